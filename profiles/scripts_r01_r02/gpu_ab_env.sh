# GPU A/B of a library experiment switch: parity tests with the switch on, then config-3 benches
# (c4 = 32 and 16 narrow plans) with it off / on, twice, and config 5 off / on.
# Usage: bash profiles/scripts_r01_r02/gpu_ab_env.sh <tag> <VAR> <value>   (uses the in-tree library built on the CPU host)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=$1; VAR=$2; VAL=$3
env $VAR=$VAL timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
for rep in 1 2; do
  for on in 0 1; do
    for c4 in 32 16; do
      if [ $on = 1 ]; then V=$VAL; else V=; fi
      env $VAR=$V timeout -k 10 200 python bench.py --plan "{\"c4\": $c4, \"lds\": 81920, \"dense\": 0}" --steps 40 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c3_on${on}_c${c4}_r${rep}.log 2>&1 || { echo BENCH FAILED; exit 1; }
    done
  done
done
for on in 0 1; do
  if [ $on = 1 ]; then V=$VAL; else V=; fi
  env $VAR=$V timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5_on${on}.log 2>&1 || { echo C5 FAILED; exit 1; }
done
echo EXIT 0
