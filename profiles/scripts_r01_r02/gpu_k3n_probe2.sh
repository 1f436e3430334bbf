# Config 5: one-workgroup-per-CU narrow kernel with / without one-batch-ahead LDS data reads.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-k3n2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
SPEC='{"c4": 16, "dense": 0, "lds": 81920}'
for v in ${VARIANTS:-base nocomp noload}; do
  if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
  for dt in f32 bf16; do
    timeout -k 10 300 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype $dt --steps 3 --warmup 1 \
      --no-cpu-baseline --no-k1 --placement-trials 2 --plan "$SPEC" > $OUT/c5_${v}_${dt}.log 2>&1 || { echo FAIL $v $dt; tail -5 $OUT/c5_${v}_${dt}.log; exit 1; }
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], sys.argv[3], round(d['roofline']['kernel_ms'],3), d['parity'])" $OUT/c5_${v}_${dt}.log $v $dt
  done
done
echo EXIT 0
