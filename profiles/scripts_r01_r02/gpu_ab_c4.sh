# A/B: config 4 (barbell, ResNet-50) with the product library vs tools/tune/libtal_agg_$1.so, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/abc4_$1; mkdir -p $OUT
for rep in 1 2; do
  for v in base $1; do
    if [ $v = base ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_$v.so; fi
    timeout -k 10 300 python bench.py --graph barbell --model resnet50 --steps 10 --no-cpu-baseline --no-k1 > $OUT/${v}_$rep.log 2>&1 || { echo FAIL $v; tail -5 $OUT/${v}_$rep.log; exit 1; }
    python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print(sys.argv[2], round(r['kernel_ms'],3), d['parity'])" $OUT/${v}_$rep.log $v
  done
done
echo EXIT 0
