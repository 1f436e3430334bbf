# Round 3 (y): K3c clique kernel at 3 waves per SIMD (launch bounds cap 168 VGPRs, probe build
# libtal_agg_cq3.so) against the product's 2 (180 VGPRs at MMAX 60), config 4 on one GPU, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03y}; mkdir -p $OUT
export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_cq3.so
B="--graph barbell --devices 128 --model resnet50 --steps 10 --warmup 3 --no-cpu-baseline --no-k1 --placement-trials 4 --no-tune"
run() {
  timeout -k 10 200 python bench.py $B > $OUT/c4_$1.log 2>&1 || { echo FAIL $1; tail -5 $OUT/c4_$1.log; return 1; }
  grep '^{' $OUT/c4_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'], d['kernel'])"
}
run base && TAL_LIB_PATH=$P run cq3 && run base2 && TAL_LIB_PATH=$P run cq3b || exit 1
