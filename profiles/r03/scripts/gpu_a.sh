# Round 3 (a): GPR-index semantics probe, the fused K1 / interface / host-cache GPU tests, the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03a}; mkdir -p $OUT
timeout -k 10 60 ./tools/tune/gpridx_probe > $OUT/gpridx.log 2>&1; echo "gpridx rc=$?"; cat $OUT/gpridx.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "agg_model or agg_f32 or agg_i64 or ring32" tests/test_gpu_interface.py tests/test_gpu_host_cache.py \
  > $OUT/tests.log 2>&1; rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity','parity_k3_vs_k1')}, d['roofline']['frac'], d['k1_per_call'], {k: v for k, v in d['cpu_baseline'].items() if k!='sample'})"
