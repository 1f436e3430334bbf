# Round 3 (b): K3r parity tests, full-size config 3/4 reference tests, config-5 K3r bench lines, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03b}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_reg.py > $OUT/reg_tests.log 2>&1; rc=$?
tail -3 $OUT/reg_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/reg_tests.log | head -20; exit $rc; }
for dt in f32 bf16; do
  timeout -k 10 300 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype $dt --steps 5 --warmup 1 \
    --no-cpu-baseline --no-k1 --placement-trials 2 --plan '{"reg": 1}' > $OUT/c5_reg_${dt}.log 2>&1 || { echo FAIL $dt; tail -5 $OUT/c5_reg_${dt}.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], 'reg', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['parity'], d['parity_k3_vs_k1'])" $OUT/c5_reg_${dt}.log $dt
done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py -k "config3 or config4" > $OUT/full_tests.log 2>&1; rc=$?
tail -3 $OUT/full_tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/full_tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity','parity_k3_vs_k1')}, d['roofline']['frac'], d['plan']['spec'], d['k1_per_call'], {k: v for k, v in d['cpu_baseline'].items() if k!='sample'})"
