# Round-2 final check: full -m gpu suite, smoke(), the driver's default bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02final2}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE FAILED; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench.log; exit 1; }
python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']; print('bench', round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), r.get('traffic'), d['plan']['spec'], d['cpu_baseline']['value'])" $OUT/bench.log
echo EXIT 0
