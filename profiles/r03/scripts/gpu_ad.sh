# Round 3 (ad): default plan = K3r for bf16 FMA rounds with per-operand weights — the K3r GPU
# tests (RoundExecutor included), then config 5 bf16 degree-centrality with the untimed default
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03ad}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_reg.py tests/test_gpu_interface.py > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --weights degcent --dtype bf16 --no-tune > $OUT/c5degcent_bf16_default.log 2>&1 || { tail -5 $OUT/c5degcent_bf16_default.log; exit 1; }
grep '^{' $OUT/c5degcent_bf16_default.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['kernel'], round(d['roofline']['kernel_ms'],3), d['parity'], d['plan'].get('spec'))"
