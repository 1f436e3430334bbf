# GPU: kernel parity tests, then config 3 (tuned) and config 5 fp32 / bf16 benches.
# Usage: bash profiles/scripts_r01_r02/gpu_k3n_check.sh <tag>   (uses the in-tree library built on the CPU host)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-k3n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo TESTS FAILED; exit 1; }
timeout -k 10 300 python bench.py --steps 40 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c3.log 2>&1 || { echo C3 FAILED; exit 1; }
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5.log 2>&1 || { echo C5 FAILED; exit 1; }
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_c5bf16.log 2>&1 || { echo C5BF16 FAILED; exit 1; }
echo EXIT 0
