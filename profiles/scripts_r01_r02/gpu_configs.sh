# GPU: distributed virtual-rank test + the BASELINE configs 2-5 on one GPU (parity-check lines).
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-cfg}
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/${TAG}_dist.log 2>&1 && \
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --steps 10 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --model resnet50 --steps 5 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c4.log 2>&1 && \
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5.log 2>&1 && \
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_c5bf16.log 2>&1 && \
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --mode exact --steps 3 --warmup 1 --no-cpu-baseline > $OUT/${TAG}_c5bf16x.log 2>&1 && \
timeout -k 10 300 python bench.py --host-path --steps 5 --no-cpu-baseline > $OUT/${TAG}_host.log 2>&1
echo EXIT $?
