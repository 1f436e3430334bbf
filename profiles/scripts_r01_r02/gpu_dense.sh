# GPU: kernel parity tests + the dense configs (4: barbell, 5: sbm / vit_b16) for kernel tuning.
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-dense}
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > $OUT/${TAG}_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --model resnet50 --steps 5 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c4.log 2>&1 && \
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5.log 2>&1
echo EXIT $?
