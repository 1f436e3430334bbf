# GPU: all gpu tests, smoke, default bench, then BASELINE configs 2/4/5 on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; TAG=${1:-all}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > $OUT/${TAG}_tests.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --cpu-seconds 5 > $OUT/${TAG}_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --steps 10 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c2.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --model resnet50 --steps 5 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c4.log 2>&1 && \
timeout -k 10 400 python bench.py --graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 > $OUT/${TAG}_c5.log 2>&1
echo EXIT $?
