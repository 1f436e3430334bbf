# Round 3: config-5 memory-side walk probe (fp32, bf16) and the current config-5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-c5walk}; mkdir -p $OUT
timeout -k 10 240 ./tools/tune/c5_walk_probe > $OUT/walk_f32.log 2>&1 && cat $OUT/walk_f32.log &&
timeout -k 10 240 ./tools/tune/c5_walk_probe bf16 > $OUT/walk_bf16.log 2>&1 && cat $OUT/walk_bf16.log &&
for dt in f32 bf16; do
  timeout -k 10 300 python bench.py --graph sbm --devices 256 --model vit_b16 --dtype $dt --steps 5 --warmup 1 \
    --no-cpu-baseline --no-k1 --placement-trials 2 --no-tune > $OUT/c5_${dt}.log 2>&1 || { echo FAIL $dt; tail -5 $OUT/c5_${dt}.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[2], round(d['roofline']['kernel_ms'],3), d['roofline']['frac'], d['parity'], d.get('plan',{}).get('spec'))" $OUT/c5_${dt}.log $dt
done
