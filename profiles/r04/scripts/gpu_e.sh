# Round 4: placement sensitivity of config 5 (windows of one arena, bf16 FMA), config 3
# window map repeated, then the PMC passes (gpu_pmc.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04e}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16"
timeout -k 10 400 python tools/window_probe.py $C5 --dtype bf16 --mode fma --windows 4 --allocs 0 --reps 2 > $OUT/window_c5_bf16.log 2>&1 || { echo W5B FAILED; tail -5 $OUT/window_c5_bf16.log; exit 1; }
tail -1 $OUT/window_c5_bf16.log
timeout -k 10 300 python tools/window_probe.py --windows 24 --allocs 8 --reps 3 > $OUT/window_map2.log 2>&1 || { echo WMAP FAILED; tail -5 $OUT/window_map2.log; exit 1; }
tail -1 $OUT/window_map2.log
timeout -k 10 200 python tools/window_probe.py --step-mb 128 --span-gb 6 --allocs 0 --reps 3 > $OUT/window_slide.log 2>&1 || { echo WSLIDE FAILED; tail -5 $OUT/window_slide.log; exit 1; }
tail -1 $OUT/window_slide.log | cut -c1-400
bash profiles/r04/scripts/gpu_pmc.sh r04pmc || exit 1
echo EXIT 0
