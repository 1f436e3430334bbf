# Round 4 (e): is the slow / fast round placement a property of the allocation or of where in HBM
# a pool's bytes sit?  Config 3: windows of one arena vs separate allocations (twice, the second
# with allocations first), sliding 128-MB windows; config 5 bf16 FMA windows of one arena.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04e}; mkdir -p $OUT
last() { tail -1 $1 | cut -c1-600; }
timeout -k 10 300 python tools/window_probe.py --windows 24 --allocs 8 --reps 3 > $OUT/window_map.log 2>&1 || { echo WMAP FAILED; tail -5 $OUT/window_map.log; exit 1; }
last $OUT/window_map.log
timeout -k 10 300 python tools/window_probe.py --windows 12 --allocs 12 --reps 3 --ballast-gb 12 > $OUT/window_ballast.log 2>&1 || { echo WBAL FAILED; tail -5 $OUT/window_ballast.log; exit 1; }
last $OUT/window_ballast.log
timeout -k 10 300 python tools/window_probe.py --step-mb 128 --span-gb 6 --allocs 0 --reps 3 > $OUT/window_slide.log 2>&1 || { echo WSLIDE FAILED; tail -5 $OUT/window_slide.log; exit 1; }
last $OUT/window_slide.log
timeout -k 10 400 python tools/window_probe.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --mode fma --windows 2 --allocs 0 --reps 2 > $OUT/window_c5_bf16.log 2>&1 || { echo W5B FAILED; tail -5 $OUT/window_c5_bf16.log; exit 1; }
last $OUT/window_c5_bf16.log
echo EXIT 0
