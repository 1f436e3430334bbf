# Round 4 (i): after the default-plan change (fp32 per-operand weights -> broadcast 8x2) and the
# DMA variant's removal: broadcast / fullsize-config-5 / K3r / interface tests, the config-5
# degree-centrality defaults, then the PMC passes before/after (gpu_pmc.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04i}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_bcast.py tests/test_gpu_reg.py tests/test_cosine_threads.py "tests/test_gpu_fullsize.py::test_config5_degree_centrality_vs_reference" "tests/test_gpu_fullsize.py::test_config5_bf16_fma_full_width_within_bound" tests/test_gpu_interface.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --weights degcent --no-tune"
for dt in f32 bf16; do
  timeout -k 10 300 python bench.py $C5 --dtype $dt > $OUT/c5dc_${dt}_default.log 2>&1 || { echo "BENCH FAILED $dt"; tail -20 $OUT/c5dc_${dt}_default.log; exit 1; }
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['plan']['spec'], json.dumps(d.get('placement'))[:300])
" $OUT/c5dc_${dt}_default.log $dt
done
bash profiles/r04/scripts/gpu_pmc.sh ${1:-r04i}_pmc || exit 1
echo EXIT 0
