# Round 4 (o): probe TAL_PROBE_ROWW_X2 (tools/tune/libtal_agg_roww2.so: ROWW passes of 8 rows x 8
# lanes, two float4 chunks per lane, at c4 = 16): ROWW parity tests through the probe library,
# then config 5 unweighted fp32 / bf16 FMA, product vs probe, interleaved twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04o}; mkdir -p $OUT
P=$GRAFT_REPO_ROOT/tools/tune/libtal_agg_roww2.so
TAL_LIB_PATH=$P timeout -k 10 600 python -u -m pytest "tests/test_gpu_kernels.py::test_round_narrow_vs_oracle" "tests/test_gpu_kernels.py::test_round_narrow_row_uniform_weights_signed_zero" "tests/test_gpu_kernels.py::test_round_narrow_sbm256_one_group" "tests/test_gpu_fullsize.py::test_config5_full_round_vs_reference" -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --no-tune --placement-trials 2"
for rep in 1 2; do
  for dt in bf16 f32; do
    for lib in prod roww2; do
      L=; [ $lib = roww2 ] && L=$P
      TAL_LIB_PATH=$L timeout -k 10 300 python bench.py $C5 --dtype $dt > $OUT/${dt}_${lib}_$rep.log 2>&1 || { echo "BENCH FAILED $dt $lib"; tail -20 $OUT/${dt}_${lib}_$rep.log; exit 1; }
      python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['parity_k3_vs_k1']['rows_differing'], d['plan']['spec'])
" $OUT/${dt}_${lib}_$rep.log ${dt}_${lib}_$rep
    done
  done
done
echo EXIT 0
