# Round 5 (r05y): A/B on one board - broadcast form with record words in SGPRs (product) vs read
# in the loop (probe build -DTAL_PROBE_BC_SMEM, round 4's form), config 5 with degree-centrality
# weights, fixed plans, two interleaved passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05y}; mkdir -p $OUT
C5="--graph sbm --devices 256 --model vit_b16 --steps 5 --warmup 1 --no-cpu-baseline --no-k1 --weights degcent --placement-trials 2"
for pass in 1 2; do
  for v in product bcsmem; do
    if [ $v = product ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$R/tools/tune/libtal_agg_$v.so; fi
    for f in "f32_8x2:--plan {\"c4\":16,\"lds\":163840,\"dense\":0,\"bcast\":8,\"bcwg\":2}" \
             "bf16_x2:--dtype bf16 --plan {\"c4\":32,\"lds\":163840,\"dense\":0,\"bcast\":16,\"bcwg\":1}" \
             "bf16_16x2:--dtype bf16 --plan {\"c4\":16,\"lds\":163840,\"dense\":0,\"bcast\":16,\"bcwg\":2}"; do
      name=${f%%:*}; args=${f#*:}
      timeout -k 10 300 python bench.py $C5 $args > $OUT/${name}_${v}_$pass.log 2>&1 || { echo FAIL $name $v; tail -5 $OUT/${name}_${v}_$pass.log; exit 1; }
      python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print('$pass', '$name', '$v', round(r['kernel_ms'],3), round(r['frac'],3), d['parity'])
" $OUT/${name}_${v}_$pass.log
    done
  done
done
echo EXIT 0
