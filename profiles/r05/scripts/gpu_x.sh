# Round 5 (r05x): broadcast form with the program's record words preloaded into SGPRs (no scalar
# load inside a record's batch, so its math starts as its first LDS read lands): parity, then
# config 5 with degree-centrality weights (fp32, bf16 FMA) on the default and tuned plans.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05x}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bcast.py tests/test_gpu_fullsize.py -k "bcast or degree or config5" > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1 --weights degcent"
for v in "f32:--no-tune" "bf16:--dtype bf16 --no-tune" "f32:" "bf16:--dtype bf16"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 400 python bench.py $C5 $args > $OUT/c5dc_${name}_$( [ -z "${args##*no-tune*}" ] && echo default || echo tuned ).log 2>&1 || { echo FAIL $v; exit 1; }
done
for f in $OUT/c5dc_*.log; do
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[1].split('/')[-1], d['dtype'], round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], (d.get('plan') or {}).get('spec'))
" $f
done
echo EXIT 0
