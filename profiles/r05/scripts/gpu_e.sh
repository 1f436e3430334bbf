# Round 5 closing (r05e): the driver's bench command under rocprofv3 --kernel-trace --stats (the
# headline's kernel time from the trace beside the bench's HIP events), smoke, and the BASELINE
# configs 2, 4, 5 table with the product's default tuning.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05e}; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o trace -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3_trace.log 2>&1 ) || { echo FAIL c3_trace; tail -20 $OUT/c3_trace.log; exit 1; }
python3 tools/summarize_trace.py $OUT/c3_trace $OUT/c3_trace.log $OUT/prof 20 "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5" || exit 1
rm -rf $OUT/c3_trace
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1"
timeout -k 10 300 python bench.py --graph ring --devices 32 --model resnet18 --degree 2 --steps 20 --no-cpu-baseline --no-k1 > $OUT/c2.log 2>&1 && \
timeout -k 10 300 python bench.py --graph barbell --devices 128 --model resnet50 --steps 10 --no-cpu-baseline --no-k1 > $OUT/c4.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 > $OUT/c5.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 > $OUT/c5bf16.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 --mode exact > $OUT/c5bf16x.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --weights degcent > $OUT/c5degcent.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --weights degcent --dtype bf16 > $OUT/c5degcent_bf16.log 2>&1 && \
timeout -k 10 300 python bench.py --host-path --steps 5 --no-cpu-baseline > $OUT/host.log 2>&1 || { echo FAILED; exit 1; }
for f in c2 c4 c5 c5bf16 c5bf16x c5degcent c5degcent_bf16 host; do
  python -c "
import json,sys
d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; r=d['roofline']
print(sys.argv[2], d['dtype'], round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],3), d['parity'], d['kernel'], (d.get('plan') or {}).get('spec'), d.get('host_path_per_call',{}).get('ms') if 'host_path_per_call' in d else '')
" $OUT/$f.log $f
done | tee $OUT/summary.txt
echo EXIT 0
