# Round 5 (r05n): cache policy of the round kernel's streams, out of place and IN PLACE (the
# product executor's form): non-temporal loads/stores (product) vs plain loads, plain stores,
# both plain (probe builds, tools/build_probe_libs.sh), config 3 default plan, 8 destinations.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=$R/gpurun_out/${1:-r05n}; mkdir -p $OUT
for v in product ldplain stplain both; do
  if [ $v = product ]; then unset TAL_LIB_PATH; else export TAL_LIB_PATH=$R/tools/tune/libtal_agg_$v.so; fi
  timeout -k 10 300 python tools/form_placement_probe.py --forms 0 --windows 4 --skip-windows 4 --allocs 4 --reps 3 --in-place > $OUT/$v.jsonl 2> $OUT/$v.err || { echo "FAIL $v"; tail -5 $OUT/$v.err; exit 1; }
  grep summary $OUT/$v.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', 'in_place' if d['in_place'] else 'out', 'windows', d['windows_ms'], 'allocs', d['allocs_ms'], 'median', d['median'])"
done
echo EXIT 0
