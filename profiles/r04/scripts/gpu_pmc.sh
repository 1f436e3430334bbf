# Round 4: config 5 with degree-centrality weights, before (K3n pairs form; K3r for bf16) and
# after (broadcast form): SQ wave states, LDS / VALU instruction counters, HBM traffic.
# One counter group per rocprofv3 pass; the summary takes the last round-kernel dispatch.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04pmc}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
WS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
LV="SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
B="--graph sbm --devices 256 --model vit_b16 --steps 2 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --weights degcent"
pmc() {  # name pass counters spec dtype
  local name=$1 pass=$2 ctr=$3 spec=$4 dt=$5
  echo "{\"spec\": $spec, \"dtype\": \"$dt\"}" > $OUT/$name.spec
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/${name}_$pass -o pmc -- \
    python3 $R/bench.py $B --dtype $dt --plan "$spec" > $OUT/${name}_$pass.log 2>&1 || { echo "FAIL $name $pass"; tail -5 $OUT/${name}_$pass.log; return 1; }
  python3 $R/tools/pmc_shrink.py $OUT/${name}_$pass || return 1  # the last round dispatch only (copy-back limit)
  echo "ok $name $pass"
}
PAIRS='{"c4":16,"lds":163840,"dense":0}'
BC16='{"c4":16,"lds":163840,"dense":0,"bcast":16,"bcwg":2}'
BC8='{"c4":16,"lds":163840,"dense":0,"bcast":8,"bcwg":2}'
REG='{"reg":1}'
X2='{"c4":32,"lds":163840,"dense":0,"bcast":16,"bcwg":1}'
for run in "bf16_pairs|$PAIRS|bf16" "bf16_bcast16|$BC16|bf16" "bf16_reg|$REG|bf16" "bf16_x2|$X2|bf16" "f32_pairs|$PAIRS|f32" "f32_bcast8|$BC8|f32" "f32_x2|$X2|f32"; do
  IFS='|' read -r name spec dt <<< "$run"
  pmc $name ws "$WS" "$spec" $dt && pmc $name lv "$LV" "$spec" $dt || exit 1
  case $name in *reg) continue;; esac
  pmc $name fetch FETCH_SIZE "$spec" $dt && pmc $name write WRITE_SIZE "$spec" $dt || exit 1
done
echo EXIT 0
