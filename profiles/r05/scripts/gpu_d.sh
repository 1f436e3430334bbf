# Round 5 (r05d): LDS counters of the bf16 config-5 round after the W16 column permutation,
# the drop-in driver rates (batched round bookkeeping), the headline bench, the whole GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05d}; mkdir -p $OUT
cd $R
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
RR="$R/tools/run_round.py --graph sbm --devices 256 --model vit_b16 --dtype bf16 --mode fma --fill randn --steps 3"
LV="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
pmc() {  # name plan-json [env]
  ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc $LV --output-format csv -d $OUT/pmc_$1 -o pmc -- \
      python3 $RR --plan "$2" > $OUT/pmc_$1.log 2>&1 ) && python3 $R/tools/pmc_shrink.py $OUT/pmc_$1 && echo "ok pmc $1"
}
pmc narrow16 '{"c4":16,"lds":81920,"dense":0}' && \
pmc x2 '{"c4":32,"lds":163840,"dense":0,"bcast":16,"bcwg":1}' && \
timeout -k 10 300 python tools/dropin_rate.py 7 > $OUT/dropin.log 2>&1 && \
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 && \
timeout -k 10 900 $PT tests > $OUT/t_all.log 2>&1
rc=$?
tail -3 $OUT/t_all.log 2>/dev/null
echo EXIT $rc
