# Round 6 (r06a): tal_fill_counter (the library's seeded-row generator) against synth, the
# smoke, and ONE run of the command that crashed in round 5 (gpurun_out/r05c/pmc_lds.log:
# SIGSEGV inside torch's bitwise_and launch of the ~20-launch torch generator under
# rocprofv3 --pmc) - now with the one-launch generator.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r06a}; mkdir -p $OUT
cd $R
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 300 $PT tests/test_fill_counter.py > $OUT/t_fill.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_lds -o pmc -- \
    python3 $R/bench.py --graph sbm --devices 256 --model vit_b16 --steps 2 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --dtype bf16 > $OUT/pmc_lds.log 2>&1 ) && \
python3 -c "import csv,sys,pathlib,collections; p=next(pathlib.Path(sys.argv[1]).rglob('*counter_collection.csv')); r=list(csv.DictReader(open(p))); d={x['Dispatch_Id']:x['Kernel_Name'] for x in r}; c=collections.Counter(v.split('(')[0][:80] for v in d.values()); print('dispatches', len(d)); [print(n, k) for k, n in c.most_common(12)]" $OUT/pmc_lds > $OUT/pmc_dispatches.txt && \
python3 tools/pmc_shrink.py $OUT/pmc_lds && \
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>$OUT/bench.err
rc=$?
echo EXIT $rc
