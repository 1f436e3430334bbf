# Round 5 (r05c): the W16 LDS column permutation (bf16 staging bank conflicts)
# and the tile-walk switch (placement, item 3).  Parity of both first, then the probes, then the
# whole GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r05c}; mkdir -p $OUT
cd $R
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
C5="--graph sbm --devices 256 --model vit_b16 --steps 3 --warmup 1 --no-cpu-baseline --no-k1"
timeout -k 10 400 $PT tests/test_gpu_walk.py tests/test_gpu_bcast.py > $OUT/t_walk_bcast.log 2>&1 && \
timeout -k 10 300 python tools/form_placement_probe.py --windows 8 --allocs 4 --reps 3 --walks 1,0,2,8 --forms 0,2,6 > $OUT/walk_probe.jsonl 2>$OUT/walk_probe.err && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 > $OUT/c5bf16.log 2>&1 && \
timeout -k 10 400 python bench.py $C5 --dtype bf16 --weights degcent > $OUT/c5degcent_bf16.log 2>&1 && \
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_lds -o pmc -- \
    python3 $R/bench.py --graph sbm --devices 256 --model vit_b16 --steps 2 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 --dtype bf16 > $OUT/pmc_lds.log 2>&1 ) && \
python3 tools/pmc_shrink.py $OUT/pmc_lds && \
timeout -k 10 900 $PT tests > $OUT/t_all.log 2>&1
rc=$?
tail -3 $OUT/t_all.log 2>/dev/null
echo EXIT $rc
