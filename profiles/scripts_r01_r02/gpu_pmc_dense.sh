# GPU: SQ counters of the dense-config round kernels (config 4, barbell) for the resident and
# streamed forms.  Two counter passes per form (8 SQ slots each), kernel-trace only.
set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; exit 1; }
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmcd}; mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INST_CYCLES_SMEM"
B="bench.py --graph barbell --model resnet50 --steps 3 --warmup 1 --no-cpu-baseline --no-k1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_stream -o kt -- python3 $B --stream-rows 64 > $OUT/stream_bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1_stream -o p1 -- python3 $B --stream-rows 64 > $OUT/p1_stream.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P2 --output-format csv -d $OUT/p2_stream -o p2 -- python3 $B --stream-rows 64 > $OUT/p2_stream.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P1 --output-format csv -d $OUT/p1_res -o p1 -- python3 $B --c4 128 > $OUT/p1_res.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc $P2 --output-format csv -d $OUT/p2_res -o p2 -- python3 $B --c4 128 > $OUT/p2_res.log 2>&1
echo EXIT $?
