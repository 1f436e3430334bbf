# Profiling pass (round 2): the driver's bench command under rocprofv3 --kernel-trace --stats
# (bench line + kernel trace from ONE process), then FETCH_SIZE / WRITE_SIZE passes per plan
# spec the tuner can pick, for tools/summarize_r02.py.   Usage: bash profiles/scripts_r01_r02/gpu_profile.sh <tag>
set -o pipefail
TAG=${1:-r02prof}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o trace -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/c3_trace.log 2>&1 || { echo FAIL c3_trace; exit 1; }
pmc() {  # name spec workload [bench args]
  local name=$1 spec=$2 wl=$3; shift 3
  echo "{\"spec\": $spec, \"workload\": \"$wl\"}" > $OUT/pmc_$name.spec
  for c in FETCH_SIZE WRITE_SIZE; do
    local s=fetch; [ $c = WRITE_SIZE ] && s=write
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${name}_$s -o pmc -- \
      python3 $R/bench.py --plan "$spec" --steps 4 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 "$@" \
      > $OUT/pmc_${name}_$s.log 2>&1 || { echo FAIL pmc $name $c; return 1; }
  done
}
# every sparse spec the tuner builds (tile width x LDS budget) on configs 3 and 2, plus config 5's
rc=0
for c4 in 16 32 64 128; do
  for lds in 81920 163840; do
    spec="{\"c4\": $c4, \"dense\": 0, \"lds\": $lds}"
    pmc c3_c${c4}_l$lds "$spec" random-64-resnet50 && \
    pmc c2_c${c4}_l$lds "$spec" ring-32-resnet18 --graph ring --model resnet18 --devices 32 --degree 2 || { rc=1; break 2; }
  done
done
# config 3's other candidates: dense row blocks (c4 >= 64) and the streamed groupings
for c4 in 64 128; do
  for lds in 81920 163840; do
    [ $rc = 0 ] && { pmc c3_c${c4}_l${lds}_d8 "{\"c4\": $c4, \"dense\": 8, \"lds\": $lds}" random-64-resnet50 || rc=1; }
  done
done
for g in "64 0" "128 0" "64 96"; do
  set -- $g
  [ $rc = 0 ] && { pmc c3_s$1_$2 "{\"stream_rows\": $1, \"stream_src\": $2}" random-64-resnet50 || rc=1; }
done
[ $rc = 0 ] && \
pmc c5_c16 '{"c4": 16, "dense": 0, "lds": 81920}' sbm-256-vit_b16 --graph sbm --model vit_b16 --devices 256 && \
pmc c5_c16_bf16 '{"c4": 16, "dense": 0, "lds": 81920}' sbm-256-vit_b16-bf16 --graph sbm --model vit_b16 --devices 256 --dtype bf16
echo PROFILE EXIT $?
