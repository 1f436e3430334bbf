# Round 3 (u): HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) of the bench's config-3
# plan and of config 5's narrow plans (fp32; bf16 with the 16-B staging lanes) on the round-3 code
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r03u}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
pmc() {  # name spec workload [bench args]
  local name=$1 spec=$2 wl=$3; shift 3
  echo "{\"spec\": $spec, \"workload\": \"$wl\"}" > $OUT/pmc_$name.spec
  for c in FETCH_SIZE WRITE_SIZE; do
    local s=fetch; [ $c = WRITE_SIZE ] && s=write
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${name}_$s -o pmc -- \
      python3 $R/bench.py --plan "$spec" --steps 4 --warmup 1 --no-cpu-baseline --no-k1 --placement-trials 2 "$@" \
      > $OUT/pmc_${name}_$s.log 2>&1 || { echo FAIL pmc $name $c; tail -5 $OUT/pmc_${name}_$s.log; return 1; }
  done
  echo ok $name
}
pmc c3_c64_l81920 '{"c4": 64, "dense": 0, "lds": 81920}' random-64-resnet50 &&
pmc c5_f32 '{"c4": 16, "dense": 0, "lds": 81920}' sbm-256-vit_b16 --graph sbm --devices 256 --model vit_b16 &&
pmc c5_bf16 '{"c4": 16, "dense": 0, "lds": 81920}' sbm-256-vit_b16-bf16 --graph sbm --devices 256 --model vit_b16 --dtype bf16 || exit 1
