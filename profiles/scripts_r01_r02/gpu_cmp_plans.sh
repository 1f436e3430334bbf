cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for spec in "64 163840" "64 81920" "16 81920" "16 163840" "32 81920" "32 163840"; do
  set -- $spec
  timeout -k 10 120 python tools/run_round.py --c4 $1 --lds $2 --steps 10 2>&1 | grep -v amdgpu.ids | tr '\n' ' '; echo
done
done
