# Build A/B probe variants of the library into tools/tune/ (not the product), with the product's
# own hipcc flags (topology_aware_learning_amd/build.py) plus the variant's.
# Usage: bash tools/build_probe_libs.sh NAME:FLAGS ...   e.g. o2:-O2  (the product source carries no
# probe switches since round 6: a variant is a -D / flag the kernels read, or a copy of the source)
cd "$(dirname "$0")/.."
base=$(python -c "from topology_aware_learning_amd.build import HIPCC_FLAGS; print(' '.join(HIPCC_FLAGS))")
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc $base $flags topology_aware_learning_amd/csrc/tal_agg.hip -o tools/tune/libtal_agg_$name.so &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
