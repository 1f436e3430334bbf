# Build A/B probe variants of the library into tools/tune/ (not the product).
# Usage: bash tools/build_probe_libs.sh NAME:FLAGS ...   e.g. nocomp:-DTAL_PROBE_NOCOMP
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}; flags=${flags//,/ }
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -mcode-object-version=5 \
    $flags topology_aware_learning_amd/csrc/tal_agg.hip -o tools/tune/libtal_agg_$name.so &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=1; done
exit $rc
