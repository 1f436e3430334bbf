"""Per-kernel register / scratch / spill report of the gfx950 library build (hipcc remarks).

usage: python tools/kernel_resources.py [substring-filter]
"""
import re
import subprocess
import sys
from pathlib import Path

SRC = Path(__file__).resolve().parents[1] / "topology_aware_learning_amd/csrc/tal_agg.hip"
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
       "-shared", "-mcode-object-version=5", "-Rpass-analysis=kernel-resource-usage", str(SRC), "-o", "/tmp/_kr.so"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|TotalSGPRs|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = r["name"]
    if flt not in n:
        continue
    short = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)[:70]
    print(f"{short:72s} sgpr={r.get('TotalSGPRs')} vgpr={r.get('VGPRs')} scratch={r.get('ScratchSize [bytes/lane]')} "
          f"sspill={r.get('SGPRs Spill')} vspill={r.get('VGPRs Spill')} occ={r.get('Occupancy [waves/SIMD]')}")
