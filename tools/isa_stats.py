"""Instruction mix of one kernel in the gfx950 build (device assembly).

usage: python tools/isa_stats.py <kernel-name-substring> [--dump FILE]
"""
import collections
import re
import subprocess
import sys
from pathlib import Path

SRC = Path(__file__).resolve().parents[1] / "topology_aware_learning_amd/csrc/tal_agg.hip"
asm = Path("/tmp/_tal_isa.s")
if not asm.exists() or asm.stat().st_mtime < SRC.stat().st_mtime:
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-mcode-object-version=5", "--cuda-device-only", "-S", str(SRC), "-o", str(asm)], check=True)
s = asm.read_text()
pat = sys.argv[1]
names = re.findall(r"^(_Z\S+):\s*;", s, re.M)
hits = [n for n in names if pat in n]
if not hits:
    sys.exit(f"no kernel matches {pat!r}")
n = hits[0]
i = s.index(n + ":")
j = s.index(".Lfunc_end", i)
body = s[i:j]
c = collections.Counter(re.findall(r"^\s+((?:s|v|ds|global|buffer|scratch)_[a-z0-9_]+)", body, re.M))
print(n, f"({len(hits)} matches)")
for k, v in c.most_common(60):
    print(f"{v:6d} {k}")
if "--dump" in sys.argv:
    Path(sys.argv[sys.argv.index("--dump") + 1]).write_text(body)
