"""Build the gfx950 HIP library (C-ABI) in-tree.

The product is ``topology_aware_learning_amd/libtal_agg.so``: hand-written CDNA4 kernels plus
the ``extern "C"`` entry points declared in ``include/tal_agg.h``.  It is compiled by hipcc for
``--offload-arch=gfx950`` only, with ``-ffp-contract=off`` so the exact-mode kernels can never
contract the reference's separate fp32 multiply and add into an FMA.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
SRC = PKG / "csrc" / "tal_agg.hip"
HDR = ROOT / "include" / "tal_agg.h"
LIB = PKG / "libtal_agg.so"
SWAP_SRC = PKG / "csrc" / "storage_swap.cpp"
SWAP_LIB = PKG / "libtal_swap.so"

HIPCC_FLAGS = [
    "--offload-arch=gfx950",
    "-O3",
    "-std=c++17",
    "-ffp-contract=off",
    "-fPIC",
    "-shared",
    # torch bundles a ROCm 7.0 HIP runtime (same soname as /opt/rocm's 7.2); code object v5
    # loads under both.
    "-mcode-object-version=5",
    # RCCL is not linked: the halo entry points dlopen it on first use (a host without RCCL
    # still loads the library; under torch its already-loaded copy is found by soname)
    "-ldl",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build_library(force: bool = False, verbose: bool = False) -> Path:
    """Compile csrc/tal_agg.hip -> libtal_agg.so (skipped when up to date)."""
    if not force and not _stale(LIB, [SRC, HDR]):
        return LIB
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc(), *HIPCC_FLAGS, str(SRC), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


def build_swap(force: bool = False, verbose: bool = False) -> Path:
    """Compile csrc/storage_swap.cpp -> libtal_swap.so (host C++ against torch's c10 headers:
    the double-buffered round's storage exchange; skipped when up to date)."""
    if not force and not _stale(SWAP_LIB, [SWAP_SRC]):
        return SWAP_LIB
    import torch

    tdir = Path(torch.__file__).resolve().parent
    tmp = SWAP_LIB.with_suffix(".so.tmp")
    cmd = [shutil.which("g++") or "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-isystem", str(tdir / "include"),
           str(SWAP_SRC), "-L" + str(tdir / "lib"), "-lc10", "-Wl,-rpath," + str(tdir / "lib"), "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, SWAP_LIB)
    return SWAP_LIB


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
    print(build_swap(force="--force" in sys.argv, verbose=True))
