"""Build the stamped diagnostic variant of the library (not part of the product):
tools/tune/libtal_agg_stamps.so = csrc/tal_agg.hip with s_memtime stamps at the phase boundaries
of k_cosine_staged (kernel start, after the plan reads, after staging, after the norms, after the
level-0 runs, end) written by thread 0 of each workgroup to a device array, and an extra export
tal_debug_stamps(out, n) that copies them out.  tools/cosine_stamps.py reads them.
usage: python tools/stamps_build.py
Historical: it patches the slab-staged K2 kernel, which the streamed column kernels replaced
(run it on a checkout of commit 17a9a02 or earlier; profiles/r06/stamps holds its output)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def patch(src: str) -> str:
    def rep(old, new):
        nonlocal src
        assert old in src, old[:80]
        src = src.replace(old, new, 1)

    rep('#include "../../include/tal_agg.h"', f'#include "{ROOT}/include/tal_agg.h"')
    rep("constexpr int kCosMaxPairs = 32;", """__device__ unsigned long long g_stamps[16384 * 8];
__device__ __forceinline__ void stamp(int k) {
  if (threadIdx.x == 0 && blockIdx.x < 16384) g_stamps[blockIdx.x * 8 + k] = __builtin_amdgcn_s_memtime();
}
constexpr int kCosMaxPairs = 32;""")
    rep("  const int L = blockIdx.x;\n  const int kq = L >> 3;\n  const int pg = kq % npg;",
        "  stamp(0);\n  const int L = blockIdx.x;\n  const int kq = L >> 3;\n  const int pg = kq % npg;")
    rep("  if (row) cos_stage<true>(gm, np + 1, nq * I, sx, I, Pr);",
        "  stamp(1);\n  if (row) cos_stage<true>(gm, np + 1, nq * I, sx, I, Pr);")
    rep("""  __syncthreads();
  const int64_t n_out = plan[1];""", """  __syncthreads();
  stamp(2);
  const int64_t n_out = plan[1];""")
    rep("""  else cos_staged_body<false, 0>(sx, mb, sn, sy, sl, sr, np, nq, I, B, Pr, s, n_out);
}""", """  else cos_staged_body<false, 0>(sx, mb, sn, sy, sl, sr, np, nq, I, B, Pr, s, n_out);
  stamp(5);
}""")
    rep("""      sy[m][g] = __fdiv_rn(1.f, nrm);
    }
  }
  __syncthreads();""", """      sy[m][g] = __fdiv_rn(1.f, nrm);
    }
  }
  __syncthreads();
  stamp(3);""")
    rep("""    sr[ia] = v;
  }
  __syncthreads();""", """    sr[ia] = v;
  }
  __syncthreads();
  stamp(4);""")
    rep("""extern "C" {

const char* tal_last_error(void) { return g_err.c_str(); }""", """extern "C" {

int32_t tal_debug_stamps(unsigned long long* out, int32_t n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * n) == hipSuccess ? 0 : 2;
}

const char* tal_last_error(void) { return g_err.c_str(); }""")
    return src


def main():
    from topology_aware_learning_amd.build import HIPCC_FLAGS, hipcc

    src = (ROOT / "topology_aware_learning_amd" / "csrc" / "tal_agg.hip").read_text()
    out = ROOT / "tools" / "tune" / "tal_stamps.hip"
    out.write_text(patch(src))
    lib = ROOT / "tools" / "tune" / "libtal_agg_stamps.so"
    subprocess.run([hipcc(), *HIPCC_FLAGS, str(out), "-o", str(lib)], check=True)
    out.unlink()
    print(lib)


if __name__ == "__main__":
    main()
