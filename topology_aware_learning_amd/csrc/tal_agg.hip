// tal_agg.hip — MI355X (gfx950 / CDNA4) kernels + C-ABI for topology-weighted neighbor-model
// aggregation.  See include/tal_agg.h for the contract and DESIGN.md for the roofline.
//
// Reference semantics (msakarvadia/topology_aware_learning, pure Python/PyTorch CPU):
//   src/decentralized_client.py:399-413   avg  = fp32(w0)*x0 ; avg += fp32(wi)*xi ; load_state_dict
//   src/decentralized_client.py:661-681   cosine_similarity (K2)
//   src/decentralized_app.py:605-641      one call per simulated device per round (K3 batches them)
//
// Numerics: EXACT mode = one rounded fp32 multiply then one rounded fp32 add per operand, in
// operand order — bit-identical to torch's `w * clone(v)` / `+=` on CPU.  This file is built
// with -ffp-contract=off and the exact kernels use explicit __fmul_rn / __fadd_rn so no FMA can
// be formed; the FMA mode uses __builtin_fmaf explicitly.
//
// The op is element-wise with arithmetic intensity ~0.1 flop/B: every kernel here is bound by
// HBM3E bandwidth (no MFMA — nothing here is a contraction).

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <type_traits>
#include <vector>

#include <dlfcn.h>
#include <rccl/rccl.h>  // types only: the functions are resolved at run time (rccl())

#include "../../include/tal_agg.h"

// The device code is gfx950 only: the inline asm below (v_mad_u32_u16 with op_sel, v_add_u32
// with an inline constant, global_load_lds_dwordx4 through M0, counted s_waitcnt vmcnt) is CDNA4
// ISA, and the kernels' tilings assume its 64-wide wavefronts and 160 KiB of LDS per CU.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "tal_agg.hip targets gfx950 (MI355X) only: build with --offload-arch=gfx950"
#endif

#pragma clang fp contract(off)

namespace {

constexpr int kAbiVersion = 25;
constexpr int kMaxOps = 256;     // operands per K1 launch (kernel-argument table, 3 KiB)
constexpr int kBlock = 256;      // 4 wavefronts of 64 lanes
constexpr uint32_t kMaskUniform = 0x80000000u;  // dense table mask flag: one weight for all rows
constexpr uint32_t kMaskSelf0 = 0x100u;          // streamed tables: bit 8+r = the entry is row r's own model
constexpr uint32_t kMaskSelf = 0xff00u;
constexpr int kMaxGrid = 256 * 8; // 256 CUs x 8 resident 256-thread blocks
constexpr int kK1Unroll = 1;     // float4 chunks per lane per K1 grid-stride step
constexpr int kK1Grid = 1 << 24; // K1 grid cap: in practice one chunk per lane and no second pass
                                 // (measured 5.98 vs 5.63 TB/s for a 4096-block grid-stride launch,
                                 // tools/tune/k1_probe.hip, ResNet-50 M = 9)

typedef float v4f __attribute__((ext_vector_type(4)));

thread_local std::string g_err;

int32_t fail(int32_t code, const std::string& msg) {
  g_err = msg;
  return code;
}

int32_t check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(TAL_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
  g_err.clear();
  return TAL_OK;
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }
inline bool aligned4(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 3u) == 0; }

// ------------------------------------------------------------------------------------------
// element arithmetic
// ------------------------------------------------------------------------------------------
template <bool EXACT>
__device__ __forceinline__ float first_term(float w, float x) {
  return __fmul_rn(w, x);
}

template <bool EXACT>
__device__ __forceinline__ float next_term(float acc, float w, float x) {
  if constexpr (EXACT) {
    return __fadd_rn(acc, __fmul_rn(w, x));
  } else {
    return __builtin_fmaf(w, x, acc);
  }
}

template <bool EXACT>
__device__ __forceinline__ float4 first4(float w, float4 x) {
  return make_float4(first_term<EXACT>(w, x.x), first_term<EXACT>(w, x.y),
                     first_term<EXACT>(w, x.z), first_term<EXACT>(w, x.w));
}

typedef float v2f_t __attribute__((ext_vector_type(2)));

// FMA mode: two packed fmas on the natural register pairs (x, y) and (z, w).  Written per
// component, the SLP vectorizer paired (x, z) / (y, w) and shuffled with 12 v_mov_b32 per batch
// of four operands in the narrow row loop (config 5 bf16: 1.46e10 VALU instructions per round).
__device__ __forceinline__ float4 fma4(float w, float4 x, float4 a) {
  const v2f_t w2 = {w, w};
  const v2f_t lo = __builtin_elementwise_fma(w2, v2f_t{x.x, x.y}, v2f_t{a.x, a.y});
  const v2f_t hi = __builtin_elementwise_fma(w2, v2f_t{x.z, x.w}, v2f_t{a.z, a.w});
  return make_float4(lo.x, lo.y, hi.x, hi.y);
}

template <bool EXACT>
__device__ __forceinline__ float4 next4(float4 a, float w, float4 x) {
  if constexpr (!EXACT) return fma4(w, x, a);
  return make_float4(next_term<EXACT>(a.x, w, x.x), next_term<EXACT>(a.y, w, x.y),
                     next_term<EXACT>(a.z, w, x.z), next_term<EXACT>(a.w, w, x.w));
}

__device__ __forceinline__ float4 mul4(float w, float4 x) {
  return make_float4(__fmul_rn(w, x.x), __fmul_rn(w, x.y), __fmul_rn(w, x.z), __fmul_rn(w, x.w));
}

__device__ __forceinline__ float4 add4(float4 a, float4 p) {
  return make_float4(__fadd_rn(a.x, p.x), __fadd_rn(a.y, p.y), __fadd_rn(a.z, p.z), __fadd_rn(a.w, p.w));
}

// by value: a ?: over two float4 lvalues would select between addresses and keep the
// arrays out of registers
__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
  return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// fp32 accumulator -> int64 the way load_state_dict's copy_ does it on x86: truncation toward
// zero; NaN and out-of-range give INT64_MIN (cvttss2si "integer indefinite").
__device__ __forceinline__ int64_t trunc_i64(float v) {
  if (!(v >= -9.2233720368547758e18f && v < 9.2233720368547758e18f)) return INT64_MIN;
  return static_cast<int64_t>(v);
}

// ------------------------------------------------------------------------------------------
// K1: one aggregation call, M operands given as a pointer table in the kernel arguments
// ------------------------------------------------------------------------------------------
struct OpTableF32 {
  const float* x[kMaxOps];
  float w[kMaxOps];
};

struct OpTableI64 {
  const int64_t* x[kMaxOps];
  float w[kMaxOps];
};

// Streamed operand loads are non-temporal: every operand byte is read exactly once per call,
// so keeping it out of the caches leaves L2/MALL to the output stream (measured +15-20 % at
// M = 9 on MI355X, tools/tune/k1_variants.hip).
__device__ __forceinline__ float4 ld_stream(const float* base, int64_t i) {
  const v4f q = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base) + i);
  return make_float4(q.x, q.y, q.z, q.w);
}

// K1 vector kernel.  Each lane owns kK1Unroll float4 chunks per grid-stride step and issues the
// loads of every operand of its chunks before the ordered accumulate: M * kK1Unroll 16-B loads
// in flight per lane.
// M_STATIC > 0: operand count known at compile time; 0: runtime count, loads in batches of 8.
// CONT: accumulate onto `out` (passes after the first when M > kMaxOps; keeps the exact order).
template <int M_STATIC, bool EXACT, bool CONT>
__global__ __launch_bounds__(kBlock) void k_agg_f32_vec(OpTableF32 t, int m_rt, float* out,
                                                        int64_t n4) {
  const int m = M_STATIC > 0 ? M_STATIC : m_rt;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock * kK1Unroll;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kBlock * kK1Unroll + threadIdx.x; i0 < n4;
       i0 += stride) {
    if constexpr (M_STATIC > 0) {
      float4 v[kK1Unroll][M_STATIC];
#pragma unroll
      for (int u = 0; u < kK1Unroll; ++u) {
        const int64_t i = i0 + u * kBlock;
        if (i < n4) {
#pragma unroll
          for (int k = 0; k < M_STATIC; ++k) v[u][k] = ld_stream(t.x[k], i);
        }
      }
#pragma unroll
      for (int u = 0; u < kK1Unroll; ++u) {
        const int64_t i = i0 + u * kBlock;
        if (i < n4) {
          float4 acc;
          int k0 = 0;
          if constexpr (CONT) {
            acc = reinterpret_cast<const float4*>(out)[i];
          } else {
            acc = first4<EXACT>(t.w[0], v[u][0]);
            k0 = 1;
          }
#pragma unroll
          for (int k = k0; k < M_STATIC; ++k) acc = next4<EXACT>(acc, t.w[k], v[u][k]);
          reinterpret_cast<float4*>(out)[i] = acc;
        }
      }
    } else {
#pragma unroll
      for (int u = 0; u < kK1Unroll; ++u) {
        const int64_t i = i0 + u * kBlock;
        if (i >= n4) break;
        float4 acc;
        int k = 0;
        if constexpr (CONT) {
          acc = reinterpret_cast<const float4*>(out)[i];
        } else {
          acc = first4<EXACT>(t.w[0], ld_stream(t.x[0], i));
          k = 1;
        }
        for (; k < m; k += 8) {
          float4 v[8];
          const int kn = min(8, m - k);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < kn) v[j] = ld_stream(t.x[k + j], i);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < kn) acc = next4<EXACT>(acc, t.w[k + j], v[j]);
        }
        reinterpret_cast<float4*>(out)[i] = acc;
      }
    }
  }
}

// Scalar form: unaligned pointers and the n % 4 tail.
template <bool EXACT, bool CONT>
__global__ __launch_bounds__(kBlock) void k_agg_f32_scalar(OpTableF32 t, int m, float* out,
                                                           int64_t e0, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = e0 + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n;
       e += stride) {
    float acc;
    int k = 0;
    if constexpr (CONT) {
      acc = out[e];
    } else {
      acc = first_term<EXACT>(t.w[0], t.x[0][e]);
      k = 1;
    }
    for (; k < m; ++k) acc = next_term<EXACT>(acc, t.w[k], t.x[k][e]);
    out[e] = acc;
  }
}

// int64 buffers (num_batches_tracked): every operand converted to fp32 (round to nearest,
// as torch's type promotion does), fp32 multiply-add chain, truncation on the store.
// Single pass: all M <= kMaxOps operands are in the table, so `out` may alias any of them.
__global__ __launch_bounds__(kBlock) void k_agg_i64(OpTableI64 t, int m, int64_t* out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
    float acc = __fmul_rn(t.w[0], static_cast<float>(t.x[0][e]));
    for (int k = 1; k < m; ++k)
      acc = __fadd_rn(acc, __fmul_rn(t.w[k], static_cast<float>(t.x[k][e])));
    out[e] = trunc_i64(acc);
  }
}

// K1m: one call over a whole model in ONE launch - the fp32 segment in float4 chunks, then (last
// block) its n % 4 tail and the int64 segment (the ~50 num_batches_tracked counters of a
// ResNet): the per-call path's three launches (vector, tail, int64) become one.  m <= kModelOps
// operands, 16-B aligned fp32 segments; the same element arithmetic as k_agg_f32_vec /
// k_agg_f32_scalar / k_agg_i64, so the result is theirs bit for bit.
constexpr int kModelOps = 64;
constexpr int kModelI64Max = 1 << 16;  // int64 elements the last block takes (else two launches)

struct OpTableModel {
  const float* x[kModelOps];
  const int64_t* xi[kModelOps];
  float w[kModelOps];
};

template <int M_STATIC, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_agg_model(OpTableModel t, int m_rt, float* out, int64_t n,
                                                      int64_t* out_i, int64_t n_i) {
  const int m = M_STATIC > 0 ? M_STATIC : m_rt;
  const int64_t n4 = n / 4;
  {
    // float4 chunks, one per lane (the last block's lanes past n4 go straight to the scalar work)
    const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i < n4) {
      if constexpr (M_STATIC > 0) {
        float4 v[M_STATIC];
#pragma unroll
        for (int k = 0; k < M_STATIC; ++k) v[k] = ld_stream(t.x[k], i);
        float4 acc = first4<EXACT>(t.w[0], v[0]);
#pragma unroll
        for (int k = 1; k < M_STATIC; ++k) acc = next4<EXACT>(acc, t.w[k], v[k]);
        reinterpret_cast<float4*>(out)[i] = acc;  // plain store: 0.154 ms vs 0.158 non-temporal (r03x)
      } else {
        float4 acc = first4<EXACT>(t.w[0], ld_stream(t.x[0], i));
        for (int k = 1; k < m; k += 8) {
          float4 v[8];
          const int kn = min(8, m - k);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < kn) v[j] = ld_stream(t.x[k + j], i);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (j < kn) acc = next4<EXACT>(acc, t.w[k + j], v[j]);
        }
        reinterpret_cast<float4*>(out)[i] = acc;
      }
    }
    if (blockIdx.x + 1 < gridDim.x) return;
  }
  // last block: the fp32 tail (< 4 elements) and the int64 segment, one element per lane
  const int64_t tail = n - 4 * n4;
  for (int64_t e = threadIdx.x; e < tail + n_i; e += kBlock) {
    if (e < tail) {
      const int64_t q = 4 * n4 + e;
      float acc = first_term<EXACT>(t.w[0], t.x[0][q]);
      for (int k = 1; k < m; ++k) acc = next_term<EXACT>(acc, t.w[k], t.x[k][q]);
      out[q] = acc;
    } else {
      const int64_t q = e - tail;
      float acc = __fmul_rn(t.w[0], static_cast<float>(t.xi[0][q]));
      for (int k = 1; k < m; ++k) acc = __fadd_rn(acc, __fmul_rn(t.w[k], static_cast<float>(t.xi[k][q])));
      out_i[q] = trunc_i64(acc);
    }
  }
}

int grid_for(int64_t work) {
  int64_t b = (work + kBlock - 1) / kBlock;
  if (b < 1) b = 1;
  if (b > kMaxGrid) b = kMaxGrid;
  return static_cast<int>(b);
}

template <bool EXACT, bool CONT>
void launch_vec(const OpTableF32& t, int m, float* out, int64_t n4, hipStream_t s) {
  int64_t nb = (n4 + kBlock * kK1Unroll - 1) / (kBlock * kK1Unroll);
  nb = std::max<int64_t>(1, std::min<int64_t>(nb, kK1Grid));
  const dim3 g(static_cast<unsigned>(nb)), b(kBlock);
#define TAL_VEC_CASE(MM) \
  case MM:               \
    k_agg_f32_vec<MM, EXACT, CONT><<<g, b, 0, s>>>(t, m, out, n4); \
    return;
  switch (m) {
    TAL_VEC_CASE(1) TAL_VEC_CASE(2) TAL_VEC_CASE(3) TAL_VEC_CASE(4) TAL_VEC_CASE(5)
    TAL_VEC_CASE(6) TAL_VEC_CASE(7) TAL_VEC_CASE(8) TAL_VEC_CASE(9) TAL_VEC_CASE(10)
    TAL_VEC_CASE(11) TAL_VEC_CASE(12) TAL_VEC_CASE(13) TAL_VEC_CASE(14) TAL_VEC_CASE(15)
    TAL_VEC_CASE(16) TAL_VEC_CASE(17)
    default:
      k_agg_f32_vec<0, EXACT, CONT><<<g, b, 0, s>>>(t, m, out, n4);
  }
#undef TAL_VEC_CASE
}

template <bool EXACT, bool CONT>
void launch_scalar(const OpTableF32& t, int m, float* out, int64_t e0, int64_t n, hipStream_t s) {
  if (n <= e0) return;
  k_agg_f32_scalar<EXACT, CONT><<<grid_for(n - e0), kBlock, 0, s>>>(t, m, out, e0, n);
}

template <bool EXACT>
void launch_pass(const OpTableF32& t, int m, bool cont, bool vec, float* out, int64_t n,
                 hipStream_t s) {
  const int64_t n4 = vec ? n / 4 : 0;
  if (cont) {
    if (n4) launch_vec<EXACT, true>(t, m, out, n4, s);
    launch_scalar<EXACT, true>(t, m, out, n4 * 4, n, s);
  } else {
    if (n4) launch_vec<EXACT, false>(t, m, out, n4, s);
    launch_scalar<EXACT, false>(t, m, out, n4 * 4, n, s);
  }
}

// ------------------------------------------------------------------------------------------
// K3: whole-round aggregation over a device pool, LDS-tiled.
//   grid = (column tiles, row groups).  A workgroup stages tile c (C4 float4 per source) of
//   every distinct source of its group into LDS (one HBM read per source per tile, however
//   many rows of the group use it), plus the group's slice of the plan; after one barrier
//   each wavefront walks rows and emits out[row][tile c] with the operands in reference order.
//   HBM traffic per tile = (sources + rows) * C4 * 16 B instead of (nnz + rows) * C4 * 16 B.
// ------------------------------------------------------------------------------------------
struct PlanView {
  const int32_t* grp_row_ptr;
  const int32_t* grp_src_ptr;
  const int32_t* src_row;
  const int32_t* row_ptr;
  const int32_t* op_slot;
  const float* op_w;
  const int32_t* out_row;
  const int32_t* grp_blk_ptr;  // dense form only
  const int32_t* blk_tab;
  const int32_t* base;         // the blob (dense tables are addressed from it)
  const int32_t* nrow_ptr;     // narrow form only
  const int32_t* npairs;
  const int32_t* nrow_w;       // narrow_roww only
  const int32_t* bc_prog;      // narrow_bcast only: [n_groups * waves] word offset of each wave's program
};

PlanView make_view(const int32_t* plan, const tal_round_plan_info& in) {
  PlanView v;
  v.grp_row_ptr = plan + in.off_grp_row_ptr;
  v.grp_src_ptr = plan + in.off_grp_src_ptr;
  v.src_row = plan + in.off_src_row;
  v.row_ptr = plan + in.off_row_ptr;
  v.op_slot = plan + in.off_op_slot;
  v.op_w = reinterpret_cast<const float*>(plan + in.off_op_w);
  v.out_row = plan + in.off_out_row;
  v.grp_blk_ptr = plan + in.off_grp_blk_ptr;
  v.blk_tab = plan + in.off_blk_tab;
  v.base = plan;
  v.nrow_ptr = plan + in.off_nrow_ptr;
  v.npairs = plan + in.off_npairs;
  v.nrow_w = plan + in.off_nrow_w;
  v.bc_prog = plan + in.off_bc_prog;
  return v;
}

// LDS carve of one workgroup (both float4 kernels and the scalar one):
//   [max_src * tile data][row_ptr (rows+1)][slot (nnz)][w (nnz)][src_row (ns)][out_row (rows)]
struct GroupLds {
  int32_t* rowptr;
  int32_t* slot;
  float* w;
  int32_t* src;
  int32_t* out;
  int ns, nr, s_beg, r_beg;
};

// Stage group g's plan slice into LDS (slots pre-multiplied by the tile width).
__device__ __forceinline__ GroupLds stage_group(const PlanView& p, int g, void* lds_tail, int tile,
                                                int nthreads) {
  GroupLds L;
  L.s_beg = p.grp_src_ptr[g];
  L.ns = p.grp_src_ptr[g + 1] - L.s_beg;
  L.r_beg = p.grp_row_ptr[g];
  L.nr = p.grp_row_ptr[g + 1] - L.r_beg;
  const int o_beg = p.row_ptr[L.r_beg];
  const int no = p.row_ptr[L.r_beg + L.nr] - o_beg;
  L.rowptr = static_cast<int32_t*>(lds_tail);
  L.slot = L.rowptr + (L.nr + 1);
  L.w = reinterpret_cast<float*>(L.slot + no);
  L.src = reinterpret_cast<int32_t*>(L.w + no);
  L.out = L.src + L.ns;
  for (int k = threadIdx.x; k <= L.nr; k += nthreads) L.rowptr[k] = p.row_ptr[L.r_beg + k] - o_beg;
  for (int k = threadIdx.x; k < no; k += nthreads) {
    L.slot[k] = p.op_slot[o_beg + k] * tile;
    L.w[k] = p.op_w[o_beg + k];
  }
  for (int k = threadIdx.x; k < L.ns; k += nthreads) L.src[k] = p.src_row[L.s_beg + k];
  for (int k = threadIdx.x; k < L.nr; k += nthreads) L.out[k] = p.out_row[L.r_beg + k];
  return L;
}

__device__ __forceinline__ void st_stream(float* base, int64_t i, float4 v) {
  const v4f q = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(base) + i);
}

// ------------------------------------------------------------------------------------------
// Storage types: fp32 (float) and bf16 (uint16_t bit patterns).  Kernels index pools in chunks
// of 4 elements (16 B fp32, 8 B bf16) and always compute in fp32.  Element k of a 32-bit bf16
// word is its low half for k = 0 (little endian).
// ------------------------------------------------------------------------------------------
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }

// fp32 pair -> bf16 pair, round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t cvt_bf16x2(float a, float b) {
  bf16x2_t r;
  r.x = static_cast<__bf16>(a);
  r.y = static_cast<__bf16>(b);
  return __builtin_bit_cast(uint32_t, r);
}

// The stored form: NaN becomes 0xFFFF, as torch's vectorized CPU fp32 -> bf16 conversion writes
// it (the reference aggregates tensors, never single elements); NaN inputs stay NaN through the
// intermediate roundings, so only the store canonicalises.
__device__ __forceinline__ uint32_t store_bf16x2(float a, float b) {
  uint32_t u = cvt_bf16x2(a, b);
  if (a != a) u |= 0x0000ffffu;
  if (b != b) u |= 0xffff0000u;
  return u;
}

// fp32 -> nearest-even bf16, kept as the fp32 it represents: one v_cvt_pk_bf16_f32 with the value
// in the HIGH half and +0.0 in the low half is that fp32 word as it stands (no shift or mask to
// unpack; a pair conversion plus unpacking costs 1.5 instructions per element instead of 1)
// (inline asm: in C++ the compiler merges two such conversions into one pair conversion plus two
// v_perm_b32, the 1.5 instructions per element this avoids)
__device__ __forceinline__ float round_bf16(float a) {
  float r;
  asm("v_cvt_pk_bf16_f32 %0, 0, %1" : "=v"(r) : "v"(a));
  return r;
}

__device__ __forceinline__ float4 round_bf16x4(float4 v) {
  return make_float4(round_bf16(v.x), round_bf16(v.y), round_bf16(v.z), round_bf16(v.w));
}

// bf16 EXACT steps on two-element vectors, so the multiplies and adds are packed (v_pk_mul_f32,
// v_pk_add_f32; IEEE, -ffp-contract=off) around the per-element roundings
typedef float bf_v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf_v2f round_bf16x2(bf_v2f a) { return bf_v2f{round_bf16(a.x), round_bf16(a.y)}; }

__device__ __forceinline__ float4 bf16x_first4(float w, float4 x) {
  const bf_v2f ww = {w, w};
  const bf_v2f p0 = round_bf16x2(ww * bf_v2f{x.x, x.y}), p1 = round_bf16x2(ww * bf_v2f{x.z, x.w});
  return make_float4(p0.x, p0.y, p1.x, p1.y);
}

__device__ __forceinline__ float4 bf16x_next4(float4 a, float w, float4 x) {
  const bf_v2f ww = {w, w};
  const bf_v2f p0 = round_bf16x2(ww * bf_v2f{x.x, x.y}), p1 = round_bf16x2(ww * bf_v2f{x.z, x.w});
  const bf_v2f s0 = round_bf16x2(bf_v2f{a.x, a.y} + p0), s1 = round_bf16x2(bf_v2f{a.z, a.w} + p1);
  return make_float4(s0.x, s0.y, s1.x, s1.y);
}

template <typename T>
struct Io;

template <>
struct Io<float> {
  typedef float4 raw_t;  // a staged chunk as loaded (converted when written to LDS)
  static __device__ __forceinline__ float4 ld(const float* b, int64_t i4) { return ld_stream(b, i4); }
  static __device__ __forceinline__ raw_t ld_raw(const float* b, int64_t i4) { return ld_stream(b, i4); }
  static __device__ __forceinline__ float4 f4(raw_t r) { return r; }
  static __device__ __forceinline__ void st(float* b, int64_t i4, float4 v) { st_stream(b, i4, v); }
  static __device__ __forceinline__ float ld1(const float* b, int64_t e) { return b[e]; }
  static __device__ __forceinline__ void st1(float* b, int64_t e, float v) { b[e] = v; }
};

template <>
struct Io<uint16_t> {
  typedef u32x2 raw_t;
  static __device__ __forceinline__ float4 ld(const uint16_t* b, int64_t i4) { return f4(ld_raw(b, i4)); }
  static __device__ __forceinline__ raw_t ld_raw(const uint16_t* b, int64_t i4) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(b) + i4);
  }
  static __device__ __forceinline__ float4 f4(raw_t q) {
    return make_float4(bf16_lo(q.x), bf16_hi(q.x), bf16_lo(q.y), bf16_hi(q.y));
  }
  static __device__ __forceinline__ u32x2 pack(float4 v) {
    u32x2 q = {cvt_bf16x2(v.x, v.y), cvt_bf16x2(v.z, v.w)};
    // NaN canonicalisation (store_bf16x2) only where a lane holds one: two unordered compares
    // on the common path instead of four compare-and-selects
    if (__builtin_isunordered(v.x, v.y) || __builtin_isunordered(v.z, v.w)) {
      q.x = store_bf16x2(v.x, v.y);
      q.y = store_bf16x2(v.z, v.w);
    }
    return q;
  }
  static __device__ __forceinline__ void st(uint16_t* b, int64_t i4, float4 v) {
    __builtin_nontemporal_store(pack(v), reinterpret_cast<u32x2*>(b) + i4);
  }
  static __device__ __forceinline__ float ld1(const uint16_t* b, int64_t e) {
    return __uint_as_float(static_cast<uint32_t>(b[e]) << 16);
  }
  static __device__ __forceinline__ void st1(uint16_t* b, int64_t e, float v) {
    b[e] = static_cast<uint16_t>(store_bf16x2(v, 0.f) & 0xffffu);
  }
};

template <typename T>
constexpr bool kIsBf16 = std::is_same<T, uint16_t>::value;

// Arithmetic per storage type.  fp32: first4 / next4.  bf16 EXACT: the reference's own ops on
// bf16 tensors (decentralized_client.py:407-411: `w * clone(v)` and `+=` each round their fp32
// result to bf16).  bf16 FMA: fp32 accumulation (fused), rounded once by the store.
template <typename T, bool EXACT>
__device__ __forceinline__ float4 first4t(float w, float4 x) {
  if constexpr (kIsBf16<T> && EXACT) return bf16x_first4(w, x);
  else return first4<EXACT>(w, x);
}

template <typename T, bool EXACT>
__device__ __forceinline__ float4 next4t(float4 a, float w, float4 x) {
  if constexpr (kIsBf16<T> && EXACT) return bf16x_next4(a, w, x);
  else return next4<EXACT>(a, w, x);
}

template <typename T, bool EXACT>
__device__ __forceinline__ float first1t(float w, float x) {
  if constexpr (kIsBf16<T> && EXACT) return round_bf16(__fmul_rn(w, x));
  else return first_term<EXACT>(w, x);
}

template <typename T, bool EXACT>
__device__ __forceinline__ float next1t(float a, float w, float x) {
  if constexpr (kIsBf16<T> && EXACT) return round_bf16(__fadd_rn(a, round_bf16(__fmul_rn(w, x))));
  else return next_term<EXACT>(a, w, x);
}

// K1 on bf16 buffers: one call, chunks of 4 elements (8 B) per lane, operand loads in batches of
// 8 ahead of the ordered accumulate.  All m <= kMaxOps operands are in the table (one pass), so
// `out` may alias any of them.
struct OpTableB16 {
  const uint16_t* x[kMaxOps];
  float w[kMaxOps];
};

template <bool EXACT>
__global__ __launch_bounds__(kBlock) void k_agg_b16_vec(OpTableB16 t, int m, uint16_t* out, int64_t n4) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock * kK1Unroll;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kBlock * kK1Unroll + threadIdx.x; i0 < n4;
       i0 += stride) {
#pragma unroll
    for (int u = 0; u < kK1Unroll; ++u) {
      const int64_t i = i0 + u * kBlock;
      if (i >= n4) break;
      float4 acc = first4t<uint16_t, EXACT>(t.w[0], Io<uint16_t>::ld(t.x[0], i));
      for (int k = 1; k < m; k += 8) {
        float4 v[8];
        const int kn = min(8, m - k);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < kn) v[j] = Io<uint16_t>::ld(t.x[k + j], i);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < kn) acc = next4t<uint16_t, EXACT>(acc, t.w[k + j], v[j]);
      }
      Io<uint16_t>::st(out, i, acc);
    }
  }
}

// unaligned operands and the n % 4 tail
template <bool EXACT>
__global__ __launch_bounds__(kBlock) void k_agg_b16_scalar(OpTableB16 t, int m, uint16_t* out, int64_t e0,
                                                           int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = e0 + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
    float acc = first1t<uint16_t, EXACT>(t.w[0], Io<uint16_t>::ld1(t.x[0], e));
    for (int k = 1; k < m; ++k) acc = next1t<uint16_t, EXACT>(acc, t.w[k], Io<uint16_t>::ld1(t.x[k], e));
    Io<uint16_t>::st1(out, e, acc);
  }
}

// K1 past kMaxOps operands for bf16 and int64 buffers: the ordered chain over m operands runs
// in passes of up to kMaxOps (one kernel-argument table each), the running sum kept in an fp32
// scratch between passes - exactly the register value the one-pass kernels carry (bf16 EXACT:
// a bf16 value; FMA and int64: the unrounded fp32 sum) - and stored to `out` (rounded /
// truncated) only by the last pass, so `out` may alias any operand.  One element per thread.
template <typename T>
struct OpTableT {
  const T* x[kMaxOps];
  float w[kMaxOps];
};

template <typename T, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_agg_chain(OpTableT<T> t, int m, bool first, bool last, float* acc,
                                                      T* out, int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n; e += stride) {
    float a;
    int k0 = 0;
    if constexpr (std::is_same<T, int64_t>::value) {
      if (first) { a = __fmul_rn(t.w[0], static_cast<float>(t.x[0][e])); k0 = 1; } else { a = acc[e]; }
      for (int k = k0; k < m; ++k) a = __fadd_rn(a, __fmul_rn(t.w[k], static_cast<float>(t.x[k][e])));
      if (last) out[e] = trunc_i64(a); else acc[e] = a;
    } else {
      if (first) { a = first1t<T, EXACT>(t.w[0], Io<T>::ld1(t.x[0], e)); k0 = 1; } else { a = acc[e]; }
      for (int k = k0; k < m; ++k) a = next1t<T, EXACT>(a, t.w[k], Io<T>::ld1(t.x[k], e));
      if (last) Io<T>::st1(out, e, a); else acc[e] = a;
    }
  }
}

// Host side of k_agg_chain: m > kMaxOps operands, an fp32 scratch of n elements allocated and
// freed in stream order (nothing persistent).
template <typename T, bool EXACT>
int32_t agg_chain(const T* const* x_host, const double* w_host, int32_t m, T* out, int64_t n, hipStream_t s,
                  const char* who) {
  float* acc = nullptr;
  if (hipMallocAsync(reinterpret_cast<void**>(&acc), static_cast<size_t>(n) * sizeof(float), s) != hipSuccess)
    return fail(TAL_ERR_HIP, std::string(who) + ": scratch allocation failed");
  for (int base = 0; base < m; base += kMaxOps) {
    OpTableT<T> t;
    const int cnt = std::min(kMaxOps, m - base);
    for (int i = 0; i < cnt; ++i) {
      t.x[i] = x_host[base + i];
      t.w[i] = static_cast<float>(w_host[base + i]);
    }
    for (int i = cnt; i < kMaxOps; ++i) { t.x[i] = nullptr; t.w[i] = 0.f; }
    k_agg_chain<T, EXACT><<<grid_for(n), kBlock, 0, s>>>(t, cnt, base == 0, base + cnt >= m, acc, out, n);
  }
  const int32_t rc = check_launch(who);
  if (hipFreeAsync(acc, s) != hipSuccess && rc == TAL_OK) return fail(TAL_ERR_HIP, std::string(who) + ": scratch free failed");
  return rc;
}

// Compute one column tile from LDS.  A wavefront owns whole rows (row index wave-uniform, so
// the plan entries — row extent, operand slots and weights — are scalar loads from the plan in
// global memory, served by the scalar cache); each lane owns C4/64 float4 columns.  Operands are
// consumed in reference order, four LDS reads in flight ahead of the ordered accumulate.
// The plan is read-only for the whole launch: reading it through the constant address space
// lets the backend use scalar (SMEM) loads for the wave-uniform entries.
typedef __attribute__((address_space(4))) const int32_t* ConstI32;
typedef __attribute__((address_space(4))) const float* ConstF32;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(4))) const i32x4* ConstI32x4;
typedef __attribute__((address_space(4))) const f32x8* ConstF32x8;

template <int C4, int NT, bool EXACT, typename T = float>
__device__ __forceinline__ void emit_tile(const float4* s_data, const PlanView& p, int r_beg, int nr,
                                          T* pout, int64_t ld_out4, int64_t c0, int64_t n4) {
  constexpr int kB = C4 >= 128 ? 8 : 4;  // operands per batch (LDS reads in flight per lane)
  static_assert(C4 % 64 == 0, "a wavefront covers 64 float4 columns");
  constexpr int kWaves = NT / 64;
  constexpr int kCpl = C4 / 64;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const ConstI32 row_ptr = (ConstI32)p.row_ptr;
  const ConstI32 out_row = (ConstI32)p.out_row;
  const ConstI32 op_slot = (ConstI32)p.op_slot;
  const ConstF32 op_w = (ConstF32)p.op_w;
  for (int r = wave; r < nr; r += kWaves) {
    const int gr = r_beg + r;
    const int q0 = row_ptr[gr];
    const int q1 = row_ptr[gr + 1];
    const int64_t orow = out_row[gr];
    float4 acc[kCpl];
    {
      const float w = op_w[q0];
      const int sl = op_slot[q0] * C4 + lane;
#pragma unroll
      for (int j = 0; j < kCpl; ++j) acc[j] = first4t<T, EXACT>(w, s_data[sl + 64 * j]);
    }
    int q = q0 + 1;
    for (; q + kB <= q1; q += kB) {
      float w[kB];
      int sl[kB];
      float4 x[kB][kCpl];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        w[u] = op_w[q + u];
        sl[u] = op_slot[q + u] * C4 + lane;
      }
#pragma unroll
      for (int u = 0; u < kB; ++u)
#pragma unroll
        for (int j = 0; j < kCpl; ++j) x[u][j] = s_data[sl[u] + 64 * j];
#pragma unroll
      for (int u = 0; u < kB; ++u)
#pragma unroll
        for (int j = 0; j < kCpl; ++j) acc[j] = next4t<T, EXACT>(acc[j], w[u], x[u][j]);
    }
    for (; q < q1; ++q) {
      const float w = op_w[q];
      const int sl = op_slot[q] * C4 + lane;
#pragma unroll
      for (int j = 0; j < kCpl; ++j) acc[j] = next4t<T, EXACT>(acc[j], w, s_data[sl + 64 * j]);
    }
#pragma unroll
    for (int j = 0; j < kCpl; ++j) {
      const int64_t col = c0 + lane + 64 * j;
      if (col < n4) Io<T>::st(pout, orow * ld_out4 + col, acc[j]);
    }
  }
}

// Dense form: a wavefront owns a block of RB rows and walks, once, the staged sources any of
// them uses (ascending); each source's LDS read serves every row of the block that uses it (row
// mask), so a row's operands are still consumed in its reference order (sorted neighbors), and
// the row's own model — the reference's last operand — is added last.  Accumulators start at
// -0.0f: -0 + fl(w*x) == fl(w*x) exactly for every x, so the first term needs no special case
// and the result is bit-identical.  Sources are walked four at a time (their LDS reads in flight
// together); masks, slots and weights are wave-uniform scalar loads.
// Block table (32-B aligned): {n_used, 7 pad words, slot[n_used], mask[n_used], w[n_used][RB]},
// n_used padded to a multiple of 4 with mask-0 entries so every vector load is aligned.
template <int C4, int NT, int RB, bool EXACT>
__device__ __forceinline__ void emit_tile_dense(const float4* s_data, const PlanView& p, int g, int r_beg,
                                                int nr, int ns, float* pout, int64_t ld_out4,
                                                int64_t c0, int64_t n4) {
  constexpr int kWaves = NT / 64;
  constexpr int kCpl = C4 / 64;
  constexpr int kU = 4;
  static_assert(RB == 8, "weights are loaded as 8-wide vectors");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const ConstI32 row_ptr = (ConstI32)p.row_ptr;
  const ConstI32 out_row = (ConstI32)p.out_row;
  const ConstI32 op_slot = (ConstI32)p.op_slot;
  const ConstF32 op_w = (ConstF32)p.op_w;
  const ConstI32 base = (ConstI32)p.base;
  const int blk0 = ((ConstI32)p.grp_blk_ptr)[g];
  const int nblk = (nr + RB - 1) / RB;
  for (int lb = wave; lb < nblk; lb += kWaves) {
    const ConstI32 tab = base + ((ConstI32)p.blk_tab)[blk0 + lb];
    const int rows_here = min(RB, nr - lb * RB);
    const int n_used = tab[0];                        // multiple of kU
    const ConstI32x4 slots4 = (ConstI32x4)(tab + 8);    // 32-B aligned (see the builder)
    const ConstI32x4 masks4 = (ConstI32x4)(tab + 8 + n_used);
    const ConstF32x8 wts8 = (ConstF32x8)(tab + 8 + 2 * n_used);
    float4 acc[RB][kCpl];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int j = 0; j < kCpl; ++j) acc[r][j] = make_float4(-0.f, -0.f, -0.f, -0.f);
    for (int e = 0; e < n_used; e += kU) {
      const i32x4 sl = slots4[e / kU];                 // s_load_dwordx4
      const i32x4 mk = masks4[e / kU];
      float4 x[kU][kCpl];
#pragma unroll
      for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int j = 0; j < kCpl; ++j) x[u][j] = s_data[sl[u] * C4 + lane + 64 * j];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const f32x8 wv = wts8[e + u];                   // s_load_dwordx8
        const uint32_t m = static_cast<uint32_t>(mk[u]);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          if (m & (1u << r)) {
#pragma unroll
            for (int j = 0; j < kCpl; ++j) acc[r][j] = next4<EXACT>(acc[r][j], wv[r], x[u][j]);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      if (r < rows_here) {
        const int gr = r_beg + lb * RB + r;
        const int q = row_ptr[gr + 1] - 1;  // the row's own model, last in reference order
        const float w = op_w[q];
        const int sl = op_slot[q] * C4 + lane;
        const int64_t orow = out_row[gr];
#pragma unroll
        for (int j = 0; j < kCpl; ++j) {
          acc[r][j] = next4<EXACT>(acc[r][j], w, s_data[sl + 64 * j]);
          const int64_t col = c0 + lane + 64 * j;
          if (col < n4) st_stream(pout, orow * ld_out4 + col, acc[r][j]);
        }
      }
    }
  }
}

constexpr int kDenseRb = 8;
constexpr int kStreamDepth = 3;        // chunks in flight ahead of the one being read
constexpr int kStreamPerWave = 2;      // sources each wavefront moves per chunk (1 KiB DMA each)
constexpr int kStreamMaxRows = 128;    // 16 wavefronts x one 8-row block
constexpr size_t stream_lds_bytes(int cs) { return static_cast<size_t>(kStreamDepth + 1) * cs * 64 * 16; }

// Persistent form (the fast path): each workgroup walks column tiles t, t+gridDim.x, ...;
// every lane owns J fixed staging slots (source, column) and keeps the next tile's J float4
// loads in flight in registers while the workgroup computes the current tile from LDS.
template <int C4, int NT, int J, bool EXACT, bool DENSE, typename T = float>
__global__ __launch_bounds__(NT) void k_round_f32_persistent(const T* __restrict__ pin,
                                                             int64_t ld_in4,
                                                             T* __restrict__ pout,
                                                             int64_t ld_out4, int64_t n4,
                                                             PlanView p, int64_t n_tiles) {
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const int s_beg = p.grp_src_ptr[g];
  const int ns = p.grp_src_ptr[g + 1] - s_beg;
  const int r_beg = p.grp_row_ptr[g];
  const int nr = p.grp_row_ptr[g + 1] - r_beg;
  // lane-fixed staging slots: slot k = j*NT + tid holds column c = tid % C4 (NT is a multiple
  // of C4) of staged source k / C4; only the source's pool row is kept per slot (-1 = unused)
  static_assert(NT % C4 == 0, "a block stages whole source tiles");
  constexpr int kLd = J, kLps = C4;  // staging as k_round_f32_narrow without its 16-B bf16 lanes
  // Branch-free staging (see k_round_f32_narrow): a slot past the group's sources reloads source
  // 0's chunk of its column and writes it where source 0's own slot does (the same value).
  // The write index and (dense form, whose registers are tight) the load addresses are recomputed
  // per tile behind an empty asm, so the compiler does not hoist them into more registers.
  const int c = threadIdx.x % C4;
  int srow[kLd];
#pragma unroll
  for (int j = 0; j < kLd; ++j) {
    const int src = (j * NT + threadIdx.x) / kLps;
    srow[j] = p.src_row[s_beg + (src < ns ? src : 0)];
  }
  typename Io<T>::raw_t v[J];
  auto load_tile = [&](int64_t tt) {
    const int64_t col = min(tt * C4 + c, n4 - 1);  // past the end: a duplicate (cache hit)
#pragma unroll
    for (int j = 0; j < J; ++j) {
      int r = srow[j];
      if constexpr (DENSE) asm volatile("" : "+v"(r));
      v[j] = Io<T>::ld_raw(pin, static_cast<int64_t>(r) * ld_in4 + col);
    }
  };
  int64_t t = blockIdx.x;
  if (t < n_tiles) load_tile(t);
  for (; t < n_tiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's readers are done with s_data
    int staged = ns * kLps;  // staging units (float4 slots) of real sources
    asm volatile("" : "+s"(staged));
#pragma unroll
    for (int j = 0; j < kLd; ++j) {
      const int k = j * NT + static_cast<int>(threadIdx.x);
      s_data[k < staged ? k : c] = Io<T>::f4(v[j]);
    }
    __syncthreads();
    if (t + gridDim.x < n_tiles) load_tile(t + gridDim.x);  // in flight during this tile's math
    if constexpr (DENSE)
      emit_tile_dense<C4, NT, kDenseRb, EXACT>(s_data, p, g, r_beg, nr, ns, pout, ld_out4, t * C4, n4);
    else
      emit_tile<C4, NT, EXACT, T>(s_data, p, r_beg, nr, pout, ld_out4, t * C4, n4);
  }
}

// Narrow-tile persistent form (C4 = 16 or 32 float4 = 256 or 512 B per source per tile): groups
// of up to 256 (C4 = 16) or 128 (C4 = 32) sources fit one LDS tile, so a whole community graph
// is one group and every source is read from HBM once per round.  A wavefront computes
// 64 / C4 rows at once (lanes [k*C4, (k+1)*C4) own row k of the set); the rows' operand counts
// differ, so the plan is per lane: the group's (slot, weight) pairs and row extents are staged in
// LDS once per workgroup, after the data tile and a tile of -0.0 in slot max_src that the
// padding pairs read (see tal_round_plan_info: every row's operands after the first come in
// whole batches of four).  Each wavefront computes the same rows for every tile, so its first
// kNarrowPasses row sets (extents, output rows) live in registers; within a row the next
// batch's pairs are read while the current batch's data reads are in flight.
constexpr int kNarrowPasses = 4;

struct NarrowLds {
  const int32_t* rowptr;  // [nr + 1], group-relative pair index (pairs form)
  const int2* pairs;      // [group pairs + 4 read-ahead] (slot * C4, fp32 weight bits)
  const int32_t* out;     // [nr] pool_out row (pairs form)
  uint32_t rec;           // ROWW: LDS byte address of the row records (16 B each, see below)
  int nr;
};

__host__ __device__ constexpr size_t narrow_lds_bytes(int64_t max_src, int64_t max_rows, int64_t max_pairs,
                                                      int c4) {
  return static_cast<size_t>((max_src + 1) * c4 * 16 + (2 * max_rows + 2 + 2 * (max_pairs + 4)) * 4 + 16);
}

// ROWW (row-uniform weights) carve: [ns + 2 tiles (-0.0, +0.0)][records][slots + 8 read-ahead].
// The rows of a pass (kRpw = 64 / c4 consecutive plan rows, one per lane group of a wavefront)
// are padded on the host to one batch count, so the row loop's trip count is wave-uniform and
// runs on the scalar unit; one 16-B record per row (rows padded to whole passes; a padding row
// reads its pass's first row and stores nothing): {LDS byte address of the row's first slot
// word, batches of four slots, fp32 weight bits, pool_out row or -1}.
__host__ __device__ constexpr int64_t narrow_roww_records(int64_t nr, int c4) {
  return (nr + 64 / c4 - 1) / (64 / c4) * (64 / c4);
}
__host__ __device__ constexpr size_t narrow_roww_lds_bytes(int64_t ns, int64_t nr, int64_t nslots, int c4) {
  return static_cast<size_t>((ns + 2) * c4 * 16 + narrow_roww_records(nr, c4) * 16 + (nslots + 8) * 2 + 16);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)p));
}

template <int C4>
__device__ __forceinline__ NarrowLds stage_narrow_roww(const PlanView& p, int g, float4* s_data, int nthreads) {
  NarrowLds L;
  const int r_beg = p.grp_row_ptr[g];
  L.nr = p.grp_row_ptr[g + 1] - r_beg;
  const int e_beg = p.nrow_ptr[r_beg];  // a multiple of 4 (every run is)
  const int ne = p.nrow_ptr[r_beg + L.nr] - e_beg;
  const int ns = p.grp_src_ptr[g + 1] - p.grp_src_ptr[g];
  constexpr int kRpw = 64 / C4;
  const int nrec = static_cast<int>(narrow_roww_records(L.nr, C4));
  // offsets in 32-bit words from s_data (index arithmetic keeps the LDS address space: a
  // pointer rebuilt from an integer would become a generic one and every read a flat load)
  int32_t* base32 = reinterpret_cast<int32_t*>(s_data);
  int32_t* rec = base32 + (ns + 2) * C4 * 4;
  uint32_t* slots = reinterpret_cast<uint32_t*>(rec + 4 * nrec);
  const uint32_t slots_addr = lds_addr(slots);
  for (int k = threadIdx.x; k < 2 * C4; k += nthreads)  // zero tiles: slot ns = -0.0, ns + 1 = +0.0
    s_data[static_cast<size_t>(ns) * C4 + k] = k < C4 ? make_float4(-0.f, -0.f, -0.f, -0.f)
                                                      : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int k = threadIdx.x; k < nrec; k += nthreads) {
    const int row = k < L.nr ? k : k / kRpw * kRpw;  // padding rows: their pass's first row
    const int q0 = p.nrow_ptr[r_beg + row] - e_beg, q1 = p.nrow_ptr[r_beg + row + 1] - e_beg;
    rec[4 * k + 0] = static_cast<int32_t>(slots_addr + 2u * static_cast<uint32_t>(q0));
    // operands the pass computes: its first (longest) row's count, as whole batches of four
    // plus a tail of 1-3; the slot storage stays padded to whole batches (8-B aligned reads)
    const int lead = r_beg + k / kRpw * kRpw;
    const int m = p.row_ptr[lead + 1] - p.row_ptr[lead];
    rec[4 * k + 1] = (m / 4) | ((m % 4) << 16);
    (void)q1;
    rec[4 * k + 2] = p.nrow_w[r_beg + row];
    rec[4 * k + 3] = k < L.nr ? p.out_row[r_beg + k] : -1;
  }
  const int nw = ne / 2;  // ne is a multiple of 4: whole words
  for (int k = threadIdx.x; k < nw + 4; k += nthreads)  // + 4 read-ahead words (never used)
    slots[k] = k < nw ? static_cast<uint32_t>(p.npairs[e_beg / 2 + k]) : 0u;
  L.rowptr = nullptr;
  L.pairs = nullptr;
  L.out = nullptr;
  L.rec = lds_addr(rec);
  return L;
}

// LDS byte address of the float4 slot in the low / high 16 bits of `word`, from the lane's
// column base: one v_mad_u32_u16 (op_sel picks the half) instead of an extract and a shift-add.
// gfx950 VOP3 encoding (see the target check at the top); the plain form is
// ((word >> (16 * half)) & 0xffff) * 16 + base, which tests/test_gpu_kernels.py's narrow cases
// check bit for bit against the oracle.
__device__ __forceinline__ uint32_t slot_addr_lo(uint32_t word, uint32_t base) {
  uint32_t a;
  asm("v_mad_u32_u16 %0, %1, 16, %2" : "=v"(a) : "v"(word), "v"(base));
  return a;
}
__device__ __forceinline__ uint32_t slot_addr_hi(uint32_t word, uint32_t base) {
  uint32_t a;
  asm("v_mad_u32_u16 %0, %1, 16, %2 op_sel:[1,0,0,0]" : "=v"(a) : "v"(word), "v"(base));
  return a;
}
__device__ __forceinline__ uint2 lds_u2(uint32_t addr) {
  typedef unsigned int u32x2_lds __attribute__((ext_vector_type(2)));
  const u32x2_lds q = *reinterpret_cast<__attribute__((address_space(3))) const u32x2_lds*>(static_cast<uintptr_t>(addr));
  return make_uint2(q.x, q.y);
}
__device__ __forceinline__ float4 lds_f4(uint32_t addr) {
  const v4f q = *reinterpret_cast<__attribute__((address_space(3))) const v4f*>(static_cast<uintptr_t>(addr));
  return make_float4(q.x, q.y, q.z, q.w);
}

__device__ __forceinline__ uint4 lds_u4(uint32_t addr) {
  typedef unsigned int u32x4_lds __attribute__((ext_vector_type(4)));
  const u32x4_lds q = *reinterpret_cast<__attribute__((address_space(3))) const u32x4_lds*>(static_cast<uintptr_t>(addr));
  return make_uint4(q.x, q.y, q.z, q.w);
}

// One ROWW row from its record: the accumulator starts at -0.0 and takes `nb` batches of four
// slots (one 8-B LDS read each, the next batch's read issued ahead of this batch's data reads),
// then a tail of `rem` < 4 slots from the word read last.  nb and rem are the same for every
// row of the pass (host padding), so the loop counts on the scalar unit: per batch 4 address +
// 16 (EXACT) or 8 (FMA) arithmetic VALU and one cursor add.  (Before the tail, rows padded to
// whole batches of four read 9.6 % zero-tile slots on config 5.)
template <typename T, bool EXACT>
__device__ __forceinline__ float4 narrow_row_tail(float4 acc, float w, uint2 e, uint32_t base, int rem) {
  // one operand at a time (a 1-3 long tail per row; read and use back to back keeps the
  // register budget of two workgroups per CU)
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    if (rem <= u) break;  // wave-uniform
    const uint32_t word = u < 2 ? e.x : e.y;
    uint32_t addr;
    addr = u == 1 ? slot_addr_hi(word, base) : slot_addr_lo(word, base);
    acc = next4t<T, EXACT>(acc, w, lds_f4(addr));
  }
  return acc;
}

template <typename T, bool EXACT>
__device__ __forceinline__ float4 narrow_row_roww(uint4 rc, uint32_t base) {
  const int nb = __builtin_amdgcn_readfirstlane(static_cast<int>(rc.y & 0xffffu));
  const int rem = __builtin_amdgcn_readfirstlane(static_cast<int>(rc.y >> 16));
  const float w = __uint_as_float(rc.z);
  uint32_t q = rc.x;
  float4 acc = make_float4(-0.f, -0.f, -0.f, -0.f);
  uint2 e = lds_u2(q);
  for (int b = 0; b < nb; ++b) {
    float4 x[4];
    x[0] = lds_f4(slot_addr_lo(e.x, base));
    x[1] = lds_f4(slot_addr_hi(e.x, base));
    x[2] = lds_f4(slot_addr_lo(e.y, base));
    x[3] = lds_f4(slot_addr_hi(e.y, base));
    asm("v_add_u32 %0, 8, %0" : "+v"(q));
    e = lds_u2(q);  // next batch (or the read-ahead pad), in flight with this batch's data reads
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = next4t<T, EXACT>(acc, w, x[u]);
    // keep the read-ahead where it is: without this the compiler sinks the next batch's slot
    // read to the loop head and waits on it before the data reads
    asm volatile("" : "+v"(e.x), "+v"(e.y));
  }
  return narrow_row_tail<T, EXACT>(acc, w, e, base, rem);
}

// one 16-B-per-lane global->LDS DMA (K3s): 64 lanes x 16 B, lane-linear from LDS byte address M0
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds_byte_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte_addr)
      : "memory");
}

// s_waitcnt vmcnt(n) lgkmcnt(0) + s_barrier, n wave-uniform (clamped: waiting longer is safe)
__device__ __forceinline__ void wait_vm_barrier(int n) {
#define TAL_WB(k) case k: asm volatile("s_waitcnt vmcnt(" #k ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
  switch (n < 0 ? 0 : (n > 31 ? 31 : n)) {
    TAL_WB(0) TAL_WB(1) TAL_WB(2) TAL_WB(3) TAL_WB(4) TAL_WB(5) TAL_WB(6) TAL_WB(7)
    TAL_WB(8) TAL_WB(9) TAL_WB(10) TAL_WB(11) TAL_WB(12) TAL_WB(13) TAL_WB(14) TAL_WB(15)
    TAL_WB(16) TAL_WB(17) TAL_WB(18) TAL_WB(19) TAL_WB(20) TAL_WB(21) TAL_WB(22) TAL_WB(23)
    TAL_WB(24) TAL_WB(25) TAL_WB(26) TAL_WB(27) TAL_WB(28) TAL_WB(29) TAL_WB(30) TAL_WB(31)
  }
#undef TAL_WB
}

// ---- broadcast form (narrow_bcast, tal_round_plan_build_bcast) ---------------------------
// A wavefront's plan is a program of records held in VGPRs for the whole launch: record lane L
// = {LDS byte offset, fp32 weight bits} of operand 16c + L % 16 of row L / 16 of a pass (4 rows;
// at C4 = 32 each lane computes two chunks, bc2_record).  Operand u reaches the 16 lanes of its
// DPP row (one row of the pass) by `row_newbcast:u`, a VALU move, so the row loop reads only
// data from LDS: no slot or weight read and no LDS round trip between a batch's slot word and
// its data reads (the addresses of a whole record are known when the record is).
constexpr int kBcRecPerWg = 128;  // records per workgroup; a wavefront holds 128 / waves of them
constexpr int kBcHdr = 8;         // program header words

template <int NT>
constexpr int bc_rec_max() { return kBcRecPerWg / (NT / 64); }

// lane U of each 16-lane row, to the row (row_newbcast:U).  As update_dpp with bound_ctrl and
// old = 0 the backend folds it into the consuming v_add_u32 (v_add_u32_dpp: the address costs
// one VALU, as the ROWW form's v_mad_u32_u16); a plain mov_dpp stays a separate v_mov_b32_dpp.
template <int U>
__device__ __forceinline__ uint32_t bc_lane(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x150 + U, 0xf, 0xf, true));
}

template <int U>
__device__ __forceinline__ float4 bc_x(int2 e, uint32_t base) { return lds_f4(bc_lane<U>(static_cast<uint32_t>(e.x)) + base); }

template <int U>
__device__ __forceinline__ float bc_w(int2 e) { return __uint_as_float(bc_lane<U>(static_cast<uint32_t>(e.y))); }

// One record: its first `cnt` (1..16) operands, in order, for this lane's row and column, as
// ceil(cnt / 4) batches of four data reads and their arithmetic (a partial last batch computes
// its identity pads: lanes past a pass's count hold the -0.0 tile with weight 1.0).  With PIPE
// the next batch's reads are issued before this batch's arithmetic (8 reads in flight: the
// 512-thread form's registers), else each batch reads, then computes (the 1024-thread form's
// 64-VGPR budget).  The scheduling barriers keep the compiler from hoisting all 16 reads at
// once (64 VGPRs, then spills).
template <int B>
__device__ __forceinline__ void bc_read4(float4 (&x)[4], int2 e, uint32_t base) {
  x[0] = bc_x<4 * B>(e, base);
  x[1] = bc_x<4 * B + 1>(e, base);
  x[2] = bc_x<4 * B + 2>(e, base);
  x[3] = bc_x<4 * B + 3>(e, base);
}

// fp32 EXACT: the four products first, then the ordered adds (each add then has independent
// work between it and the multiply it consumes: no s_nop); the other modes chain next4t.
template <typename T, bool EXACT, int B>
__device__ __forceinline__ float4 bc_math4(float4 acc, const float4 (&x)[4], int2 e) {
  if constexpr (EXACT && !kIsBf16<T>) {
    const float4 p0 = mul4(bc_w<4 * B>(e), x[0]), p1 = mul4(bc_w<4 * B + 1>(e), x[1]),
                 p2 = mul4(bc_w<4 * B + 2>(e), x[2]), p3 = mul4(bc_w<4 * B + 3>(e), x[3]);
    return add4(add4(add4(add4(acc, p0), p1), p2), p3);
  } else {
    acc = next4t<T, EXACT>(acc, bc_w<4 * B>(e), x[0]);
    acc = next4t<T, EXACT>(acc, bc_w<4 * B + 1>(e), x[1]);
    acc = next4t<T, EXACT>(acc, bc_w<4 * B + 2>(e), x[2]);
    return next4t<T, EXACT>(acc, bc_w<4 * B + 3>(e), x[3]);
  }
}

// Two operands of batch B (half H): the lean depth for the 64-VGPR fp32 EXACT form, whose records,
// staging registers and separate products leave room for two data reads in flight, not four.
template <typename T, bool EXACT, int B, int H>
__device__ __forceinline__ float4 bc_half(float4 acc, int2 e, uint32_t base) {
  const float4 x0 = bc_x<4 * B + 2 * H>(e, base), x1 = bc_x<4 * B + 2 * H + 1>(e, base);
  acc = next4t<T, EXACT>(acc, bc_w<4 * B + 2 * H>(e), x0);
  return next4t<T, EXACT>(acc, bc_w<4 * B + 2 * H + 1>(e), x1);
}

// DEPTH = data reads in flight per wavefront: 2, 4 or 8 (see bc_read4 / bc_half).
template <typename T, bool EXACT, int DEPTH>
__device__ __forceinline__ float4 bc_record(float4 acc, int2 e, uint32_t base, int cnt) {
  const int nb = (cnt + 3) >> 2;  // wave-uniform
  float4 xa[4], xb[4];
  if constexpr (DEPTH == 2) {
#define TAL_BC_LEAN(B)                                      \
    if (nb > B) {                                           \
      __builtin_amdgcn_sched_barrier(0);                    \
      acc = bc_half<T, EXACT, B, 0>(acc, e, base);          \
      __builtin_amdgcn_sched_barrier(0);                    \
      acc = bc_half<T, EXACT, B, 1>(acc, e, base);          \
    }
    TAL_BC_LEAN(0) TAL_BC_LEAN(1) TAL_BC_LEAN(2) TAL_BC_LEAN(3)
#undef TAL_BC_LEAN
    return acc;
  } else if constexpr (DEPTH == 8) {
    bc_read4<0>(xa, e, base);
    if (nb > 1) bc_read4<1>(xb, e, base);
    __builtin_amdgcn_sched_barrier(0);
    acc = bc_math4<T, EXACT, 0>(acc, xa, e);
    if (nb > 1) {
      if (nb > 2) bc_read4<2>(xa, e, base);
      __builtin_amdgcn_sched_barrier(0);
      acc = bc_math4<T, EXACT, 1>(acc, xb, e);
    }
    if (nb > 2) {
      if (nb > 3) bc_read4<3>(xb, e, base);
      __builtin_amdgcn_sched_barrier(0);
      acc = bc_math4<T, EXACT, 2>(acc, xa, e);
    }
    if (nb > 3) acc = bc_math4<T, EXACT, 3>(acc, xb, e);
  } else {
    bc_read4<0>(xa, e, base);
    acc = bc_math4<T, EXACT, 0>(acc, xa, e);
    if (nb > 1) {
      __builtin_amdgcn_sched_barrier(0);
      bc_read4<1>(xb, e, base);
      acc = bc_math4<T, EXACT, 1>(acc, xb, e);
    }
    if (nb > 2) {
      __builtin_amdgcn_sched_barrier(0);
      bc_read4<2>(xa, e, base);
      acc = bc_math4<T, EXACT, 2>(acc, xa, e);
    }
    if (nb > 3) {
      __builtin_amdgcn_sched_barrier(0);
      bc_read4<3>(xb, e, base);
      acc = bc_math4<T, EXACT, 3>(acc, xb, e);
    }
  }
  return acc;
}

// Two-chunk broadcast form (C4 = 32): a row's 16 lanes each own chunks cl and cl + 16 of the
// 32-chunk (512 B) source tile, so one broadcast address (the second read at +256 B, the
// instruction's offset) and one broadcast weight serve two float4 of the operand: per operand
// and float4 the vector ALU does (1 address + 1 weight + 2 x arithmetic) / 2, and the lane
// carries two independent accumulator chains.  Batches of four operands: 8 data reads in flight.
template <int B>
__device__ __forceinline__ void bc2_read4(float4 (&x)[8], int2 e, uint32_t base) {
#define TAL_BC2_RD(u)                                                                   \
  {                                                                                     \
    const uint32_t a = bc_lane<4 * B + u>(static_cast<uint32_t>(e.x)) + base;           \
    x[2 * u] = lds_f4(a);                                                               \
    x[2 * u + 1] = lds_f4(a + 256u);                                                    \
  }
  TAL_BC2_RD(0) TAL_BC2_RD(1) TAL_BC2_RD(2) TAL_BC2_RD(3)
#undef TAL_BC2_RD
}

template <typename T, bool EXACT, int U>
__device__ __forceinline__ void bc2_op(float4& a0, float4& a1, const float4& x0, const float4& x1, int2 e) {
  const float w = bc_w<U>(e);
  if constexpr (EXACT && !kIsBf16<T>) {  // one product live at a time (the 128-VGPR budget)
    a0 = add4(a0, mul4(w, x0));
    a1 = add4(a1, mul4(w, x1));
  } else {
    a0 = next4t<T, EXACT>(a0, w, x0);
    a1 = next4t<T, EXACT>(a1, w, x1);
  }
}

template <typename T, bool EXACT>
__device__ __forceinline__ void bc2_record(float4& a0, float4& a1, int2 e, uint32_t base, int cnt) {
  const int nb = (cnt + 3) >> 2;  // wave-uniform
  float4 x[8];
#define TAL_BC2_BATCH(B)                                        \
  if (nb > B) {                                                 \
    __builtin_amdgcn_sched_barrier(0);                          \
    bc2_read4<B>(x, e, base);                                   \
    bc2_op<T, EXACT, 4 * B + 0>(a0, a1, x[0], x[1], e);         \
    bc2_op<T, EXACT, 4 * B + 1>(a0, a1, x[2], x[3], e);         \
    bc2_op<T, EXACT, 4 * B + 2>(a0, a1, x[4], x[5], e);         \
    bc2_op<T, EXACT, 4 * B + 3>(a0, a1, x[6], x[7], e);         \
  }
  TAL_BC2_BATCH(0) TAL_BC2_BATCH(1) TAL_BC2_BATCH(2) TAL_BC2_BATCH(3)
#undef TAL_BC2_BATCH
}

template <int C4>
__device__ __forceinline__ NarrowLds stage_narrow_bc(const PlanView& p, int g, float4* s_data, int nthreads) {
  NarrowLds L;
  L.nr = p.grp_row_ptr[g + 1] - p.grp_row_ptr[g];
  const int ns = p.grp_src_ptr[g + 1] - p.grp_src_ptr[g];
  for (int k = threadIdx.x; k < C4; k += nthreads)  // the identity pads' tile of -0.0 (slot ns)
    s_data[static_cast<size_t>(ns) * C4 + k] = make_float4(-0.f, -0.f, -0.f, -0.f);
  L.rowptr = nullptr;
  L.pairs = nullptr;
  L.out = nullptr;
  L.rec = 0;
  return L;
}

template <int C4>
__device__ __forceinline__ NarrowLds stage_narrow(const PlanView& p, int g, float4* s_data, int nthreads) {
  NarrowLds L;
  const int r_beg = p.grp_row_ptr[g];
  L.nr = p.grp_row_ptr[g + 1] - r_beg;
  const int32_t* nrp = p.nrow_ptr;
  const int32_t* np = p.npairs;
  const int e_beg = nrp[r_beg];
  const int ne = nrp[r_beg + L.nr] - e_beg;
  const int ns = p.grp_src_ptr[g + 1] - p.grp_src_ptr[g];  // the -0.0 tile is slot ns
  int32_t* rowptr = reinterpret_cast<int32_t*>(s_data + static_cast<size_t>(ns + 1) * C4);
  int2* pairs = reinterpret_cast<int2*>(rowptr + ((L.nr + 2) & ~1));
  int32_t* out = reinterpret_cast<int32_t*>(pairs + ne + 4);
  for (int k = threadIdx.x; k < C4; k += nthreads)  // the padding pairs' tile of -0.0
    s_data[static_cast<size_t>(ns) * C4 + k] = make_float4(-0.f, -0.f, -0.f, -0.f);
  for (int k = threadIdx.x; k <= L.nr; k += nthreads) rowptr[k] = nrp[r_beg + k] - e_beg;
  for (int k = threadIdx.x; k < ne + 4; k += nthreads)  // + 4 read-ahead pairs (never used)
    pairs[k] = k < ne ? make_int2(np[2 * (e_beg + k)], np[2 * (e_beg + k) + 1]) : make_int2(0, 0);
  for (int k = threadIdx.x; k < L.nr; k += nthreads) out[k] = p.out_row[r_beg + k];
  L.rowptr = rowptr;
  L.pairs = pairs;
  L.out = out;
  return L;
}

// One row (pairs q0 .. q1-1, q1 - q0 - 1 a multiple of 4) for this lane's column.  PIPE: the
// next batch's pairs are read while this batch's data reads are in flight (8 more VGPRs).
template <typename T, bool EXACT, bool PIPE>
__device__ __forceinline__ float4 narrow_row(const float4* s_data, const int2* pairs, int q0, int q1, int cl) {
  const int2 f = pairs[q0];
  float4 acc = first4t<T, EXACT>(__int_as_float(f.y), s_data[f.x + cl]);
  int q = q0 + 1;
  if constexpr (!PIPE) {
    for (; q < q1; q += 4) {
      int2 e[4];
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) e[u] = pairs[q + u];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = s_data[e[u].x + cl];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = next4t<T, EXACT>(acc, __int_as_float(e[u].y), x[u]);
    }
    return acc;
  }
  if (q < q1) {
    int2 e[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) e[u] = pairs[q + u];
    do {
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = s_data[e[u].x + cl];
      int2 en[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) en[u] = pairs[q + 4 + u];  // next batch (or the read-ahead pad)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = next4t<T, EXACT>(acc, __int_as_float(e[u].y), x[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) e[u] = en[u];
      q += 4;
    } while (q < q1);
  }
  return acc;
}

// Row set of pass p for wavefront `wave`: snake order over the passes, so that with rows sorted
// by operand count no wavefront takes the longest set of every pass.
__device__ __forceinline__ int narrow_set(int p, int wave, int nwaves) {
  return p * nwaves + ((p & 1) ? nwaves - 1 - wave : wave);
}

// NP = row sets held in registers: kNarrowPasses for one resident workgroup per CU (128 VGPRs),
// 0 for two (64 VGPRs: the extents are then read from LDS each pass).
// W16 (bf16 pools): staging loads are 16 B per lane (two 4-element chunks, C4/2 lanes per source
// and tile, J/2 loads per lane) instead of 8 B; each lane writes its two chunks to LDS as two
// fp32 float4, 8 slots apart (cpos below).  Needs an even chunk count, a row stride of an even number of chunks and
// a 16-B aligned base (the launcher checks), so every pair lies inside its row.
// BC: the broadcast form (narrow_bcast plans; NT = 64 x the plan's waves per workgroup).
template <int C4, int NT, int J, int NP, bool EXACT, typename T = float, bool ROWW = false, bool W16 = false,
          bool BC = false>
__global__ __launch_bounds__(NT, NP == 0 ? 2 * NT / 256 : NT / 256) void k_round_f32_narrow(
    const T* __restrict__ pin, int64_t ld_in4, T* __restrict__ pout, int64_t ld_out4, int64_t n4,
    PlanView p, int64_t n_tiles) {
  static_assert(C4 == 16 || C4 == 32, "narrow tiles are 16 or 32 float4 wide");
  static_assert(NT % C4 == 0, "a block stages whole source tiles");
  static_assert(!W16 || (kIsBf16<T> && J % 2 == 0), "16-B staging lanes: bf16 pools, even J");
  constexpr int kLd = W16 ? J / 2 : J;       // staging loads per lane
  constexpr int kLps = W16 ? C4 / 2 : C4;    // staging lanes per source and tile
  // BC at C4 = 32: the two-chunk form (4 rows of 16 lanes per pass, like C4 = 16)
  constexpr bool kX2 = BC && C4 == 32;
  constexpr int kRpw = kX2 ? 4 : 64 / C4;
  constexpr int kW = NT / 64;
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const NarrowLds L = BC ? stage_narrow_bc<C4>(p, g, s_data, NT)
                          : ROWW ? stage_narrow_roww<C4>(p, g, s_data, NT) : stage_narrow<C4>(p, g, s_data, NT);
  const int s_beg = p.grp_src_ptr[g];
  const int ns = p.grp_src_ptr[g + 1] - s_beg;
  const int c = threadIdx.x % kLps;  // staging: the lane's chunk (W16: chunk pair) of its source
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int sub = kX2 ? lane / 16 : lane / C4;
  const int cl = kX2 ? lane % 16 : lane % C4;
  // W16: where column cl of a source sits in its LDS tile.  A staging lane holds two adjacent
  // columns 2c, 2c+1; written side by side, the eight lanes of a ds_write_b128 group span 256 B
  // and meet twice on every bank (banks are (a/4) mod 32 for writes: 2-way).
  // So within each 16-column block the even columns sit in slots 0..7 and the odd ones in 8..15
  // (column 2c'+h at slot 8h+c'): each write instruction's group covers 128 contiguous bytes, and
  // a ds_read_b128 lane group still meets each 16-B slot of a bank row once (the map is a
  // bijection on each 16-column block and every read group takes whole-block-aligned lane sets).
  const int cpos = W16 ? ((cl & ~15) | ((cl & 1) << 3) | ((cl & 15) >> 1)) : cl;
  // Staging is branch-free, so that the compiler's wait analysis sees every load land in its
  // register unconditionally (a conditional load made it wait for each load before issuing the
  // next: four serial HBM round trips per tile).  A lane past the group's sources reloads
  // source 0's chunk of its column and writes it where source 0's own lane does (same value).
  // The write index and (pairs form, whose registers are tight) the load addresses are
  // recomputed per tile behind an empty asm, so the compiler does not hoist them into J more
  // registers each (it spilled).
  int srow[kLd];
#pragma unroll
  for (int j = 0; j < kLd; ++j) {
    const int src = (j * NT + threadIdx.x) / kLps;
    srow[j] = p.src_row[s_beg + (src < ns ? src : 0)];
  }
  __syncthreads();  // plan slice staged
  // pairs form: the first NP row sets' extents in registers (ROWW reads its records instead; the
  // broadcast form has no row extents at all - stage_narrow_bc leaves L.rowptr / L.out null)
  constexpr int kNP = (NP > 0 && !ROWW && !BC) ? NP : 1;
  int rq0[kNP], rq1[kNP], rout[kNP];
  if constexpr (!ROWW && !BC) {
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int r = narrow_set(k, wave, kW) * kRpw + sub;
      rq0[k] = r < L.nr ? L.rowptr[r] : 0;
      rq1[k] = r < L.nr ? L.rowptr[r + 1] : 0;
      rout[k] = r < L.nr ? L.out[r] : 0;
    }
  }
  const int n_sets = (L.nr + kRpw - 1) / kRpw;
  // ROWW: this lane's column base in the data tile, and its record offset within a pass
  const uint32_t col_base = lds_addr(s_data + cpos);
  const uint32_t rec_lane = L.rec + 16u * static_cast<uint32_t>(sub);
  // BC: this wavefront's program (wave-uniform: scalar loads) and its records, loaded once
  // before the first staging loads (the records never wait behind them)
  constexpr int kR = BC ? bc_rec_max<NT>() : 1;
  // BC read depth: 8 data reads in flight where the registers allow it (one workgroup per CU:
  // NP = 1, 128 VGPRs at 1024 threads; 512 threads except fp32 EXACT, whose separate products
  // and the 8-VGPR staging of 8 loads per lane fill 128), 2 for fp32 EXACT at two 768- or
  // 1024-thread workgroups per CU (80 / 64 VGPRs), else 4
  constexpr bool kF32x = EXACT && !kIsBf16<T>;
  constexpr int kBcDepth = (NP == 1 || (NT <= 512 && !kF32x)) ? 8 : (kF32x && NT >= 768) ? 2 : 4;
  const int bc_off = BC ? ((ConstI32)p.bc_prog)[g * kW + wave] : 0;
  const ConstI32 prog = (ConstI32)(p.base + bc_off);
  const int bc_n = BC ? prog[0] : 0;
  int2 bc_rec[kR];
  // the program's record words, in SGPRs for the whole kernel: read in the tile loop, each was a
  // scalar load the compiler hoisted into the previous record's batch, and a scalar load in
  // flight forces lgkmcnt(0) (SMEM returns out of order) - every batch then waited for all of
  // its LDS reads before its first multiply
  int bc_d[kR];
  if constexpr (BC) {
    const int2* recs = reinterpret_cast<const int2*>(p.base + (bc_off + prog[2])) + lane;
#pragma unroll
    for (int r = 0; r < kR; ++r) bc_rec[r] = r < bc_n ? recs[64 * r] : make_int2(0, 0);
#pragma unroll
    for (int r = 0; r < kR; ++r) bc_d[r] = r < bc_n ? prog[kBcHdr + r] : 0;
  }
  // converted to fp32 when written to LDS, not when loaded
  typedef typename std::conditional<W16, u32x4, typename Io<T>::raw_t>::type raw_t;
  raw_t v[kLd];
  auto load_tile = [&](int64_t tt) {
    if constexpr (W16) {  // 16-B units: chunk pair tt * C4 / 2 + c of each row
      const int64_t col = min(tt * kLps + c, (n4 - 1) / 2);  // past the end: a duplicate
      const u32x4* b = reinterpret_cast<const u32x4*>(pin);
#pragma unroll
      for (int j = 0; j < kLd; ++j)
        v[j] = __builtin_nontemporal_load(b + static_cast<int64_t>(srow[j]) * (ld_in4 / 2) + col);
    } else {
      const int64_t col = min(tt * C4 + c, n4 - 1);  // past the end: a duplicate (cache hit)
#pragma unroll
      for (int j = 0; j < kLd; ++j) {
        int r = srow[j];
        if constexpr (!ROWW) asm volatile("" : "+v"(r));
        v[j] = Io<T>::ld_raw(pin, static_cast<int64_t>(r) * ld_in4 + col);
      }
    }
  };
  int64_t t = blockIdx.x;
  if (t < n_tiles) load_tile(t);
  for (; t < n_tiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's readers are done with s_data
    // staging units (float4 slots; W16: slot pairs) of real sources (readfirstlane: the broadcast
    // form's control flow otherwise leaves the compiler unsure that ns is uniform here)
    int staged = __builtin_amdgcn_readfirstlane(ns * kLps);
    asm volatile("" : "+s"(staged));
#pragma unroll
    for (int j = 0; j < kLd; ++j) {
      const int k = j * NT + static_cast<int>(threadIdx.x);
      if constexpr (W16) {  // unit u = source u / kLps, chunk pair c: slots cpos(2c), cpos(2c) + 8
        const int u = k < staged ? k : c;
        const int q = u + (u & ~7);
        s_data[q] = Io<T>::f4(u32x2{v[j].x, v[j].y});
        s_data[q + 8] = Io<T>::f4(u32x2{v[j].z, v[j].w});
      } else {
        s_data[k < staged ? k : c] = Io<T>::f4(v[j]);
      }
    }
    __syncthreads();
    if (t + gridDim.x < n_tiles) load_tile(t + gridDim.x);  // in flight during this tile's math
    const int64_t col = t * C4 + cl;
    if constexpr (BC) {
      // the records are loop-invariant: without this the compiler hoists every broadcast and
      // address of the tile loop out of it (hundreds of VGPRs, then spills)
#pragma unroll
      for (int r = 0; r < kR; ++r) asm volatile("" : "+v"(bc_rec[r].x), "+v"(bc_rec[r].y));
#pragma unroll
      for (int r = 0; r < kR; ++r) asm volatile("" : "+s"(bc_d[r]));
      float4 acc = make_float4(-0.f, -0.f, -0.f, -0.f);
      float4 acc1 = acc;  // kX2: chunk cl + 16
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        if (r >= bc_n) continue;  // wave-uniform (a constant trip count keeps the loop unrolled,
                                  // so the records stay in registers)
        const uint32_t d = static_cast<uint32_t>(bc_d[r]);
        if constexpr (kX2)
          bc2_record<T, EXACT>(acc, acc1, bc_rec[r], col_base, static_cast<int>(d & 0xffu));
        else
          acc = bc_record<T, EXACT, kBcDepth>(acc, bc_rec[r], col_base, static_cast<int>(d & 0xffu));
        if (d & 0x100u) {  // the pass's last record: store its rows
          const ConstI32 orow = prog + kBcHdr + kR + 4 * static_cast<int>(d >> 16);
          const int o0 = orow[0], o1 = orow[1], o2 = orow[2], o3 = orow[3];
          const int o = sub == 0 ? o0 : sub == 1 ? o1 : sub == 2 ? o2 : o3;
          if (o >= 0 && col < n4) Io<T>::st(pout, static_cast<int64_t>(o) * ld_out4 + col, acc);
          if constexpr (kX2) {
            if (o >= 0 && col + 16 < n4) Io<T>::st(pout, static_cast<int64_t>(o) * ld_out4 + col + 16, acc1);
            acc1 = make_float4(-0.f, -0.f, -0.f, -0.f);
          }
          acc = make_float4(-0.f, -0.f, -0.f, -0.f);
        }
      }
      continue;
    }
    if constexpr (ROWW) {
      for (int k = 0; k * kW < n_sets; ++k) {  // passes: row sets in snake order
        const int set = narrow_set(k, wave, kW);
        if (set >= n_sets) continue;  // wave-uniform
        const uint4 rc = lds_u4(rec_lane + 16u * static_cast<uint32_t>(set * kRpw));
        const float4 acc = narrow_row_roww<T, EXACT>(rc, col_base);
        if (static_cast<int32_t>(rc.w) >= 0 && col < n4) {
          Io<T>::st(pout, static_cast<int64_t>(static_cast<int32_t>(rc.w)) * ld_out4 + col, acc);
        }
      }
      continue;
    }
    if constexpr (!ROWW && !BC) {  // the pairs form (the other two forms continued above)
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        if (rq1[k] > rq0[k]) {
          const float4 acc = narrow_row<T, EXACT, (NP > 0)>(s_data, L.pairs, rq0[k], rq1[k], cpos);
          if (col < n4) Io<T>::st(pout, static_cast<int64_t>(rout[k]) * ld_out4 + col, acc);
        }
      }
      for (int k = NP; k * kW < n_sets; ++k) {  // row sets beyond the register-held ones
        const int r = narrow_set(k, wave, kW) * kRpw + sub;
        if (r < L.nr) {
          const float4 acc = narrow_row<T, EXACT, (NP > 0)>(s_data, L.pairs, L.rowptr[r], L.rowptr[r + 1], cpos);
          if (col < n4) Io<T>::st(pout, static_cast<int64_t>(L.out[r]) * ld_out4 + col, acc);
        }
      }
    }
  }
}

// General form (groups whose staging needs more than 8 loads per lane): one tile per
// workgroup, staging in batches of 4 independent loads per lane.
template <int C4, int NT, bool EXACT, bool DENSE, typename T = float>
__global__ __launch_bounds__(NT) void k_round_f32_tiled(const T* __restrict__ pin,
                                                        int64_t ld_in4, T* __restrict__ pout,
                                                        int64_t ld_out4, int64_t n4, PlanView p) {
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const int s_beg = p.grp_src_ptr[g];
  const int ns = p.grp_src_ptr[g + 1] - s_beg;
  const int r_beg = p.grp_row_ptr[g];
  const int nr = p.grp_row_ptr[g + 1] - r_beg;
  const int64_t c0 = static_cast<int64_t>(blockIdx.x) * C4;
  const int total = ns * C4;
  constexpr int U = 4;
  for (int k0 = 0; k0 < total; k0 += NT * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * NT + threadIdx.x;
      const int c = k % C4;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (k < total && c0 + c < n4)
        v[u] = Io<T>::ld(pin, static_cast<int64_t>(p.src_row[s_beg + k / C4]) * ld_in4 + c0 + c);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = k0 + u * NT + threadIdx.x;
      if (k < total) s_data[k] = v[u];
    }
  }
  __syncthreads();
  if constexpr (DENSE)
    emit_tile_dense<C4, NT, kDenseRb, EXACT>(s_data, p, g, r_beg, nr, ns, pout, ld_out4, c0, n4);
  else
    emit_tile<C4, NT, EXACT, T>(s_data, p, r_beg, nr, pout, ld_out4, c0, n4);
}

// Scalar tiled round: the fp32 tail (elements e0..n-1 when the float4 path ran) or whole
// unaligned pools, and the int64 segment (IS_I64: fp32 accumulate, truncation).  The tile is
// 4*c4 elements so one staged source costs the same 16*c4 LDS bytes as in the float4 kernel.
template <typename T, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_round_tiled_scalar(const T* __restrict__ pin, int64_t ld_in,
                                                               T* __restrict__ pout, int64_t ld_out,
                                                               int64_t e0, int64_t n, PlanView p,
                                                               int tile) {
  constexpr bool kI64 = std::is_same<T, int64_t>::value;
  extern __shared__ float s_f[];
  const int ns = p.grp_src_ptr[blockIdx.y + 1] - p.grp_src_ptr[blockIdx.y];
  const GroupLds L = stage_group(p, blockIdx.y, s_f + static_cast<size_t>(ns) * tile, tile, kBlock);
  __syncthreads();
  const int64_t t0 = e0 + static_cast<int64_t>(blockIdx.x) * tile;
  const int64_t cols = min(static_cast<int64_t>(tile), n - t0);
  for (int k = threadIdx.x; k < L.ns * tile; k += kBlock) {
    const int s = k / tile;
    const int c = k % tile;
    float v = 0.f;
    if (c < cols) {
      const int64_t row = L.src[s];
      if constexpr (kI64) v = static_cast<float>(pin[row * ld_in + t0 + c]);
      else v = Io<T>::ld1(pin, row * ld_in + t0 + c);
    }
    s_f[k] = v;
  }
  __syncthreads();

  for (int c = threadIdx.x; c < cols; c += kBlock) {
    for (int r = 0; r < L.nr; ++r) {
      const int q0 = L.rowptr[r];
      const int q1 = L.rowptr[r + 1];
      float acc = first1t<T, EXACT || kI64>(L.w[q0], s_f[L.slot[q0] + c]);
      for (int q = q0 + 1; q < q1; ++q) acc = next1t<T, EXACT || kI64>(acc, L.w[q], s_f[L.slot[q] + c]);
      const int64_t orow = L.out[r];
      if constexpr (kI64) pout[orow * ld_out + t0 + c] = trunc_i64(acc);
      else Io<T>::st1(pout, orow * ld_out + t0 + c, acc);
    }
  }
}

// ------------------------------------------------------------------------------------------
// K3, streamed form: sources pass through a ring of LDS chunks (global->LDS DMA), so a
// group's source count is unbounded and the workgroup needs no staging registers.
//
// Workgroup = CS wavefronts = one group of <= 8*CS rows (wavefront w owns dense row block w).
// Per column tile of 64 float4, the group's sources are consumed CS at a time: wavefront w
// DMAs source k*CS+w of chunk k (64 lanes x 16 B = 1 KiB, lane-linear in LDS) into ring slot
// (chunk index mod NBUF).  Chunks are prefetched kStreamDepth ahead across tile boundaries.
// A row's operands are ascending sources then itself, so accumulating chunk by chunk keeps the
// reference order; each row's own model is captured in registers when its chunk passes and
// added last.  The DMA is issued from inline asm (hipcc would otherwise drain vmcnt before
// every LDS read), so the kernel counts vmcnt itself: every VMEM op of a wavefront (DMA and
// output stores) retires in issue order, and chunk q is resident once at most
// (DMAs issued after it) + (stores issued after it) ops are outstanding.
// ------------------------------------------------------------------------------------------

template <int NT, bool EXACT>
__global__ __launch_bounds__(NT, 2048 / NT) void k_round_stream(const float* __restrict__ pin, int64_t ld_in4,
                                                     float* __restrict__ pout, int64_t ld_out4,
                                                     int64_t n4, PlanView p, int64_t n_tiles) {
  constexpr int NW = NT / 64;
  constexpr int D = kStreamPerWave;
  constexpr int CS = NW * D;
  constexpr int P = kStreamDepth;
  constexpr int NBUF = P + 1;
  constexpr int RB = kDenseRb;
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const ConstI32 grp_src_ptr = (ConstI32)p.grp_src_ptr;
  const ConstI32 grp_row_ptr = (ConstI32)p.grp_row_ptr;
  const ConstI32 src_row = (ConstI32)p.src_row;
  const int s_beg = grp_src_ptr[g];
  const int ns = grp_src_ptr[g + 1] - s_beg;
  const int r_beg = grp_row_ptr[g];
  const int nr = grp_row_ptr[g + 1] - r_beg;
  const int nch = (ns + CS - 1) / CS;
  const int64_t bx = blockIdx.x, gx = gridDim.x;
  const int64_t n_mine = bx < n_tiles ? (n_tiles - 1 - bx) / gx + 1 : 0;
  const int64_t total = n_mine * nch;  // chunk steps of this workgroup
  const float4* pin4 = reinterpret_cast<const float4*>(pin);
  const uint32_t lds0 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)s_data));

  // DMA cursor: (tile i, chunk k) of step qi; wavefront w moves sources k*CS + d*NW + w, d < D.
  // The pool rows of the next issue are fetched one issue ahead (off the critical path).
  int64_t qi = 0, ii = 0;
  int ik = 0;
  int next_row[D];
  auto fetch_rows = [&]() {
#pragma unroll
    for (int d = 0; d < D; ++d)  // past the last source: a duplicate (an L2 hit)
      next_row[d] = src_row[s_beg + min(ik * CS + d * NW + wave, ns - 1)];
  };
  fetch_rows();
  auto issue = [&]() {
    const int64_t t = bx + ii * gx;
    const int64_t col = min(t * 64 + lane, n4 - 1);
#pragma unroll
    for (int d = 0; d < D; ++d)
      dma16(pin4 + static_cast<int64_t>(next_row[d]) * ld_in4 + col,
            lds0 + static_cast<uint32_t>(((qi % NBUF) * CS + d * NW + wave) * 1024));
    ++qi;
    if (++ik == nch) { ik = 0; ++ii; }
    if (qi < total) fetch_rows();
  };
  for (int d = 0; d < P; ++d)
    if (qi < total) issue();

  // my row block
  const int nblk = (nr + RB - 1) / RB;
  const bool has_blk = wave < nblk;
  const int rows_here = has_blk ? min(RB, nr - wave * RB) : 0;
  const ConstI32 base = (ConstI32)p.base;
  const ConstI32 tab = has_blk ? base + ((ConstI32)p.blk_tab)[((ConstI32)p.grp_blk_ptr)[g] + wave] : base;
  const int n_used = has_blk ? tab[0] : 0;
  const ConstI32x4 slots4 = (ConstI32x4)(tab + 8);
  const ConstI32x4 masks4 = (ConstI32x4)(tab + 8 + n_used);
  const ConstF32x8 wts8 = (ConstF32x8)(tab + 8 + 2 * n_used);
  float self_w[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    self_w[r] = 0.f;
    if (r < rows_here)  // own model: the row's last operand
      self_w[r] = ((ConstF32)p.op_w)[((ConstI32)p.row_ptr)[r_beg + wave * RB + r + 1] - 1];
  }
  const float4 kNeg0 = make_float4(-0.f, -0.f, -0.f, -0.f);  // x + (-0) == x for every x
  float4 acc[RB], self_x[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    acc[r] = kNeg0;
    self_x[r] = kNeg0;
  }

  int64_t ci = 0;   // compute cursor: tile i, chunk k
  int ck = 0;
  int e = 0;        // table cursor (entries of chunks < ck consumed)
  uint32_t ends = 0;  // bit j: the step j+1 before this one ended a tile (issued stores)
  for (int64_t q = 0; q < total; ++q) {
    const int younger_dma = D * static_cast<int>(min<int64_t>(P - 1, total - 1 - q));
    const int younger_st = rows_here * __builtin_popcount(ends & ((1u << P) - 1));
    wait_vm_barrier(younger_dma + younger_st);  // chunk q resident; step q-1's readers done
    if (qi < total) issue();                    // into the slot step q-1 read
    if (has_blk) {
      const float4* buf = s_data + (q % NBUF) * CS * 64 + lane;
      const int lo = ck * CS, hi = lo + CS;
      for (; e < n_used; e += 4) {
        const i32x4 sl = slots4[e >> 2];
        if (sl.x >= hi) break;
        const i32x4 mk = masks4[e >> 2];
        float4 x[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) x[u] = buf[(sl[u] - lo) * 64];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t m = static_cast<uint32_t>(mk[u]);
          if (m & kMaskSelf) {  // this source is some rows' own model: keep it for the end
#pragma unroll
            for (int r = 0; r < RB; ++r)
              if (m & (kMaskSelf0 << r)) self_x[r] = x[u];
          }
          const f32x8 wv = wts8[e + u];
          if ((m & 0xffu) == 0) {
            // padding or own-model-only entry
          } else if (EXACT && (m & kMaskUniform)) {  // one product serves every row
            const float4 pr = mul4(wv[0], x[u]);
            if ((m & 0xffu) == 0xffu) {
#pragma unroll
              for (int r = 0; r < RB; ++r) acc[r] = add4(acc[r], pr);
            } else {
#pragma unroll
              for (int r = 0; r < RB; ++r)
                if (m & (1u << r)) acc[r] = add4(acc[r], pr);
            }
          } else if ((m & 0xffu) == 0xffu) {  // cliques: every row of the block takes this source
#pragma unroll
            for (int r = 0; r < RB; ++r) acc[r] = next4<EXACT>(acc[r], wv[r], x[u]);
          } else {
#pragma unroll
            for (int r = 0; r < RB; ++r)
              if (m & (1u << r)) acc[r] = next4<EXACT>(acc[r], wv[r], x[u]);
          }
        }
      }
    }
    ends <<= 1;
    if (ck == nch - 1) {  // tile done: own model last, store, reset
      if (has_blk) {
        const int64_t col = (bx + ci * gx) * 64 + lane;
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          if (r < rows_here) {
            acc[r] = next4<EXACT>(acc[r], self_w[r], self_x[r]);
            const int64_t orow = ((ConstI32)p.out_row)[r_beg + wave * RB + r];
            if (col < n4) st_stream(pout, orow * ld_out4 + col, acc[r]);
            acc[r] = make_float4(-0.f, -0.f, -0.f, -0.f);
          }
        }
      }
      ends |= 1u;
      ck = 0;
      ++ci;
      e = 0;
    } else {
      ++ck;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------------
// K3, wide-row form for bf16 pools (a streamed plan's groups, <= kWideRows rows each): rows with
// more distinct sources than one LDS tile holds (the reference's `unweighted_fl`, every other
// client a neighbor, decentralized_app.py:386-389) read each source once per group and column
// tile instead of once per row.  Workgroup = (column tile of kWideC4 float4, group); thread =
// (row of the group, float4 column).  The group's sources (ascending pool rows) pass through LDS
// kWideSrc at a time, converted to fp32 (the next chunk's loads in flight while the current one
// is reduced); each row walks its operands in reference order - ascending sources, its own model
// last (kept in registers when its chunk passes) - with the bf16 arithmetic of the other round
// kernels (EXACT: every product and sum rounded to bf16; FMA: fp32 fused, rounded by the store).
// ------------------------------------------------------------------------------------------
constexpr int kWideRows = 16;
constexpr int kWideC4 = 16;
constexpr int kWideSrc = 64;
constexpr int kWideThreads = kWideRows * kWideC4;  // 256
constexpr int kWideLoads = kWideSrc * kWideC4 / kWideThreads;  // 4 staged chunks per thread

template <typename T, bool EXACT>
__global__ __launch_bounds__(kWideThreads) void k_round_wide(const T* __restrict__ pin, int64_t ld_in4,
                                                            T* __restrict__ pout, int64_t ld_out4, int64_t n4,
                                                            PlanView p) {
  __shared__ float4 s_x[kWideSrc * kWideC4];  // 16 KiB
  const int g = blockIdx.y;
  const int t = threadIdx.x;
  const int rr = t / kWideC4, c = t % kWideC4;
  const int s_beg = p.grp_src_ptr[g], ns = p.grp_src_ptr[g + 1] - s_beg;
  const int r_beg = p.grp_row_ptr[g], nr = p.grp_row_ptr[g + 1] - r_beg;
  const bool live = rr < nr;
  const int row = r_beg + (live ? rr : 0);
  const int q1 = p.row_ptr[row + 1];
  int q = p.row_ptr[row];
  const int last = q1 - 1;  // the row's own model: its last operand, applied after the others
  const int self_slot = p.op_slot[last];
  const float self_w = p.op_w[last];
  const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * kWideC4;
  const int nch = (ns + kWideSrc - 1) / kWideSrc;
  typename Io<T>::raw_t v[kWideLoads];
  auto load = [&](int k) {
#pragma unroll
    for (int u = 0; u < kWideLoads; ++u) {
      const int slot = t + u * kWideThreads;
      const int src = k * kWideSrc + slot / kWideC4;
      if (src < ns)  // past the row end: a duplicate of its last chunk (never stored)
        v[u] = Io<T>::ld_raw(pin, static_cast<int64_t>(p.src_row[s_beg + src]) * ld_in4 +
                                     min(tile0 + slot % kWideC4, n4 - 1));
    }
  };
  load(0);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f), self_x = acc;
  bool started = false;
  for (int k = 0; k < nch; ++k) {
    __syncthreads();  // the previous chunk's readers are done
#pragma unroll
    for (int u = 0; u < kWideLoads; ++u) {
      const int slot = t + u * kWideThreads;
      if (k * kWideSrc + slot / kWideC4 < ns) s_x[slot] = Io<T>::f4(v[u]);
    }
    __syncthreads();
    if (k + 1 < nch) load(k + 1);  // in flight while this chunk is reduced
    if (!live) continue;
    const int lo = k * kWideSrc, hi = lo + kWideSrc;
    if (self_slot >= lo && self_slot < hi) self_x = s_x[(self_slot - lo) * kWideC4 + c];
    for (; q < last; ++q) {
      const int sl = p.op_slot[q];
      if (sl >= hi) break;
      const float4 x = s_x[(sl - lo) * kWideC4 + c];
      acc = started ? next4t<T, EXACT>(acc, p.op_w[q], x) : first4t<T, EXACT>(p.op_w[q], x);
      started = true;
    }
  }
  const int64_t col = tile0 + c;
  if (live && col < n4) {
    acc = started ? next4t<T, EXACT>(acc, self_w, self_x) : first4t<T, EXACT>(self_w, self_x);
    Io<T>::st(pout, static_cast<int64_t>(p.out_row[row]) * ld_out4 + col, acc);
  }
}

template <typename T>
int32_t launch_round_wide(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4, const PlanView& v,
                          const tal_round_plan_info& in, bool exact, hipStream_t s) {
  if (in.max_rows > kWideRows) return fail(TAL_ERR_INVALID, "wide-row round: groups of at most 16 rows");
  const int64_t tiles = (n4 + kWideC4 - 1) / kWideC4;
  if (tiles > 0x7fffffff || in.n_groups > 65535) return fail(TAL_ERR_INVALID, "wide-row round: grid too large");
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(in.n_groups));
  if (exact) k_round_wide<T, true><<<grid, kWideThreads, 0, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v);
  else k_round_wide<T, false><<<grid, kWideThreads, 0, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v);
  return check_launch("round kernel (wide rows)");
}

// Tail / int64 columns of a streamed plan: per (column chunk, group) workgroup, the group's
// sources' columns are staged in LDS (as fp32), then each thread computes (row, column) pairs
// walking the row's operands in reference order from the plan in global memory.
template <bool IS_I64, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_round_stream_scalar(const void* __restrict__ pin_v,
                                                                int64_t ld_in,
                                                                void* __restrict__ pout_v,
                                                                int64_t ld_out, int64_t e0,
                                                                int64_t n, PlanView p, int tc) {
  extern __shared__ float s_f[];
  const int g = blockIdx.y;
  const int s_beg = p.grp_src_ptr[g];
  const int ns = p.grp_src_ptr[g + 1] - s_beg;
  const int r_beg = p.grp_row_ptr[g];
  const int nr = p.grp_row_ptr[g + 1] - r_beg;
  const int64_t t0 = e0 + static_cast<int64_t>(blockIdx.x) * tc;
  const int cols = static_cast<int>(min(static_cast<int64_t>(tc), n - t0));
  for (int k = threadIdx.x; k < ns * tc; k += kBlock) {
    const int sidx = k / tc;
    const int c = k % tc;
    float v = 0.f;
    if (c < cols) {
      const int64_t row = p.src_row[s_beg + sidx];
      if constexpr (IS_I64) {
        v = static_cast<float>(static_cast<const int64_t*>(pin_v)[row * ld_in + t0 + c]);
      } else {
        v = static_cast<const float*>(pin_v)[row * ld_in + t0 + c];
      }
    }
    s_f[k] = v;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < nr * cols; k += kBlock) {
    const int r = k / cols;
    const int c = k % cols;
    const int gr = r_beg + r;
    const int q0 = p.row_ptr[gr], q1 = p.row_ptr[gr + 1];
    float acc = first_term<EXACT || IS_I64>(p.op_w[q0], s_f[p.op_slot[q0] * tc + c]);
    for (int q = q0 + 1; q < q1; ++q) acc = next_term<EXACT || IS_I64>(acc, p.op_w[q], s_f[p.op_slot[q] * tc + c]);
    const int64_t orow = p.out_row[gr];
    if constexpr (IS_I64) {
      static_cast<int64_t*>(pout_v)[orow * ld_out + t0 + c] = trunc_i64(acc);
    } else {
      static_cast<float*>(pout_v)[orow * ld_out + t0 + c] = acc;
    }
  }
}

// Few columns (the fp32 n mod 4 tail after a float4 kernel, the int64 segment): one thread per
// (row, column), the row's operands read straight from the pool (L2-served, no staging), eight
// loads in flight ahead of the ordered accumulate.  Out of place only: threads of different
// workgroups would otherwise read rows others are writing.  Serves sparse, dense and streamed
// plans alike (src_row / op_slot mean the same in every form).
constexpr int64_t kDirectMaxCols = 256;

template <typename T, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_round_direct(const T* __restrict__ pin, int64_t ld_in,
                                                         T* __restrict__ pout, int64_t ld_out,
                                                         int64_t e0, int cols, int rows, int n_groups,
                                                         PlanView p) {
  constexpr bool kI64 = std::is_same<T, int64_t>::value;
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= rows * cols) return;
  const int r = k / cols;
  const int64_t e = e0 + k % cols;
  int g = 0;
  while (g + 1 < n_groups && p.grp_row_ptr[g + 1] <= r) ++g;
  const int s_beg = p.grp_src_ptr[g];
  const int q0 = p.row_ptr[r], q1 = p.row_ptr[r + 1];
  auto load = [&](int q) -> float {
    const int64_t row = p.src_row[s_beg + p.op_slot[q]];
    if constexpr (kI64) return static_cast<float>(pin[row * ld_in + e]);
    else return Io<T>::ld1(pin, row * ld_in + e);
  };
  float acc = first1t<T, EXACT>(p.op_w[q0], load(q0));
  int q = q0 + 1;
  for (; q + 8 <= q1; q += 8) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = load(q + u);
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = next1t<T, EXACT>(acc, p.op_w[q + u], x[u]);
  }
  for (; q < q1; ++q) acc = next1t<T, EXACT>(acc, p.op_w[q], load(q));
  const int64_t orow = p.out_row[r];
  if constexpr (kI64) pout[orow * ld_out + e] = trunc_i64(acc);
  else Io<T>::st1(pout, orow * ld_out + e, acc);
}

template <typename T>
int32_t launch_round_direct(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t e0,
                            int64_t n, const PlanView& v, const tal_round_plan_info& in, bool exact,
                            hipStream_t s) {
  const int64_t cols = n - e0;
  const int64_t threads = cols * in.rows;
  if (threads > 0x7fffffffLL) return fail(TAL_ERR_INVALID, "round direct kernel: too many elements");
  const unsigned blocks = static_cast<unsigned>((threads + kBlock - 1) / kBlock);
  auto k = (std::is_same<T, int64_t>::value || exact) ? k_round_direct<T, true> : k_round_direct<T, false>;
  k<<<blocks, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, e0, static_cast<int>(cols), in.rows, in.n_groups, v);
  return check_launch("round direct kernel");
}

// the direct kernel serves the call: few columns, out of place
inline bool use_direct(const void* pin, const void* pout, int64_t e0, int64_t n) {
  return pin != pout && n > e0 && n - e0 <= kDirectMaxCols;
}

// LDS of one group in the staged scalar kernel (and the float4 kernels' tile): its sources'
// tile (16 * c4 B each) plus its plan slice [row_ptr (nr+1)][slot (no)][w (no)][src (ns)][out (nr)]
constexpr int64_t group_lds_bytes(int64_t ns, int64_t nr, int64_t no, int c4) {
  return ns * 16 * c4 + (nr + 1 + 2 * no + ns + nr) * 4;
}

// Tile width (in float4 units) of the scalar kernel (the n mod 4 tail, the int64 segment and
// unaligned pools): the plan's c4, except for narrow plans, whose scalar tiles stay at 16 so a
// 32-wide narrow tile of 256 sources (128 KiB) leaves the scalar kernel's tile + plan slice
// under 160 KiB.
constexpr int scalar_c4(int c4) { return c4 < 64 ? 16 : c4; }

std::mutex g_lds_mu;
std::vector<const void*> g_lds_raised;

int32_t ensure_lds(const void* kernel, size_t bytes) {
  // Dynamic LDS above 64 KiB must be opted in per kernel (gfx950 allows 160 KiB per workgroup).
  if (bytes > 160 * 1024) return fail(TAL_ERR_CAPACITY, "round plan needs more than 160 KiB LDS");
  if (bytes <= 64 * 1024) return TAL_OK;
  std::lock_guard<std::mutex> lk(g_lds_mu);
  if (std::find(g_lds_raised.begin(), g_lds_raised.end(), kernel) != g_lds_raised.end()) return TAL_OK;
  hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (e != hipSuccess)
    return fail(TAL_ERR_HIP, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  g_lds_raised.push_back(kernel);
  return TAL_OK;
}

int32_t validate_info(const tal_round_plan_info* info) {
  if (!info) return fail(TAL_ERR_INVALID, "null plan info");
  if (info->rows <= 0 || info->n_groups <= 0 || info->max_src <= 0)
    return fail(TAL_ERR_INVALID, "empty round plan");
  if (info->c4 != 16 && info->c4 != 32 && info->c4 != 64 && info->c4 != 128)
    return fail(TAL_ERR_INVALID, "plan c4 must be 16, 32, 64 or 128");
  if (info->c4 < 64 && info->dense_rb != 0)
    return fail(TAL_ERR_INVALID, "narrow plans (c4 16 / 32) are sparse");
  if (info->narrow_bcast != 0 &&
      (info->c4 >= 64 || (info->narrow_bcast != 8 && info->narrow_bcast != 12 && info->narrow_bcast != 16) ||
       info->bc_rec_max != kBcRecPerWg / info->narrow_bcast || info->bc_wg_per_cu < 1 || info->bc_wg_per_cu > 2))
    return fail(TAL_ERR_INVALID, "broadcast-form plan: c4 16 / 32, 8 or 16 wavefronts, 128 / waves records, "
                                 "1 or 2 workgroups per CU");
  if (info->dense_rb != 0 && info->dense_rb != kDenseRb)
    return fail(TAL_ERR_INVALID, "plan dense_rb must be 0 or 8");
  if (info->stream_cs != 0 && info->stream_cs != 8 * kStreamPerWave && info->stream_cs != 16 * kStreamPerWave)
    return fail(TAL_ERR_INVALID, "plan stream_cs must be 0 or the library's chunk size (8 or 16 wavefronts)");
  if (info->stream_cs != 0 && (info->c4 != 64 || info->dense_rb != kDenseRb ||
                               info->max_rows > kDenseRb * info->stream_cs / kStreamPerWave))
    return fail(TAL_ERR_INVALID, "streamed plan: c4 64, dense row blocks, <= 8 rows per wavefront");
  return TAL_OK;
}

template <typename T>
int32_t launch_round_scalar(const T* pin, int64_t ld_in, T* pout, int64_t ld_out,
                            int64_t e0, int64_t n, const PlanView& v,
                            const tal_round_plan_info& in, bool exact, hipStream_t s) {
  if (n <= e0) return TAL_OK;
  const int tile = 4 * scalar_c4(in.c4);
  const size_t lds = static_cast<size_t>(in.scalar_lds_bytes);  // the largest group's tile + plan slice
  const int64_t tiles = (n - e0 + tile - 1) / tile;
  if (tiles > 0x7fffffff) return fail(TAL_ERR_INVALID, "too many tiles");
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(in.n_groups));
  auto k = (std::is_same<T, int64_t>::value || exact) ? k_round_tiled_scalar<T, true> : k_round_tiled_scalar<T, false>;
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  k<<<grid, kBlock, lds, s>>>(pin, ld_in, pout, ld_out, e0, n, v, tile);
  return check_launch("round scalar kernel");
}

// Threads per round workgroup: 16 wavefronts at c4 = 64 (a 64-source tile is 4 loads per lane),
// 8 at c4 = 128 (dense rows: fewer, longer rows per wavefront).  Tuned on MI355X with
// tools/tune/round_variants.hip (config 3: 2.0-2.1 ms / round, config 4: 7.8 ms).
template <int C4>
constexpr int round_threads() { return C4 >= 128 ? 512 : 1024; }

template <int C4, int J, bool EXACT, bool DENSE, typename T = float>
int32_t launch_round_persistent(const T* pin, int64_t ld_in, T* pout, int64_t ld_out,
                                int64_t n4, const PlanView& v, const tal_round_plan_info& in,
                                size_t lds, hipStream_t s) {
  constexpr int kRoundThreads = round_threads<C4>();
  auto k = k_round_f32_persistent<C4, kRoundThreads, J, EXACT, DENSE, T>;
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const int64_t tiles = (n4 + C4 - 1) / C4;
  const int64_t per_cu = std::max<int64_t>(1, std::min<int64_t>(4, (160 * 1024) / static_cast<int64_t>(lds)));
  int64_t gx = std::max<int64_t>(1, 256 * per_cu / in.n_groups);
  gx = std::min<int64_t>(gx, tiles);
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(in.n_groups));
  k<<<grid, kRoundThreads, lds, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v, tiles);
  return check_launch("round kernel (persistent)");
}

constexpr int kNarrowThreads = 1024;

// The broadcast form's staging table - the ONE place its limits live: the launcher picks its
// instantiation from it (launch_round_bcast_nt) and the planner caps groups with it
// (bc_max_loads, round_plan_build), so a plan the planner returns always launches.
// J = float4 staging loads per lane, NT = 64 x waves threads.  Instantiated: J = 2 and 4 for
// every form, 6 at 768 threads, 8 at 512 threads and at 1024 threads with c4 = 32 and one
// workgroup per CU (the two-chunk form's 128 KiB tile; with two workgroups per CU 1024
// threads x 8 loads do not fit 64 VGPRs).
constexpr int bc_j_max(int c4, int nt, int wg_per_cu) {
  return nt == 512 ? 8 : nt == 768 ? 6 : (nt == 1024 && c4 == 32 && wg_per_cu == 1) ? 8 : 4;
}
// the J a launch of `loads` float4 staging loads per tile uses (0: more than the form stages)
constexpr int bc_j_for(int c4, int nt, int wg_per_cu, int64_t loads) {
  for (int j : {2, 4, 6, 8})
    if (j <= bc_j_max(c4, nt, wg_per_cu) && (j != 6 || nt == 768) && loads <= static_cast<int64_t>(j) * nt) return j;
  return 0;
}
// sources per group the records can address: 4096 float4 at c4 = 16, 8192 at c4 = 32 (256)
constexpr int64_t bc_max_loads(int c4, int waves, int wg_per_cu) {
  const int64_t j = bc_j_max(c4, 64 * waves, wg_per_cu);
  const int64_t cap = c4 == 32 ? 8192 : 4096;
  return j * 64 * waves < cap ? j * 64 * waves : cap;
}
static_assert(bc_j_for(16, 1024, 2, 4096) == 4 && bc_j_for(16, 1024, 2, 4097) == 0, "16 x 2");
static_assert(bc_j_for(32, 1024, 1, 8192) == 8 && bc_j_for(32, 1024, 2, 4097) == 0, "two-chunk form");
static_assert(bc_j_for(16, 768, 2, 4096) == 6 && bc_j_for(16, 512, 2, 4096) == 8, "12 x 2, 8 x 2");

// Workgroups of `kernel` resident per CU with `lds` bytes of dynamic LDS (registers and LDS both
// count), asked from the runtime once per (kernel, lds) - a persistent grid larger than what is
// resident would run a second, straggling wave of workgroups.
std::mutex g_occ_mu;
std::vector<std::tuple<const void*, size_t, int>> g_occ;

int resident_per_cu(const void* kernel, int threads, size_t lds) {
  std::lock_guard<std::mutex> lk(g_occ_mu);
  for (const auto& e : g_occ)
    if (std::get<0>(e) == kernel && std::get<1>(e) == lds) return std::get<2>(e);
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, threads, lds) != hipSuccess) nb = 1;
  nb = std::max(1, nb);
  g_occ.emplace_back(kernel, lds, nb);
  return nb;
}

// 16-B staging lanes for bf16 pools (W16 in k_round_f32_narrow): on unless TAL_NARROW_W16=0 (A/B)
bool narrow_w16_enabled() {
  static const bool on = [] {
    const char* e = getenv("TAL_NARROW_W16");
    return !(e && e[0] == '0');
  }();
  return on;
}

template <int C4, int J, bool EXACT, typename T = float, bool ROWW = false>
int32_t launch_round_narrow_jr(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                               const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  const size_t lds = static_cast<size_t>(in.lds_bytes);
  // two workgroups per CU when their LDS allows it (registers capped at 64), else one with the
  // row extents in registers
  constexpr int kNP = J >= 12 ? kNarrowPasses / 2 : kNarrowPasses;  // J = 12: VGPRs for the staging
  auto k = k_round_f32_narrow<C4, kNarrowThreads, J, kNP, EXACT, T, ROWW>;
  if constexpr (J <= 4)
    if (2 * lds <= 160 * 1024) k = k_round_f32_narrow<C4, kNarrowThreads, J, 0, EXACT, T, ROWW>;
  if constexpr (kIsBf16<T> && J >= 2 && J <= 4) {
    // whole chunk pairs per row (an even chunk count and stride) from a 16-B aligned base: no
    // pair reaches past a row's last chunk
    if (narrow_w16_enabled() && n4 % 2 == 0 && (ld_in / 4) % 2 == 0 && (reinterpret_cast<uintptr_t>(pin) & 15) == 0)
      k = 2 * lds <= 160 * 1024 ? k_round_f32_narrow<C4, kNarrowThreads, J, 0, EXACT, T, ROWW, true>
                                : k_round_f32_narrow<C4, kNarrowThreads, J, kNP, EXACT, T, ROWW, true>;
  }
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const int64_t tiles = (n4 + C4 - 1) / C4;
  const int64_t per_cu = resident_per_cu(reinterpret_cast<const void*>(k), kNarrowThreads, lds);
  int64_t gx = std::max<int64_t>(1, 256 * per_cu / in.n_groups);
  gx = std::min<int64_t>(gx, tiles);
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(in.n_groups));
  k<<<grid, kNarrowThreads, lds, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v, tiles);
  return check_launch("round kernel (narrow tiles)");
}

template <int C4, int J, bool EXACT, typename T = float>
int32_t launch_round_narrow_j(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                              const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  return in.narrow_roww ? launch_round_narrow_jr<C4, J, EXACT, T, true>(pin, ld_in, pout, ld_out, n4, v, in, s)
                        : launch_round_narrow_jr<C4, J, EXACT, T, false>(pin, ld_in, pout, ld_out, n4, v, in, s);
}

// Broadcast form: NT = 64 x the plan's waves; J staging loads per lane cover the largest group.
template <int C4, int NT, int J, bool EXACT, typename T>
int32_t launch_round_bcast_j(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                             const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  const size_t lds = static_cast<size_t>(in.lds_bytes);
  const bool one = in.bc_wg_per_cu == 1;  // one workgroup per CU: 128 VGPRs at 1024 threads
  const bool w16 = kIsBf16<T> && J % 2 == 0 && narrow_w16_enabled() && n4 % 2 == 0 && (ld_in / 4) % 2 == 0 &&
                   (reinterpret_cast<uintptr_t>(pin) & 15) == 0;
  // J = 8 at 1024 threads (the two-chunk form's 128 KiB tile) only with one workgroup per CU
  constexpr bool kOneOnly = NT == 1024 && J == 8;
  if (kOneOnly && !one) return fail(TAL_ERR_CAPACITY, "broadcast-form round plan: this tile needs one workgroup per CU");
  auto k = (one || kOneOnly) ? k_round_f32_narrow<C4, NT, J, 1, EXACT, T, false, false, true>
                             : k_round_f32_narrow<C4, NT, J, kOneOnly ? 1 : 0, EXACT, T, false, false, true>;
  if constexpr (kIsBf16<T> && J % 2 == 0) {
    if (w16)
      k = (one || kOneOnly) ? k_round_f32_narrow<C4, NT, J, 1, EXACT, T, false, true, true>
                            : k_round_f32_narrow<C4, NT, J, kOneOnly ? 1 : 0, EXACT, T, false, true, true>;
  }
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const int64_t tiles = (n4 + C4 - 1) / C4;
  const int64_t per_cu = resident_per_cu(reinterpret_cast<const void*>(k), NT, lds);
  int64_t gx = std::max<int64_t>(1, 256 * per_cu / in.n_groups);
  gx = std::min<int64_t>(gx, tiles);
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(in.n_groups));
  k<<<grid, NT, lds, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v, tiles);
  return check_launch("round kernel (narrow tiles, broadcast form)");
}

template <int C4, int NT, bool EXACT, typename T>
int32_t launch_round_bcast_nt(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                              const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  const int64_t loads = static_cast<int64_t>(in.max_src) * C4;  // float4 staging loads per tile
  switch (bc_j_for(C4, NT, in.bc_wg_per_cu, loads)) {  // the staging table (bc_j_max)
    case 2:
      return launch_round_bcast_j<C4, NT, 2, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
    case 4:
      return launch_round_bcast_j<C4, NT, 4, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
    case 6:
      if constexpr (NT == 768)
        return launch_round_bcast_j<C4, NT, 6, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
      break;
    case 8:
      if constexpr (bc_j_max(C4, NT, 1) >= 8)
        return launch_round_bcast_j<C4, NT, 8, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
      break;
    default:
      break;
  }
  // a plan from tal_round_plan_build_bcast never gets here (its groups are capped by the same
  // table); a hand-made or mismatched plan does
  return fail(TAL_ERR_CAPACITY, "broadcast-form round plan: group tile too large for the workgroup");
}

template <int C4, bool EXACT, typename T>
int32_t launch_round_bcast(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                           const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  if (in.narrow_bcast == 8) return launch_round_bcast_nt<C4, 512, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  if (in.narrow_bcast == 12) return launch_round_bcast_nt<C4, 768, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  return launch_round_bcast_nt<C4, 1024, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
}

template <int C4, bool EXACT, typename T = float>
int32_t launch_round_narrow(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                            const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  if (in.narrow_bcast) return launch_round_bcast<C4, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  const int64_t loads = static_cast<int64_t>(in.max_src) * C4;  // float4 staging loads per tile
  if (loads <= 1LL * kNarrowThreads) return launch_round_narrow_j<C4, 1, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  if (loads <= 2LL * kNarrowThreads) return launch_round_narrow_j<C4, 2, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  if (loads <= 4LL * kNarrowThreads) return launch_round_narrow_j<C4, 4, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  if (loads <= 8LL * kNarrowThreads) return launch_round_narrow_j<C4, 8, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  if (loads <= 12LL * kNarrowThreads) return launch_round_narrow_j<C4, 12, EXACT, T>(pin, ld_in, pout, ld_out, n4, v, in, s);
  return fail(TAL_ERR_CAPACITY, "narrow round plan: group tile larger than 160 KiB");
}

// ------------------------------------------------------------------------------------------
// K3c: uniform-weight cliques.  A clique block is m <= 64 sources s_0 < ... < s_{m-1} sharing
// one fp32 weight w, with output rows for (some of) its members, member i's operands being, in
// reference order, every other member ascending and then s_i itself (a complete graph's or a
// barbell's clique rows under the unweighted strategy).  The products fl(w * x_j) are the same
// for every row, and row i = ((S_i + p_{i+1}) + ... + p_{m-1}) + p_i with S_i the in-order
// prefix p_0 + ... + p_{i-1}, which all later rows extend: one thread keeps p_0..p_{m-1} of its
// two columns in registers, reads each source once from HBM, and emits every row with
// ~m^2/2 adds instead of m^2 multiply-adds.  Bitwise the reference: each row's additions are
// its own left-to-right chain (the prefix is shared, not reassociated); padding terms are -0.0
// (x + -0.0 == x for every x), S_0 = -0.0 (-0.0 + p == p).  FMA mode keeps x_j and fuses
// fma(w, x_j, acc); its padding is the zero whose product with w is -0.0.
// ------------------------------------------------------------------------------------------
constexpr int kCliqueMax = 64;
constexpr int kCliqueExtra = 4;        // attached rows per clique block
constexpr int kCliqueExtraWords = 12;  // {out, v bits, mask lo, mask hi, self member, self row,
                                       //  n_ext, ext row 0, ext row 1, ext pos 0, ext pos 1, 0}
static_assert(4 + 2 * kCliqueMax + kCliqueExtra * kCliqueExtraWords == TAL_CLIQUE_WORDS, "table layout");

typedef float v2f __attribute__((ext_vector_type(2)));

template <bool EXACT>
__device__ __forceinline__ v2f clique_term(v2f acc, float w, v2f p) {
  if constexpr (EXACT) return v2f{__fadd_rn(acc.x, p.x), __fadd_rn(acc.y, p.y)};
  else return v2f{__builtin_fmaf(w, p.x, acc.x), __builtin_fmaf(w, p.y, acc.y)};
}

typedef float v8f __attribute__((ext_vector_type(8)));

// Four clique chains stepped at once (k-th pair of lanes = chain k): one IR operation per step.
template <bool EXACT>
__device__ __forceinline__ v8f clique_term4(v8f acc, float w, v8f p) {
  if constexpr (EXACT) return acc + p;  // IEEE adds, one rounding each (no contraction: -ffp-contract=off)
  else return __builtin_elementwise_fma(v8f{w, w, w, w, w, w, w, w}, p, acc);
}

// A zero the compiler cannot see through: table reads indexed with it stay where they are
// instead of being hoisted to the top of the kernel, where 128 live row indices would spill
// the scalar register file.
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}

// Columns e and e + 1 of every row of clique block `t`.
// acc (+)= fl(v * x) for an attached row's operand (raw value x)
template <bool EXACT>
__device__ __forceinline__ v2f clique_xterm(v2f acc, float v, v2f x) {
  if constexpr (EXACT) return v2f{__fadd_rn(acc.x, __fmul_rn(v, x.x)), __fadd_rn(acc.y, __fmul_rn(v, x.y))};
  else return v2f{__builtin_fmaf(v, x.x, acc.x), __builtin_fmaf(v, x.y, acc.y)};
}

template <int MMAX, bool EXACT>
__global__ __launch_bounds__(kBlock) void k_round_clique(const float* __restrict__ pin, int64_t ld_in,
                                                         float* __restrict__ pout, int64_t ld_out,
                                                         int64_t n2, const int32_t* __restrict__ table) {
  const int32_t* t = table + static_cast<int64_t>(blockIdx.y) * TAL_CLIQUE_WORDS;
  const int64_t c2 = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (c2 >= n2) return;
  const int64_t e = 2 * c2;
  const int m = t[0];
  const float w = __int_as_float(t[1]);
  const float pad = EXACT ? -0.f : (__float_as_uint(w) >> 31 ? 0.f : -0.f);
  // every load is issued unconditionally (a padding slot re-reads member 0, an L2 hit) so all
  // MMAX loads are in flight before the first use; the padding value is selected afterwards
  v2f p[MMAX];
#pragma unroll
  for (int j = 0; j < MMAX; ++j) {
    const float* src = pin + static_cast<int64_t>(t[4 + (j < m ? j : 0) + opaque_zero()]) * ld_in + e;
    p[j] = __builtin_nontemporal_load(reinterpret_cast<const v2f*>(src));
    // batches of 8: the scheduler would otherwise compute all row addresses first
    if (j % 8 == 7) __builtin_amdgcn_sched_barrier(0);
  }
  // attached rows (a barbell's bridge nodes): most operands are members, read from the raw
  // values in registers before they become products; at most two other neighbors and an
  // optional non-member self are loaded here.  Each is its own in-order chain with its weight.
  const int n_extra = t[2];
  for (int q = 0; q < n_extra; ++q) {
    const int32_t* xr = t + 4 + 2 * kCliqueMax + q * kCliqueExtraWords + opaque_zero();
    const float v = __int_as_float(xr[1]);
    const uint32_t lo = static_cast<uint32_t>(xr[2]), hi = static_cast<uint32_t>(xr[3]);
    const int self_m = xr[4], self_e = xr[5], n_ext = xr[6];
    const int pos0 = n_ext > 0 ? xr[9] : -1, pos1 = n_ext > 1 ? xr[10] : -1;
    auto ld_row = [&](int r) {
      return __builtin_nontemporal_load(reinterpret_cast<const v2f*>(pin + static_cast<int64_t>(r) * ld_in + e));
    };
    const v2f e0 = n_ext > 0 ? ld_row(xr[7]) : v2f{0.f, 0.f};
    const v2f e1 = n_ext > 1 ? ld_row(xr[8]) : v2f{0.f, 0.f};
    v2f xs = self_e >= 0 ? ld_row(self_e) : v2f{0.f, 0.f};
    v2f acc = v2f{-0.f, -0.f};
#pragma unroll
    for (int j = 0; j <= MMAX; ++j) {
      if (pos0 == j) acc = clique_xterm<EXACT>(acc, v, e0);
      if (pos1 == j) acc = clique_xterm<EXACT>(acc, v, e1);
      if (j < MMAX) {
        if (((j < 32 ? lo >> j : hi >> (j - 32)) & 1u) != 0u) acc = clique_xterm<EXACT>(acc, v, p[j]);
        if (self_m == j) xs = p[j];
      }
    }
    acc = clique_xterm<EXACT>(acc, v, xs);
    __builtin_nontemporal_store(acc, reinterpret_cast<v2f*>(pout + static_cast<int64_t>(xr[0]) * ld_out + e));
  }
#pragma unroll
  for (int j = 0; j < MMAX; ++j) {
    if constexpr (EXACT) p[j] = v2f{__fmul_rn(w, p[j].x), __fmul_rn(w, p[j].y)};
    if (j >= m) p[j] = v2f{pad, pad};
  }
  // Rows four at a time: row r = ((S_r + p[r+1]) + ... + p[MMAX-1]) + p[r], S_{r+1} = S_r + p[r]
  // (each row its own in-order chain, as the reference sums it).  The four chains are
  // independent, so their packed adds interleave: one chain's back-to-back dependent
  // v_pk_add_f32 needed an s_nop between every pair (1,512 per column pair at MMAX 60), which
  // stretched each wavefront's compute phase and with it the time without loads in flight.
  static_assert(MMAX % 4 == 0, "rows are taken in fours");
  v2f s = v2f{-0.f, -0.f};
#pragma unroll
  for (int i = 0; i < MMAX; i += 4) {
    int orow[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) orow[k] = i + k < m ? t[4 + kCliqueMax + i + k + opaque_zero()] : -1;  // wave-uniform
    v2f sp[4];  // S_i .. S_{i+3}
    sp[0] = s;
#pragma unroll
    for (int k = 1; k < 4; ++k) sp[k] = clique_term<EXACT>(sp[k - 1], w, p[i + k - 1]);
    if (orow[0] >= 0 || orow[1] >= 0 || orow[2] >= 0 || orow[3] >= 0) {
      // heads: row i+k takes p[i+k+1 .. i+3] before the four chains run in step
      v2f a[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        a[k] = sp[k];
#pragma unroll
        for (int j = i + k + 1; j < i + 4; ++j) a[k] = clique_term<EXACT>(a[k], w, p[j]);
      }
      // the four chains as one 8-wide vector: each step is one IR operation (four packed adds
      // on natural register pairs), which the compiler can neither split into four loops nor
      // sink into the stores' branches
      v8f q = {a[0].x, a[0].y, a[1].x, a[1].y, a[2].x, a[2].y, a[3].x, a[3].y};
#pragma unroll
      for (int j = i + 4; j < MMAX; ++j) q = clique_term4<EXACT>(q, w, v8f{p[j].x, p[j].y, p[j].x, p[j].y,
                                                                           p[j].x, p[j].y, p[j].x, p[j].y});
      q = clique_term4<EXACT>(q, w, v8f{p[i].x, p[i].y, p[i + 1].x, p[i + 1].y, p[i + 2].x, p[i + 2].y,
                                        p[i + 3].x, p[i + 3].y});
#pragma unroll
      for (int k = 0; k < 4; ++k) a[k] = v2f{q[2 * k], q[2 * k + 1]};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (orow[k] >= 0)
          __builtin_nontemporal_store(a[k], reinterpret_cast<v2f*>(pout + static_cast<int64_t>(orow[k]) * ld_out + e));
    }
    s = clique_term<EXACT>(sp[3], w, p[i + 3]);
  }
}

// The last column of an odd-width round: one thread per member row, its chain in reference
// order (every other member ascending, then itself).
template <bool EXACT>
__global__ __launch_bounds__(kCliqueMax) void k_round_clique_tail(const float* __restrict__ pin, int64_t ld_in,
                                                                  float* __restrict__ pout, int64_t ld_out,
                                                                  int64_t e, const int32_t* __restrict__ table) {
  const int32_t* t = table + static_cast<int64_t>(blockIdx.x) * TAL_CLIQUE_WORDS;
  const int m = t[0];
  const int i = threadIdx.x;
  if (i >= m) return;
  const int orow = t[4 + kCliqueMax + i];
  if (orow < 0) return;
  const float w = __int_as_float(t[1]);
  float acc = -0.f;
  for (int j = 0; j <= m; ++j) {
    if (j == i) continue;
    const int k = j < m ? j : i;
    const float x = pin[static_cast<int64_t>(t[4 + k]) * ld_in + e];
    acc = EXACT ? __fadd_rn(acc, __fmul_rn(w, x)) : __builtin_fmaf(w, x, acc);
  }
  pout[static_cast<int64_t>(orow) * ld_out + e] = acc;
}

// The last column for a block's attached rows: one thread per attached row.
template <bool EXACT>
__global__ __launch_bounds__(kCliqueExtra) void k_round_clique_tail_extra(const float* __restrict__ pin,
                                                                          int64_t ld_in, float* __restrict__ pout,
                                                                          int64_t ld_out, int64_t e,
                                                                          const int32_t* __restrict__ table) {
  const int32_t* t = table + static_cast<int64_t>(blockIdx.x) * TAL_CLIQUE_WORDS;
  const int q = threadIdx.x;
  if (q >= t[2]) return;
  const int32_t* xr = t + 4 + 2 * kCliqueMax + q * kCliqueExtraWords;
  const float v = __int_as_float(xr[1]);
  const uint32_t lo = static_cast<uint32_t>(xr[2]), hi = static_cast<uint32_t>(xr[3]);
  const int n_ext = xr[6];
  auto x_of = [&](int r) { return pin[static_cast<int64_t>(r) * ld_in + e]; };
  auto term = [&](float a, float x) { return EXACT ? __fadd_rn(a, __fmul_rn(v, x)) : __builtin_fmaf(v, x, a); };
  float acc = -0.f;
  for (int j = 0; j <= kCliqueMax; ++j) {
    for (int k = 0; k < n_ext; ++k)
      if (xr[9 + k] == j) acc = term(acc, x_of(xr[7 + k]));
    if (j < kCliqueMax && (((j < 32 ? lo >> j : hi >> (j - 32)) & 1u) != 0u)) acc = term(acc, x_of(t[4 + j]));
  }
  acc = term(acc, x_of(xr[4] >= 0 ? t[4 + xr[4]] : xr[5]));
  pout[static_cast<int64_t>(xr[0]) * ld_out + e] = acc;
}

template <bool EXACT>
int32_t launch_round_clique(const float* pin, int64_t ld_in, float* pout, int64_t ld_out, int64_t n,
                            const int32_t* table, int32_t n_cliques, int32_t mmax, hipStream_t s) {
  const int64_t n2 = n / 2;
  const int64_t blocks = (n2 + kBlock - 1) / kBlock;
  if (blocks > 0x7fffffffLL || n_cliques > 65535) return fail(TAL_ERR_INVALID, "clique round: grid too large");
  if (n2 > 0) {
    const dim3 grid(static_cast<unsigned>(blocks), static_cast<unsigned>(n_cliques));
    // the chains run over MMAX slots, the ones past the largest clique adding -0.0: MMAX close
    // to the clique size keeps those no-op adds few (a 60-member barbell clique under MMAX 64
    // spent 13 % of its adds on padding)
    if (mmax <= 16) k_round_clique<16, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else if (mmax <= 32) k_round_clique<32, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else if (mmax <= 40) k_round_clique<40, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else if (mmax <= 48) k_round_clique<48, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else if (mmax <= 56) k_round_clique<56, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else if (mmax <= 60) k_round_clique<60, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    else k_round_clique<64, EXACT><<<grid, kBlock, 0, s>>>(pin, ld_in, pout, ld_out, n2, table);
    int32_t rc = check_launch("clique round kernel");
    if (rc) return rc;
  }
  if (n % 2) {
    k_round_clique_tail<EXACT><<<n_cliques, kCliqueMax, 0, s>>>(pin, ld_in, pout, ld_out, n - 1, table);
    int32_t rc = check_launch("clique round tail kernel");
    if (rc) return rc;
    k_round_clique_tail_extra<EXACT><<<n_cliques, kCliqueExtra, 0, s>>>(pin, ld_in, pout, ld_out, n - 1, table);
    return check_launch("clique round tail kernel (attached rows)");
  }
  return TAL_OK;
}

// ------------------------------------------------------------------------------------------
// K3r: rounds whose rows fall into groups of <= 64 distinct sources (community graphs, BASELINE
// config 5's stochastic block model), each group's sources held in VGPRs.
//   One wave = one item (group g, piece t): the 64 lanes load 2 elements each (fp32 8 B, bf16
//   4 B unpacked to fp32) of every source of g at columns [128 t, 128 t + 128) straight into
//   v[32 : 32 + 2 S) - no LDS, no barrier - then emit every row of g for that piece in
//   reference order.  A row's operand is read from the registers by its wave-uniform slot with
//   the VGPR index mode (s_set_gpr_idx_on / _idx / _off, SRC0): the multiply itself reads
//   v[32 + 2 slot], so the register file stands in for K3n's LDS tile and no per-operand LDS
//   read or extra move is issued.  The loads and the indexed arithmetic are inline asm on
//   fixed registers (the compiler keeps the source tuples pinned there: every asm lists them
//   as operands); rows run in pairs so that no packed instruction reads the result of the one
//   right before it (gfx950 needs a wait state there, which the pairs fill with the other row).
//   Items are handed to waves per XCD label (blockIdx % 8): the groups of one piece run on one
//   XCD at the same time, so a source shared by several groups is fetched from HBM once and
//   served to the others by that XCD's L2.
//   Arithmetic: EXACT = fp32 multiply then fp32 add per operand from -0.0 (-0 + p = p), the
//   reference's order; FMA = fused chains from -0.0 (fma(w, x0, -0) = fl(w x0)), bitwise K1-FMA.
//   bf16 pools: FMA only (fp32 accumulation, one rounding at the store).
// ------------------------------------------------------------------------------------------
typedef float v32f __attribute__((ext_vector_type(32)));
typedef __attribute__((address_space(4))) const uint64_t* ConstU64;
constexpr int kRegMaxSrc = 64;
constexpr int kRegPiece = 128;  // elements per item: 64 lanes x 2

// plain (temporal) loads: a source shared by several groups of a piece is served to the others
// by the XCD's L2 (non-temporal loads were measured fetching every group's sources from HBM:
// 4.1x the bytes on config 5)
#define TAL_RLD2(a, b, k) "global_load_dwordx2 v[" #a ":" #b "], %17, %" #k "\n\t"
#define TAL_RLD1(b, k) "global_load_dword v" #b ", %17, %" #k "\n\t"
#define TAL_RUNP(a, b) "v_lshlrev_b32 v" #a ", 16, v" #b "\n\tv_and_b32 v" #b ", 0xffff0000, v" #b "\n\t"
#define TAL_RF32_0 \
  TAL_RLD2(32,33,1) TAL_RLD2(34,35,2) TAL_RLD2(36,37,3) TAL_RLD2(38,39,4) \
  TAL_RLD2(40,41,5) TAL_RLD2(42,43,6) TAL_RLD2(44,45,7) TAL_RLD2(46,47,8) \
  TAL_RLD2(48,49,9) TAL_RLD2(50,51,10) TAL_RLD2(52,53,11) TAL_RLD2(54,55,12) \
  TAL_RLD2(56,57,13) TAL_RLD2(58,59,14) TAL_RLD2(60,61,15) TAL_RLD2(62,63,16)
#define TAL_RF32_1 \
  TAL_RLD2(64,65,1) TAL_RLD2(66,67,2) TAL_RLD2(68,69,3) TAL_RLD2(70,71,4) \
  TAL_RLD2(72,73,5) TAL_RLD2(74,75,6) TAL_RLD2(76,77,7) TAL_RLD2(78,79,8) \
  TAL_RLD2(80,81,9) TAL_RLD2(82,83,10) TAL_RLD2(84,85,11) TAL_RLD2(86,87,12) \
  TAL_RLD2(88,89,13) TAL_RLD2(90,91,14) TAL_RLD2(92,93,15) TAL_RLD2(94,95,16)
#define TAL_RF32_2 \
  TAL_RLD2(96,97,1) TAL_RLD2(98,99,2) TAL_RLD2(100,101,3) TAL_RLD2(102,103,4) \
  TAL_RLD2(104,105,5) TAL_RLD2(106,107,6) TAL_RLD2(108,109,7) TAL_RLD2(110,111,8) \
  TAL_RLD2(112,113,9) TAL_RLD2(114,115,10) TAL_RLD2(116,117,11) TAL_RLD2(118,119,12) \
  TAL_RLD2(120,121,13) TAL_RLD2(122,123,14) TAL_RLD2(124,125,15) TAL_RLD2(126,127,16)
#define TAL_RF32_3 \
  TAL_RLD2(128,129,1) TAL_RLD2(130,131,2) TAL_RLD2(132,133,3) TAL_RLD2(134,135,4) \
  TAL_RLD2(136,137,5) TAL_RLD2(138,139,6) TAL_RLD2(140,141,7) TAL_RLD2(142,143,8) \
  TAL_RLD2(144,145,9) TAL_RLD2(146,147,10) TAL_RLD2(148,149,11) TAL_RLD2(150,151,12) \
  TAL_RLD2(152,153,13) TAL_RLD2(154,155,14) TAL_RLD2(156,157,15) TAL_RLD2(158,159,16)
#define TAL_RB16_0 \
  TAL_RLD1(33,1) TAL_RLD1(35,2) TAL_RLD1(37,3) TAL_RLD1(39,4) \
  TAL_RLD1(41,5) TAL_RLD1(43,6) TAL_RLD1(45,7) TAL_RLD1(47,8) \
  TAL_RLD1(49,9) TAL_RLD1(51,10) TAL_RLD1(53,11) TAL_RLD1(55,12) \
  TAL_RLD1(57,13) TAL_RLD1(59,14) TAL_RLD1(61,15) TAL_RLD1(63,16)
#define TAL_RB16_1 \
  TAL_RLD1(65,1) TAL_RLD1(67,2) TAL_RLD1(69,3) TAL_RLD1(71,4) \
  TAL_RLD1(73,5) TAL_RLD1(75,6) TAL_RLD1(77,7) TAL_RLD1(79,8) \
  TAL_RLD1(81,9) TAL_RLD1(83,10) TAL_RLD1(85,11) TAL_RLD1(87,12) \
  TAL_RLD1(89,13) TAL_RLD1(91,14) TAL_RLD1(93,15) TAL_RLD1(95,16)
#define TAL_RB16_2 \
  TAL_RLD1(97,1) TAL_RLD1(99,2) TAL_RLD1(101,3) TAL_RLD1(103,4) \
  TAL_RLD1(105,5) TAL_RLD1(107,6) TAL_RLD1(109,7) TAL_RLD1(111,8) \
  TAL_RLD1(113,9) TAL_RLD1(115,10) TAL_RLD1(117,11) TAL_RLD1(119,12) \
  TAL_RLD1(121,13) TAL_RLD1(123,14) TAL_RLD1(125,15) TAL_RLD1(127,16)
#define TAL_RB16_3 \
  TAL_RLD1(129,1) TAL_RLD1(131,2) TAL_RLD1(133,3) TAL_RLD1(135,4) \
  TAL_RLD1(137,5) TAL_RLD1(139,6) TAL_RLD1(141,7) TAL_RLD1(143,8) \
  TAL_RLD1(145,9) TAL_RLD1(147,10) TAL_RLD1(149,11) TAL_RLD1(151,12) \
  TAL_RLD1(153,13) TAL_RLD1(155,14) TAL_RLD1(157,15) TAL_RLD1(159,16)
#define TAL_RUNP_0 \
  TAL_RUNP(32,33) TAL_RUNP(34,35) TAL_RUNP(36,37) TAL_RUNP(38,39) \
  TAL_RUNP(40,41) TAL_RUNP(42,43) TAL_RUNP(44,45) TAL_RUNP(46,47) \
  TAL_RUNP(48,49) TAL_RUNP(50,51) TAL_RUNP(52,53) TAL_RUNP(54,55) \
  TAL_RUNP(56,57) TAL_RUNP(58,59) TAL_RUNP(60,61) TAL_RUNP(62,63)
#define TAL_RUNP_1 \
  TAL_RUNP(64,65) TAL_RUNP(66,67) TAL_RUNP(68,69) TAL_RUNP(70,71) \
  TAL_RUNP(72,73) TAL_RUNP(74,75) TAL_RUNP(76,77) TAL_RUNP(78,79) \
  TAL_RUNP(80,81) TAL_RUNP(82,83) TAL_RUNP(84,85) TAL_RUNP(86,87) \
  TAL_RUNP(88,89) TAL_RUNP(90,91) TAL_RUNP(92,93) TAL_RUNP(94,95)
#define TAL_RUNP_2 \
  TAL_RUNP(96,97) TAL_RUNP(98,99) TAL_RUNP(100,101) TAL_RUNP(102,103) \
  TAL_RUNP(104,105) TAL_RUNP(106,107) TAL_RUNP(108,109) TAL_RUNP(110,111) \
  TAL_RUNP(112,113) TAL_RUNP(114,115) TAL_RUNP(116,117) TAL_RUNP(118,119) \
  TAL_RUNP(120,121) TAL_RUNP(122,123) TAL_RUNP(124,125) TAL_RUNP(126,127)
#define TAL_RUNP_3 \
  TAL_RUNP(128,129) TAL_RUNP(130,131) TAL_RUNP(132,133) TAL_RUNP(134,135) \
  TAL_RUNP(136,137) TAL_RUNP(138,139) TAL_RUNP(140,141) TAL_RUNP(142,143) \
  TAL_RUNP(144,145) TAL_RUNP(146,147) TAL_RUNP(148,149) TAL_RUNP(150,151) \
  TAL_RUNP(152,153) TAL_RUNP(154,155) TAL_RUNP(156,157) TAL_RUNP(158,159)

#define TAL_RB16(b)                                                                                 \
  "s"(b[0]), "s"(b[1]), "s"(b[2]), "s"(b[3]), "s"(b[4]), "s"(b[5]), "s"(b[6]), "s"(b[7]), "s"(b[8]), \
      "s"(b[9]), "s"(b[10]), "s"(b[11]), "s"(b[12]), "s"(b[13]), "s"(b[14]), "s"(b[15])
#define TAL_RX1 "{v[32:63]}"(X0)
#define TAL_RX2 TAL_RX1, "{v[64:95]}"(X1)
#define TAL_RX3 TAL_RX2, "{v[96:127]}"(X2)
#define TAL_RX4 TAL_RX3, "{v[128:159]}"(X3)
#define TAL_UNP(...) __VA_ARGS__
// one inline-asm statement with the NB source tuples appended to its inputs
#define TAL_RASM(TMPL, OUTS, INS)                                                      \
  do {                                                                                 \
    if constexpr (NB == 1) asm volatile(TMPL : TAL_UNP OUTS : TAL_UNP INS, TAL_RX1);   \
    else if constexpr (NB == 2) asm volatile(TMPL : TAL_UNP OUTS : TAL_UNP INS, TAL_RX2); \
    else if constexpr (NB == 3) asm volatile(TMPL : TAL_UNP OUTS : TAL_UNP INS, TAL_RX3); \
    else asm volatile(TMPL : TAL_UNP OUTS : TAL_UNP INS, TAL_RX4);                     \
  } while (0)

// 16 sources (block J) into v[32 + 32 J ...]: b = per-source byte addresses of the piece
// (wave-uniform), off = the lane's byte offset in it.  No wait: reg_wait follows all blocks.
template <int J, bool BF16>
__device__ __forceinline__ v32f reg_load_block(const uint64_t* b, uint32_t off) {
  v32f X;
#define TAL_RLOAD(TM, R) asm volatile(TM : "=&{" R "}"(X) : TAL_RB16(b), "v"(off) : "memory")
  if constexpr (!BF16) {
    if constexpr (J == 0) TAL_RLOAD(TAL_RF32_0, "v[32:63]");
    else if constexpr (J == 1) TAL_RLOAD(TAL_RF32_1, "v[64:95]");
    else if constexpr (J == 2) TAL_RLOAD(TAL_RF32_2, "v[96:127]");
    else TAL_RLOAD(TAL_RF32_3, "v[128:159]");
  } else {  // the packed pair goes to the odd register; reg_wait unpacks it in place
    if constexpr (J == 0) TAL_RLOAD(TAL_RB16_0, "v[32:63]");
    else if constexpr (J == 1) TAL_RLOAD(TAL_RB16_1, "v[64:95]");
    else if constexpr (J == 2) TAL_RLOAD(TAL_RB16_2, "v[96:127]");
    else TAL_RLOAD(TAL_RB16_3, "v[128:159]");
  }
#undef TAL_RLOAD
  return X;
}

template <int NB, bool BF16>
__device__ __forceinline__ void reg_wait(v32f& X0, v32f& X1, v32f& X2, v32f& X3) {
  if constexpr (!BF16) {
    if constexpr (NB == 1) asm volatile("s_waitcnt vmcnt(0)" : "+{v[32:63]}"(X0));
    else if constexpr (NB == 2) asm volatile("s_waitcnt vmcnt(0)" : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1));
    else if constexpr (NB == 3)
      asm volatile("s_waitcnt vmcnt(0)" : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1), "+{v[96:127]}"(X2));
    else
      asm volatile("s_waitcnt vmcnt(0)"
                   : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1), "+{v[96:127]}"(X2), "+{v[128:159]}"(X3));
  } else {  // bf16 pair (lo = element 0) -> two fp32: v[2k] = lo << 16, v[2k+1] = hi & 0xffff0000
    if constexpr (NB == 1) asm volatile("s_waitcnt vmcnt(0)\n\t" TAL_RUNP_0 : "+{v[32:63]}"(X0));
    else if constexpr (NB == 2)
      asm volatile("s_waitcnt vmcnt(0)\n\t" TAL_RUNP_0 TAL_RUNP_1 : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1));
    else if constexpr (NB == 3)
      asm volatile("s_waitcnt vmcnt(0)\n\t" TAL_RUNP_0 TAL_RUNP_1 TAL_RUNP_2
                   : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1), "+{v[96:127]}"(X2));
    else
      asm volatile("s_waitcnt vmcnt(0)\n\t" TAL_RUNP_0 TAL_RUNP_1 TAL_RUNP_2 TAL_RUNP_3
                   : "+{v[32:63]}"(X0), "+{v[64:95]}"(X1), "+{v[96:127]}"(X2), "+{v[128:159]}"(X3));
  }
}

// Operands come in RECORDS of 16 dwords, one per trip of a row pair (A, B): {A's four register
// offsets, B's four, A's four fp32 weights, B's four}; a register offset is 2 x the source's slot
// in the group, and a row with fewer operands than its trips hold is padded with the NEUTRAL
// operand (offset 32 x NB: the register pair held at -0.0 past the sources, weight +0.0), whose
// product -0.0 leaves any accumulator unchanged (x + -0 = x, also for x = +0 and NaN; fma(0,
// -0, x) = x).  A pair's trips run as ONE inline-asm loop: the next record is read into the
// other half of s[40:71] (s_load_dwordx16) while the current one computes, so a trip is one
// scalar load, the index switch per operand and four loop instructions — no copies, no address
// arithmetic per operand (v3's per-operand SALU stream was the kernel's limit).  A weight
// reaches the packed multiply as a 64-bit SGPR pair: op_sel_hi:[1,0] broadcasts its low dword,
// op_sel:[0,1] op_sel_hi:[1,1] its high dword.  The two rows' chains are interleaved, so no
// packed instruction reads the result of the one right before it (gfx950 needs a wait state
// there).  M0, which the index mode writes, is used by nothing else in this kernel (no LDS).

// one trip: i* / j* = A's / B's index SGPRs, wa* / wb* = their weight pairs
#define TAL_TRIP_E(i0, i1, i2, i3, j0, j1, j2, j3, wa01, wa23, wb01, wb23)                            \
  "s_set_gpr_idx_on " i0 ", gpr_idx(SRC0)\n\t"                                                          \
  "v_pk_mul_f32 %[t0], v[32:33], " wa01 " op_sel_hi:[1,0]\n\t"                                          \
  "s_set_gpr_idx_idx " j0 "\n\tv_pk_mul_f32 %[t4], v[32:33], " wb01 " op_sel_hi:[1,0]\n\t"              \
  "s_set_gpr_idx_idx " i1 "\n\tv_pk_mul_f32 %[t1], v[32:33], " wa01 " op_sel:[0,1] op_sel_hi:[1,1]\n\t" \
  "s_set_gpr_idx_idx " j1 "\n\tv_pk_mul_f32 %[t5], v[32:33], " wb01 " op_sel:[0,1] op_sel_hi:[1,1]\n\t" \
  "s_set_gpr_idx_idx " i2 "\n\tv_pk_mul_f32 %[t2], v[32:33], " wa23 " op_sel_hi:[1,0]\n\t"              \
  "s_set_gpr_idx_idx " j2 "\n\tv_pk_mul_f32 %[t6], v[32:33], " wb23 " op_sel_hi:[1,0]\n\t"              \
  "s_set_gpr_idx_idx " i3 "\n\tv_pk_mul_f32 %[t3], v[32:33], " wa23 " op_sel:[0,1] op_sel_hi:[1,1]\n\t" \
  "s_set_gpr_idx_idx " j3 "\n\tv_pk_mul_f32 %[t7], v[32:33], " wb23 " op_sel:[0,1] op_sel_hi:[1,1]\n\t" \
  "s_set_gpr_idx_off\n\t"                                                                               \
  "v_pk_add_f32 %[ca], %[ca], %[t0]\n\tv_pk_add_f32 %[cb], %[cb], %[t4]\n\t"                            \
  "v_pk_add_f32 %[ca], %[ca], %[t1]\n\tv_pk_add_f32 %[cb], %[cb], %[t5]\n\t"                            \
  "v_pk_add_f32 %[ca], %[ca], %[t2]\n\tv_pk_add_f32 %[cb], %[cb], %[t6]\n\t"                            \
  "v_pk_add_f32 %[ca], %[ca], %[t3]\n\tv_pk_add_f32 %[cb], %[cb], %[t7]\n\t"
#define TAL_TRIP_F(i0, i1, i2, i3, j0, j1, j2, j3, wa01, wa23, wb01, wb23)                                          \
  "s_set_gpr_idx_on " i0 ", gpr_idx(SRC0)\n\t"                                                                        \
  "v_pk_fma_f32 %[ca], v[32:33], " wa01 ", %[ca] op_sel_hi:[1,0,1]\n\t"                                               \
  "s_set_gpr_idx_idx " j0 "\n\tv_pk_fma_f32 %[cb], v[32:33], " wb01 ", %[cb] op_sel_hi:[1,0,1]\n\t"                   \
  "s_set_gpr_idx_idx " i1 "\n\tv_pk_fma_f32 %[ca], v[32:33], " wa01 ", %[ca] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"    \
  "s_set_gpr_idx_idx " j1 "\n\tv_pk_fma_f32 %[cb], v[32:33], " wb01 ", %[cb] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"    \
  "s_set_gpr_idx_idx " i2 "\n\tv_pk_fma_f32 %[ca], v[32:33], " wa23 ", %[ca] op_sel_hi:[1,0,1]\n\t"                   \
  "s_set_gpr_idx_idx " j2 "\n\tv_pk_fma_f32 %[cb], v[32:33], " wb23 ", %[cb] op_sel_hi:[1,0,1]\n\t"                   \
  "s_set_gpr_idx_idx " i3 "\n\tv_pk_fma_f32 %[ca], v[32:33], " wa23 ", %[ca] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"    \
  "s_set_gpr_idx_idx " j3 "\n\tv_pk_fma_f32 %[cb], v[32:33], " wb23 ", %[cb] op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"    \
  "s_set_gpr_idx_off\n\t"
#define TAL_TRIP_P(TRIP) TRIP("s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s[48:49]", "s[50:51]", "s[52:53]", "s[54:55]")
#define TAL_TRIP_Q(TRIP) TRIP("s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s[64:65]", "s[66:67]", "s[68:69]", "s[70:71]")
// the pair loop over records at byte offsets off, off + 64, ... (from the table base), last =
// off + 64 x trips: after a trip the offset register points one past the record being loaded,
// i.e. at off + 64 (k + 2) after record k, and record k + 1 exists iff that is <= last
#define TAL_PAIR_LOOP(TRIP)                                     \
  "s_load_dwordx16 s[40:55], %[base], %[off]\n\t"                \
  "s_add_u32 %[off], %[off], 64\n\t"                             \
  "s_waitcnt lgkmcnt(0)\n"                                       \
  "1:\n\t"                                                       \
  "s_load_dwordx16 s[56:71], %[base], %[off]\n\t"                \
  "s_add_u32 %[off], %[off], 64\n\t" TAL_TRIP_P(TRIP)           \
  "s_cmp_le_u32 %[off], %[last]\n\t"                             \
  "s_waitcnt lgkmcnt(0)\n\t"                                     \
  "s_cbranch_scc0 2f\n\t"                                        \
  "s_load_dwordx16 s[40:55], %[base], %[off]\n\t"                \
  "s_add_u32 %[off], %[off], 64\n\t" TAL_TRIP_Q(TRIP)           \
  "s_cmp_le_u32 %[off], %[last]\n\t"                             \
  "s_waitcnt lgkmcnt(0)\n\t"                                     \
  "s_cbranch_scc1 1b\n"                                          \
  "2:"
#define TAL_REC_CLOBBERS                                                                                    \
  "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", \
      "s55", "s56", "s57", "s58", "s59", "s60", "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68",     \
      "s69", "s70", "s71", "scc"

template <int NB, bool EXACT>
__device__ __forceinline__ void reg_pair(v2f_t& ca, v2f_t& cb, uint64_t base, uint32_t off, uint32_t last,
                                         const v32f& X0, const v32f& X1, const v32f& X2, const v32f& X3,
                                         const v2f_t& Z) {
#define TAL_PASM(TMPL, OUTS, ZR)                                                                             \
  do {                                                                                                       \
    if constexpr (NB == 1)                                                                                   \
      asm volatile(TMPL : TAL_UNP OUTS : [base] "s"(base), [last] "s"(last), TAL_RX1, ZR(Z) : TAL_REC_CLOBBERS); \
    else if constexpr (NB == 2)                                                                              \
      asm volatile(TMPL : TAL_UNP OUTS : [base] "s"(base), [last] "s"(last), TAL_RX2, ZR(Z) : TAL_REC_CLOBBERS); \
    else if constexpr (NB == 3)                                                                              \
      asm volatile(TMPL : TAL_UNP OUTS : [base] "s"(base), [last] "s"(last), TAL_RX3, ZR(Z) : TAL_REC_CLOBBERS); \
    else                                                                                                     \
      asm volatile(TMPL : TAL_UNP OUTS : [base] "s"(base), [last] "s"(last), TAL_RX4, ZR(Z) : TAL_REC_CLOBBERS); \
  } while (0)
#define TAL_Z1 "{v[64:65]}"
#define TAL_Z2 "{v[96:97]}"
#define TAL_Z3 "{v[128:129]}"
#define TAL_Z4 "{v[160:161]}"
  if constexpr (EXACT) {
    v2f_t t0, t1, t2, t3, t4, t5, t6, t7;
#define TAL_OUTS_E                                                                                          \
  ([ca] "+v"(ca), [cb] "+v"(cb), [off] "+s"(off), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),           \
   [t3] "=&v"(t3), [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7))
    if constexpr (NB == 1) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_E), TAL_OUTS_E, TAL_Z1);
    else if constexpr (NB == 2) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_E), TAL_OUTS_E, TAL_Z2);
    else if constexpr (NB == 3) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_E), TAL_OUTS_E, TAL_Z3);
    else TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_E), TAL_OUTS_E, TAL_Z4);
#undef TAL_OUTS_E
  } else {
#define TAL_OUTS_F ([ca] "+v"(ca), [cb] "+v"(cb), [off] "+s"(off))
    if constexpr (NB == 1) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_F), TAL_OUTS_F, TAL_Z1);
    else if constexpr (NB == 2) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_F), TAL_OUTS_F, TAL_Z2);
    else if constexpr (NB == 3) TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_F), TAL_OUTS_F, TAL_Z3);
    else TAL_PASM(TAL_PAIR_LOOP(TAL_TRIP_F), TAL_OUTS_F, TAL_Z4);
#undef TAL_OUTS_F
  }
#undef TAL_Z1
#undef TAL_Z2
#undef TAL_Z3
#undef TAL_Z4
#undef TAL_PASM
}

// Output stores with sc1: the line leaves the XCD's L2 instead of staying there (plain / nt
// stores keep it), so the outputs do not push the sources the other groups of the piece are
// about to read out of L2 (MI355X_MICROARCH.md, store flavours).
template <typename T>
__device__ __forceinline__ void reg_store(T* pout, int64_t ld_out, int32_t row, int64_t col, int64_t n, v2f_t acc) {
  if (col >= n) return;
  const int64_t e = static_cast<int64_t>(row) * ld_out + col;
  if constexpr (kIsBf16<T>) {
    uint32_t q = cvt_bf16x2(acc.x, acc.y);
    if (__builtin_isunordered(acc.x, acc.y)) q = store_bf16x2(acc.x, acc.y);
    if (col + 1 < n) asm volatile("global_store_dword %0, %1, off sc1" : : "v"(pout + e), "v"(q) : "memory");
    else pout[e] = static_cast<uint16_t>(q & 0xffffu);
  } else {
    if (col + 1 < n) asm volatile("global_store_dwordx2 %0, %1, off sc1" : : "v"(pout + e), "v"(acc) : "memory");
    else pout[e] = acc.x;
  }
}

// Table (int32, device): groups [G][4] {first source, sources, first pair, pairs}; at off_src
// the source pool rows (each group's list padded to 16 x NB entries; src_off = their byte
// offsets in the pool); at off_pairs (a multiple of 4) pair records [P][4] {out row A, out row
// B or -1, trips, byte offset of the first trip record}, a group's pairs consecutive; at off_rec
// (a multiple of 16) the trip records [T][16], followed by one record of padding (the loop reads
// one record ahead).
template <int NB, typename T, bool EXACT>
__global__ __launch_bounds__(256) void k_round_reg(const T* __restrict__ pin, T* __restrict__ pout, int64_t ld_out,
                                                   int64_t n, const int32_t* __restrict__ table,
                                                   const int64_t* __restrict__ src_off, int32_t n_groups,
                                                   int32_t off_pairs, int32_t n_pieces,
                                                   int32_t* __restrict__ ticket) {
  constexpr bool kB = kIsBf16<T>;
  constexpr int kEs = kB ? 2 : 4;
  const ConstI32 tab = (ConstI32)table;
  const ConstU64 soff = (ConstU64)src_off;
  const uint64_t base = reinterpret_cast<uint64_t>(table);
  const int lane = threadIdx.x & 63;
  const int label = static_cast<int>(blockIdx.x & 7u);
  const int pieces_l = n_pieces > label ? (n_pieces - 1 - label) / 8 + 1 : 0;
  const int items = pieces_l * n_groups;
  // Items are dealt in order by a per-label ticket counter (one atomic per item), so the items in
  // flight on an XCD stay a window of consecutive pieces: with a static round-robin the waves
  // drift apart over thousands of items and the groups of one piece no longer meet in L2
  // (profiles/r03/k3r: HBM reads 3.9x -> 1.0-1.5x the algorithmic bytes).  The next ticket is
  // taken once the current item's sources have arrived, not when the item starts: a ticket held
  // for a whole item spreads a piece's groups over two item times, and the window (pieces whose
  // sources must stay in L2) doubles past the 4 MB L2.
  int32_t* my_ticket = ticket + 16 * label;  // 64 B apart
  auto take = [&]() {
    int t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(my_ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(t);
  };
  const v2f_t zn = {-0.f, -0.f};  // the neutral operand's register pair
  int s_next = take();
  v32f X0, X1, X2, X3;
  for (;;) {
    const int s = s_next;
    if (s >= items) break;
    const int q = s / n_groups, g = s - q * n_groups;
    const int piece = q * 8 + label;
    const int s0 = tab[4 * g], p0 = tab[4 * g + 2], np = tab[4 * g + 3];
    const int64_t col = static_cast<int64_t>(piece) * kRegPiece + 2 * lane;
    const uint32_t loff = col < n ? static_cast<uint32_t>(2 * lane * kEs) : 0u;  // past n: the piece's start
    const uint64_t pbase = reinterpret_cast<uint64_t>(pin) + static_cast<uint64_t>(piece) * (kRegPiece * kEs);
    uint64_t b[16];
    // each block's 16 source offsets come in two 8-dword scalar loads, one wait
#define TAL_RBASES(J)                                                                            \
    _Pragma("unroll") for (int k = 0; k < 16; ++k)                                               \
      b[k] = pbase + static_cast<uint64_t>(soff[s0 + (J) * 16 + k]);
    TAL_RBASES(0)
    X0 = reg_load_block<0, kB>(b, loff);
    if constexpr (NB > 1) { TAL_RBASES(1) X1 = reg_load_block<1, kB>(b, loff); }
    if constexpr (NB > 2) { TAL_RBASES(2) X2 = reg_load_block<2, kB>(b, loff); }
    if constexpr (NB > 3) { TAL_RBASES(3) X3 = reg_load_block<3, kB>(b, loff); }
#undef TAL_RBASES
    reg_wait<NB, kB>(X0, X1, X2, X3);
    s_next = take();
    for (int p = 0; p < np; ++p) {
      const u32x4 pr = ((const __attribute__((address_space(4))) u32x4*)(tab + off_pairs))[p0 + p];
      v2f_t ca = {-0.f, -0.f}, cb = {-0.f, -0.f};
      const uint32_t off = pr[3];
      const uint32_t last = off + 64u * pr[2];  // the loop goes on while (next record's offset + 64) <= last
      reg_pair<NB, EXACT>(ca, cb, base, off, last, X0, X1, X2, X3, zn);
      reg_store<T>(pout, ld_out, static_cast<int32_t>(pr[0]), col, n, ca);
      if (static_cast<int32_t>(pr[1]) >= 0) reg_store<T>(pout, ld_out, static_cast<int32_t>(pr[1]), col, n, cb);
    }
  }
}

// The register round's item tickets: eight counters 64 B apart, one per XCD label, reset on the
// stream before each launch.  One buffer per (device, stream): launches on one stream are
// ordered, so they never share counters with a launch in flight elsewhere (two streams sharing
// one buffer could reset or advance each other's counters and skip items).  The library's only
// device allocations: 512 B per (device, stream) used, made on first use.
constexpr size_t kRegTicketBytes = 8 * 64;

int32_t reg_tickets(hipStream_t stream, int32_t** out) {
  static std::mutex mu;
  static std::vector<std::tuple<int, hipStream_t, int32_t*>> bufs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(TAL_ERR_HIP, "register round: no current device");
  std::lock_guard<std::mutex> lk(mu);
  for (const auto& b : bufs)
    if (std::get<0>(b) == dev && std::get<1>(b) == stream) {
      *out = std::get<2>(b);
      return TAL_OK;
    }
  void* p = nullptr;
  if (hipMalloc(&p, kRegTicketBytes) != hipSuccess) return fail(TAL_ERR_HIP, "register round: ticket allocation failed");
  bufs.emplace_back(dev, stream, static_cast<int32_t*>(p));
  *out = static_cast<int32_t*>(p);
  return TAL_OK;
}

// Compute units of the current device, asked once per device (thread-safe).
int32_t device_cus(int* n_cu) {
  static std::mutex mu;
  static std::vector<int> per_dev;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(TAL_ERR_HIP, "no current device");
  std::lock_guard<std::mutex> lk(mu);
  if (per_dev.size() <= static_cast<size_t>(dev)) per_dev.resize(dev + 1, 0);
  if (per_dev[dev] == 0 &&
      hipDeviceGetAttribute(&per_dev[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return fail(TAL_ERR_HIP, "multiprocessor count query failed");
  *n_cu = per_dev[dev];
  return TAL_OK;
}

template <int NB, typename T, bool EXACT>
int32_t launch_round_reg_nb(const T* pin, T* pout, int64_t ld_out, int64_t n, const int32_t* table,
                            const int64_t* src_off, int32_t n_groups, int32_t off_pairs, int32_t n_pieces,
                            hipStream_t s) {
  int n_cu = 0;
  if (int32_t rc = device_cus(&n_cu)) return rc;
  // resident workgroups per CU: cached per kernel under a mutex (resident_per_cu)
  const int blocks_per_cu = resident_per_cu(reinterpret_cast<const void*>(k_round_reg<NB, T, EXACT>), 256, 0);
  // persistent: every resident wave (TAL_REG_BLOCKS_PER_CU caps it: A/B probes of how many
  // pieces are in flight per XCD), a multiple of 8 blocks (XCD labels)
  int bpc = blocks_per_cu;
  if (const char* e = getenv("TAL_REG_BLOCKS_PER_CU")) bpc = std::max(1, std::min(bpc, atoi(e)));
  const int grid = std::max(8, n_cu * bpc / 8 * 8);
  int32_t* ticket = nullptr;
  if (int32_t rc = reg_tickets(s, &ticket)) return rc;
  if (hipMemsetAsync(ticket, 0, kRegTicketBytes, s) != hipSuccess)
    return fail(TAL_ERR_HIP, "register round: ticket reset failed");
  k_round_reg<NB, T, EXACT><<<grid, 256, 0, s>>>(pin, pout, ld_out, n, table, src_off, n_groups, off_pairs, n_pieces,
                                                 ticket);
  return check_launch("register round kernel");
}

template <typename T, bool EXACT>
int32_t launch_round_reg(const T* pin, T* pout, int64_t ld_out, int64_t n, const int32_t* table,
                         const int64_t* src_off, int32_t n_groups, int32_t off_pairs, int32_t max_src, hipStream_t s) {
  const int64_t n_pieces = (n + kRegPiece - 1) / kRegPiece;
  if (n_pieces * n_groups >= (1LL << 31)) return fail(TAL_ERR_INVALID, "register round: too many items");
  const int np = static_cast<int>(n_pieces);
#define TAL_REG_NB(NBV) launch_round_reg_nb<NBV, T, EXACT>(pin, pout, ld_out, n, table, src_off, n_groups, off_pairs, np, s)
  if (max_src <= 16) return TAL_REG_NB(1);
  if (max_src <= 32) return TAL_REG_NB(2);
  if (max_src <= 48) return TAL_REG_NB(3);
  return TAL_REG_NB(4);
#undef TAL_REG_NB
}

template <int NT, bool EXACT>
int32_t launch_round_stream_nt(const float* pin, int64_t ld_in, float* pout, int64_t ld_out, int64_t n4,
                               const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  auto k = k_round_stream<NT, EXACT>;
  const size_t lds = stream_lds_bytes(NT / 64 * kStreamPerWave);
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const int per_cu = resident_per_cu(reinterpret_cast<const void*>(k), NT, lds);
  const int64_t tiles = (n4 + 63) / 64;
  int64_t gx = std::max<int64_t>(1, 256LL * per_cu / in.n_groups);
  gx = std::min<int64_t>(gx, tiles);
  const dim3 grid(static_cast<unsigned>(gx), static_cast<unsigned>(in.n_groups));
  k<<<grid, NT, lds, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v, tiles);
  return check_launch("round kernel (streamed)");
}

int32_t launch_round_stream(const float* pin, int64_t ld_in, float* pout, int64_t ld_out, int64_t n4,
                            const PlanView& v, const tal_round_plan_info& in, bool exact, hipStream_t s) {
  if (in.stream_cs == 8 * kStreamPerWave)
    return exact ? launch_round_stream_nt<512, true>(pin, ld_in, pout, ld_out, n4, v, in, s)
                 : launch_round_stream_nt<512, false>(pin, ld_in, pout, ld_out, n4, v, in, s);
  return exact ? launch_round_stream_nt<1024, true>(pin, ld_in, pout, ld_out, n4, v, in, s)
               : launch_round_stream_nt<1024, false>(pin, ld_in, pout, ld_out, n4, v, in, s);
}

template <bool IS_I64>
int32_t launch_round_stream_scalar(const void* pin, int64_t ld_in, void* pout, int64_t ld_out, int64_t e0,
                                   int64_t n, const PlanView& v, const tal_round_plan_info& in, bool exact,
                                   hipStream_t s) {
  if (n <= e0) return TAL_OK;
  const int64_t tc = std::max<int64_t>(1, std::min<int64_t>(64, (160 * 1024) / (4LL * in.max_src)));
  if (in.max_src > 160 * 1024 / 4) return fail(TAL_ERR_CAPACITY, "streamed plan: group too large for the tail kernel");
  const size_t lds = static_cast<size_t>(in.max_src) * tc * 4;
  const int64_t tiles = (n - e0 + tc - 1) / tc;
  if (tiles > 0x7fffffff) return fail(TAL_ERR_INVALID, "too many tiles");
  auto k = (IS_I64 || exact) ? k_round_stream_scalar<IS_I64, true> : k_round_stream_scalar<IS_I64, false>;
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(in.n_groups));
  k<<<grid, kBlock, lds, s>>>(pin, ld_in, pout, ld_out, e0, n, v, static_cast<int>(tc));
  return check_launch("round scalar kernel (streamed plan)");
}

template <int C4, bool EXACT, bool DENSE, typename T = float>
int32_t launch_round_vec(const T* pin, int64_t ld_in, T* pout, int64_t ld_out, int64_t n4,
                         const PlanView& v, const tal_round_plan_info& in, hipStream_t s) {
  constexpr int kRoundThreads = round_threads<C4>();
  const size_t lds = static_cast<size_t>(in.max_src) * C4 * 16;
  const int64_t loads = static_cast<int64_t>(in.max_src) * C4;  // float4 staging loads per tile
  if (loads <= 1LL * kRoundThreads) return launch_round_persistent<C4, 1, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
  if (loads <= 2LL * kRoundThreads) return launch_round_persistent<C4, 2, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
  if (loads <= 4LL * kRoundThreads) return launch_round_persistent<C4, 4, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
  if (loads <= 8LL * kRoundThreads) return launch_round_persistent<C4, 8, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
  if constexpr (kRoundThreads <= 512) {  // 16-20 float4 in flight per lane: 512-thread blocks only (VGPRs)
    if (loads <= 16LL * kRoundThreads) return launch_round_persistent<C4, 16, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
    if (loads <= 20LL * kRoundThreads) return launch_round_persistent<C4, 20, EXACT, DENSE, T>(pin, ld_in, pout, ld_out, n4, v, in, lds, s);
  }
  auto k = k_round_f32_tiled<C4, kRoundThreads, EXACT, DENSE, T>;
  int32_t rc = ensure_lds(reinterpret_cast<const void*>(k), lds);
  if (rc) return rc;
  const int64_t tiles = (n4 + C4 - 1) / C4;
  if (tiles > 0x7fffffff) return fail(TAL_ERR_INVALID, "too many tiles");
  const dim3 grid(static_cast<unsigned>(tiles), static_cast<unsigned>(in.n_groups));
  k<<<grid, kRoundThreads, lds, s>>>(pin, ld_in / 4, pout, ld_out / 4, n4, v);
  return check_launch("round kernel");
}

// ------------------------------------------------------------------------------------------
// K2: the reference's model cosine similarity, bit for bit (see tal_agg.h and the C restatement
// oracle/cosine_oracle.c, which pins the operation order against the reference's own values).
// Reference: cosine_similarity, decentralized_client.py:661-681 over torch's CPU kernels:
//   n = clamp_min(vector_norm(x, 2, dim=1), 1e-6);  s = sum_dim1((x1 / n1) * (x2 / n2));
//   mean = cascade_sum(s) / numel;  result = (0 + mean_0 + mean_1 + ...) / n_params.
// Every output of a tensor viewed [A, I, B] is one element (I == 1), one row (B == 1: 8
// threads per row, one per lane of torch's 8-wide vector accumulators) or one column (B > 1:
// one thread, strided); the per-tensor means and the final average follow in two small
// kernels.  All arithmetic is single-rounding fp32 (__f*_rn), in torch's order.
// ------------------------------------------------------------------------------------------
constexpr int kCosMaxPairs = 32;
constexpr int kCosHdr = 4;         // plan words: {n_seg, n_out, torch intra-op threads, staged chunks}
constexpr int kCosMaxThreads = 1024;
constexpr int64_t kCosGrain = 32768;  // at::internal::GRAIN_SIZE
constexpr int kCosSegWords = 7;    // {offset, A, I, B, out_offset, kind, outputs per chunk}
constexpr int kCosChunkWords = 4;  // {seg, first output, count, staged (1) or direct (0)}
constexpr int kCosBlock = 256;
constexpr int kCosVw = 8;          // Vectorized<float> width of torch's sum kernel (as run)
enum { kCosElem = 0, kCosRow = 1, kCosCol = 2 };
constexpr int64_t cos_chunk_outputs(int kind) { return kind == kCosRow ? kCosBlock / kCosVw : kCosBlock; }

// Streamed column chunks (round 6): a column tensor [A, I, B] with B < 32 (the 3 x 3
// convolutions) reduces every output (o, k) over i with stride B; the direct form's lanes gather
// from ~7 slabs 18 KB apart (37.7 L1 accesses per load instruction, profiles/r05/r05k2pmc).  The
// streamed form walks i in steps of kColIc: each step moves x[o0 .. o0 + Ob, i0 .. i0 + kColIc, :]
// of every model of the workgroup (Ob contiguous runs of kColIc B floats each) into LDS with
// coalesced loads, kColDepth steps in flight in registers, and every chain - one thread per
// (output, model) or (output, pair) - advances kColIc elements from LDS in its own order.  Two
// kernels: the norms (torch's FMA chains, every distinct model once, k_cos_col_norms), then the
// products (each pair's four streams' level-0 runs, pushed into their cascades every 64 elements
// as multi_row_sum pushes them, k_cos_col_prods).  Every chain of a chunk runs at once: the
// round-6 slab-staged form ran one 512 x 9 slab per workgroup, 36 norm chains on 256 threads.
constexpr int kColIc = 16;       // i per step: a quarter of the four streams' 16-element runs
constexpr int kColThreads = 256;
constexpr int kColModels = 9;    // LDS models per workgroup: 9 models' norms, or a + 8 pairs' b
constexpr int kColPairs = 8;     // pairs per product workgroup when they share a (else 4)
constexpr int kColMS = 1024;     // LDS floats per model at most (Ob pitch-padded output blocks)
constexpr int kColDepth = 4;     // steps in flight
static_assert(31 * kColIc <= 2 * kColThreads, "a model's step is at most two elements per thread");

__host__ __device__ inline int64_t cos_log2_ceil(int64_t x) {
  int64_t r = 0;
  while ((int64_t{1} << r) < x) ++r;
  return r;
}

// torch multi_row_sum's level width over `size` elements: 2^max(4, ceil(log2 size) / 4)
__host__ __device__ inline int64_t cos_lp(int64_t size) {
  const int64_t l = cos_log2_ceil(size) / 4;
  return l > 4 ? l : 4;
}

// output blocks (B outputs each) per streamed chunk: chains Ob B <= 28 (B < 29)
__host__ __device__ inline int cos_col_ob(int64_t B) { return B >= 28 ? 1 : static_cast<int>(28 / B); }

// LDS pitch of one output block's kColIc x B floats, = B (mod 64): chain c = o B + k of model
// slot g (model stride Ob P = Ob B = C, mod 64) reads bank (g C + c + i B) mod 64 = (lane + i B)
// mod 64, so a wave's reads of one element index are conflict-free
__host__ __device__ inline int cos_col_pitch(int64_t B) {
  const int b = static_cast<int>(B);
  return b * kColIc + ((b * (1 - kColIc)) % 64 + 64) % 64;
}

// a column tensor runs the streamed form when B < 32 and its streams' level-0 runs are 16 long
// (multi_row_sum's level width 2^4: every I below 2^22)
inline bool cos_col_streamed(int kind, int64_t I, int64_t B) {
  return kind == kCosCol && B < 32 && cos_lp(I / 4) == 4 && cos_col_ob(B) * cos_col_pitch(B) <= kColMS;
}

struct CosPairs {
  const float* a[kCosMaxPairs];
  const float* b[kCosMaxPairs];
};

__device__ __forceinline__ int64_t cos_ceil_log2(int64_t x) {
  int64_t r = 0;
  while ((int64_t{1} << r) < x) ++r;
  return r;
}

// torch multi_row_sum: NR interleaved streams load(i, k), a 4-level cascade whose level
// boundaries depend only on i (so one column of a 32-column chunk is the NR = 1 case)
template <int NR, class Load>
__device__ __forceinline__ void cos_multi_row(Load load, int64_t size, float* out) {
  constexpr int kL = 4;
  const int64_t lp = cos_ceil_log2(size) / kL > 4 ? cos_ceil_log2(size) / kL : 4;
  const int64_t step = int64_t{1} << lp;
  const int64_t mask0 = step - 1;
  float acc[kL][NR];
#pragma unroll
  for (int j = 0; j < kL; ++j)
#pragma unroll
    for (int k = 0; k < NR; ++k) acc[j][k] = 0.f;
  int64_t i = 0;
  // the level-0 run of `step` (a power of two >= 16) elements in batches of kU: the batch's
  // loads are issued together, then added in order (each stream k keeps torch's order), so a
  // serial chain waits on one memory latency per batch, not per element (8 ran 0.62-0.63 ms
  // for 8 ResNet-50 pairs, 4 0.68, one element at a time 0.94)
  constexpr int kU = 8;
  while (i + step <= size) {
    for (int64_t j = 0; j < step; j += kU, i += kU) {
      float v[kU][NR];
#pragma unroll
      for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int k = 0; k < NR; ++k) v[u][k] = load(i + u, k);
#pragma unroll
      for (int u = 0; u < kU; ++u)
#pragma unroll
        for (int k = 0; k < NR; ++k) acc[0][k] = __fadd_rn(acc[0][k], v[u][k]);
    }
#pragma unroll
    for (int j = 1; j < kL; ++j) {
#pragma unroll
      for (int k = 0; k < NR; ++k) {
        acc[j][k] = __fadd_rn(acc[j][k], acc[j - 1][k]);
        acc[j - 1][k] = 0.f;
      }
      if ((i & (mask0 << (j * lp))) != 0) break;
    }
  }
  for (; i < size; ++i)
#pragma unroll
    for (int k = 0; k < NR; ++k) acc[0][k] = __fadd_rn(acc[0][k], load(i, k));
#pragma unroll
  for (int j = 1; j < kL; ++j)
#pragma unroll
    for (int k = 0; k < NR; ++k) acc[0][k] = __fadd_rn(acc[0][k], acc[j][k]);
#pragma unroll
  for (int k = 0; k < NR; ++k) out[k] = acc[0][k];
}

// torch row_sum: 4 interleaved partial sums (element 4 i + k), the remainder into partial 0,
// partials 1..3 added to partial 0 in order
template <class Load>
__device__ __forceinline__ float cos_row_sum(Load load, int64_t size) {
  float ps[4];
  const int64_t si = size / 4;
  cos_multi_row<4>([&](int64_t i, int k) { return load(i * 4 + k); }, si, ps);
  for (int64_t i = si * 4; i < size; ++i) ps[0] = __fadd_rn(ps[0], load(i));
  for (int k = 1; k < 4; ++k) ps[0] = __fadd_rn(ps[0], ps[k]);
  return ps[0];
}

// correctly rounded sqrt (llvm.sqrt.f32 under HIP's default correctly-rounded divide/sqrt);
// HIP's __fsqrt_rn is the native approximation unless OCML_BASIC_ROUNDED_OPERATIONS is set
__device__ __forceinline__ float cos_sqrt_rn(float x) { return __builtin_sqrtf(x); }

__device__ __forceinline__ float cos_clamp(float n) { return n < 1e-6f ? 1e-6f : n; }  // NaN stays NaN

// x / n with the IEEE division's result, without its scaling steps (each writes VCC, which the
// next division's v_div_fmas reads, so divisions serialise): y = RN(1 / n) once per norm, then
// q0 = RN(x y) and q = RN(q0 + RN(x - n q0) y) (both fused).  Equal to RN(x / n) for n in
// [2^-40, 2^40] and |x| in [2^-50, 2^60) (every intermediate is normal, so the result depends
// only on the two mantissas: all 2^46 pairs checked on the GPU, tools/div_exhaustive.hip,
// profiles/r05/r05div); callers take __fdiv_rn outside it.
__device__ __forceinline__ float cos_rdiv(float x, float n, float y) {
  const float q0 = __fmul_rn(x, y);
  return __fmaf_rn(__fmaf_rn(-n, q0, x), y, q0);
}
__device__ __forceinline__ bool cos_rdiv_x(float x) {  // |x| in [2^-50, 2^60)
  return (__float_as_uint(x) & 0x7fffffffu) - 0x26800000u < 0x37000000u;
}
__device__ __forceinline__ bool cos_rdiv_n(float n) {  // n in [2^-40, 2^40]
  return __float_as_uint(n) - 0x2B800000u <= 0x28000000u;
}

// Lane sums of one 8-thread group (threads g*8 .. g*8+7 of the wave) delivered to its thread 0
// in lane order: out = first + v_0 + v_1 + ... + v_7 (every thread of the wave must call it).
__device__ __forceinline__ float cos_group_fold(float first, float v, int gbase) {
  float r = first;
#pragma unroll
  for (int l = 0; l < kCosVw; ++l) r = __fadd_rn(r, __shfl(v, gbase + l, 64));
  return r;
}

__global__ __launch_bounds__(kCosBlock) void k_cosine_outputs(CosPairs pr, const int64_t* __restrict__ plan,
                                                              int n_seg, int cnt, int64_t n_direct,
                                                              float* __restrict__ s_all) {
  // XCD-aware order: dispatch deals workgroups round-robin over the 8 XCDs, so workgroup 8 k + x
  // takes pair k % cnt of direct chunk 8 (k / cnt) + x: a chunk's pairs run one after another
  // on XCD x, and all but the first find the chunk's `a` rows in that XCD's L2
  const int64_t kq = blockIdx.x >> 3;
  const int pair = static_cast<int>(kq % cnt);
  const int64_t c = kq / cnt * 8 + (blockIdx.x & 7);
  if (c >= n_direct) return;
  const int64_t n_out = plan[1];
  const int64_t* ch = plan + kCosHdr + kCosSegWords * static_cast<int64_t>(n_seg) +
                      kCosChunkWords * (plan[3] + c);  // after the streamed chunks
  const int64_t* sg = plan + kCosHdr + kCosSegWords * ch[0];
  const int64_t first = ch[1], count = ch[2];
  const int64_t I = sg[2], B = sg[3];
  const int kind = static_cast<int>(sg[5]);
  const float* a = pr.a[pair] + sg[0];
  const float* b = pr.b[pair] + sg[0];
  float* s = s_all + static_cast<int64_t>(pair) * n_out + sg[4];
  const int tid = threadIdx.x;
  if (kind == kCosElem) {  // 1-D parameter unsqueezed to [n, 1]: norm |x|, one product
    const int64_t q = first + tid;
    if (q < first + count) {
      const float x = a[q], y = b[q];
      const float n1 = cos_clamp(cos_sqrt_rn(__fmaf_rn(x, x, 0.f)));
      const float n2 = cos_clamp(cos_sqrt_rn(__fmaf_rn(y, y, 0.f)));
      s[q] = __fadd_rn(0.f, __fmul_rn(__fdiv_rn(x, n1), __fdiv_rn(y, n2)));
    }
    return;
  }
  if (kind == kCosCol) {  // B > 1: reduced dim strided by B; one thread per (row, column)
    const int64_t q = first + tid;
    if (q >= first + count) return;
    const int64_t o = q / B, k = q % B;
    const float* x1 = a + o * I * B + k;
    const float* x2 = b + o * I * B + k;
    float m1 = 0.f, m2 = 0.f;  // torch NormTwoOps: fma in index order (loads in batches of 8)
    int64_t i0 = 0;
    for (; i0 + 8 <= I; i0 += 8) {
      float u1[8], u2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        u1[u] = x1[(i0 + u) * B];
        u2[u] = x2[(i0 + u) * B];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        m1 = __fmaf_rn(u1[u], u1[u], m1);
        m2 = __fmaf_rn(u2[u], u2[u], m2);
      }
    }
    for (int64_t i = i0; i < I; ++i) {
      m1 = __fmaf_rn(x1[i * B], x1[i * B], m1);
      m2 = __fmaf_rn(x2[i * B], x2[i * B], m2);
    }
    const float n1 = cos_clamp(cos_sqrt_rn(m1)), n2 = cos_clamp(cos_sqrt_rn(m2));
    auto prod = [&](int64_t i) { return __fmul_rn(__fdiv_rn(x1[i * B], n1), __fdiv_rn(x2[i * B], n2)); };
    float r;
    if (B >= kCosVw && k < B / 32 * 32) {  // columns in chunks of 32 share one cascade
      float c[1];
      cos_multi_row<1>([&](int64_t i, int) { return prod(i); }, I, c);
      r = c[0];
    } else {  // chunks of 8 and single columns: row_sum per column
      r = cos_row_sum(prod, I);
    }
    s[q] = __fadd_rn(0.f, r);
    return;
  }
  // kCosRow (B == 1, I > 1): reduced dim contiguous; 8 threads per row (torch's vector lanes)
  const int lane = tid & 63;
  const int l = lane & (kCosVw - 1);
  const int gbase = lane & ~(kCosVw - 1);
  const int64_t q = first + tid / kCosVw;
  const bool live = q < first + count;
  const float* x1 = a + (live ? q : first) * I;
  const float* x2 = b + (live ? q : first) * I;
  const int64_t vec_end = I - I % kCosVw;
  // vector_norm (reduce-lastdim kernel): lane accumulators fma over whole vectors
  float m1 = 0.f, m2 = 0.f;
  if (live) {  // loads in batches of 8 vectors, fma in index order
    int64_t d = l;
    for (; d + 7 * kCosVw < vec_end; d += 8 * kCosVw) {
      float u1[8], u2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        u1[u] = x1[d + u * kCosVw];
        u2[u] = x2[d + u * kCosVw];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        m1 = __fmaf_rn(u1[u], u1[u], m1);
        m2 = __fmaf_rn(u2[u], u2[u], m2);
      }
    }
    for (; d < vec_end; d += kCosVw) {
      m1 = __fmaf_rn(x1[d], x1[d], m1);
      m2 = __fmaf_rn(x2[d], x2[d], m2);
    }
  }
  float t1 = __shfl(m1, gbase, 64), t2 = __shfl(m2, gbase, 64);  // lane 0 starts the fold
  for (int j = 1; j < kCosVw; ++j) {
    t1 = __fadd_rn(t1, __shfl(m1, gbase + j, 64));
    t2 = __fadd_rn(t2, __shfl(m2, gbase + j, 64));
  }
  float n1 = 0.f, n2 = 0.f;
  if (l == 0 && live) {  // the tail: groups of 4 as square-then-add, the rest fused
    int64_t d = vec_end;
    const int64_t sep = (I - vec_end) / 4 * 4;
    for (int64_t e = 0; e < sep; ++e, ++d) {
      t1 = __fadd_rn(t1, __fmul_rn(x1[d], x1[d]));
      t2 = __fadd_rn(t2, __fmul_rn(x2[d], x2[d]));
    }
    for (; d < I; ++d) {
      t1 = __fmaf_rn(x1[d], x1[d], t1);
      t2 = __fmaf_rn(x2[d], x2[d], t2);
    }
    n1 = cos_clamp(cos_sqrt_rn(t1));
    n2 = cos_clamp(cos_sqrt_rn(t2));
  }
  n1 = __shfl(n1, gbase, 64);
  n2 = __shfl(n2, gbase, 64);
  // (the reciprocal division of the streamed column kernels does not pay here: with per-element
  // range checks the row tensors ran 0.255 -> 0.335 ms for ResNet-50's, with one check per row
  // (bounds of |x| gathered in the norm loop, a templated product phase) 0.259 ms; the row kind
  // is bound by its loads, not its divisions; profiles/r06/r06k/r06k14, r06k17)
  auto prod = [&](int64_t i) { return __fmul_rn(__fdiv_rn(x1[i], n1), __fdiv_rn(x2[i], n2)); };
  if (I < kCosVw) {  // scalar_inner_sum
    if (l == 0 && live) s[q] = __fadd_rn(0.f, cos_row_sum(prod, I));
    return;
  }
  // vectorized_inner_sum: lane l sums elements 8 i + l by row_sum; then the scalar tail from 0,
  // then the lanes in order
  const int64_t nv = I / kCosVw;
  const float lane_sum = live ? cos_row_sum([&](int64_t i) { return prod(i * kCosVw + l); }, nv) : 0.f;
  float tail = 0.f;
  if (l == 0 && live)
    for (int64_t k2 = nv * kCosVw; k2 < I; ++k2) tail = __fadd_rn(tail, prod(k2));
  const float fin = cos_group_fold(tail, lane_sum, gbase);
  if (l == 0 && live) s[q] = __fadd_rn(0.f, fin);
}


// ---- streamed column chunks (see kColIc) ---------------------------------------------------
struct ColChunk {
  int I, B, C, Cf, P, MS, Ob;
  int64_t off;   // element offset of the chunk's first output block in a model
  int64_t out0;  // the chunk's first output (plan-wide)
};

__device__ __forceinline__ ColChunk col_chunk(const int64_t* __restrict__ plan, int n_seg, int64_t c) {
  const int64_t* ch = plan + kCosHdr + kCosSegWords * static_cast<int64_t>(n_seg) + kCosChunkWords * c;
  const int64_t* sg = plan + kCosHdr + kCosSegWords * ch[0];
  ColChunk k;
  k.I = static_cast<int>(sg[2]);
  k.B = static_cast<int>(sg[3]);
  k.C = static_cast<int>(ch[2]);  // the chunk's outputs: Ob B (the tensor's last chunk: fewer blocks)
  k.Ob = k.C / k.B;
  k.Cf = cos_col_ob(k.B) * k.B;   // a full chunk's chains: the thread and bank pattern
  k.P = cos_col_pitch(k.B);
  k.MS = cos_col_ob(k.B) * k.P;
  k.off = sg[0] + ch[1] * k.I;     // first output o0 B -> element o0 I B
  k.out0 = sg[4] + ch[1];
  return k;
}

// One thread's share of a step.  A model's part of a step is Ob blocks x kColIc B floats <= 2
// kColThreads (Ob B <= 31), so thread t moves elements t and t + kColThreads of every model: one
// per-thread offset pair serves all the models, whose base pointers are uniform (SGPRs).
struct ColLoads {
  const float* gm[kColModels];  // model m's first element of the chunk
  int64_t go[2];                // offset of element h kColThreads + t in a model (without i0 B)
  int lo[2];                    // its LDS index in model 0's area (+ m MS)
  int r[2];                     // its position inside its block's kColIc B run; INT_MAX: none
  int nmod, MS;
};

__device__ __forceinline__ void col_loads_init(ColLoads& L, const float* const* gm, int nmod, const ColChunk& k) {
  const int run = kColIc * k.B;
  const int per_m = k.Ob * run;
#pragma unroll
  for (int m = 0; m < kColModels; ++m) L.gm[m] = gm[m] + k.off;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int e = static_cast<int>(threadIdx.x) + h * kColThreads;
    const int o = e / run, r = e - o * run;
    L.go[h] = static_cast<int64_t>(o) * k.I * k.B + r;
    L.lo[h] = o * k.P + r;
    L.r[h] = e < per_m ? r : 0x7fffffff;
  }
  L.nmod = nmod;
  L.MS = k.MS;
}

// The chunk's steps: kColDepth steps' loads in flight in a register ring; each step waits for
// its loads, writes them to LDS and issues the loads kColDepth steps ahead, then every chain
// advances over the step's n <= kColIc elements (step(i0, n)).  The loads are unconditional
// (a load outside the chunk re-reads the model's first chunk element and is not stored) and
// the steps run in whole groups of kColDepth, so the loop body is straight-line code and each
// step waits only for its own loads.
template <class Step>
__device__ __forceinline__ void col_stream(const ColLoads& L, int I, int B, float* lds, Step step) {
  const int nsteps = (I + kColIc - 1) / kColIc;
  float ring[kColDepth][2 * kColModels];
  int64_t go[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) go[h] = L.r[h] == 0x7fffffff ? 0 : L.go[h];
  auto issue = [&](float* v, int s) {
    const int i0 = s * kColIc;
    const int lim = min(kColIc, I - i0) * B;  // <= 0 past the last step
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t a = L.r[h] < lim ? go[h] + static_cast<int64_t>(i0) * B : 0;
#pragma unroll
      for (int m = 0; m < kColModels; ++m) v[2 * m + h] = L.gm[m][a];  // m >= nmod: the last model again
    }
  };
#pragma unroll
  for (int d = 0; d < kColDepth; ++d) issue(ring[d], d);
  for (int s0 = 0; s0 < nsteps; s0 += kColDepth) {
#pragma unroll
    for (int d = 0; d < kColDepth; ++d) {
      const int s = s0 + d;
      const int n = min(kColIc, I - s * kColIc);  // <= 0: no step (the group's tail)
      __syncthreads();  // the previous step's chains are done with the LDS
#pragma unroll
      for (int m = 0; m < kColModels; ++m)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (m < L.nmod && L.r[h] < n * B) lds[m * L.MS + L.lo[h]] = ring[d][2 * m + h];
      issue(ring[d], s + kColDepth);
      __syncthreads();
      if (n > 0) step(s * kColIc, n);
    }
  }
}

// Norms: one workgroup per (streamed chunk, group of model slots); thread (g, c): model slot
// m0 + g, output c of the chunk: |x| = sqrt(fma chain over i in index order), clamped (torch's
// NormTwoOps over dim 1, cosine_similarity's clamp_min), into nrm[slot n_out + output].
__global__ __launch_bounds__(kColThreads) void k_cos_col_norms(CosPairs pr, const int64_t* __restrict__ plan, int n_seg,
                                                              int cnt, int same_a, float* __restrict__ nrm) {
  __shared__ float lds[kColModels * kColMS];
  const ColChunk k = col_chunk(plan, n_seg, blockIdx.x);
  const int n_models = same_a ? 1 + cnt : 2 * cnt;
  const int nmw = min(kColModels, kColThreads / k.Cf);
  const int m0 = static_cast<int>(blockIdx.y) * nmw;
  if (m0 >= n_models) return;
  const int nmod = min(nmw, n_models - m0);
  const float* gm[kColModels];
#pragma unroll
  for (int m = 0; m < kColModels; ++m) {
    // model slot s: one a shared by all pairs (slot 0 = a, 1 + p = b_p) or one per pair (2 p = a_p,
    // 2 p + 1 = b_p); the kernel argument is indexed in place (a reference to it would copy it
    // to scratch)
    const int sl = m0 + min(m, nmod - 1);
    gm[m] = same_a ? (sl == 0 ? pr.a[0] : pr.b[sl - 1]) : ((sl & 1) ? pr.b[sl >> 1] : pr.a[sl >> 1]);
  }
  ColLoads L;
  col_loads_init(L, gm, nmod, k);
  const int t = threadIdx.x, g = t / k.Cf, c = t - g * k.Cf;
  const bool live = g < nmod && c < k.C;
  const int o = c / k.B, kk = c - o * k.B;
  const float* x = lds + (live ? g * k.MS + o * k.P + kk : 0);
  const int B = k.B;
  float acc = 0.f;
  bool in_range = true;  // every element zero or in cos_rdiv's range
  col_stream(L, k.I, B, lds, [&](int, int n) {
    if (!live) return;
    if (n == kColIc) {
      float v[kColIc];
#pragma unroll
      for (int i = 0; i < kColIc; ++i) v[i] = x[i * B];
#pragma unroll
      for (int i = 0; i < kColIc; ++i) {
        acc = __fmaf_rn(v[i], v[i], acc);
        in_range = in_range && (cos_rdiv_x(v[i]) || v[i] == 0.f);
      }
    } else {
      for (int i = 0; i < n; ++i) {
        acc = __fmaf_rn(x[i * B], x[i * B], acc);
        in_range = in_range && (cos_rdiv_x(x[i * B]) || x[i * B] == 0.f);
      }
    }
  });
  // the norm, negated when the chain has an element outside cos_rdiv's range (the products then
  // check element by element); a NaN norm stays NaN either way
  const float nv = cos_clamp(cos_sqrt_rn(acc));
  if (live) nrm[static_cast<int64_t>(m0 + g) * plan[1] + k.out0 + c] = in_range ? nv : -nv;
}

// Products: one workgroup per (streamed chunk, group of pairs); thread (g, c): pair p0 + g, output
// c.  row_sum over the I products (x_a / n_a) (x_b / n_b): four interleaved streams of I / 4,
// each summed in 16-element level-0 runs from 0 (cos_run) that are pushed into the stream's
// cascade (cos_cascade: level 1 every run, level 2 every 16, level 3 every 256 - multi_row_sum's
// counts at width 2^4), the partial last run at the end, the I mod 4 remainder into stream 0,
// then the streams in order; s = 0 + that.  Divisions: cos_rdiv where both norms and the element
// are in its range (equal to the IEEE quotient there), else __fdiv_rn.
__global__ __launch_bounds__(kColThreads) void k_cos_col_prods(CosPairs pr, const int64_t* __restrict__ plan, int n_seg,
                                                              int cnt, int same_a, const float* __restrict__ nrm,
                                                              float* __restrict__ s_all) {
  __shared__ float lds[kColModels * kColMS];
  // chunks in the reverse of the norms' order: the first workgroups read what the norms kernel
  // read last, still in the 256 MiB last-level cache
  const ColChunk k = col_chunk(plan, n_seg, gridDim.x - 1 - blockIdx.x);
  const int ppw = same_a ? kColPairs : kColPairs / 2;
  const int p0 = static_cast<int>(blockIdx.y) * ppw;
  if (p0 >= cnt) return;
  const int np = min(ppw, cnt - p0);
  const int nmod = same_a ? 1 + np : 2 * np;
  const float* gm[kColModels];
#pragma unroll
  for (int m = 0; m < kColModels; ++m) {
    const int mm = min(m, nmod - 1);
    gm[m] = same_a ? (mm == 0 ? pr.a[p0] : pr.b[p0 + mm - 1]) : ((mm & 1) ? pr.b[p0 + (mm >> 1)] : pr.a[p0 + (mm >> 1)]);
  }
  ColLoads L;
  col_loads_init(L, gm, nmod, k);
  const int t = threadIdx.x, g = t / k.Cf, c = t - g * k.Cf;
  const bool live = g < np && c < k.C;
  const int o = c / k.B, kk = c - o * k.B;
  const int ma = same_a ? 0 : 2 * g, mb = same_a ? 1 + g : 2 * g + 1;
  const int64_t n_out = plan[1];
  float na = 1.f, nb = 1.f;
  if (live) {
    const int sa = same_a ? 0 : 2 * (p0 + g), sb = same_a ? 1 + p0 + g : 2 * (p0 + g) + 1;
    na = nrm[sa * n_out + k.out0 + c];
    nb = nrm[sb * n_out + k.out0 + c];
  }
  // a negative norm: its chain has an element outside cos_rdiv's range (k_cos_col_norms)
  const bool checked = __float_as_uint(na) >> 31 || __float_as_uint(nb) >> 31;
  na = fabsf(na);
  nb = fabsf(nb);
  const float ya = __fdiv_rn(1.f, na), yb = __fdiv_rn(1.f, nb);
  const bool fast = cos_rdiv_n(na) && cos_rdiv_n(nb);
  // both chains entirely in range (zeros included: a zero quotient's sign never reaches a sum,
  // whose terms are added to +0): the reciprocal division without element checks
  const bool sure = fast && !checked;
  const float* xa = lds + (live ? ma * k.MS + o * k.P + kk : 0);
  const float* xb = lds + (live ? mb * k.MS + o * k.P + kk : 0);
  const int B = k.B;
  const int e4 = 4 * (k.I / 4);  // the streams' elements; the rest is row_sum's remainder
  auto prod = [&](float u, float w) {
    const float qa = fast && cos_rdiv_x(u) ? cos_rdiv(u, na, ya) : __fdiv_rn(u, na);
    const float qb = fast && cos_rdiv_x(w) ? cos_rdiv(w, nb, yb) : __fdiv_rn(w, nb);
    return __fmul_rn(qa, qb);
  };
  float acc[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f}, a2[4] = {0.f, 0.f, 0.f, 0.f},
        a3[4] = {0.f, 0.f, 0.f, 0.f};
  int pushed = 0;  // elements per stream in completed runs
  col_stream(L, k.I, B, lds, [&](int i0, int n) {
    if (!live) return;
    float p[kColIc];
    if (sure && n == kColIc && i0 + kColIc <= e4) {
#pragma unroll
      for (int i = 0; i < kColIc; ++i) p[i] = __fmul_rn(cos_rdiv(xa[i * B], na, ya), cos_rdiv(xb[i * B], nb, yb));
#pragma unroll
      for (int i = 0; i < kColIc; ++i) acc[i & 3] = __fadd_rn(acc[i & 3], p[i]);
    } else if (n == kColIc && i0 + kColIc <= e4) {  // a whole step of stream elements (all but the last)
      // the reciprocal division for all 16, the IEEE one for the step if any element (or norm)
      // is outside its range: one branch per step
      bool ok = fast;
#pragma unroll
      for (int i = 0; i < kColIc; ++i) {
        const float u = xa[i * B], w = xb[i * B];
        ok = ok && cos_rdiv_x(u) && cos_rdiv_x(w);
        p[i] = __fmul_rn(cos_rdiv(u, na, ya), cos_rdiv(w, nb, yb));
      }
      if (!ok) {
#pragma unroll
        for (int i = 0; i < kColIc; ++i) p[i] = __fmul_rn(__fdiv_rn(xa[i * B], na), __fdiv_rn(xb[i * B], nb));
      }
#pragma unroll
      for (int i = 0; i < kColIc; ++i) acc[i & 3] = __fadd_rn(acc[i & 3], p[i]);
    } else {
      for (int i = 0; i < n && i0 + i < e4; ++i) acc[i & 3] = __fadd_rn(acc[i & 3], prod(xa[i * B], xb[i * B]));
    }
    if (((i0 + kColIc) & 63) == 0 && i0 + kColIc <= e4) {  // every stream's run of 16 complete
      pushed += 16;
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        a1[st] = __fadd_rn(a1[st], acc[st]);
        acc[st] = 0.f;
      }
      if ((pushed & (15 << 4)) == 0) {
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          a2[st] = __fadd_rn(a2[st], a1[st]);
          a1[st] = 0.f;
        }
        if ((pushed & (15 << 8)) == 0) {
#pragma unroll
          for (int st = 0; st < 4; ++st) {
            a3[st] = __fadd_rn(a3[st], a2[st]);
            a2[st] = 0.f;
          }
        }
      }
    }
  });
  if (!live) return;
  float ps[4];
#pragma unroll
  for (int st = 0; st < 4; ++st) ps[st] = __fadd_rn(__fadd_rn(__fadd_rn(acc[st], a1[st]), a2[st]), a3[st]);
  // the remainder (I mod 4 elements) lies in the last step, whose data is still in LDS
  const int last = (k.I - 1) / kColIc * kColIc;
  for (int gi = e4; gi < k.I; ++gi) ps[0] = __fadd_rn(ps[0], prod(xa[(gi - last) * B], xb[(gi - last) * B]));
  const float v = __fadd_rn(__fadd_rn(__fadd_rn(ps[0], ps[1]), ps[2]), ps[3]);
  s_all[static_cast<int64_t>(p0 + g) * n_out + k.out0 + c] = __fadd_rn(0.f, v);
}

// torch's serial full sum of s[0 .. n) (scalar_inner_sum below 8 elements, else
// vectorized_inner_sum: lane l sums elements 8 i + l by row_sum, then the scalar tail, then the
// lanes in order), without the store's 0 +; valid in thread 0, every thread of the wave calls it
__device__ __forceinline__ float cos_inner_sum(const float* s, int64_t n, int l) {
  if (n < kCosVw) return l == 0 ? cos_row_sum([&](int64_t i) { return s[i]; }, n) : 0.f;
  const int64_t nv = n / kCosVw;
  const float lane_sum = l < kCosVw ? cos_row_sum([&](int64_t i) { return s[i * kCosVw + l]; }, nv) : 0.f;
  float tail = 0.f;
  if (l == 0)
    for (int64_t k = nv * kCosVw; k < n; ++k) tail = __fadd_rn(tail, s[k]);
  return cos_group_fold(tail, lane_sum, 0);
}

// per (tensor, pair): mean = sum(s) / numel (torch sum then div_); 8 threads = the lanes.
// A sum over >= 32768 elements (at::internal::GRAIN_SIZE) in a process with T > 1 intra-op
// threads is torch's two-pass reduction (TensorIteratorReduce.cpp two_pass_reduction over
// at::parallel_for): nt = min(T, ceil(n / 32768)) chunks of ceil(n / nt) elements, chunk t's
// serial sum stored into a T-entry buffer of zeros (0 + sum), then the buffer's serial sum.
// T is the plan's thread word (tal_cosine_plan_set_threads; the caller's torch thread count).
__global__ void k_cosine_means(const int64_t* __restrict__ plan, int n_seg, const float* __restrict__ s_all,
                               float* __restrict__ means) {
  __shared__ float part[kCosMaxThreads];
  const int seg = blockIdx.x, pair = blockIdx.y;
  const int64_t n_out = plan[1];
  const int64_t T = plan[2];
  const int64_t* sg = plan + kCosHdr + kCosSegWords * static_cast<int64_t>(seg);
  const int64_t n = sg[1] * sg[3];
  const float* s = s_all + static_cast<int64_t>(pair) * n_out + sg[4];
  const int l = threadIdx.x & 63;
  float fin;
  if (n < kCosGrain || T <= 1) {
    fin = cos_inner_sum(s, n, l);
  } else {
    for (int64_t k = l; k < T; k += 64) part[k] = 0.f;
    __syncthreads();
    const int64_t nt = min(T, (n + kCosGrain - 1) / kCosGrain);
    const int64_t chunk = (n + nt - 1) / nt;
    for (int64_t t = 0; t < nt && t * chunk < n; ++t) {
      const float c = cos_inner_sum(s + t * chunk, min(chunk, n - t * chunk), l);
      if (l == 0) part[t] = __fadd_rn(0.f, c);
    }
    __syncthreads();
    fin = cos_inner_sum(part, T, l);
  }
  if (l == 0) means[static_cast<int64_t>(pair) * n_seg + seg] = __fdiv_rn(__fadd_rn(0.f, fin), static_cast<float>(n));
}

// avg_cos = 0 + mean_0, += mean_t in parameter order; / len(params)
__global__ void k_cosine_finish(int n_seg, const float* __restrict__ means, float* __restrict__ out, int pair0) {
  if (threadIdx.x != 0) return;
  const int pair = blockIdx.x;
  const float* m = means + static_cast<int64_t>(pair) * n_seg;
  float avg = __fadd_rn(0.f, m[0]);
  for (int t = 1; t < n_seg; ++t) avg = __fadd_rn(avg, m[t]);
  out[pair0 + pair] = __fdiv_rn(avg, static_cast<float>(n_seg));
}

// ------------------------------------------------------------------------------------------
// FedProx proximal term (reference tasks.py:277-286): prox = sum_t sum_p ||w_p - wt_p||_2 over
// neighbors t and parameter tensors p, and its gradient.  The parameters are segments of the
// flat fp32 pool rows.  Plan (int64): seg_chunk_ptr[n_seg+1], then per chunk {seg, begin, len}.
// ------------------------------------------------------------------------------------------
constexpr int kProxMaxNb = 64;             // neighbors per launch (more: host batches)
constexpr int64_t kProxChunk = 8192;       // elements per workgroup chunk
constexpr int kProxTile = 8;               // neighbors accumulated per pass over w

struct ProxPtrs {
  const float* wt[kProxMaxNb];
  float* gwt[kProxMaxNb];
};

__device__ __forceinline__ double block_sum_f64(double v, double* s_red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) s_red[wave] = v;
  __syncthreads();
  double tot = 0.0;
  for (int w = 0; w < kBlock / 64; ++w) tot += s_red[w];  // fixed order: deterministic
  return tot;
}

__global__ __launch_bounds__(kBlock) void k_prox_sumsq(const float* __restrict__ w, ProxPtrs pp, int k,
                                                       const int64_t* __restrict__ plan, int n_seg,
                                                       int n_chunks, double* __restrict__ partial) {
  __shared__ double s_red[kBlock / 64];
  const int c = blockIdx.x;
  const int64_t* ch = plan + (n_seg + 1) + 3 * static_cast<int64_t>(c);
  const int64_t beg = ch[1], len = ch[2];
  for (int t0 = 0; t0 < k; t0 += kProxTile) {
    const int nt = min(kProxTile, k - t0);
    float acc[kProxTile];
#pragma unroll
    for (int j = 0; j < kProxTile; ++j) acc[j] = 0.f;
    for (int64_t e = threadIdx.x; e < len; e += kBlock) {
      const float wv = w[beg + e];
#pragma unroll
      for (int j = 0; j < kProxTile; ++j) {
        if (j < nt) {
          const float d = wv - pp.wt[t0 + j][beg + e];
          acc[j] = fmaf(d, d, acc[j]);
        }
      }
    }
    for (int j = 0; j < nt; ++j) {
      const double tot = block_sum_f64(static_cast<double>(acc[j]), s_red);
      if (threadIdx.x == 0) partial[static_cast<int64_t>(t0 + j) * n_chunks + c] = tot;
    }
  }
}

__global__ void k_prox_finish(const int64_t* __restrict__ plan, int n_seg, int n_chunks, int k,
                              const double* __restrict__ partial, float* __restrict__ norms) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= static_cast<int64_t>(k) * n_seg) return;
  const int t = static_cast<int>(i / n_seg), sg = static_cast<int>(i % n_seg);
  double ss = 0.0;
  for (int64_t c = plan[sg]; c < plan[sg + 1]; ++c) ss += partial[static_cast<int64_t>(t) * n_chunks + c];
  norms[i] = static_cast<float>(sqrt(ss));
}

// g_w = s * sum_t (w - wt) / ||w - wt||,  g_wt = -s * (w - wt) / ||w - wt||  (0 where the
// norm is 0, as torch's norm backward); s = *scale (the upstream gradient, on the device).
__global__ __launch_bounds__(kBlock) void k_prox_grad(const float* __restrict__ w, ProxPtrs pp, int k,
                                                      const int64_t* __restrict__ plan, int n_seg,
                                                      const float* __restrict__ norms,
                                                      const float* __restrict__ scale,
                                                      float* __restrict__ gw, int accumulate) {
  __shared__ float s_c[kProxMaxNb];
  const int c = blockIdx.x;
  const int64_t* ch = plan + (n_seg + 1) + 3 * static_cast<int64_t>(c);
  const int64_t sg = ch[0], beg = ch[1], len = ch[2];
  if (threadIdx.x < k) {
    const float nrm = norms[static_cast<int64_t>(threadIdx.x) * n_seg + sg];
    s_c[threadIdx.x] = nrm > 0.f ? *scale / nrm : 0.f;
  }
  __syncthreads();
  for (int64_t e = threadIdx.x; e < len; e += kBlock) {
    const float wv = w[beg + e];
    float g = accumulate ? gw[beg + e] : 0.f;
    for (int t = 0; t < k; ++t) {
      const float d = (wv - pp.wt[t][beg + e]) * s_c[t];
      g += d;
      if (pp.gwt[t]) pp.gwt[t][beg + e] = -d;
    }
    gw[beg + e] = g;
  }
}

}  // namespace

// ==========================================================================================
// C-ABI
// ==========================================================================================
namespace {

// Row groups: consecutive rows and the union of their sources (ascending pool rows after
// finish_plan sorts them).
struct Groups {
  std::vector<int32_t> row_ptr{0};
  std::vector<std::vector<int32_t>> srcs;
};

int32_t check_csr(const char* fn, int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                  const double* w_host, const int32_t* out_row_host, int32_t* max_col) {
  if (rows <= 0 || !row_ptr_host || !col_host || !w_host || !out_row_host)
    return fail(TAL_ERR_INVALID, std::string(fn) + ": bad arguments");
  if (row_ptr_host[0] != 0) return fail(TAL_ERR_INVALID, std::string(fn) + ": row_ptr[0] != 0");
  for (int r = 0; r < rows; ++r)
    if (row_ptr_host[r + 1] <= row_ptr_host[r])
      return fail(TAL_ERR_INVALID, std::string(fn) + ": every row needs >= 1 operand");
  const int64_t nnz = row_ptr_host[rows];
  *max_col = 0;
  for (int64_t k = 0; k < nnz; ++k) {
    if (col_host[k] < 0) return fail(TAL_ERR_INVALID, std::string(fn) + ": negative source row");
    *max_col = std::max(*max_col, col_host[k]);
  }
  return TAL_OK;
}

// Reference operand order (decentralized_app.py:618-625): ascending distinct neighbors, then
// the row's own model, which does not occur among them.
bool reference_order(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host) {
  for (int r = 0; r < rows; ++r) {
    const int32_t k0 = row_ptr_host[r], k1 = row_ptr_host[r + 1];
    for (int32_t k = k0 + 1; k < k1 - 1; ++k)
      if (col_host[k] <= col_host[k - 1]) return false;
    for (int32_t k = k0; k < k1 - 1; ++k)
      if (col_host[k] == col_host[k1 - 1]) return false;
  }
  return true;
}

// Every row's operands carry one fp32 weight (bitwise): the narrow ROWW encoding applies.
bool rows_uniform_weights(int32_t rows, const int32_t* row_ptr_host, const double* w_host) {
  for (int r = 0; r < rows; ++r) {
    const float w0 = static_cast<float>(w_host[row_ptr_host[r]]);
    for (int32_t k = row_ptr_host[r] + 1; k < row_ptr_host[r + 1]; ++k) {
      const float wk = static_cast<float>(w_host[k]);
      if (memcmp(&wk, &w0, 4) != 0) return false;
    }
  }
  return true;
}

// Greedy grouping: a row joins the current group unless that breaks
// `fits(n_src, n_rows, n_ops, first_row)` (the candidate group is rows first_row .. +n_rows-1).
template <class Fits>
int32_t group_rows(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host, int32_t max_col,
                   Fits fits, Groups* out) {
  std::vector<int32_t> seen(static_cast<size_t>(max_col) + 1, -1);  // source -> group that has it
  Groups& G = *out;
  G.srcs.assign(1, {});
  int64_t cur_nnz = 0;
  auto fresh_of = [&](int r, int g, std::vector<int32_t>* fresh) {
    fresh->clear();
    for (int32_t k = row_ptr_host[r]; k < row_ptr_host[r + 1]; ++k) {
      const int32_t sr = col_host[k];
      if (seen[sr] != g && std::find(fresh->begin(), fresh->end(), sr) == fresh->end()) fresh->push_back(sr);
    }
  };
  std::vector<int32_t> fresh;
  for (int r = 0; r < rows; ++r) {
    int g = static_cast<int>(G.srcs.size()) - 1;
    fresh_of(r, g, &fresh);
    const int64_t row_nnz = row_ptr_host[r + 1] - row_ptr_host[r];
    const int64_t cur_rows = r - G.row_ptr.back();
    if (!fits(static_cast<int64_t>(G.srcs[g].size() + fresh.size()), cur_rows + 1, cur_nnz + row_nnz,
              static_cast<int64_t>(G.row_ptr.back()))) {
      if (cur_rows > 0) {
        G.row_ptr.push_back(r);
        G.srcs.emplace_back();
        cur_nnz = 0;
        g = static_cast<int>(G.srcs.size()) - 1;
        fresh_of(r, g, &fresh);
      }
      if (!fits(static_cast<int64_t>(fresh.size()), 1, row_nnz, static_cast<int64_t>(r)))
        return fail(TAL_ERR_CAPACITY, "tal_round_plan_build: row " + std::to_string(r) +
                                          " has more distinct sources than one LDS tile holds");
    }
    for (int32_t sr : fresh) {
      seen[sr] = g;
      G.srcs[g].push_back(sr);
    }
    cur_nnz += row_nnz;
  }
  G.row_ptr.push_back(rows);
  return TAL_OK;
}

// ROWW slots are 16-bit (slot * c4 float4 units, the zero tiles at ns and ns + 1 included).
bool roww_slots_fit(int32_t max_col, int32_t c4) {
  return (static_cast<int64_t>(max_col) + 3) * c4 <= 0xffff;
}

// Slots a group of rows r0 .. r0+nr-1 takes in the ROWW encoding: the narrow builder orders a
// group's rows by operand count (descending) and pads each pass of 64 / c4 consecutive rows to
// the batch count of its first (longest) row.
int64_t roww_padded_slots(const int32_t* row_ptr_host, int64_t r0, int64_t nr, int32_t c4,
                          std::vector<int32_t>* batches) {
  batches->resize(static_cast<size_t>(nr));
  for (int64_t i = 0; i < nr; ++i)
    (*batches)[i] = (row_ptr_host[r0 + i + 1] - row_ptr_host[r0 + i] + 3) / 4;
  std::sort(batches->begin(), batches->end(), std::greater<int32_t>());
  const int64_t rpw = 64 / c4;
  int64_t slots = 0;
  for (int64_t i = 0; i < nr; i += rpw) slots += 4LL * (*batches)[i] * std::min(rpw, nr - i);
  return slots;
}

// Broadcast form: a pass is 4 rows (16 lanes each: one float4 chunk per lane at c4 = 16, two
// at c4 = 32) and takes ceil(operands of its longest row / 16) records; passes are dealt to
// wavefronts longest first, each to the least loaded one.  False when a wavefront would hold
// more than rmax records.
bool bc_deal(const std::vector<int32_t>& pass_recs, int waves, int rmax, std::vector<std::vector<int32_t>>* per_wave) {
  std::vector<int32_t> order(pass_recs.size());
  for (size_t k = 0; k < order.size(); ++k) order[k] = static_cast<int32_t>(k);
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return pass_recs[a] > pass_recs[b]; });
  per_wave->assign(static_cast<size_t>(waves), {});
  std::vector<int32_t> load(static_cast<size_t>(waves), 0);
  for (int32_t k : order) {
    const int w = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
    if (load[w] + pass_recs[k] > rmax) return false;
    load[w] += pass_recs[k];
    (*per_wave)[w].push_back(k);
  }
  for (auto& v : *per_wave) std::sort(v.begin(), v.end());
  return true;
}

// Records of the passes of rows r0 .. r0+nr-1 once ordered by operand count (descending).
constexpr int32_t kBcRowsPerPass = 4;

std::vector<int32_t> bc_pass_records(const int32_t* row_ptr_host, int64_t r0, int64_t nr, bool sorted) {
  std::vector<int32_t> m(static_cast<size_t>(nr));
  for (int64_t i = 0; i < nr; ++i) m[i] = row_ptr_host[r0 + i + 1] - row_ptr_host[r0 + i];
  if (!sorted) std::sort(m.begin(), m.end(), std::greater<int32_t>());
  const int64_t rpw = kBcRowsPerPass;
  std::vector<int32_t> recs;
  for (int64_t i = 0; i < nr; i += rpw) recs.push_back((m[i] + 15) / 16);
  return recs;
}

constexpr int64_t bc_lds_bytes(int64_t ns, int c4) { return (ns + 1) * c4 * 16; }

// Lay the plan blob out (see tal_round_plan_info).  rb = dense row-block size (0 = sparse
// form only, -1 = dense when it saves LDS reads); stream_cs > 0 pads each block's entries
// chunk by chunk for the streamed kernel.
int32_t finish_plan(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                    const double* w_host, const int32_t* out_row_host, int32_t max_col,
                    Groups& grp, int32_t c4, int32_t dense_rb, int32_t stream_cs,
                    int32_t* plan_host, int64_t plan_capacity_words, tal_round_plan_info* info,
                    int32_t bc_waves = 0, int32_t bc_wg = 2) {
  const int64_t nnz = row_ptr_host[rows];
  const int32_t G = static_cast<int32_t>(grp.srcs.size());
  const std::vector<int32_t>& grp_row_ptr = grp.row_ptr;

  // staged sources of a group in ascending pool-row order; operand slots
  std::vector<int32_t> grp_src_ptr{0}, src_row, slot(nnz);
  std::vector<int32_t> map(static_cast<size_t>(max_col) + 1, -1);
  int32_t max_src = 0, max_rows = 0, max_nnz = 0;
  for (int g = 0; g < G; ++g) {
    std::vector<int32_t>& ss = grp.srcs[g];
    std::sort(ss.begin(), ss.end());
    for (size_t i = 0; i < ss.size(); ++i) map[ss[i]] = static_cast<int32_t>(i);
    for (int r = grp_row_ptr[g]; r < grp_row_ptr[g + 1]; ++r)
      for (int32_t k = row_ptr_host[r]; k < row_ptr_host[r + 1]; ++k) slot[k] = map[col_host[k]];
    src_row.insert(src_row.end(), ss.begin(), ss.end());
    grp_src_ptr.push_back(static_cast<int32_t>(src_row.size()));
    max_src = std::max<int32_t>(max_src, static_cast<int32_t>(ss.size()));
    max_rows = std::max<int32_t>(max_rows, grp_row_ptr[g + 1] - grp_row_ptr[g]);
    max_nnz = std::max<int32_t>(max_nnz, row_ptr_host[grp_row_ptr[g + 1]] - row_ptr_host[grp_row_ptr[g]]);
  }

  // dense row blocks need reference order; per block of kDenseRb rows, one LDS read per
  // table entry (distinct non-self source the block uses, padded) plus one per row for its
  // own model
  bool dense_ok = dense_rb != 0 && reference_order(rows, row_ptr_host, col_host);
  std::vector<std::vector<int32_t>> blk_used;  // per block: table slots (padded), ascending
  int64_t dense_reads = 0;
  if (dense_ok) {
    for (int g = 0; g < G; ++g) {
      for (int r0 = grp_row_ptr[g]; r0 < grp_row_ptr[g + 1]; r0 += kDenseRb) {
        std::vector<int32_t> used;
        const int r1 = std::min(r0 + kDenseRb, grp_row_ptr[g + 1]);
        for (int r = r0; r < r1; ++r)  // streamed tables also list each row's own model
          for (int32_t k = row_ptr_host[r]; k < row_ptr_host[r + 1] - (stream_cs > 0 ? 0 : 1); ++k)
            used.push_back(slot[k]);
        std::sort(used.begin(), used.end());
        used.erase(std::unique(used.begin(), used.end()), used.end());
        std::vector<int32_t> tab;
        if (stream_cs > 0) {  // each chunk's run starts on a multiple of 4 entries
          for (size_t i = 0; i < used.size();) {
            const int32_t chunk = used[i] / stream_cs;
            const int32_t first = used[i];
            while (i < used.size() && used[i] / stream_cs == chunk) tab.push_back(used[i++]);
            while (tab.size() % 4) tab.push_back(first);  // a repeated slot marks padding (mask 0)
          }
        } else {
          tab = used;
          while (tab.size() % 4) tab.push_back(-1);
        }
        dense_reads += stream_cs > 0 ? static_cast<int64_t>(tab.size()) : static_cast<int64_t>(used.size()) + (r1 - r0);
        blk_used.push_back(std::move(tab));
      }
    }
    // automatic choice: dense only when one LDS read serves >= 4 operands on average (cliques);
    // a dense entry costs every row of its block a masked multiply-add, so at the 0.69 reads per
    // operand of a random 8-regular graph the dense form ran 6.2 vs 2.45 ms (config 3)
    if (dense_rb == -1) dense_ok = dense_reads * 4 <= nnz;
  }
  if (stream_cs > 0 && !dense_ok)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_stream: rows must list operands in reference order");
  const int32_t rb = dense_ok ? kDenseRb : 0;
  std::vector<int32_t> grp_blk_ptr{0};
  int64_t dense_words = 0;
  if (rb) {
    for (int g = 0; g < G; ++g)
      grp_blk_ptr.push_back(grp_blk_ptr.back() + (grp_row_ptr[g + 1] - grp_row_ptr[g] + rb - 1) / rb);
    for (const auto& u : blk_used) dense_words += 8 + static_cast<int64_t>(u.size()) * (rb + 2);
  }
  const int32_t n_blocks = rb ? grp_blk_ptr.back() : 0;

  // narrow form: (slot * c4, weight) pairs, each row's operands after the first padded to whole
  // batches of 4 with (max_src * c4, 1.0f): the kernel's -0.0 tile makes them exact identities
  std::vector<int32_t> nrp, npr;
  int64_t max_np = 0;
  int64_t lds_need = 0;  // the largest group's LDS (exact, per group: what the kernels carve)
  for (int g = 0; g < G; ++g) {
    const int64_t nr = grp_row_ptr[g + 1] - grp_row_ptr[g];
    const int64_t no = row_ptr_host[grp_row_ptr[g + 1]] - row_ptr_host[grp_row_ptr[g]];
    lds_need = std::max(lds_need, group_lds_bytes(grp_src_ptr[g + 1] - grp_src_ptr[g], nr, no, scalar_c4(c4)));
  }
  const int64_t scalar_need = lds_need;
  const bool roww = bc_waves == 0 && c4 < 64 && rows_uniform_weights(rows, row_ptr_host, w_host) &&
                    roww_slots_fit(max_col, c4);
  std::vector<uint16_t> nsl;   // ROWW slots
  std::vector<int32_t> nrw;    // ROWW row weights
  std::vector<int32_t> bcp;    // broadcast form: program offsets (relative to the program region)
  std::vector<int32_t> bcw;    // broadcast form: the programs
  int64_t bc_records = 0;
  const int32_t bc_rmax = bc_waves > 0 ? kBcRecPerWg / bc_waves : 0;
  if (c4 < 64 && bc_waves > 0) {
    lds_need = 0;
    const int32_t rpw = kBcRowsPerPass;
    const float one = 1.0f;
    int32_t one_bits;
    memcpy(&one_bits, &one, 4);
    bcp.assign(static_cast<size_t>(G) * bc_waves, 0);
    for (int g = 0; g < G; ++g) {
      const int32_t ns = grp_src_ptr[g + 1] - grp_src_ptr[g];
      const int32_t r0 = grp_row_ptr[g], nr = grp_row_ptr[g + 1] - r0;
      lds_need = std::max<int64_t>(lds_need, bc_lds_bytes(ns, c4));
      const std::vector<int32_t> recs = bc_pass_records(row_ptr_host, r0, nr, true);
      std::vector<std::vector<int32_t>> per_wave;
      if (!bc_deal(recs, bc_waves, bc_rmax, &per_wave))
        return fail(TAL_ERR_CAPACITY, "tal_round_plan_build_bcast: a group's records exceed the wavefronts' registers");
      for (int w = 0; w < bc_waves; ++w) {
        if (bcw.size() % 2) bcw.push_back(0);
        const size_t start = bcw.size();
        bcp[static_cast<size_t>(g) * bc_waves + w] = static_cast<int32_t>(start);
        const std::vector<int32_t>& ps = per_wave[w];
        int32_t n_rec = 0;
        for (int32_t k : ps) n_rec += recs[k];
        bc_records += n_rec;
        const size_t np = ps.size();
        const size_t data_off = (kBcHdr + bc_rmax + 4 * np + 1) / 2 * 2;
        bcw.resize(start + data_off + 128 * static_cast<size_t>(n_rec), 0);
        int32_t* pr = bcw.data() + start;
        pr[0] = n_rec;
        pr[1] = static_cast<int32_t>(np);
        pr[2] = static_cast<int32_t>(data_off);
        int32_t ri = 0;
        for (size_t i = 0; i < np; ++i) {
          const int32_t k = ps[i];
          const int32_t pr0 = r0 + k * rpw, prows = std::min(rpw, r0 + nr - pr0);
          const int32_t m_lead = row_ptr_host[pr0 + 1] - row_ptr_host[pr0];
          for (int sb = 0; sb < 4; ++sb) pr[kBcHdr + bc_rmax + 4 * i + sb] = sb < prows ? out_row_host[pr0 + sb] : -1;
          for (int32_t c = 0; c < recs[k]; ++c, ++ri) {
            const int32_t cnt = std::min(16, m_lead - 16 * c);
            pr[kBcHdr + ri] = cnt | ((c == recs[k] - 1) ? 0x100 : 0) | static_cast<int32_t>(i << 16);
            int32_t* rec = pr + data_off + 128 * static_cast<size_t>(ri);
            for (int L = 0; L < 64; ++L) {
              const int32_t sb = L / 16, j = 16 * c + L % 16;
              int32_t off = ns * c4 * 16, wb = one_bits;  // identity pad: the -0.0 tile, weight 1.0
              if (sb < prows) {
                const int32_t row = pr0 + sb, k0 = row_ptr_host[row];
                if (j < row_ptr_host[row + 1] - k0) {
                  off = slot[k0 + j] * c4 * 16;
                  const float wf = static_cast<float>(w_host[k0 + j]);
                  memcpy(&wb, &wf, 4);
                }
              }
              rec[2 * L] = off;
              rec[2 * L + 1] = wb;
            }
          }
        }
      }
    }
  } else if (c4 < 64) {
    lds_need = 0;  // the narrow kernel's carve replaces the staged one
    nrp.assign(static_cast<size_t>(rows) + 1, 0);
    const float one = 1.0f;
    int32_t one_bits;
    memcpy(&one_bits, &one, 4);
    for (int g = 0; g < G; ++g) {
      const int32_t ns = grp_src_ptr[g + 1] - grp_src_ptr[g];
      const int64_t g0 = roww ? static_cast<int64_t>(nsl.size()) : static_cast<int64_t>(npr.size()) / 2;
      for (int r = grp_row_ptr[g]; r < grp_row_ptr[g + 1]; ++r) {
        const int32_t k0 = row_ptr_host[r], k1 = row_ptr_host[r + 1];
        if (roww) {  // slots only, in batches of 4, every row of a pass padded to the batch count
          // of the pass's first (longest: rows are ordered by count) row; the pad reads the zero
          // tile that keeps -0: fl(w * z) is -0.0 for z = -0.0 (w >= 0) or +0.0 (w < 0)
          const float wf = static_cast<float>(w_host[k0]);
          int32_t wb;
          memcpy(&wb, &wf, 4);
          nrw.push_back(wb);
          const int32_t lead = grp_row_ptr[g] + (r - grp_row_ptr[g]) / (64 / c4) * (64 / c4);
          const int64_t nb = (row_ptr_host[lead + 1] - row_ptr_host[lead] + 3) / 4;
          const size_t start = nsl.size();
          for (int32_t k = k0; k < k1; ++k) nsl.push_back(static_cast<uint16_t>(slot[k] * c4));
          const uint16_t zero = static_cast<uint16_t>((std::signbit(wf) ? ns + 1 : ns) * c4);
          while (nsl.size() < start + 4 * static_cast<size_t>(nb)) nsl.push_back(zero);
          nrp[r + 1] = static_cast<int32_t>(nsl.size());
          continue;
        }
        for (int32_t k = k0; k < k1; ++k) {
          const float wf = static_cast<float>(w_host[k]);
          int32_t wb;
          memcpy(&wb, &wf, 4);
          npr.push_back(slot[k] * c4);
          npr.push_back(wb);
        }
        for (int32_t pad = (4 - (k1 - k0 - 1) % 4) % 4; pad > 0; --pad) {
          npr.push_back(ns * c4);  // the group's -0.0 tile
          npr.push_back(one_bits);
        }
        nrp[r + 1] = static_cast<int32_t>(npr.size() / 2);
      }
      const int64_t gp = (roww ? static_cast<int64_t>(nsl.size()) : static_cast<int64_t>(npr.size()) / 2) - g0;
      max_np = std::max<int64_t>(max_np, gp);
      const int64_t nr = grp_row_ptr[g + 1] - grp_row_ptr[g];
      lds_need = std::max<int64_t>(lds_need, static_cast<int64_t>(
          roww ? narrow_roww_lds_bytes(ns, nr, gp, c4) : narrow_lds_bytes(ns, nr, gp, c4)));
    }
    if (roww) {  // two slots per int32 word
      npr.assign((nsl.size() + 1) / 2, 0);
      memcpy(npr.data(), nsl.data(), 2 * nsl.size());
    }
  }

  tal_round_plan_info in;
  memset(&in, 0, sizeof(in));
  in.rows = rows;
  in.nnz = static_cast<int32_t>(nnz);
  in.n_groups = G;
  in.total_src = static_cast<int32_t>(src_row.size());
  in.max_src = max_src;
  in.max_rows = max_rows;
  in.max_nnz = max_nnz;
  in.c4 = c4;
  in.dense_rb = rb;
  in.n_blocks = n_blocks;
  in.dense_reads = static_cast<int32_t>(rb ? dense_reads : nnz);
  in.stream_cs = stream_cs;
  int64_t off = 0;
  in.off_grp_row_ptr = static_cast<int32_t>(off); off += G + 1;
  in.off_grp_src_ptr = static_cast<int32_t>(off); off += G + 1;
  in.off_src_row = static_cast<int32_t>(off); off += in.total_src;
  in.off_row_ptr = static_cast<int32_t>(off); off += rows + 1;
  in.off_op_slot = static_cast<int32_t>(off); off += nnz;
  in.off_op_w = static_cast<int32_t>(off); off += nnz;
  in.off_out_row = static_cast<int32_t>(off); off += rows;
  in.off_grp_blk_ptr = static_cast<int32_t>(off); off += rb ? G + 1 : 0;
  in.off_blk_tab = static_cast<int32_t>(off); off += n_blocks;
  off = (off + 7) / 8 * 8;  // dense tables 32-B aligned (vector scalar loads)
  in.off_dense = static_cast<int32_t>(off); off += dense_words;
  in.off_nrow_ptr = static_cast<int32_t>(off); off += static_cast<int64_t>(nrp.size());
  in.off_npairs = static_cast<int32_t>(off); off += static_cast<int64_t>(npr.size());
  in.npairs = static_cast<int32_t>(roww ? nsl.size() : npr.size() / 2);
  in.max_npairs = static_cast<int32_t>(max_np);
  in.narrow_roww = roww ? 1 : 0;
  in.off_nrow_w = static_cast<int32_t>(off); off += static_cast<int64_t>(nrw.size());
  in.scalar_lds_bytes = static_cast<int32_t>(scalar_need);
  in.narrow_bcast = bc_waves > 0 && c4 < 64 ? bc_waves : 0;
  in.bc_rec_max = in.narrow_bcast ? bc_rmax : 0;
  in.bc_wg_per_cu = in.narrow_bcast ? bc_wg : 0;
  in.bc_records = static_cast<int32_t>(bc_records);
  in.off_bc_prog = static_cast<int32_t>(off); off += static_cast<int64_t>(bcp.size());
  off = (off + 1) / 2 * 2;  // programs start on an even word (8-B records)
  const int64_t bc_region = off;
  off += static_cast<int64_t>(bcw.size());
  if (off > 0x7fffffff) return fail(TAL_ERR_INVALID, "tal_round_plan_build: plan larger than 2^31 words");
  in.words = static_cast<int32_t>(off);
  in.lds_bytes = static_cast<int32_t>(stream_cs > 0 ? stream_lds_bytes(stream_cs) : lds_need);
  if (!plan_host || off > plan_capacity_words) {
    *info = in;
    return fail(TAL_ERR_CAPACITY, "tal_round_plan_build: plan buffer too small: need " +
                                      std::to_string(off) + " words");
  }

  memcpy(plan_host + in.off_grp_row_ptr, grp_row_ptr.data(), 4 * (G + 1));
  memcpy(plan_host + in.off_grp_src_ptr, grp_src_ptr.data(), 4 * (G + 1));
  memcpy(plan_host + in.off_src_row, src_row.data(), 4 * src_row.size());
  memcpy(plan_host + in.off_row_ptr, row_ptr_host, 4 * (static_cast<size_t>(rows) + 1));
  memcpy(plan_host + in.off_op_slot, slot.data(), 4 * nnz);
  for (int64_t k = 0; k < nnz; ++k) {
    const float wf = static_cast<float>(w_host[k]);
    memcpy(plan_host + in.off_op_w + k, &wf, 4);
  }
  memcpy(plan_host + in.off_out_row, out_row_host, 4 * static_cast<size_t>(rows));
  if (!nrp.empty()) {
    memcpy(plan_host + in.off_nrow_ptr, nrp.data(), 4 * nrp.size());
    memcpy(plan_host + in.off_npairs, npr.data(), 4 * npr.size());
  }
  if (!nrw.empty()) memcpy(plan_host + in.off_nrow_w, nrw.data(), 4 * nrw.size());
  for (size_t k = 0; k < bcp.size(); ++k) plan_host[in.off_bc_prog + k] = static_cast<int32_t>(bc_region + bcp[k]);
  if (!bcw.empty()) memcpy(plan_host + bc_region, bcw.data(), 4 * bcw.size());
  if (rb) {
    memcpy(plan_host + in.off_grp_blk_ptr, grp_blk_ptr.data(), 4 * (G + 1));
    int64_t pos = in.off_dense;
    int b = 0;
    for (int g = 0; g < G; ++g) {
      for (int r0 = grp_row_ptr[g]; r0 < grp_row_ptr[g + 1]; r0 += rb, ++b) {
        const std::vector<int32_t>& tabs = blk_used[b];
        const int64_t nu = static_cast<int64_t>(tabs.size());  // multiple of 4
        plan_host[in.off_blk_tab + b] = static_cast<int32_t>(pos);
        int32_t* tab = plan_host + pos;
        const int64_t words = 8 + nu * (rb + 2);  // multiple of 8: the next table stays aligned
        memset(tab, 0, 4 * static_cast<size_t>(words));
        tab[0] = static_cast<int32_t>(nu);
        int32_t* t_slot = tab + 8;
        int32_t* t_mask = t_slot + nu;
        int32_t* t_w = t_mask + nu;
        // real entries ascend strictly; padding repeats an earlier slot (or is -1: repeat the last)
        std::vector<int64_t> entry_of;  // parallel to the sorted distinct slots
        std::vector<int32_t> distinct;
        for (int64_t e = 0; e < nu; ++e) {
          const int32_t sl = tabs[e];
          const bool pad = sl < 0 || (!distinct.empty() && sl <= distinct.back());  // real slots ascend
          t_slot[e] = sl < 0 ? (e > 0 ? t_slot[e - 1] : 0) : sl;
          if (!pad) {
            distinct.push_back(sl);
            entry_of.push_back(e);
          }
        }
        std::vector<uint32_t> wbits(static_cast<size_t>(nu), 0);
        std::vector<uint8_t> uniform(static_cast<size_t>(nu), 1);
        for (int r = r0; r < std::min(r0 + rb, grp_row_ptr[g + 1]); ++r) {
          for (int32_t k = row_ptr_host[r]; k < row_ptr_host[r + 1] - 1; ++k) {  // self excluded
            const int64_t d = std::lower_bound(distinct.begin(), distinct.end(), slot[k]) - distinct.begin();
            const int64_t e = entry_of[d];
            const float wf = static_cast<float>(w_host[k]);
            uint32_t wb;
            memcpy(&wb, &wf, 4);
            if (t_mask[e] != 0 && wb != wbits[e]) uniform[e] = 0;
            wbits[e] = wb;
            t_mask[e] |= static_cast<int32_t>(1u << (r - r0));
            memcpy(t_w + e * rb + (r - r0), &wf, 4);
          }
        }
        // every row using the entry has the same fp32 weight: one product w*x serves them all
        // (identical operands round identically); the weight then fills all rb slots
        for (int64_t e = 0; e < nu; ++e) {
          if (t_mask[e] == 0 || !uniform[e] || __builtin_popcount(static_cast<uint32_t>(t_mask[e])) < 2) continue;
          t_mask[e] = static_cast<int32_t>(static_cast<uint32_t>(t_mask[e]) | kMaskUniform);
          for (int r = 0; r < rb; ++r) memcpy(t_w + e * rb + r, &wbits[e], 4);
        }
        if (stream_cs > 0) {  // bit 8+r: the entry is row r's own model (captured, added last)
          for (int r = r0; r < std::min(r0 + rb, grp_row_ptr[g + 1]); ++r) {
            const int32_t ks = row_ptr_host[r + 1] - 1;
            const int64_t d = std::lower_bound(distinct.begin(), distinct.end(), slot[ks]) - distinct.begin();
            t_mask[entry_of[d]] = static_cast<int32_t>(static_cast<uint32_t>(t_mask[entry_of[d]]) |
                                                       (kMaskSelf0 << (r - r0)));
          }
        }
        pos += words;
      }
    }
  }
  *info = in;
  g_err.clear();
  return TAL_OK;
}

}  // namespace

extern "C" {

const char* tal_last_error(void) { return g_err.c_str(); }

int32_t tal_abi_version(void) { return kAbiVersion; }

int32_t tal_agg_f32(const float* const* x_host, const double* w_host, int32_t m, float* out,
                    int64_t n, int32_t mode, void* stream) {
  if (m <= 0) return fail(TAL_ERR_INVALID, "tal_agg_f32: m must be >= 1");
  if (n < 0) return fail(TAL_ERR_INVALID, "tal_agg_f32: n < 0");
  if (!x_host || !w_host || (n > 0 && !out)) return fail(TAL_ERR_INVALID, "tal_agg_f32: null pointer");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  bool vec = aligned16(out);
  for (int i = 0; i < m; ++i) {
    if (!x_host[i]) return fail(TAL_ERR_INVALID, "tal_agg_f32: null operand pointer");
    vec = vec && aligned16(x_host[i]);
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool exact = mode == TAL_MODE_EXACT;
  // Operands beyond kMaxOps are folded in by further passes that continue the same ordered
  // chain from `out` (stored exactly in fp32, so the result is unchanged).  A later pass must
  // not read an operand that aliases `out` after out was overwritten (the reference's own
  // model is the last operand, decentralized_app.py:625): then the chain runs through an fp32
  // scratch instead and `out` is written by the last pass only.
  for (int i = kMaxOps; i < m; ++i)
    if (x_host[i] == out)
      return exact ? agg_chain<float, true>(x_host, w_host, m, out, n, s, "tal_agg_f32")
                   : agg_chain<float, false>(x_host, w_host, m, out, n, s, "tal_agg_f32");
  for (int base = 0; base < m; base += kMaxOps) {
    OpTableF32 t;
    const int cnt = std::min(kMaxOps, m - base);
    for (int i = 0; i < cnt; ++i) {
      t.x[i] = x_host[base + i];
      t.w[i] = static_cast<float>(w_host[base + i]);
    }
    for (int i = cnt; i < kMaxOps; ++i) { t.x[i] = nullptr; t.w[i] = 0.f; }
    if (exact) launch_pass<true>(t, cnt, base > 0, vec, out, n, s);
    else launch_pass<false>(t, cnt, base > 0, vec, out, n, s);
  }
  return check_launch("tal_agg_f32");
}

int32_t tal_agg_i64(const int64_t* const* x_host, const double* w_host, int32_t m, int64_t* out,
                    int64_t n, void* stream) {
  if (m <= 0) return fail(TAL_ERR_INVALID, "tal_agg_i64: m must be >= 1");
  if (n < 0) return fail(TAL_ERR_INVALID, "tal_agg_i64: n < 0");
  if (!x_host || !w_host || (n > 0 && !out)) return fail(TAL_ERR_INVALID, "tal_agg_i64: null pointer");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  if (m > kMaxOps) {  // the chain in passes through an fp32 scratch (k_agg_chain)
    for (int i = 0; i < m; ++i)
      if (!x_host[i]) return fail(TAL_ERR_INVALID, "tal_agg_i64: null operand pointer");
    return agg_chain<int64_t, true>(x_host, w_host, m, out, n, static_cast<hipStream_t>(stream), "tal_agg_i64");
  }
  OpTableI64 t;
  for (int i = 0; i < m; ++i) {
    if (!x_host[i]) return fail(TAL_ERR_INVALID, "tal_agg_i64: null operand pointer");
    t.x[i] = x_host[i];
    t.w[i] = static_cast<float>(w_host[i]);
  }
  for (int i = m; i < kMaxOps; ++i) { t.x[i] = nullptr; t.w[i] = 0.f; }
  k_agg_i64<<<grid_for(n), kBlock, 0, static_cast<hipStream_t>(stream)>>>(t, m, out, n);
  return check_launch("tal_agg_i64");
}

int32_t tal_agg_model_f32(const float* const* x_host, const int64_t* const* xi_host, const double* w_host,
                          int32_t m, float* out, int64_t n, int64_t* out_i, int64_t n_i, int32_t mode,
                          void* stream) {
  if (m <= 0) return fail(TAL_ERR_INVALID, "tal_agg_model_f32: m must be >= 1");
  if (n < 0 || n_i < 0) return fail(TAL_ERR_INVALID, "tal_agg_model_f32: n < 0");
  if (!x_host || !w_host || (n > 0 && !out) || (n_i > 0 && (!xi_host || !out_i)))
    return fail(TAL_ERR_INVALID, "tal_agg_model_f32: null pointer");
  bool fused = m <= kModelOps && n_i <= kModelI64Max && aligned16(out) && n > 0;
  for (int i = 0; i < m; ++i) {
    if ((n > 0 && !x_host[i]) || (n_i > 0 && !xi_host[i]))
      return fail(TAL_ERR_INVALID, "tal_agg_model_f32: null operand pointer");
    fused = fused && aligned16(x_host[i]);
  }
  if (!fused) {  // the segment-by-segment path (same arithmetic)
    int32_t rc = n > 0 ? tal_agg_f32(x_host, w_host, m, out, n, mode, stream) : TAL_OK;
    if (rc == TAL_OK && n_i > 0) rc = tal_agg_i64(xi_host, w_host, m, out_i, n_i, stream);
    return rc;
  }
  OpTableModel t;
  for (int i = 0; i < kModelOps; ++i) {
    t.x[i] = i < m ? x_host[i] : nullptr;
    t.xi[i] = i < m && n_i > 0 ? xi_host[i] : nullptr;
    t.w[i] = i < m ? static_cast<float>(w_host[i]) : 0.f;
  }
  const int64_t n4 = n / 4;
  // one thread per float4 chunk; the last block also takes the scalar work (an extra block
  // when the chunks fill the last one exactly)
  const int64_t nb = (n4 + kBlock - 1) / kBlock + (n4 % kBlock == 0 ? 1 : 0);
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 g(static_cast<unsigned>(nb)), b(kBlock);
  const bool exact = mode == TAL_MODE_EXACT;
#define TAL_MODEL_CASE(MM)                                                                   \
  case MM:                                                                                   \
    if (exact) k_agg_model<MM, true><<<g, b, 0, s>>>(t, m, out, n, out_i, n_i);              \
    else k_agg_model<MM, false><<<g, b, 0, s>>>(t, m, out, n, out_i, n_i);                   \
    break;
  switch (m) {
    TAL_MODEL_CASE(1) TAL_MODEL_CASE(2) TAL_MODEL_CASE(3) TAL_MODEL_CASE(4) TAL_MODEL_CASE(5)
    TAL_MODEL_CASE(6) TAL_MODEL_CASE(7) TAL_MODEL_CASE(8) TAL_MODEL_CASE(9) TAL_MODEL_CASE(10)
    TAL_MODEL_CASE(11) TAL_MODEL_CASE(12) TAL_MODEL_CASE(13) TAL_MODEL_CASE(14) TAL_MODEL_CASE(15)
    TAL_MODEL_CASE(16) TAL_MODEL_CASE(17)
    default:
      if (exact) k_agg_model<0, true><<<g, b, 0, s>>>(t, m, out, n, out_i, n_i);
      else k_agg_model<0, false><<<g, b, 0, s>>>(t, m, out, n, out_i, n_i);
  }
#undef TAL_MODEL_CASE
  return check_launch("tal_agg_model_f32");
}

int64_t tal_round_plan_words(int32_t rows, int64_t nnz) {
  if (rows < 0 || nnz < 0) return -1;
  // grp_row_ptr + grp_src_ptr (<= rows+1 each) + src_row (<= nnz) + row_ptr + slot + w + out_row
  // + the narrow form's row pointers and padded pairs
  return 2 * (static_cast<int64_t>(rows) + 1) + nnz + (rows + 1) + 2 * nnz + rows + 16 +
         (rows + 1) + 2 * (nnz + 3LL * rows) + rows;
}


}  // extern "C"

namespace {

int32_t round_plan_build(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                         const double* w_host, const int32_t* out_row_host, int32_t c4,
                         int32_t lds_bytes, int32_t dense_rb, int32_t* plan_host,
                         int64_t plan_capacity_words, tal_round_plan_info* info, int32_t bc_waves,
                         int32_t bc_wg) {
  if (!info) return fail(TAL_ERR_INVALID, "tal_round_plan_build: bad arguments");
  int32_t max_col = 0;
  int32_t rc = check_csr("tal_round_plan_build", rows, row_ptr_host, col_host, w_host, out_row_host, &max_col);
  if (rc) return rc;
  if (c4 != 16 && c4 != 32 && c4 != 64 && c4 != 128)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build: c4 must be 16, 32, 64 or 128");
  if (c4 < 64) dense_rb = 0;  // narrow tiles: sparse form (a wavefront covers 64 / c4 rows)
  if (dense_rb != 0 && dense_rb != kDenseRb && dense_rb != -1)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build: dense_rb must be 0, 8 or -1");
  // group consecutive rows while the union of their sources fits the LDS budget (both round
  // kernels stage 16*c4 bytes per source; the scalar one also the plan slice)
  const bool roww = c4 < 64 && rows_uniform_weights(rows, row_ptr_host, w_host) && roww_slots_fit(max_col, c4);
  std::vector<int32_t> batches;
  auto fits = [&](int64_t ns, int64_t nr, int64_t no, int64_t r0) {
    const int64_t sliced = group_lds_bytes(ns, nr, no, scalar_c4(c4));  // c4 >= 64: the round kernel's own
    if (c4 >= 64) return sliced <= lds_bytes;
    // narrow kernel: its own carve (exact ROWW padding; pairs: <= 3 per row) and read-ahead
    // within the budget; the staged scalar tail kernel within the hardware's 160 KiB
    if (bc_waves > 0) {
      std::vector<std::vector<int32_t>> per_wave;
      // staging: what the form's launch takes (bc_max_loads)
      return bc_lds_bytes(ns, c4) <= lds_bytes && ns * c4 <= bc_max_loads(c4, bc_waves, bc_wg) && sliced <= 160 * 1024 &&
             bc_deal(bc_pass_records(row_ptr_host, r0, nr, false), bc_waves, kBcRecPerWg / bc_waves, &per_wave);
    }
    const int64_t narrow = static_cast<int64_t>(
        roww ? narrow_roww_lds_bytes(ns, nr, roww_padded_slots(row_ptr_host, r0, nr, c4, &batches), c4)
             : narrow_lds_bytes(ns, nr, no + 3 * nr, c4));
    return narrow <= lds_bytes && sliced <= 160 * 1024;
  };
  Groups grp;
  rc = group_rows(rows, row_ptr_host, col_host, max_col, fits, &grp);
  if (rc) return rc;
  if (c4 >= 64)
    return finish_plan(rows, row_ptr_host, col_host, w_host, out_row_host, max_col, grp, c4, dense_rb, 0,
                       plan_host, plan_capacity_words, info);
  // Narrow tiles: a wavefront pass computes 64 / c4 consecutive plan rows in lock step, so the
  // rows of each group are ordered by operand count (descending, stable): rows of a pass then
  // have similar counts and few lanes idle.  Rows are independent and each names its output
  // row, so the order is free.
  std::vector<int32_t> perm(rows);
  for (int g = 0; g + 1 < static_cast<int>(grp.row_ptr.size()); ++g) {
    const int r0 = grp.row_ptr[g], r1 = grp.row_ptr[g + 1];
    for (int r = r0; r < r1; ++r) perm[r] = r;
    std::stable_sort(perm.begin() + r0, perm.begin() + r1, [&](int32_t a, int32_t b) {
      return row_ptr_host[a + 1] - row_ptr_host[a] > row_ptr_host[b + 1] - row_ptr_host[b];
    });
  }
  const int64_t nnz = row_ptr_host[rows];
  std::vector<int32_t> rp(static_cast<size_t>(rows) + 1, 0), cl(nnz), orow(rows);
  std::vector<double> wv(nnz);
  for (int r = 0; r < rows; ++r) {
    const int32_t src = perm[r], k0 = row_ptr_host[src], k1 = row_ptr_host[src + 1];
    rp[r + 1] = rp[r] + (k1 - k0);
    std::copy(col_host + k0, col_host + k1, cl.begin() + rp[r]);
    std::copy(w_host + k0, w_host + k1, wv.begin() + rp[r]);
    orow[r] = out_row_host[src];
  }
  return finish_plan(rows, rp.data(), cl.data(), wv.data(), orow.data(), max_col, grp, c4, 0, 0,
                     plan_host, plan_capacity_words, info, bc_waves, bc_wg);
}

}  // namespace

extern "C" {

int32_t tal_round_plan_build(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                             const double* w_host, const int32_t* out_row_host, int32_t c4,
                             int32_t lds_bytes, int32_t dense_rb, int32_t* plan_host,
                             int64_t plan_capacity_words, tal_round_plan_info* info) {
  return round_plan_build(rows, row_ptr_host, col_host, w_host, out_row_host, c4, lds_bytes, dense_rb,
                          plan_host, plan_capacity_words, info, 0, 2);
}

int64_t tal_round_bcast_max_loads(int32_t c4, int32_t waves, int32_t wg_per_cu) {
  if ((c4 != 16 && c4 != 32) || (waves != 8 && waves != 12 && waves != 16) || (wg_per_cu != 1 && wg_per_cu != 2))
    return -1;
  return bc_max_loads(c4, waves, wg_per_cu);
}

int32_t tal_round_plan_build_bcast(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                                   const double* w_host, const int32_t* out_row_host, int32_t c4,
                                   int32_t lds_bytes, int32_t waves, int32_t wg_per_cu, int32_t* plan_host,
                                   int64_t plan_capacity_words, tal_round_plan_info* info) {
  if (c4 != 16 && c4 != 32)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_bcast: c4 must be 16 or 32");
  if (waves != 8 && waves != 12 && waves != 16)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_bcast: waves must be 8, 12 or 16");
  if (wg_per_cu != 1 && wg_per_cu != 2)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_bcast: wg_per_cu must be 1 or 2");
  if (wg_per_cu == 2 && lds_bytes > 80 * 1024) lds_bytes = 80 * 1024;  // two groups' tiles per CU
  return round_plan_build(rows, row_ptr_host, col_host, w_host, out_row_host, c4, lds_bytes, 0, plan_host,
                          plan_capacity_words, info, waves, wg_per_cu);
}

int32_t tal_round_plan_build_stream(int32_t rows, const int32_t* row_ptr_host,
                                    const int32_t* col_host, const double* w_host,
                                    const int32_t* out_row_host, int32_t max_group_rows,
                                    int32_t max_group_src, int32_t* plan_host,
                                    int64_t plan_capacity_words, tal_round_plan_info* info) {
  if (!info) return fail(TAL_ERR_INVALID, "tal_round_plan_build_stream: bad arguments");
  int32_t max_col = 0;
  int32_t rc = check_csr("tal_round_plan_build_stream", rows, row_ptr_host, col_host, w_host, out_row_host,
                         &max_col);
  if (rc) return rc;
  if (max_group_rows < 1 || max_group_rows > kStreamMaxRows || max_group_src < 0)
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_stream: max_group_rows must be 1.." +
                                     std::to_string(kStreamMaxRows) + ", max_group_src >= 0");
  if (!reference_order(rows, row_ptr_host, col_host))
    return fail(TAL_ERR_INVALID, "tal_round_plan_build_stream: rows must list operands in reference order");
  auto fits = [&](int64_t ns, int64_t nr, int64_t, int64_t) {
    return nr <= max_group_rows && (max_group_src == 0 || ns <= max_group_src || nr == 1);
  };
  Groups grp;
  rc = group_rows(rows, row_ptr_host, col_host, max_col, fits, &grp);
  if (rc) return rc;
  int32_t max_rows = 0;
  for (size_t g = 0; g + 1 < grp.row_ptr.size(); ++g) max_rows = std::max(max_rows, grp.row_ptr[g + 1] - grp.row_ptr[g]);
  const int32_t cs = (max_rows <= 8 * 8 ? 8 : 16) * kStreamPerWave;  // one row block per wavefront
  return finish_plan(rows, row_ptr_host, col_host, w_host, out_row_host, max_col, grp, 64, kDenseRb, cs,
                     plan_host, plan_capacity_words, info);
}

int32_t tal_agg_round_f32(const float* pool_in, int64_t ld_in, float* pool_out, int64_t ld_out,
                          int64_t n, const int32_t* plan_dev, const tal_round_plan_info* info,
                          int32_t mode, void* stream) {
  int32_t rc = validate_info(info);
  if (rc) return rc;
  if (!pool_in || !pool_out || !plan_dev) return fail(TAL_ERR_INVALID, "tal_agg_round_f32: null pointer");
  if (n < 0 || ld_in < n || ld_out < n) return fail(TAL_ERR_INVALID, "tal_agg_round_f32: bad n / ld");
  if (pool_in == pool_out && info->n_groups > 1)
    return fail(TAL_ERR_INVALID,
                "tal_agg_round_f32: in-place round needs a single-group plan (snapshot semantics)");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const PlanView v = make_view(plan_dev, *info);
  const bool exact = mode == TAL_MODE_EXACT;
  const bool vec = aligned16(pool_in) && aligned16(pool_out) && ld_in % 4 == 0 && ld_out % 4 == 0;
  int64_t e_vec = 0;
  if (vec) {
    const int64_t n4 = n / 4;
    e_vec = n4 * 4;
    if (n4 > 0 && info->stream_cs > 0) {
      rc = launch_round_stream(pool_in, ld_in, pool_out, ld_out, n4, v, *info, exact, s);
      if (rc) return rc;
    } else if (n4 > 0 && info->c4 < 64) {
      if (info->c4 == 16)
        rc = exact ? launch_round_narrow<16, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s)
                   : launch_round_narrow<16, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s);
      else
        rc = exact ? launch_round_narrow<32, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s)
                   : launch_round_narrow<32, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s);
      if (rc) return rc;
    } else if (n4 > 0) {
      const bool dense = info->dense_rb > 0;
      switch (info->c4 * 4 + (exact ? 2 : 0) + (dense ? 1 : 0)) {
        case 515: rc = launch_round_vec<128, true, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 514: rc = launch_round_vec<128, true, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 513: rc = launch_round_vec<128, false, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 512: rc = launch_round_vec<128, false, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 259: rc = launch_round_vec<64, true, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 258: rc = launch_round_vec<64, true, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 257: rc = launch_round_vec<64, false, true>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        default: rc = launch_round_vec<64, false, false>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
      }
      if (rc) return rc;
    }
  }
  if (n <= e_vec) return TAL_OK;
  if (use_direct(pool_in, pool_out, e_vec, n))
    return launch_round_direct<float>(pool_in, ld_in, pool_out, ld_out, e_vec, n, v, *info, exact, s);
  if (info->stream_cs > 0)
    return launch_round_stream_scalar<false>(pool_in, ld_in, pool_out, ld_out, e_vec, n, v, *info, exact, s);
  return launch_round_scalar<float>(pool_in, ld_in, pool_out, ld_out, e_vec, n, v, *info, exact, s);
}

int32_t tal_agg_round_i64(const int64_t* pool_in, int64_t ld_in, int64_t* pool_out, int64_t ld_out,
                          int64_t n, const int32_t* plan_dev, const tal_round_plan_info* info,
                          void* stream) {
  int32_t rc = validate_info(info);
  if (rc) return rc;
  if (!pool_in || !pool_out || !plan_dev) return fail(TAL_ERR_INVALID, "tal_agg_round_i64: null pointer");
  if (n < 0 || ld_in < n || ld_out < n) return fail(TAL_ERR_INVALID, "tal_agg_round_i64: bad n / ld");
  if (pool_in == pool_out && info->n_groups > 1)
    return fail(TAL_ERR_INVALID,
                "tal_agg_round_i64: in-place round needs a single-group plan (snapshot semantics)");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  const PlanView v = make_view(plan_dev, *info);
  if (use_direct(pool_in, pool_out, 0, n))
    return launch_round_direct<int64_t>(pool_in, ld_in, pool_out, ld_out, 0, n, v, *info, true,
                                     static_cast<hipStream_t>(stream));
  if (info->stream_cs > 0)
    return launch_round_stream_scalar<true>(pool_in, ld_in, pool_out, ld_out, 0, n, v, *info, true,
                                            static_cast<hipStream_t>(stream));
  return launch_round_scalar<int64_t>(pool_in, ld_in, pool_out, ld_out, 0, n, v, *info, true,
                                   static_cast<hipStream_t>(stream));
}

int32_t tal_agg_round_clique_f32(const float* pool_in, int64_t ld_in, float* pool_out, int64_t ld_out,
                                 int64_t n, const int32_t* table_dev, int32_t n_cliques, int32_t mmax,
                                 int32_t mode, void* stream) {
  if (!pool_in || !pool_out || !table_dev)
    return fail(TAL_ERR_INVALID, "tal_agg_round_clique_f32: null pointer");
  if (pool_in == pool_out)
    return fail(TAL_ERR_INVALID, "tal_agg_round_clique_f32: the clique round runs out of place");
  if (n < 0 || ld_in < n || ld_out < n) return fail(TAL_ERR_INVALID, "tal_agg_round_clique_f32: bad n / ld");
  if (n_cliques < 0 || mmax < 1 || mmax > kCliqueMax)
    return fail(TAL_ERR_INVALID, "tal_agg_round_clique_f32: n_cliques >= 0, 1 <= mmax <= 64");
  if (!aligned8(pool_in) || !aligned8(pool_out) || ld_in % 2 || ld_out % 2)
    return fail(TAL_ERR_INVALID, "tal_agg_round_clique_f32: pools must be 8-B aligned with even ld");
  if (n == 0 || n_cliques == 0) { g_err.clear(); return TAL_OK; }
  hipStream_t s = static_cast<hipStream_t>(stream);
  return mode == TAL_MODE_EXACT
             ? launch_round_clique<true>(pool_in, ld_in, pool_out, ld_out, n, table_dev, n_cliques, mmax, s)
             : launch_round_clique<false>(pool_in, ld_in, pool_out, ld_out, n, table_dev, n_cliques, mmax, s);
}

int32_t tal_agg_round_reg(const void* pool_in, int64_t ld_in, void* pool_out, int64_t ld_out, int64_t n,
                          int32_t bf16, const int32_t* table_dev, const int64_t* src_off_dev, int32_t n_groups,
                          int32_t off_src, int32_t off_pairs, int32_t off_rec, int32_t max_src, int32_t mode,
                          void* stream) {
  if (!pool_in || !pool_out || !table_dev || !src_off_dev)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: null pointer");
  if (pool_in == pool_out)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: the register round runs out of place (snapshot semantics)");
  const int64_t n2 = n + (n & 1);  // the last lane of an odd row reads one element of padding
  if (n < 0 || ld_in < n2 || ld_out < n2 || ld_in % 2 || ld_out % 2)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: need even ld >= n rounded up to even");
  if (n_groups < 0 || max_src < 1 || max_src > kRegMaxSrc || off_src < 4 * n_groups || off_pairs % 4 ||
      off_rec % 16 || off_pairs < off_src || off_rec < off_pairs)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: bad table layout");
  if (bf16 && mode == TAL_MODE_EXACT)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: bf16 rounds take FMA mode here (EXACT: tal_agg_round_bf16)");
  if (bf16 ? !aligned4(pool_in) || !aligned4(pool_out) : !aligned8(pool_in) || !aligned8(pool_out))
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: pools must be aligned to 2 elements");
  if (reinterpret_cast<uintptr_t>(table_dev) % 64)
    return fail(TAL_ERR_INVALID, "tal_agg_round_reg: table must be 64-B aligned");
  if (n == 0 || n_groups == 0) { g_err.clear(); return TAL_OK; }
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (bf16)
    return launch_round_reg<uint16_t, false>(static_cast<const uint16_t*>(pool_in), static_cast<uint16_t*>(pool_out),
                                             ld_out, n, table_dev, src_off_dev, n_groups, off_pairs, max_src, s);
  if (mode == TAL_MODE_EXACT)
    return launch_round_reg<float, true>(static_cast<const float*>(pool_in), static_cast<float*>(pool_out), ld_out, n,
                                         table_dev, src_off_dev, n_groups, off_pairs, max_src, s);
  return launch_round_reg<float, false>(static_cast<const float*>(pool_in), static_cast<float*>(pool_out), ld_out, n,
                                        table_dev, src_off_dev, n_groups, off_pairs, max_src, s);
}

int32_t tal_agg_bf16(const uint16_t* const* x_host, const double* w_host, int32_t m, uint16_t* out,
                     int64_t n, int32_t mode, void* stream) {
  if (m <= 0) return fail(TAL_ERR_INVALID, "tal_agg_bf16: m must be >= 1");
  if (n < 0) return fail(TAL_ERR_INVALID, "tal_agg_bf16: n < 0");
  if (!x_host || !w_host || (n > 0 && !out)) return fail(TAL_ERR_INVALID, "tal_agg_bf16: null pointer");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  if (m > kMaxOps) {  // the chain in passes through an fp32 scratch (k_agg_chain)
    for (int i = 0; i < m; ++i)
      if (!x_host[i]) return fail(TAL_ERR_INVALID, "tal_agg_bf16: null operand pointer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    return mode == TAL_MODE_EXACT ? agg_chain<uint16_t, true>(x_host, w_host, m, out, n, s, "tal_agg_bf16")
                                  : agg_chain<uint16_t, false>(x_host, w_host, m, out, n, s, "tal_agg_bf16");
  }
  OpTableB16 t;
  bool vec = aligned8(out);
  for (int i = 0; i < m; ++i) {
    if (!x_host[i]) return fail(TAL_ERR_INVALID, "tal_agg_bf16: null operand pointer");
    t.x[i] = x_host[i];
    t.w[i] = static_cast<float>(w_host[i]);
    vec = vec && aligned8(x_host[i]);
  }
  for (int i = m; i < kMaxOps; ++i) { t.x[i] = nullptr; t.w[i] = 0.f; }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool exact = mode == TAL_MODE_EXACT;
  const int64_t n4 = vec ? n / 4 : 0;
  if (n4) {
    int64_t nb = (n4 + kBlock * kK1Unroll - 1) / (kBlock * kK1Unroll);
    nb = std::max<int64_t>(1, std::min<int64_t>(nb, kK1Grid));
    if (exact) k_agg_b16_vec<true><<<static_cast<unsigned>(nb), kBlock, 0, s>>>(t, m, out, n4);
    else k_agg_b16_vec<false><<<static_cast<unsigned>(nb), kBlock, 0, s>>>(t, m, out, n4);
  }
  if (n > 4 * n4) {
    if (exact) k_agg_b16_scalar<true><<<grid_for(n - 4 * n4), kBlock, 0, s>>>(t, m, out, 4 * n4, n);
    else k_agg_b16_scalar<false><<<grid_for(n - 4 * n4), kBlock, 0, s>>>(t, m, out, 4 * n4, n);
  }
  return check_launch("tal_agg_bf16");
}

int32_t tal_agg_round_bf16(const uint16_t* pool_in, int64_t ld_in, uint16_t* pool_out, int64_t ld_out,
                           int64_t n, const int32_t* plan_dev, const tal_round_plan_info* info,
                           int32_t mode, void* stream) {
  int32_t rc = validate_info(info);
  if (rc) return rc;
  const bool wide = info->stream_cs != 0;  // a streamed plan: the wide-row form (<= 16 rows per group)
  if ((info->dense_rb != 0 && !wide) || (wide && info->max_rows > kWideRows))
    return fail(TAL_ERR_INVALID, "tal_agg_round_bf16: bf16 rounds take sparse or narrow plans (dense_rb 0), or "
                                 "streamed plans of at most 16 rows per group (the wide-row form)");
  if (!pool_in || !pool_out || !plan_dev) return fail(TAL_ERR_INVALID, "tal_agg_round_bf16: null pointer");
  if (n < 0 || ld_in < n || ld_out < n) return fail(TAL_ERR_INVALID, "tal_agg_round_bf16: bad n / ld");
  if (pool_in == pool_out && info->n_groups > 1)
    return fail(TAL_ERR_INVALID,
                "tal_agg_round_bf16: in-place round needs a single-group plan (snapshot semantics)");
  if (n == 0) { g_err.clear(); return TAL_OK; }
  hipStream_t s = static_cast<hipStream_t>(stream);
  const PlanView v = make_view(plan_dev, *info);
  const bool exact = mode == TAL_MODE_EXACT;
  const bool vec = aligned8(pool_in) && aligned8(pool_out) && ld_in % 4 == 0 && ld_out % 4 == 0;
  int64_t e_vec = 0;
  if (vec) {
    const int64_t n4 = n / 4;
    e_vec = n4 * 4;
    if (n4 > 0 && wide) {
      rc = launch_round_wide<uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, exact, s);
      if (rc) return rc;
    } else if (n4 > 0) {
      switch (info->c4 * 2 + (exact ? 1 : 0)) {
        case 33: rc = launch_round_narrow<16, true, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 32: rc = launch_round_narrow<16, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 65: rc = launch_round_narrow<32, true, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 64: rc = launch_round_narrow<32, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 129: rc = launch_round_vec<64, true, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 128: rc = launch_round_vec<64, false, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        case 257: rc = launch_round_vec<128, true, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
        default: rc = launch_round_vec<128, false, false, uint16_t>(pool_in, ld_in, pool_out, ld_out, n4, v, *info, s); break;
      }
      if (rc) return rc;
    }
  }
  if (n <= e_vec) return TAL_OK;
  if (use_direct(pool_in, pool_out, e_vec, n))
    return launch_round_direct<uint16_t>(pool_in, ld_in, pool_out, ld_out, e_vec, n, v, *info, exact, s);
  return launch_round_scalar<uint16_t>(pool_in, ld_in, pool_out, ld_out, e_vec, n, v, *info, exact, s);
}

static int cos_kind(int64_t I, int64_t B) { return I == 1 ? kCosElem : (B == 1 ? kCosRow : kCosCol); }

// outputs per chunk of a tensor and whether its chunks are streamed (k_cos_col_norms /
// k_cos_col_prods: Ob output blocks of the column kind) or direct (k_cosine_outputs)
static int64_t cos_seg_per(int64_t A, int64_t I, int64_t B, bool* staged) {
  const int kind = cos_kind(I, B);
  *staged = cos_col_streamed(kind, I, B);
  (void)A;
  return *staged ? cos_col_ob(B) * B : cos_chunk_outputs(kind);
}

int64_t tal_cosine_plan_words(const int64_t* seg_host, int32_t n_seg) {
  if (!seg_host || n_seg <= 0) return -1;
  int64_t chunks = 0;
  for (int s = 0; s < n_seg; ++s) {
    const int64_t A = seg_host[4 * s + 1], I = seg_host[4 * s + 2], B = seg_host[4 * s + 3];
    if (A <= 0 || I <= 0 || B <= 0 || seg_host[4 * s] < 0) return -1;
    bool staged;
    const int64_t per = cos_seg_per(A, I, B, &staged);
    chunks += (A * B + per - 1) / per;
  }
  return kCosHdr + kCosSegWords * static_cast<int64_t>(n_seg) + kCosChunkWords * chunks;
}

int32_t tal_cosine_plan_build(const int64_t* seg_host, int32_t n_seg, int64_t* plan_host,
                              int64_t plan_capacity_words, int32_t* n_chunks) {
  const int64_t words = tal_cosine_plan_words(seg_host, n_seg);
  if (words < 0 || !plan_host || !n_chunks)
    return fail(TAL_ERR_INVALID, "tal_cosine_plan_build: bad segments");
  if (plan_capacity_words < words) return fail(TAL_ERR_INVALID, "tal_cosine_plan_build: buffer too small");
  int64_t* sg = plan_host + kCosHdr;
  int64_t* ch = sg + kCosSegWords * static_cast<int64_t>(n_seg);
  int64_t c = 0, out = 0, n_staged = 0;
  for (int s = 0; s < n_seg; ++s) {
    const int64_t A = seg_host[4 * s + 1], I = seg_host[4 * s + 2], B = seg_host[4 * s + 3];
    bool staged;
    sg[kCosSegWords * s + 0] = seg_host[4 * s];
    sg[kCosSegWords * s + 1] = A;
    sg[kCosSegWords * s + 2] = I;
    sg[kCosSegWords * s + 3] = B;
    sg[kCosSegWords * s + 4] = out;
    sg[kCosSegWords * s + 5] = cos_kind(I, B);
    sg[kCosSegWords * s + 6] = cos_seg_per(A, I, B, &staged);
    if (staged) n_staged += (A * B + sg[kCosSegWords * s + 6] - 1) / sg[kCosSegWords * s + 6];
    out += A * B;
  }
  // the streamed chunks first (k_cos_col_norms / k_cos_col_prods take chunks 0 .. n_staged - 1,
  // k_cosine_outputs the rest); a chunk writes only its own outputs, so the order is free
  for (int pass = 1; pass >= 0; --pass) {
    for (int s = 0; s < n_seg; ++s) {
      const int64_t A = sg[kCosSegWords * s + 1], B = sg[kCosSegWords * s + 3], per = sg[kCosSegWords * s + 6];
      bool staged;
      cos_seg_per(A, sg[kCosSegWords * s + 2], B, &staged);
      if (staged != (pass == 1)) continue;
      const int64_t total = A * B;
      for (int64_t f = 0; f < total; f += per) {
        ch[kCosChunkWords * c + 0] = s;
        ch[kCosChunkWords * c + 1] = f;
        ch[kCosChunkWords * c + 2] = std::min(per, total - f);
        ch[kCosChunkWords * c + 3] = staged ? 1 : 0;
        ++c;
      }
    }
  }
  if (c > 0x7fffffff) return fail(TAL_ERR_INVALID, "tal_cosine_plan_build: too many chunks");
  plan_host[0] = n_seg;
  plan_host[1] = out;
  plan_host[2] = 1;  // serial sums until tal_cosine_plan_set_threads says otherwise
  plan_host[3] = n_staged;
  *n_chunks = static_cast<int32_t>(c);
  g_err.clear();
  return TAL_OK;
}

int32_t tal_cosine_plan_set_threads(int64_t* plan_host, int32_t threads) {
  if (!plan_host || plan_host[0] <= 0 || plan_host[1] <= 0)
    return fail(TAL_ERR_INVALID, "tal_cosine_plan_set_threads: not a built plan");
  if (threads < 1 || threads > kCosMaxThreads)
    return fail(TAL_ERR_INVALID, "tal_cosine_plan_set_threads: threads must be 1..1024");
  plan_host[2] = threads;
  g_err.clear();
  return TAL_OK;
}

int64_t tal_cosine_scratch_bytes(const int64_t* plan_host, int32_t n_pairs) {
  if (!plan_host || n_pairs <= 0 || plan_host[0] <= 0 || plan_host[1] <= 0) return -1;
  // per pair of one launch: its outputs and per-tensor means, and two model slots of norms
  return static_cast<int64_t>(sizeof(float)) * (3 * plan_host[1] + plan_host[0]) * std::min(n_pairs, kCosMaxPairs);
}

// K2's side stream on the current device: created on first use and kept for the process (one
// per device, shared by every calling thread: each call joins its own caller's stream through
// its own events, so calls from several threads stay correct - their direct chunks queue on the
// one side stream).  The fork / join events are made per call and released right after their
// waits are enqueued (HIP frees a pending event's resources when it completes).
static std::mutex g_cos_side_mu;

static hipStream_t cos_side_stream() {
  static hipStream_t side[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_cos_side_mu);
  if (!side[dev] && hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking) != hipSuccess) side[dev] = nullptr;
  return side[dev];
}

// record an event on `from` and make `to` wait for it
static bool cos_stream_wait(hipStream_t to, hipStream_t from) {
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
  const bool ok = hipEventRecord(e, from) == hipSuccess && hipStreamWaitEvent(to, e, 0) == hipSuccess;
  hipEventDestroy(e);
  return ok;
}

int32_t tal_cosine_params(const float* const* a_ptrs_host, const float* const* b_ptrs_host,
                          int32_t n_pairs, const int64_t* plan_dev, const int64_t* plan_host, int32_t n_chunks,
                          void* scratch, float* out_dev, void* stream) {
  if (!a_ptrs_host || !b_ptrs_host || !plan_dev || !plan_host || !scratch || !out_dev || n_pairs <= 0 ||
      n_chunks <= 0 || plan_host[0] <= 0 || plan_host[1] <= 0)
    return fail(TAL_ERR_INVALID, "tal_cosine_params: bad arguments");
  const int n_seg = static_cast<int>(plan_host[0]);
  const int64_t n_out = plan_host[1];
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < n_pairs; base += kCosMaxPairs) {
    const int cnt = std::min(kCosMaxPairs, n_pairs - base);
    CosPairs pr;
    for (int j = 0; j < kCosMaxPairs; ++j) {
      pr.a[j] = j < cnt ? a_ptrs_host[base + j] : nullptr;
      pr.b[j] = j < cnt ? b_ptrs_host[base + j] : nullptr;
      if (j < cnt && (!pr.a[j] || !pr.b[j]))
        return fail(TAL_ERR_INVALID, "tal_cosine_params: null model pointer");
    }
    float* s_all = static_cast<float*>(scratch);
    float* means = s_all + n_out * cnt;
    const int64_t n_staged = plan_host[3];
    // pairs sharing one `a` (sim_centrality_module_avg: the client against each neighbor): its
    // norms once, and up to kColPairs pairs per product workgroup read its chunk once
    bool same_a = true;
    for (int j = 1; j < cnt; ++j) same_a = same_a && pr.a[j] == pr.a[0];
    // the direct chunks do not depend on the streamed ones: with both present they run on the
    // device's side stream, forked from and joined back into `s`, so they fill the GPU beside the
    // streamed kernels' workgroups
    const bool fork = n_staged > 0 && n_chunks > n_staged;
    hipStream_t so = s;
    if (fork) {
      so = cos_side_stream();
      if (!so) return fail(TAL_ERR_HIP, "tal_cosine_params: side stream");
      if (!cos_stream_wait(so, s)) return fail(TAL_ERR_HIP, "tal_cosine_params: fork");
    }
    if (n_chunks > n_staged) {
      const int64_t n_direct = n_chunks - n_staged;
      k_cosine_outputs<<<static_cast<unsigned>((n_direct + 7) / 8 * 8 * cnt), kCosBlock, 0, so>>>(pr, plan_dev, n_seg,
                                                                                                 cnt, n_direct, s_all);
    }
    if (n_staged > 0) {
      float* nrm = means + static_cast<int64_t>(n_seg) * cnt;  // model slots x n_out
      const int n_models = same_a ? 1 + cnt : 2 * cnt;
      const int ppw = same_a ? kColPairs : kColPairs / 2;
      k_cos_col_norms<<<dim3(static_cast<unsigned>(n_staged), (n_models + 7) / 8), kColThreads, 0, s>>>(
          pr, plan_dev, n_seg, cnt, same_a ? 1 : 0, nrm);
      k_cos_col_prods<<<dim3(static_cast<unsigned>(n_staged), (cnt + ppw - 1) / ppw), kColThreads, 0, s>>>(
          pr, plan_dev, n_seg, cnt, same_a ? 1 : 0, nrm, s_all);
    }
    if (fork && !cos_stream_wait(s, so)) return fail(TAL_ERR_HIP, "tal_cosine_params: join");
    k_cosine_means<<<dim3(n_seg, cnt), 64, 0, s>>>(plan_dev, n_seg, s_all, means);
    k_cosine_finish<<<cnt, 64, 0, s>>>(n_seg, means, out_dev, base);
  }
  return check_launch("tal_cosine_params");
}


int64_t tal_prox_plan_words(const int64_t* seg_host, int32_t n_seg) {
  if (!seg_host || n_seg <= 0) return -1;
  int64_t chunks = 0;
  for (int s = 0; s < n_seg; ++s) {
    if (seg_host[2 * s] < 0 || seg_host[2 * s + 1] <= 0) return -1;
    chunks += (seg_host[2 * s + 1] + kProxChunk - 1) / kProxChunk;
  }
  return (n_seg + 1) + 3 * chunks;
}

int32_t tal_prox_plan_build(const int64_t* seg_host, int32_t n_seg, int64_t* plan_host,
                            int64_t plan_capacity_words, int32_t* n_chunks) {
  const int64_t words = tal_prox_plan_words(seg_host, n_seg);
  if (words < 0 || !n_chunks) return fail(TAL_ERR_INVALID, "tal_prox_plan_build: bad segments");
  if (!plan_host || words > plan_capacity_words)
    return fail(TAL_ERR_CAPACITY, "tal_prox_plan_build: plan buffer too small: need " + std::to_string(words));
  const int64_t nc = (words - (n_seg + 1)) / 3;
  if (nc > 0x7fffffff) return fail(TAL_ERR_INVALID, "tal_prox_plan_build: too many chunks");
  int64_t c = 0;
  int64_t* ch = plan_host + (n_seg + 1);
  for (int s = 0; s < n_seg; ++s) {
    plan_host[s] = c;
    for (int64_t b = 0; b < seg_host[2 * s + 1]; b += kProxChunk, ++c) {
      ch[3 * c] = s;
      ch[3 * c + 1] = seg_host[2 * s] + b;
      ch[3 * c + 2] = std::min<int64_t>(kProxChunk, seg_host[2 * s + 1] - b);
    }
  }
  plan_host[n_seg] = c;
  *n_chunks = static_cast<int32_t>(nc);
  g_err.clear();
  return TAL_OK;
}

int64_t tal_prox_scratch_bytes(int32_t n_chunks, int32_t k) {
  return static_cast<int64_t>(sizeof(double)) * n_chunks * std::min<int32_t>(k, kProxMaxNb);
}

int32_t tal_prox_norms(const float* w, const float* const* wt_host, int32_t k, const int64_t* plan_dev,
                       int32_t n_chunks, int32_t n_seg, void* scratch, float* norms_out, void* stream) {
  if (!w || !wt_host || k <= 0 || !plan_dev || n_chunks <= 0 || n_seg <= 0 || !scratch || !norms_out)
    return fail(TAL_ERR_INVALID, "tal_prox_norms: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < k; base += kProxMaxNb) {
    const int cnt = std::min(kProxMaxNb, k - base);
    ProxPtrs pp{};
    for (int j = 0; j < cnt; ++j) {
      if (!wt_host[base + j]) return fail(TAL_ERR_INVALID, "tal_prox_norms: null neighbor pointer");
      pp.wt[j] = wt_host[base + j];
    }
    double* part = static_cast<double*>(scratch);
    k_prox_sumsq<<<n_chunks, kBlock, 0, s>>>(w, pp, cnt, plan_dev, n_seg, n_chunks, part);
    const int64_t outs = static_cast<int64_t>(cnt) * n_seg;
    k_prox_finish<<<static_cast<unsigned>((outs + 255) / 256), 256, 0, s>>>(
        plan_dev, n_seg, n_chunks, cnt, part, norms_out + static_cast<int64_t>(base) * n_seg);
    int32_t rc = check_launch("prox norms");
    if (rc) return rc;
  }
  g_err.clear();
  return TAL_OK;
}

int32_t tal_prox_grad(const float* w, const float* const* wt_host, int32_t k, const int64_t* plan_dev,
                      int32_t n_chunks, int32_t n_seg, const float* norms, const float* scale_dev,
                      float* gw, float* const* gwt_host, void* stream) {
  if (!w || !wt_host || k <= 0 || !plan_dev || n_chunks <= 0 || n_seg <= 0 || !norms || !scale_dev || !gw)
    return fail(TAL_ERR_INVALID, "tal_prox_grad: bad arguments");
  hipStream_t s = static_cast<hipStream_t>(stream);
  for (int base = 0; base < k; base += kProxMaxNb) {
    const int cnt = std::min(kProxMaxNb, k - base);
    ProxPtrs pp{};
    for (int j = 0; j < cnt; ++j) {
      if (!wt_host[base + j]) return fail(TAL_ERR_INVALID, "tal_prox_grad: null neighbor pointer");
      pp.wt[j] = wt_host[base + j];
      pp.gwt[j] = gwt_host ? gwt_host[base + j] : nullptr;
    }
    k_prox_grad<<<n_chunks, kBlock, 0, s>>>(w, pp, cnt, plan_dev, n_seg,
                                           norms + static_cast<int64_t>(base) * n_seg, scale_dev, gw,
                                           base > 0 ? 1 : 0);
    int32_t rc = check_launch("prox grad");
    if (rc) return rc;
  }
  g_err.clear();
  return TAL_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Synthetic pool rows: synth.py's counter generator, one launch per pool segment
// ------------------------------------------------------------------------------------------
namespace {

constexpr int kFillHeader = 8;  // {n_rows, n, n_runs, n_rv, hi, 0, 0, 0}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// counter_f32 (synth.py): random sign, exponent 121..128, the low 23 bits as mantissa
__device__ __forceinline__ uint32_t counter_f32_bits(uint64_t u) {
  return static_cast<uint32_t>(((u >> 31) & 1u) << 31 | (121u + ((u >> 23) & 7u)) << 23 | (u & 0x7FFFFFu));
}

// Block (x, r) fills columns of segment row r; each lane finds its column's generator position
// from the run table (run = {position, first column, length}, ascending columns covering
// [0, n)), starting from the run of the block's first column (found once, block-uniform) and
// stepping forward, so a lane walks at most the few runs one 256-column stretch crosses.
template <int DT>  // 0 fp32, 1 bf16 (nearest even of the fp32 value), 2 int64 (u % hi)
__global__ __launch_bounds__(kBlock) void k_fill_counter(void* __restrict__ seg, int64_t ld,
                                                         const int64_t* __restrict__ tab) {
  const int64_t n = tab[1];
  const int n_runs = static_cast<int>(tab[2]), n_rv = static_cast<int>(tab[3]);
  const uint64_t hi = static_cast<uint64_t>(tab[4]);
  const int64_t* seeds = tab + kFillHeader;
  const int64_t* runs = seeds + tab[0];
  const int64_t* rv = runs + 3 * n_runs;
  const int64_t r = blockIdx.y;
  const uint64_t key = (static_cast<uint64_t>(seeds[r]) & 0xFFFFFFFFull) << 40;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t c0 = static_cast<int64_t>(blockIdx.x) * kBlock; c0 < n; c0 += stride) {
    int lo = 0, hi_r = n_runs - 1;  // last run starting at or before c0 (uniform)
    while (lo < hi_r) {
      const int mid = (lo + hi_r + 1) >> 1;
      if (runs[3 * mid + 1] <= c0) lo = mid;
      else hi_r = mid - 1;
    }
    int vlo = 0, vhi = n_rv - 1;  // last running_var range starting at or before c0
    while (vlo < vhi) {
      const int mid = (vlo + vhi + 1) >> 1;
      if (rv[2 * mid] <= c0) vlo = mid;
      else vhi = mid - 1;
    }
    const int64_t c = c0 + threadIdx.x;
    if (c >= n) break;
    int k = lo;
    while (k + 1 < n_runs && runs[3 * (k + 1) + 1] <= c) ++k;
    const uint64_t u = splitmix64(static_cast<uint64_t>(runs[3 * k] + (c - runs[3 * k + 1])) ^ key);
    if constexpr (DT == 2) {
      static_cast<int64_t*>(seg)[r * ld + c] = static_cast<int64_t>(u % hi);
    } else {
      uint32_t bits = counter_f32_bits(u);
      if constexpr (DT == 0) {
        int v = vlo;
        while (v + 1 < n_rv && rv[2 * (v + 1)] <= c) ++v;
        if (n_rv > 0 && c >= rv[2 * v] && c < rv[2 * v] + rv[2 * v + 1])  // |v| + 0.5 in fp32
          bits = __float_as_uint(__fadd_rn(__uint_as_float(bits & 0x7FFFFFFFu), 0.5f));
        static_cast<float*>(seg)[r * ld + c] = __uint_as_float(bits);
      } else {  // finite values: nearest even is the add-and-truncate form
        static_cast<uint16_t*>(seg)[r * ld + c] = static_cast<uint16_t>((bits + 0x7FFFu + ((bits >> 16) & 1u)) >> 16);
      }
    }
  }
}

}  // namespace

extern "C" {

int32_t tal_fill_counter(void* seg, int64_t ld, int32_t dtype, const int64_t* table_dev,
                         const int64_t* table_host, void* stream) {
  if (!seg || !table_dev || !table_host || dtype < 0 || dtype > 2)
    return fail(TAL_ERR_INVALID, "tal_fill_counter: bad arguments");
  const int64_t n_rows = table_host[0], n = table_host[1], n_runs = table_host[2], n_rv = table_host[3];
  const int64_t hi = table_host[4];
  if (n_rows < 0 || n_rows > 65535 || n < 0 || n > ld || n_runs < 0 || n_rv < 0 || (dtype == 2 && hi <= 0))
    return fail(TAL_ERR_INVALID, "tal_fill_counter: bad table header");
  if (n_rows == 0 || n == 0) {
    g_err.clear();
    return TAL_OK;
  }
  // the runs must tile [0, n) in ascending columns (every lane's walk then stays in the table)
  const int64_t* runs = table_host + kFillHeader + n_rows;
  int64_t col = 0;
  for (int64_t k = 0; k < n_runs; ++k) {
    if (runs[3 * k + 1] != col || runs[3 * k + 2] <= 0 || runs[3 * k] < 0)
      return fail(TAL_ERR_INVALID, "tal_fill_counter: runs must tile the columns in order");
    col += runs[3 * k + 2];
  }
  if (col != n) return fail(TAL_ERR_INVALID, "tal_fill_counter: runs do not cover the row");
  const int64_t* rv = runs + 3 * n_runs;
  for (int64_t k = 0; k < n_rv; ++k)
    if (rv[2 * k] < 0 || rv[2 * k + 1] < 0 || (k && rv[2 * k] < rv[2 * k - 2] + rv[2 * k - 1]))
      return fail(TAL_ERR_INVALID, "tal_fill_counter: running_var ranges must ascend without overlap");
  const unsigned gx = static_cast<unsigned>(std::min<int64_t>((n + kBlock - 1) / kBlock, 4096));
  const dim3 grid(gx, static_cast<unsigned>(n_rows));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (dtype == 0) k_fill_counter<0><<<grid, kBlock, 0, s>>>(seg, ld, table_dev);
  else if (dtype == 1) k_fill_counter<1><<<grid, kBlock, 0, s>>>(seg, ld, table_dev);
  else k_fill_counter<2><<<grid, kBlock, 0, s>>>(seg, ld, table_dev);
  return check_launch("tal_fill_counter");
}

}  // extern "C"

// ------------------------------------------------------------------------------------------
// Multi-GPU halo exchange: pack kernel + RCCL group (include/tal_agg.h, halo section)
// ------------------------------------------------------------------------------------------
namespace {

// rows -> contiguous: block (x, r) copies part of row rows[r]; W = 16 or 4 bytes per lane
template <typename V>
__global__ __launch_bounds__(kBlock) void k_halo_pack(const V* __restrict__ pool, int64_t ld, int64_t pool_rows,
                                                      const int32_t* __restrict__ rows, int64_t row_n,
                                                      V* __restrict__ buf) {
  const int64_t src = rows[blockIdx.y];
  if (src < 0 || src >= pool_rows) return;  // out-of-range rows are skipped, never read
  const V* in = pool + src * ld;
  V* out = buf + static_cast<int64_t>(blockIdx.y) * row_n;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < row_n;
       i += static_cast<int64_t>(gridDim.x) * kBlock)
    out[i] = in[i];
}

// RCCL is resolved at run time (dlopen / dlsym), not linked: only the halo entry points need
// it, so a host without RCCL still loads the library (they return TAL_ERR_COMM), and under
// torch the soname lookup finds the copy torch already loaded instead of a second instance.
struct Rccl {
  bool ok = false;
  std::string why;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
      if ((h = dlopen(name, RTLD_NOW | RTLD_GLOBAL)) != nullptr) break;
    if (!h) {
      const char* e = dlerror();
      x.why = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1 not found");
      return x;
    }
    bool all = true;
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn) {
        all = false;
        x.why = std::string("RCCL lacks ") + name;
      }
    };
    sym(x.GetErrorString, "ncclGetErrorString");
    sym(x.GetUniqueId, "ncclGetUniqueId");
    sym(x.CommInitRank, "ncclCommInitRank");
    sym(x.CommInitAll, "ncclCommInitAll");
    sym(x.CommDestroy, "ncclCommDestroy");
    sym(x.CommCount, "ncclCommCount");
    sym(x.GroupStart, "ncclGroupStart");
    sym(x.GroupEnd, "ncclGroupEnd");
    sym(x.Send, "ncclSend");
    sym(x.Recv, "ncclRecv");
    x.ok = all;
    return x;
  }();
  return r;
}

int32_t comm_fail(const char* what, ncclResult_t r) {
  return fail(TAL_ERR_COMM, std::string(what) + ": " + rccl().GetErrorString(r));
}

#define TAL_NEED_RCCL(fn)                                                      \
  do {                                                                         \
    if (!rccl().ok) return fail(TAL_ERR_COMM, std::string(fn ": ") + rccl().why); \
  } while (0)

}  // namespace

extern "C" {

int32_t tal_comm_unique_id(void* id_out) {
  if (!id_out) return fail(TAL_ERR_INVALID, "tal_comm_unique_id: null output");
  TAL_NEED_RCCL("tal_comm_unique_id");
  ncclUniqueId id;
  const ncclResult_t r = rccl().GetUniqueId(&id);
  if (r != ncclSuccess) return comm_fail("ncclGetUniqueId", r);
  memcpy(id_out, &id, sizeof(id));
  g_err.clear();
  return TAL_OK;
}

int32_t tal_comm_init(void** comm_out, int32_t world, int32_t rank, const void* id, int32_t device) {
  if (!comm_out || !id || world <= 0 || rank < 0 || rank >= world || device < 0)
    return fail(TAL_ERR_INVALID, "tal_comm_init: bad arguments");
  TAL_NEED_RCCL("tal_comm_init");
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return fail(TAL_ERR_HIP, "tal_comm_init: cannot select device " + std::to_string(device));
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ncclResult_t r = rccl().CommInitRank(&c, world, uid, rank);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) return comm_fail("ncclCommInitRank", r);
  *comm_out = c;
  g_err.clear();
  return TAL_OK;
}

int32_t tal_comm_destroy(void* comm) {
  if (!comm) return fail(TAL_ERR_INVALID, "tal_comm_destroy: null communicator");
  TAL_NEED_RCCL("tal_comm_destroy");
  const ncclResult_t r = rccl().CommDestroy(static_cast<ncclComm_t>(comm));
  if (r != ncclSuccess) return comm_fail("ncclCommDestroy", r);
  g_err.clear();
  return TAL_OK;
}

int32_t tal_comm_init_local(void** comms_out, int32_t n, const int32_t* devices) {
  if (!comms_out || !devices || n <= 0) return fail(TAL_ERR_INVALID, "tal_comm_init_local: bad arguments");
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < i; ++j)
      if (devices[i] == devices[j] || devices[i] < 0)
        return fail(TAL_ERR_INVALID, "tal_comm_init_local: devices must be distinct (RCCL takes one rank per device)");
  TAL_NEED_RCCL("tal_comm_init_local");
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return fail(TAL_ERR_HIP, "tal_comm_init_local: hipGetDevice");
  std::vector<ncclComm_t> c(static_cast<size_t>(n), nullptr);
  const ncclResult_t r = rccl().CommInitAll(c.data(), n, devices);
  (void)hipSetDevice(prev);
  if (r != ncclSuccess) return comm_fail("ncclCommInitAll", r);
  for (int i = 0; i < n; ++i) comms_out[i] = c[i];
  g_err.clear();
  return TAL_OK;
}

int32_t tal_halo_exchange_local(void* const* comms, int32_t n, const void* const* send_bufs, const int64_t* send_bytes,
                                void* const* recv_bufs, const int64_t* recv_bytes, void* const* streams) {
  if (!comms || n <= 0 || !send_bytes || !recv_bytes || !streams)
    return fail(TAL_ERR_INVALID, "tal_halo_exchange_local: bad arguments");
  TAL_NEED_RCCL("tal_halo_exchange_local");
  for (int r = 0; r < n; ++r) {
    if (!comms[r]) return fail(TAL_ERR_INVALID, "tal_halo_exchange_local: null communicator");
    int cnt = 0;
    const ncclResult_t rc = rccl().CommCount(static_cast<ncclComm_t>(comms[r]), &cnt);
    if (rc != ncclSuccess) return comm_fail("ncclCommCount", rc);
    if (cnt != n) return fail(TAL_ERR_INVALID, "tal_halo_exchange_local: n differs from the communicators' size");
    for (int p = 0; p < n; ++p) {
      const int64_t k = static_cast<int64_t>(r) * n + p;
      if (send_bytes[k] < 0 || recv_bytes[k] < 0 || (send_bytes[k] && (!send_bufs || !send_bufs[k])) ||
          (recv_bytes[k] && (!recv_bufs || !recv_bufs[k])))
        return fail(TAL_ERR_INVALID, "tal_halo_exchange_local: bad buffer for rank " + std::to_string(r) + ", peer " +
                                         std::to_string(p));
    }
  }
  // one group over every local rank's sends and receives: RCCL needs them together when one
  // thread drives several of the communicator's ranks
  ncclResult_t r = rccl().GroupStart();
  if (r != ncclSuccess) return comm_fail("ncclGroupStart", r);
  ncclResult_t first = ncclSuccess;
  for (int q = 0; q < n && first == ncclSuccess; ++q) {
    ncclComm_t c = static_cast<ncclComm_t>(comms[q]);
    hipStream_t st = static_cast<hipStream_t>(streams[q]);
    for (int p = 0; p < n && first == ncclSuccess; ++p) {
      const int64_t k = static_cast<int64_t>(q) * n + p;
      if (send_bytes[k]) first = rccl().Send(send_bufs[k], static_cast<size_t>(send_bytes[k]), ncclUint8, p, c, st);
      if (first == ncclSuccess && recv_bytes[k])
        first = rccl().Recv(recv_bufs[k], static_cast<size_t>(recv_bytes[k]), ncclUint8, p, c, st);
    }
  }
  r = rccl().GroupEnd();
  if (first != ncclSuccess) return comm_fail("ncclSend / ncclRecv", first);
  if (r != ncclSuccess) return comm_fail("ncclGroupEnd", r);
  g_err.clear();
  return TAL_OK;
}

int32_t tal_halo_pack(const void* pool, int64_t ld_bytes, int64_t pool_rows, const int32_t* rows_dev,
                      int32_t n_rows, int64_t row_bytes, void* buf, void* stream) {
  if (n_rows == 0) {
    g_err.clear();
    return TAL_OK;
  }
  if (!pool || !rows_dev || !buf || n_rows < 0 || n_rows > 65535 || row_bytes <= 0 || ld_bytes < row_bytes ||
      pool_rows <= 0)
    return fail(TAL_ERR_INVALID, "tal_halo_pack: bad arguments");
  if ((row_bytes | ld_bytes) & 3 || (reinterpret_cast<uintptr_t>(pool) | reinterpret_cast<uintptr_t>(buf)) & 3)
    return fail(TAL_ERR_INVALID, "tal_halo_pack: rows, pitch and pointers must be 4-byte aligned");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool v16 = ((row_bytes | ld_bytes) & 15) == 0 && aligned16(pool) && aligned16(buf);
  const int64_t w = v16 ? 16 : 4;
  const int64_t row_n = row_bytes / w;
  const dim3 grid(static_cast<unsigned>(std::min<int64_t>((row_n + kBlock - 1) / kBlock, 1024)),
                  static_cast<unsigned>(n_rows));
  if (v16)
    k_halo_pack<uint4><<<grid, kBlock, 0, s>>>(static_cast<const uint4*>(pool), ld_bytes / 16, pool_rows, rows_dev,
                                              row_n, static_cast<uint4*>(buf));
  else
    k_halo_pack<uint32_t><<<grid, kBlock, 0, s>>>(static_cast<const uint32_t*>(pool), ld_bytes / 4, pool_rows,
                                                  rows_dev, row_n, static_cast<uint32_t*>(buf));
  return check_launch("halo pack");
}

int32_t tal_halo_exchange(void* comm, int32_t world, const void* const* send_bufs, const int64_t* send_bytes,
                          void* const* recv_bufs, const int64_t* recv_bytes, void* stream) {
  if (!comm || world <= 0 || !send_bytes || !recv_bytes)
    return fail(TAL_ERR_INVALID, "tal_halo_exchange: bad arguments");
  TAL_NEED_RCCL("tal_halo_exchange");
  ncclComm_t c = static_cast<ncclComm_t>(comm);
  int n = 0;
  ncclResult_t r = rccl().CommCount(c, &n);
  if (r != ncclSuccess) return comm_fail("ncclCommCount", r);
  if (n != world) return fail(TAL_ERR_INVALID, "tal_halo_exchange: world differs from the communicator's size");
  for (int p = 0; p < world; ++p) {
    if (send_bytes[p] < 0 || recv_bytes[p] < 0 || (send_bytes[p] && (!send_bufs || !send_bufs[p])) ||
        (recv_bytes[p] && (!recv_bufs || !recv_bufs[p])))
      return fail(TAL_ERR_INVALID, "tal_halo_exchange: bad buffer for peer " + std::to_string(p));
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  r = rccl().GroupStart();
  if (r != ncclSuccess) return comm_fail("ncclGroupStart", r);
  ncclResult_t first = ncclSuccess;
  for (int p = 0; p < world && first == ncclSuccess; ++p) {
    if (send_bytes[p]) first = rccl().Send(send_bufs[p], static_cast<size_t>(send_bytes[p]), ncclUint8, p, c, s);
    if (first == ncclSuccess && recv_bytes[p])
      first = rccl().Recv(recv_bufs[p], static_cast<size_t>(recv_bytes[p]), ncclUint8, p, c, s);
  }
  r = rccl().GroupEnd();
  if (first != ncclSuccess) return comm_fail("ncclSend / ncclRecv", first);
  if (r != ncclSuccess) return comm_fail("ncclGroupEnd", r);
  g_err.clear();
  return TAL_OK;
}

}  // extern "C"

// ==========================================================================================
// Host reduction: processes that see no GPU (BASELINE config 1 runs the reference's driver on
// CPU models, decentralized_client.py:399-413 on CPU tensors).  The same arithmetic as the
// kernels, element by element in operand order, on host pointers; a process that sees a GPU
// never calls it (aggregate.py dispatches on torch.cuda.is_available()).  Built with
// -ffp-contract=off like the rest of this file: one rounded multiply and one rounded add per
// operand in EXACT mode, as torch's `w * clone(v)` and `+=` on CPU.
// ==========================================================================================
namespace {

constexpr int64_t kHostBlock = 4096;  // elements per block: every operand of a block is read
                                      // before the block is written (out may alias an operand)

inline float host_bf16(uint16_t b) {
  const uint32_t u = static_cast<uint32_t>(b) << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// fp32 -> bf16 round to nearest even, kept as the fp32 value it represents (NaN stays NaN)
inline float host_round_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return f;
  u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
  memcpy(&f, &u, 4);
  return f;
}

// the stored bf16: NaN as 0xFFFF, as torch's vectorized conversion writes it
inline uint16_t host_store_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0xffffu;
  return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

inline int64_t host_trunc_i64(float v) {
  if (!(v >= -9.2233720368547758e18f && v < 9.2233720368547758e18f)) return INT64_MIN;
  return static_cast<int64_t>(v);
}

// Runs body(e0, e1) over [0, n) in blocks, on up to 16 threads for large n.
template <class Body>
void host_blocks(int64_t n, Body body) {
  const int64_t blocks = (n + kHostBlock - 1) / kHostBlock;
  unsigned hw = std::thread::hardware_concurrency();
  const int64_t nt = std::max<int64_t>(1, std::min<int64_t>({blocks / 64, 16, static_cast<int64_t>(hw ? hw : 1)}));
  auto run = [&](int64_t b0, int64_t b1) {
    for (int64_t b = b0; b < b1; ++b) body(b * kHostBlock, std::min(n, (b + 1) * kHostBlock));
  };
  if (nt == 1) {
    run(0, blocks);
    return;
  }
  std::vector<std::thread> th;
  for (int64_t t = 0; t < nt; ++t) th.emplace_back(run, blocks * t / nt, blocks * (t + 1) / nt);
  for (auto& t : th) t.join();
}

int32_t host_args(const char* fn, const void* const* x, const double* w, int32_t m, const void* out, int64_t n) {
  if (m <= 0) return fail(TAL_ERR_INVALID, std::string(fn) + ": m must be >= 1");
  if (n < 0) return fail(TAL_ERR_INVALID, std::string(fn) + ": n < 0");
  if (!x || !w || (n > 0 && !out)) return fail(TAL_ERR_INVALID, std::string(fn) + ": null pointer");
  for (int i = 0; i < m; ++i)
    if (!x[i]) return fail(TAL_ERR_INVALID, std::string(fn) + ": null operand pointer");
  return TAL_OK;
}

// Host cosine similarity (K2's arithmetic on host pointers, for the `*_sim` strategies in a
// process that sees no GPU).  It walks the same plan as K2 (tal_cosine_plan_build: per-tensor
// kind, output offset, 256-output chunks; the thread word) and performs the same fp32 operations
// in the same order - torch's CPU kernels' order, bit for bit: plain fp32 + and * here (this
// file is built with -ffp-contract=off), std::fma where torch fuses, sqrtss for sqrt.
struct HostCos {
  // torch multi_row_sum for one stream: the 4-level cascade whose level boundaries depend only
  // on the element index (a column of a 32-column group is this case too)
  template <class Load>
  static float cascade(Load x, int64_t size) {
    int64_t lg = 0;
    while ((int64_t{1} << lg) < size) ++lg;
    const int64_t lp = lg / 4 > 4 ? lg / 4 : 4;
    const int64_t step = int64_t{1} << lp;
    float lv[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t i = 0;
    for (; i + step <= size;) {
      for (const int64_t e = i + step; i < e; ++i) lv[0] = lv[0] + x(i);
      for (int j = 1; j < 4; ++j) {
        lv[j] = lv[j] + lv[j - 1];
        lv[j - 1] = 0.f;
        if (i & ((step - 1) << (j * lp))) break;
      }
    }
    for (; i < size; ++i) lv[0] = lv[0] + x(i);
    return ((lv[0] + lv[1]) + lv[2]) + lv[3];
  }
  // torch row_sum: four interleaved cascades (elements 4 i + k), the rest into the first, then
  // the other three added to it in order
  template <class Load>
  static float row(Load x, int64_t size) {
    const int64_t q = size / 4;
    float p[4];
    for (int k = 0; k < 4; ++k) p[k] = cascade([&](int64_t i) { return x(4 * i + k); }, q);
    for (int64_t i = 4 * q; i < size; ++i) p[0] = p[0] + x(i);
    return ((p[0] + p[1]) + p[2]) + p[3];
  }
  // torch's serial full sum of n contiguous values (without the store's 0 +): below 8 one
  // row_sum; else 8 lanes (lane l: elements 8 i + l), the tail from 0, then the lanes in order
  template <class Load>
  static float inner(Load x, int64_t n) {
    if (n < kCosVw) return row(x, n);
    const int64_t nv = n / kCosVw;
    float t = 0.f;
    for (int64_t k = nv * kCosVw; k < n; ++k) t = t + x(k);
    for (int l = 0; l < kCosVw; ++l) t = t + row([&](int64_t i) { return x(i * kCosVw + l); }, nv);
    return t;
  }
  static float clampn(float v) { return v < 1e-6f ? 1e-6f : v; }  // NaN stays NaN
  // every output of chunk ch (plan words) of one pair
  static void outputs(const int64_t* plan, int64_t ch, const float* a0, const float* b0, float* s_all) {
    const int64_t n_seg = plan[0];
    const int64_t* c = plan + kCosHdr + kCosSegWords * n_seg + kCosChunkWords * ch;
    const int64_t* sg = plan + kCosHdr + kCosSegWords * c[0];
    const int64_t I = sg[2], B = sg[3];
    const float* a = a0 + sg[0];
    const float* b = b0 + sg[0];
    float* s = s_all + sg[4];
    for (int64_t q = c[1]; q < c[1] + c[2]; ++q) {
      if (sg[5] == kCosElem) {
        const float n1 = clampn(std::sqrt(std::fma(a[q], a[q], 0.f)));
        const float n2 = clampn(std::sqrt(std::fma(b[q], b[q], 0.f)));
        s[q] = 0.f + (a[q] / n1) * (b[q] / n2);
      } else if (sg[5] == kCosCol) {  // reduced dim strided by B
        const int64_t k = q % B;
        const float* x = a + (q / B) * I * B + k;
        const float* y = b + (q / B) * I * B + k;
        float m1 = 0.f, m2 = 0.f;
        for (int64_t i = 0; i < I; ++i) {
          m1 = std::fma(x[i * B], x[i * B], m1);
          m2 = std::fma(y[i * B], y[i * B], m2);
        }
        const float n1 = clampn(std::sqrt(m1)), n2 = clampn(std::sqrt(m2));
        auto pr = [&](int64_t i) { return (x[i * B] / n1) * (y[i * B] / n2); };
        // columns in groups of 32 share one cascade; groups of 8 and single columns: row_sum
        s[q] = 0.f + ((B >= kCosVw && k < B / 32 * 32) ? cascade(pr, I) : row(pr, I));
      } else {  // kCosRow: reduced dim contiguous, torch's 8-lane norm then its inner sum
        const float* x = a + q * I;
        const float* y = b + q * I;
        const int64_t ve = I - I % kCosVw;
        float l1[kCosVw] = {}, l2[kCosVw] = {};
        for (int64_t d = 0; d < ve; d += kCosVw)
          for (int l = 0; l < kCosVw; ++l) {
            l1[l] = std::fma(x[d + l], x[d + l], l1[l]);
            l2[l] = std::fma(y[d + l], y[d + l], l2[l]);
          }
        float t1 = l1[0], t2 = l2[0];
        for (int l = 1; l < kCosVw; ++l) {
          t1 = t1 + l1[l];
          t2 = t2 + l2[l];
        }
        int64_t d = ve;
        for (const int64_t e = ve + (I - ve) / 4 * 4; d < e; ++d) {  // groups of 4: square, add
          t1 = t1 + x[d] * x[d];
          t2 = t2 + y[d] * y[d];
        }
        for (; d < I; ++d) {  // the last < 4: fused
          t1 = std::fma(x[d], x[d], t1);
          t2 = std::fma(y[d], y[d], t2);
        }
        const float n1 = clampn(std::sqrt(t1)), n2 = clampn(std::sqrt(t2));
        s[q] = 0.f + inner([&](int64_t i) { return (x[i] / n1) * (y[i] / n2); }, I);
      }
    }
  }
  // mean of one tensor's outputs: torch's sum (two-pass over T threads' chunks for >= 32768
  // outputs when T > 1) / numel
  static float mean(const int64_t* plan, int64_t seg, const float* s_all) {
    const int64_t* sg = plan + kCosHdr + kCosSegWords * seg;
    const int64_t n = sg[1] * sg[3], T = plan[2];
    const float* s = s_all + sg[4];
    float fin;
    if (n < kCosGrain || T <= 1) {
      fin = inner([&](int64_t i) { return s[i]; }, n);
    } else {
      std::vector<float> part(static_cast<size_t>(T), 0.f);
      const int64_t nt = std::min(T, (n + kCosGrain - 1) / kCosGrain);
      const int64_t chunk = (n + nt - 1) / nt;
      for (int64_t t = 0; t < nt && t * chunk < n; ++t) {
        const float* c = s + t * chunk;
        part[t] = 0.f + inner([&](int64_t i) { return c[i]; }, std::min(chunk, n - t * chunk));
      }
      fin = inner([&](int64_t i) { return part[i]; }, T);
    }
    return (0.f + fin) / static_cast<float>(n);
  }
};

}  // namespace

extern "C" {

int32_t tal_host_agg_f32(const float* const* x_host, const double* w_host, int32_t m, float* out, int64_t n,
                         int32_t mode) {
  if (int32_t rc = host_args("tal_host_agg_f32", reinterpret_cast<const void* const*>(x_host), w_host, m, out, n))
    return rc;
  std::vector<float> w(static_cast<size_t>(m));
  for (int i = 0; i < m; ++i) w[i] = static_cast<float>(w_host[i]);
  const bool exact = mode == TAL_MODE_EXACT;
  host_blocks(n, [&](int64_t e0, int64_t e1) {
    float acc[kHostBlock];
    const int64_t k = e1 - e0;
    for (int64_t e = 0; e < k; ++e) acc[e] = w[0] * x_host[0][e0 + e];
    for (int i = 1; i < m; ++i) {
      const float wi = w[i];
      const float* xi = x_host[i] + e0;
      if (exact)
        for (int64_t e = 0; e < k; ++e) acc[e] = acc[e] + wi * xi[e];
      else
        for (int64_t e = 0; e < k; ++e) acc[e] = std::fma(wi, xi[e], acc[e]);
    }
    memcpy(out + e0, acc, 4 * static_cast<size_t>(k));
  });
  g_err.clear();
  return TAL_OK;
}

int32_t tal_host_agg_i64(const int64_t* const* x_host, const double* w_host, int32_t m, int64_t* out, int64_t n) {
  if (int32_t rc = host_args("tal_host_agg_i64", reinterpret_cast<const void* const*>(x_host), w_host, m, out, n))
    return rc;
  std::vector<float> w(static_cast<size_t>(m));
  for (int i = 0; i < m; ++i) w[i] = static_cast<float>(w_host[i]);
  host_blocks(n, [&](int64_t e0, int64_t e1) {
    float acc[kHostBlock];
    const int64_t k = e1 - e0;
    for (int64_t e = 0; e < k; ++e) acc[e] = w[0] * static_cast<float>(x_host[0][e0 + e]);
    for (int i = 1; i < m; ++i)
      for (int64_t e = 0; e < k; ++e) acc[e] = acc[e] + w[i] * static_cast<float>(x_host[i][e0 + e]);
    for (int64_t e = 0; e < k; ++e) out[e0 + e] = host_trunc_i64(acc[e]);
  });
  g_err.clear();
  return TAL_OK;
}

int32_t tal_host_agg_bf16(const uint16_t* const* x_host, const double* w_host, int32_t m, uint16_t* out, int64_t n,
                          int32_t mode) {
  if (int32_t rc = host_args("tal_host_agg_bf16", reinterpret_cast<const void* const*>(x_host), w_host, m, out, n))
    return rc;
  std::vector<float> w(static_cast<size_t>(m));
  for (int i = 0; i < m; ++i) w[i] = static_cast<float>(w_host[i]);
  const bool exact = mode == TAL_MODE_EXACT;
  host_blocks(n, [&](int64_t e0, int64_t e1) {
    float acc[kHostBlock];
    const int64_t k = e1 - e0;
    for (int64_t e = 0; e < k; ++e) {
      const float p = w[0] * host_bf16(x_host[0][e0 + e]);
      acc[e] = exact ? host_round_bf16(p) : p;
    }
    for (int i = 1; i < m; ++i) {
      const float wi = w[i];
      const uint16_t* xi = x_host[i] + e0;
      if (exact)
        for (int64_t e = 0; e < k; ++e) acc[e] = host_round_bf16(acc[e] + host_round_bf16(wi * host_bf16(xi[e])));
      else
        for (int64_t e = 0; e < k; ++e) acc[e] = std::fma(wi, host_bf16(xi[e]), acc[e]);
    }
    for (int64_t e = 0; e < k; ++e) out[e0 + e] = host_store_bf16(acc[e]);
  });
  g_err.clear();
  return TAL_OK;
}

int32_t tal_host_cosine(const float* const* a_host, const float* const* b_host, int32_t n_pairs,
                        const int64_t* plan_host, float* out) {
  if (!a_host || !b_host || !plan_host || !out || n_pairs <= 0 || plan_host[0] <= 0 || plan_host[1] <= 0 ||
      plan_host[2] < 1 || plan_host[2] > kCosMaxThreads)
    return fail(TAL_ERR_INVALID, "tal_host_cosine: bad arguments");
  for (int j = 0; j < n_pairs; ++j)
    if (!a_host[j] || !b_host[j]) return fail(TAL_ERR_INVALID, "tal_host_cosine: null model pointer");
  const int64_t n_seg = plan_host[0], n_out = plan_host[1];
  int64_t n_chunks = 0;  // chunk words follow the segment words; count them from the segments
  for (int64_t t = 0; t < n_seg; ++t) {
    const int64_t* sg = plan_host + kCosHdr + kCosSegWords * t;
    n_chunks += (sg[1] * sg[3] + sg[6] - 1) / sg[6];
  }
  std::vector<float> s_all(static_cast<size_t>(n_out));
  std::vector<float> means(static_cast<size_t>(n_seg));
  for (int j = 0; j < n_pairs; ++j) {
    // outputs chunk by chunk, then the means tensor by tensor, each on up to 16 host threads
    host_blocks(n_chunks * kHostBlock, [&](int64_t e0, int64_t) {
      HostCos::outputs(plan_host, e0 / kHostBlock, a_host[j], b_host[j], s_all.data());
    });
    host_blocks(n_seg * kHostBlock, [&](int64_t e0, int64_t) {
      means[static_cast<size_t>(e0 / kHostBlock)] = HostCos::mean(plan_host, e0 / kHostBlock, s_all.data());
    });
    float avg = 0.f + means[0];  // 0 + mean_0, += mean_t in parameter order, / len(params)
    for (int64_t t = 1; t < n_seg; ++t) avg = avg + means[static_cast<size_t>(t)];
    out[j] = avg / static_cast<float>(n_seg);
  }
  g_err.clear();
  return TAL_OK;
}

}  // extern "C"
