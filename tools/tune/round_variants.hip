// Tuning harness for the K3 round kernel (not part of the product).  Builds the same tile plan
// as the library (linked: tal_round_plan_build) and times kernel variants on the BASELINE
// config-3 shape (64 ResNet-50 f32 segments, random 8-regular graph), checking every variant
// bit for bit against the library's tal_agg_round_f32.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <random>
#include "../../include/tal_agg.h"

#pragma clang fp contract(off)
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

struct PlanView { const int* grp_row_ptr; const int* grp_src_ptr; const int* src_row; const int* row_ptr; const int* op_slot; const float* op_w; const int* out_row; };

__device__ __forceinline__ float4 f4mul(float w, float4 x) { return make_float4(__fmul_rn(w,x.x), __fmul_rn(w,x.y), __fmul_rn(w,x.z), __fmul_rn(w,x.w)); }
__device__ __forceinline__ float4 f4add(float4 a, float w, float4 x) { return make_float4(__fadd_rn(a.x,__fmul_rn(w,x.x)), __fadd_rn(a.y,__fmul_rn(w,x.y)), __fadd_rn(a.z,__fmul_rn(w,x.z)), __fadd_rn(a.w,__fmul_rn(w,x.w))); }

// V2: plan + src rows staged to LDS first; data staged with UNR independent loads per batch.
template <int C4, int NT, int UNR, bool NT_LOAD, bool NT_STORE = NT_LOAD>
__global__ __launch_bounds__(NT) void k_v2(const float* __restrict__ pin, long ld_in4, float* __restrict__ pout, long ld_out4, long n4, PlanView p, int max_src) {
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const long c0 = (long)blockIdx.x * C4;
  const int s_beg = p.grp_src_ptr[g], ns = p.grp_src_ptr[g+1] - s_beg;
  const int r_beg = p.grp_row_ptr[g], nr = p.grp_row_ptr[g+1] - r_beg;
  const int o_beg = p.row_ptr[r_beg], no = p.row_ptr[r_beg+nr] - o_beg;
  int* s_rowptr = (int*)(s_data + (size_t)max_src * C4);
  int* s_slot = s_rowptr + (nr + 1);
  float* s_w = (float*)(s_slot + no);
  int* s_src = (int*)(s_w + no);
  int* s_out = s_src + ns;
  for (int k = threadIdx.x; k <= nr; k += NT) s_rowptr[k] = p.row_ptr[r_beg + k] - o_beg;
  for (int k = threadIdx.x; k < no; k += NT) { s_slot[k] = p.op_slot[o_beg + k] * C4; s_w[k] = p.op_w[o_beg + k]; }
  for (int k = threadIdx.x; k < ns; k += NT) s_src[k] = p.src_row[s_beg + k];
  for (int k = threadIdx.x; k < nr; k += NT) s_out[k] = p.out_row[r_beg + k];
  __syncthreads();
  const long cols = min((long)C4, n4 - c0);
  const int total = ns * C4;
  for (int k0 = 0; k0 < total; k0 += NT * UNR) {
    float4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int k = k0 + u * NT + threadIdx.x;
      const int s = k / C4, c = k % C4;
      v[u] = make_float4(0,0,0,0);
      if (k < total && c < cols) {
        const float4* src = reinterpret_cast<const float4*>(pin) + (long)s_src[s] * ld_in4 + c0 + c;
        if (NT_LOAD) { v4f t = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(src)); v[u] = make_float4(t.x, t.y, t.z, t.w); } else v[u] = *src;
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) { const int k = k0 + u * NT + threadIdx.x; if (k < total) s_data[k] = v[u]; }
  }
  __syncthreads();
  constexpr int RPP = NT / C4;
  const int c = threadIdx.x % C4, rsub = threadIdx.x / C4;
  if (c >= cols) return;
  for (int r = rsub; r < nr; r += RPP) {
    const int q0 = s_rowptr[r], q1 = s_rowptr[r+1];
    float4 acc = f4mul(s_w[q0], s_data[s_slot[q0] + c]);
    for (int q = q0 + 1; q < q1; ++q) acc = f4add(acc, s_w[q], s_data[s_slot[q] + c]);
    float4* dst = reinterpret_cast<float4*>(pout) + (long)s_out[r] * ld_out4 + c0 + c;
    if (NT_STORE) { v4f t = {acc.x, acc.y, acc.z, acc.w}; __builtin_nontemporal_store(t, reinterpret_cast<v4f*>(dst)); } else *dst = acc;
  }
}

// V4: persistent, register-prefetch of the next tile while computing the current one.
template <int C4, int NT, int J, bool NTL = false, bool NTS = false>   // J = float4 loads per thread per tile
__global__ __launch_bounds__(NT) void k_v4(const float* __restrict__ pin, long ld_in4, float* __restrict__ pout, long ld_out4, long n4, PlanView p, int max_src, long n_tiles) {
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const int s_beg = p.grp_src_ptr[g], ns = p.grp_src_ptr[g+1] - s_beg;
  const int r_beg = p.grp_row_ptr[g], nr = p.grp_row_ptr[g+1] - r_beg;
  const int o_beg = p.row_ptr[r_beg], no = p.row_ptr[r_beg+nr] - o_beg;
  int* s_rowptr = (int*)(s_data + (size_t)max_src * C4);
  int* s_slot = s_rowptr + (nr + 1);
  float* s_w = (float*)(s_slot + no);
  int* s_out = (int*)(s_w + no);
  for (int k = threadIdx.x; k <= nr; k += NT) s_rowptr[k] = p.row_ptr[r_beg + k] - o_beg;
  for (int k = threadIdx.x; k < no; k += NT) { s_slot[k] = p.op_slot[o_beg + k] * C4; s_w[k] = p.op_w[o_beg + k]; }
  for (int k = threadIdx.x; k < nr; k += NT) s_out[k] = p.out_row[r_beg + k];
  // per-thread source base pointers for its J staging slots (fixed across tiles)
  const float4* base[J];
  bool live[J];
  int slotk[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int k = j * NT + threadIdx.x;
    const int s = k / C4, c = k % C4;
    live[j] = s < ns;
    slotk[j] = k;
    base[j] = reinterpret_cast<const float4*>(pin) + (live[j] ? (long)p.src_row[s_beg + s] * ld_in4 : 0) + c;
  }
  const int c = threadIdx.x % C4, rsub = threadIdx.x / C4;
  constexpr int RPP = NT / C4;
  long t = blockIdx.x;
  float4 v[J];
  auto load_tile = [&](long tt) {
    const long c0 = tt * C4;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      v[j] = make_float4(0,0,0,0);
      if (live[j] && c0 + (slotk[j] % C4) < n4) { if (NTL) { v4f q = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base[j] + c0)); v[j] = make_float4(q.x, q.y, q.z, q.w); } else v[j] = base[j][c0]; }
    }
  };
  if (t < n_tiles) load_tile(t);
  for (; t < n_tiles; t += gridDim.x) {
    __syncthreads();  // previous tile's compute done reading LDS
#pragma unroll
    for (int j = 0; j < J; ++j) if (live[j]) s_data[slotk[j]] = v[j];
    __syncthreads();
    const long tn = t + gridDim.x;
    if (tn < n_tiles) load_tile(tn);     // next tile's loads fly during this tile's math
    const long c0 = t * C4;
    if (c0 + c < n4) {
      for (int r = rsub; r < nr; r += RPP) {
        const int q0 = s_rowptr[r], q1 = s_rowptr[r+1];
        float4 acc = f4mul(s_w[q0], s_data[s_slot[q0] + c]);
        for (int q = q0 + 1; q < q1; ++q) acc = f4add(acc, s_w[q], s_data[s_slot[q] + c]);
        float4* dst = reinterpret_cast<float4*>(pout) + (long)s_out[r] * ld_out4 + c0 + c;
        if (NTS) { v4f q = {acc.x, acc.y, acc.z, acc.w}; __builtin_nontemporal_store(q, reinterpret_cast<v4f*>(dst)); } else *dst = acc;
      }
    }
  }
}

template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void k_copy(const float* __restrict__ src, float* __restrict__ dst, long n4) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i0 = (long)blockIdx.x * 256 * U + threadIdx.x; i0 < n4; i0 += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * 256; if (i < n4) { const v4f* p = reinterpret_cast<const v4f*>(src) + i; v[u] = NTL ? __builtin_nontemporal_load(p) : *p; } }
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * 256; if (i < n4) { v4f* p = reinterpret_cast<v4f*>(dst) + i; if (NTS) __builtin_nontemporal_store(v[u], p); else *p = v[u]; } }
  }
}

typedef __attribute__((address_space(4))) const int* CI32;
typedef __attribute__((address_space(4))) const float* CF32;

// v5: wave-uniform rows, plan via scalar loads, operand batches of B
template <int C4, int NT, int J, int B>
__global__ __launch_bounds__(NT) void k_v5(const float* __restrict__ pin, long ld_in4, float* __restrict__ pout, long ld_out4, long n4, PlanView p, long n_tiles) {
  extern __shared__ float4 s_data[];
  const int g = blockIdx.y;
  const int s_beg = p.grp_src_ptr[g], ns = p.grp_src_ptr[g+1] - s_beg;
  const int r_beg = p.grp_row_ptr[g], nr = p.grp_row_ptr[g+1] - r_beg;
  const float* base[J]; int slotk[J]; bool live[J];
#pragma unroll
  for (int j = 0; j < J; ++j) { const int k = j * NT + threadIdx.x; const int s = k / C4; live[j] = s < ns; slotk[j] = k;
    base[j] = pin + 4 * ((live[j] ? (long)p.src_row[s_beg + s] * ld_in4 : 0) + (k % C4)); }
  float4 v[J];
  auto load_tile = [&](long tt) { const long c0 = tt * C4;
#pragma unroll
    for (int j = 0; j < J; ++j) if (live[j] && c0 + (slotk[j] % C4) < n4) { v4f q = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(base[j]) + c0); v[j] = make_float4(q.x,q.y,q.z,q.w); } };
  const CI32 row_ptr = (CI32)p.row_ptr; const CI32 out_row = (CI32)p.out_row; const CI32 op_slot = (CI32)p.op_slot; const CF32 op_w = (CF32)p.op_w;
  constexpr int kW = NT / 64; constexpr int kCpl = C4 / 64;
  const int lane = threadIdx.x & 63; const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  long t = blockIdx.x;
  if (t < n_tiles) load_tile(t);
  for (; t < n_tiles; t += gridDim.x) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) if (live[j]) s_data[slotk[j]] = v[j];
    __syncthreads();
    if (t + gridDim.x < n_tiles) load_tile(t + gridDim.x);
    const long c0 = t * C4;
    for (int r = wave; r < nr; r += kW) {
      const int gr = r_beg + r; const int q0 = row_ptr[gr], q1 = row_ptr[gr + 1]; const long orow = out_row[gr];
      float4 acc[kCpl];
      { const float w = op_w[q0]; const int sl = op_slot[q0] * C4 + lane;
#pragma unroll
        for (int j = 0; j < kCpl; ++j) acc[j] = f4mul(w, s_data[sl + 64 * j]); }
      int q = q0 + 1;
      for (; q + B <= q1; q += B) {
        float w[B]; int sl[B]; float4 x[B][kCpl];
#pragma unroll
        for (int u = 0; u < B; ++u) { w[u] = op_w[q + u]; sl[u] = op_slot[q + u] * C4 + lane; }
#pragma unroll
        for (int u = 0; u < B; ++u)
#pragma unroll
          for (int j = 0; j < kCpl; ++j) x[u][j] = s_data[sl[u] + 64 * j];
#pragma unroll
        for (int u = 0; u < B; ++u)
#pragma unroll
          for (int j = 0; j < kCpl; ++j) acc[j] = f4add(acc[j], w[u], x[u][j]);
      }
      for (; q < q1; ++q) { const float w = op_w[q]; const int sl = op_slot[q] * C4 + lane;
#pragma unroll
        for (int j = 0; j < kCpl; ++j) acc[j] = f4add(acc[j], w, s_data[sl + 64 * j]); }
#pragma unroll
      for (int j = 0; j < kCpl; ++j) { const long col = c0 + lane + 64 * j; if (col < n4) { v4f q2 = {acc[j].x, acc[j].y, acc[j].z, acc[j].w}; __builtin_nontemporal_store(q2, reinterpret_cast<v4f*>(pout) + orow * ld_out4 + col); } }
    }
  }
}

static PlanView view(const int* plan, const tal_round_plan_info& in) {
  PlanView v; v.grp_row_ptr = plan + in.off_grp_row_ptr; v.grp_src_ptr = plan + in.off_grp_src_ptr; v.src_row = plan + in.off_src_row;
  v.row_ptr = plan + in.off_row_ptr; v.op_slot = plan + in.off_op_slot; v.op_w = (const float*)(plan + in.off_op_w); v.out_row = plan + in.off_out_row; return v;
}

int main(int argc, char** argv) {
  const int rows = 64, deg = 8;
  const long n = argc > 1 ? atol(argv[1]) : 23573962L;
  const long ld = (n + 63) / 64 * 64;
  // random 8-regular-ish graph: ring offsets +-1..+-4 scrambled by a fixed permutation
  std::vector<int> perm(rows); for (int i = 0; i < rows; ++i) perm[i] = i;
  std::mt19937 rng(0); std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<int> inv(rows); for (int i = 0; i < rows; ++i) inv[perm[i]] = i;
  std::vector<int> row_ptr{0}, col, out_row; std::vector<double> w;
  const bool barbell = argc > 2 && strcmp(argv[2], "barbell") == 0;
  const int nrows = barbell ? 128 : rows;
  std::vector<std::vector<int>> adj(nrows);
  if (barbell) {
    auto edge = [&](int a, int b) { adj[a].push_back(b); adj[b].push_back(a); };
    for (int a = 0; a < 60; ++a) for (int b = a + 1; b < 60; ++b) { edge(a, b); edge(68 + a, 68 + b); }
    for (int a = 59; a < 68; ++a) edge(a, a + 1);
  } else {
    for (int r = 0; r < rows; ++r) { int pr = inv[r]; for (int d = 1; d <= deg / 2; ++d) { adj[r].push_back(perm[(pr + d) % rows]); adj[r].push_back(perm[(pr - d + rows) % rows]); } }
  }
  for (int r = 0; r < nrows; ++r) {
    std::vector<int> nb = adj[r];
    std::sort(nb.begin(), nb.end()); nb.push_back(r);
    for (int x : nb) { col.push_back(x); w.push_back(1.0 / nb.size()); }
    row_ptr.push_back(col.size()); out_row.push_back(r);
  }
  float *pin, *pref, *pout;
  const int rows_alloc = nrows;
  CK(hipMalloc(&pin, rows_alloc * ld * 4)); CK(hipMalloc(&pref, rows_alloc * ld * 4)); CK(hipMalloc(&pout, rows_alloc * ld * 4));
  { std::vector<float> h(ld); for (int r = 0; r < rows_alloc; ++r) { for (long i = 0; i < ld; ++i) h[i] = (float)((r * 131 + i * 7) % 1013) * 0.001f - 0.5f; CK(hipMemcpy(pin + r * ld, h.data(), ld * 4, hipMemcpyHostToDevice)); } }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const long n4 = n / 4;
  double bytes = 4.0 * n * (rows + rows);
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20; float best = 1e9, sum = 0;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); sum += ms; }
    CK(hipGetLastError());
    // verify
    std::vector<float> a(n), b(n); bool ok = true;
    for (int r = 0; r < nrows && ok; r += 13) { CK(hipMemcpy(a.data(), pref + r * ld, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), pout + r * ld, n * 4, hipMemcpyDeviceToHost)); ok = memcmp(a.data(), b.data(), (n / 4 * 4) * 4) == 0; }
    printf("%-34s avg %.3f ms  best %.3f ms  %.0f GB/s (avg)  %s\n", name, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9, ok ? "OK" : "MISMATCH");
    CK(hipMemset(pout, 0, (size_t)nrows * ld * 4));
  };
  for (int c4 : {64, 128}) for (int lds : {80 * 1024, 160 * 1024}) {
    std::vector<int> plan(tal_round_plan_words(nrows, col.size())); tal_round_plan_info info;
    if (tal_round_plan_build(nrows, row_ptr.data(), col.data(), w.data(), out_row.data(), c4, lds, 0, plan.data(), plan.size(), &info)) { printf("plan c4=%d lds=%d: %s\n", c4, lds, tal_last_error()); continue; }
    int* dplan; CK(hipMalloc(&dplan, info.words * 4)); CK(hipMemcpy(dplan, plan.data(), info.words * 4, hipMemcpyHostToDevice));
    bytes = 4.0 * n * (info.total_src + nrows);
    printf("== c4=%d lds_budget=%d groups=%d staged=%d max_src=%d\n", c4, lds, info.n_groups, info.total_src, info.max_src);
    CK(tal_agg_round_f32(pin, ld, pref, ld, n, dplan, &info, 1, 0) ? hipErrorUnknown : hipSuccess);
    char nm[128];
    snprintf(nm, sizeof nm, "lib c4=%d", c4);
    timeit(nm, [&]{ tal_agg_round_f32(pin, ld, pout, ld, n, dplan, &info, 1, 0); });
    PlanView v = view(dplan, info);
    const long tiles = (n4 + c4 - 1) / c4;
    const size_t ldsz = (size_t)info.max_src * c4 * 16;
#define V5(C, NTH, JJ, BB, BPC) if (c4 == C && info.max_src * C <= JJ * NTH && ldsz * BPC <= 160 * 1024) { auto k = k_v5<C, NTH, JJ, BB>; CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160*1024)); \
      const dim3 g5(std::max<long>(1, std::min<long>(tiles, 256L * BPC / info.n_groups)), info.n_groups); snprintf(nm, sizeof nm, "v5 c4=%d nt=%d J=%d B=%d bpc=%d", C, NTH, JJ, BB, BPC); timeit(nm, [&]{ k<<<g5, NTH, ldsz>>>(pin, ld/4, pout, ld/4, n4, v, tiles); }); }
    const size_t lds2 = info.lds_bytes + 4 * (info.max_src + info.max_rows) + 64;
#define V4(C, NTH, JJ, BPC, NTL, NTS) if (c4 == C && info.max_src * C <= JJ * NTH && lds2 * BPC <= 160 * 1024) { auto k = k_v4<C, NTH, JJ, NTL, NTS>; CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160*1024)); \
      const dim3 g4(std::max<long>(1, std::min<long>(tiles, 256L * BPC / info.n_groups)), info.n_groups); snprintf(nm, sizeof nm, "v4(old emit) c4=%d nt=%d J=%d bpc=%d", C, NTH, JJ, BPC); timeit(nm, [&]{ k<<<g4, NTH, lds2>>>(pin, ld/4, pout, ld/4, n4, v, info.max_src, tiles); }); }
    V4(64, 512, 8, 2, true, true) V4(64, 1024, 4, 1, true, true) V4(128, 1024, 8, 1, true, true)
    V5(64, 512, 8, 4, 2) V5(64, 1024, 4, 4, 2) V5(64, 1024, 4, 8, 2) V5(64, 1024, 8, 8, 1) V5(64, 512, 16, 8, 1)
    V5(128, 1024, 8, 4, 1) V5(128, 1024, 8, 8, 1) V5(128, 512, 16, 8, 1)
    CK(hipFree(dplan));
  }
  return 0;
}
