// Bandwidth probe (not part of the product): what the config-3 round's access pattern can reach
// on this board.  Flat copies, read-only and write-only streams, and the round kernel's own
// tile walk (64 rows x C4 float4 per tile, persistent grid, register prefetch) as a pure copy,
// each over the same 6 GB in / 6 GB out the round moves; plus the library's round kernel.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include <random>
#include "../../include/tal_agg.h"

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

template <bool NTL>
__device__ __forceinline__ v4f ld(const v4f* p) { if constexpr (NTL) return __builtin_nontemporal_load(p); else return *p; }
template <bool NTS>
__device__ __forceinline__ void st(v4f* p, v4f v) { if constexpr (NTS) __builtin_nontemporal_store(v, p); else *p = v; }

template <int NT, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_copy(const v4f* __restrict__ src, v4f* __restrict__ dst, long n4) {
  const long stride = (long)gridDim.x * NT * U;
  for (long i0 = (long)blockIdx.x * NT * U + threadIdx.x; i0 < n4; i0 += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * NT; if (i < n4) v[u] = ld<NTL>(src + i); }
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * NT; if (i < n4) st<NTS>(dst + i, v[u]); }
  }
}

template <int NT, int U, bool NTL>
__global__ __launch_bounds__(NT) void k_read(const v4f* __restrict__ src, float* __restrict__ sink, long n4) {
  const long stride = (long)gridDim.x * NT * U;
  v4f a = {0, 0, 0, 0};
  for (long i0 = (long)blockIdx.x * NT * U + threadIdx.x; i0 < n4; i0 += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * NT; v[u] = i < n4 ? ld<NTL>(src + i) : a; }
#pragma unroll
    for (int u = 0; u < U; ++u) a += v[u];
  }
  if (a.x + a.y + a.z + a.w == 123.456f) sink[threadIdx.x] = a.x;
}

template <int NT, int U, bool NTS>
__global__ __launch_bounds__(NT) void k_write(v4f* __restrict__ dst, long n4) {
  const long stride = (long)gridDim.x * NT * U;
  const v4f v = {1.f, 2.f, 3.f, 4.f};
  for (long i0 = (long)blockIdx.x * NT * U + threadIdx.x; i0 < n4; i0 += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) { long i = i0 + u * NT; if (i < n4) st<NTS>(dst + i, v); }
  }
}

// the round's tile walk as a copy: tile t = columns [t*C4, t*C4+C4) of all R rows; lane slot
// k = j*NT + tid is (row k / C4, column k % C4); next tile's loads in flight in registers
template <int C4, int NT, int J, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_tilecopy(const v4f* __restrict__ pin, v4f* __restrict__ pout, long ld4, long n4, int R, long n_tiles) {
  const int c = threadIdx.x % C4;
  int row[J];
#pragma unroll
  for (int j = 0; j < J; ++j) { int r = (j * NT + threadIdx.x) / C4; row[j] = r < R ? r : -1; }
  v4f v[J];
  long t = blockIdx.x;
  auto load = [&](long tt) { long col = tt * C4 + c; if (col < n4) {
#pragma unroll
      for (int j = 0; j < J; ++j) if (row[j] >= 0) v[j] = ld<NTL>(pin + row[j] * ld4 + col); } };
  if (t < n_tiles) load(t);
  for (; t < n_tiles; t += gridDim.x) {
    v4f w[J];
#pragma unroll
    for (int j = 0; j < J; ++j) w[j] = v[j];
    if (t + gridDim.x < n_tiles) load(t + gridDim.x);
    long col = t * C4 + c;
    if (col < n4) {
#pragma unroll
      for (int j = 0; j < J; ++j) if (row[j] >= 0) st<NTS>(pout + row[j] * ld4 + col, w[j]);
    }
  }
}

__global__ void k_fill(v4f* p, long n4, unsigned seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed; v4f v;
    for (int k = 0; k < 4; ++k) { h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; v[k] = (float)(int)(h & 0xffffff) * (1.f / 8388608.f) - 1.f; }
    p[i] = v;
  }
}

// one tile per workgroup (no persistence): the hardware dispatcher refills CUs
template <int C4, int NT, int J, bool NTL, bool NTS>
__global__ __launch_bounds__(NT) void k_tilecopy1(const v4f* __restrict__ pin, v4f* __restrict__ pout, long ld4, long n4, int R) {
  const int c = threadIdx.x % C4;
  const long col = (long)blockIdx.x * C4 + c;
  if (col >= n4) return;
  v4f v[J];
#pragma unroll
  for (int j = 0; j < J; ++j) { int r = (j * NT + threadIdx.x) / C4; if (r < R) v[j] = ld<NTL>(pin + r * ld4 + col); }
#pragma unroll
  for (int j = 0; j < J; ++j) { int r = (j * NT + threadIdx.x) / C4; if (r < R) st<NTS>(pout + r * ld4 + col, v[j]); }
}

static int ld_sweep(int argc, char** argv);
static int rows_sweep(int argc, char** argv);

int main(int argc, char** argv) {
  if (argc > 1 && strcmp(argv[1], "ld") == 0) return ld_sweep(argc, argv);
  if (argc > 1 && strcmp(argv[1], "rows") == 0) return rows_sweep(argc, argv);
  const int R = 64, deg = 8;
  const long n = 23573962L, ld = (n + 63) / 64 * 64, n4 = n / 4, ld4 = ld / 4;
  v4f *pin, *pout; float* sink;
  CK(hipMalloc(&pin, (size_t)R * ld * 4)); CK(hipMalloc(&pout, (size_t)R * ld * 4)); CK(hipMalloc(&sink, 4096));
  const bool zero = argc > 1 && strcmp(argv[1], "zero") == 0;
  if (zero) CK(hipMemset(pin, 0, (size_t)R * ld * 4)); else k_fill<<<4096, 256>>>(pin, (long)R * ld / 4, 12345u);
  CK(hipMemset(pout, 0, (size_t)R * ld * 4)); CK(hipDeviceSynchronize());
  printf("data: %s\n", zero ? "zeros" : "random");
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const long total4 = (long)R * ld4;
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize()); CK(hipGetLastError());
    const int reps = 15; float best = 1e9, sum = 0;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); sum += ms; }
    CK(hipGetLastError());
    printf("%-44s avg %.3f ms  best %.3f ms  %6.0f GB/s avg  %6.0f GB/s best\n", name, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  const double cbytes = 2.0 * 16 * total4;
  char nm[128];
#define COPY(NT_, U_, NTL_, NTS_, BPC) { snprintf(nm, sizeof nm, "copy nt=%d U=%d ntl=%d nts=%d wg/cu=%d", NT_, U_, NTL_, NTS_, BPC); \
    const int g = ncu * BPC; timeit(nm, cbytes, [&]{ k_copy<NT_, U_, NTL_, NTS_><<<g, NT_>>>(pin, pout, total4); }); }
  COPY(256, 1, true, true, 8) COPY(256, 2, true, true, 8) COPY(256, 4, true, true, 8) COPY(256, 8, true, true, 8)
  COPY(256, 4, false, false, 8) COPY(256, 4, true, false, 8) COPY(256, 4, false, true, 8)
  COPY(256, 4, true, true, 16) COPY(512, 4, true, true, 4) COPY(1024, 4, true, true, 2) COPY(1024, 2, true, true, 2)
  COPY(256, 2, true, true, 32) COPY(256, 4, true, true, 4)
  // flat copy, one grid-stride pass per element (huge grid)
  { snprintf(nm, sizeof nm, "copy nt=256 U=1 full grid"); const long g = (total4 + 255) / 256; timeit(nm, cbytes, [&]{ k_copy<256, 1, true, true><<<g, 256>>>(pin, pout, total4); }); }
  { snprintf(nm, sizeof nm, "copy nt=512 U=1 full grid"); const long g = (total4 + 511) / 512; timeit(nm, cbytes, [&]{ k_copy<512, 1, true, true><<<g, 512>>>(pin, pout, total4); }); }
  { snprintf(nm, sizeof nm, "copy nt=1024 U=1 full grid"); const long g = (total4 + 1023) / 1024; timeit(nm, cbytes, [&]{ k_copy<1024, 1, true, true><<<g, 1024>>>(pin, pout, total4); }); }
  { snprintf(nm, sizeof nm, "copy nt=256 U=2 full grid"); const long g = (total4 + 511) / 512; timeit(nm, cbytes, [&]{ k_copy<256, 2, true, true><<<g, 256>>>(pin, pout, total4); }); }
  { snprintf(nm, sizeof nm, "copy nt=256 U=4 full grid"); const long g = (total4 + 1023) / 1024; timeit(nm, cbytes, [&]{ k_copy<256, 4, true, true><<<g, 256>>>(pin, pout, total4); }); }
#define READ(NT_, U_, NTL_, BPC) { snprintf(nm, sizeof nm, "read nt=%d U=%d ntl=%d wg/cu=%d", NT_, U_, NTL_, BPC); \
    const int g = ncu * BPC; timeit(nm, cbytes / 2, [&]{ k_read<NT_, U_, NTL_><<<g, NT_>>>(pin, sink, total4); }); }
  READ(256, 4, true, 8) READ(256, 8, true, 8) READ(256, 4, false, 8) READ(1024, 4, true, 2)
#define WRITE(NT_, U_, NTS_, BPC) { snprintf(nm, sizeof nm, "write nt=%d U=%d nts=%d wg/cu=%d", NT_, U_, NTS_, BPC); \
    const int g = ncu * BPC; timeit(nm, cbytes / 2, [&]{ k_write<NT_, U_, NTS_><<<g, NT_>>>(pout, total4); }); }
  WRITE(256, 4, true, 8) WRITE(256, 4, false, 8) WRITE(1024, 4, true, 2)
#define TILE(C4_, NT_, J_, NTL_, NTS_, BPC) { snprintf(nm, sizeof nm, "tilecopy c4=%d nt=%d J=%d ntl=%d nts=%d wg/cu=%d", C4_, NT_, J_, NTL_, NTS_, BPC); \
    const long tiles = (n4 + C4_ - 1) / C4_; const long g = std::min<long>(tiles, (long)ncu * BPC); \
    timeit(nm, 2.0 * 16 * n4 * R, [&]{ k_tilecopy<C4_, NT_, J_, NTL_, NTS_><<<g, NT_>>>(pin, pout, ld4, n4, R, tiles); }); }
  TILE(64, 1024, 4, true, true, 2) TILE(64, 512, 8, true, true, 2) TILE(64, 512, 8, true, true, 4) TILE(64, 1024, 4, true, true, 4)
  TILE(64, 1024, 4, false, false, 2) TILE(64, 1024, 4, true, false, 2) TILE(128, 1024, 8, true, true, 2) TILE(32, 1024, 2, true, true, 2)
  TILE(32, 512, 4, true, true, 4) TILE(64, 256, 16, true, true, 8)
#define TILE1(C4_, NT_, J_) { snprintf(nm, sizeof nm, "tilecopy1 (tile per WG) c4=%d nt=%d J=%d", C4_, NT_, J_); \
    const long tiles = (n4 + C4_ - 1) / C4_; \
    timeit(nm, 2.0 * 16 * n4 * R, [&]{ k_tilecopy1<C4_, NT_, J_, true, true><<<tiles, NT_>>>(pin, pout, ld4, n4, R); }); }
  TILE1(64, 1024, 4) TILE1(64, 512, 8) TILE1(64, 256, 16) TILE1(32, 1024, 2) TILE1(16, 1024, 1) TILE1(128, 1024, 8)

  // the library's round kernel on a random 8-regular graph
  std::vector<int> perm(R); for (int i = 0; i < R; ++i) perm[i] = i;
  std::mt19937 rng(0); std::shuffle(perm.begin(), perm.end(), rng);
  std::vector<int> inv(R); for (int i = 0; i < R; ++i) inv[perm[i]] = i;
  std::vector<int> row_ptr{0}, col, out_row; std::vector<double> w;
  for (int r = 0; r < R; ++r) {
    std::vector<int> nb; int pr = inv[r];
    for (int d = 1; d <= deg / 2; ++d) { nb.push_back(perm[(pr + d) % R]); nb.push_back(perm[(pr - d + R) % R]); }
    std::sort(nb.begin(), nb.end()); nb.push_back(r);
    for (int x : nb) { col.push_back(x); w.push_back(1.0 / nb.size()); }
    row_ptr.push_back(col.size()); out_row.push_back(r);
  }
  std::vector<int> plan(tal_round_plan_words(R, col.size())); tal_round_plan_info info;
  if (tal_round_plan_build(R, row_ptr.data(), col.data(), w.data(), out_row.data(), 64, 160 * 1024, 0, plan.data(), plan.size(), &info)) { printf("plan: %s\n", tal_last_error()); return 1; }
  int* dplan; CK(hipMalloc(&dplan, info.words * 4)); CK(hipMemcpy(dplan, plan.data(), info.words * 4, hipMemcpyHostToDevice));
  timeit("library round (K3) c4=64", 4.0 * n * (info.total_src + R), [&]{ tal_agg_round_f32((const float*)pin, ld, (float*)pout, ld, n, dplan, &info, 1, 0); });
  return 0;
}

// row-stride sweep: the same tile walk with rows padded to different alignments
static int ld_sweep(int argc, char** argv) {
  const int R = 64;
  const long n = 23573962L, n4 = n / 4;
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const long pads[] = {64, 256, 1024, 4096, 16384, 524288, 524288 + 1024, 524288 + 64, 524288 + 4096};
  v4f *pin, *pout;
  const long maxld = (n + 524288 + 4096) / 64 * 64 + 524288 + 4096;
  CK(hipMalloc(&pin, (size_t)R * maxld * 4)); CK(hipMalloc(&pout, (size_t)R * maxld * 4));
  k_fill<<<4096, 256>>>(pin, (long)R * maxld / 4, 12345u); CK(hipDeviceSynchronize());
  char nm[160];
  for (long pad : pads) {
    long ld;
    if (pad > 524288) { ld = (n + 524287) / 524288 * 524288 + (pad - 524288); }
    else ld = (n + pad - 1) / pad * pad;
    const long ld4 = ld / 4;
    auto timeit = [&](const char* name, double bytes, auto launch) {
      for (int i = 0; i < 3; ++i) launch();
      CK(hipDeviceSynchronize()); CK(hipGetLastError());
      const int reps = 15; float sum = 0;
      for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; }
      printf("ld=%9ld (%6ld B mod 64K)  %-40s avg %.3f ms  %6.0f GB/s\n", ld, (ld * 4) % 65536, name, sum / reps, bytes / (sum / reps * 1e-3) / 1e9);
      fflush(stdout);
    };
    const long tiles = (n4 + 63) / 64;
    timeit("tilecopy persistent c4=64 nt=1024 bpc2", 2.0 * 16 * n4 * R, [&]{ k_tilecopy<64, 1024, 4, true, true><<<std::min<long>(tiles, ncu * 2), 1024>>>(pin, pout, ld4, n4, R, tiles); });
    timeit("tilecopy1 c4=64 nt=1024", 2.0 * 16 * n4 * R, [&]{ k_tilecopy1<64, 1024, 4, true, true><<<tiles, 1024>>>(pin, pout, ld4, n4, R); });
    const long tiles2 = (n4 + 127) / 128;
    timeit("tilecopy persistent c4=128 nt=1024 bpc2", 2.0 * 16 * n4 * R, [&]{ k_tilecopy<128, 1024, 8, true, true><<<std::min<long>(tiles2, ncu * 2), 1024>>>(pin, pout, ld4, n4, R, tiles2); });
  }
  return 0;
}

// many rows, small pieces: the tile walk over R rows at C4 float4 per row per tile
static int rows_sweep(int argc, char** argv) {
  const long n = 23573962L, ld = (n + 63) / 64 * 64, n4 = n / 4, ld4 = ld / 4;
  const int RMAX = 256;
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  v4f *pin, *pout;
  CK(hipMalloc(&pin, (size_t)RMAX * ld * 4)); CK(hipMalloc(&pout, (size_t)RMAX * ld * 4));
  k_fill<<<4096, 256>>>(pin, (long)RMAX * ld / 4, 12345u); CK(hipDeviceSynchronize());
  auto timeit = [&](const char* name, int R, double bytes, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize()); CK(hipGetLastError());
    const int reps = 8; float sum = 0;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; }
    printf("R=%3d %-44s avg %.3f ms  %6.0f GB/s\n", R, name, sum / reps, bytes / (sum / reps * 1e-3) / 1e9);
    fflush(stdout);
  };
#define TR(R_, C4_, NT_, J_, BPC) { const long tiles = (n4 + C4_ - 1) / C4_; char nm[96]; snprintf(nm, sizeof nm, "tilecopy c4=%d nt=%d J=%d wg/cu=%d", C4_, NT_, J_, BPC); \
    timeit(nm, R_, 2.0 * 16 * n4 * R_, [&]{ k_tilecopy<C4_, NT_, J_, true, true><<<std::min<long>(tiles, (long)ncu * BPC), NT_>>>(pin, pout, ld4, n4, R_, tiles); }); }
  TR(64, 64, 1024, 4, 2) TR(128, 32, 1024, 4, 2) TR(256, 16, 1024, 4, 2) TR(256, 32, 1024, 8, 1) TR(256, 16, 512, 8, 2) TR(256, 8, 1024, 2, 2)
  TR(128, 64, 1024, 8, 1) TR(256, 16, 1024, 4, 1) TR(256, 16, 1024, 4, 3)
#define TR1(R_, C4_, NT_, J_) { const long tiles = (n4 + C4_ - 1) / C4_; char nm[96]; snprintf(nm, sizeof nm, "tilecopy1 c4=%d nt=%d J=%d", C4_, NT_, J_); \
    timeit(nm, R_, 2.0 * 16 * n4 * R_, [&]{ k_tilecopy1<C4_, NT_, J_, true, true><<<tiles, NT_>>>(pin, pout, ld4, n4, R_); }); }
  TR1(256, 16, 1024, 4) TR1(128, 32, 1024, 4)
  return 0;
}
