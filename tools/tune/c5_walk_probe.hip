// Memory-side probe for BASELINE config 5 (not part of the product): 256 model rows of the
// ViT-B/16 layout (86,567,656 fp32 / bf16 elements), every source read once and every output
// written once per round, walked as the round kernels walk it — a persistent grid, one tile =
// C4 16-B chunks of each row of a row group, the next tile's loads in flight in registers — as a
// pure copy (row r -> row r), optionally staged through LDS with a barrier the way K3n stages.
// Reports GB/s per (tile width, rows per tile, workgroups per CU) so the narrow kernel's memory
// side can be compared with the walk it does at other widths.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <algorithm>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__device__ __forceinline__ v4f ldnt(const v4f* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void stnt(v4f* p, v4f v) { __builtin_nontemporal_store(v, p); }

// tile t -> (row group t % G, column tile t / G): the G groups of one column tile run together
template <int C4, int NT, int J, bool STAGE>
__global__ __launch_bounds__(NT) void k_walk(const v4f* __restrict__ pin, v4f* __restrict__ pout, long ld4, long n4,
                                             int RG, int G, long n_tiles) {
  extern __shared__ v4f s[];
  const int c = threadIdx.x % C4;
  int rr[J];
#pragma unroll
  for (int j = 0; j < J; ++j) rr[j] = (j * NT + threadIdx.x) / C4;  // row within the group
  v4f v[J];
  auto load = [&](long tt) {
    const long ct = tt / G, g = tt % G;
    const long col = std::min(ct * C4 + c, n4 - 1);
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int r = rr[j] < RG ? rr[j] : 0;
      v[j] = ldnt(pin + (g * RG + r) * ld4 + col);
    }
  };
  long t = blockIdx.x;
  if (t < n_tiles) load(t);
  for (; t < n_tiles; t += gridDim.x) {
    const long ct = t / G, g = t % G;
    const long col = ct * C4 + c;
    v4f w[J];
    if constexpr (STAGE) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < J; ++j) s[j * NT + threadIdx.x] = v[j];
      __syncthreads();
    } else {
#pragma unroll
      for (int j = 0; j < J; ++j) w[j] = v[j];
    }
    if (t + gridDim.x < n_tiles) load(t + gridDim.x);
    if constexpr (STAGE) {
      // read back another wave's slot of the same column (as the row passes do)
#pragma unroll
      for (int j = 0; j < J; ++j) w[j] = s[((j * NT + threadIdx.x) + 7 * C4) % (J * NT)];
    }
    if (col < n4) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int k = (j * NT + threadIdx.x + (STAGE ? 7 * C4 : 0)) % (J * NT);
        const int r = k / C4;
        if (r < RG) stnt(pout + (g * RG + r) * ld4 + col, w[j]);
      }
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

int main(int argc, char** argv) {
  const int R = 256;
  const bool bf16 = argc > 1 && strcmp(argv[1], "bf16") == 0;
  const long n_el = 86567656L;
  // bytes per row: fp32 4 B, bf16 2 B per element; chunks of 16 B either way
  const long row_bytes = n_el * (bf16 ? 2 : 4);
  const long ld4 = (row_bytes + 255) / 256 * 16, n4 = row_bytes / 16;
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  v4f *pin, *pout;
  CK(hipMalloc(&pin, (size_t)R * ld4 * 16)); CK(hipMalloc(&pout, (size_t)R * ld4 * 16));
  k_fill<<<8192, 256>>>(pin, (long)R * ld4, 12345u); CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  printf("config-5 walk probe: %s rows of %ld B, 256 in + 256 out\n", bf16 ? "bf16" : "fp32", row_bytes);
  const double bytes = 2.0 * 16 * n4 * R;
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 2; ++i) launch();
    CK(hipDeviceSynchronize()); CK(hipGetLastError());
    const int reps = 6; float sum = 0, best = 1e9;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; best = std::min(best, ms); }
    printf("%-58s avg %7.3f ms  best %7.3f  %6.0f GB/s\n", name, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9);
    fflush(stdout);
  };
#define W(C4_, NT_, J_, RG_, BPC, STG) { \
    const int G = R / RG_; const long tiles = (n4 + C4_ - 1) / C4_ * G; char nm[128]; \
    snprintf(nm, sizeof nm, "%s c4=%d (%d B) rows/tile=%d nt=%d J=%d wg/cu=%d", STG ? "staged" : "regs  ", C4_, C4_ * 16, RG_, NT_, J_, BPC); \
    const size_t lds = STG ? (size_t)J_ * NT_ * 16 : 0; \
    if (lds > 65536) CK(hipFuncSetAttribute((const void*)k_walk<C4_, NT_, J_, STG>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
    timeit(nm, [&]{ k_walk<C4_, NT_, J_, STG><<<std::min<long>(tiles, (long)ncu * BPC), NT_, lds>>>(pin, pout, ld4, n4, RG_, G, tiles); }); }
  // the narrow kernel's walk: all 256 rows per tile
  W(16, 1024, 4, 256, 2, true) W(16, 1024, 4, 256, 2, false) W(16, 1024, 4, 256, 1, false)
  W(32, 1024, 8, 256, 1, true) W(32, 1024, 8, 256, 1, false) W(32, 1024, 8, 256, 2, false)
  W(8, 1024, 2, 256, 2, false) W(8, 1024, 2, 256, 4, false)
  W(64, 1024, 16, 256, 1, false)
  // fewer rows per tile, wider pieces (community-sized groups)
  W(32, 1024, 4, 128, 2, true) W(64, 1024, 4, 64, 2, true) W(128, 1024, 4, 32, 2, true)
  W(64, 1024, 2, 32, 2, false) W(128, 1024, 4, 32, 2, false) W(128, 1024, 8, 64, 1, false)
  W(32, 512, 8, 128, 2, false) W(64, 512, 8, 64, 2, false)
  return 0;
}
