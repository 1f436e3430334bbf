// Round-kernel probe (not part of the product): compiles the library source in and times
// launch variants of the config-3 round (64 ResNet-50 fp32 rows, random 8-regular graph, self
// last, 1/9 weights, random data), each checked bit for bit against the library's launch.
#include "../../topology_aware_learning_amd/csrc/tal_agg.hip"
#include <stdio.h>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void k_fill(float4* p, long n4, unsigned seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed; float v[4];
    for (int k = 0; k < 4; ++k) { h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; v[k] = (float)(int)(h & 0xffffff) * (1.f / 8388608.f) - 1.f; }
    p[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// V9: persistent, one workgroup per CU, tile data double-buffered in LDS by global->LDS DMA
// (no staging registers); one barrier per tile.
template <int NT>
__global__ __launch_bounds__(NT, 1) void k_v9(const float* __restrict__ pin, int64_t ld_in4, float* __restrict__ pout,
                                             int64_t ld_out4, int64_t n4, PlanView p, int64_t n_tiles) {
  constexpr int C4 = 64, NW = NT / 64;
  extern __shared__ float4 s_data[];
  const int ns = p.grp_src_ptr[1] - p.grp_src_ptr[0];
  const int nr = p.grp_row_ptr[1];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  const int per_wave = (ns + NW - 1) / NW;  // sources this wave DMAs per tile (<= 8)
  const float4* pin4 = reinterpret_cast<const float4*>(pin);
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const void*)s_data));
  int srow[8];
#pragma unroll
  for (int d = 0; d < 8; ++d) { const int s = wave + d * NW; srow[d] = (d < per_wave && s < ns) ? p.src_row[s] : -1; }
  const int tile_f4 = ns * C4;
  auto issue = [&](int64_t t, int buf) {
    const int64_t col = min(t * C4 + lane, n4 - 1);
#pragma unroll
    for (int d = 0; d < 8; ++d)
      if (srow[d] >= 0) dma16(pin4 + (int64_t)srow[d] * ld_in4 + col, lds0 + (uint32_t)((buf * tile_f4 + (wave + d * NW) * C4) * 16));
  };
  int64_t t = blockIdx.x;
  int buf = 0;
  int my_dma = 0;
#pragma unroll
  for (int d = 0; d < 8; ++d) my_dma += srow[d] >= 0;
  const int my_rows = (nr - wave + NW - 1) / NW;
  if (t < n_tiles) issue(t, 0);
  bool first = true;
  for (; t < n_tiles; t += gridDim.x) {
    // this tile's DMA was issued before the previous tile's stores: wait for all but those stores
    wait_vm_barrier(first ? 0 : my_rows);
    first = false;
    if (t + gridDim.x < n_tiles) issue(t + gridDim.x, buf ^ 1);
    emit_tile<C4, NT, true>(s_data + buf * tile_f4, p, 0, nr, pout, ld_out4, t * C4, n4);
    buf ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// V10: the library's persistent kernel, but workgroup b walks a contiguous range of tiles
template <int C4, int NT, int J>
__global__ __launch_bounds__(NT) void k_v10(const float* __restrict__ pin, int64_t ld_in4, float* __restrict__ pout,
                                           int64_t ld_out4, int64_t n4, PlanView p, int64_t n_tiles) {
  extern __shared__ float4 s_data[];
  const int ns = p.grp_src_ptr[1] - p.grp_src_ptr[0];
  const int nr = p.grp_row_ptr[1];
  const int c = threadIdx.x % C4;
  int srow[J];
#pragma unroll
  for (int j = 0; j < J; ++j) { const int src = (j * NT + threadIdx.x) / C4; srow[j] = src < ns ? p.src_row[src] : -1; }
  float4 v[J];
  auto load_tile = [&](int64_t tt) {
    const int64_t col = tt * C4 + c;
    if (col < n4) {
#pragma unroll
      for (int j = 0; j < J; ++j) if (srow[j] >= 0) v[j] = ld_stream(pin, (int64_t)srow[j] * ld_in4 + col);
    }
  };
  const int64_t per = (n_tiles + gridDim.x - 1) / gridDim.x;
  const int64_t t0 = blockIdx.x * per, t1 = min(n_tiles, t0 + per);
  int64_t t = t0;
  if (t < t1) load_tile(t);
  for (; t < t1; ++t) {
    __syncthreads();
#pragma unroll
    for (int j = 0; j < J; ++j) if (srow[j] >= 0) s_data[j * NT + threadIdx.x] = v[j];
    __syncthreads();
    if (t + 1 < t1) load_tile(t + 1);
    emit_tile<C4, NT, true>(s_data, p, 0, nr, pout, ld_out4, t * C4, n4);
  }
}

int main(int argc, char** argv) {
  const int R = 64, deg = 8;
  const long n = 23573962L, ld = (n + 63) / 64 * 64, n4 = n / 4;
  float *pin, *pref, *pout;
  CK(hipMalloc(&pin, (size_t)R * ld * 4)); CK(hipMalloc(&pref, (size_t)R * ld * 4)); CK(hipMalloc(&pout, (size_t)R * ld * 4));
  k_fill<<<4096, 256>>>((float4*)pin, (long)R * ld / 4, 12345u); CK(hipDeviceSynchronize());
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
  const PlanView v = make_view(dplan, info);
  printf("groups=%d staged=%d\n", info.n_groups, info.total_src);
  CK(tal_agg_round_f32(pin, ld, pref, ld, n, dplan, &info, 1, 0) ? hipErrorUnknown : hipSuccess);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 4.0 * n * (info.total_src + R);
  std::vector<float> a(ld), b(ld);
  auto timeit = [&](const char* name, auto launch) {
    CK(hipMemset(pout, 0, (size_t)R * ld * 4));
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize()); CK(hipGetLastError());
    const int reps = 20; float sum = 0, best = 1e9;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; best = std::min(best, ms); }
    bool ok = true;
    for (int r = 0; r < R && ok; r += 7) {
      CK(hipMemcpy(a.data(), pref + r * ld, n4 * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), pout + r * ld, n4 * 16, hipMemcpyDeviceToHost));
      ok = memcmp(a.data(), b.data(), n4 * 16) == 0;
    }
    printf("%-48s avg %.3f ms  best %.3f ms  %6.0f GB/s avg  %s\n", name, sum / reps, best, bytes / (sum / reps * 1e-3) / 1e9, ok ? "OK" : "MISMATCH");
    fflush(stdout);
  };
  const int64_t tiles = (n4 + 63) / 64;
  const size_t lds = (size_t)info.max_src * 64 * 16;
  timeit("library (persistent, 2 wg/cu)", [&]{ tal_agg_round_f32(pin, ld, pout, ld, n, dplan, &info, 1, 0); });
  {
    auto k = k_round_f32_persistent<64, 1024, 4, true, false>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    for (int gx : {256, 384, 512, 1024}) {
      char nm[96]; snprintf(nm, sizeof nm, "persistent grid %d", gx);
      timeit(nm, [&]{ k<<<dim3(gx, 1), 1024, lds>>>(pin, ld / 4, pout, ld / 4, n4, v, tiles); });
    }
  }
  {
    auto k = k_round_f32_persistent<64, 512, 8, true, false>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("persistent nt=512 J=8 grid 512", [&]{ k<<<dim3(512, 1), 512, lds>>>(pin, ld / 4, pout, ld / 4, n4, v, tiles); });
  }
  {
    auto k = k_round_f32_tiled<64, 1024, true, false>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("tiled (tile per wg) nt=1024", [&]{ k<<<dim3(tiles, 1), 1024, lds>>>(pin, ld / 4, pout, ld / 4, n4, v); });
  }
  {
    auto k = k_round_f32_tiled<64, 512, true, false>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("tiled (tile per wg) nt=512", [&]{ k<<<dim3(tiles, 1), 512, lds>>>(pin, ld / 4, pout, ld / 4, n4, v); });
  }
  {
    auto k = k_v10<64, 1024, 4>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("v10 contiguous ranges grid 512", [&]{ k<<<512, 1024, lds>>>(pin, ld / 4, pout, ld / 4, n4, v, tiles); });
  }
  {
    auto k = k_v9<1024>;
    CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("v9 DMA double buffer 1 wg/cu nt=1024", [&]{ k<<<256, 1024, 2 * lds>>>(pin, ld / 4, pout, ld / 4, n4, v, tiles); });
    auto k2 = k_v9<512>;
    CK(hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    timeit("v9 DMA double buffer 1 wg/cu nt=512", [&]{ k2<<<256, 512, 2 * lds>>>(pin, ld / 4, pout, ld / 4, n4, v, tiles); });
  }
  return 0;
}
