// K1 launch-shape probe (not part of the product): the library's k_agg_f32_vec<9> on 9 ResNet-50
// operand rows of a 64-row pool (rows rotated per launch), grid-stride with capped grids vs one
// pass over a full grid; each checked bit for bit against the library launch.
#include "../../topology_aware_learning_amd/csrc/tal_agg.hip"
#include <stdio.h>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

__global__ void k_fill(float4* p, long n4, unsigned seed) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed; float v[4];
    for (int k = 0; k < 4; ++k) { h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; v[k] = (float)(int)(h & 0xffffff) * (1.f / 8388608.f) - 1.f; }
    p[i] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// one float4 chunk per lane per operand, U chunks per lane, no grid-stride loop
template <int M, int U>
__global__ __launch_bounds__(256) void k_flat(OpTableF32 t, float* out, int64_t n4) {
  const int64_t i0 = (static_cast<int64_t>(blockIdx.x) * U) * 256 + threadIdx.x;
  float4 v[U][M];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * 256;
    if (i < n4) {
#pragma unroll
      for (int k = 0; k < M; ++k) v[u][k] = ld_stream(t.x[k], i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = i0 + u * 256;
    if (i < n4) {
      float4 acc = first4<true>(t.w[0], v[u][0]);
#pragma unroll
      for (int k = 1; k < M; ++k) acc = next4<true>(acc, t.w[k], v[u][k]);
      reinterpret_cast<float4*>(out)[i] = acc;
    }
  }
}

int main() {
  const int R = 64, M = 9;
  const long n = 23573962L, ld = (n + 63) / 64 * 64, n4 = n / 4;
  float *pool, *ref, *out;
  CK(hipMalloc(&pool, (size_t)R * ld * 4)); CK(hipMalloc(&ref, ld * 4)); CK(hipMalloc(&out, ld * 4));
  k_fill<<<4096, 256>>>((float4*)pool, (long)R * ld / 4, 777u); CK(hipDeviceSynchronize());
  std::vector<OpTableF32> tabs(16);
  for (int r = 0; r < 16; ++r) {
    for (int k = 0; k < kMaxOps; ++k) { tabs[r].x[k] = nullptr; tabs[r].w[k] = 0.f; }
    for (int k = 0; k < M; ++k) { tabs[r].x[k] = pool + (size_t)((r * 4 + k * 7) % R) * ld; tabs[r].w[k] = 1.f / 9.f; }
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = 4.0 * n4 * 4 * (M + 1);
  std::vector<float> a(n4 * 4), b(n4 * 4);
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch(tabs[i]);
    CK(hipDeviceSynchronize()); CK(hipGetLastError());
    float sum = 0; const int reps = 32;
    for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(tabs[i % 16]); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; }
    launch(tabs[5]); CK(hipDeviceSynchronize());
    launch_pass<true>(tabs[5], M, false, true, ref, n4 * 4, 0); CK(hipDeviceSynchronize());
    CK(hipMemcpy(a.data(), ref, n4 * 16, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), out, n4 * 16, hipMemcpyDeviceToHost));
    printf("%-34s avg %.4f ms  %6.0f GB/s  %s\n", name, sum / reps, bytes / (sum / reps * 1e-3) / 1e9, memcmp(a.data(), b.data(), n4 * 16) ? "MISMATCH" : "OK");
    fflush(stdout);
  };
  timeit("library launch (cap 4096, U=2)", [&](const OpTableF32& t) { launch_pass<true>(t, M, false, true, out, n4 * 4, 0); });
  for (int g : {2048, 8192, 16384}) {
    char nm[64]; snprintf(nm, sizeof nm, "grid-stride U=2 grid %d", g);
    timeit(nm, [&](const OpTableF32& t) { k_agg_f32_vec<9, true, false><<<g, kBlock>>>(t, M, out, n4); });
  }
  timeit("full grid U=1", [&](const OpTableF32& t) { k_flat<9, 1><<<(n4 + 255) / 256, 256>>>(t, out, n4); });
  timeit("full grid U=2", [&](const OpTableF32& t) { k_flat<9, 2><<<(n4 + 511) / 512, 256>>>(t, out, n4); });
  timeit("full grid U=4", [&](const OpTableF32& t) { k_flat<9, 4><<<(n4 + 1023) / 1024, 256>>>(t, out, n4); });
  return 0;
}
