// Tuning harness for K1 (per-call streaming aggregation), not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include <algorithm>
#include "../../include/tal_agg.h"
#pragma clang fp contract(off)
typedef float v4f __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
struct Tab { const float* x[256]; float w[256]; };

__device__ __forceinline__ v4f mulv(float w, v4f x) { return (v4f){__fmul_rn(w,x.x), __fmul_rn(w,x.y), __fmul_rn(w,x.z), __fmul_rn(w,x.w)}; }
__device__ __forceinline__ v4f addv(v4f a, float w, v4f x) { return (v4f){__fadd_rn(a.x,__fmul_rn(w,x.x)), __fadd_rn(a.y,__fmul_rn(w,x.y)), __fadd_rn(a.z,__fmul_rn(w,x.z)), __fadd_rn(a.w,__fmul_rn(w,x.w))}; }

template <int M, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k1(Tab t, float* out, long n4) {
  const long stride = (long)gridDim.x * 256 * U;
  for (long i0 = (long)blockIdx.x * 256 * U + threadIdx.x; i0 < n4; i0 += stride) {
    v4f v[U][M];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * 256;
#pragma unroll
      for (int k = 0; k < M; ++k) {
        if (i < n4) { const v4f* p = reinterpret_cast<const v4f*>(t.x[k]) + i; v[u][k] = NTL ? __builtin_nontemporal_load(p) : *p; }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = i0 + u * 256;
      if (i < n4) {
        v4f acc = mulv(t.w[0], v[u][0]);
#pragma unroll
        for (int k = 1; k < M; ++k) acc = addv(acc, t.w[k], v[u][k]);
        v4f* o = reinterpret_cast<v4f*>(out) + i;
        if (NTS) __builtin_nontemporal_store(acc, o); else *o = acc;
      }
    }
  }
}

int main(int argc, char** argv) {
  const long n = 23573962L, ld = (n + 63) / 64 * 64;
  const int rows = 64;
  float *pool, *ref, *out;
  CK(hipMalloc(&pool, rows * ld * 4)); CK(hipMalloc(&ref, ld * 4)); CK(hipMalloc(&out, ld * 4));
  CK(hipMemset(pool, 0, rows * ld * 4));
  { std::vector<float> h(ld); for (int r = 0; r < rows; ++r) { for (long i = 0; i < ld; ++i) h[i] = (float)((r * 131 + i * 7) % 1013) * 0.001f - 0.5f; CK(hipMemcpy(pool + r * ld, h.data(), ld * 4, hipMemcpyHostToDevice)); } }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const long n4 = n / 4;
  for (int M : {3, 9, 17}) {
    auto mk = [&](int rot) { Tab t; for (int k = 0; k < M; ++k) { t.x[k] = pool + ((rot * 7 + k * 5) % rows) * ld; t.w[k] = 1.0f / M; } return t; };
    const float* xs[256]; double w[256]; Tab t0 = mk(0); for (int k = 0; k < M; ++k) { xs[k] = t0.x[k]; w[k] = 1.0 / M; }
    const double bytes = 4.0 * n * (M + 1);
    auto timeit = [&](const char* name, auto launch) {
      for (int i = 0; i < 3; ++i) launch(i);
      CK(hipDeviceSynchronize());
      float sum = 0; const int reps = 30;
      for (int i = 0; i < reps; ++i) { CK(hipEventRecord(e0)); launch(i); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); sum += ms; }
      CK(hipGetLastError());
      launch(0); CK(hipDeviceSynchronize());
      std::vector<float> a(n), b(n); CK(hipMemcpy(a.data(), ref, n * 4, hipMemcpyDeviceToHost)); CK(hipMemcpy(b.data(), out, n * 4, hipMemcpyDeviceToHost));
      bool ok = memcmp(a.data(), b.data(), (n / 4 * 4) * 4) == 0;
      printf("M=%2d %-36s %.3f ms %6.0f GB/s %s\n", M, name, sum / reps, bytes / (sum / reps * 1e-3) / 1e9, ok ? "OK" : "MISMATCH");
    };
    tal_agg_f32(xs, w, M, ref, n, 1, 0); CK(hipDeviceSynchronize());
    timeit("lib", [&](int i) { Tab t = mk(i); const float* p[256]; for (int k = 0; k < M; ++k) p[k] = t.x[k]; tal_agg_f32(i ? p : xs, w, M, out, n, 1, 0); });
    char nm[128];
#define RUN(MM, U, NL, NS, G) if (M == MM) { snprintf(nm, sizeof nm, "U=%d ntl=%d nts=%d grid=%d", U, NL, NS, G); \
      timeit(nm, [&](int i) { Tab t = mk(i); if (!i) t = t0; k1<MM, U, NL, NS><<<G, 256>>>(t, out, n4); }); }
#define SET(MM) RUN(MM,1,1,0,2048) RUN(MM,1,1,0,4096) RUN(MM,1,1,0,8192) RUN(MM,2,1,0,2048) RUN(MM,2,1,0,4096) RUN(MM,2,1,1,2048) RUN(MM,2,1,1,1024) RUN(MM,4,1,0,1024) RUN(MM,4,1,1,1024) RUN(MM,2,1,0,1024)
    SET(3) SET(9) SET(17)
  }
  // plain copy roofline reference
  {
    const double bytes = 8.0 * n;
    float sum = 0;
    for (int i = 0; i < 23; ++i) { CK(hipEventRecord(e0)); CK(hipMemcpyAsync(out, pool + ((i * 5) % rows) * ld, n * 4, hipMemcpyDeviceToDevice)); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (i >= 3) sum += ms; }
    printf("hipMemcpy D2D 94MB: %.3f ms %.0f GB/s\n", sum / 20, bytes / (sum / 20 * 1e-3) / 1e9);
  }
  return 0;
}
