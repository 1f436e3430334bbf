// Probe (not part of the product): does gfx950's VGPR index mode (s_set_gpr_idx_on, SRC0)
// offset the first source of a packed (VOP3P), a VOP3-encoded and a VOP2 instruction?  The
// register-resident round kernel would read a community's sources from VGPRs by a wave-uniform
// index this way.  Each variant multiplies X[idx] (X = 64 floats per lane in v[100:163]) by w for
// a list of indices and checks every lane's result on the host.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float v32f __attribute__((ext_vector_type(32)));
typedef float v2f __attribute__((ext_vector_type(2)));

template <int V>
__device__ __forceinline__ v2f idx_mul(const v32f& X0, const v32f& X1, int idx, float w, float wv) {
  v2f t;
  if constexpr (V == 0) {  // VOP3P: both halves, weight from an SGPR
    const v2f ww = {w, w};
    asm volatile("s_set_gpr_idx_on %3, gpr_idx(SRC0)\n\tv_pk_mul_f32 %0, v[100:101], %4\n\ts_set_gpr_idx_off"
                 : "=v"(t) : "{v[100:131]}"(X0), "{v[132:163]}"(X1), "s"(idx), "s"(ww) : "m0");
  } else if constexpr (V == 1) {  // VOP3 encoding, SGPR second source
    asm volatile("s_set_gpr_idx_on %3, gpr_idx(SRC0)\n\tv_mul_f32_e64 %0, v100, %4\n\tv_mul_f32_e64 %1, v101, %4\n\ts_set_gpr_idx_off"
                 : "=v"(t.x), "=v"(t.y) : "{v[100:131]}"(X0), "s"(idx), "s"(w), "{v[132:163]}"(X1) : "m0");
  } else {  // VOP2 (second source a VGPR)
    asm volatile("s_set_gpr_idx_on %3, gpr_idx(SRC0)\n\tv_mul_f32_e32 %0, v100, %4\n\tv_mul_f32_e32 %1, v101, %4\n\ts_set_gpr_idx_off"
                 : "=v"(t.x), "=v"(t.y) : "{v[100:131]}"(X0), "s"(idx), "v"(wv), "{v[132:163]}"(X1) : "m0");
  }
  return t;
}

template <int V>
__global__ void k(const float* in, float* out, const int* idxs, int nidx, float w) {
  v32f X0, X1;
  const int lane = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 32; ++k) { X0[k] = in[k * 64 + lane]; X1[k] = in[(k + 32) * 64 + lane]; }
  for (int i = 0; i < nidx; ++i) {
    const int id = __builtin_amdgcn_readfirstlane(idxs[i]);
    const v2f t = idx_mul<V>(X0, X1, id, w, w);
    out[(i * 64 + lane) * 2] = t.x;
    out[(i * 64 + lane) * 2 + 1] = t.y;
  }
}

int main() {
  static float h_in[64 * 64];
  for (int i = 0; i < 64 * 64; ++i) h_in[i] = (float)(i % 977) * 0.5f + 1.f;
  int h_idx[] = {0, 2, 4, 62, 30, 32, 40, 10, 12, 60};  // even: 64-bit VGPR operands are even-aligned on gfx950
  const int n = sizeof(h_idx) / sizeof(int);
  float *d_in, *d_out; int* d_idx;
  if (hipMalloc(&d_in, sizeof h_in) || hipMalloc(&d_out, n * 64 * 2 * 4) || hipMalloc(&d_idx, sizeof h_idx)) return 2;
  if (hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice) || hipMemcpy(d_idx, h_idx, sizeof h_idx, hipMemcpyHostToDevice)) return 2;
  const float w = 0.25f;
  int fails = 0;
  for (int v = 0; v < 3; ++v) {
    if (v == 0) k<0><<<1, 64>>>(d_in, d_out, d_idx, n, w);
    if (v == 1) k<1><<<1, 64>>>(d_in, d_out, d_idx, n, w);
    if (v == 2) k<2><<<1, 64>>>(d_in, d_out, d_idx, n, w);
    static float h_out[10 * 64 * 2];
    hipError_t e = hipMemcpy(h_out, d_out, n * 64 * 2 * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess) { printf("variant %d: HIP error %s\n", v, hipGetErrorString(e)); return 1; }
    int bad = 0;
    for (int i = 0; i < n; ++i)
      for (int l = 0; l < 64; ++l)
        for (int h = 0; h < 2; ++h) {
          const float want = w * h_in[(h_idx[i] + h) * 64 + l];
          if (h_out[(i * 64 + l) * 2 + h] != want) {
            if (bad < 3) printf("  v%d idx=%d lane=%d half=%d got %g want %g\n", v, h_idx[i], l, h, h_out[(i * 64 + l) * 2 + h], want);
            ++bad;
          }
        }
    printf("variant %d (%s): %s, %d mismatches\n", v, v == 0 ? "VOP3P v_pk_mul_f32" : v == 1 ? "VOP3 v_mul_f32_e64" : "VOP2 v_mul_f32_e32",
           bad ? "FAIL" : "OK", bad);
    fails += bad != 0;
  }
  return 0;
}
