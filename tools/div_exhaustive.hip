// Exhaustive check of a candidate division scheme for K2 on the GPU — a study tool, not part of
// the product (the scheme measured no faster inside K2 and is not used).
// It computes x / n as q0 = RN(x y), q = RN(q0 + RN(x - n q0) y) (both fused) with
// y = RN(1 / n) computed once per norm.  In the range it would be admitted to (n in
// [2^-40, 2^40], |x| in [2^-50, 2^60]) every intermediate is a normal number, so scaling x or n
// by a power of two scales every step exactly and the result depends only on the two
// mantissas and the signs (the scheme is odd in x).  This program compares it with the IEEE
// division for all 2^23 x 2^23 mantissa pairs (x, n in [1, 2)) and prints the mismatch count.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/div_exhaustive tools/div_exhaustive.hip
// usage: tools/div_exhaustive [corrections=1] [first_n_mantissa=0] [count=2^23]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

constexpr int kBlock = 256;
constexpr uint32_t kMant = 1u << 23;

__global__ void k_recip(float* __restrict__ y) {
  const uint32_t m = blockIdx.x * kBlock + threadIdx.x;
  if (m < kMant) y[m] = __fdiv_rn(1.0f, __uint_as_float(0x3F800000u | m));
}

template <int C>
__global__ __launch_bounds__(kBlock) void k_check(const float* __restrict__ y, uint32_t n0, uint32_t nn,
                                                  unsigned long long* __restrict__ bad,
                                                  uint32_t* __restrict__ first) {
  const uint32_t am = blockIdx.x * kBlock + threadIdx.x;
  const float x = __uint_as_float(0x3F800000u | am);
  uint32_t count = 0;
  for (uint32_t i = 0; i < nn; ++i) {
    const uint32_t nm = n0 + i;
    const float n = __uint_as_float(0x3F800000u | nm);
    const float r = y[nm];
    const float ref = __fdiv_rn(x, n);
    float q = __fmul_rn(x, r);
#pragma unroll
    for (int c = 0; c < C; ++c) q = __fmaf_rn(__fmaf_rn(-n, q, x), r, q);
    if (__float_as_uint(q) != __float_as_uint(ref)) {
      if (count == 0) {
        first[0] = am;  // any mismatching pair (vector stores only)
        first[1] = nm;
      }
      ++count;
    }
  }
  if (count) atomicAdd(bad, static_cast<unsigned long long>(count));
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 2;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const int corrections = argc > 1 ? std::atoi(argv[1]) : 1;
  const uint32_t n_first = argc > 2 ? static_cast<uint32_t>(std::atol(argv[2])) : 0;
  uint32_t n_count = argc > 3 ? static_cast<uint32_t>(std::atol(argv[3])) : kMant;
  if (n_first >= kMant) return 2;
  if (n_count > kMant - n_first) n_count = kMant - n_first;
  if (corrections != 1 && corrections != 2) return 2;
  float* y;
  unsigned long long* bad;
  uint32_t* first;
  CK(hipMalloc(&y, sizeof(float) * kMant));
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  CK(hipMalloc(&first, 2 * sizeof(uint32_t)));
  CK(hipMemset(bad, 0, sizeof(unsigned long long)));
  CK(hipMemset(first, 0xFF, 2 * sizeof(uint32_t)));
  k_recip<<<kMant / kBlock, kBlock>>>(y);
  CK(hipGetLastError());
  constexpr uint32_t kPerLaunch = 2048;
  const auto t0 = std::chrono::steady_clock::now();
  auto last = t0;
  for (uint32_t n0 = n_first; n0 < n_first + n_count; n0 += kPerLaunch) {
    const uint32_t nn = n0 + kPerLaunch <= n_first + n_count ? kPerLaunch : n_first + n_count - n0;
    if (corrections == 1)
      k_check<1><<<kMant / kBlock, kBlock>>>(y, n0, nn, bad, first);
    else
      k_check<2><<<kMant / kBlock, kBlock>>>(y, n0, nn, bad, first);
    CK(hipGetLastError());
    const auto now = std::chrono::steady_clock::now();
    if (std::chrono::duration<double>(now - last).count() > 20.0) {
      CK(hipDeviceSynchronize());
      unsigned long long b = 0;
      CK(hipMemcpy(&b, bad, sizeof b, hipMemcpyDeviceToHost));
      std::printf("progress: n mantissas %u..%u done, mismatches %llu, %.1f s\n", n_first, n0 + nn, b,
                  std::chrono::duration<double>(now - t0).count());
      std::fflush(stdout);
      last = now;
    }
  }
  CK(hipDeviceSynchronize());
  unsigned long long b = 0;
  uint32_t f[2];
  CK(hipMemcpy(&b, bad, sizeof b, hipMemcpyDeviceToHost));
  CK(hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost));
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"corrections\": %d, \"n_mantissas\": [%u, %u], \"x_mantissas\": %u, \"pairs\": %llu, "
              "\"mismatches\": %llu, \"example\": [%u, %u], \"seconds\": %.1f}\n",
              corrections, n_first, n_first + n_count, kMant,
              static_cast<unsigned long long>(n_count) * kMant, b, f[0], f[1], secs);
  return b ? 1 : 0;
}
