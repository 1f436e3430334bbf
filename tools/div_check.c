// Checks a candidate division scheme for K2 against IEEE fp32 division, on the host (a study
// tool, not part of the product; the scheme measured no faster inside K2 and is not used,
// DESIGN.md §9 item 6).  It replaces x / n, where n is a per-thread norm, by a reciprocal
// computed once (y = RN(1 / n)) and, per element, q0 = RN(x y) with Markstein corrections
// q <- RN(q + RN(x - n q) y) (fused); |x| < 2^-50, zeros, NaN and n outside [2^-40, 2^40]
// would keep the IEEE division.  Here: every fp32 mantissa of x at two exponents against
// a set of n (edge mantissas: 1, 1 + ulp, 2 - ulp, and random ones), plus random (x, n) pairs
// over the admitted range; prints the mismatch count (0 expected).
// build: gcc -O2 -fopenmp -ffp-contract=off -o /tmp/div_check tools/div_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float cos_div(float x, float n, float y, int corrections) {
  float q = x * y;
  for (int c = 0; c < corrections; ++c) q = fmaf(fmaf(-n, q, x), y, q);
  return q;
}

static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int main(int argc, char** argv) {
  const int corrections = argc > 1 ? atoi(argv[1]) : 2;
  const int n_rand_den = argc > 2 ? atoi(argv[2]) : 64;
  const long n_pairs = argc > 3 ? atol(argv[3]) : 1L << 30;
  // denominators: edge mantissas at several exponents, then random mantissas
  int nd = 0;
  float dens[4096];
  const int exps[] = {-20, -7, -1, 0, 3, 11, 30};
  const uint32_t edge[] = {0x000000u, 0x000001u, 0x7FFFFFu, 0x7FFFFEu, 0x400000u, 0x3FFFFFu, 0x555555u, 0x2AAAAAu};
  for (unsigned e = 0; e < sizeof exps / sizeof *exps; ++e)
    for (unsigned m = 0; m < sizeof edge / sizeof *edge; ++m)
      dens[nd++] = f_of(((uint32_t)(127 + exps[e]) << 23) | edge[m]);
  uint64_t seed = 12345;
  for (int i = 0; i < n_rand_den && nd < 4096; ++i)
    dens[nd++] = f_of(((uint32_t)(127 + (int)(splitmix(&seed) % 61) - 30) << 23) | (uint32_t)(splitmix(&seed) & 0x7FFFFF));
  long bad = 0, checked = 0;
  // every x mantissa, both signs, at the exponent of n and one below (|x / n| in (1/4, 2))
#pragma omp parallel for reduction(+ : bad, checked) schedule(dynamic)
  for (int d = 0; d < nd; ++d) {
    const float n = dens[d];
    const float y = 1.0f / n;
    const int en = (int)((u_of(n) >> 23) & 0xFF);
    for (int de = -1; de <= 0; ++de)
      for (uint32_t m = 0; m < (1u << 23); ++m)
        for (uint32_t s = 0; s < 2; ++s) {
          const float x = f_of((s << 31) | ((uint32_t)(en + de) << 23) | m);
          const float ref = x / n;
          const float got = cos_div(x, n, y, corrections);
          if (u_of(ref) != u_of(got)) {
            if (bad < 8) printf("mismatch x=%a n=%a ref=%a got=%a\n", x, n, ref, got);
            ++bad;
          }
          ++checked;
        }
  }
  printf("exhaustive-mantissa: corrections=%d dens=%d checked=%ld mismatches=%ld\n", corrections, nd, checked, bad);
  long bad2 = 0;
  // random pairs over the admitted range: n in [2^-40, 2^40], |x| in [2^-50, n]
#pragma omp parallel reduction(+ : bad2)
  {
    uint64_t s = 777;
#ifdef _OPENMP
    extern int omp_get_thread_num(void);
    s += 1000003ull * (uint64_t)omp_get_thread_num();
#endif
#pragma omp for
    for (long i = 0; i < n_pairs; ++i) {
      const uint64_t r = splitmix(&s);
      const int en = 127 - 40 + (int)(r % 81);
      const float n = f_of(((uint32_t)en << 23) | (uint32_t)((r >> 8) & 0x7FFFFF));
      const uint64_t r2 = splitmix(&s);
      int ex = en - (int)(r2 % 64);
      if (ex < 127 - 50) ex = 127 - 50;
      const float x = f_of((uint32_t)((r2 >> 40) & 1) << 31 | ((uint32_t)ex << 23) | (uint32_t)((r2 >> 8) & 0x7FFFFF));
      const float y = 1.0f / n;
      if (u_of(x / n) != u_of(cos_div(x, n, y, corrections))) {
        if (bad2 < 8) printf("random mismatch x=%a n=%a\n", x, n);
        ++bad2;
      }
    }
  }
  printf("random: corrections=%d pairs=%ld mismatches=%ld\n", corrections, n_pairs, bad2);
  return (bad || bad2) ? 1 : 0;
}
