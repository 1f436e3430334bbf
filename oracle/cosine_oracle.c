/*
 * oracle/cosine_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * The reference's model similarity in the exact fp32 operation order of the torch CPU kernels
 * it runs on, so that sim_centrality_module_avg's arg-min (and with it the softmax sign) can be
 * checked bit for bit, near-ties included.
 *
 * Reference: src/decentralized_client.py:661-681
 *     cos = nn.CosineSimilarity(dim=1, eps=1e-6)
 *     for w_1, w_2 in zip(params(model_1), params(model_2)):
 *         if len(w_1.shape) < 2: w_1, w_2 = w_1.unsqueeze(1), w_2.unsqueeze(1)
 *         avg_cos += cos(w_1, w_2).mean()
 *     return avg_cos / len(weights_1)
 * and torch's cosine_similarity (ATen Distance.cpp, normalize-first form):
 *     n1 = clamp_min(vector_norm(x1, 2, dim=1, keepdim), eps); n2 likewise
 *     s  = ((x1 / n1) * (x2 / n2)).sum(dim=1);   mean = s.sum() / s.numel()
 *
 * The reduction orders below are those of torch 2.10's CPU kernels as run where the golden
 * vectors are generated (AVX512 capability; the sum kernel works on 8-wide fp32 vectors), found
 * by bit-comparison against torch on random inputs and pinned by tests/test_oracle_golden.py
 * (the reference's own cosine values, bitwise):
 *   vector_norm over dim 1, reduced dim innermost (K == 1): 8 lane accumulators acc_l =
 *     fma(x, x, acc_l) over whole 8-vectors; lanes summed 0..7 in order; the tail in groups of 4
 *     with separate fp32 square and add, the last < 4 elements by fma; sqrt.
 *   vector_norm over a strided dim 1 (K > 1): acc = fma(x, x, acc) in index order; sqrt.
 *   sum (cascade_sum): row_sum = 4 interleaved partial sums (ilp) each a 4-level cascade
 *     (multi_row_sum), remainder into partial 0, partials 1..3 added to 0 in order; a
 *     contiguous reduction of n >= 8 runs it on 8-wide vectors (lane l sums elements
 *     8 i + l), then the scalar tail, then lanes 0..7; a strided one runs it per column
 *     (columns in chunks of 32 share one 4-row cascade, then chunks of 8, then single columns).
 *   a full sum over n >= 32768 elements (at::internal::GRAIN_SIZE) with T > 1 intra-op threads
 *     is torch's two_pass_reduction (TensorIteratorReduce.cpp) over at::parallel_for: nt =
 *     min(T, ceil(n / 32768)) chunks of ceil(n / nt) elements, each chunk's serial sum stored
 *     into a T-entry buffer of zeros, then the buffer's serial sum (par_sum; pinned against the
 *     reference's cosine_similarity at T = 1..32 by tests/golden/cosine_threads.json).  The
 *     per-output norms and sums split over outputs and do not depend on T.  The reference's
 *     CNNs never reach 32768 outputs per tensor (largest 4608); ViT-B/16's patch embedding has
 *     196,608.
 *
 * Built with gcc -O2 -ffp-contract=off: every float op rounds to fp32; fmaf is the single
 * rounding fused multiply-add.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define VW 8      /* Vectorized<float> width of the sum kernel */
#define ILP 4     /* row_sum interleave */
#define LEVELS 4  /* multi_row_sum cascade levels */

static int64_t ceil_log2(int64_t x) {
  int64_t r = 0;
  while ((((int64_t)1) << r) < x) ++r;
  return r;
}

/* multi_row_sum for `nrows` interleaved scalar streams: stream k's element i at
 * base[(i * row_stride + k * col_stride) * elem] - a column view: load(i, k). */
typedef float (*load_fn)(const void* ctx, int64_t i, int64_t k);

static void multi_row_sum(load_fn load, const void* ctx, int nrows, int64_t size, float* out) {
  const int64_t level_power = ceil_log2(size) / LEVELS > 4 ? ceil_log2(size) / LEVELS : 4;
  const int64_t level_step = (int64_t)1 << level_power;
  const int64_t level_mask = level_step - 1;
  float acc[LEVELS][ILP * VW];
  memset(acc, 0, sizeof(acc));
  int64_t i = 0;
  while (i + level_step <= size) {
    for (int64_t j = 0; j < level_step; ++j, ++i)
      for (int k = 0; k < nrows; ++k) acc[0][k] = acc[0][k] + load(ctx, i, k);
    for (int j = 1; j < LEVELS; ++j) {
      for (int k = 0; k < nrows; ++k) {
        acc[j][k] = acc[j][k] + acc[j - 1][k];
        acc[j - 1][k] = 0.f;
      }
      if ((i & (level_mask << (j * level_power))) != 0) break;
    }
  }
  for (; i < size; ++i)
    for (int k = 0; k < nrows; ++k) acc[0][k] = acc[0][k] + load(ctx, i, k);
  for (int j = 1; j < LEVELS; ++j)
    for (int k = 0; k < nrows; ++k) acc[0][k] = acc[0][k] + acc[j][k];
  for (int k = 0; k < nrows; ++k) out[k] = acc[0][k];
}

/* a strided scalar stream: element i at p[i * stride] */
typedef struct {
  const float* p;
  int64_t stride;
} stream_t;

static float load_ilp(const void* ctx, int64_t i, int64_t k) {
  const stream_t* s = (const stream_t*)ctx;
  return s->p[(i * ILP + k) * s->stride];
}

/* row_sum over one scalar stream of `size` elements */
static float row_sum(const float* p, int64_t stride, int64_t size) {
  float ps[ILP * VW] = {0};
  const int64_t size_ilp = size / ILP;
  stream_t s = {p, stride};
  if (size_ilp > 0) multi_row_sum(load_ilp, &s, ILP, size_ilp, ps);
  for (int64_t i = size_ilp * ILP; i < size; ++i) ps[0] = ps[0] + p[i * stride];
  for (int k = 1; k < ILP; ++k) ps[0] = ps[0] + ps[k];
  return ps[0];
}

/* full sum of a contiguous vector (vectorized_inner_sum / scalar_inner_sum), stored into a
 * zero-filled output: 0 + result */
static float inner_sum(const float* x, int64_t n) {
  if (n < VW) return 0.f + row_sum(x, 1, n);
  const int64_t vec = n / VW;
  float lane[VW];
  for (int l = 0; l < VW; ++l) lane[l] = row_sum(x + l, VW, vec);  /* lane l: elements 8 i + l */
  float fin = 0.f;
  for (int64_t k = vec * VW; k < n; ++k) fin = fin + x[k];
  for (int l = 0; l < VW; ++l) fin = fin + lane[l];
  return 0.f + fin;
}

/* torch's full sum with T intra-op threads (serial below the grain or at T == 1) */
#define GRAIN 32768
#define MAX_THREADS 1024
static float par_sum(const float* x, int64_t n, int T) {
  if (n < GRAIN || T <= 1) return inner_sum(x, n);
  if (T > MAX_THREADS) return NAN;  /* callers validate 1 <= T <= MAX_THREADS */
  float buf[MAX_THREADS];
  memset(buf, 0, sizeof(buf));
  int64_t nt = (n + GRAIN - 1) / GRAIN;
  if (nt > T) nt = T;
  const int64_t chunk = (n + nt - 1) / nt;
  for (int64_t t = 0; t < nt && t * chunk < n; ++t)
    buf[t] = inner_sum(x + t * chunk, n - t * chunk < chunk ? n - t * chunk : chunk);
  return inner_sum(buf, T);
}

typedef struct {
  const float* p;  /* p[i * K + c] */
  int64_t K;
  int64_t c0;
} cols_t;

static float load_col(const void* ctx, int64_t i, int64_t k) {
  const cols_t* s = (const cols_t*)ctx;
  return s->p[i * s->K + s->c0 + k];
}

/* sum over the strided dim of p[I][K] (vectorized_outer_sum) into out[K] */
static void outer_sum(const float* p, int64_t I, int64_t K, float* out) {
  int64_t j = 0;
  if (K >= VW) {
    for (; j + ILP * VW <= K; j += ILP * VW) {  /* 4 vectors of 8 columns share one cascade */
      float acc[ILP * VW];
      cols_t s = {p, K, j};
      multi_row_sum(load_col, &s, ILP * VW, I, acc);
      for (int k = 0; k < ILP * VW; ++k) out[j + k] = 0.f + acc[k];
    }
    for (; j + VW <= K; j += VW)
      for (int k = 0; k < VW; ++k) out[j + k] = 0.f + row_sum(p + j + k, K, I);
  }
  for (; j < K; ++j) out[j] = 0.f + row_sum(p + j, K, I);
}

static float norm_strided(const float* x, int64_t stride, int64_t I) {
  float acc = 0.f;
  for (int64_t i = 0; i < I; ++i) acc = fmaf(x[i * stride], x[i * stride], acc);
  return sqrtf(acc);
}

static float norm_lastdim(const float* x, int64_t I) {
  float acc[VW] = {0};
  int64_t d = 0;
  for (; d < I - I % VW; d += VW)
    for (int l = 0; l < VW; ++l) acc[l] = fmaf(x[d + l], x[d + l], acc[l]);
  float b = acc[0];
  for (int l = 1; l < VW; ++l) b = b + acc[l];
  const int64_t tail = I - d;
  const int64_t sep = tail / 4 * 4;
  for (int64_t k = 0; k < sep; ++k, ++d) {
    const float sq = x[d] * x[d];
    b = b + sq;
  }
  for (; d < I; ++d) b = fmaf(x[d], x[d], b);
  return sqrtf(b);
}

/* mean over the O*K outputs of cos(x1, x2) along dim 1 for one parameter tensor viewed
 * [O, I, K]; scratch: 3 * O * K + I * K floats */
static float cos_tensor(const float* a, const float* b, int64_t O, int64_t I, int64_t K, int T, float* scratch) {
  const float eps = 1e-6f;
  float* s = scratch;            /* [O * K] */
  float* n1 = s + O * K;         /* [K] */
  float* n2 = n1 + K;
  float* prod = n2 + K;          /* [I * K] */
  for (int64_t o = 0; o < O; ++o) {
    const float* x1 = a + o * I * K;
    const float* x2 = b + o * I * K;
    for (int64_t k = 0; k < K; ++k) {
      float m1, m2;
      if (K == 1 && I > 1) {
        m1 = norm_lastdim(x1, I);
        m2 = norm_lastdim(x2, I);
      } else {
        m1 = norm_strided(x1 + k, K, I);
        m2 = norm_strided(x2 + k, K, I);
      }
      n1[k] = m1 < eps ? eps : m1;  /* clamp_min_(eps); NaN stays NaN */
      n2[k] = m2 < eps ? eps : m2;
    }
    for (int64_t i = 0; i < I; ++i)
      for (int64_t k = 0; k < K; ++k) {
        const float u = x1[i * K + k] / n1[k];
        const float v = x2[i * K + k] / n2[k];
        prod[i * K + k] = u * v;
      }
    if (I == 1) {
      for (int64_t k = 0; k < K; ++k) s[o * K + k] = 0.f + prod[k];
    } else if (K == 1) {
      s[o] = inner_sum(prod, I);
    } else {
      outer_sum(prod, I, K, s + o * K);
    }
  }
  return par_sum(s, O * K, T) / (float)(O * K);
}

/* cosine_similarity(model_1, model_2) of the reference: segs = (offset, A, I, B) per parameter
 * in named_parameters order, A*I*B elements at `offset` of the flat fp32 model rows a / b
 * (1-D parameters: A = n, I = 1, B = 1).  scratch must hold oracle_cosine_scratch(segs) floats. */
int64_t oracle_cosine_scratch(const int64_t* segs, int32_t nseg) {
  int64_t m = 0;
  for (int32_t t = 0; t < nseg; ++t) {
    const int64_t O = segs[4 * t + 1], I = segs[4 * t + 2], K = segs[4 * t + 3];
    const int64_t need = O * K + 2 * K + I * K;
    if (need > m) m = need;
  }
  return m;
}

/* threads: torch's intra-op thread count of the reference's process (1..1024) */
float oracle_cosine_model_t(const float* a, const float* b, const int64_t* segs, int32_t nseg, int32_t threads,
                            float* scratch, float* per_tensor) {
  if (threads < 1 || threads > MAX_THREADS) return NAN;
  float avg = 0.f;
  for (int32_t t = 0; t < nseg; ++t) {
    const int64_t off = segs[4 * t], O = segs[4 * t + 1], I = segs[4 * t + 2], K = segs[4 * t + 3];
    const float m = cos_tensor(a + off, b + off, O, I, K, threads, scratch);
    if (per_tensor) per_tensor[t] = m;
    avg = t == 0 ? 0.f + m : avg + m;  /* python 0 + tensor, then in-place += */
  }
  return avg / (float)nseg;
}

float oracle_cosine_model(const float* a, const float* b, const int64_t* segs, int32_t nseg, float* scratch,
                          float* per_tensor) {
  return oracle_cosine_model_t(a, b, segs, nseg, 1, scratch, per_tensor);
}

/* Debug view: every tensor's per-output values s (concatenated, tensor order) and means. */
void oracle_cosine_outputs(const float* a, const float* b, const int64_t* segs, int32_t nseg, float* scratch,
                           float* s_out, float* means) {
  int64_t pos = 0;
  for (int32_t t = 0; t < nseg; ++t) {
    const int64_t off = segs[4 * t], O = segs[4 * t + 1], I = segs[4 * t + 2], K = segs[4 * t + 3];
    means[t] = cos_tensor(a + off, b + off, O, I, K, 1, scratch);
    memcpy(s_out + pos, scratch, sizeof(float) * O * K);
    pos += O * K;
  }
}
