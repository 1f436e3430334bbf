/*
 * oracle/agg_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Plain-C restatement of the reference's aggregation arithmetic, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg to check the HIP library.
 * Pinned against golden vectors generated from the reference itself
 * (tests/golden/make_golden.py); see tests/test_oracle_golden.py.
 *
 * Reference (msakarvadia/topology_aware_learning @ 2025-06-14):
 *   src/decentralized_client.py:399-413 (and the identical loops :433-446, :535-549,
 *   :597-611, :630-645):
 *       for i, client in enumerate(neighbor_futures):
 *           for name, value in model.state_dict().items():
 *               partial = w * torch.clone(value)       # python float -> fp32, one rounding
 *               avg[name] = partial  or  avg[name] += partial   # one fp32 add, no FMA
 *       client_future[1].model.load_state_dict(avg)    # int64 buffers: fp32 -> trunc
 *   Per element, in operand order i = 0..M-1:
 *       acc = fl32(fl32(w_0) * x_0);  acc = fl32(acc + fl32(fl32(w_i) * x_i))
 *   int64 operands are converted to fp32 (round to nearest even) before the multiply
 *   (torch type promotion: float scalar * int64 tensor -> default dtype fp32) and the final
 *   copy_ into the int64 buffer truncates toward zero (x86 cvttss2si: NaN/overflow ->
 *   INT64_MIN).
 *
 * Built with gcc -O2 -ffp-contract=off (x86-64 SSE: every float op rounds to fp32).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int64_t trunc_i64(float v) {
  if (!(v >= -9.2233720368547758e18f && v < 9.2233720368547758e18f)) return INT64_MIN;
  return (int64_t)v;
}

/* One aggregation call: decentralized_client.py:399-413. */
void oracle_agg_f32(const float* const* x, const double* w, int32_t m, float* out, int64_t n) {
  for (int64_t e = 0; e < n; ++e) {
    float acc = (float)w[0] * x[0][e];
    for (int32_t i = 1; i < m; ++i) {
      float p = (float)w[i] * x[i][e];
      acc = acc + p;
    }
    out[e] = acc;
  }
}

/* int64 buffers of the same call (num_batches_tracked): :407-413. */
void oracle_agg_i64(const int64_t* const* x, const double* w, int32_t m, int64_t* out,
                    int64_t n) {
  for (int64_t e = 0; e < n; ++e) {
    float acc = (float)w[0] * (float)x[0][e];
    for (int32_t i = 1; i < m; ++i) {
      float p = (float)w[i] * (float)x[i][e];
      acc = acc + p;
    }
    out[e] = trunc_i64(acc);
  }
}

/* A whole round with snapshot semantics: every row reads pool_in as it was before the round
 * (decentralized_app.py:605-641 with the aggregations' inputs taken from the round's train
 * outputs).  Row r: out_row[r] <- sum over k in [row_ptr[r], row_ptr[r+1])
 * of w[k] * pool_in[col[k]], in k order.  pool_out must not alias pool_in. */
void oracle_round_f32(const float* pool_in, int64_t ld_in, float* pool_out, int64_t ld_out,
                      int64_t n, int32_t rows, const int32_t* row_ptr, const int32_t* col,
                      const double* w, const int32_t* out_row) {
  for (int32_t r = 0; r < rows; ++r) {
    float* o = pool_out + (int64_t)out_row[r] * ld_out;
    for (int64_t e = 0; e < n; ++e) {
      int32_t k = row_ptr[r];
      float acc = (float)w[k] * pool_in[(int64_t)col[k] * ld_in + e];
      for (++k; k < row_ptr[r + 1]; ++k) {
        float p = (float)w[k] * pool_in[(int64_t)col[k] * ld_in + e];
        acc = acc + p;
      }
      o[e] = acc;
    }
  }
}

void oracle_round_i64(const int64_t* pool_in, int64_t ld_in, int64_t* pool_out, int64_t ld_out,
                      int64_t n, int32_t rows, const int32_t* row_ptr, const int32_t* col,
                      const double* w, const int32_t* out_row) {
  for (int32_t r = 0; r < rows; ++r) {
    int64_t* o = pool_out + (int64_t)out_row[r] * ld_out;
    for (int64_t e = 0; e < n; ++e) {
      int32_t k = row_ptr[r];
      float acc = (float)w[k] * (float)pool_in[(int64_t)col[k] * ld_in + e];
      for (++k; k < row_ptr[r + 1]; ++k) {
        float p = (float)w[k] * (float)pool_in[(int64_t)col[k] * ld_in + e];
        acc = acc + p;
      }
      o[e] = trunc_i64(acc);
    }
  }
}

/* ---- bf16 (uint16_t bit patterns) ------------------------------------------------------
 * The reference's loop run on bf16 state_dicts (a bf16 model): `w * clone(v)` computes the
 * product in fp32 (torch's opmath type) and rounds it to bf16; `avg += partial` adds in fp32 and
 * rounds to bf16 (c10::BFloat16 round_to_nearest_even; NaN is written as 0xFFFF by the
 * vectorized CPU conversion every full-size tensor goes through).  exact = 0 restates the
 * library's FMA mode instead: fp32 accumulation with fused multiply-adds, one rounding. */
static float bf16_to_f32(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static uint16_t f32_to_bf16(float f) {
  if (f != f) return 0xFFFF;
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

static float rbf(float f) { return bf16_to_f32(f32_to_bf16(f)); }

static uint16_t bf16_chain(const uint16_t* const* xs, const double* w, int32_t m, int64_t e,
                           int32_t exact) {
  float acc = 0.f;
  for (int32_t i = 0; i < m; ++i) {
    const float x = bf16_to_f32(xs[i][e]);
    const float wf = (float)w[i];
    if (exact) {
      const float p = rbf(wf * x);
      acc = i == 0 ? p : rbf(acc + p);
    } else {
      acc = i == 0 ? wf * x : fmaf(wf, x, acc);
    }
  }
  return f32_to_bf16(acc);
}

void oracle_agg_bf16(const uint16_t* const* x, const double* w, int32_t m, uint16_t* out, int64_t n,
                     int32_t exact) {
  for (int64_t e = 0; e < n; ++e) out[e] = bf16_chain(x, w, m, e, exact);
}

void oracle_round_bf16(const uint16_t* pool_in, int64_t ld_in, uint16_t* pool_out, int64_t ld_out,
                       int64_t n, int32_t rows, const int32_t* row_ptr, const int32_t* col,
                       const double* w, const int32_t* out_row, int32_t exact) {
  for (int32_t r = 0; r < rows; ++r) {
    const int32_t k0 = row_ptr[r], m = row_ptr[r + 1] - k0;
    const uint16_t** xs = (const uint16_t**)malloc(sizeof(*xs) * (size_t)m);
    for (int32_t i = 0; i < m; ++i) xs[i] = pool_in + (int64_t)col[k0 + i] * ld_in;
    uint16_t* o = pool_out + (int64_t)out_row[r] * ld_out;
    for (int64_t e = 0; e < n; ++e) o[e] = bf16_chain(xs, w + k0, m, e, exact);
    free(xs);
  }
}

/* elementwise conversions for the tests (same rounding as above) */
void oracle_f32_to_bf16(const float* x, uint16_t* out, int64_t n) {
  for (int64_t e = 0; e < n; ++e) out[e] = f32_to_bf16(x[e]);
}
