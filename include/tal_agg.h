/*
 * tal_agg.h — C-ABI of the MI355X (gfx950) neighbor-model aggregation library.
 *
 * The reference (msakarvadia/topology_aware_learning) is pure Python: its hot path is the
 * inner loop shared by every aggregation app,
 *
 *     src/decentralized_client.py:399-413   (weighted_module_avg)
 *     src/decentralized_client.py:433-446   (unweighted_module_avg)
 *     src/decentralized_client.py:535-549   (sim_centrality_module_avg)
 *     src/decentralized_client.py:597-611   (centrality_module_avg)
 *     src/decentralized_client.py:630-645   (scale_agg)
 *
 *         avg[name]  = w_0 * clone(sd_0[name])            # fp32(w) * x, rounded to fp32
 *         avg[name] += w_i * clone(sd_i[name])  (i=1..M-1) # separate fp32 add, no FMA
 *         model.load_state_dict(avg)                       # int64 buffers: trunc toward 0
 *
 * and its caller, the round driver src/decentralized_app.py:605-641, which submits one such
 * call per simulated device.  The reference binds no native code, so there is no FFI to
 * mirror; the entry points below are what a ctypes binding of that loop would call (see
 * INTEGRATION.md).  They replace the torch CPU ops clone/mul/add_/copy_ on that path.
 *
 * Conventions
 *   - every function returns 0 (TAL_OK) or a TAL_ERR_* code; tal_last_error() gives a
 *     thread-local message for the last failure on the calling thread.
 *   - all data pointers are DEVICE pointers owned by the caller; host arrays are named *_host.
 *   - `stream` is a hipStream_t (NULL = the default stream); calls are stream-ordered and
 *     never synchronize the device; the library allocates no device memory except 512 B of
 *     item counters per (device, stream) that tal_agg_round_reg launches on (made on first use,
 *     kept for the process: launches on different streams never share counters).
 *   - weights arrive as float64 (Python floats / numpy float64 in the reference) and are
 *     rounded to fp32 exactly as torch does for `python_float * fp32_tensor`.
 *   - mode: TAL_MODE_EXACT reproduces the reference bit for bit (ordered i=0..M-1,
 *     separate fp32 multiply and add); TAL_MODE_FMA fuses them (tolerance M*2^-24*sum|w x|).
 */
#ifndef TAL_AGG_H
#define TAL_AGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TAL_OK 0
#define TAL_ERR_INVALID 1   /* bad argument (null pointer, size, alias, plan mismatch) */
#define TAL_ERR_HIP 2       /* HIP runtime error (launch / attribute) */
#define TAL_ERR_CAPACITY 3  /* plan does not fit (a row has more sources than the LDS tile) */
#define TAL_ERR_COMM 4      /* RCCL error (multi-GPU halo exchange) */

#define TAL_MODE_FMA 0
#define TAL_MODE_EXACT 1

/* Thread-local text of the last error on this thread ("" if none). */
const char* tal_last_error(void);
/* ABI version (bumped on any signature change). */
int32_t tal_abi_version(void);

/* ---- K1: one aggregation call over M flattened operands --------------------------------
 * out[e] = sum_{i<M} fp32(w_host[i]) * x[i][e]   for e < n  (fp32 segment)
 * Replaces decentralized_client.py:399-411 (+ the fp32 part of load_state_dict :413).
 * x_host: host array of M device pointers.  out may alias any x[i] (the reference's
 * aggregating client is itself the last operand, decentralized_app.py:625).  Any M >= 1:
 * past 256 operands further passes continue the ordered chain from out, or - when an operand
 * past the first 256 aliases out - from a stream-ordered fp32 scratch (as tal_agg_bf16).  */
int32_t tal_agg_f32(const float* const* x_host, const double* w_host, int32_t m,
                    float* out, int64_t n, int32_t mode, void* stream);

/* int64 buffers (num_batches_tracked): torch promotes `python_float * int64_tensor` to
 * fp32, accumulates in fp32 and load_state_dict's copy_ truncates toward zero
 * (decentralized_client.py:407-413).  NaN / out-of-range results give INT64_MIN, as the
 * x86 cvttss2si the reference runs on does.  Any m >= 1 (past 256 operands: passes through
 * an fp32 scratch, as tal_agg_bf16); out may alias any x[i]. */
int32_t tal_agg_i64(const int64_t* const* x_host, const double* w_host, int32_t m,
                    int64_t* out, int64_t n, void* stream);

/* One call over a whole model (fp32 + int64 segments) in ONE launch: the fp32 segment as
 * tal_agg_f32 and the int64 segment as tal_agg_i64, the same arithmetic bit for bit, but the
 * per-call path's vector, n % 4 tail and int64 launches fused (decentralized_client.py:406-413
 * over every state_dict entry of a ResNet: the num_batches_tracked counters ride along).
 * xi_host may be NULL when n_i == 0.  Fused when m <= 64, n_i <= 65536 and every fp32
 * pointer is 16-byte aligned; otherwise the two segment calls above run instead. */
int32_t tal_agg_model_f32(const float* const* x_host, const int64_t* const* xi_host,
                          const double* w_host, int32_t m, float* out, int64_t n,
                          int64_t* out_i, int64_t n_i, int32_t mode, void* stream);

/* bf16 buffers (uint16_t bit patterns; bf16 models).  mode TAL_MODE_EXACT: the reference's
 * own ops on bf16 tensors (decentralized_client.py:407-411 - `w * clone(v)` and `+=` each
 * round their fp32 result to bf16, nearest even), bit-identical to it; TAL_MODE_FMA: fp32
 * fused accumulation rounded to bf16 once (|error| <= 2^-8 |result| + M 2^-24 sum|w x|).  NaN
 * results are stored as 0xFFFF (torch's vectorized conversion).  Any m >= 1: past 256
 * operands the ordered chain runs in passes of 256 through an fp32 scratch of n elements,
 * allocated and freed in stream order (hipMallocAsync), carrying the same running value the
 * one-pass kernel keeps in registers; out may alias any x[i]. */
int32_t tal_agg_bf16(const uint16_t* const* x_host, const double* w_host, int32_t m,
                     uint16_t* out, int64_t n, int32_t mode, void* stream);

/* ---- K3: one whole aggregation round over a device-resident model pool -----------------
 * Row r of the round computes pool_out[out_row[r]][e] = sum_k fp32(w[k]) * pool_in[col[k]][e]
 * over k = row_ptr[r] .. row_ptr[r+1]-1 in that (reference) order, for e < n.  All rows read
 * the pool as it was before the round ("snapshot" semantics).
 *
 * The host first turns the CSR into a tile plan (rows grouped so that each group's distinct
 * sources fit one LDS tile); the plan is a flat int32 blob the caller copies to the device.
 */
typedef struct tal_round_plan_info {
  int32_t rows;          /* rows in the round */
  int32_t nnz;           /* operands over all rows */
  int32_t n_groups;      /* row groups */
  int32_t total_src;     /* staged sources summed over groups */
  int32_t max_src;       /* largest group source count (sizes the LDS tile) */
  int32_t max_rows;      /* largest group row count */
  int32_t max_nnz;       /* largest group operand count */
  int32_t c4;            /* float4 columns per staged source row per tile (16, 32, 64 or 128) */
  int32_t lds_bytes;     /* LDS per workgroup the round kernel will request */
  /* offsets (in int32 words) of the plan's arrays inside the blob */
  int32_t off_grp_row_ptr;  /* [n_groups+1] */
  int32_t off_grp_src_ptr;  /* [n_groups+1] */
  int32_t off_src_row;      /* [total_src]  pool_in row of each staged source */
  int32_t off_row_ptr;      /* [rows+1] */
  int32_t off_op_slot;      /* [nnz] staged-source slot of each operand (within its group) */
  int32_t off_op_w;         /* [nnz] fp32 weight bits */
  int32_t off_out_row;      /* [rows] pool_out row of each row */
  int32_t words;            /* total int32 words of the blob */
  /* dense row-block form (dense_rb > 0): a wavefront computes dense_rb rows per pass over its
   * group's staged sources, each LDS read serving every row that uses that source.  Valid
   * when every row lists its operands as sources in ascending order followed by the row's own
   * (reference order: sorted neighbors, then self). */
  int32_t dense_rb;         /* rows per block (0 = sparse form only) */
  int32_t n_blocks;         /* row blocks over all groups */
  int32_t off_grp_blk_ptr;  /* [n_groups+1] first block of each group */
  int32_t off_blk_tab;      /* [n_blocks] word offset of each block's table inside the blob */
  int32_t off_dense;        /* start of the tables (32-B aligned): per block {n_used, 7 pad words,
                             * slot[n_used] (staged slots
                             * the block's rows use, ascending), mask[n_used] (bit r = row r of
                             * the block uses that slot, own model excluded; bit 31 set
                             * when all those rows have the same fp32 weight, which then
                             * fills every w slot: one product w*x serves them all),
                             * w[n_used][dense_rb] fp32}; n_used padded to a multiple of 4
                             * with mask-0 entries */
  int32_t dense_reads;      /* LDS operand reads per column in the dense form (sparse: nnz) */
  /* streamed form (stream_cs > 0, built by tal_round_plan_build_stream): a workgroup of W
   * wavefronts (W = 8 or 16) owns a group of at most 8*W rows (one dense row block per
   * wavefront) and streams the group's staged sources through a ring of LDS chunks of
   * stream_cs = 2*W sources x 64 float4 columns (two 1 KiB global->LDS DMAs per wavefront per
   * chunk), so a group's source count is not bounded by LDS.  Each block's table lists its
   * entries chunk by chunk (including the rows' own models, flagged in mask bits 8..15), every
   * chunk's run padded to a multiple of 4 with mask-0 entries. */
  int32_t stream_cs;        /* sources per chunk (16 or 32); 0 = LDS-resident groups */
  /* narrow form (c4 16 / 32): each row's operands as (slot * c4, fp32 weight bits) pairs - its
   * first operand, then the rest padded to a multiple of 4 with (max_src * c4, 1.0f) pairs that
   * read a tile of -0.0 the kernel keeps in LDS slot max_src: fl(1 * -0) = -0 and x + -0 == x
   * for every x, so padding is an exact identity.  Rows of a group are ordered by operand count
   * (descending) so that the 64 / c4 rows a wavefront computes together have similar counts. */
  int32_t off_nrow_ptr;     /* [rows+1] pair offset of each row */
  int32_t off_npairs;       /* [npairs][2] int32 */
  int32_t npairs;           /* pairs over all rows (padded) */
  int32_t max_npairs;       /* largest group pair count */
  /* narrow_roww = 1 when every row's operands share one fp32 weight (the unweighted strategy,
   * scale_agg): the pairs are replaced by 16-bit slots (slot * c4, two per int32 word), each
   * row's run padded to a multiple of 4 with a zero-tile slot (slot ns: a -0.0 tile for a
   * row weight with the sign bit clear, slot ns + 1: +0.0 otherwise, so fl(w * 0) = -0 exactly),
   * the accumulator starts at -0.0 (-0 + y == y for every y), and the row weights are in
   * off_nrow_w.  off_nrow_ptr then counts slots; npairs counts slots. */
  int32_t narrow_roww;
  int32_t off_nrow_w;       /* [rows] fp32 weight bits (narrow_roww) */
  int32_t scalar_lds_bytes; /* LDS of the staged scalar tail kernel (the largest group; its
                             * tiles are c4 float4 wide, 16 for narrow plans) */
  /* broadcast form (narrow_bcast > 0, built by tal_round_plan_build_bcast; c4 16 / 32): the
   * LDS holds only the group's data tile and one -0.0 tile (slot max_src).  Each wavefront of
   * a workgroup runs a fixed program over the group's passes (4 rows computed together, 16
   * lanes each - one float4 chunk per lane at c4 = 16, chunks cl and cl + 16 at c4 = 32 - rows
   * ordered by operand count, descending), kept in VGPRs for the whole launch: a record
   * is 64 lanes x {LDS byte offset of the operand's tile column 0, fp32 weight bits} holding
   * operands 16c .. 16c+15 of every row of the pass (lane L: row L / 16, operand 16c + L % 16;
   * past a row's count: the -0.0 tile with weight 1.0, an exact identity); the kernel hands
   * operand u to the row's lanes by a DPP row broadcast from lane u, so no per-operand plan
   * read touches LDS.  Program of wavefront w of group g at word off_bc_prog[g * narrow_bcast +
   * w] (even): {n_rec, n_pass, data offset (words from the program, even), 5 x 0},
   * bc_rec_max descriptors {operands in the record (1..16) | last of its pass << 8 | pass << 16},
   * 4 output rows per pass (-1: none), then the n_rec records (128 words each). */
  int32_t narrow_bcast;     /* wavefronts per workgroup (8, 12 or 16); 0 = not this form */
  int32_t bc_rec_max;       /* records per wavefront (128 / narrow_bcast) */
  int32_t off_bc_prog;      /* [n_groups * narrow_bcast] program offsets */
  int32_t bc_records;       /* records over all programs */
  int32_t bc_wg_per_cu;     /* resident workgroups per CU the launch sizes registers for (1: 128
                             * VGPRs at 1024 threads, deeper read pipelining; 2: two groups' tiles
                             * overlap one's staging with the other's arithmetic) */
} tal_round_plan_info;

/* Blob size in int32 words of the sparse or narrow form for `rows` rows / `nnz` operands (an upper
 * bound); the dense tables come on top — tal_round_plan_build reports the exact need. */
int64_t tal_round_plan_words(int32_t rows, int64_t nnz);

/* Build the plan on the host.  row_ptr_host[rows+1], col_host[nnz], w_host[nnz] (float64),
 * out_row_host[rows].  c4 in {16,32,64,128} (16 / 32: narrow tiles, a wavefront computes 64/c4
 * rows at once, sparse form only); lds_bytes = LDS budget per workgroup (staged tile
 * 16*c4 B per source plus the plan slice the narrow and scalar kernels stage).  Rows keep their order; consecutive rows
 * share a group while the union of their sources fits; a group's staged sources are in
 * ascending pool row order.  dense_rb: 0 = sparse form, 8 = dense row blocks of 8 (falls back
 * to sparse if a row is not in reference order), -1 = dense when it cuts the LDS operand reads
 * to at most a quarter (one read serves >= 4 operands: cliques).  Returns
 * TAL_ERR_CAPACITY if one row alone has more distinct sources than fit, or if plan_capacity_words
 * is too small (info->words then holds the size needed). */
int32_t tal_round_plan_build(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                             const double* w_host, const int32_t* out_row_host, int32_t c4,
                             int32_t lds_bytes, int32_t dense_rb, int32_t* plan_host,
                             int64_t plan_capacity_words, tal_round_plan_info* info);

/* Broadcast-form narrow plan (see narrow_bcast above): as tal_round_plan_build at c4 16 / 32,
 * with waves (8, 12 or 16) wavefronts per workgroup and wg_per_cu (1 or 2) resident workgroups per CU
 * (2 caps lds_bytes at 80 KiB; a c4 = 32 group of more than 128 sources at 1024 threads
 * launches only with wg_per_cu 1); a group also needs every wavefront's program
 * to fit 128 / waves records (TAL_ERR_CAPACITY for a row no group can take).  Per-operand
 * weights cost no LDS reads in this form (the centrality strategies on graphs whose degrees
 * differ: decentralized_client.py:572-611). */
int32_t tal_round_plan_build_bcast(int32_t rows, const int32_t* row_ptr_host, const int32_t* col_host,
                                   const double* w_host, const int32_t* out_row_host, int32_t c4,
                                   int32_t lds_bytes, int32_t waves, int32_t wg_per_cu, int32_t* plan_host,
                                   int64_t plan_capacity_words, tal_round_plan_info* info);

/* The broadcast form's staging limit: the most float4 staging loads per column tile (sources x
 * c4) one group of a (c4, waves, wg_per_cu) broadcast plan may need - the planner caps groups
 * at it and the launcher stages up to it (one table in the library for both).  -1 for a form
 * that does not exist. */
int64_t tal_round_bcast_max_loads(int32_t c4, int32_t waves, int32_t wg_per_cu);

/* Streamed plan (see stream_cs above).  Rows keep their order; consecutive rows share a group
 * while the group has at most max_group_rows rows (<= 128) and, if max_group_src > 0, at
 * most max_group_src distinct sources.  Every row must list its operands in reference order
 * (ascending distinct sources, then its own model, which does not occur before): otherwise
 * TAL_ERR_INVALID.  c4 is 64.  TAL_ERR_CAPACITY as for tal_round_plan_build. */
int32_t tal_round_plan_build_stream(int32_t rows, const int32_t* row_ptr_host,
                                    const int32_t* col_host, const double* w_host,
                                    const int32_t* out_row_host, int32_t max_group_rows,
                                    int32_t max_group_src, int32_t* plan_host,
                                    int64_t plan_capacity_words, tal_round_plan_info* info);

/* Execute the round on the fp32 segment (n elements per model; row stride ld_in / ld_out in
 * elements).  plan_dev = the blob copied to the device.  pool_out may equal pool_in only if
 * the plan has a single group (each workgroup stages every source of its tile in LDS before
 * it writes).  16-B aligned pools with ld % 4 == 0 take the float4 path; others the scalar
 * tiled path. */
int32_t tal_agg_round_f32(const float* pool_in, int64_t ld_in, float* pool_out, int64_t ld_out,
                          int64_t n, const int32_t* plan_dev, const tal_round_plan_info* info,
                          int32_t mode, void* stream);

/* The same round on the int64 segment (fp32 accumulate, truncation, as tal_agg_i64). */
int32_t tal_agg_round_i64(const int64_t* pool_in, int64_t ld_in, int64_t* pool_out,
                          int64_t ld_out, int64_t n, const int32_t* plan_dev,
                          const tal_round_plan_info* info, void* stream);

/* Clique rounds (K3c).  Rows of a round that form uniform-weight cliques — m <= 64 sources
 * s_0 < ... < s_{m-1} (pool rows) with one fp32 weight w, and for member i an output row whose
 * operands are, in reference order (decentralized_app.py:625), every other member ascending and
 * then s_i — are computed from one read of each source: the products are shared and each row's
 * in-order chain extends the shared prefix (bitwise the reference in EXACT mode; FMA mode as
 * tal_agg_f32's).  table_dev: n_cliques records of TAL_CLIQUE_WORDS int32
 *   {m, bits of w, n_att, 0, src_row[64], out_row[64], attached[4][12]}
 * (out_row -1: member without an output row) copied to the device.  An attached row (a
 * barbell's bridge node) has its own weight v and operands = members selected by a 64-bit
 * mask + at most two other rows + its own model, in reference order:
 *   {out_row, bits of v, mask lo, mask hi, self member index or -1, self pool row or -1,
 *    n_ext, ext_row[2], ext_pos[2] (members with a smaller pool row), 0}.
 * The other rows of the round run through a regular plan (a second call).  Out of place only; pools 8-B aligned with even ld.  mmax = the largest m (16, 32 or
 * 64 registers of products per lane). */
#define TAL_CLIQUE_WORDS 180
int32_t tal_agg_round_clique_f32(const float* pool_in, int64_t ld_in, float* pool_out, int64_t ld_out,
                                 int64_t n, const int32_t* table_dev, int32_t n_cliques, int32_t mmax,
                                 int32_t mode, void* stream);

/* The same round on bf16 pools (arithmetic as tal_agg_bf16, per mode).  Takes sparse plans
 * (c4 64 / 128, dense_rb 0) and narrow plans (c4 16 / 32); TAL_ERR_INVALID for dense or
 * streamed plans.  A staged tile holds the sources' values as fp32 (c4 float4 per source). */
int32_t tal_agg_round_bf16(const uint16_t* pool_in, int64_t ld_in, uint16_t* pool_out,
                           int64_t ld_out, int64_t n, const int32_t* plan_dev,
                           const tal_round_plan_info* info, int32_t mode, void* stream);

/* ---- K3r: a round over register-resident source groups ----------------------------------
 * Community graphs (BASELINE config 5's stochastic block model): the rows are grouped so that
 * each group reads <= 64 distinct sources; one wavefront loads a group's sources for a 128-
 * element piece of the columns into VGPRs and emits every row of the group for that piece, an
 * operand read from the registers by the VGPR index mode (no LDS, no barrier).  Same results
 * as tal_agg_round_f32 (EXACT: bitwise the reference; FMA: bitwise K1-FMA); bf16 pools (bf16 !=
 * 0) in FMA mode only.  Out of place (pool_in != pool_out).  Pools 2-element aligned, even ld
 * >= n rounded up to even; table_dev 64-B aligned.  table_dev (int32): n_groups records {first
 * source, sources, first pair, pairs}; at off_src the source pool rows, every group's list
 * padded to 16 x NB entries, NB = ceil(max_src / 16) (src_off_dev: int64 byte offsets of those
 * entries, row x ld_in x element size); at off_pairs (a multiple of 4) row-pair records {out
 * row A, out row B or -1, trips, byte offset from table_dev of the pair's first trip record}, a
 * group's pairs consecutive; at off_rec (a multiple of 16) trip records of 16 dwords {A's four
 * operand register offsets (2 x the source's slot in the group), B's four, A's four fp32
 * weights, B's four}, a row padded to its pair's trips with the neutral operand (offset 32 x
 * NB, weight +0.0: a -0.0 product that leaves the sum unchanged), followed by one record of
 * padding.  max_src = the largest group's sources (<= 64).  Replaces
 * decentralized_client.py:399-413 for every row of the round at once (snapshot semantics, as
 * tal_agg_round_f32). */
int32_t tal_agg_round_reg(const void* pool_in, int64_t ld_in, void* pool_out, int64_t ld_out,
                          int64_t n, int32_t bf16, const int32_t* table_dev, const int64_t* src_off_dev,
                          int32_t n_groups, int32_t off_src, int32_t off_pairs, int32_t off_rec,
                          int32_t max_src, int32_t mode, void* stream);

/* ---- K2: cosine similarity of two models' parameters, bit for bit -------------------------
 * Reference: cosine_similarity, decentralized_client.py:661-681: for each parameter tensor
 * viewed as [A, I, B] (dim 1 = the reduced dim; 1-D tensors are unsqueezed to [n, 1]),
 * nn.CosineSimilarity(dim=1, eps=1e-6) gives A*B values whose mean is taken; the result is
 * the average of those means over tensors.  Every fp32 operation is the reference's, in the
 * order of the torch CPU kernels it runs on (vector_norm, the cascade sum, sum / numel; see
 * oracle/cosine_oracle.c, pinned bitwise by the reference's own values, near-ties included):
 * the result is the reference's fp32 value, so sim_centrality_module_avg's least-similar
 * neighbor (:511-516) is the reference's.  A tensor's mean over A*B >= 32768 outputs is, in
 * torch, a two-pass parallel sum whose order depends on the process's intra-op thread count T
 * (at::parallel_for chunks of ceil(n / min(T, ceil(n / 32768))) elements, then a T-entry
 * buffer summed); the plan carries T (tal_cosine_plan_set_threads, default 1 = serial), so the
 * result is torch's for that T.
 *
 * seg_host: 4*n_seg int64 {offset (elements into the flat parameter arena), A, I, B}.
 * The plan (int64 words, tal_cosine_plan_words; copied to the device by the caller, and the
 * host copy passed too) = {n_seg, n_outputs, threads, streamed chunks}, per tensor {offset, A,
 * I, B, first output, kind, outputs per chunk}, per workgroup chunk {tensor, first output, count,
 * streamed}.  Column tensors with B < 32 (3 x 3 convolutions) run streamed (ABI 25): every
 * model's norms in one launch, then each pair's products, both walking i in 16-element steps
 * through LDS; the others one thread (or 8 lanes) per output.
 *
 * a_ptrs_host / b_ptrs_host: n_pairs device pointers; pair j compares model a_j with b_j
 * (flat fp32 parameter arenas of the same layout).  scratch: device buffer of at least
 * tal_cosine_scratch_bytes(plan_host, n_pairs) bytes (ABI 25: 4 (3 n_outputs + n_seg) per pair
 * of a launch of up to 32 pairs).  out_dev: n_pairs fp32 results. */
int64_t tal_cosine_plan_words(const int64_t* seg_host, int32_t n_seg);
int32_t tal_cosine_plan_build(const int64_t* seg_host, int32_t n_seg, int64_t* plan_host,
                              int64_t plan_capacity_words, int32_t* n_chunks);
/* Set a built plan's thread word (1..1024; the calling process's torch.get_num_threads()). */
int32_t tal_cosine_plan_set_threads(int64_t* plan_host, int32_t threads);
int64_t tal_cosine_scratch_bytes(const int64_t* plan_host, int32_t n_pairs);
int32_t tal_cosine_params(const float* const* a_ptrs_host, const float* const* b_ptrs_host,
                          int32_t n_pairs, const int64_t* plan_dev, const int64_t* plan_host,
                          int32_t n_chunks, void* scratch, float* out_dev, void* stream);

/* ---- FedProx proximal term ------------------------------------------------
 * Reference: local_train, tasks.py:277-286: loss += (prox_coeff / 2) * sum_t sum_p
 * ||w_p - wt_p||_2 over the neighbors t and the parameter tensors p.  Here the parameters are
 * segments of flat fp32 rows (a device ModelPool row per model).
 *
 * seg_host: 2*n_seg int64 {offset, length} of each parameter in the flat row.  The plan
 * (int64, copied to the device by the caller) cuts them into workgroup chunks.
 * tal_prox_norms: norms_out[t*n_seg + p] = ||w_p - wt_p||_2 (sums of squares per chunk in
 * fp32, combined in double in a fixed order: deterministic); scratch >=
 * tal_prox_scratch_bytes(n_chunks, k).
 * tal_prox_grad: gw = s * sum_t (w - wt) / ||w - wt||_p and, for each non-null gwt_host[t],
 * gwt[t] = -s * (w - wt) / ||w - wt||_p, with 0 where a norm is 0 (torch's norm backward);
 * s = *scale_dev (the upstream gradient, read on the device).  Only the parameter segments
 * of gw / gwt are written. */
int64_t tal_prox_plan_words(const int64_t* seg_host, int32_t n_seg);
int32_t tal_prox_plan_build(const int64_t* seg_host, int32_t n_seg, int64_t* plan_host,
                            int64_t plan_capacity_words, int32_t* n_chunks);
int64_t tal_prox_scratch_bytes(int32_t n_chunks, int32_t k);
int32_t tal_prox_norms(const float* w, const float* const* wt_host, int32_t k,
                       const int64_t* plan_dev, int32_t n_chunks, int32_t n_seg, void* scratch,
                       float* norms_out, void* stream);
int32_t tal_prox_grad(const float* w, const float* const* wt_host, int32_t k,
                      const int64_t* plan_dev, int32_t n_chunks, int32_t n_seg,
                      const float* norms, const float* scale_dev, float* gw,
                      float* const* gwt_host, void* stream);

/* ---- Host reduction: processes that see no GPU ------------------------------------------
 * BASELINE config 1 runs the reference's driver with CPU models and no GPU
 * (decentralized_client.py:399-413 on CPU tensors).  These compute the same arithmetic as
 * tal_agg_f32 / tal_agg_i64 / tal_agg_bf16 (EXACT: bitwise the reference; FMA as documented
 * there) on HOST pointers, elementwise in operand order, on up to 16 host threads.  out may
 * alias any x[i].  The package calls them only when torch sees no GPU; with a GPU visible
 * every aggregation runs the kernels above. */
int32_t tal_host_agg_f32(const float* const* x_host, const double* w_host, int32_t m, float* out,
                         int64_t n, int32_t mode);
int32_t tal_host_agg_i64(const int64_t* const* x_host, const double* w_host, int32_t m, int64_t* out,
                         int64_t n);
int32_t tal_host_agg_bf16(const uint16_t* const* x_host, const double* w_host, int32_t m, uint16_t* out,
                          int64_t n, int32_t mode);

/* K2's cosine similarity on HOST pointers (replaces the reference's cosine_similarity,
 * src/decentralized_client.py:661-681, where it runs: on CPU tensors inside
 * sim_centrality_module_avg, :482-490, in a process without a GPU).  out[j] = cosine of the
 * flat fp32 parameter rows a_host[j] / b_host[j] under a plan from tal_cosine_plan_build (its
 * thread word set by tal_cosine_plan_set_threads): the same fp32 operations in the same order
 * as tal_cosine_params, i.e. torch's CPU order, bit for bit.  Up to 16 host threads. */
int32_t tal_host_cosine(const float* const* a_host, const float* const* b_host, int32_t n_pairs,
                        const int64_t* plan_host, float* out);

/* ---- Synthetic pool rows (test / benchmark inputs) --------------------------
 * Not a reference interface: the reference trains its models; the benchmark and the full-size
 * parity tests need seeded models whose outputs the reference-generated sha256 fixtures pin
 * (tests/golden/full_round_c{3,4,5}_*.json).  Fills n_rows rows (pitch ld elements) of one pool
 * segment with synth.py's counter generator: element at generator position p of the row seeded
 * s is u = splitmix64(p ^ (s & 0xFFFFFFFF) << 40) turned into fp32 (dtype 0: sign bit 31,
 * exponent 121 + bits 23..25, mantissa bits 0..22; |v| + 0.5 in the running_var ranges), bf16
 * (dtype 1: that fp32 value rounded to nearest even) or int64 (dtype 2: u % hi).
 * table (int64, on the device; the host copy passed too): {n_rows, n, n_runs, n_rv, hi, 0, 0, 0},
 * seeds[n_rows], runs[n_runs] {generator position, first column, length} tiling columns
 * [0, n) in order, running_var ranges[n_rv] {first column, length} ascending (dtype 0 only).
 * One launch for the whole segment (the torch form took ~20 element-wise launches per 32 M
 * elements per row). */
int32_t tal_fill_counter(void* seg, int64_t ld, int32_t dtype, const int64_t* table_dev,
                         const int64_t* table_host, void* stream);

/* ---- Multi-GPU halo exchange (SURVEY §8(b) tal_halo_exchange, §8(e)) ---------------------
 * Reference: the models that cross workers are shipped by Parsl as Python objects
 * (decentralized_app.py:627-629, parsl_setup.py:191-203).  Sharded one process per GPU, each
 * rank needs the neighbor models other ranks own: per ordered pair (g -> h) the unique set of
 * g's rows that h's rows reference, sent once.  One RCCL communicator per process, made from a
 * unique id that rank 0 creates and the caller broadcasts (any channel: torch.distributed, a
 * file, MPI); tal_comm_init selects `device` for the communicator and restores the caller's
 * current device.
 *
 * tal_halo_pack gathers rows rows_dev[0..n_rows) (device int32, rows < pool_rows; others are
 * skipped) of a pool segment (row pitch ld_bytes) into buf, row_bytes each, back to back: the
 * message for one peer.  tal_halo_exchange posts in one RCCL group on `stream` a send of
 * send_bytes[p] bytes from send_bufs[p] and a receive of recv_bytes[p] bytes into recv_bufs[p]
 * for every peer p in [0, world) with a non-zero count (p == own rank: a local copy through
 * RCCL).  A peer's rows arrive back to back, so a contiguous block of ghost rows of the
 * receiving pool (its halo rows are grouped by owner) is a valid receive buffer and the round
 * kernels read it in place.  world must equal the communicator's size. */
#define TAL_COMM_ID_BYTES 128
int32_t tal_comm_unique_id(void* id_out);
int32_t tal_comm_init(void** comm_out, int32_t world, int32_t rank, const void* id, int32_t device);
int32_t tal_comm_destroy(void* comm);
int32_t tal_halo_pack(const void* pool, int64_t ld_bytes, int64_t pool_rows, const int32_t* rows_dev,
                      int32_t n_rows, int64_t row_bytes, void* buf, void* stream);
int32_t tal_halo_exchange(void* comm, int32_t world, const void* const* send_bufs,
                          const int64_t* send_bytes, void* const* recv_bufs,
                          const int64_t* recv_bytes, void* stream);

/* One process driving several GPUs (TAL_GPUS: the reference's single coordinator process,
 * decentralized_app.py:605-641 / parsl_setup.py:75-78, with its clients' models spread over the
 * node's GPUs).  tal_comm_init_local makes n communicators together, rank r on devices[r]
 * (ncclCommInitAll; distinct devices).  tal_halo_exchange_local posts, in ONE RCCL group (a thread
 * driving several ranks must group them), for every local rank r and peer p with a non-zero count:
 * a send of send_bytes[r n + p] bytes from send_bufs[r n + p] and a receive of recv_bytes[r n + p]
 * bytes into recv_bufs[r n + p], on rank r's stream streams[r].  The buffers obey
 * tal_halo_exchange's rules (a contiguous block of ghost rows is a valid receive buffer). */
int32_t tal_comm_init_local(void** comms_out, int32_t n, const int32_t* devices);
int32_t tal_halo_exchange_local(void* const* comms, int32_t n, const void* const* send_bufs,
                                const int64_t* send_bytes, void* const* recv_bufs,
                                const int64_t* recv_bytes, void* const* streams);

#ifdef __cplusplus
}
#endif

#endif /* TAL_AGG_H */
