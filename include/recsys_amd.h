/*
 * recsys_amd.h — C ABI of librecsys_amd.so, the MI355X (gfx950) kernels of the CTR
 * feature-interaction training path of yueshifeng/recommendSystem.
 *
 * Conventions (every entry point):
 *   - `stream` is a hipStream_t passed as void*; the call only enqueues work on it (no
 *     allocation, no host synchronisation), so any sequence of calls can be captured into a
 *     hipGraph by the caller.
 *   - all pointers are device pointers to row-major buffers owned by the caller (the caller
 *     allocates outputs and workspaces; the library never allocates or frees).
 *   - fp32 everywhere ("float"); ids are int64; hashed table rows are int32.
 *   - return value: 0 = OK, -1 = bad argument/shape, -2 = shape not compiled in,
 *     -3 = kernel launch failed.  Callers raise on non-zero (the Python host layer raises the
 *     reference's ValueError messages before launching).
 *
 * The reference is TensorFlow/Keras + tensornet Python; the "FFI" that binds this library is the
 * Python host layer (recommendsystem_amd/_lib.py, ctypes).  Each declaration cites the reference
 * interface it replaces.
 */
#ifndef RECSYS_AMD_H_
#define RECSYS_AMD_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------------------------------
 * H1/H2  Sparse embedding lookup + concat front end.
 * Replaces tn.layers.EmbeddingFeatures(embedding_column(category_column(key, bucket_size),
 * dimension, combiner))(inputs) and the expand + Concatenate(axis=1) that follows:
 *   rank/ctr/base_model.py:203-217, rank/multi_head/multidnn.py:221-238,
 *   staytime/VideoDnn.py:217-244, rough_rank/model.py:89-115, rank/finish/videodnn.py:53-68,
 *   autoint:22-26, rank/multi_head/multidnn.py:25-27,50.
 * Segment s = b*F + f holds ids[offsets[s] .. offsets[s+1]) (offsets == NULL: one id per
 * segment).  row = row_base[f] + H(id) % bucket[f] with H = identity (hash_mode 0) or
 * splitmix64 (1).  out[b*out_ld + f*out_fstride + e] = combiner(rows)[e], combiner 0 = sum,
 * 1 = mean, 2 = sqrtn; empty segment -> 0.  rows_out[k] (nullable) receives the row of ids[k].
 * table == out == NULL (rows_out required): rows only (owner-sharded tables, below).
 * ------------------------------------------------------------------------------------- */
int rs_embedding_lookup_fwd(void* stream, const int64_t* ids, const int32_t* offsets, int64_t B,
                            int F, const int64_t* row_base, const int64_t* bucket, int hash_mode,
                            int combiner, const float* table, int64_t table_rows, int dim,
                            float* out, int64_t out_ld, int64_t out_fstride, int32_t* rows_out);

/* H1 sequence lookup: embedding_column(combiner=None, seq_max_len) -> (emb3d, mask)
 * (staytime/VideoDnn.py:217-244, consumed at :58-68; the DIN keys of din.py at config 4).
 * Sample b's ids are ids[offsets[b] .. offsets[b+1]) (offsets [B+1]); the first T are looked up
 * (row = row_base + H(id) % bucket), out[b*out_ss + t*out_rs + e]; positions t >= n_b are zero,
 * mask[b*mask_ld + t] = (t < n_b), lengths[b] = min(n_b, T), rows_out[b*T + t] = row or -1
 * (all three nullable).  The sparse push skips rows < 0. */
int rs_sequence_lookup_fwd(void* stream, const int64_t* ids, const int32_t* offsets, int64_t B,
                           int T, int64_t row_base, int64_t bucket, int hash_mode,
                           const float* table, int dim, float* out, int64_t out_ss,
                           int64_t out_rs, uint8_t* mask, int64_t mask_ld, int32_t* lengths,
                           int32_t* rows_out);

/* Sparse gradient push (the backward half of EmbeddingFeatures; tensornet pushes per-feature
 * gradients to its PS): grad_table[rows[k]] += scale(s) * dout[s] for every id k of segment s.
 * Rows touched for the first time this step are claimed (flag -1 -> -2) and appended to
 * touched[*n_touched++] (capacity touched_cap).  flag[] must be all -1 between steps (the
 * optimizer entry points restore it).  touched == NULL selects SCAN mode: rows are only marked
 * (flag = -2, plain stores; no claims, n_touched unused) for rs_sparse_adam_scan /
 * rs_sparse_adagrad_scan / rs_sparse_compact_scan. */
int rs_sparse_grad_accumulate(void* stream, const int32_t* rows, const int32_t* offsets,
                              int64_t B, int F, const float* dout, int64_t dout_ld,
                              int64_t dout_fstride, int dim, int combiner, float* grad_table,
                              int32_t* flag, int32_t* touched, int32_t* n_touched,
                              int32_t touched_cap);

/* rs_sparse_grad_accumulate with a caller workspace of >= rs_sparse_push_workspace_bytes(B, F)
 * bytes: single-hot pushes (offsets == NULL) claim rows by election (plain flag stores + a claim
 * kernel, no returning atomics on hot rows' flag words; csrc/embedding.hip rs_push), rows of
 * >= 32 floats aggregated per block by a counting sort instead of LDS float atomics; multi-hot
 * pushes (offsets != NULL, no workspace needed) run a counting-sort push with CAS claims -- same
 * results and semantics.  Unaligned dout and a NULL / small workspace in single-hot list mode run
 * rs_sparse_grad_accumulate.  Graph-capturable. */
int64_t rs_sparse_push_workspace_bytes(int64_t B, int F);
int rs_sparse_grad_accumulate_ws(void* stream, const int32_t* rows, const int32_t* offsets,
                                 int64_t B, int F, const float* dout, int64_t dout_ld,
                                 int64_t dout_fstride, int dim, int combiner, float* grad_table,
                                 int32_t* flag, int32_t* touched, int32_t* n_touched,
                                 int32_t touched_cap, void* workspace, int64_t workspace_bytes);

/* Several single-hot pushes into ONE table as one launch (+ one claim launch in list mode):
 * source k pushes rows[k] [B[k], F[k]] with gradient rows dout[k] + b * dout_ld[k] +
 * f * dout_fstride[k] (16-B aligned, dim >= 32 floats).  Results and claim semantics equal one
 * rs_sparse_grad_accumulate_ws call per source (a row pushed by several sources is claimed once).
 * nsrc <= 8; workspace >= rs_sparse_push_group_workspace_bytes(nsrc, B, F) in list mode
 * (touched != NULL).  RS_ERR_UNSUPPORTED (nothing launched) for rows under 32 floats or unaligned
 * gradients: push the sources one by one.  Replaces the per-layer pushes of the
 * EmbeddingFeatures / sequence columns that share one tensornet table in one backward
 * (staytime/VideoDnn.py:217-244, one table for every feature column).  Graph-capturable. */
int64_t rs_sparse_push_group_workspace_bytes(int nsrc, const int64_t* B, const int* F);
int rs_sparse_grad_accumulate_group(void* stream, int nsrc, const int32_t* const* rows,
                                    const float* const* dout, const int64_t* B, const int* F,
                                    const int64_t* dout_ld, const int64_t* dout_fstride, int dim,
                                    float* grad_table, int32_t* flag, int32_t* touched,
                                    int32_t* n_touched, int32_t touched_cap, void* workspace,
                                    int64_t workspace_bytes);

/* Deterministic variant of rs_sparse_grad_accumulate: sort by row + segmented sum,
 * so each touched row receives the sum of its occurrences in ascending id order with one plain
 * read-modify-write -- bitwise reproducible run to run (the atomic push reproduces only the row
 * set).  Same arguments and marking/claiming semantics, plus table_rows (ids outside the table
 * push nothing), n_ids (ids in the batch: offsets[B*F], or B*F single-hot -- no host read back)
 * and a workspace of >= rs_sparse_sorted_workspace_bytes(n_ids) bytes.  dim <= 128.  Async on
 * the stream (hipcub radix sort / run-length encode / scan + two kernels): graph-capturable. */
int64_t rs_sparse_sorted_workspace_bytes(int64_t n_ids);
int rs_sparse_grad_accumulate_sorted(void* stream, const int32_t* rows, const int32_t* offsets,
                                     int64_t B, int F, const float* dout, int64_t dout_ld,
                                     int64_t dout_fstride, int dim, int combiner,
                                     int64_t table_rows, float* grad_table, int32_t* flag,
                                     int32_t* touched, int32_t* n_touched, int32_t touched_cap,
                                     void* workspace, int64_t workspace_bytes, int64_t n_ids);

/* N2 owner-sharded tables (SURVEY §8(e) owner = row % N; tensornet's PS split,
 * rank/ctr/base_model.py:89-102 / staytime/VideoDnn.py:233).  rs_embedding_lookup_fwd and
 * rs_sequence_lookup_fwd with table == out == NULL write only rows_out (and mask / lengths): the
 * id -> row half.  rs_owner_route orders the n rows by owner (stable: ascending position within an
 * owner; rows < 0 or >= table_rows dropped), writing send_local[i] = row / world, send_pos[i] =
 * the row's position and counts[w] = rows owned by w (device int32 [world]); workspace >=
 * rs_owner_route_workspace_bytes(n, world) (-1: n or world out of range; world <= 1024).
 * rs_gather_rows: dst[i] = src[idx[i]] (idx < 0: zero row); rs_scatter_rows: dst[idx[i]] =
 * src[i] (idx < 0 skipped); rows of dim floats (dim % 4 == 0), leading dimensions in floats.
 * rs_segment_expand: dE[k] = scale(s) * dout[b*dout_ld + f*dout_fstride] for every id k of
 * segment s = b*F + f (offsets [B*F+1]; the combiner's per-id gradient of a VarLen lookup).
 * rs_owner_route_fixed: the sync-free route -- the same stable owner order, but owner w's k-th
 * row goes to slot w*cap + k of send_local [world*cap] (pads -1) for k < cap, slot[i] = the slot
 * of position i (-1: invalid row or past its owner's cap, dropped); stats[0] (device int32,
 * sticky) = max(stats[0], the largest per-owner count), so stats[0] > cap means rows were
 * dropped.  Equal splits of cap per rank make the all-to-alls graph-capturable. */
int64_t rs_owner_route_workspace_bytes(int64_t n, int world);
int rs_owner_route(void* stream, const int32_t* rows, int64_t n, int world, int64_t table_rows,
                   int32_t* send_local, int32_t* send_pos, int32_t* counts, void* workspace,
                   int64_t workspace_bytes);
int rs_owner_route_fixed(void* stream, const int32_t* rows, int64_t n, int world,
                         int64_t table_rows, int cap, int32_t* send_local, int32_t* slot,
                         int32_t* stats, void* workspace, int64_t workspace_bytes);
int rs_gather_rows(void* stream, const float* src, int64_t src_ld, const int32_t* idx, int64_t n,
                   int dim, float* dst, int64_t dst_ld);
int rs_scatter_rows(void* stream, const float* src, int64_t src_ld, const int32_t* idx, int64_t n,
                    int dim, float* dst, int64_t dst_ld);
int rs_segment_expand(void* stream, const float* dout, int64_t dout_ld, int64_t dout_fstride,
                      const int32_t* offsets, int64_t B, int F, int combiner, int dim, float* dE);

/* H11 sparse optimizers on the touched rows (tensornet tn.core.Adam / tn.core.AdaGrad handed to
 * EmbeddingFeatures: rank/ctr/base_model.py:163, rank/multi_head/multidnn.py:235,
 * staytime/VideoDnn.py:233).  Zero the gradient rows, release the flags, reset the count.
 * n_touched points at int32[1 + 288] = {count, completion counters} (all zero between steps):
 * the last workgroup of the launch resets them, so no separate memset is needed.
 * max_rows bounds the grid (>= the largest possible count). */
int rs_sparse_adam(void* stream, float* table, float* m, float* v, float* grad_table,
                   int32_t* flag, const int32_t* touched, int32_t* n_touched, int dim,
                   int32_t max_rows, float lr, float beta1, float beta2, float eps,
                   float grad_scale);
int rs_sparse_adagrad(void* stream, float* table, float* g2sum, float* grad_table, int32_t* flag,
                      const int32_t* touched, int32_t* n_touched, int dim, int32_t max_rows,
                      float lr, float grad_scale);

/* Scan-mode sparse optimizers (same update forms): sweep flag[0 .. table_rows) and update every
 * row marked by a scan-mode push (rs_sparse_grad_accumulate with touched == NULL,
 * rs_il_bwd_push, rs_sparse_merge_rows with touched == NULL); zero its gradient row, clear its
 * flag.  dim % 4 == 0. */
int rs_sparse_adam_scan(void* stream, float* table, float* m, float* v, float* grad_table,
                        int32_t* flag, int64_t table_rows, int dim, float lr, float beta1,
                        float beta2, float eps, float grad_scale);
int rs_sparse_adagrad_scan(void* stream, float* table, float* g2sum, float* grad_table,
                           int32_t* flag, int64_t table_rows, int dim, float lr,
                           float grad_scale);

/* Overflow recovery for the list-mode optimizers: launch right after rs_sparse_adam /
 * rs_sparse_adagrad on the same stream (same n_touched).  Exits at once unless a push claimed more
 * rows than the touched list holds (the sticky overflow word n_touched[288] is set); then sweeps
 * the table like the scan-mode optimizer and updates the claimed rows the list could not hold. */
int rs_sparse_adam_recover(void* stream, float* table, float* m, float* v, float* grad_table,
                           int32_t* flag, const int32_t* n_touched, int64_t table_rows, int dim,
                           float lr, float beta1, float beta2, float eps, float grad_scale);
int rs_sparse_adagrad_recover(void* stream, float* table, float* g2sum, float* grad_table,
                              int32_t* flag, const int32_t* n_touched, int64_t table_rows, int dim,
                              float lr, float grad_scale);

/* Scan-mode compaction for the DP exchange: move every marked row into (rows_out, grads_out)
 * (gradient row zeroed, flag cleared), *n_out = count (slots past cap are dropped),
 * rows_out[count .. cap) = -1. */
int rs_sparse_compact_scan(void* stream, float* grad_table, int32_t* flag, int64_t table_rows,
                           int dim, int32_t* rows_out, float* grads_out, int32_t* n_out,
                           int32_t cap);

/* Data-parallel sparse exchange (replaces tensornet's PS push across workers):
 * compact moves this rank's touched rows into (rows_out, grads_out) (padding rows = -1) and
 * clears the table; merge adds one rank's list back (rows unique within a list, no atomics).
 * Merging every rank's list in rank order gives bitwise-identical sums on every replica. */
int rs_sparse_compact(void* stream, float* grad_table, int32_t* flag, const int32_t* touched,
                      int32_t* n_touched, int dim, int32_t* rows_out, float* grads_out,
                      int32_t cap);
int rs_sparse_merge_rows(void* stream, const int32_t* rows, const float* grads, int32_t count,
                         int dim, float* grad_table, int32_t* flag, int32_t* touched,
                         int32_t* n_touched, int32_t touched_cap);
/* rs_sparse_merge_rows with the counts on the device (the graph-captured DP step of the generic
 * trainer): every rank's compacted list was all-gathered as a prefix of nmax = max_r count_r
 * entries (rows_all[r * nmax], grads_all[r * nmax * dim]); counts[r * counts_stride] is rank r's
 * count; cap bounds every count (the per-rank list capacity).  Adds rank `rank`'s list. */
int rs_sparse_merge_rows_dev(void* stream, const int32_t* rows_all, const float* grads_all,
                             const int32_t* counts, int64_t counts_stride, int world, int rank,
                             int32_t cap, int dim, float* grad_table, int32_t* flag,
                             int32_t* touched, int32_t* n_touched, int32_t touched_cap);
/* rs_sparse_merge_rows_dev over a FIXED layout: rank r's list at rows_all[r * stride] (the host
 * all-gathered `stride` entries per rank without reading the counts: no host synchronisation in
 * the data-parallel step).  A rank whose count exceeds stride lost rows in transit: its count
 * is recorded in the sticky *overflow (nullable; atomicMax, never cleared by the library). */
int rs_sparse_merge_rows_dev_stride(void* stream, const int32_t* rows_all, const float* grads_all,
                                    const int32_t* counts, int64_t counts_stride, int world,
                                    int rank, int32_t stride, int dim, float* grad_table,
                                    int32_t* flag, int32_t* touched, int32_t* n_touched,
                                    int32_t touched_cap, int32_t* overflow);

/* Packed scan-mode exchange (the graph-captured DP step of the AutoInt trainer; same role as
 * compact/merge above).  pack: every marked row becomes one record [row (int32 bits) | grad[dim]]
 * of dim + 1 floats at records[u * (dim + 1)], u < *count_out (records past cap are dropped;
 * cap >= the rows one rank can touch makes that impossible); the gradient row is zeroed and the
 * flag cleared.  One all-gather then moves every rank's records as one contiguous prefix of
 * nmax = max_r count_r records.  merge_packed adds rank `rank`'s records (at
 * records + rank * nmax * (dim + 1); counts[r * counts_stride] is rank r's count, nmax is
 * recomputed on the device, so the launch needs no host-side count and is graph-capturable) and
 * scan-marks the rows.  Launching it for rank 0 .. world-1 in order gives bitwise-identical sums
 * on every replica.  Record rows outside [0, table_rows) are skipped; counts are clamped to cap
 * (each rank's record capacity). */
int rs_sparse_pack_scan(void* stream, float* grad_table, int32_t* flag, int64_t table_rows,
                        int dim, float* records, int32_t* count_out, int32_t cap);
int rs_sparse_merge_packed(void* stream, const float* records, const int32_t* counts,
                           int64_t counts_stride, int world, int rank, int dim, float* grad_table,
                           int32_t* flag, int64_t table_rows, int32_t cap);
/* rs_sparse_merge_packed over a FIXED record layout: rank r's records start at r * stride (the
 * host all-gathered every rank's whole stride-record buffer, so it never read the counts: no host
 * synchronisation in the data-parallel step). */
int rs_sparse_merge_packed_stride(void* stream, const float* records, const int32_t* counts,
                                  int64_t counts_stride, int world, int rank, int dim,
                                  float* grad_table, int32_t* flag, int64_t table_rows,
                                  int32_t cap, int32_t stride);

/* ---------------------------------------------------------------------------------------
 * Math mode (config 2's "bf16" compute mode: BASELINE.json configs[1]).
 * RS_MATH_F32 (0, default): every kernel computes in fp32, the reference's dtype.
 * RS_MATH_BF16 (1): the matrix-core GEMMs of the InteractingLayer (projections, dW, dx;
 * E = U = 16, H = 2, F <= 32) and of the fused MLP head (rs_mlp_head_train: layers 1-2, dW1,
 * dx0) take bf16-rounded operands with fp32 accumulation; activations, attention, LN, losses,
 * optimizers, weights and tables stay fp32 (fp32 master weights).  Shapes without bf16 kernels
 * return -2 in bf16 mode (never a silent fp32 run).  Process-wide, read when a launch is
 * issued: a captured hipGraph keeps the mode it was captured under.  No reference counterpart
 * (the reference trains in fp32; cf. tf.keras.mixed_precision's mixed_bfloat16 policy).
 * ------------------------------------------------------------------------------------- */
int rs_set_math_mode(int mode);
int rs_get_math_mode(void);

/* Dropout seed offset (graph-replayed training; cf. PyTorch's CUDA-graph-safe RNG offsets).
 * dev_offset: a device int64 (or NULL, the default).  While set, every dropout-using launch
 * (the InteractingLayer entry points) uses seed + *dev_offset * 0x9E3779B97F4A7C15 (mod 2^64),
 * *dev_offset read by the kernel when it runs: a graph captured once and replayed each step
 * draws a fresh mask per step when the caller's step counter lives there.  Process-wide, read
 * at launch (a captured graph keeps the pointer it was captured with). */
int rs_set_seed_offset(const int64_t* dev_offset);

/* InteractingLayer kernel variant for the AutoInt shape family (E = U = 16, H = 2, F <= 32):
 * 0 = auto (default), 1 = one wave per sample (fwd_kernel / bwd4_kernel), 2 = one 4-wave
 * workgroup per sample (il_wide.hpp: the latency-bound small-batch case and the default).  Same
 * math and outputs within fp32 summation order; the partial-row count the backward leaves for
 * rs_partials_reduce_adam follows the variant (ask rs_il_bwd_partial_blocks under the same
 * setting).  Process-wide, read when a launch is issued.  No reference counterpart. */
int rs_il_set_variant(int variant);
int rs_il_get_variant(void);

/* ---------------------------------------------------------------------------------------
 * H3  InteractingLayer (InteractingLayer.py:7-61; rank/multi_head/interacting_layer.py:7-61).
 * x [B, F, E]; W [E, 4U] = [Wq | Wk | Wv | Wr] (Keras Dense kernels), bias [4U],
 * gamma/beta [U] (LayerNormalization), layer_num L with tied weights (L > 1 needs E == U).
 * y row stride y_ld (>= F*U).  xsave [(L-1), B, F, U] receives the inputs of iterations
 * 1..L-1 for the backward (nullable when L == 1).  Dropout on the softmax weights
 * (InteractingLayer.py:53-54) uses the counter-based mask documented in csrc/common.hpp.
 * ------------------------------------------------------------------------------------- */
int rs_il_param_count(int E, int U);
int rs_il_fwd(void* stream, const float* x, int64_t B, int F, int E, int U, int H, int L,
              const float* W, const float* bias, const float* gamma, const float* beta,
              float eps, int use_res, float drop_rate, uint64_t seed, float* y, int64_t y_ld,
              float* xsave);
/* Forward with the embedding front end fused in (single-hot fields, F <= 64): replaces
 * rs_embedding_lookup_fwd(ids, offsets = NULL, ...) + rs_il_fwd(x, ...) -- the
 * EmbeddingFeatures lookup + expand/Concatenate of autoint:22-26 (rank/ctr/base_model.py:203-217)
 * followed by InteractingLayer.call (InteractingLayer.py:37-61).  x[b, f, :] =
 * table[row_base[f] + H(ids[b, f]) mod bucket[f]] is read straight into the kernel's LDS and ALSO
 * stored to x [B, F, E] (the MLP head's and the backward's input) and rows_out [B*F] (nullable;
 * the sparse push's rows).  Bit-identical to the two separate calls. */
int rs_il_fwd_gather(void* stream, const int64_t* ids, const int64_t* row_base,
                     const int64_t* bucket, int hash_mode, const float* table, int64_t table_rows,
                     float* x, int32_t* rows_out, int64_t B, int F, int E, int U, int H, int L,
                     const float* W, const float* bias, const float* gamma, const float* beta,
                     float eps, int use_res, float drop_rate, uint64_t seed, float* y,
                     int64_t y_ld, float* xsave);
/* Backward (TF autograd of the graph above).  dx [B, F, E] written (or accumulated).
 * dparams = [dW (E*4U) | dbias (4U) | dgamma (U) | dbeta (U)] written (or accumulated);
 * dparams == NULL skips the grid reduction (per-block partials stay in the workspace).
 * workspace >= rs_il_bwd_workspace_floats(B, E, U) floats. */
int64_t rs_il_bwd_workspace_floats(int64_t B, int E, int U);
int rs_il_bwd(void* stream, const float* x, const float* xsave, const float* dy, int64_t dy_ld,
              int64_t B, int F, int E, int U, int H, int L, const float* W, const float* bias,
              const float* gamma, const float* beta, float eps, int use_res, float drop_rate,
              uint64_t seed, float* dx, int dx_accumulate, float* dparams,
              int dparams_accumulate, float* workspace, int64_t workspace_floats);
/* Saved-attention pairs: the forward also writes, per (iteration, sample), the attention output
 * before the epilogue and the softmax row statistics into asave, and the backward reads them
 * instead of recomputing the attention forward.
 *   F > 64 (many-field kernels, rank/multi_head config 3): + the dropout keep bits; same results
 *     as the plain pair.
 *   F <= 32, U == 16, H == 2 (config 2): O [F][U] | (scaled max, 1/sum) [H*F][2] per (iteration,
 *     sample); the backward runs the LN backward first and the attention backward in two key
 *     sweeps (bwd4_kernel).  Within the gradient tolerance of the plain pair (the softmax weights
 *     come from the saved stats instead of a re-run of the max / sum).
 * asave >= rs_il_attn_save_floats(B, F, U, H, L) floats (0 for other shapes: there asave may be
 * NULL and the calls are exactly rs_il_fwd / rs_il_bwd). */
int64_t rs_il_attn_save_floats(int64_t B, int F, int U, int H, int L);
int rs_il_fwd_saved(void* stream, const float* x, int64_t B, int F, int E, int U, int H, int L,
                    const float* W, const float* bias, const float* gamma, const float* beta,
                    float eps, int use_res, float drop_rate, uint64_t seed, float* y,
                    int64_t y_ld, float* xsave, float* asave, int64_t asave_floats);
int rs_il_bwd_saved(void* stream, const float* x, const float* xsave, const float* dy,
                    int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L, const float* W,
                    const float* bias, const float* gamma, const float* beta, float eps,
                    int use_res, float drop_rate, uint64_t seed, float* dx, int dx_accumulate,
                    float* dparams, int dparams_accumulate, float* workspace,
                    int64_t workspace_floats, const float* asave, int64_t asave_floats);

/* ---------------------------------------------------------------------------------------
 * H6/H7  DIN behaviour-sequence attention pooling.
 *   variant 0: din.py:18-47 (DIN(**kwargs)(queries, keys, values, seq_length)):
 *              s_t = relu(relu([q, k_t, q*k_t] W1 + b1) W2 + b2), masked to 0, out = sum s_t v_t
 *   variant 1: staytime/layer.py:16-41 (DIN(**kwargs)(query, facts, mask)):
 *              z_t = sigmoid([q, f_t, q-f_t, q*f_t] W1 + b1) W2 + b2, masked -> -2**32+1,
 *              p = softmax_t(z), out = sum p_t f_t (values must be the keys tensor)
 * q [B, H] (row stride q_ld); keys / values [B, T, H] with sample stride *_ss and row stride
 * *_rs (floats; last dim contiguous, 16-byte aligned rows).  W1 [3H|4H, 16], b1 [16],
 * W2 [16, 1], b2 [1] (Keras Dense kernels).  Position t of sample b is on iff
 * (lengths == NULL || t < lengths[b]) && (mask == NULL || mask[b*mask_ld + t]).
 * H = 16 is the compiled width (configs 4, 5).  probs [B, T] (variant 1, nullable in inference)
 * receives the softmax for the backward.
 * ------------------------------------------------------------------------------------- */
int rs_din_param_count(int variant, int H);
int rs_din_fwd(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
               int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
               int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
               int64_t mask_ld, const float* W1, const float* b1, const float* W2,
               const float* b2, float* out, int64_t out_ld, float* probs);
/* Backward: dq [B, H] (row stride dq_ld) written; dkeys / dvalues [B, T, H] contiguous written
 * (nullable; dkeys == dvalues writes their sum, always the case for variant 1); dparams =
 * [dW1 | db1 | dW2 | db2] written or accumulated (nullable).  workspace >=
 * rs_din_bwd_workspace_floats(variant, B, T, H) floats (required). */
int64_t rs_din_bwd_workspace_floats(int variant, int64_t B, int T, int H);
int rs_din_bwd(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
               int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
               int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
               int64_t mask_ld, const float* W1, const float* b1, const float* W2,
               const float* b2, const float* probs, const float* dout, int64_t dout_ld,
               float* dq, int64_t dq_ld, float* dkeys, float* dvalues, float* dparams,
               int dparams_accumulate, float* workspace, int64_t workspace_floats);
/* rs_din_bwd with dkeys / dvalues rows at stride dkv_rs (>= H) and columns H .. dkv_width - 1 of
 * every row written as zeros (dkv_width <= min(dkv_rs, 2H)): the gradient of a wider facts row
 * whose first H columns the pooling reads (staytime: 32-wide sequence rows, VideoDnn.py:57-77),
 * without a zero fill and a strided copy.  rs_din_bwd = this with dkv_rs = dkv_width = H. */
int rs_din_bwd_strided(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
                       int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
                       int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
                       int64_t mask_ld, const float* W1, const float* b1, const float* W2,
                       const float* b2, const float* probs, const float* dout, int64_t dout_ld,
                       float* dq, int64_t dq_ld, float* dkeys, float* dvalues, int64_t dkv_rs,
                       int dkv_width, float* dparams, int dparams_accumulate, float* workspace,
                       int64_t workspace_floats);
/* rs_din_bwd_strided that also adds the query's other gradient: dq = dq_base + dL/dq (dq_base
 * [B, >= H] at row stride dq_base_ld, nullable; may not alias dq).  Used when the query is also
 * concatenated after the pooled output (the config-4 head's [pooled, q]). */
int rs_din_bwd_ex(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
                  int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
                  int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
                  int64_t mask_ld, const float* W1, const float* b1, const float* W2,
                  const float* b2, const float* probs, const float* dout, int64_t dout_ld,
                  float* dq, int64_t dq_ld, const float* dq_base, int64_t dq_base_ld,
                  float* dkeys, float* dvalues, int64_t dkv_rs, int dkv_width, float* dparams,
                  int dparams_accumulate, float* workspace, int64_t workspace_floats);

/* ---------------------------------------------------------------------------------------
 * H4/H5/H8/H9  Keras Dense(units, activation) towers (autoint:36-52 MultiLayerDense,
 * rank/multi_head/multidnn.py:60-127, rough_rank/layer.py:33-117 DNN,
 * staytime/VideoDnn.py:130-191).  act: 0 linear, 1 relu, 2 sigmoid.
 * Y[M, N] (ld ldy) = act(X[M, K] (ld ldx) @ W[K, N] + b).
 * ------------------------------------------------------------------------------------- */
int rs_dense_fwd(void* stream, const float* X, int64_t M, int K, int64_t ldx, const float* W,
                 const float* bias, int N, int act, float* Y, int64_t ldy);
/* dX (+)= (dY * act'(Y)) @ W^T */
int rs_dense_bwd_data(void* stream, const float* dY, int64_t lddy, const float* Y, int64_t ldy,
                      int act, const float* W, int64_t M, int K, int N, float* dX,
                      int64_t lddx, int accumulate);
/* dW (+)= X^T (dY * act'(Y)), db (+)= colsum(dY * act'(Y)); deterministic */
int64_t rs_dense_bwd_weight_workspace_floats(int64_t M, int K, int N);
int rs_dense_bwd_weight(void* stream, const float* X, int64_t ldx, const float* dY, int64_t lddy,
                        const float* Y, int64_t ldy, int act, int64_t M, int K, int N, float* dW,
                        float* db, int accumulate, float* workspace, int64_t workspace_floats);
/* The whole Dense backward in one launch: dX (+)= dZ W^T and dW / db (+)= X^T dZ / colsum dZ side by
 * side (plus the split-K reduce when the weight gradient splits; workspace as
 * rs_dense_bwd_weight_workspace_floats).  Same results as rs_dense_bwd_data + rs_dense_bwd_weight
 * (it falls back to them for unaligned operands). */
int rs_dense_bwd(void* stream, const float* X, int64_t ldx, const float* dY, int64_t lddy,
                 const float* Y, int64_t ldy, int act, const float* W, int64_t M, int K, int N,
                 float* dX, int64_t lddx, int dx_accumulate, float* dW, float* db, int w_accumulate,
                 float* workspace, int64_t workspace_floats);
/* Large GEMMs (M K N >= 2^26 multiply-adds by default; RS_GEMM_BIG=0 off, RS_GEMM_BIG_MACS=n
 * threshold) run the hand-written direct-to-LDS kernels of gemm_big.hip inside the four entries
 * above: forward with its bias / activation epilogue, data and weight gradients with
 * dZ = dY act'(Y) applied to the MFMA fragments (no dZ pass), db as the weight product's extra
 * output row, split-K weight gradients through the workspace (the workspace query covers them)
 * and a fixed-order column reduction.  rs_dense_uses_big(M, K, N): 1 when a Dense layer of that
 * shape takes these kernels.  Opt-in comparison route: RS_GEMM_BLAS=1 sends the same shapes to
 * hipBLASLt (rs_dense_uses_library(M, K, N) says which; results then equal the engine's to fp32
 * rounding, not bitwise). */
int rs_dense_uses_big(int64_t M, int K, int N);
int rs_dense_uses_library(int64_t M, int K, int N);
/* Grouped Dense: G <= 8 independent layers of one kind in ONE launch (plus one grouped split-K
 * reduce for weight gradients) -- the per-expert / per-task layers that staytime/VideoDnn.py:130-191
 * and rough_rank/layer.py:174-233 build in Python loops.  desc: G records of int64 (pointers cast):
 *   fwd        [M, K, N, ldx, ldy, act, X, W, bias, Y]                           (10 per layer)
 *   bwd_data   [M, K, N, lddy, ldy, act, dY, Y, W, dX, lddx, accumulate]         (12 per layer)
 *   bwd_weight [M, K, N, ldx, lddy, ldy, act, X, dY, Y, dW, db, accumulate]      (13 per layer;
 *              one accumulate flag for the group)
 * Same results as the per-layer calls up to summation order of split reductions. */
int rs_dense_fwd_grouped(void* stream, int G, const int64_t* desc);
int rs_dense_bwd_data_grouped(void* stream, int G, const int64_t* desc);
int64_t rs_dense_bwd_weight_grouped_workspace_floats(int G, const int64_t* desc);
int rs_dense_bwd_weight_grouped(void* stream, int G, const int64_t* desc, float* workspace,
                                int64_t workspace_floats);

/* ---------------------------------------------------------------------------------------
 * H5/H8/H9  Tower ops around the Dense GEMMs (csrc/towers.hip).  act codes as rs_dense_fwd.
 * ------------------------------------------------------------------------------------- */
/* Gate mixture (MMOE.call rough_rank/layer.py:149-162, PLE.call :212-226,
 * rank/multi_head/multidnn.py:95-120, staytime/VideoDnn.py:150-164):
 *   Y[m, t*D + d] = sum_k softmax_k(G[m, t*n_sel + k]) * act(E[m, sel[t*n_sel + k]*D + d]).
 * E holds n_exp experts of width D (pre-activation when e_act != 0), G the gate logits; both
 * may be column ranges of ONE concatenated GEMM output.  sel: device int32 [n_task*n_sel].
 * P [m, t*n_sel + k] (nullable) receives the gate probabilities.
 * Backward writes dE (= dL/d(pre-activation) when e_act != 0) and dG (gate logits). */
int rs_gate_mix_fwd(void* stream, const float* E, int64_t lde, int e_act, const float* G,
                    int64_t ldg, int64_t M, int n_exp, int D, int n_task, int n_sel,
                    const int32_t* sel, float* Y, int64_t ldy, float* P, int64_t ldp);
int rs_gate_mix_bwd(void* stream, const float* E, int64_t lde, int e_act, const float* G,
                    int64_t ldg, int64_t M, int n_exp, int D, int n_task, int n_sel,
                    const int32_t* sel, const float* dY, int64_t lddy, float* dE, int64_t ldde,
                    float* dG, int64_t lddg);
/* CrossNet (rough_rank/layer.py:236-270) / DeepCrossLayer (staytime/layer.py:44-80):
 * x_{l+1} = x0 * (x_l . W[l]) + b[l] + x_l, W, b [L, D] (L <= 4, D <= 2048).
 * Backward: dX0 written/accumulated, dparams = [dW (L*D) | db (L*D)] (nullable). */
int rs_cross_fwd(void* stream, const float* X0, int64_t ldx, int64_t M, int D, int L,
                 const float* W, const float* b, float* Y, int64_t ldy);
int64_t rs_cross_bwd_workspace_floats(int64_t M, int D, int L);
int rs_cross_bwd(void* stream, const float* X0, int64_t ldx, int64_t M, int D, int L,
                 const float* W, const float* b, const float* dY, int64_t lddy, float* dX0,
                 int64_t lddx, int dx_accumulate, float* dparams, int dparams_accumulate,
                 float* workspace, int64_t workspace_floats);
/* FM cross term with optional per-field scale (FMLayer staytime/layer.py:83-116; SENet
 * reweight + FM of staytime/VideoDnn.py:81-115): field f of row m at X[m*ldx + f*fsx + e];
 * y_f = x_f * a_scale * A[m*lda + f] (A nullable; SENet's 2 * sigmoid uses a_scale 2) -> Y[m*ldy + f*E + e] (nullable);
 * cross_e = (sum_f y_f)^2 - sum_f y_f^2 -> C (nullable); fm = 0.5 sum_e cross_e -> fm[m*ldf]. */
int rs_fm_fwd(void* stream, const float* X, int64_t ldx, int64_t fsx, int64_t M, int F, int E,
              const float* A, int64_t lda, float a_scale, float* Y, int64_t ldy, float* C, int64_t ldc,
              float* fm, int64_t ldf);
int rs_fm_bwd(void* stream, const float* X, int64_t ldx, int64_t fsx, int64_t M, int F, int E,
              const float* A, int64_t lda, float a_scale, const float* dY, int64_t lddy, const float* dC,
              int64_t lddc, const float* dfm, int64_t lddf, float* dX, int64_t lddx,
              int64_t fsdx, int dx_accumulate, float* dA, int64_t ldda);
/* ffm_block (staytime/VideoDnn.py:11-25): pair p = (i, j), i < NU user fields, j < NI item
 * fields (field k at column cols[k] of X, user fields first, E = 16):
 * Y[m, p*Dff + c] = (x_i Wx[p] + bx[p])_c * (y_j Wy[p] + by[p])_c; Mult (nullable, NU == NI)
 * = relu(x_i * y_i) (:99-105).  params = [Wx (P*E*Dff) | bx (P*Dff) | Wy | by]. */
int64_t rs_ffm_param_count(int NU, int NI, int E, int Dff);
int rs_ffm_fwd(void* stream, const float* X, int64_t ldx, int64_t M, int NU, int NI, int E,
               int Dff, const int32_t* cols, const float* Wx, const float* bx, const float* Wy,
               const float* by, float* Y, int64_t ldy, float* Mult, int64_t ldm);
int64_t rs_ffm_bwd_workspace_floats(int64_t M, int NU, int NI, int E, int Dff);
int rs_ffm_bwd(void* stream, const float* X, int64_t ldx, int64_t M, int NU, int NI, int E,
               int Dff, const int32_t* cols, const float* Wx, const float* bx, const float* Wy,
               const float* by, const float* dY, int64_t lddy, const float* dMult,
               int64_t lddm, float* dX, int64_t lddx, int dx_accumulate, float* dparams,
               int dparams_accumulate, float* workspace, int64_t workspace_floats);
/* ppnet gating (staytime/VideoDnn.py:135-146): Y = A * (scale * G) and its backward. */
int rs_mul_fwd(void* stream, const float* A, int64_t lda, const float* G, int64_t ldg, int64_t M,
               int N, float scale, float* Y, int64_t ldy);
int rs_mul_bwd(void* stream, const float* A, int64_t lda, const float* G, int64_t ldg, int64_t M,
               int N, float scale, const float* dY, int64_t lddy, float* dA, int64_t ldda,
               float* dG, int64_t lddg);
/* Grouped gating multiplies (G <= 8, one launch): desc int64 records
 *   fwd [M, N, lda, ldg, ldy, A, G, Y]                     Y = A * (scale G)
 *   bwd [M, N, lda, ldg, lddy, ldda, lddg, A, G, dY, dA, dG]  (dA / dG may be 0) */
int rs_mul_fwd_grouped(void* stream, int G, const int64_t* desc, float scale);
int rs_mul_bwd_grouped(void* stream, int G, const int64_t* desc, float scale);
/* H9/H10 staytime head (staytime/VideoDnn.py:168-179) + custom_kl_loss (staytime/model.py:20-30):
 * P[m, 0:C] = softmax(Z[m]), P[m, C] = max(P . bins, 0) (P, bins nullable); with y_true:
 * loss_rows[m] = w_m * sum_c yt log(yt / yp) (yt, yp clipped to [eps, 1]) and
 * dZ = gscale * w_m * dKL/dZ (through the clip and the softmax). */
int rs_softmax_kl(void* stream, const float* Z, int64_t ldz, int64_t M, int C, const float* bins,
                  float* P, int64_t ldp, const float* y_true, int64_t ldt, const float* sample_w,
                  float gscale, float eps, float* loss_rows, float* dZ, int64_t lddz);
/* Similarity (rough_rank/layer.py:6-30): Y[m] = [sigmoid](U[m] . V[m]); with dY: dU, dV. */
int rs_rowdot(void* stream, const float* U, int64_t ldu, const float* V, int64_t ldv, int64_t M,
              int N, int use_sigmoid, float* Y, const float* dY, float* dU, int64_t lddu,
              float* dV, int64_t lddv);
/* KDLoss (rough_rank/layer.py:272-279): loss_rows[m] = mean_j (S - T)^2,
 * dS = gscale * 2 (S - T) / N (nullable). */
int rs_mse_rows(void* stream, const float* S, int64_t lds, const float* T, int64_t ldt, int64_t M,
                int N, float gscale, float* loss_rows, float* dS, int64_t ldds);

/* T independent Dense(1, act) heads (rank/multi_head/multidnn.py:122-204 towers): head t reads
 * X columns [t*D, t*D + D), kernel W[t*D .. t*D + D), bias b[t]; Y[m*ldy + t].  T*D <= 256,
 * D a power of two <= 64.  Backward: dX (nullable), dparams = [dW (T*D) | db (T)]. */
int rs_grouped_head_fwd(void* stream, const float* X, int64_t ldx, int64_t M, int T, int D,
                        const float* W, const float* b, int act, float* Y, int64_t ldy);
int64_t rs_grouped_head_bwd_workspace_floats(int64_t M, int T, int D);
int rs_grouped_head_bwd(void* stream, const float* X, int64_t ldx, int64_t M, int T, int D,
                        const float* W, const float* Y, int64_t ldy, int act, const float* dY,
                        int64_t lddy, float* dX, int64_t lddx, float* dparams,
                        int dparams_accumulate, float* workspace, int64_t workspace_floats);
/* tf.where(mask == 1, A, B) per row (rough_rank/model.py:52-53): forward Y, or with dY the
 * routed gradients dA / dB ([M, N] contiguous, nullable). */
int rs_row_select(void* stream, const float* mask, const float* A, int64_t lda, const float* B,
                  int64_t ldb, int64_t M, int N, float* Y, int64_t ldy, const float* dY,
                  float* dA, float* dB);

/* Per-row (sample-weighted) binary cross entropy, contiguous [M, T]: staytime/model.py:33-36
 * cross_entropy with Keras sample weights; rough_rank BinaryCrossentropy with lo = eps,
 * hi = 1 - eps.  loss_rows[m] = w_m sum_t ce (nullable), dP = gscale w_m dce/dp (nullable). */
int rs_bce_rows(void* stream, const float* P, const float* Y, int64_t M, int T, float lo, float hi,
                float log_eps, const float* W, float gscale, float* loss_rows, float* dP);

/* Fused loss total (staytime/model.py:85-89 loss_weights, rough_rank/model.py:210-214):
 * out[0] = sum_k w_k * sum_i X[k*seg + i] over nseg <= 6 back-to-back per-row loss vectors
 * (rs_bce_rows / rs_softmax_kl / rs_mse_rows rows; w_k = loss_weight_k / batch).  One launch,
 * fixed summation order. */
int rs_weighted_row_sum(void* stream, const float* X, int64_t seg, int nseg, float w0, float w1,
                        float w2, float w3, float w4, float w5, float* out);

/* N1  staytime parse_input_func labels (staytime/parse.py:16-71) for a batch of B samples:
 * label [B, ld] rows = nbins Gaussian soft-label bins (sigma, width = (right - left)/(nbins - 1))
 * then the clipped watch time in seconds; short/long = watch_ms > 7000 / > 18000 (fp32 0/1);
 * weight = 5 where landing[b] != 0 (the host's regex match of extra_info against
 * ".*video_homepage_landing.*", parse.py:64), else 1.  landing, short_label, long_label and
 * weight may be NULL.  Requires ld >= nbins + 1, nbins >= 2, sigma > 0. */
int rs_staytime_labels(void* stream, const int64_t* watch_ms, const uint8_t* landing, int64_t B,
                       const float* bins, int nbins, float sigma, float left, float right,
                       float* label, int64_t ld, float* short_label, float* long_label,
                       float* weight);

/* Elementwise activation of a contiguous [n] tensor (tf.sigmoid of the rough_rank logits,
 * rough_rank/model.py:80,146): Y = act(X); backward dX = dY * act'(Y). */
int rs_act_fwd(void* stream, const float* X, int64_t n, int act, float* Y);
int rs_act_bwd(void* stream, const float* Y, const float* dY, int64_t n, int act, float* dX);

/* H4/H10  tf.clip_by_value(s, lo, hi) (autoint:52) + cross_entropy (rank/ctr/base_model.py:7-12):
 * loss[0] = mean_b sum_t [-y log(p+log_eps) - (1-y) log(1-p+log_eps)], p_out = clipped s,
 * ds = gscale[0] * dloss/ds (zero outside [lo, hi]; gscale NULL = 1).  Any output pointer
 * may be NULL. */
int rs_bce_clip_loss(void* stream, const float* s, const float* y, int64_t M, int T,
                     float clip_lo, float clip_hi, float log_eps, const float* gscale,
                     float* p_out, float* loss, float* ds);
/* The same over several workgroups: per-block sums in `workspace` (rs_bce_clip_workspace_floats;
 * its first 288 (RS_DONE_WORDS) words are completion counters that must be zero before the first call
 * and are left zero by every call), added in block order by the last block (deterministic for a
 * given M, T).  Calls sharing one workspace must not run concurrently. */
int64_t rs_bce_clip_workspace_floats(int64_t M, int T);
int rs_bce_clip_loss_ws(void* stream, const float* s, const float* y, int64_t M, int T,
                        float clip_lo, float clip_hi, float log_eps, const float* gscale,
                        float* p_out, float* loss, float* ds, float* workspace,
                        int64_t workspace_floats);

/* ---------------------------------------------------------------------------------------
 * H11  dense Adam over a flat parameter arena (tn.optimizer.Optimizer(tn.core.Adam(...)):
 * rank/ctr/base_model.py:192-193, rank/multi_head/model.py:52-53, staytime/model.py:72,
 * rough_rank/model.py:209).  step is a device int64 counter (read, then incremented).
 * zero_grad != 0 zeroes each gradient after reading it (fused optimizer.zero_grad()).
 * ------------------------------------------------------------------------------------- */
int rs_dense_adam(void* stream, float* params, float* grads, float* m, float* v, int64_t n,
                  int64_t* step, float lr, float beta1, float beta2, float eps, float grad_scale,
                  int zero_grad);
/* rs_dense_adam with the step counter advanced by the kernel's last block (done: caller-owned
 * int32[RS_DONE_WORDS = 288], zero between launches) instead of a second launch. */
int rs_dense_adam_done(void* stream, float* params, float* grads, float* m, float* v, int64_t n,
                       int64_t* step, float lr, float beta1, float beta2, float eps,
                       float grad_scale, int zero_grad, int32_t* done);

/* Keras kernel regularisers as a gradient term (L1L2 at rank/multi_head/multidnn.py:62-63,
 * L2 at :85,103 and rough_rank/layer.py:77): grads += l1 * sign(w) + 2 * l2 * w. */
int rs_l1l2_grad(void* stream, const float* params, float* grads, int64_t n, float l1, float l2);
/* The same for n <= 16 tensors in one launch: tensor k = (params[k], grads[k], counts[k] elements,
 * l1[k], l2[k]); the pointer / count arrays are host memory read at the call. */
int rs_l1l2_grad_grouped(void* stream, int n, const float* const* params, float* const* grads,
                         const int64_t* counts, const float* l1, const float* l2);

/* ---------------------------------------------------------------------------------------
 * H4 + H10 fused: the AutoInt head training pass (autoint:38-52 + rank/ctr/base_model.py:7-12).
 * Replaces, for the training step, the chain rs_dense_fwd x (deep + logits) -> rs_bce_clip_loss
 * -> rs_dense_bwd_data / rs_dense_bwd_weight x (logits + deep) that mirrors
 *   deep = MultiLayerDense([N1, N2], act)(Flatten(x0));  result = concat([deep, il], axis=1)
 *   p = clip(MultiLayerDense([T], act3)(result), lo, hi);  loss = cross_entropy(labels, p)
 * N2 = 0 means a single deep layer.  Supported (N1, N2): (32,16) (64,32) (16,0) (32,0) (64,0)
 * (16,16) (32,32) (64,16) (64,64); T <= 4; K0 % 16 == 0; S % 4 == 0; x0 / il 16-byte aligned
 * (RS_ERR_UNSUPPORTED otherwise: use the per-layer entry points).
 * Writes p_out [B, T] (may be NULL), dil = dL/d il [B, S] (row stride ld_dil), dx0 = dL/dx0 from
 * the deep tower (overwrite, or += when dx_accumulate).  Weight gradients and the loss are left
 * as per-block partial rows in `workspace` (rs_mlp_head_partial_blocks(B) rows of
 * rs_mlp_head_param_floats(...) + 1 floats, arena order [W1 b1 W2 b2 W3 b3 | loss_sum]) for
 * rs_partials_reduce_adam.  The loss partials are sums; the batch mean is sum / B.
 * ------------------------------------------------------------------------------------- */
int64_t rs_mlp_head_param_floats(int K0, int N1, int N2, int S, int T);
int64_t rs_mlp_head_workspace_floats(int64_t B, int K0, int N1, int N2, int S, int T);
int rs_mlp_head_partial_blocks(int64_t B);
int rs_mlp_head_train(void* stream, const float* x0, int64_t ldx, const float* il, int64_t ld_il,
                      int64_t B, int K0, int S, int N1, int act1, int N2, int act2, int T,
                      int act3, const float* W1, const float* b1, const float* W2,
                      const float* b2, const float* W3, const float* b3, const float* labels,
                      float clip_lo, float clip_hi, float log_eps, float* p_out, float* dil,
                      int64_t ld_dil, float* dx0, int64_t ld_dx, int dx_accumulate,
                      float* workspace, int64_t workspace_floats);
/* rs_mlp_head_train with the layer-1 weight gradient deferred: instead of a 16-row dW1 partial
 * per block (K0 x N1 floats: 57 KB per block at config 2) the kernel stores its layer-1 dz rows,
 * dz1[b * ld_dz1 + n] = dL/d(x0 W1 + b1)[b][n] (ld_dz1 >= N1), and the partial rows start at b1:
 * rs_mlp_head_dz_workspace_floats(...) = blocks x (rs_mlp_head_param_floats - K0 N1 + 1), arena
 * order [b1 W2 b2 W3 b3 | loss_sum].  dW1 = x0^T dz1 is formed by the InteractingLayer backward
 * that follows (rs_il_bwd_push_saved_xt / rs_il_bwd_saved_xt) as a few sample-range partial rows. */
int64_t rs_mlp_head_dz_workspace_floats(int64_t B, int K0, int N1, int N2, int S, int T);
int rs_mlp_head_train_dz(void* stream, const float* x0, int64_t ldx, const float* il,
                         int64_t ld_il, int64_t B, int K0, int S, int N1, int act1, int N2,
                         int act2, int T, int act3, const float* W1, const float* b1,
                         const float* W2, const float* b2, const float* W3, const float* b3,
                         const float* labels, float clip_lo, float clip_hi, float log_eps,
                         float* p_out, float* dil, int64_t ld_dil, float* dx0, int64_t ld_dx,
                         int dx_accumulate, float* workspace, int64_t workspace_floats,
                         float* dz1, int64_t ld_dz1);

/* Per-block gradient partials -> gradients (-> dense Adam), one launch (replaces the
 * column-reduce launches of the fused backward kernels plus rs_dense_adam and its step-increment
 * launch).  Segment k: partial rows parts[k][r * lds[k] + c] (r < nrows[k], c < ncols[k]) are
 * summed over r in a fixed order, scaled by scales[k] and written to outs[k][c]; if adam != 0 and
 * adam_offs[k] >= 0 the tf.keras-form Adam of rs_dense_adam is applied to arena element
 * adam_offs[k] + c with that gradient times grad_scale.  nseg <= 4.  step: device int64 Adam
 * counter (advanced once per launch); done: device int32[288] completion counters, zero between
 * launches (reset by the launch itself). */
int rs_partials_reduce_adam(void* stream, int nseg, const float* const* parts,
                            const int64_t* lds, const int32_t* nrows, const int64_t* ncols,
                            float* const* outs, const float* scales, const int64_t* adam_offs,
                            float* params, float* m, float* v, int64_t* step, int32_t* done,
                            float lr, float beta1, float beta2, float eps, float grad_scale,
                            int adam);
/* rs_partials_reduce_adam with the scan-mode sparse Adam of one table (rs_sparse_adam_scan:
 * table / m / v / grad_table / flag, lr / betas / eps / grad_scale) run by extra blocks of the
 * SAME launch: the dense reduction + Adam and the sparse flag sweep are independent, so they
 * share the chip instead of running back to back (the AutoInt step's optimizer tail). */
/* rs_partials_reduce_adam_scan whose sparse part walks the step's looked-up rows (rows[0 .. nlist),
 * -1 = none) instead of sweeping flag[]: each marked row is updated once (its flag released by an
 * atomic exchange).  Valid only when those rows are the only rows marked -- the single-GPU AutoInt
 * step, whose own push marks exactly them; dim / 4 a power of two, dim <= 256. */
int rs_partials_reduce_adam_rows(void* stream, int nseg, const float* const* parts,
                                 const int64_t* lds, const int32_t* nrows, const int64_t* ncols,
                                 float* const* outs, const float* scales, const int64_t* adam_offs,
                                 float* params, float* m, float* v, int64_t* step, int32_t* done,
                                 float lr, float beta1, float beta2, float eps, float grad_scale,
                                 int adam, float* table, float* tm, float* tv, float* grad_table,
                                 int32_t* flag, int64_t table_rows, int dim, float slr,
                                 float sbeta1, float sbeta2, float seps, float sgrad_scale,
                                 const int32_t* rows, int64_t nlist);
/* rs_partials_reduce_adam_rows over strided entries rows[i * list_stride] (i < nlist) of which,
 * when counts != NULL, segment s = i / seg_len holds counts[s * counts_stride] valid entries (the
 * packed DP records after the all-gather: rank r's [row | grad] records at r * cap, its count in
 * the gathered dense bucket) -- the marked rows of a data-parallel step are exactly those. */
int rs_partials_reduce_adam_rows_ex(void* stream, int nseg, const float* const* parts,
                                    const int64_t* lds, const int32_t* nrows, const int64_t* ncols,
                                    float* const* outs, const float* scales,
                                    const int64_t* adam_offs, float* params, float* m, float* v,
                                    int64_t* step, int32_t* done, float lr, float beta1,
                                    float beta2, float eps, float grad_scale, int adam,
                                    float* table, float* tm, float* tv, float* grad_table,
                                    int32_t* flag, int64_t table_rows, int dim, float slr,
                                    float sbeta1, float sbeta2, float seps, float sgrad_scale,
                                    const int32_t* rows, int64_t nlist, int64_t list_stride,
                                    const int32_t* counts, int64_t counts_stride, int64_t seg_len);
int rs_partials_reduce_adam_scan(void* stream, int nseg, const float* const* parts,
                                 const int64_t* lds, const int32_t* nrows, const int64_t* ncols,
                                 float* const* outs, const float* scales, const int64_t* adam_offs,
                                 float* params, float* m, float* v, int64_t* step, int32_t* done,
                                 float lr, float beta1, float beta2, float eps, float grad_scale,
                                 int adam, float* table, float* tm, float* tv, float* grad_table,
                                 int32_t* flag, int64_t table_rows, int dim, float slr,
                                 float sbeta1, float sbeta2, float seps, float sgrad_scale);

/* rs_il_bwd with the sparse push fused into its last pass (F <= 64): dL/dx of the layer input
 * is not stored; instead grad_table[rows[b * F + f]] += dL/dx[b, f] (+ dx_base[b, f] when
 * dx_base != NULL, e.g. the deep tower's share of dL/dx0) with float atomics and the rows are
 * marked scan-mode (flag = -2).  Replaces rs_il_bwd(dx_accumulate = 1) followed by
 * rs_sparse_grad_accumulate(touched = NULL) for single-id fields (rows = lookup rows_out). */
int rs_il_bwd_push(void* stream, const float* x, const float* xsave, const float* dy,
                   int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L, const float* W,
                   const float* bias, const float* gamma, const float* beta, float eps,
                   int use_res, float drop_rate, uint64_t seed, const float* dx_base,
                   const int32_t* rows, float* grad_table, int32_t* flag, float* dparams,
                   int dparams_accumulate, float* workspace, int64_t workspace_floats);

/* The saved pair's fused-front-end forward and fused-push backward (asave as rs_il_fwd_saved /
 * rs_il_bwd_saved; the AutoInt trainer's launches). */
int rs_il_fwd_gather_saved(void* stream, const int64_t* ids, const int64_t* row_base,
                           const int64_t* bucket, int hash_mode, const float* table,
                           int64_t table_rows, float* x, int32_t* rows_out, int64_t B, int F,
                           int E, int U, int H, int L, const float* W, const float* bias,
                           const float* gamma, const float* beta, float eps, int use_res,
                           float drop_rate, uint64_t seed, float* y, int64_t y_ld, float* xsave,
                           float* asave, int64_t asave_floats);
int rs_il_bwd_push_saved(void* stream, const float* x, const float* xsave, const float* dy,
                         int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                         const float* W, const float* bias, const float* gamma, const float* beta,
                         float eps, int use_res, float drop_rate, uint64_t seed,
                         const float* dx_base, const int32_t* rows, float* grad_table,
                         int32_t* flag, float* dparams, int dparams_accumulate, float* workspace,
                         int64_t workspace_floats, const float* asave, int64_t asave_floats);
/* rs_il_bwd_saved / rs_il_bwd_push_saved carrying a deferred weight gradient (the fused head's
 * dW1, rs_mlp_head_train_dz): besides the InteractingLayer backward, the launch's waves first
 * form xt_slab[sp][k][n] = sum over sample range sp of xt_x[b][k] xt_dz[b][n] for
 * sp < rs_il_xt_splits(B) (equal ranges of the batch, a function of B alone), k < xt_K0,
 * n < xt_N1 (xt_K0 % 16 == 0, xt_N1 % 16 == 0; row strides xt_ldx >= xt_K0, xt_lddz >= xt_N1);
 * xt_slab holds rs_il_xt_splits(B) x xt_K0 x xt_N1 floats, summed in range order by the
 * optimizer tail (rs_partials_reduce_adam*).  Shapes whose backward has no such kernel (no
 * attention save, F > 32, H != 2) return RS_ERR_UNSUPPORTED. */
int rs_il_xt_splits(int64_t B);
/* The grid rs_il_bwd_(push_)saved_xt would use for this shape (> 0), or 0 when the shape's
 * saved backward cannot carry the deferred weight gradient. */
int rs_il_bwd_xt_supported(int64_t B, int F, int E, int U, int H, int64_t workspace_floats);
int rs_il_bwd_saved_xt(void* stream, const float* x, const float* xsave, const float* dy,
                       int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L, const float* W,
                       const float* bias, const float* gamma, const float* beta, float eps,
                       int use_res, float drop_rate, uint64_t seed, float* dx, int dx_accumulate,
                       float* dparams, int dparams_accumulate, float* workspace,
                       int64_t workspace_floats, const float* asave, int64_t asave_floats,
                       const float* xt_x, int64_t xt_ldx, const float* xt_dz, int64_t xt_lddz,
                       int xt_K0, int xt_N1, float* xt_slab);
int rs_il_bwd_push_saved_xt(void* stream, const float* x, const float* xsave, const float* dy,
                            int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                            const float* W, const float* bias, const float* gamma,
                            const float* beta, float eps, int use_res, float drop_rate,
                            uint64_t seed, const float* dx_base, const int32_t* rows,
                            float* grad_table, int32_t* flag, float* dparams,
                            int dparams_accumulate, float* workspace, int64_t workspace_floats,
                            const float* asave, int64_t asave_floats, const float* xt_x,
                            int64_t xt_ldx, const float* xt_dz, int64_t xt_lddz, int xt_K0,
                            int xt_N1, float* xt_slab);

/* Grid (= number of per-block partial rows) rs_il_bwd / rs_il_bwd_push use for this shape and
 * workspace when dy rows are 16-B aligned (dy_ld % 4 == 0); 0 for an unsupported shape. */
int rs_il_bwd_partial_blocks(int64_t B, int F, int E, int U, int H, int64_t workspace_floats);
/* The same for the saved entry points (rs_il_bwd_saved / rs_il_bwd_push_saved with the forward's
 * attention save): shapes that have a save run other kernels with their own grid. */
int rs_il_bwd_saved_partial_blocks(int64_t B, int F, int E, int U, int H,
                                   int64_t workspace_floats);


/* ---------------------------------------------------------------------------------------
 * H2 / H12 / H13  rank/ctr BaseModel front end and the rank/ctr, rank/finish model pieces
 * (csrc/front_end.hip).  fp32, row-major, explicit leading dimensions ("_ld").
 * ------------------------------------------------------------------------------------- */
/* emb_dict[slot][:, s0:s1] slicing + Concatenate (rank/ctr/base_model.py:134-154): out[b*out_ld
 * + j] = src[b*src_ld + cols[j]] for a column plan (feature_config.SlotLayout.column_plan). */
int rs_gather_columns(void* stream, const float* src, int64_t src_ld, int64_t B,
                      const int32_t* cols, int ncols, float* out, int64_t out_ld);
/* its backward: dsrc[b*src_ld + cols[j]] += dout[b*out_ld + j] (atomic adds: a column named
 * twice in a plan receives both gradients). */
int rs_scatter_add_columns(void* stream, const float* dout, int64_t out_ld, int64_t B,
                           const int32_t* cols, int ncols, float* dsrc, int64_t src_ld);
/* The backward of several column gathers from ONE source, as one gather: out[b, c] = sum_k
 * (map[k*ncols + c] >= 0 ? srcs[k][b*src_lds[k] + map[k*ncols + c]] : 0), every out element
 * written once.  srcs / src_lds are HOST arrays (nsrc <= 8) of device pointers / row strides;
 * map is a device int32 [nsrc, ncols].  (staytime trunk fan-out, VideoDnn.py:45-47,57-77,127) */
int rs_gather_sum_columns(void* stream, int nsrc, const float* const* srcs, const int64_t* src_lds,
                          const int32_t* map, int64_t B, int ncols, float* out, int64_t out_ld);
/* SENet squeeze tf.reduce_mean(emb, axis=1, keepdims=True) per structure field
 * (rank/ctr/model_init.py:22-24): out[b*out_ld + f] = mean(x[b, seg[f] .. seg[f+1])). */
int rs_segment_mean(void* stream, const float* x, int64_t x_ld, int64_t B, const int32_t* seg,
                    int F, float* out, int64_t out_ld);
/* multiply([emb_input, senet_split_output]) per field with senet_output = alpha * s
 * (rank/ctr/model_init.py:31-40, alpha = 2): y[b, c] = x[b, c] * (alpha * s[b, colfield[c]]). */
int rs_field_scale_fwd(void* stream, const float* x, int64_t x_ld, int64_t B,
                       const int32_t* colfield, int C, const float* s, int64_t s_ld, float alpha,
                       float* y, int64_t y_ld);
/* its backward: dx[b, c] (+)= dy[b, c] alpha s[b, f(c)] (dx nullable), ds[b, f] = alpha sum_c dy x
 * (nullable). */
int rs_field_scale_bwd(void* stream, const float* dy, int64_t dy_ld, const float* x, int64_t x_ld,
                       int64_t B, const int32_t* seg, int F, const float* s, int64_t s_ld,
                       float alpha, float* dx, int64_t dx_ld, int dx_accumulate, float* ds,
                       int64_t ds_ld);
/* The per-field Dense(O) maps emb_linear_map_i (rank/ctr/model_init.py:44-46): y[b, f*O + o] =
 * sum_{c in [seg[f], seg[f+1])} x[b, c] W[c*O + o] + bias[f*O + o]; W packs every field's
 * [w_f, O] kernel as one [C, O] matrix. */
int rs_field_linear_fwd(void* stream, const float* x, int64_t x_ld, int64_t B, const int32_t* seg,
                        int F, int O, const float* W, const float* bias, float* y, int64_t y_ld);
int64_t rs_field_linear_workspace_floats(int64_t B, int C, int F, int O);
/* its backward: dx (nullable, += with dx_accumulate), dW [C, O], db [F, O] (fixed-order batch
 * reduction through the workspace). */
int rs_field_linear_bwd(void* stream, const float* dy, int64_t dy_ld, const float* x, int64_t x_ld,
                        int64_t B, const int32_t* seg, const int32_t* colfield, int C, int F, int O,
                        const float* W, float* dx, int64_t dx_ld, int dx_accumulate, float* dW,
                        float* db, int dparams_accumulate, float* workspace,
                        int64_t workspace_floats);
/* CAN per-sample matmuls (rank/ctr/model_init.py:90-98, 150-154): out = relu(relu(r W1 + b1) W2
 * + b2), W1 [8,6] | b1 [6] | W2 [6,4] | b2 [4] = the 82 columns of each sample's p row
 * (tf.split + tf.reshape, row-major).  h_save [B, 6] (nullable) keeps relu(r W1 + b1). */
int rs_can_fwd(void* stream, const float* r, int64_t r_ld, const float* p, int64_t p_ld, int64_t B,
               float* out, int64_t out_ld, float* h_save);
int rs_can_bwd(void* stream, const float* dout, int64_t dout_ld, const float* out, int64_t out_ld,
               const float* r, int64_t r_ld, const float* p, int64_t p_ld, const float* h,
               int64_t B, float* dr, int64_t dr_ld, int dr_accumulate, float* dp, int64_t dp_ld);
/* rank/finish FMLayer (rank/finish/videodnn.py:41-50): y[b] = 0.5 * sum_n ((x V)_n^2 -
 * (x^2 V^2)_n) + add[b], V = fm_matrix [K, N] (N = 4, 8, 16); add (nullable) = the layer's
 * Dense(1) linear term (rs_dense_fwd output); xv_save [B, N] nullable (needed by the backward). */
int rs_fm_proj_fwd(void* stream, const float* x, int64_t x_ld, int64_t B, int K, int N,
                   const float* V, const float* add, float* y, float* xv_save);
int64_t rs_fm_proj_workspace_floats(int64_t B, int K, int N);
int rs_fm_proj_bwd(void* stream, const float* dy, const float* x, int64_t x_ld, int64_t B, int K,
                   int N, const float* V, const float* xv, float* dx, int64_t dx_ld,
                   int dx_accumulate, float* dV, int dV_accumulate, float* workspace,
                   int64_t workspace_floats);

/* ---------------------------------------------------------------------------------------
 * Training metrics: Keras 'acc' / BinaryAccuracy(), tf.keras.metrics.AUC() and
 * tensornet tn.metric.COPC() / CTR() of the reference's model.compile calls
 * (rank/ctr/base_model.py:183-190, rough_rank/model.py:215-219, rank/multi_head/model.py:55,
 * staytime/model.py:81-82).  state: fp64 [rs_ctr_metrics_state_doubles(nthr)], zeroed by the
 * caller; rs_ctr_metrics_accumulate adds one batch (p / y / w columns with row strides; w
 * nullable = unit weights; AUC positives are y != 0, Keras's bool cast); rs_ctr_metrics_result
 * writes out[6] = {AUC (Keras: nthr thresholds, ROC, interpolation), binary accuracy (p > 0.5),
 * COPC = sum(w y) / sum(w p), CTR = sum(w y) / sum(w), mean prediction, total weight}.
 * ------------------------------------------------------------------------------------- */
int64_t rs_ctr_metrics_state_doubles(int nthr);
int rs_ctr_metrics_accumulate(void* stream, const float* p, int64_t p_ld, const float* y,
                              int64_t y_ld, const float* w, int64_t w_ld, int64_t B, int nthr,
                              double* state);
int rs_ctr_metrics_result(void* stream, const double* state, int nthr, float* out);

#ifdef __cplusplus
}
#endif

#endif /* RECSYS_AMD_H_ */
