// H1/H2 — sparse embedding lookup + concat front end, and the sparse-gradient half of the
// tensornet boundary.
//
// Reference behaviour being replaced:
//   tn.feature_column.category_column(key, bucket_size) + tf.feature_column.embedding_column(
//     dimension, combiner='mean') + tn.layers.EmbeddingFeatures(columns, sparse_opt)(inputs)
//   rank/ctr/base_model.py:203-217, rank/multi_head/multidnn.py:221-238,
//   staytime/VideoDnn.py:217-244, rough_rank/model.py:89-115, rank/finish/videodnn.py:53-68
// and the expand + Concatenate(axis=1) that follows (autoint:22-26, multidnn.py:25-27,50),
// which is folded into the store: every field's pooled row is written straight into its slot of
// the [B, F, dim] (or wider) activation.
//
// id -> row: tensornet's key->row map is not vendored, so the framework pins a documented hash
// (identical in oracle/ctr_oracle.py::hash_rows):
//   RS_HASH_MOD      row = row_base[f] + (uint64)id % bucket[f]
//   RS_HASH_SPLITMIX row = row_base[f] + splitmix64((uint64)id) % bucket[f]
// Pooling ('mean' | 'sum' | 'sqrtn') sums rows in id order in fp32, then scales; an empty
// segment yields zeros (tf.nn.embedding_lookup_sparse semantics).
//
// Layout in HBM: table [rows, dim] fp32 row-major (64 B rows at dim 16 -> one float4 per lane,
// dim/4 lanes per segment, 64/(dim/4) segments per wave instruction: a wave reads 16 whole rows
// and writes 1 KiB of contiguous [B, F, 16] output per step at config 2).
#include "common.hpp"

// RS_HASH_* and hash_row live in common.hpp (shared with the InteractingLayer's fused gather)
enum { RS_COMBINER_SUM = 0, RS_COMBINER_MEAN = 1, RS_COMBINER_SQRTN = 2 };

__device__ __forceinline__ float combiner_scale(int n, int combiner) {
  if (n <= 0) return 0.f;
  if (combiner == RS_COMBINER_MEAN) return 1.0f / (float)n;
  if (combiner == RS_COMBINER_SQRTN) return 1.0f / sqrtf((float)n);
  return 1.0f;
}

// One group of G lanes (G = dim/4 capped at 64, float4 each) pools one (b, f) segment.
template <int G>
__global__ void __launch_bounds__(256) embed_lookup_fwd_kernel(
    const int64_t* __restrict__ ids, const int32_t* __restrict__ offsets, int64_t nseg, int F,
    const int64_t* __restrict__ row_base, const int64_t* __restrict__ bucket, int hash_mode,
    int combiner, const float* __restrict__ table, int64_t table_rows, int dim,
    float* __restrict__ out, int64_t out_ld, int64_t out_fstride, int32_t* __restrict__ rows_out) {
  const int groups_per_block = blockDim.x / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int nvec = dim >> 2;
  for (int64_t s = (int64_t)blockIdx.x * groups_per_block + g; s < nseg;
       s += (int64_t)gridDim.x * groups_per_block) {
    // segment -> (b, f) in 32 bits when it fits (launch sizes here are far below 2^31)
    int f;
    int64_t b;
    if (nseg <= INT32_MAX) {
      const uint32_t s32 = (uint32_t)s, b32 = s32 / (uint32_t)F;
      b = b32;
      f = (int)(s32 - b32 * (uint32_t)F);
    } else {
      f = (int)(s % F);
      b = s / F;
    }
    const int64_t beg = offsets ? offsets[s] : s;
    const int64_t end = offsets ? offsets[s + 1] : s + 1;
    const int64_t base = row_base[f], bk = bucket[f];
    if (!table) {  // rows only (owner-sharded tables gather remotely): no table read, no store
      if (l == 0)
        for (int64_t k = beg; k < end; ++k) {
          const int64_t row = hash_row(ids[k], base, bk, hash_mode);
          rows_out[k] = (row >= 0 && row < table_rows) ? (int32_t)row : -1;
        }
      continue;
    }
    float* dst = out + b * out_ld + (int64_t)f * out_fstride;
    for (int v0 = 0; v0 < nvec; v0 += G) {
      const int v = v0 + l;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int64_t k = beg; k < end; ++k) {
        const int64_t row = hash_row(ids[k], base, bk, hash_mode);
        // a (row_base, bucket) pair outside the table (the C ABI cannot check device arrays on
        // the host): the id contributes nothing and its row index is -1, which every push skips
        const bool ok = row >= 0 && row < table_rows;
        if (v0 == 0 && l == 0 && rows_out) rows_out[k] = ok ? (int32_t)row : -1;
        if (ok && v < nvec) {
          const float4 t = reinterpret_cast<const float4*>(table + row * dim)[v];
          acc.x += t.x; acc.y += t.y; acc.z += t.z; acc.w += t.w;
        }
      }
      const float sc = combiner_scale((int)(end - beg), combiner);
      if (v < nvec) {
        if (combiner != RS_COMBINER_SUM) { acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc; }
        reinterpret_cast<float4*>(dst)[v] = acc;
      }
    }
  }
}

RS_API int rs_embedding_lookup_fwd(void* stream, const int64_t* ids, const int32_t* offsets,
                                   int64_t B, int F, const int64_t* row_base,
                                   const int64_t* bucket, int hash_mode, int combiner,
                                   const float* table, int64_t table_rows, int dim, float* out,
                                   int64_t out_ld, int64_t out_fstride, int32_t* rows_out) {
  // table == out == NULL: rows-only mode (rows_out required), the id -> row half of the lookup
  const bool rows_only = !table && !out;
  if (!ids || !row_base || !bucket || B < 0 || F <= 0 || dim <= 0) return RS_ERR_ARG;
  if (rows_only ? !rows_out : (!table || !out)) return RS_ERR_ARG;
  if (table_rows <= 0 || table_rows > INT32_MAX) return RS_ERR_ARG;  // rows_out is int32
  if (dim % 4 != 0 || out_ld % 4 != 0 || out_fstride % 4 != 0) return RS_ERR_ARG;
  const int64_t nseg = B * (int64_t)F;
  if (nseg == 0) return RS_OK;
  const int nvec = dim / 4;
  int G = 1;
  while (G < nvec && G < 64) G <<= 1;
  const int block = 256;
  int64_t grid = (nseg * G + block - 1) / block;
  if (grid > 8192) grid = 8192;
  hipStream_t s = rs_stream(stream);
#define RS_LAUNCH_EMB(GG)                                                                         \
  case GG:                                                                                        \
    embed_lookup_fwd_kernel<GG><<<(int)grid, block, 0, s>>>(ids, offsets, nseg, F, row_base,      \
                                                            bucket, hash_mode, combiner, table,  \
                                                            table_rows, dim, out, out_ld,         \
                                                            out_fstride,                          \
                                                            rows_out);                            \
    break;
  switch (G) {
    RS_LAUNCH_EMB(1) RS_LAUNCH_EMB(2) RS_LAUNCH_EMB(4) RS_LAUNCH_EMB(8) RS_LAUNCH_EMB(16)
    RS_LAUNCH_EMB(32) RS_LAUNCH_EMB(64)
    default: return RS_ERR_UNSUPPORTED;
  }
#undef RS_LAUNCH_EMB
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Sequence lookup (embedding_column(combiner=None, seq_max_len) -> (emb3d, mask);
// staytime/VideoDnn.py:217-244, consumed at :58-68; the DIN keys of din.py at config 4).
// Sample b's ids are ids[offsets[b] .. offsets[b+1]); the first T are looked up (pinned), the
// rest of the [T, dim] block is zero, mask[b, t] = t < n_b, rows_out = -1 on padding so the
// sparse push (rows < 0 skipped) needs no separate path.  One G-lane group per position.
// ---------------------------------------------------------------------------------------------
template <int G>
__global__ void __launch_bounds__(256) seq_lookup_fwd_kernel(
    const int64_t* __restrict__ ids, const int32_t* __restrict__ offsets, int64_t B, int T,
    int64_t row_base, int64_t bucket, int hash_mode, const float* __restrict__ table, int dim,
    float* __restrict__ out, int64_t out_ss, int64_t out_rs, uint8_t* __restrict__ mask,
    int64_t mask_ld, int32_t* __restrict__ lengths, int32_t* __restrict__ rows_out) {
  const int groups_per_block = blockDim.x / G;
  const int g = threadIdx.x / G;
  const int l = threadIdx.x % G;
  const int nvec = dim >> 2;
  const int64_t npos = B * (int64_t)T;
  for (int64_t p = (int64_t)blockIdx.x * groups_per_block + g; p < npos;
       p += (int64_t)gridDim.x * groups_per_block) {
    const int64_t b = p / T;
    const int t = (int)(p - b * T);
    const int64_t beg = offsets[b];
    int64_t n = offsets[b + 1] - beg;
    if (n > T) n = T;
    const bool on = t < n;
    int64_t row = -1;
    if (on) row = hash_row(ids[beg + t], row_base, bucket, hash_mode);
    if (table) {  // NULL table and out: rows / mask / lengths only
      float* dst = out + b * out_ss + (int64_t)t * out_rs;
      for (int v = l; v < nvec; v += G) {
        float4 val = make_float4(0.f, 0.f, 0.f, 0.f);
        if (on) val = reinterpret_cast<const float4*>(table + row * dim)[v];
        reinterpret_cast<float4*>(dst)[v] = val;
      }
    }
    if (l == 0) {
      if (rows_out) rows_out[p] = (int32_t)row;
      if (mask) mask[b * mask_ld + t] = on ? 1 : 0;
      if (lengths && t == 0) lengths[b] = (int32_t)n;
    }
  }
}

RS_API int rs_sequence_lookup_fwd(void* stream, const int64_t* ids, const int32_t* offsets,
                                  int64_t B, int T, int64_t row_base, int64_t bucket,
                                  int hash_mode, const float* table, int dim, float* out,
                                  int64_t out_ss, int64_t out_rs, uint8_t* mask, int64_t mask_ld,
                                  int32_t* lengths, int32_t* rows_out) {
  if (!offsets || B < 0 || T <= 0 || dim <= 0 || bucket <= 0) return RS_ERR_ARG;
  if ((!table) != (!out) || (!table && !rows_out)) return RS_ERR_ARG;  // rows-only: both NULL
  if (dim % 4 != 0 || out_ss % 4 != 0 || out_rs % 4 != 0) return RS_ERR_ARG;
  const int64_t npos = B * (int64_t)T;
  if (npos == 0) return RS_OK;
  const int nvec = dim / 4;
  int G = 1;
  while (G < nvec && G < 64) G <<= 1;
  const int block = 256;
  int64_t grid = (npos * G + block - 1) / block;
  if (grid > 8192) grid = 8192;
  hipStream_t s = rs_stream(stream);
#define RS_LAUNCH_SEQ(GG)                                                                         \
  case GG:                                                                                        \
    seq_lookup_fwd_kernel<GG><<<(int)grid, block, 0, s>>>(ids, offsets, B, T, row_base, bucket,   \
                                                          hash_mode, table, dim, out, out_ss,     \
                                                          out_rs, mask, mask_ld, lengths,         \
                                                          rows_out);                              \
    break;
  switch (G) {
    RS_LAUNCH_SEQ(1) RS_LAUNCH_SEQ(2) RS_LAUNCH_SEQ(4) RS_LAUNCH_SEQ(8) RS_LAUNCH_SEQ(16)
    RS_LAUNCH_SEQ(32) RS_LAUNCH_SEQ(64)
    default: return RS_ERR_UNSUPPORTED;
  }
#undef RS_LAUNCH_SEQ
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Sparse gradient accumulation (the "push" half of EmbeddingFeatures): every occurrence k of
// segment s adds scale(s) * dout[s] into grad_table[rows[k]].
//
// MI355X mapping: a block owns one field f and a tile of samples.  Phase 1 inserts each id's row
// into an LDS open-addressing table (CAS on the key) and adds the scaled gradient row into the
// slot with LDS float atomics; phase 2 flushes every occupied slot with ONE global float-atomic
// row add and claims the row for the optimizer (flag -1 -> -2, append to `touched`).  Zipf-hot
// ids (the top id of a field is ~18% of a Criteo-like batch) thus cost one global add per block
// instead of one per occurrence -- global atomics on one row serialise at the memory side.
// If the LDS table ever fills (long multi-hot tiles), the occurrence falls back to direct global
// atomics.  The row SET is exact; the fp32 summation order is not fixed (last-bit run-to-run
// differences).  Replicas stay identical because the cross-rank merge (rs_sparse_merge_rows)
// is rank-ordered and atomic-free.
// ---------------------------------------------------------------------------------------------
#ifdef RS_PUSH_KO_FLUSH  // timing experiments only (tools/push_prof.sh): flush by plain stores
#define RS_FLUSH_ADD(p, v) (*(p) = (v))
#else
#define RS_FLUSH_ADD(p, v) atomicAdd((p), (v))
#endif
__device__ __forceinline__ void claim_row(int32_t row, int32_t* flag, int32_t* touched,
                                          int32_t* n_touched, int32_t touched_cap) {
  if (atomicCAS(&flag[row], -1, -2) == -1) {
    const int32_t u = atomicAdd(n_touched, 1);
    if (u < touched_cap) touched[u] = row;
  }
}

__global__ void __launch_bounds__(1024) sparse_grad_accum_kernel(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ offsets, int64_t B, int F,
    const float* __restrict__ dout, int64_t dout_ld, int64_t dout_fstride, int dim, int combiner,
    int G, int tile, int cap, float* __restrict__ grad_table, int32_t* __restrict__ flag,
    int32_t* __restrict__ touched, int32_t* __restrict__ n_touched, int32_t touched_cap) {
  extern __shared__ __attribute__((aligned(16))) int32_t sm[];
  int32_t* ctl = sm;                                    // [4]: claim count, range base
  int32_t* keys = sm + 4;                               // [cap]  (lidx[cap] follows)
  float* vals = reinterpret_cast<float*>(sm + 4 + 2 * cap);  // [cap][dim]
  for (int k = threadIdx.x; k < cap; k += blockDim.x) keys[k] = -1;
  for (int k = threadIdx.x; k < cap * dim; k += blockDim.x) vals[k] = 0.f;
  __syncthreads();
  const int f = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * tile;
  const int64_t b1 = b0 + tile < B ? b0 + tile : B;
  const int per_pass = blockDim.x / G;
  const int gsub = threadIdx.x / G, l = threadIdx.x % G;
  const int leader = (threadIdx.x & 63) - l;  // lane of this group's leader within the wave
  // ---- phase 1: aggregate this tile's occurrences per row in LDS ----
  // insert one occurrence (the group's leader probes the LDS table; the group adds its elements)
  auto insert = [&](int32_t row, const float* src, float sc, float v0) {
    int slot = -1;
    if (l == 0) {
      int h = (int)(((uint32_t)row * 2654435761u) & (uint32_t)(cap - 1));
      for (int probe = 0; probe < cap; ++probe) {
        const int32_t old = atomicCAS(&keys[h], -1, row);
        if (old == -1 || old == row) { slot = h; break; }
        h = (h + 1) & (cap - 1);
      }
    }
    slot = __shfl(slot, leader, 64);
    if (slot >= 0) {
      if (src) for (int e = l; e < dim; e += G) atomicAdd(&vals[slot * dim + e], src[e] * sc);
      else if (l < dim) atomicAdd(&vals[slot * dim + l], v0);
    } else {  // LDS table full: direct global path
      if (l == 0) {
        if (touched) claim_row(row, flag, touched, n_touched, touched_cap);
        else scan_mark(flag, row);
      }
      if (src) for (int e = l; e < dim; e += G) atomicAdd(grad_table + (int64_t)row * dim + e, src[e] * sc);
      else if (l < dim) atomicAdd(grad_table + (int64_t)row * dim + l, v0);
    }
  };
  if (!offsets && dim <= G) {
    // single-hot fast path: the rows and gradient elements of CH passes are loaded before any of
    // them is inserted, so one HBM/L2 round trip covers CH samples per group (the per-pass
    // dependent load -> probe -> add chain made this launch latency-bound)
    constexpr int CH = 8;
    const float sc = combiner_scale(1, combiner);
    for (int64_t bb = b0 + gsub; bb < b1; bb += (int64_t)per_pass * CH) {
      int32_t rw[CH];
      float vv[CH];
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        const int64_t b = bb + (int64_t)u * per_pass;
        rw[u] = -1;
        vv[u] = 0.f;
        if (b < b1) {
          rw[u] = rows[b * F + f];
          if (l < dim) vv[u] = dout[b * dout_ld + (int64_t)f * dout_fstride + l] * sc;
        }
      }
#pragma unroll
      for (int u = 0; u < CH; ++u)
        if (rw[u] >= 0) insert(rw[u], nullptr, 0.f, vv[u]);
    }
  } else {
    for (int64_t b = b0 + gsub; b < b1; b += per_pass) {
      const int64_t sg = b * F + f;
      const int64_t beg = offsets ? offsets[sg] : sg;
      const int64_t end = offsets ? offsets[sg + 1] : sg + 1;
      if (end <= beg) continue;
      const float sc = combiner_scale((int)(end - beg), combiner);
      const float* src = dout + b * dout_ld + (int64_t)f * dout_fstride;
      for (int64_t k = beg; k < end; ++k) {
        const int32_t row = rows[k];
        if (row < 0) continue;  // padded sequence position (rs_sequence_lookup_fwd)
        insert(row, src, sc, 0.f);
      }
    }
  }
  __syncthreads();
  if (!touched) {
    // scan mode (touched == NULL): mark rows with a plain store (idempotent; no claims, no shared
    // counter); the scan-mode optimizer finds them by sweeping flag[]
    for (int slot = gsub; slot < cap; slot += per_pass) {
      const int32_t row = keys[slot];
      if (row < 0) continue;
      if (l == 0) scan_mark(flag, row);
      float* dst = grad_table + (int64_t)row * dim;
      for (int e = l; e < dim; e += G) RS_FLUSH_ADD(dst + e, vals[slot * dim + e]);
    }
    return;
  }
  // ---- phase 2: claim each distinct row once (flag CAS); the claims of the whole block take ONE
  //      global atomic on n_touched (a single counter word serialises ~11 ns per atomic at the
  //      memory side: 30k per-row increments would cost ~0.3 ms) ----
  int32_t* lidx = keys + cap;  // reuse: vals region follows; lidx lives in the extra cap ints
  int32_t& nclaim = ctl[0];
  int32_t& base = ctl[1];
  if (threadIdx.x == 0) nclaim = 0;
  __syncthreads();
  for (int s0 = threadIdx.x; s0 < cap; s0 += 4 * blockDim.x) {
    // four returning flag CASes in flight per thread (each is a memory-side round trip)
    int32_t rw[4], old[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int slot = s0 + u * blockDim.x;
      rw[u] = slot < cap ? keys[slot] : -1;
    }
#pragma unroll
#ifdef RS_PUSH_KO_CLAIM  // timing experiments only: no claim CASes
    for (int u = 0; u < 4; ++u) old[u] = 0;
#else
    for (int u = 0; u < 4; ++u) old[u] = rw[u] >= 0 ? atomicCAS(&flag[rw[u]], -1, -2) : 0;
#endif
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int slot = s0 + u * blockDim.x;
      if (slot < cap) lidx[slot] = (rw[u] >= 0 && old[u] == -1) ? atomicAdd(&nclaim, 1) : -1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) base = nclaim > 0 ? atomicAdd(n_touched, nclaim) : 0;
  __syncthreads();
  for (int slot = gsub; slot < cap; slot += per_pass) {
    const int32_t row = keys[slot];
    if (row < 0) continue;
    if (l == 0) {
      const int32_t li = lidx[slot];
      if (li >= 0 && base + li < touched_cap) touched[base + li] = row;
    }
    float* dst = grad_table + (int64_t)row * dim;
    for (int e = l; e < dim; e += G) RS_FLUSH_ADD(dst + e, vals[slot * dim + e]);
  }
}

// ---------------------------------------------------------------------------------------------
// Single-hot push with claims by ELECTION (rs_sparse_grad_accumulate_ws, offsets == NULL).
// PMC/timing (tools/push_prof.sh, config-4 history: 53 K ids over a 1 M-row table) split the
// atomic push's 38 us: the returning flag CASes of list mode cost most of it -- every block
// claims its hot rows, so the Zipf-hot rows' flag words take one returning CAS per block, and
// those serialise at the memory side.  Here claims take no atomics on flag words:
//   push:  block (field f, tile of samples) aggregates its occurrences in an LDS hash (one lane
//          per occurrence probes; LP lanes per occurrence add its float4s with LDS atomics; all
//          gradient loads issued before any add), then per distinct row: one global float-atomic
//          row add, and -- unless the row is already claimed (flag == -2) -- a PLAIN store
//          flag[row] = block id (the last store wins: exactly one block is elected per row) and
//          the row goes to the block's candidate list in the workspace;
//   claim: one block per push block re-reads its candidates; the elected block (flag == its id)
//          claims the row (flag = -2) and appends it to touched with one n_touched atomic per
//          block.  Single-hot tiles of T samples hold <= T distinct rows, so the 2T-slot LDS
//          table never fills (no fallback path that could claim a row twice).
// Scan mode (touched == NULL) skips the election and marks flag = -2 with plain stores.
// Row set exact; fp32 summation order not fixed (as the CAS push).
// ---------------------------------------------------------------------------------------------
RS_API int rs_sparse_grad_accumulate(void* stream, const int32_t* rows, const int32_t* offsets,
                                     int64_t B, int F, const float* dout, int64_t dout_ld,
                                     int64_t dout_fstride, int dim, int combiner,
                                     float* grad_table, int32_t* flag, int32_t* touched,
                                     int32_t* n_touched, int32_t touched_cap);

namespace rs_push {
#ifndef RS_PUSH_THREADS  // tuning builds only (tools/push_bench.py variants)
// 512: same-box push_bench medians vs 256 -- config-4 history (scan) 24.2 -> 22.7 us, config-5
// 91-field push 94.3 -> 85.6 us; a deeper chunk (8) measured no better
#define RS_PUSH_THREADS 512
#endif
#ifndef RS_PUSH_TILE
#define RS_PUSH_TILE 256
#endif
#ifndef RS_PUSH_CHUNK
#define RS_PUSH_CHUNK 4
#endif
constexpr int kThreads = RS_PUSH_THREADS;
constexpr int kTile = RS_PUSH_TILE;           // samples (= occurrences) per block
constexpr int kCap = 2 * kTile;               // LDS hash slots: never full
constexpr int kChunk = RS_PUSH_CHUNK;         // occurrences per lane group in flight

__host__ __device__ constexpr size_t lds_bytes(int dim) {
  return (4 + (size_t)kCap * (2 + dim) + 2 * (size_t)kTile) * 4;
}

template <int LP>
__global__ void __launch_bounds__(kThreads) push_elect_kernel(
    const int32_t* __restrict__ rows, int64_t B, int F, const float* __restrict__ dout,
    int64_t dout_ld, int64_t dout_fstride, int dim, float sc, int tile,
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int32_t* __restrict__ ws_cnt,
    int32_t* __restrict__ ws_rows) {
  extern __shared__ __attribute__((aligned(16))) int32_t sm[];
  int32_t* ctl = sm;                                       // [4]
  int32_t* keys = ctl + 4;                                 // [kCap]
  int32_t* orow = keys + kCap;                             // [kTile]
  int32_t* oslot = orow + kTile;                           // [kTile]
  float* vals = reinterpret_cast<float*>(oslot + kTile);  // [kCap][dim]
  const int tid = threadIdx.x;
  const int cap = 2 * tile;  // tile is a power of two <= kTile
  for (int k = tid; k < cap; k += kThreads) keys[k] = -1;
  for (int k = tid; k < cap * dim; k += kThreads) vals[k] = 0.f;
  if (tid == 0) ctl[0] = 0;
  const int f = blockIdx.y;
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * tile;
  const int n = (int)((b0 + tile < B ? b0 + tile : B) - b0);
  for (int i = tid; i < n; i += kThreads) orow[i] = rows[(b0 + i) * F + f];
  __syncthreads();
  for (int i = tid; i < n; i += kThreads) {
    const int32_t row = orow[i];
    int slot = -1;
    if (row >= 0) {
      int h = (int)(((uint32_t)row * 2654435761u) & (uint32_t)(cap - 1));
      for (;;) {  // cap > tile >= distinct rows: terminates
        const int32_t old = atomicCAS(&keys[h], -1, row);
        if (old == -1 || old == row) { slot = h; break; }
        h = (h + 1) & (cap - 1);
      }
    }
    oslot[i] = slot;
  }
  __syncthreads();
  const int ng = kThreads / LP, g = tid / LP, l = tid % LP;
  const int nvec = dim >> 2;
  for (int i0 = g; i0 < n; i0 += ng * kChunk) {
    float4 v[kChunk];
    int slot[kChunk];
#pragma unroll
    for (int u = 0; u < kChunk; ++u) {
      const int i = i0 + u * ng;
      slot[u] = i < n ? oslot[i] : -1;
      v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (slot[u] >= 0 && l < nvec)
        v[u] = reinterpret_cast<const float4*>(dout + (b0 + i) * dout_ld +
                                               (int64_t)f * dout_fstride)[l];
    }
#pragma unroll
    for (int u = 0; u < kChunk; ++u) {
      if (slot[u] < 0) continue;
      const int i = i0 + u * ng;
      for (int e4 = l; e4 < nvec; e4 += LP) {
        const float4 t = e4 == l ? v[u]
                                 : reinterpret_cast<const float4*>(
                                       dout + (b0 + i) * dout_ld + (int64_t)f * dout_fstride)[e4];
        float* d = vals + slot[u] * dim + 4 * e4;
#ifdef RS_PUSH_KO_LDSADD  // timing experiments only: the LDS adds as plain LDS stores
        *reinterpret_cast<float4*>(d) = make_float4(t.x * sc, t.y * sc, t.z * sc, t.w * sc);
        continue;
#endif
        atomicAdd(d + 0, t.x * sc); atomicAdd(d + 1, t.y * sc);
        atomicAdd(d + 2, t.z * sc); atomicAdd(d + 3, t.w * sc);
      }
    }
  }
  __syncthreads();
  // election (list mode): every slot's flag word is loaded at once (<= 2 per lane, all in
  // flight), then the plain election stores and the candidate list; scan mode: plain marks
  {
    int32_t rw[kCap / kThreads], fl[kCap / kThreads];
#pragma unroll
    for (int u = 0; u < kCap / kThreads; ++u) {
      const int slot = tid + u * kThreads;
      rw[u] = slot < cap ? keys[slot] : -1;
      fl[u] = (rw[u] >= 0 && ws_cnt) ? flag[rw[u]] : -2;
    }
#pragma unroll
    for (int u = 0; u < kCap / kThreads; ++u) {
      if (rw[u] < 0) continue;
      if (!ws_cnt) {
        scan_mark(flag, rw[u]);
      } else if (fl[u] != -2) {  // not claimed by an earlier push: stand for election
        flag[rw[u]] = blk;
        ws_rows[(int64_t)blk * kCap + atomicAdd(&ctl[0], 1)] = rw[u];
      }
    }
  }
  // gradient rows: G2 lanes per row, one dword each
  int G2 = 1;
  while (G2 < dim && G2 < 64) G2 <<= 1;
  const int per_pass = kThreads / G2, gs = tid / G2, l2 = tid % G2;
  for (int slot = gs; slot < cap; slot += per_pass) {
    const int32_t row = keys[slot];
    if (row < 0) continue;
    float* dst = grad_table + (int64_t)row * dim;
    for (int e = l2; e < dim; e += G2) RS_FLUSH_ADD(dst + e, vals[slot * dim + e]);
  }
  if (ws_cnt) {
    __syncthreads();
    if (tid == 0) ws_cnt[blk] = ctl[0];
  }
}

// The same push with the tile's occurrences grouped by row through a counting sort instead of
// LDS float atomics (tools/push_prof.sh knockouts, profiles/r06/push/: with its LDS adds as plain
// LDS stores the config-5 91-field push takes 33 instead of 68 us -- a Zipf-hot row puts dozens
// of lanes of one instruction on the same LDS words, dim atomics per occurrence):
//   probe + rank (one LDS int atomic per occurrence) -> block scan over the slots (run starts,
//   kRun-occurrence work items) -> scatter the samples into their runs -> LP lanes per item sum
//   its occurrences' gradient elements in registers (all loads in flight) into an LDS partial row
//   -> per distinct row: the election / marks as above and ONE global float-atomic row add of its
//   items' partial rows summed in item order.
constexpr int kRun = 8;                        // occurrences per work item
constexpr int kItems = kTile + kTile / kRun;   // >= sum over rows of ceil(count / kRun)
static_assert(kCap <= kThreads, "one slot per thread in the scan");

__host__ __device__ constexpr size_t sort_lds_bytes(int dim) {
  return ((size_t)16 + 4 * (size_t)kCap + 4 * (size_t)kTile + kItems) * 4 +
         (size_t)kItems * dim * 4;
}

// Push sources of one launch (rs_sparse_grad_accumulate_group): a single-hot push per source
// ([B, F] rows, dout rows of dout_ld floats with fields dout_fstride apart) into ONE table; the
// grid's y index runs over every source's fields (source k owns y in [f0, f0 + F)), so the
// pushes of several layers into a shared table (config 5: 91 fields, 52 fields and three
// 50-position sequences) run as one launch and one claim launch instead of five of each.
constexpr int kMaxSrc = 8;
struct PushSrc {
  const int32_t* rows;
  const float* dout;
  int64_t dout_ld, dout_fstride, B;
  int F, f0;
};
struct PushSrcs {
  PushSrc s[kMaxSrc];
  int n;
};

template <int LP>
__global__ void __launch_bounds__(kThreads) push_sort_kernel(
    PushSrcs srcs, int dim, float sc, int tile,
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int32_t* __restrict__ ws_cnt,
    int32_t* __restrict__ ws_rows) {
  // this block's source (block-uniform; selected field by field so the argument block is never
  // indexed dynamically)
  const int y = (int)blockIdx.y;
  const int32_t* __restrict__ rows = srcs.s[0].rows;
  const float* __restrict__ dout = srcs.s[0].dout;
  int64_t dout_ld = srcs.s[0].dout_ld, dout_fstride = srcs.s[0].dout_fstride, B = srcs.s[0].B;
  int F = srcs.s[0].F, f0 = 0;
#pragma unroll
  for (int k = 1; k < kMaxSrc; ++k)
    if (k < srcs.n && y >= srcs.s[k].f0) {
      rows = srcs.s[k].rows; dout = srcs.s[k].dout; dout_ld = srcs.s[k].dout_ld;
      dout_fstride = srcs.s[k].dout_fstride; B = srcs.s[k].B; F = srcs.s[k].F; f0 = srcs.s[k].f0;
    }
  extern __shared__ __attribute__((aligned(16))) int32_t sm[];
  int32_t* ctl = sm;                                       // [16]: list count, wave sums
  float* part = reinterpret_cast<float*>(sm + 16);        // [kItems][dim] item partial rows
  int32_t* keys = sm + 16 + kItems * dim;                  // [kCap] row of each slot
  int32_t* cnt = keys + kCap;                              // [kCap] occurrences per slot
  int32_t* sstart = cnt + kCap;                            // [kCap] run start per slot
  int32_t* sitem = sstart + kCap;                          // [kCap] first item per slot
  int32_t* orow = sitem + kCap;                            // [kTile]
  int32_t* oslot = orow + kTile;                           // [kTile]
  int32_t* orank = oslot + kTile;                          // [kTile] rank within the row's run
  int32_t* ssamp = orank + kTile;                          // [kTile] samples sorted by row
  int32_t* items = ssamp + kTile;                          // [kItems] slot | chunk << 16
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int cap = 2 * tile;  // tile is a power of two <= kTile
  for (int k = tid; k < cap; k += kThreads) {
    keys[k] = -1;
    cnt[k] = 0;
  }
  if (tid == 0) ctl[0] = 0;
  const int f = y - f0;
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * tile;
  // (a source with fewer samples than the grid's widest leaves its last blocks empty: n = 0)
  const int n = b0 < B ? (int)((b0 + tile < B ? b0 + tile : B) - b0) : 0;
  for (int i = tid; i < n; i += kThreads) orow[i] = rows[(b0 + i) * F + f];
  __syncthreads();
  for (int i = tid; i < n; i += kThreads) {
    const int32_t row = orow[i];
    int slot = -1;
    if (row >= 0) {
      int h = (int)(((uint32_t)row * 2654435761u) & (uint32_t)(cap - 1));
      for (;;) {  // cap > tile >= distinct rows: terminates
        const int32_t old = atomicCAS(&keys[h], -1, row);
        if (old == -1 || old == row) { slot = h; break; }
        h = (h + 1) & (cap - 1);
      }
      orank[i] = atomicAdd(&cnt[slot], 1);
    }
    oslot[i] = slot;
  }
  __syncthreads();
  // runs and items: one slot per thread; counts and item counts scanned together (< 2^16 each)
  const int c = tid < cap ? cnt[tid] : 0;
  const int nq = (c + kRun - 1) / kRun;
  const int packed = c + (nq << 16);
  int inc = packed;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(inc, d, 64);
    if (lane >= d) inc += t;
  }
  if (lane == 63) ctl[8 + wv] = inc;
  __syncthreads();
  int pre = inc - packed, tot = 0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    if (w < wv) pre += ctl[8 + w];
    tot += ctl[8 + w];
  }
  if (tid < cap) {
    sstart[tid] = pre & 0xffff;
    sitem[tid] = pre >> 16;
    for (int q = 0; q < nq; ++q) items[(pre >> 16) + q] = tid | (q << 16);
  }
  const int nit = tot >> 16;
  __syncthreads();
  for (int i = tid; i < n; i += kThreads) {
    const int slot = oslot[i];
    if (slot >= 0) ssamp[sstart[slot] + orank[i]] = i;
  }
  __syncthreads();
  // item partial rows: LP lanes per item, its occurrences' loads all in flight
  const int ng = kThreads / LP, g = tid / LP, l = tid % LP;
  const float* dcol = dout + (int64_t)f * dout_fstride;
  for (int it = g; it < nit; it += ng) {
    const int slot = items[it] & 0xffff, q = items[it] >> 16;
    const int kb = sstart[slot] + q * kRun;
    const int ke = min(kb + kRun, sstart[slot] + cnt[slot]);
    for (int e = l; e < dim; e += LP) {
      float v[kRun];
#pragma unroll
      for (int u = 0; u < kRun; ++u)
        v[u] = kb + u < ke ? dcol[(b0 + ssamp[kb + u]) * dout_ld + e] : 0.f;
      float acc = v[0];
#pragma unroll
      for (int u = 1; u < kRun; ++u) acc += v[u];
      part[it * dim + e] = acc * sc;
    }
  }
  __syncthreads();
  // election (list mode) or plain marks (scan mode), as push_elect_kernel
  {
    int32_t rw[kCap / kThreads], fl[kCap / kThreads];
#pragma unroll
    for (int u = 0; u < kCap / kThreads; ++u) {
      const int slot = tid + u * kThreads;
      rw[u] = slot < cap ? keys[slot] : -1;
      fl[u] = (rw[u] >= 0 && ws_cnt) ? flag[rw[u]] : -2;
    }
#pragma unroll
    for (int u = 0; u < kCap / kThreads; ++u) {
      if (rw[u] < 0) continue;
      if (!ws_cnt) {
        scan_mark(flag, rw[u]);
      } else if (fl[u] != -2) {
        flag[rw[u]] = blk;
        ws_rows[(int64_t)blk * kCap + atomicAdd(&ctl[0], 1)] = rw[u];
      }
    }
  }
  // gradient rows: G2 lanes per row, one dword each, the row's item partials summed in order
  int G2 = 1;
  while (G2 < dim && G2 < 64) G2 <<= 1;
  const int per_pass = kThreads / G2, gs = tid / G2, l2 = tid % G2;
  for (int slot = gs; slot < cap; slot += per_pass) {
    const int32_t row = keys[slot];
    if (row < 0) continue;
    const int i0 = sitem[slot], ni = (cnt[slot] + kRun - 1) / kRun;
    float* dst = grad_table + (int64_t)row * dim;
    for (int e = l2; e < dim; e += G2) {
      float v = part[i0 * dim + e];
      for (int q = 1; q < ni; ++q) v += part[(i0 + q) * dim + e];
      RS_FLUSH_ADD(dst + e, v);
    }
  }
  if (ws_cnt) {
    __syncthreads();
    if (tid == 0) ws_cnt[blk] = ctl[0];
  }
}

__global__ void __launch_bounds__(kThreads) push_claim_kernel(
    const int32_t* __restrict__ ws_cnt, const int32_t* __restrict__ ws_rows,
    int32_t* __restrict__ flag, int32_t* __restrict__ touched, int32_t* __restrict__ n_touched,
    int32_t touched_cap) {
  __shared__ int32_t lidx[kCap];
  __shared__ int32_t ctl[2];
  const int blk = blockIdx.x, tid = threadIdx.x;
  const int cnt = ws_cnt[blk];
  if (cnt == 0) return;
  if (tid == 0) ctl[0] = 0;
  __syncthreads();
  const int32_t* cand = ws_rows + (int64_t)blk * kCap;
  int32_t rw[kCap / kThreads], fl[kCap / kThreads];
#pragma unroll
  for (int u = 0; u < kCap / kThreads; ++u) {
    const int e = tid + u * kThreads;
    rw[u] = e < cnt ? cand[e] : -1;
  }
#pragma unroll
  for (int u = 0; u < kCap / kThreads; ++u) fl[u] = rw[u] >= 0 ? flag[rw[u]] : -1;
#pragma unroll
  for (int u = 0; u < kCap / kThreads; ++u) {
    const int e = tid + u * kThreads;
    if (e >= cnt) continue;
    int li = -1;
    if (fl[u] == blk) {  // elected: this block claims the row
      flag[rw[u]] = -2;
      li = atomicAdd(&ctl[0], 1);
    }
    lidx[e] = li;
  }
  __syncthreads();
  if (tid == 0) ctl[1] = ctl[0] > 0 ? atomicAdd(n_touched, ctl[0]) : 0;
  __syncthreads();
  const int base = ctl[1];
  for (int e = tid; e < cnt; e += kThreads) {
    const int li = lidx[e];
    if (li >= 0 && base + li < touched_cap) touched[base + li] = cand[e];
  }
}

// samples per block: kTile, smaller for small launches so they still spread over >= ~256 blocks
#ifndef RS_PUSH_MIN_BLOCKS  // tuning builds only
#define RS_PUSH_MIN_BLOCKS 256
#endif
inline int tile_for(int64_t B, int F) {
  int t = kTile;
  while (t > 32 && ((B + t - 1) / t) * (int64_t)F < RS_PUSH_MIN_BLOCKS) t >>= 1;
  return t;
}
inline int64_t grid_blocks(int64_t B, int F) {
  const int t = tile_for(B, F);
  return ((B + t - 1) / t) * (int64_t)F;
}

// this device's per-block LDS (queried once)
inline int64_t lds_per_block() {
  static const int64_t v = [] {
    int dev = 0, x = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&x, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
      return (int64_t)64 * 1024;
    return (int64_t)x;
  }();
  return v;
}

}  // namespace rs_push

// ---------------------------------------------------------------------------------------------
// Multi-hot push (rs_sparse_grad_accumulate_mh, offsets != NULL; config 3's 200 fields x U{1..3}
// ids over disjoint per-field row ranges).  tools/push_prof.sh knockouts on config 3's shape
// (profiles/r06/push/): the CAS push takes 132 us, 111 with its claim CASes knocked out; a
// one-thread-per-sample form with the same LDS float-atomic aggregation took 139 us, 73 with those
// adds as plain LDS stores.  So a block here aggregates without float atomics, by a counting sort
// of its occurrences by row:
//   1. one thread per sample of the tile loads its [beg, end); a block scan of the lengths gives
//      every occurrence a position (a generation holds up to kMhOcc of them);
//   2. each thread loads its ids (all in flight) into the generation's LDS occurrence list;
//   3. one lane per occurrence probes the LDS hash (kMhCap > kMhOcc slots: never full) and takes
//      its rank within the row (one LDS int atomic per occurrence);
//   4. a block scan over the slots gives each row its run in a sorted occurrence array and
//      ceil(count / kMhRun) work items; the occurrences are scattered into their runs;
//   5. LP lanes (one float each) per item sum up to kMhRun occurrences' scale x dout, all loads in
//      flight, and add the sum to the row with one global float-atomic row segment (a Zipf-hot
//      row takes count / kMhRun such adds per block, the rest one);
//   6. claims, per distinct row: a returning CAS (-1 -> -2), as the CAS push (config 3's fields
//      are disjoint row ranges: few blocks share a row); one n_touched atomic per block and
//      generation.  Scan mode (touched == NULL): plain marks.
// Row set exact; the fp32 summation order is not fixed (run order = rank order).
// ---------------------------------------------------------------------------------------------
namespace rs_push {
// tuning builds: samples per block (a power of two, 64 .. 1024).  Larger tiles aggregate more of
// a row's occurrences before its global flush (config 3: ~3.2 K -> 2.4 K distinct rows per field
// at 256 -> 1024 samples) but lengthen each block's serial chain: push 121.7 us at 256, 131.3 at
// 512, 138.6 at 1024, 142.1 at 128 (list mode; profiles/r06/push/mh_tile_size.txt)
#ifndef RS_MH_THREADS
#define RS_MH_THREADS 256
#endif
constexpr int kMhThreads = RS_MH_THREADS;  // one thread per sample of the tile
constexpr int kMhTile = kMhThreads;
constexpr int kMhOcc = 3 * kMhThreads;     // occurrences per generation (U{1..3} x the tile)
constexpr int kMhCap = 4 * kMhThreads;     // LDS hash slots (> kMhOcc >= distinct rows per generation)
constexpr int kMhRun = 8;        // occurrences summed per work item
constexpr int kMhItems = kMhOcc + kMhOcc / kMhRun;  // >= sum over rows of ceil(count / kMhRun)
#ifndef RS_MH_KO  // timing experiments only: 1 no row adds, 2 no claims / marks
#define RS_MH_KO 0
#endif

constexpr size_t mh_lds_bytes() {
  return ((size_t)16 + 3 * (size_t)kMhCap + 4 * (size_t)kMhOcc + kMhItems + kMhTile) * 4;
}

template <int LP>
__global__ void __launch_bounds__(kMhThreads) push_mh_kernel(
    const int32_t* __restrict__ rows, const int32_t* __restrict__ offsets, int64_t B, int F,
    const float* __restrict__ dout, int64_t dout_ld, int64_t dout_fstride, int dim, int combiner,
    int tile, float* __restrict__ grad_table, int32_t* __restrict__ flag,
    int32_t* __restrict__ touched, int32_t* __restrict__ n_touched, int32_t touched_cap) {
  __shared__ int32_t ctl[4 + kMhThreads / 64 > 16 ? 4 + kMhThreads / 64 : 16];  // [0] claims, [1] claim base, [2] items, [4..] waves
  extern __shared__ __attribute__((aligned(16))) int32_t sm[];
  int32_t* keys = sm;                         // [kMhCap] row of each slot
  int32_t* cnt = keys + kMhCap;               // [kMhCap] occurrences per slot
  int32_t* sstart = cnt + kMhCap;             // [kMhCap] run start per slot
  int32_t* orow = sstart + kMhCap;            // [kMhOcc] ids, then ranks within their row
  int32_t* osamp = orow + kMhOcc;             // [kMhOcc] sample of each occurrence
  int32_t* oslot = osamp + kMhOcc;            // [kMhOcc] slot of each occurrence
  int32_t* ssamp = oslot + kMhOcc;            // [kMhOcc] samples sorted by row
  int32_t* items = ssamp + kMhOcc;            // [kMhItems] slot | chunk << 16
  float* sscale = reinterpret_cast<float*>(items + kMhItems);  // [kMhTile] combiner scale
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  constexpr int NW = kMhThreads / 64;
  const int f = blockIdx.y;
  const int64_t b0 = (int64_t)blockIdx.x * tile;
  const int n = (int)((b0 + tile < B ? b0 + tile : B) - b0);
  // block exclusive scan of one int per thread (ctl[4 .. 4 + NW) hold the wave sums)
  auto block_scan = [&](int x, int& total) {
    int inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int t = __shfl_up(inc, d, 64);
      if (lane >= d) inc += t;
    }
    __syncthreads();  // ctl's wave sums free again
    if (lane == 63) ctl[4 + wv] = inc;
    __syncthreads();
    int pre = inc - x;
    total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      if (w < wv) pre += ctl[4 + w];
      total += ctl[4 + w];
    }
    return pre;
  };
  // 1. this thread's sample: its id range, scale and occurrence positions
  int64_t beg = 0;
  int len = 0;
  if (tid < n) {
    const int64_t sg = (b0 + tid) * F + f;
    beg = offsets[sg];
    const int64_t end = offsets[sg + 1];
    len = end > beg ? (int)(end - beg) : 0;
    sscale[tid] = combiner_scale(len, combiner);
  }
  for (int k = tid; k < kMhCap; k += kMhThreads) {
    keys[k] = -1;
    cnt[k] = 0;
  }
  if (tid == 0) ctl[0] = 0;
  int total;
  const int pos = block_scan(len, total);
  const int ng = kMhThreads / LP, g = tid / LP, l = tid % LP;
  constexpr int SPT = kMhCap / kMhThreads;
  for (int g0 = 0; g0 < total; g0 += kMhOcc) {
    const int gn = total - g0 < kMhOcc ? total - g0 : kMhOcc;
    // 2. this generation's ids -> LDS (a thread's loads all issued before its stores)
    {
      const int k0 = g0 > pos ? g0 - pos : 0;
      const int k1 = g0 + gn - pos < len ? g0 + gn - pos : len;
      for (int k = k0; k < k1; k += 4) {
        int32_t r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = k + u < k1 ? rows[beg + k + u] : -1;
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k + u < k1) {
            orow[pos + k + u - g0] = r[u];
            osamp[pos + k + u - g0] = tid;
          }
      }
    }
    __syncthreads();
    // 3. probe + rank (padded sequence positions, row < 0, take no slot)
    for (int j = tid; j < gn; j += kMhThreads) {
      const int32_t row = orow[j];
      int slot = -1;
      if (row >= 0) {
        int h = (int)(((uint32_t)row * 2654435761u) & (uint32_t)(kMhCap - 1));
        for (;;) {  // kMhCap > kMhOcc >= distinct rows: terminates
          const int32_t old = atomicCAS(&keys[h], -1, row);
          if (old == -1 || old == row) { slot = h; break; }
          h = (h + 1) & (kMhCap - 1);
        }
        orow[j] = atomicAdd(&cnt[slot], 1);
      }
      oslot[j] = slot;
    }
    __syncthreads();
    // 4. runs and work items: a thread owns SPT consecutive slots; counts and item counts are
    //    scanned together (both < 2^16: count in the low half, items in the high half)
    int c[SPT], packed = 0;
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      c[u] = cnt[tid * SPT + u];
      packed += c[u] + (((c[u] + kMhRun - 1) / kMhRun) << 16);
    }
    int ptot;
    int pre = block_scan(packed, ptot);
#pragma unroll
    for (int u = 0; u < SPT; ++u) {
      const int slot = tid * SPT + u;
      const int run0 = pre & 0xffff, it0 = pre >> 16, nch = (c[u] + kMhRun - 1) / kMhRun;
      sstart[slot] = run0;
      for (int q = 0; q < nch; ++q) items[it0 + q] = slot | (q << 16);
      pre += c[u] + (nch << 16);
    }
    __syncthreads();
    const int nit = ptot >> 16;
    for (int j = tid; j < gn; j += kMhThreads) {
      const int slot = oslot[j];
      if (slot >= 0) ssamp[sstart[slot] + orow[j]] = osamp[j];
    }
    __syncthreads();
    // 5. row sums: LP lanes per item, its occurrences' loads all in flight
    for (int it = g; it < ((RS_MH_KO & 1) ? 0 : nit); it += ng) {
      const int slot = items[it] & 0xffff, q = items[it] >> 16;
      const int kb = sstart[slot] + q * kMhRun;
      const int ke = min(kb + kMhRun, sstart[slot] + cnt[slot]);
      float* dst = grad_table + (int64_t)keys[slot] * dim;
      for (int e = l; e < dim; e += LP) {
        float v[kMhRun];
#pragma unroll
        for (int u = 0; u < kMhRun; ++u) {
          v[u] = 0.f;
          if (kb + u < ke) {
            const int i = ssamp[kb + u];
            v[u] = dout[(b0 + i) * dout_ld + (int64_t)f * dout_fstride + e] * sscale[i];
          }
        }
        float acc = v[0];
#pragma unroll
        for (int u = 1; u < kMhRun; ++u) acc += v[u];
        RS_FLUSH_ADD(dst + e, acc);
      }
    }
    // 6. claims (list mode: a returning CAS -1 -> -2 per distinct row, SPT in flight per thread)
    //    or marks (scan mode)
    if (!(RS_MH_KO & 2)) {
      int32_t rw[SPT], old[SPT], li[SPT];
#pragma unroll
      for (int u = 0; u < SPT; ++u) rw[u] = keys[tid * SPT + u];
      if (touched) {
#pragma unroll
        for (int u = 0; u < SPT; ++u) old[u] = rw[u] >= 0 ? atomicCAS(&flag[rw[u]], -1, -2) : 0;
#pragma unroll
        for (int u = 0; u < SPT; ++u)
          li[u] = (rw[u] >= 0 && old[u] == -1) ? atomicAdd(&ctl[0], 1) : -1;
        __syncthreads();
        if (tid == 0) ctl[1] = ctl[0] > 0 ? atomicAdd(n_touched, ctl[0]) : 0;
        __syncthreads();
        const int base = ctl[1];
#pragma unroll
        for (int u = 0; u < SPT; ++u)
          if (li[u] >= 0 && base + li[u] < touched_cap) touched[base + li[u]] = rw[u];
      } else {
#pragma unroll
        for (int u = 0; u < SPT; ++u)
          if (rw[u] >= 0) scan_mark(flag, rw[u]);
      }
    }
    if (g0 + kMhOcc < total) {  // next generation: empty table
      __syncthreads();
      if (tid == 0) ctl[0] = 0;
      for (int k = tid; k < kMhCap; k += kMhThreads) {
        keys[k] = -1;
        cnt[k] = 0;
      }
      __syncthreads();
    }
  }
}

// the multi-hot push of rs_sparse_grad_accumulate_ws; nonzero: not launched (the caller takes the
// CAS push)
inline int push_mh(hipStream_t s, const int32_t* rows, const int32_t* offsets, int64_t B, int F,
                   const float* dout, int64_t dout_ld, int64_t dout_fstride, int dim, int combiner,
                   float* grad_table, int32_t* flag, int32_t* touched, int32_t* n_touched,
                   int32_t touched_cap) {
  int tile = kMhTile;  // small launches still spread over >= ~256 blocks
  while (tile > 32 && ((B + tile - 1) / tile) * (int64_t)F < RS_PUSH_MIN_BLOCKS) tile >>= 1;
  const int64_t nbx = (B + tile - 1) / tile;
  if ((int64_t)mh_lds_bytes() > lds_per_block() || F > 65535 || nbx > INT32_MAX) return 1;
  int LP = 1;
  while (LP < dim && LP < 64) LP <<= 1;
  dim3 grid((unsigned)nbx, (unsigned)F);
  const size_t lds = mh_lds_bytes();
#define RS_PUSH_MH(LL)                                                                            \
  case LL:                                                                                        \
    push_mh_kernel<LL><<<grid, kMhThreads, lds, s>>>(rows, offsets, B, F, dout, dout_ld,         \
                                                     dout_fstride, dim, combiner, tile,           \
                                                     grad_table, flag, touched, n_touched,        \
                                                     touched_cap);                                \
    return 0;
  switch (LP) {
    RS_PUSH_MH(1) RS_PUSH_MH(2) RS_PUSH_MH(4) RS_PUSH_MH(8) RS_PUSH_MH(16) RS_PUSH_MH(32)
    RS_PUSH_MH(64)
    default: return 1;
  }
#undef RS_PUSH_MH
}

}  // namespace rs_push


RS_API int64_t rs_sparse_push_workspace_bytes(int64_t B, int F) {
  if (B < 0 || F <= 0) return -1;
  return rs_push::grid_blocks(B, F) * (1 + rs_push::kCap) * 4;
}

RS_API int rs_sparse_grad_accumulate_ws(void* stream, const int32_t* rows, const int32_t* offsets,
                                        int64_t B, int F, const float* dout, int64_t dout_ld,
                                        int64_t dout_fstride, int dim, int combiner,
                                        float* grad_table, int32_t* flag, int32_t* touched,
                                        int32_t* n_touched, int32_t touched_cap, void* workspace,
                                        int64_t workspace_bytes) {
  using namespace rs_push;
  static const bool elect_off = getenv("RS_PUSH_NO_ELECT") != nullptr;  // A/B: the CAS push
  // the election push's LDS hash must fit this device's per-block LDS: larger shapes, or a part
  // with less LDS, take the CAS push
  const int64_t lds_max = lds_per_block();
  // rows of >= 32 floats aggregate by counting sort (push_sort_kernel: config-5 91-field push
  // 69.4 -> 39.3 us), narrower ones with LDS float atomics (push_elect_kernel: config-4 pushes at
  // dim 16 6.4 / 18.6 / 16.7 us vs 7.5 / 18.6 / 17.3 sorted); RS_PUSH_LDS_ADD=0 / 1 forces either
  static const int lds_add_env = [] {
    const char* e = getenv("RS_PUSH_LDS_ADD");
    return e ? atoi(e) : -1;
  }();
  const bool lds_add = lds_add_env >= 0 ? lds_add_env != 0 : dim < 32;
  const size_t lds = lds_add ? lds_bytes(dim) : sort_lds_bytes(dim);
  // multi-hot: the counting-sort push with CAS claims (RS_PUSH_MH_CAS=1: the LDS-atomic CAS push)
  static const bool mh_off = getenv("RS_PUSH_MH_CAS") != nullptr;
  if (offsets && !mh_off && rows && dout && grad_table && flag && F > 0 && dim > 0 &&
      (!touched || n_touched) && B * (int64_t)F > 0 &&
      rs_push::push_mh(rs_stream(stream), rows, offsets, B, F, dout, dout_ld, dout_fstride, dim,
                       combiner, grad_table, flag, touched, n_touched, touched_cap) == 0)
    return rs_status_after_launch();
  const bool ok_shape = !elect_off && !offsets && dim % 4 == 0 && dout_ld % 4 == 0 && dout_fstride % 4 == 0 &&
                        ((uintptr_t)dout & 15) == 0 && (int64_t)lds <= lds_max &&
                        B <= INT32_MAX / 2 && grid_blocks(B, F) <= INT32_MAX;
  if (!ok_shape || (touched && (!workspace || workspace_bytes < rs_sparse_push_workspace_bytes(B, F))))
    return rs_sparse_grad_accumulate(stream, rows, offsets, B, F, dout, dout_ld, dout_fstride, dim,
                                     combiner, grad_table, flag, touched, n_touched, touched_cap);
  if (!rows || !dout || !grad_table || !flag || F <= 0 || dim <= 0) return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  if (B * (int64_t)F == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  const int64_t nblk = grid_blocks(B, F);
  int32_t* ws_cnt = touched ? static_cast<int32_t*>(workspace) : nullptr;
  int32_t* ws_rows = touched ? ws_cnt + nblk : nullptr;
  const float sc = 1.0f;  // one id per segment: every combiner scales by 1
  (void)combiner;
  int LP = 1;
  while (LP < dim / 4 && LP < 64) LP <<= 1;
  const int tile = tile_for(B, F);
  dim3 grid((unsigned)((B + tile - 1) / tile), (unsigned)F);
#define RS_PUSH_E(LL)                                                                             \
  case LL:                                                                                        \
    push_elect_kernel<LL><<<grid, kThreads, lds, s>>>(rows, B, F, dout, dout_ld, dout_fstride,   \
                                                      dim, sc, tile, grad_table, flag, ws_cnt,   \
                                                      ws_rows);                                  \
    break;
  PushSrcs one{};
  one.n = 1;
  one.s[0] = PushSrc{rows, dout, dout_ld, dout_fstride, B, F, 0};
#define RS_PUSH_S(LL)                                                                             \
  case LL:                                                                                        \
    push_sort_kernel<LL><<<grid, kThreads, lds, s>>>(one, dim, sc, tile, grad_table, flag,       \
                                                     ws_cnt, ws_rows);                           \
    break;
  if (lds_add) {
    switch (LP) {
      RS_PUSH_E(1) RS_PUSH_E(2) RS_PUSH_E(4) RS_PUSH_E(8) RS_PUSH_E(16) RS_PUSH_E(32) RS_PUSH_E(64)
      default: return RS_ERR_UNSUPPORTED;
    }
  } else {
    int LS = 1;  // lanes per work item: one float each
    while (LS < dim && LS < 64) LS <<= 1;
    switch (LS) {
      RS_PUSH_S(1) RS_PUSH_S(2) RS_PUSH_S(4) RS_PUSH_S(8) RS_PUSH_S(16) RS_PUSH_S(32) RS_PUSH_S(64)
      default: return RS_ERR_UNSUPPORTED;
    }
  }
#undef RS_PUSH_E
#undef RS_PUSH_S
  if (touched)
    push_claim_kernel<<<(unsigned)nblk, kThreads, 0, s>>>(ws_cnt, ws_rows, flag, touched, n_touched,
                                                          touched_cap);
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Grouped single-hot pushes into ONE table (rs_push::PushSrcs): the counting-sort push over every
// source's (tile, field) blocks in one launch, then one claim launch.  Same per-block work, row
// set and claims as one rs_sparse_grad_accumulate_ws call per source (a row pushed by several
// sources is claimed once: the election picks one block among all of them).  Rows of >= 32
// floats only (the sort push); RS_ERR_UNSUPPORTED otherwise (the caller pushes one by one).
// ---------------------------------------------------------------------------------------------
static int push_group_shape(int nsrc, const int64_t* B, const int* F, int64_t* bmax, int* ftot) {
  if (nsrc <= 0 || nsrc > rs_push::kMaxSrc || !B || !F) return RS_ERR_ARG;
  int64_t bm = 0, ft = 0;
  for (int k = 0; k < nsrc; ++k) {
    if (B[k] < 0 || F[k] <= 0) return RS_ERR_ARG;
    if (B[k] > INT32_MAX / 2) return RS_ERR_UNSUPPORTED;
    bm = B[k] > bm ? B[k] : bm;
    ft += F[k];
  }
  if (ft > 65535) return RS_ERR_UNSUPPORTED;
  *bmax = bm;
  *ftot = (int)ft;
  return RS_OK;
}

RS_API int64_t rs_sparse_push_group_workspace_bytes(int nsrc, const int64_t* B, const int* F) {
  int64_t bmax = 0;
  int ftot = 0;
  if (push_group_shape(nsrc, B, F, &bmax, &ftot) != RS_OK) return -1;
  return rs_push::grid_blocks(bmax, ftot) * (1 + rs_push::kCap) * 4;
}

RS_API int rs_sparse_grad_accumulate_group(void* stream, int nsrc, const int32_t* const* rows,
                                           const float* const* dout, const int64_t* B, const int* F,
                                           const int64_t* dout_ld, const int64_t* dout_fstride,
                                           int dim, float* grad_table, int32_t* flag,
                                           int32_t* touched, int32_t* n_touched,
                                           int32_t touched_cap, void* workspace,
                                           int64_t workspace_bytes) {
  using namespace rs_push;
  if (!rows || !dout || !dout_ld || !dout_fstride || !grad_table || !flag || dim <= 0)
    return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  int64_t bmax = 0;
  int ftot = 0;
  const int st = push_group_shape(nsrc, B, F, &bmax, &ftot);
  if (st != RS_OK) return st;
  const size_t lds = sort_lds_bytes(dim);
  if (dim < 32 || dim % 4 != 0 || (int64_t)lds > lds_per_block()) return RS_ERR_UNSUPPORTED;
  PushSrcs g{};
  g.n = nsrc;
  int f0 = 0;
  for (int k = 0; k < nsrc; ++k) {
    if (!rows[k] || !dout[k]) return RS_ERR_ARG;
    if (dout_ld[k] % 4 != 0 || dout_fstride[k] % 4 != 0 || ((uintptr_t)dout[k] & 15) != 0)
      return RS_ERR_UNSUPPORTED;
    g.s[k] = PushSrc{rows[k], dout[k], dout_ld[k], dout_fstride[k], B[k], F[k], f0};
    f0 += F[k];
  }
  if (bmax == 0) return RS_OK;
  const int64_t nblk = grid_blocks(bmax, ftot);
  if (nblk > INT32_MAX) return RS_ERR_UNSUPPORTED;
  if (touched && (!workspace || workspace_bytes < nblk * (1 + kCap) * 4)) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  int32_t* ws_cnt = touched ? static_cast<int32_t*>(workspace) : nullptr;
  int32_t* ws_rows = touched ? ws_cnt + nblk : nullptr;
  const int tile = tile_for(bmax, ftot);
  dim3 grid((unsigned)((bmax + tile - 1) / tile), (unsigned)ftot);
  int LS = 1;
  while (LS < dim && LS < 64) LS <<= 1;
  if (LS == 32)
    push_sort_kernel<32><<<grid, kThreads, lds, s>>>(g, dim, 1.0f, tile, grad_table, flag, ws_cnt, ws_rows);
  else if (LS == 64)
    push_sort_kernel<64><<<grid, kThreads, lds, s>>>(g, dim, 1.0f, tile, grad_table, flag, ws_cnt, ws_rows);
  else
    return RS_ERR_UNSUPPORTED;
  if (touched)
    push_claim_kernel<<<(unsigned)nblk, kThreads, 0, s>>>(ws_cnt, ws_rows, flag, touched, n_touched,
                                                          touched_cap);
  return rs_status_after_launch();
}

RS_API int rs_sparse_grad_accumulate(void* stream, const int32_t* rows, const int32_t* offsets,
                                     int64_t B, int F, const float* dout, int64_t dout_ld,
                                     int64_t dout_fstride, int dim, int combiner,
                                     float* grad_table, int32_t* flag, int32_t* touched,
                                     int32_t* n_touched, int32_t touched_cap) {
  if (!rows || !dout || !grad_table || !flag || F <= 0 || dim <= 0) return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  if (B * (int64_t)F == 0) return RS_OK;
  int G = 1;
  while (G < dim && G < 64) G <<= 1;
  // LDS table: cap slots of dim floats, tile = cap/2 samples (load factor <= 1/2 for single-hot
  // fields)
  // Many single-hot "fields" over one shared row space (a sequence's T positions, config 5's 91
  // fields hashed into one table) repeat the same hot rows in every field's blocks, and the
  // flush's same-row global atomics serialise: there a block takes a 4x larger tile (up to
  // 2048 slots, ~147 KB of the CU's 160 KB LDS at dim 16) so each hot row is flushed 4x less
  // often (config-4 history push 55 -> 36 us).  Few fields (config 2's 26 disjoint ranges) keep
  // the 64 KB table: more blocks in flight beat fewer flushes there.
  int cap = 1024;
#ifndef RS_PUSH_MH_BUDGET  // tuning builds only: the multi-hot table's LDS budget (KB)
#define RS_PUSH_MH_BUDGET 64
#endif
  const size_t lds_budget = (!offsets && F >= 32) ? 150 * 1024 : (size_t)RS_PUSH_MH_BUDGET * 1024;
  if (lds_budget > 64 * 1024) cap = 4096;
  while (cap > 32 && (size_t)cap * (dim + 2) * 4 > lds_budget) cap >>= 1;
  const int tile = cap / 2;
  dim3 grid((unsigned)((B + tile - 1) / tile), (unsigned)F);
  const size_t lds = ((size_t)cap * (dim + 2) + 4) * 4;
  // 1024 threads: a tile's samples are covered in ~4 passes per lane group with all their loads
  // issued up front (PMC: at 256 threads the waves spent 73 % of their cycles waiting on memory)
  sparse_grad_accum_kernel<<<grid, 1024, lds, rs_stream(stream)>>>(
      rows, offsets, B, F, dout, dout_ld, dout_fstride, dim, combiner, G, tile, cap, grad_table,
      flag, touched, n_touched, touched_cap);
  return rs_status_after_launch();
}
