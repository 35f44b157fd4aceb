// H11 — optimizers on the path.
//
// Dense: tn.optimizer.Optimizer(tn.core.Adam(lr, beta1, beta2, epsilon)) at
//   rank/ctr/base_model.py:192-193, rank/multi_head/model.py:52-53, staytime/model.py:72,
//   rough_rank/model.py:209, rank/finish/model.py:41.
// Sparse: tn.core.Adam handed to EmbeddingFeatures (rank/ctr/base_model.py:163,
//   rank/multi_head/multidnn.py:235, rough_rank/model.py:106) and tn.core.AdaGrad
//   (staytime/VideoDnn.py:233,259).
// tensornet is not vendored, so the update forms are pinned here and restated in
// oracle/ctr_oracle.py:
//   dense Adam  : t += 1; lr_t = lr*sqrt(1-b2^t)/(1-b1^t); m = b1 m + (1-b1) g;
//                 v = b2 v + (1-b2) g^2; w -= lr_t * m / (sqrt(v) + eps)      (tf.keras form)
//   sparse Adam : per touched row, no bias correction (tensornet SparseAdamValue form):
//                 m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2; w -= lr * m / (eps + sqrt(v))
//   sparse AdaGrad: g2 += g^2 (per element, initialised to initial_g2sum);
//                 w -= lr * g / sqrt(g2)
// The dense parameters of a model live in ONE flat fp32 arena (params | grads | m | v), so the
// dense step is one launch and the data-parallel all-reduce is one bucket.
#include "common.hpp"

__global__ void __launch_bounds__(256) dense_adam_kernel(float* __restrict__ p,
                                                        float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        int64_t n, int64_t* __restrict__ step,
                                                        float lr, float b1, float b2, float eps,
                                                        float grad_scale, int zero_grad,
                                                        int32_t* __restrict__ done) {
  const int64_t t = step[0] + 1;
  const float bc1 = 1.0f - powf(b1, (float)t);
  const float bc2 = 1.0f - powf(b2, (float)t);
  const float lr_t = lr * sqrtf(bc2) / bc1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * grad_scale;
    if (zero_grad) g[i] = 0.f;  // fused zero_grad: the next backward accumulates into g
    const float mi = b1 * m[i] + (1.0f - b1) * gi;
    const float vi = b2 * v[i] + (1.0f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= lr_t * mi / (sqrtf(vi) + eps);
  }
  // fused step counter: every block has read step[0] above; the last block to finish advances it
  // (no separate increment launch)
  if (done && rs_last_block(done)) step[0] = t;
}

__global__ void step_increment_kernel(int64_t* step) { step[0] += 1; }

RS_API int rs_dense_adam(void* stream, float* params, float* grads, float* m, float* v,
                         int64_t n, int64_t* step, float lr, float beta1, float beta2, float eps,
                         float grad_scale, int zero_grad) {
  if (!params || !grads || !m || !v || !step || n < 0) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  if (n > 0) {
    int64_t grid = (n + 255) / 256;
    if (grid > 2048) grid = 2048;
    dense_adam_kernel<<<(int)grid, 256, 0, s>>>(params, grads, m, v, n, step, lr, beta1, beta2,
                                                eps, grad_scale, zero_grad, nullptr);
  }
  step_increment_kernel<<<1, 1, 0, s>>>(step);
  return rs_status_after_launch();
}

RS_API int rs_dense_adam_done(void* stream, float* params, float* grads, float* m, float* v,
                              int64_t n, int64_t* step, float lr, float beta1, float beta2,
                              float eps, float grad_scale, int zero_grad, int32_t* done) {
  if (!params || !grads || !m || !v || !step || !done || n < 0) return RS_ERR_ARG;
  int64_t grid = (n + 255) / 256;
  if (grid > 2048) grid = 2048;
  if (grid < 1) grid = 1;  // n == 0: one block still advances the step
  dense_adam_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(params, grads, m, v, n, step, lr,
                                                              beta1, beta2, eps, grad_scale,
                                                              zero_grad, done);
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Sparse Adam over the rows touched this step.  One group of `lps` lanes per row; the group also
// zeroes the row's gradient slot and releases its claim flag so the next step starts clean.
// The row count lives on the device (written by rs_sparse_grad_accumulate), so the grid is sized
// by the capacity and idle groups exit: no host sync, graph-capturable.
// ---------------------------------------------------------------------------------------------
// n_touched = int32[1 + RS_DONE_WORDS]: {count, completion counters}.  Every block of a sparse
// optimizer launch reads count first; the last block to finish resets it (rs_last_block), so the
// next step's accumulate starts from zero without a separate memset launch.
// A push that claimed more rows than the touched list holds (count > cap) is an overflow: the
// optimizer updates only the first cap rows, and the last block records the count in the sticky
// word n_touched[RS_TOUCHED_OVERFLOW] (SparseTable.check_overflow raises on it).
#define RS_TOUCHED_OVERFLOW RS_DONE_WORDS
__device__ __forceinline__ void release_touched_count(int32_t* n_touched, int32_t count,
                                                      int32_t cap) {
  if (rs_last_block(n_touched + 1)) {
    if (count > cap) atomicMax(n_touched + RS_TOUCHED_OVERFLOW, count);
    atomicExch(n_touched, 0);
  }
}

__global__ void __launch_bounds__(256) sparse_adam_kernel(
    float* __restrict__ table, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ grad_table, int32_t* __restrict__ flag,
    const int32_t* __restrict__ touched, int32_t* __restrict__ n_touched, int dim,
    int32_t cap, int lps, float lr, float b1, float b2, float eps, float grad_scale) {
  const int count = *n_touched;
  const int nrows = min(count, cap);
  const int per_block = blockDim.x / lps;
  const int gi = threadIdx.x / lps;
  const int l = threadIdx.x % lps;
  for (int u = blockIdx.x * per_block + gi; u < nrows; u += gridDim.x * per_block) {
    const int64_t row = touched[u];
    const int64_t base = row * dim;
    for (int e = l; e < dim; e += lps) {
      const float g = grad_table[base + e] * grad_scale;
      const float mi = b1 * m[base + e] + (1.0f - b1) * g;
      const float vi = b2 * v[base + e] + (1.0f - b2) * g * g;
      m[base + e] = mi;
      v[base + e] = vi;
      table[base + e] -= lr * mi / (eps + sqrtf(vi));
      grad_table[base + e] = 0.f;
    }
    if (l == 0) flag[row] = -1;
  }
  release_touched_count(n_touched, count, cap);
}

__global__ void __launch_bounds__(256) sparse_adagrad_kernel(
    float* __restrict__ table, float* __restrict__ g2sum, float* __restrict__ grad_table,
    int32_t* __restrict__ flag, const int32_t* __restrict__ touched,
    int32_t* __restrict__ n_touched, int dim, int32_t cap, int lps, float lr, float grad_scale) {
  const int count = *n_touched;
  const int nrows = min(count, cap);
  const int per_block = blockDim.x / lps;
  const int gi = threadIdx.x / lps;
  const int l = threadIdx.x % lps;
  for (int u = blockIdx.x * per_block + gi; u < nrows; u += gridDim.x * per_block) {
    const int64_t row = touched[u];
    const int64_t base = row * dim;
    for (int e = l; e < dim; e += lps) {
      const float g = grad_table[base + e] * grad_scale;
      const float s2 = g2sum[base + e] + g * g;
      g2sum[base + e] = s2;
      table[base + e] -= lr * g / sqrtf(s2);
      grad_table[base + e] = 0.f;
    }
    if (l == 0) flag[row] = -1;
  }
  release_touched_count(n_touched, count, cap);
}

static int lanes_for_dim(int dim) {
  int lps = 1;
  while (lps < dim && lps < 64) lps <<= 1;
  return lps;
}

RS_API int rs_sparse_adam(void* stream, float* table, float* m, float* v, float* grad_table,
                          int32_t* flag, const int32_t* touched, int32_t* n_touched, int dim,
                          int32_t max_rows, float lr, float beta1, float beta2, float eps,
                          float grad_scale) {
  if (!table || !m || !v || !grad_table || !flag || !touched || !n_touched || dim <= 0)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int lps = lanes_for_dim(dim);
  if (max_rows > 0) {
    int64_t grid = ((int64_t)max_rows * lps + 255) / 256;
    if (grid > 1024) grid = 1024;
    sparse_adam_kernel<<<(int)grid, 256, 0, s>>>(table, m, v, grad_table, flag, touched,
                                                 n_touched, dim, max_rows, lps, lr, beta1, beta2, eps,
                                                 grad_scale);
  }
  else
    rs_fill_u32(s, n_touched, 0u, 1);
  return rs_status_after_launch();
}

RS_API int rs_sparse_adagrad(void* stream, float* table, float* g2sum, float* grad_table,
                             int32_t* flag, const int32_t* touched, int32_t* n_touched, int dim,
                             int32_t max_rows, float lr, float grad_scale) {
  if (!table || !g2sum || !grad_table || !flag || !touched || !n_touched || dim <= 0)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int lps = lanes_for_dim(dim);
  if (max_rows > 0) {
    int64_t grid = ((int64_t)max_rows * lps + 255) / 256;
    if (grid > 1024) grid = 1024;
    sparse_adagrad_kernel<<<(int)grid, 256, 0, s>>>(table, g2sum, grad_table, flag, touched,
                                                    n_touched, dim, max_rows, lps, lr, grad_scale);
  }
  else
    rs_fill_u32(s, n_touched, 0u, 1);
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Scan-mode sparse optimizers: no touched list.  The push marked every touched row with
// flag = -2 (plain stores).  The table is swept in 64-row chunks; wave w takes chunks
// w, w + W, w + 2W, ... (W = waves in the grid, one chip-full round), so the dense chunks at the
// head of each field's Zipf range are spread over many waves while every flag load stays one
// coalesced 256-B read.  Per chunk: one flag load per lane (the next chunk's is issued before
// the current one is processed), a ballot, the marked rows compacted into a wave-local LDS list
// (mbcnt rank), then processed 64 / (dim / 4) rows per pass with dim / 4 lanes per row, each
// lane moving one float4 of grad / param / m / v (one memory round trip per pass).
// ---------------------------------------------------------------------------------------------
constexpr int kScanBlock = 256;

template <bool ADAM>
struct ScanRow {
  float4 g, w, mm, vv;
  __device__ __forceinline__ void load(const float* __restrict__ table, const float* __restrict__ m,
                                       const float* __restrict__ v,
                                       const float* __restrict__ grad_table, int64_t o) {
    g = *reinterpret_cast<const float4*>(grad_table + o);
    w = *reinterpret_cast<const float4*>(table + o);
    mm = *reinterpret_cast<const float4*>(m + o);
    vv = ADAM ? *reinterpret_cast<const float4*>(v + o) : mm;
  }
  __device__ __forceinline__ void update_store(float* __restrict__ table, float* __restrict__ m,
                                               float* __restrict__ v, float* __restrict__ grad_table,
                                               int64_t o, float lr, float b1, float b2, float eps,
                                               float grad_scale) {
    float* gp = &g.x; float* wp = &w.x; float* mp = &mm.x; float* vp = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gp[k] * grad_scale;
      if (ADAM) {
        mp[k] = b1 * mp[k] + (1.0f - b1) * gk;
        vp[k] = b2 * vp[k] + (1.0f - b2) * gk * gk;
        wp[k] -= lr * mp[k] / (eps + sqrtf(vp[k]));
      } else {  // AdaGrad: m holds g2sum
        mp[k] += gk * gk;
        wp[k] -= lr * gk / sqrtf(mp[k]);
      }
    }
    *reinterpret_cast<float4*>(table + o) = w;
    *reinterpret_cast<float4*>(m + o) = mm;
    if (ADAM) *reinterpret_cast<float4*>(v + o) = vv;
    *reinterpret_cast<float4*>(grad_table + o) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
};

// Flag sweep: every wave walks its 64-row chunks (flags prefetched one chunk ahead), appends the
// marked rows to a per-wave LDS list (clearing their flags) and updates the collected rows only
// when the list is full or its chunks are done -- at ~1 % touched rows a chunk holds about one
// marked row, so batching turns one dependent HBM round trip per chunk into one per list.  The
// list is processed two passes at a time (both passes' loads issued before either's stores).
// The sweep of one wave: gw = the wave's global index, nwaves = waves in the sweep, list = its
// LCAP-entry LDS list (the standalone kernel and the fused optimizer tail share it).
constexpr int kScanLcap = 256;  // rows per wave list
template <bool ADAM>
__device__ __forceinline__ void scan_opt_wave(float* __restrict__ table, float* __restrict__ m,
                                              float* __restrict__ v, float* __restrict__ grad_table,
                                              int32_t* __restrict__ flag, int64_t nrows, int dim,
                                              float lr, float b1, float b2, float eps,
                                              float grad_scale, int64_t gw, int64_t nwaves,
                                              uint32_t* list) {
  constexpr int LCAP = kScanLcap;
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (nrows + 63) / 64;
  const int nv = dim >> 2;             // float4 per row
  const int lpr = nv < 64 ? nv : 64;   // lanes per row
  const int rpp = 64 / lpr;            // rows per pass
  const int sub = lane % lpr, slot = lane / lpr;
  int n = 0;                           // wave-uniform list length
  auto flush = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int p0 = 0; p0 < n; p0 += 2 * rpp) {
      const int k0 = p0 + slot, k1 = p0 + rpp + slot;
      const bool on0 = slot < rpp && k0 < n, on1 = slot < rpp && k1 < n;
      const int64_t r0 = on0 ? (int64_t)list[k0] : 0, r1 = on1 ? (int64_t)list[k1] : 0;
      for (int e4 = sub; e4 < nv; e4 += lpr) {
        ScanRow<ADAM> x0, x1;
        const int64_t o0 = r0 * dim + 4 * e4, o1 = r1 * dim + 4 * e4;
        if (on0) x0.load(table, m, v, grad_table, o0);
        if (on1) x1.load(table, m, v, grad_table, o1);
        if (on0) x0.update_store(table, m, v, grad_table, o0, lr, b1, b2, eps, grad_scale);
        if (on1) x1.update_store(table, m, v, grad_table, o1, lr, b1, b2, eps, grad_scale);
      }
    }
    __builtin_amdgcn_wave_barrier();  // list reuse
    n = 0;
  };
  // the flag words of PF chunks per lane are loaded at once (a chip-full grid gives each wave
  // ~5 chunks of a 2.6 M-row table: one memory round trip for all of them instead of one per
  // chunk -- the sweep was a chain of dependent flag loads)
  constexpr int PF = 8;
  for (int64_t cb = gw; cb < nchunks; cb += PF * nwaves) {
    int32_t fl[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int64_t c = cb + u * nwaves;
      fl[u] = (c < nchunks && c * 64 + lane < nrows) ? flag[c * 64 + lane] : -1;
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int64_t c = cb + u * nwaves;
      if (c >= nchunks) break;  // wave-uniform
      const int64_t row0 = c * 64;
      const bool hit = fl[u] != -1;
      const uint64_t mask = __ballot(hit);
      if (mask) {
        const int cnt = __popcll(mask);
        if (n + cnt > LCAP) flush();
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        if (hit) {
          list[n + rank] = (uint32_t)(row0 + lane);
          flag[row0 + lane] = -1;
        }
        n += cnt;
      }
    }
  }
  if (n) flush();
}

template <bool ADAM>
__global__ void __launch_bounds__(kScanBlock) sparse_scan_opt_kernel(
    float* __restrict__ table, float* __restrict__ m, float* __restrict__ v,
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int64_t nrows, int dim,
    float lr, float b1, float b2, float eps, float grad_scale, const int32_t* __restrict__ gate) {
  if (gate && *gate == 0) return;  // overflow-recovery sweep with nothing to recover
  __shared__ uint32_t lists[(kScanBlock / 64) * kScanLcap];
  const int64_t nwaves = (int64_t)gridDim.x * (kScanBlock / 64);
  const int64_t gw = (int64_t)blockIdx.x * (kScanBlock / 64) + (threadIdx.x >> 6);
  scan_opt_wave<ADAM>(table, m, v, grad_table, flag, nrows, dim, lr, b1, b2, eps, grad_scale, gw,
                      nwaves, lists + (threadIdx.x >> 6) * kScanLcap);
}

static int64_t scan_grid(int64_t nrows) {
  // one chip-full round of waves (256 CUs x 32), fewer for small tables
  const int64_t chunks = (nrows + 63) / 64;
  int64_t grid = (chunks + kScanBlock / 64 - 1) / (kScanBlock / 64);
  return grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
}

template <bool ADAM>
static void launch_scan_opt(hipStream_t s, unsigned grid, float* table, float* m, float* v,
                            float* grad, int32_t* flag, int64_t nrows, int dim, float lr, float b1,
                            float b2, float eps, float gs, const int32_t* gate = nullptr) {
  sparse_scan_opt_kernel<ADAM><<<grid, kScanBlock, 0, s>>>(table, m, v, grad, flag, nrows, dim, lr,
                                                           b1, b2, eps, gs, gate);
}

RS_API int rs_sparse_adam_scan(void* stream, float* table, float* m, float* v, float* grad_table,
                               int32_t* flag, int64_t table_rows, int dim, float lr, float beta1,
                               float beta2, float eps, float grad_scale) {
  if (!table || !m || !v || !grad_table || !flag || dim <= 0 || dim % 4 || table_rows < 0 ||
      table_rows > (int64_t)UINT32_MAX)
    return RS_ERR_ARG;
  if (table_rows == 0) return RS_OK;
  launch_scan_opt<true>(rs_stream(stream), (unsigned)scan_grid(table_rows), table, m, v,
                        grad_table, flag, table_rows, dim, lr, beta1, beta2, eps, grad_scale);
  return rs_status_after_launch();
}

RS_API int rs_sparse_adagrad_scan(void* stream, float* table, float* g2sum, float* grad_table,
                                  int32_t* flag, int64_t table_rows, int dim, float lr,
                                  float grad_scale) {
  if (!table || !g2sum || !grad_table || !flag || dim <= 0 || dim % 4 || table_rows < 0 ||
      table_rows > (int64_t)UINT32_MAX)
    return RS_ERR_ARG;
  if (table_rows == 0) return RS_OK;
  launch_scan_opt<false>(rs_stream(stream), (unsigned)scan_grid(table_rows), table, g2sum,
                         nullptr, grad_table, flag, table_rows, dim, lr, 0.f, 0.f, 0.f,
                         grad_scale);
  return rs_status_after_launch();
}

// Overflow recovery of the list-mode optimizers (rs_sparse_adam / rs_sparse_adagrad).  A push that
// claimed more rows than the touched list holds leaves the unlisted rows claimed (flag -2) with
// their gradient in grad_table; the list-mode launch then records the overflow in the sticky word
// n_touched[RS_TOUCHED_OVERFLOW].  Launched right after the list-mode optimizer on the same
// stream, this sweep reads that word and exits at once when it is zero; otherwise it is the scan
// optimizer over the whole table, which updates exactly the rows still marked (listed rows were
// released to -1 by the list launch).  The word stays set until SparseTable.check_overflow
// clears it, so every later step is swept too: overflow costs speed, never updates.
RS_API int rs_sparse_adam_recover(void* stream, float* table, float* m, float* v, float* grad_table,
                                  int32_t* flag, const int32_t* n_touched, int64_t table_rows,
                                  int dim, float lr, float beta1, float beta2, float eps,
                                  float grad_scale) {
  if (!table || !m || !v || !grad_table || !flag || !n_touched || dim <= 0 || dim % 4 ||
      table_rows < 0 || table_rows > (int64_t)UINT32_MAX)
    return RS_ERR_ARG;
  if (table_rows == 0) return RS_OK;
  launch_scan_opt<true>(rs_stream(stream), (unsigned)scan_grid(table_rows), table, m, v,
                        grad_table, flag, table_rows, dim, lr, beta1, beta2, eps, grad_scale,
                        n_touched + RS_TOUCHED_OVERFLOW);
  return rs_status_after_launch();
}

RS_API int rs_sparse_adagrad_recover(void* stream, float* table, float* g2sum, float* grad_table,
                                     int32_t* flag, const int32_t* n_touched, int64_t table_rows,
                                     int dim, float lr, float grad_scale) {
  if (!table || !g2sum || !grad_table || !flag || !n_touched || dim <= 0 || dim % 4 ||
      table_rows < 0 || table_rows > (int64_t)UINT32_MAX)
    return RS_ERR_ARG;
  if (table_rows == 0) return RS_OK;
  launch_scan_opt<false>(rs_stream(stream), (unsigned)scan_grid(table_rows), table, g2sum,
                         nullptr, grad_table, flag, table_rows, dim, lr, 0.f, 0.f, 0.f,
                         grad_scale, n_touched + RS_TOUCHED_OVERFLOW);
  return rs_status_after_launch();
}

// Scan-mode compaction for the data-parallel exchange: every marked row is moved out of the
// gradient table into (rows_out, grads_out) (gradient row zeroed, flag cleared); the slots are
// allocated with one counter atomic per block (n_out[0]; rows past `cap` are dropped and
// counted).  The list order is allocation order; the rank-ordered merge does not depend on it.
__global__ void __launch_bounds__(256) sparse_compact_scan_kernel(
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int64_t nrows, int dim,
    int32_t* __restrict__ rows_out, float* __restrict__ grads_out, int32_t* __restrict__ n_out,
    int32_t cap) {
  __shared__ int32_t cnt, base;
  for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x; r0 < nrows;
       r0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = r0 + threadIdx.x;
    const bool hit = row < nrows && flag[row] != -1;
    if (threadIdx.x == 0) cnt = 0;
    __syncthreads();
    const int li = hit ? atomicAdd(&cnt, 1) : -1;
    __syncthreads();
    if (threadIdx.x == 0) base = cnt > 0 ? atomicAdd(n_out, cnt) : 0;
    __syncthreads();
    if (hit) {
      const int32_t u = base + li;
      for (int e = 0; e < dim; e += 4) {
        if (u < cap)
          *reinterpret_cast<float4*>(grads_out + (int64_t)u * dim + e) =
              *reinterpret_cast<const float4*>(grad_table + row * dim + e);
        // over capacity the row's gradient is dropped (never left stale)
        *reinterpret_cast<float4*>(grad_table + row * dim + e) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (u < cap) rows_out[u] = (int32_t)row;
      flag[row] = -1;
    }
    __syncthreads();
  }
}

RS_API int rs_sparse_compact_scan(void* stream, float* grad_table, int32_t* flag,
                                  int64_t table_rows, int dim, int32_t* rows_out,
                                  float* grads_out, int32_t* n_out, int32_t cap) {
  if (!grad_table || !flag || !rows_out || !grads_out || !n_out || dim <= 0 || dim % 4)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  rs_fill_u32(s, n_out, 0u, 1);
  // rows past the count read -1 (the padding the rank-ordered merge skips)
  rs_fill_u32(s, rows_out, 0xFFFFFFFFu, cap);
  if (table_rows == 0) return rs_status_after_launch();
  int64_t grid = (table_rows + 255) / 256;
  if (grid > 4096) grid = 4096;
  sparse_compact_scan_kernel<<<(int)grid, 256, 0, s>>>(grad_table, flag, table_rows, dim,
                                                       rows_out, grads_out, n_out, cap);
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Data-parallel sparse exchange helpers.
//   compact: move this rank's touched rows out of the gradient table into a dense list
//            (rows_out[u], grads_out[u, :]), zero the slots and release the flags, so the
//            table is clean for the rank-ordered merge.
//   merge  : add one rank's list into the table (rows are unique within a list, so plain adds
//            with no atomics), claiming rows into `touched`.  Called once per rank in rank
//            order on every replica -> bitwise-identical sums on all replicas.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sparse_compact_kernel(
    float* __restrict__ grad_table, int32_t* __restrict__ flag, const int32_t* __restrict__ touched,
    const int32_t* __restrict__ n_touched, int dim, int lps, int32_t* __restrict__ rows_out,
    float* __restrict__ grads_out, int32_t cap) {
  const int nrows = min(*n_touched, cap);
  const int per_block = blockDim.x / lps;
  const int gi = threadIdx.x / lps;
  const int l = threadIdx.x % lps;
  for (int u = blockIdx.x * per_block + gi; u < cap; u += gridDim.x * per_block) {
    if (u < nrows) {
      const int64_t row = touched[u];
      for (int e = l; e < dim; e += lps) {
        grads_out[(int64_t)u * dim + e] = grad_table[row * dim + e];
        grad_table[row * dim + e] = 0.f;
      }
      if (l == 0) { rows_out[u] = (int32_t)row; flag[row] = -1; }
    } else {
      if (l == 0) rows_out[u] = -1;  // padding entries are skipped by the merge
    }
  }
}

__global__ void __launch_bounds__(256) sparse_merge_kernel(
    const int32_t* __restrict__ rows, const float* __restrict__ grads, int32_t count, int dim,
    int lps, float* __restrict__ grad_table, int32_t* __restrict__ flag,
    int32_t* __restrict__ touched, int32_t* __restrict__ n_touched, int32_t touched_cap,
    const int32_t* __restrict__ counts, int64_t cstride, int world, int rank,
    int32_t stride = 0, int32_t* __restrict__ overflow = nullptr) {
  // one global n_touched atomic per block (see sparse_grad_accum_kernel)
  __shared__ int32_t nclaim, base;
  __shared__ int32_t lidx[256];
  if (counts && stride > 0) {
    // fixed layout (rs_sparse_merge_rows_dev_stride): rank r's list at r * stride, whatever the
    // counts; a count past stride lost rows in transit -> the sticky overflow word
    const int c = counts[rank * cstride];
    if (overflow && c > stride && blockIdx.x == 0 && threadIdx.x == 0) atomicMax(overflow, c);
    rows += (int64_t)rank * stride;
    grads += (int64_t)rank * stride * dim;
    count = min(c, min(count, stride));
  } else if (counts) {
    // device counts (rs_sparse_merge_rows_dev): every rank's list was gathered as a prefix of
    // nmax = max_r count_r entries, count is this launch's upper bound on every count
    int nmax = 0;
    for (int r = 0; r < world; ++r) nmax = max(nmax, counts[r * cstride]);
    nmax = min(nmax, count);
    const int n = min(counts[rank * cstride], nmax);
    rows += (int64_t)rank * nmax;
    grads += (int64_t)rank * nmax * dim;
    count = n;
  }
  const int per_block = blockDim.x / lps;
  const int gi = threadIdx.x / lps;
  const int l = threadIdx.x % lps;
  for (int u0 = blockIdx.x * per_block; u0 < count; u0 += gridDim.x * per_block) {
    const int u = u0 + gi;
    const int32_t row = u < count ? rows[u] : -1;
    if (threadIdx.x == 0) nclaim = 0;
    __syncthreads();
    if (touched) {
      if (l == 0) lidx[gi] = (row >= 0 && atomicCAS(&flag[row], -1, -2) == -1) ? atomicAdd(&nclaim, 1) : -1;
      __syncthreads();
      if (threadIdx.x == 0) base = nclaim > 0 ? atomicAdd(n_touched, nclaim) : 0;
    } else if (l == 0 && row >= 0) {
      scan_mark(flag, row);  // scan mode
    }
    __syncthreads();
    if (row >= 0) {
      if (touched && l == 0 && lidx[gi] >= 0 && base + lidx[gi] < touched_cap) touched[base + lidx[gi]] = row;
      for (int e = l; e < dim; e += lps)
        grad_table[(int64_t)row * dim + e] += grads[(int64_t)u * dim + e];
    }
    __syncthreads();
  }
}

RS_API int rs_sparse_compact(void* stream, float* grad_table, int32_t* flag,
                             const int32_t* touched, int32_t* n_touched, int dim,
                             int32_t* rows_out, float* grads_out, int32_t cap) {
  if (!grad_table || !flag || !touched || !n_touched || !rows_out || !grads_out || dim <= 0)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int lps = lanes_for_dim(dim);
  if (cap > 0) {
    int64_t grid = ((int64_t)cap * lps + 255) / 256;
    if (grid > 4096) grid = 4096;
    sparse_compact_kernel<<<(int)grid, 256, 0, s>>>(grad_table, flag, touched, n_touched, dim,
                                                    lps, rows_out, grads_out, cap);
  }
  return rs_status_after_launch();
}

RS_API int rs_sparse_merge_rows(void* stream, const int32_t* rows, const float* grads,
                                int32_t count, int dim, float* grad_table, int32_t* flag,
                                int32_t* touched, int32_t* n_touched, int32_t touched_cap) {
  if (!rows || !grads || !grad_table || !flag || dim <= 0) return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  if (count <= 0) return RS_OK;
  const int lps = lanes_for_dim(dim);
  int64_t grid = ((int64_t)count * lps + 255) / 256;
  if (grid > 4096) grid = 4096;
  sparse_merge_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(
      rows, grads, count, dim, lps, grad_table, flag, touched, n_touched, touched_cap, nullptr, 0,
      1, 0);
  return rs_status_after_launch();
}

RS_API int rs_sparse_merge_rows_dev(void* stream, const int32_t* rows_all, const float* grads_all,
                                    const int32_t* counts, int64_t counts_stride, int world,
                                    int rank, int32_t cap, int dim, float* grad_table,
                                    int32_t* flag, int32_t* touched, int32_t* n_touched,
                                    int32_t touched_cap) {
  if (!rows_all || !grads_all || !counts || !grad_table || !flag || dim <= 0 || world <= 0 ||
      rank < 0 || rank >= world || counts_stride <= 0 || cap < 0)
    return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  if (cap == 0) return RS_OK;
  const int lps = lanes_for_dim(dim);
  int64_t grid = ((int64_t)cap * lps + 255) / 256;  // sized for the largest count; extra blocks exit
  if (grid > 4096) grid = 4096;
  sparse_merge_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(
      rows_all, grads_all, cap, dim, lps, grad_table, flag, touched, n_touched, touched_cap, counts,
      counts_stride, world, rank);
  return rs_status_after_launch();
}

RS_API int rs_sparse_merge_rows_dev_stride(void* stream, const int32_t* rows_all,
                                           const float* grads_all, const int32_t* counts,
                                           int64_t counts_stride, int world, int rank,
                                           int32_t stride, int dim, float* grad_table,
                                           int32_t* flag, int32_t* touched, int32_t* n_touched,
                                           int32_t touched_cap, int32_t* overflow) {
  if (!rows_all || !grads_all || !counts || !grad_table || !flag || dim <= 0 || world <= 0 ||
      rank < 0 || rank >= world || counts_stride <= 0 || stride <= 0)
    return RS_ERR_ARG;
  if (touched && !n_touched) return RS_ERR_ARG;
  const int lps = lanes_for_dim(dim);
  int64_t grid = ((int64_t)stride * lps + 255) / 256;  // sized for a full list; extra blocks exit
  if (grid > 4096) grid = 4096;
  sparse_merge_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(
      rows_all, grads_all, stride, dim, lps, grad_table, flag, touched, n_touched, touched_cap,
      counts, counts_stride, world, rank, stride, overflow);
  return rs_status_after_launch();
}

// Keras kernel regularisers folded into the gradient (rank/multi_head/multidnn.py:62-63
// L1L2(1e-5, 1e-5); :85,103 L2(0.01); rough_rank/layer.py:77 L2(l2_reg)):
//   loss += l1 * sum|w| + l2 * sum w^2   =>   grad += l1 * sign(w) + 2 * l2 * w  (tf.sign(0) = 0)
__global__ void l1l2_grad_kernel(const float* __restrict__ w, float* __restrict__ g, int64_t n,
                                 float l1, float l2) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float x = w[i];
    const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    g[i] += fmaf(l1, sg, 2.f * l2 * x);
  }
}

// Several regularised tensors in one launch (a model's regularisers apply after backward, one
// launch each cost ~5 us of launch + tail at config 3): segment k covers elements
// [start[k], start[k + 1]) of the concatenated index space.
constexpr int kL1L2MaxSeg = 16;
struct L1L2Group {
  const float* w[kL1L2MaxSeg];
  float* g[kL1L2MaxSeg];
  int64_t start[kL1L2MaxSeg + 1];
  float l1[kL1L2MaxSeg], l2[kL1L2MaxSeg];
  int n;
};

__global__ void l1l2_grad_group_kernel(L1L2Group a) {
  const int64_t total = a.start[a.n];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int k = 0;
    while (k + 1 < a.n && i >= a.start[k + 1]) ++k;
    const int64_t j = i - a.start[k];
    const float x = a.w[k][j];
    const float sg = x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f);
    a.g[k][j] += fmaf(a.l1[k], sg, 2.f * a.l2[k] * x);
  }
}

RS_API int rs_l1l2_grad_grouped(void* stream, int n, const float* const* params,
                                float* const* grads, const int64_t* counts, const float* l1,
                                const float* l2) {
  if (n < 0 || n > kL1L2MaxSeg || (n > 0 && (!params || !grads || !counts || !l1 || !l2)))
    return RS_ERR_ARG;
  L1L2Group a{};
  a.n = n;
  a.start[0] = 0;
  for (int k = 0; k < n; ++k) {
    if (!params[k] || !grads[k] || counts[k] < 0) return RS_ERR_ARG;
    a.w[k] = params[k];
    a.g[k] = grads[k];
    a.l1[k] = l1[k];
    a.l2[k] = l2[k];
    a.start[k + 1] = a.start[k] + counts[k];
  }
  if (n == 0 || a.start[n] == 0) return RS_OK;
  int64_t grid = (a.start[n] + 255) / 256;
  if (grid > 4096) grid = 4096;
  l1l2_grad_group_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(a);
  return rs_status_after_launch();
}

RS_API int rs_l1l2_grad(void* stream, const float* params, float* grads, int64_t n, float l1,
                        float l2) {
  if (!params || !grads || n < 0) return RS_ERR_ARG;
  if (n == 0) return RS_OK;
  int64_t grid = (n + 255) / 256;
  if (grid > 4096) grid = 4096;
  l1l2_grad_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(params, grads, n, l1, l2);
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Per-block gradient partials -> gradients -> dense Adam, one launch.
// The fused training kernels (InteractingLayer backward, the MLP head) leave one partial row per
// workgroup in a workspace; this kernel sums every column over its rows in a FIXED order (16 row
// groups, each in row order, then the groups in order: bitwise reproducible), writes the
// gradient, and, when adam != 0, applies the tf.keras-form Adam of rs_dense_adam to that element
// in the same pass.  Up to RS_RED_MAXSEG column segments, each mapped to an arena offset (Adam
// applies) or to a plain output (e.g. the per-block loss column -> the batch-mean loss).
// The Adam step counter is read by every block and advanced by the last block to finish
// (completion counter `done`, zero between launches), so no separate increment launch.
// ---------------------------------------------------------------------------------------------
#define RS_RED_MAXSEG 4
#ifndef RS_RED_MAXLG
#define RS_RED_MAXLG 5  // <= 32 row groups: 1536 IL partial rows -> 32 x 32 columns (measured 10.1 vs 10.8 us at 128 x 8)
#endif
struct RedSeg {
  const float* part;
  int64_t ld;
  int32_t nrows;
  int64_t ncols;
  float* out;       // gradient / output destination
  float scale;      // out = sum * scale
  int64_t adam_off; // arena index of column 0 (Adam applies), or -1
  int32_t lg;       // log2 of the row groups per block (G); columns per block = 1024 / G
  int32_t blk0;     // first block of this segment
};
struct RedArgs {
  RedSeg seg[RS_RED_MAXSEG];
  int nseg;
  float *params, *m, *v;
  const int64_t* step_in;
  int64_t* step;
  int32_t* done;
  float lr, b1, b2, eps, grad_scale;
  int adam;
  int32_t nblk_red;  // blocks of the partial reduction; the other blocks run the sparse sweep
  int32_t nblk_scan; // blocks of the sweep; scan_first: they are blocks 0 .. nblk_scan - 1
  int32_t scan_first;
  // fused sparse optimizer tail (rs_partials_reduce_adam_scan): the scan-mode sparse Adam of one
  // table, run by blocks nblk_red .. gridDim.x - 1 beside the dense reduction
  float *st_table, *st_m, *st_v, *st_grad;
  int32_t* st_flag;
  int64_t st_rows;
  int st_dim;
  float st_lr, st_b1, st_b2, st_eps, st_gscale;
  // rows mode (rs_partials_reduce_adam_rows): the step's looked-up rows instead of the flag sweep
  const int32_t* st_list;
  int64_t st_nlist;
  int64_t st_list_stride;      // int32 words between entries (packed DP records: dim + 1)
  const int32_t* st_counts;    // per-segment valid counts (packed DP: one segment per rank), or null
  int64_t st_counts_stride, st_seg_len;
  int32_t st_chunk;            // rows mode: positions per block chunk of the de-duplicating walk (0: off)
};

// Rows mode of the fused sparse Adam: the marked rows are exactly the rows the step looked up
// (single-GPU AutoInt step: only its own push marks the table), so instead of sweeping the 2.6 M
// flags the tail walks the B x F looked-up rows.  One dim/4-lane group per position: its leader
// releases the flag with an atomic exchange and the group that took the -2 updates the row (each
// marked row exactly once, whatever its multiplicity); positions of already-released rows and
// out-of-range ids (-1) do nothing.
__device__ __forceinline__ void rows_opt_block(const RedArgs& a, int vb, int nblk) {
  const int nv = a.st_dim >> 2;
  const int lpr = nv < 64 ? nv : 64;  // lanes per position (a power of two: dim / 4)
  const int per_block = 1024 / lpr;
  const int sub = (int)threadIdx.x % lpr;
  const int lead = ((int)threadIdx.x & 63) - sub;
  for (int64_t i = (int64_t)vb * per_block + threadIdx.x / lpr; i - (threadIdx.x / lpr) < a.st_nlist;
       i += (int64_t)nblk * per_block) {
    bool in = i < a.st_nlist;
    if (in && a.st_counts) {  // packed DP records: rank segment i / seg_len holds counts[seg] valid
      const int64_t seg = i / a.st_seg_len;
      in = (i - seg * a.st_seg_len) < (int64_t)a.st_counts[seg * a.st_counts_stride];
    }
    const int32_t r = in ? a.st_list[i * a.st_list_stride] : -1;
    int own = 0;
    if (sub == 0 && r >= 0 && r < a.st_rows) own = atomicExch(a.st_flag + r, -1) == -2;
    own = __shfl(own, lead, 64);
    if (own) {
      for (int e4 = sub; e4 < nv; e4 += lpr) {
        ScanRow<true> x;
        const int64_t o = (int64_t)r * a.st_dim + 4 * e4;
        x.load(a.st_table, a.st_m, a.st_v, a.st_grad, o);
        x.update_store(a.st_table, a.st_m, a.st_v, a.st_grad, o, a.st_lr, a.st_b1, a.st_b2,
                       a.st_eps, a.st_gscale);
      }
    }
  }
}

// Rows mode with a per-block de-duplication (round 5).  A Zipf batch looks the hottest row of
// each field up in ~18 % of its samples, so in rows_opt_block those rows' positions (~750 each at
// B = 4096) all race for one flag word and their atomic exchanges serialise at the memory side
// (rows mode lost to the flag sweep above B = 1024).  Here a block takes a chunk of P <= 1024
// consecutive positions (one per thread) and:
//   1. inserts their rows into an LDS hash (2P slots, linear probing, atomicCAS): one entry per
//      distinct row of the chunk -> a distinct-row list;
//   2. one thread per distinct row releases the row's flag with ONE global atomic exchange; the
//      rows it took from -2 (marked by this step's push and not yet taken by another chunk) go
//      to an owned list;
//   3. dim/4-lane groups apply the sparse Adam to the owned rows (each marked row exactly once,
//      the same per-row arithmetic as the sweep).
// A hot row now costs one exchange per chunk that holds it instead of one per position.
__device__ __forceinline__ void rows_opt_block_dedup(const RedArgs& a, int vb, int nblk, int P) {
  __shared__ int32_t keys[2048];
  __shared__ int32_t dlist[1024];
  __shared__ int32_t olist[1024];
  __shared__ int32_t ncnt[2];
  const int nv = a.st_dim >> 2;
  const int lpr = nv < 64 ? nv : 64;
  const int sub = (int)threadIdx.x % lpr;
  const int S = 2 * P;  // hash slots (a power of two)
  const int t = (int)threadIdx.x;
  for (int64_t c0 = (int64_t)vb * P; c0 < a.st_nlist; c0 += (int64_t)nblk * P) {
    for (int k = t; k < S; k += 1024) keys[k] = -1;
    if (t < 2) ncnt[t] = 0;
    __syncthreads();
    if (t < P) {
      const int64_t i = c0 + t;
      bool in = i < a.st_nlist;
      if (in && a.st_counts) {
        const int64_t seg = i / a.st_seg_len;
        in = (i - seg * a.st_seg_len) < (int64_t)a.st_counts[seg * a.st_counts_stride];
      }
      const int32_t r = in ? a.st_list[i * a.st_list_stride] : -1;
      if (r >= 0 && r < a.st_rows) {
        uint32_t h = ((uint32_t)r * 0x9E3779B1u) >> 16;
        for (;;) {
          h &= (uint32_t)(S - 1);
          const int32_t prev = atomicCAS(&keys[h], -1, r);
          if (prev == -1) { dlist[atomicAdd(&ncnt[0], 1)] = r; break; }
          if (prev == r) break;
          ++h;
        }
      }
    }
    __syncthreads();
    const int nd = ncnt[0];
    for (int k = t; k < nd; k += 1024) {
      const int32_t r = dlist[k];
      if (atomicExch(a.st_flag + r, -1) == -2) olist[atomicAdd(&ncnt[1], 1)] = r;
    }
    __syncthreads();
    const int no = ncnt[1];
    for (int k = t / lpr; k < no; k += 1024 / lpr) {
      const int32_t r = olist[k];
      for (int e4 = sub; e4 < nv; e4 += lpr) {
        ScanRow<true> x;
        const int64_t o = (int64_t)r * a.st_dim + 4 * e4;
        x.load(a.st_table, a.st_m, a.st_v, a.st_grad, o);
        x.update_store(a.st_table, a.st_m, a.st_v, a.st_grad, o, a.st_lr, a.st_b1, a.st_b2,
                       a.st_eps, a.st_gscale);
      }
    }
    __syncthreads();  // the LDS lists are rebuilt for the next chunk
  }
}

// Block shape per segment (host-chosen): G row groups x (1024 / G) columns, G the smallest power
// of two with <= 16 rows per thread (IL partials: 1024 rows -> 64 groups x 16 columns over 70
// blocks; head partials: 256 rows -> 16 x 64 over 224 blocks: the whole launch is one round).  Spreading deep segments over many CUs matters:
// one CU keeps only ~72 KB of loads in flight, so 1024 rows x 32 columns on one CU took ~11 us.
__global__ void __launch_bounds__(1024) partials_reduce_adam_kernel(RedArgs a) {
  // block roles: scan_first -> [sweep | reduction], else [reduction | sweep]; vb = the block's
  // index within its role
  const bool is_scan = a.scan_first ? (int)blockIdx.x < a.nblk_scan : (int)blockIdx.x >= a.nblk_red;
  const int vb = a.scan_first ? (is_scan ? (int)blockIdx.x : (int)blockIdx.x - a.nblk_scan)
                              : (is_scan ? (int)blockIdx.x - a.nblk_red : (int)blockIdx.x);
  if (is_scan && a.st_list) {  // rows mode
    if (a.st_chunk > 0)
      rows_opt_block_dedup(a, vb, a.nblk_scan, a.st_chunk);
    else
      rows_opt_block(a, vb, a.nblk_scan);
    return;
  }
  if (is_scan) {  // the fused sparse sweep (independent of the dense part)
    __shared__ uint32_t lists[16 * kScanLcap];
    const int64_t nwaves = (int64_t)a.nblk_scan * 16;
    const int64_t gw = (int64_t)vb * 16 + (threadIdx.x >> 6);
    scan_opt_wave<true>(a.st_table, a.st_m, a.st_v, a.st_grad, a.st_flag, a.st_rows, a.st_dim,
                        a.st_lr, a.st_b1, a.st_b2, a.st_eps, a.st_gscale, gw, nwaves,
                        lists + (threadIdx.x >> 6) * kScanLcap);
    return;
  }
  __shared__ float red[1024];
  int si = 0;
#pragma unroll
  for (int k = 1; k < RS_RED_MAXSEG; ++k)
    if (k < a.nseg && vb >= a.seg[k].blk0) si = k;  // block-uniform
  const RedSeg sg = a.seg[si];
  const int G = 1 << sg.lg, NC = 1024 >> sg.lg;
  const int lc = threadIdx.x & (NC - 1), g = threadIdx.x >> (10 - sg.lg);
  const int64_t cc = (int64_t)(vb - sg.blk0) * NC + lc;
  const bool col_ok = cc < sg.ncols;
  // Adam operands are fetched before the partial rows, so their round trip overlaps the sums
  const bool do_adam = a.adam && sg.adam_off >= 0 && g == 0 && col_ok;
  float m0 = 0.f, v0 = 0.f, p0 = 0.f, lr_t = 0.f;
  if (do_adam) {
    const int64_t i = sg.adam_off + cc;
    m0 = a.m[i]; v0 = a.v[i]; p0 = a.params[i];
    const int64_t step = a.step_in[0] + 1;
    const float bc1 = 1.0f - powf(a.b1, (float)step);
    const float bc2 = 1.0f - powf(a.b2, (float)step);
    lr_t = a.lr * sqrtf(bc2) / bc1;
  }
  float s = 0.f;
  if (col_ok) {
    const float* p = sg.part + cc;
    // every row of this thread (g, g+G, ...) is loaded before the first add (one memory round
    // trip), then summed in row order (fixed order: deterministic)
    constexpr int MAXR = 16;
    for (int r = g; r < sg.nrows; r += MAXR * G) {
      float v[MAXR];
#pragma unroll
      for (int u = 0; u < MAXR; ++u) {
        const int rr = r + u * G;
        v[u] = rr < sg.nrows ? p[(int64_t)rr * sg.ld] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < MAXR; ++u) s += v[u];
    }
  }
  red[threadIdx.x] = s;  // [g][lc]
  __syncthreads();
  for (int o = G >> 1; o > 0; o >>= 1) {  // fixed pairing: deterministic
    if (g < o) red[threadIdx.x] += red[threadIdx.x + o * NC];
    __syncthreads();
  }
  if (g == 0 && col_ok) {
    const float t = red[lc] * sg.scale;
    sg.out[cc] = t;
    if (do_adam) {
      const int64_t i = sg.adam_off + cc;
      const float gi = t * a.grad_scale;
      const float mi = a.b1 * m0 + (1.0f - a.b1) * gi;
      const float vi = a.b2 * v0 + (1.0f - a.b2) * gi * gi;
      a.m[i] = mi;
      a.v[i] = vi;
      a.params[i] = p0 - lr_t * mi / (sqrtf(vi) + a.eps);
    }
  }
  if (a.adam && a.step) {
    // every block has consumed step_in (the Adam reads above) before it arrives
    if (rs_last_block(a.done, a.nblk_red, vb)) a.step[0] = a.step_in[0] + 1;
  }
}

static int reduce_adam_impl(void* stream, int nseg, const float* const* parts,
                            const int64_t* lds, const int32_t* nrows, const int64_t* ncols,
                            float* const* outs, const float* scales, const int64_t* adam_offs,
                            float* params, float* m, float* v, int64_t* step, int32_t* done,
                            float lr, float beta1, float beta2, float eps, float grad_scale,
                            int adam, const RedArgs* tail, int64_t tail_blocks) {
  if (nseg <= 0 || nseg > RS_RED_MAXSEG || !parts || !lds || !nrows || !ncols || !outs || !scales ||
      !adam_offs)
    return RS_ERR_ARG;
  if (adam && (!params || !m || !v || !step || !done)) return RS_ERR_ARG;
  RedArgs a{};
  a.nseg = nseg;
  int64_t nblk = 0;
  for (int k = 0; k < nseg; ++k) {
    if (!parts[k] || !outs[k] || nrows[k] < 0 || ncols[k] < 0 || lds[k] < ncols[k]) return RS_ERR_ARG;
    int lg = 0;  // G = 2^lg row groups: <= 16 rows per thread, at most 1024 groups
    while (lg < RS_RED_MAXLG && ((int64_t)16 << lg) < nrows[k]) ++lg;
    const int64_t nc = 1024 >> lg;
    a.seg[k] = RedSeg{parts[k], lds[k], nrows[k], ncols[k], outs[k], scales[k], adam_offs[k], lg,
                      (int32_t)nblk};
    nblk += (ncols[k] + nc - 1) / nc;
  }
  for (int k = nseg; k < RS_RED_MAXSEG; ++k) a.seg[k].blk0 = (int32_t)nblk;
  a.params = params; a.m = m; a.v = v;
  a.step_in = step; a.step = step; a.done = done;
  a.lr = lr; a.b1 = beta1; a.b2 = beta2; a.eps = eps; a.grad_scale = grad_scale; a.adam = adam;
  a.nblk_red = (int32_t)nblk;
  a.nblk_scan = tail ? (int32_t)tail_blocks : 0;
  // the sweep's blocks first: its per-wave chains are the longer ones (same-box A/B: 0.1586 vs
  // 0.1589 ms per step reduction-first; 0.1643 ms as two launches)
  a.scan_first = tail ? 1 : 0;
  if (tail) {
    a.st_table = tail->st_table; a.st_m = tail->st_m; a.st_v = tail->st_v;
    a.st_grad = tail->st_grad; a.st_flag = tail->st_flag; a.st_rows = tail->st_rows;
    a.st_dim = tail->st_dim; a.st_lr = tail->st_lr; a.st_b1 = tail->st_b1; a.st_b2 = tail->st_b2;
    a.st_eps = tail->st_eps; a.st_gscale = tail->st_gscale;
    a.st_list = tail->st_list; a.st_nlist = tail->st_nlist; a.st_list_stride = tail->st_list_stride;
    a.st_counts = tail->st_counts; a.st_counts_stride = tail->st_counts_stride;
    a.st_seg_len = tail->st_seg_len;
    a.st_chunk = tail->st_chunk;
  }
  const int64_t total = nblk + (tail ? tail_blocks : 0);
  if (total == 0) return RS_OK;
  partials_reduce_adam_kernel<<<(unsigned)total, 1024, 0, rs_stream(stream)>>>(a);
  return rs_status_after_launch();
}

RS_API int rs_partials_reduce_adam(void* stream, int nseg, const float* const* parts,
                                   const int64_t* lds, const int32_t* nrows,
                                   const int64_t* ncols, float* const* outs, const float* scales,
                                   const int64_t* adam_offs, float* params, float* m, float* v,
                                   int64_t* step, int32_t* done, float lr, float beta1,
                                   float beta2, float eps, float grad_scale, int adam) {
  return reduce_adam_impl(stream, nseg, parts, lds, nrows, ncols, outs, scales, adam_offs, params,
                          m, v, step, done, lr, beta1, beta2, eps, grad_scale, adam, nullptr, 0);
}

RS_API int rs_partials_reduce_adam_rows_ex(
    void* stream, int nseg, const float* const* parts, const int64_t* lds, const int32_t* nrows,
    const int64_t* ncols, float* const* outs, const float* scales, const int64_t* adam_offs,
    float* params, float* m, float* v, int64_t* step, int32_t* done, float lr, float beta1,
    float beta2, float eps, float grad_scale, int adam, float* table, float* tm, float* tv,
    float* grad_table, int32_t* flag, int64_t table_rows, int dim, float slr, float sbeta1,
    float sbeta2, float seps, float sgrad_scale, const int32_t* rows, int64_t nlist,
    int64_t list_stride, const int32_t* counts, int64_t counts_stride, int64_t seg_len);

RS_API int rs_partials_reduce_adam_rows(
    void* stream, int nseg, const float* const* parts, const int64_t* lds, const int32_t* nrows,
    const int64_t* ncols, float* const* outs, const float* scales, const int64_t* adam_offs,
    float* params, float* m, float* v, int64_t* step, int32_t* done, float lr, float beta1,
    float beta2, float eps, float grad_scale, int adam, float* table, float* tm, float* tv,
    float* grad_table, int32_t* flag, int64_t table_rows, int dim, float slr, float sbeta1,
    float sbeta2, float seps, float sgrad_scale, const int32_t* rows, int64_t nlist) {
  return rs_partials_reduce_adam_rows_ex(
      stream, nseg, parts, lds, nrows, ncols, outs, scales, adam_offs, params, m, v, step, done,
      lr, beta1, beta2, eps, grad_scale, adam, table, tm, tv, grad_table, flag, table_rows, dim, slr,
      sbeta1, sbeta2, seps, sgrad_scale, rows, nlist, 1, nullptr, 0, 0);
}

RS_API int rs_partials_reduce_adam_rows_ex(
    void* stream, int nseg, const float* const* parts, const int64_t* lds, const int32_t* nrows,
    const int64_t* ncols, float* const* outs, const float* scales, const int64_t* adam_offs,
    float* params, float* m, float* v, int64_t* step, int32_t* done, float lr, float beta1,
    float beta2, float eps, float grad_scale, int adam, float* table, float* tm, float* tv,
    float* grad_table, int32_t* flag, int64_t table_rows, int dim, float slr, float sbeta1,
    float sbeta2, float seps, float sgrad_scale, const int32_t* rows, int64_t nlist,
    int64_t list_stride, const int32_t* counts, int64_t counts_stride, int64_t seg_len) {
  if (!table || !tm || !tv || !grad_table || !flag || !rows || dim <= 0 || dim % 4 ||
      (dim / 4) & (dim / 4 - 1) || dim > 256 || table_rows < 0 || nlist < 0 || list_stride < 1 ||
      (counts && (counts_stride < 1 || seg_len < 1)))
    return RS_ERR_ARG;
  RedArgs t{};
  t.st_table = table; t.st_m = tm; t.st_v = tv; t.st_grad = grad_table; t.st_flag = flag;
  t.st_rows = table_rows; t.st_dim = dim; t.st_lr = slr; t.st_b1 = sbeta1; t.st_b2 = sbeta2;
  t.st_eps = seps; t.st_gscale = sgrad_scale; t.st_list = rows; t.st_nlist = nlist;
  t.st_list_stride = list_stride; t.st_counts = counts; t.st_counts_stride = counts_stride;
  t.st_seg_len = counts ? seg_len : 1;
  // the de-duplicating walk (rows_opt_block_dedup): chunks of P positions, P in {256, 512,
  // 1024} so that the walk still spreads over >= 128 blocks; RS_ROWS_DEDUP=0 keeps the
  // one-exchange-per-position walk (A/B).  Same box, 200 steps: B = 512 0.0547 -> 0.0534 ms;
  // rows mode at B = 4096 0.1687 -> 0.1561 ms (the flag sweep, 0.1512, stays the choice there)
  static const bool dedup = [] {
    const char* e = getenv("RS_ROWS_DEDUP");
    return !(e && e[0] == '0');
  }();
  int64_t per_block = 1024 / (dim / 4 < 64 ? dim / 4 : 64);
  if (dedup) {
    int P = 1024;
    while (P > 256 && (nlist + P - 1) / P < 128) P >>= 1;
    t.st_chunk = P;
    per_block = P;
  }
  int64_t blocks = (nlist + per_block - 1) / per_block;
  if (blocks < 1) blocks = 1;
  if (blocks > 1024) blocks = 1024;
  return reduce_adam_impl(stream, nseg, parts, lds, nrows, ncols, outs, scales, adam_offs, params,
                          m, v, step, done, lr, beta1, beta2, eps, grad_scale, adam, &t, blocks);
}

RS_API int rs_partials_reduce_adam_scan(
    void* stream, int nseg, const float* const* parts, const int64_t* lds, const int32_t* nrows,
    const int64_t* ncols, float* const* outs, const float* scales, const int64_t* adam_offs,
    float* params, float* m, float* v, int64_t* step, int32_t* done, float lr, float beta1,
    float beta2, float eps, float grad_scale, int adam, float* table, float* tm, float* tv,
    float* grad_table, int32_t* flag, int64_t table_rows, int dim, float slr, float sbeta1,
    float sbeta2, float seps, float sgrad_scale) {
  if (!table || !tm || !tv || !grad_table || !flag || dim <= 0 || dim % 4 || table_rows < 0 ||
      table_rows > (int64_t)UINT32_MAX)
    return RS_ERR_ARG;
  RedArgs t{};
  t.st_table = table; t.st_m = tm; t.st_v = tv; t.st_grad = grad_table; t.st_flag = flag;
  t.st_rows = table_rows; t.st_dim = dim; t.st_lr = slr; t.st_b1 = sbeta1; t.st_b2 = sbeta2;
  t.st_eps = seps; t.st_gscale = sgrad_scale;
  // at most 256 16-wave blocks (4096 waves, ~10 chunks each at 2.6 M rows): with the ~300
  // reduction blocks the launch stays about one resident round (2 such blocks per CU)
  int64_t tail_blocks = table_rows ? (scan_grid(table_rows) * (kScanBlock / 64) + 15) / 16 : 0;
  // the sweep takes the resident round's blocks the reduction leaves (2 x 1024-thread blocks per
  // CU x 256 CUs), at least 256: each wave's flag chunks then load in one or two PF batches
  // (small batches leave few reduction blocks: B = 512 per GPU -> ~450 sweep blocks)
  int64_t nblk_red = 0;
  for (int k = 0; nrows && ncols && k < nseg && k < RS_RED_MAXSEG; ++k) {
    int lg = 0;
    while (lg < RS_RED_MAXLG && ((int64_t)16 << lg) < nrows[k]) ++lg;
    const int64_t nc = 1024 >> lg;
    nblk_red += (ncols[k] + nc - 1) / nc;
  }
  static const int64_t cap_total = [] {  // tuning runs: RS_TAIL_BLOCKS (resident-round target)
    const char* e = getenv("RS_TAIL_BLOCKS");
    const long long v = e ? atoll(e) : 0;
    return (int64_t)(v > 0 ? v : 512);
  }();
  int64_t cap_blocks = cap_total - nblk_red;
  if (cap_blocks < 256) cap_blocks = 256;
  if (tail_blocks > cap_blocks) tail_blocks = cap_blocks;
  return reduce_adam_impl(stream, nseg, parts, lds, nrows, ncols, outs, scales, adam_offs, params,
                          m, v, step, done, lr, beta1, beta2, eps, grad_scale, adam, &t,
                          tail_blocks);
}
