// Deterministic sparse push: the backward half of EmbeddingFeatures
// (tensornet's PS push; rank/ctr/base_model.py:203-217, staytime/VideoDnn.py:217-244) as
// sort + segmented sum instead of float atomics, so every touched row's gradient is the sum of
// its occurrences in ascending id order -- bitwise reproducible run to run and independent of
// scheduling (rs_sparse_grad_accumulate's LDS hash + atomics reproduce the row SET exactly but not
// the last bits of each sum).
//
//   1. keys = rows (uint32; -1 -> 0xFFFFFFFF sorts last), values = id index k
//   2. hipcub radix sort by key (stable: equal rows keep ascending k)
//   3. run-length encode the sorted keys -> unique rows, counts; exclusive scan -> run starts
//   4. one lane group per run: sum scale(segment) * dout[segment] over the run in order, add it to
//      grad_table[row] with a plain read-modify-write (the run owns its row: no atomics), mark /
//      claim the row exactly like the atomic push.
// Every step is an async launch on the caller's stream (run count stays on the device), so the
// sequence is graph-capturable; the caller provides the workspace
// (rs_sparse_sorted_workspace_bytes).
#include <hipcub/hipcub.hpp>

#include "common.hpp"

enum { RS_COMB_SUM = 0, RS_COMB_MEAN = 1, RS_COMB_SQRTN = 2 };

namespace {

__device__ __forceinline__ float comb_scale(int n, int combiner) {
  if (n <= 0) return 0.f;
  if (combiner == RS_COMB_MEAN) return 1.0f / (float)n;
  if (combiner == RS_COMB_SQRTN) return 1.0f / sqrtf((float)n);
  return 1.0f;
}

__global__ void sorted_keys_kernel(const int32_t* __restrict__ rows, int64_t n,
                                   uint32_t* __restrict__ keys, int32_t* __restrict__ idx) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    keys[k] = (uint32_t)rows[k];
    idx[k] = (int32_t)k;
  }
}

// seg[k] = the segment of id k (VarLen fields: ids of segment s are offsets[s] .. offsets[s+1])
__global__ void seg_of_kernel(const int32_t* __restrict__ offsets, int64_t nseg,
                              int32_t* __restrict__ seg) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < nseg;
       s += (int64_t)gridDim.x * blockDim.x)
    for (int32_t k = offsets[s]; k < offsets[s + 1]; ++k) seg[k] = (int32_t)s;
}

__global__ void __launch_bounds__(256) sorted_reduce_kernel(
    const uint32_t* __restrict__ ukeys, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ run_start, const int32_t* __restrict__ run_len,
    const int32_t* __restrict__ num_runs, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ offsets, int F, const float* __restrict__ dout, int64_t dout_ld,
    int64_t dout_fstride, int dim, int combiner, int G, int64_t table_rows,
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int32_t* __restrict__ touched,
    int32_t* __restrict__ n_touched, int32_t touched_cap) {
  const int per_block = blockDim.x / G;
  const int64_t r = (int64_t)blockIdx.x * per_block + threadIdx.x / G;
  const int l = threadIdx.x % G;
  if (r >= *num_runs) return;
  const uint32_t key = ukeys[r];
  if (key == 0xFFFFFFFFu || (int64_t)key >= table_rows) return;  // invalid ids push nothing
  const int32_t row = (int32_t)key;
  const int32_t beg = run_start[r], end = beg + run_len[r];
  float acc[2] = {0.f, 0.f};  // dim <= 2 * G (G = 64 at most: dim <= 128)
  for (int32_t i = beg; i < end; ++i) {
    const int32_t k = idx[i];
    const int32_t s = seg ? seg[k] : k;
    const int64_t b = s / F, f = s - b * F;
    const float sc = comb_scale(offsets ? offsets[s + 1] - offsets[s] : 1, combiner);
    const float* src = dout + b * dout_ld + f * dout_fstride;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = l + u * G;
      if (e < dim) acc[u] = fmaf(src[e], sc, acc[u]);
    }
  }
  float* dst = grad_table + (int64_t)row * dim;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = l + u * G;
    if (e < dim) dst[e] += acc[u];
  }
  if (l == 0) {
    if (touched) {
      if (atomicCAS(&flag[row], -1, -2) == -1) {
        const int32_t t = atomicAdd(n_touched, 1);
        if (t < touched_cap) touched[t] = row;
      }
    } else {
      flag[row] = -2;  // scan mark
    }
  }
}

struct SortedWs {
  uint32_t *keys_in, *keys_out, *ukeys;
  int32_t *idx_in, *idx_out, *counts, *starts, *seg, *num_runs;
  void* temp;
  size_t temp_bytes, total;
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// carve the workspace (base == nullptr: sizes only)
SortedWs carve(char* base, int64_t n) {
  SortedWs w{};
  size_t t1 = 0, t2 = 0, t3 = 0;
  const int ni = (int)(n > 0 ? n : 1);
  hipcub::DeviceRadixSort::SortPairs(nullptr, t1, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (int32_t*)nullptr, (int32_t*)nullptr, ni, 0, 32);
  hipcub::DeviceRunLengthEncode::Encode(nullptr, t2, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                        (int32_t*)nullptr, (int32_t*)nullptr, ni);
  hipcub::DeviceScan::ExclusiveSum(nullptr, t3, (int32_t*)nullptr, (int32_t*)nullptr, ni);
  w.temp_bytes = t1 > t2 ? (t1 > t3 ? t1 : t3) : (t2 > t3 ? t2 : t3);
  const size_t a = align256((size_t)ni * 4);
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off += align256(bytes); return p; };
  w.keys_in = (uint32_t*)take(a);
  w.keys_out = (uint32_t*)take(a);
  w.ukeys = (uint32_t*)take(a);
  w.idx_in = (int32_t*)take(a);
  w.idx_out = (int32_t*)take(a);
  w.counts = (int32_t*)take(a);
  w.starts = (int32_t*)take(a);
  w.seg = (int32_t*)take(a);
  w.num_runs = (int32_t*)take(4);
  w.temp = take(w.temp_bytes);
  w.total = off;
  return w;
}

}  // namespace

RS_API int64_t rs_sparse_sorted_workspace_bytes(int64_t n_ids) {
  if (n_ids < 0 || n_ids > INT32_MAX) return -1;
  return (int64_t)carve(nullptr, n_ids).total;
}

RS_API int rs_sparse_grad_accumulate_sorted(void* stream, const int32_t* rows,
                                            const int32_t* offsets, int64_t B, int F,
                                            const float* dout, int64_t dout_ld,
                                            int64_t dout_fstride, int dim, int combiner,
                                            int64_t table_rows, float* grad_table, int32_t* flag,
                                            int32_t* touched, int32_t* n_touched,
                                            int32_t touched_cap, void* workspace,
                                            int64_t workspace_bytes, int64_t n_ids) {
  if (!rows || !dout || !grad_table || !flag || !workspace || F <= 0 || B < 0) return RS_ERR_ARG;
  if (dim <= 0 || dim > 128 || table_rows <= 0 || (touched && !n_touched)) return RS_ERR_ARG;
  if (combiner < RS_COMB_SUM || combiner > RS_COMB_SQRTN) return RS_ERR_ARG;
  // n_ids: ids in the batch (offsets[B*F] with offsets; B*F without -- passed by the caller so
  // that nothing is read back to the host)
  if (!offsets && n_ids != B * (int64_t)F) return RS_ERR_ARG;
  if (n_ids < 0 || n_ids > INT32_MAX) return RS_ERR_ARG;
  if (n_ids == 0) return RS_OK;
  const SortedWs w = carve((char*)workspace, n_ids);
  if ((int64_t)w.total > workspace_bytes) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int ni = (int)n_ids;
  const int nb = (int)((n_ids + 255) / 256 < 4096 ? (n_ids + 255) / 256 : 4096);
  sorted_keys_kernel<<<nb, 256, 0, s>>>(rows, n_ids, w.keys_in, w.idx_in);
  if (offsets) {
    const int64_t nseg = B * (int64_t)F;
    const int ns = (int)((nseg + 255) / 256 < 4096 ? (nseg + 255) / 256 : 4096);
    if (nseg > 0) seg_of_kernel<<<ns, 256, 0, s>>>(offsets, nseg, w.seg);
  }
  size_t tb = w.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.keys_in, w.keys_out, w.idx_in, w.idx_out,
                                         ni, 0, 32, s) != hipSuccess)
    return RS_ERR_LAUNCH;
  tb = w.temp_bytes;
  if (hipcub::DeviceRunLengthEncode::Encode(w.temp, tb, w.keys_out, w.ukeys, w.counts, w.num_runs,
                                            ni, s) != hipSuccess)
    return RS_ERR_LAUNCH;
  tb = w.temp_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(w.temp, tb, w.counts, w.starts, ni, s) != hipSuccess)
    return RS_ERR_LAUNCH;
  int G = 1;
  while (G < dim && G < 64) G <<= 1;
  const int per_block = 256 / G;
  const int64_t grid = (n_ids + per_block - 1) / per_block;  // runs <= ids; extra groups exit
  sorted_reduce_kernel<<<(unsigned)grid, 256, 0, s>>>(
      w.ukeys, w.idx_out, w.starts, w.counts, w.num_runs, offsets ? w.seg : nullptr, offsets, F,
      dout, dout_ld, dout_fstride, dim, combiner, G, table_rows, grad_table, flag, touched,
      n_touched, touched_cap);
  return rs_status_after_launch();
}
