// Deterministic sparse push: the backward half of EmbeddingFeatures
// (tensornet's PS push; rank/ctr/base_model.py:203-217, staytime/VideoDnn.py:217-244) as
// sort + segmented sum instead of float atomics, so every touched row's gradient is the sum of
// its occurrences in a fixed order (the sorted run layout) -- bitwise reproducible run to run and independent of
// scheduling (rs_sparse_grad_accumulate's LDS hash + atomics reproduce the row SET exactly but not
// the last bits of each sum).
//
//   1. keys = rows (uint32; -1 -> 0xFFFFFFFF sorts last), values = id index k
//   2. hipcub radix sort by key (stable: equal rows keep ascending k)
//   3. run-length encode the sorted keys -> unique rows, counts; exclusive scan -> run starts
//   4. one wave per run: the lanes sum strided slices of the run's occurrences
//      (scale(segment) * dout[segment]) in order and combine them with a fixed butterfly, then add
//      the total to grad_table[row] with a plain read-modify-write (the run owns its row: no
//      atomics), and mark / claim the row exactly like the atomic push.
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

// One wave per run (grid-stride over the device run count): lane l sums the run's occurrences
// l, l + 64, l + 128, ... in order, 16 dims per pass (4 float4 loads per occurrence), then the 64
// lane sums are combined by a fixed xor butterfly and lane e writes dim e.  Every association is
// fixed by the run's layout, never by scheduling: bitwise reproducible, and a Zipf-hot row with
// thousands of occurrences costs ~count/512 load round trips instead of count.
constexpr int kRedWaves = 4;

__global__ void __launch_bounds__(64 * kRedWaves) sorted_reduce_kernel(
    const uint32_t* __restrict__ ukeys, const int32_t* __restrict__ idx,
    const int32_t* __restrict__ run_start, const int32_t* __restrict__ run_len,
    const int32_t* __restrict__ num_runs, const int32_t* __restrict__ seg,
    const int32_t* __restrict__ offsets, int F, const float* __restrict__ dout, int64_t dout_ld,
    int64_t dout_fstride, int dim, int combiner, int64_t table_rows,
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int32_t* __restrict__ touched,
    int32_t* __restrict__ n_touched, int32_t touched_cap) {
  const int lane = threadIdx.x & 63;
  const int64_t nruns = *num_runs;
  const int64_t wstride = (int64_t)gridDim.x * kRedWaves;
  for (int64_t r = (int64_t)blockIdx.x * kRedWaves + (threadIdx.x >> 6); r < nruns; r += wstride) {
    const uint32_t key = ukeys[r];
    if (key == 0xFFFFFFFFu || (int64_t)key >= table_rows) continue;  // invalid ids push nothing
    const int32_t row = (int32_t)key;
    const int32_t beg = run_start[r], end = beg + run_len[r];
    float* dst = grad_table + (int64_t)row * dim;
    for (int e0 = 0; e0 < dim; e0 += 16) {
      const int ne = dim - e0 < 16 ? dim - e0 : 16;  // dim % 4 == 0: whole float4s
      float acc[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      // UN occurrences per lane in flight: their ids, then their rows, are loaded before any is
      // accumulated (a hot run is ~count/64 dependent idx -> dout round trips otherwise); the
      // accumulation order per lane stays ascending
      constexpr int UN = 8;
      for (int32_t i0 = beg + lane; i0 < end; i0 += 64 * UN) {
        int32_t kk[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) kk[u] = i0 + 64 * u < end ? idx[i0 + 64 * u] : -1;
        float4 t[UN][4];
        float sc[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u) {
          sc[u] = 0.f;
          if (kk[u] >= 0) {
            const int32_t s = seg ? seg[kk[u]] : kk[u];
            const int64_t b = s / F, f = s - b * F;
            sc[u] = comb_scale(offsets ? offsets[s + 1] - offsets[s] : 1, combiner);
            const float4* src = reinterpret_cast<const float4*>(dout + b * dout_ld + f * dout_fstride + e0);
#pragma unroll
            for (int v = 0; v < 4; ++v) t[u][v] = 4 * v < ne ? src[v] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
        }
#pragma unroll
        for (int u = 0; u < UN; ++u) {
          if (kk[u] < 0) continue;
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            acc[4 * v + 0] = fmaf(t[u][v].x, sc[u], acc[4 * v + 0]);
            acc[4 * v + 1] = fmaf(t[u][v].y, sc[u], acc[4 * v + 1]);
            acc[4 * v + 2] = fmaf(t[u][v].z, sc[u], acc[4 * v + 2]);
            acc[4 * v + 3] = fmaf(t[u][v].w, sc[u], acc[4 * v + 3]);
          }
        }
      }
      if (end - beg > 1) {  // a single occurrence needs no combine (lane 0 holds it)
#pragma unroll
        for (int m = 1; m < 64; m <<= 1)
#pragma unroll
          for (int e = 0; e < 16; ++e) acc[e] += __shfl_xor(acc[e], m, 64);
      }
      // lane e (e < ne) writes dim e0 + e; after the butterfly every lane holds the totals, and
      // with one occurrence lane 0 holds them: broadcast lane 0's values in that case
      float mine = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float v = end - beg > 1 ? acc[e] : __shfl(acc[e], 0, 64);
        if (lane == e) mine = v;
      }
      if (lane < ne) dst[e0 + lane] += mine;
    }
    if (lane == 0) {
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
  if (dim % 4 || dout_ld % 4 || dout_fstride % 4) return RS_ERR_ARG;  // float4 rows
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
  // one wave per run, grid-stride (the run count stays on the device)
  int64_t grid = (n_ids + kRedWaves - 1) / kRedWaves;
  if (grid > 4096) grid = 4096;
  sorted_reduce_kernel<<<(unsigned)grid, 64 * kRedWaves, 0, s>>>(
      w.ukeys, w.idx_out, w.starts, w.counts, w.num_runs, offsets ? w.seg : nullptr, offsets, F,
      dout, dout_ld, dout_fstride, dim, combiner, table_rows, grad_table, flag, touched,
      n_touched, touched_cap);
  return rs_status_after_launch();
}
