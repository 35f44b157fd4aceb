// Packed scan-mode sparse exchange for the data-parallel AutoInt step.
//
// Replaces tensornet's cross-worker aggregation of the EmbeddingFeatures push (the PS push of
// rank/ctr/base_model.py:203-217 / rank/multi_head/multidnn.py:221-238 run under tensornet's MPI
// data parallelism).  Each rank's touched rows (scan-mode marks left by rs_il_bwd_push) become
// records [row (int32 bits) | grad[dim]], so a rank's whole list is ONE contiguous prefix that
// one all-gather moves; the count travels in the dense-gradient bucket.  Every replica then adds
// the gathered lists in rank order (one launch per rank, counts read on the device, so the
// launches are graph-captured): identical inputs in identical order -> bitwise-identical tables.
#include "common.hpp"

namespace {

constexpr int kBlock = 256;

int64_t sweep_grid(int64_t nrows) {  // one chip-full round of waves, fewer for small tables
  const int64_t chunks = (nrows + 63) / 64;
  int64_t grid = (chunks + kBlock / 64 - 1) / (kBlock / 64);
  return grid > 2048 ? 2048 : (grid < 1 ? 1 : grid);
}

// pack: waves sweep flag[] in 64-row chunks (chunk c to wave c mod W, so the dense chunks at the
// head of each field's Zipf range spread over many waves); per chunk one ballot, one count atomic
// per wave, the hit rows ranked by mbcnt into a wave-local LDS list, then the chunk's records are
// written as one contiguous run of n * (dim + 1) floats (coalesced) and the gradient rows zeroed.
__global__ void __launch_bounds__(kBlock) pack_scan_kernel(
    float* __restrict__ grad_table, int32_t* __restrict__ flag, int64_t nrows, int dim,
    float* __restrict__ recs, int32_t* __restrict__ count_out, int32_t cap) {
  __shared__ int32_t lists[kBlock];
  int32_t* list = lists + (threadIdx.x & ~63);
  const int lane = threadIdx.x & 63;
  const int64_t nchunks = (nrows + 63) / 64;
  const int64_t nwaves = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t gw = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const int rs = dim + 1, nv = dim >> 2;
  for (int64_t c = gw; c < nchunks; c += nwaves) {
    const int64_t row0 = c * 64;
    const bool hit = row0 + lane < nrows && flag[row0 + lane] != -1;
    const uint64_t mask = __ballot(hit);
    if (!mask) continue;
    const int n = __popcll(mask);
    const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                               __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    int base = 0;
    if (lane == 0) base = atomicAdd(count_out, n);
    base = __shfl(base, 0);
    if (hit) {
      list[rank] = lane;
      flag[row0 + lane] = -1;
    }
    wave_lds_sync();
    float* out = recs + (int64_t)base * rs;
    const int total = n * rs;
    for (int i = lane; i < total; i += 64) {
      const int k = i / rs, j = i - k * rs;
      if (base + k >= cap) break;  // k grows with i: every later element is past cap too
      const int64_t row = row0 + list[k];
      // the load is issued for every lane (the select below is branch-free), so its index must
      // stay inside the row for j == 0 too: grad_table[-1] of row 0 lies before the allocation
      const float g = grad_table[row * dim + (j > 0 ? j - 1 : 0)];
      out[i] = j == 0 ? __int_as_float((int32_t)row) : g;
    }
    wave_lds_sync();  // the zeroing below follows every lane's gradient read above
    for (int i = lane; i < n * nv; i += 64) {
      const int k = i / nv, e4 = i - k * nv;
      const int64_t row = row0 + list[k];
      *reinterpret_cast<float4*>(grad_table + row * dim + 4 * e4) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __builtin_amdgcn_wave_barrier();  // list reuse by the next chunk
  }
}

// merge: min(dim, 64) lanes per record, one float each (records are dim + 1 floats, not 16-B
// aligned); grid-stride over the rank's count, which is read on the device together with the
// other ranks' counts (nmax = their max fixes where rank r's records start).
__global__ void __launch_bounds__(kBlock) merge_packed_kernel(
    const float* __restrict__ recs, const int32_t* __restrict__ counts, int64_t cstride, int world,
    int rank, int dim, int lps, float* __restrict__ grad_table, int32_t* __restrict__ flag,
    int64_t nrows, int32_t cap, int32_t stride) {
  int nmax = 0;
  for (int r = 0; r < world; ++r) nmax = max(nmax, counts[r * cstride]);
  nmax = min(nmax, cap);  // the host refuses counts past cap; never read past the buffer
  if (stride > 0) nmax = min(nmax, stride);  // fixed layout: rank r's records at r * stride
  const int n = min(counts[rank * cstride], nmax);
  const int rs = dim + 1;
  const float* rec = recs + (int64_t)rank * (stride > 0 ? stride : nmax) * rs;
  const int per_block = kBlock / lps;
  const int gi = threadIdx.x / lps, l = threadIdx.x % lps;
  for (int u = blockIdx.x * per_block + gi; u < n; u += gridDim.x * per_block) {
    const float* r = rec + (int64_t)u * rs;
    const int64_t row = __float_as_int(r[0]);
    if (row < 0 || row >= nrows) continue;
    for (int e = l; e < dim; e += lps) grad_table[row * dim + e] += r[1 + e];
    if (l == 0) scan_mark(flag, row);
  }
}

}  // namespace

RS_API int rs_sparse_pack_scan(void* stream, float* grad_table, int32_t* flag, int64_t table_rows,
                               int dim, float* records, int32_t* count_out, int32_t cap) {
  if (!grad_table || !flag || !records || !count_out || dim <= 0 || dim % 4 || table_rows < 0 ||
      table_rows > INT32_MAX || cap < 0)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  rs_fill_u32(s, count_out, 0u, 1);
  if (table_rows == 0) return rs_status_after_launch();
  pack_scan_kernel<<<(unsigned)sweep_grid(table_rows), kBlock, 0, s>>>(
      grad_table, flag, table_rows, dim, records, count_out, cap);
  return rs_status_after_launch();
}

RS_API int rs_sparse_merge_packed_stride(void* stream, const float* records,
                                         const int32_t* counts, int64_t counts_stride, int world,
                                         int rank, int dim, float* grad_table, int32_t* flag,
                                         int64_t table_rows, int32_t cap, int32_t stride) {
  if (!records || !counts || !grad_table || !flag || dim <= 0 || world <= 0 || rank < 0 ||
      rank >= world || counts_stride <= 0 || table_rows < 0 || cap < 0 || stride < 0)
    return RS_ERR_ARG;
  const int lps = dim < 64 ? dim : 64;
  merge_packed_kernel<<<1024, kBlock, 0, rs_stream(stream)>>>(
      records, counts, counts_stride, world, rank, dim, lps, grad_table, flag, table_rows, cap,
      stride);
  return rs_status_after_launch();
}

RS_API int rs_sparse_merge_packed(void* stream, const float* records, const int32_t* counts,
                                  int64_t counts_stride, int world, int rank, int dim,
                                  float* grad_table, int32_t* flag, int64_t table_rows,
                                  int32_t cap) {
  return rs_sparse_merge_packed_stride(stream, records, counts, counts_stride, world, rank, dim,
                                       grad_table, flag, table_rows, cap, 0);
}
