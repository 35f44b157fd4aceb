// N2 owner-sharded embedding tables (SURVEY §8(e) "owner-sharded rows", §8(f) N2): under data
// parallelism over N ranks a table of R rows is split by owner = row % N (rank r holds the rows
// r, r + N, r + 2N, ... at local index row / N), so a 10M x 32 table and its optimizer slots take
// 1/N of each GPU's HBM and the sparse exchange becomes a reduce-scatter to the owners instead of
// an all-gather of every rank's touched rows.  tensornet's PS does the same split on the host
// (rank/ctr/base_model.py:89-102 feeds it; staytime/VideoDnn.py:233 names its optimizer).
//
// Per lookup (embedding.py ShardedSparseTable drives the RCCL all-to-alls between these):
//   rows      rs_embedding_lookup_fwd / rs_sequence_lookup_fwd in rows-only mode (NULL table)
//   route     rs_owner_route: stable sort of the n ids by owner (hipcub radix sort over
//             ceil(log2(N + 1)) bits, invalid rows keyed N and dropped), per-owner counts,
//             send_local[i] = row / N and send_pos[i] = the id's position, in owner order
//   gather    (owner) rs_gather_rows(shard, recv_local) -> the rows asked for
//   scatter   rs_scatter_rows(received rows, send_pos) -> per-id rows in id order (zero rows
//             for invalid ids)
// and per backward:
//   expand    rs_segment_expand: dE[k] = scale(segment of k) * dout[segment] (VarLen combiner)
//   gather    rs_gather_rows(dE, send_pos) -> gradients in owner order
//   push      (owner) rs_sparse_grad_accumulate over recv_local into the shard's gradient rows.
// All launches are async on the caller's stream; the only host sync is the count exchange.
// Sync-free form (rs_owner_route_fixed): every (requester, owner) pair gets a fixed block of cap
// slots, so the all-to-alls have equal splits known before the step (no count exchange, no host
// read, capturable in a HIP graph); pads carry row -1 (zero rows on gather, skipped by the push)
// and a per-owner count past cap is recorded in a sticky stats word.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace {

int owner_bits(int world) {
  int b = 1;
  while ((1 << b) <= world) ++b;  // keys 0 .. world (world = invalid) fit
  return b;
}

__global__ void owner_keys_kernel(const int32_t* __restrict__ rows, int64_t n, int world,
                                  int64_t table_rows, uint32_t* __restrict__ keys,
                                  int32_t* __restrict__ pos) {
  for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int32_t r = rows[k];
    keys[k] = (r >= 0 && r < table_rows) ? (uint32_t)(r % world) : (uint32_t)world;
    pos[k] = (int32_t)k;
  }
}

// counts[w] = ids owned by w (int atomics: order-independent result)
__global__ void owner_emit_kernel(const int32_t* __restrict__ rows, const uint32_t* __restrict__ keys,
                                  const int32_t* __restrict__ pos_sorted, int64_t n, int world,
                                  int32_t* __restrict__ send_local, int32_t* __restrict__ send_pos,
                                  int32_t* __restrict__ counts) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = keys[i];
    const int32_t p = pos_sorted[i];
    send_pos[i] = p;
    if (w < (uint32_t)world) {
      send_local[i] = rows[p] / world;
      atomicAdd(&counts[w], 1);
    } else {
      send_local[i] = -1;
    }
  }
}

__global__ void zero_counts_kernel(int32_t* counts, int world) {
  if (threadIdx.x < world) counts[threadIdx.x] = 0;
}

// one G-lane group per row, float4 per lane
template <bool SCATTER>
__global__ void __launch_bounds__(256) rows_move_kernel(const float* __restrict__ src, int64_t src_ld,
                                                        const int32_t* __restrict__ idx, int64_t n,
                                                        int dim, int G, float* __restrict__ dst,
                                                        int64_t dst_ld) {
  const int per_block = blockDim.x / G;
  const int l = threadIdx.x % G;
  const int nvec = dim >> 2;
  for (int64_t i = (int64_t)blockIdx.x * per_block + threadIdx.x / G; i < n;
       i += (int64_t)gridDim.x * per_block) {
    const int32_t j = idx[i];
    if (SCATTER) {  // dst[idx[i]] = src[i]   (idx < 0: dropped)
      if (j < 0) continue;
      const float4* s = reinterpret_cast<const float4*>(src + i * src_ld);
      float4* d = reinterpret_cast<float4*>(dst + (int64_t)j * dst_ld);
      for (int v = l; v < nvec; v += G) d[v] = s[v];
    } else {  // dst[i] = src[idx[i]]   (idx < 0: zero row)
      float4* d = reinterpret_cast<float4*>(dst + i * dst_ld);
      if (j < 0) {
        for (int v = l; v < nvec; v += G) d[v] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      const float4* s = reinterpret_cast<const float4*>(src + (int64_t)j * src_ld);
      for (int v = l; v < nvec; v += G) d[v] = s[v];
    }
  }
}

__device__ __forceinline__ float seg_scale(int n, int combiner) {
  if (n <= 0) return 0.f;
  if (combiner == 1) return 1.0f / (float)n;
  if (combiner == 2) return 1.0f / sqrtf((float)n);
  return 1.0f;
}

// dE[k] = scale(s) * dout[b*ld + f*fstride] for every id k of segment s = b*F + f
__global__ void __launch_bounds__(256) segment_expand_kernel(
    const float* __restrict__ dout, int64_t dout_ld, int64_t dout_fstride,
    const int32_t* __restrict__ offsets, int64_t nseg, int F, int combiner, int dim, int G,
    float* __restrict__ dE) {
  const int per_block = blockDim.x / G;
  const int l = threadIdx.x % G;
  const int nvec = dim >> 2;
  for (int64_t s = (int64_t)blockIdx.x * per_block + threadIdx.x / G; s < nseg;
       s += (int64_t)gridDim.x * per_block) {
    const int64_t b = s / F, f = s - b * F;
    const int32_t beg = offsets[s], end = offsets[s + 1];
    const float sc = seg_scale(end - beg, combiner);
    const float4* src = reinterpret_cast<const float4*>(dout + b * dout_ld + f * dout_fstride);
    for (int v = l; v < nvec; v += G) {
      float4 g = src[v];
      g.x *= sc; g.y *= sc; g.z *= sc; g.w *= sc;
      for (int32_t k = beg; k < end; ++k) reinterpret_cast<float4*>(dE + (int64_t)k * dim)[v] = g;
    }
  }
}

// fixed-capacity routing (rs_owner_route_fixed): start[w] = first sorted position of owner w
// (binary search over the sorted keys, w = 0 .. world), the largest per-owner count folded into
// the sticky stats word (device-side overflow detection / capacity measurement, no host read)
__global__ void owner_bounds_kernel(const uint32_t* __restrict__ keys, int64_t n, int world,
                                    int32_t* __restrict__ start, int32_t* __restrict__ stats) {
  __shared__ int32_t s[1025];
  for (int w = threadIdx.x; w <= world; w += blockDim.x) {
    int64_t lo = 0, hi = n;  // first i with keys[i] >= w
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < (uint32_t)w) lo = mid + 1; else hi = mid;
    }
    s[w] = (int32_t)lo;
    start[w] = (int32_t)lo;
  }
  __syncthreads();
  int32_t mx = 0;
  for (int w = threadIdx.x; w < world; w += blockDim.x) mx = max(mx, s[w + 1] - s[w]);
  for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0 && mx > 0) atomicMax(&stats[0], mx);
}

// id i (owner order) -> slot w * cap + (i - start[w]) of the fixed [world][cap] send layout;
// ids past an owner's cap and invalid rows get slot -1 (dropped; the stats word says so)
__global__ void owner_emit_fixed_kernel(const int32_t* __restrict__ rows,
                                        const uint32_t* __restrict__ keys,
                                        const int32_t* __restrict__ pos_sorted,
                                        const int32_t* __restrict__ start, int64_t n, int world,
                                        int cap, int32_t* __restrict__ send_local,
                                        int32_t* __restrict__ slot) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = keys[i];
    const int32_t p = pos_sorted[i];
    int32_t sl = -1;
    if (w < (uint32_t)world) {
      const int64_t k = i - start[w];
      if (k < cap) {
        sl = (int32_t)(w * (int64_t)cap + k);
        send_local[sl] = rows[p] / world;
      }
    }
    slot[p] = sl;
  }
}

__global__ void fill_i32_kernel(int32_t* __restrict__ p, int64_t n, int32_t v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

struct RouteWs {
  uint32_t *keys_in, *keys_out;
  int32_t *pos_in, *pos_out;
  void* temp;
  int32_t* start;  // [world + 1] (rs_owner_route_fixed)
  size_t temp_bytes, total;
};

size_t al256(size_t v) { return (v + 255) & ~(size_t)255; }

RouteWs carve_route(char* base, int64_t n, int world) {
  RouteWs w{};
  const int ni = (int)(n > 0 ? n : 1);
  size_t t = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (int32_t*)nullptr, (int32_t*)nullptr, ni, 0,
                                     owner_bits(world));
  w.temp_bytes = t;
  size_t off = 0;
  auto take = [&](size_t bytes) { char* p = base ? base + off : nullptr; off += al256(bytes); return p; };
  const size_t a = (size_t)ni * 4;
  w.keys_in = (uint32_t*)take(a);
  w.keys_out = (uint32_t*)take(a);
  w.pos_in = (int32_t*)take(a);
  w.pos_out = (int32_t*)take(a);
  w.temp = take(t);
  w.start = (int32_t*)take((size_t)(world + 1) * 4);
  w.total = off;
  return w;
}

int group_lanes(int dim) {
  int G = 1;
  while (G < dim / 4 && G < 64) G <<= 1;
  return G;
}

unsigned grid_for(int64_t items, int per_block) {
  int64_t g = (items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  return (unsigned)(g > 8192 ? 8192 : g);
}

}  // namespace

RS_API int64_t rs_owner_route_workspace_bytes(int64_t n, int world) {
  if (n < 0 || n > INT32_MAX || world < 1 || world > 1024) return -1;
  return (int64_t)carve_route(nullptr, n, world).total;
}

RS_API int rs_owner_route(void* stream, const int32_t* rows, int64_t n, int world,
                          int64_t table_rows, int32_t* send_local, int32_t* send_pos,
                          int32_t* counts, void* workspace, int64_t workspace_bytes) {
  if (!counts || world < 1 || world > 1024 || n < 0 || n > INT32_MAX || table_rows <= 0)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  zero_counts_kernel<<<1, 1024, 0, s>>>(counts, world);
  if (n == 0) return rs_status_after_launch();
  if (!rows || !send_local || !send_pos || !workspace) return RS_ERR_ARG;
  const RouteWs w = carve_route((char*)workspace, n, world);
  if ((int64_t)w.total > workspace_bytes) return RS_ERR_ARG;
  const unsigned nb = grid_for(n, 256);
  owner_keys_kernel<<<nb, 256, 0, s>>>(rows, n, world, table_rows, w.keys_in, w.pos_in);
  size_t tb = w.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.keys_in, w.keys_out, w.pos_in, w.pos_out,
                                         (int)n, 0, owner_bits(world), s) != hipSuccess)
    return RS_ERR_LAUNCH;
  owner_emit_kernel<<<nb, 256, 0, s>>>(rows, w.keys_out, w.pos_out, n, world, send_local, send_pos,
                                       counts);
  return rs_status_after_launch();
}

RS_API int rs_owner_route_fixed(void* stream, const int32_t* rows, int64_t n, int world,
                                int64_t table_rows, int cap, int32_t* send_local, int32_t* slot,
                                int32_t* stats, void* workspace, int64_t workspace_bytes) {
  if (world < 1 || world > 1024 || n < 0 || n > INT32_MAX || table_rows <= 0 || cap < 1 ||
      (int64_t)world * cap > INT32_MAX || !send_local || !stats)
    return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int64_t ns = (int64_t)world * cap;
  fill_i32_kernel<<<grid_for(ns, 256), 256, 0, s>>>(send_local, ns, -1);
  if (n == 0) return rs_status_after_launch();
  if (!rows || !slot || !workspace) return RS_ERR_ARG;
  const RouteWs w = carve_route((char*)workspace, n, world);
  if ((int64_t)w.total > workspace_bytes) return RS_ERR_ARG;
  const unsigned nb = grid_for(n, 256);
  owner_keys_kernel<<<nb, 256, 0, s>>>(rows, n, world, table_rows, w.keys_in, w.pos_in);
  size_t tb = w.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(w.temp, tb, w.keys_in, w.keys_out, w.pos_in, w.pos_out,
                                         (int)n, 0, owner_bits(world), s) != hipSuccess)
    return RS_ERR_LAUNCH;
  owner_bounds_kernel<<<1, 1024, 0, s>>>(w.keys_out, n, world, w.start, stats);
  owner_emit_fixed_kernel<<<nb, 256, 0, s>>>(rows, w.keys_out, w.pos_out, w.start, n, world, cap,
                                             send_local, slot);
  return rs_status_after_launch();
}

RS_API int rs_gather_rows(void* stream, const float* src, int64_t src_ld, const int32_t* idx,
                          int64_t n, int dim, float* dst, int64_t dst_ld) {
  if (n < 0 || dim <= 0 || dim % 4 || src_ld % 4 || dst_ld % 4) return RS_ERR_ARG;
  if (n == 0) return RS_OK;
  if (!src || !idx || !dst) return RS_ERR_ARG;
  const int G = group_lanes(dim);
  rows_move_kernel<false><<<grid_for(n, 256 / G), 256, 0, rs_stream(stream)>>>(src, src_ld, idx, n,
                                                                              dim, G, dst, dst_ld);
  return rs_status_after_launch();
}

RS_API int rs_scatter_rows(void* stream, const float* src, int64_t src_ld, const int32_t* idx,
                           int64_t n, int dim, float* dst, int64_t dst_ld) {
  if (n < 0 || dim <= 0 || dim % 4 || src_ld % 4 || dst_ld % 4) return RS_ERR_ARG;
  if (n == 0) return RS_OK;
  if (!src || !idx || !dst) return RS_ERR_ARG;
  const int G = group_lanes(dim);
  rows_move_kernel<true><<<grid_for(n, 256 / G), 256, 0, rs_stream(stream)>>>(src, src_ld, idx, n,
                                                                             dim, G, dst, dst_ld);
  return rs_status_after_launch();
}

RS_API int rs_segment_expand(void* stream, const float* dout, int64_t dout_ld, int64_t dout_fstride,
                             const int32_t* offsets, int64_t B, int F, int combiner, int dim,
                             float* dE) {
  if (B < 0 || F <= 0 || dim <= 0 || dim % 4 || dout_ld % 4 || dout_fstride % 4) return RS_ERR_ARG;
  if (combiner < 0 || combiner > 2) return RS_ERR_ARG;
  const int64_t nseg = B * (int64_t)F;
  if (nseg == 0) return RS_OK;
  if (!dout || !offsets || !dE) return RS_ERR_ARG;
  const int G = group_lanes(dim);
  segment_expand_kernel<<<grid_for(nseg, 256 / G), 256, 0, rs_stream(stream)>>>(
      dout, dout_ld, dout_fstride, offsets, nseg, F, combiner, dim, G, dE);
  return rs_status_after_launch();
}
