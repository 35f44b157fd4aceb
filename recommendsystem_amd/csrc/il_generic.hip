// H3 InteractingLayer for ANY (E, U, H) with U % H == 0 and F <= 256 -- the shapes no compiled-in
// instantiation covers (il_inst_*.hip, il_large.hip).  The reference trains whatever
// model_param['interact'] passes (autoint:30-35 -> InteractingLayer(**...)); its constructor
// defaults are layer_num 1, unit_num 128, head_num 1 (InteractingLayer.py:9-16), so dh = 128 over
// 16-dim embeddings.  Same math as the specialised kernels (InteractingLayer.py:37-61, tied
// weights, keras-layer-normalization LN, the counter-based dropout mask of common.hpp), shapes
// read at run time:
//
//   * one 256-thread workgroup per sample (grid-stride); the sample's x, Q|K|V|R (post-ReLU),
//     the attention output and, in the backward, dY / dK / dV live in LDS (row strides padded to
//     odd word counts: the thread-per-(row, key) score loops read K rows without bank conflicts);
//   * projections: thread = (row, column) over F x 4U, W from L1/L2, one fmaf chain in a fixed
//     order -- the backward recomputes Q/K/V/R with the SAME function, so the recomputed ReLU
//     masks are bit-identical to the forward's;
//   * attention per head in query tiles of QT rows (QT x F scores in LDS): scores thread =
//     (query, key), softmax one wave per row (DPP/shuffle reductions), P.V thread = (query, d);
//   * backward per tile: P, dP = dO.V^T and dS = P (dP - D_i) per (query, key) into LDS, then
//     dQ thread = (query, d) and dK / dV thread = (key, d) accumulated over the tiles (each element
//     owned by one thread: no atomics); projection backward dW / db read-modify-write into the
//     block's partial row (column_reduce over blocks, deterministic), dX = dZ W^T thread = (row, e)
//     -> the previous iteration's dY, dx, or the fused sparse push at iteration 0.
//
// The per-sample working set is F (E + 8U) + 2 QT F + small floats (backward).  When it fits the
// 160 KB LDS (e.g. the constructor defaults (E 16, U 128) up to F = 37 fields) it lives there;
// larger shapes (up to F = 256 at any E, U) run the SAME kernels with the working set in a
// per-workgroup global scratch slab (GS = true: L1 / L2-resident, one slab per workgroup of a
// 256-workgroup grid, grown on demand outside graph capture).  fp32 only (a bf16 math-mode
// request is RS_ERR_UNSUPPORTED).
#include "il_kernels.hpp"

#include <map>
#include <mutex>
#include <vector>

namespace rs_il {
namespace gen {

// threads per workgroup: 256, or 512 where one sample's working set takes more than half the LDS
// (at most two workgroups per CU either way, so twice the waves hide the MFMA / LDS latencies:
// ctor defaults backward 1093 -> 833 us, forward 203 -> 156 us; shapes with several workgroups
// per CU measured 5-15 % slower at 512, profiles/r06/generic/)
constexpr int kBigLds = 64 * 1024;
constexpr int FMAXG = 256;
constexpr size_t kLdsMax = 160 * 1024;

struct Layout {
  int XS, PS, OS;                        // row strides: x rows, Q|K|V|R rows, U-wide rows
  int QT;                                // query rows per attention tile
  int xs, P, O, G, DK, DV, S, PT, rst, hst, acc, rows, total;  // float offsets
};

__host__ __device__ inline Layout make_layout(int F, int E, int U, int H, int QT, bool bwd) {
  Layout l;
  l.XS = E + 1;
  l.PS = 4 * U + 1;
  l.OS = U + 1;
  l.QT = QT;
  int o = 0;
  l.xs = o; o += F * l.XS;  // (iterations > 0 have E == U)
  l.P = o; o += F * l.PS;
  l.O = o; o += F * l.OS;
  l.G = o; if (bwd) o += F * l.OS;
  l.DK = o; if (bwd) o += F * l.OS;
  l.DV = o; if (bwd) o += F * l.OS;
  l.S = o; o += QT * F;
  l.PT = o; if (bwd) o += QT * F;
  l.rst = o; o += 4 * F;
  l.hst = o; o += 4 * H * F;
  l.acc = o; if (bwd) o += 2 * U;
  l.rows = o; if (bwd) o += F;
  l.total = o;
  return l;
}

// the largest query tile (<= 64 rows) whose layout fits the LDS, or 0
inline int pick_qt(int F, int E, int U, int H, bool bwd) {
  for (int qt = F < 64 ? F : 64; qt >= 1; qt = qt > 1 ? qt / 2 : 0) {
    if ((size_t)make_layout(F, E, U, H, qt, bwd).total * 4 <= kLdsMax) return qt;
    if (qt == 1) break;
  }
  return 0;
}

struct GArgs {
  int64_t B;
  int F, E, U, H, L, DH, use_res, drop;
  float eps, drop_rate, inv_keep, sc2, inv_sdh;
  uint64_t seed, seed_off;
  const float *x, *xsave_in, *dy, *W, *bias, *gamma, *beta;
  int64_t dy_ld, y_ld;
  float *y, *xsave, *dx;
  int dx_accumulate;
  float* part;
  const int64_t *g_ids, *g_base, *g_bucket;
  const float* g_table;
  int64_t g_table_rows;
  int32_t* g_rows;
  int g_hash;
  const int32_t* push_rows;
  float* push_table;
  int32_t* push_flag;
  Layout lay;
  float* gscratch;  // GS kernels: lay.total floats per workgroup
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// out(m, n) = init + sum_k A(m, k) B(k, n) over an M x N output in 16 x 16 tiles spread over the
// block's waves (v_mfma_f32_16x16x4_f32, k ascending within each of NACC interleaved chains that
// are summed at the end), with A(m, k) = a[m ams + k aks], B(k, n) = b[k bks + n bns] read from
// LDS (or the GS slab / global W); rows, columns and k past the extents read 0.  init(n) seeds
// every chain-0 row of column n; epi(m, n, v) runs once per in-range output element.
template <int NACC, int NT, class Init, class Epi>
__device__ __forceinline__ void mm16(const float* a, int ams, int aks, const float* b, int bks,
                                     int bns, int M, int N, int K, Init init, Epi epi) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tm = (M + 15) >> 4, tn = (N + 15) >> 4;
  const int r16 = lane & 15, kq = lane >> 4;
  for (int t = w; t < tm * tn; t += NT / 64) {
    const int i0 = (t / tn) << 4, j0 = (t % tn) << 4;
    const int ar = i0 + r16, bc = j0 + r16;
    const bool aok = ar < M, bok = bc < N;
    const float* ap = a + (aok ? ar : 0) * ams + kq * aks;
    const float* bp = b + (bok ? bc : 0) * bns + kq * bks;
    f32x4 c[NACC];
    const float c0 = init(bok ? bc : 0);
    c[0] = f32x4{c0, c0, c0, c0};
#pragma unroll
    for (int q = 1; q < NACC; ++q) c[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
    for (; k0 + 4 * NACC <= K; k0 += 4 * NACC) {
      float av[NACC], bv[NACC];
#pragma unroll
      for (int q = 0; q < NACC; ++q) {
        av[q] = aok ? ap[(k0 + 4 * q) * aks] : 0.f;
        bv[q] = bok ? bp[(k0 + 4 * q) * bks] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < NACC; ++q)
        c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[q], bv[q], c[q], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NACC; ++q) {  // the tail: k0 + 4 q + kq may pass K
      if (k0 + 4 * q >= K) break;
      const bool kok = k0 + 4 * q + kq < K;
      const float av = (aok && kok) ? ap[(k0 + 4 * q) * aks] : 0.f;
      const float bv = (bok && kok) ? bp[(k0 + 4 * q) * bks] : 0.f;
      c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, c[q], 0, 0, 0);
    }
    f32x4 sum = c[0];
#pragma unroll
    for (int q = 1; q < NACC; ++q) sum += c[q];
    if (bok)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = i0 + 4 * kq + r;
        if (m < M) epi(m, bc, sum[r]);
      }
  }
}

__device__ __forceinline__ float zero_init(int) { return 0.f; }


// Q|K|V|R = relu(x W + b) for every (row, column) on the matrix cores: each output is bias + one
// chain over e in ascending order (forward == backward recompute, so the recomputed ReLU masks
// are the forward's)
template <int NT>
__device__ __forceinline__ void project(const GArgs& a, const float* xs, float* P) {
  const int NC = 4 * a.U, PS = a.lay.PS;
  const float* bias = a.bias;
  mm16<1, NT>(xs, a.lay.XS, 1, a.W, NC, 1, a.F, NC, a.E, [&](int n) { return bias[n]; },
          [&](int m, int n, float v) { P[m * PS + n] = fmaxf(v, 0.f); });
}

// scaled scores (base-2 domain) of head h, query rows [i0, i0 + nq) x all keys -> S[nq][F]
template <int NT>
__device__ __forceinline__ void scores(const GArgs& a, const float* P, float* S, int h, int i0,
                                       int nq) {
  const int F = a.F, PS = a.lay.PS;
  const float sc2 = a.sc2;
  mm16<2, NT>(P + i0 * PS + h * a.DH, PS, 1, P + a.U + h * a.DH, 1, PS, nq, F, a.DH, zero_init,
          [&](int m, int n, float v) { S[m * F + n] = v * sc2; });
}

// attention forward of head h, query rows [i0, i0 + nq): O rows (and, with hst, the row stats
// {scaled max, 1 / sum} into hst[(h F + i) 4 + 0..1])
template <int NT>
__device__ void attn_tile_fwd(const GArgs& a, float* sm, int h, int i0, int nq, uint32_t kb,
                              bool stats) {
  const Layout& l = a.lay;
  const int F = a.F;
  float* P = sm + l.P;
  float* S = sm + l.S;
  scores<NT>(a, P, S, h, i0, nq);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int ii = w; ii < nq; ii += NT / 64) {
    float* row = S + ii * F;
    float mx = -INFINITY;
    for (int j = lane; j < F; j += 64) mx = fmaxf(mx, row[j]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int j = lane; j < F; j += 64) {
      const float e = __builtin_amdgcn_exp2f(row[j] - mx);
      row[j] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    const float inv = 1.0f / sum;
    const int i = i0 + ii;
    for (int j = lane; j < F; j += 64) {
      float p = row[j] * inv;
      if (a.drop) p = dropout_keep_k(kb, (uint32_t)h, (uint32_t)i, (uint32_t)j, a.drop_rate) ? p * a.inv_keep : 0.f;
      row[j] = p;
    }
    if (stats && lane == 0) {
      sm[l.hst + (h * F + i) * 4 + 0] = mx;
      sm[l.hst + (h * F + i) * 4 + 1] = inv;
    }
  }
  __syncthreads();
  float* O = sm + l.O + i0 * l.OS + h * a.DH;
  const int OS = l.OS;
  mm16<1, NT>(S, F, 1, P + 2 * a.U + h * a.DH, l.PS, 1, nq, a.DH, F, zero_init,
          [&](int m, int n, float v) { O[m * OS + n] = v; });
  __syncthreads();
}

__device__ __forceinline__ uint32_t layer_key(const GArgs& a, int it, int64_t b) {
  return a.drop ? dropout_sample_key(splitmix64(rs_eff_seed(a.seed, a.seed_off) + (uint64_t)it), (uint32_t)b)
                : 0u;
}

template <bool GS, int NT>
__global__ void __launch_bounds__(NT) fwd_kernel(GArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  float* const sm = GS ? a.gscratch + (int64_t)blockIdx.x * a.lay.total : lds_;
  const Layout& l = a.lay;
  const int F = a.F, U = a.U, E = a.E, XS = l.XS;
  float* xs = sm + l.xs;
  float* P = sm + l.P;
  float* O = sm + l.O;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    for (int idx = threadIdx.x; idx < F * E; idx += NT) {
      const int f = idx / E, e = idx - f * E;
      float v;
      if (a.g_ids) {  // fused single-hot gather (rs_il_fwd_gather)
        const int64_t row = hash_row(a.g_ids[b * F + f], a.g_base[f], a.g_bucket[f], a.g_hash);
        const bool ok = row >= 0 && row < a.g_table_rows;
        v = ok ? a.g_table[row * E + e] : 0.f;
        const_cast<float*>(a.x)[b * F * E + idx] = v;
        if (e == 0 && a.g_rows) a.g_rows[b * F + f] = ok ? (int32_t)row : -1;
      } else {
        v = a.x[b * F * E + idx];
      }
      xs[f * XS + e] = v;
    }
    __syncthreads();
    for (int it = 0; it < a.L; ++it) {
      project<NT>(a, xs, P);
      __syncthreads();
      const uint32_t kb = layer_key(a, it, b);
      for (int h = 0; h < a.H; ++h)
        for (int i0 = 0; i0 < F; i0 += l.QT)
          attn_tile_fwd<NT>(a, sm, h, i0, F - i0 < l.QT ? F - i0 : l.QT, kb, false);
      // LN statistics per row
      for (int f = threadIdx.x; f < F; f += NT) {
        float mean = 0.f;
        for (int u = 0; u < U; ++u) {
          const float o = O[f * l.OS + u];
          mean += fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f);
        }
        mean *= 1.0f / U;
        float var = 0.f;
        for (int u = 0; u < U; ++u) {
          const float o = O[f * l.OS + u];
          const float z = fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f) - mean;
          var = fmaf(z, z, var);
        }
        var *= 1.0f / U;
        sm[l.rst + 4 * f] = mean;
        sm[l.rst + 4 * f + 1] = 1.0f / sqrtf(var + a.eps);
      }
      __syncthreads();
      const bool last = it == a.L - 1;
      for (int idx = threadIdx.x; idx < F * U; idx += NT) {
        const int f = idx / U, u = idx - f * U;
        const float o = O[f * l.OS + u];
        const float z = fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f);
        const float yv = fmaf((z - sm[l.rst + 4 * f]) * sm[l.rst + 4 * f + 1], a.gamma[u], a.beta[u]);
        if (last) {
          a.y[b * a.y_ld + idx] = yv;
        } else {  // E == U (tied weights): the next iteration's input
          xs[f * XS + u] = yv;
          a.xsave[((int64_t)it * a.B + b) * F * U + idx] = yv;
        }
      }
      __syncthreads();
    }
  }
}

template <bool GS, int NT>
__global__ void __launch_bounds__(NT) bwd_kernel(GArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  float* const sm = GS ? a.gscratch + (int64_t)blockIdx.x * a.lay.total : lds_;
  const Layout& l = a.lay;
  const int F = a.F, U = a.U, E = a.E, DH = a.DH, NC = 4 * U, XS = l.XS, PS = l.PS, OS = l.OS;
  const int NPARAM = E * NC + NC + 2 * U;
  float* xs = sm + l.xs;
  float* P = sm + l.P;
  float* O = sm + l.O;      // O, then dQ
  float* G = sm + l.G;      // dY -> dA (= dO) -> dY of the previous iteration
  float* DK = sm + l.DK;
  float* DV = sm + l.DV;
  float* S = sm + l.S;      // scores -> dS
  float* PT = sm + l.PT;    // P after dropout
  float* acc = sm + l.acc;  // dgamma | dbeta over the block's samples
  int32_t* rows = reinterpret_cast<int32_t*>(sm + l.rows);
  float* part = a.part + (int64_t)blockIdx.x * NPARAM;
  for (int k = threadIdx.x; k < E * NC + NC; k += NT) part[k] = 0.f;
  for (int k = threadIdx.x; k < 2 * U; k += NT) acc[k] = 0.f;
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    for (int it = a.L - 1; it >= 0; --it) {
      const float* xin = it == 0 ? a.x + b * F * E : a.xsave_in + ((int64_t)(it - 1) * a.B + b) * F * U;
      for (int idx = threadIdx.x; idx < F * E; idx += NT) {
        const int f = idx / E, e = idx - f * E;
        xs[f * XS + e] = xin[idx];
      }
      if (it == a.L - 1)
        for (int idx = threadIdx.x; idx < F * U; idx += NT) {
          const int f = idx / U, u = idx - f * U;
          G[f * l.OS + u] = a.dy[b * a.dy_ld + idx];
        }
      if (it == 0 && a.push_table)
        for (int f = threadIdx.x; f < F; f += NT) rows[f] = a.push_rows[b * F + f];
      for (int idx = threadIdx.x; idx < F * l.OS; idx += NT) { DK[idx] = 0.f; DV[idx] = 0.f; }
      __syncthreads();
      project<NT>(a, xs, P);
      __syncthreads();
      const uint32_t kb = layer_key(a, it, b);
      for (int h = 0; h < a.H; ++h)
        for (int i0 = 0; i0 < F; i0 += l.QT)
          attn_tile_fwd<NT>(a, sm, h, i0, F - i0 < l.QT ? F - i0 : l.QT, kb, true);
      // ---- epilogue backward: LN, ReLU, residual ----
      for (int f = threadIdx.x; f < F; f += NT) {
        float mean = 0.f;
        for (int u = 0; u < U; ++u) {
          const float o = O[f * l.OS + u];
          mean += fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f);
        }
        mean *= 1.0f / U;
        float var = 0.f;
        for (int u = 0; u < U; ++u) {
          const float o = O[f * l.OS + u];
          const float z = fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f) - mean;
          var = fmaf(z, z, var);
        }
        var *= 1.0f / U;
        const float rstd = 1.0f / sqrtf(var + a.eps);
        float m1 = 0.f, m2 = 0.f;
        for (int u = 0; u < U; ++u) {
          const float o = O[f * l.OS + u];
          const float z = fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f);
          const float gd = G[f * l.OS + u] * a.gamma[u];
          m1 += gd;
          m2 = fmaf(gd, (z - mean) * rstd, m2);
        }
        sm[l.rst + 4 * f] = mean;
        sm[l.rst + 4 * f + 1] = rstd;
        sm[l.rst + 4 * f + 2] = m1 * (1.0f / U);
        sm[l.rst + 4 * f + 3] = m2 * (1.0f / U);
      }
      __syncthreads();
      for (int u = threadIdx.x; u < U; u += NT) {  // dgamma, dbeta (column owners)
        float sg = 0.f, sb = 0.f;
        for (int f = 0; f < F; ++f) {
          const float o = O[f * l.OS + u];
          const float z = fmaxf(a.use_res ? o + P[f * l.PS + 3 * U + u] : o, 0.f);
          const float g = G[f * l.OS + u];
          sg = fmaf(g, (z - sm[l.rst + 4 * f]) * sm[l.rst + 4 * f + 1], sg);
          sb += g;
        }
        acc[u] += sg;
        acc[U + u] += sb;
      }
      __syncthreads();
      for (int idx = threadIdx.x; idx < F * U; idx += NT) {
        const int f = idx / U, u = idx - f * U;
        const float o = O[f * l.OS + u];
        const float r = P[f * l.PS + 3 * U + u];
        const float z = fmaxf(a.use_res ? o + r : o, 0.f);
        const float* rs = sm + l.rst + 4 * f;
        const float xh = (z - rs[0]) * rs[1];
        const float dz = rs[1] * (G[f * l.OS + u] * a.gamma[u] - rs[2] - xh * rs[3]);
        const float da = z > 0.f ? dz : 0.f;
        G[f * l.OS + u] = da;
        P[f * l.PS + 3 * U + u] = (a.use_res && r > 0.f) ? da : 0.f;  // R -> dR (masked)
      }
      __syncthreads();
      for (int idx = threadIdx.x; idx < a.H * F; idx += NT) {  // D = dO . O per (head, row)
        const int h = idx / F, i = idx - h * F;
        float d = 0.f;
        for (int k = 0; k < DH; ++k) d = fmaf(G[i * l.OS + h * DH + k], O[i * l.OS + h * DH + k], d);
        sm[l.hst + idx * 4 + 2] = d;
      }
      __syncthreads();
      // ---- attention backward per head and query tile ----
      for (int h = 0; h < a.H; ++h) {
        for (int i0 = 0; i0 < F; i0 += l.QT) {
          const int nq = F - i0 < l.QT ? F - i0 : l.QT;
          // scores and dP = dO V^T on the matrix cores, then P, dS = P (dP - D) elementwise
          scores<NT>(a, P, S, h, i0, nq);
          mm16<2, NT>(G + i0 * OS + h * DH, OS, 1, P + 2 * U + h * DH, 1, PS, nq, F, DH, zero_init,
                  [&](int m, int n, float v) { PT[m * F + n] = v; });
          __syncthreads();
          for (int idx = threadIdx.x; idx < nq * F; idx += NT) {
            const int ii = idx / F, j = idx - ii * F, i = i0 + ii;
            const float* hs = sm + l.hst + (h * F + i) * 4;
            const float p = __builtin_amdgcn_exp2f(S[idx] - hs[0]) * hs[1];
            float dp = PT[idx];
            float pd = p;
            if (a.drop) {
              const bool keep = dropout_keep_k(kb, (uint32_t)h, (uint32_t)i, (uint32_t)j, a.drop_rate);
              dp = keep ? dp * a.inv_keep : 0.f;
              pd = keep ? p * a.inv_keep : 0.f;
            }
            S[idx] = p * (dp - hs[2]);
            PT[idx] = pd;
          }
          __syncthreads();
          const float isd = a.inv_sdh;
          // dQ rows of the tile (into O: dead after D), dK / dV over the tile's query rows
          float* dq = O + i0 * OS + h * DH;
          mm16<1, NT>(S, F, 1, P + U + h * DH, PS, 1, nq, DH, F, zero_init,
                  [&](int m, int n, float v) { dq[m * OS + n] = v * isd; });
          float* dk = DK + h * DH;
          mm16<1, NT>(S, 1, F, P + i0 * PS + h * DH, PS, 1, F, DH, nq, zero_init,
                  [&](int m, int n, float v) { dk[m * OS + n] += v * isd; });
          float* dv = DV + h * DH;
          mm16<1, NT>(PT, 1, F, G + i0 * OS + h * DH, OS, 1, F, DH, nq, zero_init,
                  [&](int m, int n, float v) { dv[m * OS + n] += v; });
          __syncthreads();
        }
      }
      // ---- dZ = [dQ | dK | dV | dR] through the projection ReLUs, into P's columns (Q, K, V are
      //      dead now): one [F, 4U] operand for dW and dX ----
      for (int idx = threadIdx.x; idx < F * 3 * U; idx += NT) {
        const int f = idx / (3 * U), c = idx - f * 3 * U;
        const float* src = (c < U ? O : c < 2 * U ? DK : DV) + f * OS + (c % U);
        float* pz = P + f * PS + c;
        *pz = *pz > 0.f ? *src : 0.f;
      }
      __syncthreads();
      mm16<1, NT>(xs, 1, XS, P, PS, 1, E, NC, F, zero_init,  // dW (block partial, RMW)
              [&](int m, int n, float v) { part[m * NC + n] += v; });
      for (int c = threadIdx.x; c < NC; c += NT) {
        float s = 0.f;
        for (int f = 0; f < F; ++f) s += P[f * PS + c];
        part[E * NC + c] += s;
      }
      // dX = dZ W^T
      mm16<4, NT>(P, PS, 1, a.W, 1, NC, F, E, NC, zero_init, [&](int f, int e, float s) {
        const int idx = f * E + e;
        if (it > 0) {
          G[f * OS + e] = s;  // E == U: dY of iteration it - 1
        } else if (a.push_table) {
          const int32_t row = rows[f];
          if (row >= 0) {
            if (a.dx_accumulate) s += a.dx[b * F * E + idx];
            if (e == 0) scan_mark(a.push_flag, row);
            atomicAdd(a.push_table + (int64_t)row * E + e, s);
          }
        } else {
          float* d = a.dx + b * F * E + idx;
          *d = a.dx_accumulate ? *d + s : s;
        }
      });
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < 2 * U; k += NT) part[E * NC + NC + k] = acc[k];
}

GArgs make_args(int64_t B, int F, int E, int U, int H, int L, int use_res, float eps,
                float drop_rate, uint64_t seed) {
  GArgs a{};
  a.B = B; a.F = F; a.E = E; a.U = U; a.H = H; a.L = L; a.DH = U / H; a.use_res = use_res;
  a.drop = drop_rate > 0.f;
  a.eps = eps;
  a.drop_rate = drop_rate;
  a.inv_keep = drop_rate > 0.f ? 1.0f / (1.0f - drop_rate) : 1.0f;
  a.sc2 = 1.4426950408889634f / sqrtf((float)(U / H));
  a.inv_sdh = 1.0f / sqrtf((float)(U / H));
  a.seed = seed;
  a.seed_off = (uint64_t)(uintptr_t)rs_seed_offset_now();
  return a;
}

// GS (global-scratch) mode: workgroups of the grid, and the scratch slab shared by every GS launch
// of the process on one device (one stream at a time, like the launches themselves).  Grown only
// outside graph capture (a captured step replays the size its eager warm-up established).  A slab
// is never freed: a graph captured earlier keeps its address baked in, so growing allocates a new
// (geometrically larger) slab and retires the old one for the life of the process.
constexpr int64_t kGsGrid = 256;

float* gs_scratch(size_t floats, hipStream_t s) {
  struct Slab { float* buf = nullptr; size_t cap = 0; std::vector<float*> retired; };
  static std::mutex mu;
  static std::map<int, Slab> slabs;  // keyed by device
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  Slab& sl = slabs[dev];
  if (floats <= sl.cap) return sl.buf;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) != hipSuccess || st != hipStreamCaptureStatusNone) return nullptr;
  size_t want = sl.cap ? 2 * sl.cap : floats;
  if (want < floats) want = floats;
  float* nb = nullptr;
  if (hipMalloc(&nb, want * sizeof(float)) != hipSuccess) return nullptr;
  if (sl.buf) sl.retired.push_back(sl.buf);  // still referenced by captured graphs: kept
  sl.buf = nb;
  sl.cap = want;
  return sl.buf;
}

}  // namespace gen

int il_generic_fwd(const FwdReq& q) {
  using namespace gen;
  if (q.bf16 || q.F > FMAXG || q.U % q.H != 0 || q.E <= 0 || (q.L > 1 && q.E != q.U))
    return RS_ERR_UNSUPPORTED;
  int qt = pick_qt(q.F, q.E, q.U, q.H, false);
  const bool gs = qt == 0;
  if (gs) qt = q.F < 64 ? q.F : 64;
  if (q.B == 0) return RS_OK;
  GArgs a = make_args(q.B, q.F, q.E, q.U, q.H, q.L, q.use_res, q.eps, q.drop_rate, q.seed);
  a.x = q.x; a.W = q.W; a.bias = q.bias; a.gamma = q.gamma; a.beta = q.beta;
  a.y = q.y; a.y_ld = q.y_ld; a.xsave = q.xsave;
  a.g_ids = q.gather_ids; a.g_base = q.gather_base; a.g_bucket = q.gather_bucket;
  a.g_table = q.gather_table; a.g_table_rows = q.gather_table_rows; a.g_rows = q.gather_rows;
  a.g_hash = q.gather_hash;
  a.lay = make_layout(q.F, q.E, q.U, q.H, qt, false);
  if (gs) {
    const int64_t grid = q.B < kGsGrid ? q.B : kGsGrid;
    a.gscratch = gs_scratch((size_t)grid * a.lay.total, q.stream);
    if (!a.gscratch) return RS_ERR_UNSUPPORTED;
    fwd_kernel<true, 256><<<(int)grid, 256, 0, q.stream>>>(a);
    return rs_status_after_launch();
  }
  const int64_t grid = q.B < 4096 ? q.B : 4096;
  if ((size_t)a.lay.total * 4 > kBigLds)
    fwd_kernel<false, 512><<<(int)grid, 512, (size_t)a.lay.total * 4, q.stream>>>(a);
  else
    fwd_kernel<false, 256><<<(int)grid, 256, (size_t)a.lay.total * 4, q.stream>>>(a);
  return rs_status_after_launch();
}

int il_generic_bwd(const BwdReq& q) {
  using namespace gen;
  if (q.bf16 || q.xt_x || q.F > FMAXG || q.U % q.H != 0 || q.E <= 0 || (q.L > 1 && q.E != q.U))
    return RS_ERR_UNSUPPORTED;
  int qt = pick_qt(q.F, q.E, q.U, q.H, true);
  const bool gs = qt == 0;
  if (gs) qt = q.F < 64 ? q.F : 64;
  const int nparam = q.E * 4 * q.U + 4 * q.U + 2 * q.U;
  const int64_t gmax = gs ? kGsGrid : kMaxBwdGrid;
  int64_t grid = q.B < gmax ? q.B : gmax;
  const int64_t max_grid = q.workspace_floats / nparam;
  if (grid > max_grid) grid = max_grid;
  if (q.grid_out) { *q.grid_out = (int)(grid > 0 ? grid : 0); return RS_OK; }
  if (q.B == 0) return RS_OK;
  if (grid <= 0) return RS_ERR_ARG;
  GArgs a = make_args(q.B, q.F, q.E, q.U, q.H, q.L, q.use_res, q.eps, q.drop_rate, q.seed);
  a.x = q.x; a.xsave_in = q.xsave; a.dy = q.dy; a.dy_ld = q.dy_ld;
  a.W = q.W; a.bias = q.bias; a.gamma = q.gamma; a.beta = q.beta;
  a.dx = q.dx; a.dx_accumulate = q.dx_accumulate; a.part = q.workspace;
  a.push_rows = q.push_rows; a.push_table = q.push_table; a.push_flag = q.push_flag;
  a.lay = make_layout(q.F, q.E, q.U, q.H, qt, true);
  if (gs) {
    a.gscratch = gs_scratch((size_t)grid * a.lay.total, q.stream);
    if (!a.gscratch) return RS_ERR_UNSUPPORTED;
    bwd_kernel<true, 256><<<(int)grid, 256, 0, q.stream>>>(a);
  } else {
    if ((size_t)a.lay.total * 4 > kBigLds)
      bwd_kernel<false, 512><<<(int)grid, 512, (size_t)a.lay.total * 4, q.stream>>>(a);
    else
      bwd_kernel<false, 256><<<(int)grid, 256, (size_t)a.lay.total * 4, q.stream>>>(a);
  }
  int st = rs_status_after_launch();
  if (st || !q.dparams) return st;
  reduce_params(q.stream, q.workspace, (int)grid, nparam, q.dparams, q.dparams_accumulate);
  return rs_status_after_launch();
}

}  // namespace rs_il
