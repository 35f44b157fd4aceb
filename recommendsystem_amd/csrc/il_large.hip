// H3/H5 — InteractingLayer for many fields (F in (64, 256]): the rank/multi_head ranker runs
// IL(layer_num 1, unit_num 8, head_num 2, dropout 0.2, res) over 200 fields
// (rank/multi_head/multidnn.py:54).  Same math as il_kernels.hpp
// (InteractingLayer.py:37-61, tied weights, keras-layer-normalization LN, the counter-based
// dropout mask of common.hpp), different MI355X mapping:
//
//   * one 256-thread workgroup per sample (grid-stride): at F = 200 the sample's x, Q, K, V, R
//     and attention output are 38 KB of LDS (4 blocks / CU in forward);
//   * projections: thread = (column of [Wq|Wk|Wv|Wr], row group), the column's E weights in
//     VGPRs, x rows as broadcast float4 LDS reads;
//   * attention: thread = query row covering every head (a K/V row is read once per key for all
//     heads, as broadcast float4 LDS reads); the F x F scores are never stored: a max pass and an
//     exp pass (one v_exp_f32 per score, base-2 domain);
//   * the forward can save O, the softmax row stats and the dropout keep bits per sample
//     (rs_il_fwd_saved, 21 KB at F = 200); the backward then skips the attention recompute and
//     the mask hashing (without a save it recomputes them into LDS), and makes two passes over
//     the score matrix: pass A with thread = query row (dQ), pass B with thread = key row (dK,
//     dV), each row's gradient in VGPRs -- no F x F buffer, no atomics;
//   * weight gradients in registers across the block's samples, one partial row per block,
//     column_reduce over blocks (deterministic).
#include "il_kernels.hpp"

namespace rs_il {
namespace large {

constexpr int NT = 256;
#ifndef RS_ILL_SKIP
#define RS_ILL_SKIP 0  // profiling variants only: bit 1 passes A/B, 2 projection bwd, 4 epilogue
#endif
constexpr int FMAXL = 256;

template <int E_, int U_, int H_>
struct LC {
  static constexpr int E = E_, U = U_, H = H_, NC = 4 * U, DH = U / H;
  static constexpr int NPARAM = E * NC + NC + 2 * U;
  static constexpr int NRG = NT / NC;   // projection row groups
  static constexpr int WK = (E * NC + NT - 1) / NT;  // dW entries per thread
  static_assert(DH % 4 == 0 && E % 4 == 0 && U % 4 == 0, "16-byte rows");
  static_assert(NC <= NT && NT % NC == 0, "projection mapping");
  static_assert(NT % E == 0, "dx mapping");
};

struct LFwd {
  const float *x, *W, *bias, *gamma, *beta;
  int64_t B;
  int F, L, use_res, drop;
  float eps, drop_rate, inv_keep, sc2, inv_sdh;
  uint64_t seed;
  uint64_t seed_off;  // rs_set_seed_offset source address (0 = none)
  float *y, *xsave;
  int64_t y_ld;
  float* asave;  // attention save (rs_il_fwd_saved) or null
};

struct LBwd {
  const float *x, *xsave, *dy, *W, *bias, *gamma, *beta;
  int64_t dy_ld, B;
  int F, L, use_res, drop;
  float eps, drop_rate, inv_keep, sc2, inv_sdh;
  uint64_t seed;
  uint64_t seed_off;
  float* dx;
  int dx_accumulate;
  float* part;
  const float* asave;  // forward's attention save (rs_il_bwd_saved) or null: no recompute
};

// Attention save of one (iteration, sample): O [F][U] (attention output before the epilogue) |
// row stats [F][H] x {scaled max, 1 / sum} | dropout keep bits [F][ceil(F/32)][H] (uint32: query
// row, key word, head -- both heads' words adjacent for one 8-byte LDS read).
// Written by the forward, it lets the backward skip the max pass, the O pass and the per-pair
// mask hashing.  The stride is padded to 4 floats so every sample's save starts 16-B aligned
// (float4 accesses of O).
__host__ __device__ inline int64_t save_stride(int F, int U, int H) {
  const int64_t n = (int64_t)F * U + 2 * (int64_t)H * F + (int64_t)H * F * ((F + 31) / 32);
  return (n + 3) & ~(int64_t)3;
}

template <int N>
__device__ __forceinline__ void ld(float (&v)[N], const float* p) {
#pragma unroll
  for (int k = 0; k < N / 4; ++k) {
    const float4 t = reinterpret_cast<const float4*>(p)[k];
    v[4 * k] = t.x; v[4 * k + 1] = t.y; v[4 * k + 2] = t.z; v[4 * k + 3] = t.w;
  }
}
template <int N>
__device__ __forceinline__ void st(float* p, const float (&v)[N]) {
#pragma unroll
  for (int k = 0; k < N / 4; ++k)
    reinterpret_cast<float4*>(p)[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
}
// dot product of head h's DH-slice of two U-rows, packed (v_pk_fma_f32: even / odd partial
// sums, added at the end)
template <class C>
__device__ __forceinline__ float hdot(const float (&a)[C::U], const float (&b)[C::U], int h) {
  f32x2v acc = {0.f, 0.f};
#pragma unroll
  for (int d = 0; d < C::DH; d += 2)
    acc = __builtin_elementwise_fma(f32x2v{a[h * C::DH + d], a[h * C::DH + d + 1]},
                                    f32x2v{b[h * C::DH + d], b[h * C::DH + d + 1]}, acc);
  return acc.x + acc.y;
}
// init + dot product of head h's DH-slice (the score's -max folded into the accumulator)
template <class C>
__device__ __forceinline__ float hdot_from(const float (&a)[C::U], const float (&b)[C::U], int h,
                                           float init) {
  f32x2v acc = {init, 0.f};
#pragma unroll
  for (int d = 0; d < C::DH; d += 2)
    acc = __builtin_elementwise_fma(f32x2v{a[h * C::DH + d], a[h * C::DH + d + 1]},
                                    f32x2v{b[h * C::DH + d], b[h * C::DH + d + 1]}, acc);
  return acc.x + acc.y;
}
// v if bit `bit` of the keep word m is set, else +0 (v_bfe_i32 -> all-ones / zero mask, one AND)
__device__ __forceinline__ float keep_bit(float v, uint32_t m, uint32_t bit) {
  const uint32_t msk = (uint32_t)__builtin_amdgcn_sbfe((int)m, bit, 1u);
  return __uint_as_float(__float_as_uint(v) & msk);
}
// o[h-slice] += p * x[h-slice], packed
template <class C>
__device__ __forceinline__ void haxpy(float (&o)[C::U], float p, const float (&x)[C::U], int h) {
  const f32x2v pp = {p, p};
#pragma unroll
  for (int d = 0; d < C::DH; d += 2) {
    const f32x2v r = __builtin_elementwise_fma(pp, f32x2v{x[h * C::DH + d], x[h * C::DH + d + 1]},
                                               f32x2v{o[h * C::DH + d], o[h * C::DH + d + 1]});
    o[h * C::DH + d] = r.x;
    o[h * C::DH + d + 1] = r.y;
  }
}

// projection: P_c[f] = relu(x_f . W[:, c] + b_c) into the Q|K|V|R region of column c
template <class C>
__device__ __forceinline__ void project(const float* xs, float* Qs, int F, const float (&wcol)[C::E],
                                        float bc) {
  const int t = threadIdx.x, c = t % C::NC, rg = t / C::NC;
  float* dst = Qs + (c / C::U) * F * C::U + (c % C::U);
  for (int f = rg; f < F; f += C::NRG) {
    float xr[C::E];
    ld<C::E>(xr, xs + f * C::E);
    float acc = bc;
#pragma unroll
    for (int e = 0; e < C::E; ++e) acc = fmaf(xr[e], wcol[e], acc);
    dst[f * C::U] = fmaxf(acc, 0.f);
  }
}

// Attention forward, one thread per query row i covering every head (K/V rows are read once per
// key for all heads, as broadcast float4 LDS reads): a max pass, then an exp pass accumulating O
// and the keep bits word by word.  O -> Os (LDS); optionally stats -> st4[i*H+h].xy (LDS),
// keep bits -> mask (LDS), and O / stats / bits -> sv (the global attention save).
template <class C>
__device__ __forceinline__ void attn_rows(const float* Qs, const float* Ks, const float* Vs,
                                          float* Os, int F, float sc2, bool drop, uint32_t kb,
                                          float drop_rate, float inv_keep, float4* st4,
                                          uint32_t* mask, float* sv) {
  const int W32 = (F + 31) / 32;
  const uint32_t thr16 = dropout_thr16(drop_rate);
  for (int i = threadIdx.x; i < F; i += NT) {
    float q[C::U];
    ld<C::U>(q, Qs + i * C::U);
#pragma unroll
    for (int u = 0; u < C::U; ++u) q[u] *= sc2;  // scores straight into the exp2 domain
    float mx[C::H];
#pragma unroll
    for (int h = 0; h < C::H; ++h) mx[h] = -INFINITY;
#pragma unroll 4
    for (int j = 0; j < F; ++j) {
      float k[C::U];
      ld<C::U>(k, Ks + j * C::U);
#pragma unroll
      for (int h = 0; h < C::H; ++h) mx[h] = fmaxf(mx[h], hdot<C>(q, k, h));
    }
    float msc[C::H], l[C::H], o[C::U];
    uint32_t kbh[C::H];  // the dropout counter's (head, row) part: per key pair one xor (j < 4096)
#pragma unroll
    for (int h = 0; h < C::H; ++h) {
      msc[h] = mx[h];
      l[h] = 0.f;
      kbh[h] = kb ^ (((uint32_t)h << 24) | ((uint32_t)i << 12));
    }
#pragma unroll
    for (int u = 0; u < C::U; ++u) o[u] = 0.f;
    for (int w = 0; w < W32; ++w) {
      const int jn = F - 32 * w < 32 ? F - 32 * w : 32;
      uint32_t bits[C::H], draw[C::H];
#pragma unroll
      for (int h = 0; h < C::H; ++h) { bits[h] = 0u; draw[h] = 0u; }
#pragma unroll 2
      for (int jj = 0; jj < jn; ++jj) {
        const int j = 32 * w + jj;
        float k[C::U], v[C::U];
        ld<C::U>(k, Ks + j * C::U);
        ld<C::U>(v, Vs + j * C::U);
        // one draw per key pair (words start at even keys: jj even <=> j even)
        if (drop && (jj & 1) == 0) {
#pragma unroll
          for (int h = 0; h < C::H; ++h) draw[h] = fmix32(kbh[h] ^ (uint32_t)j);
        }
#pragma unroll
        for (int h = 0; h < C::H; ++h) {
          const float e = __builtin_amdgcn_exp2f(hdot_from<C>(q, k, h, -msc[h]));
          l[h] += e;
          const bool keep = !drop || dropout_half(draw[h], (uint32_t)j) >= thr16;
          bits[h] |= (uint32_t)keep << jj;
          const float ek = keep ? e : 0.f;
          haxpy<C>(o, ek, v, h);
        }
      }
      if (drop) {
#pragma unroll
        for (int h = 0; h < C::H; ++h) {
          if (mask) mask[(i * W32 + w) * C::H + h] = bits[h];
          if (sv) reinterpret_cast<uint32_t*>(sv + F * C::U + 2 * C::H * F)[(i * W32 + w) * C::H + h] = bits[h];
        }
      }
    }
#pragma unroll
    for (int h = 0; h < C::H; ++h) {
      const float il = 1.0f / l[h];
      const float inv = (drop ? inv_keep : 1.f) * il;
#pragma unroll
      for (int d = 0; d < C::DH; ++d) o[h * C::DH + d] *= inv;
      if (st4) { st4[i * C::H + h].x = msc[h]; st4[i * C::H + h].y = il; }
      if (sv) {
        sv[F * C::U + 2 * (i * C::H + h)] = msc[h];
        sv[F * C::U + 2 * (i * C::H + h) + 1] = il;
      }
    }
    st<C::U>(Os + i * C::U, o);
    if (sv) st<C::U>(sv + i * C::U, o);
  }
}

template <class C>
__global__ void __launch_bounds__(NT) fwd_kernel(LFwd a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int F = a.F;
  float* xs = sm;                          // [F][E]
  float* Qs = xs + F * C::E;               // [F][U] x {Q, K, V, R}
  float* Ks = Qs + F * C::U;
  float* Vs = Ks + F * C::U;
  float* Rs = Vs + F * C::U;
  float* Os = Rs + F * C::U;               // [F][U]
  const int t = threadIdx.x;
  float wcol[C::E];
  {
    const int c = t % C::NC;
#pragma unroll
    for (int e = 0; e < C::E; ++e) wcol[e] = a.W[e * C::NC + c];
  }
  const float bc = a.bias[t % C::NC];
  float gam[C::U], bet[C::U];
#pragma unroll
  for (int u = 0; u < C::U; ++u) { gam[u] = a.gamma[u]; bet[u] = a.beta[u]; }
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    const float4* xg = reinterpret_cast<const float4*>(a.x + b * F * C::E);
    for (int k = t; k < F * C::E / 4; k += NT) reinterpret_cast<float4*>(xs)[k] = xg[k];
    __syncthreads();
    for (int it = 0; it < a.L; ++it) {
      const uint32_t kb = a.drop ? dropout_sample_key(splitmix64(rs_eff_seed(a.seed, a.seed_off) + (uint64_t)it), (uint32_t)b) : 0u;
      project<C>(xs, Qs, F, wcol, bc);
      __syncthreads();
      float* sv = a.asave ? a.asave + ((int64_t)it * a.B + b) * save_stride(F, C::U, C::H) : nullptr;
      attn_rows<C>(Qs, Ks, Vs, Os, F, a.sc2, a.drop, kb, a.drop_rate, a.inv_keep, nullptr, nullptr, sv);
      __syncthreads();
      const bool last = it == a.L - 1;
      for (int i = t; i < F; i += NT) {
        float z[C::U], r[C::U];
        ld<C::U>(z, Os + i * C::U);
        ld<C::U>(r, Rs + i * C::U);
        float mean = 0.f;
#pragma unroll
        for (int u = 0; u < C::U; ++u) {
          z[u] = fmaxf(a.use_res ? z[u] + r[u] : z[u], 0.f);
          mean += z[u];
        }
        mean *= 1.0f / C::U;
        float var = 0.f;
#pragma unroll
        for (int u = 0; u < C::U; ++u) var = fmaf(z[u] - mean, z[u] - mean, var);
        var *= 1.0f / C::U;
        const float rstd = 1.0f / sqrtf(var + a.eps);
#pragma unroll
        for (int u = 0; u < C::U; ++u) z[u] = fmaf((z[u] - mean) * rstd, gam[u], bet[u]);
        if (last) {
          st<C::U>(a.y + b * a.y_ld + i * C::U, z);
        } else {  // E == U (tied weights): the output is the next iteration's input
          st<C::U>(xs + i * C::E, z);
          st<C::U>(a.xsave + ((int64_t)it * a.B + b) * F * C::U + i * C::U, z);
        }
      }
      __syncthreads();
    }
  }
}

template <class C>
__global__ void __launch_bounds__(NT) bwd_kernel(LBwd a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int F = a.F;
  const int W32 = (F + 31) / 32;
  float* xs = sm;                          // [F][E]
  float* Qs = xs + F * C::E;               // Q | K | V | R (R becomes dR)
  float* Ks = Qs + F * C::U;
  float* Vs = Ks + F * C::U;
  float* Rs = Vs + F * C::U;
  float* Os = Rs + F * C::U;               // O, then dQ
  float* Gs = Os + F * C::U;               // dY -> dA (= dO) -> dx of this iteration
  float* DKs = Gs + F * C::U;
  float* DVs = DKs + F * C::U;
  float4* st4 = reinterpret_cast<float4*>(DVs + F * C::U);   // [F][H] {scaled max, 1/sum, D, -}
  uint32_t* mask = reinterpret_cast<uint32_t*>(st4 + F * C::H);  // [F][W32][H]
  const int t = threadIdx.x;
  float wcol[C::E];
  {
    const int c = t % C::NC;
#pragma unroll
    for (int e = 0; e < C::E; ++e) wcol[e] = a.W[e * C::NC + c];
  }
  const float bc = a.bias[t % C::NC];
  float gam[C::U];
#pragma unroll
  for (int u = 0; u < C::U; ++u) gam[u] = a.gamma[u];
  // dx mapping: thread -> (row group, e); the row of W for e in registers
  const int xe = t % C::E, xrg = t / C::E;
  constexpr int XRG = NT / C::E;
  float wrow[C::NC];
#pragma unroll
  for (int c = 0; c < C::NC; ++c) wrow[c] = a.W[xe * C::NC + c];
  float dw[C::WK];
#pragma unroll
  for (int k = 0; k < C::WK; ++k) dw[k] = 0.f;
  float dbc = 0.f, dg[C::U], dbt[C::U];
#pragma unroll
  for (int u = 0; u < C::U; ++u) { dg[u] = 0.f; dbt[u] = 0.f; }

  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    for (int it = a.L - 1; it >= 0; --it) {
      const float* xin = it == 0 ? a.x + b * F * C::E : a.xsave + ((int64_t)(it - 1) * a.B + b) * F * C::U;
      for (int k = t; k < F * C::E / 4; k += NT)
        reinterpret_cast<float4*>(xs)[k] = reinterpret_cast<const float4*>(xin)[k];
      if (it == a.L - 1) {
        for (int k = t; k < F * C::U / 4; k += NT) {
          const int i = k / (C::U / 4), q4 = k % (C::U / 4);
          reinterpret_cast<float4*>(Gs)[k] =
              reinterpret_cast<const float4*>(a.dy + b * a.dy_ld + i * C::U)[q4];
        }
      }
      if (a.asave) {
        // the forward's O, row stats and keep bits into their LDS regions
        const float* sv = a.asave + ((int64_t)it * a.B + b) * save_stride(F, C::U, C::H);
        for (int k = t; k < F * C::U / 4; k += NT)
          reinterpret_cast<float4*>(Os)[k] = reinterpret_cast<const float4*>(sv)[k];
        for (int k = t; k < C::H * F; k += NT) {
          const float2 mi = reinterpret_cast<const float2*>(sv + F * C::U)[k];
          st4[k].x = mi.x;
          st4[k].y = mi.y;
        }
        if (a.drop) {
          const uint32_t* mg = reinterpret_cast<const uint32_t*>(sv + F * C::U + 2 * C::H * F);
          for (int k = t; k < C::H * F * W32; k += NT) mask[k] = mg[k];
        }
        __syncthreads();
        project<C>(xs, Qs, F, wcol, bc);
        __syncthreads();
      } else {
        const uint64_t lseed = splitmix64(rs_eff_seed(a.seed, a.seed_off) + (uint64_t)it);
        const uint32_t kb = a.drop ? dropout_sample_key(lseed, (uint32_t)b) : 0u;
        __syncthreads();
        project<C>(xs, Qs, F, wcol, bc);
        __syncthreads();
        attn_rows<C>(Qs, Ks, Vs, Os, F, a.sc2, a.drop, kb, a.drop_rate, a.inv_keep, st4, mask, nullptr);
        __syncthreads();
      }
      // ---- epilogue backward: LN, ReLU, residual; D = dO . O per (row, head) ----
      for (int i = t; i < F && (RS_ILL_SKIP & 4) == 0; i += NT) {
        float o[C::U], r[C::U], z[C::U], g[C::U];
        ld<C::U>(o, Os + i * C::U);
        ld<C::U>(r, Rs + i * C::U);
        ld<C::U>(g, Gs + i * C::U);
        float mean = 0.f;
#pragma unroll
        for (int u = 0; u < C::U; ++u) {
          z[u] = fmaxf(a.use_res ? o[u] + r[u] : o[u], 0.f);
          mean += z[u];
        }
        mean *= 1.0f / C::U;
        float var = 0.f;
#pragma unroll
        for (int u = 0; u < C::U; ++u) var = fmaf(z[u] - mean, z[u] - mean, var);
        var *= 1.0f / C::U;
        const float rstd = 1.0f / sqrtf(var + a.eps);
        float m1 = 0.f, m2 = 0.f, xh[C::U];
#pragma unroll
        for (int u = 0; u < C::U; ++u) {
          xh[u] = (z[u] - mean) * rstd;
          dg[u] = fmaf(g[u], xh[u], dg[u]);
          dbt[u] += g[u];
          const float gd = g[u] * gam[u];
          m1 += gd;
          m2 = fmaf(gd, xh[u], m2);
        }
        m1 *= 1.0f / C::U;
        m2 *= 1.0f / C::U;
        float da[C::U], dr[C::U];
#pragma unroll
        for (int u = 0; u < C::U; ++u) {
          const float dz = rstd * (g[u] * gam[u] - m1 - xh[u] * m2);
          da[u] = z[u] > 0.f ? dz : 0.f;
          dr[u] = (a.use_res && r[u] > 0.f) ? da[u] : 0.f;
        }
        st<C::U>(Rs + i * C::U, dr);
        // passes A / B read the softmax 1/sum and the dropout scale pre-folded (they are per
        // (row, head) constants of dS_ij = P_ij (keep inv_keep dO_i . v_j - D_i) with
        // P_ij = e_ij / sum_i):  dS_ij = e_ij (keep (g'_i . v_j) - D'_i) with
        // g'_i = dO_i inv_keep / sum_i and D'_i = D_i / sum_i, and dV_j += keep e_ij g'_i -- two
        // to three multiplies fewer per score and head in the VALU-bound passes
        const float ks = a.drop ? a.inv_keep : 1.f;
#pragma unroll
        for (int h = 0; h < C::H; ++h) {
          const float inv = st4[i * C::H + h].y;
          st4[i * C::H + h].z = hdot<C>(da, o, h) * inv;
          const float gs = inv * ks;
#pragma unroll
          for (int d = 0; d < C::DH; ++d) da[h * C::DH + d] *= gs;
        }
        st<C::U>(Gs + i * C::U, da);
      }
      __syncthreads();
      // ---- passes A and B side by side: threads [0, NT/2) run pass A (dQ -> Os) over query
      // rows {r, r + NH}, threads [NT/2, NT) pass B (dK, dV) over key rows {r, r + NH}, NH =
      // ceil(F/2).  Two rows per thread halve the broadcast K/V (pass A) and Q/dO/stats (pass B)
      // LDS reads per score -- the passes are LDS-read bound -- and the two halves overlap.
      {
        const int NH = (F + 1) / 2;
        const int half = t / (NT / 2), r = t % (NT / 2);
        const int r1 = r + NH;
        const bool has1 = r1 < F;
        const int rr1 = has1 ? r1 : r;  // duplicate row 0's work when F is odd (not stored)
        if ((RS_ILL_SKIP & 1) == 0 && half == 0 && r < NH) {
          float q0[C::U], g0[C::U], q1[C::U], g1[C::U], dq0[C::U], dq1[C::U];
          ld<C::U>(q0, Qs + r * C::U);
          ld<C::U>(g0, Gs + r * C::U);
          ld<C::U>(q1, Qs + rr1 * C::U);
          ld<C::U>(g1, Gs + rr1 * C::U);
#pragma unroll
          for (int u = 0; u < C::U; ++u) {
            dq0[u] = 0.f; dq1[u] = 0.f;
            q0[u] *= a.sc2; q1[u] *= a.sc2;  // scores in the exp2 domain (signs, the dq ReLU masks, kept)
          }
          float4 s0[C::H], s1[C::H];
#pragma unroll
          for (int h = 0; h < C::H; ++h) { s0[h] = st4[r * C::H + h]; s1[h] = st4[rr1 * C::H + h]; }
          for (int w = 0; w < W32; ++w) {
            const int jn = F - 32 * w < 32 ? F - 32 * w : 32;
            uint32_t m0[C::H], m1[C::H];
#pragma unroll
            for (int h = 0; h < C::H; ++h) {
              m0[h] = a.drop ? mask[(r * W32 + w) * C::H + h] : ~0u;
              m1[h] = a.drop ? mask[(rr1 * W32 + w) * C::H + h] : ~0u;
            }
#pragma unroll 1
            for (int jj = 0; jj < jn; ++jj) {
              const int j = 32 * w + jj;
              float k[C::U], v[C::U];
              ld<C::U>(k, Ks + j * C::U);
              ld<C::U>(v, Vs + j * C::U);
#pragma unroll
              for (int h = 0; h < C::H; ++h) {
                const float pe0 = __builtin_amdgcn_exp2f(hdot_from<C>(q0, k, h, -s0[h].x));
                const float pe1 = __builtin_amdgcn_exp2f(hdot_from<C>(q1, k, h, -s1[h].x));
                float dP0 = hdot<C>(g0, v, h), dP1 = hdot<C>(g1, v, h);
                if (a.drop) {
                  dP0 = keep_bit(dP0, m0[h], (uint32_t)jj);
                  dP1 = keep_bit(dP1, m1[h], (uint32_t)jj);
                }
                haxpy<C>(dq0, pe0 * (dP0 - s0[h].z), k, h);
                haxpy<C>(dq1, pe1 * (dP1 - s1[h].z), k, h);
              }
            }
          }
#pragma unroll
          for (int u = 0; u < C::U; ++u) {
            dq0[u] = q0[u] > 0.f ? dq0[u] * a.inv_sdh : 0.f;
            dq1[u] = q1[u] > 0.f ? dq1[u] * a.inv_sdh : 0.f;
          }
          st<C::U>(Os + r * C::U, dq0);
          if (has1) st<C::U>(Os + r1 * C::U, dq1);
        } else if ((RS_ILL_SKIP & 1) == 0 && half == 1 && r < NH) {
          float k0[C::U], v0[C::U], k1[C::U], v1[C::U];
          float dk0[C::U], dv0[C::U], dk1[C::U], dv1[C::U];
          ld<C::U>(k0, Ks + r * C::U);
          ld<C::U>(v0, Vs + r * C::U);
          ld<C::U>(k1, Ks + rr1 * C::U);
          ld<C::U>(v1, Vs + rr1 * C::U);
#pragma unroll
          for (int u = 0; u < C::U; ++u) {
            dk0[u] = 0.f; dv0[u] = 0.f; dk1[u] = 0.f; dv1[u] = 0.f;
            k0[u] *= a.sc2; k1[u] *= a.sc2;  // (signs, the dk ReLU masks, kept)
          }
          const int jw0 = r >> 5, jb0 = r & 31, jw1 = rr1 >> 5, jb1 = rr1 & 31;
#pragma unroll 1
          for (int i = 0; i < F; ++i) {
            float q[C::U], g[C::U];
            ld<C::U>(q, Qs + i * C::U);
            ld<C::U>(g, Gs + i * C::U);
#pragma unroll
            for (int h = 0; h < C::H; ++h) {
              const float4 sh = st4[i * C::H + h];
              const float pe0 = __builtin_amdgcn_exp2f(hdot_from<C>(q, k0, h, -sh.x));
              const float pe1 = __builtin_amdgcn_exp2f(hdot_from<C>(q, k1, h, -sh.x));
              float dP0 = hdot<C>(g, v0, h), pd0 = pe0;
              float dP1 = hdot<C>(g, v1, h), pd1 = pe1;
              if (a.drop) {
                const uint32_t* mr = mask + i * W32 * C::H + h;  // [i][w][h]: both heads' words adjacent
                const uint32_t w0 = mr[jw0 * C::H], w1 = mr[jw1 * C::H];
                dP0 = keep_bit(dP0, w0, (uint32_t)jb0);
                pd0 = keep_bit(pe0, w0, (uint32_t)jb0);
                dP1 = keep_bit(dP1, w1, (uint32_t)jb1);
                pd1 = keep_bit(pe1, w1, (uint32_t)jb1);
              }
              haxpy<C>(dk0, pe0 * (dP0 - sh.z), q, h);
              haxpy<C>(dv0, pd0, g, h);
              haxpy<C>(dk1, pe1 * (dP1 - sh.z), q, h);
              haxpy<C>(dv1, pd1, g, h);
            }
          }
#pragma unroll
          for (int u = 0; u < C::U; ++u) {
            dk0[u] = k0[u] > 0.f ? dk0[u] * a.inv_sdh : 0.f;
            dv0[u] = v0[u] > 0.f ? dv0[u] : 0.f;
            dk1[u] = k1[u] > 0.f ? dk1[u] * a.inv_sdh : 0.f;
            dv1[u] = v1[u] > 0.f ? dv1[u] : 0.f;
          }
          st<C::U>(DKs + r * C::U, dk0);
          st<C::U>(DVs + r * C::U, dv0);
          if (has1) {
            st<C::U>(DKs + r1 * C::U, dk1);
            st<C::U>(DVs + r1 * C::U, dv1);
          }
        }
      }
      __syncthreads();
      // ---- projection backward: dZ = [dQ (Os) | dK | dV | dR (Rs)] ----
      auto dzb = [&](int c) -> const float* {
        const int g = c / C::U;
        return (g == 0 ? Os : g == 1 ? DKs : g == 2 ? DVs : Rs) + (c % C::U);
      };
#pragma unroll
      for (int k = 0; k < C::WK; ++k) {
        const int idx = t + NT * k;
        if ((RS_ILL_SKIP & 2) == 0 && idx < C::E * C::NC) {
          const int e = idx / C::NC, c = idx % C::NC;
          const float* dz = dzb(c);
          float s = 0.f;
          for (int f = 0; f < F; ++f) s = fmaf(xs[f * C::E + e], dz[f * C::U], s);
          dw[k] += s;
        }
      }
      if (t < C::NC) {
        const float* dz = dzb(t);
        float s = 0.f;
        for (int f = 0; f < F; ++f) s += dz[f * C::U];
        dbc += s;
      }
      for (int f = xrg; f < F && (RS_ILL_SKIP & 2) == 0; f += XRG) {
        float s = 0.f;
#pragma unroll
        for (int c = 0; c < C::NC; ++c) s = fmaf(dzb(c)[f * C::U], wrow[c], s);
        if (it == 0) {
          float* dst = a.dx + b * F * C::E + f * C::E + xe;
          *dst = a.dx_accumulate ? *dst + s : s;
        } else {
          Gs[f * C::U + xe] = s;  // E == U: dY of iteration it - 1
        }
      }
      __syncthreads();
    }
  }
  // ---- block partial: [dW (E*NC) | db (NC) | dgamma (U) | dbeta (U)] ----
  float* red = sm;  // [NT][2U]
#pragma unroll
  for (int u = 0; u < C::U; ++u) {
    red[t * 2 * C::U + u] = dg[u];
    red[t * 2 * C::U + C::U + u] = dbt[u];
  }
  __syncthreads();
  float* pr = a.part + (int64_t)blockIdx.x * C::NPARAM;
#pragma unroll
  for (int k = 0; k < C::WK; ++k) {
    const int idx = t + NT * k;
    if (idx < C::E * C::NC) pr[idx] = dw[k];
  }
  if (t < C::NC) pr[C::E * C::NC + t] = dbc;
  if (t < 2 * C::U) {
    float s = 0.f;
    for (int r = 0; r < NT; ++r) s += red[r * 2 * C::U + t];
    pr[C::E * C::NC + C::NC + t] = s;
  }
}

inline size_t fwd_lds(int F, int E, int U) { return (size_t)F * (E + 5 * U) * 4; }
inline size_t bwd_lds(int F, int E, int U, int H) {
  const size_t main = (size_t)F * (E + 8 * U) * 4 + (size_t)4 * H * F * 4 +
                      (size_t)H * F * ((F + 31) / 32) * 4;
  const size_t red = (size_t)NT * 2 * U * 4;
  return main > red ? main : red;
}

template <int E, int U, int H>
int run_fwd(const FwdReq& q) {
  using C = LC<E, U, H>;
  LFwd a{q.x, q.W, q.bias, q.gamma, q.beta, q.B, q.F, q.L, q.use_res, q.drop_rate > 0.f,
         q.eps, q.drop_rate, q.drop_rate > 0.f ? 1.0f / (1.0f - q.drop_rate) : 1.0f,
         1.4426950408889634f / sqrtf((float)C::DH), 1.0f / sqrtf((float)C::DH), q.seed, (uint64_t)(uintptr_t)rs_seed_offset_now(), q.y,
         q.xsave, q.y_ld, q.asave};
  if (q.B == 0) return RS_OK;
  const size_t lds = fwd_lds(q.F, E, U);
  int64_t grid = q.B < 4096 ? q.B : 4096;
  fwd_kernel<C><<<(int)grid, NT, lds, q.stream>>>(a);
  return rs_status_after_launch();
}

template <int E, int U, int H>
int run_bwd(const BwdReq& q) {
  using C = LC<E, U, H>;
  int64_t grid = q.B < kMaxBwdGrid ? q.B : kMaxBwdGrid;
  if (q.grid_out) {  // dry run (rs_il_bwd_partial_blocks)
    const int64_t by_ws = q.workspace_floats / C::NPARAM;
    *q.grid_out = (int)(grid < by_ws ? grid : by_ws);
    return RS_OK;
  }
  if (q.B == 0) return RS_OK;
  if (q.workspace_floats < grid * C::NPARAM) return RS_ERR_ARG;
  LBwd a{q.x, q.xsave, q.dy, q.W, q.bias, q.gamma, q.beta, q.dy_ld, q.B, q.F, q.L, q.use_res,
         q.drop_rate > 0.f, q.eps, q.drop_rate,
         q.drop_rate > 0.f ? 1.0f / (1.0f - q.drop_rate) : 1.0f,
         1.4426950408889634f / sqrtf((float)C::DH), 1.0f / sqrtf((float)C::DH), q.seed, (uint64_t)(uintptr_t)rs_seed_offset_now(), q.dx,
         q.dx_accumulate, q.workspace, q.asave};
  const size_t lds = bwd_lds(q.F, E, U, H);
  bwd_kernel<C><<<(int)grid, NT, lds, q.stream>>>(a);
  int st = rs_status_after_launch();
  if (st || !q.dparams) return st;
  launch_column_reduce(q.stream, q.workspace, (int)grid, C::NPARAM, C::NPARAM, C::NPARAM,
                       q.dparams, nullptr, q.dparams_accumulate);
  return rs_status_after_launch();
}

}  // namespace large

int64_t il_attn_save_floats(int64_t B, int F, int U, int H, int L) {
  if (F > 64) return (int64_t)L * B * large::save_stride(F, U, H);
  // F <= 32, two heads of 8 (il_inst_a.hip shapes): O + softmax stats for bwd4_kernel
  if (F <= 32 && U == 16 && H == 2) return (int64_t)L * B * small_save_stride(F, U, H);
  return 0;
}

// F in (64, 256]: the many-field instantiations (config 3 is E = U = 8, H = 2).
int il_large_fwd(const FwdReq& q) {
  if (q.bf16) return RS_ERR_UNSUPPORTED;  // fp32 only (bf16 mode: il_inst_a.hip shapes)
  if (q.F > large::FMAXL || (q.L > 1 && q.E != q.U)) return RS_ERR_UNSUPPORTED;
  if (large::fwd_lds(q.F, q.E, q.U) > 64 * 1024) return RS_ERR_UNSUPPORTED;
  if (q.E == 8 && q.U == 8 && q.H == 2) return large::run_fwd<8, 8, 2>(q);
  if (q.E == 8 && q.U == 8 && q.H == 1) return large::run_fwd<8, 8, 1>(q);
  if (q.E == 16 && q.U == 16 && q.H == 2) return large::run_fwd<16, 16, 2>(q);
  return RS_ERR_UNSUPPORTED;
}

int il_large_bwd(const BwdReq& q) {
  if (q.bf16) return RS_ERR_UNSUPPORTED;
  if (q.F > large::FMAXL || (q.L > 1 && q.E != q.U)) return RS_ERR_UNSUPPORTED;
  if (large::bwd_lds(q.F, q.E, q.U, q.H) > 160 * 1024) return RS_ERR_UNSUPPORTED;
  if (q.E == 8 && q.U == 8 && q.H == 2) return large::run_bwd<8, 8, 2>(q);
  if (q.E == 8 && q.U == 8 && q.H == 1) return large::run_bwd<8, 8, 1>(q);
  if (q.E == 16 && q.U == 16 && q.H == 2) return large::run_bwd<16, 16, 2>(q);
  return RS_ERR_UNSUPPORTED;
}

}  // namespace rs_il
