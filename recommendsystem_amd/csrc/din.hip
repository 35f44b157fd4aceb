// H6/H7 — DIN behaviour-sequence attention pooling, forward and backward.
//
// Two reference variants share one kernel family (template VAR):
//   VAR 0  din.py:18-47            a_t = [q, k_t, q*k_t] (3H) -> Dense(16, relu) -> Dense(1, relu)
//                                  -> masked to 0 (sequence_mask(seq_length)) -> out = sum_t s_t v_t
//                                  (no softmax)
//   VAR 1  staytime/layer.py:16-41 a_t = [q, f_t, q-f_t, q*f_t] (4H) -> Dense(16, sigmoid) ->
//                                  Dense(1) -> masked positions = -2**32+1 -> softmax over T ->
//                                  out = sum_t p_t f_t
//
// Algebra (exact up to fp32 rounding, no approximation): the first Dense factorises per sample,
//   a_t W1 + b1 = c + k_t W1',   c = q Wq + b1,   W1' = Wk + diag(q) Wqk
//   VAR 0: Wq = W1[0:H], Wk = W1[H:2H],          Wqk = W1[2H:3H]
//   VAR 1: Wq = W1[0:H] + W1[2H:3H], Wk = W1[H:2H] - W1[2H:3H], Wqk = W1[3H:4H]
// so the per-position work is one [16 x H] x [H x 16] product instead of a [3H|4H] x 16 one, and
// the tiled [B, T, 3H|4H] concat the reference materialises (78.6 MB per step at config 4) never
// exists.  The backward uses the same identity: with dZ_t = dL/d(pre-activation of layer 1),
//   G = sum_t k_t^T dZ_t (H x 16),  gsum = sum_t dZ_t
//   dWq-part = q (x) gsum,  dWk-part = G,  dWqk-part = diag(q) G,  db1 = gsum
//   dk_t = dZ_t W1'^T,      dq_i = sum_j Wq[i][j] gsum_j + sum_j Wqk[i][j] G[i][j]
//
// MI355X mapping (H = 16, hidden = 16): one wave per sample, 16 positions per step.
//   * The key rows t0..t0+15 are ONE coalesced 1 KiB float4 load: lane l reads row t0 + (l&15),
//     columns 4(l>>4)..+3, which is exactly an MFMA A fragment with a permuted reduction index;
//     W1' is the matching B fragment (4 VGPRs, rebuilt per sample from 3 fragments and q).
//     4 x v_mfma_f32_16x16x4_f32 give the 16x16 layer-1 pre-activations (exact fp32 FMAs).
//   * The MFMA result layout (lane (g = l>>4, j = l&15) holds rows 4g..4g+3, column j) is used
//     as is: layer 2 is a 16-lane DPP reduction, the value rows are read in the same layout, and
//     in the backward the dZ tile is already the B fragment of G = K^T dZ (reduction over t).
//     Only dK = dZ W1'^T needs dZ as an A fragment: a 16x16 transpose through 1.25 KiB of LDS.
//   * Masks: positions t >= T are dropped; position t of sample b is "on" iff
//     (lengths == NULL || t < lengths[b]) && (mask == NULL || mask[b * mask_ld + t] != 0).
//   * Weight gradients: per-lane register accumulators across a wave's samples -> per-block LDS
//     sum in wave order -> per-block partial rows -> column_reduce (fixed order: deterministic).
// Roofline: HBM-bound at config 4 (12.9 KB of keys+values per sample vs ~19 KFLOP after the
// factorisation); the backward re-reads the same rows (L2-resident within a wave).
#include "common.hpp"

namespace rs_din {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int HD = 16;            // embedding width (configs 4 and 5 pool 16-wide rows)
constexpr int D1 = 16;            // layer-1 width: Dense(16) in both references
constexpr int WPB = 4;            // waves per block
constexpr int TT_LD = 20;         // LDS transpose tile row stride (floats; 16B aligned)
constexpr float PAD = -4294967296.0f;  // fp32(-2**32 + 1), staytime/layer.py:32

__host__ __device__ constexpr int nblk(int var) { return var == 0 ? 3 : 4; }
__host__ __device__ constexpr int nparam(int var) { return nblk(var) * HD * D1 + D1 + D1 + 1; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + __expf(-v)); }

struct Geo {
  const float* q; int64_t q_ld;
  const float* k; int64_t k_ss, k_rs;
  const float* v; int64_t v_ss, v_rs;
  int64_t B; int T;
  const int32_t* lengths;
  const uint8_t* mask; int64_t mask_ld;
};

__device__ __forceinline__ bool pos_on(const Geo& g, int64_t b, int t, int len) {
  if (t >= len) return false;
  if (g.mask && g.mask[b * g.mask_ld + t] == 0) return false;
  return true;
}

// Per-lane weight fragments (lane (g, j), rows i = 4g + r):
//   rq/rk/rqk[r] = Wq/Wk/Wqk[4g + r][j]        (B fragment of W1', dq epilogue)
//   tk/tqk[r]    = Wk/Wqk[j][4g + r]           (B fragment of W1'^T, for dK)
template <int VAR>
struct Frags {
  float rq[4], rk[4], rqk[4], tk[4], tqk[4];
  float b1, w2, b2;
  __device__ __forceinline__ void load(const float* __restrict__ W1, const float* __restrict__ b1p,
                                       const float* __restrict__ W2, const float* __restrict__ b2p) {
    const int l = lane_id(), g = l >> 4, j = l & 15;
    auto w = [&](int blk, int i, int c) { return W1[(blk * HD + i) * D1 + c]; };
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * g + r;
      if (VAR == 0) {
        rq[r] = w(0, i, j); rk[r] = w(1, i, j); rqk[r] = w(2, i, j);
        tk[r] = w(1, j, i); tqk[r] = w(2, j, i);
      } else {
        rq[r] = w(0, i, j) + w(2, i, j); rk[r] = w(1, i, j) - w(2, i, j); rqk[r] = w(3, i, j);
        tk[r] = w(1, j, i) - w(2, j, i); tqk[r] = w(3, j, i);
      }
    }
    b1 = b1p[j]; w2 = W2[j]; b2 = b2p[0];
  }
};

// Per-sample setup: q fragment, c_j and the W1' B fragment.
template <int VAR>
struct SampleW {
  float qv[4], bw[4], c;
  __device__ __forceinline__ void build(const Frags<VAR>& fr, const float* __restrict__ qrow) {
    const int l = lane_id(), g = l >> 4;
    const float4 q4 = *reinterpret_cast<const float4*>(qrow + 4 * g);
    qv[0] = q4.x; qv[1] = q4.y; qv[2] = q4.z; qv[3] = q4.w;
    float p = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      p = fmaf(qv[r], fr.rq[r], p);
      bw[r] = fmaf(qv[r], fr.rqk[r], fr.rk[r]);
    }
    p += __shfl_xor(p, 16, 64);
    p += __shfl_xor(p, 32, 64);
    c = p + fr.b1;
  }
};

// The key rows t0 .. t0 + 15 as this lane's A fragment (row t0 + (l & 15), columns 4 (l >> 4)..).
// The sweeps load step t0 + 16's keys / values while step t0 computes (one step ahead), so a
// wave's per-step HBM round trip overlaps its MFMA / DPP work instead of serialising with it.
__device__ __forceinline__ float4 load_keys(const float* __restrict__ krow0, int64_t k_rs, int t0,
                                            int T) {
  const int l = lane_id();
  const int row = t0 + (l & 15);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (row < T) a = *reinterpret_cast<const float4*>(krow0 + (int64_t)row * k_rs + 4 * (l >> 4));
  return a;
}
// values (or any [T, >= 16] row set) of rows t0 + 4g + r, column j, r < 4
struct Vals { float v[4]; };
__device__ __forceinline__ Vals load_vals(const float* __restrict__ vrow0, int64_t v_rs, int t0,
                                          int T) {
  const int l = lane_id(), g = l >> 4, j = l & 15;
  Vals out;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int t = t0 + 4 * g + r;
    out.v[r] = t < T ? vrow0[(int64_t)t * v_rs + j] : 0.f;
  }
  return out;
}
// Layer-1 pre-activations of rows t0 + 4g + r (column j) minus nothing: z1[r] = acc[r] + c.
__device__ __forceinline__ f32x4 layer1_frag(float4 a, const float bw[4]) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = mfma4(a.x, bw[0], acc);
  acc = mfma4(a.y, bw[1], acc);
  acc = mfma4(a.z, bw[2], acc);
  acc = mfma4(a.w, bw[3], acc);
  return acc;
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
template <int VAR>
__global__ void __launch_bounds__(64 * WPB) din_fwd_kernel(Geo geo, const float* __restrict__ W1,
                                                           const float* __restrict__ b1,
                                                           const float* __restrict__ W2,
                                                           const float* __restrict__ b2,
                                                           float* __restrict__ out, int64_t out_ld,
                                                           float* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int l = lane_id(), g = l >> 4, j = l & 15;
  const int T = geo.T;
  float* sbuf = smem + wave_id() * T;  // VAR 1: scores, then exp(scores - max)
  Frags<VAR> fr;
  fr.load(W1, b1, W2, b2);
  for (int64_t b = (int64_t)blockIdx.x * WPB + wave_id(); b < geo.B; b += (int64_t)gridDim.x * WPB) {
    SampleW<VAR> sw;
    sw.build(fr, geo.q + b * geo.q_ld);
    const float* krow0 = geo.k + b * geo.k_ss;
    const float* vrow0 = geo.v + b * geo.v_ss;
    const int len = geo.lengths ? min(geo.lengths[b], T) : T;
    float o = 0.f, mx = -INFINITY;
    float4 an = load_keys(krow0, geo.k_rs, 0, T);
    Vals vn{};
    if (VAR == 0) vn = load_vals(vrow0, geo.v_rs, 0, T);
    for (int t0 = 0; t0 < T; t0 += 16) {
      const float4 a = an;
      const Vals vc = vn;
      if (t0 + 16 < T) {
        an = load_keys(krow0, geo.k_rs, t0 + 16, T);
        if (VAR == 0) vn = load_vals(vrow0, geo.v_rs, t0 + 16, T);
      }
      const f32x4 acc = layer1_frag(a, sw.bw);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z1 = acc[r] + sw.c;
        const float h = VAR == 0 ? fmaxf(z1, 0.f) : sigm(z1);
        const float z2 = group_sum<16>(h * fr.w2) + fr.b2;
        const int t = t0 + 4 * g + r;
        if (t < T) {
          const bool on = pos_on(geo, b, t, len);
          if (VAR == 0) {
            const float s = on ? fmaxf(z2, 0.f) : 0.f;
            o = fmaf(s, vc.v[r], o);
          } else {
            const float sc = on ? z2 : PAD;
            mx = fmaxf(mx, sc);
            if (j == 0) sbuf[t] = sc;
          }
        }
      }
    }
    if (VAR == 1) {
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      wave_lds_sync();
      float lsum = 0.f;
      Vals fn = load_vals(vrow0, geo.v_rs, 0, T);
      for (int t0 = 0; t0 < T; t0 += 16) {
        const Vals fc = fn;
        if (t0 + 16 < T) fn = load_vals(vrow0, geo.v_rs, t0 + 16, T);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = t0 + 4 * g + r;
          if (t < T) {
            const float e = __expf(sbuf[t] - mx);
            lsum += e;
            o = fmaf(e, fc.v[r], o);
          }
        }
      }
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
      const float inv = 1.0f / lsum;
      o *= inv;
      if (probs) {
        for (int t = l; t < T; t += 64) probs[b * T + t] = __expf(sbuf[t] - mx) * inv;
      }
      wave_lds_sync();
    }
    o += __shfl_xor(o, 16, 64);
    o += __shfl_xor(o, 32, 64);
    if (g == 0) out[b * out_ld + j] = o;
  }
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
template <int VAR>
__global__ void __launch_bounds__(64 * WPB) din_bwd_kernel(
    Geo geo, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ probs,
    const float* __restrict__ dout, int64_t dout_ld, float* __restrict__ dq, int64_t dq_ld,
    float* __restrict__ dk, float* __restrict__ dv, float* __restrict__ part, int64_t dkv_rs,
    int dkv_pad, const float* __restrict__ dq_base, int64_t dqb_ld) {
  constexpr int NP = nparam(VAR);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int l = lane_id(), g = l >> 4, j = l & 15, w = wave_id();
  const int T = geo.T;
  float* tt = smem + w * (16 * TT_LD);                 // [16][TT_LD] transpose tile
  float* sbuf = smem + WPB * 16 * TT_LD + w * T;       // VAR 1: dp_t
  float* red = smem;                                   // [WPB][NP], aliases the above at the end
  const bool alias_kv = geo.k == geo.v;
  const bool alias_d = dk != nullptr && dk == dv;
  Frags<VAR> fr;
  fr.load(W1, b1, W2, b2);
  float accA[4] = {0.f, 0.f, 0.f, 0.f}, accG[4] = {0.f, 0.f, 0.f, 0.f};
  float accQG[4] = {0.f, 0.f, 0.f, 0.f};
  float accb1 = 0.f, accw2 = 0.f, accb2 = 0.f;
  for (int64_t b = (int64_t)blockIdx.x * WPB + w; b < geo.B; b += (int64_t)gridDim.x * WPB) {
    SampleW<VAR> sw;
    const float* qrow = geo.q + b * geo.q_ld;
    sw.build(fr, qrow);
    const float qi = qrow[j];
    float tb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tb[r] = fmaf(qi, fr.tqk[r], fr.tk[r]);  // W1'[j][4g + r]
    const float* krow0 = geo.k + b * geo.k_ss;
    const float* vrow0 = geo.v + b * geo.v_ss;
    const int len = geo.lengths ? min(geo.lengths[b], T) : T;
    const float doj = dout[b * dout_ld + j];
    const float* prow = VAR == 1 ? probs + b * T : nullptr;
    float sdp = 0.f;
    if (VAR == 1) {  // pass 1: dp_t = dout . f_t, sum_t p_t dp_t
      Vals fn = load_vals(vrow0, geo.v_rs, 0, T);
      for (int t0 = 0; t0 < T; t0 += 16) {
        const Vals fc = fn;
        if (t0 + 16 < T) fn = load_vals(vrow0, geo.v_rs, t0 + 16, T);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = t0 + 4 * g + r;
          const float fv = fc.v[r];
          const float dp = group_sum<16>(doj * fv);
          if (t < T) {
            sdp = fmaf(prow[t], dp, sdp);
            if (j == 0) sbuf[t] = dp;
          }
        }
      }
      sdp += __shfl_xor(sdp, 16, 64);
      sdp += __shfl_xor(sdp, 32, 64);
      wave_lds_sync();
    }
    f32x4 G = {0.f, 0.f, 0.f, 0.f};
    float gs = 0.f;
    float4 an = load_keys(krow0, geo.k_rs, 0, T);
    Vals vn = load_vals(vrow0, geo.v_rs, 0, T);
    for (int t0 = 0; t0 < T; t0 += 16) {
      const float4 a = an;
      const Vals vc = vn;
      if (t0 + 16 < T) {
        an = load_keys(krow0, geo.k_rs, t0 + 16, T);
        vn = load_vals(vrow0, geo.v_rs, t0 + 16, T);
      }
      const f32x4 acc = layer1_frag(a, sw.bw);
      float dz1[4], kv[4], dvv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + 4 * g + r;
        const bool in = t < T;
        const float z1 = acc[r] + sw.c;
        const float h = VAR == 0 ? fmaxf(z1, 0.f) : sigm(z1);
        const bool on = in && pos_on(geo, b, t, len);
        float dz2, vval;
        if (VAR == 0) {
          const float z2 = group_sum<16>(h * fr.w2) + fr.b2;
          vval = vc.v[r];
          const float ds = group_sum<16>(doj * vval);
          const float s = on ? fmaxf(z2, 0.f) : 0.f;
          dz2 = (on && z2 > 0.f) ? ds : 0.f;
          dvv[r] = s * doj;                                   // d values
          kv[r] = alias_kv ? vval : (in ? krow0[(int64_t)t * geo.k_rs + j] : 0.f);
          dz1[r] = h > 0.f ? dz2 * fr.w2 : 0.f;
        } else {
          const float p = in ? prow[t] : 0.f;
          dz2 = on ? p * (sbuf[in ? t : 0] - sdp) : 0.f;
          vval = vc.v[r];
          dvv[r] = p * doj;                                   // d facts through the pooling
          kv[r] = vval;
          dz1[r] = dz2 * fr.w2 * h * (1.0f - h);
        }
        accw2 = fmaf(h, dz2, accw2);
        if (j == 0) accb2 += dz2;
        gs += dz1[r];
      }
      // G += K^T dZ (reduction over the 16 positions of this step)
#pragma unroll
      for (int r = 0; r < 4; ++r) G = mfma4(kv[r], dz1[r], G);
      // dK = dZ W1'^T: transpose dZ into an A fragment through LDS
#pragma unroll
      for (int r = 0; r < 4; ++r) tt[(4 * g + r) * TT_LD + j] = dz1[r];
      wave_lds_sync();
      const float4 az = *reinterpret_cast<const float4*>(tt + (l & 15) * TT_LD + 4 * g);
      wave_lds_sync();
      f32x4 DK = {0.f, 0.f, 0.f, 0.f};
      DK = mfma4(az.x, tb[0], DK);
      DK = mfma4(az.y, tb[1], DK);
      DK = mfma4(az.z, tb[2], DK);
      DK = mfma4(az.w, tb[3], DK);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int t = t0 + 4 * g + r;
        if (t < T) {
          float* base = (float*)nullptr;
          // row stride dkv_rs >= HD; columns HD .. dkv_pad - 1 of each row are written as zeros
          // (the gradient of a wider facts row whose first HD columns the pooling reads)
          const int64_t off = (b * T + t) * dkv_rs + j;
          const bool zpad = j + HD < dkv_pad;
          if (VAR == 1 || alias_d) {
            // VAR 1: keys and values are the same facts tensor -> one gradient
            base = dk ? dk : dv;
            if (base) {
              base[off] = DK[r] + dvv[r];
              if (zpad) base[off + HD] = 0.f;
            }
          } else {
            if (dk) { dk[off] = DK[r]; if (zpad) dk[off + HD] = 0.f; }
            if (dv) { dv[off] = dvv[r]; if (zpad) dv[off + HD] = 0.f; }
          }
        }
      }
    }
    gs += __shfl_xor(gs, 16, 64);
    gs += __shfl_xor(gs, 32, 64);  // gsum_j, in every lane of column j
    float dqv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dqv[r] = group_sum<16>(fmaf(fr.rq[r], gs, fr.rqk[r] * G[r]));
      accA[r] = fmaf(sw.qv[r], gs, accA[r]);
      accG[r] += G[r];
      accQG[r] = fmaf(sw.qv[r], G[r], accQG[r]);
    }
    if (g == 0) accb1 += gs;
    if (j == 0) {
      if (dq_base) {  // dq = the query's other gradient + this one (no separate sum launch)
#pragma unroll
        for (int r = 0; r < 4; ++r) dqv[r] += dq_base[b * dqb_ld + 4 * g + r];
      }
      *reinterpret_cast<float4*>(dq + b * dq_ld + 4 * g) = make_float4(dqv[0], dqv[1], dqv[2], dqv[3]);
    }
  }
  // ---- weight-gradient partials: wave -> block (LDS, wave order) -> part[blockIdx] ----
  accw2 += __shfl_xor(accw2, 16, 64);
  accw2 += __shfl_xor(accw2, 32, 64);
  accb2 += __shfl_xor(accb2, 16, 64);
  accb2 += __shfl_xor(accb2, 32, 64);
  __syncthreads();
  float* mine = red + w * NP;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * g + r;
    mine[(0 * HD + i) * D1 + j] = accA[r];
    mine[(1 * HD + i) * D1 + j] = accG[r];
    if (VAR == 0) {
      mine[(2 * HD + i) * D1 + j] = accQG[r];
    } else {
      mine[(2 * HD + i) * D1 + j] = accA[r] - accG[r];
      mine[(3 * HD + i) * D1 + j] = accQG[r];
    }
  }
  constexpr int OB = nblk(VAR) * HD * D1;
  if (g == 0) {
    mine[OB + j] = accb1;
    mine[OB + D1 + j] = accw2;
  }
  if (l == 0) mine[OB + 2 * D1] = accb2;
  __syncthreads();
  for (int c = threadIdx.x; c < NP; c += blockDim.x) {
    float s = red[c];
#pragma unroll
    for (int ww = 1; ww < WPB; ++ww) s += red[ww * NP + c];
    part[(int64_t)blockIdx.x * NP + c] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// Split form: TWO waves per sample (a block = 2 samples), wave half h taking the 16-position steps
// t0 = 16 (2 c + h): each wave's dependent chain of steps is half as long (the one-wave form is
// latency-bound at one wave per SIMD for config 4).  The halves meet through LDS: the softmax max
// and sum (VAR 1), the pooled partial sums, and in the backward sum_t p_t dp_t (VAR 1) and the
// per-sample G / gsum partials, which half 0 combines (in half order) for dq and the weight
// accumulators.  Every wave of a block runs the same number of sample iterations and barriers.
// ---------------------------------------------------------------------------------------------
template <int VAR>
__global__ void __launch_bounds__(64 * WPB) din_fwd_split_kernel(
    Geo geo, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, float* __restrict__ out,
    int64_t out_ld, float* __restrict__ probs) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int l = lane_id(), g = l >> 4, j = l & 15, w = wave_id(), pr = w >> 1, hf = w & 1;
  const int T = geo.T;
  float* sbuf = smem + pr * T;              // VAR 1: the pair's scores
  float* xo = smem + 2 * T + pr * 24;       // [16] half 1's pooled partial, [16..17] max, [18..19] sum
  Frags<VAR> fr;
  fr.load(W1, b1, W2, b2);
  const int64_t per_it = (int64_t)gridDim.x * 2;
  const int64_t n_it = (geo.B + per_it - 1) / per_it;
  for (int64_t it = 0; it < n_it; ++it) {
    const int64_t b = it * per_it + (int64_t)blockIdx.x * 2 + pr;
    const bool live = b < geo.B;
    const int64_t bb = live ? b : 0;
    SampleW<VAR> sw;
    sw.build(fr, geo.q + bb * geo.q_ld);
    const float* krow0 = geo.k + bb * geo.k_ss;
    const float* vrow0 = geo.v + bb * geo.v_ss;
    const int len = geo.lengths ? min(geo.lengths[bb], T) : T;
    float o = 0.f, mx = -INFINITY;
    if (live) {
      float4 an = load_keys(krow0, geo.k_rs, 16 * hf, T);
      Vals vn{};
      if (VAR == 0) vn = load_vals(vrow0, geo.v_rs, 16 * hf, T);
      for (int t0 = 16 * hf; t0 < T; t0 += 32) {
        const float4 a = an;
        const Vals vc = vn;
        if (t0 + 32 < T) {
          an = load_keys(krow0, geo.k_rs, t0 + 32, T);
          if (VAR == 0) vn = load_vals(vrow0, geo.v_rs, t0 + 32, T);
        }
        const f32x4 acc = layer1_frag(a, sw.bw);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z1 = acc[r] + sw.c;
          const float h = VAR == 0 ? fmaxf(z1, 0.f) : sigm(z1);
          const float z2 = group_sum<16>(h * fr.w2) + fr.b2;
          const int t = t0 + 4 * g + r;
          if (t < T) {
            const bool on = pos_on(geo, bb, t, len);
            if (VAR == 0) {
              o = fmaf(on ? fmaxf(z2, 0.f) : 0.f, vc.v[r], o);
            } else {
              const float sc = on ? z2 : PAD;
              mx = fmaxf(mx, sc);
              if (j == 0) sbuf[t] = sc;
            }
          }
        }
      }
    }
    float inv = 1.f;
    if (VAR == 1) {
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      if (l == 0) xo[16 + hf] = mx;
      __syncthreads();  // both halves' scores and maxima
      mx = fmaxf(xo[16], xo[17]);
      float lsum = 0.f;
      if (live) {
        Vals fn = load_vals(vrow0, geo.v_rs, 16 * hf, T);
        for (int t0 = 16 * hf; t0 < T; t0 += 32) {
          const Vals fc = fn;
          if (t0 + 32 < T) fn = load_vals(vrow0, geo.v_rs, t0 + 32, T);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = t0 + 4 * g + r;
            if (t < T) {
              const float e = __expf(sbuf[t] - mx);
              lsum += e;
              o = fmaf(e, fc.v[r], o);
            }
          }
        }
      }
      lsum += __shfl_xor(lsum, 16, 64);
      lsum += __shfl_xor(lsum, 32, 64);
      if (l == 0) xo[18 + hf] = lsum;
    }
    o += __shfl_xor(o, 16, 64);
    o += __shfl_xor(o, 32, 64);
    if (hf == 1 && g == 0) xo[j] = o;
    __syncthreads();  // half 1's partials (and both sums)
    if (VAR == 1) inv = 1.0f / (xo[18] + xo[19]);
    if (live && hf == 0 && g == 0) out[b * out_ld + j] = (o + xo[j]) * inv;
    if (VAR == 1 && live && probs) {
      for (int t = l + 64 * hf; t < T; t += 128) probs[b * T + t] = __expf(sbuf[t] - mx) * inv;
    }
    __syncthreads();  // sbuf / exchange reuse
  }
}

template <int VAR>
__global__ void __launch_bounds__(64 * WPB) din_bwd_split_kernel(
    Geo geo, const float* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ W2, const float* __restrict__ b2, const float* __restrict__ probs,
    const float* __restrict__ dout, int64_t dout_ld, float* __restrict__ dq, int64_t dq_ld,
    float* __restrict__ dk, float* __restrict__ dv, float* __restrict__ part, int64_t dkv_rs,
    int dkv_pad, const float* __restrict__ dq_base, int64_t dqb_ld) {
  constexpr int NP = nparam(VAR);
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int l = lane_id(), g = l >> 4, j = l & 15, w = wave_id(), pr = w >> 1, hf = w & 1;
  const int T = geo.T;
  float* tt = smem + w * (16 * TT_LD);                      // [16][TT_LD] transpose tile
  float* sbuf = smem + WPB * 16 * TT_LD + pr * T;           // VAR 1: the pair's dp_t
  float* xg = smem + WPB * 16 * TT_LD + 2 * T + pr * (64 * 5 + 4);  // [64][5] half 1, [320..] sdp
  float* red = smem;                                        // [WPB][NP], aliases the above at the end
  const bool alias_kv = geo.k == geo.v;
  const bool alias_d = dk != nullptr && dk == dv;
  Frags<VAR> fr;
  fr.load(W1, b1, W2, b2);
  float accA[4] = {0.f, 0.f, 0.f, 0.f}, accG[4] = {0.f, 0.f, 0.f, 0.f};
  float accQG[4] = {0.f, 0.f, 0.f, 0.f};
  float accb1 = 0.f, accw2 = 0.f, accb2 = 0.f;
  const int64_t per_it = (int64_t)gridDim.x * 2;
  const int64_t n_it = (geo.B + per_it - 1) / per_it;
  for (int64_t it = 0; it < n_it; ++it) {
    const int64_t b = it * per_it + (int64_t)blockIdx.x * 2 + pr;
    const bool live = b < geo.B;
    const int64_t bb = live ? b : 0;
    SampleW<VAR> sw;
    const float* qrow = geo.q + bb * geo.q_ld;
    sw.build(fr, qrow);
    const float qi = qrow[j];
    float tb[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) tb[r] = fmaf(qi, fr.tqk[r], fr.tk[r]);  // W1'[j][4g + r]
    const float* krow0 = geo.k + bb * geo.k_ss;
    const float* vrow0 = geo.v + bb * geo.v_ss;
    const int len = geo.lengths ? min(geo.lengths[bb], T) : T;
    const float doj = dout[bb * dout_ld + j];
    const float* prow = VAR == 1 ? probs + bb * T : nullptr;
    float sdp = 0.f;
    if (VAR == 1) {  // pass 1: dp_t = dout . f_t over this half's steps, sum_t p_t dp_t
      if (live) {
        Vals fn = load_vals(vrow0, geo.v_rs, 16 * hf, T);
        for (int t0 = 16 * hf; t0 < T; t0 += 32) {
          const Vals fc = fn;
          if (t0 + 32 < T) fn = load_vals(vrow0, geo.v_rs, t0 + 32, T);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int t = t0 + 4 * g + r;
            const float dp = group_sum<16>(doj * fc.v[r]);
            if (t < T) {
              sdp = fmaf(prow[t], dp, sdp);
              if (j == 0) sbuf[t] = dp;
            }
          }
        }
      }
      sdp += __shfl_xor(sdp, 16, 64);
      sdp += __shfl_xor(sdp, 32, 64);
      if (l == 0) xg[320 + hf] = sdp;
      __syncthreads();
      sdp = xg[320] + xg[321];
    }
    f32x4 G = {0.f, 0.f, 0.f, 0.f};
    float gs = 0.f;
    if (live) {
      float4 an = load_keys(krow0, geo.k_rs, 16 * hf, T);
      Vals vn = load_vals(vrow0, geo.v_rs, 16 * hf, T);
      for (int t0 = 16 * hf; t0 < T; t0 += 32) {
        const float4 a = an;
        const Vals vc = vn;
        if (t0 + 32 < T) {
          an = load_keys(krow0, geo.k_rs, t0 + 32, T);
          vn = load_vals(vrow0, geo.v_rs, t0 + 32, T);
        }
        const f32x4 acc = layer1_frag(a, sw.bw);
        float dz1[4], kv[4], dvv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = t0 + 4 * g + r;
          const bool in = t < T;
          const float z1 = acc[r] + sw.c;
          const float h = VAR == 0 ? fmaxf(z1, 0.f) : sigm(z1);
          const bool on = in && pos_on(geo, bb, t, len);
          float dz2, vval;
          if (VAR == 0) {
            const float z2 = group_sum<16>(h * fr.w2) + fr.b2;
            vval = vc.v[r];
            const float ds = group_sum<16>(doj * vval);
            const float s = on ? fmaxf(z2, 0.f) : 0.f;
            dz2 = (on && z2 > 0.f) ? ds : 0.f;
            dvv[r] = s * doj;
            kv[r] = alias_kv ? vval : (in ? krow0[(int64_t)t * geo.k_rs + j] : 0.f);
            dz1[r] = h > 0.f ? dz2 * fr.w2 : 0.f;
          } else {
            const float p = in ? prow[t] : 0.f;
            dz2 = on ? p * (sbuf[in ? t : 0] - sdp) : 0.f;
            vval = vc.v[r];
            dvv[r] = p * doj;
            kv[r] = vval;
            dz1[r] = dz2 * fr.w2 * h * (1.0f - h);
          }
          accw2 = fmaf(h, dz2, accw2);
          if (j == 0) accb2 += dz2;
          gs += dz1[r];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) G = mfma4(kv[r], dz1[r], G);
#pragma unroll
        for (int r = 0; r < 4; ++r) tt[(4 * g + r) * TT_LD + j] = dz1[r];
        wave_lds_sync();
        const float4 az = *reinterpret_cast<const float4*>(tt + (l & 15) * TT_LD + 4 * g);
        wave_lds_sync();
        f32x4 DK = {0.f, 0.f, 0.f, 0.f};
        DK = mfma4(az.x, tb[0], DK);
        DK = mfma4(az.y, tb[1], DK);
        DK = mfma4(az.z, tb[2], DK);
        DK = mfma4(az.w, tb[3], DK);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int t = t0 + 4 * g + r;
          if (t < T) {
            const int64_t off = (b * T + t) * dkv_rs + j;
            const bool zpad = j + HD < dkv_pad;
            if (VAR == 1 || alias_d) {
              float* base = dk ? dk : dv;
              if (base) {
                base[off] = DK[r] + dvv[r];
                if (zpad) base[off + HD] = 0.f;
              }
            } else {
              if (dk) { dk[off] = DK[r]; if (zpad) dk[off + HD] = 0.f; }
              if (dv) { dv[off] = dvv[r]; if (zpad) dv[off + HD] = 0.f; }
            }
          }
        }
      }
    }
    gs += __shfl_xor(gs, 16, 64);
    gs += __shfl_xor(gs, 32, 64);  // this half's gsum_j, in every lane of column j
    if (hf == 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) xg[l * 5 + r] = G[r];
      xg[l * 5 + 4] = gs;
    }
    __syncthreads();  // half 1's G / gsum
    if (hf == 0 && live) {
#pragma unroll
      for (int r = 0; r < 4; ++r) G[r] += xg[l * 5 + r];
      gs += xg[l * 5 + 4];
      float dqv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dqv[r] = group_sum<16>(fmaf(fr.rq[r], gs, fr.rqk[r] * G[r]));
        accA[r] = fmaf(sw.qv[r], gs, accA[r]);
        accG[r] += G[r];
        accQG[r] = fmaf(sw.qv[r], G[r], accQG[r]);
      }
      if (g == 0) accb1 += gs;
      if (j == 0) {
        if (dq_base) {
#pragma unroll
          for (int r = 0; r < 4; ++r) dqv[r] += dq_base[b * dqb_ld + 4 * g + r];
        }
        *reinterpret_cast<float4*>(dq + b * dq_ld + 4 * g) = make_float4(dqv[0], dqv[1], dqv[2], dqv[3]);
      }
    }
    __syncthreads();  // exchange / sbuf reuse
  }
  // ---- weight-gradient partials: wave -> block (LDS, wave order) -> part[blockIdx] ----
  accw2 += __shfl_xor(accw2, 16, 64);
  accw2 += __shfl_xor(accw2, 32, 64);
  accb2 += __shfl_xor(accb2, 16, 64);
  accb2 += __shfl_xor(accb2, 32, 64);
  __syncthreads();
  float* mine = red + w * NP;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = 4 * g + r;
    mine[(0 * HD + i) * D1 + j] = accA[r];
    mine[(1 * HD + i) * D1 + j] = accG[r];
    if (VAR == 0) {
      mine[(2 * HD + i) * D1 + j] = accQG[r];
    } else {
      mine[(2 * HD + i) * D1 + j] = accA[r] - accG[r];
      mine[(3 * HD + i) * D1 + j] = accQG[r];
    }
  }
  constexpr int OB = nblk(VAR) * HD * D1;
  if (g == 0) {
    mine[OB + j] = accb1;
    mine[OB + D1 + j] = accw2;
  }
  if (l == 0) mine[OB + 2 * D1] = accb2;
  __syncthreads();
  for (int c = threadIdx.x; c < NP; c += blockDim.x) {
    float s = red[c];
#pragma unroll
    for (int ww = 1; ww < WPB; ++ww) s += red[ww * NP + c];
    part[(int64_t)blockIdx.x * NP + c] = s;
  }
}

// Two waves per sample while one wave per sample would leave fewer than two waves per SIMD
// (B < 2048 on 1024 SIMDs): config 4 (B = 1024, T = 100) 0.0998 -> 0.0975 ms; at config 5
// (B = 2048, T = 50) the split measured 1.780 -> 1.797 ms (twice the partial rows, and the chip
// already holds two waves per SIMD), profiles/r05/split_ab/.  Tuning runs: RS_DIN_SPLIT=0 / 1.
static bool din_split(int64_t B) {
  static const int mode = [] {
    const char* e = getenv("RS_DIN_SPLIT");
    return e && *e ? atoi(e) : -1;
  }();
  return mode >= 0 ? mode != 0 : B < 2048;
}

static int fwd_grid(int64_t B) {
  const int spb = din_split(B) ? WPB / 2 : WPB;  // samples per block
  int64_t g = (B + spb - 1) / spb;
  return (int)(g > 4096 ? 4096 : g);
}
static int bwd_grid(int64_t B) {
  // one sample per wave: the per-sample chain is latency-bound, so waves beat fewer partial rows
  // (two samples per wave: config 4 0.1222 ms, config 5 1.890 ms; one: 0.1115 / 1.861 ms,
  // profiles/r05/din_spw/); tuning runs: RS_DIN_BWD_SPW
  static const int spw = [] {
    const char* e = getenv("RS_DIN_BWD_SPW");
    return e && atoi(e) > 0 ? atoi(e) : 1;
  }();
  const int64_t spb = din_split(B) ? WPB / 2 : (int64_t)spw * WPB;  // samples per block
  int64_t g = (B + spb - 1) / spb;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace rs_din

using namespace rs_din;

RS_API int rs_din_param_count(int variant, int H) {
  if ((variant != 0 && variant != 1) || H != HD) return RS_ERR_UNSUPPORTED;
  return nparam(variant);
}

RS_API int64_t rs_din_bwd_workspace_floats(int variant, int64_t B, int T, int H) {
  (void)T;
  if ((variant != 0 && variant != 1) || H != HD || B <= 0) return 0;
  return (int64_t)bwd_grid(B) * nparam(variant);
}

static int din_check(int variant, const float* q, int64_t q_ld, const float* k, int64_t k_ss,
                     int64_t k_rs, const float* v, int64_t v_ss, int64_t v_rs, int64_t B, int T,
                     int H) {
  if (variant != 0 && variant != 1) return RS_ERR_ARG;
  if (H != HD) return RS_ERR_UNSUPPORTED;
  if (!q || !k || !v || B < 0 || T <= 0) return RS_ERR_ARG;
  if (q_ld % 4 || k_rs % 4 || k_ss % 4 || q_ld < H || k_rs < H || v_rs < H) return RS_ERR_ARG;
  if (variant == 1 && (v != k || v_ss != k_ss || v_rs != k_rs)) return RS_ERR_ARG;
  if (T > 8192) return RS_ERR_UNSUPPORTED;
  return RS_OK;
}

RS_API int rs_din_fwd(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
                      int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
                      int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
                      int64_t mask_ld, const float* W1, const float* b1, const float* W2,
                      const float* b2, float* out, int64_t out_ld, float* probs) {
  int st = din_check(variant, q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T, H);
  if (st) return st;
  if (!W1 || !b1 || !W2 || !b2 || !out || out_ld < H) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  Geo geo{q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T, lengths, mask, mask_ld};
  hipStream_t s = rs_stream(stream);
  if (din_split(B)) {
    const size_t lds = ((size_t)2 * T + 48) * 4;
    if (variant == 0)
      din_fwd_split_kernel<0><<<fwd_grid(B), 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, out, out_ld,
                                                                 probs);
    else
      din_fwd_split_kernel<1><<<fwd_grid(B), 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, out, out_ld,
                                                                 probs);
    return rs_status_after_launch();
  }
  const size_t lds = variant == 1 ? (size_t)WPB * T * 4 : 0;
  if (variant == 0)
    din_fwd_kernel<0><<<fwd_grid(B), 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, out, out_ld, probs);
  else
    din_fwd_kernel<1><<<fwd_grid(B), 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, out, out_ld, probs);
  return rs_status_after_launch();
}

RS_API int rs_din_bwd_ex(void* stream, int variant, const float* q, int64_t q_ld,
                         const float* keys, int64_t k_ss, int64_t k_rs, const float* values,
                         int64_t v_ss, int64_t v_rs, int64_t B, int T, int H,
                         const int32_t* lengths, const uint8_t* mask, int64_t mask_ld,
                         const float* W1, const float* b1, const float* W2, const float* b2,
                         const float* probs, const float* dout, int64_t dout_ld, float* dq,
                         int64_t dq_ld, const float* dq_base, int64_t dq_base_ld, float* dkeys,
                         float* dvalues, int64_t dkv_rs, int dkv_width, float* dparams,
                         int dparams_accumulate, float* workspace, int64_t workspace_floats) {
  int st = din_check(variant, q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T, H);
  if (st) return st;
  if (dkv_rs < H || dkv_width < H || dkv_width > dkv_rs || dkv_width > 2 * H) return RS_ERR_ARG;
  if (!W1 || !b1 || !W2 || !b2 || !dout || !dq || dq_ld % 4 || dq_ld < H) return RS_ERR_ARG;
  if (dq_base && dq_base_ld < H) return RS_ERR_ARG;
  if (variant == 1 && !probs) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  const int grid = bwd_grid(B);
  const int np = nparam(variant);
  if (dparams && (!workspace || workspace_floats < (int64_t)grid * np)) return RS_ERR_ARG;
  Geo geo{q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T, lengths, mask, mask_ld};
  hipStream_t s = rs_stream(stream);
  const bool split = din_split(B);
  size_t lds = split ? ((size_t)WPB * 16 * TT_LD + 2 * (size_t)T + 2 * (64 * 5 + 4)) * 4
                     : ((size_t)WPB * 16 * TT_LD + (variant == 1 ? (size_t)WPB * T : 0)) * 4;
  const size_t red = (size_t)WPB * np * 4;
  if (lds < red) lds = red;
  // without dparams the partials still need somewhere to go: the caller must pass a workspace
  if (!workspace || workspace_floats < (int64_t)grid * np) return RS_ERR_ARG;
  if (split && variant == 0)
    din_bwd_split_kernel<0><<<grid, 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, probs, dout, dout_ld,
                                                        dq, dq_ld, dkeys, dvalues, workspace,
                                                        dkv_rs, dkv_width, dq_base, dq_base_ld);
  else if (split)
    din_bwd_split_kernel<1><<<grid, 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, probs, dout, dout_ld,
                                                        dq, dq_ld, dkeys, dvalues, workspace,
                                                        dkv_rs, dkv_width, dq_base, dq_base_ld);
  else if (variant == 0)
    din_bwd_kernel<0><<<grid, 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, probs, dout, dout_ld, dq,
                                                  dq_ld, dkeys, dvalues, workspace, dkv_rs,
                                                  dkv_width, dq_base, dq_base_ld);
  else
    din_bwd_kernel<1><<<grid, 64 * WPB, lds, s>>>(geo, W1, b1, W2, b2, probs, dout, dout_ld, dq,
                                                  dq_ld, dkeys, dvalues, workspace, dkv_rs,
                                                  dkv_width, dq_base, dq_base_ld);
  st = rs_status_after_launch();
  if (st || !dparams) return st;
  launch_column_reduce(s, workspace, grid, np, np, np, dparams, dparams, dparams_accumulate);
  return rs_status_after_launch();
}

RS_API int rs_din_bwd_strided(void* stream, int variant, const float* q, int64_t q_ld,
                              const float* keys, int64_t k_ss, int64_t k_rs, const float* values,
                              int64_t v_ss, int64_t v_rs, int64_t B, int T, int H,
                              const int32_t* lengths, const uint8_t* mask, int64_t mask_ld,
                              const float* W1, const float* b1, const float* W2, const float* b2,
                              const float* probs, const float* dout, int64_t dout_ld, float* dq,
                              int64_t dq_ld, float* dkeys, float* dvalues, int64_t dkv_rs,
                              int dkv_width, float* dparams, int dparams_accumulate,
                              float* workspace, int64_t workspace_floats) {
  return rs_din_bwd_ex(stream, variant, q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T, H,
                       lengths, mask, mask_ld, W1, b1, W2, b2, probs, dout, dout_ld, dq, dq_ld,
                       nullptr, 0, dkeys, dvalues, dkv_rs, dkv_width, dparams, dparams_accumulate,
                       workspace, workspace_floats);
}

RS_API int rs_din_bwd(void* stream, int variant, const float* q, int64_t q_ld, const float* keys,
                      int64_t k_ss, int64_t k_rs, const float* values, int64_t v_ss, int64_t v_rs,
                      int64_t B, int T, int H, const int32_t* lengths, const uint8_t* mask,
                      int64_t mask_ld, const float* W1, const float* b1, const float* W2,
                      const float* b2, const float* probs, const float* dout, int64_t dout_ld,
                      float* dq, int64_t dq_ld, float* dkeys, float* dvalues, float* dparams,
                      int dparams_accumulate, float* workspace, int64_t workspace_floats) {
  return rs_din_bwd_strided(stream, variant, q, q_ld, keys, k_ss, k_rs, values, v_ss, v_rs, B, T,
                            H, lengths, mask, mask_ld, W1, b1, W2, b2, probs, dout, dout_ld, dq,
                            dq_ld, dkeys, dvalues, H, H, dparams, dparams_accumulate, workspace,
                            workspace_floats);
}
