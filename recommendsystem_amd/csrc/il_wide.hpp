// InteractingLayer forward / backward for the AutoInt CTR shape family (E = U = 16, H = 2,
// F <= 32), ONE 256-THREAD WORKGROUP (4 waves) PER SAMPLE.
//
// Reference: InteractingLayer.py:37-61 (the math is restated in il_kernels.hpp's header).
//
// Why a second kernel pair (round 4): the per-sample-wave kernels (fwd_kernel, bwd4_kernel) keep
// one sample on one wave, so one sample-iteration is a serial chain of ~1.7 K VALU + 96 MFMA
// instructions on one SIMD.  At 255 VGPRs the backward holds 2 waves per SIMD and its PMC shows
// 40 % issue / 30 % waiting (latency-bound); below ~2 K samples per GPU (the strong-scaling
// series: 512 per GPU at N = 8) most SIMDs are idle and the step time is one sample's latency.
// Here the four waves of a workgroup split every phase of one sample:
//   * MFMA phases by 16-wide column tile: wave w owns projection columns [16w, 16w + 16)
//     (Q, K, V, R for w = 0..3), the matching dW tile (no cross-wave reduction: the tiles are
//     disjoint) and the k-chunk 16w.. of dx = G W^T (4 partial tiles summed in wave order in
//     LDS).  Each wave's weight fragments (4 + 4 floats + bias) stay in VGPRs for the kernel.
//   * attention sweeps by KEY (or query) across the waves: lane = (head, row) = h F + i as in
//     the one-wave kernels, wave w takes keys j = w, w + 4, ... -- the key rows are wave-uniform
//     (broadcast LDS reads, scalar loop control, no per-lane address math), so each wave runs
//     the lean bwd4-style sweep over a quarter of the keys.  The waves' partials meet in LDS:
//     forward (m_w, l_w, o_w) combined flash-style in the LN epilogue; backward dq partials
//     (Q-pass, 4 waves) and dv (waves 0, 1) / dk (waves 2, 3) partials (K-pass, queries split
//     in two) summed in wave order by a combine phase that also applies the ReLU masks.
//   * LN (forward epilogue / backward) by (row, column pair): 8 lanes per row, DPP row sums.
// Per sample-iteration the backward stores P (dropout-applied) and dS = P (dP - D) in LDS in the
// Q-pass, so the K-pass (dV, dK) does no dP recompute.  A workgroup needs ~49 KB of LDS in the
// backward (3 per CU, 135 VGPRs) and ~23 KB in the forward.
//
// Numerics: fp32 everywhere (bf16 math mode: the same bf16 MFMA operand rounding as the
// per-sample-wave kernels); the projections use mfma tiles identical to mfma_project (bitwise the
// same Q/K/V/R); scores q . k in even/odd fma pairs (dot_reg_pk) in the forward and the backward
// (bitwise the same S); softmax / attention / LN sums in a different fixed order than the
// per-sample-wave kernels (partials per wave, combined in wave order): deterministic, within fp32
// rounding of them.
#pragma once
#ifndef RS_ILW_PRIO
#define RS_ILW_PRIO 0
#endif

namespace rs_il {

template <class C>
constexpr bool kWide = C::E == 16 && C::U == 16 && C::H == 2 && C::FMAX <= 32 && C::NC == 64;

constexpr int kWideThreads = 256;
constexpr int kWideRows = 32;  // every per-sample buffer holds 32 rows (2 MFMA row tiles)

// threadIdx.x through an empty asm (as lane_id()): indices derived from it are re-derived in
// each phase instead of being hoisted and kept live across the whole sample loop
__device__ __forceinline__ int tid_v() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ float quad_sum(float v) {
  v += dpp_mov<0xB1>(v);  // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);  // quad_perm [2,3,0,1]
  return v;
}
__device__ __forceinline__ float quad_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  return v;
}

// 8 floats from LDS (two ds_read_b128)
__device__ __forceinline__ void ld8(float (&v)[8], const float* p) {
  const float4 a = reinterpret_cast<const float4*>(p)[0];
  const float4 b = reinterpret_cast<const float4*>(p)[1];
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// wave w's projection: PR[f][16w + j] = relu(X[f] . W[:, 16w + j] + b) for both row tiles
// (the bias as the accumulator's initial value and the k order of mfma_project: bitwise the
// same values); rows >= F are written too (PR and X hold kWideRows rows; X's rows >= F are 0)
template <class C>
__device__ __forceinline__ void wide_project(const float* X, float* PR, const float (&wp)[4],
                                             float bp, int w) {
  const int q = lane_id() >> 4, j = lane_id() & 15;
  f32x4 acc[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    acc[rt] = f32x4{bp, bp, bp, bp};
    const float4 v = *reinterpret_cast<const float4*>(X + (16 * rt + j) * 16 + 4 * q);
    if constexpr (C::BF) {
      acc[rt] = mfma_bf16(pack_bf16(v.x, v.y), pack_bf16(v.z, v.w), wp[0], wp[1], acc[rt]);
    } else {
      acc[rt] = mfma_16x16x4(v.x, wp[0], acc[rt]);
      acc[rt] = mfma_16x16x4(v.y, wp[1], acc[rt]);
      acc[rt] = mfma_16x16x4(v.z, wp[2], acc[rt]);
      acc[rt] = mfma_16x16x4(v.w, wp[3], acc[rt]);
    }
  }
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      PR[(16 * rt + 4 * q + r) * C::PRS + 16 * w + j] = fmaxf(acc[rt][r], 0.f);
}

// this wave's weight fragments: projection B (W[4q + t][16w + j]), bias, dx B (W[j][16w + 4q + t])
template <class C>
__device__ __forceinline__ void wide_load_w(const float* __restrict__ W, const float* __restrict__ bias,
                                            int w, float (&wp)[4], float& bp, float (&wx)[4]) {
  const int q = lane_id() >> 4, j = lane_id() & 15;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    wp[t] = W[(4 * q + t) * C::NC + 16 * w + j];
    wx[t] = W[j * C::NC + 16 * w + 4 * q + t];
  }
  bp = bias[16 * w + j];
  if constexpr (C::BF) {
    wp[0] = pack_bf16(wp[0], wp[1]);
    wp[1] = pack_bf16(wp[2], wp[3]);
    wx[0] = pack_bf16(wx[0], wx[1]);
    wx[1] = pack_bf16(wx[2], wx[3]);
  }
}

// ============================== forward =======================================================
template <class C>
struct WideFwdLayout {
  int xb, pr, total;
  __host__ __device__ WideFwdLayout() {
    xb = 0;
    pr = xb + kWideRows * C::E;
    total = pr + kWideRows * C::PRS;
  }
};

// SKIP (diagnostic instantiations only, tools/il_variants.hip; 0 in the library): bits drop phases
// to time them by elimination (results are wrong).  Forward: 1 projection, 2 attention, 4 LN
// epilogue, 8 input load.  Backward: 1 P1, 2 P3, 4 Q-pass, 8 K-pass, 16 P7, 32 dx sum / push.
template <class C, bool DROP, int SKIP = 0>
__global__ void __launch_bounds__(kWideThreads, 2) wfwd_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ y,
    int64_t y_ld, float* __restrict__ xsave, Args a) {
  static_assert(kWide<C>, "wide kernels: E = U = 16, H = 2, F <= 32");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int U = C::U, DH = C::DH;
  constexpr int MQ = (C::FMAX + 3) / 4;  // keys per lane (quarter)
  const WideFwdLayout<C> lay;
  float* const X = smem + lay.xb;
  float* const PR = smem + lay.pr;
  const int tid = threadIdx.x;
  const int w = wave_id();
#if RS_ILW_PRIO  // tuning builds: static priority for every other workgroup (all its waves)
  if (blockIdx.x & 1) __builtin_amdgcn_s_setprio(1);
#endif
  const int F = C::EXACT ? C::FMAX : a.F;
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);

  float wp[4], bp, wx[4];
  wide_load_w<C>(W, bias, w, wp, bp, wx);
  // LN lanes: row lf, columns u0, u0 + 1
  const int lf = tid >> 3, u0 = 2 * (tid & 7);
  const float gm0 = gamma[u0], gm1 = gamma[u0 + 1], bt0 = beta[u0], bt1 = beta[u0 + 1];
  // attention lanes: (head ah, query row ai), keys qq + 4m
  const int ag = tid >> 2, ah = ag >> 5, ai0 = ag & 31, qq = tid & 3;
  const bool aact = ai0 < F;
  const int ai = aact ? ai0 : 0;
  // X rows F .. 31 stay zero (the projection reads both row tiles unguarded)
  for (int k = F * C::E + tid; k < kWideRows * C::E; k += kWideThreads) X[k] = 0.f;

  IL_STAMP_DECL
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    IL_STAMP(0)
    // ---- the sample's field embeddings -> X ----
    constexpr int QV = C::E / 4;
    if (SKIP & 8) {
    } else if (a.g_table) {
      // fused single-hot gather (as fwd_kernel): float4 k = quarter k % 4 of field k / 4's row
      float4* xo = reinterpret_cast<float4*>(const_cast<float*>(x) + b * F * C::E);
      if (tid < F * QV) {
        const int f = tid / QV, qv = tid - f * QV;
        const int64_t row = hash_row(a.g_ids[b * F + f], a.g_base[f], a.g_bucket[f], a.g_hash);
        const bool ok = row >= 0 && row < a.g_table_rows;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) v = reinterpret_cast<const float4*>(a.g_table + row * C::E)[qv];
        reinterpret_cast<float4*>(X)[tid] = v;
        xo[tid] = v;
        if (qv == 0 && a.g_rows) a.g_rows[b * F + f] = ok ? (int32_t)row : -1;
      }
    } else if (tid < F * QV) {
      reinterpret_cast<float4*>(X)[tid] = reinterpret_cast<const float4*>(x + b * F * C::E)[tid];
    }
    lds_barrier();
    IL_STAMP(1)
    for (int it = 0; it < a.L; ++it) {
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      // ---- projections (wave w: columns 16w..16w+15) ----
      if constexpr (!(SKIP & 1)) wide_project<C>(X, PR, wp, bp, w);
      lds_barrier();
      IL_STAMP(2)
      // ---- attention: (head, query) quad, keys qq + 4m ----
      if constexpr (!(SKIP & 2)) {
        float qv[DH];
        ld8(qv, PR + ai * C::PRS + ah * DH);
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] *= a.sc2;  // scores straight in the exp2 domain
        const float* kb = PR + U + ah * DH;
        const float* vb = PR + 2 * U + ah * DH;
        float s[MQ];
        float mx = -INFINITY;
#pragma unroll
        for (int m = 0; m < MQ; ++m) {
          const int j = qq + 4 * m;
          const bool ok = (C::EXACT && 4 * m + 3 < C::FMAX) || j < F;
          float kv[DH];
          ld8(kv, kb + (ok ? j : 0) * C::PRS);
          s[m] = dot_reg_pk(qv, kv);
          mx = ok ? fmaxf(mx, s[m]) : mx;
        }
        mx = quad_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int m = 0; m < MQ; ++m) {
          const int j = qq + 4 * m;
          const bool ok = (C::EXACT && 4 * m + 3 < C::FMAX) || j < F;
          s[m] = ok ? __builtin_amdgcn_exp2f(s[m] - mx) : 0.f;
          sum += s[m];
        }
        sum = quad_sum(sum);
        const float inv = 1.0f / sum;
        float o[DH];
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] = 0.f;
        const uint32_t kb_drop = DROP ? dropout_sample_key(lseed, (uint32_t)b) : 0u;
#pragma unroll
        for (int m = 0; m < MQ; ++m) {
          const int j = qq + 4 * m;
          const bool ok = (C::EXACT && 4 * m + 3 < C::FMAX) || j < F;
          float p = s[m] * inv;
          if (DROP) p = dropout_keep_k(kb_drop, ah, ai, j, a.drop_rate) ? p * a.drop_scale : 0.f;
          float vv[DH];
          ld8(vv, vb + (ok ? j : 0) * C::PRS);
          axpy_reg_pk(o, p, vv);
        }
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] = quad_sum(o[d]);
        // O_i over Q_i in place (only this quad read Q_i, all four lanes before the sums)
        float2 mine = make_float2(o[0], o[1]);
        if (qq == 1) mine = make_float2(o[2], o[3]);
        if (qq == 2) mine = make_float2(o[4], o[5]);
        if (qq == 3) mine = make_float2(o[6], o[7]);
        if (aact) {
          *reinterpret_cast<float2*>(PR + ai * C::PRS + ah * DH + 2 * qq) = mine;
          if (a.osave) {  // the saved path: O row and (max, 1 / sum) for the backward
            float* gs = a.osave + ((int64_t)it * a.B + b) * small_save_stride(F, U, C::H);
            *reinterpret_cast<float2*>(gs + ai * U + ah * DH + 2 * qq) = mine;
            if (qq == 0) *reinterpret_cast<float2*>(gs + F * U + 2 * (ah * F + ai)) = make_float2(mx, inv);
          }
        }
      }
      lds_barrier();
      IL_STAMP(3)
      // ---- z = relu(O + R); y = LN(z): 8 lanes per row, two columns each ----
      if constexpr (!(SKIP & 4)) {
        const bool act = lf < F;
        const int f = act ? lf : 0;
        const float2 o2 = *reinterpret_cast<const float2*>(PR + f * C::PRS + u0);
        float2 r2 = *reinterpret_cast<const float2*>(PR + f * C::PRS + 3 * U + u0);
        if (!a.use_res) r2 = make_float2(0.f, 0.f);
        const float z0 = fmaxf(o2.x + r2.x, 0.f), z1 = fmaxf(o2.y + r2.y, 0.f);
        const float mean = group_sum<8>(z0 + z1) * (1.0f / (float)U);
        const float d0 = z0 - mean, d1 = z1 - mean;
        const float var = group_sum<8>(d0 * d0 + d1 * d1) * (1.0f / (float)U);
        const float rstd = 1.0f / sqrtf(var + a.eps);
        const float2 yv = make_float2(d0 * rstd * gm0 + bt0, d1 * rstd * gm1 + bt1);
        if (it == a.L - 1) {
          if (act) *reinterpret_cast<float2*>(y + b * y_ld + f * U + u0) = yv;
        } else {  // (X is its own buffer: no barrier between these reads and the X stores)
          if (act) {
            *reinterpret_cast<float2*>(X + f * C::E + u0) = yv;  // E == U when L > 1
            if (xsave)
              *reinterpret_cast<float2*>(xsave + ((int64_t)it * a.B + b) * F * U + f * U + u0) = yv;
          }
        }
      }
      lds_barrier();
      IL_STAMP(4)
    }
  }
  IL_STAMP_FLUSH(a.stamps)
}

// ============================== backward (saved path) =========================================
template <class C>
struct WideBwdLayout {
  int xb0, xb1, sb0, sb1, dy, pr, pm, pd, dl, qp, hf1, total;
  __host__ __device__ WideBwdLayout(int F) {
    const int sv = (int)small_save_stride(F, C::U, C::H);
    hf1 = C::H * F + 1;  // attention rows h F + i, plus one dummy row for the idle lanes
    int off = 0;
    xb0 = off; off += kWideRows * C::E;
    xb1 = off; off += kWideRows * C::E;
    sb0 = off; off += (sv + 3) & ~3;
    sb1 = off; off += (sv + 3) & ~3;
    dy = off; off += (F * C::U + 3) & ~3;
    pr = off; off += kWideRows * C::PRS;
    // P and dS, one row per attention lane.  Once the K-pass sweep is done PM + PD also hold its
    // dv / dk partials (4 x hf1 x 8), and in P7 the 4 x 2 x 4 x 64 dx partial tiles (2 048)
    const int pmn = (hf1 * C::PMS + 3) & ~3;
    const int need = 4 * hf1 * 8 > 2048 ? 4 * hf1 * 8 : 2048;
    const int pmd = 2 * pmn > need ? pmn : (need + 1) / 2 + 4;
    pm = off; off += pmd;
    pd = off; off += pmd;
    dl = off; off += (C::H * kWideRows + 3) & ~3;
    qp = off; off += 4 * hf1 * 8;  // the Q-pass's dq partials [wave][row][8]
    total = off;
  }
};

template <class C>
__host__ __forceinline__ size_t wbwd_lds_bytes(int F) {
  return (size_t)WideBwdLayout<C>(F).total * 4;
}

template <class C, bool DROP, int SKIP = 0>
__global__ void __launch_bounds__(kWideThreads, 4) wbwd_kernel(
    const float* __restrict__ x, const float* __restrict__ xsave, const float* __restrict__ dy,
    int64_t dy_ld, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ dx,
    int dx_accumulate, float* __restrict__ partials, Args a) {
  static_assert(kWide<C>, "wide kernels: E = U = 16, H = 2, F <= 32");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int U = C::U, DH = C::DH, E = C::E;
  constexpr int MQ = (C::FMAX + 3) / 4;
  const int F = C::EXACT ? C::FMAX : a.F;
  const WideBwdLayout<C> lay(F);
  float* XB = smem + lay.xb0;  // this iteration's input X (rows >= F zero)
  float* XN = smem + lay.xb1;  // the next iteration's (prefetch)
  float* SB = smem + lay.sb0;  // this iteration's save: O | stats; O becomes dO in P3
  float* SN = smem + lay.sb1;
  float* const DY = smem + lay.dy;
  float* const PR = smem + lay.pr;
  float* const PM = smem + lay.pm;  // P (dropout applied)  [h][i][j]
  float* const PD = smem + lay.pd;  // dS = P (dP - D)       [h][i][j]
  float* const DL = smem + lay.dl;  // D_{h,i} = dO_i . O_i
  float* const QP = smem + lay.qp;
  float* const KVP = PM;            // K-pass partials, after its sweep (PM / PD are dead then)
  float* const XS = PM;             // P7: the 4 waves' dx partial tiles
  const int HF1 = lay.hf1;          // partial rows per wave
  const int w = wave_id();
  const int sv = (int)small_save_stride(F, U, C::H);
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);

  float wp[4], bp, wx[4];
  wide_load_w<C>(W, bias, w, wp, bp, wx);
  const float gm0 = gamma[2 * (threadIdx.x & 7)], gm1 = gamma[2 * (threadIdx.x & 7) + 1];
  // per-phase lane roles, re-derived where used (tid_v):
  //   LN (P3): row tid / 8, columns 2 (tid % 8) + {0, 1}
  //   attention: (head, row) = (tid / 128, tid / 4 % 32), quarter tid % 4
  //   MFMA fragments: q = lane / 16, j = lane % 16
#define RS_W_ATTN_IDX                                                       \
  const int t_ = tid_v();                                                   \
  const int ah = t_ >> 7, ai0 = (t_ >> 2) & 31, qq = t_ & 3;                \
  const bool aact = ai0 < F;                                                \
  const int ai = aact ? ai0 : 0;

  // zero once: X rows >= F of both buffers (read by the projection's unguarded row tiles)
  for (int k = F * E + (int)threadIdx.x; k < kWideRows * E; k += kWideThreads) {
    smem[lay.xb0 + k] = 0.f;
    smem[lay.xb1 + k] = 0.f;
  }

  f32x4 dwacc = f32x4{0.f, 0.f, 0.f, 0.f};  // dW[4q + r][16w + jx]
  float dbp = 0.f;                           // db[16w + jx] over this lane's rows
  float dg0 = 0.f, dg1 = 0.f, dbt0 = 0.f, dbt1 = 0.f;

  const int nx4 = F * E / 4, ns4 = sv / 4, ny4 = F * U / 4;
  auto x_src = [&](int64_t bb, int itx) -> const float* {
    return itx == 0 ? x + bb * F * E : xsave + ((int64_t)(itx - 1) * a.B + bb) * F * U;
  };
  auto s_src = [&](int64_t bb, int itx) -> const float* {
    return a.osave_in + ((int64_t)itx * a.B + bb) * sv;
  };
  const bool push = a.push_table != nullptr;
  const bool with_base = push && dx_accumulate;
  const int64_t b0 = blockIdx.x, bstep = gridDim.x;
  if (b0 < a.B) {
    glds_copy(XB, x_src(b0, a.L - 1), nx4);
    glds_copy(SB, s_src(b0, a.L - 1), ns4);
    glds_copy(DY, dy + b0 * dy_ld, ny4);
  }
  // the deferred weight-gradient jobs, while the first sample's operands stream in
  xt_wave_jobs(a, (int64_t)blockIdx.x * 4 + w, (int64_t)gridDim.x * 4);
  IL_STAMP_DECL
  for (int64_t b = b0; b < a.B; b += bstep) {
    for (int it = a.L - 1; it >= 0; --it) {
      IL_STAMP(0)
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      const int64_t bn = it > 0 ? b : b + bstep;  // the next iteration's sample
      const int itn = it > 0 ? it - 1 : a.L - 1;
      const bool has_next = bn < a.B;
      // fused push: this thread's two output cells (rows pf and pf + 16, column jx of tid's
      // 16-lane group) -- their table rows and the head's share, loaded now, used in P7
      const int pf = (int)(threadIdx.x >> 4), pe = (int)(threadIdx.x & 15);
      int32_t rw0 = -1, rw1 = -1;
      float bv0 = 0.f, bv1 = 0.f;
      if (it == 0 && push) {
        if (pf < F) {
          rw0 = a.push_rows[b * F + pf];
          if (with_base) bv0 = dx[(b * F + pf) * E + pe];
        }
        if (pf + 16 < F) {
          rw1 = a.push_rows[b * F + pf + 16];
          if (with_base) bv1 = dx[(b * F + pf + 16) * E + pe];
        }
      }
      vm_wait_all();  // this wave's prefetches of X / save (/ dy) for this iteration
      lds_barrier();
      IL_STAMP(1)
      // ---- P1: projections (wave w: columns 16w..) and dW's X operand into registers ----
      if constexpr (!(SKIP & 1)) wide_project<C>(XB, PR, wp, bp, w);
      float xa[2][4];
      const int q = lane_id() >> 4, jx = lane_id() & 15;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int t = 0; t < 4; ++t) xa[rt][t] = XB[(16 * rt + 4 * q + t) * E + jx];
      // the next iteration's input and save stream into the spare buffers meanwhile
      if (has_next) {
        glds_copy(XN, x_src(bn, itn), nx4);
        glds_copy(SN, s_src(bn, itn), ns4);
      }
      lds_barrier();
      IL_STAMP(2)
      // ---- P3: z = relu(O + R); LN + ReLU backward -> dO (SB), gR (PR's R slot), D ----
      if constexpr (!(SKIP & 2)) {
        const int t_ = tid_v();
        const int lf = t_ >> 3, u0 = 2 * (t_ & 7);
        const bool act = lf < F;
        const int f = act ? lf : 0;
        const float2 o2 = *reinterpret_cast<const float2*>(SB + f * U + u0);
        const float2 r2 = *reinterpret_cast<const float2*>(PR + f * C::PRS + 3 * U + u0);
        float2 y2 = *reinterpret_cast<const float2*>(DY + f * U + u0);
        if (!act) y2 = make_float2(0.f, 0.f);
        const float rr0 = a.use_res ? r2.x : 0.f, rr1 = a.use_res ? r2.y : 0.f;
        const float z0 = fmaxf(o2.x + rr0, 0.f), z1 = fmaxf(o2.y + rr1, 0.f);
        const float mean = group_sum<8>(z0 + z1) * (1.0f / (float)U);
        const float c0 = z0 - mean, c1 = z1 - mean;
        const float var = group_sum<8>(c0 * c0 + c1 * c1) * (1.0f / (float)U);
        const float rstd = 1.0f / sqrtf(var + a.eps);
        const float zh0 = c0 * rstd, zh1 = c1 * rstd;
        dg0 = fmaf(y2.x, zh0, dg0);
        dg1 = fmaf(y2.y, zh1, dg1);
        dbt0 += y2.x;
        dbt1 += y2.y;
        const float g0 = y2.x * gm0, g1 = y2.y * gm1;
        const float sg = group_sum<8>(g0 + g1) * (1.0f / (float)U);
        const float sgz = group_sum<8>(g0 * zh0 + g1 * zh1) * (1.0f / (float)U);
        const float dz0 = (g0 - sg - zh0 * sgz) * rstd, dz1 = (g1 - sg - zh1 * sgz) * rstd;
        const float dt0 = z0 > 0.f ? dz0 : 0.f, dt1 = z1 > 0.f ? dz1 : 0.f;
        // D_{h,f} = dO_f . O_f over head h = the 4 lanes of this column quad
        const float dd = quad_sum(fmaf(o2.x, dt0, o2.y * dt1));
        if (act) {
          // dO and D stored x the row's softmax 1/sum (as bwd4): the sweeps use e_ij for P_ij
          const float isum = SB[F * U + 2 * ((u0 >> 3) * F + f) + 1];
          *reinterpret_cast<float2*>(PR + f * C::PRS + 3 * U + u0) =
              make_float2((a.use_res && r2.x > 0.f) ? dt0 : 0.f, (a.use_res && r2.y > 0.f) ? dt1 : 0.f);
          *reinterpret_cast<float2*>(SB + f * U + u0) = make_float2(dt0 * isum, dt1 * isum);
          if ((t_ & 3) == 0) DL[(u0 >> 3) * F + f] = dd * isum;
        }
      }
      lds_barrier();
      IL_STAMP(3)
      // ---- Q-pass: lane = (head, query i) (lane = h F + i), wave w takes keys j = w, w + 4, ...
      //      (wave-uniform key rows: broadcast LDS reads, scalar loop): P, dS -> PM / PD row
      //      `lane`; this wave's dq partial -> QP[w][lane] ----
      if constexpr (!(SKIP & 4)) {
        const int lane = lane_id();
        const bool act = lane < C::H * F;
        const int h = act ? (lane >= F ? 1 : 0) : 0;
        const int i = act ? lane - h * F : 0;
        float qv[DH], dO[DH], dq[DH];
        ld8(qv, PR + i * C::PRS + h * DH);
        ld8(dO, SB + i * U + h * DH);  // x 1/sum_i (P3)
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] *= a.sc2;  // scores straight in the exp2 domain
        const float2 stt = *reinterpret_cast<const float2*>(SB + F * U + 2 * (h * F + i));
        const float D = DL[h * F + i];  // x 1/sum_i
        const float* kb = PR + U + h * DH;
        const float* vb = PR + 2 * U + h * DH;
        // row = lane = h F + i; the idle lanes (>= H F) share the dummy row H F (never read)
        const int prow = act ? lane : C::H * F;
        float* const pm_row = PM + prow * C::PMS;
        float* const pd_row = PD + prow * C::PMS;
        const uint32_t kb_drop = DROP ? dropout_sample_key(lseed, (uint32_t)b) : 0u;
#pragma unroll
        for (int d = 0; d < DH; ++d) dq[d] = 0.f;
        const int nk = (F - w + 3) >> 2;  // keys w + 4m < F
        auto ld = [&](float (&kv)[DH], float (&vv)[DH], int m) {
          const int mm = m < nk ? m : (nk > 0 ? nk - 1 : 0);
          const int j = w + 4 * mm;
          ld8(kv, kb + j * C::PRS);
          ld8(vv, vb + j * C::PRS);
        };
        auto key = [&](int m, const float (&kv)[DH], const float (&vv)[DH]) {
          const int j = w + 4 * m;
          // sv_ = s_ij - max_i and (without dropout) dp = dP_ij - D_i by the dots' initial
          // values; p = e_ij = P_ij sum_i, with dO and D already x 1/sum_i
          float sv_, dp;
          dot2_reg_pk(qv, kv, dO, vv, sv_, dp, -stt.x, DROP ? 0.f : -D);
          const float p = __builtin_amdgcn_exp2f(sv_);
          float pdrop = p;
          if (DROP) {
            const bool keep = dropout_keep_k(kb_drop, h, i, j, a.drop_rate);
            pdrop = keep ? p * a.drop_scale : 0.f;
            dp = (keep ? dp * a.drop_scale : 0.f) - D;
          }
          const float ds = p * dp;
          pm_row[j] = pdrop;
          pd_row[j] = ds;
          axpy_reg_pk(dq, ds, kv);
        };
        // software-pipelined by one key (two register sets), as bwd4's sweeps
        float k0[DH], v0[DH], k1[DH], v1[DH];
        ld(k0, v0, 0);
        for (int m = 0; m < nk; m += 2) {
          ld(k1, v1, m + 1);
          key(m, k0, v0);
          ld(k0, v0, m + 2);
          if (m + 1 < nk) key(m + 1, k1, v1);
        }
        float4* qp = reinterpret_cast<float4*>(QP + (w * HF1 + prow) * 8);
        qp[0] = make_float4(dq[0], dq[1], dq[2], dq[3]);
        qp[1] = make_float4(dq[4], dq[5], dq[6], dq[7]);
      }
      lds_barrier();
      IL_STAMP(4)
      // ---- K-pass: lane = (head, key j); waves 0, 1: dv_j = sum_i Pd_ij dO_i over queries
      //      i = w, w + 2, ...; waves 2, 3: dk_j = sum_i dS_ij q_i over i = w - 2, w, ... ->
      //      KVP[w][lane] ----
      if constexpr (!(SKIP & 8)) {
        const int lane = lane_id();
        const bool act = lane < C::H * F;
        const int h = act ? (lane >= F ? 1 : 0) : 0;
        const int j = act ? lane - h * F : 0;
        const bool isv = w < 2;  // wave-uniform
        const int i0 = w & 1;
        const int ni = (F - i0 + 1) >> 1;
        const float* col = (isv ? PM : PD) + h * F * C::PMS + j;
        const float* vec = (isv ? SB : PR) + h * DH;
        const int vs = isv ? U : C::PRS;
        float acc[DH];
#pragma unroll
        for (int d = 0; d < DH; ++d) acc[d] = 0.f;
        auto ld = [&](float (&v)[DH], float& c, int m) {
          const int mm = m < ni ? m : (ni > 0 ? ni - 1 : 0);
          const int i = i0 + 2 * mm;
          ld8(v, vec + i * vs);
          c = col[i * C::PMS];
        };
        float v0[DH], v1[DH], c0, c1;
        ld(v0, c0, 0);
        for (int m = 0; m < ni; m += 2) {
          ld(v1, c1, m + 1);
          axpy_reg_pk(acc, c0, v0);
          ld(v0, c0, m + 2);
          if (m + 1 < ni) axpy_reg_pk(acc, c1, v1);
        }
        lds_barrier();  // every wave's P / dS reads are done: the partials go over PM / PD
        float4* kp = reinterpret_cast<float4*>(KVP + (w * HF1 + (act ? lane : C::H * F)) * 8);
        kp[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        kp[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
      } else {
        lds_barrier();
      }
      lds_barrier();
      IL_STAMP(5)
      // ---- combine (wave order, fixed): gQ = relu'(Q) sum_w dq_w / sqrt(dh), gK = relu'(K)
      //      (dk_2 + dk_3) / sqrt(dh), gV = relu'(V) (dv_0 + dv_1) -> PR's Q, K, V slots ----
      {
        const int n4 = 12 * F;  // (slot Q / K / V, row f, head, half) float4 items
        for (int t4 = tid_v(); t4 < n4; t4 += kWideThreads) {
          const int half = t4 & 1, hh = (t4 >> 1) & 1, rest = t4 >> 2;
          const int sl = rest >= 2 * F ? 2 : (rest >= F ? 1 : 0);
          const int f = rest - sl * F;
          const int l = hh * F + f;
          float* g = PR + f * C::PRS + sl * U + hh * DH + 4 * half;
          const float4 cur = *reinterpret_cast<const float4*>(g);
          float4 sum;
          float sc = a.inv_sdh;
          if (sl == 0) {
            const float* qp = QP + l * 8 + 4 * half;
            const int ws = HF1 * 8;
            const float4 p0 = *reinterpret_cast<const float4*>(qp);
            const float4 p1 = *reinterpret_cast<const float4*>(qp + ws);
            const float4 p2 = *reinterpret_cast<const float4*>(qp + 2 * ws);
            const float4 p3 = *reinterpret_cast<const float4*>(qp + 3 * ws);
            sum = make_float4(((p0.x + p1.x) + p2.x) + p3.x, ((p0.y + p1.y) + p2.y) + p3.y,
                              ((p0.z + p1.z) + p2.z) + p3.z, ((p0.w + p1.w) + p2.w) + p3.w);
          } else {
            const int ws = HF1 * 8;
            const float* kp = KVP + (sl == 1 ? 2 * ws : 0) + l * 8 + 4 * half;
            const float4 p0 = *reinterpret_cast<const float4*>(kp);
            const float4 p1 = *reinterpret_cast<const float4*>(kp + ws);
            sum = make_float4(p0.x + p1.x, p0.y + p1.y, p0.z + p1.z, p0.w + p1.w);
            if (sl == 2) sc = 1.f;
          }
          *reinterpret_cast<float4*>(g) =
              make_float4(cur.x > 0.f ? sum.x * sc : 0.f, cur.y > 0.f ? sum.y * sc : 0.f,
                          cur.z > 0.f ? sum.z * sc : 0.f, cur.w > 0.f ? sum.w * sc : 0.f);
        }
      }
      lds_barrier();
      IL_STAMP(6)
      // dO (SB) is dead: at the last iteration of the sample the next sample's dy streams into
      // DY once P7's barrier has passed (below)
      // ---- P7: G = [gQ | gK | gV | gR] column tile w; dW += X^T G, db; dx partial = G W_w^T ----
      if constexpr (!(SKIP & 16)) {
        // G rows of this lane for dW (B operand: k = f = 16rt + 4q + t, n = 16w + jx) and for dx
        // (A operand: m = f = 16rt + jx, k = 16w + 4q + t)
        const int q = lane_id() >> 4, jx = lane_id() & 15;
        const int lane = lane_id();
        float gb[2][4], ga[2][4];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int f = 16 * rt + 4 * q + t;
            const float g = PR[f * C::PRS + 16 * w + jx];
            gb[rt][t] = f < F ? g : 0.f;
            dbp += gb[rt][t];
          }
          const int fa = 16 * rt + jx;
          const float4 g4 = *reinterpret_cast<const float4*>(PR + fa * C::PRS + 16 * w + 4 * q);
          ga[rt][0] = g4.x; ga[rt][1] = g4.y; ga[rt][2] = g4.z; ga[rt][3] = g4.w;
        }
        f32x4 acc[2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (C::BF) {
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            dwacc = mfma_bf16(pack_bf16(xa[rt][0], xa[rt][1]), pack_bf16(xa[rt][2], xa[rt][3]),
                              pack_bf16(gb[rt][0], gb[rt][1]), pack_bf16(gb[rt][2], gb[rt][3]), dwacc);
            acc[rt] = mfma_bf16(pack_bf16(ga[rt][0], ga[rt][1]), pack_bf16(ga[rt][2], ga[rt][3]),
                                wx[0], wx[1], acc[rt]);
          }
        } else {
#pragma unroll
          for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              dwacc = mfma_16x16x4(xa[rt][t], gb[rt][t], dwacc);
              acc[rt] = mfma_16x16x4(ga[rt][t], wx[t], acc[rt]);
            }
        }
        // partial tile of wave w -> XS[w][rt][r][lane] (PM / PD are dead since the K-pass)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) XS[((w * 2 + rt) * 4 + r) * 64 + lane] = acc[rt][r];
      }
      lds_barrier();
      IL_STAMP(7)
      if (it == 0 && has_next) glds_copy(DY, dy + bn * dy_ld, ny4);  // the next sample's dy
      // ---- dx = sum of the 4 partial tiles (wave order), cells (pf, pe) and (pf + 16, pe):
      //      -> DY (the next iteration's dy), or the fused push, or dx ----
      if constexpr (!(SKIP & 32)) {
        // cell (f, e): row tile f / 16, r = f % 4, q = (f % 16) / 4, lane = 16 q + e
        float v[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int f = pf + 16 * k;
          const int rt = f >> 4, r = f & 3, ql = (f & 15) >> 2;
          const int idx = (rt * 4 + r) * 64 + 16 * ql + pe;
          v[k] = ((XS[idx] + XS[512 + idx]) + XS[1024 + idx]) + XS[1536 + idx];
        }
        if (it > 0) {
          // (DY's dq was last read in P7, before the barrier above)
          if (pf < F) DY[pf * U + pe] = v[0];
          if (pf + 16 < F) DY[(pf + 16) * U + pe] = v[1];
        } else if (push) {
          if (rw0 >= 0) {
            if (pe == 0) scan_mark(a.push_flag, rw0);
            atomicAdd(a.push_table + (int64_t)rw0 * E + pe, v[0] + bv0);
          }
          if (rw1 >= 0) {
            if (pe == 0) scan_mark(a.push_flag, rw1);
            atomicAdd(a.push_table + (int64_t)rw1 * E + pe, v[1] + bv1);
          }
        } else {
          float* d = dx + b * F * E;
          if (pf < F) d[pf * E + pe] = dx_accumulate ? d[pf * E + pe] + v[0] : v[0];
          if (pf + 16 < F) d[(pf + 16) * E + pe] = dx_accumulate ? d[(pf + 16) * E + pe] + v[1] : v[1];
        }
      }
      if (it > 0) { IL_STAMP(8) } else { IL_STAMP(9) }
      float* t = XB; XB = XN; XN = t;
      t = SB; SB = SN; SN = t;
    }
  }
  // ---- block partials: dW tiles are disjoint per wave (no reduction), db over q, dgamma / dbeta
  //      over rows (lanes) then waves, fixed order ----
#undef RS_W_ATTN_IDX
  IL_STAMP_FLUSH(a.stamps)
  const int tid = threadIdx.x, lane = lane_id(), q = lane >> 4, jx = lane & 15;
  dbp += __shfl_xor(dbp, 16, 64);
  dbp += __shfl_xor(dbp, 32, 64);
#pragma unroll
  for (int o = 8; o < 64; o <<= 1) {
    dg0 += __shfl_xor(dg0, o, 64);
    dg1 += __shfl_xor(dg1, o, 64);
    dbt0 += __shfl_xor(dbt0, o, 64);
    dbt1 += __shfl_xor(dbt1, o, 64);
  }
  float* const out = partials + (int64_t)blockIdx.x * C::NPARAM;
#pragma unroll
  for (int r = 0; r < 4; ++r) out[(4 * q + r) * C::NC + 16 * w + jx] = dwacc[r];
  if (q == 0) out[E * C::NC + 16 * w + jx] = dbp;
  lds_barrier();
  float* const RED = smem;  // [wave][gamma 16 | beta 16]
  if (lane < 8) {
    RED[w * 32 + 2 * lane] = dg0;
    RED[w * 32 + 2 * lane + 1] = dg1;
    RED[w * 32 + 16 + 2 * lane] = dbt0;
    RED[w * 32 + 16 + 2 * lane + 1] = dbt1;
  }
  lds_barrier();
  if (tid < 32)
    out[E * C::NC + C::NC + tid] = ((RED[tid] + RED[32 + tid]) + RED[64 + tid]) + RED[96 + tid];
}

}  // namespace rs_il
