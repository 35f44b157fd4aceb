// H3 — AutoInt InteractingLayer (multi-head self-attention over field embeddings), fused.
//
// Reference: InteractingLayer.py:7-61 (byte-identical rank/multi_head/interacting_layer.py:7-61).
// Per iteration it < layer_num, with the SAME Dense/LN objects every iteration (tied weights,
// InteractingLayer.py:41-46):
//   Q,K,V = relu(x Wq + bq), relu(x Wk + bk), relu(x Wv + bv)           :42-44
//   R     = relu(x Wr + br)                    (use_res)                 :45-46
//   heads = split(., H, axis=2) concat axis 0 -> [H*B, F, dh]            :47-49
//   S     = Qh Kh^T / sqrt(dh)                 (dh = post-split width)   :50-51
//   P     = softmax(S) ; dropout(P) when use_dropout (train)             :52-54
//   O     = merge_heads(P Vh)                                            :55-56
//   x     = LN(relu(O + R))                    (keras-layer-normalization form,
//           (z - mean)/sqrt(var + eps) * gamma + beta; eps pinned by the caller)  :57-60
//
// MI355X mapping (one wave = one sample; samples are independent):
//   * the sample's x, the four projections, the attention output (and in backward the softmax
//     matrix and every gradient) live in LDS: only x_in, x_out and the per-iteration inputs saved
//     for backward touch HBM.  The TF graph materialises ~15 intermediates per iteration
//     including the [H*B, F, F] scores; here scores never leave LDS/VGPRs.
//   * projections: lane = output column of [Wq|Wk|Wv|Wr] (4U = 64 columns at U = 16), the
//     column's E weights in VGPRs, x rows broadcast from LDS (one address per wave).
//   * attention: lane = (head, query row); the row's scores stay in VGPRs (softmax per lane:
//     exp(s - max) * (1/sum), TF's order, evaluated as v_exp_f32 in the base-2 domain with
//     log2(e)/sqrt(dh) folded into one multiply; no fp32 divisions in any loop); K/V rows are
//     broadcast LDS reads.  Key rows F..FMAX-1
//     are zero and masked to -inf, so the j loops are unguarded and fully unrolled with
//     compile-time LDS offsets (no per-key branch, no runtime stride arithmetic).
//   * epilogue: U lanes per field row; LN mean/var by xor-butterfly inside the U-lane group.
//   * backward recomputes the iteration from its saved input (only x_it is stored: 1.7 KB per
//     sample per iteration), back-propagates LN, ReLU, attention and projections in LDS, keeps
//     dW/db/dgamma/dbeta in VGPRs across every sample a wave visits, then reduces wave -> block
//     (fixed order) -> grid (fixed order): deterministic weight gradients, no float atomics.
// All arithmetic is fp32, as in the reference.
#pragma once
#include "common.hpp"

#include <cstdlib>

namespace rs_il {

struct FwdReq {
  hipStream_t stream;
  const float *x, *W, *bias, *gamma, *beta;
  int64_t B;
  int F, E, U, H, L, use_res;
  float eps, drop_rate;
  uint64_t seed;
  float *y, *xsave;
  int64_t y_ld;  // row stride of y (>= F*U): lets the layer write into a concat buffer
  // many-field path (F > 64): the attention save the backward reads instead of recomputing
  // (rs_il_fwd_saved; layout il_large.hip::save_stride), or null
  float* asave = nullptr;
  // fused single-hot gather (rs_il_fwd_gather): x[b, f, :] = table[hash(ids[b, f])] is read
  // straight into LDS, stored to x (the head's and the backward's input) and the hashed rows to
  // gather_rows -- replaces the rs_embedding_lookup_fwd launch and the re-read of x
  const int64_t* gather_ids = nullptr;
  const int64_t* gather_base = nullptr;
  const int64_t* gather_bucket = nullptr;
  const float* gather_table = nullptr;
  int64_t gather_table_rows = 0;
  int32_t* gather_rows = nullptr;
  int gather_hash = 0;
  int bf16 = 0;  // RS_MATH_BF16 (rs_set_math_mode): bf16 operands on the matrix cores
};

struct BwdReq {
  hipStream_t stream;
  const float *x, *xsave, *dy, *W, *bias, *gamma, *beta;
  int64_t dy_ld;  // row stride of dy (>= F*U)
  int64_t B;
  int F, E, U, H, L, use_res;
  float eps, drop_rate;
  uint64_t seed;
  float* dx;
  int dx_accumulate;
  float* dparams;
  int dparams_accumulate;
  float* workspace;
  int64_t workspace_floats;
  const float* asave = nullptr;  // rs_il_bwd_saved: the forward's attention save (F > 64)
  // fused sparse push (rs_il_bwd_push): dL/dx of the first iteration is added (with dx's
  // current contents when dx_accumulate) straight into push_table rows push_rows[b * F + f],
  // marking push_flag[row] = -2 (scan mode) instead of being stored to dx
  const int32_t* push_rows = nullptr;
  float* push_table = nullptr;
  int32_t* push_flag = nullptr;
  // dry run: write the grid (= number of per-block partial rows) the launch would use and
  // return without launching (rs_il_bwd_partial_blocks)
  int* grid_out = nullptr;
  int bf16 = 0;  // RS_MATH_BF16 (rs_set_math_mode): bf16 operands on the matrix cores
  // a deferred weight gradient carried by this launch (rs_il_bwd_saved_xt): the fused head's
  // dW1 = xt_x^T xt_dz over the batch, as xt_splits(B) sample-range partial rows in xt_slab
  const float* xt_x = nullptr;
  const float* xt_dz = nullptr;
  int64_t xt_ldx = 0, xt_lddz = 0;
  int xt_K0 = 0, xt_N1 = 0;
  float* xt_slab = nullptr;
};

constexpr int kMaxFwdWaves = 4;
constexpr int kFwdSpreadBlocks = 512;
constexpr int kMaxBwdWaves = 2;
#ifndef RS_IL_BWD_GRID
#define RS_IL_BWD_GRID 1536
#endif
constexpr int kMaxBwdGrid = RS_IL_BWD_GRID;
constexpr size_t kLdsBytes = 160 * 1024;

template <int E_, int U_, int H_, int FMAX_, bool EXACT_ = false, bool BF_ = false>
struct Cfg {
  static constexpr int E = E_, U = U_, H = H_, FMAX = FMAX_;
  static constexpr bool EXACT = EXACT_;                // F == FMAX: no padded keys to mask
  // bf16 math mode (rs_set_math_mode): projection / dW / dx MFMAs take bf16-rounded operands
  // (v_mfma_f32_16x16x16_bf16, fp32 accumulate); attention, LN, storage and weights stay fp32
  static constexpr bool BF = BF_;
  static constexpr int NC = 4 * U;                     // [Q | K | V | R] projection columns
  static constexpr int DH = U / H;
  static constexpr int NCOLW = NC < 64 ? NC : 64;      // lanes per projection row
  static constexpr int RPI = 64 / NCOLW;               // rows per projection step
  static constexpr int CPLP = NC / NCOLW;              // column chunks per lane
  static constexpr int LPR = U < 64 ? U : 64;          // lanes per row in the LN epilogue
  static constexpr int RG = 64 / LPR;                  // rows per epilogue step
  static constexpr int CPLN = U / LPR;                 // LN columns per lane
  static constexpr int RGE = 64 / E;                   // rows per dx step (E <= 64)
  static constexpr int NPARAM = E * NC + NC + 2 * U;   // W | b | gamma | beta
  // LDS row strides (floats), compile-time: every access inside an unrolled loop is
  // base + immediate.  Region bases depend on the runtime F and are per-wave scalars.
  static constexpr int PRS = NC + 4;                   // projection row stride (16-B aligned)
  static constexpr int OS = U + 4;                     // attention-output row stride
  static constexpr int PMS = FMAX + 1;                 // softmax-matrix row stride
  static constexpr int WPS = NC + 4;                   // padded W row stride in LDS (dx phase)

  static_assert(U % H == 0, "unit_num must be divisible by head_num");
  static_assert(E % 4 == 0 && DH % 4 == 0, "E and dh must be multiples of 4");
  static_assert(E <= 64, "E <= 64");
};

// Diagnostic build only (-DRS_IL_STAMPS): per-phase s_memtime deltas summed per wave and added to
// a global u64 array (cdna_hip_programming.md §7 "In-kernel stamps"); shares, not absolute time.
#ifdef RS_IL_STAMPS
#define IL_STAMP_DECL uint64_t st_prev_ = 0, st_acc_[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define IL_STAMP(k)                                                                    \
  {                                                                                    \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    uint64_t t_;                                                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");         \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    if ((k) > 0) st_acc_[(k)-1] += t_ - st_prev_;                                      \
    st_prev_ = t_;                                                                     \
  }
#define IL_STAMP_FLUSH(ptr)                                                            \
  if ((ptr) && lane_id() == 0)                                                         \
    for (int k_ = 0; k_ < 10; ++k_) atomicAdd((unsigned long long*)(ptr) + k_, st_acc_[k_]);
#else
#define IL_STAMP_DECL
#define IL_STAMP(k)
#define IL_STAMP_FLUSH(ptr)
#endif

struct Args {
  int B, F, L, use_res, ncol;
  float eps, sdh, drop_rate, drop_scale;
  float inv_sdh;    // 1 / sqrt(dh)
  float sc2;        // log2(e) / sqrt(dh): scores go straight to the exp2 domain
  uint64_t seed;
  uint64_t seed_off;           // rs_set_seed_offset source address (0 = none): seed + *src * K
  int l_x, l_pr, l_o, l_gpr, l_dy, l_pm, l_st, per_wave;  // per-wave LDS carve-up (floats)
  int l_tmp;                   // bwd2 only: partial-row exchange / dV buffer
  int l_x2, l_w, l_b;          // bwd2 only: second X buffer (prefetch), W and bias in LDS
  int dy_vec;                  // bwd2 only: dy rows 16-B aligned (async LDS copy)
  unsigned long long* stamps;  // diagnostic build only
  const int32_t* push_rows;    // fused sparse push (see BwdReq)
  float* push_table;
  int32_t* push_flag;
  const int64_t* g_ids;        // fused gather (see FwdReq); g_table == nullptr: read x
  const int64_t* g_base;
  const int64_t* g_bucket;
  const float* g_table;
  int32_t* g_rows;
  int64_t g_table_rows;
  int g_hash;
  // F <= 32 saved path (rs_il_fwd_saved / rs_il_bwd_saved, small_save_stride): per (iteration,
  // sample) the forward writes the attention output O [F][U] and the softmax row stats
  // [H*F] x {scaled max, 1 / sum}; the backward reads them instead of re-running the softmax
  float* osave;
  const float* osave_in;
  // deferred weight gradient (BwdReq::xt_*): slab[sp][k][n] = sum over sample range sp of
  // x[b][k] dz[b][n]; xt_nsplit ranges, jobs = (K0 / 16) x (N1 / 16) x nsplit 16 x 16 tiles
  const float* xt_x;
  const float* xt_dz;
  int64_t xt_ldx, xt_lddz;
  int xt_K0, xt_N1, xt_nsplit;
  float* xt_slab;
};

// sample ranges of the deferred weight gradient (a function of B alone: the partial rows, their
// fixed-order sum and so every bit of the result depend on B only)
__host__ __device__ inline int xt_splits(int64_t B) {
  const int64_t n = (B + 15) / 16;
  return (int)(n < 1 ? 1 : (n > 32 ? 32 : n));
}

// The deferred weight-gradient jobs of one wave (wave gw of nw in the grid): each job is a
// 16 x 16 tile (k tile, n tile) of x^T dz over one sample range, v_mfma_f32_16x16x4f32 with 4
// samples per step (A = x[b + q][16 kt + j], B = dz[b + q][16 nt + j]); eight steps' loads are
// issued before their MFMAs.  The tile goes to slab row sp (row-major [K0][N1]): the optimizer
// tail sums the nsplit rows in order.  Runs before the wave's first sample, while its first
// sample's operands stream into LDS.
__device__ __forceinline__ void xt_wave_jobs(const Args& a, int64_t gw, int64_t nw) {
  if (!a.xt_x) return;
  const int lane = threadIdx.x & 63, q = lane >> 4, j = lane & 15;
  const int nkt = a.xt_K0 >> 4, nnt = a.xt_N1 >> 4, ns = a.xt_nsplit;
  const int64_t njobs = (int64_t)nkt * nnt * ns;
  const int64_t per = ((((int64_t)a.B + ns - 1) / ns) + 3) & ~(int64_t)3;
  for (int64_t job = gw; job < njobs; job += nw) {
    const int sp = (int)(job % ns);
    const int64_t t = job / ns;
    const int kt = (int)(t % nkt), nt = (int)(t / nkt);
    const int64_t lo = sp * per;
    const int64_t hi = lo + per < (int64_t)a.B ? lo + per : (int64_t)a.B;
    const float* xp = a.xt_x + 16 * kt + j;
    const float* dp = a.xt_dz + 16 * nt + j;
    float __attribute__((ext_vector_type(4))) acc = {0.f, 0.f, 0.f, 0.f};
    constexpr int KB = 8;
    for (int64_t g = lo; g < hi; g += 4 * KB) {
      float xv[KB], dv[KB];
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const int64_t b = g + 4 * u + q;
        const bool ok = b < hi;
        xv[u] = ok ? xp[b * a.xt_ldx] : 0.f;
        dv[u] = ok ? dp[b * a.xt_lddz] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < KB; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv[u], dv[u], acc, 0, 0, 0);
    }
    float* o = a.xt_slab + (int64_t)sp * a.xt_K0 * a.xt_N1 + (int64_t)(16 * kt) * a.xt_N1 + 16 * nt + j;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[(int64_t)(4 * q + r) * a.xt_N1] = acc[r];
  }
}

static inline int r4(int v) { return (v + 3) & ~3; }

// floats per (iteration, sample) of the small-F attention save: O [F][U] | stats [H*F][2],
// padded to 16 B
__host__ __device__ inline int64_t small_save_stride(int F, int U, int H) {
  return ((int64_t)F * U + 2 * (int64_t)H * F + 3) & ~(int64_t)3;
}

template <class C>
Args make_args(int64_t B, int F, int L, int use_res, float eps, float drop_rate, uint64_t seed,
               bool bwd) {
  Args a;
  a.B = (int)B; a.F = F; a.L = L; a.use_res = use_res;
  a.xt_x = nullptr; a.xt_dz = nullptr; a.xt_slab = nullptr;
  a.xt_ldx = a.xt_lddz = 0; a.xt_K0 = a.xt_N1 = 0; a.xt_nsplit = 1;
  a.ncol = use_res ? C::NC : 3 * C::U;
  a.eps = eps;
  a.sdh = (float)__builtin_sqrt((double)C::DH);   // Python float dh ** 0.5 -> fp32 constant
  a.inv_sdh = (float)(1.0 / __builtin_sqrt((double)C::DH));
  a.sc2 = (float)(1.4426950408889634 / __builtin_sqrt((double)C::DH));
  a.drop_rate = drop_rate;
  a.drop_scale = drop_rate > 0.f ? (float)(1.0 / (1.0 - (double)drop_rate)) : 1.f;
  a.seed = seed;
  a.seed_off = (uint64_t)(uintptr_t)rs_seed_offset_now();
  int off = 0;
  a.l_x = off; off += r4(F * C::E);
  a.l_pr = off; off += r4(C::FMAX * C::PRS);  // FMAX rows: padded key/value rows stay zero
  a.l_o = 0;  // forward: the attention output aliases the Q columns of PR
  a.l_gpr = a.l_dy = a.l_pm = a.l_st = 0;
  if (bwd) {
    a.l_o = off; off += r4(F * C::OS);
    a.l_gpr = off; off += r4(F * C::PRS);
    a.l_dy = off; off += r4(F * C::U);
    a.l_pm = off; off += r4(C::H * F * C::PMS);
    a.l_st = off; off += r4(2 * C::H * F);   // LN stats / the split-j D partials
  }
  a.per_wave = off;
  a.l_tmp = 0;
  a.l_x2 = a.l_w = a.l_b = 0;
  a.dy_vec = 0;
#ifdef RS_IL_STAMPS
  extern unsigned long long* g_il_stamps;
  a.stamps = g_il_stamps;
#else
  a.stamps = nullptr;
#endif
  a.push_rows = nullptr;
  a.push_table = nullptr;
  a.push_flag = nullptr;
  a.g_ids = a.g_base = a.g_bucket = nullptr;
  a.g_table = nullptr;
  a.g_rows = nullptr;
  a.g_table_rows = 0;
  a.g_hash = 0;
  a.osave = nullptr;
  a.osave_in = nullptr;
  return a;
}

// bwd2 carve-up (one block = one sample at a time, two waves): W and bias resident for the whole
// kernel, two X buffers, no separate gradient region (the projection gradients overwrite Q/K/V/R
// in place once each is dead), a TMP region for partial rows / dV, and ST holding
// [m0 | m1 | l0 | l1] (forward recompute) then the D partials.
template <class C>
Args make_args2(int64_t B, int F, int L, int use_res, float eps, float drop_rate, uint64_t seed) {
  Args a = make_args<C>(B, F, L, use_res, eps, drop_rate, seed, false);
  int off = 0;
  a.l_w = off; off += r4(C::E * C::WPS);        // W [E][NC] (row stride WPS), block-resident
  a.l_b = off; off += r4(C::NC);                // bias
  a.l_x = off; off += r4(F * C::E);             // X, double-buffered: the next iteration's
  a.l_x2 = off; off += r4(F * C::E);            // input streams in while this one runs
  a.l_pr = off; off += r4(C::FMAX * C::PRS);
  a.l_o = off; off += r4(F * C::OS);
  a.l_dy = off; off += r4(F * C::U);
  a.l_tmp = off; off += r4(F * C::U);           // == DH * H * F
  a.l_pm = off; off += r4(C::H * F * C::PMS);
  a.l_st = off; off += r4(4 * C::H * F);
  a.l_gpr = 0;
  a.per_wave = off;
  return a;
}

// zero the padded projection rows F..FMAX-1 (done once per kernel; projections never write them)
template <class C>
__device__ __forceinline__ void zero_pad_rows(float* PR, int F) {
  for (int k = F * C::PRS + lane_id(); k < C::FMAX * C::PRS; k += 64) PR[k] = 0.f;
}

template <int N>
__device__ __forceinline__ void load_row(float (&v)[N], const float* p) {
  const float4* p4 = reinterpret_cast<const float4*>(p);
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) {
    const float4 t = p4[d4];
    v[4 * d4] = t.x; v[4 * d4 + 1] = t.y; v[4 * d4 + 2] = t.z; v[4 * d4 + 3] = t.w;
  }
}

template <int N>
__device__ __forceinline__ void store_row(float* p, const float (&v)[N]) {
  float4* p4 = reinterpret_cast<float4*>(p);
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) p4[d4] = make_float4(v[4 * d4], v[4 * d4 + 1], v[4 * d4 + 2], v[4 * d4 + 3]);
}

template <int N>
__device__ __forceinline__ float dot_row(const float (&q)[N], const float* p) {
  const float4* p4 = reinterpret_cast<const float4*>(p);
  float acc = 0.f;
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) {
    const float4 k = p4[d4];
    acc = fmaf(q[4 * d4], k.x, acc);
    acc = fmaf(q[4 * d4 + 1], k.y, acc);
    acc = fmaf(q[4 * d4 + 2], k.z, acc);
    acc = fmaf(q[4 * d4 + 3], k.w, acc);
  }
  return acc;
}

template <int N>
__device__ __forceinline__ void axpy_row(float (&o)[N], float p, const float* v) {
  const float4* v4 = reinterpret_cast<const float4*>(v);
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) {
    const float4 t = v4[d4];
    o[4 * d4] = fmaf(p, t.x, o[4 * d4]);
    o[4 * d4 + 1] = fmaf(p, t.y, o[4 * d4 + 1]);
    o[4 * d4 + 2] = fmaf(p, t.z, o[4 * d4 + 2]);
    o[4 * d4 + 3] = fmaf(p, t.w, o[4 * d4 + 3]);
  }
}

// packed-fp32 forms (v_pk_fma_f32: two fmas per lane per instruction, twice the v_fma_f32 rate;
// the attention phases of the backward are VALU-issue bound).  Dot products keep two interleaved
// partial sums (even / odd d), added at the end.  They need even-aligned register pairs: the
// 128-VGPR forward kernel keeps the scalar forms (the packed ones spill there).
typedef float f32x2v __attribute__((ext_vector_type(2)));

template <int N>
__device__ __forceinline__ float dot_row_pk(const float (&q)[N], const float* p) {
  const float4* p4 = reinterpret_cast<const float4*>(p);
  f32x2v acc = {0.f, 0.f};
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) {
    const float4 k = p4[d4];
    acc = __builtin_elementwise_fma(f32x2v{q[4 * d4], q[4 * d4 + 1]}, f32x2v{k.x, k.y}, acc);
    acc = __builtin_elementwise_fma(f32x2v{q[4 * d4 + 2], q[4 * d4 + 3]}, f32x2v{k.z, k.w}, acc);
  }
  return acc.x + acc.y;
}

template <int N>
__device__ __forceinline__ void axpy_row_pk(float (&o)[N], float p, const float* v) {
  const float4* v4 = reinterpret_cast<const float4*>(v);
  const f32x2v pp = {p, p};
#pragma unroll
  for (int d4 = 0; d4 < N / 4; ++d4) {
    const float4 t = v4[d4];
    const f32x2v lo = __builtin_elementwise_fma(pp, f32x2v{t.x, t.y}, f32x2v{o[4 * d4], o[4 * d4 + 1]});
    const f32x2v hi = __builtin_elementwise_fma(pp, f32x2v{t.z, t.w}, f32x2v{o[4 * d4 + 2], o[4 * d4 + 3]});
    o[4 * d4] = lo.x; o[4 * d4 + 1] = lo.y; o[4 * d4 + 2] = hi.x; o[4 * d4 + 3] = hi.y;
  }
}


// =============================================================================================
// GEMM-shaped phases on the matrix cores: v_mfma_f32_16x16x4_f32 (fp32 in, fp32 accumulate,
// exact: a k-ordered fma chain).  D[16x16] += A[16x4] B[4x16]; lane l = (q = l >> 4, j = l & 15)
// supplies A[j][k_q] and B[k_q][j] and holds D[4q + r][j] (r < 4).  The k index is PERMUTED
// consistently for A and B (k-step t takes k = 16s + 4q + t), so one ds_read_b128 of 4
// consecutive floats feeds 4 k-steps.  W lives in VGPRs for the whole kernel in both layouts
// (projection B operand and dx B operand), so only activations / gradients come from LDS:
// this replaces the per-row broadcast ds_read_b128 streams of the VALU version, which made the
// backward LDS-throughput bound (PMC: ~2.6K LDS instructions per sample-iteration).
// =============================================================================================
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma_16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// bf16 math mode: pack_bf16 / mfma_bf16 (common.hpp) take the same lane fragments.

template <class C>
struct MfmaW {
  static constexpr int KS = (C::E + 15) / 16;  // 16-wide k chunks of E
  static constexpr int NT = C::NC / 16;        // 16-wide column tiles of [Wq|Wk|Wv|Wr]
  static constexpr int ET = (C::E + 15) / 16;  // 16-wide e tiles (dx / dW rows)
  static constexpr int CS = C::NC / 16;        // 16-wide c chunks (dx reduction)
  float wp[KS][4][NT];  // projection B: W[16ks + 4q + t][16nt + j]
  float wx[CS][4][ET];  // dx B       : W[16et + j][16cs + 4q + t]
  // (bf16 mode: [..][0] / [..][1] hold the packed pairs t = 0,1 / 2,3; [2], [3] are never
  // touched and take no registers)
  float bp[NT];         // bias[16nt + j] (loop-invariant: kept out of the per-row loops)

  __device__ __forceinline__ void load(const float* __restrict__ W, const float* __restrict__ bias) {
    load_proj(W, bias);
    load_dx(W);
  }
  // projection B operand + bias only
  __device__ __forceinline__ void load_proj(const float* __restrict__ W,
                                            const float* __restrict__ bias) {
    const int q = lane_id() >> 4, j = lane_id() & 15;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bp[nt] = bias[16 * nt + j];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int k = 16 * ks + 4 * q + t;
          wp[ks][t][nt] = k < C::E ? W[k * C::NC + 16 * nt + j] : 0.f;
        }
    pack_proj();
  }
  __device__ __forceinline__ void pack_proj() {
    if constexpr (C::BF) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const float p01 = pack_bf16(wp[ks][0][nt], wp[ks][1][nt]);
          const float p23 = pack_bf16(wp[ks][2][nt], wp[ks][3][nt]);
          wp[ks][0][nt] = p01;
          wp[ks][1][nt] = p23;
        }
    }
  }
  __device__ __forceinline__ void pack_dx() {
    if constexpr (C::BF) {
#pragma unroll
      for (int cs = 0; cs < CS; ++cs)
#pragma unroll
        for (int et = 0; et < ET; ++et) {
          const float p01 = pack_bf16(wx[cs][0][et], wx[cs][1][et]);
          const float p23 = pack_bf16(wx[cs][2][et], wx[cs][3][et]);
          wx[cs][0][et] = p01;
          wx[cs][1][et] = p23;
        }
    }
  }
  // the same fragments from a block-resident LDS copy of W ([E][NC], row stride C::WPS) and bias
  __device__ __forceinline__ void load_proj_lds(const float* WL, const float* BL) {
    const int q = lane_id() >> 4, j = lane_id() & 15;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bp[nt] = BL[16 * nt + j];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int k = 16 * ks + 4 * q + t;
          wp[ks][t][nt] = k < C::E ? WL[k * C::WPS + 16 * nt + j] : 0.f;
        }
    pack_proj();
  }
  __device__ __forceinline__ void load_dx_lds(const float* WL) {
    const int q = lane_id() >> 4, j = lane_id() & 15;
#pragma unroll
    for (int cs = 0; cs < CS; ++cs)
#pragma unroll
      for (int et = 0; et < ET; ++et) {
        const int e = 16 * et + j;
        // the 4 t-values are consecutive columns: one ds_read_b128
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < C::E) v = *reinterpret_cast<const float4*>(WL + e * C::WPS + 16 * cs + 4 * q);
        wx[cs][0][et] = v.x; wx[cs][1][et] = v.y; wx[cs][2][et] = v.z; wx[cs][3][et] = v.w;
      }
    pack_dx();
  }
  // dx B operand only
  __device__ __forceinline__ void load_dx(const float* __restrict__ W) {
    const int q = lane_id() >> 4, j = lane_id() & 15;
#pragma unroll
    for (int cs = 0; cs < CS; ++cs)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int et = 0; et < ET; ++et) {
          const int e = 16 * et + j;
          wx[cs][t][et] = e < C::E ? W[e * C::NC + 16 * cs + 4 * q + t] : 0.f;
        }
    pack_dx();
  }
};

// PR[f][c] = relu(X[f] . W[:, c] + b[c]) for the 16 rows of row tile rt (rows >= F skipped)
template <class C, bool ALL_ROWS = false>
__device__ __forceinline__ void mfma_project(const float* X, float* PR, int F, int rt,
                                             const MfmaW<C>& w) {
  const int q = lane_id() >> 4, j = lane_id() & 15;
  using M = MfmaW<C>;
  f32x4 acc[M::NT];
  // the bias is the accumulator's initial value (column 16nt + j in every row): no add per
  // output.  Every IL kernel (forward and the recomputing backwards) projects through this one
  // function, so the backward's Q / K / V / R equal the forward's bit for bit.
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) {
    const float bc = w.bp[nt];
    acc[nt] = f32x4{bc, bc, bc, bc};
  }
  const int arow = 16 * rt + j;  // A row of this lane (rows >= F give discarded outputs)
#pragma unroll
  for (int ks = 0; ks < M::KS; ++ks) {
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    if (16 * ks + 4 * q < C::E && arow < F) {
      const float4 v = *reinterpret_cast<const float4*>(X + arow * C::E + 16 * ks + 4 * q);
      a4[0] = v.x; a4[1] = v.y; a4[2] = v.z; a4[3] = v.w;
    }
    if constexpr (C::BF) {
      const float a01 = pack_bf16(a4[0], a4[1]), a23 = pack_bf16(a4[2], a4[3]);
#pragma unroll
      for (int nt = 0; nt < M::NT; ++nt)
        acc[nt] = mfma_bf16(a01, a23, w.wp[ks][0][nt], w.wp[ks][1][nt], acc[nt]);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int nt = 0; nt < M::NT; ++nt) acc[nt] = mfma_16x16x4(a4[t], w.wp[ks][t][nt], acc[nt]);
    }
  }
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) {
    const int c = 16 * nt + j;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * rt + 4 * q + r;
      // ALL_ROWS: the caller's layout has dead space for rows F .. 16 * ceil(F / 16) - 1 (no
      // per-element branch)
      if (ALL_ROWS || f < F) PR[f * C::PRS + c] = fmaxf(acc[nt][r], 0.f);
    }
  }
}

// dW[e][c] += sum_{f in tile rt} X[f][e] G[f][c] (acc[et][nt], D row = e, col = c);
// db partial: dbp[nt] += sum over this lane's 4 rows of G[f][16nt + j]
template <class C>
__device__ __forceinline__ void mfma_dw(const float* X, const float* G, int F, int rt,
                                        f32x4 (&acc)[MfmaW<C>::ET][MfmaW<C>::NT],
                                        float (&dbp)[MfmaW<C>::NT]) {
  using M = MfmaW<C>;
  const int q = lane_id() >> 4, j = lane_id() & 15;
  float xa[4][M::ET];
  float gb[4][M::NT];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int f = 16 * rt + 4 * q + t;
    const bool ok = f < F;
#pragma unroll
    for (int et = 0; et < M::ET; ++et) {
      const int e = 16 * et + j;
      xa[t][et] = (ok && e < C::E) ? X[f * C::E + e] : 0.f;
    }
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) {
      gb[t][nt] = ok ? G[f * C::PRS + 16 * nt + j] : 0.f;
      dbp[nt] += gb[t][nt];
    }
  }
  if constexpr (C::BF) {
    float xp[2][M::ET], gp[2][M::NT];
#pragma unroll
    for (int et = 0; et < M::ET; ++et) {
      xp[0][et] = pack_bf16(xa[0][et], xa[1][et]);
      xp[1][et] = pack_bf16(xa[2][et], xa[3][et]);
    }
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) {
      gp[0][nt] = pack_bf16(gb[0][nt], gb[1][nt]);
      gp[1][nt] = pack_bf16(gb[2][nt], gb[3][nt]);
    }
#pragma unroll
    for (int et = 0; et < M::ET; ++et)
#pragma unroll
      for (int nt = 0; nt < M::NT; ++nt)
        acc[et][nt] = mfma_bf16(xp[0][et], xp[1][et], gp[0][nt], gp[1][nt], acc[et][nt]);
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int et = 0; et < M::ET; ++et)
#pragma unroll
        for (int nt = 0; nt < M::NT; ++nt)
          acc[et][nt] = mfma_16x16x4(xa[t][et], gb[t][nt], acc[et][nt]);
  }
}

// dx[f][e] = sum_c G[f][c] W[e][c] for row tile rt; writes rows < F to out[f * ld + e]
// (accumulate: adds to out's contents, whose loads are issued before the MFMAs so that one
// memory round trip overlaps them instead of one per row)
template <class C>
__device__ __forceinline__ void mfma_dx(const float* G, int F, int rt, const MfmaW<C>& w,
                                        float* out, int ld, bool accumulate) {
  using M = MfmaW<C>;
  const int q = lane_id() >> 4, j = lane_id() & 15;
  float prev[M::ET][4];
#pragma unroll
  for (int et = 0; et < M::ET; ++et)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * rt + 4 * q + r, e = 16 * et + j;
      prev[et][r] = (accumulate && f < F && e < C::E) ? out[f * ld + e] : 0.f;
    }
  f32x4 acc[M::ET];
#pragma unroll
  for (int et = 0; et < M::ET; ++et) acc[et] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = 16 * rt + j;
#pragma unroll
  for (int cs = 0; cs < M::CS; ++cs) {
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    if (arow < F) {
      const float4 v = *reinterpret_cast<const float4*>(G + arow * C::PRS + 16 * cs + 4 * q);
      a4[0] = v.x; a4[1] = v.y; a4[2] = v.z; a4[3] = v.w;
    }
    if constexpr (C::BF) {
      const float a01 = pack_bf16(a4[0], a4[1]), a23 = pack_bf16(a4[2], a4[3]);
#pragma unroll
      for (int et = 0; et < M::ET; ++et)
        acc[et] = mfma_bf16(a01, a23, w.wx[cs][0][et], w.wx[cs][1][et], acc[et]);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int et = 0; et < M::ET; ++et) acc[et] = mfma_16x16x4(a4[t], w.wx[cs][t][et], acc[et]);
    }
  }
#pragma unroll
  for (int et = 0; et < M::ET; ++et) {
    const int e = 16 * et + j;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * rt + 4 * q + r;
      if (f < F && e < C::E) out[f * ld + e] = acc[et][r] + prev[et][r];
    }
  }
}

// dx of row tile rt as in mfma_dx, but pushed into the sparse gradient table: for each row f,
// grad_table[rows[f]][e] += dx[f][e] (+ base[f * E + e] when base != NULL: the deep tower's share
// of dL/dx0 written earlier) with float atomics, and flag[rows[f]] = -2 (scan-mode mark).
// This replaces the store of dx0 and the separate push kernel that re-read it.  The row indices
// and base values are loaded before the MFMAs (one overlapped round trip, not two per row).
template <class C>
__device__ __forceinline__ void mfma_dx_push(const float* G, int F, int rt, const MfmaW<C>& w,
                                             const float* base, const int32_t* rows,
                                             float* table, int32_t* flag) {
  using M = MfmaW<C>;
  const int q = lane_id() >> 4, j = lane_id() & 15;
  int32_t rw[4];
  float bv[M::ET][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int f = 16 * rt + 4 * q + r;
    rw[r] = f < F ? rows[f] : -1;
#pragma unroll
    for (int et = 0; et < M::ET; ++et) {
      const int e = 16 * et + j;
      bv[et][r] = (base && f < F && e < C::E) ? base[f * C::E + e] : 0.f;
    }
  }
  f32x4 acc[M::ET];
#pragma unroll
  for (int et = 0; et < M::ET; ++et) acc[et] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int arow = 16 * rt + j;
#pragma unroll
  for (int cs = 0; cs < M::CS; ++cs) {
    float a4[4] = {0.f, 0.f, 0.f, 0.f};
    if (arow < F) {
      const float4 v = *reinterpret_cast<const float4*>(G + arow * C::PRS + 16 * cs + 4 * q);
      a4[0] = v.x; a4[1] = v.y; a4[2] = v.z; a4[3] = v.w;
    }
    if constexpr (C::BF) {
      const float a01 = pack_bf16(a4[0], a4[1]), a23 = pack_bf16(a4[2], a4[3]);
#pragma unroll
      for (int et = 0; et < M::ET; ++et)
        acc[et] = mfma_bf16(a01, a23, w.wx[cs][0][et], w.wx[cs][1][et], acc[et]);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int et = 0; et < M::ET; ++et) acc[et] = mfma_16x16x4(a4[t], w.wx[cs][t][et], acc[et]);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int32_t row = rw[r];
    if (row >= 0) {  // f >= F and rows < 0 (invalid ids) push nothing
      if (j == 0) scan_mark(flag, row);
      float* dst = table + (int64_t)row * C::E;
#pragma unroll
      for (int et = 0; et < M::ET; ++et) {
        const int e = 16 * et + j;
        if (e < C::E) atomicAdd(dst + e, acc[et][r] + bv[et][r]);
      }
    }
  }
}

// dx of ALL row tiles of the sample at once (one wave owns the sample): the tiles' MFMA chains
// (and, with RS_IL_DX_KH > 1, k parts of each tile) run as independent accumulators, then each
// result goes to `emit(rt, et, r, f, e, value)`
// (rt, et, r compile-time after unrolling: per-lane arrays indexed by them stay in registers).
// Summation per k part in c order, parts added in order -- fixed, deterministic.
template <class C, class Emit, bool ALL_ROWS = false>
__device__ __forceinline__ void mfma_dx_all(const float* G, int F, const MfmaW<C>& w, Emit emit) {
  using M = MfmaW<C>;
  constexpr int NRT = (C::FMAX + 15) / 16;
#ifndef RS_IL_DX_KH
#define RS_IL_DX_KH 1
#endif
  constexpr int KH = M::CS % RS_IL_DX_KH == 0 ? RS_IL_DX_KH : 1;  // independent k parts
  constexpr int CSH = M::CS / KH;
  const int q = lane_id() >> 4, j = lane_id() & 15;
  f32x4 acc[NRT][KH][M::ET];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int kh = 0; kh < KH; ++kh)
#pragma unroll
      for (int et = 0; et < M::ET; ++et) acc[rt][kh][et] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cc = 0; cc < CSH; ++cc) {
    float a4[NRT][KH][4];
#pragma unroll
    for (int rt = 0; rt < NRT; ++rt) {
      const int arow = 16 * rt + j;
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) {
        const int cs = kh * CSH + cc;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (arow < F) v = *reinterpret_cast<const float4*>(G + arow * C::PRS + 16 * cs + 4 * q);
        a4[rt][kh][0] = v.x; a4[rt][kh][1] = v.y; a4[rt][kh][2] = v.z; a4[rt][kh][3] = v.w;
      }
    }
    if constexpr (C::BF) {
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int kh = 0; kh < KH; ++kh) {
          const float a01 = pack_bf16(a4[rt][kh][0], a4[rt][kh][1]);
          const float a23 = pack_bf16(a4[rt][kh][2], a4[rt][kh][3]);
#pragma unroll
          for (int et = 0; et < M::ET; ++et)
            acc[rt][kh][et] = mfma_bf16(a01, a23, w.wx[kh * CSH + cc][0][et],
                                        w.wx[kh * CSH + cc][1][et], acc[rt][kh][et]);
        }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
          for (int kh = 0; kh < KH; ++kh)
#pragma unroll
            for (int et = 0; et < M::ET; ++et)
              acc[rt][kh][et] = mfma_16x16x4(a4[rt][kh][t], w.wx[kh * CSH + cc][t][et], acc[rt][kh][et]);
    }
  }
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int et = 0; et < M::ET; ++et) {
      const int e = 16 * et + j;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int f = 16 * rt + 4 * q + r;
        float v = acc[rt][0][et][r];
#pragma unroll
        for (int kh = 1; kh < KH; ++kh) v += acc[rt][kh][et][r];
        if ((ALL_ROWS || f < F) && e < C::E) emit(rt, et, r, f, e, v);
      }
    }
}

// ---- phase: attention forward; optionally keeps P (pre-dropout) for backward ----------------
template <class C, bool STORE_P, bool DROP, int OSTR = C::OS, bool PK = false>
__device__ __forceinline__ void attention_fwd(const float* PR, float* O, float* PM,
                                              const Args& a, int64_t b, uint64_t lseed,
                                              float* gsave = nullptr) {
  const int lane = lane_id();
  const int F = a.F;
  for (int r0 = 0; r0 < C::H * F; r0 += 64) {
    const int r = r0 + lane;
    const bool act = r < C::H * F;
    const int h = act ? r / F : 0, i = act ? r % F : 0;
    float q[C::DH];
    load_row(q, PR + i * C::PRS + h * C::DH);
    const float* kb = PR + C::U + h * C::DH;
    // softmax(QK^T / sqrt(dh)) as exp2((QK^T) * log2(e)/sqrt(dh) - max): one multiply per score,
    // a hardware v_exp_f32 per key, one reciprocal per row (TF: exp(x - max) * (1 / sum)).
    float s[C::FMAX];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < C::FMAX; ++j) {
      const float acc = PK ? dot_row_pk(q, kb + j * C::PRS) : dot_row(q, kb + j * C::PRS);
      s[j] = (C::EXACT || j < F) ? acc * a.sc2 : -INFINITY;
      mx = fmaxf(mx, s[j]);
    }
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < C::FMAX; ++j) { s[j] = __builtin_amdgcn_exp2f(s[j] - mx); sum += s[j]; }
    const float inv = 1.0f / sum;
    float o[C::DH];
#pragma unroll
    for (int d = 0; d < C::DH; ++d) o[d] = 0.f;
    const float* vb = PR + 2 * C::U + h * C::DH;
    float* pm_row = PM + (h * F + i) * C::PMS;
#pragma unroll
    for (int j = 0; j < C::FMAX; ++j) {
      float p = s[j] * inv;
      if (STORE_P && act) pm_row[j] = p;
      if (DROP) p = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? p * a.drop_scale : 0.f;
      if constexpr (PK) axpy_row_pk(o, p, vb + j * C::PRS);
      else axpy_row(o, p, vb + j * C::PRS);
    }
    if (act) {
      float4* orow = reinterpret_cast<float4*>(O + i * OSTR + h * C::DH);
#pragma unroll
      for (int d4 = 0; d4 < C::DH / 4; ++d4)
        orow[d4] = make_float4(o[4 * d4], o[4 * d4 + 1], o[4 * d4 + 2], o[4 * d4 + 3]);
      if (gsave) {  // the saved path: O row and (max, 1/sum) for the backward (bwd4_kernel)
        float4* g = reinterpret_cast<float4*>(gsave + i * C::U + h * C::DH);
#pragma unroll
        for (int d4 = 0; d4 < C::DH / 4; ++d4)
          g[d4] = make_float4(o[4 * d4], o[4 * d4 + 1], o[4 * d4 + 2], o[4 * d4 + 3]);
        *reinterpret_cast<float2*>(gsave + F * C::U + 2 * (h * F + i)) = make_float2(mx, inv);
      }
    }
  }
}

// ---- phase: z = relu(O + R); y = LN(z).  MODE 0: write y (to LDS X or to global).
//      MODE 1 (backward recompute): keep z in O, (mean, std) per row in ST. -----------------
template <class C, int MODE, int OSTR = C::OS>
__device__ __forceinline__ void epilogue(float* O, const float* PR, float* ST, float* Y,
                                         int y_stride, const Args& a, const float (&gam)[C::CPLN],
                                         const float (&bet)[C::CPLN]) {
  const int lane = lane_id();
  const int u0 = lane % C::LPR;
  const int F = a.F;
  for (int f0 = 0; f0 < F; f0 += C::RG) {
    const int f = f0 + lane / C::LPR;
    const bool act = f < F;
    float z[C::CPLN];
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < C::CPLN; ++c) {
      const int u = u0 + c * C::LPR;
      float t = act ? O[f * OSTR + u] : 0.f;
      if (a.use_res && act) t += PR[f * C::PRS + 3 * C::U + u];
      z[c] = fmaxf(t, 0.f);
      sum += z[c];
    }
    const float mean = group_sum<C::LPR>(sum) * (1.0f / (float)C::U);
    float sq = 0.f;
#pragma unroll
    for (int c = 0; c < C::CPLN; ++c) { const float d = z[c] - mean; sq += d * d; }
    const float var = group_sum<C::LPR>(sq) * (1.0f / (float)C::U);
    const float rstd = 1.0f / sqrtf(var + a.eps);  // (x - mean) / sqrt(var + eps)
    if (act) {
#pragma unroll
      for (int c = 0; c < C::CPLN; ++c) {
        const int u = u0 + c * C::LPR;
        if (MODE == 0) Y[f * y_stride + u] = (z[c] - mean) * rstd * gam[c] + bet[c];
        else O[f * OSTR + u] = z[c];
      }
      if (MODE == 1 && u0 == 0) { ST[2 * f] = mean; ST[2 * f + 1] = rstd; }
    }
  }
}

// ============================== forward kernel ===============================================
#ifndef RS_IL_FWD_PK
#define RS_IL_FWD_PK 0  // packed-fp32 (v_pk_fma_f32) score dots / PV axpys in the forward
#endif
template <class C, bool DROP>
__global__ void __launch_bounds__(256, 4) fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ y,
    int64_t y_ld, float* __restrict__ xsave, Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);  // dropout seed of this launch
  float* base = smem + wave_id() * a.per_wave;
  float* X = base + a.l_x;
  float* PR = base + a.l_pr;
  const int lane = lane_id();
  const int wpb = blockDim.x >> 6;
  const int F = a.F;
  zero_pad_rows<C>(PR, F);
  MfmaW<C> mw;
  mw.load(W, bias);
  float gam[C::CPLN], bet[C::CPLN];
#pragma unroll
  for (int c = 0; c < C::CPLN; ++c) {
    gam[c] = gamma[lane % C::LPR + c * C::LPR];
    bet[c] = beta[lane % C::LPR + c * C::LPR];
  }
  for (int64_t b = (int64_t)blockIdx.x * wpb + wave_id(); b < a.B; b += (int64_t)gridDim.x * wpb) {
    if (a.g_table) {
      // fused gather: float4 k of the sample is quarter k % (E/4) of field k / (E/4)'s row; the
      // E/4 lanes of a field hash the same id (one cached 8-B load), lane q == 0 records the row
      constexpr int QV = C::E / 4;
      float4* xo = reinterpret_cast<float4*>(const_cast<float*>(x) + b * F * C::E);
      for (int k = lane; k < F * QV; k += 64) {
        const int f = k / QV, q = k - f * QV;
        const int64_t row = hash_row(a.g_ids[b * F + f], a.g_base[f], a.g_bucket[f], a.g_hash);
        // rows outside the table (bad row_base / bucket): a zero embedding, row index -1
        const bool ok = row >= 0 && row < a.g_table_rows;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) v = reinterpret_cast<const float4*>(a.g_table + row * C::E)[q];
        reinterpret_cast<float4*>(X)[k] = v;
        xo[k] = v;
        if (q == 0 && a.g_rows) a.g_rows[b * F + f] = ok ? (int32_t)row : -1;
      }
    } else {
      const float4* src = reinterpret_cast<const float4*>(x + b * F * C::E);
      for (int k = lane; k < F * C::E / 4; k += 64) reinterpret_cast<float4*>(X)[k] = src[k];
    }
    wave_lds_sync();
    for (int it = 0; it < a.L; ++it) {
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      for (int rt = 0; rt * 16 < F; ++rt) mfma_project<C>(X, PR, F, rt, mw);
      wave_lds_sync();
      // O_i overwrites Q_i in place (only lane (h, i) ever reads Q_i, before writing O_i)
      float* gsave = a.osave ? a.osave + ((int64_t)it * a.B + b) * small_save_stride(F, C::U, C::H)
                             : nullptr;
      attention_fwd<C, false, DROP, C::PRS, RS_IL_FWD_PK != 0>(PR, PR, nullptr, a, b, lseed, gsave);
      wave_lds_sync();
      if (it == a.L - 1) {
        epilogue<C, 0, C::PRS>(PR, PR, nullptr, y + b * y_ld, C::U, a, gam, bet);
      } else {
        epilogue<C, 0, C::PRS>(PR, PR, nullptr, X, C::E, a, gam, bet);  // E == U when L > 1
        wave_lds_sync();
        if (xsave) {
          float4* dst = reinterpret_cast<float4*>(xsave + ((int64_t)it * a.B + b) * F * C::U);
          for (int k = lane; k < F * C::U / 4; k += 64) dst[k] = reinterpret_cast<float4*>(X)[k];
        }
      }
      wave_lds_sync();
    }
  }
}

// ============================== backward kernel, v2 ===========================================
// One workgroup = one sample at a time, TWO waves sharing the sample's LDS (row-parallel phases
// split rows between the waves; attention phases keep lane = (head, row) and split the inner
// loop -- keys for the softmax / dS / dQ passes, queries for dV / dK -- the partials meeting in
// LDS regions dead in that phase; round 1's first backward, since removed, had this split with a
// separate gradient region), laid out for occupancy:
//   * no gradient region: the projection gradients overwrite Q, K, V, R in place as each input
//     dies (R after the LN backward; V after dS; K after dQ; Q after dK), dV / dQ wait in
//     TMP / DY / O meanwhile -> ~20 KB of LDS per sample instead of ~26 KB;
//   * W is not held in VGPRs across the kernel: its MFMA fragments are loaded (L1/L2 hits) in
//     the two phases that use them -> <= 128 VGPRs (4 waves per SIMD instead of 2);
//   * the forward-recompute partials exchange through ST (m, l) and TMP (o of wave 1).
// Phases per sample and iteration (barriers between them):
//   P1 projection recompute (MFMA)      P2 attention recompute (keys split), P, O
//   P3 LN + ReLU backward: O <- dt, R <- gR
//   P4 dV (queries split) -> DY         P5 dS (in place of P), dQ (keys split) -> O
//   P6 dK (queries split) -> K <- gK;  V <- gV (DY), Q <- gQ (O)
//   P7 dW, db += X^T G; dx = G W^T -> DY (next iteration's dy) or the input gradient / push
#ifndef RS_IL_BWD2_OCC
#define RS_IL_BWD2_OCC 3
#endif
template <class C, bool DROP>
__global__ void __launch_bounds__(128, RS_IL_BWD2_OCC) bwd2_kernel(
    const float* __restrict__ x, const float* __restrict__ xsave, const float* __restrict__ dy,
    int64_t dy_ld, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ dx,
    int dx_accumulate, float* __restrict__ partials, Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);  // dropout seed of this launch
  constexpr int JH = (C::FMAX + 1) / 2;  // keys (or queries) per wave in the split passes
  float* const X0 = smem + a.l_x;
  float* const X1 = smem + a.l_x2;
  float* const WL = smem + a.l_w;
  float* const BL = smem + a.l_b;
  float* PR = smem + a.l_pr;
  float* O = smem + a.l_o;
  float* DY = smem + a.l_dy;
  float* TMP = smem + a.l_tmp;
  float* PM = smem + a.l_pm;
  float* ST = smem + a.l_st;
  const int lane = lane_id();
  const int w = wave_id();  // 0 or 1
  const int F = C::EXACT ? C::FMAX : a.F;  // compile-time for exact-F shapes
  const int HF = C::H * F;
  const int j0 = w * JH;

  for (int k = F * C::PRS + threadIdx.x; k < C::FMAX * C::PRS; k += blockDim.x) PR[k] = 0.f;
  // W and bias stay in LDS for the whole kernel (the MFMA fragments are re-read per phase from
  // there instead of from L1/L2: a global round trip at the head of two phases per iteration)
  for (int k = threadIdx.x; k < C::E * C::NC; k += blockDim.x)
    WL[(k / C::NC) * C::WPS + k % C::NC] = W[k];
  for (int k = threadIdx.x; k < C::NC; k += blockDim.x) BL[k] = bias[k];
  // iteration inputs stream in asynchronously one iteration ahead (X double buffer; dy of the
  // next sample during the last iteration's dW/dx phase)
  auto x_src = [&](int64_t bb, int itx) -> const float* {
    return itx == 0 ? x + bb * F * C::E : xsave + ((int64_t)(itx - 1) * a.B + bb) * F * C::U;
  };
  auto load_dy = [&](int64_t bb) {
    const float* src = dy + bb * dy_ld;
    if (a.dy_vec) glds_copy(DY, src, F * C::U / 4);
    else for (int k = threadIdx.x; k < F * C::U; k += blockDim.x) DY[k] = src[k];
  };
  if ((int64_t)blockIdx.x < a.B) {
    glds_copy(X0, x_src(blockIdx.x, a.L - 1), F * C::E / 4);
    load_dy(blockIdx.x);
  }
  int par = 0;

  using M = MfmaW<C>;
  f32x4 dwacc[M::ET][M::NT];
  float dbp[M::NT];
#pragma unroll
  for (int et = 0; et < M::ET; ++et)
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) dwacc[et][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) dbp[nt] = 0.f;
  float dg[C::CPLN], dbt[C::CPLN], gam[C::CPLN];
  const int u0 = lane % C::LPR;
#pragma unroll
  for (int c = 0; c < C::CPLN; ++c) { dg[c] = 0.f; dbt[c] = 0.f; gam[c] = gamma[u0 + c * C::LPR]; }
  const int nrt = (F + 15) / 16;

  IL_STAMP_DECL
  for (int64_t b = blockIdx.x; b < a.B; b += gridDim.x) {
    for (int it = a.L - 1; it >= 0; --it) {
      IL_STAMP(0)
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      float* const X = par ? X1 : X0;
      vm_wait_all();  // this wave's share of X (and of dy at it == L-1) has landed
      lds_barrier();
      {  // prefetch the next iteration's input into the other buffer
        const int64_t bn = it > 0 ? b : b + gridDim.x;
        if (bn < a.B) glds_copy(par ? X0 : X1, x_src(bn, it > 0 ? it - 1 : a.L - 1), F * C::E / 4);
      }
      IL_STAMP(1)
      // ---- P1: projections (row tiles split between the waves) ----
      {
        // launder W / bias so the fragment loads are NOT hoisted out of the sample loop (they
        // would then stay live in 36 VGPRs across every phase): reloading them costs a few
        // L1 hits per iteration, keeping them costs two waves per SIMD
        MfmaW<C> mw;
        mw.load_proj_lds(WL, BL);
        for (int rt = w; rt < nrt; rt += 2) mfma_project<C>(X, PR, F, rt, mw);
      }
      lds_barrier();
      IL_STAMP(2)
      // ---- P2: attention recompute, keys split; m / l through ST, wave 1's o through TMP ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, i = act ? r % F : 0;
        float q[C::DH];
        load_row(q, PR + i * C::PRS + h * C::DH);
        const float* kb = PR + C::U + h * C::DH;
        float s[JH];
        float mx = -INFINITY;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj) {
          const int j = j0 + jj;
          const float acc = (j < C::FMAX) ? dot_row(q, kb + j * C::PRS) : 0.f;
          s[jj] = (j < F) ? acc * a.sc2 : -INFINITY;
          mx = fmaxf(mx, s[jj]);
        }
        if (act) ST[w * HF + r] = mx;
        lds_barrier();
        const float m = act ? fmaxf(ST[r], ST[HF + r]) : 0.f;
        float l = 0.f;
        float o[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) o[d] = 0.f;
        const float* vb = PR + 2 * C::U + h * C::DH;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj) {
          const int j = j0 + jj;
          s[jj] = __builtin_amdgcn_exp2f(s[jj] - m);
          l += s[jj];
          float e = s[jj];
          if (DROP && j < F) e = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? e * a.drop_scale : 0.f;
          if (j < C::FMAX) axpy_row(o, e, vb + j * C::PRS);
        }
        if (act) {
          ST[(2 + w) * HF + r] = l;
          if (w == 1) {
#pragma unroll
            for (int d = 0; d < C::DH; ++d) TMP[d * HF + r] = o[d];
          }
        }
        lds_barrier();
        if (act) {
          const float inv = 1.0f / (ST[2 * HF + r] + ST[3 * HF + r]);
          float* pm_row = PM + (h * F + i) * C::PMS;
#pragma unroll
          for (int jj = 0; jj < JH; ++jj)
            if (j0 + jj < C::FMAX) pm_row[j0 + jj] = s[jj] * inv;
          if (w == 0) {
            float ov[C::DH];
#pragma unroll
            for (int d = 0; d < C::DH; ++d) ov[d] = (o[d] + TMP[d * HF + r]) * inv;
            store_row(O + i * C::OS + h * C::DH, ov);
          }
        }
        lds_barrier();
      }
      IL_STAMP(3)
      // ---- P3: z = relu(O + R), LN stats, LN + ReLU backward (rows split):
      //      O <- dt; R <- gR = dt * (R > 0) (R dies here) ----
      {
        for (int f0 = w * C::RG; f0 < F; f0 += 2 * C::RG) {
          const int f = f0 + lane / C::LPR;
          const bool act = f < F;
          float z[C::CPLN], rr[C::CPLN];
          float sum = 0.f;
#pragma unroll
          for (int c = 0; c < C::CPLN; ++c) {
            const int u = u0 + c * C::LPR;
            float t = act ? O[f * C::OS + u] : 0.f;
            rr[c] = (a.use_res && act) ? PR[f * C::PRS + 3 * C::U + u] : 0.f;
            t += rr[c];
            z[c] = fmaxf(t, 0.f);
            sum += z[c];
          }
          const float mean = group_sum<C::LPR>(sum) * (1.0f / (float)C::U);
          float sq = 0.f;
#pragma unroll
          for (int c = 0; c < C::CPLN; ++c) { const float d = z[c] - mean; sq += d * d; }
          const float var = group_sum<C::LPR>(sq) * (1.0f / (float)C::U);
          const float rstd = 1.0f / sqrtf(var + a.eps);
          float zh[C::CPLN], g[C::CPLN];
          float sg = 0.f, sgz = 0.f;
#pragma unroll
          for (int c = 0; c < C::CPLN; ++c) {
            const int u = u0 + c * C::LPR;
            zh[c] = (z[c] - mean) * rstd;
            const float dyv = act ? DY[f * C::U + u] : 0.f;
            dg[c] = fmaf(dyv, zh[c], dg[c]);
            dbt[c] += dyv;
            g[c] = dyv * gam[c];
            sg += g[c];
            sgz += g[c] * zh[c];
          }
          sg = group_sum<C::LPR>(sg) * (1.0f / (float)C::U);
          sgz = group_sum<C::LPR>(sgz) * (1.0f / (float)C::U);
          if (act) {
#pragma unroll
            for (int c = 0; c < C::CPLN; ++c) {
              const int u = u0 + c * C::LPR;
              const float dz = (g[c] - sg - zh[c] * sgz) * rstd;
              const float dt = z[c] > 0.f ? dz : 0.f;  // TF ReluGrad: x > 0
              O[f * C::OS + u] = dt;
              // without use_res the R columns carry no gradient (their dW / db must be zero)
              PR[f * C::PRS + 3 * C::U + u] = (a.use_res && rr[c] > 0.f) ? dt : 0.f;
            }
          }
        }
      }
      lds_barrier();
      IL_STAMP(4)
      // ---- P4: dV_j = sum_i Pd_ij dO_i (lane = (h, j); queries split) -> DY[j][h dh + d] ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, j = act ? r % F : 0;
        float dv[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dv[d] = 0.f;
#pragma unroll 2
        for (int ii = 0; ii < JH; ++ii) {
          const int i = j0 + ii;
          if (C::EXACT ? (i < C::FMAX) : (i < F)) {
            float p = PM[(h * F + i) * C::PMS + j];
            if (DROP) p = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? p * a.drop_scale : 0.f;
            axpy_row(dv, p, O + i * C::OS + h * C::DH);
          }
        }
        if (act && w == 1) {
#pragma unroll
          for (int d = 0; d < C::DH; ++d) TMP[d * HF + r] = dv[d];
        }
        lds_barrier();
        if (act && w == 0) {
#pragma unroll
          for (int d = 0; d < C::DH; ++d) dv[d] += TMP[d * HF + r];
          store_row(DY + j * C::U + h * C::DH, dv);
        }
        lds_barrier();
      }
      IL_STAMP(5)
      // ---- P5: dS (in place of P) and dQ (lane = (h, i); keys split) -> O (dO dies here) ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, i = act ? r % F : 0;
        float dO[C::DH];
        load_row(dO, O + i * C::OS + h * C::DH);
        const float* vb = PR + 2 * C::U + h * C::DH;
        const float* kb = PR + C::U + h * C::DH;
        float* pm_row = PM + (h * F + i) * C::PMS;
        float s[JH];
        float Dw = 0.f;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj) {
          const int j = j0 + jj;
          float dp = (j < C::FMAX) ? dot_row(dO, vb + j * C::PRS) : 0.f;
          if (DROP && j < F) dp = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? dp * a.drop_scale : 0.f;
          const float p = (j < C::FMAX) ? pm_row[j] : 0.f;
          Dw = fmaf(p, dp, Dw);
          s[jj] = dp;
        }
        if (act) ST[w * HF + r] = Dw;
        lds_barrier();
        const float D = act ? ST[r] + ST[HF + r] : 0.f;
        float dq[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dq[d] = 0.f;
#pragma unroll
        for (int jj = 0; jj < JH; ++jj) {
          const int j = j0 + jj;
          if (j < C::FMAX) {
            const float ds = pm_row[j] * (s[jj] - D) * a.inv_sdh;
            axpy_row(dq, ds, kb + j * C::PRS);
            if (act) pm_row[j] = ds;
          }
        }
        if (act && w == 1) {
#pragma unroll
          for (int d = 0; d < C::DH; ++d) TMP[d * HF + r] = dq[d];
        }
        lds_barrier();
        if (act && w == 0) {
#pragma unroll
          for (int d = 0; d < C::DH; ++d) dq[d] += TMP[d * HF + r];
          store_row(O + i * C::OS + h * C::DH, dq);
        }
        lds_barrier();
      }
      IL_STAMP(6)
      // ---- P6: dK_j = sum_i dS_ij Q_i (lane = (h, j); queries split); then K <- gK (wave 0),
      //      V <- gV from DY and Q <- gQ from O (wave 1) ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, j = act ? r % F : 0;
        float dk[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dk[d] = 0.f;
#pragma unroll 2
        for (int ii = 0; ii < JH; ++ii) {
          const int i = j0 + ii;
          if (C::EXACT ? (i < C::FMAX) : (i < F))
            axpy_row(dk, PM[(h * F + i) * C::PMS + j], PR + i * C::PRS + h * C::DH);
        }
        if (act && w == 1) {
#pragma unroll
          for (int d = 0; d < C::DH; ++d) TMP[d * HF + r] = dk[d];
        }
        lds_barrier();
        if (act && w == 0) {
          float kr[C::DH], pt[C::DH];
          load_row(kr, PR + j * C::PRS + C::U + h * C::DH);
#pragma unroll
          for (int d = 0; d < C::DH; ++d) pt[d] = TMP[d * HF + r];  // unconditional: no branches
#pragma unroll
          for (int d = 0; d < C::DH; ++d) kr[d] = kr[d] > 0.f ? dk[d] + pt[d] : 0.f;
          store_row(PR + j * C::PRS + C::U + h * C::DH, kr);
        }
        if (w == 1 && r0 + 64 >= HF) {  // once, after the last row chunk's dK reads of Q
          for (int k = lane; k < F * C::U; k += 64) {
            const int f = k / C::U, c = k % C::U;
            float* vq = PR + f * C::PRS + 2 * C::U + c;
            float* qq = PR + f * C::PRS + c;
            const float gv = DY[k], gq = O[f * C::OS + c];  // unconditional loads, then select
            const float v0 = *vq, q0 = *qq;
            *vq = v0 > 0.f ? gv : 0.f;
            *qq = q0 > 0.f ? gq : 0.f;
          }
        }
        lds_barrier();
      }
      IL_STAMP(7)
      // ---- P7: dW += X^T G, db += colsum G; dx = G W^T (row tiles split; MFMA) ----
      for (int rt = w; rt < nrt; rt += 2) mfma_dw<C>(X, PR, F, rt, dwacc, dbp);
      __builtin_amdgcn_sched_barrier(0);  // keep the dx pass's loads out of the dW pass
      {
        MfmaW<C> mw;
        mw.load_dx_lds(WL);
        for (int rt = w; rt < nrt; rt += 2) {
          if (it > 0) mfma_dx<C>(PR, F, rt, mw, DY, C::U, false);  // dL/d(previous output)
          else if (a.push_table)
            mfma_dx_push<C>(PR, F, rt, mw, dx_accumulate ? dx + b * F * C::E : nullptr,
                            a.push_rows + b * F, a.push_table, a.push_flag);
          else mfma_dx<C>(PR, F, rt, mw, dx + b * F * C::E, C::E, dx_accumulate != 0);
        }
      }
      // the next sample's dy (DY is dead after P6 at it == 0); issued after the push's own
      // loads so that their waits do not also wait for this copy
      if (it == 0 && b + gridDim.x < a.B) load_dy(b + gridDim.x);
      lds_barrier();
      IL_STAMP(8)
      par ^= 1;
    }
  }
  vm_wait_all();
  IL_STAMP_FLUSH(a.stamps)

  // ---- lanes -> wave -> block (wave order) ----
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) {
    dbp[nt] += __shfl_xor(dbp[nt], 16, 64);
    dbp[nt] += __shfl_xor(dbp[nt], 32, 64);
  }
#pragma unroll
  for (int c = 0; c < C::CPLN; ++c) {
#pragma unroll
    for (int o = C::LPR; o < 64; o <<= 1) {
      dg[c] += __shfl_xor(dg[c], o, 64);
      dbt[c] += __shfl_xor(dbt[c], o, 64);
    }
  }
  float* RED = smem;
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x) RED[k] = 0.f;
  __syncthreads();
  {
    const int q = lane >> 4, jx = lane & 15;
    for (int ww = 0; ww < 2; ++ww) {
      if (w == ww) {
#pragma unroll
        for (int et = 0; et < M::ET; ++et)
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int e = 16 * et + 4 * q + r;
              if (e < C::E) RED[e * C::NC + 16 * nt + jx] += dwacc[et][nt][r];
            }
        if (q == 0) {
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt) RED[C::E * C::NC + 16 * nt + jx] += dbp[nt];
        }
        if (lane < C::LPR) {
#pragma unroll
          for (int c = 0; c < C::CPLN; ++c) {
            const int u = u0 + c * C::LPR;
            RED[C::E * C::NC + C::NC + u] += dg[c];
            RED[C::E * C::NC + C::NC + C::U + u] += dbt[c];
          }
        }
      }
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x)
    partials[(int64_t)blockIdx.x * C::NPARAM + k] = RED[k];
}

// ============================== backward kernel, v3 ===========================================
// One wave = one sample at a time, kWpb3 waves (samples) per block sharing the block-resident W
// and bias in LDS.  Every phase is wave-local: no workgroup barrier and no partial-row exchange
// inside the sample loop (v2's 17 barriers and split-j exchanges per sample-iteration were where
// its waves parked), at the price of 2 waves per SIMD (LDS: ~18 KB per sample).  The next
// iteration's input rows and the next sample's dy rows are prefetched into registers while the
// current iteration runs, and written to LDS at the next iteration's start.
//   P1 projections (MFMA, both row tiles)      P2 attention recompute (lane = (head, row),
//   P3 LN + ReLU backward (O <- dt, R <- gR)       every key; P stored pre-dropout)
//   P4 dV (lane = (head, key)) -> DY           P5 dS (in place of P), dQ -> O
//   P6 dK -> K <- gK; V <- gV, Q <- gQ         P7 dW, db += X^T G; dx = G W^T (-> DY / push)
constexpr int kWpb3 = 4;

// P3 can form D_i = dO_i . O_i per head when a head's columns sit in whole lane groups of the
// LN epilogue mapping (DH <= LPR, LPR % DH == 0)
template <class C>
constexpr bool kDRowDot = C::DH <= C::LPR && C::LPR % C::DH == 0;

// P3 with lane = (row, head) when H == 2 and the rows fit one pass: each lane owns one head's DH
// columns of one row, so the LN sums need one DPP step (the row's other head) instead of
// log2(LPR) per sum, D_i is lane-local, and the row's loads/stores are float4s
template <class C>
constexpr bool kLnPair = C::H == 2 && C::DH % 4 == 0 && C::DH <= 16 && C::FMAX <= 32;

template <class C>
struct Bwd3Layout {
  // per-wave region (floats): XA | XB | PR (FMAX rows) | DY | PM | ST (the fused push's table
  // rows).  XA / XB alternate as X (this iteration's input rows, stride E) and O (attention
  // output, stride OS): once O is dead (after P6) the next iteration's input streams into it
  // (global_load_lds, no registers) while P7 runs, and the two swap.
  int xa, xb, pr, dy, pm, st, per_wave;
  __host__ __device__ Bwd3Layout(int F) {
    const int xo = ((F * C::E > F * C::OS ? F * C::E : F * C::OS) + 3) & ~3;
    int off = 0;
    xa = off; off += xo;
    xb = off; off += xo;
    pr = off; off += (C::FMAX * C::PRS + 3) & ~3;
    dy = off; off += (F * C::U + 3) & ~3;
    pm = off; off += (C::H * F * C::PMS + 3) & ~3;
    st = off; off += (2 * F + 3) & ~3;
    per_wave = off;
  }
  static constexpr int shared_floats() {  // W [E][WPS] | bias [NC] | gamma [U]
    return ((C::E * C::WPS + 3) & ~3) + ((C::NC + 3) & ~3) + ((C::U + 3) & ~3);
  }
};

// n4 float4 of a global row block -> registers (PF float4 per lane) / registers -> LDS
template <int PF>
__device__ __forceinline__ void row_prefetch(float4 (&r)[PF], const float* src, int n4) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int i = lane + 64 * k;
    if (i < n4) r[k] = reinterpret_cast<const float4*>(src)[i];
  }
}

template <int PF>
__device__ __forceinline__ void row_commit(float* dst, const float4 (&r)[PF], int n4) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int i = lane + 64 * k;
    if (i < n4) reinterpret_cast<float4*>(dst)[i] = r[k];
  }
}

template <class C, bool DROP>
#ifndef RS_IL_BWD3_OCC
#define RS_IL_BWD3_OCC 2
#endif
__global__ void __launch_bounds__(64 * kWpb3, RS_IL_BWD3_OCC) bwd3_kernel(
    const float* __restrict__ x, const float* __restrict__ xsave, const float* __restrict__ dy,
    int64_t dy_ld, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ dx,
    int dx_accumulate, float* __restrict__ partials, Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);  // dropout seed of this launch
  const int F = C::EXACT ? C::FMAX : a.F;
  const Bwd3Layout<C> lay(F);
  float* const WL = smem;
  float* const BL = smem + ((C::E * C::WPS + 3) & ~3);
  float* const base = smem + Bwd3Layout<C>::shared_floats() + wave_id() * lay.per_wave;
  float* X = base + lay.xa;
  float* const PR = base + lay.pr;
  float* O = base + lay.xb;
  float* const DY = base + lay.dy;
  float* const PM = base + lay.pm;
  float* const ST = base + lay.st;
  const int lane = lane_id();
  const int w = wave_id();
  const int HF = C::H * F;
  const int nrt = (F + 15) / 16;

  for (int k = threadIdx.x; k < C::E * C::NC; k += blockDim.x)
    WL[(k / C::NC) * C::WPS + k % C::NC] = W[k];
  for (int k = threadIdx.x; k < C::NC; k += blockDim.x) BL[k] = bias[k];
  float* const GL = BL + ((C::NC + 3) & ~3);
  for (int k = threadIdx.x; k < C::U; k += blockDim.x) GL[k] = gamma[k];
  zero_pad_rows<C>(PR, F);
  __syncthreads();  // the only workgroup barrier before the final reduction

  using M = MfmaW<C>;
  f32x4 dwacc[M::ET][M::NT];
  float dbp[M::NT];
#pragma unroll
  for (int et = 0; et < M::ET; ++et)
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) dwacc[et][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) dbp[nt] = 0.f;
  float dg[C::CPLN], dbt[C::CPLN], gam[C::CPLN];
  const int u0 = lane % C::LPR;
#pragma unroll
  for (int c = 0; c < C::CPLN; ++c) { dg[c] = 0.f; dbt[c] = 0.f; gam[c] = gamma[u0 + c * C::LPR]; }
  float dg2[C::DH], dbt2[C::DH];  // kLnPair: this lane's head columns (lane & 1), all its rows
#pragma unroll
  for (int d = 0; d < C::DH; ++d) { dg2[d] = 0.f; dbt2[d] = 0.f; }

  const int nx4 = F * C::E / 4, ny4 = F * C::U / 4;
  auto x_src = [&](int64_t bb, int itx) -> const float* {
    return itx == 0 ? x + bb * F * C::E : xsave + ((int64_t)(itx - 1) * a.B + bb) * F * C::U;
  };
  // wave w of block k starts at sample k + w * grid: below 4 * grid samples the active waves
  // spread over every block (every CU) instead of filling the first blocks (bwd3_grid)
  const int64_t b_first = (int64_t)blockIdx.x + (int64_t)gridDim.x * w;
  const int64_t b_step = (int64_t)gridDim.x * kWpb3;
  if (b_first < a.B) {  // the first sample's input rows and dy (dy_vec: rows 16-B aligned)
    glds_copy_wave(X, x_src(b_first, a.L - 1), nx4);
    glds_copy_wave(DY, dy + b_first * dy_ld, ny4);
  }

  IL_STAMP_DECL
  for (int64_t b = b_first; b < a.B; b += b_step) {
    for (int it = a.L - 1; it >= 0; --it) {
      IL_STAMP(0)
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      // fused push (it == 0): this sample's table rows, parked in ST (unused by v3) after P1,
      // so the push at the end of the iteration reads them from LDS
      vm_wait_all();  // X (and DY at it == L-1) streamed in by the previous iteration
      int32_t rowv = -1;
      const bool push_rows_now = it == 0 && a.push_table != nullptr;
      if (push_rows_now && lane < F) rowv = a.push_rows[b * F + lane];
      wave_lds_sync();
      IL_STAMP(1)
      // ---- P1: projections ----
      {
        MfmaW<C> mw;
        mw.load_proj_lds(WL, BL);
        for (int rt = 0; rt < nrt; ++rt) mfma_project<C>(X, PR, F, rt, mw);
      }
      if (push_rows_now && lane < F) reinterpret_cast<int32_t*>(ST)[lane] = rowv;
      wave_lds_sync();
      IL_STAMP(2)
      // ---- P2: attention recompute; P (pre-dropout) -> PM, O ----
      attention_fwd<C, true, DROP, C::OS, true>(PR, O, PM, a, b, lseed);
      wave_lds_sync();
      IL_STAMP(3)
      // ---- P3: z = relu(O + R), LN stats, LN + ReLU backward: O <- dt; R <- gR ----
      if constexpr (kLnPair<C>) {
        const int ln = lane_id(), f = ln >> 1, h = ln & 1;
        const bool act = f < F;
        const int fr = act ? f : 0;
        float oa[C::DH], rr[C::DH], dyv[C::DH], gm[C::DH], z[C::DH];
        load_row(oa, O + fr * C::OS + h * C::DH);
        load_row(rr, PR + fr * C::PRS + 3 * C::U + h * C::DH);
        load_row(dyv, DY + fr * C::U + h * C::DH);
        load_row(gm, GL + h * C::DH);
        float sum = 0.f;
#pragma unroll
        for (int d = 0; d < C::DH; ++d) {
          if (!a.use_res) rr[d] = 0.f;
          if (!act) dyv[d] = 0.f;
          z[d] = fmaxf(oa[d] + rr[d], 0.f);
          sum += z[d];
        }
        const float mean = group_sum<2>(sum) * (1.0f / (float)C::U);
        float sq = 0.f;
#pragma unroll
        for (int d = 0; d < C::DH; ++d) { const float t = z[d] - mean; sq += t * t; }
        const float var = group_sum<2>(sq) * (1.0f / (float)C::U);
        const float rstd = 1.0f / sqrtf(var + a.eps);
        float sg = 0.f, sgz = 0.f;
#pragma unroll
        for (int d = 0; d < C::DH; ++d) {
          const float zh = (z[d] - mean) * rstd;
          dg2[d] = fmaf(dyv[d], zh, dg2[d]);
          dbt2[d] += dyv[d];
          const float g = dyv[d] * gm[d];
          sg += g;
          sgz += g * zh;
          rr[d] = z[d] > 0.f ? 1.f : 0.f;  // ReLU mask of z (TF ReluGrad: x > 0)
          z[d] = zh;
          gm[d] = g;
        }
        sg = group_sum<2>(sg) * (1.0f / (float)C::U);
        sgz = group_sum<2>(sgz) * (1.0f / (float)C::U);
        float dt[C::DH];
        float dd = 0.f;
#pragma unroll
        for (int d = 0; d < C::DH; ++d) {
          const float dz = (gm[d] - sg - z[d] * sgz) * rstd;
          dt[d] = rr[d] != 0.f ? dz : 0.f;
          dd = fmaf(oa[d], dt[d], dd);
        }
        if (act) {
          // gR = dt where the residual projection R > 0 (its own ReLU)
          float rv[C::DH], gr[C::DH];
          load_row(rv, PR + f * C::PRS + 3 * C::U + h * C::DH);
#pragma unroll
          for (int d = 0; d < C::DH; ++d) gr[d] = (a.use_res && rv[d] > 0.f) ? dt[d] : 0.f;
          store_row(O + f * C::OS + h * C::DH, dt);
          store_row(PR + f * C::PRS + 3 * C::U + h * C::DH, gr);
          // D_{h,f} = dO_f . O_f over head h (see kDRowDot), lane-local here
          PM[(h * F + f) * C::PMS + C::FMAX] = dd;
        }
      } else
      for (int f0 = 0; f0 < F; f0 += C::RG) {
        const int f = f0 + lane / C::LPR;
        const bool act = f < F;
        float z[C::CPLN], rr[C::CPLN], oa[C::CPLN];
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < C::CPLN; ++c) {
          const int u = u0 + c * C::LPR;
          float t = act ? O[f * C::OS + u] : 0.f;
          oa[c] = t;  // the attention output (for D below)
          rr[c] = (a.use_res && act) ? PR[f * C::PRS + 3 * C::U + u] : 0.f;
          t += rr[c];
          z[c] = fmaxf(t, 0.f);
          sum += z[c];
        }
        const float mean = group_sum<C::LPR>(sum) * (1.0f / (float)C::U);
        float sq = 0.f;
#pragma unroll
        for (int c = 0; c < C::CPLN; ++c) { const float d = z[c] - mean; sq += d * d; }
        const float var = group_sum<C::LPR>(sq) * (1.0f / (float)C::U);
        const float rstd = 1.0f / sqrtf(var + a.eps);
        float zh[C::CPLN], g[C::CPLN];
        float sg = 0.f, sgz = 0.f;
#pragma unroll
        for (int c = 0; c < C::CPLN; ++c) {
          const int u = u0 + c * C::LPR;
          zh[c] = (z[c] - mean) * rstd;
          const float dyv = act ? DY[f * C::U + u] : 0.f;
          dg[c] = fmaf(dyv, zh[c], dg[c]);
          dbt[c] += dyv;
          g[c] = dyv * gam[c];
          sg += g[c];
          sgz += g[c] * zh[c];
        }
        sg = group_sum<C::LPR>(sg) * (1.0f / (float)C::U);
        sgz = group_sum<C::LPR>(sgz) * (1.0f / (float)C::U);
#pragma unroll
        for (int c = 0; c < C::CPLN; ++c) {
          const int u = u0 + c * C::LPR;
          const float dz = (g[c] - sg - zh[c] * sgz) * rstd;
          const float dt = z[c] > 0.f ? dz : 0.f;  // TF ReluGrad: x > 0
          if (act) {
            O[f * C::OS + u] = dt;
            PR[f * C::PRS + 3 * C::U + u] = (a.use_res && rr[c] > 0.f) ? dt : 0.f;
          }
          if constexpr (kDRowDot<C>) {
            // D_{h,f} = sum_j P_fj dP_fj = dO_f . O_f over head h's columns (O = sum_j Pd_fj V_j,
            // dropout included), reduced over the DH lanes of the head: P5 then needs one pass
            // over the keys instead of two.  Parked in PM's pad column FMAX of row (h, f).
            const float dd = group_sum<C::DH>(oa[c] * dt);
            if (act && u % C::DH == 0) PM[((u / C::DH) * F + f) * C::PMS + C::FMAX] = dd;
          }
        }
      }
      wave_lds_sync();
      IL_STAMP(4)
      // ---- P4: dV_j = sum_i Pd_ij dO_i (lane = (h, j)) -> DY[j][h dh + d] ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, j = act ? r % F : 0;
        float dv[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dv[d] = 0.f;
#pragma unroll 4
        for (int i = 0; i < F; ++i) {
          float p = PM[(h * F + i) * C::PMS + j];
          if (DROP) p = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? p * a.drop_scale : 0.f;
          axpy_row_pk(dv, p, O + i * C::OS + h * C::DH);
        }
        if (act) store_row(DY + j * C::U + h * C::DH, dv);
      }
      wave_lds_sync();
      IL_STAMP(5)
      // ---- P5: dS (in place of P) and dQ (lane = (h, i)) -> O ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, i = act ? r % F : 0;
        float dO[C::DH];
        load_row(dO, O + i * C::OS + h * C::DH);
        const float* vb = PR + 2 * C::U + h * C::DH;
        const float* kb = PR + C::U + h * C::DH;
        float* pm_row = PM + (h * F + i) * C::PMS;
        // D_i from P3 (kDRowDot) and one pass over the keys; otherwise two passes (dP_ij
        // recomputed in the second) rather than a dP row in registers: 26 live dP values per lane
        // pushed v3 past 256 VGPRs into scratch
        float D = 0.f;
        if constexpr (kDRowDot<C>) {
          D = pm_row[C::FMAX];  // from P3
        } else {
#pragma unroll 2
          for (int j = 0; j < F; ++j) {
            float dp = dot_row_pk(dO, vb + j * C::PRS);
            if (DROP) dp = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? dp * a.drop_scale : 0.f;
            D = fmaf(pm_row[j], dp, D);
          }
        }
        float dq[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dq[d] = 0.f;
#pragma unroll 2
        for (int j = 0; j < F; ++j) {
          float dp = dot_row_pk(dO, vb + j * C::PRS);
          if (DROP) dp = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? dp * a.drop_scale : 0.f;
          const float ds = pm_row[j] * (dp - D) * a.inv_sdh;
          axpy_row_pk(dq, ds, kb + j * C::PRS);
          if (act) pm_row[j] = ds;
        }
        if (act) store_row(O + i * C::OS + h * C::DH, dq);  // dO_i (read above) dies here
      }
      wave_lds_sync();
      IL_STAMP(6)
      // ---- P6: dK_j = sum_i dS_ij Q_i (lane = (h, j)); K <- gK ----
      for (int r0 = 0; r0 < HF; r0 += 64) {
        const int r = r0 + lane;
        const bool act = r < HF;
        const int h = act ? r / F : 0, j = act ? r % F : 0;
        float dk[C::DH];
#pragma unroll
        for (int d = 0; d < C::DH; ++d) dk[d] = 0.f;
#pragma unroll 4
        for (int i = 0; i < F; ++i) axpy_row_pk(dk, PM[(h * F + i) * C::PMS + j], PR + i * C::PRS + h * C::DH);
        float kr[C::DH];
        load_row(kr, PR + j * C::PRS + C::U + h * C::DH);
#pragma unroll
        for (int d = 0; d < C::DH; ++d) kr[d] = kr[d] > 0.f ? dk[d] : 0.f;
        // every lane's K reads (here) precede any K write of the same row: row j is read only
        // by lane (h, j) in this pass
        if (act) store_row(PR + j * C::PRS + C::U + h * C::DH, kr);
      }
      wave_lds_sync();  // all dK reads of Q done
      for (int k = lane; k < F * C::U; k += 64) {  // V <- gV (DY), Q <- gQ (O)
        const int f = k / C::U, c = k % C::U;
        float* vq = PR + f * C::PRS + 2 * C::U + c;
        float* qq = PR + f * C::PRS + c;
        const float gv = DY[k], gq = O[f * C::OS + c];
        const float v0 = *vq, q0 = *qq;
        *vq = v0 > 0.f ? gv : 0.f;
        *qq = q0 > 0.f ? gq : 0.f;
      }
      wave_lds_sync();
      {  // O is dead: stream the next iteration's input rows into it (and at it == 0, when DY is
         // dead too, the next sample's dy) while P7 runs
        const int64_t bn = it > 0 ? b : b + b_step;
        if (bn < a.B) {
          glds_copy_wave(O, x_src(bn, it > 0 ? it - 1 : a.L - 1), nx4);
          if (it == 0) glds_copy_wave(DY, dy + bn * dy_ld, ny4);
        }
      }
      IL_STAMP(7)
      // ---- P7: dW += X^T G, db += colsum G; dx = G W^T ----
      // fused push with the head's share (dx_base): its values for this lane's (row, col)
      // slots, loaded before the dW MFMAs so dW + dx cover the round trip
      constexpr int NRT7 = (C::FMAX + 15) / 16;
      float bv[NRT7][M::ET][4];
      if (it == 0 && a.push_table && dx_accumulate) {
        const float* base_g = dx + b * F * C::E;
        // lane re-derived (laundered): keeps LLVM from turning the 8 slot addresses into
        // loop-carried pointers over b (they were spilled to scratch)
        const int ln = lane_id(), q = ln >> 4, jx = ln & 15;
#pragma unroll
        for (int rt = 0; rt < NRT7; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int et = 0; et < M::ET; ++et) {
              const int f = 16 * rt + 4 * q + r, e = 16 * et + jx;
              bv[rt][et][r] = (f < F && e < C::E) ? base_g[f * C::E + e] : 0.f;
            }
      } else {
#pragma unroll
        for (int rt = 0; rt < NRT7; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int et = 0; et < M::ET; ++et) bv[rt][et][r] = 0.f;
      }
      for (int rt = 0; rt < nrt; ++rt) mfma_dw<C>(X, PR, F, rt, dwacc, dbp);
      __builtin_amdgcn_sched_barrier(0);
      IL_STAMP(8)
      {
        MfmaW<C> mw;
        mw.load_dx_lds(WL);
        if (it > 0) {  // dL/d(previous output) -> DY
          mfma_dx_all<C>(PR, F, mw, [&](int, int, int, int f, int e, float v) { DY[f * C::U + e] = v; });
        } else if (a.push_table) {
          // fused sparse push: row index and the head's share loaded before the MFMAs; rows
          // f >= F and rows < 0 (ids outside the table) push nothing
          constexpr int NRT = (C::FMAX + 15) / 16;
          const int q = lane >> 4, jx = lane & 15;
          int32_t rw[NRT][4];
          const int32_t* rows = reinterpret_cast<const int32_t*>(ST);  // parked after P1
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int f = 16 * rt + 4 * q + r;
              rw[rt][r] = f < F ? rows[f] : -1;
            }
          (void)jx;
          mfma_dx_all<C>(PR, F, mw, [&](int rt, int et, int r, int, int e, float v) {
            const int32_t row = rw[rt][r];
            if (row >= 0) {
              if (e == 0) scan_mark(a.push_flag, row);
              atomicAdd(a.push_table + (int64_t)row * C::E + e, v + bv[rt][et][r]);
            }
          });
        } else {
          float* d = dx + b * F * C::E;
          if (dx_accumulate)
            mfma_dx_all<C>(PR, F, mw, [&](int, int, int, int f, int e, float v) { d[f * C::E + e] += v; });
          else
            mfma_dx_all<C>(PR, F, mw, [&](int, int, int, int f, int e, float v) { d[f * C::E + e] = v; });
        }
      }
      wave_lds_sync();
      if (it > 0) { IL_STAMP(9) } else { IL_STAMP(10) }  // dx -> DY / dx -> push (it == 0)
      float* const t = X;  // the next iteration's input is in O's buffer
      X = O;
      O = t;
    }
  }
  IL_STAMP_FLUSH(a.stamps)

  // ---- lanes -> wave -> block (wave order 0..kWpb3-1): deterministic ----
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) {
    dbp[nt] += __shfl_xor(dbp[nt], 16, 64);
    dbp[nt] += __shfl_xor(dbp[nt], 32, 64);
  }
  if constexpr (kLnPair<C>) {  // lanes of one head parity hold the same columns
#pragma unroll
    for (int d = 0; d < C::DH; ++d)
#pragma unroll
      for (int o = 2; o < 64; o <<= 1) {
        dg2[d] += __shfl_xor(dg2[d], o, 64);
        dbt2[d] += __shfl_xor(dbt2[d], o, 64);
      }
  } else {
#pragma unroll
    for (int c = 0; c < C::CPLN; ++c) {
#pragma unroll
      for (int o = C::LPR; o < 64; o <<= 1) {
        dg[c] += __shfl_xor(dg[c], o, 64);
        dbt[c] += __shfl_xor(dbt[c], o, 64);
      }
    }
  }
  __syncthreads();
  float* RED = smem;  // W / per-wave regions are dead now
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x) RED[k] = 0.f;
  __syncthreads();
  {
    const int q = lane >> 4, jx = lane & 15;
    for (int ww = 0; ww < kWpb3; ++ww) {
      if (w == ww) {
#pragma unroll
        for (int et = 0; et < M::ET; ++et)
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int e = 16 * et + 4 * q + r;
              if (e < C::E) RED[e * C::NC + 16 * nt + jx] += dwacc[et][nt][r];
            }
        if (q == 0) {
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt) RED[C::E * C::NC + 16 * nt + jx] += dbp[nt];
        }
        if constexpr (kLnPair<C>) {
          if (lane < 2) {
#pragma unroll
            for (int d = 0; d < C::DH; ++d) {
              const int u = lane * C::DH + d;
              RED[C::E * C::NC + C::NC + u] += dg2[d];
              RED[C::E * C::NC + C::NC + C::U + u] += dbt2[d];
            }
          }
        } else if (lane < C::LPR) {
#pragma unroll
          for (int c = 0; c < C::CPLN; ++c) {
            const int u = u0 + c * C::LPR;
            RED[C::E * C::NC + C::NC + u] += dg[c];
            RED[C::E * C::NC + C::NC + C::U + u] += dbt[c];
          }
        }
      }
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x)
    partials[(int64_t)blockIdx.x * C::NPARAM + k] = RED[k];
}

// v3 fits when kWpb3 sample regions + W give 2 blocks per CU; otherwise v2 runs
template <class C>
__host__ __forceinline__ size_t bwd3_lds_bytes(int F) {
  return ((size_t)Bwd3Layout<C>::shared_floats() + (size_t)kWpb3 * Bwd3Layout<C>(F).per_wave) * 4;
}

// ============================== backward kernel, v4 (saved path) ===============================
// rs_il_bwd_saved / rs_il_bwd_push_saved for F <= 32 with two heads: the forward wrote, per
// (iteration, sample), the attention output O and the softmax row stats (scaled max, 1 / sum)
// (small_save_stride).  With O known, the LN + ReLU backward runs right after the projections,
// so dO and D_i = dO_i . O_i are known before the attention backward, and the attention backward
// needs two passes over the keys instead of v3's four (recompute, dV, dS/dQ, dK):
//   Q-pass, lane = (head, query i), one sweep over the keys j:
//     P_ij = exp2(q_i . k_j * log2e / sqrt(dh) - max_i) / sum_i   (saved stats: no max/sum pass)
//     dP_ij = dO_i . v_j ;  dS_ij = P_ij (dP_ij - D_i) / sqrt(dh) ;  dq_i += dS_ij k_j
//     (P_ij parked in PM for the K-pass; dq_i to DY)
//   K-pass, lane = (head, key j), one sweep over the queries i:
//     dv_j += Pd_ij dO_i ;  dS_ij recomputed from P_ij and dP_ij = dO_i . v_j (v_j in registers,
//     the same fma order as the Q-pass, so the same value) ;  dk_j += dS_ij q_i
// Per sample-iteration that is 4 LDS row reads per key instead of v3's 12, and no PV product.
// Buffers per wave: BA / BB alternate as X (the iteration's input) and S (the saved O | stats;
// after the LN backward it holds dO).  The X operand of dW is taken into registers right after
// the projections, so BA takes the next iteration's save straight away (global_load_lds) and BB
// the next iteration's input once dO is dead (after the K-pass).  The fused push's row indices
// and the head's dx share are fetched at the start of iteration 0 by loads the compiler does not
// track, and waited for with an explicit vmcnt that leaves the younger prefetches in flight.
template <class C>
constexpr bool kSaved4 = kLnPair<C> && C::H * C::FMAX <= 64;
// unroll of the two key sweeps (a full unroll of 26 keys lets the scheduler hoist every LDS row
// read and spills)
#ifndef RS_IL4_EXP
#define RS_IL4_EXP 0
#endif
#ifndef RS_IL4_WREG
#define RS_IL4_WREG 0
#endif
#ifndef RS_IL4_UNROLL_Q
#define RS_IL4_UNROLL_Q 2
#endif
#ifndef RS_IL4_UNROLL_K
#define RS_IL4_UNROLL_K 2
#endif
#define RS_PRAGMA_(x) _Pragma(#x)
#define RS_UNROLL(n) RS_PRAGMA_(unroll n)

// RS_IL4_ROT (round 6): three rotating buffers instead of two + DY, so the next iteration's input
// is issued right after the LN backward (when the dy it replaces is consumed) instead of after the
// K-pass; dq stays in registers through the K-pass; the push rows come to registers
#ifndef RS_IL4_ROT
#define RS_IL4_ROT 1
#endif
// static priority (cdna guide "two waves per SIMD", item 4): the wave in an odd SIMD slot runs at
// s_setprio 1, so the two co-resident waves stop trading VALU issue slot by slot (same box, 300
// steps x 3: IL backward 78.4 -> 77.9 us, profiles/r06/rot/)
#ifndef RS_IL4_PRIO
#define RS_IL4_PRIO 1
#endif
// RS_IL4_MQ (round 6, opt-in): the Q-pass's score, dP and dq products on the matrix cores (f32,
// no dropout, two heads of dh = 8, F <= 32, three rotating buffers).  Correct (the whole GPU
// suite, 338 tests, passed with it on) but SLOWER: same box, 300 steps x 2, the backward launch
// 77.6 / 78.1 -> 90.4 / 90.2 us (0.1456 / 0.1482 -> 0.1579 / 0.1587 ms per step); one
// accumulator per key tile (RS_IL4_MQ_SPLIT) 92.3 / 91.3 us (profiles/r06/mq/).  Each 16 x 16
// tile is a dependent chain (S / dP MFMAs -> exp / dS on the VALU -> 4 dq MFMAs) with 37 % of
// the tile padding (26 of 32 rows and keys) and the dq^T tile half padding (dh 8 of 16 rows),
// and the 16 packed dq registers held through the K-pass push the kernel past 256 VGPRs (148 B
// of scratch); the VALU pass's per-lane key loop keeps two waves per SIMD issuing instead.
#ifndef RS_IL4_MQ
#define RS_IL4_MQ 0
#endif
#ifndef RS_IL4_MQ_SPLIT
#define RS_IL4_MQ_SPLIT 0
#endif
template <class C, bool DROP>
constexpr bool kMQ = RS_IL4_MQ && RS_IL4_ROT && !DROP && !C::BF && C::H == 2 && C::DH == 8 &&
                     C::FMAX <= 32;
template <class C>
struct Bwd4Layout {
  int ba, bb, bc, pr, dy, pm, st, rows, sv, per_wave;
  __host__ __device__ Bwd4Layout(int F) {
    sv = (int)small_save_stride(F, C::U, C::H);
    const int xe = F * C::E;
    const int f16 = (F + 15) & ~15;
    int xo = ((xe > sv ? xe : sv) + 3) & ~3;
#if RS_IL4_ROT
    // a buffer also takes the dx rows of iterations > 0 (exact F: all 16 * ceil(F / 16) rows)
    const int dyr = (C::EXACT ? f16 : F) * C::U;
    if (xo < dyr) xo = (dyr + 3) & ~3;
#endif
    int off = 0;
    ba = off; off += xo;
    bb = off; off += xo;
#if RS_IL4_ROT
    bc = off; off += xo;
#else
    bc = 0;
#endif
    // PR's rows F .. 16 * ceil(F / 16) - 1 (written by the unguarded projection stores) land in
    // PM, dead at the projections; DY's (the dx rows of iterations > 0) land in ST / RW / pad,
    // dead in P7 of those iterations
    pr = off; off += (C::FMAX * C::PRS + 3) & ~3;
    pm = off; off += (C::H * F * C::PMS + 3) & ~3;
#if RS_IL4_ROT
    dy = 0;
    st = off; off += (C::H * F + 3) & ~3;     // D_i per (head, row)
    rows = off; off += (F + 3) & ~3;          // the Q-pass's dead-lane P stores
#else
    dy = off; off += (F * C::U + 3) & ~3;
    st = off; off += (C::H * F + 3) & ~3;     // D_i per (head, row)
    rows = off; off += (F + 3) & ~3;          // the fused push's table rows (int32)
    const int dy_slack = C::EXACT ? (f16 - F) * C::U - (off - dy - F * C::U) : 0;
    if (dy_slack > 0) off += (dy_slack + 3) & ~3;
#endif
    per_wave = off;
  }
};

template <class C>
__host__ __forceinline__ size_t bwd4_lds_bytes(int F) {
  return ((size_t)Bwd3Layout<C>::shared_floats() + (size_t)kWpb3 * Bwd4Layout<C>(F).per_wave) * 4;
}

#ifndef RS_IL4_PK  // 0: the same even / odd accumulator pairs as scalar v_fma_f32 (tuning builds)
#define RS_IL4_PK 1
#endif
// init: the even chain's starting value (a bias folded into the dot for free)
template <int N>
__device__ __forceinline__ float dot_reg_pk(const float (&a)[N], const float (&b)[N],
                                            float init = 0.f) {
  if constexpr (!RS_IL4_PK) {
    float e = init, o = 0.f;
#pragma unroll
    for (int d = 0; d < N; d += 2) { e = fmaf(a[d], b[d], e); o = fmaf(a[d + 1], b[d + 1], o); }
    return e + o;
  }
  f32x2v acc = {init, 0.f};
#pragma unroll
  for (int d = 0; d < N; d += 2)
    acc = __builtin_elementwise_fma(f32x2v{a[d], a[d + 1]}, f32x2v{b[d], b[d + 1]}, acc);
  return acc.x + acc.y;
}

// two independent dot products, their packed-fma chains interleaved (back-to-back dependent
// v_pk_fma_f32 need a wait state between them)
template <int N>
__device__ __forceinline__ void dot2_reg_pk(const float (&a)[N], const float (&b)[N],
                                            const float (&c)[N], const float (&d)[N], float& ab,
                                            float& cd, float ab0 = 0.f, float cd0 = 0.f) {
  if constexpr (!RS_IL4_PK) {
    ab = dot_reg_pk(a, b, ab0);
    cd = dot_reg_pk(c, d, cd0);
    return;
  }
  f32x2v x = {ab0, 0.f}, y = {cd0, 0.f};
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    x = __builtin_elementwise_fma(f32x2v{a[k], a[k + 1]}, f32x2v{b[k], b[k + 1]}, x);
    y = __builtin_elementwise_fma(f32x2v{c[k], c[k + 1]}, f32x2v{d[k], d[k + 1]}, y);
  }
  ab = x.x + x.y;
  cd = y.x + y.y;
}

template <int N>
__device__ __forceinline__ void axpy_reg_pk(float (&o)[N], float p, const float (&v)[N]) {
  if constexpr (!RS_IL4_PK) {
#pragma unroll
    for (int d = 0; d < N; ++d) o[d] = fmaf(p, v[d], o[d]);
    return;
  }
  const f32x2v pp = {p, p};
#pragma unroll
  for (int d = 0; d < N; d += 2) {
    const f32x2v r = __builtin_elementwise_fma(pp, f32x2v{v[d], v[d + 1]}, f32x2v{o[d], o[d + 1]});
    o[d] = r.x; o[d + 1] = r.y;
  }
}

// dW += X^T G over row tile rt with the X operand already in registers (xa[t][et] = X[16rt+4q+t]
// [16et+j], as mfma_dw loads it)
template <class C>
__device__ __forceinline__ void mfma_dw_xreg(const float (&xa)[4][MfmaW<C>::ET], const float* G,
                                             int F, int rt,
                                             f32x4 (&acc)[MfmaW<C>::ET][MfmaW<C>::NT],
                                             float (&dbp)[MfmaW<C>::NT]) {
  using M = MfmaW<C>;
  const int q = lane_id() >> 4, j = lane_id() & 15;
  float gb[4][M::NT];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int f = 16 * rt + 4 * q + t;
    const bool ok = f < F;
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) {
      gb[t][nt] = ok ? G[f * C::PRS + 16 * nt + j] : 0.f;
      dbp[nt] += gb[t][nt];
    }
  }
  if constexpr (C::BF) {
    float xp[2][M::ET], gp[2][M::NT];
#pragma unroll
    for (int et = 0; et < M::ET; ++et) {
      xp[0][et] = pack_bf16(xa[0][et], xa[1][et]);
      xp[1][et] = pack_bf16(xa[2][et], xa[3][et]);
    }
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) {
      gp[0][nt] = pack_bf16(gb[0][nt], gb[1][nt]);
      gp[1][nt] = pack_bf16(gb[2][nt], gb[3][nt]);
    }
#pragma unroll
    for (int et = 0; et < M::ET; ++et)
#pragma unroll
      for (int nt = 0; nt < M::NT; ++nt)
        acc[et][nt] = mfma_bf16(xp[0][et], xp[1][et], gp[0][nt], gp[1][nt], acc[et][nt]);
  } else {
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int et = 0; et < M::ET; ++et)
#pragma unroll
        for (int nt = 0; nt < M::NT; ++nt)
          acc[et][nt] = mfma_16x16x4(xa[t][et], gb[t][nt], acc[et][nt]);
  }
}

// glds wave instructions a copy of n4 float4 (n words) issues
__host__ __device__ constexpr int glds_instrs4(int n4) { return (n4 + 63) / 64; }

template <class C, bool DROP>
#ifndef RS_IL_BWD4_OCC
#define RS_IL_BWD4_OCC 2
#endif
__global__ void __launch_bounds__(64 * kWpb3, RS_IL_BWD4_OCC) bwd4_kernel(
    const float* __restrict__ x, const float* __restrict__ xsave, const float* __restrict__ dy,
    int64_t dy_ld, const float* __restrict__ W, const float* __restrict__ bias,
    const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ dx,
    int dx_accumulate, float* __restrict__ partials, Args a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  static_assert(kSaved4<C>, "bwd4 needs H == 2, F <= 32 (one lane per (head, row))");
  // PR's unguarded rows up to the next multiple of 16 must fit in PM (Bwd4Layout); the
  // non-exact instantiations (FMAX 32) have no such rows
  static_assert(!C::EXACT ||
                (((C::FMAX + 15) & ~15) - C::FMAX) * C::PRS <= C::H * C::FMAX * C::PMS,
                "PM too small for PR's padded rows");
  static_assert(C::EXACT || C::FMAX % 16 == 0, "non-exact FMAX must be a multiple of 16");
  const uint64_t seed0 = rs_eff_seed(a.seed, a.seed_off);
  const int F = C::EXACT ? C::FMAX : a.F;
  const Bwd4Layout<C> lay(F);
  float* const WL = smem;
  float* const BL = smem + ((C::E * C::WPS + 3) & ~3);
  float* const GL = BL + ((C::NC + 3) & ~3);
  float* const base = smem + Bwd3Layout<C>::shared_floats() + wave_id() * lay.per_wave;
  float* XB = base + lay.ba;  // this iteration's input X
  float* SB = base + lay.bb;  // this iteration's save: O | stats, then dO
  float* const PR = base + lay.pr;
#if RS_IL4_ROT
  float* DY = base + lay.bc;  // this iteration's dy, then (after P3) the next iteration's X
#else
  float* const DY = base + lay.dy;
#endif
  float* const PM = base + lay.pm;
  float* const DL = base + lay.st;
  int32_t* const RW = reinterpret_cast<int32_t*>(base + lay.rows);
  const int lane = lane_id();
  const int w = wave_id();
  constexpr int H = C::H, DH = C::DH, U = C::U;
  const int HF = H * F;
  const int nrt = (F + 15) / 16;
  const int sv = lay.sv;

  for (int k = threadIdx.x; k < C::E * C::NC; k += blockDim.x)
    WL[(k / C::NC) * C::WPS + k % C::NC] = W[k];
  for (int k = threadIdx.x; k < C::NC; k += blockDim.x) BL[k] = bias[k];
  for (int k = threadIdx.x; k < C::U; k += blockDim.x) GL[k] = gamma[k];
  zero_pad_rows<C>(PR, F);
  __syncthreads();

  using M = MfmaW<C>;
  constexpr int NRT = (C::FMAX + 15) / 16;
  f32x4 dwacc[M::ET][M::NT];
  float dbp[M::NT];
#pragma unroll
  for (int et = 0; et < M::ET; ++et)
#pragma unroll
    for (int nt = 0; nt < M::NT; ++nt) dwacc[et][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) dbp[nt] = 0.f;
  float dg2[DH], dbt2[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) { dg2[d] = 0.f; dbt2[d] = 0.f; }

  const int nx4 = F * C::E / 4, ny4 = F * U / 4, ns4 = sv / 4;
  auto x_src = [&](int64_t bb, int itx) -> const float* {
    return itx == 0 ? x + bb * F * C::E : xsave + ((int64_t)(itx - 1) * a.B + bb) * F * U;
  };
  auto s_src = [&](int64_t bb, int itx) -> const float* {
    return a.osave_in + ((int64_t)itx * a.B + bb) * sv;
  };
  // wave w of block k starts at sample k + w * grid: below 4 * grid samples the active waves
  // spread over every block (every CU) instead of filling the first blocks (bwd3_grid)
  const int64_t b_first = (int64_t)blockIdx.x + (int64_t)gridDim.x * w;
  const int64_t b_step = (int64_t)gridDim.x * kWpb3;
  if (b_first < a.B) {
    glds_copy_wave(XB, x_src(b_first, a.L - 1), nx4);
    glds_copy_wave(SB, s_src(b_first, a.L - 1), ns4);
    glds_copy_wave(DY, dy + b_first * dy_ld, ny4);
  }
  xt_wave_jobs(a, (int64_t)blockIdx.x * kWpb3 + w, (int64_t)gridDim.x * kWpb3);
  // the fused push's share of the head (dx_accumulate): 4 rows x ET columns per row tile
  const bool push = a.push_table != nullptr;
  const bool with_base = push && dx_accumulate;
#if RS_IL4_WREG
  MfmaW<C> mwp;  // the projection fragments stay in registers for the whole kernel
  mwp.load_proj_lds(WL, BL);
#endif

#if RS_IL4_PRIO
  {  // static priority for the wave in an odd SIMD slot (its co-resident partner keeps 0)
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    if (hw & 1u) __builtin_amdgcn_s_setprio(1);
  }
#endif
  IL_STAMP_DECL
  for (int64_t b = b_first; b < a.B; b += b_step) {
    for (int it = a.L - 1; it >= 0; --it) {
      IL_STAMP(0)
      const uint64_t lseed = splitmix64(seed0 + (uint64_t)it);
      const int64_t bn = it > 0 ? b : b + b_step;  // the next iteration's sample
      const int itn = it > 0 ? it - 1 : a.L - 1;
      const bool has_next = bn < a.B;
      vm_wait_all();  // X, the save (and dy) of this iteration, and the previous push's atomics
      wave_lds_sync();
      if (it == a.L - 1) { IL_STAMP(10) } else { IL_STAMP(1) }
      const bool push_now = it == 0 && push;
      float bv[NRT][M::ET][4];
#if RS_IL4_ROT
      int32_t rw[NRT][4];
#endif
      if (push_now) {
#if RS_IL4_ROT
        {
          const int q = lane >> 4;
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int f = 16 * rt + 4 * q + r;
              rw[rt][r] = __float_as_int(gload_untracked(
                  reinterpret_cast<const float*>(a.push_rows + b * F + (f < F ? f : F - 1))));
            }
        }
#else
        glds_copy_wave_u32(RW, a.push_rows + b * F, F);
#endif
        if (with_base) {
          const float* base_g = dx + b * F * C::E;
          const int q = lane >> 4, jx = lane & 15;
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int et = 0; et < M::ET; ++et)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int f = 16 * rt + 4 * q + r, e = 16 * et + jx;
                const int fc = f < F ? f : F - 1;
                bv[rt][et][r] = gload_untracked(base_g + fc * C::E + (e < C::E ? e : 0));
              }
        }
      }
      // ---- P1: projections (MFMA); dW's X operand into registers ----
      if (RS_IL4_EXP != 5) {
#if RS_IL4_WREG
        for (int rt = 0; rt < nrt; ++rt) mfma_project<C, true>(XB, PR, F, rt, mwp);
#else
        MfmaW<C> mw;
        mw.load_proj_lds(WL, BL);
        for (int rt = 0; rt < nrt; ++rt) mfma_project<C, true>(XB, PR, F, rt, mw);
#endif
      }
      float xa[NRT][4][M::ET];
      {
        const int q = lane >> 4, jx = lane & 15;
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int et = 0; et < M::ET; ++et) {
              const int f = 16 * rt + 4 * q + t, e = 16 * et + jx;
              xa[rt][t][et] = (f < F && e < C::E) ? XB[f * C::E + e] : 0.f;
            }
      }
      wave_lds_sync();  // X dead: the next iteration's save streams into its buffer
      if (has_next) glds_copy_wave(XB, s_src(bn, itn), ns4);
      IL_STAMP(2)
      // ---- P3: z = relu(O + R), LN + ReLU backward (lane = (row, head)): SB <- dO, R <- gR,
      //      D_{h,f} = dO_f . O_f over head h ----
      if (RS_IL4_EXP != 6) {
        const int f = lane >> 1, h = lane & 1;
        const bool act = f < F;
        const int fr = act ? f : 0;
        float oa[DH], rr[DH], dyv[DH], gm[DH], z[DH];
        load_row(oa, SB + fr * U + h * DH);
        load_row(rr, PR + fr * C::PRS + 3 * U + h * DH);
        load_row(dyv, DY + fr * U + h * DH);
        load_row(gm, GL + h * DH);
        float sum = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          if (!a.use_res) rr[d] = 0.f;
          if (!act) dyv[d] = 0.f;
          z[d] = fmaxf(oa[d] + rr[d], 0.f);
          sum += z[d];
        }
        const float mean = group_sum<2>(sum) * (1.0f / (float)U);
        float sq = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) { const float t = z[d] - mean; sq += t * t; }
        const float var = group_sum<2>(sq) * (1.0f / (float)U);
        const float rstd = 1.0f / sqrtf(var + a.eps);
        float sg = 0.f, sgz = 0.f;
        float gr[DH];
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          const float zh = (z[d] - mean) * rstd;
          dg2[d] = fmaf(dyv[d], zh, dg2[d]);
          dbt2[d] += dyv[d];
          const float g = dyv[d] * gm[d];
          sg += g;
          sgz += g * zh;
          gr[d] = rr[d];         // R (for its ReLU mask below)
          rr[d] = z[d] > 0.f ? 1.f : 0.f;
          z[d] = zh;
          gm[d] = g;
        }
        sg = group_sum<2>(sg) * (1.0f / (float)U);
        sgz = group_sum<2>(sgz) * (1.0f / (float)U);
        float dt[DH];
        float dd = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          const float dz = (gm[d] - sg - z[d] * sgz) * rstd;
          dt[d] = rr[d] != 0.f ? dz : 0.f;
          dd = fmaf(oa[d], dt[d], dd);
          gr[d] = (a.use_res && gr[d] > 0.f) ? dt[d] : 0.f;
        }
        if (act) {
          // dO and D stored pre-multiplied by the row's softmax 1/sum, so both key sweeps use
          // the unnormalised e_ij = exp2(s_ij - max_i) for P_ij (one multiply per score fewer)
          const float isum = SB[F * U + 2 * (h * F + f) + 1];
          store_row(PR + f * C::PRS + 3 * U + h * DH, gr);
#pragma unroll
          for (int d = 0; d < DH; ++d) dt[d] *= isum;
          store_row(SB + f * U + h * DH, dt);
          DL[h * F + f] = dd * isum;
        }
      }
      wave_lds_sync();
#if RS_IL4_ROT
      // dy consumed: its buffer takes the next iteration's input now (a Q- and K-pass ahead)
      if (has_next) glds_copy_wave(DY, x_src(bn, itn), nx4);
#endif
      IL_STAMP(3)
      // ---- Q-pass (lane = (h, i)): P -> PM, dq -> DY (ROT: dq stays in registers) ----
#if RS_IL4_ROT
      float dqk[DH];
      // MQ: dq per head, packed: lanes of group g < 2 hold query tile 0's d = 4g + r, lanes of
      // group g >= 2 query tile 1's d = 4(g - 2) + r (the dq^T accumulators' rows d >= 8 are
      // padding, so the two tiles share one register set)
      f32x4 dqm[kMQ<C, DROP> ? 2 : 1];
#endif
      if constexpr (kMQ<C, DROP>) {
        // Q-pass on the matrix cores (RS_IL4_MQ): per head and 16 x 16 (key j, query i) tile
        //   S^T = K Q^T, dP^T = V dO^T          two v_mfma_f32_16x16x4_f32 each (dh = 8; lane
        //                                       group g takes d = 2g + s in instruction s)
        //   e = exp2(S sc2 - max_i) -> PM,  dS^T = e (dP^T - D_i)    (lane (g, i): j = 4g + r)
        //   dq^T += K^T dS^T                    the dS^T accumulators ARE the B operand (register
        //                                       r <-> k-step r: key 4g + r); A = K^T, rows d < 8
        // Every K / V / Q / dO row is read once per 16 lanes (b64) instead of once per lane and
        // key (the VALU pass: 4 ds_read_b128 per key and lane).  Rows past F (PR's padded rows
        // alias PM) read as zeros; invalid (i, j) give e = dS = 0 and store nothing.
        const int g = lane >> 4, ii = lane & 15;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 dqt[2];
#pragma unroll
          for (int it = 0; it < 2; ++it) {
            f32x4 dq = {0.f, 0.f, 0.f, 0.f};
#if RS_IL4_MQ_SPLIT
            f32x4 dq1 = {0.f, 0.f, 0.f, 0.f};
#endif
            if (it < nrt) {
              const int i = 16 * it + ii;
              const bool iv = i < F;
              const int ic = iv ? i : 0;
              float2 qb = *reinterpret_cast<const float2*>(PR + ic * C::PRS + h * DH + 2 * g);
              float2 ob = *reinterpret_cast<const float2*>(SB + ic * U + h * DH + 2 * g);
              const float2 stt = *reinterpret_cast<const float2*>(SB + F * U + 2 * (h * F + ic));
              const float Dv = DL[h * F + ic];  // x 1/sum_i (P3)
              if (!iv) { qb = make_float2(0.f, 0.f); ob = qb; }
              float* pm_row = PM + (h * F + ic) * C::PMS;
#pragma unroll
              for (int jt = 0; jt < 2; ++jt) {
                if (jt >= nrt) break;
                const int ja = 16 * jt + ii;
                const bool jav = ja < F;
                const int jc = jav ? ja : 0;
                float2 ka = *reinterpret_cast<const float2*>(PR + jc * C::PRS + U + h * DH + 2 * g);
                float2 va = *reinterpret_cast<const float2*>(PR + jc * C::PRS + 2 * U + h * DH + 2 * g);
                if (!jav) { ka = make_float2(0.f, 0.f); va = ka; }
                f32x4 s = {0.f, 0.f, 0.f, 0.f}, p = {0.f, 0.f, 0.f, 0.f};
                s = mfma_16x16x4(ka.x, qb.x, s);
                p = mfma_16x16x4(va.x, ob.x, p);
                s = mfma_16x16x4(ka.y, qb.y, s);
                p = mfma_16x16x4(va.y, ob.y, p);
                // A of dq^T: K[16 jt + 4g + t][d = ii] (d < 8)
                float kt[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                  const int j = 16 * jt + 4 * g + t;
                  kt[t] = (ii < DH && j < F) ? PR[j * C::PRS + U + h * DH + ii] : 0.f;
                }
                float ds[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int j = 16 * jt + 4 * g + r;
                  const bool v = iv && j < F;
                  const float e = v ? __builtin_amdgcn_exp2f(fmaf(s[r], a.sc2, -stt.x)) : 0.f;
                  if (v) pm_row[j] = e;
                  ds[r] = e * (p[r] - Dv);
                }
#if RS_IL4_MQ_SPLIT  // one accumulator per key tile: two 4-long MFMA chains instead of one 8-long
                if (jt == 0) {
#pragma unroll
                  for (int t = 0; t < 4; ++t) dq = mfma_16x16x4(kt[t], ds[t], dq);
                } else {
#pragma unroll
                  for (int t = 0; t < 4; ++t) dq1 = mfma_16x16x4(kt[t], ds[t], dq1);
                }
#else
#pragma unroll
                for (int t = 0; t < 4; ++t) dq = mfma_16x16x4(kt[t], ds[t], dq);
#endif
              }
            }
#if RS_IL4_MQ_SPLIT
            dq += dq1;
#endif
            dqt[it] = dq;
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float t1 = __shfl_xor(dqt[1][r], 32, 64);
            dqm[kMQ<C, DROP> ? h : 0][r] = (g < 2 ? dqt[0][r] : t1) * a.inv_sdh;
          }
        }
      } else if (RS_IL4_EXP != 3) {
        const bool act = lane < HF;
        const int h = act ? lane / F : 0, i = act ? lane - h * F : 0;
        float qv[DH], dO[DH], dq[DH];
        load_row(qv, PR + i * C::PRS + h * DH);
        load_row(dO, SB + i * U + h * DH);  // x 1/sum_i (P3)
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] *= a.sc2;  // scores straight in the exp2 domain
        const float2 stt = *reinterpret_cast<const float2*>(SB + F * U + 2 * (h * F + i));
        const float D = DL[h * F + i];  // x 1/sum_i
        const float* kb = PR + U + h * DH;
        const float* vb = PR + 2 * U + h * DH;
        // lanes past H * F store their P values into DY (dead until this pass's dq stores,
        // which come after the loop in program order and cover DY[0 .. 2U)): an unconditional
        // ds_write per key instead of an exec-mask save / restore around each (ROT: into RW,
        // whose F floats nothing else uses)
#if RS_IL4_ROT
        float* pm_row = act ? PM + (h * F + i) * C::PMS : reinterpret_cast<float*>(RW);
#else
        float* pm_row = act ? PM + (h * F + i) * C::PMS : DY;
#endif
        const float nm = -stt.x;
#pragma unroll
        for (int d = 0; d < DH; ++d) dq[d] = 0.f;
        const int nj = C::EXACT ? C::FMAX : F;
        // software-pipelined by one key: the next key's K / V rows are in flight while this
        // key's products run (two register sets, unrolled by two)
        float k0[DH], v0[DH], k1[DH], v1[DH];
        auto ld = [&](float (&k)[DH], float (&v)[DH], int j) {
          load_row(k, kb + j * C::PRS);
          load_row(v, vb + j * C::PRS);
        };
        auto key = [&](int j, const float (&k)[DH], const float (&v)[DH]) {
          // sv = s_ij - max_i (-max as the dot's initial value); without dropout dp = dP_ij - D_i
          // the same way, both already x 1/sum_i
          float sv, dp;
          dot2_reg_pk(qv, k, dO, v, sv, dp, nm, DROP ? 0.f : -D);
          const float p = __builtin_amdgcn_exp2f(sv);  // e_ij; P_ij = e_ij / sum_i
          pm_row[j] = p;
          if (DROP) {
            dp = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate) ? dp * a.drop_scale : 0.f;
            dp -= D;
          }
          axpy_reg_pk(dq, p * dp, k);  // (x 1/sqrt(dh) once, after the loop)
        };
        ld(k0, v0, 0);
RS_UNROLL(RS_IL4_UNROLL_Q)
        for (int j = 0; j < nj; j += 2) {
          const bool two = (C::EXACT && C::FMAX % 2 == 0) || j + 1 < nj;
          ld(k1, v1, two ? j + 1 : j);
          key(j, k0, v0);
          ld(k0, v0, j + 2 < nj ? j + 2 : nj - 1);  // (the last one re-reads a row: unused)
          if (two) key(j + 1, k1, v1);
        }
#pragma unroll
        for (int d = 0; d < DH; ++d) dq[d] *= a.inv_sdh;
#if RS_IL4_ROT
#pragma unroll
        for (int d = 0; d < DH; ++d) dqk[d] = dq[d];
#else
        if (act) store_row(DY + i * U + h * DH, dq);
#endif
      }
      wave_lds_sync();
      IL_STAMP(4)
      // ---- K-pass (lane = (h, j)): dV, dK -> V, K slots as gV, gK ----
      if (RS_IL4_EXP != 4) {
        const bool act = lane < HF;
        const int h = act ? lane / F : 0, j = act ? lane - h * F : 0;
        float vj[DH], dv[DH], dk[DH];
        load_row(vj, PR + j * C::PRS + 2 * U + h * DH);
#pragma unroll
        for (int d = 0; d < DH; ++d) { dv[d] = 0.f; dk[d] = 0.f; }
        const float* pcol = PM + h * F * C::PMS + j;
        const float* dl = DL + h * F;
        const int ni = C::EXACT ? C::FMAX : F;
        // pipelined by one query like the Q-pass: P_ij, D_i, dO_i and Q_i of the next query in
        // flight while this one's products run
        float o0[DH], q0[DH], o1[DH], q1[DH], p0, p1, d0, d1;
        auto ld = [&](float (&o)[DH], float (&qq)[DH], float& P, float& D, int i) {
          load_row(o, SB + i * U + h * DH);
          load_row(qq, PR + i * C::PRS + h * DH);
          P = pcol[i * C::PMS];
          D = dl[i];
        };
        auto query = [&](int i, const float (&dOi)[DH], const float (&qi)[DH], float P, float D) {
          // P = e_ij, dO_i and D_i x 1/sum_i (P3): the products are P_ij dO_i and P_ij (dP - D)
          float pd = P;
          float dp = dot_reg_pk(dOi, vj, DROP ? 0.f : -D);
          if (DROP) {
            const bool keep = dropout_keep(lseed, (uint32_t)b, h, i, j, a.drop_rate);
            pd = keep ? P * a.drop_scale : 0.f;
            dp = (keep ? dp * a.drop_scale : 0.f) - D;
          }
          axpy_reg_pk(dv, pd, dOi);
          axpy_reg_pk(dk, P * dp, qi);  // (x 1/sqrt(dh) once, after the loop)
        };
        ld(o0, q0, p0, d0, 0);
RS_UNROLL(RS_IL4_UNROLL_K)
        for (int i = 0; i < ni; i += 2) {
          const bool two = (C::EXACT && C::FMAX % 2 == 0) || i + 1 < ni;
          ld(o1, q1, p1, d1, two ? i + 1 : i);
          query(i, o0, q0, p0, d0);
          ld(o0, q0, p0, d0, i + 2 < ni ? i + 2 : ni - 1);
          if (two) query(i + 1, o1, q1, p1, d1);
        }
        float kj[DH];
        load_row(kj, PR + j * C::PRS + U + h * DH);
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          dv[d] = vj[d] > 0.f ? dv[d] : 0.f;
          dk[d] = kj[d] > 0.f ? dk[d] * a.inv_sdh : 0.f;
        }
        // row j's K / V are read only by this lane in this pass
        if (act) {
          store_row(PR + j * C::PRS + 2 * U + h * DH, dv);
          store_row(PR + j * C::PRS + U + h * DH, dk);
        }
      }
      wave_lds_sync();  // every lane's Q-row reads are done
      IL_STAMP(5)
#if RS_IL4_ROT
      if constexpr (kMQ<C, DROP>) {  // Q <- gQ from the packed dq registers: lane (g, i)
        const int g = lane >> 4, ii = lane & 15, it = g >> 1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 16 * it + ii;
          if (it < nrt && i < F) {
              float4* qp = reinterpret_cast<float4*>(PR + i * C::PRS + h * DH + 4 * (g & 1));
              float4 qv = *qp;
              const f32x4 dq = dqm[kMQ<C, DROP> ? h : 0];
              qv.x = qv.x > 0.f ? dq[0] : 0.f;
              qv.y = qv.y > 0.f ? dq[1] : 0.f;
              qv.z = qv.z > 0.f ? dq[2] : 0.f;
              qv.w = qv.w > 0.f ? dq[3] : 0.f;
              *qp = qv;
          }
        }
      } else if (lane < HF) {  // Q <- gQ, lane (h, i) as in the Q-pass
        const int h = lane / F, i = lane - h * F;
        float qv[DH];
        load_row(qv, PR + i * C::PRS + h * DH);
#pragma unroll
        for (int d = 0; d < DH; ++d) qv[d] = qv[d] > 0.f ? dqk[d] : 0.f;
        store_row(PR + i * C::PRS + h * DH, qv);
      }
      wave_lds_sync();
      // dO (SB) is dead: it takes the next sample's dy (iteration 0) or this iteration's dx (P7)
      if (has_next && it == 0) glds_copy_wave(SB, dy + bn * dy_ld, ny4);
#else
      for (int k = lane; k < F * U; k += 64) {  // Q <- gQ (dq in DY)
        const int f = k / U, c = k - f * U;
        float* qq = PR + f * C::PRS + c;
        *qq = *qq > 0.f ? DY[k] : 0.f;
      }
      wave_lds_sync();
#endif
#if !RS_IL4_ROT
      // dO (SB) and dq (DY) are dead: the next iteration's input (and the next sample's dy)
      if (has_next) {
#if RS_IL4_EXP == 2
        if (it > 0)
#endif
        glds_copy_wave(SB, x_src(bn, itn), nx4);
#if RS_IL4_EXP != 2
        if (it == 0) glds_copy_wave(DY, dy + bn * dy_ld, ny4);
#endif
      }
#endif  // !RS_IL4_ROT
      IL_STAMP(6)
      // ---- P7: dW += X^T G, db += colsum G; dx = G W^T ----
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
        if (rt < nrt && RS_IL4_EXP != 7) mfma_dw_xreg<C>(xa[rt], PR, F, rt, dwacc, dbp);
      __builtin_amdgcn_sched_barrier(0);
      IL_STAMP(7)
      {
        MfmaW<C> mw;
        mw.load_dx_lds(WL);
#if RS_IL4_EXP == 1
        if (true) {
#else
        if (it > 0) {
#endif
#if RS_IL4_ROT
          float* const ndy = SB;  // the next iteration's dy buffer
#else
          float* const ndy = DY;
#endif
          auto to_dy = [&](int, int, int, int f, int e, float v) { ndy[f * U + e] = v; };
          // (exact F: all NRT * 16 rows, the ones past F land in DY's slack; otherwise the
          // tiles past ceil(F / 16) would not fit it)
          mfma_dx_all<C, decltype(to_dy), C::EXACT>(PR, F, mw, to_dy);
        } else if (push) {
          // the rows (and the head's share) were fetched at the start of this iteration; the
          // prefetches issued since (the next save, input and dy) stay in flight
          if (has_next) {
            constexpr int kYoung = C::EXACT
                ? glds_instrs4((int)(((C::FMAX * C::U + 2 * C::H * C::FMAX + 3) & ~3) / 4)) +
                      glds_instrs4(C::FMAX * C::E / 4) + glds_instrs4(C::FMAX * C::U / 4)
                : 3;
            asm volatile("s_waitcnt vmcnt(%0)" :: "n"(kYoung) : "memory");
          } else {
            vm_wait_all();
          }
          // the asm loads' registers: tie them to the wait (no use may move above it)
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int et = 0; et < M::ET; ++et)
#pragma unroll
              for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(bv[rt][et][r]));
          const int q = lane >> 4;
#if RS_IL4_ROT
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              asm volatile("" : "+v"(rw[rt][r]));
              if (16 * rt + 4 * q + r >= F) rw[rt][r] = -1;
            }
#else
          wave_lds_sync();  // RW landed in LDS
          int32_t rw[NRT][4];
#pragma unroll
          for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int f = 16 * rt + 4 * q + r;
              rw[rt][r] = f < F ? RW[f] : -1;
            }
#endif
          mfma_dx_all<C>(PR, F, mw, [&](int rt, int et, int r, int, int e, float v) {
            const int32_t row = rw[rt][r];
            if (row >= 0) {
              if (e == 0) scan_mark(a.push_flag, row);
              atomicAdd(a.push_table + (int64_t)row * C::E + e, with_base ? v + bv[rt][et][r] : v);
            }
          });
        } else {
          float* d = dx + b * F * C::E;
          if (dx_accumulate)
            mfma_dx_all<C>(PR, F, mw, [&](int, int, int, int f, int e, float v) { d[f * C::E + e] += v; });
          else
            mfma_dx_all<C>(PR, F, mw, [&](int, int, int, int f, int e, float v) { d[f * C::E + e] = v; });
        }
      }
      wave_lds_sync();
      if (it > 0) { IL_STAMP(8) } else { IL_STAMP(9) }
#if RS_IL4_ROT
      float* const t = XB;  // XB holds the next save, DY the next input, SB the next dy
      XB = DY;
      DY = SB;
      SB = t;
#else
      float* const t = XB;  // XB holds the next save, SB the next input
      XB = SB;
      SB = t;
#endif
    }
  }

  IL_STAMP_FLUSH(a.stamps)
  // ---- lanes -> wave -> block (wave order 0..kWpb3-1): deterministic ----
#pragma unroll
  for (int nt = 0; nt < M::NT; ++nt) {
    dbp[nt] += __shfl_xor(dbp[nt], 16, 64);
    dbp[nt] += __shfl_xor(dbp[nt], 32, 64);
  }
#pragma unroll
  for (int d = 0; d < DH; ++d)
#pragma unroll
    for (int o = 2; o < 64; o <<= 1) {
      dg2[d] += __shfl_xor(dg2[d], o, 64);
      dbt2[d] += __shfl_xor(dbt2[d], o, 64);
    }
  __syncthreads();
  float* RED = smem;
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x) RED[k] = 0.f;
  __syncthreads();
  {
    const int q = lane >> 4, jx = lane & 15;
    for (int ww = 0; ww < kWpb3; ++ww) {
      if (w == ww) {
#pragma unroll
        for (int et = 0; et < M::ET; ++et)
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int e = 16 * et + 4 * q + r;
              if (e < C::E) RED[e * C::NC + 16 * nt + jx] += dwacc[et][nt][r];
            }
        if (q == 0) {
#pragma unroll
          for (int nt = 0; nt < M::NT; ++nt) RED[C::E * C::NC + 16 * nt + jx] += dbp[nt];
        }
        if (lane < 2) {
#pragma unroll
          for (int d = 0; d < DH; ++d) {
            const int u = lane * DH + d;
            RED[C::E * C::NC + C::NC + u] += dg2[d];
            RED[C::E * C::NC + C::NC + C::U + u] += dbt2[d];
          }
        }
      }
      __syncthreads();
    }
  }
  for (int k = threadIdx.x; k < C::NPARAM; k += blockDim.x)
    partials[(int64_t)blockIdx.x * C::NPARAM + k] = RED[k];
}

// ---- one workgroup per sample (il_wide.hpp) -------------------------------------------------
// Kernel variant (rs_il_set_variant, process-wide like the math mode, read when a launch is
// issued): 0 = auto, 1 = the per-sample-wave kernels (fwd_kernel / bwd4_kernel), 2 = the wide
// kernels wherever they apply.
enum { RS_IL_VARIANT_AUTO = 0, RS_IL_VARIANT_WAVE = 1, RS_IL_VARIANT_WIDE = 2 };
int rs_il_variant_now();
}  // namespace rs_il
#include "il_wide.hpp"
namespace rs_il {
// grids: one workgroup per sample up to these, then persistent workgroups looping over samples
// (the backward's grid is also the number of per-block partial rows)
// the forward runs one workgroup per sample up to 4096 samples: ~6 resident per CU (78 VGPRs),
// so a 2048-workgroup grid at B = 4096 left a second round of 512 workgroups with 2 samples each
// (same box, 200 steps: 0.1542 -> 0.1508 ms per step; 1536: 0.1535; 1024: 0.1575)
constexpr int kWideFwdGrid = 4096;
// tuning runs: RS_IL_WIDE_FWD_GRID overrides the forward's persistent grid (read once)
inline int64_t wide_fwd_grid() {
  static const int64_t g = [] {
    const char* e = getenv("RS_IL_WIDE_FWD_GRID");
    const long v = e ? atol(e) : 0L;
    return (int64_t)(v >= 64 && v <= 65536 ? v : kWideFwdGrid);
  }();
  return g;
}
constexpr int kWideBwdGrid = 1024;
// auto: the wide forward everywhere (B = 512: 10.1 vs 19.9 us, 4096: 34.6 vs 34.1 us, same-box
// HIP events); the wide backward up to this batch (512: 22.7 vs 31.2 us, 1024: 36 vs 40.5 us; at
// 4096 it is throughput-bound at 111 vs 78 us: the one-wave kernel keeps its sweeps' key
// addresses wave-uniform and needs no cross-wave exchange), profiles/r04_wide_sb
constexpr int64_t kWideBwdAutoMaxB = 1536;

// one resident round of v3 blocks on MI355X (2 per CU x 256 CUs); callers size the per-block
// partial rows with rs_il_bwd_partial_blocks, which applies the same rule
constexpr int kBwd3Grid = 512;
// v3 / v4 grid: one block per sample up to kBwd3Grid samples (one active wave per block, the
// blocks spread over every CU -- B = 512 runs one wave on each of 512 SIMDs instead of four per
// CU on 128 CUs), then kBwd3Grid blocks whose waves take every (grid)th sample
__host__ __forceinline__ int64_t bwd3_grid(int64_t B) { return B < kBwd3Grid ? B : kBwd3Grid; }

// grid-level reduction of the per-block partials, fixed order (deterministic); interacting.hip
void reduce_params(hipStream_t s, const float* partials, int nblocks, int nparam, float* out,
                   int accumulate);

// ---------------------------------------------------------------------------------------------
template <class C, bool DROP>
int fwd_launch(const FwdReq& q) {
  if (q.F > C::FMAX) return RS_ERR_UNSUPPORTED;
  Args a = make_args<C>(q.B, q.F, q.L, q.use_res, q.eps, q.drop_rate, q.seed, false);
  a.g_ids = q.gather_ids;
  a.g_base = q.gather_base;
  a.g_bucket = q.gather_bucket;
  a.g_table = q.gather_table;
  a.g_table_rows = q.gather_table_rows;
  a.g_rows = q.gather_rows;
  a.g_hash = q.gather_hash;
  if constexpr (kSaved4<C>) a.osave = q.asave;  // the saved path's O + softmax stats
  if constexpr (kWide<C>) {
    if (rs_il_variant_now() != RS_IL_VARIANT_WAVE) {
      const size_t lds = (size_t)WideFwdLayout<C>().total * sizeof(float);
      const int64_t gmax = wide_fwd_grid();
      const int64_t grid = q.B < gmax ? q.B : gmax;
      if (grid == 0) return RS_OK;
      wfwd_kernel<C, DROP><<<(int)grid, kWideThreads, lds, q.stream>>>(
          q.x, q.W, q.bias, q.gamma, q.beta, q.y, q.y_ld, q.xsave, a);
      return rs_status_after_launch();
    }
  }
  const size_t per_wave = (size_t)a.per_wave * sizeof(float);
  int wpb = (int)(kLdsBytes / per_wave);
  if (wpb > kMaxFwdWaves) wpb = kMaxFwdWaves;
  if (wpb < 1) return RS_ERR_UNSUPPORTED;
  // small batches: fewer waves per block so the samples spread over >= 512 blocks (all CUs)
  // instead of filling B / wpb blocks
  if (q.B < (int64_t)kFwdSpreadBlocks * wpb) {
    const int64_t w = q.B / kFwdSpreadBlocks;
    wpb = w < 1 ? 1 : (int)w;
  }
  int64_t grid = (q.B + wpb - 1) / wpb;
  if (grid > 4096) grid = 4096;
  if (grid == 0) return RS_OK;
  fwd_kernel<C, DROP><<<(int)grid, 64 * wpb, per_wave * wpb, q.stream>>>(
      q.x, q.W, q.bias, q.gamma, q.beta, q.y, q.y_ld, q.xsave, a);
  return rs_status_after_launch();
}

template <class C, bool DROP>
int bwd_launch(const BwdReq& q) {
  if (q.F > C::FMAX) return RS_ERR_UNSUPPORTED;
  Args a = make_args2<C>(q.B, q.F, q.L, q.use_res, q.eps, q.drop_rate, q.seed);
  a.push_rows = q.push_rows;
  a.push_table = q.push_table;
  a.push_flag = q.push_flag;
  a.dy_vec = (q.dy_ld % 4 == 0) && ((uintptr_t)q.dy % 16 == 0);
  if (q.xt_x) {
    if (!q.xt_dz || !q.xt_slab || q.xt_K0 <= 0 || q.xt_K0 % 16 || q.xt_N1 <= 0 || q.xt_N1 % 16 ||
        q.xt_ldx < q.xt_K0 || q.xt_lddz < q.xt_N1)
      return RS_ERR_ARG;
    a.xt_x = q.xt_x; a.xt_dz = q.xt_dz; a.xt_ldx = q.xt_ldx; a.xt_lddz = q.xt_lddz;
    a.xt_K0 = q.xt_K0; a.xt_N1 = q.xt_N1; a.xt_nsplit = xt_splits(q.B); a.xt_slab = q.xt_slab;
  }
  // x / xsave rows are copied 16 B at a time
  if ((uintptr_t)q.x % 16 || (q.xsave && (uintptr_t)q.xsave % 16)) return RS_ERR_ARG;
#ifndef RS_IL_BWD_NO_V3
  if constexpr (kWide<C>) {  // one workgroup per sample over the forward's save (il_wide.hpp)
    const int var = rs_il_variant_now();
    if ((var == RS_IL_VARIANT_WIDE || (var == RS_IL_VARIANT_AUTO && q.B <= kWideBwdAutoMaxB)) &&
        q.asave && a.dy_vec && q.F >= 1) {
      int64_t grid = q.B < kWideBwdGrid ? q.B : kWideBwdGrid;
      const int64_t max_grid = q.workspace_floats / C::NPARAM;
      if (grid > max_grid) grid = max_grid;
      if (q.grid_out) { *q.grid_out = (int)(grid > 0 ? grid : 0); return RS_OK; }
      if (grid <= 0) return q.B == 0 ? RS_OK : RS_ERR_ARG;
      a.osave_in = q.asave;
      wbwd_kernel<C, DROP><<<(int)grid, kWideThreads, wbwd_lds_bytes<C>(q.F), q.stream>>>(
          q.x, q.xsave, q.dy, q.dy_ld, q.W, q.bias, q.gamma, q.beta, q.dx, q.dx_accumulate,
          q.workspace, a);
      if (q.dparams)
        reduce_params(q.stream, q.workspace, (int)grid, C::NPARAM, q.dparams, q.dparams_accumulate);
      return rs_status_after_launch();
    }
  }
  if constexpr (kSaved4<C>) {  // v4: the forward's O + softmax stats (rs_il_bwd_saved)
    const size_t lds3 = bwd3_lds_bytes<C>(q.F), lds4 = bwd4_lds_bytes<C>(q.F);
    if (q.asave && a.dy_vec && lds3 <= kLdsBytes / 2 && lds4 <= kLdsBytes / 2 &&
        (size_t)C::NPARAM * 4 <= lds4 && q.F <= C::FMAX && q.F >= 1) {
      // same grid rule as v3 (rs_il_bwd_partial_blocks answers for both)
      int64_t grid = bwd3_grid(q.B);
      const int64_t max_grid = q.workspace_floats / C::NPARAM;
      if (grid > kBwd3Grid) grid = kBwd3Grid;
      if (grid > max_grid) grid = max_grid;
      if (q.grid_out) { *q.grid_out = (int)(grid > 0 ? grid : 0); return RS_OK; }
      if (grid <= 0) return q.B == 0 ? RS_OK : RS_ERR_ARG;
      a.osave_in = q.asave;
      bwd4_kernel<C, DROP><<<(int)grid, 64 * kWpb3, lds4, q.stream>>>(
          q.x, q.xsave, q.dy, q.dy_ld, q.W, q.bias, q.gamma, q.beta, q.dx, q.dx_accumulate,
          q.workspace, a);
      if (q.dparams)
        reduce_params(q.stream, q.workspace, (int)grid, C::NPARAM, q.dparams, q.dparams_accumulate);
      return rs_status_after_launch();
    }
  }
  // the deferred weight gradient rides on the wide / v4 kernels only
  if (q.xt_x) return RS_ERR_UNSUPPORTED;
  {  // v3 (one wave per sample, no workgroup barriers) when its LDS gives 2 blocks per CU
    const size_t lds3 = bwd3_lds_bytes<C>(q.F);
    if (a.dy_vec && lds3 <= kLdsBytes / 2 && (size_t)C::NPARAM * 4 <= lds3) {
      int64_t grid = bwd3_grid(q.B);
      const int64_t max_grid = q.workspace_floats / C::NPARAM;
      if (grid > kBwd3Grid) grid = kBwd3Grid;
      if (grid > max_grid) grid = max_grid;
      if (q.grid_out) { *q.grid_out = (int)(grid > 0 ? grid : 0); return RS_OK; }
      if (grid <= 0) return q.B == 0 ? RS_OK : RS_ERR_ARG;
      bwd3_kernel<C, DROP><<<(int)grid, 64 * kWpb3, lds3, q.stream>>>(
          q.x, q.xsave, q.dy, q.dy_ld, q.W, q.bias, q.gamma, q.beta, q.dx, q.dx_accumulate,
          q.workspace, a);
      if (q.dparams)
        reduce_params(q.stream, q.workspace, (int)grid, C::NPARAM, q.dparams, q.dparams_accumulate);
      return rs_status_after_launch();
    }
  }
#endif
  const size_t lds = (size_t)a.per_wave * sizeof(float);
  if (lds > kLdsBytes || (size_t)C::NPARAM > (size_t)a.per_wave) return RS_ERR_UNSUPPORTED;
  // kMaxBwdGrid = one resident round of this kernel on MI355X (6 blocks per CU x 256 CUs at
  // config 2), so no block waits for a second round while others idle.  A fixed rule (not an
  // occupancy query) because callers size the partial-row reduction with
  // rs_il_bwd_partial_blocks.
  int64_t grid = q.B;
  const int64_t max_grid = q.workspace_floats / C::NPARAM;
  if (grid > kMaxBwdGrid) grid = kMaxBwdGrid;
  if (grid > max_grid) grid = max_grid;
  if (q.grid_out) { *q.grid_out = (int)(grid > 0 ? grid : 0); return RS_OK; }
  if (grid <= 0) return q.B == 0 ? RS_OK : RS_ERR_ARG;
  bwd2_kernel<C, DROP><<<(int)grid, 128, lds, q.stream>>>(
      q.x, q.xsave, q.dy, q.dy_ld, q.W, q.bias, q.gamma, q.beta, q.dx, q.dx_accumulate,
      q.workspace, a);
  if (q.dparams)  // NULL: leave the per-block partials in the workspace
    reduce_params(q.stream, q.workspace, (int)grid, C::NPARAM, q.dparams, q.dparams_accumulate);
  return rs_status_after_launch();
}

// EXACT instantiations (F == FMAX) drop the padded-key mask entirely.
// BF16: this shape also has bf16-math-mode instantiations (only the shapes a bf16 benchmark
// or model runs: each one doubles the unit's compile); without them a bf16 request is
// RS_ERR_UNSUPPORTED, never a silent fp32 run.
template <int E, int U, int H, int FMAX, bool EXACT = false, bool BF16 = false>
int try_fwd(const FwdReq& q) {
  if (q.E != E || q.U != U || q.H != H || q.F > FMAX || (EXACT && q.F != FMAX))
    return RS_ERR_UNSUPPORTED;
  if (q.bf16) {
    if constexpr (BF16)
      return q.drop_rate > 0.f ? fwd_launch<Cfg<E, U, H, FMAX, EXACT, true>, true>(q)
                               : fwd_launch<Cfg<E, U, H, FMAX, EXACT, true>, false>(q);
    return RS_ERR_UNSUPPORTED;
  }
  return q.drop_rate > 0.f ? fwd_launch<Cfg<E, U, H, FMAX, EXACT>, true>(q)
                           : fwd_launch<Cfg<E, U, H, FMAX, EXACT>, false>(q);
}

template <int E, int U, int H, int FMAX, bool EXACT = false, bool BF16 = false>
int try_bwd(const BwdReq& q) {
  if (q.E != E || q.U != U || q.H != H || q.F > FMAX || (EXACT && q.F != FMAX))
    return RS_ERR_UNSUPPORTED;
  if (q.bf16) {
    if constexpr (BF16)
      return q.drop_rate > 0.f ? bwd_launch<Cfg<E, U, H, FMAX, EXACT, true>, true>(q)
                               : bwd_launch<Cfg<E, U, H, FMAX, EXACT, true>, false>(q);
    return RS_ERR_UNSUPPORTED;
  }
  return q.drop_rate > 0.f ? bwd_launch<Cfg<E, U, H, FMAX, EXACT>, true>(q)
                           : bwd_launch<Cfg<E, U, H, FMAX, EXACT>, false>(q);
}

// Each instantiation unit (il_inst_*.hip) defines one pair of these.
#define RS_IL_DECLARE_UNIT(name)          \
  int name##_fwd(const rs_il::FwdReq& q); \
  int name##_bwd(const rs_il::BwdReq& q);

}  // namespace rs_il
