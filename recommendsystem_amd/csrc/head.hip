// H4 + H10 — the AutoInt head as ONE training kernel: deep MultiLayerDense over the flattened
// embeddings, concat [deep, interacting], logits Dense(T, act), clip_by_value, cross_entropy,
// and the whole backward of that head down to dL/d(interacting output) and dL/dx0.
//
// Reference: autoint:38-52 (deep = MultiLayerDense(mlp.hidden_units)(Flatten(all_inputs)),
// result = concat([deep, autoint], axis=1), logits = MultiLayerDense(logits.hidden_units)(result),
// output = clip_by_value(logits, 1e-6, 1.0)) and cross_entropy at rank/ctr/base_model.py:7-12
// (-y log(p + 1e-6) - (1 - y) log(1 - p + 1e-6), summed over the label axis, batch mean).
// The same pattern is rank/multi_head/multidnn.py:60-64 (deep Dense(32) -> Dense(16)).
//
// Why one kernel: at config 2 the head is 4096 x [416 -> 32 -> 16] + [432 -> 1]: 85 KFLOP per
// sample, ~1.7 us of fp32 MFMA time on the chip, but as separate GEMM / loss / reduce launches it
// cost ~100 us per step (nine launches, each latency-bound on a skinny K = 416 reduction, plus
// split-K partial reductions).  Here a workgroup owns RB = 16 samples end to end:
//   x0 tile and interacting-output tile -> LDS (coalesced float4, read once from HBM)
//   h1 = act(x0 W1 + b1)     v_mfma_f32_16x16x4_f32, K split over the waves, fixed-order combine
//   h2 = act(h1 W2 + b2)     MFMA
//   z  = [h2 | il] W3 + b3   VALU dot + DPP row sums;  y = act(z);  p = clip(y, lo, hi)
//   loss rows, dL/dz (clip gate: TF ClipByValue grad passes only inside [lo, hi]; act grad)
//   d il   = dz W3[D:]^T     -> global (the InteractingLayer backward's dy, row stride ld_dil)
//   d h2 -> d h1 -> dx0 = dz1 W1^T (MFMA) -> global (overwrite)
//   dW1 = x0^T dz1 (MFMA), dW2, dW3, db*: per-block partial rows in ARENA ORDER
//   [W1 | b1 | W2 | b2 | W3 | b3 | loss] -> rs_partials_reduce_adam sums them over blocks in a
// fixed order (deterministic, no float atomics) and runs the dense Adam in the same pass.
// W1 (53 KB at config 2), W2, W3 are staged once per block into LDS (row stride N1 + 4: the
// dx0 pass reads W1 rows as conflict-free float4s), so no MFMA waits on an L2 round trip.
// All arithmetic is fp32 (the reference's dtype); only the summation order differs from TF.
// (bf16 math mode, [N1, N2] = [32, 16] only: the MFMA operands are rounded to bf16.)
#include "common.hpp"

namespace rs_head {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2 };

__device__ __forceinline__ float act_f(float v, int act) {
  if (act == ACT_RELU) return fmaxf(v, 0.f);
  if (act == ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
  return v;
}

__device__ __forceinline__ float act_b(float dy, float y, int act) {
  if (act == ACT_RELU) return y > 0.f ? dy : 0.f;  // TF ReluGrad: y > 0
  if (act == ACT_SIGMOID) return dy * y * (1.0f - y);
  return dy;
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// diagnostic builds only (-DRS_HEAD_SKIP=bits, tools/head_bench.py): 1 = no W1 staging, 2 = no
// layer-1 backward, 4 = no dW1 partial stores, 8 = no x0 / il staging
#ifndef RS_HEAD_SKIP
#define RS_HEAD_SKIP 0
#endif
#ifdef RS_HEAD_STAMPS  // diagnostic build: block 0's phase times (s_memtime) -> d il row 0
#define HEAD_STAMP(k) \
  if (tid == 0) { uint64_t t_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)); st_[k] = t_; }
#else
#define HEAD_STAMP(k)
#endif
constexpr int RB = 16;   // samples per workgroup (one MFMA row tile)
constexpr int NTH = 1024; // 16 waves: 4 per SIMD at one block per CU (the LDS footprint)
constexpr int NW = NTH / 64;
constexpr int TMAX = 4;  // logits units

struct Args {
  const float* x0; int64_t ldx;            // [B, K0]
  const float* il; int64_t ld_il;          // [B, S]   (slice of the concat buffer)
  const float *W1, *b1, *W2, *b2, *W3, *b3;
  const float* labels;                     // [B, T]
  int64_t B;
  int K0, S, T, act1, act2, act3;
  float lo, hi, log_eps, inv_batch;
  float* p_out;                            // [B, T] clipped prediction (or null)
  float* dil; int64_t ld_dil;              // [B, S]
  float* dx0; int64_t ld_dx; int dx_accumulate;
  float* part; int64_t np;                 // [gridDim.x, np]
  float* dz1; int64_t ld_dz1;              // deferred dW1 (rs_mlp_head_train_dz): [B, N1], else null
};

// LDS carve-up (floats).  Row strides are padded by 4 (16-byte aligned rows, staggered banks).
template <int N1, int N2>
struct Lay {
  static constexpr int D = N2 > 0 ? N2 : N1;   // deep output width
  static constexpr int H1S = N1 + 4, H2S = (N2 > 0 ? N2 : 4) + 4;
  static constexpr int W1S = N1 + 4;  // W1 row stride in LDS: conflict-free float4 column reads
  int xs, xo, is, io, h1, h2, dz1, dzd, red, z3, lred, w1, w2, w3, total;
  __device__ __host__ Lay(int K0, int S, int T) {
    xs = K0 + 4; is = S + 4;
    int o = 0;
    w1 = o; o += K0 * W1S;
    w2 = o; o += (N1 * N2 + 3) & ~3;
    w3 = o; o += (((N2 > 0 ? N2 : N1) + S) * T + 3) & ~3;
    xo = o; o += RB * xs;
    io = o; o += RB * is;
    h1 = o; o += RB * H1S;
    h2 = o; o += RB * H2S;
    dz1 = o; o += RB * H1S;
    dzd = o; o += RB * (D + 4);
    red = o; o += NW * 256;         // per-wave 16x16 accumulator tiles (layer-1 K split)
    z3 = o; o += RB * TMAX;
    lred = o; o += NW;
    total = o;
  }
};

// rows x (n4 float4) of a row-major global matrix (row stride ld floats) -> LDS (row stride
// lds_stride); rows >= valid are zero-filled.  Split into issue (first BATCH * NTH float4 into
// registers) and commit (LDS stores, then any remainder synchronously), so the caller can put the
// loads of every source in flight before the first store: ONE memory round trip for the whole
// prologue instead of one per source.
template <int BATCH>
struct StageRows {
  float4 v[BATCH];
  float* dst; int lds_stride; const float* src; int64_t ld; int rows, n4, valid;
  __device__ __forceinline__ StageRows(float* d, int ls, const float* sp, int64_t l, int r, int n,
                                       int va)
      : dst(d), lds_stride(ls), src(sp), ld(l), rows(r), n4(n), valid(va) {}
  __device__ __forceinline__ float4 ld4(int idx) const {
    const int r = idx / n4, c = (idx - r * n4) * 4;
    float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (idx < rows * n4 && r < valid) z = *reinterpret_cast<const float4*>(src + r * ld + c);
    return z;
  }
  __device__ __forceinline__ void st4(int idx, float4 x) const {
    const int r = idx / n4, c = (idx - r * n4) * 4;
    if (idx < rows * n4) *reinterpret_cast<float4*>(dst + r * lds_stride + c) = x;
  }
  __device__ __forceinline__ void issue(int tid) {
#pragma unroll
    for (int u = 0; u < BATCH; ++u) v[u] = ld4(u * NTH + tid);
  }
  __device__ __forceinline__ void commit(int tid) {
#pragma unroll
    for (int u = 0; u < BATCH; ++u) st4(u * NTH + tid, v[u]);
    for (int base = BATCH * NTH; base < rows * n4; base += NTH) st4(base + tid, ld4(base + tid));
  }
};

// BF: bf16 math mode (rs_set_math_mode): the layer-1/2 and dx0/dW1 MFMAs take bf16-rounded
// operands (mfma_bf16, one instruction per 16-deep k chunk, fp32 accumulate); the logits dot,
// the loss and every stored value stay fp32.
// TT: the logits width T at compile time (1: every reference head -- AutoInt's Dense(1), the
// multi_head towers), 0: runtime T <= TMAX.  With T known the per-row / per-column T loops unroll
// into straight-line code (the runtime form measured 9.2 K cycles for the logits backward phase).
// DZ: deferred dW1 (rs_mlp_head_train_dz): the block stores its layer-1 dz rows (dz1 [B, N1])
// instead of a 16-row dW1 partial (K0 x N1 floats per block: 57 KB at config 2, 14.6 MB per
// B = 4096 step, written here and read back by the reduction); the optimizer tail forms
// dW1 = x0^T dz1 over the whole batch (rs_partials_reduce_adam_ex).  The partial row then starts
// at b1.
template <int N1, int N2, bool BF, int TT = 0, bool DZ = false>
__global__ void __launch_bounds__(NTH) head_train_kernel(Args a) {
  using L = Lay<N1, N2>;
  constexpr int D = L::D;
  constexpr int NT1 = N1 / 16;           // column tiles of layer 1
  constexpr int KSPLIT = NW / NT1;       // waves sharing one layer-1 tile (K split)
  static_assert(N1 % 16 == 0 && N1 <= 64 && N2 % 16 == 0 && N2 <= 64, "deep widths");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const L lay(a.K0, a.S, a.T);
  float* Xs = sm + lay.xo;
  float* Is = sm + lay.io;
  float* H1 = sm + lay.h1;
  float* H2 = sm + lay.h2;
  float* DZ1 = sm + lay.dz1;
  float* DZD = sm + lay.dzd;
  float* RED = sm + lay.red;
  float* Z3 = sm + lay.z3;
  float* LRED = sm + lay.lred;
  float* W1s = sm + lay.w1;
  float* W2s = sm + lay.w2;
  float* W3s = sm + lay.w3;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, q = l >> 4, j = l & 15;
  const int64_t b0 = (int64_t)blockIdx.x * RB;
#ifdef RS_HEAD_STAMPS
  uint64_t st_[16] = {};
#endif
  HEAD_STAMP(0)
  const int nrow = (int)(a.B - b0 < RB ? a.B - b0 : RB);
  const int K0 = a.K0, S = a.S, T = TT > 0 ? TT : a.T, C = D + S;
  const int xs = lay.xs, is = lay.is;

  // ---- weights (L2-resident, shared by every block) and the x0 / interacting tiles -> LDS
  //      (rows >= nrow are zero): every MFMA / dot operand below comes from LDS ----
  // the per-phase scalars (biases, labels) are loaded into registers with the staging batch:
  // no global round trip inside the phases below
  const int h1n = tid % N1;
  const float b1v = tid < RB * N1 ? a.b1[h1n] : 0.f;
  const float b2v = (N2 > 0 && w < N2 / 16) ? a.b2[16 * w + j] : 0.f;
  float b3v[TMAX], ylv[TMAX];
#pragma unroll
  for (int t = 0; t < TMAX; ++t) {
    const bool ok = t < T && l == 0 && w < nrow;
    b3v[t] = ok ? a.b3[t] : 0.f;
    ylv[t] = ok ? a.labels[(b0 + w) * T + t] : 0.f;
  }
  {
    // every source's first batch is in flight before the first LDS store: the block waits for
    // ~one L2/HBM round trip for the whole prologue (a load -> store loop waits per element)
    constexpr int n4 = N1 / 4;
    StageRows<4> sw1(W1s, L::W1S, a.W1, N1, K0, n4, K0);
    StageRows<2> sx(Xs, xs, a.x0 + b0 * a.ldx, a.ldx, RB, K0 >> 2, nrow);
    StageRows<2> si(Is, is, a.il + b0 * a.ld_il, a.ld_il, RB, S >> 2, nrow);
    if (!(RS_HEAD_SKIP & 1)) sw1.issue(tid);
    if (!(RS_HEAD_SKIP & 8)) { sx.issue(tid); si.issue(tid); }
    float w2v = tid < N1 * N2 ? a.W2[tid] : 0.f;
    float w3v = tid < C * T ? a.W3[tid] : 0.f;
    if (!(RS_HEAD_SKIP & 1)) sw1.commit(tid);
    if (!(RS_HEAD_SKIP & 8)) { sx.commit(tid); si.commit(tid); }
    if (tid < N1 * N2) W2s[tid] = w2v;
    if (tid < C * T) W3s[tid] = w3v;
    for (int idx = tid + NTH; idx < N1 * N2; idx += NTH) W2s[idx] = a.W2[idx];
    for (int idx = tid + NTH; idx < C * T; idx += NTH) W3s[idx] = a.W3[idx];
  }
  // LDS-only barriers from here on: no wave reads another wave's global writes (d il, dx0 and
  // the partial rows), so no phase boundary waits for the stores in flight (__syncthreads would)
  lds_barrier();
  HEAD_STAMP(1)

  // ---- layer 1: h1 = act1(x0 W1 + b1); wave w -> column tile w % NT1, K chunks w / NT1 :: KSPLIT
  //      (16-wide chunks; one ds_read_b128 of x0 feeds 4 k-steps; k permuted consistently) ----
  {
    const int nt = w % NT1, ks0 = w / NT1;
    const int nks = K0 >> 4;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    const float* wcol = W1s + 16 * nt + j;
    int s = ks0;
    for (; s + KSPLIT < nks; s += 2 * KSPLIT) {
      const float4 x4 = *reinterpret_cast<const float4*>(Xs + j * xs + 16 * s + 4 * q);
      const float4 y4 = *reinterpret_cast<const float4*>(Xs + j * xs + 16 * (s + KSPLIT) + 4 * q);
      const float* wk = wcol + (16 * s + 4 * q) * L::W1S;
      const float* wk2 = wcol + (16 * (s + KSPLIT) + 4 * q) * L::W1S;
      const float w0 = wk[0], w1 = wk[L::W1S], w2 = wk[2 * L::W1S], w3 = wk[3 * L::W1S];
      const float v0 = wk2[0], v1 = wk2[L::W1S], v2 = wk2[2 * L::W1S], v3 = wk2[3 * L::W1S];
      if constexpr (BF) {
        acc0 = mfma_bf16(pack_bf16(x4.x, x4.y), pack_bf16(x4.z, x4.w), pack_bf16(w0, w1),
                         pack_bf16(w2, w3), acc0);
        acc1 = mfma_bf16(pack_bf16(y4.x, y4.y), pack_bf16(y4.z, y4.w), pack_bf16(v0, v1),
                         pack_bf16(v2, v3), acc1);
      } else {
        acc0 = mfma(x4.x, w0, acc0); acc1 = mfma(y4.x, v0, acc1);
        acc0 = mfma(x4.y, w1, acc0); acc1 = mfma(y4.y, v1, acc1);
        acc0 = mfma(x4.z, w2, acc0); acc1 = mfma(y4.z, v2, acc1);
        acc0 = mfma(x4.w, w3, acc0); acc1 = mfma(y4.w, v3, acc1);
      }
    }
    for (; s < nks; s += KSPLIT) {
      const float4 x4 = *reinterpret_cast<const float4*>(Xs + j * xs + 16 * s + 4 * q);
      const float* wk = wcol + (16 * s + 4 * q) * L::W1S;
      if constexpr (BF) {
        acc0 = mfma_bf16(pack_bf16(x4.x, x4.y), pack_bf16(x4.z, x4.w),
                         pack_bf16(wk[0], wk[L::W1S]), pack_bf16(wk[2 * L::W1S], wk[3 * L::W1S]),
                         acc0);
      } else {
        acc0 = mfma(x4.x, wk[0], acc0);
        acc0 = mfma(x4.y, wk[L::W1S], acc0);
        acc0 = mfma(x4.z, wk[2 * L::W1S], acc0);
        acc0 = mfma(x4.w, wk[3 * L::W1S], acc0);
      }
    }
    // lane holds D[4q + r][j] of tile nt: stash per wave, combine in wave order below
#pragma unroll
    for (int r = 0; r < 4; ++r) RED[w * 256 + (4 * q + r) * 16 + j] = acc0[r] + acc1[r];
  }
  lds_barrier();
  HEAD_STAMP(2)
  static_assert(RB * N1 <= NTH, "one H1 element per thread");
  if (tid < RB * N1) {
    const int r = tid / N1, n = h1n, nt = n >> 4, jj = n & 15;
    float v = 0.f;
#pragma unroll
    for (int ks = 0; ks < KSPLIT; ++ks) v += RED[(ks * NT1 + nt) * 256 + r * 16 + jj];
    H1[r * L::H1S + n] = act_f(v + b1v, a.act1);
  }
  lds_barrier();
  HEAD_STAMP(3)

  // ---- layer 2: h2 = act2(h1 W2 + b2) (K = N1), wave w < N2/16 owns column tile w ----
  if (N2 > 0) {
    if (w < N2 / 16) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < N1 / 16; ++s) {
        const float4 x4 = *reinterpret_cast<const float4*>(H1 + j * L::H1S + 16 * s + 4 * q);
        const float* wk = W2s + (16 * s + 4 * q) * N2 + 16 * w + j;
        if constexpr (BF) {
          acc = mfma_bf16(pack_bf16(x4.x, x4.y), pack_bf16(x4.z, x4.w), pack_bf16(wk[0], wk[N2]),
                          pack_bf16(wk[2 * N2], wk[3 * N2]), acc);
        } else {
          acc = mfma(x4.x, wk[0], acc);
          acc = mfma(x4.y, wk[N2], acc);
          acc = mfma(x4.z, wk[2 * N2], acc);
          acc = mfma(x4.w, wk[3 * N2], acc);
        }
      }
      const float bb = b2v;
#pragma unroll
      for (int r = 0; r < 4; ++r) H2[(4 * q + r) * L::H2S + 16 * w + j] = act_f(acc[r] + bb, a.act2);
    }
    lds_barrier();
  HEAD_STAMP(4)
  }
  const float* HD = N2 > 0 ? H2 : H1;
  constexpr int HDS = N2 > 0 ? L::H2S : L::H1S;

  // ---- logits: z[r][t] = sum_c cat[r][c] W3[c][t] + b3[t]; one wave per row (RB = NW).  The
  //      row's wave goes straight on with its share of the backward: d il[r] = dz[r] W3[D:]^T
  //      (global) and the deep output's dz (DZD row r) -- no barrier between the loss and them;
  //      the cross-row sums (dW3, db3, loss) wait for the layer-2 backward phase ----
  static_assert(NW == RB, "logits pass maps one wave to one row");
  float lsum = 0.f;
  {
    const int r = w, c0 = l;
    float dzt[TMAX] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {  // unrolled: b3v / ylv stay registers
      if (t >= T) break;
      float acc = 0.f;
      for (int c = c0; c < C; c += 64) {
        const float xv = c < D ? HD[r * HDS + c] : Is[r * is + (c - D)];
        acc = fmaf(xv, W3s[c * T + t], acc);
      }
      acc = group_sum<64>(acc);
      float dz = 0.f;
      if (c0 == 0) {
        if (r < nrow) {
          const float y = act_f(acc + b3v[t], a.act3);
          const float p = fminf(fmaxf(y, a.lo), a.hi);
          const float yl = ylv[t];
          lsum += -yl * logf(p + a.log_eps) - (1.0f - yl) * logf(1.0f - p + a.log_eps);
          if (a.p_out) a.p_out[(b0 + r) * T + t] = p;
          const float dp = (-yl / (p + a.log_eps) + (1.0f - yl) / (1.0f - p + a.log_eps)) * a.inv_batch;
          dz = act_b((y >= a.lo && y <= a.hi) ? dp : 0.f, y, a.act3);
        }
        Z3[r * TMAX + t] = dz;
      }
      dzt[t] = __shfl(dz, 0, 64);  // the row's dz to every lane of its wave
    }
    // d(concat)[r][c] = sum_t dz[r][t] W3[c][t]: the interacting part -> d il (global), the deep
    // part -> DZD (with the deep output activation's gradient)
    for (int c = c0; c < C; c += 64) {
      float g = 0.f;
#pragma unroll
      for (int t = 0; t < TMAX; ++t)
        if (t < T) g = fmaf(dzt[t], W3s[c * T + t], g);
      if (c < D) {
        DZD[r * (D + 4) + c] = act_b(g, HD[r * HDS + c], N2 > 0 ? a.act2 : a.act1);
      } else if (r < nrow) {
        a.dil[(b0 + r) * a.ld_dil + (c - D)] = g;
      }
    }
  }
  if (l == 0) LRED[w] = lsum;  // lane 0 of each wave holds its row's loss terms
  lds_barrier();
  HEAD_STAMP(5)
  HEAD_STAMP(6)

  float* part = a.part + (int64_t)blockIdx.x * a.np;
  const int o_b1 = DZ ? 0 : K0 * N1, o_w2 = o_b1 + N1, o_b2 = o_w2 + N1 * N2, o_w3 = o_b2 + N2;
  const int o_b3 = o_w3 + C * T, o_loss = o_b3 + T;
  // ---- logits' cross-row sums: dW3 / db3 partials and the block's loss ----
  for (int c = tid; c < C; c += NTH) {
    float g[TMAX] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const float xv = c < D ? HD[r * HDS + c] : Is[r * is + (c - D)];
#pragma unroll
      for (int t = 0; t < TMAX; ++t)
        if (t < T) g[t] = fmaf(xv, Z3[r * TMAX + t], g[t]);
    }
    for (int t = 0; t < T; ++t) part[o_w3 + c * T + t] = g[t];
  }
  if (tid < T) {
    float g = 0.f;
    for (int r = 0; r < RB; ++r) g += Z3[r * TMAX + tid];
    part[o_b3 + tid] = g;
  }
  if (tid == 0) {
    float s = 0.f;
    for (int k = 0; k < NW; ++k) s += LRED[k];
    part[o_loss] = s;
  }

  // ---- layer 2 backward: dW2 = h1^T dz2, db2, dz1 = act1'(dz2 W2^T) ----
  if (N2 > 0) {
    for (int idx = tid; idx < N1 * N2; idx += NTH) {
      const int k = idx / N2, n = idx - k * N2;
      float g = 0.f;
#pragma unroll
      for (int r = 0; r < RB; ++r) g = fmaf(H1[r * L::H1S + k], DZD[r * (D + 4) + n], g);
      part[o_w2 + idx] = g;
    }
    if (tid < N2) {
      float g = 0.f;
#pragma unroll
      for (int r = 0; r < RB; ++r) g += DZD[r * (D + 4) + tid];
      part[o_b2 + tid] = g;
    }
    for (int idx = tid; idx < RB * N1; idx += NTH) {
      const int r = idx / N1, k = idx - r * N1;
      float g = 0.f;
#pragma unroll
      for (int n = 0; n < N2; ++n) g = fmaf(DZD[r * (D + 4) + n], W2s[k * N2 + n], g);
      DZ1[r * L::H1S + k] = act_b(g, H1[r * L::H1S + k], a.act1);
    }
  } else {
    for (int idx = tid; idx < RB * N1; idx += NTH) {
      const int r = idx / N1, k = idx - r * N1;
      DZ1[r * L::H1S + k] = DZD[r * (D + 4) + k];
    }
  }
  lds_barrier();
  HEAD_STAMP(7)
  if (tid < N1) {
    float g = 0.f;
#pragma unroll
    for (int r = 0; r < RB; ++r) g += DZ1[r * L::H1S + tid];
    part[o_b1 + tid] = g;
  }
  if constexpr (DZ) {
    for (int idx = tid; idx < nrow * N1; idx += NTH) {
      const int r = idx / N1, n = idx - r * N1;
      a.dz1[(b0 + r) * a.ld_dz1 + n] = DZ1[r * L::H1S + n];
    }
  }

  // ---- layer 1 backward (MFMA), e tiles of 16 spread over the waves:
  //      dx0[r][e] = sum_n dz1[r][n] W1[e][n]    (A = dz1, B = W1 rows, both from LDS)
  //      dW1[e][n] = sum_r x0[r][e] dz1[r][n]    (A = x0^T from LDS, B = dz1 from LDS) ----
  if (!(RS_HEAD_SKIP & 2)) {
    const int net = K0 >> 4;
    float4 dzf[N1 / 16];
#pragma unroll
    for (int s = 0; s < N1 / 16; ++s)
      dzf[s] = *reinterpret_cast<const float4*>(DZ1 + j * L::H1S + 16 * s + 4 * q);
    float dzb[4][NT1];  // B of dW1: dz1[4q + t][16 nt + j]
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt) dzb[t][nt] = DZ ? 0.f : DZ1[(4 * q + t) * L::H1S + 16 * nt + j];
    for (int et = w; et < net; et += NW) {
      const int e = 16 * et + j;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < N1 / 16; ++s) {
        const float4 w4 = *reinterpret_cast<const float4*>(W1s + e * L::W1S + 16 * s + 4 * q);
        if constexpr (BF) {
          acc = mfma_bf16(pack_bf16(dzf[s].x, dzf[s].y), pack_bf16(dzf[s].z, dzf[s].w),
                          pack_bf16(w4.x, w4.y), pack_bf16(w4.z, w4.w), acc);
        } else {
          acc = mfma(dzf[s].x, w4.x, acc);
          acc = mfma(dzf[s].y, w4.y, acc);
          acc = mfma(dzf[s].z, w4.z, acc);
          acc = mfma(dzf[s].w, w4.w, acc);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 4 * q + r;
        if (row < nrow) {
          float* d = a.dx0 + (b0 + row) * a.ld_dx + e;
          *d = a.dx_accumulate ? *d + acc[r] : acc[r];
        }
      }
      if constexpr (DZ) continue;
      float xa[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) xa[t] = Xs[(4 * q + t) * xs + e];
#pragma unroll
      for (int nt = 0; nt < NT1; ++nt) {
        f32x4 g = {0.f, 0.f, 0.f, 0.f};
        if constexpr (BF) {
          g = mfma_bf16(pack_bf16(xa[0], xa[1]), pack_bf16(xa[2], xa[3]),
                        pack_bf16(dzb[0][nt], dzb[1][nt]), pack_bf16(dzb[2][nt], dzb[3][nt]), g);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) g = mfma(xa[t], dzb[t][nt], g);
        }
        // D[4q + r][j] = dW1[16 et + 4q + r][16 nt + j]
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (!(RS_HEAD_SKIP & 4)) part[(16 * et + 4 * q + r) * N1 + 16 * nt + j] = g[r];
      }
    }
  }
  HEAD_STAMP(8)
#ifdef RS_HEAD_STAMPS
  if (tid == 0 && blockIdx.x == 0)
    for (int q2 = 1; q2 <= 8; ++q2) a.dil[q2 - 1] = (float)(st_[q2] - st_[q2 - 1]);
#endif
}

template <int N1, int N2, bool BF16_OK = false, int TT = 0, bool DZ = false>
int launch_mode(hipStream_t s, const Args& a, int64_t grid) {
  const Lay<N1, N2> lay(a.K0, a.S, a.T);
  const size_t lds = (size_t)lay.total * sizeof(float);
  if (lds > 160 * 1024) return RS_ERR_UNSUPPORTED;
  if (TT > 0 && a.T != TT) return RS_ERR_ARG;
  if (rs_math_mode_now() == RS_MATH_BF16) {
    if constexpr (!BF16_OK) return RS_ERR_UNSUPPORTED;  // never a silent fp32 run
    else head_train_kernel<N1, N2, true, TT, DZ><<<(unsigned)grid, NTH, lds, s>>>(a);
  } else {
    head_train_kernel<N1, N2, false, TT, DZ><<<(unsigned)grid, NTH, lds, s>>>(a);
  }
  return rs_status_after_launch();
}

template <int N1, int N2, bool BF16_OK = false, int TT = 0>
int launch(hipStream_t s, const Args& a, int64_t grid) {
  return a.dz1 ? launch_mode<N1, N2, BF16_OK, TT, true>(s, a, grid)
               : launch_mode<N1, N2, BF16_OK, TT, false>(s, a, grid);
}

}  // namespace rs_head

static int64_t head_np(int K0, int N1, int N2, int S, int T, bool dz = false) {
  const int D = N2 > 0 ? N2 : N1;
  return (dz ? 0 : (int64_t)K0 * N1) + N1 + (int64_t)N1 * N2 + N2 + (int64_t)(D + S) * T + T + 1;
}

RS_API int64_t rs_mlp_head_param_floats(int K0, int N1, int N2, int S, int T) {
  return head_np(K0, N1, N2, S, T) - 1;
}

RS_API int64_t rs_mlp_head_workspace_floats(int64_t B, int K0, int N1, int N2, int S, int T) {
  return ((B + rs_head::RB - 1) / rs_head::RB) * head_np(K0, N1, N2, S, T);
}

RS_API int64_t rs_mlp_head_dz_workspace_floats(int64_t B, int K0, int N1, int N2, int S, int T) {
  return ((B + rs_head::RB - 1) / rs_head::RB) * head_np(K0, N1, N2, S, T, true);
}

RS_API int rs_mlp_head_partial_blocks(int64_t B) {
  return (int)((B + rs_head::RB - 1) / rs_head::RB);
}

static int head_train_impl(void* stream, const float* x0, int64_t ldx, const float* il,
                           int64_t ld_il, int64_t B, int K0, int S, int N1, int act1, int N2,
                           int act2, int T, int act3, const float* W1, const float* b1,
                           const float* W2, const float* b2, const float* W3, const float* b3,
                           const float* labels, float clip_lo, float clip_hi, float log_eps,
                           float* p_out, float* dil, int64_t ld_dil, float* dx0, int64_t ld_dx,
                           int dx_accumulate, float* workspace, int64_t workspace_floats,
                           float* dz1, int64_t ld_dz1) {
  using namespace rs_head;
  if (!x0 || !il || !W1 || !b1 || !W3 || !b3 || !labels || !dil || !dx0 || !workspace)
    return RS_ERR_ARG;
  if (N2 > 0 && (!W2 || !b2)) return RS_ERR_ARG;
  if (B < 0 || K0 <= 0 || S <= 0 || T <= 0) return RS_ERR_ARG;
  if (dz1 && ld_dz1 < N1) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  if (T > TMAX || K0 % 16 != 0 || S % 4 != 0 || ldx % 4 != 0 || ld_il % 4 != 0)
    return RS_ERR_UNSUPPORTED;
  if (((uintptr_t)x0 & 15) || ((uintptr_t)il & 15)) return RS_ERR_UNSUPPORTED;
  for (int act : {act1, act2, act3})
    if (act < ACT_NONE || act > ACT_SIGMOID) return RS_ERR_ARG;
  const int64_t grid = (B + RB - 1) / RB;
  const int64_t np = head_np(K0, N1, N2, S, T, dz1 != nullptr);
  if (workspace_floats < grid * np) return RS_ERR_ARG;
  Args a{x0, ldx, il, ld_il, W1, b1, W2, b2, W3, b3, labels, B, K0, S, T, act1, act2, act3,
         clip_lo, clip_hi, log_eps, 1.0f / (float)B, p_out, dil, ld_dil, dx0, ld_dx,
         dx_accumulate, workspace, np, dz1, ld_dz1};
  hipStream_t s = rs_stream(stream);
#define RS_HEAD(A, Bn) if (N1 == A && N2 == Bn) return launch<A, Bn>(s, a, grid);
  if (N1 == 32 && N2 == 16)  // config 2 (bf16 too)
    return T == 1 ? launch<32, 16, true, 1>(s, a, grid) : launch<32, 16, true>(s, a, grid);
  RS_HEAD(64, 32) RS_HEAD(16, 0) RS_HEAD(32, 0) RS_HEAD(64, 0)
  RS_HEAD(16, 16) RS_HEAD(32, 32) RS_HEAD(64, 16) RS_HEAD(64, 64)
#undef RS_HEAD
  return RS_ERR_UNSUPPORTED;
}

RS_API int rs_mlp_head_train(void* stream, const float* x0, int64_t ldx, const float* il,
                             int64_t ld_il, int64_t B, int K0, int S, int N1, int act1, int N2,
                             int act2, int T, int act3, const float* W1, const float* b1,
                             const float* W2, const float* b2, const float* W3, const float* b3,
                             const float* labels, float clip_lo, float clip_hi, float log_eps,
                             float* p_out, float* dil, int64_t ld_dil, float* dx0, int64_t ld_dx,
                             int dx_accumulate, float* workspace, int64_t workspace_floats) {
  return head_train_impl(stream, x0, ldx, il, ld_il, B, K0, S, N1, act1, N2, act2, T, act3, W1, b1,
                         W2, b2, W3, b3, labels, clip_lo, clip_hi, log_eps, p_out, dil, ld_dil, dx0,
                         ld_dx, dx_accumulate, workspace, workspace_floats, nullptr, 0);
}

RS_API int rs_mlp_head_train_dz(void* stream, const float* x0, int64_t ldx, const float* il,
                                int64_t ld_il, int64_t B, int K0, int S, int N1, int act1, int N2,
                                int act2, int T, int act3, const float* W1, const float* b1,
                                const float* W2, const float* b2, const float* W3, const float* b3,
                                const float* labels, float clip_lo, float clip_hi, float log_eps,
                                float* p_out, float* dil, int64_t ld_dil, float* dx0,
                                int64_t ld_dx, int dx_accumulate, float* workspace,
                                int64_t workspace_floats, float* dz1, int64_t ld_dz1) {
  if (!dz1) return RS_ERR_ARG;
  return head_train_impl(stream, x0, ldx, il, ld_il, B, K0, S, N1, act1, N2, act2, T, act3, W1, b1,
                         W2, b2, W3, b3, labels, clip_lo, clip_hi, log_eps, p_out, dil, ld_dil, dx0,
                         ld_dx, dx_accumulate, workspace, workspace_floats, dz1, ld_dz1);
}
