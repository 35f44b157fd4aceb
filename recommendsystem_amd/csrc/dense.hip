// H4/H5/H8/H9 MLP towers — Keras Dense(units, activation) on the CTR path, forward and backward.
//
// Reference call sites: autoint:36-52 (MultiLayerDense deep/logits towers),
// rank/multi_head/multidnn.py:60-64 (deep Dense(32, 16) relu), :80-127 (experts, gates, heads),
// rough_rank/layer.py:33-117 (DNN), staytime/VideoDnn.py:130-191 (experts / towers).
// Keras Dense = tensordot(x, kernel) + bias, then activation (kernel stored [in, out]).
//
// MI355X mapping: fp32 in / fp32 accumulate on the matrix cores (v_mfma_f32_16x16x4_f32: exact
// f32, a k-ordered fma chain, so the numerics equal an fp32 CPU dot product up to summation
// order).  One tiled GEMM engine (below) serves forward, data and weight gradients.  Leading
// dimensions are explicit so a layer reads a slice of a concatenated activation and writes
// straight into its slot of the next concat (the tf.concat on autoint:44 costs nothing).
//   forward      Y  = act(X W + b)
//   backward     dZ = dY * act'(Y) (recomputed on load, never stored)
//                dX = dZ W^T       (optionally accumulated)
//                dW = X^T dZ, db = colsum(dZ): split over M chunks -> per-chunk partials ->
//                fixed-order reduce (deterministic, no float atomics)
#include "blas.hpp"
#include "common.hpp"
#include "gemm_big.hpp"

#include <cstdint>
#include <cstdio>
#include <cstdlib>

enum { RS_ACT_NONE = 0, RS_ACT_RELU = 1, RS_ACT_SIGMOID = 2 };

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float act_fwd(float v, int act) {
  if (act == RS_ACT_RELU) return fmaxf(v, 0.f);
  if (act == RS_ACT_SIGMOID) return 1.0f / (1.0f + expf(-v));
  return v;
}

// dL/dz from dL/dy and the saved activation output y (TF ReluGrad / SigmoidGrad forms)
__device__ __forceinline__ float act_bwd(float dy, float y, int act) {
  if (act == RS_ACT_RELU) return y > 0.f ? dy : 0.f;
  if (act == RS_ACT_SIGMOID) return dy * y * (1.0f - y);
  return dy;
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// One MFMA GEMM engine for all three products (C[Mo, No] = sum_r A(m, r) B(r, n)):
//   forward       Y  = act(X W + b)          A = X  (row-major)      B = W  (row-major)
//   bwd data      dX (+)= dZ W^T             A = dZ (row-major, Z)   B(r=n, c=k) = W[k][n] (col)
//   bwd weight    dW = X^T dZ, db = colsum   A(k, m) = X[m][k] (col) B = dZ (row-major, Z)
// "Z" operands are dY * act'(Y) computed on load (dZ is never stored).
// Block = 256 threads (4 waves), tile BM x BN in {32, 64}^2, reduction staged through LDS in
// 16-deep slabs, double-buffered (the next slab's global loads are in flight while the current
// one feeds the MFMAs; one barrier per slab).  Each lane's float4 fragment read from LDS covers
// four k-steps of v_mfma_f32_16x16x4_f32 (the k index is permuted consistently in A and B), so a
// slab costs one ds_read_b128 per operand tile and 4 MFMAs per output tile.  The reduction can
// be split over gridDim.z (bwd weight with a small [K, N] and a batch-sized M): per-split
// partial rows, then column_reduce in split order (deterministic).
// ---------------------------------------------------------------------------------------------
enum { LAY_ROW = 0, LAY_COL = 1 };
enum { EPI_FWD = 0, EPI_STORE = 1, EPI_PARTIAL = 2 };

constexpr int GBK = 32;       // reduction slab
constexpr int LDP = GBK + 4;  // LDS row stride (floats): 16-byte aligned rows
constexpr int RQ = GBK / 4;   // float4s per row along r

struct GemmArgs {
  const float* a; int64_t lda; const float* ay; int64_t lday;   // ay: Y of a Z operand
  const float* b; int64_t ldb; const float* by; int64_t ldby;
  int64_t M, N, R, rchunk;
  int act_z;          // activation of the Z operand
  int epi, act;       // epilogue mode, forward activation
  const float* bias;
  float* out; int64_t ldo; int accumulate;
  float* db;          // bwd weight: column sums of B (row m-chunk z) or NULL
};

// Load one operand slab (tile rows [x0, x0 + BX) x reduction [r0, r0 + GBK)) into NL = BX/32
// float4 registers per thread.  ALONG_R: contiguous along r (A row / B col layouts), else
// contiguous along x (A col / B row).  Z operands keep dY and Y raw in registers: dZ = dY act'(Y)
// is formed only when the slab is stored to LDS, after the MFMAs of the current slab, so no wait
// on the prefetch lands in front of them (out-of-range elements load as dY = Y = 0 -> dZ = 0).
template <int BX, bool Z>
struct Slab {
  static constexpr int NL = BX * GBK / 4 / 256;  // float4 per thread
  float4 v[NL];
  float4 y[Z ? NL : 1];
  unsigned ok;  // VEC loads: bit u set when float4 u is in range
};

template <int BX, bool ALONG_R, bool Z, bool VEC>
__device__ __forceinline__ void load_one(float4& v, float4& yv, const float* p, int64_t ld,
                                         const float* y, int64_t ldy, int64_t x0, int64_t X,
                                         int64_t r0, int64_t R, int idx) {
  v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (Z) yv = v;
  int64_t x, r, xs, rs;  // element (x, r); strides of the four consecutive elements
  if (ALONG_R) {
    x = x0 + idx / RQ;
    r = r0 + 4 * (idx % RQ);
    if (x >= X) return;
    if (VEC && r + 3 < R) {
      v = *reinterpret_cast<const float4*>(p + x * ld + r);
      if (Z) yv = *reinterpret_cast<const float4*>(y + x * ldy + r);
      return;
    }
    xs = 0; rs = 1;
  } else {
    r = r0 + idx / (BX / 4);
    x = x0 + 4 * (idx % (BX / 4));
    if (r >= R) return;
    if (VEC && x + 3 < X) {
      v = *reinterpret_cast<const float4*>(p + r * ld + x);
      if (Z) yv = *reinterpret_cast<const float4*>(y + r * ldy + x);
      return;
    }
    xs = 1; rs = 0;
  }
  float e[4], f[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const bool ok = x + i * xs < X && r + i * rs < R;
    e[i] = ok ? p[(x + i * xs) * (ALONG_R ? ld : 1) + (r + i * rs) * (ALONG_R ? 1 : ld)] : 0.f;
    f[i] = (Z && ok) ? y[(x + i * xs) * (ALONG_R ? ldy : 1) + (r + i * rs) * (ALONG_R ? 1 : ldy)] : 0.f;
  }
  v = make_float4(e[0], e[1], e[2], e[3]);
  if (Z) yv = make_float4(f[0], f[1], f[2], f[3]);
}

// VEC operands (16-B aligned rows, extents along the contiguous axis multiples of 4) load every
// float4 unconditionally: an out-of-range one reads element 0 instead and is zeroed when stored
// (bit u of Slab::ok).  Branch-free loads let the compiler wait for exactly the older slab's loads
// before storing it; with per-lane branches it waited for every outstanding load, which
// serialised the slab's loads and the two-slab prefetch.
template <int BX, bool ALONG_R, bool Z, bool VEC>
__device__ __forceinline__ void load_slab(Slab<BX, Z>& sl, const float* p, int64_t ld, const float* y,
                                          int64_t ldy, int64_t x0, int64_t X, int64_t r0,
                                          int64_t R, int t) {
  if constexpr (VEC) {
    sl.ok = 0;
#pragma unroll
    for (int u = 0; u < Slab<BX, Z>::NL; ++u) {
      const int idx = t + 256 * u;
      int64_t x, r;
      if (ALONG_R) { x = x0 + idx / RQ; r = r0 + 4 * (idx % RQ); }
      else { r = r0 + idx / (BX / 4); x = x0 + 4 * (idx % (BX / 4)); }
      const bool ok = x < X && r < R;
      sl.ok |= ok ? 1u << u : 0u;
      const int64_t o = ok ? (ALONG_R ? x * ld + r : r * ld + x) : 0;
      sl.v[u] = *reinterpret_cast<const float4*>(p + o);
      if (Z) {
        const int64_t oy = ok ? (ALONG_R ? x * ldy + r : r * ldy + x) : 0;
        sl.y[u] = *reinterpret_cast<const float4*>(y + oy);
      }
    }
  } else {
    sl.ok = ~0u;
#pragma unroll
    for (int u = 0; u < Slab<BX, Z>::NL; ++u)
      load_one<BX, ALONG_R, Z, VEC>(sl.v[u], sl.y[Z ? u : 0], p, ld, y, ldy, x0, X, r0, R, t + 256 * u);
  }
}

// LDS image of one operand slab.  ALONG_R operands (contiguous along the reduction in global
// memory) keep rows of x: [x][GBK + 4], and a lane's float4 along r covers four k-steps.  The
// others keep the global orientation, rows of r: [GBK][BX + pad] (float4 stores, no transpose:
// a transposing scalar store into [x][r] rows hit the same few banks from every lane), and a
// lane reads its four k-steps as four ds_read_b32 -- pad 4 (MF 16: the four lane groups' rows
// 4 apart land 16 banks apart) or 8 (MF 32: the two half-waves' rows land 32 banks apart).
template <int BX, int MF, bool ALONG_R>
struct OpLay {
  static constexpr int LDX = BX + (MF == 32 ? 8 : 4);
  static constexpr int SIZE = ALONG_R ? BX * LDP : GBK * LDX;
};

template <int BX, int MF, bool ALONG_R, bool Z>
__device__ __forceinline__ void store_slab(float* s, const Slab<BX, Z>& sl, int act, int t) {
#pragma unroll
  for (int u = 0; u < Slab<BX, Z>::NL; ++u) {
    const int idx = t + 256 * u;
    float4 v = sl.v[u];
    if (!((sl.ok >> u) & 1u)) v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (Z) {
      const float4 yv = sl.y[u];
      v.x = act_bwd(v.x, yv.x, act); v.y = act_bwd(v.y, yv.y, act);
      v.z = act_bwd(v.z, yv.z, act); v.w = act_bwd(v.w, yv.w, act);
    }
    if (ALONG_R) {
      *reinterpret_cast<float4*>(s + (idx / RQ) * LDP + 4 * (idx % RQ)) = v;
    } else {
      const int ri = idx / (BX / 4), xq = idx % (BX / 4);
      *reinterpret_cast<float4*>(s + ri * OpLay<BX, MF, false>::LDX + 4 * xq) = v;
    }
  }
}

// the operand values at (x, kb + j), j = 0..3 (the k-steps of four consecutive MFMAs)
template <int BX, int MF, bool ALONG_R>
__device__ __forceinline__ float4 frag4(const float* s, int x, int kb) {
  if (ALONG_R) return *reinterpret_cast<const float4*>(s + x * LDP + kb);
  constexpr int LDX = OpLay<BX, MF, false>::LDX;
  return make_float4(s[kb * LDX + x], s[(kb + 1) * LDX + x], s[(kb + 2) * LDX + x],
                     s[(kb + 3) * LDX + x]);
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

// MF = 16: 16x16 output tiles on v_mfma_f32_16x16x4_f32 (32 x 32 / 32 x 64 / 64 x 64 blocks; small
// and medium GEMMs).  MF = 32: 32x32 tiles on v_mfma_f32_32x32x2_f32 for the large GEMMs (64 / 128
// square-or-oblong blocks): the four waves form a 2 x 2 grid, each owning (BM/2) x (BN/2) as
// 32x32 tiles, so per 8 k a wave reads BM/64 A and BN/64 B fragments (one ds_read_b128 each) for
// (BM/64)(BN/64) x 4 MFMAs -- twice the flops per operand read of the 16x16 form, and a 64 x 128 /
// 128 x 128 block moves 2-4x less L2 traffic per flop than a 32 x 64 one.  The k index inside each
// 8-slab is permuted as in the 16x16 form (lane half h supplies k = 4h + j to MFMA j, in A and B).
template <int BM, int BN, int MF, int ALAY, int BLAY, bool AZ, bool BZ, bool VEC>
__device__ __forceinline__ void gemm_block(const GemmArgs& g, const int64_t bx, const int64_t by,
                                           const int64_t bz) {
  static_assert(MF == 16 || MF == 32, "MFMA tile");
  constexpr int TM = BM / MF, TN = BN / MF;
  constexpr int WT = MF == 16 ? TM * TN / 4 : 1;            // 16x16 tiles per wave
  constexpr int WM = MF == 32 ? BM / 64 : 1, WN = MF == 32 ? BN / 64 : 1;  // 32x32 tiles per wave
  static_assert(MF == 16 ? WT >= 1 : (BM % 64 == 0 && BN % 64 == 0), "tile too small for 4 waves");
  constexpr bool A_ALONG_R = ALAY == LAY_ROW, B_ALONG_R = BLAY == LAY_COL;
  __shared__ __attribute__((aligned(16))) float As[2][OpLay<BM, MF, A_ALONG_R>::SIZE];
  __shared__ __attribute__((aligned(16))) float Bs[2][OpLay<BN, MF, B_ALONG_R>::SIZE];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int64_t m0 = bx * BM, n0 = by * BN;
  const int64_t rb = bz * g.rchunk;
  const int64_t re = rb + g.rchunk < g.R ? rb + g.rchunk : g.R;
  const bool do_db = g.db != nullptr && bx == 0;
  float csum = 0.f;
  f32x4 acc[WT];
  f32x16 acc32[WM][WN];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < WT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc32[i][j][e] = 0.f;
  }
  const int wr = w >> 1, wc = w & 1;  // MF = 32: the wave's quadrant
  // one slab in flight in registers: slab s + 1 loads while slab s feeds the MFMAs
  Slab<BM, AZ> ra;
  Slab<BN, BZ> rbv;
  auto load = [&](int64_t r) {
    load_slab<BM, A_ALONG_R, AZ, VEC>(ra, g.a, g.lda, g.ay, g.lday, m0, g.M, r, re, t);
    load_slab<BN, B_ALONG_R, BZ, VEC>(rbv, g.b, g.ldb, g.by, g.ldby, n0, g.N, r, re, t);
  };
  auto store = [&](int sbuf) {
    store_slab<BM, MF, A_ALONG_R, AZ>(As[sbuf], ra, g.act_z, t);
    store_slab<BN, MF, B_ALONG_R, BZ>(Bs[sbuf], rbv, g.act_z, t);
  };
  auto compute = [&](int cb) {
    if (do_db && t < BN) {
#pragma unroll
      for (int k = 0; k < GBK; ++k)
        csum += B_ALONG_R ? Bs[cb][t * LDP + k] : Bs[cb][k * OpLay<BN, MF, false>::LDX + t];
    }
    if constexpr (MF == 16) {
#pragma unroll
      for (int kg = 0; kg < GBK / 16; ++kg) {
#pragma unroll
        for (int i = 0; i < WT; ++i) {
          const int q = w * WT + i, rt = q / TN, ct = q % TN;
          const float4 af = frag4<BM, MF, A_ALONG_R>(As[cb], rt * 16 + (l & 15), kg * 16 + 4 * (l >> 4));
          const float4 bf = frag4<BN, MF, B_ALONG_R>(Bs[cb], ct * 16 + (l & 15), kg * 16 + 4 * (l >> 4));
          acc[i] = mfma4(af.x, bf.x, acc[i]);
          acc[i] = mfma4(af.y, bf.y, acc[i]);
          acc[i] = mfma4(af.z, bf.z, acc[i]);
          acc[i] = mfma4(af.w, bf.w, acc[i]);
        }
      }
    } else {
#pragma unroll
      for (int kg = 0; kg < GBK / 8; ++kg) {
        float4 af[WM], bf[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i)
          af[i] = frag4<BM, MF, A_ALONG_R>(As[cb], wr * (BM / 2) + i * 32 + (l & 31), kg * 8 + 4 * (l >> 5));
#pragma unroll
        for (int j = 0; j < WN; ++j)
          bf[j] = frag4<BN, MF, B_ALONG_R>(Bs[cb], wc * (BN / 2) + j * 32 + (l & 31), kg * 8 + 4 * (l >> 5));
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
          for (int j = 0; j < WN; ++j) {
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].x, bf[j].x, acc32[i][j], 0, 0, 0);
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].y, bf[j].y, acc32[i][j], 0, 0, 0);
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].z, bf[j].z, acc32[i][j], 0, 0, 0);
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].w, bf[j].w, acc32[i][j], 0, 0, 0);
          }
      }
    }
  };
  load(rb);
  store(0);
  __syncthreads();
  int buf = 0;
  for (int64_t r0 = rb; r0 < re; r0 += GBK) {
    load(r0 + GBK);  // (beyond re: masked loads of element 0, never stored)
    compute(buf);
    if (r0 + GBK < re) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  // ---- epilogue ----
  auto emit = [&](int64_t m, int64_t n, float v) {
    if (m < g.M && n < g.N) {
      if (g.epi == EPI_FWD) {
        g.out[m * g.ldo + n] = act_fwd(v + g.bias[n], g.act);
      } else if (g.epi == EPI_STORE) {
        float* d = g.out + m * g.ldo + n;
        *d = g.accumulate ? *d + v : v;
      } else {
        g.out[bz * (g.M * g.N + g.N) + m * g.N + n] = v;
      }
    }
  };
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < WT; ++i) {
      const int q = w * WT + i, rt = q / TN, ct = q % TN;
      const int64_t n = n0 + ct * 16 + (l & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) emit(m0 + rt * 16 + (l >> 4) * 4 + j, n, acc[i][j]);
    }
  } else {
    // 32x32 accumulator: register 4 i + j holds row 8 i + 4 (lane / 32) + j, column lane % 32
#pragma unroll
    for (int ti = 0; ti < WM; ++ti)
#pragma unroll
      for (int tj = 0; tj < WN; ++tj) {
        const int64_t n = n0 + wc * (BN / 2) + tj * 32 + (l & 31);
        const int64_t mb = m0 + wr * (BM / 2) + ti * 32 + 4 * (l >> 5);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) emit(mb + 8 * i + j, n, acc32[ti][tj][4 * i + j]);
      }
  }
  if (do_db && t < BN && n0 + t < g.N) {
    if (g.epi == EPI_PARTIAL) g.out[bz * (g.M * g.N + g.N) + g.M * g.N + n0 + t] = csum;
    else g.db[n0 + t] = g.accumulate ? g.db[n0 + t] + csum : csum;
  }
}

template <int BM, int BN, int MF, int ALAY, int BLAY, bool AZ, bool BZ, bool VEC>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  gemm_block<BM, BN, MF, ALAY, BLAY, AZ, BZ, VEC>(g, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Grouped launch: up to kMaxGroup independent GEMMs of one operand form and block shape (the
// expert / gate / tower layers of the configs-3/5 models that a Python loop launched one by one).
// Linear block b -> problem p (start[p] <= b < start[p + 1]) -> (split, tile row, tile column).
// The problem index is block-uniform, so its arguments are read with scalar loads.
constexpr int kMaxGroup = 8;
struct GemmGroup {
  GemmArgs g[kMaxGroup];
  int start[kMaxGroup + 1];
  int tx[kMaxGroup], ty[kMaxGroup];
  int n;
};

template <int BM, int BN, int MF, int ALAY, int BLAY, bool AZ, bool BZ, bool VEC>
__global__ void __launch_bounds__(256) gemm_group_kernel(GemmGroup gg) {
  const int b = (int)blockIdx.x;
  int p = 0;
#pragma unroll
  for (int k = 1; k < kMaxGroup; ++k) p += (k < gg.n && b >= gg.start[k]) ? 1 : 0;
  const int local = b - gg.start[p];
  const int per = gg.tx[p] * gg.ty[p];
  const int bz = local / per, rem = local - bz * per;
  gemm_block<BM, BN, MF, ALAY, BLAY, AZ, BZ, VEC>(gg.g[p], rem % gg.tx[p], rem / gg.tx[p], bz);
}

// Grouped deterministic column reduction of split-K partials: problem p's partial rows (one per
// split, K N weights then N biases) summed in split order into dW / db, blocks of 64 columns x 16
// row groups exactly as column_reduce_kernel.
struct ReduceGroup {
  const float* part[kMaxGroup];
  float* dw[kMaxGroup];
  float* db[kMaxGroup];
  int64_t kn[kMaxGroup], total[kMaxGroup];
  int nrows[kMaxGroup];
  int start[kMaxGroup + 1];
  int accumulate, n;
};

__global__ void __launch_bounds__(1024) column_reduce_group_kernel(ReduceGroup rg) {
  constexpr int G = 16;
  __shared__ float red[G][64];
  const int b = (int)blockIdx.x;
  int p = 0;
#pragma unroll
  for (int k = 1; k < kMaxGroup; ++k) p += (k < rg.n && b >= rg.start[k]) ? 1 : 0;
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t total = rg.total[p];
  const int64_t c = (int64_t)(b - rg.start[p]) * 64 + lc;
  const float* part = rg.part[p];
  const int nrows = rg.nrows[p];
  float s = 0.f;
  if (c < total) {
#pragma unroll 4
    for (int r = g; r < nrows; r += G) s += part[(int64_t)r * total + c];
  }
  red[g][lc] = s;
  __syncthreads();
  if (g == 0 && c < total) {
    float t = red[0][lc];
#pragma unroll
    for (int k = 1; k < G; ++k) t += red[k][lc];
    float* d = c < rg.kn[p] ? rg.dw[p] + c : rg.db[p] + (c - rg.kn[p]);
    *d = rg.accumulate ? (*d + t) : t;
  }
}

struct GemmPlan { int bm, bn, mf, splits; int64_t rchunk; };

// Tile / split-K policy.  256 CUs take ~4 resident 256-thread GEMM blocks each, so a launch wants
// ~1k blocks: 64-row tiles only when that still gives >= big_min tiles, and reductions split
// (deterministic partials + column_reduce) while the tile count is below split_below, towards
// split_target blocks with >= min_rows reduction rows per split; launches that cannot split
// (forward, data gradient) take 32-column tiles below narrow_below tiles.  GEMMs of >= big_macs
// multiply-adds may take the 32x32-MFMA blocks instead (64 x 64 .. 128 x 128), sized by the MFMA
// time of the busiest CU plus any split-K round trip, larger blocks on ties -- off by default:
// on the configs 3 / 5 shapes they measured no better than the 16x16 blocks at ~4 resident
// blocks per CU (the loads, not the MFMAs, bound these GEMMs).
// RS_GEMM_TUNE="a,b,c,d[,e[,f]]" overrides (host-side, read once; tools/gemm_tune.sh); f > 0
// enables the large-GEMM blocks from f multiply-adds.
struct GemmTune { int big_min, split_below, split_target, min_rows, narrow_below; int64_t big_macs; };
static const GemmTune& gemm_tune() {
  static const GemmTune t = [] {
    // round 4 (after the slab-pipeline change, tools/r04_tune*.sh, 50 steps): 64-row tiles from
    // 256 tiles, split below 256, narrow below 256 -- config 5 2.60 -> 2.53 ms, config 3 2.01 ->
    // 2.02, config 4 unchanged; the 32x32 blocks opt-in (f = 2^28: DESIGN 5.6)
    GemmTune v{256, 256, 1024, 128, 256, INT64_MAX};
    if (const char* e = getenv("RS_GEMM_TUNE")) {
      GemmTune o = v;
      long long bm = (long long)v.big_macs;
      const int n = sscanf(e, "%d,%d,%d,%d,%d,%lld", &o.big_min, &o.split_below, &o.split_target,
                           &o.min_rows, &o.narrow_below, &bm);
      o.big_macs = bm > 0 ? (int64_t)bm : INT64_MAX;
      if (n >= 4 && o.split_target > 0 && o.min_rows >= GBK)
        v = o;
    }
    return v;
  }();
  return t;
}

static int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

static GemmPlan finish_plan(GemmPlan p, int64_t R) {
  int64_t rc = cdiv(R, p.splits);
  rc = cdiv(rc, GBK) * GBK;
  p.rchunk = rc < GBK ? GBK : rc;
  p.splits = (int)cdiv(R, p.rchunk);
  if (p.splits < 1) p.splits = 1;
  return p;
}

static GemmPlan plan_gemm(int64_t M, int64_t N, int64_t R, bool allow_split) {
  const GemmTune& tu = gemm_tune();
  // degenerate extents (size queries of empty or invalid shapes; the launches reject them
  // before planning) plan as one tile: no tile count of 0 divides below
  if (M < 1) M = 1;
  if (N < 1) N = 1;
  if (R < 0) R = 0;
  GemmPlan p;
  p.mf = 16;
  if (M * N * R >= tu.big_macs) {
    // large GEMM: 32x32-MFMA blocks; cost = rounds over 256 CUs x block area x rows per split
    static const int cand[4][2] = {{128, 128}, {128, 64}, {64, 128}, {64, 64}};
    double best = 0;
    for (const auto& c : cand) {
      const int64_t tiles = cdiv(M, c[0]) * cdiv(N, c[1]);
      int64_t s = 1;
      if (allow_split) {  // fill one round of 256 CUs, >= 256 reduction rows per split
        s = 256 / tiles;
        const int64_t max_s = R / 256;
        if (s > max_s) s = max_s;
        if (s < 1) s = 1;
      }
      // us: MFMA time of the busiest CU (614 GFLOP/s per CU) + the split partials' round trip
      // (written and re-read by column_reduce at ~4 TB/s) and the reduce launch
      double cost = (double)cdiv(tiles * s, 256) * c[0] * c[1] * (double)cdiv(R, s) * 2.0 / 6.14e5;
      if (s > 1) cost += (double)s * M * N * 8.0 / 4.0e6 + 3.0;
      if (best == 0 || cost < best * 0.999) {
        best = cost;
        p.bm = c[0]; p.bn = c[1]; p.splits = (int)s;
      }
    }
    p.mf = 32;
    static const int forced = [] {  // tuning runs: RS_GEMM_BIG_TILE=BMxBN forces the block
      const char* e = getenv("RS_GEMM_BIG_TILE");
      int bm = 0, bn = 0;
      if (e && sscanf(e, "%dx%d", &bm, &bn) == 2 && (bm == 64 || bm == 128) && (bn == 64 || bn == 128))
        return bm * 1000 + bn;
      return 0;
    }();
    if (forced) {
      p.bm = forced / 1000; p.bn = forced % 1000;
      const int64_t tiles = cdiv(M, p.bm) * cdiv(N, p.bn);
      int64_t sp = allow_split ? 512 / tiles : 1;
      if (sp > R / 256) sp = R / 256;
      p.splits = (int)(sp < 1 ? 1 : sp);
    }
    return finish_plan(p, R);
  }
  p.bn = N <= 32 ? 32 : 64;
  const int64_t tn = (N + p.bn - 1) / p.bn;
  p.bm = ((M + 63) / 64) * tn >= tu.big_min ? 64 : 32;
  int64_t tiles = ((M + p.bm - 1) / p.bm) * tn;
  if (!allow_split && p.bn == 64 && tiles < tu.narrow_below) {  // no split-K: narrower tiles
    p.bn = 32;
    tiles = ((M + p.bm - 1) / p.bm) * ((N + 31) / 32);
  }
  p.splits = 1;
  if (allow_split && tiles < tu.split_below) {
    int64_t s = (tu.split_target + tiles - 1) / tiles;
    const int64_t max_s = (R + tu.min_rows - 1) / tu.min_rows;  // >= min_rows rows per split
    if (s > max_s) s = max_s;
    p.splits = (int)(s < 1 ? 1 : s);
  }
  return finish_plan(p, R);
}

template <int ALAY, int BLAY, bool AZ, bool BZ>
static void launch_gemm(hipStream_t s, const GemmPlan& p, const GemmArgs& g, bool vec) {
  dim3 grid((unsigned)((g.M + p.bm - 1) / p.bm), (unsigned)((g.N + p.bn - 1) / p.bn), (unsigned)p.splits);
#define RS_GEMM(BMM, BNN, MF, V) gemm_kernel<BMM, BNN, MF, ALAY, BLAY, AZ, BZ, V><<<grid, 256, 0, s>>>(g)
#define RS_GEMM_V(V)                                                   \
  if (p.mf == 32) {                                                    \
    if (p.bm == 128 && p.bn == 128) RS_GEMM(128, 128, 32, V);          \
    else if (p.bm == 128) RS_GEMM(128, 64, 32, V);                     \
    else if (p.bn == 128) RS_GEMM(64, 128, 32, V);                     \
    else RS_GEMM(64, 64, 32, V);                                       \
  } else {                                                             \
    if (p.bm == 64 && p.bn == 64) RS_GEMM(64, 64, 16, V);              \
    else if (p.bm == 64) RS_GEMM(64, 32, 16, V);                       \
    else if (p.bn == 64) RS_GEMM(32, 64, 16, V);                       \
    else RS_GEMM(32, 32, 16, V);                                       \
  }
  if (vec) {
    RS_GEMM_V(true)
  } else {
    RS_GEMM_V(false)
  }
#undef RS_GEMM_V
#undef RS_GEMM
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ---------------------------------------------------------------------------------------------
// The library route (blas.hpp) for the large plain GEMMs.  Row-major C[M, N] = A B is the
// column-major C^T = B^T A^T, so every call below swaps its operands:
//   forward   Y^T [N x M] = W^T-view (W row-major [K, N] = col-major N x K) . X^T-view, + bias, relu
//   data      dX^T [K x M] = op_T(W col-major N x K) . dZ^T-view (col-major N x M)
//   weight    dW^T [N x K] = dZ^T-view (N x M) . op_T(X^T-view col-major K x M)
// dZ = dY act'(Y) is materialised once in the workspace (act != none) by dz_partial_kernel,
// which also forms db's column partials per row split (fixed order; column_reduce sums them).
// ---------------------------------------------------------------------------------------------
constexpr int kDzMaxSplits = 256;

__global__ void __launch_bounds__(1024) dz_partial_kernel(const float* __restrict__ dY, int64_t lddy,
                                                          const float* __restrict__ Y, int64_t ldy,
                                                          int act, int64_t M, int N, int64_t rchunk,
                                                          float* __restrict__ dz,
                                                          float* __restrict__ part) {
  __shared__ float red[16][64];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lc;
  const int64_t r0 = (int64_t)blockIdx.y * rchunk;
  const int64_t r1 = r0 + rchunk < M ? r0 + rchunk : M;
  float s = 0.f;
  if (c < N) {
    for (int64_t r = r0 + g; r < r1; r += 16) {
      const float v = act_bwd(dY[r * lddy + c], act ? Y[r * ldy + c] : 0.f, act);
      if (dz) dz[r * N + c] = v;
      s += v;
    }
  }
  red[g][lc] = s;
  __syncthreads();
  if (g == 0 && c < N) {
    float t = red[0][lc];
#pragma unroll
    for (int k = 1; k < 16; ++k) t += red[k][lc];
    part[(int64_t)blockIdx.y * N + c] = t;
  }
}

static int64_t dz_splits(int64_t M, int N) {
  int64_t s = cdiv(256, cdiv(N, 64));
  const int64_t max_s = cdiv(M, 64);
  if (s > max_s) s = max_s;
  if (s > kDzMaxSplits) s = kDzMaxSplits;
  return s < 1 ? 1 : s;
}

static int64_t blas_bwd_workspace_floats(int64_t M, int N) {
  return M * N + (int64_t)kDzMaxSplits * N;
}

// 0: done; nonzero: nothing but workspace was written (the caller runs its own kernels)
static int blas_dense_bwd(hipStream_t s, const float* X, int64_t ldx, const float* dY, int64_t lddy,
                          const float* Y, int64_t ldy, int act, const float* W, int64_t M, int K,
                          int N, float* dX, int64_t lddx, int dx_accumulate, float* dW, float* db,
                          int w_accumulate, float* ws, int64_t wsf) {
  if (!ws || wsf < blas_bwd_workspace_floats(M, N)) return 1;
  const int64_t S = dz_splits(M, N), rc = cdiv(M, S);
  float* dz = act != RS_ACT_NONE ? ws : nullptr;
  float* part = ws + M * N;
  const float* Z = dz ? dz : dY;
  const int64_t ldz = dz ? N : lddy;
  dz_partial_kernel<<<dim3((unsigned)cdiv(N, 64), (unsigned)cdiv(M, rc)), 1024, 0, s>>>(
      dY, lddy, Y, ldy, act, M, N, rc, dz, part);
  if (rs_blas_gemm_cm(s, false, true, N, K, M, Z, ldz, X, ldx, w_accumulate ? 1.f : 0.f, dW, N,
                      nullptr, false))
    return 1;
  launch_column_reduce(s, part, (int)cdiv(M, rc), N, N, N, db, nullptr, w_accumulate);
  if (dX && rs_blas_gemm_cm(s, true, false, K, M, N, W, N, Z, ldz, dx_accumulate ? 1.f : 0.f, dX,
                            lddx, nullptr, false)) {
    // the data gradient on the engine (dZ recomputed from dY, Y on load)
    GemmArgs g{dY, lddy, Y, ldy, W, N, nullptr, 0, M, K, N, 0, act, EPI_STORE, 0, nullptr, dX, lddx,
               dx_accumulate, nullptr};
    GemmPlan p = plan_gemm(M, K, N, false);
    g.rchunk = p.rchunk;
    const bool vec = aligned16(dY) && aligned16(Y) && aligned16(W) && lddy % 4 == 0 &&
                     ldy % 4 == 0 && N % 4 == 0;
    launch_gemm<LAY_ROW, LAY_COL, true, false>(s, p, g, vec);
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// The large GEMMs (>= 2^26 multiply-adds: rs_big::wanted) run the direct-to-LDS kernels of
// gemm_big.hip; the library route (hipBLASLt, RS_GEMM_BLAS=1) is kept as an opt-in comparison.
// Each helper returns 0 when it launched, nonzero when the caller runs its own kernels.
// ---------------------------------------------------------------------------------------------
static int big_fwd(hipStream_t s, const float* X, int64_t M, int K, int64_t ldx, const float* W,
                   const float* bias, int N, int act, float* Y, int64_t ldy) {
  if (!rs_big::wanted_fwd(M, N, K)) return 1;
  return rs_big::fwd(s, X, M, K, ldx, W, bias, N, act, Y, ldy);
}

static int big_data(hipStream_t s, const float* dY, int64_t lddy, const float* Y, int64_t ldy,
                    int act, const float* W, int64_t M, int K, int N, float* dX, int64_t lddx,
                    int accumulate) {
  if (!rs_big::wanted(M, K, N)) return 1;
  const bool z = act != RS_ACT_NONE;
  const rs_big::Plan p = rs_big::plan(M, K, N, false, z);
  rs_big::Args g{};
  g.a = rs_big::Operand{dY, z ? Y : nullptr, lddy, ldy, M, 0};
  g.b = rs_big::Operand{W, nullptr, N, 0, K, 0};
  g.M = M; g.N = K; g.R = N; g.act_z = act;
  g.epi = rs_big::EPI_STORE; g.out = dX; g.ldo = lddx; g.accumulate = accumulate; g.Mreal = M;
  return rs_big::launch(s, rs_big::FORM_DATA, p, g);
}

// dZ = dY act'(Y) materialised once (the weight product's B operand is contiguous along its
// output, so a fused act' would read Y beside dY as four ds_read_b32 per fragment: measured
// 154 vs 109 us at 2048 x 1712 x 960, against ~4 us for this pass)
__global__ void __launch_bounds__(256) dz_kernel(const float* __restrict__ dY, int64_t lddy,
                                                 const float* __restrict__ Y, int64_t ldy, int act,
                                                 int64_t M, int N, float* __restrict__ dz) {
  const int64_t n4 = (int64_t)M * N;
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += (int64_t)gridDim.x * 256) {
    const int64_t m = k / N, n = k - m * N;
    dz[k] = act_bwd(dY[m * lddy + n], Y[m * ldy + n], act);
  }
}
static void launch_dz(hipStream_t s, const float* dY, int64_t lddy, const float* Y, int64_t ldy,
                      int act, int64_t M, int N, float* dz) {
  int64_t blocks = cdiv((int64_t)M * N, 256);
  if (blocks > 4096) blocks = 4096;
  dz_kernel<<<(unsigned)blocks, 256, 0, s>>>(dY, lddy, Y, ldy, act, M, N, dz);
}

// weight gradient dW [K, N] and db [N] as one product of K + 1 output rows (row K: db); with an
// activation the workspace holds dZ [M, N] first, then the split-K partials
static rs_big::Plan big_weight_plan(int64_t M, int K, int N, int act) {
  (void)act;
  return rs_big::plan((int64_t)K + 1, N, M, true, false);
}
static int64_t big_weight_ws(int64_t M, int K, int N, int act) {
  const rs_big::Plan p = big_weight_plan(M, K, N, act);
  return (p.splits > 1 ? (int64_t)p.splits * ((int64_t)K * N + N) : 0) +
         (act != RS_ACT_NONE ? (M * N + 3) / 4 * 4 : 0);
}
// dz: dZ already materialised by the caller (rs_dense_bwd), or nullptr
static int big_weight(hipStream_t s, const float* X, int64_t ldx, const float* dY, int64_t lddy,
                      const float* Y, int64_t ldy, int act, int64_t M, int K, int N, float* dW,
                      float* db, int accumulate, float* ws, int64_t wsf, const float* dz = nullptr) {
  if (!rs_big::wanted(K, N, M)) return 1;
  const bool z = act != RS_ACT_NONE;
  const rs_big::Plan p = big_weight_plan(M, K, N, act);
  const bool split = p.splits > 1;
  const int64_t total = (int64_t)K * N + N;
  if (!ws || wsf < big_weight_ws(M, K, N, act)) {
    if (split || (z && !dz)) return 1;
  }
  const int64_t zoff = z ? (M * N + 3) / 4 * 4 : 0;
  if (z && !dz) {
    launch_dz(s, dY, lddy, Y, ldy, act, M, N, ws);
    dz = ws;
  }
  float* part = ws + zoff;
  rs_big::Args g{};
  g.a = rs_big::Operand{X, nullptr, ldx, 0, K, 1};
  g.b = z ? rs_big::Operand{dz, nullptr, N, 0, N, 0}
          : rs_big::Operand{dY, nullptr, lddy, 0, N, 0};
  g.M = (int64_t)K + 1; g.N = N; g.R = M; g.act_z = act;
  g.Mreal = K;
  if (split) {
    g.epi = rs_big::EPI_PARTIAL; g.out = part; g.slab = total;
  } else {
    g.epi = rs_big::EPI_STORE; g.out = dW; g.ldo = N; g.db = db; g.accumulate = accumulate;
  }
  if (rs_big::launch(s, rs_big::FORM_WEIGHT, p, g)) return 1;
  if (split) launch_column_reduce(s, part, p.splits, total, total, (int64_t)K * N, dW, db, accumulate);
  return 0;
}

RS_API int rs_dense_fwd(void* stream, const float* X, int64_t M, int K, int64_t ldx,
                        const float* W, const float* bias, int N, int act, float* Y,
                        int64_t ldy) {
  if (!X || !W || !bias || !Y || M < 0 || K <= 0 || N <= 0 || ldx < K || ldy < N) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  if (act != RS_ACT_SIGMOID && rs_blas_wanted(M, N, K) &&
      rs_blas_gemm_cm(rs_stream(stream), false, false, N, M, K, W, N, X, ldx, 0.f, Y, ldy, bias,
                      act == RS_ACT_RELU) == 0)
    return rs_status_after_launch();
  if (big_fwd(rs_stream(stream), X, M, K, ldx, W, bias, N, act, Y, ldy) == 0)
    return rs_status_after_launch();
  GemmArgs g{X, ldx, nullptr, 0, W, N, nullptr, 0, M, N, K, 0, 0, EPI_FWD, act, bias, Y, ldy, 0, nullptr};
  GemmPlan p = plan_gemm(M, N, K, false);
  g.rchunk = p.rchunk;
  // VEC: every operand float4 lies wholly inside or wholly outside its extent
  const bool vec = aligned16(X) && aligned16(W) && ldx % 4 == 0 && N % 4 == 0 && K % 4 == 0;
  launch_gemm<LAY_ROW, LAY_ROW, false, false>(rs_stream(stream), p, g, vec);
  return rs_status_after_launch();
}

RS_API int rs_dense_bwd_data(void* stream, const float* dY, int64_t lddy, const float* Y,
                             int64_t ldy, int act, const float* W, int64_t M, int K, int N,
                             float* dX, int64_t lddx, int accumulate) {
  if (!dY || !Y || !W || !dX || M < 0 || K <= 0 || N <= 0 || lddx < K) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  // (the library route needs dZ = dY: no workspace here to materialise it)
  if (act == RS_ACT_NONE && rs_blas_wanted(M, K, N) &&
      rs_blas_gemm_cm(rs_stream(stream), true, false, K, M, N, W, N, dY, lddy,
                      accumulate ? 1.f : 0.f, dX, lddx, nullptr, false) == 0)
    return rs_status_after_launch();
  if (big_data(rs_stream(stream), dY, lddy, Y, ldy, act, W, M, K, N, dX, lddx, accumulate) == 0)
    return rs_status_after_launch();
  // C[M, K] = dZ[M, N] . W^T : B(r = n, c = k) = W[k * N + n] (column layout, ldb = N)
  GemmArgs g{dY, lddy, Y, ldy, W, N, nullptr, 0, M, K, N, 0, act, EPI_STORE, 0, nullptr, dX, lddx,
             accumulate, nullptr};
  GemmPlan p = plan_gemm(M, K, N, false);
  g.rchunk = p.rchunk;
  const bool vec = aligned16(dY) && aligned16(Y) && aligned16(W) && lddy % 4 == 0 && ldy % 4 == 0 &&
                   N % 4 == 0;
  launch_gemm<LAY_ROW, LAY_COL, true, false>(rs_stream(stream), p, g, vec);
  return rs_status_after_launch();
}

RS_API int rs_dense_uses_library(int64_t M, int K, int N) {
  return rs_blas_wanted(K, N, M) ? 1 : 0;
}

RS_API int rs_dense_uses_big(int64_t M, int K, int N) {
  return !rs_blas_wanted(K, N, M) && rs_big::wanted(K, N, M) ? 1 : 0;
}

RS_API int64_t rs_dense_bwd_weight_workspace_floats(int64_t M, int K, int N) {
  if (M < 0 || K <= 0 || N <= 0) return 0;  // (rs_dense_bwd_weight rejects these shapes)
  const GemmPlan p = plan_gemm(K, N, M, true);
  int64_t own = (int64_t)p.splits * ((int64_t)K * N + N);
  if (rs_big::wanted(K, N, M)) {  // either activation form (the caller's act is not known here)
    const int64_t b0 = big_weight_ws(M, K, N, RS_ACT_NONE), b1 = big_weight_ws(M, K, N, RS_ACT_RELU);
    own = own > b0 ? own : b0;
    own = own > b1 ? own : b1;
  }
  if (!rs_blas_wanted(K, N, M)) return own;
  const int64_t lib = blas_bwd_workspace_floats(M, N);  // (or the engine's, if the library declines)
  return lib > own ? lib : own;
}

RS_API int rs_dense_bwd_weight(void* stream, const float* X, int64_t ldx, const float* dY,
                               int64_t lddy, const float* Y, int64_t ldy, int act, int64_t M,
                               int K, int N, float* dW, float* db, int accumulate,
                               float* workspace, int64_t workspace_floats) {
  if (!X || !dY || !Y || !dW || !db || M < 0 || K <= 0 || N <= 0) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  if (M == 0) {
    if (!accumulate) {
      rs_fill_u32(s, dW, 0u, (int64_t)K * N);
      rs_fill_u32(s, db, 0u, N);
    }
    return rs_status_after_launch();
  }
  if (rs_blas_wanted(K, N, M) &&
      blas_dense_bwd(s, X, ldx, dY, lddy, Y, ldy, act, nullptr, M, K, N, nullptr, 0, 0, dW, db,
                     accumulate, workspace, workspace_floats) == 0)
    return rs_status_after_launch();
  if (big_weight(s, X, ldx, dY, lddy, Y, ldy, act, M, K, N, dW, db, accumulate, workspace,
                 workspace_floats) == 0)
    return rs_status_after_launch();
  // C[K, N] = sum_m X[m][k] dZ[m][n]: A(k, m) = X[m * ldx + k] (column layout), B = dZ rows
  const GemmPlan p = plan_gemm(K, N, M, true);
  const bool split = p.splits > 1;
  if (split && (!workspace || workspace_floats < (int64_t)p.splits * ((int64_t)K * N + N)))
    return RS_ERR_ARG;
  GemmArgs g{X, ldx, nullptr, 0, dY, lddy, Y, ldy, K, N, M, p.rchunk, act,
             split ? EPI_PARTIAL : EPI_STORE, 0, nullptr, split ? workspace : dW, N, accumulate,
             db};
  const bool vec = aligned16(X) && aligned16(dY) && aligned16(Y) && ldx % 4 == 0 && lddy % 4 == 0 &&
                   ldy % 4 == 0 && K % 4 == 0 && N % 4 == 0;
  launch_gemm<LAY_COL, LAY_ROW, false, true>(s, p, g, vec);
  if (split) {
    const int64_t total = (int64_t)K * N + N;
    launch_column_reduce(s, workspace, p.splits, total, total, (int64_t)K * N, dW, db, accumulate);
  }
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// One Dense layer's backward as ONE launch: blocks [0, nd) form the data gradient dX = dZ W^T,
// blocks [nd, ...) the weight gradient (its splits) -- two independent GEMMs of different operand
// forms side by side instead of back to back (one kernel boundary less per layer, and the small
// layers' two half-empty launches fill the chip together).  Both forms' LDS tiles are static, so a
// block reserves the sum; the branch is block-uniform.
// ---------------------------------------------------------------------------------------------
template <int BMD, int BND, int BMW, int BNW>
__global__ void __launch_bounds__(256) dense_bwd_dual_kernel(GemmArgs gd, GemmArgs gw, int nd,
                                                             int txd, int txw, int tyw) {
  const int b = (int)blockIdx.x;
  if (b < nd) {
    gemm_block<BMD, BND, 16, LAY_ROW, LAY_COL, true, false, true>(gd, b % txd, b / txd, 0);
  } else {
    const int l = b - nd, per = txw * tyw;
    const int bz = l / per, r = l - bz * per;
    gemm_block<BMW, BNW, 16, LAY_COL, LAY_ROW, false, true, true>(gw, r % txw, r / txw, bz);
  }
}

template <int BMD, int BND>
static void launch_dual_w(hipStream_t s, unsigned grid, const GemmArgs& gd, const GemmArgs& gw,
                          int nd, int txd, int txw, int tyw, int bmw, int bnw) {
#define RS_DUAL(BMW, BNW) \
  dense_bwd_dual_kernel<BMD, BND, BMW, BNW><<<grid, 256, 0, s>>>(gd, gw, nd, txd, txw, tyw)
  if (bmw == 64 && bnw == 64) RS_DUAL(64, 64);
  else if (bmw == 64) RS_DUAL(64, 32);
  else if (bnw == 64) RS_DUAL(32, 64);
  else RS_DUAL(32, 32);
#undef RS_DUAL
}

static void launch_dual(hipStream_t s, unsigned grid, const GemmArgs& gd, const GemmArgs& gw, int nd,
                        int txd, int txw, int tyw, int bmd, int bnd, int bmw, int bnw) {
  if (bmd == 64 && bnd == 64) launch_dual_w<64, 64>(s, grid, gd, gw, nd, txd, txw, tyw, bmw, bnw);
  else if (bmd == 64) launch_dual_w<64, 32>(s, grid, gd, gw, nd, txd, txw, tyw, bmw, bnw);
  else if (bnd == 64) launch_dual_w<32, 64>(s, grid, gd, gw, nd, txd, txw, tyw, bmw, bnw);
  else launch_dual_w<32, 32>(s, grid, gd, gw, nd, txd, txw, tyw, bmw, bnw);
}

RS_API int rs_dense_bwd(void* stream, const float* X, int64_t ldx, const float* dY, int64_t lddy,
                        const float* Y, int64_t ldy, int act, const float* W, int64_t M, int K,
                        int N, float* dX, int64_t lddx, int dx_accumulate, float* dW, float* db,
                        int w_accumulate, float* workspace, int64_t workspace_floats) {
  if (!X || !dY || !Y || !W || !dX || !dW || !db || M < 0 || K <= 0 || N <= 0 || lddx < K)
    return RS_ERR_ARG;
  if (M > 0 && rs_blas_wanted(K, N, M) &&
      blas_dense_bwd(rs_stream(stream), X, ldx, dY, lddy, Y, ldy, act, W, M, K, N, dX, lddx,
                     dx_accumulate, dW, db, w_accumulate, workspace, workspace_floats) == 0)
    return rs_status_after_launch();
  if (M > 0 && rs_big::wanted(K, N, M)) {
    // two big launches (data, weight); the data gradient of a shape below the big threshold
    // (M K N is the same product) cannot occur here
    hipStream_t s = rs_stream(stream);
    const bool z = act != RS_ACT_NONE;
    if (workspace && workspace_floats >= big_weight_ws(M, K, N, act)) {
      // dZ once into the workspace: the data product reads it plain, the weight product too
      if (z) launch_dz(s, dY, lddy, Y, ldy, act, M, N, workspace);
      const float* Z = z ? workspace : dY;
      const int64_t ldz = z ? N : lddy;
      if (big_data(s, Z, ldz, nullptr, 0, RS_ACT_NONE, W, M, K, N, dX, lddx, dx_accumulate) == 0) {
        if (big_weight(s, X, ldx, dY, lddy, Y, ldy, act, M, K, N, dW, db, w_accumulate, workspace,
                       workspace_floats, z ? workspace : nullptr) == 0)
          return rs_status_after_launch();
        return rs_dense_bwd_weight(stream, X, ldx, dY, lddy, Y, ldy, act, M, K, N, dW, db,
                                   w_accumulate, workspace, workspace_floats);
      }
    }
  }
  const GemmPlan pd = plan_gemm(M, K, N, false);
  const GemmPlan pw = plan_gemm(K, N, M, true);
  const bool vec_d = aligned16(dY) && aligned16(Y) && aligned16(W) && lddy % 4 == 0 && ldy % 4 == 0 &&
                     N % 4 == 0;
  const bool vec_w = aligned16(X) && aligned16(dY) && aligned16(Y) && ldx % 4 == 0 && lddy % 4 == 0 &&
                     ldy % 4 == 0 && K % 4 == 0 && N % 4 == 0;
  const int64_t txd = cdiv(M, pd.bm), tyd = cdiv(K, pd.bn);
  const int64_t txw = cdiv(K, pw.bm), tyw = cdiv(N, pw.bn);
  const int64_t nd = txd * tyd, nw = txw * tyw * pw.splits;
  if (M == 0 || pd.mf != 16 || pw.mf != 16 || !vec_d || !vec_w || nd + nw > ((int64_t)1 << 30)) {
    int st = M == 0 ? RS_OK
                    : rs_dense_bwd_data(stream, dY, lddy, Y, ldy, act, W, M, K, N, dX, lddx, dx_accumulate);
    if (st) return st;
    return rs_dense_bwd_weight(stream, X, ldx, dY, lddy, Y, ldy, act, M, K, N, dW, db, w_accumulate,
                               workspace, workspace_floats);
  }
  const bool split = pw.splits > 1;
  if (split && (!workspace || workspace_floats < (int64_t)pw.splits * ((int64_t)K * N + N)))
    return RS_ERR_ARG;
  GemmArgs gd{dY, lddy, Y, ldy, W, N, nullptr, 0, M, K, N, pd.rchunk, act, EPI_STORE, 0, nullptr, dX,
              lddx, dx_accumulate, nullptr};
  GemmArgs gw{X, ldx, nullptr, 0, dY, lddy, Y, ldy, K, N, M, pw.rchunk, act,
              split ? EPI_PARTIAL : EPI_STORE, 0, nullptr, split ? workspace : dW, N, w_accumulate, db};
  hipStream_t s = rs_stream(stream);
  launch_dual(s, (unsigned)(nd + nw), gd, gw, (int)nd, (int)txd, (int)txw, (int)tyw, pd.bm, pd.bn,
              pw.bm, pw.bn);
  if (split) {
    const int64_t total = (int64_t)K * N + N;
    launch_column_reduce(s, workspace, pw.splits, total, total, (int64_t)K * N, dW, db, w_accumulate);
  }
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// Grouped Dense launches (G <= kMaxGroup independent layers of one kind in ONE launch each): the
// per-expert / per-task / per-tower layers of the configs-3/5 models (staytime/VideoDnn.py:130-191
// ppnet gates and expert stacks, MMoE gate layers, task towers).  Host descriptors, int64 per
// problem (pointers as integers):
//   fwd         [M, K, N, ldx, ldy, act, X, W, bias, Y]
//   bwd_data    [M, K, N, lddy, ldy, act, dY, Y, W, dX, lddx, accumulate]
//   bwd_weight  [M, K, N, ldx, lddy, ldy, act, X, dY, Y, dW, db, accumulate]
// One block shape for the group (the largest problem's plan); weight gradients split their
// reduction per problem by the single-launch rule applied to the group's total tile count, and
// the split problems' partials are reduced by ONE grouped column_reduce launch.
// ---------------------------------------------------------------------------------------------
enum { GD_FWD = 10, GD_BWD_DATA = 12, GD_BWD_WEIGHT = 13 };

template <typename T>
static T* dptr(int64_t v) { return reinterpret_cast<T*>((uintptr_t)v); }

template <int ALAY, int BLAY, bool AZ, bool BZ>
static void launch_group(hipStream_t s, int bm, int bn, bool vec, const GemmGroup& gg) {
  const unsigned grid = (unsigned)gg.start[gg.n];
#define RS_GG(BMM, BNN, V) gemm_group_kernel<BMM, BNN, 16, ALAY, BLAY, AZ, BZ, V><<<grid, 256, 0, s>>>(gg)
#define RS_GG_V(V)                                   \
  if (bm == 64 && bn == 64) RS_GG(64, 64, V);        \
  else if (bm == 64) RS_GG(64, 32, V);               \
  else if (bn == 64) RS_GG(32, 64, V);               \
  else RS_GG(32, 32, V);
  if (vec) {
    RS_GG_V(true)
  } else {
    RS_GG_V(false)
  }
#undef RS_GG_V
#undef RS_GG
}

struct GroupPlan {
  int bm, bn;
  int splits[kMaxGroup];
  int64_t rchunk[kMaxGroup];
};

// (Mo, No, R) per problem: output extent and reduction length
static bool plan_group(int G, const int64_t (*shape)[3], bool allow_split, GroupPlan& gp) {
  if (G < 1 || G > kMaxGroup) return false;
  int big = 0;
  for (int p = 1; p < G; ++p)
    if (shape[p][0] * shape[p][1] * shape[p][2] > shape[big][0] * shape[big][1] * shape[big][2]) big = p;
  GemmPlan bp = plan_gemm(shape[big][0], shape[big][1], shape[big][2], allow_split);
  if (bp.mf != 16) { bp.bm = 64; bp.bn = 64; }
  gp.bm = bp.bm; gp.bn = bp.bn;
  const GemmTune& tu = gemm_tune();
  int64_t tiles = 0;
  for (int p = 0; p < G; ++p) tiles += cdiv(shape[p][0], gp.bm) * cdiv(shape[p][1], gp.bn);
  int64_t sp = 1;
  if (allow_split && tiles < tu.split_below) sp = cdiv(tu.split_target, tiles);
  for (int p = 0; p < G; ++p) {
    GemmPlan q;
    q.bm = gp.bm; q.bn = gp.bn; q.mf = 16;
    int64_t s = sp;
    const int64_t max_s = cdiv(shape[p][2], tu.min_rows);
    if (s > max_s) s = max_s;
    q.splits = (int)(s < 1 ? 1 : s);
    q = finish_plan(q, shape[p][2]);
    gp.splits[p] = q.splits;
    gp.rchunk[p] = q.rchunk;
  }
  return true;
}

static void group_blocks(GemmGroup& gg, int G, const GroupPlan& gp) {
  gg.n = G;
  gg.start[0] = 0;
  for (int p = 0; p < G; ++p) {
    gg.tx[p] = (int)cdiv(gg.g[p].M, gp.bm);
    gg.ty[p] = (int)cdiv(gg.g[p].N, gp.bn);
    gg.start[p + 1] = gg.start[p] + gg.tx[p] * gg.ty[p] * gp.splits[p];
  }
  for (int p = G; p < kMaxGroup; ++p) gg.start[p + 1] = gg.start[G];
}

RS_API int rs_dense_fwd_grouped(void* stream, int G, const int64_t* desc) {
  if (!desc || G < 1 || G > kMaxGroup) return RS_ERR_ARG;
  GemmGroup gg{};
  int64_t shape[kMaxGroup][3];
  bool vec = true;
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + GD_FWD * p;
    const int64_t M = d[0], K = d[1], N = d[2], ldx = d[3], ldy = d[4];
    const float* X = dptr<const float>(d[6]);
    const float* W = dptr<const float>(d[7]);
    const float* bias = dptr<const float>(d[8]);
    float* Y = dptr<float>(d[9]);
    if (!X || !W || !bias || !Y || M <= 0 || K <= 0 || N <= 0 || ldx < K || ldy < N) return RS_ERR_ARG;
    gg.g[p] = GemmArgs{X, ldx, nullptr, 0, W, N, nullptr, 0, M, N, K, 0, 0, EPI_FWD, (int)d[5],
                       bias, Y, ldy, 0, nullptr};
    shape[p][0] = M; shape[p][1] = N; shape[p][2] = K;
    vec = vec && aligned16(X) && aligned16(W) && ldx % 4 == 0 && N % 4 == 0 && K % 4 == 0;
  }
  GroupPlan gp;
  if (!plan_group(G, shape, false, gp)) return RS_ERR_ARG;
  for (int p = 0; p < G; ++p) gg.g[p].rchunk = gp.rchunk[p];
  group_blocks(gg, G, gp);
  launch_group<LAY_ROW, LAY_ROW, false, false>(rs_stream(stream), gp.bm, gp.bn, vec, gg);
  return rs_status_after_launch();
}

RS_API int rs_dense_bwd_data_grouped(void* stream, int G, const int64_t* desc) {
  if (!desc || G < 1 || G > kMaxGroup) return RS_ERR_ARG;
  GemmGroup gg{};
  int64_t shape[kMaxGroup][3];
  bool vec = true;
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + GD_BWD_DATA * p;
    const int64_t M = d[0], K = d[1], N = d[2], lddy = d[3], ldy = d[4], lddx = d[10];
    const float* dY = dptr<const float>(d[6]);
    const float* Y = dptr<const float>(d[7]);
    const float* W = dptr<const float>(d[8]);
    float* dX = dptr<float>(d[9]);
    if (!dY || !Y || !W || !dX || M <= 0 || K <= 0 || N <= 0 || lddx < K) return RS_ERR_ARG;
    gg.g[p] = GemmArgs{dY, lddy, Y, ldy, W, N, nullptr, 0, M, K, N, 0, (int)d[5], EPI_STORE, 0,
                       nullptr, dX, lddx, (int)d[11], nullptr};
    shape[p][0] = M; shape[p][1] = K; shape[p][2] = N;
    vec = vec && aligned16(dY) && aligned16(Y) && aligned16(W) && lddy % 4 == 0 && ldy % 4 == 0 &&
          N % 4 == 0;
  }
  GroupPlan gp;
  if (!plan_group(G, shape, false, gp)) return RS_ERR_ARG;
  for (int p = 0; p < G; ++p) gg.g[p].rchunk = gp.rchunk[p];
  group_blocks(gg, G, gp);
  launch_group<LAY_ROW, LAY_COL, true, false>(rs_stream(stream), gp.bm, gp.bn, vec, gg);
  return rs_status_after_launch();
}

static bool weight_group_plan(int G, const int64_t* desc, GroupPlan& gp) {
  int64_t shape[kMaxGroup][3];
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + GD_BWD_WEIGHT * p;
    if (d[0] <= 0 || d[1] <= 0 || d[2] <= 0) return false;  // (M, K, N)
    shape[p][0] = d[1]; shape[p][1] = d[2]; shape[p][2] = d[0];  // C[K, N] over M rows
  }
  return plan_group(G, shape, true, gp);
}

RS_API int64_t rs_dense_bwd_weight_grouped_workspace_floats(int G, const int64_t* desc) {
  if (!desc || G < 1 || G > kMaxGroup) return -1;
  GroupPlan gp;
  if (!weight_group_plan(G, desc, gp)) return -1;
  int64_t n = 0;
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + GD_BWD_WEIGHT * p;
    if (gp.splits[p] > 1) n += (int64_t)gp.splits[p] * (d[1] * d[2] + d[2]);
  }
  return n;
}

RS_API int rs_dense_bwd_weight_grouped(void* stream, int G, const int64_t* desc, float* workspace,
                                       int64_t workspace_floats) {
  if (!desc || G < 1 || G > kMaxGroup) return RS_ERR_ARG;
  GroupPlan gp;
  if (!weight_group_plan(G, desc, gp)) return RS_ERR_ARG;
  GemmGroup gg{};
  ReduceGroup rg{};
  int nred = 0;
  int64_t off = 0;
  bool vec = true;
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + GD_BWD_WEIGHT * p;
    const int64_t M = d[0], K = d[1], N = d[2], ldx = d[3], lddy = d[4], ldy = d[5];
    const float* X = dptr<const float>(d[7]);
    const float* dY = dptr<const float>(d[8]);
    const float* Y = dptr<const float>(d[9]);
    float* dW = dptr<float>(d[10]);
    float* db = dptr<float>(d[11]);
    const int acc = (int)d[12];
    if (!X || !dY || !Y || !dW || !db || M <= 0 || K <= 0 || N <= 0) return RS_ERR_ARG;
    const bool split = gp.splits[p] > 1;
    float* part = nullptr;
    if (split) {
      const int64_t need = (int64_t)gp.splits[p] * (K * N + N);
      if (!workspace || off + need > workspace_floats) return RS_ERR_ARG;
      part = workspace + off;
      off += need;
      rg.part[nred] = part; rg.dw[nred] = dW; rg.db[nred] = db;
      rg.kn[nred] = K * N; rg.total[nred] = K * N + N; rg.nrows[nred] = gp.splits[p];
      rg.accumulate = acc;  // (one flag per call: the Python group passes the same for every layer)
      ++nred;
    }
    gg.g[p] = GemmArgs{X, ldx, nullptr, 0, dY, lddy, Y, ldy, K, N, M, gp.rchunk[p], (int)d[6],
                       split ? EPI_PARTIAL : EPI_STORE, 0, nullptr, split ? part : dW, N, acc, db};
    vec = vec && aligned16(X) && aligned16(dY) && aligned16(Y) && ldx % 4 == 0 && lddy % 4 == 0 &&
          ldy % 4 == 0 && K % 4 == 0 && N % 4 == 0;
  }
  for (int p = 1; p < G; ++p)
    if ((int)desc[GD_BWD_WEIGHT * p + 12] != (int)desc[12]) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  group_blocks(gg, G, gp);
  launch_group<LAY_COL, LAY_ROW, false, true>(s, gp.bm, gp.bn, vec, gg);
  if (nred) {
    rg.n = nred;
    rg.start[0] = 0;
    for (int q = 0; q < nred; ++q) rg.start[q + 1] = rg.start[q] + (int)cdiv(rg.total[q], 64);
    for (int q = nred; q < kMaxGroup; ++q) rg.start[q + 1] = rg.start[nred];
    column_reduce_group_kernel<<<rg.start[nred], 1024, 0, s>>>(rg);
  }
  return rs_status_after_launch();
}

// ---------------------------------------------------------------------------------------------
// H4/H10 head: p = clip(s, lo, hi) (autoint:52 tf.clip_by_value(output, 1e-6, 1.0)) and
// cross_entropy (rank/ctr/base_model.py:7-12):
//   loss = mean_b sum_t [ -y log(p + 1e-6) - (1 - y) log(1 - p + 1e-6) ]
// One workgroup (deterministic block reduction for the scalar loss) also writes
// ds = dloss/ds, with the clip gradient (1 inside [lo, hi], 0 outside: TF ClipByValue grad).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) bce_clip_kernel(const float* __restrict__ s,
                                                        const float* __restrict__ y, int64_t M,
                                                        int T, float lo, float hi, float log_eps,
                                                        const float* __restrict__ gscale,
                                                        float* __restrict__ p_out,
                                                        float* __restrict__ loss,
                                                        float* __restrict__ ds) {
  __shared__ float red[1024];
  const int64_t n = M * T;
  const float inv_m = 1.0f / (float)M;
  const float gs = gscale ? gscale[0] * inv_m : inv_m;
  float acc = 0.f;
  // U elements per thread have their loads issued before any is used (one block walks all M T
  // elements: a load -> use chain per element made this launch latency-bound, 23 us at 4096 x 7);
  // each thread still adds its elements i = tid, tid + 1024, ... in order
  constexpr int U = 8;
  const int64_t step = (int64_t)blockDim.x;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += U * step) {
    float sv[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * step;
      sv[u] = i < n ? s[i] : 0.f;
      yv[u] = i < n ? y[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * step;
      if (i >= n) break;
      const float p = fminf(fmaxf(sv[u], lo), hi);
      const float li = -yv[u] * logf(p + log_eps) - (1.0f - yv[u]) * logf(1.0f - p + log_eps);
      acc += li;
      if (p_out) p_out[i] = p;
      if (ds) {
        const float dp = (-yv[u] / (p + log_eps) + (1.0f - yv[u]) / (1.0f - p + log_eps)) * gs;
        ds[i] = (sv[u] >= lo && sv[u] <= hi) ? dp : 0.f;
      }
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && loss) loss[0] = red[0] * inv_m;
}

// Multi-block form: each block sums its elements (same per-element arithmetic), the block sums
// go to ws partials, and the last block (rs_last_block over the counters at the head of ws) adds
// them in block order -> a fixed summation order for a given (M, T).  One workgroup was issue-
// bound on its own CU at config 3 (4096 x 7 elements, two logs and two divides each: 17.5 us).
constexpr int kBceThreads = 256;
constexpr int kBceMaxBlocks = 64;
static int bce_blocks(int64_t n) {
  const int64_t b = (n + 4 * kBceThreads - 1) / (4 * kBceThreads);
  return (int)(b < 1 ? 1 : (b > kBceMaxBlocks ? kBceMaxBlocks : b));
}

__global__ void __launch_bounds__(kBceThreads) bce_clip_multi_kernel(
    const float* __restrict__ s, const float* __restrict__ y, int64_t M, int T, float lo, float hi,
    float log_eps, const float* __restrict__ gscale, float* __restrict__ p_out,
    float* __restrict__ loss, float* __restrict__ ds, int32_t* __restrict__ ctr,
    float* __restrict__ partials) {
  __shared__ float red[kBceThreads / 64];
  const int64_t n = M * T;
  const float inv_m = 1.0f / (float)M;
  const float gs = gscale ? gscale[0] * inv_m : inv_m;
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float sv = s[i];
    const float p = fminf(fmaxf(sv, lo), hi);
    const float yv = y[i];
    acc += -yv * logf(p + log_eps) - (1.0f - yv) * logf(1.0f - p + log_eps);
    if (p_out) p_out[i] = p;
    if (ds) {
      const float dp = (-yv / (p + log_eps) + (1.0f - yv) / (1.0f - p + log_eps)) * gs;
      ds[i] = (sv >= lo && sv <= hi) ? dp : 0.f;
    }
  }
  acc = group_sum<64>(acc);
  if (lane_id() == 0) red[wave_id()] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float b = 0.f;
#pragma unroll
    for (int w = 0; w < kBceThreads / 64; ++w) b += red[w];
    partials[blockIdx.x] = b;
    __threadfence();  // release this block's partial before it counts as done
  }
  if (rs_last_block(ctr)) {
    __threadfence();  // acquire: every block's partial is visible
    float t = 0.f;
    for (int k = 0; k < (int)gridDim.x; ++k) t += partials[k];
    if (loss) loss[0] = t * inv_m;
  }
}

RS_API int64_t rs_bce_clip_workspace_floats(int64_t M, int T) {
  if (M <= 0 || T <= 0) return 0;
  return RS_DONE_WORDS + bce_blocks(M * (int64_t)T);
}

RS_API int rs_bce_clip_loss_ws(void* stream, const float* s, const float* y, int64_t M, int T,
                               float clip_lo, float clip_hi, float log_eps, const float* gscale,
                               float* p_out, float* loss, float* ds, float* workspace,
                               int64_t workspace_floats) {
  if (!s || !y || M <= 0 || T <= 0) return RS_ERR_ARG;
  if (!workspace || workspace_floats < rs_bce_clip_workspace_floats(M, T)) return RS_ERR_ARG;
  int32_t* ctr = reinterpret_cast<int32_t*>(workspace);
  bce_clip_multi_kernel<<<bce_blocks(M * (int64_t)T), kBceThreads, 0, rs_stream(stream)>>>(
      s, y, M, T, clip_lo, clip_hi, log_eps, gscale, p_out, loss, ds, ctr,
      workspace + RS_DONE_WORDS);
  return rs_status_after_launch();
}

RS_API int rs_bce_clip_loss(void* stream, const float* s, const float* y, int64_t M, int T,
                            float clip_lo, float clip_hi, float log_eps, const float* gscale,
                            float* p_out, float* loss, float* ds) {
  if (!s || !y || M <= 0 || T <= 0) return RS_ERR_ARG;
  bce_clip_kernel<<<1, 1024, 0, rs_stream(stream)>>>(s, y, M, T, clip_lo, clip_hi, log_eps, gscale,
                                                     p_out, loss, ds);
  return rs_status_after_launch();
}
