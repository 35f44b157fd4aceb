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
#include "common.hpp"

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

template <bool Z>
__device__ __forceinline__ float opval(const float* p, const float* y, int64_t i, int64_t iy, int act) {
  if (!Z) return p[i];
  return act_bwd(p[i], y[iy], act);
}

template <bool Z>
__device__ __forceinline__ float4 opval4(const float* p, const float* y, int64_t i, int64_t iy, int act) {
  float4 v = *reinterpret_cast<const float4*>(p + i);
  if (Z) {
    const float4 yv = *reinterpret_cast<const float4*>(y + iy);
    v.x = act_bwd(v.x, yv.x, act); v.y = act_bwd(v.y, yv.y, act);
    v.z = act_bwd(v.z, yv.z, act); v.w = act_bwd(v.w, yv.w, act);
  }
  return v;
}

// Load one operand slab (tile rows [x0, x0 + BX) x reduction [r0, r0 + GBK)) into NL = BX/32
// float4 registers per thread.  ALONG_R: contiguous along r (A row / B col layouts), else
// contiguous along x (A col / B row).
template <int BX, bool ALONG_R, bool Z, bool VEC>
__device__ __forceinline__ float4 load_one(const float* p, int64_t ld, const float* y, int64_t ldy,
                                           int act, int64_t x0, int64_t X, int64_t r0, int64_t R,
                                           int idx) {
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t x, r;
  if (ALONG_R) {
    x = x0 + idx / RQ;
    r = r0 + 4 * (idx % RQ);
    if (x >= X) return v;
    if (VEC && r + 3 < R) return opval4<Z>(p, y, x * ld + r, x * ldy + r, act);
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = (r + i < R) ? opval<Z>(p, y, x * ld + r + i, x * ldy + r + i, act) : 0.f;
    return make_float4(e[0], e[1], e[2], e[3]);
  } else {
    r = r0 + idx / (BX / 4);
    x = x0 + 4 * (idx % (BX / 4));
    if (r >= R) return v;
    if (VEC && x + 3 < X) return opval4<Z>(p, y, r * ld + x, r * ldy + x, act);
    float e[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = (x + i < X) ? opval<Z>(p, y, r * ld + x + i, r * ldy + x + i, act) : 0.f;
    return make_float4(e[0], e[1], e[2], e[3]);
  }
}

template <int BX>
struct Slab {
  static constexpr int NL = BX * GBK / 4 / 256;  // float4 per thread
  float4 v[NL];
};

template <int BX, bool ALONG_R, bool Z, bool VEC>
__device__ __forceinline__ void load_slab(Slab<BX>& sl, const float* p, int64_t ld, const float* y,
                                          int64_t ldy, int act, int64_t x0, int64_t X, int64_t r0,
                                          int64_t R, int t) {
#pragma unroll
  for (int u = 0; u < Slab<BX>::NL; ++u)
    sl.v[u] = load_one<BX, ALONG_R, Z, VEC>(p, ld, y, ldy, act, x0, X, r0, R, t + 256 * u);
}

template <int BX, bool ALONG_R>
__device__ __forceinline__ void store_slab(float* s, const Slab<BX>& sl, int t) {
#pragma unroll
  for (int u = 0; u < Slab<BX>::NL; ++u) {
    const int idx = t + 256 * u;
    const float4 v = sl.v[u];
    if (ALONG_R) {
      *reinterpret_cast<float4*>(s + (idx / RQ) * LDP + 4 * (idx % RQ)) = v;
    } else {
      const int ri = idx / (BX / 4), xq = idx % (BX / 4);
      s[(4 * xq + 0) * LDP + ri] = v.x;
      s[(4 * xq + 1) * LDP + ri] = v.y;
      s[(4 * xq + 2) * LDP + ri] = v.z;
      s[(4 * xq + 3) * LDP + ri] = v.w;
    }
  }
}

template <int BM, int BN, int ALAY, int BLAY, bool AZ, bool BZ, bool VEC>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g) {
  constexpr int TM = BM / 16, TN = BN / 16, WT = TM * TN / 4;
  static_assert(WT >= 1, "tile too small for 4 waves");
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDP];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDP];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  const int64_t m0 = (int64_t)blockIdx.x * BM, n0 = (int64_t)blockIdx.y * BN;
  const int64_t rb = (int64_t)blockIdx.z * g.rchunk;
  const int64_t re = rb + g.rchunk < g.R ? rb + g.rchunk : g.R;
  const bool do_db = g.db != nullptr && blockIdx.x == 0;
  float csum = 0.f;
  f32x4 acc[WT];
#pragma unroll
  for (int i = 0; i < WT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr bool A_ALONG_R = ALAY == LAY_ROW, B_ALONG_R = BLAY == LAY_COL;
  Slab<BM> ra;
  Slab<BN> rbv;
  load_slab<BM, A_ALONG_R, AZ, VEC>(ra, g.a, g.lda, g.ay, g.lday, g.act_z, m0, g.M, rb, re, t);
  load_slab<BN, B_ALONG_R, BZ, VEC>(rbv, g.b, g.ldb, g.by, g.ldby, g.act_z, n0, g.N, rb, re, t);
  store_slab<BM, A_ALONG_R>(As[0], ra, t);
  store_slab<BN, B_ALONG_R>(Bs[0], rbv, t);
  __syncthreads();
  int buf = 0;
  for (int64_t r0 = rb; r0 < re; r0 += GBK) {
    const bool more = r0 + GBK < re;
    if (more) {
      load_slab<BM, A_ALONG_R, AZ, VEC>(ra, g.a, g.lda, g.ay, g.lday, g.act_z, m0, g.M, r0 + GBK, re, t);
      load_slab<BN, B_ALONG_R, BZ, VEC>(rbv, g.b, g.ldb, g.by, g.ldby, g.act_z, n0, g.N, r0 + GBK, re, t);
    }
    if (do_db && t < BN) {
#pragma unroll
      for (int k = 0; k < GBK; ++k) csum += Bs[buf][t * LDP + k];
    }
#pragma unroll
    for (int kg = 0; kg < GBK / 16; ++kg) {
#pragma unroll
      for (int i = 0; i < WT; ++i) {
        const int q = w * WT + i, rt = q / TN, ct = q % TN;
        const float4 af = *reinterpret_cast<const float4*>(
            &As[buf][(rt * 16 + (l & 15)) * LDP + kg * 16 + 4 * (l >> 4)]);
        const float4 bf = *reinterpret_cast<const float4*>(
            &Bs[buf][(ct * 16 + (l & 15)) * LDP + kg * 16 + 4 * (l >> 4)]);
        acc[i] = mfma4(af.x, bf.x, acc[i]);
        acc[i] = mfma4(af.y, bf.y, acc[i]);
        acc[i] = mfma4(af.z, bf.z, acc[i]);
        acc[i] = mfma4(af.w, bf.w, acc[i]);
      }
    }
    if (more) {
      store_slab<BM, A_ALONG_R>(As[buf ^ 1], ra, t);
      store_slab<BN, B_ALONG_R>(Bs[buf ^ 1], rbv, t);
    }
    __syncthreads();
    buf ^= 1;
  }
  // ---- epilogue ----
#pragma unroll
  for (int i = 0; i < WT; ++i) {
    const int q = w * WT + i, rt = q / TN, ct = q % TN;
    const int64_t n = n0 + ct * 16 + (l & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t m = m0 + rt * 16 + (l >> 4) * 4 + j;
      if (m < g.M && n < g.N) {
        const float v = acc[i][j];
        if (g.epi == EPI_FWD) {
          g.out[m * g.ldo + n] = act_fwd(v + g.bias[n], g.act);
        } else if (g.epi == EPI_STORE) {
          float* d = g.out + m * g.ldo + n;
          *d = g.accumulate ? *d + v : v;
        } else {
          g.out[(int64_t)blockIdx.z * (g.M * g.N + g.N) + m * g.N + n] = v;
        }
      }
    }
  }
  if (do_db && t < BN && n0 + t < g.N) {
    if (g.epi == EPI_PARTIAL) g.out[(int64_t)blockIdx.z * (g.M * g.N + g.N) + g.M * g.N + n0 + t] = csum;
    else g.db[n0 + t] = g.accumulate ? g.db[n0 + t] + csum : csum;
  }
}

struct GemmPlan { int bm, bn, splits; int64_t rchunk; };

// Tile / split-K policy.  256 CUs take ~4 resident 256-thread GEMM blocks each, so a launch wants
// ~1k blocks: 64-row tiles only when that still gives >= big_min tiles, and reductions split
// (deterministic partials + column_reduce) while the tile count is below split_below, towards
// split_target blocks with >= min_rows reduction rows per split; launches that cannot split
// (forward, data gradient) take 32-column tiles below narrow_below tiles.  RS_GEMM_TUNE="a,b,c,d[,e]"
// overrides (host-side, read once; tools/gemm_tune.sh).
struct GemmTune { int big_min, split_below, split_target, min_rows, narrow_below; };
static const GemmTune& gemm_tune() {
  static const GemmTune t = [] {
    GemmTune v{512, 512, 1024, 128, 512};
    if (const char* e = getenv("RS_GEMM_TUNE")) {
      GemmTune o = v;
      const int n = sscanf(e, "%d,%d,%d,%d,%d", &o.big_min, &o.split_below, &o.split_target,
                           &o.min_rows, &o.narrow_below);
      if (n >= 4 && o.split_target > 0 && o.min_rows >= GBK)
        v = o;
    }
    return v;
  }();
  return t;
}

static GemmPlan plan_gemm(int64_t M, int64_t N, int64_t R, bool allow_split) {
  const GemmTune& tu = gemm_tune();
  GemmPlan p;
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
  int64_t rc = (R + p.splits - 1) / p.splits;
  rc = (rc + GBK - 1) / GBK * GBK;
  p.rchunk = rc < GBK ? GBK : rc;
  p.splits = (int)((R + p.rchunk - 1) / p.rchunk);
  if (p.splits < 1) p.splits = 1;
  return p;
}

template <int ALAY, int BLAY, bool AZ, bool BZ>
static void launch_gemm(hipStream_t s, const GemmPlan& p, const GemmArgs& g, bool vec) {
  dim3 grid((unsigned)((g.M + p.bm - 1) / p.bm), (unsigned)((g.N + p.bn - 1) / p.bn), (unsigned)p.splits);
#define RS_GEMM(BMM, BNN, V) gemm_kernel<BMM, BNN, ALAY, BLAY, AZ, BZ, V><<<grid, 256, 0, s>>>(g)
  if (vec) {
    if (p.bm == 64 && p.bn == 64) RS_GEMM(64, 64, true);
    else if (p.bm == 64) RS_GEMM(64, 32, true);
    else if (p.bn == 64) RS_GEMM(32, 64, true);
    else RS_GEMM(32, 32, true);
  } else {
    if (p.bm == 64 && p.bn == 64) RS_GEMM(64, 64, false);
    else if (p.bm == 64) RS_GEMM(64, 32, false);
    else if (p.bn == 64) RS_GEMM(32, 64, false);
    else RS_GEMM(32, 32, false);
  }
#undef RS_GEMM
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

RS_API int rs_dense_fwd(void* stream, const float* X, int64_t M, int K, int64_t ldx,
                        const float* W, const float* bias, int N, int act, float* Y,
                        int64_t ldy) {
  if (!X || !W || !bias || !Y || M < 0 || K <= 0 || N <= 0 || ldx < K || ldy < N) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  GemmArgs g{X, ldx, nullptr, 0, W, N, nullptr, 0, M, N, K, 0, 0, EPI_FWD, act, bias, Y, ldy, 0, nullptr};
  GemmPlan p = plan_gemm(M, N, K, false);
  g.rchunk = p.rchunk;
  const bool vec = aligned16(X) && aligned16(W) && ldx % 4 == 0 && N % 4 == 0;
  launch_gemm<LAY_ROW, LAY_ROW, false, false>(rs_stream(stream), p, g, vec);
  return rs_status_after_launch();
}

RS_API int rs_dense_bwd_data(void* stream, const float* dY, int64_t lddy, const float* Y,
                             int64_t ldy, int act, const float* W, int64_t M, int K, int N,
                             float* dX, int64_t lddx, int accumulate) {
  if (!dY || !Y || !W || !dX || M < 0 || K <= 0 || N <= 0 || lddx < K) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
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

RS_API int64_t rs_dense_bwd_weight_workspace_floats(int64_t M, int K, int N) {
  const GemmPlan p = plan_gemm(K, N, M, true);
  return (int64_t)p.splits * ((int64_t)K * N + N);
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
  // C[K, N] = sum_m X[m][k] dZ[m][n]: A(k, m) = X[m * ldx + k] (column layout), B = dZ rows
  const GemmPlan p = plan_gemm(K, N, M, true);
  const bool split = p.splits > 1;
  if (split && (!workspace || workspace_floats < (int64_t)p.splits * ((int64_t)K * N + N)))
    return RS_ERR_ARG;
  GemmArgs g{X, ldx, nullptr, 0, dY, lddy, Y, ldy, K, N, M, p.rchunk, act,
             split ? EPI_PARTIAL : EPI_STORE, 0, nullptr, split ? workspace : dW, N, accumulate,
             db};
  const bool vec = aligned16(X) && aligned16(dY) && aligned16(Y) && ldx % 4 == 0 && lddy % 4 == 0 &&
                   ldy % 4 == 0;
  launch_gemm<LAY_COL, LAY_ROW, false, true>(s, p, g, vec);
  if (split) {
    const int64_t total = (int64_t)K * N + N;
    launch_column_reduce(s, workspace, p.splits, total, total, (int64_t)K * N, dW, db, accumulate);
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
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const float sv = s[i];
    const float p = fminf(fmaxf(sv, lo), hi);
    const float yv = y[i];
    const float li = -yv * logf(p + log_eps) - (1.0f - yv) * logf(1.0f - p + log_eps);
    acc += li;
    if (p_out) p_out[i] = p;
    if (ds) {
      const float dp = (-yv / (p + log_eps) + (1.0f - yv) / (1.0f - p + log_eps)) * gs;
      ds[i] = (sv >= lo && sv <= hi) ? dp : 0.f;
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

RS_API int rs_bce_clip_loss(void* stream, const float* s, const float* y, int64_t M, int T,
                            float clip_lo, float clip_hi, float log_eps, const float* gscale,
                            float* p_out, float* loss, float* ds) {
  if (!s || !y || M <= 0 || T <= 0) return RS_ERR_ARG;
  bce_clip_kernel<<<1, 1024, 0, rs_stream(stream)>>>(s, y, M, T, clip_lo, clip_hi, log_eps, gscale,
                                                     p_out, loss, ds);
  return rs_status_after_launch();
}
