// H4/H5/H8/H9 MLP towers — Keras Dense(units, activation) on the CTR path, forward and backward.
//
// Reference call sites: autoint:36-52 (MultiLayerDense deep/logits towers),
// rank/multi_head/multidnn.py:60-64 (deep Dense(32, 16) relu), :80-127 (experts, gates, heads),
// rough_rank/layer.py:33-117 (DNN), staytime/VideoDnn.py:130-191 (experts / towers).
// Keras Dense = tensordot(x, kernel) + bias, then activation (kernel stored [in, out]).
//
// MI355X mapping: fp32 in / fp32 accumulate on the matrix cores (v_mfma_f32_16x16x4_f32: exact
// f32, a k-ordered fma chain, so the numerics equal an fp32 CPU dot product up to summation
// order).  64x64 block tile, 4 waves x (16 rows x 64 columns), K staged through LDS in 32-deep
// slabs with coalesced row loads.  Leading dimensions are explicit so a layer reads a slice of
// a concatenated activation and writes straight into its slot of the next concat (the
// tf.concat on autoint:44 costs nothing).
//   forward      Y  = act(X W + b)
//   backward     dZ = dY * act'(Y) (recomputed on load, never stored)
//                dX = dZ W^T       (optionally accumulated)
//                dW = X^T dZ, db = colsum(dZ): split over M chunks -> per-chunk partials ->
//                fixed-order reduce (deterministic, no float atomics)
#include "common.hpp"

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

constexpr int BT = 64;  // block tile (rows and columns)
constexpr int BK = 32;  // K slab

// ------------------------------- forward ------------------------------------------------------
// Block = 16 rows x 64 columns, 4 waves splitting K (a batch-sized M with N <= 64 and K up to a
// few thousand is the shape of every tower layer on the path, so the grid is M/16 blocks rather
// than M/64).  X rows are staged through LDS in 256-deep slabs (coalesced); W is read straight
// from L2 (it is a few KB to a few hundred KB and shared by every block).  The 4 wave partials
// are summed in wave order (deterministic), then bias + activation.
constexpr int FM = 16;    // rows per block
constexpr int FKS = 256;  // K slab staged in LDS

__global__ void __launch_bounds__(256) dense_fwd_kernel(const float* __restrict__ X, int64_t M,
                                                        int K, int64_t ldx,
                                                        const float* __restrict__ W,
                                                        const float* __restrict__ bias, int N,
                                                        int act, float* __restrict__ Y,
                                                        int64_t ldy) {
  __shared__ float As[FM][FKS + 4];
  __shared__ float red[4][FM][BT + 1];
  const int64_t m_blk = (int64_t)blockIdx.x * FM;
  const int n_blk = blockIdx.y * BT;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int lr = l & 15, lk = l >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += FKS) {
    for (int t = threadIdx.x; t < FM * FKS; t += 256) {
      const int r = t / FKS, c = t % FKS;
      const int64_t m = m_blk + r;
      const int k = k0 + c;
      As[r][c] = (m < M && k < K) ? X[m * ldx + k] : 0.f;
    }
    __syncthreads();
    // wave w takes k-steps kk = w*4, w*4 + 16, ... of this slab (interleaved -> balanced tails)
    for (int kk = w * 4; kk < FKS && k0 + kk < K; kk += 16) {
      const int k = k0 + kk + lk;
      const float a = As[lr][kk + lk];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int n = n_blk + t * 16 + lr;
        const float bv = (k < K && n < N) ? W[(int64_t)k * N + n] : 0.f;
        acc[t] = mfma4(a, bv, acc[t]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][lk * 4 + r][t * 16 + lr] = acc[t][r];
  __syncthreads();
  for (int o = threadIdx.x; o < FM * BT; o += 256) {
    const int r = o / BT, c = o % BT;
    const int64_t m = m_blk + r;
    const int n = n_blk + c;
    if (m < M && n < N) {
      const float v = ((red[0][r][c] + red[1][r][c]) + red[2][r][c]) + red[3][r][c];
      Y[m * ldy + n] = act_fwd(v + bias[n], act);
    }
  }
}

// ------------------------------- backward: data ----------------------------------------------
// dX[m][k] (+)= sum_n dZ[m][n] W[k][n]
__global__ void __launch_bounds__(256) dense_bwd_data_kernel(
    const float* __restrict__ dY, int64_t lddy, const float* __restrict__ Y, int64_t ldy, int act,
    const float* __restrict__ W, int64_t M, int K, int N, float* __restrict__ dX, int64_t lddx,
    int accumulate) {
  __shared__ float As[BT][BK + 1];  // dZ[m][n]
  __shared__ float Bs[BK][BT + 1];  // W^T[n][k]
  const int64_t m_blk = (int64_t)blockIdx.x * BT;
  const int k_blk = blockIdx.y * BT;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int n0 = 0; n0 < N; n0 += BK) {
    for (int t = threadIdx.x; t < BT * BK; t += 256) {
      const int r = t / BK, c = t % BK;
      const int64_t m = m_blk + r;
      const int n = n0 + c;
      As[r][c] = (m < M && n < N) ? act_bwd(dY[m * lddy + n], Y[m * ldy + n], act) : 0.f;
    }
    for (int t = threadIdx.x; t < BK * BT; t += 256) {
      const int kr = t / BK, c = t % BK;  // coalesced along n within a W row
      const int k = k_blk + kr, n = n0 + c;
      Bs[c][kr] = (k < K && n < N) ? W[(int64_t)k * N + n] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const float a = As[w * 16 + (l & 15)][kk + (l >> 4)];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = mfma4(a, Bs[kk + (l >> 4)][t * 16 + (l & 15)], acc[t]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int k = k_blk + t * 16 + (l & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t m = m_blk + w * 16 + (l >> 4) * 4 + r;
      if (m < M && k < K) {
        float* d = dX + m * lddx + k;
        *d = accumulate ? (*d + acc[t][r]) : acc[t][r];
      }
    }
  }
}

// ------------------------------- backward: weights -------------------------------------------
// partial[chunk][k][n] = sum_{m in chunk} X[m][k] dZ[m][n];  partial[chunk][K*N + n] = colsum dZ
constexpr int MCH = 64;  // rows per M chunk (2 x 64 x 65 floats of LDS)

__global__ void __launch_bounds__(256) dense_bwd_weight_kernel(
    const float* __restrict__ X, int64_t ldx, const float* __restrict__ dY, int64_t lddy,
    const float* __restrict__ Y, int64_t ldy, int act, int64_t M, int K, int N,
    float* __restrict__ partials) {
  __shared__ float Xs[MCH][BT + 1];
  __shared__ float Zs[MCH][BT + 1];
  const int64_t m_blk = (int64_t)blockIdx.x * MCH;
  const int k_blk = blockIdx.y * BT;
  const int n_blk = blockIdx.z * BT;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int t = threadIdx.x; t < MCH * BT; t += 256) {
    const int r = t / BT, c = t % BT;
    const int64_t m = m_blk + r;
    const int k = k_blk + c, n = n_blk + c;
    Xs[r][c] = (m < M && k < K) ? X[m * ldx + k] : 0.f;
    Zs[r][c] = (m < M && n < N) ? act_bwd(dY[m * lddy + n], Y[m * ldy + n], act) : 0.f;
  }
  __syncthreads();
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int mm = 0; mm < MCH; mm += 4) {
    const float a = Xs[mm + (l >> 4)][w * 16 + (l & 15)];
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma4(a, Zs[mm + (l >> 4)][t * 16 + (l & 15)], acc[t]);
  }
  float* part = partials + (int64_t)blockIdx.x * ((int64_t)K * N + N);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = n_blk + t * 16 + (l & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k_blk + w * 16 + (l >> 4) * 4 + r;
      if (k < K && n < N) part[(int64_t)k * N + n] = acc[t][r];
    }
  }
  if (blockIdx.y == 0) {  // column sums of dZ (bias gradient), in row order
    for (int c = threadIdx.x; c < BT; c += 256) {
      const int n = n_blk + c;
      if (n < N) {
        float s = 0.f;
        for (int r = 0; r < MCH; ++r) s += Zs[r][c];
        part[(int64_t)K * N + n] = s;
      }
    }
  }
}

RS_API int rs_dense_fwd(void* stream, const float* X, int64_t M, int K, int64_t ldx,
                        const float* W, const float* bias, int N, int act, float* Y,
                        int64_t ldy) {
  if (!X || !W || !bias || !Y || M < 0 || K <= 0 || N <= 0 || ldx < K || ldy < N) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  dim3 grid((unsigned)((M + FM - 1) / FM), (unsigned)((N + BT - 1) / BT));
  dense_fwd_kernel<<<grid, 256, 0, rs_stream(stream)>>>(X, M, K, ldx, W, bias, N, act, Y, ldy);
  return rs_status_after_launch();
}

RS_API int rs_dense_bwd_data(void* stream, const float* dY, int64_t lddy, const float* Y,
                             int64_t ldy, int act, const float* W, int64_t M, int K, int N,
                             float* dX, int64_t lddx, int accumulate) {
  if (!dY || !Y || !W || !dX || M < 0 || K <= 0 || N <= 0 || lddx < K) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  dim3 grid((unsigned)((M + BT - 1) / BT), (unsigned)((K + BT - 1) / BT));
  dense_bwd_data_kernel<<<grid, 256, 0, rs_stream(stream)>>>(dY, lddy, Y, ldy, act, W, M, K, N,
                                                              dX, lddx, accumulate);
  return rs_status_after_launch();
}

RS_API int64_t rs_dense_bwd_weight_workspace_floats(int64_t M, int K, int N) {
  const int64_t nchunks = (M + MCH - 1) / MCH;
  return (nchunks < 1 ? 1 : nchunks) * ((int64_t)K * N + N);
}

RS_API int rs_dense_bwd_weight(void* stream, const float* X, int64_t ldx, const float* dY,
                               int64_t lddy, const float* Y, int64_t ldy, int act, int64_t M,
                               int K, int N, float* dW, float* db, int accumulate,
                               float* workspace, int64_t workspace_floats) {
  if (!X || !dY || !Y || !dW || !db || !workspace || M < 0 || K <= 0 || N <= 0) return RS_ERR_ARG;
  if (workspace_floats < rs_dense_bwd_weight_workspace_floats(M, K, N)) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
  const int nchunks = (int)((M + MCH - 1) / MCH);
  if (nchunks > 0) {
    dim3 grid((unsigned)nchunks, (unsigned)((K + BT - 1) / BT), (unsigned)((N + BT - 1) / BT));
    dense_bwd_weight_kernel<<<grid, 256, 0, s>>>(X, ldx, dY, lddy, Y, ldy, act, M, K, N,
                                                 workspace);
  }
  const int64_t total = (int64_t)K * N + N;
  launch_column_reduce(s, workspace, nchunks, total, total, (int64_t)K * N, dW, db, accumulate);
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
