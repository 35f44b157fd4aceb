// H5/H8/H9/H10 — the tower-side ops around the MLP GEMMs (csrc/dense.hip), each fused into one
// HBM pass over its rows, forward and backward:
//
//   gate_mix     MMOE / PLE / multi_head / staytime MMoE combine: out_t = sum_k softmax(g_t)_k *
//                act(expert_{sel[t,k]}) (rough_rank/layer.py:155-166, 212-226;
//                rank/multi_head/multidnn.py:95-120; staytime/VideoDnn.py:150-164).  Experts and
//                gate logits come straight out of ONE concatenated GEMM when they share an input
//                (all experts + all gates of a layer are one [K, sum N] Dense), so the mixture
//                kernel is the only extra pass.
//   cross        CrossNet (rough_rank/layer.py:236-270) == DeepCrossLayer (staytime/layer.py:44-80):
//                x_{l+1} = x0 * (x_l . w_l) + b_l + x_l, evaluated in closed form (one batched
//                reduction per row).
//   fm           FMLayer (staytime/layer.py:83-116, rank/finish/videodnn.py:23-52) and the SENet
//                reweight + FM cross term of staytime/VideoDnn.py:81-115: y_f = x_f * a_f,
//                cross = (sum_f y_f)^2 - sum_f y_f^2, fm = 0.5 * sum_e cross.
//   ffm          ffm_block (staytime/VideoDnn.py:11-25,118-120): per (user, item) field pair,
//                Dense(8)(x) * Dense(8)(y); plus the user x item multiply-ReLU (:99-105).
//   mul          ppnet gating deep * (scale * gate) (staytime/VideoDnn.py:135-146).
//   softmax_kl   400-bin staytime head softmax + expected bins (:168-179) and custom_kl_loss
//                (staytime/model.py:20-30), fused forward + backward.
//   rowdot       Similarity (rough_rank/layer.py:6-30); mse_rows: KDLoss (:272-279).
//
// All reductions over rows are per-block partials + column_reduce (fixed order, deterministic).
#include "common.hpp"

namespace rs_tw {

enum { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2 };

__device__ __forceinline__ float act_f(float z, int act) {
  if (act == ACT_RELU) return fmaxf(z, 0.f);
  if (act == ACT_SIGMOID) return 1.0f / (1.0f + expf(-z));
  return z;
}
// d/dz given z (relu: TF ReluGrad on the output, y > 0 <=> z > 0)
__device__ __forceinline__ float act_d(float z, int act) {
  if (act == ACT_RELU) return z > 0.f ? 1.f : 0.f;
  if (act == ACT_SIGMOID) { const float y = 1.0f / (1.0f + expf(-z)); return y * (1.f - y); }
  return 1.f;
}

// Block-wide sum of one float per thread (256 threads = 4 waves); `red` = 8 floats of LDS,
// double-buffered by `phase` so back-to-back reductions need one barrier each.
__device__ __forceinline__ float block_sum256(float v, float* red, int phase) {
  v = group_sum<64>(v);
  float* r = red + (phase & 1) * 4;
  if (lane_id() == 0) r[wave_id()] = v;
  __syncthreads();
  return (r[0] + r[1]) + (r[2] + r[3]);
}

// =============================================================================================
// gate_mix
// =============================================================================================
constexpr int GM_MAXSEL = 16;
constexpr int GM_MAXCH = 4;  // D <= 256

struct GM {
  const float* E; int64_t lde; int e_act;
  const float* G; int64_t ldg;
  int64_t M; int n_exp, D, n_task, n_sel;
  const int32_t* sel;
};

// Per row: the activations of the row's experts are staged once in LDS (each lane stages and
// reads only its own columns d = dl + c DP, so no barrier) when `stage` (RPB n_exp D floats of
// dynamic LDS), and each task's gate softmax is formed once in registers (one exp per gate):
// every task re-reads every selected expert, and the per-(task, expert, column) exp and global
// load made this kernel latency-bound.  p_k = exp(g_k - max) / sum exactly as before.
template <int DP>
__global__ void __launch_bounds__(256) gate_mix_fwd_kernel(GM a, float* __restrict__ Y, int64_t ldy,
                                                           float* __restrict__ P, int64_t ldp,
                                                           int stage) {
  constexpr int RPB = 256 / DP;
  extern __shared__ float act_all[];  // [RPB][n_exp][D] when stage
  __shared__ int32_t sel[GM_MAXSEL * 8];
  for (int i = threadIdx.x; i < a.n_task * a.n_sel; i += blockDim.x) sel[i] = a.sel[i];
  __syncthreads();
  const int rl = threadIdx.x / DP, dl = threadIdx.x % DP;
  const int nch = (a.D + DP - 1) / DP;
  float* ar = act_all + (int64_t)rl * a.n_exp * a.D;
  for (int64_t m = (int64_t)blockIdx.x * RPB + rl; m < a.M; m += (int64_t)gridDim.x * RPB) {
    const float* g = a.G + m * a.ldg;
    const float* e = a.E + m * a.lde;
    if (stage) {
      for (int x = 0; x < a.n_exp; ++x)
#pragma unroll
        for (int c = 0; c < GM_MAXCH; ++c) {
          const int d = dl + c * DP;
          if (c < nch && d < a.D) ar[x * a.D + d] = act_f(e[(int64_t)x * a.D + d], a.e_act);
        }
    }
    for (int t = 0; t < a.n_task; ++t) {
      float pk[GM_MAXSEL];
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) {
        pk[k] = k < a.n_sel ? g[t * a.n_sel + k] : -INFINITY;
        mx = fmaxf(mx, pk[k]);
      }
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) {
        pk[k] = k < a.n_sel ? expf(pk[k] - mx) : 0.f;
        sum += pk[k];
      }
      const float inv = 1.0f / sum;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) pk[k] *= inv;
#pragma unroll
      for (int c = 0; c < GM_MAXCH; ++c) {
        const int d = dl + c * DP;
        if (c >= nch || d >= a.D) continue;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < GM_MAXSEL; ++k) {
          if (k < a.n_sel) {
            const int x = sel[t * a.n_sel + k];
            const float v = stage ? ar[x * a.D + d] : act_f(e[(int64_t)x * a.D + d], a.e_act);
            acc = fmaf(pk[k], v, acc);
          }
        }
        Y[m * ldy + (int64_t)t * a.D + d] = acc;
      }
      if (P) {
#pragma unroll
        for (int k = 0; k < GM_MAXSEL; ++k)
          if (k < a.n_sel && (k % DP) == dl) P[m * ldp + t * a.n_sel + k] = pk[k];
      }
    }
  }
}

template <int DP>
__global__ void __launch_bounds__(256) gate_mix_bwd_kernel(GM a, const float* __restrict__ dY,
                                                           int64_t lddy, float* __restrict__ dE,
                                                           int64_t ldde, float* __restrict__ dG,
                                                           int64_t lddg, int stage) {
  constexpr int RPB = 256 / DP;
  extern __shared__ float acc_all[];  // [RPB][n_exp][D] (+ [RPB][n_exp][D] activations: stage)
  __shared__ int32_t sel[GM_MAXSEL * 8];
  for (int i = threadIdx.x; i < a.n_task * a.n_sel; i += blockDim.x) sel[i] = a.sel[i];
  __syncthreads();
  const int rl = threadIdx.x / DP, dl = threadIdx.x % DP;
  float* acc = acc_all + (int64_t)rl * a.n_exp * a.D;
  float* ar = acc_all + (int64_t)(RPB + rl) * a.n_exp * a.D;
  const int nch = (a.D + DP - 1) / DP;
  // every thread walks the same number of rows (so the group reductions stay converged)
  const int64_t nrow_iter = (a.M + (int64_t)gridDim.x * RPB - 1) / ((int64_t)gridDim.x * RPB);
  for (int64_t it = 0; it < nrow_iter; ++it) {
    const int64_t m = ((int64_t)it * gridDim.x + blockIdx.x) * RPB + rl;
    const bool live = m < a.M;
    const int64_t mm = live ? m : 0;
    const float* g = a.G + mm * a.ldg;
    const float* e = a.E + mm * a.lde;
    for (int x = 0; x < a.n_exp; ++x)
#pragma unroll
      for (int c = 0; c < GM_MAXCH; ++c) {
        const int d = dl + c * DP;
        if (c < nch && d < a.D) {
          acc[x * a.D + d] = 0.f;
          if (stage) ar[x * a.D + d] = act_f(e[(int64_t)x * a.D + d], a.e_act);
        }
      }
    for (int t = 0; t < a.n_task; ++t) {
      float dy[GM_MAXCH];
#pragma unroll
      for (int c = 0; c < GM_MAXCH; ++c) {
        const int d = dl + c * DP;
        dy[c] = (c < nch && d < a.D && live) ? dY[mm * lddy + (int64_t)t * a.D + d] : 0.f;
      }
      float p[GM_MAXSEL], s[GM_MAXSEL];
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) {
        p[k] = k < a.n_sel ? g[t * a.n_sel + k] : -INFINITY;
        mx = fmaxf(mx, p[k]);
      }
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) {
        p[k] = k < a.n_sel ? expf(p[k] - mx) : 0.f;
        sum += p[k];
      }
      const float inv = 1.0f / sum;
      float ps = 0.f;
#pragma unroll
      for (int k = 0; k < GM_MAXSEL; ++k) {
        p[k] *= inv;
        s[k] = 0.f;
        if (k < a.n_sel) {
          const int64_t col = (int64_t)sel[t * a.n_sel + k] * a.D;
          float part = 0.f;
#pragma unroll
          for (int c = 0; c < GM_MAXCH; ++c) {
            const int d = dl + c * DP;
            if (c < nch && d < a.D)
              part = fmaf(dy[c], stage ? ar[col + d] : act_f(e[col + d], a.e_act), part);
          }
          s[k] = group_sum<DP>(part);
          ps = fmaf(p[k], s[k], ps);
#pragma unroll
          for (int c = 0; c < GM_MAXCH; ++c) {
            const int d = dl + c * DP;
            if (c < nch && d < a.D) acc[sel[t * a.n_sel + k] * a.D + d] += p[k] * dy[c];
          }
        }
      }
      if (live && dG) {
#pragma unroll
        for (int k = 0; k < GM_MAXSEL; ++k)
          if (k < a.n_sel && (k % DP) == dl) dG[m * lddg + t * a.n_sel + k] = p[k] * (s[k] - ps);
      }
    }
    if (live && dE) {
      for (int x = 0; x < a.n_exp; ++x)
        for (int c = 0; c < nch; ++c) {
          const int d = dl + c * DP;
          if (d < a.D) {
            const float z = e[(int64_t)x * a.D + d];
            dE[m * ldde + (int64_t)x * a.D + d] = acc[x * a.D + d] * act_d(z, a.e_act);
          }
        }
    }
  }
}

// =============================================================================================
// cross (CrossNet / DeepCrossLayer)
// =============================================================================================
constexpr int CR_MAXL = 4;

// Closed form of the recurrence x_{l+1} = x0 (x_l . w_l) + b_l + x_l: by induction every layer
// is x_l = A_l x0 + B_l with a per-row scalar A_l and a row-independent vector
// B_l = sum_{k<l} b_k, so with q_l = x0 . w_l and the per-model constants c_l = B_l . w_l
//     s_l = x_l . w_l = A_l q_l + c_l,   A_0 = 1,   A_{l+1} = A_l + s_l,   y = A_L x0 + B_L.
// One batched block reduction per row (the L dots q_l) replaces L dependent ones.
// Backward (g_l = dL/dx_{l+1}, g_{L-1} = dY):  ds_l = g_l . x0 = p + sum_{k>l} ds_k q_k with
// p = dY . x0, so the whole chain is again ONE batched reduction {q_l, p} plus scalar algebra:
//     dX0  = A_L dY + sum_l (A_l ds_l) w_l
//     dW_l = sum_rows (A_l ds_l) x0 + B_l sum_rows ds_l
//     db_l = sum_rows dY + sum_{k>l} w_k sum_rows ds_k.
// The row pass writes dX0 and the per-row scalars (A_l ds_l, ds_l); a column pass forms the three
// row sums in fixed order (per-split partials) and a finalize pass assembles dW and db.

// Block-wide sums of K floats per thread (256 threads = 4 waves); `red` = 2 * 4 * K floats of LDS,
// double-buffered by `phase` like block_sum256.
template <int K>
__device__ __forceinline__ void block_sumk(float (&v)[K], float* red, int phase) {
  float* r = red + (phase & 1) * 4 * K;
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = group_sum<64>(v[k]);
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) r[wave_id() * K + k] = v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = (r[k] + r[K + k]) + (r[2 * K + k] + r[3 * K + k]);
}

// w_l in registers, c_l = B_l . w_l (block-reduced once), B_L returned in `bl`.
// Thread owns columns c = threadIdx.x + 256 v (v < NV).
template <int NV, int L>
__device__ __forceinline__ void cross_setup(const float* __restrict__ W,
                                            const float* __restrict__ bias, int D,
                                            float (&w)[L][NV], float (&cl)[L], float (&bl)[NV],
                                            float* red) {
#pragma unroll
  for (int v = 0; v < NV; ++v) bl[v] = 0.f;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    float part = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + 256 * v;
      w[l][v] = c < D ? W[(int64_t)l * D + c] : 0.f;
      part = fmaf(bl[v], w[l][v], part);
      bl[v] += c < D ? bias[(int64_t)l * D + c] : 0.f;
    }
    cl[l] = part;
  }
  block_sumk<L>(cl, red, 0);  // red: its own 4 L floats, not the row loop's buffer
}

// s_l recursion: A[l] = A_l for l <= L
template <int L>
__device__ __forceinline__ void cross_scales(const float (&q)[L], const float (&cl)[L],
                                             float (&A)[L + 1]) {
  A[0] = 1.f;
#pragma unroll
  for (int l = 0; l < L; ++l) A[l + 1] = A[l] + fmaf(A[l], q[l], cl[l]);
}

template <int NV, int L>
__global__ void __launch_bounds__(256) cross_fwd_kernel(const float* __restrict__ X0, int64_t ldx,
                                                        int64_t M, int D,
                                                        const float* __restrict__ W,
                                                        const float* __restrict__ bias,
                                                        float* __restrict__ Y, int64_t ldy) {
  __shared__ float red0[4 * L], red[2 * 4 * L];
  float w[L][NV], cl[L], bl[NV];
  cross_setup<NV, L>(W, bias, D, w, cl, bl, red0);
  int phase = 0;
  for (int64_t m = blockIdx.x; m < M; m += gridDim.x) {
    float x0[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + 256 * v;
      x0[v] = c < D ? X0[m * ldx + c] : 0.f;
    }
    float q[L];
#pragma unroll
    for (int l = 0; l < L; ++l) {
      q[l] = 0.f;
#pragma unroll
      for (int v = 0; v < NV; ++v) q[l] = fmaf(x0[v], w[l][v], q[l]);
    }
    block_sumk<L>(q, red, phase++);
    float A[L + 1];
    cross_scales<L>(q, cl, A);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + 256 * v;
      if (c < D) Y[m * ldy + c] = fmaf(A[L], x0[v], bl[v]);
    }
  }
}

// Row pass of the backward: dX0 and coef[m] = [A_l ds_l (l < L) | ds_l (l < L)].
template <int NV, int L>
__global__ void __launch_bounds__(256) cross_bwd_rows_kernel(
    const float* __restrict__ X0, int64_t ldx, int64_t M, int D, const float* __restrict__ W,
    const float* __restrict__ bias, const float* __restrict__ dY, int64_t lddy,
    float* __restrict__ dX0, int64_t lddx, int dx_accumulate, float* __restrict__ coef) {
  __shared__ float red0[4 * L], red[2 * 4 * (L + 1)];
  float w[L][NV], cl[L], bl[NV];
  cross_setup<NV, L>(W, bias, D, w, cl, bl, red0);
  int phase = 0;
  for (int64_t m = blockIdx.x; m < M; m += gridDim.x) {
    float x0[NV], g[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + 256 * v;
      x0[v] = c < D ? X0[m * ldx + c] : 0.f;
      g[v] = c < D ? dY[m * lddy + c] : 0.f;
    }
    float r[L + 1];  // q_0 .. q_{L-1}, p
#pragma unroll
    for (int l = 0; l <= L; ++l) r[l] = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int l = 0; l < L; ++l) r[l] = fmaf(x0[v], w[l][v], r[l]);
      r[L] = fmaf(g[v], x0[v], r[L]);
    }
    block_sumk<L + 1>(r, red, phase++);
    float q[L];
#pragma unroll
    for (int l = 0; l < L; ++l) q[l] = r[l];
    float A[L + 1];
    cross_scales<L>(q, cl, A);
    float ds[L], al[L];
#pragma unroll
    for (int l = L - 1; l >= 0; --l) {
      float d = r[L];
#pragma unroll
      for (int k = l + 1; k < L; ++k) d = fmaf(ds[k], q[k], d);
      ds[l] = d;
      al[l] = A[l] * d;
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int c = threadIdx.x + 256 * v;
      if (c < D) {
        float val = A[L] * g[v];
#pragma unroll
        for (int l = 0; l < L; ++l) val = fmaf(al[l], w[l][v], val);
        float* dst = dX0 + m * lddx + c;
        *dst = dx_accumulate ? *dst + val : val;
      }
    }
    if (threadIdx.x < 2 * L) {
      float o = 0.f;
#pragma unroll
      for (int l = 0; l < L; ++l) {
        if (threadIdx.x == l) o = al[l];
        if (threadIdx.x == L + l) o = ds[l];
      }
      coef[m * 2 * L + threadIdx.x] = o;
    }
  }
}

// Column pass: split s of gridDim.y sums rows [m0, m1) of  x0 * (A_l ds_l)  (l < L) and dY into
// part[s][(L+1) D], and (column tile 0) the row sums of ds_l into part[s][(L+1) D + l].
template <int L>
__global__ void __launch_bounds__(256) cross_bwd_cols_kernel(
    const float* __restrict__ X0, int64_t ldx, int64_t M, int D, const float* __restrict__ dY,
    int64_t lddy, const float* __restrict__ coef, int64_t rows_per_split,
    float* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per_split;
  const int64_t m1 = m0 + rows_per_split < M ? m0 + rows_per_split : M;
  const bool col = c < D;
  float acc[L + 1], t[L];
#pragma unroll
  for (int l = 0; l <= L; ++l) acc[l] = 0.f;
#pragma unroll
  for (int l = 0; l < L; ++l) t[l] = 0.f;
  int64_t m = m0;
  for (; m + 4 <= m1; m += 4) {
    float x[4], g[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] = col ? X0[(m + u) * ldx + c] : 0.f;
      g[u] = col ? dY[(m + u) * lddy + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float* cf = coef + (m + u) * 2 * L;
#pragma unroll
      for (int l = 0; l < L; ++l) { acc[l] = fmaf(x[u], cf[l], acc[l]); t[l] += cf[L + l]; }
      acc[L] += g[u];
    }
  }
  for (; m < m1; ++m) {
    const float x = col ? X0[m * ldx + c] : 0.f;
    const float g = col ? dY[m * lddy + c] : 0.f;
    const float* cf = coef + m * 2 * L;
#pragma unroll
    for (int l = 0; l < L; ++l) { acc[l] = fmaf(x, cf[l], acc[l]); t[l] += cf[L + l]; }
    acc[L] += g;
  }
  float* pr = part + (int64_t)blockIdx.y * ((L + 1) * (int64_t)D + L);
  if (col) {
#pragma unroll
    for (int l = 0; l <= L; ++l) pr[(int64_t)l * D + c] = acc[l];
  }
  if (blockIdx.x == 0 && threadIdx.x < L) {
    float o = 0.f;
#pragma unroll
    for (int l = 0; l < L; ++l)
      if (threadIdx.x == l) o = t[l];
    pr[(int64_t)(L + 1) * D + threadIdx.x] = o;
  }
}

// Finalize: dW_l = R_l + B_l T_l, db_l = S + sum_{k>l} w_k T_k (R, S, T summed over the splits)
// -> dparams [dW (L D) | db (L D)], written or accumulated.  Block = 64 columns x 16 split groups
// (thread group g sums splits g, g+16, ... in order, the groups are combined in g order, as
// column_reduce_kernel): a fixed summation order.
template <int L>
__global__ void __launch_bounds__(64 * 16) cross_bwd_final_kernel(
    const float* __restrict__ part, int nsplit, int D, const float* __restrict__ W,
    const float* __restrict__ bias, float* __restrict__ dparams, int accumulate) {
  constexpr int G = 16;
  __shared__ float red[G][L + 1][64];
  __shared__ float redt[G][L];
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const int64_t stride = (L + 1) * (int64_t)D + L;
  float R[L + 1], T[L];
#pragma unroll
  for (int l = 0; l <= L; ++l) R[l] = 0.f;
#pragma unroll
  for (int l = 0; l < L; ++l) T[l] = 0.f;
#pragma unroll 4
  for (int s = g; s < nsplit; s += G) {
    const float* pr = part + s * stride;
    if (c < D) {
#pragma unroll
      for (int l = 0; l <= L; ++l) R[l] += pr[(int64_t)l * D + c];
    }
#pragma unroll
    for (int l = 0; l < L; ++l) T[l] += pr[(int64_t)(L + 1) * D + l];
  }
#pragma unroll
  for (int l = 0; l <= L; ++l) red[g][l][lc] = R[l];
  if (lc < L) {
#pragma unroll
    for (int l = 0; l < L; ++l)
      if (lc == l) redt[g][l] = T[l];
  }
  __syncthreads();
  if (g != 0 || c >= D) return;
#pragma unroll
  for (int k = 1; k < G; ++k) {
#pragma unroll
    for (int l = 0; l <= L; ++l) R[l] += red[k][l][lc];
  }
#pragma unroll
  for (int l = 0; l < L; ++l) {
    float t = redt[0][l];
#pragma unroll
    for (int k = 1; k < G; ++k) t += redt[k][l];
    T[l] = t;
  }
  float B = 0.f;
#pragma unroll
  for (int l = 0; l < L; ++l) {
    const float dw = fmaf(B, T[l], R[l]);
    float db = R[L];
#pragma unroll
    for (int k = l + 1; k < L; ++k) db = fmaf(W[(int64_t)k * D + c], T[k], db);
    float* pw = dparams + (int64_t)l * D + c;
    float* pb = dparams + (int64_t)(L + l) * D + c;
    *pw = accumulate ? *pw + dw : dw;
    *pb = accumulate ? *pb + db : db;
    B += bias[(int64_t)l * D + c];
  }
}

static int64_t cross_rows_per_split(int64_t M) {
  const int64_t rps = 32;  // B = 2048, D = 1712: 64 splits x 7 column tiles = 448 blocks
  const int64_t nsplit = (M + rps - 1) / rps;
  return nsplit <= 128 ? rps : (M + 127) / 128;
}
static int cross_nsplit(int64_t M) {
  const int64_t rps = cross_rows_per_split(M);
  return (int)((M + rps - 1) / rps);
}

// =============================================================================================
// fm (+ optional per-field scale = SENet reweight)
// =============================================================================================
struct FM {
  const float* X; int64_t ldx; int64_t fsx;      // x[m*ldx + f*fsx + e]
  int64_t M; int F, E;
  const float* A; int64_t lda;                   // scale a[m*lda + f] (nullable)
  float as;                                      // y = x * (as * a)
};

template <int EW>
__global__ void __launch_bounds__(256) fm_fwd_kernel(FM a, float* __restrict__ Y, int64_t ldy,
                                                     float* __restrict__ C, int64_t ldc,
                                                     float* __restrict__ FMo, int64_t ldf) {
  constexpr int NG = 64 / EW;
  const int l = lane_id(), e = l % EW, fg = l / EW;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < a.M; m += (int64_t)gridDim.x * 4) {
    float S = 0.f, Q = 0.f;
    if (e < a.E) {
#pragma unroll 8
      for (int f = fg; f < a.F; f += NG) {
        float y = a.X[m * a.ldx + (int64_t)f * a.fsx + e];
        if (a.A) y *= a.as * a.A[m * a.lda + f];
        if (Y) Y[m * ldy + (int64_t)f * a.E + e] = y;
        S += y;
        Q = fmaf(y, y, Q);
      }
    }
#pragma unroll
    for (int o = EW; o < 64; o <<= 1) {
      S += __shfl_xor(S, o, 64);
      Q += __shfl_xor(Q, o, 64);
    }
    const float cr = S * S - Q;
    if (C && fg == 0 && e < a.E) C[m * ldc + e] = cr;
    if (FMo) {
      const float t = group_sum<EW>(e < a.E ? cr : 0.f);
      if (l == 0) FMo[m * ldf] = 0.5f * t;
    }
  }
}

template <int EW>
__global__ void __launch_bounds__(256) fm_bwd_kernel(FM a, const float* __restrict__ dY,
                                                     int64_t lddy, const float* __restrict__ dC,
                                                     int64_t lddc, const float* __restrict__ dFM,
                                                     int64_t lddf, float* __restrict__ dX,
                                                     int64_t lddx, int64_t fsdx, int dx_accumulate,
                                                     float* __restrict__ dA, int64_t ldda) {
  constexpr int NG = 64 / EW;
  const int l = lane_id(), e = l % EW, fg = l / EW;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < a.M; m += (int64_t)gridDim.x * 4) {
    float S = 0.f;
    if (e < a.E) {
      for (int f = fg; f < a.F; f += NG) {
        float y = a.X[m * a.ldx + (int64_t)f * a.fsx + e];
        if (a.A) y *= a.as * a.A[m * a.lda + f];
        S += y;
      }
    }
#pragma unroll
    for (int o = EW; o < 64; o <<= 1) S += __shfl_xor(S, o, 64);
    const float dc = (dC && e < a.E) ? dC[m * lddc + e] : 0.f;
    const float dfm = dFM ? dFM[m * lddf] : 0.f;
    // F is the same for every lane group; loop over field rounds so group reductions converge
    for (int f0 = 0; f0 < a.F; f0 += NG) {
      const int f = f0 + fg;
      const bool ok = f < a.F && e < a.E;
      float x = 0.f, sc = 1.f, dyt = 0.f;
      if (ok) {
        x = a.X[m * a.ldx + (int64_t)f * a.fsx + e];
        if (a.A) sc = a.as * a.A[m * a.lda + f];
        const float y = x * sc;
        // d/dy of cross_e = 2 (S_e - y), of fm = (S_e - y)
        dyt = (dY ? dY[m * lddy + (int64_t)f * a.E + e] : 0.f) + (2.f * dc + dfm) * (S - y);
      }
      if (dX && ok) {
        float* dst = dX + m * lddx + (int64_t)f * fsdx + e;
        const float v = dyt * sc;
        *dst = dx_accumulate ? *dst + v : v;
      }
      if (dA) {
        const float t = group_sum<EW>(dyt * x);
        if (e == 0 && f < a.F) dA[m * ldda + f] = a.as * t;
      }
    }
  }
}

// =============================================================================================
// ffm + user x item multiply-ReLU
// =============================================================================================
constexpr int FF_E = 16;      // field width (general inputs are the 0:16 column slice)
constexpr int FF_MAXF = 8;    // user + item fields

struct FFM {
  const float* X; int64_t ldx;                 // field f at column cols[f] (user fields first)
  int64_t M; int NU, NI, Dff;
  const int32_t* cols;
  const float *Wx, *bx, *Wy, *by;              // [P][E][Dff], [P][Dff]
};

__global__ void __launch_bounds__(256) ffm_fwd_kernel(FFM a, float* __restrict__ Y, int64_t ldy,
                                                      float* __restrict__ Mu, int64_t ldm) {
  extern __shared__ float sw[];  // Wx | bx | Wy | by
  const int P = a.NU * a.NI, nw = P * FF_E * a.Dff, nb = P * a.Dff;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) { sw[i] = a.Wx[i]; sw[nw + nb + i] = a.Wy[i]; }
  for (int i = threadIdx.x; i < nb; i += blockDim.x) { sw[nw + i] = a.bx[i]; sw[2 * nw + nb + i] = a.by[i]; }
  __shared__ int32_t cols[FF_MAXF];
  if (threadIdx.x < a.NU + a.NI) cols[threadIdx.x] = a.cols[threadIdx.x];
  __syncthreads();
  const float* Wx = sw; const float* bx = sw + nw; const float* Wy = sw + nw + nb;
  const float* by = sw + 2 * nw + nb;
  const int l = lane_id();
  const int nout = P * a.Dff;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < a.M; m += (int64_t)gridDim.x * 4) {
    const float* row = a.X + m * a.ldx;
    for (int o = l; o < nout; o += 64) {
      const int p = o / a.Dff, c = o % a.Dff;
      const int xi = p / a.NI, yi = p % a.NI;
      const float* xe = row + cols[xi];
      const float* ye = row + cols[a.NU + yi];
      float xo = bx[p * a.Dff + c], yo = by[p * a.Dff + c];
#pragma unroll
      for (int e = 0; e < FF_E; ++e) {
        xo = fmaf(xe[e], Wx[(p * FF_E + e) * a.Dff + c], xo);
        yo = fmaf(ye[e], Wy[(p * FF_E + e) * a.Dff + c], yo);
      }
      Y[m * ldy + o] = xo * yo;
    }
    if (Mu) {
      for (int o = l; o < a.NU * FF_E; o += 64) {
        const int i = o / FF_E, e = o % FF_E;
        Mu[m * ldm + o] = fmaxf(row[cols[i] + e] * row[cols[a.NU + i] + e], 0.f);
      }
    }
  }
}

// Backward: phase 1 (lane = output o): dxo/dyo into LDS and the per-lane dW/db accumulators;
// phase 2 (lane = (field, e)): dx of each field = sum over its pairs (fixed order) + multiply.
constexpr int FF_MAXOUT = 2;  // outputs per lane: P * Dff <= 128

__global__ void __launch_bounds__(256) ffm_bwd_kernel(FFM a, const float* __restrict__ dY,
                                                      int64_t lddy, const float* __restrict__ dMu,
                                                      int64_t lddm, float* __restrict__ dX,
                                                      int64_t lddx, int dx_accumulate,
                                                      float* __restrict__ part) {
  extern __shared__ float sw[];  // Wx | bx | Wy | by | per-wave dxo/dyo [4][2][P*Dff]
  const int P = a.NU * a.NI, nw = P * FF_E * a.Dff, nb = P * a.Dff;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) { sw[i] = a.Wx[i]; sw[nw + nb + i] = a.Wy[i]; }
  for (int i = threadIdx.x; i < nb; i += blockDim.x) { sw[nw + i] = a.bx[i]; sw[2 * nw + nb + i] = a.by[i]; }
  __shared__ int32_t cols[FF_MAXF];
  if (threadIdx.x < a.NU + a.NI) cols[threadIdx.x] = a.cols[threadIdx.x];
  __syncthreads();
  const float* Wx = sw; const float* bx = sw + nw; const float* Wy = sw + nw + nb;
  const float* by = sw + 2 * nw + nb;
  float* dxo_s = sw + 2 * (nw + nb) + wave_id() * 2 * nb;
  float* dyo_s = dxo_s + nb;
  const int l = lane_id();
  const int nout = P * a.Dff;
  float gWx[FF_MAXOUT][FF_E], gWy[FF_MAXOUT][FF_E], gbx[FF_MAXOUT], gby[FF_MAXOUT];
#pragma unroll
  for (int j = 0; j < FF_MAXOUT; ++j) {
    gbx[j] = gby[j] = 0.f;
#pragma unroll
    for (int e = 0; e < FF_E; ++e) gWx[j][e] = gWy[j][e] = 0.f;
  }
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < a.M; m += (int64_t)gridDim.x * 4) {
    const float* row = a.X + m * a.ldx;
#pragma unroll
    for (int j = 0; j < FF_MAXOUT; ++j) {
      const int o = l + 64 * j;
      if (o < nout) {
        const int p = o / a.Dff, c = o % a.Dff;
        const int xi = p / a.NI, yi = p % a.NI;
        const float* xe = row + cols[xi];
        const float* ye = row + cols[a.NU + yi];
        float xv[FF_E], yv[FF_E];
        float xo = bx[p * a.Dff + c], yo = by[p * a.Dff + c];
#pragma unroll
        for (int e = 0; e < FF_E; ++e) {
          xv[e] = xe[e]; yv[e] = ye[e];
          xo = fmaf(xv[e], Wx[(p * FF_E + e) * a.Dff + c], xo);
          yo = fmaf(yv[e], Wy[(p * FF_E + e) * a.Dff + c], yo);
        }
        const float d = dY[m * lddy + o];
        const float dxo = d * yo, dyo = d * xo;
        dxo_s[o] = dxo;
        dyo_s[o] = dyo;
        gbx[j] += dxo;
        gby[j] += dyo;
#pragma unroll
        for (int e = 0; e < FF_E; ++e) {
          gWx[j][e] = fmaf(xv[e], dxo, gWx[j][e]);
          gWy[j][e] = fmaf(yv[e], dyo, gWy[j][e]);
        }
      }
    }
    wave_lds_sync();
    // phase 2: lane -> (field i, e)
    for (int q = l; q < (a.NU + a.NI) * FF_E; q += 64) {
      const int i = q / FF_E, e = q % FF_E;
      float v = 0.f;
      if (i < a.NU) {
        for (int yi = 0; yi < a.NI; ++yi) {
          const int p = i * a.NI + yi;
          for (int c = 0; c < a.Dff; ++c) v = fmaf(Wx[(p * FF_E + e) * a.Dff + c], dxo_s[p * a.Dff + c], v);
        }
      } else {
        const int yi = i - a.NU;
        for (int xi = 0; xi < a.NU; ++xi) {
          const int p = xi * a.NI + yi;
          for (int c = 0; c < a.Dff; ++c) v = fmaf(Wy[(p * FF_E + e) * a.Dff + c], dyo_s[p * a.Dff + c], v);
        }
      }
      if (dMu) {  // multiply-ReLU: field i pairs with field i of the other side
        const int k = i < a.NU ? i : i - a.NU;
        const float u = row[cols[k] + e], w = row[cols[a.NU + k] + e];
        const float dm = dMu[m * lddm + k * FF_E + e];
        if (u * w > 0.f) v = fmaf(dm, i < a.NU ? w : u, v);
      }
      float* dst = dX + m * lddx + cols[i] + e;
      *dst = dx_accumulate ? *dst + v : v;
    }
    wave_lds_sync();
  }
  // per-wave partials -> block partial via LDS (reuse the weight region after a barrier)
  __syncthreads();
  float* red = sw;  // [4][2*(nw+nb)]
  const int np = 2 * (nw + nb);
  float* mine = red + wave_id() * np;
#pragma unroll
  for (int j = 0; j < FF_MAXOUT; ++j) {
    const int o = l + 64 * j;
    if (o < nout) {
      const int p = o / a.Dff, c = o % a.Dff;
#pragma unroll
      for (int e = 0; e < FF_E; ++e) {
        mine[(p * FF_E + e) * a.Dff + c] = gWx[j][e];
        mine[nw + nb + (p * FF_E + e) * a.Dff + c] = gWy[j][e];
      }
      mine[nw + o] = gbx[j];
      mine[2 * nw + nb + o] = gby[j];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np; i += blockDim.x)
    part[(int64_t)blockIdx.x * np + i] = (red[i] + red[np + i]) + (red[2 * np + i] + red[3 * np + i]);
}

static int ffm_grid(int64_t M) {
  // 8 rows per block, <= 512 blocks: config 5 (B = 2048) runs 256 blocks, not 128 (16 rows /
  // 256 blocks: 1.855 ms, 8 / 512: 1.846 ms, profiles/r05/ffm_ab/); tuning runs: RS_FFM_RPB,
  // RS_FFM_MAXGRID
  static const int rpb = [] {
    const char* e = getenv("RS_FFM_RPB");
    return e && atoi(e) > 0 ? atoi(e) : 8;
  }();
  static const int cap = [] {
    const char* e = getenv("RS_FFM_MAXGRID");
    return e && atoi(e) > 0 ? atoi(e) : 512;
  }();
  int64_t g = (M + rpb - 1) / rpb;
  return (int)(g > cap ? cap : (g < 1 ? 1 : g));
}

// =============================================================================================
// elementwise gate multiply, softmax-KL head, rowdot, mse
// =============================================================================================
__global__ void mul_fwd_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ G,
                               int64_t ldg, int64_t M, int N, float scale, float* __restrict__ Y,
                               int64_t ldy) {
  const int64_t n = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, c = i % N;
    Y[m * ldy + c] = A[m * lda + c] * (scale * G[m * ldg + c]);
  }
}

__global__ void mul_bwd_kernel(const float* __restrict__ A, int64_t lda, const float* __restrict__ G,
                               int64_t ldg, int64_t M, int N, float scale,
                               const float* __restrict__ dY, int64_t lddy, float* __restrict__ dA,
                               int64_t ldda, float* __restrict__ dG, int64_t lddg) {
  const int64_t n = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, c = i % N;
    const float d = dY[m * lddy + c] * scale;
    const float a = A[m * lda + c], g = G[m * ldg + c];
    if (dA) dA[m * ldda + c] = d * g;
    if (dG) dG[m * lddg + c] = d * a;
  }
}

constexpr int SK_MAXCH = 8;  // C <= 512

__global__ void __launch_bounds__(256) softmax_kl_kernel(
    const float* __restrict__ Z, int64_t ldz, int64_t M, int C, const float* __restrict__ bins,
    float* __restrict__ Pout, int64_t ldp, const float* __restrict__ Yt, int64_t ldt,
    const float* __restrict__ sw, float gscale, float eps, float* __restrict__ loss_rows,
    float* __restrict__ dZ, int64_t lddz) {
  const int l = lane_id();
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < M; m += (int64_t)gridDim.x * 4) {
    float z[SK_MAXCH];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < SK_MAXCH; ++c) {
      const int j = l + 64 * c;
      z[c] = j < C ? Z[m * ldz + j] : -INFINITY;
      mx = fmaxf(mx, z[c]);
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int c = 0; c < SK_MAXCH; ++c) {
      const int j = l + 64 * c;
      z[c] = j < C ? expf(z[c] - mx) : 0.f;
      sum += z[c];
    }
    sum = group_sum<64>(sum);
    const float inv = 1.0f / sum;
    float ev = 0.f;
#pragma unroll
    for (int c = 0; c < SK_MAXCH; ++c) {
      const int j = l + 64 * c;
      z[c] *= inv;  // p
      if (j < C) {
        if (Pout) Pout[m * ldp + j] = z[c];
        if (bins) ev = fmaf(z[c], bins[j], ev);
      }
    }
    if (Pout && bins) {
      ev = group_sum<64>(ev);
      if (l == 0) Pout[m * ldp + C] = ev < 0.f ? 0.f : ev;  // tf.where(pred < 0, 0, pred)
    }
    if (!Yt) continue;
    const float w = sw ? sw[m] : 1.f;
    float kl = 0.f, pdp = 0.f, dp[SK_MAXCH];
#pragma unroll
    for (int c = 0; c < SK_MAXCH; ++c) {
      const int j = l + 64 * c;
      dp[c] = 0.f;
      if (j < C) {
        const float yt = fminf(fmaxf(Yt[m * ldt + j], eps), 1.f);
        const float p = z[c];
        const float yp = fminf(fmaxf(p, eps), 1.f);
        kl = fmaf(yt, logf(yt / yp), kl);
        dp[c] = (p >= eps && p <= 1.f) ? -yt / yp * (w * gscale) : 0.f;
        pdp = fmaf(p, dp[c], pdp);
      }
    }
    kl = group_sum<64>(kl);
    pdp = group_sum<64>(pdp);
    if (loss_rows && l == 0) loss_rows[m] = kl * w;
    if (dZ) {
#pragma unroll
      for (int c = 0; c < SK_MAXCH; ++c) {
        const int j = l + 64 * c;
        if (j < C) dZ[m * lddz + j] = z[c] * (dp[c] - pdp);
      }
    }
  }
}

__global__ void __launch_bounds__(256) rowdot_kernel(const float* __restrict__ U, int64_t ldu,
                                                     const float* __restrict__ V, int64_t ldv,
                                                     int64_t M, int N, int sigm,
                                                     float* __restrict__ Y,
                                                     const float* __restrict__ dY,
                                                     float* __restrict__ dU, int64_t lddu,
                                                     float* __restrict__ dV, int64_t lddv) {
  const int l = lane_id();
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < M; m += (int64_t)gridDim.x * 4) {
    float s = 0.f;
    for (int j = l; j < N; j += 64) s = fmaf(U[m * ldu + j], V[m * ldv + j], s);
    s = group_sum<64>(s);
    const float y = sigm ? 1.0f / (1.0f + expf(-s)) : s;
    if (Y && l == 0) Y[m] = y;
    if (dY) {
      const float d = dY[m] * (sigm ? y * (1.f - y) : 1.f);
      for (int j = l; j < N; j += 64) {
        const float u = U[m * ldu + j], v = V[m * ldv + j];
        if (dU) dU[m * lddu + j] = d * v;
        if (dV) dV[m * lddv + j] = d * u;
      }
    }
  }
}

__global__ void __launch_bounds__(256) mse_rows_kernel(const float* __restrict__ S, int64_t lds,
                                                       const float* __restrict__ T, int64_t ldt,
                                                       int64_t M, int N, float gscale,
                                                       float* __restrict__ loss_rows,
                                                       float* __restrict__ dS, int64_t ldds) {
  const int l = lane_id();
  const float invN = 1.0f / (float)N;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < M; m += (int64_t)gridDim.x * 4) {
    float q = 0.f;
    for (int j = l; j < N; j += 64) {
      const float d = S[m * lds + j] - T[m * ldt + j];
      q = fmaf(d, d, q);
      if (dS) dS[m * ldds + j] = 2.f * d * invN * gscale;
    }
    q = group_sum<64>(q);
    if (loss_rows && l == 0) loss_rows[m] = q * invN;
  }
}

static int rows_grid(int64_t M, int rows_per_block) {
  int64_t g = (M + rows_per_block - 1) / rows_per_block;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace rs_tw

using namespace rs_tw;

// ------------------------------- gate_mix ------------------------------------------------------
static int gm_dp(int D) {
  int dp = 8;
  while (dp < D && dp < 64) dp <<= 1;
  return dp;
}

static int gm_check(const GM& a) {
  if (!a.E || !a.G || !a.sel || a.M < 0 || a.D <= 0 || a.n_exp <= 0 || a.n_task <= 0 ||
      a.n_sel <= 0)
    return RS_ERR_ARG;
  if (a.n_sel > GM_MAXSEL || a.n_task * a.n_sel > GM_MAXSEL * 8 || a.D > 64 * GM_MAXCH)
    return RS_ERR_UNSUPPORTED;
  return RS_OK;
}

RS_API int rs_gate_mix_fwd(void* stream, const float* E, int64_t lde, int e_act, const float* G,
                           int64_t ldg, int64_t M, int n_exp, int D, int n_task, int n_sel,
                           const int32_t* sel, float* Y, int64_t ldy, float* P, int64_t ldp) {
  GM a{E, lde, e_act, G, ldg, M, n_exp, D, n_task, n_sel, sel};
  int st = gm_check(a);
  if (st || !Y) return st ? st : RS_ERR_ARG;
  if (M == 0) return RS_OK;
  const int dp = gm_dp(D);
  const int grid = rows_grid(M, 256 / dp);
  const size_t act_lds = (size_t)(256 / dp) * n_exp * D * 4;
  const int stage = act_lds <= 32 * 1024;
  const size_t lds = stage ? act_lds : 0;
  hipStream_t s = rs_stream(stream);
  switch (dp) {
    case 8: gate_mix_fwd_kernel<8><<<grid, 256, lds, s>>>(a, Y, ldy, P, ldp, stage); break;
    case 16: gate_mix_fwd_kernel<16><<<grid, 256, lds, s>>>(a, Y, ldy, P, ldp, stage); break;
    case 32: gate_mix_fwd_kernel<32><<<grid, 256, lds, s>>>(a, Y, ldy, P, ldp, stage); break;
    default: gate_mix_fwd_kernel<64><<<grid, 256, lds, s>>>(a, Y, ldy, P, ldp, stage); break;
  }
  return rs_status_after_launch();
}

RS_API int rs_gate_mix_bwd(void* stream, const float* E, int64_t lde, int e_act, const float* G,
                           int64_t ldg, int64_t M, int n_exp, int D, int n_task, int n_sel,
                           const int32_t* sel, const float* dY, int64_t lddy, float* dE,
                           int64_t ldde, float* dG, int64_t lddg) {
  GM a{E, lde, e_act, G, ldg, M, n_exp, D, n_task, n_sel, sel};
  int st = gm_check(a);
  if (st || !dY) return st ? st : RS_ERR_ARG;
  if (M == 0) return RS_OK;
  const int dp = gm_dp(D);
  const int rpb = 256 / dp;
  const size_t acc_lds = (size_t)rpb * n_exp * D * 4;
  if (acc_lds > 64 * 1024) return RS_ERR_UNSUPPORTED;
  // the staged activations double the LDS: kept while the total stays <= 64 KB
  const int stage = 2 * acc_lds <= 64 * 1024;
  const size_t lds = stage ? 2 * acc_lds : acc_lds;
  const int grid = rows_grid(M, rpb);
  hipStream_t s = rs_stream(stream);
  switch (dp) {
    case 8: gate_mix_bwd_kernel<8><<<grid, 256, lds, s>>>(a, dY, lddy, dE, ldde, dG, lddg, stage); break;
    case 16: gate_mix_bwd_kernel<16><<<grid, 256, lds, s>>>(a, dY, lddy, dE, ldde, dG, lddg, stage); break;
    case 32: gate_mix_bwd_kernel<32><<<grid, 256, lds, s>>>(a, dY, lddy, dE, ldde, dG, lddg, stage); break;
    default: gate_mix_bwd_kernel<64><<<grid, 256, lds, s>>>(a, dY, lddy, dE, ldde, dG, lddg, stage); break;
  }
  return rs_status_after_launch();
}

// ------------------------------- cross ---------------------------------------------------------
RS_API int64_t rs_cross_bwd_workspace_floats(int64_t M, int D, int L) {
  if (M <= 0 || D <= 0 || L <= 0) return 0;
  return M * 2 * L + (int64_t)cross_nsplit(M) * ((int64_t)(L + 1) * D + L);
}

static int cross_nv(int D) {
  const int nv = (D + 255) / 256;
  return nv <= 1 ? 1 : nv <= 2 ? 2 : nv <= 4 ? 4 : 8;
}

#define RS_CROSS_SWITCH(NVV, LL, CALL) \
  switch (NVV * 10 + LL) {              \
    case 11: CALL(1, 1); break;         \
    case 12: CALL(1, 2); break;         \
    case 13: CALL(1, 3); break;         \
    case 14: CALL(1, 4); break;         \
    case 21: CALL(2, 1); break;         \
    case 22: CALL(2, 2); break;         \
    case 23: CALL(2, 3); break;         \
    case 24: CALL(2, 4); break;         \
    case 41: CALL(4, 1); break;         \
    case 42: CALL(4, 2); break;         \
    case 43: CALL(4, 3); break;         \
    case 44: CALL(4, 4); break;         \
    case 81: CALL(8, 1); break;         \
    case 82: CALL(8, 2); break;         \
    case 83: CALL(8, 3); break;         \
    default: CALL(8, 4); break;         \
  }

static int cross_row_grid(int64_t M, bool fwd) {
  static const int cap[2] = {[] {  // tuning runs: RS_CROSS_GRID_BWD / RS_CROSS_GRID_FWD
    const char* e = getenv("RS_CROSS_GRID_BWD");
    return e && atoi(e) > 0 ? atoi(e) : 1024;
  }(), [] {
    const char* e = getenv("RS_CROSS_GRID_FWD");
    return e && atoi(e) > 0 ? atoi(e) : 1024;
  }()};
  const int c = cap[fwd ? 1 : 0];
  return (int)(M > c ? c : M);
}

RS_API int rs_cross_fwd(void* stream, const float* X0, int64_t ldx, int64_t M, int D, int L,
                        const float* W, const float* b, float* Y, int64_t ldy) {
  if (!X0 || !W || !b || !Y || M < 0 || D <= 0 || L <= 0) return RS_ERR_ARG;
  if (L > CR_MAXL || D > 256 * 8) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  const int nv = cross_nv(D);
  const int grid = cross_row_grid(M, true);
  hipStream_t s = rs_stream(stream);
#define RS_CF(NV, LL) cross_fwd_kernel<NV, LL><<<grid, 256, 0, s>>>(X0, ldx, M, D, W, b, Y, ldy)
  RS_CROSS_SWITCH(nv, L, RS_CF)
#undef RS_CF
  return rs_status_after_launch();
}

RS_API int rs_cross_bwd(void* stream, const float* X0, int64_t ldx, int64_t M, int D, int L,
                        const float* W, const float* b, const float* dY, int64_t lddy, float* dX0,
                        int64_t lddx, int dx_accumulate, float* dparams, int dparams_accumulate,
                        float* workspace, int64_t workspace_floats) {
  if (!X0 || !W || !b || !dY || !dX0 || M < 0 || D <= 0 || L <= 0) return RS_ERR_ARG;
  if (L > CR_MAXL || D > 256 * 8) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  if (!workspace || workspace_floats < rs_cross_bwd_workspace_floats(M, D, L)) return RS_ERR_ARG;
  const int nv = cross_nv(D);
  const int grid = cross_row_grid(M, false);
  float* coef = workspace;
  float* part = workspace + M * 2 * L;
  hipStream_t s = rs_stream(stream);
#define RS_CB(NV, LL)                                                                           \
  cross_bwd_rows_kernel<NV, LL><<<grid, 256, 0, s>>>(X0, ldx, M, D, W, b, dY, lddy, dX0, lddx,  \
                                                     dx_accumulate, coef)
  RS_CROSS_SWITCH(nv, L, RS_CB)
#undef RS_CB
  int st = rs_status_after_launch();
  if (st || !dparams) return st;
  const int64_t rps = cross_rows_per_split(M);
  const int nsplit = cross_nsplit(M);
  const dim3 cgrid((D + 255) / 256, nsplit);
  const int fgrid = (D + 63) / 64;
  switch (L) {
#define RS_CC(LL)                                                                                \
  case LL:                                                                                       \
    cross_bwd_cols_kernel<LL><<<cgrid, 256, 0, s>>>(X0, ldx, M, D, dY, lddy, coef, rps, part);   \
    cross_bwd_final_kernel<LL><<<fgrid, 64 * 16, 0, s>>>(part, nsplit, D, W, b, dparams,             \
                                                     dparams_accumulate);                        \
    break;
    RS_CC(1) RS_CC(2) RS_CC(3) RS_CC(4)
#undef RS_CC
  }
  return rs_status_after_launch();
}

// ------------------------------- fm ------------------------------------------------------------
RS_API int rs_fm_fwd(void* stream, const float* X, int64_t ldx, int64_t fsx, int64_t M, int F,
                     int E, const float* A, int64_t lda, float a_scale, float* Y, int64_t ldy, float* C,
                     int64_t ldc, float* fm, int64_t ldf) {
  if (!X || M < 0 || F <= 0 || E <= 0) return RS_ERR_ARG;
  if (E > 64) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  FM a{X, ldx, fsx, M, F, E, A, lda, a_scale};
  const int grid = rows_grid(M, 4);
  hipStream_t s = rs_stream(stream);
  if (E <= 8) fm_fwd_kernel<8><<<grid, 256, 0, s>>>(a, Y, ldy, C, ldc, fm, ldf);
  else if (E <= 16) fm_fwd_kernel<16><<<grid, 256, 0, s>>>(a, Y, ldy, C, ldc, fm, ldf);
  else if (E <= 32) fm_fwd_kernel<32><<<grid, 256, 0, s>>>(a, Y, ldy, C, ldc, fm, ldf);
  else fm_fwd_kernel<64><<<grid, 256, 0, s>>>(a, Y, ldy, C, ldc, fm, ldf);
  return rs_status_after_launch();
}

RS_API int rs_fm_bwd(void* stream, const float* X, int64_t ldx, int64_t fsx, int64_t M, int F, int E,
                     const float* A, int64_t lda, float a_scale, const float* dY, int64_t lddy, const float* dC,
                     int64_t lddc, const float* dfm, int64_t lddf, float* dX, int64_t lddx,
                     int64_t fsdx, int dx_accumulate, float* dA, int64_t ldda) {
  if (!X || M < 0 || F <= 0 || E <= 0) return RS_ERR_ARG;
  if (E > 64) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  FM a{X, ldx, fsx, M, F, E, A, lda, a_scale};
  const int grid = rows_grid(M, 4);
  hipStream_t s = rs_stream(stream);
#define RS_FMB(EW)                                                                              \
  fm_bwd_kernel<EW><<<grid, 256, 0, s>>>(a, dY, lddy, dC, lddc, dfm, lddf, dX, lddx, fsdx,      \
                                         dx_accumulate, dA, ldda)
  if (E <= 8) RS_FMB(8);
  else if (E <= 16) RS_FMB(16);
  else if (E <= 32) RS_FMB(32);
  else RS_FMB(64);
#undef RS_FMB
  return rs_status_after_launch();
}

// ------------------------------- ffm -----------------------------------------------------------
static int ffm_check(int64_t M, int NU, int NI, int E, int Dff) {
  if (M < 0 || NU <= 0 || NI <= 0 || Dff <= 0) return RS_ERR_ARG;
  if (E != FF_E || NU + NI > FF_MAXF || NU * NI * Dff > 64 * FF_MAXOUT) return RS_ERR_UNSUPPORTED;
  return RS_OK;
}

RS_API int64_t rs_ffm_param_count(int NU, int NI, int E, int Dff) {
  return 2 * ((int64_t)NU * NI * E * Dff + (int64_t)NU * NI * Dff);
}

RS_API int64_t rs_ffm_bwd_workspace_floats(int64_t M, int NU, int NI, int E, int Dff) {
  if (ffm_check(M, NU, NI, E, Dff)) return 0;
  return (int64_t)ffm_grid(M) * rs_ffm_param_count(NU, NI, E, Dff);
}

RS_API int rs_ffm_fwd(void* stream, const float* X, int64_t ldx, int64_t M, int NU, int NI, int E,
                      int Dff, const int32_t* cols, const float* Wx, const float* bx,
                      const float* Wy, const float* by, float* Y, int64_t ldy, float* Mult,
                      int64_t ldm) {
  int st = ffm_check(M, NU, NI, E, Dff);
  if (st) return st;
  if (!X || !cols || !Wx || !bx || !Wy || !by || !Y) return RS_ERR_ARG;
  if (Mult && NU != NI) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  FFM a{X, ldx, M, NU, NI, Dff, cols, Wx, bx, Wy, by};
  const size_t lds = (size_t)rs_ffm_param_count(NU, NI, E, Dff) * 4;
  ffm_fwd_kernel<<<rows_grid(M, 4), 256, lds, rs_stream(stream)>>>(a, Y, ldy, Mult, ldm);
  return rs_status_after_launch();
}

RS_API int rs_ffm_bwd(void* stream, const float* X, int64_t ldx, int64_t M, int NU, int NI, int E,
                      int Dff, const int32_t* cols, const float* Wx, const float* bx,
                      const float* Wy, const float* by, const float* dY, int64_t lddy,
                      const float* dMult, int64_t lddm, float* dX, int64_t lddx,
                      int dx_accumulate, float* dparams, int dparams_accumulate, float* workspace,
                      int64_t workspace_floats) {
  int st = ffm_check(M, NU, NI, E, Dff);
  if (st) return st;
  if (!X || !cols || !Wx || !bx || !Wy || !by || !dY || !dX) return RS_ERR_ARG;
  if (dMult && NU != NI) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  const int grid = ffm_grid(M);
  const int64_t np = rs_ffm_param_count(NU, NI, E, Dff);
  if (!workspace || workspace_floats < grid * np) return RS_ERR_ARG;
  FFM a{X, ldx, M, NU, NI, Dff, cols, Wx, bx, Wy, by};
  const int nb = NU * NI * Dff;
  size_t lds = (size_t)(np + 4 * 2 * nb) * 4;
  if (lds < (size_t)4 * np * 4) lds = (size_t)4 * np * 4;
  hipStream_t s = rs_stream(stream);
  ffm_bwd_kernel<<<grid, 256, lds, s>>>(a, dY, lddy, dMult, lddm, dX, lddx, dx_accumulate,
                                        workspace);
  st = rs_status_after_launch();
  if (st || !dparams) return st;
  launch_column_reduce(s, workspace, grid, np, np, np, dparams, dparams, dparams_accumulate);
  return rs_status_after_launch();
}

// ------------------------------- elementwise / heads / losses ---------------------------------
RS_API int rs_mul_fwd(void* stream, const float* A, int64_t lda, const float* G, int64_t ldg,
                      int64_t M, int N, float scale, float* Y, int64_t ldy) {
  if (!A || !G || !Y || M < 0 || N <= 0) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  int64_t grid = (M * N + 255) / 256;
  if (grid > 8192) grid = 8192;
  mul_fwd_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(A, lda, G, ldg, M, N, scale, Y, ldy);
  return rs_status_after_launch();
}

RS_API int rs_mul_bwd(void* stream, const float* A, int64_t lda, const float* G, int64_t ldg,
                      int64_t M, int N, float scale, const float* dY, int64_t lddy, float* dA,
                      int64_t ldda, float* dG, int64_t lddg) {
  if (!A || !G || !dY || M < 0 || N <= 0) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  int64_t grid = (M * N + 255) / 256;
  if (grid > 8192) grid = 8192;
  mul_bwd_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(A, lda, G, ldg, M, N, scale, dY, lddy,
                                                           dA, ldda, dG, lddg);
  return rs_status_after_launch();
}

// Grouped ppnet gating (staytime/VideoDnn.py:139-146, one multiply per expert): G <= 8 problems,
// one element per thread, block b -> problem p by start offsets (a block-uniform index).
//   fwd desc [M, N, lda, ldg, ldy, A, G, Y]                    Y = A * (scale G)
//   bwd desc [M, N, lda, ldg, lddy, ldda, lddg, A, G, dY, dA, dG]
constexpr int kMulGroup = 8;
struct MulGroup {
  const float* a[kMulGroup]; const float* g[kMulGroup]; const float* dy[kMulGroup];
  float* y[kMulGroup]; float* da[kMulGroup]; float* dg[kMulGroup];
  int64_t lda[kMulGroup], ldg[kMulGroup], ldy[kMulGroup], ldda[kMulGroup], lddg[kMulGroup];
  int64_t M[kMulGroup];
  int N[kMulGroup];
  int start[kMulGroup + 1];
  int n;
  float scale;
};

template <bool BWD>
__global__ void __launch_bounds__(256) mul_group_kernel(MulGroup mg) {
  const int b = (int)blockIdx.x;
  int p = 0;
#pragma unroll
  for (int k = 1; k < kMulGroup; ++k) p += (k < mg.n && b >= mg.start[k]) ? 1 : 0;
  const int64_t i = (int64_t)(b - mg.start[p]) * 256 + threadIdx.x;
  const int N = mg.N[p];
  if (i >= mg.M[p] * N) return;
  const int64_t m = i / N, c = i - m * N;
  const float a = mg.a[p][m * mg.lda[p] + c], g = mg.g[p][m * mg.ldg[p] + c];
  if (!BWD) {
    mg.y[p][m * mg.ldy[p] + c] = a * (mg.scale * g);
  } else {
    const float d = mg.dy[p][m * mg.ldy[p] + c] * mg.scale;
    if (mg.da[p]) mg.da[p][m * mg.ldda[p] + c] = d * g;
    if (mg.dg[p]) mg.dg[p][m * mg.lddg[p] + c] = d * a;
  }
}

template <typename T>
static T* mptr(int64_t v) { return reinterpret_cast<T*>((uintptr_t)v); }

static int mul_group_launch(void* stream, int G, const int64_t* desc, float scale, bool bwd) {
  if (!desc || G < 1 || G > kMulGroup) return RS_ERR_ARG;
  MulGroup mg{};
  mg.n = G;
  mg.scale = scale;
  mg.start[0] = 0;
  for (int p = 0; p < G; ++p) {
    const int64_t* d = desc + (bwd ? 12 : 8) * p;
    mg.M[p] = d[0]; mg.N[p] = (int)d[1]; mg.lda[p] = d[2]; mg.ldg[p] = d[3]; mg.ldy[p] = d[4];
    if (bwd) {
      mg.ldda[p] = d[5]; mg.lddg[p] = d[6];
      mg.a[p] = mptr<const float>(d[7]); mg.g[p] = mptr<const float>(d[8]);
      mg.dy[p] = mptr<const float>(d[9]); mg.da[p] = mptr<float>(d[10]); mg.dg[p] = mptr<float>(d[11]);
      if (!mg.dy[p]) return RS_ERR_ARG;
    } else {
      mg.a[p] = mptr<const float>(d[5]); mg.g[p] = mptr<const float>(d[6]); mg.y[p] = mptr<float>(d[7]);
      if (!mg.y[p]) return RS_ERR_ARG;
    }
    if (!mg.a[p] || !mg.g[p] || mg.M[p] < 0 || mg.N[p] <= 0) return RS_ERR_ARG;
    const int64_t blocks = (mg.M[p] * mg.N[p] + 255) / 256;
    if (mg.start[p] + blocks > (int64_t)1 << 30) return RS_ERR_ARG;
    mg.start[p + 1] = mg.start[p] + (int)blocks;
  }
  for (int p = G; p < kMulGroup; ++p) mg.start[p + 1] = mg.start[G];
  if (mg.start[G] == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  if (bwd) mul_group_kernel<true><<<mg.start[G], 256, 0, s>>>(mg);
  else mul_group_kernel<false><<<mg.start[G], 256, 0, s>>>(mg);
  return rs_status_after_launch();
}

RS_API int rs_mul_fwd_grouped(void* stream, int G, const int64_t* desc, float scale) {
  return mul_group_launch(stream, G, desc, scale, false);
}

RS_API int rs_mul_bwd_grouped(void* stream, int G, const int64_t* desc, float scale) {
  return mul_group_launch(stream, G, desc, scale, true);
}

RS_API int rs_softmax_kl(void* stream, const float* Z, int64_t ldz, int64_t M, int C,
                         const float* bins, float* P, int64_t ldp, const float* y_true,
                         int64_t ldt, const float* sample_w, float gscale, float eps,
                         float* loss_rows, float* dZ, int64_t lddz) {
  if (!Z || M < 0 || C <= 0) return RS_ERR_ARG;
  if (C > 64 * SK_MAXCH) return RS_ERR_UNSUPPORTED;
  if ((loss_rows || dZ) && !y_true) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  softmax_kl_kernel<<<rows_grid(M, 4), 256, 0, rs_stream(stream)>>>(
      Z, ldz, M, C, bins, P, ldp, y_true, ldt, sample_w, gscale, eps, loss_rows, dZ, lddz);
  return rs_status_after_launch();
}

RS_API int rs_rowdot(void* stream, const float* U, int64_t ldu, const float* V, int64_t ldv,
                     int64_t M, int N, int use_sigmoid, float* Y, const float* dY, float* dU,
                     int64_t lddu, float* dV, int64_t lddv) {
  if (!U || !V || M < 0 || N <= 0) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  rowdot_kernel<<<rows_grid(M, 4), 256, 0, rs_stream(stream)>>>(U, ldu, V, ldv, M, N, use_sigmoid,
                                                               Y, dY, dU, lddu, dV, lddv);
  return rs_status_after_launch();
}

RS_API int rs_mse_rows(void* stream, const float* S, int64_t lds, const float* T, int64_t ldt,
                       int64_t M, int N, float gscale, float* loss_rows, float* dS, int64_t ldds) {
  if (!S || !T || M < 0 || N <= 0) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  mse_rows_kernel<<<rows_grid(M, 4), 256, 0, rs_stream(stream)>>>(S, lds, T, ldt, M, N, gscale,
                                                                 loss_rows, dS, ldds);
  return rs_status_after_launch();
}

// ------------------------------- grouped per-task heads ----------------------------------------
// T independent Dense(1, act) heads, head t reading columns [t*D, (t+1)*D) of X
// (rank/multi_head/multidnn.py:122-204: one Dense(1, sigmoid) tower per gated task output).
// W [T*D] (head t's kernel is W[t*D .. t*D+D)), b [T].  One wave per row, D-lane groups reduce.
namespace rs_tw {
template <int D>
__global__ void __launch_bounds__(256) grouped_head_fwd_kernel(const float* __restrict__ X,
                                                               int64_t ldx, int64_t M, int T,
                                                               const float* __restrict__ W,
                                                               const float* __restrict__ b,
                                                               int act, float* __restrict__ Y,
                                                               int64_t ldy) {
  const int l = lane_id();
  const int n = T * D;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < M; m += (int64_t)gridDim.x * 4) {
    for (int c0 = 0; c0 < n; c0 += 64) {
      const int idx = c0 + l;
      const float v = idx < n ? X[m * ldx + idx] * W[idx] : 0.f;
      const float s = group_sum<D>(v);
      const int t = idx / D;
      if (idx < n && (idx % D) == 0) Y[m * ldy + t] = act_f(s + b[t], act);
    }
  }
}

template <int D>
__global__ void __launch_bounds__(256) grouped_head_bwd_kernel(
    const float* __restrict__ X, int64_t ldx, int64_t M, int T, const float* __restrict__ W,
    const float* __restrict__ Y, int64_t ldy, int act, const float* __restrict__ dY, int64_t lddy,
    float* __restrict__ dX, int64_t lddx, float* __restrict__ part) {
  // part[block][T*D + T]: dW then db; lanes own columns idx = c0 + lane
  constexpr int MAXC = 4;  // T*D <= 256
  const int l = lane_id();
  const int n = T * D;
  float gw[MAXC] = {0.f, 0.f, 0.f, 0.f}, gb[MAXC] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t m = (int64_t)blockIdx.x * 4 + wave_id(); m < M; m += (int64_t)gridDim.x * 4) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int idx = c * 64 + l;
      if (idx < n) {
        const int t = idx / D;
        const float y = Y[m * ldy + t];
        float dz = dY[m * lddy + t];
        if (act == ACT_RELU) dz = y > 0.f ? dz : 0.f;
        else if (act == ACT_SIGMOID) dz *= y * (1.f - y);
        const float x = X[m * ldx + idx];
        if (dX) dX[m * lddx + idx] = dz * W[idx];
        gw[c] = fmaf(x, dz, gw[c]);
        if (idx % D == 0) gb[c] += dz;
      }
    }
  }
  __shared__ float red[4][256 + 64];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int idx = c * 64 + l;
    red[wave_id()][idx] = gw[c];
    if (idx % D == 0 && idx < n) red[wave_id()][256 + idx / D] = gb[c];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n + T; i += blockDim.x) {
    const int src = i < n ? i : 256 + (i - n);
    part[(int64_t)blockIdx.x * (n + T) + i] = (red[0][src] + red[1][src]) + (red[2][src] + red[3][src]);
  }
}

__global__ void row_select_kernel(const float* __restrict__ mask, const float* __restrict__ A,
                                  int64_t lda, const float* __restrict__ Bm, int64_t ldb,
                                  int64_t M, int N, float* __restrict__ Y, int64_t ldy,
                                  const float* __restrict__ dY, float* __restrict__ dA,
                                  float* __restrict__ dB) {
  const int64_t n = M * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, c = i % N;
    const bool on = mask[m] == 1.0f;
    if (Y) Y[m * ldy + c] = on ? A[m * lda + c] : Bm[m * ldb + c];
    if (dY) {
      const float d = dY[m * ldy + c];
      if (dA) dA[m * N + c] = on ? d : 0.f;
      if (dB) dB[m * N + c] = on ? 0.f : d;
    }
  }
}
}  // namespace rs_tw

static int gh_grid(int64_t M) { return (int)(M < 4 * 256 ? (M + 3) / 4 : 256); }

RS_API int64_t rs_grouped_head_bwd_workspace_floats(int64_t M, int T, int D) {
  if (M <= 0 || T <= 0 || D <= 0) return 0;
  return (int64_t)gh_grid(M) * (T * D + T);
}

#define RS_GH_SWITCH(DD, CALL) \
  switch (DD) {                \
    case 1: CALL(1); break;    \
    case 2: CALL(2); break;    \
    case 4: CALL(4); break;    \
    case 8: CALL(8); break;    \
    case 16: CALL(16); break;  \
    case 32: CALL(32); break;  \
    case 64: CALL(64); break;  \
    default: return RS_ERR_UNSUPPORTED; \
  }

RS_API int rs_grouped_head_fwd(void* stream, const float* X, int64_t ldx, int64_t M, int T, int D,
                               const float* W, const float* b, int act, float* Y, int64_t ldy) {
  if (!X || !W || !b || !Y || M < 0 || T <= 0 || D <= 0) return RS_ERR_ARG;
  if (T * D > 256) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  const int grid = rows_grid(M, 4);
#define RS_GHF(DD) grouped_head_fwd_kernel<DD><<<grid, 256, 0, s>>>(X, ldx, M, T, W, b, act, Y, ldy)
  RS_GH_SWITCH(D, RS_GHF)
#undef RS_GHF
  return rs_status_after_launch();
}

RS_API int rs_grouped_head_bwd(void* stream, const float* X, int64_t ldx, int64_t M, int T, int D,
                               const float* W, const float* Y, int64_t ldy, int act,
                               const float* dY, int64_t lddy, float* dX, int64_t lddx,
                               float* dparams, int dparams_accumulate, float* workspace,
                               int64_t workspace_floats) {
  if (!X || !W || !Y || !dY || M < 0 || T <= 0 || D <= 0) return RS_ERR_ARG;
  if (T * D > 256) return RS_ERR_UNSUPPORTED;
  if (M == 0) return RS_OK;
  const int grid = gh_grid(M);
  const int64_t np = (int64_t)T * D + T;
  if (!workspace || workspace_floats < grid * np) return RS_ERR_ARG;
  hipStream_t s = rs_stream(stream);
#define RS_GHB(DD)                                                                               \
  grouped_head_bwd_kernel<DD><<<grid, 256, 0, s>>>(X, ldx, M, T, W, Y, ldy, act, dY, lddy, dX,   \
                                                   lddx, workspace)
  RS_GH_SWITCH(D, RS_GHB)
#undef RS_GHB
  int st = rs_status_after_launch();
  if (st || !dparams) return st;
  launch_column_reduce(s, workspace, grid, np, np, np, dparams, dparams, dparams_accumulate);
  return rs_status_after_launch();
}

RS_API int rs_row_select(void* stream, const float* mask, const float* A, int64_t lda,
                         const float* Bm, int64_t ldb, int64_t M, int N, float* Y, int64_t ldy,
                         const float* dY, float* dA, float* dB) {
  if (!mask || M < 0 || N <= 0 || (!Y && !dY)) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  int64_t grid = (M * N + 255) / 256;
  if (grid > 8192) grid = 8192;
  row_select_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(mask, A, lda, Bm, ldb, M, N, Y, ldy,
                                                            dY, dA, dB);
  return rs_status_after_launch();
}

// ------------------------------- elementwise activation ----------------------------------------
// tf.sigmoid / relu on a [M, N] tensor (rough_rank/model.py:30-33,80 teacher / student
// probabilities from their logits).
namespace rs_tw {
__global__ void act_fwd_kernel(const float* __restrict__ X, int64_t n, int act, float* __restrict__ Y) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    Y[i] = act_f(X[i], act);
}
__global__ void act_bwd_kernel(const float* __restrict__ Y, const float* __restrict__ dY, int64_t n,
                               int act, float* __restrict__ dX) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float y = Y[i];
    float d = dY[i];
    if (act == ACT_RELU) d = y > 0.f ? d : 0.f;
    else if (act == ACT_SIGMOID) d *= y * (1.f - y);
    dX[i] = d;
  }
}
}  // namespace rs_tw

RS_API int rs_act_fwd(void* stream, const float* X, int64_t n, int act, float* Y) {
  if (!X || !Y || n < 0) return RS_ERR_ARG;
  if (n == 0) return RS_OK;
  int64_t grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  act_fwd_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(X, n, act, Y);
  return rs_status_after_launch();
}

RS_API int rs_act_bwd(void* stream, const float* Y, const float* dY, int64_t n, int act, float* dX) {
  if (!Y || !dY || !dX || n < 0) return RS_ERR_ARG;
  if (n == 0) return RS_OK;
  int64_t grid = (n + 255) / 256;
  if (grid > 8192) grid = 8192;
  act_bwd_kernel<<<(int)grid, 256, 0, rs_stream(stream)>>>(Y, dY, n, act, dX);
  return rs_status_after_launch();
}

// ------------------------------- per-row weighted cross entropy --------------------------------
// staytime/model.py:33-36 cross_entropy (per element, p unclipped, +1e-6 inside the logs) with
// Keras sample weights (parse.py:64): loss_rows[m] = w_m * sum_t ce(y, clip(p)); ds = gscale *
// w_m * dce/dp (zero outside [lo, hi], TF ClipByValue gradient).
namespace rs_tw {
__global__ void bce_rows_kernel(const float* __restrict__ P, const float* __restrict__ Y, int64_t M,
                                int T, float lo, float hi, float log_eps,
                                const float* __restrict__ W, float gscale,
                                float* __restrict__ loss_rows, float* __restrict__ dP) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < M;
       m += (int64_t)gridDim.x * blockDim.x) {
    const float w = W ? W[m] : 1.f;
    float l = 0.f;
    for (int t = 0; t < T; ++t) {
      const float p0 = P[m * T + t], y = Y[m * T + t];
      const float p = fminf(fmaxf(p0, lo), hi);
      l += -y * logf(p + log_eps) - (1.f - y) * logf(1.f - p + log_eps);
      if (dP) {
        const float d = -y / (p + log_eps) + (1.f - y) / (1.f - p + log_eps);
        dP[m * T + t] = (p0 >= lo && p0 <= hi) ? gscale * w * d : 0.f;
      }
    }
    if (loss_rows) loss_rows[m] = w * l;
  }
}
}  // namespace rs_tw

RS_API int rs_bce_rows(void* stream, const float* P, const float* Y, int64_t M, int T, float lo,
                       float hi, float log_eps, const float* W, float gscale, float* loss_rows,
                       float* dP) {
  if (!P || !Y || M < 0 || T <= 0) return RS_ERR_ARG;
  if (M == 0) return RS_OK;
  // one row per thread, 64-thread blocks: B = 2048 rows spread over 32 CUs instead of 8
  int64_t grid = (M + 63) / 64;
  if (grid > 4096) grid = 4096;
  bce_rows_kernel<<<(int)grid, 64, 0, rs_stream(stream)>>>(P, Y, M, T, lo, hi, log_eps, W, gscale,
                                                         loss_rows, dP);
  return rs_status_after_launch();
}

// ------------------------------- fused loss total ------------------------------------------------
// The compiled Keras loss of a multi-output model is sum_k loss_weight_k * mean_batch(rows_k):
// the per-row loss vectors of every output (rs_softmax_kl / rs_bce_rows / rs_mse_rows rows, laid
// out back to back, seg floats each) are reduced with their weights in ONE launch instead of a
// reduction, a scale and an add per output (staytime/model.py:85-89, rough_rank/model.py:210-214).
// One workgroup, fixed summation order (deterministic).
namespace rs_tw {
constexpr int kWsumThreads = 1024;
__global__ void __launch_bounds__(kWsumThreads) weighted_row_sum_kernel(
    const float* __restrict__ X, int64_t seg, int nseg, float w0, float w1, float w2, float w3,
    float w4, float w5, float* __restrict__ out) {
  __shared__ float red[kWsumThreads / 64];
  const float ws[6] = {w0, w1, w2, w3, w4, w5};
  float acc = 0.f;
  for (int k = 0; k < nseg; ++k) {
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < seg; i += kWsumThreads) s += X[k * seg + i];
    acc = fmaf(ws[k], s, acc);
  }
  acc = group_sum<64>(acc);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < kWsumThreads / 64; ++k) t += red[k];
    out[0] = t;
  }
}
}  // namespace rs_tw

RS_API int rs_weighted_row_sum(void* stream, const float* X, int64_t seg, int nseg, float w0,
                               float w1, float w2, float w3, float w4, float w5, float* out) {
  if (!X || !out || seg < 0 || nseg < 1 || nseg > 6) return RS_ERR_ARG;
  rs_tw::weighted_row_sum_kernel<<<1, rs_tw::kWsumThreads, 0, rs_stream(stream)>>>(
      X, seg, nseg, w0, w1, w2, w3, w4, w5, out);
  return rs_status_after_launch();
}
