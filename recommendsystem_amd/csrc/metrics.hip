// Training metrics compiled into every reference model: Keras 'acc' /
// tf.keras.metrics.BinaryAccuracy(), tf.keras.metrics.AUC() and tensornet's tn.metric.COPC() /
// tn.metric.CTR() (rank/ctr/base_model.py:183-190, rough_rank/model.py:215-219,
// rank/multi_head/model.py:55, staytime/model.py:81-82), accumulated on the device over the
// predictions a training step already holds (no host read per step, graph-capturable).
//
// AUC follows tf.keras.metrics.AUC's defaults (num_thresholds = 200, curve ROC, summation
// 'interpolation'): thresholds t_0 = -1e-7, t_i = i / (nthr - 1) (i = 1 .. nthr - 2, rounded to
// fp32), t_{nthr-1} = 1 + 1e-7; a prediction counts as positive at t_i when p > t_i.  Each sample
// falls in bucket k = #{i : t_i < p}, so TP(t_i) = sum_{k > i} pos[k] and FP(t_i) = sum_{k > i}
// neg[k]; the result is sum_i (FPR_i - FPR_{i+1}) (TPR_i + TPR_{i+1}) / 2.  Binary accuracy uses
// threshold 0.5 (p > 0.5).  COPC (tensornet, not vendored; pinned form): sum(w y) / sum(w p);
// CTR: sum(w y) / sum(w).  Weighted (weighted_metrics with a sample weight) or unit weights.
// Accumulators are fp64 (exact integer counts for unit weights).
#include "common.hpp"

namespace {

constexpr int kMaxThr = 1024;

// bucket of p among the fp32 thresholds (the comparison Keras makes in fp32)
__device__ __forceinline__ int auc_bucket(float p, int nthr) {
  if (!(p > -1e-7f)) return 0;                 // p <= t_0 (or NaN): below every threshold
  const int m = nthr - 1;                      // interior thresholds i = 1 .. m - 1 are i / m
  int k = (int)floorf(p * (float)m);           // guess: i / m < p for i <= k (fp32 rounding aside)
  k = k < 0 ? 0 : (k > m - 1 ? m - 1 : k);
  while (k > 0 && !((float)((double)k / (double)m) < p)) --k;
  while (k + 1 <= m - 1 && (float)((double)(k + 1) / (double)m) < p) ++k;
  // k interior thresholds below p, plus t_0; t_{nthr-1} = 1 + 1e-7 as well when p exceeds it
  return 1 + k + (p > 1.0f + 1e-7f ? 1 : 0);
}

// state: hist[2][nthr + 1] (negatives, positives) | sums[4] = {sum w y, sum w p, sum w correct,
// sum w} -- all fp64
__global__ void __launch_bounds__(256) metrics_accumulate_kernel(
    const float* __restrict__ p, int64_t p_ld, const float* __restrict__ y, int64_t y_ld,
    const float* __restrict__ w, int64_t w_ld, int64_t B, int nthr, double* __restrict__ state) {
  __shared__ double hist[2 * (kMaxThr + 1)];
  __shared__ double red[4][4];
  const int nb = nthr + 1;
  for (int k = threadIdx.x; k < 2 * nb; k += blockDim.x) hist[k] = 0.0;
  __syncthreads();
  double sy = 0.0, sp = 0.0, sc = 0.0, sw = 0.0;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < B;
       b += (int64_t)gridDim.x * blockDim.x) {
    const float pv = p[b * p_ld], yv = y[b * y_ld];
    const float wv = w ? w[b * w_ld] : 1.0f;
    const bool pos = yv != 0.f;  // Keras AUC: cast(y_true, bool)
    atomicAdd(&hist[(pos ? nb : 0) + auc_bucket(pv, nthr)], (double)wv);
    sy += (double)wv * yv;
    sp += (double)wv * pv;
    sc += (yv == (pv > 0.5f ? 1.f : 0.f)) ? (double)wv : 0.0;  // binary_accuracy, threshold 0.5
    sw += wv;
  }
  // sums: wave butterflies, then 4 waves in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sy += __shfl_xor(sy, o, 64);
    sp += __shfl_xor(sp, o, 64);
    sc += __shfl_xor(sc, o, 64);
    sw += __shfl_xor(sw, o, 64);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[wave][0] = sy; red[wave][1] = sp; red[wave][2] = sc; red[wave][3] = sw;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    double t = 0.0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += red[k][threadIdx.x];
    atomicAdd(state + 2 * nb + threadIdx.x, t);
  }
  for (int k = threadIdx.x; k < 2 * nb; k += blockDim.x)
    if (hist[k] != 0.0) atomicAdd(state + k, hist[k]);
}

// out[6] = {auc, binary accuracy, copc, ctr, mean prediction, total weight}
__global__ void __launch_bounds__(64) metrics_result_kernel(const double* __restrict__ state,
                                                            int nthr, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const int nb = nthr + 1;
  const double* neg = state;
  const double* pos = state + nb;
  double P = 0.0, N = 0.0;
  for (int k = 0; k < nb; ++k) { P += pos[k]; N += neg[k]; }
  // TP(t_i) / FP(t_i): samples in buckets k > i; walk i upward, removing bucket i
  double tp = P, fp = N, auc = 0.0;
  double tpr_prev = 0.0, fpr_prev = 0.0;
  for (int i = 0; i < nthr; ++i) {
    tp -= pos[i];
    fp -= neg[i];
    const double tpr = (tp + 0.0) / (P > 0.0 ? P : 1.0);  // Keras: tp / (tp + fn), divide_no_nan
    const double fpr = (fp + 0.0) / (N > 0.0 ? N : 1.0);
    if (i > 0) auc += (fpr_prev - fpr) * (tpr_prev + tpr) * 0.5;
    tpr_prev = tpr;
    fpr_prev = fpr;
  }
  const double* s = state + 2 * nb;
  out[0] = (float)auc;
  out[1] = (float)(s[3] > 0.0 ? s[2] / s[3] : 0.0);
  out[2] = (float)(s[1] > 0.0 ? s[0] / s[1] : 0.0);
  out[3] = (float)(s[3] > 0.0 ? s[0] / s[3] : 0.0);
  out[4] = (float)(s[3] > 0.0 ? s[1] / s[3] : 0.0);
  out[5] = (float)s[3];
}

}  // namespace

RS_API int64_t rs_ctr_metrics_state_doubles(int nthr) {
  if (nthr < 3 || nthr > kMaxThr) return -1;
  return 2 * (int64_t)(nthr + 1) + 4;
}

RS_API int rs_ctr_metrics_accumulate(void* stream, const float* p, int64_t p_ld, const float* y,
                                     int64_t y_ld, const float* w, int64_t w_ld, int64_t B,
                                     int nthr, double* state) {
  if (!p || !y || !state || B < 0 || nthr < 3 || nthr > kMaxThr || p_ld < 1 || y_ld < 1 ||
      (w && w_ld < 1))
    return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  int64_t grid = (B + 255) / 256;
  if (grid > 256) grid = 256;
  metrics_accumulate_kernel<<<(unsigned)grid, 256, 0, rs_stream(stream)>>>(p, p_ld, y, y_ld, w,
                                                                           w_ld, B, nthr, state);
  return rs_status_after_launch();
}

RS_API int rs_ctr_metrics_result(void* stream, const double* state, int nthr, float* out) {
  if (!state || !out || nthr < 3 || nthr > kMaxThr) return RS_ERR_ARG;
  metrics_result_kernel<<<1, 64, 0, rs_stream(stream)>>>(state, nthr, out);
  return rs_status_after_launch();
}
