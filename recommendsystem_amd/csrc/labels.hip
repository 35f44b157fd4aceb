// the staytime label construction of parse_input_func (staytime/parse.py:16-71)
// as one device pass over a batch, so a data-parallel rank hands the trainer raw watch times and
// never builds the [B, 401] soft label on the host.
//
// Per sample b (reference op order, fp32 throughout, as the TF graph computes it):
//   short[b] = watch_ms[b] > 7000  ? 1 : 0                       (parse.py:30-34, int64 compare)
//   long[b]  = watch_ms[b] > 18000 ? 1 : 0                       (parse.py:36-38)
//   wt       = min(float(watch_ms[b]) / 1000, 160)               (parse.py:40-42; tf.where(wt > 160))
//   label[b, i] = exp(|bins[i] - wt|^2 / (-2 sigma^2)) / (sqrt(2 pi) sigma) * width, i < nbins
//                                                                (parse.py:45-61)
//   label[b, nbins] = wt                                         (parse.py:62, concat [label, wt])
//   weight[b] = landing[b] ? 5 : 1                               (parse.py:64; the regex
//                      ".*video_homepage_landing.*" over extra_info is string work: the host
//                      evaluates it and passes one byte per sample)
//
// Layout: one wave per sample row; the 64 lanes sweep the nbins + 1 columns, so every store of a
// wave is one contiguous 256-B run of the row (HBM-bound: 4 (nbins + 1) + 8 + 1 + 12 bytes per
// sample).  At B = 16384 it measures 14.9 us (profiles/r01c): VALU-bound on the correctly rounded
// fp32 division and the exp per element (staging the bins in LDS measured slower, 16.6 us).
#include <cmath>

#include "common.hpp"

namespace {

constexpr int kLabelThreads = 256;  // 4 waves = 4 sample rows per block

__global__ __launch_bounds__(kLabelThreads) void staytime_label_kernel(
    const int64_t* __restrict__ watch_ms, const uint8_t* __restrict__ landing, int64_t B,
    const float* __restrict__ bins, int nbins, float neg_two_sigma2, bool pow2_div,
    float inv_neg_two_sigma2, float norm, float width,
    float* __restrict__ label, int64_t ld, float* __restrict__ short_label,
    float* __restrict__ long_label, float* __restrict__ weight) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (kLabelThreads / 64);
  for (int64_t b = (int64_t)blockIdx.x * (kLabelThreads / 64) + (threadIdx.x >> 6); b < B;
       b += waves) {
    const int64_t w = watch_ms[b];
    float wt = (float)w / 1000.0f;
    wt = wt > 160.0f ? 160.0f : wt;
    float* row = label + b * ld;
    for (int i = lane; i < nbins; i += 64) {
      const float d = fabsf(bins[i] - wt);
      // tf.divide(absSquareDist, -2 sigma^2): a true fp32 division; when -2 sigma^2 is a power of
      // two (sigma = 4: -32) the product with its reciprocal is the same correctly rounded value.
      const float q = pow2_div ? (d * d) * inv_neg_two_sigma2 : (d * d) / neg_two_sigma2;
      const float e = expf(q);
      row[i] = (e / norm) * width;
    }
    if (lane == 0) {
      row[nbins] = wt;
      if (short_label) short_label[b] = w > 7000 ? 1.0f : 0.0f;
      if (long_label) long_label[b] = w > 18000 ? 1.0f : 0.0f;
      if (weight) weight[b] = (landing && landing[b]) ? 5.0f : 1.0f;
    }
  }
}

}  // namespace

RS_API int rs_staytime_labels(void* stream, const int64_t* watch_ms, const uint8_t* landing,
                              int64_t B, const float* bins, int nbins, float sigma, float left,
                              float right, float* label, int64_t ld, float* short_label,
                              float* long_label, float* weight) {
  if (B < 0 || nbins <= 1 || !(sigma > 0.f) || ld < (int64_t)nbins + 1)
    return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  if (!watch_ms || !bins || !label) return RS_ERR_ARG;
  // Python-float constants of parse.py:55-59, rounded to fp32 the way TF converts them.
  const double s = (double)sigma;
  const float neg_two_sigma2 = (float)(-2.0 * s * s);
  const float norm = (float)(2.5066282746310002 * s);  // math.sqrt(2 * math.pi) * sigma
  const float width = (float)(((double)right - (double)left) / (double)(nbins - 1));
  int exp2;
  const bool pow2_div = std::frexp((double)neg_two_sigma2, &exp2) == -0.5;
  int64_t grid = (B + 3) / 4;
  if (grid > 8192) grid = 8192;
  staytime_label_kernel<<<(int)grid, kLabelThreads, 0, rs_stream(stream)>>>(
      watch_ms, landing, B, bins, nbins, neg_two_sigma2, pow2_div, 1.0f / neg_two_sigma2, norm, width, label, ld, short_label,
      long_label, weight);
  return rs_status_after_launch();
}
