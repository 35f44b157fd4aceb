// H2 / H12 / H13 -- the rank/ctr BaseModel front end and the per-sample pieces of the rank/ctr
// and rank/finish models.
//
//   rs_gather_columns / rs_scatter_add_columns
//       emb_dict[slot][:, s0:s1] interval slicing + Concatenate of the BaseModel front end
//       (rank/ctr/base_model.py:134-154): out[b, j] = src[b, cols[j]] over a column plan
//       (feature_config.SlotLayout.column_plan); backward adds into the source columns.
//   rs_segment_mean
//       the SENet squeeze tf.reduce_mean(emb, axis=1) per structure field (model_init.py:22-24).
//   rs_field_scale_fwd / _bwd
//       multiply([emb_input, senet_split_output]) per field (model_init.py:38-40).
//   rs_field_linear_fwd / _bwd
//       the 175 per-field Dense(8) maps (model_init.py:44-46): field f's columns [seg[f],
//       seg[f+1]) times its own [w_f, O] kernel; the kernels are stored packed as one [C, O]
//       matrix (row c belongs to the field that owns column c).
//   rs_can_fwd / _bwd
//       the CAN per-sample matmuls (model_init.py:90-98, 150-154): relu(relu(r W1 + b1) W2 + b2)
//       with W1 [8, 6], b1, W2 [6, 4], b2 sliced out of each sample's Dense(82) row.
//   rs_fm_proj_fwd / _bwd
//       rank/finish FMLayer.call's second-order term (rank/finish/videodnn.py:41-50):
//       0.5 * sum_k ((x V)_k^2 - (x^2 V^2)_k) with the learned fm_matrix V [D, 8].
//
// All fp32, one thread per output element (these are VALU-light, HBM-bound gathers and tiny
// per-sample products); weight gradients reduce over the batch in fixed-order chunks
// (per-chunk partial rows + column_reduce_kernel): deterministic.
#include "common.hpp"

namespace {

constexpr int kBlk = 256;
constexpr int kChunk = 256;  // samples per partial row of a batch reduction

unsigned grid_for(int64_t n) {
  int64_t g = (n + kBlk - 1) / kBlk;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

// ---- column gather / scatter-add ------------------------------------------------------------
__global__ void __launch_bounds__(kBlk) gather_cols_kernel(const float* __restrict__ src,
                                                           int64_t src_ld, int64_t B,
                                                           const int32_t* __restrict__ cols,
                                                           int ncols, float* __restrict__ out,
                                                           int64_t out_ld) {
  const int64_t n = B * ncols;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / ncols;
    const int j = (int)(i - b * ncols);
    out[b * out_ld + j] = src[b * src_ld + cols[j]];
  }
}

__global__ void __launch_bounds__(kBlk) scatter_add_cols_kernel(const float* __restrict__ dout,
                                                                int64_t out_ld, int64_t B,
                                                                const int32_t* __restrict__ cols,
                                                                int ncols, float* __restrict__ dsrc,
                                                                int64_t src_ld) {
  const int64_t n = B * ncols;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / ncols;
    const int j = (int)(i - b * ncols);
    // a plan may name a column twice (the same interval sliced twice): the gradients add up, so
    // the update is an atomic (no-return global f32 add; as cheap as a plain RMW when unique)
    atomicAdd(dsrc + b * src_ld + cols[j], dout[b * out_ld + j]);
  }
}

// ---- per-field reductions / scaling -----------------------------------------------------------
__global__ void __launch_bounds__(kBlk) segment_mean_kernel(const float* __restrict__ x,
                                                            int64_t x_ld, int64_t B,
                                                            const int32_t* __restrict__ seg, int F,
                                                            float* __restrict__ out,
                                                            int64_t out_ld) {
  const int64_t n = B * F;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / F;
    const int f = (int)(i - b * F);
    const int c0 = seg[f], c1 = seg[f + 1];
    float s = 0.f;
    for (int c = c0; c < c1; ++c) s += x[b * x_ld + c];  // TF reduce_mean: sum, then / n
    out[b * out_ld + f] = c1 > c0 ? s / (float)(c1 - c0) : 0.f;
  }
}

__global__ void __launch_bounds__(kBlk) field_scale_fwd_kernel(
    const float* __restrict__ x, int64_t x_ld, int64_t B, const int32_t* __restrict__ colfield,
    int C, const float* __restrict__ s, int64_t s_ld, float alpha, float* __restrict__ y,
    int64_t y_ld) {
  const int64_t n = B * C;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / C;
    const int c = (int)(i - b * C);
    // TF: multiply(x, alpha * s) -- alpha = 2 (a power of two) makes x * (2 s) == 2 (x s) exactly
    y[b * y_ld + c] = x[b * x_ld + c] * (alpha * s[b * s_ld + colfield[c]]);
  }
}

// one thread per (b, f): dx over the field's columns, ds = sum_c dy * x
__global__ void __launch_bounds__(kBlk) field_scale_bwd_kernel(
    const float* __restrict__ dy, int64_t dy_ld, const float* __restrict__ x, int64_t x_ld,
    int64_t B, const int32_t* __restrict__ seg, int F, const float* __restrict__ s, int64_t s_ld,
    float alpha, float* __restrict__ dx, int64_t dx_ld, int dx_accumulate, float* __restrict__ ds,
    int64_t ds_ld) {
  const int64_t n = B * F;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / F;
    const int f = (int)(i - b * F);
    const float sv = alpha * s[b * s_ld + f];
    float acc = 0.f;
    for (int c = seg[f]; c < seg[f + 1]; ++c) {
      const float g = dy[b * dy_ld + c];
      acc = fmaf(g, x[b * x_ld + c], acc);
      if (dx) {
        float* d = dx + b * dx_ld + c;
        *d = dx_accumulate ? *d + g * sv : g * sv;
      }
    }
    if (ds) ds[b * ds_ld + f] = alpha * acc;  // d/ds of x * (alpha s)
  }
}

// ---- per-field Dense(O) ------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlk) field_linear_fwd_kernel(
    const float* __restrict__ x, int64_t x_ld, int64_t B, const int32_t* __restrict__ seg, int F,
    int O, const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ y,
    int64_t y_ld) {
  const int64_t n = B * F * O;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / ((int64_t)F * O);
    const int r = (int)(i - b * F * O), f = r / O, o = r - f * O;
    float acc = 0.f;
    for (int c = seg[f]; c < seg[f + 1]; ++c) acc = fmaf(x[b * x_ld + c], W[(int64_t)c * O + o], acc);
    y[b * y_ld + r] = acc + bias[r];  // tensordot, then bias_add (Keras Dense)
  }
}

// dx[b, c] (+)= sum_o dy[b, f(c), o] W[c, o]
__global__ void __launch_bounds__(kBlk) field_linear_dx_kernel(
    const float* __restrict__ dy, int64_t dy_ld, int64_t B, const int32_t* __restrict__ colfield,
    int C, int O, const float* __restrict__ W, float* __restrict__ dx, int64_t dx_ld,
    int accumulate) {
  const int64_t n = B * C;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / C;
    const int c = (int)(i - b * C);
    const float* g = dy + b * dy_ld + (int64_t)colfield[c] * O;
    float acc = 0.f;
    for (int o = 0; o < O; ++o) acc = fmaf(g[o], W[(int64_t)c * O + o], acc);
    float* d = dx + b * dx_ld + c;
    *d = accumulate ? *d + acc : acc;
  }
}

// batch-chunk partials: part[chunk][c * O + o] = sum_{b in chunk} x[b, c] dy[b, f(c), o];
// part[chunk][C * O + f * O + o] = sum_{b in chunk} dy[b, f, o]
__global__ void __launch_bounds__(kBlk) field_linear_dw_kernel(
    const float* __restrict__ dy, int64_t dy_ld, const float* __restrict__ x, int64_t x_ld,
    int64_t B, const int32_t* __restrict__ colfield, int C, int F, int O,
    float* __restrict__ part) {
  const int64_t J = (int64_t)C * O + (int64_t)F * O;
  const int64_t j = (int64_t)blockIdx.x * kBlk + threadIdx.x;
  if (j >= J) return;
  const int64_t b0 = (int64_t)blockIdx.y * kChunk;
  const int64_t b1 = b0 + kChunk < B ? b0 + kChunk : B;
  float acc = 0.f;
  if (j < (int64_t)C * O) {
    const int c = (int)(j / O), o = (int)(j - (int64_t)c * O);
    const int64_t go = (int64_t)colfield[c] * O + o;
    for (int64_t b = b0; b < b1; ++b) acc = fmaf(x[b * x_ld + c], dy[b * dy_ld + go], acc);
  } else {
    const int64_t r = j - (int64_t)C * O;
    for (int64_t b = b0; b < b1; ++b) acc += dy[b * dy_ld + r];
  }
  part[(int64_t)blockIdx.y * J + j] = acc;
}

// ---- CAN ----------------------------------------------------------------------------------------
// p row layout (tf.split(can_inputs, [8*6, 6, 6*4, 4])): W1 [8][6] at 0, b1 at 48, W2 [6][4] at
// 54, b2 at 78 (tf.reshape keeps row-major order).
constexpr int kCanIn = 8, kCanH = 6, kCanOut = 4, kCanP = 82;

__global__ void __launch_bounds__(kBlk) can_fwd_kernel(const float* __restrict__ r, int64_t r_ld,
                                                       const float* __restrict__ p, int64_t p_ld,
                                                       int64_t B, float* __restrict__ out,
                                                       int64_t out_ld, float* __restrict__ h_save) {
  for (int64_t b = (int64_t)blockIdx.x * kBlk + threadIdx.x; b < B; b += (int64_t)gridDim.x * kBlk) {
    const float* pr = p + b * p_ld;
    float x[kCanIn], h[kCanH];
#pragma unroll
    for (int i = 0; i < kCanIn; ++i) x[i] = r[b * r_ld + i];
#pragma unroll
    for (int j = 0; j < kCanH; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < kCanIn; ++i) acc = fmaf(x[i], pr[i * kCanH + j], acc);
      h[j] = fmaxf(acc + pr[48 + j], 0.f);  // matmul + can_bias1, ReLU
      if (h_save) h_save[b * kCanH + j] = h[j];
    }
#pragma unroll
    for (int k = 0; k < kCanOut; ++k) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < kCanH; ++j) acc = fmaf(h[j], pr[54 + j * kCanOut + k], acc);
      out[b * out_ld + k] = fmaxf(acc + pr[78 + k], 0.f);
    }
  }
}

__global__ void __launch_bounds__(kBlk) can_bwd_kernel(
    const float* __restrict__ dout, int64_t dout_ld, const float* __restrict__ out, int64_t out_ld,
    const float* __restrict__ r, int64_t r_ld, const float* __restrict__ p, int64_t p_ld,
    const float* __restrict__ h, int64_t B, float* __restrict__ dr, int64_t dr_ld,
    int dr_accumulate, float* __restrict__ dp, int64_t dp_ld) {
  for (int64_t b = (int64_t)blockIdx.x * kBlk + threadIdx.x; b < B; b += (int64_t)gridDim.x * kBlk) {
    const float* pr = p + b * p_ld;
    float* dpr = dp + b * dp_ld;
    float dz2[kCanOut], dh[kCanH];
#pragma unroll
    for (int k = 0; k < kCanOut; ++k) {
      dz2[k] = out[b * out_ld + k] > 0.f ? dout[b * dout_ld + k] : 0.f;  // ReluGrad: out > 0
      dpr[78 + k] = dz2[k];
    }
#pragma unroll
    for (int j = 0; j < kCanH; ++j) {
      const float hj = h[b * kCanH + j];
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < kCanOut; ++k) {
        dpr[54 + j * kCanOut + k] = hj * dz2[k];
        acc = fmaf(pr[54 + j * kCanOut + k], dz2[k], acc);
      }
      dh[j] = hj > 0.f ? acc : 0.f;
      dpr[48 + j] = dh[j];
    }
#pragma unroll
    for (int i = 0; i < kCanIn; ++i) {
      const float xi = r[b * r_ld + i];
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < kCanH; ++j) {
        dpr[i * kCanH + j] = xi * dh[j];
        acc = fmaf(pr[i * kCanH + j], dh[j], acc);
      }
      float* d = dr + b * dr_ld + i;
      *d = dr_accumulate ? *d + acc : acc;
    }
  }
}

// ---- FM projection (rank/finish FMLayer) ---------------------------------------------------------
// one wave-segment of N (<= 64, power of two) lanes per sample: lane n forms (xV)_n and
// (x^2 V^2)_n, the group sums 0.5 * ((xV)_n^2 - (x^2 V^2)_n) over n
template <int N>
__global__ void __launch_bounds__(kBlk) fm_proj_fwd_kernel(const float* __restrict__ x,
                                                           int64_t x_ld, int64_t B, int K,
                                                           const float* __restrict__ V,
                                                           const float* __restrict__ add,
                                                           float* __restrict__ y,
                                                           float* __restrict__ xv_save) {
  const int n = threadIdx.x % N;
  for (int64_t b = ((int64_t)blockIdx.x * kBlk + threadIdx.x) / N; b < B;
       b += (int64_t)gridDim.x * (kBlk / N)) {
    const float* xr = x + b * x_ld;
    float s1 = 0.f, s2 = 0.f;
    for (int c = 0; c < K; ++c) {
      const float xc = xr[c], v = V[(int64_t)c * N + n];
      s1 = fmaf(xc, v, s1);                   // matmul(inputs, fm_matrix)
      s2 = fmaf(xc * xc, v * v, s2);          // matmul(square(inputs), square(fm_matrix))
    }
    if (xv_save) xv_save[b * N + n] = s1;
    float t = s1 * s1 - s2;
    t = group_sum<N>(t);
    if (n == 0) y[b] = add ? 0.5f * t + add[b] : 0.5f * t;  // tf.math.add(high_order, linear)
  }
}

// dx[b, c] (+)= dy[b] * sum_n (xv[b, n] V[c, n] - x[b, c] V[c, n]^2)
__global__ void __launch_bounds__(kBlk) fm_proj_dx_kernel(const float* __restrict__ dy,
                                                          const float* __restrict__ x,
                                                          int64_t x_ld, int64_t B, int K, int N,
                                                          const float* __restrict__ V,
                                                          const float* __restrict__ xv,
                                                          float* __restrict__ dx, int64_t dx_ld,
                                                          int accumulate) {
  const int64_t total = B * K;
  for (int64_t i = (int64_t)blockIdx.x * kBlk + threadIdx.x; i < total; i += (int64_t)gridDim.x * kBlk) {
    const int64_t b = i / K;
    const int c = (int)(i - b * K);
    const float xc = x[b * x_ld + c];
    float acc = 0.f;
    for (int n = 0; n < N; ++n) {
      const float v = V[(int64_t)c * N + n];
      acc = fmaf(xv[b * N + n] - xc * v, v, acc);
    }
    float* d = dx + b * dx_ld + c;
    *d = accumulate ? fmaf(dy[b], acc, *d) : dy[b] * acc;
  }
}

// part[chunk][c * N + n] = sum_{b in chunk} dy[b] (xv[b, n] x[b, c] - x[b, c]^2 V[c, n])
__global__ void __launch_bounds__(kBlk) fm_proj_dv_kernel(const float* __restrict__ dy,
                                                          const float* __restrict__ x,
                                                          int64_t x_ld, int64_t B, int K, int N,
                                                          const float* __restrict__ V,
                                                          const float* __restrict__ xv,
                                                          float* __restrict__ part) {
  const int64_t J = (int64_t)K * N;
  const int64_t j = (int64_t)blockIdx.x * kBlk + threadIdx.x;
  if (j >= J) return;
  const int c = (int)(j / N), n = (int)(j - (int64_t)c * N);
  const float v = V[j];
  const int64_t b0 = (int64_t)blockIdx.y * kChunk;
  const int64_t b1 = b0 + kChunk < B ? b0 + kChunk : B;
  float acc = 0.f;
  for (int64_t b = b0; b < b1; ++b) {
    const float xc = x[b * x_ld + c];
    acc = fmaf(dy[b], xc * (xv[b * N + n] - xc * v), acc);
  }
  part[(int64_t)blockIdx.y * J + j] = acc;
}

int64_t chunks(int64_t B) { return (B + kChunk - 1) / kChunk; }

}  // namespace

RS_API int rs_gather_columns(void* stream, const float* src, int64_t src_ld, int64_t B,
                             const int32_t* cols, int ncols, float* out, int64_t out_ld) {
  if (!src || !cols || !out || B < 0 || ncols < 0 || out_ld < ncols) return RS_ERR_ARG;
  if (B * ncols == 0) return RS_OK;
  gather_cols_kernel<<<grid_for(B * ncols), kBlk, 0, rs_stream(stream)>>>(src, src_ld, B, cols,
                                                                          ncols, out, out_ld);
  return rs_status_after_launch();
}

RS_API int rs_scatter_add_columns(void* stream, const float* dout, int64_t out_ld, int64_t B,
                                  const int32_t* cols, int ncols, float* dsrc, int64_t src_ld) {
  if (!dout || !cols || !dsrc || B < 0 || ncols < 0 || out_ld < ncols) return RS_ERR_ARG;
  if (B * ncols == 0) return RS_OK;
  scatter_add_cols_kernel<<<grid_for(B * ncols), kBlk, 0, rs_stream(stream)>>>(
      dout, out_ld, B, cols, ncols, dsrc, src_ld);
  return rs_status_after_launch();
}

RS_API int rs_segment_mean(void* stream, const float* x, int64_t x_ld, int64_t B,
                           const int32_t* seg, int F, float* out, int64_t out_ld) {
  if (!x || !seg || !out || B < 0 || F <= 0 || out_ld < F) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  segment_mean_kernel<<<grid_for(B * F), kBlk, 0, rs_stream(stream)>>>(x, x_ld, B, seg, F, out,
                                                                       out_ld);
  return rs_status_after_launch();
}

RS_API int rs_field_scale_fwd(void* stream, const float* x, int64_t x_ld, int64_t B,
                              const int32_t* colfield, int C, const float* s, int64_t s_ld,
                              float alpha, float* y, int64_t y_ld) {
  if (!x || !colfield || !s || !y || B < 0 || C <= 0 || y_ld < C) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  field_scale_fwd_kernel<<<grid_for(B * C), kBlk, 0, rs_stream(stream)>>>(x, x_ld, B, colfield, C,
                                                                          s, s_ld, alpha, y, y_ld);
  return rs_status_after_launch();
}

RS_API int rs_field_scale_bwd(void* stream, const float* dy, int64_t dy_ld, const float* x,
                              int64_t x_ld, int64_t B, const int32_t* seg, int F, const float* s,
                              int64_t s_ld, float alpha, float* dx, int64_t dx_ld,
                              int dx_accumulate, float* ds, int64_t ds_ld) {
  if (!dy || !x || !seg || !s || B < 0 || F <= 0 || (!dx && !ds)) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  field_scale_bwd_kernel<<<grid_for(B * F), kBlk, 0, rs_stream(stream)>>>(
      dy, dy_ld, x, x_ld, B, seg, F, s, s_ld, alpha, dx, dx_ld, dx_accumulate, ds, ds_ld);
  return rs_status_after_launch();
}

RS_API int rs_field_linear_fwd(void* stream, const float* x, int64_t x_ld, int64_t B,
                               const int32_t* seg, int F, int O, const float* W,
                               const float* bias, float* y, int64_t y_ld) {
  if (!x || !seg || !W || !bias || !y || B < 0 || F <= 0 || O <= 0 || y_ld < (int64_t)F * O)
    return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  field_linear_fwd_kernel<<<grid_for(B * F * O), kBlk, 0, rs_stream(stream)>>>(
      x, x_ld, B, seg, F, O, W, bias, y, y_ld);
  return rs_status_after_launch();
}

RS_API int64_t rs_field_linear_workspace_floats(int64_t B, int C, int F, int O) {
  return chunks(B) * ((int64_t)C * O + (int64_t)F * O);
}

// dx: NULL to skip; dW [C, O] and db [F, O] are overwritten (dparams_accumulate = 0) or added to
RS_API int rs_field_linear_bwd(void* stream, const float* dy, int64_t dy_ld, const float* x,
                               int64_t x_ld, int64_t B, const int32_t* seg,
                               const int32_t* colfield, int C, int F, int O, const float* W,
                               float* dx, int64_t dx_ld, int dx_accumulate, float* dW, float* db,
                               int dparams_accumulate, float* workspace,
                               int64_t workspace_floats) {
  if (!dy || !x || !seg || !colfield || !W || B < 0 || C <= 0 || F <= 0 || O <= 0 || !dW || !db)
    return RS_ERR_ARG;
  if (workspace_floats < rs_field_linear_workspace_floats(B, C, F, O) || !workspace) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  if (dx)
    field_linear_dx_kernel<<<grid_for(B * C), kBlk, 0, s>>>(dy, dy_ld, B, colfield, C, O, W, dx,
                                                           dx_ld, dx_accumulate);
  const int64_t J = (int64_t)C * O + (int64_t)F * O;
  dim3 grid((unsigned)((J + kBlk - 1) / kBlk), (unsigned)chunks(B));
  field_linear_dw_kernel<<<grid, kBlk, 0, s>>>(dy, dy_ld, x, x_ld, B, colfield, C, F, O, workspace);
  launch_column_reduce(s, workspace, (int)chunks(B), J, J, (int64_t)C * O, dW, db,
                       dparams_accumulate);
  return rs_status_after_launch();
}

RS_API int rs_can_fwd(void* stream, const float* r, int64_t r_ld, const float* p, int64_t p_ld,
                      int64_t B, float* out, int64_t out_ld, float* h_save) {
  if (!r || !p || !out || B < 0 || r_ld < kCanIn || p_ld < kCanP || out_ld < kCanOut) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  can_fwd_kernel<<<grid_for(B), kBlk, 0, rs_stream(stream)>>>(r, r_ld, p, p_ld, B, out, out_ld,
                                                             h_save);
  return rs_status_after_launch();
}

RS_API int rs_can_bwd(void* stream, const float* dout, int64_t dout_ld, const float* out,
                      int64_t out_ld, const float* r, int64_t r_ld, const float* p, int64_t p_ld,
                      const float* h, int64_t B, float* dr, int64_t dr_ld, int dr_accumulate,
                      float* dp, int64_t dp_ld) {
  if (!dout || !out || !r || !p || !h || !dr || !dp || B < 0 || dp_ld < kCanP) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  can_bwd_kernel<<<grid_for(B), kBlk, 0, rs_stream(stream)>>>(dout, dout_ld, out, out_ld, r, r_ld,
                                                             p, p_ld, h, B, dr, dr_ld,
                                                             dr_accumulate, dp, dp_ld);
  return rs_status_after_launch();
}

RS_API int rs_fm_proj_fwd(void* stream, const float* x, int64_t x_ld, int64_t B, int K, int N,
                          const float* V, const float* add, float* y, float* xv_save) {
  if (!x || !V || !y || B < 0 || K <= 0 || x_ld < K) return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  const unsigned grid = grid_for(B * N);
  switch (N) {
    case 4: fm_proj_fwd_kernel<4><<<grid, kBlk, 0, s>>>(x, x_ld, B, K, V, add, y, xv_save); break;
    case 8: fm_proj_fwd_kernel<8><<<grid, kBlk, 0, s>>>(x, x_ld, B, K, V, add, y, xv_save); break;
    case 16: fm_proj_fwd_kernel<16><<<grid, kBlk, 0, s>>>(x, x_ld, B, K, V, add, y, xv_save); break;
    default: return RS_ERR_UNSUPPORTED;
  }
  return rs_status_after_launch();
}

RS_API int64_t rs_fm_proj_workspace_floats(int64_t B, int K, int N) {
  return chunks(B) * (int64_t)K * N;
}

RS_API int rs_fm_proj_bwd(void* stream, const float* dy, const float* x, int64_t x_ld, int64_t B,
                          int K, int N, const float* V, const float* xv, float* dx, int64_t dx_ld,
                          int dx_accumulate, float* dV, int dV_accumulate, float* workspace,
                          int64_t workspace_floats) {
  if (!dy || !x || !V || !xv || !dV || B < 0 || K <= 0 || N <= 0 || !workspace ||
      workspace_floats < rs_fm_proj_workspace_floats(B, K, N))
    return RS_ERR_ARG;
  if (B == 0) return RS_OK;
  hipStream_t s = rs_stream(stream);
  if (dx)
    fm_proj_dx_kernel<<<grid_for(B * K), kBlk, 0, s>>>(dy, x, x_ld, B, K, N, V, xv, dx, dx_ld,
                                                      dx_accumulate);
  const int64_t J = (int64_t)K * N;
  dim3 grid((unsigned)((J + kBlk - 1) / kBlk), (unsigned)chunks(B));
  fm_proj_dv_kernel<<<grid, kBlk, 0, s>>>(dy, x, x_ld, B, K, N, V, xv, workspace);
  launch_column_reduce(s, workspace, (int)chunks(B), J, J, J, dV, nullptr, dV_accumulate);
  return rs_status_after_launch();
}

// ---- the backward of several column gathers from one source, as one gather ------------------
// out[b, c] = sum_k (map[k][c] >= 0 ? src_k[b * ld_k + map[k][c]] : 0) for c < ncols: every output
// element written once (no zero fill, no atomics, no accumulate chain).  The staytime trunk reads
// general = emb[:, :, 0:16], the DIN queries general[:, q] and the gate input emb[:, bias, 16:32]
// from the field embeddings (VideoDnn.py:45-47, 57-77, 127); their gradients meet in d_emb here.
namespace {
constexpr int kMaxSumSrc = 8;
struct SumSrc {
  const float* p[kMaxSumSrc];
  int64_t ld[kMaxSumSrc];
};

// 2-D grid: a thread owns one output column c (its nsrc map entries in registers) and walks rows
// b = blockIdx.y, + gridDim.y, ... (the flat form paid a 64-bit division and nsrc map loads per
// element: 33.5 us for config 5's 2048 x 2912 d_emb).
__global__ void __launch_bounds__(kBlk) gather_sum_cols_kernel(SumSrc src, int nsrc,
                                                               const int32_t* __restrict__ map,
                                                               int64_t B, int ncols,
                                                               float* __restrict__ out,
                                                               int64_t out_ld) {
  const int c = blockIdx.x * kBlk + threadIdx.x;
  if (c >= ncols) return;
  int32_t sc[kMaxSumSrc];
#pragma unroll
  for (int k = 0; k < kMaxSumSrc; ++k) sc[k] = k < nsrc ? map[(int64_t)k * ncols + c] : -1;
  for (int64_t b = blockIdx.y; b < B; b += gridDim.y) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < kMaxSumSrc; ++k)
      if (sc[k] >= 0) v += src.p[k][b * src.ld[k] + sc[k]];
    out[b * out_ld + c] = v;
  }
}
}  // namespace

RS_API int rs_gather_sum_columns(void* stream, int nsrc, const float* const* srcs,
                                 const int64_t* src_lds, const int32_t* map, int64_t B, int ncols,
                                 float* out, int64_t out_ld) {
  if (nsrc < 1 || nsrc > kMaxSumSrc || !srcs || !src_lds || !map || !out || B < 0 || ncols < 0 ||
      out_ld < ncols)
    return RS_ERR_ARG;
  SumSrc s{};
  for (int k = 0; k < nsrc; ++k) {  // host arrays of device pointers / strides
    if (!srcs[k]) return RS_ERR_ARG;
    s.p[k] = srcs[k];
    s.ld[k] = src_lds[k];
  }
  if (B * ncols == 0) return RS_OK;
  const unsigned gx = (unsigned)((ncols + kBlk - 1) / kBlk);
  int64_t gy = (2048 + gx - 1) / gx;  // ~2048 blocks in all
  if (gy > B) gy = B;
  if (gy > 65535) gy = 65535;
  gather_sum_cols_kernel<<<dim3(gx, (unsigned)gy), kBlk, 0, rs_stream(stream)>>>(s, nsrc, map, B,
                                                                                 ncols, out, out_ld);
  return rs_status_after_launch();
}
