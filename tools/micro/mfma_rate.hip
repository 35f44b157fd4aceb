// Microbenchmark: back-to-back f32 MFMA throughput per SIMD from one or two waves per SIMD
// (v_mfma_f32_16x16x4_f32 on 8 independent accumulators, v_mfma_f32_32x32x2_f32 on 2).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256) k16(float* out, int iters) {
  f4 acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k32(float* out, int iters) {
  f16v acc[2];
  for (int i = 0; i < 2; ++i) for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 2; ++i) for (int e = 0; e < 16; ++e) s += acc[i][e];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 24);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 4000;
  for (int wps = 1; wps <= 2; ++wps) {
    const int blocks = 256 * wps;  // 4 waves per block: wps waves per SIMD
    for (int kind = 0; kind < 2; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (kind == 0) k16<<<blocks, 256>>>(out, iters); else k32<<<blocks, 256>>>(out, iters);
        hipEventRecord(b);
        hipEventSynchronize(b);
      }
      float ms; hipEventElapsedTime(&ms, a, b);
      // per SIMD: wps waves x iters x 32 MFMAs (16x16x4: 1024 MAC; 32x32x2: 2048 MAC, 16 per iter)
      const double macs = (double)blocks * 4 * iters * 32 * 1024.0;  // both kinds: 32K MAC/iter/wave
      const double tf = 2 * macs / (ms * 1e-3) / 1e12;
      const double mf = kind == 0 ? 32.0 : 16.0;
      printf("%s waves/SIMD=%d: %.3f ms, %.1f TF/s, %.1f cycles/MFMA/SIMD at 2.4 GHz\n",
             kind == 0 ? "16x16x4" : "32x32x2", wps, ms, tf, ms * 1e-3 * 2.4e9 / (wps * iters * mf));
    }
  }
  return 0;
}
