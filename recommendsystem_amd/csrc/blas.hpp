// Library GEMMs (hipBLASLt) behind the Dense entry points: the large plain fp32 GEMMs of the
// configs-3/5 towers.  The hand-written engine in dense.hip keeps every GEMM below
// the size threshold, every fused form the library has no epilogue for (sigmoid forward, the
// grouped launches) and any shape the library returns no algorithm for.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// Column-major D[m x n] = op(A) op(B) (+ beta D) (+ bias[row]) (relu): op(A) is m x k, op(B) k x n.
// Returns 0 when the product was enqueued on s, nonzero when the library cannot run it (no
// algorithm, not initialised, disabled): the caller then runs its own kernel.
int rs_blas_gemm_cm(hipStream_t s, bool trans_a, bool trans_b, int64_t m, int64_t n, int64_t k,
                    const float* A, int64_t lda, const float* B, int64_t ldb, float beta,
                    float* D, int64_t ldd, const float* bias, bool relu);

// Whether a GEMM of m * n * k multiply-adds goes to the library (RS_GEMM_BLAS=0 disables it,
// RS_GEMM_BLAS_MACS sets the threshold).
bool rs_blas_wanted(int64_t m, int64_t n, int64_t k);
