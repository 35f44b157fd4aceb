// hipBLASLt for the large plain fp32 GEMMs of the Dense layers (blas.hpp).  One handle and one
// workspace per process, created on the first eligible call (an eager step: graph capture
// replays the plans a warm-up step made); one plan per (shape, layout, epilogue): matmul
// descriptor, four matrix layouts and an algorithm, cached.  The algorithm is the fastest of the
// heuristic's top candidates (32; RS_GEMM_BLAS_CANDS), each timed on scratch operands of the plan's shape on a private
// stream when the plan is made outside a graph capture (the heuristic's first pick otherwise, or
// with RS_GEMM_BLAS_TUNE=0).  The bias pointer is set on the cached descriptor per call
// (host-side attribute; a captured launch keeps the one it was recorded with).
#include "blas.hpp"

#include <hipblaslt/hipblaslt.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace {

constexpr size_t kWsBytes = (size_t)64 << 20;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

using Key = std::tuple<int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int>;

struct Ctx {
  std::mutex mu;
  bool tried = false, ok = false;
  hipblasLtHandle_t h = nullptr;
  void* ws = nullptr;
  std::map<Key, Plan> plans;
};

Ctx& ctx() {
  static Ctx c;
  return c;
}

bool init_locked(Ctx& c) {
  if (c.tried) return c.ok;
  c.tried = true;
  if (hipblasLtCreate(&c.h) != HIPBLAS_STATUS_SUCCESS) return false;
  if (hipMalloc(&c.ws, kWsBytes) != hipSuccess) {
    c.ws = nullptr;
    return false;
  }
  c.ok = true;
  return true;
}

int64_t env_i64(const char* name, int64_t dflt) {
  const char* e = getenv(name);
  if (!e || !*e) return dflt;
  return (int64_t)strtoll(e, nullptr, 10);
}

// Times each usable candidate (1 warm-up + 5 timed runs) on zero-filled scratch operands of the
// plan's shape; returns the index of the fastest (`dflt` if anything fails).
int time_candidates(Ctx& c, Plan& p, const hipblasLtMatmulHeuristicResult_t* res, int got, int dflt,
                    bool ta, bool tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
                    int64_t ldd, int epi, bool beta) {
  const size_t na = (size_t)lda * (size_t)(ta ? m : k), nb = (size_t)ldb * (size_t)(tb ? k : n);
  const size_t nd = (size_t)ldd * (size_t)n, nbias = (size_t)(m > n ? m : n);
  float *A = nullptr, *B = nullptr, *D = nullptr, *bias = nullptr;
  hipStream_t ts = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int pick = dflt;
  const bool ok = hipMalloc(&A, na * 4) == hipSuccess && hipMalloc(&B, nb * 4) == hipSuccess &&
                  hipMalloc(&D, nd * 4) == hipSuccess && hipMalloc(&bias, nbias * 4) == hipSuccess &&
                  hipStreamCreateWithFlags(&ts, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess &&
                  hipMemsetAsync(A, 0, na * 4, ts) == hipSuccess &&
                  hipMemsetAsync(B, 0, nb * 4, ts) == hipSuccess &&
                  hipMemsetAsync(D, 0, nd * 4, ts) == hipSuccess &&
                  hipMemsetAsync(bias, 0, nbias * 4, ts) == hipSuccess;
  if (ok) {
    if (epi != HIPBLASLT_EPILOGUE_DEFAULT)
      hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias,
                                      sizeof(bias));
    const float alpha = 1.f, bt = beta ? 1.f : 0.f;
    float best_ms = 1e30f;
    for (int i = 0; i < got; ++i) {
      if (res[i].workspaceSize > kWsBytes) continue;
      bool good = true;
      for (int r = 0; r < 6 && good; ++r) {
        if (r == 1) good = hipEventRecord(e0, ts) == hipSuccess;
        good = good && hipblasLtMatmul(c.h, p.desc, &alpha, A, p.a, B, p.b, &bt, D, p.d, D, p.d,
                                       &res[i].algo, c.ws, kWsBytes, ts) == HIPBLAS_STATUS_SUCCESS;
      }
      float ms = 0.f;
      good = good && hipEventRecord(e1, ts) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
             hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
      if (good && ms < best_ms) { best_ms = ms; pick = i; }
    }
    hipStreamSynchronize(ts);
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (ts) hipStreamDestroy(ts);
  hipFree(A); hipFree(B); hipFree(D); hipFree(bias);
  (void)hipGetLastError();
  return pick;
}

Plan make_plan(Ctx& c, bool ta, bool tb, int64_t m, int64_t n, int64_t k, int64_t lda, int64_t ldb,
               int64_t ldd, int epi, bool beta, bool tune) {
  Plan p;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS)
    return p;
  const hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  const hipblasLtEpilogue_t e = (hipblasLtEpilogue_t)epi;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  if (epi != HIPBLASLT_EPILOGUE_DEFAULT) {
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  // stored shapes: A is m x k (k x m transposed), B k x n (n x k transposed)
  hipblasLtMatrixLayoutCreate(&p.a, HIP_R_32F, ta ? k : m, ta ? m : k, lda);
  hipblasLtMatrixLayoutCreate(&p.b, HIP_R_32F, tb ? n : k, tb ? k : n, ldb);
  hipblasLtMatrixLayoutCreate(&p.d, HIP_R_32F, m, n, ldd);
  hipblasLtMatmulPreference_t pref = nullptr;
  hipblasLtMatmulPreferenceCreate(&pref);
  const uint64_t wsb = kWsBytes;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb,
                                        sizeof(wsb));
  constexpr int kCand = 32;
  static const int ncand = [] {  // tuning runs: RS_GEMM_BLAS_CANDS (candidates timed)
    const int64_t v = env_i64("RS_GEMM_BLAS_CANDS", 32);
    return (int)(v < 1 ? 1 : (v > kCand ? kCand : v));
  }();
  hipblasLtMatmulHeuristicResult_t res[kCand];
  int got = 0;
  const int want = tune ? ncand : 1;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(c.h, p.desc, p.a, p.b, p.d, p.d, pref,
                                                             want, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || got <= 0) return p;
  int best = -1;
  for (int i = 0; i < got && best < 0; ++i)
    if (res[i].workspaceSize <= kWsBytes) best = i;
  if (best < 0) return p;
  if (tune && got > 1) best = time_candidates(c, p, res, got, best, ta, tb, m, n, k, lda, ldb, ldd,
                                              epi, beta);
  p.algo = res[best].algo;
  p.ok = true;
  return p;
}

}  // namespace

bool rs_blas_wanted(int64_t m, int64_t n, int64_t k) {
  // measured (tools/gemm_vs_blas.py, profiles/r05/blas/gemm.log): the library leads
  // on the towers' weight / data gradients from ~0.4 G multiply-adds (1.3-4x on the trunks); with
  // the timed algorithm choice it also wins from 67 M (config 3 1.586 -> 1.570 ms, config 5
  // 1.791 -> 1.784 ms against the 268 M threshold, profiles/r05/thr/)
  static const int64_t thr = env_i64("RS_GEMM_BLAS_MACS", (int64_t)1 << 26);
  static const bool on = env_i64("RS_GEMM_BLAS", 0) != 0;  // opt-in (round 6: gemm_big.hip)
  return on && m > 0 && n > 0 && k > 0 && m * n * k >= thr;
}

int rs_blas_gemm_cm(hipStream_t s, bool ta, bool tb, int64_t m, int64_t n, int64_t k,
                    const float* A, int64_t lda, const float* B, int64_t ldb, float beta, float* D,
                    int64_t ldd, const float* bias, bool relu) {
  Ctx& c = ctx();
  const int epi = bias ? (relu ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                       : (relu ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
  Plan* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (!init_locked(c)) return 1;
    const Key key{ta, tb, m, n, k, lda, ldb, ldd, epi, beta != 0.f};
    auto it = c.plans.find(key);
    if (it == c.plans.end()) {
      static const bool tune_on = env_i64("RS_GEMM_BLAS_TUNE", 1) != 0;
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      const bool capturing = hipStreamIsCapturing(s, &cs) != hipSuccess ||
                             cs != hipStreamCaptureStatusNone;
      it = c.plans.emplace(key, make_plan(c, ta, tb, m, n, k, lda, ldb, ldd, epi, beta != 0.f,
                                          tune_on && !capturing)).first;
    }
    p = &it->second;
    if (!p->ok) return 1;
    if (bias)
      hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias));
    const float alpha = 1.f;
    const hipblasStatus_t st = hipblasLtMatmul(c.h, p->desc, &alpha, A, p->a, B, p->b, &beta, D, p->d,
                                               D, p->d, &p->algo, c.ws, kWsBytes, s);
    return st == HIPBLAS_STATUS_SUCCESS ? 0 : 1;
  }
}
