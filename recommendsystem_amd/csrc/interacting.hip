// C-ABI entry points of the fused InteractingLayer (kernels: il_kernels.hpp, instantiations:
// il_inst_*.hip).  Replaces InteractingLayer.call (InteractingLayer.py:37-61) forward and the
// TF autograd of that graph for backward.
#include "il_kernels.hpp"

namespace rs_il {
RS_IL_DECLARE_UNIT(il_unit_a)
RS_IL_DECLARE_UNIT(il_unit_b)
RS_IL_DECLARE_UNIT(il_unit_c)
int il_large_fwd(const FwdReq& q);  // il_large.hip: F in (64, 256]
int il_large_bwd(const BwdReq& q);
int il_generic_fwd(const FwdReq& q);  // il_generic.hip: any (E, U, H), F <= 256, LDS-bounded
int il_generic_bwd(const BwdReq& q);
int64_t il_attn_save_floats(int64_t B, int F, int U, int H, int L);

void reduce_params(hipStream_t s, const float* partials, int nblocks, int nparam, float* out,
                   int accumulate) {
  launch_column_reduce(s, partials, nblocks, nparam, nparam, nparam, out, nullptr, accumulate);
}
}  // namespace rs_il

#ifdef RS_IL_STAMPS
namespace rs_il { unsigned long long* g_il_stamps = nullptr; }
// diagnostic build only (not part of include/recsys_amd.h)
RS_API void rs_il_debug_set_stamps(unsigned long long* p) { rs_il::g_il_stamps = p; }
#endif

// process-wide math mode (common.hpp); relaxed atomics: a mode change is ordered with the
// launches of the thread that made it, and other threads see it at their next launch
static int g_math_mode = RS_MATH_F32;
int rs_math_mode_now() { return __atomic_load_n(&g_math_mode, __ATOMIC_RELAXED); }

RS_API int rs_set_math_mode(int mode) {
  if (mode != RS_MATH_F32 && mode != RS_MATH_BF16) return RS_ERR_ARG;
  __atomic_store_n(&g_math_mode, mode, __ATOMIC_RELAXED);
  return RS_OK;
}

RS_API int rs_get_math_mode(void) { return rs_math_mode_now(); }

// InteractingLayer kernel variant (il_kernels.hpp: RS_IL_VARIANT_*), process-wide like the math mode
static int g_il_variant = rs_il::RS_IL_VARIANT_AUTO;
namespace rs_il {
int rs_il_variant_now() { return __atomic_load_n(&g_il_variant, __ATOMIC_RELAXED); }
}  // namespace rs_il

RS_API int rs_il_set_variant(int variant) {
  if (variant < rs_il::RS_IL_VARIANT_AUTO || variant > rs_il::RS_IL_VARIANT_WIDE) return RS_ERR_ARG;
  __atomic_store_n(&g_il_variant, variant, __ATOMIC_RELAXED);
  return RS_OK;
}

RS_API int rs_il_get_variant(void) { return rs_il::rs_il_variant_now(); }

static const int64_t* g_seed_offset = nullptr;
const int64_t* rs_seed_offset_now() { return __atomic_load_n(&g_seed_offset, __ATOMIC_RELAXED); }

RS_API int rs_set_seed_offset(const int64_t* dev_offset) {
  __atomic_store_n(&g_seed_offset, dev_offset, __ATOMIC_RELAXED);
  return RS_OK;
}

RS_API int rs_il_param_count(int E, int U) { return E * 4 * U + 4 * U + 2 * U; }

RS_API int64_t rs_il_bwd_workspace_floats(int64_t B, int E, int U) {
  int64_t grid = B < 1 ? 1 : B;
  if (grid > rs_il::kMaxBwdGrid) grid = rs_il::kMaxBwdGrid;
  return grid * (int64_t)rs_il_param_count(E, U);
}

// RS_IL_FORCE_GENERIC=1: every shape the generic kernels take runs them (A/B timing against the
// compiled-in instantiations; read once)
static bool force_generic() {
  static const bool on = [] {
    const char* e = getenv("RS_IL_FORCE_GENERIC");
    return e && e[0] == '1';
  }();
  return on;
}

static int il_fwd_impl(void* stream, const float* x, int64_t B, int F, int E, int U, int H,
                       int L, const float* W, const float* bias, const float* gamma,
                       const float* beta, float eps, int use_res, float drop_rate, uint64_t seed,
                       float* y, int64_t y_ld, float* xsave, float* asave) {
  if (!x || !W || !bias || !gamma || !beta || !y || B < 0 || F <= 0 || L <= 0 || H <= 0)
    return RS_ERR_ARG;
  if (U % H != 0 || (L > 1 && (E != U || !xsave))) return RS_ERR_ARG;
  if (drop_rate < 0.f || drop_rate >= 1.f || y_ld < (int64_t)F * U) return RS_ERR_ARG;
  rs_il::FwdReq q{rs_stream(stream), x, W, bias, gamma, beta, B, F, E, U, H, L, use_res,
                  eps, drop_rate, seed, y, xsave, y_ld};
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  q.asave = asave;
  if (force_generic()) {
    const int g = rs_il::il_generic_fwd(q);
    if (g != RS_ERR_UNSUPPORTED) return g;
  }
  int r = F > 64 ? rs_il::il_large_fwd(q) : rs_il::il_unit_a_fwd(q);
  if (F <= 64 && r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_b_fwd(q);
  if (F <= 64 && r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_c_fwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_generic_fwd(q);  // shapes with no instantiation
  return r;
}

RS_API int rs_il_fwd(void* stream, const float* x, int64_t B, int F, int E, int U, int H, int L,
                     const float* W, const float* bias, const float* gamma, const float* beta,
                     float eps, int use_res, float drop_rate, uint64_t seed, float* y,
                     int64_t y_ld, float* xsave) {
  return il_fwd_impl(stream, x, B, F, E, U, H, L, W, bias, gamma, beta, eps, use_res, drop_rate,
                     seed, y, y_ld, xsave, nullptr);
}

RS_API int64_t rs_il_attn_save_floats(int64_t B, int F, int U, int H, int L) {
  if (B < 0 || F <= 0 || U <= 0 || H <= 0 || L <= 0) return 0;
  return rs_il::il_attn_save_floats(B, F, U, H, L);
}

RS_API int rs_il_fwd_saved(void* stream, const float* x, int64_t B, int F, int E, int U, int H,
                           int L, const float* W, const float* bias, const float* gamma,
                           const float* beta, float eps, int use_res, float drop_rate,
                           uint64_t seed, float* y, int64_t y_ld, float* xsave, float* asave,
                           int64_t asave_floats) {
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need > 0 && (!asave || asave_floats < need)) return RS_ERR_ARG;
  return il_fwd_impl(stream, x, B, F, E, U, H, L, W, bias, gamma, beta, eps, use_res, drop_rate,
                     seed, y, y_ld, xsave, need > 0 ? asave : nullptr);
}

static int il_fwd_gather_impl(void* stream, const int64_t* ids, const int64_t* row_base,
                              const int64_t* bucket, int hash_mode, const float* table,
                              int64_t table_rows, float* x, int32_t* rows_out, int64_t B, int F,
                              int E, int U, int H, int L, const float* W, const float* bias,
                              const float* gamma, const float* beta, float eps, int use_res,
                              float drop_rate, uint64_t seed, float* y, int64_t y_ld,
                              float* xsave, float* asave) {
  if (!ids || !row_base || !bucket || !table || !x || !W || !bias || !gamma || !beta || !y ||
      B < 0 || F <= 0 || L <= 0 || H <= 0 || (hash_mode != RS_HASH_MOD && hash_mode != RS_HASH_SPLITMIX))
    return RS_ERR_ARG;
  if (U % H != 0 || (L > 1 && (E != U || !xsave))) return RS_ERR_ARG;
  if (drop_rate < 0.f || drop_rate >= 1.f || y_ld < (int64_t)F * U) return RS_ERR_ARG;
  if (F > 64) return RS_ERR_UNSUPPORTED;  // the many-field kernels read x (rs_embedding_lookup_fwd)
  if (table_rows <= 0 || table_rows > INT32_MAX) return RS_ERR_ARG;
  rs_il::FwdReq q{rs_stream(stream), x, W, bias, gamma, beta, B, F, E, U, H, L, use_res,
                  eps, drop_rate, seed, y, xsave, y_ld};
  q.gather_ids = ids;
  q.gather_base = row_base;
  q.gather_bucket = bucket;
  q.gather_table = table;
  q.gather_table_rows = table_rows;
  q.gather_rows = rows_out;
  q.gather_hash = hash_mode;
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  q.asave = asave;
  int r = rs_il::il_unit_a_fwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_b_fwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_c_fwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_generic_fwd(q);
  return r;
}

RS_API int rs_il_fwd_gather(void* stream, const int64_t* ids, const int64_t* row_base,
                            const int64_t* bucket, int hash_mode, const float* table,
                            int64_t table_rows, float* x, int32_t* rows_out, int64_t B, int F,
                            int E, int U, int H, int L, const float* W, const float* bias,
                            const float* gamma, const float* beta, float eps, int use_res,
                            float drop_rate, uint64_t seed, float* y, int64_t y_ld, float* xsave) {
  return il_fwd_gather_impl(stream, ids, row_base, bucket, hash_mode, table, table_rows, x,
                            rows_out, B, F, E, U, H, L, W, bias, gamma, beta, eps, use_res,
                            drop_rate, seed, y, y_ld, xsave, nullptr);
}

RS_API int rs_il_fwd_gather_saved(void* stream, const int64_t* ids, const int64_t* row_base,
                                  const int64_t* bucket, int hash_mode, const float* table,
                                  int64_t table_rows, float* x, int32_t* rows_out, int64_t B,
                                  int F, int E, int U, int H, int L, const float* W,
                                  const float* bias, const float* gamma, const float* beta,
                                  float eps, int use_res, float drop_rate, uint64_t seed, float* y,
                                  int64_t y_ld, float* xsave, float* asave, int64_t asave_floats) {
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need > 0 && (!asave || asave_floats < need)) return RS_ERR_ARG;
  return il_fwd_gather_impl(stream, ids, row_base, bucket, hash_mode, table, table_rows, x,
                            rows_out, B, F, E, U, H, L, W, bias, gamma, beta, eps, use_res,
                            drop_rate, seed, y, y_ld, xsave, need > 0 ? asave : nullptr);
}

static int bwd_small(const rs_il::BwdReq& q) {
  if (force_generic() && !q.xt_x) {
    const int g = rs_il::il_generic_bwd(q);
    if (g != RS_ERR_UNSUPPORTED) return g;
  }
  int r = rs_il::il_unit_a_bwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_b_bwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_unit_c_bwd(q);
  if (r == RS_ERR_UNSUPPORTED) r = rs_il::il_generic_bwd(q);  // shapes with no instantiation
  return r;
}

// F > 64: the many-field instantiations, else the generic kernel
static int bwd_large(const rs_il::BwdReq& q) {
  const int r = rs_il::il_large_bwd(q);
  return r == RS_ERR_UNSUPPORTED ? rs_il::il_generic_bwd(q) : r;
}

// the deferred weight gradient a backward launch carries (rs_il_bwd_saved_xt /
// rs_il_bwd_push_saved_xt)
struct XtArgs {
  const float* x; int64_t ldx; const float* dz; int64_t lddz; int K0, N1; float* slab;
};
static void set_xt(rs_il::BwdReq& q, const XtArgs* xt) {
  if (!xt) return;
  q.xt_x = xt->x; q.xt_ldx = xt->ldx; q.xt_dz = xt->dz; q.xt_lddz = xt->lddz;
  q.xt_K0 = xt->K0; q.xt_N1 = xt->N1; q.xt_slab = xt->slab;
}

static int il_bwd_impl(void* stream, const float* x, const float* xsave, const float* dy,
                       int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                       const float* W, const float* bias, const float* gamma, const float* beta,
                       float eps, int use_res, float drop_rate, uint64_t seed, float* dx,
                       int dx_accumulate, float* dparams, int dparams_accumulate,
                       float* workspace, int64_t workspace_floats, const float* asave,
                       const XtArgs* xt = nullptr) {
  if (!x || !dy || !W || !bias || !gamma || !beta || !dx || !workspace) return RS_ERR_ARG;
  if (B < 0 || F <= 0 || L <= 0 || H <= 0 || U % H != 0 || (L > 1 && (E != U || !xsave)))
    return RS_ERR_ARG;
  if (drop_rate < 0.f || drop_rate >= 1.f || dy_ld < (int64_t)F * U) return RS_ERR_ARG;
  rs_il::BwdReq q{rs_stream(stream), x, xsave, dy, W, bias, gamma, beta, dy_ld, B, F, E, U, H, L,
                  use_res, eps, drop_rate, seed, dx, dx_accumulate, dparams, dparams_accumulate,
                  workspace, workspace_floats};
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  q.asave = asave;
  set_xt(q, xt);
  if (F > 64) return xt ? RS_ERR_UNSUPPORTED : bwd_large(q);
  return bwd_small(q);
}

RS_API int rs_il_bwd(void* stream, const float* x, const float* xsave, const float* dy,
                     int64_t dy_ld, int64_t B,
                     int F, int E, int U, int H, int L, const float* W, const float* bias,
                     const float* gamma, const float* beta, float eps, int use_res,
                     float drop_rate, uint64_t seed, float* dx, int dx_accumulate,
                     float* dparams, int dparams_accumulate, float* workspace,
                     int64_t workspace_floats) {
  return il_bwd_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta, eps,
                     use_res, drop_rate, seed, dx, dx_accumulate, dparams, dparams_accumulate,
                     workspace, workspace_floats, nullptr);
}

RS_API int rs_il_bwd_saved(void* stream, const float* x, const float* xsave, const float* dy,
                           int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                           const float* W, const float* bias, const float* gamma,
                           const float* beta, float eps, int use_res, float drop_rate,
                           uint64_t seed, float* dx, int dx_accumulate, float* dparams,
                           int dparams_accumulate, float* workspace, int64_t workspace_floats,
                           const float* asave, int64_t asave_floats) {
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need > 0 && (!asave || asave_floats < need)) return RS_ERR_ARG;
  return il_bwd_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta, eps,
                     use_res, drop_rate, seed, dx, dx_accumulate, dparams, dparams_accumulate,
                     workspace, workspace_floats, need > 0 ? asave : nullptr);
}

static int il_bwd_push_impl(void* stream, const float* x, const float* xsave, const float* dy,
                            int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                            const float* W, const float* bias, const float* gamma,
                            const float* beta, float eps, int use_res, float drop_rate,
                            uint64_t seed, const float* dx_base, const int32_t* rows,
                            float* grad_table, int32_t* flag, float* dparams,
                            int dparams_accumulate, float* workspace, int64_t workspace_floats,
                            const float* asave, const XtArgs* xt = nullptr) {
  if (!x || !dy || !W || !bias || !gamma || !beta || !rows || !grad_table || !flag || !workspace)
    return RS_ERR_ARG;
  if (B < 0 || F <= 0 || L <= 0 || H <= 0 || U % H != 0 || (L > 1 && (E != U || !xsave)))
    return RS_ERR_ARG;
  if (drop_rate < 0.f || drop_rate >= 1.f || dy_ld < (int64_t)F * U) return RS_ERR_ARG;
  rs_il::BwdReq q{rs_stream(stream), x, xsave, dy, W, bias, gamma, beta, dy_ld, B, F, E, U, H, L,
                  use_res, eps, drop_rate, seed, const_cast<float*>(dx_base), dx_base != nullptr,
                  dparams, dparams_accumulate, workspace, workspace_floats};
  q.push_rows = rows;
  q.push_table = grad_table;
  q.push_flag = flag;
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  q.asave = asave;
  set_xt(q, xt);
  // F > 64: only the generic kernel fuses the push (the many-field instantiations do not)
  return F > 64 ? rs_il::il_generic_bwd(q) : bwd_small(q);
}

RS_API int rs_il_bwd_push(void* stream, const float* x, const float* xsave, const float* dy,
                          int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                          const float* W, const float* bias, const float* gamma,
                          const float* beta, float eps, int use_res, float drop_rate,
                          uint64_t seed, const float* dx_base, const int32_t* rows,
                          float* grad_table, int32_t* flag, float* dparams,
                          int dparams_accumulate, float* workspace, int64_t workspace_floats) {
  return il_bwd_push_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta,
                          eps, use_res, drop_rate, seed, dx_base, rows, grad_table, flag, dparams,
                          dparams_accumulate, workspace, workspace_floats, nullptr);
}

RS_API int rs_il_bwd_push_saved(void* stream, const float* x, const float* xsave, const float* dy,
                                int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                                const float* W, const float* bias, const float* gamma,
                                const float* beta, float eps, int use_res, float drop_rate,
                                uint64_t seed, const float* dx_base, const int32_t* rows,
                                float* grad_table, int32_t* flag, float* dparams,
                                int dparams_accumulate, float* workspace,
                                int64_t workspace_floats, const float* asave,
                                int64_t asave_floats) {
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need > 0 && (!asave || asave_floats < need)) return RS_ERR_ARG;
  return il_bwd_push_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta,
                          eps, use_res, drop_rate, seed, dx_base, rows, grad_table, flag, dparams,
                          dparams_accumulate, workspace, workspace_floats,
                          need > 0 ? asave : nullptr);
}

RS_API int rs_il_xt_splits(int64_t B) { return rs_il::xt_splits(B); }

static bool xt_ok(const XtArgs& t) {
  return t.x && t.dz && t.slab && t.K0 > 0 && t.K0 % 16 == 0 && t.N1 > 0 && t.N1 % 16 == 0 &&
         t.ldx >= t.K0 && t.lddz >= t.N1;
}

RS_API int rs_il_bwd_saved_xt(void* stream, const float* x, const float* xsave, const float* dy,
                              int64_t dy_ld, int64_t B, int F, int E, int U, int H, int L,
                              const float* W, const float* bias, const float* gamma,
                              const float* beta, float eps, int use_res, float drop_rate,
                              uint64_t seed, float* dx, int dx_accumulate, float* dparams,
                              int dparams_accumulate, float* workspace, int64_t workspace_floats,
                              const float* asave, int64_t asave_floats, const float* xt_x,
                              int64_t xt_ldx, const float* xt_dz, int64_t xt_lddz, int xt_K0,
                              int xt_N1, float* xt_slab) {
  const XtArgs xt{xt_x, xt_ldx, xt_dz, xt_lddz, xt_K0, xt_N1, xt_slab};
  if (!xt_ok(xt)) return RS_ERR_ARG;
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need <= 0 || !asave || asave_floats < need) return need <= 0 ? RS_ERR_UNSUPPORTED : RS_ERR_ARG;
  return il_bwd_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta, eps,
                     use_res, drop_rate, seed, dx, dx_accumulate, dparams, dparams_accumulate,
                     workspace, workspace_floats, asave, &xt);
}

RS_API int rs_il_bwd_push_saved_xt(void* stream, const float* x, const float* xsave,
                                   const float* dy, int64_t dy_ld, int64_t B, int F, int E, int U,
                                   int H, int L, const float* W, const float* bias,
                                   const float* gamma, const float* beta, float eps, int use_res,
                                   float drop_rate, uint64_t seed, const float* dx_base,
                                   const int32_t* rows, float* grad_table, int32_t* flag,
                                   float* dparams, int dparams_accumulate, float* workspace,
                                   int64_t workspace_floats, const float* asave,
                                   int64_t asave_floats, const float* xt_x, int64_t xt_ldx,
                                   const float* xt_dz, int64_t xt_lddz, int xt_K0, int xt_N1,
                                   float* xt_slab) {
  const XtArgs xt{xt_x, xt_ldx, xt_dz, xt_lddz, xt_K0, xt_N1, xt_slab};
  if (!xt_ok(xt)) return RS_ERR_ARG;
  const int64_t need = rs_il_attn_save_floats(B, F, U, H, L);
  if (need <= 0 || !asave || asave_floats < need) return need <= 0 ? RS_ERR_UNSUPPORTED : RS_ERR_ARG;
  return il_bwd_push_impl(stream, x, xsave, dy, dy_ld, B, F, E, U, H, L, W, bias, gamma, beta,
                          eps, use_res, drop_rate, seed, dx_base, rows, grad_table, flag, dparams,
                          dparams_accumulate, workspace, workspace_floats, asave, &xt);
}

static int il_partial_blocks(int64_t B, int F, int E, int U, int H, int64_t workspace_floats,
                             bool saved) {
  // the kernels pick a variant per shape: ask the dispatch (dry run, nothing launched).
  // Pointers only need the alignment the real call has (the fused trainer's dy is 16-B aligned);
  // saved: the entry points that read the forward's attention save (another kernel pair for the
  // shapes that have one)
  static const float kDummy[4] __attribute__((aligned(16))) = {0.f, 0.f, 0.f, 0.f};
  int grid = 0;
  rs_il::BwdReq q{nullptr, kDummy, kDummy, kDummy, kDummy, kDummy, kDummy, kDummy,
                  (int64_t)F * U, B, F, E, U, H, 1, 1, 1e-14f, 0.f, 0, nullptr, 0, nullptr, 0,
                  nullptr, workspace_floats};
  q.grid_out = &grid;
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  if (saved && rs_il_attn_save_floats(B < 1 ? 1 : B, F, U, H, 1) > 0) q.asave = kDummy;
  if ((F > 64 ? bwd_large(q) : bwd_small(q)) != RS_OK) return 0;
  return grid < 0 ? 0 : grid;
}

RS_API int rs_il_bwd_partial_blocks(int64_t B, int F, int E, int U, int H,
                                    int64_t workspace_floats) {
  return il_partial_blocks(B, F, E, U, H, workspace_floats, false);
}

RS_API int rs_il_bwd_saved_partial_blocks(int64_t B, int F, int E, int U, int H,
                                          int64_t workspace_floats) {
  return il_partial_blocks(B, F, E, U, H, workspace_floats, true);
}

// whether the saved backward of this shape can carry a deferred weight gradient
// (rs_il_bwd_saved_xt / rs_il_bwd_push_saved_xt): its grid, or 0
RS_API int rs_il_bwd_xt_supported(int64_t B, int F, int E, int U, int H, int64_t workspace_floats) {
  if (F > 64 || rs_il_attn_save_floats(B < 1 ? 1 : B, F, U, H, 1) <= 0) return 0;
  static const float kDummy[16] __attribute__((aligned(16))) = {};
  int grid = 0;
  rs_il::BwdReq q{nullptr, kDummy, kDummy, kDummy, kDummy, kDummy, kDummy, kDummy,
                  (int64_t)F * U, B, F, E, U, H, 1, 1, 1e-14f, 0.f, 0, nullptr, 0, nullptr, 0,
                  nullptr, workspace_floats};
  q.grid_out = &grid;
  q.bf16 = rs_math_mode_now() == RS_MATH_BF16;
  q.asave = kDummy;
  q.xt_x = kDummy; q.xt_dz = kDummy; q.xt_ldx = 16; q.xt_lddz = 16; q.xt_K0 = 16; q.xt_N1 = 16;
  q.xt_slab = const_cast<float*>(kDummy);
  if (bwd_small(q) != RS_OK) return 0;
  return grid;
}
