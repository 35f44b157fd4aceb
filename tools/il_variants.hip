// Diagnostic only (not part of librecsys_amd.so): the wide InteractingLayer kernels with phases
// dropped (il_wide.hpp SKIP bits), to time each phase by elimination (tools/il_variants.py).
// Built by tools/il_variants.py into _gpuvar/libilvar.so; outputs of SKIP != 0 are wrong.
#include "../recommendsystem_amd/csrc/il_kernels.hpp"
namespace rs_il {
int rs_il_variant_now() { return RS_IL_VARIANT_WIDE; }
}
const int64_t* rs_seed_offset_now() { return nullptr; }
int rs_math_mode_now() { return RS_MATH_F32; }
using namespace rs_il;
using C = Cfg<16, 16, 2, 26, true, false>;

template <int S>
static void fwd_v(hipStream_t st, const float* x, const float* W, const float* b, const float* g,
                  const float* be, float* y, float* xs, float* asave, int64_t B) {
  Args a = make_args<C>(B, 26, 3, 1, 1e-14f, 0.f, 0, false);
  a.osave = asave;
  const int64_t grid = B < kWideFwdGrid ? B : kWideFwdGrid;
  wfwd_kernel<C, false, S><<<(int)grid, kWideThreads, WideFwdLayout<C>().total * 4, st>>>(
      x, W, b, g, be, y, 26 * 16, xs, a);
}
template <int S>
static void bwd_v(hipStream_t st, const float* x, const float* xs, const float* dy, const float* W,
                  const float* b, const float* g, const float* be, float* dx, float* ws,
                  const float* asave, int64_t B) {
  Args a = make_args2<C>(B, 26, 3, 1, 1e-14f, 0.f, 0);
  a.osave_in = asave;
  const int64_t grid = B < kWideBwdGrid ? B : kWideBwdGrid;
  wbwd_kernel<C, false, S><<<(int)grid, kWideThreads, wbwd_lds_bytes<C>(26), st>>>(
      x, xs, dy, 26 * 16, W, b, g, be, dx, 0, ws, a);
}

#define FV(S) case S: fwd_v<S>(st, x, W, b, g, be, y, xs, asave, B); break;
#define BV(S) case S: bwd_v<S>(st, x, xs, dy, W, b, g, be, dx, ws, asave, B); break;
extern "C" int ilvar_fwd(int skip, void* s, const float* x, const float* W, const float* b,
                         const float* g, const float* be, float* y, float* xs, float* asave,
                         int64_t B) {
  hipStream_t st = (hipStream_t)s;
  switch (skip) { FV(0) FV(1) FV(2) FV(4) FV(8) FV(3) FV(7) default: return -1; }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
extern "C" int ilvar_bwd(int skip, void* s, const float* x, const float* xs, const float* dy,
                         const float* W, const float* b, const float* g, const float* be, float* dx,
                         float* ws, const float* asave, int64_t B) {
  hipStream_t st = (hipStream_t)s;
  switch (skip) { BV(0) BV(1) BV(2) BV(4) BV(8) BV(12) BV(16) BV(32) BV(63) default: return -1; }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
