// InteractingLayer FORWARD instantiations of the AutoInt CTR shape (E = U = 16, H = 2; SURVEY §8
// config 2).  A unit of its own because build.py compiles it with -fno-slp-vectorize: the forward's
// scalar score dots / PV axpys, re-packed into v_pk_fma_f32 by the SLP vectorizer, cost 128 VGPRs
// plus scratch spills at 4 waves per SIMD; scalar they take 118 VGPRs, no spills (same-box
// tools/il_bench.py: fwd_saved 37.1 -> 34.6 us).  The backward keeps its explicit packed FMAs
// (il_inst_a.hip; without SLP there it measured 76.9 -> 78.2 us).
#include "il_kernels.hpp"
namespace rs_il {
RS_IL_DECLARE_UNIT(il_unit_a)
int il_unit_a_fwd(const FwdReq& q) {
  if (q.F == 26) return try_fwd<16, 16, 2, 26, true, true>(q);
#ifndef RS_MIN_BUILD
  if (q.F <= 32) return try_fwd<16, 16, 2, 32, false, true>(q);
  return try_fwd<16, 16, 2, 64>(q);
#endif
  return RS_ERR_UNSUPPORTED;
}
}  // namespace rs_il
