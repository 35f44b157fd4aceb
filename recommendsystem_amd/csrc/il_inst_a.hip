// InteractingLayer instantiations: the AutoInt CTR shape (E = U = 16, H = 2),
// backward kernels (the forward kernels are il_inst_a_fwd.hip, built without SLP vectorization).
// FMAX = 26 is the Criteo field count (no padded keys); 32 and 64 cover other field counts.
// F <= 32 also has the bf16-math-mode kernels (config 2's bf16 mode, BASELINE.json configs[1]).
#include "il_kernels.hpp"
namespace rs_il {
RS_IL_DECLARE_UNIT(il_unit_a)
int il_unit_a_bwd(const BwdReq& q) {
  if (q.F == 26) return try_bwd<16, 16, 2, 26, true, true>(q);
#ifndef RS_MIN_BUILD
  if (q.F <= 32) return try_bwd<16, 16, 2, 32, false, true>(q);
  return try_bwd<16, 16, 2, 64>(q);
#endif
  return RS_ERR_UNSUPPORTED;
}
}  // namespace rs_il
