// InteractingLayer instantiations: other 16-wide shapes (head counts 1 and 4, unit_num 8/32 on
// 16-dim embeddings; layer_num > 1 needs E == U).
#include "il_kernels.hpp"
namespace rs_il {
RS_IL_DECLARE_UNIT(il_unit_b)
template <int E, int U, int H>
static int fwd32(const FwdReq& q) { return q.F <= 32 ? try_fwd<E, U, H, 32>(q) : try_fwd<E, U, H, 64>(q); }
template <int E, int U, int H>
static int bwd32(const BwdReq& q) { return q.F <= 32 ? try_bwd<E, U, H, 32>(q) : try_bwd<E, U, H, 64>(q); }
int il_unit_b_fwd(const FwdReq& q) {
#ifdef RS_MIN_BUILD
  return RS_ERR_UNSUPPORTED;
#endif
  if (q.E == 16 && q.U == 16 && q.H == 1) return fwd32<16, 16, 1>(q);
  if (q.E == 16 && q.U == 16 && q.H == 4) return fwd32<16, 16, 4>(q);
  if (q.E == 16 && q.U == 8 && q.H == 2) return fwd32<16, 8, 2>(q);
  if (q.E == 16 && q.U == 32 && q.H == 2) return fwd32<16, 32, 2>(q);
  // (the constructor defaults, unit_num 128 / head_num 1, run il_generic.hip both ways: its
  // forward took 590 vs 972 us for this one-wave instantiation at B = 2048, F = 26)
  return RS_ERR_UNSUPPORTED;
}
int il_unit_b_bwd(const BwdReq& q) {
#ifdef RS_MIN_BUILD
  return RS_ERR_UNSUPPORTED;
#endif
  if (q.E == 16 && q.U == 16 && q.H == 1) return bwd32<16, 16, 1>(q);
  if (q.E == 16 && q.U == 16 && q.H == 4) return bwd32<16, 16, 4>(q);
  if (q.E == 16 && q.U == 8 && q.H == 2) return bwd32<16, 8, 2>(q);
  if (q.E == 16 && q.U == 32 && q.H == 2) return bwd32<16, 32, 2>(q);
  return RS_ERR_UNSUPPORTED;
}
}  // namespace rs_il
