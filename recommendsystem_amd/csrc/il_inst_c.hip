// InteractingLayer instantiations: 8-wide (rank/multi_head IL(1, 8, 2), rank/ctr/model_init.py:54)
// and 32-wide embeddings.
#include "il_kernels.hpp"
namespace rs_il {
RS_IL_DECLARE_UNIT(il_unit_c)
template <int E, int U, int H>
static int fwd32(const FwdReq& q) { return q.F <= 32 ? try_fwd<E, U, H, 32>(q) : try_fwd<E, U, H, 64>(q); }
template <int E, int U, int H>
static int bwd32(const BwdReq& q) { return q.F <= 32 ? try_bwd<E, U, H, 32>(q) : try_bwd<E, U, H, 64>(q); }
int il_unit_c_fwd(const FwdReq& q) {
#ifdef RS_MIN_BUILD
  return RS_ERR_UNSUPPORTED;
#endif
  if (q.E == 8 && q.U == 8 && q.H == 2) return fwd32<8, 8, 2>(q);
  if (q.E == 8 && q.U == 8 && q.H == 1) return fwd32<8, 8, 1>(q);
  if (q.E == 32 && q.U == 32 && q.H == 2) return fwd32<32, 32, 2>(q);
  if (q.E == 32 && q.U == 32 && q.H == 4) return fwd32<32, 32, 4>(q);
  return RS_ERR_UNSUPPORTED;
}
int il_unit_c_bwd(const BwdReq& q) {
#ifdef RS_MIN_BUILD
  return RS_ERR_UNSUPPORTED;
#endif
  if (q.E == 8 && q.U == 8 && q.H == 2) return bwd32<8, 8, 2>(q);
  if (q.E == 8 && q.U == 8 && q.H == 1) return bwd32<8, 8, 1>(q);
  if (q.E == 32 && q.U == 32 && q.H == 2) return bwd32<32, 32, 2>(q);
  if (q.E == 32 && q.U == 32 && q.H == 4) return bwd32<32, 32, 4>(q);
  return RS_ERR_UNSUPPORTED;
}
}  // namespace rs_il
