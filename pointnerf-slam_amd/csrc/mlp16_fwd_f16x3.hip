// mlp16_fwd_f16x3.hip -- k_mlp_fwd16 instantiated for PNR_PREC_F16X3 (own translation unit: the
// fully unrolled kernels compile in parallel).
#include "mlp16.h"

namespace pnr {
#if defined(PNR_EXP_TIMELINE)
__device__ unsigned long long g_pnr_dbg[4][48];
extern "C" int pnr_dbg_read(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pnr_dbg), sizeof(g_pnr_dbg), 0, hipMemcpyDeviceToHost);
}
#endif
int launch_fwd16_f16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save) {
  return launch16<PNR_PREC_F16X3>(mode, grid, st, a, hasc, save);
}
}  // namespace pnr
