// mlp16_fwd_bf16.hip -- k_mlp_fwd16 instantiated for PNR_PREC_BF16 (own translation unit: the
// fully unrolled kernels compile in parallel).
#include "mlp16.h"

namespace pnr {
#if defined(PNR_EXP_TIMELINE)  // each TU's code object holds its own copy (no -fgpu-rdc)
__device__ unsigned long long g_pnr_dbg[4][48];
#endif
int launch_fwd16_bf16(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save) {
  return launch16<PNR_PREC_BF16>(mode, grid, st, a, hasc, save);
}
}  // namespace pnr
