// mlp16_fwd_bf16x3.hip -- k_mlp_fwd16 instantiated for PNR_PREC_BF16X3 (own translation unit: the
// fully unrolled kernels compile in parallel).
#include "mlp16.h"

namespace pnr {
int launch_fwd16_bf16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save) {
  return launch16<PNR_PREC_BF16X3>(mode, grid, st, a, hasc, save);
}
}  // namespace pnr
