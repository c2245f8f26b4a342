// mlp16w_fwd.hip -- k_mlp_fwd16w (mlp16w.h), the f16x3 forward in 16-point waves, and its launcher.
#include "mlp16w.h"

namespace pnr {

template <int SV>
static int launch16w_sv(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a) {
  auto kern = k_mlp_fwd16w<SV>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               W16Geo::kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, grid, dim3(512), W16Geo::kLds, st, a, mode);
  return hip_status(hipGetLastError());
}

int launch_fwd16w(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, int save) {
  switch (save) {
    case 0: return launch16w_sv<0>(mode, grid, st, a);
    case 1: return launch16w_sv<1>(mode, grid, st, a);
    default: return launch16w_sv<2>(mode, grid, st, a);
  }
}

}  // namespace pnr
