// mlp16w_fwd.hip -- k_mlp_fwd16w (mlp16w.h), the f16x3 forward in 16-point waves, and its launcher.
#include <cstdlib>

#include "mlp16w.h"

namespace pnr {

template <int SV, int NW>
static int launch16w_sv(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, const MapRowsArgs& mr) {
  auto kern = k_mlp_fwd16w<SV, NW>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               W16Geo::kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, grid, dim3(64 * NW), W16Geo::kLds, st, a, mode, mr);
  return hip_status(hipGetLastError());
}

// Grid: one persistent workgroup per CU at most.  A batch whose 128-point tiles would fill at most half
// the CUs once (the Mapper's fine pass: 12,032 points = 94 tiles on 256 CUs) runs 64-point tiles of 4
// waves instead -- twice the workgroups, one 16-point wave per SIMD (PNR_W16_NW4=0: always 8 waves)
int launch_fwd16w(int mode, hipStream_t st, const BfFwdArgs& a, int save, const MapRowsArgs* mrp) {
  if ((mode == kMapRows) != (mrp != nullptr) || (mode == kMapRows && save != 1)) return PNR_E_ARG;
  static const MapRowsArgs kNone{};
  const MapRowsArgs& mr = mrp ? *mrp : kNone;
  static const bool nw4_ok = !(getenv("PNR_W16_NW4") && getenv("PNR_W16_NW4")[0] == '0');
  const int64_t ncu = device_cu_count();
  const int64_t t128 = (a.P + 127) / 128;
  if (nw4_ok && save != 2 && 2 * t128 <= ncu) {
    const dim3 grid((unsigned)((a.P + 63) / 64));
    return save == 0 ? launch16w_sv<0, 4>(mode, grid, st, a, mr) : launch16w_sv<1, 4>(mode, grid, st, a, mr);
  }
  const dim3 grid((unsigned)(t128 < ncu ? t128 : ncu));
  switch (save) {
    case 0: return launch16w_sv<0, 8>(mode, grid, st, a, mr);
    case 1: return launch16w_sv<1, 8>(mode, grid, st, a, mr);
    default: return launch16w_sv<2, 8>(mode, grid, st, a, mr);
  }
}

}  // namespace pnr
