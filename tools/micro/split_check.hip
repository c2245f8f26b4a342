// Check: the packed f16 hi/lo split (v_cvt_pk_f16_f32 + v_fma_mixlo/mixhi_f16, dev_common.h split2)
// against the scalar form the kernels used before (hi = f16(x), lo = f16(x - float(hi))), bit for bit,
// over values spanning the f16 range and its subnormals, signed zeros, the overflow edge, inf, NaN.
//   hipcc --offload-arch=gfx950 -O3 -I pointnerf-slam_amd/csrc tools/micro/split_check.hip -o /tmp/split_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include "dev_common.h"

__global__ void k(const float* x, uint32_t* hi_a, uint32_t* lo_a, uint32_t* hi_b, uint32_t* lo_b, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const float x0 = x[2 * i], x1 = x[2 * i + 1];
  uint32_t h, l;
  pnr::split2(x0, x1, h, l);
  hi_a[i] = h;
  lo_a[i] = l;
  const _Float16 h0 = (_Float16)x0, h1 = (_Float16)x1;
  const _Float16 l0 = (_Float16)(x0 - (float)h0), l1 = (_Float16)(x1 - (float)h1);
  hi_b[i] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
  lo_b[i] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
}

int main() {
  const int n = 1 << 22;
  float* hx = new float[n];
  uint64_t s = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;
    const int e = (int)((s >> 3) % 60) - 40;            // 2^-40 .. 2^19
    float v = (float)((1.0 + u) * std::ldexp(1.0, e));
    if (s & 1) v = -v;
    hx[i] = v;
  }
  const float specials[] = {0.f, -0.f, 65504.f, 65519.f, 65520.f, -65520.f, 1e-8f, 6.1e-5f, 5.96e-8f,
                            INFINITY, -INFINITY, NAN, 1.0f + 1.0f / 4096, 2049.f, 3.0e-5f, 1.0e30f};
  for (int i = 0; i < (int)(sizeof(specials) / 4); ++i) hx[i] = specials[i];
  float* dx;
  uint32_t *ha, *la, *hb, *lb;
  hipMalloc(&dx, n * 4);
  hipMalloc(&ha, n * 2); hipMalloc(&la, n * 2); hipMalloc(&hb, n * 2); hipMalloc(&lb, n * 2);
  hipMemcpy(dx, hx, n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 2 / 256), dim3(256), 0, 0, dx, ha, la, hb, lb, n);
  uint32_t *a = new uint32_t[n / 2], *b = new uint32_t[n / 2], *c = new uint32_t[n / 2], *d = new uint32_t[n / 2];
  hipMemcpy(a, ha, n * 2, hipMemcpyDeviceToHost); hipMemcpy(b, la, n * 2, hipMemcpyDeviceToHost);
  hipMemcpy(c, hb, n * 2, hipMemcpyDeviceToHost); hipMemcpy(d, lb, n * 2, hipMemcpyDeviceToHost);
  long bad_hi = 0, bad_lo = 0, bad_lo_nan = 0;
  for (int i = 0; i < n / 2; ++i) {
    bad_hi += a[i] != c[i];
    if (b[i] != d[i]) {
      // both NaN (any payload) counts as equal
      const bool nan_a = ((b[i] & 0x7c00) == 0x7c00 && (b[i] & 0x3ff)) || ((b[i] & 0x7c000000) == 0x7c000000 && (b[i] & 0x3ff0000));
      if (nan_a) ++bad_lo_nan; else ++bad_lo;
      if (bad_lo < 5 && !nan_a) printf("lo mismatch x=(%g, %g) new %08x old %08x\n", hx[2 * i], hx[2 * i + 1], b[i], d[i]);
    }
  }
  printf("pairs %d: hi mismatches %ld, lo mismatches %ld (NaN-payload only: %ld)\n", n / 2, bad_hi, bad_lo, bad_lo_nan);
  printf(bad_hi == 0 && bad_lo == 0 ? "SPLIT_OK\n" : "SPLIT_MISMATCH\n");
  return 0;
}
