// Microbenchmark: cycles per v_mfma_f32_32x32x16_f16 for the decoder's group pattern
// (8 accumulator tiles, each a dependent chain of 6 MFMAs per step), one wave per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma_chain.hip -o /tmp/mfma_chain && /tmp/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(const f16x8* in, float* out, unsigned long long* t) {
  __shared__ f16x8 lds[4096];
  for (int i = threadIdx.x; i < 4096; i += 256) lds[i] = in[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  f16x8 b0 = in[lane], b1 = in[lane + 64];
  f16x8 a[8];
  for (int i = 0; i < 8; ++i) a[i] = in[128 + 64 * i + lane];
  f32x16 acc[8];
  for (int i = 0; i < 8; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < 64; ++it) {
    if (MODE == 2) __syncthreads();
    if (MODE == 3) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int T = 0; T < 8; ++T) {
      f16x8 x = a[T], y = a[(T + 1) & 7];
      if (MODE >= 1) {  // operands from LDS like the decoder (4 frags per tile)
        x = lds[(T * 4 + 0) * 64 + lane];
        y = lds[(T * 4 + 1) * 64 + lane];
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(y, b0, acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, b1, acc[T], 0, 0, 0);
        acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, b0, acc[T], 0, 0, 0);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 7) t[MODE] = t1 - t0;
}

int main() {
  f16x8* in;
  float* out;
  unsigned long long* t;
  hipMalloc(&in, 8192 * 16);
  hipMemset(in, 0, 8192 * 16);
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&t, 64);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k<0>, dim3(1024), dim3(256), 0, 0, in, out, t);
    hipLaunchKernelGGL(k<1>, dim3(1024), dim3(256), 0, 0, in, out, t);
    hipLaunchKernelGGL(k<2>, dim3(1024), dim3(256), 0, 0, in, out, t);
    hipLaunchKernelGGL(k<3>, dim3(1024), dim3(256), 0, 0, in, out, t);
  }
  unsigned long long h[4];
  hipMemcpy(h, t, 32, hipMemcpyDeviceToHost);
  const double n = 64.0 * 48;
  printf("register operands: %.1f cycles/MFMA\nLDS operands:      %.1f cycles/MFMA\n", h[0] / n, h[1] / n);
  printf("+ __syncthreads per 48: %.1f\n+ s_barrier per 48:     %.1f\n", h[2] / n, h[3] / n);
  return 0;
}
