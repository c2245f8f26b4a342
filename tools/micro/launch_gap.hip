// launch_gap.hip -- where do the ~5 us boundaries of the room0 iteration come from?
// A HIP graph of back-to-back dependent launches of synthetic kernels that differ in ONE property each
// (block size, dynamic LDS, grid size, registers / scratch, bytes written), replayed many times; the
// boundaries are read from a rocprofv3 kernel trace (tools/micro/launch_gap.py).
//   hipcc -O3 --offload-arch=gfx950 tools/micro/launch_gap.hip -o /tmp/launch_gap
//   rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lgap -o g -- /tmp/launch_gap
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// small: 64 blocks x 256 threads, one store per thread
__global__ __launch_bounds__(256) void k_small(float* out) {
  out[blockIdx.x * 256 + threadIdx.x] += 1.f;
}
// big: 256 blocks x 512 threads; dynamic LDS of the launch (0 or 152 KiB) touched once; one store per thread
__global__ __launch_bounds__(512, 1) void k_big(float* out) {
  extern __shared__ float lds[];
  lds[threadIdx.x] = (float)threadIdx.x;
  __syncthreads();
  out[blockIdx.x * 512 + threadIdx.x] += lds[511 - threadIdx.x];
}
// big writer: the same grid, each thread writes 64 KiB / 512 ... = `n` floats (dirty lines at the end)
__global__ __launch_bounds__(512, 1) void k_big_write(float* out, int n) {
  float* o = out + (size_t)blockIdx.x * 512 * n;
  for (int i = 0; i < n; ++i) o[(size_t)i * 512 + threadIdx.x] = (float)i;
}
// big persistent-like: each block spins for ~`cyc` cycles (busy, no memory)
__global__ __launch_bounds__(512, 1) void k_big_spin(float* out, long cyc) {
  const long t0 = clock64();
  float a = 0.f;
  while (clock64() - t0 < cyc) a += 1.f;
  if (a < 0.f) out[threadIdx.x] = a;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 40;
  float* buf;
  const size_t nbuf = (size_t)256 * 512 * 1024;  // 512 MB of floats for the writer
  CK(hipMalloc(&buf, nbuf * sizeof(float)));
  CK(hipMemset(buf, 0, nbuf * sizeof(float)));
  const int kLds = 152 * 1024;
  CK(hipFuncSetAttribute((const void*)k_big, hipFuncAttributeMaxDynamicSharedMemorySize, kLds));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  // sequence (names in the trace tell the pairs apart):
  //   small small small | big(0 LDS) small | big(152K) small | small big(152K) | big(152K) big(152K)
  //   | big_write(32 MB) small | big_spin(20 us) small | big_spin big_spin
  auto body = [&]() {
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_big, dim3(256), dim3(512), 0, st, buf);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_big, dim3(256), dim3(512), kLds, st, buf);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_big, dim3(256), dim3(512), kLds, st, buf);
    hipLaunchKernelGGL(k_big, dim3(256), dim3(512), kLds, st, buf);
    hipLaunchKernelGGL(k_big_write, dim3(256), dim3(512), 0, st, buf, 64);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_big_spin, dim3(256), dim3(512), 0, st, buf, 48000L);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
    hipLaunchKernelGGL(k_big_spin, dim3(256), dim3(512), 0, st, buf, 48000L);
    hipLaunchKernelGGL(k_big_spin, dim3(256), dim3(512), 0, st, buf, 48000L);
    hipLaunchKernelGGL(k_small, dim3(64), dim3(256), 0, st, buf);
  };
  // eager once (warm-up), then the captured graph
  body();
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  body();
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  printf("launch_gap: %d replays done\n", reps);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(buf));
  return 0;
}
