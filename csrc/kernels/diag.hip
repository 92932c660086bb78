// Diagnostics kernels (not on any training path).
//
// comm_emulator: stands in for an RCCL collective that shares the GPU with the backward
// pass.  RCCL's generic kernel (librccl gfx950 code object metadata: 37,664 B of LDS, up to
// 512 threads, 248-256 VGPRs per wave) occupies `blocks` CUs for the duration of a
// collective; the persistent conv kernels (146-150 KB of LDS per block) cannot share a CU
// with it.  bench.py --emulate-comm launches this on a side stream when the classifier's
// gradient lands - the moment the data-parallel bucketer starts its first all-reduce - so
// the single-GPU step shows what overlapping comm costs the compute kernels.
#include "common.h"
#include "api.h"

namespace mpa {

__global__ __launch_bounds__(512) void comm_emulator_kernel(float* __restrict__ sink,
                                                            long long cycles) {
  extern __shared__ float buf[];
  buf[threadIdx.x] = (float)threadIdx.x;  // touch the LDS allocation
  __syncthreads();
  const long long t0 = wall_clock64();
  float acc = buf[(threadIdx.x + 1) % blockDim.x];
  while (wall_clock64() - t0 < cycles) acc = acc * 0.999f + 1.f;
  if (acc == -1.f) sink[blockIdx.x] = acc;  // never true; keeps the loop
}

void comm_emulator(int blocks, int threads, int lds_bytes, double us, float* sink, hipStream_t s) {
  int dev = 0, khz = 100000;  // wall_clock64 ticks at the device's fixed reference clock
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
  const long long cycles = (long long)(us * 1e-3 * khz);
  hipLaunchKernelGGL(comm_emulator_kernel, dim3(blocks), dim3(threads), (size_t)lds_bytes, s,
                     sink, cycles);
}

// atomic_latency: `iters` dependent device-scope atomicAdds (or, mode 3, dependent loads) by
// thread 0 of each of `blocks` blocks; the kernel time / iters is the round trip the
// persistent kernels' work-queue tickets must hide.  mode 0: one counter for all blocks,
// 1: one per XCD (block % 8), 2: one per block, 3: loads of a per-block word.
__global__ void atomic_latency_kernel(int* q, int iters, int mode) {
  if (threadIdx.x != 0) return;
  const int b = blockIdx.x;
  int* c = q + (mode == 0 ? 0 : mode == 1 ? (b & 7) * 32 : b * 32);
  int r = 0;
  if (mode == 3) {
    for (int i = 0; i < iters; ++i) r += __atomic_load_n(c + (r >> 30), __ATOMIC_RELAXED) & 1;
  } else {
    for (int i = 0; i < iters; ++i) r = atomicAdd(c + (r >> 30), 1);
  }
  if (r == -7) q[1 << 20] = r;  // never true: keeps the chain
}

void atomic_latency(int blocks, int iters, int mode, int* q, hipStream_t s) {
  hipLaunchKernelGGL(atomic_latency_kernel, dim3(blocks), dim3(64), 0, s, q, iters, mode);
}

}  // namespace mpa
