// LDS-DMA staging-rate probe for the halo conv kernels (conv_halo.hip).
//
// Question: what limits the halo kernels' item rate (ResNet-18 layer1: 2.9 us per 37 KB
// item per CU, ~13 GB/s/CU, MFMA ~33 % busy)?  The probe runs the halo kernels' staging
// skeleton without the convolution: persistent blocks (one per CU), 4 producer waves
// issuing buffer_load ... lds into an S-stage ring, 4 consumer waves that pass one barrier
// per item and optionally burn a fixed number of MFMAs on registers (the compute an item
// carries), over a [pixels][64 ch] bf16 tensor the size of layer1's (411 MB at N = 1024).
//
//   mode 0 (chunk64): an item is PX pixels x one 64-B channel chunk (the halo kernels'
//                     layout: 16 pixels per 1-KiB wave-instruction, half of each 128-B line)
//   mode 1 (full128): an item is PX/2 pixels x both chunks (8 whole 128-B pixels per
//                     instruction): same bytes per item, half the lines
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/kernels tools/dma_probe.hip -o dma_probe
// Run:   ./dma_probe            (prints one line per configuration)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "igemm_common.h"

using namespace mpa;

template <int S, int MODE, int KB>
__global__ __launch_bounds__(512, 1) void probe_kernel(const char* x, uint32_t xbytes, int tiles,
                                                       int nmfma, float* sink) {
  constexpr int ITEM = KB * 1024;
  constexpr int IPW = KB / 4;  // 1-KiB DMA instructions per producer wave per item
  __shared__ __attribute__((aligned(16))) char smem[S * ITEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, G8 = gridDim.x >> 3;
  const int tbeg = (int)((int64_t)xcd * tiles / 8), tend = (int)((int64_t)(xcd + 1) * tiles / 8);
  const int ntiles = tbeg + loc < tend ? (tend - tbeg - loc + G8 - 1) / G8 : 0;
  const int nitems = ntiles * 2;  // two items per tile: channel chunks (mode 0) / halves (1)
  // pixels per item: mode 0 ITEM / 64 B, mode 1 ITEM / 128 B; a tile = 2 items
  constexpr int PXI = MODE == 0 ? ITEM / 64 : ITEM / 128;
  constexpr int PXT = MODE == 0 ? PXI : 2 * PXI;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(x, xbytes);
  const uint32_t s32 = lds_base(smem);
  auto src = [&](int k, int j) -> uint32_t {
    const int t = tbeg + loc + (k >> 1) * G8, half = k & 1;
    const int ins = (wave - 4) * IPW + j;  // instruction index within the item
    if (MODE == 0) {
      const uint32_t px = (uint32_t)t * PXT + ins * 16 + (lane >> 2);
      return px * 128u + half * 64 + (lane & 3) * 16;
    } else {
      const uint32_t px = (uint32_t)t * PXT + half * PXI + ins * 8 + (lane >> 3);
      return px * 128u + (lane & 7) * 16;
    }
  };
  auto issue = [&](int k) {
    const uint32_t st = s32 + (k % S) * ITEM;
#pragma unroll
    for (int j = 0; j < IPW; ++j) {
      uint32_t o = src(k, j);
      if (o >= xbytes) o = 0x80000000u;
      buf_lds16_at(r, st + ((wave - 4) * IPW + j) * 1024, o);
    }
  };
  if (wave >= 4) {  // producers
    for (int k = 0; k < S - 1 && k < nitems; ++k) issue(k);
    for (int k = 0; k < nitems; ++k) {
      // item k landed: at most (S - 2) younger items of this wave still in flight
      if constexpr (S == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (S == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(IPW) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * IPW) : "memory");
      __builtin_amdgcn_s_barrier();
      if (k + S - 1 < nitems) issue(k + S - 1);
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    return;
  }
  f32x4 acc[4] = {};
  bf16x8 a = {}, b = {};
  for (int k = 0; k < nitems; ++k) {
    __builtin_amdgcn_s_barrier();
    // touch the stage (one fragment read) and run the item's MFMAs (4 independent chains)
    a = *(const bf16x8*)(smem + (k % S) * ITEM + (tid & 255) * 16);
    for (int i = 0; i < nmfma; i += 4) {
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] = mfma16(a, b, acc[c]);
    }
  }
  if (acc[0][0] + acc[1][0] + acc[2][0] + acc[3][0] == 12345.f) sink[tid] = acc[0][1];
}

template <int S, int MODE, int KB>
static void run(const char* x, uint32_t bytes, int cus, int nmfma, float* sink) {
  const int item = KB * 1024;
  const int tiles = (int)(bytes / (2ull * item));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  probe_kernel<S, MODE, KB><<<cus, 512>>>(x, bytes, tiles, nmfma, sink);  // warm
  hipEventRecord(e0);
  const int reps = 5;
  for (int i = 0; i < reps; ++i) probe_kernel<S, MODE, KB><<<cus, 512>>>(x, bytes, tiles, nmfma, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double moved = 2.0 * tiles * item;
  const double items_per_cu = 2.0 * tiles / cus;
  printf("S=%d mode=%s item=%3d KB mfma/item/wave=%3d : %8.1f us  %6.2f TB/s  %6.1f GB/s/CU  %5.2f us/item\n",
         S, MODE ? "full128" : "chunk64", KB, nmfma, ms * 1e3, moved / (ms * 1e-3) / 1e12,
         moved / (ms * 1e-3) / cus / 1e9, ms * 1e3 / items_per_cu);
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) cus = prop.multiProcessorCount;
  const size_t bytes = (size_t)1024 * 56 * 56 * 64 * 2;  // layer1 activation, batch 1024
  char* x = nullptr;
  float* sink = nullptr;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&sink, 4096) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(x, 1, bytes);
  printf("# dma_probe: %d CUs, %.0f MB tensor\n", cus, bytes / 1e6);
  const uint32_t b32 = (uint32_t)bytes;
  for (int nm : {0, 144}) {
    run<2, 0, 36>(x, b32, cus, nm, sink);
    run<2, 1, 36>(x, b32, cus, nm, sink);
    run<3, 0, 36>(x, b32, cus, nm, sink);
    run<3, 1, 36>(x, b32, cus, nm, sink);
    run<4, 0, 36>(x, b32, cus, nm, sink);
    run<2, 0, 24>(x, b32, cus, nm, sink);
    run<3, 0, 24>(x, b32, cus, nm, sink);
    run<4, 0, 24>(x, b32, cus, nm, sink);
    run<2, 0, 48>(x, b32, cus, nm, sink);
    run<3, 0, 48>(x, b32, cus, nm, sink);
    run<3, 1, 48>(x, b32, cus, nm, sink);
  }
  hipError_t e = hipDeviceSynchronize();
  printf("# status %s\n", hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
