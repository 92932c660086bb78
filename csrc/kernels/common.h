// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels.
// Wave64 throughout; bf16 storage as raw 16-bit words; fp32 accumulation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

#define MPA_CHECK_LAUNCH() (void)hipGetLastError()

namespace mpa {

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even f32 -> bf16 (hipcc emits v_cvt_pk_bf16_f32 for the plain cast;
// NaN stays NaN, see MI355X_MICROARCH.md "Correctness boundaries")
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// Streaming 16-B accesses with the nontemporal hint (BN passes over tensors far larger than
// L2: every byte is touched once per pass)
__device__ __forceinline__ uint4 ld_stream(const void* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load((const v4u*)p);
  return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void st_stream(void* p, uint4 v) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, (v4u*)p);
}

__device__ __forceinline__ void unpack8(const uint4& v, float* f) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack2(f[0], f[1]);
  r.y = pack2(f[2], f[3]);
  r.z = pack2(f[4], f[5]);
  r.w = pack2(f[6], f[7]);
  return r;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that the dispatcher places on the same XCD (b % 8) get a
// contiguous range of tile ids, so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int x = b & 7, i = b >> 3;
  const int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

// Split-K rows GEMM launches (grid = tiles x 1 x splits) with a multiple of 8 splits place
// whole splits on one XCD: split z runs on XCD z % 8, so its k-slab of A and B
// comes from HBM once into that XCD's L2 and every tile of the split reuses it.  With
// xcd_remap's tile-contiguous placement each k-slab is fetched by every XCD that holds a
// tile of its row / column (the classifier dgrad, 4 x 4 tiles x 16 splits: 2-4x the HBM
// bytes; tools/bench_head.py: 74.5 -> 66 us).  Dispatch order is the flattened id
// L = x + gx * z, XCD = L % 8.  The mapping is a bijection of (x, z), so a wrong guess of
// the order costs locality, never correctness.  (The split-pixel weight-gradient kernels
// keep xcd_remap: there the step's autotuned plans came out mixed.)
__device__ __forceinline__ bool split_major() {
  return gridDim.z >= 8 && (gridDim.z & 7) == 0 && gridDim.y == 1;
}
__device__ __forceinline__ int block_split() {
  if (!split_major()) return blockIdx.z;
  const int L = blockIdx.x + gridDim.x * blockIdx.z;
  return (L & 7) + 8 * ((L >> 3) / gridDim.x);
}
__device__ __forceinline__ int block_tile(int tiles_total) {
  if (!split_major()) return xcd_remap(blockIdx.x, tiles_total);
  const int L = blockIdx.x + gridDim.x * blockIdx.z;
  return (L >> 3) % gridDim.x;
}

}  // namespace mpa
