// Image preprocessing (K15) and dropout (K14).
//
// preprocess: uint8 HWC images -> resize -> (x/255 - mean)/std -> bf16 NHWC with the
// channel dim optionally zero-padded (so the stem conv can take 16-B channel vectors).
//   mode 0: bilinear, align_corners=False, no antialias - the train transform
//           ToTensor -> Resize(tensor) -> Normalize of main.py:62-65 (torchvision 0.9.1
//           resizes tensors with F.interpolate bilinear, antialias off);
//   mode 1: bicubic (a = -0.5) with antialias, separable PIL-style support scaling - the
//           eval path's PIL Image.resize default (evaluation_pipeline.py:89).
// Replaces three pipeline ranks of the reference (read/resize/normalize) with one kernel.
//
// dropout: counter-based hash RNG (seed, call offset, element index) -> keep mask (uint8),
// inverted scaling; deterministic per (seed, offset) and graph-replay safe.
#include "common.h"
#include "api.h"
#include <algorithm>

namespace mpa {

__device__ __forceinline__ float cubic_w(float x) {
  const float a = -0.5f;
  x = fabsf(x);
  if (x < 1.f) return ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
  if (x < 2.f) return (((x - 5.f) * x + 8.f) * x - 4.f) * a;
  return 0.f;
}

// One output pixel: 3 normalized channels + zero channels up to cpad, one 8-B store for
// the 4-channel pixel-pair stem layout, one 16-B store for 8 channels.
__device__ __forceinline__ void store_px(bf16_t* o, float c0, float c1, float c2, int cpad) {
  const uint32_t lo = (uint32_t)f2bf(c0) | ((uint32_t)f2bf(c1) << 16);
  const uint32_t hi = (uint32_t)f2bf(c2);
  if (cpad == 4) {
    *(uint2*)o = make_uint2(lo, hi);
  } else if (cpad == 8) {
    *(uint4*)o = make_uint4(lo, hi, 0u, 0u);
  } else {
    o[0] = (bf16_t)(lo & 0xffff); o[1] = (bf16_t)(lo >> 16); o[2] = (bf16_t)hi;
    for (int ch = 3; ch < cpad; ++ch) o[ch] = 0;
  }
}

// Output geometry: the resized image sits at (pad.top, pad.left) of a zero-bordered
// [OH + top + bottom][OW + left + right] canvas (the pre-padded input of a pixel-pair
// stem conv, models/layers.py); a thread per canvas pixel, border pixels write zeros.
__device__ __forceinline__ bool canvas_px(int64_t t, const OutPad& pd, int OH, int OW, int& b,
                                          int& oy, int& ox) {
  const int owp = OW + pd.left + pd.right, ohp = OH + pd.top + pd.bottom;
  const int px = (int)(t % owp);
  const int64_t r = t / owp;
  const int py = (int)(r % ohp);
  b = (int)(r / ohp);
  oy = py - pd.top;
  ox = px - pd.left;
  return (unsigned)oy < (unsigned)OH && (unsigned)ox < (unsigned)OW;
}

__global__ __launch_bounds__(256) void preprocess_bilinear_kernel(
    const uint8_t* __restrict__ img, int B, int H, int W, int OH, int OW,
    Norm3 nrm, int cpad, OutPad pd, bf16_t* __restrict__ out) {
  const float* mean = nrm.mean;
  const float* stdv = nrm.std;
  const int64_t total = (int64_t)B * (OH + pd.top + pd.bottom) * (OW + pd.left + pd.right);
  const float sh = (float)H / OH, sw = (float)W / OW;
  const float m0 = mean[0], m1 = mean[1], m2 = mean[2];
  const float i0 = 1.f / (255.f * stdv[0]), i1 = 1.f / (255.f * stdv[1]), i2 = 1.f / (255.f * stdv[2]);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int b, oy, ox;
    if (!canvas_px(t, pd, OH, OW, b, oy, ox)) {
      store_px(out + t * cpad, 0.f, 0.f, 0.f, cpad);
      continue;
    }
    float sy = fmaxf((oy + 0.5f) * sh - 0.5f, 0.f);
    float sx = fmaxf((ox + 0.5f) * sw - 0.5f, 0.f);
    int y0 = min((int)sy, H - 1), x0 = min((int)sx, W - 1);
    const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
    const float ly = sy - y0, lx = sx - x0;
    const uint8_t* base = img + (size_t)b * H * W * 3;
    float c[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const float v00 = base[((size_t)y0 * W + x0) * 3 + ch];
      const float v01 = base[((size_t)y0 * W + x1) * 3 + ch];
      const float v10 = base[((size_t)y1 * W + x0) * 3 + ch];
      const float v11 = base[((size_t)y1 * W + x1) * 3 + ch];
      c[ch] = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
    }
    store_px(out + t * cpad, c[0] * i0 - m0 / stdv[0], c[1] * i1 - m1 / stdv[1],
             c[2] * i2 - m2 / stdv[2], cpad);
  }
}

// antialiased bicubic: separable weights computed on the fly (support scales with the
// downsampling factor, PIL/torch "aa" semantics)
__device__ __forceinline__ void aa_window(int i, int in, int out, int& xmin, int& xsize,
                                          float& center, float& invscale, float& support) {
  const float scale = (float)in / out;
  support = (scale >= 1.f) ? 2.f * scale : 2.f;
  invscale = (scale >= 1.f) ? 1.f / scale : 1.f;
  center = scale * (i + 0.5f);
  xmin = max((int)(center - support + 0.5f), 0);
  xsize = min((int)(center + support + 0.5f), in) - xmin;
}

__global__ __launch_bounds__(256) void preprocess_bicubic_aa_kernel(
    const uint8_t* __restrict__ img, int B, int H, int W, int OH, int OW,
    Norm3 nrm, int cpad, OutPad pd, bf16_t* __restrict__ out) {
  const float* mean = nrm.mean;
  const float* stdv = nrm.std;
  const int64_t total = (int64_t)B * (OH + pd.top + pd.bottom) * (OW + pd.left + pd.right);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int b, oy, ox;
    if (!canvas_px(t, pd, OH, OW, b, oy, ox)) {
      store_px(out + t * cpad, 0.f, 0.f, 0.f, cpad);
      continue;
    }
    int ymin, ysize, xmin, xsize;
    float cy, isy, suy, cx, isx, sux;
    aa_window(oy, H, OH, ymin, ysize, cy, isy, suy);
    aa_window(ox, W, OW, xmin, xsize, cx, isx, sux);
    float wsy = 0.f, wsx = 0.f;
    for (int j = 0; j < ysize; ++j) wsy += cubic_w((j + ymin - cy + 0.5f) * isy);
    for (int j = 0; j < xsize; ++j) wsx += cubic_w((j + xmin - cx + 0.5f) * isx);
    const float ny = wsy != 0.f ? 1.f / wsy : 0.f, nx = wsx != 0.f ? 1.f / wsx : 0.f;
    const uint8_t* base = img + (size_t)b * H * W * 3;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int j = 0; j < ysize; ++j) {
      const float wy = cubic_w((j + ymin - cy + 0.5f) * isy) * ny;
      float row[3] = {0.f, 0.f, 0.f};
      const uint8_t* rp = base + (size_t)(ymin + j) * W * 3;
      for (int k = 0; k < xsize; ++k) {
        const float wx = cubic_w((k + xmin - cx + 0.5f) * isx) * nx;
        const uint8_t* px = rp + (size_t)(xmin + k) * 3;
        row[0] += wx * px[0];
        row[1] += wx * px[1];
        row[2] += wx * px[2];
      }
      acc[0] += wy * row[0];
      acc[1] += wy * row[1];
      acc[2] += wy * row[2];
    }
    store_px(out + t * cpad, (acc[0] / 255.f - mean[0]) / stdv[0],
             (acc[1] / 255.f - mean[1]) / stdv[1], (acc[2] / 255.f - mean[2]) / stdv[2], cpad);
  }
}

__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // murmur3-style finalizer over a mixed triple
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ c * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x85EBCA6Bu;
  h ^= h >> 13; h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

__global__ void dropout_fwd_kernel(const bf16_t* __restrict__ x, int64_t n, float p, uint32_t seed,
                                   uint32_t offset, bf16_t* __restrict__ y,
                                   uint8_t* __restrict__ mask) {
  const float scale = 1.f / (1.f - p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hash3(seed, offset, (uint32_t)i);
    const float u = (h >> 8) * (1.f / 16777216.f);
    const bool keep = u >= p;
    mask[i] = keep ? 1 : 0;
    y[i] = keep ? f2bf(bf2f(x[i]) * scale) : (bf16_t)0;
  }
}

__global__ void dropout_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                                   int64_t n, float p, bf16_t* __restrict__ dx) {
  const float scale = 1.f / (1.f - p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = mask[i] ? f2bf(bf2f(dy[i]) * scale) : (bf16_t)0;
}

static int blocks_n(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

void preprocess(const uint8_t* img, int B, int H, int W, int OH, int OW, Norm3 nrm, int mode,
                int cpad, OutPad pd, bf16_raw* out, hipStream_t s) {
  const int64_t total = (int64_t)B * (OH + pd.top + pd.bottom) * (OW + pd.left + pd.right);
  if (mode == 0)
    hipLaunchKernelGGL(preprocess_bilinear_kernel, dim3(blocks_n(total)), dim3(256), 0, s, img, B,
                       H, W, OH, OW, nrm, cpad, pd, out);
  else
    hipLaunchKernelGGL(preprocess_bicubic_aa_kernel, dim3(blocks_n(total)), dim3(256), 0, s, img,
                       B, H, W, OH, OW, nrm, cpad, pd, out);
}

void dropout_fwd(const bf16_raw* x, int64_t n, float p, uint64_t seed, uint64_t offset,
                 bf16_raw* y, uint8_t* mask, hipStream_t s) {
  hipLaunchKernelGGL(dropout_fwd_kernel, dim3(blocks_n(n)), dim3(256), 0, s, x, n, p,
                     (uint32_t)seed, (uint32_t)offset, y, mask);
}

void dropout_bwd(const bf16_raw* dy, const uint8_t* mask, int64_t n, float p, bf16_raw* dx,
                 hipStream_t s) {
  hipLaunchKernelGGL(dropout_bwd_kernel, dim3(blocks_n(n)), dim3(256), 0, s, dy, mask, n, p, dx);
}

}  // namespace mpa
