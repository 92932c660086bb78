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
#include <cstdlib>

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
// stem conv, models/layers.py); border pixels are written as zeros.
//
// Bilinear (the training path, one launch per batch): a block owns PP_ROWS canvas rows of
// one image (a work item; blocks stride over the items).  Phase 1 stages the two source
// rows of every one of those rows' bilinear taps into LDS with independent 16-B (or dword,
// or byte) loads - one memory round trip per block; phase 2 has lane i compute canvas
// pixel i of each row from LDS and store 8 B (pixel-pair layout) or 16 B, consecutive
// lanes -> consecutive pixels.  (A pixel-per-thread grid-stride version with 64-bit index
// math and byte gathers from global memory streamed ~1.5 TB/s; a row-at-a-time LDS
// version was round-trip bound.)  The taps are LDS reads on purpose: a global (or flat)
// load after the previous pixel's store makes the in-order vmcnt wait for that store too,
// so every pixel paid a full store round trip.  Source rows wider than PP_MAXW pixels
// (STAGED = false) read their taps from global memory.
constexpr int PP_ROWS = 8;
constexpr int PP_MAXW = 1344;  // 2 x 8 staged rows x 1344 px x 3 B = 63 KiB of LDS

// VEC: staging load width (16, 4 or 1 bytes; alignment of the source rows); CPAD: 4 or 8
// output channels with one 8-B / 16-B store per pixel, 0 = any (scalar stores)
template <bool STAGED, int VEC, int CPAD>
__global__ __launch_bounds__(256) void preprocess_bilinear_kernel(
    const uint8_t* __restrict__ img, int B, int H, int W, int OH, int OW,
    Norm3 nrm, int cpad_rt, OutPad pd, bf16_t* __restrict__ out, const int* __restrict__ ext) {
  const int cpad = CPAD ? CPAD : cpad_rt;
  extern __shared__ __attribute__((aligned(16))) uint8_t srow[];  // [PP_ROWS][2][rb]
  const float* mean = nrm.mean;
  const float* stdv = nrm.std;
  const float i0 = 1.f / (255.f * stdv[0]), i1 = 1.f / (255.f * stdv[1]), i2 = 1.f / (255.f * stdv[2]);
  const float o0 = mean[0] / stdv[0], o1 = mean[1] / stdv[1], o2 = mean[2] / stdv[2];
  const int ohp = OH + pd.top + pd.bottom, owp = OW + pd.left + pd.right;
  const int ngroups = (ohp + PP_ROWS - 1) / PP_ROWS;  // row groups per image
  const int rb = W * 3;                     // source row bytes (the slot pitch)
  const int rbp = (rb + 15) & ~15;          // staged row pitch
  constexpr int vec = VEC;
  // work items (image, row group), strided over a grid of at most ~2k blocks: per-wave
  // start-up (kernel arguments, the normalisation divides) is paid once per block
  for (int item = blockIdx.x; item < B * ngroups; item += gridDim.x) {
    const int b = item / ngroups;
    const int row0 = (item - b * ngroups) * PP_ROWS;
    const int nrows = min(PP_ROWS, ohp - row0);
    const uint8_t* base = img + (size_t)b * H * W * 3;
    // this image's extent inside the [H][W] pitch (real images of different sizes share
    // one padded slot); the full pitch when ext is null
    const int ih = ext ? ext[2 * b] : H, iw = ext ? ext[2 * b + 1] : W;
    const float sh = (float)ih / OH, sw = (float)iw / OW;
    const int per = (iw * 3 + vec - 1) / vec;  // vectors per staged source row
    auto tap_rows = [&](int r, int& y0, int& y1, float& ly) {
      const int oy = row0 + r - pd.top;
      const float sy = fmaxf((oy + 0.5f) * sh - 0.5f, 0.f);
      y0 = min((int)sy, ih - 1);
      y1 = min(y0 + 1, ih - 1);
      ly = sy - y0;
    };
    if constexpr (STAGED) {  // phase 1: every (row, tap) source row; 4 loads in flight per
                             // thread before any LDS write (one round trip per batch)
      __syncthreads();       // the previous item's readers are done with srow
      const int total = nrows * 2 * per;
      for (int j0 = threadIdx.x; j0 < total; j0 += 4 * blockDim.x) {
        uint4 v[4];
        int dsto[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int i = j0 + k * blockDim.x;
          dsto[k] = -1;
          if (i >= total) continue;
          const int rt = i / per, e = i - rt * per;  // rt = 2 * row + tap
          const int oy = row0 + (rt >> 1) - pd.top;
          if ((unsigned)oy >= (unsigned)OH) continue;  // border row: nothing to stage
          int y0, y1;
          float ly;
          tap_rows(rt >> 1, y0, y1, ly);
          const uint8_t* src = base + (size_t)((rt & 1) ? y1 : y0) * rb;
          dsto[k] = rt * rbp + e * vec;
          if constexpr (vec == 16) v[k] = ((const uint4*)src)[e];
          else if constexpr (vec == 4) v[k].x = ((const uint32_t*)src)[e];
          else v[k].x = src[e];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (dsto[k] < 0) continue;
          if constexpr (vec == 16) *(uint4*)(srow + dsto[k]) = v[k];
          else if constexpr (vec == 4) *(uint32_t*)(srow + dsto[k]) = v[k].x;
          else srow[dsto[k]] = (uint8_t)v[k].x;
        }
      }
      __syncthreads();
    }
    for (int r = 0; r < nrows; ++r) {  // phase 2
      const int oy = row0 + r - pd.top;
      bf16_t* orow = out + ((size_t)b * ohp + row0 + r) * owp * cpad;
      const bool brow = (unsigned)oy >= (unsigned)OH;
      int y0, y1;
      float ly;
      tap_rows(r, y0, y1, ly);
      const uint8_t* t0;
      const uint8_t* t1;
      if constexpr (STAGED) {
        t0 = srow + (2 * r) * rbp;
        t1 = srow + (2 * r + 1) * rbp;
      } else {
        t0 = base + (size_t)y0 * rb;
        t1 = base + (size_t)y1 * rb;
      }
      for (int px = threadIdx.x; px < owp; px += blockDim.x) {
        const int ox = px - pd.left;
        bf16_t* o = orow + (size_t)px * cpad;
        if (brow || (unsigned)ox >= (unsigned)OW) {
          store_px(o, 0.f, 0.f, 0.f, cpad);
          continue;
        }
        const float sx = fmaxf((ox + 0.5f) * sw - 0.5f, 0.f);
        const int x0 = min((int)sx, iw - 1), x1 = min(x0 + 1, iw - 1);
        const float lx = sx - x0;
        float c[3];
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
          const float v00 = t0[x0 * 3 + ch], v01 = t0[x1 * 3 + ch];
          const float v10 = t1[x0 * 3 + ch], v11 = t1[x1 * 3 + ch];
          c[ch] = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
        }
        store_px(o, c[0] * i0 - o0, c[1] * i1 - o1, c[2] * i2 - o2, cpad);
      }
    }
  }
}

// Identity resize (OH == H, OW == W: bilinear weights are exactly 0 / 1, so the result is
// bitwise the bilinear kernel's) into the 4-channel pixel-pair stem canvas - the training
// benchmark's synthetic images arrive at the output size.  A pure stream (u8 in, 8-B bf16
// pixels out): a block owns 4 canvas rows (one wave each, no grid stride, so no load ever
// queues behind an earlier store in the in-order vmcnt); lane g < W/4 converts source
// pixels 4g..4g+3 (three aligned dwords -> four 8-B stores), the next lanes write the row's
// left / right border pixels, and border rows are zero-filled.
__global__ __launch_bounds__(256) void preprocess_copy4_kernel(
    const uint8_t* __restrict__ img, int B, int H, int W, Norm3 nrm, OutPad pd,
    bf16_t* __restrict__ out) {
  const float* mean = nrm.mean;
  const float* stdv = nrm.std;
  const float i0 = 1.f / (255.f * stdv[0]), i1 = 1.f / (255.f * stdv[1]), i2 = 1.f / (255.f * stdv[2]);
  const float o0 = mean[0] / stdv[0], o1 = mean[1] / stdv[1], o2 = mean[2] / stdv[2];
  const int ohp = H + pd.top + pd.bottom, owp = W + pd.left + pd.right;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);  // canvas row of all images
  if (row >= B * ohp) return;
  const int lane = threadIdx.x & 63;
  const int b = row / ohp, cy = row - b * ohp, y = cy - pd.top;
  bf16_t* orow = out + (size_t)row * owp * 4;
  if ((unsigned)y >= (unsigned)H) {
    for (int px = lane; px < owp; px += 64) *(uint2*)(orow + px * 4) = make_uint2(0u, 0u);
    return;
  }
  const int G = W >> 2, bw = pd.left + pd.right;
  const uint32_t* src = (const uint32_t*)(img + ((size_t)b * H + y) * W * 3);
  for (int g = lane; g < G + bw; g += 64) {
    if (g >= G) {  // border pixel of an interior row
      const int k = g - G;
      const int px = k < pd.left ? k : W + k;
      *(uint2*)(orow + px * 4) = make_uint2(0u, 0u);
      continue;
    }
    const uint32_t w0 = src[3 * g], w1 = src[3 * g + 1], w2 = src[3 * g + 2];
    const uint32_t v[12] = {w0 & 255u, (w0 >> 8) & 255u, (w0 >> 16) & 255u, w0 >> 24,
                            w1 & 255u, (w1 >> 8) & 255u, (w1 >> 16) & 255u, w1 >> 24,
                            w2 & 255u, (w2 >> 8) & 255u, (w2 >> 16) & 255u, w2 >> 24};
    bf16_t* o = orow + (pd.left + 4 * g) * 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float c0 = (float)v[3 * q], c1 = (float)v[3 * q + 1], c2 = (float)v[3 * q + 2];
      store_px(o + 4 * q, c0 * i0 - o0, c1 * i1 - o1, c2 * i2 - o2, 4);
    }
  }
}

// Bicubic-AA (eval path): one block per canvas row (blockIdx.x = row, blockIdx.y =
// image); the per-pixel filter windows dominate, not the indexing.
struct CanvasRow {
  int owp, oy;     // canvas row width; resized-image row (outside [0, OH): border row)
  bool border;
  bf16_t* out;     // first pixel of this canvas row
};

__device__ __forceinline__ CanvasRow canvas_row(const OutPad& pd, int OH, int OW, int cpad,
                                                bf16_t* out) {
  CanvasRow r;
  const int ohp = OH + pd.top + pd.bottom;
  r.owp = OW + pd.left + pd.right;
  r.oy = (int)blockIdx.x - pd.top;
  r.border = (unsigned)r.oy >= (unsigned)OH;
  r.out = out + (((size_t)blockIdx.y * ohp + blockIdx.x) * r.owp) * cpad;
  return r;
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
  const CanvasRow cr = canvas_row(pd, OH, OW, cpad, out);
  const float* mean = nrm.mean;
  const float* stdv = nrm.std;
  const int oy = cr.oy;
  for (int px = threadIdx.x; px < cr.owp; px += blockDim.x) {
    const int ox = px - pd.left;
    bf16_t* o = cr.out + (size_t)px * cpad;
    if (cr.border || (unsigned)ox >= (unsigned)OW) {
      store_px(o, 0.f, 0.f, 0.f, cpad);
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
    const uint8_t* base = img + (size_t)blockIdx.y * H * W * 3;
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
    store_px(o, (acc[0] / 255.f - mean[0]) / stdv[0],
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

// offset: host part of the stream position; dev_off (optional): a device counter added to
// it, advanced by dropout_counter_inc after every call - a HIP graph replays the read and
// the increment, so every replay draws a fresh mask (a host offset is frozen at capture)
__global__ void dropout_fwd_kernel(const bf16_t* __restrict__ x, int64_t n, float p, uint32_t seed,
                                   uint32_t offset, const uint32_t* __restrict__ dev_off,
                                   bf16_t* __restrict__ y, uint8_t* __restrict__ mask) {
  const float scale = 1.f / (1.f - p);
  if (dev_off) offset += *dev_off;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hash3(seed, offset, (uint32_t)i);
    const float u = (h >> 8) * (1.f / 16777216.f);
    const bool keep = u >= p;
    mask[i] = keep ? 1 : 0;
    y[i] = keep ? f2bf(bf2f(x[i]) * scale) : (bf16_t)0;
  }
}

__global__ void dropout_counter_inc_kernel(uint32_t* c) { c[0] += 1u; }

__global__ void dropout_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ mask,
                                   int64_t n, float p, bf16_t* __restrict__ dx) {
  const float scale = 1.f / (1.f - p);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dx[i] = mask[i] ? f2bf(bf2f(dy[i]) * scale) : (bf16_t)0;
}

// ---------------------------------------------------------------- PIL-exact bicubic (eval)
// Pillow's 8-bpc resampler (evaluation_pipeline.py:89 -> data/pil_resize.py): integer
// tables (22-bit fixed point) built on the host exactly as Pillow builds them, a horizontal
// pass rounded + clipped to uint8, then a vertical pass over that uint8 image, then
// ToTensor/Normalize in fp32 with torchvision's operation order.  Every image b of the batch
// has its own source extent ext[b] = (h, w) inside the [Hp][Wp] slot pitch (real JPEGs of
// different sizes decoded into one padded ring slot) and its own tables sel[b] = (width
// table, height table).  The output equals PIL's uint8 image exactly before normalisation.
constexpr int PIL_PREC = 22;

__device__ __forceinline__ int pil_clip8(int v) { return min(max(v >> PIL_PREC, 0), 255); }

// tmp[b][y][ox] (RGBx, 4 B) for the rows y < h_b: one thread per output column
__global__ __launch_bounds__(256) void pil_hpass_kernel(const uint8_t* __restrict__ img, int Hp,
                                                        int Wp, const int* __restrict__ ext,
                                                        const int* __restrict__ sel,
                                                        const int* __restrict__ hb,
                                                        const int* __restrict__ hk, int kh, int OW,
                                                        uint32_t* __restrict__ tmp) {
  const int b = blockIdx.z, y = blockIdx.y;
  const int ox = blockIdx.x * blockDim.x + threadIdx.x;
  const int h = ext ? ext[2 * b] : Hp;
  if (y >= h || ox >= OW) return;
  const int tab = sel[2 * b];
  const int xmin = hb[2 * (tab * OW + ox)], xs = hb[2 * (tab * OW + ox) + 1];
  const int* k = hk + (size_t)(tab * OW + ox) * kh;
  const uint8_t* p = img + (((size_t)b * Hp + y) * Wp + xmin) * 3;
  int s0 = 1 << (PIL_PREC - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < xs; ++t) {
    const int kt = k[t];
    s0 += (int)p[3 * t] * kt;
    s1 += (int)p[3 * t + 1] * kt;
    s2 += (int)p[3 * t + 2] * kt;
  }
  tmp[((size_t)b * Hp + y) * OW + ox] =
      (uint32_t)pil_clip8(s0) | ((uint32_t)pil_clip8(s1) << 8) | ((uint32_t)pil_clip8(s2) << 16);
}

// one block per canvas row (blockIdx.x) of image blockIdx.y; threads over its pixels
__global__ __launch_bounds__(256) void pil_vpass_kernel(const uint32_t* __restrict__ tmp, int Hp,
                                                        const int* __restrict__ sel,
                                                        const int* __restrict__ vb,
                                                        const int* __restrict__ vk, int kv, int OH,
                                                        int OW, Norm3 nrm, int cpad, OutPad pd,
                                                        bf16_t* __restrict__ out) {
  const CanvasRow cr = canvas_row(pd, OH, OW, cpad, out);
  const int b = blockIdx.y, oy = cr.oy;
  int ymin = 0, ys = 0;
  const int* k = nullptr;
  if (!cr.border) {
    const int tab = sel[2 * b + 1];
    ymin = vb[2 * (tab * OH + oy)];
    ys = vb[2 * (tab * OH + oy) + 1];
    k = vk + (size_t)(tab * OH + oy) * kv;
  }
  for (int px = threadIdx.x; px < cr.owp; px += blockDim.x) {
    const int ox = px - pd.left;
    bf16_t* o = cr.out + (size_t)px * cpad;
    if (cr.border || (unsigned)ox >= (unsigned)OW) {
      store_px(o, 0.f, 0.f, 0.f, cpad);
      continue;
    }
    const uint32_t* col = tmp + ((size_t)b * Hp + ymin) * OW + ox;
    int s0 = 1 << (PIL_PREC - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < ys; ++t) {
      const uint32_t v = col[(size_t)t * OW];
      const int kt = k[t];
      s0 += (int)(v & 255u) * kt;
      s1 += (int)((v >> 8) & 255u) * kt;
      s2 += (int)((v >> 16) & 255u) * kt;
    }
    // ToTensor (u8 / 255) then Normalize ((x - mean) / std), each step in fp32
    const float c0 = ((float)pil_clip8(s0) / 255.f - nrm.mean[0]) / nrm.std[0];
    const float c1 = ((float)pil_clip8(s1) / 255.f - nrm.mean[1]) / nrm.std[1];
    const float c2 = ((float)pil_clip8(s2) / 255.f - nrm.mean[2]) / nrm.std[2];
    store_px(o, c0, c1, c2, cpad);
  }
}

void preprocess_pil(const uint8_t* img, int B, int Hp, int Wp, const int* ext, const int* sel,
                    const int* hb, const int* hk, int kh, const int* vb, const int* vk, int kv,
                    int OH, int OW, Norm3 nrm, int cpad, OutPad pd, uint32_t* tmp, bf16_raw* out,
                    hipStream_t s) {
  if (B <= 0) return;
  const int tx = OW >= 256 ? 256 : std::max(64, (OW + 63) / 64 * 64);
  hipLaunchKernelGGL(pil_hpass_kernel, dim3((OW + tx - 1) / tx, Hp, B), dim3(tx), 0, s, img, Hp,
                     Wp, ext, sel, hb, hk, kh, OW, tmp);
  const int ohp = OH + pd.top + pd.bottom, owp = OW + pd.left + pd.right;
  const dim3 block(owp >= 256 ? 256 : std::max(64, (owp + 63) / 64 * 64));
  hipLaunchKernelGGL(pil_vpass_kernel, dim3(ohp, B), block, 0, s, tmp, Hp, sel, vb, vk, kv, OH,
                     OW, nrm, cpad, pd, (bf16_t*)out);
}

static int blocks_n(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

// identity-size fast path (preprocess_copy4_kernel); MPA_PRE_COPY=0 / the setter disable it
static int g_pre_copy = [] {
  const char* e = getenv("MPA_PRE_COPY");
  return e ? atoi(e) : 1;
}();
void preprocess_set_copy(int on) { g_pre_copy = on; }

void preprocess(const uint8_t* img, int B, int H, int W, int OH, int OW, Norm3 nrm, int mode,
                int cpad, OutPad pd, bf16_raw* out, hipStream_t s, const int* ext) {
  if (B <= 0) return;  // bicubic: gridDim.y = images (<= 65535)
  const int ohp = OH + pd.top + pd.bottom, owp = OW + pd.left + pd.right;
  if (mode == 0 && !ext && g_pre_copy && H == OH && W == OW && cpad == 4 && W % 4 == 0 &&
      reinterpret_cast<uintptr_t>(img) % 4 == 0 && (int64_t)B * ohp < (1ll << 30)) {
    hipLaunchKernelGGL(preprocess_copy4_kernel, dim3((B * ohp + 3) / 4), dim3(256), 0, s, img, B,
                       H, W, nrm, pd, out);
    return;
  }
  if (mode == 0) {
    const int items = B * ((ohp + PP_ROWS - 1) / PP_ROWS);
    const dim3 grid(std::min(items, 2048));
    const size_t lds = (size_t)PP_ROWS * 2 * ((W * 3 + 15) & ~15);
    const int rb = W * 3;
    const uintptr_t ia = (uintptr_t)img;
    const int vec = (rb % 16 == 0 && ia % 16 == 0) ? 16 : (rb % 4 == 0 && ia % 4 == 0) ? 4 : 1;
#define PP_LAUNCH(ST, V, CP, L)                                                                 \
  hipLaunchKernelGGL((preprocess_bilinear_kernel<ST, V, CP>), grid, dim3(256), L, s, img, B, H, \
                     W, OH, OW, nrm, cpad, pd, out, ext)
#define PP_CPAD(ST, V, L)                                      \
  do {                                                         \
    if (cpad == 4) PP_LAUNCH(ST, V, 4, L);                     \
    else if (cpad == 8) PP_LAUNCH(ST, V, 8, L);                \
    else PP_LAUNCH(ST, V, 0, L);                               \
  } while (0)
    if (W > PP_MAXW) PP_CPAD(false, 1, 0);
    else if (vec == 16) PP_CPAD(true, 16, lds);
    else if (vec == 4) PP_CPAD(true, 4, lds);
    else PP_CPAD(true, 1, lds);
#undef PP_CPAD
#undef PP_LAUNCH
  } else {
    const dim3 block(owp >= 256 ? 256 : std::max(64, (owp + 63) / 64 * 64));
    hipLaunchKernelGGL(preprocess_bicubic_aa_kernel, dim3(ohp, B), block, 0, s, img, B, H, W, OH,
                       OW, nrm, cpad, pd, out);
  }
}

void dropout_fwd(const bf16_raw* x, int64_t n, float p, uint64_t seed, uint64_t offset,
                 uint32_t* counter, bf16_raw* y, uint8_t* mask, hipStream_t s) {
  hipLaunchKernelGGL(dropout_fwd_kernel, dim3(blocks_n(n)), dim3(256), 0, s, x, n, p,
                     (uint32_t)seed, (uint32_t)offset, (const uint32_t*)counter, y, mask);
  if (counter) hipLaunchKernelGGL(dropout_counter_inc_kernel, dim3(1), dim3(1), 0, s, counter);
}

void dropout_bwd(const bf16_raw* dy, const uint8_t* mask, int64_t n, float p, bf16_raw* dx,
                 hipStream_t s) {
  hipLaunchKernelGGL(dropout_bwd_kernel, dim3(blocks_n(n)), dim3(256), 0, s, dy, mask, n, p, dx);
}

}  // namespace mpa
