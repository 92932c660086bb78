// Channel concat / split of NHWC bf16 activations (K13 of SURVEY.md §2.7): DenseNet's dense
// blocks, Inception's branch joins and SqueezeNet's Fire expand pair (reference
// models.py:59-95 -> torchvision torch.cat(dim=1) over NCHW).
//
// In NHWC a channel concat is a per-pixel concatenation of contiguous channel runs, so the
// op is a pure strided copy of 16-B vectors (8 channels).  Grid = (pixel chunks, segment):
// the segment index is blockIdx.y, so each block's source pointer, channel offset and run
// length are wave-uniform scalar loads from the kernarg table - no per-lane segment search.
// The same kernel runs forward (gather the inputs into the output rows) and backward
// (scatter the dy rows into per-input gradients), so the split costs one read and one
// write of the activation, like the forward.  Up to CAT_MAXSEG segments per launch; the
// host issues one launch per CAT_MAXSEG-chunk (DenseNet-121's block 3 joins 25 inputs).
#include "common.h"
#include "api.h"
#include <algorithm>

namespace mpa {

struct CatArgs {
  bf16_raw* seg[CAT_MAXSEG];  // input (concat) / gradient output (split) of each segment
  int off[CAT_MAXSEG];        // channel offset / 8 of the segment in the joined row
  int cs[CAT_MAXSEG];         // channels / 8 of the segment
  int cv;                     // joined row channels / 8
};

template <bool SPLIT>
__global__ void __launch_bounds__(256) concat_kernel(CatArgs a, bf16_raw* __restrict__ y,
                                                     int pixels) {
  const int sidx = blockIdx.y;
  const int cs = a.cs[sidx];
  const int off = a.off[sidx];
  uint4* __restrict__ seg = reinterpret_cast<uint4*>(a.seg[sidx]);
  uint4* __restrict__ row = reinterpret_cast<uint4*>(y);
  const unsigned n = (unsigned)pixels * (unsigned)cs;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned px = i / (unsigned)cs;
    const unsigned v = i - px * (unsigned)cs;
    const int64_t r = (int64_t)px * a.cv + off + v;
    if (SPLIT)
      seg[i] = row[r];
    else
      row[r] = seg[i];
  }
}

static void launch(bool split, bf16_raw* const* segs, const int* chans, int nseg, int pixels,
                   int ctotal, bf16_raw* y, hipStream_t s) {
  int base = 0;
  for (int s0 = 0; s0 < nseg; s0 += CAT_MAXSEG) {
    const int ns = std::min(CAT_MAXSEG, nseg - s0);
    CatArgs a{};
    a.cv = ctotal / 8;
    int maxcs = 1;
    for (int i = 0; i < ns; ++i) {
      a.seg[i] = segs[s0 + i];
      a.off[i] = base / 8;
      a.cs[i] = chans[s0 + i] / 8;
      base += chans[s0 + i];
      maxcs = std::max(maxcs, a.cs[i]);
    }
    const int64_t work = (int64_t)pixels * maxcs;
    const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256,
                                                               std::max(64, 4096 / ns)));
    if (split)
      hipLaunchKernelGGL(concat_kernel<true>, dim3(gx, ns), dim3(256), 0, s, a, y, pixels);
    else
      hipLaunchKernelGGL(concat_kernel<false>, dim3(gx, ns), dim3(256), 0, s, a, y, pixels);
  }
}

void concat_channels(const bf16_raw* const* xs, const int* chans, int nseg, int pixels,
                     int ctotal, bf16_raw* y, hipStream_t s) {
  launch(false, const_cast<bf16_raw* const*>(xs), chans, nseg, pixels, ctotal, y, s);
}

void chan_insert(bf16_raw* dst, int ld, int off, const bf16_raw* src, int cs, int rows,
                 hipStream_t s) {
  CatArgs a{};
  a.cv = ld / 8;
  a.seg[0] = const_cast<bf16_raw*>(src);
  a.off[0] = off / 8;
  a.cs[0] = cs / 8;
  const int64_t work = (int64_t)rows * a.cs[0];
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 4096));
  hipLaunchKernelGGL(concat_kernel<false>, dim3(gx, 1), dim3(256), 0, s, a, dst, rows);
}

void chan_slice(const bf16_raw* src, int ld, int off, bf16_raw* dst, int cs, int rows,
                hipStream_t s) {
  CatArgs a{};
  a.cv = ld / 8;
  a.seg[0] = dst;
  a.off[0] = off / 8;
  a.cs[0] = cs / 8;
  const int64_t work = (int64_t)rows * a.cs[0];
  const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 4096));
  hipLaunchKernelGGL(concat_kernel<true>, dim3(gx, 1), dim3(256), 0, s, a,
                     const_cast<bf16_raw*>(src), rows);
}

void split_channels(const bf16_raw* dy, const int* chans, int nseg, int pixels, int ctotal,
                    bf16_raw* const* dxs, hipStream_t s) {
  launch(true, dxs, chans, nseg, pixels, ctotal, const_cast<bf16_raw*>(dy), s);
}

// ------------------------------------------------------- fp32 channel-range accumulator
// A dense block's gradient buffer G [pixels][ldg] (fp32): every layer's input gradient
// (bf16, channels [0, cs) of the block's joined features) is ADDED into G's first cs
// channels, and each layer reads its output gradient back as a bf16 channel range - one
// launch per layer instead of autograd's split + one elementwise add per earlier feature
// (models/densenet.py).  8 channels per thread (16-B bf16 / 32-B fp32 vectors).
__global__ void __launch_bounds__(256) chan_accum_kernel(float* __restrict__ g, int ldg8, int off8,
                                                         const bf16_raw* __restrict__ src, int cs8,
                                                         int pixels, int assign) {
  const unsigned n = (unsigned)pixels * (unsigned)cs8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned px = i / (unsigned)cs8, v = i - px * (unsigned)cs8;
    const uint4 b = reinterpret_cast<const uint4*>(src)[i];
    float4* d = reinterpret_cast<float4*>(g + ((int64_t)px * ldg8 + off8 + v) * 8);
    const float4 lo = make_float4(__uint_as_float(b.x << 16), __uint_as_float(b.x & 0xffff0000u),
                                  __uint_as_float(b.y << 16), __uint_as_float(b.y & 0xffff0000u));
    const float4 hi = make_float4(__uint_as_float(b.z << 16), __uint_as_float(b.z & 0xffff0000u),
                                  __uint_as_float(b.w << 16), __uint_as_float(b.w & 0xffff0000u));
    if (assign) {
      d[0] = lo;
      d[1] = hi;
    } else {
      float4 a = d[0], c = d[1];
      d[0] = make_float4(a.x + lo.x, a.y + lo.y, a.z + lo.z, a.w + lo.w);
      d[1] = make_float4(c.x + hi.x, c.y + hi.y, c.z + hi.z, c.w + hi.w);
    }
  }
}

__global__ void __launch_bounds__(256) chan_extract_kernel(const float* __restrict__ g, int ldg8,
                                                           int off8, bf16_raw* __restrict__ dst,
                                                           int cs8, int pixels) {
  const unsigned n = (unsigned)pixels * (unsigned)cs8;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned px = i / (unsigned)cs8, v = i - px * (unsigned)cs8;
    const float4* s4 = reinterpret_cast<const float4*>(g + ((int64_t)px * ldg8 + off8 + v) * 8);
    const float4 a = s4[0], c = s4[1];
    reinterpret_cast<uint4*>(dst)[i] = make_uint4(pack2(a.x, a.y), pack2(a.z, a.w),
                                                  pack2(c.x, c.y), pack2(c.z, c.w));
  }
}

static int chan_grid(int64_t work) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 8192));
}

void chan_accum(float* g, int ldg, int off, const bf16_raw* src, int cs, int pixels, bool assign,
                hipStream_t s) {
  hipLaunchKernelGGL(chan_accum_kernel, dim3(chan_grid((int64_t)pixels * cs / 8)), dim3(256), 0, s,
                     g, ldg / 8, off / 8, src, cs / 8, pixels, assign ? 1 : 0);
}

void chan_extract(const float* g, int ldg, int off, bf16_raw* dst, int cs, int pixels,
                  hipStream_t s) {
  hipLaunchKernelGGL(chan_extract_kernel, dim3(chan_grid((int64_t)pixels * cs / 8)), dim3(256), 0,
                     s, g, ldg / 8, off / 8, dst, cs / 8, pixels);
}

}  // namespace mpa
