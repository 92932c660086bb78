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

void split_channels(const bf16_raw* dy, const int* chans, int nseg, int pixels, int ctotal,
                    bf16_raw* const* dxs, hipStream_t s) {
  launch(true, dxs, chans, nseg, pixels, ctotal, const_cast<bf16_raw*>(dy), s);
}

}  // namespace mpa
