// Fused flat-arena optimizers (K11): ONE streaming pass over the fp32 master weights,
// gradients and optimizer state of the whole model.  Applies the data-parallel 1/N
// gradient scale (the average of mpi_tools.py:36 folded in), L2 weight decay, the
// torch.optim.Adam / torch.optim.SGD update rule, and writes the bf16 weight shadow the
// MFMA kernels read (no separate cast pass).  The step counter lives on the device so the
// update is HIP-graph capturable.  Reference: Adam(lr=4e-4) at main.py:125,155.
#include "common.h"
#include "api.h"
#include <algorithm>

namespace mpa {

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16_t* __restrict__ shadow,
                                                    const float* __restrict__ step, int64_t n4,
                                                    float lr, float b1, float b2, float eps,
                                                    float wd, float gs) {
  const float t = step[0] + 1.f;
  const float bc1 = 1.f - powf(b1, t);
  const float bc2s = sqrtf(1.f - powf(b2, t));
  const float step_size = lr / bc1;
  // streaming-bound: 1.33 GB per step at 44 M parameters in ~213 us (6.2 TB/s); the
  // correctly rounded sqrt / divide keep torch.optim.Adam's update bit-for-bit
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i];
    const float4 gg = ((const float4*)g)[i];
    float4 mm = ((float4*)m)[i];
    float4 vv = ((float4*)v)[i];
    float* pf = (float*)&pp;
    const float* gf = (const float*)&gg;
    float* mf = (float*)&mm;
    float* vf = (float*)&vv;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = gf[j] * gs;
      if (wd != 0.f) gr += wd * pf[j];
      mf[j] = b1 * mf[j] + (1.f - b1) * gr;
      vf[j] = b2 * vf[j] + (1.f - b2) * gr * gr;
      const float denom = sqrtf(vf[j]) / bc2s + eps;
      pf[j] -= step_size * mf[j] / denom;
    }
    ((float4*)p)[i] = pp;
    ((float4*)m)[i] = mm;
    ((float4*)v)[i] = vv;
    if (shadow) ((uint2*)shadow)[i] = make_uint2(pack2(pf[0], pf[1]), pack2(pf[2], pf[3]));
  }
}

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ buf, bf16_t* __restrict__ shadow,
                                                   const float* __restrict__ step, int64_t n4,
                                                   float lr, float momentum, float dampening,
                                                   float wd, int nesterov, float gs) {
  const bool first = step[0] == 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i];
    const float4 gg = ((const float4*)g)[i];
    float4 bb = ((float4*)buf)[i];
    float* pf = (float*)&pp;
    const float* gf = (const float*)&gg;
    float* bf = (float*)&bb;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gr = gf[j] * gs;
      if (wd != 0.f) gr += wd * pf[j];
      if (momentum != 0.f) {
        bf[j] = first ? gr : momentum * bf[j] + (1.f - dampening) * gr;
        gr = nesterov ? gr + momentum * bf[j] : bf[j];
      }
      pf[j] -= lr * gr;
    }
    ((float4*)p)[i] = pp;
    if (momentum != 0.f) ((float4*)buf)[i] = bb;
    if (shadow) ((uint2*)shadow)[i] = make_uint2(pack2(pf[0], pf[1]), pack2(pf[2], pf[3]));
  }
}

__global__ void cast_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float4 f = ((const float4*)x)[i];
    ((uint2*)y)[i] = make_uint2(pack2(f.x, f.y), pack2(f.z, f.w));
  }
}

static int blocks_for(int64_t n4) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 4096));
}

void adam_step(float* p, const float* g, float* m, float* v, bf16_raw* shadow, const float* step,
               int64_t n, float lr, float b1, float b2, float eps, float wd, float gs,
               hipStream_t s) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n4)), dim3(256), 0, s, p, g, m, v, shadow, step,
                     n4, lr, b1, b2, eps, wd, gs);
}

void sgd_step(float* p, const float* g, float* buf, bf16_raw* shadow, const float* step,
              int64_t n, float lr, float momentum, float dampening, float wd, int nesterov,
              float gs, hipStream_t s) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(sgd_kernel, dim3(blocks_for(n4)), dim3(256), 0, s, p, g, buf, shadow, step,
                     n4, lr, momentum, dampening, wd, nesterov, gs);
}

void cast_f32_bf16(const float* x, bf16_raw* y, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(cast_kernel, dim3(blocks_for(n4)), dim3(256), 0, s, x, y, n4);
}

static void step_inc_launch(float* step, hipStream_t s);

// ------------------------------------------------------------ transposed weight shadow
// wt[c][t][k] = w[k][t][c] for every registered conv / linear weight, from the bf16 shadow
// the optimizer just wrote: dgrad then reads its B operand K-contiguous, exactly like the
// forward GEMM.  seg: [nseg][6] int64 = (src_off, dst_off, K, RS, C, first_tile); one
// 64x64 (k, c) tile of one tap per block, tiles of all weights in one flat grid.
__global__ __launch_bounds__(256) void transpose_krsc_kernel(const bf16_t* __restrict__ w,
                                                              bf16_t* __restrict__ wt,
                                                              const int64_t* __restrict__ seg,
                                                              int nseg, int total_tiles,
                                                              float* __restrict__ step_inc) {
  // the optimizer kernel that read the step counter has completed (stream order): count
  // the step here instead of in a launch of its own
  if (step_inc && blockIdx.x == 0 && threadIdx.x == 0) *step_inc += 1.f;
  // 64 (k) x 64 (c) tile, rows of eight 16-B chunks; chunk q of row r is stored at
  // position q ^ ((r >> 3) & 7), so the store phase's column gathers (8 lanes per k-row
  // group, one k-row from each of 8 row groups) hit 8 distinct chunk positions: no bank
  // conflicts (with a padded [64][72] tile they were 4-way)
  __shared__ __attribute__((aligned(16))) bf16_t tile[64][64];
  // one tile per block (a grid-stride loop over tiles with 2,048 blocks measured slower)
  for (int b = blockIdx.x; b < total_tiles; b += gridDim.x) {
    __syncthreads();  // previous tile's gathers done before the tile is overwritten
    int lo = 0, hi = nseg - 1;  // last segment whose first_tile <= b (uniform)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (seg[mid * 6 + 5] <= b) lo = mid; else hi = mid - 1;
    }
    const int64_t* d = seg + lo * 6;
    const int64_t so = d[0], dof = d[1];
    const int K = (int)d[2], RS = (int)d[3], C = (int)d[4];  // K % 8 == 0, C % 8 == 0
    const int tk = (K + 63) / 64, tc = (C + 63) / 64;
    int r = b - (int)d[5];
    const int t = r / (tk * tc);
    r -= t * tk * tc;
    const int k0 = (r / tc) * 64, c0 = (r % tc) * 64;
    // load: 512 16-B chunks (64 k-rows x 8 c-chunks), 2 per thread
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = threadIdx.x + 256 * h;
      const int row = q >> 3, ch = q & 7;
      const int k = k0 + row, c = c0 + ch * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < K && c < C) v = *(const uint4*)(w + so + ((size_t)k * RS + t) * C + c);
      *(uint4*)&tile[row][(ch ^ ((row >> 3) & 7)) * 8] = v;
    }
    __syncthreads();
    // store: 512 16-B chunks (64 c-rows x 8 k-chunks), each gathered from a tile column
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q = threadIdx.x + 256 * h;
      const int crow = q >> 3, kk = (q & 7) * 8;
      const int c = c0 + crow, k = k0 + kk;
      if (c < C && k < K) {
        const int cpos = crow & 7, cq = crow >> 3;
        const int col = ((cq ^ (q & 7)) << 3) + cpos;  // rows kk..kk+7 share (row >> 3) = q & 7
        uint32_t e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          e[u] = (uint32_t)tile[kk + 2 * u][col] | ((uint32_t)tile[kk + 2 * u + 1][col] << 16);
        *(uint4*)(wt + dof + ((size_t)c * RS + t) * K + k) = make_uint4(e[0], e[1], e[2], e[3]);
      }
    }
  }
}

void transpose_krsc(const bf16_raw* w, bf16_raw* wt, const int64_t* seg, int nseg,
                    int total_tiles, hipStream_t s, float* step_inc) {
  if (nseg <= 0 || total_tiles <= 0) {
    if (step_inc) step_inc_launch(step_inc, s);
    return;
  }
  hipLaunchKernelGGL(transpose_krsc_kernel, dim3(total_tiles), dim3(256), 0, s, w, wt, seg, nseg,
                     total_tiles, step_inc);
}

// ------------------------------------------------------------------------ small helpers
__global__ __launch_bounds__(256) void zero_f32_kernel(float4* __restrict__ t, int64_t n4) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x)
    t[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ void step_inc_kernel(float* step) { *step += 1.f; }

// dst[i] += src[i] (fp32; small vectors: a bias gradient from a fused reduction)
__global__ __launch_bounds__(256) void add_f32_kernel(float* __restrict__ dst,
                                                     const float* __restrict__ src, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] += src[i];
}

// t viewed as [rows][period] fp32: zero columns [first, first + count) of every row (the
// pixel-pair stem's weight-gradient column past the kernel, layers.Conv2d.fix_grad)
__global__ __launch_bounds__(256) void zero_cols_f32_kernel(float* __restrict__ t, int64_t rows,
                                                            int period, int first, int count) {
  const int64_t n = rows * count;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / count;
    t[r * period + first + (int)(i - r * count)] = 0.f;
  }
}

// a += b over bf16 vectors (fp32 add, one rounding): two computed gradient contributions
// of one activation (GradJoin) summed without an ATen elementwise kernel
__global__ __launch_bounds__(256) void add_bf16_kernel(uint4* __restrict__ a,
                                                       const uint4* __restrict__ b, int64_t n8) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float x[8], y[8];
    unpack8(a[i], x);
    unpack8(b[i], y);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] += y[j];
    a[i] = pack8(x);
  }
}

void zero_cols_f32(float* t, int64_t rows, int period, int first, int count, hipStream_t s) {
  const int64_t n = rows * count;
  if (n > 0)
    hipLaunchKernelGGL(zero_cols_f32_kernel, dim3(blocks_for((n + 3) / 4)), dim3(256), 0, s, t,
                       rows, period, first, count);
}

void add_bf16(bf16_raw* a, const bf16_raw* b, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  if (n8 > 0)
    hipLaunchKernelGGL(add_bf16_kernel, dim3(blocks_for((n8 + 1) / 2)), dim3(256), 0, s,
                       (uint4*)a, (const uint4*)b, n8);
}

void zero_f32(float* t, int64_t n, hipStream_t s) {
  const int64_t n4 = n / 4;
  if (n4 > 0)
    hipLaunchKernelGGL(zero_f32_kernel, dim3(blocks_for(n4)), dim3(256), 0, s, (float4*)t, n4);
}

void add_f32(float* dst, const float* src, int64_t n, hipStream_t s) {
  if (n > 0)
    hipLaunchKernelGGL(add_f32_kernel, dim3(std::min<int64_t>((n + 255) / 256, 1024)), dim3(256),
                       0, s, dst, src, n);
}

static void step_inc_launch(float* step, hipStream_t s) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
}
void step_inc(float* step, hipStream_t s) { step_inc_launch(step, s); }

}  // namespace mpa
