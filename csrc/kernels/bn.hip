// BatchNorm (train/eval, fwd/bwd) with fused residual add + ReLU, activation backward with
// fused bias-gradient reduction, and ReLU.  NHWC => a [M][C] row-major matrix with C
// contiguous; every kernel moves 16-B (8 x bf16) chunks.
//
// Thread mapping (all kernels): a block owns up to 256 8-channel chunk columns
// (blockIdx.y selects the column window) and sweeps rows; each thread keeps the SAME 8
// channels for its whole life, so per-channel coefficients live in registers and
// per-channel sums accumulate in registers, reduced once per block through LDS and
// added with one fp32 atomic per channel per block.
//
// Reference ops replaced: ATen batch_norm train/eval + backward, relu, residual add
// (SURVEY.md §2.5, K4/K5/K8).  BN statistics of conv outputs arrive pre-reduced from the
// implicit-GEMM epilogue (igemm.hip), so the forward is a single read+write pass.
#include "common.h"
#include "api.h"
#include <algorithm>
#include <cstdlib>

namespace mpa {

struct ColMap {
  int cw, rpi, cc, r0;
  bool active;
};

__device__ __forceinline__ ColMap colmap(int cpr) {
  ColMap m;
  const int y0 = blockIdx.y * 256;
  m.cw = min(256, cpr - y0);
  m.rpi = 256 / m.cw;
  m.cc = y0 + (int)threadIdx.x % m.cw;
  m.r0 = (int)threadIdx.x / m.cw;
  m.active = m.r0 < m.rpi;
  return m;
}

// Tuning knobs (tools/bench_bn.py): MPA_BN_GRID = target block count, MPA_BN_UNR = rows in
// flight per thread (1, 2 or 4).
static int bn_grid_target() {  // 0: size-based default
  static const int v = [] {
    const char* e = getenv("MPA_BN_GRID");
    return e ? std::max(64, atoi(e)) : 0;
  }();
  return v;
}
static int bn_unr() {
  static const int v = [] {
    const char* e = getenv("MPA_BN_UNR");
    const int u = e ? atoi(e) : 1;
    return (u == 2 || u == 4) ? u : 1;
  }();
  return v;
}
#define BN_LAUNCH(kern, grid, ...)                                                        \
  do {                                                                                    \
    const int u_ = bn_unr();                                                              \
    if (u_ == 4) hipLaunchKernelGGL(kern<4>, grid, dim3(256), 0, __VA_ARGS__);            \
    else if (u_ == 2) hipLaunchKernelGGL(kern<2>, grid, dim3(256), 0, __VA_ARGS__);       \
    else hipLaunchKernelGGL(kern<1>, grid, dim3(256), 0, __VA_ARGS__);                    \
  } while (0)

// Default block count, measured on the ResNet-18 batch-256 shapes (tools/bench_bn.py,
// profiles/bn_grid_sweep.txt): 512 blocks stream 5.5 TB/s on the 411 MB stem activations
// (1024: 5.2, 2048: 4.7 - more blocks only add slab rows and tail waves); tensors under
// 2M 16-B chunks (layer3/4) are tail-bound and fastest at 256.
static dim3 grid_for(int M, int C, int target = 0) {
  if (target <= 0) target = bn_grid_target();
  if (target <= 0) target = ((int64_t)M * (C / 8) >= (2 << 20)) ? 512 : 256;
  const int cpr = C / 8;
  const int gy = (cpr + 255) / 256;
  const int cw = std::min(256, cpr);
  const int rpi = 256 / cw;
  int gx = (M + rpi - 1) / rpi;
  gx = std::max(1, std::min(gx, std::max(1, target / gy)));
  return dim3(gx, gy);
}

// Row sweep with UNR rows in flight per thread: every row's loads are issued before any
// row is consumed, so a thread keeps UNR x (tensors) 16-B loads outstanding (one load per
// thread leaves ~8 MB in flight chip-wide, half of HBM bandwidth x latency).
template <int UNR, typename F>
__device__ __forceinline__ void sweep_rows(const ColMap& cm, int M, F&& body) {
  const int stride = gridDim.x * cm.rpi;
  int r = blockIdx.x * cm.rpi + cm.r0;
  for (; r + (UNR - 1) * stride < M; r += UNR * stride) body(r, stride, UNR);
  for (; r < M; r += stride) body(r, stride, 1);
}

// block-reduce 8-channel partials held per thread; returns sums in threads with r0 == 0
__device__ __forceinline__ void block_reduce8(float* v, const ColMap& cm, float* red) {
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x * 8 + j] = cm.active ? v[j] : 0.f;
  __syncthreads();
  if (cm.active && cm.r0 == 0) {
    for (int r = 1; r < cm.rpi; ++r) {
      const int t = r * cm.cw + (threadIdx.x % cm.cw);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += red[t * 8 + j];
    }
  }
}

// ---------------------------------------------------------------------- statistics
template <int UNR>
__global__ __launch_bounds__(256) void bn_stats_kernel(const bf16_t* __restrict__ x, int M,
                                                        int C, const float* __restrict__ shift,
                                                        float* __restrict__ slab,
                                                        float* __restrict__ sums) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float s[8], q[8], k[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; k[j] = 0.f; }
  if (cm.active) {
    if (blockIdx.x == 0 && cm.r0 == 0) {  // slab_reduce accumulates into these afterwards
#pragma unroll
      for (int j = 0; j < 8; ++j) { sums[cm.cc * 8 + j] = 0.f; sums[C + cm.cc * 8 + j] = 0.f; }
    }
    if (shift) {
#pragma unroll
      for (int j = 0; j < 8; ++j) k[j] = shift[cm.cc * 8 + j];
    }
    sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
      uint4 v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (u < n) v[u] = *(const uint4*)(x + (size_t)(r + u * st) * C + cm.cc * 8);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u >= n) break;
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float d = f[j] - k[j];
          s[j] += d;
          q[j] += d * d;
        }
      }
    });
  }
  block_reduce8(s, cm, red);
  block_reduce8(q, cm, red);
  if (cm.active && cm.r0 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      slab[(size_t)blockIdx.x * 2 * C + cm.cc * 8 + j] = s[j];
      slab[(size_t)blockIdx.x * 2 * C + C + cm.cc * 8 + j] = q[j];
    }
  }
}

// y = relu?(x * sc + sh (+ res)) over this thread's rows
template <int UNR>
__device__ __forceinline__ void bn_apply_rows(const ColMap& cm, int M, int C, int c0,
                                              const float* sc, const float* sh,
                                              const bf16_t* __restrict__ x,
                                              const bf16_t* __restrict__ res, int relu,
                                              bf16_t* __restrict__ y) {
  sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
    uint4 xv[UNR], rv[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u < n) {
        const size_t off = (size_t)(r + u * st) * C + c0;
        xv[u] = *(const uint4*)(x + off);
        if (res) rv[u] = *(const uint4*)(res + off);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u >= n) break;
      float f[8];
      unpack8(xv[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = f[j] * sc[j] + sh[j];
      if (res) {
        float g[8];
        unpack8(rv[u], g);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] += g[j];
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      *(uint4*)(y + (size_t)(r + u * st) * C + c0) = pack8(f);
    }
  });
}

// ------------------------------------------------------------------- forward (train)
template <int UNR>
__global__ __launch_bounds__(256) void bn_fwd_train_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, const bf16_t* __restrict__ res, int relu, int M, int C,
    bf16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    unsigned long long* __restrict__ counter) {
  if (counter && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(counter, 1ull);
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mu = stats[c0 + j];       // finalized (mean, biased var)
    const float var = stats[C + c0 + j];
    const float rs = rsqrtf(var + eps);
    sc[j] = gamma[c0 + j] * rs;
    sh[j] = beta[c0 + j] - mu * sc[j];
    if (blockIdx.x == 0 && cm.r0 == 0) {
      mean_out[c0 + j] = mu;
      rstd_out[c0 + j] = rs;
      const float unb = var * ((float)M / (float)max(M - 1, 1));
      rmean[c0 + j] = (1.f - momentum) * rmean[c0 + j] + momentum * mu;
      rvar[c0 + j] = (1.f - momentum) * rvar[c0 + j] + momentum * unb;
    }
  }
  bn_apply_rows<UNR>(cm, M, C, c0, sc, sh, x, res, relu, y);
}

// -------------------------------------------------------------------- forward (eval)
template <int UNR>
__global__ __launch_bounds__(256) void bn_fwd_eval_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
    const bf16_t* __restrict__ res, int relu, int M, int C, bf16_t* __restrict__ y) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float rs = rsqrtf(rvar[c0 + j] + eps);
    sc[j] = gamma[c0 + j] * rs;
    sh[j] = beta[c0 + j] - rmean[c0 + j] * sc[j];
  }
  bn_apply_rows<UNR>(cm, M, C, c0, sc, sh, x, res, relu, y);
}

// ---------------------------------------------------------------------- backward
// pass 1: ws[0:C] += sum(g), ws[C:2C] += sum(g * xhat), g = dy * (y > 0 if relu)
template <int UNR>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd, int M, int C,
    float* __restrict__ slab, float* __restrict__ sums) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sgx[j] = 0.f; }
  if (cm.active) {
    const int c0 = cm.cc * 8;
    if (blockIdx.x == 0 && cm.r0 == 0) {  // slab_reduce accumulates into these afterwards
#pragma unroll
      for (int j = 0; j < 8; ++j) { sums[c0 + j] = 0.f; sums[C + c0 + j] = 0.f; }
    }
    float mu[8], rs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
    sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
      uint4 dv[UNR], xr[UNR], yr[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u < n) {
          const size_t off = (size_t)(r + u * st) * C + c0;
          dv[u] = *(const uint4*)(dy + off);
          xr[u] = *(const uint4*)(x + off);
          if (y) yr[u] = *(const uint4*)(y + off);
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u >= n) break;
        float g[8], xv[8];
        unpack8(dv[u], g);
        unpack8(xr[u], xv);
        if (y) {
          float yv[8];
          unpack8(yr[u], yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sg[j] += g[j];
          sgx[j] += g[j] * (xv[j] - mu[j]) * rs[j];
        }
      }
    });
  }
  block_reduce8(sg, cm, red);
  block_reduce8(sgx, cm, red);
  if (cm.active && cm.r0 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      slab[(size_t)blockIdx.x * 2 * C + cm.cc * 8 + j] = sg[j];
      slab[(size_t)blockIdx.x * 2 * C + C + cm.cc * 8 + j] = sgx[j];
    }
  }
}

// pass 2: dx = a*g + b + c*x ; optionally write g (residual-branch gradient); block 0
// folds the sums into dgamma/dbeta.
template <int UNR>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ ws, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int M, int C, bf16_t* __restrict__ dx, bf16_t* __restrict__ gout) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float a[8], b[8], cco[8];
  const float invM = 1.f / (float)M;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sg = ws[c0 + j], sgx = ws[C + c0 + j];
    const float rs = rstd[c0 + j];
    const float sc = gamma[c0 + j] * rs;
    a[j] = sc;
    cco[j] = -sc * rs * sgx * invM;
    b[j] = -sc * sg * invM - cco[j] * mean[c0 + j];
    if (blockIdx.x == 0 && cm.r0 == 0) {
      if (dgamma) dgamma[c0 + j] += sgx;
      if (dbeta) dbeta[c0 + j] += sg;
    }
  }
  if (!dx && !gout) return;
  sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
    uint4 dv[UNR], xr[UNR], yr[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u < n) {
        const size_t off = (size_t)(r + u * st) * C + c0;
        dv[u] = *(const uint4*)(dy + off);
        if (y) yr[u] = *(const uint4*)(y + off);
        if (dx) xr[u] = *(const uint4*)(x + off);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if (u >= n) break;
      const size_t off = (size_t)(r + u * st) * C + c0;
      float g[8];
      unpack8(dv[u], g);
      if (y) {
        float yv[8];
        unpack8(yr[u], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
        if (gout) *(uint4*)(gout + off) = pack8(g);
      } else if (gout) {
        *(uint4*)(gout + off) = dv[u];
      }
      if (dx) {
        float xv[8];
        unpack8(xr[u], xv);
#pragma unroll
        for (int j = 0; j < 8; ++j) xv[j] = a[j] * g[j] + b[j] + cco[j] * xv[j];
        *(uint4*)(dx + off) = pack8(xv);
      }
    }
  });
}

// g = dy * (y > 0) ; dbias += colsum(g)
template <int UNR>
__global__ __launch_bounds__(256) void act_bwd_kernel(const bf16_t* __restrict__ dy,
                                                       const bf16_t* __restrict__ y,
                                                       float* __restrict__ slab, int M, int C,
                                                       bf16_t* __restrict__ g) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (cm.active) {
    const int c0 = cm.cc * 8;
    sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
      uint4 dv[UNR], yr[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u < n) {
          const size_t off = (size_t)(r + u * st) * C + c0;
          dv[u] = *(const uint4*)(dy + off);
          if (y) yr[u] = *(const uint4*)(y + off);
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u >= n) break;
        float f[8];
        unpack8(dv[u], f);
        if (y) {
          float yv[8];
          unpack8(yr[u], yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = yv[j] > 0.f ? f[j] : 0.f;
          *(uint4*)(g + (size_t)(r + u * st) * C + c0) = pack8(f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    });
  }
  if (!slab) return;
  block_reduce8(s, cm, red);
  if (cm.active && cm.r0 == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) slab[(size_t)blockIdx.x * C + cm.cc * 8 + j] = s[j];
  }
}

// any C (e.g. a 64,500-wide classifier head): one thread per column, rows in a loop
__global__ __launch_bounds__(256) void act_bwd_generic_kernel(const bf16_t* __restrict__ dy,
                                                               const bf16_t* __restrict__ y,
                                                               float* __restrict__ dbias, int M,
                                                               int C, bf16_t* __restrict__ g) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int r = 0; r < M; ++r) {
    const size_t off = (size_t)r * C + c;
    float f = bf2f(dy[off]);
    if (y) {
      f = bf2f(y[off]) > 0.f ? f : 0.f;
      g[off] = f2bf(f);
    }
    s += f;
  }
  if (dbias) dbias[c] += s;
}

__global__ void relu_kernel(const bf16_t* __restrict__ x, int64_t n8, bf16_t* __restrict__ y) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8;
       i += (int64_t)gridDim.x * blockDim.x) {
    float f[8];
    unpack8(((const uint4*)x)[i], f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    ((uint4*)y)[i] = pack8(f);
  }
}

// Cross-block reduction of per-block partial sums (replaces same-address fp32 atomics,
// which serialise at the memory-side atomic unit when thousands of blocks target the
// same 2*C words - MI355X_MICROARCH.md "Global float atomics", contention row).
// out[w] += sum_s slab[s*W + w]; 64 columns x 4 slab groups per block, <= 32 adds/word.
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ slab, int S,
                                                           int W, float* __restrict__ out) {
  __shared__ float red[256];
  const int w = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  float acc = 0.f;
  if (w < W)
    for (int s_ = blockIdx.y * 4 + g; s_ < S; s_ += gridDim.y * 4) acc += slab[(size_t)s_ * W + w];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && w < W) {
    acc = red[threadIdx.x] + red[threadIdx.x + 64] + red[threadIdx.x + 128] + red[threadIdx.x + 192];
    if (gridDim.y == 1) out[w] += acc;
    else atomicAdd(out + w, acc);
  }
}

// out must hold its starting value (the producer kernels zero it in their first block
// when the reduction should start from 0; zero_out=true is only a fallback memset)
void slab_reduce(const float* slab, int S, int W, float* out, bool zero_out, hipStream_t s) {
  if (zero_out) (void)hipMemsetAsync(out, 0, sizeof(float) * W, s);
  const int gy = std::max(1, std::min(32, (S + 63) / 64));
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((W + 63) / 64, gy), dim3(256), 0, s, slab, S, W, out);
}

int64_t bn_ws_floats(int M, int C) {
  const dim3 g = grid_for(M, C);
  return (int64_t)g.x * 2 * C + 2 * C;
}

__global__ void stats_finalize_kernel(const float* __restrict__ sums, const float* __restrict__ shift,
                                      int M, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.f / (float)M;
  const float d = sums[c] * inv;  // mean of (x - K)
  const float k = shift ? shift[c] : 0.f;
  out[c] = k + d;
  out[C + c] = fmaxf(sums[C + c] * inv - d * d, 0.f);
}

void stats_finalize(const float* sums, const float* shift, int M, int C, float* out,
                    hipStream_t s) {
  hipLaunchKernelGGL(stats_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, sums, shift,
                     M, C, out);
}

// ------------------------------------------------------------------------ launchers
void bn_stats(const bf16_raw* x, int M, int C, const float* shift, float* stats, float* ws,
              hipStream_t s) {
  const dim3 g = grid_for(M, C);
  float* sums = ws + (int64_t)g.x * 2 * C;
  BN_LAUNCH(bn_stats_kernel, g, s, x, M, C, shift, ws, sums);
  slab_reduce(ws, g.x, 2 * C, sums, false, s);
  stats_finalize(sums, shift, M, C, stats, s);
}

void bn_fwd_train(const bf16_raw* x, const float* stats, const float* gamma, const float* beta,
                  float* rmean, float* rvar, float momentum, float eps, const bf16_raw* res,
                  int relu, int M, int C, bf16_raw* y, float* mean, float* rstd,
                  int64_t* counter, hipStream_t s) {
  BN_LAUNCH(bn_fwd_train_kernel, grid_for(M, C), s, x, stats, gamma,
                     beta, rmean, rvar, momentum, eps, res, relu, M, C, y, mean, rstd,
                     (unsigned long long*)counter);
}

void bn_fwd_eval(const bf16_raw* x, const float* gamma, const float* beta, const float* rmean,
                 const float* rvar, float eps, const bf16_raw* res, int relu, int M, int C,
                 bf16_raw* y, hipStream_t s) {
  BN_LAUNCH(bn_fwd_eval_kernel, grid_for(M, C), s, x, gamma, beta, rmean,
                     rvar, eps, res, relu, M, C, y);
}

void bn_bwd(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
            const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M, int C,
            bf16_raw* dx, bf16_raw* g, float* ws, hipStream_t s) {
  // ws layout: [2C] final sums | [gx][2C] per-block partials
  const dim3 gr = grid_for(M, C);
  float* slab = ws + 2 * C;
  BN_LAUNCH(bn_bwd_reduce_kernel, gr, s, dy, x, y, mean, rstd, M, C, slab,
                     ws);
  slab_reduce(slab, gr.x, 2 * C, ws, false, s);
  BN_LAUNCH(bn_bwd_apply_kernel, grid_for(M, C), s, dy, x, y, mean, rstd,
                     gamma, ws, dgamma, dbeta, M, C, dx, g);
}

// apply pass only, with the reduction sums [sum g | sum g*xhat] already in `sums` (e.g.
// from the fused dgrad epilogue, igemm_rows_dgrad_bnred)
void bn_bwd_apply(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
                  const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M,
                  int C, bf16_raw* dx, bf16_raw* g, const float* sums, hipStream_t s) {
  BN_LAUNCH(bn_bwd_apply_kernel, grid_for(M, C), s, dy, x, y, mean, rstd, gamma, sums, dgamma,
            dbeta, M, C, dx, g);
}

void act_bwd(const bf16_raw* dy, const bf16_raw* y, float* dbias, int M, int C, bf16_raw* g,
             float* ws, hipStream_t s) {
  if (C % 8 == 0) {
    const dim3 gr = grid_for(M, C);
    BN_LAUNCH(act_bwd_kernel, gr, s, dy, y, dbias ? ws : (float*)nullptr, M,
                       C, g);
    if (dbias) slab_reduce(ws, gr.x, C, dbias, false, s);
  } else
    hipLaunchKernelGGL(act_bwd_generic_kernel, dim3((C + 255) / 256), dim3(256), 0, s, dy, y,
                       dbias, M, C, g);
}

void relu_fwd(const bf16_raw* x, int64_t n, bf16_raw* y, hipStream_t s) {
  const int64_t n8 = n / 8;
  const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 4096);
  hipLaunchKernelGGL(relu_kernel, dim3(std::max(blocks, 1)), dim3(256), 0, s, x, n8, y);
}

}  // namespace mpa
