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

// Rows in flight per thread: 2 (batch-512 ResNet-18 step 13.47 ms against 13.63 with 1
// and 13.49 with 4, round 1 gpu_ab.sh, two alternating repeats).
// as BN_LAUNCH, for kernels with a second (bool) template parameter
#define BN_LAUNCH_T(kern, T, grid, ...) \
  hipLaunchKernelGGL((kern<2, T>), grid, dim3(256), 0, __VA_ARGS__)
#define BN_LAUNCH(kern, grid, ...) hipLaunchKernelGGL(kern<2>, grid, dim3(256), 0, __VA_ARGS__)

// Default block count, measured on the ResNet-18 batch-256 shapes (tools/bench_bn.py,
// profiles/bn_grid_sweep.txt): 512 blocks stream 5.5 TB/s on the 411 MB stem activations
// (1024: 5.2, 2048: 4.7 - more blocks only add slab rows and tail waves); tensors under
// 2M 16-B chunks (layer3/4) are tail-bound and fastest at 256.
static dim3 grid_for(int M, int C, int target = 0) {
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

// Software-pipelined row sweep for the kernels that STORE per row: the loads of the next
// UNR rows are issued before the current rows are processed and stored.  On CDNA, loads
// and stores share the in-order vmcnt, so in the plain sweep the wait for row i+1's loads
// also waited for row i's stores - a full write round trip per iteration.  Here the wait
// for the prefetched rows leaves the stores issued after them in flight.
// load(r, regs[u]) fills the NT 16-B vectors of row r; proc(r, regs[u]) consumes them.
template <int UNR, int NT, typename L, typename P>
__device__ __forceinline__ void sweep_rows_pl(const ColMap& cm, int M, L&& load, P&& proc) {
  const int stride = gridDim.x * cm.rpi;
  int r = blockIdx.x * cm.rpi + cm.r0;
  if (r >= M) return;
  uint4 cur[UNR][NT], nxt[UNR][NT];
#pragma unroll
  for (int u = 0; u < UNR; ++u)
    if (r + u * stride < M) load(r + u * stride, cur[u]);
  for (;;) {
    const int rn = r + UNR * stride;
    const bool more = rn < M;
    if (more) {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (rn + u * stride < M) load(rn + u * stride, nxt[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u)
      if (r + u * stride < M) proc(r + u * stride, cur[u]);
    if (!more) break;
    for (int u = 0; u < UNR; ++u)
      for (int t = 0; t < NT; ++t) cur[u][t] = nxt[u][t];
    r = rn;
  }
}

// Nontemporal hint for tensors of >= 40 M elements (ResNet-18 layer1 / layer2 at batch
// >= 1024): +4-8 % on their BN passes (tools/bench_bn.py, profiles/bn_nt_r6.txt); the
// L2-sized layer3/4 tensors were 5-15 % slower with it (their consumer re-reads them)
__device__ __forceinline__ bool stream_hint(int M, int C) {
  return (int64_t)M * C >= (40ll << 20);
}
__device__ __forceinline__ uint4 ld16(const bf16_t* p, bool nt) {
  return nt ? ld_stream(p) : *(const uint4*)p;
}
__device__ __forceinline__ void st16(bf16_t* p, uint4 v, bool nt) {
  if (nt) st_stream(p, v);
  else *(uint4*)p = v;
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

// bit j = (bf16 element j of the 16-B vector > 0): the ReLU mask of a stored output
__device__ __forceinline__ uint32_t posmask8(uint4 p) {
  const uint32_t w[4] = {p.x, p.y, p.z, p.w};
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t lo = w[i] & 0xffffu, hi = w[i] >> 16;
    m |= (uint32_t)(lo - 1u < 0x7fffu) << (2 * i);  // 1 .. 0x7fff: positive
    m |= (uint32_t)(hi - 1u < 0x7fffu) << (2 * i + 1);
  }
  return m;
}

// y = relu?(x * sc + sh (+ res)) over this thread's rows; ym (optional): the ReLU mask of y,
// one bit per element (byte r * C/8 + c0/8), which the backward reads instead of y.  x rows
// have stride ldx >= C (a channel prefix of a wider buffer: DenseNet's block features)
// rsc / rsh (optional, this thread's 8 channels): the residual enters as res * rsc + rsh -
// a residual branch's own BN (ResNet's downsample) applied while it is read, so that BN's
// output is never written
template <int UNR, bool YM = false>
__device__ __forceinline__ void bn_apply_rows(const ColMap& cm, int M, int C, int ldx, int c0,
                                              const float* sc, const float* sh,
                                              const bf16_t* __restrict__ x,
                                              const bf16_t* __restrict__ res, int relu,
                                              bf16_t* __restrict__ y,
                                              uint8_t* __restrict__ ym = nullptr,
                                              const float* rsc = nullptr,
                                              const float* rsh = nullptr, int ldy = 0) {
  if (ldy <= 0) ldy = C;
  const bool nt = stream_hint(M, C);
  sweep_rows_pl<UNR, 2>(
      cm, M,
      [&](int r, uint4 (&v)[2]) {
        const size_t off = (size_t)r * C + c0;
        v[0] = ld16(x + (size_t)r * ldx + c0, nt);
        if (res) v[1] = ld16(res + off, nt);
      },
      [&](int r, uint4 (&v)[2]) {
        float f[8];
        unpack8(v[0], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = __builtin_fmaf(f[j], sc[j], sh[j]);
        if (res) {
          float g[8];
          unpack8(v[1], g);
          if (rsc) {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += __builtin_fmaf(g[j], rsc[j], rsh[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] += g[j];
          }
        }
        if (relu) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
        }
        const uint4 pk = pack8(f);
        st16(y + (size_t)r * ldy + c0, pk, nt);
        if constexpr (YM) ym[(size_t)r * (C / 8) + c0 / 8] = (uint8_t)posmask8(pk);
      });
}

// y = relu?(x * aff[c] + aff[C + c]): a BN whose affine was computed by bn_stats_affine,
// materialized (the fallback of the operand-path BN when the consumer's kernel cannot apply
// it while staging)
template <int UNR>
__global__ __launch_bounds__(256) void affine_act_kernel(const bf16_t* __restrict__ x,
                                                         const float* __restrict__ aff, int relu,
                                                         int M, int C, bf16_t* __restrict__ y) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = aff[c0 + j];
    sh[j] = aff[C + c0 + j];
  }
  bn_apply_rows<UNR>(cm, M, C, C, c0, sc, sh, x, nullptr, relu, y);
}

// ------------------------------------------------------------------- forward (train)
template <int UNR, bool YM>
__global__ __launch_bounds__(256) void bn_fwd_train_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, const bf16_t* __restrict__ res, int relu, int M, int C,
    bf16_t* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    unsigned long long* __restrict__ counter, uint8_t* __restrict__ ymask, int ldx, int lds,
    const float* __restrict__ res_aff, int ldy) {
  if (counter && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(counter, 1ull);
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float sc[8], sh[8], rsc[8], rsh[8];
  if (res_aff) {  // [2][C]: the residual's BN scale | shift
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      rsc[j] = res_aff[c0 + j];
      rsh[j] = res_aff[C + c0 + j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mu = stats[c0 + j];       // finalized (mean, biased var); rows lds apart
    const float var = stats[lds + c0 + j];
    const float rs = rsqrtf(var + eps);
    sc[j] = gamma[c0 + j] * rs;
    sh[j] = __builtin_fmaf(-mu, sc[j], beta[c0 + j]);
    if (blockIdx.x == 0 && cm.r0 == 0) {
      mean_out[c0 + j] = mu;
      rstd_out[c0 + j] = rs;
      const float unb = var * ((float)M / (float)max(M - 1, 1));
      rmean[c0 + j] = (1.f - momentum) * rmean[c0 + j] + momentum * mu;
      rvar[c0 + j] = (1.f - momentum) * rvar[c0 + j] + momentum * unb;
    }
  }
  if (res_aff)
    bn_apply_rows<UNR, YM>(cm, M, C, ldx, c0, sc, sh, x, res, relu, y, ymask, rsc, rsh, ldy);
  else
    bn_apply_rows<UNR, YM>(cm, M, C, ldx, c0, sc, sh, x, res, relu, y, ymask, nullptr, nullptr,
                           ldy);
}

// Train-mode BN whose apply pass is deferred to its consumer (bn_fwd_train's res_aff): the
// batch mean / rstd from finalized statistics, the running-stat update, num_batches_tracked,
// and the affine [scale | shift] = [gamma rstd | beta - mean gamma rstd] - one thread per
// channel, same arithmetic as bn_fwd_train
__global__ __launch_bounds__(256) void bn_stats_affine_kernel(
    const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, int M, int C, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, float* __restrict__ aff, unsigned long long* __restrict__ counter) {
  if (counter && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(counter, 1ull);
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float mu = stats[c], var = stats[C + c];
  const float rs = rsqrtf(var + eps);
  const float sc = gamma[c] * rs;
  mean_out[c] = mu;
  rstd_out[c] = rs;
  aff[c] = sc;
  aff[C + c] = __builtin_fmaf(-mu, sc, beta[c]);
  const float unb = var * ((float)M / (float)max(M - 1, 1));
  rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
  rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
}

// relu(bn(z)) -> 2x2 / stride-2 average pool in one pass (DenseNet transitions, whose pool
// runs ahead of the 1x1 conv): thread = 8 channels of one pooled pixel, the four inputs
// loaded together; the BN output is never written.  aff [2][C] = scale | shift
// (bn_stats_affine).  The backward reuses avgpool_bwd + bn_bwd (mask recomputed from z).
__global__ __launch_bounds__(256) void bn_relu_avgpool2_fwd_kernel(
    const bf16_t* __restrict__ z, const float* __restrict__ aff, int N, int H, int W, int C,
    bf16_t* __restrict__ y) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = aff[c0 + j];
    sh[j] = aff[C + c0 + j];
  }
  const int P = H / 2, Q = W / 2, MP = N * P * Q;
  for (int r = blockIdx.x * cm.rpi + cm.r0; r < MP; r += gridDim.x * cm.rpi) {
    const int q = r % Q, t = r / Q, p = t % P, n = t / P;
    const size_t i00 = (((size_t)n * H + 2 * p) * W + 2 * q) * C + c0;
    const uint4 v0 = *(const uint4*)(z + i00), v1 = *(const uint4*)(z + i00 + C);
    const uint4 v2 = *(const uint4*)(z + i00 + (size_t)W * C);
    const uint4 v3 = *(const uint4*)(z + i00 + (size_t)W * C + C);
    float a[8], b[8], acc[8];
    unpack8(v0, a);
    unpack8(v1, b);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = fmaxf(__builtin_fmaf(a[j], sc[j], sh[j]), 0.f) +
               fmaxf(__builtin_fmaf(b[j], sc[j], sh[j]), 0.f);
    unpack8(v2, a);
    unpack8(v3, b);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      acc[j] = 0.25f * (acc[j] + fmaxf(__builtin_fmaf(a[j], sc[j], sh[j]), 0.f) +
                        fmaxf(__builtin_fmaf(b[j], sc[j], sh[j]), 0.f));
    *(uint4*)(y + (size_t)r * C + c0) = pack8(acc);
  }
}

// -------------------------------------------------------------------- forward (eval)
template <int UNR>
__global__ __launch_bounds__(256) void bn_fwd_eval_kernel(
    const bf16_t* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ rmean, const float* __restrict__ rvar, float eps,
    const bf16_t* __restrict__ res, int relu, int M, int C, bf16_t* __restrict__ y, int ldx) {
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
  bn_apply_rows<UNR>(cm, M, C, ldx, c0, sc, sh, x, res, relu, y);
}

// ---------------------------------------------------------------------- backward
// pass 1: ws[0:C] += sum(g), ws[C:2C] += sum(g * xhat), g = dy * (y > 0 if relu)
// ReLU mask of y = relu(bn(x)) recomputed from x exactly as bn_fwd_train rounded it
// (same fma affine, same bf16 rounding): the backward of a BN+ReLU whose output carries no
// residual then never reads y - one activation-sized read less in each of its two passes
__device__ __forceinline__ void bn_relu_coeffs(const float* gamma, const float* beta,
                                               const float* mean, const float* rstd, int c0,
                                               float* sc, float* sh) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = gamma[c0 + j] * rstd[c0 + j];
    sh[j] = __builtin_fmaf(-mean[c0 + j], sc[j], beta[c0 + j]);
  }
}
__device__ __forceinline__ bool bn_relu_live(float x, float sc, float sh) {
  return bf2f(f2bf(__builtin_fmaf(x, sc, sh))) > 0.f;
}

// ReLU mask, in order of preference: ym (bit mask written by the forward), zmask (beta !=
// null, y == null: recomputed from x via bn_relu_live), y (the stored output).  (Here ym is
// a runtime pointer: the compile-time variant scheduled the byte load between the row
// loads and waited for each - 117 vs 78 us on layer1; the apply pass is the other way
// round, see there.)
template <int UNR>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int M, int C,
    float* __restrict__ slab, float* __restrict__ sums, const uint8_t* __restrict__ ym, int ldx,
    int lddy) {
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
    float mu[8], rs[8], msc[8], msh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
    const bool zmask = !ym && !y && beta;
    if (zmask) bn_relu_coeffs(gamma, beta, mean, rstd, c0, msc, msh);
    sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
      uint4 dv[UNR], xr[UNR], yr[UNR];
      uint32_t mb[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u < n) {
          const size_t off = (size_t)(r + u * st) * C + c0;
          dv[u] = *(const uint4*)(dy + (size_t)(r + u * st) * lddy + c0);
          xr[u] = *(const uint4*)(x + (size_t)(r + u * st) * ldx + c0);
          if (ym) mb[u] = ym[off / 8];
          else if (y) yr[u] = *(const uint4*)(y + off);
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u >= n) break;
        float g[8], xv[8];
        unpack8(dv[u], g);
        unpack8(xr[u], xv);
        if (ym) {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = (mb[u] >> j) & 1u ? g[j] : 0.f;
        } else if (y) {
          float yv[8];
          unpack8(yr[u], yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
        } else if (zmask) {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = bn_relu_live(xv[j], msc[j], msh[j]) ? g[j] : 0.f;
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
// folds the sums into dgamma/dbeta.  YM (mask from bn_fwd_train) is a template parameter:
// a runtime mask pointer slowed every variant of this pass by 10-40 % (its row loads no
// longer stayed in flight).  x rows have stride ldx.  ACC: dx is ADDED into gacc [M][ldg]
// (a dense block's gradient accumulator; its rows are loaded with the others) instead of
// being written as bf16 - ACC 1: fp32 accumulator, ACC 2: bf16 accumulator (one rounding
// per contribution, as autograd's own bf16 sums; half the accumulator traffic).
template <int UNR, bool YM, int ACC = 0>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ y,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ ws,
    float* __restrict__ dgamma, float* __restrict__ dbeta, int M, int C,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ gout, const uint8_t* __restrict__ ym, int ldx,
    float* __restrict__ gacc, int ldg, int lddx, int lddy) {
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
  if (!ACC && !dx && !gout) return;
  const bool zmask = !YM && !y && beta;
  float msc[8], msh[8];
  if (zmask) bn_relu_coeffs(gamma, beta, mean, rstd, c0, msc, msh);
  const bool need_x = ACC || dx || zmask;
  const bool nt = stream_hint(M, C);
  sweep_rows_pl<UNR, ACC == 1 ? 5 : (ACC == 2 ? 4 : 3)>(
      cm, M,
      [&](int r, uint4 (&v)[ACC == 1 ? 5 : (ACC == 2 ? 4 : 3)]) {
        const size_t off = (size_t)r * C + c0;
        v[0] = ld16(dy + (size_t)r * lddy + c0, nt);
        if constexpr (YM) v[2].x = ym[off / 8];
        else if (y) v[2] = ld16(y + off, nt);
        if (need_x) v[1] = ld16(x + (size_t)r * ldx + c0, nt);
        if constexpr (ACC == 1) {
          const uint4* gp = (const uint4*)(gacc + (size_t)r * ldg + c0);
          v[3] = gp[0];
          v[4] = gp[1];
        } else if constexpr (ACC == 2) {
          v[3] = *(const uint4*)((const bf16_t*)gacc + (size_t)r * ldg + c0);
        }
      },
      [&](int r, uint4 (&v)[ACC == 1 ? 5 : (ACC == 2 ? 4 : 3)]) {
        const size_t off = (size_t)r * C + c0;
        float g[8];
        unpack8(v[0], g);
        if constexpr (YM) {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = (v[2].x >> j) & 1u ? g[j] : 0.f;
          if (gout) *(uint4*)(gout + off) = pack8(g);
        } else if (y) {
          float yv[8];
          unpack8(v[2], yv);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = yv[j] > 0.f ? g[j] : 0.f;
          if (gout) *(uint4*)(gout + off) = pack8(g);
        } else if (zmask) {
          float xv[8];
          unpack8(v[1], xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = bn_relu_live(xv[j], msc[j], msh[j]) ? g[j] : 0.f;
          if (gout) *(uint4*)(gout + off) = pack8(g);
        } else if (gout) {
          *(uint4*)(gout + off) = v[0];
        }
        if (ACC || dx) {
          float xv[8];
          unpack8(v[1], xv);
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = a[j] * g[j] + b[j] + cco[j] * xv[j];
          if constexpr (ACC == 2) {
            float gv[8];
            unpack8(v[3], gv);
#pragma unroll
            for (int j = 0; j < 8; ++j) gv[j] += xv[j];
            *(uint4*)((bf16_t*)gacc + (size_t)r * ldg + c0) = pack8(gv);
          } else if constexpr (ACC == 1) {
            const uint32_t gw[8] = {v[3].x, v[3].y, v[3].z, v[3].w, v[4].x, v[4].y, v[4].z, v[4].w};
            uint4 o[2];
            uint32_t* ow = (uint32_t*)o;
#pragma unroll
            for (int j = 0; j < 8; ++j) ow[j] = __float_as_uint(__uint_as_float(gw[j]) + xv[j]);
            uint4* gp = (uint4*)(gacc + (size_t)r * ldg + c0);
            gp[0] = o[0];
            gp[1] = o[1];
          } else {
            st16(dx + (size_t)r * lddx + c0, pack8(xv), nt);
          }
        }
      });
}

// ------------------------------------------------------- 2x2 / stride-2 max pool (VGG)
// The generic kernels above split every flat index with 64-bit divisions, loop over
// window bounds and move the argmax byte by byte.  A 2x2/s2/p0 pool over an even image
// tiles the input exactly: one thread = one pooled pixel x 8 channels, four 16-B loads in,
// one 16-B value + one 8-B argmax out (forward), or one 2x2 block of 16-B stores (backward:
// every input pixel is written exactly once, no gather, no atomics).
__global__ __launch_bounds__(256) void maxpool2_fwd_kernel(const bf16_t* __restrict__ x, int NP,
                                                           int Q, int C, bf16_t* __restrict__ y,
                                                           uint8_t* __restrict__ idx) {
  const int cv = C / 8;
  const int total = NP * Q * cv;  // (n, p) rows x Q x chunks (host: < 2^31)
  const size_t W2C = (size_t)2 * Q * C;
  // thread item t -> the four 16-B input vectors of its window; the next item's loads are
  // issued before this item's stores (loads and stores share the in-order vmcnt)
  auto load = [&](int t, uint4 (&v)[4]) {
    const int cc = t % cv, r = t / cv;  // r = (n * P + p) * Q + q
    const int q = r % Q, np_ = r / Q;
    // input pixel (n, 2p + a, 2q + b) = row 2 * np_ + a of the [N * H] rows, width 2Q
    const size_t o = ((size_t)(2 * np_) * (2 * Q) + 2 * q) * C + cc * 8;
    v[0] = *(const uint4*)(x + o);
    v[1] = *(const uint4*)(x + o + C);
    v[2] = *(const uint4*)(x + o + W2C);
    v[3] = *(const uint4*)(x + o + W2C + C);
  };
  const int stride = gridDim.x * 256;
  int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= total) return;
  uint4 v[4], vn[4];
  load(t, v);
  for (;;) {
    const int tn = t + stride;
    if (tn < total) load(tn, vn);
    float best[8], f[8];
    uint32_t bi[8];
    unpack8(v[0], best);
#pragma unroll
    for (int j = 0; j < 8; ++j) bi[j] = 0;
#pragma unroll
    for (int u = 1; u < 4; ++u) {
      unpack8(v[u], f);
      // window tap of input (a, b) in a 2x2 window: a * 2 + b (first max wins, NaN wins)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (f[j] > best[j] || (f[j] != f[j] && best[j] == best[j])) {
          best[j] = f[j];
          bi[j] = u;
        }
    }
    const size_t o = (size_t)t * 8;  // == ((n * P + p) * Q + q) * C + cc * 8
    *(uint4*)(y + o) = pack8(best);
    uint2 ib;
    ib.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | (bi[3] << 24);
    ib.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | (bi[7] << 24);
    *(uint2*)(idx + o) = ib;
    if (tn >= total) break;
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = vn[u];
    t = tn;
  }
}

// RELU: the pooled tensor is a ReLU output whose producer's backward is handed over
// (Fn.BNLink): the gradient routes only where the pooled value is > 0 (the argmax element
// IS the pooled value, so that is the producer's own y > 0 mask), and the per-channel sum
// of the routed gradient - the producer's bias gradient - is slab-reduced here.
template <bool RELU>
__global__ __launch_bounds__(256) void maxpool2_bwd_kernel(
    const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ yp,
    int NP, int Q, int C, bf16_t* __restrict__ dx, float* __restrict__ slab,
    float* __restrict__ sums) {
  const ColMap cm = colmap(C / 8);
  float sg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) sg[j] = 0.f;
  if (cm.active) {
    const int c0 = cm.cc * 8;
    if (RELU && blockIdx.x == 0 && cm.r0 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) sums[c0 + j] = 0.f;
    }
    const int M = NP * Q;
    const size_t W2C = (size_t)2 * Q * C;
    // v[0] dy, v[1] = (idx pair, -), v[2] pooled y; next row's loads before this row's stores
    sweep_rows_pl<1, 3>(
        cm, M,
        [&](int r, uint4 (&v)[3]) {
          const size_t o = (size_t)r * C + c0;
          v[0] = *(const uint4*)(dy + o);
          const uint2 iv = *(const uint2*)(idx + o);
          v[1] = make_uint4(iv.x, iv.y, 0u, 0u);
          if constexpr (RELU) v[2] = *(const uint4*)(yp + o);
        },
        [&](int r, uint4 (&v)[3]) {
          float g[8];
          unpack8(v[0], g);
          if constexpr (RELU) {
            float yv[8];
            unpack8(v[2], yv);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              g[j] = yv[j] > 0.f ? g[j] : 0.f;
              sg[j] += g[j];
            }
          }
          const int q = r % Q, np_ = r / Q;
          const size_t row0 = (size_t)(2 * np_) * (2 * Q) + 2 * q;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            float d[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t w = j < 4 ? v[1].x : v[1].y;
              d[j] = ((w >> (8 * (j & 3))) & 0xff) == (uint32_t)u ? g[j] : 0.f;
            }
            bf16_t* p = dx + (row0 + (u & 1)) * C + (u >> 1) * W2C + c0;
            *(uint4*)p = pack8(d);
          }
        });
  }
  if constexpr (RELU) {
    __shared__ float red[256 * 8];
    block_reduce8(sg, cm, red);
    if (cm.active && cm.r0 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) slab[(size_t)blockIdx.x * C + cm.cc * 8 + j] = sg[j];
    }
  }
}

// ---------------------------------------------------------------- residual BN pair
// Backward of y = relu(bn(x) + bn2(x2)) when BOTH BNs are train-mode (ResNet's bn2 and the
// deferred downsample BN it applies on read, Fn.BNDefer): both see the same upstream
// g = dy * mask, so one reduce pass yields [sum g | sum g*xhat | sum g*xhat2] and one apply
// pass writes dx AND dx2 - g is never materialised, and the second BN's own reduce and
// apply passes (read g, x2; read g, x2, write dx2) disappear.  Mask: the forward's bit mask.
template <int UNR>
__global__ __launch_bounds__(256) void bn_bwd_pair_reduce_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
    const uint8_t* __restrict__ ym, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ mean2, const float* __restrict__ rstd2, int M, int C,
    float* __restrict__ slab, float* __restrict__ sums) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float sg[8], sgx[8], sgx2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sgx[j] = 0.f; sgx2[j] = 0.f; }
  if (cm.active) {
    const int c0 = cm.cc * 8;
    if (blockIdx.x == 0 && cm.r0 == 0) {  // slab_reduce accumulates into these afterwards
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sums[c0 + j] = 0.f;
        sums[C + c0 + j] = 0.f;
        sums[2 * C + c0 + j] = 0.f;
      }
    }
    float mu[8], rs[8], mu2[8], rs2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j];
      mu2[j] = mean2[c0 + j]; rs2[j] = rstd2[c0 + j];
    }
    sweep_rows<UNR>(cm, M, [&](int r, int st, int n) {
      uint4 dv[UNR], xr[UNR], x2r[UNR];
      uint32_t mb[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u < n) {
          const size_t off = (size_t)(r + u * st) * C + c0;
          dv[u] = *(const uint4*)(dy + off);
          xr[u] = *(const uint4*)(x + off);
          x2r[u] = *(const uint4*)(x2 + off);
          mb[u] = ym[off / 8];
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (u >= n) break;
        float g[8], xv[8], x2v[8];
        unpack8(dv[u], g);
        unpack8(xr[u], xv);
        unpack8(x2r[u], x2v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gj = (mb[u] >> j) & 1u ? g[j] : 0.f;
          sg[j] += gj;
          sgx[j] += gj * (xv[j] - mu[j]) * rs[j];
          sgx2[j] += gj * (x2v[j] - mu2[j]) * rs2[j];
        }
      }
    });
  }
  block_reduce8(sg, cm, red);
  block_reduce8(sgx, cm, red);
  block_reduce8(sgx2, cm, red);
  if (cm.active && cm.r0 == 0) {
    float* row = slab + (size_t)blockIdx.x * 3 * C + cm.cc * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      row[j] = sg[j];
      row[C + j] = sgx[j];
      row[2 * C + j] = sgx2[j];
    }
  }
}

// dx = a*g + b + c*x, dx2 = a2*g + b2 + c2*x2; block 0 folds the sums into both BNs'
// dgamma / dbeta
template <int UNR>
__global__ __launch_bounds__(256) void bn_bwd_pair_apply_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ x2,
    const uint8_t* __restrict__ ym, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ mean2,
    const float* __restrict__ rstd2, const float* __restrict__ gamma2,
    const float* __restrict__ ws, float* __restrict__ dgamma, float* __restrict__ dbeta,
    float* __restrict__ dgamma2, float* __restrict__ dbeta2, int M, int C,
    bf16_t* __restrict__ dx, bf16_t* __restrict__ dx2) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  float a[8], b[8], cc[8], a2[8], b2[8], cc2[8];
  const float invM = 1.f / (float)M;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sg = ws[c0 + j], sgx = ws[C + c0 + j], sgx2 = ws[2 * C + c0 + j];
    const float rs = rstd[c0 + j], sc = gamma[c0 + j] * rs;
    a[j] = sc;
    cc[j] = -sc * rs * sgx * invM;
    b[j] = -sc * sg * invM - cc[j] * mean[c0 + j];
    const float rs2_ = rstd2[c0 + j], sc2 = gamma2[c0 + j] * rs2_;
    a2[j] = sc2;
    cc2[j] = -sc2 * rs2_ * sgx2 * invM;
    b2[j] = -sc2 * sg * invM - cc2[j] * mean2[c0 + j];
    if (blockIdx.x == 0 && cm.r0 == 0) {
      if (dgamma) dgamma[c0 + j] += sgx;
      if (dbeta) dbeta[c0 + j] += sg;
      if (dgamma2) dgamma2[c0 + j] += sgx2;
      if (dbeta2) dbeta2[c0 + j] += sg;
    }
  }
  sweep_rows_pl<UNR, 4>(
      cm, M,
      [&](int r, uint4 (&v)[4]) {
        const size_t off = (size_t)r * C + c0;
        v[0] = *(const uint4*)(dy + off);
        v[3].x = ym[off / 8];
        v[1] = *(const uint4*)(x + off);
        v[2] = *(const uint4*)(x2 + off);
      },
      [&](int r, uint4 (&v)[4]) {
        const size_t off = (size_t)r * C + c0;
        float g[8], xv[8], x2v[8];
        unpack8(v[0], g);
        unpack8(v[1], xv);
        unpack8(v[2], x2v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          g[j] = (v[3].x >> j) & 1u ? g[j] : 0.f;
          xv[j] = a[j] * g[j] + b[j] + cc[j] * xv[j];
          x2v[j] = a2[j] * g[j] + b2[j] + cc2[j] * x2v[j];
        }
        *(uint4*)(dx + off) = pack8(xv);
        *(uint4*)(dx2 + off) = pack8(x2v);
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
// out[w] += sum_s slab[s*W + w]; 64 columns x SG slab-row groups per block.  Each thread
// keeps eight independent partial sums, so eight slab loads are in flight per iteration:
// these kernels are latency-bound (a few hundred KiB just written by other XCDs, one add
// chain per thread), and with 16 row groups a 256-row slab takes two round trips instead
// of sixteen (slab_stats ~10 us -> ~3 us per BN layer).
constexpr int SG = 16;  // slab-row groups per block (blockDim = 64 * SG)
__device__ __forceinline__ float slab_col_sum(const float* __restrict__ slab, size_t rstride,
                                              int s0, int S, int step) {
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s_ = s0;
  for (; s_ + 7 * step < S; s_ += 8 * step) {
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] += slab[(size_t)(s_ + u * step) * rstride];
  }
  for (; s_ < S; s_ += step) a[0] += slab[(size_t)s_ * rstride];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// fixed-order sum of the SG groups' partials of column (threadIdx.x & 63) held in red[]
__device__ __forceinline__ float group_sum(const float* red, int t) {
  float v = 0.f;
#pragma unroll
  for (int g = 0; g < SG; ++g) v += red[g * 64 + t];
  return v;
}

__global__ __launch_bounds__(64 * SG) void slab_reduce_kernel(float* __restrict__ slab, int S,
                                                               int W, float* __restrict__ out,
                                                               int det) {
  __shared__ float red[64 * SG];
  const int w = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  float acc = 0.f;
  if (w < W) acc = slab_col_sum(slab + w, W, blockIdx.y * SG + g, S, gridDim.y * SG);
  red[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && w < W) {
    acc = group_sum(red, threadIdx.x);
    if (gridDim.y == 1) out[w] += acc;
    else if (det) slab[(size_t)blockIdx.y * SG * W + w] = acc;  // a row only this block read
    else atomicAdd(out + w, acc);
  }
}

// deterministic second pass: out[w] += the blocks' partials, in block order
__global__ __launch_bounds__(256) void slab_partials_kernel(const float* __restrict__ slab, int gy,
                                                            int W, float* __restrict__ out) {
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (w >= W) return;
  float a = 0.f;
  for (int y = 0; y < gy; ++y) a += slab[(size_t)y * SG * W + w];
  out[w] += a;
}

static bool g_det = [] {
  const char* e = getenv("MPA_DETERMINISTIC");
  return e && e[0] == '1';
}();
void set_deterministic(int on) { g_det = on != 0; }
bool deterministic() { return g_det; }

// out must hold its starting value (the producer kernels zero it in their first block
// when the reduction should start from 0; zero_out=true is only a fallback memset).
// Deterministic mode (MPA_DETERMINISTIC=1): the cross-block combine of a multi-block
// reduction is a fixed-order second pass over per-block partials (stored into the slab
// rows each block owns) instead of float atomics, whose order varies between launches.
void slab_reduce(const float* slab, int S, int W, float* out, bool zero_out, hipStream_t s) {
  if (zero_out) (void)hipMemsetAsync(out, 0, sizeof(float) * W, s);
  const int gy = std::max(1, std::min(32, (S + 255) / 256));
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((W + 63) / 64, gy), dim3(64 * SG), 0, s,
                     const_cast<float*>(slab), S, W, out, (int)g_det);
  if (gy > 1 && g_det)
    hipLaunchKernelGGL(slab_partials_kernel, dim3((W + 255) / 256), dim3(256), 0, s, slab, gy, W,
                       out);
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

// Statistics slab [S][2C] (rows of shifted (sum, sum of squares)) -> sums [2C] and the
// finalized [mean(C), biased var(C)], in ONE launch for slabs of <= 64 rows (the slab
// reduction and the finalize used to be two dependent launches per BN layer).  Larger
// slabs (the 3.2 M-pixel stem: 25,088 rows) first fold each chunk of `chunk` rows into
// the chunk's first row in place (deterministic, no atomics; every block owns its chunk),
// then the finalize kernel reads the chunk heads.  Thread (g, c) sums rows g, g+4, ... of
// columns c and C + c; the 4 groups combine through LDS in a fixed order.
__global__ __launch_bounds__(64 * SG) void slab_fold_kernel(float* __restrict__ slab, int S,
                                                             int W, int chunk) {
  __shared__ float red[64 * SG];
  const int w = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int r0 = blockIdx.y * chunk;
  const int r1 = min(S, r0 + chunk);
  float acc = 0.f;
  if (w < W) acc = slab_col_sum(slab + w, W, r0 + g, r1, SG);
  red[threadIdx.x] = acc;
  __syncthreads();
  if (g == 0 && w < W) slab[(size_t)r0 * W + w] = group_sum(red, threadIdx.x);
}

__global__ __launch_bounds__(64 * SG) void slab_stats_kernel(const float* __restrict__ slab,
                                                              int S, int rstep, int C,
                                                              const float* __restrict__ shift,
                                                              int M, float* __restrict__ sums,
                                                              float* __restrict__ out, int ld) {
  __shared__ float red[2][64 * SG];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const size_t W = 2 * (size_t)C;
  float a = 0.f, b = 0.f;
  if (c < C) {
    a = slab_col_sum(slab + c, W * rstep, g, S, SG);
    b = slab_col_sum(slab + C + c, W * rstep, g, S, SG);
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = b;
  __syncthreads();
  if (g == 0 && c < C) {
    const int t = threadIdx.x;
    a = group_sum(red[0], t);
    b = group_sum(red[1], t);
    sums[c] = a;
    sums[C + c] = b;
    const float inv = 1.f / (float)M;
    const float d = a * inv;  // mean of (x - K)
    const float k = shift ? shift[c] : 0.f;
    out[c] = k + d;
    out[ld + c] = fmaxf(b * inv - d * d, 0.f);
  }
}

void slab_stats(float* slab, int S, int C, const float* shift, int M, float* sums, float* out,
                hipStream_t s, int out_ld) {
  int rstep = 1, rows = S;
  if (S > 256) {  // fold to <= 64 chunk heads (one launch up to 256 rows: halo-conv slabs)
    const int chunk = (S + 63) / 64;
    rows = (S + chunk - 1) / chunk;
    rstep = chunk;
    hipLaunchKernelGGL(slab_fold_kernel, dim3((2 * C + 63) / 64, rows), dim3(64 * SG), 0, s, slab,
                       S, 2 * C, chunk);
  }
  hipLaunchKernelGGL(slab_stats_kernel, dim3((C + 63) / 64), dim3(64 * SG), 0, s, slab, rows,
                     rstep, C, shift, M, sums, out, out_ld > 0 ? out_ld : C);
}

// ----------------------------------------------- BN + ReLU + max-pool (network stems)
// conv -> BN -> ReLU -> max-pool (ResNet / DenseNet stems) as ONE pass over z: the BN
// output (411 MB for ResNet at batch 256) is never materialised.  Forward writes the pooled
// output and the window argmax; backward gathers the pooled gradient through the argmax
// and recomputes the ReLU mask from z (bn(z) > 0), so neither pass reads or writes the
// full-size activation gradient either.
struct PoolGeom {
  int N, H, W, P, Q, kh, kw, sh, sw, ph, pw;
};

__device__ __forceinline__ void bn_coeffs(const float* __restrict__ mean,
                                          const float* __restrict__ rstd,
                                          const float* __restrict__ gamma,
                                          const float* __restrict__ beta, int c0, float* sc,
                                          float* sh) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = gamma[c0 + j] * rstd[c0 + j];
    sh[j] = beta[c0 + j] - mean[c0 + j] * sc[j];
  }
}

// MODE 0: any window; 1: 3x3 / stride 2 / pad 1; 2: 3x3 / stride 2 / pad 0 (Inception's
// valid pools: every window lies inside the image, no clamp, no mask)
template <int MODE>
__global__ __launch_bounds__(256) void bn_relu_maxpool_fwd_kernel(
    const bf16_t* __restrict__ z, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, int C, PoolGeom g, bf16_t* __restrict__ y,
    uint8_t* __restrict__ idx, float* __restrict__ mean_out, float* __restrict__ rstd_out,
    unsigned long long* __restrict__ counter, bf16_t* __restrict__ zsel, int xmap) {
  if (counter && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(counter, 1ull);
  const ColMap cm = colmap(C / 8);
  // xmap (grid % 8 == 0): XCD x runs logical blocks [x G/8, (x+1) G/8), i.e. one contiguous
  // run of pooled rows per sweep, so the z row two vertically adjacent windows share is
  // fetched into one L2 (with the plain order, neighbouring blocks sit on different XCDs)
  const int xb = xmap ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  const int M = g.N * g.H * g.W;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float mu = stats[c0 + j], var = stats[C + c0 + j];
    const float rs = rsqrtf(var + eps);
    sc[j] = gamma[c0 + j] * rs;
    sh[j] = __builtin_fmaf(-mu, sc[j], beta[c0 + j]);
    if (blockIdx.x == 0 && cm.r0 == 0) {
      mean_out[c0 + j] = mu;
      rstd_out[c0 + j] = rs;
      const float unb = var * ((float)M / (float)max(M - 1, 1));
      rmean[c0 + j] = (1.f - momentum) * rmean[c0 + j] + momentum * mu;
      rvar[c0 + j] = (1.f - momentum) * rvar[c0 + j] + momentum * unb;
    }
  }
  const int MP = g.N * g.P * g.Q;
  // pooled output r -> (n, p, q), writes of (best, argmax, z at argmax)
  auto emit = [&](int r, const float* best, const int* bi, const float* bz) {
    const size_t o = (size_t)r * C + c0;
    *(uint4*)(y + o) = pack8(best);
    uint2 ib;
    ib.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    ib.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *(uint2*)(idx + o) = ib;
    if (zsel) *(uint4*)(zsel + o) = pack8(bz);  // bf16 -> f32 -> bf16: exact
  };
  for (int r = xb * cm.rpi + cm.r0; r < MP; r += gridDim.x * cm.rpi) {
    const int q = r % g.Q;
    const int t = r / g.Q;
    const int p = t % g.P;
    const int n = t / g.P;
    float best[8], bz[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; bi[j] = 0; bz[j] = 0.f; }
    if constexpr (MODE != 0) {
      // 3x3 / stride 2 / pad 1: all nine loads issued before any is consumed (out-of-range
      // taps read a clamped in-range pixel and are masked).  (Prefetching the next
      // output's nine loads ahead of this output's stores measured slower: 300 -> 384 us.)
      const int h0 = 2 * p - (MODE == 1 ? 1 : 0), w0 = 2 * q - (MODE == 1 ? 1 : 0);
      uint4 v9[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int h = min(max(h0 + i, 0), g.H - 1), w = min(max(w0 + k, 0), g.W - 1);
          v9[i * 3 + k] = *(const uint4*)(z + (((size_t)n * g.H + h) * g.W + w) * C + c0);
        }
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const bool ok = MODE == 2 ||
                          ((unsigned)(h0 + i) < (unsigned)g.H && (unsigned)(w0 + k) < (unsigned)g.W);
          float f[8];
          unpack8(v9[i * 3 + k], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float v = fmaxf(f[j] * sc[j] + sh[j], 0.f);
            if (ok && v > best[j]) { best[j] = v; bi[j] = i * 3 + k; bz[j] = f[j]; }
          }
        }
    } else {
      const int h0 = p * g.sh - g.ph, w0 = q * g.sw - g.pw;
      for (int i = 0; i < g.kh; ++i) {
        const int h = h0 + i;
        if ((unsigned)h >= (unsigned)g.H) continue;
        for (int k = 0; k < g.kw; ++k) {
          const int w = w0 + k;
          if ((unsigned)w >= (unsigned)g.W) continue;
          float f[8];
          unpack8(*(const uint4*)(z + (((size_t)n * g.H + h) * g.W + w) * C + c0), f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float v = fmaxf(f[j] * sc[j] + sh[j], 0.f);
            if (v > best[j]) { best[j] = v; bi[j] = i * g.kw + k; bz[j] = f[j]; }
          }
        }
      }
    }
    // a window whose every tap is ReLU-dead (best == 0) passes no gradient: its argmax byte
    // is 255, which no backward tap comparison matches - the pooled weight gradient then
    // needs no ReLU mask per pixel (stem_pool_wgrad)
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(best[j] > 0.f)) bi[j] = 255;
    emit(r, best, bi, bz);
  }
}

// Backward reduction of the fused stem from POOLED tensors only: the pool gradient reaches
// input pixel (n,h,w,c) only from windows whose argmax it is, and the ReLU mask there is
// bn(z_argmax) > 0, so  sum_pixels g = sum_windows dp * [bn(zsel) > 0]  and
// sum_pixels g * xhat = sum_windows dp * [bn(zsel) > 0] * xhat(zsel), with zsel the raw conv
// output at each window's argmax (saved by the forward).  Reads dp + zsel (2 x pooled size)
// instead of z + dp + idx (4 x + 1.5 x pooled size for a 3x3/s2 stem).
__global__ __launch_bounds__(256) void maxpool_bn_bwd_sel_reduce_kernel(
    const bf16_t* __restrict__ dp, const bf16_t* __restrict__ zsel,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int C, int MP,
    float* __restrict__ slab, float* __restrict__ sums) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sgx[j] = 0.f; }
  if (cm.active) {
    const int c0 = cm.cc * 8;
    if (blockIdx.x == 0 && cm.r0 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sums[c0 + j] = 0.f; sums[C + c0 + j] = 0.f; }
    }
    float sc[8], sh[8], mu[8], rs[8];
    bn_coeffs(mean, rstd, gamma, beta, c0, sc, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
#pragma unroll 2
    for (int r = blockIdx.x * cm.rpi + cm.r0; r < MP; r += gridDim.x * cm.rpi) {
      const size_t o = (size_t)r * C + c0;
      float d[8], zr[8];
      unpack8(*(const uint4*)(dp + o), d);
      unpack8(*(const uint4*)(zsel + o), zr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gr = (zr[j] * sc[j] + sh[j] > 0.f) ? d[j] : 0.f;
        sg[j] += gr;
        sgx[j] += gr * (zr[j] - mu[j]) * rs[j];
      }
    }
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

// gradient at input pixel (n, h, w): pooled gradients whose argmax is this pixel, times
// the ReLU mask bn(z) > 0; also returns z
__device__ __forceinline__ void pool_bn_grad(const bf16_t* __restrict__ dp,
                                             const uint8_t* __restrict__ idx,
                                             const bf16_t* __restrict__ z, int C, int c0,
                                             const PoolGeom& g, int r, const float* sc,
                                             const float* sh, float* gr, float* zr) {
  const int w = r % g.W;
  const int t = r / g.W;
  const int h = t % g.H;
  const int n = t / g.H;
#pragma unroll
  for (int j = 0; j < 8; ++j) gr[j] = 0.f;
  const int plo = max(0, (h + g.ph - g.kh + g.sh) / g.sh), phi = min(g.P - 1, (h + g.ph) / g.sh);
  const int qlo = max(0, (w + g.pw - g.kw + g.sw) / g.sw), qhi = min(g.Q - 1, (w + g.pw) / g.sw);
  for (int p = plo; p <= phi; ++p) {
    const int i = h - (p * g.sh - g.ph);
    if (i < 0 || i >= g.kh) continue;
    for (int q = qlo; q <= qhi; ++q) {
      const int k = w - (q * g.sw - g.pw);
      if (k < 0 || k >= g.kw) continue;
      const size_t o = (((size_t)n * g.P + p) * g.Q + q) * C + c0;
      const uint2 ib = *(const uint2*)(idx + o);
      const int me = i * g.kw + k;
      float d[8];
      unpack8(*(const uint4*)(dp + o), d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t word = j < 4 ? ib.x : ib.y;
        if ((int)((word >> (8 * (j & 3))) & 0xff) == me) gr[j] += d[j];
      }
    }
  }
  unpack8(*(const uint4*)(z + (size_t)r * C + c0), zr);
#pragma unroll
  for (int j = 0; j < 8; ++j) gr[j] = (zr[j] * sc[j] + sh[j] > 0.f) ? gr[j] : 0.f;
}

__global__ __launch_bounds__(256) void maxpool_bn_bwd_reduce_kernel(
    const bf16_t* __restrict__ dp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int C, PoolGeom g,
    float* __restrict__ slab, float* __restrict__ sums) {
  __shared__ float red[256 * 8];
  const ColMap cm = colmap(C / 8);
  float sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sgx[j] = 0.f; }
  if (cm.active) {
    const int c0 = cm.cc * 8;
    if (blockIdx.x == 0 && cm.r0 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { sums[c0 + j] = 0.f; sums[C + c0 + j] = 0.f; }
    }
    float sc[8], sh[8], mu[8], rs[8];
    bn_coeffs(mean, rstd, gamma, beta, c0, sc, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
    const int M = g.N * g.H * g.W;
    for (int r = blockIdx.x * cm.rpi + cm.r0; r < M; r += gridDim.x * cm.rpi) {
      float gr[8], zr[8];
      pool_bn_grad(dp, idx, z, C, c0, g, r, sc, sh, gr, zr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg[j] += gr[j];
        sgx[j] += gr[j] * (zr[j] - mu[j]) * rs[j];
      }
    }
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

__global__ __launch_bounds__(256) void maxpool_bn_bwd_apply_kernel(
    const bf16_t* __restrict__ dp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ sums, float* __restrict__ dgamma, float* __restrict__ dbeta, int C,
    PoolGeom g, bf16_t* __restrict__ dz) {
  const ColMap cm = colmap(C / 8);
  if (!cm.active) return;
  const int c0 = cm.cc * 8;
  const int M = g.N * g.H * g.W;
  float sc[8], sh[8], a[8], b[8], cco[8];
  bn_coeffs(mean, rstd, gamma, beta, c0, sc, sh);
  const float invM = 1.f / (float)M;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sgv = sums[c0 + j], sgx = sums[C + c0 + j];
    const float rs = rstd[c0 + j];
    a[j] = sc[j];
    cco[j] = -sc[j] * rs * sgx * invM;
    b[j] = -sc[j] * sgv * invM - cco[j] * mean[c0 + j];
    if (blockIdx.x == 0 && cm.r0 == 0) {
      if (dgamma) dgamma[c0 + j] += sgx;
      if (dbeta) dbeta[c0 + j] += sgv;
    }
  }
  for (int r = blockIdx.x * cm.rpi + cm.r0; r < M; r += gridDim.x * cm.rpi) {
    float gr[8], zr[8];
    pool_bn_grad(dp, idx, z, C, c0, g, r, sc, sh, gr, zr);
#pragma unroll
    for (int j = 0; j < 8; ++j) zr[j] = a[j] * gr[j] + b[j] + cco[j] * zr[j];
    *(uint4*)(dz + (size_t)r * C + c0) = pack8(zr);
  }
}

// 3x3 / stride 2 pool, thread = one 2x2 input cell (2p..2p+1, 2q..2q+1) x 8 channels.
// PAD 1 over an even H x W (H == 2P, W == 2Q; ResNet / DenseNet stems): row 2p is covered
// only by window row p (tap 1), row 2p+1 by window p (tap 2) and p+1 (tap 0), so the cell
// needs the pooled positions (p|p+1, q|q+1).  PAD 0 over H == 2P+1, W == 2Q+1 (Inception's
// valid pools): row 2p by window p (tap 0) and p-1 (tap 2), row 2p+1 by window p (tap 1)
// only; cells run over (P+1) x (Q+1) so the last row / column (2P, 2Q) is covered, and the
// pooled positions are (p-1|p, q-1|q).  Every load is independent.
// APPLY = false: reduce (sum g, sum g*xhat) into the slab; true: write dz.
template <bool APPLY, int PAD = 1>
__global__ __launch_bounds__(256) void maxpool_bn_bwd_cell_kernel(
    const bf16_t* __restrict__ dp, const uint8_t* __restrict__ idx, const bf16_t* __restrict__ z,
    const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ sums, float* __restrict__ dgamma, float* __restrict__ dbeta, int C,
    PoolGeom g, float* __restrict__ slab, float* __restrict__ zsums, bf16_t* __restrict__ dz) {
  __shared__ float red[APPLY ? 1 : 256 * 8];
  const ColMap cm = colmap(C / 8);
  float sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sg[j] = 0.f; sgx[j] = 0.f; }
  if (cm.active) {
    const int c0 = cm.cc * 8;
    float sc[8], sh[8], mu[8], rs[8], a[8], b[8], cco[8];
    bn_coeffs(mean, rstd, gamma, beta, c0, sc, sh);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = mean[c0 + j]; rs[j] = rstd[c0 + j]; }
    if constexpr (APPLY) {
      const float invM = 1.f / (float)(g.N * g.H * g.W);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sgv = sums[c0 + j], sgxv = sums[C + c0 + j];
        a[j] = sc[j];
        cco[j] = -sc[j] * rs[j] * sgxv * invM;
        b[j] = -sc[j] * sgv * invM - cco[j] * mu[j];
        if (blockIdx.x == 0 && cm.r0 == 0) {
          if (dgamma) dgamma[c0 + j] += sgxv;
          if (dbeta) dbeta[c0 + j] += sgv;
        }
      }
    } else if (blockIdx.x == 0 && cm.r0 == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) { zsums[c0 + j] = 0.f; zsums[C + c0 + j] = 0.f; }
    }
    // cell grid: P x Q (PAD 1) or (P+1) x (Q+1) (PAD 0)
    const int CP = g.P + (PAD ? 0 : 1), CQ = g.Q + (PAD ? 0 : 1);
    const int cells = g.N * CP * CQ;
    // pooled neighbours (dp, idx) at window rows p + dp0 + (u >> 1), cols q + dq0 + (u & 1)
    // with dp0 = dq0 = 0 (PAD 1) or -1 (PAD 0); out-of-range neighbours load an in-range
    // one and are masked in proc.  Register image per cell: dp 0..3, idx pairs 4..5, z 6..9
    // (pixels past the image load a clamped one, never stored).  The next cell's loads are
    // issued before this cell's dz stores (sweep_rows_pl: a load after a store would wait
    // for the store in the in-order vmcnt).
    constexpr int D0 = PAD ? 0 : -1;
    auto nb_ok = [&](int p, int q, int u) {
      const int pp = p + D0 + (u >> 1), qq = q + D0 + (u & 1);
      return (unsigned)pp < (unsigned)g.P && (unsigned)qq < (unsigned)g.Q;
    };
    auto load = [&](int r, uint4 (&v)[10]) {
      const int q = r % CQ, t = r / CQ, p = t % CP, n = t / CP;
      uint2 iv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bool ok = nb_ok(p, q, u);
        const int pp = ok ? p + D0 + (u >> 1) : min(p, g.P - 1);
        const int qq = ok ? q + D0 + (u & 1) : min(q, g.Q - 1);
        const size_t o = (((size_t)n * g.P + pp) * g.Q + qq) * C + c0;
        v[u] = *(const uint4*)(dp + o);
        iv[u] = *(const uint2*)(idx + o);
      }
      v[4] = make_uint4(iv[0].x, iv[0].y, iv[1].x, iv[1].y);
      v[5] = make_uint4(iv[2].x, iv[2].y, iv[3].x, iv[3].y);
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const int h = min(2 * p + (w4 >> 1), g.H - 1), w = min(2 * q + (w4 & 1), g.W - 1);
        v[6 + w4] = *(const uint4*)(z + (((size_t)n * g.H + h) * g.W + w) * C + c0);
      }
    };
    auto proc = [&](int r, uint4 (&v)[10]) {
      const int q = r % CQ, t = r / CQ, p = t % CP, n = t / CP;
      uint2 iv[4] = {make_uint2(v[4].x, v[4].y), make_uint2(v[4].z, v[4].w),
                     make_uint2(v[5].x, v[5].y), make_uint2(v[5].z, v[5].w)};
      float d[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (!nb_ok(p, q, u)) iv[u] = make_uint2(~0u, ~0u);  // argmax 255 never matches a tap
        unpack8(v[u], d[u]);
      }
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const int a0 = w4 >> 1, b0 = w4 & 1;  // input pixel (2p+a0, 2q+b0)
        if (2 * p + a0 >= g.H || 2 * q + b0 >= g.W) continue;  // PAD 0: past the last row
        float zr[8], gr[8];
        unpack8(v[6 + w4], zr);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float acc = 0.f;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int du = u >> 1, eu = u & 1;
            int ti, tk;
            if constexpr (PAD) {
              // rows {p: tap 1+a0} (+ {p+1: tap 0} if a0), cols likewise
              if ((du && !a0) || (eu && !b0)) continue;
              ti = du ? 0 : 1 + a0;
              tk = eu ? 0 : 1 + b0;
            } else {
              // rows {p: tap a0} (+ {p-1: tap 2} if !a0), cols likewise
              if ((!du && a0) || (!eu && b0)) continue;
              ti = du ? a0 : 2;
              tk = eu ? b0 : 2;
            }
            const uint32_t word = j < 4 ? iv[u].x : iv[u].y;
            if ((int)((word >> (8 * (j & 3))) & 0xff) == ti * 3 + tk) acc += d[u][j];
          }
          gr[j] = (zr[j] * sc[j] + sh[j] > 0.f) ? acc : 0.f;
        }
        if constexpr (APPLY) {
#pragma unroll
          for (int j = 0; j < 8; ++j) zr[j] = a[j] * gr[j] + b[j] + cco[j] * zr[j];
          const int h = 2 * p + a0, w = 2 * q + b0;
          *(uint4*)(dz + (((size_t)n * g.H + h) * g.W + w) * C + c0) = pack8(zr);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            sg[j] += gr[j];
            sgx[j] += gr[j] * (zr[j] - mu[j]) * rs[j];
          }
        }
      }
    };
    sweep_rows_pl<1, 10>(cm, cells, load, proc);
  }
  if constexpr (!APPLY) {
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
}

static bool pool_k3s2p1_even(const PoolGeom& g) {
  return g.kh == 3 && g.kw == 3 && g.sh == 2 && g.sw == 2 && g.ph == 1 && g.pw == 1 &&
         g.H == 2 * g.P && g.W == 2 * g.Q;
}

static bool pool_k3s2p0_odd(const PoolGeom& g) {
  return g.kh == 3 && g.kw == 3 && g.sh == 2 && g.sw == 2 && g.ph == 0 && g.pw == 0 &&
         g.H == 2 * g.P + 1 && g.W == 2 * g.Q + 1;
}

// --------------------------------------- deferred BN-backward corrections (DenseNet)
// A dense block's norm1 layers all normalise channel c with the SAME batch statistics (the
// block table, taken once when the feature is produced), so their backward terms
//   dx_i = a_i g_i - a_i mean(g_i) - a_i mean(g_i xhat) xhat,   a_i = gamma_i rstd
// split into a per-layer local part a_i g_i - added into the block gradient G by the
// consumer conv's dgrad epilogue (ep_gacc) - and per-channel constants that SUM over layers:
//   K1[c] = -sum_i a_i mean(g_i),  K2[c] = -sum_i a_i mean(g_i xhat),
// applied once per channel as G += K1 + K2 xhat when the channel's gradient is complete.
// One launch after layer i's dgrad: block 0 folds layer i's sums into K (channels < s0) and
// the (gamma, beta) gradients; every block applies the now-final correction (K plus layer
// i's own term) to the channels [s0, Ci) no later layer reads (layer i-1's 32 outputs, or
// the block input for i = 0).  Thread = 8 channels x rows strided by the grid.
template <bool F32>
__global__ __launch_bounds__(256) void bn_defer_step_kernel(
    const float* __restrict__ sums, const float* __restrict__ gamma,
    const float* __restrict__ mean, const float* __restrict__ rstd, int Ci, int s0, int M,
    float invM, float* __restrict__ k12, int ldk, float* __restrict__ dgamma,
    float* __restrict__ dbeta, void* __restrict__ G, int ldg, const bf16_t* __restrict__ x,
    int ldx, bf16_t* __restrict__ out) {
  if (blockIdx.x == 0) {
    for (int c = threadIdx.x; c < Ci; c += 256) {
      const float sg = sums[c], sgx = sums[Ci + c];
      if (dgamma) dgamma[c] += sgx;
      if (dbeta) dbeta[c] += sg;
      if (c < s0) {
        const float a = gamma[c] * rstd[c];
        k12[c] -= a * sg * invM;
        k12[ldk + c] -= a * sgx * invM;
      }
    }
  }
  const int cg = (Ci - s0) / 8, rpp = 256 / cg;  // host: 256 % cg == 0
  const int c0 = s0 + (threadIdx.x % cg) * 8;
  float k1[8], k2[8], mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    const float a = gamma[c] * rstd[c];
    k1[j] = k12[c] - a * sums[c] * invM;
    k2[j] = k12[ldk + c] - a * sums[Ci + c] * invM;
    mu[j] = mean[c];
    rs[j] = rstd[c];
  }
  const int rstep = gridDim.x * rpp;
  if constexpr (F32) {
    for (int m = blockIdx.x * rpp + (int)threadIdx.x / cg; m < M; m += rstep) {
      float xv[8];
      unpack8(*(const uint4*)(x + (size_t)m * ldx + c0), xv);
      float d[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = k1[j] + k2[j] * ((xv[j] - mu[j]) * rs[j]);
      f32x4* gp = (f32x4*)((float*)G + (size_t)m * ldg + c0);
      f32x4 g0 = gp[0], g1 = gp[1];
#pragma unroll
      for (int j = 0; j < 4; ++j) { g0[j] += d[j]; g1[j] += d[4 + j]; }
      if (out) {  // the finished slice goes to its consumer only: G's copy is never read again
        float gv[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        *(uint4*)(out + (size_t)m * (Ci - s0) + (c0 - s0)) = pack8(gv);
      } else {
        gp[0] = g0;
        gp[1] = g1;
      }
    }
  } else {
    // two rows per iteration, both rows' loads issued before either is used
    auto fin = [&](int m, uint4 xq, uint4 gq) {
      float xv[8], gv[8];
      unpack8(xq, xv);
      unpack8(gq, gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] += k1[j] + k2[j] * ((xv[j] - mu[j]) * rs[j]);
      const uint4 pk = pack8(gv);
      if (out) *(uint4*)(out + (size_t)m * (Ci - s0) + (c0 - s0)) = pk;
      else *(uint4*)((bf16_t*)G + (size_t)m * ldg + c0) = pk;
    };
    for (int m = blockIdx.x * rpp + (int)threadIdx.x / cg; m < M; m += 2 * rstep) {
      const int m2 = m + rstep;
      const uint4 xa = *(const uint4*)(x + (size_t)m * ldx + c0);
      const uint4 ga = *(const uint4*)((const bf16_t*)G + (size_t)m * ldg + c0);
      uint4 xb = make_uint4(0u, 0u, 0u, 0u), gb = xb;
      if (m2 < M) {
        xb = *(const uint4*)(x + (size_t)m2 * ldx + c0);
        gb = *(const uint4*)((const bf16_t*)G + (size_t)m2 * ldg + c0);
      }
      fin(m, xa, ga);
      if (m2 < M) fin(m2, xb, gb);
    }
  }
}

// ------------------------------------------------------------------------ launchers
void bn_stats(const bf16_raw* x, int M, int C, const float* shift, float* stats, float* ws,
              hipStream_t s) {
  const dim3 g = grid_for(M, C);
  float* sums = ws + (int64_t)g.x * 2 * C;
  BN_LAUNCH(bn_stats_kernel, g, s, x, M, C, shift, ws, sums);
  slab_stats(ws, g.x, C, shift, M, sums, stats, s);
}

void bn_fwd_train(const bf16_raw* x, const float* stats, const float* gamma, const float* beta,
                  float* rmean, float* rvar, float momentum, float eps, const bf16_raw* res,
                  int relu, int M, int C, bf16_raw* y, float* mean, float* rstd,
                  int64_t* counter, hipStream_t s, uint8_t* ymask, int ldx, int lds,
                  const float* res_aff, int ldy) {
  if (ldx <= 0) ldx = C;
  if (lds <= 0) lds = C;
  if (ldy <= 0) ldy = C;
  if (ymask)
    BN_LAUNCH_T(bn_fwd_train_kernel, true, grid_for(M, C), s, x, stats, gamma, beta, rmean, rvar,
                momentum, eps, res, relu, M, C, y, mean, rstd, (unsigned long long*)counter, ymask,
                ldx, lds, res_aff, ldy);
  else
    BN_LAUNCH_T(bn_fwd_train_kernel, false, grid_for(M, C), s, x, stats, gamma, beta, rmean, rvar,
                momentum, eps, res, relu, M, C, y, mean, rstd, (unsigned long long*)counter, ymask,
                ldx, lds, res_aff, ldy);
}

void bn_stats_affine(const float* stats, const float* gamma, const float* beta, float* rmean,
                     float* rvar, float momentum, float eps, int M, int C, float* mean,
                     float* rstd, float* aff, int64_t* counter, hipStream_t s) {
  hipLaunchKernelGGL(bn_stats_affine_kernel, dim3((C + 255) / 256), dim3(256), 0, s, stats,
                     gamma, beta, rmean, rvar, momentum, eps, M, C, mean, rstd, aff,
                     (unsigned long long*)counter);
}

void affine_act(const bf16_raw* x, const float* aff, int relu, int M, int C, bf16_raw* y,
                hipStream_t s) {
  BN_LAUNCH(affine_act_kernel, grid_for(M, C), s, (const bf16_t*)x, aff, relu, M, C, (bf16_t*)y);
}

void bn_fwd_eval(const bf16_raw* x, const float* gamma, const float* beta, const float* rmean,
                 const float* rvar, float eps, const bf16_raw* res, int relu, int M, int C,
                 bf16_raw* y, hipStream_t s, int ldx) {
  BN_LAUNCH(bn_fwd_eval_kernel, grid_for(M, C), s, x, gamma, beta, rmean,
                     rvar, eps, res, relu, M, C, y, ldx > 0 ? ldx : C);
}

void bn_bwd(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
            const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M, int C,
            bf16_raw* dx, bf16_raw* g, float* ws, hipStream_t s, const float* zmask_beta,
            const uint8_t* ymask, int ldx, float* gacc, int ldg, int lddx, bool gacc_bf16,
            int lddy) {
  // ws layout: [2C] final sums | [gx][2C] per-block partials
  if (ldx <= 0) ldx = C;
  if (lddx <= 0) lddx = C;
  if (lddy <= 0) lddy = C;
  const dim3 gr = grid_for(M, C);
  float* slab = ws + 2 * C;
  const float* zb = (y || ymask) ? nullptr : zmask_beta;
  if (ymask) y = nullptr;
  BN_LAUNCH(bn_bwd_reduce_kernel, gr, s, dy, x, y, mean, rstd, gamma, zb, M, C, slab, ws, ymask,
            ldx, lddy);
  slab_reduce(slab, gr.x, 2 * C, ws, false, s);
  if (gacc) {  // dense-block accumulator: dx added into gacc (no ymask, no g)
    const dim3 ga = grid_for(M, C);
#define BN_ACC_LAUNCH(U, A)                                                                 \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<U, false, A>), ga, dim3(256), 0, s, dy, x, y, mean, \
                     rstd, gamma, zb, ws, dgamma, dbeta, M, C, (bf16_t*)nullptr,             \
                     (bf16_t*)nullptr, (const uint8_t*)nullptr, ldx, gacc, ldg, C, lddy)
    if (gacc_bf16) BN_ACC_LAUNCH(2, 2);
    else BN_ACC_LAUNCH(2, 1);
#undef BN_ACC_LAUNCH
  } else if (ymask)
    BN_LAUNCH_T(bn_bwd_apply_kernel, true, grid_for(M, C), s, dy, x, y, mean, rstd, gamma, zb, ws,
                dgamma, dbeta, M, C, dx, g, ymask, ldx, (float*)nullptr, 0, lddx, lddy);
  else
    BN_LAUNCH_T(bn_bwd_apply_kernel, false, grid_for(M, C), s, dy, x, y, mean, rstd, gamma, zb,
                ws, dgamma, dbeta, M, C, dx, g, ymask, ldx, (float*)nullptr, 0, lddx, lddy);
}

// apply pass only, with the reduction sums [sum g | sum g*xhat] already in `sums` (e.g.
// from the fused dgrad epilogue, igemm_rows_dgrad_bnred)
void bn_bwd_apply(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
                  const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M,
                  int C, bf16_raw* dx, bf16_raw* g, const float* sums, hipStream_t s, int lddy) {
  if (lddy <= 0) lddy = C;
  BN_LAUNCH_T(bn_bwd_apply_kernel, false, grid_for(M, C), s, dy, x, y, mean, rstd, gamma,
              (const float*)nullptr, sums, dgamma, dbeta, M, C, dx, g, (const uint8_t*)nullptr, C,
              (float*)nullptr, 0, C, lddy);
}


bool maxpool2_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw) {
  return kh == 2 && kw == 2 && sh == 2 && sw == 2 && ph == 0 && pw == 0 && H % 2 == 0 &&
         W % 2 == 0 && C % 8 == 0 && (int64_t)N * H * W * C < (1ll << 31);
}

void maxpool2_fwd(const bf16_raw* x, int N, int H, int W, int C, bf16_raw* y, uint8_t* idx,
                  hipStream_t s) {
  const int NP = N * (H / 2), Q = W / 2;
  const int64_t total = (int64_t)NP * Q * (C / 8);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
  hipLaunchKernelGGL(maxpool2_fwd_kernel, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, NP, Q, C,
                     (bf16_t*)y, idx);
}

int64_t maxpool2_ws_floats(int N, int H, int W, int C) {
  return (int64_t)(grid_for(N * (H / 2) * (W / 2), C).x + 1) * C;
}

void maxpool2_bwd(const bf16_raw* dy, const uint8_t* idx, const bf16_raw* yp, int N, int H, int W,
                  int C, bf16_raw* dx, float* sums, float* ws, hipStream_t s) {
  const int NP = N * (H / 2), Q = W / 2;
  const dim3 gr = grid_for(NP * Q, C);
  if (yp && sums) {
    float* slab = ws;
    hipLaunchKernelGGL(maxpool2_bwd_kernel<true>, gr, dim3(256), 0, s, (const bf16_t*)dy, idx,
                       (const bf16_t*)yp, NP, Q, C, (bf16_t*)dx, slab, sums);
    slab_reduce(slab, gr.x, C, sums, false, s);
  } else {
    hipLaunchKernelGGL(maxpool2_bwd_kernel<false>, gr, dim3(256), 0, s, (const bf16_t*)dy, idx,
                       (const bf16_t*)nullptr, NP, Q, C, (bf16_t*)dx, (float*)nullptr,
                       (float*)nullptr);
  }
}

int64_t bn_pair_ws_floats(int M, int C) { return (int64_t)3 * C * (1 + grid_for(M, C).x); }

void bn_bwd_pair(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* x2, const uint8_t* ymask,
                 const float* mean, const float* rstd, const float* gamma, const float* mean2,
                 const float* rstd2, const float* gamma2, float* dgamma, float* dbeta,
                 float* dgamma2, float* dbeta2, int M, int C, bf16_raw* dx, bf16_raw* dx2,
                 float* ws, hipStream_t s) {
  // ws layout: [3C] final sums | [gx][3C] per-block partials
  const dim3 gr = grid_for(M, C);
  float* slab = ws + 3 * C;
  BN_LAUNCH(bn_bwd_pair_reduce_kernel, gr, s, dy, x, x2, ymask, mean, rstd, mean2, rstd2, M, C,
            slab, ws);
  slab_reduce(slab, gr.x, 3 * C, ws, false, s);
  BN_LAUNCH(bn_bwd_pair_apply_kernel, gr, s, dy, x, x2, ymask, mean, rstd, gamma, mean2, rstd2,
            gamma2, ws, dgamma, dbeta, dgamma2, dbeta2, M, C, dx, dx2);
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

// grid targets of the fused stem kernels (forward, backward reduce, backward apply); the
// gathers are latency-bound, so they want more waves in flight than the streaming passes
static int stem_grid(int which) {
  static const int v[3] = {1024, 1024, 4096};
  return v[which];
}

void bn_relu_maxpool_fwd(const bf16_raw* z, const float* stats, const float* gamma,
                         const float* beta, float* rmean, float* rvar, float momentum, float eps,
                         int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                         int ph, int pw, bf16_raw* y, uint8_t* idx, float* mean, float* rstd,
                         int64_t* counter, hipStream_t s, bf16_raw* zsel) {
  const PoolGeom g{N, H, W, P, Q, kh, kw, sh, sw, ph, pw};
  const bool k3 = kh == 3 && kw == 3 && sh == 2 && sw == 2;
  const int mode = (k3 && ph == 1 && pw == 1) ? 1
                   : (k3 && ph == 0 && pw == 0 && 2 * P + 1 <= H && 2 * Q + 1 <= W) ? 2 : 0;
  const dim3 grid = grid_for(N * P * Q, C, stem_grid(0));
  // (XCD-contiguous order: step time neutral, 4 alternating runs, profiles/halo_wxmap_r6.txt)
  const int xmap = grid.x % 8 == 0;
  hipLaunchKernelGGL(mode == 1   ? bn_relu_maxpool_fwd_kernel<1>
                     : mode == 2 ? bn_relu_maxpool_fwd_kernel<2>
                                 : bn_relu_maxpool_fwd_kernel<0>,
                     grid, dim3(256), 0, s, z, stats, gamma, beta,
                     rmean, rvar, momentum, eps, C, g, y, idx, mean, rstd,
                     (unsigned long long*)counter, zsel, xmap);
}

__global__ void bn_sums_grad_kernel(const float* __restrict__ sums, int C,
                                    float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dgamma) dgamma[c] += sums[C + c];
  if (dbeta) dbeta[c] += sums[c];
}

// the fused stem backward's pooled-only half: (sum g, sum g xhat) into ws[0 .. 2C) and the
// (gamma, beta) gradients; the dz pass itself runs inside the stem weight gradient
// (stem_pool_wgrad, conv_stem.hip)
void maxpool_bn_bwd_sums(const bf16_raw* dp, const bf16_raw* zsel, const float* mean,
                         const float* rstd, const float* gamma, const float* beta, float* dgamma,
                         float* dbeta, int MP, int C, float* ws, hipStream_t s) {
  float* slab = ws + 2 * C;
  const dim3 gr = grid_for(MP, C, stem_grid(1));
  hipLaunchKernelGGL(maxpool_bn_bwd_sel_reduce_kernel, gr, dim3(256), 0, s, dp, zsel, mean, rstd,
                     gamma, beta, C, MP, slab, ws);
  slab_reduce(slab, gr.x, 2 * C, ws, false, s);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(bn_sums_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, C, dgamma,
                       dbeta);
}

int64_t maxpool_bn_ws_floats(int M, int C) {
  return (int64_t)grid_for(M, C, stem_grid(1)).x * 2 * C + 2 * C;
}

void maxpool_bn_bwd(const bf16_raw* dp, const uint8_t* idx, const bf16_raw* z, const float* mean,
                    const float* rstd, const float* gamma, const float* beta, float* dgamma,
                    float* dbeta, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh,
                    int sw, int ph, int pw, bf16_raw* dz, float* ws, hipStream_t s,
                    const bf16_raw* zsel) {
  // ws layout: [2C] final sums | [gx][2C] per-block partials (as bn_bwd)
  const PoolGeom g{N, H, W, P, Q, kh, kw, sh, sw, ph, pw};
  const int M = N * H * W;
  float* slab = ws + 2 * C;
  bool reduced = false;
  if (zsel) {
    const dim3 gr = grid_for(N * P * Q, C, stem_grid(1));
    hipLaunchKernelGGL(maxpool_bn_bwd_sel_reduce_kernel, gr, dim3(256), 0, s, dp, zsel, mean,
                       rstd, gamma, beta, C, N * P * Q, slab, ws);
    slab_reduce(slab, gr.x, 2 * C, ws, false, s);
    reduced = true;
  }
  if (pool_k3s2p1_even(g)) {
    const int cells = N * P * Q;
    if (!reduced) {
      const dim3 gr = grid_for(cells, C, stem_grid(1));
      hipLaunchKernelGGL(maxpool_bn_bwd_cell_kernel<false>, gr, dim3(256), 0, s, dp, idx, z, mean,
                         rstd, gamma, beta, nullptr, nullptr, nullptr, C, g, slab, ws, nullptr);
      slab_reduce(slab, gr.x, 2 * C, ws, false, s);
    }
    hipLaunchKernelGGL(maxpool_bn_bwd_cell_kernel<true>, grid_for(cells, C, stem_grid(2)),
                       dim3(256), 0, s, dp, idx, z, mean, rstd, gamma, beta, ws, dgamma, dbeta, C,
                       g, nullptr, nullptr, dz);
    return;
  }
  if (pool_k3s2p0_odd(g)) {
    const int cells = N * (P + 1) * (Q + 1);
    if (!reduced) {
      const dim3 gr = grid_for(cells, C, stem_grid(1));
      hipLaunchKernelGGL((maxpool_bn_bwd_cell_kernel<false, 0>), gr, dim3(256), 0, s, dp, idx, z,
                         mean, rstd, gamma, beta, nullptr, nullptr, nullptr, C, g, slab, ws,
                         nullptr);
      slab_reduce(slab, gr.x, 2 * C, ws, false, s);
    }
    hipLaunchKernelGGL((maxpool_bn_bwd_cell_kernel<true, 0>), grid_for(cells, C, stem_grid(2)),
                       dim3(256), 0, s, dp, idx, z, mean, rstd, gamma, beta, ws, dgamma, dbeta, C,
                       g, nullptr, nullptr, dz);
    return;
  }
  if (!reduced) {
    const dim3 gr = grid_for(M, C, stem_grid(1));
    hipLaunchKernelGGL(maxpool_bn_bwd_reduce_kernel, gr, dim3(256), 0, s, dp, idx, z, mean, rstd,
                       gamma, beta, C, g, slab, ws);
    slab_reduce(slab, gr.x, 2 * C, ws, false, s);
  }
  hipLaunchKernelGGL(maxpool_bn_bwd_apply_kernel, grid_for(M, C, stem_grid(2)), dim3(256), 0, s, dp, idx, z,
                     mean, rstd, gamma, beta, ws, dgamma, dbeta, C, g, dz);
}

}  // namespace mpa

namespace mpa {
void bn_defer_step(const float* sums, const float* gamma, const float* mean, const float* rstd,
                   int Ci, int s0, int M, float* k12, int ldk, float* dgamma, float* dbeta,
                   void* G, bool g_f32, int ldg, const bf16_raw* x, int ldx, bf16_raw* out,
                   hipStream_t s) {
  const int cg = (Ci - s0) / 8, rpp = 256 / cg;
  const int blocks = std::max(1, std::min(2048, (M + rpp - 1) / rpp));
  if (g_f32)
    hipLaunchKernelGGL(bn_defer_step_kernel<true>, dim3(blocks), dim3(256), 0, s, sums, gamma,
                       mean, rstd, Ci, s0, M, 1.f / (float)M, k12, ldk, dgamma, dbeta, G, ldg,
                       (const bf16_t*)x, ldx, (bf16_t*)out);
  else
    hipLaunchKernelGGL(bn_defer_step_kernel<false>, dim3(blocks), dim3(256), 0, s, sums, gamma,
                       mean, rstd, Ci, s0, M, 1.f / (float)M, k12, ldk, dgamma, dbeta, G, ldg,
                       (const bf16_t*)x, ldx, (bf16_t*)out);
}
}  // namespace mpa

namespace mpa {
void bn_relu_avgpool2_fwd(const bf16_raw* z, const float* aff, int N, int H, int W, int C,
                          bf16_raw* y, hipStream_t s) {
  hipLaunchKernelGGL(bn_relu_avgpool2_fwd_kernel, grid_for(N * (H / 2) * (W / 2), C), dim3(256),
                     0, s, (const bf16_t*)z, aff, N, H, W, C, (bf16_t*)y);
}
}  // namespace mpa
