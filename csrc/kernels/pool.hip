// Max / average / adaptive-average pooling, forward and backward, NHWC (K6/K7 of
// SURVEY.md §2.7).  One thread per output (forward) or input (backward) pixel and 8-channel
// chunk (16-B vectors) when C % 8 == 0, scalar channels otherwise.  Backward passes are
// GATHER formulations - each input pixel sums the windows that cover it - so they need no
// atomics and are deterministic.  Max pooling stores the window-local argmax (uint8) in
// forward; backward compares against it (first-max tie rule, like ATen).
#include "common.h"
#include "api.h"
#include <algorithm>

namespace mpa {

template <int V>
struct Vec;
template <>
struct Vec<8> {
  static __device__ __forceinline__ void load(const bf16_t* p, float* f) {
    unpack8(*(const uint4*)p, f);
  }
  static __device__ __forceinline__ void store(bf16_t* p, const float* f) {
    *(uint4*)p = pack8(f);
  }
};
template <>
struct Vec<1> {
  static __device__ __forceinline__ void load(const bf16_t* p, float* f) { f[0] = bf2f(p[0]); }
  static __device__ __forceinline__ void store(bf16_t* p, const float* f) { p[0] = f2bf(f[0]); }
};

static inline int grid1d(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

// ------------------------------------------------------------------------------ max
template <int V>
__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int H, int W, int C,
                                   int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                                   bf16_t* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * P * Q * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int q = (int)(r % Q); r /= Q;
    const int p = (int)(r % P);
    const int n = (int)(r / P);
    float best[V];
    int bi[V];
#pragma unroll
    for (int j = 0; j < V; ++j) { best[j] = -INFINITY; bi[j] = 0; }
    const int h0 = p * sh - ph, w0 = q * sw - pw;
    for (int i = 0; i < kh; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int k = 0; k < kw; ++k) {
        const int w = w0 + k;
        if ((unsigned)w >= (unsigned)W) continue;
        float f[V];
        Vec<V>::load(x + (((size_t)n * H + h) * W + w) * C + cc * V, f);
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (f[j] > best[j] || (f[j] != f[j] && best[j] == best[j])) {
            best[j] = f[j];
            bi[j] = i * kw + k;
          }
      }
    }
    const size_t o = (((size_t)n * P + p) * Q + q) * C + cc * V;
    Vec<V>::store(y + o, best);
#pragma unroll
    for (int j = 0; j < V; ++j) idx[o + j] = (uint8_t)bi[j];
  }
}

template <int V>
__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx,
                                   int N, int H, int W, int C, int P, int Q, int kh, int kw,
                                   int sh, int sw, int ph, int pw, bf16_t* __restrict__ dx) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    // outputs p with p*sh - ph <= h <= p*sh - ph + kh - 1
    const int plo = max(0, (h + ph - kh + sh) / sh), phi = min(P - 1, (h + ph) / sh);
    const int qlo = max(0, (w + pw - kw + sw) / sw), qhi = min(Q - 1, (w + pw) / sw);
    for (int p = plo; p <= phi; ++p) {
      const int i = h - (p * sh - ph);
      if (i < 0 || i >= kh) continue;
      for (int q = qlo; q <= qhi; ++q) {
        const int k = w - (q * sw - pw);
        if (k < 0 || k >= kw) continue;
        const size_t o = (((size_t)n * P + p) * Q + q) * C + cc * V;
        float g[V];
        Vec<V>::load(dy + o, g);
        const int me = i * kw + k;
#pragma unroll
        for (int j = 0; j < V; ++j)
          if (idx[o + j] == me) acc[j] += g[j];
      }
    }
    Vec<V>::store(dx + (((size_t)n * H + h) * W + w) * C + cc * V, acc);
  }
}

// -------------------------------------------------------------------------- average
__device__ __forceinline__ float avg_div(int p, int q, int H, int W, int kh, int kw, int sh,
                                         int sw, int ph, int pw, int cip) {
  int hs = p * sh - ph, ws = q * sw - pw;
  int he = min(hs + kh, H + ph), we = min(ws + kw, W + pw);
  const int pool = (he - hs) * (we - ws);
  hs = max(hs, 0); ws = max(ws, 0);
  he = min(he, H); we = min(we, W);
  const int cnt = cip ? pool : (he - hs) * (we - ws);
  return cnt > 0 ? 1.f / (float)cnt : 0.f;
}

template <int V>
__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, int N, int H, int W, int C,
                                   int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                                   int cip, bf16_t* __restrict__ y, int ldx) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * P * Q * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int q = (int)(r % Q); r /= Q;
    const int p = (int)(r % P);
    const int n = (int)(r / P);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    const int h0 = p * sh - ph, w0 = q * sw - pw;
    for (int i = 0; i < kh; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int k = 0; k < kw; ++k) {
        const int w = w0 + k;
        if ((unsigned)w >= (unsigned)W) continue;
        float f[V];
        Vec<V>::load(x + (((size_t)n * H + h) * W + w) * ldx + cc * V, f);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += f[j];
      }
    }
    const float d = avg_div(p, q, H, W, kh, kw, sh, sw, ph, pw, cip);
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] *= d;
    Vec<V>::store(y + (((size_t)n * P + p) * Q + q) * C + cc * V, acc);
  }
}

template <int V>
__global__ void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, int N, int H, int W, int C,
                                   int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw,
                                   int cip, bf16_t* __restrict__ dx, int ldo) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    const int plo = max(0, (h + ph - kh + sh) / sh), phi = min(P - 1, (h + ph) / sh);
    const int qlo = max(0, (w + pw - kw + sw) / sw), qhi = min(Q - 1, (w + pw) / sw);
    for (int p = plo; p <= phi; ++p) {
      const int i = h - (p * sh - ph);
      if (i < 0 || i >= kh) continue;
      for (int q = qlo; q <= qhi; ++q) {
        const int k = w - (q * sw - pw);
        if (k < 0 || k >= kw) continue;
        const float d = avg_div(p, q, H, W, kh, kw, sh, sw, ph, pw, cip);
        float g[V];
        Vec<V>::load(dy + (((size_t)n * P + p) * Q + q) * C + cc * V, g);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += g[j] * d;
      }
    }
    Vec<V>::store(dx + (((size_t)n * H + h) * W + w) * ldo + cc * V, acc);
  }
}

// ------------------------------------------------------------------------- adaptive
__device__ __forceinline__ int ad_start(int i, int in, int out) { return (i * in) / out; }
__device__ __forceinline__ int ad_end(int i, int in, int out) {
  return ((i + 1) * in + out - 1) / out;
}

template <int V>
__global__ void adaptive_fwd_kernel(const bf16_t* __restrict__ x, int N, int H, int W, int C,
                                    int P, int Q, bf16_t* __restrict__ y) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * P * Q * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int q = (int)(r % Q); r /= Q;
    const int p = (int)(r % P);
    const int n = (int)(r / P);
    const int hs = ad_start(p, H, P), he = ad_end(p, H, P);
    const int ws = ad_start(q, W, Q), we = ad_end(q, W, Q);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        float f[V];
        Vec<V>::load(x + (((size_t)n * H + h) * W + w) * C + cc * V, f);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += f[j];
      }
    const float d = 1.f / (float)((he - hs) * (we - ws));
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] *= d;
    Vec<V>::store(y + (((size_t)n * P + p) * Q + q) * C + cc * V, acc);
  }
}

template <int V>
__global__ void adaptive_bwd_kernel(const bf16_t* __restrict__ dy, int N, int H, int W, int C,
                                    int P, int Q, bf16_t* __restrict__ dx) {
  const int cv = C / V;
  const int64_t total = (int64_t)N * H * W * cv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int cc = (int)(t % cv);
    int64_t r = t / cv;
    const int w = (int)(r % W); r /= W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    const int plo = max(0, (h * P) / H - 1), phi = min(P - 1, ((h + 1) * P) / H + 1);
    const int qlo = max(0, (w * Q) / W - 1), qhi = min(Q - 1, ((w + 1) * Q) / W + 1);
    for (int p = plo; p <= phi; ++p) {
      const int hs = ad_start(p, H, P), he = ad_end(p, H, P);
      if (h < hs || h >= he) continue;
      for (int q = qlo; q <= qhi; ++q) {
        const int ws = ad_start(q, W, Q), we = ad_end(q, W, Q);
        if (w < ws || w >= we) continue;
        const float d = 1.f / (float)((he - hs) * (we - ws));
        float g[V];
        Vec<V>::load(dy + (((size_t)n * P + p) * Q + q) * C + cc * V, g);
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] += g[j] * d;
      }
    }
    Vec<V>::store(dx + (((size_t)n * H + h) * W + w) * C + cc * V, acc);
  }
}

// ------------------------------------------------------------------------ launchers
#define POOL_LAUNCH(K, total, ...)                                                        \
  do {                                                                                    \
    if (C % 8 == 0)                                                                       \
      hipLaunchKernelGGL(K<8>, dim3(grid1d((total) / 8)), dim3(256), 0, s, __VA_ARGS__);  \
    else                                                                                  \
      hipLaunchKernelGGL(K<1>, dim3(grid1d(total)), dim3(256), 0, s, __VA_ARGS__);        \
  } while (0)

void maxpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, bf16_raw* y, uint8_t* idx, hipStream_t s) {
  POOL_LAUNCH(maxpool_fwd_kernel, (int64_t)N * P * Q * C, x, N, H, W, C, P, Q, kh, kw, sh, sw,
              ph, pw, y, idx);
}
void maxpool_bwd(const bf16_raw* dy, const uint8_t* idx, int N, int H, int W, int C, int P,
                 int Q, int kh, int kw, int sh, int sw, int ph, int pw, bf16_raw* dx,
                 hipStream_t s) {
  POOL_LAUNCH(maxpool_bwd_kernel, (int64_t)N * H * W * C, dy, idx, N, H, W, C, P, Q, kh, kw, sh,
              sw, ph, pw, dx);
}
void avgpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, int cip, bf16_raw* y, hipStream_t s, int ldx) {
  if (ldx <= 0) ldx = C;
  POOL_LAUNCH(avgpool_fwd_kernel, (int64_t)N * P * Q * C, x, N, H, W, C, P, Q, kh, kw, sh, sw,
              ph, pw, cip, y, ldx);
}
void avgpool_bwd(const bf16_raw* dy, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, int cip, bf16_raw* dx, hipStream_t s, int ldo) {
  if (ldo <= 0) ldo = C;
  POOL_LAUNCH(avgpool_bwd_kernel, (int64_t)N * H * W * C, dy, N, H, W, C, P, Q, kh, kw, sh, sw,
              ph, pw, cip, dx, ldo);
}
void adaptive_avgpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q,
                          bf16_raw* y, hipStream_t s) {
  POOL_LAUNCH(adaptive_fwd_kernel, (int64_t)N * P * Q * C, x, N, H, W, C, P, Q, y);
}
void adaptive_avgpool_bwd(const bf16_raw* dy, int N, int H, int W, int C, int P, int Q,
                          bf16_raw* dx, hipStream_t s) {
  POOL_LAUNCH(adaptive_bwd_kernel, (int64_t)N * H * W * C, dy, N, H, W, C, P, Q, dx);
}

}  // namespace mpa
