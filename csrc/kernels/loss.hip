// Fused softmax cross-entropy (K10) and argmax accuracy (K12).
//
// Forward: one workgroup per row makes ONE pass over the logits with an online
// (running max, rescaled sum) log-sum-exp - no max pass, no materialised softmax - and
// adds (lse - logit[label]) / B into the scalar loss.  Backward recomputes
// softmax = exp(logit - lse) from the saved per-row LSE and writes
// (softmax - onehot) * grad_out / B in bf16: logits are read twice in total, the
// gradient written once.  Reference: nn.CrossEntropyLoss at main.py:134,150 over a
// 64,500-wide head (utils.py:39); argmax accuracy at main.py:182-183.
//
// Rows may be padded (row stride ld >= NC): classifier heads store their output dim
// rounded up to a multiple of 32 so every GEMM of the head stays 16-B granular; the
// backward writes zeros into the padding columns of dlogits.
#include "common.h"
#include "api.h"
#include <cstdlib>
#include <algorithm>

namespace mpa {

template <int V>
__device__ __forceinline__ void load_v(const bf16_t* p, float* f) {
  if constexpr (V == 8) {
    unpack8(*(const uint4*)p, f);
  } else if constexpr (V == 4) {
    const uint2 u = *(const uint2*)p;
    f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
    f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  } else {
    f[0] = bf2f(p[0]);
  }
}

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

template <int V>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const bf16_t* __restrict__ logits,
                                                      const int64_t* __restrict__ labels, int B,
                                                      int NC, int ld, float* __restrict__ row_loss,
                                                      float* __restrict__ lse_out) {
  const int row = blockIdx.x;
  const bf16_t* x = logits + (size_t)row * ld;
  float m = -INFINITY, s = 0.f;
  const int nv = NC / V;
  for (int i = threadIdx.x; i < nv; i += 256) {
    float f[V];
    load_v<V>(x + (size_t)i * V, f);
    float lm = f[0];
#pragma unroll
    for (int j = 1; j < V; ++j) lm = fmaxf(lm, f[j]);
    const float mn = fmaxf(m, lm);
    float acc = s * __expf(m - mn);
#pragma unroll
    for (int j = 0; j < V; ++j) acc += __expf(f[j] - mn);
    m = mn;
    s = acc;
  }
  // wave reduce (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  __shared__ float sm[4], ss[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) lse_merge(M, S, sm[i], ss[i]);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    const float picked = (lab >= 0 && lab < NC) ? bf2f(x[lab]) : lse;
    row_loss[row] = (lse - picked) / (float)B;
  }
}

// Padded rows (ld % 8 == 0, 16-B aligned; the 64,500-class head has ld = 64,512): 16-B
// loads over the whole padded row with columns >= NC masked to -inf, U loads issued before
// any is consumed.  The unpadded kernel above walked 64,500 columns in 8-B loads, one load
// per online-LSE step, and streamed ~2.2 TB/s (30 us per 66 MB of logits).
template <int U>
__global__ __launch_bounds__(256) void ce_fwd_padded_kernel(const bf16_t* __restrict__ logits,
                                                             const int64_t* __restrict__ labels,
                                                             int B, int NC, int ld,
                                                             float* __restrict__ row_loss,
                                                             float* __restrict__ lse_out) {
  const int row = blockIdx.x;
  const bf16_t* x = logits + (size_t)row * ld;
  float m = -INFINITY, s = 0.f;
  const int nv = ld / 8;
  for (int i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * 256;
      v[u] = i < nv ? *(const uint4*)(x + (size_t)i * 8) : make_uint4(0u, 0u, 0u, 0u);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c0 = (i0 + u * 256) * 8;
      if (c0 >= NC) continue;
      float f[8];
      unpack8(v[u], f);
      float lm = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c0 + j >= NC) f[j] = -INFINITY;
        lm = fmaxf(lm, f[j]);
      }
      const float mn = fmaxf(m, lm);
      float acc = s * __expf(m - mn);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += __expf(f[j] - mn);
      m = mn;
      s = acc;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  __shared__ float sm[4], ss[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sm[w] = m; ss[w] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) lse_merge(M, S, sm[i], ss[i]);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t lab = labels[row];
    const float picked = (lab >= 0 && lab < NC) ? bf2f(x[lab]) : lse;
    row_loss[row] = (lse - picked) / (float)B;
  }
}

template <int V>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const bf16_t* __restrict__ logits,
                                                      const int64_t* __restrict__ labels,
                                                      const float* __restrict__ lse,
                                                      const float* __restrict__ grad_out, int B,
                                                      int NC, int ld, bf16_t* __restrict__ dlogits,
                                                      float weight) {
  const float scale = grad_out[0] * weight / (float)B;
  const int nv = ld / V;  // whole padded row: columns >= NC get zero gradient
  const int64_t total = (int64_t)B * nv;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int row = (int)(t / nv);
    const int c0 = (int)(t - (int64_t)row * nv) * V;
    const float l = lse[row];
    const int64_t lab = labels[row];
    float f[V];
    const size_t off = (size_t)row * ld + c0;
    load_v<V>(logits + off, f);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      float p = __expf(f[j] - l);
      if (c0 + j == lab) p -= 1.f;
      f[j] = (c0 + j < NC) ? p * scale : 0.f;
    }
    if constexpr (V == 8) {
      *(uint4*)(dlogits + off) = pack8(f);
    } else if constexpr (V == 4) {
      *(uint2*)(dlogits + off) = make_uint2(pack2(f[0], f[1]), pack2(f[2], f[3]));
    } else {
      dlogits[off] = f2bf(f[0]);
    }
  }
}

__global__ __launch_bounds__(256) void argmax_kernel(const bf16_t* __restrict__ logits,
                                                      const int64_t* __restrict__ labels, int NC,
                                                      int ld, unsigned long long* __restrict__ count) {
  const int row = blockIdx.x;
  const bf16_t* x = logits + (size_t)row * ld;
  float best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < NC; i += 256) {
    const float v = bf2f(x[i]);
    if (v > best) { best = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(best, o, 64);
    const int i2 = __shfl_xor(bi, o, 64);
    if (v2 > best || (v2 == best && i2 < bi)) { best = v2; bi = i2; }
  }
  __shared__ float sv[4];
  __shared__ int si[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[w] = best; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 4; ++i)
      if (sv[i] > best || (sv[i] == best && si[i] < bi)) { best = sv[i]; bi = si[i]; }
    if ((int64_t)bi == labels[row]) atomicAdd(count, 1ull);
  }
}

// loss = sum of the per-row terms in a FIXED order (strided per-thread partial sums, then a
// fixed tree): bitwise reproducible, unlike one float atomic per row (whose order varies
// between launches), and one launch like the memset it replaces.
__global__ __launch_bounds__(256) void ce_loss_sum_kernel(const float* __restrict__ row_loss, int B,
                                                          float* __restrict__ loss, int accumulate,
                                                          float weight, float* __restrict__ acc) {
  __shared__ float red[256];
  float a = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) a += row_loss[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float v = weight * red[0];
    if (accumulate) *loss += v;
    else *loss = v;
    if (acc) *acc += v;  // the trainer's running loss sum (one host sync per epoch)
  }
}

// loss: [1 + B] floats - the mean loss at [0], the per-row terms after it
void ce_fwd(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld, float* loss,
            float* lse, hipStream_t s) {
  float* rows = loss + 1;
  ce_fwd_rows(logits, labels, B, NC, ld, rows, lse, s);
  hipLaunchKernelGGL(ce_loss_sum_kernel, dim3(1), dim3(256), 0, s, rows, B, loss,
                     0, 1.f, (float*)nullptr);
}

// out[0] = (or +=) weight * mean CE; acc[0] += the same (when acc is set).  rows: B floats of
// scratch.  Several heads (Inception's main + 0.4 * aux) sum into one loss this way.
void ce_fwd_weighted(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld,
                     float* out, float* acc, float weight, bool accumulate, float* rows,
                     float* lse, hipStream_t s) {
  ce_fwd_rows(logits, labels, B, NC, ld, rows, lse, s);
  hipLaunchKernelGGL(ce_loss_sum_kernel, dim3(1), dim3(256), 0, s, rows, B, out,
                     accumulate ? 1 : 0, weight, acc);
}

void ce_fwd_rows(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld, float* loss,
                 float* lse, hipStream_t s) {
  if (ld % 8 == 0 && ld >= NC && reinterpret_cast<uintptr_t>(logits) % 16 == 0) {
    hipLaunchKernelGGL(ce_fwd_padded_kernel<4>, dim3(B), dim3(256), 0, s, logits, labels, B, NC,
                       ld, loss, lse);
    return;
  }
  const int g = NC % 8 == 0 && ld % 8 == 0 ? 8 : (NC % 4 == 0 && ld % 4 == 0 ? 4 : 1);
  if (g == 8)
    hipLaunchKernelGGL(ce_fwd_kernel<8>, dim3(B), dim3(256), 0, s, logits, labels, B, NC, ld, loss,
                       lse);
  else if (g == 4)
    hipLaunchKernelGGL(ce_fwd_kernel<4>, dim3(B), dim3(256), 0, s, logits, labels, B, NC, ld, loss,
                       lse);
  else
    hipLaunchKernelGGL(ce_fwd_kernel<1>, dim3(B), dim3(256), 0, s, logits, labels, B, NC, ld, loss,
                       lse);
}

void ce_bwd(const bf16_raw* logits, const int64_t* labels, const float* lse,
            const float* grad_out, int B, int NC, int ld, bf16_raw* dlogits, hipStream_t s,
            float weight) {
  const int V = (ld % 8 == 0) ? 8 : (ld % 4 == 0 ? 4 : 1);
  const int64_t total = (int64_t)B * (ld / V);
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
  if (V == 8)
    hipLaunchKernelGGL(ce_bwd_kernel<8>, dim3(blocks), dim3(256), 0, s, logits, labels, lse,
                       grad_out, B, NC, ld, dlogits, weight);
  else if (V == 4)
    hipLaunchKernelGGL(ce_bwd_kernel<4>, dim3(blocks), dim3(256), 0, s, logits, labels, lse,
                       grad_out, B, NC, ld, dlogits, weight);
  else
    hipLaunchKernelGGL(ce_bwd_kernel<1>, dim3(blocks), dim3(256), 0, s, logits, labels, lse,
                       grad_out, B, NC, ld, dlogits, weight);
}

void argmax_correct(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld,
                    int64_t* count, hipStream_t s) {
  hipLaunchKernelGGL(argmax_kernel, dim3(B), dim3(256), 0, s, logits, labels, NC, ld,
                     (unsigned long long*)count);
}

}  // namespace mpa
