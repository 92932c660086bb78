// Implicit-GEMM convolution / linear engine on CDNA4 MFMA (gfx950, wave64).
//
// One engine serves every GEMM-shaped op the reference reaches through ATen
// (SURVEY.md §2.7 K1/K2/K3/K9): conv forward, conv dgrad, conv wgrad and Linear
// fwd/dgrad/wgrad.  Activations are NHWC bf16, conv weights KRSC bf16, accumulation fp32
// on v_mfma_f32_16x16x32_bf16.
//
//  * fwd / dgrad kernel ("igemm_rows"): GEMM rows = output pixels (gathered im2col rows of
//    an NHWC tensor, K-contiguous), GEMM cols = output channels.  A per-launch TAP TABLE
//    (dh, dw, weight-tap) describes the gather, so one kernel covers every kernel shape
//    (7x7, 11x11, 1x7/7x1 asymmetric, 1x1) and, for dgrad, every stride phase of a strided
//    conv (sub-pixel decomposition: each output phase is a stride-1 conv over the valid
//    taps only - no zero-stuffed MFMA work).  Weights are read K-contiguous (fwd, [K][RSC])
//    or N-contiguous (dgrad: B(kk=(tap,k), n=c) = w[k][tap][c]) through the hardware
//    transpose read ds_read_b64_tr_b16 - no transposed weight copy is ever materialised.
//    Epilogue: +bias, ReLU, bf16 store of 4 consecutive channels per lane (the MFMA is
//    issued with the channel operand first so each lane owns 4 adjacent channels), and
//    per-channel BatchNorm sum / sum-of-squares reduced in-wave and added with one fp32
//    atomic per channel per wave (K4's statistics pass disappears).
//  * wgrad kernel ("igemm_wgrad"): GEMM rows = output channels, cols = (r,s,c), reduction
//    over pixels.  Both operands are pixel-major in memory, so both are staged
//    [pixel][channel] in LDS and read as MFMA fragments with ds_read_b64_tr_b16.  Split-K
//    over pixels with fp32 atomic accumulation straight into the flat gradient arena.
//
// LDS images are XOR-swizzled so fragment reads are bank-conflict free (derivation in
// docs/KERNELS.md); staging is register double-buffered: global loads for tile k+1 are in
// flight while tile k's MFMAs run, one barrier per K-step.  Blocks are remapped so tiles
// sharing an operand panel land on the same XCD (private L2).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include "igemm_common.h"

namespace mpa {

// ======================================================================================
//  fwd / dgrad kernel
// ======================================================================================
template <int BM, int BN, int WM, int WN, int VW, bool BKC, bool SPLIT, int OCC>
__global__ __launch_bounds__(256, OCC) void igemm_rows_kernel(IGemmArgs p) {
  constexpr int NA = BM / 64;                 // A chunks / thread
  constexpr int A_BYTES = BM * 64;
  constexpr int B_BYTES = BN * 64;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  constexpr int NB_KC = (BN * 4 + 255) / 256;  // B chunks / thread (K-contig)
  constexpr int CPR = BN / 8;                  // N-contig: chunks per k-row
  constexpr int NB_MN = (BK * CPR + 255) / 256;
  constexpr int NB = BKC ? NB_KC : NB_MN;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int tile = block_tile(p.tiles_total);
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;

  const int ktiles = (p.Ktot + BK - 1) / BK;
  const int kbeg = block_split() * p.ktiles_per_split;
  const int kend = min(ktiles, kbeg + p.ktiles_per_split);

  // ---- per-thread A rows (fixed for the whole K loop)
  const int akc = tid & 3;
  int a_img[NA], a_bh[NA], a_bw[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (tid >> 2) + 64 * i;
    if (m < p.M) {
      const int hw = p.oH * p.oW;
      const int img = (int)fdiv((uint32_t)m, p.fd_hw);
      const int r = m - img * hw;
      const int oh = (int)fdiv((uint32_t)r, p.fd_ow);
      const int ow = r - oh * p.oW;
      a_img[i] = img * p.aH * p.aW;
      a_bh[i] = oh * p.Uh + p.Oh;
      a_bw[i] = ow * p.Uw + p.Ow;
    } else {
      a_img[i] = -1;
      a_bh[i] = 0;
      a_bw[i] = 0;
    }
  }

  u32x4 ra[NA], rb[NB];

  auto load_A = [&](int kt) {
    const int kk0 = kt * BK + akc * 8;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (VW == 8) {
        const int t = kk0 / p.aC;
        const int c = kk0 - t * p.aC;
        bool ok = (a_img[i] >= 0) && (kk0 < p.Ktot);
        int ih = 0, iw = 0;
        if (ok) {
          ih = a_bh[i] + p.taps.dh[t];
          iw = a_bw[i] + p.taps.dw[t];
          ok = (unsigned)ih < (unsigned)p.aH && (unsigned)iw < (unsigned)p.aW;
        }
        ra[i] = ld_chunk<8>(p.A + (size_t)(a_img[i] + ih * p.aW + iw) * p.aC + c, ok ? 8 : 0);
      } else {
        constexpr int SUB = (VW == 4) ? 2 : 8;
        constexpr int SW = 8 / SUB;
        uint16_t e[8];
#pragma unroll
        for (int s = 0; s < SUB; ++s) {
          const int kk = kk0 + s * SW;
          const int t = kk / p.aC;
          const int c = kk - t * p.aC;
          bool ok = (a_img[i] >= 0) && (kk < p.Ktot);
          int ih = 0, iw = 0;
          if (ok) {
            ih = a_bh[i] + p.taps.dh[t];
            iw = a_bw[i] + p.taps.dw[t];
            ok = (unsigned)ih < (unsigned)p.aH && (unsigned)iw < (unsigned)p.aW;
          }
          const bf16_t* src = p.A + (size_t)(a_img[i] + ih * p.aW + iw) * p.aC + c;
          if constexpr (SW == 4) {
            u32x2 v = u32x2{0u, 0u};
            if (ok) v = *(const u32x2*)src;
            e[4 * s] = v.x & 0xffff; e[4 * s + 1] = v.x >> 16;
            e[4 * s + 2] = v.y & 0xffff; e[4 * s + 3] = v.y >> 16;
          } else {
            e[s] = ok ? src[0] : (uint16_t)0;
          }
        }
        ra[i] = u32x4_make(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16),
                           e[6] | (e[7] << 16));
      }
    }
  };

  auto load_B = [&](int kt) {
    if constexpr (BKC) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i;
        const int row = c >> 2, kc = c & 3;
        const int n = n0 + row;
        const int kk = kt * BK + kc * 8;
        if constexpr (VW == 1) {
          uint16_t e[8];
#pragma unroll
          for (int j = 0; j < 8; ++j)
            e[j] = (row < BN && n < p.N && kk + j < p.Ktot) ? p.B[(size_t)n * p.ldb + kk + j] : 0;
          rb[i] = u32x4_make(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16),
                             e[6] | (e[7] << 16));
        } else {
          const bool ok = (row < BN) && (n < p.N);
          int kb = kk;
          if (VW == 8 && p.b_tapmap && kk < p.Ktot) {  // weight-tap row map (dgrad, wT)
            const int t = kk / p.aC;
            kb = p.taps.bt[t] * p.aC + (kk - t * p.aC);
          }
          rb[i] = ld_chunk<VW>(p.B + (size_t)n * p.ldb + kb, ok ? nvalid(kk, p.Ktot) : 0);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i;
        const int krow = c / CPR, cc = c % CPR;
        const int kk = kt * BK + krow;
        const int n = n0 + cc * 8;
        const bool ok = (krow < BK) && (kk < p.Ktot) && (n < p.N);
        int t = 0, k = 0;
        if (ok) {
          t = kk / p.aC;
          k = kk - t * p.aC;
        }
        rb[i] = ld_chunk<VW>(p.B + ((size_t)k * p.RS + p.taps.bt[t]) * p.ldb + n,
                              ok ? nvalid(n, p.N) : 0);
      }
    }
  };

  auto store_tiles = [&](char* st) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int row = (tid >> 2) + 64 * i;
      *LDS_PTR(u32x4, st + kc_off(row, akc)) = ra[i];
    }
    char* bimg = st + A_BYTES;
    if constexpr (BKC) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i;
        const int row = c >> 2, kc = c & 3;
        if (row < BN) *LDS_PTR(u32x4, bimg + kc_off(row, kc)) = rb[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int c = tid + 256 * i;
        const int krow = c / CPR, cc = c % CPR;
        if (krow < BK) *LDS_PTR(u32x4, bimg + mn_off<BN>(krow, cc * 8)) = rb[i];
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wrow0 = wm * (BM / WM);
  const int wcol0 = wn * (BN / WN);

  if (kbeg < kend) {
    load_A(kbeg);
    load_B(kbeg);
    store_tiles(smem);
    __syncthreads();
    int cur = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
      const bool more = kt + 1 < kend;
      if (more) {
        load_A(kt + 1);
        load_B(kt + 1);
      }
      const char* st = smem + cur * STAGE;
      const char* bimg = st + A_BYTES;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_kc(st, wrow0 + i * 16 + (lane & 15), lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (BKC) bfr[j] = frag_kc(bimg, wcol0 + j * 16 + (lane & 15), lane);
        else bfr[j] = frag_mn<BN>(bimg, wcol0 + j * 16, lane);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
      if (more) store_tiles(smem + (cur ^ 1) * STAGE);
      __syncthreads();
      cur ^= 1;
    }
  }
  rows_epilogue<BM, BN, WM, WN, SPLIT>(p, acc, smem, mt, m0, n0, wm, wrow0, wcol0, tid,
                                       RowsGeom{p.M, p.oH, p.oW, p.Poh, p.Pow, p.fd_hw, p.fd_ow});
}

// ======================================================================================
//  wgrad kernel: dW[m = kout][n = (r,s,c)] += sum_pix dy[pix][m] * im2col(x)[pix][n]
// ======================================================================================
template <int BM, int BN, int WM, int WN, int VWA, int VWB, int OCC>
__global__ __launch_bounds__(256, OCC) void igemm_wgrad_kernel(WGradArgs p) {
  constexpr int A_BYTES = BK * BM * 2;
  constexpr int B_BYTES = BK * BN * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int CPRA = BM / 8, CPRB = BN / 8;
  constexpr int NA = (BK * CPRA + 255) / 256;
  constexpr int NB = (BK * CPRB + 255) / 256;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int tile = xcd_remap(blockIdx.x, p.tiles_total);
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ktiles = (p.Mpix + BK - 1) / BK;
  const int kbeg = blockIdx.z * p.ktiles_per_split;
  const int kend = min(ktiles, kbeg + p.ktiles_per_split);
  if (kbeg >= kend) return;

  // ---- B column decode (fixed per thread): n -> (r, s, c)
  constexpr int NE = (VWB == 1) ? 8 : 1;
  int b_dh[NB][NE], b_dw[NB][NE], b_c[NB][NE];
  bool b_ok[NB][NE];
  // pixel iterators (incremental), one per B chunk
  int pix_img[NB], pix_oh[NB], pix_ow[NB];
  const int PQ = p.P * p.Q;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c = tid + 256 * i;
    const int krow = c / CPRB, cc = c % CPRB;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int n = n0 + cc * 8 + e;
      const int tap = n / p.C;
      const int ch = n - tap * p.C;
      const int r = tap / p.S, s = tap - (tap / p.S) * p.S;
      b_dh[i][e] = r - p.ph;
      b_dw[i][e] = s - p.pw;
      b_c[i][e] = ch;
      b_ok[i][e] = (krow < BK) && (n < p.Ncols);
    }
    const int pix = kbeg * BK + krow;
    const int img = pix / PQ;
    const int rr = pix - img * PQ;
    pix_img[i] = img;
    pix_oh[i] = rr / p.Q;
    pix_ow[i] = rr - (rr / p.Q) * p.Q;
  }

  u32x4 ra[NA], rb[NB];

  auto load_A = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i;
      const int krow = c / CPRA, cc = c % CPRA;
      const int pix = kt * BK + krow;
      const int m = m0 + cc * 8;
      const bool ok = (krow < BK) && (pix < p.Mpix);
      ra[i] = ld_chunk<VWA>(p.dy + (size_t)pix * p.Kout + m, ok ? nvalid(m, p.Kout) : 0);
    }
  };

  auto load_B = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + 256 * i;
      const int krow = c / CPRB;
      const int pix = kt * BK + krow;
      const bool pok = (krow < BK) && (pix < p.Mpix);
      const int bh = pix_oh[i] * p.sh, bw = pix_ow[i] * p.sw;
      const size_t ibase = (size_t)pix_img[i] * p.H * p.W;
      if constexpr (VWB == 1) {
        uint16_t e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ih = bh + b_dh[i][j], iw = bw + b_dw[i][j];
          const bool ok = pok && b_ok[i][j] && (unsigned)ih < (unsigned)p.H &&
                          (unsigned)iw < (unsigned)p.W;
          e[j] = ok ? p.x[(ibase + ih * p.W + iw) * p.C + b_c[i][j]] : (uint16_t)0;
        }
        rb[i] = u32x4_make(e[0] | (e[1] << 16), e[2] | (e[3] << 16), e[4] | (e[5] << 16),
                           e[6] | (e[7] << 16));
      } else {
        const int ih = bh + b_dh[i][0], iw = bw + b_dw[i][0];
        const bool ok = pok && b_ok[i][0] && (unsigned)ih < (unsigned)p.H &&
                        (unsigned)iw < (unsigned)p.W;
        rb[i] = ld_chunk<VWB>(p.x + (ibase + ih * p.W + iw) * p.C + b_c[i][0], ok ? 8 : 0);
      }
      // advance this chunk's pixel by BK for the next K-step
      int ow = pix_ow[i] + BK, oh = pix_oh[i], img = pix_img[i];
      while (ow >= p.Q) { ow -= p.Q; ++oh; }
      while (oh >= p.P) { oh -= p.P; ++img; }
      pix_ow[i] = ow; pix_oh[i] = oh; pix_img[i] = img;
    }
  };

  auto store_tiles = [&](char* st) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int c = tid + 256 * i;
      const int krow = c / CPRA, cc = c % CPRA;
      if (krow < BK) *LDS_PTR(u32x4, st + mn_off<BM>(krow, cc * 8)) = ra[i];
    }
    char* bimg = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c = tid + 256 * i;
      const int krow = c / CPRB, cc = c % CPRB;
      if (krow < BK) *LDS_PTR(u32x4, bimg + mn_off<BN>(krow, cc * 8)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * (BM / WM);
  const int wcol0 = wn * (BN / WN);

  load_A(kbeg);
  load_B(kbeg);
  store_tiles(smem);
  __syncthreads();
  int cur = 0;
  for (int kt = kbeg; kt < kend; ++kt) {
    const bool more = kt + 1 < kend;
    if (more) {
      load_A(kt + 1);
      load_B(kt + 1);
    }
    const char* st = smem + cur * STAGE;
    const char* bimg = st + A_BYTES;
    bf16x8 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = frag_mn<BM>(st, wrow0 + i * 16, lane);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = frag_mn<BN>(bimg, wcol0 + j * 16, lane);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
    if (more) store_tiles(smem + (cur ^ 1) * STAGE);
    __syncthreads();
    cur ^= 1;
  }
  wgrad_epilogue<BM, BN, WM, WN>(p, acc, m0, n0, wrow0, wcol0, lane);

}

// dw[i] += sum_z slab[z][i] (dw[i] = ... when overwrite).  A block owns 64 float4 columns; its 4 waves sum disjoint
// quarters of the splits (4 float4 loads in flight per lane), then reduce through LDS.
// With ~100 splits of a small layer (ResNet-18 layer1: 64 x 576 outputs) a
// one-thread-per-column walk over the splits ran at ~0.6 TB/s on 36 blocks.
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ slab, int S,
                                                            int64_t n, float* __restrict__ dw,
                                                            int overwrite) {
  __shared__ f32x4 red[4][64];
  const int64_t n4 = n / 4;
  const int64_t c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  if (c < n4) {
    const f32x4* src = (const f32x4*)slab + c;
    const int64_t stride = n4;  // one split = n4 float4
    int z = g;
    for (; z + 12 < S; z += 16) {
      const f32x4 a = src[(int64_t)z * stride], b = src[(int64_t)(z + 4) * stride];
      const f32x4 d = src[(int64_t)(z + 8) * stride], e = src[(int64_t)(z + 12) * stride];
      acc += (a + b) + (d + e);
    }
    for (; z < S; z += 4) acc += src[(int64_t)z * stride];
  }
  red[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g == 0 && c < n4) {
    const int t = threadIdx.x;
    f32x4 v = overwrite ? f32x4{0.f, 0.f, 0.f, 0.f} : ((f32x4*)dw)[c];
    v += (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
    ((f32x4*)dw)[c] = v;
  }
}

// any n (split rows not 16-B aligned when n % 4 != 0): one thread per element
__global__ __launch_bounds__(256) void wgrad_reduce_scalar_kernel(const float* __restrict__ slab,
                                                                   int S, int64_t n,
                                                                   float* __restrict__ dw,
                                                                   int overwrite) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float a = overwrite ? 0.f : dw[i];
    for (int z = 0; z < S; ++z) a += slab[(size_t)z * n + i];
    dw[i] = a;
  }
}

// ----------------------------------------------------------- split-K finalize (fp32->bf16)
// Sums the S split partials [S][M][N] (+ the existing output when beta).  A block owns CW
// columns (CW = 32 for 32-wide GEMMs, so no lane idles) and 256 / CW rows per pass, rows
// strided by gridDim.y; two rows per thread are in flight per pass (the S loads of both are
// independent).  Statistics go to the per-block-row slab [gridDim.y][2N].  (The round-2
// form, 64 columns x 4 rows per block and at most 64 block rows, left a 32-wide 12,544-row
// finalize at 59 us: 64 blocks, half their lanes idle, one dependent row at a time.)
template <int CW>
__global__ __launch_bounds__(256) void splitk_finalize_kernel(
    const float* __restrict__ ws, int S, bf16_t* __restrict__ out, int M, int N,
    const float* __restrict__ bias, int relu, float* __restrict__ slab,
    const float* __restrict__ shift, float* __restrict__ sums, int beta) {
  constexpr int RP = 256 / CW;
  __shared__ float red[2][256];
  const int n = blockIdx.x * CW + (threadIdx.x % CW);
  const int r0 = blockIdx.y * RP + threadIdx.x / CW;
  const int rstep = gridDim.y * RP;
  const size_t MN = (size_t)M * N;
  float s = 0.f, q = 0.f;
  const float b = (bias && n < N) ? bias[n] : 0.f;
  const float k = (shift && n < N) ? shift[n] : 0.f;
  auto fin = [&](int m, float v) {
    if (beta) v += bf2f(out[(size_t)m * N + n]);
    if (relu) v = fmaxf(v, 0.f);
    const bf16_t o = f2bf(v);
    out[(size_t)m * N + n] = o;
    const float rv = bf2f(o) - k;
    s += rv;
    q += rv * rv;
  };
  if (n < N) {
    int m = r0;
    for (; m + rstep < M; m += 2 * rstep) {
      float v0 = b, v1 = b;
      const float* w0 = ws + (size_t)m * N + n;
      const float* w1 = w0 + (size_t)rstep * N;
      for (int z = 0; z < S; ++z) {
        v0 += w0[z * MN];
        v1 += w1[z * MN];
      }
      fin(m, v0);
      fin(m + rstep, v1);
    }
    if (m < M) {
      float v = b;
      for (int z = 0; z < S; ++z) v += ws[z * MN + (size_t)m * N + n];
      fin(m, v);
    }
  }
  if (slab) {
    if (blockIdx.y == 0 && threadIdx.x < CW && n < N) {  // start value of the slab reduction
      sums[n] = 0.f;
      sums[N + n] = 0.f;
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = q;
    __syncthreads();
    if (threadIdx.x < CW && n < N) {
      const int t = threadIdx.x;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int r = 0; r < RP; ++r) {
        a0 += red[0][t + r * CW];
        a1 += red[1][t + r * CW];
      }
      slab[(size_t)blockIdx.y * 2 * N + n] = a0;
      slab[(size_t)blockIdx.y * 2 * N + N + n] = a1;
    }
  }
}

// ======================================================================================
//  host-side launch logic
// ======================================================================================
// Occupancy target (waves per SIMD) for the MFMA kernels: 3 fits every tile in <= 168
// VGPRs with no spills (accumulators move from AGPRs to VGPRs); 4 (<= 128 VGPRs) spills a
// few registers on the large tiles.
static int occ_target() { return 3; }

// Staging engine for 16-B-granular operands: 0 = register-staged (this file),
// 1 = tuned default: LDS-DMA (igemm_dma.hip) for the rows GEMMs (fwd / dgrad / linear);
//     for wgrad the 8-wave generic DMA tile where it wins (wgrad_big), the incremental
//     DMA kernel where it applies, register staging elsewhere,
// 2 = LDS-DMA for every GEMM.  MPA_IGEMM_ENGINE=0|1|2 sets the start value;
// igemm_set_engine switches at run time (A/B benchmarks, cross-checking tests).
static int g_engine = -1;
int igemm_engine() {
  if (g_engine < 0) {
    const char* e = getenv("MPA_IGEMM_ENGINE");
    g_engine = e ? std::min(2, std::max(0, atoi(e))) : 1;
  }
  return g_engine;
}
void igemm_set_engine(int e) { g_engine = std::min(2, std::max(0, e)); }

// Tile override for measurement (tools/bench_kernels.py): igemm_force_tile(BM, BN, splits);
// zeros restore the heuristics.  Applies to both plans (rows and wgrad, BM x BN of the
// respective GEMM) when the requested tile exists for the engine in use.
static int g_force_bm = 0, g_force_bn = 0, g_force_splits = 0;
void igemm_force_tile(int bm, int bn, int splits) {
  g_force_bm = bm; g_force_bn = bn; g_force_splits = splits;
}

// ---------------------------------------------------------------------- tile autotuner
// The static plans (rows_plan / wgrad_plan) were fitted on a few shapes and miss by 10-25 %
// elsewhere (tools/bench_kernels.py sweep at batch 512: layer4's strided conv runs 24 %
// faster on 256x128, layer2's strided wgrad 10 % faster on 128x256, layer3's 15 % faster on
// 128x128).  Like cudnn.benchmark, the first launch of each GEMM shape on the LDS-DMA
// engine times every eligible tile on scratch outputs (a warm-up run, then 3 timed ones)
// and caches the fastest; later launches reuse it.  The sweep costs a few ms once per shape
// (the warm-up steps of a training run), is skipped while a HIP graph is being captured
// (the static plan runs then) and is off with MPA_TUNE=0.  Tiles never change a result's
// summation order except through the split-K count, which candidates may not raise past
// the caller's workspace.
static bool g_tune = [] {
  const char* e = getenv("MPA_TUNE");
  return !(e && e[0] == '0');
}();
void igemm_set_tune(int on) { g_tune = on != 0; }
// Drain the whole device before timing a tuner candidate (single GPU: side / branch
// streams may still run kernels whose overlap would bias the choice).  Off under data
// parallelism (parallel/dist.py init_world): the drain would also wait for the overlapped
// RCCL all-reduces of the first step; the compute stream alone is synchronized then.
static bool g_tune_drain = true;
void igemm_set_tune_drain(int on) { g_tune_drain = on != 0; }

struct TunedTile {
  int bm, bn;
};
static std::mutex g_tune_mu;
static std::map<std::string, TunedTile> g_tuned;
// held for a whole tuning pass (scratch growth + candidate launches + timing): a second
// host thread tuning on the same device must not free the scratch buffer that this
// thread's candidate kernels are still writing
static std::mutex g_tune_pass_mu;

static bool stream_capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// grow-only per-device scratch for the candidates' outputs
static char* tune_scratch(size_t bytes) {
  static char* buf[64] = {};
  static size_t cap[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (bytes > cap[dev]) {
    if (buf[dev]) (void)hipFree(buf[dev]);
    buf[dev] = nullptr;
    cap[dev] = 0;
    if (hipMalloc(&buf[dev], bytes) != hipSuccess) return nullptr;
    cap[dev] = bytes;
  }
  return buf[dev];
}

// Timing of one tuner candidate: the device is drained first (the first training step tunes
// while side / branch streams may still run other kernels, whose overlap would bias the
// choice - an intermittent 3x slower SqueezeNet step in round 5), then the best of two
// rounds of three launches.  Tuning only runs on a shape's first launch outside a capture.
template <class F>
static float time_launches(F&& fn, hipStream_t s) {
  if (g_tune_drain) (void)hipDeviceSynchronize();
  else (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  fn();
  float best = 1e30f;
  for (int r = 0; r < 2; ++r) {
    (void)hipEventRecord(e0, s);
    for (int i = 0; i < 3; ++i) fn();
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = std::min(best, ms / 3.f);
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

static bool tuned_lookup(const std::string& key, int& bm, int& bn) {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  auto it = g_tuned.find(key);
  if (it == g_tuned.end()) return false;
  bm = it->second.bm;
  bn = it->second.bn;
  return true;
}
static void tuned_store(const std::string& key, int bm, int bn) {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  g_tuned[key] = TunedTile{bm, bn};
}

// number of tuned shapes and a readable dump ("key -> BMxBN" lines) for diagnostics
std::string igemm_tuned_table() {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  std::string out;
  for (const auto& kv : g_tuned)
    out += kv.first + " -> " + std::to_string(kv.second.bm) + "x" + std::to_string(kv.second.bn) + "\n";
  return out;
}

// load a table in igemm_tuned_table()'s format ("key -> BMxBN" lines); replace: drop every
// entry first.  Data-parallel ranks adopt rank 0's table this way, so every rank runs the
// same tiles (parallel/comm.py agree_tuned_tiles).  Returns the entries loaded.
int igemm_tuned_load(const std::string& table, bool replace) {
  std::lock_guard<std::mutex> lock(g_tune_mu);
  if (replace) g_tuned.clear();
  int n = 0;
  size_t pos = 0;
  while (pos < table.size()) {
    size_t end = table.find('\n', pos);
    if (end == std::string::npos) end = table.size();
    const std::string line = table.substr(pos, end - pos);
    pos = end + 1;
    const size_t arrow = line.rfind(" -> ");
    if (arrow == std::string::npos) continue;
    int bm = 0, bn = 0;
    if (sscanf(line.c_str() + arrow + 4, "%dx%d", &bm, &bn) != 2 || bm <= 0 || bn <= 0) continue;
    g_tuned[line.substr(0, arrow)] = TunedTile{bm, bn};
    ++n;
  }
  return n;
}

template <int BM, int BN, int WM, int WN, int VW, bool BKC, bool SPLIT>
static void launch_rows(const IGemmArgs& a0, int splits, hipStream_t s) {
  IGemmArgs a = a0;
  igemm_set_fastdiv(a);
  dim3 grid(a.tiles_total, 1, splits);
  const int o = occ_target();
  if (o == 4)
    hipLaunchKernelGGL((igemm_rows_kernel<BM, BN, WM, WN, VW, BKC, SPLIT, 4>), grid, dim3(256), 0,
                       s, a);
  else if (o == 2)
    hipLaunchKernelGGL((igemm_rows_kernel<BM, BN, WM, WN, VW, BKC, SPLIT, 2>), grid, dim3(256), 0,
                       s, a);
  else
    hipLaunchKernelGGL((igemm_rows_kernel<BM, BN, WM, WN, VW, BKC, SPLIT, 3>), grid, dim3(256), 0,
                       s, a);
}

template <int BM, int BN, int WM, int WN, bool BKC, bool SPLIT>
static void dispatch_vw(const IGemmArgs& a, int vw, int splits, hipStream_t s) {
  if (vw == 8) launch_rows<BM, BN, WM, WN, 8, BKC, SPLIT>(a, splits, s);
  else if (vw == 4) launch_rows<BM, BN, WM, WN, 4, BKC, SPLIT>(a, splits, s);
  else launch_rows<BM, BN, WM, WN, 1, BKC, SPLIT>(a, splits, s);
}

template <int BM, int BN, int WM, int WN, bool BKC>
static void dispatch_split(const IGemmArgs& a, int vw, int splits, hipStream_t s) {
  if (splits > 1) dispatch_vw<BM, BN, WM, WN, BKC, true>(a, vw, splits, s);
  else dispatch_vw<BM, BN, WM, WN, BKC, false>(a, vw, splits, s);
}

static int choose_bn(int N) {
  if (N <= 32) return 32;
  if (N <= 64 || (N % 128 != 0 && N % 64 == 0 && N < 256)) return 64;
  return 128;
}

// Split-K for grids smaller than the chip (< 256 tiles): each split stores its partial
// tile with plain 16-B stores into a [splits][M][N] fp32 slab and splitk_finalize sums
// them (+bias, ReLU, bf16, BN statistics) - no atomics.  Slab traffic is
// 2 * splits * M * N * 4 bytes, small next to the GEMM for these deep-K shapes.
static int choose_splits(int tiles, int ktiles) {
  if (tiles >= 256 || ktiles < 16) return 1;
  int s = (512 + tiles - 1) / tiles;
  s = std::min(s, ktiles / 8);
  s = std::min(s, 64);
  return std::max(s, 1);
}

static void finish_split_plan(int ktiles, int& splits, int& per_split) {
  per_split = ktiles > 0 ? (ktiles + splits - 1) / splits : 1;
  splits = ktiles > 0 ? (ktiles + per_split - 1) / per_split : 1;
}

// dma: the LDS-DMA engine will run it (adds the 8-wave 256x128 / 256x256 tiles, reachable
// through igemm_force_tile; tools/bench_kernels.py sweep measures them slower than 128x128
// on every ResNet layer: they leave the grid under one block per CU or force split-K,
// whose fp32 partial slab costs more than the tile saves).
static bool rows_tile_ok(int bm, int bn, bool dma) {
  const bool ok_reg = (bm == 128 && bn == 128) || (bm == 256 && bn == 64) || (bm == 128 && bn == 32);
  const bool ok_dma = ok_reg || (bm == 256 && (bn == 256 || bn == 128)) || (bm == 128 && bn == 64);
  return dma ? ok_dma : ok_reg;
}

// tbm / tbn: a tile chosen by the autotuner (0: the heuristic); igemm_force_tile wins
static void rows_plan(IGemmArgs& a, int& BM, int& BN, int& splits, bool allow_split, bool dma,
                      int tbm = 0, int tbn = 0) {
  BN = choose_bn(a.N);
  // 64-wide GEMMs: the DMA engine's 128x64 tile (36 KiB ring, 4 blocks/CU) beats 256x64
  // (60 KiB, 2 blocks/CU) on every ResNet-18 64-channel layer by 8-20 % (tile sweep)
  BM = (BN == 64 && !dma) ? 256 : 128;
  const int ktiles = (a.Ktot + BK - 1) / BK;
  if (tbm && tbn && rows_tile_ok(tbm, tbn, dma)) { BM = tbm; BN = tbn; }
  if (g_force_bm && g_force_bn && rows_tile_ok(g_force_bm, g_force_bn, dma)) {
    BM = g_force_bm;
    BN = g_force_bn;
  }
  a.tiles_n = (a.N + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  a.tiles_total = tiles_m * a.tiles_n;
  splits = allow_split ? choose_splits(a.tiles_total, ktiles) : 1;
  if (allow_split && g_force_splits > 0) splits = std::min(g_force_splits, std::max(ktiles, 1));
  finish_split_plan(ktiles, splits, a.ktiles_per_split);
}

static bool use_dma(int vw) { return vw == 8 && igemm_engine() >= 1; }

int64_t igemm_ws_floats(int M, int N, int Ktot) {
  int64_t best = 0;
  for (int dma = 0; dma < 2; ++dma) {  // sized for whichever engine ends up running it
    IGemmArgs a{};
    a.M = M; a.N = N; a.Ktot = Ktot;
    int BM, BN, splits;
    rows_plan(a, BM, BN, splits, true, dma == 1);
    if (splits > 1) best = std::max(best, (int64_t)splits * M * N);
  }
  return best;
}

// statistics slab rows: one per 128-row M-tile (the smallest BM of any plan), per halo /
// stem block or per splitk_finalize block row (<= slab_rows_max), then the [2][N] sums
static int64_t slab_rows_max(int M) {
  return std::max<int64_t>((M + 127) / 128, std::max(64, HALO_MAX_ROWS));
}

int64_t igemm_slab_floats(int M, int N) { return slab_rows_max(M) * 2 * N + 2 * N; }

static void rows_run_plan(IGemmArgs a, bool bkc, int vw, float* ws, float* slab, hipStream_t s,
                          int tbm, int tbn);

static std::string rows_key(const IGemmArgs& a, bool bkc, bool split) {
  char k[256];
  snprintf(k, sizeof k, "rows%d%d M%d N%d K%d a%dx%dx%d o%dx%d U%d,%d O%d,%d T%d s%d b%d r%d p%d",
           (int)bkc, (int)split, a.M, a.N, a.Ktot, a.aH, a.aW, a.aC, a.oH, a.oW, a.Uh, a.Uw,
           a.Oh, a.Ow, a.T, a.stap, a.beta, a.relu, a.nphase);
  std::string key(k);
  for (int i = 0; i < a.nphase; ++i)
    key += " " + std::to_string(a.ph[i].M) + "," + std::to_string(a.ph[i].Ktot);
  return key;
}

static const int kRowsCands[][2] = {{128, 128}, {256, 128}, {128, 64}, {256, 64}, {128, 32},
                                    {256, 256}};

// The 8-wave 256 x 256 rows tile is not an autotuner candidate: same-box A/B, round 3 -
// ResNet-18 b1024 47.73k/47.89k vs 47.67k/47.85k img/s, Inception 7.24k vs 7.26k,
// ResNet-34 25.35k vs 25.39k (noise) - for a longer first-step tuning pass.

static bool rows_cand_ok(int bm, int bn, int N) {
  if (bm == 256 && bn == 256) return false;
  if (bn == 128 && N <= 64) return false;  // half-empty tiles
  if (bn == 64 && (N <= 32 || N > 1024)) return false;
  if (bn == 32 && N > 32) return false;
  return true;
}

// autotuned tile of a rows GEMM (fills tbm / tbn; leaves them 0 to keep the heuristic)
static void tuned_rows_tile(const IGemmArgs& a, bool bkc, int vw, bool allow_split, hipStream_t s,
                            int& tbm, int& tbn) {
  if (!g_tune || deterministic() || (g_force_bm && g_force_bn) || a.M <= 0 || stream_capturing(s))
    return;
  const std::string key = rows_key(a, bkc, allow_split);
  if (tuned_lookup(key, tbm, tbn)) return;
  std::lock_guard<std::mutex> pass(g_tune_pass_mu);
  if (tuned_lookup(key, tbm, tbn)) return;  // tuned by another thread meanwhile
  const int64_t ws_cap = allow_split ? igemm_ws_floats(a.M, a.N, a.Ktot) : 0;
  const int64_t cbytes = ((int64_t)a.M * std::max(a.ldc, a.N) * 2 + 255) / 256 * 256;
  const int64_t sbytes = (igemm_slab_floats(a.M, a.N) + 2 * a.N) * 4;
  float best = 1e30f;
  int bbm = 0, bbn = 0;
  for (const auto& c : kRowsCands) {
    if (!rows_cand_ok(c[0], c[1], a.N)) continue;
    IGemmArgs b = a;
    int BM, BN, sp;
    rows_plan(b, BM, BN, sp, allow_split, true, c[0], c[1]);
    if (BM != c[0] || BN != c[1]) continue;
    if (sp > 1 && (int64_t)sp * a.M * a.N > ws_cap) continue;
    const int64_t wbytes = sp > 1 ? (int64_t)sp * a.M * a.N * 4 : 0;
    char* scr = tune_scratch(cbytes + sbytes + wbytes + 512);
    if (!scr) return;
    b = a;
    b.C = scr;
    float* slab = (float*)(scr + cbytes);
    if (a.stats) b.stats = slab + igemm_slab_floats(a.M, a.N);  // [2][N] after the slab
    b.stats_ld = 0;
    float* ws = sp > 1 ? (float*)(scr + cbytes + sbytes) : nullptr;
    if (!allow_split) ws = nullptr;
    else if (!ws) ws = (float*)(scr + cbytes + sbytes);  // (unused: no split)
    const float t = time_launches([&] { rows_run_plan(b, bkc, vw, ws, slab, s, c[0], c[1]); }, s);
    if (t < best) { best = t; bbm = c[0]; bbn = c[1]; }
  }
  if (!bbm) return;
  tuned_store(key, bbm, bbn);
  tbm = bbm;
  tbn = bbn;
}

static const bool g_kpad = [] {
  const char* e = getenv("MPA_KPAD");
  return !(e && e[0] == '0');
}();

static void run_rows(IGemmArgs a, bool bkc, int vw, float* ws, float* slab, hipStream_t s) {
  const bool dma = use_dma(vw);
  if (dma && bkc && conv_stem_ok(a)) {  // 7x7 pixel-pair stem: row-staged direct conv
    float* stats = a.stats;
    float* sums = stats ? slab + slab_rows_max(a.M) * 2 * a.N : nullptr;
    a.stats = stats ? slab : nullptr;
    const int rows = conv_stem(a, s);
    if (stats) slab_stats(slab, rows, a.N, a.stats_shift, a.M, sums, stats, s, a.stats_ld);
    return;
  }
  if (dma && bkc && conv3_halo_ok(a)) {  // 3x3 / stride 1: halo-staged direct conv
    float* stats = a.stats;
    float* sums = stats ? slab + slab_rows_max(a.M) * 2 * a.N : nullptr;
    a.stats = stats ? slab : nullptr;
    a.stats_sums = sums;
    const int rows = conv3_halo(a, s);
    if (stats) slab_stats(slab, rows, a.N, a.stats_shift, a.M, sums, stats, s, a.stats_ld);
    return;
  }
  // 16-B but not 32-granular channel counts (Inception 48 / 80): the uniform-tap kernel
  // with each tap's K padded to 32 (MPA_KPAD=0: the generic gather kernel); no split-K (the
  // caller's workspace was sized for the unpadded K)
  if (dma && g_kpad && igemm_rows_kpad_ok(a, bkc)) {
    a.Ktot = a.T * ((a.aC + BK - 1) / BK) * BK;
    a.kpad = 1;
    ws = nullptr;
  }
  int tbm = 0, tbn = 0;
  if (dma) tuned_rows_tile(a, bkc, vw, ws != nullptr, s, tbm, tbn);
  rows_run_plan(a, bkc, vw, ws, slab, s, tbm, tbn);
}

// the GEMM part of run_rows for a given (tuned) tile
static void rows_run_plan(IGemmArgs a, bool bkc, int vw, float* ws, float* slab, hipStream_t s,
                          int tbm, int tbn) {
  int BM, BN, splits;
  const bool dma = use_dma(vw);
  rows_plan(a, BM, BN, splits, ws != nullptr, dma, tbm, tbn);
  const int tiles_m = (a.M + BM - 1) / BM;
  void* final_out = a.C;
  float* stats = a.stats;
  float* sums = stats ? slab + slab_rows_max(a.M) * 2 * a.N : nullptr;
  a.stats = stats ? slab : nullptr;
  a.stats_sums = sums;
  if (splits > 1) {
    a.C = ws;
    a.ldc = a.N;
  }
  if (dma && igemm_rows_dma(a, BM, BN, bkc, splits, s)) {
    // LDS-DMA engine (igemm_dma.hip)
  } else if (a.kpad) {  // (unreachable: every planned tile has a kernel)
    fprintf(stderr, "rows_run_plan: padded-K launch without an LDS-DMA kernel\n");
    abort();
  } else if (bkc) {
    if (BN == 128) dispatch_split<128, 128, 2, 2, true>(a, vw, splits, s);
    else if (BN == 64) dispatch_split<256, 64, 4, 1, true>(a, vw, splits, s);
    else dispatch_split<128, 32, 4, 1, true>(a, vw, splits, s);
  } else {
    if (BN == 128) dispatch_split<128, 128, 2, 2, false>(a, vw, splits, s);
    else if (BN == 64) dispatch_split<256, 64, 4, 1, false>(a, vw, splits, s);
    else dispatch_split<128, 32, 4, 1, false>(a, vw, splits, s);
  }
  int slab_rows = tiles_m;
  if (splits > 1) {
    // ~512+ blocks (two rows in flight per thread), at most one slab row per block row
    const int cw = a.N <= 32 ? 32 : 64, rp = 256 / cw, gx = (a.N + cw - 1) / cw;
    const int gy = (int)std::min<int64_t>(slab_rows_max(a.M),
                                          std::max(1, std::min((a.M + 2 * rp - 1) / (2 * rp),
                                                               (1024 + gx - 1) / gx)));
    dim3 grid(gx, gy);
    if (cw == 32)
      hipLaunchKernelGGL(splitk_finalize_kernel<32>, grid, dim3(256), 0, s, ws, splits,
                         (bf16_t*)final_out, a.M, a.N, a.bias, a.relu,
                         stats ? slab : (float*)nullptr, a.stats_shift, sums, a.beta);
    else
      hipLaunchKernelGGL(splitk_finalize_kernel<64>, grid, dim3(256), 0, s, ws, splits,
                         (bf16_t*)final_out, a.M, a.N, a.bias, a.relu,
                         stats ? slab : (float*)nullptr, a.stats_shift, sums, a.beta);
    slab_rows = gy;
  }
  if (stats) slab_stats(slab, slab_rows, a.N, a.stats_shift, a.M, sums, stats, s, a.stats_ld);
}

// `a.stats` (if set) receives the finalized per-column statistics [mean(N), var(N)]
// (biased variance, from sums shifted by a.stats_shift); `slab` is a workspace of
// igemm_slab_floats(M, N) floats; `ws` holds igemm_ws_floats(M, N, Ktot) floats for the
// split-K partials (nullptr disables split-K, e.g. for strided output mappings).
void igemm_rows(IGemmArgs a, int vw, float* ws, float* slab, hipStream_t s) {
  run_rows(a, true, vw, ws, slab, s);
}

void igemm_rows_dgrad(IGemmArgs a, int vw, float* ws, hipStream_t s, bool bkc) {
  a.stats = nullptr;
  a.nphase = 0;
  run_rows(a, bkc, vw, ws, nullptr, s);
}

// dgrad + fused BN-backward reduction (LDS-DMA engine only: one launch, dense slab rows)
int64_t igemm_bnred_slab_floats(int M, int N, int nphase) {
  const int64_t rows = std::max<int64_t>((int64_t)((M + 127) / 128 + 1) * std::max(nphase, 1),
                                         HALO_MAX_ROWS);
  return rows * 2 * N;
}

// tile plan of a merged stride-phase launch; returns the number of (phase, m-tile) rows
static int plan_phases(IGemmArgs& a, int& BM, int& BN, int tbm = 0, int tbn = 0) {
  IGemmArgs probe = a;
  probe.M = 0;
  probe.Ktot = 0;
  for (int i = 0; i < a.nphase; ++i) {
    probe.M = std::max(probe.M, a.ph[i].M);
    probe.Ktot = std::max(probe.Ktot, a.ph[i].Ktot);
  }
  int splits;
  rows_plan(probe, BM, BN, splits, false, true, tbm, tbn);
  a.tiles_n = (a.N + BN - 1) / BN;
  int most = 0, rows = 0;
  for (int i = 0; i < a.nphase; ++i) {
    const int mts = (a.ph[i].M + BM - 1) / BM;
    a.ph[i].tiles = mts * a.tiles_n;
    most = std::max(most, a.ph[i].tiles);
    rows += mts;
  }
  a.tiles_total = most * a.nphase;
  a.ktiles_per_split = 1 << 30;
  return rows;
}

void igemm_rows_dgrad_bnred(IGemmArgs a, int vw, bool bkc, float* slab, float* sums,
                            hipStream_t s) {
  (void)vw;  // callers guarantee 16-B granular operands (LDS-DMA engine)
  a.bias = nullptr;
  a.relu = 0;
  a.stats_shift = nullptr;
  a.ep_bnred = 1;
  a.stats = slab;
  a.stats_sums = sums;
  int BM, BN, rows;
  if (a.nphase == 0 && bkc) {
    IGemmArgs t = a;
    if (t.ep_gamma && t.ep_beta) t.ep_y = nullptr;  // the halo kernel's z-mask form
    if (conv3_halo_ok(t)) {
      rows = conv3_halo(t, s);
      slab_reduce(slab, rows, 2 * a.N, sums, false, s);
      return;
    }
  }
  if (a.nphase > 0) {
    rows = plan_phases(a, BM, BN);
  } else {
    int splits;
    rows_plan(a, BM, BN, splits, false, true);
    rows = (a.M + BM - 1) / BM;
  }
  igemm_rows_dma(a, BM, BN, bkc, 1, s);
  slab_reduce(slab, rows, 2 * a.N, sums, false, s);
}

// All stride phases in ONE launch on the LDS-DMA engine: a stride-2 conv's dgrad is 4
// GEMMs of a quarter of the pixels each; launched separately each fills a fraction of the
// 256 CUs (ResNet-18 layer4 at batch 256: 196 tiles per phase), merged they fill it.
bool igemm_dgrad_src2_ok(const IGemmArgs& a, int vw, bool bkc) {
  return use_dma(vw) && a.nphase > 0 && a.nphase <= MAXPH && igemm_rows_uni_src2_ok(a, bkc);
}

void igemm_rows_dgrad_phases(IGemmArgs a, int vw, hipStream_t s, bool bkc) {
  a.stats = nullptr;
  a.bias = nullptr;
  if (a.nphase <= 0) return;
  if (a.A2 && !igemm_dgrad_src2_ok(a, vw, bkc)) {
    fprintf(stderr, "igemm_rows_dgrad_phases: second source on an ineligible launch\n");
    abort();
  }
  if (use_dma(vw) && a.nphase <= MAXPH) {
    int tbm = 0, tbn = 0;
    if (g_tune && !deterministic() && !(g_force_bm && g_force_bn) && !stream_capturing(s)) {
      const std::string key = rows_key(a, bkc, false);
      std::unique_lock<std::mutex> pass(g_tune_pass_mu, std::defer_lock);
      if (!tuned_lookup(key, tbm, tbn) && (pass.lock(), !tuned_lookup(key, tbm, tbn))) {
        // time the merged launch per candidate tile
        const int64_t hw0 = std::max(1, a.ph[0].oH * a.ph[0].oW);
        const int64_t rows = (a.ph[0].M + hw0 - 1) / hw0 * a.dH * a.dW;  // dx pixels
        const int64_t cbytes = rows * std::max(a.ldc, a.N) * 2;
        char* scr = tune_scratch(cbytes + 256);
        float best = 1e30f;
        for (const auto& c : kRowsCands) {
          if (!scr || !rows_cand_ok(c[0], c[1], a.N)) continue;
          IGemmArgs b = a;
          int BM, BN;
          plan_phases(b, BM, BN, c[0], c[1]);
          if (BM != c[0] || BN != c[1] || b.tiles_total <= 0) continue;
          b.C = scr;
          const float t = time_launches([&] { igemm_rows_dma(b, BM, BN, bkc, 1, s); }, s);
          if (t < best) { best = t; tbm = c[0]; tbn = c[1]; }
        }
        if (tbm) tuned_store(key, tbm, tbn);
      }
    }
    int BM, BN;
    plan_phases(a, BM, BN, tbm, tbn);
    if (a.tiles_total > 0 && igemm_rows_dma(a, BM, BN, bkc, 1, s)) return;
  }
  if (a.A2) {  // (unreachable: every planned tile has a kernel)
    fprintf(stderr, "igemm_rows_dgrad_phases: no merged launch for a second source\n");
    abort();
  }
  for (int i = 0; i < a.nphase; ++i) {  // one launch per phase
    const PhaseDesc& d = a.ph[i];
    IGemmArgs b = a;
    b.nphase = 0;
    b.M = d.M; b.oH = d.oH; b.oW = d.oW; b.Ktot = d.Ktot; b.T = d.T;
    b.Poh = d.Poh; b.Pow = d.Pow;
    for (int t = 0; t < d.T; ++t) {
      b.taps.dh[t] = a.taps.dh[d.tap0 + t];
      b.taps.dw[t] = a.taps.dw[d.tap0 + t];
      b.taps.bt[t] = a.taps.bt[d.tap0 + t];
    }
    run_rows(b, bkc, vw, nullptr, nullptr, s);
  }
}

template <int BM, int BN, int WM, int WN, int VWA, int VWB>
static void launch_wgrad(const WGradArgs& a, int splits, hipStream_t s) {
  dim3 grid(a.tiles_total, 1, splits);
  const int o = occ_target();
  if (o == 4)
    hipLaunchKernelGGL((igemm_wgrad_kernel<BM, BN, WM, WN, VWA, VWB, 4>), grid, dim3(256), 0, s, a);
  else if (o == 2)
    hipLaunchKernelGGL((igemm_wgrad_kernel<BM, BN, WM, WN, VWA, VWB, 2>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_wgrad_kernel<BM, BN, WM, WN, VWA, VWB, 3>), grid, dim3(256), 0, s, a);
}

template <int BM, int BN>
static void wgrad_vw(const WGradArgs& a, int vwa, int vwb, int splits, hipStream_t s) {
  if (vwb == 1) {
    if (vwa == 8) launch_wgrad<BM, BN, 2, 2, 8, 1>(a, splits, s);
    else if (vwa == 4) launch_wgrad<BM, BN, 2, 2, 4, 1>(a, splits, s);
    else launch_wgrad<BM, BN, 2, 2, 1, 1>(a, splits, s);
  } else {
    if (vwa == 8) launch_wgrad<BM, BN, 2, 2, 8, 8>(a, splits, s);
    else if (vwa == 4) launch_wgrad<BM, BN, 2, 2, 4, 8>(a, splits, s);
    else launch_wgrad<BM, BN, 2, 2, 1, 8>(a, splits, s);
  }
}

// split over pixels: ~512 blocks (2 per CU), >= 16 K-steps per split, slab <= 64 MiB;
// stem-shaped reductions (see wgrad_plan) target ~1024 blocks instead
// big: the 8-wave 128x256 LDS-DMA tile (measured +20..40 % over the 4-wave tiles for
// Kout >= 256 and for the stem's tiny-output / huge-pixel-count reduction)
static bool wgrad_big(const WGradArgs& a, bool dma_ok) {
  return dma_ok && (a.Kout >= 256 || ((int64_t)a.Kout * a.Ncols <= 32768 && a.Mpix >= (1 << 20)));
}

static bool wgrad_tile_ok(int bm, int bn, bool dma) {
  const bool ok_reg = (bm == 64 || bm == 128) && bn == 128;
  const bool ok_dma = ok_reg || (bn == 256 && (bm == 64 || bm == 128 || bm == 256));
  return dma ? ok_dma : ok_reg;
}

static void wgrad_plan(WGradArgs& a, int& BM, int& BN, int& splits, bool dma, bool big,
                       int tbm = 0, int tbn = 0) {
  BM = (a.Kout <= 64) ? 64 : 128;
  BN = 128;
  // few 128-row tiles (e.g. a 1x1 downsample: Ncols = C_in): halve BM for parallelism
  if (dma && BM == 128 && ((a.Kout + 127) / 128) * ((a.Ncols + 127) / 128) < 4) BM = 64;
  if (big) BN = 256, BM = (a.Kout <= 64) ? 64 : 128;  // 64-row stems: no half-empty tile
  const bool tuned = tbm && tbn && wgrad_tile_ok(tbm, tbn, dma);
  if (tuned) { BM = tbm; BN = tbn; }
  if (g_force_bm && g_force_bn && wgrad_tile_ok(g_force_bm, g_force_bn, dma)) {
    BM = g_force_bm;
    BN = g_force_bn;
  }
  a.tiles_n = (a.Ncols + BN - 1) / BN;
  const int tiles_m = (a.Kout + BM - 1) / BM;
  a.tiles_total = tiles_m * a.tiles_n;
  const int ktiles = (a.Mpix + BK - 1) / BK;
  // stem-shaped reductions (64 output rows, 129..256 columns, >= 1M pixels): two 64x128
  // column tiles x 512 splits instead of one 64x256 tile x 512 splits
  // (profiles/stem_sweep_b512.txt, batch 512: 64x128/s512 439.4 us, 64x128/s1024 449.2 us,
  // 64x256/s512 493.7 us). 512 splits keep the fp32 slab at 29 MB (1024: 58.7 MB).
  const bool stem2 = big && BM == 64 && BN == 256 && !(g_force_bm && g_force_bn) && !tuned &&
                     a.Ncols > 128 && a.Ncols <= 256;
  if (stem2) {
    BN = 128;
    a.tiles_n = (a.Ncols + BN - 1) / BN;
    a.tiles_total = tiles_m * a.tiles_n;
  }
  splits = std::max(1, ((stem2 ? 1024 : 512) + a.tiles_total - 1) / a.tiles_total);
  splits = std::min(splits, std::max(1, ktiles / 16));
  if (g_force_splits > 0) splits = std::min(g_force_splits, std::max(ktiles, 1));
  const int64_t out = (int64_t)a.Kout * a.Ncols;
  splits = (int)std::min<int64_t>(splits, std::max<int64_t>(1, (16ll << 20) / out));
  finish_split_plan(ktiles, splits, a.ktiles_per_split);
}

int64_t igemm_wgrad_ws_floats(int Kout, int Ncols, int Mpix) {
  int64_t best = conv3_halo_wgrad_ws_floats(Kout, Ncols);
  if (Kout == 64 && Ncols == 224) best = std::max(best, stem_wgrad_ws_floats());
  for (int dma = 0; dma < 3; ++dma) {  // register, DMA, DMA big tile
    WGradArgs a{};
    a.Kout = Kout; a.Ncols = Ncols; a.Mpix = Mpix;
    int BM, BN, splits;
    wgrad_plan(a, BM, BN, splits, dma >= 1, dma == 2);
    if (splits > 1) best = std::max(best, (int64_t)splits * Kout * Ncols);
  }
  return best;
}

static void wgrad_run_plan(WGradArgs a, int vwa, int vwb, hipStream_t s, int tbm, int tbn);

void igemm_stem_pool_wgrad(WGradArgs a, StemPoolArgs q, hipStream_t s) {
  const int z = stem_pool_wgrad(a, q, s);
  const int64_t n = (int64_t)a.Kout * a.Ncols;
  const int blocks = (int)std::max<int64_t>(1, (n / 4 + 63) / 64);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, a.slab, z, n, a.dw,
                     a.overwrite);
}

static const int kWgradCands[][2] = {{64, 128}, {128, 128}, {64, 256}, {128, 256}, {256, 256}};

// autotuned tile of a (non-halo) weight-gradient GEMM; candidates run on a scratch slab
// and a scratch dw, and may not need more split slab than the caller allocated
static void tuned_wgrad_tile(const WGradArgs& a, int vwa, int vwb, hipStream_t s, int& tbm,
                             int& tbn) {
  if (!g_tune || deterministic() || (g_force_bm && g_force_bn) || a.Mpix <= 0 ||
      stream_capturing(s))
    return;
  char k[200];
  snprintf(k, sizeof k, "wgrad K%d N%d P%d x%dx%dx%d o%dx%d f%dx%d s%d,%d p%d,%d", a.Kout, a.Ncols,
           a.Mpix, a.H, a.W, a.C, a.P, a.Q, a.R, a.S, a.sh, a.sw, a.ph, a.pw);
  const std::string key(k);
  if (tuned_lookup(key, tbm, tbn)) return;
  std::lock_guard<std::mutex> pass(g_tune_pass_mu);
  if (tuned_lookup(key, tbm, tbn)) return;
  const int64_t out = (int64_t)a.Kout * a.Ncols;
  const int64_t cap = igemm_wgrad_ws_floats(a.Kout, a.Ncols, a.Mpix);
  float best = 1e30f;
  for (const auto& c : kWgradCands) {
    if (c[0] > 64 && a.Kout <= 64) continue;  // half-empty tiles
    if (c[1] == 256 && a.Ncols <= 128) continue;
    WGradArgs b = a;
    int BM, BN, sp;
    const bool big = c[1] == 256;
    wgrad_plan(b, BM, BN, sp, true, big, c[0], c[1]);
    if (BM != c[0] || BN != c[1]) continue;
    if (sp > 1 && (int64_t)sp * out > cap) continue;
    char* scr = tune_scratch((size_t)(out + (sp > 1 ? sp * out : 0)) * 4 + 256);
    if (!scr) return;
    b = a;
    b.dw = (float*)scr;
    b.slab = a.slab ? (float*)scr + out : nullptr;
    const float t = time_launches([&] { wgrad_run_plan(b, vwa, vwb, s, c[0], c[1]); }, s);
    if (t < best) { best = t; tbm = c[0]; tbn = c[1]; }
  }
  if (tbm) tuned_store(key, tbm, tbn);
}

void igemm_wgrad(WGradArgs a, int vwa, int vwb, hipStream_t s) {
  if (igemm_engine() >= 1 && conv3_halo_wgrad_ok(a)) {  // 3x3 / stride 1: halo-staged
    const int z = conv3_halo_wgrad(a, s);
    const int64_t n = (int64_t)a.Kout * a.Ncols;  // Ncols = 9C, C % 32 == 0: float4 rows
    const int blocks = (int)std::max<int64_t>(1, (n / 4 + 63) / 64);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, a.slab, z, n, a.dw,
                       a.overwrite);
    return;
  }
  if (igemm_engine() >= 1 && stem_wgrad_ok(a)) {  // pixel-pair 7x7 stem: halo-staged
    const int z = stem_wgrad(a, s);
    const int64_t n = (int64_t)a.Kout * a.Ncols;
    const int blocks = (int)std::max<int64_t>(1, (n / 4 + 63) / 64);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, a.slab, z, n, a.dw,
                       a.overwrite);
    return;
  }
  const bool dma_ok = vwa == 8 && vwb == 8 && igemm_engine() >= 1;
  int tbm = 0, tbn = 0;
  if (dma_ok) tuned_wgrad_tile(a, vwa, vwb, s, tbm, tbn);
  wgrad_run_plan(a, vwa, vwb, s, tbm, tbn);
}

// the GEMM + split reduction of igemm_wgrad for a given (tuned) tile
static void wgrad_run_plan(WGradArgs a, int vwa, int vwb, hipStream_t s, int tbm, int tbn) {
  int BM, BN, splits;
  const bool dma_ok = vwa == 8 && vwb == 8 && igemm_engine() >= 1;
  const bool big = (tbm && tbn) ? tbn == 256 : wgrad_big(a, dma_ok);
  // engine 1: big 8-wave tile where it wins, else the incremental-pixel DMA kernel
  // (tools/bench_kernels.py sweep: equal or faster than register staging on every
  // ResNet-18 wgrad shape it covers), else register staging
  const bool dma = big || (dma_ok && (igemm_engine() == 2 || igemm_wgrad_inc_ok(a)));
  wgrad_plan(a, BM, BN, splits, dma, big, tbm, tbn);
  if (dma && igemm_wgrad_dma(a, BM, BN, splits, s)) {
    // LDS-DMA engine (igemm_dma.hip)
  } else if (BM == 64) {
    wgrad_vw<64, 128>(a, vwa, vwb, splits, s);
  } else {
    wgrad_vw<128, 128>(a, vwa, vwb, splits, s);
  }
  if (splits > 1) {
    const int64_t n = (int64_t)a.Kout * a.Ncols;
    if (n % 4 == 0) {  // float4 path: 16-B aligned split rows
      const int blocks = (int)std::max<int64_t>(1, (n / 4 + 63) / 64);
      hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, s, a.slab, splits, n,
                         a.dw, a.overwrite);
    } else {
      const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096));
      hipLaunchKernelGGL(wgrad_reduce_scalar_kernel, dim3(blocks), dim3(256), 0, s, a.slab,
                         splits, n, a.dw, a.overwrite);
    }
  }
}

}  // namespace mpa
