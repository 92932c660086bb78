// DenseNet norm1 -> conv1 backward hand-off (SURVEY.md §2.7 K2 + K4; models/densenet.py
// _DenseBlockGrad): the 1x1 / stride-1 dgrad of conv1,
//     dy[m][c] = sum_k dz[m][k] * W[k][c]          (c < Ci, the block buffer's prefix),
// with norm1's backward folded into the epilogue: g = bf16(dy) * [ReLU(BN(x)) > 0] is never
// written; instead  G[m][c] += gamma_c * rstd_c * g  goes straight into the block gradient
// and (sum g, sum g * xhat) are reduced per column.  The remaining, per-channel part of the
// BN backward is deferred and summed over layers (bn_defer_step, bn.hip).
//
// Why a kernel of its own: the epilogue moves 3 activation-sized streams (x, G in; G out)
// against one for a plain dgrad.  In the shared rows epilogue (fragment layout: each
// 8-byte access covers 4 columns of one row, 16 rows per instruction) that ran at ~1.4 TB/s
// and made the hand-off slower than the three passes it replaces.  Here the tile's g goes
// through LDS once, and the sweep reads / writes whole 256-byte row segments (16 lanes x
// 16 B), all 8 rows of a thread's loads in flight before any use.
//
// GEMM part: 128 x 128 tile, 4 waves (2 x 2, 64 x 64 each), K in 32-deep steps through a
// 3-stage LDS-DMA ring (buffer_load ... lds), the swizzled K-contiguous images and fragment
// reads of the rows engine (igemm_dma.hip).
#include "igemm_common.h"

namespace mpa {

namespace {
constexpr int GB_BM = 128, GB_BN = 128, GB_NW = 4;
constexpr int GB_A = GB_BM * 64, GB_B = GB_BN * 64, GB_STAGE = GB_A + GB_B;  // 16 KiB
constexpr int GB_IAW = GB_BM / 16 / GB_NW;  // A DMA instructions per wave and stage (2)
constexpr int GB_IBW = GB_BN / 16 / GB_NW;  // B (2)
constexpr int GB_TP = 136;                  // g tile pitch in bf16 (272 B: rows 4 banks apart)
constexpr int GB_LDS = 3 * GB_STAGE;        // 48 KiB; the epilogue reuses it

template <int N>
__device__ __forceinline__ void gb_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// logical 16-B chunk a DMA lane fetches so that it lands where kc_off expects it
__device__ __forceinline__ int gb_lane_chunk(int lane) {
  const int sub = lane >> 2;
  return (lane & 3) ^ ((4 - ((sub >> 2) & 3)) & 3);
}
}  // namespace

template <bool F32>
__global__ __launch_bounds__(256, 2) void dense_gacc_kernel(IGemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[GB_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tile = block_tile(p.tiles_total);
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int m0 = mt * GB_BM, n0 = nt * GB_BN;
  const int M = p.M, N = p.N, K = p.Ktot;
  const int ktiles = K / BK;

  // ---- epilogue operands first: this thread's 8 columns (cg) x rows r0, r0 + 16, ...,
  // r0 + 112 of x and G do not depend on the GEMM, so their loads are in flight under it
  // (the first ring wait then waits for them too: one exposed latency, not two)
  const int cg = tid & 15, r0 = tid >> 4;
  const int n = n0 + cg * 8;
  const bool nok = n < N;  // N % 8 == 0: a group is all in or all out
  float sc[8], sh[8], mu[8], rs[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = nok ? n + j : 0;
    mu[j] = p.ep_mean[c];
    rs[j] = p.ep_rstd[c];
    sc[j] = p.ep_gamma[c] * rs[j];
    sh[j] = __builtin_fmaf(-mu[j], sc[j], p.ep_beta[c]);
  }
  const size_t ld = (size_t)p.ldc;
  uint4 zq[8], gq[8], gq2[F32 ? 8 : 1];
#pragma unroll
  for (int pss = 0; pss < 8; ++pss) {  // every load of the thread in flight first
    const int m = m0 + r0 + 16 * pss;
    const bool ok = nok && m < M;
    const size_t o = (size_t)(ok ? m : 0) * ld + (ok ? n : 0);
    zq[pss] = ok ? *(const uint4*)(p.ep_z + o) : make_uint4(0u, 0u, 0u, 0u);
    if constexpr (F32) {
      const uint4* gp = (const uint4*)((const float*)p.ep_gacc + o);
      gq[pss] = ok ? gp[0] : make_uint4(0u, 0u, 0u, 0u);
      gq2[pss] = ok ? gp[1] : make_uint4(0u, 0u, 0u, 0u);
    } else {
      gq[pss] = ok ? *(const uint4*)((const bf16_t*)p.ep_gacc + o) : make_uint4(0u, 0u, 0u, 0u);
    }
  }
  // ---- GEMM: DMA lanes (rows past M / columns past N clamp; their results are dropped)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, 0x7fffffffu);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, 0x7fffffffu);
  const uint32_t s32 = lds_base(smem);
  const int kch = gb_lane_chunk(lane);
  uint32_t a_off[GB_IAW], b_off[GB_IBW];
#pragma unroll
  for (int i = 0; i < GB_IAW; ++i) {
    const int m = min(m0 + 16 * (wave * GB_IAW + i) + (lane >> 2), M - 1);
    a_off[i] = (uint32_t)(((size_t)m * K + kch * 8) * 2);
  }
#pragma unroll
  for (int i = 0; i < GB_IBW; ++i) {
    const int n = min(n0 + 16 * (wave + GB_NW * i) + (lane >> 2), N - 1);
    b_off[i] = (uint32_t)(((size_t)n * p.ldb + kch * 8) * 2);
  }
  auto issue = [&](int kt, uint32_t st) {
    const uint32_t kb = (uint32_t)kt * BK * 2;
#pragma unroll
    for (int i = 0; i < GB_IAW; ++i)
      buf_lds16_at(ra, st + (wave * GB_IAW + i) * 1024, a_off[i] + kb);
#pragma unroll
    for (int i = 0; i < GB_IBW; ++i)
      buf_lds16_at(rb, st + GB_A + (wave + GB_NW * i) * 1024, b_off[i] + kb);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * 64, wcol0 = wn * 64;
  if (ktiles > 0) issue(0, s32);
  if (ktiles > 1) issue(1, s32 + GB_STAGE);
  for (int kt = 0; kt < ktiles; ++kt) {
    if (kt + 1 < ktiles) gb_wait_barrier<GB_IAW + GB_IBW>();
    else gb_wait_barrier<0>();
    if (kt + 2 < ktiles) issue(kt + 2, s32 + ((kt + 2) % 3) * GB_STAGE);
    const char* st = smem + (kt % 3) * GB_STAGE;
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag_kc(st, wrow0 + i * 16 + (lane & 15), lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag_kc(st + GB_A, wcol0 + j * 16 + (lane & 15), lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(bfr[j], af[i], acc[i][j]);
  }
  __syncthreads();  // every DMA waited (vmcnt(0) on the last step): LDS free

  // ---- g = bf16(dy) tile into LDS: lane owns rows wrow0 + 16 i + lane%16, columns
  // wcol0 + 16 j + 4 (lane/16) .. +3
  bf16_t* tg = (bf16_t*)smem;
  {
    const int nl = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wrow0 + i * 16 + (lane & 15), col = wcol0 + j * 16 + nl;
        *(uint2*)(tg + row * GB_TP + col) =
            make_uint2(pack2(acc[i][j][0], acc[i][j][1]), pack2(acc[i][j][2], acc[i][j][3]));
      }
  }
  __syncthreads();

  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s[j] = 0.f; q[j] = 0.f; }
#pragma unroll
  for (int pss = 0; pss < 8; ++pss) {
    const int row = r0 + 16 * pss, m = m0 + row;
    if (!nok || m >= M) continue;
    float g[8], z[8];
    const uint4 gl = *(const uint4*)(tg + row * GB_TP + cg * 8);
    unpack8(gl, g);
    unpack8(zq[pss], z);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool live = bf2f(f2bf(__builtin_fmaf(z[j], sc[j], sh[j]))) > 0.f;
      g[j] = live ? g[j] : 0.f;
      s[j] += g[j];
      q[j] += g[j] * (z[j] - mu[j]) * rs[j];
    }
    const size_t o = (size_t)m * ld + n;
    if constexpr (F32) {
      f32x4 a = __builtin_bit_cast(f32x4, gq[pss]), b = __builtin_bit_cast(f32x4, gq2[pss]);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a[j] += sc[j] * g[j];
        b[j] += sc[4 + j] * g[4 + j];
      }
      f32x4* gp = (f32x4*)((float*)p.ep_gacc + o);
      gp[0] = a;
      gp[1] = b;
    } else {
      float gv[8];
      unpack8(gq[pss], gv);
#pragma unroll
      for (int j = 0; j < 8; ++j) gv[j] += sc[j] * g[j];
      *(uint4*)((bf16_t*)p.ep_gacc + o) = pack8(gv);
    }
  }
  // ---- column sums: the 4 row groups of a wave share cg (lanes l, l^16, l^32, l^48), then
  // the 4 waves through LDS; one slab row per M-tile (dense rows, slab_reduce sums them)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] += __shfl_xor(s[j], 16, 64);
    s[j] += __shfl_xor(s[j], 32, 64);
    q[j] += __shfl_xor(q[j], 16, 64);
    q[j] += __shfl_xor(q[j], 32, 64);
  }
  __syncthreads();  // done with the g tile
  float* red = (float*)smem;  // [4 waves][128 cols][2]
  if (lane < 16) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * GB_BN + cg * 8 + j) * 2] = s[j];
      red[(wave * GB_BN + cg * 8 + j) * 2 + 1] = q[j];
    }
  }
  __syncthreads();
  if (tid < GB_BN && n0 + tid < N) {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int w = 0; w < GB_NW; ++w) {
      a += red[(w * GB_BN + tid) * 2];
      b += red[(w * GB_BN + tid) * 2 + 1];
    }
    p.stats[(size_t)mt * 2 * N + n0 + tid] = a;
    p.stats[(size_t)mt * 2 * N + N + n0 + tid] = b;
    if (mt == 0) {  // start value of the slab reduction that runs after this kernel
      p.stats_sums[n0 + tid] = 0.f;
      p.stats_sums[N + n0 + tid] = 0.f;
    }
  }
}

// a: the dgrad as a plain GEMM (A = dz [M][K], B = the transposed 1x1 weight [N][ldb]),
// ep_z / ep_gacc / ldc the block buffer and gradient, ep_mean / ep_rstd / ep_gamma /
// ep_beta norm1's vectors; slab >= ceil(M / 128) x 2N floats, sums [2N]
bool dense_gacc_ok(const IGemmArgs& a) {
  return a.Ktot % BK == 0 && a.N % 8 == 0 && a.ldc % 8 == 0 && a.M > 0 &&
         (int64_t)a.M * a.Ktot * 2 < (1ll << 31) && (int64_t)a.N * a.ldb * 2 < (1ll << 31);
}

void dense_gacc(IGemmArgs a, float* slab, float* sums, hipStream_t s) {
  const int tiles_m = (a.M + GB_BM - 1) / GB_BM;
  a.tiles_n = (a.N + GB_BN - 1) / GB_BN;
  a.tiles_total = tiles_m * a.tiles_n;
  a.stats = slab;
  a.stats_sums = sums;
  if (a.ep_gacc_f32)
    hipLaunchKernelGGL(dense_gacc_kernel<true>, dim3(a.tiles_total), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(dense_gacc_kernel<false>, dim3(a.tiles_total), dim3(256), 0, s, a);
  slab_reduce(slab, tiles_m, 2 * a.N, sums, false, s);
}

}  // namespace mpa
