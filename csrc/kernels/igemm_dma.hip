// LDS-DMA implicit-GEMM engine for gfx950 (MI355X / CDNA4).
//
// Same GEMM decomposition, tap tables, LDS images, fragment reads and epilogues as the
// register-staged engine in igemm.hip (conv fwd / dgrad / linear "rows" kernel and the
// wgrad kernel), but both operands are staged with
// global_load_lds_dwordx4: each lane DMA's one 16-B chunk straight from HBM/L2 into LDS,
// no VGPR round trip and no ds_write pass.  Why: per 32-deep K-step a 128x128 block reads
// 32 KiB of fragments (~128 LDS clk at 256 B/clk) but the register path also writes 16 KiB
// with ds_write_b128 (~79 B/clk/CU, ~207 clk) - against 256 clk of MFMA per SIMD the
// register-staged kernel is LDS-write bound (MI355X_MICROARCH.md §LDS).
//
//  * An LDS-DMA instruction writes wave-uniform base + 16*lane, so the images stay in the
//    engine's XOR-swizzled layouts by permuting the SOURCE: the lane that lands on chunk
//    position p of a row fetches logical chunk p ^ swz(row) (the same involution the
//    fragment reads apply).  Lanes whose element is padding / out of range fetch a 16-B
//    zero page instead, so halo and tail handling cost nothing in the loop.
//  * 3-stage ring, one raw s_barrier per K-step, counted `s_waitcnt vmcnt(N)`: tile kt+1's
//    DMAs stay in flight across the barrier while tile kt is multiplied, and the DMA for
//    tile kt+2 is issued right after the barrier into the stage tile kt-1 just vacated.
//  * No ordinary VGPR-destination global load inside the loop (hipcc would drain the DMA
//    queue with vmcnt(0) at its first use): the per-launch tap table is copied to LDS at
//    kernel start and read with ds_read; every other loop operand is a kernel argument.
//  * All LDS lives in one __shared__ array (a second LDS object makes hipcc insert a
//    vmcnt(0) before the first ds_read of every K-step).
// Requires 16-B granularity on both operands (the VW = 8 case of igemm.hip); the host
// falls back to the register-staged engine otherwise.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include "igemm_common.h"

namespace mpa {

// 16-B zero page: the DMA source of every padded / out-of-range lane
static __device__ __attribute__((aligned(16))) uint32_t g_zero16[4];

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16,
                                   0, 0);
}

// wait until at most N of this wave's vector-memory ops are outstanding and all its LDS
// reads have returned, then barrier; the memory clobber pins LDS reads/DMAs on their side
template <int N>
__device__ __forceinline__ void wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// logical 16-B chunk fetched by `lane` for K-contiguous images (kc_off layout): the lane
// lands on row 16j + lane/4, position lane&3; kc_off's XOR depends on (row>>2)&3 only
__device__ __forceinline__ int kc_lane_chunk(int lane) {
  const int sub = lane >> 2;
  return (lane & 3) ^ ((4 - ((sub >> 2) & 3)) & 3);
}

// waves per SIMD allowed by the 3-stage ring's LDS (160 KiB per CU) for a block of `nw`
// waves, capped at 3 (<= 168 VGPRs per lane): the occupancy target of __launch_bounds__.
// (A cap of 4 for 8-wave blocks forces 22-44 spilled VGPRs on the fast-path kernels.)
constexpr int dma_occ(int lds_bytes, int nw) {
  return ((160 * 1024) / lds_bytes) * nw / 4 >= 3 ? 3
         : (((160 * 1024) / lds_bytes) * nw / 4 >= 2 ? 2 : 1);
}

// ======================================================================================
//  rows kernel (fwd / dgrad / linear): C[m][n] = sum_k im2col(A)[m][k] * B(k, n)
// ======================================================================================
template <int BM, int BN, int WM, int WN, bool BKC, bool SPLIT, bool PH>
__global__ __launch_bounds__(WM * WN * 64, dma_occ(3 * (BM + BN) * 64 + MAXT * 8, WM * WN))
void igemm_rows_dma_kernel(IGemmArgs p) {
  constexpr int NW = WM * WN, NT = NW * 64;  // waves / threads per block
  constexpr int NS = 3;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, STAGE = A_BYTES + B_BYTES;
  constexpr int IA = BM / 16, IB = BN / 16;  // 1-KiB DMA instructions per tile
  constexpr int IAW = IA / NW;               // A instructions per wave
  constexpr int IBW = (IB + NW - 1) / NW;    // B instructions per wave (max)
  constexpr int WAITN = IAW + IB / NW;       // DMAs per wave per tile (min over waves)
  constexpr int CPR = BN / 8, RPI = 64 / CPR;  // N-contig B image: chunks / row, rows / instr
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  static_assert(IA % NW == 0 && (NW == 4 || NW == 8), "tile");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + MAXT * 8];
  int* tap_hw = (int*)(smem + NS * STAGE);  // (dh << 16) | (dw & 0xffff)
  int* tap_b = tap_hw + MAXT;               // weight tap of the N-contig operand

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  int tile = block_tile(p.tiles_total);
  // merged stride-phase launch: the block's phase sets output geometry, K and taps
  RowsGeom g{p.M, p.oH, p.oW, p.Poh, p.Pow, p.fd_hw, p.fd_ow};
  int Ktot = p.Ktot, T = p.T, tap0 = 0, kps = p.ktiles_per_split;
  int row_base = 0;  // statistics-slab row of m-tile 0 of this block's phase (dense rows)
  if constexpr (PH) {
    const int ph = tile % p.nphase;
    tile /= p.nphase;
    const PhaseDesc& d = p.ph[ph];
    if (tile >= d.tiles) return;  // padding tile of a shorter phase (whole block)
    for (int q = 0; q < ph; ++q) row_base += p.ph[q].tiles / p.tiles_n;
    g = RowsGeom{d.M, d.oH, d.oW, d.Poh, d.Pow, d.fd_hw, d.fd_ow};
    Ktot = d.Ktot;
    T = d.T;
    tap0 = d.tap0;
    kps = (Ktot + BK - 1) / BK;
  }
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ktiles = (Ktot + BK - 1) / BK;
  const int kbeg = block_split() * kps;
  const int kend = min(ktiles, kbeg + kps);

  for (int t = tid; t < T; t += NT) {
    tap_hw[t] = ((int)p.taps.dh[tap0 + t] << 16) | ((int)p.taps.dw[tap0 + t] & 0xffff);
    tap_b[t] = p.taps.bt[tap0 + t];
  }
  __syncthreads();
  const int tlast = max(T - 1, 0);
  const bf16_t* const zp = (const bf16_t*)g_zero16;

  // ---- A: this lane's rows (one per DMA instruction) and its k-chunk state
  const int kch = kc_lane_chunk(lane);
  int a_img[IAW], a_bh[IAW], a_bw[IAW];
#pragma unroll
  for (int i = 0; i < IAW; ++i) {
    const int m = m0 + 16 * (wave * IAW + i) + (lane >> 2);
    if (m < g.M) {
      const int hw = g.oH * g.oW;
      const int img = (int)fdiv((uint32_t)m, g.fd_hw);
      const int r = m - img * hw;
      const int oh = (int)fdiv((uint32_t)r, g.fd_ow);
      a_img[i] = img * p.aH * p.aW;
      a_bh[i] = oh * p.Uh + p.Oh;
      a_bw[i] = (r - oh * g.oW) * p.Uw + p.Ow;
    } else {
      a_img[i] = -1;
      a_bh[i] = 0;
      a_bw[i] = 0;
    }
  }
  // tap / channel of k = kt*BK + 8*kch, advanced incrementally by BK per issued tile
  int a_t, a_c;
  {
    const int kk = kbeg * BK + kch * 8;
    a_t = kk / p.aC;
    a_c = kk - a_t * p.aC;
  }
  // ---- B (N-contig, dgrad): per instruction k-row state
  int b_t[IBW], b_k[IBW], b_col[IBW];
  if constexpr (!BKC) {
#pragma unroll
    for (int i = 0; i < IBW; ++i) {
      const int jb = wave + NW * i;
      const int krow = RPI * jb + lane / CPR;
      b_col[i] = n0 + (((lane % CPR) ^ mn_swz<BN>(krow)) << 3);
      const int kk = kbeg * BK + krow;
      b_t[i] = kk / p.aC;
      b_k[i] = kk - b_t[i] * p.aC;
    }
  }

  auto issue = [&](int kt, int stage) {
    char* st = smem + stage * STAGE;
    const int kk = kt * BK + kch * 8;
    const bool kok = kk < Ktot;
    const int hwv = tap_hw[min(a_t, tlast)];
    const int dh = hwv >> 16, dw = (short)(hwv & 0xffff);
#pragma unroll
    for (int i = 0; i < IAW; ++i) {
      const int ih = a_bh[i] + dh, iw = a_bw[i] + dw;
      const bool ok = kok & (a_img[i] >= 0) & ((unsigned)ih < (unsigned)p.aH) &
                      ((unsigned)iw < (unsigned)p.aW);
      const bf16_t* src = ok ? p.A + (size_t)(a_img[i] + ih * p.aW + iw) * p.aC + a_c
                             : zp;
      glds16(src, st + (wave * IAW + i) * 1024);
    }
    char* bimg = st + A_BYTES;
    if constexpr (BKC) {
#pragma unroll
      for (int i = 0; i < IBW; ++i) {
        const int jb = wave + NW * i;
        if (jb < IB) {
          const int n = n0 + 16 * jb + (lane >> 2);
          const bool ok = kok & (n < p.N);
          // K index of the weight row: GEMM k, or (weight tap of a_t, channel a_c)
          const int kb = p.b_tapmap ? tap_b[min(a_t, tlast)] * p.aC + a_c : kk;
          const bf16_t* src = ok ? p.B + (size_t)n * p.ldb + kb : zp;
          glds16(src, bimg + jb * 1024);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < IBW; ++i) {
        const int jb = wave + NW * i;
        if (jb < IB) {
          const int kr = kt * BK + RPI * jb + lane / CPR;
          const bool ok = (kr < Ktot) & (b_col[i] < p.N);
          const bf16_t* src =
              ok ? p.B + ((size_t)b_k[i] * p.RS + tap_b[min(b_t[i], tlast)]) * p.ldb + b_col[i]
                 : zp;
          glds16(src, bimg + jb * 1024);
          b_k[i] += BK;
          while (b_k[i] >= p.aC) { b_k[i] -= p.aC; ++b_t[i]; }
        }
      }
    }
    a_c += BK;
    while (a_c >= p.aC) { a_c -= p.aC; ++a_t; }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * (BM / WM);
  const int wcol0 = wn * (BN / WN);

  if (kbeg < kend) {
    issue(kbeg, 0);
    if (kbeg + 1 < kend) issue(kbeg + 1, 1);
    int s = 0;
    for (int kt = kbeg; kt < kend; ++kt) {
      if (kt + 1 < kend) wait_barrier<WAITN>();
      else wait_barrier<0>();
      if (kt + 2 < kend) issue(kt + 2, s == 0 ? 2 : s - 1);
      const char* st = smem + s * STAGE;
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
      s = (s == 2) ? 0 : s + 1;
    }
  }
  __syncthreads();  // every DMA waited (vmcnt(0) on the last step); LDS free for the epilogue
  rows_epilogue<BM, BN, WM, WN, SPLIT>(p, acc, smem, mt, m0, n0, wm, wrow0, wcol0, tid, g,
                                       row_base + mt);
}

// ======================================================================================
//  rows kernel, uniform-tap fast path (K-dim channels aC % 32 == 0: every layer but the
//  8-channel stem).  A 32-deep K tile then lies inside one tap, so tap, channel offset and
//  the weight-tap index are wave-uniform scalars per K-step:
//   * A row i keeps a 64-bit base pointer and its (bh, bw) origin; per step its DMA source
//     is base + scalar tap offset, valid iff (bh + dh, bw + dw) is inside the image (two
//     compares) - vs a per-lane tap decode, table lookup and 64-bit multiply-add before;
//   * B rows / columns past the edge are clamped to the last valid one instead of masked:
//     they only feed output rows / columns the epilogue discards, so a B DMA is one
//     64-bit add;
//   * the K loop is unrolled over the 3 ring stages, so every LDS address is an
//     immediate offset.
// PMC on the generic kernel (ResNet-18 layer3, batch 256): 5.5 VALU + 3.6 SALU per MFMA,
// MFMA busy 19 % - issue-bound on address arithmetic, not on LDS or memory.
// ======================================================================================
template <int BM, int BN, int WM, int WN, bool BKC, bool SPLIT, bool PH>
__global__ __launch_bounds__(WM * WN * 64, dma_occ(3 * (BM + BN) * 64 + MAXT * 16, WM * WN))
void igemm_rows_dma_uni_kernel(IGemmArgs p) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, STAGE = A_BYTES + B_BYTES;
  constexpr int IA = BM / 16, IB = BN / 16;
  constexpr int IAW = IA / NW;
  constexpr int IBW = (IB + NW - 1) / NW;
  constexpr int WAITN = IAW + IB / NW;
  constexpr int CPR = BN / 8, RPI = 64 / CPR;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  static_assert(IA % NW == 0 && (NW == 4 || NW == 8), "tile");
  __shared__ __attribute__((aligned(16))) char smem[3 * STAGE + MAXT * 16];
  int* tap_hw = (int*)(smem + 3 * STAGE);  // (dh << 16) | (dw & 0xffff)
  int* tap_b = tap_hw + MAXT;              // weight tap (| super-tap column count << 12)
  int* tap_ab = tap_b + MAXT;              // byte offsets: A pixel shift [MAXT], B tap [MAXT]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  int tile = block_tile(p.tiles_total);
  RowsGeom g{p.M, p.oH, p.oW, p.Poh, p.Pow, p.fd_hw, p.fd_ow};
  int Ktot = p.Ktot, T = p.T, tap0 = 0, kps = p.ktiles_per_split;
  int row_base = 0;  // statistics-slab row of m-tile 0 of this block's phase (dense rows)
  if constexpr (PH) {
    const int ph = tile % p.nphase;
    tile /= p.nphase;
    const PhaseDesc& d = p.ph[ph];
    if (tile >= d.tiles) return;
    for (int q = 0; q < ph; ++q) row_base += p.ph[q].tiles / p.tiles_n;
    g = RowsGeom{d.M, d.oH, d.oW, d.Poh, d.Pow, d.fd_hw, d.fd_ow};
    Ktot = d.Ktot;
    T = d.T;
    tap0 = d.tap0;
    kps = (Ktot + BK - 1) / BK;
  }
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int m0 = mt * BM, n0 = nt * BN;
  const int ktiles = Ktot / BK;  // aC % 32 == 0 => Ktot % 32 == 0
  const int kbeg = block_split() * kps;
  const int kend = min(ktiles, kbeg + kps);
  const int aC = p.aC;

  for (int t = tid; t < T; t += NT) {
    const int dh = p.taps.dh[tap0 + t], dw = p.taps.dw[tap0 + t], bt = p.taps.bt[tap0 + t];
    tap_hw[t] = (dh << 16) | (dw & 0xffff);
    tap_b[t] = bt;
    tap_ab[t] = (dh * p.aW + dw) * aC * 2;
    // (bit 31: a second-source tap, see IGemmArgs::A2; its B rows have stride ldb2)
    tap_ab[MAXT + t] = (PH && (bt & TAP_SRC2)) ? (int)(0x80000000u | (uint32_t)((bt & 0xfff) * aC * 2))
                       : BKC ? (bt & 0xfff) * aC * 2 : (bt & 0xfff) * p.ldb * 2;
  }
  __syncthreads();

  // Operands as buffer descriptors with 32-bit byte offsets (the host keeps both tensors
  // under 2 GiB); a lane past an edge gets offset 2^31 >= num_records and DMAs zeros.  Per
  // K-step an A DMA is one add and one select, a B DMA is free: the weight tap's offset
  // rides in the scalar soffset.  (The 64-bit pointer form cost ~9 VALU + 5 SALU per MFMA:
  // issue-bound, MFMA busy ~25 %.)
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(p.A, 0x7fffffffu);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(p.B, 0x7fffffffu);
  // second source (PH, BKC only): its own descriptors; null -> the first (never selected)
  const __amdgpu_buffer_rsrc_t ra2 = make_rsrc(PH && p.A2 ? p.A2 : p.A, 0x7fffffffu);
  const __amdgpu_buffer_rsrc_t rb2 = make_rsrc(PH && p.B2 ? p.B2 : p.B, 0x7fffffffu);
  const uint32_t s32 = lds_base(smem);
  const int kch = kc_lane_chunk(lane);
  // K elements per tap-table entry: aC, or 32 for super-taps (4 kernel columns x 8 ch), or
  // aC rounded up to 32 (kpad: the chunks past aC read zeros on both operands)
  const int kpt = p.stap ? BK : (p.kpad ? (aC + BK - 1) / BK * BK : aC);
  // ---- A rows (rows past M clamp to M-1: their outputs are discarded)
  uint32_t a_off[IAW];
  int a_bh[IAW], a_bw[IAW];
#pragma unroll
  for (int i = 0; i < IAW; ++i) {
    const int m = min(m0 + 16 * (wave * IAW + i) + (lane >> 2), g.M - 1);
    const int hw = g.oH * g.oW;
    const int img = (int)fdiv((uint32_t)m, g.fd_hw);
    const int r = m - img * hw;
    const int oh = (int)fdiv((uint32_t)r, g.fd_ow);
    a_bh[i] = oh * p.Uh + p.Oh;
    a_bw[i] = (r - oh * g.oW) * p.Uw + p.Ow;
    // (may be "negative" for a padded origin; the valid taps bring it back in range)
    a_off[i] = (uint32_t)((((img * p.aH + a_bh[i]) * p.aW + a_bw[i]) * aC + kch * 8) * 2);
    if (p.stap) a_bw[i] += kch;  // super-tap: chunk kch is the input pixel kch columns right
  }
  // ---- B rows (K-contig) or k-rows x column chunks (N-contig), clamped
  uint32_t b_off[IBW];
#pragma unroll
  for (int i = 0; i < IBW; ++i) {
    const int jb = min(wave + NW * i, IB - 1);
    if constexpr (BKC) {
      const int n = min(n0 + 16 * jb + (lane >> 2), p.N - 1);
      b_off[i] = (uint32_t)((n * p.ldb + kch * 8) * 2);
    } else {
      const int krow = RPI * jb + lane / CPR;
      const int col = min(n0 + (((lane % CPR) ^ mn_swz<BN>(krow)) << 3), p.N - 8);
      b_off[i] = (uint32_t)((krow * p.RS * p.ldb + col) * 2);
    }
  }

  // K-step state (wave-uniform): tap index and channel offset of k = kt * 32
  int t_s = (kbeg * BK) / kpt;
  int c_s = kbeg * BK - t_s * kpt;
  auto issue = [&](uint32_t st) {  // st: the stage's LDS byte address
    const int hwv = __builtin_amdgcn_readfirstlane(tap_hw[t_s]);
    const int dh = hwv >> 16, dw = (short)(hwv & 0xffff);
    const int toff = __builtin_amdgcn_readfirstlane(tap_ab[t_s]) + c_s * 2;
    const int braw = __builtin_amdgcn_readfirstlane(tap_ab[MAXT + t_s]);
    const bool x2 = PH && BKC && braw < 0;  // wave-uniform: a second-source tap
    const __amdgpu_buffer_rsrc_t rA = x2 ? ra2 : ra;
    const __amdgpu_buffer_rsrc_t rB = x2 ? rb2 : rb;
    const bool cok = !p.kpad || c_s + kch * 8 < aC;  // (kpad: this lane's chunk exists)
#pragma unroll
    for (int i = 0; i < IAW; ++i) {
      const bool ok = ((unsigned)(a_bh[i] + dh) < (unsigned)p.aH) &
                      ((unsigned)(a_bw[i] + dw) < (unsigned)p.aW) & cok;
      buf_lds16_at(rA, st + (wave * IAW + i) * 1024, ok ? a_off[i] + toff : 0x80000000u);
    }
    const uint32_t bst = st + A_BYTES;
    const int boff = (braw & 0x7fffffff) + (BKC ? c_s * 2 : c_s * p.RS * p.ldb * 2);
    // super-tap: chunks past the kernel's last column read zeros (ns valid columns)
    const bool bok = (!p.stap || kch < (__builtin_amdgcn_readfirstlane(tap_b[t_s]) >> 12)) & cok;
#pragma unroll
    for (int i = 0; i < IBW; ++i) {
      const int jb = wave + NW * i;
      uint32_t bo = b_off[i];
      if constexpr (PH && BKC) {
        // second-source rows (stride ldb2): recomputed on its few K-steps, not held
        if (x2) bo = (uint32_t)((min(n0 + 16 * min(jb, IB - 1) + (lane >> 2), p.N - 1) * p.ldb2 +
                                 kch * 8) * 2);
      }
      if (jb < IB) buf_lds16_so(rB, bst + jb * 1024, bok ? bo : 0x80000000u, boff);
    }
    c_s += BK;
    if (c_s >= kpt) { c_s = 0; ++t_s; }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wrow0 = wm * (BM / WM);
  const int wcol0 = wn * (BN / WN);

  auto compute = [&](const char* st) {
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
  };

  if (kbeg < kend) {
    issue(s32);
    if (kbeg + 1 < kend) issue(s32 + STAGE);
    int kt = kbeg;
    // one ring revolution per iteration: stage offsets are compile-time constants.  The
    // DMAs are inline asm (invisible to the compiler's waits): the counted wait_barrier is
    // the only thing that orders them before the fragment reads.
    auto step = [&](auto sc) {
      constexpr int S = decltype(sc)::value;
      if (kt + 1 < kend) wait_barrier<WAITN>();
      else wait_barrier<0>();
      if (kt + 2 < kend) issue(s32 + ((S + 2) % 3) * STAGE);
      compute(smem + S * STAGE);
      ++kt;
    };
    while (kt + 3 <= kend) {
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
    }
    if (kt < kend) step(std::integral_constant<int, 0>{});
    if (kt < kend) step(std::integral_constant<int, 1>{});
  }
  __syncthreads();
  rows_epilogue<BM, BN, WM, WN, SPLIT>(p, acc, smem, mt, m0, n0, wm, wrow0, wcol0, tid, g,
                                       row_base + mt);
}

// ======================================================================================
//  wgrad kernel: dW[m = kout][n = (r,s,c)] += sum_pix dy[pix][m] * im2col(x)[pix][n]
// ======================================================================================
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, dma_occ(3 * (BM + BN) * 64, WM * WN))
void igemm_wgrad_dma_kernel(WGradArgs p) {
  constexpr int NW = WM * WN;
  constexpr int NS = 3;
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int CPRA = BM / 8, RPIA = 64 / CPRA;
  constexpr int CPRB = BN / 8, RPIB = 64 / CPRB;
  constexpr int IA = BM / 16, IB = BN / 16;
  constexpr int IAW = (IA + NW - 1) / NW, IBW = (IB + NW - 1) / NW;
  constexpr int WAITN = IA / NW + IB / NW;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  static_assert(NW == 4 || NW == 8, "tile");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

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
  const bf16_t* const zp = (const bf16_t*)g_zero16;

  // ---- A (dy, [pix][Kout]): per instruction pixel row and output-channel chunk
  int a_row[IAW], a_m[IAW];
#pragma unroll
  for (int i = 0; i < IAW; ++i) {
    const int ja = wave + NW * i;
    a_row[i] = RPIA * ja + lane / CPRA;
    a_m[i] = m0 + (((lane % CPRA) ^ mn_swz<BM>(a_row[i])) << 3);
  }
  // ---- B (im2col(x)): per instruction column decode n -> (dh, dw, c) and pixel iterator
  const int PQ = p.P * p.Q;
  int b_dh[IBW], b_dw[IBW], b_c[IBW], b_img[IBW], b_oh[IBW], b_ow[IBW];
  bool b_ok[IBW];
#pragma unroll
  for (int i = 0; i < IBW; ++i) {
    const int jb = wave + NW * i;
    const int krow = RPIB * jb + lane / CPRB;
    const int n = n0 + (((lane % CPRB) ^ mn_swz<BN>(krow)) << 3);
    const int tap = n / p.C;
    const int r = tap / p.S;
    b_dh[i] = r - p.ph;
    b_dw[i] = tap - r * p.S - p.pw;
    b_c[i] = n - tap * p.C;
    b_ok[i] = n < p.Ncols;
    const int pix = kbeg * BK + krow;
    const int img = pix / PQ;
    const int rr = pix - img * PQ;
    b_img[i] = img;
    b_oh[i] = rr / p.Q;
    b_ow[i] = rr - b_oh[i] * p.Q;
  }

  auto issue = [&](int kt, int stage) {
    char* st = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < IAW; ++i) {
      const int ja = wave + NW * i;
      if (ja < IA) {
        const int pix = kt * BK + a_row[i];
        const bool ok = (pix < p.Mpix) & (a_m[i] < p.Kout);
        const bf16_t* src = ok ? p.dy + (size_t)pix * p.Kout + a_m[i] : zp;
        glds16(src, st + ja * 1024);
      }
    }
    char* bimg = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < IBW; ++i) {
      const int jb = wave + NW * i;
      if (jb < IB) {
        const int pix = kt * BK + RPIB * jb + lane / CPRB;
        const int ih = b_oh[i] * p.sh + b_dh[i], iw = b_ow[i] * p.sw + b_dw[i];
        const bool ok = b_ok[i] & (pix < p.Mpix) & ((unsigned)ih < (unsigned)p.H) &
                        ((unsigned)iw < (unsigned)p.W);
        const bf16_t* src =
            ok ? p.x + (((size_t)b_img[i] * p.H + ih) * p.W + iw) * p.C + b_c[i]
               : zp;
        glds16(src, bimg + jb * 1024);
        if (PQ == 1) {  // Linear (1x1 "image"): the pixel IS the image index
          b_img[i] += BK;
        } else {
          int ow = b_ow[i] + BK, oh = b_oh[i], img = b_img[i];
          while (ow >= p.Q) { ow -= p.Q; ++oh; }
          while (oh >= p.P) { oh -= p.P; ++img; }
          b_ow[i] = ow; b_oh[i] = oh; b_img[i] = img;
        }
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

  issue(kbeg, 0);
  if (kbeg + 1 < kend) issue(kbeg + 1, 1);
  int s = 0;
  for (int kt = kbeg; kt < kend; ++kt) {
    if (kt + 1 < kend) wait_barrier<WAITN>();
    else wait_barrier<0>();
    if (kt + 2 < kend) issue(kt + 2, s == 0 ? 2 : s - 1);
    const char* st = smem + s * STAGE;
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
    s = (s == 2) ? 0 : s + 1;
  }
  wgrad_epilogue<BM, BN, WM, WN>(p, acc, m0, n0, wrow0, wcol0, lane);
}

// ======================================================================================
//  wgrad kernel, incremental fast path.  Each lane's pixel (kt*32 + its k-row) advances
//  by exactly 32 per K-step, i.e. by (dP, dQ) = (32 / Q, 32 % Q) output rows/cols; with
//  32/Q + 1 <= P the column wrap and the image wrap are each ONE conditional, so the
//  lane keeps (oh*sh, ow*sw, input element offset) as 32-bit state updated by scalar
//  constants with no division, no 64-bit multiply and no divergent loop.  Output
//  channels past Kout and columns past R*S*C are clamped instead of masked (their
//  results are never stored); pixels past Mpix read the zero page.
// ======================================================================================
struct WInc {   // per-launch scalar constants of the pixel walk
  int dq_s, dp_s;          // sw * (32 % Q), sh * (32 / Q): per-step ow*sw / oh*sh advance
  int qwrap, pwrap;        // Q * sw, P * sh: wrap thresholds of ow*sw and oh*sh
  int step_off;            // input offset advance per step (no wrap)
  int qwrap_off, pwrap_off;  // extra input offset on a column / image wrap
};

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64, dma_occ(3 * (BM + BN) * 64, WM * WN))
void igemm_wgrad_dma_inc_kernel(WGradArgs p, WInc w) {
  constexpr int NW = WM * WN;
  constexpr int A_BYTES = BK * BM * 2, B_BYTES = BK * BN * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int CPRA = BM / 8, RPIA = 64 / CPRA;
  constexpr int CPRB = BN / 8, RPIB = 64 / CPRB;
  constexpr int IA = BM / 16, IB = BN / 16;
  constexpr int IAW = (IA + NW - 1) / NW, IBW = (IB + NW - 1) / NW;
  constexpr int WAITN = IA / NW + IB / NW;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  static_assert(NW == 4 || NW == 8, "tile");
  __shared__ __attribute__((aligned(16))) char smem[3 * STAGE];

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
  const bf16_t* const zp = (const bf16_t*)g_zero16;

  // ---- A (dy [pix][Kout]): row pointer walks by 32 pixels per step
  const bf16_t* a_ptr[IAW];
  int a_pix[IAW];
#pragma unroll
  for (int i = 0; i < IAW; ++i) {
    const int ja = min(wave + NW * i, IA - 1);
    const int row = RPIA * ja + lane / CPRA;
    const int m = min(m0 + (((lane % CPRA) ^ mn_swz<BM>(row)) << 3), p.Kout - 8);
    a_pix[i] = kbeg * BK + row;
    a_ptr[i] = p.dy + (size_t)a_pix[i] * p.Kout + m;
  }
  // ---- B (im2col(x)): fixed column (tap, channel) + incremental pixel state
  int b_dh[IBW], b_dw[IBW], b_col[IBW], b_pix[IBW], b_ohs[IBW], b_ows[IBW], b_off[IBW];
  const int PQ = p.P * p.Q;
#pragma unroll
  for (int i = 0; i < IBW; ++i) {
    const int jb = min(wave + NW * i, IB - 1);
    const int krow = RPIB * jb + lane / CPRB;
    const int n = min(n0 + (((lane % CPRB) ^ mn_swz<BN>(krow)) << 3), p.Ncols - 8);
    const int tap = n / p.C;
    const int r = tap / p.S;
    b_dh[i] = r - p.ph;
    b_dw[i] = tap - r * p.S - p.pw;
    b_col[i] = (b_dh[i] * p.W + b_dw[i]) * p.C + (n - tap * p.C);
    const int pix = kbeg * BK + krow;
    const int img = pix / PQ;
    const int rr = pix - img * PQ;
    const int oh = rr / p.Q;
    const int ow = rr - oh * p.Q;
    b_pix[i] = pix;
    b_ohs[i] = oh * p.sh;
    b_ows[i] = ow * p.sw;
    b_off[i] = ((img * p.H + b_ohs[i]) * p.W + b_ows[i]) * p.C;
  }

  auto issue = [&](char* st) {
#pragma unroll
    for (int i = 0; i < IAW; ++i) {
      const int ja = wave + NW * i;
      if (ja < IA) {
        glds16(a_pix[i] < p.Mpix ? a_ptr[i] : zp, st + ja * 1024);
        a_pix[i] += BK;
        a_ptr[i] += (size_t)BK * p.Kout;
      }
    }
    char* bimg = st + A_BYTES;
#pragma unroll
    for (int i = 0; i < IBW; ++i) {
      const int jb = wave + NW * i;
      if (jb < IB) {
        const bool ok = (b_pix[i] < p.Mpix) &
                        ((unsigned)(b_ohs[i] + b_dh[i]) < (unsigned)p.H) &
                        ((unsigned)(b_ows[i] + b_dw[i]) < (unsigned)p.W);
        glds16(ok ? p.x + (b_off[i] + b_col[i]) : zp, bimg + jb * 1024);
        // advance this lane's pixel by 32: at most one column wrap, one image wrap
        b_pix[i] += BK;
        b_ows[i] += w.dq_s;
        b_ohs[i] += w.dp_s;
        b_off[i] += w.step_off;
        const bool qw = b_ows[i] >= w.qwrap;
        b_ows[i] -= qw ? w.qwrap : 0;
        b_ohs[i] += qw ? p.sh : 0;
        b_off[i] += qw ? w.qwrap_off : 0;
        const bool pw_ = b_ohs[i] >= w.pwrap;
        b_ohs[i] -= pw_ ? w.pwrap : 0;
        b_off[i] += pw_ ? w.pwrap_off : 0;
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
  auto compute = [&](const char* st) {
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
  };

  issue(smem);
  if (kbeg + 1 < kend) issue(smem + STAGE);
  int kt = kbeg;
  auto step = [&](auto sc) {
    constexpr int S = decltype(sc)::value;
    if (kt + 1 < kend) wait_barrier<WAITN>();
    else wait_barrier<0>();
    if (kt + 2 < kend) issue(smem + ((S + 2) % 3) * STAGE);
    compute(smem + S * STAGE);
    ++kt;
  };
  while (kt + 3 <= kend) {
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
  }
  if (kt < kend) step(std::integral_constant<int, 0>{});
  if (kt < kend) step(std::integral_constant<int, 1>{});
  wgrad_epilogue<BM, BN, WM, WN>(p, acc, m0, n0, wrow0, wcol0, lane);
}

// ======================================================================================
//  host launchers (plans are made by igemm.hip)
// ======================================================================================
// uniform-tap fast path on/off (A/B and cross-checking; MPA_DMA_UNI=0 disables)
static bool g_dma_uni = [] {
  const char* e = getenv("MPA_DMA_UNI");
  return !(e && e[0] == '0');
}();
void igemm_set_dma_uni(int on) { g_dma_uni = on != 0; }
bool igemm_stap_ok() { return g_dma_uni && igemm_engine() >= 1; }
// byte extents of the rows kernel's operands: the uniform-tap kernel addresses both with
// 32-bit offsets
static bool rows_uni_fits(const IGemmArgs& a, bool bkc) {
  const PhaseDesc* d = a.nphase > 0 ? &a.ph[0] : nullptr;
  const int64_t hw = d ? (int64_t)d->oH * d->oW : (int64_t)a.oH * a.oW;
  const int64_t m = d ? d->M : a.M;
  const int64_t nimg = hw > 0 ? (m + hw - 1) / hw : 0;
  const int64_t abytes = nimg * a.aH * a.aW * a.aC * 2;
  const int64_t bbytes = (bkc ? (int64_t)a.N : (int64_t)a.aC * a.RS) * a.ldb * 2;
  const int64_t b2bytes = (int64_t)a.N * a.ldb2 * 2;
  return abytes < (1ll << 31) && bbytes < (1ll << 31) && b2bytes < (1ll << 31);
}

// a second GEMM source is read only by the uniform-tap kernel's phase form with K-contiguous
// B (launch_rows_dma_v picks that kernel under exactly these conditions)
// kpad form available: the uniform-tap kernel with K-contiguous B takes the launch
bool igemm_rows_kpad_ok(const IGemmArgs& a, bool bkc) {
  return bkc && g_dma_uni && !a.stap && a.nphase == 0 && a.aC % BK != 0 && a.aC % 8 == 0 &&
         rows_uni_fits(a, bkc);
}

bool igemm_rows_uni_src2_ok(const IGemmArgs& a, bool bkc) {
  return bkc && a.nphase > 0 && a.aC % BK == 0 && !a.stap && g_dma_uni && rows_uni_fits(a, bkc);
}

template <int BM, int BN, int WM, int WN, bool BKC, bool SPLIT, bool PH>
static void launch_rows_dma_v(const IGemmArgs& a0, dim3 grid, hipStream_t s) {
  IGemmArgs a = a0;
  igemm_set_fastdiv(a);
  if ((a.aC % BK == 0 || a.stap || (a.kpad && BKC)) && g_dma_uni && rows_uni_fits(a, BKC))
    hipLaunchKernelGGL((igemm_rows_dma_uni_kernel<BM, BN, WM, WN, BKC, SPLIT, PH>), grid,
                       dim3(WM * WN * 64), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_rows_dma_kernel<BM, BN, WM, WN, BKC, SPLIT, PH>), grid,
                       dim3(WM * WN * 64), 0, s, a);
}

template <int BM, int BN, int WM, int WN, bool BKC>
static void launch_rows_dma(const IGemmArgs& a, int splits, hipStream_t s) {
  dim3 grid(a.tiles_total, 1, splits);
  if (a.nphase > 0) {  // merged stride phases (dgrad): never split
    launch_rows_dma_v<BM, BN, WM, WN, BKC, false, true>(a, grid, s);
    return;
  }
  if (splits > 1) launch_rows_dma_v<BM, BN, WM, WN, BKC, true, false>(a, grid, s);
  else launch_rows_dma_v<BM, BN, WM, WN, BKC, false, false>(a, grid, s);
}

template <bool BKC>
static bool rows_dma_tile(const IGemmArgs& a, int BM, int BN, int splits, hipStream_t s) {
  if (BM == 256 && BN == 256) launch_rows_dma<256, 256, 2, 4, BKC>(a, splits, s);
  else if (BM == 256 && BN == 128) launch_rows_dma<256, 128, 2, 2, BKC>(a, splits, s);
  else if (BM == 128 && BN == 128) launch_rows_dma<128, 128, 2, 2, BKC>(a, splits, s);
  else if (BM == 256 && BN == 64) launch_rows_dma<256, 64, 4, 1, BKC>(a, splits, s);
  else if (BM == 128 && BN == 64) launch_rows_dma<128, 64, 2, 2, BKC>(a, splits, s);
  else if (BM == 128 && BN == 32) launch_rows_dma<128, 32, 4, 1, BKC>(a, splits, s);
  else return false;
  return true;
}

bool igemm_rows_dma(const IGemmArgs& a, int BM, int BN, bool bkc, int splits, hipStream_t s) {
  return bkc ? rows_dma_tile<true>(a, BM, BN, splits, s) : rows_dma_tile<false>(a, BM, BN, splits, s);
}

// incremental pixel walk applicable: one wrap per step suffices, 32-bit offsets, and
// 16-B granular operands on both sides (callers guarantee Kout % 8 == 0, C % 8 == 0)
bool igemm_wgrad_inc_ok(const WGradArgs& a) {
  return g_dma_uni && (BK / a.Q) + 1 <= a.P && a.Ncols >= 8 && a.Kout >= 8 &&
         (int64_t)a.Mpix / (a.P * a.Q) * a.H * a.W * a.C < (1ll << 31);
}

template <int BM, int BN, int WM, int WN>
static void launch_wgrad_inc(const WGradArgs& a, dim3 grid, hipStream_t s) {
  WInc w;
  w.dq_s = a.sw * (BK % a.Q);
  w.dp_s = a.sh * (BK / a.Q);
  w.qwrap = a.Q * a.sw;
  w.pwrap = a.P * a.sh;
  w.step_off = (w.dp_s * a.W + w.dq_s) * a.C;
  w.qwrap_off = (a.sh * a.W - a.Q * a.sw) * a.C;
  w.pwrap_off = (a.H - a.P * a.sh) * a.W * a.C;
  hipLaunchKernelGGL((igemm_wgrad_dma_inc_kernel<BM, BN, WM, WN>), grid, dim3(WM * WN * 64), 0,
                     s, a, w);
}

bool igemm_wgrad_dma(const WGradArgs& a, int BM, int BN, int splits, hipStream_t s) {
  dim3 grid(a.tiles_total, 1, splits);
  // incremental kernel for the 4-wave tiles; the 8-wave tiles keep the generic kernel
  // (the extra per-lane pixel state costs them their second block per CU: 124 -> 166 VGPR)
  if (igemm_wgrad_inc_ok(a) && BN == 128 && (BM == 128 || BM == 64)) {
    if (BM == 128) launch_wgrad_inc<128, 128, 2, 2>(a, grid, s);
    else launch_wgrad_inc<64, 128, 2, 2>(a, grid, s);
    return true;
  }
  if (BM == 256 && BN == 256)
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<256, 256, 2, 4>), grid, dim3(512), 0, s, a);
  else if (BM == 128 && BN == 256)
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<128, 256, 2, 4>), grid, dim3(512), 0, s, a);
  else if (BM == 64 && BN == 256)
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<64, 256, 2, 4>), grid, dim3(512), 0, s, a);
  else if (BM == 128 && BN == 128)
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<128, 128, 2, 2>), grid, dim3(256), 0, s, a);
  else if (BM == 64 && BN == 128)
    hipLaunchKernelGGL((igemm_wgrad_dma_kernel<64, 128, 2, 2>), grid, dim3(256), 0, s, a);
  else
    return false;
  return true;
}

}  // namespace mpa
