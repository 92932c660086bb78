// Halo-staged direct 3x3 / stride-1 convolution for gfx950 (MI355X / CDNA4): the forward
// and the stride-1 dgrad of every 3x3 "same" conv (ResNet-18 has 13
// such convs = 26 of its 34 rows-GEMM launches per step).
//
// Why a second engine: the implicit GEMM (igemm_dma.hip) gathers a fresh A tile for every
// tap, so each input pixel crosses L2 -> LDS nine times and the weight tile once per
// 128-row M-tile: 21 (64-channel) to 32 (128-channel) MAC per staged byte.  The measured
// L2 -> LDS gather rate is ~30 B/clk/CU (MI355X_MICROARCH.md "Indexed rows") against 2048
// bf16 MAC/clk/CU of MFMA, so those layers ran at 16-25 % of the matrix peak
// (profiles/conv_kernels_tuned_b256.txt).  Here a block stages, per 32-channel chunk, the
// input rows its 256 output pixels touch plus a one-pixel halo ONCE, and runs all nine taps
// out of LDS: 67-77 MAC per staged byte, and 185 when the whole weight tile stays resident.
//
//  * LDS halo image: "slots" of P pixels, one input row per slot, P = W + 1 rounded up to
//    8: a row's right border column is the next row's left border (one shared zero column),
//    and one zero slot separates consecutive images, so every tap is a uniform pixel offset
//    dh*P + dw and no lane ever tests a border.  Slot s of a tile whose first output row
//    is (img0, oh0) holds input row v = s + oh0 - 1 of the image sequence with period H+1
//    (row H of each period = the zero separator).
//  * Pixel rows are 64 B (32 bf16 channels, four 16-B chunks).  Chunk c of row r sits at
//    position c ^ (2 * ((r >> 2) & 1)): a fragment read (ds_read_b128, lane l: row l%16,
//    chunk l/16) of ANY 16 consecutive rows - the taps shift halo rows by arbitrary
//    amounts - touches every bank once per lane group (brute-force checked for all 64
//    alignments; the engine's aligned-row swizzle kc_off conflicts 2-way off alignment).
//    The weight image [tap][64 cols][32 k] uses the same rows and swizzle.  P % 8 == 0, so
//    a row tap never moves the swizzle bit and A addresses are precomputed per column tap.
//  * Staging is buffer_load_dwordx4 ... lds: the swizzle moves to the source (lane on
//    chunk position q of row r fetches chunk q ^ (2 * ((r>>2)&1))), border / out-of-tensor
//    lanes get an offset past num_records and the hardware returns zeros, the chunk step
//    moves the descriptor base (scalar), so a DMA costs no VALU.  The next item's DMAs are
//    issued inside the current item's MFMA stream (an LDS-DMA costs its wave 60-180
//    cycles of issue; as a burst in front of the wait they stalled every item).
//  * Persistent blocks (one 4-wave block per CU, 146 KiB LDS): work items (tile, chunk) run
//    through a 2-stage ring; XCD x owns a contiguous share of the tile list.
//  * WRES (64-wide outputs, <= 64 input channels, e.g. ResNet layer1): the 64 x 9 x C weight
//    tile is loaded once per block and only the halo streams.
//  * Lean epilogue (bias, ReLU, BN statistics, fused BN-backward reduction, accumulate for
//    GradJoin) after each tile; BN statistics accumulate in registers across all of a
//    block's tiles and are written once per block.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <type_traits>
#include "igemm_common.h"

namespace mpa {

constexpr int HB_BM = 256, HB_BN = 64, HB_NW = 4;
constexpr int HB_HIW = 9;                       // halo DMA instructions per wave per chunk
constexpr int HB_HPX = 16 * HB_NW * HB_HIW;     // 576 halo pixels per chunk
constexpr int HB_HBYTES = HB_HPX * 64;          // 36 KiB
constexpr int HB_WIW = 9;                       // weight DMA instructions per wave per chunk
constexpr int HB_WBYTES = 9 * HB_BN * 64;       // 36 KiB: [tap][64 cols][32 k]
constexpr int HB_RED = HB_NW * HB_BN * 2 * 4;   // epilogue cross-wave statistics
constexpr int HB_COLS = 4 * HB_BN * 4;          // per-column epilogue operands [4][64]
constexpr int HB_LDS = 2 * HB_HBYTES + 2 * HB_WBYTES + HB_RED + HB_COLS;  // 150,528 B

struct HaloPlan {
  int w2;               // halo row pitch P: W + 1 (one shared zero column) rounded up to 8
  int btoff[9];         // tap t = (dh + 1) * 3 + (dw + 1): byte offset bt * aC * 2 of its
                        // weight row segment (the host orders any 3x3 tap table this way)
  uint32_t mag_w, mag_w2, mag_h1, mag_hw;  // floor(2^32 / d) + 1: exact n / d for n*d < 2^32
  int tiles_m, tiles_total, cc;
  uint32_t a_bytes, b_bytes;
};

__device__ __forceinline__ bf16x8 frag16(const char* lds_byte) {
  return __builtin_bit_cast(bf16x8, *LDS_PTR(const u32x4, lds_byte));
}

// Epilogue flavours (compile-time, so the fused epilogue below is one straight-line block)
enum : int { EP_RELU = 1, EP_BETA = 2, EP_BNRED = 4, EP_STATS = 8, EP_BIAS = 16 };

// Per-tile operands the epilogue reads from memory (accumulate: the old output; fused
// BN-backward reduction: z, whose ReLU mask is recomputed like bn_fwd_train rounded y, so
// y is never read), loaded at the start of the tile's second-to-last item so they are in
// registers long before the epilogue runs.
template <int MI = 4>
struct EpiInT {
  uint2 a[MI][4];
  uint2 mk[MI];  // (accumulate from ep_res) row i's 64 ReLU mask bits of the column tile
};
typedef EpiInT<4> EpiIn;

// the accumulate operand of element e: the old output, or the residual gradient ep_res
// (its ReLU mask is applied at the epilogue, see masked_acc: applying it here would make the
// MFMA waves wait for the mask load at preload time)
__device__ __forceinline__ uint2 acc_operand(const IGemmArgs& p, uint32_t e) {
  return *(const uint2*)((const bf16_t*)(p.ep_res ? p.ep_res : p.C) + e);
}

// row i's 64 mask bits of the block's column tile (row element e0 = m * ldc + n0, n0 % 64 == 0)
__device__ __forceinline__ uint2 acc_mask(const IGemmArgs& p, uint32_t e0) {
  return p.ep_rmask ? *(const uint2*)(p.ep_rmask + (e0 >> 3)) : make_uint2(~0u, ~0u);
}

// fragment (jn, jq)'s 4 channels 16 jn + 4 jq .. +3 of the preloaded operand, masked
__device__ __forceinline__ uint2 masked_acc(uint2 v, uint2 mk, int jn, int jq) {
  const uint32_t word = jn < 2 ? mk.x : mk.y;
  const uint32_t nib = (word >> ((16 * jn + 4 * jq) & 31)) & 15u;
  v.x &= ((nib & 1u) ? 0xffffu : 0u) | ((nib & 2u) ? 0xffff0000u : 0u);
  v.y &= ((nib & 4u) ? 0xffffu : 0u) | ((nib & 8u) ? 0xffff0000u : 0u);
  return v;
}

template <int EPI, int NJ, int MI = 4>
__device__ __forceinline__ void epi_preload(const IGemmArgs& p, EpiInT<MI>& in, int m0, int n0,
                                            int wave, int lane) {
  if constexpr (!(EPI & (EP_BETA | EP_BNRED))) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int jn = 0; jn < 4; ++jn) in.a[i][jn] = make_uint2(0u, 0u);
  } else {
    const int nl = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = min(m0 + wave * 16 * MI + i * 16 + (lane & 15), p.M - 1);  // rows >= M: unused
      const uint32_t orow = (uint32_t)m * p.ldc + n0 + nl;
      if constexpr (!(EPI & EP_BNRED)) in.mk[i] = acc_mask(p, (uint32_t)m * p.ldc + n0);
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) {
        if constexpr (EPI & EP_BNRED) {
          in.a[i][jn] = *(const uint2*)(p.ep_z + orow + jn * 16);
        } else {
          in.a[i][jn] = acc_operand(p, orow + jn * 16);
        }
      }
    }
  }
}

__device__ __forceinline__ float lo_f(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Epilogue of one 256 x 64 tile (lane: 4 consecutive channels n = n0 + 16 jn + 4 (lane/16)
// of pixel m = m0 + 64 wave + 16 i + lane%16).  N % 64 == 0 (no column guards), dense
// [M][ldc] output with 32-bit offsets, per-column operands in registers for the block's
// whole life (its column tile never changes), and the BN statistics accumulated in
// registers across ALL of the block's tiles (ss/sq), reduced and written once per block by
// halo_stats_flush.  epi_frag handles fragment (i, jn); the fused form calls it between the
// next tile's taps (branch-free), the MASKED form after the block's last tile.
// (BN reduction: cb / cs = mean / rstd, mc / mh = bn_fwd_train's scale / shift)
template <int EPI, bool FULL, bool ST = true>
__device__ __forceinline__ uint2 epi_frag(const IGemmArgs& p, const f32x4& acc, uint2 ia, bool ok,
                                         int jn, uint32_t orow, const f32x4& cb, const f32x4& cs,
                                         const f32x4& mc, const f32x4& mh, float (&ssj)[4],
                                         float (&sqj)[4]) {
  bf16_t* const out = (bf16_t*)p.C;
  float v[4];
  if constexpr (EPI & EP_BNRED) {
    // dy (bf16-rounded) masked by ReLU(bn(z)) > 0; reduction (sum g, sum g * xhat)
    const uint2 z = ia;
    const float zr[4] = {lo_f(z.x), hi_f(z.x), lo_f(z.y), hi_f(z.y)};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float d = bf2f(f2bf(acc[r]));
      const bool live = bf2f(f2bf(__builtin_fmaf(zr[r], mc[r], mh[r]))) > 0.f;
      v[r] = ((FULL || ok) && live) ? d : 0.f;
      ssj[r] += v[r];
      sqj[r] += v[r] * (zr[r] - cb[r]) * cs[r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (EPI & EP_BIAS) ? acc[r] + cb[r] : acc[r];
    if constexpr (EPI & EP_BETA) {
      const uint2 o = ia;
      v[0] += lo_f(o.x); v[1] += hi_f(o.x); v[2] += lo_f(o.y); v[3] += hi_f(o.y);
    }
    if constexpr (EPI & EP_RELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
    }
  }
  const uint32_t lo = pack2(v[0], v[1]), hi = pack2(v[2], v[3]);
  if constexpr (ST) {
    if (FULL || ok) *(uint2*)(out + orow + jn * 16) = make_uint2(lo, hi);
  }
  if constexpr ((EPI & EP_STATS) && !(EPI & EP_BNRED)) {
    // shifted statistics of the bf16-rounded values BN will read
    float rv[4] = {lo_f(lo) - cs[0], hi_f(lo) - cs[1], lo_f(hi) - cs[2], hi_f(hi) - cs[3]};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (!FULL) rv[r] = ok ? rv[r] : 0.f;
      ssj[r] += rv[r];
      sqj[r] += rv[r] * rv[r];
    }
  }
  return make_uint2(lo, hi);
}

// 16-B epilogue stores (round 6; MI300-class store-issue rule, cdna_hip_programming.md T21):
// a lane holds 4 channels of column groups jn and jn + 1 of one pixel; v_permlane16_swap
// trades the even lane row's jn + 1 half for the odd row's jn half, so the even lane
// (jq = 0, 2) writes channels 16 jn + 4 jq .. + 7 and the odd lane (jq = 1, 3) channels
// 16 (jn + 1) + 4 (jq - 1) .. + 7: one dwordx4 per lane and fragment pair instead of two
// scattered dwordx2 (same bytes, half the store instructions).  prow = m * ldc + n0.
__device__ __forceinline__ void store_pair16(bf16_t* out, uint32_t prow, int jn, int jq,
                                             uint2 x, uint2 y, bool ok) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(x.x, y.x, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x.y, y.y, false, false);
  const uint32_t off = prow + jn * 16 + jq * 4 + ((jq & 1) ? 12 : 0);
  if (ok) *(uint4*)(out + off) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
}

// Sum over the 16 lanes of a DPP row (the 16 pixel lanes of one column group), result in
// every lane of the row: quad swaps, then the half-row and row mirrors (4 VALU ops).
__device__ __forceinline__ float row16_sum(float v) {
  auto dpp = [](float x, auto ctrl) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x),
                                                              decltype(ctrl)::value, 0xF, 0xF,
                                                              true));
  };
  v += dpp(v, std::integral_constant<int, 0xB1>{});   // quad_perm [1,0,3,2]
  v += dpp(v, std::integral_constant<int, 0x4E>{});   // quad_perm [2,3,0,1]
  v += dpp(v, std::integral_constant<int, 0x141>{});  // row_half_mirror
  v += dpp(v, std::integral_constant<int, 0x140>{});  // row_mirror
  return v;
}

// Block-level statistics: reduce the per-lane sums of the block's tiles and write slab row
// blockIdx.x ([2][N]: the block's 64 columns, zeros elsewhere, so every row is complete);
// block 0 zeroes the final-sum vector the slab reduction accumulates into.
// TRED: the per-wave sums are already in `red` (per-tile LDS accumulation).
template <bool TRED = false>
__device__ __forceinline__ void halo_stats_flush(const IGemmArgs& p, float (&ss)[4][4],
                                                 float (&sq)[4][4], char* red, int n0, int wave,
                                                 int tid) {
  const int lane = tid & 63, nl = (lane >> 4) * 4;
  float* rd = (float*)red;
  if constexpr (!TRED) {
#pragma unroll
  for (int jn = 0; jn < 4; ++jn)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = ss[jn][r], b = sq[jn][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
      }
      ss[jn][r] = a;
      sq[jn][r] = b;
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int jn = 0; jn < 4; ++jn)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rd[(wave * 64 + jn * 16 + nl + r) * 2] = ss[jn][r];
        rd[(wave * 64 + jn * 16 + nl + r) * 2 + 1] = sq[jn][r];
      }
  }
  }
  __syncthreads();
  float* row = p.stats + (size_t)blockIdx.x * 2 * p.N;
  for (int c = tid; c < p.N; c += 256) {
    float a = 0.f, b = 0.f;
    if (c >= n0 && c < n0 + 64) {
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        a += rd[(w * 64 + c - n0) * 2];
        b += rd[(w * 64 + c - n0) * 2 + 1];
      }
    }
    row[c] = a;
    row[p.N + c] = b;
    if (blockIdx.x == 0) {
      p.stats_sums[c] = 0.f;
      p.stats_sums[p.N + c] = 0.f;
    }
  }
}

// NJ: 16-column fragment groups per wave (4: 64-wide column tiles; 2: N == 32 - the weight
// image's upper 32 columns are zero-filled DMAs and never read, no MFMA touches them)
// MI: 16-pixel row fragments per MFMA wave.  4: 256-pixel linear tiles (576-pixel halo
// stages, 9 DMAs per producer wave).  7 (round 6, resident weights): 448-pixel tiles of 8
// whole image rows (ResNet layer1, W = 56): the 10-slot halo stage (640 pixels, 10 DMAs per
// producer wave) feeds 1.75x the MFMA work of a 576-pixel stage, so the layer's staging -
// HBM-latency-bound at one item in flight per CU (tools/dma_probe.hip) - is paid per 448
// output pixels instead of per 256; A fragments stream one row fragment behind its MFMAs.
template <bool WRES, int EPI, bool FULL, int NJ, int MI = 4>
__global__ __launch_bounds__(MI == 4 ? 512 : 256, 1) void conv3_halo_kernel(IGemmArgs p,
                                                                          HaloPlan h) {
  // SELF (MI = 7): 4-wave blocks whose MFMA waves issue their own DMAs.  The 448-pixel
  // tile's 112 accumulator registers do not fit the 256 registers per wave of an 8-wave
  // block (92-158 B/lane of scratch, 1.8x slower); alone on its SIMD a wave has 512.
  constexpr bool SELF = MI != 4;
  // 16-B epilogue stores (store_pair16) in the 448-pixel flavours; the 256-pixel ones keep
  // 8-B stores (their pair form spills 1-18 B/lane at 256 registers)
  constexpr bool WIDE = SELF;
  constexpr int BM = 64 * MI;                        // tile pixels: 16 MI per MFMA wave
  constexpr int HIW = MI == 4 ? HB_HIW : 10;         // halo DMAs per producer wave per item
  constexpr int HBYTES = 16 * HB_NW * HIW * 64;      // halo stage bytes
  static_assert(MI == 4 || (MI == 7 && WRES), "448-pixel tiles: resident weights only");
  static_assert(2 * HBYTES + 2 * HB_WBYTES + HB_RED + HB_COLS <= 163840, "LDS budget");
  __shared__ __attribute__((aligned(16))) char smem[2 * HBYTES + 2 * HB_WBYTES + HB_RED + HB_COLS];
  char* const hal = smem;
  char* const wst = smem + 2 * HBYTES;
  char* const red = smem + 2 * HBYTES + 2 * HB_WBYTES;
  float* const cst = (float*)(red + HB_RED);  // [4][64] per-column epilogue operands

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wave_all & (HB_NW - 1);  // MFMA wave / DMA lane group
  const int H = p.aH, W = p.aW, HW = H * W, W2 = h.w2, aC = p.aC;
  const int nimg = p.M / HW;
  const int jq = lane >> 4, l15 = lane & 15;

  // persistent tile list: XCD x = blockIdx % 8 owns tiles [x*T/8, (x+1)*T/8); the host
  // makes G8 a multiple of tiles_n, so a block's tiles all share one column tile nt
  const int T = h.tiles_total;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, G8 = gridDim.x >> 3;
  const int tbeg = (int)((int64_t)xcd * T / 8), tend = (int)((int64_t)(xcd + 1) * T / 8);
  const int ntiles = tbeg + loc < tend ? (tend - tbeg - loc + G8 - 1) / G8 : 0;
  const int CC = h.cc;
  const int nitems = ntiles * CC;
  const int nt = (tbeg + loc) % p.tiles_n;
  const int n0 = nt * HB_BN;
  auto tile_of = [&](int tk) { return tbeg + loc + tk * G8; };
  auto m0_of = [&](int tk) { return (tile_of(tk) / p.tiles_n) * BM; };

  // ---- staging: the DMA lanes of lane group `wave` and the instructions of one item
  auto stager = [&](auto body) {
    // halo lanes: tile-independent (slot, column, logical chunk) of each DMA lane
    uint32_t hsc[HIW];  // slot | (col + 1) << 10 | chunk << 18
#pragma unroll
    for (int j = 0; j < HIW; ++j) {
      const uint32_t hp = 16 * (wave * HIW + j) + (lane >> 2);
      const uint32_t s = udiv(hp, h.mag_w2);
      const uint32_t colp = hp - s * W2;
      const uint32_t lc = (lane & 3) ^ (((hp >> 2) & 1) << 1);
      hsc[j] = s | (colp << 10) | (lc << 18);
    }
    // weight lanes: row r = 16 q + lane/4 of the [tap][64][32] image, tap = q / 4; the
    // block's column tile is fixed, so the offsets are too
    uint32_t wv[HB_WIW];
#pragma unroll
    for (int j = 0; j < HB_WIW; ++j) {
      const int q = wave * HB_WIW + j;
      const int r = 16 * q + (lane >> 2);
      const int n = r & 63;
      const int lc = (lane & 3) ^ (((r >> 2) & 1) << 1);
      wv[j] = (n0 + n < p.N) ? (uint32_t)(n0 + n) * p.ldb * 2 + h.btoff[q >> 2] + lc * 16
                             : 0x80000000u;
    }
    uint32_t hv[HIW];
    auto prep_tile = [&](int tk) {  // DMA source offsets of a tile's halo
      const int m0 = m0_of(tk);
      const int img0 = m0 / HW;
      const int oh0 = (m0 - img0 * HW) / W;
#pragma unroll
      for (int j = 0; j < HIW; ++j) {
        const int s = hsc[j] & 1023, col = (int)((hsc[j] >> 10) & 255) - 1;
        const int v = s + oh0 - 1;                                     // >= -1
        const int d = (int)udiv((uint32_t)(v + H + 1), h.mag_h1) - 1;  // floor(v / (H+1))
        const int row = v - d * (H + 1);
        const int img = img0 + d;
        const bool ok = row < H && (unsigned)col < (unsigned)W && img < nimg;
        hv[j] = ok ? ((((uint32_t)img * H + row) * W + col) * aC) * 2 + (hsc[j] >> 18) * 16
                   : 0x80000000u;
      }
    };
    // DMA instruction j (halo 0..8, then weights 9..17 unless resident) of item (cc, stage)
    auto dma = [&](int cc, int stage, int j) {
      if (j < HIW) {
        const __amdgpu_buffer_rsrc_t ra = make_rsrc((const char*)p.A + cc * 64, h.a_bytes);
        // (SELF: as asm, invisible to the compiler, which would otherwise wait for these
        // DMAs before the MFMA waves' next ds_read of the other stage)
        if constexpr (SELF) buf_lds16_asm(ra, hal + stage * HBYTES + (wave * HIW + j) * 1024, hv[j]);
        else buf_lds16(ra, hal + stage * HBYTES + (wave * HIW + j) * 1024, hv[j]);
      } else if (!WRES && j < HIW + HB_WIW) {
        const __amdgpu_buffer_rsrc_t rb = make_rsrc((const char*)p.B + cc * 64, h.b_bytes);
        buf_lds16(rb, wst + stage * HB_WBYTES + (wave * HB_WIW + j - HIW) * 1024,
                  wv[j - HIW]);
      }
    };
    auto issue = [&](int cc, int stage) {
#pragma unroll
      for (int j = 0; j < HIW + HB_WIW; ++j) dma(cc, stage, j);
    };
    if (nitems > 0) {
      if constexpr (WRES) {  // whole weight tile (tiles_n == 1, CC <= 2) once per block
        for (int cc = 0; cc < CC; ++cc) {
          const __amdgpu_buffer_rsrc_t rb = make_rsrc((const char*)p.B + cc * 64, h.b_bytes);
          char* wdst = wst + cc * HB_WBYTES + wave * HB_WIW * 1024;
#pragma unroll
          for (int j = 0; j < HB_WIW; ++j) buf_lds16(rb, wdst + j * 1024, wv[j]);
        }
      }
      prep_tile(0);
      issue(0, 0);
    }
    body(prep_tile, dma, issue);
  };

  {
    // Producer waves 4..7: all of the block's LDS-DMAs.  Item k's top barrier publishes
    // stage k & 1 (every producer has waited for its DMAs) and frees stage (k + 1) & 1 (every
    // MFMA wave is done with item k - 1), so item k + 1's DMAs go out right behind it and get
    // the whole of item k to land.  The MFMA waves' instruction streams carry no DMA at all:
    // issuing the 18 per item between the MFMAs cost those waves ~10 % (round-2 A/B,
    // docs/KERNELS.md), waiting for them nothing measurable.  Barrier count per wave:
    // nitems (+1 for the statistics flush) on both sides.
    if (!SELF && wave_all >= HB_NW) {
      stager([&](auto& prep_tile, auto&, auto& issue) {
        int cc1 = 0;
        for (int k = 0; k < nitems; ++k) {
          wait_all_barrier();
          if (++cc1 == CC) cc1 = 0;
          if (k + 1 < nitems) {
            if (cc1 == 0) prep_tile((k + 1) / CC);
            issue(cc1, (k + 1) & 1);
          }
        }
      });
      if constexpr (EPI & (EP_STATS | EP_BNRED)) __syncthreads();  // halo_stats_flush's
      return;
    }
  }

  // per-column epilogue operands of the block's 64 columns: bias (or BN mean) and stats
  // shift (or BN rstd), parked in LDS rather than in 32 VGPRs held through every MFMA; the
  // first item's barrier publishes them
  if (tid < 16 * NJ) {
    const float* bsrc = (EPI & EP_BNRED) ? p.ep_mean : p.bias;
    const float* ssrc = (EPI & EP_BNRED) ? p.ep_rstd : p.stats_shift;
    const float b = bsrc ? bsrc[n0 + tid] : 0.f, sv = ssrc ? ssrc[n0 + tid] : 0.f;
    cst[tid] = b;
    cst[HB_BN + tid] = sv;
    if constexpr (EPI & EP_BNRED) {  // the ReLU mask's affine, as bn_fwd_train computed it
      const float sc = p.ep_gamma[n0 + tid] * sv;
      cst[2 * HB_BN + tid] = sc;
      cst[3 * HB_BN + tid] = __builtin_fmaf(-b, sc, p.ep_beta[n0 + tid]);
    }
  }
  // TRED (fused BN-backward reduction): the column sums are reduced per tile and column
  // group (DPP over the 16 pixel lanes) and accumulated in this wave's slot of `red`, so
  // no sums live in registers through the MFMA stream and at most 8 through the epilogue.
  // Holding them for the block's life (as the statistics flavours do) put this flavour at
  // 256 VGPRs with 344-556 B/lane of scratch spills - the round-2/3 "BN link is slower"
  // measurements were those spills.
  // (SELF, statistics epilogue: the same per-tile reduction - 32 sums held for the block's
  // life beside 112 accumulators put the 448-pixel flavour at ~600 registers)
  constexpr bool TRED = (EPI & EP_BNRED) != 0 || (SELF && (EPI & EP_STATS) != 0);
  if constexpr (TRED) ((float2*)red)[tid] = make_float2(0.f, 0.f);  // own wave's slot
  float ss[4][4], sq[4][4];
#pragma unroll
  for (int jn = 0; jn < 4; ++jn)
#pragma unroll
    for (int r = 0; r < 4; ++r) { ss[jn][r] = 0.f; sq[jn][r] = 0.f; }

  // B fragment byte offsets (tap 0, column group 0): row l15 of the [tap][64][32] image
  const int boff = l15 * 64 + ((jq ^ ((l15 >> 1) & 2)) << 4);
  // Swizzled LDS byte address of this lane's A row in each row fragment for column tap
  // dw = d - 1: X = 64 * (pixel + dw) + 16 * chunk, chunk position flipped by pixel bit 2
  // (X bit 8).  The pitch is a multiple of 8 pixels, so a row tap dh adds dh*P*64 without
  // touching bits 0..8: a tap's address is xbw[i][dw + 1] + dh*P*64 (+ stage) - 1 VALU.
  int xbw[MI][3];
  EpiInT<MI> ein;
  f32x4 acc[MI][4];

  // Epilogue of fragment (i, jn) of the tile at m0e (operands from epi_preload).
  auto epi_fr = [&](int i, int jn, int m0e, auto full, float (&es)[4][4], float (&eq)[4][4]) {
    constexpr bool F = decltype(full)::value;
    const int m = m0e + wave * 16 * MI + i * 16 + l15;
    const uint32_t orow = (uint32_t)m * p.ldc + n0 + jq * 4;
    // (BN reduction: volatile, read where used - hoisted out of the tile loop, its four
    // vectors would hold 64 VGPRs through every MFMA.  Volatile reads in the other
    // flavours made them 12-30 % slower.)
    const int c = jn * 16 + jq * 4;
    f32x4 colb, cols, mc = {0.f, 0.f, 0.f, 0.f}, mh = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI & EP_BNRED) {
      auto col = [&](int row) { return *(const volatile f32x4*)(cst + row * HB_BN + c); };
      colb = col(0);
      cols = col(1);
      mc = col(2);
      mh = col(3);
    } else {
      colb = *(const f32x4*)(cst + c);
      cols = *(const f32x4*)(cst + HB_BN + c);
    }
    uint2 av = ein.a[i][jn];
    if constexpr ((EPI & EP_BETA) != 0) {
      if (p.ep_rmask) av = masked_acc(av, ein.mk[i], jn, jq);
    }
    return epi_frag<EPI, F, false>(p, acc[i][jn], av, m < p.M, jn, orow, colb, cols, mc, mh,
                                   es[jn], eq[jn]);
  };
  // Epilogue of a whole tile (see TRED)
  auto epi_tile = [&](int m0e, auto full) {
    if constexpr (TRED) {
      constexpr bool F = decltype(full)::value;
      float* rd = (float*)red;
      if constexpr (WIDE) {
#pragma unroll
      for (int jp = 0; jp < NJ; jp += 2) {
        // this column-group pair's mean / rstd / mask affine, read from LDS per tile (an
        // empty asm memory clobber keeps the compiler from hoisting 64 VGPRs of them out of
        // the tile loop); its sums live only across its row fragments (32 live sums spilled)
        asm volatile("" ::: "memory");
        f32x4 colb[2], cols[2], mc[2], mh[2];
        float ts[2][4], tq[2][4];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int c = (jp + e) * 16 + jq * 4;
          colb[e] = *LDS_PTR(const f32x4, cst + c);
          cols[e] = *LDS_PTR(const f32x4, cst + HB_BN + c);
          mc[e] = f32x4{0.f, 0.f, 0.f, 0.f};
          mh[e] = f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr ((EPI & EP_BNRED) != 0) {
            mc[e] = *LDS_PTR(const f32x4, cst + 2 * HB_BN + c);
            mh[e] = *LDS_PTR(const f32x4, cst + 3 * HB_BN + c);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) { ts[e][r] = 0.f; tq[e][r] = 0.f; }
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0e + wave * 16 * MI + i * 16 + l15;
          const uint32_t prow = (uint32_t)m * p.ldc + n0;
          const uint32_t orow = prow + jq * 4;
          uint2 v[2];
#pragma unroll
          for (int e = 0; e < 2; ++e)
            v[e] = epi_frag<EPI, F, false>(p, acc[i][jp + e], ein.a[i][jp + e], m < p.M, jp + e,
                                           orow, colb[e], cols[e], mc[e], mh[e], ts[e], tq[e]);
          store_pair16((bf16_t*)p.C, prow, jp, jq, v[0], v[1], F || m < p.M);
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            ts[e][r] = row16_sum(ts[e][r]);
            tq[e][r] = row16_sum(tq[e][r]);
          }
          if (l15 == 0) {  // columns (jp+e)*16 + 4 jq .. +3 of this wave: [sum, sum2] pairs
            f32x4* q = (f32x4*)(rd + (wave * 64 + (jp + e) * 16 + jq * 4) * 2);
            f32x4 q0 = q[0], q1 = q[1];
            q0[0] += ts[e][0]; q0[1] += tq[e][0]; q0[2] += ts[e][1]; q0[3] += tq[e][1];
            q1[0] += ts[e][2]; q1[1] += tq[e][2]; q1[2] += ts[e][3]; q1[3] += tq[e][3];
            q[0] = q0;
            q[1] = q1;
          }
        }
      }
      } else {
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) {
        // this column group's mean / rstd / mask affine, read from LDS per tile (an empty
        // asm memory clobber keeps the compiler from hoisting 64 VGPRs of them out of the
        // tile loop); its sums live only across its 4 row fragments (32 live sums spilled)
        asm volatile("" ::: "memory");
        const int c = jn * 16 + jq * 4;
        const f32x4 colb = *LDS_PTR(const f32x4, cst + c);
        const f32x4 cols = *LDS_PTR(const f32x4, cst + HB_BN + c);
        f32x4 mc = {0.f, 0.f, 0.f, 0.f}, mh = {0.f, 0.f, 0.f, 0.f};
        if constexpr ((EPI & EP_BNRED) != 0) {
          mc = *LDS_PTR(const f32x4, cst + 2 * HB_BN + c);
          mh = *LDS_PTR(const f32x4, cst + 3 * HB_BN + c);
        }
        float ts[4][4], tq[4][4];  // (only row jn is used)
#pragma unroll
        for (int r = 0; r < 4; ++r) { ts[jn][r] = 0.f; tq[jn][r] = 0.f; }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int m = m0e + wave * 16 * MI + i * 16 + l15;
          const uint32_t orow = (uint32_t)m * p.ldc + n0 + jq * 4;
          epi_frag<EPI, F>(p, acc[i][jn], ein.a[i][jn], m < p.M, jn, orow, colb, cols, mc, mh,
                           ts[jn], tq[jn]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ts[jn][r] = row16_sum(ts[jn][r]);
          tq[jn][r] = row16_sum(tq[jn][r]);
        }
        if (l15 == 0) {  // columns jn*16 + 4 jq .. +3 of this wave: [sum, sum2] pairs
          f32x4* q = (f32x4*)(rd + (wave * 64 + jn * 16 + jq * 4) * 2);
          f32x4 q0 = q[0], q1 = q[1];
          q0[0] += ts[jn][0]; q0[1] += tq[jn][0]; q0[2] += ts[jn][1]; q0[3] += tq[jn][1];
          q1[0] += ts[jn][2]; q1[1] += tq[jn][2]; q1[2] += ts[jn][3]; q1[3] += tq[jn][3];
          q[0] = q0;
          q[1] = q1;
        }
      }
      }
    } else {
      // (the per-column operands are re-read from LDS per tile: an empty asm memory clobber
      // keeps the compiler from hoisting 32 VGPRs of them out of the tile loop)
      asm volatile("" ::: "memory");
      if constexpr (WIDE) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int m = m0e + wave * 16 * MI + i * 16 + l15;
#pragma unroll
        for (int jn = 0; jn < NJ; jn += 2) {
          const uint2 v0 = epi_fr(i, jn, m0e, full, ss, sq);
          const uint2 v1 = epi_fr(i, jn + 1, m0e, full, ss, sq);
          store_pair16((bf16_t*)p.C, (uint32_t)m * p.ldc + n0, jn, jq, v0, v1,
                       decltype(full)::value || m < p.M);
        }
      }
      } else {
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int jn = 0; jn < NJ; ++jn) {
            const int m = m0e + wave * 16 * MI + i * 16 + l15;
            const uint2 v = epi_fr(i, jn, m0e, full, ss, sq);
            if (decltype(full)::value || m < p.M)
              *(uint2*)((bf16_t*)p.C + (uint32_t)m * p.ldc + n0 + jq * 4 + jn * 16) = v;
          }
      }
    }
  };

  // One 32-channel chunk, all 9 taps, tap-outer: per tap 4 A + NJ B fragments (the next
  // tap's reads issued ahead of this tap's 4 NJ MFMAs).  FIRST: the tile's first chunk
  // (accumulators start at 0).  (Measured: fencing the reads a tap ahead with
  // sched_barrier and zeroing the accumulators per tile instead of the FIRST path was 7-10 %
  // faster in isolation but 0.7 % slower in the training step with side-stream weight
  // gradients - profiles/halo_sched_r5.txt; a row-major body that held the chunk's B
  // fragments in registers and ran the previous tile's epilogue interleaved with the next
  // tile's MFMAs was 10-15 % slower.)
  auto mma_chunk = [&](int st, int cc, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    const int hbase = st * HBYTES;
    const char* wimg = (WRES ? wst + cc * HB_WBYTES : wst + st * HB_WBYTES) + boff;
    if constexpr (MI != 4) {
      // (MI = 7: row fragment i of tap t + 1 is read into its register right after tap t's
      // MFMAs on row i consumed it - one A set instead of a double buffer - and a
      // scheduling fence per row group keeps the compiler from hoisting those reads, which
      // would need the double buffer's registers: the 8-wave block has 256 per wave)
      bf16x8 a1[MI], b2[2][4];
      auto lda = [&](int t, int i) {
        a1[i] = frag16(hal + hbase + (t / 3 - 1) * W2 * 64 + xbw[i][t % 3]);
      };
      auto ldb = [&](int t, int b) {
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn) b2[b][jn] = frag16(wimg + t * (HB_BN * 64) + jn * 1024);
      };
#pragma unroll
      for (int i = 0; i < MI; ++i) lda(0, i);
      ldb(0, 0);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t + 1 < 9) ldb(t + 1, (t + 1) & 1);
#pragma unroll
        for (int i = 0; i < MI; ++i) {
#pragma unroll
          for (int jn = 0; jn < NJ; ++jn)
            acc[i][jn] = mfma16(b2[t & 1][jn], a1[i],
                                (FIRST && t == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][jn]);
          if (t + 1 < 9) lda(t + 1, i);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      return;
    }
    bf16x8 a2[2][4], b2[2][4];
    auto ld = [&](int t, int b) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a2[b][i] = frag16(hal + hbase + (t / 3 - 1) * W2 * 64 + xbw[i][t % 3]);
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) b2[b][jn] = frag16(wimg + t * (HB_BN * 64) + jn * 1024);
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn)
          acc[i][jn] = mfma16(b2[t & 1][jn], a2[t & 1][i],
                              (FIRST && t == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][jn]);
    }
  };

  // One tile: CC items through the 2-stage ring, then its epilogue.  The epilogue operands
  // (accumulate: old output; fused BN reduction: z, y) are loaded right after the top wait
  // of the tile's second-to-last item, so they are in flight under its MFMAs (a load issued
  // in front of a wait would be waited for with the DMAs).
  auto run_tile = [&](int tk, auto hook) {
    const int m0 = m0_of(tk);
    for (int cc = 0; cc < CC; ++cc) {
      const int k = tk * CC + cc;
      const int st = k & 1;
      // this item's DMAs were issued by the producers during the previous item (stage st ^ 1
      // was freed by this barrier); the MFMA waves have no DMA of their own to wait for
      // (SELF: this wave's own DMAs of item k - issued at item k - 1's top - have landed;
      // the previous tile's epilogue stores, issued after them, may stay in flight)
      if constexpr (SELF) {
        if (cc == 0 && tk > 0) {
          static_assert(MI * NJ == 28, "vmcnt below counts one store per epilogue fragment");
          asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
        } else {
          __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
        }
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      hook(k);  // (SELF: item k + 1's DMAs into the stage this barrier freed)
      if (cc == max(CC - 2, 0)) epi_preload<EPI, NJ, MI>(p, ein, m0, n0, wave, lane);
      if (cc == 0) {
        const int img0 = m0 / HW;
        const int r0 = m0 - img0 * HW;
        const int oh0 = r0 / W;
        const int mlast = p.M - 1 - img0 * HW;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const uint32_t n = (uint32_t)min(r0 + wave * 16 * MI + i * 16 + l15, mlast);
          const uint32_t di = udiv(n, h.mag_hw);
          const uint32_t rem = n - di * HW;
          const uint32_t oh = udiv(rem, h.mag_w);
          const uint32_t ow = rem - oh * W;
          const int hp = ((int)(di * (H + 1) + oh) - oh0 + 1) * W2 + (int)ow + 1;
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const int x = ((hp + d - 1) << 6) + (jq << 4);
            xbw[i][d] = x ^ ((x >> 3) & 32);
          }
        }
        mma_chunk(st, 0, std::true_type{});
      } else {
        mma_chunk(st, cc, std::false_type{});
      }
      if (cc == CC - 1 && tk + 1 < ntiles)  // full tile (only the last can end past M)
        epi_tile(m0, std::true_type{});
      // (no barrier here: item k + 2's DMAs into stage st are issued during item k + 1,
      // after its top barrier, which every wave passes only once done reading stage st)
    }
  };

  if constexpr (SELF) {
    stager([&](auto& prep_tile, auto&, auto& issue) {
      int cc1 = 0;
      auto next = [&](int k) {
        if (++cc1 == CC) cc1 = 0;
        if (k + 1 < nitems) {
          if (cc1 == 0) prep_tile((k + 1) / CC);
          issue(cc1, (k + 1) & 1);
        }
      };
      for (int tk = 0; tk < ntiles; ++tk) run_tile(tk, next);
    });
  } else {
    for (int tk = 0; tk < ntiles; ++tk) run_tile(tk, [](int) {});
  }
  if (ntiles > 0) epi_tile(m0_of(ntiles - 1), std::integral_constant<bool, FULL>{});
  if constexpr (EPI & (EP_STATS | EP_BNRED)) halo_stats_flush<TRED>(p, ss, sq, red, n0, wave, tid);
}

// ======================================================================================
//  Strip-tiled 3x3 / stride-1 convolution (same engine, 2-D tiles)
//
//  conv3_halo_kernel's tiles are 256 consecutive pixels of the flattened (image, row, col)
//  sequence; its halo image must hold every input row those pixels touch plus one above and
//  below, so an image wider than ~60 pixels (VGG's 224^2 / 112^2 layers, Inception's 147^2 /
//  73^2) does not fit a 36 KiB stage and runs on the implicit GEMM, which gathers every input
//  pixel nine times.  Here a tile is TR rows x TW columns of ONE image (TW = W, or W split
//  into equal strips of <= 128 columns; TR*TW <= 256 MFMA rows, the rest masked), and the
//  stage holds (TR + 2) slot rows of pitch P = TW + 2 (left / right halo columns, rounded up
//  to 8): every tap is still one uniform offset dh*P + dw, the A fragment addresses are
//  tile-independent (computed once per block), and only (TR+2)*P pixels are staged:
//  ResNet layer1 (W 56): 4 x 56 tiles, 384 pixels per item instead of 576.
//
//  NS = 3 (resident weights, <= 6 halo DMAs per producer wave): two items in flight while a
//  third is multiplied.  The layer1 halo kernel stages 37 KB per 2.9 us item per CU
//  (~13 GB/s/CU): one item in flight per CU is HBM latency-bound, not bandwidth-bound
//  (tools/dma_probe.hip).
//  Producer waves only (8-wave blocks), 64-wide column tiles (N % 64 == 0).
// ======================================================================================
struct StripPlan {
  int tr, tw, p;            // tile rows / columns, LDS pitch (pixels)
  int hiw;                  // halo DMA instructions per producer wave per item (<= 9)
  int tiles_c, tiles_img;   // column strips per row band, tiles per image
  int tiles_total, cc;
  uint32_t mag_tw, mag_p, mag_tc, mag_timg;  // floor(2^32 / d) + 1 (0: d == 1)
  int btoff[9];
  uint32_t a_bytes, b_bytes;
  int ch, cw;               // tap-set centre shift: output (i, j) reads input rows / cols
                            // i + ch - 1 .. i + ch + 1 (same conv 0, valid 1, its dgrad -1)
};

// n / d from udiv's magic, with magic 0 standing for d == 1 (floor(2^32 / 1) + 1 wraps)
__device__ __forceinline__ uint32_t udiv1(uint32_t n, uint32_t mag) {
  return mag ? udiv(n, mag) : n;
}

// s_waitcnt vmcnt(n) for the run-time per-item DMA counts of the strip producers
__device__ __forceinline__ void strip_wait(int n) {
  switch (n) {
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <bool WRES, int EPI, int NS, int NJ>
__global__ __launch_bounds__(512, 1) void conv3_strip_kernel(IGemmArgs p, StripPlan h) {
  __shared__ __attribute__((aligned(16))) char smem[HB_LDS];
  const int HBY = h.hiw * 4096;  // halo stage bytes (4 producer waves x hiw KiB)
  char* const hal = smem;
  char* const wst = smem + NS * HBY;
  char* const red = smem + 2 * HB_HBYTES + 2 * HB_WBYTES;
  float* const cst = (float*)(red + HB_RED);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wave_all & (HB_NW - 1);
  const int H = p.aH, W = p.aW, P = h.p, aC = p.aC;  // input image
  const int OH = p.oH, OW = p.oW;                      // output image (tiles)
  const int TR = h.tr, TW = h.tw;
  const int jq = lane >> 4, l15 = lane & 15;

  const int T = h.tiles_total;
  const int xcd = blockIdx.x & 7, loc = blockIdx.x >> 3, G8 = gridDim.x >> 3;
  const int tbeg = (int)((int64_t)xcd * T / 8), tend = (int)((int64_t)(xcd + 1) * T / 8);
  const int ntiles = tbeg + loc < tend ? (tend - tbeg - loc + G8 - 1) / G8 : 0;
  const int CC = h.cc;
  const int nitems = ntiles * CC;
  const int nt = (tbeg + loc) % p.tiles_n;
  const int n0 = nt * HB_BN;
  // tile tk of this block -> (image, first row, first column)
  auto origin = [&](int tk, int& img, int& r0, int& c0) {
    const uint32_t mt = (uint32_t)((tbeg + loc + tk * G8) / p.tiles_n);
    img = (int)udiv1(mt, h.mag_timg);
    const uint32_t rem = mt - (uint32_t)img * h.tiles_img;
    const uint32_t tr = udiv1(rem, h.mag_tc);
    r0 = (int)tr * TR;
    c0 = (int)(rem - tr * h.tiles_c) * TW;
  };

  if (wave_all >= HB_NW) {
    // ---- producers: halo lanes (slot row, column, logical chunk) are tile-independent
    const int hiw = h.hiw;
    uint32_t hsc[9];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const uint32_t hp = 16 * (wave * hiw + j) + (lane >> 2);
      const uint32_t s = udiv(hp, h.mag_p);
      const uint32_t col = hp - s * P;
      const uint32_t lc = (lane & 3) ^ (((hp >> 2) & 1) << 1);
      hsc[j] = s | (col << 10) | (lc << 20);
    }
    uint32_t wv[HB_WIW];
#pragma unroll
    for (int j = 0; j < HB_WIW; ++j) {
      const int q = wave * HB_WIW + j;
      const int r = 16 * q + (lane >> 2);
      const int n = r & 63;
      const int lc = (lane & 3) ^ (((r >> 2) & 1) << 1);
      wv[j] = (n0 + n < p.N) ? (uint32_t)(n0 + n) * p.ldb * 2 + h.btoff[q >> 2] + lc * 16
                             : 0x80000000u;
    }
    uint32_t hv[9];
    auto prep_tile = [&](int tk) {
      int img, r0, c0;
      origin(tk, img, r0, c0);
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int s = hsc[j] & 1023, col = (hsc[j] >> 10) & 1023;
        const int ih = r0 + h.ch - 1 + s, iw = c0 + h.cw - 1 + col;
        const bool ok = s < TR + 2 && col < TW + 2 && (unsigned)ih < (unsigned)H &&
                        (unsigned)iw < (unsigned)W;
        hv[j] = ok ? ((((uint32_t)img * H + ih) * W + iw) * aC) * 2 + (hsc[j] >> 20) * 16
                   : 0x80000000u;
      }
    };
    auto issue = [&](int cc, int stage) {
      const __amdgpu_buffer_rsrc_t ra = make_rsrc((const char*)p.A + cc * 64, h.a_bytes);
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (j < hiw) buf_lds16(ra, hal + stage * HBY + (wave * hiw + j) * 1024, hv[j]);
      if constexpr (!WRES) {
        const __amdgpu_buffer_rsrc_t rb = make_rsrc((const char*)p.B + cc * 64, h.b_bytes);
#pragma unroll
        for (int j = 0; j < HB_WIW; ++j)
          buf_lds16(rb, wst + stage * HB_WBYTES + (wave * HB_WIW + j) * 1024, wv[j]);
      }
    };
    const int dpi = hiw + (WRES ? 0 : HB_WIW);  // DMAs per item per producer wave
    if (nitems > 0) {
      if constexpr (WRES) {
        for (int cc = 0; cc < CC; ++cc) {
          const __amdgpu_buffer_rsrc_t rb = make_rsrc((const char*)p.B + cc * 64, h.b_bytes);
          char* wdst = wst + cc * HB_WBYTES + wave * HB_WIW * 1024;
#pragma unroll
          for (int j = 0; j < HB_WIW; ++j) buf_lds16(rb, wdst + j * 1024, wv[j]);
        }
      }
    }
    int ki = 0;  // next item to issue (issue order == item order)
    auto issue_next = [&]() {
      const int tk = ki / CC, cc = ki - tk * CC;
      if (cc == 0) prep_tile(tk);
      issue(cc, ki % NS);
      ++ki;
    };
    while (ki < NS - 1 && ki < nitems) issue_next();
    for (int k = 0; k < nitems; ++k) {
      strip_wait((ki - k - 1) * dpi);  // item k landed; younger items stay in flight
      __builtin_amdgcn_s_barrier();    // publishes stage k % NS, frees stage (k - 1) % NS
      if (ki < nitems) issue_next();
    }
    if constexpr (EPI & (EP_STATS | EP_BNRED)) __syncthreads();  // halo_stats_flush's
    return;
  }

  // ---- MFMA waves
  if (tid < 16 * NJ) {
    const float* bsrc = (EPI & EP_BNRED) ? p.ep_mean : p.bias;
    const float* ssrc = (EPI & EP_BNRED) ? p.ep_rstd : p.stats_shift;
    const float b = bsrc ? bsrc[n0 + tid] : 0.f, sv = ssrc ? ssrc[n0 + tid] : 0.f;
    cst[tid] = b;
    cst[HB_BN + tid] = sv;
    if constexpr (EPI & EP_BNRED) {
      const float sc = p.ep_gamma[n0 + tid] * sv;
      cst[2 * HB_BN + tid] = sc;
      cst[3 * HB_BN + tid] = __builtin_fmaf(-b, sc, p.ep_beta[n0 + tid]);
    }
  }
  constexpr bool TRED = (EPI & EP_BNRED) != 0;
  if constexpr (TRED) ((float2*)red)[tid] = make_float2(0.f, 0.f);
  float ss[4][4], sq[4][4];
#pragma unroll
  for (int jn = 0; jn < 4; ++jn)
#pragma unroll
    for (int r = 0; r < 4; ++r) { ss[jn][r] = 0.f; sq[jn][r] = 0.f; }

  const int boff = l15 * 64 + ((jq ^ ((l15 >> 1) & 2)) << 4);
  // A row addresses (tile-independent): local pixel li -> slot (lr + 1), column (lc + 1),
  // column tap dw = d - 1; rows past the tile read its last pixel (their outputs are masked)
  int xbw[4][3], lrc[4];
  const int tpx = TR * TW;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int li = min(wave * 64 + i * 16 + l15, tpx - 1);
    const int lr = (int)udiv((uint32_t)li, h.mag_tw), lc = li - lr * TW;
    lrc[i] = (wave * 64 + i * 16 + l15 < tpx) ? (lr << 16) | lc : -1;
    const int hp = (lr + 1) * P + lc + 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int x = ((hp + d - 1) << 6) + (jq << 4);
      xbw[i][d] = x ^ ((x >> 3) & 32);
    }
  }
  EpiIn ein;
  f32x4 acc[4][4];
  int mrow[4];  // output pixel of each row fragment's lane in the current tile (-1: masked)
  auto set_rows = [&](int tk) {
    int img, r0, c0;
    origin(tk, img, r0, c0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lr = lrc[i] >> 16, lc = lrc[i] & 0xffff;
      mrow[i] = (lrc[i] >= 0 && r0 + lr < OH && c0 + lc < OW)
                    ? (img * OH + r0 + lr) * OW + c0 + lc : -1;
    }
  };
  auto preload = [&]() {
    if constexpr (EPI & (EP_BETA | EP_BNRED)) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t orow = (uint32_t)max(mrow[i], 0) * p.ldc + n0 + jq * 4;
        if constexpr (!(EPI & EP_BNRED))
          ein.mk[i] = acc_mask(p, (uint32_t)max(mrow[i], 0) * p.ldc + n0);
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn) {
          if constexpr (EPI & EP_BNRED) ein.a[i][jn] = *(const uint2*)(p.ep_z + orow + jn * 16);
          else ein.a[i][jn] = acc_operand(p, orow + jn * 16);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) ein.a[i][jn] = make_uint2(0u, 0u);
    }
  };
  auto epi_tile = [&]() {
    if constexpr (TRED) {
      float* rd = (float*)red;
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) {
        asm volatile("" ::: "memory");
        const int c = jn * 16 + jq * 4;
        const f32x4 colb = *LDS_PTR(const f32x4, cst + c);
        const f32x4 cols = *LDS_PTR(const f32x4, cst + HB_BN + c);
        const f32x4 mc = *LDS_PTR(const f32x4, cst + 2 * HB_BN + c);
        const f32x4 mh = *LDS_PTR(const f32x4, cst + 3 * HB_BN + c);
        float ts[4][4], tq[4][4];
#pragma unroll
        for (int r = 0; r < 4; ++r) { ts[jn][r] = 0.f; tq[jn][r] = 0.f; }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t orow = (uint32_t)max(mrow[i], 0) * p.ldc + n0 + jq * 4;
          epi_frag<EPI, false>(p, acc[i][jn], ein.a[i][jn], mrow[i] >= 0, jn, orow, colb, cols,
                               mc, mh, ts[jn], tq[jn]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          ts[jn][r] = row16_sum(ts[jn][r]);
          tq[jn][r] = row16_sum(tq[jn][r]);
        }
        if (l15 == 0) {
          f32x4* q = (f32x4*)(rd + (wave * 64 + jn * 16 + jq * 4) * 2);
          f32x4 q0 = q[0], q1 = q[1];
          q0[0] += ts[jn][0]; q0[1] += tq[jn][0]; q0[2] += ts[jn][1]; q0[3] += tq[jn][1];
          q1[0] += ts[jn][2]; q1[1] += tq[jn][2]; q1[2] += ts[jn][3]; q1[3] += tq[jn][3];
          q[0] = q0;
          q[1] = q1;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn) {
          const int c = jn * 16 + jq * 4;
          const f32x4 colb = *(const f32x4*)(cst + c);
          const f32x4 cols = *(const f32x4*)(cst + HB_BN + c);
          const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
          const uint32_t orow = (uint32_t)max(mrow[i], 0) * p.ldc + n0 + jq * 4;
          uint2 av = ein.a[i][jn];
          if constexpr ((EPI & EP_BETA) != 0) {
            if (p.ep_rmask) av = masked_acc(av, ein.mk[i], jn, jq);
          }
          epi_frag<EPI, false>(p, acc[i][jn], av, mrow[i] >= 0, jn, orow, colb, cols,
                               z4, z4, ss[jn], sq[jn]);
        }
    }
  };
  // one 32-channel chunk, all 9 taps (as conv3_halo_kernel's mma_chunk)
  auto mma_chunk = [&](int st, int cc, auto first) {
    constexpr bool FIRST = decltype(first)::value;
    const int hbase = st * HBY;
    const char* wimg = (WRES ? wst + cc * HB_WBYTES : wst + st * HB_WBYTES) + boff;
    bf16x8 a2[2][4], b2[2][4];
    auto ld = [&](int t, int b) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a2[b][i] = frag16(hal + hbase + (t / 3 - 1) * P * 64 + xbw[i][t % 3]);
#pragma unroll
      for (int jn = 0; jn < NJ; ++jn) b2[b][jn] = frag16(wimg + t * (HB_BN * 64) + jn * 1024);
    };
    ld(0, 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ld(t + 1, (t + 1) & 1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int jn = 0; jn < NJ; ++jn)
          acc[i][jn] = mfma16(b2[t & 1][jn], a2[t & 1][i],
                              (FIRST && t == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[i][jn]);
    }
  };
  for (int tk = 0; tk < ntiles; ++tk) {
    set_rows(tk);
    for (int cc = 0; cc < CC; ++cc) {
      const int k = tk * CC + cc;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      if (cc == max(CC - 2, 0)) preload();
      if (cc == 0) mma_chunk(k % NS, 0, std::true_type{});
      else mma_chunk(k % NS, cc, std::false_type{});
    }
    epi_tile();
  }
  if constexpr (EPI & (EP_STATS | EP_BNRED)) halo_stats_flush<TRED>(p, ss, sq, red, n0, wave, tid);
}

// ======================================================================================
//  Halo-staged 3x3 / stride-1 weight gradient:
//    dW[k][t = 3r+s][c] += sum_pix dy[pix][k] * x[pix + (r-1, s-1)][c]
//  The implicit-GEMM wgrad gathers an im2col column panel per (tap, channel) tile, i.e.
//  every x pixel nine times.  Here a block owns a 64 (k) x 64 (c) x 9 (taps) output
//  partition and streams 128-pixel tiles: the dy tile [128 px][64 k] and the x halo of
//  those pixels (both 32-channel chunks of the partition) are staged once per tile, and the
//  nine taps read shifted halo rows.  Reduction dim = pixels: both operands are read
//  pixel-major with ds_read_b64_tr_b16 (dy image in the engine's mn_off<64> layout; halo
//  rows 64 B with chunk c at position c ^ (2 * ((row >> 3) & 1)), so the 2 x 4 pixel rows
//  one 32-lane half reads hit every bank once).  Wave w owns 16 channels (chunk w/2) for
//  all 64 k and 9 taps: 36 accumulators of 16x16.  Partials go to a [Z][K][9C] slab
//  (Z = blocks per partition), summed into the fp32 gradient arena by wgrad_reduce.
// ======================================================================================
constexpr int HW_BM = 128;                    // pixels per tile
constexpr int HW_HIW = 7;                     // halo DMA instructions per wave per chunk
constexpr int HW_HPX = 16 * 4 * HW_HIW;       // 448 halo pixels
constexpr int HW_HBYTES = HW_HPX * 64;        // 28 KiB per chunk
constexpr int HW_DBYTES = HW_BM * 64 * 2;     // 16 KiB: dy tile, 4 k-steps x [32 px][64 k]
constexpr int HW_STAGE = HW_DBYTES + 2 * HW_HBYTES;  // 72 KiB
constexpr int HW_LDS = 2 * HW_STAGE;                 // 147,456 B

struct HaloWPlan {
  int toff[9];
  int w2;  // halo row pitch in pixels: W + 2 rounded up to 16 (see the B-address note)
  uint32_t mag_w, mag_w2, mag_h1, mag_hw;
  int tiles_m, parts, kparts, Z;
  uint32_t dy_bytes, x_bytes;
  // STRIP: tiles of tr rows x tw columns of one image (w2 = tw + 2 rounded up to 16), for
  // images too wide for the 128-pixel linear tiles' halo (VGG 224^2 / 112^2)
  int tr, tw, tiles_c, tiles_img;
  uint32_t mag_tw, mag_tc, mag_timg;  // (0: divisor 1)
  // XCD-grouped block order (grid % 8 == 0): logical block L = xcd * (grid / 8) + slot, so
  // one XCD's blocks are consecutive (z, part) ids - they share z lanes and cover a run of
  // partitions, and each staged dy / x tile is read into that XCD's L2 by the blocks that
  // consume it, instead of every XCD fetching every x (or dy) panel
  int xmap;
};

// W2T: the halo pitch as a compile-time constant (16 / 32 / 48 / 64: every ResNet and
// Inception size), so a tap's row offset is an immediate DS offset; 0 = runtime pitch.
// ONECH (C == 32, images too wide for a 448-pixel halo, e.g. Inception's 147 x 147
// Conv2d_2b): the partition's second channel chunk does not exist, so the two chunk areas
// of a stage hold ONE 896-pixel halo image of the first chunk (14 DMA instructions per
// wave instead of 2 x 7).  Waves 2 and 3 then read chunk 0 as well; their partials are
// duplicates of waves 0 / 1 and are not stored.
// PROD: 8-wave blocks; waves 4..7 are producers (every tile's index math and LDS-DMAs),
// waves 0..3 run only fragment reads and MFMAs.  One barrier per tile on both sides: tile
// k's barrier publishes stage k & 1 and frees stage (k + 1) & 1.
// KM: 16-row k fragments per partition (4; 2 when Kout == 32 - DenseNet's growth-rate
// convs - so the partition's zero upper half costs no MFMA and no fragment read)
template <int W2T, bool ONECH = false, bool STRIP = false, bool PROD = false, int KM = 4>
__global__ __launch_bounds__(PROD ? 512 : 256, 1) void conv3_halo_wgrad_kernel(WGradArgs p, HaloWPlan h) {
  constexpr int HIW = ONECH ? 2 * HW_HIW : HW_HIW;  // halo DMA instructions per wave (chunk)
  __shared__ __attribute__((aligned(16))) char smem[HW_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wave_all & 3;  // MFMA channel group / DMA lane group
  const int H = p.H, W = p.W, HW = H * W, W2 = W2T ? W2T : h.w2, C = p.C, K = p.Kout;
  const int M = p.Mpix, nimg = M / HW;
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;

  const int bid = h.xmap ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
  const int part = bid % h.parts, z = bid / h.parts;
  const int k0 = (part % h.kparts) * 64, c0 = (part / h.kparts) * 64;
  const int ntiles = z < h.tiles_m ? (h.tiles_m - z + h.Z - 1) / h.Z : 0;

  // ---- DMA lanes.  dy: instruction j of this wave = rows 8 (4 wave + j) + lane/8 of the
  // tile (k-step image (row >> 5), mn_off<64> swizzle at the source)
  // (K % 64 == 32: the last k partition's upper 32 k read zeros - kok - and are not stored)
  uint32_t drow[4];
  bool kok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int row = 8 * (4 * wave + j) + (lane >> 3);
    const int chunk = (lane & 7) ^ mn_swz<64>(row & 31);
    // linear: + pixel0 * K * 2 per tile; STRIP: + (the row's pixel) * K * 2
    drow[j] = ((uint32_t)(STRIP ? 0 : row) * K + k0 + chunk * 8) * 2;
    kok[j] = k0 + chunk * 8 < K;
  }
  // halo: instruction j = pixels 16 (7 wave + j) + lane/4 of the image; chunk 1 of the
  // partition is the same lanes with the descriptor base 64 B further
  uint32_t hsc[HIW];
#pragma unroll
  for (int j = 0; j < HIW; ++j) {
    const uint32_t hp = 16 * (wave * HIW + j) + (lane >> 2);
    const uint32_t sl = udiv(hp, h.mag_w2);
    const uint32_t colp = hp - sl * W2;
    const uint32_t lc = (lane & 3) ^ (((hp >> 3) & 1) << 1);
    hsc[j] = sl | (colp << 10) | (lc << 18);
  }
  // buffer descriptors, once: dy and the partition's two 32-channel halo chunks
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(p.dy, h.dy_bytes);
  const __amdgpu_buffer_rsrc_t rx0 = make_rsrc(p.x, h.x_bytes);
  // (C % 64 == 32: the last channel partition's second chunk is an empty buffer: zeros)
  const __amdgpu_buffer_rsrc_t rx1 =
      make_rsrc((const char*)p.x + 64, c0 + 32 < C ? h.x_bytes : 0u);
  uint32_t hv[HIW], dv[4];
  // this wave's 16 channels: chunk (wave >> 1) of the halo, 16-B chunks 2 (wave & 1) + pp/2
  const int cbyte = ((2 * (wave & 1) + (pp >> 1)) << 4) + 8 * (pp & 1);
  // B-row addresses per (k-step, lo/hi, column tap dw): the swizzle bit is pixel bit 3,
  // and the row pitch W2 is a multiple of 16, so a tap's row offset dh * W2 never changes
  // it - the swizzled address of pixel (hp + dh*W2 + dw) is hbw[dw] + dh*W2*64.  hbw holds
  // the CURRENT tile's addresses at row tap dh = -1 including its stage's base (one set of
  // 24 registers: the MFMA waves of an 8-wave block have 256), and the next tile's are
  // computed after the current tile's MFMAs are issued
  const int hoff = HW_DBYTES + (ONECH ? 0 : (wave >> 1) * HW_HBYTES);
  auto stage_base = [&](int st) { return st * HW_STAGE + hoff - W2 * 64; };
  int hbw[4][2][3];
  const int tpx = STRIP ? h.tr * h.tw : HW_BM;
  if constexpr (STRIP) {
    // B-row addresses are tile-independent: local pixel n -> slot (lr + 1), column (lc + 1);
    // rows past the tile (dy rows zero) read its last pixel
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const uint32_t n = (uint32_t)min(ks * 32 + 8 * g + 4 * e + q, tpx - 1);
        const uint32_t lr = udiv1(n, h.mag_tw), lc = n - lr * h.tw;
        const int hp = (int)(lr + 1) * W2 + (int)lc + 1;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const int x = (hp + d - 1) * 64 + cbyte;
          hbw[ks][e][d] = (x ^ ((x >> 4) & 32)) + stage_base(0);
        }
      }
  }
  // a tile's DMA source offsets (halo hv, dy rows dv)
  auto prep_dma = [&](int mt) {
    if constexpr (STRIP) {
      const int img = (int)udiv1((uint32_t)mt, h.mag_timg);
      const uint32_t rem = (uint32_t)(mt - img * h.tiles_img);
      const uint32_t band = udiv1(rem, h.mag_tc);
      const int r0 = (int)band * h.tr, cs0 = (int)(rem - band * h.tiles_c) * h.tw;
#pragma unroll
      for (int j = 0; j < HIW; ++j) {
        const int sl = hsc[j] & 1023, col = (int)((hsc[j] >> 10) & 255);
        // (valid conv, pad 0: output (i, j) reads input rows i .. i + 2)
        const int ih = r0 - p.ph + sl, iw = cs0 - p.pw + col;
        const bool ok = sl < h.tr + 2 && col < h.tw + 2 && (unsigned)ih < (unsigned)H &&
                        (unsigned)iw < (unsigned)W;
        hv[j] = ok ? ((((uint32_t)img * H + ih) * W + iw) * C + c0) * 2 + (hsc[j] >> 18) * 16
                   : 0x80000000u;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t row = 8 * (4 * wave + j) + (lane >> 3);
        const uint32_t lr = udiv1(row, h.mag_tw), lc = row - lr * h.tw;
        const bool ok = (int)row < tpx && r0 + (int)lr < p.P && cs0 + (int)lc < p.Q && kok[j];
        dv[j] = ok ? drow[j] + (((uint32_t)img * p.P + r0 + lr) * p.Q + cs0 + lc) * (uint32_t)K * 2
                   : 0x80000000u;
      }
      return;
    }
    const int m0 = mt * HW_BM;
    const int img0 = m0 / HW;
    const int r0 = m0 - img0 * HW;
    const int oh0 = r0 / W;
#pragma unroll
    for (int j = 0; j < HIW; ++j) {
      const int sl = hsc[j] & 1023, col = (int)((hsc[j] >> 10) & 255) - 1;
      const int v = sl + oh0 - 1;
      const int d = (int)udiv((uint32_t)(v + H + 1), h.mag_h1) - 1;
      const int row = v - d * (H + 1);
      const int img = img0 + d;
      const bool ok = row < H && (unsigned)col < (unsigned)W && img < nimg;
      hv[j] = ok ? ((((uint32_t)img * H + row) * W + col) * C + c0) * 2 + (hsc[j] >> 18) * 16
                 : 0x80000000u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = 8 * (4 * wave + j) + (lane >> 3);
      dv[j] = (m0 + row < M && kok[j]) ? drow[j] + (uint32_t)m0 * K * 2 : 0x80000000u;
    }
  };
  // tile mt's B-row addresses in stage st (STRIP: tile-independent, only the stage moves)
  auto prep_b = [&](int mt, int st) {
    if constexpr (STRIP) {
      const int dlt = st ? HW_STAGE : -HW_STAGE;  // called for alternating stages
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int d = 0; d < 3; ++d) hbw[ks][e][d] += dlt;
    } else {
      const int hb0 = stage_base(st);
      const int m0 = mt * HW_BM;
      const int img0 = m0 / HW;
      const int r0 = m0 - img0 * HW;
      const int oh0 = r0 / W;
      const int mlast = M - 1 - img0 * HW;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const uint32_t n = (uint32_t)min(r0 + ks * 32 + 8 * g + 4 * e + q, mlast);
          const uint32_t di = udiv(n, h.mag_hw);
          const uint32_t rem = n - di * HW;
          const uint32_t oh = udiv(rem, h.mag_w);
          const uint32_t ow = rem - oh * W;
          const int hp = ((int)(di * (H + 1) + oh) - oh0 + 1) * W2 + (int)ow + 1;
#pragma unroll
          for (int d = 0; d < 3; ++d) {
            const int x = (hp + d - 1) * 64 + cbyte;
            hbw[ks][e][d] = (x ^ ((x >> 4) & 32)) + hb0;
          }
        }
    }
  };
  // DMA instruction j of a tile: dy rows (0..3), halo chunk 0 (4..10), halo chunk 1 (11..17)
  const uint32_t sw = lds_base(smem) + wave * 4096;  // this wave's DMA pieces: + 1 KiB each
  auto dmaw = [&](int stage, int j) {
    const uint32_t st = sw + stage * HW_STAGE;
    if (j < 4) {
      buf_lds16_at(rdy, st + j * 1024, dv[j]);
    } else if constexpr (ONECH) {
      const int jj = j - 4;
      buf_lds16_at(rx0, st - wave * 4096 + HW_DBYTES + (wave * HIW + jj) * 1024, hv[jj]);
    } else {
      const int ch = (j - 4) / HW_HIW, jj = (j - 4) % HW_HIW;
      buf_lds16_at(ch ? rx1 : rx0, st - wave * 4096 + HW_DBYTES + ch * HW_HBYTES +
                                       (wave * HW_HIW + jj) * 1024, hv[jj]);
    }
  };
  auto issue = [&](int stage) {
#pragma unroll
    for (int j = 0; j < 4 + 2 * HW_HIW; ++j) dmaw(stage, j);
  };

  if constexpr (PROD) {
    if (wave_all >= 4) {
      // ---- producers
      if (ntiles > 0) {
        prep_dma(z);
        issue(0);
      }
      for (int k = 0; k < ntiles; ++k) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile k landed (this wave's part)
        __builtin_amdgcn_s_barrier();  // publishes stage k & 1, frees stage (k + 1) & 1
        if (k + 1 < ntiles) {
          prep_dma(z + (k + 1) * h.Z);
          issue((k + 1) & 1);
        }
      }
      return;
    }
  }

  f32x4 acc[KM][9];
#pragma unroll
  for (int km = 0; km < KM; ++km)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[km][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (ntiles > 0) {
    if constexpr (!STRIP) prep_b(z, 0);
    if constexpr (!PROD) {
      prep_dma(z);
      issue(0);
    }
  }
  // tile k from stage k & 1; MORE (all but the block's last tile): prepare tile k + 1 and
  // (without producer waves) issue its 18 DMAs into the other stage inside this tile's MFMA
  // stream, one per two tap-steps.  The last tile is peeled so the loop body carries no
  // per-DMA branch.
  auto tile = [&](int k, auto nmore) {
    constexpr bool MORE = decltype(nmore)::value;
    const int st = k & 1;
    if constexpr (PROD) {
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    } else {
      wait_all_barrier();
    }
    // (hbw: this tile's B-row bases at row tap dh = -1 in stage st; tap dh adds
    // (dh+1)*W2*64, an immediate offset when W2T != 0)
    // 4-wave form: this tile's B-row bases are copied (hbk) and the next tile's DMA offsets
    // and bases computed up front, where their index math overlaps this tile's MFMA stream
    // (computed after the MFMAs instead, as the producer-wave form must for its register
    // budget, the 4-wave kernel was ~7 % slower: round-5 bisection)
    int hbk[4][2][3];
    if constexpr (!PROD) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int d = 0; d < 3; ++d) hbk[ks][e][d] = hbw[ks][e][d];
      if constexpr (MORE) {
        prep_dma(z + (k + 1) * h.Z);
        if constexpr (!STRIP) prep_b(z + (k + 1) * h.Z, st ^ 1);
      }
    }
    const char* sbase = smem + st * HW_STAGE;
    auto ld_b = [&](int j, s16x4& lo, s16x4& hi) {  // B fragment of step j = 9 ks + t
      const int ks = j / 9, t = j % 9, off = (t / 3) * W2 * 64;
      const int (&hb)[4][2][3] = PROD ? hbw : hbk;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + hb[ks][0][t % 3] + off));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, smem + hb[ks][1][t % 3] + off));
    };
    auto mma = [&](int t, const s16x4& lo, const s16x4& hi, const bf16x8 (&af)[KM]) {
      s16x8 r;
      r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
      r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, r);
#pragma unroll
      for (int km = 0; km < KM; ++km) acc[km][t] = mfma16(bfr, af[km], acc[km][t]);
    };
    if constexpr (PROD) {
      // Fenced schedule (sched_barrier), as the halo forward: the B fragment of step j + PD
      // and the next k-step's A fragments (4 steps ahead) are read in front of step j's
      // MFMAs and cannot sink below them.  Left to itself the scheduler read each tap's B
      // fragment right in front of its KM MFMAs (64 / 32 cycles), exposing an LDS round
      // trip per tap.  With KM = 2 for DenseNet's 32-output convs: +0.9 % DenseNet-121,
      // ResNet-18 within noise (round-5 same-box A/B, profiles/halo_sched_r5.txt).
      constexpr int PD = KM == 2 ? 6 : 3;
      s16x4 blo[PD + 1], bhi[PD + 1];
      bf16x8 af[2][KM];
#pragma unroll
      for (int km = 0; km < KM; ++km) af[0][km] = frag_mn<64>(sbase, 16 * km, lane);
#pragma unroll
      for (int j = 0; j < PD; ++j) ld_b(j, blo[j], bhi[j]);
#pragma unroll
      for (int j = 0; j < 36; ++j) {
        const int ks = j / 9, t = j % 9;
        if (j + PD < 36) ld_b(j + PD, blo[(j + PD) % (PD + 1)], bhi[(j + PD) % (PD + 1)]);
        if (t == 4 && ks + 1 < 4) {
#pragma unroll
          for (int km = 0; km < KM; ++km)
            af[(ks + 1) & 1][km] = frag_mn<64>(sbase + (ks + 1) * 4096, 16 * km, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(t, blo[j % (PD + 1)], bhi[j % (PD + 1)], af[ks & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bf16x8 af[KM];
#pragma unroll
        for (int km = 0; km < KM; ++km) af[km] = frag_mn<64>(sbase + ks * 4096, 16 * km, lane);
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          s16x4 lo, hi;
          ld_b(ks * 9 + t, lo, hi);
          mma(t, lo, hi, af);
          if constexpr (MORE && !PROD) {
            if (((ks * 9 + t) & 1) == 0) dmaw(st ^ 1, (ks * 9 + t) >> 1);
          }
        }
      }
    }
    // the next tile's B-row addresses (its stage is the other one), after this tile's last
    // fragment reads
    if constexpr (MORE && (PROD || STRIP)) prep_b(z + (k + 1) * h.Z, st ^ 1);
    // (no barrier: tile k + 2's DMAs into stage st follow tile k + 1's top barrier)
  };
  for (int k = 0; k + 1 < ntiles; ++k) tile(k, std::true_type{});
  if (ntiles > 0) tile(ntiles - 1, std::false_type{});
  // partial of this block -> slab z: dw[k][t][c] at k = k0 + 16 km + lane%16,
  // c = c0 + 16 wave + 4 (lane/16) .. +3
  const int64_t ncols = 9 * (int64_t)C;
  float* dst = p.slab + (int64_t)z * K * ncols;
  const int cw = c0 + 16 * wave;  // this wave's 16 channels (wave-uniform validity)
#pragma unroll
  for (int km = 0; km < KM; ++km) {
    const int kk = k0 + 16 * km + li;
    if (k0 + 16 * km >= K || cw >= C) continue;
#pragma unroll
    for (int t = 0; t < 9; ++t)
      *(f32x4*)(dst + (int64_t)kk * ncols + t * C + cw + 4 * g) = acc[km][t];
  }
}

// ------------------------------------------------------------------------------ host
static bool g_halo = [] {
  const char* e = getenv("MPA_HALO");
  return !(e && e[0] == '0');
}();
void igemm_set_halo(int on) { g_halo = on != 0; }
bool igemm_halo_enabled() { return g_halo; }

static uint32_t magic(uint32_t d) { return (uint32_t)((1ull << 32) / d + 1); }

static int num_cus() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        v <= 0)
      v = 256;
    return v;
  }();
  return n;
}

// CUs held by an overlapping collective (set by the host between kernel launches, read at
// launch time: a launch enqueued after a bucket's collective runs after it in stream order)
static std::atomic<int> g_comm_reserve{0};
void set_comm_reserve(int cus) { g_comm_reserve.store(std::max(0, cus)); }
int comm_reserve() { return g_comm_reserve.load(); }
int active_cus() {
  const int n = num_cus();
  const int r = g_comm_reserve.load();
  if (r <= 0) return n;
  // whole CUs per XCD: the persistent tile schedules split their blocks XCD-contiguously
  return std::max(8, (n - r) / 8 * 8);
}

// halo row pitch: W pixels + one zero column shared by consecutive rows (a row's right
// border is the next row's left border), rounded up to 8 pixels
static int halo_pitch(int W) { return (W + 1 + 7) / 8 * 8; }

// epilogue flavour of a launch; -1: not instantiated (the implicit GEMM runs it)
static int halo_epi(const IGemmArgs& a) {
  int e = 0;
  // fused BN reduction: the z-mask form only (y is never read; see EpiIn)
  if (a.ep_bnred)
    return (a.beta || a.relu || a.bias || a.ep_y || !a.ep_gamma || !a.ep_beta || !a.ep_mean ||
            !a.ep_rstd)
               ? -1
               : EP_BNRED;
  if (a.relu) e |= EP_RELU;
  if (a.beta) e |= EP_BETA;
  if (a.stats) e |= EP_STATS;
  if (a.bias) e |= EP_BIAS;
  switch (e) {
    case 0: case EP_BETA: case EP_STATS: case EP_BIAS | EP_RELU: case EP_BIAS | EP_STATS:
      return e;
    default:
      return -1;
  }
}

// eligibility of the halo engine (either tiling); `linear`: the 256-pixel linear tiles fit
// centre shift (ch, cw) of a 3x3 stride-1 tap set: the taps Oh + dh cover ch-1 .. ch+1 (same
// conv 0; valid conv 1; the valid conv's dgrad, padding 2, -1) and the output is the input
// less 2*ch rows / 2*cw columns
static bool tap_shift(const IGemmArgs& a, int& ch, int& cw) {
  int mh = 1 << 20, mw = 1 << 20;
  for (int t = 0; t < 9; ++t) {
    mh = std::min(mh, a.Oh + a.taps.dh[t]);
    mw = std::min(mw, a.Ow + a.taps.dw[t]);
  }
  ch = mh + 1;
  cw = mw + 1;
  if (ch < -1 || ch > 1 || cw < -1 || cw > 1) return false;
  int seen = 0;  // every relative (dh, dw) in {-1,0,1}^2 exactly once
  for (int t = 0; t < 9; ++t) {
    const int dh = a.Oh + a.taps.dh[t] - ch, dw = a.Ow + a.taps.dw[t] - cw;
    if (dh < -1 || dh > 1 || dw < -1 || dw > 1) return false;
    seen |= 1 << ((dh + 1) * 3 + dw + 1);
  }
  return seen == 511 && a.oH == a.aH - 2 * ch && a.oW == a.aW - 2 * cw;
}

static bool halo_ok_impl(const IGemmArgs& a, bool& linear) {
  linear = false;
  if (!g_halo || a.nphase > 0 || a.stap || a.T != 9 || a.Uh != 1 || a.Uw != 1) return false;
  if (a.aC % 32 != 0 || a.M <= 0 || a.oH <= 0 || a.oW <= 0) return false;
  // 64-wide column tiles, or one 32-wide tile (DenseNet's growth-rate convs, Inception's
  // Conv2d_2a) in the flavours instantiated for it (strip tiles: also accumulate / BN link)
  const int e32 = halo_epi(a);
  const bool n32_lin = a.N == 32 && (e32 == 0 || e32 == EP_STATS);
  if (a.N % HB_BN != 0 && !(a.N == 32 && (n32_lin || e32 == EP_BETA || e32 == EP_BNRED)))
    return false;
  // dense [M][ldc] output (stride-1 geometry), 32-bit element offsets in the epilogue
  if (a.dH != a.oH || a.dW != a.oW || a.Uoh != 1 || a.Uow != 1 || a.Poh != 0 || a.Pow != 0)
    return false;
  if ((int64_t)a.M * a.ldc >= (1ll << 31) || a.ldc < a.N) return false;
  if (halo_epi(a) < 0) return false;  // an epilogue flavour without an instantiation
  if (a.Ktot != 9 * a.aC) return false;
  int ch, cw;
  if (!tap_shift(a, ch, cw)) return false;
  const int64_t HW = (int64_t)a.aH * a.aW, OHW = (int64_t)a.oH * a.oW;
  if (a.M % OHW != 0) return false;
  if ((int64_t)(a.M / OHW) * HW * a.aC * 2 >= (1ll << 31)) return false;
  if ((int64_t)a.N * a.ldb * 2 >= (1ll << 31)) return false;
  // (strip tiles only: shifted tap sets - valid convs and their dgrads - and wide images)
  if (ch != 0 || cw != 0 || HW + HB_BM >= 65536 || a.aW + 2 > 255) return true;
  // halo slots of any 256-pixel tile: rows touched + 2 halo rows + image separators
  const int64_t rows = (HB_BM - 1 + a.aW - 1) / a.aW + 1;
  const int64_t seps = (HB_BM - 1) / HW + 1;
  // (+1: with P == W + 1 the last slot's right border is the next pixel)
  const int P = halo_pitch(a.aW);
  linear = (rows + 2 + seps) * P + (P == a.aW + 1 ? 1 : 0) <= HB_HPX &&
           (a.N % HB_BN == 0 || n32_lin);
  return true;
}

// MPA_HALO_WRES=0: no resident-weight variant (A/B of the 64-channel layers)
static const bool g_halo_wres = [] {
  const char* e = getenv("MPA_HALO_WRES");
  return !(e && atoi(e) == 0);
}();

// ------------------------------------------------------------------ strip tiles (host)
// MPA_HALO_STRIP: 0 off; 1 (default) images too wide for the linear tiles; 2 also the
// resident-weight layers whose strips leave room for a third stage (ResNet layer1)
static int g_strip = [] {
  const char* e = getenv("MPA_HALO_STRIP");
  return e ? atoi(e) : 1;
}();
void igemm_set_halo_strip(int mode) { g_strip = mode; }

static bool strip_plan(const IGemmArgs& a, StripPlan& h, bool& wres, int& ns) {
  const int W = a.oW, H = a.oH;  // tiles cover the output image
  if ((a.N % HB_BN != 0 && a.N != 32) || W < 8) return false;
  if (!tap_shift(a, h.ch, h.cw)) return false;
  const int nstrip = (W + 127) / 128;
  const int TW = (W + nstrip - 1) / nstrip;
  int TR = std::max(1, std::min(H, HB_BM / TW));
  const int P = (TW + 2 + 7) / 8 * 8;
  while (TR > 1 && ((TR + 2) * P + 63) / 64 > HB_HIW) --TR;
  const int hiw = ((TR + 2) * P + 63) / 64;
  if (hiw > HB_HIW || 2 * TR * TW < HB_BM) return false;  // at least half the MFMA rows live
  h.tr = TR;
  h.tw = TW;
  h.p = P;
  h.hiw = hiw;
  h.tiles_c = (W + TW - 1) / TW;
  h.tiles_img = ((H + TR - 1) / TR) * h.tiles_c;
  h.cc = a.aC / 32;
  const int nimg = a.M / (H * W);  // (output pixels per image)
  wres = g_halo_wres && (a.N + HB_BN - 1) / HB_BN == 1 && h.cc <= 2;
  const int lds = 2 * HB_HBYTES + 2 * HB_WBYTES;
  ns = 2;
  if (wres && 3 * hiw * 4096 + h.cc * HB_WBYTES <= lds) ns = 3;
  if (ns * hiw * 4096 + (wres ? h.cc : ns) * HB_WBYTES > lds) return false;
  h.mag_tw = magic(TW);
  h.mag_p = magic(P);
  h.mag_tc = h.tiles_c > 1 ? magic(h.tiles_c) : 0u;
  h.mag_timg = h.tiles_img > 1 ? magic(h.tiles_img) : 0u;
  h.tiles_total = nimg * h.tiles_img * ((a.N + HB_BN - 1) / HB_BN);
  return (int64_t)nimg * h.tiles_img < (1 << 24);
}

template <int EPI, int NJ = 4>
static void launch_strip(bool wres, int ns, int grid, const IGemmArgs& a, const StripPlan& h,
                         hipStream_t s) {
  if (wres && ns == 3)
    hipLaunchKernelGGL((conv3_strip_kernel<true, EPI, 3, NJ>), dim3(grid), dim3(512), 0, s, a, h);
  else if (wres)
    hipLaunchKernelGGL((conv3_strip_kernel<true, EPI, 2, NJ>), dim3(grid), dim3(512), 0, s, a, h);
  else
    hipLaunchKernelGGL((conv3_strip_kernel<false, EPI, 2, NJ>), dim3(grid), dim3(512), 0, s, a, h);
}

static int conv3_strip(IGemmArgs a, hipStream_t s) {
  StripPlan h{};
  bool wres;
  int ns;
  strip_plan(a, h, wres, ns);
  for (int t = 0; t < 9; ++t) {
    const int r = (a.Oh + a.taps.dh[t] - h.ch + 1) * 3 + (a.Ow + a.taps.dw[t] - h.cw + 1);
    h.btoff[r] = a.taps.bt[t] * a.aC * 2;
  }
  h.a_bytes = (uint32_t)((int64_t)(a.M / ((int64_t)a.oH * a.oW)) * a.aH * a.aW * a.aC * 2);
  h.b_bytes = (uint32_t)((int64_t)a.N * a.ldb * 2);
  a.tiles_n = (a.N + HB_BN - 1) / HB_BN;
  a.tiles_total = h.tiles_total;
  int g8 = std::min(std::min(active_cus(), HALO_MAX_ROWS) / 8, (h.tiles_total + 7) / 8);
  g8 = std::max(a.tiles_n, g8 / a.tiles_n * a.tiles_n);
  const int grid = 8 * g8;
  if (a.N == 32) {  // one 32-wide column tile (NJ = 2)
    switch (halo_epi(a)) {
      case 0: launch_strip<0, 2>(wres, ns, grid, a, h, s); break;
      case EP_STATS: launch_strip<EP_STATS, 2>(wres, ns, grid, a, h, s); break;
      case EP_BETA: launch_strip<EP_BETA, 2>(wres, ns, grid, a, h, s); break;
      default: launch_strip<EP_BNRED, 2>(wres, ns, grid, a, h, s); break;
    }
    return grid;
  }
  switch (halo_epi(a)) {
    case 0: launch_strip<0>(wres, ns, grid, a, h, s); break;
    case EP_BETA: launch_strip<EP_BETA>(wres, ns, grid, a, h, s); break;
    case EP_STATS: launch_strip<EP_STATS>(wres, ns, grid, a, h, s); break;
    case EP_BIAS | EP_RELU: launch_strip<EP_BIAS | EP_RELU>(wres, ns, grid, a, h, s); break;
    case EP_BIAS | EP_STATS: launch_strip<EP_BIAS | EP_STATS>(wres, ns, grid, a, h, s); break;
    default: launch_strip<EP_BNRED>(wres, ns, grid, a, h, s); break;
  }
  return grid;
}

// strip tiles for this launch: images the linear tiles cannot hold, or (MPA_HALO_STRIP=2)
// resident-weight layers that get a third stage
static bool use_strip(const IGemmArgs& a, bool linear) {
  if (g_strip < 1) return false;
  StripPlan h{};
  bool wres;
  int ns;
  if (!strip_plan(a, h, wres, ns)) return false;
  return !linear || (g_strip >= 2 && ns == 3);
}

bool conv3_halo_ok(const IGemmArgs& a) {
  bool linear;
  if (!halo_ok_impl(a, linear)) return false;
  return linear || use_strip(a, linear);
}

// Producer waves (PROD: 8-wave blocks, DMAs off the MFMA waves; each MFMA wave then has
// 256 registers, which every flavour fits) for every launch: issuing the DMAs between the
// MFMAs cost the MFMA waves ~10 % (round-2 A/B), and the fused BN-backward reduction
// flavour, reduced per column group (TRED), fits 256 registers without scratch

template <int EPI, int NJ>
static void launch_halo_k(bool wres, int grid, const IGemmArgs& a, const HaloPlan& h,
                          hipStream_t s, bool mi7 = false) {
  if constexpr (NJ == 4 && (EPI == 0 || EPI == EP_STATS)) {
    if (mi7) {  // (halo_mi7_ok: resident weights, whole 448-pixel tiles)
      hipLaunchKernelGGL((conv3_halo_kernel<true, EPI, true, 4, 7>), dim3(grid), dim3(256), 0, s,
                         a, h);
      return;
    }
  }
  const bool full = a.M % HB_BM == 0;  // no tile ends past M: branch-free epilogue everywhere
  if (wres && full)
    hipLaunchKernelGGL((conv3_halo_kernel<true, EPI, true, NJ>), dim3(grid), dim3(512), 0, s, a, h);
  else if (wres)
    hipLaunchKernelGGL((conv3_halo_kernel<true, EPI, false, NJ>), dim3(grid), dim3(512), 0, s, a, h);
  else if (full)
    hipLaunchKernelGGL((conv3_halo_kernel<false, EPI, true, NJ>), dim3(grid), dim3(512), 0, s, a, h);
  else
    hipLaunchKernelGGL((conv3_halo_kernel<false, EPI, false, NJ>), dim3(grid), dim3(512), 0, s, a, h);
}

template <int EPI>
static void launch_halo(bool wres, int grid, const IGemmArgs& a, const HaloPlan& h,
                        hipStream_t s, bool mi7 = false) {
  launch_halo_k<EPI, 4>(wres, grid, a, h, s, mi7);
}

// MPA_HALO_MI7=0: keep the 256-pixel tiles for the resident-weight layers (A/B)
static int g_halo_mi7 = [] {
  const char* e = getenv("MPA_HALO_MI7");
  return e ? atoi(e) : 1;
}();
void igemm_set_halo_mi7(int on) { g_halo_mi7 = on; }

// 448-pixel tiles (MI = 7): same-conv tap set, one resident 64-wide weight tile, tiles of
// whole image rows that never cross an image (HW % 448 == 0, 448 % W == 0) and whose
// (448 / W + 2)-slot halo fits the 640-pixel stage
static bool halo_mi7_ok(const IGemmArgs& a, int epi, bool wres) {
  if (!g_halo_mi7 || !wres || a.N != HB_BN) return false;
  // (the accumulate / BN-link dgrad flavours spill 92-102 B/lane at 448 pixels: not yet)
  if (epi != 0 && epi != EP_STATS) return false;
  int ch, cw;
  if (!tap_shift(a, ch, cw) || ch != 0 || cw != 0) return false;
  const int64_t HW = (int64_t)a.aH * a.aW;
  constexpr int BM7 = 448;
  if (HW % BM7 != 0 || BM7 % a.aW != 0 || a.M % BM7 != 0) return false;
  return (BM7 / a.aW + 2) * halo_pitch(a.aW) <= 640;
}

// N == 32 (plain and statistics epilogues only; producer-wave blocks)
template <int EPI>
static void launch_halo32(bool wres, int grid, const IGemmArgs& a, const HaloPlan& h,
                          hipStream_t s) {
  launch_halo_k<EPI, 2>(wres, grid, a, h, s);
}

// Launch (conv3_halo_ok(a) must hold; B K-contiguous with the tap map in a.taps.bt);
// returns the number of statistics-slab rows written (one per block, <= HALO_MAX_ROWS).
int conv3_halo(IGemmArgs a, hipStream_t s) {
  {
    bool linear;
    halo_ok_impl(a, linear);
    if (use_strip(a, linear)) return conv3_strip(a, s);
  }
  HaloPlan h{};
  const int W2 = halo_pitch(a.aW);
  h.w2 = W2;
  for (int t = 0; t < 9; ++t) {  // raster (dh, dw) order, whatever order the table had
    const int r = (a.Oh + a.taps.dh[t] + 1) * 3 + (a.Ow + a.taps.dw[t] + 1);
    h.btoff[r] = a.taps.bt[t] * a.aC * 2;
  }
  h.mag_w = magic(a.aW);
  h.mag_w2 = magic(W2);
  h.mag_h1 = magic(a.aH + 1);
  h.mag_hw = magic(a.aH * a.aW);
  h.cc = a.aC / 32;
  const bool wres = g_halo_wres && (a.N + HB_BN - 1) / HB_BN == 1 && h.cc <= 2;
  const bool mi7 = halo_mi7_ok(a, halo_epi(a), wres);
  h.tiles_m = mi7 ? a.M / 448 : (a.M + HB_BM - 1) / HB_BM;
  a.tiles_n = (a.N + HB_BN - 1) / HB_BN;
  h.tiles_total = h.tiles_m * a.tiles_n;
  a.tiles_total = h.tiles_total;
  h.a_bytes = (uint32_t)((int64_t)a.M * a.aC * 2);
  h.b_bytes = (uint32_t)((int64_t)a.N * a.ldb * 2);
  // persistent grid: G8 blocks per XCD, a multiple of tiles_n (fixed column tile per block)
  int g8 = std::min(std::min(active_cus(), HALO_MAX_ROWS) / 8, (h.tiles_total + 7) / 8);
  g8 = std::max(a.tiles_n, g8 / a.tiles_n * a.tiles_n);
  const int grid = 8 * g8;
  if (a.N == 32) {
    if (halo_epi(a) == EP_STATS) launch_halo32<EP_STATS>(wres, grid, a, h, s);
    else launch_halo32<0>(wres, grid, a, h, s);
    return grid;
  }
  switch (halo_epi(a)) {
    case 0: launch_halo<0>(wres, grid, a, h, s, mi7); break;
    case EP_BETA: launch_halo<EP_BETA>(wres, grid, a, h, s); break;
    case EP_STATS: launch_halo<EP_STATS>(wres, grid, a, h, s, mi7); break;
    case EP_BIAS | EP_RELU: launch_halo<EP_BIAS | EP_RELU>(wres, grid, a, h, s); break;
    case EP_BIAS | EP_STATS: launch_halo<EP_BIAS | EP_STATS>(wres, grid, a, h, s); break;
    default: launch_halo<EP_BNRED>(wres, grid, a, h, s); break;
  }
  return grid;
}

// ------------------------------------------------------------------ halo wgrad host
static int halo_wgrad_pitch(int W) { return (W + 2 + 15) / 16 * 16; }

// shape checks shared by the linear and strip tilings
// (pad 1: same conv; pad 0: valid conv, strip tiles only - its dy is the smaller image)
static bool halo_wgrad_base(const WGradArgs& a) {
  if (!g_halo || a.R != 3 || a.S != 3 || a.sh != 1 || a.sw != 1) return false;
  if (a.ph < 0 || a.ph > 1 || a.pw < 0 || a.pw > 1) return false;
  if (a.P != a.H + 2 * a.ph - 2 || a.Q != a.W + 2 * a.pw - 2 || a.P <= 0 || a.Q <= 0) return false;
  // 64 x 64 partitions; a 32-wide remainder in either dimension is zero-filled
  if (a.C % 32 != 0 || a.Kout % 32 != 0) return false;
  const int64_t PQ = (int64_t)a.P * a.Q;
  if (a.Mpix % PQ != 0) return false;
  const int64_t nimg = a.Mpix / PQ;
  return nimg * a.H * a.W * a.C * 2 < (1ll << 31) && (int64_t)a.Mpix * a.Kout * 2 < (1ll << 31);
}

// strip tiling of the weight gradient (images too wide for the linear tiles): the TR x TW
// tile (TR * TW <= 128 pixels) minimising tiles x (128 MFMA rows + staged halo pixels)
static bool halo_wgrad_strip_plan(const WGradArgs& a, HaloWPlan& h) {
  if (g_strip < 1 || !halo_wgrad_base(a)) return false;
  const int OH = a.P, OW = a.Q;  // tiles cover dy (the conv output)
  const int64_t nimg = a.Mpix / ((int64_t)OH * OW);
  int64_t best = -1;
  for (int n = 1; n <= OW; ++n) {
    const int tw = (OW + n - 1) / n;
    if (tw > 126 || (n > 1 && (OW + tw - 1) / tw != n)) continue;
    if (tw < 8) break;
    const int pitch = (tw + 2 + 15) / 16 * 16;
    int tr = std::max(1, std::min(OH, HW_BM / tw));
    while (tr > 1 && (tr + 2) * pitch > HW_HPX) --tr;
    if ((tr + 2) * pitch > HW_HPX) continue;
    const int64_t tiles = nimg * ((OH + tr - 1) / tr) * n;
    const int64_t cost = tiles * (HW_BM + (tr + 2) * pitch);
    if (best < 0 || cost < best) {
      best = cost;
      h.tr = tr;
      h.tw = tw;
      h.w2 = pitch;
      h.tiles_c = n;
      h.tiles_img = ((OH + tr - 1) / tr) * n;
      h.tiles_m = (int)tiles;
    }
  }
  if (best < 0 || h.tiles_m <= 0) return false;
  h.mag_tw = magic(h.tw);
  h.mag_tc = h.tiles_c > 1 ? magic(h.tiles_c) : 0u;
  h.mag_timg = h.tiles_img > 1 ? magic(h.tiles_img) : 0u;
  return true;
}

static bool halo_wgrad_geom(const WGradArgs& a) {
  if (!halo_wgrad_base(a) || a.ph != 1 || a.pw != 1) return false;
  const int64_t HW = (int64_t)a.H * a.W;
  if (HW + HW_BM >= 65536 || a.W + 2 > 255) return false;
  const int64_t rows = (HW_BM - 1 + a.W - 1) / a.W + 1;
  const int64_t seps = (HW_BM - 1) / HW + 1;
  // 32-channel partitions may use both chunk areas for one wider halo image (ONECH)
  return (rows + 2 + seps) * halo_wgrad_pitch(a.W) <= (a.C == 32 ? 2 : 1) * HW_HPX;
}

// one 32-channel chunk whose halo needs the combined image
static bool halo_wgrad_onech(const WGradArgs& a) {
  const int64_t HW = (int64_t)a.H * a.W;
  const int64_t rows = (HW_BM - 1 + a.W - 1) / a.W + 1;
  const int64_t seps = (HW_BM - 1) / HW + 1;
  return a.C == 32 && (rows + 2 + seps) * halo_wgrad_pitch(a.W) > HW_HPX;
}

int64_t conv3_halo_wgrad_ws_floats(int Kout, int Ncols) {
  if (Ncols % 9 != 0 || (Ncols / 9) % 32 != 0 || Kout % 32 != 0) return 0;
  return (int64_t)HALO_MAX_ROWS * 64 * 64 * 9;  // <= 256 blocks x one 64x9x64 partition
}

bool conv3_halo_wgrad_ok(const WGradArgs& a) {
  if (a.slab == nullptr) return false;
  if (halo_wgrad_geom(a)) return true;
  HaloWPlan h{};
  return halo_wgrad_strip_plan(a, h);
}

// Producer-wave weight-gradient kernels (PROD) for the linear tiles: the 13 ResNet-18 halo
// weight gradients take 3.14 ms instead of 3.63 ms per b1024 step, +2.4 % single-stream
// (round-5 A/B, profiles/wprod_pre_ab_r5.txt).  MPA_HALO_WPROD=0: the 4-wave form (the
// MFMA waves issue the DMAs).
// XCD-grouped weight-gradient block order (HaloWPlan::xmap); MPA_HALO_WXMAP=0: plain order
static bool g_wxmap = [] {
  const char* e = getenv("MPA_HALO_WXMAP");
  return !(e && e[0] == '0');
}();

static bool g_wprod = [] {
  const char* e = getenv("MPA_HALO_WPROD");
  return !(e && e[0] == '0');
}();
void igemm_set_halo_wprod(int on) { g_wprod = on != 0; }
void igemm_set_halo_wxmap(int on) { g_wxmap = on != 0; }

// (8-wave forms use the run-time pitch: with a compile-time pitch the MFMA waves' hoisted
// tap addresses spill past their 256 registers)
template <int W2T, bool ONECH = false, bool STRIP = false>
static void launch_halo_wgrad(const WGradArgs& a, const HaloWPlan& h, dim3 grid, hipStream_t s) {
  if constexpr (!STRIP) {
    if (g_wprod) {
      if (a.Kout == 32)
        hipLaunchKernelGGL((conv3_halo_wgrad_kernel<0, ONECH, false, true, 2>), grid,
                           dim3(512), 0, s, a, h);
      else
        hipLaunchKernelGGL((conv3_halo_wgrad_kernel<0, ONECH, false, true>), grid,
                           dim3(512), 0, s, a, h);
      return;
    }
  }
  hipLaunchKernelGGL((conv3_halo_wgrad_kernel<W2T, ONECH, STRIP>), grid, dim3(256), 0, s, a, h);
}

// slab partials -> returns Z (slabs of [Kout][9C] to sum into dw)
int conv3_halo_wgrad(WGradArgs a, hipStream_t s) {
  HaloWPlan h{};
  if (!halo_wgrad_geom(a) && halo_wgrad_strip_plan(a, h)) {
    const int W2 = h.w2;
    for (int t = 0; t < 9; ++t) h.toff[t] = (t / 3 - 1) * W2 + (t % 3 - 1);
    h.mag_w2 = magic(W2);
    h.kparts = (a.Kout + 63) / 64;
    h.parts = h.kparts * ((a.C + 63) / 64);
    const int G = std::min(active_cus(), HALO_MAX_ROWS);
    h.Z = std::max(1, std::min(G / h.parts, h.tiles_m));
    h.dy_bytes = (uint32_t)((int64_t)a.Mpix * a.Kout * 2);
    h.x_bytes = (uint32_t)((int64_t)(a.Mpix / ((int64_t)a.P * a.Q)) * a.H * a.W * a.C * 2);
    h.xmap = g_wxmap && (h.parts * h.Z) % 8 == 0;
    launch_halo_wgrad<0, false, true>(a, h, dim3(h.parts * h.Z), s);
    return h.Z;
  }
  const int W2 = halo_wgrad_pitch(a.W);
  h.w2 = W2;
  for (int t = 0; t < 9; ++t) h.toff[t] = (t / 3 - 1) * W2 + (t % 3 - 1);
  h.mag_w = magic(a.W);
  h.mag_w2 = magic(W2);
  h.mag_h1 = magic(a.H + 1);
  h.mag_hw = magic(a.H * a.W);
  h.tiles_m = (a.Mpix + HW_BM - 1) / HW_BM;
  h.kparts = (a.Kout + 63) / 64;
  h.parts = h.kparts * ((a.C + 63) / 64);
  const int G = std::min(active_cus(), HALO_MAX_ROWS);
  h.Z = std::max(1, std::min(G / h.parts, h.tiles_m));
  h.dy_bytes = (uint32_t)((int64_t)a.Mpix * a.Kout * 2);
  h.x_bytes = (uint32_t)((int64_t)a.Mpix * a.C * 2);
  const dim3 grid(h.parts * h.Z);
  h.xmap = g_wxmap && (h.parts * h.Z) % 8 == 0;
  if (halo_wgrad_onech(a)) {
    launch_halo_wgrad<0, true>(a, h, grid, s);
    return h.Z;
  }
  switch (W2) {
    case 16: launch_halo_wgrad<16>(a, h, grid, s); break;
    case 32: launch_halo_wgrad<32>(a, h, grid, s); break;
    case 48: launch_halo_wgrad<48>(a, h, grid, s); break;
    case 64: launch_halo_wgrad<64>(a, h, grid, s); break;
    default: launch_halo_wgrad<0>(a, h, grid, s); break;
  }
  return h.Z;
}

}  // namespace mpa
