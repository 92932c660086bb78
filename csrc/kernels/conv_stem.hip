// Direct, row-staged forward of the pixel-pair image stem (ResNet-18/34 and DenseNet-121's
// 7x7 / stride-2 conv, 3 -> 64 channels; reference models.py:24-30, 74-80 reach it through
// torchvision).  models/layers.py stores the image as a zero-bordered canvas of 8-channel
// pixel pairs, which makes the stem a stride-(sh, 1) conv with a 7 x 4 kernel over 8
// channels: per kernel row dh exactly one 32-deep MFMA K step (4 pairs x 8 channels).
//
// Why a dedicated kernel: as an implicit GEMM (igemm_rows_dma_uni_kernel) the stem is
// K = 224 deep - 7 K steps per 128 x 64 tile - so each tile is dominated by its fixed costs
// (row-address divisions, the 3-stage DMA ring fill, the per-tile BN-statistics reduction
// through LDS and a slab row per tile) and by the 4x re-fetch of overlapping A rows
// (neighbouring output pixels read 64-B windows 16 B apart).  Measured 660-700 us per
// batch-512 pass against a 121 us write floor (tools/stem_sweep.py).
//
// Design (gfx950, 64-wide waves, 160 KB LDS per CU):
//   * persistent blocks of 8 waves, one per CU (grid <= 256 = one statistics-slab row
//     each; MPA_STEM_CFG=1: 4 waves, two per CU); a work item is 8 (4) output rows of one
//     image;
//   * the item's (8 - 1) * sh + 7 canvas rows are staged ONCE into LDS (16-B vectors, plain
//     loads into registers issued before the current item's MFMAs, written after them), so
//     every A fragment - row q + kchunk of canvas row 2 pr + dh - is one ds_read_b128;
//   * all 7 x 4 weight fragments (64 channels x 224) live in 112 VGPRs for the whole kernel;
//   * per 16-pixel subtile: 7 dh x 4 channel blocks = 28 MFMA 16x16x32 bf16, then the
//     epilogue in registers: + bias, ReLU, bf16 store (8 B per lane, full 128-B pixel rows
//     across the 4 channel blocks), and the shifted BN sums of the bf16-rounded outputs
//     accumulated PER LANE across all the block's items - reduced once at the end (shuffles
//     over the 16 pixel lanes, LDS across the 8 waves) into the block's slab row.
#include "common.h"
#include "api.h"
#include "igemm_common.h"
#include <algorithm>
#include <cstdlib>

namespace mpa {

namespace {
constexpr int STEM_R = 7;             // kernel rows (7x7 stem)
constexpr int STEM_MAX_WP = 120;      // canvas pairs per row (image width <= 232)
}  // namespace

struct StemPlan {
  int items;        // N * ceil(P / 8)
  int items_img;    // ceil(P / 8)
  int crows;        // canvas rows per item: (8 - 1) * sh + 7
  int qsub;         // 16-pixel subtiles per output row: ceil(Q / 16)
};

// STEM_NW waves per block, STEM_ROWS output rows per item, STEM_OCC waves per SIMD
template <int STEM_NW, int STEM_ROWS, int STEM_OCC>
__global__ __launch_bounds__(STEM_NW * 64, STEM_OCC) void conv_stem_kernel(IGemmArgs p,
                                                                           StemPlan h) {
  constexpr int STEM_MAX_CROWS = (STEM_ROWS - 1) * 2 + STEM_R;  // canvas rows, sh <= 2
  constexpr int STEM_LDS = STEM_MAX_CROWS * STEM_MAX_WP * 16;
  constexpr int STEM_PREF = (STEM_LDS / 16 + STEM_NW * 64 - 1) / (STEM_NW * 64);  // vec/thread
  __shared__ __attribute__((aligned(16))) char canvas[STEM_LDS];
  __shared__ float red[STEM_NW][2][64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kc = lane >> 4, li = lane & 15;
  const int Wp = p.aW, P = p.oH, Q = p.oW, sh = p.Uh;
  const int rowvec = Wp;                       // 16-B vectors per canvas row
  const int itemvec = h.crows * rowvec;        // vectors staged per item
  const bf16_t* __restrict__ A = (const bf16_t*)p.A;
  bf16_t* __restrict__ out = (bf16_t*)p.C;

  static_assert(STEM_PREF * STEM_NW * 64 * 16 >= STEM_LDS, "prefetch covers the stage");
  // weights: lane holds W[n = 16 nb + li][dh][pair kc][0..7] for every (dh, nb)
  bf16x8 wf[STEM_R][4];
#pragma unroll
  for (int dh = 0; dh < STEM_R; ++dh)
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
      wf[dh][nb] = __builtin_bit_cast(
          bf16x8, *(const u32x4*)((const bf16_t*)p.B + (size_t)(16 * nb + li) * p.ldb + dh * 32 +
                                  kc * 8));
  // epilogue constants of this lane's 16 channels n = 16 nb + 4 kc + r
  float bias[4][4], shift[4][4], s[4][4], q2[4][4];
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * nb + 4 * kc + r;
      bias[nb][r] = p.bias ? p.bias[n] : 0.f;
      shift[nb][r] = p.stats_shift ? p.stats_shift[n] : 0.f;
      s[nb][r] = 0.f;
      q2[nb][r] = 0.f;
    }

  auto item_src = [&](int it) -> const u32x4* {
    const int img = it / h.items_img, p0 = (it - img * h.items_img) * STEM_ROWS;
    return (const u32x4*)(A + ((size_t)img * p.aH + (size_t)p0 * sh) * Wp * 8);
  };
  // rows past the canvas (last item of an image, P % 8 != 0) are clamped: they only feed
  // output rows that are not stored
  auto item_rows_avail = [&](int it) -> int {
    const int img = it / h.items_img, p0 = (it - img * h.items_img) * STEM_ROWS;
    return min(h.crows, p.aH - p0 * sh);
  };
  u32x4 pref[STEM_PREF];
  auto prefetch = [&](int it) {
    const u32x4* src = item_src(it);
    const int lim = item_rows_avail(it) * rowvec;
#pragma unroll
    for (int i = 0; i < STEM_PREF; ++i) {
      const int v = tid + i * STEM_NW * 64;
      pref[i] = (v < itemvec) ? src[min(v, lim - 1)] : u32x4{0, 0, 0, 0};
    }
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < STEM_PREF; ++i) {
      const int v = tid + i * STEM_NW * 64;
      if (v < itemvec) *LDS_PTR(u32x4, canvas + v * 16) = pref[i];
    }
  };

  int it = blockIdx.x;
  if (it < h.items) {
    prefetch(it);
    commit();
  }
  __syncthreads();
  const int nsub = STEM_ROWS * h.qsub;
  for (; it < h.items; it += gridDim.x) {
    const int nxt = it + gridDim.x;
    if (nxt < h.items) prefetch(nxt);  // lands during this item's MFMAs
    const int img = it / h.items_img, p0 = (it - img * h.items_img) * STEM_ROWS;
    for (int t = wave; t < nsub; t += STEM_NW) {
      const int pr = t / h.qsub;                 // wave-uniform
      const int q0 = (t - pr * h.qsub) * 16;
      if (p0 + pr >= P) break;                   // t grows with pr: the rest is past P too
      const int q = min(q0 + li, Q - 1);
      f32x4 acc[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* abase = canvas + ((pr * sh) * rowvec + q + kc) * 16;
#pragma unroll
      for (int dh = 0; dh < STEM_R; ++dh) {
        const bf16x8 af =
            __builtin_bit_cast(bf16x8, *LDS_PTR(const u32x4, abase + dh * rowvec * 16));
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[nb] = mfma16(wf[dh][nb], af, acc[nb]);
      }
      if (q0 + li < Q) {
        bf16_t* orow = out + ((size_t)(img * P + p0 + pr) * Q + q0 + li) * p.ldc + 4 * kc;
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t2 = acc[nb][r] + bias[nb][r];
            if (p.relu) t2 = fmaxf(t2, 0.f);
            v[r] = t2;
          }
          const uint32_t lo = pack2(v[0], v[1]), hi = pack2(v[2], v[3]);
          *(uint2*)(orow + 16 * nb) = make_uint2(lo, hi);
          // statistics of the stored (bf16-rounded) values, shifted
          const float r0 = bf2f(lo & 0xffff) - shift[nb][0], r1 = bf2f(lo >> 16) - shift[nb][1];
          const float r2 = bf2f(hi & 0xffff) - shift[nb][2], r3 = bf2f(hi >> 16) - shift[nb][3];
          s[nb][0] += r0; q2[nb][0] = __builtin_fmaf(r0, r0, q2[nb][0]);
          s[nb][1] += r1; q2[nb][1] = __builtin_fmaf(r1, r1, q2[nb][1]);
          s[nb][2] += r2; q2[nb][2] = __builtin_fmaf(r2, r2, q2[nb][2]);
          s[nb][3] += r3; q2[nb][3] = __builtin_fmaf(r3, r3, q2[nb][3]);
        }
      }
    }
    __syncthreads();  // every wave is done reading this item's canvas rows
    if (nxt < h.items) commit();
    __syncthreads();
  }

  if (!p.stats) return;
  // reduce over the 16 pixel lanes that share kc, then across the waves
#pragma unroll
  for (int nb = 0; nb < 4; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float a = s[nb][r], b = q2[nb][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
      }
      if (li == 0) {
        red[wave][0][16 * nb + 4 * kc + r] = a;
        red[wave][1][16 * nb + 4 * kc + r] = b;
      }
    }
  __syncthreads();
  if (tid < 128) {
    const int which = tid >> 6, n = tid & 63;
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < STEM_NW; ++w) acc += red[w][which][n];
    p.stats[(size_t)blockIdx.x * 2 * 64 + which * 64 + n] = acc;
  }
}

static int g_stem_on = [] {
  const char* e = getenv("MPA_STEM_DIRECT");
  return e ? atoi(e) : 1;
}();
void igemm_set_stem(int on) { g_stem_on = on; }

bool conv_stem_ok(const IGemmArgs& a) {
  if (!g_stem_on || !a.stap || a.aC != 8 || a.N != 64 || a.ldc != 64 || a.T != STEM_R || a.Ktot != 224 ||
      a.ldb != 224 || a.Uw != 1 || a.Oh != 0 || a.Ow != 0 || a.beta || a.nphase || a.ep_bnred ||
      a.Uh < 1 || a.Uh > 2 || a.aW != a.oW + 3 || a.aW > STEM_MAX_WP)
    return false;
  if ((reinterpret_cast<uintptr_t>(a.A) | reinterpret_cast<uintptr_t>(a.B) |
       reinterpret_cast<uintptr_t>(a.C)) & 15)
    return false;
  if (a.aH < (a.oH - 1) * a.Uh + STEM_R || a.M % (a.oH * a.oW) != 0) return false;
  for (int t = 0; t < STEM_R; ++t)  // one super-tap per kernel row: dh = t, dw = 0, 4 columns
    if (a.taps.dh[t] != t || a.taps.dw[t] != 0 || a.taps.bt[t] != ((t * 4) | (4 << 12)))
      return false;
  return true;
}

// block shape: 0 = 8 waves x 8-row items, one block per CU; 1 = 4 waves x 4-row items, two
// blocks per CU (one block's barrier / LDS-commit phase overlaps the other's MFMAs).
// Measured equal at batch 512 (37.96k vs 38.01k img/s), so the default is the simpler 0.
static int g_stem_cfg = [] {
  const char* e = getenv("MPA_STEM_CFG");
  return e ? atoi(e) : 0;
}();

template <int NW, int ROWS, int OCC>
static int launch_stem(IGemmArgs a, int max_blocks, hipStream_t s) {
  StemPlan h{};
  h.items_img = (a.oH + ROWS - 1) / ROWS;
  const int nimg = a.M / (a.oH * a.oW);
  h.items = nimg * h.items_img;
  h.crows = (ROWS - 1) * a.Uh + STEM_R;
  h.qsub = (a.oW + 15) / 16;
  const int grid = std::max(1, std::min(h.items, max_blocks));
  hipLaunchKernelGGL((conv_stem_kernel<NW, ROWS, OCC>), dim3(grid), dim3(NW * 64), 0, s, a, h);
  return grid;
}

int conv_stem(IGemmArgs a, hipStream_t s) {
  // one statistics-slab row per block: the caller's slab holds >= slab_rows_max(M) rows
  if (g_stem_cfg == 1 && (a.M + 127) / 128 >= 512) return launch_stem<4, 4, 2>(a, 512, s);
  return launch_stem<8, 8, 1>(a, HALO_MAX_ROWS, s);
}

}  // namespace mpa
