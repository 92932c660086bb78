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

constexpr int SP_MAXQ = 112;  // PF: output width the z image holds

// PF pooling of one item (output rows p0 .. p0 + 7 of image img) from its LDS z image:
// thread = (pooled pixel, 8-channel chunk).  Window (pp, qq) covers output rows 2 pp - 1 ..
// 2 pp + 1 and columns 2 qq - 1 .. 2 qq + 1 (tap 3 i + k); taps are scanned in order with a
// strict comparison, so the first extreme wins, as in bn_relu_maxpool_fwd_kernel.  gamma < 0
// channels take the minimum (relu(bn(z)) decreases in z there).
__device__ __forceinline__ void stem_pool_item(const IGemmArgs& p, const StemPlan& h,
                                               const char* zimg, int img, int p0) {
  const int Q = p.oW, PQ = Q >> 1, PP = p.oH >> 1;
  const int pp0 = p0 >> 1, item = p0 >> 3, nthr = blockDim.x;
  auto chunk = [&](int r, int q, int c8) -> uint4 {
    const u32x4 v = *LDS_PTR(const u32x4, zimg + (r * SP_MAXQ + q) * 128 + ((c8 ^ (q & 7)) << 4));
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  // main records: pooled rows pp0 .. pp0 + 3, window rows inside the item
  for (int u = threadIdx.x; u < 4 * PQ * 8; u += nthr) {
    const int c8 = u & 7, t = u >> 3, qq = t % PQ, pr = t / PQ;
    float sg[8], best[8], bz[8];
    int bt[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sg[j] = p.sp_gamma[c8 * 8 + j] < 0.f ? -1.f : 1.f;
      best[j] = -INFINITY;
      bz[j] = 0.f;
      bt[j] = 0;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int r = 2 * pr - 1 + i;  // (>= -1, <= 7)
      if (r < 0) continue;            // the previous item's bottom row (stem_pool_apply)
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = 2 * qq - 1 + k;
        if (q < 0) continue;          // left padding
        float f[8];
        const uint4 cv = chunk(r, q, c8);
        unpack8(cv, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = sg[j] * f[j];
          if (v > best[j]) { best[j] = v; bz[j] = f[j]; bt[j] = 3 * i + k; }
        }
      }
    }
    const size_t o = (((size_t)img * PP + pp0 + pr) * PQ + qq) * 64 + c8 * 8;
    *(uint4*)((bf16_t*)p.sp_zsel + o) = pack8(bz);  // bf16 -> f32 -> bf16: exact
    uint2 ib;
    ib.x = (uint32_t)bt[0] | ((uint32_t)bt[1] << 8) | ((uint32_t)bt[2] << 16) | ((uint32_t)bt[3] << 24);
    ib.y = (uint32_t)bt[4] | ((uint32_t)bt[5] << 8) | ((uint32_t)bt[6] << 16) | ((uint32_t)bt[7] << 24);
    *(uint2*)(p.sp_idx + o) = ib;
  }
  // bottom record: output row p0 + 7 is window row 0 (taps 0..2) of the next item's first
  // pooled row pp0 + 4
  if (item + 1 < h.items_img) {
    for (int u = threadIdx.x; u < PQ * 8; u += nthr) {
      const int c8 = u & 7, qq = u >> 3;
      float sg[8], best[8], bz[8];
      int bt[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sg[j] = p.sp_gamma[c8 * 8 + j] < 0.f ? -1.f : 1.f;
        best[j] = -INFINITY;
        bz[j] = 0.f;
        bt[j] = 0;
      }
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const int q = 2 * qq - 1 + k;
        if (q < 0) continue;
        float f[8];
        const uint4 cv = chunk(7, q, c8);
        unpack8(cv, f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = sg[j] * f[j];
          if (v > best[j]) { best[j] = v; bz[j] = f[j]; bt[j] = k; }
        }
      }
      const size_t o = (((size_t)img * h.items_img + item + 1) * PQ + qq) * 64 + c8 * 8;
      *(uint4*)((bf16_t*)p.sp_bz + o) = pack8(bz);
      uint2 ib;
      ib.x = (uint32_t)bt[0] | ((uint32_t)bt[1] << 8) | ((uint32_t)bt[2] << 16) | ((uint32_t)bt[3] << 24);
      ib.y = (uint32_t)bt[4] | ((uint32_t)bt[5] << 8) | ((uint32_t)bt[6] << 16) | ((uint32_t)bt[7] << 24);
      *(uint2*)(p.sp_bidx + o) = ib;
    }
  }
}

// STEM_NW waves per block, STEM_ROWS output rows per item, STEM_OCC waves per SIMD.
// PF (round 6): the stem max-pool fused in (IGemmArgs::sp_zsel).  Every subtile's bf16 z also
// goes to an LDS image of the item's 8 x Q outputs (16-B chunks swizzled by pixel), and
// after the item's MFMAs the block takes each pooled window's extreme from it: the
// separate pool pass no longer reads z back from memory.
template <int STEM_NW, int STEM_ROWS, int STEM_OCC, bool PF = false>
__global__ __launch_bounds__(STEM_NW * 64, STEM_OCC) void conv_stem_kernel(IGemmArgs p,
                                                                           StemPlan h) {
  constexpr int STEM_MAX_CROWS = (STEM_ROWS - 1) * 2 + STEM_R;  // canvas rows, sh <= 2
  constexpr int STEM_LDS = STEM_MAX_CROWS * STEM_MAX_WP * 16;
  constexpr int STEM_PREF = (STEM_LDS / 16 + STEM_NW * 64 - 1) / (STEM_NW * 64);  // vec/thread
  __shared__ __attribute__((aligned(16))) char canvas[STEM_LDS];
  __shared__ float red[STEM_NW][2][64];
  __shared__ __attribute__((aligned(16))) char zimg[PF ? STEM_ROWS * SP_MAXQ * 128 : 16];
  static_assert(!PF || STEM_ROWS == 8, "fused pool: 8-row items (4 pooled rows)");
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
          if constexpr (PF) {  // channels 16 nb + 4 kc .. +3: half of 16-B chunk 2 nb + kc / 2
            const int q = q0 + li, ch = 2 * nb + (kc >> 1);
            *LDS_PTR(u32x2, zimg + (pr * SP_MAXQ + q) * 128 + ((ch ^ (q & 7)) << 4) +
                                ((kc & 1) << 3)) = u32x2{lo, hi};
          }
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
    // (PF: after the commit, whose prefetch registers are then dead; the z image is not
    // rewritten before the next item's MFMAs, behind the barrier below)
    if constexpr (PF) stem_pool_item(p, h, zimg, img, p0);
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
  if (a.sp_zsel &&  // fused pool: whole 8-row items, an even width the z image holds
      (a.oH % 8 != 0 || a.oW % 2 != 0 || a.oW > SP_MAXQ || !a.sp_idx || !a.sp_bz ||
       !a.sp_bidx || !a.sp_gamma || a.relu || a.bias ||
       ((reinterpret_cast<uintptr_t>(a.sp_zsel) | reinterpret_cast<uintptr_t>(a.sp_bz)) & 15) ||
       ((reinterpret_cast<uintptr_t>(a.sp_idx) | reinterpret_cast<uintptr_t>(a.sp_bidx)) & 7)))
    return false;
  for (int t = 0; t < STEM_R; ++t)  // one super-tap per kernel row: dh = t, dw = 0, 4 columns
    if (a.taps.dh[t] != t || a.taps.dw[t] != 0 || a.taps.bt[t] != ((t * 4) | (4 << 12)))
      return false;
  return true;
}

// block shape: 8 waves x 8-row items, one block per CU (4 waves x 4-row items, two blocks
// per CU, measured equal at batch 512 - 37.96k vs 38.01k img/s - and was removed)

template <int NW, int ROWS, int OCC, bool PF = false>
static int launch_stem(IGemmArgs a, int max_blocks, hipStream_t s) {
  StemPlan h{};
  h.items_img = (a.oH + ROWS - 1) / ROWS;
  const int nimg = a.M / (a.oH * a.oW);
  h.items = nimg * h.items_img;
  h.crows = (ROWS - 1) * a.Uh + STEM_R;
  h.qsub = (a.oW + 15) / 16;
  const int grid = std::max(1, std::min(h.items, max_blocks));
  hipLaunchKernelGGL((conv_stem_kernel<NW, ROWS, OCC, PF>), dim3(grid), dim3(NW * 64), 0, s, a, h);
  return grid;
}

int conv_stem(IGemmArgs a, hipStream_t s) {
  // one statistics-slab row per block: the caller's slab holds >= slab_rows_max(M) rows
  // (PF: 4-wave blocks, one wave per SIMD with 512 registers: the 112 weight registers held
  // for the kernel's life plus the pooling pass spill at the 256 of an 8-wave block)
  if (a.sp_zsel) return launch_stem<4, 8, 1, true>(a, std::min(HALO_MAX_ROWS, active_cus()), s);
  return launch_stem<8, 8, 1>(a, std::min(HALO_MAX_ROWS, active_cus()), s);
}

// stem_pool_apply: thread = (pooled pixel, 8-channel chunk); the BN affine as
// bn_relu_maxpool_fwd_kernel computes it (rsqrt of the batch variance, fma shift)
__global__ __launch_bounds__(256) void stem_pool_apply_kernel(
    IGemmArgs p, int items_img, const float* __restrict__ stats, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, bf16_t* __restrict__ y, float* __restrict__ mean_out,
    float* __restrict__ rstd_out, unsigned long long* __restrict__ counter) {
  const int C = 64, PQ = p.oW >> 1, PP = p.oH >> 1;
  const int nimg = p.M / (p.oH * p.oW);
  const int64_t rows = (int64_t)nimg * PP * PQ;
  if (blockIdx.x == 0 && threadIdx.x < C) {
    const int c = threadIdx.x;
    const float mu = stats[c], var = stats[C + c];
    const int64_t M = p.M;
    mean_out[c] = mu;
    rstd_out[c] = rsqrtf(var + eps);
    const float unb = var * ((float)M / (float)(M > 1 ? M - 1 : 1));
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * mu;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * unb;
    if (counter && c == 0) atomicAdd(counter, 1ull);
  }
  const int c8 = threadIdx.x & 7;
  float sc[8], sh[8], sg[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c8 * 8 + j;
    const float rs = rsqrtf(stats[C + c] + eps);
    sc[j] = gamma[c] * rs;
    sh[j] = __builtin_fmaf(-stats[c], sc[j], beta[c]);
    sg[j] = gamma[c] < 0.f ? -1.f : 1.f;
  }
  bf16_t* const zsel = (bf16_t*)p.sp_zsel;
  for (int64_t r = (int64_t)blockIdx.x * 32 + (threadIdx.x >> 3); r < rows;
       r += (int64_t)gridDim.x * 32) {
    const int qq = (int)(r % PQ);
    const int64_t t = r / PQ;
    const int pp = (int)(t % PP), img = (int)(t / PP);
    const size_t o = (size_t)r * C + c8 * 8;
    float z[8];
    unpack8(*(const uint4*)(zsel + o), z);
    if ((pp & 3) == 0 && pp > 0) {  // merge the previous item's bottom row (taps 0..2 first)
      const size_t ob = (((size_t)img * items_img + (pp >> 2)) * PQ + qq) * C + c8 * 8;
      float zb[8];
      unpack8(*(const uint4*)((const bf16_t*)p.sp_bz + ob), zb);
      const uint2 ib = *(const uint2*)(p.sp_bidx + ob);
      uint2 im = *(const uint2*)(p.sp_idx + o);
      uint32_t w[2] = {im.x, im.y};
      const uint32_t wb[2] = {ib.x, ib.y};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (sg[j] * zb[j] >= sg[j] * z[j]) {  // (a tie keeps the earlier tap: the bottom row)
          z[j] = zb[j];
          const int sft = 8 * (j & 3);
          w[j >> 2] = (w[j >> 2] & ~(0xffu << sft)) | (((wb[j >> 2] >> sft) & 0xffu) << sft);
        }
      }
      *(uint4*)(zsel + o) = pack8(z);
      *(uint2*)(p.sp_idx + o) = make_uint2(w[0], w[1]);
    }
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(z[j] * sc[j] + sh[j], 0.f);
    *(uint4*)(y + o) = pack8(v);
    // ReLU-dead windows: argmax byte 255, as bn_relu_maxpool_fwd writes it
    uint32_t dead[2] = {0u, 0u};
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (!(v[j] > 0.f)) dead[j >> 2] |= 0xffu << (8 * (j & 3));
    if (dead[0] | dead[1]) {
      const uint2 im = *(const uint2*)(p.sp_idx + o);
      *(uint2*)(p.sp_idx + o) = make_uint2(im.x | dead[0], im.y | dead[1]);
    }
  }
}

void stem_pool_apply(const IGemmArgs& a, const float* stats, const float* gamma,
                     const float* beta, float* rmean, float* rvar, float momentum, float eps,
                     bf16_raw* y, float* mean, float* rstd, int64_t* counter, hipStream_t s) {
  const int items_img = a.oH / 8;
  const int64_t rows = (int64_t)(a.M / (a.oH * a.oW)) * (a.oH / 2) * (a.oW / 2);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((rows + 31) / 32, 4096));
  hipLaunchKernelGGL(stem_pool_apply_kernel, dim3(grid), dim3(256), 0, s, a, items_img, stats,
                     gamma, beta, rmean, rvar, momentum, eps, (bf16_t*)y, mean, rstd,
                     (unsigned long long*)counter);
}

// ======================================================================================
//  Stem weight gradient, halo-staged (pixel-pair layout of the forward above):
//    dW[k][r][s][c] += sum_pix dz[pix][k] * canvas[n][2 oh + r][ow + s][c]
//  k < 64 output channels; (r < 7, s < 4 pair columns, c < 8) = 224 columns; the reduction
//  runs over every output pixel (6.4 M at batch 512).  As an implicit GEMM (igemm_wgrad_dma_
//  inc_kernel) every 16-B canvas vector was gathered once per (r, s) tap it feeds - 14x -
//  and the kernel waited on those gathers 57 % of its wave time.  Here a block owns the
//  whole 64 x 224 output and streams items of 2 output rows of one image:
//    * the item's dz rows (2 Q pixels x 128 B, contiguous) and its 9 canvas rows (contiguous:
//      the 7 x 4 windows of every output pixel of the item) are staged ONCE per item,
//      register-staged: the next item's 16-B loads are issued at the top of the current
//      item and written to the other LDS stage after its MFMAs (LDS-DMA pieces cost the
//      issuing wave 60-180 cycles each; as DMAs the 45 per item were 37 % of the kernel);
//    * both operands are pixel-major and read with ds_read_b64_tr_b16: dz through the
//      engine's mn_off<64> image, the canvas straight from its rows - a lane's 8-B granule
//      of column fragment j (tap row r = j/2, pair columns 2 (j%2) + {0,1}) for pixel
//      (row, ow) sits at ((2 row + r) Wc + ow + s) * 16 + 8 * (channel half): a per-lane
//      base plus a wave-uniform tap offset;
//    * the KS K-steps of an item are unrolled at compile time and software-pipelined (the
//      next K-step's fragments are read under this one's MFMAs);
//    * wave w accumulates all 64 k x column fragments {w, w+4, w+8, w+12} (< 14) in
//      registers for the block's whole life; one [64][224] fp32 partial per block goes to
//      the slab that wgrad_reduce adds into the gradient arena.
// ======================================================================================
namespace {
constexpr int SW_KS = 8;                             // <= 8 K-steps: 2 Q <= 256 pixels
constexpr int SW_DZ = SW_KS * 4096;                  // [K-step][32 px][64 k] bf16, mn_off<64>
constexpr int SW_CROWS = 9;                          // canvas rows per item: 2 (2-1) + 7
constexpr int SW_CVV = SW_CROWS * STEM_MAX_WP;       // canvas 16-B vectors per item (<= 1080)
constexpr int SW_CVPT = (SW_CVV + 255) / 256;        // canvas vectors per thread (5)
constexpr int SW_STAGE = SW_DZ + SW_CVV * 16;
constexpr int SW_LDS = 2 * SW_STAGE;                 // 100,096 B
}  // namespace

struct StemWPlan {
  int items, items_img;  // items = N * ceil(P / 2)
  int ks;                // K-steps per item: ceil(2 Q / 32) (= the kernel's KS)
};

// one item's MFMAs: all KS K-steps of (dz stage sdz, canvas scv), software-pipelined (the
// next K-step's fragments are read under this one's MFMAs).  Waves 2 and 3 own three column
// fragments; their fourth (a duplicate of fragment 13) keeps the MFMA stream branch-free -
// those waves would idle at the item barrier anyway - and is never stored.
// (BBQ: the B granule offsets are recomputed per K-step from Q instead of held in 2 KS
// registers - the pooled form's MFMA waves also carry a dz unit)
template <int KS, bool BBQ = false>
__device__ __forceinline__ void stem_wgrad_item(const char* sdz, const char* scv,
                                                const int (&bb)[KS][2], int Wc, int wave,
                                                int lane, f32x4 (&acc)[4][4], int Q = 0) {
  auto load_frags = [&](int ks, bf16x8(&af)[4], bf16x8(&bf)[4]) {
#pragma unroll
    for (int km = 0; km < 4; ++km) af[km] = frag_mn<64>(sdz + ks * 4096, 16 * km, lane);
    int b0, b1;
    if constexpr (BBQ) {
      const int g = lane >> 4, li = lane & 15, qd = li >> 2, pp = li & 3;
      int bo[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int pl = min(32 * ks + 8 * g + qd + 4 * e, 2 * Q - 1);
        const int prow = pl >= Q ? 1 : 0;
        bo[e] = ((2 * prow) * Wc + pl - prow * Q + (pp >> 1)) * 16 + (pp & 1) * 8;
      }
      b0 = bo[0];
      b1 = bo[1];
    } else {
      b0 = bb[ks][0];
      b1 = bb[ks][1];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = min(wave + 4 * i, 13);
      const int toff = ((j >> 1) * Wc + 2 * (j & 1)) * 16;  // tap row r, pair column s0
      const s16x4 lo =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, scv + b0 + toff));
      const s16x4 hi =
          __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, scv + b1 + toff));
      s16x8 r;
      r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
      r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
      bf[i] = __builtin_bit_cast(bf16x8, r);
    }
  };
  bf16x8 af[2][4], bf[2][4];
  load_frags(0, af[0], bf[0]);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    if (ks + 1 < KS) load_frags(ks + 1, af[(ks + 1) & 1], bf[(ks + 1) & 1]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int km = 0; km < 4; ++km)
        acc[km][i] = mfma16(bf[ks & 1][i], af[ks & 1][km], acc[km][i]);
  }
}

// a block's partial -> its slab row: dw[k][col], k = 16 km + lane % 16,
// col = 16 j + 4 (lane / 16) .. +3
__device__ __forceinline__ void stem_wgrad_store(float* dst, const f32x4 (&acc)[4][4], int nfr,
                                                 int wave, int li, int g) {
#pragma unroll
  for (int km = 0; km < 4; ++km)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nfr) break;
      const int j = wave + 4 * i;
      *(f32x4*)(dst + (16 * km + li) * 224 + 16 * j + 4 * g) = acc[km][i];
    }
}

// per-lane canvas byte offsets of the B granules (item independent): K-step ks, half e ->
// item pixel pl = 32 ks + 8 g + qd + 4 e -> (row, ow); pixels past 2 Q are clamped (their
// dz rows are zero)
template <int KS>
__device__ __forceinline__ void stem_wgrad_boffs(int (&bb)[KS][2], int Q, int Wc, int lane) {
  const int g = lane >> 4, li = lane & 15, qd = li >> 2, pp = li & 3;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int pl = min(32 * ks + 8 * g + qd + 4 * e, 2 * Q - 1);
      const int prow = pl >= Q ? 1 : 0;
      const int ow = pl - prow * Q;
      bb[ks][e] = ((2 * prow) * Wc + ow + (pp >> 1)) * 16 + (pp & 1) * 8;
    }
}

// XCD-contiguous item order for the persistent stem kernels: block b (XCD b % 8) starts at
// item (b % 8) * G / 8 + b / 8 and strides G, so at any step the G / 8 blocks of one XCD work
// on consecutive items (neighbouring row pairs / row groups of one image), whose shared
// canvas rows then hit that XCD's L2.  (G % 8 != 0: the plain order.)
__device__ __forceinline__ int stem_first_item(int G) {
  const int b = blockIdx.x;
  return (G & 7) ? b : (b & 7) * (G >> 3) + (b >> 3);
}

template <int KS>
__global__ __launch_bounds__(256, 1) void stem_wgrad_kernel(WGradArgs p, StemWPlan h) {
  __shared__ __attribute__((aligned(16))) char smem[SW_LDS];
  constexpr int CVPT = SW_CVPT;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int P = p.P, Q = p.Q, Hc = p.H, Wc = p.W;
  const int g = lane >> 4, li = lane & 15;
  const int nfr = wave < 2 ? 4 : 3;  // column fragments j = wave + 4 i < 14
  int bb[KS][2];
  stem_wgrad_boffs<KS>(bb, Q, Wc, lane);
  // this thread's staging slots: dz vector tid + 256 i (row = v >> 3, chunk = v & 7) and
  // canvas vector tid + 256 i
  int dzoff[KS];
#pragma unroll
  for (int i = 0; i < KS; ++i) {
    const int v = tid + 256 * i, row = v >> 3, chunk = v & 7;
    dzoff[i] = (row >> 5) * 4096 + mn_off<64>(row & 31, chunk * 8);
  }
  const u32x4* const dzsrc = (const u32x4*)p.dy;   // [pix][8 vectors]
  const u32x4* const cvsrc = (const u32x4*)p.x;    // [n][Hc][Wc] pair vectors
  u32x4 pdz[KS], pcv[CVPT];
  auto fetch = [&](int it) {  // item it's vectors into registers (zeros past its end)
    const int n = it / h.items_img, oh0 = (it - n * h.items_img) * 2;
    const size_t cv0 = ((size_t)n * Hc + 2 * oh0) * Wc;
    const int cvlim = min(SW_CROWS, Hc - 2 * oh0) * Wc;
    const int pix0 = (n * P + oh0) * Q, nval = min(2, P - oh0) * Q;
#pragma unroll
    for (int i = 0; i < KS; ++i) {
      const int v = tid + 256 * i;
      pdz[i] = (v >> 3) < nval ? dzsrc[(size_t)(pix0 + (v >> 3)) * 8 + (v & 7)]
                               : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < CVPT; ++i) {
      const int v = tid + 256 * i;
      pcv[i] = v < cvlim ? cvsrc[cv0 + v] : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto commit = [&](int stage) {
    char* st = smem + stage * SW_STAGE;
#pragma unroll
    for (int i = 0; i < KS; ++i) *LDS_PTR(u32x4, st + dzoff[i]) = pdz[i];
#pragma unroll
    for (int i = 0; i < CVPT; ++i) {
      const int v = tid + 256 * i;
      if (v < SW_CVV) *LDS_PTR(u32x4, st + SW_DZ + v * 16) = pcv[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int km = 0; km < 4; ++km)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[km][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int G = gridDim.x;
  int it = stem_first_item(G);
  if (it < h.items) {
    fetch(it);
    commit(0);
  }
  for (int k = 0; it < h.items; ++k, it += G) {
    const int st = k & 1;
    __syncthreads();  // item k's stage written; every wave is done with item k-1's stage
    const bool more = it + G < h.items;
    if (more) fetch(it + G);  // lands under this item's MFMAs
    const char* sdz = smem + st * SW_STAGE;
    stem_wgrad_item<KS>(sdz, sdz + SW_DZ, bb, Wc, wave, lane, acc);
    if (more) commit(st ^ 1);
  }
  stem_wgrad_store(p.slab + (size_t)blockIdx.x * 64 * 224, acc, nfr, wave, li, g);
}

// ---------------------------------------------------------------------------------------
// POOL form (round 6): the stem's BN + ReLU + 3x3/s2/p1 max-pool backward runs INSIDE the
// weight gradient's staging, so the full-resolution dz is never written or read back.
// An item (output rows 2t, 2t+1) is exactly one row of 2x2 cells; cell (t, c) is covered
// by the pooled windows (t | t+1, c | c+1).  Per (cell, 8 channels) unit a thread gathers
// the 4 windows' pooled gradient dp and argmax taps plus the cell's 4 z vectors (issued one
// item ahead), then writes
//   dz = a g + b + cco z,  g = sum of dp over windows whose argmax is this pixel
//        (a = gamma rstd, b / cco from the pooled sums (sum g, sum g xhat))
// to the dz stage - the arithmetic of maxpool_bn_bwd_cell_kernel<true> (bn.hip), so the
// staged operand is the one the two-pass form wrote to memory.  The ReLU mask bn(z) > 0 of
// that form is implied: the forward gives a ReLU-dead window the argmax byte 255, and a
// live window's argmax pixel is live, so g is already zero wherever the mask would be.  Reference: the stem
// conv1 -> bn1 -> relu -> maxpool of torchvision resnet / densenet (models.py:24-30, 74-80).
// (StemPoolArgs: api.h)
//
// 8-wave blocks.  The dz formation (~500 VALU per unit) bounds the kernel, and one wave
// alone issues a VALU instruction only every ~4 cycles (MI355X_MICROARCH.md), so it is
// split over BOTH wave sets: waves 4..7 (producers) form units 0..255 and stage the canvas,
// waves 0..3 form units 256.. (4 Q units per item) right after their item's MFMAs - their
// gathers are issued before those MFMAs and land under them.  The two waves of a SIMD then
// interleave their VALU streams in the issue slots the MFMAs leave.  (Producers forming all
// 4 Q units: 0.88-0.93 ms per b1024 step; with the gathers and z LDS-DMAed into a 3-stage
// ring instead: no faster, profiles/stem_pool_r6.txt.)
template <int KS>
__global__ __launch_bounds__(512, 1) void stem_pool_wgrad_kernel(WGradArgs p, StemWPlan h,
                                                                  StemPoolArgs pa) {
  __shared__ __attribute__((aligned(16))) char smem[SW_LDS + 1024];
  constexpr int CVPT = SW_CVPT;
  const int lane = threadIdx.x & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P = p.P, Q = p.Q, Hc = p.H, Wc = p.W;
  const bool prod = wave_all >= 4;
  // this thread's unit: producers 0..255, MFMA waves 256..511 (valid below 4 Q)
  const int u = prod ? (int)threadIdx.x - 256 : (int)threadIdx.x + 256;
  const bool uok = u < 4 * Q;
  const int cq = uok ? (u >> 3) : 0;
  const int pch = (threadIdx.x & 7) * 8;
  // per-channel BN-backward constants (bn_coeffs + maxpool_bn_bwd_cell_kernel<true>) as
  // an LDS table [scale, shift, b, cco][64], read per unit (as registers: 32 per thread)
  float* tab = (float*)(smem + SW_LDS);
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    const float mu = pa.mean[c], rs = pa.rstd[c];
    const float sc = pa.gamma[c] * rs;
    const float cc = -sc * rs * pa.sums[64 + c] * pa.invM;
    tab[c] = sc;
    tab[64 + c] = pa.beta[c] - mu * sc;
    tab[128 + c] = -sc * pa.sums[c] * pa.invM - cc * mu;
    tab[192 + c] = cc;
  }
  {  // K-step rows past 2 Q are never staged: zero them once in both stages
    const int r0 = 2 * Q;
    const int zb = (r0 >> 5) * 4096 + (r0 & 31) * 128, ze = KS * 4096;
    for (int s2 = 0; s2 < 2; ++s2)
      for (int b = zb + (int)threadIdx.x * 16; b < ze; b += 512 * 16)
        *LDS_PTR(u32x4, smem + s2 * SW_STAGE + b) = u32x4{0u, 0u, 0u, 0u};
  }
  const u32x4* const zsrc = (const u32x4*)p.dy;    // z: [pix][8 vectors]
  const u32x4* const cvsrc = (const u32x4*)p.x;    // [n][Hc][Wc] pair vectors
  // the unit's 4 windows (out-of-range ones load a clamped window, masked at commit) and
  // its cell's 4 z vectors, for item it
  struct Unit {
    u32x4 dp[4], z[4];
    u32x2 ix[4];
  };
  auto fetch_unit = [&](int it, Unit& q) {
    const int n = it / h.items_img, t = it - n * h.items_img, oh0 = 2 * t;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int wp = min(t + (w >> 1), pa.PP - 1), wq = min(cq + (w & 1), pa.PQ - 1);
      const size_t o = (((size_t)n * pa.PP + wp) * pa.PQ + wq) * 64 + pch;
      q.dp[w] = *(const u32x4*)(pa.dp + o);
      q.ix[w] = *(const u32x2*)(pa.idx + o);
    }
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4)
      q.z[w4] = zsrc[((size_t)(n * P + oh0 + (w4 >> 1)) * Q + 2 * cq + (w4 & 1)) * 8 +
                    (pch >> 3)];
  };
  auto commit_unit = [&](int stage, int it, const Unit& q) {
    if (!uok) return;
    char* st = smem + stage * SW_STAGE;
    const int t = it - (it / h.items_img) * h.items_img;  // cell row = oh0 / 2
    f32x4 bsc[2], bb0[2], bcc[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      bsc[h2] = *LDS_PTR(const f32x4, tab + pch + 4 * h2);
      bb0[h2] = *LDS_PTR(const f32x4, tab + 128 + pch + 4 * h2);
      bcc[h2] = *LDS_PTR(const f32x4, tab + 192 + pch + 4 * h2);
    }
    uint2 iv[4];
    float d[4][8];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const bool ok = t + (w >> 1) < pa.PP && cq + (w & 1) < pa.PQ;
      iv[w] = ok ? make_uint2(q.ix[w][0], q.ix[w][1]) : make_uint2(~0u, ~0u);
      unpack8(make_uint4(q.dp[w][0], q.dp[w][1], q.dp[w][2], q.dp[w][3]), d[w]);
    }
#pragma unroll
    for (int w4 = 0; w4 < 4; ++w4) {
      const int a0 = w4 >> 1, b0 = w4 & 1;  // pixel (2t + a0, 2 cq + b0)
      float zr[8];
      unpack8(make_uint4(q.z[w4][0], q.z[w4][1], q.z[w4][2], q.z[w4][3]), zr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int du = w >> 1, eu = w & 1;
          // rows {t: tap 1 + a0} (+ {t + 1: tap 0} if a0), columns likewise
          if ((du && !a0) || (eu && !b0)) continue;
          const int ti = du ? 0 : 1 + a0, tk = eu ? 0 : 1 + b0;
          const uint32_t word = j < 4 ? iv[w].x : iv[w].y;
          if ((int)((word >> (8 * (j & 3))) & 0xff) == ti * 3 + tk) acc += d[w][j];
        }
        // (no ReLU mask: a dead window's argmax byte is 255 and matched no tap above)
        zr[j] = bsc[j >> 2][j & 3] * acc + bb0[j >> 2][j & 3] + bcc[j >> 2][j & 3] * zr[j];
      }
      const int pl = a0 * Q + 2 * cq + b0;
      const uint4 o = pack8(zr);
      *LDS_PTR(u32x4, st + (pl >> 5) * 4096 + mn_off<64>(pl & 31, pch)) =
          u32x4{o.x, o.y, o.z, o.w};
    }
  };

  const int G = gridDim.x;
  int it = stem_first_item(G);
  if (prod) {  // ------------------------------------------------------------- producers
    // (item k + 2's loads issued before forming item k + 1, two register sets: 1.00 ms vs
    // 0.89 ms - the spills cost more than the latency it hides)
    const int tid = (int)threadIdx.x - 256;
    u32x4 pcv[CVPT];
    auto fetch_canvas = [&](int it) {
      const int n = it / h.items_img, oh0 = (it - n * h.items_img) * 2;
      const size_t cv0 = ((size_t)n * Hc + 2 * oh0) * Wc;
      const int cvlim = min(SW_CROWS, Hc - 2 * oh0) * Wc;
#pragma unroll
      for (int i = 0; i < CVPT; ++i) {
        const int v = tid + 256 * i;
        pcv[i] = v < cvlim ? cvsrc[cv0 + v] : u32x4{0u, 0u, 0u, 0u};
      }
    };
    auto commit_canvas = [&](int stage) {
      char* st = smem + stage * SW_STAGE;
#pragma unroll
      for (int i = 0; i < CVPT; ++i) {
        const int v = tid + 256 * i;
        if (v < SW_CVV) *LDS_PTR(u32x4, st + SW_DZ + v * 16) = pcv[i];
      }
    };
    Unit qp;
    if (it < h.items) {
      fetch_unit(it, qp);
      fetch_canvas(it);
      commit_unit(0, it, qp);
      commit_canvas(0);
    }
    for (int k = 0; it < h.items; ++k, it += G) {
      __syncthreads();  // item k's stage published; item k - 1's stage free
      if (it + G < h.items) {
        fetch_unit(it + G, qp);
        fetch_canvas(it + G);
        commit_unit((k + 1) & 1, it + G, qp);
        commit_canvas((k + 1) & 1);
      }
    }
    return;
  }
  // ---------------------------------------------------------------------------- MFMA waves
  const int wave = wave_all;
  const int g = lane >> 4, li = lane & 15;
  const int nfr = wave < 2 ? 4 : 3;
  const int bb[KS][2] = {};  // (unused: BBQ)
  f32x4 acc[4][4];
#pragma unroll
  for (int km = 0; km < 4; ++km)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[km][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  Unit qm;
  if (it < h.items) {
    fetch_unit(it, qm);
    commit_unit(0, it, qm);
  }
  for (int k = 0; it < h.items; ++k, it += G) {
    const int st = k & 1;
    __syncthreads();  // item k's stage written; every wave is done with item k-1's stage
    const bool more = it + G < h.items;
    if (more) fetch_unit(it + G, qm);  // lands under this item's MFMAs
    const char* sdz = smem + st * SW_STAGE;
    stem_wgrad_item<KS, true>(sdz, sdz + SW_DZ, bb, Wc, wave, lane, acc, Q);
    if (more) commit_unit(st ^ 1, it + G, qm);
  }
  stem_wgrad_store(p.slab + (size_t)blockIdx.x * 64 * 224, acc, nfr, wave, li, g);
}

bool stem_wgrad_ok(const WGradArgs& a) {
  if (!g_stem_on || a.R != STEM_R || a.S != 4 || a.C != 8 || a.sh != 2 || a.sw != 1 || a.ph != 0 ||
      a.pw != 0 || a.Kout != 64 || a.Ncols != 224 || a.slab == nullptr)
    return false;
  if (a.P != (a.H - STEM_R) / 2 + 1 || a.Q != a.W - 3 || a.Q < 16 || 2 * a.Q > 32 * SW_KS ||
      a.W > STEM_MAX_WP || a.Mpix % (a.P * a.Q) != 0)
    return false;
  return ((reinterpret_cast<uintptr_t>(a.dy) | reinterpret_cast<uintptr_t>(a.x) |
           reinterpret_cast<uintptr_t>(a.slab)) & 15) == 0;
}

int64_t stem_wgrad_ws_floats() { return (int64_t)HALO_MAX_ROWS * 64 * 224; }

// partials into a.slab ([Z][64][224]); returns Z
int stem_wgrad(WGradArgs a, hipStream_t s) {
  StemWPlan h{};
  const int nimg = a.Mpix / (a.P * a.Q);
  h.items_img = (a.P + 1) / 2;
  h.items = nimg * h.items_img;
  h.ks = (2 * a.Q + 31) / 32;
  const int grid = std::max(1, std::min(h.items, std::min(HALO_MAX_ROWS, active_cus())));
  switch (h.ks) {
#define SW_CASE(K)                                                                 \
  case K:                                                                          \
    hipLaunchKernelGGL((stem_wgrad_kernel<K>), dim3(grid), dim3(256), 0, s, a, h); \
    break;
    SW_CASE(1) SW_CASE(2) SW_CASE(3) SW_CASE(4) SW_CASE(5) SW_CASE(6) SW_CASE(7) SW_CASE(8)
#undef SW_CASE
  }
  return grid;
}

bool stem_pool_wgrad_ok(const WGradArgs& a, const StemPoolArgs& q) {
  // 3x3 / s2 / p1 pool over an even conv output: every item is one full row of 2x2 cells
  return stem_wgrad_ok(a) && a.P % 2 == 0 && a.Q % 2 == 0 && q.PP * 2 == a.P &&
         q.PQ * 2 == a.Q && q.dp && q.idx && q.mean && q.rstd && q.gamma && q.beta && q.sums &&
         ((reinterpret_cast<uintptr_t>(q.dp) | reinterpret_cast<uintptr_t>(q.idx)) & 15) == 0;
}

int stem_pool_wgrad(WGradArgs a, StemPoolArgs q, hipStream_t s) {
  StemWPlan h{};
  const int nimg = a.Mpix / (a.P * a.Q);
  h.items_img = a.P / 2;
  h.items = nimg * h.items_img;
  h.ks = (2 * a.Q + 31) / 32;
  q.invM = 1.f / (float)a.Mpix;
  const int grid = std::max(1, std::min(h.items, std::min(HALO_MAX_ROWS, active_cus())));
  switch (h.ks) {
#define SW_CASE(K)                                                                       \
  case K:                                                                                \
    hipLaunchKernelGGL((stem_pool_wgrad_kernel<K>), dim3(grid), dim3(512), 0, s, a, h, q); \
    break;
    SW_CASE(1) SW_CASE(2) SW_CASE(3) SW_CASE(4) SW_CASE(5) SW_CASE(6) SW_CASE(7) SW_CASE(8)
#undef SW_CASE
  }
  return grid;
}

}  // namespace mpa
