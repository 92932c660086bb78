// Host-side launcher API of the gfx950 kernel library.  Plain pointers + POD argument
// structs, no torch headers: the .hip translation units compile in seconds and the
// torch-facing binding layer (csrc/bindings.cpp) validates shapes and allocates.
#pragma once
#include <algorithm>
#include <string>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mpa {

typedef uint16_t bf16_raw;
constexpr int MAXT = 128;  // max taps in one implicit-GEMM launch (11x11 = 121)

struct Taps {
  short dh[MAXT];
  short dw[MAXT];
  short bt[MAXT];
};

// One stride phase of a merged dgrad launch: its output sub-grid (oH x oW pixels at
// rows/cols Poh + Uoh*i, Pow + Uow*j of dx), its taps [tap0, tap0 + T) of the shared table,
// and its tile count.  Tile g of the launch belongs to phase g % nphase (phases interleaved
// so every XCD's contiguous share of the tile list holds an equal mix of long and short
// phases), local tile g / nphase; phases are padded to the longest tile count.
// n / d for 0 <= n < 2^31 as one multiply-high and a shift (Granlund-Montgomery: m =
// ceil(2^(31 + l) / d), l = ceil(log2 d)); m == 0 encodes d == 1.  The rows kernels split
// a pixel index into (image, row, column) with these instead of two 32-bit integer divisions
// (~40 VALU each) per row in the prologue and again in the epilogue.
struct FastDiv {
  uint32_t m, s;
};
inline FastDiv make_fastdiv(uint32_t d) {
  if (d <= 1) return FastDiv{0u, 0u};
  const uint32_t l = 32u - (uint32_t)__builtin_clz(d - 1u);
  return FastDiv{(uint32_t)(((1ull << (31 + l)) + d - 1) / d), l - 1u};
}

constexpr int MAXPH = 16;
struct PhaseDesc {
  int M, oH, oW, Ktot, tap0, T, Poh, Pow, tiles;
  FastDiv fd_hw, fd_ow;  // oH * oW, oW (set by the launchers: igemm_set_fastdiv)
};

// implicit GEMM whose rows are pixels of a gathered NHWC tensor (conv fwd / dgrad / linear)
struct IGemmArgs {
  const bf16_raw* A;
  int aH, aW, aC;
  int oH, oW;
  int M;
  int Uh, Uw, Oh, Ow;
  int T;
  int Ktot;
  const bf16_raw* B;
  int N;
  int RS;
  int ldb;
  void* C;
  int ldc;
  int dH, dW, Uoh, Uow, Poh, Pow;
  const float* bias;
  float* stats;              // [2][N]: finalized (mean, biased var) of the bf16 output
  const float* stats_shift;  // per-column shift K for the sums (BN running mean) or null
  float* stats_sums;         // [2][N] final sums: zeroed by the epilogue's mt == 0 blocks
  int stats_ld;              // row stride of the finalized [2][N] statistics (0: N)
  int relu;
  int ktiles_per_split;
  int tiles_n;
  int tiles_total;
  Taps taps;
  int nphase;             // > 0: merged stride-phase dgrad launch (igemm_rows_dgrad_phases)
  PhaseDesc ph[MAXPH];
  int b_tapmap;           // K-contiguous B whose rows are indexed by weight tap: B element of
                          // GEMM k = (t, c) is B[n][taps.bt[t] * aC + c] (dgrad from the
                          // transposed weight [C][RS][K]); 0: B[n][k]
  // fused BN-backward reduction (dgrad epilogue, ep_bnred = 1): the GEMM output v is the
  // gradient dy of a ReLU(BN(z)) whose z / y / mean / rstd are given (same layout as C);
  // the epilogue writes g = dy * (y > 0) and slab-reduces (sum g, sum g * (z - mean) * rstd)
  // per column into `stats` exactly like the forward statistics (row `stat` of the slab)
  int ep_bnred;
  const bf16_raw* ep_z;
  const bf16_raw* ep_y;
  const float* ep_mean;
  const float* ep_rstd;
  // ep_gamma / ep_beta (optional): the 3x3/s1 halo kernel then recomputes the ReLU mask
  // from z exactly as bn_fwd_train rounded y (bf16(fma(z, gamma*rstd, fma(-mean,
  // gamma*rstd, beta))) > 0) and never reads y; the implicit GEMM always reads ep_y
  const float* ep_gamma;
  const float* ep_beta;
  // ep_gacc (dense_gacc.hip only): no output is written; gamma*rstd * g is ADDED into
  // ep_gacc (same row stride ldc as ep_z; bf16 with one rounding, or fp32 when
  // ep_gacc_f32) - the DenseNet block gradient, whose per-channel BN-backward corrections
  // are deferred (bn_defer_step)
  void* ep_gacc;
  int ep_gacc_f32;
  int stap;               // 8-channel "super-tap" forward: each tap entry = 4 adjacent kernel
                          // columns (dw .. dw+3, weight taps bt .. bt+ns-1), Ktot = 32 * T
  int beta;               // 1: accumulate, C = acc + C (bf16 read-add-write, one rounding):
                          // a second gradient contribution lands in the first one's buffer
  FastDiv fd_hw, fd_ow;   // oH * oW, oW (igemm_set_fastdiv, right before a launch)
  // second GEMM source (merged stride-phase dgrad, uniform-tap LDS-DMA kernel only): tap
  // entries with bt & TAP_SRC2 read A2 (same pixel grid and channel count as A) and B2
  // (K-contiguous, row stride ldb2) - the dgrad of a second conv that reads the same input
  // with the same stride (ResNet's 1x1/s2 shortcut) lands as extra K of the phase its
  // taps belong to, so dx is written once
  const bf16_raw* A2;
  const bf16_raw* B2;
  int ldb2;
  // kpad (uniform-tap LDS-DMA kernel, K-contiguous B): aC is 16-B but not 32-granular
  // (Inception's 48 / 80 channels): every tap's K is padded to a multiple of 32, Ktot =
  // T * round32(aC), and the chunks past aC read zeros
  int kpad;
  // accumulate (beta = 1) from ep_res instead of the old C, masked by the ReLU bit mask
  // ep_rmask (bit e % 8 of byte e / 8 for element e): a residual block's shortcut gradient
  // dy * (y > 0) added in the conv1 dgrad epilogue without being written first (halo
  // kernels only; dense [M][N] rows)
  const bf16_raw* ep_res;
  const uint8_t* ep_rmask;
  // the stem's 3x3/s2/p1 max-pool fused into the pixel-pair stem forward (conv_stem.hip;
  // sp_zsel set): per pooled window and channel the extreme z of the window rows inside the
  // kernel's 8-row item - the max where gamma >= 0, the min where gamma < 0, which is where
  // relu(bn(z)) is largest - and its tap 3 i + k ([N][P/2][Q/2][N] each).  An item's first
  // pooled row lacks its top window row: the previous item leaves that row's horizontal
  // extreme in sp_bz / sp_bidx ([N][P/8][Q/2][N]) and stem_pool_apply merges the two.
  bf16_raw* sp_zsel;
  uint8_t* sp_idx;
  bf16_raw* sp_bz;
  uint8_t* sp_bidx;
  const float* sp_gamma;
};
constexpr short TAP_SRC2 = 0x2000;

// fill the FastDiv fields of a rows launch (and of its stride phases)
inline void igemm_set_fastdiv(IGemmArgs& a) {
  a.fd_hw = make_fastdiv((uint32_t)std::max(1, a.oH * a.oW));
  a.fd_ow = make_fastdiv((uint32_t)std::max(1, a.oW));
  for (int i = 0; i < a.nphase && i < MAXPH; ++i) {
    a.ph[i].fd_hw = make_fastdiv((uint32_t)std::max(1, a.ph[i].oH * a.ph[i].oW));
    a.ph[i].fd_ow = make_fastdiv((uint32_t)std::max(1, a.ph[i].oW));
  }
}

struct WGradArgs {
  const bf16_raw* dy;
  const bf16_raw* x;
  float* dw;
  float* slab;  // split partials [splits][Kout][Ncols] (igemm_wgrad_ws_floats), or null
  int Kout, C, H, W, P, Q, R, S, sh, sw, ph, pw;
  int Mpix;
  int Ncols;
  int ktiles_per_split;
  int tiles_n, tiles_total;
  int overwrite;  // 1: dw holds nothing to keep (first gradient since zero_grad): store, no
                  // read-modify-write of the fp32 arena
};

// igemm.hip
int64_t igemm_slab_floats(int M, int N);
void igemm_rows(IGemmArgs a, int vw, float* ws, float* slab, hipStream_t s);  // B K-contig
// dgrad GEMMs: B N-contiguous (the forward weight, read with transposing LDS loads) or,
// with bkc, K-contiguous (the transposed weight copy; set a.b_tapmap)
void igemm_rows_dgrad(IGemmArgs a, int vw, float* ws, hipStream_t s, bool bkc = false);
// all stride phases of a strided-conv dgrad (a.nphase, a.ph[], shared a.taps) in one launch
// on the LDS-DMA engine when eligible, else one igemm_rows_dgrad per phase
void igemm_rows_dgrad_phases(IGemmArgs a, int vw, hipStream_t s, bool bkc = false);
// whether a merged-phase dgrad with a second source (a.A2) runs on the kernel that reads it
bool igemm_dgrad_src2_ok(const IGemmArgs& a, int vw, bool bkc);
// dgrad with the fused BN-backward reduction (a.ep_* set): sums[2][N] receives
// (sum g, sum g * xhat); slab holds igemm_bnred_slab_floats(a) floats
int64_t igemm_bnred_slab_floats(int M, int N, int nphase);
void igemm_rows_dgrad_bnred(IGemmArgs a, int vw, bool bkc, float* slab, float* sums,
                            hipStream_t s);
void igemm_wgrad(WGradArgs a, int vwa, int vwb, hipStream_t s);
int64_t igemm_ws_floats(int M, int N, int Ktot);          // split-K partials (0: no split)
int64_t igemm_wgrad_ws_floats(int Kout, int Ncols, int Mpix);  // wgrad split slab (0: none)
int igemm_engine();  // 0 register staging, 1 LDS-DMA rows GEMMs (default), 2 LDS-DMA all
void igemm_set_engine(int engine);
void igemm_force_tile(int bm, int bn, int splits);  // measurement override (0: auto)
// tile autotuner (igemm.hip): on by default (MPA_TUNE=0 off); the cached choices as text
void igemm_set_tune(int on);
void igemm_set_tune_drain(int on);  // tuner drains the device (1) or its stream (0)
std::string igemm_tuned_table();
// adopt a table in igemm_tuned_table()'s format (replace: drop the current entries first)
int igemm_tuned_load(const std::string& table, bool replace);
void igemm_set_dma_uni(int on);  // LDS-DMA uniform-tap fast path (default on)
bool igemm_stap_ok();  // super-tap forward available (engine >= 1 and fast path on)
// conv_halo.hip: halo-staged direct 3x3 / stride-1 conv (forward and stride-1 dgrad with
// a K-contiguous B); run_rows / the fused-reduction dgrad take it when conv3_halo_ok
bool conv3_halo_ok(const IGemmArgs& a);
int conv3_halo(IGemmArgs a, hipStream_t s);  // returns the statistics-slab rows written
constexpr int HALO_MAX_ROWS = 256;           // its slab rows (one per persistent block)
void igemm_set_halo(int on);                 // MPA_HALO=0 disables (A/B, bitwise tests)
void igemm_set_halo_mi7(int on);     // MPA_HALO_MI7 (448-pixel resident-weight tiles)
void igemm_set_halo_strip(int mode);  // MPA_HALO_STRIP (0 off, 1 wide images, 2 + layer1 3-stage)
// halo-staged 3x3/s1 weight gradient: partials into a.slab ([Z][Kout][9C]); returns Z
// halo-staged pixel-pair stem weight gradient (conv_stem.hip): partials into a.slab
// ([Z][64][224], <= stem_wgrad_ws_floats()); returns Z
bool stem_wgrad_ok(const WGradArgs& a);
int stem_wgrad(WGradArgs a, hipStream_t s);
int64_t stem_wgrad_ws_floats();
// the same weight gradient with the stem's BN + ReLU + 3x3/s2/p1 max-pool backward formed in
// its operand staging (a.dy = the conv output z; dz is never written): partials into a.slab
struct StemPoolArgs {
  const bf16_raw* dp;    // pooled gradient [N][PP][PQ][64]
  const uint8_t* idx;    // window argmax tap (3 i + k) [N][PP][PQ][64]
  const float *mean, *rstd, *gamma, *beta;
  const float* sums;     // [2][64]: sum g, sum g xhat over the batch (maxpool_bn_bwd_sums)
  int PP, PQ;            // pooled extent (P / 2, Q / 2)
  float invM;            // set by stem_pool_wgrad
};
bool stem_pool_wgrad_ok(const WGradArgs& a, const StemPoolArgs& q);
int stem_pool_wgrad(WGradArgs a, StemPoolArgs q, hipStream_t s);
// stem_pool_wgrad + the slab reduction into a.dw
void igemm_stem_pool_wgrad(WGradArgs a, StemPoolArgs q, hipStream_t s);
bool conv3_halo_wgrad_ok(const WGradArgs& a);
void igemm_set_halo_wxmap(int on);  // XCD-grouped halo weight-gradient blocks (MPA_HALO_WXMAP)
void igemm_set_halo_wprod(int on);  // producer-wave halo weight gradients (MPA_HALO_WPROD)
int conv3_halo_wgrad(WGradArgs a, hipStream_t s);
int64_t conv3_halo_wgrad_ws_floats(int Kout, int Ncols);
bool igemm_halo_enabled();
// Comm-aware persistent grids (conv_halo.hip).  While a data-parallel collective overlaps
// backward, its CTAs hold CUs that a persistent conv block (146-150 KB of LDS) cannot
// share; a block whose static tile share is queued behind one starts late and stretches
// the whole kernel.  The bucketer reserves the collective's CTA count while a bucket is in
// flight, and the persistent launches (halo fwd/dgrad and wgrad, stem fwd and wgrad) size
// their grids to the CUs left: active_cus() = CU count - reserve, a multiple of 8 (XCDs).
void set_comm_reserve(int cus);
int comm_reserve();
int active_cus();
// conv_stem.hip: direct row-staged forward of the 7x7 pixel-pair stem (super-tap layout,
// 64 output channels); run_rows takes it when conv_stem_ok.  Returns the slab rows written.
bool conv_stem_ok(const IGemmArgs& a);
int conv_stem(IGemmArgs a, hipStream_t s);
// the pooled half of the fused stem forward: merges each item's first pooled row with the
// previous item's bottom row (a.sp_bz), then y = relu(bn(zsel)) with the batch statistics
// `stats` ([2][C] mean, biased var); mean / rstd out, running stats (momentum) and the
// batch counter updated like bn_relu_maxpool_fwd
void stem_pool_apply(const IGemmArgs& a, const float* stats, const float* gamma,
                     const float* beta, float* rmean, float* rvar, float momentum, float eps,
                     bf16_raw* y, float* mean, float* rstd, int64_t* counter, hipStream_t s);
void igemm_set_stem(int on);  // MPA_STEM_DIRECT=0 disables (A/B, tests)

// bn.hip  (x/y/res/dy/dx: [M][C] bf16 rows; per-channel fp32 vectors)
// ws: float workspace of bn_ws_floats(M, C) elements (per-block partial-sum slab)
int64_t bn_ws_floats(int M, int C);
void slab_reduce(const float* slab, int S, int W, float* out, bool zero_out, hipStream_t s);
// deferred BN-backward corrections of a dense block (bn.hip, bn_defer_step_kernel); the host
// guarantees (Ci - s0) % 8 == 0 and 256 % ((Ci - s0) / 8) == 0
// DenseNet norm1 -> conv1 dgrad hand-off kernel (dense_gacc.hip)
bool dense_gacc_ok(const IGemmArgs& a);
void dense_gacc(IGemmArgs a, float* slab, float* sums, hipStream_t s);
void bn_defer_step(const float* sums, const float* gamma, const float* mean, const float* rstd,
                   int Ci, int s0, int M, float* k12, int ldk, float* dgamma, float* dbeta,
                   void* G, bool g_f32, int ldg, const bf16_raw* x, int ldx, bf16_raw* out,
                   hipStream_t s);
// MPA_DETERMINISTIC: fixed-order cross-block reductions, no timing-based tile autotuning
void set_deterministic(int on);
bool deterministic();
// sums [2][C] of (x - shift) and (x - shift)^2 over M rows -> out [mean(C), var(C)]
// slab [S][2C] of shifted (sum, sumsq) rows -> sums [2C] and out [mean(C), var(C)] (the
// slab may be folded in place); replaces slab_reduce + stats_finalize
void slab_stats(float* slab, int S, int C, const float* shift, int M, float* sums, float* out,
                hipStream_t s, int out_ld = 0);
void stats_finalize(const float* sums, const float* shift, int M, int C, float* out,
                    hipStream_t s);
void bn_stats(const bf16_raw* x, int M, int C, const float* shift, float* stats, float* ws,
              hipStream_t s);
void bn_fwd_train(const bf16_raw* x, const float* stats, const float* gamma, const float* beta,
                  float* rmean, float* rvar, float momentum, float eps, const bf16_raw* res,
                  int relu, int M, int C, bf16_raw* y, float* mean, float* rstd,
                  int64_t* counter, hipStream_t s,  // counter (num_batches_tracked) += 1
                  uint8_t* ymask = nullptr,  // optional ReLU bit mask of y ([M*C/8] bytes)
                  int ldx = 0,   // x row stride (0: C) - a channel prefix of a wider buffer
                  int lds = 0,   // stats = [mean | var] rows lds apart (0: C)
                  const float* res_aff = nullptr,  // [2][C]: res enters as res * aff0 + aff1
                  int ldy = 0);  // y row stride (0: C) - a channel window of a wider buffer
// mean / rstd / running stats / num_batches_tracked of a train-mode BN whose apply pass is
// deferred to its consumer; aff [2][C] = [gamma rstd | beta - mean gamma rstd]
void bn_stats_affine(const float* stats, const float* gamma, const float* beta, float* rmean,
                     float* rvar, float momentum, float eps, int M, int C, float* mean,
                     float* rstd, float* aff, int64_t* counter, hipStream_t s);
// avgpool2x2/s2(relu(z * aff0 + aff1)) without writing the BN output (H, W even, C % 8 == 0)
void bn_relu_avgpool2_fwd(const bf16_raw* z, const float* aff, int N, int H, int W, int C,
                          bf16_raw* y, hipStream_t s);
// y = relu?(x * aff[c] + aff[C + c]) (aff [2][C]: bn_stats_affine's scale | shift)
void affine_act(const bf16_raw* x, const float* aff, int relu, int M, int C, bf16_raw* y,
                hipStream_t s);
void bn_fwd_eval(const bf16_raw* x, const float* gamma, const float* beta, const float* rmean,
                 const float* rvar, float eps, const bf16_raw* res, int relu, int M, int C,
                 bf16_raw* y, hipStream_t s, int ldx = 0);
// zmask_beta (y == null): the ReLU mask of y = relu(bn(x)) is recomputed from x with this
// beta (no residual in the forward), so y is never read
void bn_bwd(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
            const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M, int C,
            bf16_raw* dx, bf16_raw* g, float* ws, hipStream_t s,
            const float* zmask_beta = nullptr,
            const uint8_t* ymask = nullptr,  // bit mask from bn_fwd_train, used instead of y
            int ldx = 0,             // x row stride (0: C)
            float* gacc = nullptr,   // non-null: dx ADDED in fp32 into gacc [M][ldg] (dx unused)
            int ldg = 0,
            int lddx = 0,            // dx row stride (0: C) - a channel window of a wider buffer
            bool gacc_bf16 = false,  // gacc holds bf16 (cast the pointer) instead of fp32
            int lddy = 0);           // dy row stride (0: C) - a channel window of a wider buffer
// backward of relu(bn(x) + bn2(x2)), both train-mode BNs (bn2: a deferred downsample BN
// applied on read): dx and dx2 from one reduce and one apply pass, mask = the forward's bit
// mask; ws holds bn_pair_ws_floats(M, C) floats
// 2x2 / stride-2 / pad-0 max pool over an even image (VGG): one pooled pixel x 8 channels
// per thread; backward with yp + sums: the pooled tensor is a ReLU output whose producer's
// mask and bias-gradient sum are applied / reduced here (sums [C]; ws maxpool2_ws_floats)
bool maxpool2_ok(int N, int H, int W, int C, int kh, int kw, int sh, int sw, int ph, int pw);
void maxpool2_fwd(const bf16_raw* x, int N, int H, int W, int C, bf16_raw* y, uint8_t* idx,
                  hipStream_t s);
int64_t maxpool2_ws_floats(int N, int H, int W, int C);
void maxpool2_bwd(const bf16_raw* dy, const uint8_t* idx, const bf16_raw* yp, int N, int H, int W,
                  int C, bf16_raw* dx, float* sums, float* ws, hipStream_t s);
int64_t bn_pair_ws_floats(int M, int C);
void bn_bwd_pair(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* x2, const uint8_t* ymask,
                 const float* mean, const float* rstd, const float* gamma, const float* mean2,
                 const float* rstd2, const float* gamma2, float* dgamma, float* dbeta,
                 float* dgamma2, float* dbeta2, int M, int C, bf16_raw* dx, bf16_raw* dx2,
                 float* ws, hipStream_t s);
void bn_bwd_apply(const bf16_raw* dy, const bf16_raw* x, const bf16_raw* y, const float* mean,
                  const float* rstd, const float* gamma, float* dgamma, float* dbeta, int M,
                  int C, bf16_raw* dx, bf16_raw* g, const float* sums, hipStream_t s,
                  int lddy = 0);
void act_bwd(const bf16_raw* dy, const bf16_raw* y, float* dbias, int M, int C, bf16_raw* g,
             float* ws, hipStream_t s);
void relu_fwd(const bf16_raw* x, int64_t n, bf16_raw* y, hipStream_t s);
// fused BN(train) + ReLU + max-pool (stems): z [N][H][W][C] -> y [N][P][Q][C] + argmax idx;
// backward: dp, idx, z -> dz (BN backward of the ReLU(BN) through the pool), ws of
// maxpool_bn_ws_floats(N*H*W, C) floats; C % 8 == 0.  zsel (optional, [N][P][Q][C]): the raw
// z at each window's argmax, written by the forward; with it the backward's reduction pass
// reads only pooled-size tensors
void bn_relu_maxpool_fwd(const bf16_raw* z, const float* stats, const float* gamma,
                         const float* beta, float* rmean, float* rvar, float momentum, float eps,
                         int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                         int ph, int pw, bf16_raw* y, uint8_t* idx, float* mean, float* rstd,
                         int64_t* counter, hipStream_t s, bf16_raw* zsel = nullptr);
int64_t maxpool_bn_ws_floats(int M, int C);
// pooled-only backward reduction of the fused stem: sums (ws[0 .. 2C)) and dgamma / dbeta
void maxpool_bn_bwd_sums(const bf16_raw* dp, const bf16_raw* zsel, const float* mean,
                         const float* rstd, const float* gamma, const float* beta, float* dgamma,
                         float* dbeta, int MP, int C, float* ws, hipStream_t s);
void maxpool_bn_bwd(const bf16_raw* dp, const uint8_t* idx, const bf16_raw* z, const float* mean,
                    const float* rstd, const float* gamma, const float* beta, float* dgamma,
                    float* dbeta, int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh,
                    int sw, int ph, int pw, bf16_raw* dz, float* ws, hipStream_t s,
                    const bf16_raw* zsel = nullptr);

// pool.hip  (NHWC)
void maxpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, bf16_raw* y, uint8_t* idx, hipStream_t s);
void maxpool_bwd(const bf16_raw* dy, const uint8_t* idx, int N, int H, int W, int C, int P,
                 int Q, int kh, int kw, int sh, int sw, int ph, int pw, bf16_raw* dx,
                 hipStream_t s);
// ldx / ldo: pixel stride of x / dx (0: C) - a channel window of a wider NHWC buffer
void avgpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, int count_include_pad, bf16_raw* y,
                 hipStream_t s, int ldx = 0);
void avgpool_bwd(const bf16_raw* dy, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                 int sh, int sw, int ph, int pw, int count_include_pad, bf16_raw* dx,
                 hipStream_t s, int ldo = 0);
void adaptive_avgpool_fwd(const bf16_raw* x, int N, int H, int W, int C, int P, int Q,
                          bf16_raw* y, hipStream_t s);
void adaptive_avgpool_bwd(const bf16_raw* dy, int N, int H, int W, int C, int P, int Q,
                          bf16_raw* dx, hipStream_t s);

// concat.hip (NHWC channel concat / split; every segment's channels % 8 == 0)
constexpr int CAT_MAXSEG = 32;
// fp32 gradient buffer G [pixels][ldg]: G[:, off:off+cs] (+)= src (bf16 [pixels][cs]) /
// dst = bf16(G[:, off:off+cs]); ldg, off, cs multiples of 8
void chan_accum(float* g, int ldg, int off, const bf16_raw* src, int cs, int pixels, bool assign,
                hipStream_t s);
void chan_extract(const float* g, int ldg, int off, bf16_raw* dst, int cs, int pixels,
                  hipStream_t s);
void concat_channels(const bf16_raw* const* xs, const int* chans, int nseg, int pixels,
                     int ctotal, bf16_raw* y, hipStream_t s);
// dst [rows][ld] (16-bit units) at unit offset off <- src [rows][cs]; ld, off, cs % 8 == 0
// (bf16 activations, or fp32 rows as pairs of units)
void chan_insert(bf16_raw* dst, int ld, int off, const bf16_raw* src, int cs, int rows,
                 hipStream_t s);
// dst [rows][cs] <- src [rows][ld] at unit offset off (the inverse of chan_insert)
void chan_slice(const bf16_raw* src, int ld, int off, bf16_raw* dst, int cs, int rows,
                hipStream_t s);
void split_channels(const bf16_raw* dy, const int* chans, int nseg, int pixels, int ctotal,
                    bf16_raw* const* dxs, hipStream_t s);

// loss.hip
// logits rows have stride ld >= NC (padded heads); ce_bwd writes dlogits with stride ld and
// zeros in columns NC..ld-1
void ce_fwd_rows(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld, float* row_loss,
                 float* lse, hipStream_t s);
// loss: [1 + B] floats (mean at [0], per-row terms after it; fixed-order sum)
void ce_fwd(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld, float* loss,
            float* lse, hipStream_t s);
void ce_bwd(const bf16_raw* logits, const int64_t* labels, const float* lse,
            const float* grad_out, int B, int NC, int ld, bf16_raw* dlogits, hipStream_t s,
            float weight = 1.f);
void ce_fwd_weighted(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld,
                     float* out, float* acc, float weight, bool accumulate, float* rows,
                     float* lse, hipStream_t s);
// fp32 t[0:n) = 0 (n % 4 == 0, 16-B aligned); step[0] += 1
void zero_f32(float* t, int64_t n, hipStream_t s);
void add_f32(float* dst, const float* src, int64_t n, hipStream_t s);  // dst += src
// t as [rows][period] fp32: zero columns [first, first + count)
void zero_cols_f32(float* t, int64_t rows, int period, int first, int count, hipStream_t s);
// a += b, bf16 [n] (n % 8 == 0, 16-B aligned)
void add_bf16(bf16_raw* a, const bf16_raw* b, int64_t n, hipStream_t s);
void step_inc(float* step, hipStream_t s);
void argmax_correct(const bf16_raw* logits, const int64_t* labels, int B, int NC, int ld,
                    int64_t* count, hipStream_t s);

// optim.hip (flat fp32 arenas)
void adam_step(float* p, const float* g, float* m, float* v, bf16_raw* shadow,
               const float* step, int64_t n, float lr, float b1, float b2, float eps, float wd,
               float grad_scale, hipStream_t s);
void sgd_step(float* p, const float* g, float* buf, bf16_raw* shadow, const float* step,
              int64_t n, float lr, float momentum, float dampening, float wd, int nesterov,
              float grad_scale, hipStream_t s);
void cast_f32_bf16(const float* x, bf16_raw* y, int64_t n, hipStream_t s);
// wt[c][t][k] = w[k][t][c] per segment (src_off, dst_off, K, RS, C, first_tile) of seg
// step_inc (optional): the optimizer's step counter, incremented by the same launch
void transpose_krsc(const bf16_raw* w, bf16_raw* wt, const int64_t* seg, int nseg,
                    int total_tiles, hipStream_t s, float* step_inc = nullptr);

// preprocess.hip
struct Norm3 {
  float mean[3];
  float std[3];
};
// zero border around the resized image (pre-padded pixel-pair stem input); all 0 = none
struct OutPad {
  int top, bottom, left, right;
};
void preprocess_set_copy(int on);  // identity-size fast path on/off (tests, A/B)
// ext (optional): per-image source extents [B][2] = (h, w) inside the [H][W] pitch (mode 0)
void preprocess(const uint8_t* img, int B, int H, int W, int OH, int OW, Norm3 nrm, int mode,
                int cpad, OutPad pad, bf16_raw* out, hipStream_t s, const int* ext = nullptr);
// PIL-exact bicubic (eval transform): per-image extents ext [B][2] (h, w) inside the
// [Hp][Wp] pitch (nullptr: all full), per-image table selectors sel [B][2]; tmp holds
// B * Hp * OW RGBx words
void preprocess_pil(const uint8_t* img, int B, int Hp, int Wp, const int* ext, const int* sel,
                    const int* hb, const int* hk, int kh, const int* vb, const int* vk, int kv,
                    int OH, int OW, Norm3 nrm, int cpad, OutPad pd, uint32_t* tmp, bf16_raw* out,
                    hipStream_t s);
// counter (optional, device uint32): added to offset and incremented after the launch
void dropout_fwd(const bf16_raw* x, int64_t n, float p, uint64_t seed, uint64_t offset,
                 uint32_t* counter, bf16_raw* y, uint8_t* mask, hipStream_t s);
void dropout_bwd(const bf16_raw* dy, const uint8_t* mask, int64_t n, float p, bf16_raw* dx,
                 hipStream_t s);

// diag.hip: stand-in for a concurrent RCCL collective (bench.py --emulate-comm)
void comm_emulator(int blocks, int threads, int lds_bytes, double us, float* sink, hipStream_t s);
void atomic_latency(int blocks, int iters, int mode, int* q, hipStream_t s);  // diag.hip

}  // namespace mpa
