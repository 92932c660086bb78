// Torch-facing binding layer for the gfx950 kernel library (module mpi_pytorch_amd._C).
//
// Responsibilities: validate dtypes/shapes/contiguity (so a kernel never sees operands its
// grid does not expect), allocate outputs on the caller's device, build the implicit-GEMM
// tap tables, and launch on the current HIP stream (so everything composes with HIP
// graphs and the RCCL comm stream).  The function set mirrors ops/ref.py one-to-one.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>

#include <vector>

#include "kernels/api.h"
#include "runtime/runtime.h"

using torch::Tensor;

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_BF16(x) \
  TORCH_CHECK((x).scalar_type() == torch::kBFloat16, #x " must be bfloat16, got ", (x).scalar_type())
#define CHECK_F32(x) \
  TORCH_CHECK((x).scalar_type() == torch::kFloat32, #x " must be float32, got ", (x).scalar_type())
#define CHECK_ACT(x) \
  CHECK_CUDA(x);     \
  CHECK_CONTIG(x);   \
  CHECK_BF16(x)

inline const mpa::bf16_raw* bp(const Tensor& t) {
  return reinterpret_cast<const mpa::bf16_raw*>(t.data_ptr());
}
inline mpa::bf16_raw* bpm(const Tensor& t) { return reinterpret_cast<mpa::bf16_raw*>(t.data_ptr()); }
inline bool has(const Tensor& t) { return t.defined() && t.numel() > 0; }
inline const float* fopt(const Tensor& t) {
  if (!has(t)) return nullptr;
  CHECK_CUDA(t);
  CHECK_F32(t);
  CHECK_CONTIG(t);
  return t.data_ptr<float>();
}
inline float* fopt_mut(const Tensor& t) { return const_cast<float*>(fopt(t)); }
inline const mpa::bf16_raw* bopt(const Tensor& t) {
  if (!has(t)) return nullptr;
  CHECK_ACT(t);
  return bp(t);
}

inline int vec_width(int64_t c) { return (c % 8 == 0) ? 8 : ((c % 4 == 0) ? 4 : 1); }

float* alloc_ws(Tensor& holder, const Tensor& like, int64_t n) {
  if (n <= 0) return nullptr;
  holder = torch::empty({n}, like.options().dtype(torch::kFloat32));
  return holder.data_ptr<float>();
}

Tensor empty_like_shape(const Tensor& ref, at::IntArrayRef shape, torch::Dtype dt) {
  return torch::empty(shape, ref.options().dtype(dt));
}

// ------------------------------------------------------------------------------- conv
// out (optional): a bf16 channel-window view [N, P, Q, K] of a wider NHWC buffer (DenseNet's
// block buffer) the output is written into (row stride out.stride(2)); stats may then be a
// [2, K] window of a wider statistics table (row stride stats.stride(0))
Tensor affine_act(Tensor x, Tensor aff, bool relu) {
  CHECK_ACT(x);
  CHECK_CUDA(aff);
  const int C = x.size(-1);
  TORCH_CHECK(C % 8 == 0 && aff.numel() == 2 * C && aff.scalar_type() == torch::kFloat32 &&
                  aff.is_contiguous(),
              "affine_act: x [..., C] (C % 8 == 0), aff [2, C] fp32");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = torch::empty_like(x);
  mpa::affine_act(bp(x), aff.data_ptr<float>(), relu ? 1 : 0, (int)(x.numel() / C), C, bpm(y),
                  cur_stream());
  return y;
}

// pooled outputs of the fused stem forward (conv_stem_pool_fwd): when set, conv_fwd_impl
// returns an undefined tensor unless the pixel-pair stem kernel takes the launch
struct StemPoolOut {
  Tensor zsel, idx, bz, bidx;
  const float* gamma;
};

static Tensor conv_fwd_impl(Tensor x, Tensor w, Tensor bias, int64_t sh, int64_t sw, int64_t ph,
                            int64_t pw, bool relu, Tensor stats, Tensor shift, const Tensor* out,
                            StemPoolOut* spo = nullptr, mpa::IGemmArgs* args_out = nullptr) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4, "conv_fwd: x NHWC, w KRSC");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(w.size(3) == C, "conv_fwd: channel mismatch");
  TORCH_CHECK(R * S <= mpa::MAXT, "conv_fwd: too many taps");
  const int P = (H + 2 * ph - R) / sh + 1, Q = (W + 2 * pw - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0, "conv_fwd: empty output");
  if (has(bias)) TORCH_CHECK(bias.numel() == K, "conv_fwd: bias size");
  int stats_ld = 0;
  if (has(stats)) {
    TORCH_CHECK(stats.numel() == 2 * K, "conv_fwd: stats size");
    if (out) {
      TORCH_CHECK(stats.dim() == 2 && stats.size(0) == 2 && stats.stride(1) == 1 &&
                      stats.stride(0) >= K,
                  "conv_fwd_into: stats must be a [2, K] row-window");
      stats_ld = (int)stats.stride(0);
    }
  }
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y;
  int ldc = K;
  if (out) {
    CHECK_CUDA((*out));
    CHECK_BF16((*out));
    TORCH_CHECK(out->dim() == 4 && out->size(0) == N && out->size(1) == P && out->size(2) == Q &&
                    out->size(3) == K && out->stride(3) == 1 &&
                    out->stride(1) == (int64_t)Q * out->stride(2) &&
                    out->stride(0) == (int64_t)P * out->stride(1) && out->stride(2) % 8 == 0,
                "conv_fwd_into: out must be a channel window [N, P, Q, K] of an NHWC buffer");
    y = *out;
    ldc = (int)out->stride(2);
  } else {
    y = empty_like_shape(x, {N, P, Q, K}, torch::kBFloat16);
  }
  mpa::IGemmArgs a{};
  a.A = bp(x); a.aH = H; a.aW = W; a.aC = C;
  a.oH = P; a.oW = Q; a.M = N * P * Q;
  a.Uh = sh; a.Uw = sw; a.Oh = -ph; a.Ow = -pw;
  a.T = R * S;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      const int t = r * S + s;
      a.taps.dh[t] = r; a.taps.dw[t] = s; a.taps.bt[t] = t;
    }
  a.Ktot = a.T * C;
  a.B = bp(w); a.N = K; a.RS = R * S; a.ldb = a.Ktot;
  if (C == 8 && S > 1 && mpa::igemm_stap_ok()) {
    // 8-channel image stem: group 4 adjacent kernel columns into one 32-deep K tile (their
    // input pixels are 64 contiguous bytes in NHWC), so the stem takes the uniform-tap
    // fast path; columns past S get zero weights.  K grows from R*S*8 to R*ceil(S/4)*32.
    int t = 0;
    for (int r = 0; r < R; ++r)
      for (int s0 = 0; s0 < S; s0 += 4, ++t) {
        a.taps.dh[t] = r; a.taps.dw[t] = s0;
        a.taps.bt[t] = (short)((r * S + s0) | (std::min(4, S - s0) << 12));
      }
    a.T = t;
    a.Ktot = t * 32;
    a.stap = 1;
  }
  a.C = y.data_ptr(); a.ldc = ldc;
  a.dH = P; a.dW = Q; a.Uoh = 1; a.Uow = 1; a.Poh = 0; a.Pow = 0;
  a.bias = fopt(bias);
  if (stats_ld) {  // a checked [2, K] row-window of a wider table
    CHECK_CUDA(stats);
    CHECK_F32(stats);
    a.stats = stats.data_ptr<float>();
  } else {
    a.stats = fopt_mut(stats);
  }
  a.stats_ld = stats_ld;
  a.stats_shift = fopt(shift);
  if (a.stats_shift) TORCH_CHECK(shift.numel() == K, "conv_fwd: shift size");
  a.relu = relu ? 1 : 0;
  if (spo) {
    const int PP = P / 2, PQ = Q / 2, P8 = std::max(1, P / 8);
    spo->zsel = empty_like_shape(x, {N, PP, PQ, K}, torch::kBFloat16);
    spo->idx = empty_like_shape(x, {N, PP, PQ, K}, torch::kUInt8);
    spo->bz = empty_like_shape(x, {N, P8, PQ, K}, torch::kBFloat16);
    spo->bidx = empty_like_shape(x, {N, P8, PQ, K}, torch::kUInt8);
    a.sp_zsel = bpm(spo->zsel);
    a.sp_idx = spo->idx.data_ptr<uint8_t>();
    a.sp_bz = bpm(spo->bz);
    a.sp_bidx = spo->bidx.data_ptr<uint8_t>();
    a.sp_gamma = spo->gamma;
    if (!(vec_width(C) == 8 && mpa::igemm_engine() >= 1 && a.stats && mpa::conv_stem_ok(a)))
      return Tensor();
  }
  if (args_out) *args_out = a;
  Tensor ws;
  // (split-K's finalize writes dense [M][N] rows: none into a window)
  float* wsp = ldc == K ? alloc_ws(ws, x, mpa::igemm_ws_floats(a.M, a.N, a.Ktot)) : nullptr;
  Tensor slab;
  if (a.stats)
    slab = torch::empty({mpa::igemm_slab_floats(a.M, a.N)}, x.options().dtype(torch::kFloat32));
  mpa::igemm_rows(a, vec_width(C), wsp, a.stats ? slab.data_ptr<float>() : nullptr,
                  cur_stream());
  return y;
}

Tensor conv_fwd(Tensor x, Tensor w, Tensor bias, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                bool relu, Tensor stats, Tensor shift) {
  return conv_fwd_impl(x, w, bias, sh, sw, ph, pw, relu, stats, shift, nullptr);
}

void conv_fwd_into(Tensor x, Tensor w, Tensor bias, int64_t sh, int64_t sw, int64_t ph,
                   int64_t pw, bool relu, Tensor stats, Tensor shift, Tensor out) {
  conv_fwd_impl(x, w, bias, sh, sw, ph, pw, relu, stats, shift, &out);
}

// The ResNet / DenseNet stem forward, conv -> BN(train) -> ReLU -> 3x3/s2/p1 max-pool, with
// the pool taken inside the conv kernel (conv_stem.hip, PF) and the BN + ReLU applied to the
// pooled extremes only (stem_pool_apply).  Returns [y, idx, mean, rstd, z, zsel] like
// bn_relu_maxpool_fwd (+ conv_fwd's z), or None when the stem kernel cannot take the launch.
c10::optional<std::vector<Tensor>> conv_stem_pool_fwd(Tensor x, Tensor w, int64_t sh, int64_t sw,
                                                      int64_t ph, int64_t pw, Tensor stats,
                                                      Tensor shift, Tensor gamma, Tensor beta,
                                                      Tensor rmean, Tensor rvar,
                                                      double momentum, double eps,
                                                      c10::optional<Tensor> counter) {
  CHECK_CUDA(gamma);
  CHECK_F32(gamma);
  TORCH_CHECK(gamma.numel() == w.size(0) && beta.numel() == w.size(0), "conv_stem_pool_fwd: BN size");
  StemPoolOut spo;
  spo.gamma = gamma.data_ptr<float>();
  mpa::IGemmArgs a{};
  Tensor z = conv_fwd_impl(x, w, Tensor(), sh, sw, ph, pw, false, stats, shift, nullptr, &spo, &a);
  if (!z.defined()) return c10::nullopt;
  const int K = w.size(0);
  Tensor y = torch::empty_like(spo.zsel);
  Tensor mean = torch::empty({K}, gamma.options());
  Tensor rstd = torch::empty({K}, gamma.options());
  mpa::stem_pool_apply(a, stats.data_ptr<float>(), gamma.data_ptr<float>(), fopt(beta),
                       fopt_mut(rmean), fopt_mut(rvar), (float)momentum, (float)eps, bpm(y),
                       mean.data_ptr<float>(), rstd.data_ptr<float>(),
                       (counter && counter->defined() && counter->numel() == 1)
                           ? counter->data_ptr<int64_t>() : nullptr,
                       cur_stream());
  return std::vector<Tensor>{y, spo.idx, mean, rstd, z, spo.zsel};
}

// wt (optional): the transposed weight [C][R*S][K] (arena shadow_t) - the dgrad GEMM then
// reads B K-contiguous like the forward GEMM.  bnred (optional): fuse the backward
// reduction of the ReLU(BN) that produced this conv's input (see igemm_rows_dgrad_bnred);
// then dx = g (masked) and bnred->sums receives [sum g | sum g*xhat].
struct BnRed {
  Tensor z, y, mean, rstd, sums, gamma, beta;
};
// src2: a second conv reading the same input with the same stride (its dy2 on dy's pixel
// grid with dy's channel count, weight w2 [K][R2][S2][C], transposed wt2 [C][R2*S2][K], pad
// ph2 / pw2): its taps join the stride phases they belong to (IGemmArgs::A2)
struct DgradSrc2 {
  Tensor dy2, w2, wt2;
  int ph2, pw2;
};

static Tensor conv_dgrad_impl(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t sh, int64_t sw,
                              int64_t ph, int64_t pw, c10::optional<Tensor> wt_opt,
                              BnRed* bnred, c10::optional<Tensor> accum = c10::nullopt,
                              const DgradSrc2* src2 = nullptr) {
  CHECK_ACT(dy);
  CHECK_ACT(w);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  const int Kw = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(Kw == K, "conv_dgrad: channel mismatch");
  TORCH_CHECK(R * S <= mpa::MAXT, "conv_dgrad: too many taps");
  const c10::OptionalDeviceGuard g(device_of(dy));
  // accum: dx accumulates into this tensor (a second gradient contribution to the same
  // activation, e.g. a residual block's input: conv1 dgrad + shortcut) - no separate add
  const bool acc = accum && accum->defined();
  Tensor dx;
  if (acc) {
    CHECK_ACT((*accum));
    TORCH_CHECK(accum->dim() == 4 && accum->size(0) == N && accum->size(1) == H &&
                    accum->size(2) == W && accum->size(3) == C,
                "conv_dgrad: accum shape mismatch");
    TORCH_CHECK(!bnred, "conv_dgrad: accum and the fused BN reduction are exclusive");
    dx = *accum;
  } else {
    dx = empty_like_shape(dy, {N, (int64_t)H, (int64_t)W, C}, torch::kBFloat16);
  }
  const int vw = std::min(vec_width(K), vec_width(C));
  // sub-pixel decomposition: output phase (a_, b_) of dx is a stride-1 conv of dy with the
  // taps (r, s) congruent to it; stride 1 has one phase
  mpa::IGemmArgs a{};
  a.A = bp(dy); a.aH = P; a.aW = Q; a.aC = K;
  a.Uh = 1; a.Uw = 1; a.Oh = 0; a.Ow = 0;
  a.B = bp(w); a.N = C; a.RS = R * S; a.ldb = C;
  const bool bkc = wt_opt && wt_opt->defined() && wt_opt->numel() == w.numel() && vw == 8;
  if (bkc) {
    CHECK_ACT((*wt_opt));
    a.B = bp(*wt_opt);
    a.ldb = R * S * K;
    a.b_tapmap = 1;
  }
  a.C = dx.data_ptr(); a.ldc = C;
  a.dH = H; a.dW = W; a.Uoh = sh; a.Uow = sw;
  a.bias = nullptr; a.stats = nullptr; a.relu = 0;
  a.beta = acc ? 1 : 0;
  int T = 0, nph = 0;
  for (int a_ = 0; a_ < sh; ++a_)
    for (int b_ = 0; b_ < sw; ++b_) {
      const int Hp = (H - a_ + sh - 1) / sh, Wp = (W - b_ + sw - 1) / sw;
      if (Hp <= 0 || Wp <= 0) continue;
      const int t0 = T;
      for (int r = 0; r < R; ++r) {
        if (((a_ + ph - r) % sh) != 0) continue;
        for (int s = 0; s < S; ++s) {
          if (((b_ + pw - s) % sw) != 0) continue;
          a.taps.dh[T] = (a_ + ph - r) / sh;
          a.taps.dw[T] = (b_ + pw - s) / sw;
          a.taps.bt[T] = r * S + s;
          ++T;
        }
      }
      if (src2) {
        const int R2 = src2->w2.size(1), S2 = src2->w2.size(2);
        for (int r = 0; r < R2; ++r) {
          if (((a_ + src2->ph2 - r) % sh) != 0) continue;
          for (int s = 0; s < S2; ++s) {
            if (((b_ + src2->pw2 - s) % sw) != 0) continue;
            TORCH_CHECK(T < mpa::MAXT, "conv_dgrad: too many taps");
            a.taps.dh[T] = (a_ + src2->ph2 - r) / sh;
            a.taps.dw[T] = (b_ + src2->pw2 - s) / sw;
            a.taps.bt[T] = (short)((r * S2 + s) | mpa::TAP_SRC2);
            ++T;
          }
        }
      }
      TORCH_CHECK(nph < mpa::MAXPH, "conv_dgrad: too many stride phases");
      a.ph[nph++] = mpa::PhaseDesc{N * Hp * Wp, Hp, Wp, (T - t0) * K, t0, T - t0, a_, b_, 0};
    }
  if (bnred) {
    a.ep_z = bp(bnred->z);
    a.ep_y = bopt(bnred->y);
    a.ep_mean = fopt(bnred->mean);
    a.ep_rstd = fopt(bnred->rstd);
    a.ep_gamma = fopt(bnred->gamma);
    a.ep_beta = fopt(bnred->beta);
    // without y (BN in the operand path: never written) every kernel recomputes the ReLU
    // mask from z with gamma / beta
    TORCH_CHECK(a.ep_y || (a.ep_gamma && a.ep_beta),
                "conv_dgrad_bnred: needs y or gamma / beta for the ReLU mask");
    TORCH_CHECK(!a.ep_gamma == !a.ep_beta, "conv_dgrad_bnred: gamma and beta go together");
    for (const Tensor* t : {&bnred->mean, &bnred->rstd, &bnred->gamma, &bnred->beta})
      TORCH_CHECK(!has(*t) || t->numel() == C, "conv_dgrad_bnred: per-channel vector size");
    bnred->sums = torch::empty({2 * C}, dy.options().dtype(torch::kFloat32));
    int k = 0;
    bool empty = false;
    for (int i = 0; i < nph; ++i) {
      empty |= a.ph[i].T == 0;
      if (a.ph[i].T > 0) a.ph[k++] = a.ph[i];
    }
    if (empty) dx.zero_();
    if (sh == 1 && sw == 1) {
      const mpa::PhaseDesc& d = a.ph[0];
      a.M = d.M; a.oH = d.oH; a.oW = d.oW; a.T = d.T; a.Ktot = d.Ktot; a.Poh = 0; a.Pow = 0;
      a.nphase = 0;
    } else {
      a.nphase = k;
    }
    TORCH_CHECK(!empty, "conv_dgrad_bnred: stride-phase without taps");
    Tensor slab = torch::empty({mpa::igemm_bnred_slab_floats(N * H * W, C, std::max(a.nphase, 1))},
                               dy.options().dtype(torch::kFloat32));
    mpa::igemm_rows_dgrad_bnred(a, vw, bkc, slab.data_ptr<float>(),
                                bnred->sums.data_ptr<float>(), cur_stream());
    return dx;
  }
  if (sh == 1 && sw == 1) {
    const mpa::PhaseDesc& d = a.ph[0];
    a.M = d.M; a.oH = d.oH; a.oW = d.oW; a.T = d.T; a.Ktot = d.Ktot; a.Poh = 0; a.Pow = 0;
    Tensor ws;
    float* wsp = alloc_ws(ws, dy, mpa::igemm_ws_floats(a.M, a.N, a.Ktot));
    mpa::igemm_rows_dgrad(a, vw, wsp, cur_stream(), bkc);
  } else {
    // phases with no taps (stride > kernel) leave their dx pixels zero (or, accumulating,
    // untouched)
    bool empty = false;
    for (int i = 0; i < nph; ++i) empty |= a.ph[i].T == 0;
    int k = 0;
    for (int i = 0; i < nph; ++i)
      if (a.ph[i].T > 0) a.ph[k++] = a.ph[i];
    a.nphase = k;
    if (src2) {
      a.A2 = bp(src2->dy2);
      a.B2 = bp(src2->wt2);
      a.ldb2 = src2->w2.size(1) * src2->w2.size(2) * K;
      if (!mpa::igemm_dgrad_src2_ok(a, vw, bkc)) return Tensor();  // caller runs them apart
    }
    if (empty && !acc) dx.zero_();
    mpa::igemm_rows_dgrad_phases(a, vw, cur_stream(), bkc);
  }
  return dx;
}

Tensor conv_dgrad(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t sh, int64_t sw, int64_t ph,
                  int64_t pw, c10::optional<Tensor> wt_opt, c10::optional<Tensor> accum) {
  return conv_dgrad_impl(dy, w, H, W, sh, sw, ph, pw, wt_opt, nullptr, accum);
}

// stride-1 dgrad plus a residual block's shortcut gradient dy_res * (y > 0) (y's ReLU bit
// mask from bn_fwd_train) added in the halo kernel's epilogue: the masked shortcut gradient
// is never written.  None when the launch would not run on the halo kernel.
c10::optional<Tensor> conv_dgrad_res(Tensor dy, Tensor w, Tensor wt, int64_t H, int64_t W,
                                     int64_t ph, int64_t pw, Tensor res, Tensor rmask) {
  CHECK_ACT(dy);
  CHECK_ACT(w);
  CHECK_ACT(res);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  const int R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(w.size(0) == K, "conv_dgrad_res: channel mismatch");
  TORCH_CHECK(res.dim() == 4 && res.size(0) == N && res.size(1) == H && res.size(2) == W &&
                  res.size(3) == C,
              "conv_dgrad_res: the residual gradient must have dx's shape");
  TORCH_CHECK(rmask.scalar_type() == torch::kUInt8 && rmask.is_contiguous() &&
                  rmask.numel() == res.numel() / 8 && rmask.device() == res.device(),
              "conv_dgrad_res: ReLU mask must be contiguous uint8 [numel / 8]");
  if (!(wt.defined() && wt.numel() == w.numel()) || vec_width(K) != 8 || vec_width(C) != 8 ||
      mpa::igemm_engine() < 1)
    return c10::nullopt;
  if (P != H + 2 * ph - R + 1 || Q != W + 2 * pw - S + 1) return c10::nullopt;
  if (C % 64 != 0) return c10::nullopt;  // (a column tile's 64 mask bits: one aligned 8-B load)
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = empty_like_shape(dy, {N, H, W, C}, torch::kBFloat16);
  mpa::IGemmArgs a{};
  a.A = bp(dy); a.aH = P; a.aW = Q; a.aC = K;
  a.Uh = 1; a.Uw = 1; a.Oh = 0; a.Ow = 0;
  a.B = bp(wt); a.N = C; a.RS = R * S; a.ldb = R * S * K; a.b_tapmap = 1;
  a.C = dx.data_ptr(); a.ldc = C;
  a.dH = H; a.dW = W; a.Uoh = 1; a.Uow = 1;
  a.beta = 1;
  a.ep_res = bp(res);
  a.ep_rmask = rmask.data_ptr<uint8_t>();
  int T = 0;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      a.taps.dh[T] = ph - r;
      a.taps.dw[T] = pw - s;
      a.taps.bt[T] = r * S + s;
      ++T;
    }
  a.T = T;
  a.M = N * H * W; a.oH = H; a.oW = W; a.Ktot = T * K; a.Poh = 0; a.Pow = 0;
  if (!mpa::conv3_halo_ok(a)) return c10::nullopt;
  mpa::igemm_rows_dgrad(a, 8, nullptr, cur_stream(), true);
  return dx;
}

// dx of two convs that read the same input with the same stride (a residual stage's 3x3/s2
// conv1 and its 1x1/s2 shortcut) in ONE merged stride-phase launch: the shortcut's taps
// are extra K of the phases they hit, so dx is written once, with no accumulate pass.
// Returns None when that launch is not available (the caller runs the two dgrads apart).
c10::optional<Tensor> conv_dgrad_pair(Tensor dy, Tensor w, Tensor wt, int64_t H, int64_t W,
                                      int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                                      Tensor dy2, Tensor w2, Tensor wt2, int64_t ph2,
                                      int64_t pw2, c10::optional<Tensor> accum) {
  CHECK_ACT(dy2);
  CHECK_ACT(w2);
  CHECK_ACT(wt2);
  TORCH_CHECK(dy2.sizes() == dy.sizes(), "conv_dgrad_pair: dy2 must have dy's shape");
  TORCH_CHECK(w2.dim() == 4 && w2.size(0) == w.size(0) && w2.size(3) == w.size(3) &&
                  wt2.numel() == w2.numel(),
              "conv_dgrad_pair: w2 [K][R2][S2][C] with w's K and C, and its transpose");
  if (sh == 1 && sw == 1) return c10::nullopt;
  if (!(wt.defined() && wt.numel() == w.numel())) return c10::nullopt;
  // the two convs' output grids must coincide: P = (H + 2 ph - R) / sh + 1 for both
  const int P2 = (H + 2 * ph2 - w2.size(1)) / sh + 1, Q2 = (W + 2 * pw2 - w2.size(2)) / sw + 1;
  if (P2 != dy.size(1) || Q2 != dy.size(2)) return c10::nullopt;
  DgradSrc2 s2{dy2, w2, wt2, (int)ph2, (int)pw2};
  Tensor dx = conv_dgrad_impl(dy, w, H, W, sh, sw, ph, pw, wt, nullptr, accum, &s2);
  if (!dx.defined()) return c10::nullopt;
  return dx;
}

// fused-reduction dgrad available: LDS-DMA engine, 16-B granular dy (K) and dx (C), and
// the transposed weight (K-contiguous B)
bool conv_bnred_ok(int64_t K, int64_t C) {
  return mpa::igemm_engine() >= 1 && vec_width(K) == 8 && vec_width(C) == 8 && C % 8 == 0;
}

std::vector<Tensor> conv_dgrad_bnred(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t sh,
                                     int64_t sw, int64_t ph, int64_t pw, Tensor wt, Tensor z,
                                     Tensor y, Tensor mean, Tensor rstd,
                                     c10::optional<Tensor> gamma, c10::optional<Tensor> beta) {
  CHECK_ACT(z);
  TORCH_CHECK(conv_bnred_ok(w.size(0), w.size(3)), "conv_dgrad_bnred: unsupported shape/engine");
  TORCH_CHECK(wt.defined() && wt.numel() == w.numel(), "conv_dgrad_bnred: needs the transposed weight");
  BnRed r{z, y, mean, rstd, Tensor(), gamma.value_or(Tensor()), beta.value_or(Tensor())};
  Tensor dx = conv_dgrad_impl(dy, w, H, W, sh, sw, ph, pw, wt, &r);
  TORCH_CHECK(z.sizes() == dx.sizes(), "conv_dgrad_bnred: z must have dx's shape");
  return {dx, r.sums};
}

// DenseNet norm1 -> conv1 (1x1, stride 1) backward hand-off: conv1's dgrad with the ReLU(BN)
// mask, the (sum g, sum g * xhat) reduction and G[..., :Ci] += gamma*rstd * g in ONE GEMM
// epilogue (ep_gacc); no dy tensor is written.  zbuf / G: the block feature buffer and
// block gradient, [..., Ctot] with the same row stride; returns the sums [2 * Ci] for
// bn_defer_step.
Tensor conv_dgrad_bnred_gacc(Tensor dz, Tensor w, Tensor wt, Tensor zbuf, Tensor mean,
                             Tensor rstd, Tensor gamma, Tensor beta, Tensor G) {
  CHECK_ACT(dz);
  CHECK_ACT(w);
  CHECK_ACT(wt);
  CHECK_ACT(zbuf);
  CHECK_CUDA(G);
  CHECK_CONTIG(G);
  const int N = dz.size(0), H = dz.size(1), W = dz.size(2), K = dz.size(3);
  const int Ci = w.size(3);
  TORCH_CHECK(w.size(0) == K && w.size(1) == 1 && w.size(2) == 1 && wt.numel() == w.numel(),
              "conv_dgrad_bnred_gacc: 1x1 weight [K][1][1][Ci] and its transpose");
  TORCH_CHECK(zbuf.is_contiguous() && zbuf.dim() == 4 && zbuf.size(0) == N &&
                  zbuf.size(1) == H && zbuf.size(2) == W && zbuf.size(3) >= Ci,
              "conv_dgrad_bnred_gacc: zbuf must be the contiguous [N, H, W, >= Ci] buffer");
  TORCH_CHECK(G.sizes() == zbuf.sizes(), "conv_dgrad_bnred_gacc: G must have zbuf's shape");
  TORCH_CHECK(G.scalar_type() == torch::kBFloat16 || G.scalar_type() == torch::kFloat32,
              "conv_dgrad_bnred_gacc: G must be bf16 or fp32");
  TORCH_CHECK(conv_bnred_ok(K, Ci) && Ci % 8 == 0 && zbuf.size(3) % 8 == 0,
              "conv_dgrad_bnred_gacc: unsupported shape/engine");
  for (const Tensor* t : {&mean, &rstd, &gamma, &beta}) {
    CHECK_CUDA(*t);
    CHECK_F32(*t);
    TORCH_CHECK(t->numel() >= Ci, "conv_dgrad_bnred_gacc: per-channel vector size");
  }
  const c10::OptionalDeviceGuard g(device_of(dz));
  mpa::IGemmArgs a{};
  a.A = bp(dz); a.aH = H; a.aW = W; a.aC = K;
  a.oH = H; a.oW = W; a.M = N * H * W;
  a.Uh = 1; a.Uw = 1; a.Oh = 0; a.Ow = 0;
  a.T = 1;
  a.taps.dh[0] = 0; a.taps.dw[0] = 0; a.taps.bt[0] = 0;
  a.Ktot = K;
  a.B = bp(wt); a.N = Ci; a.RS = 1; a.ldb = K; a.b_tapmap = 1;
  a.C = G.data_ptr(); a.ldc = (int)zbuf.size(3);
  a.dH = H; a.dW = W; a.Uoh = 1; a.Uow = 1; a.Poh = 0; a.Pow = 0;
  a.ep_z = bp(zbuf);
  a.ep_y = nullptr;
  a.ep_mean = mean.data_ptr<float>();
  a.ep_rstd = rstd.data_ptr<float>();
  a.ep_gamma = gamma.data_ptr<float>();
  a.ep_beta = beta.data_ptr<float>();
  a.ep_gacc = G.data_ptr();
  a.ep_gacc_f32 = G.scalar_type() == torch::kFloat32 ? 1 : 0;
  Tensor sums = torch::empty({2 * Ci}, dz.options().dtype(torch::kFloat32));
  TORCH_CHECK(mpa::dense_gacc_ok(a), "conv_dgrad_bnred_gacc: operand sizes");
  Tensor slab = torch::empty({(int64_t)((a.M + 127) / 128) * 2 * Ci},
                             dz.options().dtype(torch::kFloat32));
  mpa::dense_gacc(a, slab.data_ptr<float>(), sums.data_ptr<float>(), cur_stream());
  return sums;
}

// see mpa::bn_defer_step (bn.hip): fold layer sums into the block's deferred-correction
// table k12 [2, Ctot] and apply the final correction to G's channels [s0, Ci)
// out (optional, bf16 contiguous [..., Ci - s0]): receives the finished slice (the gradient
// its consumer reads) INSTEAD of G's channels [s0, Ci), which nothing reads again - no
// separate slice copy, no write-back
void bn_defer_step(Tensor sums, Tensor gamma, Tensor mean, Tensor rstd, int64_t s0, Tensor k12,
                   Tensor dgamma, Tensor dbeta, Tensor G, Tensor x, c10::optional<Tensor> out) {
  CHECK_CUDA(G);
  CHECK_CONTIG(G);
  CHECK_ACT(x);
  CHECK_F32(k12);
  CHECK_CONTIG(k12);
  const int Ci = sums.numel() / 2;
  const int ctot = x.size(-1);
  const int M = x.numel() / ctot;
  TORCH_CHECK(x.is_contiguous() && G.sizes() == x.sizes() && k12.numel() == 2 * ctot,
              "bn_defer_step: G / x / k12 shapes");
  TORCH_CHECK(s0 >= 0 && s0 < Ci && Ci <= ctot && (Ci - s0) % 8 == 0 &&
                  256 % ((Ci - s0) / 8) == 0,
              "bn_defer_step: slice [s0, Ci) must be 8-channel groups dividing 256");
  for (const Tensor* t : {&gamma, &mean, &rstd}) {
    CHECK_F32(*t);
    TORCH_CHECK(t->numel() >= Ci, "bn_defer_step: per-channel vector size");
  }
  const bool into = out && out->defined() && out->numel() > 0;
  if (into) {
    CHECK_ACT((*out));
    TORCH_CHECK(out->is_contiguous() && out->size(-1) == Ci - s0 && out->numel() / (Ci - s0) == M,
                "bn_defer_step: out must be a contiguous bf16 [..., Ci - s0]");
  }
  const c10::OptionalDeviceGuard g(device_of(x));
  mpa::bn_defer_step(sums.data_ptr<float>(), gamma.data_ptr<float>(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), Ci, (int)s0, M, k12.data_ptr<float>(), ctot,
                     fopt_mut(dgamma), fopt_mut(dbeta), G.data_ptr(),
                     G.scalar_type() == torch::kFloat32, ctot, bp(x), ctot,
                     into ? bpm(*out) : nullptr, cur_stream());
}

static int row_stride(const Tensor& t);  // (below, with the BN helpers)

std::vector<Tensor> bn_bwd_apply(Tensor dy, Tensor x, Tensor y, Tensor mean, Tensor rstd,
                                 Tensor gamma, Tensor dgamma, Tensor dbeta, Tensor sums,
                                 bool want_dx, bool want_g) {
  CHECK_CUDA(dy);
  CHECK_BF16(dy);
  const int lddy = row_stride(dy);  // (a channel window of a wider buffer, or contiguous)
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && sums.numel() == 2 * C && dy.size(-1) == C && lddy % 8 == 0,
              "bn_bwd_apply: shapes");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor dx = want_dx ? torch::empty_like(x) : Tensor();
  Tensor gout = want_g ? torch::empty_like(x) : Tensor();
  mpa::bn_bwd_apply(bp(dy), bp(x), bopt(y), fopt(mean), fopt(rstd), fopt(gamma),
                    fopt_mut(dgamma), fopt_mut(dbeta), M, C, want_dx ? bpm(dx) : nullptr,
                    want_g ? bpm(gout) : nullptr, fopt(sums), cur_stream(), lddy);
  return {dx, gout};
}

void conv_wgrad(Tensor dy, Tensor x, Tensor dw, int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                bool overwrite) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  CHECK_CUDA(dw);
  CHECK_F32(dw);
  CHECK_CONTIG(dw);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  TORCH_CHECK(dw.dim() == 4 && dw.size(0) == K && dw.size(3) == C, "conv_wgrad: dw shape");
  const int R = dw.size(1), S = dw.size(2);
  TORCH_CHECK(dy.size(0) == N, "conv_wgrad: batch mismatch");
  const c10::OptionalDeviceGuard g(device_of(dy));
  mpa::WGradArgs a{};
  a.dy = bp(dy); a.x = bp(x); a.dw = dw.data_ptr<float>();
  a.Kout = K; a.C = C; a.H = H; a.W = W; a.P = P; a.Q = Q; a.R = R; a.S = S;
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.Mpix = N * P * Q;
  a.Ncols = R * S * C;
  a.overwrite = overwrite ? 1 : 0;
  Tensor slab;
  a.slab = alloc_ws(slab, dy, mpa::igemm_wgrad_ws_floats(a.Kout, a.Ncols, a.Mpix));
  mpa::igemm_wgrad(a, vec_width(K), (C % 8 == 0) ? 8 : 1, cur_stream());
}

Tensor act_bwd(Tensor dy, Tensor y, Tensor dbias) {
  CHECK_ACT(dy);
  const int C = dy.size(-1);
  const int M = dy.numel() / C;
  const bool hy = has(y);
  if (!hy && !has(dbias)) return dy;
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor out = hy ? torch::empty_like(dy) : dy;
  Tensor ws;
  float* wsp = nullptr;
  if (has(dbias) && C % 8 == 0) {
    ws = torch::empty({mpa::bn_ws_floats(M, C)}, dy.options().dtype(torch::kFloat32));
    wsp = ws.data_ptr<float>();
  }
  mpa::act_bwd(bp(dy), hy ? bopt(y) : nullptr, fopt_mut(dbias), M, C, hy ? bpm(out) : nullptr,
               wsp, cur_stream());
  return out;
}

// -------------------------------------------------------------------------------- BN
static uint8_t* ymask_ptr(const c10::optional<Tensor>& m, const Tensor& like) {
  if (!m || !m->defined() || m->numel() == 0) return nullptr;
  TORCH_CHECK(m->scalar_type() == torch::kUInt8 && m->is_contiguous() && m->numel() == like.numel() / 8 &&
                  m->device() == like.device(),
              "bn: ReLU mask must be contiguous uint8 [numel / 8] on the activation's device");
  return m->data_ptr<uint8_t>();
}

// mask (optional, uint8 [numel / 8]): receives the ReLU bit mask of y (bit j of byte i =
// element 8 i + j > 0) for bn_bwd(ymask=...), which then never reads y
// channels > 0: x is a wider buffer [..., ldx] and the BN runs on its first `channels`
// channels (a DenseNet block's feature prefix); stats may then be a wider [2, lds] buffer
// whose first `channels` columns hold [mean | var]
// Row stride of a channel-window view [..., C] of a wider NHWC buffer (x[..., a:b]): unit
// channel stride and uniformly strided rows; a contiguous tensor has row stride C
static int row_stride(const Tensor& t) {
  TORCH_CHECK(t.dim() >= 1 && t.stride(-1) == 1, "bn: channels must be contiguous");
  if (t.dim() == 1) return (int)t.size(0);
  const int64_t ld = t.stride(-2);
  int64_t expect = ld * t.size(-2);
  for (int64_t d = t.dim() - 3; d >= 0; --d) {
    TORCH_CHECK(t.size(d) == 1 || t.stride(d) == expect, "bn: rows must be uniformly strided");
    expect *= t.size(d);
  }
  TORCH_CHECK(ld >= t.size(-1), "channel window: row stride below the row width");
  return (int)ld;
}

// x: the BN input - contiguous, or a channel-window view (row stride ldx); channels > 0:
// x is contiguous [..., ldx] and the BN runs on its first `channels` channels
static void bn_prefix(const Tensor& x, int64_t channels, int* C, int* ldx, int* M) {
  CHECK_CUDA(x);
  CHECK_BF16(x);
  if (channels > 0) {
    CHECK_CONTIG(x);
    *ldx = x.size(-1);
    *C = (int)channels;
  } else {
    *ldx = row_stride(x);
    *C = x.size(-1);
  }
  TORCH_CHECK(*C <= *ldx && *C % 8 == 0 && *ldx % 8 == 0,
              "bn: channels must be a multiple of 8 within the row");
  *M = x.numel() / x.size(-1);
}

static std::vector<int64_t> with_last(const Tensor& x, int64_t c) {
  std::vector<int64_t> shape(x.sizes().begin(), x.sizes().end());
  shape.back() = c;
  return shape;
}

// res_affine (optional, fp32 [2, C] = scale | shift): the residual's own BN applied as it
// is read (bn_stats_affine of a deferred BN), so res holds that BN's raw input
std::vector<Tensor> bn_fwd_train(Tensor x, Tensor stats, Tensor gamma, Tensor beta, Tensor rmean,
                                 Tensor rvar, double momentum, double eps, Tensor res, bool relu,
                                 c10::optional<Tensor> counter, c10::optional<Tensor> mask,
                                 int64_t channels, c10::optional<Tensor> res_affine,
                                 c10::optional<Tensor> out) {
  int C, ldx, M;
  bn_prefix(x, channels, &C, &ldx, &M);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor st = stats;
  int lds = C;
  if (has(st)) {
    CHECK_CUDA(st);
    CHECK_F32(st);
    // [2C] contiguous, or a [2, >= C] (view) whose rows hold mean | var: rows stride(0) apart
    if (st.dim() == 2) {
      TORCH_CHECK(st.size(0) == 2 && st.size(1) >= C && st.stride(1) == 1,
                  "bn_fwd_train: stats must be [2, >= C] (mean | var)");
      lds = (int)st.stride(0);
    } else {
      CHECK_CONTIG(st);
      TORCH_CHECK(st.numel() == 2 * C, "bn_fwd_train: stats must be [2, >= C] (mean | var)");
    }
  } else {
    TORCH_CHECK(ldx == C, "bn_fwd_train: a channel prefix needs precomputed stats");
    st = torch::empty({2, C}, x.options().dtype(torch::kFloat32));
    Tensor ws = torch::empty({mpa::bn_ws_floats(M, C)}, x.options().dtype(torch::kFloat32));
    mpa::bn_stats(bp(x), M, C, fopt(rmean), st.data_ptr<float>(), ws.data_ptr<float>(),
                  cur_stream());
  }
  // out (optional): write y into this bf16 channel window of a wider NHWC buffer (a block
  // output at the branch's channel offset: concat without a copy)
  const bool into = out && out->defined() && out->numel() > 0;
  int ldy = C;
  Tensor y;
  if (into) {
    CHECK_CUDA(*out);
    CHECK_BF16(*out);
    TORCH_CHECK(out->sizes() == c10::IntArrayRef(with_last(x, C)) && !has(res) &&
                    !(mask && mask->defined() && mask->numel()),
                "bn_fwd_train: out must have the output's shape (no residual / mask)");
    ldy = row_stride(*out);
    TORCH_CHECK(ldy % 8 == 0, "bn_fwd_train: out row stride must be a multiple of 8");
    y = *out;
  } else {
    y = torch::empty(with_last(x, C), x.options());
  }
  if (has(res)) TORCH_CHECK(res.numel() == y.numel(), "bn_fwd_train: residual shape");
  const float* raff = nullptr;
  if (res_affine && res_affine->defined() && res_affine->numel() > 0) {
    TORCH_CHECK(has(res) && res_affine->numel() == 2 * C, "bn_fwd_train: res_affine [2, C]");
    raff = fopt(*res_affine);
  }
  Tensor mean = torch::empty({C}, x.options().dtype(torch::kFloat32));
  Tensor rstd = torch::empty({C}, x.options().dtype(torch::kFloat32));
  mpa::bn_fwd_train(bp(x), st.data_ptr<float>(), fopt(gamma), fopt(beta), fopt_mut(rmean), fopt_mut(rvar),
                    (float)momentum, (float)eps, bopt(res), relu ? 1 : 0, M, C, bpm(y),
                    mean.data_ptr<float>(), rstd.data_ptr<float>(),
                    (counter && counter->defined() && counter->numel() == 1)
                        ? counter->data_ptr<int64_t>() : nullptr,
                    cur_stream(), into ? nullptr : ymask_ptr(mask, y), ldx, lds, raff, ldy);
  return {y, mean, rstd};
}

// a train-mode BN's statistics half (see mpa::bn_stats_affine): returns mean, rstd and the
// [2, C] affine its consumer applies (bn_fwd_train(res_affine=)).  x is the BN input
// (unused here: the statistics are finalized already; the CPU oracle recomputes them)
std::vector<Tensor> bn_stats_affine(Tensor x, Tensor stats, Tensor gamma, Tensor beta,
                                    Tensor rmean, Tensor rvar, double momentum, double eps,
                                    c10::optional<Tensor> counter) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(has(stats) && stats.numel() == 2 * C, "bn_stats_affine: stats [2, C]");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor mean = torch::empty({C}, x.options().dtype(torch::kFloat32));
  Tensor rstd = torch::empty({C}, x.options().dtype(torch::kFloat32));
  Tensor aff = torch::empty({2, C}, x.options().dtype(torch::kFloat32));
  mpa::bn_stats_affine(fopt(stats), fopt(gamma), fopt(beta), fopt_mut(rmean), fopt_mut(rvar),
                       (float)momentum, (float)eps, M, C, mean.data_ptr<float>(),
                       rstd.data_ptr<float>(), aff.data_ptr<float>(),
                       (counter && counter->defined() && counter->numel() == 1)
                           ? counter->data_ptr<int64_t>() : nullptr,
                       cur_stream());
  return {mean, rstd, aff};
}

// avgpool2x2/s2(relu(bn(z))) with the BN as its [2, C] affine (bn_stats_affine)
Tensor bn_relu_avgpool2_fwd(Tensor z, Tensor aff) {
  CHECK_ACT(z);
  TORCH_CHECK(z.dim() == 4 && z.size(1) % 2 == 0 && z.size(2) % 2 == 0 && z.size(3) % 8 == 0,
              "bn_relu_avgpool2_fwd: z [N, H, W, C] with even H, W and C % 8 == 0");
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  TORCH_CHECK(aff.numel() == 2 * C, "bn_relu_avgpool2_fwd: aff [2, C]");
  const c10::OptionalDeviceGuard g(device_of(z));
  Tensor y = empty_like_shape(z, {N, H / 2, W / 2, C}, torch::kBFloat16);
  mpa::bn_relu_avgpool2_fwd(bp(z), fopt(aff), N, H, W, C, bpm(y), cur_stream());
  return y;
}

// per-channel batch statistics [2, C] = [mean | biased var] of x [..., C] (shift: optional
// per-channel value subtracted before the sums, e.g. the running mean, for precision)
Tensor bn_stats(Tensor x, Tensor shift) {
  CHECK_ACT(x);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && M > 0, "bn_stats: channels must be a multiple of 8");
  if (has(shift)) TORCH_CHECK(shift.numel() == C && shift.is_contiguous(), "bn_stats: shift");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor st = torch::empty({2, C}, x.options().dtype(torch::kFloat32));
  Tensor ws = torch::empty({mpa::bn_ws_floats(M, C)}, x.options().dtype(torch::kFloat32));
  mpa::bn_stats(bp(x), M, C, fopt(shift), st.data_ptr<float>(), ws.data_ptr<float>(),
                cur_stream());
  return st;
}

Tensor bn_fwd_eval(Tensor x, Tensor gamma, Tensor beta, Tensor rmean, Tensor rvar, double eps,
                   Tensor res, bool relu, int64_t channels) {
  int C, ldx, M;
  bn_prefix(x, channels, &C, &ldx, &M);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = torch::empty(with_last(x, C), x.options());
  if (has(res)) TORCH_CHECK(res.numel() == y.numel(), "bn_fwd_eval: residual shape");
  mpa::bn_fwd_eval(bp(x), fopt(gamma), fopt(beta), fopt(rmean), fopt(rvar), (float)eps,
                   bopt(res), relu ? 1 : 0, M, C, bpm(y), cur_stream(), ldx);
  return y;
}

// x may be wider than dy (a channel prefix: ldx = x.size(-1)); gacc (fp32 [..., ldg]): dx is
// ADDED into its first C channels instead of being returned (a dense block's accumulator)
std::vector<Tensor> bn_bwd(Tensor dy, Tensor x, Tensor y, Tensor mean, Tensor rstd, Tensor gamma,
                           Tensor dgamma, Tensor dbeta, bool want_dx, bool want_g,
                           c10::optional<Tensor> zmask_beta, c10::optional<Tensor> ymask,
                           c10::optional<Tensor> gacc, c10::optional<Tensor> dx_out) {
  // dy: contiguous or a channel window of a wider buffer (a branch's slice of a block
  // output gradient), row stride lddy
  CHECK_CUDA(dy);
  CHECK_BF16(dy);
  const int lddy = row_stride(dy);
  CHECK_CUDA(x);
  CHECK_BF16(x);
  const int C = dy.size(-1);
  TORCH_CHECK(lddy % 8 == 0, "bn_bwd: dy row stride must be a multiple of 8");
  // x: same channels as dy (contiguous or a channel-window view), or a contiguous wider
  // buffer whose first C channels are the BN input (a DenseNet block prefix)
  const int ldx = (x.size(-1) > C) ? (x.is_contiguous() ? (int)x.size(-1) : -1) : row_stride(x);
  TORCH_CHECK(ldx > 0, "bn_bwd: a wider x must be contiguous");
  const int M = dy.numel() / C;
  TORCH_CHECK(C % 8 == 0 && ldx % 8 == 0 && ldx >= C, "bn: channels must be a multiple of 8");
  TORCH_CHECK(x.numel() / x.size(-1) == M && x.dim() == dy.dim(), "bn_bwd: dy/x shape mismatch");
  const bool acc = gacc && gacc->defined() && gacc->numel() > 0;
  if (acc) {
    CHECK_CUDA(*gacc);
    CHECK_CONTIG(*gacc);
    TORCH_CHECK(gacc->scalar_type() == torch::kFloat32 || gacc->scalar_type() == torch::kBFloat16,
                "bn_bwd: gradient accumulator must be fp32 or bf16");
    TORCH_CHECK(gacc->numel() / gacc->size(-1) == M && gacc->size(-1) >= C &&
                    gacc->size(-1) % 8 == 0 && !want_g,
                "bn_bwd: gradient accumulator must be fp32 [..., >= C] with dy's rows");
  }
  // dx_out: write dx into this (contiguous or channel-window) bf16 view of dy's shape
  const bool into = dx_out && dx_out->defined() && dx_out->numel() > 0;
  int lddx = C;
  if (into) {
    CHECK_CUDA(*dx_out);
    CHECK_BF16(*dx_out);
    TORCH_CHECK(dx_out->sizes() == dy.sizes() && !acc, "bn_bwd: dx_out must have dy's shape");
    lddx = row_stride(*dx_out);
    TORCH_CHECK(lddx % 8 == 0, "bn_bwd: dx_out row stride must be a multiple of 8");
  }
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor dx = (want_dx && !acc)
                  ? (into ? *dx_out : torch::empty(dy.sizes(), dy.options()))
                  : Tensor();
  Tensor gout = want_g ? torch::empty(dy.sizes(), dy.options()) : Tensor();
  Tensor ws = torch::empty({mpa::bn_ws_floats(M, C)}, x.options().dtype(torch::kFloat32));
  const Tensor zb = (zmask_beta && zmask_beta->defined()) ? *zmask_beta : Tensor();
  if (has(zb)) TORCH_CHECK(zb.numel() == C, "bn_bwd: zmask beta size");
  mpa::bn_bwd(bp(dy), bp(x), bopt(y), fopt(mean), fopt(rstd), fopt(gamma), fopt_mut(dgamma),
              fopt_mut(dbeta), M, C, (want_dx && !acc) ? bpm(dx) : nullptr,
              want_g ? bpm(gout) : nullptr, ws.data_ptr<float>(), cur_stream(), fopt(zb),
              ymask_ptr(ymask, dy), ldx, acc ? (float*)gacc->data_ptr() : nullptr,
              acc ? (int)gacc->size(-1) : 0, lddx,
              acc && gacc->scalar_type() == torch::kBFloat16, lddy);
  return {dx, gout};
}

// backward of relu(bn(x) + bn2(x2)) with both BNs in train mode (ResNet bn2 + the deferred
// downsample BN): returns [dx, dx2]; both BNs' dgamma/dbeta receive their sums
std::vector<Tensor> bn_bwd_pair(Tensor dy, Tensor x, Tensor ymask, Tensor mean, Tensor rstd,
                                Tensor gamma, Tensor dgamma, Tensor dbeta, Tensor x2, Tensor mean2,
                                Tensor rstd2, Tensor gamma2, Tensor dgamma2, Tensor dbeta2) {
  CHECK_CUDA(dy);
  CHECK_BF16(dy);
  dy = dy.contiguous();
  CHECK_ACT(x);
  CHECK_ACT(x2);
  const int C = dy.size(-1);
  const int M = dy.numel() / C;
  TORCH_CHECK(C % 8 == 0, "bn_bwd_pair: channels must be a multiple of 8");
  TORCH_CHECK(x.sizes() == dy.sizes() && x2.sizes() == dy.sizes(), "bn_bwd_pair: shape mismatch");
  for (const Tensor* t : {&mean, &rstd, &gamma, &mean2, &rstd2, &gamma2}) {
    CHECK_CUDA(*t);
    CHECK_F32(*t);
    TORCH_CHECK(t->numel() == C, "bn_bwd_pair: per-channel vector size");
  }
  const uint8_t* ym = ymask_ptr(ymask, dy);
  TORCH_CHECK(ym, "bn_bwd_pair: needs the forward's ReLU bit mask");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor dx = torch::empty(dy.sizes(), dy.options());
  Tensor dx2 = torch::empty(dy.sizes(), dy.options());
  Tensor ws = torch::empty({mpa::bn_pair_ws_floats(M, C)}, x.options().dtype(torch::kFloat32));
  mpa::bn_bwd_pair(bp(dy), bp(x), bp(x2), ym, fopt(mean), fopt(rstd), fopt(gamma), fopt(mean2),
                   fopt(rstd2), fopt(gamma2), fopt_mut(dgamma), fopt_mut(dbeta), fopt_mut(dgamma2),
                   fopt_mut(dbeta2), M, C, bpm(dx), bpm(dx2), ws.data_ptr<float>(), cur_stream());
  return {dx, dx2};
}

Tensor relu_fwd(Tensor x) {
  CHECK_ACT(x);
  TORCH_CHECK(x.numel() % 8 == 0, "relu: numel must be a multiple of 8");
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = torch::empty_like(x);
  mpa::relu_fwd(bp(x), x.numel(), bpm(y), cur_stream());
  return y;
}

// ------------------------------------------------------------------------------ pools
int pool_out(int H, int k, int s, int p, bool ceil) {
  int o;
  if (ceil) {
    o = (H + 2 * p - k + s - 1) / s + 1;
    if ((o - 1) * s >= H + p) --o;
  } else {
    o = (H + 2 * p - k) / s + 1;
  }
  return o;
}

std::vector<Tensor> maxpool_fwd(Tensor x, int64_t kh, int64_t kw, int64_t sh, int64_t sw,
                                int64_t ph, int64_t pw, bool ceil) {
  CHECK_ACT(x);
  TORCH_CHECK(kh * kw <= 256, "maxpool: window too large for uint8 argmax");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = pool_out(H, kh, sh, ph, ceil), Q = pool_out(W, kw, sw, pw, ceil);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = empty_like_shape(x, {N, P, Q, C}, torch::kBFloat16);
  Tensor idx = empty_like_shape(x, {N, P, Q, C}, torch::kUInt8);
  if (mpa::maxpool2_ok(N, H, W, C, kh, kw, sh, sw, ph, pw))
    mpa::maxpool2_fwd(bp(x), N, H, W, C, bpm(y), idx.data_ptr<uint8_t>(), cur_stream());
  else
    mpa::maxpool_fwd(bp(x), N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw, bpm(y),
                     idx.data_ptr<uint8_t>(), cur_stream());
  return {y, idx};
}

Tensor maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh,
                   int64_t sw, int64_t ph, int64_t pw, bool ceil) {
  CHECK_ACT(dy);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  (void)ceil;
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = empty_like_shape(dy, {N, H, W, C}, torch::kBFloat16);
  if (mpa::maxpool2_ok(N, H, W, C, kh, kw, sh, sw, ph, pw))
    mpa::maxpool2_bwd(bp(dy), idx.data_ptr<uint8_t>(), nullptr, N, H, W, C, bpm(dx), nullptr,
                      nullptr, cur_stream());
  else
    mpa::maxpool_bwd(bp(dy), idx.data_ptr<uint8_t>(), N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw,
                     bpm(dx), cur_stream());
  return dx;
}

// max-pool backward whose input is a ReLU output handed over by its producer (Fn.BNLink):
// the gradient routes only where the pooled value is > 0, and the per-channel sum of what
// is routed (the producer's bias gradient) comes back with it.  None: not a 2x2/s2 pool.
c10::optional<std::vector<Tensor>> maxpool_bwd_relu(Tensor dy, Tensor idx, Tensor y, int64_t H,
                                                    int64_t W, int64_t kh, int64_t kw,
                                                    int64_t sh, int64_t sw, int64_t ph,
                                                    int64_t pw) {
  CHECK_ACT(dy);
  CHECK_ACT(y);
  const int N = dy.size(0), C = dy.size(3);
  if (!mpa::maxpool2_ok(N, H, W, C, kh, kw, sh, sw, ph, pw)) return c10::nullopt;
  TORCH_CHECK(y.sizes() == dy.sizes() && idx.sizes() == dy.sizes() &&
                  idx.scalar_type() == torch::kUInt8 && idx.is_contiguous(),
              "maxpool_bwd_relu: pooled tensors");
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = empty_like_shape(dy, {N, H, W, C}, torch::kBFloat16);
  Tensor sums = torch::empty({C}, dy.options().dtype(torch::kFloat32));
  Tensor ws = torch::empty({mpa::maxpool2_ws_floats(N, H, W, C)},
                           dy.options().dtype(torch::kFloat32));
  mpa::maxpool2_bwd(bp(dy), idx.data_ptr<uint8_t>(), bp(y), N, H, W, C, bpm(dx),
                    sums.data_ptr<float>(), ws.data_ptr<float>(), cur_stream());
  return std::vector<Tensor>{dx, sums};
}

// conv -> BN -> ReLU -> max-pool stem: z is the raw conv output, stats its (shifted)
// epilogue statistics; returns the pooled activation, argmax, batch mean and rstd
std::vector<Tensor> bn_relu_maxpool_fwd(Tensor z, Tensor stats, Tensor gamma, Tensor beta,
                                        Tensor rmean, Tensor rvar, double momentum, double eps,
                                        int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                                        int64_t pw, bool ceil, c10::optional<Tensor> counter,
                                        c10::optional<Tensor> zsel_out) {
  CHECK_ACT(z);
  TORCH_CHECK(kh * kw <= 256, "bn_relu_maxpool: window too large for uint8 argmax");
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  TORCH_CHECK(C % 8 == 0 && stats.numel() == 2 * C, "bn_relu_maxpool: shapes");
  const int P = pool_out(H, kh, sh, ph, ceil), Q = pool_out(W, kw, sw, pw, ceil);
  const c10::OptionalDeviceGuard g(device_of(z));
  Tensor y = empty_like_shape(z, {N, P, Q, C}, torch::kBFloat16);
  Tensor idx = empty_like_shape(z, {N, P, Q, C}, torch::kUInt8);
  Tensor mean = torch::empty({C}, z.options().dtype(torch::kFloat32));
  Tensor rstd = torch::empty({C}, z.options().dtype(torch::kFloat32));
  mpa::bf16_raw* zsel = nullptr;
  if (zsel_out && zsel_out->defined()) {
    CHECK_ACT(*zsel_out);
    TORCH_CHECK(zsel_out->sizes() == y.sizes(), "bn_relu_maxpool: zsel_out must be [N,P,Q,C]");
    zsel = bpm(*zsel_out);
  }
  mpa::bn_relu_maxpool_fwd(bp(z), fopt(stats), fopt(gamma), fopt(beta), fopt_mut(rmean),
                           fopt_mut(rvar), (float)momentum, (float)eps, N, H, W, C, P, Q, kh, kw,
                           sh, sw, ph, pw, bpm(y), idx.data_ptr<uint8_t>(), mean.data_ptr<float>(),
                           rstd.data_ptr<float>(),
                           (counter && counter->defined() && counter->numel() == 1)
                               ? counter->data_ptr<int64_t>() : nullptr,
                           cur_stream(), zsel);
  return {y, idx, mean, rstd};
}

Tensor maxpool_bn_bwd(Tensor dp, Tensor idx, Tensor z, Tensor mean, Tensor rstd, Tensor gamma,
                      Tensor beta, Tensor dgamma, Tensor dbeta, int64_t kh, int64_t kw, int64_t sh,
                      int64_t sw, int64_t ph, int64_t pw, c10::optional<Tensor> zsel) {
  CHECK_ACT(dp);
  CHECK_ACT(z);
  const mpa::bf16_raw* zs = nullptr;
  if (zsel && zsel->defined()) {
    CHECK_ACT(*zsel);
    TORCH_CHECK(zsel->sizes() == dp.sizes(), "maxpool_bn_bwd: zsel must match dp");
    zs = bp(*zsel);
  }
  const int N = z.size(0), H = z.size(1), W = z.size(2), C = z.size(3);
  const int P = dp.size(1), Q = dp.size(2);
  TORCH_CHECK(dp.size(0) == N && dp.size(3) == C && idx.sizes() == dp.sizes() && C % 8 == 0,
              "maxpool_bn_bwd: shapes");
  const c10::OptionalDeviceGuard g(device_of(z));
  Tensor dz = torch::empty_like(z);
  Tensor ws = torch::empty({mpa::maxpool_bn_ws_floats(N * H * W, C)},
                           z.options().dtype(torch::kFloat32));
  mpa::maxpool_bn_bwd(bp(dp), idx.data_ptr<uint8_t>(), bp(z), fopt(mean), fopt(rstd), fopt(gamma),
                      fopt(beta), fopt_mut(dgamma), fopt_mut(dbeta), N, H, W, C, P, Q, kh, kw, sh,
                      sw, ph, pw, bpm(dz), ws.data_ptr<float>(), cur_stream(), zs);
  return dz;
}

// ---- fused stem backward (round 6): pooled-only sums, then the weight gradient that forms
// dz in its operand staging (conv_stem.hip stem_wgrad_kernel<KS, true>)
Tensor maxpool_bn_bwd_sums(Tensor dp, Tensor zsel, Tensor mean, Tensor rstd, Tensor gamma,
                           Tensor beta, Tensor dgamma, Tensor dbeta) {
  CHECK_ACT(dp);
  CHECK_ACT(zsel);
  TORCH_CHECK(zsel.sizes() == dp.sizes() && dp.dim() == 4 && dp.size(3) % 8 == 0,
              "maxpool_bn_bwd_sums: shapes");
  const int C = dp.size(3);
  const int MP = dp.numel() / C;
  const c10::OptionalDeviceGuard g(device_of(dp));
  Tensor ws = torch::empty({mpa::maxpool_bn_ws_floats(MP, C)}, dp.options().dtype(torch::kFloat32));
  mpa::maxpool_bn_bwd_sums(bp(dp), bp(zsel), fopt(mean), fopt(rstd), fopt(gamma), fopt(beta),
                           fopt_mut(dgamma), fopt_mut(dbeta), MP, C, ws.data_ptr<float>(),
                           cur_stream());
  return ws.narrow(0, 0, 2 * C);
}

static mpa::WGradArgs stem_pool_args(const Tensor& z, const Tensor& x, const Tensor& dw,
                                     int64_t sh, int64_t sw, int64_t ph, int64_t pw,
                                     bool overwrite) {
  mpa::WGradArgs a{};
  a.dy = bp(z); a.x = bp(x); a.dw = dw.data_ptr<float>();
  a.Kout = z.size(3); a.C = x.size(3); a.H = x.size(1); a.W = x.size(2);
  a.P = z.size(1); a.Q = z.size(2); a.R = dw.size(1); a.S = dw.size(2);
  a.sh = sh; a.sw = sw; a.ph = ph; a.pw = pw;
  a.Mpix = z.size(0) * a.P * a.Q;
  a.Ncols = a.R * a.S * a.C;
  a.overwrite = overwrite ? 1 : 0;
  return a;
}

static mpa::StemPoolArgs stem_pool_q(const Tensor& dp, const Tensor& idx, const Tensor& mean,
                                     const Tensor& rstd, const Tensor& gamma, const Tensor& beta,
                                     const Tensor& sums) {
  mpa::StemPoolArgs q{};
  q.dp = bp(dp); q.idx = idx.data_ptr<uint8_t>();
  q.mean = fopt(mean); q.rstd = fopt(rstd); q.gamma = fopt(gamma); q.beta = fopt(beta);
  q.sums = fopt(sums);
  q.PP = dp.size(1); q.PQ = dp.size(2);
  return q;
}

bool stem_pool_wgrad_ok(Tensor dp, Tensor idx, Tensor z, Tensor x, Tensor dw, int64_t sh,
                        int64_t sw, int64_t ph, int64_t pw) {
  if (!dp.is_cuda() || !z.is_cuda() || !x.is_cuda() || dp.dim() != 4 || z.dim() != 4 ||
      x.dim() != 4 || dw.dim() != 4 || !dp.is_contiguous() || !z.is_contiguous() ||
      !x.is_contiguous() || !idx.is_contiguous() || idx.sizes() != dp.sizes() ||
      dp.size(0) != z.size(0) || x.size(0) != z.size(0) || dp.size(3) != z.size(3) ||
      dw.size(0) != z.size(3) || dw.size(3) != x.size(3) ||
      dp.scalar_type() != torch::kBFloat16 || z.scalar_type() != torch::kBFloat16 ||
      x.scalar_type() != torch::kBFloat16 || dw.scalar_type() != torch::kFloat32)
    return false;
  mpa::WGradArgs a = stem_pool_args(z, x, dw, sh, sw, ph, pw, false);
  a.slab = reinterpret_cast<float*>(16);  // (checked for presence and alignment only)
  mpa::StemPoolArgs q{};
  q.dp = bp(dp); q.idx = idx.data_ptr<uint8_t>();
  q.mean = q.rstd = q.gamma = q.beta = q.sums = reinterpret_cast<const float*>(16);
  q.PP = dp.size(1); q.PQ = dp.size(2);
  return mpa::igemm_engine() >= 1 && mpa::stem_pool_wgrad_ok(a, q);
}

void stem_pool_wgrad(Tensor dp, Tensor idx, Tensor z, Tensor mean, Tensor rstd, Tensor gamma,
                     Tensor beta, Tensor sums, Tensor x, Tensor dw, int64_t sh, int64_t sw,
                     int64_t ph, int64_t pw, bool overwrite) {
  CHECK_ACT(dp);
  CHECK_ACT(z);
  CHECK_ACT(x);
  CHECK_F32(dw);
  CHECK_CONTIG(dw);
  const c10::OptionalDeviceGuard g(device_of(z));
  mpa::WGradArgs a = stem_pool_args(z, x, dw, sh, sw, ph, pw, overwrite);
  Tensor slab;
  a.slab = alloc_ws(slab, z, mpa::igemm_wgrad_ws_floats(a.Kout, a.Ncols, a.Mpix));
  const mpa::StemPoolArgs q = stem_pool_q(dp, idx, mean, rstd, gamma, beta, sums);
  TORCH_CHECK(mpa::stem_pool_wgrad_ok(a, q), "stem_pool_wgrad: unsupported geometry");
  mpa::igemm_stem_pool_wgrad(a, q, cur_stream());
}

// x: contiguous NHWC or a channel-window view of a wider buffer (pixel stride ldx)
Tensor avgpool_fwd(Tensor x, int64_t kh, int64_t kw, int64_t sh, int64_t sw, int64_t ph,
                   int64_t pw, bool ceil, bool cip) {
  CHECK_CUDA(x);
  CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 4, "avgpool: NHWC input");
  const int ldx = row_stride(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(ldx == C || (C % 8 == 0 && ldx % 8 == 0), "avgpool: window must be 16-B aligned");
  const int P = pool_out(H, kh, sh, ph, ceil), Q = pool_out(W, kw, sw, pw, ceil);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = empty_like_shape(x, {N, P, Q, C}, torch::kBFloat16);
  mpa::avgpool_fwd(bp(x), N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw, cip ? 1 : 0, bpm(y),
                   cur_stream(), ldx);
  return y;
}

// dx_out (optional): write dx into this [N, H, W, C] view (a channel window of a wider
// buffer) instead of a new tensor
Tensor avgpool_bwd(Tensor dy, int64_t H, int64_t W, int64_t kh, int64_t kw, int64_t sh,
                   int64_t sw, int64_t ph, int64_t pw, bool ceil, bool cip,
                   c10::optional<Tensor> dx_out) {
  CHECK_ACT(dy);
  (void)ceil;
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx;
  int ldo = C;
  if (dx_out && dx_out->defined() && dx_out->numel() > 0) {
    dx = *dx_out;
    CHECK_CUDA(dx);
    CHECK_BF16(dx);
    TORCH_CHECK(dx.dim() == 4 && dx.size(0) == N && dx.size(1) == H && dx.size(2) == W &&
                    dx.size(3) == C, "avgpool_bwd: dx_out shape");
    ldo = row_stride(dx);
    TORCH_CHECK(ldo == C || (C % 8 == 0 && ldo % 8 == 0), "avgpool: window must be 16-B aligned");
  } else {
    dx = empty_like_shape(dy, {N, H, W, C}, torch::kBFloat16);
  }
  mpa::avgpool_bwd(bp(dy), N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw, cip ? 1 : 0, bpm(dx),
                   cur_stream(), ldo);
  return dx;
}

Tensor adaptive_avgpool_fwd(Tensor x, int64_t P, int64_t Q) {
  CHECK_ACT(x);
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = empty_like_shape(x, {N, P, Q, C}, torch::kBFloat16);
  mpa::adaptive_avgpool_fwd(bp(x), N, H, W, C, P, Q, bpm(y), cur_stream());
  return y;
}

Tensor adaptive_avgpool_bwd(Tensor dy, int64_t H, int64_t W) {
  CHECK_ACT(dy);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = empty_like_shape(dy, {N, H, W, C}, torch::kBFloat16);
  mpa::adaptive_avgpool_bwd(bp(dy), N, H, W, C, P, Q, bpm(dx), cur_stream());
  return dx;
}

// ----------------------------------------------------------------------------- linear
Tensor linear_fwd(Tensor x, Tensor w, Tensor bias, bool relu) {
  CHECK_ACT(x);
  CHECK_ACT(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "linear_fwd: shapes");
  const int B = x.size(0), Cin = x.size(1), Cout = w.size(0);
  const c10::OptionalDeviceGuard g(device_of(x));
  Tensor y = empty_like_shape(x, {B, Cout}, torch::kBFloat16);
  mpa::IGemmArgs a{};
  a.A = bp(x); a.aH = 1; a.aW = 1; a.aC = Cin;
  a.oH = 1; a.oW = 1; a.M = B;
  a.Uh = 1; a.Uw = 1; a.Oh = 0; a.Ow = 0;
  a.T = 1; a.taps.dh[0] = 0; a.taps.dw[0] = 0; a.taps.bt[0] = 0;
  a.Ktot = Cin;
  a.B = bp(w); a.N = Cout; a.RS = 1; a.ldb = Cin;
  a.C = y.data_ptr(); a.ldc = Cout;
  a.dH = 1; a.dW = 1; a.Uoh = 1; a.Uow = 1; a.Poh = 0; a.Pow = 0;
  a.bias = fopt(bias); a.stats = nullptr; a.relu = relu ? 1 : 0;
  Tensor ws;
  float* wsp = alloc_ws(ws, x, mpa::igemm_ws_floats(a.M, a.N, a.Ktot));
  mpa::igemm_rows(a, vec_width(Cin), wsp, nullptr, cur_stream());
  return y;
}

Tensor linear_dgrad(Tensor dy, Tensor w, c10::optional<Tensor> wt_opt) {
  CHECK_ACT(dy);
  CHECK_ACT(w);
  const int B = dy.size(0), Cout = dy.size(1), Cin = w.size(1);
  TORCH_CHECK(w.size(0) == Cout, "linear_dgrad: shapes");
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = empty_like_shape(dy, {B, Cin}, torch::kBFloat16);
  mpa::IGemmArgs a{};
  a.A = bp(dy); a.aH = 1; a.aW = 1; a.aC = Cout;
  a.oH = 1; a.oW = 1; a.M = B;
  a.Uh = 1; a.Uw = 1; a.Oh = 0; a.Ow = 0;
  a.T = 1; a.taps.dh[0] = 0; a.taps.dw[0] = 0; a.taps.bt[0] = 0;
  a.Ktot = Cout;
  a.B = bp(w); a.N = Cin; a.RS = 1; a.ldb = Cin;
  const int vw = std::min(vec_width(Cout), vec_width(Cin));
  const bool bkc = wt_opt && wt_opt->defined() && wt_opt->numel() == w.numel() && vw == 8;
  if (bkc) {  // transposed weight [Cin][Cout]: B K-contiguous
    CHECK_ACT((*wt_opt));
    a.B = bp(*wt_opt);
    a.ldb = Cout;
  }
  a.C = dx.data_ptr(); a.ldc = Cin;
  a.dH = 1; a.dW = 1; a.Uoh = 1; a.Uow = 1; a.Poh = 0; a.Pow = 0;
  Tensor ws;
  float* wsp = alloc_ws(ws, dy, mpa::igemm_ws_floats(a.M, a.N, a.Ktot));
  mpa::igemm_rows_dgrad(a, vw, wsp, cur_stream(), bkc);
  return dx;
}

void linear_wgrad(Tensor dy, Tensor x, Tensor dw, bool overwrite) {
  CHECK_ACT(dy);
  CHECK_ACT(x);
  CHECK_CUDA(dw);
  CHECK_F32(dw);
  const int B = dy.size(0), Cout = dy.size(1), Cin = x.size(1);
  TORCH_CHECK(dw.size(0) == Cout && dw.size(1) == Cin, "linear_wgrad: dw shape");
  const c10::OptionalDeviceGuard g(device_of(dy));
  mpa::WGradArgs a{};
  a.dy = bp(dy); a.x = bp(x); a.dw = dw.data_ptr<float>();
  a.Kout = Cout; a.C = Cin; a.H = 1; a.W = 1; a.P = 1; a.Q = 1; a.R = 1; a.S = 1;
  a.sh = 1; a.sw = 1; a.ph = 0; a.pw = 0;
  a.Mpix = B; a.Ncols = Cin;
  a.overwrite = overwrite ? 1 : 0;
  Tensor slab;
  a.slab = alloc_ws(slab, dy, mpa::igemm_wgrad_ws_floats(a.Kout, a.Ncols, a.Mpix));
  mpa::igemm_wgrad(a, vec_width(Cout), (Cin % 8 == 0) ? 8 : 1, cur_stream());
}

void comm_emulator(int64_t blocks, int64_t threads, int64_t lds_bytes, double us, Tensor sink) {
  CHECK_CUDA(sink);
  CHECK_F32(sink);
  TORCH_CHECK(sink.numel() >= blocks && threads <= 512 && lds_bytes <= 160 * 1024,
              "comm_emulator: args");
  const c10::OptionalDeviceGuard g(device_of(sink));
  mpa::comm_emulator(blocks, threads, lds_bytes, us, sink.data_ptr<float>(), cur_stream());
}

void atomic_latency(int64_t blocks, int64_t iters, int64_t mode, Tensor q) {
  CHECK_CUDA(q);
  TORCH_CHECK(q.scalar_type() == at::kInt && q.numel() >= std::max<int64_t>(blocks * 32, 1 << 20) + 1,
              "atomic_latency: q int32 with >= max(32 blocks, 2^20) + 1 words");
  const c10::OptionalDeviceGuard g(device_of(q));
  mpa::atomic_latency(blocks, iters, mode, q.data_ptr<int>(), cur_stream());
}

// ------------------------------------------------------------------------ loss / acc
// logits: [B][NC] bf16 with unit column stride; rows may be padded (stride(0) >= NC, a
// view of a classifier's padded output)
static int logits_ld(const Tensor& logits) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == torch::kBFloat16 && logits.dim() == 2,
              "logits must be a 2-D bf16 GPU tensor");
  TORCH_CHECK(logits.stride(1) == 1 && logits.stride(0) >= logits.size(1),
              "logits: rows must be unit-stride");
  return (int)logits.stride(0);
}

std::vector<Tensor> ce_fwd(Tensor logits, Tensor labels) {
  const int ld = logits_ld(logits);
  CHECK_CUDA(labels);
  TORCH_CHECK(labels.scalar_type() == torch::kInt64, "labels must be int64");
  const int B = logits.size(0), NC = logits.size(1);
  const c10::OptionalDeviceGuard g(device_of(logits));
  Tensor buf = torch::empty({1 + B}, logits.options().dtype(torch::kFloat32));
  Tensor lse = torch::empty({B}, logits.options().dtype(torch::kFloat32));
  mpa::ce_fwd(bp(logits), labels.contiguous().data_ptr<int64_t>(), B, NC, ld,
              buf.data_ptr<float>(), lse.data_ptr<float>(), cur_stream());
  return {buf.narrow(0, 0, 1), lse};
}

// returns dlogits with the same row stride as logits (a view of a zero-padded buffer when
// the logits are padded)
// out[0] = (or +=, accumulate) weight * mean CE and acc[0] += the same (acc optional);
// returns the per-row log-sum-exp for the backward
Tensor ce_fwd_weighted(Tensor logits, Tensor labels, Tensor out, Tensor acc, double weight,
                       bool accumulate) {
  const int ld = logits_ld(logits);
  CHECK_CUDA(labels);
  TORCH_CHECK(labels.scalar_type() == torch::kInt64, "labels must be int64");
  CHECK_CUDA(out);
  CHECK_F32(out);
  TORCH_CHECK(out.numel() >= 1, "ce_fwd_weighted: out must hold one float");
  const int B = logits.size(0), NC = logits.size(1);
  TORCH_CHECK(labels.numel() == B, "ce_fwd_weighted: one label per row");
  const c10::OptionalDeviceGuard g(device_of(logits));
  Tensor rows = torch::empty({B}, logits.options().dtype(torch::kFloat32));
  Tensor lse = torch::empty({B}, logits.options().dtype(torch::kFloat32));
  mpa::ce_fwd_weighted(bp(logits), labels.contiguous().data_ptr<int64_t>(), B, NC, ld,
                       out.data_ptr<float>(), fopt_mut(acc), (float)weight, accumulate,
                       rows.data_ptr<float>(), lse.data_ptr<float>(), cur_stream());
  return lse;
}

Tensor ce_bwd(Tensor logits, Tensor labels, Tensor lse, Tensor grad_out, double weight) {
  const int ld = logits_ld(logits);
  const int B = logits.size(0), NC = logits.size(1);
  const c10::OptionalDeviceGuard g(device_of(logits));
  Tensor d = torch::empty({B, ld}, logits.options());
  mpa::ce_bwd(bp(logits), labels.contiguous().data_ptr<int64_t>(), fopt(lse), fopt(grad_out), B,
              NC, ld, bpm(d), cur_stream(), (float)weight);
  return ld == NC ? d : d.narrow(1, 0, NC);
}

void argmax_correct(Tensor logits, Tensor labels, Tensor count) {
  const int ld = logits_ld(logits);
  TORCH_CHECK(count.scalar_type() == torch::kInt64, "count must be int64");
  const c10::OptionalDeviceGuard g(device_of(logits));
  mpa::argmax_correct(bp(logits), labels.contiguous().data_ptr<int64_t>(), logits.size(0),
                      logits.size(1), ld, count.data_ptr<int64_t>(), cur_stream());
}

// ----------------------------------------------------------------------------- optim
void adam_step(Tensor p, Tensor g, Tensor m, Tensor v, Tensor shadow, Tensor step, double lr,
               double b1, double b2, double eps, double wd, double gs) {
  CHECK_F32(p);
  TORCH_CHECK(p.numel() % 4 == 0 && g.numel() >= p.numel(), "adam: sizes");
  const c10::OptionalDeviceGuard gd(device_of(p));
  mpa::adam_step(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                 v.data_ptr<float>(), has(shadow) ? bpm(shadow) : nullptr, step.data_ptr<float>(),
                 p.numel(), lr, b1, b2, eps, wd, gs, cur_stream());
}

void sgd_step(Tensor p, Tensor g, Tensor buf, Tensor shadow, Tensor step, double lr,
              double momentum, double dampening, double wd, bool nesterov, double gs) {
  CHECK_F32(p);
  TORCH_CHECK(p.numel() % 4 == 0, "sgd: sizes");
  const c10::OptionalDeviceGuard gd(device_of(p));
  mpa::sgd_step(p.data_ptr<float>(), g.data_ptr<float>(), buf.data_ptr<float>(),
                has(shadow) ? bpm(shadow) : nullptr, step.data_ptr<float>(), p.numel(), lr,
                momentum, dampening, wd, nesterov ? 1 : 0, gs, cur_stream());
}

void transpose_krsc(Tensor w, Tensor wt, Tensor seg, int64_t total_tiles,
                    c10::optional<Tensor> step_inc) {
  CHECK_CUDA(w);
  CHECK_CUDA(wt);
  CHECK_CUDA(seg);
  TORCH_CHECK(seg.scalar_type() == torch::kInt64 && seg.dim() == 2 && seg.size(1) == 6,
              "transpose_krsc: seg [n][6] int64");
  const c10::OptionalDeviceGuard g(device_of(w));
  mpa::transpose_krsc(bp(w), bpm(wt), seg.contiguous().data_ptr<int64_t>(), (int)seg.size(0),
                      (int)total_tiles, cur_stream(),
                      step_inc ? fopt_mut(*step_inc) : nullptr);
}

void zero_cols_f32(Tensor t, int64_t period, int64_t first, int64_t count) {
  CHECK_CUDA(t);
  CHECK_CONTIG(t);
  CHECK_F32(t);
  TORCH_CHECK(period > 0 && first >= 0 && count >= 0 && first + count <= period &&
                  t.numel() % period == 0, "zero_cols_f32: columns outside the row");
  const c10::OptionalDeviceGuard g(device_of(t));
  mpa::zero_cols_f32(t.data_ptr<float>(), t.numel() / period, (int)period, (int)first,
                     (int)count, cur_stream());
}

void add_bf16_(Tensor a, Tensor b) {
  CHECK_ACT(a);
  CHECK_ACT(b);
  TORCH_CHECK(a.numel() == b.numel() && a.numel() % 8 == 0, "add_bf16_: same size, % 8");
  const c10::OptionalDeviceGuard g(device_of(a));
  mpa::add_bf16(bpm(a), bp(b), a.numel(), cur_stream());
}

void zero_f32(Tensor t) {
  CHECK_CUDA(t);
  CHECK_CONTIG(t);
  CHECK_F32(t);
  TORCH_CHECK(t.numel() % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              "zero_f32: numel % 4 == 0 and 16-B alignment required");
  const c10::OptionalDeviceGuard g(device_of(t));
  mpa::zero_f32(t.data_ptr<float>(), t.numel(), cur_stream());
}

void add_f32_(Tensor dst, Tensor src) {
  CHECK_CUDA(dst);
  CHECK_F32(dst);
  CHECK_F32(src);
  TORCH_CHECK(dst.is_contiguous() && src.is_contiguous() && dst.numel() == src.numel() &&
                  src.device() == dst.device(),
              "add_f32_: contiguous fp32 tensors of equal size on one device");
  const c10::OptionalDeviceGuard g(device_of(dst));
  mpa::add_f32(dst.data_ptr<float>(), src.data_ptr<float>(), dst.numel(), cur_stream());
}

void step_inc(Tensor step) {
  CHECK_CUDA(step);
  CHECK_F32(step);
  const c10::OptionalDeviceGuard g(device_of(step));
  mpa::step_inc(step.data_ptr<float>(), cur_stream());
}

void cast_f32_bf16(Tensor x, Tensor y) {
  CHECK_F32(x);
  CHECK_BF16(y);
  TORCH_CHECK(x.numel() % 4 == 0 && y.numel() == x.numel(), "cast: sizes");
  const c10::OptionalDeviceGuard g(device_of(x));
  mpa::cast_f32_bf16(x.data_ptr<float>(), bpm(y), x.numel(), cur_stream());
}

// ------------------------------------------------------------------------ preprocess
// pad: (top, bottom, left, right) zero border of the output canvas (empty = none)
Tensor preprocess(Tensor img, int64_t OH, int64_t OW, std::vector<double> mean,
                  std::vector<double> stdv, int64_t mode, int64_t cpad, std::vector<int64_t> pad,
                  c10::optional<Tensor> ext) {
  CHECK_CUDA(img);
  CHECK_CONTIG(img);
  TORCH_CHECK(img.scalar_type() == torch::kUInt8 && img.dim() == 4 && img.size(3) == 3,
              "preprocess: expects uint8 [B,H,W,3]");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3 && cpad >= 3, "preprocess: args");
  TORCH_CHECK(pad.empty() || pad.size() == 4, "preprocess: pad = (top, bottom, left, right)");
  mpa::OutPad pd{0, 0, 0, 0};
  if (pad.size() == 4) pd = mpa::OutPad{(int)pad[0], (int)pad[1], (int)pad[2], (int)pad[3]};
  TORCH_CHECK(pd.top >= 0 && pd.bottom >= 0 && pd.left >= 0 && pd.right >= 0, "preprocess: pad");
  const c10::OptionalDeviceGuard g(device_of(img));
  const int B = img.size(0), H = img.size(1), W = img.size(2);
  Tensor out = empty_like_shape(
      img, {B, OH + pd.top + pd.bottom, OW + pd.left + pd.right, cpad}, torch::kBFloat16);
  mpa::Norm3 n;
  for (int i = 0; i < 3; ++i) { n.mean[i] = mean[i]; n.std[i] = stdv[i]; }
  const int* extp = nullptr;
  if (ext && ext->defined() && ext->numel() > 0) {
    // per-image extents (h, w) inside the [H][W] pitch; the caller (ops/functional.py)
    // checked them on its host copy, so no device sync here
    TORCH_CHECK(mode == 0, "preprocess: extents with mode 0 (mode 1 is preprocess_pil)");
    CHECK_CUDA((*ext));
    CHECK_CONTIG((*ext));
    TORCH_CHECK(ext->scalar_type() == torch::kInt32 && ext->numel() == 2 * (int64_t)B,
                "preprocess: ext must be int32 [B,2]");
    extp = ext->data_ptr<int>();
  }
  mpa::preprocess(img.data_ptr<uint8_t>(), B, H, W, OH, OW, n, mode, cpad, pd, bpm(out),
                  cur_stream(), extp);
  return out;
}

// PIL-exact bicubic resize + ToTensor + Normalize (data/pil_resize.py builds the tables)
Tensor preprocess_pil(Tensor img, Tensor ext, Tensor sel, Tensor hb, Tensor hk, int64_t kh,
                      Tensor vb, Tensor vk, int64_t kv, int64_t OH, int64_t OW,
                      std::vector<double> mean, std::vector<double> stdv, int64_t cpad,
                      std::vector<int64_t> pad) {
  CHECK_CUDA(img);
  CHECK_CONTIG(img);
  TORCH_CHECK(img.scalar_type() == torch::kUInt8 && img.dim() == 4 && img.size(3) == 3,
              "preprocess_pil: expects uint8 [B,H,W,3]");
  TORCH_CHECK(mean.size() == 3 && stdv.size() == 3 && cpad >= 3, "preprocess_pil: args");
  TORCH_CHECK(pad.empty() || pad.size() == 4, "preprocess_pil: pad = (top, bottom, left, right)");
  const int B = img.size(0), Hp = img.size(1), Wp = img.size(2);
  auto i32 = [&](const Tensor& t, int64_t n, const char* what) {
    CHECK_CUDA(t);
    CHECK_CONTIG(t);
    TORCH_CHECK(t.scalar_type() == torch::kInt32 && t.numel() == n, "preprocess_pil: ", what);
    return t.data_ptr<int>();
  };
  const int* selp = i32(sel, 2 * (int64_t)B, "sel [B,2]");
  TORCH_CHECK(hb.numel() % (2 * OW) == 0 && vb.numel() % (2 * OH) == 0, "preprocess_pil: bounds");
  const int64_t nw = hb.numel() / (2 * OW), nh = vb.numel() / (2 * OH);
  const int* hbp = i32(hb, nw * 2 * OW, "hb");
  const int* hkp = i32(hk, nw * OW * kh, "hk");
  const int* vbp = i32(vb, nh * 2 * OH, "vb");
  const int* vkp = i32(vk, nh * OH * kv, "vk");
  // (the window of every table entry lies inside its image's extent and every extent inside
  // the pitch: data/pil_resize.TableCache checks that on the host copies it builds, so this
  // launch path never syncs the device)
  const int* extp = has(ext) ? i32(ext, 2 * (int64_t)B, "ext [B,2]") : nullptr;
  mpa::OutPad pd{0, 0, 0, 0};
  if (pad.size() == 4) pd = mpa::OutPad{(int)pad[0], (int)pad[1], (int)pad[2], (int)pad[3]};
  TORCH_CHECK(pd.top >= 0 && pd.bottom >= 0 && pd.left >= 0 && pd.right >= 0, "preprocess_pil: pad");
  const c10::OptionalDeviceGuard g(device_of(img));
  Tensor out = empty_like_shape(
      img, {B, OH + pd.top + pd.bottom, OW + pd.left + pd.right, cpad}, torch::kBFloat16);
  Tensor tmp = torch::empty({(int64_t)B * Hp * OW}, img.options().dtype(torch::kInt32));
  mpa::Norm3 n;
  for (int i = 0; i < 3; ++i) { n.mean[i] = mean[i]; n.std[i] = stdv[i]; }
  mpa::preprocess_pil(img.data_ptr<uint8_t>(), B, Hp, Wp, extp, selp, hbp, hkp, (int)kh, vbp, vkp,
                      (int)kv, (int)OH, (int)OW, n, (int)cpad, pd,
                      reinterpret_cast<uint32_t*>(tmp.data_ptr<int>()), bpm(out), cur_stream());
  return out;
}

// counter: optional device int32 [1] added to offset and advanced by one per call on the
// stream (graph-replay-safe dropout streams, ops/functional.py DropoutRNG)
std::vector<Tensor> dropout_fwd(Tensor x, double p, int64_t seed, int64_t offset,
                                c10::optional<Tensor> counter) {
  CHECK_ACT(x);
  const c10::OptionalDeviceGuard g(device_of(x));
  uint32_t* ctr = nullptr;
  if (counter && counter->defined() && counter->numel()) {
    TORCH_CHECK(counter->is_cuda() && counter->scalar_type() == torch::kInt32 &&
                    counter->numel() == 1 && counter->device() == x.device(),
                "dropout_fwd: counter must be one int32 on the input's device");
    ctr = reinterpret_cast<uint32_t*>(counter->data_ptr<int>());
  }
  Tensor y = torch::empty_like(x);
  Tensor mask = torch::empty(x.sizes(), x.options().dtype(torch::kUInt8));
  mpa::dropout_fwd(bp(x), x.numel(), p, seed, offset, ctr, bpm(y), mask.data_ptr<uint8_t>(),
                   cur_stream());
  return {y, mask};
}

Tensor dropout_bwd(Tensor dy, Tensor mask, double p) {
  CHECK_ACT(dy);
  const c10::OptionalDeviceGuard g(device_of(dy));
  Tensor dx = torch::empty_like(dy);
  mpa::dropout_bwd(bp(dy), mask.data_ptr<uint8_t>(), dy.numel(), p, bpm(dx), cur_stream());
  return dx;
}

// ----------------------------------------------------------------------- channel concat
Tensor concat_channels(std::vector<Tensor> xs) {
  TORCH_CHECK(!xs.empty(), "concat_channels: no inputs");
  const Tensor& x0 = xs[0];
  TORCH_CHECK(x0.dim() >= 2, "concat_channels: inputs must be [..., C]");
  const int64_t pixels = x0.numel() / x0.size(-1);
  std::vector<const mpa::bf16_raw*> ptrs;
  std::vector<int> chans;
  int64_t ctot = 0;
  for (const Tensor& x : xs) {
    CHECK_ACT(x);
    TORCH_CHECK(x.dim() == x0.dim() && x.get_device() == x0.get_device(),
                "concat_channels: rank/device mismatch");
    for (int d = 0; d + 1 < x.dim(); ++d)
      TORCH_CHECK(x.size(d) == x0.size(d), "concat_channels: leading dims differ");
    TORCH_CHECK(x.size(-1) % 8 == 0, "concat_channels: channels must be a multiple of 8");
    ptrs.push_back(bp(x));
    chans.push_back((int)x.size(-1));
    ctot += x.size(-1);
  }
  TORCH_CHECK(pixels * (ctot / 8) < (int64_t(1) << 31), "concat_channels: too large");
  const c10::OptionalDeviceGuard g(device_of(x0));
  std::vector<int64_t> shape(x0.sizes().begin(), x0.sizes().end());
  shape.back() = ctot;
  Tensor y = torch::empty(shape, x0.options());
  if (pixels > 0)
    mpa::concat_channels(ptrs.data(), chans.data(), (int)xs.size(), (int)pixels, (int)ctot,
                         bpm(y), cur_stream());
  return y;
}

// G[..., off:off+C] (+)= src  (G fp32 [..., Ctot], src bf16 [..., C], same leading dims)
void chan_accum(Tensor g, int64_t off, Tensor src, bool assign) {
  CHECK_ACT(src);
  CHECK_CUDA(g);
  CHECK_CONTIG(g);
  CHECK_F32(g);
  const int64_t ctot = g.size(-1), cs = src.size(-1);
  TORCH_CHECK(g.dim() == src.dim() && g.numel() / ctot == src.numel() / cs,
              "chan_accum: leading dims differ");
  TORCH_CHECK(ctot % 8 == 0 && cs % 8 == 0 && off % 8 == 0 && off >= 0 && off + cs <= ctot,
              "chan_accum: channel range outside G (multiples of 8 required)");
  const int64_t pixels = src.numel() / cs;
  TORCH_CHECK(pixels * (cs / 8) < (int64_t(1) << 31), "chan_accum: too large");
  const c10::OptionalDeviceGuard gd(device_of(g));
  if (pixels > 0)
    mpa::chan_accum(g.data_ptr<float>(), (int)ctot, (int)off, bp(src), (int)cs, (int)pixels, assign,
                    cur_stream());
}

// dst[..., off:off+C] = src (same dtype: bf16 activations or fp32 rows, e.g. BN statistics
// [2, C] into a block's [2, Ctot]); same leading element count
void chan_insert(Tensor dst, int64_t off, Tensor src) {
  CHECK_CUDA(dst);
  CHECK_CUDA(src);
  CHECK_CONTIG(dst);
  CHECK_CONTIG(src);
  TORCH_CHECK(dst.scalar_type() == src.scalar_type() &&
                  (src.scalar_type() == torch::kBFloat16 || src.scalar_type() == torch::kFloat32),
              "chan_insert: bf16 or fp32, same dtype");
  const int64_t u = src.element_size() / 2;  // 16-bit units per element
  const int64_t ld = dst.size(-1), cs = src.size(-1);
  TORCH_CHECK(dst.numel() / ld == src.numel() / cs && off >= 0 && off + cs <= ld,
              "chan_insert: shapes");
  TORCH_CHECK((ld * u) % 8 == 0 && (cs * u) % 8 == 0 && (off * u) % 8 == 0,
              "chan_insert: 16-byte aligned channel runs required");
  const int64_t rows = src.numel() / cs;
  TORCH_CHECK(rows * (cs * u / 8) < (int64_t(1) << 31), "chan_insert: too large");
  const c10::OptionalDeviceGuard gd(device_of(dst));
  if (rows > 0)
    mpa::chan_insert((mpa::bf16_raw*)dst.data_ptr(), (int)(ld * u), (int)(off * u),
                     (const mpa::bf16_raw*)src.data_ptr(), (int)(cs * u), (int)rows,
                     cur_stream());
}

// dense copy of src[..., off:off+cs] (bf16 or fp32)
Tensor chan_slice(Tensor src, int64_t off, int64_t cs) {
  CHECK_CUDA(src);
  CHECK_CONTIG(src);
  TORCH_CHECK(src.scalar_type() == torch::kBFloat16 || src.scalar_type() == torch::kFloat32,
              "chan_slice: bf16 or fp32");
  const int64_t u = src.element_size() / 2;
  const int64_t ld = src.size(-1);
  TORCH_CHECK(off >= 0 && cs > 0 && off + cs <= ld && (ld * u) % 8 == 0 && (cs * u) % 8 == 0 &&
                  (off * u) % 8 == 0, "chan_slice: 16-byte aligned channel runs required");
  const int64_t rows = src.numel() / ld;
  TORCH_CHECK(rows * (cs * u / 8) < (int64_t(1) << 31), "chan_slice: too large");
  const c10::OptionalDeviceGuard gd(device_of(src));
  std::vector<int64_t> shape(src.sizes().begin(), src.sizes().end());
  shape.back() = cs;
  Tensor out = torch::empty(shape, src.options());
  if (rows > 0)
    mpa::chan_slice((const mpa::bf16_raw*)src.data_ptr(), (int)(ld * u), (int)(off * u),
                    (mpa::bf16_raw*)out.data_ptr(), (int)(cs * u), (int)rows, cur_stream());
  return out;
}

// bf16 copy of G[..., off:off+C]
Tensor chan_extract(Tensor g, int64_t off, int64_t cs) {
  CHECK_CUDA(g);
  CHECK_CONTIG(g);
  CHECK_F32(g);
  const int64_t ctot = g.size(-1);
  TORCH_CHECK(ctot % 8 == 0 && cs % 8 == 0 && off % 8 == 0 && off >= 0 && off + cs <= ctot && cs > 0,
              "chan_extract: channel range outside G (multiples of 8 required)");
  const int64_t pixels = g.numel() / ctot;
  TORCH_CHECK(pixels * (cs / 8) < (int64_t(1) << 31), "chan_extract: too large");
  const c10::OptionalDeviceGuard gd(device_of(g));
  std::vector<int64_t> shape(g.sizes().begin(), g.sizes().end());
  shape.back() = cs;
  Tensor out = torch::empty(shape, g.options().dtype(torch::kBFloat16));
  if (pixels > 0)
    mpa::chan_extract(g.data_ptr<float>(), (int)ctot, (int)off, bpm(out), (int)cs, (int)pixels,
                      cur_stream());
  return out;
}

std::vector<Tensor> split_channels(Tensor dy, std::vector<int64_t> sizes) {
  CHECK_ACT(dy);
  TORCH_CHECK(dy.dim() >= 2 && !sizes.empty(), "split_channels: dy must be [..., C]");
  int64_t ctot = 0;
  for (int64_t c : sizes) {
    TORCH_CHECK(c > 0 && c % 8 == 0, "split_channels: channels must be a multiple of 8");
    ctot += c;
  }
  TORCH_CHECK(ctot == dy.size(-1), "split_channels: sizes do not sum to C");
  const int64_t pixels = dy.numel() / ctot;
  TORCH_CHECK(pixels * (ctot / 8) < (int64_t(1) << 31), "split_channels: too large");
  const c10::OptionalDeviceGuard g(device_of(dy));
  std::vector<Tensor> out;
  std::vector<mpa::bf16_raw*> ptrs;
  std::vector<int> chans;
  std::vector<int64_t> shape(dy.sizes().begin(), dy.sizes().end());
  for (int64_t c : sizes) {
    shape.back() = c;
    out.push_back(torch::empty(shape, dy.options()));
    ptrs.push_back(bpm(out.back()));
    chans.push_back((int)c);
  }
  if (pixels > 0)
    mpa::split_channels(bp(dy), chans.data(), (int)sizes.size(), (int)pixels, (int)ctot,
                        ptrs.data(), cur_stream());
  return out;
}

}  // namespace

extern "C" const char* mpa_src_hash();  // build/src_hash.cpp (setup.py)

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "mpi_pytorch_amd native gfx950 kernels + runtime";
  m.def("src_hash", [] { return std::string(mpa_src_hash()); },
        "hash of the csrc/ sources this binary was built from (setup.py source_hash)");
  m.def("igemm_engine", &mpa::igemm_engine, "GEMM staging engine: 1 LDS-DMA, 0 register");
  m.def("igemm_set_engine", &mpa::igemm_set_engine);
  m.def("igemm_force_tile", &mpa::igemm_force_tile, "override GEMM tile (BM, BN, splits); 0 = auto");
  m.def("igemm_set_tune", &mpa::igemm_set_tune, "tile autotuner on/off (MPA_TUNE)");
  m.def("igemm_set_tune_drain", &mpa::igemm_set_tune_drain,
        "tuner candidates: drain the whole device (1, single GPU) or only their stream (0)");
  m.def("set_deterministic", &mpa::set_deterministic,
        "fixed-order reductions + no timing-based autotuning (MPA_DETERMINISTIC)");
  m.def("deterministic", &mpa::deterministic);
  m.def("igemm_tuned_table", &mpa::igemm_tuned_table, "autotuned GEMM tiles so far");
  m.def("igemm_tuned_load", &mpa::igemm_tuned_load, py::arg("table"), py::arg("replace") = true,
        "adopt an igemm_tuned_table() dump (data-parallel ranks take rank 0's)");
  m.def("igemm_set_dma_uni", &mpa::igemm_set_dma_uni, "LDS-DMA uniform-tap fast path on/off");
  m.def("igemm_set_halo", &mpa::igemm_set_halo, "halo-staged direct 3x3/s1 conv on/off");
  m.def("igemm_set_halo_mi7", &mpa::igemm_set_halo_mi7, "448-pixel halo tiles on/off");
  m.def("igemm_set_halo_strip", &mpa::igemm_set_halo_strip,
        "strip-tiled halo conv: 0 off, 1 images too wide for linear tiles, 2 also layer1");
  m.def("igemm_halo_enabled", &mpa::igemm_halo_enabled);
  m.def("igemm_set_stem", &mpa::igemm_set_stem, "direct row-staged 7x7 pixel-pair stem on/off");
  m.def("preprocess_set_copy", &mpa::preprocess_set_copy,
        "identity-size preprocess fast path on/off (MPA_PRE_COPY)");
  m.def("set_comm_reserve", &mpa::set_comm_reserve,
        "CUs held by an overlapping collective (persistent conv grids use the rest)");
  m.def("comm_reserve", &mpa::comm_reserve, "current collective CU reservation");
  m.def("active_cus", &mpa::active_cus, "CUs the persistent conv grids size for");
  m.def("igemm_set_halo_wprod", &mpa::igemm_set_halo_wprod,
        "halo weight gradients on producer-wave blocks on/off (MPA_HALO_WPROD)");
  m.def("igemm_set_halo_wxmap", &mpa::igemm_set_halo_wxmap,
        "XCD-grouped halo weight-gradient block order on/off (MPA_HALO_WXMAP)");
  m.def("affine_act", &affine_act, "relu?(x * aff[0] + aff[1]) per channel (aff [2, C])");
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("relu"), py::arg("stats"),
        py::arg("shift"), "conv forward (+ BN statistics of its output)");
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("w"), py::arg("H"), py::arg("W"),
        py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("wt") = py::none(),
        py::arg("accum") = py::none());
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("overwrite") = false,
        "weight gradient into dw (+=; overwrite: dw = ..., the first gradient since zero)");
  m.def("conv_bnred_ok", &conv_bnred_ok);
  m.def("conv_dgrad_bnred_gacc", &conv_dgrad_bnred_gacc);
  m.def("conv_dgrad_res", &conv_dgrad_res);
  m.def("conv_dgrad_pair", &conv_dgrad_pair, py::arg("dy"), py::arg("w"), py::arg("wt"),
        py::arg("H"), py::arg("W"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("dy2"), py::arg("w2"), py::arg("wt2"), py::arg("ph2"), py::arg("pw2"),
        py::arg("accum") = py::none());
  m.def("bn_defer_step", &bn_defer_step, py::arg("sums"), py::arg("gamma"), py::arg("mean"),
        py::arg("rstd"), py::arg("s0"), py::arg("k12"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("G"), py::arg("x"), py::arg("out") = py::none());
  m.def("conv_fwd_into", &conv_fwd_into);
  m.def("conv_dgrad_bnred", &conv_dgrad_bnred, py::arg("dy"), py::arg("w"), py::arg("H"),
        py::arg("W"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("wt"),
        py::arg("z"), py::arg("y"), py::arg("mean"), py::arg("rstd"),
        py::arg("gamma") = py::none(), py::arg("beta") = py::none());
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("act_bwd", &act_bwd);
  m.def("bn_fwd_train", &bn_fwd_train, py::arg("x"), py::arg("stats"), py::arg("gamma"),
        py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("momentum"), py::arg("eps"),
        py::arg("res"), py::arg("relu"), py::arg("counter") = py::none(),
        py::arg("mask") = py::none(), py::arg("channels") = 0,
        py::arg("res_affine") = py::none(), py::arg("out") = py::none());
  m.def("bn_stats_affine", &bn_stats_affine, py::arg("x"), py::arg("stats"), py::arg("gamma"),
        py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("momentum"),
        py::arg("eps"), py::arg("counter") = py::none());
  m.def("bn_stats", &bn_stats, "[mean | biased var] of x [..., C]");
  m.def("bn_relu_avgpool2_fwd", &bn_relu_avgpool2_fwd);
  m.def("bn_fwd_eval", &bn_fwd_eval, py::arg("x"), py::arg("gamma"), py::arg("beta"),
        py::arg("rmean"), py::arg("rvar"), py::arg("eps"), py::arg("res"), py::arg("relu"),
        py::arg("channels") = 0);
  m.def("bn_bwd_pair", &bn_bwd_pair);
  m.def("maxpool_bwd_relu", &maxpool_bwd_relu);
  m.def("bn_bwd", &bn_bwd, py::arg("dy"), py::arg("x"), py::arg("y"), py::arg("mean"),
        py::arg("rstd"), py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("want_dx"), py::arg("want_g"), py::arg("zmask_beta") = py::none(),
        py::arg("ymask") = py::none(), py::arg("gacc") = py::none(),
        py::arg("dx_out") = py::none());
  m.def("relu_fwd", &relu_fwd);
  m.def("comm_emulator", &comm_emulator, "diagnostics: occupy CUs like a concurrent collective");
  m.def("atomic_latency", &atomic_latency, "diagnostics: dependent atomic round trips");
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("bn_relu_maxpool_fwd", &bn_relu_maxpool_fwd, py::arg("z"), py::arg("stats"),
        py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("momentum"),
        py::arg("eps"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"),
        py::arg("pw"), py::arg("ceil"), py::arg("counter") = py::none(),
        py::arg("zsel_out") = py::none());
  m.def("maxpool_bn_bwd_sums", &maxpool_bn_bwd_sums);
  m.def("conv_stem_pool_fwd", &conv_stem_pool_fwd, py::arg("x"), py::arg("w"), py::arg("sh"),
        py::arg("sw"), py::arg("ph"), py::arg("pw"), py::arg("stats"),
        py::arg("shift"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"),
        py::arg("momentum"), py::arg("eps"), py::arg("counter") = py::none());
  m.def("stem_pool_wgrad_ok", &stem_pool_wgrad_ok);
  m.def("stem_pool_wgrad", &stem_pool_wgrad);
  m.def("maxpool_bn_bwd", &maxpool_bn_bwd, py::arg("dp"), py::arg("idx"), py::arg("z"),
        py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("beta"), py::arg("dgamma"),
        py::arg("dbeta"), py::arg("kh"), py::arg("kw"), py::arg("sh"), py::arg("sw"),
        py::arg("ph"), py::arg("pw"), py::arg("zsel") = py::none());
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd, py::arg("dy"), py::arg("H"), py::arg("W"), py::arg("kh"),
        py::arg("kw"), py::arg("sh"), py::arg("sw"), py::arg("ph"), py::arg("pw"),
        py::arg("ceil"), py::arg("cip"), py::arg("dx_out") = py::none());
  m.def("adaptive_avgpool_fwd", &adaptive_avgpool_fwd);
  m.def("adaptive_avgpool_bwd", &adaptive_avgpool_bwd);
  m.def("linear_fwd", &linear_fwd);
  m.def("linear_dgrad", &linear_dgrad, py::arg("dy"), py::arg("w"), py::arg("wt") = py::none());
  m.def("linear_wgrad", &linear_wgrad, py::arg("dy"), py::arg("x"), py::arg("dw"),
        py::arg("overwrite") = false);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd, py::arg("logits"), py::arg("labels"), py::arg("lse"),
        py::arg("grad_out"), py::arg("weight") = 1.0);
  m.def("ce_fwd_weighted", &ce_fwd_weighted);
  m.def("argmax_correct", &argmax_correct);
  m.def("adam_step", &adam_step);
  m.def("sgd_step", &sgd_step);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("transpose_krsc", &transpose_krsc, py::arg("w"), py::arg("wt"), py::arg("seg"),
        py::arg("total_tiles"), py::arg("step_inc") = py::none());
  m.def("zero_f32", &zero_f32, "t.zero_() on the native path");
  m.def("zero_cols_f32", &zero_cols_f32, "zero columns [first, first+count) of t as [-1, period]");
  m.def("add_bf16_", &add_bf16_, "a += b (bf16, fp32 add)");
  m.def("add_f32_", &add_f32_, "dst += src (fp32)");
  m.def("step_inc", &step_inc);
  m.def("chan_accum", &chan_accum, "fp32 G[..., off:off+C] (+)= bf16 src");
  m.def("chan_extract", &chan_extract, "bf16 copy of fp32 G[..., off:off+C]");
  m.def("chan_insert", &chan_insert, "dst[..., off:off+C] = src (bf16 or fp32)");
  m.def("chan_slice", &chan_slice, "dense copy of src[..., off:off+C] (bf16 or fp32)");
  m.def("preprocess_pil", &preprocess_pil, "PIL-exact bicubic resize + ToTensor + Normalize");
  m.def("preprocess", &preprocess, py::arg("img"), py::arg("OH"), py::arg("OW"), py::arg("mean"),
        py::arg("std"), py::arg("mode"), py::arg("cpad"),
        py::arg("pad") = std::vector<int64_t>{}, py::arg("ext") = py::none());
  m.def("dropout_fwd", &dropout_fwd, py::arg("x"), py::arg("p"), py::arg("seed"),
        py::arg("offset"), py::arg("counter") = py::none());
  m.def("dropout_bwd", &dropout_bwd);
  m.def("concat_channels", &concat_channels);
  m.def("split_channels", &split_channels);
  mpa_runtime::register_bindings(m);
}
