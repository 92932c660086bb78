// Device-side building blocks shared by the implicit-GEMM kernels (igemm.hip: register-
// staged engine; igemm_dma.hip: LDS-DMA engine): LDS image swizzles, MFMA fragment reads,
// vector loaders and the two epilogues.  Layout derivations: docs/KERNELS.md.
#pragma once
#include "common.h"
#include "api.h"

namespace mpa {

__device__ __forceinline__ u32x4 u32x4_make(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return u32x4{a, b, c, d};
}

constexpr int BK = 32;

// ---------------------------------------------------------------------- LDS swizzles
// K-contiguous image: [rows][32] bf16, 64-B rows, 4 x 16-B chunks per row.
__device__ __forceinline__ int kc_off(int row, int chunk) {
  return row * 64 + ((chunk ^ ((4 - ((row >> 2) & 3)) & 3)) << 4);
}

// N-contiguous image: [32 k-rows][COLS] bf16.  Chunk XOR keeps 8-B granules intact for
// the transposed read and spreads the 8 rows read by one 32-lane half over all banks.
template <int COLS>
__device__ __forceinline__ int mn_swz(int k) {
  if constexpr (COLS >= 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else if constexpr (COLS == 64) return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
  else return 2 * ((k >> 3) & 1);
}
template <int COLS>
__device__ __forceinline__ int mn_off(int k, int col) {
  const int chunk = col >> 3;
  return k * (COLS * 2) + (((chunk ^ mn_swz<COLS>(k))) << 4) + ((col & 7) << 1);
}

// fragment (8 consecutive k of one row) from a K-contiguous image
__device__ __forceinline__ bf16x8 frag_kc(const char* img, int row, int lane) {
  const u32x4 v = *LDS_PTR(const u32x4, img + kc_off(row, lane >> 4));
  return __builtin_bit_cast(bf16x8, v);
}

// fragment (8 consecutive k of one column) from an N-contiguous image, two tr reads
template <int COLS>
__device__ __forceinline__ bf16x8 frag_mn(const char* img, int col0, int lane) {
  const int g = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int col = col0 + 4 * pp;
  const int k0 = 8 * g + q;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, img + mn_off<COLS>(k0, col)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, img + mn_off<COLS>(k0 + 4, col)));
  s16x8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return __builtin_bit_cast(bf16x8, r);
}

// ------------------------------------------------- buffer-descriptor LDS-DMA helpers
// (conv_halo.hip, conv_stem.hip).  Exact n / d for n * d < 2^32 with mag = floor(2^32/d)+1.
__device__ __forceinline__ uint32_t udiv(uint32_t n, uint32_t mag) { return __umulhi(n, mag); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                           0x00020000);
}

__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, 0, 0, 0);
}

// The same DMA as inline asm: the compiler does not see an LDS write, so it inserts no
// vmcnt(0) before the following ds_read_b64_tr_b16 (whose intrinsic it cannot prove
// disjoint from the DMA target - with the builtin, every DMA issued between transposed
// reads was followed by a full wait).  Safe for the compiler's own vmcnt accounting: it
// only undercounts outstanding ops, so its waits get stronger, never weaker; the kernel
// waits for these DMAs itself (wait_all_barrier) before reading their stage.
__device__ __forceinline__ void buf_lds16_asm(__amdgpu_buffer_rsrc_t r, const char* lds,
                                              uint32_t voff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)lds);
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(m0), "v"(voff), "s"(r)
               : "memory", "m0");
}

// The same with the LDS byte address as a wave-uniform 32-bit value (lds_base(smem) +
// offset): converting a generic pointer per DMA costs a null check (s_cmp_lg_u64 +
// s_cselect) and a 64-bit add on the scalar unit every time.
__device__ __forceinline__ uint32_t lds_base(const void* smem) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)smem;
}
__device__ __forceinline__ void buf_lds16_at(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r)
               : "memory", "m0");
}

// ... and with a wave-uniform soffset added to every lane's address (a per-step scalar
// offset, e.g. the weight tap, at no VALU cost); soff must be >= 0
__device__ __forceinline__ void buf_lds16_so(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff,
                                             int soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r),
                 "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory", "m0");
}

template <int N>
__device__ __forceinline__ void halo_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// all of this wave's VMEM (LDS-DMAs, loads, stores) done, then the workgroup barrier; as a
// builtin s_waitcnt (vmcnt 0, lgkmcnt 0) the compiler's wait insertion knows the loads are
// complete, so it adds no vmcnt(0) later that would also wait for DMAs issued afterwards
__device__ __forceinline__ void wait_all_barrier() {
  __builtin_amdgcn_s_waitcnt(0x0070);
  __builtin_amdgcn_s_barrier();
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------- vector loaders
// Load 8 consecutive bf16 (one 16-B chunk) with VW-wide accesses.  `nv` = number of
// valid leading elements (0..8); VW=8 callers guarantee nv is 0 or 8 (alignment).
template <int VW>
__device__ __forceinline__ u32x4 ld_chunk(const bf16_t* p, int nv) {
  u32x4 r = u32x4{0, 0, 0, 0};
  if constexpr (VW == 8) {
    if (nv >= 8) r = *(const u32x4*)p;
  } else if constexpr (VW == 4) {
    if (nv >= 4) {
      const u32x2 a = *(const u32x2*)p;
      r.x = a.x; r.y = a.y;
    }
    if (nv >= 8) {
      const u32x2 b = *(const u32x2*)(p + 4);
      r.z = b.x; r.w = b.y;
    }
  } else {
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i)
      if (i < nv) w[i >> 1] |= (uint32_t)p[i] << (16 * (i & 1));
    r = u32x4{w[0], w[1], w[2], w[3]};
  }
  return r;
}

__device__ __forceinline__ int nvalid(int idx, int lim) {
  const int d = lim - idx;
  return d <= 0 ? 0 : (d >= 8 ? 8 : d);
}

// -------------------------------------------------------------------------- epilogues
// Rows engine (fwd / dgrad / linear).  The MFMA is issued channel-operand first, so lane
// owns D[n = nb + r][m = lane&15], r = 0..3: four consecutive output channels of one row.
//   SPLIT: plain 16-B fp32 stores of this split's partial into [z][M][N] (summed by
//          splitk_finalize) - no atomics.
//   else : +bias, ReLU, bf16 store (8 B per lane), and per-column shifted BN statistics of
//          the bf16-rounded outputs, reduced in-wave, across the WM waves through LDS
//          (`smem` must be free: the caller has passed a barrier after its last LDS read),
//          and written as this M-tile's row of the statistics slab p.stats [tiles_m][2N].
// output-row geometry of the rows engine (per stride phase in a merged dgrad launch)
struct RowsGeom {
  int M, oH, oW, Poh, Pow;
  FastDiv fd_hw, fd_ow;
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
  return f.m ? (__umulhi(n, f.m) >> f.s) : n;
}

template <int BM, int BN, int WM, int WN, bool SPLIT>
__device__ __forceinline__ void rows_epilogue(const IGemmArgs& p,
                                              f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                              char* smem, int mt, int m0, int n0, int wm,
                                              int wrow0, int wcol0, int tid, const RowsGeom& g,
                                              int stat_row = -1) {
  if (stat_row < 0) stat_row = mt;
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  const int lane = tid & 63;
  const int nl = (lane >> 4) * 4;
  if constexpr (SPLIT) {
    float* out = (float*)p.C + (size_t)block_split() * g.M * p.N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wrow0 + i * 16 + (lane & 15);
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wcol0 + j * 16 + nl;
        if (n + 3 < p.N && (p.N & 3) == 0) {
          *(f32x4*)(out + (size_t)m * p.N + n) = acc[i][j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (n + r < p.N) out[(size_t)m * p.N + n + r] = acc[i][j][r];
        }
      }
    }
  } else {
    bf16_t* out = (bf16_t*)p.C;
    float s[TN][4], q[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) { s[j][r] = 0.f; q[j][r] = 0.f; }
    // bias / stats shift; in BN-reduce mode the same registers carry mean / rstd
    f32x4 bias[TN], shift[TN];
    const bool bnred = p.ep_bnred != 0;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bias[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      shift[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int n = n0 + wcol0 + j * 16 + nl;
      const float* bsrc = bnred ? p.ep_mean : p.bias;
      const float* ssrc = bnred ? p.ep_rstd : p.stats_shift;
      if (bsrc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[j][r] = (n + r < p.N) ? bsrc[n + r] : 0.f;
      }
      if (ssrc) {
#pragma unroll
        for (int r = 0; r < 4; ++r) shift[j][r] = (n + r < p.N) ? ssrc[n + r] : 0.f;
      }
    }
    size_t orows[TM];
    bool moks[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wrow0 + i * 16 + (lane & 15);
      moks[i] = m < g.M;
      orows[i] = 0;
      if (moks[i]) {
        const int hw = g.oH * g.oW;
        const int img = (int)fdiv((uint32_t)m, g.fd_hw);
        const int rr = m - img * hw;
        const int oh = (int)fdiv((uint32_t)rr, g.fd_ow);
        const int ow = rr - oh * g.oW;
        orows[i] = ((size_t)img * p.dH * p.dW + (size_t)(oh * p.Uoh + g.Poh) * p.dW +
                    (ow * p.Uow + g.Pow)) * p.ldc;
      }
    }
    // accumulate mode: issue every read of the existing output up front (one exposed
    // latency for the tile instead of one per fragment)
    uint2 oldv[TM][TN];
    if (p.beta) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + wcol0 + j * 16 + nl;
          oldv[i][j] = (moks[i] && n + 3 < p.N) ? *(const uint2*)(out + orows[i] + n)
                                                 : make_uint2(0u, 0u);
        }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool mok = moks[i];
      const size_t orow = orows[i];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wcol0 + j * 16 + nl;
        float v[4];
        float zr[4] = {0.f, 0.f, 0.f, 0.f};
        if (bnred) {
          // dy (bf16-rounded like the unfused path) masked by ReLU(y); x_hat from z
          bool live[4] = {true, true, true, true};
          if (mok && n + 3 < p.N) {
            const uint2 zz = *(const uint2*)(p.ep_z + orow + n);
            zr[0] = bf2f(zz.x & 0xffff); zr[1] = bf2f(zz.x >> 16);
            zr[2] = bf2f(zz.y & 0xffff); zr[3] = bf2f(zz.y >> 16);
            if (p.ep_y) {
              const uint2 yy = *(const uint2*)(p.ep_y + orow + n);
              live[0] = (yy.x & 0x7fff) != 0 && !(yy.x & 0x8000);
              live[1] = ((yy.x >> 16) & 0x7fff) != 0 && !(yy.x & 0x80000000u);
              live[2] = (yy.y & 0x7fff) != 0 && !(yy.y & 0x8000);
              live[3] = ((yy.y >> 16) & 0x7fff) != 0 && !(yy.y & 0x80000000u);
            }
          } else if (mok) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (n + r < p.N) {
                zr[r] = bf2f(p.ep_z[orow + n + r]);
                if (p.ep_y) live[r] = bf2f(p.ep_y[orow + n + r]) > 0.f;
              }
            }
          }
          if (!p.ep_y && p.ep_gamma && p.ep_beta && mok) {
            // y never written (BN in the operand path): the mask from z with the forward's
            // exact affine and rounding, as the halo kernels recompute it
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (n + r < p.N) {
                const float sc = p.ep_gamma[n + r] * shift[j][r];
                const float sh = __builtin_fmaf(-bias[j][r], sc, p.ep_beta[n + r]);
                live[r] = bf2f(f2bf(__builtin_fmaf(zr[r], sc, sh))) > 0.f;
              }
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float d = bf2f(f2bf(acc[i][j][r]));
            v[r] = live[r] ? d : 0.f;
          }
        } else {
          float old[4] = {0.f, 0.f, 0.f, 0.f};
          if (p.beta && mok) {
            if (n + 3 < p.N) {
              const uint2 oo = oldv[i][j];
              old[0] = bf2f(oo.x & 0xffff); old[1] = bf2f(oo.x >> 16);
              old[2] = bf2f(oo.y & 0xffff); old[3] = bf2f(oo.y >> 16);
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (n + r < p.N) old[r] = bf2f(out[orow + n + r]);
            }
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float t = acc[i][j][r] + bias[j][r] + old[r];
            if (p.relu) t = fmaxf(t, 0.f);
            v[r] = t;
          }
        }
        const uint32_t lo = pack2(v[0], v[1]), hi = pack2(v[2], v[3]);
        if (mok) {
          if (n + 3 < p.N) {
            *(uint2*)(out + orow + n) = make_uint2(lo, hi);
          } else {
            const uint16_t e[4] = {(uint16_t)(lo & 0xffff), (uint16_t)(lo >> 16),
                                   (uint16_t)(hi & 0xffff), (uint16_t)(hi >> 16)};
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (n + r < p.N) out[orow + n + r] = e[r];
          }
          if (bnred) {
            // (sum g, sum g * (z - mean) * rstd) - BN backward's reduction
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s[j][r] += v[r];
              q[j][r] += v[r] * (zr[r] - bias[j][r]) * shift[j][r];
            }
          } else {
            // statistics on the bf16-rounded values BN will read, shifted by K ~ mean
            // (BN running mean) so the sum of squares does not cancel when |mean| >> std
            const float rv[4] = {bf2f(lo & 0xffff) - shift[j][0], bf2f(lo >> 16) - shift[j][1],
                                 bf2f(hi & 0xffff) - shift[j][2], bf2f(hi >> 16) - shift[j][3]};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s[j][r] += rv[r];
              q[j][r] += rv[r] * rv[r];
            }
          }
        }
      }
    }
    if (p.stats) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a = s[j][r], b = q[j][r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            a += __shfl_xor(a, o, 64);
            b += __shfl_xor(b, o, 64);
          }
          s[j][r] = a;
          q[j][r] = b;
        }
      float* red = (float*)smem;
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wcol0 + j * 16 + nl;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            red[(wm * BN + col + r) * 2] = s[j][r];
            red[(wm * BN + col + r) * 2 + 1] = q[j][r];
          }
        }
      }
      __syncthreads();
      if (stat_row == 0 && block_split() == 0 && tid < BN && n0 + tid < p.N) {
        // start value of the slab reduction that runs after this kernel (no memset)
        p.stats_sums[n0 + tid] = 0.f;
        p.stats_sums[p.N + n0 + tid] = 0.f;
      }
      if (tid < BN && n0 + tid < p.N) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          a += red[(w * BN + tid) * 2];
          b += red[(w * BN + tid) * 2 + 1];
        }
        p.stats[(size_t)stat_row * 2 * p.N + n0 + tid] = a;
        p.stats[(size_t)stat_row * 2 * p.N + p.N + n0 + tid] = b;
      }
    }
  }
}

// Wgrad engine.  The MFMA is issued with the column (r,s,c) operand first, so lane owns
// D[n = nb + r][m = lane&15]: four consecutive weight-gradient columns of one output
// channel -> one 16-B fp32 access per lane.  One split: read-modify-write straight into
// the fp32 gradient arena (a plain store when p.overwrite: the classifier's 132 MB gradient
// is then written once instead of read and written).  Several splits: plain stores of this split's partial into the
// slab [z][Kout][Ncols]; wgrad_reduce sums the slab into the arena afterwards.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void wgrad_epilogue(const WGradArgs& p,
                                               f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                               int m0, int n0, int wrow0, int wcol0,
                                               int lane) {
  constexpr int TM = BM / WM / 16;
  constexpr int TN = BN / WN / 16;
  const int nl = (lane >> 4) * 4;
  const bool direct = gridDim.z == 1;
  const bool vec = (p.Ncols & 3) == 0;
  float* dst = direct ? p.dw : p.slab + (size_t)blockIdx.z * p.Kout * p.Ncols;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wrow0 + i * 16 + (lane & 15);
    if (m >= p.Kout) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wcol0 + j * 16 + nl;
      float* q = dst + (size_t)m * p.Ncols + n;
      if (vec && n + 3 < p.Ncols) {
        f32x4 v = acc[i][j];
        if (direct && !p.overwrite) v += *(const f32x4*)q;
        *(f32x4*)q = v;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < p.Ncols) q[r] = (direct && !p.overwrite) ? q[r] + acc[i][j][r] : acc[i][j][r];
      }
    }
  }
}

// ------------------------------------------------- LDS-DMA engine (igemm_dma.hip)
// Launch the LDS-DMA variant of a planned rows / wgrad GEMM (16-B operand granularity
// required).  Return false when no instantiation covers the tile shape.
bool igemm_rows_dma(const IGemmArgs& a, int BM, int BN, bool bkc, int splits, hipStream_t s);
bool igemm_rows_uni_src2_ok(const IGemmArgs& a, bool bkc);
bool igemm_rows_kpad_ok(const IGemmArgs& a, bool bkc);
bool igemm_wgrad_dma(const WGradArgs& a, int BM, int BN, int splits, hipStream_t s);
bool igemm_wgrad_inc_ok(const WGradArgs& a);  // incremental-pixel wgrad kernel applies

}  // namespace mpa
