// NHWC bf16 implicit-GEMM convolution on MFMA (v_mfma_f32_16x16x32_bf16), gfx950.
//
// One forward-style kernel covers every conv GEMM that writes activations:
//   * forward        Y[m, co]  = Σ_{tap, ci} X[n, y*s + dy_t, x*s + dx_t, ci] · W[co, tap, ci]
//   * dgrad stride 1 dX[m, ci] = Σ_{tap, co} dY[n, y + dy_t, x + dx_t, co] · Wt[ci, tap, co]
//                    (tap offsets dy_t = p − kh encode the 180° kernel flip)
//   * dgrad stride 2 one launch per output parity class (a, b): rows m = (n, y, x) are the
//                    output pixels (2y+a, 2x+b); only the taps with kh ≡ a+p (mod 2) are
//                    visited, so no MFMA work is spent on the 3/4 structural zeros.
// The per-launch geometry is an arithmetic tap grid (ConvGeom) expanded into an LDS
// table once per block.
//
// Tiling (CDNA4, wave64): BM×BN block tile, BK = 64 (one 128-B row per tile row),
// 4 waves each owning a (BM/WM)×(BN/WN) sub-tile as 16×16 MFMA blocks; the LDS image
// is row-major with the 16-B chunk XOR-swizzle  chunk ^ ((row >> 1) & 7), which makes
// every ds_read_b128 fragment read of the 16x16x32 operand map and every 8-lane
// ds_write_b128 group conflict-free (see docs/KERNELS.md for the derivation).
// Global→LDS staging is register-double-buffered: tile k+1 is loaded into VGPRs
// before the MFMAs of tile k and written to the other LDS buffer after them, so one
// barrier per K-tile suffices.  The epilogue stages the fp32 tile through LDS to emit
// fully coalesced 16-B bf16 stores, optionally adds a residual/accumulate tensor, and
// reduces per-channel Σy and Σy² (BatchNorm batch statistics) from the fp32
// accumulators into a per-row-tile slab — BN statistics cost no extra pass over Y.
//
// Weight gradient (igemm_wgrad): dW[co, tap, ci] = Σ_m dY[m, co] · X_im2col[m, (tap, ci)]
// reduces over m, which is the row index of both operands in memory, so both tiles
// are staged [m][cols] and read with the CDNA4 transpose read ds_read_b64_tr_b16.
// The reduction is split over blocks into fp32 slabs and combined by a fixed-order
// reduce that also permutes to the OIHW fp32 gradient layout and applies beta.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <cstdint>
#include <stdexcept>
#include <string>

#include <type_traits>

namespace dm {


// ------------------------------------------------------------------ forward / dgrad, v3
// Register-staged buffer loads (as igemm_fwd_kernel<...,BUF=true>) with
//   * cheaper per-tile addressing: each staged row keeps its pixel base and its
//     (y*isy, x*isx) origin, so a chunk costs one add + two unsigned bound checks;
//   * MF32 = true: v_mfma_f32_32x32x16_bf16 (half the MFMA issues of 16x16x32 for the
//     same 64x64 wave tile; same LDS bytes per FLOP; the chunk swizzle stays
//     conflict-free for its 32-row fragment reads).
template <int BM, int BN, int WM, int WN, bool MF32, int DEPTH, bool SEG2 = false, bool RED = false>
__global__ void __launch_bounds__(WM * WN * 64, (WM * WN > 4 ? 1 : 2)) igemm_fwd3_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeomSet gs, unsigned xbytes, unsigned wbytes, DgradSeg2 s2,
    BnBwdRed red) {
  // blockIdx.z selects the geometry: the parity classes of a stride-2 dgrad (disjoint
  // output pixels, 1..4 taps each) run as ONE launch instead of four small serial ones
  const ConvGeom g = gs.g[blockIdx.z];
  if ((long long)blockIdx.x * BM >= g.M) {  // classes with fewer rows (odd sizes)
    if constexpr (RED) {  // every part row is summed by the consumer: write this one's zeros
      const long long row = (long long)blockIdx.z * gridDim.x + blockIdx.x;
      for (int c = threadIdx.x; c < 2 * g.Ncols; c += blockDim.x) red.part[row * 2 * g.Ncols + c] = 0.f;
    }
    return;
  }
  constexpr int BK = 64;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = MF32 ? 32 : 16;                 // MFMA block edge
  constexpr int RM = TM / FM, RN = TN / FM;
  constexpr int NT = WM * WN * 64, RPP = NT / 8;   // threads, staged rows per pass
  constexpr int AR = BM / RPP, BR = BN / RPP;
  static_assert(AR * RPP == BM && BR * RPP == BN, "tile rows must be a multiple of NT/8");
  static_assert(DEPTH == 1 || DEPTH == 2, "register prefetch depth");
  constexpr unsigned OOB = 0x80000000u;
  typedef typename std::conditional<MF32, f32x16, f32x4>::type accT;
  constexpr int NR = MF32 ? 16 : 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);
  bf16_t* Bs = As + 2 * BM * BK;
  int4* taps = reinterpret_cast<int4*>(Bs + 2 * BN * BK);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const long long m0 = (long long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int ntaps = g.nth * g.ntw;
  if (tid < MAXTAPS) {  // every entry written: the loader reads it without a branch
    int4 e = make_int4(0, 0, 0, 0);
    if (tid < ntaps) {
      const int th = tid / g.ntw, tw = tid % g.ntw;
      const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
      // .w = pixel offset of the tap (dy*W + dx)
      e = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * g.C,
                    dy * g.W + dx);
    }
    taps[tid] = e;
  }
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, (int)wbytes, 0x00020000);
  const int chunk = tid & 7;
  int a_y[AR], a_x[AR];
  unsigned a_pix[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const long long m = m0 + (tid >> 3) + RPP * i;
    if (m < g.M) {
      const unsigned t = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - t * (unsigned)g.Wg);
      const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
      const int y = (int)(t - n * (unsigned)g.Hg);
      a_y[i] = y * g.isy;
      a_x[i] = x * g.isx;
      a_pix[i] = (n * (unsigned)g.H + (unsigned)a_y[i]) * (unsigned)g.W + (unsigned)a_x[i];
    } else {
      a_y[i] = -(1 << 28);
      a_x[i] = 0;
      a_pix[i] = 0;
    }
  }
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + (tid >> 3) + RPP * i;
    b_off[i] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u : OOB;
  }
  __syncthreads();
  uint4 ra[DEPTH > 1 ? 2 : 1][AR], rb[DEPTH > 1 ? 2 : 1][BR];
  const int nk1 = (g.K + BK - 1) / BK;
  int nk = nk1;
  const unsigned C2 = (unsigned)g.C * 2u;
  // SEG2: K tiles nk1.. of geometry s2.z read X2 at the row's own pixel and W2 (block-uniform)
  unsigned b_off2[SEG2 ? BR : 1];
  const auto rsx2 = __builtin_amdgcn_make_buffer_rsrc((void*)(SEG2 ? s2.X2 : (const void*)X), (short)0,
                                                      (int)(SEG2 ? s2.x2bytes : 0u), 0x00020000);
  const auto rsw2 = __builtin_amdgcn_make_buffer_rsrc((void*)(SEG2 ? s2.W2 : (const void*)Wp), (short)0,
                                                      (int)(SEG2 ? s2.w2bytes : 0u), 0x00020000);
  if constexpr (SEG2) {
    if ((int)blockIdx.z == s2.z) nk += s2.C2 / BK;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + (tid >> 3) + RPP * i;
      b_off2[i] = n < g.Ncols ? (unsigned)n * (unsigned)s2.C2 * 2u : OOB;
    }
  }

  auto load = [&](int kt, auto S) {
    if constexpr (SEG2) {
      if (kt >= nk1) {
        const unsigned c0b = (unsigned)(((kt - nk1) * (BK / 8) + chunk) * 16);
        const unsigned P2 = (unsigned)s2.C2 * 2u;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const unsigned off = a_y[i] >= 0 ? a_pix[i] * P2 + c0b : OOB;
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx2, off, 0, 0);
          ra[S][i] = make_uint4(v[0], v[1], v[2], v[3]);
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
          const unsigned off = b_off2[i] != OOB ? b_off2[i] + c0b : OOB;
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsw2, off, 0, 0);
          rb[S][i] = make_uint4(v[0], v[1], v[2], v[3]);
        }
        return;
      }
    }
    const int kc = kt * (BK / 8) + chunk;
    const int tap = kc >> g.lgC8;
    const unsigned c0b = (unsigned)((kc & ((1 << g.lgC8) - 1)) * 16);  // byte offset in pixel
    const bool kval = tap < ntaps;
    const int4 tp = taps[tap < MAXTAPS ? tap : MAXTAPS - 1];
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const bool ok = kval && (unsigned)(a_y[i] + tp.x) < (unsigned)g.H &&
                      (unsigned)(a_x[i] + tp.y) < (unsigned)g.W;
      const unsigned off = ok ? (a_pix[i] + (unsigned)tp.w) * C2 + c0b : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      ra[S][i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const unsigned off = (kval && b_off[i] != OOB) ? b_off[i] + (unsigned)tp.z * 2u + c0b : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsw, off, 0, 0);
      rb[S][i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store = [&](int buf, auto S) {
    bf16_t* as = As + buf * BM * BK;
    bf16_t* bs = Bs + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int r = (tid >> 3) + RPP * i;
      *reinterpret_cast<uint4*>(as + r * BK + swz(r, chunk) * 8) = ra[S][i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = (tid >> 3) + RPP * i;
      *reinterpret_cast<uint4*>(bs + r * BK + swz(r, chunk) * 8) = rb[S][i];
    }
  };


  accT acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;

  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, (DEPTH > 1 ? 1 : 0)>;
  auto compute = [&](int buf, auto post) {
      const bf16_t* as = As + buf * BM * BK;
      const bf16_t* bs = Bs + buf * BN * BK;
      if constexpr (MF32) {
        // fragments double-buffered across the 4 k-substeps: the reads of substep ks+1
        // are in flight while the MFMAs of substep ks issue
        bf16x8 af[2][RM], bfr[2][RN];
        auto frag = [&](int ks, int set) {
          const int ch = ks * 2 + (lane >> 5);
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            const int r = wm * TM + i * 32 + (lane & 31);
            af[set][i] = *reinterpret_cast<const bf16x8*>(as + r * BK + swz(r, ch) * 8);
          }
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            const int r = wn * TN + j * 32 + (lane & 31);
            bfr[set][j] = *reinterpret_cast<const bf16x8*>(bs + r * BK + swz(r, ch) * 8);
          }
        };
        frag(0, 0);
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
          if (ks + 1 < BK / 16) frag(ks + 1, (ks + 1) & 1);
          __builtin_amdgcn_sched_barrier(0);  // keep those reads ahead of this substep's MFMAs
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bfr[ks & 1][j],
                                                                  acc[i][j], 0, 0, 0);
          post(ks);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
          const int ch = ks * 4 + (lane >> 4);
          bf16x8 af[RM], bfr[RN];
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            const int r = wm * TM + i * 16 + (lane & 15);
            af[i] = *reinterpret_cast<const bf16x8*>(as + r * BK + swz(r, ch) * 8);
          }
#pragma unroll
          for (int j = 0; j < RN; ++j) {
            const int r = wn * TN + j * 16 + (lane & 15);
            bfr[j] = *reinterpret_cast<const bf16x8*>(bs + r * BK + swz(r, ch) * 8);
          }
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
          post(ks);
        }
      }
  };
  auto nopost = [](int) {};
  if constexpr (DEPTH == 1) {
    load(0, S0{});
    store(0, S0{});
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int buf = kt & 1;
      if (kt + 1 < nk) load(kt + 1, S0{});
      compute(buf, nopost);
      if (kt + 1 < nk) store(buf ^ 1, S0{});
      __syncthreads();
    }
  } else {
    // tile t is staged through register set t & 1, issued two tiles ahead of its use
    load(0, S0{});
    if (nk > 1) load(1, S1{});
    store(0, S0{});
    __syncthreads();
    for (int kt = 0; kt < nk; kt += 2) {
      if (kt + 2 < nk) load(kt + 2, S0{});
      compute(0, nopost);
      if (kt + 1 < nk) store(1, S1{});
      __syncthreads();
      if (kt + 1 >= nk) break;
      if (kt + 3 < nk) load(kt + 3, S1{});
      compute(1, nopost);
      if (kt + 2 < nk) store(0, S0{});
      __syncthreads();
    }
  }

  mfma_tile_epilogue<BM, BN, WM, WN, MF32, 1, RED>(acc, smem, m0, n0, blockIdx.z * gridDim.x + blockIdx.x,
                                                    stats, g, Y, ADD, red);
}

// ------------------------------------------------------------------ weight gradient
// grid: (ceil(Ncols/BM), ceil(K/BN), S).  Block reduces m in [s*mchunk, min(M,(s+1)*mchunk)).
// A = dY (rows m, cols co), B = im2col(X) (rows m, cols k); LDS images [m][cols+PAD].
// Weight gradient, v2: 64 m-rows per barrier (two MFMA k-steps), branch-free buffer
// loads with range-check zero fill, magic-number row decomposition.
template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256, 2) igemm_wgrad2_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY, float* __restrict__ slab,
    ConvGeom g, long long mchunk, unsigned xbytes, unsigned dybytes) {
  constexpr int BKM = 64;
  constexpr int PAD = 16;
  constexpr int LA = BM + PAD, LB = BN + PAD;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int RM = TM / 16, RN = TN / 16;
  constexpr int ACH = BM / 8, BCH = BN / 8;
  constexpr int AIT = BKM * ACH / 256, BIT = BKM * BCH / 256;
  constexpr unsigned OOB = 0x80000000u;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);           // [2][BKM][LA]
  bf16_t* Bs = As + 2 * BKM * LA;                         // [2][BKM][LB]
  int4* taps = reinterpret_cast<int4*>(Bs + 2 * BKM * LB);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int co0 = blockIdx.x * BM, k0 = blockIdx.y * BN;
  const unsigned mb = (unsigned)((long long)blockIdx.z * mchunk);
  const unsigned me = (unsigned)min(g.M, (long long)mb + mchunk);
  const int ntaps = g.nth * g.ntw;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    taps[tid] = make_int4(g.dy0 + th * g.dys, g.dx0 + tw * g.dxs, 0, 0);
  }
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsd = __builtin_amdgcn_make_buffer_rsrc((void*)DY, (short)0, (int)dybytes, 0x00020000);
  // per-thread fixed column chunks (the row varies with the step)
  const int acol = tid % ACH, arow0 = tid / ACH;          // A: rows arow0 + it*(256/ACH)
  const int bcol = tid % BCH, brow0 = tid / BCH;
  const bool a_colok = co0 + acol * 8 < g.Ncols;
  const int kc = (k0 >> 3) + bcol;
  const int btap = kc >> g.lgC8;
  const unsigned bc0 = (unsigned)((kc & ((1 << g.lgC8) - 1)) * 8);
  __syncthreads();
  const bool b_ok = btap < ntaps;
  int4 btp = make_int4(0, 0, 0, 0);
  if (b_ok) btp = taps[btap];

  uint4 ra[AIT], rb[BIT];
  auto load = [&](unsigned mt) {
#pragma unroll
    for (int it = 0; it < AIT; ++it) {
      const unsigned m = mt + arow0 + it * (256 / ACH);
      const unsigned off = (m < me && a_colok) ? (m * (unsigned)g.Ncols + co0 + acol * 8) * 2u : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsd, off, 0, 0);
      ra[it] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
      const unsigned m = mt + brow0 + it * (256 / BCH);
      unsigned off = OOB;
      if (m < me && b_ok) {
        const unsigned t = fdiv(m, g.wg_mul, g.wg_shr);
        const int x = (int)(m - t * (unsigned)g.Wg);
        const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
        const int y = (int)(t - n * (unsigned)g.Hg);
        const int iy = y * g.isy + btp.x, ix = x * g.isx + btp.y;
        if ((unsigned)iy < (unsigned)g.H && (unsigned)ix < (unsigned)g.W)
          off = (((n * (unsigned)g.H + (unsigned)iy) * (unsigned)g.W + (unsigned)ix) * (unsigned)g.C + bc0) * 2u;
      }
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rb[it] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store = [&](int buf) {
    bf16_t* as = As + buf * BKM * LA;
    bf16_t* bs = Bs + buf * BKM * LB;
#pragma unroll
    for (int it = 0; it < AIT; ++it)
      *reinterpret_cast<uint4*>(as + (arow0 + it * (256 / ACH)) * LA + acol * 8) = ra[it];
#pragma unroll
    for (int it = 0; it < BIT; ++it)
      *reinterpret_cast<uint4*>(bs + (brow0 + it * (256 / BCH)) * LB + bcol * 8) = rb[it];
  };

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int nsteps = me > mb ? (int)((me - mb + BKM - 1) / BKM) : 0;
  if (nsteps > 0) {
    load(mb);
    store(0);
  }
  __syncthreads();
  typedef short s4 __attribute__((ext_vector_type(4)));
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    if (st + 1 < nsteps) load(mb + (unsigned)(st + 1) * BKM);
    const bf16_t* as = As + buf * BKM * LA;
    const bf16_t* bs = Bs + buf * BKM * LB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = ks * 32 + grp * 4 + q;
      bf16x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const int col = wm * TM + i * 16 + 4 * p;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(as + r0 * LA + col));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(as + (r0 + 16) * LA + col));
        af[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int col = wn * TN + j * 16 + 4 * p;
        const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(bs + r0 * LB + col));
        const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) s4*)(bs + (r0 + 16) * LB + col));
        bfr[j] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (st + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  float* out = slab + (long long)blockIdx.z * g.Ncols * g.K;
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
        const int k = k0 + wn * TN + j * 16 + (lane & 15);
        if (co < g.Ncols && k < g.K) out[(long long)co * g.K + k] = acc[i][j][r];
      }
}

// dw[co][ci][kh][kw] = beta*dw + Σ_s slab[s][co][(kh*KW+kw)*C + ci]   (ci < Cin)
typedef float f32x4v __attribute__((ext_vector_type(4)));
template <bool NT, int V>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab,
                                                           int S, int Cout, int C, int Cin,
                                                           int KH, int KW,
                                                           float* __restrict__ dw, float beta,
                                                           int lanes) {
  // block = (256 / lanes) threads of V consecutive slab elements x `lanes` split lanes; lane l
  // sums the slabs l, l + lanes, ... in order, up to 8 V-wide loads in flight (the last
  // batch predicated, so a short S still issues its loads together), lanes combine in fixed
  // order.  Reads follow the slab layout [S][Cout][K] (coalesced, V = 4 needs C % 4 == 0);
  // the OIHW write is a permutation.
  typedef typename std::conditional<V == 4, f32x4v, float>::type vec;
  __shared__ vec red[256];
  const long long K = (long long)KH * KW * C;
  const long long total = (long long)Cout * K;
  const long long plane = total / V;
  const int E = 256 / lanes;
  const int el = threadIdx.x % E, ln = threadIdx.x / E;
  const long long e = ((long long)blockIdx.x * E + el) * V;
  vec acc = 0.f;
  if (e < total) {
    const vec* src = reinterpret_cast<const vec*>(slab + e);
    for (int i = ln; i < S; i += 8 * lanes) {
      vec v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const vec* a = src + (long long)(i + j * lanes) * plane;
        v[j] = i + j * lanes < S ? (NT ? __builtin_nontemporal_load(a) : *a) : vec(0.f);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (i + j * lanes < S) acc += v[j];
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (ln != 0 || e >= total) return;
  vec sum = 0.f;
  for (int l = 0; l < lanes; ++l) sum += red[l * E + el];
  const int co = (int)(e / K);
  const int k0 = (int)(e - (long long)co * K);
  const int tap = k0 / C, ci0 = k0 - tap * C;  // V | C: the V elements share co and tap
  const int kh = tap / KW, kw = tap - kh * KW;
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int ci = ci0 + u;
    if (ci >= Cin) break;  // channel padding of the packed input
    const long long o = (((long long)co * Cin + ci) * KH + kh) * KW + kw;
    float su;
    if constexpr (V == 4) su = sum[u]; else su = sum;
    dw[o] = (beta != 0.f ? beta * dw[o] : 0.f) + su;
  }
}

// ------------------------------------------------------------------ weight packing
// fp32 OIHW -> bf16 [Cout][KH][KW][Cpad] (forward) and optionally
// bf16 [Cin][KH][KW][Cout] (dgrad; transpose only — the flip is in the tap offsets),
// one element per thread
__global__ void __launch_bounds__(256) pack_weights_any_kernel(const float* __restrict__ w,
                                                               bf16_t* __restrict__ wf,
                                                               bf16_t* __restrict__ wd, int Cout,
                                                               int Cin, int Cpad, int KH, int KW) {
  const long long total = (long long)Cout * KH * KW * Cpad;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int ci = o % Cpad;
    long long t = o / Cpad;
    const int kw = t % KW;
    t /= KW;
    const int kh = t % KH;
    const int co = t / KH;
    const float v = ci < Cin ? w[(((long long)co * Cin + ci) * KH + kh) * KW + kw] : 0.f;
    const bf16_t b = f2bf(v);
    wf[o] = b;
    if (wd && ci < Cin) wd[(((long long)ci * KH + kh) * KW + kw) * Cout + co] = b;
  }
}

// All conv layers of a model in one launch: desc[l] = {w, wf, wd, Cout, Cin, Cpad, KH, KW}
// (pointers as int64), prefix[l] = first packed element of layer l (prefix[nl] = total).
__global__ void __launch_bounds__(256) pack_weights_multi_kernel(const long long* __restrict__ desc,
                                                                 const long long* __restrict__ prefix,
                                                                 int nl) {
  __shared__ long long pre[33];
  for (int i = threadIdx.x; i <= nl; i += blockDim.x) pre[i] = prefix[i];
  __syncthreads();
  const long long total = pre[nl];
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    int l = 0;
    while (l + 1 < nl && o >= pre[l + 1]) ++l;
    const long long* d = desc + 8 * l;
    const float* w = (const float*)d[0];
    bf16_t* wf = (bf16_t*)d[1];
    bf16_t* wd = (bf16_t*)d[2];
    const int Cout = (int)d[3], Cin = (int)d[4], Cpad = (int)d[5], KH = (int)d[6], KW = (int)d[7];
    const unsigned e = (unsigned)(o - pre[l]);
    const int ci = (int)(e % (unsigned)Cpad);
    unsigned t = e / (unsigned)Cpad;
    const int kw = (int)(t % (unsigned)KW);
    t /= (unsigned)KW;
    const int kh = (int)(t % (unsigned)KH);
    const int co = (int)(t / (unsigned)KH);
    const float v = ci < Cin ? w[(((long long)co * Cin + ci) * KH + kh) * KW + kw] : 0.f;
    const bf16_t b = f2bf(v);
    wf[e] = b;
    if (wd && ci < Cin) wd[(((long long)ci * KH + kh) * KW + kw) * Cout + co] = b;
  }
}

// All conv layers in one launch, LDS-tiled: block = (layer, 32 co, 32 ci) over all taps
// (tap chunks of <= 9).  Reads are contiguous OIHW runs of 32*T floats, both packed
// layouts are written as contiguous 64-B rows (2 bf16 per lane), so neither the strided
// fp32 reads nor the scattered 2-byte dgrad-layout writes of the element-per-thread
// kernel remain (that kernel: ~100 us for ResNet-18's 11.2 M conv weights).
// tprefix[l] = first tile of layer l (tprefix[nl] = number of blocks).
__global__ void __launch_bounds__(256) pack_weights_tiled_kernel(const long long* __restrict__ desc,
                                                                 const int* __restrict__ tprefix,
                                                                 int nl) {
  __shared__ float tile[32 * 9 * 33];
  __shared__ int pre[33];
  for (int i = threadIdx.x; i <= nl; i += blockDim.x) pre[i] = tprefix[i];
  __syncthreads();
  int l = 0;
  while (l + 1 < nl && (int)blockIdx.x >= pre[l + 1]) ++l;
  const long long* d = desc + 8 * l;
  const float* w = (const float*)d[0];
  bf16_t* wf = (bf16_t*)d[1];
  bf16_t* wd = (bf16_t*)d[2];
  const int Cout = (int)d[3], Cin = (int)d[4], Cpad = (int)d[5];
  const int T = (int)(d[6] * d[7]);
  const int CI = Cpad > Cin ? Cpad : Cin;
  const int nci = (CI + 31) / 32;
  const int tl = (int)blockIdx.x - pre[l];
  const int co0 = (tl / nci) * 32, ci0 = (tl % nci) * 32;
  for (int t0 = 0; t0 < T; t0 += 9) {
    const int TT = T - t0 < 9 ? T - t0 : 9;
    if (t0) __syncthreads();
    if (TT == T && Cin % 32 == 0) {
      // whole-tap tile of full channel groups: 32 contiguous runs of 32*T floats, read as
      // float4 with every load of the thread issued before the first LDS store
      const int R4 = 8 * T;
      float4 v[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int e = threadIdx.x + k * 256;
        const int co = e / R4;
        v[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (e < 32 * R4 && co0 + co < Cout)
          v[k] = reinterpret_cast<const float4*>(w + ((long long)(co0 + co) * Cin + ci0) * T)[e - co * R4];
      }
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int e = threadIdx.x + k * 256;
        if (e >= 32 * R4) break;
        const int co = e / R4, f = 4 * (e - co * R4);
        const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int ci = (f + j) / T, t = (f + j) - ci * T;
          tile[(co * TT + t) * 33 + ci] = vv[j];
        }
      }
    } else
    for (int e = threadIdx.x; e < 32 * 32 * TT; e += 256) {
      const int co = e / (32 * TT), r = e - co * (32 * TT);
      const int ci = r / TT, t = r - ci * TT;
      float v = 0.f;
      if (co0 + co < Cout && ci0 + ci < Cin) v = w[((long long)(co0 + co) * Cin + ci0 + ci) * T + t0 + t];
      tile[(co * TT + t) * 33 + ci] = v;
    }
    __syncthreads();
    // wf[co][t][ci]: pairs of channels (Cpad is a multiple of 8)
    for (int e = threadIdx.x; e < 32 * TT * 16; e += 256) {
      const int ci = 2 * (e & 15), r = e >> 4;
      const int t = r % TT, co = r / TT;
      if (co0 + co < Cout && ci0 + ci < Cpad) {
        const float* q = tile + (co * TT + t) * 33 + ci;
        *reinterpret_cast<uint32_t*>(wf + ((long long)(co0 + co) * T + t0 + t) * Cpad + ci0 + ci) =
            pack_bf2(q[0], q[1]);
      }
    }
    if (wd) {
      // wd[ci][t][co]: pairs of output channels (Cout even)
      for (int e = threadIdx.x; e < 32 * TT * 16; e += 256) {
        const int co = 2 * (e & 15), r = e >> 4;
        const int t = r % TT, ci = r / TT;
        if (co0 + co < Cout && ci0 + ci < Cin)
          *reinterpret_cast<uint32_t*>(wd + ((long long)(ci0 + ci) * T + t0 + t) * Cout + co0 + co) =
              pack_bf2(tile[(co * TT + t) * 33 + ci], tile[((co + 1) * TT + t) * 33 + ci]);
      }
    }
  }
}

void pack_weights_multi(const long long* desc, const long long* prefix, int nl, long long total,
                        hipStream_t st) {
  pack_weights_multi_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(desc, prefix, nl);
}

void pack_weights_tiled(const long long* desc, const int* tprefix, int nl, int ntiles,
                        hipStream_t st) {
  pack_weights_tiled_kernel<<<ntiles, 256, 0, st>>>(desc, tprefix, nl);
}

// Space-to-depth stem weights: W[co][c][7][7] -> W'[co][4][4][Cp] with
// W'[co][u][v][(dy*2+dx)*C + c] = W[co][c][2u+dy-1][2v+dx-1] (0 outside the 7x7 window)
__global__ void __launch_bounds__(256) pack_weights_s2d_kernel(const float* __restrict__ w,
                                                               bf16_t* __restrict__ wf, int Cout,
                                                               int C, int Cp) {
  const long long total = (long long)Cout * 16 * Cp;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long o = (long long)blockIdx.x * blockDim.x + threadIdx.x; o < total; o += stride) {
    const int ch = o % Cp;
    const int uv = (o / Cp) % 16;
    const int co = o / (Cp * 16);
    const int u = uv / 4, v = uv % 4;
    const int sub = ch / C, c = ch % C;
    float val = 0.f;
    if (sub < 4) {
      const int kh = 2 * u + (sub >> 1) - 1, kw = 2 * v + (sub & 1) - 1;
      if (kh >= 0 && kh < 7 && kw >= 0 && kw < 7) val = w[(((long long)co * C + c) * 7 + kh) * 7 + kw];
    }
    wf[o] = f2bf(val);
  }
}

// dw[co][c][kh][kw] = beta*dw + Σ_s slab[s][co][(u*4+v)*Cp + (dy*2+dx)*C + c]
// Reduced in the slab's own layout [S][Cout][16*Cp] (coalesced reads), the S-sum split over
// `lanes` lanes per element with 8 loads in flight each, lanes combined in fixed order
// (deterministic); the write is the s2d -> 7x7 permutation (slab elements that fall outside
// the 7x7 window or into channel padding are structural zeros of the packed weight and
// are dropped).  The stem wgrad has many m-splits (S = 256) over few elements (64 x 256), so
// one thread per output element (9408 threads summing 256 dependent loads) was ~80 us.
__global__ void __launch_bounds__(256) wgrad_reduce_s2d_kernel(const float* __restrict__ slab,
                                                               int S, int Cout, int C, int Cp,
                                                               float* __restrict__ dw, float beta,
                                                               int lanes) {
  __shared__ float red[256];
  const long long K = 16LL * Cp;
  const long long total = (long long)Cout * K;
  const int E = 256 / lanes;
  const int el = threadIdx.x % E, ln = threadIdx.x / E;
  const long long e = (long long)blockIdx.x * E + el;
  float acc = 0.f;
  if (e < total) {
    const float* src = slab + e;
    int i = ln;
    for (; i + 7 * lanes < S; i += 8 * lanes) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = src[(long long)(i + j * lanes) * total];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += v[j];
    }
    for (; i < S; i += lanes) acc += src[(long long)i * total];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (ln != 0 || e >= total) return;
  float sum = 0.f;
  for (int l = 0; l < lanes; ++l) sum += red[l * E + el];
  const int co = (int)(e / K);
  const int k = (int)(e - (long long)co * K);
  const int uv = k / Cp, ch = k - uv * Cp;
  const int sub = ch / C, c = ch - sub * C;
  if (sub >= 4) return;
  const int kh = 2 * (uv >> 2) + (sub >> 1) - 1, kw = 2 * (uv & 3) + (sub & 1) - 1;
  if (kh < 0 || kh >= 7 || kw < 0 || kw >= 7) return;
  const long long o = (((long long)co * C + c) * 7 + kh) * 7 + kw;
  dw[o] = (beta != 0.f ? beta * dw[o] : 0.f) + sum;
}

void pack_weights_s2d(const float* w, bf16_t* wf, int Cout, int C, int Cp, hipStream_t st) {
  const long long total = (long long)Cout * 16 * Cp;
  pack_weights_s2d_kernel<<<grid_for(total, 256), 256, 0, st>>>(w, wf, Cout, C, Cp);
}

void wgrad_reduce_s2d(const float* slab, int S, int Cout, int C, int Cp, float* dw, float beta,
                      hipStream_t st) {
  const long long total = (long long)Cout * 16 * Cp;
  int lanes = 1;
  while (lanes < 16 && lanes * 8 < S) lanes *= 2;
  const int E = 256 / lanes;
  wgrad_reduce_s2d_kernel<<<(unsigned)((total + E - 1) / E), 256, 0, st>>>(slab, S, Cout, C, Cp,
                                                                          dw, beta, lanes);
}

// ------------------------------------------------------------------ launchers
static size_t fwd_smem(int BM, int BN) {
  const size_t main = (size_t)2 * (BM + BN) * 64 * 2 + MAXTAPS * 16;
  const size_t epi = (size_t)BM * (BN + 4) * 4;
  return main > epi ? main : epi;
}

template <int BM, int BN, int WM, int WN, bool MF32, int DEPTH, bool SEG2 = false, bool RED = false>
static void launch_fwd3_set(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                            float* stats, const ConvGeomSet& gs, int ng, hipStream_t st,
                            const DgradSeg2* seg2 = nullptr, const BnBwdRed* red = nullptr) {
  const ConvGeom& g = gs.g[0];
  long long mmax = 0;
  for (int i = 0; i < ng; ++i) mmax = gs.g[i].M > mmax ? gs.g[i].M : mmax;
  const size_t sm = fwd_smem(BM, BN);
  dim3 grid((unsigned)((mmax + BM - 1) / BM), (g.Ncols + BN - 1) / BN, ng);
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  const DgradSeg2 s2 = seg2 ? *seg2 : DgradSeg2{};
  const BnBwdRed rd = red ? *red : BnBwdRed{};
  auto k = igemm_fwd3_kernel<BM, BN, WM, WN, MF32, DEPTH, SEG2, RED>;
  set_smem_attr(k, sm);
  k<<<grid, WM * WN * 64, sm, st>>>(X, Wp, Y, ADD, stats, gs, xb, wb, s2, rd);
}

// the multi-geometry launch with the optional merged segment / reduction epilogue variants
template <int BM, int BN, int WM, int WN, bool MF32, int DEPTH>
static void launch_fwd3_multi(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                              float* stats, const ConvGeomSet& gs, int ng, hipStream_t st,
                              const DgradSeg2* seg2, const BnBwdRed* red) {
  if (seg2 && red)
    launch_fwd3_set<BM, BN, WM, WN, MF32, DEPTH, true, true>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red);
  else if (seg2)
    launch_fwd3_set<BM, BN, WM, WN, MF32, DEPTH, true, false>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red);
  else if (red)
    launch_fwd3_set<BM, BN, WM, WN, MF32, DEPTH, false, true>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red);
  else
    launch_fwd3_set<BM, BN, WM, WN, MF32, DEPTH>(X, Wp, Y, ADD, stats, gs, ng, st);
}

template <int BM, int BN, int WM, int WN, bool MF32, int DEPTH>
static void launch_fwd3(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                        float* stats, const ConvGeom& g, hipStream_t st) {
  launch_fwd3_set<BM, BN, WM, WN, MF32, DEPTH>(X, Wp, Y, ADD, stats, ConvGeomSet::one(g), 1,
                                               st);
}

// up to four geometries sharing X / W / Y (the parity classes of a stride-2 dgrad) in one
// launch on the v3 128x128 mf32 tile (no statistics: the classes' row tiles would collide)
bool igemm_fwd_multi(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                     const ConvGeomSet& gs, int ng, int cfg, hipStream_t st, const DgradSeg2* seg2,
                     const BnBwdRed* red) {
  if (seg2 && (seg2->C2 % 64 != 0 || seg2->z < 0 || seg2->z >= ng))
    throw std::runtime_error("igemm_fwd_multi: seg2 needs C2 % 64 == 0 and a valid geometry");
  switch (cfg) {  // the v3 mf32 tiles of igemm_fwd (12/13: one tile of prefetch, 15/16: two)
    case 12: launch_fwd3_multi<128, 128, 2, 2, true, 1>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    case 13: launch_fwd3_multi<128, 64, 2, 2, true, 1>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    case 15: launch_fwd3_multi<128, 128, 2, 2, true, 2>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    case 16: launch_fwd3_multi<128, 64, 2, 2, true, 2>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    // the 64x64 16x16x32 tiles (small grids: few images per GPU)
    case 11: case 14: launch_fwd3_multi<64, 64, 2, 2, false, 1>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    case 17: launch_fwd3_multi<64, 64, 2, 2, false, 2>(X, Wp, Y, ADD, stats, gs, ng, st, seg2, red); return true;
    default: return false;
  }
}

// part rows of a multi-geometry launch with the BN-backward reduction epilogue (blockIdx.z
// major, blockIdx.x minor; every block writes its row)
long long igemm_multi_rows(const ConvGeomSet& gs, int ng, int cfg) {
  long long mmax = 0;
  for (int i = 0; i < ng; ++i) mmax = gs.g[i].M > mmax ? gs.g[i].M : mmax;
  const int bm = (cfg == 12 || cfg == 13 || cfg == 15 || cfg == 16) ? 128
                 : (cfg == 11 || cfg == 14 || cfg == 17) ? 64 : 0;
  if (!bm) return 0;
  return (long long)ng * ((mmax + bm - 1) / bm);
}

// halo-kernel configs (conv_halo.hip): 42 = 128-pixel tile of 2 x 2 waves, BN 128, with
// two weight tiles of register prefetch (waves bit 8); 39 = 256-pixel tile of 4 x 2 waves,
// BN 64; 41 = 256-pixel tile of 4 x 1 waves of 64 x 64.  (The round-2 tiles 20 / 21, 42
// without the prefetch and BN 64, lost on every layer and are removed.)
int igemm_fwd_rowtile(int cfg);
bool halo_cfg(int cfg, int& bn, int& waves) {
  switch (cfg) {
    case 42: bn = 128; waves = 4 | 0x100; return true;
    case 39: bn = 64; waves = 16; return true;
    case 41: bn = 64; waves = 32; return true;
    default: return false;
  }
}

// Forward-style conv GEMM (forward, stride-1 dgrad, one dgrad parity class), by cfg:
//   9 / 10 / 11  v3 tiles 128x128 / 128x64 / 64x64 (2 x 2 waves) on 16x16x32 MFMA
//   12 / 13 / 14 the same on 32x32x16 MFMA (64x64 as 16x16x32: 14 == 11)
//   15 / 16 / 17 12 / 13 / 11 with two tiles of register prefetch
//   20 / 21 / 42 / 39 / 41  halo-staged unit-stride tiles (conv_halo.hip, see halo_cfg)
//   60           space-to-depth stem kernel (conv_stem.hip)
//   80           persistent resident-weight 64 -> 64 channel 3x3 conv (conv_res64.hip)
//   90 - 93      pipelined LDS-DMA tiles (conv_pipe.hip)
// Shapes a specialised kernel does not cover fall back to a v3 tile with the same row tile,
// so the statistics slab rows (igemm_fwd_rowtile) still match.
void igemm_fwd(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int cfg, hipStream_t st) {
  if (cfg >= 90 && cfg <= 93) {
    if (conv_pipe_supported(g, cfg)) return conv_pipe(X, Wp, Y, ADD, stats, g, cfg, st);
    if (g.Ncols % 128 == 0) return launch_fwd3<256, 128, 4, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
    return launch_fwd3<256, 64, 4, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
  }
  if (cfg == 80) return conv_res64(X, Wp, Y, ADD, stats, g, st);  // throws if unsupported
  if (cfg == 60) {
    if (!ADD && stem_conv_supported(g)) return stem_conv(X, Wp, Y, stats, g, st);
    return launch_fwd3<256, 64, 4, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
  }
  int bn, waves;
  if (halo_cfg(cfg, bn, waves)) {
    if (conv_halo_supported(g)) return conv_halo(X, Wp, Y, ADD, stats, g, bn, waves, st);
    if (igemm_fwd_rowtile(cfg) == 256) {
      if (bn == 128) return launch_fwd3<256, 128, 4, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
      return launch_fwd3<256, 64, 4, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
    }
    cfg = bn == 128 ? 12 : 13;
  }
  switch (cfg) {
    case 9: return launch_fwd3<128, 128, 2, 2, false, 1>(X, Wp, Y, ADD, stats, g, st);
    case 10: return launch_fwd3<128, 64, 2, 2, false, 1>(X, Wp, Y, ADD, stats, g, st);
    case 11: case 14: return launch_fwd3<64, 64, 2, 2, false, 1>(X, Wp, Y, ADD, stats, g, st);
    case 12: return launch_fwd3<128, 128, 2, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
    case 13: return launch_fwd3<128, 64, 2, 2, true, 1>(X, Wp, Y, ADD, stats, g, st);
    case 15: return launch_fwd3<128, 128, 2, 2, true, 2>(X, Wp, Y, ADD, stats, g, st);
    case 16: return launch_fwd3<128, 64, 2, 2, true, 2>(X, Wp, Y, ADD, stats, g, st);
    case 17: return launch_fwd3<64, 64, 2, 2, false, 2>(X, Wp, Y, ADD, stats, g, st);
    default: throw std::runtime_error("igemm_fwd: unknown cfg " + std::to_string(cfg));
  }
}

int igemm_fwd_rowtile(int cfg) {
  if ((cfg >= 90 && cfg <= 93) || cfg == 60 || cfg == 39 || cfg == 41) return 256;
  return (cfg == 11 || cfg == 14 || cfg == 17) ? 64 : 128;
}

void igemm_wgrad(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                 long long mchunk, int cfg, hipStream_t st) {
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned db = (unsigned)(g.M * g.Ncols * 2);
  // 8: row-streaming 64 -> 64 channel 3x3 kernel (wgrad_res64.hip), one slab per workgroup;
  // 4 / 5: halo-staged 3x3 unit-stride kernel (wgrad_halo.hip) with 9 / 3 taps per block;
  // other shapes fall back to the v2 tiles: 2 = 128x128, 3 = 64x128, 6 = 64x256
  if (cfg == 8) return wgrad_res64(X, DY, slab, g, S, st);  // throws if unsupported
  // 7: stride-2 parity-plane kernel (wgrad_halo.hip), 3x3 only (other shapes: v2 tiles)
  if (cfg == 7) {
    if (wgrad_s2_supported(g)) return wgrad_s2(X, DY, slab, g, S, mchunk, st);
    cfg = g.Ncols % 128 == 0 ? 2 : 3;
  }
  if (cfg == 4 || cfg == 5) {
    if (wgrad_halo_supported(g)) return wgrad_halo(X, DY, slab, g, S, mchunk, cfg == 4 ? 3 : 1, st);
    cfg = g.Ncols % 128 == 0 ? 2 : 3;
  }
  if (cfg != 2 && cfg != 3 && cfg != 6)
    throw std::runtime_error("igemm_wgrad: cfg must be 2, 3, 4, 5 or 6");
  if (cfg == 2) {
    dim3 grid((g.Ncols + 127) / 128, (g.K + 127) / 128, S);
    auto k = igemm_wgrad2_kernel<128, 128, 2, 2>;
    const size_t sm = 2 * 64 * ((128 + 16) + (128 + 16)) * 2 + MAXTAPS * 16;
    set_smem_attr(k, sm);
    k<<<grid, 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db);
  } else if (cfg == 6) {
    // 64 x 256: the whole K of the s2d stem (4x4 taps x 16 ch) in one tile, so every dY
    // row is read once instead of once per 128-column K tile
    dim3 grid((g.Ncols + 63) / 64, (g.K + 255) / 256, S);
    auto k = igemm_wgrad2_kernel<64, 256, 2, 2>;
    const size_t sm = 2 * 64 * ((64 + 16) + (256 + 16)) * 2 + MAXTAPS * 16;
    set_smem_attr(k, sm);
    k<<<grid, 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db);
  } else {
    dim3 grid((g.Ncols + 63) / 64, (g.K + 127) / 128, S);
    auto k = igemm_wgrad2_kernel<64, 128, 2, 2>;
    const size_t sm = 2 * 64 * ((64 + 16) + (128 + 16)) * 2 + MAXTAPS * 16;
    set_smem_attr(k, sm);
    k<<<grid, 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db);
  }
}

void wgrad_reduce(const float* slab, int S, int Cout, int C, int Cin, int KH, int KW, float* dw,
                  float beta, hipStream_t st) {
  const long long total = (long long)Cout * KH * KW * C;
  int lanes = 1;  // split the S-sum over lanes so small gradients with many slabs stay parallel
  while (lanes < 16 && lanes * 8 < S) lanes *= 2;
  const int E = 256 / lanes;
  // non-temporal slab loads: every slab is read once (profiles/nt_pool_wgrad_reduce_ab_r4aa.txt)
  // 16-byte slab loads: isolated 0.333 -> 0.276 ms per ResNet-18 step, the step itself equal
  // (profiles/wgrad_reduce_vec_ab_r4au.txt)
  if (C % 4 == 0 && (reinterpret_cast<uintptr_t>(slab) & 15) == 0) {
    const long long nv = total / 4;
    wgrad_reduce_kernel<true, 4><<<(unsigned)((nv + E - 1) / E), 256, 0, st>>>(
        slab, S, Cout, C, Cin, KH, KW, dw, beta, lanes);
    return;
  }
  wgrad_reduce_kernel<true, 1><<<(unsigned)((total + E - 1) / E), 256, 0, st>>>(
      slab, S, Cout, C, Cin, KH, KW, dw, beta, lanes);
}

void pack_weights(const float* w, bf16_t* wf, bf16_t* wd, int Cout, int Cin, int Cpad, int KH,
                  int KW, hipStream_t st) {
  // element-per-thread: measured faster than the LDS-tiled transpose (pack_weights_kernel)
  // on the ResNet-18 shapes, whose small layers give the tiled grid too few workgroups
  const long long total = (long long)Cout * KH * KW * Cpad;
  pack_weights_any_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(w, wf, wd, Cout, Cin, Cpad, KH, KW);
}

}  // namespace dm
