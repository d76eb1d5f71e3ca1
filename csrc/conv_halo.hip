// Halo-staged implicit-GEMM convolution for unit-stride tap grids (|dy|, |dx| <= 1), gfx950.
//
// The igemm kernels (conv_igemm.hip) stage one (tap, 64-channel) slice of the implicit
// im2col matrix per K-tile, so every input pixel is fetched from L2 once per tap — 9x
// for a 3x3 conv — and written to LDS 9x.  Measured on MI355X that staging traffic,
// not the MFMA issue rate, bounds those kernels at ~600-700 TFLOP/s.
//
// Here a block owns 128 consecutive output pixels m (flattened n, y, x).  Because the
// tap grid is unit-stride, all of their taps live inside the contiguous flattened input
// row range [r0 - 1, r1 + 1] (r = n*H + y), the "halo": at most (ceil(127/W) + 3) * W
// pixels.  The halo of one 64-channel chunk is staged into LDS ONCE and every tap's A
// fragment is read straight out of it:
//     A[p, tap] = halo[(m0 + p) - hbase + dy*W + dx]          (hbase = (r0 - 1) * W)
// — consecutive output pixels are consecutive halo rows, so the XOR-swizzled fragment
// reads stay conflict-free.  A tap that leaves the image (x+dx or y+dy out of range, or
// rows past M) is redirected to an all-zero LDS row, which is exactly the conv's zero
// padding (and crosses image/row boundaries of the flattened layout correctly).
//
// Per (chunk, tap) step the block stages only the weight tile (BN x 64 bf16), double
// buffered through registers as in the igemm kernels; the next chunk's halo is loaded
// into VGPRs while the current chunk's taps run and written once per chunk.  Per-step
// L2->LDS traffic drops from 16 KB (A) + BN*128 B (B) to ~2.5-5 KB + BN*128 B.
//
// Used for: stride-1 forward convs (3x3/p1, 1x1/p0), stride-1 dgrad (tap flip) and the
// parity classes of stride-2 dgrad (their dY grid is the launch grid, taps are unit-
// stride).  MFMA v_mfma_f32_32x32x16_bf16, 4 waves each owning 64 x BN/2.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <stdexcept>

namespace dm {

namespace {
constexpr int HBM = 128;  // output pixels per block (default tile)
constexpr int HBK = 64;   // channels per chunk (one 128-B LDS row per pixel)
constexpr unsigned OOB = 0x80000000u;

// 8-wave BN-64 tiles must stay <= 128 VGPRs to keep two workgroups (4 waves) per SIMD
// PF: weight-tile register prefetch depth (1: the tile of step s+1 is loaded during step s;
// 2: the tile of step s+2, so a load has two steps of MFMA work to land in)
// PRE: 0 = X as stored; 1 = X is a conv's raw output y, operand relu(y*sc + sh) (forward BN +
// ReLU of the previous layer)
// waves per SIMD the 8-wave 64-channel tile (cfg 39) is compiled for: 4 = its LDS-bound
// occupancy (2 workgroups per CU).  Built with 2: 43.9k vs 44.8k img/s
// (profiles/halo39_launch_bounds_r2c.jsonl)
#ifndef DM_HALO39_MINB
#define DM_HALO39_MINB 4
#endif
// RED: the data gradient's epilogue also reduces the consumer BatchNorm's backward sums
// (mfma_tile_epilogue RED)
// BWD (data gradients): X is a BatchNorm's OUTPUT gradient dz and the operand is that BN's
// backward dy = a*dz' + b*y + c (kernels.h BnBwdIn), computed while staging: the BN-backward
// apply pass and its dy tensor do not exist
template <int BN, int HR, int WM, int WN, int BMH, bool PRE, int PF, bool RED = false, bool BWD = false>
__global__ void __launch_bounds__(WM * WN * 64, (WM * WN == 8 && BN == 64) ? DM_HALO39_MINB : 2) conv_halo_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, unsigned wbytes,
    const float* __restrict__ pre_sc, const float* __restrict__ pre_sh,
    int xcd, int mtiles, BnBwdRed red, BnBwdIn bwd) {
  static_assert(!(PRE && BWD), "one operand transform");
  // pre_sc/pre_sh (optional): X is a conv's raw output y; the operand is relu(y*sc + sh)
  // (BatchNorm-apply + ReLU of the previous layer fused into the halo staging).  Out-of-
  // image taps still read the zero row, i.e. the padding stays zero AFTER the BN.
  constexpr int TM = BMH / WM, TN = BN / WN;
  constexpr int RM = TM / 32, RN = TN / 32;
  constexpr int NT = WM * WN * 64, RPP = NT / 8;     // threads, staged rows per pass
  constexpr int BR = BN / RPP;
  static_assert(BR * RPP == BN && RM >= 1 && RN >= 1, "tile / wave layout");
  constexpr int HP_MAX = RPP * HR;                   // halo rows the LDS image holds
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hs = reinterpret_cast<bf16_t*>(smem);      // [HP_MAX + 1][64], last row = zeros
  bf16_t* Bs = Hs + (HP_MAX + 1) * HBK;              // [2][BN][64]
  int4* taps = reinterpret_cast<int4*>(Bs + 2 * BN * HBK);
  float* btab = reinterpret_cast<float*>(taps + MAXTAPS);  // BWD: [5][C] coefficients

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // block -> (M tile, N tile).  xcd > 0 (1-D grid): the N tiles of one M tile are
  // consecutive blocks on the same XCD (blocks go to the XCDs round-robin, b % 8), so the
  // input halo the N tiles share is fetched into that XCD's L2 once, not once per N tile
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int b = blockIdx.x, j = b >> 3;
    by = j % xcd;
    bx = (j / xcd) * 8 + (b & 7);
    if (bx >= mtiles) return;  // padding of the M tiles to a multiple of 8
  }
  const long long m0 = (long long)bx * BMH;
  const int n0 = by * BN;
  const int ntaps = g.nth * g.ntw;
  const int nchunk = g.C / HBK;
  const int HW = g.H * g.W;
  const int NHW = g.N * HW;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    taps[tid] = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * g.C,
                          dy * g.W + dx);
  }
  if (tid < 8) *reinterpret_cast<uint4*>(Hs + HP_MAX * HBK + tid * 8) = make_uint4(0, 0, 0, 0);
  if constexpr (BWD) bwd_tab_fill(btab, bwd, 0, g.C, tid, WM * WN * 64);

  // halo extent (flattened rows r0-1 .. r1+1)
  const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
  const long long mlast = (m0 + BMH - 1 < g.M) ? m0 + BMH - 1 : g.M - 1;
  const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
  const int hbase = (r0 - 1) * g.W;
  const int hp = (r1 - r0 + 3) * g.W;

  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, (int)wbytes, 0x00020000);
  const int chunk = tid & 7;

  // per-lane A-fragment rows: halo row of the centre tap and the pixel coordinates
  int a_h[RM], a_x[RM], a_y[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const long long m = m0 + wm * TM + i * 32 + (lane & 31);
    const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
    a_x[i] = (int)((unsigned)m - r * (unsigned)g.W);
    const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
    a_y[i] = (m < g.M) ? (int)(r - n * (unsigned)g.H) : -(1 << 28);  // rows >= M: never valid
    a_h[i] = (int)(m - hbase);
  }
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + (tid >> 3) + RPP * i;
    b_off[i] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u : OOB;
  }
  __syncthreads();

  uint4 rh[HR], rb[BR];
  // BWD: the BN input y of the same chunks and their mask bytes, loaded with rh
  uint4 ry[BWD ? HR : 1];
  unsigned rmk[BWD ? HR : 1];
  const auto rsy = __builtin_amdgcn_make_buffer_rsrc((void*)(BWD ? (const void*)bwd.y : (const void*)X),
                                                     (short)0, (int)(BWD ? xbytes : 0u), 0x00020000);
  auto load_halo = [&](int cc) __attribute__((always_inline)) {
    const unsigned cb = (unsigned)(cc * HBK + chunk * 8) * 2u;
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      const int gp = hbase + hh;
      const bool ok = hh < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? (unsigned)gp * (unsigned)g.C * 2u + cb : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
      if constexpr (BWD) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rsy, off, 0, 0);
        ry[j] = make_uint4(w[0], w[1], w[2], w[3]);
        rmk[j] = bwd_mask_byte(bwd, off, xbytes >> 4);  // off is OOB (reads 0) past the tensor
      }
    }
  };
  auto store_halo = [&](int cc) __attribute__((always_inline)) {
    if constexpr (BWD) {
      // rows outside the tensor become garbage here: no valid tap reads them (zero row)
#pragma unroll
      for (int j = 0; j < HR; ++j) rh[j] = bwd_apply(btab, g.C, cc * HBK + chunk * 8, rh[j], ry[j], rmk[j]);
    }
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      *reinterpret_cast<uint4*>(Hs + hh * HBK + swz(hh, chunk) * 8) = rh[j];
    }
    if constexpr (PRE) {
      // normalise in place once the staging registers are dead (each thread rewrites
      // only its own chunks: program order suffices, no barrier), so the fused BN costs
      // no registers across the tap loop
      PreBN pbn;
      pbn.load(pre_sc, pre_sh, cc * HBK + chunk * 8);
#pragma unroll
      for (int j = 0; j < HR; ++j) {
        const int hh = (tid >> 3) + RPP * j;
        uint4* q = reinterpret_cast<uint4*>(Hs + hh * HBK + swz(hh, chunk) * 8);
        *q = pbn.apply(*q);
      }
    }
  };
  auto load_b_into = [&](uint4 (&dst)[BR], int cc, int t) {
    const unsigned kb = (unsigned)(taps[t].z + cc * HBK + chunk * 8) * 2u;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const unsigned off = b_off[i] != OOB ? b_off[i] + kb : OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsw, off, 0, 0);
      dst[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_b_from = [&](const uint4 (&src)[BR], int buf) {
    bf16_t* bs = Bs + buf * BN * HBK;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = (tid >> 3) + RPP * i;
      *reinterpret_cast<uint4*>(bs + r * HBK + swz(r, chunk) * 8) = src[i];
    }
  };
  auto load_b = [&](int cc, int t) { load_b_into(rb, cc, t); };
  auto store_b = [&](int buf) { store_b_from(rb, buf); };

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf, int t) {
    const int4 tp = taps[t];
    int hrow[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const bool ok = (unsigned)(a_x[i] + tp.y) < (unsigned)g.W &&
                      (unsigned)(a_y[i] + tp.x) < (unsigned)g.H;
      hrow[i] = ok ? a_h[i] + tp.w : HP_MAX;
    }
    const bf16_t* bs = Bs + buf * BN * HBK;
    // fragments double-buffered across the 4 k-substeps (reads of ks+1 overlap MFMAs of ks)
    bf16x8 af[2][RM], bfr[2][RN];
    auto frag = [&](int ks, int set) {
      const int ch = ks * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < RM; ++i)
        af[set][i] = *reinterpret_cast<const bf16x8*>(Hs + hrow[i] * HBK + swz(hrow[i], ch) * 8);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int r = wn * TN + j * 32 + (lane & 31);
        bfr[set][j] = *reinterpret_cast<const bf16x8*>(bs + r * HBK + swz(r, ch) * 8);
      }
    };
    frag(0, 0);
#pragma unroll
    for (int ks = 0; ks < HBK / 16; ++ks) {
      if (ks + 1 < HBK / 16) frag(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bfr[ks & 1][j],
                                                              acc[i][j], 0, 0, 0);
    }
  };

  const int S = nchunk * ntaps;
  if constexpr (PF == 1) {
    load_halo(0);
    load_b(0, 0);
    store_halo(0);
    store_b(0);
    __syncthreads();
    if (nchunk > 1) load_halo(1);
    int cc = 0, t = 0;
    for (int s = 0; s < S; ++s) {
      int nt = t + 1, ncc = cc;
      if (nt == ntaps) {
        nt = 0;
        ++ncc;
      }
      if (s + 1 < S) load_b(ncc, nt);
      compute(s & 1, t);
      if (s + 1 < S) store_b((s + 1) & 1);
      __syncthreads();
      if (ncc != cc && s + 1 < S) {
        store_halo(ncc);  // every wave is past the last tap of chunk cc
        __syncthreads();
        if (ncc + 1 < nchunk) load_halo(ncc + 1);
      }
      t = nt;
      cc = ncc;
    }
  } else {
    // two weight tiles in flight: step s computes from LDS buffer s&1, stores tile s+1
    // (loaded during step s-1) and issues the loads of tile s+2 into the register set
    // that tile s used; the loop is unrolled by two so each set is a static register array
    uint4 rb2[BR];
    auto nxt = [&](int& cc_, int& t_) {
      if (++t_ == ntaps) {
        t_ = 0;
        ++cc_;
      }
    };
    load_halo(0);
    load_b_into(rb, 0, 0);
    int lc = 0, lt = 0;  // (chunk, tap) of the next tile to load
    nxt(lc, lt);
    store_halo(0);
    store_b_from(rb, 0);
    if (S > 1) load_b_into(rb2, lc, lt);  // tile 1
    nxt(lc, lt);
    __syncthreads();
    if (nchunk > 1) load_halo(1);
    int cc = 0, t = 0;
    auto step = [&](int s, uint4 (&rnext)[BR], uint4 (&rfree)[BR]) {
      // rnext holds tile s+1; rfree receives tile s+2
      int nt = t + 1, ncc = cc;
      if (nt == ntaps) {
        nt = 0;
        ++ncc;
      }
      if (s + 2 < S) load_b_into(rfree, lc, lt);
      nxt(lc, lt);
      compute(s & 1, t);
      if (s + 1 < S) store_b_from(rnext, (s + 1) & 1);
      __syncthreads();
      if (ncc != cc && s + 1 < S) {
        store_halo(ncc);
        __syncthreads();
        if (ncc + 1 < nchunk) load_halo(ncc + 1);
      }
      t = nt;
      cc = ncc;
    };
    for (int s = 0; s < S; s += 2) {
      step(s, rb2, rb);
      if (s + 1 < S) step(s + 1, rb, rb2);
    }
  }
  mfma_tile_epilogue<BMH, BN, WM, WN, true, BMH / 128, RED>(acc, smem, m0, n0, bx, stats, g, Y, ADD,
                                                           red);
}

int halo_rows_needed(const ConvGeom& g, int bm = HBM) {
  // worst case over blocks: a bm-pixel run starting at the last pixel of a row
  return ((g.W - 1 + bm - 1) / g.W + 3) * g.W;
}

template <int BN, int HR, int WM, int WN, int BMH = HBM, int PF = 1, bool RED = false, bool BWD = false>
void launch_halo(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                 const ConvGeom& g, const float* pre_sc, const float* pre_sh, hipStream_t st,
                 const BnBwdRed* red = nullptr, const BnBwdIn* bwd = nullptr) {
  constexpr int RPP = WM * WN * 8;
  const size_t main = (size_t)(RPP * HR + 1) * HBK * 2 + (size_t)2 * BN * HBK * 2 + MAXTAPS * 16 +
                      (BWD ? (size_t)5 * g.C * 4 : 0);
  const size_t epi = (size_t)128 * (BN + 4) * 4;  // staged in 128-row bands
  const size_t sm = main > epi ? main : epi;
  const unsigned mt = (unsigned)((g.M + BMH - 1) / BMH), nt = (g.Ncols + BN - 1) / BN;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  auto k = (RED || BWD) ? conv_halo_kernel<BN, HR, WM, WN, BMH, false, PF, RED, BWD>
         : pre_sc ? conv_halo_kernel<BN, HR, WM, WN, BMH, true, PF>
                  : conv_halo_kernel<BN, HR, WM, WN, BMH, false, PF>;
  const BnBwdRed rarg = red ? *red : BnBwdRed{};
  const BnBwdIn barg = bwd ? *bwd : BnBwdIn{};
  set_smem_attr(k, sm);
  // XCD-aware 1-D grid over the M tiles (padded to a multiple of 8) x N tiles: the N tiles of
  // one M tile share an XCD's L2.  Measured (tools/bench_conv.py, batch 512): layer3 fwd
  // 845 -> 880 TF/s, dgrad 859 -> 892; layer2 / layer4 +2-7 %
  if (nt > 1) {
    const unsigned mt8 = (mt + 7) / 8 * 8;
    k<<<dim3(mt8 * nt), WM * WN * 64, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, wb, pre_sc, pre_sh,
                                                (int)nt, (int)mt, rarg, barg);
    return;
  }
  k<<<dim3(mt, nt), WM * WN * 64, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, wb, pre_sc, pre_sh,
                                            0, (int)mt, rarg, barg);
}
}  // namespace

bool conv_halo_supported(const ConvGeom& g) {
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W) return false;
  if (g.C % HBK != 0 || g.nth * g.ntw > 16 || g.nth < 1 || g.ntw < 1) return false;
  const int dya = g.dy0, dyb = g.dy0 + (g.nth - 1) * g.dys;
  const int dxa = g.dx0, dxb = g.dx0 + (g.ntw - 1) * g.dxs;
  auto in1 = [](int v) { return v >= -1 && v <= 1; };
  if (!in1(dya) || !in1(dyb) || !in1(dxa) || !in1(dxb)) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  if ((long long)g.Ncols * g.wK * 2 >= (1LL << 31)) return false;
  return halo_rows_needed(g) <= 32 * 12 && halo_rows_needed(g, 256) <= 32 * 14;
}

// tiles (igemm_fwd's halo cfgs): waves 4 | 0x100 = 128 px as 2 x 2 waves of 64 x 64 with two
// weight tiles of register prefetch (cfg 42); 16 = 256 px as 4 x 2 waves of 64 x 32 (cfg 39);
// 32 = 256 px as 4 x 1 waves of 64 x 64 (cfg 41)
template <bool RED, bool BWD>
static void launch_halo42(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                          float* stats, const ConvGeom& g, int hp, hipStream_t st,
                          const BnBwdRed* red, const BnBwdIn* bwd) {
  const int hr = hp <= 192 ? 6 : hp <= 256 ? 8 : 12;
  if (hr == 6) launch_halo<128, 6, 2, 2, HBM, 2, RED, BWD>(X, Wp, Y, ADD, stats, g, nullptr, nullptr, st, red, bwd);
  else if (hr == 8) launch_halo<128, 8, 2, 2, HBM, 2, RED, BWD>(X, Wp, Y, ADD, stats, g, nullptr, nullptr, st, red, bwd);
  else launch_halo<128, 12, 2, 2, HBM, 2, RED, BWD>(X, Wp, Y, ADD, stats, g, nullptr, nullptr, st, red, bwd);
}

void conv_halo(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int bn, int waves, hipStream_t st, const float* pre_sc,
               const float* pre_sh, const BnBwdRed* red, const BnBwdIn* bwd) {
  const int hp = halo_rows_needed(g), hp2 = halo_rows_needed(g, 256);
  if (red || bwd) {
    // the BN-backward reduction epilogue and the folded BN-backward operand are built for the
    // cfg 42 tile (layer2's data gradient)
    if (waves != (4 | 0x100) || bn != 128 || pre_sc)
      throw std::runtime_error("conv_halo: BN-backward reduction / operand needs cfg 42, no PRE input");
    if (bwd && (!bwd->y || !bwd->coef || bwd->C != g.C))
      throw std::runtime_error("conv_halo: BN-backward operand needs y, coef and C == input channels");
    if (red && bwd) launch_halo42<true, true>(X, Wp, Y, ADD, stats, g, hp, st, red, bwd);
    else if (red) launch_halo42<true, false>(X, Wp, Y, ADD, stats, g, hp, st, red, bwd);
    else launch_halo42<false, true>(X, Wp, Y, ADD, stats, g, hp, st, red, bwd);
    DM_CHECK(hipGetLastError());
    return;
  }
  if (waves == (4 | 0x100) && bn == 128) {
    const int hr = hp <= 192 ? 6 : hp <= 256 ? 8 : 12;
    if (hr == 6) launch_halo<128, 6, 2, 2, HBM, 2>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else if (hr == 8) launch_halo<128, 8, 2, 2, HBM, 2>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else launch_halo<128, 12, 2, 2, HBM, 2>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
  } else if (waves == 16 && bn == 64) {
    const int hr = (hp2 + 63) / 64;
    if (hr <= 5) launch_halo<64, 5, 4, 2, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else if (hr <= 6) launch_halo<64, 6, 4, 2, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else launch_halo<64, 7, 4, 2, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
  } else if (waves == 32 && bn == 64) {
    const int hr = (hp2 + 31) / 32;
    if (hr <= 10) launch_halo<64, 10, 4, 1, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else if (hr <= 12) launch_halo<64, 12, 4, 1, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
    else launch_halo<64, 14, 4, 1, 256>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st);
  } else {
    throw std::runtime_error("conv_halo: unknown tile (cfg 39 / 41 / 42)");
  }
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
