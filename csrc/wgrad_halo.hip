// Halo-staged weight gradient for 3x3 / unit-stride / pad-1 convolutions, gfx950.
//
//   dW[co, tap, c] = Σ_m dY[m, co] · X[m + dy_t*W + dx_t, c]        (m = flattened n, y, x)
//
// The igemm wgrad kernel (conv_igemm.hip) stages one (tap, channel) column block of the
// implicit im2col matrix per K-tile, so each block re-fetches the same input pixels once
// per tap and re-stages the dY tile for every K-tile — measured 250-470 TFLOP/s.
//
// Here a block owns 64 output channels x ALL 9 taps x 64 input channels (a 64 x 576
// gradient tile) and walks a slice of m in steps of 64 pixels.  Per step it stages
//   * the dY tile   [64 m][64 co]                      (8 KB), and
//   * the input halo [64 + 2W + 2 pixels][64 c]        (the pixels every tap of the 64
//     rows touches: m0 - W - 1 ... m0 + 64 + W, contiguous in the flattened NHWC layout)
// once, and the 9 taps read their B fragments straight out of the halo at row offset
// dy*W + dx.  One dY fragment feeds 9 MFMAs; per step the block issues 2 x 4 x 9 x 4
// v_mfma_f32_16x16x32_bf16 against ~31 KB of staging (vs 2.1 MFLOP per 24 KB before).
// A tap whose source pixel leaves the image (x+dx or y+dy out of range) reads an all-zero
// LDS row instead — exactly the conv's zero padding, also across the row / image
// boundaries of the flattened layout.  Rows past the block's m-slice have zero dY.
//
// Both operands are m-major in memory and in LDS, so fragments come from the CDNA4
// transpose read ds_read_b64_tr_b16 (row pitch 80 elements: conflict-free, see
// docs/KERNELS.md).  Waves split the 64 input channels (16 each) and share the dY
// fragments.  The m reduction is split over blocks into fp32 slabs [S][Cout][9*C] reduced
// by wgrad_reduce (fixed order, deterministic).
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <stdexcept>

namespace dm {

namespace {
constexpr int WBM = 64;    // output channels per block
constexpr int WBC = 64;    // input channels per block
constexpr int WBK = 64;    // m rows per step
constexpr int WPITCH = 80; // LDS row pitch (elements) for the transpose reads
constexpr unsigned WOOB = 0x80000000u;

typedef short s4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4*)p);
}

// NTY = kernel rows (dy values) per block: 3 = all 9 taps share the dY fragments; 1 = one
// row of 3 taps (smaller halo, 3x more output tiles -> 3x fewer m-splits and slab bytes)
// BWD: DY is a BatchNorm's OUTPUT gradient dz; the dY operand is that BN's backward
// dy = a*dz' + b*y + c (kernels.h BnBwdIn), computed while staging (no dy tensor)
template <int HRN, int NTY, bool PRE, bool BWD = false>
__global__ void __launch_bounds__(256, 2) wgrad_halo_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY, float* __restrict__ slab,
    ConvGeom g, long long mchunk, unsigned xbytes, unsigned dybytes,
    const float* __restrict__ pre_sc, const float* __restrict__ pre_sh, int xy, int gx, int nz,
    BnBwdIn bwd) {
  // pre_sc/pre_sh (optional): X is the previous conv's raw output; the operand is
  // relu(x*sc + sh) applied while staging (out-of-image taps read the zero row)
  constexpr int HROWS_MAX = HRN * 32;  // halo rows a buffer holds (8 chunks per row)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);            // [2][64][WPITCH] dY
  bf16_t* Hs = As + 2 * WBK * WPITCH;                       // [2][HROWS_MAX][WPITCH] input
  bf16_t* Zr = Hs + 2 * HROWS_MAX * WPITCH;                 // one zero row
  float* btab = reinterpret_cast<float*>(Zr + WPITCH);      // BWD: [5][64] coefficients

  constexpr int NT = 3 * NTY;  // taps per block
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // block -> (co tile bx, channel/row tile by, m slice bz).  xy > 0 (1-D grid): the xy tiles
  // of one m slice are consecutive blocks on one XCD (blocks go to the XCDs round-robin), so
  // the slice's dY rows and input halo are fetched into that XCD's L2 once
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (xy) {
    const int b = blockIdx.x, j = b >> 3, t = j % xy;
    bz = (j / xy) * 8 + (b & 7);
    if (bz >= nz) return;  // padding of the m slices to a multiple of 8
    bx = t % gx;
    by = t / gx;
  }
  const int co0 = bx * WBM;
  const int cc0 = (by / (3 / NTY)) * WBC;
  const int dy_lo = -1 + (int)(by % (3 / NTY)) * NTY;  // first kernel row of the block
  const long long mb = (long long)bz * mchunk;
  const long long me = min(g.M, mb + mchunk);
  const int W = g.W, H = g.H;
  const int hrows = WBK + 2 + (NTY - 1) * W;  // pixels m0 + dy_lo*W - 1 ... m0 + (dy_hi)*W + 64
  const int NHW = g.N * H * W;
  if (tid < WPITCH / 8) *reinterpret_cast<uint4*>(Zr + tid * 8) = make_uint4(0, 0, 0, 0);
  if constexpr (BWD) {
    bwd_tab_fill(btab, bwd, co0, WBM, tid, 256);
    __syncthreads();  // the first store below reads it
  }

  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsd = __builtin_amdgcn_make_buffer_rsrc((void*)DY, (short)0, (int)dybytes, 0x00020000);
  const int chunk = tid & 7, row0 = tid >> 3;  // staging: 32 rows x 8 chunks per pass

  uint4 ra[2], rh[HRN];
  unsigned raoff[BWD ? 2 : 1];  // BWD: the dY chunks' byte offsets (y and mask read at store)
  const auto rsy = __builtin_amdgcn_make_buffer_rsrc((void*)(BWD ? (const void*)bwd.y : (const void*)DY),
                                                     (short)0, (int)(BWD ? dybytes : 0u), 0x00020000);
  auto load = [&](long long m0) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long long m = m0 + row0 + 32 * i;
      const unsigned off = m < me ? (unsigned)((m * g.Ncols + co0 + chunk * 8) * 2) : WOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsd, off, 0, 0);
      ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
      if constexpr (BWD) raoff[i] = off;
    }
    const long long hb = m0 + dy_lo * W - 1;
#pragma unroll
    for (int j = 0; j < HRN; ++j) {
      const int h = row0 + 32 * j;
      const long long p = hb + h;
      const bool ok = h < hrows && p >= 0 && p < NHW;
      const unsigned off = ok ? (unsigned)((p * g.C + cc0 + chunk * 8) * 2) : WOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store = [&](int buf, long long m0) __attribute__((always_inline)) {
    bf16_t* as = As + buf * WBK * WPITCH;
    bf16_t* hs = Hs + buf * HROWS_MAX * WPITCH;
    if constexpr (BWD) {
      // rows past the m-slice keep their zero dY (the conv's reduction must not see them).
      // y and the mask are read here, not with the dY prefetch: held across the MFMA loop
      // they pushed the kernel (144 accumulator registers) into spills
      uint4 ry[2];
      unsigned rmk[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const auto w = __builtin_amdgcn_raw_buffer_load_b128(rsy, raoff[i], 0, 0);
        ry[i] = make_uint4(w[0], w[1], w[2], w[3]);
        rmk[i] = bwd_mask_byte(bwd, raoff[i], dybytes >> 4);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const uint4 v = bwd_apply<false>(btab, WBM, chunk * 8, ra[i], ry[i], rmk[i]);
        if (m0 + row0 + 32 * i < me) ra[i] = v;
      }
      __builtin_amdgcn_sched_barrier(0);  // its coefficients are dead before PreBN's load
    }
    PreBN pbn;  // PRE: loaded per store (L1 hits) instead of 16 registers live all kernel
    if constexpr (PRE) pbn.load(pre_sc, pre_sh, cc0 + chunk * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      *reinterpret_cast<uint4*>(as + (row0 + 32 * i) * WPITCH + chunk * 8) = ra[i];
#pragma unroll
    for (int j = 0; j < HRN; ++j)
      *reinterpret_cast<uint4*>(hs + (row0 + 32 * j) * WPITCH + chunk * 8) =
          PRE ? pbn.apply(rh[j]) : rh[j];
  };

  f32x4 acc[4][NT];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // transpose-read lane roles (as igemm_wgrad2): row grp*4+q (+16), column 4p
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int rbase = grp * 4 + q;
  const int nsteps = me > mb ? (int)((me - mb + WBK - 1) / WBK) : 0;
  if (nsteps > 0) {
    load(mb);
    store(0, mb);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const long long m0 = mb + (long long)s * WBK;
    if (s + 1 < nsteps) load(m0 + WBK);
    const bf16_t* as = As + buf * WBK * WPITCH;
    const bf16_t* hs = Hs + buf * HROWS_MAX * WPITCH;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      // pixel coordinates of this lane's two rows (lo: r, hi: r + 16)
      int xr[2], yr[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned m = (unsigned)(m0 + ks * 32 + rbase + 16 * u);
        const unsigned t = fdiv(m, g.wg_mul, g.wg_shr);
        xr[u] = (int)(m - t * (unsigned)W);
        const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
        yr[u] = (int)(t - n * (unsigned)H);
      }
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * p;
        const s4 lo = tr_read(as + (ks * 32 + rbase) * WPITCH + col);
        const s4 hi = tr_read(as + (ks * 32 + rbase + 16) * WPITCH + col);
        af[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int bcol = wid * 16 + 4 * p;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int dyl = t / 3, dx = t % 3 - 1;  // kernel row relative to dy_lo
        const int dy = dy_lo + dyl;
        const bf16_t* src[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bool ok = (unsigned)(xr[u] + dx) < (unsigned)W && (unsigned)(yr[u] + dy) < (unsigned)H;
          const int h = ks * 32 + rbase + 16 * u + 1 + dyl * W + dx;
          src[u] = ok ? hs + h * WPITCH + bcol : Zr + 4 * p;
        }
        const s4 lo = tr_read(src[0]);
        const s4 hi = tr_read(src[1]);
        const bf16x8 bfr = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][t], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) store(buf ^ 1, m0 + WBK);
    __syncthreads();
  }
  // slab[z][co][tap*C + c]; 16x16 C map: col = lane & 15 (channel), row = (lane>>4)*4 + r (co)
  float* out = slab + (long long)bz * g.Ncols * g.K;
  const int c = cc0 + wid * 16 + (lane & 15);
  const int t0 = (dy_lo + 1) * 3;  // global tap index of the block's first tap
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + i * 16 + (lane >> 4) * 4 + r;
        if (co < g.Ncols) out[(long long)co * g.K + (t0 + t) * g.C + c] = acc[i][t][r];
      }
}

// ---------------------------------------------------------------- stride 2 (wgrad cfg 7)
// 3x3 / stride-2 / pad-1 weight gradient of an even-sized input (the first conv of layers
// 2-4).  Output pixel m = (n, y, x) reads input (2y + dy, 2x + dx), dy, dx in {-1, 0, 1}.
// The input splits into four parity planes P(a, b) = pixels (2i + a, 2j + b), each indexed
// exactly like the output (q = (n*Ho + i)*Wo + j), and tap (dy, dx) of pixel m reads plane
// (dy & 1, dx & 1) at q = m + di*Wo + dj with di = (dy < 0 ? -1 : 0), dj likewise: per plane a
// CONSTANT offset, as in the stride-1 kernel.  A step stages MR dY rows and, per plane, the
// flattened range [m0 - lead, m0 + MR) its taps touch (lead 0, 1, Wo, Wo + 1 for planes
// (0,0), (0,1), (1,0), (1,1): 4 MR + 2 Wo + 2 rows), and all 9 taps read B fragments from it.
// MR: m rows per step (32: two workgroups per CU fit the LDS)
template <int HRN, int MR>
__global__ void __launch_bounds__(256, MR == 32 ? 2 : 1) wgrad_s2_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY, float* __restrict__ slab,
    ConvGeom g, long long mchunk, unsigned xbytes, unsigned dybytes, int xy, int gx, int nz) {
  constexpr int HROWS_MAX = HRN * 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);            // [2][MR][WPITCH] dY
  bf16_t* Hs = As + 2 * MR * WPITCH;                        // [2][HROWS_MAX][WPITCH] planes
  bf16_t* Zr = Hs + 2 * HROWS_MAX * WPITCH;                 // one zero row
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (xy) {  // XCD-grouped 1-D grid, as the stride-1 kernel
    const int b = blockIdx.x, j = b >> 3, t = j % xy;
    bz = (j / xy) * 8 + (b & 7);
    if (bz >= nz) return;
    bx = t % gx;
    by = t / gx;
  }
  const int co0 = bx * WBM;
  const int cc0 = by * WBC;
  const long long mb = (long long)bz * mchunk;
  const long long me = min(g.M, mb + mchunk);
  const int Wo = g.Wg, Ho = g.Hg, Wi = g.W, Hi = g.H;
  // plane row bases in LDS and leads: plane p = a*2 + b
  const int lead1 = 1, lead2 = Wo, lead3 = Wo + 1;
  const int base1 = MR, base2 = base1 + MR + lead1, base3 = base2 + MR + lead2;
  const int hrows = base3 + MR + lead3;
  const long long NQ = g.M;  // plane positions (= output pixels)
  if (tid < WPITCH / 8) *reinterpret_cast<uint4*>(Zr + tid * 8) = make_uint4(0, 0, 0, 0);

  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsd = __builtin_amdgcn_make_buffer_rsrc((void*)DY, (short)0, (int)dybytes, 0x00020000);
  const int chunk = tid & 7, row0 = tid >> 3;

  uint4 ra[MR / 32], rh[HRN];
  auto load = [&](long long m0) {
#pragma unroll
    for (int i = 0; i < MR / 32; ++i) {
      const long long m = m0 + row0 + 32 * i;
      const unsigned off = m < me ? (unsigned)((m * g.Ncols + co0 + chunk * 8) * 2) : WOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsd, off, 0, 0);
      ra[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
#pragma unroll
    for (int j = 0; j < HRN; ++j) {
      const int h = row0 + 32 * j;
      int a, b;
      long long q;
      if (h < base1) { a = 0; b = 0; q = m0 + h; }
      else if (h < base2) { a = 0; b = 1; q = m0 - lead1 + (h - base1); }
      else if (h < base3) { a = 1; b = 0; q = m0 - lead2 + (h - base2); }
      else { a = 1; b = 1; q = m0 - lead3 + (h - base3); }
      unsigned off = WOOB;
      if (h < hrows && q >= 0 && q < NQ) {
        const unsigned t = fdiv((unsigned)q, g.wg_mul, g.wg_shr);
        const int jj = (int)((unsigned)q - t * (unsigned)Wo);
        const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
        const int ii = (int)(t - n * (unsigned)Ho);
        const int yi = 2 * ii + a, xi = 2 * jj + b;
        if (yi < Hi && xi < Wi)
          off = (unsigned)(((((long long)n * Hi + yi) * Wi + xi) * g.C + cc0 + chunk * 8) * 2);
      }
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store = [&](int buf) {
    bf16_t* as = As + buf * MR * WPITCH;
    bf16_t* hs = Hs + buf * HROWS_MAX * WPITCH;
#pragma unroll
    for (int i = 0; i < MR / 32; ++i)
      *reinterpret_cast<uint4*>(as + (row0 + 32 * i) * WPITCH + chunk * 8) = ra[i];
#pragma unroll
    for (int j = 0; j < HRN; ++j)
      *reinterpret_cast<uint4*>(hs + (row0 + 32 * j) * WPITCH + chunk * 8) = rh[j];
  };

  constexpr int NTAP = 9;
  f32x4 acc[4][NTAP];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NTAP; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int grp = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int rbase = grp * 4 + q4;
  const int nsteps = me > mb ? (int)((me - mb + MR - 1) / MR) : 0;
  if (nsteps > 0) {
    load(mb);
    store(0);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    const long long m0 = mb + (long long)s * MR;
    if (s + 1 < nsteps) load(m0 + MR);
    const bf16_t* as = As + buf * MR * WPITCH;
    const bf16_t* hs = Hs + buf * HROWS_MAX * WPITCH;
#pragma unroll
    for (int ks = 0; ks < MR / 32; ++ks) {
      int xr[2], yr[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const unsigned m = (unsigned)(m0 + ks * 32 + rbase + 16 * u);
        const unsigned t = fdiv(m, g.wg_mul, g.wg_shr);
        xr[u] = (int)(m - t * (unsigned)Wo);
        const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
        yr[u] = (int)(t - n * (unsigned)Ho);
      }
      bf16x8 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = i * 16 + 4 * p4;
        const s4 lo = tr_read(as + (ks * 32 + rbase) * WPITCH + col);
        const s4 hi = tr_read(as + (ks * 32 + rbase + 16) * WPITCH + col);
        af[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const int bcol = wid * 16 + 4 * p4;
#pragma unroll
      for (int t = 0; t < NTAP; ++t) {
        const int dy = t / 3 - 1, dx = t % 3 - 1;
        const int a = dy & 1, b = dx & 1;
        const int pbase = a ? (b ? base3 + lead3 : base2 + lead2) : (b ? base1 + lead1 : 0);
        const int poff = (dy < 0 ? -Wo : 0) + (dx < 0 ? -1 : 0);
        const bf16_t* src[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const bool ok = (unsigned)(2 * xr[u] + dx) < (unsigned)Wi &&
                          (unsigned)(2 * yr[u] + dy) < (unsigned)Hi;
          const int h = pbase + ks * 32 + rbase + 16 * u + poff;
          src[u] = ok ? hs + h * WPITCH + bcol : Zr + 4 * p4;
        }
        const s4 lo = tr_read(src[0]);
        const s4 hi = tr_read(src[1]);
        const bf16x8 bfr = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[i][t], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }
  float* out = slab + (long long)bz * g.Ncols * g.K;
  const int c = cc0 + wid * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < NTAP; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + i * 16 + (lane >> 4) * 4 + r;
        if (co < g.Ncols) out[(long long)co * g.K + t * g.C + c] = acc[i][t][r];
      }
}

template <int HRN, int MR>
void launch_wgrad_s2(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                     long long mchunk, hipStream_t st) {
  const size_t sm = ((size_t)2 * MR * WPITCH + (size_t)2 * HRN * 32 * WPITCH + WPITCH) * 2;
  dim3 grid((g.Ncols + WBM - 1) / WBM, g.C / WBC, S);
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned db = (unsigned)(g.M * g.Ncols * 2);
  auto k = wgrad_s2_kernel<HRN, MR>;
  set_smem_attr(k, sm);
  const int xy = (int)(grid.x * grid.y);
  if (xy > 1 && S > 1) {
    const unsigned z8 = (unsigned)((S + 7) / 8 * 8);
    k<<<dim3(z8 * xy), 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db, xy, (int)grid.x, S);
    return;
  }
  k<<<grid, 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db, 0, (int)grid.x, S);
}

template <int HRN, int NTY, bool BWD = false>
void launch_wgrad_halo(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                       long long mchunk, hipStream_t st, const float* pre_sc,
                       const float* pre_sh, const BnBwdIn* bwd = nullptr) {
  const size_t sm = ((size_t)2 * WBK * WPITCH + (size_t)2 * HRN * 32 * WPITCH + WPITCH) * 2 +
                    (BWD ? (size_t)5 * WBM * 4 : 0);
  dim3 grid((g.Ncols + WBM - 1) / WBM, (g.C / WBC) * (3 / NTY), S);
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned db = (unsigned)(g.M * g.Ncols * 2);
  const BnBwdIn barg = bwd ? *bwd : BnBwdIn{};
  auto k = pre_sc ? wgrad_halo_kernel<HRN, NTY, true, BWD> : wgrad_halo_kernel<HRN, NTY, false, BWD>;
  set_smem_attr(k, sm);
  // XCD-grouped order for the 9-tap tiles.  Measured (tools/bench_conv.py, one call): 9-tap
  // layer2 +2-4 %, layer3/4 within 1 %, step 11.55 vs 11.57 ms; the 3-tap tiles lose (layer1
  // 526 -> 475 TF/s) and keep the 3-D grid
  const int xy = (int)(grid.x * grid.y);
  if (NTY == 3 && xy > 1 && S > 1) {
    const unsigned z8 = (unsigned)((S + 7) / 8 * 8);
    k<<<dim3(z8 * xy), 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db, pre_sc, pre_sh, xy,
                                       (int)grid.x, S, barg);
    return;
  }
  k<<<grid, 256, sm, st>>>(X, DY, slab, g, mchunk, xb, db, pre_sc, pre_sh, 0, (int)grid.x, S, barg);
}
}  // namespace

bool wgrad_halo_supported(const ConvGeom& g) {
  // 3x3, unit stride, pad 1, tap order (kh, kw) row-major with dy = kh - 1, dx = kw - 1
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W) return false;
  if (g.nth != 3 || g.ntw != 3 || g.dy0 != -1 || g.dys != 1 || g.dx0 != -1 || g.dxs != 1) return false;
  if (g.kh0 != 0 || g.khs != 1 || g.kw0 != 0 || g.kws != 1 || g.KW != 3) return false;
  if (g.C % WBC != 0 || g.Ncols % 8 != 0 || g.K != 9 * g.C) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31) || g.M * g.Ncols * 2 >= (1LL << 31))
    return false;
  return WBK + 2 * g.W + 2 <= 6 * 32;
}

bool wgrad_s2_supported(const ConvGeom& g) {
  // 3x3, stride 2, pad 1, even input (output = input / 2), tap order (kh, kw) row-major
  if (g.isy != 2 || g.isx != 2 || g.H != 2 * g.Hg || g.W != 2 * g.Wg) return false;
  if (g.nth != 3 || g.ntw != 3 || g.dy0 != -1 || g.dys != 1 || g.dx0 != -1 || g.dxs != 1) return false;
  if (g.kh0 != 0 || g.khs != 1 || g.kw0 != 0 || g.kws != 1 || g.KW != 3) return false;
  if (g.C % WBC != 0 || g.Ncols % 8 != 0 || g.K != 9 * g.C) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31) || g.M * g.Ncols * 2 >= (1LL << 31))
    return false;
  return 4 * 32 + 2 * g.Wg + 2 <= 6 * 32;
}

void wgrad_s2(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
              long long mchunk, hipStream_t st) {
  if (!wgrad_s2_supported(g)) throw std::runtime_error("wgrad_s2: unsupported geometry");
  // 32-row steps: 72 KB of LDS, two workgroups per CU (64-row steps, one per CU, lost 0.7 %:
  // profiles/wgrad_s2_ab_r4al.txt, profiles/wgrad_s2_mr_ab_r4am.txt)
  const int rows = 4 * 32 + 2 * g.Wg + 2;
  if (rows <= 5 * 32) launch_wgrad_s2<5, 32>(X, DY, slab, g, S, mchunk, st);
  else launch_wgrad_s2<6, 32>(X, DY, slab, g, S, mchunk, st);
  DM_CHECK(hipGetLastError());
}

void wgrad_halo(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                long long mchunk, int nty, hipStream_t st, const float* pre_sc,
                const float* pre_sh, const BnBwdIn* bwd) {
  if (bwd) {  // the folded BN-backward dY operand: the 9-tap tiles (wgrad cfg 4)
    if (nty != 3 || !bwd->y || !bwd->coef || bwd->C != g.Ncols)
      throw std::runtime_error("wgrad_halo: BN-backward operand needs the 9-tap tile, y, coef, "
                               "C == output channels");
    const int rows = WBK + 2 * g.W + 2;
    if (rows <= 96) launch_wgrad_halo<3, 3, true>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh, bwd);
    else if (rows <= 128) launch_wgrad_halo<4, 3, true>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh, bwd);
    else launch_wgrad_halo<6, 3, true>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh, bwd);
    DM_CHECK(hipGetLastError());
    return;
  }
  if (nty == 1) {
    launch_wgrad_halo<3, 1>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh);  // 66 rows
  } else {
    const int rows = WBK + 2 * g.W + 2;
    if (rows <= 96) launch_wgrad_halo<3, 3>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh);
    else if (rows <= 128) launch_wgrad_halo<4, 3>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh);
    else launch_wgrad_halo<6, 3>(X, DY, slab, g, S, mchunk, st, pre_sc, pre_sh);
  }
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
