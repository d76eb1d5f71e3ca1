// Stride-2 3x3 data gradient with all four parity classes in one block over one dY halo.
//
// dX of a 3x3/s2/p1 conv splits into the parity classes (a, b) of the input pixel
// (2p + a, 2q + b).  Each class is a unit-stride conv of dY over the dY grid (p, q) with
// 1, 2, 2 or 4 taps whose dY offsets lie in {0, +1}:
//     a = 0: kh = 1, dY row p          a = 1: kh = 0 -> dY row p + 1, kh = 2 -> dY row p
// The igemm path (conv_igemm.hip igemm_fwd_multi) runs the classes as blockIdx.z slices,
// each with its own 128-position tile and only 1-4 K-tiles of work (class (0,0): K = Cout),
// so prologue and epilogue dominate: layer2's dgrad ran at ~230 TFLOP/s.
//
// Here a block owns 128 consecutive dY positions m (flattened n, p, q) and all 9 (class,
// tap) steps of every 64-channel chunk: the dY halo rows r0-1 .. r1+1 of a chunk are staged
// into LDS once (as in conv_halo.hip) and every class reads its taps' A fragments from it;
// only the 64 x BN weight tile is staged per step (double-buffered through registers).  The
// four classes accumulate into four register tiles, written by the shared MFMA epilogue with
// the class's output geometry (pixel (2p + a, 2q + b)).  Requires even input H, W, so every
// class grid is the dY grid.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int S2BM = 128;  // dY positions per block
constexpr int S2BK = 64;   // dY channels per chunk
constexpr unsigned S2OOB = 0x80000000u;

// taps of the 4 classes, class-major: (dy, dx, packed-weight k offset, dy*W + dx)
struct S2Taps {
  int4 t[16];
  int end[4];  // cumulative tap count after class c
};

template <int BN, int HR, int WM, int WN>
__global__ void __launch_bounds__(WM * WN * 64, 2) dgrad_s2_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    ConvGeomSet set, S2Taps tp, unsigned xbytes, unsigned wbytes, int xcd, int mtiles, int diag) {
  // diag (DMLAB_S2_DIAG, timing only; results wrong when set): bit 0 drops the MFMAs, bit 1
  // the per-step weight loads, bit 2 the epilogue, bit 3 the per-step barriers
  const ConvGeom& g = set.g[0];  // the dY grid (shared by all classes)
  constexpr int TM = S2BM / WM, TN = BN / WN;
  constexpr int RM = TM / 32, RN = TN / 32;
  constexpr int NT = WM * WN * 64, RPP = NT / 8;
  constexpr int BR = BN / RPP;
  static_assert(BR * RPP == BN && RM >= 1 && RN >= 1, "tile / wave layout");
  constexpr int HP_MAX = RPP * HR;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hs = reinterpret_cast<bf16_t*>(smem);  // [HP_MAX + 1][64], last row = zeros
  bf16_t* Bs = Hs + (HP_MAX + 1) * S2BK;          // [2][BN][64]
  int4* taps = reinterpret_cast<int4*>(Bs + 2 * BN * S2BK);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  // xcd > 0: the N tiles of one M tile run back to back on one XCD (as in conv_halo.hip)
  int bx = blockIdx.x, by = blockIdx.y;
  if (xcd) {
    const int b = blockIdx.x, j = b >> 3;
    by = j % xcd;
    bx = (j / xcd) * 8 + (b & 7);
    if (bx >= mtiles) return;
  }
  const long long m0 = (long long)bx * S2BM;
  const int n0 = by * BN;
  const int ntaps = tp.end[3];
  const int nchunk = g.C / S2BK;
  const int NHW = g.N * g.H * g.W;
  if (tid < ntaps) taps[tid] = tp.t[tid];
  if (tid < 8) *reinterpret_cast<uint4*>(Hs + HP_MAX * S2BK + tid * 8) = make_uint4(0, 0, 0, 0);

  const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
  const long long mlast = (m0 + S2BM - 1 < g.M) ? m0 + S2BM - 1 : g.M - 1;
  const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
  const int hbase = (r0 - 1) * g.W;
  const int hp = (r1 - r0 + 3) * g.W;

  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, (int)wbytes, 0x00020000);
  const int chunk = tid & 7;

  int a_h[RM], a_x[RM], a_y[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const long long m = m0 + wm * TM + i * 32 + (lane & 31);
    const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
    a_x[i] = (int)((unsigned)m - r * (unsigned)g.W);
    const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
    a_y[i] = (m < g.M) ? (int)(r - n * (unsigned)g.H) : -(1 << 28);
    a_h[i] = (int)(m - hbase);
  }
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = n0 + (tid >> 3) + RPP * i;
    b_off[i] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u : S2OOB;
  }
  __syncthreads();

  uint4 rh[HR], rb[BR];
  auto load_halo = [&](int cc) {
    const unsigned cb = (unsigned)(cc * S2BK + chunk * 8) * 2u;
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      const int gp = hbase + hh;
      const bool ok = hh < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? (unsigned)gp * (unsigned)g.C * 2u + cb : S2OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      *reinterpret_cast<uint4*>(Hs + hh * S2BK + swz(hh, chunk) * 8) = rh[j];
    }
  };
  auto load_b = [&](int cc, int t) {
    if (diag & 2) return;
    const unsigned kb = (unsigned)(taps[t].z + cc * S2BK + chunk * 8) * 2u;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const unsigned off = b_off[i] != S2OOB ? b_off[i] + kb : S2OOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsw, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_b = [&](int buf) {
    bf16_t* bs = Bs + buf * BN * S2BK;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = (tid >> 3) + RPP * i;
      *reinterpret_cast<uint4*>(bs + r * S2BK + swz(r, chunk) * 8) = rb[i];
    }
  };

  f32x16 acc[4][RM][RN];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[c][i][j][r] = 0.f;

  auto compute = [&](f32x16 (&ac)[RM][RN], int buf, int t) {
    if (diag & 1) return;
    const int4 tv = taps[t];
    int hrow[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const bool ok = (unsigned)(a_x[i] + tv.y) < (unsigned)g.W &&
                      (unsigned)(a_y[i] + tv.x) < (unsigned)g.H;
      hrow[i] = ok ? a_h[i] + tv.w : HP_MAX;
    }
    const bf16_t* bs = Bs + buf * BN * S2BK;
    bf16x8 af[2][RM], bfr[2][RN];
    auto frag = [&](int ks, int s) {
      const int ch = ks * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < RM; ++i)
        af[s][i] = *reinterpret_cast<const bf16x8*>(Hs + hrow[i] * S2BK + swz(hrow[i], ch) * 8);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int r = wn * TN + j * 32 + (lane & 31);
        bfr[s][j] = *reinterpret_cast<const bf16x8*>(bs + r * S2BK + swz(r, ch) * 8);
      }
    };
    frag(0, 0);
#pragma unroll
    for (int ks = 0; ks < S2BK / 16; ++ks) {
      if (ks + 1 < S2BK / 16) frag(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          ac[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bfr[ks & 1][j],
                                                             ac[i][j], 0, 0, 0);
    }
  };

  const int S = nchunk * ntaps;
  load_halo(0);
  load_b(0, 0);
  store_halo();
  store_b(0);
  __syncthreads();
  if (nchunk > 1) load_halo(1);
  int s = 0;
  for (int cc = 0; cc < nchunk; ++cc) {
    int t = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int tend = tp.end[c];
      for (; t < tend; ++t, ++s) {
        int nt = t + 1, ncc = cc;
        if (nt == ntaps) {
          nt = 0;
          ++ncc;
        }
        if (s + 1 < S) load_b(ncc, nt);
        compute(acc[c], s & 1, t);
        if (s + 1 < S) store_b((s + 1) & 1);
        if (!(diag & 8)) __syncthreads();
      }
    }
    if (cc + 1 < nchunk) {
      store_halo();  // every wave is past the last tap of chunk cc
      __syncthreads();
      if (cc + 2 < nchunk) load_halo(cc + 2);
    }
  }
  if (diag & 4) return;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c) __syncthreads();  // the previous class's staged tile has been read
    mfma_tile_epilogue<S2BM, BN, WM, WN, true, 1>(acc[c], smem, m0, n0, 0, nullptr, set.g[c], Y,
                                                  ADD);
  }
}

int s2_halo_rows(const ConvGeom& g) { return ((g.W - 1 + S2BM - 1) / g.W + 3) * g.W; }

template <int BN, int HR, int WM, int WN>
void launch_s2(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
               const ConvGeomSet& set, const S2Taps& tp, hipStream_t st) {
  const ConvGeom& g = set.g[0];
  constexpr int RPP = WM * WN * 8;
  const size_t main = (size_t)(RPP * HR + 1) * S2BK * 2 + (size_t)2 * BN * S2BK * 2 + 16 * 16;
  const size_t epi = (size_t)S2BM * (BN + 4) * 4;
  const size_t sm = main > epi ? main : epi;
  const unsigned gx = (unsigned)((g.M + S2BM - 1) / S2BM), gy = (g.Ncols + BN - 1) / BN;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  auto k = dgrad_s2_kernel<BN, HR, WM, WN>;
  set_smem_attr(k, sm);
  static const int diag = getenv("DMLAB_S2_DIAG") ? atoi(getenv("DMLAB_S2_DIAG")) : 0;
  if (gy > 1) {
    const unsigned mt8 = (gx + 7) / 8 * 8;
    k<<<dim3(mt8 * gy), WM * WN * 64, sm, st>>>(X, Wp, Y, ADD, set, tp, xb, wb, (int)gy, (int)gx, diag);
  } else {
    k<<<dim3(gx, 1), WM * WN * 64, sm, st>>>(X, Wp, Y, ADD, set, tp, xb, wb, 0, (int)gx, diag);
  }
}
}  // namespace

bool dgrad_s2_supported(const ConvGeomSet& set, int ng) {
  if (ng != 4) return false;
  const ConvGeom& g = set.g[0];
  if (g.C % S2BK != 0 || g.Ncols % 64 != 0) return false;
  int ntaps = 0;
  for (int c = 0; c < 4; ++c) {
    const ConvGeom& q = set.g[c];
    // every class grid is the dY grid (even input size), unit-stride taps within +-1
    if (q.Hg != g.H || q.Wg != g.W || q.H != g.H || q.W != g.W || q.M != g.M) return false;
    if (q.isy != 1 || q.isx != 1 || q.osy != 2 || q.osx != 2) return false;
    const int dya = q.dy0, dyb = q.dy0 + (q.nth - 1) * q.dys;
    const int dxa = q.dx0, dxb = q.dx0 + (q.ntw - 1) * q.dxs;
    auto in1 = [](int v) { return v >= -1 && v <= 1; };
    if (!in1(dya) || !in1(dyb) || !in1(dxa) || !in1(dxb)) return false;
    ntaps += q.nth * q.ntw;
  }
  if (ntaps > 16) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  if ((long long)g.Ncols * g.wK * 2 >= (1LL << 31)) return false;
  if (g.M >= (1LL << 31)) return false;
  return s2_halo_rows(g) <= 32 * 8;
}

void dgrad_s2(const bf16_t* dY, const bf16_t* Wd, bf16_t* dX, const bf16_t* ADD,
              const ConvGeomSet& set, hipStream_t st) {
  S2Taps tp{};
  int k = 0;
  for (int c = 0; c < 4; ++c) {
    const ConvGeom& q = set.g[c];
    for (int th = 0; th < q.nth; ++th)
      for (int tw = 0; tw < q.ntw; ++tw) {
        const int dy = q.dy0 + th * q.dys, dx = q.dx0 + tw * q.dxs;
        const int wz = ((q.kh0 + th * q.khs) * q.KW + (q.kw0 + tw * q.kws)) * q.C;
        tp.t[k++] = make_int4(dy, dx, wz, dy * q.W + dx);
      }
    tp.end[c] = k;
  }
  const int hr = (s2_halo_rows(set.g[0]) + 31) / 32;
  if (hr <= 5) launch_s2<64, 5, 2, 2>(dY, Wd, dX, ADD, set, tp, st);
  else if (hr <= 6) launch_s2<64, 6, 2, 2>(dY, Wd, dX, ADD, set, tp, st);
  else if (hr <= 7) launch_s2<64, 7, 2, 2>(dY, Wd, dX, ADD, set, tp, st);
  else launch_s2<64, 8, 2, 2>(dY, Wd, dX, ADD, set, tp, st);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
