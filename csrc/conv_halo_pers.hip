// Persistent variant of the single-chunk halo conv (cfg 39 shape: 64 input channels, 64
// output channels, 256-pixel tiles, 4 x 2 waves), gfx950.
//
// With one 64-channel chunk (ResNet layer 1) the per-tile kernel (conv_halo.hip) starts every
// block by loading its whole input halo (~57 KB) and the first weight tile, and nothing hides
// that latency but the other resident block.  Here two workgroups per CU loop over the M
// tiles: while tile i finishes, the halo of tile i+1 is already in flight in the
// staging registers (issued before tile i's epilogue, so it lands while the epilogue runs:
// held across the tap loop the 28 staging registers would spill at 128 VGPRs), and the last
// tap step loads tile i+1's first weight tile.  The epilogue (BN statistics, LDS staging,
// coalesced stores) is unchanged and still follows the taps of each tile.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int PBK = 64;    // channels (the single chunk)
constexpr int PBN = 64;    // output channels
constexpr int PBM = 256;   // pixels per tile
constexpr int PWM = 4, PWN = 2;
constexpr unsigned POOB = 0x80000000u;

template <int HR, bool PRE>
__global__ void __launch_bounds__(PWM * PWN * 64, 4) conv_halo_pers_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, unsigned wbytes,
    const float* __restrict__ pre_sc, const float* __restrict__ pre_sh, int mtiles) {
  constexpr int TM = PBM / PWM, TN = PBN / PWN;
  constexpr int RM = TM / 32, RN = TN / 32;
  constexpr int NT = PWM * PWN * 64, RPP = NT / 8;
  constexpr int BR = PBN / RPP;
  constexpr int HP_MAX = RPP * HR;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hs = reinterpret_cast<bf16_t*>(smem);  // [HP_MAX + 1][64], last row = zeros
  bf16_t* Bs = Hs + (HP_MAX + 1) * PBK;           // [2][64][64]
  int4* taps = reinterpret_cast<int4*>(Bs + 2 * PBN * PBK);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / PWN, wn = wid % PWN;
  const int ntaps = g.nth * g.ntw;
  const int NHW = g.N * g.H * g.W;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    taps[tid] = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * g.C,
                          dy * g.W + dx);
  }
  if (tid < 8) *reinterpret_cast<uint4*>(Hs + HP_MAX * PBK + tid * 8) = make_uint4(0, 0, 0, 0);
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)Wp, (short)0, (int)wbytes, 0x00020000);
  const int chunk = tid & 7;
  unsigned b_off[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int n = (tid >> 3) + RPP * i;
    b_off[i] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u : POOB;
  }
  // halo extent of a tile: flattened rows r0-1 .. r1+1
  auto geom = [&](int tile, int& hbase, int& hp) {
    const long long m0 = (long long)tile * PBM;
    const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
    const long long mlast = (m0 + PBM - 1 < g.M) ? m0 + PBM - 1 : g.M - 1;
    const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
    hbase = (r0 - 1) * g.W;
    hp = (r1 - r0 + 3) * g.W;
  };
  uint4 rh[HR], rb[BR];
  auto load_halo = [&](int hbase, int hp) {
    const unsigned cb = (unsigned)(chunk * 8) * 2u;
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      const int gp = hbase + hh;
      const bool ok = hh < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? (unsigned)gp * (unsigned)g.C * 2u + cb : POOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int j = 0; j < HR; ++j) {
      const int hh = (tid >> 3) + RPP * j;
      *reinterpret_cast<uint4*>(Hs + hh * PBK + swz(hh, chunk) * 8) = rh[j];
    }
    if constexpr (PRE) {
      PreBN pbn;
      pbn.load(pre_sc, pre_sh, chunk * 8);
#pragma unroll
      for (int j = 0; j < HR; ++j) {
        const int hh = (tid >> 3) + RPP * j;
        uint4* q = reinterpret_cast<uint4*>(Hs + hh * PBK + swz(hh, chunk) * 8);
        *q = pbn.apply(*q);
      }
    }
  };
  auto load_b = [&](int t) {
    const unsigned kb = (unsigned)(taps[t].z + chunk * 8) * 2u;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const unsigned off = b_off[i] != POOB ? b_off[i] + kb : POOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsw, off, 0, 0);
      rb[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_b = [&](int buf) {
    bf16_t* bs = Bs + buf * PBN * PBK;
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = (tid >> 3) + RPP * i;
      *reinterpret_cast<uint4*>(bs + r * PBK + swz(r, chunk) * 8) = rb[i];
    }
  };
  __syncthreads();  // taps table

  int tile = blockIdx.x;
  int hbase, hp;
  geom(tile, hbase, hp);
  load_halo(hbase, hp);
  load_b(0);
  int s = 0;  // global tap step (LDS weight buffer parity)
  for (; tile < mtiles; tile += gridDim.x) {
    const long long m0 = (long long)tile * PBM;
    const int cur_hbase = hbase;
    __syncthreads();  // the previous tile's epilogue has read the staging LDS
    store_halo();
    store_b(s & 1);
    if (tid < 8) *reinterpret_cast<uint4*>(Hs + HP_MAX * PBK + tid * 8) = make_uint4(0, 0, 0, 0);
    int a_h[RM], a_x[RM], a_y[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const long long m = m0 + wm * TM + i * 32 + (lane & 31);
      const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      a_x[i] = (int)((unsigned)m - r * (unsigned)g.W);
      const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
      a_y[i] = (m < g.M) ? (int)(r - n * (unsigned)g.H) : -(1 << 28);
      a_h[i] = (int)(m - cur_hbase);
    }
    __syncthreads();
    const int next = tile + (int)gridDim.x;
    f32x16 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int t = 0; t < ntaps; ++t, ++s) {
      const bool more = t + 1 < ntaps;
      if (more || next < mtiles) load_b(more ? t + 1 : 0);  // the next tile's tap 0 at the end
      const int4 tp = taps[t];
      int hrow[RM];
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        const bool ok = (unsigned)(a_x[i] + tp.y) < (unsigned)g.W &&
                        (unsigned)(a_y[i] + tp.x) < (unsigned)g.H;
        hrow[i] = ok ? a_h[i] + tp.w : HP_MAX;
      }
      const bf16_t* bs = Bs + (s & 1) * PBN * PBK;
      // single-buffered fragments: the next tile's halo occupies the registers the
      // per-tile kernel spends on reading k-substep ks+1 during the MFMAs of ks
#pragma unroll
      for (int ks = 0; ks < PBK / 16; ++ks) {
        const int ch = ks * 2 + (lane >> 5);
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i)
          af[i] = *reinterpret_cast<const bf16x8*>(Hs + hrow[i] * PBK + swz(hrow[i], ch) * 8);
#pragma unroll
        for (int j = 0; j < RN; ++j) {
          const int r = wn * TN + j * 32 + (lane & 31);
          bfr[j] = *reinterpret_cast<const bf16x8*>(bs + r * PBK + swz(r, ch) * 8);
        }
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
      if (more) store_b((s + 1) & 1);
      __syncthreads();
    }
    if (next < mtiles) {  // the next tile's halo lands while this tile's epilogue runs
      geom(next, hbase, hp);
      load_halo(hbase, hp);
    }
    mfma_tile_epilogue<PBM, PBN, PWM, PWN, true, PBM / 128>(acc, smem, m0, 0, tile, stats, g, Y,
                                                            ADD);
  }
}
}  // namespace

// Opt-in (DMLAB_HALO_PERS=1): measured slower.  Held through the epilogue, the prefetched
// halo pushes the kernel past 128 VGPRs (29-46 spilled) and the tap loop reads its fragments
// single-buffered: layer-1 forward 475 vs 525-534 TFLOP/s, dgrad 506-520 vs 567-570, end to
// end 43.17-43.22k vs 43.72-43.88k img/s (profiles/conv_halo_pers_r2c.txt)
bool conv_halo_pers_ok(const ConvGeom& g) {
  static const bool on = getenv("DMLAB_HALO_PERS") && atoi(getenv("DMLAB_HALO_PERS"));
  return on && g.C == PBK && g.Ncols == PBN && conv_halo_supported(g);
}

int conv_halo_pers_rows(const ConvGeom& g) { return ((g.W - 1 + PBM - 1) / g.W + 3) * g.W; }

void conv_halo_pers(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                    const ConvGeom& g, const float* pre_sc, const float* pre_sh, hipStream_t st) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int hr = (conv_halo_pers_rows(g) + 63) / 64;
  const int mtiles = (int)((g.M + PBM - 1) / PBM);
  const int grid = mtiles < 2 * cus ? mtiles : 2 * cus;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  auto go = [&](auto kern, int HRv) {
    const size_t main = (size_t)(64 * HRv + 1) * PBK * 2 + (size_t)2 * PBN * PBK * 2 + MAXTAPS * 16;
    const size_t epi = (size_t)128 * (PBN + 4) * 4;
    const size_t sm = main > epi ? main : epi;
    set_smem_attr(kern, sm);
    kern<<<grid, PWM * PWN * 64, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, wb, pre_sc, pre_sh, mtiles);
  };
  if (hr <= 5) go(pre_sc ? conv_halo_pers_kernel<5, true> : conv_halo_pers_kernel<5, false>, 5);
  else if (hr <= 6) go(pre_sc ? conv_halo_pers_kernel<6, true> : conv_halo_pers_kernel<6, false>, 6);
  else go(pre_sc ? conv_halo_pers_kernel<7, true> : conv_halo_pers_kernel<7, false>, 7);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
