// Persistent resident-weight conv for 64 -> 64 channel unit-stride 3x3 layers (ResNet-18
// layer1: forward and data gradient), gfx950.
//
// With C = Cout = 64 the whole weight tensor of a 3x3 conv is 9 x 64 x 64 bf16 = 72 KB: it fits
// in LDS next to one 256-pixel input halo (<= 8 rows of W = 56 pixels x 128 B).  So instead of
// conv_halo.hip's one (tap) step per barrier with the weight tile re-staged every step, a
// block here is PERSISTENT (one per CU):
//
//  * the weights are staged once per block and stay resident;
//  * per 256-pixel output tile the block runs all 9 taps x 4 k-substeps back to back with no
//    barrier (A fragments from the halo at row offset dy*W + dx, B fragments from the
//    resident weights), 72 v_mfma_f32_32x32x16_bf16 per wave;
//  * the NEXT tile's halo is loaded into registers while the current tile computes and runs
//    its epilogue, then written to LDS (with the fused BN-apply of the previous layer, PRE);
//  * the epilogue (BN statistics + coalesced bf16 stores, optional ADD) is the shared tile
//    epilogue, staged through the halo buffer once the taps are done.
// 8 waves (2 per SIMD) x (32 pixels x 64 channels).  Stats slab rows = 256-pixel tiles, as
// the other 256-row configs, so the BN finalize is unchanged.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int LBM = 256;   // output pixels per tile
constexpr int LC = 64;     // channels (in and out)
constexpr int LNT = 512;   // threads
constexpr int LHR = 7;     // halo registers per thread: 7 x 64 rows = 448 rows
constexpr int LHP = LHR * (LNT / 8);
constexpr unsigned LOOB = 0x80000000u;

template <bool PRE>
__global__ void __launch_bounds__(LNT, 1) conv_l1_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, const float* __restrict__ pre_sc,
    const float* __restrict__ pre_sh, int ntiles) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem);          // [9 taps][64 co][64 c]
  bf16_t* Hs = Ws + 9 * LC * LC;                          // [LHP + 1][64], last row zeros
  int4* taps = reinterpret_cast<int4*>(Hs + (LHP + 1) * LC);
  float* psc = reinterpret_cast<float*>(taps + MAXTAPS);  // [64] (PRE)
  float* psh = psc + LC;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntaps = g.nth * g.ntw;
  const int NHW = g.N * g.H * g.W;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    taps[tid] = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * LC,
                          dy * g.W + dx);
  }
  if (tid < 8) *reinterpret_cast<uint4*>(Hs + LHP * LC + tid * 8) = make_uint4(0, 0, 0, 0);
  if (PRE && tid < LC) {
    psc[tid] = pre_sc[tid];
    psh[tid] = pre_sh[tid];
  }
  __syncthreads();  // taps table
  // resident weights: packed row co holds tap t's 64 channels at taps[t].z -> LDS [t][co][c]
  for (int e = tid; e < ntaps * LC * 8; e += LNT) {
    const int ch = e & 7, co = (e >> 3) & (LC - 1), t = e >> 9;
    const uint4 v = *reinterpret_cast<const uint4*>(Wp + (long long)co * g.wK + taps[t].z + ch * 8);
    *reinterpret_cast<uint4*>(Ws + (t * LC + co) * LC + swz(co, ch) * 8) = v;
  }

  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  const int chunk = tid & 7;
  uint4 rh[LHR];
  int hbase_next = 0;
  auto halo_of = [&](int tile, int& hbase, int& hp) {
    const long long m0 = (long long)tile * LBM;
    const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
    const long long mlast = (m0 + LBM - 1 < g.M) ? m0 + LBM - 1 : g.M - 1;
    const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
    hbase = (r0 - 1) * g.W;
    hp = (r1 - r0 + 3) * g.W;
  };
  auto load_halo = [&](int tile) {
    int hb, hp;
    halo_of(tile, hb, hp);
    hbase_next = hb;
#pragma unroll
    for (int j = 0; j < LHR; ++j) {
      const int hh = (tid >> 3) + (LNT / 8) * j;
      const int gp = hb + hh;
      const bool ok = hh < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? (unsigned)gp * (unsigned)(LC * 2) + (unsigned)chunk * 16u : LOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      rh[j] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int j = 0; j < LHR; ++j) {
      const int hh = (tid >> 3) + (LNT / 8) * j;
      uint4 v = rh[j];
      if constexpr (PRE) {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int c = chunk * 8 + 2 * q;
          const float lo = fmaxf(bf2f((bf16_t)(w[q] & 0xffff)) * psc[c] + psh[c], 0.f);
          const float hi = fmaxf(bf2f((bf16_t)(w[q] >> 16)) * psc[c + 1] + psh[c + 1], 0.f);
          o[q] = pack_bf2(lo, hi);
        }
        v = make_uint4(o[0], o[1], o[2], o[3]);
      }
      *reinterpret_cast<uint4*>(Hs + hh * LC + swz(hh, chunk) * 8) = v;
    }
  };

  int tile = blockIdx.x;
  if (tile < ntiles) load_halo(tile);
  for (; tile < ntiles; tile += gridDim.x) {
    const int hbase = hbase_next;
    store_halo();
    __syncthreads();  // halo visible
    const int next = tile + gridDim.x;
    if (next < ntiles) load_halo(next);  // in flight during the taps and the epilogue
    const long long m0 = (long long)tile * LBM;
    // this wave's 32 pixels: halo row of the zero-offset tap and coordinates
    const long long m = m0 + wid * 32 + (lane & 31);
    const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
    const int ax = (int)((unsigned)m - r * (unsigned)g.W);
    const unsigned nimg = fdiv(r, g.hg_mul, g.hg_shr);
    const int ay = (m < g.M) ? (int)(r - nimg * (unsigned)g.H) : -(1 << 28);
    const int ah = (int)(m - hbase);

    f32x16 acc[1][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[0][j][q] = 0.f;
    // fragments of (tap, k-substep) u+1 are read while u's MFMAs issue; u = t*4 + ks
    auto frags = [&](int u, bf16x8& af, bf16x8 (&bf)[2]) {
      const int t = u >> 2, ks = u & 3;
      const int4 tp = taps[t];
      const bool ok = (unsigned)(ax + tp.y) < (unsigned)g.W && (unsigned)(ay + tp.x) < (unsigned)g.H;
      const int hrow = ok ? ah + tp.w : LHP;
      const int ch = ks * 2 + (lane >> 5);
      af = *reinterpret_cast<const bf16x8*>(Hs + hrow * LC + swz(hrow, ch) * 8);
      const bf16_t* ws = Ws + t * LC * LC;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int co = j * 32 + (lane & 31);
        bf[j] = *reinterpret_cast<const bf16x8*>(ws + co * LC + swz(co, ch) * 8);
      }
    };
    constexpr int nu = 9 * 4;  // 3x3 taps (conv_l1_supported) x 4 k-substeps: fully unrolled
    bf16x8 a0, a1, b0[2], b1[2];
    frags(0, a0, b0);
#pragma unroll
    for (int u = 0; u < nu; u += 2) {
      if (u + 1 < nu) frags(u + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b0[j], acc[0][j], 0, 0, 0);
      if (u + 1 >= nu) break;
      if (u + 2 < nu) frags(u + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[0][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b1[j], acc[0][j], 0, 0, 0);
    }
    __syncthreads();  // every wave is done with the halo: the epilogue stages through it
    mfma_tile_epilogue<LBM, LC, 8, 1, true, 2>(acc, reinterpret_cast<unsigned char*>(Hs), m0, 0,
                                                tile, stats, g, Y, ADD);
    __syncthreads();  // staging reads done before the next halo overwrites it
  }
}
}  // namespace

bool conv_l1_supported(const ConvGeom& g) {
  if (g.C != LC || g.Ncols != LC || g.wK != 9 * LC || g.nth != 3 || g.ntw != 3) return false;
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W || g.OC != LC) return false;
  const int dya = g.dy0, dyb = g.dy0 + 2 * g.dys, dxa = g.dx0, dxb = g.dx0 + 2 * g.dxs;
  auto in1 = [](int v) { return v >= -1 && v <= 1; };
  if (!in1(dya) || !in1(dyb) || !in1(dxa) || !in1(dxb)) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  // worst-case halo over tiles: a 256-pixel run starting at the last pixel of a row
  return ((g.W - 1 + LBM - 1) / g.W + 3) * g.W <= LHP;
}

void conv_l1(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
             const ConvGeom& g, hipStream_t st, const float* pre_sc, const float* pre_sh) {
  const size_t sm = (size_t)9 * LC * LC * 2 + (size_t)(LHP + 1) * LC * 2 + MAXTAPS * 16 + 2 * LC * 4;
  const int ntiles = (int)((g.M + LBM - 1) / LBM);
  static int cus = 0;  // one persistent block per CU
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int grid = ntiles < cus ? ntiles : cus;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  auto k = pre_sc ? conv_l1_kernel<true> : conv_l1_kernel<false>;
  set_smem_attr(k, sm);
  k<<<grid, LNT, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, pre_sc, pre_sh, ntiles);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
