// Persistent halo-pipelined 3x3 convolution for the 64- and 128-channel ResNet layers
// ("hpipe", cfg 94/95), gfx950.
//
// The layer-1/2 3x3 convs (56x56x64, 28x28x128) were the least efficient convs of the step
// (docs/KERNELS.md: cfg 39 at ~612 TF/s isolated, ~420 TF/s inside the two-stream step, 4.5 of
// 31.5 ms of kernel time at batch 1024).  Their K is short (9 taps x 64 or 128 channels), so a
// per-tile kernel spends a large share of its life in the halo prologue and the epilogue, and two
// resident workgroups per CU only partly overlap those phases with MFMA work.  Here:
//
//  * a workgroup is PERSISTENT: it walks items (128-pixel x BN-channel tiles) b, b+G, b+2G, ...
//    and its K loop never drains at an item boundary: the input halo of the NEXT (item, 64-channel
//    chunk) is prefetched while the current chunk's 9 taps run, and the first two weight tiles of
//    the next item are in flight while the current item's last taps run;
//  * the halo (the contiguous flattened pixel range [m0 - W - 1, m0 + 128 + W + 1) of one chunk,
//    every tap's A fragment is a row-shifted read of it, out-of-image taps read a zero row) and the
//    per-tap weight tiles go global -> LDS by LDS-DMA (no staging VGPRs, no ds_write pass).  The
//    halo's 8-row pieces are spread one per tap over the first 8 taps, so each K step's single
//    barrier (s_waitcnt vmcnt(0)) only ever waits for DMA issued one step earlier;
//  * LDS per workgroup <= 80 KB (two halo buffers + two weight stages), so two workgroups share a
//    CU and one's epilogue overlaps the other's MFMA work; 4 waves (2 x 2) of 64 x BN/2;
//  * PRE: relu(x * sc + sh) of the previous conv's raw output is applied ONCE per halo (by the
//    thread whose DMA landed the chunk), not once per tap as the per-tile im2col kernels must;
//  * epilogue: BN statistics straight from the accumulators into one slab row per 64-pixel wave
//    row (no LDS, no cross-wave barrier); outputs staged per wave in 16-row bands through the
//    halo buffer the item just finished with, stored as 16-B bf16 chunks (optional ADD).
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <type_traits>

namespace dm {

namespace {
constexpr int QBM = 128;  // output pixels per item
constexpr unsigned QOOB = 0x80000000u;

template <int BN, int HR, bool PRE>
__global__ void __launch_bounds__(256, 2) conv_hpipe_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, unsigned wbytes, int mtiles, int ntN,
    int nitems, int ipb, const float* __restrict__ pre_sc, const float* __restrict__ pre_sh) {
  constexpr int NW = 4, WN = 2;
  constexpr int TN = BN / WN;             // wave tile 64 x TN
  constexpr int RM = 2, RN = TN / 32;     // 32x32 blocks per wave
  constexpr int NP = HR / 8;              // halo pieces (8 rows x 128 B) per chunk
  constexpr int PPW = (NP + NW - 1) / NW; // pieces per wave, two per tap over taps 0-3
  constexpr int BI = BN / 32;             // weight pieces per wave per K step
  constexpr unsigned HB = HR * 128u, BB = BN * 128u;
  constexpr int ZROW = HR - 1;            // never DMA'd as a real row: stays zero
  static_assert(PPW <= 8 && HR % 8 == 0 && 2 * HB + 2 * BB <= 81920u, "halo / LDS budget");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int hsel = lane >> 5;
  const pi32x4 rsx = prsrc(X, xbytes);
  const pi32x4 rsw = prsrc(Wp, wbytes);
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)smem;

  const int W = g.W, H = g.H, C = g.C;
  const int NHW = g.N * H * W;
  const int hp = QBM + 2 * W + 2;  // halo rows an item reads (< HR: row HR-1 stays zero)
  const int nchunk = C / 64;
  const int SI = 9 * nchunk;       // K steps per item
  // items of this workgroup: ipb > 0: the contiguous run [b*ipb, b*ipb + ipb) (the hardware
  // balances the blocks over the CUs; a block prefetches across its own items only);
  // ipb == 0: persistent, items b, b+G, b+2G, ...
  const int G = gridDim.x;
  const int nmine = ipb > 0 ? min(ipb, nitems - (int)blockIdx.x * ipb)
                            : (nitems - (int)blockIdx.x + G - 1) / G;
  const int S = nmine * SI;

  // DMA lane geometry: lane l of piece p fills row 8p + l/8, physical 16-B slot l%8, which holds
  // logical chunk (l%8) ^ ((row >> 1) & 7) = (l%8) ^ ((4p + l/16) & 7); every piece of this wave
  // has p = wid + 4j, so the chunk a lane fetches is the same for all of them
  const int dch = (lane & 7) ^ ((4 * wid + (lane >> 4)) & 7);
  const unsigned choff = (unsigned)dch * 16u;

  auto item_mn = [&](int k, int& mt, int& nt) __attribute__((always_inline)) {
    const int j = ipb > 0 ? (int)blockIdx.x * ipb + k : (int)blockIdx.x + k * G;
    if (ntN == 1 || ipb > 0) {  // contiguous runs: a block takes all N tiles of its M tiles
      mt = j / ntN;
      nt = j - mt * ntN;
      return;
    }
    if (ntN == 1) {
      mt = j;
      nt = 0;
      return;
    }
    const int loc = j >> 3;  // the N tiles of one M tile: items j, j+8, ... (one XCD)
    nt = loc % ntN;
    mt = (loc / ntN) * 8 + (j & 7);
  };
  auto tap_off = [&](int t) __attribute__((always_inline)) {
    const int th = t / 3, tw = t - 3 * th;
    return (g.dy0 + th * g.dys) * W + (g.dx0 + tw * g.dxs);
  };
  auto tap_w = [&](int t) __attribute__((always_inline)) {
    const int th = t / 3, tw = t - 3 * th;
    return ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * C;
  };
  // this lane's two A rows of an item: centre halo row and 9-bit mask of in-image taps
  auto item_rows = [&](int k, int (&lr)[RM], unsigned (&mk)[RM], int& m0, int& n0, int& mt)
      __attribute__((always_inline)) {
    int nt;
    item_mn(k, mt, nt);
    m0 = mt * QBM;
    n0 = nt * BN;
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int r = wm * 64 + i * 32 + (lane & 31);
      const int m = m0 + r;
      lr[i] = r + W + 1;
      unsigned b = 0;
      if (mt < mtiles && m < g.M) {
        const unsigned rr = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
        const int x = m - (int)rr * W;
        const unsigned n = fdiv(rr, g.hg_mul, g.hg_shr);
        const int y = (int)rr - (int)n * H;
#pragma unroll
        for (int th = 0; th < 3; ++th) {
          const int yy = y + g.dy0 + th * g.dys;
#pragma unroll
          for (int tw = 0; tw < 3; ++tw) {
            const int xx = x + g.dx0 + tw * g.dxs;
            if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) b |= 1u << (th * 3 + tw);
          }
        }
      }
      mk[i] = b;
    }
  };

  // ---- halo pieces: piece j of this wave (p = wid + 4j) for chunk cc of an item at pixel m0 ----
  auto halo_off = [&](int j, int m0, int cc) __attribute__((always_inline)) {
    const int row = 8 * (wid + 4 * j) + (lane >> 3);
    const int pix = m0 - W - 1 + row;
    const bool ok = row < hp && pix >= 0 && pix < NHW;
    return ok ? (unsigned)pix * (unsigned)C * 2u + (unsigned)cc * 128u + choff : QOOB;
  };
  auto halo_lds = [&](int j, int hb) __attribute__((always_inline)) {
    return lds0 + (unsigned)hb * HB + (unsigned)(wid + 4 * j) * 1024u;
  };
  // PRE: scale / shift of the 8 channels this thread's halo chunks hold (one 64-channel chunk)
  float psc[PRE ? 8 : 1], psh[PRE ? 8 : 1];
  auto load_pre = [&](int cc) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const int c0 = cc * 64 + dch * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        psc[q] = pre_sc[c0 + q];
        psh[q] = pre_sh[c0 + q];
      }
    }
  };
  auto xform = [&](int j, int hb) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const int row = 8 * (wid + 4 * j) + (lane >> 3);
      if (j >= PPW || wid + 4 * j >= NP || row >= hp) return;
      uint4* q = reinterpret_cast<uint4*>(smem + hb * HB + (wid + 4 * j) * 1024 + lane * 16);
      const uint4 v = *q;
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(bf2f((bf16_t)(w[k] & 0xffff)) * psc[2 * k] + psh[2 * k], 0.f);
        const float hi = fmaxf(bf2f((bf16_t)(w[k] >> 16)) * psc[2 * k + 1] + psh[2 * k + 1], 0.f);
        o[k] = pack_bf2(lo, hi);
      }
      *q = make_uint4(o[0], o[1], o[2], o[3]);
    }
  };

  // ---- weight pieces: B rows n0 + 8(wid + 4q) + l/8 of K step (chunk cc, tap t) ----
  auto b_off = [&](int q, int n0, int cc, int t) __attribute__((always_inline)) {
    const int n = n0 + 8 * (wid + 4 * q) + (lane >> 3);
    return (unsigned)n * (unsigned)g.wK * 2u + (unsigned)(tap_w(t) + cc * 64) * 2u + choff;
  };

  // ---- fragment reads ----
  const int brow = wn * TN + (lane & 31);
  const unsigned boff_frag = 2 * HB + (unsigned)brow * 128u;
  const int bsw = (brow >> 1) & 7;  // same for rows +32
  constexpr int NMF = RM * RN, NRD = RM + RN;
  bf16x8 f0[NRD], f1[NRD];
  auto rd1 = [&](bf16x8 (&f)[NRD], int r, unsigned hbo, const int (&ha)[RM], unsigned sto, int ks)
      __attribute__((always_inline)) {
    const int ch = ks * 2 + hsel;
    if (r < RM) {
      const int row = ha[r];
      f[r] = *reinterpret_cast<const bf16x8*>(smem + hbo + row * 128 + ((ch ^ ((row >> 1) & 7)) << 4));
    } else {
      f[r] = *reinterpret_cast<const bf16x8*>(smem + sto + boff_frag + (r - RM) * 4096 + ((ch ^ bsw) << 4));
    }
  };
  f32x16 acc[RM][RN];
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };
  zero_acc();
  // one 16-deep substep: the MFMAs of `fc` interleaved with the reads of the next substep into
  // `fn` and (DMA) the weight pieces of a later K step into stage `bst`
  constexpr int NQ = NMF > NRD ? (NMF > BI ? NMF : BI) : (NRD > BI ? NRD : BI);
  unsigned bdo[BI];
  auto sub = [&](const bf16x8 (&fc)[NRD], bf16x8 (&fn)[NRD], unsigned hbo, const int (&ha)[RM],
                 unsigned sto, int ks, auto DMA_, unsigned bst) __attribute__((always_inline)) {
    constexpr bool DMA = decltype(DMA_)::value;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < NMF) {
        const int i = q / RN, j = q % RN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fc[i], fc[RM + j], acc[i][j], 0, 0, 0);
      }
      if (q < NRD) rd1(fn, q, hbo, ha, sto, ks);
      if (DMA && q < BI) pdma16(rsw, lds0 + 2 * HB + bst + (unsigned)(wid + 4 * q) * 1024u, bdo[q]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < NMF) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (q < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };

  // ---- epilogue of one item (stage: the halo buffer hbo this item just finished with) ----
  constexpr int LDC = TN + 4;
  constexpr int CPR = TN / 8, RPI = 64 / CPR;
  auto epilogue = [&](int m0, int n0, int mt, unsigned hbo) __attribute__((always_inline)) {
    if (stats && mt < mtiles && (long long)(mt * 2 + wm) * 64 < g.M) {
      const long long srow = (long long)mt * 2 + wm;  // slab row: 64 pixels of this wave row
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        float sm = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = acc[i][j][r];
            sm += v;
            sq += v * v;
          }
        sm += __shfl_xor(sm, 32, 64);
        sq += __shfl_xor(sq, 32, 64);
        if (lane < 32) {
          const int col = n0 + wn * TN + j * 32 + lane;
          stats[(srow * 2 + 0) * g.Ncols + col] = sm;
          stats[(srow * 2 + 1) * g.Ncols + col] = sq;
        }
      }
    }
    float* cs = reinterpret_cast<float*>(smem + hbo) + wid * 16 * LDC;
    const int cq = lane % CPR, rsub = lane / CPR;
    const int col = n0 + wn * TN + cq * 8;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 8 * b; r < 8 * b + 8; ++r)
            cs[((r & 3) + 8 * ((r >> 2) & 1) + 4 * hsel) * LDC + j * 32 + (lane & 31)] = acc[i][j][r];
        // (a wave's LDS accesses complete in order: no barrier between its write and read)
#pragma unroll
        for (int it = 0; it < 16 / RPI; ++it) {
          const int rr = it * RPI + rsub;
          const int m = m0 + wm * 64 + i * 32 + b * 16 + rr;
          if (mt >= mtiles || m >= g.M) continue;
          const long long o = (long long)m * g.OC + col;
          const float4 v0 = *reinterpret_cast<const float4*>(cs + rr * LDC + cq * 8);
          const float4 v1 = *reinterpret_cast<const float4*>(cs + rr * LDC + cq * 8 + 4);
          float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
          if (ADD) {
            const uint4 a = *reinterpret_cast<const uint4*>(ADD + o);
            const uint32_t aw[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              v[2 * q] += bf2f((bf16_t)(aw[q] & 0xffff));
              v[2 * q + 1] += bf2f((bf16_t)(aw[q] >> 16));
            }
          }
          *reinterpret_cast<uint4*>(Y + o) = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]),
                                                        pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
        }
      }
  };

  // ---- cursors ----
  // compute: item kc (rows lr/mk, origin m0c/n0c/mtc), chunk ccc, tap tc, halo buffer hbc
  int kc = 0, ccc = 0, tc = 0, hbc = 0;
  int m0c, n0c, mtc;
  int lr[RM];
  unsigned mk[RM];
  item_rows(0, lr, mk, m0c, n0c, mtc);
  // weight DMA of K step s + 2: item kb (n0b), chunk ccb, tap tb
  int kb = 0, ccb = 0, tb = 0, n0b = n0c;
  auto b_advance = [&]() __attribute__((always_inline)) {
    if (++tb == 9) {
      tb = 0;
      if (++ccb == nchunk) {
        ccb = 0;
        ++kb;
        int mt_, nt_;
        item_mn(kb, mt_, nt_);
        n0b = nt_ * BN;
      }
    }
  };
  // next (item, chunk) after the current one: the halo prefetch target
  int kn = 0, ccn = 0, m0n = 0;
  bool hasn = false;
  auto next_chunk = [&]() __attribute__((always_inline)) {
    kn = kc;
    ccn = ccc + 1;
    if (ccn == nchunk) {
      ccn = 0;
      ++kn;
    }
    hasn = kn < nmine;
    int mt_, nt_;
    item_mn(kn, mt_, nt_);
    m0n = mt_ * QBM;
  };

  // ---- prologue: item 0 chunk 0 halo + weight tiles of K steps 0 and 1 ----
  load_pre(0);
#pragma unroll
  for (int j = 0; j < PPW; ++j)
    if (wid + 4 * j < NP) pdma16(rsx, halo_lds(j, 0), halo_off(j, m0c, 0));
#pragma unroll
  for (int st = 0; st < 2; ++st) {
#pragma unroll
    for (int q = 0; q < BI; ++q)
      pdma16(rsw, lds0 + 2 * HB + (unsigned)st * BB + (unsigned)(wid + 4 * q) * 1024u,
             kb < nmine ? b_off(q, n0b, ccb, tb) : QOOB);
    b_advance();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int j = 0; j < PPW; ++j) xform(j, 0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  next_chunk();
  if (nchunk > 1) load_pre(ccn);
  int ha[RM];
  {
    const int o = tap_off(0);
#pragma unroll
    for (int i = 0; i < RM; ++i) ha[i] = (mk[i] & 1u) ? lr[i] + o : ZROW;
  }
#pragma unroll
  for (int r = 0; r < NRD; ++r) rd1(f0, r, 0u, ha, 0u, 0);

  using T_ = std::true_type;
  using F_ = std::false_type;
  int xpend = -1;  // PRE: halo pieces 2j, 2j+1 issued at the previous DMA slot (transformed
  int xhb = 0;     // after this step's barrier: nobody reads them before the next chunk)
  for (int s = 0; s < S; ++s) {
    const unsigned sto = (unsigned)(s & 1) * BB;
    const unsigned hbo = (unsigned)hbc * HB;
    sub(f0, f1, hbo, ha, sto, 1, F_{}, 0u);
    sub(f1, f0, hbo, ha, sto, 2, F_{}, 0u);
    // weight DMA of step s + 2 (zero loads past the end, into a stage nobody reads again)
#pragma unroll
    for (int q = 0; q < BI; ++q) bdo[q] = kb < nmine ? b_off(q, n0b, ccb, tb) : QOOB;
    sub(f0, f1, hbo, ha, sto, 3, F_{}, 0u);
    // ---- the step's barrier: everything issued at the previous DMA slot has landed ----
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (xpend >= 0) {
      xform(2 * xpend, xhb);
      xform(2 * xpend + 1, xhb);
    }
    // halo pieces 2tc, 2tc + 1 of the next chunk (this wave's share, taps 0-3): landed by the
    // next barrier, transformed after it, read from the next chunk on (>= 4 barriers later)
    xpend = -1;
    if (hasn && 2 * tc < PPW) {
      if (wid + 8 * tc < NP) pdma16(rsx, halo_lds(2 * tc, hbc ^ 1), halo_off(2 * tc, m0n, ccn));
      if (2 * tc + 1 < PPW && wid + 4 * (2 * tc + 1) < NP)
        pdma16(rsx, halo_lds(2 * tc + 1, hbc ^ 1), halo_off(2 * tc + 1, m0n, ccn));
      xpend = tc;
      xhb = hbc ^ 1;
    }
    // rows of step s + 1
    const bool item_end = tc == 8 && ccc == nchunk - 1;
    int ntc = tc + 1, nhb = hbc;
    int lr2[RM];
    unsigned mk2[RM];
    int m0x = m0c, n0x = n0c, mtx = mtc;
    if (tc == 8) {
      ntc = 0;
      nhb = hbc ^ 1;
    }
    if (item_end && kc + 1 < nmine) {
      item_rows(kc + 1, lr2, mk2, m0x, n0x, mtx);
    } else {
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        lr2[i] = lr[i];
        mk2[i] = mk[i];
      }
    }
    int han[RM];
    {
      const int o = tap_off(ntc);
#pragma unroll
      for (int i = 0; i < RM; ++i) han[i] = ((mk2[i] >> ntc) & 1u) ? lr2[i] + o : ZROW;
    }
    sub(f1, f0, (unsigned)nhb * HB, han, sto ^ BB, 0, T_{}, sto);
    b_advance();
    if (item_end) {
      epilogue(m0c, n0c, mtc, hbo);
      zero_acc();
      ++kc;
      ccc = 0;
      m0c = m0x;
      n0c = n0x;
      mtc = mtx;
#pragma unroll
      for (int i = 0; i < RM; ++i) {
        lr[i] = lr2[i];
        mk[i] = mk2[i];
      }
    } else if (tc == 8) {
      ++ccc;
    }
    if (tc == 8) {
      hbc ^= 1;
      next_chunk();
      if (nchunk > 1) load_pre(ccn);
    }
    tc = ntc;
#pragma unroll
    for (int i = 0; i < RM; ++i) ha[i] = han[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int hpipe_hr(const ConvGeom& g) {
  const int hp = QBM + 2 * g.W + 2;
  return hp < 192 ? 192 : hp < 248 ? 248 : 0;
}

int num_cus_cached() {
  static int cus[64] = {0};
  int dev = 0;
  DM_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev]) DM_CHECK(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return cus[dev];
}

// items per workgroup (DMLAB_HPIPE_IPB; 0 = persistent, two workgroups per CU)
int hpipe_ipb() {
  static const int v = getenv("DMLAB_HPIPE_IPB") ? atoi(getenv("DMLAB_HPIPE_IPB")) : 4;
  return v < 0 ? 0 : v;
}

template <int BN, int HR>
void launch_hpipe(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                  const ConvGeom& g, hipStream_t st, const float* pre_sc, const float* pre_sh) {
  const int mtiles = (int)((g.M + QBM - 1) / QBM);
  const int ntN = g.Ncols / BN;
  const int ipb = hpipe_ipb();
  const int nitems = (ntN == 1 || ipb > 0) ? mtiles * ntN : (mtiles + 7) / 8 * 8 * ntN;
  int grid;
  if (ipb > 0) {
    grid = (nitems + ipb - 1) / ipb;
  } else {
    grid = 2 * num_cus_cached();
    if (grid > nitems) grid = nitems;
  }
  const size_t sm = (size_t)2 * HR * 128 + (size_t)2 * BN * 128;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  auto k = pre_sc ? conv_hpipe_kernel<BN, HR, true> : conv_hpipe_kernel<BN, HR, false>;
  set_smem_attr(k, sm);
  k<<<grid, 256, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, wb, mtiles, ntN, nitems, ipb, pre_sc,
                           pre_sh);
  DM_CHECK(hipGetLastError());
}
}  // namespace

bool conv_hpipe_supported(const ConvGeom& g, int cfg) {
  const int bn = cfg == 95 ? 128 : 64;
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W) return false;
  if (g.osy != 1 || g.osx != 1 || g.oy0 != 0 || g.ox0 != 0 || g.OH != g.H || g.OW != g.W) return false;
  if (g.nth != 3 || g.ntw != 3) return false;
  auto in1 = [](int v) { return v >= -1 && v <= 1; };
  if (!in1(g.dy0) || !in1(g.dy0 + 2 * g.dys) || !in1(g.dx0) || !in1(g.dx0 + 2 * g.dxs)) return false;
  if (g.C % 64 != 0 || g.Ncols % bn != 0 || g.OC != g.Ncols) return false;
  const int hr = hpipe_hr(g);
  if (hr == 0 || (bn == 128 && hr > 192)) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  if ((long long)g.Ncols * g.wK * 2 >= (1LL << 31)) return false;
  if (g.M * g.OC >= (1LL << 31)) return false;
  return true;
}

// cfg 94: 128 x 64 items (2 x 2 waves of 64 x 32); 95: 128 x 128 items (2 x 2 waves of 64 x 64)
void conv_hpipe(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                const ConvGeom& g, int cfg, hipStream_t st, const float* pre_sc,
                const float* pre_sh) {
  const int hr = hpipe_hr(g);
  if (cfg == 95) launch_hpipe<128, 192>(X, Wp, Y, ADD, stats, g, st, pre_sc, pre_sh);
  else if (hr == 192) launch_hpipe<64, 192>(X, Wp, Y, ADD, stats, g, st, pre_sc, pre_sh);
  else launch_hpipe<64, 248>(X, Wp, Y, ADD, stats, g, st, pre_sc, pre_sh);
}

}  // namespace dm
