// Pipelined implicit-GEMM convolution ("pipe" kernels, cfg 90/91), gfx950.
//
// Round 3 rebuild of the conv main loop around what the register-staged tiles could not do
// (docs/KERNELS.md "Where the ceiling is"): the v3/halo kernels keep 64x64 per wave, stage
// every operand through VGPRs and ds_write, and run at 2 workgroups per CU with a barrier per
// 64-deep K step; their MFMA pipe is busy ~30 % of the time.  Here:
//
//  * one 256-pixel x BN-channel tile per workgroup, 4 waves (2 x 2), each wave owning a
//    128 x BN/2 sub-tile as 4 x BN/64 blocks of v_mfma_f32_32x32x16_bf16 (the 256 fp32
//    accumulators of the BN = 256 tile live in the AGPR half of the unified register file):
//    0.5 LDS fragment reads per MFMA (v3: 1.0);
//  * both operands go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds): no staging
//    VGPRs, no ds_write pass.  The A operand is the implicit im2col matrix gathered row by
//    row — each DMA lane supplies the address of its own output pixel's tap source, padding
//    taps read 0 through the buffer range check — so one kernel serves every tap geometry
//    ConvGeom describes (3x3 and 1x1, stride 1 and 2, forward and the data gradient);
//  * two LDS stages; the ONE barrier of a K step sits after the last fragment reads of the
//    step (before its last 16-deep substep), so the DMA of tile t+2 is issued right after it
//    and has a full K step to land while the other stage is consumed; the first fragments of
//    the next tile are read under the last substep's MFMAs (no read latency at the seam);
//  * the DMA is issued from inline asm so the compiler's alias-blind LDS-DMA bookkeeping does
//    not drain the queue before every ds_read (docs/KERNELS.md, conv_h5 notes); the loop
//    retires it with its own s_waitcnt vmcnt(0) at the barrier.  The loop has no other VMEM
//    op, so nothing else waits on the queue.
//  * epilogue: per-column BN statistics straight from the accumulators (no LDS pass), then
//    each wave stages its own 32-row bands through a private LDS region and stores 16-B bf16
//    chunks (optional residual add), so no cross-wave barrier and no 2-pass 133 KB image.
//
// LDS swizzle: the 16-B chunk c of tile row r lives at slot c ^ ((r >> 1) & 7) (igemm_common.h
// swz), conflict-free for the 32x32x16 fragment reads; the DMA image is lane-linear (base +
// 16 * lane), so the swizzle is applied to the SOURCE chunk each lane fetches.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <stdexcept>
#include <type_traits>

namespace dm {

namespace {
constexpr int PBM = 256;   // output pixels per tile
constexpr int PBK = 64;    // K per step (one 128-B LDS row per tile row)
constexpr unsigned POOB = 0x80000000u;
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));

// BN output channels per tile (256 / 128 / 64); WM x WN waves, wave tile 256/WM x BN/WN;
// MINW waves per SIMD the register budget is sized for.  (A PRE variant that applied the
// previous BN + ReLU to the landed A chunks between the vmcnt wait and the barrier was removed
// in round 4: materialising that BN output is 1.7 % faster per step on layers 3-4,
// profiles/pipe_pre_materialise_ab_r4q.txt)
// RED (data gradients): the backward reduction of the BatchNorm whose output gradient Y is
// (kernels.h BnBwdRed) runs in the store loop -- each lane's 8 channels of the stored bf16
// value against that BN's input y -- and leaves one [2][Ncols] row per M tile in red.part
// SEG2 (stride-2 data gradients): geometry s2.z (parity class (0,0)) runs C2/64 more K steps
// over X2 / W2 at the row's own pixel -- the block's 1x1/s2 projection (conv_geom.h DgradSeg2;
// here X2 has X's channel count, so the row's pixel base is shared)
template <int BN, int WM, int WN, int MINW, bool RED = false, bool SEG2 = false>
__global__ void __launch_bounds__(WM * WN * 64, MINW) conv_pipe_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeomSet gs, unsigned xbytes, unsigned wbytes, int ntN,
    int mtiles_max, int xcd, BnBwdRed red, DgradSeg2 s2) {
  // blockIdx.y selects one of up to four geometries sharing X / W / Y (the parity classes of a
  // stride-2 data gradient, which write disjoint output pixels); one geometry otherwise
  const ConvGeom g = gs.g[blockIdx.y];
  const int mtiles = (int)((g.M + PBM - 1) / PBM);
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = PBM / WM, TN = BN / WN;  // wave tile
  constexpr int RM = TM / 32, RN = TN / 32;   // 32x32 blocks per wave
  constexpr int AI = PBM * 8 / NT;            // A DMA instructions per thread per tile
  constexpr int BI = BN * 8 / NT;             // B DMA instructions per thread per tile
  static_assert(AI * NT == PBM * 8 && BI * NT == BN * 8 && RM >= 1 && RN >= 1, "tile");
  constexpr unsigned ABYTES = PBM * PBK * 2;
  constexpr unsigned STG = ABYTES + BN * PBK * 2;  // one pipeline stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  // block -> (M tile, N tile): the N tiles of one M tile are blocks b, b+8, ... (one XCD)
  int bx = blockIdx.x, by = 0;
  if (xcd) {
    const int b = blockIdx.x, j = b >> 3;
    by = j % ntN;
    bx = (j / ntN) * 8 + (b & 7);
  } else {
    bx = blockIdx.x % mtiles_max;
    by = blockIdx.x / mtiles_max;
  }
  // part row of this block (RED): parity classes of a multi-geometry launch stack their M tiles
  const long long prow = (long long)blockIdx.y * mtiles_max + bx;
  if (bx >= mtiles) {  // padding of the grid, or a smaller parity class
    if constexpr (RED) {  // every part row is summed by the consumer
      if (bx < mtiles_max && by == 0)
        for (int c = threadIdx.x; c < 2 * g.Ncols; c += blockDim.x) red.part[prow * 2 * g.Ncols + c] = 0.f;
    }
    return;
  }
  const int m0 = bx * PBM;
  const int n0 = by * BN;
  const int ntaps = g.nth * g.ntw;
  const int nchunk = g.C / PBK;
  const int S1 = ntaps * nchunk;
  const int S = S1 + ((SEG2 && (int)blockIdx.y == s2.z) ? s2.C2 / PBK : 0);

  const pi32x4 rsx = prsrc(X, xbytes);
  const pi32x4 rsw = prsrc(Wp, wbytes);
  const pi32x4 rsx2 = prsrc(SEG2 ? s2.X2 : (const void*)X, SEG2 ? s2.x2bytes : 0u);
  const pi32x4 rsw2 = prsrc(SEG2 ? s2.W2 : (const void*)Wp, SEG2 ? s2.w2bytes : 0u);
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)smem;

  // ---- DMA lane geometry: instruction j of wave w fills tile rows 8 NW j + 8w + lane/8 ----
  const int drow = 8 * wid + (lane >> 3);                 // row within an 8 NW-row group
  const int dch = (lane & 7) ^ ((drow >> 1) & 7);         // logical chunk this lane fetches
  const unsigned choff = (unsigned)dch * 16u;
  unsigned abase[AI], amask[AI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = m0 + 8 * NW * j + drow;
    unsigned base = 0, mk = 0;
    if (m < g.M) {
      const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - r * (unsigned)g.Wg);
      const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
      const int y = (int)(r - n * (unsigned)g.Hg);
      const int iy = y * g.isy, ix = x * g.isx;
      base = (((unsigned)n * g.H + iy) * g.W + ix) * (unsigned)g.C * 2u + choff;
      for (int th = 0; th < g.nth; ++th) {
        const int yy = iy + g.dy0 + th * g.dys;
        if ((unsigned)yy >= (unsigned)g.H) continue;
        for (int tw = 0; tw < g.ntw; ++tw) {
          const int xx = ix + g.dx0 + tw * g.dxs;
          if ((unsigned)xx < (unsigned)g.W) mk |= 1u << (th * g.ntw + tw);
        }
      }
    }
    abase[j] = base;
    amask[j] = mk;
  }
  unsigned bbase[BI], bbase2[SEG2 ? BI : 1];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int n = n0 + 8 * NW * j + drow;
    bbase[j] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u + choff : POOB;
    if constexpr (SEG2) bbase2[j] = n < g.Ncols ? (unsigned)n * (unsigned)s2.C2 * 2u + choff : POOB;
  }

  // DMA of the next K step (chunk icc, tap ith/itw): prep() computes this thread's source
  // offsets and advances the counters; one(q, st) issues DMA instruction q into stage st
  constexpr int ND = AI + BI;
  int icc = 0, ith = 0, itw = 0;
  unsigned doff[ND];
  bool dseg = false;  // the prepared step reads the second segment
  auto prep = [&]() __attribute__((always_inline)) {
    if constexpr (SEG2) {
      // after the geometry's own steps (icc == nchunk), C2/64 steps of the projection: one
      // 64-channel chunk each, the row's own pixel (abase: X2 has X's channel count)
      const int c2 = icc - nchunk;
      dseg = c2 >= 0 && c2 * PBK < s2.C2 && (int)blockIdx.y == s2.z;
      if (dseg) {
        ++icc;
        const unsigned co = (unsigned)(c2 * PBK * 2);
#pragma unroll
        for (int j = 0; j < AI; ++j) doff[j] = amask[j] ? abase[j] + co : POOB;
#pragma unroll
        for (int j = 0; j < BI; ++j) doff[AI + j] = bbase2[j] != POOB ? bbase2[j] + co : POOB;
        return;
      }
    }
    const int cc = icc, th = ith, tw = itw;
    const int t = th * g.ntw + tw;
    if (++itw == g.ntw) {
      itw = 0;
      if (++ith == g.nth) {
        ith = 0;
        ++icc;
      }
    }
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    const bool live = cc < nchunk;  // steps past the end load zeros
    const unsigned tapd = (unsigned)((dy * g.W + dx) * g.C * 2 + cc * PBK * 2);
    const unsigned wko =
        (unsigned)((((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * g.C + cc * PBK) * 2);
#pragma unroll
    for (int j = 0; j < AI; ++j) doff[j] = live && ((amask[j] >> t) & 1u) ? abase[j] + tapd : POOB;
#pragma unroll
    for (int j = 0; j < BI; ++j) doff[AI + j] = live && bbase[j] != POOB ? bbase[j] + wko : POOB;
  };
  const unsigned ldsw = lds0 + (unsigned)wid * 1024u;
  auto one = [&](int q, int st) __attribute__((always_inline)) {
    if (q < AI)
      pdma16(SEG2 && dseg ? rsx2 : rsx, ldsw + (unsigned)st * STG + (unsigned)q * (NW * 1024u), doff[q]);
    else
      pdma16(SEG2 && dseg ? rsw2 : rsw, ldsw + (unsigned)st * STG + ABYTES + (unsigned)(q - AI) * (NW * 1024u),
             doff[q]);
  };

  // ---- fragment reads: A rows wm*TM + i*32 + (lane&31), B rows wn*TN + j*32 + (lane&31) ----
  const int frow_a = wm * TM + (lane & 31);
  const int frow_b = wn * TN + (lane & 31);
  const int fsw_a = (frow_a >> 1) & 7, fsw_b = (frow_b >> 1) & 7;  // same for +32k rows
  const int hsel = lane >> 5;
  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  constexpr int NMF = RM * RN;  // MFMAs per 16-deep substep
  constexpr int NRD = RM + RN;  // fragment reads per substep
  bf16x8 f0[NRD], f1[NRD];      // [0, RM) A fragments, [RM, NRD) B fragments
  auto rd1 = [&](bf16x8 (&f)[NRD], int r, int st, int ks) __attribute__((always_inline)) {
    const int ch = ks * 2 + hsel;
    if (r < RM)
      f[r] = *reinterpret_cast<const bf16x8*>(smem + st * STG + frow_a * 128 +
                                              ((ch ^ fsw_a) << 4) + r * 4096);
    else
      f[r] = *reinterpret_cast<const bf16x8*>(smem + st * STG + ABYTES + frow_b * 128 +
                                              ((ch ^ fsw_b) << 4) + (r - RM) * 4096);
  };
  auto rdall = [&](bf16x8 (&f)[NRD], int st, int ks) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < NRD; ++r) rd1(f, r, st, ks);
  };
  // one 16-deep substep: the MFMAs of fragment set `fc`, interleaved (one MFMA, one read, then
  // the DMA share) with the reads of the next substep's fragments into `fn` (RD) and the DMA
  // of the next-but-one K step into stage dst (DMA)
  constexpr int NQ = NMF > NRD ? (NMF > ND ? NMF : ND) : (NRD > ND ? NRD : ND);
  auto sub = [&](const bf16x8 (&fc)[NRD], bf16x8 (&fn)[NRD], int rst, int rks, auto RD_, auto DMA_,
                 int dst) __attribute__((always_inline)) {
    constexpr bool RD = decltype(RD_)::value, DMA = decltype(DMA_)::value;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < NMF) {
        const int i = q / RN, j = q % RN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fc[i], fc[RM + j], acc[i][j], 0, 0, 0);
      }
      if (RD && q < NRD) rd1(fn, q, rst, rks);
      if (DMA && q < ND) one(q, dst);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q < NMF) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      if (RD && q < NRD) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  // tile of stage `nst` landed; publish it (every wave is done reading the other stage)
  auto barrier_vm0 = [&](int nst) __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // ---- prologue: tiles 0 and 1 in flight, tile 0 published, its first fragments read ----
  // (with S == 1 the second DMA loads zeros into stage 1, which is never read)
  prep();
#pragma unroll
  for (int q = 0; q < ND; ++q) one(q, 0);
  prep();
#pragma unroll
  for (int q = 0; q < ND; ++q) one(q, 1);
  if constexpr (ND == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if constexpr (ND == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if constexpr (ND == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  else if constexpr (ND == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  rdall(f0, 0, 0);

  // one K step from stage cur; MODE 2: barrier, next tile's first reads, DMA of step t+2 into
  // cur; 1: barrier and reads only (t+2 >= S); 0: last step
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto step = [&](int cur, auto MODE_) __attribute__((always_inline)) {
    constexpr int MODE = decltype(MODE_)::value;
    sub(f0, f1, cur, 1, T_{}, F_{}, 0);
    sub(f1, f0, cur, 2, T_{}, F_{}, 0);
    if constexpr (MODE == 2) prep();
    sub(f0, f1, cur, 3, T_{}, F_{}, 0);
    if constexpr (MODE > 0) barrier_vm0(cur ^ 1);  // tile t+1 landed; stage cur is free
    sub(f1, f0, cur ^ 1, 0, std::integral_constant<bool, (MODE > 0)>{},
        std::integral_constant<bool, (MODE == 2)>{}, cur);
  };
  using M2 = std::integral_constant<int, 2>;
  using M0 = std::integral_constant<int, 0>;
  // steps past the end (t + 2 >= S) issue zero-DMAs into a stage nobody reads again and read
  // fragments nobody uses: one uniform loop body (the tail copies of the step cost spills)
  int t = 0;
  for (; t + 1 < S; t += 2) {
    step(0, M2{});
    step(1, M2{});
  }
  if (t < S) step(0, M0{});

  // ---- epilogue ----
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the stage buffers (LDS reused below)
  float* sred = reinterpret_cast<float*>(smem);  // [WM][BN][2] statistics partials
  if (stats) {
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = acc[i][j][r];
          sm += v;
          q += v * v;
        }
      sm += __shfl_xor(sm, 32, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < 32) {
        const int c = wn * TN + j * 32 + lane;
        sred[(wm * BN + c) * 2 + 0] = sm;
        sred[(wm * BN + c) * 2 + 1] = q;
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      if (n0 + c < g.Ncols) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          a += sred[(w * BN + c) * 2 + 0];
          b += sred[(w * BN + c) * 2 + 1];
        }
        stats[((long long)bx * 2 + 0) * g.Ncols + n0 + c] = a;
        stats[((long long)bx * 2 + 1) * g.Ncols + n0 + c] = b;
      }
    }
    __syncthreads();
  }
  // per-wave staging region: 32 rows x (TN + 4) floats
  constexpr int LDC = TN + 4;
  float* cs = reinterpret_cast<float*>(smem) + wid * 32 * LDC;
  constexpr int CPR = TN / 8;            // 16-B output chunks per row
  constexpr int RPI = 64 / CPR;          // rows per wave instruction
  const int cq = lane % CPR, rsub = lane / CPR;
  const int col = n0 + wn * TN + cq * 8;
  const int fcol = lane & 31;
  float rsc[8], rsh[8], rmu[8], rs[8], rq[8];
  if constexpr (RED) {
    // 8 consecutive channels' constants as 16-byte loads when aligned (profiles/
    // red_const_loads_ab_r6.txt); Ncols % 8 == 0, a group past the edge reads channel 0's
    const int cb = col + 8 <= g.Ncols ? col : 0;
    auto ld8 = [&](const float* p, float (&v)[8]) __attribute__((always_inline)) {
      if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        const float4 a = *reinterpret_cast<const float4*>(p + cb);
        const float4 b = *reinterpret_cast<const float4*>(p + cb + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = p[cb + j];
      }
    };
    ld8(red.mu, rmu);
    if (red.mask) {
#pragma unroll
      for (int j = 0; j < 8; ++j) rsc[j] = rsh[j] = 0.f;
    } else {
      ld8(red.sc, rsc);
      ld8(red.sh, rsh);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) rs[j] = rq[j] = 0.f;
  }
  // RED: the y chunks (and 1-bit masks) of row block i + 1 are loaded while block i is
  // staged and stored (a load per chunk in the store loop left its latency exposed: layer4's
  // 1.5 workgroups per CU have nothing else to run)
  // The residual ADD chunks (and identity-skip masks) of block i are loaded before block i
  // is staged, for the same reason.
  constexpr int NIT = 32 / RPI;
  uint4 ypf[2][NIT], apf[NIT];
  unsigned mpf[2][NIT], ampf[NIT];
  auto aload = [&](int i) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + wm * TM + i * 32 + it * RPI + rsub;
      apf[it] = make_uint4(0, 0, 0, 0);
      ampf[it] = 0xffu;
      if (m >= g.M || col >= g.Ncols) continue;
      const unsigned t = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - t * (unsigned)g.Wg);
      const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
      const int y = (int)(t - n * (unsigned)g.Hg);
      const long long o =
          (((long long)n * g.OH + (y * g.osy + g.oy0)) * g.OW + (x * g.osx + g.ox0)) * g.OC + col;
      apf[it] = *reinterpret_cast<const uint4*>(ADD + o);
      if (g.addm) ampf[it] = g.addm[o >> 3];
    }
  };
  auto yload = [&](int i, int bsel) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int m = m0 + wm * TM + i * 32 + it * RPI + rsub;
      ypf[bsel][it] = make_uint4(0, 0, 0, 0);
      mpf[bsel][it] = 0u;
      if (m >= g.M || col >= g.Ncols) continue;
      const unsigned t = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - t * (unsigned)g.Wg);
      const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
      const int y = (int)(t - n * (unsigned)g.Hg);
      const long long o =
          (((long long)n * g.OH + (y * g.osy + g.oy0)) * g.OW + (x * g.osx + g.ox0)) * g.OC + col;
      ypf[bsel][it] = *reinterpret_cast<const uint4*>(red.y + o);
      if (red.mask) mpf[bsel][it] = red.mask[o >> 3];
    }
  };
  if constexpr (RED) yload(0, 0);
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    if (ADD) aload(i);
    if constexpr (RED) {
      if (i + 1 < RM) yload(i + 1, (i + 1) & 1);
    }
    // stage rows wm*128 + i*32 .. +31 of this wave's columns
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        cs[((r & 3) + 8 * (r >> 2) + 4 * hsel) * LDC + j * 32 + fcol] = acc[i][j][r];
    // (a wave's LDS accesses complete in order: no barrier between its own write and read)
#pragma unroll
    for (int it = 0; it < 32 / RPI; ++it) {
      const int rr = it * RPI + rsub;
      const int m = m0 + wm * TM + i * 32 + rr;
      if (m >= g.M || col >= g.Ncols) continue;
      const unsigned t = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - t * (unsigned)g.Wg);
      const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
      const int y = (int)(t - n * (unsigned)g.Hg);
      const long long o =
          (((long long)n * g.OH + (y * g.osy + g.oy0)) * g.OW + (x * g.osx + g.ox0)) * g.OC + col;
      const float4 v0 = *reinterpret_cast<const float4*>(cs + rr * LDC + cq * 8);
      const float4 v1 = *reinterpret_cast<const float4*>(cs + rr * LDC + cq * 8 + 4);
      float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
      if (ADD) {
        const uint4 a = apf[it];
        const unsigned mb = ampf[it];  // identity-skip ReLU mask
        const uint32_t aw[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[2 * q] += ((mb >> (2 * q)) & 1u) ? bf2f((bf16_t)(aw[q] & 0xffff)) : 0.f;
          v[2 * q + 1] += ((mb >> (2 * q + 1)) & 1u) ? bf2f((bf16_t)(aw[q] >> 16)) : 0.f;
        }
      }
      const uint4 ov = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]),
                                  pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
      {  // non-temporal store (profiles/conv_nt_stores_ab_r4ab.txt)
        u32x4_nt v;
        v.x = ov.x; v.y = ov.y; v.z = ov.z; v.w = ov.w;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4_nt*>(Y + o));
      }
      if constexpr (RED) {
        // dz = the stored gradient where the reduced BN's ReLU passed (1-bit mask, or
        // y*sc + sh > 0); Σdz and Σdz (y - mu) per channel
        const uint4 yv = ypf[i & 1][it];
        const unsigned mb = mpf[i & 1][it];
        const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w}, ow[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float yj = __uint_as_float((j & 1) ? (yw[j >> 1] & 0xffff0000u) : (yw[j >> 1] << 16));
          const float gj = __uint_as_float((j & 1) ? (ow[j >> 1] & 0xffff0000u) : (ow[j >> 1] << 16));
          const bool pass = red.mask ? ((mb >> j) & 1u) != 0u : yj * rsc[j] + rsh[j] > 0.f;
          const float dz = pass ? gj : 0.f;
          rs[j] += dz;
          rq[j] += dz * (yj - rmu[j]);
        }
      }
    }
  }
  if constexpr (RED) {
    // lanes of one channel chunk (same cq, rsub = lane / CPR) add up, then the WM waves of
    // one channel range, in LDS past every wave's staging region
#pragma unroll
    for (int sft = CPR; sft < 64; sft <<= 1)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        rs[j] += __shfl_xor(rs[j], sft, 64);
        rq[j] += __shfl_xor(rq[j], sft, 64);
      }
    float* rr2 = reinterpret_cast<float*>(smem) + NW * 32 * LDC;  // [WM][BN][2]
    if (lane < CPR)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = wn * TN + cq * 8 + j;
        rr2[(wm * BN + c) * 2 + 0] = rs[j];
        rr2[(wm * BN + c) * 2 + 1] = rq[j];
      }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      if (n0 + c < g.Ncols) {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          a += rr2[(w * BN + c) * 2 + 0];
          b += rr2[(w * BN + c) * 2 + 1];
        }
        red.part[(prow * 2 + 0) * g.Ncols + n0 + c] = a;
        red.part[(prow * 2 + 1) * g.Ncols + n0 + c] = b * red.is[n0 + c];
      }
    }
  }
}

template <int BN, int WM, int WN, int MINW>
void launch_pipe(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                 const ConvGeomSet& gs, int ng, hipStream_t st, const BnBwdRed* red = nullptr,
                 const DgradSeg2* seg2 = nullptr) {
  const ConvGeom& g = gs.g[0];
  constexpr size_t STG = (size_t)PBM * PBK * 2 + (size_t)BN * PBK * 2;
  const size_t sm_main = 2 * STG;
  const size_t sm_epi = (size_t)WM * WN * 32 * (BN / WN + 4) * 4 + (red ? (size_t)WM * BN * 8 : 0);
  const size_t sm = sm_main > sm_epi ? sm_main : sm_epi;
  long long mmax = 0;
  for (int i = 0; i < ng; ++i) mmax = gs.g[i].M > mmax ? gs.g[i].M : mmax;
  const int mtiles = (int)((mmax + PBM - 1) / PBM);
  const int ntN = (g.Ncols + BN - 1) / BN;
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  if (seg2 && (seg2->C2 != g.C || seg2->z < 0 || seg2->z >= ng))
    throw std::runtime_error("conv_pipe: the merged segment needs X's channel count");
  auto k = red ? (seg2 ? conv_pipe_kernel<BN, WM, WN, MINW, true, true>
                       : conv_pipe_kernel<BN, WM, WN, MINW, true, false>)
               : (seg2 ? conv_pipe_kernel<BN, WM, WN, MINW, false, true>
                       : conv_pipe_kernel<BN, WM, WN, MINW, false, false>);
  const BnBwdRed rarg = red ? *red : BnBwdRed{};
  const DgradSeg2 sarg = seg2 ? *seg2 : DgradSeg2{};
  constexpr int NT = WM * WN * 64;
  set_smem_attr(k, sm);
  if (ntN > 1) {
    const unsigned mt8 = (unsigned)((mtiles + 7) / 8 * 8);
    k<<<dim3(mt8 * ntN, ng), NT, sm, st>>>(X, Wp, Y, ADD, stats, gs, xb, wb, ntN, mtiles, 1, rarg,
                                            sarg);
  } else {
    k<<<dim3((unsigned)mtiles, ng), NT, sm, st>>>(X, Wp, Y, ADD, stats, gs, xb, wb, 1, mtiles, 0,
                                                  rarg, sarg);
  }
  DM_CHECK(hipGetLastError());
}

template <int BN, int WM, int WN, int MINW>
void launch_pipe1(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                  const ConvGeom& g, hipStream_t st, const BnBwdRed* red) {
  launch_pipe<BN, WM, WN, MINW>(X, Wp, Y, ADD, stats, ConvGeomSet::one(g), 1, st, red);
}
}  // namespace

int pipe_bn(int cfg) { return cfg == 90 ? 256 : cfg == 93 ? 64 : 128; }

bool conv_pipe_supported(const ConvGeom& g, int cfg) {
  const int bn = pipe_bn(cfg);
  if (g.C % PBK != 0 || g.nth * g.ntw > 32 || g.Ncols % bn != 0) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  if ((long long)g.Ncols * g.wK * 2 >= (1LL << 31)) return false;
  if (g.M >= (1LL << 31) || g.C > 2048) return false;
  return true;
}

void conv_pipe(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int cfg, hipStream_t st, const BnBwdRed* red) {
  // 90: 256 x 256, 8 waves (2 x 4) of 128 x 64; 91: 256 x 128, 8 waves (4 x 2) of 64 x 64;
  // 92: 256 x 128, 4 waves (2 x 2) of 128 x 64; 93: 256 x 64, 4 waves (4 x 1) of 64 x 64,
  // two workgroups per CU (80 KB of LDS each)
  if (cfg == 90) launch_pipe1<256, 2, 4, 1>(X, Wp, Y, ADD, stats, g, st, red);
  else if (cfg == 91) launch_pipe1<128, 4, 2, 1>(X, Wp, Y, ADD, stats, g, st, red);
  else if (cfg == 92) launch_pipe1<128, 2, 2, 1>(X, Wp, Y, ADD, stats, g, st, red);
  else launch_pipe1<64, 4, 1, 2>(X, Wp, Y, ADD, stats, g, st, red);
}

// the parity classes of a stride-2 data gradient (no statistics) in one launch
bool conv_pipe_multi(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                     const ConvGeomSet& gs, int ng, int cfg, hipStream_t st, const DgradSeg2* seg2,
                     const BnBwdRed* red) {
  if (ng < 1 || ng > 4) return false;
  for (int i = 0; i < ng; ++i)
    if (!conv_pipe_supported(gs.g[i], cfg)) return false;
  if (seg2 && seg2->C2 != gs.g[0].C) return false;
  if (cfg == 90) launch_pipe<256, 2, 4, 1>(X, Wp, Y, ADD, nullptr, gs, ng, st, red, seg2);
  else if (cfg == 91) launch_pipe<128, 4, 2, 1>(X, Wp, Y, ADD, nullptr, gs, ng, st, red, seg2);
  else if (cfg == 92) launch_pipe<128, 2, 2, 1>(X, Wp, Y, ADD, nullptr, gs, ng, st, red, seg2);
  else launch_pipe<64, 4, 1, 2>(X, Wp, Y, ADD, nullptr, gs, ng, st, red, seg2);
  return true;
}

// part rows of a multi-geometry pipelined launch with the reduction epilogue
long long pipe_multi_rows(const ConvGeomSet& gs, int ng) {
  long long mmax = 0;
  for (int i = 0; i < ng; ++i) mmax = gs.g[i].M > mmax ? gs.g[i].M : mmax;
  return (long long)ng * ((mmax + PBM - 1) / PBM);
}

}  // namespace dm
