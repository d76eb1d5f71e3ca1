// Register-resident-weight 3x3 convolution for 64 -> 64 channels (ResNet-18 layer1: forward and
// the stride-1 data gradient), gfx950.  cfg 80.
//
// Layer1 runs 8 of these convs per step (4 forward, 4 data gradients) over 1024 x 56 x 56
// pixels.  With only 64 output channels the halo tile (conv_halo.hip cfg 39) re-stages a
// 64 x 64 weight tile through LDS at every tap (9 barriers per tile, 72 KB of weight traffic
// per 256 pixels) and its single-chunk halo prologue is exposed: ~400-450 TF/s in the step.
// The whole weight tensor is only 9 x 64 x 64 bf16 = 72 KB, so here it never touches LDS:
//
//  * 4 waves per workgroup, 2 (64-pixel halves) x 2 (32-channel halves).  Each wave keeps the
//    MFMA B fragments of its 32 output channels for all 9 taps x 4 k-substeps in VGPRs
//    (144 registers, loaded once: the kernel is persistent) and reads only A fragments from
//    LDS: per 16-deep substep 2 ds_read_b128 feed 2 v_mfma_f32_32x32x16_bf16.
//  * A 128-pixel output tile reads the flattened input rows m0-W-1 .. m0+128+W (the halo),
//    landed by LDS-DMA (buffer_load_dwordx4 ... lds) into a 144-B-pitch image: with 36-dword
//    rows, any 16 consecutive rows of a fragment read fall on distinct banks for EVERY tap
//    shift, so the tap's row offset is a plain add (no per-tap swizzle) and the k-substep is
//    the instruction's immediate offset.  The 9th 16-B slot of a row is the DMA's pad (reads
//    zero through the buffer range check).  A tap that leaves the image reads a zero row.
//  * One barrier per tile.  The next tile's halo DMA is issued right after it, into the same
//    stage, and lands while this wave runs its epilogue; two workgroups per CU (56 KB of LDS
//    each) keep the MFMA pipe fed while the other one waits for its DMA.
//  * Epilogue: per-channel BN statistics accumulate in two registers per lane across all the
//    workgroup's tiles (one stats row per workgroup, reduced once at exit); the fp32 tile goes
//    through a per-wave LDS band to 16-B bf16 buffer stores (optional residual ADD), no
//    cross-wave barrier.
//  * PRE: the input is the previous conv's raw output and the operand is relu(x*sc + sh):
//    each thread rewrites the 16-B chunks its own DMA landed before the publishing barrier.
//
// Workgroups own contiguous tile ranges, so the 2W+2 halo rows two consecutive tiles share
// are re-read from this XCD's L2, not HBM.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <stdexcept>

namespace dm {

namespace {
constexpr int RT = 128;                 // output pixels per tile
constexpr int RC = 64;                  // channels in and out
constexpr int RNT = 256;                // threads: 4 waves
constexpr int RPITCH = 144;             // LDS bytes per halo row (128 B + 16 B DMA pad)
constexpr int RDMA = 9;                 // LDS-DMA instructions per wave per tile
constexpr int RSLOTS = RDMA * RNT;      // 16-B slots of the halo image (9 per row)
constexpr int RHMAX = RSLOTS / 9;       // halo rows the image holds (256: W <= 63)
constexpr unsigned ROOB = 0x80000000u;
constexpr unsigned R_PADOFF = 0x40000000u;  // DMA pad pieces: past every supported tensor
constexpr int R_ZROW = RSLOTS * 16;     // zero row
constexpr int R_TAB = R_ZROW + RPITCH;  // PRE scale / shift (2 x 64 floats)
constexpr int R_EPI = R_TAB + 2 * RC * 4;
constexpr int R_LDC = 36;               // epilogue band pitch (floats): 32 rows x 32 columns
constexpr int R_SMEM = R_EPI + 4 * 32 * R_LDC * 4;
// RED (BN-backward reduction of the next layer, dgrad only): the reduced BN's sc / sh / mu,
// per-lane running sums [4 waves][64 lanes][2], and the tile's y (that BN's input) landed by
// LDS-DMA as [channel half][128 pixels][32 channels].  Nothing of it lives in registers
// across tiles: the kernel already holds 240 of its 256 VGPRs.
constexpr int R_RTAB = R_SMEM;
constexpr int R_RACC = R_RTAB + 3 * RC * 4;
constexpr int R_Y = R_RACC + RNT * 2 * 4;
constexpr int R_MK = R_Y + RT * RC * 2;  // the tile's 1-bit ReLU mask (8 B per pixel)
constexpr int R_SMEM_RED = R_MK + RT * 8;
typedef unsigned v4u32_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int div9(int s) { return (s * 7282) >> 16; }  // exact for s < 3584
// an opaque copy: values derived from it are recomputed per tile instead of being hoisted out
// of the tile loop (18 tap addresses + 27 DMA slot terms would not fit the 256-register budget)
__device__ __forceinline__ unsigned opq(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}

template <bool PRE, bool RED>
__global__ void __launch_bounds__(RNT, 2) conv_res64_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, unsigned ybytes,
    const float* __restrict__ pre_sc, const float* __restrict__ pre_sh, int ntiles,
    BnBwdRed red) {
  static_assert(!(PRE && RED), "RED is a data-gradient epilogue (no PRE input)");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const int hsel = lane >> 5, l32 = lane & 31;

  // contiguous tile range of this workgroup
  const int G = gridDim.x, b = blockIdx.x;
  const int per = ntiles / G, rem = ntiles % G;
  const int t_begin = b * per + (b < rem ? b : rem);
  const int t_end = t_begin + per + (b < rem ? 1 : 0);

  // B fragments (k = 16 ks + 8 hsel .. +7, column = output channel) of all taps -> VGPRs
  bf16x8 wr[9][4];
  {
    const int co = wn * 32 + l32;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int th = t / 3, tw = t % 3;
      const int kt = (g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws);
      const bf16_t* wp = Wp + (long long)co * g.wK + kt * RC + hsel * 8;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) wr[t][ks] = *reinterpret_cast<const bf16x8*>(wp + ks * 16);
    }
  }
  // tap t reads halo row p + W + 1 + (dy W + dx): byte offsets of the shift
  int toff[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int th = t / 3, tw = t % 3;
    toff[t] = ((g.dy0 + th * g.dys) * g.W + (g.dx0 + tw * g.dxs)) * RPITCH;
  }
  if (tid < 9) *reinterpret_cast<uint4*>(smem + R_ZROW + tid * 16) = make_uint4(0, 0, 0, 0);
  float* tab = reinterpret_cast<float*>(smem + R_TAB);
  if (PRE && tid < RC) {
    tab[tid] = pre_sc[tid];
    tab[RC + tid] = pre_sh[tid];
  }
  if (RED) {
    float* rtab = reinterpret_cast<float*>(smem + R_RTAB);
    if (tid < RC) {
      rtab[tid] = red.sc[tid];
      rtab[RC + tid] = red.sh[tid];
      rtab[2 * RC + tid] = red.mu[tid];
    }
    reinterpret_cast<float2*>(smem + R_RACC)[tid] = make_float2(0.f, 0.f);
  }

  const pi32x4 rsx = prsrc(X, xbytes);
  const auto rsy = __builtin_amdgcn_make_buffer_rsrc((void*)Y, (short)0, (int)ybytes, 0x00020000);
  const auto rsa =
      __builtin_amdgcn_make_buffer_rsrc((void*)(ADD ? ADD : Y), (short)0, (int)ybytes, 0x00020000);
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)smem;

  // halo of tile tt -> LDS image: piece s (16 B) of the image is piece s % 9 of halo row s / 9.
  // pb[j]: byte offset of this thread's piece j relative to the halo's first pixel (pad pieces
  // pushed past any tensor), so a tile's source offset is ONE add: the buffer range check turns
  // rows before the tensor (negative, wrapped) or past it into zeros
  unsigned pb[RDMA];
#pragma unroll
  for (int j = 0; j < RDMA; ++j) {
    const int s = (j * 4 + wid) * 64 + lane;
    const int row = div9(s), c = s - row * 9;
    pb[j] = c < 8 ? (unsigned)(row * 128 + c * 16) : R_PADOFF;
  }
  // RED: y of tile tt -> R_Y; LDS piece s = (j*4 + wid)*64 + lane is channel half s >> 9,
  // pixel (s >> 2) & 127, 16-B chunk s & 3 (rows past M read zero)
  const pi32x4 rsr = prsrc(RED ? (const void*)red.y : (const void*)X, ybytes);
  const pi32x4 rsm = prsrc(RED && red.mask ? (const void*)red.mask : (const void*)X, ybytes >> 4);
  auto ydma = [&](int tt) __attribute__((always_inline)) {
    // the 1-bit mask of the tile's 128 pixels is 1 KB: one instruction of wave 0
    if (red.mask && wid == 0) pdma16(rsm, lds0 + (unsigned)R_MK, (unsigned)tt * (RT * 8u) + lane * 16u);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const unsigned s = (unsigned)(j * 4 + wid) * 64u + opq((unsigned)lane);
      const unsigned off = (unsigned)tt * (RT * 128u) + ((s >> 2) & 127u) * 128u + (s >> 9) * 64u +
                           (s & 3u) * 16u;
      pdma16(rsr, lds0 + (unsigned)(R_Y + (j * 4 + wid) * 1024), off);
    }
  };
  auto dma = [&](int tt) __attribute__((always_inline)) {
    const unsigned hs = (unsigned)((tt * RT - g.W - 1) * 128);
#pragma unroll
    for (int j = 0; j < RDMA; ++j) pdma16(rsx, lds0 + (unsigned)(j * 4 + wid) * 1024u, hs + pb[j]);
  };
  // PRE: BN + ReLU of the chunks this thread's DMA landed (pad pieces stay zero; rows outside
  // the image are never read: their taps go to the zero row)
  auto transform = [&]() __attribute__((always_inline)) {
    if constexpr (PRE) {
#pragma unroll
      for (int j = 0; j < RDMA; ++j) {
        if (pb[j] < R_PADOFF) {
          const int c = (int)((pb[j] >> 4) & 7u);
          uint4* q = reinterpret_cast<uint4*>(smem + ((j * 4 + wid) * 64 + lane) * 16);
          const float4 s0 = *reinterpret_cast<const float4*>(tab + c * 8);
          const float4 s1 = *reinterpret_cast<const float4*>(tab + c * 8 + 4);
          const float4 h0 = *reinterpret_cast<const float4*>(tab + RC + c * 8);
          const float4 h1 = *reinterpret_cast<const float4*>(tab + RC + c * 8 + 4);
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
          const uint4 v = *q;
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float lo = fmaxf(__uint_as_float(w[k] << 16) * sc[2 * k] + sh[2 * k], 0.f);
            const float hi = fmaxf(__uint_as_float(w[k] & 0xffff0000u) * sc[2 * k + 1] + sh[2 * k + 1], 0.f);
            o[k] = pack_bf2(lo, hi);
          }
          *q = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
    }
  };

  // fragment rows: lane's pixel p = wm*64 + i*32 + l32 of the tile, halo row p + W + 1
  unsigned hb[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) hb[i] = (unsigned)((wm * 64 + i * 32 + l32 + g.W + 1) * RPITCH + hsel * 16);
  const unsigned zad = (unsigned)(R_ZROW + hsel * 16);

  float* cs = reinterpret_cast<float*>(smem + R_EPI) + wid * 32 * R_LDC;
  float ssum = 0.f, ssq = 0.f;

  if (t_begin < t_end) {
    __syncthreads();  // zero row / table written
    dma(t_begin);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    transform();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  for (int tt = t_begin; tt < t_end; ++tt) {
    const int m0 = tt * RT;
    // every wave is past the previous tile's epilogue (loop-end barrier): y(tt) may land
    if (RED) ydma(tt);
    // taps inside the image, per fragment row (bit th*3 + tw)
    unsigned mk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = m0 + wm * 64 + i * 32 + l32;
      const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - r * (unsigned)g.W);
      const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
      const int y = (int)(r - n * (unsigned)g.H);
      unsigned xm = 0, ym = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        xm |= ((unsigned)(x + g.dx0 + k * g.dxs) < (unsigned)g.W ? 1u : 0u) << k;
        ym |= ((unsigned)(y + g.dy0 + k * g.dys) < (unsigned)g.H ? 1u : 0u) << k;
      }
      unsigned v = ((ym & 1u) ? xm : 0u) | ((ym & 2u) ? xm << 3 : 0u) | ((ym & 4u) ? xm << 6 : 0u);
      mk[i] = m < g.M ? v : 0u;
    }
    f32x16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    // 36 (tap, 16-deep substep) steps of two MFMAs (one per 32-pixel row block)
    const unsigned hbt[2] = {opq(hb[0]), opq(hb[1])};
    auto addr = [&](int i, int t) __attribute__((always_inline)) {
      return ((mk[i] >> t) & 1u) ? hbt[i] + toff[t] : zad;
    };
    bf16x8 fr[3][2];
    auto rd = [&](int set, int u) __attribute__((always_inline)) {
      const int t = u >> 2, ks = u & 3;
      fr[set][0] = *reinterpret_cast<const bf16x8*>(smem + addr(0, t) + ks * 32);
      fr[set][1] = *reinterpret_cast<const bf16x8*>(smem + addr(1, t) + ks * 32);
    };
    // reads run two steps ahead of the MFMAs (three fragment sets); sched_barrier keeps the
    // compiler from regrouping the two accumulator chains and re-using one fragment register
    rd(0, 0);
    rd(1, 1);
#pragma unroll
    for (int u = 0; u < 36; ++u) {
      if (u + 2 < 36) rd((u + 2) % 3, u + 2);
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[u % 3][0], wr[u >> 2][u & 3], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[u % 3][1], wr[u >> 2][u & 3], acc[1], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave is done reading the halo image: the next tile's DMA may overwrite it
    // (RED: and every wave's share of y(tt), issued a whole tile ago, has landed)
    if (RED) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const bool more = tt + 1 < t_end;
    if (more) dma(tt + 1);

    // epilogue: statistics, then 32-row bands through this wave's LDS region to 16-B stores
    // RED: this lane's channel (its MFMA output column) is fixed; its BN constants are
    // re-read per tile through a laundered address (kept out of the register budget)
    float rsc = 0.f, rsh = 0.f, rmu = 0.f;
    red_f2 rs2 = {0.f, 0.f}, rq2 = {0.f, 0.f};
    const unsigned char* ybase = smem;
    const unsigned char* mbase = smem;
    if constexpr (RED) {
      ybase = smem + opq((unsigned)(R_Y + wn * 8192 + (wm * 64 + 4 * hsel) * 64 + l32 * 2));
      mbase = smem + opq((unsigned)(R_MK + (wm * 64 + 4 * hsel) * 8 + wn * 4 + (l32 >> 3)));
      const float* rt = reinterpret_cast<const float*>(smem + opq((unsigned)(R_RTAB + (wn * 32 + l32) * 4)));
      rsc = rt[0];
      rsh = rt[RC];
      rmu = rt[2 * RC];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v = acc[i][r];
        if constexpr (!RED) {  // (data gradients have no statistics)
          ssum += v;
          ssq += v * v;
        }
        cs[((r & 3) + 8 * (r >> 2) + 4 * hsel) * R_LDC + l32] = v;
      }
#pragma unroll
      for (int it = 0; it < 2; ++it) {
        const int rr = it * 16 + (lane >> 2), cq = lane & 3;
        const int m = m0 + wm * 64 + i * 32 + rr;
        const unsigned off =
            m < g.M ? ((unsigned)m * (unsigned)RC + (unsigned)(wn * 32 + cq * 8)) * 2u : ROOB;
        const float4 v0 = *reinterpret_cast<const float4*>(cs + rr * R_LDC + cq * 8);
        const float4 v1 = *reinterpret_cast<const float4*>(cs + rr * R_LDC + cq * 8 + 4);
        float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        if (ADD) {
          const auto a = __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0);
          // identity-skip ReLU mask: one byte per 16-B chunk (byte offset / 16)
          const unsigned mb = (g.addm && off != ROOB) ? g.addm[off >> 4] : 0xffu;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            v[2 * q] += ((mb >> (2 * q)) & 1u) ? __uint_as_float((unsigned)a[q] << 16) : 0.f;
            v[2 * q + 1] += ((mb >> (2 * q + 1)) & 1u) ? __uint_as_float((unsigned)a[q] & 0xffff0000u) : 0.f;
          }
        }
        const v4u32_t o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                           pack_bf2(v[6], v[7])};
        // non-temporal (aux bit 1): the output streams past L2/MALL (+1.1 % per step with
        // the other conv epilogues, profiles/conv_nt_stores_ab_r4ab.txt)
        __builtin_amdgcn_raw_buffer_store_b128(o, rsy, off, 0, 2);
        if (RED && ADD) {  // the band keeps the stored values for the reduction below
          *reinterpret_cast<float4*>(cs + rr * R_LDC + cq * 8) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(cs + rr * R_LDC + cq * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
      if constexpr (RED) {
        // dz = the stored (bf16) gradient where the reduced BN's ReLU passed, read back from
        // the band in the MFMA layout (this lane's channel is its column)
        // (rows r, r + 1 as a packed pair: one bf16 rounding for both, packed fp32 FMA/add;
        // the mask / ReLU-condition choice is made once, outside the row loop: a per-element
        // uniform branch split the loop into blocks and kept the LDS reads unpaired)
        auto rows = [&](auto mtag) __attribute__((always_inline)) {
          constexpr bool MK = decltype(mtag)::value;
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            red_f2 v2, y2, g2;
            unsigned mk[2];
            float vv[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int rh = r + h;
              const int row = (rh & 3) + 8 * (rh >> 2) + 4 * hsel;
              const int pr = i * 32 + (rh & 3) + 8 * (rh >> 2);  // + wm*64 + 4*hsel in ybase
              vv[h] = cs[row * R_LDC + l32];
              y2[h] = __uint_as_float(
                  (unsigned)*reinterpret_cast<const unsigned short*>(ybase + pr * 64) << 16);
              // bit -> all-ones / zero (mask mode), then AND
              mk[h] = MK ? (unsigned)((int)((unsigned)mbase[pr * 8] << (31 - (l32 & 7))) >> 31)
                         : 0xffffffffu;
            }
            const unsigned pk = pack_bf2(vv[0], vv[1]);  // the stored values
            v2.x = __uint_as_float((pk << 16) & mk[0]);
            v2.y = __uint_as_float(pk & 0xffff0000u & mk[1]);
            if constexpr (MK) {
              g2 = v2;
            } else {
              const red_f2 t = y2 * red_f2{rsc, rsc} + red_f2{rsh, rsh};
              g2.x = t.x > 0.f ? v2.x : 0.f;
              g2.y = t.y > 0.f ? v2.y : 0.f;
            }
            rs2 += g2;
            rq2 += g2 * (y2 - red_f2{rmu, rmu});
            // bound the LDS reads in flight (the scheduler would hoist all of them)
            if ((r & 3) == 2) __builtin_amdgcn_sched_barrier(0);
          }
        };
        if (red.mask) rows(std::true_type{});
        else rows(std::false_type{});
      }
    }
    if constexpr (RED) {
      float2* ra = reinterpret_cast<float2*>(smem + R_RACC) + tid;
      const float2 o = *ra;
      *ra = make_float2(o.x + (rs2.x + rs2.y), o.y + (rq2.x + rq2.y));
    }
    if (more) {
      // the DMA is older than the 4 stores above: vmcnt(4) retires it, not them
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      transform();
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }

  if constexpr (RED) {
    // workgroup row: both row halves (hsel) and the two pixel-half waves (wm) add up;
    // Σdz(y - mu) scales by invstd
    // lane slot tid = (wm*2 + wn)*64 + hsel*32 + l32 holds channel wn*32 + l32
    __syncthreads();
    const float2* ra = reinterpret_cast<const float2*>(smem + R_RACC);
    if (tid < RC) {
      const int h = tid >> 5, c = tid & 31;
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < 2; ++w)
#pragma unroll
        for (int hs = 0; hs < 2; ++hs) {
          const float2 v = ra[(w * 2 + h) * 64 + hs * 32 + c];
          s += v.x;
          q += v.y;
        }
      red.part[(long long)b * 2 * RC + tid] = s;
      red.part[(long long)b * 2 * RC + RC + tid] = q * red.is[tid];
    }
  }
  if (!RED && stats) {
    ssum += __shfl_xor(ssum, 32, 64);
    ssq += __shfl_xor(ssq, 32, 64);
    __syncthreads();  // staging bands free
    float* red = reinterpret_cast<float*>(smem + R_EPI);
    if (lane < 32) {
      red[(wm * RC + wn * 32 + l32) * 2 + 0] = ssum;
      red[(wm * RC + wn * 32 + l32) * 2 + 1] = ssq;
    }
    __syncthreads();
    if (tid < RC) {
      stats[((long long)b * 2 + 0) * RC + tid] = red[tid * 2 + 0] + red[(RC + tid) * 2 + 0];
      stats[((long long)b * 2 + 1) * RC + tid] = red[tid * 2 + 1] + red[(RC + tid) * 2 + 1];
    }
  }
}

int cu_count() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return cus;
}
}  // namespace

int res64_grid(long long M) {
  const long long ntiles = (M + RT - 1) / RT;
  const long long g = 2LL * cu_count();  // two workgroups per CU
  return (int)(ntiles < g ? ntiles : g);
}

bool conv_res64_supported(const ConvGeom& g) {
  if (g.C != RC || g.Ncols != RC || g.OC != RC || g.wK != 9 * RC) return false;
  if (g.nth != 3 || g.ntw != 3 || g.KW != 3) return false;
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W) return false;
  if (g.OH != g.H || g.OW != g.W || g.osy != 1 || g.osx != 1 || g.oy0 != 0 || g.ox0 != 0) return false;
  auto in1 = [](int v) { return v >= -1 && v <= 1; };
  if (!in1(g.dy0) || !in1(g.dy0 + 2 * g.dys) || !in1(g.dx0) || !in1(g.dx0 + 2 * g.dxs)) return false;
  if (RT + 2 * g.W + 2 > RHMAX) return false;
  // pad pieces sit at R_PADOFF + (halo start) bytes: the tensor must end below 2^30 - 2^14
  if ((long long)g.N * g.H * g.W * RC * 2 >= (1LL << 30) - (1LL << 14) ||
      g.M != (long long)g.N * g.H * g.W)
    return false;
  return true;
}

void conv_res64(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                const ConvGeom& g, hipStream_t st, const float* pre_sc, const float* pre_sh,
                const BnBwdRed* red) {
  if (!conv_res64_supported(g)) throw std::runtime_error("conv_res64: unsupported geometry");
  const int grid = res64_grid(g.M);
  const unsigned bytes = (unsigned)(g.M * RC * 2);
  const int ntiles = (int)((g.M + RT - 1) / RT);
  if (red) {
    if (pre_sc || !red->y || !red->sc || !red->sh || !red->mu || !red->is ||
        !red->part)
      throw std::runtime_error("conv_res64: BN-backward reduction needs y, sc, sh, mu, is, part "
                               "(no PRE input)");
    set_smem_attr(conv_res64_kernel<false, true>, R_SMEM_RED);
    conv_res64_kernel<false, true><<<grid, RNT, R_SMEM_RED, st>>>(
        X, Wp, Y, ADD, stats, g, bytes, bytes, pre_sc, pre_sh, ntiles, *red);
  } else {
    auto k = pre_sc ? conv_res64_kernel<true, false> : conv_res64_kernel<false, false>;
    set_smem_attr(k, R_SMEM);
    k<<<grid, RNT, R_SMEM, st>>>(X, Wp, Y, ADD, stats, g, bytes, bytes, pre_sc, pre_sh, ntiles,
                                 BnBwdRed{});
  }
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
