// Row-streaming weight gradient for 64 -> 64 channel 3x3 / stride-1 / pad-1 convolutions
// (ResNet-18 layer1), gfx950.  wgrad cfg 8.
//
//   dW[co, tap, c] = Σ_(n,y,x) dY[n,y,x, co] · X[n, y+dy_t, x+dx_t, c]
//
// The halo wgrad (wgrad_halo.hip) walks flattened 64-pixel chunks, so every transposed
// fragment read of every tap needs a per-lane image-boundary test and a select (the padding),
// and for layer1 (one 64 x 64 channel tile) it splits the 9 taps over 3 blocks that each
// re-stage the same dY tile: ~480-540 TF/s at batch 1024.  Here the unit of work is one image
// ROW, padded to 64 pixel slots:
//
//  * LDS holds a ring of input rows, each [66 slots][64 c] with zero slots at x = -1 and
//    x >= W, and a ring of dY rows [64 slots][64 co] with zero slots at x >= W (W <= 60).  A
//    tap (dy, dx) of output pixel x reads input slot x + 1 + dx of row y + dy, so EVERY
//    fragment address is a per-lane base plus a compile-time offset: no boundary tests in the
//    MFMA loop (rows outside the image read an all-zero row; the pad slots are the x padding
//    and the dY pad slots make the 64 - W dummy pixels contribute nothing).
//  * a persistent workgroup (8 waves, one per CU) owns a contiguous range of image rows and
//    accumulates the WHOLE 64 x 576 gradient in registers (72 per lane: wave w owns input
//    channels 16 (w & 3) .. +15 x output channels 32 (w >> 2) .. +31 x 9 taps); per row and
//    32-pixel k-step it reads 2 dY^T fragments and 9 shifted input fragments
//    (ds_read_b64_tr_b16, 160-B slot pitch: conflict-free) for 18 v_mfma_f32_16x16x32_bf16;
//  * rows stream in by LDS-DMA, two rows per iteration and two iterations ahead (5
//    instructions per wave per iteration; 60 lanes = 6 slots x 10 pieces, the last two pieces
//    of a slot and pixels x >= W read zero through the buffer range check), one barrier per
//    two rows, the fragments of k-step s+1 read while step s issues its MFMAs; the fused
//    pre-BN transform (PRE: the input
//    is the previous conv's raw output, the operand relu(x*sc + sh)) rewrites each thread's
//    landed input pieces before the barrier that publishes them;
//  * each workgroup writes one fp32 slab [64][576], reduced in fixed order by wgrad_reduce.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

#include <stdexcept>

namespace dm {

namespace {
constexpr int QC = 64;                    // channels (in and out)
constexpr int QP = 160;                   // LDS bytes per pixel slot (80 bf16: tr-read pitch)
constexpr int QXS = 66;                   // input slots per row (x = -1 .. 64)
constexpr int QDS = 64;                   // dY slots per row
constexpr int QRX = 8;                    // input-row ring
constexpr int QRD = 6;                    // dY-row ring
constexpr int Q_XROW = QXS * QP;          // 10,560 B
constexpr int Q_DROW = QDS * QP;          // 10,240 B
constexpr int Q_X = 0;                    // QRX input rows
constexpr int Q_Z = Q_X + QRX * Q_XROW;   // the all-zero input row
constexpr int Q_D = Q_Z + Q_XROW;         // QRD dY rows
constexpr int Q_SCR = Q_D + QRD * Q_DROW; // end of the zero-initialised region
constexpr int Q_TAB = Q_SCR;              // PRE scale / shift
constexpr int Q_SMEM = Q_TAB + 2 * QC * 4;
constexpr unsigned QOOB = 0x80000000u;

typedef short s4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ s4 qtr(unsigned lds_byte) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s4*)(size_t)lds_byte);
}

template <bool PRE>
__global__ void __launch_bounds__(512, 2) wgrad_res64_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ DY, float* __restrict__ slab,
    ConvGeom g, unsigned xbytes, unsigned dybytes, const float* __restrict__ pre_sc,
    const float* __restrict__ pre_sh, int nrows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = wid & 3, ch = wid >> 2;  // input-channel block (16), output-channel half (32)
  const int W = g.W, H = g.H;

  // contiguous range of flattened image rows r = n*H + y
  const int G = gridDim.x, b = blockIdx.x;
  const int per = nrows / G, rem = nrows % G;
  const int r0 = b * per + (b < rem ? b : rem);
  const int r1 = r0 + per + (b < rem ? 1 : 0);

  // zero everything once: the pad slots and the zero row are never written again
  for (int i = tid; i < Q_SCR / 16; i += 512)
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(0, 0, 0, 0);
  float* tab = reinterpret_cast<float*>(smem + Q_TAB);
  if (PRE && tid < QC) {
    tab[tid] = pre_sc[tid];
    tab[QC + tid] = pre_sh[tid];
  }

  const pi32x4 rsx = prsrc(X, xbytes);
  const pi32x4 rsd = prsrc(DY, dybytes);
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)smem;

  // DMA: a row is 10 instructions of 60 lanes (6 slots x 10 pieces; lanes 60-63 masked off).
  // lane l: slot l / 10, piece l % 10 (pieces 8, 9 = slot pad)
  const int dslot = lane / 10, dpiece = lane - dslot * 10;
  const bool dlane = lane < 60;
  // instruction jj (0..9) of a row: pixels 6 jj .. 6 jj + 5
  auto dma_row = [&](const pi32x4& rs, int row, int jj, unsigned lds_row, int rows_total) {
    const int x = 6 * jj + dslot;
    const bool ok = dpiece < 8 && x < W && (unsigned)row < (unsigned)rows_total;
    const unsigned off = ok ? (unsigned)((row * W + x) * 128 + dpiece * 16) : QOOB;
    if (dlane) pdma16(rs, lds_row + (unsigned)(jj * 6 * QP), off);
  };
  const int NR = g.N * H;  // image rows of the tensor
  auto xslot = [&](int row) { return (unsigned)(Q_X + ((row % QRX + QRX) % QRX) * Q_XROW); };
  auto dslotb = [&](int row) { return (unsigned)(Q_D + (row % QRD) * Q_DROW); };
  // the batch of iteration k (output rows r0 + 2k, +1): input rows r0 + 2k + 1, +2 and dY rows
  // r0 + 2k, +1 = 40 instructions, wave w issues w, w + 8, ..., w + 32 (input row pieces
  // j < 20 into slot x = 0 = byte QP of their ring slot, then dY rows)
  auto batch = [&](int k) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int j = wid + 8 * u;
      if (j < 20) {
        const int rx = r0 + 2 * k + 1 + j / 10;
        dma_row(rsx, rx, j % 10, lds0 + xslot(rx) + QP, NR);
      } else {
        const int rd = r0 + 2 * k + (j - 20) / 10;
        dma_row(rsd, rd, (j - 20) % 10, lds0 + dslotb(rd), NR);
      }
    }
  };
  // input-row-only loads (prologue): instructions w, w + 8 of 10
  auto xonly = [&](int rx) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = wid + 8 * u;
      if (j < 10) dma_row(rsx, rx, j, lds0 + xslot(rx) + QP, NR);
    }
  };
  // PRE: BN + ReLU of this thread's landed pieces of input row rx (piece instruction j)
  auto tpiece = [&](int rx, int j) __attribute__((always_inline)) {
    if constexpr (PRE) {
      const int x = 6 * j + dslot;
      if (dlane && dpiece < 8 && x < W) {
        uint4* p = reinterpret_cast<uint4*>(smem + xslot(rx) + QP + j * 6 * QP + lane * 16);
        const float4 s0 = *reinterpret_cast<const float4*>(tab + dpiece * 8);
        const float4 s1 = *reinterpret_cast<const float4*>(tab + dpiece * 8 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(tab + QC + dpiece * 8);
        const float4 h1 = *reinterpret_cast<const float4*>(tab + QC + dpiece * 8 + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        const uint4 v = *p;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float lo = fmaxf(__uint_as_float(w[q] << 16) * sc[2 * q] + sh[2 * q], 0.f);
          const float hi = fmaxf(__uint_as_float(w[q] & 0xffff0000u) * sc[2 * q + 1] + sh[2 * q + 1], 0.f);
          o[q] = pack_bf2(lo, hi);
        }
        *p = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  };
  auto xform_batch = [&](int k) __attribute__((always_inline)) {  // input rows of batch k
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int j = wid + 8 * u;
      if (j < 20) tpiece(r0 + 2 * k + 1 + j / 10, j % 10);
    }
  };
  auto xform_row = [&](int rx) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = wid + 8 * u;
      if (j < 10) tpiece(rx, j);
    }
  };

  // transpose-read lane roles (as wgrad_halo): rows grp*4 + q and +16 of a 32-pixel k-step,
  // columns 4p .. 4p+3 of a 16-channel block
  const int grp = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int rbase = grp * 4 + q4;
  const unsigned a_lane = (unsigned)(rbase * QP + (ch * 32 + 4 * p4) * 2);  // + i*32 B per co block
  const unsigned b_lane = (unsigned)(rbase * QP + (cb * 16 + 4 * p4) * 2);

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int niter = (r1 - r0 + 1) / 2;
  if (niter > 0) {
    __syncthreads();  // zeroed LDS before any DMA lands
    xonly(r0 - 1);
    xonly(r0);
    batch(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    xform_row(r0 - 1);
    xform_row(r0);
    __syncthreads();
    batch(1);
  }
  for (int it = 0; it < niter; ++it) {
    // this wave's batch it landed (batch it+1, 5 instructions, may not have)
    asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    xform_batch(it);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // the ring slots of iteration it-1's rows are free: prefetch two iterations ahead
    batch(it + 2);

    const int R = r0 + 2 * it;
    const bool two = R + 1 < r1;  // the second row belongs to this workgroup
    // input row bases per (output row ro, kernel row dyi): zero row outside the image
    unsigned xb[2][3], ab[2];
#pragma unroll
    for (int ro = 0; ro < 2; ++ro) {
      const int y = (R + ro) % H;
      xb[ro][0] = lds0 + (y > 0 ? xslot(R + ro - 1) : (unsigned)Q_Z) + b_lane;
      xb[ro][1] = lds0 + xslot(R + ro) + b_lane;
      xb[ro][2] = lds0 + (y + 1 < H ? xslot(R + ro + 1) : (unsigned)Q_Z) + b_lane;
      ab[ro] = lds0 + dslotb(R + ro) + a_lane;
    }
    // four 32-pixel k-steps (row ro = ks >> 1, half kb = ks & 1), fragments of step ks+1 read
    // while step ks issues its 18 MFMAs
    bf16x8 fa[2][2], fb[2][9];
    auto rdk = [&](int set, int ks) __attribute__((always_inline)) {
      const int ro = ks >> 1, kb = ks & 1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const s4 lo = qtr(ab[ro] + (kb * 32) * QP + i * 32);
        const s4 hi = qtr(ab[ro] + (kb * 32 + 16) * QP + i * 32);
        fa[set][i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dyi = t / 3, dxo = t % 3;  // input slot = x + dxo, row y + dyi - 1
        const s4 lo = qtr(xb[ro][dyi] + (kb * 32 + dxo) * QP);
        const s4 hi = qtr(xb[ro][dyi] + (kb * 32 + 16 + dxo) * QP);
        fb[set][t] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
    };
    auto mm = [&](int set) __attribute__((always_inline)) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[set][i], fb[set][t], acc[i][t], 0, 0, 0);
    };
    rdk(0, 0);
    rdk(1, 1);
    __builtin_amdgcn_sched_barrier(0);
    mm(0);
    __builtin_amdgcn_sched_barrier(0);
    if (two) {
      rdk(0, 2);
      __builtin_amdgcn_sched_barrier(0);
      mm(1);
      __builtin_amdgcn_sched_barrier(0);
      rdk(1, 3);
      __builtin_amdgcn_sched_barrier(0);
      mm(0);
      __builtin_amdgcn_sched_barrier(0);
      mm(1);
    } else {
      mm(1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetches past the range

  // slab[b][co][tap*64 + c]; 16x16 C map: col = lane & 15 (c), row = (lane>>4)*4 + r (co)
  float* out = slab + (long long)b * QC * 9 * QC;
  const int c = cb * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = ch * 32 + i * 16 + (lane >> 4) * 4 + rr;
        out[co * 9 * QC + t * QC + c] = acc[i][t][rr];
      }
}
}  // namespace

bool wgrad_res64_supported(const ConvGeom& g) {
  if (g.C != QC || g.Ncols != QC || g.K != 9 * QC) return false;
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W || g.W > 60) return false;
  if (g.nth != 3 || g.ntw != 3 || g.dy0 != -1 || g.dys != 1 || g.dx0 != -1 || g.dxs != 1) return false;
  if (g.kh0 != 0 || g.khs != 1 || g.kw0 != 0 || g.kws != 1 || g.KW != 3) return false;
  return (long long)g.N * g.H * g.W * QC * 2 < (1LL << 31);
}

// S = slab count = workgroups (each owns a contiguous range of the N*H image rows)
void wgrad_res64(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                 hipStream_t st, const float* pre_sc, const float* pre_sh) {
  if (!wgrad_res64_supported(g)) throw std::runtime_error("wgrad_res64: unsupported geometry");
  const int nrows = g.N * g.H;
  if (S < 1 || S > nrows) throw std::runtime_error("wgrad_res64: S must be in [1, N*H]");
  const unsigned bytes = (unsigned)((long long)g.N * g.H * g.W * QC * 2);
  auto k = pre_sc ? wgrad_res64_kernel<true> : wgrad_res64_kernel<false>;
  set_smem_attr(k, Q_SMEM);
  k<<<S, 512, Q_SMEM, st>>>(X, DY, slab, g, bytes, bytes, pre_sc, pre_sh, nrows);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
