// Shared device helpers of the implicit-GEMM conv kernels (conv_igemm.hip, conv_halo.hip).
#pragma once
#include "common.h"
#include "conv_geom.h"
#include "kernels.h"

#include <type_traits>

namespace dm {

template <typename K>
static void set_smem_attr(K kernel, size_t bytes) {
  // dynamic LDS above 64 KiB must be opted into per kernel (idempotent, cheap)
  if (bytes > 65536)
    DM_CHECK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)bytes));
}

__device__ __forceinline__ unsigned fdiv(unsigned n, unsigned mul, unsigned shr) {
  return (__umulhi(n, mul) + n) >> shr;
}

// 16-B chunk swizzle of a 128-B LDS row: conflict-free for 8-lane row writes and for the
// 16- and 32-row fragment reads of both MFMA shapes
__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// Buffer resource for LDS-DMA issued from inline asm (range-checked: offsets >= bytes read 0)
typedef int pi32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ pi32x4 prsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  pi32x4 r;
  r[0] = (int)(unsigned)a;
  r[1] = (int)(unsigned)(a >> 32) & 0xffff;
  r[2] = (int)bytes;
  r[3] = 0x00020000;
  return r;
}

// LDS-DMA: lane l's 16 bytes at buffer byte `off` -> LDS byte lds + 16*l (lds wave-uniform).
// Issued from inline asm so the compiler's alias-blind LDS-DMA tracking does not put a
// vmcnt(0) before every ds_read; the caller retires it with its own s_waitcnt vmcnt.
__device__ __forceinline__ void pdma16(const pi32x4& rs, unsigned lds, unsigned off) {
  lds = __builtin_amdgcn_readfirstlane(lds);  // keep M0's source an SGPR under register pressure
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %2, 0 offen lds"
      :
      : "v"(off), "s"(lds), "s"(rs)
      : "memory");
}

// Fused BatchNorm-apply + ReLU of a staged 16-B chunk (8 bf16 channels c0..c0+7):
// v = max(v * sc[c] + sh[c], 0).  Used by the halo kernels to read a conv's RAW output and
// consume BN(y) directly, so the normalised activation is never written to memory.
struct PreBN {
  float sc[8], sh[8];
  __device__ __forceinline__ void load(const float* __restrict__ scale,
                                       const float* __restrict__ shift, int c0) {
    const float4 a = *reinterpret_cast<const float4*>(scale + c0);
    const float4 b = *reinterpret_cast<const float4*>(scale + c0 + 4);
    const float4 c = *reinterpret_cast<const float4*>(shift + c0);
    const float4 d = *reinterpret_cast<const float4*>(shift + c0 + 4);
    sc[0] = a.x; sc[1] = a.y; sc[2] = a.z; sc[3] = a.w;
    sc[4] = b.x; sc[5] = b.y; sc[6] = b.z; sc[7] = b.w;
    sh[0] = c.x; sh[1] = c.y; sh[2] = c.z; sh[3] = c.w;
    sh[4] = d.x; sh[5] = d.y; sh[6] = d.z; sh[7] = d.w;
  }
  __device__ __forceinline__ uint4 apply(uint4 v) const {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float lo = fmaxf(bf2f((bf16_t)(w[q] & 0xffff)) * sc[2 * q] + sh[2 * q], 0.f);
      const float hi = fmaxf(bf2f((bf16_t)(w[q] >> 16)) * sc[2 * q + 1] + sh[2 * q + 1], 0.f);
      o[q] = pack_bf2(lo, hi);
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
  }
};

// BatchNorm backward of a staged 16-B chunk of that BN's output gradient (8 bf16 channels,
// kernels.h BnBwdIn): dy = a*dz' + b*y + c, the arithmetic of bn_bwd_apply_kernel.  The
// coefficients live in an LDS table [5][n] (a, b, c, sc, sh of n channels, bwd_tab_fill) and
// are read per chunk through an opaque address, so they occupy no registers across the
// consumer's MFMA loop (held in VGPRs they spilled both halo kernels: 76 / 220 spills).
__device__ __forceinline__ unsigned opq_u(unsigned v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void bwd_tab_fill(float* tab, const BnBwdIn& in, int cbase, int n,
                                             int tid, int nt) {
  for (int i = tid; i < 5 * n; i += nt) {
    const int k = i / n, c = cbase + i % n;
    float v;
    if (k < 3) v = in.coef[k * in.C + c];
    else if (in.mode == 2) v = (k == 3 ? in.sc : in.sh)[c];
    else v = k == 3 ? 0.f : 1.f;  // no ReLU from y: y*0 + 1 > 0, every element passes
    tab[i] = v;
  }
}

// tab: the table, n its channel count, ci the chunk's first channel (relative to the table);
// mb: the chunk's mask byte (mode 4) or 0xff.  Two halves of 4 channels, so at most 20
// coefficients are live at a time.
// SB: a scheduling barrier after each half (keeps the halves' coefficients from being loaded
// together; helps the data-gradient tile, hurts the weight-gradient one)
template <bool SB = true>
__device__ __forceinline__ uint4 bwd_apply(const float* tab, int n, int ci, uint4 dz, uint4 y,
                                           unsigned mb) {
  const uint32_t dw[4] = {dz.x, dz.y, dz.z, dz.w};
  const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
  uint32_t o[4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float* t = tab + opq_u((unsigned)(ci + 4 * h));
    const float4 va = *reinterpret_cast<const float4*>(t);
    const float4 vb = *reinterpret_cast<const float4*>(t + n);
    const float4 vc = *reinterpret_cast<const float4*>(t + 2 * n);
    const float4 vs = *reinterpret_cast<const float4*>(t + 3 * n);
    const float4 vh = *reinterpret_cast<const float4*>(t + 4 * n);
    const float a[4] = {va.x, va.y, va.z, va.w}, b[4] = {vb.x, vb.y, vb.z, vb.w};
    const float c[4] = {vc.x, vc.y, vc.z, vc.w}, sc[4] = {vs.x, vs.y, vs.z, vs.w};
    const float sh[4] = {vh.x, vh.y, vh.z, vh.w};
#pragma unroll
    for (int q2 = 0; q2 < 2; ++q2) {
      const int q = 2 * h + q2;
      float r[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int jj = 2 * q2 + hh, j = 2 * q + hh;
        const float d = __uint_as_float(hh ? (dw[q] & 0xffff0000u) : (dw[q] << 16));
        const float yv = __uint_as_float(hh ? (yw[q] & 0xffff0000u) : (yw[q] << 16));
        const bool pass = ((mb >> j) & 1u) && (yv * sc[jj] + sh[jj]) > 0.f;
        r[hh] = a[jj] * (pass ? d : 0.f) + b[jj] * yv + c[jj];
      }
      o[q] = pack_bf2(r[0], r[1]);
    }
    if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// the mask byte of the 16-B chunk at byte offset `off` of an NHWC bf16 tensor (mode 4), or 0xff:
// a range-checked buffer load (0-byte resource when there is no mask), never a branch
__device__ __forceinline__ unsigned bwd_mask_byte(const BnBwdIn& in, unsigned off, unsigned mbytes) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(in.mask ? in.mask : (const uint8_t*)in.coef),
                                                    (short)0, (int)(in.mask ? mbytes : 0u), 0x00020000);
  const unsigned v = __builtin_amdgcn_raw_buffer_load_b8(rs, off >> 4, 0, 0);
  return in.mode == 4 ? v : 0xffu;
}

template <bool MF32>
using mfma_acc_t = typename std::conditional<MF32, f32x16, f32x4>::type;

// Epilogue of a BM x BN MFMA tile held by WM x WN waves (each TM x TN as FM x FM blocks).
// C/D maps: 16x16 col = l&15, row = (l>>4)*4 + r;  32x32 col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
//  * optional BN statistics: per-column Σy, Σy² of the fp32 tile -> stats[stat_row][2][Ncols]
//  * fp32 tile staged through LDS (row pitch BN+4) -> coalesced 16-B bf16 stores at the
//    output pixel (y*osy+oy0, x*osx+ox0), optionally adding ADD (which may alias Y).
// Rows >= g.M must hold zeros when stats are requested.  Requires (BM/PASSES)*(BN+4)*4 B of
// LDS: with PASSES > 1 the tile is staged one band of BM/PASSES rows (whole wave rows) at a time.
// RED (data gradients, kernels.h BnBwdRed): the backward reduction of the BatchNorm whose
// output gradient Y is, from the stored bf16 values and that BN's input y (prefetched with
// the ADD chunks): one [2][Ncols] row per stat_row in red.part.
typedef float red_f2 __attribute__((ext_vector_type(2)));
// RED epilogue, one output row of 8 channels: dz = the stored (bf16) gradient o where the
// consumer's ReLU passed (bit j of the 1-bit mask, or y*sc + sh > 0), rs += dz,
// rq += dz (y - mu), channel pairs packed (the sums are those of the values the unfused
// reduction would re-read)
template <bool MASK>
__device__ __forceinline__ void red_acc8(const uint4& ov, const uint4& yv, unsigned ym,
                                         red_f2 (&rs)[4], red_f2 (&rq)[4], const red_f2 (&sc)[4],
                                         const red_f2 (&sh)[4], const red_f2 (&mu)[4]) {
  const uint32_t yw[4] = {yv.x, yv.y, yv.z, yv.w}, ow[4] = {ov.x, ov.y, ov.z, ov.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    red_f2 y2, g2;
    y2.x = __uint_as_float(yw[q] << 16);
    y2.y = __uint_as_float(yw[q] & 0xffff0000u);
    if constexpr (MASK) {
      // bit -> all-ones / zero (one signed bit-field extract), then AND: no compare, no select
      g2.x = __uint_as_float((ow[q] << 16) & (unsigned)((int)(ym << (31 - 2 * q)) >> 31));
      g2.y = __uint_as_float(ow[q] & 0xffff0000u & (unsigned)((int)(ym << (30 - 2 * q)) >> 31));
    } else {
      const red_f2 t = y2 * sc[q] + sh[q];
      g2.x = t.x > 0.f ? __uint_as_float(ow[q] << 16) : 0.f;
      g2.y = t.y > 0.f ? __uint_as_float(ow[q] & 0xffff0000u) : 0.f;
    }
    rs[q] += g2;
    rq[q] += g2 * (y2 - mu[q]);
  }
}

template <int BM, int BN, int WM, int WN, bool MF32, int PASSES = 1, bool RED = false>
__device__ __forceinline__ void mfma_tile_epilogue(mfma_acc_t<MF32> (&acc)[BM / WM / (MF32 ? 32 : 16)][BN / WN / (MF32 ? 32 : 16)],
                                                   unsigned char* smem, long long m0, int n0,
                                                   int stat_row, float* stats, const ConvGeom& g,
                                                   bf16_t* Y, const bf16_t* ADD,
                                                   const BnBwdRed& red = BnBwdRed{}) {
  float* fstats = stats;  // Σy, Σy² of the fp32 tile
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = MF32 ? 32 : 16;
  constexpr int RM = TM / FM, RN = TN / FM;
  constexpr int NR = MF32 ? 16 : 4;
  constexpr int NT = WM * WN * 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  auto frow = [&](int r) { return MF32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : (lane >> 4) * 4 + r; };
  const int fcol = MF32 ? (lane & 31) : (lane & 15);
  float* sred = reinterpret_cast<float*>(smem);
  if (fstats) {
#pragma unroll
    for (int j = 0; j < RN; ++j) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const float v = acc[i][j][r];
          sm += v;
          q += v * v;
        }
      if (!MF32) {
        sm += __shfl_xor(sm, 16, 64);
        q += __shfl_xor(q, 16, 64);
      }
      sm += __shfl_xor(sm, 32, 64);
      q += __shfl_xor(q, 32, 64);
      if (lane < FM) {
        const int c = wn * TN + j * FM + lane;
        sred[(wm * BN + c) * 2 + 0] = sm;
        sred[(wm * BN + c) * 2 + 1] = q;
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        sm += sred[(w * BN + c) * 2 + 0];
        q += sred[(w * BN + c) * 2 + 1];
      }
      if (n0 + c < g.Ncols) {
        fstats[((long long)stat_row * 2 + 0) * g.Ncols + n0 + c] = sm;
        fstats[((long long)stat_row * 2 + 1) * g.Ncols + n0 + c] = q;
      }
    }
    __syncthreads();
  }
  constexpr int LDC = BN + 4;
  constexpr int RPB = BM / PASSES;  // rows per band
  static_assert(RPB % TM == 0, "a band holds whole wave rows");
  float* cs = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / 8;
  static_assert(NT % CPR == 0, "a thread keeps one 8-column group across rows");
  constexpr int ITERS = RPB * CPR / NT;
  static_assert(ITERS * NT == RPB * CPR, "rows per band divisible by the block");
  const int cc = tid % CPR;
  const int col = n0 + cc * 8;
  // output offset of row `row` of band pb (and whether it is a real output)
  auto row_off = [&](int pb, int row, long long& o, bool& ok) {
    const long long m = m0 + pb * RPB + row;
    ok = m < g.M && col < g.Ncols;
    const long long mm = ok ? m : m0;
    const unsigned t = fdiv((unsigned)mm, g.wg_mul, g.wg_shr);
    const int x = (int)((unsigned)mm - t * (unsigned)g.Wg);
    const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
    const int y = (int)(t - n * (unsigned)g.Hg);
    o = (((long long)n * g.OH + (y * g.osy + g.oy0)) * g.OW + (x * g.osx + g.ox0)) * g.OC + col;
  };
  auto stage_band = [&](int pb) {
    if (PASSES > 1) __syncthreads();  // previous band's LDS reads done
    if (wm * TM >= pb * RPB && wm * TM < (pb + 1) * RPB) {
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
#pragma unroll
          for (int r = 0; r < NR; ++r)
            cs[(wm * TM - pb * RPB + i * FM + frow(r)) * LDC + wn * TN + j * FM + fcol] = acc[i][j][r];
    }
    __syncthreads();
  };
  auto tile_vals = [&](int row, const uint4& a, unsigned mb, float (&v)[8]) {
    const float4 v0 = *reinterpret_cast<const float4*>(cs + row * LDC + cc * 8);
    const float4 v1 = *reinterpret_cast<const float4*>(cs + row * LDC + cc * 8 + 4);
    v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
    v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    if (ADD) {
      const uint32_t aw[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[2 * q] += ((mb >> (2 * q)) & 1u) ? bf2f((bf16_t)(aw[q] & 0xffff)) : 0.f;
        v[2 * q + 1] += ((mb >> (2 * q + 1)) & 1u) ? bf2f((bf16_t)(aw[q] >> 16)) : 0.f;
      }
    }
  };
  {
    // store phase: the ADD loads of ALL bands are issued before the first accumulator
    // goes to LDS, so their latency overlaps the staging instead of being exposed per row
    // group (the main loop's staging registers are dead here: no rise in the kernel's peak)
    constexpr int NLD = PASSES * ITERS;
    long long o[NLD];
    bool ok[NLD];
    uint4 av[NLD];
    unsigned mb[NLD];
    uint4 yv[RED ? NLD : 1];
    unsigned ym[RED ? NLD : 1];
#pragma unroll
    for (int k = 0; k < NLD; ++k) {
      row_off(k / ITERS, (tid + (k % ITERS) * NT) / CPR, o[k], ok[k]);
      av[k] = make_uint4(0, 0, 0, 0);
      mb[k] = 0xffu;
      if (ADD && ok[k]) {
        av[k] = *reinterpret_cast<const uint4*>(ADD + o[k]);
        if (g.addm) mb[k] = g.addm[o[k] >> 3];
      }
      if constexpr (RED) {
        yv[k] = make_uint4(0, 0, 0, 0);
        ym[k] = 0u;
        if (ok[k]) {
          yv[k] = *reinterpret_cast<const uint4*>(red.y + o[k]);
          if (red.mask) ym[k] = red.mask[o[k] >> 3];
        }
      }
    }
    // RED: this thread's 8 channels are fixed (col); Σdz, Σdz (y - mu) accumulate in registers
    // as channel pairs (packed fp32 FMA/add: half the VALU issues of the scalar form)
    float rs[8], rq[8];
    red_f2 rs2[4], rq2[4], rsc[4], rsh[4], rmu[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) rs2[q] = rq2[q] = red_f2{0.f, 0.f};
    if constexpr (RED) {
      // this thread's 8 consecutive channels' constants as 16-byte loads (24 dword loads
      // per tile before; Ncols % 8 == 0, a column group past the edge reads channel 0's)
      const int cb = col + 8 <= g.Ncols ? col : 0;
      auto ld8 = [&](const float* p, red_f2 (&v)[4]) __attribute__((always_inline)) {
        if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {  // (tensor views at any offset)
          const float4 a = *reinterpret_cast<const float4*>(p + cb);
          const float4 b = *reinterpret_cast<const float4*>(p + cb + 4);
          v[0] = red_f2{a.x, a.y}; v[1] = red_f2{a.z, a.w};
          v[2] = red_f2{b.x, b.y}; v[3] = red_f2{b.z, b.w};
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = red_f2{p[cb + 2 * q], p[cb + 2 * q + 1]};
        }
      };
      ld8(red.mu, rmu);
      if (red.mask) {
#pragma unroll
        for (int q = 0; q < 4; ++q) rsc[q] = rsh[q] = red_f2{0.f, 0.f};
      } else {
        ld8(red.sc, rsc);
        ld8(red.sh, rsh);
      }
    }
#pragma unroll
    for (int pb = 0; pb < PASSES; ++pb) {
      stage_band(pb);
#pragma unroll
      for (int i = 0; i < ITERS; ++i) {
        const int k = pb * ITERS + i;
        if (!ok[k]) continue;
        float v[8];
        tile_vals((tid + i * NT) / CPR, av[k], mb[k], v);
        const uint32_t ow[4] = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                                pack_bf2(v[6], v[7])};
        {  // non-temporal store (profiles/conv_nt_stores_ab_r4ab.txt)
          typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
          u32x4_nt v;
          v.x = ow[0]; v.y = ow[1]; v.z = ow[2]; v.w = ow[3];
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4_nt*>(Y + o[k]));
        }
        if constexpr (RED) {
          const uint4 ov = make_uint4(ow[0], ow[1], ow[2], ow[3]);
          if constexpr (BM * BN >= 128 * 64) {
            if (red.mask) red_acc8<true>(ov, yv[k], ym[k], rs2, rq2, rsc, rsh, rmu);
            else red_acc8<false>(ov, yv[k], ym[k], rs2, rq2, rsc, rsh, rmu);
          } else {  // 64x64 tiles: the pair alignment would cost an occupancy step (78 -> 82 VGPRs)
            const uint32_t yw[4] = {yv[k].x, yv[k].y, yv[k].z, yv[k].w};
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int q = j >> 1;
              const float yj = __uint_as_float((j & 1) ? (yw[q] & 0xffff0000u) : (yw[q] << 16));
              const float gj = __uint_as_float((j & 1) ? (ow[q] & 0xffff0000u) : (ow[q] << 16));
              const bool pass = red.mask ? ((ym[k] >> j) & 1u) != 0u
                                         : yj * rsc[q][j & 1] + rsh[q][j & 1] > 0.f;
              const float dz = pass ? gj : 0.f;
              rs2[q][j & 1] += dz;
              rq2[q][j & 1] += dz * (yj - rmu[q][j & 1]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      rs[2 * q] = rs2[q].x; rs[2 * q + 1] = rs2[q].y;
      rq[2 * q] = rq2[q].x; rq[2 * q + 1] = rq2[q].y;
    }
    if constexpr (RED) {
      // threads of one channel group (tid % CPR) add up: with CPR 8 the two lanes of a
      // 16-lane row by a DPP rotate (row_ror:8 == lane ^ 8; the bpermute shuffles cost 3 VALU
      // + 1 LDS op each), then every row's partials in LDS
      static_assert(CPR == 8 || CPR == 16, "RED epilogue: 64- or 128-column tiles");
      if constexpr (CPR == 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          rs[j] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(rs[j]), 0x128, 0xf, 0xf, false));
          rq[j] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(rq[j]), 0x128, 0xf, 0xf, false));
        }
      }
      constexpr int NRW = NT / 16;  // 16-lane rows of the block
      __syncthreads();  // staging reads done: the LDS is reused below
      float2* rr2 = reinterpret_cast<float2*>(smem);  // [NRW][BN]
      if ((lane & 15) < CPR)
#pragma unroll
        for (int j = 0; j < 8; ++j) rr2[(tid >> 4) * BN + cc * 8 + j] = make_float2(rs[j], rq[j]);
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        if (n0 + c < g.Ncols) {
          float a = 0.f, b = 0.f;
#pragma unroll
          for (int w = 0; w < NRW; ++w) {
            const float2 v = rr2[w * BN + c];
            a += v.x;
            b += v.y;
          }
          red.part[((long long)stat_row * 2 + 0) * g.Ncols + n0 + c] = a;
          red.part[((long long)stat_row * 2 + 1) * g.Ncols + n0 + c] = b * red.is[n0 + c];
        }
      }
    }
  }
}


}  // namespace dm
