// Shared device helpers of the implicit-GEMM conv kernels (conv_igemm.hip, conv_halo.hip).
#pragma once
#include "common.h"
#include "conv_geom.h"

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

template <bool MF32>
using mfma_acc_t = typename std::conditional<MF32, f32x16, f32x4>::type;

// Epilogue of a BM x BN MFMA tile held by WM x WN waves (each TM x TN as FM x FM blocks).
// C/D maps: 16x16 col = l&15, row = (l>>4)*4 + r;  32x32 col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).
//  * optional BN statistics: per-column Σy, Σy² of the fp32 tile -> stats[stat_row][2][Ncols]
//  * fp32 tile staged through LDS (row pitch BN+4) -> coalesced 16-B bf16 stores at the
//    output pixel (y*osy+oy0, x*osx+ox0), optionally adding ADD (which may alias Y).
// Rows >= g.M must hold zeros when stats are requested.  Requires (BM/PASSES)*(BN+4)*4 B of
// LDS: with PASSES > 1 the tile is staged one band of BM/PASSES rows (whole wave rows) at a time.
template <int BM, int BN, int WM, int WN, bool MF32, int PASSES = 1>
__device__ __forceinline__ void mfma_tile_epilogue(mfma_acc_t<MF32> (&acc)[BM / WM / (MF32 ? 32 : 16)][BN / WN / (MF32 ? 32 : 16)],
                                                   unsigned char* smem, long long m0, int n0,
                                                   int stat_row, float* stats, const ConvGeom& g,
                                                   bf16_t* Y, const bf16_t* ADD) {
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = MF32 ? 32 : 16;
  constexpr int RM = TM / FM, RN = TN / FM;
  constexpr int NR = MF32 ? 16 : 4;
  constexpr int NT = WM * WN * 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  auto frow = [&](int r) { return MF32 ? (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5) : (lane >> 4) * 4 + r; };
  const int fcol = MF32 ? (lane & 31) : (lane & 15);
  float* red = reinterpret_cast<float*>(smem);
  if (stats) {
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
        red[(wm * BN + c) * 2 + 0] = sm;
        red[(wm * BN + c) * 2 + 1] = q;
      }
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float sm = 0.f, q = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        sm += red[(w * BN + c) * 2 + 0];
        q += red[(w * BN + c) * 2 + 1];
      }
      if (n0 + c < g.Ncols) {
        stats[((long long)stat_row * 2 + 0) * g.Ncols + n0 + c] = sm;
        stats[((long long)stat_row * 2 + 1) * g.Ncols + n0 + c] = q;
      }
    }
    __syncthreads();
  }
  constexpr int LDC = BN + 4;
  constexpr int RPB = BM / PASSES;  // rows per band
  static_assert(RPB % TM == 0, "a band holds whole wave rows");
  float* cs = reinterpret_cast<float*>(smem);
  constexpr int CPR = BN / 8;
#pragma unroll
  for (int pb = 0; pb < PASSES; ++pb) {
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
    for (int e = tid; e < RPB * CPR; e += NT) {
      const int row = e / CPR, cc = e % CPR;
      const long long m = m0 + pb * RPB + row;
      const int col = n0 + cc * 8;
      if (m >= g.M || col >= g.Ncols) continue;
      const unsigned t = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      const int x = (int)((unsigned)m - t * (unsigned)g.Wg);
      const unsigned n = fdiv(t, g.hg_mul, g.hg_shr);
      const int y = (int)(t - n * (unsigned)g.Hg);
      const long long o =
          (((long long)n * g.OH + (y * g.osy + g.oy0)) * g.OW + (x * g.osx + g.ox0)) * g.OC + col;
      const float4 v0 = *reinterpret_cast<const float4*>(cs + row * LDC + cc * 8);
      const float4 v1 = *reinterpret_cast<const float4*>(cs + row * LDC + cc * 8 + 4);
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
}


}  // namespace dm
