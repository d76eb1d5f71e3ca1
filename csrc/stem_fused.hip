// ResNet stem, fused: 7x7/s2/p3 conv (3 -> 64) + BatchNorm statistics + 3x3/s2/p1 max-pool,
// with the raw dataset gather/normalisation folded into the kernel and a K-dense GEMM layout.
//
// Reference: the stem is not in the reference (SURVEY §2.5 "Extensions required by
// BASELINE.json": ResNet-18-shaped CNN); it replaces cuDNN conv + BN + ReLU + max-pool.
//
// Forward (stem_fwd_kernel), one persistent 768-thread workgroup per CU walking whole images,
// one conv-row PAIR (2i, 2i+1) per step, warp-specialised: 4 MFMA waves, 8 VALU waves (raw
// staging, E expansion, pooling), the two kinds a step apart on double-buffered tiles:
//
//  * K-dense operand.  Input row iy is expanded once in LDS into E[iy][ox][24]: the 7 x 3
//    (kx, c) taps of output column ox (21 values + 3 zero pad, 48 B).  The A fragment of
//    output pixel (oy, ox) at kernel row ky is E[2oy-3+ky][ox][...]: K = 7 x 24 = 168 -> 11
//    k-steps of v_mfma_f32_32x32x16_bf16 (147 real taps: 84 % of the MFMA lanes; the s2d
//    4x4 layout of conv_stem.hip used 256, 57 %).  E rows live in a 13-row ring; a pair
//    needs 9 of them and stages 4 new ones.
//  * Raw input.  Rows are read straight from the dataset through the batch's row index (the
//    loader's gather), u8 / fp32 / bf16 channels-last, normalised per channel, converted to
//    bf16 (S buffer, then the E expansion): no packed copy of the batch exists.
//  * Pool in the epilogue.  BN is a per-channel affine with scale gamma * invstd, whose sign
//    is the sign of gamma, known before the batch statistics: max-pool(relu(s*y + t)) =
//    relu(s * ext(y) + t) with ext = max for s >= 0, min for s < 0.  The kernel writes the
//    pooled extremum of the RAW conv output and its 4-bit window code (the tie-break rank
//    (2-kh) << 2 | (2-kw) of an integer max: the first extremum in PyTorch's scan order); the
//    full-resolution conv output (1.6 GB at batch 1024) never reaches memory.  A small pass
//    then applies BN + ReLU to the pooled tensor and masks the codes of zero outputs (15).
//  * BN statistics (sum, sum of squares) from the fp32 accumulators, one row per workgroup.
//
// Backward (stem_bwd_kernel), same walk, 16 waves: with the BN backward dy = a*dz + b*y + cc
// (dz: the pooled gradient routed to its window's selected pixel),
//     dW = a * dz^T X + b * W (X^T X) + cc * colsum(X)
// (X: the im2col rows).  8 VALU waves route pair i's pooled gradient into a bf16 dz tile (a
// 2x2 quad of conv pixels shares its 4 windows: 9 code tests per channel) and stage the raw
// rows; 8 MFMA waves accumulate pair i-1's D = dz^T X and G = X^T X tiles in fp32 and expand
// the E rows.  y never exists in the backward, and the mean-subtraction terms b*W G and
// cc*colsum cancel in fp32 in stem_wcombine_kernel (colsum(X) is row 93 of G: E element 21
// of every in-image row is 1.0, a zero-weight column).  Rejected on the way (docs/KERNELS.md
// "Round 5"): (a dz + cc) x_col with cc rounded to bf16 per element (7-90 % gradient error),
// and recomputing y for an in-place dy tile (slower: a conflicted read-modify-write epilogue).
// stem_slab_reduce_kernel + stem_wcombine_kernel sum the per-workgroup slabs in fixed order
// and form the OIHW gradient.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {

constexpr int SCO = 64;     // output channels
constexpr int SKP = 176;    // packed weight row: 7 ky x 24 + 8 pad
constexpr int SKH = 192;    // H / D' columns per slab row (6 k-blocks of 32)
constexpr int RING = 13;    // E-row ring

typedef short s4v __attribute__((ext_vector_type(4)));
typedef unsigned int nt4 __attribute__((ext_vector_type(4)));
typedef unsigned int nt2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s4v tr4(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)p);
}

struct StemGeo {
  int Hin, Win, Hout, Wout, PH, PW;
  int ROWB;   // E row bytes = Wout * 48
  int SP;     // S row pitch (elements) = 3 * Win + 24
};

struct RawUnit {
  uint4 w;  // the raw bits of 4 consecutive row elements (u8: .x, bf16: .x .y, fp32: all)
};

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not its
// global loads (__syncthreads' fence drains vmcnt too, which would expose the raw-row and
// pooled-row prefetches -- issued a step ahead -- at every step boundary).
// s_memtime stamp (timing experiments: DMLAB_STEM_TRACE); one asm statement with its wait
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// E-ring row of input row iy (iy >= -5)
__device__ __forceinline__ int ring_of(int iy) { return (iy + 13 * 8) % RING; }

// Division-free staging maps, computed once per thread (the loops then only add offsets).
// Raw rows: a group of NT threads loads up to 4 rows = 3W units of 4 elements; thread t owns
// units t, t + NT, ... (at most RU of them).  E rows: thread t < 3 Wout owns chunk (ox, part)
// = (t / 3, t % 3) of every row it builds.
template <int NT, int RU>
struct RawMap {
  int r[RU], k[RU];  // row within the staging, unit within the row (r = -1: none)
  unsigned valid;    // bit u: unit u of the last load lies inside the image
  float sc[RU][4], bi[RU][4];  // normalisation of the unit's 4 elements (channel (k + j) % 3)
  __device__ __forceinline__ void init(int t, int Win, const float (&nsc)[3], const float (&nbi)[3]) {
    const int upr = 3 * Win / 4;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int e = t + NT * u;
      r[u] = e < 4 * upr ? e / upr : -1;
      k[u] = e - (e / upr) * upr;
      // register selects of the (scalar) kernel arguments: no memory reads, so no vmcnt
      // wait on the in-flight prefetches where the values are used
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = (k[u] + j) % 3;
        sc[u][j] = c == 0 ? nsc[0] : c == 1 ? nsc[1] : nsc[2];
        bi[u][j] = c == 0 ? nbi[0] : c == 1 ? nbi[1] : nbi[2];
      }
    }
  }
  // issue the loads only: the conversion waits for them in store(), a step later.  Every
  // lane loads (out-of-range units read a clamped in-image address and are zeroed in store()):
  // a conditionally loaded register would be merged with a copy at the branch join, and that
  // copy waits for the load on the spot.
  template <int DT>
  __device__ __forceinline__ void load(RawUnit (&ru)[RU], const void* img, long long rowbase, int Hin,
                                       int Win, int iy0, int nrows) {
    valid = 0;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int iy = iy0 + r[u];
      const bool ok = r[u] >= 0 && r[u] < nrows && iy >= 0 && iy < Hin;
      valid |= ok ? 1u << u : 0u;
      const int iyc = min(max(iy, 0), Hin - 1);
      const long long off = rowbase + (long long)iyc * Win * 3 + 4LL * (r[u] >= 0 ? k[u] : 0);
      if (DT == 0) {
        ru[u].w = *reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(img) + off);
      } else if (DT == 1) {
        const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(img) + off);
        ru[u].w = make_uint4(w.x, w.y, 0, 0);
      } else {
        ru[u].w = make_uint4(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(img) + off), 0, 0, 0);
      }
    }
  }
  // normalise (x = raw * nsc[c] + nbi[c]; rows outside the image stay 0), round to bf16, write
  // S[row r][t], t = f + 9 (9 zero pad elements on the left, >= 15 on the right)
  template <int DT>
  __device__ __forceinline__ void store(const RawUnit (&ru)[RU], bf16_t* S, int SP, int nrows) const {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (r[u] < 0 || r[u] >= nrows) continue;
      float x[4];
      const uint4 w = ru[u].w;
      if (DT == 0) {
        x[0] = __uint_as_float(w.x); x[1] = __uint_as_float(w.y);
        x[2] = __uint_as_float(w.z); x[3] = __uint_as_float(w.w);
      } else if (DT == 1) {
        x[0] = __uint_as_float(w.x << 16); x[1] = __uint_as_float(w.x & 0xffff0000u);
        x[2] = __uint_as_float(w.y << 16); x[3] = __uint_as_float(w.y & 0xffff0000u);
      } else {
        x[0] = (float)(w.x & 0xff); x[1] = (float)((w.x >> 8) & 0xff);
        x[2] = (float)((w.x >> 16) & 0xff); x[3] = (float)(w.x >> 24);
      }
      const bool ok = (valid >> u) & 1;
#pragma unroll
      for (int j = 0; j < 4; ++j) x[j] = ok ? fmaf(x[j], sc[u][j], bi[u][j]) : 0.f;
      bf16_t* p = S + r[u] * SP + 4 * k[u] + 9;  // odd element index
      p[0] = f2bf(x[0]);
      *reinterpret_cast<uint32_t*>(p + 1) = pack_bf2(x[1], x[2]);
      p[3] = f2bf(x[3]);
    }
  }
};

struct EMap {
  bool act;
  int soff, eoff;  // S element offset 6 ox + 8 part, E byte offset 48 ox + 16 part
  int part;
  __device__ __forceinline__ void init(int t, int Wout) {
    act = t < 3 * Wout;
    const int ox = t / 3;
    part = t - 3 * ox;
    soff = 6 * ox + 8 * part;
    eoff = 48 * ox + 16 * part;
  }
  // E rows iy0 .. iy0 + nrows - 1; S row of iy is srow0 + (iy - iy0) (rows outside [0, Hin):
  // zeros, no S read)
  // (all the rows' S reads are issued before the first E write: one LDS round trip, not nrows)
  __device__ __forceinline__ void build(unsigned char* E, const bf16_t* S, const StemGeo& G, int iy0,
                                        int nrows, int srow0) const {
    if (!act) return;
    if (nrows == 4) build_n<4>(E, S, G, iy0, srow0);
    else if (nrows == 2) build_n<2>(E, S, G, iy0, srow0);
    else for (int q = 0; q < nrows; ++q) build_n<1>(E, S, G, iy0 + q, srow0 + q);
  }
  template <int NR>
  __device__ __forceinline__ void build_n(unsigned char* E, const bf16_t* S, const StemGeo& G,
                                          int iy0, int srow0) const {
    uint32_t w[NR][4];
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      // rows outside the image read a clamped in-buffer row (zeroed below: no branch joins)
      const int sr = min(max(srow0 + q, 0), 3);
      const uint32_t* sp = reinterpret_cast<const uint32_t*>(S + sr * G.SP + soff);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[q][j] = sp[j];
    }
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int iy = iy0 + q;
      const bool in = iy >= 0 && iy < G.Hin;
      uint4 v = make_uint4(in ? w[q][0] : 0u, in ? w[q][1] : 0u, in ? w[q][2] : 0u, in ? w[q][3] : 0u);
      if (part == 2) {  // elements 21..23 of the expanded row: 1.0 (the backward's all-ones
        v.z = in ? (v.z & 0xffffu) | 0x3f800000u : 0u;  // X column, zero weight), 0, 0
        v.w = 0;
      }
      *reinterpret_cast<uint4*>(E + ring_of(iy) * G.ROWB + eoff) = v;
    }
  }
};

// Window code of pooling-window position (kh, kw): (2 - kh) << 2 | (2 - kw), the tie-break
// rank of the forward's integer max (largest rank = first in PyTorch's scan order); 15 =
// no gradient (the BN+ReLU output is 0).  Channel 2k in the low nibble of byte k.
__host__ __device__ constexpr unsigned wcode(int kh, int kw) { return (unsigned)((2 - kh) << 2 | (2 - kw)); }

// monotone 16-bit key of a bf16 bit pattern (signed int16 order = float order); involution
__device__ __forceinline__ uint32_t mono2(uint32_t w) {  // two packed bf16 -> two keys
  const uint32_t s = (w >> 15) & 0x00010001u;
  return w ^ (s * 0x7fffu);
}

// Y-tile chunk swizzle: [2 slots][Wout px][8 chunks of 8 channels], chunk ^ f(px) with
// f = ((px >> 1) & 1) << 2 | ((px >> 2) & 3): the 4-row x 32-channel transposed reads of the
// wgrad MFMAs stay conflict-free (bit 2 alternates over same-parity rows) and the 32-pixel
// column accesses of the MFMA epilogues spread over all 8 chunk positions (2-way, the
// minimum for 8-byte lanes; bit 2 alone left them 8-way)
__device__ __forceinline__ int yoff(int slot, int px, int c8, int Wout) {
  return ((slot * Wout + px) * 8 + (c8 ^ ((((px >> 1) & 1) << 2) | ((px >> 2) & 3)))) * 16;
}

// One 32-channel x 32-pixel conv tile: acc = W (registers, 11 k-steps of 16) x E^T, the E
// fragment of k-step s at byte rowoff[ky] + 16 part + pxoff with (ky, part) = divmod(2s + hh, 3)
// (ky clamped to 6: k-step 10's upper half has zero weights).  rowoff is wave-uniform, so a
// k-step's address is one select between two scalar sums; the reads run PF k-steps ahead of
// the MFMAs.
template <int PF>
__device__ __forceinline__ f32x16 conv_tile(const bf16x8 (&wa)[11], const unsigned char* E,
                                            const int (&rowoff)[7], int pxoff, bool hh) {
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  bf16x8 bq[11];
#pragma unroll
  for (int s = 0; s < 11 + PF; ++s) {
    if (s < 11) {
      const int j0 = 2 * s, j1 = 2 * s + 1;
      const int k0 = j0 / 3 > 6 ? 6 : j0 / 3, k1 = j1 / 3 > 6 ? 6 : j1 / 3;
      const int a0 = rowoff[k0] + 16 * (j0 % 3), a1 = rowoff[k1] + 16 * (j1 % 3);
      bq[s] = *reinterpret_cast<const bf16x8*>(E + (hh ? a1 : a0) + pxoff);
    }
    if (s >= PF) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s - PF], bq[s - PF], acc, 0, 0, 0);
  }
  return acc;
}

// byte offsets of the ring rows of input rows iy0 + r, r = 0..6 (iy0 >= -5)
__device__ __forceinline__ void ring_rows(int (&ro)[7], int iy0, int ROWB) {
  const int r0 = ring_of(iy0);
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int x = r0 + r;
    ro[r] = (x >= RING ? x - RING : x) * ROWB;
  }
}

// The wgrad MFMAs of one conv-row pair: acc[kb] (32 co x 32 k, 3 k-blocks) += T[slot][m][co]^T *
// E[m][k] over both slots' Wout pixels.  Wave w (0..3): co-block w & 1, k-blocks
// 3*((w >> 1) & 1) + 0..2.  T is the bf16 dy tile, E the ring rows of the pair.  The 8
// transposed reads of each (t, slot) stage are issued one stage ahead of its 3 MFMAs.
__device__ __forceinline__ void pair_wgrad(f32x16 (&acc)[3], const unsigned char* T,
                                           const unsigned char* E, const StemGeo& G, int i,
                                           int wid, int lane) {
  const int cb = wid & 1, kq = (wid >> 1) & 1;
  const int g = lane >> 4, h = g >> 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  // A: rows m = 16t + 4h + q (+8), channels co = 32cb + 16(g&1) + 4p .. +3
  const int c8 = 4 * cb + 2 * (g & 1) + (p >> 1);
  // rows m and m + 8 (the swizzle is invariant under m + 16, not m + 8)
  int ta[2], ta8[2], boff[2][3];
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    ta[sl] = yoff(sl, 4 * h + q, c8, G.Wout) + 8 * (p & 1);
    ta8[sl] = yoff(sl, 4 * h + q + 8, c8, G.Wout) + 8 * (p & 1);
    const int oy = 2 * i + sl;
    // B: rows m (same), columns k = 32kb + 16(g&1) + 4p .. +3
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int k = 32 * (3 * kq + u) + 16 * (g & 1) + 4 * p;
      int ky = k / 24, kk = k - 24 * ky;
      if (ky > 6) ky = 6;  // the pad columns k >= 168 read finite data (their results are unused)
      boff[sl][u] = ring_of(2 * oy - 3 + ky) * G.ROWB + (4 * h + q) * 48 + 2 * kk;
    }
  }
  struct Stage {
    s4v a0, a1, b0[3], b1[3];
  };
  auto load = [&](Stage& S, int t, int sl) {
    const int mo = 16 * t;
    S.a0 = tr4(T + ta[sl] + mo * 128);
    S.a1 = tr4(T + ta8[sl] + mo * 128);
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      S.b0[u] = tr4(E + boff[sl][u] + mo * 48);
      S.b1[u] = tr4(E + boff[sl][u] + (mo + 8) * 48);
    }
  };
  auto mma = [&](const Stage& S) {
    const bf16x8 af = (bf16x8){S.a0[0], S.a0[1], S.a0[2], S.a0[3], S.a1[0], S.a1[1], S.a1[2], S.a1[3]};
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const bf16x8 bf = (bf16x8){S.b0[u][0], S.b0[u][1], S.b0[u][2], S.b0[u][3],
                                 S.b1[u][0], S.b1[u][1], S.b1[u][2], S.b1[u][3]};
      acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[u], 0, 0, 0);
    }
  };
  const int nt = G.Wout >> 4;
  Stage s0, s1;
  load(s0, 0, 0);
  for (int t = 0; t < nt; ++t) {
    load(s1, t, 1);
    mma(s0);
    if (t + 1 < nt) load(s0, t + 1, 0);
    mma(s1);
  }
}

}  // namespace

struct StemFwdArgs {
  const void* img;
  const long long* idx;  // batch row -> dataset row (nullptr: identity)
  float nsc[3], nbi[3];  // x = raw * nsc[c] + nbi[c]
  const bf16_t* wk;      // [64][SKP]
  const float* gamma;    // BN weight: sign picks max / min pooling
  bf16_t* pext;          // [N][PH][PW][64]
  uint8_t* code;         // [N][PH][PW][32]: window codes, 4 bits per channel (see wcode)
  float* stats;          // [grid][2][64] or nullptr
  int N, nimg;           // batch rows, image rows (idx values are clamped to it)
  int ablate;            // timing experiments only (DMLAB_STEM_ABLATE): skip parts of the work
  StemGeo G;
};

// Warp-specialised forward: 4 MFMA waves compute pair i's conv into key tile Y[i & 1] while
// 8 VALU waves pool pair i-1 from the other tile, expand the E rows pair i+1 needs and load
// the raw rows of the step after; one barrier per step.  Per image the step stream is
// [stage rows -3..3, stage rows 4..5, pair 0, ..., pair PH-1]; the last pair is pooled in the
// next image's first step.  The tile holds monotone 16-bit keys of the bf16 conv output
// (complemented where gamma < 0), so the pooled extremum and its first-in-scan-order window
// position fall out of 32-bit integer max3s of (key << 16 | rank).
constexpr int FNT = 768;                 // 12 waves: 0-3 MFMA, 4-11 VALU
constexpr int FVT = FNT - 256;           // VALU threads
constexpr int FRU = 2;                   // raw units per VALU thread per staging (4 rows)

template <int DT>
__global__ void __launch_bounds__(FNT, 1) stem_fwd_kernel(StemFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StemGeo G = a.G;
  const int YB = 2 * G.Wout * 128;       // one key tile: [2 slots][Wout][64]
  const int SB = 4 * G.SP;               // one S buffer (elements)
  unsigned char* E = smem;                                   // [RING][Wout][24] bf16
  unsigned char* Y = E + RING * G.ROWB;                      // [2][YB]
  bf16_t* S = reinterpret_cast<bf16_t*>(Y + 2 * YB);         // [2][4][SP]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool train = a.stats != nullptr;
  {
    const int tot16 = (RING * G.ROWB + 2 * YB + 2 * SB * 2) / 16;
    for (int e = tid; e < tot16; e += FNT) reinterpret_cast<uint4*>(smem)[e] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  const int nimg = a.N > (int)blockIdx.x ? (a.N - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int SPI = G.PH + 2;              // steps per image
  const int nsteps = nimg * SPI;         // + 1 final pooling-only step
  auto img_base = [&](int q) -> long long {
    const int n = (int)blockIdx.x + q * (int)gridDim.x;
    long long row = a.idx ? a.idx[n] : (long long)n;
    row = row < 0 ? 0 : row >= a.nimg ? a.nimg - 1 : row;
    return row * G.Hin * G.Win * 3;
  };
  const bool mw = wid < 4;
  if (mw) {
    // ================================================================ MFMA waves
    // wave w: conv row 2i + (w >> 1) of the pair, output channels 32 (w & 1) .. +31, all
    // pixel blocks.  C = W x E^T: lane = pixel (lane & 31), register r = channel
    // 32cb + (r & 3) + 8 (r >> 2) + 4 hh -- 4 consecutive channels per register quad, one
    // 8-byte key store each.  The weights (A) stay in registers.
    const int slot = wid >> 1, cb = wid & 1, hh = lane >> 5;
    bf16x8 wa[11];
#pragma unroll
    for (int s = 0; s < 11; ++s)
      wa[s] = *reinterpret_cast<const bf16x8*>(a.wk + (32 * cb + (lane & 31)) * SKP + 16 * s + 8 * hh);
    uint32_t flm[4][2];  // complement masks (gamma < 0) of the register quads' channel pairs
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int co = 32 * cb + 8 * g4 + 4 * hh + 2 * h;
        flm[g4][h] = (a.gamma[co] < 0.f ? 0xffffu : 0u) | (a.gamma[co + 1] < 0.f ? 0xffff0000u : 0u);
      }
    float st_s[16], st_q[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) st_s[r] = st_q[r] = 0.f;
    for (int st = 0; st <= nsteps; ++st) {
      lds_barrier();  // step boundary (the previous step's tile reads / E writes are done)
      if (st == nsteps) break;
      const int kk = st % SPI;
      if (kk < 2) continue;
      const int i = kk - 2;
      unsigned char* Yt = Y + (st & 1) * YB;
      int ro[7];
      ring_rows(ro, 4 * i - 3 + 2 * slot, G.ROWB);  // conv row 2i + slot: input rows 2oy-3 ..
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) {
        if (32 * mb >= G.Wout || (a.ablate & 1)) break;
        const int px = 32 * mb + (lane & 31);
        const int pxb = min(px, G.Wout - 1);
        f32x16 acc = conv_tile<4>(wa, E, ro, pxb * 48, hh);
        const bool valid = px < G.Wout;
        if (32 * mb + 32 > G.Wout) {  // partial block: drop the clamped duplicates
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = valid ? acc[r] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          st_s[r] += acc[r];
          st_q[r] = fmaf(acc[r], acc[r], st_q[r]);
        }
        if (valid) {
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const uint32_t k0 = mono2(pack_bf2(acc[4 * g4 + 0], acc[4 * g4 + 1])) ^ flm[g4][0];
            const uint32_t k1 = mono2(pack_bf2(acc[4 * g4 + 2], acc[4 * g4 + 3])) ^ flm[g4][1];
            *reinterpret_cast<uint2*>(Yt + yoff(slot, px, 4 * cb + g4, G.Wout) + 8 * hh) = make_uint2(k0, k1);
          }
        }
      }
    }
    if (!train) return;
    // statistics: [wave][r][lane] partials -> per channel, summed in fixed order
    float* red = reinterpret_cast<float*>(smem);  // 4 waves x 2 x 16 x 64 floats
    __syncthreads();  // the VALU waves' last pooling reads of the tiles are done
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      red[((wid * 2 + 0) * 16 + r) * 64 + lane] = st_s[r];
      red[((wid * 2 + 1) * 16 + r) * 64 + lane] = st_q[r];
    }
    __syncthreads();
    if (tid < 2 * SCO) {
      const int co = tid & 63, which = tid >> 6;
      const int c = co >> 5, cl = co & 31, h = (cl >> 2) & 1, r = (cl & 3) + 4 * (cl >> 3);
      float sum = 0.f;
      for (int sl = 0; sl < 2; ++sl) {
        const float* rp = red + (((2 * sl + c) * 2 + which) * 16 + r) * 64 + 32 * h;
        for (int l = 0; l < 32; ++l) sum += rp[l];
      }
      a.stats[(long long)blockIdx.x * 2 * SCO + which * SCO + co] = sum;
    }
    return;
  }
  // ================================================================== VALU waves
  const int vt = tid - 256;
  RawMap<FVT, FRU> rm;
  rm.init(vt, G.Win, a.nsc, a.nbi);
  EMap em;
  em.init(vt, G.Wout);
  RawUnit ru[FRU];
  // pooling thread (j, c8)
  const bool pact = vt < G.PW * 8;
  const int pj = vt >> 3, pc8 = vt & 7;
  uint32_t pflip[4];  // per channel pair of this chunk: complement masks (gamma < 0)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = pc8 * 8 + 2 * k;
    pflip[k] = (pact && a.gamma[c] < 0.f ? 0xffffu : 0u) |
               (pact && a.gamma[c + 1] < 0.f ? 0xffff0000u : 0u);
  }
  int pv[8];  // previous odd row's horizontal max keys (key << 16 | 2 - kw)
  // raw rows for step 0: image 0 rows 0..3
  // dataset row bases of the current and the next image, read once per image (a per-step
  // index read is a vector load whose wait would drain the in-flight prefetches and stores)
  long long bcur = nimg > 0 ? img_base(0) : 0, bnext = nimg > 1 ? img_base(1) : 0;
  int bq = 0;  // image of bcur
  auto base = [&](int qq) {
    if (qq != bq) {  // advance (images are visited in order)
      bcur = bnext;
      bq = qq;
      bnext = qq + 1 < nimg ? img_base(qq + 1) : 0;
    }
    return bcur;
  };
  // raw rows expanded at step t (stored into S[(t - 1) & 1] at the top of step t - 1, loaded
  // during step t - 2: a whole step in flight)
  auto plan = [&](int t, int& pq, int& piy) -> int {
    if (t >= nsteps) return 0;
    pq = t / SPI;
    const int k = t - pq * SPI;
    if (k == 0) { piy = 0; return 4; }
    if (k == 1) { piy = 4; return 2; }
    if (k - 2 + 1 < G.PH) { piy = 4 * (k - 2) + 6; return 4; }
    return 0;
  };
  int pend = 0;  // rows in flight in ru (for step st + 1)
  if (nimg > 0) {
    rm.load<DT>(ru, a.img, bcur, G.Hin, G.Win, 0, 4);
    rm.store<DT>(ru, S + 1 * SB, G.SP, 4);  // consumed by step 0 from S[(0 - 1) & 1] = S[1]
    int pq = 0, piy = 0;
    pend = plan(1, pq, piy);
    if (pend) rm.load<DT>(ru, a.img, base(pq), G.Hin, G.Win, piy, pend);
  }
  for (int st = 0; st <= nsteps; ++st) {
    lds_barrier();
    const int q = st / SPI, kk = st - q * SPI;
    // (c) the rows of step st + 1 into S, then the loads of step st + 2's
    if (pend) rm.store<DT>(ru, S + (st & 1) * SB, G.SP, pend);
    {
      int pq = 0, piy = 0;
      pend = plan(st + 2, pq, piy);
      if (pend) rm.load<DT>(ru, a.img, base(pq), G.Hin, G.Win, piy, pend);
    }
    // (a) pooling of the pair the MFMA waves computed in the previous step
    if (st >= 1) {
      const int ps = st - 1, pq = ps / SPI, pk = ps - pq * SPI;
      if (pk >= 2 && pact && !(a.ablate & 4)) {
        const int i = pk - 2;
        const unsigned char* Yt = Y + (ps & 1) * YB;
        if (i == 0) {
#pragma unroll
          for (int c = 0; c < 8; ++c) pv[c] = INT_MIN;
        }
        int hk[2][8];
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
          uint4 w[3];
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int px = 2 * pj - 1 + kw;
            w[kw] = (px >= 0 && px < G.Wout) ? *reinterpret_cast<const uint4*>(Yt + yoff(sl, px, pc8, G.Wout))
                                             : make_uint4(0x80008000u, 0x80008000u, 0x80008000u, 0x80008000u);
          }
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const int sh = 16 * (c & 1);
            int k3[3];
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
              const uint32_t ww[4] = {w[kw].x, w[kw].y, w[kw].z, w[kw].w};
              const uint32_t d = ww[c >> 1];
              k3[kw] = (int)((sh ? (d & 0xffff0000u) : (d << 16)) | (uint32_t)(2 - kw));
            }
            hk[sl][c] = max(max(k3[0], k3[1]), k3[2]);
          }
        }
        uint32_t o[4] = {0, 0, 0, 0}, cd = 0;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const int v = max(max(pv[c] | 8, hk[0][c] | 4), hk[1][c]);  // kh rank 2 - kh in bits 2-3
          cd |= ((uint32_t)v & 15u) << (4 * c);  // the rank nibble is the window code
          o[c >> 1] |= ((uint32_t)v >> 16) << (16 * (c & 1));
          pv[c] = hk[1][c];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = mono2(o[k] ^ pflip[k]);  // keys -> bf16 bits
        const int n = (int)blockIdx.x + pq * (int)gridDim.x;
        const long long po = (((long long)n * G.PH + i) * G.PW + pj) * SCO + pc8 * 8;
        __builtin_nontemporal_store((nt4){o[0], o[1], o[2], o[3]}, reinterpret_cast<nt4*>(a.pext + po));
        __builtin_nontemporal_store(cd, reinterpret_cast<uint32_t*>(a.code + po / 2));
      }
    }
    // (b) E rows for the next step's MFMA, from the raw rows staged in the previous step
    if (st < nsteps && !(a.ablate & 8)) {
      const bf16_t* Sp = S + ((st - 1) & 1) * SB;
      if (kk == 0) em.build(E, Sp, G, -3, 7, -3);
      else if (kk == 1) em.build(E, Sp, G, 4, 2, 0);
      else if (kk - 2 + 1 < G.PH) em.build(E, Sp, G, 4 * (kk - 2) + 6, 4, 0);
    }
  }
  if (train) {  // the MFMA waves' statistics exchange (overwrites the tiles)
    __syncthreads();
    __syncthreads();
  }
}

// out = relu(scale * pext + shift); code4 (optional) = the forward's window codes with 15
// where that output is <= 0 (no gradient flows).  Four 8-channel chunks per thread, all loads
// issued first.
__global__ void __launch_bounds__(256) stem_pool_apply_kernel(const bf16_t* __restrict__ pext,
                                                              const uint32_t* __restrict__ code,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              bf16_t* __restrict__ out,
                                                              uint32_t* __restrict__ code4,
                                                              long long n8) {
  constexpr int U = 4;
  const long long b = (long long)blockIdx.x * 256 * U + threadIdx.x;
  nt4 v[U];
  uint32_t cd[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long e = b + 256LL * u;
    if (e < n8) {
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(pext) + e);
      cd[u] = code4 ? __builtin_nontemporal_load(code + e) : 0u;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long e = b + 256LL * u;
    if (e >= n8) continue;
    const int c0 = (int)(e & 7) * 8;
    const uint32_t w[4] = {v[u][0], v[u][1], v[u][2], v[u][3]};
    uint32_t o[4], keep = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float r[2];
#pragma unroll
      for (int hlf = 0; hlf < 2; ++hlf) {
        const int c = c0 + 2 * k + hlf;
        const float z = bf2f((bf16_t)((w[k] >> (16 * hlf)) & 0xffff)) * scale[c] + shift[c];
        r[hlf] = z > 0.f ? z : 0.f;
        keep |= z > 0.f ? 15u << (4 * (2 * k + hlf)) : 0u;
      }
      o[k] = pack_bf2(r[0], r[1]);
    }
    __builtin_nontemporal_store((nt4){o[0], o[1], o[2], o[3]}, reinterpret_cast<nt4*>(out) + e);
    if (code4) code4[e] = (cd[u] & keep) | ~keep;
  }
}

// ------------------------------------------------------------------------------- backward
// ------------------------------------------------------------------ backward MFMA plans
// dW = a*D + b*(W G) + cc*colsum(X), with D = dz^T X (dz: the routed pooled gradient, bf16
// tile T) and G = X^T X (X: the im2col rows of the conv, straight from the E ring), both
// fp32 MFMA accumulations over the workgroup's images.  y = X W^T never exists: b * sum y X
// is W G, exactly, in the combine kernel (the mean-subtraction terms cancel in fp32 there).
// colsum(X) is row 93 of G: E element 21 of every in-image row is 1.0 (X column 3*24 + 21,
// centre kernel row, zero weight).  6 k-blocks of 32: G's 21 upper-triangle tiles and D's
// 12 tiles over 8 MFMA waves; a wave loads the X fragments of its blocks (and the T
// fragment of its co-block) once per 16-row m-step and feeds all its tiles.
constexpr int GK = 192;   // G rows / columns (6 k-blocks)
constexpr int GONE = 93;  // the all-ones X column
struct WavePlan {
  int nb, blk[4];         // X blocks loaded
  int tcb;                // T co-block loaded (-1: none)
  int nt, kind[5], x[5], y[5];  // tiles: kind 0 = G(blk[x], blk[y]), 1 = D(tcb, blk[y])
};
__device__ constexpr WavePlan kPlans[8] = {
    {2, {0, 1, 0, 0}, 0, 5, {0, 0, 0, 1, 1}, {0, 0, 1, 0, 0}, {0, 1, 1, 0, 1}},
    {2, {2, 3, 0, 0}, 0, 5, {0, 0, 0, 1, 1}, {0, 0, 1, 0, 0}, {0, 1, 1, 0, 1}},
    {2, {4, 5, 0, 0}, 0, 5, {0, 0, 0, 1, 1}, {0, 0, 1, 0, 0}, {0, 1, 1, 0, 1}},
    {4, {0, 1, 2, 3}, -1, 4, {0, 0, 0, 0, 0}, {0, 0, 1, 1, 0}, {2, 3, 2, 3, 0}},
    {4, {0, 1, 4, 5}, -1, 4, {0, 0, 0, 0, 0}, {0, 0, 1, 1, 0}, {2, 3, 2, 3, 0}},
    {4, {2, 3, 4, 5}, -1, 4, {0, 0, 0, 0, 0}, {0, 0, 1, 1, 0}, {2, 3, 2, 3, 0}},
    {3, {0, 1, 2, 0}, 1, 3, {1, 1, 1, 0, 0}, {0, 0, 0, 0, 0}, {0, 1, 2, 0, 0}},
    {3, {3, 4, 5, 0}, 1, 3, {1, 1, 1, 0, 0}, {0, 0, 0, 0, 0}, {0, 1, 2, 0, 0}},
};

struct BwdFrags {
  bf16x8 xf[4], tf;
};

// MFMA work of m-steps [t0, t1) of one slot (conv row 2i + slot) of a pair for wave W
template <int W>
__device__ __forceinline__ void gram_slot(f32x16 (&acc)[5], const unsigned char* T,
                                          const unsigned char* E, const StemGeo& G, int i,
                                          int slot, int t0, int t1, int lane) {
  constexpr WavePlan P = kPlans[W];
  const int g = lane >> 4, h = g >> 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int oy = 2 * i + slot;
  int boff[4];
#pragma unroll
  for (int b = 0; b < P.nb; ++b) {
    const int k = 32 * P.blk[b] + 16 * (g & 1) + 4 * p;
    int ky = k / 24;
    const int kk = k - 24 * ky;
    if (ky > 6) ky = 6;  // pad columns k >= 168: finite data, unused results
    boff[b] = ring_of(2 * oy - 3 + ky) * G.ROWB + (4 * h + q) * 48 + 2 * kk;
  }
  int ta = 0, ta8 = 0;
  if (P.tcb >= 0) {
    const int c8 = 4 * P.tcb + 2 * (g & 1) + (p >> 1);
    ta = yoff(slot, 4 * h + q, c8, G.Wout) + 8 * (p & 1);
    ta8 = yoff(slot, 4 * h + q + 8, c8, G.Wout) + 8 * (p & 1);  // swizzle: m + 16 invariant only
  }
  auto load = [&](BwdFrags& F, int t) {
    const int mo = 16 * t;
#pragma unroll
    for (int b = 0; b < P.nb; ++b) {
      const s4v v0 = tr4(E + boff[b] + mo * 48), v1 = tr4(E + boff[b] + (mo + 8) * 48);
      F.xf[b] = (bf16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
    if (P.tcb >= 0) {
      const s4v v0 = tr4(T + ta + mo * 128), v1 = tr4(T + ta8 + mo * 128);
      F.tf = (bf16x8){v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    }
  };
  auto mma = [&](const BwdFrags& F) {
#pragma unroll
    for (int j = 0; j < P.nt; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(P.kind[j] ? F.tf : F.xf[P.x[j]], F.xf[P.y[j]],
                                                       acc[j], 0, 0, 0);
  };
  // (two MFMA waves per SIMD cover each other's fragment-read latency)
  for (int t = t0; t < t1; ++t) {
    BwdFrags f;
    load(f, t);
    mma(f);
  }
}

template <int W>
__device__ __forceinline__ void gram_store(const f32x16 (&acc)[5], float* dslab, float* gslab,
                                           int lane) {
  constexpr WavePlan P = kPlans[W];
#pragma unroll
  for (int j = 0; j < P.nt; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int col = 32 * P.blk[P.y[j]] + (lane & 31);
      if (P.kind[j])
        dslab[(long long)blockIdx.x * SCO * SKH + (32 * P.tcb + row) * SKH + col] = acc[j][r];
      else
        gslab[(long long)blockIdx.x * GK * GK + (32 * P.blk[P.x[j]] + row) * GK + col] = acc[j][r];
    }
}

template <int W>
__device__ __forceinline__ void gram_zero(f32x16 (&acc)[5]) {
#pragma unroll
  for (int j = 0; j < 5; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
}

struct StemBwdArgs2 {
  const void* img;
  const long long* idx;
  float nsc[3], nbi[3];
  const bf16_t* wk;      // [64][SKP] packed weights (the forward's)
  const bf16_t* pdy;     // [N][PH][PW][64] pooled gradient
  const uint8_t* code4;  // [N][PH][PW][32] window positions, 4 bits per channel, 15 = masked
  float* dslab;          // [grid][64][SKH]: D = dz^T X partials
  float* gslab;          // [grid][GK][GK]: G = X^T X partials (upper-triangle tiles)
  int N, nimg;
  int ablate;            // timing experiments only (DMLAB_STEM_ABLATE)
  int split;             // m-steps of a pair's MFMA work before the mid-step barrier
  unsigned long long* trace;  // timing experiments: [step][8] stamps of workgroup 0
  StemGeo G;
};

constexpr int PRING = 3;  // pooled-row ring: rows i, i+1 in use, i+2 staged
constexpr int BNT = 1024;  // 16 waves: 0-7 MFMA, 8-15 VALU
constexpr int BMW = 8;     // MFMA waves
constexpr int BVT = BNT - 64 * BMW;

// Warp-specialised backward.  Step stream per image: [stage raw rows 0..1 + pooled rows 0..2,
// expand E rows -3..1, pair 0, ..., pair PH-1, (drain)]; the VALU waves route pair i's pooled
// gradient into the dz tile T[i & 1] (and stage its E rows) while the MFMA waves accumulate
// pair i-1's D and G tiles (slot 0 before the mid-step barrier, slot 1 after).  The barriers:
// T and E hand-offs (step start) and the VALU waves' S reads before the next raw rows
// overwrite it (mid-step).
template <int DT>
__global__ void __launch_bounds__(BNT, 1) stem_bwd_kernel(StemBwdArgs2 a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StemGeo G = a.G;
  const int TB = 2 * G.Wout * 128;                           // one tile: [2 slots][Wout][64]
  unsigned char* E = smem;                                   // [RING][Wout][24]
  unsigned char* T = E + RING * G.ROWB;                      // [2][TB]
  bf16_t* S = reinterpret_cast<bf16_t*>(T + 2 * TB);         // [4][SP]
  const int PRB = G.PW * SCO;                                // pooled row elements
  bf16_t* Pg = S + 4 * G.SP;                                 // [PRING][PW][64] grads
  uint8_t* Pc = reinterpret_cast<uint8_t*>(Pg + PRING * PRB);  // [PRING][PW][32] 4-bit codes
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  {
    const int tot16 = (RING * G.ROWB + 2 * TB + 4 * G.SP * 2) / 16;
    for (int e = tid; e < tot16; e += BNT) reinterpret_cast<uint4*>(smem)[e] = make_uint4(0, 0, 0, 0);
  }
  const int nimg = a.N > (int)blockIdx.x ? (a.N - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int SPI = G.PH + 2;
  const int nsteps = nimg * SPI;  // + 1 drain step (the last pair's MFMA work)
  auto img_of = [&](int q) { return (int)blockIdx.x + q * (int)gridDim.x; };
  auto img_base = [&](int q) -> long long {
    long long row = a.idx ? a.idx[img_of(q)] : (long long)img_of(q);
    row = row < 0 ? 0 : row >= a.nimg ? a.nimg - 1 : row;
    return row * G.Hin * G.Win * 3;
  };
  if (wid < BMW) {
    // ================================================================ MFMA waves
    f32x16 acc[5];
    gram_zero<0>(acc);
    __syncthreads();  // zeroed LDS
    EMap em;  // the E expansion runs here, after the step's Gram work (the VALU waves are the
    em.init(tid, G.Wout);  // busier side): rows of pair kk-2 from the S rows stored this step
    auto run = [&](auto wtag) {
      constexpr int W = decltype(wtag)::value;
      const bool tr = a.trace && blockIdx.x == 0 && W == 0;
      for (int st = 0; st <= nsteps; ++st) {
        if (tr) a.trace[st * 8 + 4] = stamp();
        lds_barrier();  // step start: T[(st-1) & 1] (dz of the pair) and its E rows are ready
        if (tr) a.trace[st * 8 + 5] = stamp();
        const int ps = st - 1;
        const int pk = ps >= 0 ? ps % SPI : -1;
        const bool work = ps >= 0 && pk >= 2 && !(a.ablate & 1);
        const unsigned char* Tt = T + (ps & 1) * TB;
        // the VALU waves' gather runs before the mid-step barrier, their staging after it:
        // m-steps [0, split) of the 2 * Wout / 16 before, the rest after
        const int nt = G.Wout >> 4, split = min(a.split, 2 * nt);
        if (work) {
          gram_slot<W>(acc, Tt, E, G, pk - 2, 0, 0, min(split, nt), lane);
          if (split > nt) gram_slot<W>(acc, Tt, E, G, pk - 2, 1, 0, split - nt, lane);
        }
        if (tr) a.trace[st * 8 + 6] = stamp();
        lds_barrier();  // mid-step
        if (tr) a.trace[st * 8 + 7] = stamp();
        if (work) {
          if (split < nt) gram_slot<W>(acc, Tt, E, G, pk - 2, 0, split, nt, lane);
          gram_slot<W>(acc, Tt, E, G, pk - 2, 1, max(split - nt, 0), nt, lane);
        }
        // E rows: kk = 1 -> rows -3..1 (S rows 0..1), kk = i + 2 -> rows 4i+2..4i+5 (pair i's
        // new rows; pair i-1's 4i-7..4i+1 are being read: 13 live rows, the ring)
        if (st < nsteps && !(a.ablate & 8)) {
          const int kk = st % SPI;
          if (kk == 1) em.build(E, S, G, -3, 5, -3);
          else if (kk >= 2) em.build(E, S, G, 4 * (kk - 2) + 2, 4, 0);
        }
      }
      gram_store<W>(acc, a.dslab, a.gslab, lane);
    };
    switch (wid) {
      case 0: run(std::integral_constant<int, 0>{}); break;
      case 1: run(std::integral_constant<int, 1>{}); break;
      case 2: run(std::integral_constant<int, 2>{}); break;
      case 3: run(std::integral_constant<int, 3>{}); break;
      case 4: run(std::integral_constant<int, 4>{}); break;
      case 5: run(std::integral_constant<int, 5>{}); break;
      case 6: run(std::integral_constant<int, 6>{}); break;
      default: run(std::integral_constant<int, 7>{}); break;
    }
    return;
  }
  // ================================================================== VALU waves
  // Per image (SPI = PH + 2 steps): kk = 0 stages pooled rows 0..2 (the MFMA waves finish the
  // previous image's last pair); kk = 1 stores raw rows 0..1 (expanded to E rows -3..1 by the
  // MFMA waves after the mid-step barrier); kk = i + 2 stores rows 4i+2..4i+5 (pair i's new
  // rows) and routes pair i's pooled gradient into the dz tile T.  The MFMA waves read pair
  // i-1's rows 4i-7..4i+1 meanwhile: 13 live rows, the ring's size.
  const int vt = tid - 64 * BMW;
  RawMap<BVT, FRU> rm;
  rm.init(vt, G.Win, a.nsc, a.nbi);
  RawUnit ru[FRU];
  // pooled rows: PW * 8 chunks of (8 grads, 8 4-bit codes) per row; thread vt < PW*8 owns one
  const bool pl = vt < G.PW * 8;
  uint4 pg_r;
  uint32_t pc_r;
  bool p_ok = false;
  // branch-free like RawMap::load: clamped addresses, validity applied at the store
  auto pload = [&](int q, int r) {
    p_ok = pl && r < G.PH;
    const int rc = min(r, G.PH - 1), vc = pl ? vt : 0;
    const long long o = (((long long)img_of(min(q, nimg - 1)) * G.PH + rc) * G.PW) * SCO + vc * 8;
    pg_r = *reinterpret_cast<const uint4*>(a.pdy + o);
    pc_r = *reinterpret_cast<const uint32_t*>(a.code4 + o / 2);
  };
  auto pstore = [&](int r) {
    if (!pl) return;
    const int sl = r % PRING;
    *reinterpret_cast<uint4*>(Pg + sl * PRB + vt * 8) = p_ok ? pg_r : make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint32_t*>(Pc + (sl * PRB + vt * 8) / 2) = p_ok ? pc_r : 0xffffffffu;
  };
  const int qb = vt >> 3, qc = vt & 7, c0 = qc * 8;
  __syncthreads();  // zeroed LDS
  // dz of quad pixel pp = (ddy, ddx), channels c0 + 4 hf .. +3: the sum of the grads of the
  // covering windows whose code names this pixel (window (wa, wb) sees it at
  // kh = ddy ? (wa ? 0 : 2) : 1, same for kw).  Half a chunk at a time keeps the live set small.
  // per-thread constants of the gather: the quad's two window columns (clamped; a column past
  // the row is masked by its code) and its 4 pixels' tile offsets
  const bool colok = qb + 1 < G.PW;
  const int ocol0 = qb * SCO + c0, ocol1 = (colok ? qb + 1 : qb) * SCO + c0;
  int toff[4];
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) toff[pp] = yoff(pp >> 1, 2 * qb + (pp & 1), qc, G.Wout);
  uint2 gres[4];  // channels 0..3 of the 4 pixels, held across the mid-step barrier
  auto gquad = [&](uint2 (&res)[4], int i, int hf) {
    uint2 qg[4];     // the quad's windows: 4 pooled grads each
    uint32_t qi[4];  // and their codes (15 everywhere for a window outside the image)
    const int sl0 = i % PRING, sl1 = sl0 + 1 == PRING ? 0 : sl0 + 1;  // rows i, i+1 (uniform)
    const bool rowok = i + 1 < G.PH;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int wa = w >> 1, wb = w & 1;
      const int o = (wa ? sl1 : sl0) * PRB + (wb ? ocol1 : ocol0);
      qg[w] = *reinterpret_cast<const uint2*>(Pg + o + 4 * hf);
      const uint32_t c = *reinterpret_cast<const uint16_t*>(Pc + o / 2 + 2 * hf);
      qi[w] = ((wa && !rowok) || (wb && !colok)) ? 0xffffu : c;
    }
#pragma unroll
    for (int pp = 0; pp < 4; ++pp) {
      const int ddy = pp >> 1, ddx = pp & 1;
      float d[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int wa = w >> 1, wb = w & 1;
        if ((wa && !ddy) || (wb && !ddx)) continue;
        const uint32_t gw[2] = {qg[w].x, qg[w].y};
        const unsigned code = wcode(ddy ? (wa ? 0 : 2) : 1, ddx ? (wb ? 0 : 2) : 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t g = gw[j >> 1];
          const float gf = __uint_as_float((j & 1) ? (g & 0xffff0000u) : (g << 16));
          d[j] += (qi[w] & (15u << (4 * j))) == (code << (4 * j)) ? gf : 0.f;
        }
      }
      res[pp] = make_uint2(pack_bf2(d[0], d[1]), pack_bf2(d[2], d[3]));
    }
  };


  // dataset row bases of the current and the next image, read once per image (a per-step
  // index read is a vector load whose wait would drain the in-flight prefetches)
  long long bcur = nimg > 0 ? img_base(0) : 0, bnext = nimg > 1 ? img_base(1) : 0;
  int bq = 0;
  auto base = [&](int qq) {
    if (qq != bq) {
      bcur = bnext;
      bq = qq;
      bnext = qq + 1 < nimg ? img_base(qq + 1) : 0;
    }
    return bcur;
  };
  const bool trv = a.trace && blockIdx.x == 0 && vt < 64;
  // raw rows: stored into S before the mid-step barrier of step kk (the MFMA waves expand them
  // after it), loaded during step kk - 1: kk = 1 rows 0..1, kk = i + 2 rows 4i+2..4i+5
  for (int st = 0; st <= nsteps; ++st) {
    const int q = st / SPI, kk = st - q * SPI;
    if (trv) a.trace[st * 8 + 0] = stamp();
    lds_barrier();  // (MFMA waves: step start)
    if (trv) a.trace[st * 8 + 1] = stamp();
    // ---- phase 1 (MFMA waves: the first m-steps of the previous step's pair)
    if (st < nsteps) {
      if (kk == 0) {
        pload(q, 0);
        pstore(0);
        pload(q, 1);
        pstore(1);
        pload(q, 2);  // stored at pair 0
      } else if (kk == 1) {
        rm.store<DT>(ru, S, G.SP, 2);  // rows 0..1
      } else {
        const int i = kk - 2;
        // pooled ring: rows i, i+1 are gathered this step (both phases); row i+2 goes into
        // the slot of row i-1 (last read in the previous step); row i+3 is loaded
        pstore(i + 2);
        pload(q, i + 3);
        rm.store<DT>(ru, S, G.SP, 4);  // rows 4i+2..4i+5
        // the quad's 4 windows: pooled rows i (+1), columns qb (+1); channels 0..3 of the
        // chunk now, 4..7 after the mid-step barrier (each half reloads its windows)
        if (pl && !(a.ablate & 4)) gquad(gres, i, 0);
      }
    }
    if (trv) a.trace[st * 8 + 2] = stamp();
    lds_barrier();  // (MFMA waves: mid-step) this step's S and pooled-ring reads are done
    if (trv) a.trace[st * 8 + 3] = stamp();
    // ---- phase 2 (MFMA waves: the rest of the pair, then the E expansion)
    if (st < nsteps) {
      if (kk == 0) {
        rm.load<DT>(ru, a.img, base(q), G.Hin, G.Win, 0, 2);
      } else if (kk == 1) {
        rm.load<DT>(ru, a.img, base(q), G.Hin, G.Win, 2, 4);
      } else {
        const int i = kk - 2;
        if (pl && !(a.ablate & 4)) {
          uint2 r1[4];
          gquad(r1, i, 1);
          // whole 16-byte chunks: 8-lane groups of ds_write_b128 fill a pixel row, conflict-free
          // (half-chunk 8-byte writes of same-parity pixels were 4-way bank conflicts)
          unsigned char* Tt = T + (st & 1) * TB;
#pragma unroll
          for (int pp = 0; pp < 4; ++pp)
            *reinterpret_cast<uint4*>(Tt + toff[pp]) = make_uint4(gres[pp].x, gres[pp].y, r1[pp].x, r1[pp].y);
        }
        if (trv) a.trace[16384 + st * 4 + 0] = stamp();
        if (trv) a.trace[16384 + st * 4 + 1] = stamp();
        if (trv) a.trace[16384 + st * 4 + 2] = stamp();
        if (i + 1 < G.PH) rm.load<DT>(ru, a.img, base(q), G.Hin, G.Win, 4 * i + 6, 4);
      }
    }
  }
}

// Fixed-order sums of the per-workgroup D and G slabs (one thread per element, 4 partial
// chains combined in order): dsum [64][SKH], gsum [GK][GK] (upper-triangle tiles meaningful)
__global__ void __launch_bounds__(256) stem_slab_reduce_kernel(const float* __restrict__ dslab,
                                                               const float* __restrict__ gslab,
                                                               int GD, float* __restrict__ dsum,
                                                               float* __restrict__ gsum) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int nd = SCO * SKH, ng = GK * GK;
  if (e >= nd + ng) return;
  const float* src = e < nd ? dslab + e : gslab + (e - nd);
  const long long stride = e < nd ? nd : ng;
  float s4[4] = {0.f, 0.f, 0.f, 0.f};
  int gi = 0;
  for (; gi + 4 <= GD; gi += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) s4[u] += src[(long long)(gi + u) * stride];
  for (; gi < GD; ++gi) s4[0] += src[(long long)gi * stride];
  const float v = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  if (e < nd) dsum[e] = v;
  else gsum[e - nd] = v;
}

// dW[co][c][ky][kx] = beta * dW + a D[co][k] + b (W G)[co][k] + cc G[GONE][k], k = ky*24 + kx*3 + c
__global__ void __launch_bounds__(256) stem_wcombine_kernel(const float* __restrict__ dsum,
                                                            const float* __restrict__ gsum,
                                                            const bf16_t* __restrict__ wk,
                                                            const float* __restrict__ coef,
                                                            float* __restrict__ dw, float beta) {
  __shared__ float wrow[SKP];
  const int co = blockIdx.x, t = threadIdx.x;
  for (int k = t; k < SKP; k += 256) wrow[k] = bf2f(wk[co * SKP + k]);
  __syncthreads();
  if (t >= 147) return;
  const int ky = t / 21, rem = t - 21 * ky, kx = rem / 3, c = rem - 3 * kx;
  const int k = ky * 24 + kx * 3 + c;
  float wg = 0.f;
  for (int j = 0; j < SKP; ++j) {
    const float gv = j <= k ? gsum[j * GK + k] : gsum[k * GK + j];  // symmetric: upper tiles
    wg = fmaf(wrow[j], gv, wg);
  }
  const float colsum = GONE <= k ? gsum[GONE * GK + k] : gsum[k * GK + GONE];
  const float d = coef[co] * dsum[co * SKH + k] + coef[SCO + co] * wg + coef[2 * SCO + co] * colsum;
  float* o = dw + ((co * 3 + c) * 7 + ky) * 7 + kx;
  *o = (beta != 0.f ? beta * *o : 0.f) + d;
}

// OIHW fp32 [64][3][7][7] -> [64][SKP] bf16, k = ky*24 + kx*3 + c (pads zero)
__global__ void __launch_bounds__(256) stem_pack_weights_kernel(const float* __restrict__ w,
                                                                bf16_t* __restrict__ wk) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= SCO * SKP) return;
  const int co = e / SKP, k = e - co * SKP;
  const int ky = k / 24, kk = k - 24 * ky, kx = kk / 3, c = kk - 3 * kx;
  float v = 0.f;
  if (ky < 7 && kk < 21) v = w[((co * 3 + c) * 7 + ky) * 7 + kx];
  wk[e] = f2bf(v);
}

// ------------------------------------------------------------------------------- host side
static StemGeo stem_geo(int Hin, int Win) {
  StemGeo G;
  G.Hin = Hin;
  G.Win = Win;
  G.Hout = Hin / 2;
  G.Wout = Win / 2;
  G.PH = G.Hout / 2;
  G.PW = G.Wout / 2;
  G.ROWB = G.Wout * 48;
  G.SP = 3 * Win + 24;
  return G;
}

bool stem_fused_supported(int Hin, int Win) {
  // Wout a multiple of 16 (wgrad m-steps) and <= 128 (4 M-blocks); rows in 4-element units
  // (LDS: the backward's weights + 13 E rows + tile + staging + pooled-row ring fit 160 KB
  // up to W 224: 160,704 B there)
  return Hin >= 8 && Hin % 4 == 0 && Win % 32 == 0 && Win <= 224;
}

static size_t fwd_smem(const StemGeo& G) {
  const size_t tiles = (size_t)RING * G.ROWB + (size_t)2 * 2 * G.Wout * 128 + (size_t)2 * 4 * G.SP * 2;
  const size_t red = (size_t)4 * 2 * 16 * 64 * 4;  // the statistics exchange at exit (32 KB)
  return tiles > red ? tiles : red;
}
static size_t bwd_smem(const StemGeo& G) {
  // E ring + 2 dz tiles + S (4 rows) + pooled ring (bf16 grads + 4-bit codes)
  return (size_t)RING * G.ROWB + (size_t)2 * 2 * G.Wout * 128 + (size_t)4 * G.SP * 2 +
         (size_t)PRING * G.PW * SCO * 2 + (size_t)PRING * G.PW * SCO / 2;
}

// DMLAB_STEM_ABLATE=<bits>: timing experiments (wrong results): 1 conv MFMAs, 2 wgrad MFMAs,
// 4 pooling / gather, 8 E expansion
static int stem_ablate() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("DMLAB_STEM_ABLATE");
    v = e ? atoi(e) : 0;
  }
  return v;
}

int stem_fused_grid(int N) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const char* e = getenv("DMLAB_STEM_GRID");  // tuning: workgroups (default one per CU)
    if (e && atoi(e) > 0 && atoi(e) < cus) cus = atoi(e);
  }
  return N < cus ? N : cus;
}

void stem_fwd_fused(const void* img, int dtype, const long long* idx, const float* nsc,
                    const float* nbi, const bf16_t* wk, const float* gamma, bf16_t* pext,
                    uint8_t* code, float* stats, int N, int nimg, int Hin, int Win, int grid,
                    hipStream_t st) {
  StemFwdArgs a;
  a.img = img;
  a.idx = idx;
  for (int c = 0; c < 3; ++c) {
    a.nsc[c] = nsc[c];
    a.nbi[c] = nbi[c];
  }
  a.wk = wk;
  a.gamma = gamma;
  a.pext = pext;
  a.code = code;
  a.stats = stats;
  a.N = N;
  a.nimg = nimg;
  a.G = stem_geo(Hin, Win);
  a.ablate = stem_ablate();
  const size_t sm = fwd_smem(a.G);
#define DM_SF(DT)                                              \
  do {                                                         \
    set_smem_attr(stem_fwd_kernel<DT>, sm);                    \
    stem_fwd_kernel<DT><<<grid, FNT, sm, st>>>(a);             \
  } while (0)
  if (dtype == 0) DM_SF(0);
  else if (dtype == 1) DM_SF(1);
  else DM_SF(2);
#undef DM_SF
  DM_CHECK(hipGetLastError());
}

void stem_pool_apply(const bf16_t* pext, const uint8_t* code, const float* scale,
                     const float* shift, bf16_t* out, uint8_t* code4, long long n, hipStream_t st) {
  const long long n8 = n / 8;
  stem_pool_apply_kernel<<<(unsigned)((n8 + 1023) / 1024), 256, 0, st>>>(
      pext, reinterpret_cast<const uint32_t*>(code), scale, shift, out,
      reinterpret_cast<uint32_t*>(code4), n8);
  DM_CHECK(hipGetLastError());
}

void stem_bwd_fused2(const void* img, int dtype, const long long* idx, const float* nsc,
                     const float* nbi, const bf16_t* wk, const bf16_t* pdy, const uint8_t* code4,
                     float* dslab, float* gslab, int N, int nimg, int Hin, int Win, int grid,
                     hipStream_t st) {
  StemBwdArgs2 a;
  a.img = img;
  a.idx = idx;
  for (int c = 0; c < 3; ++c) {
    a.nsc[c] = nsc[c];
    a.nbi[c] = nbi[c];
  }
  a.wk = wk;
  a.pdy = pdy;
  a.code4 = code4;
  a.dslab = dslab;
  a.gslab = gslab;
  a.N = N;
  a.nimg = nimg;
  a.G = stem_geo(Hin, Win);
  a.ablate = stem_ablate();
  {
    static int sp = -1;
    if (sp < 0) {
      const char* e = getenv("DMLAB_STEM_SPLIT");  // tuning: default 10 of 14 at W 224
      sp = e ? atoi(e) : 0;
    }
    a.split = sp > 0 ? sp : (2 * (a.G.Wout >> 4) * 5 + 6) / 7;
  }
  static unsigned long long* trace_buf = nullptr;
  const bool trace = getenv("DMLAB_STEM_TRACE") != nullptr;
  const int nst = ((N + grid - 1) / grid) * (a.G.PH + 2) + 1;
  if (trace && !trace_buf) {
    DM_CHECK(hipMalloc(&trace_buf, 8 * 8 * 4096));
    DM_CHECK(hipMemset(trace_buf, 0, 8 * 8 * 4096));
  }
  // [0, nst*8) per-step stamps, [16384, 16384 + nst*4) the second region: disjoint for nst <= 2048
  a.trace = trace && nst <= 2048 ? trace_buf : nullptr;
  const size_t sm = bwd_smem(a.G);
#define DM_SB(DT)                                              \
  do {                                                         \
    set_smem_attr(stem_bwd_kernel<DT>, sm);                    \
    stem_bwd_kernel<DT><<<grid, BNT, sm, st>>>(a);             \
  } while (0)
  if (dtype == 0) DM_SB(0);
  else if (dtype == 1) DM_SB(1);
  else DM_SB(2);
#undef DM_SB
  DM_CHECK(hipGetLastError());
  if (a.trace) {  // per-step medians of workgroup 0's phases (s_memtime units)
    std::vector<unsigned long long> h((size_t)nst * 8), h2((size_t)nst * 4);
    DM_CHECK(hipStreamSynchronize(st));
    DM_CHECK(hipMemcpy(h.data(), a.trace, h.size() * 8, hipMemcpyDeviceToHost));
    DM_CHECK(hipMemcpy(h2.data(), a.trace + 16384, h2.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> col[12];
    for (int s2 = 1; s2 + 1 < nst; ++s2) {
      const unsigned long long* r = &h[(size_t)s2 * 8];
      const unsigned long long* nx = &h[(size_t)(s2 + 1) * 8];
      const unsigned long long* r2 = &h2[(size_t)s2 * 4];
      col[0].push_back((double)(r[2] - r[1]));   // VALU phase 1
      col[1].push_back((double)(r[3] - r[2]));   // VALU mid wait
      col[2].push_back((double)(nx[0] - r[3]));  // VALU phase 2
      col[3].push_back((double)(nx[1] - nx[0])); // VALU step-start wait
      col[4].push_back((double)(r[6] - r[5]));   // MFMA phase 1
      col[5].push_back((double)(r[7] - r[6]));
      col[6].push_back((double)(nx[4] - r[7]));
      col[7].push_back((double)(nx[5] - nx[4]));
      col[8].push_back((double)(nx[0] - r[0]));  // whole step
      if (r2[0] >= r[3] && r2[2] <= nx[0] && r2[0]) {
        col[9].push_back((double)(r2[0] - r[3]));
        col[10].push_back((double)(r2[2] - r2[0]));
        col[11].push_back((double)(nx[0] - r2[2]));
      }
    }
    auto med = [](std::vector<double> v) {
      if (v.empty()) return 0.0;
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    const double tot = (double)(h[(size_t)(nst - 1) * 8] - h[8]) / (nst - 2);
    fprintf(stderr,
            "stem_bwd trace (medians, units/step; mean step %.0f): step %.0f | VALU p1 %.0f wait %.0f "
            "p2 %.0f wait %.0f [p2: gather %.0f raw %.0f rest %.0f] | MFMA p1 %.0f wait %.0f p2 %.0f "
            "wait %.0f\n",
            tot, med(col[8]), med(col[0]), med(col[1]), med(col[2]), med(col[3]), med(col[9]),
            med(col[10]), med(col[11]), med(col[4]), med(col[5]), med(col[6]), med(col[7]));
  }

}

void stem_wcombine(const float* dslab, const float* gslab, int GD, const bf16_t* wk,
                   const float* coef, float* sums, float* dw, float beta, hipStream_t st) {
  const int n = SCO * SKH + GK * GK;
  float* dsum = sums;
  float* gsum = sums + SCO * SKH;
  stem_slab_reduce_kernel<<<(n + 255) / 256, 256, 0, st>>>(dslab, gslab, GD, dsum, gsum);
  DM_CHECK(hipGetLastError());
  stem_wcombine_kernel<<<SCO, 256, 0, st>>>(dsum, gsum, wk, coef, dw, beta);
  DM_CHECK(hipGetLastError());
}
int stem_gram_cols() { return GK; }
int stem_sums_len() { return SCO * SKH + GK * GK; }

void stem_pack_weights(const float* w, bf16_t* wk, hipStream_t st) {
  stem_pack_weights_kernel<<<(SCO * SKP + 255) / 256, 256, 0, st>>>(w, wk);
  DM_CHECK(hipGetLastError());
}

int stem_slab_cols() { return SKH; }
int stem_wk_cols() { return SKP; }

}  // namespace dm
