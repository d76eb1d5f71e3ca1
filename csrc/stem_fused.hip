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
//    pooled extremum of the RAW conv output and its window position (code kh*3 + kw, the
//    first extremum in PyTorch's scan order); the full-resolution conv output (1.6 GB at
//    batch 1024) never reaches memory.  A small pass then applies BN + ReLU to the pooled
//    tensor and marks relu-masked windows (code 15).
//  * BN statistics (sum, sum of squares) from the fp32 accumulators, one row per workgroup.
//
// Backward (stem_bwd_kernel), same walk: the weight gradient of y = conv(x) under the BN
// backward  dy = a*dz + b*y + cc  (dz: the pooled gradient routed to its window's selected
// pixel).  y is not stored, so the kernel RECOMPUTES it: per row pair, (1) a*dz from the
// pooled gradient and codes (a 2x2 quad of pixels shares its 4 windows) into a bf16 tile,
// (2) the conv MFMAs again (fp32 y in registers, the tile read/updated in place:
// dy = a*dz + b*y + cc in fp32, then bf16 -- the mean-subtraction terms b*y + cc cancel in
// fp32 per element, as in the unfused BN backward), (3) dW += dy^T x_col from the tile and
// the E rows.  The 1.6 GB full-resolution y is neither written nor read: 1/3 more stem MFMA
// work instead.  (Splitting dW = sum (a dz + cc) x_col + b * sum y x_col was built first and
// rejected: the bf16 rounding of the large per-channel constant cc does not cancel against
// b * sum y x_col -- 7-90 % gradient error on inputs with a large mean.)
// Warp-specialised like the forward: 8 VALU waves do (1) and the E staging of pair i while the
// 4 MFMA waves (their conv weights resident in registers) do (2) and (3) of pair i-1; the
// window codes travel as 4-bit nibbles (the pooled-row ring then fits LDS beside the ring,
// two tiles and the staging rows).
//  stem_wreduce_kernel sums the per-workgroup slabs in fixed order into the OIHW gradient.
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
  float v[4];
};

// E-ring row of input row iy (iy >= -5)
__device__ __forceinline__ int ring_of(int iy) { return (iy + 13 * 8) % RING; }

// Division-free staging maps, computed once per thread (the loops then only add offsets).
// Raw rows: a group of NT threads loads up to 4 rows = 3W units of 4 elements; thread t owns
// units t, t + NT, ... (at most RU of them).  E rows: thread t < 3 Wout owns chunk (ox, part)
// = (t / 3, t % 3) of every row it builds.
template <int NT, int RU>
struct RawMap {
  int r[RU], k[RU];  // row within the staging, unit within the row (r = -1: none)
  __device__ __forceinline__ void init(int t, int Win) {
    const int upr = 3 * Win / 4;
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const int e = t + NT * u;
      r[u] = e < 4 * upr ? e / upr : -1;
      k[u] = e - (e / upr) * upr;
    }
  }
  template <int DT>
  __device__ __forceinline__ void load(RawUnit (&ru)[RU], const void* img, long long rowbase, int Hin,
                                       int Win, int iy0, int nrows, const float* nsc,
                                       const float* nbi) const {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      const int iy = iy0 + r[u];
      if (r[u] >= 0 && r[u] < nrows && iy >= 0 && iy < Hin) {
        const long long off = rowbase + (long long)iy * Win * 3 + 4LL * k[u];
        if (DT == 0) {
          const float4 f = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(img) + off);
          x[0] = f.x; x[1] = f.y; x[2] = f.z; x[3] = f.w;
        } else if (DT == 1) {
          const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(img) + off);
          x[0] = bf2f((bf16_t)(w.x & 0xffff)); x[1] = bf2f((bf16_t)(w.x >> 16));
          x[2] = bf2f((bf16_t)(w.y & 0xffff)); x[3] = bf2f((bf16_t)(w.y >> 16));
        } else {
          const uint32_t w = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(img) + off);
          x[0] = (float)(w & 0xff); x[1] = (float)((w >> 8) & 0xff);
          x[2] = (float)((w >> 16) & 0xff); x[3] = (float)(w >> 24);
        }
        const int c0 = k[u] % 3;  // channel of element 4k + j is (k + j) % 3
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = (c0 + j) % 3;
          x[j] = x[j] * nsc[c] + nbi[c];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) ru[u].v[j] = x[j];
    }
  }
  __device__ __forceinline__ void store(const RawUnit (&ru)[RU], bf16_t* S, int SP, int nrows) const {
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      if (r[u] < 0 || r[u] >= nrows) continue;
      bf16_t* p = S + r[u] * SP + 4 * k[u] + 9;  // odd element index
      p[0] = f2bf(ru[u].v[0]);
      *reinterpret_cast<uint32_t*>(p + 1) = pack_bf2(ru[u].v[1], ru[u].v[2]);
      p[3] = f2bf(ru[u].v[3]);
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
  __device__ __forceinline__ void build(unsigned char* E, const bf16_t* S, const StemGeo& G, int iy0,
                                        int nrows, int srow0) const {
    if (!act) return;
    for (int q = 0; q < nrows; ++q) {
      const int iy = iy0 + q;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (iy >= 0 && iy < G.Hin) {
        const uint32_t* sp = reinterpret_cast<const uint32_t*>(S + (srow0 + q) * G.SP + soff);
        v = make_uint4(sp[0], sp[1], sp[2], sp[3]);
        if (part == 2) {  // elements 21..23 of the expanded row are the zero pad
          v.z &= 0xffffu;
          v.w = 0;
        }
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

// The wgrad MFMAs of one conv-row pair: acc[kb] (32 co x 32 k, 3 k-blocks per wave) +=
// T[slot][m][co]^T * E[m][k] over the slot's Wout pixels.  Wave w: slot w >> 2, co-block w & 1,
// k-blocks 3*((w >> 1) & 1) + 0..2.  T is the bf16 tile (y in the forward, a*dz + cc in the
// backward), E the ring rows of the pair (base = ring row of iy = 4i - 3).
__device__ __forceinline__ void pair_wgrad(f32x16 (&acc)[3], const unsigned char* T,
                                           const unsigned char* E, const StemGeo& G, int i,
                                           int wid, int lane) {
  const int slot = wid >> 2, cb = wid & 1, kq = (wid >> 1) & 1;
  const int g = lane >> 4, h = g >> 1, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
  const int oy = 2 * i + slot;
  // A: rows m = 16t + 4h + q (+8), channels co = 32cb + 16(g&1) + 4p .. +3
  const int c8 = 4 * cb + 2 * (g & 1) + (p >> 1);
  // rows m and m + 8 (the swizzle is invariant under m + 16, not m + 8)
  const unsigned char* ta = T + yoff(slot, 4 * h + q, c8, G.Wout) + 8 * (p & 1);
  const unsigned char* ta8 = T + yoff(slot, 4 * h + q + 8, c8, G.Wout) + 8 * (p & 1);
  // B: rows m (same), columns k = 32kb + 16(g&1) + 4p .. +3
  int boff[3];
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int k = 32 * (3 * kq + u) + 16 * (g & 1) + 4 * p;
    int ky = k / 24, kk = k - 24 * ky;
    if (ky > 6) ky = 6;  // the pad columns k >= 168 read finite data (their results are unused)
    boff[u] = ring_of(2 * oy - 3 + ky) * G.ROWB + (4 * h + q) * 48 + 2 * kk;
  }
  const int nt = G.Wout >> 4;
  for (int t = 0; t < nt; ++t) {
    const int mo = 16 * t;
    const s4v a0 = tr4(ta + mo * 128), a1 = tr4(ta8 + mo * 128);
    const bf16x8 af = (bf16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const s4v b0 = tr4(E + boff[u] + mo * 48), b1 = tr4(E + boff[u] + (mo + 8) * 48);
      const bf16x8 bf = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[u], 0, 0, 0);
    }
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
      __syncthreads();  // step boundary (the previous step's tile reads / E writes are done)
      if (st == nsteps) break;
      const int kk = st % SPI;
      if (kk < 2) continue;
      const int i = kk - 2;
      unsigned char* Yt = Y + (st & 1) * YB;
      const int ring0 = (4 * i - 3 + 2 * slot + 13 * 8) % RING;  // ring row of ky = 0
#pragma unroll 1
      for (int mb = 0; mb < 4; ++mb) {
        if (32 * mb >= G.Wout) break;
        const int px = 32 * mb + (lane & 31);
        const int pxb = min(px, G.Wout - 1);
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < 11; ++s) {
          const int j = 2 * s + hh;
          int ky = j / 3;
          const int part = j - 3 * ky;
          if (ky > 6) ky = 6;  // k-step 10's upper half: zero weights, finite data
          int rr = ring0 + ky;
          rr = rr >= RING ? rr - RING : rr;
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(E + rr * G.ROWB + pxb * 48 + part * 16);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], bfr, acc, 0, 0, 0);
        }
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
  rm.init(vt, G.Win);
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
  if (nimg > 0) {
    rm.load<DT>(ru, a.img, img_base(0), G.Hin, G.Win, 0, 4, a.nsc, a.nbi);
    rm.store(ru, S + 1 * SB, G.SP, 4);  // consumed by step 0 from S[(0 - 1) & 1] = S[1]
  }
  for (int st = 0; st <= nsteps; ++st) {
    __syncthreads();
    const int q = st / SPI, kk = st - q * SPI;
    // (c) raw rows for the NEXT step's E build, issued first (consumed at this step's end)
    int nrows = 0, niy = 0, nq = q;
    if (st + 1 < nsteps) {
      const int k1 = kk + 1 == SPI ? 0 : kk + 1;
      if (k1 == 0) { nq = q + 1; nrows = 4; niy = 0; }
      else if (k1 == 1) { nrows = 2; niy = 4; }
      else if (k1 - 2 + 1 < G.PH) { nrows = 4; niy = 4 * (k1 - 2) + 6; }
      if (nrows) rm.load<DT>(ru, a.img, img_base(nq), G.Hin, G.Win, niy, nrows, a.nsc, a.nbi);
    }
    // (a) pooling of the pair the MFMA waves computed in the previous step
    if (st >= 1) {
      const int ps = st - 1, pq = ps / SPI, pk = ps - pq * SPI;
      if (pk >= 2 && pact) {
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
    if (st < nsteps) {
      const bf16_t* Sp = S + ((st - 1) & 1) * SB;
      if (kk == 0) em.build(E, Sp, G, -3, 7, -3);
      else if (kk == 1) em.build(E, Sp, G, 4, 2, 0);
      else if (kk - 2 + 1 < G.PH) em.build(E, Sp, G, 4 * (kk - 2) + 6, 4, 0);
    }
    if (nrows) rm.store(ru, S + (st & 1) * SB, G.SP, nrows);
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
struct StemBwdArgs2 {
  const void* img;
  const long long* idx;
  float nsc[3], nbi[3];
  const bf16_t* wk;      // [64][SKP] packed weights (the forward's)
  const bf16_t* pdy;     // [N][PH][PW][64] pooled gradient
  const uint8_t* code4;  // [N][PH][PW][32] window positions, 4 bits per channel, 15 = masked
  const float* coef;     // [3][64] a, b, cc
  float* dslab;          // [grid][64][SKH]
  int N, nimg;
  StemGeo G;
};

constexpr int PRING = 3;  // pooled-row ring: rows i, i+1 in use, i+2 staged
constexpr int BNT = 768;  // 12 waves: 0-3 MFMA, 4-11 VALU
constexpr int BVT = BNT - 256;

// Warp-specialised backward.  Step stream per image: [stage E rows -3..3 + pooled rows 0..2,
// stage rows 4..5, pair 0, ..., pair PH-1, (drain)]; the VALU waves build pair i's a*dz tile
// T[i & 1] (and stage pair i+1's E rows) while the MFMA waves process pair i-1: recompute
// its conv output y (weights resident in registers, C = [co][px]), turn T into
// dy = a*dz + b*y + cc in place, then reduce dy^T x_col.  Two barriers per step: the y pass
// of every MFMA wave completes before any wgrad read of T, and the VALU waves' S reads before
// the raw rows of the next step overwrite it.
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
  float* cf = reinterpret_cast<float*>(Pc + PRING * PRB / 2);  // a, b, cc
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  {
    const int tot16 = (RING * G.ROWB + 2 * TB + 4 * G.SP * 2) / 16;
    for (int e = tid; e < tot16; e += BNT) reinterpret_cast<uint4*>(smem)[e] = make_uint4(0, 0, 0, 0);
  }
  if (tid < 3 * SCO) cf[tid] = a.coef[tid];
  const int nimg = a.N > (int)blockIdx.x ? (a.N - 1 - (int)blockIdx.x) / (int)gridDim.x + 1 : 0;
  const int SPI = G.PH + 2;
  const int nsteps = nimg * SPI;  // + 1 drain step (the last pair's MFMA work)
  auto img_of = [&](int q) { return (int)blockIdx.x + q * (int)gridDim.x; };
  auto img_base = [&](int q) -> long long {
    long long row = a.idx ? a.idx[img_of(q)] : (long long)img_of(q);
    row = row < 0 ? 0 : row >= a.nimg ? a.nimg - 1 : row;
    return row * G.Hin * G.Win * 3;
  };
  if (wid < 4) {
    // ================================================================ MFMA waves
    // y pass: wave w owns co-block cb = w & 1 and px-blocks (w >> 1) * 2 + {0, 1} of BOTH
    // slots (4 units); its A fragments (the weights of its 32 channels, 11 k-steps) stay in
    // registers.  wgrad pass: pair_wgrad's wave roles with w and w + 4 of the 8-wave layout
    // (slot, co-block, k-blocks) folded onto 4 waves: wave w does roles w and w + 4.
    const int cb = wid & 1, hh = lane >> 5;
    bf16x8 wa[11];
#pragma unroll
    for (int s = 0; s < 11; ++s)
      wa[s] = *reinterpret_cast<const bf16x8*>(a.wk + (32 * cb + (lane & 31)) * SKP + 16 * s + 8 * hh);
    f32x16 dacc[3];
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) dacc[u][r] = 0.f;
    __syncthreads();  // cf, zeroed LDS
    for (int st = 0; st <= nsteps; ++st) {
      __syncthreads();  // step start: T[(st-1) & 1] (a dz of the pair) and its E rows are ready
      const int ps = st - 1;
      const int pk = ps >= 0 ? ps % SPI : -1;
      const bool work = ps >= 0 && pk >= 2;
      const int i = pk - 2;
      unsigned char* Tt = T + (ps & 1) * TB;
      if (work) {
        const int ring0 = (4 * i - 3 + 13 * 8) % RING;  // ring row of iy = 4i - 3
#pragma unroll 1
        for (int u = 0; u < 4; ++u) {
          const int slot = u >> 1, mb = 2 * (wid >> 1) + (u & 1);
          if (32 * mb >= G.Wout) continue;
          const int pxb = min(32 * mb + (lane & 31), G.Wout - 1);
          const int pxo = 32 * mb + (lane & 31);
          f32x16 acc;
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
          for (int s = 0; s < 11; ++s) {
            const int j = 2 * s + hh;
            int ky = j / 3;
            const int part = j - 3 * ky;
            if (ky > 6) ky = 6;
            int rr = ring0 + 2 * slot + ky;  // iy = 2 oy - 3 + ky, oy = 2i + slot
            rr = rr >= RING ? rr - RING : rr;
            rr = rr >= RING ? rr - RING : rr;
            const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(E + rr * G.ROWB + pxb * 48 + part * 16);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wa[s], bfr, acc, 0, 0, 0);
          }
          // C: col = px (lane & 31), row = co = 32 cb + (r & 3) + 8 (r >> 2) + 4 hh
          if (pxo < G.Wout) {
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
              const int co = 32 * cb + 8 * g4 + 4 * hh;
              unsigned char* tp = Tt + yoff(slot, pxo, co >> 3, G.Wout) + 2 * (co & 7);
              const uint2 t = *reinterpret_cast<const uint2*>(tp);
              const float4 bv = *reinterpret_cast<const float4*>(cf + SCO + co);
              const float4 cv = *reinterpret_cast<const float4*>(cf + 2 * SCO + co);
              const float d0 = bf2f((bf16_t)(t.x & 0xffff)) + bv.x * acc[4 * g4 + 0] + cv.x;
              const float d1 = bf2f((bf16_t)(t.x >> 16)) + bv.y * acc[4 * g4 + 1] + cv.y;
              const float d2 = bf2f((bf16_t)(t.y & 0xffff)) + bv.z * acc[4 * g4 + 2] + cv.z;
              const float d3 = bf2f((bf16_t)(t.y >> 16)) + bv.w * acc[4 * g4 + 3] + cv.w;
              *reinterpret_cast<uint2*>(tp) = make_uint2(pack_bf2(d0, d1), pack_bf2(d2, d3));
            }
          }
        }
      }
      __syncthreads();  // mid-step: every wave's dy is in T
      if (work) {
        pair_wgrad(dacc, Tt, E, G, i, wid, lane);      // slot 0
        pair_wgrad(dacc, Tt, E, G, i, wid + 4, lane);  // slot 1
      }
    }
    // slab: both slots' partials are in dacc (same co / k positions)
    const int kq = (wid >> 1) & 1;
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = 32 * (3 * kq + u) + (lane & 31);
        a.dslab[(long long)blockIdx.x * SCO * SKH + co * SKH + k] = dacc[u][r];
      }
    return;
  }
  // ================================================================== VALU waves
  // Per image (SPI = PH + 2 steps): kk = 0 stages raw rows 0..1 and pooled rows 0..2 (the
  // MFMA waves finish the previous image's last pair); kk = 1 expands E rows -3..1; kk = i + 2
  // expands rows 4i+2..4i+5 (the new rows of pair i) and gathers pair i's a*dz into T.  The
  // MFMA waves read pair i-1's rows 4i-7..4i+1 meanwhile: 13 live rows, the ring's size.
  // Raw rows are stored into S after the mid-step barrier (the step's S reads are done) and
  // expanded the step after.
  const int vt = tid - 256;
  RawMap<BVT, FRU> rm;
  rm.init(vt, G.Win);
  EMap em;
  em.init(vt, G.Wout);
  RawUnit ru[FRU];
  // pooled rows: PW * 8 chunks of (8 grads, 8 4-bit codes) per row; thread vt < PW*8 owns one
  const bool pl = vt < G.PW * 8;
  uint4 pg_r = make_uint4(0, 0, 0, 0);
  uint32_t pc_r = 0xffffffffu;
  auto pload = [&](int q, int r) {
    pg_r = make_uint4(0, 0, 0, 0);
    pc_r = 0xffffffffu;  // rows past the image: masked windows
    if (pl && r < G.PH) {
      const long long o = (((long long)img_of(q) * G.PH + r) * G.PW) * SCO + vt * 8;
      pg_r = *reinterpret_cast<const uint4*>(a.pdy + o);
      pc_r = *reinterpret_cast<const uint32_t*>(a.code4 + o / 2);
    }
  };
  auto pstore = [&](int r) {
    if (!pl) return;
    const int sl = r % PRING;
    *reinterpret_cast<uint4*>(Pg + sl * PRB + vt * 8) = pg_r;
    *reinterpret_cast<uint32_t*>(Pc + (sl * PRB + vt * 8) / 2) = pc_r;
  };
  const int qb = vt >> 3, qc = vt & 7, c0 = qc * 8;
  __syncthreads();  // cf, zeroed LDS
  float ka[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ka[j] = cf[c0 + j];
  uint4 qg[4];     // the quad's windows: 8 pooled grads each
  uint32_t qi[4];  // and their codes (15 everywhere for a window outside the image)
  // a*dz of quad pixel pp = (ddy, ddx): the sum of the grads of the covering windows whose
  // code names this pixel (window (wa, wb) sees it at kh = ddy ? (wa ? 0 : 2) : 1, same for kw)
  auto gpix = [&](unsigned char* Tt, int pp) {
    const int ddy = pp >> 1, ddx = pp & 1;
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int wa = w >> 1, wb = w & 1;
      if ((wa && !ddy) || (wb && !ddx)) continue;
      const uint32_t gw[4] = {qg[w].x, qg[w].y, qg[w].z, qg[w].w};
      const unsigned code = wcode(ddy ? (wa ? 0 : 2) : 1, ddx ? (wb ? 0 : 2) : 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t g = gw[j >> 1];
        const float gf = __uint_as_float((j & 1) ? (g & 0xffff0000u) : (g << 16));
        d[j] += (qi[w] & (15u << (4 * j))) == (code << (4 * j)) ? gf : 0.f;
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = pack_bf2(ka[2 * k] * d[2 * k], ka[2 * k + 1] * d[2 * k + 1]);
    *reinterpret_cast<uint4*>(Tt + yoff(ddy, 2 * qb + ddx, qc, G.Wout)) = make_uint4(o[0], o[1], o[2], o[3]);
  };
  if (nimg > 0) rm.load<DT>(ru, a.img, img_base(0), G.Hin, G.Win, 0, 2, a.nsc, a.nbi);
  for (int st = 0; st <= nsteps; ++st) {
    const int q = st / SPI, kk = st - q * SPI;
    __syncthreads();  // (MFMA waves: step start)
    // ---- phase 1 (MFMA waves: y pass of the previous step's pair)
    if (st < nsteps) {
      if (kk == 0) {
        rm.store(ru, S, G.SP, 2);  // rows 0..1
        pload(q, 0);
        pstore(0);
        pload(q, 1);
        pstore(1);
        pload(q, 2);
        pstore(2);
        pload(q, 3);
        rm.load<DT>(ru, a.img, img_base(q), G.Hin, G.Win, 2, 4, a.nsc, a.nbi);
      } else if (kk == 1) {
        em.build(E, S, G, -3, 5, -3);
      } else {
        const int i = kk - 2;
        em.build(E, S, G, 4 * i + 2, 4, 0);
        if (pl) {
          // the quad's 4 windows: pooled rows i (+1), columns qb (+1); pixels (0,0), (1,1) now,
          // (0,1), (1,0) after the mid-step barrier (5 + 4 window tests: balances the phases)
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int wa = w >> 1, wb = w & 1;
            const bool okw = i + wa < G.PH && qb + wb < G.PW;
            const int sl = (i + wa) % PRING, col = okw ? qb + wb : qb;
            qg[w] = *reinterpret_cast<const uint4*>(Pg + sl * PRB + col * SCO + c0);
            qi[w] = okw ? *reinterpret_cast<const uint32_t*>(Pc + (sl * PRB + col * SCO + c0) / 2)
                        : 0xffffffffu;
          }
          gpix(T + (st & 1) * TB, 0);
          gpix(T + (st & 1) * TB, 3);
        }
      }
    }
    __syncthreads();  // (MFMA waves: mid-step) this step's S and pooled-ring reads are done
    // ---- phase 2 (MFMA waves: wgrad of the previous step's pair)
    if (st < nsteps) {
      if (kk == 1) {
        rm.store(ru, S, G.SP, 4);  // rows 2..5
        if (G.PH > 1) rm.load<DT>(ru, a.img, img_base(q), G.Hin, G.Win, 6, 4, a.nsc, a.nbi);
      } else if (kk >= 2) {
        const int i = kk - 2;
        if (pl) {
          gpix(T + (st & 1) * TB, 1);
          gpix(T + (st & 1) * TB, 2);
        }
        if (i + 1 < G.PH) {
          rm.store(ru, S, G.SP, 4);  // rows 4i+6..4i+9 (pair i+1's new rows)
          pstore(i + 3);             // row i's slot: its last reader was this step's gather
          pload(q, i + 4);
        }
        if (i + 2 < G.PH) rm.load<DT>(ru, a.img, img_base(q), G.Hin, G.Win, 4 * i + 10, 4, a.nsc, a.nbi);
        else if (i + 2 == G.PH && q + 1 < nimg)
          rm.load<DT>(ru, a.img, img_base(q + 1), G.Hin, G.Win, 0, 2, a.nsc, a.nbi);
      }
    }
  }
}

// dW[co][c][ky][kx] = beta * dW + sum_g slab[g][co][k], k = ky*24 + kx*3 + c.  One
// workgroup per output channel; each of the 4 lane groups sums a quarter of the slabs in
// order, the quarters are combined in order (deterministic).
__global__ void __launch_bounds__(256) stem_wreduce_kernel(const float* __restrict__ dslab, int GD,
                                                           float* __restrict__ dw, float beta) {
  __shared__ float part[4][SKH];
  const int co = blockIdx.x, t = threadIdx.x, k = t & 63, gq = t >> 6;
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    float s = 0.f;
    for (int g = gq; g < GD; g += 4) s += dslab[((long long)g * SCO + co) * SKH + k + 64 * u];
    part[gq][k + 64 * u] = s;
  }
  __syncthreads();
  for (int e = t; e < 147; e += 256) {
    const int ky = e / 21, rem = e - 21 * ky, kx = rem / 3, c = rem - 3 * kx;
    const int kk = ky * 24 + kx * 3 + c;
    const float d = ((part[0][kk] + part[1][kk]) + part[2][kk]) + part[3][kk];
    float* o = dw + ((co * 3 + c) * 7 + ky) * 7 + kx;
    *o = (beta != 0.f ? beta * *o : 0.f) + d;
  }
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
  return (size_t)RING * G.ROWB + (size_t)2 * 2 * G.Wout * 128 + (size_t)2 * 4 * G.SP * 2;
}
static size_t bwd_smem(const StemGeo& G) {
  // E ring + 2 tiles + S (4 rows) + pooled ring (bf16 grads + 4-bit codes) + coefficients
  return (size_t)RING * G.ROWB + (size_t)2 * 2 * G.Wout * 128 + (size_t)4 * G.SP * 2 +
         (size_t)PRING * G.PW * SCO * 2 + (size_t)PRING * G.PW * SCO / 2 + 3 * SCO * 4;
}

int stem_fused_grid(int N) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
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
                     const float* coef, float* dslab, int N, int nimg, int Hin, int Win, int grid,
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
  a.coef = coef;
  a.dslab = dslab;
  a.N = N;
  a.nimg = nimg;
  a.G = stem_geo(Hin, Win);
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
}

void stem_wreduce(const float* dslab, int GD, float* dw, float beta, hipStream_t st) {
  stem_wreduce_kernel<<<SCO, 256, 0, st>>>(dslab, GD, dw, beta);
  DM_CHECK(hipGetLastError());
}

void stem_pack_weights(const float* w, bf16_t* wk, hipStream_t st) {
  stem_pack_weights_kernel<<<(SCO * SKP + 255) / 256, 256, 0, st>>>(w, wk);
  DM_CHECK(hipGetLastError());
}

int stem_slab_cols() { return SKH; }
int stem_wk_cols() { return SKP; }

}  // namespace dm
