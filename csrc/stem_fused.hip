// ResNet stem, fused: 7x7/s2/p3 conv (3 -> 64) + BatchNorm statistics + 3x3/s2/p1 max-pool,
// with the raw dataset gather/normalisation folded into the kernel and a K-dense GEMM layout.
//
// Reference: the stem is not in the reference (SURVEY §2.5 "Extensions required by
// BASELINE.json": ResNet-18-shaped CNN); it replaces cuDNN conv + BN + ReLU + max-pool.
//
// Forward (stem_fwd_kernel), one persistent 512-thread workgroup per CU walking whole images,
// one conv-row PAIR (2i, 2i+1) per step:
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
//  stem_wreduce_kernel sums the per-workgroup slabs in fixed order into the OIHW gradient.
#include "common.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {

constexpr int SNT = 512;    // threads per workgroup (8 waves)
constexpr int SCO = 64;     // output channels
constexpr int SKP = 176;    // packed weight row: 7 ky x 24 + 8 pad
constexpr int SWP = 184;    // weight row pitch in LDS (368 B: conflict-free B-fragment reads)
constexpr int SKH = 192;    // H / D' columns per slab row (6 k-blocks of 32)
constexpr int RING = 13;    // E-row ring
constexpr int SROWS = 6;    // raw rows staged at once (image prologue: rows 0..5)
constexpr int UPT = 3;      // raw 4-element units per thread per staging (<= 6 x 3*256/4 / 512)

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

template <int DT>
__device__ __forceinline__ void raw_load(RawUnit (&u)[UPT], const void* img, long long rowbase_elems,
                                         int Hin, int Win, int iy0, int nrows, const float* nsc,
                                         const float* nbi, int tid) {
  // units of 4 consecutive row elements; unit e of the block: row e / (3W/4), k = e % (3W/4)
  const int upr = 3 * Win / 4;
  const int total = nrows * upr;
#pragma unroll
  for (int t = 0; t < UPT; ++t) {
    const int e = tid + SNT * t;
    const int r = e / upr, k = e - r * upr;
    const int iy = iy0 + r;
    float x[4] = {0.f, 0.f, 0.f, 0.f};
    if (e < total && iy >= 0 && iy < Hin) {
      const long long off = rowbase_elems + (long long)iy * Win * 3 + 4LL * k;
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
      // channel of element 4k + j is (4k + j) % 3 = (k + j) % 3
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = (k + j) % 3;
        x[j] = x[j] * nsc[c] + nbi[c];
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) u[t].v[j] = x[j];
  }
}

// S[row r][t], t = f + 9 (9 zero pad elements on the left, >= 15 on the right)
__device__ __forceinline__ void raw_store(const RawUnit (&u)[UPT], bf16_t* S, int SP, int Win,
                                          int nrows, int tid) {
  const int upr = 3 * Win / 4;
  const int total = nrows * upr;
#pragma unroll
  for (int t = 0; t < UPT; ++t) {
    const int e = tid + SNT * t;
    if (e >= total) continue;
    const int r = e / upr, k = e - r * upr;
    bf16_t* p = S + r * SP + 4 * k + 9;  // odd element index
    p[0] = f2bf(u[t].v[0]);
    *reinterpret_cast<uint32_t*>(p + 1) = pack_bf2(u[t].v[1], u[t].v[2]);
    p[3] = f2bf(u[t].v[3]);
  }
}

// E rows iy0 .. iy0+nrows-1 from S rows srow0.. (rows outside [0, Hin) are written as zeros)
__device__ __forceinline__ void e_build(unsigned char* E, const bf16_t* S, const StemGeo& G, int iy0,
                                        int nrows, int srow0, int tid) {
  const int per_row = 3 * G.Wout;
  const int total = nrows * per_row;
  for (int e = tid; e < total; e += SNT) {
    const int q = e / per_row, rem = e - q * per_row;
    const int ox = rem / 3, part = rem - ox * 3;
    const int iy = iy0 + q;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (iy >= 0 && iy < G.Hin) {
      const uint32_t* s = reinterpret_cast<const uint32_t*>(S + (srow0 + q) * G.SP + 6 * ox + 8 * part);
      v = make_uint4(s[0], s[1], s[2], s[3]);
      if (part == 2) {  // elements 21..23 of the expanded row are the zero pad
        v.z &= 0xffffu;
        v.w = 0;
      }
    }
    *reinterpret_cast<uint4*>(E + ring_of(iy) * G.ROWB + ox * 48 + part * 16) = v;
  }
}

// Y-tile chunk swizzle: [2 slots][Wout px][8 chunks of 8 channels], chunk ^ (((px >> 1) & 1) << 2)
// -> the 4-row x 32-channel transposed reads of the wgrad MFMAs are conflict-free
__device__ __forceinline__ int yoff(int slot, int px, int c8, int Wout) {
  return ((slot * Wout + px) * 8 + (c8 ^ (((px >> 1) & 1) << 2))) * 16;
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
  const unsigned char* ta = T + yoff(slot, 4 * h + q, c8, G.Wout) + 8 * (p & 1);
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
    const s4v a0 = tr4(ta + mo * 128), a1 = tr4(ta + (mo + 8) * 128);
    const bf16x8 af = (bf16x8){a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const s4v b0 = tr4(E + boff[u] + mo * 48), b1 = tr4(E + boff[u] + (mo + 8) * 48);
      const bf16x8 bf = (bf16x8){b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bf, acc[u], 0, 0, 0);
    }
  }
}

// slab[blk][co][SKH]: the two slot groups' partials summed in fixed order through LDS
__device__ __forceinline__ void write_wslab(const f32x16 (&acc)[3], float* red, float* slab, int wid,
                                            int lane) {
  const int slot = wid >> 2, cb = wid & 1, kq = (wid >> 1) & 1;
  // C layout: col = lane & 31 (k), row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) (co)
  if (slot == 1) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = 32 * (3 * kq + u) + (lane & 31);
        red[co * SKH + k] = acc[u][r];
      }
  }
  __syncthreads();
  if (slot == 0) {
#pragma unroll
    for (int u = 0; u < 3; ++u)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int co = 32 * cb + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int k = 32 * (3 * kq + u) + (lane & 31);
        slab[(long long)blockIdx.x * SCO * SKH + co * SKH + k] = acc[u][r] + red[co * SKH + k];
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
  uint8_t* code;         // [N][PH][PW][64]
  float* stats;          // [grid][2][64] or nullptr
  int N, nimg;           // batch rows, image rows (idx values are clamped to it)
  StemGeo G;
};

template <int DT>
__global__ void __launch_bounds__(SNT, 1) stem_fwd_kernel(StemFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StemGeo G = a.G;
  unsigned char* Ws = smem;                                  // [64][SWP] bf16
  unsigned char* E = Ws + SCO * SWP * 2;                     // [RING][Wout][24] bf16
  unsigned char* Y = E + RING * G.ROWB;                      // [2][Wout][64] bf16 (swizzled)
  bf16_t* S = reinterpret_cast<bf16_t*>(Y + 2 * G.Wout * 128);  // [SROWS][SP]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool train = a.stats != nullptr;   // batch statistics

  // zero everything once (S pads, E pad pixels are never read uninitialised)
  {
    const int tot16 = (SCO * SWP * 2 + RING * G.ROWB + 2 * G.Wout * 128 + SROWS * G.SP * 2) / 16;
    for (int e = tid; e < tot16; e += SNT) reinterpret_cast<uint4*>(smem)[e] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  for (int e = tid; e < SCO * SKP / 8; e += SNT) {
    const int co = e / (SKP / 8), ch = e - co * (SKP / 8);
    *reinterpret_cast<uint4*>(Ws + co * SWP * 2 + ch * 16) =
        *reinterpret_cast<const uint4*>(a.wk + co * SKP + ch * 8);
  }

  // ------------------------------------------------------------------ per-lane roles
  // y MFMA: slot w >> 2 (conv row 2i + slot), M-block w & 3 (32 px), both co-blocks
  const int yslot = wid >> 2, mb = wid & 3;
  const int hh = lane >> 5;
  const bool yact = 32 * mb < G.Wout;
  const int pxa = min(32 * mb + (lane & 31), G.Wout - 1);  // A row (pad lanes re-read px W-1)
  // pooling: thread (j, c8)
  const bool pact = tid < G.PW * 8;
  const int pj = tid >> 3, pc8 = tid & 7;
  float psg[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) psg[c] = (pact && a.gamma[pc8 * 8 + c] < 0.f) ? -1.f : 1.f;

  float st_s[2] = {0.f, 0.f}, st_q[2] = {0.f, 0.f};

  RawUnit ru[UPT];
  auto img_base = [&](int n) -> long long {
    long long row = a.idx ? a.idx[n] : (long long)n;
    row = row < 0 ? 0 : row >= a.nimg ? a.nimg - 1 : row;
    return row * G.Hin * G.Win * 3;
  };
  // prologue: image blockIdx.x, rows 0..5 (rows -3..-1 are zero rows)
  int n = blockIdx.x;
  if (n < a.N) {
    raw_load<DT>(ru, a.img, img_base(n), G.Hin, G.Win, 0, SROWS, a.nsc, a.nbi, tid);
    raw_store(ru, S, G.SP, G.Win, SROWS, tid);
  }
  __syncthreads();
  if (n < a.N) e_build(E, S, G, -3, 9, -3, tid);
  __syncthreads();

  for (; n < a.N; n += gridDim.x) {
    const int nnext = n + gridDim.x;
    float pv[8];
    uint32_t pk = 0;  // previous odd row's horizontal extremum and kw (2 bits per channel)
#pragma unroll
    for (int c = 0; c < 8; ++c) pv[c] = -INFINITY;
    for (int i = 0; i < G.PH; ++i) {
      // ---------------------------------------------------------------- phase A
      // raw rows of the next step: pair i+1 needs rows 4i+6 .. 4i+9; after the image's last
      // pair, the next image's rows 0..5
      const bool last = i + 1 == G.PH;
      const bool more = !last || nnext < a.N;
      int srows = 0, siy = 0;
      if (!last) {
        srows = 4;
        siy = 4 * i + 6;
        raw_load<DT>(ru, a.img, img_base(n), G.Hin, G.Win, siy, 4, a.nsc, a.nbi, tid);
      } else if (nnext < a.N) {
        srows = SROWS;
        siy = 0;
        raw_load<DT>(ru, a.img, img_base(nnext), G.Hin, G.Win, 0, SROWS, a.nsc, a.nbi, tid);
      }
      if (yact) {
        const int oy = 2 * i + yslot;
        const int rb = 2 * oy - 3;
        f32x16 acc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
        const unsigned char* wb = Ws + (lane & 31) * SWP * 2 + 16 * hh;
#pragma unroll
        for (int s = 0; s < 11; ++s) {
          const int j = 2 * s + hh;
          int ky = j / 3;
          const int part = j - 3 * ky;
          if (ky > 6) ky = 6;  // k-step 10's upper half: zero weights, finite data
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(E + ring_of(rb + ky) * G.ROWB + pxa * 48 + part * 16);
          const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(wb + 32 * s);
          const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(wb + 32 * SWP * 2 + 32 * s);
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, acc[1], 0, 0, 0);
        }
        // C: col = co (lane & 31), row = px
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int co = 32 * c + (lane & 31);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int px = 32 * mb + (r & 3) + 8 * (r >> 2) + 4 * hh;
            if (px < G.Wout) {
              const float v = acc[c][r];
              st_s[c] += v;
              st_q[c] += v * v;
              *reinterpret_cast<bf16_t*>(Y + yoff(yslot, px, co >> 3, G.Wout) + 2 * (co & 7)) = f2bf(v);
            }
          }
        }
      }
      if (srows) raw_store(ru, S, G.SP, G.Win, srows, tid);
      __syncthreads();
      // ---------------------------------------------------------------- phase B
      if (pact) {
        float hv[2][8];
        uint32_t hk[2] = {0, 0};
#pragma unroll
        for (int sl = 0; sl < 2; ++sl) {
#pragma unroll
          for (int c = 0; c < 8; ++c) hv[sl][c] = -INFINITY;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int px = 2 * pj - 1 + kw;
            if (px < 0 || px >= G.Wout) continue;
            const uint4 w = *reinterpret_cast<const uint4*>(Y + yoff(sl, px, pc8, G.Wout));
            const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
              const float v = psg[c] * bf2f((bf16_t)((ww[c >> 1] >> (16 * (c & 1))) & 0xffff));
              if (v > hv[sl][c]) {
                hv[sl][c] = v;
                hk[sl] = (hk[sl] & ~(3u << (2 * c))) | ((uint32_t)kw << (2 * c));
              }
            }
          }
        }
        uint32_t o[4];
        uint32_t cd[2] = {0, 0};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float b = pv[c];
          uint32_t code = (pk >> (2 * c)) & 3;  // kh = 0
          if (hv[0][c] > b) {
            b = hv[0][c];
            code = 3 + ((hk[0] >> (2 * c)) & 3);
          }
          if (hv[1][c] > b) {
            b = hv[1][c];
            code = 6 + ((hk[1] >> (2 * c)) & 3);
          }
          const float val = psg[c] * b;  // exact: b is a bf16 value times +-1
          if (c & 1) o[c >> 1] |= (uint32_t)f2bf(val) << 16;
          else o[c >> 1] = f2bf(val);
          cd[c >> 2] |= code << (8 * (c & 3));
          pv[c] = hv[1][c];
        }
        pk = hk[1];
        const long long po = (((long long)n * G.PH + i) * G.PW + pj) * SCO + pc8 * 8;
        __builtin_nontemporal_store((nt4){o[0], o[1], o[2], o[3]}, reinterpret_cast<nt4*>(a.pext + po));
        __builtin_nontemporal_store((nt2){cd[0], cd[1]}, reinterpret_cast<nt2*>(a.code + po));
      }
      if (!last) e_build(E, S, G, 4 * i + 6, 4, 0, tid);
      __syncthreads();
      if (last && more) {  // the next image's first rows: after this pair's MFMA reads of E
        e_build(E, S, G, -3, 9, -3, tid);
        __syncthreads();
      }
    }
  }
  if (!train) return;
  // ------------------------------------------------------------------ statistics
  float* red = reinterpret_cast<float*>(smem);  // reuse: [8 waves][2 halves][64][2]
  __syncthreads();
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int co = 32 * c + (lane & 31);
    red[((wid * 2 + hh) * SCO + co) * 2 + 0] = st_s[c];
    red[((wid * 2 + hh) * SCO + co) * 2 + 1] = st_q[c];
  }
  __syncthreads();
  if (tid < 2 * SCO) {
    const int co = tid & 63, which = tid >> 6;
    float s = 0.f;
    for (int k = 0; k < 16; ++k) s += red[(k * SCO + co) * 2 + which];
    a.stats[(long long)blockIdx.x * 2 * SCO + which * SCO + co] = s;
  }
}

// out = relu(scale * pext + shift); code = 15 where that is <= 0 (no gradient flows)
__global__ void __launch_bounds__(256) stem_pool_apply_kernel(const bf16_t* __restrict__ pext,
                                                              uint8_t* __restrict__ code,
                                                              const float* __restrict__ scale,
                                                              const float* __restrict__ shift,
                                                              bf16_t* __restrict__ out, long long n8) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n8) return;
  const int c0 = (int)(e & 7) * 8;
  const nt4 v = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(pext) + e);
  uint2 cd = code ? reinterpret_cast<const uint2*>(code)[e] : make_uint2(0, 0);
  const uint32_t w[4] = {v[0], v[1], v[2], v[3]};
  uint32_t o[4];
  uint32_t cw[2] = {cd.x, cd.y};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float r[2];
#pragma unroll
    for (int hlf = 0; hlf < 2; ++hlf) {
      const int c = c0 + 2 * k + hlf;
      const float z = bf2f((bf16_t)((w[k] >> (16 * hlf)) & 0xffff)) * scale[c] + shift[c];
      r[hlf] = z > 0.f ? z : 0.f;
      if (!(z > 0.f)) {
        const int b = 2 * k + hlf;
        cw[b >> 2] = (cw[b >> 2] & ~(0xffu << (8 * (b & 3)))) | (15u << (8 * (b & 3)));
      }
    }
    o[k] = pack_bf2(r[0], r[1]);
  }
  __builtin_nontemporal_store((nt4){o[0], o[1], o[2], o[3]}, reinterpret_cast<nt4*>(out) + e);
  if (code) reinterpret_cast<uint2*>(code)[e] = make_uint2(cw[0], cw[1]);
}

// ------------------------------------------------------------------------------- backward
struct StemBwdArgs2 {
  const void* img;
  const long long* idx;
  float nsc[3], nbi[3];
  const bf16_t* wk;      // [64][SKP] packed weights (the forward's)
  const bf16_t* pdy;     // [N][PH][PW][64] pooled gradient
  const uint8_t* code;   // [N][PH][PW][64] window position, 15 = masked
  const float* coef;     // [3][64] a, b, cc
  float* dslab;          // [grid][64][SKH]
  int N, nimg;
  StemGeo G;
};

constexpr int PRING = 3;  // pooled-row ring: rows i, i+1 in use, i+2 staged (i+3 in flight)
constexpr int BROWS = 4;  // raw rows staged at once in the backward

template <int DT>
__global__ void __launch_bounds__(SNT, 1) stem_bwd_kernel(StemBwdArgs2 a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const StemGeo G = a.G;
  unsigned char* Ws = smem;                                  // [64][SWP] bf16
  unsigned char* E = Ws + SCO * SWP * 2;                     // [RING][Wout][24]
  unsigned char* T = E + RING * G.ROWB;                      // [2][Wout][64]: a dz, then dy
  bf16_t* S = reinterpret_cast<bf16_t*>(T + 2 * G.Wout * 128);  // [BROWS][SP]
  const int PRB = G.PW * SCO;                                // pooled row elements
  bf16_t* Pg = S + BROWS * G.SP;                             // [PRING][PW][64] grads
  uint8_t* Pc = reinterpret_cast<uint8_t*>(Pg + PRING * PRB);  // [PRING][PW][64] codes
  float* cf = reinterpret_cast<float*>(Pc + PRING * PRB);   // a, b, cc
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  {
    const int tot16 = (SCO * SWP * 2 + RING * G.ROWB + 2 * G.Wout * 128 + BROWS * G.SP * 2) / 16;
    for (int e = tid; e < tot16; e += SNT) reinterpret_cast<uint4*>(smem)[e] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  for (int e = tid; e < SCO * SKP / 8; e += SNT) {
    const int co = e / (SKP / 8), ch = e - co * (SKP / 8);
    *reinterpret_cast<uint4*>(Ws + co * SWP * 2 + ch * 16) =
        *reinterpret_cast<const uint4*>(a.wk + co * SKP + ch * 8);
  }
  if (tid < 3 * SCO) cf[tid] = a.coef[tid];
  f32x16 dacc[3];
#pragma unroll
  for (int u = 0; u < 3; ++u)
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[u][r] = 0.f;
  RawUnit ru[UPT];
  auto img_base = [&](int n) -> long long {
    long long row = a.idx ? a.idx[n] : (long long)n;
    row = row < 0 ? 0 : row >= a.nimg ? a.nimg - 1 : row;
    return row * G.Hin * G.Win * 3;
  };
  // pooled rows: PW * 8 chunks of (8 grads, 8 codes) per row; thread tid < PW*8 owns one
  const bool pl = tid < G.PW * 8;
  uint4 pg_r;
  uint2 pc_r;
  auto pload = [&](int n, int r) {
    pg_r = make_uint4(0, 0, 0, 0);
    pc_r = make_uint2(0x0f0f0f0fu, 0x0f0f0f0fu);  // rows past the image: masked windows
    if (pl && r < G.PH) {
      const long long o = (((long long)n * G.PH + r) * G.PW) * SCO + tid * 8;
      pg_r = *reinterpret_cast<const uint4*>(a.pdy + o);
      pc_r = *reinterpret_cast<const uint2*>(a.code + o);
    }
  };
  auto pstore = [&](int r) {
    if (!pl) return;
    const int s = r % PRING;
    *reinterpret_cast<uint4*>(Pg + s * PRB + tid * 8) = pg_r;
    *reinterpret_cast<uint2*>(Pc + s * PRB + tid * 8) = pc_r;
  };
  // synchronous staging of raw rows iy0 .. iy0+nr-1 (nr <= BROWS) and E rows e0 .. iy0+nr-1
  auto stage_sync = [&](int n, int iy0, int nr, int e0) {
    raw_load<DT>(ru, a.img, img_base(n), G.Hin, G.Win, iy0, nr, a.nsc, a.nbi, tid);
    raw_store(ru, S, G.SP, G.Win, nr, tid);
    __syncthreads();
    e_build(E, S, G, e0, iy0 + nr - e0, e0 - iy0, tid);
    __syncthreads();
  };
  // quad items: (qb, chunk) = pixels (2i + ddy, 2qb + ddx), ddy, ddx in {0, 1}, 8 channels
  const bool qact = tid < G.PW * 8;
  const int qb = tid >> 3, qc = tid & 7, c0 = qc * 8;
  // y MFMA (recompute), C = W x E^T: [co][px] -- wave w: slot w >> 2, px block w & 3
  const int yslot = wid >> 2, mb = wid & 3, hh = lane >> 5;
  const bool yact = 32 * mb < G.Wout;
  const int pxb = min(32 * mb + (lane & 31), G.Wout - 1);  // B column (pad lanes re-read W-1)
  const int pxo = 32 * mb + (lane & 31);                     // the output pixel of this lane
  __syncthreads();
  for (int n = blockIdx.x; n < a.N; n += gridDim.x) {
    // image prologue: E rows -3..5 (data rows 0..5 in two stagings), pooled rows 0, 1 + 2
    pload(n, 0);
    pstore(0);
    pload(n, 1);
    pstore(1);
    pload(n, 2);
    stage_sync(n, 0, 4, -3);
    stage_sync(n, 4, 2, 4);
    float ka[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ka[j] = cf[c0 + j];
    for (int i = 0; i < G.PH; ++i) {
      const bool last = i + 1 == G.PH;
      // ---------------------------------------------------------------- phase A: a dz
      if (!last) raw_load<DT>(ru, a.img, img_base(n), G.Hin, G.Win, 4 * i + 6, 4, a.nsc, a.nbi, tid);
      if (qact) {
        // the quad's 4 windows: pooled rows i (+1), columns qb (+1)
        uint4 qg[4];
        uint2 qi[4];
        unsigned ok = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int wa = w >> 1, wb = w & 1;
          ok |= (i + wa < G.PH && qb + wb < G.PW) ? 1u << w : 0u;
          const int s = (i + wa) % PRING, col = qb + wb < G.PW ? qb + wb : qb;
          qg[w] = *reinterpret_cast<const uint4*>(Pg + s * PRB + col * SCO + c0);
          qi[w] = *reinterpret_cast<const uint2*>(Pc + s * PRB + col * SCO + c0);
        }
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
          const int ddy = pp >> 1, ddx = pp & 1;
          float d[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int wa = w >> 1, wb = w & 1;
            if (wa == 1 && ddy == 0) continue;
            if (wb == 1 && ddx == 0) continue;
            if (!(ok & (1u << w))) continue;
            const uint32_t gw[4] = {qg[w].x, qg[w].y, qg[w].z, qg[w].w};
            const uint32_t aw[2] = {qi[w].x, qi[w].y};
            const unsigned code = (unsigned)((ddy ? (wa ? 0 : 2) : 1) * 3 + (ddx ? (wb ? 0 : 2) : 1));
#pragma unroll
            for (int j = 0; j < 8; ++j)
              if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == code)
                d[j] += bf2f((bf16_t)((gw[j >> 1] >> (16 * (j & 1))) & 0xffff));
          }
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = pack_bf2(ka[2 * k] * d[2 * k], ka[2 * k + 1] * d[2 * k + 1]);
          *reinterpret_cast<uint4*>(T + yoff(ddy, 2 * qb + ddx, qc, G.Wout)) = make_uint4(o[0], o[1], o[2], o[3]);
        }
      }
      // pooled row i + 2 (loaded one pair ago) into the slot of row i - 1; load row i + 3
      pstore(i + 2);
      pload(n, i + 3);
      if (!last) raw_store(ru, S, G.SP, G.Win, 4, tid);
      __syncthreads();
      // ---------------------------------------------------------------- phase B: dy
      if (yact) {
        const int oy = 2 * i + yslot;
        const int rb = 2 * oy - 3;
        f32x16 acc[2];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
        const unsigned char* wa0 = Ws + (lane & 31) * SWP * 2 + 16 * hh;
#pragma unroll
        for (int s = 0; s < 11; ++s) {
          const int j = 2 * s + hh;
          int ky = j / 3;
          const int part = j - 3 * ky;
          if (ky > 6) ky = 6;  // k-step 10's upper half: zero weights, finite data
          const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(E + ring_of(rb + ky) * G.ROWB + pxb * 48 + part * 16);
          const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(wa0 + 32 * s);
          const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(wa0 + 32 * SWP * 2 + 32 * s);
          acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bfr, acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bfr, acc[1], 0, 0, 0);
        }
        // C: col = px (lane & 31), row = co = 32 c + (r & 3) + 8 (r >> 2) + 4 hh
        if (pxo < G.Wout) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int g4 = 0; g4 < 4; ++g4) {
              const int co = 32 * c + 8 * g4 + 4 * hh;
              unsigned char* tp = T + yoff(yslot, pxo, co >> 3, G.Wout) + 2 * (co & 7);
              const uint2 t = *reinterpret_cast<const uint2*>(tp);
              const float4 bv = *reinterpret_cast<const float4*>(cf + SCO + co);
              const float4 cv = *reinterpret_cast<const float4*>(cf + 2 * SCO + co);
              const float d0 = bf2f((bf16_t)(t.x & 0xffff)) + bv.x * acc[c][4 * g4 + 0] + cv.x;
              const float d1 = bf2f((bf16_t)(t.x >> 16)) + bv.y * acc[c][4 * g4 + 1] + cv.y;
              const float d2 = bf2f((bf16_t)(t.y & 0xffff)) + bv.z * acc[c][4 * g4 + 2] + cv.z;
              const float d3 = bf2f((bf16_t)(t.y >> 16)) + bv.w * acc[c][4 * g4 + 3] + cv.w;
              *reinterpret_cast<uint2*>(tp) = make_uint2(pack_bf2(d0, d1), pack_bf2(d2, d3));
            }
        }
      }
      if (!last) e_build(E, S, G, 4 * i + 6, 4, 0, tid);
      __syncthreads();
      // ---------------------------------------------------------------- phase C: dW
      pair_wgrad(dacc, T, E, G, i, wid, lane);
      __syncthreads();
    }
  }
  float* red = reinterpret_cast<float*>(smem);
  write_wslab(dacc, red, a.dslab, wid, lane);
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
  return (size_t)SCO * SWP * 2 + (size_t)RING * G.ROWB + (size_t)2 * G.Wout * 128 +
         (size_t)SROWS * G.SP * 2;
}
static size_t bwd_smem(const StemGeo& G) {
  return (size_t)SCO * SWP * 2 + (size_t)RING * G.ROWB + (size_t)2 * G.Wout * 128 +
         (size_t)BROWS * G.SP * 2 + (size_t)PRING * G.PW * SCO * 3 + 3 * SCO * 4;
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
    stem_fwd_kernel<DT><<<grid, SNT, sm, st>>>(a);             \
  } while (0)
  if (dtype == 0) DM_SF(0);
  else if (dtype == 1) DM_SF(1);
  else DM_SF(2);
#undef DM_SF
  DM_CHECK(hipGetLastError());
}

void stem_pool_apply(const bf16_t* pext, uint8_t* code, const float* scale, const float* shift,
                     bf16_t* out, long long n, hipStream_t st) {
  const long long n8 = n / 8;
  stem_pool_apply_kernel<<<(unsigned)((n8 + 255) / 256), 256, 0, st>>>(pext, code, scale, shift,
                                                                       out, n8);
  DM_CHECK(hipGetLastError());
}

void stem_bwd_fused2(const void* img, int dtype, const long long* idx, const float* nsc,
                     const float* nbi, const bf16_t* wk, const bf16_t* pdy, const uint8_t* code,
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
  a.code = code;
  a.coef = coef;
  a.dslab = dslab;
  a.N = N;
  a.nimg = nimg;
  a.G = stem_geo(Hin, Win);
  const size_t sm = bwd_smem(a.G);
#define DM_SB(DT)                                              \
  do {                                                         \
    set_smem_attr(stem_bwd_kernel<DT>, sm);                    \
    stem_bwd_kernel<DT><<<grid, SNT, sm, st>>>(a);             \
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
