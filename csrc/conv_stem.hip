// Stem convolution on the space-to-depth input (4x4/s1 taps over 16 channels), gfx950.
//
// The ResNet stem (7x7/s2 over RGB) runs as a 4x4/s1 conv over the s2d-packed input
// [N][112][112][16] (conv_igemm.hip pack_input_s2d): M = N*112*112 output pixels, 64 output
// channels, K = 16 taps x 16 channels = 256.  The generic implicit-GEMM tiles stage one
// (4-tap, 16-channel) K-slice of the im2col matrix per step, so every input pixel is fetched
// 16 times and the weight tile is re-staged 4 times per 128 output pixels.  Here:
//
//  * a block owns 256 consecutive output pixels and stages, ONCE, (a) the whole packed weight
//    matrix [64][256] (32 KB, L2-resident across blocks) and (b) the input halo: the flattened
//    pixel rows r0-2 .. r1+1 that all 16 taps of the 256 pixels touch (<= 7 x 112 pixels x 32 B);
//  * each tap is exactly one v_mfma_f32_32x32x16_bf16 k-step (16 channels): per tap a wave
//    reads its 2 A fragments from the halo at row offset dy*W + dx (out-of-image taps read a
//    zero row = the conv's zero padding) and 2 B fragments from the resident weights;
//  * 4 waves x (64 px x 64 ch), 2 x 2 MFMA blocks each, 64 MFMAs per wave, then the shared
//    tile epilogue (BN statistics from the fp32 tile + coalesced bf16 stores).
//
// Bank layout: a weight row is 512 B (32 16-B chunks), so the 16-B chunk index is XORed with
// (row & 15): the 32 lanes of a B-fragment read (32 rows, same k) hit 16 distinct slots per
// 16-lane group.  A halo pixel is 32 B (two 16-B halves); its halves are swapped when
// (pixel >> 3) & 1, so 16 consecutive pixels reading the same half cover all 16 slots.
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int SBM = 256;        // output pixels per block
constexpr int SC = 16;          // input channels (s2d: 4 x RGB padded to 16)
constexpr int SCO = 64;         // output channels
constexpr int SK = 256;         // K = 16 taps x 16 channels
constexpr int SHP = 8 * 112;    // halo pixel capacity (W = 112: <= 4 + 3 rows; smaller W: more rows)
constexpr unsigned SOOB = 0x80000000u;

__device__ __forceinline__ int wswz(int row, int chunk) { return chunk ^ (row & 15); }
__device__ __forceinline__ int hswz(int pix, int half) { return half ^ ((pix >> 3) & 1); }

// Persistent: two workgroups per CU loop over the 256-pixel tiles.  The 32 KB weight
// matrix is staged ONCE per workgroup (the per-tile kernel re-reads it from L2 for every one
// of the 25088 tiles at batch 512: as many bytes as the conv writes), and the input halo of
// tile i+1 is loaded into registers while tile i runs its MFMAs and epilogue.  The epilogue
// stages the fp32 tile in two 128-row bands in the LDS after the weights (the halo's space),
// so weights + halo/epilogue still fit two workgroups per CU.
__device__ __forceinline__ void stem_tile_geom(const ConvGeom& g, long long m0, int dymin, int dymax,
                                               int& hbase, int& hp) {
  const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
  const long long mlast = (m0 + SBM - 1 < g.M) ? m0 + SBM - 1 : g.M - 1;
  const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
  hbase = (r0 + dymin) * g.W;
  hp = (r1 - r0 + 1 + dymax - dymin) * g.W;
}

__global__ void __launch_bounds__(256, 2) stem_conv_pers_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, int ntiles) {
  constexpr int HI = (2 * SHP + 255) / 256;
  constexpr size_t RBYTES = (size_t)(SHP + 1) * SC * 2 > (size_t)128 * (SCO + 4) * 4
                                ? (size_t)(SHP + 1) * SC * 2
                                : (size_t)128 * (SCO + 4) * 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Ws = reinterpret_cast<bf16_t*>(smem);                        // [64][256]
  unsigned char* R = smem + SCO * SK * 2;                              // halo | epilogue band
  bf16_t* Hs = reinterpret_cast<bf16_t*>(R);                           // [SHP + 1][16]
  int4* taps = reinterpret_cast<int4*>(R + RBYTES);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntaps = g.nth * g.ntw;
  const int NHW = g.N * g.H * g.W;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    taps[tid] = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * SC,
                          dy * g.W + dx);
  }
  const int dymin = g.dys > 0 ? g.dy0 : g.dy0 + (g.nth - 1) * g.dys;
  const int dymax = g.dys > 0 ? g.dy0 + (g.nth - 1) * g.dys : g.dy0;
  const auto rsx = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)xbytes, 0x00020000);
  uint4 hv[HI];
  auto load_halo = [&](int tile) {
    int hbase, hp;
    stem_tile_geom(g, (long long)tile * SBM, dymin, dymax, hbase, hp);
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int e = tid + 256 * i, pix = e >> 1, half = e & 1;
      const int gp = hbase + pix;
      const bool ok = pix < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? ((unsigned)gp * SC + half * 8) * 2u : SOOB;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsx, off, 0, 0);
      hv[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  int tile = blockIdx.x;
  {
    uint4 wv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, row = e >> 5, ch = e & 31;
      wv[i] = *reinterpret_cast<const uint4*>(Wp + row * SK + ch * 8);
    }
    load_halo(tile);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i, row = e >> 5, ch = e & 31;
      *reinterpret_cast<uint4*>(Ws + row * SK + wswz(row, ch) * 8) = wv[i];
    }
  }
  const int h = lane >> 5;  // k half: channels 8h..8h+7 of the tap
  for (; tile < ntiles; tile += gridDim.x) {
    const long long m0 = (long long)tile * SBM;
    int hbase, hp;
    stem_tile_geom(g, m0, dymin, dymax, hbase, hp);
    __syncthreads();  // the previous tile's epilogue has finished reading the LDS band
#pragma unroll
    for (int i = 0; i < HI; ++i) {
      const int e = tid + 256 * i, pix = e >> 1, half = e & 1;
      if (pix < SHP) *reinterpret_cast<uint4*>(Hs + pix * SC + hswz(pix, half) * 8) = hv[i];
    }
    if (tid < 2) *reinterpret_cast<uint4*>(Hs + SHP * SC + tid * 8) = make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (tile + (int)gridDim.x < ntiles) load_halo(tile + gridDim.x);  // lands during this tile
    int a_h[2], a_x[2], a_y[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const long long m = m0 + wid * 64 + i * 32 + (lane & 31);
      const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
      a_x[i] = (int)((unsigned)m - r * (unsigned)g.W);
      const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
      a_y[i] = (m < g.M) ? (int)(r - n * (unsigned)g.H) : -(1 << 28);
      a_h[i] = (int)(m - hbase);
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    auto frags = [&](int t, bf16x8 (&af)[2], bf16x8 (&bf)[2]) {
      const int4 tp = taps[t];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = (unsigned)(a_x[i] + tp.y) < (unsigned)g.W &&
                        (unsigned)(a_y[i] + tp.x) < (unsigned)g.H;
        const int pix = ok ? a_h[i] + tp.w : SHP;
        af[i] = *reinterpret_cast<const bf16x8*>(Hs + pix * SC + hswz(pix, h) * 8);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int row = j * 32 + (lane & 31);
        bf[j] = *reinterpret_cast<const bf16x8*>(Ws + row * SK + wswz(row, (tp.z >> 3) + h) * 8);
      }
    };
    bf16x8 a0[2], b0[2], a1[2], b1[2];
    auto mma = [&](const bf16x8 (&af)[2], const bf16x8 (&bf)[2]) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    };
    frags(0, a0, b0);
#pragma unroll
    for (int t = 0; t < 16; t += 2) {
      frags(t + 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0);
      if (t + 2 < 16) frags(t + 2, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1);
    }
    __syncthreads();  // the epilogue band overwrites the halo
    mfma_tile_epilogue<SBM, SCO, 4, 1, true, 2>(acc, R, m0, 0, tile, stats, g, Y, nullptr);
  }
}

// ------------------------------------------------------------------ fused stem backward
// Weight gradient of the s2d stem with the stem's BatchNorm backward applied on the fly:
//
//   dW[co][tap*16 + c] = Σ_m dy[m][co] · xs[m + off(tap)][c]
//   dy = a·dz + b·y + cc      dz = max-pool gradient gathered at its argmax pixels, masked
//                              by relu(y·sc + sh) (3x3/s2/p1 pool over even H, W)
//
// The unfused path writes dy at full resolution (bn_bwd_apply_quad: read y + pooled grad +
// codes, write dy) and the wgrad re-reads it; here each block walks image row PAIRS
// (2 x W pixels = the W/2 pooling quads of one pooled row band), gathers dz for every quad
// exactly as bn_bwd_apply_quad does (4 pixels share their 4 candidate windows), writes the
// bf16 dy tile straight into LDS (bit-identical to the unfused dy), stages the 5 input rows
// the 4x4 taps touch, and reduces over the pair's pixels with v_mfma_f32_16x16x32_bf16 from
// transposed LDS reads (ds_read_b64_tr_b16), as wgrad_halo.hip.  dy never reaches memory.
// 8 waves: wave w owns kernel row w & 3 (4 taps) x output channels 32*(w >> 2) .. +31 x 16
// input channels; one quad item (4 pixels x 8 channels) per thread.  The next row pair's
// loads are in flight while the current one computes.  One block per CU (512 threads hold
// the staging registers of a whole row pair); blocks own contiguous ranges of row pairs and
// write fp32 slabs [block][64][256] (fixed-order reduce after).
struct StemBwdArgs {
  const bf16_t* xs;     // [N][H][W][16] s2d input
  const bf16_t* y;      // [N][H][W][64] raw stem conv output
  const bf16_t* pdy;    // [N][H/2][W/2][64] max-pool output gradient
  const uint8_t* pidx;  // argmax codes (kh*3 + kw), same shape
  const float* coef;    // [3][64] a, b, cc of dy = a·dz + b·y + cc
  const float* sc;      // forward BN scale / shift (ReLU mask)
  const float* sh;
  float* slab;          // [gridDim.x][64][256]
  int N, H, W;
  int spb;              // row pairs per block
};

__device__ __forceinline__ void s_unpack8(const uint4& v, float f[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f[2 * k] = bf2f((bf16_t)(w[k] & 0xffff));
    f[2 * k + 1] = bf2f((bf16_t)(w[k] >> 16));
  }
}

typedef short s4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s4v tr_read4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v*)p);
}

constexpr int FW = 112;        // widest row supported (ResNet stem at 224: 112)
constexpr int FDP = 80;        // dY tile pitch (elements, 160 B rows: conflict-free tr reads)
constexpr int FR = 2 * FW;     // pixel rows per row pair
constexpr int FXH = 5 * FW;    // input halo pixels (rows y0-2 .. y0+2)
constexpr int FWP = FW + 3;    // padded halo row: 2 zero pixels left, 1 right (x = -2 .. W)

// Per row pair the work is mostly VALU (the quad gather + BN apply of 4 x 8 values per thread
// and, in the first version, ~60 address instructions per MFMA k-step), so the loop keeps the
// VALU side lean: the halo rows carry zero pad columns (every 4x4 tap read is in bounds, the
// zero padding comes from the pads and from the zero rows outside the image), every LDS
// address of the k-loop is a per-lane base + a compile-time offset, and the global offsets
// are 32-bit (all tensors < 2^31 elements, checked by stem_wgrad_fused_supported).
// ------------------------------------------------------------------ warp-specialised kernel
// The VALU-heavy dy construction (quad gather + BN apply, ~70 % of a single-role kernel's
// cycles, where every wave alternated building dy and reducing it) and the MFMA reduction run
// in different waves.  Waves 0-7 (producers) build the dy tile of pair s+1 while waves 8-11
// (consumers) reduce pair s; the tiles (dy and the input halo) are double-buffered in LDS
// and one barrier per pair hands them over.  Waves w, w+4 and w+8 share a SIMD (a
// workgroup's waves go to the SIMDs cyclically), so every SIMD runs two producers (one
// producer alone cannot hide its own VALU / LDS latencies) beside one consumer.  Measured:
// 4 + 4 waves 478 us, 8 + 4 420, 8 + 8 438 (128-VGPR budget: 1-deep y prefetch).
//   producers: one quad item per thread; its y rows are loaded two pairs ahead; the pooled
//              gradient rows come from a 3-slot LDS ring
//   consumers: wave 8 + t owns kernel row t, all 64 output channels x 4 taps x 16 channels
//              (16 accumulators); they also stage the next pair's halo and the pooled
//              gradient rows into LDS
__global__ void __launch_bounds__(768) stem_wgrad_ws_kernel(StemBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Ds0 = reinterpret_cast<bf16_t*>(smem);  // [2][FR][FDP] dy tiles
  bf16_t* Xs0 = Ds0 + 2 * FR * FDP;               // [2][5][FWP][16] padded halos
  // pooled-gradient rows in a PSL-slot ring: pair s reads pooled rows s and s + 1 (global
  // row index = pair index); the consumers store row s + 3 while pair s + 1 is being built
  // (loaded one iteration earlier, so a whole iteration covers its latency)
  constexpr int PSL = 4;
  bf16_t* Gs = Xs0 + 2 * 5 * FWP * SC;                            // [PSL][FW / 2 * 64] grads
  uint8_t* Is = reinterpret_cast<uint8_t*>(Gs + PSL * (FW / 2) * 64);  // [PSL][FW / 2 * 64] codes
  float* cf = reinterpret_cast<float*>(Is + PSL * (FW / 2) * 64);  // [3][64] a, b, cc
  constexpr int DSZ = FR * FDP, XSZ = 5 * FWP * SC, GSZ = (FW / 2) * 64;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int W = a.W, H = a.H, W2 = W >> 1, H2 = H >> 1;
  const int R = 2 * W, nks = (R + 31) >> 5;
  const int WP = W + 3;
  const long long total = (long long)a.N * H2;
  const long long s0 = (long long)blockIdx.x * a.spb;
  const long long s1 = s0 + a.spb < total ? s0 + a.spb : total;
  const int np = s1 > s0 ? (int)(s1 - s0) : 0;

  for (int i = tid; i < 2 * DSZ / 8; i += 768)
    reinterpret_cast<uint4*>(Ds0)[i] = make_uint4(0, 0, 0, 0);  // rows >= R stay zero
  for (int i = tid; i < 2 * XSZ / 8; i += 768)
    reinterpret_cast<uint4*>(Xs0)[i] = make_uint4(0, 0, 0, 0);  // pad columns stay zero
  for (int c = tid; c < 64; c += 768) {
    cf[c] = a.coef[c];
    cf[64 + c] = a.coef[64 + c];
    cf[128 + c] = a.coef[128 + c];
  }
  const unsigned npix = (unsigned)a.N * H * W, npool = (unsigned)a.N * H2 * W2;
  __syncthreads();

  if (wid < 8) {
    // ---------------------------------------------------------------- producers
    const auto ry = __builtin_amdgcn_make_buffer_rsrc((void*)a.y, (short)0, (int)(npix * 128u), 0x00020000);
    const int nitems = W2 * 8;
    struct Item {
      uint4 qy[4];
    };
    auto load = [&](Item& I, int it, long long s) {
      if (it >= nitems) return;
      const int chunk = it & 7, qb = it >> 3;
      const int n = (int)(s / H2), qa = (int)(s - (long long)n * H2);
      const unsigned pix0 = ((unsigned)n * H + 2 * qa) * W + 2 * qb;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(
            ry, (pix0 + (p >> 1) * W + (p & 1)) * 128u + chunk * 16u, 0, 0);
        I.qy[p] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    };
    // dz gathered from the pooled gradient (masked windows carry code 15), dy = a dz + b y + cc
    auto store = [&](const Item& I, int it, long long s, bf16_t* Ds) {
      if (it >= nitems) return;
      const int chunk = it & 7, qb = it >> 3, c0 = chunk * 8;
      const int qa = (int)(s % H2);
      // the quad's 4 windows: pooled rows s (+1), columns qb (+1); masked off the image
      uint4 qg[4];
      uint2 qi[4];
      unsigned ok = 0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const int wa = w >> 1, wb = w & 1;
        ok |= (qa + wa < H2 && qb + wb < W2) ? 1u << w : 0u;
        const int slot = (int)((s + wa) % PSL), col = qb + wb < W2 ? qb + wb : qb;
        qg[w] = *reinterpret_cast<const uint4*>(Gs + slot * GSZ + col * 64 + c0);
        qi[w] = *reinterpret_cast<const uint2*>(Is + slot * GSZ + col * 64 + c0);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int ddy = p >> 1, ddx = p & 1;
        float d[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const int wa = w >> 1, wb = w & 1;
          if (wa == 1 && ddy == 0) continue;
          if (wb == 1 && ddx == 0) continue;
          if (!(ok & (1u << w))) continue;
          float gg[8];
          s_unpack8(qg[w], gg);
          const uint32_t aw[2] = {qi[w].x, qi[w].y};
          const unsigned code = (unsigned)((ddy ? (wa ? 0 : 2) : 1) * 3 + (ddx ? (wb ? 0 : 2) : 1));
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == code) d[j] += gg[j];
        }
        float yv[8];
        s_unpack8(I.qy[p], yv);
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const float4 ca = *reinterpret_cast<const float4*>(cf + c0 + 4 * h);
          const float4 cb = *reinterpret_cast<const float4*>(cf + 64 + c0 + 4 * h);
          const float4 cc = *reinterpret_cast<const float4*>(cf + 128 + c0 + 4 * h);
          const float av[4] = {ca.x, ca.y, ca.z, ca.w}, bv[4] = {cb.x, cb.y, cb.z, cb.w};
          const float cv[4] = {cc.x, cc.y, cc.z, cc.w};
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int j0 = 4 * h + 2 * k;
            o[2 * h + k] = pack_bf2(av[2 * k] * d[j0] + bv[2 * k] * yv[j0] + cv[2 * k],
                                    av[2 * k + 1] * d[j0 + 1] + bv[2 * k + 1] * yv[j0 + 1] + cv[2 * k + 1]);
          }
        }
        const int lp = ddy * W + 2 * qb + ddx;
        *reinterpret_cast<uint4*>(Ds + lp * FDP + c0) = make_uint4(o[0], o[1], o[2], o[3]);
      }
    };
    // one quad item per producer thread; y of pair s sits in register set (s - s0) & 1 and is
    // loaded two pairs ahead
    const int it = tid;
    Item A0, A1;
    if (np > 0) load(A0, it, s0);
    if (np > 1) load(A1, it, s0 + 1);
    __syncthreads();  // pooled rows s0 .. s0 + 2 staged
    if (np > 0) {
      store(A0, it, s0, Ds0);
      if (np > 2) load(A0, it, s0 + 2);
    }
    __syncthreads();
    auto step = [&](int i, Item& A) {
      if (i + 1 < np) {
        bf16_t* Dn = Ds0 + ((i + 1) & 1) * DSZ;
        const long long sn = s0 + i + 1;
        store(A, it, sn, Dn);
        if (i + 3 < np) load(A, it, sn + 2);
      }
      __syncthreads();
    };
    for (int i = 0; i < np; i += 2) {
      step(i, A1);
      if (i + 1 < np) step(i + 1, A0);
    }
    return;
  }
  // ------------------------------------------------------------------ consumers
  const int ct = tid - 512;  // 0..255
  const int th = wid - 8;    // kernel row of this wave: dy = th - 2
  const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)a.xs, (short)0, (int)(npix * 32u), 0x00020000);
  constexpr int XC = (2 * FXH + 255) / 256;  // halo pieces per consumer thread
  int xh_row[XC], xh_lds[XC];
#pragma unroll
  for (int i = 0; i < XC; ++i) {
    const int e = ct + 256 * i, pix = e >> 1;
    const int hr = pix / W, x = pix - hr * W;
    xh_row[i] = pix < 5 * W ? hr : 1 << 20;
    xh_lds[i] = ((hr * WP + x + 2) * SC + (e & 1) * 8) * 2;
  }
  uint4 xv[XC];
  // pooled row r (global index; rows past the tensor read as zeros): 448 16-B grad pieces and
  // 448 8-B code pieces, two of each per consumer thread
  const auto rg = __builtin_amdgcn_make_buffer_rsrc((void*)a.pdy, (short)0, (int)(npool * 128u), 0x00020000);
  const auto ri = __builtin_amdgcn_make_buffer_rsrc((void*)a.pidx, (short)0, (int)(npool * 64u), 0x00020000);
  const int npc = W2 * 8;  // pieces per pooled row
  uint4 pg[2];
  uint2 pi[2];
  auto pload = [&](long long r) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = ct + 256 * u;
      const unsigned off = (unsigned)r * (unsigned)npc + (unsigned)e;  // piece index
      const bool ok = e < npc && r < total;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rg, ok ? off * 16u : 0x80000000u, 0, 0);
      pg[u] = make_uint4(v[0], v[1], v[2], v[3]);
      const auto w = __builtin_amdgcn_raw_buffer_load_b64(ri, ok ? off * 8u : 0x80000000u, 0, 0);
      pi[u] = make_uint2(w[0], w[1]);
    }
  };
  auto pstore = [&](long long r) {
    const int slot = (int)(r % PSL);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = ct + 256 * u;
      if (e < npc) {
        *reinterpret_cast<uint4*>(Gs + slot * GSZ + e * 8) = pg[u];
        *reinterpret_cast<uint2*>(Is + slot * GSZ + e * 8) = pi[u];
      }
    }
  };
  auto xload = [&](long long s) {
    const int n = (int)(s / H2), qa = (int)(s - (long long)n * H2);
    const int ylo = 2 - 2 * qa, yhi = H + 2 - 2 * qa;
    const unsigned xb = ((unsigned)n * H + 2 * qa - 2) * (unsigned)W * 32u;
#pragma unroll
    for (int i = 0; i < XC; ++i) {
      xv[i] = make_uint4(0, 0, 0, 0);
      if (xh_row[i] >= ylo && xh_row[i] < yhi) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rx, xb + (ct + 256 * i) * 16u, 0, 0);
        xv[i] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    }
  };
  auto xstore = [&](bf16_t* Xs) {
#pragma unroll
    for (int i = 0; i < XC; ++i)
      if (xh_row[i] < 5)
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned char*>(Xs) + xh_lds[i]) = xv[i];
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int rbase = grp * 4 + q;
  auto xrow = [&](const bf16_t* Xs, int r) -> const bf16_t* {
    if (r >= R) r = 0;  // dy rows past the pair are zero: any in-bounds halo pixel will do
    const int rr = r >= W ? 1 : 0;
    return Xs + ((rr + th) * WP + (r - rr * W)) * SC + 4 * pp;
  };
  struct Frag {
    bf16x8 af[4], bf[4];
  };
  auto frag = [&](Frag& F, const bf16_t* Ds, const bf16_t* Xs, int ks) {
    const bf16_t* dk = Ds + (ks * 32 + rbase) * FDP + 4 * pp;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s4v lo = tr_read4(dk + i * 16);
      const s4v hi = tr_read4(dk + 16 * FDP + i * 16);
      F.af[i] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
    const bf16_t* x0 = xrow(Xs, ks * 32 + rbase);
    const bf16_t* x1 = xrow(Xs, ks * 32 + rbase + 16);
#pragma unroll
    for (int tw = 0; tw < 4; ++tw) {
      const s4v lo = tr_read4(x0 + tw * SC);
      const s4v hi = tr_read4(x1 + tw * SC);
      F.bf[tw] = (bf16x8){lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  };
  auto mma = [&](const Frag& F) {
#pragma unroll
    for (int tw = 0; tw < 4; ++tw)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i][tw] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(F.af[i], F.bf[tw], acc[i][tw], 0, 0, 0);
  };
  if (np > 0) {
#pragma unroll 1
    for (int r = 0; r < 3; ++r) {
      pload(s0 + r);
      pstore(s0 + r);
    }
    if (np > 2) pload(s0 + 3);
  }
  __syncthreads();  // pooled rows s0 .. s0 + 2 staged
  if (np > 0) {
    xload(s0);
    xstore(Xs0);
    if (np > 1) xload(s0 + 1);
  }
  __syncthreads();
  Frag F0;
  for (int i = 0; i < np; ++i) {
    // pooled row s0 + i + 3 (loaded one iteration ago) goes to the slot of row s0 + i - 1,
    // last read in iteration i - 2; the producers of iteration i + 1 read it.  Row s0 + i + 4
    // is loaded now and stored next iteration.
    if (i + 2 < np) pstore(s0 + i + 3);
    if (i + 3 < np) pload(s0 + i + 4);
    if (i + 1 < np) {
      xstore(Xs0 + ((i + 1) & 1) * XSZ);  // that buffer was last read in iteration i - 1
      if (i + 2 < np) xload(s0 + i + 2);
    }
    const bf16_t* Ds = Ds0 + (i & 1) * DSZ;
    const bf16_t* Xs = Xs0 + (i & 1) * XSZ;
    // one fragment set (the registers go to the producers' share); the two producer waves
    // on this SIMD cover the LDS latency
    for (int ks = 0; ks < nks; ++ks) {
      frag(F0, Ds, Xs, ks);
      mma(F0);
    }
    __syncthreads();
  }
  // slab[b][co][tap*16 + c]; 16x16 C map: col = lane & 15 (channel), row = (lane>>4)*4 + r (co)
  float* out = a.slab + (long long)blockIdx.x * 64 * SK;
  const int c = lane & 15;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int tw = 0; tw < 4; ++tw)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = i * 16 + (lane >> 4) * 4 + r;
        out[(long long)co * SK + (th * 4 + tw) * SC + c] = acc[i][tw][r];
      }
}

}  // namespace

bool stem_conv_supported(const ConvGeom& g) {
  if (g.C != SC || g.Ncols != SCO || g.wK != SK || g.nth * g.ntw != 16) return false;
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W || g.OC != SCO) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  const int span = (g.nth - 1) * (g.dys < 0 ? -g.dys : g.dys);
  // worst-case halo over blocks: a 256-pixel run starting at the last pixel of a row
  const int rows = (g.W - 1 + SBM - 1) / g.W + 1 + span;
  return rows * g.W <= SHP && (g.dxs == 1 || g.dxs == -1);
}

bool stem_wgrad_fused_supported(int N, int H, int W, int C, int Cpad) {
  return C == 64 && Cpad == SC && H % 2 == 0 && W % 2 == 0 && W <= FW && H >= 2 &&
         (long long)N * H * W * 64 < (1LL << 31);
}

// one 768-thread workgroup per CU (256 row-pair slices); each slice's slab is 64 KB
int stem_wgrad_fused_blocks(int N, int H) {
  const long long pairs = (long long)N * (H / 2);
  const long long b = pairs < 256 ? pairs : 256;
  const long long spb = (pairs + b - 1) / b;
  return (int)((pairs + spb - 1) / spb);
}

void stem_wgrad_fused(const bf16_t* xs, const bf16_t* y, const bf16_t* pdy, const uint8_t* pidx,
                      const float* coef, const float* sc, const float* sh, float* slab, int N,
                      int H, int W, int S, hipStream_t st) {
  const long long pairs = (long long)N * (H / 2);
  StemBwdArgs a{xs, y, pdy, pidx, coef, sc, sh, slab, N, H, W, (int)((pairs + S - 1) / S)};
  const size_t sm = (size_t)2 * FR * FDP * 2 + (size_t)2 * 5 * FWP * SC * 2 +
                    (size_t)4 * (FW / 2) * 64 * 3 + 3 * 64 * 4;
  set_smem_attr(stem_wgrad_ws_kernel, sm);
  stem_wgrad_ws_kernel<<<S, 768, sm, st>>>(a);
  DM_CHECK(hipGetLastError());
}

void stem_conv(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, float* stats, const ConvGeom& g,
               hipStream_t st) {
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const int ntiles = (int)((g.M + SBM - 1) / SBM);
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    DM_CHECK(hipGetDevice(&dev));
    DM_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const size_t hal = (size_t)(SHP + 1) * SC * 2, band = (size_t)128 * (SCO + 4) * 4;
  const size_t smp = (size_t)SCO * SK * 2 + (hal > band ? hal : band) + MAXTAPS * 16;
  set_smem_attr(stem_conv_pers_kernel, smp);
  const int grid = ntiles < 2 * cus ? ntiles : 2 * cus;
  stem_conv_pers_kernel<<<grid, 256, smp, st>>>(X, Wp, Y, stats, g, xb, ntiles);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
