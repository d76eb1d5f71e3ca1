// BatchNorm (train-mode batch statistics), fused BN-apply/residual/ReLU, BN backward,
// max/avg pooling and input packing — NHWC bf16, 16-B vectorised (8 channels/lane).
//
// Forward BN statistics are produced by the conv epilogue (conv_igemm.hip) as
// per-row-tile slabs [T][2][C]; here they are reduced in two fixed-order passes
// (deterministic) and turned into per-channel scale/shift plus the running-stat
// update (PyTorch semantics: unbiased variance for running_var, momentum 0.1).
// BN backward is two memory passes: a reduction of Σdz and Σdz·x̂ (dz = ReLU-masked
// upstream grad) and an apply pass dy = a·dz + b·y + c that also emits the residual
// branch gradient dz when the block has a skip connection.
#include "common.h"

#include <cstdlib>

namespace dm {

__device__ __forceinline__ void unpack8(const uint4& v, float f[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f[2 * q] = bf2f((bf16_t)(w[q] & 0xffff));
    f[2 * q + 1] = bf2f((bf16_t)(w[q] >> 16));
  }
}
__device__ __forceinline__ uint4 pack8(const float f[8]) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]),
                    pack_bf2(f[6], f[7]));
}

// ------------------------------------------------------------------ slab column reduce
// Fixed-order (deterministic) reductions of per-tile partial rows [T][W] fp32.  Every
// lane keeps 8 independent loads in flight: these reductions are latency-bound chains
// otherwise (a 6272-row slab summed one dependent load at a time costs ~40 us).
__device__ __forceinline__ double sum_rows8(const float* __restrict__ p, int r, int rend, int step,
                                            long long W) {
  double acc = 0.0;
  for (; r + 7 * step < rend; r += 8 * step) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = p[(long long)(r + j * step) * W];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += v[j];
  }
  for (; r < rend; r += step) acc += p[(long long)r * W];
  return acc;
}

// in: [T][W] -> out: [G][W] (G = gridDim.y); group gi sums rows [gi*R, (gi+1)*R), R = ceil(T/G)
__global__ void __launch_bounds__(256) slab_colsum_kernel(const float* __restrict__ in, int T,
                                                          int W, float* __restrict__ out) {
  const int G = gridDim.y, gi = blockIdx.y;
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;  // 4 row lanes
  const int R = (T + G - 1) / G;
  const int r0 = gi * R, r1 = min(T, r0 + R);
  __shared__ double red[4][64];
  red[rl][threadIdx.x & 63] = col < W ? sum_rows8(in + col, r0 + rl, r1, 4, W) : 0.0;
  __syncthreads();
  if (rl == 0 && col < W)
    out[(long long)gi * W + col] = (float)(red[0][threadIdx.x] + red[1][threadIdx.x] +
                                           red[2][threadIdx.x] + red[3][threadIdx.x]);
}

// Σ over the G rows of part[G][2C] for channels c (Σ) and C+c (second moment): NT/CH row
// lanes x CH channels per block, 8 loads in flight per lane, lanes combined in a fixed order
// (groups of RLN/16 lanes, then the 16 groups); the result is valid in threads 0..CH-1
// (channel blockIdx.x*CH + threadIdx.x).  CH = 4 (64 row lanes) sums up to fin_direct_rows()
// rows without the slab_colsum pre-pass: one dependent launch fewer per finalize, in 4-wave
// blocks (a 1024-thread block waited for a whole free CU next to the side stream: 23 us)
constexpr int FIN_CH = 16;
template <int NT, int CH>
__device__ __forceinline__ void block_sum2(const float* __restrict__ part, int G, int C, int c,
                                           double& s, double& q) {
  constexpr int RLN = NT / CH;
  __shared__ double red[2][RLN][CH];
  const int rl = threadIdx.x / CH, cl = threadIdx.x % CH;
  const long long W = 2LL * C;
  red[0][rl][cl] = c < C ? sum_rows8(part + c, rl, G, RLN, W) : 0.0;
  red[1][rl][cl] = c < C ? sum_rows8(part + C + c, rl, G, RLN, W) : 0.0;
  __syncthreads();
  if constexpr (RLN > 16) {
    // first level: 16 groups of RLN/16 consecutive lanes, in order
    constexpr int PER = RLN / 16;
    double a = 0.0, b = 0.0;
    if (threadIdx.x < 16 * CH) {
#pragma unroll
      for (int l = 0; l < PER; ++l) {
        a += red[0][rl * PER + l][cl];
        b += red[1][rl * PER + l][cl];
      }
    }
    __syncthreads();
    if (threadIdx.x < 16 * CH) {
      red[0][rl][cl] = a;
      red[1][rl][cl] = b;
    }
    __syncthreads();
  }
  s = 0.0;
  q = 0.0;
  if (threadIdx.x < CH)
    for (int l = 0; l < 16; ++l) {
      s += red[0][l][cl];
      q += red[1][l][cl];
    }
}

// rows a 4-channel finalize block sums directly (DMLAB_FIN_DIRECT, default 2048; 256 = the
// round-4 path: slab_colsum pre-pass above 256 rows)
static int fin_direct_rows() {
  static const int v = [] {
    const char* e = getenv("DMLAB_FIN_DIRECT");
    return e ? atoi(e) : 2048;
  }();
  return v;
}

// level-1 groups for a [T][2C] slab: none when the finalize block can sum it directly
static inline int colsum_groups(int T) {
  return (T <= 256 || T <= fin_direct_rows()) ? 0 : min(256, (T + 31) / 32);
}

// Per-channel finalize math of the forward / backward finalize kernels (the one-launch
// last-block finalizes measured slower and were removed: docs/KERNELS.md round 2).
struct FinFwd {
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  float momentum, eps;
  float* scale;
  float* shift;
  float* mean_out;
  float* invstd_out;
  long long* num_batches;
};
struct FinBwd {
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float gbeta;
  float* coef;
};

__device__ __forceinline__ void fin_fwd_channel(const FinFwd& f, int c, double s, double q,
                                                double count) {
  const double mean = s / count;
  double var = q / count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + f.eps));
  const float sc = f.gamma[c] * invstd;
  f.scale[c] = sc;
  f.shift[c] = f.beta[c] - (float)mean * sc;
  f.mean_out[c] = (float)mean;
  f.invstd_out[c] = invstd;
  if (f.rmean) {
    const double unbiased = count > 1 ? var * count / (count - 1) : var;
    f.rmean[c] = (1.f - f.momentum) * f.rmean[c] + f.momentum * (float)mean;
    f.rvar[c] = (1.f - f.momentum) * f.rvar[c] + f.momentum * (float)unbiased;
  }
}

__device__ __forceinline__ void fin_bwd_channel(const FinBwd& f, int c, int C, double s, double q,
                                                double count) {
  f.dbeta[c] = (f.gbeta != 0.f ? f.gbeta * f.dbeta[c] : 0.f) + (float)s;
  f.dgamma[c] = (f.gbeta != 0.f ? f.gbeta * f.dgamma[c] : 0.f) + (float)q;
  const float a = f.gamma[c] * f.invstd[c];
  const float inv_m = (float)(1.0 / count);
  const float b = -a * f.invstd[c] * (float)q * inv_m;
  const float cc = -a * (float)s * inv_m - b * f.mean[c];
  f.coef[c] = a;
  f.coef[C + c] = b;
  f.coef[2 * C + c] = cc;
}

// stats: [G][2][C] partial (Σy, Σy²) -> scale/shift, mean/invstd; running stats update.
// grid ceil(C/16) x 256 threads
template <int NT, int CH>
__global__ void __launch_bounds__(NT) bn_finalize_kernel(const float* __restrict__ part, int G,
                                                         int C, double count, FinFwd f) {
  const int c = blockIdx.x * CH + (threadIdx.x % CH);
  if (f.num_batches && blockIdx.x == 0 && threadIdx.x == 0) *f.num_batches += 1;
  double s, q;
  block_sum2<NT, CH>(part, G, C, c, s, q);
  if (threadIdx.x >= CH || c >= C) return;
  fin_fwd_channel(f, c, s, q, count);
}

// eval mode: scale/shift from running stats
__global__ void bn_eval_coeffs_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rmean, const float* __restrict__ rvar,
                                      float eps, int C, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rvar[c] + eps);
  scale[c] = gamma[c] * inv;
  shift[c] = beta[c] - rmean[c] * gamma[c] * inv;
}

// out = [relu](y*scale + shift [+ res])
// mask (optional, RELU only): one bit per element, (out > 0) of the stored bf16 value, one
// byte per 8-channel chunk -- the BN backward's ReLU mask source for residual layers
// (mode 4) at 1/16 of the bytes of re-reading `out`.
__device__ __forceinline__ uint32_t pos_bits8(const uint4& v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t b = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t lo = w[q] & 0xffff, hi = w[q] >> 16;
    b |= (uint32_t)(!(lo & 0x8000) && (lo & 0x7fff)) << (2 * q);
    b |= (uint32_t)(!(hi & 0x8000) && (hi & 0x7fff)) << (2 * q + 1);
  }
  return b;
}

// Streaming passes: block b covers U*256 consecutive 16-B chunks (no grid stride: the
// dispatcher balances the blocks) and the loads/stores are non-temporal (the activation
// tensors of a batch-1024 step exceed the 256 MB MALL; keeping them out of L2/MALL leaves
// those to the kernels that reuse data).  At 1024x56x56x64 the residual apply runs at
// 6.4 TB/s against 4.5 for the earlier grid-strided, cached version (torch's add: 6.0), and
// the step gains 1.9 % with the backward passes done the same way
// (profiles/bn_apply_variants_r4x.jsonl, profiles/bn_stream_variants_ab_r4z.txt).
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld16(const bf16_t* p, long long i) {
  if constexpr (NT) {
    const u32x4v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p) + i);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return reinterpret_cast<const uint4*>(p)[i];
  }
}
template <bool NT>
__device__ __forceinline__ void st16(bf16_t* p, long long i, const uint4& o) {
  if constexpr (NT) {
    u32x4v v;
    v.x = o.x; v.y = o.y; v.z = o.z; v.w = o.w;
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(p) + i);
  } else {
    reinterpret_cast<uint4*>(p)[i] = o;
  }
}
// out = [relu](y*scale + shift [+ res])
// mask (optional, RELU only): one bit per element, (out > 0) of the stored bf16 value, one
// byte per 8-channel chunk -- the BN backward's ReLU mask source for residual layers
// (mode 4) at 1/16 of the bytes of re-reading `out`.
template <bool RES, bool RELU, int U = 4, bool NT = true>
__global__ void __launch_bounds__(256) bn_apply_kernel(const bf16_t* __restrict__ y,
                                                            const bf16_t* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            bf16_t* __restrict__ out, long long n8,
                                                            int C, uint8_t* __restrict__ mask) {
  extern __shared__ float sc_sh[];  // [2][C]
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    sc_sh[i] = scale[i];
    sc_sh[C + i] = shift[i];
  }
  __syncthreads();
  const long long i0 = (long long)blockIdx.x * (U * 256) + threadIdx.x;
  const int C8 = C >> 3;
  uint4 yr[U], rr[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * 256 < n8 ? i0 + u * 256 : 0;
    yr[u] = ld16<NT>(y, i);
    if (RES) rr[u] = ld16<NT>(res, i);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * 256;
    if (i >= n8) continue;
    const int c0 = (int)((unsigned long long)i & (unsigned)(C8 - 1)) * 8;
    float f[8], r[8];
    unpack8(yr[u], f);
    if (RES) unpack8(rr[u], r);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = f[j] * sc_sh[c0 + j] + sc_sh[C + c0 + j];
      if (RES) v += r[j];
      if (RELU) v = fmaxf(v, 0.f);
      f[j] = v;
    }
    const uint4 o = pack8(f);
    st16<NT>(out, i, o);
    if (RELU && mask) mask[i] = (uint8_t)pos_bits8(o);
  }
}

// ------------------------------------------------------------------ BN backward
// dz = upstream grad with the ReLU mask; sources (template MODE):
//   0  dout tensor, no ReLU
//   1  dout tensor, mask from the saved output (out > 0)          -- residual layers
//   2  dout tensor, mask recomputed from y (y*scale + shift > 0)   -- no `out` read
//   3  gathered from a following 3x3/s2 max-pool's grads + argmax codes, mask from y
//      (stem: neither `out` nor the unpooled gradient is ever materialised)
//   4  dout tensor, mask from the forward's 1-bit (out > 0) mask    -- residual layers
struct BnBwdArgs {
  const bf16_t* dout;
  const bf16_t* out;
  const bf16_t* y;
  const float* mean;
  const float* invstd;
  const float* scale;   // forward BN scale/shift (modes 2, 3)
  const float* shift;
  const bf16_t* pdy;    // mode 3: pooled-output gradient [N][OH][OW][C]
  const uint8_t* pidx;  //         argmax codes (kh*K + kw), same shape
  int H, W, OH, OW, K, S, P;
  long long M;
  int C;
  const uint8_t* mask;  // mode 4: bit j of byte i = (out > 0) of chunk i, channel j
};

// mode 3: dz of one 8-channel chunk of input pixel r, gathered from the pool windows
// that contain it.  For K <= 2S a pixel lies in at most 2 x 2 windows: all candidate
// (codes, grads) are loaded up front — 8 independent loads instead of a chain of
// dependent ones — then matched against the pixel's position in each window.
__device__ __forceinline__ void gather_pool_dz(const BnBwdArgs& a, long long r, int chunk, int C8,
                                               float d[8]) {
  const unsigned ru = (unsigned)r;  // pixel counts < 2^31: 32-bit divisions
  const unsigned tq = ru / (unsigned)a.W;
  const int iw = (int)(ru - tq * (unsigned)a.W);
  const int n = (int)(tq / (unsigned)a.H);
  const int ih = (int)(tq - (unsigned)n * (unsigned)a.H);
#pragma unroll
  for (int j = 0; j < 8; ++j) d[j] = 0.f;
  const int oh_lo = max(0, (ih + a.P - a.K + a.S) / a.S), oh_hi = min(a.OH - 1, (ih + a.P) / a.S);
  const int ow_lo = max(0, (iw + a.P - a.K + a.S) / a.S), ow_hi = min(a.OW - 1, (iw + a.P) / a.S);
  if (a.K <= 2 * a.S) {
    uint2 ix[4];
    uint4 gv[4];
    bool ok[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int oh = oh_lo + (w >> 1), ow = ow_lo + (w & 1);
      ok[w] = oh <= oh_hi && ow <= ow_hi;
      const long long o = (((long long)n * a.OH + min(oh, oh_hi)) * a.OW + min(ow, ow_hi)) * C8 + chunk;
      ix[w] = reinterpret_cast<const uint2*>(a.pidx)[o];
      gv[w] = reinterpret_cast<const uint4*>(a.pdy)[o];
    }
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (!ok[w]) continue;
      const int oh = oh_lo + (w >> 1), ow = ow_lo + (w & 1);
      const unsigned code = (ih - (oh * a.S - a.P)) * a.K + (iw - (ow * a.S - a.P));
      const uint32_t aw[2] = {ix[w].x, ix[w].y};
      float g[8];
      unpack8(gv[w], g);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == code) d[j] += g[j];
    }
    return;
  }
  for (int oh = oh_lo; oh <= oh_hi; ++oh)
    for (int ow = ow_lo; ow <= ow_hi; ++ow) {
      const unsigned code = (ih - (oh * a.S - a.P)) * a.K + (iw - (ow * a.S - a.P));
      const long long o = (((long long)n * a.OH + oh) * a.OW + ow) * C8 + chunk;
      const uint2 ix = reinterpret_cast<const uint2*>(a.pidx)[o];
      const uint32_t aw[2] = {ix.x, ix.y};
      float g[8];
      unpack8(reinterpret_cast<const uint4*>(a.pdy)[o], g);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == code) d[j] += g[j];
    }
}

// Raw operands of U grid-strided 8-channel chunks i0 + u*stride, all loads issued before
// any is consumed (memory-level parallelism: these kernels are pure HBM streams).
template <int MODE, int U>
struct BnBwdBatch {
  uint4 y[U], dout[U], out[U];
  uint32_t mk[U];
  bool ok[U];
  template <bool NT = false>
  __device__ __forceinline__ void load(const BnBwdArgs& a, long long i0, long long stride,
                                       long long n8) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = i0 + u * stride;
      ok[u] = i < n8;
      const long long ii = ok[u] ? i : 0;
      y[u] = ld16<NT>(a.y, ii);
      if (MODE != 3) dout[u] = ld16<NT>(a.dout, ii);
      if (MODE == 1) out[u] = ld16<NT>(a.out, ii);
      if (MODE == 4) mk[u] = a.mask[ii];
    }
  }
  // dz (upstream grad with the ReLU mask) and y of chunk u
  __device__ __forceinline__ void dz(const BnBwdArgs& a, int u, long long i, int chunk, int C8,
                                     const float* sc, const float* sh, float d[8],
                                     float yv[8]) const {
    unpack8(y[u], yv);
    if (MODE == 3) gather_pool_dz(a, (long long)((unsigned long long)i >> (31 - __builtin_clz(C8))), chunk, C8, d);
    else unpack8(dout[u], d);
    if (MODE == 1) {
      float o[8];
      unpack8(out[u], o);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = o[j] > 0.f ? d[j] : 0.f;
    } else if (MODE == 4) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = (mk[u] >> j) & 1u ? d[j] : 0.f;
    } else if (MODE >= 2) {
      const int c0 = chunk * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = (yv[j] * sc[c0 + j] + sh[c0 + j]) > 0.f ? d[j] : 0.f;
    }
  }
};

// grid (G); block 256; thread t owns channel chunk t % C8 of the rows ≡ t / C8 (mod 256 / C8)
template <int MODE, int UU = 4, bool NT = false>
__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(BnBwdArgs a, float* __restrict__ part) {
  constexpr int U = MODE == 3 ? 2 : UU;
  extern __shared__ float red[];  // [256][16] partials, then [2][C] scale/shift
  const int C = a.C, C8 = C >> 3;
  float* sc = red + 256 * 16;
  float* sh = sc + C;
  if (MODE == 2 || MODE == 3)
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      sc[c] = a.scale[c];
      sh[c] = a.shift[c];
    }
  __syncthreads();
  const int chunk = threadIdx.x % C8;
  const int rl = threadIdx.x / C8;
  const int RL = blockDim.x / C8;
  const int c0 = chunk * 8;
  float mu[8], is[8], s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = a.mean[c0 + j];
    is[j] = a.invstd[c0 + j];
    s[j] = 0.f;
    q[j] = 0.f;
  }
  // chunk index i = r*C8 + chunk; rows strided by gridDim.x*RL keep the channel fixed
  const long long n8 = a.M * C8;
  const long long rstride = (long long)gridDim.x * RL;
  const long long stride = rstride * C8;
  for (long long i0 = ((long long)blockIdx.x * RL + rl) * C8 + chunk; i0 < n8; i0 += U * stride) {
    BnBwdBatch<MODE, U> bt;
    bt.template load<NT>(a, i0, stride, n8);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!bt.ok[u]) continue;
      float d[8], yv[8];
      bt.dz(a, u, i0 + u * stride, chunk, C8, sc, sh, d, yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] += d[j];
        q[j] += d[j] * (yv[j] - mu[j]) * is[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x * 16 + j] = s[j];
    red[threadIdx.x * 16 + 8 + j] = q[j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < C8 * 16; e += blockDim.x) {
    const int ch = e / 16, j = e % 16;
    float acc = 0.f;
    for (int l = 0; l < RL; ++l) acc += red[(l * C8 + ch) * 16 + j];
    const int c = ch * 8 + (j & 7);
    part[(long long)blockIdx.x * 2 * C + (j < 8 ? 0 : C) + c] = acc;
  }
}

// finalize: Σ over G partials -> dgamma, dbeta (written with beta-accumulate into grad
// slots) and the affine dy coefficients a, b, c.  grid ceil(C/16) x 256 threads.
template <int NT, int CH>
__global__ void __launch_bounds__(NT) bn_bwd_finalize_kernel(const float* __restrict__ part,
                                                             int G, int C, double count,
                                                             FinBwd f) {
  const int c = blockIdx.x * CH + (threadIdx.x % CH);
  double s, q;
  block_sum2<NT, CH>(part, G, C, c, s, q);
  if (threadIdx.x >= CH || c >= C) return;
  fin_bwd_channel(f, c, C, s, q, count);
}

// dy = a·dz + b·y + c ; optional dres = dz
template <int MODE, bool DRES, int UU = 4, bool FLAT = false, bool NT = false>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(BnBwdArgs a, const float* __restrict__ coef,
                                                           bf16_t* __restrict__ dy,
                                                           bf16_t* __restrict__ dres) {
  constexpr int U = MODE == 3 ? 2 : UU;
  extern __shared__ float cf[];  // [3][C] coefficients, [2][C] forward scale/shift
  const int C = a.C, C8 = C >> 3;
  for (int i = threadIdx.x; i < 3 * C; i += blockDim.x) cf[i] = coef[i];
  float* sc = cf + 3 * C;
  float* sh = sc + C;
  if (MODE == 2 || MODE == 3)
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      sc[c] = a.scale[c];
      sh[c] = a.shift[c];
    }
  __syncthreads();
  const long long n8 = a.M * C8;
  // FLAT: block b covers U*256 consecutive chunks (no grid stride); else grid-strided
  const long long stride = FLAT ? (long long)blockDim.x : (long long)gridDim.x * blockDim.x;
  // With C8 | blockDim (C <= 2048) a thread's channel chunk never changes across the
  // grid-stride loop: its 24 coefficients live in registers instead of being re-read
  // from LDS per element (lanes 8 floats apart: the kernel's LDS bank conflicts).
  const bool hoist = (blockDim.x % C8) == 0;
  float ka[8], kb[8], kc[8];
  if (hoist) {
    const int c0 = (threadIdx.x & (C8 - 1)) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ka[j] = cf[c0 + j];
      kb[j] = cf[C + c0 + j];
      kc[j] = cf[2 * C + c0 + j];
    }
  }
  const long long ib = FLAT ? (long long)blockIdx.x * U * blockDim.x : (long long)blockIdx.x * blockDim.x;
  for (long long i0 = ib + threadIdx.x; i0 < n8; i0 += FLAT ? n8 : U * stride) {
    BnBwdBatch<MODE, U> bt;
    bt.template load<NT>(a, i0, stride, n8);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!bt.ok[u]) continue;
      const long long i = i0 + u * stride;
      const int chunk = (int)((unsigned long long)i & (unsigned)(C8 - 1));
      const int c0 = chunk * 8;
      float d[8], yv[8];
      bt.dz(a, u, i, chunk, C8, sc, sh, d, yv);
      if (DRES) st16<NT>(dres, i, pack8(d));
      float r[8];
      if (hoist) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] = ka[j] * d[j] + kb[j] * yv[j] + kc[j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          r[j] = cf[c0 + j] * d[j] + cf[C + c0 + j] * yv[j] + cf[2 * C + c0 + j];
      }
      st16<NT>(dy, i, pack8(r));
    }
  }
}

// ------------------------------------------------------------------ stem BN backward, quads
// 3x3/s2/p1 max-pool after the stem (even H, W): the 2x2 pixel quad (2qa+dy, 2qb+dx) is
// covered by exactly the pooled windows (qa+wa, qb+wb), wa, wb in {0, 1}; pixel row dy=0
// lies in window row 1 of wa=0 only, dy=1 in row 2 of wa=0 and row 0 of wa=1 (same for
// columns).  One thread handles a quad x 8 channels: the 4 pooled gradients + argmax codes
// are loaded once for 4 pixels (the per-pixel gather loaded them for every pixel: 4x the
// L2 traffic, which bound those passes at ~2.4 TB/s).
struct QuadPool {
  uint4 y[4];
  uint4 gv[4];
  uint2 ix[4];
  bool ok[4];
  float d[4][8];
  long long pix0;
  // issue every load of quad q (8 channels `chunk`); consumed by finish()
  __device__ __forceinline__ void load(const BnBwdArgs& a, unsigned q, int chunk, int C8) {
    const int W2 = a.W >> 1, H2 = a.H >> 1;
    const unsigned qb = q % (unsigned)W2;
    const unsigned t = q / (unsigned)W2;
    const unsigned qa = t % (unsigned)H2;
    const unsigned n = t / (unsigned)H2;
    pix0 = ((long long)n * a.H + 2 * qa) * a.W + 2 * qb;
#pragma unroll
    for (int p = 0; p < 4; ++p)
      y[p] = reinterpret_cast<const uint4*>(a.y)[(pix0 + (p >> 1) * a.W + (p & 1)) * C8 + chunk];
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const unsigned oh = qa + (w >> 1), ow = qb + (w & 1);
      ok[w] = oh < (unsigned)a.OH && ow < (unsigned)a.OW;
      const long long o = (((long long)n * a.OH + (ok[w] ? oh : qa)) * a.OW + (ok[w] ? ow : qb)) * C8 + chunk;
      ix[w] = reinterpret_cast<const uint2*>(a.pidx)[o];
      gv[w] = reinterpret_cast<const uint4*>(a.pdy)[o];
    }
  }
  // d[p] = ReLU-masked gradient of pixel p gathered from the windows whose argmax it is
  __device__ __forceinline__ void finish(int chunk, const float* sc, const float* sh) {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int j = 0; j < 8; ++j) d[p][j] = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (!ok[w]) continue;
      const int wa = w >> 1, wb = w & 1;
      float g[8];
      unpack8(gv[w], g);
      const uint32_t aw[2] = {ix[w].x, ix[w].y};
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int dy = p >> 1, dx = p & 1;
        if (wa == 1 && dy == 0) continue;  // pixel row outside the window
        if (wb == 1 && dx == 0) continue;
        const unsigned code = (unsigned)((dy ? (wa ? 0 : 2) : 1) * 3 + (dx ? (wb ? 0 : 2) : 1));
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == code) d[p][j] += g[j];
      }
    }
    const int c0 = chunk * 8;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float yv[8];
      unpack8(y[p], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[p][j] = (yv[j] * sc[c0 + j] + sh[c0 + j]) > 0.f ? d[p][j] : 0.f;
    }
  }
};

__global__ void __launch_bounds__(256) bn_bwd_reduce_quad_kernel(BnBwdArgs a, float* __restrict__ part) {
  extern __shared__ float red[];  // [256][16] partials, then [2][C] scale/shift
  const int C = a.C, C8 = C >> 3;
  float* sc = red + 256 * 16;
  float* sh = sc + C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sc[c] = a.scale[c];
    sh[c] = a.shift[c];
  }
  __syncthreads();
  const int chunk = threadIdx.x % C8, rl = threadIdx.x / C8, RL = blockDim.x / C8;
  const int c0 = chunk * 8;
  float mu[8], is[8], s[8], qq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mu[j] = a.mean[c0 + j];
    is[j] = a.invstd[c0 + j];
    s[j] = 0.f;
    qq[j] = 0.f;
  }
  const unsigned nq = (unsigned)(a.M >> 2);
  const unsigned qs = gridDim.x * RL;
  // two quads in flight per thread (all 24 loads issued before either is consumed)
  for (unsigned q = blockIdx.x * RL + rl; q < nq; q += 2 * qs) {
    QuadPool qp[2];
    const bool two = q + qs < nq;
    qp[0].load(a, q, chunk, C8);
    qp[1].load(a, two ? q + qs : q, chunk, C8);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && !two) break;
      qp[u].finish(chunk, sc, sh);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        float yv[8];
        unpack8(qp[u].y[p], yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] += qp[u].d[p][j];
          qq[j] += qp[u].d[p][j] * (yv[j] - mu[j]) * is[j];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[threadIdx.x * 16 + j] = s[j];
    red[threadIdx.x * 16 + 8 + j] = qq[j];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < C8 * 16; e += blockDim.x) {
    const int ch = e / 16, j = e % 16;
    float acc = 0.f;
    for (int l = 0; l < RL; ++l) acc += red[(l * C8 + ch) * 16 + j];
    const int c = ch * 8 + (j & 7);
    part[(long long)blockIdx.x * 2 * C + (j < 8 ? 0 : C) + c] = acc;
  }
}

__global__ void __launch_bounds__(256) bn_bwd_apply_quad_kernel(BnBwdArgs a, const float* __restrict__ coef,
                                                                bf16_t* __restrict__ dy) {
  extern __shared__ float cf[];  // [3][C] coefficients, [2][C] forward scale/shift
  const int C = a.C, C8 = C >> 3;
  for (int i = threadIdx.x; i < 3 * C; i += blockDim.x) cf[i] = coef[i];
  float* sc = cf + 3 * C;
  float* sh = sc + C;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    sc[c] = a.scale[c];
    sh[c] = a.shift[c];
  }
  __syncthreads();
  const unsigned n8 = (unsigned)((a.M >> 2) * C8);
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int chunk = (int)(i & (unsigned)(C8 - 1));
    const unsigned q = i >> (31 - __builtin_clz(C8));
    QuadPool qp;
    qp.load(a, q, chunk, C8);
    qp.finish(chunk, sc, sh);
    const int c0 = chunk * 8;
    const long long pix0 = qp.pix0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float yv[8], r[8];
      unpack8(qp.y[p], yv);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        r[j] = cf[c0 + j] * qp.d[p][j] + cf[C + c0 + j] * yv[j] + cf[2 * C + c0 + j];
      reinterpret_cast<uint4*>(dy)[(pix0 + (p >> 1) * a.W + (p & 1)) * C8 + chunk] = pack8(r);
    }
  }
}

// Fused stem tail: pooled = maxpool_KxK/S(relu(y*scale + shift)) with argmax codes; the
// BN output itself is never written.
// yarg (optional): the raw conv output y at each window's argmax.  The stem's BN-backward
// sums Σdz, Σdz·x̂ then reduce over the POOLED grid (pooled grad masked by relu at the
// argmax, x̂ from yarg) instead of gathering over the full-resolution y: 2 pooled-size
// tensors instead of y + pooled grad + codes (~2.7x fewer bytes); same terms, regrouped.
__global__ void __launch_bounds__(256) bn_relu_maxpool_kernel(
    const bf16_t* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    bf16_t* __restrict__ out, uint8_t* __restrict__ idx, bf16_t* __restrict__ yarg, int N, int H,
    int W, int C, int OH, int OW, int K, int S, int P) {
  extern __shared__ float ss[];  // [2][C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    ss[c] = scale[c];
    ss[C + c] = shift[c];
  }
  __syncthreads();
  const int C8 = C >> 3;
  const long long total = (long long)N * OH * OW * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const unsigned iu = (unsigned)i;  // element counts < 2^31: 32-bit index math
    const int c8 = (int)(iu % (unsigned)C8);
    unsigned t = iu / (unsigned)C8;
    const int ow = (int)(t % (unsigned)OW);
    t /= (unsigned)OW;
    const int oh = (int)(t % (unsigned)OH);
    const int n = (int)(t / (unsigned)OH);
    const int c0 = c8 * 8;
    float best[8], raw[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; raw[j] = 0.f; }
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - P + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * S - P + kw;
        if (iw < 0 || iw >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(y + (((long long)n * H + ih) * W + iw) * C + c0), f);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = fmaxf(f[j] * ss[c0 + j] + ss[C + c0 + j], 0.f);
          if (v > best[j]) { best[j] = v; arg[j] = kh * K + kw; raw[j] = f[j]; }
        }
      }
    }
    reinterpret_cast<uint4*>(out)[i] = pack8(best);
    if (yarg) reinterpret_cast<uint4*>(yarg)[i] = pack8(raw);  // raw is bf16-exact
    // a window whose max is 0 (every BN value <= 0) passes no gradient: its ReLU mask at
    // the argmax is 0.  Code 15 (no window position) says so, so the backward gathers need
    // no mask of their own (the stem's fused weight-gradient kernel relies on this)
#pragma unroll
    for (int j = 0; j < 8; ++j) arg[j] = best[j] > 0.f ? arg[j] : 15;
    uint2 a2;
    a2.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    a2.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = a2;
  }
}

// The stem's 3x3/s2/p1 case of bn_relu_maxpool_kernel: a thread owns two horizontally
// adjacent pooled outputs (they share one input column: 15 loads instead of 18) and issues
// all 15 16-B loads before any compare (the generic kernel's guarded loop keeps only a few
// in flight).  Same scan order and strict '>' (first max wins), same codes and yarg.
template <bool NT>
__global__ void __launch_bounds__(256) bn_relu_maxpool3s2_kernel(
    const bf16_t* __restrict__ y, const float* __restrict__ scale, const float* __restrict__ shift,
    bf16_t* __restrict__ out, uint8_t* __restrict__ idx, bf16_t* __restrict__ yarg, int N, int H,
    int W, int C, int OH, int OW) {
  extern __shared__ float ss[];  // [2][C]
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    ss[c] = scale[c];
    ss[C + c] = shift[c];
  }
  __syncthreads();
  const unsigned C8 = (unsigned)(C >> 3), OWP = (unsigned)((OW + 1) >> 1);
  const unsigned total = (unsigned)N * (unsigned)OH * OWP * C8;  // < 2^31 (host check)
  const unsigned stride = gridDim.x * blockDim.x;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % C8);
    unsigned t = i / C8;
    const int owp = (int)(t % OWP);
    t /= OWP;
    const int oh = (int)(t % (unsigned)OH);
    const int n = (int)(t / (unsigned)OH);
    const int c0 = c8 * 8, ow0 = owp * 2;
    const bool two = ow0 + 1 < OW;
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = ss[c0 + j];
      sh[j] = ss[C + c0 + j];
    }
    // rows 2oh-1..2oh+1, columns 2ow0-1..2ow0+3; an out-of-image tap loads the (always
    // valid) window centre and is skipped in the compare
    const unsigned ctr = (((unsigned)n * H + 2 * oh) * W + 2 * ow0) * C + c0;
    uint4 v[3][5];
    bool ok[3][5];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        const int iw = 2 * ow0 - 1 + q;
        ok[kh][q] = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W && (q < 3 || two);
        const unsigned off = ok[kh][q] ? (((unsigned)n * H + ih) * W + iw) * C + c0 : ctr;
        v[kh][q] = *reinterpret_cast<const uint4*>(y + off);
      }
    }
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      if (o == 1 && !two) break;
      float best[8], raw[8];
      int arg[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; raw[j] = 0.f; }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int q = 2 * o + kw;
          if (!ok[kh][q]) continue;
          float f[8];
          unpack8(v[kh][q], f);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float val = fmaxf(f[j] * sc[j] + sh[j], 0.f);
            if (val > best[j]) { best[j] = val; arg[j] = kh * 3 + kw; raw[j] = f[j]; }
          }
        }
      const unsigned oi = (((unsigned)n * OH + oh) * OW + ow0 + o) * C8 + c8;
      st16<NT>(out, oi, pack8(best));
      if (yarg) st16<NT>(yarg, oi, pack8(raw));
#pragma unroll
      for (int j = 0; j < 8; ++j) arg[j] = best[j] > 0.f ? arg[j] : 15;
      uint2 a2;
      a2.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
      a2.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
      reinterpret_cast<uint2*>(idx)[oi] = a2;
    }
  }
}

// ------------------------------------------------------------------ max pool (NHWC)
// out[n,oh,ow,c] = max window; idx = argmax position in window (0..K*K-1), first max wins
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, int N, int H,
                                                          int W, int C, int OH, int OW, int K,
                                                          int S, int P) {
  const int C8 = C >> 3;
  const long long total = (long long)N * OH * OW * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const unsigned iu = (unsigned)i;  // element counts < 2^31: 32-bit index math
    const int c8 = (int)(iu % (unsigned)C8);
    unsigned t = iu / (unsigned)C8;
    const int ow = (int)(t % (unsigned)OW);
    t /= (unsigned)OW;
    const int oh = (int)(t % (unsigned)OH);
    const int n = (int)(t / (unsigned)OH);
    float best[8];
    int arg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { best[j] = -INFINITY; arg[j] = 0; }
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh * S - P + kh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow * S - P + kw;
        if (iw < 0 || iw >= W) continue;
        float f[8];
        unpack8(*reinterpret_cast<const uint4*>(x + (((long long)n * H + ih) * W + iw) * C + c8 * 8), f);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (f[j] > best[j]) { best[j] = f[j]; arg[j] = kh * K + kw; }
      }
    }
    reinterpret_cast<uint4*>(y)[i] = pack8(best);
    uint2 a;
    a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24);
    a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = a;
  }
}

// dx[n,ih,iw,c] = Σ_{windows (oh,ow) containing (ih,iw) whose argmax is (ih,iw)} dy
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx,
                                                          bf16_t* __restrict__ dx, int N, int H,
                                                          int W, int C, int OH, int OW, int K,
                                                          int S, int P) {
  const int C8 = C >> 3;
  const long long total = (long long)N * H * W * C8;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const unsigned iu = (unsigned)i;
    const int c8 = (int)(iu % (unsigned)C8);
    unsigned t = iu / (unsigned)C8;
    const int iw = (int)(t % (unsigned)W);
    t /= (unsigned)W;
    const int ih = (int)(t % (unsigned)H);
    const int n = (int)(t / (unsigned)H);
    float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // output windows covering ih: oh in [ceil((ih+P-K+1)/S), floor((ih+P)/S)]
    const int oh_lo = max(0, (ih + P - K + S) / S), oh_hi = min(OH - 1, (ih + P) / S);
    const int ow_lo = max(0, (iw + P - K + S) / S), ow_hi = min(OW - 1, (iw + P) / S);
    for (int oh = oh_lo; oh <= oh_hi; ++oh)
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int code = (ih - (oh * S - P)) * K + (iw - (ow * S - P));
        const long long o = (((long long)n * OH + oh) * OW + ow) * C8 + c8;
        const uint2 a = reinterpret_cast<const uint2*>(idx)[o];
        float d[8];
        unpack8(reinterpret_cast<const uint4*>(dy)[o], d);
        const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (((aw[j >> 2] >> (8 * (j & 3))) & 0xff) == (uint32_t)code) g[j] += d[j];
      }
    reinterpret_cast<uint4*>(dx)[i] = pack8(g);
  }
}

// ------------------------------------------------------------------ global average pool
// x [N][HW][C] -> y [N][C] (bf16), fp32 accumulation; one block per (n, 8-channel group)
// One thread per (image, 8-channel chunk) sums its HW pixels in order, 7 loads in flight
// (consecutive threads read consecutive 16-B chunks of a pixel row).  The previous
// block-per-(image, chunk) tree reduction ran 32768 blocks of 256 threads with 49 busy
// threads each and 8 barriers: 40 us for 26 MB at batch 512.
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ y, int N, int HW,
                                                          int C) {
  const int C8 = C >> 3;
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)N * C8) return;
  const int n = (int)(t / C8), c = (int)(t % C8) * 8;
  const bf16_t* px = x + (long long)n * HW * C + c;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int p = 0;
  for (; p + 7 <= HW; p += 7) {
    uint4 v[7];
#pragma unroll
    for (int u = 0; u < 7; ++u) v[u] = *reinterpret_cast<const uint4*>(px + (long long)(p + u) * C);
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      float f[8];
      unpack8(v[u], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
  for (; p < HW; ++p) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(px + (long long)p * C), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] += f[j];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] /= HW;
  *reinterpret_cast<uint4*>(y + (long long)n * C + c) = pack8(s);
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          bf16_t* __restrict__ dx, int N, int HW,
                                                          int C) {
  const int C8 = C >> 3;
  const long long total = (long long)N * HW * C8;
  const float inv = 1.f / HW;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = i % C8;
    const int n = (i / C8) / HW;
    float d[8];
    unpack8(reinterpret_cast<const uint4*>(dy)[(long long)n * C8 + c8], d);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= inv;
    reinterpret_cast<uint4*>(dx)[i] = pack8(d);
  }
}

// ------------------------------------------------------------------ input packing
// x: fp32 or bf16 with arbitrary NCHW strides (sn, sc, sh, sw in elements) -> NHWC bf16,
// channels zero-padded to Cp (multiple of 8)
template <typename T>
__global__ void __launch_bounds__(256) pack_input_kernel(const T* __restrict__ x,
                                                         bf16_t* __restrict__ y, int N, int C,
                                                         int H, int W, int Cp, long long sn,
                                                         long long sc, long long sh, long long sw) {
  const long long total = (long long)N * H * W;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int w = i % W;
    long long t = i / W;
    const int h = t % H;
    const int n = t / H;
    const T* src = x + n * sn + h * sh + w * sw;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c0 + j;
        if (c < C) {
          if constexpr (sizeof(T) == 4) f[j] = src[c * sc];
          else f[j] = bf2f(src[c * sc]);
        } else {
          f[j] = 0.f;
        }
      }
      *reinterpret_cast<uint4*>(y + i * Cp + c0) = pack8(f);
    }
  }
}

// Space-to-depth input packing for the 7x7/s2 stem: (N,C,H,W) -> (N,H/2,W/2,Cp) with
// channel (dy*2+dx)*C + c holding x[n, c, 2i+dy, 2j+dx]; the stem then runs as a
// 4x4/s1 conv over 4C (<= Cp) channels: K = 16*16 = 256 instead of 49*8 = 392
// (padded to 448), and every tap is one contiguous 32-B channel vector.
// idx (optional): output image n is source row idx[n] of a device-resident dataset (the
// data loader's gather fused into the packing pass; clamped to [0, nsrc)).
__device__ __forceinline__ long long s2d_src_row(const long long* idx, long long n, long long nsrc) {
  if (idx == nullptr) return n;
  const long long r = idx[n];
  return r < 0 ? 0 : (r >= nsrc ? nsrc - 1 : r);
}

template <typename T>
__global__ void __launch_bounds__(256) pack_input_s2d_kernel(const T* __restrict__ x,
                                                             bf16_t* __restrict__ y, int N, int C,
                                                             int H2, int W2, int Cp, long long sn,
                                                             long long sc, long long sh,
                                                             long long sw,
                                                             const long long* __restrict__ idx,
                                                             long long nsrc) {
  const long long total = (long long)N * H2 * W2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int j = i % W2;
    long long t = i / W2;
    const int r = t % H2;
    const int n = t / H2;
    for (int c0 = 0; c0 < Cp; c0 += 8) {
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int ch = c0 + q;
        const int sub = ch / C, c = ch % C;
        if (sub < 4) {
          const int dy = sub >> 1, dx = sub & 1;
          const T v = x[s2d_src_row(idx, n, nsrc) * sn + c * sc + (2 * r + dy) * sh + (2 * j + dx) * sw];
          if constexpr (sizeof(T) == 4) f[q] = v;
          else f[q] = bf2f(v);
        } else {
          f[q] = 0.f;
        }
      }
      *reinterpret_cast<uint4*>(y + i * Cp + c0) = pack8(f);
    }
  }
}

// Fast path of the stem packing for the common input: fp32 channels_last RGB
// (c stride 1, x stride 3, row stride 3W) into Cp = 16.  A thread owns two adjacent output
// pixels (2q, 2q+1) of row r: their 2 x 4 source pixels are 12 contiguous floats (48 B,
// 16-B aligned) in each of the source rows 2r and 2r+1 -> 6 float4 loads and one 64-B run
// of bf16 stores, instead of 24 scalar loads.
__global__ void __launch_bounds__(256) pack_input_s2d_cl3_kernel(const float* __restrict__ x,
                                                                 bf16_t* __restrict__ y, int N,
                                                                 int H2, int W2, long long sn,
                                                                 const long long* __restrict__ idx,
                                                                 long long nsrc) {
  const int Q = W2 >> 1;
  const long long total = (long long)N * H2 * Q;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long rowf = (long long)W2 * 2 * 3;  // floats per source row
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int q = (int)(i % Q);
    const long long t = i / Q;
    const int r = (int)(t % H2);
    const int n = (int)(t / H2);
    const float* a = x + s2d_src_row(idx, n, nsrc) * sn + (long long)(2 * r) * rowf + 12LL * q;
    float A[12], B[12];
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      const float4 fa = reinterpret_cast<const float4*>(a)[v];
      const float4 fb = reinterpret_cast<const float4*>(a + rowf)[v];
      A[4 * v] = fa.x; A[4 * v + 1] = fa.y; A[4 * v + 2] = fa.z; A[4 * v + 3] = fa.w;
      B[4 * v] = fb.x; B[4 * v + 1] = fb.y; B[4 * v + 2] = fb.z; B[4 * v + 3] = fb.w;
    }
    uint4* o = reinterpret_cast<uint4*>(y + ((long long)(n * H2 + r) * W2 + 2 * q) * 16);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      // channel (dy*2 + dx)*3 + c  <-  source (2r+dy, 2(2q+p)+dx, c); 12..15 zero
      const float* ra = A + 6 * p;
      const float* rb = B + 6 * p;
      const float lo[8] = {ra[0], ra[1], ra[2], ra[3], ra[4], ra[5], rb[0], rb[1]};
      const float hi[8] = {rb[2], rb[3], rb[4], rb[5], 0.f, 0.f, 0.f, 0.f};
      o[2 * p] = pack8(lo);
      o[2 * p + 1] = pack8(hi);
    }
  }
}

// ------------------------------------------------------------------ launchers
void pack_input_s2d(const void* x, bool bf16, bf16_t* y, int N, int C, int H2, int W2, int Cp,
                    long long sn, long long sc, long long sh, long long sw, const long long* idx,
                    long long nsrc, hipStream_t st) {
  const long long total = (long long)N * H2 * W2;
  if (!bf16 && C == 3 && Cp == 16 && sc == 1 && sw == 3 && sh == 3LL * 2 * W2 && W2 % 2 == 0 &&
      ((uintptr_t)x & 15) == 0 && sn % 4 == 0) {
    // (non-temporal loads/stores measured slower here: the step's two alternating input
    // batches partly stay in the MALL, profiles/nt_pack_stem_bwd_rejected_r4ad.txt)
    pack_input_s2d_cl3_kernel<<<grid_for(total / 2, 256, 8192), 256, 0, st>>>(
        (const float*)x, y, N, H2, W2, sn, idx, nsrc);
    return;
  }
  if (bf16)
    pack_input_s2d_kernel<bf16_t><<<grid_for(total, 256, 8192), 256, 0, st>>>(
        (const bf16_t*)x, y, N, C, H2, W2, Cp, sn, sc, sh, sw, idx, nsrc);
  else
    pack_input_s2d_kernel<float><<<grid_for(total, 256, 8192), 256, 0, st>>>(
        (const float*)x, y, N, C, H2, W2, Cp, sn, sc, sh, sw, idx, nsrc);
}

void bn_stats_finalize(const float* stats, int T, int C, double count, const float* gamma,
                       const float* beta, float* rmean, float* rvar, float momentum, float eps,
                       float* scale, float* shift, float* mean, float* invstd, float* work,
                       long long* num_batches, hipStream_t st) {
  const int W = 2 * C;
  const int G = colsum_groups(T);
  const FinFwd f{gamma, beta, rmean, rvar, momentum, eps, scale, shift, mean, invstd, num_batches};
  const float* fin = stats;
  if (G) {
    slab_colsum_kernel<<<dim3((W + 63) / 64, G), 256, 0, st>>>(stats, T, W, work);
    fin = work;
  }
  const int rows = G ? G : T;
  if (rows > 256)
    bn_finalize_kernel<256, 4><<<(C + 3) / 4, 256, 0, st>>>(fin, rows, C, count, f);
  else
    bn_finalize_kernel<256, FIN_CH><<<(C + FIN_CH - 1) / FIN_CH, 256, 0, st>>>(fin, rows, C, count, f);
}

void bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                    float eps, int C, float* scale, float* shift, hipStream_t st) {
  bn_eval_coeffs_kernel<<<(C + 255) / 256, 256, 0, st>>>(gamma, beta, rmean, rvar, eps, C, scale,
                                                         shift);
}

void bn_apply(const bf16_t* y, const bf16_t* res, const float* scale, const float* shift,
              bf16_t* out, long long n, int C, bool relu, hipStream_t st, uint8_t* mask) {
  const long long n8 = n / 8;
  const size_t sh = sizeof(float) * 2 * C;
  constexpr int U = 4;
  const int gf = (int)((n8 + U * 256 - 1) / (U * 256));
  if (res) {
    if (relu) bn_apply_kernel<true, true><<<gf, 256, sh, st>>>(y, res, scale, shift, out, n8, C, mask);
    else bn_apply_kernel<true, false><<<gf, 256, sh, st>>>(y, res, scale, shift, out, n8, C, nullptr);
  } else {
    if (relu) bn_apply_kernel<false, true><<<gf, 256, sh, st>>>(y, res, scale, shift, out, n8, C, mask);
    else bn_apply_kernel<false, false><<<gf, 256, sh, st>>>(y, res, scale, shift, out, n8, C, nullptr);
  }
}

int bn_bwd_groups(long long M, int C);
int bn_bwd_groups(long long M, int C) {
  const int RL = 256 / (C / 8);
  // >= 16 rows per row lane (4 batched iterations): enough workgroups to keep every CU
  // streaming on the small late layers (C 512 x 12544 rows -> 196 groups, not 49)
  long long g = (M + RL * 16 - 1) / (RL * 16);
  if (g > 2048) g = 2048;  // 4096 / 8192 measure the same (profiles/bn_bwd_groups_ab_r4ak.txt)
  if (g < 1) g = 1;
  return (int)g;
}

void bn_backward(const bf16_t* dout, const bf16_t* out, const bf16_t* y, const float* mean,
                 const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                 float gbeta, long long M, int C, int mode, const float* scale,
                 const float* shift, const bf16_t* pdy, const uint8_t* pidx, int H, int W,
                 int OH, int OW, int K, int S, int P, bf16_t* dy, bf16_t* dres, float* work,
                 hipStream_t st, const float* pre_part, int pre_rows, const uint8_t* mask) {
  // pre_part (optional): [pre_rows][2C] partial Σdz, Σdz·x̂ already reduced by the producing
  // kernel (the stem's pooled-domain sums) — the reduction pass over dout and y is skipped
  // work: [G][2C] partials + [3C] coefficients + [<=256][2C] second-level partials
  BnBwdArgs a{dout, out, y, mean, invstd, scale, shift, pdy, pidx, H, W, OH, OW, K, S, P, M, C,
              mask};
  // stem 3x3/s2/p1 pool with even H, W: quad gather (4 pixels share their 4 windows)
  const bool quad = mode == 3 && K == 3 && S == 2 && P == 1 && H % 2 == 0 && W % 2 == 0 &&
                    OH == H / 2 && OW == W / 2 && !dres && (long long)M * C / 8 < (1LL << 31);
  const int G = pre_part ? pre_rows : quad ? bn_bwd_groups(M / 4, C) : bn_bwd_groups(M, C);
  float* part = pre_part ? const_cast<float*>(pre_part) : work;
  float* coef = pre_part ? work : work + (long long)G * 2 * C;
  float* part2 = coef + 3 * C;
  const size_t shr = sizeof(float) * (256 * 16 + 2 * C);
  if (pre_part) {
  } else if (quad) bn_bwd_reduce_quad_kernel<<<G, 256, shr, st>>>(a, part);
  else switch (mode) {
    // 4 16-B chunks per operand in flight per thread (8 measured neutral for the reduce and
    // forward apply, -1.2 % for the backward apply: profiles/bn_loads_in_flight_r2c.jsonl)
    // non-temporal loads: the reduce streams its inputs once (the apply pass re-reads them
    // from HBM either way at these sizes)
    case 0: bn_bwd_reduce_kernel<0, 4, true><<<G, 256, shr, st>>>(a, part); break;
    case 1: bn_bwd_reduce_kernel<1, 4, true><<<G, 256, shr, st>>>(a, part); break;
    case 2: bn_bwd_reduce_kernel<2, 4, true><<<G, 256, shr, st>>>(a, part); break;
    case 4: bn_bwd_reduce_kernel<4, 4, true><<<G, 256, shr, st>>>(a, part); break;
    default: bn_bwd_reduce_kernel<3><<<G, 256, shr, st>>>(a, part); break;
  }
  const int G2 = colsum_groups(G);
  const FinBwd fb{gamma, mean, invstd, dgamma, dbeta, gbeta, coef};
  const float* fin = part;
  if (G2) {  // parallel fixed-order pre-reduction so the finalize sums stay short
    slab_colsum_kernel<<<dim3((2 * C + 63) / 64, G2), 256, 0, st>>>(part, G, 2 * C, part2);
    fin = part2;
  }
  const int rows = G2 ? G2 : G;
  if (rows > 256)
    bn_bwd_finalize_kernel<256, 4><<<(C + 3) / 4, 256, 0, st>>>(fin, rows, C, (double)M, fb);
  else
    bn_bwd_finalize_kernel<256, FIN_CH><<<(C + FIN_CH - 1) / FIN_CH, 256, 0, st>>>(fin, rows, C,
                                                                            (double)M, fb);
  if (!dy) return;  // coefficients only (a consumer kernel applies dy = a·dz + b·y + c itself)
  const long long n8 = M * C / 8;
  // grid-strided mode 3: workgroup cap 4096 (1024-8192 within noise,
  // profiles/bn_bwd_apply_grid_ab_r3s3.txt)
  const int grid = grid_for(n8, 256, 4096);
  const size_t sh = sizeof(float) * 5 * C;
  // streaming modes: flat blocks of 4 x 256 chunks, non-temporal (see bn_apply_kernel); the
  // stem's pool-gather mode keeps its grid-strided loop
  const int gflat = (int)((n8 + 4 * 256 - 1) / (4 * 256));
#define DM_BNB(MD, D)                                                                              \
  do {                                                                                             \
    if (MD != 3)                                                                                   \
      bn_bwd_apply_kernel<MD, D, 4, true, true><<<gflat, 256, sh, st>>>(a, coef, dy, dres);        \
    else                                                                                           \
      bn_bwd_apply_kernel<MD, D><<<grid, 256, sh, st>>>(a, coef, dy, dres);                        \
  } while (0)
  if (quad) {
    bn_bwd_apply_quad_kernel<<<grid_for(n8 / 4, 256, 4096), 256, sh, st>>>(a, coef, dy);
    return;
  }
  switch (mode * 2 + (dres ? 1 : 0)) {
    case 0: DM_BNB(0, false); break;
    case 1: DM_BNB(0, true); break;
    case 2: DM_BNB(1, false); break;
    case 3: DM_BNB(1, true); break;
    case 4: DM_BNB(2, false); break;
    case 5: DM_BNB(2, true); break;
    case 6: DM_BNB(3, false); break;
    case 7: DM_BNB(3, true); break;
    case 8: DM_BNB(4, false); break;
    default: DM_BNB(4, true); break;
  }
#undef DM_BNB
}


void bn_relu_maxpool(const bf16_t* y, const float* scale, const float* shift, bf16_t* out,
                     uint8_t* idx, int N, int H, int W, int C, int OH, int OW, int K, int S,
                     int P, hipStream_t st, bf16_t* yarg) {
  const long long total = (long long)N * OH * OW * (C / 8);
  if (K == 3 && S == 2 && P == 1 && OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 &&
      (long long)N * H * W * C < (1LL << 31)) {
    const long long pairs = (long long)N * OH * ((OW + 1) / 2) * (C / 8);
    // non-temporal stores of out / yarg (+0.1-0.2 %, profiles/nt_pool_wgrad_reduce_ab_r4aa.txt);
    // the overlapping window loads stay cached
    // (an uncapped, one-pass grid measures the same: profiles/pool_pack_grid_ab_r4as.txt)
    bn_relu_maxpool3s2_kernel<true><<<grid_for(pairs, 256, 8192), 256, sizeof(float) * 2 * C, st>>>(
        y, scale, shift, out, idx, yarg, N, H, W, C, OH, OW);
    return;
  }
  bn_relu_maxpool_kernel<<<grid_for(total, 256, 8192), 256, sizeof(float) * 2 * C, st>>>(
      y, scale, shift, out, idx, yarg, N, H, W, C, OH, OW, K, S, P);
}

// Σdz, Σdz·x̂ partial rows [G][2C] of a mode-2 operand pair (dz = dout masked by
// y*scale + shift > 0) over M rows; returns G (= bn_bwd_groups(M, C)).  Used for the stem's
// pooled-domain sums (dout = pooled grad, y = yarg), handed to bn_backward as pre_part.
int bn_bwd_reduce_masked(const bf16_t* dout, const bf16_t* y, const float* mean,
                         const float* invstd, const float* scale, const float* shift, long long M,
                         int C, float* part, hipStream_t st) {
  BnBwdArgs a{dout, nullptr, y, mean, invstd, scale, shift, nullptr, nullptr, 0, 0, 0, 0, 0, 0, 0,
              M, C, nullptr};
  const int G = bn_bwd_groups(M, C);
  const size_t shr = sizeof(float) * (256 * 16 + 2 * C);
  bn_bwd_reduce_kernel<2, 4, true><<<G, 256, shr, st>>>(a, part);
  return G;
}

void maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH,
                 int OW, int K, int S, int P, hipStream_t st) {
  const long long total = (long long)N * OH * OW * (C / 8);
  maxpool_fwd_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(x, y, idx, N, H, W, C, OH, OW, K, S, P);
}

void maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                 int OH, int OW, int K, int S, int P, hipStream_t st) {
  const long long total = (long long)N * H * W * (C / 8);
  maxpool_bwd_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(dy, idx, dx, N, H, W, C, OH, OW, K, S, P);
}

void avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st) {
  const long long threads = (long long)N * (C / 8);
  avgpool_fwd_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, st>>>(x, y, N, HW, C);
}

void avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  const long long total = (long long)N * HW * (C / 8);
  avgpool_bwd_kernel<<<grid_for(total, 256, 8192), 256, 0, st>>>(dy, dx, N, HW, C);
}

void pack_input(const void* x, bool bf16, bf16_t* y, int N, int C, int H, int W, int Cp,
                long long sn, long long sc, long long sh, long long sw, hipStream_t st) {
  const long long total = (long long)N * H * W;
  if (bf16)
    pack_input_kernel<bf16_t><<<grid_for(total, 256, 8192), 256, 0, st>>>(
        (const bf16_t*)x, y, N, C, H, W, Cp, sn, sc, sh, sw);
  else
    pack_input_kernel<float><<<grid_for(total, 256, 8192), 256, 0, st>>>(
        (const float*)x, y, N, C, H, W, Cp, sn, sc, sh, sw);
}

}  // namespace dm
