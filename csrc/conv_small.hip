// Direct convolution for tiny channel counts (LeNet: C = 1 → 6 → 16), NCHW fp32/bf16.
//
// with N = 6/16 output channels and K = 25/150 the
// convs are far too thin for MFMA tiles (a 16×16 tile would be ≥60 % padding),
// so they run on the VALU with the weights of one output channel (forward) or
// one input channel (backward-data) staged in LDS, and everything elementwise
// fused in:
//   fwd : conv + bias + ReLU + 2×2 max-pool, writing the pooled map and a 2-bit
//         argmax code per pooled element (uint8) instead of int64 indices
//   bwd : (1) unpool+ReLU-mask → dense conv-output gradient
//         (2) backward-data with W[:, ci] in LDS
//         (3) backward-weight + bias, split over batch slices into fp32 partial
//             slabs, then a fixed-order slab reduce (deterministic, no atomics)
//             that also applies the accumulate (beta) semantics of .grad.
#include "common.h"

namespace dm {

template <typename T> __device__ __forceinline__ float ld(const T* p, long long i);
template <> __device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) {
  return bf2f(p[i]);
}
template <typename T> __device__ __forceinline__ void st(T* p, long long i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, long long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, long long i, float v) {
  p[i] = f2bf(v);
}

// ---------------------------------------------------------------- forward
// grid: (ceil(PH*PW/256), B*Cout); block 256.  POOL ∈ {1,2}.
template <typename T, int K, int POOL>
__global__ void __launch_bounds__(256) conv_small_fwd_kernel(
    const T* __restrict__ x, const float* __restrict__ w, const float* __restrict__ bias,
    T* __restrict__ y, uint8_t* __restrict__ mask, int Cin, int H, int W, int Cout, int pad,
    int relu, int PH, int PW) {
  extern __shared__ float ws[];  // Cin*K*K
  const int bc = blockIdx.y;
  const int b = bc / Cout, co = bc % Cout;
  const int nw = Cin * K * K;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) ws[i] = w[(long long)co * nw + i];
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= PH * PW) return;
  const int ph = idx / PW, pw = idx % PW;
  const int oh0 = ph * POOL, ow0 = pw * POOL;
  float acc[POOL * POOL];
#pragma unroll
  for (int i = 0; i < POOL * POOL; ++i) acc[i] = 0.f;
  constexpr int P = K + POOL - 1;  // input patch edge
  for (int ci = 0; ci < Cin; ++ci) {
    const T* xp = x + ((long long)b * Cin + ci) * H * W;
    float patch[P][P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const int ih = oh0 - pad + r;
#pragma unroll
      for (int c = 0; c < P; ++c) {
        const int iw = ow0 - pad + c;
        patch[r][c] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? ld(xp, (long long)ih * W + iw) : 0.f;
      }
    }
    const float* wc = ws + ci * K * K;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const float wv = wc[kh * K + kw];
#pragma unroll
        for (int dy = 0; dy < POOL; ++dy)
#pragma unroll
          for (int dx = 0; dx < POOL; ++dx) acc[dy * POOL + dx] += wv * patch[dy + kh][dx + kw];
      }
  }
  float best = acc[0];
  int arg = 0;
#pragma unroll
  for (int i = 1; i < POOL * POOL; ++i)
    if (acc[i] > best) { best = acc[i]; arg = i; }
  float v = best + (bias ? bias[co] : 0.f);
  if (relu) v = fmaxf(v, 0.f);
  const long long o = ((long long)b * Cout + co) * PH * PW + idx;
  st(y, o, v);
  if (POOL > 1 && mask) mask[o] = (uint8_t)arg;
}

// ---------------------------------------------------------------- backward (1): unpool + relu mask
// dyc[b,co,oh,ow] (dense conv-output grad, fp32) from pooled grad dp and pooled output yp.
template <typename T, int POOL>
__global__ void __launch_bounds__(256) unpool_relu_bwd_kernel(
    const T* __restrict__ dp, const T* __restrict__ yp, const uint8_t* __restrict__ mask,
    float* __restrict__ dyc, long long total, int OH, int OW, int PH, int PW, int relu) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int ow = i % OW;
    const long long t = i / OW;
    const int oh = t % OH;
    const long long plane = t / OH;
    float g = 0.f;
    const int ph = oh / POOL, pw = ow / POOL;
    if (ph < PH && pw < PW) {
      const long long pi = plane * PH * PW + ph * PW + pw;
      const int code = (oh - ph * POOL) * POOL + (ow - pw * POOL);
      const bool hit = POOL == 1 || mask[pi] == code;
      const bool live = !relu || ld(yp, pi) > 0.f;
      if (hit && live) g = ld(dp, pi);
    }
    dyc[i] = g;
  }
}

// ---------------------------------------------------------------- backward (2): data
// dx[b,ci,ih,iw] = sum_{co,kh,kw} dyc[b,co,ih+pad-kh, iw+pad-kw] * w[co,ci,kh,kw]
// grid: (ceil(H*W/256), B*Cin)
template <typename T, int K>
__global__ void __launch_bounds__(256) conv_small_bwd_data_kernel(
    const float* __restrict__ dyc, const float* __restrict__ w, T* __restrict__ dx, int Cin,
    int H, int W, int Cout, int OH, int OW, int pad) {
  // LDS: Cout*K*K weights of this ci, then image b's upstream gradient [Cout][OH][OW] with a
  // zero border of K-1 on every side (18 x 18 per channel for LeNet conv2, 20.7 KB): staged
  // with coalesced loads once, so the 16 x 25 tap loop reads LDS at compile-time offsets with
  // no bounds branches (a dependent L2 load per tap: 35 us at batch 32; guarded LDS taps at
  // 3 waves per CU: 23 us)
  extern __shared__ float ws[];
  float* gs = ws + Cout * K * K;
  const int PH = OH + 2 * (K - 1), PW = OW + 2 * (K - 1);
  const int bc = blockIdx.y;
  const int b = bc / Cin, ci = bc % Cin;
  for (int i = threadIdx.x; i < Cout * K * K; i += blockDim.x) {
    const int co = i / (K * K), r = i % (K * K);
    ws[i] = w[((long long)co * Cin + ci) * K * K + r];
  }
  const float* gb = dyc + (long long)b * Cout * OH * OW;
  for (int i = threadIdx.x; i < Cout * PH * PW; i += blockDim.x) {
    const int co = i / (PH * PW), r = i % (PH * PW);
    const int oh = r / PW - (K - 1), ow = r % PW - (K - 1);
    gs[i] = (oh >= 0 && oh < OH && ow >= 0 && ow < OW) ? gb[(co * OH + oh) * OW + ow] : 0.f;
  }
  __syncthreads();
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= H * W) return;
  const int ih = idx / W, iw = idx % W;
  // tap (kh, kw) reads padded (ih + pad + K-1 - kh, iw + pad + K-1 - kw)
  const int base = (ih + pad + K - 1) * PW + (iw + pad + K - 1);
  float part[K];
#pragma unroll
  for (int kh = 0; kh < K; ++kh) part[kh] = 0.f;
  for (int co = 0; co < Cout; ++co) {
    const float* g = gs + co * PH * PW + base;
    const float* wc = ws + co * K * K;
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) part[kh] += g[-kh * PW - kw] * wc[kh * K + kw];
  }
  float acc = 0.f;
#pragma unroll
  for (int kh = 0; kh < K; ++kh) acc += part[kh];
  st(dx, ((long long)b * Cin + ci) * H * W + idx, acc);
}

// ---------------------------------------------------------------- backward (3): weight partials
// grid: (Cout*Cin, S) ; block 256.  Block (co,ci,s) reduces over images
// [s*bs, min(B,(s+1)*bs)) and all output pixels; writes K*K weight partials and
// (ci==0) the bias partial into part[s][...].
template <typename T, int K>
__global__ void __launch_bounds__(256) conv_small_bwd_w_kernel(
    const float* __restrict__ dyc, const T* __restrict__ x, float* __restrict__ part, int B,
    int Cin, int H, int W, int Cout, int OH, int OW, int pad, int bs, int nout) {
  __shared__ float red[4][K * K + 1];
  const int co = blockIdx.x / Cin, ci = blockIdx.x % Cin;
  const int s = blockIdx.y;
  const int b0 = s * bs, b1 = min(B, b0 + bs);
  float acc[K * K + 1];
#pragma unroll
  for (int i = 0; i <= K * K; ++i) acc[i] = 0.f;
  const long long npix = (long long)(b1 - b0) * OH * OW;
  for (long long p = threadIdx.x; p < npix; p += blockDim.x) {
    const int ow = p % OW;
    const long long t = p / OW;
    const int oh = t % OH;
    const int b = b0 + (int)(t / OH);
    const float g = dyc[(((long long)b * Cout + co) * OH + oh) * OW + ow];
    if (g == 0.f) continue;  // pooled grads are 3/4 zeros
    const T* xp = x + ((long long)b * Cin + ci) * H * W;
#pragma unroll
    for (int kh = 0; kh < K; ++kh) {
      const int ih = oh - pad + kh;
      const bool okh = ih >= 0 && ih < H;
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int iw = ow - pad + kw;
        const float xv = (okh && iw >= 0 && iw < W) ? ld(xp, (long long)ih * W + iw) : 0.f;
        acc[kh * K + kw] += g * xv;
      }
    }
    acc[K * K] += g;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i <= K * K; ++i) {
    float v = wave_sum(acc[i]);
    if (lane == 0) red[wid][i] = v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i <= K * K; i += blockDim.x) {
    const float v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    float* ps = part + (long long)s * nout;
    if (i < K * K)
      ps[((long long)co * Cin + ci) * K * K + i] = v;
    else if (ci == 0)
      ps[(long long)Cout * Cin * K * K + co] = v;
  }
}

// out[j] = beta*out[j] + sum_s part[s][j]   (fixed order → deterministic)
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ part,
                                                          int S, int n, float* __restrict__ outw,
                                                          int nw, float* __restrict__ outb,
                                                          float beta) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  float s = 0.f;
  for (int i = 0; i < S; ++i) s += part[(long long)i * n + j];
  if (j < nw) {
    outw[j] = beta * outw[j] + s;
  } else if (outb) {
    outb[j - nw] = beta * outb[j - nw] + s;
  }
}

// ---------------------------------------------------------------- launchers
template <typename T>
static void fwd_dispatch(const T* x, const float* w, const float* bias, T* y, uint8_t* mask,
                         int B, int Cin, int H, int W, int Cout, int K, int pad, int pool,
                         int relu, hipStream_t st) {
  const int OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  const int PH = OH / pool, PW = OW / pool;
  dim3 grid((PH * PW + 255) / 256, B * Cout);
  const size_t sh = sizeof(float) * Cin * K * K;
  if (K == 5 && pool == 2)
    conv_small_fwd_kernel<T, 5, 2><<<grid, 256, sh, st>>>(x, w, bias, y, mask, Cin, H, W, Cout,
                                                          pad, relu, PH, PW);
  else if (K == 5 && pool == 1)
    conv_small_fwd_kernel<T, 5, 1><<<grid, 256, sh, st>>>(x, w, bias, y, mask, Cin, H, W, Cout,
                                                          pad, relu, PH, PW);
  else if (K == 3 && pool == 2)
    conv_small_fwd_kernel<T, 3, 2><<<grid, 256, sh, st>>>(x, w, bias, y, mask, Cin, H, W, Cout,
                                                          pad, relu, PH, PW);
  else if (K == 3 && pool == 1)
    conv_small_fwd_kernel<T, 3, 1><<<grid, 256, sh, st>>>(x, w, bias, y, mask, Cin, H, W, Cout,
                                                          pad, relu, PH, PW);
  else
    abort();
}

void conv_small_fwd(const void* x, const float* w, const float* bias, void* y, uint8_t* mask,
                    int B, int Cin, int H, int W, int Cout, int K, int pad, int pool, int relu,
                    bool bf16, hipStream_t st) {
  if (bf16)
    fwd_dispatch<bf16_t>((const bf16_t*)x, w, bias, (bf16_t*)y, mask, B, Cin, H, W, Cout, K, pad,
                         pool, relu, st);
  else
    fwd_dispatch<float>((const float*)x, w, bias, (float*)y, mask, B, Cin, H, W, Cout, K, pad,
                        pool, relu, st);
}

// Full backward of one fused conv stage.  `work` must hold
// B*Cout*OH*OW (dyc) + S*nout (partials) floats, S = ceil(B / bs).
template <typename T>
static void bwd_impl(const T* x, const float* w, const T* dp, const T* yp, const uint8_t* mask,
                     T* dx, float* dw, float* db, float* work, int B, int Cin, int H, int W,
                     int Cout, int K, int pad, int pool, int relu, float beta, int bs,
                     hipStream_t st) {
  const int OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  const int PH = OH / pool, PW = OW / pool;
  const long long total = (long long)B * Cout * OH * OW;
  float* dyc = work;
  const int S = (B + bs - 1) / bs;
  const int nw = Cout * Cin * K * K;
  const int nout = nw + Cout;
  float* part = work + ((total + 63) / 64) * 64;
  if (pool == 2)
    unpool_relu_bwd_kernel<T, 2><<<grid_for(total, 256), 256, 0, st>>>(dp, yp, mask, dyc, total,
                                                                       OH, OW, PH, PW, relu);
  else
    unpool_relu_bwd_kernel<T, 1><<<grid_for(total, 256), 256, 0, st>>>(dp, yp, mask, dyc, total,
                                                                       OH, OW, PH, PW, relu);
  if (dx) {
    dim3 g((H * W + 255) / 256, B * Cin);
    const size_t sh = sizeof(float) * (Cout * K * K + Cout * (OH + 2 * (K - 1)) * (OW + 2 * (K - 1)));
    if (K == 5)
      conv_small_bwd_data_kernel<T, 5><<<g, 256, sh, st>>>(dyc, w, dx, Cin, H, W, Cout, OH, OW, pad);
    else
      conv_small_bwd_data_kernel<T, 3><<<g, 256, sh, st>>>(dyc, w, dx, Cin, H, W, Cout, OH, OW, pad);
  }
  dim3 gw(Cout * Cin, S);
  if (K == 5)
    conv_small_bwd_w_kernel<T, 5><<<gw, 256, 0, st>>>(dyc, x, part, B, Cin, H, W, Cout, OH, OW,
                                                      pad, bs, nout);
  else
    conv_small_bwd_w_kernel<T, 3><<<gw, 256, 0, st>>>(dyc, x, part, B, Cin, H, W, Cout, OH, OW,
                                                      pad, bs, nout);
  slab_reduce_kernel<<<(nout + 255) / 256, 256, 0, st>>>(part, S, nout, dw, nw, db, beta);
}

void conv_small_bwd(const void* x, const float* w, const void* dp, const void* yp,
                    const uint8_t* mask, void* dx, float* dw, float* db, float* work, int B,
                    int Cin, int H, int W, int Cout, int K, int pad, int pool, int relu,
                    float beta, int bs, bool bf16, hipStream_t st) {
  if (bf16)
    bwd_impl<bf16_t>((const bf16_t*)x, w, (const bf16_t*)dp, (const bf16_t*)yp, mask,
                     (bf16_t*)dx, dw, db, work, B, Cin, H, W, Cout, K, pad, pool, relu, beta, bs,
                     st);
  else
    bwd_impl<float>((const float*)x, w, (const float*)dp, (const float*)yp, mask, (float*)dx, dw,
                    db, work, B, Cin, H, W, Cout, K, pad, pool, relu, beta, bs, st);
}

}  // namespace dm
