// Strided GEMM on the fp32-input MFMA (v_mfma_f32_16x16x4_f32) for Linear layers.
//
//   C[m,n] = alpha * sum_k A(m,k) * B(k,n)  (+ beta*C)  (+ bias[n])  (ReLU)
//   A(m,k) = A[m*sam + k*sak] (optionally masked by Amask(m,k) > 0: ReLU backward
//            fused into the operand load), B(k,n) = B[k*sbk + n*sbn]
//
// One kernel serves all three Linear GEMMs:
//   fwd   Y  = X  · Wᵀ     A=X[M,K] (sam=K,sak=1)   B=Wᵀ (sbk=1, sbn=K)
//   dgrad dX = dY · W      A=dY (masked)           B=W  (sbk=K_in... row-major)
//   wgrad dW = dYᵀ · X     A=dYᵀ (sam=1, sak=N)     B=X
// The operands are tiny (LeNet fc 400→120, MLP ≤784×512, ResNet fc 512→1000), so
// the kernel is latency-oriented: 64×64 tile, 4 waves each owning a 32×32
// quadrant as 2×2 MFMA 16×16 blocks, BK=64 staged through padded LDS (16 independent
// loads per thread and operand in flight: with BK=16 LeNet's fc1, K=400, was 25 serial
// load round trips, 59 us for 1.5 MFLOP).  Inputs may be fp32 or bf16 (converted on the
// LDS store; exact fp32 MFMA math either way).
// Exact f32 numerics: the MFMA is a k-ordered fmaf chain (guide §3).
#include "common.h"

namespace dm {

template <typename T> __device__ __forceinline__ float ldx(const T* p, long long i);
template <> __device__ __forceinline__ float ldx<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ldx<bf16_t>(const bf16_t* p, long long i) {
  return bf2f(p[i]);
}

constexpr int GBM = 64, GBN = 64, GBK = 16;
constexpr int FBK = 64;  // k per LDS stage of the fp32 kernel

template <typename TA, typename TB, typename TC>
__global__ void __launch_bounds__(256) gemm_f32mfma_kernel(
    const TA* __restrict__ A, const TA* __restrict__ Amask, const TB* __restrict__ B,
    TC* __restrict__ C, float* __restrict__ C32, const float* __restrict__ bias, int M, int N,
    int K, long long sam, long long sak, long long sbk, long long sbn, long long scm,
    float alpha, float beta, int relu, float* __restrict__ part, int kchunk) {
  // split-K (part != nullptr): block z reduces k in [z*kchunk, (z+1)*kchunk) into
  // part[z][M][N] (alpha applied); gemm_splitk_reduce_kernel sums z in order + epilogue
  __shared__ float As[FBK][GBM + 4];
  __shared__ float Bs[FBK][GBN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  constexpr int NA = FBK * GBM / 256, NB = FBK * GBN / 256;
  const int kb = part ? blockIdx.z * kchunk : 0;
  const int ke = part ? min(K, kb + kchunk) : K;
  for (int k0 = kb; k0 < ke; k0 += FBK) {
    // stage A tile [FBK][GBM] and B tile [FBK][GBN]: 16 elements each per thread.  Every
    // load is issued first (out-of-range elements read element 0 and are zeroed by a select,
    // no branch), then all LDS stores: a guarded load-then-store per element made the
    // compiler wait on each load in turn
    float va[NA], vb[NB];
#pragma unroll
    for (int r = 0; r < NA; ++r) {
      const int e = tid + r * 256;
      int mm, kk;
      if (sak == 1) { mm = e / FBK; kk = e % FBK; }   // k contiguous: walk k fastest
      else { kk = e / GBM; mm = e % GBM; }            // m contiguous
      const int gm = m0 + mm, gk = k0 + kk;
      const bool ok = gm < M && gk < ke;
      const long long o = ok ? (long long)gm * sam + (long long)gk * sak : 0;
      float v = ldx(A, o);
      if (Amask) v = ldx(Amask, o) > 0.f ? v : 0.f;
      va[r] = ok ? v : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const int e = tid + r * 256;
      int nn, kk;
      if (sbk == 1) { nn = e / FBK; kk = e % FBK; }
      else { kk = e / GBN; nn = e % GBN; }
      const int gn = n0 + nn, gk = k0 + kk;
      const bool ok = gn < N && gk < ke;
      const float v = ldx(B, ok ? (long long)gk * sbk + (long long)gn * sbn : 0);
      vb[r] = ok ? v : 0.f;
    }
    if (k0 > kb) __syncthreads();  // the previous tile's MFMA reads are done
#pragma unroll
    for (int r = 0; r < NA; ++r) {
      const int e = tid + r * 256;
      if (sak == 1) As[e % FBK][e / FBK] = va[r];
      else As[e / GBM][e % GBM] = va[r];
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const int e = tid + r * 256;
      if (sbk == 1) Bs[e % FBK][e / FBK] = vb[r];
      else Bs[e / GBN][e % GBN] = vb[r];
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < FBK; ks += 4) {
      const int kk = ks + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const float a = As[kk][wm + i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float b = Bs[kk][wn + j * 16 + (lane & 15)];
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + r
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        const int gn = n0 + wn + j * 16 + (lane & 15);
        if (gm < M && gn < N) {
          float v = alpha * acc[i][j][r];
          if (part) {
            part[((long long)blockIdx.z * M + gm) * N + gn] = v;
            continue;
          }
          const long long o = (long long)gm * scm + gn;
          if (beta != 0.f) v += beta * (C32 ? C32[o] : ldx(C, o));
          if (bias) v += bias[gn];
          if (relu) v = fmaxf(v, 0.f);
          if (C32) C32[o] = v;
          if (C) {
            if constexpr (sizeof(TC) == 4) C[o] = v;
            else C[o] = f2bf(v);
          }
        }
      }
}

// bf16 operands on v_mfma_f32_16x16x32_bf16 (fp32 accumulation): the ResNet classifier head
// (A = bf16 activations / gradients, B = bf16 or the fp32 master weight, rounded to bf16 while
// staging).  Same strided semantics and epilogue as gemm_f32mfma_kernel.  Tile 64x64, 4 waves
// of 32x32, BK 32; LDS rows k-contiguous (pitch 40 elements) for the 8-k fragment reads.
template <typename TB, typename TC>
__global__ void __launch_bounds__(256) gemm_bf16mfma_kernel(
    const bf16_t* __restrict__ A, const bf16_t* __restrict__ Amask, const TB* __restrict__ B,
    TC* __restrict__ C, float* __restrict__ C32, const float* __restrict__ bias, int M, int N,
    int K, long long sam, long long sak, long long sbk, long long sbn, long long scm,
    float alpha, float beta, int relu, float* __restrict__ part, int kchunk) {
  // split-K (part != nullptr): block z reduces k in [z*kchunk, (z+1)*kchunk) and stores
  // alpha*acc into part[z][M][N]; gemm_splitk_reduce_kernel applies the epilogue
  constexpr int BK = 32, P = 40;
  __shared__ __attribute__((aligned(16))) bf16_t As[GBM][P];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[GBN][P];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  const int wm = (wid >> 1) * 32, wn = (wid & 1) * 32;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int kb = part ? blockIdx.z * kchunk : 0;
  const int ke = part ? min(K, kb + kchunk) : K;
  for (int k0 = kb; k0 < ke; k0 += BK) {
    // 64 x 32 elements per operand, 8 per thread, walking the contiguous dimension fastest.
    // All 16 loads first (out-of-range elements read element 0, zeroed by a select), then
    // the LDS stores: a guarded load-then-store per element waited on each load in turn
    bf16_t va[8], vb[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + r * 256;
      int mm, kk;
      if (sak == 1) { mm = e / BK; kk = e % BK; }
      else { kk = e / GBM; mm = e % GBM; }
      const int gm = m0 + mm, gk = k0 + kk;
      const bool ok = gm < M && gk < ke;
      const long long o = ok ? (long long)gm * sam + (long long)gk * sak : 0;
      bf16_t v = A[o];
      if (Amask) v = bf2f(Amask[o]) > 0.f ? v : (bf16_t)0;
      va[r] = ok ? v : (bf16_t)0;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + r * 256;
      int nn, kk;
      if (sbk == 1) { nn = e / BK; kk = e % BK; }
      else { kk = e / GBN; nn = e % GBN; }
      const int gn = n0 + nn, gk = k0 + kk;
      const bool ok = gn < N && gk < ke;
      const long long o = ok ? (long long)gk * sbk + (long long)gn * sbn : 0;
      bf16_t v;
      if constexpr (sizeof(TB) == 4) v = f2bf(B[o]);
      else v = B[o];
      vb[r] = ok ? v : (bf16_t)0;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + r * 256;
      if (sak == 1) As[e / BK][e % BK] = va[r];
      else As[e % GBM][e / GBM] = va[r];
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int e = tid + r * 256;
      if (sbk == 1) Bs[e / BK][e % BK] = vb[r];
      else Bs[e % GBN][e / GBN] = vb[r];
    }
    __syncthreads();
    const int kq = (lane >> 4) * 8;
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) af[i] = *reinterpret_cast<const bf16x8*>(&As[wm + i * 16 + (lane & 15)][kq]);
#pragma unroll
    for (int j = 0; j < 2; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(&Bs[wn + j * 16 + (lane & 15)][kq]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + (lane >> 4) * 4 + r;
        const int gn = n0 + wn + j * 16 + (lane & 15);
        if (gm < M && gn < N) {
          float v = alpha * acc[i][j][r];
          if (part) {
            part[((long long)blockIdx.z * M + gm) * N + gn] = v;
            continue;
          }
          const long long o = (long long)gm * scm + gn;
          if (beta != 0.f) v += beta * (C32 ? C32[o] : ldx(C, o));
          if (bias) v += bias[gn];
          if (relu) v = fmaxf(v, 0.f);
          if (C32) C32[o] = v;
          if (C) {
            if constexpr (sizeof(TC) == 4) C[o] = v;
            else C[o] = f2bf(v);
          }
        }
      }
}

template <typename TC>
__global__ void __launch_bounds__(256) gemm_splitk_reduce_kernel(
    const float* __restrict__ part, int S, int M, int N, TC* __restrict__ C,
    float* __restrict__ C32, const float* __restrict__ bias, long long scm, float beta, int relu) {
  const long long total = (long long)M * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int z = 0; z < S; ++z) v += part[z * total + e];  // fixed order: deterministic
    const int gm = (int)(e / N), gn = (int)(e % N);
    const long long o = (long long)gm * scm + gn;
    if (beta != 0.f) v += beta * (C32 ? C32[o] : ldx(C, o));
    if (bias) v += bias[gn];
    if (relu) v = fmaxf(v, 0.f);
    if (C32) C32[o] = v;
    if (C) {
      if constexpr (sizeof(TC) == 4) C[o] = v;
      else C[o] = f2bf(v);
    }
  }
}

// db[n] = beta*db[n] + sum_m A(m,n) [masked by Amask(m,n) > 0]   (bias gradient)
template <typename T>
__global__ void __launch_bounds__(256) colsum_kernel(const T* __restrict__ A,
                                                     const T* __restrict__ Amask,
                                                     float* __restrict__ out, int M, int N,
                                                     float beta) {
  // block = 256 threads: 64 columns x 4 row-groups
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < N)
    for (int m = rg; m < M; m += 4) {
      const long long o = (long long)m * N + c;
      float v = ldx(A, o);
      if (Amask && !(ldx(Amask, o) > 0.f)) v = 0.f;
      s += v;
    }
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < N) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                    red[3][threadIdx.x];
    out[c] = beta * out[c] + t;
  }
}

// ------------------------------------------------------------------ launchers
// dtype codes: 0 = fp32, 1 = bf16
void gemm_strided(const void* A, const void* Amask, int a_bf16, const void* B, int b_bf16,
                  void* C, int c_bf16, float* C32, const float* bias, int M, int N, int K,
                  long long sam, long long sak, long long sbk, long long sbn, long long scm,
                  float alpha, float beta, int relu, int lowp, float* part, int S,
                  hipStream_t st) {
  dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
  if (lowp && a_bf16) {  // bf16 MFMA (B rounded to bf16 while staging)
    const int kchunk = S > 1 ? ((K + S - 1) / S + 31) / 32 * 32 : K;
    if (S > 1) grid.z = S;
    float* pp = S > 1 ? part : nullptr;
#define DM_GEMM16(TB, TC)                                                                    \
  gemm_bf16mfma_kernel<TB, TC><<<grid, 256, 0, st>>>(                                        \
      (const bf16_t*)A, (const bf16_t*)Amask, (const TB*)B, (TC*)C, C32, bias, M, N, K, sam, \
      sak, sbk, sbn, scm, alpha, beta, relu, pp, kchunk)
    if (b_bf16 && c_bf16) DM_GEMM16(bf16_t, bf16_t);
    else if (b_bf16) DM_GEMM16(bf16_t, float);
    else if (c_bf16) DM_GEMM16(float, bf16_t);
    else DM_GEMM16(float, float);
#undef DM_GEMM16
    if (S > 1) {
      const int g = grid_for((long long)M * N, 256, 2048);
      if (c_bf16)
        gemm_splitk_reduce_kernel<bf16_t><<<g, 256, 0, st>>>(part, S, M, N, (bf16_t*)C, C32, bias,
                                                              scm, beta, relu);
      else
        gemm_splitk_reduce_kernel<float><<<g, 256, 0, st>>>(part, S, M, N, (float*)C, C32, bias,
                                                             scm, beta, relu);
    }
    return;
  }
  // split-K for the fp32 kernel: the caller sized part for S chunks of K (LeNet fc1: 2
  // output tiles, K = 400 = 7 serial LDS stages -> 7 blocks of one stage each + a reduce)
  const int kchunk32 = S > 1 ? ((K + S - 1) / S + FBK - 1) / FBK * FBK : K;
  float* pp32 = S > 1 ? part : nullptr;
  if (S > 1) grid.z = (K + kchunk32 - 1) / kchunk32;
#define DM_GEMM(TA, TB, TC)                                                                  \
  gemm_f32mfma_kernel<TA, TB, TC><<<grid, 256, 0, st>>>(                                     \
      (const TA*)A, (const TA*)Amask, (const TB*)B, (TC*)C, C32, bias, M, N, K, sam, sak, sbk, \
      sbn, scm, alpha, beta, relu, pp32, kchunk32)
  if (!a_bf16 && !b_bf16 && !c_bf16) DM_GEMM(float, float, float);
  else if (!a_bf16 && !b_bf16 && c_bf16) DM_GEMM(float, float, bf16_t);
  else if (a_bf16 && !b_bf16 && !c_bf16) DM_GEMM(bf16_t, float, float);
  else if (a_bf16 && !b_bf16 && c_bf16) DM_GEMM(bf16_t, float, bf16_t);
  else if (a_bf16 && b_bf16 && !c_bf16) DM_GEMM(bf16_t, bf16_t, float);
  else if (a_bf16 && b_bf16 && c_bf16) DM_GEMM(bf16_t, bf16_t, bf16_t);
  else if (!a_bf16 && b_bf16 && !c_bf16) DM_GEMM(float, bf16_t, float);
  else DM_GEMM(float, bf16_t, bf16_t);
#undef DM_GEMM
  if (S > 1) {
    const int g = grid_for((long long)M * N, 256, 2048);
    if (c_bf16)
      gemm_splitk_reduce_kernel<bf16_t><<<g, 256, 0, st>>>(part, (int)grid.z, M, N, (bf16_t*)C,
                                                            C32, bias, scm, beta, relu);
    else
      gemm_splitk_reduce_kernel<float><<<g, 256, 0, st>>>(part, (int)grid.z, M, N, (float*)C, C32,
                                                           bias, scm, beta, relu);
  }
}

void colsum(const void* A, const void* Amask, int bf16, float* out, int M, int N, float beta,
            hipStream_t st) {
  dim3 grid((N + 63) / 64);
  if (bf16)
    colsum_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)A, (const bf16_t*)Amask, out, M,
                                                N, beta);
  else
    colsum_kernel<float><<<grid, 256, 0, st>>>((const float*)A, (const float*)Amask, out, M, N,
                                               beta);
}

// out = act(y + bias) (fp32 -> fp32 or bf16): the tensor-parallel row-split head's epilogue,
// after the all-reduce of the partial products (parallel/tensor_parallel.py RowParallelLinear)
__global__ void __launch_bounds__(256) bias_act_kernel(const float* __restrict__ y,
                                                       const float* __restrict__ bias, void* out,
                                                       long long n, int N, int relu, int obf) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    float v = y[i] + (bias ? bias[i % N] : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    if (obf) reinterpret_cast<bf16_t*>(out)[i] = f2bf(v);
    else reinterpret_cast<float*>(out)[i] = v;
  }
}

void bias_act(const float* y, const float* bias, void* out, int out_bf16, int M, int N, int relu,
              hipStream_t st) {
  const long long n = (long long)M * N;
  if (n == 0) return;
  bias_act_kernel<<<grid_for(n, 256), 256, 0, st>>>(y, bias, out, n, N, relu, out_bf16);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
