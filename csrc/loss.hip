// Cross-entropy (fused log-softmax + NLL + backward seed), evaluation counter and
// a device spin kernel.
//
// the reference runs log_softmax, nll_loss (mean) and, in
// backward, their two gradients as separate ATen kernels.  Here ONE pass per row
// computes the row loss AND d(logits) = (softmax − onehot) * scale (scale = 1/B
// for the mean), so backward only rescales by the incoming grad.  Per-row losses
// are summed by a second single-block kernel in fixed order (deterministic).
// K26: the eval loop's argmax/eq/sum/.item() per batch becomes an on-device
// argmax+compare+counter with one D2H read per evaluation.
#include "common.h"

namespace dm {

template <typename T> __device__ __forceinline__ float ldv(const T* p, long long i);
template <> __device__ __forceinline__ float ldv<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ldv<bf16_t>(const bf16_t* p, long long i) {
  return bf2f(p[i]);
}

// one wave per row; block = 256 (4 rows)
template <typename T>
__global__ void __launch_bounds__(256) ce_fwd_bwd_kernel(const T* __restrict__ logits,
                                                         const long long* __restrict__ labels,
                                                         float* __restrict__ rowloss,
                                                         T* __restrict__ dlogits, int B, int C,
                                                         float scale, int ignore_index) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* x = logits + (long long)row * C;
  float m = -INFINITY;
  for (int c = lane; c < C; c += 64) m = fmaxf(m, ldv(x, c));
  m = wave_max(m);
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += __expf(ldv(x, c) - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  const long long y = labels[row];
  const bool valid = y != ignore_index && y >= 0 && y < C;
  if (lane == 0) rowloss[row] = valid ? (lse - ldv(x, y)) : 0.f;
  if (dlogits) {
    T* d = dlogits + (long long)row * C;
    const float inv = 1.f / s;
    for (int c = lane; c < C; c += 64) {
      float g = valid ? (__expf(ldv(x, c) - m) * inv - (c == y ? 1.f : 0.f)) * scale : 0.f;
      if constexpr (sizeof(T) == 4) d[c] = g;
      else d[c] = f2bf(g);
    }
  }
}

__global__ void __launch_bounds__(256) sum_scale_kernel(const float* __restrict__ v, int n,
                                                        float scale, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) out[0] = s * scale;
}

// correct[0] += #rows with argmax(logits[row]) == label[row]
template <typename T>
__global__ void __launch_bounds__(256) argmax_count_kernel(const T* __restrict__ logits,
                                                           const long long* __restrict__ labels,
                                                           int B, int C,
                                                           unsigned long long* __restrict__ correct) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* x = logits + (long long)row * C;
  float best = -INFINITY;
  int arg = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = ldv(x, c);
    if (v > best) { best = v; arg = c; }  // first max within the lane's strided set
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oa = __shfl_xor(arg, o, 64);
    if (ob > best || (ob == best && oa < arg)) { best = ob; arg = oa; }  // torch: first index
  }
  if (lane == 0 && arg == labels[row]) atomicAdd(correct, 1ull);
}

// Busy-wait on the device for `us` microseconds (straggler injection, graph-safe).
__global__ void spin_kernel(unsigned long long cycles) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

// ------------------------------------------------------------------ launchers
void cross_entropy(const void* logits, const long long* labels, float* rowloss, float* loss,
                   void* dlogits, int B, int C, float scale, int ignore_index, bool bf16,
                   hipStream_t st) {
  const int grid = (B + 3) / 4;
  if (bf16)
    ce_fwd_bwd_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)logits, labels, rowloss,
                                                    (bf16_t*)dlogits, B, C, scale, ignore_index);
  else
    ce_fwd_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)logits, labels, rowloss,
                                                   (float*)dlogits, B, C, scale, ignore_index);
  sum_scale_kernel<<<1, 256, 0, st>>>(rowloss, B, scale, loss);
}

void argmax_count(const void* logits, const long long* labels, int B, int C,
                  unsigned long long* correct, bool bf16, hipStream_t st) {
  const int grid = (B + 3) / 4;
  if (bf16)
    argmax_count_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)logits, labels, B, C, correct);
  else
    argmax_count_kernel<float><<<grid, 256, 0, st>>>((const float*)logits, labels, B, C, correct);
}

void spin_us(double us, hipStream_t st) {
  // s_memrealtime runs at a constant 100 MHz on CDNA
  const unsigned long long cycles = (unsigned long long)(us * 100.0);
  spin_kernel<<<1, 64, 0, st>>>(cycles);
}

}  // namespace dm
