// One-shot all-reduce over xGMI peer memory (single node, one process per GPU), gfx950.
//
// RCCL's ring all-reduce pays 2(W-1) latency-bound steps; for the small gradient buckets
// of the labs' LeNet (207 KB in total) the step count, not bandwidth, is the cost.  Here
// every rank exposes an IPC-shared, uncached device buffer (hipExtMallocWithFlags
// hipDeviceMallocUncached + hipIpcGetMemHandle), opened by every peer
// (hipIpcOpenMemHandle).  One kernel per call:
//   1. block b copies its slice of the input into this rank's shared data buffer
//      (buffer parity = call epoch & 1: a slice is rewritten two calls later, after every
//      peer has passed the previous call's flag wait, so it has finished reading it);
//   2. system-scope release fence, then block b stores the epoch into flag[b][rank] of
//      EVERY rank (remote stores over xGMI);
//   3. block b waits until its own flag[b][0..W) all carry the epoch (bounded spin: a peer
//      that never arrives sets *err and the kernel exits instead of hanging the GPU);
//   4. block b reads slice b of all W buffers (remote loads over xGMI), sums them in a fixed
//      rank order (bitwise-identical results on every rank) and writes out = scale * sum.
// Blocks synchronise only with their namesakes on the peers — no grid-wide barrier.
//
// The call epoch lives on the DEVICE (state[1]), not in a kernel argument: every block reads
// epoch = state[1] + 1 on entry, and the last block to leave (a done-counter, state[2])
// publishes it.  A hipGraph replay therefore advances the epoch (and flips the parity half)
// exactly like an eager call; a host counter frozen into the captured arguments would replay
// the same epoch and let the flag waits pass at once.  state[0] is the timeout flag.
//
// Two-shot variant (large buckets, e.g. ResNet-18's 25 MB): the one-shot kernel reads W
// full copies per rank, (W-1)·n remote bytes.  Two-shot splits the message into W rank
// slices; block b of rank r
//   1. copies chunk b of every slice into its shared buffer, flags phase A on every rank;
//   2. after all W phase-A flags: reduces chunk b of ITS slice r from the W buffers (rank
//      order), writes scale·sum to out and back into its own buffer (only rank r ever
//      reads slice r of its own buffer during phase 2, so the in-place write is safe),
//      flags phase B on every rank;
//   3. after all W phase-B flags: gathers chunk b of every other slice q from rank q's
//      buffer.
// 2·(W-1)/W·n remote bytes per rank, spread over all W-1 xGMI links at once (a ring uses
// one).  Parity halves: a peer can only rewrite the half read here two calls later, after
// passing a phase-A wait on OUR next call, which starts after this kernel has drained.
#include "common.h"

#include <cstring>

namespace dm {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_BLOCKS = 64;        // one-shot grid
constexpr int XG2_BLOCKS = 256;      // two-shot grid (bandwidth-bound: more loads in flight)
constexpr int XG_FLAG_BLOCKS = 256;  // flag slots per phase

struct XgmiPtrs {
  float* data[XG_MAX_RANKS];        // each rank's shared buffer: [2][cap] floats (parity halves)
  unsigned* flags[XG_MAX_RANKS];    // each rank's flags: [2 phases][XG_FLAG_BLOCKS][XG_MAX_RANKS]
};

// block b announces `epoch` in slot (phase, b, rank) of every rank (remote stores over xGMI)
__device__ inline void xg_signal(const XgmiPtrs& p, int phase, int b, int rank, int W,
                                 unsigned epoch) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < W) {
    unsigned* f = p.flags[threadIdx.x] + (phase * XG_FLAG_BLOCKS + b) * XG_MAX_RANKS + rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

constexpr unsigned long long XG_TIMEOUT_TICKS = 400000000ull;  // 4 s at 100 MHz

// wait until every rank's slot (phase, b, q) carries >= epoch; bounded spin -> false when a
// peer never arrives (the caller reports through *err and exits instead of hanging the GPU)
__device__ inline bool xg_wait(const XgmiPtrs& p, int phase, int b, int rank, int W,
                               unsigned epoch) {
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if (threadIdx.x < W) {
    const unsigned* f = p.flags[rank] + (phase * XG_FLAG_BLOCKS + b) * XG_MAX_RANKS + threadIdx.x;
    // bounded by wall time (s_memrealtime: 100 MHz), not by a spin count: a peer may lag by
    // host work (logging, a checkpoint) or, with several ranks on one GPU, by the hardware
    // scheduler time-slicing their queues; 4 s still frees the GPU when one never comes
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > XG_TIMEOUT_TICKS) {
        timed_out = 1;
        break;
      }
    }
  }
  __syncthreads();
  const bool ok = !timed_out;
  __syncthreads();
  if (ok) __threadfence_system();
  return ok;
}

// epoch of this call: one past the last published one (read before this block can finish,
// so before the last block of the grid can publish)
__device__ inline unsigned xg_epoch(const unsigned* state) {
  return __hip_atomic_load(state + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
}

// every block calls this exactly once on every exit path; the last one publishes the epoch
__device__ inline void xg_finish(unsigned* state, unsigned epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(state + 2, 1u, __ATOMIC_ACQ_REL,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(state + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state + 1, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int VEC>
struct XgVec;
template <>
struct XgVec<1> {
  using T = float;
  static __device__ inline T add(T a, T b) { return a + b; }
  static __device__ inline T mul(T a, float s) { return a * s; }
};
template <>
struct XgVec<4> {
  using T = float4;
  static __device__ inline T add(T a, T b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
  static __device__ inline T mul(T a, float s) {
    return make_float4(a.x * s, a.y * s, a.z * s, a.w * s);
  }
};

// n, cap in units of VEC floats
template <int VEC>
__global__ void __launch_bounds__(256) xgmi_allreduce2_kernel(const float* __restrict__ in_,
                                                              float* __restrict__ out_, long long n,
                                                              long long cap, XgmiPtrs p, int rank,
                                                              int W, float scale,
                                                              unsigned* __restrict__ state) {
  using V = typename XgVec<VEC>::T;
  const unsigned epoch = xg_epoch(state);
  const V* in = reinterpret_cast<const V*>(in_);
  V* out = reinterpret_cast<V*>(out_);
  const int b = blockIdx.x, G = gridDim.x;
  const long long S = (n + W - 1) / W, C = (S + G - 1) / G;
  const long long half = (long long)(epoch & 1u) * cap;
  auto buf = [&](int q) { return reinterpret_cast<V*>(p.data[q]) + half; };
  auto range = [&](int q, long long& lo, long long& hi) {
    lo = q * S + b * C;
    long long e = (q + 1) * S < n ? (q + 1) * S : n;
    hi = lo + C < e ? lo + C : e;
  };
  V* mine = buf(rank);
  long long lo, hi;
  for (int q = 0; q < W; ++q) {
    range(q, lo, hi);
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = in[i];
  }
  xg_signal(p, 0, b, rank, W, epoch);
  if (!xg_wait(p, 0, b, rank, W, epoch)) {
    if (threadIdx.x == 0) atomicExch(state, 1u);
    xg_finish(state, epoch);
    return;
  }
  range(rank, lo, hi);
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    V s = buf(0)[i];
    for (int q = 1; q < W; ++q) s = XgVec<VEC>::add(s, buf(q)[i]);
    s = XgVec<VEC>::mul(s, scale);
    mine[i] = s;
    out[i] = s;
  }
  xg_signal(p, 1, b, rank, W, epoch);
  if (!xg_wait(p, 1, b, rank, W, epoch)) {
    if (threadIdx.x == 0) atomicExch(state, 1u);
    xg_finish(state, epoch);
    return;
  }
  for (int q = 0; q < W; ++q) {
    if (q == rank) continue;
    const V* src = buf(q);
    range(q, lo, hi);
    for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) out[i] = src[i];
  }
  xg_finish(state, epoch);
}

__global__ void __launch_bounds__(256) xgmi_allreduce_kernel(const float* __restrict__ in,
                                                             float* __restrict__ out, long long n,
                                                             long long cap, XgmiPtrs p, int rank,
                                                             int W, float scale,
                                                             unsigned* __restrict__ state) {
  const int b = blockIdx.x;
  const unsigned epoch = xg_epoch(state);
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long lo = b * per, hi = lo + per < n ? lo + per : n;
  const long long half = (long long)(epoch & 1u) * cap;
  float* mine = p.data[rank] + half;
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = in[i];
  xg_signal(p, 0, b, rank, W, epoch);
  // >=: a fast peer may already have stored epoch+1 (it then waits for OUR epoch+1 flag,
  // so it cannot reach epoch+2 and overwrite the parity half this call reads)
  if (!xg_wait(p, 0, b, rank, W, epoch)) {
    if (threadIdx.x == 0) atomicExch(state, 1u);
    xg_finish(state, epoch);
    return;
  }
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < W; ++q) s += p.data[q][half + i];
    out[i] = s * scale;
  }
  xg_finish(state, epoch);
}

void* xgmi_alloc(size_t bytes) {
  void* ptr = nullptr;
  DM_CHECK(hipExtMallocWithFlags(&ptr, bytes, hipDeviceMallocUncached));
  DM_CHECK(hipMemset(ptr, 0, bytes));
  DM_CHECK(hipDeviceSynchronize());
  return ptr;
}

void xgmi_free(void* ptr) { DM_CHECK(hipFree(ptr)); }

void xgmi_get_handle(void* ptr, void* handle64) {
  hipIpcMemHandle_t h;
  DM_CHECK(hipIpcGetMemHandle(&h, ptr));
  static_assert(sizeof(h) == 64, "IPC handle size");
  std::memcpy(handle64, &h, sizeof(h));
}

void* xgmi_open_handle(const void* handle64) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle64, sizeof(h));
  void* ptr = nullptr;
  DM_CHECK(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess));
  return ptr;
}

void xgmi_close_handle(void* ptr) { DM_CHECK(hipIpcCloseMemHandle(ptr)); }

// share: ranks whose kernels run on this same GPU (1 on a node with one rank per GPU).  Every
// block of the spinning kernels must be resident together with its namesakes on the peers;
// W ranks sharing one device divide its CUs, so the grids shrink by that factor
void xgmi_allreduce(const float* in, float* out, long long n, long long cap, void* const* data,
                    void* const* flags, int rank, int W, float scale, unsigned* state, int algo,
                    hipStream_t st, int share) {
  if (share < 1) share = 1;
  const int g1 = XG_BLOCKS / share > 8 ? XG_BLOCKS / share : 8;
  const int g2 = XG2_BLOCKS / share > 16 ? XG2_BLOCKS / share : 16;
  XgmiPtrs p{};
  for (int q = 0; q < W; ++q) {
    p.data[q] = (float*)data[q];
    p.flags[q] = (unsigned*)flags[q];
  }
  if (algo == 0) {
    xgmi_allreduce_kernel<<<g1, 256, 0, st>>>(in, out, n, cap, p, rank, W, scale,
                                                     state);
    return;
  }
  // two-shot: float4 when every rank's view is 16-B aligned (cap % 4 == 0 keeps the parity
  // halves aligned; the caller checks n % 4 and the tensor addresses)
  const bool v4 = n % 4 == 0 && cap % 4 == 0 && ((uintptr_t)in % 16) == 0 &&
                  ((uintptr_t)out % 16) == 0;
  if (v4)
    xgmi_allreduce2_kernel<4><<<g2, 256, 0, st>>>(in, out, n / 4, cap / 4, p, rank, W,
                                                          scale, state);
  else
    xgmi_allreduce2_kernel<1><<<g2, 256, 0, st>>>(in, out, n, cap, p, rank, W, scale,
                                                          state);
}

}  // namespace dm
