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
#include "common.h"

#include <cstring>

namespace dm {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_BLOCKS = 64;

struct XgmiPtrs {
  float* data[XG_MAX_RANKS];        // each rank's shared buffer: [2][cap] floats (parity halves)
  unsigned* flags[XG_MAX_RANKS];    // each rank's flag array: [XG_BLOCKS][XG_MAX_RANKS]
};

__global__ void __launch_bounds__(256) xgmi_allreduce_kernel(const float* __restrict__ in,
                                                             float* __restrict__ out, long long n,
                                                             long long cap, XgmiPtrs p, int rank,
                                                             int W, unsigned epoch, float scale,
                                                             int* __restrict__ err) {
  const int b = blockIdx.x;
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long lo = b * per, hi = lo + per < n ? lo + per : n;
  const long long half = (long long)(epoch & 1u) * cap;
  float* mine = p.data[rank] + half;
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) mine[i] = in[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x < W) {
    unsigned* f = p.flags[threadIdx.x] + b * XG_MAX_RANKS + rank;
    __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // wait for every rank's slice b of this epoch
  __shared__ int timed_out;
  if (threadIdx.x == 0) timed_out = 0;
  __syncthreads();
  if (threadIdx.x < W) {
    const unsigned* f = p.flags[rank] + b * XG_MAX_RANKS + threadIdx.x;
    long long spins = 0;
    // >=: a fast peer may already have stored epoch+1 (it then waits for OUR epoch+1 flag,
    // so it cannot reach epoch+2 and overwrite the parity half this call reads)
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1LL << 22)) {  // ~0.5-1 s: a peer is missing -> report, do not hang
        timed_out = 1;
        break;
      }
    }
  }
  __syncthreads();
  if (timed_out) {
    if (threadIdx.x == 0) atomicExch(err, 1);
    return;
  }
  __threadfence_system();
  for (long long i = lo + threadIdx.x; i < hi; i += blockDim.x) {
    float s = 0.f;
    for (int q = 0; q < W; ++q) s += p.data[q][half + i];
    out[i] = s * scale;
  }
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

void xgmi_allreduce(const float* in, float* out, long long n, long long cap, void* const* data,
                    void* const* flags, int rank, int W, unsigned epoch, float scale, int* err,
                    hipStream_t st) {
  XgmiPtrs p{};
  for (int q = 0; q < W; ++q) {
    p.data[q] = (float*)data[q];
    p.flags[q] = (unsigned*)flags[q];
  }
  xgmi_allreduce_kernel<<<XG_BLOCKS, 256, 0, st>>>(in, out, n, cap, p, rank, W, epoch, scale, err);
}

}  // namespace dm
