// Stage-to-stage point-to-point transport over xGMI peer memory (lab 4 pipeline), gfx950.
//
// SURVEY §2.7 asks for a native stage transport (`comm/p2p.cpp`): the reference relays every
// activation through the driver process over TensorPipe RPC (codes/task4/model.py:57-60, 82),
// and RCCL send/recv pairs serialise on one communicator stream per peer pair.
//
// A channel carries messages in ONE direction, sender S -> receiver R.  R owns the landing
// zone: an IPC-shared, uncached ring of NSLOT slots of `cap` bytes plus a `full` flag per
// slot; S owns a small IPC-shared `free` (ack) array.  Message i uses slot i % NSLOT:
//   send (on S's stream): wait until free[slot] >= i - NSLOT + 1 (R has consumed message
//     i - NSLOT from that slot), copy the payload into R's slot (remote stores over xGMI),
//     system-scope release, then the LAST block to finish stores full[slot] = i + 1;
//   recv (on R's stream): every block waits until full[slot] >= i + 1 (acquire), copies its
//     share of the slot into the destination tensor, and the last block stores
//     free[slot] = i + 1 into S's ack array (remote store).
// The message counter i lives on the device (state[0]; state[1] = done-block counter,
// state[2] = timeout flag), advanced by the last block of each call, so a captured hipGraph
// replays correctly.  Waits are bounded: a peer that never arrives sets the timeout flag and
// the kernel exits instead of hanging the GPU.  Up to NSLOT messages can be in flight per
// channel, so a receiver can post its receives ahead of the compute that needs them (the
// pipeline's prefetch) without blocking the sender.
#include "common.h"

namespace dm {

namespace {
constexpr int P2P_BLOCKS = 32;

// bounded by wall time (s_memrealtime, 100 MHz): the peer stage may be busy with its own
// compute for a while; 8 s still frees the GPU when it never sends
constexpr unsigned long long P2P_TIMEOUT_TICKS = 800000000ull;

__device__ inline bool p2p_wait_ge(const unsigned* f, unsigned v, unsigned* state) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - v) < 0) {
    __builtin_amdgcn_s_sleep(2);
    if (__builtin_amdgcn_s_memrealtime() - t0 > P2P_TIMEOUT_TICKS) {
      atomicExch(state + 2, 1u);
      return false;
    }
  }
  return true;
}

// call counter (read by every block before the last one can advance it)
__device__ inline unsigned p2p_seq(const unsigned* state) {
  return __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every block arrives once; the last one runs `last` and advances the call counter
template <typename F>
__device__ inline void p2p_finish(unsigned* state, unsigned seq, F last) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev =
        __hip_atomic_fetch_add(state + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      last();
      __hip_atomic_store(state + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state, seq + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__global__ void __launch_bounds__(256) p2p_send_kernel(const uint4* __restrict__ src, long long n16,
                                                        uint4* ring, unsigned* full,
                                                        const unsigned* free_, long long slot16,
                                                        int nslot, unsigned* state) {
  const unsigned seq = p2p_seq(state);
  const int slot = (int)(seq % (unsigned)nslot);
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    if (seq >= (unsigned)nslot) ok = p2p_wait_ge(free_ + slot, seq - nslot + 1u, state);
  }
  __syncthreads();
  if (ok) {
    uint4* dst = ring + (long long)slot * slot16;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (long long)gridDim.x * blockDim.x)
      dst[i] = src[i];
    __threadfence_system();
  }
  p2p_finish(state, seq, [&]() {
    __threadfence_system();
    if (ok) __hip_atomic_store(full + slot, seq + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  });
}

__global__ void __launch_bounds__(256) p2p_recv_kernel(uint4* __restrict__ dst, long long n16,
                                                        const uint4* ring, const unsigned* full,
                                                        unsigned* free_, long long slot16,
                                                        int nslot, unsigned* state) {
  const unsigned seq = p2p_seq(state);
  const int slot = (int)(seq % (unsigned)nslot);
  __shared__ int ok;
  if (threadIdx.x == 0) ok = p2p_wait_ge(full + slot, seq + 1u, state);
  __syncthreads();
  if (ok) {
    __threadfence_system();
    const uint4* src = ring + (long long)slot * slot16;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (long long)gridDim.x * blockDim.x)
      dst[i] = src[i];
  }
  p2p_finish(state, seq, [&]() {
    __threadfence_system();
    __hip_atomic_store(free_ + slot, seq + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  });
}
}  // namespace

// bytes: payload size (multiple of 16); slot_bytes: ring slot size (multiple of 16)
void p2p_xgmi_send(const void* src, long long bytes, void* ring, void* full, const void* free_,
                   long long slot_bytes, int nslot, unsigned* state, hipStream_t st) {
  const long long n16 = bytes / 16;
  int blocks = (int)((n16 + 255) / 256);
  blocks = blocks < 1 ? 1 : blocks > P2P_BLOCKS ? P2P_BLOCKS : blocks;
  p2p_send_kernel<<<blocks, 256, 0, st>>>((const uint4*)src, n16, (uint4*)ring, (unsigned*)full,
                                          (const unsigned*)free_, slot_bytes / 16, nslot, state);
  DM_CHECK(hipGetLastError());
}

void p2p_xgmi_recv(void* dst, long long bytes, const void* ring, const void* full, void* free_,
                   long long slot_bytes, int nslot, unsigned* state, hipStream_t st) {
  const long long n16 = bytes / 16;
  int blocks = (int)((n16 + 255) / 256);
  blocks = blocks < 1 ? 1 : blocks > P2P_BLOCKS ? P2P_BLOCKS : blocks;
  p2p_recv_kernel<<<blocks, 256, 0, st>>>((uint4*)dst, n16, (const uint4*)ring,
                                          (const unsigned*)full, (unsigned*)free_, slot_bytes / 16,
                                          nslot, state);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
