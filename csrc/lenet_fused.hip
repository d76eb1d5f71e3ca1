// Fused LeNet training step (the reference `Net`, codes/task1/pytorch/model.py:12-35, trained by
// the task3 loop, codes/task3/model.py:50-64), gfx950.
//
// The reference step is ~50-70 kernel launches; the layer-by-layer native
// Program was 22 dispatches / 206 us at batch 32 (profiles/rocprof_lenet_b32_step_r2c.txt).
// The whole model is 78 MFLOP per step: the step is launch- and latency-bound, so it is
// restructured around the batch dimension instead of the layers:
//
//  K1 lenet_sample_kernel — ONE workgroup per sample runs the entire forward AND backward of
//     that sample in LDS: conv1+bias+ReLU+2x2 max-pool, conv2+bias+ReLU+pool, fc1+ReLU, fc2,
//     softmax cross-entropy (loss and the (softmax - onehot)/B seed), fc2/fc1 data gradients,
//     unpooling through the argmax codes, the conv2 data gradient, and the per-sample
//     conv1/conv2 weight- and bias-gradient contributions.  Everything a layer hands to the
//     next stays in LDS; the only global traffic is the input, the weights (L2-resident,
//     207 KB) and a per-sample record for K2: h0 (400), h1 (120), dh1 (120), dlogits (10)
//     and the conv gradient partials (2572 floats).
//  K2 lenet_grad_kernel — one thread per parameter (51,902): the batch reduction of every
//     gradient in a fixed order (deterministic; fc weights as sum_b dY[b] (x) X[b] rank-1
//     terms from the K1 records, conv weights as sums of the per-sample partials), written
//     into the flat gradient buffer, optionally followed in the same thread by the SGD
//     (momentum / dampening / nesterov / weight decay) update of that parameter, and the mean
//     loss (block 0).  With data parallelism K2 writes gradients only; the bucket all-reduce
//     and the fused SGD kernel (optim.hip) follow.
//
// So a single-GPU training step is 2 dispatches (3 with DDP, plus the collective), none of
// them ATen.  All accumulation is fp32; the bf16 variant reads bf16 input images.
#include "common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int LT = 1024;  // threads per sample workgroup (16 waves: the long phases split)
// per-sample conv gradient partials: conv2 w (2400), conv2 b (16), conv1 w (150), conv1 b (6)
constexpr int CS = 2400 + 16 + 150 + 6;
constexpr int NPROBE = 16;

template <typename XT>
__device__ __forceinline__ float ldx(const XT* p);
template <>
__device__ __forceinline__ float ldx<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ldx<bf16_t>(const bf16_t* p) { return bf2f(*p); }

template <bool PROBE>
__device__ __forceinline__ void probe_stamp(unsigned long long* probe, int b, int tid, int k) {
  if constexpr (PROBE) {
    if (tid == 0 && k < NPROBE) probe[(long long)b * NPROBE + k] = __builtin_amdgcn_s_memrealtime();
  }
}

template <typename XT, bool PROBE>
__global__ void __launch_bounds__(LT) lenet_sample_kernel(
    const XT* __restrict__ X, const long long* __restrict__ labels,
    const float* __restrict__ c1w, const float* __restrict__ c1b, const float* __restrict__ c2w,
    const float* __restrict__ c2b, const float* __restrict__ f1w, const float* __restrict__ f1b,
    const float* __restrict__ f2w, const float* __restrict__ f2b, float* __restrict__ rec,
    float* __restrict__ cslab, float* __restrict__ rowloss, float inv_b,
    const long long* __restrict__ sidx, const int* __restrict__ cursor, long long nrows,
    unsigned long long* __restrict__ probe) {
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // probe (development, tools/lenet_phases.py; null otherwise): the 100 MHz real-time clock at
  // the start and after every phase barrier, NPROBE stamps per sample
  probe_stamp<PROBE>(probe, b, tid, 0);
  // device-resident loader: sample b of this step is dataset row sidx[cursor * B + b] (the
  // epoch's sampler order, uploaded once per epoch; the cursor advances on the device in the
  // gradient kernel, so a captured graph walks the epoch); clamped, never out of bounds
  long long row = b;
  if (sidx != nullptr) {
    const long long r = sidx[(long long)(*cursor) * gridDim.x + b];
    row = r < 0 ? 0 : (r >= nrows ? nrows - 1 : r);
  }
  __shared__ float xs[32 * 32];            // input with the conv1 zero padding (2)
  __shared__ float w1[152], bb1[8], w2[2400], bb2[16], fw2[1200], fb2[16];
  __shared__ float p1[6 * 196];            // relu(conv1) max-pooled
  __shared__ short pos1[6 * 196];          // xs offset of the window's argmax conv output
  __shared__ float p2[400];                // relu(conv2) max-pooled = h0 (flatten order)
  __shared__ short pos2[400];              // p1 offset of the argmax conv2 output
  __shared__ float h1[128], lg[16], dl[16], dh1[128], g2[400], g1[6 * 196];
  __shared__ float dc2[16 * 18 * 18];      // unpooled conv2 gradient, 4-pixel zero border
  __shared__ float4 red4[10 * 100];        // cross-thread partials (fc1 dgrad, conv2, conv1 dw)
  // cross-thread partials: conv2 forward [6 input channels][16][10][10], later the conv2 data
  // gradient [16 output channels][6][14][14] (the phases are separated by barriers)
  __shared__ float big[16 * 1176];
  float* pc2 = big;
  float* pdq = big;
  float* red = reinterpret_cast<float*>(red4);

  // ---- stage input and the small weights (fc1's 192 KB stream from L2 instead) ----
  for (int i = tid; i < 1024; i += LT) {
    const int y = (i >> 5) - 2, x = (i & 31) - 2;
    xs[i] = ((unsigned)y < 28u && (unsigned)x < 28u) ? ldx<XT>(X + row * 784 + y * 28 + x)
                                                     : 0.f;
  }
  for (int i = tid; i < 2400; i += LT) w2[i] = c2w[i];
  for (int i = tid; i < 1200; i += LT) fw2[i] = f2w[i];
  for (int i = tid; i < 16 * 18 * 18; i += LT) dc2[i] = 0.f;
  if (tid < 150) w1[tid] = c1w[tid];
  if (tid < 6) bb1[tid] = c1b[tid];
  if (tid < 16) bb2[tid] = c2b[tid];
  if (tid < 10) fb2[tid] = f2b[tid];
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 1);

  // ---- conv1 (1 -> 6, 5x5, pad 2) + bias + ReLU + 2x2 max-pool ----
  for (int q = tid; q < 1176; q += LT) {
    const int c = q / 196, r = q - c * 196, py = r / 14, px = r - py * 14;
    float win[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) win[i][j] = xs[(2 * py + i) * 32 + 2 * px + j];
    float best = 0.f;
    int code = -1;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int ay = a >> 1, ax = a & 1;
      float acc = bb1[c];
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc += win[ay + kh][ax + kw] * w1[c * 25 + kh * 5 + kw];
      if (acc > best) {  // first maximum; a window whose max is <= 0 passes no gradient
        best = acc;
        code = a;
      }
    }
    p1[q] = best;
    pos1[q] = code < 0 ? (short)-1 : (short)((2 * py + (code >> 1)) * 32 + 2 * px + (code & 1));
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 2);

  // ---- conv2 (6 -> 16, 5x5): item (input channel c, output channel o, row oy) computes
  //      the 10 outputs of one row from a 5 x 14 window read one row at a time (70 + 25 LDS
  //      reads for 250 FMAs), partial sums per input channel into pc2 ----
  if (tid < 960) {
    const int c = tid / 160, r160 = tid - c * 160, o = r160 / 10, oy = r160 - o * 10;
    const float* src = p1 + c * 196 + oy * 14;
    const float* wo = w2 + o * 150 + c * 25;
    float acc[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) acc[q] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh) {
      float row[14];
#pragma unroll
      for (int q = 0; q < 14; ++q) row[q] = src[kh * 14 + q];
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const float wv = wo[kh * 5 + kw];
#pragma unroll
        for (int q = 0; q < 10; ++q) acc[q] += row[q + kw] * wv;
      }
    }
    float* dst = pc2 + c * 1600 + o * 100 + oy * 10;
#pragma unroll
    for (int q = 0; q < 10; ++q) dst[q] = acc[q];
  }
  __syncthreads();
  // ---- + bias (channel partials summed in a fixed order) + ReLU + 2x2 max-pool ----
  if (tid < 400) {
    const int o = tid / 25, r = tid - o * 25, py = r / 5, px = r - py * 5;
    float best = 0.f;
    int code = -1;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int e = o * 100 + (2 * py + (a >> 1)) * 10 + 2 * px + (a & 1);
      float v = bb2[o];
#pragma unroll
      for (int c = 0; c < 6; ++c) v += pc2[c * 1600 + e];
      if (v > best) {  // first maximum; a window whose max is <= 0 passes no gradient
        best = v;
        code = a;
      }
    }
    p2[tid] = best;
    pos2[tid] = code < 0 ? (short)-1 : (short)((2 * py + (code >> 1)) * 14 + 2 * px + (code & 1));
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 3);

  // ---- fc1 (400 -> 120) + ReLU: 8 threads per output, thread p loading float4 columns
  //      p, p+8, ... of the row (all 12-13 in flight together; the 8 threads of an output
  //      read 128 contiguous bytes per step), combined by lane shuffles ----
  if (tid < 960) {
    const int u = tid >> 3, part = tid & 7;
    const float4* wr = reinterpret_cast<const float4*>(f1w + u * 400);
    const float4* hr = reinterpret_cast<const float4*>(p2);
    float4 wv[13];
#pragma unroll
    for (int j = 0; j < 13; ++j) wv[j] = part + 8 * j < 100 ? wr[part + 8 * j] : make_float4(0.f, 0.f, 0.f, 0.f);
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 13; ++j) {
      const float4 h = part + 8 * j < 100 ? hr[part + 8 * j] : make_float4(0.f, 0.f, 0.f, 0.f);
      acc += wv[j].x * h.x + wv[j].y * h.y + wv[j].z * h.z + wv[j].w * h.w;
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
    acc += __shfl_xor(acc, 4, 64);
    if (part == 0) h1[u] = fmaxf(acc + f1b[u], 0.f);
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 4);

  // ---- fc2 (120 -> 10) from LDS, one wave per output ----
  for (int o = wid; o < 10; o += LT / 64) {
    float acc = lane < 56 ? fw2[o * 120 + lane] * h1[lane] + fw2[o * 120 + 64 + lane] * h1[64 + lane]
                          : fw2[o * 120 + lane] * h1[lane];
    acc = wave_sum(acc);
    if (lane == 0) lg[o] = acc + fb2[o];
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 5);
  // ---- softmax cross-entropy: loss and the (softmax - onehot) / B seed ----
  if (wid == 0) {
    const float z = lane < 10 ? lg[lane] : -INFINITY;
    const float mx = wave_max(z);
    const float e = lane < 10 ? __expf(z - mx) : 0.f;
    const float se = wave_sum(e);
    const int lab = (int)labels[row];
    const float zl = __shfl(z, lab, 64);
    if (lane < 10) dl[lane] = (e / se - (lane == lab ? 1.f : 0.f)) * inv_b;
    if (lane == 0) rowloss[b] = mx + __logf(se) - zl;
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 6);

  // ---- fc2 data gradient, masked by fc1's ReLU ----
  if (tid < 120) {
    float acc = 0.f;
#pragma unroll
    for (int o = 0; o < 10; ++o) acc += dl[o] * fw2[o * 120 + tid];
    dh1[tid] = h1[tid] > 0.f ? acc : 0.f;
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 7);

  // ---- fc1 data gradient: thread (k4, u-group of 12) streams coalesced float4 rows ----
  if (tid < 1000) {
    const int k4 = tid % 100, ug = tid / 100;
    float4 wv[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) wv[j] = reinterpret_cast<const float4*>(f1w + (ug * 12 + j) * 400)[k4];
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      const float d = dh1[ug * 12 + j];
      a.x += d * wv[j].x;
      a.y += d * wv[j].y;
      a.z += d * wv[j].z;
      a.w += d * wv[j].w;
    }
    red4[ug * 100 + k4] = a;
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 8);
  float* r = rec + (long long)b * 656;  // per-sample record: h0 | h1 | dh1 | dl (+ pad)
  if (tid < 400) {
    float d = 0.f;
#pragma unroll
    for (int g = 0; g < 10; ++g) d += red[g * 400 + tid];
    const int ps = pos2[tid];
    const float gv = ps >= 0 ? d : 0.f;
    g2[tid] = gv;
    if (ps >= 0) {  // scatter into the unpooled, zero-bordered conv2 gradient
      const int o = tid / 25, y = ps / 14, x = ps - (ps / 14) * 14;
      dc2[o * 324 + (y + 4) * 18 + x + 4] = gv;
    }
    r[tid] = p2[tid];
  }
  if (tid < 120) {
    r[400 + tid] = h1[tid];
    r[520 + tid] = dh1[tid];
  }
  if (tid < 10) r[640 + tid] = dl[tid];
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 9);

  float* cs = cslab + (long long)b * CS;
  // ---- conv2 data gradient (full correlation of the unpooled, zero-bordered gradient dc2
  //      with the flipped kernel) on threads 0..447: thread (output channel o, row y, 7-column
  //      half) computes the 6 x 7 outputs of every input channel from one 5 x 11 window of
  //      dc2[o], read one row at a time (55 window + 150 weight reads for 1050 FMAs); the 16
  //      per-o partials are summed in a fixed order after the barrier ----
  // ---- conv2 weight gradient on threads 448..1023: item (o, c, kh) = the 5 taps kw of one
  //      kernel row, summed over the 25 argmax positions of channel o ----
  if (tid < 448) {
    const int o = tid / 28, r28 = tid - o * 28, y0 = r28 >> 1, x0 = 7 * (r28 & 1);
    float acc[6][7];
#pragma unroll
    for (int c = 0; c < 6; ++c)
#pragma unroll
      for (int q = 0; q < 7; ++q) acc[c][q] = 0.f;
    const float* d = dc2 + o * 324 + y0 * 18 + x0;
#pragma unroll 1
    for (int kh = 0; kh < 5; ++kh) {  // output row y0 reads window row 4 - kh
      float row[11];
#pragma unroll
      for (int q = 0; q < 11; ++q) row[q] = d[(4 - kh) * 18 + q];
#pragma unroll
      for (int c = 0; c < 6; ++c)
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const float wv = w2[o * 150 + c * 25 + kh * 5 + kw];
#pragma unroll
          for (int q = 0; q < 7; ++q) acc[c][q] += row[q + 4 - kw] * wv;
        }
    }
    float* pg = pdq + o * 1176 + y0 * 14 + x0;
#pragma unroll
    for (int c = 0; c < 6; ++c)
#pragma unroll
      for (int q = 0; q < 7; ++q) pg[c * 196 + q] = acc[c][q];
  } else {
    for (int i = tid - 448; i < 480; i += LT - 448) {
      const int o = i / 30, r30 = i - o * 30, c = r30 / 5, kh = r30 - c * 5;
      const float* pc = p1 + c * 196 + kh * 14;
      float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 5
      for (int j = 0; j < 25; ++j) {
        const int ps = pos2[o * 25 + j];
        const float gv = g2[o * 25 + j];
        const float* q = pc + (ps < 0 ? 0 : ps);
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) acc[kw] += gv * q[kw];
      }
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) cs[o * 150 + c * 25 + kh * 5 + kw] = acc[kw];
    }
    if (tid >= 1008) {  // conv2 bias: 16 channels
      const int o = tid - 1008;
      float acc = 0.f;
      for (int j = 0; j < 25; ++j) acc += g2[o * 25 + j];
      cs[2400 + o] = acc;
    }
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 10);
  for (int idx = tid; idx < 1176; idx += LT) {  // output-channel partials in order, unpool1
    float sacc = 0.f;
#pragma unroll
    for (int o = 0; o < 16; ++o) sacc += pdq[o * 1176 + idx];
    g1[idx] = pos1[idx] >= 0 ? sacc : 0.f;
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 11);

  // ---- conv1 weight/bias gradient partials: 150 weights x 196 pooled positions, 6 threads
  //      per weight, combined in a fixed order ----
  if (tid < 900) {
    const int i = tid / 6, part = tid - i * 6;
    const int c = i / 25, t = i - c * 25, kh = t / 5, kw = t - kh * 5;
    const float* xc = xs + kh * 32 + kw;
    float acc = 0.f;
#pragma unroll 4
    for (int j = part; j < 196; j += 6) {
      const int ps = pos1[c * 196 + j];
      acc += g1[c * 196 + j] * xc[ps < 0 ? 0 : ps];
    }
    red[tid] = acc;
  }
  __syncthreads();
  probe_stamp<PROBE>(probe, b, tid, 12);
  if (tid < 150)
    cs[2416 + tid] = red[6 * tid] + red[6 * tid + 1] + red[6 * tid + 2] + red[6 * tid + 3] +
                     red[6 * tid + 4] + red[6 * tid + 5];
  if (tid >= 192 && tid < 192 + 6 * 32) {  // conv1 bias: 6 channels x 32 lanes
    const int c = (tid - 192) >> 5, l = (tid - 192) & 31;
    float acc = 0.f;
    for (int j = l; j < 196; j += 32) acc += g1[c * 196 + j];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 32);
    if (l == 0) cs[2566 + c] = acc;
  }
  probe_stamp<PROBE>(probe, b, tid, 13);
}

// Flat-buffer segment j (fc2.w, fc2.b, fc1.w, fc1.b, conv2.w, conv2.b, conv1.w, conv1.b in the
// Program's reverse-execution order) starts at off[j].
struct LenetFlat {
  int off[8];
};
__device__ __forceinline__ int seg_n(int s) {
  switch (s) {
    case 0: return 1200;
    case 1: return 10;
    case 2: return 48000;
    case 3: return 120;
    case 4: return 2400;
    case 5: return 16;
    case 6: return 150;
    default: return 6;
  }
}

__global__ void __launch_bounds__(256) lenet_grad_kernel(
    const float* __restrict__ rec, const float* __restrict__ cslab, int B, float* __restrict__ grad,
    LenetFlat fl, float* __restrict__ p, float* __restrict__ mom, float lr, float momentum,
    float dampening, float wd, float gscale, int nesterov, int first, int do_sgd,
    const float* __restrict__ rowloss, float* __restrict__ loss, int* __restrict__ cursor,
    int nbatch, float* __restrict__ loss_sum) {
  // two lanes per parameter: each sums half of the batch (16 loads in flight), the halves
  // are added by a lane shuffle in a fixed order
  const int half = threadIdx.x & 1;
  int i = blockIdx.x * 128 + (threadIdx.x >> 1);
  const int bh = (B + 1) >> 1, blo = half ? bh : 0, bhi = half ? B : bh;
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // mean loss, fixed order
    float a = 0.f;
    for (int j = threadIdx.x; j < B; j += 64) a += rowloss[j];
    a = wave_sum(a);
    if (threadIdx.x == 0) {
      *loss = a / (float)B;
      if (loss_sum != nullptr) *loss_sum += a / (float)B;  // device-side running sum (logging)
      // next batch of the epoch (the sample kernel that read the cursor has finished)
      if (cursor != nullptr) *cursor = (*cursor + 1 >= nbatch) ? 0 : *cursor + 1;
    }
  }
  int seg = 0;
  while (seg < 8 && i >= seg_n(seg)) {
    i -= seg_n(seg);
    ++seg;
  }
  if (seg == 8) return;
  float g = 0.f;
  if (seg == 0) {  // fc2.w[o][u] = sum_b dl[b][o] h1[b][u]
    const int o = i / 120, u = i - o * 120;
#pragma unroll 16
    for (int b = blo; b < bhi; ++b) g += rec[b * 656 + 640 + o] * rec[b * 656 + 400 + u];
  } else if (seg == 1) {
    for (int b = blo; b < bhi; ++b) g += rec[b * 656 + 640 + i];
  } else if (seg == 2) {  // fc1.w[u][k] = sum_b dh1[b][u] h0[b][k]
    const int u = i / 400, k = i - u * 400;
#pragma unroll 16
    for (int b = blo; b < bhi; ++b) g += rec[b * 656 + 520 + u] * rec[b * 656 + k];
  } else if (seg == 3) {
    for (int b = blo; b < bhi; ++b) g += rec[b * 656 + 520 + i];
  } else {
    const int base = seg == 4 ? 0 : seg == 5 ? 2400 : seg == 6 ? 2416 : 2566;
#pragma unroll 16
    for (int b = blo; b < bhi; ++b) g += cslab[(long long)b * CS + base + i];
  }
  g += __shfl_xor(g, 1, 64);  // both lanes: first half + second half
  if (half) return;
  const int o = fl.off[seg] + i;
  grad[o] = g;
  if (!do_sgd) return;
  float d = g * gscale;
  const float pv = p[o];
  if (wd != 0.f) d += wd * pv;
  if (momentum != 0.f) {
    const float bv = first ? d : momentum * mom[o] + (1.f - dampening) * d;
    mom[o] = bv;
    d = nesterov ? d + momentum * bv : bv;
  }
  p[o] = pv - lr * d;
}
}  // namespace

int lenet_record_floats() { return 656; }
int lenet_slab_floats() { return CS; }
int lenet_probe_stamps() { return NPROBE; }

void lenet_fused_step(const void* x, bool x_bf16, const long long* labels, int B,
                      const float* const* w, float* rec, float* cslab, float* rowloss, float* grad,
                      const int* off, float* p, float* mom, float lr, float momentum,
                      float dampening, float wd, float gscale, bool nesterov, bool first,
                      bool do_sgd, float* loss, const long long* sidx, int* cursor,
                      long long nrows, int nbatch, float* loss_sum, hipStream_t st,
                      unsigned long long* probe) {
  const float inv_b = 1.f / (float)B;
  // the probed variant is a separate instantiation: the normal kernel carries none of it
  if (x_bf16) {
    auto k = probe ? lenet_sample_kernel<bf16_t, true> : lenet_sample_kernel<bf16_t, false>;
    k<<<B, LT, 0, st>>>((const bf16_t*)x, labels, w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7],
                        rec, cslab, rowloss, inv_b, sidx, cursor, nrows, probe);
  } else {
    auto k = probe ? lenet_sample_kernel<float, true> : lenet_sample_kernel<float, false>;
    k<<<B, LT, 0, st>>>((const float*)x, labels, w[0], w[1], w[2], w[3], w[4], w[5], w[6], w[7],
                        rec, cslab, rowloss, inv_b, sidx, cursor, nrows, probe);
  }
  DM_CHECK(hipGetLastError());
  LenetFlat fl;
  for (int j = 0; j < 8; ++j) fl.off[j] = off[j];
  const int total = 1200 + 10 + 48000 + 120 + 2400 + 16 + 150 + 6;
  lenet_grad_kernel<<<(2 * total + 255) / 256, 256, 0, st>>>(rec, cslab, B, grad, fl, p, mom, lr,
                                                         momentum, dampening, wd, gscale,
                                                         nesterov ? 1 : 0, first ? 1 : 0,
                                                         do_sgd ? 1 : 0, rowloss, loss,
                                                         sidx != nullptr ? cursor : nullptr,
                                                         nbatch, loss_sum);
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
