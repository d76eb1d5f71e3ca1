// Halo conv, LDS-DMA pipeline ("h5"): unit-stride tap grids (3x3/s1 forward and dgrad), gfx950.
//
// Same decomposition as conv_halo.hip — a block owns BMH consecutive output pixels, the input
// halo of one 64-channel chunk is staged once and all taps read their A fragments from it,
// only the BN x 64 weight tile changes per (chunk, tap) step — but the staging pipeline is
// rebuilt around buffer_load ... lds (LDS-DMA) instead of register staging:
//
//  * every staged byte goes HBM/L2 -> LDS directly: no staging VGPRs, no ds_write pass, no
//    waits on the loads before the stores (conv_halo.hip's per-step critical path);
//  * the weight tiles run in a 3-deep LDS ring: step s computes from buffer s%3 while tile s+1
//    is in flight (issued one step earlier) and tile s+2 is issued at the top of step s; a
//    COUNTED `s_waitcnt vmcnt(N)` before the step's one barrier retires only tile s+1 (N =
//    the DMA instructions issued after it), so loads stay in flight across barriers;
//  * the halo is double-buffered: chunk c+1's halo is issued at the first tap of chunk c and
//    retired by the same counted waits, 9 steps later for a 3x3 conv;
//  * 8 waves (512 threads) per block, one block per CU: BMH x BN = 256 x 128 as 4 x 2 waves of
//    64 x 64 (v_mfma_f32_32x32x16_bf16, 2 x 2 per wave, 16 MFMAs per wave per step), or
//    512 x 64 as 8 x 1 waves for the single-chunk 64-channel layer;
//  * the LDS image is lane-linear per DMA instruction (base + lane*16); the bank swizzle is
//    applied to the SOURCE address (lane (row, p) fetches chunk p ^ f(row)) and to the
//    fragment reads, so every read sees the same XOR layout as conv_halo.hip (swz()).
//
// Fused pre-BN (PRE): the operand is relu(y*sc + sh) of the previous conv's raw output.  Each
// thread normalises, in place, exactly the 16-B chunks its own DMA instructions wrote, after
// its counted wait and before the barrier that publishes them (scale/shift for all C channels
// are staged in LDS once).  Out-of-image taps still read the zero row.
//
// The loop holds no ordinary global load (only DMA and LDS traffic), so the compiler's own
// waits cannot drain the DMA queue; the barrier is a raw s_barrier preceded by lgkmcnt(0)
// (this wave's fragment reads of the buffer that the next step refills are complete).
#include "common.h"
#include "conv_geom.h"
#include "igemm_common.h"
#include "kernels.h"

namespace dm {

namespace {
constexpr int H5K = 64;  // channels per chunk: one 128-B LDS row per pixel
constexpr unsigned H5OOB = 0x80000000u;

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// buffer descriptor: base, stride 0, num_records = bytes (out-of-range offsets read as 0)
__device__ __forceinline__ i32x4 make_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  i32x4 r;
  r[0] = (int)(unsigned)a;
  r[1] = (int)(unsigned)(a >> 32) & 0xffff;
  r[2] = (int)bytes;
  r[3] = 0x00020000;
  return r;
}

// One 16-B-per-lane LDS-DMA (buffer_load_dwordx4 ... lds): lane l's 16 bytes at byte `off`
// of the buffer land at LDS byte m0 + 16*l.  Issued from inline asm so the compiler does not
// track it: its alias-blind LDS-DMA bookkeeping would otherwise wait vmcnt(0) before the
// first ds_read after every DMA (measured in the .s), draining the pipeline each step.  The
// kernel retires these loads itself with counted vmcnt waits.  M0 is written in the same
// statement (compiler-reserved, not preserved across statements).
__device__ __forceinline__ void lds_dma16(const i32x4& rs, const void* lds_wave_base, unsigned off) {
  const unsigned lds =
      __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds_wave_base);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %0, %2, 0 offen lds"
      :
      : "v"(off), "s"(lds), "s"(rs)
      : "memory");
}

// BMH output pixels x BN output channels per block, WM x WN waves; HRI halo DMA instructions
// per thread (halo capacity HRI * NW * 8 rows); NHB halo buffers (1: single-chunk layers)
template <int BN, int WM, int WN, int BMH, int HRI, int NHB, bool PRE>
__global__ void __launch_bounds__(WM * WN * 64) conv_h5_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp, bf16_t* Y, const bf16_t* ADD,
    float* __restrict__ stats, ConvGeom g, unsigned xbytes, unsigned wbytes,
    const float* __restrict__ pre_sc, const float* __restrict__ pre_sh, BnBwdEpi bnb) {
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int TM = BMH / WM, TN = BN / WN;
  constexpr int RM = TM / 32, RN = TN / 32;
  constexpr int HP = HRI * NW * 8;       // halo rows per buffer (+1 zero row after them)
  constexpr int BI = BN * 8 / NT;        // weight-tile DMA instructions per thread
  constexpr int NB = 3;                  // weight-tile ring depth
  static_assert(BI >= 1 && BI * NT == BN * 8, "weight tile = whole DMA rounds");
  static_assert(RM >= 1 && RN >= 1 && TM % 32 == 0 && TN % 32 == 0, "wave tile");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* Hs = reinterpret_cast<bf16_t*>(smem);              // [NHB][HP + 1][64]
  bf16_t* Bs = Hs + NHB * (HP + 1) * H5K;                    // [NB][BN][64]
  int4* taps = reinterpret_cast<int4*>(Bs + NB * BN * H5K);  // [MAXTAPS]
  float* psc = reinterpret_cast<float*>(taps + MAXTAPS);     // [C] (PRE)
  float* psh = psc + g.C;                                    // [C] (PRE)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const long long m0 = (long long)blockIdx.x * BMH;
  const int n0 = blockIdx.y * BN;
  const int ntaps = g.nth * g.ntw;
  const int nchunk = g.C / H5K;
  const int HW = g.H * g.W;
  const int NHW = g.N * HW;
  if (tid < ntaps) {
    const int th = tid / g.ntw, tw = tid % g.ntw;
    const int dy = g.dy0 + th * g.dys, dx = g.dx0 + tw * g.dxs;
    taps[tid] = make_int4(dy, dx, ((g.kh0 + th * g.khs) * g.KW + (g.kw0 + tw * g.kws)) * g.C,
                          dy * g.W + dx);
  }
  if (tid < 8 * NHB)
    *reinterpret_cast<uint4*>(Hs + ((tid >> 3) * (HP + 1) + HP) * H5K + (tid & 7) * 8) =
        make_uint4(0, 0, 0, 0);
  if constexpr (PRE) {
    for (int c = tid; c < g.C; c += NT) {
      psc[c] = pre_sc[c];
      psh[c] = pre_sh[c];
    }
  }

  // halo extent (flattened rows r0-1 .. r1+1)
  const int r0 = (int)fdiv((unsigned)m0, g.wg_mul, g.wg_shr);
  const long long mlast = (m0 + BMH - 1 < g.M) ? m0 + BMH - 1 : g.M - 1;
  const int r1 = (int)fdiv((unsigned)mlast, g.wg_mul, g.wg_shr);
  const int hbase = (r0 - 1) * g.W;
  const int hp = (r1 - r0 + 3) * g.W;

  const i32x4 rsx = make_rsrc(X, xbytes);
  const i32x4 rsw = make_rsrc(Wp, wbytes);
  // DMA lane geometry: instruction i of wave w fills LDS rows (i*NW + w)*8 + lane/8, chunk
  // position lane%8, with the source chunk pre-swizzled so the image equals swz() layout
  const int drow = lane >> 3, dpos = lane & 7;

  // per-lane A-fragment rows: halo row of the centre tap and the pixel coordinates
  int a_h[RM], a_x[RM], a_y[RM];
#pragma unroll
  for (int i = 0; i < RM; ++i) {
    const long long m = m0 + wm * TM + i * 32 + (lane & 31);
    const unsigned r = fdiv((unsigned)m, g.wg_mul, g.wg_shr);
    a_x[i] = (int)((unsigned)m - r * (unsigned)g.W);
    const unsigned n = fdiv(r, g.hg_mul, g.hg_shr);
    a_y[i] = (m < g.M) ? (int)(r - n * (unsigned)g.H) : -(1 << 28);  // rows >= M: never valid
    a_h[i] = (int)(m - hbase);
  }
  unsigned b_off[BI];
  int b_gc[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int r = (i * NW + wid) * 8 + drow;
    const int n = n0 + r;
    b_gc[i] = dpos ^ ((r >> 1) & 7);
    b_off[i] = n < g.Ncols ? (unsigned)n * (unsigned)g.wK * 2u + (unsigned)b_gc[i] * 16u : H5OOB;
  }
  __syncthreads();  // taps, zero rows, scale/shift visible

  auto issue_halo = [&](int cc, int hb) {
    bf16_t* hs = Hs + hb * (HP + 1) * H5K;
#pragma unroll
    for (int j = 0; j < HRI; ++j) {
      const int hh = (j * NW + wid) * 8 + drow;
      const int gp = hbase + hh;
      const int gc = dpos ^ ((hh >> 1) & 7);
      const bool ok = hh < hp && (unsigned)gp < (unsigned)NHW;
      const unsigned off = ok ? (unsigned)gp * (unsigned)g.C * 2u + (unsigned)(cc * H5K + gc * 8) * 2u
                              : H5OOB;
      lds_dma16(rsx, hs + (j * NW + wid) * 8 * H5K, off);
    }
  };
  auto issue_b = [&](int cc, int t, int b) {
    bf16_t* bs = Bs + b * BN * H5K;
    const unsigned kb = (unsigned)(taps[t].z + cc * H5K) * 2u;
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const unsigned off = b_off[i] != H5OOB ? b_off[i] + kb : H5OOB;
      lds_dma16(rsw, bs + (i * NW + wid) * 8 * H5K, off);
    }
  };
  // PRE: normalise the chunks this thread's halo DMA wrote (after its wait retired them)
  auto normalise_halo = [&](int cc, int hb) {
    if constexpr (PRE) {
      bf16_t* hs = Hs + hb * (HP + 1) * H5K;
#pragma unroll
      for (int j = 0; j < HRI; ++j) {
        const int hh = (j * NW + wid) * 8 + drow;
        const int gc = dpos ^ ((hh >> 1) & 7);
        const int c0 = cc * H5K + gc * 8;
        uint4* q = reinterpret_cast<uint4*>(hs + hh * H5K + dpos * 8);
        const uint4 v = *q;
        const float4 s0 = *reinterpret_cast<const float4*>(psc + c0);
        const float4 s1 = *reinterpret_cast<const float4*>(psc + c0 + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(psh + c0);
        const float4 h1 = *reinterpret_cast<const float4*>(psh + c0 + 4);
        const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
        const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float lo = fmaxf(bf2f((bf16_t)(w[k] & 0xffff)) * sc[2 * k] + sh[2 * k], 0.f);
          const float hi = fmaxf(bf2f((bf16_t)(w[k] >> 16)) * sc[2 * k + 1] + sh[2 * k + 1], 0.f);
          o[k] = pack_bf2(lo, hi);
        }
        *q = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  };
  // retire all but the `young` youngest DMA instructions of this thread
  auto wait_young = [&](int young) {
    if (young == 0) vm_wait<0>();
    else if (young == BI) vm_wait<BI>();
    else if (young == HRI) vm_wait<HRI>();
    else vm_wait<BI + HRI>();
  };
  auto barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };

  f32x16 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int hb, int b, int t) {
    const int4 tp = taps[t];
    const bf16_t* hs = Hs + hb * (HP + 1) * H5K;
    int hrow[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const bool ok = (unsigned)(a_x[i] + tp.y) < (unsigned)g.W &&
                      (unsigned)(a_y[i] + tp.x) < (unsigned)g.H;
      hrow[i] = ok ? a_h[i] + tp.w : HP;
    }
    const bf16_t* bs = Bs + b * BN * H5K;
    bf16x8 af[2][RM], bfr[2][RN];
    auto frag = [&](int ks, int set) {
      const int ch = ks * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < RM; ++i)
        af[set][i] = *reinterpret_cast<const bf16x8*>(hs + hrow[i] * H5K + swz(hrow[i], ch) * 8);
#pragma unroll
      for (int j = 0; j < RN; ++j) {
        const int r = wn * TN + j * 32 + (lane & 31);
        bfr[set][j] = *reinterpret_cast<const bf16x8*>(bs + r * H5K + swz(r, ch) * 8);
      }
    };
    frag(0, 0);
#pragma unroll
    for (int ks = 0; ks < H5K / 16; ++ks) {
      if (ks + 1 < H5K / 16) frag(ks + 1, (ks + 1) & 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[ks & 1][i], bfr[ks & 1][j],
                                                              acc[i][j], 0, 0, 0);
    }
  };

  const int S = nchunk * ntaps;
  // prologue: halo 0, weight tiles 0 and 1
  issue_halo(0, 0);
  issue_b(0, 0, 0);
  int lc = 0, lt = 1;  // (chunk, tap) of the next weight tile to issue
  if (lt == ntaps) {
    lt = 0;
    ++lc;
  }
  if (S > 1) {
    issue_b(lc, lt, 1);
    if (++lt == ntaps) {
      lt = 0;
      ++lc;
    }
    vm_wait<BI>();
  } else {
    vm_wait<0>();
  }
  normalise_halo(0, 0);
  barrier();

  int cc = 0, t = 0, bcur = 0;
  for (int s = 0; s < S; ++s) {
    const bool hiss = NHB == 2 && t == 0 && cc + 1 < nchunk;
    if (hiss) issue_halo(cc + 1, (cc + 1) & 1);
    const bool bis = s + 2 < S;
    if (bis) {
      const int b2 = bcur == 0 ? 2 : bcur - 1;  // (s + 2) % 3
      issue_b(lc, lt, b2);
      if (++lt == ntaps) {
        lt = 0;
        ++lc;
      }
    }
    compute(NHB == 2 ? (cc & 1) : 0, bcur, t);
    int nt = t + 1, ncc = cc;
    if (nt == ntaps) {
      nt = 0;
      ++ncc;
    }
    if (s + 1 < S) {
      // retire weight tile s+1 (and, at a chunk's last tap, halo cc+1): only tile s+2 and a
      // halo issued this step for a LATER chunk boundary may stay in flight
      wait_young((bis ? BI : 0) + ((hiss && nt != 0) ? HRI : 0));
      if (ncc != cc) normalise_halo(ncc, ncc & 1);
      barrier();
    }
    t = nt;
    cc = ncc;
    bcur = bcur == 2 ? 0 : bcur + 1;
  }
  vm_wait<0>();
  __syncthreads();  // the epilogue reuses the staging LDS
  constexpr int PASSES = (BMH * (BN + 4) * 4 > 80 * 1024) ? 2 : 1;
  mfma_tile_epilogue<BMH, BN, WM, WN, true, PASSES>(acc, smem, m0, n0, blockIdx.x, stats, g, Y, ADD,
                                                   bnb);
}

template <int BN, int WM, int WN, int BMH, int HRI, int NHB>
void launch_h5(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, const float* pre_sc, const float* pre_sh, hipStream_t st,
               const BnBwdEpi& bnb) {
  constexpr int NW = WM * WN;
  constexpr int HP = HRI * NW * 8;
  const size_t main = (size_t)NHB * (HP + 1) * H5K * 2 + (size_t)3 * BN * H5K * 2 + MAXTAPS * 16 +
                      (pre_sc ? (size_t)g.C * 8 : 0);
  constexpr int PASSES = (BMH * (BN + 4) * 4 > 80 * 1024) ? 2 : 1;
  const size_t epi = (size_t)(BMH / PASSES) * (BN + 4) * 4;
  const size_t sm = main > epi ? main : epi;
  dim3 grid((unsigned)((g.M + BMH - 1) / BMH), (g.Ncols + BN - 1) / BN);
  const unsigned xb = (unsigned)((long long)g.N * g.H * g.W * g.C * 2);
  const unsigned wb = (unsigned)((long long)g.Ncols * g.wK * 2);
  auto k = pre_sc ? conv_h5_kernel<BN, WM, WN, BMH, HRI, NHB, true>
                  : conv_h5_kernel<BN, WM, WN, BMH, HRI, NHB, false>;
  set_smem_attr(k, sm);
  k<<<grid, NW * 64, sm, st>>>(X, Wp, Y, ADD, stats, g, xb, wb, pre_sc, pre_sh, bnb);
}

int h5_halo_rows(const ConvGeom& g, int bm) {
  // worst case over blocks: a bm-pixel run starting at the last pixel of a row
  return ((g.W - 1 + bm - 1) / g.W + 3) * g.W;
}
}  // namespace

int conv_h5_rowtile(int cfg) { return cfg == 51 ? 512 : 256; }

// 50: 256 px x BN 128 (4 x 2 waves), two halo buffers; 51: 512 px x BN 64 (8 x 1 waves),
// one halo buffer (single 64-channel chunk only)
bool conv_h5_supported(const ConvGeom& g, int cfg) {
  if (g.isy != 1 || g.isx != 1 || g.Hg != g.H || g.Wg != g.W) return false;
  if (g.C % H5K != 0 || g.nth * g.ntw > 16 || g.nth < 1 || g.ntw < 1) return false;
  const int dya = g.dy0, dyb = g.dy0 + (g.nth - 1) * g.dys;
  const int dxa = g.dx0, dxb = g.dx0 + (g.ntw - 1) * g.dxs;
  auto in1 = [](int v) { return v >= -1 && v <= 1; };
  if (!in1(dya) || !in1(dyb) || !in1(dxa) || !in1(dxb)) return false;
  if ((long long)g.N * g.H * g.W * g.C * 2 >= (1LL << 31)) return false;
  if ((long long)g.Ncols * g.wK * 2 >= (1LL << 31)) return false;
  if (g.C > 512) return false;  // PRE scale/shift staging
  if (cfg == 50) return g.Ncols % 128 == 0 && h5_halo_rows(g, 256) <= 6 * 64;
  if (cfg == 51) return g.Ncols % 64 == 0 && g.C == 64 && h5_halo_rows(g, 512) <= 12 * 64;
  return false;
}

void conv_h5(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
             const ConvGeom& g, int cfg, hipStream_t st, const float* pre_sc, const float* pre_sh,
             const BnBwdEpi* bnbp) {
  const BnBwdEpi bnb = bnbp ? *bnbp : BnBwdEpi{};
  if (cfg == 50) {
    const int hr = (h5_halo_rows(g, 256) + 63) / 64;
    if (hr <= 5) launch_h5<128, 4, 2, 256, 5, 2>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st, bnb);
    else launch_h5<128, 4, 2, 256, 6, 2>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st, bnb);
  } else {
    const int hr = (h5_halo_rows(g, 512) + 63) / 64;
    if (hr <= 8) launch_h5<64, 8, 1, 512, 8, 1>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st, bnb);
    else launch_h5<64, 8, 1, 512, 12, 1>(X, Wp, Y, ADD, stats, g, pre_sc, pre_sh, st, bnb);
  }
  DM_CHECK(hipGetLastError());
}

}  // namespace dm
