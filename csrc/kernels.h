// Host-side launcher declarations for every dmlab HIP kernel.
// All launchers are allocation-free and sync-free (hipGraph-capturable).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dm {
typedef unsigned short bf16_t;

// optim.hip
void sgd_step(float* p, const float* g, float* mom, bf16_t* pbf, long long n, float lr,
              float momentum, float dampening, float wd, float gscale, bool nesterov,
              bool first, hipStream_t st);
void adam_step(float* p, const float* g, float* m, float* v, bf16_t* pbf, long long n,
               float lr, float b1, float b2, float eps, float wd, float gscale, float bc1,
               float bc2, hipStream_t st);
void cast_f32_bf16(const float* x, bf16_t* y, long long n, hipStream_t st);
void rows_mean(const float* x, float* out, int rows, long long n, float scale,
               hipStream_t st);
void scale_inplace(float* x, long long n, float s, hipStream_t st);

}  // namespace dm

namespace dm {
// conv_small.hip  (NCHW, tiny channel counts; x/y/dx fp32 or bf16, weights fp32)
void conv_small_fwd(const void* x, const float* w, const float* bias, void* y, uint8_t* mask,
                    int B, int Cin, int H, int W, int Cout, int K, int pad, int pool, int relu,
                    bool bf16, hipStream_t st);
void conv_small_bwd(const void* x, const float* w, const void* dp, const void* yp,
                    const uint8_t* mask, void* dx, float* dw, float* db, float* work, int B,
                    int Cin, int H, int W, int Cout, int K, int pad, int pool, int relu,
                    float beta, int bs, bool bf16, hipStream_t st);
// gemm.hip
void gemm_strided(const void* A, const void* Amask, int a_bf16, const void* B, int b_bf16,
                  void* C, int c_bf16, float* C32, const float* bias, int M, int N, int K,
                  long long sam, long long sak, long long sbk, long long sbn, long long scm,
                  float alpha, float beta, int relu, int lowp, float* part, int S,
                  hipStream_t st);
void bias_act(const float* y, const float* bias, void* out, int out_bf16, int M, int N, int relu,
              hipStream_t st);
void colsum(const void* A, const void* Amask, int bf16, float* out, int M, int N, float beta,
            hipStream_t st);
// loss.hip
void cross_entropy(const void* logits, const long long* labels, float* rowloss, float* loss,
                   void* dlogits, int B, int C, float scale, int ignore_index, bool bf16,
                   hipStream_t st);
void argmax_count(const void* logits, const long long* labels, int B, int C,
                  unsigned long long* correct, bool bf16, hipStream_t st);
void spin_us(double us, hipStream_t st);
// lenet_fused.hip: the whole LeNet training step in 2 dispatches
int lenet_record_floats();
int lenet_slab_floats();
void lenet_fused_step(const void* x, bool x_bf16, const long long* labels, int B,
                      const float* const* w, float* rec, float* cslab, float* rowloss, float* grad,
                      const int* off, float* p, float* mom, float lr, float momentum,
                      float dampening, float wd, float gscale, bool nesterov, bool first,
                      bool do_sgd, float* loss, const long long* sidx, int* cursor,
                      long long nrows, int nbatch, float* loss_sum, hipStream_t st,
                      unsigned long long* probe = nullptr);
int lenet_probe_stamps();
}  // namespace dm

namespace dm {
// comm_xgmi.hip
void* xgmi_alloc(size_t bytes);
void xgmi_free(void* ptr);
void xgmi_get_handle(void* ptr, void* handle64);
void* xgmi_open_handle(const void* handle64);
void xgmi_close_handle(void* ptr);
void xgmi_allreduce(const float* in, float* out, long long n, long long cap, void* const* data,
                    void* const* flags, int rank, int W, float scale, unsigned* state, int algo,
                    hipStream_t st, int share = 1);
// p2p_xgmi.hip: one-direction stage-to-stage channel over IPC peer memory
void p2p_xgmi_send(const void* src, long long bytes, void* ring, void* full, const void* free_,
                   long long slot_bytes, int nslot, unsigned* state, hipStream_t st);
void p2p_xgmi_recv(void* dst, long long bytes, const void* ring, const void* full, void* free_,
                   long long slot_bytes, int nslot, unsigned* state, hipStream_t st);
// conv_igemm.hip
struct ConvGeom;
struct ConvGeomSet;
struct DgradSeg2;
struct BnBwdRed;
// seg2 (optional): a second K segment of geometry seg2->z (a 1x1/s2 projection's data
// gradient merged into the stride-2 dgrad's parity class (0,0)); red (optional): the consumer
// BatchNorm's backward sums in the epilogue (one part row per block: igemm_multi_rows)
bool igemm_fwd_multi(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                     const ConvGeomSet& gs, int ng, int cfg, hipStream_t st,
                     const DgradSeg2* seg2 = nullptr, const BnBwdRed* red = nullptr);
long long igemm_multi_rows(const ConvGeomSet& gs, int ng, int cfg);
void igemm_fwd(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int cfg, hipStream_t st);
// conv_stem.hip: s2d stem (16 channels, 16 taps, 64 outputs) with resident weights (cfg 60)
bool stem_conv_supported(const ConvGeom& g);
void stem_conv(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, float* stats, const ConvGeom& g,
               hipStream_t st);
// fused stem BN backward (quad max-pool gather) + s2d weight gradient -> slabs [S][64][256]
bool stem_wgrad_fused_supported(int N, int H, int W, int C, int Cpad);
int stem_wgrad_fused_blocks(int N, int H);
void stem_wgrad_fused(const bf16_t* xs, const bf16_t* y, const bf16_t* pdy, const uint8_t* pidx,
                      const float* coef, const float* sc, const float* sh, float* slab, int N,
                      int H, int W, int S, hipStream_t st);
// stem_fused.hip: K-dense fused stem (raw-input gather + 7x7/s2 conv + BN statistics + pooled
// extremum), pooled BN apply, backward (y recomputed, dy = a dz + b y + cc) wgrad, reduce
bool stem_fused_supported(int Hin, int Win);
int stem_fused_grid(int N);
int stem_slab_cols();
int stem_wk_cols();
void stem_fwd_fused(const void* img, int dtype, const long long* idx, const float* nsc,
                    const float* nbi, const bf16_t* wk, const float* gamma, bf16_t* pext,
                    uint8_t* code, float* stats, int N, int nimg, int Hin, int Win, int grid,
                    hipStream_t st);
void stem_pool_apply(const bf16_t* pext, const uint8_t* code, const float* scale,
                     const float* shift, bf16_t* out, uint8_t* code4, long long n, hipStream_t st);
void stem_bwd_fused2(const void* img, int dtype, const long long* idx, const float* nsc,
                     const float* nbi, const bf16_t* wk, const bf16_t* pdy, const uint8_t* code4,
                     float* dslab, float* gslab, int N, int nimg, int Hin, int Win, int grid,
                     hipStream_t st);
void stem_wcombine(const float* dslab, const float* gslab, int GD, const bf16_t* wk,
                   const float* coef, float* sums, float* dw, float beta, hipStream_t st);
int stem_gram_cols();
int stem_sums_len();
void stem_pack_weights(const float* w, bf16_t* wk, hipStream_t st);
// The BatchNorm backward reduction of the layer whose output gradient a data gradient
// produces, done in that dgrad's epilogue: with dz = Y * relu-mask (mask from y*sc + sh > 0,
// or the 1-bit `mask` when set), part[wg][0][c] = Σ dz and part[wg][1][c] = Σ dz (y - mu) is
// (one row per workgroup, the layout bn_backward's pre_part consumes)
struct BnBwdRed {
  const bf16_t* y;
  const uint8_t* mask;
  const float* sc;
  const float* sh;
  const float* mu;
  const float* is;
  float* part;
};
// The BatchNorm backward apply folded into a consumer's operand staging (the data and weight
// gradients of the conv that produced that BN's input): the staged operand is the BN's OUTPUT
// gradient dz, and the kernel stages dy = a*dz' + b*y + c (dz' = dz where the ReLU passed:
// y*sc + sh > 0 when sc is set, bit j of the 1-bit mask when mask is set, everywhere when
// neither) instead of reading a materialised dy.  coef: [3][C] a, b, c (bn_backward, dy None).
// Every pointer is valid (sc / sh alias coef when unused) and `mode` says which mask applies
// (0: none, 2: y*sc + sh > 0, 4: the 1-bit mask), so the kernels load unconditionally: a load
// under a branch leaves a phi that makes the compiler drain every prefetch in flight.
struct BnBwdIn {
  const bf16_t* y;
  const uint8_t* mask;  // null unless mode 4 (read through a range-checked buffer resource)
  const float* coef;
  const float* sc;
  const float* sh;
  int C;
  int mode;
};
// conv_pipe.hip: pipelined LDS-DMA implicit-GEMM conv (cfg 90-93: 256-pixel tiles)
bool conv_pipe_supported(const ConvGeom& g, int cfg);
bool conv_pipe_multi(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD,
                     const ConvGeomSet& gs, int ng, int cfg, hipStream_t st,
                     const DgradSeg2* seg2 = nullptr, const BnBwdRed* red = nullptr);
long long pipe_multi_rows(const ConvGeomSet& gs, int ng);
void conv_pipe(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int cfg, hipStream_t st, const BnBwdRed* red = nullptr);
// conv_res64.hip: persistent register-resident-weight 3x3 conv, 64 -> 64 channels (cfg 80);
// statistics rows = res64_grid(M) (one per workgroup)
bool conv_res64_supported(const ConvGeom& g);
int res64_grid(long long M);
void conv_res64(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
                const ConvGeom& g, hipStream_t st, const float* pre_sc = nullptr,
                const float* pre_sh = nullptr, const BnBwdRed* red = nullptr);
bool conv_halo_supported(const ConvGeom& g);
bool halo_cfg(int cfg, int& bn, int& waves);
void conv_halo(const bf16_t* X, const bf16_t* Wp, bf16_t* Y, const bf16_t* ADD, float* stats,
               const ConvGeom& g, int bn, int waves, hipStream_t st,
               const float* pre_sc = nullptr, const float* pre_sh = nullptr,
               const BnBwdRed* red = nullptr, const BnBwdIn* bwd = nullptr);
bool wgrad_halo_supported(const ConvGeom& g);
// stride-2 3x3 weight gradient over the four input parity planes (wgrad cfg 7)
bool wgrad_s2_supported(const ConvGeom& g);
void wgrad_s2(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
              long long mchunk, hipStream_t st);
// wgrad_res64.hip: row-streaming 64 -> 64 channel 3x3 weight gradient (wgrad cfg 8); S slabs
bool wgrad_res64_supported(const ConvGeom& g);
void wgrad_res64(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                 hipStream_t st, const float* pre_sc = nullptr, const float* pre_sh = nullptr);
void wgrad_halo(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                long long mchunk, int nty, hipStream_t st, const float* pre_sc = nullptr,
                const float* pre_sh = nullptr, const BnBwdIn* bwd = nullptr);
void pack_weights_multi(const long long* desc, const long long* prefix, int nl, long long total,
                        hipStream_t st);
void pack_weights_tiled(const long long* desc, const int* tprefix, int nl, int ntiles,
                        hipStream_t st);
int igemm_fwd_rowtile(int cfg);
void igemm_wgrad(const bf16_t* X, const bf16_t* DY, float* slab, const ConvGeom& g, int S,
                 long long mchunk, int cfg, hipStream_t st);
void wgrad_reduce(const float* slab, int S, int Cout, int C, int Cin, int KH, int KW, float* dw,
                  float beta, hipStream_t st);
void pack_weights(const float* w, bf16_t* wf, bf16_t* wd, int Cout, int Cin, int Cpad, int KH,
                  int KW, hipStream_t st);
// bn_pool.hip
void bn_stats_finalize(const float* stats, int T, int C, double count, const float* gamma,
                       const float* beta, float* rmean, float* rvar, float momentum, float eps,
                       float* scale, float* shift, float* mean, float* invstd, float* work, long long* num_batches,
                       hipStream_t st);
void bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                    float eps, int C, float* scale, float* shift, hipStream_t st);
void bn_apply(const bf16_t* y, const bf16_t* res, const float* scale, const float* shift,
              bf16_t* out, long long n, int C, bool relu, hipStream_t st, uint8_t* mask = nullptr);
int bn_bwd_groups(long long M, int C);
void bn_backward(const bf16_t* dout, const bf16_t* out, const bf16_t* y, const float* mean,
                 const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                 float gbeta, long long M, int C, int mode, const float* scale,
                 const float* shift, const bf16_t* pdy, const uint8_t* pidx, int H, int W,
                 int OH, int OW, int K, int S, int P, bf16_t* dy, bf16_t* dres, float* work,
                 hipStream_t st, const float* pre_part = nullptr, int pre_rows = 0,
                 const uint8_t* mask = nullptr);
void bn_relu_maxpool(const bf16_t* y, const float* scale, const float* shift, bf16_t* out,
                     uint8_t* idx, int N, int H, int W, int C, int OH, int OW, int K, int S,
                     int P, hipStream_t st, bf16_t* yarg = nullptr);
int bn_bwd_groups(long long M, int C);
int bn_bwd_reduce_masked(const bf16_t* dout, const bf16_t* y, const float* mean,
                         const float* invstd, const float* scale, const float* shift, long long M,
                         int C, float* part, hipStream_t st);
void maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH,
                 int OW, int K, int S, int P, hipStream_t st);
void maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C,
                 int OH, int OW, int K, int S, int P, hipStream_t st);
void avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st);
void avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st);
void pack_input(const void* x, bool bf16, bf16_t* y, int N, int C, int H, int W, int Cp,
                long long sn, long long sc, long long sh, long long sw, hipStream_t st);
void pack_input_s2d(const void* x, bool bf16, bf16_t* y, int N, int C, int H2, int W2, int Cp,
                    long long sn, long long sc, long long sh, long long sw, const long long* idx,
                    long long nsrc, hipStream_t st);
void pack_weights_s2d(const float* w, bf16_t* wf, int Cout, int C, int Cp, hipStream_t st);
void wgrad_reduce_s2d(const float* slab, int S, int Cout, int C, int Cp, float* dw, float beta,
                      hipStream_t st);
}  // namespace dm
