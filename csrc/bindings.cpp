// Python bindings for the dmlab HIP kernels (module dmlab._C).
// Each binding validates shapes/dtypes on the host, then launches on the
// current PyTorch HIP stream so kernels compose with RCCL/torch streams and
// hipGraph capture.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "kernels.h"

namespace {

inline hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}
using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;

#define CHECK_CUDA(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP device tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_ALIGN16(t) \
  TORCH_CHECK((reinterpret_cast<uintptr_t>((t).data_ptr()) & 15) == 0, #t " must be 16-B aligned")

inline dm::bf16_t* bfp(const at::Tensor& t) {
  return reinterpret_cast<dm::bf16_t*>(t.data_ptr());
}
inline dm::bf16_t* opt_bfp(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_CUDA(*t);
  CHECK_BF16(*t);
  CHECK_ALIGN16(*t);
  return bfp(*t);
}

void sgd_step(at::Tensor p, at::Tensor g, c10::optional<at::Tensor> mom,
              c10::optional<at::Tensor> pbf, double lr, double momentum, double dampening,
              double wd, double gscale, bool nesterov, bool first) {
  CHECK_CUDA(p); CHECK_CUDA(g); CHECK_F32(p); CHECK_F32(g);
  CHECK_CONTIG(p); CHECK_CONTIG(g);
  TORCH_CHECK(p.numel() == g.numel(), "param/grad size mismatch");
  float* mp = nullptr;
  if (momentum != 0.0) {
    TORCH_CHECK(mom.has_value() && mom->defined(), "momentum buffer required");
    CHECK_CUDA(*mom); CHECK_F32(*mom);
    TORCH_CHECK(mom->numel() == p.numel(), "momentum size mismatch");
    mp = mom->data_ptr<float>();
  }
  dm::bf16_t* pb = opt_bfp(pbf);
  if (pb) TORCH_CHECK(pbf->numel() == p.numel(), "bf16 shadow size mismatch");
  const DeviceGuard guard(p.device());
  dm::sgd_step(p.data_ptr<float>(), g.data_ptr<float>(), mp, pb, p.numel(), (float)lr,
               (float)momentum, (float)dampening, (float)wd, (float)gscale, nesterov, first,
               cur_stream());
}

void adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v,
               c10::optional<at::Tensor> pbf, double lr, double b1, double b2, double eps,
               double wd, double gscale, double bc1, double bc2) {
  for (auto* t : {&p, &g, &m, &v}) {
    CHECK_CUDA(*t); CHECK_F32(*t); CHECK_CONTIG(*t); CHECK_ALIGN16(*t);
    TORCH_CHECK(t->numel() == p.numel(), "adam buffer size mismatch");
  }
  dm::bf16_t* pb = opt_bfp(pbf);
  const DeviceGuard guard(p.device());
  dm::adam_step(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                v.data_ptr<float>(), pb, p.numel(), (float)lr, (float)b1, (float)b2,
                (float)eps, (float)wd, (float)gscale, (float)bc1, (float)bc2, cur_stream());
}

void cast_f32_bf16(at::Tensor x, at::Tensor y) {
  CHECK_CUDA(x); CHECK_CUDA(y); CHECK_F32(x); CHECK_BF16(y);
  CHECK_CONTIG(x); CHECK_CONTIG(y); CHECK_ALIGN16(x); CHECK_ALIGN16(y);
  TORCH_CHECK(x.numel() == y.numel(), "size mismatch");
  const DeviceGuard guard(x.device());
  dm::cast_f32_bf16(x.data_ptr<float>(), bfp(y), x.numel(), cur_stream());
}

void rows_mean(at::Tensor x, at::Tensor out, double scale) {
  CHECK_CUDA(x); CHECK_CUDA(out); CHECK_F32(x); CHECK_F32(out);
  CHECK_CONTIG(x); CHECK_CONTIG(out);
  TORCH_CHECK(x.dim() == 2 && x.size(1) == out.numel(), "x must be [rows, N]");
  const DeviceGuard guard(x.device());
  dm::rows_mean(x.data_ptr<float>(), out.data_ptr<float>(), (int)x.size(0), out.numel(),
                (float)scale, cur_stream());
}

void scale_inplace(at::Tensor x, double s) {
  CHECK_CUDA(x); CHECK_F32(x); CHECK_CONTIG(x);
  const DeviceGuard guard(x.device());
  dm::scale_inplace(x.data_ptr<float>(), x.numel(), (float)s, cur_stream());
}

// ------------------------------------------------------------------ small conv (LeNet)
inline bool is_bf16(const at::Tensor& t) { return t.scalar_type() == at::kBFloat16; }
inline void check_act(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a HIP tensor");
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
  TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, n,
              " must be fp32/bf16");
}
inline const void* optp(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}

void conv_small_fwd(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, at::Tensor y,
                    c10::optional<at::Tensor> mask, int64_t pad, int64_t pool, bool relu) {
  check_act(x, "x"); check_act(y, "y"); CHECK_F32(w); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(1) == x.size(1) && w.size(2) == w.size(3));
  TORCH_CHECK(is_bf16(x) == is_bf16(y), "x/y dtype mismatch");
  const int B = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int Cout = w.size(0), K = w.size(2);
  TORCH_CHECK(K == 3 || K == 5, "conv_small supports K in {3,5}");
  TORCH_CHECK(pool == 1 || pool == 2, "pool must be 1 or 2");
  const int OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  TORCH_CHECK(y.size(0) == B && y.size(1) == Cout && y.size(2) == OH / pool && y.size(3) == OW / pool,
              "y shape mismatch");
  if (pool > 1) TORCH_CHECK(mask.has_value() && mask->numel() == y.numel(), "mask required");
  const DeviceGuard guard(x.device());
  dm::conv_small_fwd(x.data_ptr(), w.data_ptr<float>(),
                     bias.has_value() ? bias->data_ptr<float>() : nullptr, y.data_ptr(),
                     pool > 1 ? (uint8_t*)mask->data_ptr() : nullptr, B, Cin, H, W, Cout, K,
                     (int)pad, (int)pool, relu ? 1 : 0, is_bf16(x), cur_stream());
}

void conv_small_bwd(at::Tensor x, at::Tensor w, at::Tensor dp, at::Tensor yp,
                    c10::optional<at::Tensor> mask, c10::optional<at::Tensor> dx, at::Tensor dw,
                    c10::optional<at::Tensor> db, at::Tensor work, int64_t pad, int64_t pool,
                    bool relu, double beta, int64_t bs) {
  check_act(x, "x"); check_act(dp, "dp"); check_act(yp, "yp");
  CHECK_F32(w); CHECK_F32(dw); CHECK_F32(work);
  const int B = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int Cout = w.size(0), K = w.size(2);
  const int OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  const long long total = (long long)B * Cout * OH * OW;
  const int S = (B + bs - 1) / bs;
  const long long need = (total + 63) / 64 * 64 + (long long)S * (Cout * Cin * K * K + Cout);
  TORCH_CHECK(work.numel() >= need, "workspace too small");
  TORCH_CHECK(dw.numel() == w.numel(), "dw size");
  if (dx.has_value()) { check_act(*dx, "dx"); TORCH_CHECK(dx->numel() == x.numel()); }
  if (pool > 1) TORCH_CHECK(mask.has_value() && mask->numel() == dp.numel(), "mask required");
  const DeviceGuard guard(x.device());
  dm::conv_small_bwd(x.data_ptr(), w.data_ptr<float>(), dp.data_ptr(), yp.data_ptr(),
                     pool > 1 ? (const uint8_t*)mask->data_ptr() : nullptr,
                     dx.has_value() ? dx->data_ptr() : nullptr, dw.data_ptr<float>(),
                     db.has_value() ? db->data_ptr<float>() : nullptr, work.data_ptr<float>(), B,
                     Cin, H, W, Cout, K, (int)pad, (int)pool, relu ? 1 : 0, (float)beta, (int)bs,
                     is_bf16(x), cur_stream());
}

int64_t conv_small_workspace(int64_t B, int64_t Cin, int64_t H, int64_t W, int64_t Cout,
                             int64_t K, int64_t pad, int64_t bs) {
  const long long OH = H + 2 * pad - K + 1, OW = W + 2 * pad - K + 1;
  const long long total = B * Cout * OH * OW;
  const long long S = (B + bs - 1) / bs;
  return (total + 63) / 64 * 64 + S * (Cout * Cin * K * K + Cout);
}

// ------------------------------------------------------------------ strided GEMM
// C[m,n] = alpha * sum_k A(m,k) B(k,n) + beta*C + bias ; strides in elements.
void gemm(at::Tensor A, c10::optional<at::Tensor> Amask, at::Tensor B, c10::optional<at::Tensor> C,
          c10::optional<at::Tensor> C32, c10::optional<at::Tensor> bias, int64_t M, int64_t N,
          int64_t K, int64_t sam, int64_t sak, int64_t sbk, int64_t sbn, int64_t scm,
          double alpha, double beta, bool relu, bool lowp) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda());
  auto span_ok = [](const at::Tensor& t, int64_t r, int64_t c, int64_t sr, int64_t sc) {
    return (r - 1) * sr + (c - 1) * sc < t.numel();
  };
  TORCH_CHECK(span_ok(A, M, K, sam, sak), "A too small for M,K,strides");
  TORCH_CHECK(span_ok(B, K, N, sbk, sbn), "B too small for K,N,strides");
  if (Amask.has_value()) TORCH_CHECK(Amask->scalar_type() == A.scalar_type() && Amask->numel() >= A.numel());
  void* cp = nullptr;
  int cbf = 0;
  if (C.has_value()) { cp = C->data_ptr(); cbf = is_bf16(*C); TORCH_CHECK(span_ok(*C, M, N, scm, 1)); }
  float* c32 = nullptr;
  if (C32.has_value()) { CHECK_F32(*C32); c32 = C32->data_ptr<float>(); TORCH_CHECK(span_ok(*C32, M, N, scm, 1)); }
  TORCH_CHECK(cp || c32, "an output is required");
  if (bias.has_value()) { CHECK_F32(*bias); TORCH_CHECK(bias->numel() >= N); }
  const DeviceGuard guard(A.device());
  // bf16 path: split K over blocks when the output tile grid alone cannot fill the chip
  // (the ResNet head: 64 output tiles), partial sums in an fp32 workspace reduced in order
  int S = 1;
  at::Tensor part;
  if (lowp && is_bf16(A)) {
    const long long tiles = ((M + 63) / 64) * ((N + 63) / 64);
    while (S < 16 && tiles * S < 256 && K / (S * 2) >= 64) S *= 2;
    if (S > 1) part = at::empty({(long long)S * M * N}, A.options().dtype(at::kFloat));
  } else if (K >= 4 * 64) {
    // fp32 kernel: its 64-deep LDS stages run serially per block, so a K of >= 4 stages on
    // few output tiles is split over blocks (one or two stages each) + an ordered reduce
    const long long tiles = ((M + 63) / 64) * ((N + 63) / 64);
    while (S < 16 && tiles * S < 256 && K / (S * 2) >= 32) S *= 2;
    if (S > 1) part = at::empty({(long long)S * M * N}, A.options().dtype(at::kFloat));
  }
  dm::gemm_strided(A.data_ptr(), optp(Amask), is_bf16(A), B.data_ptr(), is_bf16(B), cp, cbf, c32,
                   bias.has_value() ? bias->data_ptr<float>() : nullptr, M, N, K, sam, sak, sbk,
                   sbn, scm, (float)alpha, (float)beta, relu ? 1 : 0, lowp ? 1 : 0,
                   S > 1 ? part.data_ptr<float>() : nullptr, S, cur_stream());
}

// ------------------------------------------------------------ CU-masked streams
// A stream whose kernels may only use the CUs set in `mask` (32 CUs per word).  Its own
// hardware queue carries the mask, so two processes on one GPU can each own a disjoint CU
// partition: the lab-4 pipeline uses it to give every stage a "device" of its own.
int64_t cu_mask_stream(std::vector<int64_t> mask) {
  TORCH_CHECK(!mask.empty(), "empty CU mask");
  std::vector<uint32_t> m(mask.begin(), mask.end());
  hipStream_t st = nullptr;
  TORCH_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()) == hipSuccess,
              "hipExtStreamCreateWithCUMask failed");
  return (int64_t)(uintptr_t)st;
}
std::vector<int64_t> cu_mask_of(int64_t stream, int64_t words) {
  std::vector<uint32_t> m((size_t)words, 0u);
  TORCH_CHECK(hipExtStreamGetCUMask((hipStream_t)(uintptr_t)stream, (uint32_t)words, m.data()) ==
              hipSuccess, "hipExtStreamGetCUMask failed");
  return std::vector<int64_t>(m.begin(), m.end());
}
void stream_destroy(int64_t stream) {
  TORCH_CHECK(hipStreamDestroy((hipStream_t)(uintptr_t)stream) == hipSuccess);
}

// ------------------------------------------------------------ xGMI one-/two-shot all-reduce
int64_t xgmi_alloc(int64_t bytes) { return (int64_t)(uintptr_t)dm::xgmi_alloc((size_t)bytes); }
void xgmi_free(int64_t ptr) { dm::xgmi_free((void*)(uintptr_t)ptr); }
py::bytes xgmi_get_handle(int64_t ptr) {
  char h[64];
  dm::xgmi_get_handle((void*)(uintptr_t)ptr, h);
  return py::bytes(h, 64);
}
int64_t xgmi_open_handle(py::bytes handle) {
  std::string h = handle;
  TORCH_CHECK(h.size() == 64, "IPC handle must be 64 bytes");
  return (int64_t)(uintptr_t)dm::xgmi_open_handle(h.data());
}
void xgmi_close_handle(int64_t ptr) { dm::xgmi_close_handle((void*)(uintptr_t)ptr); }
void xgmi_allreduce(at::Tensor in, at::Tensor out, int64_t cap, std::vector<int64_t> data,
                    std::vector<int64_t> flags, int64_t rank, double scale, at::Tensor state,
                    int64_t algo, int64_t share) {
  CHECK_F32(in);
  CHECK_F32(out);
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel());
  TORCH_CHECK(in.numel() <= cap, "tensor larger than the shared buffer");
  const int W = data.size();
  TORCH_CHECK(W >= 1 && W <= 8 && (int)flags.size() == W && rank >= 0 && rank < W);
  // [timeout flag, last published epoch, done-block counter, pad] on the device
  TORCH_CHECK(state.scalar_type() == at::kInt && state.is_cuda() && state.numel() >= 3 &&
              state.device() == in.device());
  std::vector<void*> d(W), f(W);
  for (int q = 0; q < W; ++q) {
    d[q] = (void*)(uintptr_t)data[q];
    f[q] = (void*)(uintptr_t)flags[q];
  }
  const DeviceGuard guard(in.device());
  dm::xgmi_allreduce(in.data_ptr<float>(), out.data_ptr<float>(), in.numel(), cap, d.data(),
                     f.data(), (int)rank, W, (float)scale,
                     reinterpret_cast<unsigned*>(state.data_ptr<int>()), (int)algo, cur_stream(),
                     (int)share);
}

// P2P channel (csrc/p2p_xgmi.hip): src/dst tensors contiguous, 16-B aligned, bytes % 16 == 0;
// ring/full/free are raw device addresses (own or IPC-opened), state an int32[4] device tensor
void p2p_xgmi_send(at::Tensor src, int64_t ring, int64_t full, int64_t free_, int64_t slot_bytes,
                   int64_t nslot, at::Tensor state) {
  CHECK_CUDA(src); CHECK_CONTIG(src); CHECK_ALIGN16(src); CHECK_CUDA(state);
  const int64_t bytes = src.numel() * src.element_size();
  TORCH_CHECK(bytes % 16 == 0 && bytes <= slot_bytes && slot_bytes % 16 == 0 && nslot >= 1,
              "p2p send: payload must be a multiple of 16 B and fit a ring slot");
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() >= 4, "state: int32[4]");
  const DeviceGuard guard(src.device());
  dm::p2p_xgmi_send(src.data_ptr(), bytes, (void*)(uintptr_t)ring, (void*)(uintptr_t)full,
                    (const void*)(uintptr_t)free_, slot_bytes, (int)nslot,
                    reinterpret_cast<unsigned*>(state.data_ptr<int>()), cur_stream());
}

void p2p_xgmi_recv(at::Tensor dst, int64_t ring, int64_t full, int64_t free_, int64_t slot_bytes,
                   int64_t nslot, at::Tensor state) {
  CHECK_CUDA(dst); CHECK_CONTIG(dst); CHECK_ALIGN16(dst); CHECK_CUDA(state);
  const int64_t bytes = dst.numel() * dst.element_size();
  TORCH_CHECK(bytes % 16 == 0 && bytes <= slot_bytes && slot_bytes % 16 == 0 && nslot >= 1,
              "p2p recv: payload must be a multiple of 16 B and fit a ring slot");
  TORCH_CHECK(state.scalar_type() == at::kInt && state.numel() >= 4, "state: int32[4]");
  const DeviceGuard guard(dst.device());
  dm::p2p_xgmi_recv(dst.data_ptr(), bytes, (const void*)(uintptr_t)ring,
                    (const void*)(uintptr_t)full, (void*)(uintptr_t)free_, slot_bytes, (int)nslot,
                    reinterpret_cast<unsigned*>(state.data_ptr<int>()), cur_stream());
}

void colsum(at::Tensor A, c10::optional<at::Tensor> Amask, at::Tensor out, double beta) {
  TORCH_CHECK(A.is_cuda() && A.dim() == 2 && A.is_contiguous());
  CHECK_F32(out);
  TORCH_CHECK(out.numel() == A.size(1));
  const DeviceGuard guard(A.device());
  dm::colsum(A.data_ptr(), optp(Amask), is_bf16(A), out.data_ptr<float>(), A.size(0), A.size(1),
             (float)beta, cur_stream());
}

void bias_act(at::Tensor y, c10::optional<at::Tensor> bias, at::Tensor out, bool relu) {
  CHECK_F32(y);
  TORCH_CHECK(y.is_cuda() && y.dim() == 2 && y.is_contiguous());
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.sizes() == y.sizes() &&
              (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16));
  if (bias.has_value()) { CHECK_F32(*bias); TORCH_CHECK(bias->numel() == y.size(1)); }
  const DeviceGuard guard(y.device());
  dm::bias_act(y.data_ptr<float>(), bias.has_value() ? bias->data_ptr<float>() : nullptr,
               out.data_ptr(), is_bf16(out), y.size(0), y.size(1), relu ? 1 : 0, cur_stream());
}

// ------------------------------------------------------------------ loss / eval / spin
void cross_entropy(at::Tensor logits, at::Tensor labels, at::Tensor rowloss, at::Tensor loss,
                   c10::optional<at::Tensor> dlogits, double scale) {
  check_act(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && labels.scalar_type() == at::kLong && labels.numel() == logits.size(0));
  CHECK_F32(rowloss); CHECK_F32(loss);
  TORCH_CHECK(rowloss.numel() >= logits.size(0));
  if (dlogits.has_value()) { check_act(*dlogits, "dlogits"); TORCH_CHECK(dlogits->sizes() == logits.sizes() && is_bf16(*dlogits) == is_bf16(logits)); }
  const DeviceGuard guard(logits.device());
  dm::cross_entropy(logits.data_ptr(), (const long long*)labels.data_ptr(), rowloss.data_ptr<float>(),
                    loss.data_ptr<float>(), dlogits.has_value() ? dlogits->data_ptr() : nullptr,
                    logits.size(0), logits.size(1), (float)scale, -100, is_bf16(logits),
                    cur_stream());
}

void argmax_count(at::Tensor logits, at::Tensor labels, at::Tensor correct) {
  check_act(logits, "logits");
  TORCH_CHECK(correct.scalar_type() == at::kLong && labels.scalar_type() == at::kLong);
  const DeviceGuard guard(logits.device());
  dm::argmax_count(logits.data_ptr(), (const long long*)labels.data_ptr(), logits.size(0), logits.size(1),
                   (unsigned long long*)correct.data_ptr(), is_bf16(logits), cur_stream());
}

void spin_us(double us) { dm::spin_us(us, cur_stream()); }

// One LeNet training step (csrc/lenet_fused.hip).  w: conv1.w, conv1.b, conv2.w, conv2.b,
// fc1.w, fc1.b, fc2.w, fc2.b (fp32 masters); off: flat-buffer offsets of fc2.w, fc2.b, fc1.w,
// fc1.b, conv2.w, conv2.b, conv1.w, conv1.b; p/mom given: the SGD update runs in the same
// dispatch as the gradient reduction (p = the flat fp32 parameters, mom its momentum buffer).
void lenet_fused_step(at::Tensor x, at::Tensor labels, std::vector<at::Tensor> w, at::Tensor rec,
                      at::Tensor cslab, at::Tensor rowloss, at::Tensor grad,
                      std::vector<int64_t> off, c10::optional<at::Tensor> p,
                      c10::optional<at::Tensor> mom, double lr, double momentum, double dampening,
                      double wd, double gscale, bool nesterov, bool first, at::Tensor loss,
                      c10::optional<at::Tensor> sidx, c10::optional<at::Tensor> cursor,
                      int64_t batch, c10::optional<at::Tensor> loss_sum,
                      c10::optional<at::Tensor> probe) {
  CHECK_CUDA(x); CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4 && x.size(1) == 1 && x.size(2) == 28 && x.size(3) == 28,
              "x: [B, 1, 28, 28]");
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16, "x: fp32 or bf16");
  // sidx given: x / labels are the whole device-resident dataset; this step's samples are rows
  // sidx[cursor*batch : (cursor+1)*batch] (sampler order), the cursor advancing on the device
  const bool indexed = sidx.has_value() && sidx->defined();
  const int B = indexed ? (int)batch : (int)x.size(0);
  int nbatch = 0;
  if (indexed) {
    CHECK_CUDA(*sidx); CHECK_CONTIG(*sidx);
    TORCH_CHECK(sidx->scalar_type() == at::kLong && batch >= 1, "sidx: int64 row indices");
    TORCH_CHECK(cursor.has_value() && cursor->is_cuda() && cursor->scalar_type() == at::kInt &&
                    cursor->numel() == 1, "cursor: int32 [1] on the device");
    nbatch = (int)(sidx->numel() / batch);
    TORCH_CHECK(nbatch >= 1, "sidx holds fewer than one batch");
    TORCH_CHECK(labels.numel() == x.size(0), "labels: one per dataset row");
  }
  TORCH_CHECK(B >= 1 && labels.is_cuda() && labels.scalar_type() == at::kLong &&
                  labels.is_contiguous() && (indexed || labels.numel() == B), "labels: int64 [B]");
  TORCH_CHECK(w.size() == 8 && off.size() == 8, "8 parameter tensors / offsets");
  const int64_t want[8] = {150, 6, 2400, 16, 48000, 120, 1200, 10};
  const float* wp[8];
  for (int i = 0; i < 8; ++i) {
    CHECK_CUDA(w[i]); CHECK_F32(w[i]); CHECK_CONTIG(w[i]);
    TORCH_CHECK(w[i].numel() == want[i], "parameter ", i, " has the wrong size");
    wp[i] = w[i].data_ptr<float>();
  }
  for (auto* t : {&rec, &cslab, &rowloss, &grad, &loss}) { CHECK_CUDA(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  TORCH_CHECK(rec.numel() >= (int64_t)B * dm::lenet_record_floats() &&
                  cslab.numel() >= (int64_t)B * dm::lenet_slab_floats() && rowloss.numel() >= B &&
                  loss.numel() == 1, "workspace too small");
  const int64_t segn[8] = {1200, 10, 48000, 120, 2400, 16, 150, 6};
  int o[8];
  for (int i = 0; i < 8; ++i) {
    TORCH_CHECK(off[i] >= 0 && off[i] + segn[i] <= grad.numel(), "flat offset out of range");
    o[i] = (int)off[i];
  }
  float* pp = nullptr;
  float* mp = nullptr;
  if (p.has_value()) {
    CHECK_CUDA(*p); CHECK_F32(*p); CHECK_CONTIG(*p);
    TORCH_CHECK(p->numel() == grad.numel(), "p: the flat parameter buffer");
    pp = p->data_ptr<float>();
    if (momentum != 0.0) {
      TORCH_CHECK(mom.has_value() && mom->numel() == grad.numel() && mom->scalar_type() == at::kFloat,
                  "mom: the flat momentum buffer");
      mp = mom->data_ptr<float>();
    }
  }
  float* lsum = nullptr;
  if (loss_sum.has_value() && loss_sum->defined()) {
    CHECK_CUDA(*loss_sum); CHECK_F32(*loss_sum);
    TORCH_CHECK(loss_sum->numel() == 1, "loss_sum: fp32 [1] on the device");
    lsum = loss_sum->data_ptr<float>();
  }
  unsigned long long* pr = nullptr;
  if (probe.has_value() && probe->defined()) {  // phase timestamps (tools/lenet_phases.py)
    CHECK_CUDA(*probe); CHECK_CONTIG(*probe);
    TORCH_CHECK(probe->scalar_type() == at::kLong && probe->numel() >= (int64_t)B * dm::lenet_probe_stamps(),
                "probe: int64 [B * lenet_probe_stamps()]");
    pr = reinterpret_cast<unsigned long long*>(probe->data_ptr<int64_t>());
  }
  const DeviceGuard guard(x.device());
  dm::lenet_fused_step(x.data_ptr(), x.scalar_type() == at::kBFloat16,
                       reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()),
                       B, wp, rec.data_ptr<float>(), cslab.data_ptr<float>(),
                       rowloss.data_ptr<float>(), grad.data_ptr<float>(), o, pp, mp, (float)lr,
                       (float)momentum, (float)dampening, (float)wd, (float)gscale, nesterov,
                       first, pp != nullptr, loss.data_ptr<float>(),
                       indexed ? reinterpret_cast<const long long*>(sidx->data_ptr<int64_t>()) : nullptr,
                       indexed ? cursor->data_ptr<int>() : nullptr, x.size(0), nbatch, lsum,
                       cur_stream(), pr);
}

int num_cus(int device) {
  int n = 0;
  TORCH_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess);
  return n;
}

}  // namespace

void register_resnet(pybind11::module_& m);
void register_reducer(pybind11::module_& m);

// generated per build by dmlab/_build.py (build/native/source_hash.cpp): sha256 of the csrc/
// tree and build configuration this library was linked from
extern "C" const char* dmlab_source_hash();

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("source_hash", []() { return std::string(dmlab_source_hash()); },
        "sha256 of the csrc/ sources + build flags this extension was built from");
  register_resnet(m);
  register_reducer(m);
  m.doc() = "dmlab native HIP kernels for MI355X (gfx950)";
  m.def("num_cus", &num_cus);
  m.def("sgd_step", &sgd_step, "fused flat SGD/GD step");
  m.def("adam_step", &adam_step, "fused flat Adam step");
  m.def("cast_f32_bf16", &cast_f32_bf16, "fp32 -> bf16 cast");
  m.def("rows_mean", &rows_mean, "[rows,N] -> [N] scaled row sum");
  m.def("scale_inplace", &scale_inplace, "x *= s");
  m.def("conv_small_fwd", &conv_small_fwd);
  m.def("conv_small_bwd", &conv_small_bwd);
  m.def("conv_small_workspace", &conv_small_workspace);
  m.def("gemm", &gemm, py::arg("A"), py::arg("Amask"), py::arg("B"), py::arg("C"), py::arg("C32"),
        py::arg("bias"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("sam"), py::arg("sak"),
        py::arg("sbk"), py::arg("sbn"), py::arg("scm"), py::arg("alpha"), py::arg("beta"),
        py::arg("relu"), py::arg("lowp") = false);
  m.def("colsum", &colsum);
  m.def("bias_act", &bias_act, py::arg("y"), py::arg("bias"), py::arg("out"), py::arg("relu"));
  m.def("cu_mask_stream", &cu_mask_stream);
  m.def("cu_mask_of", &cu_mask_of);
  m.def("stream_destroy", &stream_destroy);
  m.def("xgmi_alloc", &xgmi_alloc);
  m.def("xgmi_free", &xgmi_free);
  m.def("xgmi_get_handle", &xgmi_get_handle);
  m.def("xgmi_open_handle", &xgmi_open_handle);
  m.def("xgmi_close_handle", &xgmi_close_handle);
  m.def("xgmi_allreduce", &xgmi_allreduce, py::arg("in"), py::arg("out"), py::arg("cap"),
        py::arg("data"), py::arg("flags"), py::arg("rank"), py::arg("scale"), py::arg("state"),
        py::arg("algo"), py::arg("share") = 1);
  m.def("p2p_xgmi_send", &p2p_xgmi_send);
  m.def("p2p_xgmi_recv", &p2p_xgmi_recv);
  m.def("cross_entropy", &cross_entropy);
  m.def("argmax_count", &argmax_count);
  m.def("spin_us", &spin_us);
  m.def("lenet_fused_step", &lenet_fused_step, "one fused LeNet training step (2 dispatches)",
        py::arg("x"), py::arg("labels"), py::arg("w"), py::arg("rec"), py::arg("cslab"),
        py::arg("rowloss"), py::arg("grad"), py::arg("off"), py::arg("p"), py::arg("mom"),
        py::arg("lr"), py::arg("momentum"), py::arg("dampening"), py::arg("wd"),
        py::arg("gscale"), py::arg("nesterov"), py::arg("first"), py::arg("loss"),
        py::arg("sidx") = py::none(), py::arg("cursor") = py::none(), py::arg("batch") = 0,
        py::arg("loss_sum") = py::none(), py::arg("probe") = py::none());
  m.def("lenet_record_floats", &dm::lenet_record_floats);
  m.def("lenet_slab_floats", &dm::lenet_slab_floats);
  m.def("lenet_probe_stamps", &dm::lenet_probe_stamps);
  m.attr("arch") = "gfx950";
}
