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

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "dmlab native HIP kernels for MI355X (gfx950)";
  m.def("sgd_step", &sgd_step, "fused flat SGD/GD step");
  m.def("adam_step", &adam_step, "fused flat Adam step");
  m.def("cast_f32_bf16", &cast_f32_bf16, "fp32 -> bf16 cast");
  m.def("rows_mean", &rows_mean, "[rows,N] -> [N] scaled row sum");
  m.def("scale_inplace", &scale_inplace, "x *= s");
  m.attr("arch") = "gfx950";
}
