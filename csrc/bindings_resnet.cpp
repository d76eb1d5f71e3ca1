// Bindings for the NHWC bf16 ResNet kernels: implicit-GEMM conv (fwd / dgrad /
// wgrad), BatchNorm, pooling, input/weight packing.  Geometry (ConvGeom) is built
// here on the host from plain conv parameters, so Python never sees kernel structs.
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "conv_geom.h"
#include "kernels.h"

namespace {

inline hipStream_t cur_stream() {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}
using DeviceGuard = c10::hip::HIPGuardMasqueradingAsCUDA;
using bf = dm::bf16_t;

inline bf* bp(const at::Tensor& t) { return reinterpret_cast<bf*>(t.data_ptr()); }
inline float* fp(const at::Tensor& t) { return t.data_ptr<float>(); }

void need_bf16_nhwc(const at::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.dim() == 4,
              n, " must be a contiguous 4-D bf16 HIP tensor [N,H,W,C]");
  TORCH_CHECK(t.size(3) % 8 == 0, n, ": channels must be a multiple of 8");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, n, " must be 16-B aligned");
}
void need_f32(const at::Tensor& t, const char* n, int64_t numel = -1) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), n,
              " must be a contiguous fp32 HIP tensor");
  if (numel >= 0) TORCH_CHECK(t.numel() >= numel, n, " too small");
}
int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  TORCH_CHECK((1 << l) == v, "C/8 must be a power of two");
  return l;
}

dm::ConvGeom fwd_geom(const at::Tensor& x, int Cout, int KH, int KW, int stride, int pad, int OH,
                      int OW) {
  dm::ConvGeom g{};
  g.N = x.size(0); g.H = x.size(1); g.W = x.size(2); g.C = x.size(3);
  g.lgC8 = ilog2(g.C / 8);
  g.Hg = OH; g.Wg = OW; g.isy = stride; g.isx = stride;
  g.OH = OH; g.OW = OW; g.OC = Cout; g.osy = 1; g.osx = 1; g.oy0 = 0; g.ox0 = 0;
  g.nth = KH; g.ntw = KW; g.dy0 = -pad; g.dys = 1; g.dx0 = -pad; g.dxs = 1;
  g.kh0 = 0; g.khs = 1; g.kw0 = 0; g.kws = 1; g.KW = KW;
  g.Ncols = Cout; g.wK = KH * KW * g.C;
  g.M = (long long)g.N * OH * OW;
  g.K = KH * KW * g.C;
  TORCH_CHECK(KH * KW <= dm::MAXTAPS, "too many taps");
  dm::geom_finalize(g);
  return g;
}

int64_t conv_stats_rows(int64_t M, int64_t cfg, int64_t ncols);

// The folded BatchNorm-backward operand (kernels.h BnBwdIn) of a data / weight gradient whose
// dY argument is that BN's OUTPUT gradient dz: y (its input, dz's shape), coef [3][C] (bn_backward
// with dy None), scale/shift (ReLU mask from y) or the 1-bit mask, neither: no ReLU
dm::BnBwdIn bwd_in(const at::Tensor& dz, const at::Tensor& y, const at::Tensor& coef,
                   const c10::optional<at::Tensor>& sc, const c10::optional<at::Tensor>& sh,
                   const c10::optional<at::Tensor>& mask) {
  need_bf16_nhwc(y, "bwd_y");
  TORCH_CHECK(y.sizes() == dz.sizes(), "bwd_y: the gradient's shape");
  const int C = dz.size(3);
  need_f32(coef, "bwd_coef", 3 * C);
  // unused scale/shift alias coef: the kernels load them unconditionally (kernels.h BnBwdIn)
  dm::BnBwdIn b{bp(y), nullptr, fp(coef), fp(coef), fp(coef), C, 0};
  TORCH_CHECK(!(mask.has_value() && sc.has_value()), "bwd: mask or scale/shift, not both");
  if (sc.has_value()) {
    TORCH_CHECK(sh.has_value(), "bwd_scale needs bwd_shift");
    need_f32(*sc, "bwd_scale", C);
    need_f32(*sh, "bwd_shift", C);
    b.sc = fp(*sc);
    b.sh = fp(*sh);
    b.mode = 2;
  }
  if (mask.has_value()) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() * 8 == dz.numel(), "bwd_mask: uint8 [numel/8]");
    b.mask = mask->data_ptr<uint8_t>();
    b.mode = 4;
  }
  return b;
}

// y = conv(x, w)  (+add) ; stats [T][2][Cout] optional
void conv_fwd(at::Tensor x, at::Tensor wpack, at::Tensor y, c10::optional<at::Tensor> stats,
              c10::optional<at::Tensor> add, int64_t KH, int64_t KW, int64_t stride, int64_t pad,
              int64_t cfg, c10::optional<at::Tensor> pre_scale,
              c10::optional<at::Tensor> pre_shift) {
  // pre_scale/pre_shift: x is the previous conv's raw output and the conv consumes
  // relu(x*pre_scale + pre_shift) (fused BN-apply + ReLU; halo kernels only)
  need_bf16_nhwc(x, "x");
  need_bf16_nhwc(y, "y");
  const int Cout = y.size(3), OH = y.size(1), OW = y.size(2);
  // pad is the top/left padding; the output size (taken from y) may imply a smaller
  // bottom/right padding (space-to-depth stem), never a larger one
  TORCH_CHECK(OH <= (x.size(1) + 2 * pad - KH) / stride + 1 && OW <= (x.size(2) + 2 * pad - KW) / stride + 1,
              "output spatial size mismatch");
  TORCH_CHECK(wpack.scalar_type() == at::kBFloat16 && wpack.numel() == (int64_t)Cout * KH * KW * x.size(3),
              "wpack must be bf16 [Cout][KH][KW][C]");
  auto g = fwd_geom(x, Cout, KH, KW, stride, pad, OH, OW);
  float* sp = nullptr;
  if (stats.has_value()) {
    need_f32(*stats, "stats", conv_stats_rows(g.M, cfg, Cout) * 2 * Cout);
    sp = fp(*stats);
  }
  const bf* ap = nullptr;
  if (add.has_value()) { need_bf16_nhwc(*add, "add"); TORCH_CHECK(add->sizes() == y.sizes()); ap = bp(*add); }
  const DeviceGuard guard(x.device());
  if (pre_scale.has_value()) {
    int bn, waves;
    TORCH_CHECK(pre_shift.has_value(), "pre_scale needs pre_shift");
    need_f32(*pre_scale, "pre_scale", x.size(3));
    need_f32(*pre_shift, "pre_shift", x.size(3));
    if (cfg == 80) {
      dm::conv_res64(bp(x), bp(wpack), bp(y), ap, sp, g, cur_stream(), fp(*pre_scale), fp(*pre_shift));
      return;
    }
    // the pipelined tiles take no fused pre-BN (measured slower than materialising it): the
    // halo tile with the same 256-row stats slab does
    if (cfg >= 90 && cfg <= 93) cfg = 41;
    TORCH_CHECK(dm::halo_cfg((int)cfg, bn, waves) && dm::conv_halo_supported(g),
                "fused pre-BN needs a halo-kernel cfg and a unit-stride 3x3 geometry");
    dm::conv_halo(bp(x), bp(wpack), bp(y), ap, sp, g, bn, waves, cur_stream(), fp(*pre_scale),
                  fp(*pre_shift));
    return;
  }
  dm::igemm_fwd(bp(x), bp(wpack), bp(y), ap, sp, g, cfg, cur_stream());
}

// statistics rows a forward conv of this cfg writes (one per row tile, or per workgroup of the
// persistent cfg 80); ncols is unused
// The BN-backward apply of a 3x3/s1/p1 conv's BatchNorm can fold into both consumers: the data
// gradient on the cfg 42 halo tile and the 9-tap halo weight gradient (conv_dgrad / conv_wgrad
// bwd_*).  x: the conv's input [N,H,W,Cin]; Cout its output channels.
bool bn_fold_supported(int64_t N, int64_t H, int64_t W, int64_t Cin, int64_t Cout) {
  if (Cin % 64 || Cout % 64 || ((Cout / 8) & (Cout / 8 - 1)) || ((Cin / 8) & (Cin / 8 - 1)))
    return false;
  dm::ConvGeom d{};  // data gradient (conv_dgrad stride 1)
  d.N = N; d.H = H; d.W = W; d.C = Cout; d.lgC8 = ilog2(Cout / 8);
  d.OH = H; d.OW = W; d.OC = Cin; d.KW = 3; d.Ncols = Cin; d.wK = 9 * Cout;
  d.Hg = H; d.Wg = W; d.isy = 1; d.isx = 1; d.osy = 1; d.osx = 1; d.oy0 = 0; d.ox0 = 0;
  d.nth = 3; d.ntw = 3; d.dy0 = 1; d.dys = -1; d.dx0 = 1; d.dxs = -1;
  d.kh0 = 0; d.khs = 1; d.kw0 = 0; d.kws = 1; d.M = N * H * W; d.K = 9 * Cout;
  dm::geom_finalize(d);
  dm::ConvGeom w{};  // weight gradient (fwd_geom of the conv)
  w.N = N; w.H = H; w.W = W; w.C = Cin; w.lgC8 = ilog2(Cin / 8);
  w.Hg = H; w.Wg = W; w.isy = 1; w.isx = 1; w.OH = H; w.OW = W; w.OC = Cout;
  w.osy = 1; w.osx = 1; w.oy0 = 0; w.ox0 = 0; w.nth = 3; w.ntw = 3; w.dy0 = -1; w.dys = 1;
  w.dx0 = -1; w.dxs = 1; w.kh0 = 0; w.khs = 1; w.kw0 = 0; w.kws = 1; w.KW = 3;
  w.Ncols = Cout; w.wK = 9 * Cin; w.M = N * H * W; w.K = 9 * Cin;
  dm::geom_finalize(w);
  return dm::conv_halo_supported(d) && dm::wgrad_halo_supported(w);
}

// part rows of a stride-2 data gradient with the reduction epilogue (conv_dgrad red_part)
int64_t dgrad_s2_red_rows(int64_t N, int64_t H, int64_t W, int64_t cfg) {
  dm::ConvGeomSet set{};
  int ng = 0;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      auto& g = set.g[ng++];
      g.M = N * ((H - a + 1) / 2) * ((W - b + 1) / 2);
    }
  if (cfg >= 90 && cfg <= 93) return dm::pipe_multi_rows(set, ng);
  return dm::igemm_multi_rows(set, ng, (int)cfg);
}

int64_t conv_stats_rows(int64_t M, int64_t cfg, int64_t ncols) {
  if (cfg == 80) return dm::res64_grid(M);
  const int bm = dm::igemm_fwd_rowtile(cfg);
  return (M + bm - 1) / bm;
}

// dx = conv_transpose(dy, w) for stride 1 or 2; add: tensor added to the result (may alias dx
// for in-place accumulation)
void conv_dgrad(at::Tensor dy, at::Tensor wd, at::Tensor dx, int64_t KH, int64_t KW,
                int64_t stride, int64_t pad, c10::optional<at::Tensor> add, int64_t cfg,
                c10::optional<at::Tensor> add_mask, c10::optional<at::Tensor> red_y,
                c10::optional<at::Tensor> red_scale, c10::optional<at::Tensor> red_shift,
                c10::optional<at::Tensor> red_mean, c10::optional<at::Tensor> red_invstd,
                c10::optional<at::Tensor> red_part, c10::optional<at::Tensor> red_mask,
                c10::optional<at::Tensor> dy2, c10::optional<at::Tensor> wd2,
                c10::optional<at::Tensor> bwd_y, c10::optional<at::Tensor> bwd_coef,
                c10::optional<at::Tensor> bwd_scale, c10::optional<at::Tensor> bwd_shift,
                c10::optional<at::Tensor> bwd_mask) {
  // bwd_* (optional, stride 1, cfg 42): dy is a BatchNorm's OUTPUT gradient; the kernel stages
  // that BN's backward a*dz' + b*y + c itself (bwd_in)
  // dy2 / wd2 (optional, stride 2): a 1x1/s2/p0 projection's output gradient and packed data-
  // gradient weights [Cin][1][1][C2]; its data gradient is merged into this launch (parity
  // class (0,0) gets a second K segment), so dx is written once, complete
  // red_* (optional, cfg 80 only): the backward reduction of the BatchNorm + ReLU whose
  // output gradient dx is (its input red_y, forward scale/shift, mean/invstd) runs in this
  // dgrad's epilogue -> red_part [res64_grid(M)][2][Cin] (bn_backward's pre_slab)
  // add_mask (optional, stride 1): 1-bit mask of `add` (bit j of byte i = element 8i + j), so
  // the identity-skip gradient dres = add * mask is added without being materialised
  need_bf16_nhwc(dy, "dy");
  need_bf16_nhwc(dx, "dx");
  const int N = dy.size(0), OH = dy.size(1), OW = dy.size(2), Cout = dy.size(3);
  const int H = dx.size(1), W = dx.size(2), Cin = dx.size(3);
  TORCH_CHECK(dx.size(0) == N);
  TORCH_CHECK(OH == (H + 2 * pad - KH) / stride + 1 && OW == (W + 2 * pad - KW) / stride + 1,
              "dgrad shape mismatch");
  TORCH_CHECK(wd.scalar_type() == at::kBFloat16 && wd.numel() == (int64_t)Cin * KH * KW * Cout,
              "wd must be bf16 [Cin][KH][KW][Cout]");
  TORCH_CHECK(stride == 1 || stride == 2, "stride must be 1 or 2");
  const bf* addp = nullptr;
  if (add.has_value()) { need_bf16_nhwc(*add, "add"); TORCH_CHECK(add->sizes() == dx.sizes()); addp = bp(*add); }
  const bool accumulate = addp != nullptr;
  TORCH_CHECK(stride == 1 || !accumulate || addp == bp(dx),
              "stride-2 dgrad accumulates only in place (add must alias dx)");
  const DeviceGuard guard(dy.device());
  auto st = cur_stream();
  dm::ConvGeom base{};
  base.N = N; base.H = OH; base.W = OW; base.C = Cout; base.lgC8 = ilog2(Cout / 8);
  base.OH = H; base.OW = W; base.OC = Cin;
  base.KW = KW; base.Ncols = Cin; base.wK = KH * KW * Cout;
  const unsigned char* addm = nullptr;
  if (add_mask.has_value()) {
    TORCH_CHECK(addp && stride == 1 && addp != bp(dx),
                "add_mask needs a separate add tensor and a stride-1 data gradient");
    TORCH_CHECK(add_mask->is_cuda() && add_mask->scalar_type() == at::kByte &&
                    add_mask->is_contiguous() && add_mask->numel() * 8 >= dx.numel(),
                "add_mask: uint8 [numel/8] on the device");
    addm = add_mask->data_ptr<uint8_t>();
  }
  dm::BnBwdIn bwd{};
  const bool has_bwd = bwd_y.has_value();
  if (has_bwd) {
    TORCH_CHECK(stride == 1 && cfg == 42 && bwd_coef.has_value(),
                "bwd_*: a stride-1 cfg 42 (halo) data gradient with bwd_coef");
    bwd = bwd_in(dy, *bwd_y, *bwd_coef, bwd_scale, bwd_shift, bwd_mask);
  }
  if (stride == 1) {
    auto g = base;
    g.addm = addm;
    g.Hg = H; g.Wg = W; g.isy = 1; g.isx = 1; g.osy = 1; g.osx = 1; g.oy0 = 0; g.ox0 = 0;
    g.nth = KH; g.ntw = KW; g.dy0 = pad; g.dys = -1; g.dx0 = pad; g.dxs = -1;
    g.kh0 = 0; g.khs = 1; g.kw0 = 0; g.kws = 1;
    g.M = (long long)N * H * W; g.K = KH * KW * Cout;
    dm::geom_finalize(g);
    if (has_bwd) {
      int hbn = 0, hwv = 0;
      TORCH_CHECK(dm::halo_cfg((int)cfg, hbn, hwv) && dm::conv_halo_supported(g),
                  "bwd_*: the geometry must suit the halo kernel");
    }
    if (red_y.has_value()) {
      const bool pipe = cfg >= 90 && cfg <= 93 && dm::conv_pipe_supported(g, (int)cfg);
      int hbn = 0, hwv = 0;
      const bool halo = cfg == 42 && dm::halo_cfg((int)cfg, hbn, hwv) && dm::conv_halo_supported(g);
      TORCH_CHECK(cfg == 80 || pipe || halo,
                  "red_*: a cfg 80, pipelined (90-93) or cfg 42 data gradient");
      need_bf16_nhwc(*red_y, "red_y");
      TORCH_CHECK(red_y->sizes() == dx.sizes(), "red_y: dx's shape");
      TORCH_CHECK(red_scale && red_shift && red_mean && red_invstd && red_part,
                  "red_*: scale, shift, mean, invstd and part are all required");
      need_f32(*red_scale, "red_scale", Cin);
      need_f32(*red_shift, "red_shift", Cin);
      need_f32(*red_mean, "red_mean", Cin);
      need_f32(*red_invstd, "red_invstd", Cin);
      need_f32(*red_part, "red_part", conv_stats_rows(g.M, cfg, Cin) * 2 * Cin);
      const unsigned char* rmask = nullptr;
      if (red_mask.has_value()) {
        TORCH_CHECK(red_mask->is_cuda() && red_mask->scalar_type() == at::kByte &&
                        red_mask->is_contiguous() && red_mask->numel() * 8 >= dx.numel(),
                    "red_mask: uint8 [numel/8] on the device");
        rmask = red_mask->data_ptr<uint8_t>();
      }
      const dm::BnBwdRed red{bp(*red_y), rmask, fp(*red_scale), fp(*red_shift), fp(*red_mean),
                             fp(*red_invstd), fp(*red_part)};
      if (pipe)
        dm::conv_pipe(bp(dy), bp(wd), bp(dx), addp, nullptr, g, (int)cfg, st, &red);
      else if (halo)
        dm::conv_halo(bp(dy), bp(wd), bp(dx), addp, nullptr, g, hbn, hwv, st, nullptr, nullptr, &red,
                      has_bwd ? &bwd : nullptr);
      else
        dm::conv_res64(bp(dy), bp(wd), bp(dx), addp, nullptr, g, st, nullptr, nullptr, &red);
      return;
    }
    if (has_bwd) {
      int hbn = 0, hwv = 0;
      dm::halo_cfg((int)cfg, hbn, hwv);
      dm::conv_halo(bp(dy), bp(wd), bp(dx), addp, nullptr, g, hbn, hwv, st, nullptr, nullptr, nullptr,
                    &bwd);
      return;
    }
    dm::igemm_fwd(bp(dy), bp(wd), bp(dx), addp, nullptr, g, cfg, st);
    return;
  }
  TORCH_CHECK(!has_bwd, "bwd_*: stride-1 data gradients only");
  // parity classes write disjoint output pixels; a class with no taps (e.g. the odd
  // pixels of a 1x1/s2 conv) is exactly zero, so zero-fill once up front when needed
  bool any_empty = false;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      const int kh0 = (a + pad) & 1, kw0 = (b + pad) & 1;
      if ((KH - kh0 + 1) / 2 <= 0 || (KW - kw0 + 1) / 2 <= 0) any_empty = true;
    }
  if (any_empty && !accumulate)
    TORCH_CHECK(hipMemsetAsync(dx.data_ptr(), 0, dx.numel() * 2, st) == hipSuccess);
  dm::ConvGeomSet set{};
  int ng = 0;
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      auto g = base;
      g.Hg = (H - a + 1) / 2; g.Wg = (W - b + 1) / 2;
      if (g.Hg <= 0 || g.Wg <= 0) continue;
      const int kh0 = (a + pad) & 1, kw0 = (b + pad) & 1;
      const int nth = (KH - kh0 + 1) / 2, ntw = (KW - kw0 + 1) / 2;
      if (nth <= 0 || ntw <= 0) continue;
      g.isy = 1; g.isx = 1; g.osy = 2; g.osx = 2; g.oy0 = a; g.ox0 = b;
      g.nth = nth; g.ntw = ntw;
      g.dy0 = (a + pad - kh0) / 2; g.dys = -1; g.dx0 = (b + pad - kw0) / 2; g.dxs = -1;
      g.kh0 = kh0; g.khs = 2; g.kw0 = kw0; g.kws = 2;
      g.M = (long long)N * g.Hg * g.Wg; g.K = nth * ntw * Cout;
      dm::geom_finalize(g);
      set.g[ng++] = g;
    }
  const bool multi_igemm = cfg == 11 || cfg == 12 || cfg == 13 || cfg == 14 || cfg == 15 ||
                           cfg == 16 || cfg == 17;
  // the pipelined tiles merge a projection of dy's own channel count (ResNet: always)
  const bool multi_pipe = cfg >= 90 && cfg <= 93;
  dm::DgradSeg2 seg2{};
  const bool merged = dy2.has_value();
  if (merged) {
    TORCH_CHECK((multi_igemm || (multi_pipe && dy2->size(3) == Cout)) && !accumulate && ng == 4 &&
                    pad == 1 && KH == 3 && KW == 3,
                "dy2: a 3x3/s2/p1 data gradient on an igemm tile (cfg 11-17) or a pipelined tile "
                "(cfg 90-93, projection channels == dy's), no add");
    need_bf16_nhwc(*dy2, "dy2");
    TORCH_CHECK(dy2->size(0) == N && dy2->size(1) == OH && dy2->size(2) == OW && dy2->size(3) % 64 == 0,
                "dy2: [N, OH, OW, C2] with dy's grid, C2 % 64 == 0");
    TORCH_CHECK(wd2.has_value() && wd2->scalar_type() == at::kBFloat16 && wd2->is_contiguous() &&
                    wd2->numel() == (int64_t)Cin * dy2->size(3),
                "wd2 must be bf16 [Cin][1][1][C2]");
    // class (a, b) = (0, 0) is geometry 0 (the a-major loop above): rows (y, x) are the output
    // pixels (2y, 2x), read dY at (y, x) through the centre tap -- the 1x1/s2/p0 map
    TORCH_CHECK(set.g[0].oy0 == 0 && set.g[0].ox0 == 0 && set.g[0].Hg == OH && set.g[0].Wg == OW,
                "dy2: parity class (0,0) must cover dy's grid");
    seg2.X2 = dy2->data_ptr();
    seg2.W2 = wd2->data_ptr();
    seg2.x2bytes = (unsigned)(dy2->numel() * 2);
    seg2.w2bytes = (unsigned)(wd2->numel() * 2);
    seg2.C2 = (int)dy2->size(3);
    seg2.z = 0;
  }
  if (red_y.has_value()) {
    TORCH_CHECK((multi_igemm || multi_pipe) && !accumulate && !any_empty && ng == 4,
                "red_* with stride 2: a complete data gradient (all 4 parity classes, no add) on "
                "an igemm (cfg 11-17) or pipelined (cfg 90-93) tile");
    need_bf16_nhwc(*red_y, "red_y");
    TORCH_CHECK(red_y->sizes() == dx.sizes(), "red_y: dx's shape");
    TORCH_CHECK(red_scale && red_shift && red_mean && red_invstd && red_part,
                "red_*: scale, shift, mean, invstd and part are all required");
    need_f32(*red_scale, "red_scale", Cin);
    need_f32(*red_shift, "red_shift", Cin);
    need_f32(*red_mean, "red_mean", Cin);
    need_f32(*red_invstd, "red_invstd", Cin);
    need_f32(*red_part, "red_part",
             (multi_pipe ? dm::pipe_multi_rows(set, ng) : dm::igemm_multi_rows(set, ng, (int)cfg)) *
                 2 * Cin);
    const unsigned char* rmask = nullptr;
    if (red_mask.has_value()) {
      TORCH_CHECK(red_mask->is_cuda() && red_mask->scalar_type() == at::kByte &&
                      red_mask->is_contiguous() && red_mask->numel() * 8 >= dx.numel(),
                  "red_mask: uint8 [numel/8] on the device");
      rmask = red_mask->data_ptr<uint8_t>();
    }
    const dm::BnBwdRed red{bp(*red_y), rmask, fp(*red_scale), fp(*red_shift), fp(*red_mean),
                           fp(*red_invstd), fp(*red_part)};
    const bool ok = multi_pipe
        ? dm::conv_pipe_multi(bp(dy), bp(wd), bp(dx), nullptr, set, ng, (int)cfg, st,
                              merged ? &seg2 : nullptr, &red)
        : dm::igemm_fwd_multi(bp(dy), bp(wd), bp(dx), nullptr, nullptr, set, ng, (int)cfg, st,
                              merged ? &seg2 : nullptr, &red);
    TORCH_CHECK(ok, "stride-2 dgrad with reduction: unsupported cfg / geometry");
    return;
  }
  if (merged) {
    const bool ok = multi_pipe
        ? dm::conv_pipe_multi(bp(dy), bp(wd), bp(dx), nullptr, set, ng, (int)cfg, st, &seg2, nullptr)
        : dm::igemm_fwd_multi(bp(dy), bp(wd), bp(dx), nullptr, nullptr, set, ng, (int)cfg, st, &seg2,
                              nullptr);
    TORCH_CHECK(ok, "merged stride-2 dgrad: unsupported cfg / geometry");
    return;
  }
  // pipelined tiles: all parity classes in one launch (blockIdx.y = class)
  if (cfg >= 90 && cfg <= 93 && ng > 0 &&
      dm::conv_pipe_multi(bp(dy), bp(wd), bp(dx), accumulate ? bp(dx) : nullptr, set, ng, (int)cfg, st))
    return;
  // all parity classes in one launch (blockIdx.z = class) when the tile supports it
  if (ng > 0 && dm::igemm_fwd_multi(bp(dy), bp(wd), bp(dx), accumulate ? bp(dx) : nullptr, nullptr,
                                    set, ng, (int)cfg, st))
    return;
  for (int i = 0; i < ng; ++i)
    dm::igemm_fwd(bp(dy), bp(wd), bp(dx), accumulate ? bp(dx) : nullptr, nullptr, set.g[i], cfg, st);
}

// dw (fp32 OIHW [Cout][Cin][KH][KW]) = beta*dw + Σ_m dy ⊗ im2col(x)
void conv_wgrad(at::Tensor x, at::Tensor dy, at::Tensor dw, at::Tensor slab, int64_t Cin,
                int64_t KH, int64_t KW, int64_t stride, int64_t pad, double beta, int64_t S,
                int64_t cfg, bool s2d, c10::optional<at::Tensor> pre_scale,
                c10::optional<at::Tensor> pre_shift, c10::optional<at::Tensor> bwd_y,
                c10::optional<at::Tensor> bwd_coef, c10::optional<at::Tensor> bwd_scale,
                c10::optional<at::Tensor> bwd_shift, c10::optional<at::Tensor> bwd_mask) {
  // s2d: x/dy are the space-to-depth stem operands (4x4/s1 conv over 4*Cin channels);
  // dw is the original [Cout][Cin][7][7] gradient
  // bwd_* (optional, cfg 4): dy is a BatchNorm's OUTPUT gradient; the halo weight gradient
  // stages that BN's backward a*dz' + b*y + c itself (bwd_in)
  need_bf16_nhwc(x, "x");
  need_bf16_nhwc(dy, "dy");
  const int Cout = dy.size(3);
  need_f32(dw, "dw", s2d ? (int64_t)Cout * Cin * 49 : (int64_t)Cout * Cin * KH * KW);
  auto g = fwd_geom(x, Cout, KH, KW, stride, pad, dy.size(1), dy.size(2));
  TORCH_CHECK(dy.size(0) == x.size(0));
  need_f32(slab, "slab", (int64_t)S * Cout * g.K);
  const long long steps = (g.M + 63) / 64;
  const long long mchunk = ((steps + S - 1) / S) * 64;  // multiple of both kernels' row step
  const DeviceGuard guard(x.device());
  auto st = cur_stream();
  if (bwd_y.has_value()) {
    TORCH_CHECK(cfg == 4 && !s2d && bwd_coef.has_value() && dm::wgrad_halo_supported(g),
                "bwd_*: the 9-tap halo weight gradient (cfg 4), a 3x3/s1/p1 geometry, bwd_coef");
    const dm::BnBwdIn bwd = bwd_in(dy, *bwd_y, *bwd_coef, bwd_scale, bwd_shift, bwd_mask);
    const float *psc = nullptr, *psh = nullptr;
    if (pre_scale.has_value()) {
      TORCH_CHECK(pre_shift.has_value(), "pre_scale needs pre_shift");
      need_f32(*pre_scale, "pre_scale", x.size(3));
      need_f32(*pre_shift, "pre_shift", x.size(3));
      psc = fp(*pre_scale);
      psh = fp(*pre_shift);
    }
    dm::wgrad_halo(bp(x), bp(dy), fp(slab), g, (int)S, mchunk, 3, st, psc, psh, &bwd);
  } else if (pre_scale.has_value()) {
    // x = previous conv's raw output, operand relu(x*sc + sh)
    TORCH_CHECK(pre_shift.has_value() && !s2d, "pre_scale needs pre_shift (not with s2d)");
    need_f32(*pre_scale, "pre_scale", x.size(3));
    need_f32(*pre_shift, "pre_shift", x.size(3));
    const float *psc = fp(*pre_scale), *psh = fp(*pre_shift);
    if (cfg == 8) {
      dm::wgrad_res64(bp(x), bp(dy), fp(slab), g, (int)S, st, psc, psh);
    } else {
      TORCH_CHECK((cfg == 4 || cfg == 5) && dm::wgrad_halo_supported(g),
                  "fused pre-BN needs the halo wgrad (cfg 4/5/8) and a 3x3/s1/p1 geometry");
      dm::wgrad_halo(bp(x), bp(dy), fp(slab), g, (int)S, mchunk, cfg == 4 ? 3 : 1, st, psc, psh);
    }
  } else {
    dm::igemm_wgrad(bp(x), bp(dy), fp(slab), g, (int)S, mchunk, cfg, st);
  }
  if (s2d)
    dm::wgrad_reduce_s2d(fp(slab), (int)S, Cout, (int)Cin, g.C, fp(dw), (float)beta, st);
  else
    dm::wgrad_reduce(fp(slab), (int)S, Cout, g.C, (int)Cin, KH, KW, fp(dw), (float)beta, st);
}

void pack_weights_s2d(at::Tensor w, at::Tensor wf) {
  need_f32(w, "w");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 7 && w.size(3) == 7, "s2d stem needs a 7x7 kernel");
  const int Cout = w.size(0), C = w.size(1);
  TORCH_CHECK(wf.scalar_type() == at::kBFloat16 && wf.numel() % (Cout * 16) == 0);
  const int Cp = wf.numel() / (Cout * 16);
  TORCH_CHECK(Cp % 8 == 0 && Cp >= 4 * C);
  const DeviceGuard guard(w.device());
  dm::pack_weights_s2d(fp(w), bp(wf), Cout, C, Cp, cur_stream());
}

// idx (optional, int64 [y.size(0)] on the device): y's image n is x's row idx[n] -- the
// device-resident loader's batch gather fused into the packing pass (x = the whole dataset)
void pack_input_s2d(at::Tensor x, at::Tensor y, c10::optional<at::Tensor> idx) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16);
  need_bf16_nhwc(y, "y");
  TORCH_CHECK(x.size(2) % 2 == 0 && x.size(3) % 2 == 0, "s2d needs even H, W");
  const bool gather = idx.has_value() && idx->defined();
  if (gather) {
    TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kLong && idx->is_contiguous() &&
                    idx->numel() == y.size(0), "idx: int64 [N] row indices on the device");
  } else {
    TORCH_CHECK(y.size(0) == x.size(0));
  }
  TORCH_CHECK(y.size(1) * 2 == x.size(2) && y.size(2) * 2 == x.size(3) && y.size(3) >= 4 * x.size(1));
  const DeviceGuard guard(x.device());
  dm::pack_input_s2d(x.data_ptr(), x.scalar_type() == at::kBFloat16, bp(y), y.size(0), x.size(1),
                     y.size(1), y.size(2), y.size(3), x.stride(0), x.stride(1), x.stride(2),
                     x.stride(3),
                     gather ? reinterpret_cast<const long long*>(idx->data_ptr<int64_t>()) : nullptr,
                     x.size(0), cur_stream());
}

void pack_weights(at::Tensor w, at::Tensor wf, c10::optional<at::Tensor> wd, int64_t Cpad) {
  need_f32(w, "w");
  TORCH_CHECK(w.dim() == 4);
  const int Cout = w.size(0), Cin = w.size(1), KH = w.size(2), KW = w.size(3);
  TORCH_CHECK(wf.scalar_type() == at::kBFloat16 && wf.numel() == (int64_t)Cout * KH * KW * Cpad);
  bf* wdp = nullptr;
  if (wd.has_value()) {
    TORCH_CHECK(wd->scalar_type() == at::kBFloat16 && wd->numel() == (int64_t)Cin * KH * KW * Cout);
    wdp = bp(*wd);
  }
  const DeviceGuard guard(w.device());
  dm::pack_weights(fp(w), bp(wf), wdp, Cout, Cin, Cpad, KH, KW, cur_stream());
}

// ------------------------------------------------------------------ BN
// every conv layer's weight packing in one launch (see pack_weights_multi_kernel)
void pack_weights_multi(at::Tensor desc, at::Tensor prefix, int64_t total) {
  TORCH_CHECK(desc.is_cuda() && prefix.is_cuda() && desc.scalar_type() == at::kLong &&
              prefix.scalar_type() == at::kLong, "desc/prefix: int64 device tensors");
  const int nl = prefix.numel() - 1;
  TORCH_CHECK(nl >= 1 && nl <= 32 && desc.numel() == 8 * nl, "pack_weights_multi: 1..32 layers");
  const DeviceGuard guard(desc.device());
  dm::pack_weights_multi((const long long*)desc.data_ptr(), (const long long*)prefix.data_ptr(), nl,
                         total, cur_stream());
}

// LDS-tiled variant: tprefix[l] = first 32x32 (co, ci) tile of layer l
void pack_weights_tiled(at::Tensor desc, at::Tensor tprefix, int64_t ntiles) {
  TORCH_CHECK(desc.is_cuda() && tprefix.is_cuda() && desc.scalar_type() == at::kLong &&
              tprefix.scalar_type() == at::kInt, "desc int64 / tprefix int32 device tensors");
  const int nl = tprefix.numel() - 1;
  TORCH_CHECK(nl >= 1 && nl <= 32 && desc.numel() == 8 * nl, "pack_weights_tiled: 1..32 layers");
  TORCH_CHECK(ntiles >= 1 && ntiles < (1 << 24), "pack_weights_tiled: tile count");
  const DeviceGuard guard(desc.device());
  dm::pack_weights_tiled((const long long*)desc.data_ptr(), tprefix.data_ptr<int>(), nl, (int)ntiles,
                         cur_stream());
}

void bn_stats_finalize(at::Tensor stats, int64_t T, double count, at::Tensor gamma, at::Tensor beta,
                       c10::optional<at::Tensor> rmean, c10::optional<at::Tensor> rvar,
                       double momentum, double eps, at::Tensor scale, at::Tensor shift,
                       at::Tensor mean, at::Tensor invstd, at::Tensor work,
                       c10::optional<at::Tensor> num_batches) {
  const int C = gamma.numel();
  need_f32(stats, "stats", T * 2 * C);
  long long* nb = nullptr;  // BatchNorm num_batches_tracked, incremented in the finalize kernel
  if (num_batches.has_value()) {
    TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1 &&
                num_batches->device() == stats.device(), "num_batches: int64 scalar on the device");
    nb = (long long*)num_batches->data_ptr();
  }
  need_f32(work, "work", 256 * 2 * C);
  for (auto* t : {&gamma, &beta, &scale, &shift, &mean, &invstd}) need_f32(*t, "bn vec", C);
  const DeviceGuard guard(stats.device());
  dm::bn_stats_finalize(fp(stats), T, C, count, fp(gamma), fp(beta),
                        rmean.has_value() ? fp(*rmean) : nullptr, rvar.has_value() ? fp(*rvar) : nullptr,
                        momentum, eps, fp(scale), fp(shift), fp(mean), fp(invstd), fp(work), nb,
                        cur_stream());
}

void bn_eval_coeffs(at::Tensor gamma, at::Tensor beta, at::Tensor rmean, at::Tensor rvar, double eps,
                    at::Tensor scale, at::Tensor shift) {
  const int C = gamma.numel();
  const DeviceGuard guard(gamma.device());
  dm::bn_eval_coeffs(fp(gamma), fp(beta), fp(rmean), fp(rvar), eps, C, fp(scale), fp(shift),
                     cur_stream());
}

void bn_apply(at::Tensor y, c10::optional<at::Tensor> res, at::Tensor scale, at::Tensor shift,
              at::Tensor out, bool relu, c10::optional<at::Tensor> mask) {
  need_bf16_nhwc(y, "y");
  need_bf16_nhwc(out, "out");
  const int C = y.size(3);
  need_f32(scale, "scale", C);
  need_f32(shift, "shift", C);
  const bf* rp = nullptr;
  if (res.has_value()) { need_bf16_nhwc(*res, "res"); TORCH_CHECK(res->sizes() == y.sizes()); rp = bp(*res); }
  TORCH_CHECK(out.sizes() == y.sizes());
  const DeviceGuard guard(y.device());
  uint8_t* mp = nullptr;
  if (mask.has_value()) {
    TORCH_CHECK(relu, "mask: ReLU outputs only");
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                mask->numel() == y.numel() / 8, "mask: contiguous uint8, one byte per 8 channels");
    mp = (uint8_t*)mask->data_ptr();
  }
  dm::bn_apply(bp(y), rp, fp(scale), fp(shift), bp(out), y.numel(), C, relu, cur_stream(), mp);
}

int64_t bn_bwd_work(int64_t M, int64_t C) { return (int64_t)dm::bn_bwd_groups(M, C) * 2 * C + 3 * C + 256 * 2 * C; }

// mode: 0 no ReLU, 1 mask from `out`, 2 mask from y*scale+shift, 3 (stem) dz gathered
// from the following max-pool's gradient (pdy, pidx; pool K/S/P) with mask from y, 4 mask
// from the 1-bit (out > 0) mask that bn_apply wrote in the forward.
// Stem backward without the full-resolution dy: BN-backward coefficients from the pooled-
// domain sums (pre_slab, bn_bwd_reduce_masked), then the fused gather + apply + s2d weight
// gradient (conv_stem.hip) into slab, then the fixed-order reduce into dw [Cout][Cin][7][7].
bool stem_bwd_fused_supported(at::Tensor y, at::Tensor xs) {
  return y.dim() == 4 && xs.dim() == 4 && y.size(0) == xs.size(0) && y.size(1) == xs.size(1) &&
         y.size(2) == xs.size(2) &&
         dm::stem_wgrad_fused_supported(y.size(0), y.size(1), y.size(2), y.size(3), xs.size(3));
}

int64_t stem_bwd_slab_floats(int64_t N, int64_t H) {
  return (int64_t)dm::stem_wgrad_fused_blocks((int)N, (int)H) * 64 * 256;
}

void stem_bwd_fused(at::Tensor y, at::Tensor mean, at::Tensor invstd, at::Tensor gamma,
                    at::Tensor dgamma, at::Tensor dbeta, double gbeta, at::Tensor scale,
                    at::Tensor shift, at::Tensor pdy, at::Tensor pidx, at::Tensor pre_slab,
                    int64_t pre_rows, at::Tensor xs, int64_t Cin, at::Tensor dw, double wbeta,
                    at::Tensor work, at::Tensor slab) {
  need_bf16_nhwc(y, "y");
  need_bf16_nhwc(xs, "xs");
  need_bf16_nhwc(pdy, "pdy");
  TORCH_CHECK(stem_bwd_fused_supported(y, xs), "stem_bwd_fused: unsupported shape");
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  TORCH_CHECK(pdy.size(0) == N && pdy.size(1) == H / 2 && pdy.size(2) == W / 2 && pdy.size(3) == C,
              "pdy must be the 3x3/s2/p1 pooled gradient");
  TORCH_CHECK(pidx.is_cuda() && pidx.scalar_type() == at::kByte && pidx.is_contiguous() &&
              pidx.numel() == pdy.numel());
  const long long M = (long long)N * H * W;
  need_f32(work, "work", bn_bwd_work(M, C));
  need_f32(pre_slab, "pre_slab", pre_rows * 2 * C);
  need_f32(scale, "scale", C);
  need_f32(shift, "shift", C);
  need_f32(dw, "dw", (int64_t)C * Cin * 49);
  const int S = dm::stem_wgrad_fused_blocks(N, H);
  need_f32(slab, "slab", (int64_t)S * 64 * 256);
  const DeviceGuard guard(y.device());
  auto st = cur_stream();
  // mode 3, dy = nullptr: finalize only; with pre_part the coefficients land at work[0, 3C)
  dm::bn_backward(nullptr, nullptr, bp(y), fp(mean), fp(invstd), fp(gamma), fp(dgamma), fp(dbeta),
                  (float)gbeta, M, C, 3, fp(scale), fp(shift), bp(pdy),
                  (const uint8_t*)pidx.data_ptr(), H, W, H / 2, W / 2, 3, 2, 1, nullptr, nullptr,
                  fp(work), st, fp(pre_slab), (int)pre_rows, nullptr);
  dm::stem_wgrad_fused(bp(xs), bp(y), bp(pdy), (const uint8_t*)pidx.data_ptr(), fp(work),
                       fp(scale), fp(shift), fp(slab), N, H, W, S, st);
  dm::wgrad_reduce_s2d(fp(slab), S, C, (int)Cin, xs.size(3), fp(dw), (float)wbeta, st);
}


void wgrad_reduce_s2d(at::Tensor slab, int64_t S, int64_t Cout, int64_t Cin, int64_t Cp,
                      at::Tensor dw, double beta) {
  need_f32(slab, "slab", S * Cout * 16 * Cp);
  need_f32(dw, "dw", Cout * Cin * 49);
  const DeviceGuard guard(slab.device());
  dm::wgrad_reduce_s2d(fp(slab), (int)S, (int)Cout, (int)Cin, (int)Cp, fp(dw), (float)beta,
                       cur_stream());
}

void bn_backward(c10::optional<at::Tensor> dout, c10::optional<at::Tensor> out, at::Tensor y,
                 at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor dgamma,
                 at::Tensor dbeta, double gbeta, int64_t mode, c10::optional<at::Tensor> scale,
                 c10::optional<at::Tensor> shift, c10::optional<at::Tensor> pdy,
                 c10::optional<at::Tensor> pidx, int64_t K, int64_t S, int64_t P,
                 c10::optional<at::Tensor> dy, c10::optional<at::Tensor> dres, at::Tensor work,
                 c10::optional<at::Tensor> pre_slab, int64_t pre_rows,
                 c10::optional<at::Tensor> mask) {
  // dy None: reduce + finalize only -- dgamma/dbeta and the coefficients a, b, cc of
  // dy = a*dz + b*y + cc are left in work (bn_bwd_coef_offset) for a consumer kernel that
  // applies them while staging its operand (conv_dgrad / conv_wgrad bwd_*)
  need_bf16_nhwc(y, "y");
  if (dy.has_value()) {
    need_bf16_nhwc(*dy, "dy");
    TORCH_CHECK(dy->sizes() == y.sizes());
  } else {
    TORCH_CHECK(!dres.has_value() && mode != 3, "dy None: no residual gradient, no pool mode");
  }
  TORCH_CHECK(mode >= 0 && mode <= 4);
  const int C = y.size(3);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "bn_backward: C/8 must divide 256");
  const long long M = y.numel() / C;
  need_f32(work, "work", bn_bwd_work(M, C));
  if (pre_slab.has_value()) {
    TORCH_CHECK(pre_rows >= 1, "pre_slab: >= 1 row");
    need_f32(*pre_slab, "pre_slab", pre_rows * 2 * C);
  }
  const bf* doutp = nullptr;
  if (mode != 3) {
    TORCH_CHECK(dout.has_value());
    need_bf16_nhwc(*dout, "dout");
    TORCH_CHECK(dout->sizes() == y.sizes());
    doutp = bp(*dout);
  }
  const bf* outp = nullptr;
  if (mode == 1) {
    TORCH_CHECK(out.has_value());
    need_bf16_nhwc(*out, "out");
    TORCH_CHECK(out->sizes() == y.sizes());
    outp = bp(*out);
  }
  const float *scp = nullptr, *shp = nullptr;
  if (mode == 2 || mode == 3) {
    TORCH_CHECK(scale.has_value() && shift.has_value());
    need_f32(*scale, "scale", C);
    need_f32(*shift, "shift", C);
    scp = fp(*scale);
    shp = fp(*shift);
  }
  const bf* pdyp = nullptr;
  const uint8_t* pidxp = nullptr;
  int OH = 0, OW = 0;
  if (mode == 3) {
    TORCH_CHECK(pdy.has_value() && pidx.has_value());
    need_bf16_nhwc(*pdy, "pdy");
    TORCH_CHECK(pidx->scalar_type() == at::kByte && pidx->numel() == pdy->numel());
    TORCH_CHECK(pdy->size(0) == y.size(0) && pdy->size(3) == C);
    OH = pdy->size(1);
    OW = pdy->size(2);
    TORCH_CHECK(OH == (y.size(1) + 2 * P - K) / S + 1 && OW == (y.size(2) + 2 * P - K) / S + 1);
    pdyp = bp(*pdy);
    pidxp = (const uint8_t*)pidx->data_ptr();
  }
  const uint8_t* mp = nullptr;
  if (mode == 4) {
    TORCH_CHECK(mask.has_value() && mask->is_cuda() && mask->scalar_type() == at::kByte &&
                mask->is_contiguous() && mask->numel() == y.numel() / 8, "mode 4 needs the uint8 mask");
    mp = (const uint8_t*)mask->data_ptr();
  }
  bf* drp = nullptr;
  if (dres.has_value()) { need_bf16_nhwc(*dres, "dres"); drp = bp(*dres); }
  const DeviceGuard guard(y.device());
  dm::bn_backward(doutp, outp, bp(y), fp(mean), fp(invstd), fp(gamma), fp(dgamma), fp(dbeta),
                  (float)gbeta, M, C, (int)mode, scp, shp, pdyp, pidxp, y.size(1), y.size(2), OH,
                  OW, K, S, P, dy.has_value() ? bp(*dy) : nullptr, drp, fp(work), cur_stream(), pre_slab.has_value() ? fp(*pre_slab) : nullptr,
                  (int)pre_rows, mp);
}

void bn_relu_maxpool(at::Tensor y, at::Tensor scale, at::Tensor shift, at::Tensor out,
                     at::Tensor idx, int64_t K, int64_t S, int64_t P,
                     c10::optional<at::Tensor> yarg) {
  need_bf16_nhwc(y, "y");
  need_bf16_nhwc(out, "out");
  const int C = y.size(3);
  need_f32(scale, "scale", C);
  need_f32(shift, "shift", C);
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == out.numel());
  TORCH_CHECK(out.size(1) == (y.size(1) + 2 * P - K) / S + 1 && out.size(2) == (y.size(2) + 2 * P - K) / S + 1);
  const DeviceGuard guard(y.device());
  bf* yargp = nullptr;
  if (yarg.has_value()) {
    need_bf16_nhwc(*yarg, "yarg");
    TORCH_CHECK(yarg->sizes() == out.sizes(), "yarg: pooled shape");
    yargp = bp(*yarg);
  }
  dm::bn_relu_maxpool(bp(y), fp(scale), fp(shift), bp(out), (uint8_t*)idx.data_ptr(), y.size(0),
                      y.size(1), y.size(2), C, out.size(1), out.size(2), K, S, P, cur_stream(),
                      yargp);
}

int64_t bn_bwd_rows(int64_t M, int64_t C) { return dm::bn_bwd_groups(M, C); }

// element offset of the [3][C] backward coefficients in bn_backward's work buffer
int64_t bn_bwd_coef_offset(int64_t M, int64_t C, bool pre_sums) {
  return pre_sums ? 0 : (int64_t)dm::bn_bwd_groups(M, C) * 2 * C;
}

// Σdz, Σdz·x̂ partials of (dout masked by y*scale+shift > 0) -> part [rows][2C]; returns rows
int64_t bn_bwd_reduce_masked(at::Tensor dout, at::Tensor y, at::Tensor mean, at::Tensor invstd,
                             at::Tensor scale, at::Tensor shift, at::Tensor part) {
  need_bf16_nhwc(dout, "dout");
  need_bf16_nhwc(y, "y");
  TORCH_CHECK(dout.sizes() == y.sizes());
  const int C = y.size(3);
  TORCH_CHECK(C % 8 == 0 && 256 % (C / 8) == 0, "C/8 must divide 256");
  need_f32(mean, "mean", C);
  need_f32(invstd, "invstd", C);
  need_f32(scale, "scale", C);
  need_f32(shift, "shift", C);
  const long long M = y.numel() / C;
  need_f32(part, "part", (int64_t)dm::bn_bwd_groups(M, C) * 2 * C);
  const DeviceGuard guard(y.device());
  return dm::bn_bwd_reduce_masked(bp(dout), bp(y), fp(mean), fp(invstd), fp(scale), fp(shift), M,
                                  C, fp(part), cur_stream());
}

// ------------------------------------------------------------------ pooling / packing
void maxpool_fwd(at::Tensor x, at::Tensor y, at::Tensor idx, int64_t K, int64_t S, int64_t P) {
  need_bf16_nhwc(x, "x");
  need_bf16_nhwc(y, "y");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == y.numel());
  const DeviceGuard guard(x.device());
  dm::maxpool_fwd(bp(x), bp(y), (uint8_t*)idx.data_ptr(), x.size(0), x.size(1), x.size(2), x.size(3),
                  y.size(1), y.size(2), K, S, P, cur_stream());
}

void maxpool_bwd(at::Tensor dy, at::Tensor idx, at::Tensor dx, int64_t K, int64_t S, int64_t P) {
  need_bf16_nhwc(dy, "dy");
  need_bf16_nhwc(dx, "dx");
  const DeviceGuard guard(dy.device());
  dm::maxpool_bwd(bp(dy), (const uint8_t*)idx.data_ptr(), bp(dx), dx.size(0), dx.size(1), dx.size(2),
                  dx.size(3), dy.size(1), dy.size(2), K, S, P, cur_stream());
}

void avgpool_fwd(at::Tensor x, at::Tensor y) {
  need_bf16_nhwc(x, "x");
  TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.numel() == x.size(0) * x.size(3));
  const DeviceGuard guard(x.device());
  dm::avgpool_fwd(bp(x), bp(y), x.size(0), x.size(1) * x.size(2), x.size(3), cur_stream());
}

void avgpool_bwd(at::Tensor dy, at::Tensor dx) {
  need_bf16_nhwc(dx, "dx");
  TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && dy.numel() == dx.size(0) * dx.size(3));
  const DeviceGuard guard(dx.device());
  dm::avgpool_bwd(bp(dy), bp(dx), dx.size(0), dx.size(1) * dx.size(2), dx.size(3), cur_stream());
}

void pack_input(at::Tensor x, at::Tensor y) {
  TORCH_CHECK(x.is_cuda() && x.dim() == 4);
  TORCH_CHECK(x.scalar_type() == at::kFloat || x.scalar_type() == at::kBFloat16);
  need_bf16_nhwc(y, "y");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == x.size(2) && y.size(2) == x.size(3) &&
              y.size(3) >= x.size(1));
  const DeviceGuard guard(x.device());
  dm::pack_input(x.data_ptr(), x.scalar_type() == at::kBFloat16, bp(y), x.size(0), x.size(1),
                 x.size(2), x.size(3), y.size(3), x.stride(0), x.stride(1), x.stride(2), x.stride(3),
                 cur_stream());
}

}  // namespace

// ----------------------------------------------------------------- fused K-dense stem
// img: the raw input as stored -- (N, 3, H, W) channels_last or (N, H, W, 3) contiguous, fp32 /
// bf16 / u8; idx (optional int64 [B]): batch row -> image row (the loader's gather)
struct ImgView {
  const void* ptr;
  int dtype, N, H, W;
};
ImgView img_view(const at::Tensor& img) {
  TORCH_CHECK(img.is_cuda() && img.dim() == 4, "stem input must be a 4-D HIP tensor");
  ImgView v{img.data_ptr(), 0, (int)img.size(0), 0, 0};
  if (img.size(1) == 3 && img.size(3) != 3) {
    TORCH_CHECK(img.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem input (N,3,H,W) must be channels_last");
    v.H = img.size(2);
    v.W = img.size(3);
  } else {
    TORCH_CHECK(img.size(3) == 3 && img.is_contiguous(), "stem input (N,H,W,3) must be contiguous");
    v.H = img.size(1);
    v.W = img.size(2);
  }
  const auto t = img.scalar_type();
  TORCH_CHECK(t == at::kFloat || t == at::kBFloat16 || t == at::kByte,
              "stem input must be fp32, bf16 or uint8");
  v.dtype = t == at::kFloat ? 0 : t == at::kBFloat16 ? 1 : 2;
  return v;
}

bool stem_fused_supported(int64_t Hin, int64_t Win) { return dm::stem_fused_supported(Hin, Win); }
int64_t stem_fused_grid(int64_t N) { return dm::stem_fused_grid((int)N); }
int64_t stem_slab_cols() { return dm::stem_slab_cols(); }
// floats of the backward's slab workspace for `grid` workgroups: D and G partials + their sums
int64_t stem_bwd_slab_len(int64_t grid) {
  const int64_t gk = dm::stem_gram_cols();
  return grid * (64 * dm::stem_slab_cols() + gk * gk) + dm::stem_sums_len();
}

const long long* idx_ptr(const c10::optional<at::Tensor>& idx, int B, int Nimg) {
  if (!idx.has_value()) {
    TORCH_CHECK(B <= Nimg, "stem: batch larger than the image tensor");
    return nullptr;
  }
  TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kLong && idx->is_contiguous() &&
                  idx->numel() == B, "stem: idx must be a contiguous int64 HIP tensor of B rows");
  return reinterpret_cast<const long long*>(idx->data_ptr());
}

void stem_fwd_fused(at::Tensor img, c10::optional<at::Tensor> idx, std::vector<double> nsc,
                    std::vector<double> nbi, at::Tensor wk, at::Tensor gamma, at::Tensor pext,
                    at::Tensor code, c10::optional<at::Tensor> stats, int64_t grid) {
  const ImgView v = img_view(img);
  TORCH_CHECK(dm::stem_fused_supported(v.H, v.W), "fused stem: unsupported input size");
  need_bf16_nhwc(pext, "pext");
  const int B = pext.size(0);
  TORCH_CHECK(pext.size(1) == v.H / 4 && pext.size(2) == v.W / 4 && pext.size(3) == 64,
              "pext must be [B, H/4, W/4, 64]");
  TORCH_CHECK(code.is_cuda() && code.scalar_type() == at::kByte && code.is_contiguous() &&
              code.numel() * 2 == pext.numel(), "code must be uint8 [N][PH][PW][32] (4-bit codes)");
  TORCH_CHECK(wk.is_cuda() && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous() &&
              wk.numel() == 64 * dm::stem_wk_cols(), "wk must be packed [64][176] bf16");
  need_f32(gamma, "gamma", 64);
  TORCH_CHECK(nsc.size() == 3 && nbi.size() == 3, "3 normalisation scales / biases");
  TORCH_CHECK(grid >= 1 && grid <= B, "grid must be in [1, B]");
  if (stats.has_value()) need_f32(*stats, "stats", grid * 128);
  const float s3[3] = {(float)nsc[0], (float)nsc[1], (float)nsc[2]};
  const float b3[3] = {(float)nbi[0], (float)nbi[1], (float)nbi[2]};
  const DeviceGuard guard(pext.device());
  dm::stem_fwd_fused(v.ptr, v.dtype, idx_ptr(idx, B, v.N), s3, b3, bp(wk), fp(gamma), bp(pext),
                     (uint8_t*)code.data_ptr(), stats ? fp(*stats) : nullptr, B, v.N, v.H, v.W,
                     (int)grid, cur_stream());
}

// out = relu(scale * pext + shift); with code4: the backward's 4-bit window codes (15 where
// the output is 0) from the forward's byte codes
void stem_pool_apply(at::Tensor pext, c10::optional<at::Tensor> code, at::Tensor scale,
                     at::Tensor shift, at::Tensor out, c10::optional<at::Tensor> code4) {
  need_bf16_nhwc(pext, "pext");
  need_bf16_nhwc(out, "out");
  TORCH_CHECK(out.numel() == pext.numel() && pext.size(3) == 64, "pooled shapes");
  TORCH_CHECK(code.has_value() == code4.has_value(), "code and code4 go together");
  if (code.has_value()) {
    TORCH_CHECK(code->is_cuda() && code->scalar_type() == at::kByte && code->is_contiguous() &&
                    code->numel() * 2 == pext.numel(), "code must be uint8 [N][PH][PW][32]");
    TORCH_CHECK(code4->is_cuda() && code4->scalar_type() == at::kByte && code4->is_contiguous() &&
                    code4->numel() * 2 == pext.numel(), "code4 must be uint8 [N][PH][PW][32]");
  }
  need_f32(scale, "scale", 64);
  need_f32(shift, "shift", 64);
  const DeviceGuard guard(pext.device());
  dm::stem_pool_apply(bp(pext), code ? (const uint8_t*)code->data_ptr() : nullptr, fp(scale),
                      fp(shift), bp(out), code4 ? (uint8_t*)code4->data_ptr() : nullptr,
                      pext.numel(), cur_stream());
}

// BN-backward coefficients (a, b, cc) from the pooled-domain sums (pre_slab); the per-workgroup
// D = dz^T X and G = X^T X partials into dslab; dW = beta dW + a D + b W G + cc colsum(X)
void stem_bwd_fused2(at::Tensor img, c10::optional<at::Tensor> idx, std::vector<double> nsc,
                     std::vector<double> nbi, at::Tensor wk, at::Tensor pdy, at::Tensor code4,
                     at::Tensor mean, at::Tensor invstd, at::Tensor gamma, at::Tensor dgamma,
                     at::Tensor dbeta, double gbeta, at::Tensor pre_slab, int64_t pre_rows,
                     at::Tensor dw, double wbeta, at::Tensor work, at::Tensor dslab, int64_t grid) {
  const ImgView v = img_view(img);
  TORCH_CHECK(dm::stem_fused_supported(v.H, v.W), "fused stem: unsupported input size");
  need_bf16_nhwc(pdy, "pdy");
  const int B = pdy.size(0), C = 64;
  TORCH_CHECK(pdy.size(1) == v.H / 4 && pdy.size(2) == v.W / 4 && pdy.size(3) == C, "pdy shape");
  TORCH_CHECK(code4.is_cuda() && code4.scalar_type() == at::kByte && code4.is_contiguous() &&
                  code4.numel() * 2 == pdy.numel(), "code4 must be uint8 [N][PH][PW][32]");
  const long long M = (long long)B * (v.H / 2) * (v.W / 2);
  need_f32(work, "work", bn_bwd_work(M, C));
  need_f32(pre_slab, "pre_slab", pre_rows * 2 * C);
  need_f32(dw, "dw", (int64_t)C * 3 * 49);
  TORCH_CHECK(wk.is_cuda() && wk.scalar_type() == at::kBFloat16 && wk.is_contiguous() &&
              wk.numel() == 64 * dm::stem_wk_cols(), "wk must be packed [64][176] bf16");
  TORCH_CHECK(grid >= 1 && grid <= B, "grid must be in [1, B]");
  need_f32(dslab, "dslab", stem_bwd_slab_len(grid));
  const float s3[3] = {(float)nsc[0], (float)nsc[1], (float)nsc[2]};
  const float b3[3] = {(float)nbi[0], (float)nbi[1], (float)nbi[2]};
  const DeviceGuard guard(pdy.device());
  auto st = cur_stream();
  // mode 3, dy = nullptr: coefficients only (work[0, 3C) = a, b, cc) + dgamma / dbeta
  dm::bn_backward(nullptr, nullptr, nullptr, fp(mean), fp(invstd), fp(gamma), fp(dgamma), fp(dbeta),
                  (float)gbeta, M, C, 3, nullptr, nullptr, nullptr, nullptr, v.H / 2, v.W / 2,
                  v.H / 4, v.W / 4, 3, 2, 1, nullptr, nullptr, fp(work), st, fp(pre_slab),
                  (int)pre_rows, nullptr);
  float* d_part = fp(dslab);
  float* g_part = d_part + grid * C * dm::stem_slab_cols();
  float* sums = g_part + grid * dm::stem_gram_cols() * dm::stem_gram_cols();
  dm::stem_bwd_fused2(v.ptr, v.dtype, idx_ptr(idx, B, v.N), s3, b3, bp(wk), bp(pdy),
                      (const uint8_t*)code4.data_ptr(), d_part, g_part, B, v.N, v.H, v.W,
                      (int)grid, st);
  dm::stem_wcombine(d_part, g_part, (int)grid, bp(wk), fp(work), sums, fp(dw), (float)wbeta, st);
}

void stem_pack_weights(at::Tensor w, at::Tensor wk) {
  need_f32(w, "w", 64 * 3 * 49);
  TORCH_CHECK(w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7,
              "stem weight must be [64][3][7][7]");
  TORCH_CHECK(wk.scalar_type() == at::kBFloat16 && wk.numel() == 64 * dm::stem_wk_cols(), "wk");
  const DeviceGuard guard(w.device());
  dm::stem_pack_weights(fp(w), bp(wk), cur_stream());
}

void register_resnet(pybind11::module_& m) {
  m.def("conv_fwd", &conv_fwd, py::arg("x"), py::arg("wpack"), py::arg("y"), py::arg("stats"),
        py::arg("add"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("cfg"), py::arg("pre_scale") = py::none(), py::arg("pre_shift") = py::none());
  m.def("conv_stats_rows", &conv_stats_rows, py::arg("M"), py::arg("cfg"), py::arg("ncols") = -1);
  m.def("conv_dgrad", &conv_dgrad, py::arg("dy"), py::arg("wd"), py::arg("dx"), py::arg("KH"),
        py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("add") = py::none(), py::arg("cfg") = 12, py::arg("add_mask") = py::none(),
        py::arg("red_y") = py::none(), py::arg("red_scale") = py::none(),
        py::arg("red_shift") = py::none(), py::arg("red_mean") = py::none(),
        py::arg("red_invstd") = py::none(), py::arg("red_part") = py::none(),
        py::arg("red_mask") = py::none(), py::arg("dy2") = py::none(),
        py::arg("wd2") = py::none(), py::arg("bwd_y") = py::none(),
        py::arg("bwd_coef") = py::none(), py::arg("bwd_scale") = py::none(),
        py::arg("bwd_shift") = py::none(), py::arg("bwd_mask") = py::none());
  m.def("bn_fold_supported", &bn_fold_supported);
  m.def("dgrad_s2_red_rows", &dgrad_s2_red_rows, py::arg("N"), py::arg("H"), py::arg("W"),
        py::arg("cfg"));
  m.def("conv_wgrad", &conv_wgrad, py::arg("x"), py::arg("dy"), py::arg("dw"), py::arg("slab"),
        py::arg("Cin"), py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"),
        py::arg("beta"), py::arg("S"), py::arg("cfg"), py::arg("s2d"),
        py::arg("pre_scale") = py::none(), py::arg("pre_shift") = py::none(),
        py::arg("bwd_y") = py::none(), py::arg("bwd_coef") = py::none(),
        py::arg("bwd_scale") = py::none(), py::arg("bwd_shift") = py::none(),
        py::arg("bwd_mask") = py::none());
  m.def("pack_weights", &pack_weights);
  m.def("pack_weights_multi", &pack_weights_multi);
  m.def("pack_weights_tiled", &pack_weights_tiled);
  m.def("bn_stats_finalize", &bn_stats_finalize, py::arg("stats"), py::arg("T"), py::arg("count"),
        py::arg("gamma"), py::arg("beta"), py::arg("rmean"), py::arg("rvar"), py::arg("momentum"),
        py::arg("eps"), py::arg("scale"), py::arg("shift"), py::arg("mean"), py::arg("invstd"),
        py::arg("work"), py::arg("num_batches") = py::none());
  m.def("bn_eval_coeffs", &bn_eval_coeffs);
  m.def("bn_apply", &bn_apply, py::arg("y"), py::arg("res"), py::arg("scale"), py::arg("shift"),
        py::arg("out"), py::arg("relu"), py::arg("mask") = py::none());
  m.def("bn_bwd_work", &bn_bwd_work);
  m.def("stem_bwd_fused_supported", &stem_bwd_fused_supported);
  m.def("stem_bwd_slab_floats", &stem_bwd_slab_floats);
  m.def("stem_bwd_fused", &stem_bwd_fused, py::arg("y"), py::arg("mean"), py::arg("invstd"),
        py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"), py::arg("gbeta"), py::arg("scale"),
        py::arg("shift"), py::arg("pdy"), py::arg("pidx"), py::arg("pre_slab"), py::arg("pre_rows"),
        py::arg("xs"), py::arg("Cin"), py::arg("dw"), py::arg("wbeta"), py::arg("work"),
        py::arg("slab"));
  m.def("wgrad_reduce_s2d", &wgrad_reduce_s2d);
  m.def("bn_backward", &bn_backward, py::arg("dout"), py::arg("out"), py::arg("y"), py::arg("mean"), py::arg("invstd"), py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"), py::arg("gbeta"), py::arg("mode"), py::arg("scale"), py::arg("shift"), py::arg("pdy"), py::arg("pidx"), py::arg("K"), py::arg("S"), py::arg("P"), py::arg("dy"), py::arg("dres"), py::arg("work"),
        py::arg("pre_slab") = py::none(), py::arg("pre_rows") = 0, py::arg("mask") = py::none());
  m.def("bn_relu_maxpool", &bn_relu_maxpool, py::arg("y"), py::arg("scale"), py::arg("shift"),
        py::arg("out"), py::arg("idx"), py::arg("K"), py::arg("S"), py::arg("P"),
        py::arg("yarg") = py::none());
  m.def("bn_bwd_rows", &bn_bwd_rows);
  m.def("bn_bwd_coef_offset", &bn_bwd_coef_offset);
  m.def("bn_bwd_reduce_masked", &bn_bwd_reduce_masked);
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("pack_input", &pack_input);
  m.def("pack_input_s2d", &pack_input_s2d, py::arg("x"), py::arg("y"),
        py::arg("idx") = py::none());
  m.def("pack_weights_s2d", &pack_weights_s2d);
  m.def("stem_fused_supported", &stem_fused_supported);
  m.def("stem_fused_grid", &stem_fused_grid);
  m.def("stem_slab_cols", &stem_slab_cols);
  m.def("stem_bwd_slab_len", &stem_bwd_slab_len);
  m.def("stem_fwd_fused", &stem_fwd_fused, py::arg("img"), py::arg("idx"), py::arg("nsc"),
        py::arg("nbi"), py::arg("wk"), py::arg("gamma"), py::arg("pext"), py::arg("code"),
        py::arg("stats"), py::arg("grid"));
  m.def("stem_pool_apply", &stem_pool_apply, py::arg("pext"), py::arg("code"), py::arg("scale"),
        py::arg("shift"), py::arg("out"), py::arg("code4") = py::none());
  m.def("stem_bwd_fused2", &stem_bwd_fused2, py::arg("img"), py::arg("idx"), py::arg("nsc"),
        py::arg("nbi"), py::arg("wk"), py::arg("pdy"), py::arg("code4"), py::arg("mean"),
        py::arg("invstd"), py::arg("gamma"), py::arg("dgamma"), py::arg("dbeta"),
        py::arg("gbeta"), py::arg("pre_slab"), py::arg("pre_rows"), py::arg("dw"),
        py::arg("wbeta"), py::arg("work"), py::arg("dslab"), py::arg("grid"));
  m.def("stem_pack_weights", &stem_pack_weights);
}
