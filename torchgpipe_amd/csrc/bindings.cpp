// ATen bindings: registers the framework kernels as torch.ops.tgpipe.* (CUDA == HIP
// dispatch key on ROCm builds) and validates shapes / dtypes / devices before launching.
#include <algorithm>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>

#include <vector>

#include "kernels.h"

namespace tgpipe {
namespace {

hipStream_t stream_of(const at::Tensor& t) {
  return at::hip::getCurrentHIPStream(t.device().index()).stream();
}

// Optional device-resident Philox state: int64 [2] (seed, base offset) on the op's device.
const int64_t* rng_state(const c10::optional<at::Tensor>& rng, const at::Device& device) {
  if (!rng.has_value() || !rng->defined()) return nullptr;
  TORCH_CHECK(rng->is_cuda() && rng->device() == device && rng->scalar_type() == at::kLong &&
                  rng->is_contiguous() && rng->numel() == 2,
              "rng must be a contiguous int64 [2] (seed, offset) tensor on the op's device");
  return rng->data_ptr<int64_t>();
}

void check_f32_gpu(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

std::vector<at::Tensor> dna_forward(const at::Tensor& x, double p, double eps, double slope,
                                    int64_t seed, int64_t offset, bool dropout,
                                    const c10::optional<at::Tensor>& rng) {
  check_f32_gpu(x, "x");
  TORCH_CHECK(x.dim() >= 3, "expected (N, C, *spatial) input");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout probability must be in [0, 1)");
  const int64_t planes = x.size(0) * x.size(1);
  const int64_t s = planes == 0 ? 0 : x.numel() / planes;
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty_like(x);
  auto opts = x.options();
  auto mean = at::empty({planes}, opts);
  auto rstd = at::empty({planes}, opts);
  auto scale = at::empty({planes}, opts);
  launch_dna_forward(x.data_ptr<float>(), y.data_ptr<float>(), mean.data_ptr<float>(),
                     rstd.data_ptr<float>(), scale.data_ptr<float>(), planes, s,
                     static_cast<float>(p), static_cast<float>(eps), static_cast<float>(slope),
                     static_cast<uint64_t>(seed), static_cast<uint64_t>(offset), dropout,
                     rng_state(rng, x.device()), stream_of(x));
  return {y, mean, rstd, scale};
}

at::Tensor dna_backward(const at::Tensor& dy_in, const at::Tensor& x, const at::Tensor& mean,
                        const at::Tensor& rstd, const at::Tensor& scale, double slope) {
  check_f32_gpu(x, "x");
  auto dy = dy_in.contiguous();
  check_f32_gpu(dy, "dy");
  TORCH_CHECK(dy.sizes() == x.sizes(), "dy and x must have the same shape");
  const int64_t planes = x.size(0) * x.size(1);
  const int64_t s = planes == 0 ? 0 : x.numel() / planes;
  TORCH_CHECK(mean.numel() == planes && rstd.numel() == planes && scale.numel() == planes,
              "saved statistics must have N*C elements");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto dx = at::empty_like(x);
  launch_dna_backward(dy.data_ptr<float>(), x.data_ptr<float>(), mean.data_ptr<float>(),
                      rstd.data_ptr<float>(), scale.data_ptr<float>(), dx.data_ptr<float>(),
                      planes, s, static_cast<float>(slope), stream_of(x));
  return dx;
}

at::Tensor dropout(const at::Tensor& x_in, double p, int64_t seed, int64_t offset,
                   const c10::optional<at::Tensor>& rng) {
  auto x = x_in.contiguous();
  check_f32_gpu(x, "x");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout probability must be in [0, 1)");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty_like(x);
  launch_dropout(x.data_ptr<float>(), y.data_ptr<float>(), x.numel(), static_cast<float>(p),
                 static_cast<uint64_t>(seed), static_cast<uint64_t>(offset),
                 rng_state(rng, x.device()), stream_of(x));
  return y;
}

at::Tensor philox_uniform(int64_t n, int64_t seed, int64_t offset, at::Device device,
                          const c10::optional<at::Tensor>& rng) {
  TORCH_CHECK(device.is_cuda(), "philox_uniform runs on the GPU");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(device);
  auto out = at::empty({n}, at::TensorOptions().dtype(at::kFloat).device(device));
  launch_philox_uniform(out.data_ptr<float>(), n, static_cast<uint64_t>(seed),
                        static_cast<uint64_t>(offset), rng_state(rng, out.device()),
                        stream_of(out));
  return out;
}

void spin(int64_t ns, at::Device device) {
  TORCH_CHECK(device.is_cuda(), "spin runs on the GPU");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(device);
  launch_spin(static_cast<uint64_t>(ns),
              at::hip::getCurrentHIPStream(device.index()).stream());
}

void copy_segments(at::TensorList srcs, at::TensorList dsts) {
  TORCH_CHECK(srcs.size() == dsts.size(), "srcs and dsts must pair up");
  if (srcs.empty()) return;
  const auto device = srcs[0].device();
  TORCH_CHECK(device.is_cuda(), "copy_segments runs on the GPU");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(device);
  std::vector<Segment> segs;
  for (size_t i = 0; i < srcs.size(); ++i) {
    TORCH_CHECK(srcs[i].is_contiguous() && dsts[i].is_contiguous(), "segments must be contiguous");
    TORCH_CHECK(srcs[i].device() == device && dsts[i].device() == device,
                "segments must live on one device");
    const int64_t bytes = srcs[i].numel() * srcs[i].element_size();
    TORCH_CHECK(bytes == dsts[i].numel() * dsts[i].element_size(), "segment size mismatch");
    segs.push_back({srcs[i].data_ptr(), dsts[i].data_ptr(), bytes});
  }
  const hipStream_t stream = at::hip::getCurrentHIPStream(device.index()).stream();
  for (size_t i = 0; i < segs.size(); i += kMaxSegments) {
    const int count = static_cast<int>(std::min<size_t>(kMaxSegments, segs.size() - i));
    launch_segments_copy(segs.data() + i, count, stream);
  }
}

// `out` (optional): an existing transform of the same shape to overwrite in place (the
// per-step cache refresh, ops/conv.py) instead of a new tensor plus a copy.
at::Tensor transform_out(const c10::optional<at::Tensor>& out, at::IntArrayRef shape,
                         const at::Tensor& like) {
  if (!out.has_value() || !out->defined()) return at::empty(shape, like.options());
  check_f32_gpu(*out, "out");
  TORCH_CHECK(out->sizes() == shape && out->device() == like.device(),
              "out must be the transform's shape on the weight's device");
  return *out;
}

at::Tensor wino_weight(const at::Tensor& w, bool flip, const c10::optional<at::Tensor>& out) {
  check_f32_gpu(w, "weight");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "weight must be [K][C][3][3]");
  const int64_t out_channels = flip ? w.size(1) : w.size(0);
  const int64_t red_channels = flip ? w.size(0) : w.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  auto u = transform_out(
      out, {wino_pad_reduction(red_channels), wino_pad_output(out_channels), 16}, w);
  launch_wino_weight(w.data_ptr<float>(), u.data_ptr<float>(), out_channels, red_channels, flip,
                     stream_of(w));
  return u;
}

at::Tensor wino_conv(const at::Tensor& x_in, const at::Tensor& u,
                     const c10::optional<at::Tensor>& bias, int64_t out_channels,
                     int64_t variant, int64_t splits) {
  auto x = x_in.contiguous();
  check_f32_gpu(x, "x");
  check_f32_gpu(u, "u");
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  const int64_t n = x.size(0), r = x.size(1), h = x.size(2), w = x.size(3);
  TORCH_CHECK(u.dim() == 3 && u.size(2) == 16 && u.size(0) == wino_pad_reduction(r) &&
                  u.size(1) == wino_pad_output(out_channels),
              "transformed weight does not match the input/output channels");
  TORCH_CHECK(u.device() == x.device(), "u must live on the input's device");
  TORCH_CHECK(n * ((h + 1) / 2) * ((w + 1) / 2) < (int64_t{1} << 31) * 32,
              "too many output tiles for one launch");
  TORCH_CHECK(r * h * w < (int64_t{1} << 31) && out_channels < (1 << 24),
              "plane too large for 32-bit channel offsets");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_f32_gpu(*bias, "bias");
    TORCH_CHECK(bias->numel() == out_channels, "bias must have K elements");
    bptr = bias->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(variant >= -1 && variant <= 2, "variant must be -1 (auto), 0, 1 or 2");
  auto y = at::empty({n, out_channels, h, w}, x.options());
  if (y.numel() == 0) return y;
  const WinoPlan plan = wino_plan(n, r, h, w, out_channels, static_cast<int>(variant),
                                  static_cast<int>(splits));
  at::Tensor ws;
  if (plan.workspace > 0) ws = at::empty({plan.workspace}, x.options());
  launch_wino_conv(x.data_ptr<float>(), u.data_ptr<float>(), bptr, y.data_ptr<float>(),
                   plan.workspace > 0 ? ws.data_ptr<float>() : nullptr, n, r, h, w, out_channels,
                   plan, stream_of(x));
  return y;
}

at::Tensor wino4_weight(const at::Tensor& w, bool flip, const c10::optional<at::Tensor>& out) {
  check_f32_gpu(w, "weight");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "weight must be [K][C][3][3]");
  const int64_t out_channels = flip ? w.size(1) : w.size(0);
  const int64_t red_channels = flip ? w.size(0) : w.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  auto u = transform_out(
      out, {wino4_pad_reduction(red_channels), wino4_pad_output(out_channels), 36}, w);
  launch_wino4_weight(w.data_ptr<float>(), u.data_ptr<float>(), out_channels, red_channels, flip,
                      stream_of(w));
  return u;
}

at::Tensor wino4_conv(const at::Tensor& x_in, const at::Tensor& u,
                      const c10::optional<at::Tensor>& bias, int64_t out_channels,
                      int64_t variant, int64_t splits) {
  auto x = x_in.contiguous();
  check_f32_gpu(x, "x");
  check_f32_gpu(u, "u");
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  const int64_t n = x.size(0), r = x.size(1), h = x.size(2), w = x.size(3);
  // the kernel's 36-float weight rows, channel padding and index ranges
  TORCH_CHECK(u.dim() == 3 && u.size(2) == 36 && u.size(0) == wino4_pad_reduction(r) &&
                  u.size(1) == wino4_pad_output(out_channels),
              "F(4x4) transformed weight does not match the input/output channels");
  TORCH_CHECK(u.device() == x.device(), "u must live on the input's device");
  TORCH_CHECK(wino4_supported(n, r, h, w, out_channels),
              "input too large for the F(4x4) kernel (needs < 1 GiB); use wino_conv");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_f32_gpu(*bias, "bias");
    TORCH_CHECK(bias->numel() == out_channels, "bias must have K elements");
    bptr = bias->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({n, out_channels, h, w}, x.options());
  if (y.numel() == 0) return y;
  TORCH_CHECK(variant == -1 || (variant >= 4 && variant <= 15 && variant != 11 && variant != 13) ||
                  variant == 18,
              "variant must be -1, 4-10, 12, 14, 15 or 18");
  const WinoPlan plan = wino4_plan(n, r, h, w, out_channels, static_cast<int>(variant),
                                   static_cast<int>(splits));
  at::Tensor ws;
  if (plan.workspace > 0) ws = at::empty({plan.workspace}, x.options());
  launch_wino4_conv(x.data_ptr<float>(), u.data_ptr<float>(), bptr, y.data_ptr<float>(),
                    plan.workspace > 0 ? ws.data_ptr<float>() : nullptr, n, r, h, w,
                    out_channels, plan, stream_of(x));
  return y;
}

// Weight-gradient destination: a new tensor, or `into` (an existing .grad, contiguous
// fp32 [K][C][3][3]) that the kernels add into (gradient-accumulation fusion).
at::Tensor wgrad_destination(const c10::optional<at::Tensor>& into, const at::Tensor& x,
                             int64_t k, int64_t c) {
  if (!into.has_value()) return at::empty({k, c, 3, 3}, x.options());
  const at::Tensor& d = *into;
  TORCH_CHECK(d.is_contiguous() && d.scalar_type() == at::kFloat && d.device() == x.device() &&
                  d.dim() == 4 && d.size(0) == k && d.size(1) == c && d.size(2) == 3 &&
                  d.size(3) == 3,
              "into must be a contiguous fp32 [K][C][3][3] tensor on x's device");
  return d;
}

at::Tensor wino_wgrad(const at::Tensor& x_in, const at::Tensor& dy_in, int64_t splits,
                      int64_t variant, const c10::optional<at::Tensor>& into) {
  auto x = x_in.contiguous();
  auto dy = dy_in.contiguous();
  check_f32_gpu(x, "x");
  check_f32_gpu(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4, "x and dy must be NCHW");
  const int64_t n = x.size(0), c = x.size(1), h = x.size(2), w = x.size(3), k = dy.size(1);
  TORCH_CHECK(dy.size(0) == n && dy.size(2) == h && dy.size(3) == w,
              "dy must be [N][K][H][W] of a 3x3/s1/p1 convolution of x");
  TORCH_CHECK(dy.device() == x.device(), "x and dy must share a device");
  TORCH_CHECK(c * h * w < (int64_t{1} << 31) && k * h * w < (int64_t{1} << 31),
              "plane too large for 32-bit channel offsets");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const bool accum = into.has_value();
  auto dw = wgrad_destination(into, x, k, c);
  if (n == 0 || h == 0 || w == 0) return accum ? dw : dw.zero_();
  TORCH_CHECK(variant == -1 || variant == 0 || variant == 2, "variant must be -1, 0 or 2");
  // auto: the 64 x 64 double-buffered kernel, except for <= 32 output channels where
  // half of its 64-wide k block would idle (benchmarks/wgrad_variants.py).  Variant 2
  // decodes tile indices through a float reciprocal: exact below 2^24 tiles.
  const int64_t tiles = n * ((h + 1) / 2) * ((w + 1) / 2);
  int v = variant >= 0 ? static_cast<int>(variant) : (k <= 32 ? 0 : 2);
  if (v == 2 && tiles >= (int64_t{1} << 24)) v = 0;
  // every split must own >= 1 step of 8 tiles (both variants step 8 tiles)
  const int64_t steps = (tiles + 7) / 8;
  const int s = static_cast<int>(std::min<int64_t>(
      splits > 0 ? splits : wino_wgrad_splits(n, c, k, h, w, v), steps));
  at::Tensor ws;
  if (s > 1) ws = at::empty({s * k * c * 9}, x.options());
  launch_wino_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), dw.data_ptr<float>(),
                    s > 1 ? ws.data_ptr<float>() : nullptr, n, c, k, h, w, s, v, accum,
                    stream_of(x));
  return dw;
}

at::Tensor wino4_wgrad(const at::Tensor& x_in, const at::Tensor& dy_in, int64_t splits,
                       int64_t variant, const c10::optional<at::Tensor>& into) {
  auto x = x_in.contiguous();
  auto dy = dy_in.contiguous();
  check_f32_gpu(x, "x");
  check_f32_gpu(dy, "dy");
  TORCH_CHECK(x.dim() == 4 && dy.dim() == 4, "x and dy must be NCHW");
  const int64_t n = x.size(0), c = x.size(1), h = x.size(2), w = x.size(3), k = dy.size(1);
  TORCH_CHECK(dy.size(0) == n && dy.size(2) == h && dy.size(3) == w,
              "dy must be [N][K][H][W] of a 3x3/s1/p1 convolution of x");
  TORCH_CHECK(dy.device() == x.device(), "x and dy must share a device");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  const bool accum = into.has_value();
  auto dw = wgrad_destination(into, x, k, c);
  if (n == 0 || h == 0 || w == 0 || c == 0 || k == 0) return accum ? dw : dw.zero_();
  // 32-bit buffer offsets and tile indices
  TORCH_CHECK(wino4_wgrad_supported(n, c, k, h, w),
              "input too large for the F(4x4) weight-gradient kernel (needs < 1 GiB); "
              "use wino_wgrad");
  TORCH_CHECK(variant >= 0 && variant <= 2,
              "variant must be 0 (fused), 1 (non-fused) or 2 (split-bf16 batched GEMM)");
  // every split owns >= 1 step (of 4 tiles; of 16 for the split-bf16 GEMM)
  const int64_t tiles = n * ((h + 3) / 4) * ((w + 3) / 4);
  const int64_t steps = variant == 2 ? (tiles + 15) / 16 : (tiles + 3) / 4;
  const int s = static_cast<int>(std::min<int64_t>(
      splits > 0 ? splits
                 : (variant == 2 ? wino4_wgrad_emu_splits(n, c, k, h, w)
                                 : wino4_wgrad_splits(n, c, k, h, w)),
      steps));
  const int64_t wsize = wino4_wgrad_workspace(n, c, k, h, w, s, static_cast<int>(variant));
  at::Tensor ws;
  if (wsize > 0) ws = at::empty({wsize}, x.options());
  launch_wino4_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), dw.data_ptr<float>(),
                     wsize > 0 ? ws.data_ptr<float>() : nullptr, n, c, k, h, w, s,
                     static_cast<int>(variant), accum, stream_of(x));
  return dw;
}

// Batched-GEMM Winograd F(4x4): weights in the GEMM operand layout (cached per step by
// ops/conv.py), and the convolution (input transform, 36 GEMMs, output transform).
at::Tensor bg_weight(const at::Tensor& w, bool flip, int64_t kind,
                     const c10::optional<at::Tensor>& out, int64_t emu) {
  check_f32_gpu(w, "weight");
  TORCH_CHECK(w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "weight must be [K][C][3][3]");
  auto wc = w.contiguous();
  const int64_t out_channels = flip ? w.size(1) : w.size(0);
  const int64_t red_channels = flip ? w.size(0) : w.size(1);
  c10::hip::HIPGuardMasqueradingAsCUDA guard(w.device());
  TORCH_CHECK(kind == 4 || kind == 2, "kind must be 4 (F(4x4)) or 2 (F(2x2))");
  auto a =
      transform_out(out, {bg_weight_numel(out_channels, red_channels, static_cast<int>(kind),
                                          static_cast<int>(emu))}, w);
  launch_bg_weight(wc.data_ptr<float>(), a.data_ptr<float>(), out_channels, red_channels, flip,
                   static_cast<int>(kind), stream_of(w), static_cast<int>(emu));
  return a;
}

at::Tensor bg_conv(const at::Tensor& x_in, const at::Tensor& a,
                   const c10::optional<at::Tensor>& bias, int64_t out_channels, int64_t bn,
                   int64_t splits, int64_t kind, int64_t waves, int64_t sub, int64_t emu,
                   const c10::optional<at::Tensor>& stats) {
  auto x = x_in.contiguous();
  check_f32_gpu(x, "x");
  check_f32_gpu(a, "a");
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  const int64_t n = x.size(0), r = x.size(1), h = x.size(2), w = x.size(3);
  TORCH_CHECK(kind == 4 || kind == 2, "kind must be 4 (F(4x4)) or 2 (F(2x2))");
  TORCH_CHECK(a.dim() == 1 && a.numel() == bg_weight_numel(out_channels, r, static_cast<int>(kind),
                                                           static_cast<int>(emu)),
              "batched-GEMM transformed weight does not match the input/output channels");
  TORCH_CHECK(a.device() == x.device(), "a must live on the input's device");
  TORCH_CHECK(wino4_supported(n, r, h, w, out_channels),
              "input too large for the F(4x4) kernels (needs < 1 GiB)");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_f32_gpu(*bias, "bias");
    TORCH_CHECK(bias->numel() == out_channels, "bias must have K elements");
    bptr = bias->data_ptr<float>();
  }
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({n, out_channels, h, w}, x.options());
  if (n == 0 || h == 0 || w == 0 || out_channels == 0) return y;
  const BgPlan plan = bg_plan(n, r, h, w, out_channels, static_cast<int>(bn),
                              static_cast<int>(splits), static_cast<int>(kind),
                              static_cast<int>(waves), static_cast<int>(sub),
                              static_cast<int>(emu));
  // 32-bit tile / element indices of the GEMM and transform kernels
  TORCH_CHECK(plan.ksteps * 16 * plan.np < (int64_t{1} << 31) &&
                  plan.mp * plan.np < (int64_t{1} << 31),
              "operands too large for the batched-GEMM kernels");
  // stats: the BatchNorm (mean, M2) partials of y, [2][groups][out_channels] with groups =
  // ceil(n / bg_stats_ipg(n, h, w, kind)) -- the caller's bn_train_forward reads them
  float* pm = nullptr;
  int ipg = 0;
  if (stats.has_value() && stats->defined()) {
    check_f32_gpu(*stats, "stats");
    ipg = bg_stats_ipg(n, h, w, static_cast<int>(kind));
    const int64_t groups = (n + ipg - 1) / ipg;
    TORCH_CHECK(stats->device() == x.device() && stats->is_contiguous() &&
                    stats->numel() == 2 * groups * out_channels,
                "stats must be a contiguous [2][ceil(n / bg_stats_ipg)][K] float32 tensor");
    pm = stats->data_ptr<float>();
  }
  auto ws = at::empty({plan.workspace}, x.options());
  launch_bg_conv(x.data_ptr<float>(), a.data_ptr<float>(), bptr, y.data_ptr<float>(),
                 ws.data_ptr<float>(), n, r, h, w, out_channels, plan, stream_of(x), pm,
                 pm == nullptr ? nullptr : pm + stats->numel() / 2, ipg);
  return y;
}

int64_t bg_stats_images(int64_t n, int64_t h, int64_t w, int64_t kind) {
  return bg_stats_ipg(n, h, w, static_cast<int>(kind));
}

// Split-K count of the F(4x4) kernels for one convolution: variant 0 = the weight gradient,
// otherwise that forward / backward-data variant (wino4_plan).
int64_t wino4_splits(int64_t n, int64_t c, int64_t k, int64_t h, int64_t w, int64_t variant) {
  if (variant == 0) {
    const int64_t steps = (n * ((h + 3) / 4) * ((w + 3) / 4) + 3) / 4;
    return std::min<int64_t>(wino4_wgrad_splits(n, c, k, h, w), steps);
  }
  return wino4_plan(n, c, h, w, k, static_cast<int>(variant), 0).splits;
}

}  // namespace
}  // namespace tgpipe

TORCH_LIBRARY(tgpipe, m) {
  m.def("dna_forward(Tensor x, float p, float eps, float slope, int seed, int offset, "
        "bool dropout, Tensor? rng=None) -> Tensor[]");
  m.def("dna_backward(Tensor dy, Tensor x, Tensor mean, Tensor rstd, Tensor scale, "
        "float slope) -> Tensor");
  m.def("dropout(Tensor x, float p, int seed, int offset, Tensor? rng=None) -> Tensor");
  m.def("philox_uniform(int n, int seed, int offset, Device device, Tensor? rng=None) -> Tensor");
  m.def("spin(int ns, Device device) -> ()");
  m.def("copy_segments(Tensor[] srcs, Tensor(a!)[] dsts) -> ()");
  m.def("wino_weight(Tensor w, bool flip, Tensor? out=None) -> Tensor");
  m.def("wino_wgrad(Tensor x, Tensor dy, int splits=0, int variant=-1, Tensor? into=None) -> Tensor");
  m.def("wino_conv(Tensor x, Tensor u, Tensor? bias, int out_channels, int variant=-1, "
        "int splits=0) -> Tensor");
  m.def("wino4_weight(Tensor w, bool flip, Tensor? out=None) -> Tensor");
  m.def("wino4_wgrad(Tensor x, Tensor dy, int splits=0, int variant=0, Tensor? into=None) -> Tensor");
  m.def("wino4_conv(Tensor x, Tensor u, Tensor? bias, int out_channels, int variant=-1, "
        "int splits=0) -> Tensor");
  m.def("bg_weight(Tensor w, bool flip, int kind=4, Tensor? out=None, int emu=-1) -> Tensor");
  // split-K counts the F(4x4) host heuristics pick (host only, CPU-testable)
  m.def("wino4_splits(int n, int c, int k, int h, int w, int variant) -> int",
        &tgpipe::wino4_splits);
  m.def("bg_conv(Tensor x, Tensor a, Tensor? bias, int out_channels, int bn=0, int splits=0, "
        "int kind=4, int waves=0, int sub=0, int emu=-1, Tensor(b!)? stats=None) -> Tensor");
  // images per BatchNorm-statistics group of bg_conv's `stats` (host only)
  m.def("bg_stats_images(int n, int h, int w, int kind) -> int", &tgpipe::bg_stats_images);
}

TORCH_LIBRARY_IMPL(tgpipe, CUDA, m) {
  m.impl("dna_forward", &tgpipe::dna_forward);
  m.impl("dna_backward", &tgpipe::dna_backward);
  m.impl("dropout", &tgpipe::dropout);
  m.impl("copy_segments", &tgpipe::copy_segments);
  m.impl("wino_weight", &tgpipe::wino_weight);
  m.impl("wino_conv", &tgpipe::wino_conv);
  m.impl("wino_wgrad", &tgpipe::wino_wgrad);
  m.impl("wino4_weight", &tgpipe::wino4_weight);
  m.impl("wino4_conv", &tgpipe::wino4_conv);
  m.impl("wino4_wgrad", &tgpipe::wino4_wgrad);
  m.impl("bg_weight", &tgpipe::bg_weight);
  m.impl("bg_conv", &tgpipe::bg_conv);
}

TORCH_LIBRARY_IMPL(tgpipe, CompositeExplicitAutograd, m) {
  m.impl("philox_uniform", &tgpipe::philox_uniform);
  m.impl("spin", &tgpipe::spin);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "torchgpipe_amd native HIP kernels (gfx950)";
}
