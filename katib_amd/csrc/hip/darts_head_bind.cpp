// torch bindings of the fused DARTS head kernels (darts_head.hip), with the shape / dtype /
// device checks their one-workgroup-per-sample grids rely on.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <optional>

#include "darts_head.h"
#include "darts_ops.h"

namespace py = pybind11;
using at::Tensor;
namespace H_ = katib_hip::head;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

float* f32(const Tensor& t, const char* name, std::initializer_list<int64_t> shape, const Tensor& ref) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name,
              " must be a contiguous float32 GPU tensor");
  TORCH_CHECK(t.device() == ref.device(), name, " must be on the device of x");
  TORCH_CHECK(t.sizes().equals(shape), name, " has shape ", t.sizes(), ", expected ", at::IntArrayRef(shape));
  return t.data_ptr<float>();
}

struct Dims {
  int N, C, HW, K, nodes;
};

// x: [N][C][H][W], or node-major [nodes][N][C / nodes][H][W] (a DARTS cell output kept as its nodes)
Dims dims_of(const Tensor& x, const Tensor& w) {
  TORCH_CHECK(x.dim() == 4 || x.dim() == 5, "head: x must be [N][C][H][W] or node-major [nodes][N][C/nodes][H][W]");
  const bool nm = x.dim() == 5;
  Dims d{static_cast<int>(nm ? x.size(1) : x.size(0)), static_cast<int>(nm ? x.size(0) * x.size(2) : x.size(1)),
         static_cast<int>(nm ? x.size(3) * x.size(4) : x.size(2) * x.size(3)), static_cast<int>(w.size(0)),
         static_cast<int>(nm ? x.size(0) : 1)};
  TORCH_CHECK(w.dim() == 2 && w.size(1) == d.C, "head: w must be [K][C]");
  TORCH_CHECK(d.N >= 1 && d.C >= 1 && d.HW >= 1 && d.K >= 1, "head: empty operand");
  TORCH_CHECK(d.C <= H_::kMaxC && d.K <= H_::kMaxK, "head: C must be <= ", H_::kMaxC, " and K <= ", H_::kMaxK);
  TORCH_CHECK(x.numel() < (int64_t(1) << 31), "head: x too large");
  return d;
}

void fwd(const Tensor& x, const Tensor& w, const Tensor& b, const Tensor& y, const Tensor& pooled,
         const Tensor& logits, const Tensor& dl, const Tensor& loss_n) {
  const Dims d = dims_of(x, w);
  H_::FwdArgs a;
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kFloat && x.is_contiguous(), "head: x must be contiguous fp32");
  a.x = x.data_ptr<float>();
  a.nodes = d.nodes;
  a.w = f32(w, "w", {d.K, d.C}, x);
  a.b = f32(b, "b", {d.K}, x);
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kLong && y.is_contiguous() && y.dim() == 1 && y.size(0) == d.N &&
                  y.device() == x.device(),
              "head: y must be a contiguous int64 [N] GPU tensor");
  a.y = y.data_ptr<int64_t>();
  a.pooled = f32(pooled, "pooled", {d.N, d.C}, x);
  a.logits = f32(logits, "logits", {d.N, d.K}, x);
  a.dl = f32(dl, "dl", {d.N, d.K}, x);
  a.loss_n = f32(loss_n, "loss_n", {d.N}, x);
  a.N = d.N;
  a.C = d.C;
  a.HW = d.HW;
  a.K = d.K;
  H_::launch_fwd(a, stream());
}

void loss(const Tensor& loss_n, const Tensor& out) {
  TORCH_CHECK(loss_n.dim() == 1 && loss_n.size(0) >= 1, "head: loss_n must be [N]");
  H_::launch_loss(f32(loss_n, "loss_n", {loss_n.size(0)}, loss_n), static_cast<int>(loss_n.size(0)),
                  f32(out, "loss", {}, loss_n), stream());
}

void bwd(const Tensor& x_like, const Tensor& dl, const Tensor& pooled, const Tensor& w, const Tensor& gout,
         std::optional<Tensor> dx, std::optional<Tensor> gw, int64_t gw_stride, std::optional<Tensor> gb,
         int64_t gb_stride) {
  const Dims d = dims_of(x_like, w);
  H_::BwdArgs a;
  a.dl = f32(dl, "dl", {d.N, d.K}, x_like);
  a.pooled = f32(pooled, "pooled", {d.N, d.C}, x_like);
  a.w = f32(w, "w", {d.K, d.C}, x_like);
  TORCH_CHECK(gout.numel() == 1, "head: upstream gradient must be a scalar");
  a.gout = f32(gout, "gout", {}, x_like);
  if (dx) {
    TORCH_CHECK(dx->is_cuda() && dx->scalar_type() == at::kFloat && dx->is_contiguous() &&
                    dx->sizes() == x_like.sizes() && dx->device() == x_like.device(),
                "head: dx must be a contiguous fp32 tensor shaped like x");
  }
  a.dx = dx ? dx->data_ptr<float>() : nullptr;
  a.nodes = d.nodes;
  // replicated gradient rows: replica r at + r * stride, kRep rows must fit the buffer the view lives in
  auto rep_ptr = [&](const std::optional<Tensor>& g, int64_t stride, int64_t numel, const char* name) -> float* {
    if (!g) return nullptr;
    const Tensor& t = *g;
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == numel &&
                    t.device() == x_like.device(),
                name, ": contiguous float32 GPU tensor of ", numel, " elements expected");
    TORCH_CHECK(stride >= numel, name, ": replica stride smaller than the gradient");
    const auto& st = t.storage();
    const int64_t need = (t.storage_offset() + (int64_t)(katib_hip::kRep - 1) * stride + numel) * 4;
    TORCH_CHECK(need <= (int64_t)st.nbytes(), name, ": ", katib_hip::kRep, " replica rows do not fit its storage");
    return t.data_ptr<float>();
  };
  a.gw = rep_ptr(gw, gw_stride, (int64_t)d.K * d.C, "gw");
  a.gw_stride = static_cast<int>(gw_stride);
  a.gb = rep_ptr(gb, gb_stride, d.K, "gb");
  a.gb_stride = static_cast<int>(gb_stride);
  a.N = d.N;
  a.C = d.C;
  a.HW = d.HW;
  a.K = d.K;
  H_::launch_bwd(a, stream());
}

}  // namespace

void register_darts_head(py::module& m) {
  m.def("head_fwd", &fwd, "fused gap + classifier + cross-entropy forward (per-sample losses, dlogits)");
  m.def("head_loss", &loss, "mean of the per-sample losses (fixed order)");
  m.def("head_bwd", &bwd, "fused head backward: pooled-feature gradient + replicated weight / bias gradients",
        py::arg("x_like"), py::arg("dl"), py::arg("pooled"), py::arg("w"), py::arg("gout"), py::arg("dx"),
        py::arg("gw"), py::arg("gw_stride"), py::arg("gb"), py::arg("gb_stride"));
}
