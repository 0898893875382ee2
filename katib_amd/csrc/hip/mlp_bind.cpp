// torch bindings of the fused MLP kernels (mlp.hip), with the shape / dtype / alignment /
// index-range checks the kernels and their grids rely on.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "mlp.h"

namespace py = pybind11;
using at::Tensor;
namespace M_ = katib_hip::mlp;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
M_::bf16* bp(const Tensor& t) { return reinterpret_cast<M_::bf16*>(t.data_ptr()); }
void ok(hipError_t e, const char* w) { TORCH_CHECK(e == hipSuccess, w, ": ", hipGetErrorString(e)); }

void chk(const Tensor& t, at::ScalarType dt, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous() && t.numel() == n, name,
              " must be a contiguous ", c10::toString(dt), " GPU tensor of ", n, " elements (got ", t.numel(), ")");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
// the gather index must address rows of x: the kernels trust it
void chk_idx(const c10::optional<Tensor>& idx, int64_t M) {
  if (!idx.has_value()) return;
  TORCH_CHECK(idx->is_cuda() && idx->scalar_type() == at::kLong && idx->is_contiguous() && idx->numel() == M,
              "idx must be a contiguous int64 GPU tensor with one entry per row");
}

void lin_fwd(const Tensor& x, const c10::optional<Tensor>& idx, const Tensor& w, const c10::optional<Tensor>& bias,
             const c10::optional<Tensor>& mask, const Tensor& y, bool relu) {
  TORCH_CHECK(w.dim() == 2 && y.dim() == 2 && x.dim() == 2, "lin_fwd: 2-D operands");
  const int64_t N = w.size(0), K = w.size(1), M = y.size(0);
  TORCH_CHECK(K % 8 == 0 && K == x.size(1) && y.size(1) == N, "lin_fwd: K % 8 == 0 and matching shapes");
  TORCH_CHECK(idx.has_value() || x.size(0) == M, "lin_fwd: x rows must match y rows without a gather");
  chk(x, at::kBFloat16, x.numel(), "x");
  chk(w, at::kBFloat16, N * K, "w");
  chk(y, at::kBFloat16, M * N, "y");
  chk_idx(idx, M);
  if (bias.has_value()) chk(*bias, at::kFloat, N, "bias");
  if (mask.has_value()) chk(*mask, at::kBFloat16, M * N, "mask");
  ok(M_::lin_fwd(bp(x), idx.has_value() ? idx->data_ptr<int64_t>() : nullptr, bp(w),
                 bias.has_value() ? bias->data_ptr<float>() : nullptr, mask.has_value() ? bp(*mask) : nullptr, bp(y),
                 (int)M, (int)N, (int)K, relu ? 1 : 0, stream()),
     "lin_fwd");
}

void lin_wgrad_sgd(const Tensor& dy, const Tensor& x, const c10::optional<Tensor>& idx, const Tensor& w,
                   const Tensor& wm, const Tensor& w16, const Tensor& w16t, const c10::optional<Tensor>& bias,
                   const c10::optional<Tensor>& bm, const Tensor& lr, double momentum) {
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && w.dim() == 2, "lin_wgrad_sgd: 2-D operands");
  const int64_t M = dy.size(0), N = dy.size(1), K = w.size(1);
  TORCH_CHECK(w.size(0) == N && x.size(1) == K && N % 8 == 0 && K % 8 == 0, "lin_wgrad_sgd: N, K % 8 == 0");
  TORCH_CHECK(idx.has_value() || x.size(0) == M, "lin_wgrad_sgd: x rows must match dy rows without a gather");
  chk(dy, at::kBFloat16, M * N, "dy");
  chk(x, at::kBFloat16, x.numel(), "x");
  chk_idx(idx, M);
  chk(w, at::kFloat, N * K, "w");
  chk(wm, at::kFloat, N * K, "wm");
  chk(w16, at::kBFloat16, N * K, "w16");
  chk(w16t, at::kBFloat16, N * K, "w16t");
  TORCH_CHECK(bias.has_value() == bm.has_value(), "bias and its momentum buffer go together");
  if (bias.has_value()) {
    chk(*bias, at::kFloat, N, "bias");
    chk(*bm, at::kFloat, N, "bias momentum");
  }
  TORCH_CHECK(lr.is_cuda() && lr.scalar_type() == at::kFloat && lr.numel() == 1, "lr must be a GPU fp32 scalar");
  ok(M_::lin_wgrad_sgd(bp(dy), bp(x), idx.has_value() ? idx->data_ptr<int64_t>() : nullptr, (int)M, (int)N, (int)K,
                       w.data_ptr<float>(), wm.data_ptr<float>(), bp(w16), bp(w16t),
                       bias.has_value() ? bias->data_ptr<float>() : nullptr,
                       bm.has_value() ? bm->data_ptr<float>() : nullptr, lr.data_ptr<float>(), (float)momentum,
                       stream()),
     "lin_wgrad_sgd");
}

void xent_small(const Tensor& logits, const Tensor& y, const c10::optional<Tensor>& idx, const Tensor& dl,
                int64_t C, const Tensor& stats) {
  TORCH_CHECK(logits.dim() == 2, "logits must be [M, ld]");
  const int64_t M = logits.size(0), ld = logits.size(1);
  TORCH_CHECK(C > 0 && C <= ld && ld <= 64, "xent_small: 0 < C <= ld <= 64");
  chk(logits, at::kBFloat16, M * ld, "logits");
  chk(dl, at::kBFloat16, M * ld, "dl");
  TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kLong && y.is_contiguous(), "labels must be int64 on the GPU");
  chk_idx(idx, M);
  TORCH_CHECK(idx.has_value() || y.numel() == M, "labels must have one entry per row without a gather");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kFloat && stats.numel() == 2, "stats: fp32[2]");
  ok(M_::xent_small(bp(logits), y.data_ptr<int64_t>(), idx.has_value() ? idx->data_ptr<int64_t>() : nullptr, bp(dl),
                    (int)M, (int)C, (int)ld, stats.data_ptr<float>(), stream()),
     "xent_small");
}

}  // namespace

void register_mlp(py::module& m) {
  m.def("lin_fwd", &lin_fwd, "fused linear (+bias, +ReLU or ReLU-derivative mask), optional row gather");
  m.def("lin_wgrad_sgd", &lin_wgrad_sgd, "weight/bias gradient with fused SGD-momentum update");
  m.def("xent_small", &xent_small, "softmax cross-entropy + gradient for a few classes");
}
