// torch bindings of the NHWC batch-norm kernels (batchnorm.hip); shapes, dtypes and
// alignment are checked against what the kernels index before every launch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "batchnorm.h"

namespace py = pybind11;
using at::Tensor;
namespace B_ = katib_hip::bn;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }
B_::bf16* bp(const Tensor& t) { return reinterpret_cast<B_::bf16*>(t.data_ptr()); }
const B_::bf16* obp(const c10::optional<Tensor>& t) { return t.has_value() ? bp(*t) : nullptr; }

void chk_act(const Tensor& t, int64_t P, int64_t C, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous() && t.numel() == P * C, name,
              " must be a contiguous bf16 [P, C] GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
void chk_vec(const Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, name,
              " must be a contiguous fp32 GPU tensor of ", n, " elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
void dims(const Tensor& x, int64_t& P, int64_t& C) {
  TORCH_CHECK(x.dim() == 2, "activations must be viewed as [P, C]");
  P = x.size(0);
  C = x.size(1);
  TORCH_CHECK(P > 0 && C > 0 && C % 8 == 0 && P * C < (1ll << 31), "bn: C % 8 == 0, P * C < 2^31");
}
void ok(hipError_t e, const char* w) { TORCH_CHECK(e == hipSuccess, w, ": ", hipGetErrorString(e)); }

void bn_fwd_train(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& y, const Tensor& gamma,
                  const Tensor& beta, const c10::optional<Tensor>& rmean, const c10::optional<Tensor>& rvar,
                  const Tensor& mean, const Tensor& invstd, double eps, double momentum, bool relu,
                  const c10::optional<Tensor>& num_batches) {
  int64_t P, C;
  dims(x, P, C);
  chk_act(x, P, C, "x");
  chk_act(y, P, C, "y");
  if (res.has_value()) chk_act(*res, P, C, "res");
  chk_vec(gamma, C, "gamma");
  chk_vec(beta, C, "beta");
  chk_vec(mean, C, "mean");
  chk_vec(invstd, C, "invstd");
  TORCH_CHECK(rmean.has_value() == rvar.has_value(), "running mean and var go together");
  if (rmean.has_value()) {
    chk_vec(*rmean, C, "running_mean");
    chk_vec(*rvar, C, "running_var");
  }
  int R, rows, cvb;
  B_::plan((int)P, (int)C, &R, &rows, &cvb);
  auto part = at::empty({(int64_t)R * 2 * C}, x.options().dtype(at::kFloat));
  auto ss = at::empty({2 * C}, x.options().dtype(at::kFloat));
  ok(B_::fwd_train(bp(x), obp(res), bp(y), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                   rmean.has_value() ? rmean->data_ptr<float>() : nullptr,
                   rvar.has_value() ? rvar->data_ptr<float>() : nullptr, mean.data_ptr<float>(),
                   invstd.data_ptr<float>(), ss.data_ptr<float>(), part.data_ptr<float>(), (int)P, (int)C, (float)eps,
                   (float)momentum, relu ? 1 : 0, stream(),
                   num_batches.has_value() ? reinterpret_cast<long long*>(num_batches->data_ptr<int64_t>()) : nullptr),
     "bn_fwd_train");
}

void bn_fwd_eval(const Tensor& x, const c10::optional<Tensor>& res, const Tensor& y, const Tensor& gamma,
                 const Tensor& beta, const Tensor& rmean, const Tensor& rvar, double eps, bool relu) {
  int64_t P, C;
  dims(x, P, C);
  chk_act(x, P, C, "x");
  chk_act(y, P, C, "y");
  if (res.has_value()) chk_act(*res, P, C, "res");
  chk_vec(gamma, C, "gamma");
  chk_vec(beta, C, "beta");
  chk_vec(rmean, C, "running_mean");
  chk_vec(rvar, C, "running_var");
  auto ss = at::empty({2 * C}, x.options().dtype(at::kFloat));
  ok(B_::fwd_eval(bp(x), obp(res), bp(y), gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(),
                  rvar.data_ptr<float>(), ss.data_ptr<float>(), (int)P, (int)C, (float)eps, relu ? 1 : 0, stream()),
     "bn_fwd_eval");
}

void bn_bwd(const Tensor& dy, const c10::optional<Tensor>& y, const Tensor& x, const Tensor& gamma,
            const Tensor& mean, const Tensor& invstd, const Tensor& dx, const c10::optional<Tensor>& dres,
            const Tensor& dgamma, const Tensor& dbeta, bool accumulate) {
  int64_t P, C;
  dims(x, P, C);
  chk_act(dy, P, C, "dy");
  chk_act(x, P, C, "x");
  chk_act(dx, P, C, "dx");
  if (y.has_value()) chk_act(*y, P, C, "y");
  if (dres.has_value()) chk_act(*dres, P, C, "dres");
  chk_vec(gamma, C, "gamma");
  chk_vec(mean, C, "mean");
  chk_vec(invstd, C, "invstd");
  chk_vec(dgamma, C, "dgamma");
  chk_vec(dbeta, C, "dbeta");
  int R, rows, cvb;
  B_::plan((int)P, (int)C, &R, &rows, &cvb);
  auto part = at::empty({(int64_t)R * 2 * C}, x.options().dtype(at::kFloat));
  auto coef = at::empty({3 * C}, x.options().dtype(at::kFloat));
  ok(B_::bwd(bp(dy), obp(y), bp(x), gamma.data_ptr<float>(), mean.data_ptr<float>(), invstd.data_ptr<float>(), bp(dx),
             dres.has_value() ? bp(*dres) : nullptr, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
             coef.data_ptr<float>(), part.data_ptr<float>(), (int)P, (int)C, stream(), accumulate ? 1 : 0),
     "bn_bwd");
}

void channel_sum(const Tensor& x, const Tensor& out) {
  int64_t P, C;
  dims(x, P, C);
  chk_act(x, P, C, "x");
  chk_vec(out, C, "out");
  int R, rows, cvb;
  B_::plan((int)P, (int)C, &R, &rows, &cvb);
  auto part = at::empty({(int64_t)R * 2 * C}, x.options().dtype(at::kFloat));
  ok(B_::channel_sum(bp(x), out.data_ptr<float>(), part.data_ptr<float>(), (int)P, (int)C, stream()), "channel_sum");
}

}  // namespace

void register_batchnorm(py::module& m) {
  m.def("channel_sum", &channel_sum, "per-channel sum of a [P, C] bf16 activation (bias gradients), graph-safe");
  m.def("bn_fwd_train", &bn_fwd_train, "NHWC bf16 batch norm (+residual, +ReLU), training statistics",
        py::arg("x"), py::arg("res"), py::arg("y"), py::arg("gamma"), py::arg("beta"), py::arg("rmean"),
        py::arg("rvar"), py::arg("mean"), py::arg("invstd"), py::arg("eps"), py::arg("momentum"), py::arg("relu"),
        py::arg("num_batches") = py::none());
  m.def("bn_fwd_eval", &bn_fwd_eval, "NHWC bf16 batch norm (+residual, +ReLU) with running statistics");
  m.def("bn_bwd", &bn_bwd, "NHWC bf16 batch norm backward (ReLU mask from the output, residual gradient)",
        py::arg("dy"), py::arg("y"), py::arg("x"), py::arg("gamma"), py::arg("mean"), py::arg("invstd"), py::arg("dx"),
        py::arg("dres"), py::arg("dgamma"), py::arg("dbeta"), py::arg("accumulate") = false);
}
