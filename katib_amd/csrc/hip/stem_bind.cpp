// torch bindings of the DARTS stem convolution kernels (stem_conv.hip), with the shape /
// dtype / contiguity checks their grids and LDS slab rely on.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <optional>

#include "darts_ops.h"
#include "stem_conv.h"

namespace py = pybind11;
using at::Tensor;
namespace S_ = katib_hip::stem;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name,
              " must be a contiguous float32 GPU tensor");
}

// x [N][Cin][H][W], w [Cout][Cin][3][3]; Cin in {1, 3}, Cout <= kMaxCout
void check_shapes(const Tensor& x, const Tensor& w) {
  chk(x, "x");
  chk(w, "w");
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3, "stem: 4-D x and 3x3 w");
  TORCH_CHECK(w.size(1) == x.size(1) && (x.size(1) == 1 || x.size(1) == 3), "stem: Cin must be 1 or 3 and match w");
  TORCH_CHECK(w.size(0) >= 1 && w.size(0) <= S_::kMaxCout, "stem: Cout must be in [1, ", S_::kMaxCout, "]");
  TORCH_CHECK(x.numel() < (int64_t(1) << 31) / 64, "stem: input too large for 32-bit pixel indexing");
  TORCH_CHECK(x.device() == w.device(), "stem: operands on one device");
}

void fwd(const Tensor& x, const Tensor& w, const Tensor& y) {
  check_shapes(x, w);
  chk(y, "y");
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Cout = w.size(0);
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == Cout && y.size(2) == H && y.size(3) == W,
              "stem: y must be [N][Cout][H][W]");
  S_::launch_fwd(x.data_ptr<float>(), w.data_ptr<float>(), y.data_ptr<float>(), N, Cin, Cout, H, W, stream());
}

void wgrad(const Tensor& x, const Tensor& dy, const Tensor& partial, const Tensor& dw) {
  check_shapes(x, dw);
  chk(dy, "dy");
  chk(partial, "partial");
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Cout = dw.size(0);
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == Cout && dy.size(2) == H && dy.size(3) == W,
              "stem: dy must be [N][Cout][H][W]");
  TORCH_CHECK(partial.dim() == 2 && partial.size(1) == Cout * Cin * 9, "stem: partial must be [chunks][Cout*Cin*9]");
  const int chunks = partial.size(0);
  TORCH_CHECK(chunks >= 1 && chunks <= 65535 && chunks <= (int64_t)N * H * W, "stem: bad chunk count");
  S_::launch_wgrad(x.data_ptr<float>(), dy.data_ptr<float>(), partial.data_ptr<float>(), dw.data_ptr<float>(), N, Cin,
                   Cout, H, W, chunks, stream());
}

void chk64(const Tensor& t, const char* name, int64_t min_numel) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kDouble && t.is_contiguous() && t.numel() >= min_numel, name,
              " must be a contiguous float64 GPU tensor with >= ", min_numel, " elements");
}

// y = conv(x, w) and BN statistics into stats[kRep][2*Cout] (must be zeroed by the caller)
void fwd_stats(const Tensor& x, const Tensor& w, const Tensor& y, const Tensor& stats) {
  check_shapes(x, w);
  chk(y, "y");
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Cout = w.size(0);
  TORCH_CHECK(y.dim() == 4 && y.size(0) == N && y.size(1) == Cout && y.size(2) == H && y.size(3) == W,
              "stem: y must be [N][Cout][H][W]");
  chk64(stats, "stats", (int64_t)katib_hip::kRep * 2 * Cout);
  TORCH_CHECK(stats.device() == x.device(), "stem: stats on the device of x");
  S_::launch_fwd_stats(x.data_ptr<float>(), w.data_ptr<float>(), y.data_ptr<float>(), stats.data_ptr<double>(), N,
                       Cin, Cout, H, W, stream());
}

// weight gradient through the affine BN backward (dy = gradient of the BN output)
void wgrad_bn(const Tensor& x, const Tensor& dy, const Tensor& z, const Tensor& red, const Tensor& stats,
              const Tensor& gamma, double eps, std::optional<Tensor> dgamma, std::optional<Tensor> dbeta,
              const Tensor& partial, const Tensor& dw, int64_t world, bool accumulate) {
  check_shapes(x, dw);
  TORCH_CHECK(world >= 1, "stem: world must be >= 1");
  chk(dy, "dy");
  chk(z, "z");
  chk(partial, "partial");
  chk(gamma, "gamma");
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Cout = dw.size(0);
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == Cout && dy.size(2) == H && dy.size(3) == W,
              "stem: dy must be [N][Cout][H][W]");
  TORCH_CHECK(z.sizes() == dy.sizes(), "stem: z must match dy");
  TORCH_CHECK(gamma.numel() == Cout, "stem: gamma must have Cout elements");
  chk64(red, "red", 2 * Cout);
  chk64(stats, "stats", 2 * Cout);
  TORCH_CHECK(partial.dim() == 2 && partial.size(1) == Cout * Cin * 9, "stem: partial must be [chunks][Cout*Cin*9]");
  const int chunks = partial.size(0);
  TORCH_CHECK(chunks >= 1 && chunks <= 65535 && chunks <= (int64_t)N * H * W, "stem: bad chunk count");
  S_::BnBwd bn{};
  bn.z = z.data_ptr<float>();
  bn.red = red.data_ptr<double>();
  bn.stats = stats.data_ptr<double>();
  bn.gamma = gamma.data_ptr<float>();
  // SyncBN (world > 1): stats / red are sums over every rank's batch
  bn.inv_count = static_cast<float>(1.0 / ((double)N * H * W * world));
  bn.red_scale = static_cast<float>(1.0 / world);
  bn.eps = static_cast<float>(eps);
  if (dgamma) {
    chk(*dgamma, "dgamma");
    TORCH_CHECK(dgamma->numel() == Cout, "stem: dgamma must have Cout elements");
    bn.dgamma = dgamma->data_ptr<float>();
  }
  if (dbeta) {
    chk(*dbeta, "dbeta");
    TORCH_CHECK(dbeta->numel() == Cout, "stem: dbeta must have Cout elements");
    bn.dbeta = dbeta->data_ptr<float>();
  }
  for (const Tensor* t : {&dy, &z, &red, &stats, &gamma, &partial})
    TORCH_CHECK(t->device() == x.device(), "stem: operands on one device");
  S_::launch_wgrad_bn(x.data_ptr<float>(), dy.data_ptr<float>(), bn, partial.data_ptr<float>(), dw.data_ptr<float>(),
                      N, Cin, Cout, H, W, chunks, stream(), accumulate);
}

}  // namespace

void register_stem(py::module& m) {
  m.def("stem_conv_fwd_stats", &fwd_stats, "stem conv forward + BN statistics into kRep fp64 replicas");
  m.def("stem_conv_wgrad_bn", &wgrad_bn, "stem conv weight gradient through the affine BN backward",
        py::arg("x"), py::arg("dy"), py::arg("z"), py::arg("red"), py::arg("stats"), py::arg("gamma"), py::arg("eps"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("partial"), py::arg("dw"), py::arg("world") = 1,
        py::arg("accumulate") = false);
  m.def("stem_conv_fwd", &fwd, "direct 3x3 stem conv forward (fp32 NCHW)");
  m.def("stem_conv_wgrad", &wgrad, "stem conv weight gradient (chunk partials + fixed-order sum)");
}
