// torch bindings of the DARTS search-step optimizer kernels (darts_optim.hip), with the
// dtype / size / device checks the kernels rely on.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "darts_optim.h"

namespace py = pybind11;
using at::Tensor;
namespace O_ = katib_hip::optim;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

float* f32(const Tensor& t, const char* name, int64_t numel, const Tensor& ref) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), name,
              " must be a contiguous float32 GPU tensor");
  TORCH_CHECK(t.device() == ref.device(), name, " must be on the device of the parameters");
  TORCH_CHECK(numel < 0 || t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  TORCH_CHECK(t.numel() < (int64_t(1) << 31), name, " too large for 32-bit indexing");
  return t.data_ptr<float>();
}

double* parts_ptr(const Tensor& p, const Tensor& ref) {
  TORCH_CHECK(p.is_cuda() && p.scalar_type() == at::kDouble && p.is_contiguous() && p.numel() >= O_::kMaxParts,
              "parts must be a contiguous float64 GPU tensor with >= ", O_::kMaxParts, " elements");
  TORCH_CHECK(p.device() == ref.device(), "parts must be on the device of the parameters");
  return p.data_ptr<double>();
}

// one fp64 partial per workgroup into parts[0:P]; returns P
int sumsq(const Tensor& x, const Tensor& parts) {
  const float* px = f32(x, "x", -1, x);
  double* pp = parts_ptr(parts, x);
  const int n = static_cast<int>(x.numel());
  O_::launch_sumsq(px, n, pp, stream());
  return O_::sumsq_parts(n);
}

void virtual_step(const Tensor& wv, const Tensor& w, const Tensor& mom, const Tensor& g, const Tensor& lr, double mu,
                  double wd, const Tensor& av, const Tensor& a, const Tensor& zero_w, const Tensor& zero_a) {
  const int64_t n = w.numel(), na = a.numel();
  O_::VirtualStepArgs p;
  p.wv = f32(wv, "wv", n, w);
  p.w = f32(w, "w", n, w);
  p.mom = f32(mom, "mom", n, w);
  p.g = f32(g, "g", n, w);
  p.lr = f32(lr, "lr", 1, w);
  p.mu = static_cast<float>(mu);
  p.wd = static_cast<float>(wd);
  p.n = static_cast<int>(n);
  p.av = f32(av, "av", na, w);
  p.a = f32(a, "a", na, w);
  p.na = static_cast<int>(na);
  p.zero_w = f32(zero_w, "zero_w", -1, w);
  p.n_zero_w = static_cast<int>(zero_w.numel());
  p.zero_a = f32(zero_a, "zero_a", na, w);
  TORCH_CHECK(na <= (int64_t(1) << 20), "too many architecture weights");
  O_::launch_virtual_step(p, stream());
}

void hessian(int phase, const Tensor& w, const Tensor& d, const Tensor& eps, const Tensor& parts, int nparts,
             const Tensor& ga, const Tensor& gap, const Tensor& gav, const Tensor& alpha_grad, const Tensor& lr) {
  TORCH_CHECK(phase >= 0 && phase <= 2, "hessian: phase must be 0, 1 or 2");
  TORCH_CHECK(nparts >= 1 && nparts <= O_::kMaxParts, "hessian: bad partial count");
  const int64_t n = w.numel(), na = ga.numel();
  O_::HessianArgs p;
  p.w = f32(w, "w", n, w);
  p.d = f32(d, "d", n, w);
  p.n = static_cast<int>(n);
  p.eps = f32(eps, "eps", 1, w);
  p.parts = parts_ptr(parts, w);
  p.nparts = nparts;
  p.ga = f32(ga, "ga", na, w);
  p.gap = f32(gap, "gap", na, w);
  p.gav = f32(gav, "gav", na, w);
  p.alpha_grad = f32(alpha_grad, "alpha_grad", na, w);
  p.lr = f32(lr, "lr", 1, w);
  p.na = static_cast<int>(na);
  p.phase = phase;
  O_::launch_hessian(p, stream());
}

// concurrent Hessian passes: phase 3 (wp, wm, eps, zeroed alpha accumulators, BN snapshots) and
// the final phase 2 without a weight update (alpha gradient + merged BN running statistics)
void hessian_split(int phase, const Tensor& w, const Tensor& d, const Tensor& eps, const Tensor& parts, int nparts,
                   const Tensor& ga, const Tensor& gap, const Tensor& gav, const Tensor& alpha_grad, const Tensor& lr,
                   const Tensor& wp, const Tensor& wm, const Tensor& bn, const Tensor& bn_plus, const Tensor& bn_zero,
                   double momentum) {
  TORCH_CHECK(phase == 2 || phase == 3, "hessian_split: phase must be 3 (split) or 2 (merge)");
  TORCH_CHECK(nparts >= 1 && nparts <= O_::kMaxParts, "hessian_split: bad partial count");
  const int64_t n = w.numel(), na = ga.numel(), nbn = bn.numel();
  O_::HessianArgs p;
  p.w = f32(w, "w", n, w);
  p.d = f32(d, "d", n, w);
  p.n = phase == 3 ? static_cast<int>(n) : 0;
  p.eps = f32(eps, "eps", 1, w);
  p.parts = parts_ptr(parts, w);
  p.nparts = nparts;
  p.ga = f32(ga, "ga", na, w);
  p.gap = f32(gap, "gap", na, w);
  p.gav = f32(gav, "gav", na, w);
  p.alpha_grad = f32(alpha_grad, "alpha_grad", na, w);
  p.lr = f32(lr, "lr", 1, w);
  p.na = static_cast<int>(na);
  p.phase = phase;
  p.wp = f32(wp, "wp", n, w);
  p.wm = f32(wm, "wm", n, w);
  p.bn = f32(bn, "bn", nbn, w);
  p.bn_plus = f32(bn_plus, "bn_plus", nbn, w);
  p.bn_zero = f32(bn_zero, "bn_zero", nbn, w);
  p.nbn = static_cast<int>(nbn);
  p.bn_momentum = static_cast<float>(momentum);
  O_::launch_hessian(p, stream());
}

void adam(const Tensor& a, const Tensor& grad, const Tensor& m, const Tensor& v, const Tensor& t, double lr, double b1,
          double b2, double wd, double eps, const Tensor& zero) {
  const int64_t n = a.numel();
  O_::AdamArgs p;
  p.a = f32(a, "a", n, a);
  p.grad = f32(grad, "grad", n, a);
  p.m = f32(m, "m", n, a);
  p.v = f32(v, "v", n, a);
  p.t = f32(t, "t", 1, a);
  p.lr = static_cast<float>(lr);
  p.b1 = static_cast<float>(b1);
  p.b2 = static_cast<float>(b2);
  p.wd = static_cast<float>(wd);
  p.eps = static_cast<float>(eps);
  p.n = static_cast<int>(n);
  p.zero = f32(zero, "zero", -1, a);
  p.nzero = static_cast<int>(zero.numel());
  TORCH_CHECK(n <= (int64_t(1) << 20) && p.nzero <= (1 << 20), "adam: single-workgroup kernel, too many elements");
  O_::launch_adam(p, stream());
}

void sgd_clip(const Tensor& w, const Tensor& g, const Tensor& mom, const Tensor& lr, const Tensor& parts, int nparts,
              double clip, double mu, double wd) {
  TORCH_CHECK(nparts >= 1 && nparts <= O_::kMaxParts, "sgd_clip: bad partial count");
  const int64_t n = w.numel();
  O_::SgdArgs p;
  p.w = f32(w, "w", n, w);
  p.g = f32(g, "g", n, w);
  p.mom = f32(mom, "mom", n, w);
  p.lr = f32(lr, "lr", 1, w);
  p.parts = parts_ptr(parts, w);
  p.nparts = nparts;
  p.clip = static_cast<float>(clip);
  p.mu = static_cast<float>(mu);
  p.wd = static_cast<float>(wd);
  p.n = static_cast<int>(n);
  O_::launch_sgd_clip(p, stream());
}

}  // namespace

void register_darts_optim(py::module& m) {
  m.attr("OPTIM_MAX_PARTS") = O_::kMaxParts;
  m.def("optim_sumsq", &sumsq, "fp64 sum-of-squares partials (one per workgroup); returns the partial count");
  m.def("optim_virtual_step", &virtual_step, "architect virtual step w' = w - lr (mu m + g + wd w), alpha' = alpha");
  m.def("optim_hessian_split", &hessian_split,
        "concurrent finite-difference Hessian passes: split (phase 3) / merge (phase 2)");
  m.def("optim_hessian", &hessian, "finite-difference Hessian perturbation phase 0/1/2");
  m.def("optim_adam", &adam, "Adam (L2 weight decay) on the architecture weights, device step counter");
  m.def("optim_sgd_clip", &sgd_clip, "global-norm clip + momentum SGD with weight decay");
}
