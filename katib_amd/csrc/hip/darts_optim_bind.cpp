// torch bindings of the DARTS search-step optimizer kernels (darts_optim.hip), with the
// dtype / size / device checks the kernels rely on.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <algorithm>
#include <optional>
#include <vector>

#include "darts_optim.h"
#include "darts_ops.h"  // kRep

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
                  double wd, const Tensor& av, const Tensor& a, const Tensor& zero_w, const Tensor& zero_a, bool zero_g) {
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
  p.g_zero = zero_g ? const_cast<float*>(p.g) : nullptr;
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

// softmax of the (normal[, reduce]) alpha matrices -> weights; optionally zeroes an f64 buffer
void alpha_softmax(std::vector<Tensor> alphas, std::vector<Tensor> outs, std::optional<Tensor> zero) {
  TORCH_CHECK(!alphas.empty() && alphas.size() <= 2 && alphas.size() == outs.size(), "alpha_softmax: 1 or 2 matrices");
  O_::AlphaSoftmaxArgs p{};
  p.nmat = alphas.size();
  p.K = alphas[0].size(1);
  TORCH_CHECK(p.K >= 1 && p.K <= 16, "alpha_softmax: K in [1, 16]");
  for (int m = 0; m < p.nmat; ++m) {
    TORCH_CHECK(alphas[m].dim() == 2 && alphas[m].size(1) == p.K && outs[m].sizes() == alphas[m].sizes(),
                "alpha_softmax: [rows][K] matrices");
    p.a[m] = f32(alphas[m], "alpha", -1, alphas[0]);
    p.w[m] = f32(outs[m], "weights", alphas[m].numel(), alphas[0]);
    p.rows[m] = alphas[m].size(0);
  }
  if (zero.has_value() && zero->defined()) {
    TORCH_CHECK(zero->is_cuda() && zero->scalar_type() == at::kDouble && zero->is_contiguous() &&
                    zero->device() == alphas[0].device(), "alpha_softmax: zero must be contiguous f64 on the device");
    p.zero = zero->data_ptr<double>();
    p.nzero = zero->numel();
  }
  O_::launch_alpha_softmax(p, stream());
}

// entries: (g: f64 tensor holding kRep replicas of [K], rstride, softmax weight row [K], destination row [K]);
// entries sharing a destination row are summed (grouped here; the kernel runs a workgroup per row)
void alpha_grad(std::vector<py::tuple> entries, bool accumulate) {
  TORCH_CHECK(!entries.empty() && (int)entries.size() <= O_::kAlphaGradMax, "alpha_grad: 1..kAlphaGradMax entries");
  O_::AlphaGradArgs p{};
  p.accumulate = accumulate;
  struct Ent { const double* g; int rs; const float* w; float* d; };
  std::vector<Ent> ents;
  std::vector<float*> rows;
  for (size_t e = 0; e < entries.size(); ++e) {
    const py::tuple& t = entries[e];
    Tensor g = t[0].cast<Tensor>(), w = t[2].cast<Tensor>(), d = t[3].cast<Tensor>();
    const int rs = t[1].cast<int>();
    const int K = w.numel();
    if (e == 0) p.K = K;
    TORCH_CHECK(K == p.K && K >= 1 && K <= 16 && d.numel() == K, "alpha_grad: rows of K <= 16");
    TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kDouble && g.is_contiguous() &&
                    g.numel() >= (int64_t)(katib_hip::kRep - 1) * rs + K && rs >= K,
                "alpha_grad: g must hold kRep f64 replicas of [K]");
    Ent x{g.data_ptr<double>(), rs, f32(w, "w", K, w), f32(d, "dst", K, w)};
    ents.push_back(x);
    if (std::find(rows.begin(), rows.end(), x.d) == rows.end()) rows.push_back(x.d);
  }
  p.nrows = rows.size();
  p.n = 0;
  for (int r = 0; r < p.nrows; ++r) {
    p.dst[r] = rows[r];
    p.row_start[r] = p.n;
    for (const Ent& x : ents)
      if (x.d == rows[r]) {
        p.g[p.n] = x.g;
        p.rstride[p.n] = x.rs;
        p.w[p.n] = x.w;
        ++p.n;
      }
  }
  p.row_start[p.nrows] = p.n;
  O_::launch_alpha_grad(p, stream());
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
              double clip, double mu, double wd, bool zero_g) {
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
  p.zero_g = zero_g ? 1 : 0;
  O_::launch_sgd_clip(p, stream());
}

}  // namespace

void register_darts_optim(py::module& m) {
  m.attr("OPTIM_MAX_PARTS") = O_::kMaxParts;
  m.def("optim_sumsq", &sumsq, "fp64 sum-of-squares partials (one per workgroup); returns the partial count");
  m.def("optim_virtual_step", &virtual_step, "architect virtual step w' = w - lr (mu m + g + wd w), alpha' = alpha");
  m.def("alpha_softmax", &alpha_softmax, "softmax over the primitives of the alpha matrices (+ optional f64 zeroing)",
        py::arg("alphas"), py::arg("outs"), py::arg("zero") = py::none());
  m.def("alpha_grad", &alpha_grad, "d alpha from replicated d(softmax weight) through the softmax Jacobian",
        py::arg("entries"), py::arg("accumulate"));
  m.def("optim_hessian_split", &hessian_split,
        "concurrent finite-difference Hessian passes: split (phase 3) / merge (phase 2)");
  m.def("optim_hessian", &hessian, "finite-difference Hessian perturbation phase 0/1/2");
  m.def("optim_adam", &adam, "Adam (L2 weight decay) on the architecture weights, device step counter");
  m.def("optim_sgd_clip", &sgd_clip, "global-norm clip + momentum SGD with weight decay");
}
