// torch bindings of the NHWC depthwise convolution kernels (dwconv.hip). The geometry is
// checked against every tensor before launch: the kernels' gathers are bounds-checked per
// tap, and these checks keep the grid and the 16-byte vector accesses inside the tensors.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "dwconv.h"
#include "pool_nhwc.h"

namespace py = pybind11;
using at::Tensor;
namespace D = katib_hip::dwconv;

namespace {

D::Geom make_geom(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 11, "geometry: N,H,W,C,DM,K,S,pt,pl,OH,OW");
  D::Geom g{};
  int* f[11] = {&g.N, &g.H, &g.W, &g.C, &g.DM, &g.K, &g.S, &g.pt, &g.pl, &g.OH, &g.OW};
  for (int i = 0; i < 11; ++i) {
    TORCH_CHECK(v[i] >= 0 && v[i] < (1 << 30), "geometry value out of range");
    *f[i] = (int)v[i];
  }
  TORCH_CHECK(g.N > 0 && g.H > 0 && g.W > 0 && g.OH > 0 && g.OW > 0, "empty geometry");
  TORCH_CHECK(g.C % 8 == 0, "depthwise conv: C must be a multiple of 8");
  TORCH_CHECK(g.DM == 1 || g.DM == 2, "depth multiplier must be 1 or 2");
  TORCH_CHECK(g.K == 3 || g.K == 5 || g.K == 7, "kernel size must be 3, 5 or 7");
  TORCH_CHECK(g.S == 1 || g.S == 2, "stride must be 1 or 2");
  TORCH_CHECK(g.pt < g.K && g.pl < g.K, "padding must be smaller than the kernel");
  TORCH_CHECK((int64_t)(g.OH - 1) * g.S - g.pt < g.H && (int64_t)(g.OW - 1) * g.S - g.pl < g.W,
              "output size inconsistent with the geometry");
  TORCH_CHECK((int64_t)g.N * g.H * g.W * g.C * g.DM < (1ll << 40), "tensor too large");
  return g;
}

void check(const Tensor& t, at::ScalarType ty, int64_t numel, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == ty && t.is_contiguous(), name, " must be a contiguous ",
              ty == at::kBFloat16 ? "bf16" : "fp32", " GPU tensor");
  TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, geometry needs ", numel);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

const __hip_bfloat16* bf(const Tensor& t) { return reinterpret_cast<const __hip_bfloat16*>(t.data_ptr()); }
__hip_bfloat16* bfm(const Tensor& t) { return reinterpret_cast<__hip_bfloat16*>(t.data_ptr()); }

// x [N,H,W,C] bf16, w [K*K][C*DM] fp32 (tap-major), bias [C*DM] fp32 or None, y [N,OH,OW,C*DM] bf16
void dw_fwd(const Tensor& x, const Tensor& w, const c10::optional<Tensor>& bias, const Tensor& y,
            const std::vector<int64_t>& geom) {
  const D::Geom g = make_geom(geom);
  const int64_t Co = (int64_t)g.C * g.DM;
  check(x, at::kBFloat16, (int64_t)g.N * g.H * g.W * g.C, "x");
  check(w, at::kFloat, g.K * g.K * Co, "w");
  check(y, at::kBFloat16, (int64_t)g.N * g.OH * g.OW * Co, "y");
  const float* b = nullptr;
  if (bias.has_value() && bias->defined()) {
    check(*bias, at::kFloat, Co, "bias");
    b = bias->data_ptr<float>();
  }
  TORCH_CHECK(D::launch_fwd(g, bf(x), w.data_ptr<float>(), b, bfm(y), stream()) == hipSuccess, "dw_fwd launch failed");
}

void dw_dgrad(const Tensor& gy, const Tensor& w, const Tensor& gx, const std::vector<int64_t>& geom) {
  const D::Geom g = make_geom(geom);
  const int64_t Co = (int64_t)g.C * g.DM;
  check(gy, at::kBFloat16, (int64_t)g.N * g.OH * g.OW * Co, "gy");
  check(w, at::kFloat, g.K * g.K * Co, "w");
  check(gx, at::kBFloat16, (int64_t)g.N * g.H * g.W * g.C, "gx");
  TORCH_CHECK(D::launch_dgrad(g, bf(gy), w.data_ptr<float>(), bfm(gx), stream()) == hipSuccess, "dw_dgrad launch failed");
}

// part [rows][C*DM][K*K] fp32 partial weight gradients (rows = dw_wgrad_rows(geom))
void dw_wgrad(const Tensor& x, const Tensor& gy, const Tensor& part, const std::vector<int64_t>& geom) {
  const D::Geom g = make_geom(geom);
  const int64_t Co = (int64_t)g.C * g.DM;
  const int rows = D::wgrad_rows(g);
  check(x, at::kBFloat16, (int64_t)g.N * g.H * g.W * g.C, "x");
  check(gy, at::kBFloat16, (int64_t)g.N * g.OH * g.OW * Co, "gy");
  check(part, at::kFloat, (int64_t)rows * Co * g.K * g.K, "part");
  TORCH_CHECK(D::launch_wgrad(g, bf(x), bf(gy), part.data_ptr<float>(), rows, stream()) == hipSuccess,
              "dw_wgrad launch failed");
}

// ---- NHWC bf16 pooling (pool_nhwc.hip): geometry (N, H, W, C, P, S)
katib_hip::poolnhwc::Geom pool_geom(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 6, "pool geometry: N,H,W,C,P,S");
  for (int64_t e : v) TORCH_CHECK(e > 0 && e < (1 << 30), "pool geometry value out of range");
  katib_hip::poolnhwc::Geom g{(int)v[0], (int)v[1], (int)v[2], (int)v[3], (int)v[4], (int)v[5], 0, 0};
  TORCH_CHECK(g.C % 8 == 0, "pool: C must be a multiple of 8");
  TORCH_CHECK(g.P <= 16 && g.P <= g.H && g.P <= g.W, "pool window must fit the input (and be <= 16)");
  g.OH = (g.H - g.P) / g.S + 1;
  g.OW = (g.W - g.P) / g.S + 1;
  TORCH_CHECK((int64_t)g.N * g.H * g.W * g.C < (1ll << 40), "tensor too large");
  return g;
}

// x [N,H,W,C] bf16 -> y [N,OH,OW,C] bf16 (+ arg uint8, max pooling)
void pool_fwd(const Tensor& x, const Tensor& y, const c10::optional<Tensor>& arg, bool is_max,
              const std::vector<int64_t>& geom) {
  const auto g = pool_geom(geom);
  check(x, at::kBFloat16, (int64_t)g.N * g.H * g.W * g.C, "x");
  check(y, at::kBFloat16, (int64_t)g.N * g.OH * g.OW * g.C, "y");
  void* a = nullptr;
  if (is_max) {
    TORCH_CHECK(arg.has_value() && arg->defined(), "max pooling needs the argmax buffer");
    check(*arg, at::kByte, (int64_t)g.N * g.OH * g.OW * g.C, "arg");
    a = arg->data_ptr();
  }
  TORCH_CHECK(katib_hip::poolnhwc::launch_fwd(g, is_max, x.data_ptr(), y.data_ptr(), a, stream()) == hipSuccess,
              "pool_fwd launch failed");
}

void pool_bwd(const Tensor& gy, const c10::optional<Tensor>& arg, const Tensor& gx, bool is_max,
              const std::vector<int64_t>& geom) {
  const auto g = pool_geom(geom);
  check(gy, at::kBFloat16, (int64_t)g.N * g.OH * g.OW * g.C, "gy");
  check(gx, at::kBFloat16, (int64_t)g.N * g.H * g.W * g.C, "gx");
  const void* a = nullptr;
  if (is_max) {
    TORCH_CHECK(arg.has_value() && arg->defined(), "max pooling backward needs the argmax buffer");
    check(*arg, at::kByte, (int64_t)g.N * g.OH * g.OW * g.C, "arg");
    a = arg->data_ptr();
  }
  TORCH_CHECK(katib_hip::poolnhwc::launch_bwd(g, is_max, gy.data_ptr(), a, gx.data_ptr(), stream()) == hipSuccess,
              "pool_bwd launch failed");
}

}  // namespace

void register_dwconv(py::module& m) {
  m.def("pool_nhwc_fwd", &pool_fwd, "max / avg pooling forward (NHWC bf16, valid padding)");
  m.def("pool_nhwc_bwd", &pool_bwd, "max / avg pooling backward (NHWC bf16, gather, no atomics)");
  m.def("dw_fwd", &dw_fwd, "depthwise conv forward (NHWC bf16)", py::arg("x"), py::arg("w"), py::arg("bias"),
        py::arg("y"), py::arg("geom"));
  m.def("dw_dgrad", &dw_dgrad, "depthwise conv input gradient (NHWC bf16)");
  m.def("dw_wgrad", &dw_wgrad, "depthwise conv weight gradient partials (fp32)");
  m.def("dw_wgrad_rows", [](const std::vector<int64_t>& geom) { return D::wgrad_rows(make_geom(geom)); });
}
