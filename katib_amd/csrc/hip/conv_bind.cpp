// torch bindings of the implicit-GEMM convolution kernels (conv_igemm.hip).
// Tensors are NHWC-contiguous bf16 views (x.permute(0, 2, 3, 1) of a channels_last
// tensor); geometry is passed explicitly and checked against every tensor size before
// launch, so the grid and the kernels' gathers never leave the allocations.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "conv_igemm.h"

namespace py = pybind11;
using at::Tensor;
using katib_hip::conv::ConvGeom;

namespace {

ConvGeom make_geom(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 15, "geometry: N,H,W,C,K,R,S,OH,OW,sh,sw,ph,pw,dh,dw");
  ConvGeom g{};
  int* f[15] = {&g.N, &g.H, &g.W, &g.C, &g.K, &g.R, &g.S, &g.OH, &g.OW, &g.sh, &g.sw, &g.ph, &g.pw, &g.dh, &g.dw};
  for (int i = 0; i < 15; ++i) {
    TORCH_CHECK(v[i] >= 0 && v[i] < (1 << 30), "geometry value out of range");
    *f[i] = (int)v[i];
  }
  TORCH_CHECK(g.N > 0 && g.H > 0 && g.W > 0 && g.C > 0 && g.K > 0 && g.R > 0 && g.S > 0, "empty geometry");
  TORCH_CHECK(g.sh > 0 && g.sw > 0 && g.dh > 0 && g.dw > 0, "stride / dilation must be positive");
  // (ph, pw) is the top/left padding; the bottom/right padding is implied by (OH, OW), which
  // allows TF-style asymmetric 'same' padding. Every gather is bounds-checked in the kernels.
  TORCH_CHECK(g.OH > 0 && g.OW > 0 && g.ph < g.dh * g.R && g.pw < g.dw * g.S &&
                  (int64_t)(g.OH - 1) * g.sh <= (int64_t)g.H + g.ph && (int64_t)(g.OW - 1) * g.sw <= (int64_t)g.W + g.pw,
              "output size inconsistent with the geometry");
  TORCH_CHECK((int64_t)g.N * g.H * g.W * g.C < (1ll << 31) && (int64_t)g.N * g.OH * g.OW * g.K < (1ll << 31),
              "tensor too large for 32-bit pixel indexing");
  return g;
}

void check_bf16(const Tensor& t, int64_t numel, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), name,
              " must be a contiguous bf16 GPU tensor");
  TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, geometry needs ", numel);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void conv_fwd(const Tensor& x, const Tensor& w, const Tensor& y, const std::vector<int64_t>& geom) {
  const ConvGeom g = make_geom(geom);
  TORCH_CHECK(g.C % 8 == 0, "conv_fwd: C must be a multiple of 8 (pad channels)");
  check_bf16(x, (int64_t)g.N * g.H * g.W * g.C, "x");
  check_bf16(w, (int64_t)g.K * g.R * g.S * g.C, "w");
  TORCH_CHECK(y.is_cuda() && y.is_contiguous() && y.numel() == (int64_t)g.N * g.OH * g.OW * g.K, "y shape");
  float* y32 = nullptr;
  __hip_bfloat16* yb = nullptr;
  if (y.scalar_type() == at::kFloat)
    y32 = y.data_ptr<float>();
  else {
    TORCH_CHECK(y.scalar_type() == at::kBFloat16, "y must be bf16 or fp32");
    yb = reinterpret_cast<__hip_bfloat16*>(y.data_ptr());
  }
  auto e = katib_hip::conv::launch_fwd(g, reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                                       reinterpret_cast<const __hip_bfloat16*>(w.data_ptr()), yb, y32, stream());
  TORCH_CHECK(e == hipSuccess, "conv_fwd launch: ", hipGetErrorString(e));
}

void conv_dgrad(const Tensor& dy, const Tensor& wt, const Tensor& dx, const std::vector<int64_t>& geom,
                const c10::optional<Tensor>& add_d, const c10::optional<Tensor>& add_y) {
  const ConvGeom g = make_geom(geom);
  TORCH_CHECK(g.K % 8 == 0, "conv_dgrad: K must be a multiple of 8");
  check_bf16(dy, (int64_t)g.N * g.OH * g.OW * g.K, "dy");
  check_bf16(wt, (int64_t)g.C * g.R * g.S * g.K, "wt");
  check_bf16(dx, (int64_t)g.N * g.H * g.W * g.C, "dx");
  TORCH_CHECK(add_d.has_value() || !add_y.has_value(), "conv_dgrad: add_y masks add_d");
  if (add_d.has_value()) check_bf16(*add_d, (int64_t)g.N * g.H * g.W * g.C, "add_d");
  if (add_y.has_value()) check_bf16(*add_y, (int64_t)g.N * g.H * g.W * g.C, "add_y");
  auto cp = [](const c10::optional<Tensor>& t) {
    return t.has_value() ? reinterpret_cast<const __hip_bfloat16*>(t->data_ptr()) : nullptr;
  };
  auto e = katib_hip::conv::launch_dgrad(g, reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr()),
                                         reinterpret_cast<const __hip_bfloat16*>(wt.data_ptr()),
                                         reinterpret_cast<__hip_bfloat16*>(dx.data_ptr()), stream(), cp(add_d),
                                         cp(add_y));
  TORCH_CHECK(e == hipSuccess, "conv_dgrad launch: ", hipGetErrorString(e));
}

void conv_wgrad(const Tensor& x, const Tensor& dy, const Tensor& dw32, const std::vector<int64_t>& geom) {
  const ConvGeom g = make_geom(geom);
  TORCH_CHECK(g.C % 8 == 0 && g.K % 8 == 0, "conv_wgrad: C and K must be multiples of 8");
  check_bf16(x, (int64_t)g.N * g.H * g.W * g.C, "x");
  check_bf16(dy, (int64_t)g.N * g.OH * g.OW * g.K, "dy");
  TORCH_CHECK(dw32.is_cuda() && dw32.scalar_type() == at::kFloat && dw32.is_contiguous() &&
                  dw32.numel() == (int64_t)g.K * g.R * g.S * g.C,
              "dw32 must be a contiguous fp32 [K][R*S*C] tensor");
  auto e = katib_hip::conv::launch_wgrad(g, reinterpret_cast<const __hip_bfloat16*>(x.data_ptr()),
                                         reinterpret_cast<const __hip_bfloat16*>(dy.data_ptr()),
                                         dw32.data_ptr<float>(), stream());
  TORCH_CHECK(e == hipSuccess, "conv_wgrad launch: ", hipGetErrorString(e));
}

}  // namespace

void register_conv(py::module& m) {
  m.def("conv_fwd", &conv_fwd, "implicit-GEMM conv forward (NHWC bf16, MFMA)");
  m.def("conv_dgrad", &conv_dgrad, "implicit-GEMM conv input gradient (+ optional ReLU-masked residual gradient)",
        py::arg("dy"), py::arg("wt"), py::arg("dx"), py::arg("geom"), py::arg("add_d") = py::none(),
        py::arg("add_y") = py::none());
  m.def("conv_wgrad", &conv_wgrad, "implicit-GEMM conv weight gradient (fp32 atomics, caller zeroes dw32)");
}
