// torch bindings of the fused ResNet-18 step kernels (resnet_step.hip). Every tensor is checked
// against the sizes the kernels index; the SGD segment table is validated once when it is built
// and copied to the device (the captured step then only passes its pointer).
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstring>
#include <vector>

#include "resnet_step.h"

namespace py = pybind11;
using at::Tensor;
namespace R_ = katib_hip::rn;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const Tensor& t, at::ScalarType dt, int64_t numel, const char* name, const Tensor& ref) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous(), name, " must be a contiguous ",
              c10::toString(dt), " GPU tensor");
  TORCH_CHECK(t.device() == ref.device(), name, " must be on the device of the other operands");
  TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
}

// tx: [n_src, H, W, C] bf16 (NHWC), idx: [B] int64, xb: [B, H, W, C8] bf16
void gather(const Tensor& tx, const Tensor& idx, const Tensor& xb) {
  TORCH_CHECK(tx.dim() == 4 && xb.dim() == 4 && idx.dim() == 1, "rn_gather: tx / xb are [N, H, W, C], idx [B]");
  const int64_t B = idx.size(0), H = tx.size(1), W = tx.size(2), C = tx.size(3), C8 = xb.size(3);
  TORCH_CHECK(xb.size(0) == B && xb.size(1) == H && xb.size(2) == W && C8 % 8 == 0 && C <= C8,
              "rn_gather: xb must be [B, H, W, C8 >= C], C8 % 8 == 0");
  chk(tx, at::kBFloat16, tx.size(0) * H * W * C, "tx", xb);
  chk(idx, at::kLong, B, "idx", xb);
  chk(xb, at::kBFloat16, B * H * W * C8, "xb", xb);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(xb.data_ptr()) % 16 == 0, "rn_gather: xb must be 16-byte aligned");
  TORCH_CHECK(B * H * W < (1ll << 31), "rn_gather: batch too large");
  TORCH_CHECK(R_::launch_gather(reinterpret_cast<const R_::bf16*>(tx.data_ptr()), idx.data_ptr<int64_t>(),
                                reinterpret_cast<R_::bf16*>(xb.data_ptr()), (int)B, (int)(H * W), (int)C, (int)C8,
                                tx.size(0), stream()) == hipSuccess,
              "rn_gather launch failed");
}

// x: [B, HW, C] bf16, w: [K, C] fp32, bias [K], ty: int64 labels, idx [B]
void head(const Tensor& x, const Tensor& w, const Tensor& bias, const Tensor& ty, const Tensor& idx, const Tensor& dx,
          const Tensor& pooled, const Tensor& dl, const Tensor& loss_n, const Tensor& gw, const Tensor& gb,
          const c10::optional<Tensor>& loss_acc) {
  TORCH_CHECK(x.dim() == 3 && w.dim() == 2, "rn_head: x is [B, HW, C], w [K, C]");
  const int64_t B = x.size(0), HW = x.size(1), C = x.size(2), K = w.size(0);
  TORCH_CHECK(w.size(1) == C && B >= 1 && HW >= 1 && C % 8 == 0 && C <= R_::kHeadMaxC && K >= 1 &&
                  K <= R_::kHeadMaxK,
              "rn_head: C % 8 == 0, C <= ", R_::kHeadMaxC, ", K <= ", R_::kHeadMaxK);
  chk(x, at::kBFloat16, B * HW * C, "x", x);
  chk(dx, at::kBFloat16, B * HW * C, "dx", x);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dx.data_ptr()) % 16 == 0,
              "rn_head: x / dx must be 16-byte aligned");
  chk(w, at::kFloat, K * C, "w", x);
  chk(bias, at::kFloat, K, "bias", x);
  TORCH_CHECK(ty.dim() == 1, "rn_head: ty must be 1-D");
  chk(ty, at::kLong, ty.numel(), "ty", x);
  chk(idx, at::kLong, B, "idx", x);
  chk(pooled, at::kFloat, B * C, "pooled", x);
  chk(dl, at::kFloat, B * K, "dl", x);
  chk(loss_n, at::kFloat, B, "loss_n", x);
  chk(gw, at::kFloat, K * C, "gw", x);
  chk(gb, at::kFloat, K, "gb", x);
  if (loss_acc.has_value()) chk(*loss_acc, at::kFloat, 1, "loss_acc", x);
  R_::HeadArgs a;
  a.x = reinterpret_cast<const R_::bf16*>(x.data_ptr());
  a.w = w.data_ptr<float>();
  a.bias = bias.data_ptr<float>();
  a.ty = ty.data_ptr<int64_t>();
  a.idx = idx.data_ptr<int64_t>();
  a.n_labels = ty.numel();
  a.dx = reinterpret_cast<R_::bf16*>(dx.data_ptr());
  a.pooled = pooled.data_ptr<float>();
  a.dl = dl.data_ptr<float>();
  a.loss_n = loss_n.data_ptr<float>();
  a.gw = gw.data_ptr<float>();
  a.gb = gb.data_ptr<float>();
  a.loss_acc = loss_acc.has_value() ? loss_acc->data_ptr<float>() : nullptr;
  a.B = (int)B;
  a.HW = (int)HW;
  a.C = (int)C;
  a.K = (int)K;
  TORCH_CHECK(R_::launch_head(a, stream()) == hipSuccess, "rn_head launch failed");
}

// One entry per parameter tensor: (p, g, m, wk or None, wt or None, K, C, C8, RS); returns
// (device table as a uint8 tensor, segment count, total workgroups).
py::tuple sgd_table(const std::vector<py::tuple>& entries) {
  TORCH_CHECK(!entries.empty(), "rn_sgd_table: no parameters");
  std::vector<R_::SgdSeg> segs;
  int tiles = 0;
  c10::optional<at::Device> dev;
  for (const auto& e : entries) {
    TORCH_CHECK(e.size() == 9, "rn_sgd_table: entries are (p, g, m, wk, wt, K, C, C8, RS)");
    const Tensor p = e[0].cast<Tensor>(), g = e[1].cast<Tensor>(), m = e[2].cast<Tensor>();
    const int64_t K = e[5].cast<int64_t>(), C = e[6].cast<int64_t>(), C8 = e[7].cast<int64_t>(),
                  RS = e[8].cast<int64_t>();
    if (!dev) dev = p.device();
    R_::SgdSeg s{};
    chk(p, at::kFloat, p.numel(), "p", p);
    TORCH_CHECK(p.device() == *dev, "rn_sgd_table: every tensor on one device");
    TORCH_CHECK(p.numel() < (1ll << 31), "rn_sgd_table: parameter too large");
    s.p = p.data_ptr<float>();
    s.n = (int)p.numel();
    if (!e[3].is_none()) {
      const Tensor wk = e[3].cast<Tensor>();
      TORCH_CHECK(K >= 1 && C >= 1 && RS >= 1 && C8 >= C && C8 % 8 == 0 && p.numel() == K * RS * C,
                  "rn_sgd_table: filter geometry does not match p");
      chk(g, at::kFloat, K * RS * C8, "g", p);
      chk(m, at::kFloat, K * RS * C, "m", p);
      chk(wk, at::kBFloat16, K * RS * C8, "wk", p);
      s.wk = reinterpret_cast<R_::bf16*>(wk.data_ptr());
      if (!e[4].is_none()) {
        const Tensor wt = e[4].cast<Tensor>();
        chk(wt, at::kBFloat16, K * RS * C8, "wt", p);
        s.wt = reinterpret_cast<R_::bf16*>(wt.data_ptr());
      }
      s.K = (int)K;
      s.C = (int)C;
      s.C8 = (int)C8;
      s.RS = (int)RS;
    } else {
      chk(g, at::kFloat, p.numel(), "g", p);
      chk(m, at::kFloat, p.numel(), "m", p);
    }
    s.g = g.data_ptr<float>();
    s.m = m.data_ptr<float>();
    s.tile0 = tiles;
    tiles += R_::sgd_tiles(s);
    segs.push_back(s);
  }
  auto host = at::empty({(int64_t)(segs.size() * sizeof(R_::SgdSeg))}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(host.data_ptr(), segs.data(), segs.size() * sizeof(R_::SgdSeg));
  Tensor devt = host.to(*dev);
  return py::make_tuple(devt, (int64_t)segs.size(), (int64_t)tiles);
}

void sgd(const Tensor& table, int64_t nseg, int64_t tiles, double lr, double momentum, double wd, bool nesterov,
         bool update) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte &&
                  table.numel() == nseg * (int64_t)sizeof(R_::SgdSeg) && nseg >= 1 && tiles >= 1,
              "rn_sgd: table must come from rn_sgd_table");
  TORCH_CHECK(R_::launch_sgd(reinterpret_cast<const R_::SgdSeg*>(table.data_ptr()), (int)nseg, (int)tiles, (float)lr,
                             (float)momentum, (float)wd, nesterov ? 1 : 0, update ? 1 : 0, stream()) == hipSuccess,
              "rn_sgd launch failed");
}

}  // namespace

void register_resnet(py::module& m) {
  m.def("rn_gather", &gather, "batch gather of NHWC images by index + channel zero-pad to C8");
  m.def("rn_head", &head,
        "fused global-avg-pool + linear + cross-entropy forward and backward (input, weight, bias gradients, "
        "+= mean loss)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("ty"), py::arg("idx"), py::arg("dx"), py::arg("pooled"),
        py::arg("dl"), py::arg("loss_n"), py::arg("gw"), py::arg("gb"), py::arg("loss_acc") = py::none());
  m.def("rn_sgd_table", &sgd_table, "validate + upload the fused-SGD segment table");
  m.def("rn_sgd", &sgd,
        "one-launch SGD (momentum, Nesterov, weight decay) over every segment; zeroes the gradients and "
        "re-emits the bf16 filter images (update=False: images only)");
}
