// torch bindings for the ENAS controller kernel (module katib_amd._hipkern, enas_* entry points).
// Shapes, dtypes, devices and the LDS budget are validated here before the launch.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "enas_ctrl.h"

using at::Tensor;
namespace E = katib_hip::enas;

namespace {

void check(const Tensor& t, at::ScalarType ty, int64_t n, const char* name, const Tensor& ref) {
  TORCH_CHECK(t.is_cuda() && t.device() == ref.device(), name, " must be on the controller's GPU");
  TORCH_CHECK(t.scalar_type() == ty, name, " has the wrong dtype");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() >= n, name, " is too small (", t.numel(), " < ", n, ")");
}

E::Args make_args(Tensor P, int64_t L, int64_t n_ops, int64_t H, py::dict cfg) {
  TORCH_CHECK(H >= 1 && H <= E::kMaxH, "controller_hidden_size must be in [1, ", E::kMaxH, "] for the HIP controller");
  TORCH_CHECK(n_ops >= 1 && n_ops <= E::kMaxOps, "number of operations out of range for the HIP controller");
  TORCH_CHECK(L >= 1 && L <= E::kMaxLayers, "num_layers out of range for the HIP controller");
  TORCH_CHECK(E::lds_bytes(H, n_ops, L) <= 160 * 1024, "controller does not fit the 160 KB LDS");
  const E::Offsets o = E::offsets(H, n_ops);
  check(P, at::kFloat, o.n, "params", P);
  E::Args a{};
  a.P = P.data_ptr<float>();
  a.L = L;
  a.n_ops = n_ops;
  a.H = H;
  auto opt = [&](const char* k, int& use, float& val) {
    py::object v = cfg[k];
    use = v.is_none() ? 0 : 1;
    val = v.is_none() ? 0.f : v.cast<float>();
  };
  opt("temperature", a.use_temp, a.temperature);
  opt("tanh_const", a.use_tanh, a.tanh_c);
  opt("entropy_weight", a.use_ew, a.entropy_weight);
  opt("skip_weight", a.use_sw, a.skip_weight);
  a.skip_target = cfg["skip_target"].cast<float>();
  a.baseline_decay = cfg["baseline_decay"].cast<float>();
  a.lr = cfg["lr"].cast<float>();
  a.beta1 = cfg["beta1"].cast<float>();
  a.beta2 = cfg["beta2"].cast<float>();
  a.eps = cfg["eps"].cast<float>();
  const double decay = cfg["baseline_decay"].cast<double>(), b1 = cfg["beta1"].cast<double>(),
               b2 = cfg["beta2"].cast<double>();
  a.baseline_rate = (float)(1.0 - decay);  // as torch: the Python-double difference, then fp32
  a.omb1 = (float)(1.0 - b1);
  a.omb2 = (float)(1.0 - b2);
  TORCH_CHECK(a.skip_target > 0.f && a.skip_target < 1.f, "skip_target must be in (0, 1)");
  TORCH_CHECK(!a.use_temp || a.temperature != 0.f, "temperature must be non-zero");
  TORCH_CHECK(!a.use_tanh || a.tanh_c != 0.f, "tanh_const must be non-zero");
  return a;
}

void set_forced(E::Args& a, const c10::optional<Tensor>& forced, int64_t rows, const Tensor& P) {
  if (!forced.has_value() || !forced->defined()) return;
  const int alen = E::arc_len(a.L);
  check(*forced, at::kInt, alen, "forced", P);
  TORCH_CHECK(forced->numel() == alen || forced->numel() == rows * alen, "forced arcs: one arc or one per row");
  a.forced = forced->data_ptr<int>();
  a.forced_stride = forced->numel() == alen ? 0 : alen;
  auto f = forced->cpu();
  const int* fp = f.data_ptr<int>();
  for (int64_t r = 0; r < forced->numel() / alen; ++r)
    for (int l = 0, pos = 0; l < a.L; pos += l + 1, ++l) {
      TORCH_CHECK(fp[r * alen + pos] >= 0 && fp[r * alen + pos] < a.n_ops, "forced op index out of range");
      for (int i = 0; i < l; ++i) TORCH_CHECK(fp[r * alen + pos + 1 + i] == 0 || fp[r * alen + pos + 1 + i] == 1,
                                              "forced skip must be 0 or 1");
    }
}

// one arc per row of `arcs` [n, arc_len] (int32); tape [n, tape_floats]
void enas_sample(Tensor P, Tensor arcs, Tensor tape, int64_t L, int64_t n_ops, int64_t H, py::dict cfg,
                 int64_t seed, int64_t rng_offset, c10::optional<Tensor> forced) {
  E::Args a = make_args(P, L, n_ops, H, cfg);
  const int64_t n = arcs.size(0);
  TORCH_CHECK(arcs.dim() == 2 && arcs.size(1) == E::arc_len(L) && n >= 1, "arcs must be [n, arc_len]");
  check(arcs, at::kInt, n * E::arc_len(L), "arcs", P);
  check(tape, at::kFloat, n * E::tape_floats(H, n_ops, L), "tape", P);
  a.arcs = arcs.data_ptr<int>();
  a.tape = tape.data_ptr<float>();
  a.seed = (unsigned long long)seed;
  a.rng_offset = (unsigned long long)rng_offset;
  a.nsteps = 0;
  set_forced(a, forced, n, P);
  E::launch(a, (int)n, c10::hip::getCurrentHIPStream().stream());
}

// `nsteps` REINFORCE steps in one launch: arcs [nsteps, arc_len], logs [nsteps, 8]
void enas_train(Tensor P, Tensor M, Tensor V, Tensor G, Tensor tape, Tensor arcs, Tensor logs, Tensor baseline,
                int64_t L, int64_t n_ops, int64_t H, py::dict cfg, double reward, int64_t nsteps, int64_t adam_t0,
                int64_t seed, int64_t rng_offset, c10::optional<Tensor> forced, c10::optional<Tensor> phase_clocks) {
  E::Args a = make_args(P, L, n_ops, H, cfg);
  const int64_t n = E::offsets(H, n_ops).n;
  if (phase_clocks.has_value() && phase_clocks->defined()) {
    check(*phase_clocks, at::kLong, 5, "phase_clocks", P);
    a.phase_clocks = reinterpret_cast<long long*>(phase_clocks->data_ptr<int64_t>());
  }
  TORCH_CHECK(nsteps >= 1, "nsteps >= 1");
  check(M, at::kFloat, n, "adam m", P);
  check(V, at::kFloat, n, "adam v", P);
  check(G, at::kFloat, n, "grad", P);
  check(tape, at::kFloat, E::tape_floats(H, n_ops, L), "tape", P);
  check(arcs, at::kInt, nsteps * E::arc_len(L), "arcs", P);
  check(logs, at::kFloat, nsteps * E::kLogFields, "logs", P);
  check(baseline, at::kFloat, 1, "baseline", P);
  a.M = M.data_ptr<float>();
  a.V = V.data_ptr<float>();
  a.G = G.data_ptr<float>();
  a.tape = tape.data_ptr<float>();
  a.arcs = arcs.data_ptr<int>();
  a.logs = logs.data_ptr<float>();
  a.baseline = baseline.data_ptr<float>();
  a.reward = (float)reward;
  a.nsteps = (int)nsteps;
  a.adam_t0 = (int)adam_t0;
  a.seed = (unsigned long long)seed;
  a.rng_offset = (unsigned long long)rng_offset;
  set_forced(a, forced, nsteps, P);
  E::launch(a, 1, c10::hip::getCurrentHIPStream().stream());
}

}  // namespace

void register_enas(py::module& m) {
  m.def("enas_sample", &enas_sample, "ENAS controller: sample one arc per workgroup");
  m.def("enas_train", &enas_train, "ENAS controller: nsteps REINFORCE steps (sample, BPTT, Adam) in one workgroup",
        py::arg("P"), py::arg("M"), py::arg("V"), py::arg("G"), py::arg("tape"), py::arg("arcs"), py::arg("logs"),
        py::arg("baseline"), py::arg("L"), py::arg("n_ops"), py::arg("H"), py::arg("cfg"), py::arg("reward"),
        py::arg("nsteps"), py::arg("adam_t0"), py::arg("seed"), py::arg("rng_offset"), py::arg("forced"),
        py::arg("phase_clocks") = py::none());
  m.def("enas_tape_floats", [](int64_t H, int64_t n_ops, int64_t L) { return E::tape_floats(H, n_ops, L); });
  m.def("enas_n_params", [](int64_t H, int64_t n_ops) { return E::offsets(H, n_ops).n; });
  m.def("enas_lds_bytes", [](int64_t H, int64_t n_ops, int64_t L) { return E::lds_bytes(H, n_ops, L); });
  m.attr("ENAS_LOG_FIELDS") = E::kLogFields;
  m.attr("ENAS_MAX_H") = E::kMaxH;
  m.attr("ENAS_MAX_OPS") = E::kMaxOps;
  m.attr("ENAS_MAX_LAYERS") = E::kMaxLayers;
  m.attr("ENAS_LDS_LIMIT") = 160 * 1024;
}
