// hipBLASLt GEMMs with fused epilogues for the GPT-2 trial (models/gpt2.py), the plain-library GEMM
// path of the trial kernels. The weight-gradient GEMMs of the layers whose bias gradient no other
// kernel already sums (MLP fc1, attention qkv) take hipBLASLt's BGRADB epilogue: dW and db in one
// pass over dY instead of the GEMM + a colsum_k pass over the same 16k x 3072 / 16k x 2304 gradient.
// Reference parity: the PBT GPT-2 member trains HF GPT2LMHeadModel (reference
// examples/v1beta1/trial-images/simple-pbt + SURVEY.md §2.9). Row-major torch tensors are handed to
// hipBLASLt as their column-major transposes. gfx950 solutions (scripts/lt_probe.py,
// profiles/lt_epilogue_r05.log): BIAS / GELU / GELU_BIAS for every layout, BGRADB for (N, T) only,
// none for GELU_AUX*, DGELU*, BGRADA - so the GELU forward / backward stay in gemm_nt / gelu_bwd_k.
// Measured on MI355X: the BGRADB solutions are unsplit 256x128 MI32x32 tiles, 197 / 115 us per fc1 /
// qkv wgrad against 65-72 us for the split-K form + 14.5 us colsum, so the path is opt-in
// (KATIB_LT_EPILOGUE=1). Every entry returns false (nothing launched) when hipBLASLt has no
// solution, and the caller keeps its two-kernel path.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <tuple>

namespace py = pybind11;
using at::Tensor;

namespace {

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  size_t ws = 0;
  bool ok = false;
};

// (device, transA, transB, m, n, k, lda, ldb, ldd, epilogue, bias type)
using Key = std::tuple<int, int, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int, int>;

std::mutex g_mu;
std::map<int, hipblasLtHandle_t> g_handles;
std::map<Key, Plan> g_plans;
constexpr uint64_t kMaxWs = 32ull << 20;

hipblasLtHandle_t handle(int dev) {
  auto it = g_handles.find(dev);
  if (it != g_handles.end()) return it->second;
  hipblasLtHandle_t h = nullptr;
  TORCH_CHECK(hipblasLtCreate(&h) == HIPBLAS_STATUS_SUCCESS, "hipblasLtCreate failed");
  g_handles[dev] = h;
  return h;
}

template <class T>
bool set(hipblasLtMatmulDesc_t d, hipblasLtMatmulDescAttributes_t a, const T& v) {
  return hipblasLtMatmulDescSetAttribute(d, a, &v, sizeof(T)) == HIPBLAS_STATUS_SUCCESS;
}

// Build (once per shape) the descriptor + layouts and pick hipBLASLt's first heuristic solution.
// Pointers are set per call; the algorithm does not depend on them.
Plan& plan(int dev, hipblasOperation_t ta, hipblasOperation_t tb, int64_t m, int64_t n, int64_t k, int64_t lda,
           int64_t ldb, int64_t ldd, hipblasLtEpilogue_t epi, hipDataType bias_t, const void* bias, const void* aux,
           int64_t ldaux) {
  Key key{dev, (int)ta, (int)tb, m, n, k, lda, ldb, ldd, (int)epi, (int)bias_t};
  auto it = g_plans.find(key);
  if (it != g_plans.end()) return it->second;
  Plan& p = g_plans[key];
  hipblasLtHandle_t h = handle(dev);
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return p;
  const int32_t ta32 = (int32_t)ta, tb32 = (int32_t)tb;
  bool good = set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, ta32) && set(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, tb32) &&
              set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, epi) &&
              set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, (int32_t)bias_t) &&
              set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, bias) &&
              set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, aux) &&
              set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, ldaux);
  const int64_t ar = ta == HIPBLAS_OP_N ? m : k, ac = ta == HIPBLAS_OP_N ? k : m;
  const int64_t br = tb == HIPBLAS_OP_N ? k : n, bc = tb == HIPBLAS_OP_N ? n : k;
  good = good && hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ar, ac, lda) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, br, bc, ldb) == HIPBLAS_STATUS_SUCCESS &&
         hipblasLtMatrixLayoutCreate(&p.d, HIP_R_16BF, m, n, ldd) == HIPBLAS_STATUS_SUCCESS;
  if (!good) return p;
  hipblasLtMatmulPreference_t pref = nullptr;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return p;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &kMaxWs, sizeof(kMaxWs));
  hipblasLtMatmulHeuristicResult_t res[1];
  int got = 0;
  const auto st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.d, p.d, pref, 1, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st == HIPBLAS_STATUS_SUCCESS && got > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS) {
    p.algo = res[0].algo;
    p.ws = res[0].workspaceSize;
    p.ok = true;
  }
  return p;
}

void chk(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous(), name, " must be a contiguous ",
              c10::toString(dt), " GPU tensor");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

bool run(Plan& p, int dev, const void* A, const void* B, void* D, const void* bias, const void* aux) {
  if (!p.ok) return false;
  if (!set(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, bias) ||
      !set(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_POINTER, aux))
    return false;
  Tensor ws;
  void* wsp = nullptr;
  if (p.ws) {
    ws = at::empty({(int64_t)p.ws}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
    wsp = ws.data_ptr();
  }
  const float one = 1.f, zero = 0.f;
  const auto st = hipblasLtMatmul(handle(dev), p.desc, &one, A, p.a, B, p.b, &zero, D, p.d, D, p.d, &p.algo, wsp,
                                  p.ws, c10::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(st == HIPBLAS_STATUS_SUCCESS, "hipblasLtMatmul (epilogue) failed: ", (int)st);
  return true;
}

// dw[N, K] = dy[M, N]^T x[M, K] and db[N] = column sums of dy, in one GEMM (BGRADB: the bias gradient
// reduced from operand B while it is streamed for the product).
bool lt_wgrad_bgrad(const Tensor& dy, const Tensor& x, const Tensor& dw, const Tensor& db) {
  chk(dy, at::kBFloat16, "dy");
  chk(x, at::kBFloat16, "x");
  chk(dw, at::kBFloat16, "dw");
  chk(db, at::kBFloat16, "db");
  TORCH_CHECK(dy.dim() == 2 && x.dim() == 2 && dy.size(0) == x.size(0), "lt_wgrad_bgrad: dy [M, N], x [M, K]");
  const int64_t M = dy.size(0), N = dy.size(1), K = x.size(1);
  TORCH_CHECK(dw.numel() == N * K && db.numel() == N, "lt_wgrad_bgrad: dw [N, K], db [N]");
  const int dev = dy.get_device();
  std::lock_guard<std::mutex> lk(g_mu);
  // column-major: dw^T [K, N] = X^T ([K, M] stored, N) . dY ([N, M] stored, T)
  Plan& p = plan(dev, HIPBLAS_OP_N, HIPBLAS_OP_T, K, N, M, K, N, K, HIPBLASLT_EPILOGUE_BGRADB, HIP_R_16BF,
                 db.data_ptr(), nullptr, K);
  return run(p, dev, x.data_ptr(), dy.data_ptr(), dw.data_ptr(), db.data_ptr(), nullptr);
}

// Diagnostic: how many heuristic solutions hipBLASLt returns for an epilogue / layout / type combination
// (bf16 A, B, D; fp32 compute). Negative: the hipblasStatus_t of the failing call. No GPU memory is touched.
int64_t lt_probe(int64_t epi, int64_t ta, int64_t tb, int64_t m, int64_t n, int64_t k, int64_t bias_t,
                 int64_t aux_t, int64_t dev) {
  std::lock_guard<std::mutex> lk(g_mu);
  hipblasLtHandle_t h = handle((int)dev);
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, d = nullptr;
  auto st = hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F, HIP_R_32F);
  if (st != HIPBLAS_STATUS_SUCCESS) return -(int64_t)st - 1000;
  const auto opa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, opb = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  set(desc, HIPBLASLT_MATMUL_DESC_TRANSA, (int32_t)opa);
  set(desc, HIPBLASLT_MATMUL_DESC_TRANSB, (int32_t)opb);
  set(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, (hipblasLtEpilogue_t)epi);
  if (bias_t >= 0) set(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, (int32_t)bias_t);
  if (aux_t >= 0) set(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_DATA_TYPE, (int32_t)aux_t);
  set(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE_AUX_LD, (int64_t)m);
  const int64_t ar = ta ? k : m, ac = ta ? m : k, br = tb ? n : k, bc = tb ? k : n;
  hipblasLtMatrixLayoutCreate(&a, HIP_R_16BF, ar, ac, ar);
  hipblasLtMatrixLayoutCreate(&b, HIP_R_16BF, br, bc, br);
  hipblasLtMatrixLayoutCreate(&d, HIP_R_16BF, m, n, m);
  hipblasLtMatmulPreference_t pref = nullptr;
  hipblasLtMatmulPreferenceCreate(&pref);
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &kMaxWs, sizeof(kMaxWs));
  hipblasLtMatmulHeuristicResult_t res[8];
  int got = 0;
  st = hipblasLtMatmulAlgoGetHeuristic(h, desc, a, b, d, d, pref, 8, res, &got);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(a);
  hipblasLtMatrixLayoutDestroy(b);
  hipblasLtMatrixLayoutDestroy(d);
  hipblasLtMatmulDescDestroy(desc);
  return st == HIPBLAS_STATUS_SUCCESS ? got : -(int64_t)st;
}

}  // namespace

void register_lt_epilogue(py::module& m) {
  m.def("lt_wgrad_bgrad", &lt_wgrad_bgrad, "hipBLASLt weight-gradient GEMM + bias gradient (BGRADB epilogue)",
        py::arg("dy"), py::arg("x"), py::arg("dw"), py::arg("db"));
  m.def("lt_probe", &lt_probe, "number of hipBLASLt heuristic solutions for an epilogue / layout / type", py::arg("epi"),
        py::arg("ta"), py::arg("tb"), py::arg("m"), py::arg("n"), py::arg("k"), py::arg("bias_t") = -1,
        py::arg("aux_t") = -1, py::arg("dev") = 0);
}
