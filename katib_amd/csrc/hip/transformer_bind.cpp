// torch bindings of the GPT-2 trial kernels (transformer.hip). Every entry point checks
// dtype, contiguity, device, alignment and the element counts the kernel and its grid
// assume before launching on the current HIP stream (graph-capturable: no host syncs).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "gemm_bf16.h"
#include "transformer.h"

namespace py = pybind11;
using at::Tensor;
namespace T_ = katib_hip::tfm;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void chk(const Tensor& t, at::ScalarType dt, int64_t numel, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == dt && t.is_contiguous(), name, " must be a contiguous ",
              c10::toString(dt), " GPU tensor");
  TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}
T_::bf16* bp(const Tensor& t) { return reinterpret_cast<T_::bf16*>(t.data_ptr()); }
void ok(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e)); }

void ln_fwd(const Tensor& x32, const c10::optional<Tensor>& r, const c10::optional<Tensor>& xo, const Tensor& gamma,
            const Tensor& beta, const Tensor& y, const Tensor& mean, const Tensor& rstd, double eps) {
  TORCH_CHECK(x32.dim() == 2, "x32 must be [M, D]");
  const int64_t M = x32.size(0), D = x32.size(1);
  TORCH_CHECK(D % 256 == 0 && D / 256 >= 1 && D / 256 <= 8 && D / 256 != 7, "ln_fwd: D must be 256*{1..6,8}");
  chk(x32, at::kFloat, M * D, "x32");
  chk(gamma, at::kBFloat16, D, "gamma");
  chk(beta, at::kBFloat16, D, "beta");
  chk(y, at::kBFloat16, M * D, "y");
  chk(mean, at::kFloat, M, "mean");
  chk(rstd, at::kFloat, M, "rstd");
  const T_::bf16* rp = nullptr;
  float* xop = nullptr;
  if (r.has_value()) {
    TORCH_CHECK(xo.has_value(), "ln_fwd: residual add needs xo");
    chk(*r, at::kBFloat16, M * D, "r");
    chk(*xo, at::kFloat, M * D, "xo");
    rp = bp(*r);
    xop = xo->data_ptr<float>();
  }
  ok(T_::ln_fwd(x32.data_ptr<float>(), rp, xop, bp(gamma), bp(beta), bp(y), mean.data_ptr<float>(),
                rstd.data_ptr<float>(), (int)M, (int)D, (float)eps, stream()),
     "ln_fwd");
}

int64_t ln_bwd_blocks(int64_t M) { return T_::ln_bwd_blocks((int)M); }

void ln_bwd(const Tensor& dy, const Tensor& xin, const Tensor& mean, const Tensor& rstd, const Tensor& gamma,
            const c10::optional<Tensor>& dres, const Tensor& dx, const c10::optional<Tensor>& dr,
            const Tensor& part_g, const Tensor& part_b, const c10::optional<Tensor>& part_r) {
  TORCH_CHECK(xin.dim() == 2, "xin must be [M, D]");
  const int64_t M = xin.size(0), D = xin.size(1);
  TORCH_CHECK(D % 256 == 0 && D / 256 >= 1 && D / 256 <= 8 && D / 256 != 7, "ln_bwd: D must be 256*{1..6,8}");
  chk(dy, at::kBFloat16, M * D, "dy");
  chk(xin, at::kFloat, M * D, "xin");
  chk(mean, at::kFloat, M, "mean");
  chk(rstd, at::kFloat, M, "rstd");
  chk(gamma, at::kBFloat16, D, "gamma");
  chk(dx, at::kFloat, M * D, "dx");
  const int64_t nb = T_::ln_bwd_blocks((int)M);
  chk(part_g, at::kFloat, nb * D, "part_g");
  chk(part_b, at::kFloat, nb * D, "part_b");
  const float* dresp = nullptr;
  if (dres.has_value()) {
    chk(*dres, at::kFloat, M * D, "dres");
    dresp = dres->data_ptr<float>();
  }
  T_::bf16* drp = nullptr;
  if (dr.has_value()) {
    chk(*dr, at::kBFloat16, M * D, "dr");
    drp = bp(*dr);
  }
  float* prp = nullptr;
  if (part_r.has_value()) {
    TORCH_CHECK(drp != nullptr, "ln_bwd: part_r (bias-gradient column sums of dr) needs dr");
    chk(*part_r, at::kFloat, nb * D, "part_r");
    prp = part_r->data_ptr<float>();
  }
  ok(T_::ln_bwd(bp(dy), xin.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), bp(gamma), dresp,
                dx.data_ptr<float>(), drp, part_g.data_ptr<float>(), part_b.data_ptr<float>(), (int)M, (int)D,
                stream(), prp),
     "ln_bwd");
}

void ln_reduce(const Tensor& part_g, const Tensor& part_b, const Tensor& dgamma, const Tensor& dbeta,
               const c10::optional<Tensor>& part_r, const c10::optional<Tensor>& dbias) {
  const int64_t D = dgamma.numel();
  TORCH_CHECK(D > 0 && part_g.numel() % D == 0, "ln_reduce: partials must be [nblk, D]");
  const int64_t nb = part_g.numel() / D;
  chk(part_g, at::kFloat, nb * D, "part_g");
  chk(part_b, at::kFloat, nb * D, "part_b");
  chk(dgamma, at::kBFloat16, D, "dgamma");
  chk(dbeta, at::kBFloat16, D, "dbeta");
  TORCH_CHECK(part_r.has_value() == dbias.has_value(), "ln_reduce: part_r and dbias go together");
  if (part_r.has_value()) {
    chk(*part_r, at::kFloat, nb * D, "part_r");
    chk(*dbias, at::kBFloat16, D, "dbias");
  }
  ok(T_::ln_reduce_params(part_g.data_ptr<float>(), part_b.data_ptr<float>(), (int)nb, (int)D, bp(dgamma), bp(dbeta),
                          stream(), part_r.has_value() ? part_r->data_ptr<float>() : nullptr,
                          dbias.has_value() ? bp(*dbias) : nullptr),
     "ln_reduce");
}

void gelu_fwd(const Tensor& u, const Tensor& g) {
  TORCH_CHECK(u.numel() % 8 == 0, "gelu: numel must be a multiple of 8");
  chk(u, at::kBFloat16, u.numel(), "u");
  chk(g, at::kBFloat16, u.numel(), "g");
  ok(T_::gelu_fwd(bp(u), bp(g), u.numel(), stream()), "gelu_fwd");
}

void gelu_bwd(const Tensor& u, const Tensor& dy, const Tensor& du) {
  TORCH_CHECK(u.numel() % 8 == 0, "gelu: numel must be a multiple of 8");
  chk(u, at::kBFloat16, u.numel(), "u");
  chk(dy, at::kBFloat16, u.numel(), "dy");
  chk(du, at::kBFloat16, u.numel(), "du");
  ok(T_::gelu_bwd(bp(u), bp(dy), bp(du), u.numel(), stream()), "gelu_bwd");
}

void xent_fwd(const Tensor& logits, const Tensor& tgt, const Tensor& loss, const Tensor& lse, int64_t V) {
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, Vp]");
  const int64_t N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V > 0 && V <= Vp, "xent: Vp % 8 == 0 and 0 < V <= Vp");
  chk(logits, at::kBFloat16, N * Vp, "logits");
  TORCH_CHECK(tgt.is_cuda() && tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == N, "tgt");
  chk(loss, at::kFloat, N, "loss");
  chk(lse, at::kFloat, N, "lse");
  ok(T_::xent_fwd(bp(logits), tgt.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(), (int)N, (int)V,
                  (int)Vp, stream()),
     "xent_fwd");
}

void xent_eval(const Tensor& logits, const Tensor& tgt, const Tensor& loss, const Tensor& hit, int64_t V) {
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, Vp]");
  const int64_t N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V > 0 && V <= Vp, "xent: Vp % 8 == 0 and 0 < V <= Vp");
  chk(logits, at::kBFloat16, N * Vp, "logits");
  TORCH_CHECK(tgt.is_cuda() && tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == N, "tgt");
  chk(loss, at::kFloat, N, "loss");
  chk(hit, at::kFloat, N, "hit");
  ok(T_::xent_eval(bp(logits), tgt.data_ptr<int64_t>(), loss.data_ptr<float>(), hit.data_ptr<float>(), (int)N, (int)V,
                   (int)Vp, stream()),
     "xent_eval");
}

void xent_bwd(const Tensor& logits, const Tensor& tgt, const Tensor& lse, const Tensor& gscale, double inv_n,
              int64_t V) {
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, Vp]");
  const int64_t N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V > 0 && V <= Vp, "xent: Vp % 8 == 0 and 0 < V <= Vp");
  chk(logits, at::kBFloat16, N * Vp, "logits");
  TORCH_CHECK(tgt.is_cuda() && tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == N, "tgt");
  chk(lse, at::kFloat, N, "lse");
  TORCH_CHECK(gscale.is_cuda() && gscale.scalar_type() == at::kFloat && gscale.numel() == 1, "gscale");
  ok(T_::xent_bwd(bp(logits), tgt.data_ptr<int64_t>(), lse.data_ptr<float>(), gscale.data_ptr<float>(), (float)inv_n,
                  (int)N, (int)V, (int)Vp, stream()),
     "xent_bwd");
}

bool xent_fused(const Tensor& logits, const Tensor& tgt, const Tensor& loss, const Tensor& lse, const Tensor& gscale,
                double inv_n, int64_t V) {
  TORCH_CHECK(logits.dim() == 2, "logits must be [N, Vp]");
  const int64_t N = logits.size(0), Vp = logits.size(1);
  TORCH_CHECK(Vp % 8 == 0 && V > 0 && V <= Vp, "xent: Vp % 8 == 0 and 0 < V <= Vp");
  chk(logits, at::kBFloat16, N * Vp, "logits");
  TORCH_CHECK(tgt.is_cuda() && tgt.scalar_type() == at::kLong && tgt.is_contiguous() && tgt.numel() == N, "tgt");
  chk(loss, at::kFloat, N, "loss");
  chk(lse, at::kFloat, N, "lse");
  TORCH_CHECK(gscale.is_cuda() && gscale.scalar_type() == at::kFloat && gscale.numel() == 1, "gscale");
  if (Vp / 8 > 512 * 13) return false;  // the caller falls back to xent_fwd + xent_bwd
  ok(T_::xent_fused(bp(logits), tgt.data_ptr<int64_t>(), loss.data_ptr<float>(), lse.data_ptr<float>(),
                    gscale.data_ptr<float>(), (float)inv_n, (int)N, (int)V, (int)Vp, stream()),
     "xent_fused");
  return true;
}

void grad_sumsq(const Tensor& g, const Tensor& sumsq) {
  TORCH_CHECK(g.numel() % 8 == 0, "grad_sumsq: numel must be a multiple of 8");
  chk(g, at::kBFloat16, g.numel(), "g");
  TORCH_CHECK(sumsq.is_cuda() && sumsq.scalar_type() == at::kFloat && sumsq.numel() == 1, "sumsq");
  ok(T_::grad_sumsq(bp(g), g.numel(), sumsq.data_ptr<float>(), stream()), "grad_sumsq");
}

void adamw(const Tensor& p, const Tensor& g, const Tensor& m, const Tensor& v, const Tensor& w16, const Tensor& lr,
           const Tensor& step, double b1, double b2, double eps, double wd, const Tensor& sumsq, double max_norm) {
  const int64_t n = p.numel();
  TORCH_CHECK(n % 8 == 0, "adamw: flat buffers must be padded to a multiple of 8");
  chk(p, at::kFloat, n, "p");
  chk(g, at::kBFloat16, n, "g");
  chk(m, at::kFloat, n, "m");
  chk(v, at::kFloat, n, "v");
  chk(w16, at::kBFloat16, n, "w16");
  for (const Tensor* s : {&lr, &step, &sumsq})
    TORCH_CHECK(s->is_cuda() && s->scalar_type() == at::kFloat && s->numel() == 1, "adamw scalars must be fp32[1]");
  ok(T_::adamw(p.data_ptr<float>(), bp(g), m.data_ptr<float>(), v.data_ptr<float>(), bp(w16), n, lr.data_ptr<float>(),
               step.data_ptr<float>(), (float)b1, (float)b2, (float)eps, (float)wd, sumsq.data_ptr<float>(),
               (float)max_norm, stream()),
     "adamw");
}

void reduce_rows(const Tensor& part, const Tensor& out) {
  const int64_t n = out.numel();
  TORCH_CHECK(n > 0 && n % 4 == 0 && part.numel() % n == 0, "reduce_rows: part must be [R, n], n % 4 == 0");
  chk(part, at::kFloat, part.numel(), "part");
  chk(out, at::kBFloat16, n, "out");
  ok(T_::reduce_rows(part.data_ptr<float>(), (int)(part.numel() / n), n, bp(out), stream()), "reduce_rows");
}

void colsum(const Tensor& x, const Tensor& out) {
  TORCH_CHECK(x.dim() == 2, "colsum: x must be [M, N]");
  const int64_t M = x.size(0), N = x.size(1);
  TORCH_CHECK(N % 8 == 0 && M > 0 && M < (1ll << 31), "colsum: N % 8 == 0");
  chk(x, at::kBFloat16, M * N, "x");
  chk(out, at::kBFloat16, N, "out");
  auto part = at::empty({T_::colsum_chunks((int)M, (int)N), N}, x.options().dtype(at::kFloat));
  ok(T_::colsum(bp(x), (int)M, (int)N, part.data_ptr<float>(), bp(out), stream()), "colsum");
}

void check_attn(int64_t B, int64_t Tn, int64_t H) {
  TORCH_CHECK(B > 0 && H > 0 && Tn > 0 && Tn % 128 == 0, "attention: T must be a positive multiple of 128");
  TORCH_CHECK(B * Tn * 3 * H * 64 < (1ll << 31), "attention: tensor too large for 32-bit row indexing");
}

void attn_fwd(const Tensor& qkv, const Tensor& o, const Tensor& lse, int64_t B, int64_t Tn, int64_t H,
              double sm_scale) {
  check_attn(B, Tn, H);
  chk(qkv, at::kBFloat16, B * Tn * 3 * H * 64, "qkv");
  chk(o, at::kBFloat16, B * Tn * H * 64, "o");
  chk(lse, at::kFloat, B * H * Tn, "lse");
  ok(T_::attn_fwd(bp(qkv), bp(o), lse.data_ptr<float>(), (int)B, (int)Tn, (int)H, (float)sm_scale, stream()),
     "attn_fwd");
}

void attn_bwd(const Tensor& qkv, const Tensor& o, const Tensor& dout, const Tensor& lse, const Tensor& delta,
              const Tensor& dqkv, int64_t B, int64_t Tn, int64_t H, double sm_scale) {
  check_attn(B, Tn, H);
  chk(qkv, at::kBFloat16, B * Tn * 3 * H * 64, "qkv");
  chk(o, at::kBFloat16, B * Tn * H * 64, "o");
  chk(dout, at::kBFloat16, B * Tn * H * 64, "dout");
  chk(lse, at::kFloat, B * H * Tn, "lse");
  chk(delta, at::kFloat, B * H * Tn, "delta");
  chk(dqkv, at::kBFloat16, B * Tn * 3 * H * 64, "dqkv");
  ok(T_::attn_bwd(bp(qkv), bp(o), bp(dout), lse.data_ptr<float>(), delta.data_ptr<float>(), bp(dqkv), (int)B,
                  (int)Tn, (int)H, (float)sm_scale, stream()),
     "attn_bwd");
}

// C[M][N] = A[M][K] . W[N][K]^T (+ bias[N]); G given: C = pre-activation, G = gelu_tanh(C)
void gemm_nt(const Tensor& A, const Tensor& W, const c10::optional<Tensor>& bias, const Tensor& C,
             const c10::optional<Tensor>& G) {
  TORCH_CHECK(A.dim() == 2 && W.dim() == 2 && C.dim() == 2, "gemm_nt: 2-D operands");
  const int64_t M = A.size(0), K = A.size(1), N = W.size(0);
  TORCH_CHECK(W.size(1) == K && C.size(0) == M && C.size(1) == N, "gemm_nt: shapes");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm_nt: dims");
  TORCH_CHECK(katib_hip::gemm::supported((int)M, (int)N, (int)K), "gemm_nt: M, N % 128 and K % 64 required");
  chk(A, at::kBFloat16, M * K, "A");
  chk(W, at::kBFloat16, N * K, "W");
  chk(C, at::kBFloat16, M * N, "C");
  const void* bp_ = nullptr;
  if (bias.has_value() && bias->defined()) {
    chk(*bias, at::kBFloat16, N, "bias");
    bp_ = bias->data_ptr();
  }
  void* gp = nullptr;
  if (G.has_value() && G->defined()) {
    chk(*G, at::kBFloat16, M * N, "G");
    gp = G->data_ptr();
  }
  ok(katib_hip::gemm::launch_nt(A.data_ptr(), W.data_ptr(), bp_, C.data_ptr(), gp, (int)M, (int)N, (int)K, stream()),
     "gemm_nt");
}

// C = op(A) op(B) on the layout-native MFMA kernel (gemm_bf16.hip gemm_lt_kernel): a_mn: A stored
// [K][M] (else [M][K]); b_mn: B stored [K][N] (else [N][K]). C: bf16 [M][N] (splitk 1, optional
// bias) or fp32 [splitk][M][N] slabs (one per K slice, summed by the caller).
void gemm_lt(const Tensor& A, bool a_mn, const Tensor& B, bool b_mn, const c10::optional<Tensor>& bias,
             const Tensor& C, int64_t splitk, const c10::optional<Tensor>& gelu_u,
             const c10::optional<Tensor>& colpart) {
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gemm_lt: 2-D operands");
  const int64_t M = a_mn ? A.size(1) : A.size(0), K = a_mn ? A.size(0) : A.size(1);
  const int64_t N = b_mn ? B.size(1) : B.size(0), KB = b_mn ? B.size(0) : B.size(1);
  TORCH_CHECK(KB == K, "gemm_lt: inner dimensions differ");
  TORCH_CHECK(M % 128 == 0 && N % 128 == 0 && splitk >= 1 && K % (64 * splitk) == 0,
              "gemm_lt: M, N % 128 and K % (64 splitk) required");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm_lt: dims");
  chk(A, at::kBFloat16, M * K, "A");
  chk(B, at::kBFloat16, N * K, "B");
  const bool f32 = C.scalar_type() == at::kFloat;
  if (f32) chk(C, at::kFloat, splitk * M * N, "C");
  else {
    TORCH_CHECK(splitk == 1, "gemm_lt: a bf16 output needs splitk 1");
    chk(C, at::kBFloat16, M * N, "C");
  }
  const void* bp_ = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(!f32, "gemm_lt: bias only with a bf16 output");
    chk(*bias, at::kBFloat16, N, "bias");
    bp_ = bias->data_ptr();
  }
  const void* gu = nullptr;
  if (gelu_u.has_value() && gelu_u->defined()) {
    TORCH_CHECK(!f32, "gemm_lt: the GELU-backward epilogue needs a bf16 output");
    chk(*gelu_u, at::kBFloat16, M * N, "gelu_u");
    gu = gelu_u->data_ptr();
  }
  float* cp = nullptr;
  if (colpart.has_value() && colpart->defined()) {
    TORCH_CHECK(!f32, "gemm_lt: column partial sums need a bf16 output");
    chk(*colpart, at::kFloat, (M / 64) * N, "colpart");
    cp = colpart->data_ptr<float>();
  }
  ok(katib_hip::gemm::launch_lt(A.data_ptr(), (int)A.size(1), a_mn, B.data_ptr(), (int)B.size(1), b_mn, bp_,
                                C.data_ptr(), f32, (int)splitk, (int)M, (int)N, (int)K, stream(), gu, cp),
     "gemm_lt");
}

// C = op(A) op(B) on the 256 x 256-tile 8-wave ping-pong kernel (gemm256.hip): operand layouts as
// gemm_lt; bf16 C (+ bias) with G = gelu_tanh(C) when G is given, or fp32 [splitk][M][N] slabs.
void gemm256(const Tensor& A, bool a_mn, const Tensor& B, bool b_mn, const c10::optional<Tensor>& bias,
             const Tensor& C, const c10::optional<Tensor>& G, int64_t splitk) {
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "gemm256: 2-D operands");
  const int64_t M = a_mn ? A.size(1) : A.size(0), K = a_mn ? A.size(0) : A.size(1);
  const int64_t N = b_mn ? B.size(1) : B.size(0), KB = b_mn ? B.size(0) : B.size(1);
  TORCH_CHECK(KB == K, "gemm256: inner dimensions differ");
  TORCH_CHECK(M < (1 << 30) && N < (1 << 30) && K < (1 << 30), "gemm256: dims");
  TORCH_CHECK(katib_hip::gemm::supported256((int)M, (int)N, (int)K, (int)splitk),
              "gemm256: M, N % 128 and K % (64 splitk) required");
  chk(A, at::kBFloat16, M * K, "A");
  chk(B, at::kBFloat16, N * K, "B");
  const bool f32 = C.scalar_type() == at::kFloat;
  if (f32) chk(C, at::kFloat, splitk * M * N, "C");
  else {
    TORCH_CHECK(splitk == 1, "gemm256: a bf16 output needs splitk 1");
    chk(C, at::kBFloat16, M * N, "C");
  }
  const void* bp_ = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(!f32, "gemm256: bias only with a bf16 output");
    chk(*bias, at::kBFloat16, N, "bias");
    bp_ = bias->data_ptr();
  }
  void* gp = nullptr;
  if (G.has_value() && G->defined()) {
    TORCH_CHECK(!f32, "gemm256: the GELU output needs a bf16 C");
    chk(*G, at::kBFloat16, M * N, "G");
    gp = G->data_ptr();
  }
  ok(katib_hip::gemm::launch_g256(A.data_ptr(), (int)A.size(1), a_mn, B.data_ptr(), (int)B.size(1), b_mn, bp_,
                                  C.data_ptr(), gp, f32, (int)splitk, (int)M, (int)N, (int)K, stream()),
     "gemm256");
}

}  // namespace

void register_transformer(py::module& m) {
  m.def("gemm256", &gemm256, "C = op(A) op(B), 256^2 tile 8-wave ping-pong (bias / GELU / split-K fp32 slabs)",
        py::arg("A"), py::arg("a_mn"), py::arg("B"), py::arg("b_mn"), py::arg("bias"), py::arg("C"),
        py::arg("G") = py::none(), py::arg("splitk") = 1);
  m.def("gemm256_ablate", [](const Tensor& A, const Tensor& B, const Tensor& C, int64_t variant) {
    ok(katib_hip::gemm::launch_g256_ablate(A.data_ptr(), B.data_ptr(), C.data_ptr(), (int)A.size(0), (int)B.size(0),
                                           (int)A.size(1), (int)variant, stream()), "gemm256_ablate");
  }, "measurement only: gemm256 NT with parts of the K loop removed (wrong results)");
  m.def("gemm256_supported", [](int64_t M, int64_t N, int64_t K, int64_t splitk) {
    return M < (1 << 30) && N < (1 << 30) && K < (1 << 30) && katib_hip::gemm::supported256((int)M, (int)N, (int)K, (int)splitk);
  }, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("splitk") = 1);
  m.def("gemm_lt", &gemm_lt, "bf16 C = op(A) op(B), layout-native operands (NN / TN / NT), split-K fp32 slabs",
        py::arg("A"), py::arg("a_mn"), py::arg("B"), py::arg("b_mn"), py::arg("bias"), py::arg("C"),
        py::arg("splitk") = 1, py::arg("gelu_u") = py::none(), py::arg("colpart") = py::none());
  m.def("gemm_nt", &gemm_nt, "bf16 C = A W^T (+ bias) (+ GELU) on MFMA (gemm_bf16.hip)", py::arg("A"), py::arg("W"),
        py::arg("bias"), py::arg("C"), py::arg("G"));
  m.def("gemm_nt_supported", [](int64_t M, int64_t N, int64_t K) {
    return M < (1 << 30) && N < (1 << 30) && K < (1 << 30) && katib_hip::gemm::supported((int)M, (int)N, (int)K);
  });
  m.def("ln_fwd", &ln_fwd, "residual add + LayerNorm forward (fp32 stream, bf16 out)");
  m.def("ln_bwd", &ln_bwd, "LayerNorm backward (+ residual grad), per-block dgamma/dbeta (+ dr column-sum) partials",
        py::arg("dy"), py::arg("xin"), py::arg("mean"), py::arg("rstd"), py::arg("gamma"), py::arg("dres"),
        py::arg("dx"), py::arg("dr"), py::arg("part_g"), py::arg("part_b"), py::arg("part_r") = py::none());
  m.def("ln_bwd_blocks", &ln_bwd_blocks);
  m.def("ln_reduce", &ln_reduce, "sum LayerNorm parameter-gradient partials into bf16 grads (+ a bias gradient)",
        py::arg("part_g"), py::arg("part_b"), py::arg("dgamma"), py::arg("dbeta"), py::arg("part_r") = py::none(),
        py::arg("dbias") = py::none());
  m.def("xent_eval", &xent_eval, "per-row cross-entropy loss + top-1 hit in one pass over bf16 logits");
  m.def("gelu_fwd", &gelu_fwd);
  m.def("gelu_bwd", &gelu_bwd);
  m.def("xent_fwd", &xent_fwd, "vocabulary cross-entropy forward (per-row loss and lse)");
  m.def("xent_bwd", &xent_bwd, "cross-entropy backward, in place over the logits");
  m.def("xent_fused", &xent_fused,
        "training cross-entropy in one pass over the logits: per-row loss / lse + the gradient in place "
        "(False: row too wide, use xent_fwd + xent_bwd)");
  m.def("grad_sumsq", &grad_sumsq);
  m.def("adamw", &adamw, "flat AdamW with global-norm clip, writes bf16 shadow weights");
  m.def("reduce_rows", &reduce_rows, "bf16 out = sum of fp32 partial rows (split-K reduction)");
  m.def("colsum", &colsum, "bf16 column sums of a [M, N] bf16 matrix (bias gradients)");
  m.def("attn_fwd", &attn_fwd, "causal flash attention forward, head dim 64 (MFMA)");
  m.def("attn_bwd", &attn_bwd, "causal flash attention backward (delta, dK/dV, dQ)");
}
