// torch bindings for the DARTS HIP kernels (module katib_amd._hipkern).
// Every entry point validates shapes/dtypes/devices against what the kernel's grid
// and LDS layout assume before launching on the current HIP stream (graph-capture safe:
// no allocation, no synchronisation here).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include "darts_ops.h"

using namespace katib_hip;
using at::Tensor;
using OptT = c10::optional<Tensor>;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

// per-op intermediates (d, z): fp32, or bf16 in the KATIB_DARTS_ZBF16 build (darts_ops.h zt)
constexpr at::ScalarType kZType = kZbf16 ? at::kBFloat16 : at::kFloat;

void check_z(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == kZType, name, " must be ", kZbf16 ? "bfloat16" : "float32",
              " (the per-op intermediates' storage type of this build)");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

zt* zptr(const Tensor& t) { return reinterpret_cast<zt*>(t.data_ptr()); }

template <typename T>
T* ptr_or_null(const OptT& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// bn tuple: (sums: Optional[f64 tensor], rmean, rvar, inv_count, eval, eps, rep, rstride)
BNRef make_bn(const py::tuple& b, int C) {
  BNRef r{};
  TORCH_CHECK(b.size() == 8, "bn tuple has 8 fields");
  OptT sums = b[0].cast<OptT>(), rm = b[1].cast<OptT>(), rv = b[2].cast<OptT>();
  r.rep = b[6].cast<int>();
  r.rstride = b[7].cast<int>();
  TORCH_CHECK(r.rep >= 1 && r.rep <= kRep && r.rstride >= 2 * C, "bn replica layout");
  if (sums.has_value() && sums->defined()) {
    TORCH_CHECK(sums->scalar_type() == at::kDouble && sums->is_contiguous() &&
                    sums->numel() >= (int64_t)(r.rep - 1) * r.rstride + 2 * C,
                "bn sums must be f64 with rep x rstride doubles");
  }
  r.sums = ptr_or_null<double>(sums);
  r.rmean = ptr_or_null<float>(rm);
  r.rvar = ptr_or_null<float>(rv);
  r.inv_count = b[3].cast<float>();
  r.eval = b[4].cast<bool>() ? 1 : 0;
  r.eps = b[5].cast<float>();
  r.C = C;
  TORCH_CHECK(r.eval ? (r.rmean && r.rvar) : (r.sums != nullptr), "bn reference lacks its statistics");
  return r;
}

// grad source tuple: (g, z, S1 (f64 view), S2 (f64 view), bn tuple, w: Optional, widx, rep, rstride)
// replica r of S1/S2 starts r*rstride doubles after the view's first element
int64_t storage_doubles_after(const Tensor& t) {
  return (int64_t)(t.storage().nbytes() / sizeof(double)) - t.storage_offset();
}

int64_t gs_numel(const py::tuple& t) {
  return t[1].cast<Tensor>().numel();  // z, the pre-BN output the gradient is evaluated on
}

GradSrc make_gs(const py::tuple& t, int C) {
  GradSrc g{};
  TORCH_CHECK(t.size() == 9, "grad-source tuple has 9 fields");
  Tensor gt = t[0].cast<Tensor>(), zt = t[1].cast<Tensor>();
  check_f32(gt, "g");
  check_z(zt, "z");
  g.g = gt.data_ptr<float>();
  g.z = zptr(zt);
  OptT s1 = t[2].cast<OptT>(), s2 = t[3].cast<OptT>();
  g.S1 = ptr_or_null<double>(s1);
  g.S2 = ptr_or_null<double>(s2);
  g.bn = make_bn(t[4].cast<py::tuple>(), C);
  g.eval = g.bn.eval;
  TORCH_CHECK(g.eval || (g.S1 && g.S2), "training-mode BN backward needs S1/S2 reductions");
  OptT w = t[5].cast<OptT>();
  g.w = ptr_or_null<float>(w);
  g.widx = t[6].cast<int>();
  g.rep = t[7].cast<int>();
  g.rstride = t[8].cast<int>();
  TORCH_CHECK(g.rep >= 1 && g.rep <= kRep, "replicas");
  if (!g.eval) {
    for (int k = 2; k <= 3; ++k) {
      Tensor sv = *t[k].cast<OptT>();
      TORCH_CHECK(sv.scalar_type() == at::kDouble &&
                      storage_doubles_after(sv) >= (int64_t)(g.rep - 1) * g.rstride + C,
                  "S1/S2 replicas exceed their buffer");
    }
  }
  return g;
}

// ------------------------------------------------------------------------------------------------
// Self-folding launches (darts_ops.h FoldTail): a per-device ring of zeroed arrival counters,
// registered once from Python outside any graph capture (set_fold_counters); every launch that
// produces replicated f64 sums takes the next counter. Off unless set_selffold(true) (the
// Python side then launches fold_f64 as before; selffold_ready() tells it which mode is live).
// ------------------------------------------------------------------------------------------------
struct CtrRing {
  unsigned* base = nullptr;
  int size = 0;
  int cursor = 0;
};
CtrRing g_ring[64];
bool g_selffold = false;  // self-folding launches (set_selffold): measured slower, tests only

void set_selffold(bool on) { g_selffold = on; }

int cur_device() {
  int d = 0;
  TORCH_CHECK(hipGetDevice(&d) == hipSuccess, "hipGetDevice");
  return d;
}

void set_fold_counters(Tensor t) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() >= 4 * kFoldCtrSlot,
              "fold counters: contiguous int32 GPU tensor of >= 4 launch slots");
  const int d = t.get_device();
  TORCH_CHECK(d >= 0 && d < 64, "device index");
  g_ring[d] = CtrRing{reinterpret_cast<unsigned*>(t.data_ptr<int>()), (int)(t.numel() / kFoldCtrSlot), 0};
}

bool selffold_ready() { return g_selffold && g_ring[cur_device()].base != nullptr; }

void tail_begin(FoldTail& t) {
  t.nseg = 0;
  t.ctr = nullptr;
  if (!g_selffold) return;
  CtrRing& r = g_ring[cur_device()];
  if (!r.base) return;
  t.ctr = r.base + (size_t)r.cursor * kFoldCtrSlot;  // size counts launch slots
  r.cursor = (r.cursor + 1) % r.size;
}

void tail_add(FoldTail& t, double* p, int n, int rs) {
  if (!t.ctr || !p) return;
  for (int s = 0; s < t.nseg; ++s)
    if (t.p[s] == p) {
      t.n[s] = std::max(t.n[s], n);
      return;
    }
  TORCH_CHECK(t.nseg < kTailSeg, "self-fold: too many reduction segments in one launch");
  // (a launch with no segment keeps ctr == nullptr: see tail_close)
  t.p[t.nseg] = p;
  t.n[t.nseg] = n;
  t.rs[t.nseg] = rs;
  ++t.nseg;
}

// a launch that ended up with nothing to fold (eval mode: no statistics) skips the epilogue
void tail_close(FoldTail& t) {
  if (t.nseg == 0) t.ctr = nullptr;
}

int pick_chunk(int C, int per_channel_floats, int fixed_floats) {
  // keep dynamic LDS <= 64 KB so several blocks stay resident per CU
  const int budget = 16384 - fixed_floats;
  int ch = C;
  while (ch > 1 && ch * per_channel_floats > budget) ch = (ch + 1) / 2;
  return std::max(ch, 1);
}

// ------------------------------------------------------------------------------------------------
// Edge-batched entry points: `calls` is a list of per-edge argument tuples that share shapes;
// one launch covers all of them (blockIdx.y = edge).
// ------------------------------------------------------------------------------------------------
template <typename Bt>
void check_batch(const std::vector<py::tuple>& calls) {
  TORCH_CHECK(!calls.empty() && (int)calls.size() <= Bt::kCap, "batch of 1..", Bt::kCap, " edges");
}

#define SAME_SHAPE(b, fld) TORCH_CHECK(b.e[i].fld == b.e[0].fld, "edges in a batch must share " #fld)

// one entry of a dw-pw stage: (x, dw, pw, inbn|None, d, z, stats|None); returns whether it has an input BN
static bool fill_dwpw(const py::tuple& t, DwPwFwdArgs& a, int64_t K, int64_t dil, int64_t S, int64_t pad, int nentries,
                      bool use_mfma) {
  Tensor x = t[0].cast<Tensor>(), dw = t[1].cast<Tensor>(), pw = t[2].cast<Tensor>();
  auto inbn = t[3].cast<c10::optional<py::tuple>>();
  Tensor d = t[4].cast<Tensor>(), z = t[5].cast<Tensor>();
  OptT stats = t[6].cast<OptT>();
  const bool has_inbn = t[3].cast<c10::optional<py::tuple>>().has_value();
  if (has_inbn) check_z(x, "x (previous stage z)");
  else check_f32(x, "x");
  check_f32(dw, "dw"); check_f32(pw, "pw"); check_z(d, "d"); check_z(z, "z");
  TORCH_CHECK(x.dim() == 4, "x must be NCHW");
  TORCH_CHECK((K == 3 || K == 5) && (dil == 1 || dil == 2) && (S == 1 || S == 2), "K in {3,5}, dil, S in {1,2}");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int Ho = z.size(2), Wo = z.size(3);
  TORCH_CHECK(dw.numel() == C * K * K && pw.numel() == C * C, "weight shapes");
  TORCH_CHECK(z.size(0) == N && z.size(1) == C && d.sizes() == z.sizes(), "output shapes");
  TORCH_CHECK(64 % Wo == 0 && Ho % (64 / Wo) == 0, "tile constraint: 64 % Wo == 0 and Ho % (64/Wo) == 0");
  TORCH_CHECK(C <= kMaxC, "C too large");
  TORCH_CHECK(Ho == (H + 2 * pad - dil * (K - 1) - 1) / S + 1, "output height mismatch");
  a.x = x.data_ptr(); a.dw = dw.data_ptr<float>(); a.pw = pw.data_ptr<float>();
  a.d = zptr(d); a.z = zptr(z); a.stats = ptr_or_null<double>(stats);
  if (a.stats) TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->numel() >= kRep * 2 * C, "stats f64 [kRep][2C]");
  a.N = N; a.C = C; a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.pad = pad;
  const int TR = 64 / Wo;
  const int IR = (TR - 1) * S + (K - 1) * dil + 1, IW = (Wo - 1) * S + (K - 1) * dil + 1;
  a.chunk = pick_chunk(C, IR * IW, C * 64 + 4 * C);
  if (C == 4 || C == 8 || C == 16) {
    // dwpw_plane: `chunk` = row bands per image, ~2048 workgroups per launch and >= 4
    // output rows per band, capped so the staged band fits 64 KB of LDS
    int nb = std::max(1, std::min(Ho / 4, 2048 / std::max(N * nentries, 1)));
    auto band_bytes = [&](int b) {
      const int BR = (Ho + b - 1) / b;
      return (size_t)C * ((BR - 1) * S + (K - 1) * dil + 1) * (W + 2 * pad) * sizeof(float);
    };
    while (band_bytes(nb) > 65536 && nb < Ho) ++nb;
    a.chunk = nb;
  }
  a.use_mfma = (use_mfma && C % 16 == 0) ? 1 : 0;
  const bool prebn = inbn.has_value();
  if (prebn) a.inbn = make_bn(*inbn, C);
  a.variant = (((K == 5) * 4 + (dil == 2) * 2 + (S == 2)) * 4) + (prebn ? 2 : 0);
  return prebn;
}

// (x, dw, pw, inbn|None, d, z, stats|None)
void dwpw_fwd(std::vector<py::tuple> calls, int64_t K, int64_t dil, int64_t S, int64_t pad, bool use_mfma) {
  check_batch<DwPwFwdBatch>(calls);
  DwPwFwdBatch bt{};
  bt.n = calls.size();
  bool prebn = false;
  for (int i = 0; i < bt.n; ++i) {
    const bool pb = fill_dwpw(calls[i], bt.e[i], K, dil, S, pad, bt.n, use_mfma);
    if (i == 0) prebn = pb;
    TORCH_CHECK(pb == prebn, "edges in a batch must agree on the input BN");
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C); SAME_SHAPE(bt, H); SAME_SHAPE(bt, W);
  }
  tail_begin(bt.tail);
  for (int i = 0; i < bt.n; ++i) tail_add(bt.tail, bt.e[i].stats, 2 * bt.e[i].C, 2 * bt.e[i].C);
  tail_close(bt.tail);
  launch_dwpw_fwd(bt, K, dil, S, prebn, cur_stream());
}

// Mixed (K, dil, S, input-BN) entries of one node stage in one launch:
// (x, dw, pw, inbn|None, d, z, stats|None, K, dil, S, pad) per entry. Entries that do not fit the
// plane kernels (channel counts, alignment) run as per-group launches instead.
static void fill_dwpw_multi(const std::vector<py::tuple>& calls, DwPwMultiBatch& bt, int64_t* kk, int64_t* dd,
                            int64_t* ss, int64_t* pp, bool* pre) {
  TORCH_CHECK(!calls.empty() && (int)calls.size() <= DwPwMultiBatch::kCap, "1..", DwPwMultiBatch::kCap, " entries");
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    TORCH_CHECK(t.size() == 11, "dwpw_fwd_multi entry: (x, dw, pw, inbn, d, z, stats, K, dil, S, pad)");
    kk[i] = t[7].cast<int64_t>(); dd[i] = t[8].cast<int64_t>(); ss[i] = t[9].cast<int64_t>(); pp[i] = t[10].cast<int64_t>();
    pre[i] = fill_dwpw(t, bt.e[i], kk[i], dd[i], ss[i], pp[i], bt.n, true);
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C); SAME_SHAPE(bt, Ho); SAME_SHAPE(bt, Wo);
  }
  tail_begin(bt.tail);
  for (int i = 0; i < bt.n; ++i) tail_add(bt.tail, bt.e[i].stats, 2 * bt.e[i].C, 2 * bt.e[i].C);
  tail_close(bt.tail);
}

void dwpw_fwd_multi(std::vector<py::tuple> calls) {
  DwPwMultiBatch bt{};
  int64_t kk[DwPwMultiBatch::kCap], dd[DwPwMultiBatch::kCap], ss[DwPwMultiBatch::kCap], pp[DwPwMultiBatch::kCap];
  bool pre[DwPwMultiBatch::kCap];
  fill_dwpw_multi(calls, bt, kk, dd, ss, pp, pre);
  if (launch_dwpw_multi(bt, cur_stream())) return;
  for (int i = 0; i < bt.n; ++i) {  // fallback: one launch per entry (the plane path's band count is per batch)
    DwPwFwdBatch one{};
    one.n = 1;
    one.tail = bt.tail;  // sequential launches may share the counter (each re-arms it)
    fill_dwpw(calls[i], one.e[0], kk[i], dd[i], ss[i], pp[i], 1, true);
    launch_dwpw_fwd(one, kk[i], dd[i], ss[i], pre[i], cur_stream());
  }
}

// (x, pw, z, stats|None, co_off, off)
void pw_fwd(std::vector<py::tuple> calls, int64_t S) {
  check_batch<PwFwdBatch>(calls);
  PwFwdBatch bt{};
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    Tensor x = t[0].cast<Tensor>(), pw = t[1].cast<Tensor>(), z = t[2].cast<Tensor>();
    OptT stats = t[3].cast<OptT>();
    const int co_off = t[4].cast<int>(), off = t[5].cast<int>();
    check_f32(x, "x"); check_f32(pw, "pw"); check_z(z, "z");
    // a 5-D x is node-major [nodes][N][C / nodes][H][W] (a DARTS cell output kept as its nodes' buffers)
    const bool nm = x.dim() == 5;
    const int xnodes = nm ? x.size(0) : 1;
    const int N = nm ? x.size(1) : x.size(0), Cin = nm ? x.size(0) * x.size(2) : x.size(1);
    const int H = x.size(nm ? 3 : 2), W = x.size(nm ? 4 : 3);
    const int Cout = pw.size(0), Ho = z.size(2), Wo = z.size(3);
    TORCH_CHECK(pw.size(1) == Cin && co_off + Cout <= z.size(1) && z.size(0) == N, "pw shapes");
    TORCH_CHECK((Ho * Wo) % 64 == 0, "Ho*Wo must be a multiple of 64");
    TORCH_CHECK(Cin <= kMaxC && Cout <= kMaxC, "channels");
    PwFwdArgs& a = bt.e[i];
    a.x = x.data_ptr<float>(); a.pw = pw.data_ptr<float>(); a.z = zptr(z);
    a.stats = ptr_or_null<double>(stats);
    if (a.stats)
      TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->numel() >= kRep * 2 * z.size(1), "stats [kRep][2Ctot]");
    a.N = N; a.Cin = Cin; a.Cout = Cout; a.CoutTotal = z.size(1); a.co_off = co_off;
    a.H = H; a.W = W; a.Ho = Ho; a.Wo = Wo; a.S = S; a.off = off; a.relu = 1; a.xnodes = xnodes;
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, Cin); SAME_SHAPE(bt, Cout); SAME_SHAPE(bt, Ho); SAME_SHAPE(bt, Wo);
  }
  tail_begin(bt.tail);
  for (int i = 0; i < bt.n; ++i) tail_add(bt.tail, bt.e[i].stats, 2 * bt.e[i].CoutTotal, 2 * bt.e[i].CoutTotal);
  tail_close(bt.tail);
  launch_pw_fwd(bt, cur_stream());
}

// (x, zavg, zmax, stats_avg|None, stats_max|None, amax|None[, S]); S < 0: per-entry S (7th field)
static void fill_pool_fwd(const std::vector<py::tuple>& calls, int64_t S_all, PoolFwdBatch& bt) {
  check_batch<PoolFwdBatch>(calls);
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    const int64_t S = S_all > 0 ? S_all : t[6].cast<int64_t>();
    TORCH_CHECK(S == 1 || S == 2, "pool stride must be 1 or 2");
    bt.e[i].S = (int)S;
    Tensor x = t[0].cast<Tensor>(), zavg = t[1].cast<Tensor>(), zmax = t[2].cast<Tensor>();
    OptT sa = t[3].cast<OptT>(), sm = t[4].cast<OptT>(), amax = t[5].cast<OptT>();
    check_f32(x, "x"); check_z(zavg, "zavg"); check_z(zmax, "zmax");
    PoolFwdArgs& a = bt.e[i];
    if (amax.has_value() && amax->defined()) {
      TORCH_CHECK(amax->scalar_type() == at::kByte && amax->numel() == zmax.numel(), "amax must be uint8 like zmax");
      a.amax = amax->data_ptr<uint8_t>();
    }
    a.x = x.data_ptr<float>(); a.zavg = zptr(zavg); a.zmax = zptr(zmax);
    a.stats_avg = ptr_or_null<double>(sa); a.stats_max = ptr_or_null<double>(sm);
    if (a.stats_avg) TORCH_CHECK(sa->scalar_type() == at::kDouble && sa->numel() >= kRep * 2 * x.size(1), "stats");
    if (a.stats_max) TORCH_CHECK(sm->scalar_type() == at::kDouble && sm->numel() >= kRep * 2 * x.size(1), "stats");
    a.N = x.size(0); a.C = x.size(1); a.H = x.size(2); a.W = x.size(3); a.Ho = zavg.size(2); a.Wo = zavg.size(3);
    TORCH_CHECK(a.Ho == (a.H - 1) / S + 1 && zmax.sizes() == zavg.sizes(), "pool shapes");
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C);
    if (S_all > 0) { SAME_SHAPE(bt, H); SAME_SHAPE(bt, W); }
  }
  tail_begin(bt.tail);
  for (int i = 0; i < bt.n; ++i) {
    tail_add(bt.tail, bt.e[i].stats_avg, 2 * bt.e[i].C, 2 * bt.e[i].C);
    tail_add(bt.tail, bt.e[i].stats_max, 2 * bt.e[i].C, 2 * bt.e[i].C);
  }
  tail_close(bt.tail);
}

static void pool_fwd_impl(std::vector<py::tuple> calls, int64_t S_all) {
  PoolFwdBatch bt{};
  fill_pool_fwd(calls, S_all, bt);
  if (S_all > 0) launch_pool_fwd(bt, S_all, cur_stream());
  else launch_pool_fwd_multi(bt, cur_stream());
}

void pool_fwd(std::vector<py::tuple> calls, int64_t S) { pool_fwd_impl(calls, S); }
// stride-1 and stride-2 pools of a node in one launch: (..., amax|None, S) per entry
void pool_fwd_multi(std::vector<py::tuple> calls) { pool_fwd_impl(calls, -1); }

// a node's stage-1 dw-pw entries and its pools (both read only the node inputs) in ONE launch
// when the fused narrow-layer plane path applies; otherwise the two launches above
void dwpw_pool_fwd_multi(std::vector<py::tuple> dcalls, std::vector<py::tuple> pcalls) {
  DwPwMultiBatch bt{};
  int64_t kk[DwPwMultiBatch::kCap], dd[DwPwMultiBatch::kCap], ss[DwPwMultiBatch::kCap], pp[DwPwMultiBatch::kCap];
  bool pre[DwPwMultiBatch::kCap];
  fill_dwpw_multi(dcalls, bt, kk, dd, ss, pp, pre);
  PoolFwdBatch pb{};
  fill_pool_fwd(pcalls, -1, pb);
  if (launch_dwpw_pool_multi(bt, pb, cur_stream())) return;
  dwpw_fwd_multi(dcalls);
  launch_pool_fwd_multi(pb, cur_stream());
}

// calls: per edge (zs, bns, widx, w|None, id_idx, xid|None, upd); all edges summed into `out`
void combine_fwd(std::vector<py::tuple> calls, OptT gamma, OptT beta, Tensor out, double momentum,
                 bool update_running, bool accumulate) {
  check_f32(out, "out");
  check_batch<CombineFwdBatch>(calls);
  CombineFwdBatch bt{};
  bt.n = calls.size();
  const int C = out.size(1);
  TORCH_CHECK(C <= kMaxC, "C too large");
  TORCH_CHECK((int64_t)2 * bt.n * kMaxOps * C * 4 <= 65536, "combine LDS budget exceeded");
  for (int e = 0; e < bt.n; ++e) {
    const py::tuple& t = calls[e];
    auto zs = t[0].cast<std::vector<Tensor>>();
    auto bns = t[1].cast<std::vector<py::tuple>>();
    auto widx = t[2].cast<std::vector<int64_t>>();
    OptT w = t[3].cast<OptT>();
    const int id_idx = t[4].cast<int>();
    OptT xid = t[5].cast<OptT>();
    auto upd = t[6].cast<std::vector<py::tuple>>();
    TORCH_CHECK(zs.size() == bns.size() && zs.size() == widx.size() && (int)zs.size() <= kMaxOps, "ops");
    CombineFwdArgs& a = bt.e[e];
    a.N = out.size(0); a.C = C; a.HW = out.size(2) * out.size(3);
    a.nops = zs.size();
    for (size_t k = 0; k < zs.size(); ++k) {
      check_z(zs[k], "z");
      TORCH_CHECK(zs[k].sizes() == out.sizes(), "combine input shape");
      a.z[k] = zptr(zs[k]);
      a.bn[k] = make_bn(bns[k], C);
      a.widx[k] = widx[k];
    }
    TORCH_CHECK((int)upd.size() <= kMaxUpd, "too many update-only BN layers");
    a.nupd = upd.size();
    for (size_t k = 0; k < upd.size(); ++k) a.upd[k] = make_bn(upd[k], C);
    a.w = ptr_or_null<float>(w); a.id_idx = id_idx; a.xid = ptr_or_null<float>(xid);
    if (a.xid) {
      check_f32(*xid, "xid");
      TORCH_CHECK(xid->sizes() == out.sizes(), "identity shape");
    }
    a.gamma = ptr_or_null<float>(gamma); a.beta = ptr_or_null<float>(beta);
    a.out = out.data_ptr<float>(); a.momentum = momentum; a.update_running = update_running;
    a.accumulate = accumulate;
  }
  launch_combine_fwd(bt, cur_stream());
}

// (dout, zs, bns, xid|None, red, widx, id_idx, gw|None)
void combine_bwd_reduce(std::vector<py::tuple> calls) {
  check_batch<CombineBwdBatch>(calls);
  CombineBwdBatch bt{};
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    Tensor dout = t[0].cast<Tensor>();
    auto zs = t[1].cast<std::vector<Tensor>>();
    auto bns = t[2].cast<std::vector<py::tuple>>();
    OptT xid = t[3].cast<OptT>();
    Tensor red = t[4].cast<Tensor>();
    auto widx = t[5].cast<std::vector<int64_t>>();
    const int id_idx = t[6].cast<int>();
    OptT gw = t[7].cast<OptT>();
    check_f32(dout, "dout");
    TORCH_CHECK(red.scalar_type() == at::kDouble, "red must be f64");
    CombineBwdArgs& a = bt.e[i];
    a.N = dout.size(0); a.C = dout.size(1); a.HW = dout.size(2) * dout.size(3);
    a.nops = zs.size();
    a.rstride = (a.nops + 1) * a.C + 1;
    TORCH_CHECK(a.nops <= kMaxOps && red.numel() >= (int64_t)kRep * a.rstride, "red size [kRep][(nops+1)C+1]");
    for (int k = 0; k < a.nops; ++k) {
      TORCH_CHECK(zs[k].sizes() == dout.sizes(), "z shape");
      check_z(zs[k], "z");
      a.z[k] = zptr(zs[k]);
      a.bn[k] = make_bn(bns[k], a.C);
    }
    a.dout = dout.data_ptr<float>(); a.xid = ptr_or_null<float>(xid); a.red = red.data_ptr<double>();
    a.gw = ptr_or_null<double>(gw); a.id_idx = id_idx;
    if (a.gw) {
      TORCH_CHECK(gw->scalar_type() == at::kDouble && gw->numel() % kRep == 0, "gw must be f64 [kRep][nw]");
      a.gwstride = gw->numel() / kRep;
      TORCH_CHECK((int)widx.size() == a.nops, "widx per op");
      for (int k = 0; k < a.nops; ++k) {
        TORCH_CHECK(widx[k] >= 0 && widx[k] < a.gwstride, "widx out of range");
        a.widx[k] = widx[k];
      }
      TORCH_CHECK(id_idx < a.gwstride, "id_idx out of range");
    }
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C); SAME_SHAPE(bt, HW);
  }
  tail_begin(bt.tail);
  for (int i = 0; i < bt.n; ++i) {
    tail_add(bt.tail, bt.e[i].red, bt.e[i].rstride, bt.e[i].rstride);
    tail_add(bt.tail, bt.e[i].gw, bt.e[i].gwstride, bt.e[i].gwstride);
  }
  tail_close(bt.tail);
  launch_combine_bwd_reduce(bt, cur_stream());
}

// gW replica r lives gstride floats after replica 0 (gstride == 0: one accumulator)
void check_grad_sink(const OptT& gW, int64_t numel, int64_t gstride) {
  if (!gW.has_value() || !gW->defined()) return;
  TORCH_CHECK(gW->scalar_type() == at::kFloat && gW->is_contiguous() && gW->numel() == numel, "gW shape");
  TORCH_CHECK(gstride == 0 || (gstride >= numel && (int64_t)(gW->storage().nbytes() / sizeof(float)) -
                                                           gW->storage_offset() >= (kRep - 1) * gstride + numel),
              "gW replicas exceed their buffer");
}

// (gs, pw, ain|None, x, dd|None, gx|None, gW|None, co_off, off, gstride)
void pw_bwd(std::vector<py::tuple> calls, int64_t S, int64_t mode, bool need_dx) {
  check_batch<PwBwdBatch>(calls);
  PwBwdBatch bt{};
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    py::tuple gs = t[0].cast<py::tuple>();
    Tensor pw = t[1].cast<Tensor>();
    OptT ain = t[2].cast<OptT>();
    Tensor x = t[3].cast<Tensor>();
    OptT dd = t[4].cast<OptT>(), gx = t[5].cast<OptT>(), gW = t[6].cast<OptT>();
    const int co_off = t[7].cast<int>(), off = t[8].cast<int>();
    const int64_t gstride = t[9].cast<int64_t>();
    const bool overwrite = t.size() > 10 && t[10].cast<bool>();
    check_f32(pw, "pw");
    if (mode != 0) check_f32(x, "x");  // mode 0 reads only the shape of x (the stage input, maybe a zt z)
    PwBwdArgs& a = bt.e[i];
    a.overwrite = overwrite;
    TORCH_CHECK(!overwrite || (mode == 1 && S == 1 && off == 0), "gx overwrite needs the stride-1 full-coverage form");
    const int Cout = pw.size(0), Cin = pw.size(1);
    Tensor g = gs[0].cast<Tensor>();
    a.N = g.size(0); a.CoutTotal = g.size(1); a.Ho = g.size(2); a.Wo = g.size(3);
    a.gs = make_gs(gs, a.CoutTotal);
    a.Cin = Cin; a.Cout = Cout; a.co_off = co_off; a.S = S; a.off = off; a.mode = mode;
    a.need_dx = need_dx;
    // mode 1 with a 5-D x: node-major [nodes][N][Cin / nodes][H][W] input and input gradient
    const bool nm = mode != 0 && x.dim() == 5;
    a.xnodes = nm ? x.size(0) : 1;
    a.H = x.size(nm ? 3 : 2); a.W = x.size(nm ? 4 : 3);
    if (mode != 0) {
      TORCH_CHECK(x.numel() == (int64_t)a.N * Cin * a.H * a.W && (!nm || x.size(1) == a.N),
                  "pw_bwd: x must be [N][Cin][H][W] or node-major [nodes][N][Cin/nodes][H][W]");
      if (gx.has_value() && gx->defined()) TORCH_CHECK(gx->sizes() == x.sizes(), "pw_bwd: gx must have the shape of x");
    }
    TORCH_CHECK(Cin * Cout <= 8192, "pw_bwd supports Cin*Cout <= 8192");
    TORCH_CHECK((a.Ho * a.Wo) % 64 == 0, "Ho*Wo % 64");
    a.pw = pw.data_ptr<float>(); a.x = mode != 0 ? x.data_ptr<float>() : nullptr;
    if (ain.has_value() && ain->defined()) check_z(*ain, "ain (depthwise output d)");
    a.ain = ain.has_value() && ain->defined() ? zptr(*ain) : nullptr;
    a.dd = ptr_or_null<float>(dd); a.gx = ptr_or_null<float>(gx);
    a.gW = ptr_or_null<float>(gW);
    if (mode == 0) {
      TORCH_CHECK(a.ain && (!need_dx || a.dd), "mode 0 needs ain (and dd)");
    } else {
      TORCH_CHECK(!need_dx || a.gx, "mode 1 needs gx");
    }
    check_grad_sink(gW, (int64_t)Cin * Cout, gstride);
    a.gstride = gstride;
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, Cin); SAME_SHAPE(bt, Cout); SAME_SHAPE(bt, Ho); SAME_SHAPE(bt, Wo);
  }
  launch_pw_bwd(bt, cur_stream());
}

// (x, inbn|None, dw, dd, gout, gW|None, red|None, gstride, overwrite)
void dw_bwd_fill(std::vector<py::tuple>& calls, DwBwdBatch& bt, const int64_t* Ks, const int64_t* dils,
                 const int64_t* Ss, bool& prebn);

void dw_bwd(std::vector<py::tuple> calls, int64_t K, int64_t dil, int64_t S, int64_t pad) {
  check_batch<DwBwdBatch>(calls);
  DwBwdBatch bt{};
  int64_t Ks[DwBwdBatch::kCap], Ds[DwBwdBatch::kCap], Ss[DwBwdBatch::kCap];
  for (int i = 0; i < DwBwdBatch::kCap; ++i) Ks[i] = K, Ds[i] = dil, Ss[i] = S;
  TORCH_CHECK(pad == (K - 1) / 2 * dil, "dw_bwd padding must be 'same'");
  bool prebn = false;
  dw_bwd_fill(calls, bt, Ks, Ds, Ss, prebn);
  tail_close(bt.tail);
  launch_dw_bwd(bt, K, dil, S, prebn, cur_stream());
}

// Depthwise backward entries of mixed kernel size / dilation / stride that write DISTINCT outputs,
// in one launch: (x, inbn, dw, dd, gout, gW|None, red|None, gstride, overwrite, K[, dil, S]) -
// a node's separable second stages (input BN), or its stage-1 separable and dilated convolutions
// each writing its own input-gradient buffer (overwrite). One launch when the plane kernel fits,
// else one launch per (K, dil, S) group.
void dw_bwd_multi(std::vector<py::tuple> calls) {
  check_batch<DwBwdBatch>(calls);
  DwBwdBatch bt{};
  int64_t Ks[DwBwdBatch::kCap], Ds[DwBwdBatch::kCap], Ss[DwBwdBatch::kCap];
  for (size_t i = 0; i < calls.size(); ++i) {
    TORCH_CHECK(calls[i].size() == 10 || calls[i].size() == 12,
                "dw_bwd_multi entry: (x, inbn, dw, dd, gout, gW, red, gstride, overwrite, K[, dil, S])");
    Ks[i] = calls[i][9].cast<int64_t>();
    Ds[i] = calls[i].size() == 12 ? calls[i][10].cast<int64_t>() : 1;
    Ss[i] = calls[i].size() == 12 ? calls[i][11].cast<int64_t>() : 1;
    TORCH_CHECK((Ks[i] == 3 || Ks[i] == 5) && (Ds[i] == 1 || Ds[i] == 2) && (Ss[i] == 1 || Ss[i] == 2),
                "K in {3, 5}, dil and S in {1, 2}");
  }
  bool prebn = false;
  dw_bwd_fill(calls, bt, Ks, Ds, Ss, prebn);
  for (int i = 0; i < bt.n; ++i) {
    TORCH_CHECK(prebn || bt.e[i].overwrite, "dw_bwd_multi: input-gradient entries must own (overwrite) their output");
    TORCH_CHECK(!prebn || (Ds[i] == 1 && Ss[i] == 1), "dw_bwd_multi: input-BN entries are stride-1 separable stages");
    bt.e[i].variant = dw_bwd_variant((int)Ks[i], (int)Ds[i], (int)Ss[i], prebn);
  }
  for (int i = 0; i < bt.n; ++i)  // no ordering between entries: distinct outputs
    for (int j = i + 1; j < bt.n; ++j) TORCH_CHECK(bt.e[i].gout != bt.e[j].gout, "dw_bwd_multi entries share an output");
  tail_close(bt.tail);
  if (launch_dw_bwd_multi(bt, cur_stream())) return;
  for (int v = 0; v < 16; ++v) {  // fallback: per variant, sharing the counter (sequential launches)
    DwBwdBatch one{};
    one.tail = bt.tail;
    for (int i = 0; i < bt.n; ++i)
      if (bt.e[i].variant == v) one.e[one.n++] = bt.e[i];
    if (one.n) launch_dw_bwd(one, dw_variant_k(v), dw_variant_dil(v), dw_variant_s(v), prebn, cur_stream());
  }
}

void dw_bwd_fill(std::vector<py::tuple>& calls, DwBwdBatch& bt, const int64_t* Ks, const int64_t* dils,
                 const int64_t* Ss, bool& prebn) {
  bt.n = calls.size();
  bool has_gw = false;
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    const int64_t K = Ks[i], dil = dils[i], S = Ss[i], pad = (K - 1) / 2 * dil;
    Tensor x = t[0].cast<Tensor>();
    auto inbn = t[1].cast<c10::optional<py::tuple>>();
    Tensor dw = t[2].cast<Tensor>(), dd = t[3].cast<Tensor>(), gout = t[4].cast<Tensor>();
    OptT gW = t[5].cast<OptT>(), red = t[6].cast<OptT>();
    const int64_t gstride = t[7].cast<int64_t>();
    const bool overwrite = t[8].cast<bool>();
    if (inbn.has_value()) check_z(x, "x (stage-1 z)");
    else check_f32(x, "x");
    check_f32(dw, "dw"); check_f32(dd, "dd"); check_f32(gout, "gout");
    DwBwdArgs& a = bt.e[i];
    a.N = x.size(0); a.C = x.size(1); a.H = x.size(2); a.W = x.size(3); a.Ho = dd.size(2); a.Wo = dd.size(3);
    TORCH_CHECK(64 % a.Wo == 0 && a.Ho % (64 / a.Wo) == 0, "tile constraint");
    TORCH_CHECK(a.H == a.Ho * S && a.W == a.Wo * S, "dw_bwd needs H == Ho*S");
    TORCH_CHECK(gout.sizes() == x.sizes(), "gout shape");
    TORCH_CHECK(dw.numel() == a.C * K * K && dd.size(1) == a.C, "dw_bwd weight / grad shapes");
    a.x = x.data_ptr(); a.dw = dw.data_ptr<float>(); a.dd = dd.data_ptr<float>();
    a.gout = gout.data_ptr<float>(); a.gW = ptr_or_null<float>(gW); a.red = ptr_or_null<double>(red);
    check_grad_sink(gW, (int64_t)a.C * K * K, gstride);
    a.gstride = gstride;
    a.overwrite = overwrite;
    if (a.red) TORCH_CHECK(red->scalar_type() == at::kDouble && red->numel() >= kRep * 2 * a.C, "red [kRep][2C]");
    a.pad = pad;
    if (i == 0) {
      prebn = inbn.has_value();
      has_gw = a.gW != nullptr;
    }
    TORCH_CHECK(inbn.has_value() == prebn, "edges in a batch must agree on the input BN");
    TORCH_CHECK((a.gW != nullptr) == has_gw, "edges in a batch must agree on weight-gradient sinks");
    TORCH_CHECK(!(prebn && overwrite), "overwrite applies to the input-gradient (non-BN) form");
    const int TR = 64 / a.Wo, r = (K - 1) / 2 * dil, h = (r + S - 1) / S, OR = TR + 2 * h;
    const int IR = (TR - 1) * S + (K - 1) * dil + 1, IW = (a.Wo - 1) * S + (K - 1) * dil + 1;
    a.chunk = pick_chunk(a.C, OR * a.Wo + IR * IW, 4 * a.C + (a.gW ? a.C * (int)(K * K) : 0));
    if (prebn) a.inbn = make_bn(*inbn, a.C);
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C); SAME_SHAPE(bt, Ho); SAME_SHAPE(bt, Wo);
  }
  tail_begin(bt.tail);
  if (prebn)
    for (int i = 0; i < bt.n; ++i) tail_add(bt.tail, bt.e[i].red, 2 * bt.e[i].C, 2 * bt.e[i].C);
}

// (ga|None, gm|None, x, dout_id|None, w|None, id_idx, gx, amax|None, overwrite[, S]); S < 0: per entry
static void pool_bwd_impl(std::vector<py::tuple> calls, int64_t S_all) {
  check_batch<PoolBwdBatch>(calls);
  PoolBwdBatch bt{};
  bt.n = calls.size();
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    const int64_t S = S_all > 0 ? S_all : t[9].cast<int64_t>();
    TORCH_CHECK(S == 1 || S == 2, "pool stride must be 1 or 2");
    bt.e[i].S = (int)S;
    auto ga = t[0].cast<c10::optional<py::tuple>>(), gm = t[1].cast<c10::optional<py::tuple>>();
    Tensor x = t[2].cast<Tensor>();
    OptT dout_id = t[3].cast<OptT>(), w = t[4].cast<OptT>();
    const int id_idx = t[5].cast<int>();
    Tensor gx = t[6].cast<Tensor>();
    OptT amax = t[7].cast<OptT>();
    check_f32(x, "x"); check_f32(gx, "gx");
    PoolBwdArgs& a = bt.e[i];
    a.N = x.size(0); a.C = x.size(1); a.H = x.size(2); a.W = x.size(3);
    a.Ho = (a.H - 1) / S + 1; a.Wo = (a.W - 1) / S + 1;
    TORCH_CHECK(a.Ho * a.Wo <= 8192, "pool_bwd stages one output plane in LDS (Ho*Wo <= 8192)");
    TORCH_CHECK(gx.sizes() == x.sizes(), "gx shape");
    TORCH_CHECK(!gm.has_value() || (amax.has_value() && amax->defined() && amax->scalar_type() == at::kByte &&
                                    amax->numel() == (int64_t)a.N * a.C * a.Ho * a.Wo),
                "max-pool backward needs the uint8 argmax from pool_fwd");
    if (amax.has_value() && amax->defined()) a.amax = amax->data_ptr<uint8_t>();
    if (ga.has_value()) a.ga = make_gs(*ga, a.C);
    if (gm.has_value()) a.gm = make_gs(*gm, a.C);
    a.x = x.data_ptr<float>(); a.dout_id = ptr_or_null<float>(dout_id); a.w = ptr_or_null<float>(w);
    if (a.dout_id) TORCH_CHECK(dout_id->sizes() == x.sizes(), "identity gradient shape");
    a.id_idx = id_idx; a.gx = gx.data_ptr<float>();
    a.overwrite = t[8].cast<bool>();
    if (S_all <= 0 && t.size() > 10) {  // (..., S, extras): other input-gradient parts to sum in
      auto ex = t[10].cast<std::vector<Tensor>>();
      TORCH_CHECK(ex.size() <= 4, "pool_bwd: at most 4 extra gradient parts");
      a.nextra = ex.size();
      for (size_t j = 0; j < ex.size(); ++j) {
        check_f32(ex[j], "extra");
        TORCH_CHECK(ex[j].sizes() == gx.sizes(), "extra gradient part shape");
        TORCH_CHECK(ex[j].data_ptr() != gx.data_ptr(), "extra part aliases gx");
        a.extra[j] = ex[j].data_ptr<float>();
      }
    }
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C);
    if (S_all > 0) { SAME_SHAPE(bt, H); SAME_SHAPE(bt, W); }
  }
  // entries of one launch must write distinct input gradients (no ordering between them)
  for (int i = 0; i < bt.n; ++i)
    for (int j = i + 1; j < bt.n; ++j) TORCH_CHECK(bt.e[i].gx != bt.e[j].gx, "pool_bwd entries share a gx buffer");
  if (S_all > 0) launch_pool_bwd(bt, S_all, cur_stream());
  else launch_pool_bwd_multi(bt, cur_stream());
}

void pool_bwd(std::vector<py::tuple> calls, int64_t S) { pool_bwd_impl(calls, S); }

// Whole input gradient of up to 4 edges of one node (distinct gx buffers), one launch:
// per edge (x, gx, overwrite, convs, ga|None, gm|None, amax|None, dout_id|None, w|None, id_idx, S);
// convs = 4 slots (sep 3x3, sep 5x5, dil 3x3, dil 5x5), each None or (dw, dd, gW|None, gstride).
// Returns false (nothing launched) when the shapes fall outside the fused kernel.
bool edge_bwd(std::vector<py::tuple> calls) {
  check_batch<EdgeBwdBatch>(calls);
  EdgeBwdBatch bt{};
  bt.n = calls.size();
  const int Ks[4] = {3, 5, 3, 5};
  for (int i = 0; i < bt.n; ++i) {
    const py::tuple& t = calls[i];
    TORCH_CHECK(t.size() == 11, "edge_bwd entry: (x, gx, overwrite, convs, ga, gm, amax, dout_id, w, id_idx, S)");
    Tensor x = t[0].cast<Tensor>(), gx = t[1].cast<Tensor>();
    check_f32(x, "x"); check_f32(gx, "gx");
    TORCH_CHECK(x.dim() == 4 && gx.sizes() == x.sizes(), "gx shape");
    EdgeBwdArgs& a = bt.e[i];
    a.x = x.data_ptr<float>(); a.gx = gx.data_ptr<float>(); a.overwrite = t[2].cast<bool>();
    a.S = t[10].cast<int>();
    TORCH_CHECK(a.S == 1 || a.S == 2, "stride");
    a.N = x.size(0); a.C = x.size(1); a.H = x.size(2); a.W = x.size(3);
    a.Ho = (a.H - 1) / a.S + 1; a.Wo = (a.W - 1) / a.S + 1;
    auto convs = t[3].cast<std::vector<py::object>>();
    TORCH_CHECK(convs.size() == 4, "4 conv slots");
    for (int v = 0; v < 4; ++v) {
      if (convs[v].is_none()) continue;
      py::tuple c = convs[v].cast<py::tuple>();
      Tensor dw = c[0].cast<Tensor>(), dd = c[1].cast<Tensor>();
      OptT gW = c[2].cast<OptT>();
      const int64_t gstride = c[3].cast<int64_t>();
      check_f32(dw, "dw"); check_f32(dd, "dd");
      TORCH_CHECK(dw.numel() == a.C * Ks[v] * Ks[v], "dw shape");
      TORCH_CHECK(dd.dim() == 4 && dd.size(0) == a.N && dd.size(1) == a.C && dd.size(2) == a.Ho && dd.size(3) == a.Wo,
                  "dd shape");
      check_grad_sink(gW, (int64_t)a.C * Ks[v] * Ks[v], gstride);
      a.dw[v] = dw.data_ptr<float>(); a.dd[v] = dd.data_ptr<float>(); a.gW[v] = ptr_or_null<float>(gW);
      a.gstride[v] = gstride;
      a.conv_mask |= 1 << v;
    }
    auto ga = t[4].cast<c10::optional<py::tuple>>(), gm = t[5].cast<c10::optional<py::tuple>>();
    OptT amax = t[6].cast<OptT>(), dout_id = t[7].cast<OptT>(), w = t[8].cast<OptT>();
    if (ga.has_value()) {
      a.ga = make_gs(*ga, a.C);
      TORCH_CHECK(gs_numel(*ga) == (int64_t)a.N * a.C * a.Ho * a.Wo, "avg-pool gradient source shape");
    }
    if (gm.has_value()) {
      a.gm = make_gs(*gm, a.C);
      TORCH_CHECK(gs_numel(*gm) == (int64_t)a.N * a.C * a.Ho * a.Wo, "max-pool gradient source shape");
      TORCH_CHECK(amax.has_value() && amax->defined() && amax->scalar_type() == at::kByte &&
                      amax->numel() == (int64_t)a.N * a.C * a.Ho * a.Wo,
                  "max-pool backward needs the uint8 argmax from pool_fwd");
      a.amax = amax->data_ptr<uint8_t>();
    }
    a.dout_id = ptr_or_null<float>(dout_id); a.w = ptr_or_null<float>(w); a.id_idx = t[9].cast<int>();
    if (a.dout_id) {
      check_f32(*dout_id, "dout_id");
      TORCH_CHECK(dout_id->sizes() == x.sizes() && a.S == 1, "identity gradient shape");
    }
    SAME_SHAPE(bt, N); SAME_SHAPE(bt, C);
  }
  for (int i = 0; i < bt.n; ++i)
    for (int j = i + 1; j < bt.n; ++j) TORCH_CHECK(bt.e[i].gx != bt.e[j].gx, "edge_bwd entries share a gx buffer");
  return launch_edge_bwd(bt, cur_stream());
}
void pool_bwd_multi(std::vector<py::tuple> calls) { pool_bwd_impl(calls, -1); }

void fold_rows(Tensor buf) {
  check_f32(buf, "buf");
  TORCH_CHECK(buf.dim() == 2, "buf must be [rows][n]");
  FoldArgs a{};
  a.buf = buf.data_ptr<float>();
  a.rows = buf.size(0);
  a.n = buf.size(1);
  launch_fold_rows(a, cur_stream());
}

// segments: (f64 tensor holding kRep replicas, n, rstride)
void fold_f64(std::vector<py::tuple> segs) {
  TORCH_CHECK(!segs.empty() && (int)segs.size() <= kMaxSeg, "1..kMaxSeg segments");
  FoldF64Args a{};
  a.nseg = segs.size();
  for (int k = 0; k < a.nseg; ++k) {
    Tensor t = segs[k][0].cast<Tensor>();
    int n = segs[k][1].cast<int>(), rs = segs[k][2].cast<int>();
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kDouble && t.is_contiguous(), "fold segment must be f64");
    TORCH_CHECK(n >= 1 && rs >= n && t.numel() >= (int64_t)(kRep - 1) * rs + n, "fold segment size");
    a.p[k] = t.data_ptr<double>();
    a.n[k] = n;
    a.rstride[k] = rs;
    a.total += n;
  }
  launch_fold_f64(a, cur_stream());
}

}  // namespace

void register_xgmi(py::module& m);  // xgmi_bind.cpp
void register_conv(py::module& m);  // conv_bind.cpp
void register_transformer(py::module& m);  // transformer_bind.cpp
void register_batchnorm(py::module& m);  // batchnorm_bind.cpp
void register_mlp(py::module& m);  // mlp_bind.cpp
void register_stem(py::module& m);  // stem_bind.cpp
void register_enas(py::module& m);  // enas_bind.cpp
void register_dwconv(py::module& m);  // dwconv_bind.cpp
void register_darts_optim(py::module& m);  // darts_optim_bind.cpp
void register_darts_head(py::module& m);  // darts_head_bind.cpp
void register_resnet(py::module& m);  // resnet_bind.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "katib_amd HIP kernels for gfx950 (DARTS edge ops, implicit-GEMM conv, transformer, xGMI all-reduce)";
  m.def("dwpw_fwd", &dwpw_fwd);
  m.def("pw_fwd", &pw_fwd);
  m.def("pool_fwd", &pool_fwd);
  m.def("combine_fwd", &combine_fwd);
  m.def("combine_bwd_reduce", &combine_bwd_reduce);
  m.def("pw_bwd", &pw_bwd);
  m.def("dw_bwd", &dw_bwd);
  m.def("dw_bwd_multi", &dw_bwd_multi, "separable second-stage depthwise backward of mixed kernel size in one launch");
  m.def("pool_bwd", &pool_bwd);
  m.def("dwpw_fwd_multi", &dwpw_fwd_multi, "mixed (K, dil, S) dw-pw entries of one node stage in one launch");
  m.def("pool_fwd_multi", &pool_fwd_multi, "stride-1 and stride-2 pools in one launch");
  m.def("dwpw_pool_fwd_multi", &dwpw_pool_fwd_multi, "a node's stage-1 dw-pw entries and its pools in one launch");
  m.def("pool_bwd_multi", &pool_bwd_multi, "stride-1 and stride-2 pool backward in one launch");
  m.def("edge_bwd", &edge_bwd, "whole input gradient of a node's edges (convs, pools, identity) in one launch");
  m.def("set_max_blocks", &set_max_blocks);
  m.def("stamps_arm", [](int kind, int call, torch::Tensor buf) {
    TORCH_CHECK(!buf.defined() || kind == 0 || (buf.is_cuda() && buf.scalar_type() == torch::kInt64 &&
                                               buf.is_contiguous() && buf.numel() >= 65536 * 8),
                "stamps_arm: int64 CUDA buffer of >= 65536 * 8 entries");
    stamps_arm(kind, call, kind == 0 ? nullptr : reinterpret_cast<unsigned long long*>(buf.data_ptr<int64_t>()));
  }, "diagnostic build: phase-stamp the call-th launch of kind (StampKind) into buf[wg * 8 + phase]");
  m.def("stamps_compiled", &stamps_compiled);
  m.def("fold_rows", &fold_rows);
  m.def("fold_f64", &fold_f64);
  m.def("set_fold_counters", &set_fold_counters, "register the current device's self-fold counter ring (int32, zeroed)");
  m.def("selffold_ready", &selffold_ready, "launches on the current device fold their own f64 replicas");
  m.def("set_selffold", &set_selffold, "turn self-folding launches on / off (default off: measured slower)");
  m.attr("REP") = kRep;
  m.attr("ZBF16") = kZbf16;  // per-op intermediates stored as bf16 (the _hipkern_zbf16 variant)
  m.def("max_blocks", &max_blocks);
  register_xgmi(m);
  register_conv(m);
  register_transformer(m);
  register_batchnorm(m);
  register_enas(m);
  register_dwconv(m);
  register_mlp(m);
  register_stem(m);
  register_darts_optim(m);
  register_darts_head(m);
  register_resnet(m);
}
