// torch binding of the one-shot xGMI all-reduce workspace (class katib_amd._hipkern.XgmiWorkspace).
//
// Life cycle (driven by katib_amd/parallel/xgmi.py):
//   ws = XgmiWorkspace(device, cap_floats, blocks)   hipMalloc staging [2][cap] + uncached signal page
//   h  = ws.handles()                                 64-byte IPC handles of both allocations
//   ... exchange h between ranks (any process group) ...
//   ws.open(rank, world, [h_0, ..., h_{W-1}], timeout_s)   map every peer's allocations
//   ws.allreduce(x, out, scale)                       on the current HIP stream (graph-capturable)
//   ws.error()                                        non-zero if a wait ever timed out
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "xgmi_allreduce.h"

namespace py = pybind11;
using namespace katib_hip::xgmi;

namespace {

#define XG_CHECK(expr)                                                                  \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    TORCH_CHECK(e_ == hipSuccess, #expr " failed: ", hipGetErrorString(e_));            \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int d) {
    XG_CHECK(hipGetDevice(&prev));
    if (prev != d) XG_CHECK(hipSetDevice(d));
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

class XgmiWorkspace {
 public:
  XgmiWorkspace(int device, int64_t cap, int blocks) : device_(device), cap_((cap + 3) / 4 * 4), blocks_(blocks) {
    TORCH_CHECK(cap_ > 0, "capacity must be positive");
    TORCH_CHECK(blocks_ >= 1 && blocks_ <= kMaxBlocks, "blocks must be in [1, ", kMaxBlocks, "]");
    DeviceGuard g(device_);
    XG_CHECK(hipMalloc(reinterpret_cast<void**>(&buf_), sizeof(float) * 2 * cap_));
    const size_t sbytes = sizeof(uint32_t) * kSigWords;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sbytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      XG_CHECK(hipExtMallocWithFlags(reinterpret_cast<void**>(&sig_), sbytes, hipDeviceMallocFinegrained));
    }
    XG_CHECK(hipMemset(sig_, 0, sbytes));
    XG_CHECK(hipMemset(buf_, 0, sizeof(float) * 2 * cap_));
    XG_CHECK(hipDeviceSynchronize());
  }

  ~XgmiWorkspace() {
    DeviceGuard g(device_);
    for (int p = 0; p < world_; ++p) {
      if (p == rank_) continue;
      if (args_.buf[p]) (void)hipIpcCloseMemHandle(args_.buf[p]);
      if (args_.sig[p]) (void)hipIpcCloseMemHandle(args_.sig[p]);
    }
    if (buf_) (void)hipFree(buf_);
    if (sig_) (void)hipFree(sig_);
  }

  py::bytes handles() const {
    hipIpcMemHandle_t h[2];
    XG_CHECK(hipIpcGetMemHandle(&h[0], buf_));
    XG_CHECK(hipIpcGetMemHandle(&h[1], sig_));
    return py::bytes(reinterpret_cast<const char*>(h), sizeof(h));
  }

  void open(int rank, int world, const std::vector<std::string>& hs, double timeout_s) {
    TORCH_CHECK(world_ == 0, "workspace already opened");
    TORCH_CHECK(world >= 1 && world <= kMaxRanks, "world size must be in [1, ", kMaxRanks, "]");
    TORCH_CHECK(rank >= 0 && rank < world, "bad rank");
    TORCH_CHECK((int)hs.size() == world, "need one handle blob per rank");
    DeviceGuard g(device_);
    rank_ = rank;
    world_ = world;
    for (int p = 0; p < world; ++p) {
      TORCH_CHECK(hs[p].size() == 2 * sizeof(hipIpcMemHandle_t), "bad handle blob from rank ", p);
      if (p == rank) {
        args_.buf[p] = buf_;
        args_.sig[p] = sig_;
        continue;
      }
      hipIpcMemHandle_t h[2];
      memcpy(h, hs[p].data(), sizeof(h));
      void* pb = nullptr;
      void* ps = nullptr;
      XG_CHECK(hipIpcOpenMemHandle(&pb, h[0], hipIpcMemLazyEnablePeerAccess));
      XG_CHECK(hipIpcOpenMemHandle(&ps, h[1], hipIpcMemLazyEnablePeerAccess));
      args_.buf[p] = static_cast<float*>(pb);
      args_.sig[p] = static_cast<uint32_t*>(ps);
    }
    args_.cap = cap_;
    args_.rank = rank;
    args_.world = world;
    args_.timeout_ticks = (uint64_t)(timeout_s * 1e8);  // 100 MHz constant clock
  }

  // out = scale * sum over ranks of x (out may alias x)
  void allreduce(const at::Tensor& x, const at::Tensor& out, double scale) {
    TORCH_CHECK(world_ > 0, "workspace not opened");
    TORCH_CHECK(x.is_cuda() && out.is_cuda() && x.get_device() == device_ && out.get_device() == device_,
                "tensors must live on the workspace's device");
    TORCH_CHECK(x.scalar_type() == at::kFloat && out.scalar_type() == at::kFloat, "float32 only");
    TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "tensors must be contiguous");
    TORCH_CHECK(x.numel() == out.numel(), "size mismatch");
    TORCH_CHECK(x.numel() <= cap_, "message larger than the workspace capacity");
    if (x.numel() == 0) return;
    AllReduceArgs a = args_;
    a.in = x.data_ptr<float>();
    a.out = out.data_ptr<float>();
    a.n = x.numel();
    a.scale = (float)scale;
    const bool vec4 = (reinterpret_cast<uintptr_t>(a.in) % 16 == 0) && (reinterpret_cast<uintptr_t>(a.out) % 16 == 0);
    XG_CHECK(launch_oneshot(a, blocks_, vec4, c10::hip::getCurrentHIPStream(device_).stream()));
  }

  // SyncBN: fold_f64 segments (f64 tensor holding kRep replicas, n, rstride[, sync]); segments with
  // sync (default true) are also summed over the ranks
  void fold_sync(std::vector<py::tuple> segs) {
    TORCH_CHECK(world_ > 0, "workspace not opened");
    TORCH_CHECK(!segs.empty() && (int)segs.size() <= 64, "fold_sync: 1..64 segments (one sync-mask bit each)");
    katib_hip::FoldF64Args f{};
    uint64_t mask = 0;
    f.nseg = segs.size();
    for (int k = 0; k < f.nseg; ++k) {
      at::Tensor t = segs[k][0].cast<at::Tensor>();
      const int n = segs[k][1].cast<int>(), rs = segs[k][2].cast<int>();
      TORCH_CHECK(t.is_cuda() && t.get_device() == device_ && t.scalar_type() == at::kDouble && t.is_contiguous(),
                  "fold segment must be a contiguous f64 tensor on the workspace's device");
      TORCH_CHECK(n >= 1 && rs >= n && t.numel() >= (int64_t)(katib_hip::kRep - 1) * rs + n, "fold segment size");
      f.p[k] = t.data_ptr<double>();
      f.n[k] = n;
      f.rstride[k] = rs;
      f.total += n;
      const bool sync = segs[k].size() < 4 || segs[k][3].cast<bool>();
      if (sync) mask |= (1ull << k);
    }
    TORCH_CHECK(f.total <= katib_hip::xgmi::kSmallFold || (int64_t)f.total <= cap_ / 2 - katib_hip::xgmi::kSmallFold,
                "fold_sync: segments exceed the workspace capacity");
    TORCH_CHECK(cap_ / 2 >= 2 * katib_hip::xgmi::kSmallFold, "fold_sync: workspace too small for the small-fold region");
    XG_CHECK(launch_fold_sync(args_, f, mask, blocks_, c10::hip::getCurrentHIPStream(device_).stream()));
  }

  int error() const {
    DeviceGuard g(device_);
    uint32_t e = 0;
    XG_CHECK(hipMemcpy(&e, sig_ + kSigErr, sizeof(e), hipMemcpyDeviceToHost));
    return (int)e;
  }

  void clear_error() {
    DeviceGuard g(device_);
    XG_CHECK(hipMemset(sig_ + kSigErr, 0, sizeof(uint32_t)));
    XG_CHECK(hipDeviceSynchronize());
  }

  int64_t capacity() const { return cap_; }
  int blocks() const { return blocks_; }

 private:
  int device_;
  int64_t cap_;
  int blocks_;
  float* buf_ = nullptr;
  uint32_t* sig_ = nullptr;
  int rank_ = -1, world_ = 0;
  AllReduceArgs args_{};
};

}  // namespace

void register_xgmi(py::module& m) {
  py::class_<XgmiWorkspace>(m, "XgmiWorkspace")
      .def(py::init<int, int64_t, int>(), py::arg("device"), py::arg("capacity"), py::arg("blocks"))
      .def("handles", &XgmiWorkspace::handles)
      .def("open", &XgmiWorkspace::open, py::arg("rank"), py::arg("world"), py::arg("handles"),
           py::arg("timeout_s") = 10.0)
      .def("allreduce", &XgmiWorkspace::allreduce, py::arg("x"), py::arg("out"), py::arg("scale") = 1.0)
      .def("fold_sync", &XgmiWorkspace::fold_sync, "SyncBN: fold f64 replicas, sum synchronised segments over ranks")
      .def("error", &XgmiWorkspace::error)
      .def("clear_error", &XgmiWorkspace::clear_error)
      .def_property_readonly("capacity", &XgmiWorkspace::capacity)
      .def_property_readonly("blocks", &XgmiWorkspace::blocks);
  m.attr("XGMI_MAX_RANKS") = kMaxRanks;
}
