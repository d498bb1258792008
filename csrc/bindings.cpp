// Python bindings: mlapi_amd._C
//
// Kernels take raw device pointers (ints) + a hipStream_t (int), so torch tensors are passed as
// tensor.data_ptr() / torch.cuda.current_stream().cuda_stream without linking libtorch.
// Blocking calls release the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <cmath>
#include <mutex>

#include "dist/comm.h"
#include "dist/p2p.h"
#include "http/loadgen.h"
#include "http/json_body.h"
#include "http/server.h"
#include "http/dispatch.h"
#include "mlapi/common.h"
#include "mlapi/kernels.h"
#include "runtime/engine.h"
#include "runtime/float_repr.h"
#include "runtime/split_merge.h"

namespace py = pybind11;
using namespace mlapi;

namespace {

template <typename T>
T* ptr(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// Completion sink for Python/asyncio: the engine's completer thread appends and signals an
// eventfd; Python watches the fd (loop.add_reader) and drains.
class PySink : public Sink {
 public:
  PySink() {
    fd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (fd_ < 0) throw std::runtime_error("eventfd failed");
  }
  ~PySink() override { close(fd_); }
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>& m) override {
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (size_t i = 0; i < n; ++i) {
        items_.push_back(c[i]);
        versions_.push_back(m ? m->version : 0);
      }
    }
    const uint64_t one = 1;
    ssize_t r = write(fd_, &one, sizeof one);
    (void)r;
  }
  int fd() const { return fd_; }
  py::list drain() {
    std::vector<Completion> items;
    std::vector<uint64_t> vers;
    {
      uint64_t v;
      ssize_t r = read(fd_, &v, sizeof v);
      (void)r;
      std::lock_guard<std::mutex> lk(mu_);
      items.swap(items_);
      vers.swap(versions_);
    }
    py::list out;
    for (size_t i = 0; i < items.size(); ++i)
      out.append(py::make_tuple(items[i].tag, items[i].idx, items[i].status, items[i].p, items[i].latency_ns,
                                vers[i]));
    return out;
  }

 private:
  int fd_;
  std::mutex mu_;
  std::vector<Completion> items_;
  std::vector<uint64_t> versions_;
};

py::dict stats_dict(const EngineStats& s) {
  py::dict d;
  d["requests"] = s.requests;
  d["batches"] = s.batches;
  d["errors"] = s.errors;
  py::list bh, lh;
  for (auto v : s.batch_hist) bh.append(v);
  for (auto v : s.latency_hist) lh.append(v);
  d["batch_hist"] = bh;
  d["latency_hist_us_pow2"] = lh;
  d["latency_sum_us"] = s.latency_sum_us;
  d["device_us_sum"] = s.device_us_sum;
  d["queue_wait_us_sum"] = s.queue_wait_us_sum;
  {
    py::dict bn, cn;
    const char* bs[4] = {"take", "slot", "launch", "book"};
    for (int i = 0; i < 4; ++i) bn[bs[i]] = s.batcher_ns[i];
    cn["wait_gpu"] = s.completer_ns[0];
    cn["deliver"] = s.completer_ns[1];
    d["batcher_ns"] = bn;
    py::dict ln;
    const char* ls[3] = {"pack", "flush", "kernel"};
    for (int i = 0; i < 3; ++i) ln[ls[i]] = s.launch_ns[i];
    d["launch_ns"] = ln;
    d["completer_ns"] = cn;
  }
  d["queue_depth"] = s.queue_depth;
  d["model_version"] = s.model_version;
  d["healthy"] = s.healthy;
  d["dropped"] = s.dropped;
  d["rejected"] = s.rejected;
  py::dict paths;
  static const char* names[PATH_COUNT] = {"small", "gemv", "gemm", "generic", "wide"};
  for (int i = 0; i < PATH_COUNT; ++i) paths[names[i]] = s.path_batches[i];
  d["path_batches"] = paths;
  d["inline_batches"] = s.inline_batches;
  d["direct_batches"] = s.direct_batches;
  d["direct_wide_batches"] = s.direct_wide_batches;
  d["idle_batches"] = s.idle_batches;
  d["resident_rows"] = s.resident_rows;
  d["resident_stale"] = s.resident_stale;
  d["resident_launches"] = s.resident_launches;
  d["resident_hb_restarts"] = s.resident_hb_restarts;
  d["resident_ring_restarts"] = s.resident_ring_restarts;
  d["resident_self_exits"] = s.resident_self_exits;
  d["resident_queue_faults"] = s.resident_queue_faults;
  d["resident_abandoned"] = s.resident_abandoned;
  d["resident_heartbeat"] = s.resident_heartbeat;
  d["resident_rings"] = s.resident_rings;
  d["resident_live"] = s.resident_live;
  d["generic_models"] = s.generic_models;
  d["xcd_errors"] = s.xcd_errors;
  d["bar_batches"] = s.bar_batches;
  d["direct_dispatch"] = s.direct_dispatch;
  d["direct_device_kernargs"] = s.direct_device_kernargs;
  return d;
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "mlapi_amd native runtime: gfx950 HIP kernels, batching engine, HTTP server, load generator";

  m.attr("KIND_BINARY") = (int)KIND_BINARY;
  m.attr("KIND_BINARY_SOFTMAX") = (int)KIND_BINARY_SOFTMAX;
  m.attr("KIND_MULTINOMIAL") = (int)KIND_MULTINOMIAL;
  m.attr("KIND_OVR") = (int)KIND_OVR;
  m.attr("DT_F64") = (int)DT_F64;
  m.attr("DT_F32") = (int)DT_F32;
  m.attr("DT_BF16") = (int)DT_BF16;

  m.def("device_count", [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("py_float_repr", [](double v) {
    std::string s;
    if (!append_py_float(s, v)) throw std::invalid_argument("non-finite");
    return s;
  });
  m.def("parse_predict_body", [](const std::string& body, const std::vector<std::string>& names) -> py::object {
    std::vector<double> out(names.size());
    if (!parse_predict_body(body.data(), body.size(), names, out.data())) return py::none();
    return py::cast(out);
  });

  // ---------------------------------------------------------------- kernels
  m.def(
      "linear_small",
      [](int dt, uintptr_t X, int64_t ldx, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind,
         uintptr_t out_idx, uintptr_t out_p, uintptr_t stream) {
        launch_linear_small(dt, ptr<void>(X), ldx, ptr<void>(W), ptr<void>(b), B, F, K, kind, ptr<int32_t>(out_idx),
                            ptr<void>(out_p), stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("ldx"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("out_idx"), py::arg("out_p"), py::arg("stream") = 0);
  m.def(
      "gemv_binary",
      [](int dt, uintptr_t X, uintptr_t w, float bias, int64_t B, int F, int kind, uintptr_t out_idx,
         uintptr_t out_p, uintptr_t stream) {
        launch_gemv_binary(dt, ptr<void>(X), ptr<void>(w), bias, B, F, kind, ptr<int32_t>(out_idx),
                           ptr<float>(out_p), stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("w"), py::arg("bias"), py::arg("B"), py::arg("F"), py::arg("kind"),
      py::arg("out_idx"), py::arg("out_p"), py::arg("stream") = 0);
  m.def("gemm_softmax_workspace", &gemm_softmax_workspace);
  m.def("gemm_softmax_plan", [](int64_t B, int K, int F) {
    int64_t o[5];
    gemm_softmax_plan_info(B, K, F, o);
    static const char* kernels[] = {"tiles", "t32", "rows"};
    py::dict d;
    d["kernel"] = kernels[o[0]];
    d["nt"] = o[1];
    d["splits"] = o[2];
    d["classes_per_split"] = o[3];
    d["row_blocks"] = o[4];
    return d;
  });
  m.def("gemm_softmax_set_rows_g2", &gemm_softmax_set_rows_g2, py::arg("on"));
  m.def("gemm_softmax_set_w_packed", &gemm_softmax_set_w_packed, py::arg("on"));
  m.def("gemm_softmax_force_plan", &gemm_softmax_force_plan, py::arg("nt") = 0, py::arg("splits") = 0,
        py::arg("kernel") = 0);
  m.def("gemm_softmax_set_stamps", [](uintptr_t p) { gemm_softmax_set_stamps(reinterpret_cast<void*>(p)); });
  m.def(
      "gemm_softmax",
      [](uintptr_t X, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind, uintptr_t out_idx,
         uintptr_t out_p, uintptr_t ws, size_t ws_bytes, uintptr_t stream) {
        launch_gemm_softmax(ptr<void>(X), ptr<void>(W), ptr<float>(b), B, F, K, kind, ptr<int32_t>(out_idx),
                            ptr<float>(out_p), ptr<void>(ws), ws_bytes, stream_of(stream));
      },
      py::arg("X"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"), py::arg("K"), py::arg("kind"),
      py::arg("out_idx"), py::arg("out_p"), py::arg("ws"), py::arg("ws_bytes"), py::arg("stream") = 0);
  m.def(
      "linear_wide_plan",
      [](int dt, int F, int K) {
        const WidePlan p = linear_wide_plan(dt, F, K);
        py::dict d;
        d["ncb"] = p.ncb;
        d["nfs"] = p.nfs;
        d["ldx"] = p.ldx;
        d["fsteps"] = p.fsteps;
        return d;
      },
      py::arg("dt"), py::arg("F"), py::arg("K"));
  m.def("linear_wide_set_probe", &linear_wide_set_probe, py::arg("probe"));
  m.def("linear_wide_set_trace", [](uintptr_t p) { linear_wide_set_trace(reinterpret_cast<void*>(p)); },
        py::arg("data_ptr"));
  m.def("linear_wide_workspace", &linear_wide_workspace, py::arg("B"), py::arg("dt"), py::arg("F"), py::arg("K"));
  m.def(
      "linear_wide",
      [](int dt, uintptr_t X, int64_t ldx, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind,
         uintptr_t out_idx, uintptr_t out_p, uintptr_t ws, size_t ws_bytes, uintptr_t stream) {
        launch_linear_wide(dt, ptr<void>(X), ldx, ptr<void>(W), ptr<double>(b), B, F, K, kind, ptr<int32_t>(out_idx),
                           ptr<double>(out_p), ptr<void>(ws), ws_bytes, stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("ldx"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("out_idx"), py::arg("out_p"), py::arg("ws"), py::arg("ws_bytes"),
      py::arg("stream") = 0);
  m.def("linear_split_supported", &linear_split_supported);
  m.def("linear_split_workspace", &linear_split_workspace);
  m.def("linear_split_xcd_err_offset", &linear_split_xcd_err_offset);
  m.def("linear_split_set_xcd", &linear_split_set_xcd);
  m.def("gemm_softmax_xcd_err_offset", &gemm_softmax_xcd_err_offset);
  m.def("xcd_placement_state", &xcd_placement_state, py::arg("device") = 0);
  m.def("xcd_placement_mismatches", &xcd_placement_mismatches, py::arg("device") = 0);
  m.def("xcd_local_errors", &xcd_local_errors, py::arg("device") = 0);
  m.def("xcd_local_inject", &xcd_local_inject, py::arg("launches"));
  m.def("xcd_local_reset", &xcd_local_reset, py::arg("device") = 0);
  m.def(
      "linear_split",
      [](int dt, uintptr_t X, int64_t ldx, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind,
         uintptr_t out_idx, uintptr_t out_p, uintptr_t ws, size_t ws_bytes, uintptr_t stream) {
        launch_linear_split(dt, ptr<void>(X), ldx, ptr<void>(W), ptr<float>(b), B, F, K, kind, ptr<int32_t>(out_idx),
                            ptr<float>(out_p), ptr<void>(ws), ws_bytes, stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("ldx"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("out_idx"), py::arg("out_p"), py::arg("ws"), py::arg("ws_bytes"),
      py::arg("stream") = 0);
  m.def(
      "gemm_logits",
      [](uintptr_t X, uintptr_t W, uintptr_t b, int64_t B, int F, int K, uintptr_t Z, uintptr_t stream) {
        launch_gemm_logits(ptr<void>(X), ptr<void>(W), ptr<float>(b), B, F, K, ptr<float>(Z), stream_of(stream));
      },
      py::arg("X"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"), py::arg("K"), py::arg("Z"),
      py::arg("stream") = 0);
  m.def(
      "gemm_rowstate",
      [](uintptr_t X, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind, uintptr_t out, uintptr_t ws,
         size_t ws_bytes, uintptr_t stream) {
        launch_gemm_rowstate(ptr<void>(X), ptr<void>(W), ptr<float>(b), B, F, K, kind, ptr<void>(out), ptr<void>(ws),
                             ws_bytes, stream_of(stream));
      },
      py::arg("X"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"), py::arg("K"), py::arg("kind"),
      py::arg("out"), py::arg("ws"), py::arg("ws_bytes"), py::arg("stream") = 0);
  m.def(
      "merge_split_records",
      [](const std::vector<int32_t>& bi, const std::vector<float>& m, const std::vector<float>& sm, bool ovr) {
        // one row's per-block states in block order -> (label, p): the completer's host merge
        const size_t ns = bi.size();
        if (ns == 0 || ns > 64 || m.size() != ns || sm.size() != ns)
          throw std::invalid_argument("merge_split_records: 1..64 blocks, equal lengths");
        SplitRecord r[64];
        for (size_t k = 0; k < ns; ++k) r[k] = SplitRecord{0u, bi[k], m[k], sm[k]};
        int32_t label = 0;
        const double p = merge_split_records(r, (int)ns, ovr, &label);
        return py::make_tuple(label, p);
      },
      py::arg("argmax"), py::arg("max"), py::arg("sum"), py::arg("ovr"));
  m.def(
      "merge_rowstates",
      [](uintptr_t parts, int nparts, int64_t B, std::vector<int> offsets, int kind, uintptr_t out_idx,
         uintptr_t out_p, uintptr_t stream) {
        if ((int)offsets.size() != nparts) throw std::invalid_argument("merge_rowstates: one offset per shard");
        if (nparts < 1 || nparts > ShardOffsets::MAX) throw std::invalid_argument("merge_rowstates: 1..64 shards");
        ShardOffsets o{};
        for (int i = 0; i < nparts; ++i) o.off[i] = offsets[i];
        launch_merge_rowstates(ptr<void>(parts), nparts, B, o, kind, ptr<int32_t>(out_idx), ptr<float>(out_p),
                               stream_of(stream));
      },
      py::arg("parts"), py::arg("nparts"), py::arg("B"), py::arg("offsets"), py::arg("kind"), py::arg("out_idx"),
      py::arg("out_p"), py::arg("stream") = 0);
  m.def(
      "logits_epilogue",
      [](uintptr_t Z, uintptr_t b, int64_t B, int K, int kind, uintptr_t out_idx, uintptr_t out_p, uintptr_t stream) {
        launch_logits_epilogue(ptr<float>(Z), ptr<float>(b), B, K, kind, ptr<int32_t>(out_idx), ptr<float>(out_p),
                               stream_of(stream));
      },
      py::arg("Z"), py::arg("b"), py::arg("B"), py::arg("K"), py::arg("kind"), py::arg("out_idx"), py::arg("out_p"),
      py::arg("stream") = 0);
  m.def("train_binary_workspace", &train_binary_workspace);
  m.def("train_binary_set_max_blocks", &train_binary_set_max_blocks, py::arg("n") = 0);
  m.def(
      "train_binary_grad",
      [](int dt, uintptr_t X, uintptr_t y, uintptr_t w, uintptr_t b, int64_t B, int F, uintptr_t out, uintptr_t ws,
         size_t ws_bytes, uintptr_t stream) {
        launch_train_binary_grad(dt, ptr<void>(X), ptr<float>(y), ptr<float>(w), 0.f, ptr<float>(b), B, F,
                                 ptr<float>(out), ptr<void>(ws), ws_bytes, stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("y"), py::arg("w"), py::arg("b"), py::arg("B"), py::arg("F"),
      py::arg("out"), py::arg("ws"), py::arg("ws_bytes"), py::arg("stream") = 0);
  m.def(
      "train_binary_step",
      [](int dt, uintptr_t X, uintptr_t y, uintptr_t params, uintptr_t mom, int64_t B, int F, uintptr_t grad_out,
         uintptr_t ws, size_t ws_bytes, float lr, float inv_n, float l2, float momentum, uintptr_t stream,
         P2PAllReduce* p2p, int timeout_ms) {
        launch_train_binary_step(dt, ptr<void>(X), ptr<float>(y), ptr<float>(params), ptr<float>(mom), B, F,
                                 ptr<float>(grad_out), ptr<void>(ws), ws_bytes, lr, inv_n, l2, momentum,
                                 stream_of(stream), p2p, timeout_ms);
      },
      py::arg("dt"), py::arg("X"), py::arg("y"), py::arg("params"), py::arg("mom"), py::arg("B"), py::arg("F"),
      py::arg("grad_out"), py::arg("ws"), py::arg("ws_bytes"), py::arg("lr"), py::arg("inv_n"), py::arg("l2"),
      py::arg("momentum"), py::arg("stream") = 0, py::arg("p2p") = nullptr, py::arg("timeout_ms") = 60000);
  m.def("train_small_workspace", &train_small_workspace);
  m.def(
      "train_small_grad",
      [](int dt, uintptr_t X, uintptr_t y, uintptr_t W, uintptr_t b, int64_t B, int F, int K, int kind,
         uintptr_t out, uintptr_t ws, size_t ws_bytes, uintptr_t stream) {
        launch_train_small_grad(dt, ptr<void>(X), ptr<int32_t>(y), ptr<void>(W), ptr<void>(b), B, F, K, kind,
                                ptr<void>(out), ptr<void>(ws), ws_bytes, stream_of(stream));
      },
      py::arg("dt"), py::arg("X"), py::arg("y"), py::arg("W"), py::arg("b"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("out"), py::arg("ws"), py::arg("ws_bytes"), py::arg("stream") = 0);
  m.def(
      "sgd_update",
      [](uintptr_t params, uintptr_t grad, uintptr_t mom, int64_t n, int64_t n_pen, float lr, float inv_n, float l2,
         float momentum, uintptr_t stream) {
        launch_sgd_update(ptr<float>(params), ptr<float>(grad), ptr<float>(mom), n, n_pen, lr, inv_n, l2, momentum,
                          stream_of(stream));
      },
      py::arg("params"), py::arg("grad"), py::arg("mom"), py::arg("n"), py::arg("n_pen"), py::arg("lr"),
      py::arg("inv_n"), py::arg("l2"), py::arg("momentum"), py::arg("stream") = 0);
  m.def("softmax_grad_dw_supported", &softmax_grad_dw_supported);
  m.def("softmax_grad_dw_force_plan", &softmax_grad_dw_force_plan, py::arg("row_groups") = 0, py::arg("nc") = 0);
  m.def("softmax_grad_dw_workspace", &softmax_grad_dw_workspace);
  m.def(
      "softmax_grad_dw",
      [](uintptr_t X_aug, int64_t ldx, uintptr_t W, uintptr_t b, uintptr_t y, int64_t B, int F, int K, int kind,
         uintptr_t dW_out, uintptr_t stats_out, uintptr_t ws, size_t ws_bytes, uintptr_t stream, uintptr_t params,
         uintptr_t mom, uintptr_t shadow_w, uintptr_t shadow_b, int pen_cols, float lr, float inv_n, float l2,
         float momentum, P2PAllReduce* p2p, int timeout_ms) {
        Sgd2D u;
        u.params = ptr<float>(params);
        u.mom = ptr<float>(mom);
        u.shadow_w = ptr<uint16_t>(shadow_w);
        u.shadow_b = ptr<float>(shadow_b);
        u.cols = F + 8;
        u.pen_cols = pen_cols;
        u.lr = lr;
        u.inv_n = inv_n;
        u.l2 = l2;
        u.momentum = momentum;
        launch_softmax_grad_dw(ptr<void>(X_aug), ldx, ptr<void>(W), ptr<float>(b), ptr<int32_t>(y), B, F, K, kind,
                               ptr<float>(dW_out), ptr<float>(stats_out), ptr<void>(ws), ws_bytes, stream_of(stream),
                               params != 0 ? &u : nullptr, p2p, timeout_ms);
      },
      py::arg("X_aug"), py::arg("ldx"), py::arg("W"), py::arg("b"), py::arg("y"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("dW_out"), py::arg("stats_out"), py::arg("ws"), py::arg("ws_bytes"),
      py::arg("stream") = 0, py::arg("params") = 0, py::arg("mom") = 0, py::arg("shadow_w") = 0,
      py::arg("shadow_b") = 0, py::arg("pen_cols") = 0, py::arg("lr") = 0.f, py::arg("inv_n") = 0.f,
      py::arg("l2") = 0.f, py::arg("momentum") = 0.f, py::arg("p2p") = nullptr, py::arg("timeout_ms") = 60000);
  m.def(
      "gdw_reduce",
      [](uintptr_t slabs, int nslabs, int K, int F_aug, uintptr_t dW_out, uintptr_t stat_slabs, int nstat,
         uintptr_t stats_out, uintptr_t stream, P2PAllReduce* p2p, int timeout_ms) {
        launch_gdw_reduce(ptr<float>(slabs), nslabs, K, F_aug, ptr<float>(dW_out), ptr<float>(stat_slabs), nstat,
                          ptr<float>(stats_out), nullptr, p2p, timeout_ms, stream_of(stream));
      },
      py::arg("slabs"), py::arg("nslabs"), py::arg("K"), py::arg("F_aug"), py::arg("dW_out"), py::arg("stat_slabs"),
      py::arg("nstat"), py::arg("stats_out"), py::arg("stream") = 0, py::arg("p2p") = nullptr,
      py::arg("timeout_ms") = 60000);
  m.def("softmax_grad_wide_supported", &softmax_grad_wide_supported);
  m.def("softmax_grad_wide_workspace", &softmax_grad_wide_workspace);
  m.def("softmax_grad_wide_set_zbuf", &softmax_grad_wide_set_zbuf);
  m.def(
      "softmax_grad_wide",
      [](uintptr_t X_aug, int64_t ldx, uintptr_t W, uintptr_t b, uintptr_t y, int64_t B, int F, int K, int kind,
         uintptr_t dW_out, uintptr_t stats_out, uintptr_t ws, size_t ws_bytes, uintptr_t stream, uintptr_t params,
         uintptr_t mom, uintptr_t shadow_w, uintptr_t shadow_b, int pen_cols, float lr, float inv_n, float l2,
         float momentum, P2PAllReduce* p2p, int timeout_ms) {
        Sgd2D u;
        u.params = ptr<float>(params);
        u.mom = ptr<float>(mom);
        u.shadow_w = ptr<uint16_t>(shadow_w);
        u.shadow_b = ptr<float>(shadow_b);
        u.cols = F + 8;
        u.pen_cols = pen_cols;
        u.lr = lr;
        u.inv_n = inv_n;
        u.l2 = l2;
        u.momentum = momentum;
        launch_softmax_grad_wide(ptr<void>(X_aug), ldx, ptr<void>(W), ptr<float>(b), ptr<int32_t>(y), B, F, K, kind,
                                 ptr<float>(dW_out), ptr<float>(stats_out), ptr<void>(ws), ws_bytes, stream_of(stream),
                                 params != 0 ? &u : nullptr, p2p, timeout_ms);
      },
      py::arg("X_aug"), py::arg("ldx"), py::arg("W"), py::arg("b"), py::arg("y"), py::arg("B"), py::arg("F"),
      py::arg("K"), py::arg("kind"), py::arg("dW_out"), py::arg("stats_out"), py::arg("ws"), py::arg("ws_bytes"),
      py::arg("stream") = 0, py::arg("params") = 0, py::arg("mom") = 0, py::arg("shadow_w") = 0,
      py::arg("shadow_b") = 0, py::arg("pen_cols") = 0, py::arg("lr") = 0.f, py::arg("inv_n") = 0.f,
      py::arg("l2") = 0.f, py::arg("momentum") = 0.f, py::arg("p2p") = nullptr, py::arg("timeout_ms") = 60000);
  m.def(
      "sgd_update_2d",
      [](uintptr_t params, uintptr_t grad, uintptr_t mom, int64_t rows, int cols, int pen_cols, float lr,
         float inv_n, float l2, float momentum, uintptr_t shadow_w, uintptr_t shadow_b, uintptr_t stream) {
        launch_sgd_update_2d(ptr<float>(params), ptr<float>(grad), ptr<float>(mom), rows, cols, pen_cols, lr, inv_n,
                             l2, momentum, ptr<uint16_t>(shadow_w), ptr<float>(shadow_b), stream_of(stream));
      },
      py::arg("params"), py::arg("grad"), py::arg("mom"), py::arg("rows"), py::arg("cols"), py::arg("pen_cols"),
      py::arg("lr"), py::arg("inv_n"), py::arg("l2"), py::arg("momentum"), py::arg("shadow_w"),
      py::arg("shadow_b"), py::arg("stream") = 0);
  m.def(
      "cast",
      [](int src_dt, uintptr_t src, int dst_dt, uintptr_t dst, int64_t n, uintptr_t stream) {
        launch_cast(src_dt, ptr<void>(src), dst_dt, ptr<void>(dst), n, stream_of(stream));
      },
      py::arg("src_dt"), py::arg("src"), py::arg("dst_dt"), py::arg("dst"), py::arg("n"), py::arg("stream") = 0);

  // ---------------------------------------------------------------- engine
  py::class_<EngineConfig>(m, "EngineConfig")
      .def(py::init<>())
      .def_readwrite("device", &EngineConfig::device)
      .def_readwrite("max_batch", &EngineConfig::max_batch)
      .def_readwrite("max_wait_us", &EngineConfig::max_wait_us)
      .def_readwrite("slots", &EngineConfig::slots)
      .def_readwrite("dtype", &EngineConfig::dtype)
      .def_readwrite("max_features", &EngineConfig::max_features)
      .def_readwrite("watchdog_ms", &EngineConfig::watchdog_ms)
      .def_readwrite("fail_every", &EngineConfig::fail_every)
      .def_readwrite("delay_us", &EngineConfig::delay_us)
      .def_readwrite("spin_us", &EngineConfig::spin_us)
      .def_readwrite("wide_dtype", &EngineConfig::wide_dtype)
      .def_readwrite("split_max_rows", &EngineConfig::split_max_rows)
      .def_readwrite("bar_rows", &EngineConfig::bar_rows)
      .def_readwrite("host_merge_rows", &EngineConfig::host_merge_rows)
      .def_readwrite("inline_args", &EngineConfig::inline_args)
      .def_readwrite("idle_inline_rows", &EngineConfig::idle_inline_rows)
      .def_readwrite("resident", &EngineConfig::resident)
      .def_readwrite("resident_depth", &EngineConfig::resident_depth)
      .def_readwrite("resident_lease_ms", &EngineConfig::resident_lease_ms)
      .def_readwrite("resident_idle_polls", &EngineConfig::resident_idle_polls)
      .def_readwrite("resident_idle_sleep", &EngineConfig::resident_idle_sleep)
      .def_readwrite("f32_gemv", &EngineConfig::f32_gemv)
      .def_readwrite("wide_host_merge_blocks", &EngineConfig::wide_host_merge_blocks)
      .def_readwrite("completers", &EngineConfig::completers)
      .def_readwrite("batchers", &EngineConfig::batchers)
      .def_readwrite("gemv_record_rows", &EngineConfig::gemv_record_rows)
      .def_readwrite("direct_wide", &EngineConfig::direct_wide)
      .def_readwrite("direct_wide_max_weight_bytes", &EngineConfig::direct_wide_max_weight_bytes)
      .def_readwrite("record_completion", &EngineConfig::record_completion)
      .def_readwrite("stage_wide", &EngineConfig::stage_wide)
      .def_readwrite("direct_dispatch", &EngineConfig::direct_dispatch)
      .def_readwrite("hsaco_path", &EngineConfig::hsaco_path)
      .def_readwrite("max_queue", &EngineConfig::max_queue);

  py::class_<PySink>(m, "PySink").def(py::init<>()).def("fd", &PySink::fd).def("drain", &PySink::drain);

  py::class_<Engine>(m, "Engine")
      .def(py::init<const EngineConfig&>(), py::call_guard<py::gil_scoped_release>())
      .def(
          "load_model",
          [](Engine& e, int kind, py::array_t<double, py::array::c_style | py::array::forcecast> W,
             py::array_t<double, py::array::c_style | py::array::forcecast> b, std::vector<std::string> labels) {
            if (W.ndim() != 2) throw std::invalid_argument("W must be 2-D");
            const int K = (int)W.shape(0), F = (int)W.shape(1);
            if (b.size() != K) throw std::invalid_argument("b must have K entries");
            const double* wp = W.data();
            const double* bp = b.data();
            py::gil_scoped_release rel;
            return e.load_model(kind, F, K, wp, bp, labels);
          },
          py::arg("kind"), py::arg("W"), py::arg("b"), py::arg("labels"))
      .def("unload_model", &Engine::unload_model)
      .def("model_version",
           [](Engine& e) -> uint64_t {
             auto mm = e.model();
             return mm ? mm->version : 0;
           })
      .def("n_features",
           [](Engine& e) -> int {
             auto mm = e.model();
             return mm ? mm->F : 0;
           })
      .def("model_path",
           [](Engine& e) -> std::string {
             static const char* names[PATH_COUNT] = {"small", "gemv", "gemm", "generic", "wide"};
             auto mm = e.model();
             return mm ? names[mm->path] : "";
           })
      .def("inject_drop", &Engine::inject_drop, py::arg("on"))
      // resident-path fault injection (tests): "stall" | "stall_sticky" (kept across relaunches) |
      // "exit_ring" (arg = ring) | "ignore_stop" | "lease_starve" (arg = ms) | "queue_fault" | "none"
      // (clear); False = no live instance to inject into
      .def(
          "resident_inject",
          [](Engine& e, const std::string& mode, int arg) {
            int m = -1;
            if (mode == "none") m = RES_FAULT_NONE;
            else if (mode == "stall") m = RES_FAULT_STALL;
            else if (mode == "stall_sticky") m = Engine::RES_INJECT_STALL_STICKY;
            else if (mode == "exit_ring") m = RES_FAULT_EXIT_RING;
            else if (mode == "ignore_stop") m = RES_FAULT_IGNORE_STOP;
            else if (mode == "lease_starve") m = Engine::RES_INJECT_LEASE_STARVE;
            else if (mode == "queue_fault") m = Engine::RES_INJECT_QUEUE_FAULT;
            else throw std::invalid_argument("unknown resident fault " + mode);
            return e.resident_inject(m, arg);
          },
          py::arg("mode"), py::arg("arg") = 0)
      .def("mark_healthy", &Engine::mark_healthy)
      .def(
          "submit",
          [](Engine& e, py::array_t<double, py::array::c_style | py::array::forcecast> x, uint64_t tag, PySink& sink) {
            // 1 accepted, 0 engine stopping / malformed, -1 (Engine::SUBMIT_BUSY) queue full
            const uint64_t t = tag;
            return e.submit_many(x.data(), 1, (int)x.size(), &t, &sink);
          },
          py::arg("x"), py::arg("tag"), py::arg("sink"))
      .def(
          "submit_many",
          [](Engine& e, py::array_t<double, py::array::c_style | py::array::forcecast> X, uint64_t tag0,
             PySink& sink) {
            if (X.ndim() != 2) throw std::invalid_argument("X must be 2-D");
            const int64_t B = X.shape(0);
            const int F = (int)X.shape(1);
            const double* xp = X.data();
            int64_t ok = 0;
            for (int64_t r = 0; r < B; ++r) ok += e.submit(xp + r * F, F, tag0 + (uint64_t)r, &sink);
            return ok;
          },
          py::arg("X"), py::arg("tag0"), py::arg("sink"))
      .def("predict",
           [](Engine& e, py::array_t<double, py::array::c_style | py::array::forcecast> X) {
             if (X.ndim() != 2) throw std::invalid_argument("X must be 2-D");
             const int64_t B = X.shape(0);
             const int F = (int)X.shape(1);
             py::array_t<int32_t> idx(B), st(B);
             py::array_t<double> p(B);
             const double* xp = X.data();
             int32_t* ip = idx.mutable_data();
             double* pp = p.mutable_data();
             int32_t* sp = st.mutable_data();
             {
               py::gil_scoped_release rel;
               e.predict(xp, B, F, ip, pp, sp);
             }
             return py::make_tuple(idx, p, st);
           })
      .def("stats", [](Engine& e) { return stats_dict(e.stats()); })
      .def("healthy", &Engine::healthy)
      .def("stop", &Engine::stop, py::call_guard<py::gil_scoped_release>());

  // ---------------------------------------------------------------- HTTP server
  py::class_<ServerConfig>(m, "ServerConfig")
      .def(py::init<>())
      .def_readwrite("host", &ServerConfig::host)
      .def_readwrite("port", &ServerConfig::port)
      .def_readwrite("io_threads", &ServerConfig::io_threads)
      .def_readwrite("reuseport", &ServerConfig::reuseport)
      .def_readwrite("feature_names", &ServerConfig::feature_names)
      .def_readwrite("predict_path", &ServerConfig::predict_path)
      .def_readwrite("server_header", &ServerConfig::server_header)
      .def_readwrite("fast_path", &ServerConfig::fast_path)
      .def_readwrite("max_body", &ServerConfig::max_body)
      .def_readwrite("pipeline_cap", &ServerConfig::pipeline_cap)
      .def_readwrite("io_spin_us", &ServerConfig::io_spin_us)
      .def_readwrite("io_wait_spin_us", &ServerConfig::io_wait_spin_us)
      .def_readwrite("io_ring_spin_us", &ServerConfig::io_ring_spin_us)
      .def_readwrite("io_ring_sleep_us", &ServerConfig::io_ring_sleep_us)
      .def_readwrite("idle_max_conns", &ServerConfig::idle_max_conns)
      .def_readwrite("io_spin_lowload_us", &ServerConfig::io_spin_lowload_us)
      .def_readwrite("io_spin_max_conns", &ServerConfig::io_spin_max_conns)
      .def_readwrite("io_steer", &ServerConfig::io_steer)
      .def_readwrite("steer_every", &ServerConfig::steer_every)
      .def_readwrite("steer_stable", &ServerConfig::steer_stable)
      .def_readwrite("io_cpus", &ServerConfig::io_cpus)
      .def_readwrite("access_log", &ServerConfig::access_log)
      .def_readwrite("access_log_fd", &ServerConfig::access_log_fd)
      .def_readwrite("health_dispatch", &ServerConfig::health_dispatch)
      .def_readwrite("health_probe_ms", &ServerConfig::health_probe_ms)
      .def_readwrite("backlog", &ServerConfig::backlog)
      .def_readwrite("dispatch", &ServerConfig::dispatch)
      .def_readwrite("stage_timing", &ServerConfig::stage_timing)
      .def_readwrite("dispatch_group", &ServerConfig::dispatch_group)
      .def_readwrite("dispatch_rank", &ServerConfig::dispatch_rank)
      .def_readwrite("dispatch_claim", &ServerConfig::dispatch_claim);

  // ---- native RCCL communicator (csrc/dist/comm.h)
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](py::bytes id, int rank, int world, int device) {
             std::string uid = id;  // copy while holding the GIL, then release it for ncclCommInitRank
             py::gil_scoped_release nogil;
             return new RcclComm(uid, rank, world, device);
           }),
           py::arg("unique_id"), py::arg("rank"), py::arg("world"), py::arg("device"))
      .def_static("unique_id", []() { return py::bytes(RcclComm::unique_id()); })
      .def_static("version", &RcclComm::version)
      .def_static("library_path", &RcclComm::library_path)
      .def("all_reduce",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t stream) {
             c.all_reduce(ptr<void>(send), ptr<void>(recv), count, dtype, op, stream_of(stream));
           },
           py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("op"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int root, uintptr_t stream) {
             c.broadcast(ptr<void>(send), ptr<void>(recv), count, dtype, root, stream_of(stream));
           },
           py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("root"),
           py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def("all_gather",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, uintptr_t stream) {
             c.all_gather(ptr<void>(send), ptr<void>(recv), count, dtype, stream_of(stream));
           },
           py::arg("send"), py::arg("recv"), py::arg("count_per_rank"), py::arg("dtype"), py::arg("stream"),
           py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter",
           [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int op, uintptr_t stream) {
             c.reduce_scatter(ptr<void>(send), ptr<void>(recv), count, dtype, op, stream_of(stream));
           },
           py::arg("send"), py::arg("recv"), py::arg("recv_count"), py::arg("dtype"), py::arg("op"),
           py::arg("stream"), py::call_guard<py::gil_scoped_release>())
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("wait", [](RcclComm& c, uintptr_t stream, int timeout_ms) { return c.wait(stream_of(stream), timeout_ms); },
           py::arg("stream"), py::arg("timeout_ms") = 0, py::call_guard<py::gil_scoped_release>())
      .def("barrier",
           [](RcclComm& c, uintptr_t stream, int timeout_ms) { return c.barrier(stream_of(stream), timeout_ms); },
           py::arg("stream"), py::arg("timeout_ms") = 0, py::call_guard<py::gil_scoped_release>())
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("device", &RcclComm::device)
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def("comm_count", &RcclComm::comm_count)
      .def("comm_device", &RcclComm::comm_device)
      .def("comm_rank", &RcclComm::comm_rank);

  // ---- one-shot P2P all-reduce over IPC-mapped peer buffers (csrc/dist/p2p.h)
  py::class_<P2PAllReduce>(m, "P2PAllReduce")
      .def(py::init<int, int, int, size_t>(), py::arg("rank"), py::arg("world"), py::arg("device"),
           py::arg("max_bytes"))
      .def("data_handle", [](const P2PAllReduce& p) { return py::bytes(p.data_handle()); })
      .def("flag_handle", [](const P2PAllReduce& p) { return py::bytes(p.flag_handle()); })
      .def("open_peers",
           [](P2PAllReduce& p, const std::vector<py::bytes>& d, const std::vector<py::bytes>& f) {
             std::vector<std::string> ds, fs;
             for (const auto& x : d) ds.emplace_back(x);
             for (const auto& x : f) fs.emplace_back(x);
             py::gil_scoped_release nogil;
             p.open_peers(ds, fs);
           },
           py::arg("data_handles"), py::arg("flag_handles"))
      .def("all_reduce",
           [](P2PAllReduce& p, uintptr_t buf, size_t count, int dtype, uintptr_t stream, int timeout_ms) {
             p.all_reduce(ptr<void>(buf), count, dtype, stream_of(stream), timeout_ms);
           },
           py::arg("buf"), py::arg("count"), py::arg("dtype"), py::arg("stream"), py::arg("timeout_ms") = 60000,
           py::call_guard<py::gil_scoped_release>())
      .def("status", &P2PAllReduce::status, py::call_guard<py::gil_scoped_release>())
      .def("status_now", &P2PAllReduce::status_now)
      .def("selftest_write", &P2PAllReduce::selftest_write, py::arg("corrupt") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("selftest_verify", &P2PAllReduce::selftest_verify, py::call_guard<py::gil_scoped_release>())
      .def("inject_skip_publish", &P2PAllReduce::inject_skip_publish)
      .def_property_readonly("epoch", &P2PAllReduce::epoch)
      .def_property_readonly("max_bytes", &P2PAllReduce::max_bytes);

  py::class_<HttpServer>(m, "HttpServer")
      .def(py::init<Engine*, const ServerConfig&>(), py::keep_alive<1, 2>())
      .def("start", &HttpServer::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &HttpServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("port", &HttpServer::port)
      .def(
          "next_slow",
          [](HttpServer& s, int timeout_ms) -> py::object {
            SlowRequest r;
            bool got;
            {
              py::gil_scoped_release rel;
              got = s.next_slow(&r, timeout_ms);
            }
            if (!got) return py::none();
            py::list headers;
            for (auto& h : r.headers) headers.append(py::make_tuple(py::bytes(h.first), py::bytes(h.second)));
            py::dict d;
            d["token"] = r.token;
            d["method"] = r.method;
            d["target"] = py::bytes(r.target);
            d["http_version"] = r.http_version;
            d["headers"] = headers;
            d["body"] = py::bytes(r.body);
            d["client"] = py::make_tuple(r.client_host, r.client_port);
            d["server"] = py::make_tuple(r.server_host, r.server_port);
            return d;
          },
          py::arg("timeout_ms") = 100)
      .def(
          "respond",
          [](HttpServer& s, uint64_t token, int status, const std::string& reason, py::list headers, py::bytes body,
             bool close) {
            std::vector<std::pair<std::string, std::string>> hs;
            for (auto h : headers) {
              auto t = h.cast<py::tuple>();
              hs.emplace_back(t[0].cast<std::string>(), t[1].cast<std::string>());
            }
            std::string b = body;
            py::gil_scoped_release rel;
            s.respond(token, status, reason, hs, b, close);
          },
          py::arg("token"), py::arg("status"), py::arg("reason"), py::arg("headers"), py::arg("body"),
          py::arg("close") = false)
      .def("stats", [](HttpServer& s) {
        const ServerStats st = s.stats();
        py::dict d;
        d["fast"] = st.fast;
        d["slow"] = st.slow;
        d["responses"] = st.responses;
        d["connections"] = st.connections;
        d["errors"] = st.errors;
        d["bad_requests"] = st.bad_requests;
        d["listen_closes"] = st.listen_closes;
        d["steered"] = st.steered;
        d["steer_pauses"] = st.steer_pauses;
        d["conns_per_thread"] = st.conns_per_thread;
        d["steer_plan"] = st.steer_plan;
        d["accepting"] = st.accepting;
        d["listeners"] = s.listeners();
        py::dict stg;
        for (int i = 0; i < SS_COUNT; ++i) stg[server_stage_name(i)] = st.stage_ns[i];
        d["stage_ns"] = stg;
        py::list lh;
        for (int i = 0; i < HTTP_LAT_BUCKETS; ++i) lh.append(st.http_latency_hist[i]);
        d["http_latency_hist_us_pow2"] = lh;
        d["http_latency_sum_ns"] = st.http_latency_sum_ns;
        d["http_latency_count"] = st.http_latency_count;
        if (const ConnDispatcher* dp = s.dispatcher()) {
          py::dict x;
          x["leader"] = dp->leader();
          x["group"] = dp->group();
          x["received"] = dp->received();
          x["elections"] = dp->elections();
          py::list ts;
          for (const auto& t : dp->targets()) ts.append(py::make_tuple(t.rank, t.conns, t.healthy));
          x["targets"] = ts;
          d["dispatch"] = x;
        }
        return d;
      });

  // ---------------------------------------------------------------- load generator
  py::class_<Loadgen>(m, "Loadgen")
      .def(py::init<const std::string&, int, const std::string&, int, int, double>(), py::arg("host"), py::arg("port"),
           py::arg("request"), py::arg("conns"), py::arg("threads"), py::arg("timeout_s") = 30.0)
      .def(
          "run",
          [](Loadgen& lg, int64_t n, bool record) {
            LoadgenResult r;
            {
              py::gil_scoped_release rel;
              r = lg.run(n, record);
            }
            py::dict d;
            d["elapsed_s"] = r.elapsed_s;
            d["completed"] = r.completed;
            d["errors"] = r.errors;
            d["failed"] = r.failed;
            d["body_mismatches"] = r.body_mismatches;
            py::array_t<int64_t> lat((py::ssize_t)r.latencies_ns.size());
            if (!r.latencies_ns.empty())
              std::memcpy(lat.mutable_data(), r.latencies_ns.data(), r.latencies_ns.size() * sizeof(int64_t));
            d["latencies_ns"] = lat;
            py::dict sc;
            for (int s = 0; s < 600; ++s)
              if (r.status_counts[s]) sc[py::int_(s)] = r.status_counts[s];
            d["status_counts"] = sc;
            return d;
          },
          py::arg("requests_per_conn"), py::arg("record") = true)
      .def("set_workload", &Loadgen::set_workload, py::arg("requests"), py::arg("expected"),
           py::arg("rel_tol") = 0.0)
      .def("set_conn_map", &Loadgen::set_conn_map, py::arg("mode"), py::arg("seed") = 1)
      .def("set_thread_cpus", &Loadgen::set_thread_cpus, py::arg("cpus"))
      .def("close", &Loadgen::close_all);
}
