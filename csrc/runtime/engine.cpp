// Serving engine implementation (see engine.h for the design).
#include "engine.h"
#include "split_merge.h"

#include <immintrin.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>

#include "mlapi/kernels.h"
#include "trace.h"

namespace mlapi {

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

Model::~Model() {
  if (device >= 0) {
    int prev = 0;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (dW) (void)hipFree(dW);
    if (db) (void)hipFree(db);
    if (ws) (void)hipFree(ws);
    if (ws_split) (void)hipFree(ws_split);
    if (ws_wide) (void)hipFree(ws_wide);
    (void)hipSetDevice(prev);
  }
}

// Same epilogue formulas as linear_small.hip (float64).
void cpu_linear_predict(const Model& m, const double* X, int64_t B, int32_t* idx, double* p) {
  const int F = m.F, K = m.K;
  std::vector<double> z((size_t)K);
  for (int64_t r = 0; r < B; ++r) {
    const double* x = X + r * F;
    for (int k = 0; k < K; ++k) {
      double acc = 0.0;
      for (int f = 0; f < F; ++f) acc = std::fma(x[f], m.W[(size_t)k * F + f], acc);
      z[k] = acc + m.b[k];
    }
    int32_t id = 0;
    double pm;
    if (m.kind == KIND_BINARY) {
      const double p1 = 1.0 / (1.0 + std::exp(-z[0]));
      const double p0 = 1.0 - p1;
      id = z[0] > 0.0;
      pm = std::isnan(p1) ? p1 : (p0 > p1 ? p0 : p1);
    } else if (m.kind == KIND_BINARY_SOFTMAX) {
      const double zz = z[0], mm = std::fabs(zz);
      const double e0 = std::exp(-zz - mm), e1 = std::exp(zz - mm), s = e0 + e1;
      const double q0 = e0 / s, q1 = e1 / s;
      id = zz > 0.0;
      pm = std::isnan(s) ? s : (q0 > q1 ? q0 : q1);
    } else if (m.kind == KIND_MULTINOMIAL) {
      double mx = z[0];
      bool nan = std::isnan(z[0]);
      for (int k = 1; k < K; ++k) {
        nan |= std::isnan(z[k]);
        if (z[k] > mx) { mx = z[k]; id = k; }
      }
      double s = 0.0;
      for (int k = 0; k < K; ++k) s += std::exp(z[k] - mx);
      pm = nan ? std::nan("") : 1.0 / s;
    } else {
      double mx = z[0];
      for (int k = 1; k < K; ++k)
        if (z[k] > mx) { mx = z[k]; id = k; }
      double s = 0.0, smax = 0.0;
      for (int k = 0; k < K; ++k) {
        const double sg = 1.0 / (1.0 + std::exp(-z[k]));
        s += sg;
        smax = sg > smax ? sg : smax;
      }
      pm = smax / s;
    }
    idx[r] = id;
    p[r] = pm;
  }
}

namespace {
// rows of every path are padded to at most this multiple (GEMM: F -> 32..512 power of two)
size_t padded_features(int F) {
  const size_t f = (size_t)std::max(F, 1);
  return f <= 512 ? std::max<size_t>(32, size_t(1) << (64 - __builtin_clzll(f - 1 | 1))) : (f + 511) / 512 * 512;
}

inline uint16_t f32_to_bf16(float f) {  // round to nearest even (inputs are finite)
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// Kernel-argument batch: W + b of the model and n rows (row(i): the row's features, nullptr if its
// feature count does not match the model -> zeroed, ST_SHAPE in pre[i]) into `a`, in the model's
// small-path dtype.
template <class RowFn>
void fill_inline(InlineBatch& a, const Model& m, int64_t n, RowFn row, int32_t* pre) {
  a.n = (int32_t)n;
  a.F = m.F;
  a.K = m.K;
  a.kind = m.kind;
  const size_t kf = (size_t)m.K * m.F;
  if (m.xdt == DT_F64) {
    double* wb = reinterpret_cast<double*>(a.wb);
    std::memcpy(wb, m.W.data(), kf * sizeof(double));
    std::memcpy(wb + kf, m.b.data(), (size_t)m.K * sizeof(double));
    double* x = reinterpret_cast<double*>(a.x);
    for (int64_t i = 0; i < n; ++i) {
      const double* r = row(i);
      if (r == nullptr) pre[i] = ST_SHAPE;
      if (r != nullptr)
        std::memcpy(x + i * m.F, r, sizeof(double) * m.F);
      else
        std::memset(x + i * m.F, 0, sizeof(double) * m.F);
    }
  } else {
    float* wb = reinterpret_cast<float*>(a.wb);
    for (size_t i = 0; i < kf; ++i) wb[i] = (float)m.W[i];
    for (int k = 0; k < m.K; ++k) wb[kf + k] = (float)m.b[k];
    float* x = reinterpret_cast<float*>(a.x);
    for (int64_t i = 0; i < n; ++i) {
      const double* r = row(i);
      if (r == nullptr) pre[i] = ST_SHAPE;
      for (int f = 0; f < m.F; ++f) x[i * m.F + f] = r != nullptr ? (float)r[f] : 0.f;
    }
  }
}
}  // namespace

Engine::Engine(const EngineConfig& cfg) : cfg_(cfg) {
  if (cfg_.max_batch < 1) cfg_.max_batch = 1;
  if (cfg_.slots < 1) cfg_.slots = 1;
  if (cfg_.dtype != DT_F64 && cfg_.dtype != DT_F32) throw std::invalid_argument("engine dtype must be f64 or f32");
  if (cfg_.wide_dtype != DT_F64 && cfg_.wide_dtype != DT_F32 && cfg_.wide_dtype != DT_BF16)
    throw std::invalid_argument("engine wide_dtype must be f64, f32 or bf16");
  if (cfg_.max_features < 1) cfg_.max_features = 1;
  q_meta_.reserve(4096);
  q_x_.reserve(4096 * 8);
  if (cfg_.device >= 0) {
    MLAPI_HIP_CHECK(hipSetDevice(cfg_.device));
    int lo = 0, hi = 0;
    MLAPI_HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    MLAPI_HIP_CHECK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
    slots_.resize(cfg_.slots);
    slot_row_bytes_ = padded_features(cfg_.max_features) * sizeof(double);
    for (int f = 1; f <= cfg_.max_features; ++f)  // WIDE models' padded rows (plan width, either storage)
      slot_row_bytes_ = std::max({slot_row_bytes_, (size_t)linear_wide_plan(DT_F64, f, 1).ldx * sizeof(double),
                                  (size_t)linear_wide_plan(DT_F32, f, 1).ldx * sizeof(float)});
    const size_t xb = (size_t)cfg_.max_batch * slot_row_bytes_;
    const size_t done_bytes = sizeof(uint32_t) * SIGNAL_STRIDE * cfg_.slots;
    MLAPI_HIP_CHECK(hipHostMalloc((void**)&done_h_, done_bytes, hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(done_h_, 0, done_bytes);
    MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&done_d_, done_h_, 0));
    MLAPI_HIP_CHECK(hipMalloc((void**)&sig_counter_, sizeof(uint32_t)));
    MLAPI_HIP_CHECK(hipMemset(sig_counter_, 0, sizeof(uint32_t)));
    MLAPI_HIP_CHECK(hipDeviceSynchronize());
    if (cfg_.direct_dispatch && !cfg_.hsaco_path.empty()) {
      std::string why;
      direct_ = make_direct_dispatcher(cfg_.device, cfg_.hsaco_path, cfg_.slots, &why);
      if (!direct_) std::fprintf(stderr, "[mlapi engine] direct dispatch off (%s): using hipLaunchKernel\n", why.c_str());
    }
    if (direct_ && cfg_.resident > 0) {
      // resident kernel: rings + records + control block in host-coherent memory the waves poll
      const size_t rb = (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * RESIDENT_ENTRY_BYTES;
      const size_t cb = (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * sizeof(ServeRecord);
      MLAPI_HIP_CHECK(hipHostMalloc((void**)&res_rings_h_, rb, hipHostMallocMapped | hipHostMallocCoherent));
      MLAPI_HIP_CHECK(hipHostMalloc((void**)&res_recs_h_, cb, hipHostMallocMapped | hipHostMallocCoherent));
      MLAPI_HIP_CHECK(hipHostMalloc((void**)&res_ctl_h_, sizeof(ResidentCtl), hipHostMallocMapped | hipHostMallocCoherent));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&res_rings_d_, res_rings_h_, 0));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&res_recs_d_, res_recs_h_, 0));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&res_ctl_d_, res_ctl_h_, 0));
    }
    for (int i = 0; i < cfg_.slots; ++i) {
      Slot& s = slots_[i];
      MLAPI_HIP_CHECK(hipHostMalloc(&s.hx, xb, hipHostMallocMapped));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer(&s.dx, s.hx, 0));
      MLAPI_HIP_CHECK(hipMalloc(&s.dstage, xb));
      MLAPI_HIP_CHECK(hipHostMalloc((void**)&s.hidx, (size_t)cfg_.max_batch * sizeof(int32_t), hipHostMallocMapped));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&s.didx, s.hidx, 0));
      MLAPI_HIP_CHECK(hipHostMalloc(&s.hp, (size_t)cfg_.max_batch * sizeof(double), hipHostMallocMapped));
      MLAPI_HIP_CHECK(hipHostGetDevicePointer(&s.dp, s.hp, 0));
      const size_t rb = (size_t)cfg_.max_batch * sizeof(ServeRecord);
      MLAPI_HIP_CHECK(hipHostMalloc((void**)&s.hrec, rb, hipHostMallocMapped | hipHostMallocCoherent));
      std::memset(s.hrec, 0, rb);  // seq 0 is never launched
      MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&s.drec, s.hrec, 0));
      if (direct_ && cfg_.bar_rows > 0) s.xbar = direct_->bar_alloc((size_t)cfg_.bar_rows * slot_row_bytes_);
      if (cfg_.host_merge_rows > 0) {
        // linear_split: [64 blocks][32 rows] SplitRecord; linear_wide: [64 blocks][32 rows][2] WideRecord
        const size_t sb = (size_t)64 * 32 * 2 * sizeof(WideRecord);
        MLAPI_HIP_CHECK(hipHostMalloc((void**)&s.hsrec, sb, hipHostMallocMapped | hipHostMallocCoherent));
        std::memset(s.hsrec, 0, sb);
        MLAPI_HIP_CHECK(hipHostGetDevicePointer((void**)&s.dsrec, s.hsrec, 0));
      }
      s.metas.reserve(cfg_.max_batch);
      free_slots_.push_back(i);
    }
  }
  if (cfg_.device < 0 && cfg_.resident > 0) {
    // CPU backend: same layouts in plain memory, the supervisor thread plays the resident kernel
    res_cpu_ = true;
    const size_t rb = (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * RESIDENT_ENTRY_BYTES;
    const size_t cb = (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * sizeof(ServeRecord);
    res_rings_h_ = res_rings_d_ = static_cast<unsigned char*>(std::aligned_alloc(64, rb));
    res_recs_h_ = res_recs_d_ = static_cast<ServeRecord*>(std::aligned_alloc(64, cb));
    res_ctl_h_ = res_ctl_d_ = static_cast<ResidentCtl*>(std::aligned_alloc(64, sizeof(ResidentCtl)));
  }
  if (res_ctl_h_ != nullptr) {
    // position 0xffffffff with meta 0 never matches a live row; records start with seq 0xffffffff
    std::memset(res_rings_h_, 0xff, (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * RESIDENT_ENTRY_BYTES);
    std::memset(res_recs_h_, 0xff, (size_t)RESIDENT_MAX_RINGS * RESIDENT_RING * sizeof(ServeRecord));
    std::memset(res_ctl_h_, 0, sizeof(ResidentCtl));
    if (!res_cpu_) resident_register(true);
    res_thread_ = std::thread([this] { resident_loop(); });
  }
  for (int i = 0; i < std::max(1, cfg_.batchers); ++i) batchers_.emplace_back([this] { batcher_loop(); });
  if (cfg_.device >= 0)
    for (int i = 0; i < std::max(1, cfg_.completers); ++i) completers_.emplace_back([this] { completer_loop(); });
}

Engine::~Engine() {
  stop();
  if (res_cpu_) {
    std::free(res_rings_h_);
    std::free(res_recs_h_);
    std::free(res_ctl_h_);
  }
  if (cfg_.device >= 0) {
    (void)hipSetDevice(cfg_.device);
    if (stream_) (void)hipStreamSynchronize(stream_);
    if (done_h_) (void)hipHostFree(done_h_);
    if (sig_counter_) (void)hipFree(sig_counter_);
    if (res_ctl_h_ != nullptr && !res_leaked_) {  // the supervisor has stopped its instance (stop())
      (void)hipHostFree(res_rings_h_);
      (void)hipHostFree(res_recs_h_);
      (void)hipHostFree(res_ctl_h_);
    }
    for (Slot& s : slots_) {
      if (s.hx) (void)hipHostFree(s.hx);
      if (s.dstage) (void)hipFree(s.dstage);
      if (s.hidx) (void)hipHostFree(s.hidx);
      if (s.hp) (void)hipHostFree(s.hp);
      if (s.hrec) (void)hipHostFree(s.hrec);
      if (s.hsrec) (void)hipHostFree(s.hsrec);
    }
    {
      std::lock_guard<std::mutex> lk(model_mu_);
      model_.reset();
    }
    if (stream_) (void)hipStreamDestroy(stream_);
  }
}

void Engine::stop() {
  {
    std::lock_guard<std::mutex> lk(res_mu_);
    res_stop_ = true;
  }
  res_cv_.notify_all();
  if (res_thread_.joinable()) res_thread_.join();  // the resident instance has ended (or is abandoned)
  if (res_ctl_h_ != nullptr && !res_cpu_) resident_register(false);
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    stopping_ = true;
  }
  q_cv_.notify_all();
  for (std::thread& t : batchers_)
    if (t.joinable()) t.join();
  s_cv_.notify_all();
  for (std::thread& t : completers_)
    if (t.joinable()) t.join();
}

uint64_t Engine::load_model(int kind, int F, int K, const double* W, const double* b,
                            const std::vector<std::string>& label_json) {
  if (F <= 0 || K <= 0) throw std::invalid_argument("load_model: empty model");
  if (F > cfg_.max_features) throw std::invalid_argument("load_model: F exceeds engine max_features");
  auto m = std::make_shared<Model>();
  m->kind = kind;
  m->F = F;
  m->K = K;
  m->dtype = cfg_.dtype;
  m->W.assign(W, W + (size_t)K * F);
  m->b.assign(b, b + K);
  m->label_json = label_json;
  // ---- kernel path (see engine.h); the CPU backend ignores it
  const bool binary = kind == KIND_BINARY || kind == KIND_BINARY_SOFTMAX;
  if (F <= 32 && K <= 16) {
    m->path = PATH_SMALL;
    m->xdt = cfg_.dtype;
    m->ldx = F;
  } else if (binary && K == 1 && (cfg_.wide_dtype == DT_BF16 ? F <= 4096 : cfg_.wide_dtype == DT_F32 && cfg_.f32_gemv && F <= 2048)) {
    // bf16 binary models (and f32 ones with f32_gemv): the GEMV kernel, f32 accumulation; f32 / f64
    // storage otherwise takes WIDE below (f64 accumulation: rel 1e-11 / 1e-12 of the oracle, and
    // measured no slower at serving batch sizes: profiles/r4_s20/)
    m->path = PATH_GEMV;
    m->xdt = cfg_.wide_dtype;
    const int ne = cfg_.wide_dtype == DT_BF16 ? 8 : 4;  // elements per 16-byte chunk
    m->ldx = (F + ne - 1) / ne * ne;
  } else if (!binary && K >= 2 && cfg_.wide_dtype == DT_BF16 && F <= 4096) {
    // F <= 512: the tiles kernels at a power-of-two width; wider: the row-group kernel at a
    // multiple of 512 (it loops F in 256-feature slices inside one launch)
    m->path = PATH_GEMM;
    m->xdt = DT_BF16;
    m->ldx = (int)padded_features(F);
  } else if (binary ? K == 1 : K >= 2) {
    // f64 accumulation on the matrix cores, any width: f64 storage (wide_dtype f64) or f32 (bf16
    // models beyond the bf16 kernels' F <= 4096 are stored f32 here: more precision, not less)
    m->path = PATH_WIDE;
    m->xdt = cfg_.wide_dtype == DT_F64 ? DT_F64 : DT_F32;
    m->wplan = linear_wide_plan(m->xdt, F, K);
    m->ldx = m->wplan.ldx;
  } else {
    m->path = PATH_GENERIC;
    m->xdt = cfg_.wide_dtype == DT_F64 ? DT_F64 : DT_F32;
    m->ldx = F;
  }
  if (m->path == PATH_GENERIC) {
    std::fprintf(stderr, "[mlapi engine] warning: model kind %d F=%d K=%d runs on the scalar GENERIC kernel\n", kind, F,
                 K);
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.generic_models++;
  }
  m->pdt = (m->path == PATH_GEMV || m->path == PATH_GEMM) ? DT_F32 : m->xdt;
  if (m->path == PATH_WIDE) m->pdt = DT_F64;
  m->bias0 = (float)b[0];
  m->version = next_version_.fetch_add(1);
  if (cfg_.device >= 0) {
    MLAPI_HIP_CHECK(hipSetDevice(cfg_.device));
    m->device = cfg_.device;
    // W as the kernel reads it: [K][ldx] in xdt, zero-padded columns
    const size_t wn = (size_t)K * m->ldx;
    std::vector<unsigned char> wbuf(wn * dtype_size(m->xdt), 0);
    for (int k = 0; k < K; ++k)
      for (int f = 0; f < F; ++f) {
        const double v = W[(size_t)k * F + f];
        const size_t i = (size_t)k * m->ldx + f;
        if (m->xdt == DT_F64)
          reinterpret_cast<double*>(wbuf.data())[i] = v;
        else if (m->xdt == DT_F32)
          reinterpret_cast<float*>(wbuf.data())[i] = (float)v;
        else
          reinterpret_cast<uint16_t*>(wbuf.data())[i] = f32_to_bf16((float)v);
      }
    MLAPI_HIP_CHECK(hipMalloc(&m->dW, wbuf.size()));
    MLAPI_HIP_CHECK(hipMemcpy(m->dW, wbuf.data(), wbuf.size(), hipMemcpyHostToDevice));
    // bias: xdt for SMALL / GENERIC (the kernels' T), f64 for WIDE, f32 for GEMM (GEMV takes a scalar)
    const int bdt = m->path == PATH_SMALL || m->path == PATH_GENERIC ? m->xdt : m->path == PATH_WIDE ? DT_F64 : DT_F32;
    MLAPI_HIP_CHECK(hipMalloc(&m->db, (size_t)K * dtype_size(bdt)));
    if (bdt == DT_F64 && m->path == PATH_WIDE && m->xdt == DT_F32) {
      // f32 storage: the intercept is rounded like W and the rows (the f32 model, exactly)
      std::vector<double> bd(K);
      for (int k = 0; k < K; ++k) bd[k] = (double)(float)b[k];
      MLAPI_HIP_CHECK(hipMemcpy(m->db, bd.data(), (size_t)K * 8, hipMemcpyHostToDevice));
    } else if (bdt == DT_F64) {
      MLAPI_HIP_CHECK(hipMemcpy(m->db, b, (size_t)K * 8, hipMemcpyHostToDevice));
    } else {
      std::vector<float> bf(b, b + K);
      MLAPI_HIP_CHECK(hipMemcpy(m->db, bf.data(), bf.size() * 4, hipMemcpyHostToDevice));
    }
    if (m->path == PATH_GEMM) {
      // the split plan depends on the batch size: size for the largest any batch can need
      if (m->xdt == DT_BF16)
        for (int64_t B = 1; B <= cfg_.max_batch; ++B)
          m->ws_bytes = std::max(m->ws_bytes, gemm_softmax_workspace(B, K, m->ldx));
      if (m->ws_bytes) {
        MLAPI_HIP_CHECK(hipMalloc(&m->ws, m->ws_bytes));
        MLAPI_HIP_CHECK(hipMemset(m->ws, 0, m->ws_bytes));
      }
      if (linear_split_supported(m->xdt, m->ldx)) {
        m->ws_split_bytes = linear_split_workspace(cfg_.max_batch, K);
        MLAPI_HIP_CHECK(hipMalloc(&m->ws_split, m->ws_split_bytes));
        MLAPI_HIP_CHECK(hipMemset(m->ws_split, 0, m->ws_split_bytes));
      }
    }
    if (m->path == PATH_WIDE) {
      // one workspace per batch slot (256-byte aligned): batches in flight never share tickets, so
      // their direct-dispatched packets need no barrier and overlap on the GPU
      m->ws_wide_bytes = (linear_wide_workspace(cfg_.max_batch, m->xdt, F, K) + 255) & ~size_t(255);
      const size_t total = m->ws_wide_bytes * (size_t)std::max(1, cfg_.slots);
      MLAPI_HIP_CHECK(hipMalloc(&m->ws_wide, total));
      MLAPI_HIP_CHECK(hipMemset(m->ws_wide, 0, total));
    }
    MLAPI_HIP_CHECK(hipDeviceSynchronize());
  }
  std::shared_ptr<const Model> cm = m;
  {
    std::lock_guard<std::mutex> lk(model_mu_);
    model_.swap(cm);
  }
  {
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.model_version = m->version;
  }
  kick_resident();
  return m->version;  // old model (cm) released here unless an in-flight batch still holds it
}

void Engine::unload_model() {
  {
    std::lock_guard<std::mutex> lk(model_mu_);
    model_.reset();
  }
  kick_resident();
}

void Engine::kick_resident() {
  {
    std::lock_guard<std::mutex> lk(res_mu_);
    ++res_kick_;
  }
  res_cv_.notify_all();
}

std::shared_ptr<const Model> Engine::model() const {
  std::lock_guard<std::mutex> lk(model_mu_);
  return model_;
}

bool Engine::submit(const double* x, int nf, uint64_t tag, Sink* sink) {
  return submit_many(x, 1, nf, &tag, sink) == 1;
}

// One lock acquisition for a whole group of requests (an IO thread submits everything it parsed
// in one epoll round), and a futex wake only when the batcher is actually asleep: at high load
// the batcher is busy launching and the notify would be a wasted syscall per request.
int Engine::submit_many(const double* X, int n, int nf, const uint64_t* tags, Sink* sink) {
  if (nf < 0 || nf > cfg_.max_features || n <= 0) return 0;
  const int64_t t = now_ns();
  bool wake;
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (stopping_) return 0;
    // Backpressure: accept the prefix that still fits under max_queue, refuse the rest (the caller
    // answers those 503). All-or-nothing would refuse a whole epoll round's worth of requests
    // because of the last one.
    const int64_t room = (int64_t)cfg_.max_queue - (int64_t)q_meta_.size();
    if (room < n) {
      std::lock_guard<std::mutex> sl(st_mu_);
      stats_.rejected += (uint64_t)(n - std::max<int64_t>(room, 0));
      if (room <= 0) return SUBMIT_BUSY;
      n = (int)room;
    }
    int32_t off = (int32_t)q_x_.size();
    q_x_.insert(q_x_.end(), X, X + (size_t)n * nf);
    for (int i = 0; i < n; ++i, off += nf) q_meta_.push_back(Meta{tags[i], sink, t, nf, off});
    q_count_.store((int)q_meta_.size(), std::memory_order_release);
    wake = batchers_sleeping_ > 0;
  }
  if (wake) q_cv_.notify_one();
  return n;
}

namespace {
struct BlockingSink : Sink {
  std::mutex mu;
  std::condition_variable cv;
  int64_t remaining = 0;
  int32_t* idx;
  double* p;
  int32_t* st;
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>&) override {
    std::lock_guard<std::mutex> lk(mu);
    for (size_t i = 0; i < n; ++i) {
      idx[c[i].tag] = c[i].idx;
      p[c[i].tag] = c[i].p;
      st[c[i].tag] = c[i].status;
    }
    remaining -= (int64_t)n;
    if (remaining == 0) cv.notify_all();
  }
};
}  // namespace

void Engine::predict(const double* X, int64_t B, int F, int32_t* idx, double* p, int32_t* status) {
  BlockingSink sink;
  sink.idx = idx;
  sink.p = p;
  sink.st = status;
  sink.remaining = B;
  int64_t submitted = 0;
  for (int64_t r = 0; r < B; ++r) {
    if (!submit(X + r * F, F, (uint64_t)r, &sink)) {
      idx[r] = 0;
      p[r] = std::nan("");
      status[r] = ST_SHUTDOWN;
    } else {
      ++submitted;
    }
  }
  std::unique_lock<std::mutex> lk(sink.mu);
  sink.remaining -= (B - submitted);
  sink.cv.wait(lk, [&] { return sink.remaining <= 0; });
}

void Engine::record_batch(size_t n) {
  int b = 0;
  while ((size_t(1) << (b + 1)) <= n && b < 11) ++b;
  std::lock_guard<std::mutex> lk(st_mu_);
  stats_.batches++;
  stats_.batch_hist[b]++;
}

void Engine::deliver(std::vector<Meta>& metas, const int32_t* idx, const double* p, const int32_t* st,
                     const std::shared_ptr<const Model>& m, int64_t now) {
  const size_t n = metas.size();
  auto status = [&](size_t j) {
    const int32_t s = st[j];
    return s == ST_OK && !std::isfinite(p[j]) ? (int32_t)ST_NONFINITE : s;
  };
  // stats first: a sink's waiter may read them as soon as its on_complete has run (counted after
  // the hand-off, a predict() could return before its own requests were in `requests`)
  {
    uint64_t errors = 0;
    uint64_t lat_hist[24] = {0};
    double lat_sum = 0;
    for (size_t j = 0; j < n; ++j) {
      if (status(j) != ST_OK) ++errors;
      const double us = (double)(now - metas[j].t_enq) * 1e-3;
      lat_sum += us;
      int bkt = 0;
      while (bkt < 23 && (double)(int64_t(1) << bkt) <= us) ++bkt;
      lat_hist[bkt]++;
    }
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.requests += n;
    stats_.errors += errors;
    stats_.latency_sum_us += lat_sum;
    for (int b = 0; b < 24; ++b) stats_.latency_hist[b] += lat_hist[b];
  }
  // group by sink, preserving submission order inside each sink
  std::vector<Completion> buf;
  buf.reserve(n);
  std::vector<char> done(n, 0);
  for (size_t i = 0; i < n; ++i) {
    if (done[i]) continue;
    Sink* sk = metas[i].sink;
    buf.clear();
    for (size_t j = i; j < n; ++j) {
      if (done[j] || metas[j].sink != sk) continue;
      done[j] = 1;
      buf.push_back(Completion{metas[j].tag, idx[j], status(j), p[j], now - metas[j].t_enq});
    }
    if (sk) sk->on_complete(buf.data(), buf.size(), m);
  }
}

void Engine::run_cpu(std::vector<Meta>& metas, const std::vector<double>& xs, const std::shared_ptr<const Model>& m) {
  const size_t n = metas.size();
  std::vector<int32_t> idx(n, 0), st(n, ST_OK);
  std::vector<double> p(n, 0.0);
  if (!m) {
    std::fill(st.begin(), st.end(), (int32_t)ST_NO_MODEL);
  } else {
    std::vector<double> X((size_t)n * m->F, 0.0);
    for (size_t i = 0; i < n; ++i) {
      if (metas[i].nf != m->F) {
        st[i] = ST_SHAPE;
        continue;
      }
      std::memcpy(&X[i * m->F], &xs[metas[i].off], sizeof(double) * m->F);
    }
    cpu_linear_predict(*m, X.data(), (int64_t)n, idx.data(), p.data());
    if (drop_.load(std::memory_order_relaxed)) {
      std::fill(st.begin(), st.end(), (int32_t)ST_DEVICE_ERROR);
      healthy_.store(false);
    } else if (cfg_.fail_every > 0 && (++batch_counter_ % (uint64_t)cfg_.fail_every) == 0) {
      std::fill(st.begin(), st.end(), (int32_t)ST_DEVICE_ERROR);
    }
  }
  if (cfg_.delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(cfg_.delay_us));
  record_batch(n);
  deliver(metas, idx.data(), p.data(), st.data(), m, now_ns());
}

// Rows of the batch -> the slot's pinned buffer in the model's row layout (xdt, stride ldx,
// zero padding). A row whose feature count does not match the model is zeroed and answered
// ST_SHAPE.
void Engine::pack_rows(Slot& s, const std::vector<double>& xs, const Model& m, void* dst) {
  const int F = m.F, ld = m.ldx;
  const size_t n = (size_t)s.n;
  // MLAPI_PACK_STAGED=1: stage each row in a scratch row (below). Off by default: interleaved x2 on
  // one box it was 0-7 % slower end to end than converting straight into dst
  // (profiles/r3_pack_staged/), though its own pack stage was shorter at K = 1000.
  static const bool staged = [] {
    const char* e = getenv("MLAPI_PACK_STAGED");
    return e != nullptr && atoi(e) != 0;
  }();
  const size_t es = dtype_size(m.xdt);
  // staged: each row is converted in a cached scratch row (branch-free loops the compiler
  // vectorises) and then copied out in one memcpy - dst is often the BAR (write-combined,
  // uncached device memory), where element-by-element stores with a per-element select were
  // the batcher's largest cost on wide models
  thread_local std::vector<unsigned char> row;
  if (staged && row.size() < (size_t)ld * es) row.resize((size_t)ld * es);
  for (size_t i = 0; i < n; ++i) {
    const bool ok = s.metas[i].nf == F;
    if (!ok) s.pre_status[i] = ST_SHAPE;
    const double* src = &xs[s.metas[i].off];
    unsigned char* d = static_cast<unsigned char*>(dst) + i * ld * es;
    if (staged) {
      if (!ok) {
        std::memset(d, 0, (size_t)ld * es);
        continue;
      }
      if (m.xdt == DT_F64) {
        std::memcpy(d, src, sizeof(double) * F);
        if (ld > F) std::memset(d + sizeof(double) * F, 0, sizeof(double) * (ld - F));
        continue;
      }
      if (m.xdt == DT_F32) {
        float* t = reinterpret_cast<float*>(row.data());
        for (int f = 0; f < F; ++f) t[f] = (float)src[f];
        for (int f = F; f < ld; ++f) t[f] = 0.f;
      } else {
        uint16_t* t = reinterpret_cast<uint16_t*>(row.data());
        for (int f = 0; f < F; ++f) t[f] = f32_to_bf16((float)src[f]);
        for (int f = F; f < ld; ++f) t[f] = 0;
      }
      std::memcpy(d, row.data(), (size_t)ld * es);
      continue;
    }
    if (m.xdt == DT_F64) {
      double* dd = reinterpret_cast<double*>(d);
      if (ok)
        std::memcpy(dd, src, sizeof(double) * F);
      else
        std::memset(dd, 0, sizeof(double) * F);
      for (int f = F; f < ld; ++f) dd[f] = 0.0;
    } else if (m.xdt == DT_F32) {
      float* df = reinterpret_cast<float*>(d);
      for (int f = 0; f < F; ++f) df[f] = ok ? (float)src[f] : 0.f;
      for (int f = F; f < ld; ++f) df[f] = 0.f;
    } else {
      uint16_t* dh = reinterpret_cast<uint16_t*>(d);
      for (int f = 0; f < F; ++f) dh[f] = ok ? f32_to_bf16((float)src[f]) : 0;
      for (int f = F; f < ld; ++f) dh[f] = 0;
    }
  }
}

// One launch for the whole batch on the model's kernel path (engine.h).
void Engine::launch_batch(Slot& s, const Model& m, const std::vector<double>& xs) {
  const int64_t n = s.n;
  const int si = (int)(&s - slots_.data());
  ServeSignal sig;
  sig.done = done_d_ + (size_t)si * SIGNAL_STRIDE;
  sig.seq = ++s.seq;
  sig.counter = sig_counter_;
  if (m.path == PATH_SMALL && cfg_.inline_args && linear_inline_fits(m.xdt, n, m.F, m.K)) {
    // rows, W and b ride in the kernel-argument block
    InlineBatch& a = inline_;
    a.out_idx = s.didx;
    a.out_p = s.dp;
    s.rec_mode = cfg_.record_completion ? REC_ROWS : 0;
    a.done = s.rec_mode ? nullptr : sig.done;
    a.rec = s.rec_mode ? s.drec : nullptr;
    a.rec_scatter = 0;
    a.seq = sig.seq;
    fill_inline(
        a, m, n,
        [&](int64_t i) -> const double* { return s.metas[i].nf == m.F ? &xs[s.metas[i].off] : nullptr; },
        s.pre_status.data());
    if (direct_)
      direct_->launch(m.xdt, a);  // ~0.03 us: one packet into the engine's own HSA queue
    else
      launch_linear_inline(m.xdt, a, stream_);
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.path_batches[PATH_SMALL]++;
    stats_.inline_batches++;
    if (direct_) stats_.direct_batches++;
    return;
  }
  s.rec_mode = 0;
  const size_t bytes = (size_t)n * m.ldx * dtype_size(m.xdt);
  const bool bar = s.xbar != nullptr && m.path != PATH_SMALL && n <= cfg_.bar_rows &&
                   bytes <= (size_t)cfg_.bar_rows * slot_row_bytes_;
  // class-split and record-completing GEMV batches go into the direct dispatcher's own queue: ~0.1 us of batcher time instead of hipLaunchKernel's ~3 us, and that launch's HDP flush
  // also covers the BAR rows (no flush of their own)
  const bool split_path = m.path != PATH_SMALL && m.path != PATH_GENERIC && m.path != PATH_GEMV &&
                          m.ws_split != nullptr && n <= cfg_.split_max_rows;
  const bool gemv_rec = m.path == PATH_GEMV && cfg_.gemv_record_rows > 0 && n >= cfg_.gemv_record_rows;
  // ... for models whose weights stay small: the packet's agent-scope acquire (it covers the
  // kernarg block written through the BAR) invalidates L2, so every batch re-reads W - measured
  // +4 us on the GPU leg for a 1 MB f32 K = 1000 model, which outweighs the ~2 us of batcher time
  // saved (profiles/r3_direct_wide/)
  const size_t w_bytes = (size_t)(m.path == PATH_GEMV ? 1 : m.K) * m.ldx * dtype_size(m.xdt);
  const bool direct_wide = direct_ && cfg_.direct_wide && cfg_.record_completion &&
                           (split_path || gemv_rec || m.path == PATH_WIDE) &&
                           w_bytes <= (size_t)cfg_.direct_wide_max_weight_bytes;
  const int64_t t_p0 = now_ns();
  pack_rows(s, xs, m, bar ? s.xbar : s.hx);
  const int64_t t_p1 = now_ns();
  // rows: written into device HBM through the BAR (small wide batches: every wave then reads them
  // from HBM / L2), zero-copy from the pinned slot (one host-link round trip per reading wave), or
  // staged by a copy first (a blit kernel of its own: ~4 us at serving sizes)
  const void* X = s.dx;
  if (bar) {
    if (!direct_wide) direct_->bar_flush();
    X = s.xbar;
  } else if (m.path != PATH_SMALL && cfg_.stage_wide) {
    MLAPI_HIP_CHECK(hipMemcpyAsync(s.dstage, s.hx, bytes, hipMemcpyHostToDevice, stream_));
    X = s.dstage;
  }
  const int64_t t_p2 = now_ns();
  bool direct_wide_used = false;
  if (m.path == PATH_SMALL || m.path == PATH_GENERIC) {
    launch_linear_small(m.xdt, X, m.ldx, m.dW, m.db, n, m.F, m.K, m.kind, s.didx, s.dp, stream_, sig);
  } else {
    // GEMM: completion records written by the kernel's result stores (no trailing one-wave
    // serve_signal launch: 3.9 us of GPU time and a hipLaunchKernel per batch). GEMV: records from
    // gemv_record_rows rows up - a batch-1 leg measured 6.3-6.9 us with records vs 5.6-6.0 with the
    // signal kernel (profiles/r2_records/wide_ab/), but under load the signal kernel's second
    // hipLaunchKernel is batcher time, and the batcher is what queues the rows (engine stage
    // clocks: launch ~10 us per GEMV batch at c=64, profiles/r3_s19/).
    RecOut ro;
    if (cfg_.record_completion && (m.path == PATH_GEMM || gemv_rec)) {
      ro.rec = s.drec;
      ro.seq = sig.seq;
      s.rec_mode = REC_ROWS;
    }
    // a kernel the code object lacks falls back to hipLaunchKernel: flush the BAR rows first
    struct Direct final : KernelLauncher {
      InlineDispatcher* d;
      bool flush_on_miss, used = false;
      bool launch_kernel(const char* name, const void* args, size_t bytes, unsigned gx, unsigned gy, unsigned block,
                         bool ordered) override {
        if (d->launch_kernel(name, args, bytes, gx, gy, block, ordered)) return used = true;
        if (flush_on_miss) d->bar_flush();
        return false;
      }
    } dl;
    dl.d = direct_.get();
    dl.flush_on_miss = bar;
    if (m.path == PATH_WIDE) {
      // f64 accumulation; per-row records from the kernel's in-kernel class merge (default), or -
      // with wide_host_merge_blocks set - per-(class block, row) records the completer merges
      WideRecOut hro;
      const bool binary = m.kind == KIND_BINARY || m.kind == KIND_BINARY_SOFTMAX;
      if (cfg_.record_completion && s.hsrec != nullptr && !binary && n <= cfg_.host_merge_rows && n <= 32 &&
          m.wplan.ncb > 1 && m.wplan.ncb <= std::min(64, cfg_.wide_host_merge_blocks)) {
        hro.rec = reinterpret_cast<WideRecord*>(s.dsrec);
        hro.seq = sig.seq;
        ro = RecOut();
        s.rec_mode = REC_WIDE;
        s.rec_nsplit = m.wplan.ncb;
      } else if (cfg_.record_completion) {
        ro.rec = s.drec;
        ro.seq = sig.seq;
        s.rec_mode = REC_ROWS;
      }
      launch_linear_wide(m.xdt, X, m.ldx, m.dW, static_cast<const double*>(m.db), n, m.F, m.K, m.kind, s.didx,
                         static_cast<double*>(s.dp), static_cast<unsigned char*>(m.ws_wide) + (size_t)si * m.ws_wide_bytes,
                         m.ws_wide_bytes, stream_, ro, hro, direct_wide ? &dl : nullptr, /*ws_private=*/true);
    } else if (m.path == PATH_GEMV)
      launch_gemv_binary(m.xdt, X, m.dW, m.bias0, n, m.ldx, m.kind, s.didx, static_cast<float*>(s.dp), stream_, ro,
                         direct_wide && ro.rec != nullptr ? &dl : nullptr);
    else if (m.ws_split != nullptr && n <= cfg_.split_max_rows) {
      // small batches: the class-split kernel. Serving-sized batches end in
      // per-block records the completer merges; larger ones merge in-kernel (one round trip).
      SplitRecOut sro;
      const int ns = linear_split_nsplit(m.K);
      if (s.hsrec != nullptr && n <= cfg_.host_merge_rows && n <= 32 && ns <= 64) {
        sro.rec = s.dsrec;
        sro.seq = sig.seq;
        ro = RecOut();
        s.rec_mode = REC_SPLITS;
        s.rec_nsplit = ns;
      }
      // one launch covers at most LINEAR_SPLIT_MAX_ROWS rows (its ticket region): larger batches
      // (max_batch above it) go in row chunks, in order on one queue, sharing the workspace
      for (int64_t r0 = 0; r0 < n; r0 += LINEAR_SPLIT_MAX_ROWS) {
        const int64_t nb = std::min<int64_t>(LINEAR_SPLIT_MAX_ROWS, n - r0);
        RecOut roc = ro;
        if (roc.rec != nullptr) roc.rec += r0;
        launch_linear_split(m.xdt, static_cast<const unsigned char*>(X) + (size_t)r0 * m.ldx * dtype_size(m.xdt),
                            m.ldx, m.dW, static_cast<const float*>(m.db), nb, m.ldx, m.K, m.kind, s.didx + r0,
                            static_cast<float*>(s.dp) + r0, m.ws_split, m.ws_split_bytes, stream_, roc, sro,
                            direct_wide ? &dl : nullptr);
      }
    } else
      launch_gemm_softmax(X, m.dW, static_cast<const float*>(m.db), n, m.ldx, m.K, m.kind, s.didx,
                          static_cast<float*>(s.dp), m.ws, m.ws_bytes, stream_, ro);
    if (!s.rec_mode) launch_serve_signal(sig, stream_);
    direct_wide_used = dl.used;
  }
  const int64_t t_p3 = now_ns();
  std::lock_guard<std::mutex> lk(st_mu_);
  stats_.path_batches[m.path]++;
  if (bar) stats_.bar_batches++;
  if (direct_wide_used) stats_.direct_wide_batches++;
  stats_.launch_ns[0] += (double)(t_p1 - t_p0);
  stats_.launch_ns[1] += (double)(t_p2 - t_p1);
  stats_.launch_ns[2] += (double)(t_p3 - t_p2);
}

void Engine::batcher_loop() {
  pthread_setname_np(pthread_self(), "mlapi-batch");
  if (cfg_.device >= 0) (void)hipSetDevice(cfg_.device);
  std::vector<Meta> metas, chunk;
  std::vector<double> xs;
  metas.reserve(4096);
  chunk.reserve(4096);
  xs.reserve(4096 * 8);
  int64_t t_take = 0;
  for (;;) {
    if (cfg_.spin_us > 0 && q_count_.load(std::memory_order_acquire) == 0) {
      // Adaptive spin: under load the next request arrives within microseconds; polling the
      // queue counter avoids the submitter's futex wake (several us on the request path).
      const int64_t until = now_ns() + (int64_t)cfg_.spin_us * 1000;
      while (q_count_.load(std::memory_order_acquire) == 0 && now_ns() < until) _mm_pause();
    }
    {
      std::unique_lock<std::mutex> lk(q_mu_);
      const bool slept = q_meta_.empty();
      if (slept) ++batchers_sleeping_;
      q_cv_.wait(lk, [&] { return stopping_ || !q_meta_.empty(); });
      if (slept) --batchers_sleeping_;
      if (q_meta_.empty() && stopping_) break;  // (another batcher may have taken the last rows)
      if (cfg_.max_wait_us > 0 && (int)q_meta_.size() < cfg_.max_batch && !stopping_) {
        q_cv_.wait_for(lk, std::chrono::microseconds(cfg_.max_wait_us),
                       [&] { return stopping_ || (int)q_meta_.size() >= cfg_.max_batch; });
      }
      t_take = now_ns();
      metas.swap(q_meta_);
      xs.swap(q_x_);
      q_meta_.clear();
      q_x_.clear();
      q_count_.store(0, std::memory_order_release);
    }
    const std::shared_ptr<const Model> m = model();
    int64_t t_prev = now_ns();
    double take_ns = (double)(t_prev - t_take);  // charged to the first batch of this take
    size_t pos = 0;
    while (pos < metas.size()) {
      const size_t n = std::min(metas.size() - pos, (size_t)cfg_.max_batch);
      // no allocation per batch: chunk and the slots' meta vectors trade buffers (s.metas.swap
      // below hands this one to the slot and takes back the slot's cleared one)
      chunk.assign(metas.begin() + pos, metas.begin() + pos + n);
      pos += n;
      if (cfg_.device < 0 || !m) {
        run_cpu(chunk, xs, m);
        continue;
      }
      // ---- GPU path: acquire a slot, pack, launch
      int si;
      {
        std::unique_lock<std::mutex> lk(s_mu_);
        s_cv_.wait(lk, [&] { return !free_slots_.empty(); });
        si = free_slots_.front();
        free_slots_.pop_front();
      }
      const int64_t t_slot = now_ns();
      Slot& s = slots_[si];
      TraceRange tr("mlapi.batch.launch");
      s.metas.swap(chunk);
      s.model = m;
      s.n = (int)n;
      s.failed = false;
      s.launched = false;
      s.pre_status.assign(n, ST_OK);
      if (drop_.load(std::memory_order_relaxed)) {
        s.failed = true;
        healthy_.store(false);
      } else if (cfg_.fail_every > 0 && (++batch_counter_ % (uint64_t)cfg_.fail_every) == 0) {
        s.failed = true;
      } else {
        try {
          std::lock_guard<std::mutex> lk(launch_mu_);
          launch_batch(s, *m, xs);
          s.launched = true;
        } catch (const std::exception&) {
          s.failed = true;
          healthy_.store(false);
        }
      }
      s.t_launch = now_ns();
      {
        double qw = 0;
        for (const Meta& mt : s.metas) qw += (double)(s.t_launch - mt.t_enq);
        std::lock_guard<std::mutex> lk(st_mu_);
        stats_.queue_wait_us_sum += qw * 1e-3;
        stats_.batcher_ns[0] += take_ns;
        stats_.batcher_ns[1] += (double)(t_slot - t_prev);
        stats_.batcher_ns[2] += (double)(s.t_launch - t_slot);
      }
      take_ns = 0;
      {
        std::lock_guard<std::mutex> lk(s_mu_);
        inflight_.push_back(si);
        inflight_n_.fetch_add(1, std::memory_order_release);
      }
      s_cv_.notify_all();
      const int64_t t_end = now_ns();
      {
        std::lock_guard<std::mutex> lk(st_mu_);
        stats_.batcher_ns[3] += (double)(t_end - s.t_launch);
      }
      t_prev = t_end;
    }
    metas.clear();
    xs.clear();
  }
  {
    std::lock_guard<std::mutex> lk(s_mu_);
    ++batchers_done_;
  }
  s_cv_.notify_all();
}

// Spin on the slot's done word (the kernel publishes s.seq with a system-scope release); back off
// after ~50 us, check the stream / direct queue for a fault now and then, and give up on the batch
// (ST_DEVICE_ERROR) after 10x the watchdog.
namespace {
// One 16-byte load (atomic on x86-64 with AVX): seq, idx and p of a record from the same store.
inline __m128i load_record(const ServeRecord* r) {
  asm volatile("" ::: "memory");  // re-read every poll
  return _mm_load_si128(reinterpret_cast<const __m128i*>(r));
}
}  // namespace

void Engine::wait_done(Slot& s) {
  const int si = (int)(&s - slots_.data());
  volatile uint32_t* dw = done_h_ + (size_t)si * SIGNAL_STRIDE;
  const int64_t t0 = now_ns();
  uint32_t spins = 0;
  int next_row = 0;  // record mode: rows [0, next_row) seen complete
  const int nrec = s.rec_mode == REC_SPLITS ? s.rec_nsplit * s.n : s.rec_mode == REC_WIDE ? 2 * s.rec_nsplit * s.n : s.n;
  auto done = [&]() -> bool {
    if (!s.rec_mode) return __atomic_load_n(dw, __ATOMIC_ACQUIRE) == s.seq;
    if (s.rec_mode == REC_WIDE) {  // unit k: block k / (2n), row (k / 2) % n, half k % 2 (at [block][32][2])
      const WideRecord* base = reinterpret_cast<const WideRecord*>(s.hsrec);
      while (next_row < nrec) {
        const int cb = next_row / (2 * s.n), rem = next_row - cb * 2 * s.n;
        const WideRecord* r = base + ((size_t)cb * 32 + rem / 2) * 2 + (rem & 1);
        if ((uint32_t)_mm_cvtsi128_si32(load_record(reinterpret_cast<const ServeRecord*>(r))) != s.seq) break;
        ++next_row;
      }
      return next_row == nrec;
    }
    if (s.rec_mode == REC_SPLITS) {  // record k: split k / n, row k % n (at [split][32])
      while (next_row < nrec) {
        const int sp = next_row / s.n, row = next_row - sp * s.n;
        const SplitRecord* r = s.hsrec + (size_t)sp * 32 + row;
        if ((uint32_t)_mm_cvtsi128_si32(load_record(reinterpret_cast<const ServeRecord*>(r))) != s.seq) break;
        ++next_row;
      }
      return next_row == nrec;
    }
    while (next_row < s.n && (uint32_t)_mm_cvtsi128_si32(load_record(s.hrec + next_row)) == s.seq) ++next_row;
    return next_row == s.n;
  };
  while (!done()) {
    ++spins;
    if (spins < 20000) {
      _mm_pause();
      continue;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(spins < 40000 ? 2 : 50));
    if ((spins & 63) == 0) {
      const hipError_t q = hipStreamQuery(stream_);
      if ((q != hipSuccess && q != hipErrorNotReady) || (direct_ && direct_->faulted())) {
        s.failed = true;
        healthy_.store(false);
        return;
      }
      const int64_t waited = now_ns() - t0;
      if (cfg_.watchdog_ms > 0 && waited > (int64_t)cfg_.watchdog_ms * 1000000) healthy_.store(false);
      if (cfg_.watchdog_ms > 0 && waited > (int64_t)cfg_.watchdog_ms * 10000000) {
        s.failed = true;
        return;
      }
    }
  }
}

const int32_t* Engine::collect(Slot& s, std::vector<int32_t>& st, std::vector<double>& pd, std::vector<int32_t>& idx) {
  const size_t n = (size_t)s.n;
  st.assign(s.pre_status.begin(), s.pre_status.end());
  pd.resize(n);
  if (s.failed) {
    std::fill(st.begin(), st.end(), (int32_t)ST_DEVICE_ERROR);
    std::fill(pd.begin(), pd.end(), 0.0);
    idx.assign(n, 0);
    return idx.data();
  }
  if (s.rec_mode == REC_WIDE) {
    // host merge of linear_wide's per-class-block f64 states, in block order
    idx.resize(n);
    const bool ovr = s.model->kind == KIND_OVR;
    const int ncb = s.rec_nsplit;
    const WideRecord* base = reinterpret_cast<const WideRecord*>(s.hsrec);
    for (size_t i = 0; i < n; ++i) {
      alignas(16) WideRecord r[128];
      for (int cb = 0; cb < ncb; ++cb)
        for (int u = 0; u < 2; ++u)
          _mm_store_si128(reinterpret_cast<__m128i*>(&r[2 * cb + u]),
                          load_record(reinterpret_cast<const ServeRecord*>(base + ((size_t)cb * 32 + i) * 2 + u)));
      pd[i] = merge_wide_records(r, ncb, ovr, &idx[i]);
    }
    return idx.data();
  }
  if (s.rec_mode == REC_SPLITS) {
    // host merge of the class-split kernel's per-block states, in block order (deterministic), in
    // double: max (first max wins on ties, like numpy's argmax), then the rescaled sums
    idx.resize(n);
    const bool ovr = s.model->kind == KIND_OVR;
    const int ns = s.rec_nsplit;
    for (size_t i = 0; i < n; ++i) {
      alignas(16) SplitRecord r[64];
      for (int sp = 0; sp < ns; ++sp)
        _mm_store_si128(reinterpret_cast<__m128i*>(&r[sp]),
                        load_record(reinterpret_cast<const ServeRecord*>(s.hsrec + (size_t)sp * 32 + i)));
      pd[i] = merge_split_records(r, ns, ovr, &idx[i]);
    }
    return idx.data();
  }
  if (s.rec_mode) {
    idx.resize(n);
    for (size_t i = 0; i < n; ++i) {
      alignas(16) ServeRecord r;
      _mm_store_si128(reinterpret_cast<__m128i*>(&r), load_record(s.hrec + i));
      idx[i] = r.idx;
      pd[i] = r.p;
    }
    xcd_check(idx.data(), st, pd);
    return idx.data();
  }
  if (s.model->pdt == DT_F64) {
    std::memcpy(pd.data(), s.hp, n * sizeof(double));
  } else {
    const float* pf = static_cast<const float*>(s.hp);
    for (size_t i = 0; i < n; ++i) pd[i] = pf[i];
  }
  xcd_check(s.hidx, st, pd);
  return s.hidx;
}

// Rows an XCD-local split merge marked as misplaced (XCD_BAD_IDX: a partial came from another
// XCD's L2, so the merged state may be stale) fail with ST_DEVICE_ERROR instead of answering, and
// the protocol is switched off for the device: every later launch uses the agent-scope merge.
void Engine::xcd_check(const int32_t* idx, std::vector<int32_t>& st, std::vector<double>& pd) {
  uint64_t bad = 0, timeouts = 0;
  for (size_t i = 0; i < st.size(); ++i)
    if (idx[i] == XCD_BAD_IDX || idx[i] == WIDE_TIMEOUT_IDX) {
      st[i] = ST_DEVICE_ERROR;
      pd[i] = 0.0;
      ++(idx[i] == XCD_BAD_IDX ? bad : timeouts);
    }
  if (timeouts != 0)
    std::fprintf(stderr, "[mlapi] wide class merge timed out: %llu row(s) failed\n", (unsigned long long)timeouts);
  if (bad == 0) return;
  xcd_local_report_error(cfg_.device);
  std::fprintf(stderr, "[mlapi] XCD-local split merge read a misplaced partial: %llu row(s) failed, protocol off\n",
               (unsigned long long)bad);
  std::lock_guard<std::mutex> lk(st_mu_);
  stats_.xcd_errors += bad;
}

namespace {
struct CollectSink : Sink {
  std::vector<Completion>* out;
  void on_complete(const Completion* c, size_t n, const std::shared_ptr<const Model>&) override {
    out->insert(out->end(), c, c + n);
  }
};
}  // namespace

// Idle-engine fast path. At batch = 1 the queued path costs two thread hand-offs before the
// response can be written (submitter -> batcher futex wake, completer -> submitter eventfd wake),
// several us each; with nothing queued or in flight there is no batch to join, so the submitting
// thread launches and waits itself. The check is a heuristic (a request submitted by another
// thread right after it simply takes the queued path and runs concurrently in another slot).
bool Engine::run_idle(const double* X, int n, int nf, const uint64_t* tags, std::vector<Completion>& out,
                      std::shared_ptr<const Model>& m_out, bool allow_wide) {
  if (cfg_.idle_inline_rows <= 0 || n <= 0 || n > cfg_.idle_inline_rows) return false;
  if (nf < 0 || nf > cfg_.max_features) return false;
  if (drop_.load(std::memory_order_relaxed) || cfg_.fail_every > 0 || cfg_.delay_us > 0) return false;
  if (inflight_n_.load(std::memory_order_acquire) != 0) return false;
  std::shared_ptr<const Model> m = model();
  // SMALL models only: their batches are kernel-argument packets (~0.03 us to dispatch) with a
  // ~4 us GPU leg. Wide models are bound by the IO threads' JSON parsing; blocking one on a GEMV /
  // GEMM launch + leg cost c=64 throughput (F=256 binary: 265k vs 306-310k req/s) - unless the
  // caller vouches for low load (allow_wide).
  if (!m || (m->path != PATH_SMALL && !allow_wide)) return false;
  const int64_t t = now_ns();
  {
    std::lock_guard<std::mutex> lk(q_mu_);
    if (stopping_ || !q_meta_.empty() || batchers_sleeping_ < (int)batchers_.size()) return false;
  }
  CollectSink sink;
  sink.out = &out;
  if (cfg_.device < 0) {  // CPU backend: the float64 oracle, in this thread
    thread_local std::vector<Meta> metas;
    thread_local std::vector<double> xs;
    xs.assign(X, X + (size_t)n * nf);
    metas.clear();
    for (int i = 0; i < n; ++i) metas.push_back(Meta{tags[i], &sink, t, nf, i * nf});
    run_cpu(metas, xs, m);
    {
      std::lock_guard<std::mutex> lk(st_mu_);
      stats_.idle_batches++;
    }
    m_out = std::move(m);
    return true;
  }
  int si;
  {
    std::lock_guard<std::mutex> lk(s_mu_);
    if (free_slots_.empty() || !inflight_.empty()) return false;
    si = free_slots_.front();
    free_slots_.pop_front();
  }
  Slot& s = slots_[si];
  thread_local std::vector<double> xs;
  xs.assign(X, X + (size_t)n * nf);
  s.metas.clear();
  for (int i = 0; i < n; ++i) s.metas.push_back(Meta{tags[i], nullptr, t, nf, i * nf});
  s.model = m;
  s.n = n;
  s.failed = false;
  s.launched = false;
  s.pre_status.assign((size_t)n, ST_OK);
  try {
    std::lock_guard<std::mutex> lk(launch_mu_);
    launch_batch(s, *m, xs);
    s.launched = true;
  } catch (const std::exception&) {
    s.failed = true;
    healthy_.store(false);
  }
  s.t_launch = now_ns();
  if (s.launched) wait_done(s);
  const int64_t now = now_ns();
  thread_local std::vector<int32_t> st, ix;
  thread_local std::vector<double> pd;
  const int32_t* idx = collect(s, st, pd, ix);
  {
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.device_us_sum += (double)(now - s.t_launch) * 1e-3;
    stats_.idle_batches++;
  }
  record_batch((size_t)n);
  for (Meta& mt : s.metas) mt.sink = &sink;
  deliver(s.metas, idx, pd.data(), st.data(), m, now);
  s.metas.clear();
  s.model.reset();
  m_out = std::move(m);
  {
    std::lock_guard<std::mutex> lk(s_mu_);
    free_slots_.push_back(si);
  }
  s_cv_.notify_all();
  return true;
}

void Engine::completer_loop() {
  pthread_setname_np(pthread_self(), "mlapi-compl");
  (void)hipSetDevice(cfg_.device);
  std::vector<int32_t> st, ix;
  std::vector<double> pd;
  std::vector<Meta> dmetas;  // the batch being delivered, after its slot went back to the batcher
  dmetas.reserve(4096);
  for (;;) {
    int si;
    if (cfg_.spin_us > 0 && inflight_n_.load(std::memory_order_acquire) == 0) {
      // as the batcher: poll for the next launched batch before paying a futex wake
      const int64_t until = now_ns() + (int64_t)cfg_.spin_us * 1000;
      while (inflight_n_.load(std::memory_order_acquire) == 0 && now_ns() < until) _mm_pause();
    }
    {
      std::unique_lock<std::mutex> lk(s_mu_);
      s_cv_.wait(lk, [&] { return !inflight_.empty() || batchers_done_ >= (int)batchers_.size(); });
      if (inflight_.empty()) break;  // batcher has exited and nothing is in flight
      si = inflight_.front();
      inflight_.pop_front();
      inflight_n_.fetch_sub(1, std::memory_order_relaxed);
    }
    Slot& s = slots_[si];
    const int64_t t_w0 = now_ns();
    if (s.launched) {
      TraceRange tw("mlapi.batch.wait_gpu");
      wait_done(s);
    }
    if (cfg_.delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(cfg_.delay_us));
    TraceRange td("mlapi.batch.deliver");
    const int64_t now = now_ns();
    const size_t n = (size_t)s.n;
    const int32_t* idx = collect(s, st, pd, ix);
    if (idx != ix.data()) {  // results still in the slot's buffers: copy them out
      ix.assign(idx, idx + n);
      idx = ix.data();
    }
    {
      std::lock_guard<std::mutex> lk(st_mu_);
      stats_.device_us_sum += (double)(now - s.t_launch) * 1e-3;
    }
    record_batch(n);
    std::shared_ptr<const Model> m = std::move(s.model);
    // The slot goes back to the batcher BEFORE the delivery: waking the batch's IO threads (an
    // eventfd write per sink, ~1 us each with a sleeping reader) measured ~6 us per batch, and
    // while it ran the slot was not free, so the batcher queued behind it (engine stage clocks,
    // profiles/r3_s16).
    dmetas.swap(s.metas);
    {
      std::lock_guard<std::mutex> lk(s_mu_);
      free_slots_.push_back(si);
    }
    s_cv_.notify_all();
    deliver(dmetas, idx, pd.data(), st.data(), m, now);
    dmetas.clear();
    {
      const int64_t t_d1 = now_ns();
      std::lock_guard<std::mutex> lk(st_mu_);
      stats_.completer_ns[0] += (double)(now - t_w0);
      stats_.completer_ns[1] += (double)(t_d1 - now);
    }
  }
}

// ---- resident SMALL-path kernel: per-IO-thread rings (ServeRing) and the supervisor ---------------
namespace {
// Engines with a resident kernel: a process that exits without stopping its engines (interpreter
// exit with a server still up) halts their instances first, so no wave is still polling when the
// HIP runtime tears the queues down (the lease rule would end it within resident_lease_ms anyway).
std::mutex g_res_mu;
std::vector<Engine*>& res_engines() {
  static std::vector<Engine*>* v = new std::vector<Engine*>();  // never destroyed: used at exit
  return *v;
}
void halt_residents_at_exit() {
  std::lock_guard<std::mutex> lk(g_res_mu);
  for (Engine* e : res_engines()) e->resident_halt(500);
}
}  // namespace

void Engine::resident_register(bool on) {
  static bool hooked = false;
  std::lock_guard<std::mutex> lk(g_res_mu);
  auto& v = res_engines();
  if (on) {
    v.push_back(this);
    if (!hooked) {
      hooked = true;
      std::atexit(halt_residents_at_exit);
    }
  } else {
    v.erase(std::remove(v.begin(), v.end(), this), v.end());
  }
}

void Engine::resident_halt(int timeout_ms) {
  // under the instance lock: a launch that already passed its halt check cannot clear this stop
  // afterwards, and the dispatcher's resident queue / signal are not swapped under the wait
  std::lock_guard<std::mutex> lk(res_inst_mu_);
  res_halt_.store(true, std::memory_order_release);  // the supervisor launches nothing from now on
  res_live_.store(false, std::memory_order_release);
  if (res_ctl_h_ == nullptr) return;
  __atomic_store_n(&res_ctl_h_->fault, (uint32_t)RES_FAULT_NONE, __ATOMIC_RELAXED);  // an injected ignore-stop too
  __atomic_store_n(&res_ctl_h_->stop, 1u, __ATOMIC_RELEASE);
  if (!res_cpu_ && direct_) (void)direct_->resident_wait(timeout_ms);
}

ServeRing* Engine::open_ring() {
  if (cfg_.resident <= 0 || res_ctl_h_ == nullptr) return nullptr;
  ServeRing* r = nullptr;
  {
    std::lock_guard<std::mutex> lk(rings_mu_);
    if (!free_rings_.empty()) {
      r = free_rings_.back();
      free_rings_.pop_back();
    } else if ((int)rings_.size() < RESIDENT_MAX_RINGS) {
      rings_.push_back(std::unique_ptr<ServeRing>(new ServeRing(this, (int)rings_.size())));
      r = rings_.back().get();
      rings_open_.store((int)rings_.size(), std::memory_order_release);
    }
  }
  if (r != nullptr) kick_resident();  // a new ring: the instance's grid grows
  return r;
}

void Engine::close_ring(ServeRing* ring) {
  if (ring == nullptr) return;
  std::vector<Completion> c;
  std::vector<ServeRing::Seg> segs;
  const int64_t until = now_ns() + 2000000000LL;
  int rq = 0;
  while (ring->poll(c, segs, nullptr, &rq) > 0 && now_ns() < until) {
    c.clear();
    segs.clear();
    _mm_pause();
  }
  // rows still pending after 2 s: poisoned, with their tags and models dropped, so the ring's next
  // owner (another IO thread, whose connection ids overlap this one's) never renders their answers
  // and never rewrites their slots before the GPU is done with them
  const int gave_up = ring->abandon_pending();
  if (gave_up > 0) {
    healthy_.store(false);
    std::fprintf(stderr, "[mlapi engine] resident ring %d closed with %d rows unanswered\n", ring->idx_, gave_up);
  }
  std::lock_guard<std::mutex> lk(rings_mu_);
  free_rings_.push_back(ring);
}

int ServeRing::abandon_pending() {
  int n = 0;
  for (uint32_t pos = tail_; pos != next_; ++pos) {
    Pend& p = pend_[pos & (RESIDENT_RING - 1)];
    if (!p.live) continue;
    p.live = false;
    p.poisoned = true;
    p.tag = 0;
    p.model.reset();
    ++n;
  }
  live_n_ = 0;
  tail_ = next_;
  return n;
}

bool ServeRing::reclaim(Pend& p) {
  if (!p.poisoned) return true;
  if (!landed(p.pos)) return false;
  p.poisoned = false;
  return true;
}

ServeRing::ServeRing(Engine* e, int index) : eng_(e), idx_(index) {
  ring_ = reinterpret_cast<ResidentGranule*>(e->res_rings_h_ + (size_t)index * RESIDENT_RING * RESIDENT_ENTRY_BYTES);
  rec_ = e->res_recs_h_ + (size_t)index * RESIDENT_RING;
  // positions continue from the ring's head (a pooled ring keeps next_ itself)
  next_ = tail_ = __atomic_load_n(&e->res_ctl_h_->heads[index], __ATOMIC_ACQUIRE);
}

// A record is {seq, idx, p} from one 16-byte store (kernel) or p, idx then seq (CPU backend); its slot
// is rewritten only after this thread consumed it, so seq (acquire) then idx / p is consistent.
bool ServeRing::landed(uint32_t pos) const {
  return __atomic_load_n(&rec_[pos & (RESIDENT_RING - 1)].seq, __ATOMIC_ACQUIRE) == pos;
}

bool ServeRing::submit(const double* X, int n, int nf, const uint64_t* tags) {
  Engine& e = *eng_;
  // measurement: MLAPI_RESIDENT_SHADOW=1 keeps the resident kernel polling while every row takes the
  // engine queue (the polling's cost to the host, isolated from the path itself)
  static const bool shadow = [] {
    const char* v = getenv("MLAPI_RESIDENT_SHADOW");
    return v != nullptr && atoi(v) != 0;
  }();
  if (shadow) return false;
  if (n <= 0 || n > RESIDENT_RING / 2 || next_ - tail_ + (uint32_t)n > (uint32_t)RESIDENT_RING) return false;
  if (!e.res_live_.load(std::memory_order_acquire) || idx_ >= e.res_nrings_.load(std::memory_order_acquire)) return false;
  if (e.drop_.load(std::memory_order_relaxed) || e.cfg_.fail_every > 0 || e.cfg_.delay_us > 0) return false;
  std::shared_ptr<const Model> m = e.model();
  const uint32_t mver = e.res_mver_.load(std::memory_order_acquire);
  if (!m || m->path != PATH_SMALL || nf != m->F || resident_mver(m->version) != mver) return false;
  // slots of given-up rows are not rewritten until their late records land (the GPU may still
  // read the entry and answer it)
  for (int i = 0; i < n; ++i)
    if (!reclaim(pend_[(next_ + (uint32_t)i) & (RESIDENT_RING - 1)])) return false;
  const int64_t t = now_ns();
  const uint32_t meta = mver << 8 | (uint32_t)nf;
  for (int i = 0; i < n; ++i) {
    const uint32_t pos = next_ + (uint32_t)i;
    const uint32_t ei = pos & (RESIDENT_RING - 1);
    Pend& p = pend_[ei];
    p.tag = tags[i];
    p.t_enq = t;
    p.model = m;
    p.pos = pos;
    p.nf = nf;
    p.live = true;
    // every granule {x_f, pos, meta}: the value, then its tag word (x86 stores become visible in
    // program order, and the wave reads each 16-byte granule in one load, so a granule whose tag
    // it sees carries this row's value); the wave accepts the row once all F tags carry this position
    ResidentGranule* g = ring_ + (size_t)ei * RESIDENT_FMAX;
    const uint64_t tag = (uint64_t)meta << 32 | pos;
    for (int f = 0; f < nf; ++f) {
      g[f].x = X[(size_t)i * nf + f];
      __atomic_store_n(reinterpret_cast<uint64_t*>(&g[f].pos), tag, __ATOMIC_RELEASE);
    }
  }
  next_ += (uint32_t)n;
  live_n_ += n;
  return true;
}

bool ServeRing::wait_any(int64_t ns) const {
  if (tail_ == next_) return false;
  const int64_t until = now_ns() + ns;
  for (;;) {
    for (uint32_t pos = tail_; pos != next_; ++pos) {
      const Pend& p = pend_[pos & (RESIDENT_RING - 1)];
      if (p.live && landed(pos)) return true;
    }
    if (now_ns() >= until) return false;
    for (int i = 0; i < 8; ++i) _mm_pause();
  }
}

int ServeRing::poll(std::vector<Completion>& out, std::vector<Seg>& segs, Sink* sink, int* requeued) {
  Engine& e = *eng_;
  if (tail_ == next_) return 0;
  const int64_t now = now_ns();
  const int64_t wd = (int64_t)e.cfg_.watchdog_ms * 1000000;
  int done = 0, errors = 0, stale = 0;
  double lat_sum = 0;
  uint64_t lat_hist[24] = {0};
  const Model* last = nullptr;
  for (uint32_t pos = tail_; pos != next_; ++pos) {
    Pend& p = pend_[pos & (RESIDENT_RING - 1)];
    if (!p.live) continue;
    const ServeRecord* rp = rec_ + (pos & (RESIDENT_RING - 1));
    ServeRecord r{};
    r.seq = __atomic_load_n(&rp->seq, __ATOMIC_ACQUIRE);
    if (r.seq == pos) {
      r.idx = rp->idx;
      r.p = rp->p;
    }
    bool fail = false;
    if (r.seq != pos) {
      const int64_t waited = now - p.t_enq;
      if (wd > 0 && waited > 10 * wd) {
        fail = true;  // the record may still land later: this slot is never written again
      } else {
        if (wd > 0 && waited > wd) {
          // this ring's wave stopped answering (it exited or hung while block 0 still beats): the
          // supervisor restarts the instance, whose waves resume from the published ring heads
          e.healthy_.store(false);
          if (!e.res_ring_stall_.exchange(true)) e.kick_resident();
        }
        continue;
      }
    }
    if (!fail && r.idx == RESIDENT_STALE_IDX) {
      // parsed for another model version: the engine queue answers it with the current model
      ++stale;
      const ResidentGranule* g = ring_ + (size_t)(pos & (RESIDENT_RING - 1)) * RESIDENT_FMAX;
      double x[RESIDENT_FMAX];
      for (int f = 0; f < p.nf; ++f) x[f] = g[f].x;
      const uint64_t tag = p.tag;
      p.live = false;
      p.model.reset();
      --live_n_;
      if (sink != nullptr) {
        const int k = e.submit_many(x, 1, p.nf, &tag, sink);
        if (k == 1) {
          ++*requeued;
          continue;
        }
      }
      // not accepted (stopping / backpressure / no sink): answered as a device error
      out.push_back(Completion{tag, 0, (int32_t)ST_DEVICE_ERROR, 0.0, now - p.t_enq});
      if (segs.empty() || last != nullptr) {
        segs.push_back(Seg{out.size() - 1, nullptr});
        last = nullptr;
      }
      ++errors;
      ++done;
      continue;
    }
    int32_t st = fail ? (int32_t)ST_DEVICE_ERROR : (int32_t)ST_OK;
    const int32_t idx = fail ? 0 : r.idx;
    const double pv = fail ? 0.0 : r.p;
    if (st == ST_OK && !std::isfinite(pv)) st = ST_NONFINITE;
    if (fail) {
      e.healthy_.store(false);
      p.poisoned = true;
    }
    errors += st != ST_OK;
    if (segs.empty() || p.model.get() != last) {
      segs.push_back(Seg{out.size(), p.model});
      last = p.model.get();
    }
    const int64_t lat = now - p.t_enq;
    out.push_back(Completion{p.tag, idx, st, pv, lat});
    const double us = (double)lat * 1e-3;
    lat_sum += us;
    int b = 0;
    while (b < 23 && (double)(int64_t(1) << b) <= us) ++b;
    lat_hist[b]++;
    ++done;
    p.live = false;
    p.model.reset();
    --live_n_;
  }
  // consumed and given-up rows alike leave the window (a poisoned slot is reclaimed by submit once
  // its late record lands)
  while (tail_ != next_ && !pend_[tail_ & (RESIDENT_RING - 1)].live) ++tail_;
  if (done > 0 || stale > 0) {
    std::lock_guard<std::mutex> lk(e.st_mu_);
    e.stats_.requests += (uint64_t)done;
    e.stats_.errors += (uint64_t)errors;
    e.stats_.resident_rows += (uint64_t)(done - errors);
    e.stats_.resident_stale += (uint64_t)stale;
    e.stats_.latency_sum_us += lat_sum;
    for (int b = 0; b < 24; ++b) e.stats_.latency_hist[b] += lat_hist[b];
  }
  return live_n_;
}

namespace {
int resident_lpe(int F) { return F <= 4 ? 4 : F <= 8 ? 8 : 32; }
}  // namespace

bool Engine::resident_launch(const std::shared_ptr<const Model>& m, uint32_t mver, int nrings, bool bounce) {
  if (!res_fault_sticky_.load(std::memory_order_relaxed))  // injections are per instance unless sticky
    __atomic_store_n(&res_ctl_h_->fault, (uint32_t)RES_FAULT_NONE, __ATOMIC_RELAXED);
  if (res_cpu_) return true;  // the supervisor polls the rings itself
  if (!direct_) return false;
  ResidentArgs a{};
  a.rings = res_rings_d_;
  a.recs = res_recs_d_;
  a.ctl = res_ctl_d_;
  const int F = bounce ? 32 : m->F;
  const int lpe = resident_lpe(F);
  a.F = bounce ? lpe : m->F;
  a.K = bounce ? 0 : m->K;
  a.kind = bounce ? 0 : m->kind;
  a.W = bounce ? nullptr : m->dW;
  a.b = bounce ? nullptr : m->db;
  a.mver = bounce ? 0u : mver;
  a.lease_ticks = (uint64_t)std::max(20, cfg_.resident_lease_ms) * 100000ull;
  a.idle_exit_ticks = bounce ? 1000000ull : 0ull;  // the bounce instance: 10 ms without a row
  a.idle_polls = (uint32_t)std::max(1, cfg_.resident_idle_polls);
  a.idle_sleep = (uint32_t)std::max(0, cfg_.resident_idle_sleep);
  const int depth = cfg_.resident_depth >= 4 ? 4 : cfg_.resident_depth >= 2 ? 2 : 1;
  const bool f64 = bounce ? true : m->xdt == DT_F64;
  char name[64];
  std::snprintf(name, sizeof name, "mlapi_resident_%s_r%d_d%d", f64 ? "f64" : "f32", lpe, depth);
  std::lock_guard<std::mutex> lk(res_inst_mu_);
  if (res_halt_.load(std::memory_order_acquire)) return false;  // halted since the supervisor's check
  __atomic_store_n(&res_ctl_h_->stop, 0u, __ATOMIC_RELEASE);
  return direct_->resident_launch(name, &a, sizeof a, (unsigned)nrings, 64);
}

bool Engine::resident_stop_instance(int timeout_ms) {
  std::lock_guard<std::mutex> lk(res_inst_mu_);
  __atomic_store_n(&res_ctl_h_->stop, 1u, __ATOMIC_RELEASE);
  if (res_cpu_) return true;
  if (direct_->resident_wait(timeout_ms)) return true;
  // never ended: keep its memory alive and leave it to its lease (the supervisor stops bumping it
  // while res_leaked_ is set); its queue is freed and the path resumes once it has ended
  std::fprintf(stderr, "[mlapi engine] resident kernel did not stop within %d ms: abandoned to its lease\n",
               timeout_ms);
  direct_->resident_abandon(/*track=*/true);
  res_leaked_ = true;
  healthy_.store(false);
  std::lock_guard<std::mutex> sl(st_mu_);
  stats_.resident_abandoned++;
  return false;
}

bool Engine::resident_inject(int mode, int arg) {
  if (res_ctl_h_ == nullptr) return false;
  if (mode == RES_FAULT_NONE) {  // clear (a sticky injection too)
    res_fault_sticky_.store(false);
    __atomic_store_n(&res_ctl_h_->fault, (uint32_t)RES_FAULT_NONE, __ATOMIC_RELEASE);
    return true;
  }
  if (!res_live_.load(std::memory_order_acquire)) return false;
  if (mode == RES_INJECT_STALL_STICKY) {  // a hang that survives restarts: the rows' give-up path
    res_fault_sticky_.store(true);
    mode = RES_FAULT_STALL;
  }
  switch (mode) {
    case RES_FAULT_STALL:
    case RES_FAULT_EXIT_RING:
    case RES_FAULT_IGNORE_STOP:
      // the CPU backend's host poller plays a hang (STALL) but has no waves to exit or to ignore stop
      if (res_cpu_ && mode != RES_FAULT_STALL) return false;
      __atomic_store_n(&res_ctl_h_->fault_arg, (uint32_t)arg, __ATOMIC_RELAXED);
      __atomic_store_n(&res_ctl_h_->fault, (uint32_t)mode, __ATOMIC_RELEASE);
      return true;
    case RES_INJECT_LEASE_STARVE:
      res_starve_until_.store(now_ns() + (int64_t)std::max(0, arg) * 1000000);
      return true;
    case RES_INJECT_QUEUE_FAULT: {
      if (res_cpu_ || !direct_) return false;
      std::lock_guard<std::mutex> lk(res_inst_mu_);
      res_fault_queue_.store(true);
      direct_->inject_resident_fault();
      __atomic_store_n(&res_ctl_h_->stop, 1u, __ATOMIC_RELEASE);  // the instance ends; its queue reads as failed
      return true;
    }
    default:
      return false;
  }
}

// CPU backend: one pass of the resident kernel's protocol over every ring (the same tag rules).
int Engine::resident_cpu_poll(const std::shared_ptr<const Model>& m, uint32_t mver, int nrings, bool bounce) {
  // an injected hang: no row answered, no heartbeat (the watchdogs' tests on GPU-less hosts)
  if (__atomic_load_n(&res_ctl_h_->fault, __ATOMIC_ACQUIRE) == RES_FAULT_STALL) return 0;
  __atomic_store_n(&res_ctl_h_->heartbeat, res_ctl_h_->heartbeat + 1, __ATOMIC_RELAXED);
  int rows = 0;
  for (int r = 0; r < nrings; ++r) {
    uint32_t head = __atomic_load_n(&res_ctl_h_->heads[r], __ATOMIC_ACQUIRE);
    const ResidentGranule* ring =
        reinterpret_cast<const ResidentGranule*>(res_rings_h_ + (size_t)r * RESIDENT_RING * RESIDENT_ENTRY_BYTES);
    for (;;) {
      const ResidentGranule* g = ring + (size_t)(head & (RESIDENT_RING - 1)) * RESIDENT_FMAX;
      auto tag_of = [&](int f) {  // {pos, meta} of granule f (acquire: its value was written before)
        return __atomic_load_n(reinterpret_cast<const uint64_t*>(&g[f].pos), __ATOMIC_ACQUIRE);
      };
      const uint64_t t0 = tag_of(0);
      if ((uint32_t)t0 != head) break;
      const uint32_t meta = (uint32_t)(t0 >> 32);
      const int rf = (int)(meta & 0xffu);
      double x[RESIDENT_FMAX];
      bool full = rf >= 1 && rf <= RESIDENT_FMAX;
      for (int f = 0; f < rf && full; ++f) {
        full = (uint32_t)tag_of(f) == head;
        if (full) x[f] = g[f].x;
      }
      if (!full) break;
      // a hang injected while this call was already past its check answers nothing more
      if (__atomic_load_n(&res_ctl_h_->fault, __ATOMIC_ACQUIRE) == RES_FAULT_STALL) break;
      int32_t idx = RESIDENT_STALE_IDX;
      double p = 0.0;
      if (!bounce && m && (meta >> 8) == mver && rf == m->F) cpu_linear_predict(*m, x, 1, &idx, &p);
      ServeRecord* rc = res_recs_h_ + (size_t)r * RESIDENT_RING + (head & (RESIDENT_RING - 1));
      rc->idx = idx;
      rc->p = p;
      __atomic_store_n(&rc->seq, head, __ATOMIC_RELEASE);
      ++head;
      ++rows;
    }
    __atomic_store_n(&res_ctl_h_->heads[r], head, __ATOMIC_RELEASE);
  }
  return rows;
}

void Engine::resident_loop() {
  pthread_setname_np(pthread_self(), "mlapi-resid");
  if (cfg_.device >= 0) (void)hipSetDevice(cfg_.device);
  bool running = false;      // an instance is up
  bool inst_bounce = false;  // ... answering every row stale (no SMALL model to serve)
  uint32_t inst_mver = 0;
  int inst_rings = 0;
  std::shared_ptr<const Model> inst_model;
  uint64_t seen_kick = ~uint64_t(0);
  uint64_t last_hb = 0;
  int64_t t_hb = now_ns(), t_retry = 0, t_row = 0, t_ring_restart = 0;
  bool served = false;  // an instance has served rows that a successor may have to bounce
  auto set_live = [&](bool live) {
    res_live_.store(live, std::memory_order_release);
    std::lock_guard<std::mutex> lk(st_mu_);
    stats_.resident_live = live;
    stats_.resident_rings = running ? inst_rings : 0;
  };
  auto stop_inst = [&]() {
    res_live_.store(false, std::memory_order_release);
    if (running) resident_stop_instance(1000);
    running = false;
    inst_model.reset();
    set_live(false);
  };
  for (;;) {
    bool stopping;
    {
      std::unique_lock<std::mutex> lk(res_mu_);
      if (res_cpu_ && running) {
        lk.unlock();
        const int64_t t = now_ns();
        if (resident_cpu_poll(inst_model, inst_mver, inst_rings, inst_bounce) > 0 || t_row == 0) t_row = t;
        if (inst_bounce && t - t_row > 10000000) {  // the bounce instance's idle exit
          running = false;
          served = false;
          t_row = 0;
        }
        lk.lock();
      } else {
        res_cv_.wait_for(lk, std::chrono::milliseconds(10), [&] { return res_stop_ || res_kick_ != seen_kick; });
      }
      stopping = res_stop_;
      seen_kick = res_kick_;
    }
    // the lease: not while an abandoned instance (one that ignored its stop word) still owns the
    // rings - it then ends on the lease rule - and not while a starvation is injected
    if (!res_leaked_ && now_ns() >= res_starve_until_.load(std::memory_order_relaxed))
      __atomic_fetch_add(&res_ctl_h_->lease, 1u, __ATOMIC_RELEASE);
    if (res_leaked_) {
      // the resident path stays off until the abandoned instance has ended (its queue is then freed)
      bool done;
      {
        std::lock_guard<std::mutex> lk(res_inst_mu_);
        done = direct_->resident_abandoned_done();
      }
      if (stopping) break;
      if (!done) continue;
      std::fprintf(stderr, "[mlapi engine] abandoned resident kernel ended: resident path resumes\n");
      res_leaked_ = false;
    }
    bool ended = false;
    if (running && !res_cpu_) {
      std::lock_guard<std::mutex> lk(res_inst_mu_);
      ended = direct_->resident_wait(0);
      if (ended && direct_->resident_faulted()) {
        std::fprintf(stderr, "[mlapi engine] resident kernel queue error: restarting on a fresh queue\n");
        // an injected fault ended cleanly: its queue is freed once seen ended; a real one is forgotten
        direct_->resident_abandon(/*track=*/res_fault_queue_.exchange(false));
        healthy_.store(false);
        std::lock_guard<std::mutex> sl(st_mu_);
        stats_.resident_queue_faults++;
      }
      (void)direct_->resident_abandoned_done();
    }
    if (ended) {
      // ended by itself: the bounce instance's idle exit, a lease expiry (this thread starved), an
      // early wave exit or a fault
      running = false;
      if (inst_bounce) served = false;
      set_live(false);
      std::lock_guard<std::mutex> sl(st_mu_);
      stats_.resident_self_exits++;
    }
    if (stopping) {
      stop_inst();
      break;
    }
    const std::shared_ptr<const Model> m = model();
    const bool small = m && m->path == PATH_SMALL && m->F <= RESIDENT_FMAX && m->K <= 16;
    const uint32_t want = small ? resident_mver(m->version) : 0u;
    const int nr = rings_open_.load(std::memory_order_acquire);
    if (running && (inst_rings != nr || (inst_bounce ? small : want != inst_mver))) stop_inst();
    const int64_t now = now_ns();
    // (never next to an abandoned instance: it may still be polling the same rings)
    if (!running && nr > 0 && (small || served) && now >= t_retry && !res_leaked_ &&
        !res_halt_.load(std::memory_order_acquire)) {
      const bool bounce = !small;
      if (resident_launch(m, want, nr, bounce)) {
        running = true;
        inst_bounce = bounce;
        inst_mver = want;
        inst_rings = nr;
        inst_model = m;
        served = true;
        last_hb = __atomic_load_n(&res_ctl_h_->heartbeat, __ATOMIC_ACQUIRE);
        t_hb = now;
        t_row = 0;
        res_mver_.store(want, std::memory_order_release);
        res_nrings_.store(nr, std::memory_order_release);
        {
          std::lock_guard<std::mutex> lk(st_mu_);
          stats_.resident_launches++;
        }
        set_live(small);
      } else {
        // no resident kernel in the code object (or the queue failed): the batcher path serves
        t_retry = now + 1000000000LL;
        set_live(false);
      }
    }
    if (running && !inst_bounce && cfg_.watchdog_ms > 0) {
      const uint64_t hb = __atomic_load_n(&res_ctl_h_->heartbeat, __ATOMIC_ACQUIRE);
      if (hb != last_hb) {
        last_hb = hb;
        t_hb = now;
      } else if (now - t_hb > (int64_t)cfg_.watchdog_ms * 1000000) {
        // the waves stopped polling: off the request path, restart (a fresh queue if it never ends)
        std::fprintf(stderr, "[mlapi engine] resident kernel heartbeat stalled: restarting\n");
        healthy_.store(false);
        stop_inst();
        t_hb = now;
        t_ring_restart = now;
        std::lock_guard<std::mutex> sl(st_mu_);
        stats_.resident_hb_restarts++;
      }
    }
    if (res_ring_stall_.load(std::memory_order_relaxed)) {
      // a ring's row waited past the watchdog: restart the instance (at most once per watchdog
      // period; an instance that is not running is relaunched above anyway)
      const bool act = running && !inst_bounce && now - t_ring_restart > (int64_t)cfg_.watchdog_ms * 1000000;
      if (act || !running) res_ring_stall_.store(false);
      if (act) {
        std::fprintf(stderr, "[mlapi engine] resident ring stalled: restarting the instance\n");
        stop_inst();
        t_ring_restart = now;
        t_hb = now;
        std::lock_guard<std::mutex> sl(st_mu_);
        stats_.resident_ring_restarts++;
      }
    }
  }
}

EngineStats Engine::stats() const {
  EngineStats s;
  {
    std::lock_guard<std::mutex> lk(st_mu_);
    s = stats_;
  }
  {
    std::lock_guard<std::mutex> lk(const_cast<std::mutex&>(q_mu_));
    s.queue_depth = q_meta_.size();
  }
  s.healthy = healthy_.load();
  s.dropped = drop_.load();
  if (res_ctl_h_ != nullptr) s.resident_heartbeat = __atomic_load_n(&res_ctl_h_->heartbeat, __ATOMIC_RELAXED);
  s.direct_dispatch = direct_ != nullptr;
  s.direct_device_kernargs = direct_ != nullptr && direct_->device_kernargs();
  return s;
}

}  // namespace mlapi
