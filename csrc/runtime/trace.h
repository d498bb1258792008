// Optional roctx ranges (SURVEY 5.1 tracing). libroctx64 is dlopen'ed lazily so the extension has
// no hard dependency on it; ranges are emitted only when MLAPI_ROCTX=1, so a normal run pays one
// relaxed atomic load per range. Visible in `rocprofv3 --marker-trace` timelines.
#pragma once
#include <dlfcn.h>

#include <atomic>
#include <cstdlib>

namespace mlapi {

struct Roctx {
  using push_fn = int (*)(const char*);
  using pop_fn = int (*)();
  push_fn push = nullptr;
  pop_fn pop = nullptr;
  bool enabled = false;

  static Roctx& get() {
    static Roctx r = [] {
      Roctx x;
      const char* e = std::getenv("MLAPI_ROCTX");
      if (e && e[0] == '1') {
        // rocprofiler-sdk's roctx first: rocprofv3 --marker-trace intercepts that library (the
        // legacy libroctx64 ranges are not recorded by rocprofv3)
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
          x.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
          x.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
          x.enabled = x.push && x.pop;
        }
      }
      return x;
    }();
    return r;
  }
};

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(Roctx::get().enabled) {
    if (on_) Roctx::get().push(name);
  }
  ~TraceRange() {
    if (on_) Roctx::get().pop();
  }

 private:
  bool on_;
};

}  // namespace mlapi
