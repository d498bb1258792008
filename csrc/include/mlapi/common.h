// Shared definitions between the HIP kernels, the C++ runtime and the Python bindings.
// Model kinds mirror mlapi_amd/models/linear.py::Kind (sklearn predict/predict_proba semantics,
// SURVEY Appendix B; reference call sites main.py:21-22).
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

namespace mlapi {

enum Kind : int32_t {
  KIND_BINARY = 0,          // p_max = sigmoid(|z|), label = z > 0
  KIND_BINARY_SOFTMAX = 1,  // softmax([-z, z]) -> p_max = sigmoid(2|z|)
  KIND_MULTINOMIAL = 2,     // p_max = 1 / sum_k exp(z_k - z_max), label = first argmax
  KIND_OVR = 3,             // p_k = sigmoid(z_k) / sum_j sigmoid(z_j)
};

enum DType : int32_t { DT_F64 = 0, DT_F32 = 1, DT_BF16 = 2 };

inline size_t dtype_size(int dt) { return dt == DT_F64 ? 8 : dt == DT_F32 ? 4 : 2; }

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

}  // namespace mlapi

#define MLAPI_HIP_CHECK(expr)                                                                  \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) {                                                                    \
      throw ::mlapi::HipError(std::string(#expr " failed: ") + hipGetErrorString(_e) + " at " + \
                              __FILE__ + ":" + std::to_string(__LINE__));                      \
    }                                                                                          \
  } while (0)
