// Host launchers of the binary GEMV predict (gemv_binary.h: design and roofline).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <stdexcept>

#include "gemv_binary.h"

namespace mlapi {
namespace {

using gemv::Chunk;
using gemv::GemvArgs;

template <typename T, int LPR, int CPL, int U>
__global__ __launch_bounds__(256) void gemv_binary_kernel(GemvArgs a) {
  gemv::gemv_rows<T, LPR, CPL, U>(a);
}

template <typename T, int LPR, int CPL, int U>
void launch(GemvArgs a, hipStream_t stream, KernelLauncher* direct) {
  constexpr int rows_per_block_iter = 4 * U * (64 / LPR);
  int64_t blocks = (a.B + rows_per_block_iter - 1) / rows_per_block_iter;
  const int64_t cap = 256 * 8;  // 256 CUs x 8 resident blocks: grid-stride beyond that
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  a.blocks = (int32_t)blocks;
  if (direct != nullptr) {
    // the same kernel, unmangled, in the serving code object (serve_direct.hip)
    char name[64];
    std::snprintf(name, sizeof name, "mlapi_gemv_%s_l%d_c%d_u%d", sizeof(T) == 2 ? "bf16" : "f32", LPR, CPL, U);
    // results go out as write-through records (the engine passes `direct` only then): unordered
    if (direct->launch_kernel(name, &a, sizeof a, (unsigned)blocks, 1, 256, false)) return;
  }
  hipLaunchKernelGGL((gemv_binary_kernel<T, LPR, CPL, U>), dim3((unsigned)blocks), dim3(256), 0, stream, a);
  MLAPI_HIP_CHECK(hipGetLastError());
}

template <typename T>
void dispatch(const GemvArgs& a, hipStream_t stream, KernelLauncher* direct) {
  constexpr int NE = Chunk<T>::N;
  if (a.F % NE != 0) throw std::invalid_argument("gemv_binary: F must be a multiple of 16 bytes of elements");
  const int chunks = a.F / NE;
  if (chunks <= 4)
    launch<T, 4, 1, 4>(a, stream, direct);
  else if (chunks <= 8)
    launch<T, 8, 1, 8>(a, stream, direct);
  else if (chunks <= 16)
    launch<T, 16, 1, 8>(a, stream, direct);
  else if (chunks <= 32)
    launch<T, 32, 1, 8>(a, stream, direct);
  else if (chunks <= 64)
    launch<T, 64, 1, 8>(a, stream, direct);
  else if (chunks <= 128)
    launch<T, 64, 2, 4>(a, stream, direct);
  else if (chunks <= 256)
    launch<T, 64, 4, 2>(a, stream, direct);
  else if (chunks <= 512)
    launch<T, 64, 8, 1>(a, stream, direct);
  else
    throw std::invalid_argument("gemv_binary: F too large (max 4096 bf16 / 2048 f32)");
}

}  // namespace

void launch_gemv_binary(int dt, const void* X, const void* w, float bias, int64_t B, int F, int kind,
                        int32_t* out_idx, float* out_p, hipStream_t stream, RecOut ro, KernelLauncher* direct) {
  if (B <= 0) return;
  if (reinterpret_cast<uintptr_t>(X) % 16 || reinterpret_cast<uintptr_t>(w) % 16)
    throw std::invalid_argument("gemv_binary: X and w must be 16-byte aligned");
  GemvArgs a{};
  a.X = X;
  a.w = w;
  a.bias = bias;
  a.F = F;
  a.B = B;
  a.kind = kind;
  a.out_idx = out_idx;
  a.out_p = out_p;
  a.ro = ro;
  if (dt == DT_BF16)
    dispatch<uint16_t>(a, stream, direct);
  else if (dt == DT_F32)
    dispatch<float>(a, stream, direct);
  else
    throw std::invalid_argument("gemv_binary: dtype must be bf16 or f32");
}

}  // namespace mlapi
