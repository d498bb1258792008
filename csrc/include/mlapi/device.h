// Device-side helpers shared by the kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace mlapi {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

// 16-byte non-temporal (streamed-once) load: global_load_dwordx4 ... nt.
__device__ __forceinline__ uint4 load_nt16(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

}  // namespace mlapi
