// Host plan of the f64-accumulating wide predict (linear_wide.h): pure arithmetic, shared by the
// launcher (linear_wide.hip) and host-only builds (csrc/tests/kernel_stubs.cpp), where the engine
// still plans models it then serves on the CPU backend.
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <stdexcept>

#include "mlapi/common.h"
#include "mlapi/kernels.h"

namespace mlapi {
namespace wide_plan {

constexpr int CB = 16;     // classes per block
constexpr int RG = 32;     // rows of a row group's workspace region (a launch's groups have 16 or 32)
constexpr int WAVES = 4;   // waves per block (feature quarters)
constexpr int SMAX = 32;   // wave steps per feature split before the features are split over blocks

inline WidePlan plan(int dt, int F, int K) {
  if (dt != DT_F64 && dt != DT_F32) throw std::invalid_argument("linear_wide: f64 or f32 storage");
  if (F < 1 || K < 1) throw std::invalid_argument("linear_wide: empty model");
  const int E = dt == DT_F64 ? 2 : 4;  // elements per 16-byte load
  const int unit = WAVES * 4 * E;      // features one step of every wave covers
  WidePlan p;
  p.ncb = (K + CB - 1) / CB;
  p.nfs = std::max(1, (F + unit * SMAX - 1) / (unit * SMAX));
  const int per = unit * p.nfs;
  p.ldx = (F + per - 1) / per * per;
  p.fsteps = p.ldx / per;
  return p;
}

// 16-row tiles per row group: one (NB = 1) while the grid of 16-row groups stays within one block
// per CU - small serving batches then spread their MFMA work over twice the CUs (B = 24: 126
// blocks of one tile instead of 63 of two; tools/wide_trace.py) - else two (W read once per 32 rows)
inline int tiles_per_group(int64_t B, const WidePlan& p) {
  return (std::max<int64_t>(B, 1) + 15) / 16 * p.ncb * p.nfs <= 256 ? 1 : 2;
}
inline int row_groups(int64_t B, int nb) { return (int)((std::max<int64_t>(B, 1) + 16 * nb - 1) / (16 * nb)); }

// one region per row group (linear_wide.h WideArgs): tickets | split partials | row states
struct Layout {
  size_t cnt_bytes, part_bytes, rg_bytes;
};
inline Layout layout(const WidePlan& p) {
  Layout l;
  l.cnt_bytes = (((size_t)p.ncb + 1) * sizeof(unsigned) + 255) & ~size_t(255);
  l.part_bytes = p.nfs > 1 ? (size_t)p.ncb * p.nfs * (2 * 4 * 64) * sizeof(double) : 0;
  l.rg_bytes = l.cnt_bytes + l.part_bytes + (size_t)p.ncb * RG * 4 * sizeof(double);
  return l;
}

// enough for every launch of at most B rows (16-row groups are the most regions a launch uses)
inline size_t workspace(int64_t B, int dt, int F, int K) {
  return (size_t)row_groups(B, 1) * layout(plan(dt, F, K)).rg_bytes;
}

}  // namespace wide_plan
}  // namespace mlapi
