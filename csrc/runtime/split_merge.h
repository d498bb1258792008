// Host merge of the class-split kernel's per-block row states (linear_split.hip host-record mode):
// ns records {seq, argmax, m, s} of one row, one per 64-class block in block order, -> (label, p).
// In double: the max (first max wins on ties - lower block, then the block's own first index -
// like numpy's argmax), then the sums rescaled to it. Softmax: p = 1 / sum_b s_b exp(m_b - M);
// OvR: p = sigmoid(M) / sum_b s_b. The engine's completer runs it (Engine::collect); pure so CPU
// tests can check it against the float64 oracle.
#pragma once
#include <cmath>
#include <cstdint>

#include "mlapi/kernels.h"

namespace mlapi {

inline double merge_split_records(const SplitRecord* r, int ns, bool ovr, int32_t* label) {
  double M = -INFINITY;
  int bi = 0x7fffffff;
  for (int sp = 0; sp < ns; ++sp) {
    const double m = r[sp].m;
    if (m > M || (m == M && r[sp].bi < bi)) {
      M = m;
      bi = r[sp].bi;
    }
  }
  double S = 0;
  for (int sp = 0; sp < ns; ++sp) {
    if (ovr)
      S += r[sp].s;
    else if (r[sp].m != -INFINITY)
      S += (double)r[sp].s * std::exp((double)r[sp].m - M);
  }
  *label = bi;
  return ovr ? (1.0 / (1.0 + std::exp(-M))) / S : 1.0 / S;
}

// Host class merge of linear_wide's per-block row states (WideRecOut): ncb blocks x 2 units of
// one row, r[2 * cb] = {seq, argmax, m}, r[2 * cb + 1] = {seq, 0, s}, all f64, merged in block
// order (the kernel's in-kernel merge sums the same terms in its own fixed order: both within
// float64 rounding of the oracle, tests/test_wide_gpu.py).
inline double merge_wide_records(const WideRecord* r, int ncb, bool ovr, int32_t* label) {
  double M = -INFINITY, S = 0.0;
  int bi = 0x7fffffff;
  for (int b = 0; b < ncb; ++b) {
    const double m = r[2 * b].x, s = r[2 * b + 1].x;
    const int i = r[2 * b].v;
    const bool take = (m > M) || (m == M && i < bi);
    const double nm = take ? m : M;
    if (ovr) {
      S = S + s;
    } else {
      const double sa = M == -INFINITY ? 0.0 : S * std::exp(M - nm);
      const double sb = m == -INFINITY ? 0.0 : s * std::exp(m - nm);
      S = sa + sb;
    }
    if (take) {
      M = m;
      bi = i;
    }
    if (std::isnan(m)) M = m;  // a NaN state poisons the row (the kernel's merge does the same)
  }
  *label = bi;
  return ovr ? (1.0 / (1.0 + std::exp(-M))) / S : 1.0 / S;
}

}  // namespace mlapi
