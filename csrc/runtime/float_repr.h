// Python-compatible float rendering (repr(float) == json.dumps(float)).
//
// The reference returns the probability as a numpy float64 that FastAPI serializes with
// json.dumps -> float.__repr__ (shortest round-trip digits, SURVEY Appendix A "Float rendering").
// The native fast path must produce byte-identical JSON, so this reproduces CPython's
// format_float_short(..., 'r'): shortest digits (std::to_chars), fixed notation when
// -4 < decpt <= 16, otherwise d.ddde[+-]XX with at least two exponent digits; ".0" appended to
// integral fixed values.
#pragma once
#include <charconv>
#include <cmath>
#include <cstring>
#include <string>

namespace mlapi {

// Appends repr(v) to out. Returns false for non-finite values (json.dumps(allow_nan=False) raises).
inline bool append_py_float(std::string& out, double v) {
  if (!std::isfinite(v)) return false;
  if (v == 0.0) {
    out += std::signbit(v) ? "-0.0" : "0.0";
    return true;
  }
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  *res.ptr = '\0';
  // buf = [-]d[.ddd]e[+-]XX
  const char* p = buf;
  bool neg = false;
  if (*p == '-') { neg = true; ++p; }
  char digits[32];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int exp10 = 0;
  if (*p == 'e') exp10 = std::atoi(p + 1);
  // strip trailing zeros of the mantissa (to_chars shortest never emits them, be safe)
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  const int decpt = exp10 + 1;  // value = 0.d1d2... * 10^decpt
  if (neg) out += '-';
  if (decpt <= -4 || decpt > 16) {
    out += digits[0];
    if (nd > 1) {
      out += '.';
      out.append(digits + 1, nd - 1);
    }
    out += 'e';
    const int e = decpt - 1;
    out += e < 0 ? '-' : '+';
    const int ae = e < 0 ? -e : e;
    if (ae < 10) out += '0';
    out += std::to_string(ae);
  } else if (decpt <= 0) {
    out += "0.";
    out.append((size_t)(-decpt), '0');
    out.append(digits, nd);
  } else if (decpt >= nd) {
    out.append(digits, nd);
    out.append((size_t)(decpt - nd), '0');
    out += ".0";
  } else {
    out.append(digits, decpt);
    out += '.';
    out.append(digits + decpt, nd - decpt);
  }
  return true;
}

}  // namespace mlapi
