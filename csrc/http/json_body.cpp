// /predict body parser (json_body.h).
#include "json_body.h"

#include <cmath>
#include <cstdlib>
#include <cstring>

namespace mlapi {
namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }
inline bool is_hex(char c) { return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F'); }
// short-key compare, inlined (a memcmp call per key costs more than the compare itself)
inline bool same_bytes(const char* a, const char* b, size_t len) {
  for (; len >= 8; a += 8, b += 8, len -= 8) {
    uint64_t x, y;
    memcpy(&x, a, 8);
    memcpy(&y, b, 8);
    if (x != y) return false;
  }
  if (len >= 4) {
    uint32_t x, y;
    memcpy(&x, a, 4);
    memcpy(&y, b, 4);
    if (x != y) return false;
    a += 4;
    b += 4;
    len -= 4;
  }
  for (; len > 0; --len)
    if (*a++ != *b++) return false;
  return true;
}
inline unsigned digit(char c) { return (unsigned)(unsigned char)c - (unsigned)'0'; }  // > 9: not a digit

// RFC 8259 number grammar (no value conversion): -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
bool scan_number(const char* p, size_t n, size_t& i) {
  if (i < n && p[i] == '-') ++i;
  if (i >= n) return false;
  if (p[i] == '0') {
    ++i;
  } else if (p[i] >= '1' && p[i] <= '9') {
    while (i < n && digit(p[i]) <= 9) ++i;
  } else {
    return false;
  }
  if (i < n && p[i] == '.') {
    ++i;
    if (i >= n || digit(p[i]) > 9) return false;
    while (i < n && digit(p[i]) <= 9) ++i;
  }
  if (i < n && (p[i] == 'e' || p[i] == 'E')) {
    ++i;
    if (i < n && (p[i] == '+' || p[i] == '-')) ++i;
    if (i >= n || digit(p[i]) > 9) return false;
    while (i < n && digit(p[i]) <= 9) ++i;
  }
  return true;
}

// Skip one JSON value starting at p[i]; returns false on malformed input, and also on anything
// json.loads might judge differently from a strict scanner (non-ASCII bytes in strings, which
// depend on the body's UTF-8 validity): those requests go to the Python slow path instead.
bool skip_value(const char* p, size_t n, size_t& i, int depth) {
  if (depth > 64) return false;
  while (i < n && is_ws(p[i])) ++i;
  if (i >= n) return false;
  const char c = p[i];
  if (c == '"') {
    ++i;
    while (i < n) {
      const unsigned char ch = (unsigned char)p[i];
      if (ch == '\\') {
        if (i + 1 >= n) return false;
        const char e = p[i + 1];
        if (e == 'u') {
          if (n - i < 6 || !is_hex(p[i + 2]) || !is_hex(p[i + 3]) || !is_hex(p[i + 4]) || !is_hex(p[i + 5]))
            return false;
          i += 6;
        } else if (e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't') {
          i += 2;
        } else {
          return false;
        }
        continue;
      }
      if (ch < 0x20 || ch >= 0x80) return false;
      ++i;
      if (ch == '"') return true;
    }
    return false;
  }
  if (c == '{' || c == '[') {
    const char close = c == '{' ? '}' : ']';
    ++i;
    while (i < n && is_ws(p[i])) ++i;
    if (i < n && p[i] == close) {
      ++i;
      return true;
    }
    for (;;) {
      if (c == '{') {
        while (i < n && is_ws(p[i])) ++i;
        if (i >= n || p[i] != '"') return false;
        if (!skip_value(p, n, i, depth + 1)) return false;
        while (i < n && is_ws(p[i])) ++i;
        if (i >= n || p[i] != ':') return false;
        ++i;
      }
      if (!skip_value(p, n, i, depth + 1)) return false;
      while (i < n && is_ws(p[i])) ++i;
      if (i >= n) return false;
      if (p[i] == ',') {
        ++i;
        continue;
      }
      if (p[i] == close) {
        ++i;
        return true;
      }
      return false;
    }
  }
  // literals / numbers: strictness only matters for the required keys (parsed separately), an odd
  // extra value just needs to be skippable.
  if (c == 't' && n - i >= 4 && memcmp(p + i, "true", 4) == 0) { i += 4; return true; }
  if (c == 'f' && n - i >= 5 && memcmp(p + i, "false", 5) == 0) { i += 5; return true; }
  if (c == 'n' && n - i >= 4 && memcmp(p + i, "null", 4) == 0) { i += 4; return true; }
  if (c == '-' || digit(c) <= 9) return scan_number(p, n, i);
  return false;  // NaN / Infinity / garbage -> slow path
}

const double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                           1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Slow number path: grammar scan, then strtod on a NUL-terminated copy (finite values only).
bool parse_number_strtod(const char* p, size_t n, size_t& i, double* out) {
  const size_t s = i;
  if (!scan_number(p, n, i)) return false;
  const size_t len = i - s;
  if (len > 400) return false;  // absurd literals: let Python decide
  char buf[416];
  memcpy(buf, p + s, len);
  buf[len] = '\0';
  char* end = nullptr;
  const double v = strtod(buf, &end);
  if (end != buf + len || !std::isfinite(v)) return false;
  *out = v;
  return true;
}

// ---- SWAR digit runs (8 bytes at a time, little-endian): the digit loops of a short decimal
// ("-0.891") are data-dependent branches that mispredict once or twice per number; counting a
// run with one mask and converting it with three multiplies has none.
inline uint64_t load8(const char* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
// leading ASCII digits among the 8 bytes (a +6 carry out of a byte >= 0xFA only reaches bytes
// after that non-digit, so the leading run is exact)
inline int digit_run8(uint64_t v) {
  const uint64_t hi = v & 0xF0F0F0F0F0F0F0F0ull;
  const uint64_t hi6 = (v + 0x0606060606060606ull) & 0xF0F0F0F0F0F0F0F0ull;
  const uint64_t x = (hi ^ 0x3030303030303030ull) | (hi6 ^ 0x3030303030303030ull);  // byte != 0: not a digit
  const uint64_t y = (((x & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full) | x) & 0x8080808080808080ull;
  return y == 0 ? 8 : __builtin_ctzll(y) >> 3;
}
// value of the first c (1..8) digits: bytes past the run may borrow upward only, and the shift
// drops them; the zero bytes shifted in are leading zeros
inline uint64_t digits_value(uint64_t v, int c) {
  uint64_t t = (v - 0x3030303030303030ull) << (8 * (8 - c));
  t = (t * 10 + (t >> 8)) & 0x00FF00FF00FF00FFull;
  t = (t * 100 + (t >> 16)) & 0x0000FFFF0000FFFFull;
  return (t * 10000 + (t >> 32)) & 0xFFFFFFFFull;
}
const uint64_t kPow10u[9] = {1, 10, 100, 1000, 10000, 100000, 1000000, 10000000, 100000000};

// Strict JSON number -> finite double, scanned and converted in one pass. Significand digits
// accumulate into m (leading zeros skipped); e10 is the decimal exponent of m's last digit.
// Exact (Clinger) when m has <= 15 significant digits and |e10| <= 22; otherwise strtod.
inline bool parse_number(const char* p, size_t n, size_t& i, double* out) {
  size_t j = i;
  const bool neg = j < n && p[j] == '-';
  j += neg;
  if (j >= n) return false;
  if (n - j >= 24) {  // SWAR fast path: int part and fraction of <= 7 digits each, no exponent
    const uint64_t v = load8(p + j);
    const int c1 = digit_run8(v);
    if (c1 == 0) return false;
    if (c1 > 1 && p[j] == '0') return false;  // leading zero: not JSON
    if (c1 < 8) {
      size_t k = j + (size_t)c1;
      uint64_t m = digits_value(v, c1);
      int c2 = 0;
      if (p[k] == '.') {
        const uint64_t w = load8(p + k + 1);
        c2 = digit_run8(w);
        if (c2 == 0) return false;
        if (c2 < 8) {
          m = m * kPow10u[c2] + digits_value(w, c2);
          k += 1 + (size_t)c2;
        }
      }
      if (c2 < 8 && (p[k] | 0x20) != 'e') {  // c1 + c2 <= 14 digits: m < 2^53, Clinger exact
        const double d = m == 0 ? 0.0 : (c2 == 0 ? (double)m : (double)m / kPow10[c2]);
        // an integer literal is a Python int: "-0" is 0, not -0.0
        *out = neg && (m != 0 || c2 != 0) ? -d : d;
        i = k;
        return true;
      }
    }
  }
  uint64_t m = 0;
  int sig = 0, e10 = 0;
  unsigned d = digit(p[j]);
  if (d == 0) {
    ++j;
  } else if (d <= 9) {
    do {
      m = m * 10 + d;
      ++sig;
      ++j;
    } while (j < n && (d = digit(p[j])) <= 9);
  } else {
    return false;
  }
  bool is_int = true;  // no fraction, no exponent
  if (j < n && p[j] == '.') {
    is_int = false;
    ++j;
    if (j >= n || digit(p[j]) > 9) return false;
    while (j < n && (d = digit(p[j])) <= 9) {
      --e10;
      sig += m != 0 || d != 0;
      m = m * 10 + d;
      ++j;
    }
  }
  if (j < n && (p[j] | 0x20) == 'e') {
    is_int = false;
    ++j;
    bool eneg = false;
    if (j < n && (p[j] == '+' || p[j] == '-')) eneg = p[j++] == '-';
    if (j >= n || digit(p[j]) > 9) return false;
    int x = 0;
    while (j < n && (d = digit(p[j])) <= 9) {
      if (x < 100000) x = x * 10 + (int)d;
      ++j;
    }
    e10 += eneg ? -x : x;
  }
  if (sig > 15 || e10 > 22 || e10 < -22) return parse_number_strtod(p, n, i, out);  // i: token start
  const double v = m == 0 ? 0.0 : (e10 >= 0 ? (double)m * kPow10[e10] : (double)m / kPow10[-e10]);
  *out = neg && !(m == 0 && is_int) ? -v : v;  // "-0" is the Python int 0
  i = j;
  return true;
}

}  // namespace

PredictBodyParser::PredictBodyParser(std::vector<std::string> names) : names_(std::move(names)) {
  quoted_.resize(names_.size());
  for (size_t k = 0; k < names_.size(); ++k) {
    bool clean = true;
    for (const char ch : names_[k]) {
      const unsigned char u = (unsigned char)ch;
      if (u == '"' || u == '\\' || u < 0x20 || u >= 0x80) clean = false;
    }
    // a key the scan below would reject (escapes, control or non-ASCII bytes) never matches
    if (clean) quoted_[k] = names_[k] + '"';
  }
}

bool PredictBodyParser::parse(const char* p, size_t n, double* out) const {
  const size_t nk = names_.size();
  if (nk > 4096) return false;
  uint64_t seen_bits[64];  // no per-request allocation: one bit per feature name
  std::memset(seen_bits, 0, ((nk + 63) / 64) * sizeof(uint64_t));
  size_t i = 0, hint = 0;
  while (i < n && is_ws(p[i])) ++i;
  if (i >= n || p[i] != '{') return false;
  ++i;
  while (i < n && is_ws(p[i])) ++i;
  if (i < n && p[i] == '}') {
    ++i;
  } else {
    for (;;) {
      while (i < n && is_ws(p[i])) ++i;
      if (i >= n || p[i] != '"') return false;
      ++i;
      // keys usually arrive in schema order: the one after the last match is tried first with a
      // single compare of name + closing quote (a clean name matched byte for byte is exactly the
      // key the scan below would find), so a wide body parses in O(F)
      int which = -1;
      if (hint < nk) {
        const std::string& q = quoted_[hint];
        if (!q.empty() && n - i >= q.size() && same_bytes(p + i, q.data(), q.size())) {
          which = (int)hint;
          i += q.size();
        }
      }
      if (which < 0) {
        const size_t ks = i;
        while (i < n && p[i] != '"') {
          // escaped or non-ASCII keys -> slow path
          if (p[i] == '\\' || (unsigned char)p[i] < 0x20 || (unsigned char)p[i] >= 0x80) return false;
          ++i;
        }
        if (i >= n) return false;
        const size_t klen = i - ks;
        ++i;
        for (size_t k = 0; k < nk; ++k) {
          if (names_[k].size() == klen && memcmp(names_[k].data(), p + ks, klen) == 0) {
            which = (int)k;
            break;
          }
        }
      }
      while (i < n && is_ws(p[i])) ++i;
      if (i >= n || p[i] != ':') return false;
      ++i;
      while (i < n && is_ws(p[i])) ++i;
      if (which >= 0) {
        hint = (size_t)which + 1;
        double v;
        if (!parse_number(p, n, i, &v)) return false;
        out[which] = v;
        seen_bits[(size_t)which >> 6] |= uint64_t(1) << ((size_t)which & 63);
      } else {
        if (!skip_value(p, n, i, 0)) return false;
      }
      while (i < n && is_ws(p[i])) ++i;
      if (i >= n) return false;
      if (p[i] == ',') {
        ++i;
        continue;
      }
      if (p[i] == '}') {
        ++i;
        break;
      }
      return false;
    }
  }
  while (i < n && is_ws(p[i])) ++i;
  if (i != n) return false;
  for (size_t k = 0; k < nk; ++k)
    if (!(seen_bits[k >> 6] >> (k & 63) & 1)) return false;
  return true;
}

bool parse_predict_body(const char* p, size_t n, const std::vector<std::string>& names, double* out) {
  return PredictBodyParser(names).parse(p, n, out);
}

}  // namespace mlapi
