// Strict JSON body parser of the /predict fast path (reference contract: the pydantic model
// `IrisSpecies` of /root/reference/main.py:10-14, generalised to a model's feature names).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mlapi {

// Parses a JSON object in which every name in `names` appears with a finite JSON-number value
// (last duplicate wins, like json.loads); extra keys may hold any JSON value. Anything else -
// malformed JSON, NaN / Infinity, escaped or non-ASCII keys, a missing key - returns false and
// the request goes to the Python slow path, which decides exactly like FastAPI.
//
// Built once per server (the names never change while it runs). The common body - keys in schema
// order, short decimal numbers - parses in one pass: the expected key is matched with one memcmp
// (name + closing quote), and each number is scanned and converted in the same loop (Clinger's
// fast path: <= 15 significant digits, |power of ten| <= 22 -> one correctly rounded multiply or
// divide, the value strtod / float() return). Longer numbers fall back to strtod.
class PredictBodyParser {
 public:
  explicit PredictBodyParser(std::vector<std::string> names);
  bool parse(const char* p, size_t n, double* out) const;
  size_t size() const { return names_.size(); }

 private:
  std::vector<std::string> names_;
  std::vector<std::string> quoted_;  // name + '"' (empty for names a JSON key can only spell escaped)
};

// One-shot form (tests, the Python binding): builds a parser per call.
bool parse_predict_body(const char* p, size_t n, const std::vector<std::string>& names, double* out);

}  // namespace mlapi
