// Shared definitions for the tensorframes_amd native runtime.
//
// The reference delegates all of this to libtensorflow's C++ runtime over JNI
// (reference: src/main/scala/org/tensorframes/impl/TensorFlowOps.scala:76-95).
// Here it is our own: a GraphDef decoder, a graph IR with static shape/dtype
// inference, a planner and an executor that launches hand-written HIP kernels.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace tfa {

// TensorFlow DataType enum values (reference: src/main/protobuf/tensorflow/core/framework/types.proto:9-57).
enum class DType : int {
  INVALID = 0,
  F32 = 1,
  F64 = 2,
  I32 = 3,
  U8 = 4,
  I16 = 5,
  I8 = 6,
  STRING = 7,
  C64 = 8,
  I64 = 9,
  BOOL = 10,
  BF16 = 14,
  F16 = 19,
};

// A positive integer from the environment; unset, unparsable or < 1 values
// fall back to `dflt` (a bad override must never produce a 0-block grid).
inline int64_t env_positive(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  char* end = nullptr;
  long long v = std::strtoll(e, &end, 10);
  if (end == e || *end != '\0' || v < 1) return dflt;
  return static_cast<int64_t>(v);
}

const char* dtype_name(DType d);
int64_t dtype_size(DType d);
bool dtype_is_float(DType d);
bool dtype_is_int(DType d);

// User-facing errors. Python maps the prefix to a typed exception.
struct GraphError : std::runtime_error {
  explicit GraphError(const std::string& m) : std::runtime_error(m) {}
};

template <typename... Args>
std::string str_cat(Args&&... args) {
  std::ostringstream os;
  (os << ... << args);
  return os.str();
}

#define TFA_CHECK(cond, ...)                                               \
  do {                                                                     \
    if (!(cond)) throw ::tfa::GraphError(::tfa::str_cat(__VA_ARGS__));     \
  } while (0)

// A (possibly partially unknown) shape. dim == -1 is unknown
// (reference: src/main/scala/org/tensorframes/Shape.scala:16-109).
struct Shape {
  bool unknown_rank = false;
  std::vector<int64_t> dims;

  Shape() = default;
  explicit Shape(std::vector<int64_t> d) : dims(std::move(d)) {}
  static Shape unknown() {
    Shape s;
    s.unknown_rank = true;
    return s;
  }
  int rank() const { return unknown_rank ? -1 : static_cast<int>(dims.size()); }
  bool fully_known() const {
    if (unknown_rank) return false;
    for (auto d : dims)
      if (d < 0) return false;
    return true;
  }
  int64_t num_elements() const {
    if (!fully_known()) return -1;
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
  bool operator==(const Shape& o) const {
    return unknown_rank == o.unknown_rank && dims == o.dims;
  }
  std::string str() const;
};

}  // namespace tfa
