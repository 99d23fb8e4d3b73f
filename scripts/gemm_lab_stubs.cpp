// Minimal definitions the kernel objects reference (the full runtime lives in
// csrc/proto/graphdef.cpp); only for the standalone kernel lab.
#include "common.h"

namespace tfa {
const char* dtype_name(DType d) { return d == DType::F32 ? "float32" : d == DType::F64 ? "float64" : "other"; }
int64_t dtype_size(DType d) {
  switch (d) {
    case DType::F64: case DType::I64: return 8;
    case DType::F32: case DType::I32: return 4;
    default: return 1;
  }
}
bool dtype_is_float(DType d) { return d == DType::F32 || d == DType::F64; }
bool dtype_is_int(DType d) { return d == DType::I32 || d == DType::I64; }
}  // namespace tfa
