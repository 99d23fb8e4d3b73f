// Internal launchers shared between the GEMM translation units.
#pragma once

#include "kernels.h"

namespace tfa {
namespace k {
void gemm_f64_launch(const GemmArgs& g, hipStream_t s);
void gemm_int_launch(DType dt, const GemmArgs& g, hipStream_t s);
}  // namespace k
}  // namespace tfa
