// Internal launchers shared between the GEMM translation units.
#pragma once

#include "kernels.h"

namespace tfa {
namespace k {
void gemm_f64_launch(const GemmArgs& g, hipStream_t s);
void gemm_int_launch(DType dt, const GemmArgs& g, hipStream_t s);

// implicit-GEMM conv geometry (NHWC input, filter viewed as [KH*KW*C, OC])
struct Im2colGeom {
  int H, W, C, KW, OH, OW, sh, sw, dh, dw, pt, pl;
};

// reduced-precision f32 GEMM on bf16 MFMA (gemm_bf16.hip); mode 1 = bf16, 2 = bf16x3
size_t bf16_workspace_bytes(int mode, int64_t N, int64_t K);
bool bf16_gemm_eligible(const GemmArgs& g, bool conv, int64_t conv_c);
void bf16_gemm_launch(int mode, const GemmArgs& g, bool conv, const Im2colGeom& cg, hipStream_t s);
// direct small-reduction conv (conv_smallc.hip): KH*KW*C <= 32, OC <= 64,
// no fused siblings / epilogue chain; bitwise equal to the implicit-GEMM core
bool conv_smallc_eligible(const ConvArgs& a);
void conv_smallc_launch(const ConvArgs& a, hipStream_t s);
// direct conv for C in {32, 64}, OC <= 96 stem layers (conv_direct.hip):
// filter in LDS, A straight to registers; chosen by shape only
bool conv_direct_eligible(const ConvArgs& a);
void conv_direct_launch(const ConvArgs& a, hipStream_t s);
// Winograd F(2x2,3x3) (conv_wino.hip): a.wino set by the planner, 3x3/s1,
// C % 4 == 0, OC % 4 == 0, cheap epilogue, 16-byte aligned outputs
bool conv_wino_eligible(const ConvArgs& a);
void conv_wino_launch(const ConvArgs& a, hipStream_t s);
}  // namespace k
}  // namespace tfa
