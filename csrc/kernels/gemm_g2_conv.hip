// g2 core tiles (gemm_g2_core.h) for the implicit-GEMM Conv2D: im2col rows of
// the NHWC input as A (C % 4 == 0: one 16-byte DMA piece = 4 channels of one
// tap), the HWIO filter as B [KH*KW*C][OC].
#include "gemm_g2_core.h"

namespace tfa {
namespace k {
namespace g2 {

void launch_conv(const F32Plan& p, const GemmArgs& g, const ConvGeom& cg, hipStream_t s) {
  if (cg.C % 16 == 0) launch_cfg<A_CONV16, B_RC>(p, g, cg, s);
  else launch_cfg<A_CONV, B_RC>(p, g, cg, s);
}

}  // namespace g2
}  // namespace k
}  // namespace tfa
