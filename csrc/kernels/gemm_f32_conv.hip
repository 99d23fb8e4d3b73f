// f32 core tile kernels for conv (im2col-on-the-fly A loader): every tile of
// gemm_f32_core.h instantiated for this A loader (one translation unit per
// loader, so the builds run in parallel).
#include "gemm_f32_core.h"

namespace tfa {
namespace k {
namespace f32core {

void launch_conv(const F32Plan& p, const GemmArgs& g, bool vec, const ConvGeom& cg, hipStream_t s) {
  if (vec) launch_cfg<A_CONV, false, true>(p, g, cg, s);
  else launch_cfg<A_CONV, false, false>(p, g, cg, s);
}

}  // namespace f32core
}  // namespace k
}  // namespace tfa
