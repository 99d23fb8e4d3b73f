// g2 core tiles (gemm_g2_core.h) for k-contiguous A (row-major [M][K]: the
// map_blocks MatMul and the 1x1 convs), with B [K][N] or B^T [N][K].
#include "gemm_g2_core.h"

namespace tfa {
namespace k {
namespace g2 {

void launch_kc(const F32Plan& p, const GemmArgs& g, hipStream_t s) {
  if (g.tb) launch_cfg<A_KCONTIG, B_KC>(p, g, ConvGeom{}, s);
  else launch_cfg<A_KCONTIG, B_RC>(p, g, ConvGeom{}, s);
}

}  // namespace g2
}  // namespace k
}  // namespace tfa
