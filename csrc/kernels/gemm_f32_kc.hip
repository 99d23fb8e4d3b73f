// f32 core tile kernels for k-contiguous A (row-major [M][K]: the map_blocks MatMul and the 1x1 convs): every tile of
// gemm_f32_core.h instantiated for this A loader (one translation unit per
// loader, so the builds run in parallel).
#include "gemm_f32_core.h"

namespace tfa {
namespace k {
namespace f32core {

void launch_kcontig_b(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s) {
  if (vec) launch_cfg<A_KCONTIG, false, true>(p, g, ConvGeom{}, s);
  else launch_cfg<A_KCONTIG, false, false>(p, g, ConvGeom{}, s);
}

void launch_kcontig_bt(const F32Plan& p, const GemmArgs& g, bool vec, hipStream_t s) {
  if (vec) launch_cfg<A_KCONTIG, true, true>(p, g, ConvGeom{}, s);
  else launch_cfg<A_KCONTIG, true, false>(p, g, ConvGeom{}, s);
}

}  // namespace f32core
}  // namespace k
}  // namespace tfa
