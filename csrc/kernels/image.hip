// Image resize kernels (NHWC) for the image-scoring preprocessing graphs
// (TF ResizeBilinear / ResizeNearestNeighbor semantics, incl. align_corners
// and half_pixel_centers).
//
// One thread per output pixel x 4 channels: the 2 (nearest: 1) source rows
// are read as contiguous channel runs, so loads coalesce along C.
#include <cmath>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

__device__ __forceinline__ float src_coord(int64_t dst, float scale, int mode) {
  return mode == 2 ? ((float)dst + 0.5f) * scale - 0.5f : (float)dst * scale;
}

template <typename T>
__global__ __launch_bounds__(256) void resize_bilinear_kernel(ResizeArgs a, int64_t n) {
  const T* x = static_cast<const T*>(a.x);
  float* y = static_cast<float*>(a.y);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t c = i % a.C;
    int64_t t = i / a.C;
    const int64_t ow = t % a.OW;
    t /= a.OW;
    const int64_t oh = t % a.OH;
    const int64_t nn = t / a.OH;
    const float iy = src_coord(oh, a.sh, a.mode), ix = src_coord(ow, a.sw, a.mode);
    const float fy = floorf(iy), fx = floorf(ix);
    const int64_t y0 = max((int64_t)fy, (int64_t)0), y1 = min((int64_t)ceilf(iy), a.H - 1);
    const int64_t x0 = max((int64_t)fx, (int64_t)0), x1 = min((int64_t)ceilf(ix), a.W - 1);
    const float ly = iy - fy, lx = ix - fx;
    const T* base = x + nn * a.H * a.W * a.C + c;
    const float tl = (float)base[(y0 * a.W + x0) * a.C], tr = (float)base[(y0 * a.W + x1) * a.C];
    const float bl = (float)base[(y1 * a.W + x0) * a.C], br = (float)base[(y1 * a.W + x1) * a.C];
    const float top = tl + (tr - tl) * lx;
    const float bot = bl + (br - bl) * lx;
    y[i] = top + (bot - top) * ly;
  }
}

template <typename E>
__global__ __launch_bounds__(256) void resize_nearest_kernel(ResizeArgs a, int64_t n) {
  const E* x = static_cast<const E*>(a.x);
  E* y = static_cast<E*>(a.y);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t c = i % a.C;
    int64_t t = i / a.C;
    const int64_t ow = t % a.OW;
    t /= a.OW;
    const int64_t oh = t % a.OH;
    const int64_t nn = t / a.OH;
    int64_t sy, sx;
    if (a.mode == 1) {
      sy = (int64_t)roundf((float)oh * a.sh);
      sx = (int64_t)roundf((float)ow * a.sw);
    } else if (a.mode == 2) {
      sy = (int64_t)floorf(((float)oh + 0.5f) * a.sh);
      sx = (int64_t)floorf(((float)ow + 0.5f) * a.sw);
    } else {
      sy = (int64_t)floorf((float)oh * a.sh);
      sx = (int64_t)floorf((float)ow * a.sw);
    }
    sy = min(max(sy, (int64_t)0), a.H - 1);
    sx = min(max(sx, (int64_t)0), a.W - 1);
    y[i] = x[((nn * a.H + sy) * a.W + sx) * a.C + c];
  }
}

}  // namespace

void resize_bilinear(DType dt, const ResizeArgs& a, hipStream_t s) {
  const int64_t n = a.N * a.OH * a.OW * a.C;
  if (n <= 0) return;
  TFA_CHECK(a.H > 0 && a.W > 0, "resize_bilinear: empty input image");
  const dim3 g(ew_grid(n)), b(256);
  switch (dt) {
    case DType::F32: hipLaunchKernelGGL((resize_bilinear_kernel<float>), g, b, 0, s, a, n); break;
    case DType::F64: hipLaunchKernelGGL((resize_bilinear_kernel<double>), g, b, 0, s, a, n); break;
    case DType::U8: hipLaunchKernelGGL((resize_bilinear_kernel<uint8_t>), g, b, 0, s, a, n); break;
    case DType::I32: hipLaunchKernelGGL((resize_bilinear_kernel<int32_t>), g, b, 0, s, a, n); break;
    case DType::I64: hipLaunchKernelGGL((resize_bilinear_kernel<int64_t>), g, b, 0, s, a, n); break;
    default: TFA_CHECK(false, "resize_bilinear: dtype ", dtype_name(dt), " not supported");
  }
  TFA_LAUNCH_CHECK("resize_bilinear");
}

void resize_nearest(int64_t elem_size, const ResizeArgs& a, hipStream_t s) {
  const int64_t n = a.N * a.OH * a.OW * a.C;
  if (n <= 0) return;
  TFA_CHECK(a.H > 0 && a.W > 0, "resize_nearest: empty input image");
  const dim3 g(ew_grid(n)), b(256);
  switch (elem_size) {
    case 1: hipLaunchKernelGGL((resize_nearest_kernel<uint8_t>), g, b, 0, s, a, n); break;
    case 2: hipLaunchKernelGGL((resize_nearest_kernel<uint16_t>), g, b, 0, s, a, n); break;
    case 4: hipLaunchKernelGGL((resize_nearest_kernel<uint32_t>), g, b, 0, s, a, n); break;
    case 8: hipLaunchKernelGGL((resize_nearest_kernel<uint64_t>), g, b, 0, s, a, n); break;
    default: TFA_CHECK(false, "resize_nearest: element size ", elem_size);
  }
  TFA_LAUNCH_CHECK("resize_nearest");
}

}  // namespace k
}  // namespace tfa
