// Image resize kernels (NHWC) for the image-scoring preprocessing graphs
// (TF ResizeBilinear / ResizeNearestNeighbor semantics, incl. align_corners
// and half_pixel_centers), and the batched ragged pre-stage of the reference's
// JPEG scoring graph (read_image.py:35-75: decode -> cast -> resize -> central
// crop -> mean subtraction, one image per row): every decoded image of a
// map_rows chunk in ONE ragged uint8 buffer, one kernel producing the
// [rows, h, w, C] float batch the CNN reads (instead of a short program per
// row).
//
// One thread per output pixel x 4 channels: the 2 (nearest: 1) source rows
// are read as contiguous channel runs, so loads coalesce along C.
#include <algorithm>
#include <cmath>

#include "hip_common.h"

namespace tfa {
namespace k {

namespace {

// Both helpers round after every operation (no fused multiply-add), as the
// host oracle (ir/ops_nn.cpp, one ATen op per step) does: the GPU resize, the
// batched pre-stage and the CPU executor give the same bits.
__device__ __forceinline__ float src_coord(int64_t dst, float scale, int mode) {
#pragma clang fp contract(off)
  return mode == 2 ? ((float)dst + 0.5f) * scale - 0.5f : (float)dst * scale;
}

// the bilinear blend shared by both resize paths
__device__ __forceinline__ float bilerp(float tl, float tr, float bl, float br, float lx, float ly) {
#pragma clang fp contract(off)
  const float top = tl + (tr - tl) * lx;
  const float bot = bl + (br - bl) * lx;
  return top + (bot - top) * ly;
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
    const int64_t y0 = min(max((int64_t)fy, (int64_t)0), a.H - 1), y1 = min((int64_t)ceilf(iy), a.H - 1);
    const int64_t x0 = min(max((int64_t)fx, (int64_t)0), a.W - 1), x1 = min((int64_t)ceilf(ix), a.W - 1);
    const float ly = iy - fy, lx = ix - fx;
    const T* base = x + nn * a.H * a.W * a.C + c;
    const float tl = (float)base[(y0 * a.W + x0) * a.C], tr = (float)base[(y0 * a.W + x1) * a.C];
    const float bl = (float)base[(y1 * a.W + x0) * a.C], br = (float)base[(y1 * a.W + x1) * a.C];
    y[i] = bilerp(tl, tr, bl, br, lx, ly);
  }
}

// one output pixel (image blockIdx.y, crop pixel p) of the batched
// pre-stage, all its channels: the bilinear sample of the resized image at
// (oy + yy, ox + xx), computed exactly as resize_bilinear_kernel does on the
// cast image (so a batch equals the per-row program bit for bit), then the
// elementwise steps in graph order. With a.rp the resize size and crop offset
// are the row's own (rp[4n..4n+3] = OH, OW, oy, ox: an aspect-preserving
// resize and its central crop, evaluated per row on the host). 32-bit index
// math per pixel and compile-time indices into the step constants (a runtime
// index would move the kernel arguments to scratch).
__global__ __launch_bounds__(256) void ragged_prep_kernel(RaggedPrepArgs a, int n0) {
#pragma clang fp contract(off)
  const int64_t nn = n0 + (int64_t)blockIdx.y;
  const int C = a.C, npix = a.h * a.w;
  const int H = a.hw[2 * nn], W = a.hw[2 * nn + 1];
  int OH = a.OH, OW = a.OW, oy = a.oy, ox = a.ox;
  if (a.rp) {
    const int4 pr = reinterpret_cast<const int4*>(a.rp)[nn];
    OH = pr.x; OW = pr.y; oy = pr.z; ox = pr.w;
  }
  const float sh = (a.mode == 1 && OH > 1) ? float(H - 1) / float(OH - 1) : float(H) / float(OH);
  const float sw = (a.mode == 1 && OW > 1) ? float(W - 1) / float(OW - 1) : float(W) / float(OW);
  const uint8_t* img = a.x + a.offs[nn];
  float* out = a.y + nn * (int64_t)npix * C;
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < npix; p += gridDim.x * blockDim.x) {
    const int yy = p / a.w, xx = p - yy * a.w;
    const float iy = src_coord(oy + yy, sh, a.mode), ix = src_coord(ox + xx, sw, a.mode);
    const float fy = floorf(iy), fx = floorf(ix);
    const int y0 = min(max((int)fy, 0), H - 1), y1 = min((int)ceilf(iy), H - 1);
    const int x0 = min(max((int)fx, 0), W - 1), x1 = min((int)ceilf(ix), W - 1);
    const float ly = iy - fy, lx = ix - fx;
    const uint8_t* r0 = img + y0 * W * C;
    const uint8_t* r1 = img + y1 * W * C;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= C) break;
      const float tl = (float)r0[x0 * C + c], tr = (float)r0[x1 * C + c];
      const float bl = (float)r1[x0 * C + c], br = (float)r1[x1 * C + c];
      float v = bilerp(tl, tr, bl, br, lx, ly);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= a.nops) break;
        const float k = a.op_chan[q] ? a.op_val[q][c] : a.op_val[q][0];
        switch (a.op_kind[q]) {
          case 0: v = v + k; break;
          case 1: v = v - k; break;
          case 2: v = v * k; break;
          default: v = v / k; break;
        }
      }
      out[(int64_t)p * C + c] = v;
    }
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

void ragged_image_prep(const RaggedPrepArgs& a, hipStream_t s) {
  const int64_t total = a.n * a.h * a.w * a.C;
  if (total <= 0) return;
  TFA_CHECK((int64_t)a.h * a.w * a.C < (int64_t(1) << 31), "ragged_image_prep: crop too large");
  TFA_CHECK(a.C >= 1 && a.C <= 4 && a.nops >= 0 && a.nops <= 4, "ragged_image_prep: bad args");
  // per-row sizes and offsets (a.rp) are checked by the caller, on the host copy
  TFA_CHECK(a.rp || (a.OH > 0 && a.OW > 0 && a.oy >= 0 && a.ox >= 0 && a.oy + a.h <= a.OH && a.ox + a.w <= a.OW),
            "ragged_image_prep: crop outside");
  const int npix = a.h * a.w;
  const unsigned gx = (unsigned)std::min<int64_t>((npix + 255) / 256, 64);
  for (int64_t n0 = 0; n0 < a.n; n0 += 65535) {  // grid y: one image per block row
    const unsigned gy = (unsigned)std::min<int64_t>(a.n - n0, 65535);
    hipLaunchKernelGGL(ragged_prep_kernel, dim3(gx, gy), dim3(256), 0, s, a, (int)n0);
  }
  TFA_LAUNCH_CHECK("ragged_image_prep");
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
