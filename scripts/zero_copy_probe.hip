// PCIe transfer probe for the host-resident pipeline: DMA copies (SDMA) vs
// kernels that read / write page-locked host memory directly ("zero-copy"),
// alone and concurrently. Prints one JSON object.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/zero_copy_probe.hip -o build/zero_copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

// dst[i] = src[i], 16 bytes per lane, 4 vectors in flight per lane
__global__ __launch_bounds__(256) void copy16(const float4* __restrict__ src, float4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    float4 a = src[i], b = src[i + stride], c = src[i + 2 * stride], d = src[i + 3 * stride];
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2 * stride] = c;
    dst[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

struct Timer {
  hipEvent_t a, b;
  hipStream_t s;
  explicit Timer(hipStream_t st) : s(st) {
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
  }
  void start() { CK(hipEventRecord(a, s)); }
  void stop() { CK(hipEventRecord(b, s)); }
  float ms() {
    CK(hipEventSynchronize(b));
    float m = 0;
    CK(hipEventElapsedTime(&m, a, b));
    return m;
  }
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048ull) << 20;
  const int blocks = argc > 2 ? std::atoi(argv[2]) : 1024;
  const size_t n4 = bytes / 16;
  void *h_in, *h_out, *d_in, *d_out;
  CK(hipHostMalloc(&h_in, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&h_out, bytes, hipHostMallocDefault));
  CK(hipMalloc(&d_in, bytes));
  CK(hipMalloc(&d_out, bytes));
  CK(hipMemset(d_in, 1, bytes));
  CK(hipMemset(d_out, 2, bytes));
  std::memset(h_in, 3, bytes);
  std::memset(h_out, 4, bytes);
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  void *h_in_dev = nullptr, *h_out_dev = nullptr;
  CK(hipHostGetDevicePointer(&h_in_dev, h_in, 0));
  CK(hipHostGetDevicePointer(&h_out_dev, h_out, 0));
  const double gb = bytes / 1e9;
  std::vector<std::pair<const char*, double>> out;
  auto run = [&](const char* name, auto fn, int streams) {
    for (int warm = 0; warm < 2; ++warm) {
      Timer t1(s1), t2(s2);
      CK(hipDeviceSynchronize());
      t1.start();
      if (streams == 2) {
        CK(hipStreamWaitEvent(s2, t1.a, 0));
      }
      fn();
      if (streams == 2) {
        CK(hipEventRecord(t2.b, s2));
        CK(hipStreamWaitEvent(s1, t2.b, 0));
      }
      t1.stop();
      float ms = t1.ms();
      if (warm) out.push_back({name, gb / (ms / 1e3) * (streams == 2 ? 2 : 1)});
    }
  };
  run("h2d_dma_GBps", [&] { CK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1)); }, 1);
  run("d2h_dma_GBps", [&] { CK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s1)); }, 1);
  run("bidir_dma_total_GBps", [&] {
    CK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1));
    CK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s2));
  }, 2);
  run("d2h_kernel_write_GBps", [&] {
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s1, (const float4*)d_out, (float4*)h_out_dev, n4);
  }, 1);
  run("h2d_kernel_read_GBps", [&] {
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s1, (const float4*)h_in_dev, (float4*)d_in, n4);
  }, 1);
  run("h2d_dma_plus_d2h_kernel_total_GBps", [&] {
    CK(hipMemcpyAsync(d_in, h_in, bytes, hipMemcpyHostToDevice, s1));
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s2, (const float4*)d_out, (float4*)h_out_dev, n4);
  }, 2);
  run("h2d_kernel_plus_d2h_kernel_total_GBps", [&] {
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s1, (const float4*)h_in_dev, (float4*)d_in, n4);
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s2, (const float4*)d_out, (float4*)h_out_dev, n4);
  }, 2);
  run("h2d_kernel_plus_d2h_dma_total_GBps", [&] {
    hipLaunchKernelGGL(copy16, dim3(blocks), dim3(256), 0, s1, (const float4*)h_in_dev, (float4*)d_in, n4);
    CK(hipMemcpyAsync(h_out, d_out, bytes, hipMemcpyDeviceToHost, s2));
  }, 2);
  std::printf("{\"bytes\": %zu, \"blocks\": %d", bytes, blocks);
  for (auto& kv : out) std::printf(", \"%s\": %.2f", kv.first, kv.second);
  std::printf("}\n");
  return 0;
}
