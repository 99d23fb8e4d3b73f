// Kernel lab for the f32 MFMA GEMM / implicit-GEMM conv core (csrc/kernels/gemm.hip):
// times tfa::k::gemm / conv2d_nhwc on device-resident operands with HIP events
// and checks sampled outputs against a double-accumulated reference kernel.
//
//   scripts/build_gemm_lab.sh            (hipcc, links build/hip/*.o)
//   [TFA_GEMM_TILE=cfg] [TFA_PRECISION=f32|bf16|bf16x3] ./build/gemm_lab [iters]
//
// One JSON line per shape: {"kind", "shape", "ms", "tflops", "max_rel_err"}.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels/kernels.h"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void fill_uniform(float* p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    p[i] = (float)(x & 0xffffff) / 8388608.0f - 1.0f;
  }
}

// sampled reference: out[s] = act(sum_k A[m][k] * B[k][n] + bias[n]) in double
__global__ void ref_gemm(const float* A, const float* B, const float* bias, int64_t N, int64_t K, bool tb,
                         const int64_t* rows, const int64_t* cols, int ns, double* out, double* mag, int act) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  const int64_t m = rows[s], n = cols[s];
  double acc = 0, a2 = 0;
  for (int64_t k = 0; k < K; ++k) {
    const double a = A[m * K + k], b = tb ? B[n * K + k] : B[k * N + n];
    acc += a * b;
    a2 += fabs(a * b);
  }
  if (bias) acc += bias[n];
  if (act == 1) acc = acc > 0 ? acc : 0;
  out[s] = acc;
  mag[s] = a2 + 1e-30;
}

__global__ void ref_conv(const float* x, const float* w, const float* bias, tfa::k::ConvArgs a, const int64_t* rows,
                         const int64_t* cols, int ns, double* out, double* mag) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= ns) return;
  const int64_t m = rows[s], oc = cols[s];
  const int64_t ow = m % a.OW, oh = (m / a.OW) % a.OH, n = m / (a.OW * a.OH);
  double acc = 0, a2 = 0;
  for (int64_t kh = 0; kh < a.KH; ++kh)
    for (int64_t kw = 0; kw < a.KW; ++kw) {
      const int64_t ih = oh * a.sh - a.pad_t + kh * a.dh, iw = ow * a.sw - a.pad_l + kw * a.dw;
      if (ih < 0 || ih >= a.H || iw < 0 || iw >= a.W) continue;
      for (int64_t c = 0; c < a.C; ++c) {
        const double xv = x[((n * a.H + ih) * a.W + iw) * a.C + c];
        const double wv = w[((kh * a.KW + kw) * a.C + c) * a.OC + oc];
        acc += xv * wv;
        a2 += fabs(xv * wv);
      }
    }
  if (bias) acc += bias[oc];
  acc = acc > 0 ? acc : 0;
  out[s] = acc;
  mag[s] = a2 + 1e-30;
}

struct Samples {
  int ns;
  int64_t *rows, *cols;
  double *ref, *mag;
  std::vector<int64_t> hr, hc;
  Samples(int64_t M, int64_t N, int n) : ns(n) {
    hr.resize(n);
    hc.resize(n);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      hr[i] = (i < 8) ? (M - 1 - i) : (int64_t)(s % (uint64_t)M);  // always include the last rows (edge tiles)
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      hc[i] = (i < 8) ? (N - 1 - i % N) : (int64_t)(s % (uint64_t)N);
    }
    CK(hipMalloc(&rows, n * 8)); CK(hipMalloc(&cols, n * 8));
    CK(hipMalloc(&ref, n * 8)); CK(hipMalloc(&mag, n * 8));
    CK(hipMemcpy(rows, hr.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(cols, hc.data(), n * 8, hipMemcpyHostToDevice));
  }
  double check(const float* C, int64_t ldc) {
    std::vector<double> r(ns), mg(ns);
    CK(hipMemcpy(r.data(), ref, ns * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(mg.data(), mag, ns * 8, hipMemcpyDeviceToHost));
    double worst = 0;
    for (int i = 0; i < ns; ++i) {
      float got;
      CK(hipMemcpy(&got, C + hr[i] * ldc + hc[i], 4, hipMemcpyDeviceToHost));
      worst = std::fmax(worst, std::fabs(got - r[i]) / mg[i]);
    }
    return worst;
  }
};

float* dev_uniform(int64_t n, uint32_t seed) {
  float* p;
  CK(hipMalloc(&p, n * 4));
  hipLaunchKernelGGL(fill_uniform, dim3(2048), dim3(256), 0, 0, p, n, seed);
  return p;
}

template <typename F>
double time_ms(F f, int iters) {
  f();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 10;
  const char* mode = std::getenv("TFA_GEMM_TILE");
  const char* st = std::getenv("TFA_PRECISION");
  struct G { int64_t M, N, K; bool tb, bias; };
  const G gemms[] = {{2500000, 512, 512, false, true}, {262144, 512, 512, false, true}, {4096, 4096, 4096, false, false},
                     {8192, 1024, 1024, false, false}, {1000000, 64, 256, false, true}, {4096, 4096, 4096, true, false},
                     {100003, 500, 300, false, true}, {777, 260, 1000, true, false}};
  for (const G& s : gemms) {
    float* A = dev_uniform(s.M * s.K, 1);
    float* B = dev_uniform(s.K * s.N, 2);
    float* bias = s.bias ? dev_uniform(s.N, 3) : nullptr;
    float* C;
    CK(hipMalloc(&C, s.M * s.N * 4));
    tfa::k::GemmArgs g{};
    g.M = s.M; g.N = s.N; g.K = s.K;
    g.A = A; g.lda = s.K; g.B = B; g.ldb = s.tb ? s.K : s.N; g.C = C; g.ldc = s.N;
    g.tb = s.tb; g.bias = bias; g.act = s.bias ? 1 : 0; g.batch = 1;
    size_t wsb = tfa::k::gemm_workspace_bytes(tfa::DType::F32, g);
    void* ws = nullptr;
    if (wsb) CK(hipMalloc(&ws, wsb));
    g.workspace = ws;
    const double ms = time_ms([&] { tfa::k::gemm(tfa::DType::F32, g, 0); }, iters);
    Samples smp(s.M, s.N, 512);
    hipLaunchKernelGGL(ref_gemm, dim3(2), dim3(256), 0, 0, A, B, bias, s.N, s.K, s.tb, smp.rows, smp.cols, smp.ns,
                       smp.ref, smp.mag, g.act);
    CK(hipDeviceSynchronize());
    const double err = smp.check(C, s.N);
    std::printf("{\"kind\": \"gemm\", \"tile\": \"%s\", \"precision\": \"%s\", \"shape\": [%ld, %ld, %ld, %d], "
                "\"ms\": %.4f, \"tflops\": %.2f, \"max_rel_err\": %.3e}\n",
                mode ? mode : "default", st ? st : "default", (long)s.M, (long)s.N, (long)s.K, (int)s.tb, ms,
                2.0 * s.M * s.N * s.K / ms / 1e9, err);
    std::fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C));
    if (bias) CK(hipFree(bias));
    if (ws) CK(hipFree(ws));
  }
  struct Cv { int64_t N, H, W, C, KH, KW, OC, s; bool same; };
  const Cv convs[] = {{512, 111, 111, 32, 3, 3, 32, 1, false}, {512, 109, 109, 32, 3, 3, 64, 1, true},
                      {512, 25, 25, 48, 5, 5, 64, 1, true},    {512, 25, 25, 64, 3, 3, 96, 1, true},
                      {512, 12, 12, 128, 1, 7, 128, 1, true},  {512, 12, 12, 160, 7, 1, 192, 1, true},
                      {512, 5, 5, 448, 3, 3, 384, 1, true},    {512, 25, 25, 288, 3, 3, 384, 2, false},
                      {64, 224, 224, 3, 3, 3, 32, 2, false},   {512, 12, 12, 160, 1, 7, 160, 1, true},
                      {512, 5, 5, 1280, 1, 1, 320, 1, true},   {512, 5, 5, 2048, 1, 1, 448, 1, true},
                      {512, 12, 12, 768, 1, 1, 192, 1, true},  {512, 25, 25, 256, 1, 1, 48, 1, true}};
  for (const Cv& c : convs) {
    tfa::k::ConvArgs a{};
    a.N = c.N; a.H = c.H; a.W = c.W; a.C = c.C; a.KH = c.KH; a.KW = c.KW; a.OC = c.OC;
    a.sh = a.sw = c.s; a.dh = a.dw = 1;
    if (c.same) {
      a.OH = (c.H + c.s - 1) / c.s; a.OW = (c.W + c.s - 1) / c.s;
      const int64_t ph = std::max<int64_t>(0, (a.OH - 1) * c.s + c.KH - c.H);
      const int64_t pw = std::max<int64_t>(0, (a.OW - 1) * c.s + c.KW - c.W);
      a.pad_t = ph / 2; a.pad_l = pw / 2;
    } else {
      a.OH = (c.H - c.KH) / c.s + 1; a.OW = (c.W - c.KW) / c.s + 1;
    }
    float* x = dev_uniform(c.N * c.H * c.W * c.C, 4);
    float* w = dev_uniform(c.KH * c.KW * c.C * c.OC, 5);
    float* bias = dev_uniform(c.OC, 6);
    float* y;
    const int64_t M = a.N * a.OH * a.OW;
    CK(hipMalloc(&y, M * c.OC * 4));
    a.x = x; a.w = w; a.y = y; a.bias = bias; a.act = 1;
    size_t wsb = tfa::k::conv2d_workspace_bytes(tfa::DType::F32, a);
    void* ws = nullptr;
    if (wsb) CK(hipMalloc(&ws, wsb));
    a.workspace = ws;
    const double ms = time_ms([&] { tfa::k::conv2d_nhwc(tfa::DType::F32, a, 0); }, iters);
    Samples smp(M, c.OC, 512);
    hipLaunchKernelGGL(ref_conv, dim3(2), dim3(256), 0, 0, x, w, bias, a, smp.rows, smp.cols, smp.ns, smp.ref,
                       smp.mag);
    CK(hipDeviceSynchronize());
    const double err = smp.check(y, c.OC);
    const double flop = 2.0 * M * c.OC * c.KH * c.KW * c.C;
    std::printf("{\"kind\": \"conv\", \"tile\": \"%s\", \"precision\": \"%s\", \"shape\": [%ld, %ld, %ld, %ld, %ld, "
                "%ld, %ld, %ld, \"%s\"], \"ms\": %.4f, \"tflops\": %.2f, \"max_rel_err\": %.3e}\n",
                mode ? mode : "default", st ? st : "default", (long)c.N, (long)c.H, (long)c.W, (long)c.C,
                (long)c.KH, (long)c.KW, (long)c.OC, (long)c.s, c.same ? "SAME" : "VALID", ms, flop / ms / 1e9, err);
    std::fflush(stdout);
    CK(hipFree(x)); CK(hipFree(w)); CK(hipFree(y)); CK(hipFree(bias));
    if (ws) CK(hipFree(ws));
  }
  return 0;
}
