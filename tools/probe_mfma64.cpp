// Probe (round 4): FP64 matrix-core vs vector FMA throughput on this device (the design choice for
// the Q2 application in dse_eig2.hip).  One JSON line: TFLOP/s of v_mfma_f64_16x16x4_f64 (8
// independent accumulators per wave) and of v_fma_f64 (8 independent chains).
//   hipcc --offload-arch=gfx950 -O3 tools/probe_mfma64.cpp -o tools/bin/probe_mfma64
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kIter = 4096;

__global__ void __launch_bounds__(256) k_mfma(double* out, double a, double b) {
  f64x4 c[8];
  for (int i = 0; i < 8; ++i) c[i] = f64x4{0.0, 0.0, 0.0, (double)threadIdx.x};
  double x = a + threadIdx.x * 1e-9, y = b;
  for (int it = 0; it < kIter; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c[i], 0, 0, 0);
  double s = 0.0;
  for (int i = 0; i < 8; ++i) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fma(double* out, double a, double b) {
  double c[8];
  for (int i = 0; i < 8; ++i) c[i] = threadIdx.x + i;
  const double x = a + threadIdx.x * 1e-9;
  for (int it = 0; it < kIter * 4; ++it)
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = fma(c[i], x, b);
  double s = 0.0;
  for (int i = 0; i < 8; ++i) s += c[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int blocks = p.multiProcessorCount * 8;
  double* out;
  hipMalloc(&out, (size_t)blocks * 256 * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms_m = 0, ms_f = 0;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_m, e0, e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, 1.0000001, 0.9999999);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms_f, e0, e1);
  }
  const double waves = (double)blocks * 4;
  const double fl_m = waves * kIter * 8 * 2.0 * 16 * 16 * 4;  // flops per MFMA: 2 x 16 x 16 x 4
  const double fl_f = (double)blocks * 256 * kIter * 4 * 8 * 2.0;
  std::printf("{\"cus\": %d, \"mfma_f64_tflops\": %.1f, \"vector_fma_f64_tflops\": %.1f, \"ms\": [%.3f, %.3f]}\n",
              p.multiProcessorCount, fl_m / ms_m * 1e-9, fl_f / ms_f * 1e-9, ms_m, ms_f);
  return 0;
}
