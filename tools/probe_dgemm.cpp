// Probe (round 5): rocBLAS DGEMM rate for the dense engine's output product Psi = V P
// (dse_runtime.hip `outputs`: M = K = dim, N = 2 x TB output columns, column-major, no transposes).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe_dgemm.cpp -lrocblas -o tools/bin/probe_dgemm
//   probe_dgemm <dim> <N>...      one JSON line per N: ms per call (median of 5) and TF/s
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    if ((x) != hipSuccess) {                                         \
      std::fprintf(stderr, "%s:%d HIP error\n", __FILE__, __LINE__); \
      return 2;                                                      \
    }                                                                \
  } while (0)

__global__ void k_fill(double* a, size_t n, unsigned seed) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) a[i] = (double)((i * 2654435761u ^ seed) & 1023u) / 1024.0 - 0.5;
}

int main(int argc, char** argv) {
  if (argc < 3) return 1;
  const int dim = std::atoi(argv[1]);
  int nmax = 0;
  for (int a = 2; a < argc; ++a) nmax = std::max(nmax, std::atoi(argv[a]));
  double *V, *P, *C;
  const size_t nv = (size_t)dim * dim, np = (size_t)dim * nmax;
  CK(hipMalloc(&V, nv * 8));
  CK(hipMalloc(&P, np * 8));
  CK(hipMalloc(&C, np * 8));
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, 0, V, nv, 1u);
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, 0, P, np, 2u);
  rocblas_handle h;
  rocblas_create_handle(&h);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double one = 1.0, zero = 0.0;
  for (int a = 2; a < argc; ++a) {
    const int N = std::atoi(argv[a]);
    std::vector<float> ms;
    for (int r = 0; r < 6; ++r) {
      CK(hipEventRecord(e0, 0));
      rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, dim, N, dim, &one, V, dim, P, dim, &zero, C, dim);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0.f;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r > 0) ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    std::printf("{\"dim\": %d, \"N\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n", dim, N, med,
                2.0 * dim * (double)dim * N / (med * 1e-3) / 1e12);
    std::fflush(stdout);
  }
  rocblas_destroy_handle(h);
  return 0;
}
