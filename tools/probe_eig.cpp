// Planning probe (round 3): throughput of rocSOLVER dsyevd on one MI355X when several large
// symmetric eigendecompositions run at once (one host thread, HIP stream and rocBLAS handle
// each), against one at a time.  Also times the phases of one solve (dsytrd alone).
//
//   hipcc --offload-arch=gfx950 -O2 tools/probe_eig.cpp -lrocsolver -lrocblas -o /tmp/probe_eig
//   probe_eig <dim> <max_concurrent>
//
// Matrices: a banded-plus-diagonal symmetric matrix with the spectral spread of the N = 14
// rotated H' (diagonal ~ field terms, off-diagonal entries at the bit-flip positions of a
// 2-local operator), so that divide and conquer deflates like the engine's matrices do.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                        \
    }                                                                      \
  } while (0)

__global__ void k_fill(double* A, int dim, int nbits, unsigned seed) {
  const unsigned x = blockIdx.x * 256u + threadIdx.x;
  if (x >= (unsigned)dim) return;
  double* col = A + (size_t)x * dim;
  // diagonal: a field-like sum over the bits, plus a small hashed term
  double d = 0.0;
  for (int b = 0; b < nbits; ++b) d += (0.5 - (double)((x >> b) & 1u)) * (1.0 + 0.37 * b);
  unsigned h = x * 2654435761u ^ seed;
  h ^= h >> 15;
  d += 1e-3 * (double)(h & 1023u);
  col[x] = d;
  for (int b = 0; b < nbits; ++b) col[x ^ (1u << b)] = 0.25;  // drive-like flips
  for (int i = 0; i < nbits; ++i)
    for (int j = i + 1; j < nbits; ++j)
      if (!(((x >> i) ^ (x >> j)) & 1u)) col[x ^ ((1u << i) | (1u << j))] = -0.01 * (1 + ((i * 7 + j) % 5));
}

struct Solver {
  int dim;
  hipStream_t st;
  rocblas_handle h;
  double *A, *w, *e;
  rocblas_int* info;
};

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int dim = argc > 1 ? std::atoi(argv[1]) : 16384;
  const int kmax = argc > 2 ? std::atoi(argv[2]) : 4;
  int nbits = 0;
  while ((1 << nbits) < dim) ++nbits;
  std::vector<Solver> S(kmax);
  for (int i = 0; i < kmax; ++i) {
    S[i].dim = dim;
    CK(hipStreamCreateWithFlags(&S[i].st, hipStreamNonBlocking));
    rocblas_create_handle(&S[i].h);
    rocblas_set_stream(S[i].h, S[i].st);
    CK(hipMalloc(&S[i].A, (size_t)dim * dim * sizeof(double)));
    CK(hipMalloc(&S[i].w, dim * sizeof(double)));
    CK(hipMalloc(&S[i].e, dim * sizeof(double)));
    CK(hipMalloc(&S[i].info, sizeof(rocblas_int)));
  }
  auto fill = [&](Solver& s, unsigned seed) {
    CK(hipMemsetAsync(s.A, 0, (size_t)dim * dim * sizeof(double), s.st));
    hipLaunchKernelGGL(k_fill, dim3((dim + 255) / 256), dim3(256), 0, s.st, s.A, dim, nbits, seed);
    CK(hipStreamSynchronize(s.st));
  };
  auto solve = [&](Solver& s) {
    rocsolver_dsyevd(s.h, rocblas_evect_original, rocblas_fill_upper, dim, s.A, dim, s.w, s.e, s.info);
    CK(hipStreamSynchronize(s.st));
  };
  // warm-up (library kernels loaded, workspace sized)
  fill(S[0], 1);
  solve(S[0]);
  // phases of one solve: tridiagonalisation alone
  {
    fill(S[0], 2);
    double* tau;
    CK(hipMalloc(&tau, dim * sizeof(double)));
    const double t0 = now_ms();
    rocsolver_dsytrd(S[0].h, rocblas_fill_upper, dim, S[0].A, dim, S[0].w, S[0].e, tau);
    CK(hipStreamSynchronize(S[0].st));
    const double t1 = now_ms();
    std::printf("{\"dim\": %d, \"op\": \"dsytrd\", \"ms\": %.1f}\n", dim, t1 - t0);
    CK(hipFree(tau));
  }
  for (int k = 1; k <= kmax; k *= 2) {
    for (int i = 0; i < k; ++i) fill(S[i], 10 + i);
    CK(hipDeviceSynchronize());
    const double t0 = now_ms();
    std::vector<std::thread> th;
    for (int i = 0; i < k; ++i) th.emplace_back([&, i] { solve(S[i]); });
    for (auto& x : th) x.join();
    const double t1 = now_ms();
    int bad = 0;
    for (int i = 0; i < k; ++i) {
      rocblas_int inf = 0;
      CK(hipMemcpy(&inf, S[i].info, sizeof(inf), hipMemcpyDeviceToHost));
      bad += inf != 0;
    }
    std::printf("{\"dim\": %d, \"op\": \"dsyevd\", \"concurrent\": %d, \"wall_ms\": %.1f, \"ms_per_solve\": %.1f, \"failed\": %d}\n",
                dim, k, t1 - t0, (t1 - t0) / k, bad);
    std::fflush(stdout);
  }
  for (auto& s : S) {
    (void)hipFree(s.A), (void)hipFree(s.w), (void)hipFree(s.e), (void)hipFree(s.info);
    rocblas_destroy_handle(s.h);
    (void)hipStreamDestroy(s.st);
  }
  return 0;
}
