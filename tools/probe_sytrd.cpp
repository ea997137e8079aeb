// Probe (round 3): the half-matrix tridiagonalisation (dse_sytrd.hip) against rocSOLVER.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iquantumsimulations_amd/csrc tools/probe_sytrd.cpp \
//         quantumsimulations_amd/csrc/dse_sytrd.hip -lrocsolver -lrocblas -o /tmp/probe_sytrd
//   probe_sytrd <dim> [check | split]
// Matrix as tools/probe_eig.cpp (spectrum and sparsity of the N = 14 rotated H').  Prints one JSON
// line per timing and, with check, max |lam - lam_dsyevd| / max |lam|, max |A V - V diag(lam)| /
// max |lam| and max |V^T V - I|.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "dse_dense.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(2);                                                                  \
    }                                                                                \
  } while (0)

__global__ void k_fill(double* A, int dim, int nbits, unsigned seed) {
  const unsigned x = blockIdx.x * 256u + threadIdx.x;
  if (x >= (unsigned)dim) return;
  double* col = A + (size_t)x * dim;
  double d = 0.0;
  for (int b = 0; b < nbits; ++b) d += (0.5 - (double)((x >> b) & 1u)) * (1.0 + 0.37 * b);
  unsigned h = x * 2654435761u ^ seed;
  h ^= h >> 15;
  d += 1e-3 * (double)(h & 1023u);
  col[x] = d;
  for (int b = 0; b < nbits; ++b) col[x ^ (1u << b)] = 0.25;
  for (int i = 0; i < nbits; ++i)
    for (int j = i + 1; j < nbits; ++j)
      if (!(((x >> i) ^ (x >> j)) & 1u)) col[x ^ ((1u << i) | (1u << j))] = -0.01 * (1 + ((i * 7 + j) % 5));
}

__global__ void k_eye(double* R, int dim) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= (size_t)dim * dim) return;
  R[k] = (k % dim == k / dim) ? 1.0 : 0.0;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 2048;
  const bool check = argc > 2 && std::string(argv[2]) == "check";
  int nbits = 0;
  while ((1 << nbits) < n) ++nbits;
  const size_t nn = (size_t)n * n;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  rocblas_handle h;
  rocblas_create_handle(&h);
  rocblas_set_stream(h, st);
  double *A0, *A, *V, *lam, *lref, *e, *tau, *work;
  rocblas_int* info;
  CK(hipMalloc(&A0, nn * 8));
  CK(hipMalloc(&A, nn * 8));
  CK(hipMalloc(&V, nn * 8));
  CK(hipMalloc(&lam, n * 8));
  CK(hipMalloc(&lref, n * 8));
  CK(hipMalloc(&e, n * 8));
  CK(hipMalloc(&tau, n * 8));
  CK(hipMalloc(&work, dse::sytrd_workspace(n)));
  CK(hipMalloc(&info, sizeof(rocblas_int)));
  CK(hipMemsetAsync(A0, 0, nn * 8, st));
  hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, st, A0, n, nbits, 7u);
  auto reset = [&] {
    CK(hipMemcpyAsync(A, A0, nn * 8, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
  };
  auto timed = [&](const char* op, auto&& f) {
    reset();
    const double t0 = now_ms();
    const int rc = f();
    CK(hipStreamSynchronize(st));
    const double t1 = now_ms();
    std::printf("{\"dim\": %d, \"op\": \"%s\", \"ms\": %.1f, \"rc\": %d}\n", n, op, t1 - t0, rc);
    std::fflush(stdout);
  };
  // warm-up both
  reset();
  rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, n, A, n, lref, e, info);
  reset();
  CK(hipMemsetAsync(lam, 0, n * 8, st));
  dse::eig_sym_lower(h, st, n, A, n, lam, V, n, e, tau, work, info);
  CK(hipStreamSynchronize(st));
  if (argc > 2 && std::string(argv[2]) == "split") {
    // the phases of eig_sym_lower, and sytrd_lower alone three times (for kernel traces)
    for (int rep = 0; rep < 3; ++rep) timed("sytrd_lower", [&] { return dse::sytrd_lower(h, st, n, A, n, lam, e, tau, work); });
    reset();
    dse::sytrd_lower(h, st, n, A, n, lam, e, tau, work);
    CK(hipStreamSynchronize(st));
    double t0 = now_ms();
    rocsolver_dstedc(h, rocblas_evect_tridiagonal, n, lam, e, V, n, info);
    CK(hipStreamSynchronize(st));
    double t1 = now_ms();
    // Z kept in V0 for the second back-transformation
    const double ms_stedc = t1 - t0;
    double* V0 = A0;  // A0 no longer needed
    CK(hipMemcpyAsync(V0, V, nn * 8, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
    t1 = now_ms();
    rocsolver_dormtr(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, n, n, A, n, tau, V, n);
    CK(hipStreamSynchronize(st));
    double t2 = now_ms();
    const int rc = dse::ormtr_lower(h, st, n, A, n, tau, V0, n, work);
    CK(hipStreamSynchronize(st));
    double t3 = now_ms();
    // max |V_dormtr - V_ormtr_lower|
    const double mone = -1.0;
    rocblas_daxpy(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), &mone, V, 1, V0, 1);
    rocblas_int ia = 0;
    rocblas_idamax(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), V0, 1, &ia);
    double dv = 0.0;
    CK(hipMemcpy(&dv, V0 + (ia - 1), 8, hipMemcpyDeviceToHost));
    std::printf("{\"dim\": %d, \"op\": \"dstedc\", \"ms\": %.1f}\n{\"dim\": %d, \"op\": \"dormtr\", \"ms\": %.1f}\n"
                "{\"dim\": %d, \"op\": \"ormtr_lower\", \"ms\": %.1f, \"rc\": %d, \"max_diff_vs_dormtr\": %.3e}\n",
                n, ms_stedc, n, t2 - t1, n, t3 - t2, rc, std::fabs(dv));
    return 0;
  }
  for (int rep = 0; rep < 2; ++rep) {
    timed("rocsolver_dsytrd", [&] { return (int)rocsolver_dsytrd(h, rocblas_fill_lower, n, A, n, lam, e, tau); });
    timed("sytrd_lower", [&] { return dse::sytrd_lower(h, st, n, A, n, lam, e, tau, work); });
    timed("rocsolver_dsyevd", [&] {
      return (int)rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, n, A, n, lref, e, info);
    });
    timed("eig_sym_lower", [&] { return dse::eig_sym_lower(h, st, n, A, n, lam, V, n, e, tau, work, info); });
  }
  if (check) {
    // lref from the last dsyevd; lam, V from the last eig_sym_lower
    std::vector<double> a(n), b(n);
    CK(hipMemcpy(a.data(), lam, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), lref, n * 8, hipMemcpyDeviceToHost));
    double dl = 0.0, ml = 0.0;
    for (int k = 0; k < n; ++k) dl = std::max(dl, std::fabs(a[k] - b[k])), ml = std::max(ml, std::fabs(b[k]));
    // residual A0 V - V diag(lam) into A
    const double one = 1.0, mone = -1.0, zero = 0.0;
    rocblas_ddgmm(h, rocblas_side_right, n, n, V, n, lam, 1, A, n);
    rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, n, n, n, &one, A0, n, V, n, &mone, A, n);
    rocblas_int ia = 0;
    rocblas_set_pointer_mode(h, rocblas_pointer_mode_host);
    rocblas_idamax(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), A, 1, &ia);
    double res = 0.0;
    CK(hipMemcpy(&res, A + (ia - 1), 8, hipMemcpyDeviceToHost));
    // orthogonality V^T V - I
    hipLaunchKernelGGL(k_eye, dim3((nn + 255) / 256), dim3(256), 0, st, A, n);
    rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, n, n, n, &one, V, n, V, n, &mone, A, n);
    rocblas_idamax(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), A, 1, &ia);
    double orth = 0.0;
    CK(hipMemcpy(&orth, A + (ia - 1), 8, hipMemcpyDeviceToHost));
    rocblas_int inf = 0;
    CK(hipMemcpy(&inf, info, sizeof(inf), hipMemcpyDeviceToHost));
    std::printf("{\"dim\": %d, \"check\": 1, \"lam_rel\": %.3e, \"resid_rel\": %.3e, \"orth\": %.3e, \"info\": %d, "
                "\"lam_max\": %.4f}\n",
                n, dl / ml, std::fabs(res) / ml, std::fabs(orth), inf, ml);
  }
  return 0;
}
