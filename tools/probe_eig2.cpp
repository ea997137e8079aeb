// Probe (round 4): the two-stage eigensolver (dse_eig2.hip) against rocSOLVER dsyevd.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DDSE_EIG2_VARIANTS -Iquantumsimulations_amd/csrc tools/probe_eig2.cpp \
//         quantumsimulations_amd/csrc/dse_eig2.hip quantumsimulations_amd/csrc/dse_sytrd.hip \
//         -lrocsolver -lrocblas -o tools/bin/probe_eig2
//   probe_eig2 <dim> [random]
// Exit codes: 0 ok; 2 HIP error; 3 band reduction error; 4 a bounded poll gave up (band void, the
// later stages are not run); 5 dstedc info != 0; 6 / 7 Q2 / Q1 error.
// Matrix: tools/probe_sytrd.cpp's (spectrum and sparsity of the N = 14 rotated H') or, with
// "random", a dense symmetric one.  One JSON line per stage timing, then the check: max |lam -
// lam_dsyevd| / max |lam|, max |A V - V diag(lam)| / max |lam|, max |V^T V - I|.
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
  for (int b = 0; b < nbits; ++b)
    if ((x ^ (1u << b)) < (unsigned)dim) col[x ^ (1u << b)] = 0.25;
  for (int i = 0; i < nbits; ++i)
    for (int j = i + 1; j < nbits; ++j)
      if (!(((x >> i) ^ (x >> j)) & 1u) && (x ^ ((1u << i) | (1u << j))) < (unsigned)dim)
        col[x ^ ((1u << i) | (1u << j))] = -0.01 * (1 + ((i * 7 + j) % 5));
}

__global__ void k_rand(double* A, int dim, unsigned seed) {
  const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= (size_t)dim * dim) return;
  const unsigned r = (unsigned)(k % dim), c = (unsigned)(k / dim);
  const unsigned a = std::min(r, c), b = std::max(r, c);
  unsigned h = (a * 2654435761u) ^ (b * 40503u) ^ seed;
  h ^= h >> 13;
  h *= 0x5bd1e995u;
  h ^= h >> 15;
  A[k] = (double)(h & 0xffffu) / 65536.0 - 0.5;
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
  const bool rnd = argc > 2 && std::string(argv[2]) == "random";
  int nbits = 0;
  while ((1 << nbits) < n) ++nbits;
  const size_t nn = (size_t)n * n;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  rocblas_handle h;
  rocblas_create_handle(&h);
  rocblas_set_stream(h, st);
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int n_cu = prop.multiProcessorCount;
  double *A0, *A, *V, *lam, *lref, *e;
  void* work;
  rocblas_int* info;
  CK(hipMalloc(&A0, nn * 8));
  CK(hipMalloc(&A, nn * 8));
  CK(hipMalloc(&V, nn * 8));
  CK(hipMalloc(&lam, n * 8));
  CK(hipMalloc(&lref, n * 8));
  CK(hipMalloc(&e, n * 8));
  CK(hipMalloc(&work, dse::eig2_workspace(n)));
  CK(hipMalloc(&info, sizeof(rocblas_int)));
  if (std::getenv("EIG2_Q2")) dse::set_eig2_q2_variant(std::atoi(std::getenv("EIG2_Q2")));
  if (std::getenv("EIG2_CHASE")) dse::set_eig2_chase_variant(std::atoi(std::getenv("EIG2_CHASE")));
  if (std::getenv("EIG2_SYR2K_TRI")) dse::set_eig2_syr2k_tri(std::atoi(std::getenv("EIG2_SYR2K_TRI")));
  // EIG2_CHASE_DBG=1: the chase's per-worker phase times (k_sb2st<true>)
  long long* dbg = nullptr;
  const bool chase_dbg = std::getenv("EIG2_CHASE_DBG") && std::atoi(std::getenv("EIG2_CHASE_DBG"));
  const size_t ntr = n <= 4096 ? (size_t)n * (1 + (n - 2) / 32) * 8 : 0;
  const size_t ndbg = (size_t)5 * 4096 + 6 * (size_t)n + ntr;
  if (chase_dbg) CK(hipMalloc(&dbg, ndbg * 8));
  CK(hipMemsetAsync(A0, 0, nn * 8, st));
  if (rnd)
    hipLaunchKernelGGL(k_rand, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st, A0, n, 7u);
  else
    hipLaunchKernelGGL(k_fill, dim3((n + 255) / 256), dim3(256), 0, st, A0, n, nbits, 7u);
  auto reset = [&] {
    CK(hipMemcpyAsync(A, A0, nn * 8, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
  };
  // reference eigenvalues
  reset();
  rocsolver_dsyevd(h, rocblas_evect_none, rocblas_fill_lower, n, A, n, lref, e, info);
  CK(hipStreamSynchronize(st));
  for (int rep = 0; rep < 2; ++rep) {
    reset();
    double t[6];
    t[0] = now_ms();
    int rc1 = dse::sy2sb_lower(h, st, n, A, n, work);
    CK(hipStreamSynchronize(st));
    t[1] = now_ms();
    if (rc1 != 0) {  // a launch or argument error of the band reduction: nothing after it is valid
      std::fprintf(stderr, "sy2sb_lower rc %d: stopping before the chase\n", rc1);
      return 3;
    }
    int rc2 = dse::sb2st_lower(st, n, A, n, lam, e, work, n_cu, dse::kEig2DefaultSpin, dbg);
    CK(hipStreamSynchronize(st));
    t[2] = now_ms();
    if (rc2 != 0) {
      // kEig2PollTimeout: a bounded cross-workgroup poll of the panel QR or of the chase gave up (the
      // error word sy2sb_lower and sb2st_lower share), so the band / tridiagonal is void.  Round 5
      // ran dstedc, Q2 and Q1 on such a void band under rocprofv3 --pmc and ended in a host SIGSEGV;
      // stop here instead (libdse.so's dense engine re-solves such a register with dsyevd).
      std::printf("{\"dim\": %d, \"rep\": %d, \"sy2sb_ms\": %.1f, \"sb2st_ms\": %.1f, \"rc\": [%d, %d], "
                  "\"poll_gave_up\": %d}\n", n, rep, t[1] - t[0], t[2] - t[1], rc1, rc2,
                  rc2 == dse::kEig2PollTimeout);
      std::fflush(stdout);
      return 4;
    }
    rocsolver_dstedc(h, rocblas_evect_tridiagonal, n, lam, e, V, n, info);
    CK(hipStreamSynchronize(st));
    t[3] = now_ms();
    rocblas_int hinfo = 0;
    CK(hipMemcpy(&hinfo, info, sizeof(hinfo), hipMemcpyDeviceToHost));
    if (hinfo != 0) {
      std::fprintf(stderr, "dstedc info %d: stopping before Q2\n", (int)hinfo);
      return 5;
    }
    int rc3 = dse::q2_apply(st, n, V, n, work);
    CK(hipStreamSynchronize(st));
    t[4] = now_ms();
    // Q1 via the public two-stage entry's last step: ormtr_lower(offset 32) on the stage-1 reflectors
    if (rc3 != 0) {
      std::fprintf(stderr, "q2_apply rc %d: stopping before Q1\n", rc3);
      return 6;
    }
    int rc4 = dse::eig2_q1(h, st, n, A, n, V, n, work);
    CK(hipStreamSynchronize(st));
    if (rc4 != 0) {
      std::fprintf(stderr, "eig2_q1 rc %d\n", rc4);
      return 7;
    }
    t[5] = now_ms();
    std::printf("{\"dim\": %d, \"rep\": %d, \"sy2sb_ms\": %.1f, \"sb2st_ms\": %.1f, \"stedc_ms\": %.1f, \"q2_ms\": %.1f, "
                "\"q1_ms\": %.1f, \"total_ms\": %.1f, \"rc\": [%d, %d, %d, %d]}\n",
                n, rep, t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], t[5] - t[0], rc1, rc2, rc3,
                rc4);
    std::fflush(stdout);
    if (chase_dbg) {
      std::vector<long long> h(ndbg, 0);
      CK(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
      double sum[5] = {0, 0, 0, 0, 0};
      int workers = 0;
      for (int w = 0; w < 4096; ++w)
        if (h[5 * w + 4] > 0) {
          ++workers;
          for (int q = 0; q < 5; ++q) sum[q] += (double)h[5 * w + q];
        }
      // 100 MHz ticks -> us per task
      std::printf("{\"dim\": %d, \"chase_dbg\": 1, \"workers\": %d, \"tasks\": %.0f, \"us_per_task\": {\"wait\": %.2f, "
                  "\"load\": %.2f, \"compute_store\": %.2f, \"drain_flag\": %.2f}}\n",
                  n, workers, sum[4], sum[0] / sum[4] / 100.0, sum[1] / sum[4] / 100.0, sum[2] / sum[4] / 100.0,
                  sum[3] / sum[4] / 100.0);
      // critical chain: sweep s starts task 0 after sweep s - 1 flagged task 2
      double acc[6] = {0, 0, 0, 0, 0, 0};  // busy0, wait1, busy1, wait2, busy2, flag2(s-1) -> start0(s)
      int cntl = 0;
      for (int q = 1; q < n - 1; ++q) {
        const long long* c = &h[5 * 4096 + 6 * q];
        const long long* p = &h[5 * 4096 + 6 * (q - 1)];
        if (!c[5] || !p[5]) continue;
        acc[0] += c[1] - c[0], acc[1] += c[2] - c[1], acc[2] += c[3] - c[2], acc[3] += c[4] - c[3], acc[4] += c[5] - c[4];
        acc[5] += c[0] - p[5];
        ++cntl;
      }
      std::printf("{\"dim\": %d, \"chase_chain\": 1, \"sweeps\": %d, \"us\": {\"busy0\": %.2f, \"wait1\": %.2f, "
                  "\"busy1\": %.2f, \"wait2\": %.2f, \"busy2\": %.2f, \"flag2_to_next_start\": %.2f}}\n", n, cntl,
                  acc[0] / cntl / 100, acc[1] / cntl / 100, acc[2] / cntl / 100, acc[3] / cntl / 100, acc[4] / cntl / 100,
                  acc[5] / cntl / 100);
      if (std::getenv("EIG2_CHASE_TRACE") && ntr) {  // every task's 4 times, raw int64, (s nt(0) + t) 4
        FILE* f = std::fopen(std::getenv("EIG2_CHASE_TRACE"), "wb");
        if (f) {
          std::fwrite(&h[5 * 4096 + 6 * (size_t)n], 8, ntr, f);
          std::fclose(f);
        }
      }
      CK(hipMemset(dbg, 0, ndbg * 8));
    }
  }
  std::vector<double> a(n), b(n);
  CK(hipMemcpy(a.data(), lam, n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), lref, n * 8, hipMemcpyDeviceToHost));
  double dl = 0.0, ml = 0.0;
  for (int k = 0; k < n; ++k) dl = std::max(dl, std::fabs(a[k] - b[k])), ml = std::max(ml, std::fabs(b[k]));
  const double one = 1.0, mone = -1.0;
  rocblas_set_pointer_mode(h, rocblas_pointer_mode_host);
  rocblas_ddgmm(h, rocblas_side_right, n, n, V, n, lam, 1, A, n);
  rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, n, n, n, &one, A0, n, V, n, &mone, A, n);
  rocblas_int ia = 0;
  rocblas_idamax(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), A, 1, &ia);
  double res = 0.0;
  CK(hipMemcpy(&res, A + (ia - 1), 8, hipMemcpyDeviceToHost));
  hipLaunchKernelGGL(k_eye, dim3((unsigned)((nn + 255) / 256)), dim3(256), 0, st, A, n);
  rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, n, n, n, &one, V, n, V, n, &mone, A, n);
  rocblas_idamax(h, (rocblas_int)std::min(nn, (size_t)0x7fffffff), A, 1, &ia);
  double orth = 0.0;
  CK(hipMemcpy(&orth, A + (ia - 1), 8, hipMemcpyDeviceToHost));
  rocblas_int inf = 0;
  CK(hipMemcpy(&inf, info, sizeof(inf), hipMemcpyDeviceToHost));
  std::printf("{\"dim\": %d, \"matrix\": \"%s\", \"check\": 1, \"lam_rel\": %.3e, \"resid_rel\": %.3e, \"orth\": %.3e, "
              "\"info\": %d, \"lam_max\": %.4f, \"workspace_mb\": %.1f}\n",
              n, rnd ? "random" : "h14-like", dl / ml, std::fabs(res) / ml, std::fabs(orth), inf, ml,
              dse::eig2_workspace(n) / 1048576.0);
  return 0;
}
