// dse_dense.h -- the dense eigen-propagator engine (dse_dense.hip): SURVEY.md §8(a) K4.
//
// For a register of n <= kDenseMaxQubits qubits whose drives are all purely imaginary (drive
// phase pi/2, the sweep's case) or all real, H is brought to a REAL symmetric form
//     H' = D H D^dagger,   D |x> = i^{popcount(x)} |x>
// (a drive flip changes popcount by 1, a double-quantum pair flip by 2: i * (i a) and i^2 g are
// real), diagonalised once on the device (rocSOLVER dsyevd: H' = V diag(lambda) V^T), and every
// output is then exact at any time, independent of ||H|| t:
//     psi'(tau_j) = V (c * exp(-i lambda tau_j)),   c = V^T e_{x0}   (a row of V)
// Psi' for a block of output times is one real GEMM (rocBLAS dgemm: V times the [cos | -sin]
// phase columns), the observables are read from its columns (k_dense_obs).  The reference's
// own default workload (n_sea = 6, 30 s / 20 000 outputs, sweep_sea_detuning.py:1223-1240) needs
// ~1e8 Chebyshev terms per evolution and one 128 x 128 eigendecomposition this way.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

namespace dse {

constexpr int kDenseMaxQubits = 14;  // 2^14 x 2^14 fp64 = 2 GiB per eigenvector matrix

struct DenseProb {
  int n;              // qubits (engine bit order: bit b = site b)
  int rot;            // 1: drives imaginary, H' = D H D^dagger; 0: drives real, H' = H
  int refine;         // 1: refined eigenvalues and double-double phases (option dense_refine);
                      // 0: the eigensolver's eigenvalues, phases sincos(lam tau) in fp64
  uint64_t sea_mask;
  int rare_bit;       // -1: none in the register
  int n_sea;          // popcount(sea_mask)
  uint64_t x0;        // psi(t0) = e_{x0}
  double shift;       // scalar part of H (a global phase; left out of H')
  const double* field;  // [n]     sum_b field[b] s_b
  const double* zz;     // [n * n] sum_{i<j} zz[i n + j] s_i s_j
  const double* pair;   // [n * n] pair flip coefficient g_ij (i < j), applies iff bit_i == bit_j
  const double* flip;   // [4 n]   drive flip of bit b: re0 im0 re1 im1 by the output bit value
  double* V;            // [dim * dim] column-major: H' in, eigenvectors out (rocSOLVER)
  double* lam;          // [dim] eigenvalues (ascending); after k_dense_rq the high part of each
                        // refined eigenvalue (double-double lam + lam_lo)
  double* lam_lo;       // [dim] low parts (zero without the refinement)
  double* diag_dd;      // [2 dim] the exact diagonal <x|H'|x> as double-double (hi, lo), for k_dense_rq
  double* obs;          // [n_t][8] raw observable sums of this problem (finish_obs order)
  double2* final_state; // [dim] psi(t_last) in the reference frame (dse_get_state), or null
};

// H' of every problem into its (zeroed) V
hipError_t launch_dense_h(const DenseProb* d, int count, int dim, hipStream_t st);
// Rayleigh-quotient refinement of every eigenvalue in double-double arithmetic: lam_a = v_a^T H' v_a
// / v_a^T v_a with H' applied from the coefficient tables (the same fp64 matrix k_dense_h built).
// The eigensolver's eigenvalues carry errors ~eps ||H'|| sqrt(dim) (a phase error growing like that
// times t); the quotient of its eigenvector is exact to ~(eps ||H'||)^2 / gap + eps^2 ||H'||.
// (launch_dense_rq first writes diag_dd: one exact diagonal per row, not one per row and column)
hipError_t launch_dense_rq(const DenseProb* d, int count, int dim, hipStream_t st);
// phase columns of output times tau[0 .. tb): P[a + j dim] = c_a cos(lambda_a tau_j),
// P[a + (tb + j) dim] = -c_a sin(lambda_a tau_j); problem p's block at P + p * pstride
hipError_t launch_dense_phase(const DenseProb* d, int count, int dim, const double* tau, int tb,
                              double* P, size_t pstride, hipStream_t st);
// observables of the tb columns of Psi' (re | im blocks as P) into d[p].obs rows t0 .. t0 + tb
hipError_t launch_dense_obs(const DenseProb* d, int count, int dim, const double* Psi, size_t pstride,
                            int tb, int t0, hipStream_t st);
// observables of n_states complex states (dim amplitudes each, consecutive) of one problem
// (d->rot = 0: the computational frame) into d->obs rows t0 .. t0 + n_states
hipError_t launch_state_obs(const DenseProb* d, int dim, const double2* states, int n_states, int t0,
                            hipStream_t st);
// psi(t_last) from column tb - 1 of Psi' into d[p].final_state (frame rotation, psi0 phase and
// the shift's phase exp(-i shift tau_last) included)
hipError_t launch_dense_final(const DenseProb* d, int count, int dim, const double* Psi, size_t pstride,
                              int tb, double tau_last, hipStream_t st);
// the same two for ONE problem whose tb output columns are interleaved complex (column j = dim
// double2 at Psi + 2 j dim: the non-uniform FFT's output, dse_nufft.hip)
hipError_t launch_dense_obs_c(const DenseProb* d, int dim, const double* Psi, int tb, int t0, hipStream_t st);
hipError_t launch_dense_final_c(const DenseProb* d, int dim, const double* Psi, int tb, double tau_last,
                                hipStream_t st);

// ---- output times by a type-1 non-uniform FFT (dse_nufft.hip) ---------------------------------
// On a uniform grid tau_j = j s + delta_j (|delta_j| lambda_max <= 1e-7) psi'(tau_j) of every output
// from W-point spreading of the eigenvalue phases theta_a = lambda_a s mod 2 pi onto M >= 2T grid
// points, M-point FFTs per row and deconvolution, instead of the dim^2 T GEMM.
constexpr int kNufftW = 15;          // kernel width in grid points (error ~3e-14, beta = 2.30 W)
constexpr int kNufftMinDim = 1024;   // smaller registers keep the GEMM (its cost is small there)
constexpr int kNufftMinOutputs = 2048;  // option dense_nufft 1: grids of at least this many outputs
struct NufftGrid {
  int T = 0, M = 0, half = 0, W = 0;
  double s = 0.0, h = 0.0, alpha = 0.0, beta = 0.0;
  std::vector<double> delta;  // tau_j - j s (exact)
  std::vector<double> scale;  // (2 pi / M) / phi_hat(j - half)
};
// false: the grid is not uniform enough (or too short) for the transform
bool nufft_grid(const double* tau, int n_t, double lam_max, NufftGrid& g);
struct NufftScratch {  // device buffers of one dense_run (sized for its largest register)
  double2 *U = nullptr, *U2 = nullptr;  // [M][dim] each
  double* c = nullptr;                  // [dim]
  int *off = nullptr, *src = nullptr;   // [M + 1], [nnz_cap]
  double* wt = nullptr;                 // [4 nnz_cap]
  size_t nnz_cap = 0;
  double *scale = nullptr, *delta = nullptr;  // [T] each (uploaded from NufftGrid)
};
struct NufftCache;  // rocFFT plans (per context)
void nufft_release(NufftCache* c);
size_t nufft_scratch_doubles(const NufftGrid& g, int dim);
// psi' of every output of one register (V column-major dim x dim, refined eigenvalues, psi0 = e_x0)
// into Psi in blocks of TB interleaved complex columns, per_block(tb0, tb) called after each block
// (the observables, the final state); 0 on success
int nufft_outputs(NufftCache*& cache, hipStream_t st, const NufftGrid& g, const NufftScratch& S, const double* V,
                  const double* lam_hi, const double* lam_lo, uint64_t x0, int dim, double* Psi, int TB,
                  const std::function<int(int tb0, int tb)>& per_block);

}  // namespace dse

typedef struct _rocblas_handle* rocblas_handle;

namespace dse {

// ---- the half-matrix tridiagonalisation (dse_sytrd.hip): LAPACK dsytrd's lower layout (d, e, tau,
// reflectors below the subdiagonal of A), the trailing-matrix products over the lower-triangle
// tiles only.  work: sytrd_workspace(n) bytes.  0 on success.
size_t sytrd_workspace(int n);
int sytrd_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* d, double* e, double* tau,
                double* work);
// Z = Q Z for the Q of sytrd_lower's reflectors in A (rocsolver_dormtr's left / lower / no-transpose
// case), blocks of 256 reflectors; work: sytrd_workspace(n) bytes.  off: reflector q (column q of A,
// unit element at row q + off) -- 1 for sytrd_lower, the bandwidth for sy2sb_lower's panels
int ormtr_lower(rocblas_handle h, hipStream_t st, int n, const double* A, int lda, const double* tau, double* Z,
                int ldz, double* work, int off = 1);
// A = V diag(lam) V^T (lower triangle of A read, A overwritten): sytrd_lower, rocsolver_dstedc,
// ormtr_lower.  e, tau: n doubles each; V: n x n, ldv >= n; info: rocsolver_dstedc's
int eig_sym_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* lam, double* V, int ldv,
                  double* e, double* tau, double* work, int* info);

// ---- the two-stage eigensolver (dse_eig2.hip): dense -> band 32 (sy2sb_lower), band ->
// tridiagonal by bulge chasing (sb2st_lower), rocsolver_dstedc, Z <- Q2 Z (q2_apply), Z <- Q1 Z
// (ormtr_lower, offset 32).  work: eig2_workspace(n) bytes (the chase's reflectors: ~n^2 / 2
// doubles); n_cu: compute units (the chase's workgroups are co-resident)
size_t eig2_workspace(int n);
#ifdef DSE_EIG2_VARIANTS
// A/B variants (probe builds only: tools/probe_eig2.cpp; dse_eig2.hip g_q2_variant, ...)
void set_eig2_q2_variant(int v);
void set_eig2_chase_variant(int v);
void set_eig2_syr2k_tri(int v);
#endif
// spin: rounds a cross-workgroup poll waits before it gives up (option eig_spin_limit; < 0: fail at
// once, tests).  A give-up makes sb2st_lower / eig_sym_2stage return kEig2PollTimeout (the band or
// tridiagonal is then void; the dense engine re-solves the register with rocSOLVER dsyevd).
constexpr int kEig2PollTimeout = -9;
constexpr int kEig2DefaultSpin = 1 << 22;
int sy2sb_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, void* work, int spin = kEig2DefaultSpin);
int sb2st_lower(hipStream_t st, int n, const double* A, int lda, double* d, double* e, void* work, int n_cu,
                int spin = kEig2DefaultSpin, long long* dbg = nullptr);
int q2_apply(hipStream_t st, int n, double* Z, int ldz, void* work);
int eig2_q1(rocblas_handle h, hipStream_t st, int n, const double* A, int lda, double* Z, int ldz, void* work);
int eig_sym_2stage(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* lam, double* V, int ldv,
                   double* e, void* work, int* info, int n_cu, int spin = kEig2DefaultSpin);

}  // namespace dse

namespace dse {

// ---- propagator-matrix mode (dse_runtime.hip matrix_run): y = U x for the column-built
// U = exp(-iH dt) of a register whose rotated form is symmetric, U_cr = s_r s_c U_rc with
// s_x = (-1)^popcount(x) (imaginary drives; s = 1 for real ones).  Only the kSymvBlock^2 tiles on
// or above the diagonal are read (half the matrix): tile (I, J) adds U_IJ x_J to row block I and,
// below the diagonal by symmetry, s (U_IJ^T (s x_I)) to row block J.  Per-tile partial sums
// partial[B][k][kSymvBlock] (k = the other block index) are summed in fixed order by the reduce kernel:
// deterministic, no atomics.
constexpr int kSymvBlock = 64;
// tile storage of U for k_symv: the kSymvBlock^2 tiles (I, J), I <= J, in the row-major order of the
// upper triangle of nb x nb blocks, each column-major (64 KiB contiguous)
__host__ __device__ inline size_t symv_tile_index(int I, int J, int nb) {
  return (size_t)I * nb - (size_t)I * (I - 1) / 2 + (size_t)(J - I);
}
// cnt (nb zeroed ints) non-null: the reduction into y in the same launch (k_symv<FUSED>), counters
// left zeroed; null: partials only, then launch_symv_reduce
hipError_t launch_symv(const double2* U, int dim, const double2* x, double2* partial, int parity,
                       hipStream_t st, int* cnt = nullptr, double2* y = nullptr);
hipError_t launch_symv_reduce(const double2* partial, int dim, double2* y, hipStream_t st);

// Column build in real arithmetic (dse_matrix.hip, k_ucols): U e_c for columns col0 .. col0 +
// n_cols - 1 of a one-tile register (n == L, drives all imaginary (rot = 1) or all real (rot = 0)),
// one workgroup per column.  probs: one DevProb with beta and s1 = 1 / alpha of the interval;
// cf[k] = (-1)^{floor(k/2)} (2 - delta_k0) J_k(alpha dt), k = 0..deg; (phr, phi) = e^{-i beta dt}.
// U in the computational frame, in k_symv's tile storage (the tiles on and above the diagonal);
// column c1 also whole (2^L amplitudes) into psi1.
bool ucols_supported(int L);
hipError_t launch_ucols(int L, const struct DevProb* probs, const double* cf, int deg, int rot, double phr,
                        double phi, double2* U, int n_cols, int col0, int c1, double2* psi1, hipStream_t st);

}  // namespace dse
