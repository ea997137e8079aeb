// dse_nufft.hip -- the dense engine's output times by a type-1 non-uniform FFT (gfx950).
//
// The dense eigen-propagator (dse_dense.h) needs psi'(tau_j) = V (c o exp(-i lambda tau_j)) at every
// output time.  As one real GEMM per block of times (V times the [cos | -sin] phase columns) that
// is 4 dim^2 T flops per register: 2.1e13 at dim 2^14 on the reference's 20 000-output grid
// (sweep_sea_detuning.py:1223-1224), 0.36 s at the FP64 MFMA rate and ~a quarter of the full
// sweep's device work.  On a uniform grid tau_j = j s + delta_j (np.linspace: |delta_j| ~ an ulp)
//     psi'_x(tau_j) = sum_a V_xa c_a e^{-i j theta_a} (1 - i lambda_a delta_j) + O((lambda delta)^2),
//     theta_a = lambda_a s mod 2 pi,
// and for one row x the sum over the eigenvectors a is a type-1 non-uniform discrete Fourier
// transform: 'sources' at theta_a with strengths w_xa = V_xa c_a, evaluated at the integer modes
// j = 0 .. T-1 (centred: j = k + T/2, the factor e^{-i (T/2) theta_a} folded into the strengths).
// Each source is spread onto a uniform grid of M >= 2T points with the exponential-of-semicircle
// kernel phi(z) = exp(beta (sqrt(1 - z^2) - 1)) over W = 15 points (beta = 2.30 W), every row is
// transformed by an M-point FFT (rocFFT, batched over the rows, stride dim), and mode k is divided
// by the kernel's Fourier transform: error ~3e-14 of sum_a |w_xa| <= 1 (numpy prototype; the
// GPU tests hold the result to the GEMM path and to the 30 s oracles).  The lambda_a delta_j term
// is a second transform with strengths lambda_a w_xa (G), spread in the same pass.  ~60 GB of HBM
// traffic and ~1e11 flops per 2^14 register instead of 2.1e13 flops.
//
// theta_a, the centring phase and delta_j are formed on the host in double-double from the refined
// eigenvalues (lambda_hi + lambda_lo), and the kernel's offsets x_m - theta_a in double-double, so
// the phases keep the dense engine's 30 s accuracy: the only rounding left is that of
// e^{-i j theta} inside the FFT, a relative 1e-16 per source.
//
// Layouts: U[m dim + x] (the spreading kernel's writes coalesced over x; the FFT runs along m with
// stride dim), the outputs interleaved complex, column j = dim amplitudes (k_dense_obs' es = 2 form).
#include <rocfft/rocfft.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <vector>

#include "dse_dense.h"

namespace dse {
namespace {

// ---- host double-double (value = hi + lo), std::fma exact ----
struct hdd {
  double hi, lo;
};
hdd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
hdd fast_sum(double a, double b) {
  const double s = a + b;
  return {s, b - (s - a)};
}
hdd two_prod(double a, double b) {
  const double p = a * b;
  return {p, std::fma(a, b, -p)};
}
hdd dd_add(hdd a, hdd b) {
  hdd s = two_sum(a.hi, b.hi);
  s.lo += a.lo + b.lo;
  return fast_sum(s.hi, s.lo);
}
hdd dd_mul(hdd a, hdd b) {
  hdd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_sum(p.hi, p.lo);
}
constexpr hdd kTwoPi = {0x1.921fb54442d18p+2, 0x1.1a62633145c07p-52};
// x mod 2 pi into [0, 2 pi)
hdd dd_mod2pi(hdd x) {
  const double k = std::nearbyint(x.hi / kTwoPi.hi);
  const hdd p = two_prod(k, kTwoPi.hi);
  hdd r = dd_add(x, hdd{-p.hi, -p.lo});
  r = dd_add(r, hdd{-k * kTwoPi.lo, 0.0});
  if (r.hi < 0.0) r = dd_add(r, kTwoPi);
  return r;
}

int nice_fft_length(int m) {  // smallest 2^a 3^b 5^c >= m
  for (int n = std::max(m, 2);; ++n) {
    int r = n;
    for (int p : {2, 3, 5})
      while (r % p == 0) r /= p;
    if (r == 1) return n;
  }
}

// Gauss-Legendre nodes and weights on [-1, 1]
void gauss_legendre(int q, std::vector<double>& x, std::vector<double>& w) {
  x.assign(q, 0.0);
  w.assign(q, 0.0);
  for (int i = 0; i < q; ++i) {
    double z = std::cos(M_PI * (i + 0.75) / (q + 0.5)), dp = 0.0;
    for (int it = 0; it < 100; ++it) {
      double p0 = 1.0, p1 = z;
      for (int k = 2; k <= q; ++k) {
        const double p2 = ((2 * k - 1) * z * p1 - (k - 1) * p0) / k;
        p0 = p1;
        p1 = p2;
      }
      dp = q * (z * p1 - p0) / (z * z - 1.0);
      const double dz = p1 / dp;
      z -= dz;
      if (std::fabs(dz) < 1e-17) break;
    }
    x[i] = z;
    w[i] = 2.0 / ((1.0 - z * z) * dp * dp);
  }
}

constexpr int kSpreadRows = 256;  // rows x per workgroup
constexpr int kSpreadMB = 16;     // grid points m per workgroup

// U[m dim + x] = sum_e V[src_e dim + x] wt_e.xy, U2 the same with wt_e.zw (the lambda-weighted
// strengths of the delta_j correction); the entries of grid point m are off[m] .. off[m + 1]
// (uniform across the workgroup: scalar loads), V's column reads coalesced over x
__global__ void __launch_bounds__(kSpreadRows)
k_nufft_spread(const double* __restrict__ V, int dim, int M, const int* __restrict__ off,
               const int* __restrict__ src, const double4* __restrict__ wt, double2* __restrict__ U,
               double2* __restrict__ U2) {
  const int x = blockIdx.x * kSpreadRows + threadIdx.x;
  const int m0 = blockIdx.y * kSpreadMB;
  if (x >= dim) return;
#pragma unroll 1
  for (int mm = 0; mm < kSpreadMB; ++mm) {
    const int m = m0 + mm;
    if (m >= M) break;
    double2 a = make_double2(0.0, 0.0), b = make_double2(0.0, 0.0);
    const int e1 = off[m + 1];
#pragma unroll 2
    for (int e = off[m]; e < e1; ++e) {
      const double v = V[(size_t)src[e] * dim + x];
      const double4 c = wt[e];
      a.x = fma(v, c.x, a.x);
      a.y = fma(v, c.y, a.y);
      b.x = fma(v, c.z, b.x);
      b.y = fma(v, c.w, b.y);
    }
    U[(size_t)m * dim + x] = a;
    U2[(size_t)m * dim + x] = b;
  }
}

// output j = tb0 + blockIdx.y: mode k = j - half of the transforms, deconvolved (scale_j), plus the
// first-order delta_j term: psi'_x = scale_j (F - i delta_j G), interleaved into column blockIdx.y
__global__ void __launch_bounds__(256)
k_nufft_extract(const double2* __restrict__ U, const double2* __restrict__ U2, int dim, int M, int half,
                const double* __restrict__ scale, const double* __restrict__ delta, int tb0,
                double2* __restrict__ Psi) {
  const int x = blockIdx.x * 256 + threadIdx.x;
  if (x >= dim) return;
  const int j = tb0 + (int)blockIdx.y;
  const int k = j - half;
  const size_t ik = (size_t)(k < 0 ? k + M : k);
  const double2 f = U[ik * dim + x], g = U2[ik * dim + x];
  const double sc = scale[j], dl = delta[j];
  Psi[(size_t)blockIdx.y * dim + x] = make_double2(sc * fma(dl, g.y, f.x), sc * fma(-dl, g.x, f.y));
}

// c_a = <v_a | e_x0> = V[x0 + a dim] (row x0 of the eigenvector matrix)
__global__ void __launch_bounds__(256)
k_nufft_row(const double* __restrict__ V, int dim, uint64_t x0, double* __restrict__ c) {
  const int a = blockIdx.x * 256 + threadIdx.x;
  if (a < dim) c[a] = V[x0 + (size_t)a * dim];
}

}  // namespace

// ---- grid ----------------------------------------------------------------------------------

bool nufft_grid(const double* tau, int n_t, double lam_max, NufftGrid& g) {
  if (n_t < 2 || !(tau[1] > 0.0)) return false;
  g = NufftGrid{};
  g.T = n_t;
  g.half = n_t / 2;
  g.s = tau[1] - tau[0];  // tau[0] = 0 in the dense engine (times relative to the first)
  g.delta.resize(n_t);
  double dmax = 0.0;
  for (int j = 0; j < n_t; ++j) {  // delta_j = tau_j - j s, exact in double-double
    const hdd p = two_prod((double)j, g.s);
    const double d = (tau[j] - p.hi) - p.lo;
    g.delta[j] = d;
    dmax = std::max(dmax, std::fabs(d));
  }
  // first order in lambda delta: the dropped term is (lambda delta)^2 / 2 <= 5e-15
  if (!(dmax * lam_max <= 1e-7)) return false;
  g.M = nice_fft_length(2 * n_t);
  g.W = kNufftW;
  g.beta = 2.30 * kNufftW;
  g.h = 2.0 * M_PI / g.M;
  g.alpha = 0.5 * kNufftW * g.h;
  // scale_j = (2 pi / M) / phi_hat(k), phi_hat(k) = alpha int_{-1}^{1} phi(z) cos(k alpha z) dz
  std::vector<double> gx, gw;
  gauss_legendre(200, gx, gw);
  std::vector<double> ph(gx.size());
  for (size_t q = 0; q < gx.size(); ++q) ph[q] = gw[q] * std::exp(g.beta * (std::sqrt(1.0 - gx[q] * gx[q]) - 1.0));
  g.scale.resize(n_t);
  for (int j = 0; j < n_t; ++j) {
    const double k = (double)(j - g.half);
    double s = 0.0;
    for (size_t q = 0; q < gx.size(); ++q) s += ph[q] * std::cos(k * g.alpha * gx[q]);
    g.scale[j] = (2.0 * M_PI / g.M) / (g.alpha * s);
  }
  return true;
}

// ---- spreading tables of one register -------------------------------------------------------

void nufft_sources(const NufftGrid& g, int dim, const double* lam_hi, const double* lam_lo, const double* c,
                   std::vector<int>& off, std::vector<int>& src, std::vector<double>& wt) {
  const int M = g.M;
  const hdd two_pi_m = {kTwoPi.hi / M, 0.0};
  // 2 pi / M in double-double
  hdd hm = two_pi_m;
  {
    const hdd back = dd_mul(hm, hdd{(double)M, 0.0});
    const hdd r = dd_add(kTwoPi, hdd{-back.hi, -back.lo});
    hm = dd_add(hm, hdd{r.hi / M, 0.0});
  }
  const hdd hs = two_prod((double)g.half, g.s);  // exact: half < 2^31, s fp64
  struct Ent {
    int a;
    double zr;  // (x_m - theta_a) / alpha
  };
  std::vector<int> cnt(M + 1, 0);
  std::vector<double> th(dim), dre(dim), dim_(dim);
  for (int a = 0; a < dim; ++a) {
    const hdd lam = {lam_hi[a], lam_lo[a]};
    const hdd theta = dd_mod2pi(dd_mul(lam, hdd{g.s, 0.0}));
    const hdd phase = dd_mod2pi(dd_mul(lam, hs));  // (T/2) lambda s mod 2 pi: the centring factor
    th[a] = theta.hi + theta.lo;  // position for the window search only
    const double ph = phase.hi + phase.lo;
    dre[a] = c[a] * std::cos(ph);
    dim_[a] = -c[a] * std::sin(ph);
    const int mlo = (int)std::ceil((th[a] - g.alpha) / g.h), mhi = (int)std::floor((th[a] + g.alpha) / g.h);
    for (int m = mlo; m <= mhi; ++m) ++cnt[((m % M) + M) % M + 1];
  }
  off.assign(M + 1, 0);
  for (int m = 0; m < M; ++m) off[m + 1] = off[m] + cnt[m + 1];
  const int nnz = off[M];
  src.assign(nnz, 0);
  wt.assign(4 * (size_t)nnz, 0.0);
  std::vector<int> fill(off.begin(), off.end() - 1);
  for (int a = 0; a < dim; ++a) {
    const hdd lam = {lam_hi[a], lam_lo[a]};
    const hdd theta = dd_mod2pi(dd_mul(lam, hdd{g.s, 0.0}));
    const int mlo = (int)std::ceil((th[a] - g.alpha) / g.h), mhi = (int)std::floor((th[a] + g.alpha) / g.h);
    for (int m = mlo; m <= mhi; ++m) {
      // x_m - theta_a in double-double (x_m = m 2 pi / M, m may run one period below 0 or above M)
      const hdd xm = dd_mul(hm, hdd{(double)m, 0.0});
      const hdd dx = dd_add(xm, hdd{-theta.hi, -theta.lo});
      const double z = (dx.hi + dx.lo) / g.alpha;
      const double phi = std::fabs(z) < 1.0 ? std::exp(g.beta * (std::sqrt(1.0 - z * z) - 1.0)) : 0.0;
      const int mm = ((m % M) + M) % M;
      const int e = fill[mm]++;
      src[e] = a;
      wt[4 * (size_t)e + 0] = dre[a] * phi;
      wt[4 * (size_t)e + 1] = dim_[a] * phi;
      wt[4 * (size_t)e + 2] = lam.hi * dre[a] * phi;
      wt[4 * (size_t)e + 3] = lam.hi * dim_[a] * phi;
    }
  }
}

// ---- rocFFT plans --------------------------------------------------------------------------

struct NufftCache {
  struct Plan {
    rocfft_plan plan = nullptr;
    rocfft_execution_info info = nullptr;
    void* work = nullptr;
    size_t work_b = 0;
  };
  std::map<std::pair<int, int>, Plan> plans;  // (M, dim)
  bool setup = false;
};

void nufft_release(NufftCache* c) {
  if (!c) return;
  for (auto& kv : c->plans) {
    if (kv.second.info) rocfft_execution_info_destroy(kv.second.info);
    if (kv.second.plan) rocfft_plan_destroy(kv.second.plan);
    if (kv.second.work) (void)hipFree(kv.second.work);
  }
  delete c;
}

// in-place forward FFT along m of U[m dim + x] for every row x (batch dim, stride dim, distance 1)
static int nufft_fft(NufftCache*& cache, int M, int dim, double2* U, hipStream_t st) {
  if (!cache) cache = new NufftCache;
  if (!cache->setup) {
    if (rocfft_setup() != rocfft_status_success) return -1;
    cache->setup = true;
  }
  auto key = std::make_pair(M, dim);
  auto it = cache->plans.find(key);
  if (it == cache->plans.end()) {
    NufftCache::Plan p;
    rocfft_plan_description desc = nullptr;
    if (rocfft_plan_description_create(&desc) != rocfft_status_success) return -1;
    const size_t stride = (size_t)dim, dist = 1, len = (size_t)M;
    rocfft_status s = rocfft_plan_description_set_data_layout(
        desc, rocfft_array_type_complex_interleaved, rocfft_array_type_complex_interleaved, nullptr, nullptr, 1,
        &stride, dist, 1, &stride, dist);
    if (s == rocfft_status_success)
      s = rocfft_plan_create(&p.plan, rocfft_placement_inplace, rocfft_transform_type_complex_forward,
                             rocfft_precision_double, 1, &len, (size_t)dim, desc);
    rocfft_plan_description_destroy(desc);
    if (s != rocfft_status_success) return -2;
    if (rocfft_plan_get_work_buffer_size(p.plan, &p.work_b) != rocfft_status_success) return -2;
    if (p.work_b && hipMalloc(&p.work, p.work_b) != hipSuccess) {
      rocfft_plan_destroy(p.plan);
      return -3;
    }
    if (rocfft_execution_info_create(&p.info) != rocfft_status_success) return -2;
    if (p.work_b && rocfft_execution_info_set_work_buffer(p.info, p.work, p.work_b) != rocfft_status_success)
      return -2;
    it = cache->plans.emplace(key, p).first;
  }
  if (rocfft_execution_info_set_stream(it->second.info, st) != rocfft_status_success) return -2;
  void* buf[1] = {U};
  return rocfft_execute(it->second.plan, buf, nullptr, it->second.info) == rocfft_status_success ? 0 : -2;
}

size_t nufft_scratch_doubles(const NufftGrid& g, int dim) {
  // U, U2 (complex), the row c, the per-output tables; the source tables are per register
  return 2 * 2 * (size_t)g.M * dim + dim + 2 * (size_t)g.T;
}

int nufft_outputs(NufftCache*& cache, hipStream_t st, const NufftGrid& g, const NufftScratch& S, const double* V,
                  const double* lam_hi, const double* lam_lo, uint64_t x0, int dim, double* Psi, int TB,
                  const std::function<int(int tb0, int tb)>& per_block) {
  // eigenvalues (refined) and c = row x0 of V to the host
  hipLaunchKernelGGL(k_nufft_row, dim3((dim + 255) / 256), dim3(256), 0, st, V, dim, x0, S.c);
  std::vector<double> lh(dim), ll(dim), c(dim);
  if (hipMemcpyAsync(lh.data(), lam_hi, dim * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(ll.data(), lam_lo, dim * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(c.data(), S.c, dim * sizeof(double), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return -1;
  std::vector<int> off, src;
  std::vector<double> wt;
  nufft_sources(g, dim, lh.data(), ll.data(), c.data(), off, src, wt);
  const size_t nnz = src.size();
  if (nnz > S.nnz_cap) return -4;
  if (hipMemcpyAsync(S.off, off.data(), off.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(S.src, src.data(), nnz * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess ||
      hipMemcpyAsync(S.wt, wt.data(), wt.size() * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess)
    return -1;
  hipLaunchKernelGGL(k_nufft_spread, dim3((dim + kSpreadRows - 1) / kSpreadRows, (g.M + kSpreadMB - 1) / kSpreadMB),
                     dim3(kSpreadRows), 0, st, V, dim, g.M, S.off, S.src, (const double4*)S.wt, S.U, S.U2);
  if (hipGetLastError() != hipSuccess) return -1;
  int rc = nufft_fft(cache, g.M, dim, S.U, st);
  if (rc == 0) rc = nufft_fft(cache, g.M, dim, S.U2, st);
  if (rc) return rc;
  for (int tb0 = 0; tb0 < g.T; tb0 += TB) {
    const int tb = std::min(TB, g.T - tb0);
    hipLaunchKernelGGL(k_nufft_extract, dim3((dim + 255) / 256, tb), dim3(256), 0, st, S.U, S.U2, dim, g.M, g.half,
                       S.scale, S.delta, tb0, (double2*)Psi);
    if (hipGetLastError() != hipSuccess) return -1;
    if ((rc = per_block(tb0, tb))) return rc;
  }
  // (the host tables above stay alive until here: the copies are asynchronous)
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

}  // namespace dse
