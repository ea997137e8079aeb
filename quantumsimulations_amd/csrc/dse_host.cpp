// dse_host.cpp -- device-independent pieces of libdse: spectral bounds and Chebyshev
// (Bessel) coefficients.  Pure C++, callable without a GPU (tests use them on CPU).
//
// The reference integrates i d/dt psi = H psi with QuTiP's sesolve (ZVODE-Adams,
// dipolar_ensemble_with_rare.py:653-666).  H is time independent (the rf drive is static in
// the rotating frame, :469-471, :514-530), so the engine propagates each output interval
// exactly:  exp(-i H dt) = exp(-i beta dt) sum_k (2 - delta_k0) (-i)^k J_k(alpha dt) T_k(Ht),
// Ht = (H - beta)/alpha with spectrum(H) inside [beta - alpha, beta + alpha].
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/dse.h"

extern "C" int dse_abi_version(void) { return DSE_ABI_VERSION; }

extern "C" int dse_spectral_bounds(int n, const double* field, const double* zz, const double* pair,
                                   const double* flip, double shift, double* e_min, double* e_max) {
  if (n < 1 || n > DSE_MAX_QUBITS || !field || !zz || !pair || !flip || !e_min || !e_max)
    return DSE_ERR_ARG;
  // Weyl: lambda_min(sum A_k) >= sum lambda_min(A_k), same for max.
  double lo = shift, hi = shift;
  for (int k = 0; k < n; ++k) {
    const double c = std::hypot(flip[4 * k + 2], flip[4 * k + 3]);
    const double r = std::sqrt(0.25 * field[k] * field[k] + c * c);  // field*s_k + drive: +-r
    lo -= r;
    hi += r;
  }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      // zz s_i s_j + pair flip on {00,11}: zz/4 +- |g|; on {01,10}: -zz/4
      const double q = 0.25 * zz[i * n + j], g = std::fabs(pair[i * n + j]);
      lo += std::fmin(q - g, -q);
      hi += std::fmax(q + g, -q);
    }
  *e_min = lo;
  *e_max = hi;
  return DSE_OK;
}

// J_k(z) for k = 0..kmax by Miller's backward recurrence J_{k-1} = (2k/z) J_k - J_{k+1},
// started far above max(kmax, z) and normalised with J_0 + 2 sum_{k>=1} J_{2k} = 1.
extern "C" int dse_bessel_j(double z, int kmax, double* out, double tol, int* degree) {
  if (kmax < 1 || !out || !(z >= 0.0) || !std::isfinite(z)) return DSE_ERR_ARG;
  if (z == 0.0) {
    out[0] = 1.0;
    for (int k = 1; k <= kmax; ++k) out[k] = 0.0;
    if (degree) *degree = 1;
    return DSE_OK;
  }
  // start index: beyond both kmax and the turning point z, plus a margin for decay below 1e-300
  const int m0 = (int)std::ceil(std::fmax((double)kmax, z) + 60.0 + 12.0 * std::cbrt(z + 1.0));
  const int m = m0 + (m0 & 1);  // even
  std::vector<double> j(m + 2, 0.0);
  j[m] = 1e-300;
  for (int k = m; k >= 1; --k) {
    j[k - 1] = (2.0 * k / z) * j[k] - j[k + 1];
    if (std::fabs(j[k - 1]) > 1e250)  // rescale everything computed so far
      for (int q = k - 1; q <= m + 1; ++q) j[q] *= 1e-250;
  }
  double norm = j[0];
  for (int k = 2; k <= m; k += 2) norm += 2.0 * j[k];
  const double inv = 1.0 / norm;
  for (int k = 0; k <= kmax; ++k) out[k] = j[k] * inv;
  if (degree) {
    int d = 1;
    for (int k = (int)std::fmin((double)m, (double)kmax); k >= 1; --k)
      if (std::fabs(j[k] * inv) > tol) { d = k; break; }
    // the tail beyond d sums below ~tol because |J_k| decays super-exponentially past z
    *degree = d < 1 ? 1 : d;
  }
  return DSE_OK;
}
