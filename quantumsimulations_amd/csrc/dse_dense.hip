// dse_dense.hip -- kernels of the dense eigen-propagator engine (dse_dense.h).
//
// The eigendecomposition (rocSOLVER dsyevd) and the Psi' = V P product (rocBLAS dgemm, MFMA
// FP64) are library calls made by the runtime (dse_runtime.hip, dense_run); the kernels here
// build H' from the coefficient tables, form the phase columns, and reduce the observables.
#include "dse_dense.h"

namespace dse {
namespace {

// i^m for m mod 4, as (re, im)
__device__ __forceinline__ double2 ipow(int m) {
  m &= 3;
  return make_double2(m == 0 ? 1.0 : (m == 2 ? -1.0 : 0.0), m == 1 ? 1.0 : (m == 3 ? -1.0 : 0.0));
}

// Diagonal element <x|H'|x> (fp64, one fixed order: k_dense_h and k_dense_rq must agree bitwise).
__device__ __forceinline__ double dense_diag(const DenseProb& P, uint32_t x) {
  const int n = P.n;
  double d = 0.0;
  for (int i = 0; i < n; ++i) {
    const double si = 0.5 - (double)((x >> i) & 1u);
    d += P.field[i] * si;
    for (int j = i + 1; j < n; ++j) d += P.zz[i * n + j] * si * (0.5 - (double)((x >> j) & 1u));
  }
  return d;
}

// Off-diagonal elements <y|H'|x> of column x: f(y, value) for every drive flip and pair flip.
template <typename F>
__device__ __forceinline__ void dense_offdiag(const DenseProb& P, uint32_t x, F&& f) {
  const int n = P.n;
  const int px = __popc(x);
  for (int b = 0; b < n; ++b) {
    const double* fl = P.flip + 4 * b;
    if (fl[0] == 0.0 && fl[1] == 0.0 && fl[2] == 0.0 && fl[3] == 0.0) continue;
    const uint32_t y = x ^ (1u << b);
    const uint32_t vb = (y >> b) & 1u;  // output bit value selects the coefficient
    const double cr = vb ? fl[2] : fl[0], ci = vb ? fl[3] : fl[1];
    double v = cr;
    if (P.rot) {  // i^{|y| - |x|} c, real by construction (imaginary drive)
      const double2 ph = ipow(__popc(y) - px);
      v = ph.x * cr - ph.y * ci;
    }
    f(y, v);
  }
  for (int i = 0; i < n; ++i)
    for (int j = i + 1; j < n; ++j) {
      const double g = P.pair[i * n + j];
      if (g == 0.0 || (((x >> i) ^ (x >> j)) & 1u)) continue;
      f(x ^ ((1u << i) | (1u << j)), P.rot ? -g : g);  // i^{+-2} = -1
    }
}

// Column x of H' (rows y with <y|H'|x> != 0); V is zero on entry.  Matrix elements follow
// dipolar_ensemble_with_rare.py:453-588 in the bitwise form of SURVEY.md Appendix A.
__global__ void __launch_bounds__(256)
k_dense_h(const DenseProb* __restrict__ probs, int dim) {
  const DenseProb& P = probs[blockIdx.y];
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= (uint32_t)dim) return;
  double* col = P.V + (size_t)x * dim;
  col[x] = dense_diag(P, x);
  dense_offdiag(P, x, [&](uint32_t y, double v) { col[y] = v; });
}

// ---- double-double arithmetic (value = hi + lo, |lo| <= ulp(hi) / 2) ----
// No FMA contraction from here to the end of k_dense_phase: HIP compiles with -ffp-contract=fast,
// and a contracted p.hi + p.lo (p.hi = a * b) is fma(a, b, p.lo), which counts the product's
// rounding error twice -- every double-double product then carries an fp64-sized error, and the
// refined eigenvalues were no better than ~eps |H| (round 4's 1.3e-8 at 30 s; 1e-13 without it).
// The explicit fma() calls below are the intended ones.
#pragma clang fp contract(off)
struct ddv {
  double hi, lo;
};
__device__ __forceinline__ ddv dd_two_sum(double a, double b) {
  const double s = a + b;
  const double bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ ddv dd_fast(double a, double b) {  // |a| >= |b|
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ ddv dd_add(ddv a, ddv b) {
  ddv s = dd_two_sum(a.hi, b.hi);
  s.lo += a.lo + b.lo;
  return dd_fast(s.hi, s.lo);
}
__device__ __forceinline__ ddv dd_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
__device__ __forceinline__ ddv dd_mul_d(ddv a, double b) {
  ddv p = dd_prod(a.hi, b);
  p.lo = fma(a.lo, b, p.lo);
  return dd_fast(p.hi, p.lo);
}
__device__ __forceinline__ ddv dd_div(ddv a, ddv b) {
  const double q1 = a.hi / b.hi;
  ddv r = dd_add(a, dd_mul_d(b, -q1));
  const double q2 = r.hi / b.hi;
  return dd_fast(q1, q2);
}

// The diagonal element <x|H'|x> EXACTLY (to double-double): every term field_i s_i, zz_ij s_i s_j is
// an fp64 coefficient times +-1/2 or +-1/4 (exact), so only the sum rounds -- k_dense_h's fp64
// diagonal carries a few ulp of it (~|H| 1e-16), which at the reference grid's 30 s would be a
// phase of ~1e-8.  The refined eigenvalues are therefore those of H' with the exact diagonal.
__device__ __forceinline__ ddv dense_diag_dd(const DenseProb& P, uint32_t x) {
  const int n = P.n;
  ddv d = {0.0, 0.0};
  for (int i = 0; i < n; ++i) {
    const double si = 0.5 - (double)((x >> i) & 1u);
    d = dd_add(d, ddv{P.field[i] * si, 0.0});
    for (int j = i + 1; j < n; ++j) d = dd_add(d, ddv{P.zz[i * n + j] * (si * (0.5 - (double)((x >> j) & 1u))), 0.0});
  }
  return d;
}

// the exact diagonal of every row, once (k_dense_rq reads it for every eigenvector)
__global__ void __launch_bounds__(256)
k_dense_diag(const DenseProb* __restrict__ probs, int dim) {
  const DenseProb& P = probs[blockIdx.y];
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= (uint32_t)dim) return;
  const ddv d = dense_diag_dd(P, x);
  P.diag_dd[2 * (size_t)x] = d.hi;
  P.diag_dd[2 * (size_t)x + 1] = d.lo;
}

// Rayleigh quotient of eigenvector a (column a of V) in double-double: one workgroup per
// (eigenvector, problem); thread partials summed in a fixed order (deterministic)
__global__ void __launch_bounds__(256)
k_dense_rq(const DenseProb* __restrict__ probs, int dim) {
  __shared__ double red[4][256];
  const DenseProb& P = probs[blockIdx.y];
  const uint32_t a = blockIdx.x;
  const double* v = P.V + (size_t)a * dim;
  const double2* dg = reinterpret_cast<const double2*>(P.diag_dd);
  ddv num = {0.0, 0.0}, den = {0.0, 0.0};
  for (uint32_t x = threadIdx.x; x < (uint32_t)dim; x += 256u) {
    const double vx = v[x];
    const double2 dx = dg[x];
    ddv y = dd_mul_d(ddv{dx.x, dx.y}, vx);
    dense_offdiag(P, x, [&](uint32_t yy, double c) { y = dd_add(y, dd_prod(c, v[yy])); });
    num = dd_add(num, dd_mul_d(y, vx));
    den = dd_add(den, dd_prod(vx, vx));
  }
  const int t = threadIdx.x;
  red[0][t] = num.hi, red[1][t] = num.lo, red[2][t] = den.hi, red[3][t] = den.lo;
  __syncthreads();
  if (t == 0) {
    ddv sn = {0.0, 0.0}, sd = {0.0, 0.0};
    for (int i = 0; i < 256; ++i) {
      sn = dd_add(sn, ddv{red[0][i], red[1][i]});
      sd = dd_add(sd, ddv{red[2][i], red[3][i]});
    }
    const ddv lam = dd_div(sn, sd);
    P.lam[a] = lam.hi;
    P.lam_lo[a] = lam.lo;
  }
}

// cos and sin of (lam_hi + lam_lo) tau: the product in double-double, reduced modulo 2 pi with a
// three-part 2 pi (the first part 27 significant bits, so k C1 is exact for |k| < 2^26, i.e.
// |lam tau| < 4e8 rad), then sincos of the reduced angle's high part corrected by its low part.
// A plain fp64 product lam * tau rounds the angle by ulp(lam tau): 1.5e-8 rad at 1.5e8 rad,
// the reference grid's 30 s at |lam| ~ 5e6 rad/s.
__device__ __forceinline__ void dd_sincos(double lh, double ll, double tau, double* s, double* c) {
  constexpr double C1 = 0x1.921fb54p+2;            // 2 pi, high 27 bits
  constexpr double C2 = 0x1.10b4611a62633p-28;     // next 53 bits
  constexpr double C3 = 0x1.45c06e0e68948p-84;     // next 53 bits
  constexpr double INV = 0.15915494309189533576888376337251436;
  const ddv p = dd_mul_d(ddv{lh, ll}, tau);
  const double k = rint(p.hi * INV);
  ddv r = dd_two_sum(p.hi, -k * C1);  // k C1 exact
  r = dd_add(r, dd_prod(-k, C2));
  r.lo = fma(-k, C3, r.lo + p.lo);
  r = dd_fast(r.hi, r.lo);
  double sh, ch;
  sincos(r.hi, &sh, &ch);
  *s = fma(ch, r.lo, sh);
  *c = fma(-sh, r.lo, ch);
}

__global__ void __launch_bounds__(256)
k_dense_phase(const DenseProb* __restrict__ probs, int dim, const double* __restrict__ tau, int tb,
              double* __restrict__ Pm, size_t pstride) {
  const DenseProb& P = probs[blockIdx.z];
  const uint32_t a = blockIdx.x * 256u + threadIdx.x;
  const int j = blockIdx.y;
  if (a >= (uint32_t)dim) return;
  const double c = P.V[P.x0 + (size_t)a * dim];  // <v_a | e_x0>
  double s, co;
  if (P.refine)
    dd_sincos(P.lam[a], P.lam_lo[a], tau[j], &s, &co);
  else
    sincos(P.lam[a] * tau[j], &s, &co);
  double* blk = Pm + blockIdx.z * pstride;
  blk[a + (size_t)j * dim] = c * co;
  blk[a + (size_t)(tb + j) * dim] = -c * s;
}
#pragma clang fp contract(fast)

// block sum of 7 values (256 threads = 4 waves)
__device__ __forceinline__ void block_sum7(double* v, double (*red)[8]) {
#pragma unroll
  for (int k = 0; k < 7; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 7; ++k) red[w][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < 7; ++k) v[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// Same sums as k_obs (dse_kernels.hip): 0 Ix_sea, 1 Iy_sea, 2 Iz_sea, 3 Iz_R, 4 Ix_R, 5 Iy_R,
// 6 ||psi||^2, with <Ix_k> = sum_{bit_k(x)=0} Re(conj(psi_x) psi_{x^e_k}), <Iy_k> = Im(...).  In the
// rotated frame psi_x = i^{-|x|} psi'_x, so conj(psi_x) psi_{x^e_k} = -i conj(psi'_x) psi'_{x^e_k}.
// Columns j of Psi' at Psi + p pstride + j colstride (real parts), imaginary parts imoff further,
// elements es doubles apart: the dense engine's [re | im] blocks (colstride dim, imoff tb dim,
// es 1) or interleaved complex states (colstride 2 dim, imoff 1, es 2).
__global__ void __launch_bounds__(256)
k_dense_obs(const DenseProb* __restrict__ probs, int dim, const double* __restrict__ Psi, size_t pstride,
            size_t colstride, size_t imoff, int es, int t0) {
  __shared__ double red[4][8];
  const DenseProb& P = probs[blockIdx.y];
  const int j = blockIdx.x;
  const double* re = Psi + blockIdx.y * pstride + (size_t)j * colstride;
  const double* im = re + imoff;
  const int n = P.n;
  const double half_sea = 0.5 * (double)P.n_sea;
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  for (uint32_t x = threadIdx.x; x < (uint32_t)dim; x += 256u) {
    const double ar = re[(size_t)x * es], ai = im[(size_t)x * es];
    const double p2 = ar * ar + ai * ai;
    v[6] += p2;
    v[2] += p2 * (half_sea - (double)__popcll((uint64_t)x & P.sea_mask));
    if (P.rare_bit >= 0) v[3] += p2 * (0.5 - (double)((x >> P.rare_bit) & 1u));
    for (int b = 0; b < n; ++b) {
      if ((x >> b) & 1u) continue;
      const bool sea = (P.sea_mask >> b) & 1ull;
      const bool rr = (b == P.rare_bit);
      if (!sea && !rr) continue;
      const uint32_t y = x | (1u << b);
      const double br = re[(size_t)y * es], bi = im[(size_t)y * es];
      double zr = ar * br + ai * bi, zi = ar * bi - ai * br;  // conj(a) b
      if (P.rot) {  // -i z
        const double t = zr;
        zr = zi;
        zi = -t;
      }
      if (sea) v[0] += zr, v[1] += zi;
      if (rr) v[4] += zr, v[5] += zi;
    }
  }
  block_sum7(v, red);
  if (threadIdx.x == 0) {
    double* o = P.obs + (size_t)(t0 + j) * 8;
#pragma unroll
    for (int k = 0; k < 7; ++k) o[k] = v[k];
    o[7] = 0.0;
  }
}

// column tb - 1 of Psi' (layout as k_dense_obs: colstride, imoff, es)
__global__ void __launch_bounds__(256)
k_dense_final(const DenseProb* __restrict__ probs, int dim, const double* __restrict__ Psi, size_t pstride,
              size_t colstride, size_t imoff, int es, int tb, double tau_last) {
  const DenseProb& P = probs[blockIdx.y];
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  if (x >= (uint32_t)dim || !P.final_state) return;
  const double* re = Psi + blockIdx.y * pstride + (size_t)(tb - 1) * colstride;
  const double* im = re + imoff;
  // psi_x = exp(-i shift tau) i^{|x0| - |x|} psi'_x   (rot; psi'(0) = e_x0 stands for i^{|x0|} e_x0)
  double s, c;
  if (P.refine)
    dd_sincos(-P.shift, 0.0, tau_last, &s, &c);
  else
    sincos(-P.shift * tau_last, &s, &c);
  double2 ph = make_double2(c, s);
  if (P.rot) {
    const double2 q = ipow(__popcll(P.x0) - __popc(x));
    ph = make_double2(ph.x * q.x - ph.y * q.y, ph.x * q.y + ph.y * q.x);
  }
  const double ar = re[(size_t)x * es], ai = im[(size_t)x * es];
  P.final_state[x] = make_double2(ph.x * ar - ph.y * ai, ph.x * ai + ph.y * ar);
}

}  // namespace

hipError_t launch_dense_h(const DenseProb* d, int count, int dim, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_h, dim3((dim + 255) / 256, count), dim3(256), 0, st, d, dim);
  return hipGetLastError();
}

hipError_t launch_dense_rq(const DenseProb* d, int count, int dim, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_diag, dim3((dim + 255) / 256, count), dim3(256), 0, st, d, dim);
  hipLaunchKernelGGL(k_dense_rq, dim3(dim, count), dim3(256), 0, st, d, dim);
  return hipGetLastError();
}

hipError_t launch_dense_phase(const DenseProb* d, int count, int dim, const double* tau, int tb,
                              double* P, size_t pstride, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_phase, dim3((dim + 255) / 256, tb, count), dim3(256), 0, st, d, dim, tau,
                     tb, P, pstride);
  return hipGetLastError();
}

hipError_t launch_dense_obs(const DenseProb* d, int count, int dim, const double* Psi, size_t pstride,
                            int tb, int t0, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_obs, dim3(tb, count), dim3(256), 0, st, d, dim, Psi, pstride, (size_t)dim,
                     (size_t)tb * dim, 1, t0);
  return hipGetLastError();
}

hipError_t launch_state_obs(const DenseProb* d, int dim, const double2* states, int n_states, int t0,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_dense_obs, dim3(n_states, 1), dim3(256), 0, st, d, dim, (const double*)states,
                     (size_t)0, (size_t)2 * dim, (size_t)1, 2, t0);
  return hipGetLastError();
}

hipError_t launch_dense_final(const DenseProb* d, int count, int dim, const double* Psi, size_t pstride,
                              int tb, double tau_last, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_final, dim3((dim + 255) / 256, count), dim3(256), 0, st, d, dim, Psi,
                     pstride, (size_t)dim, (size_t)tb * dim, 1, tb, tau_last);
  return hipGetLastError();
}

hipError_t launch_dense_obs_c(const DenseProb* d, int dim, const double* Psi, int tb, int t0, hipStream_t st) {
  hipLaunchKernelGGL(k_dense_obs, dim3(tb, 1), dim3(256), 0, st, d, dim, Psi, (size_t)0, (size_t)2 * dim,
                     (size_t)1, 2, t0);
  return hipGetLastError();
}

hipError_t launch_dense_final_c(const DenseProb* d, int dim, const double* Psi, int tb, double tau_last,
                                hipStream_t st) {
  hipLaunchKernelGGL(k_dense_final, dim3((dim + 255) / 256, 1), dim3(256), 0, st, d, dim, Psi, (size_t)0,
                     (size_t)2 * dim, (size_t)1, 2, tb, tau_last);
  return hipGetLastError();
}

}  // namespace dse
