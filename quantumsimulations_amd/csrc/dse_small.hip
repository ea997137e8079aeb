// dse_small.hip -- persistent engine for small registers (n <= 9 qubits: the reference's default
// sweep, n_sea = 6 -> N = 7, sweep_sea_detuning.py:1240).
//
// A register of n <= 9 qubits is at most 512 amplitudes (8 KiB): one wave holds it.  Workgroup =
// one wave = one problem; lane l owns the amplitudes x = r * 64 + l, r < R = 2^(n-6) (n >= 6; a
// smaller register uses its first 2^n lanes).  One launch runs a chunk of output intervals of
// every small problem of the context completely on chip:
//   LDS        w_{k-1} of the register (the operand of H)
//   registers  o (w_k being formed: starts as -w_{k-2} / (2 s1), see k_interval), the propagator
//              sum acc of the interval (ONE output per series: the coarse-grid regime these
//              registers live in, alpha dt ~ 1e3..1e4 on the reference's 30 s grid), D(x) - beta
// At each output time acc = psi(t_m) goes to LDS, the 7 observable sums are reduced over the wave
// and written to out[problem][m][8], and acc becomes w_0 of the next interval.  Between launches
// the state lives in the problem's buffer.  Every term is compile-time structure (the masks of
// all n drives and n (n - 1) / 2 pairs are known for a given n; coefficients come from LDS), so
// a term costs n + n(n-1)/2 LDS partner reads per amplitude and no other memory traffic.
// Launches: ceil((n_t - 1) / chunk), independent of the Chebyshev degree (the per-term streaming
// kernels would need one launch per term: ~1e8 for a 30 s N = 7 evolution).
#include "dse_device.h"
#include "dse_small.h"

namespace dse {
namespace {

template <int N>
struct SmallGeo {
  static constexpr int DIM = 1 << N;
  static constexpr int R = N >= 6 ? (1 << (N - 6)) : 1;
  static constexpr int NP = N * (N - 1) / 2;
};

template <int N>
__global__ void __launch_bounds__(64)
k_small(const SmallProb* __restrict__ probs, const int* __restrict__ sel, int m0, int n_int,
        const int* __restrict__ iv_set, double* __restrict__ out) {
  using G = SmallGeo<N>;
  constexpr int R = G::R, DIM = G::DIM, NP = G::NP;
  __shared__ double2 w[DIM];
  __shared__ double2 fl[N][2];  // drive coefficient of bit b for output bit value v
  __shared__ double pg[NP > 0 ? NP : 1];
  __shared__ int pm[NP > 0 ? NP : 1];   // pair masks e_i | e_j
  __shared__ double red[8];

  const SmallProb& P = probs[sel[blockIdx.x]];
  const int lane = threadIdx.x;
  const bool live = lane < DIM;
  const gd2* gst_ = gptr((const double2*)P.state);

  // tables -> LDS; the diagonal D(x) - beta of the owned amplitudes -> registers
  if (lane < N) {
    fl[lane][0] = make_double2(P.flip[4 * lane + 0], P.flip[4 * lane + 1]);
    fl[lane][1] = make_double2(P.flip[4 * lane + 2], P.flip[4 * lane + 3]);
  }
  for (int e = lane; e < NP; e += 64) {
    int i = 0, rem = e;
    while (rem >= N - 1 - i) rem -= N - 1 - i, ++i;
    pg[e] = P.pair[i * N + i + 1 + rem];
    pm[e] = (1 << i) | (1 << (i + 1 + rem));
  }
  double dmb[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int x = r * 64 + lane;
    double d = P.shift - P.beta;
    for (int b = 0; b < N; ++b) {
      const double sb = 0.5 - (double)((x >> b) & 1);
      d += P.field[b] * sb;
      for (int c = b + 1; c < N; ++c) d += P.zz[b * N + c] * (sb * (0.5 - (double)((x >> c) & 1)));
    }
    dmb[r] = d;
    if (live) w[x] = gld(gst_, x);
  }
  __syncthreads();

  const double s1 = P.s1, inv2s1 = 0.5 / s1;
  for (int mi = 0; mi < n_int; ++mi) {
    const int m = m0 + mi;  // interval [t_m, t_{m+1}]
    const int set = iv_set[m];
    const cptr<double> a = (cptr<double>)(P.coef + (size_t)set * P.kcap1);  // a_k = (a[2k], a[2k+1])
    const int K = P.deg[set];
    double2 o[R], acc[R];
    {
      const double2 a0 = make_double2(a[0], a[1]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double2 v = live ? w[r * 64 + lane] : make_double2(0.0, 0.0);
        acc[r] = cmad(make_double2(0.0, 0.0), a0.x, a0.y, v);
        o[r] = make_double2(0.0, 0.0);
      }
    }
    for (int k = 1; k <= K; ++k) {
      double2 own[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int x = r * 64 + lane;
        own[r] = live ? w[x] : make_double2(0.0, 0.0);
        o[r].x = fma(dmb[r], own[r].x, o[r].x);
        o[r].y = fma(dmb[r], own[r].y, o[r].y);
      }
#pragma unroll
      for (int b = 0; b < N; ++b) {
        const double2 c0 = fl[b][0], c1 = fl[b][1];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int x = r * 64 + lane;
          if (!live) continue;
          const double2 c = ((x >> b) & 1) ? c1 : c0;
          o[r] = cmad(o[r], c.x, c.y, w[x ^ (1 << b)]);
        }
      }
      if (N <= 7) {  // every pair's mask at compile time
        int e = 0;
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = i + 1; j < N; ++j, ++e) {
            const double g = pg[e];
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int x = r * 64 + lane;
              if (!live || (((x >> i) ^ (x >> j)) & 1)) continue;
              const double2 v = w[x ^ ((1 << i) | (1 << j))];
              o[r].x = fma(g, v.x, o[r].x);
              o[r].y = fma(g, v.y, o[r].y);
            }
          }
      } else {  // 28 / 36 pairs: a loop (an unrolled one hoists every coefficient into registers)
#pragma unroll 1
        for (int e = 0; e < NP; ++e) {
          const double g = pg[e];
          const int m = pm[e];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const int x = r * 64 + lane;
            if (!live || (__popc(x & m) & 1)) continue;
            const double2 v = w[x ^ m];
            o[r].x = fma(g, v.x, o[r].x);
            o[r].y = fma(g, v.y, o[r].y);
          }
        }
      }
      const double sc = (k == 1) ? s1 : 2.0 * s1;
      const double2 ak = make_double2(a[2 * k], a[2 * k + 1]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        o[r].x *= sc;
        o[r].y *= sc;
        acc[r] = cmad(acc[r], ak.x, ak.y, o[r]);
      }
      __syncthreads();  // all reads of w_{k-1} done
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int x = r * 64 + lane;
        if (live) w[x] = o[r];
        o[r] = make_double2(-inv2s1 * own[r].x, -inv2s1 * own[r].y);  // the next term's -w_{k-2}/(2 s1)
      }
      __syncthreads();
    }
    // psi(t_{m+1}) = acc -> LDS (w_0 of the next interval), then its observables
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (live) w[r * 64 + lane] = acc[r];
    __syncthreads();
    double v[7] = {0, 0, 0, 0, 0, 0, 0};
    if (live) {
      const double half_sea = 0.5 * (double)__popcll(P.sea_mask);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int x = r * 64 + lane;
        const double2 p = acc[r];
        const double p2 = p.x * p.x + p.y * p.y;
        v[6] += p2;
        v[2] += p2 * (half_sea - (double)__popcll((uint64_t)x & P.sea_mask));
        if (P.rare_bit >= 0) v[3] += p2 * (0.5 - (double)((x >> P.rare_bit) & 1));
#pragma unroll
        for (int b = 0; b < N; ++b) {
          const bool sea = (P.sea_mask >> b) & 1ull, rr = (b == P.rare_bit);
          if ((!sea && !rr) || ((x >> b) & 1)) continue;
          const double2 s = w[x ^ (1 << b)];
          const double re = p.x * s.x + p.y * s.y, im = p.x * s.y - p.y * s.x;
          if (sea) v[0] += re, v[1] += im;
          if (rr) v[4] += re, v[5] += im;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double t = v[j];
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);
      if (lane == 0) red[j] = t;
    }
    __syncthreads();
    if (lane < 8) out[((size_t)sel[blockIdx.x] * P.n_t + (m + 1)) * 8 + lane] = lane < 7 ? red[lane] : 0.0;
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (live) gst(gptr((double2*)P.state), r * 64 + lane, w[r * 64 + lane]);
}

// observables of the initial state (output 0)
template <int N>
__global__ void __launch_bounds__(64)
k_small_obs0(const SmallProb* __restrict__ probs, const int* __restrict__ sel, double* __restrict__ out) {
  using G = SmallGeo<N>;
  constexpr int R = G::R, DIM = G::DIM;
  __shared__ double2 w[DIM];
  const SmallProb& P = probs[sel[blockIdx.x]];
  const int lane = threadIdx.x;
  const bool live = lane < DIM;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (live) w[r * 64 + lane] = gld(gptr((const double2*)P.state), r * 64 + lane);
  __syncthreads();
  double v[7] = {0, 0, 0, 0, 0, 0, 0};
  if (live) {
    const double half_sea = 0.5 * (double)__popcll(P.sea_mask);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int x = r * 64 + lane;
      const double2 p = w[x];
      const double p2 = p.x * p.x + p.y * p.y;
      v[6] += p2;
      v[2] += p2 * (half_sea - (double)__popcll((uint64_t)x & P.sea_mask));
      if (P.rare_bit >= 0) v[3] += p2 * (0.5 - (double)((x >> P.rare_bit) & 1));
      for (int b = 0; b < N; ++b) {
        const bool sea = (P.sea_mask >> b) & 1ull, rr = (b == P.rare_bit);
        if ((!sea && !rr) || ((x >> b) & 1)) continue;
        const double2 s = w[x ^ (1 << b)];
        const double re = p.x * s.x + p.y * s.y, im = p.x * s.y - p.y * s.x;
        if (sea) v[0] += re, v[1] += im;
        if (rr) v[4] += re, v[5] += im;
      }
    }
  }
  for (int j = 0; j < 7; ++j) {
    double t = v[j];
    for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);
    v[j] = t;
  }
  if (lane == 0) {
    double* o = out + (size_t)sel[blockIdx.x] * P.n_t * 8;
    for (int j = 0; j < 7; ++j) o[j] = v[j];
    o[7] = 0.0;
  }
}

}  // namespace

#define DSE_SMALL_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9)

hipError_t launch_small(int n, const SmallProb* probs, const int* sel, int count, int m0, int n_int,
                        const int* iv_set, double* out, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  switch (n) {
#define X(q) \
  case q: hipLaunchKernelGGL((k_small<q>), dim3(count), dim3(64), 0, st, probs, sel, m0, n_int, iv_set, out); break;
    DSE_SMALL_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_small_obs0(int n, const SmallProb* probs, const int* sel, int count, double* out,
                             hipStream_t st) {
  if (count <= 0) return hipSuccess;
  switch (n) {
#define X(q) \
  case q: hipLaunchKernelGGL((k_small_obs0<q>), dim3(count), dim3(64), 0, st, probs, sel, out); break;
    DSE_SMALL_CASES(X)
#undef X
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace dse
