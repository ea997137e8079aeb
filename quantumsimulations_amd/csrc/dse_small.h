// dse_small.h -- the small-register engine (dse_small.hip): registers of n <= 9 qubits, one wave
// per problem, all Chebyshev terms and the observables of a chunk of output intervals per launch.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dse {

constexpr int kSmallMaxQubits = 9;

struct SmallProb {
  double2* state;          // [2^n] the state at the start of the next launch
  const double* field;     // [n]
  const double* zz;        // [n*n]
  const double* pair;      // [n*n]
  const double* flip;      // [4n] re0 im0 re1 im1 (output bit value 0 / 1)
  const double2* coef;     // [n_sets][kcap1] a_k = e^{-i beta tau} (2 - d_k0) (-i)^k J_k(alpha tau)
  const int* deg;          // [n_sets] Chebyshev degree K of each interval length
  uint64_t sea_mask;
  double shift, beta, s1;
  int n, rare_bit, kcap1, n_t;
};

// One launch: intervals m0 .. m0 + n_int - 1 of problems sel[0 .. count) (all with n qubits);
// out[problem][m + 1][8] = raw observable sums of psi(t_{m+1}) (dse_runtime.hip finish_obs).
hipError_t launch_small(int n, const SmallProb* probs, const int* sel, int count, int m0, int n_int,
                        const int* iv_set, double* out, hipStream_t st);
// out[problem][0][8] = observable sums of the state buffer (psi0)
hipError_t launch_small_obs0(int n, const SmallProb* probs, const int* sel, int count, double* out,
                             hipStream_t st);

}  // namespace dse
