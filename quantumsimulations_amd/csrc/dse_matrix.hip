// dse_matrix.hip -- propagator-matrix mode for a lone register (dse_runtime.hip, matrix_run).
//
// simulate_rare(params) hands libdse ONE register at a time (the reference's own call pattern,
// sweep_sea_detuning.py:671-673).  On a uniform output grid its evolution is psi_{j+1} = U psi_j
// with U = exp(-iH dt), so the whole chip builds U once and the outputs are a chain of products:
//
//   k_ucols   one workgroup per column c: U e_c by the Chebyshev series over one interval, in REAL
//             arithmetic.  When the drives are all imaginary (the sweep's phase pi/2) or all real,
//             H' = D H D^dagger (D|x> = i^{popcount x}|x>) is real symmetric (dse_dense.h), so the
//             Chebyshev vectors T_k(H~') e_c are real and
//               U' e_c = e^{-i beta dt} (A_c - i S_c),  A_c = sum_{k even} (-1)^{k/2} c_k T_k e_c,
//                                                      S_c = sum_{k odd} (-1)^{(k-1)/2} c_k T_k e_c
//             (c_k = (2 - delta_k0) J_k(alpha dt)); U_rc = i^{|c| - |r|} U'_rc is written in the
//             computational frame.  Half the FP64 work and half the LDS bytes of the complex
//             column build, no input columns in HBM, and the two sums stay in registers.
//   k_symv    y = U x over the 128 x 128 tiles on and above the diagonal (U_cr = s_r s_c U_rc),
//   k_symv_reduce   the per-tile partial sums in fixed order (deterministic, no atomics).
#include <type_traits>

#include "dse_dense.h"
#include "dse_device.h"

namespace dse {
namespace {

// thread pairs per fused iteration: ceil(C(TB, 2) / TB) (padded with zero pairs)
template <int L>
struct UcGeo {
  static constexpr int TB = RB<L>::TB;
  static constexpr int NPI = (TB * (TB - 1) / 2 + TB - 1) / TB;
};

template <int L>
struct UcShared {
  double w[2][1 << L];                // T_{k-1} e_c and T_{k-2} e_c (roles alternate by term)
  double c[L + 1];                    // F_i and C - beta of the (single) tile
  double zz[L * L];                   // in-register zz couplings (upper triangle)
  double zr[kRegAmps];                // register-bit ZZ part of the diagonal per r
  double sw[RB<L>::TB][8];            // thread bit j: drive (output bit 0 / 1), pairs with register bits 0..3
  DPair tt[RB<L>::TB * UcGeo<L>::NPI];  // pairs of two thread bits (rotated coefficient), zero-padded
};

// rotated real drive coefficient of a flip whose output bit value is v: <y|H'|x> = i^{|y|-|x|} c_v
__device__ __forceinline__ double rot_drive(int rot, int v, double re, double im) {
  return rot ? (v ? -im : im) : re;
}

// LDS vectors keep rows 2p and 2p + 1 of thread t side by side, at w[2 (p NT + t) + (r & 1)]:
// one conflict-free ds_read_b128 per row pair (ds_read_b64 needs ~4 waves per SIMD for full rate,
// MI355X_MICROARCH.md §LDS; this kernel runs 2)
template <int NT>
__device__ __forceinline__ int lidx(int r, int t) {
  return 2 * ((r >> 1) * NT + t) + (r & 1);
}
typedef __attribute__((address_space(3))) dv2 lv2;
// rows r0 .. r0 + n - 1 (r0, n even) of thread t
template <int NT, int N>
__device__ __forceinline__ void ldrows(const double* w, int t, int r0, double* v) {
#pragma unroll
  for (int p = 0; p < N / 2; ++p) {
    const dv2 d = *(const lv2*)(w + 2 * ((r0 / 2 + p) * NT + t));
    v[2 * p] = d.x;
    v[2 * p + 1] = d.y;
  }
}
template <int NT>
__device__ __forceinline__ void ld16(const double* w, int t, double* v) {
  ldrows<NT, kRegAmps>(w, t, 0, v);
}

// U e_c for columns c = col0 + blockIdx.x of a one-tile register (n == L), see the file comment.
// P: the problem (beta, s1 = 1/alpha of the interval set by the caller); cf[k] = (-1)^{floor(k/2)}
// c_k, k = 0..deg; (phr, phi) = e^{-i beta dt}.
// Per term: w_{k-1} in LDS buffer A is read by every thread (its own rows, then one partner per
// thread bit and per thread pair); w_{k-2} in buffer B only by its owner, which overwrites it with
// w_k -- so one barrier per term, and w_{k-2} needs no registers.  Thread t holds out, and the two
// sums A_c, S_c (16 rows each).  The fused loop visits thread bit j: the sweep of partner t ^ e_j
// (drive of j, pairs (j, register bit i)) and NPI thread pairs, each next partner's rows loaded
// before the FMAs of the current one.
template <int L>
__global__ void __launch_bounds__(RB<L>::NT, 2)
k_ucols(const DevProb* __restrict__ probs, const double* __restrict__ cf, int deg, int rot, double phr,
        double phi, double2* __restrict__ U, int col0, int c1, double2* __restrict__ psi1) {
  constexpr int NT = RB<L>::NT, R = kRegAmps, TB = RB<L>::TB, NPI = UcGeo<L>::NPI;
  constexpr int T = 1 << L;
  __shared__ UcShared<L> S;
  const DevProb& P = *probs;
  const int tid = threadIdx.x;
  const uint32_t c = (uint32_t)(col0 + blockIdx.x);
  const int ntt = P.n_pairs_tt;

  // ---- tables (rotated real coefficients), w_0 = e_c, w_{-1} = 0 ----
  for (int e = tid; e < L * L; e += NT) {
    const int i = e / L, j = e % L;
    S.zz[e] = (j > i) ? P.zz[i * P.n + j] : 0.0;
  }
  tile_diag_coeffs<L>(P, 0u, P.beta, S.c, tid);
  if (tid < TB) {
    const DSweep& d = P.sweeps[tid];
    S.sw[tid][0] = rot_drive(rot, 0, d.re0, d.im0);
    S.sw[tid][1] = rot_drive(rot, 1, d.re1, d.im1);
#pragma unroll
    for (int i = 0; i < kRegBits; ++i) S.sw[tid][2 + i] = rot ? -d.g[i] : d.g[i];
    S.sw[tid][6] = S.sw[tid][7] = 0.0;
  }
  // iteration j takes NPI pairs for j < ja, NPI - 1 after (no padded pair is executed when the
  // list fills TB * (NPI - 1) .. TB * NPI slots); slots beyond the list hold zero pairs
  const int ja = min(TB, max(0, ntt - TB * (NPI - 1)));
  for (int p = tid; p < TB * NPI; p += NT) {
    const int j = p / NPI, q = p % NPI;
    const int nj = j < ja ? NPI : NPI - 1;
    const int idx = j * NPI - max(0, j - ja) + q;
    DPair e;
    e.mask_lo = 0u, e.tile_xor = 0u, e.g = 0.0;  // the own rows with coefficient 0
    if (q < nj && idx < ntt) {
      e = P.pairs_tt[idx];
      e.g = rot ? -e.g : e.g;
    }
    S.tt[p] = e;
  }
  for (int x = tid; x < T; x += NT) {
    S.w[0][lidx<NT>(x / NT, x % NT)] = (x == (int)c) ? 1.0 : 0.0;
    S.w[1][x] = 0.0;
  }
  __syncthreads();
  if (tid < kRegAmps) {
    double v = 0.0;
    for (int a = 0; a < kRegBits; ++a)
      for (int b = a + 1; b < kRegBits; ++b)
        v += S.zz[(TB + a) * L + TB + b] * ((0.5 - ((tid >> a) & 1)) * (0.5 - ((tid >> b) & 1)));
    S.zr[tid] = v;
  }
  // per-thread diagonal D(r) = zt + sum_i hr[i] s_i(r) + zr[r]
  double zt = S.c[L];
  double hr[kRegBits];
#pragma unroll
  for (int i = 0; i < kRegBits; ++i) hr[i] = S.c[TB + i];
#pragma unroll 1
  for (int j = 0; j < TB; ++j) {
    const double sj = 0.5 - (double)((tid >> j) & 1);
    double a = S.c[j];
#pragma unroll 1
    for (int i = j + 1; i < TB; ++i) a += S.zz[j * L + i] * (0.5 - (double)((tid >> i) & 1));
    zt += a * sj;
#pragma unroll
    for (int i = 0; i < kRegBits; ++i) hr[i] += S.zz[j * L + TB + i] * sj;
  }
  // register-bit drives and pairs (rotated, uniform)
  double rd[kRegBits][2], rg[kRegPairs];
#pragma unroll
  for (int i = 0; i < kRegBits; ++i) {
    const bool on = (P.rflip_mask >> i) & 1;
    rd[i][0] = on ? rot_drive(rot, 0, P.rflip[i][0], P.rflip[i][1]) : 0.0;
    rd[i][1] = on ? rot_drive(rot, 1, P.rflip[i][2], P.rflip[i][3]) : 0.0;
  }
#pragma unroll
  for (int q = 0; q < kRegPairs; ++q) rg[q] = rot ? -P.rr_g[q] : P.rr_g[q];
  __syncthreads();  // S.zr

  const double s1 = P.s1;
  double ac[R], as[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    ac[r] = ((uint32_t)(r * NT + tid) == c) ? cf[0] : 0.0;
    as[r] = 0.0;
  }

#pragma unroll 1
  for (int k = 1; k <= deg; ++k) {
    const double* A = S.w[(k - 1) & 1];  // w_{k-1}
    double* B = S.w[k & 1];              // w_{k-2}, then w_k
    double out[R];
    {
      double own[R];
      ld16<NT>(A, tid, own);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        double d = zt + S.zr[r];
#pragma unroll
        for (int i = 0; i < kRegBits; ++i) d += ((r >> i) & 1 ? -0.5 : 0.5) * hr[i];
        out[r] = d * own[r];
      }
#pragma unroll
      for (int i = 0; i < kRegBits; ++i)
#pragma unroll
        for (int r = 0; r < R; ++r) out[r] = fma(rd[i][(r >> i) & 1], own[r ^ (1 << i)], out[r]);
#pragma unroll
      for (int a = 0; a < kRegBits; ++a)
#pragma unroll
        for (int b = a + 1; b < kRegBits; ++b)
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (((r >> a) ^ (r >> b)) & 1) continue;  // compile-time
            out[r] = fma(rg[rr_index(a, b)], own[r ^ ((1 << a) | (1 << b))], out[r]);
          }
    }
    // fused iteration j with NQ thread pairs (compile-time: NPI for j < ja, NPI - 1 after)
    // BJ = -1: j is a lane bit; 0 / 1: a wave bit (j >= 6) of that value, so the sweep's pairs
    // (j, register bit i) touch only the rows r_i == BJ (half its pair FMAs skipped at compile time)
    auto iteration = [&](const int j, auto nq_tag, auto bj_tag) {
      constexpr int NQ = decltype(nq_tag)::value;
      constexpr int BJ = decltype(bj_tag)::value;
      const int bj = BJ >= 0 ? BJ : (tid >> j) & 1;
      const DPair* qs = S.tt + j * NPI;
      // the iteration's pair masks and coefficients, wave-uniform: scalar registers
      int pm[NQ];
      double pg[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        pm[q] = __builtin_amdgcn_readfirstlane((int)qs[q].mask_lo);
        const long long gb = __double_as_longlong(qs[q].g);
        pg[q] = __longlong_as_double(((long long)__builtin_amdgcn_readfirstlane((int)(gb >> 32)) << 32) |
                                     (unsigned)__builtin_amdgcn_readfirstlane((int)gb));
      }
      // load units of 8 rows: 0, 1 the sweep's halves (partner t ^ e_j), 2 + 2q + h half h of thread
      // pair q; two buffers, unit u + 1 loaded before the FMAs of unit u
      constexpr int NU = 2 + 2 * NQ, NH = R / 2;
      auto unit_load = [&](int u, double* v) {
        const int t = u < 2 ? (tid ^ (1 << j)) : (tid ^ pm[(u - 2) >> 1]);
        const int h = u < 2 ? u : ((u - 2) & 1);
        ldrows<NT, NH>(A, t, h * NH, v);
      };
      const double cd = bj ? S.sw[j][1] : S.sw[j][0];
      double ba[NH], bb[NH];
      unit_load(0, ba);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        double* cur = (u & 1) ? bb : ba;
        if (u + 1 < NU) unit_load(u + 1, (u & 1) ? ba : bb);
        if (u < 2) {
          // sweep half hh = u: drive of j; pairs (j, register bit i < 3) inside the half; (j, register
          // bit 3) from this half's rows into the other half's (rows with r_i == x_j)
          const int hh = u;
          double* oh = out + hh * NH;
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) oh[rr] = fma(cd, cur[rr], oh[rr]);
#pragma unroll
          for (int i = 0; i < 3; ++i) {
            const double g = S.sw[j][2 + i];
            const double g0 = bj ? 0.0 : g, g1 = bj ? g : 0.0;
#pragma unroll
            for (int rr = 0; rr < NH; ++rr) {
              if (BJ >= 0 && (int)((rr >> i) & 1) != BJ) continue;
              oh[rr] = fma((rr >> i) & 1 ? g1 : g0, cur[rr ^ (1 << i)], oh[rr]);
            }
          }
          if (BJ < 0 || 1 - hh == BJ) {
            const double g = S.sw[j][5];
            const double g3 = ((1 - hh) == bj) ? g : 0.0;  // output rows r_3 = 1 - hh
            double* oo = out + (1 - hh) * NH;
#pragma unroll
            for (int rr = 0; rr < NH; ++rr) oo[rr] = fma(g3, cur[rr], oo[rr]);
          }
        } else {
          // thread pair q, half h (partner t ^ m on the rows with x_i == x_j: coefficient zero in the
          // other lanes, one branch-free block)
          const int q = (u - 2) >> 1, h = (u - 2) & 1;
          const double g = par32((uint32_t)(tid & pm[q])) ? 0.0 : pg[q];
          double* oh = out + h * NH;
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) oh[rr] = fma(g, cur[rr], oh[rr]);
        }
        // keep the next unit's loads behind this point: at most two units' rows in registers (the
        // scheduler would otherwise hoist every load of the iteration and spill)
        asm volatile("" ::: "memory");
      }
    };
    using LANE = std::integral_constant<int, -1>;
    using W0 = std::integral_constant<int, 0>;
    using W1 = std::integral_constant<int, 1>;
    using QA = std::integral_constant<int, NPI>;
    using QB = std::integral_constant<int, NPI - 1>;
    constexpr int JW = TB < 6 ? TB : 6;  // thread bits 6.. index the wave
#pragma unroll 1
    for (int j = 0; j < min(ja, JW); ++j) iteration(j, QA{}, LANE{});
#pragma unroll 1
    for (int j = ja; j < JW; ++j) iteration(j, QB{}, LANE{});
#pragma unroll 1
    for (int j = JW; j < TB; ++j) {
      const bool wb = __builtin_amdgcn_readfirstlane((tid >> j) & 1);
      if (j < ja) {
        if (wb) iteration(j, QA{}, W1{}); else iteration(j, QA{}, W0{});
      } else {
        if (wb) iteration(j, QB{}, W1{}); else iteration(j, QB{}, W0{});
      }
    }
    // recurrence (w_{k-2} from B, own rows) and the two sums (k odd: the sine part); w_k -> B
    const double ck = cf[k];
    {
      double pr[R];
      ld16<NT>(B, tid, pr);
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = (k == 1) ? s1 * out[r] : fma(2.0 * s1, out[r], -pr[r]);
#pragma unroll
      for (int p = 0; p < R / 2; ++p) {
        dv2 d;
        d.x = out[2 * p];
        d.y = out[2 * p + 1];
        *(lv2*)(B + 2 * (p * NT + tid)) = d;
      }
    }
    if (k & 1) {
#pragma unroll
      for (int r = 0; r < R; ++r) as[r] = fma(ck, out[r], as[r]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) ac[r] = fma(ck, out[r], ac[r]);
    }
    __syncthreads();  // w_k complete in B; every read of A done (A takes w_{k+1} next term)
  }
  // U_xc = e^{-i beta dt} i^{|c| - |x|} (A - i S)   (rot; without the i power for real drives), into
  // the tiles on and above the diagonal (symv_tile_index), column c1 also whole into psi1
  constexpr int BS = kSymvBlock, NB = T / BS;
  const int J = (int)c / BS, jj = (int)c % BS;
  const int pc = __popc(c);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint32_t x = (uint32_t)(r * NT + tid);
    double vr = phr * ac[r] + phi * as[r], vi = phi * ac[r] - phr * as[r];
    if (rot) {
      switch ((pc - __popc(x)) & 3) {
        case 1: { const double t = vr; vr = -vi; vi = t; break; }
        case 2: vr = -vr, vi = -vi; break;
        case 3: { const double t = vr; vr = vi; vi = -t; break; }
        default: break;
      }
    }
    const int I = (int)x / BS;
    if (I <= J) U[(symv_tile_index(I, J, NB) * BS + jj) * (size_t)BS + x % BS] = make_double2(vr, vi);
    if ((int)c == c1) psi1[x] = make_double2(vr, vi);
  }
}

// One BS x BS tile (I, J), I <= J, of U in tile storage (symv_tile_index; column-major inside a
// tile, the tiles in the row-major order of the upper triangle, blockIdx.x = the tile); 256 threads:
// wave w takes columns w * BS / 4 .. of the tile, lane l rows l + 64 q (q < BS / 64), in chunks of
// 8 columns.  Below the diagonal (I < J) the same elements give s (U_IJ^T (s x_I)) for row block J:
// each lane's 8 column partials are summed over the wave by a butterfly reduce-scatter (xor 32, 16,
// 8 halve the set, xor 4, 2, 1 finish it: 10 complex exchanges per chunk instead of 48).  Small
// tiles (BS = 64: 2080 of 64 KiB at N = 12) spread the matrix evenly over the CUs (with 128 x 128
// tiles 528 of 256 KiB left 16 CUs three tiles: the product took as long as those).
//
// FUSED: the reduction as well -- every workgroup counts itself in the agent-scope counters of its
// two row blocks after an agent release (MI355X_MICROARCH.md, valid forms: plain stores, vmcnt(0)
// per wave, barrier, lane-0 release, counter), and the workgroup whose add completes a block's count
// (nb contributions) acquires and sums that block's partials in the fixed k order of k_symv_reduce,
// then resets the counter for the next product: one launch per product instead of two.
template <bool FUSED>
__global__ void __launch_bounds__(256)
k_symv(const double2* __restrict__ U, int dim, const double2* __restrict__ x, double2* __restrict__ partial,
       int parity, int* __restrict__ cnt, double2* __restrict__ y) {
  constexpr int BS = kSymvBlock, RL = BS / 64, CW = BS / 4;
  const int nb = dim / BS;
  // blockIdx.x -> (I, J) with I <= J, row-major over the upper triangle
  int I = 0, rem = (int)blockIdx.x;
  while (rem >= nb - I) rem -= nb - I, ++I;
  const int J = I + rem;
  __shared__ double2 xs[2][BS];   // x_J, s * x_I
  __shared__ double2 red[4][BS];  // per-wave direct partials
  __shared__ double2 tr[4][CW];   // per-wave transposed sums of the wave's columns
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < BS) {
    xs[0][tid] = x[J * BS + tid];
    const int r = I * BS + tid;
    const double2 v = x[r];
    const double s = (parity && (__popc(r) & 1)) ? -1.0 : 1.0;
    xs[1][tid] = make_double2(s * v.x, s * v.y);
  }
  __syncthreads();
  const bool off = I < J;
  // the wave's columns: CW * BS * 16 B contiguous
  const double2* col0 = U + ((size_t)blockIdx.x * BS + w * CW) * BS;
  double2 a[RL], sx[RL];
#pragma unroll
  for (int q = 0; q < RL; ++q) {
    a[q] = make_double2(0.0, 0.0);
    sx[q] = xs[1][lane + 64 * q];
  }
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1, b3 = (lane >> 3) & 1;
#pragma unroll 1
  for (int c0 = 0; c0 < CW; c0 += 8) {
    double2 u[8][RL];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int q = 0; q < RL; ++q) u[c][q] = col0[(size_t)(c0 + c) * BS + lane + 64 * q];
    double px[8], py[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const double2 xj = xs[0][w * CW + c0 + c];
      double tx = 0.0, ty = 0.0;
#pragma unroll
      for (int q = 0; q < RL; ++q) {
        a[q].x = fma(u[c][q].x, xj.x, fma(-u[c][q].y, xj.y, a[q].x));
        a[q].y = fma(u[c][q].x, xj.y, fma(u[c][q].y, xj.x, a[q].y));
        tx = fma(u[c][q].x, sx[q].x, fma(-u[c][q].y, sx[q].y, tx));
        ty = fma(u[c][q].x, sx[q].y, fma(u[c][q].y, sx[q].x, ty));
      }
      px[c] = tx;
      py[c] = ty;
    }
    if (off) {
      // xor 32: keep columns 4 b5 .. 4 b5 + 3
      double kx[4], ky[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double sxv = b5 ? px[i] : px[4 + i], syv = b5 ? py[i] : py[4 + i];
        kx[i] = (b5 ? px[4 + i] : px[i]) + __shfl_xor(sxv, 32, 64);
        ky[i] = (b5 ? py[4 + i] : py[i]) + __shfl_xor(syv, 32, 64);
      }
      // xor 16: keep 2 of them
      double mx[2], my[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const double sxv = b4 ? kx[i] : kx[2 + i], syv = b4 ? ky[i] : ky[2 + i];
        mx[i] = (b4 ? kx[2 + i] : kx[i]) + __shfl_xor(sxv, 16, 64);
        my[i] = (b4 ? ky[2 + i] : ky[i]) + __shfl_xor(syv, 16, 64);
      }
      // xor 8: keep 1, then the full sum over xor 4, 2, 1
      double vx = (b3 ? mx[1] : mx[0]) + __shfl_xor(b3 ? mx[0] : mx[1], 8, 64);
      double vy = (b3 ? my[1] : my[0]) + __shfl_xor(b3 ? my[0] : my[1], 8, 64);
#pragma unroll
      for (int o = 4; o > 0; o >>= 1) {
        vx += __shfl_xor(vx, o, 64);
        vy += __shfl_xor(vy, o, 64);
      }
      if ((lane & 7) == 0) tr[w][c0 + 4 * b5 + 2 * b4 + b3] = make_double2(vx, vy);
    }
  }
#pragma unroll
  for (int q = 0; q < RL; ++q) red[w][lane + 64 * q] = a[q];
  __syncthreads();
  // direct partial of row block I from this tile (contributor k = J), fixed wave order
  if (tid < BS) {
    double2 s = red[0][tid];
#pragma unroll
    for (int q = 1; q < 4; ++q) s.x += red[q][tid].x, s.y += red[q][tid].y;
    partial[((size_t)I * nb + J) * BS + tid] = s;
  }
  // transposed partial of row block J (contributor k = I): s_c * sum, column c = w * CW + lane
  if (off && lane < CW) {
    const int c = w * CW + lane;
    const double sc = (parity && (__popc(J * BS + c) & 1)) ? -1.0 : 1.0;
    const double2 t = tr[w][lane];
    partial[((size_t)J * nb + I) * BS + c] = make_double2(sc * t.x, sc * t.y);
  }
  if constexpr (FUSED) {
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int last = 0;
      if (__hip_atomic_fetch_add(cnt + I, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) last |= 1;
      if (off && __hip_atomic_fetch_add(cnt + J, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) last |= 2;
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      s_last = last;
    }
    __syncthreads();
    const int last = s_last;
    for (int which = 0; which < 2; ++which) {
      if (!((last >> which) & 1)) continue;
      const int B = which ? J : I;
      // 256 threads: row tid % 64 of block B, quarter tid / 64 of the k range, then the quarters
      const int rr = tid & 63, part = tid >> 6;
      double2 a = make_double2(0.0, 0.0);
      if (rr < BS) {
        const int k0 = part * nb / 4, k1 = (part + 1) * nb / 4;
        for (int k = k0; k < k1; ++k) {
          const double2 v = partial[((size_t)B * nb + k) * BS + rr];
          a.x += v.x;
          a.y += v.y;
        }
      }
      red[part][rr] = a;
      __syncthreads();
      if (part == 0 && rr < BS) {
#pragma unroll
        for (int q = 1; q < 4; ++q) a.x += red[q][rr].x, a.y += red[q][rr].y;
        y[B * BS + rr] = a;
      }
      if (tid == 0) cnt[B] = 0;  // the next product is the next launch (stream order)
      __syncthreads();
    }
  }
}

// y[r] = sum_k partial[r / BS][k][r % BS] in fixed k order: a workgroup of 256 threads takes 16
// rows; thread (row tid % 16, part tid / 16) sums nb / 16 consecutive k, then the parts in order
// (256 workgroups: the chain's per-product reduction is latency-, not bandwidth-bound)
__global__ void __launch_bounds__(256)
k_symv_reduce(const double2* __restrict__ partial, int dim, double2* __restrict__ y) {
  constexpr int BS = kSymvBlock, RW = 16, NP = 256 / RW;
  __shared__ double2 q[NP][RW];
  const int nb = dim / BS;
  const int tid = threadIdx.x, rl = tid % RW, part = tid / RW;
  const int r = blockIdx.x * RW + rl;
  double2 s = make_double2(0.0, 0.0);
  if (r < dim) {
    const int B = r / BS, rr = r % BS;
    const int k0 = part * nb / NP, k1 = (part + 1) * nb / NP;
    for (int k = k0; k < k1; ++k) {
      const double2 v = partial[((size_t)B * nb + k) * BS + rr];
      s.x += v.x;
      s.y += v.y;
    }
  }
  q[part][rl] = s;
  __syncthreads();
  if (part == 0 && r < dim) {
#pragma unroll
    for (int p = 1; p < NP; ++p) s.x += q[p][rl].x, s.y += q[p][rl].y;
    y[r] = s;
  }
}

}  // namespace

bool ucols_supported(int L) { return L >= kRegBlockMinTile && L <= kMaxTile; }

hipError_t launch_ucols(int L, const DevProb* probs, const double* cf, int deg, int rot, double phr, double phi,
                        double2* U, int n_cols, int col0, int c1, double2* psi1, hipStream_t st) {
  if (n_cols <= 0) return hipSuccess;
  switch (L) {
#define X(l)                                                                                      \
  case l:                                                                                         \
    hipLaunchKernelGGL(k_ucols<l>, dim3(n_cols), dim3(RB<l>::NT), 0, st, probs, cf, deg, rot, phr, \
                       phi, U, col0, c1, psi1);                                                   \
    return hipGetLastError();
    X(10) X(11) X(12) X(13)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_symv(const double2* U, int dim, const double2* x, double2* partial, int parity,
                       hipStream_t st, int* cnt, double2* y) {
  const int nb = dim / kSymvBlock;
  if (cnt)
    hipLaunchKernelGGL(k_symv<true>, dim3(nb * (nb + 1) / 2), dim3(256), 0, st, U, dim, x, partial, parity, cnt, y);
  else
    hipLaunchKernelGGL(k_symv<false>, dim3(nb * (nb + 1) / 2), dim3(256), 0, st, U, dim, x, partial, parity,
                       cnt, y);
  return hipGetLastError();
}

hipError_t launch_symv_reduce(const double2* partial, int dim, double2* y, hipStream_t st) {
  hipLaunchKernelGGL(k_symv_reduce, dim3((dim + 15) / 16), dim3(256), 0, st, partial, dim, y);
  return hipGetLastError();
}

}  // namespace dse
