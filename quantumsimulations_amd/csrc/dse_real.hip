// dse_real.hip -- the real-component Chebyshev interval kernel (gfx950): one workgroup per real
// component of a whole register, no cross-workgroup traffic inside a launch.
//
// The sweep's drives are purely imaginary (phase pi/2, sweep_sea_detuning.py:1227-1228), so in
// the rotated frame D|x> = i^popcount(x) |x> the Hamiltonian H' = D H D^dagger is REAL symmetric
// (a drive flip changes popcount by 1: i * (i a) is real; a double-quantum pair flip by 2:
// i^2 g = -g; the diagonal is untouched -- dse_dense.h).  T_k(H~') therefore maps real vectors to
// real vectors, and the rotated state phi = a + i b (phi(0) = e_x0, the phase i^|x0| of D psi0
// factored out) propagates over an interval as
//     phi(t + tau) = acc_a + i acc_b,   acc_c = sum_k c_k T_k(H~') c      (c = a, b)
// with the complex Chebyshev coefficients c_k of dse_interval.hip.  The two recurrences are
// independent: one workgroup runs each, and a real vector of 2^14 amplitudes is 128 KiB, so the
// WHOLE N = 14 register sits in one CU's LDS.  k_interval splits such a register into two 2^13
// complex tiles that exchange 128 KiB through the fabric every term (sc1 hand-off: 27.8 us per
// term against 19.1 for one tile); here the per-thread work of a term is the same (32 real rows
// instead of 16 complex ones: the same bytes, the same FMAs) and nothing crosses workgroups.
//
// Thread t of 512 owns the rows x = r * 512 + t, r < R = 2^(n - 9); in LDS rows 2p and 2p + 1 of
// a thread sit side by side (one ds_read_b128 per row pair).  Register bit 0 is the row pair's
// component, the top register bit splits the rows into halves (partner reads in halves, as
// k_interval's register bit 3).  One H application: phase 1 (diagonal, drives and pairs among
// register bits), then per thread bit j the sweep (partner t ^ e_j: drive of j, pairs (j, register
// bit)) fused with the iteration's four thread-bit pairs (canonical schedule), software-pipelined;
// phase 5: w_k = 2 (H' - beta) w_{k-1} / alpha - w_{k-2}, complex propagator sums of the launch's
// outputs every third term (acc += c0 w_{k-2} + c1 w_{k-1} + c2 w_k, complex c times real w).
//
// k_real_combine then forms psi = i^{|x0| - |x|} (acc_a + i acc_b) of every output in the
// computational frame (the buffers k_obs reads, dse_get_state's final state) and the next
// interval's [a | b].
#include <type_traits>

#include "dse_device.h"

namespace dse {

namespace {

typedef __attribute__((address_space(3))) const dv2 ldv2;
typedef __attribute__((address_space(3))) dv2 sdv2;

constexpr int kRealNT = 512;
constexpr int kRealTB = 9;

template <typename T>
__device__ __forceinline__ uint32_t lds_u32(const T* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) T*)p;
}

// The canonical thread-pair schedule (as dse_span.hip span_pair_mask): pair p = (a, b), a < b < 9,
// lexicographic, iteration p / 4, slot p % 4 (36 pairs, 4 per iteration)
__host__ __device__ constexpr uint32_t real_pair_mask(int j, int q) {
  int p = j * 4 + q;
  int a = 0;
  while (p >= kRealTB - 1 - a) {
    p -= kRealTB - 1 - a;
    ++a;
  }
  return (1u << a) | (1u << (a + 1 + p));
}

struct RealShared {
  dv2 w[16 * kRealNT];   // the register's w_{k-1} (2^14 doubles as row pairs)
  dv2 td[3][kRealNT];    // per-thread diagonal: (zt, hr0) (hr1, hr2) (hr3, hr4)
  double zr[32];         // register-bit ZZ part of the diagonal per row
  double cf[16];         // field per bit (scratch for the diagonal)
  double zz[14 * 14];
  dv2 it[kRealTB][6];    // coefficient rows (RealTab::it)
};

// rows 2 (hh * HRP + pp) + {0, 1}, pp < NP, of thread tp (one ds_read_b128 per row pair); the second
// half starts past ds_read's 16-bit offset at n = 14: an opaque base, not per-row adds
template <int HRP, int NP>
__device__ __forceinline__ void rd_pairs(uint32_t wbase, int tp, int hh, int pp0, double* v) {
  uint32_t a = wbase + (uint32_t)tp * 16u;
  constexpr uint32_t HALF = (uint32_t)HRP * kRealNT * 16u;
  if (hh) {
    if (HALF >= 65536u)
      asm("v_add_u32_e32 %0, %1, %2" : "=v"(a) : "i"(HALF), "v"(a));
    else
      a += HALF;
  }
#pragma unroll
  for (int pp = 0; pp < NP; ++pp) {
    const dv2 d = *(ldv2*)(size_t)(a + (uint32_t)(pp0 + pp) * kRealNT * 16u);
    v[2 * pp] = d.x;
    v[2 * pp + 1] = d.y;
  }
}

// diagnostics builds only (-DDSE_DIAG; option real_ablate, separate instantiations; results become
// wrong): 1 phase 1, 2 the sweeps' FMAs, 4 the thread pairs, 8 the propagator sums' global loads and
// stores, 16 the w_k stores
#ifdef DSE_DIAG
int g_real_ablate = 0;
#endif

template <int L, int ABL>
__device__ __forceinline__ void real_body(RealShared& S, const DevProb& P, int comp, int set, int n_out) {
  constexpr int NT = kRealNT, TB = kRealTB, RB = L - TB, R = 1 << RB, RP = R / 2, HRP = RP / 2;
  constexpr int RH = R / 2;  // rows per half
  constexpr int AB = R >= 32 ? 2 : 4;  // rows per propagator-sum block
  static_assert(RB >= 4 && RB <= kRealRB, "register bits");
  const int tid = threadIdx.x;
  const int K = P.degree;
  const double s1 = P.s1;
  const size_t nn = size_t(1) << L;
  const RealTab* tab = P.rtab;
  const cptr<RealTab> ctab = cst(tab);
  const double* crow = (const double*)coef_row(P, set, 0);
  const size_t rstride = 2 * (size_t)(P.kcap1 + 1);
  int dj[kMaxOut];
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) dj[j] = j < n_out ? (int)crow[j * rstride] : 0;

  // ---- setup: coefficient rows, the component -> LDS, per-thread diagonal ----
  {
    const gd2* src = (const gd2*)tab->it;
    for (int e = tid; e < TB * 6; e += NT) (&S.it[0][0])[e] = src[e];
    const gdbl* zz = gptr(P.zz);
    for (int e = tid; e < L * L; e += NT) S.zz[e] = zz[e];
    if (tid < L) S.cf[tid] = P.field[tid];
    const gdbl* in = gptr(P.rin + (size_t)comp * nn);
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      dv2 d;
      d.x = in[(size_t)(2 * p) * NT + tid];
      d.y = in[(size_t)(2 * p + 1) * NT + tid];
      S.w[p * NT + tid] = d;
    }
  }
  __syncthreads();
  if (tid < R) {
    double v = 0.0;
    for (int a = 0; a < RB; ++a)
      for (int b = a + 1; b < RB; ++b)
        v += S.zz[(TB + a) * L + TB + b] * ((0.5 - ((tid >> a) & 1)) * (0.5 - ((tid >> b) & 1)));
    S.zr[tid] = v;
  }
  {
    // D(x) = shift - beta + sum_i field_i s_i + sum_{i<j} zz_ij s_i s_j, x = r * 512 + t:
    // zt(t) + sum_i hr_i(t) s_i(r) + zr(r)
    double zt = P.shift - P.beta;
    double hr[kRealRB];
#pragma unroll
    for (int i = 0; i < kRealRB; ++i) hr[i] = i < RB ? S.cf[TB + i] : 0.0;
#pragma unroll 1
    for (int j = 0; j < TB; ++j) {
      const double sj = 0.5 - (double)((tid >> j) & 1);
      double a = S.cf[j];
#pragma unroll 1
      for (int i = j + 1; i < TB; ++i) a += S.zz[j * L + i] * (0.5 - (double)((tid >> i) & 1));
      zt += a * sj;
#pragma unroll
      for (int i = 0; i < RB; ++i) hr[i] += S.zz[j * L + TB + i] * sj;
    }
    dv2 v;
    v.x = zt, v.y = hr[0];
    S.td[0][tid] = v;
    v.x = hr[1], v.y = hr[2];
    S.td[1][tid] = v;
    v.x = hr[3], v.y = hr[4];
    S.td[2][tid] = v;
  }
  __syncthreads();

  double prev[R];
#pragma unroll
  for (int r = 0; r < R; ++r) prev[r] = 0.0;
  const uint32_t wb = lds_u32(&S.w[0]);
  const int rfm = ctab->rflip_mask;
  constexpr int ab = ABL;

  for (int k = 1; k <= K; ++k) {
    // ---- phase 1: diagonal, drives and pairs among register bits (own rows), one half of the
    // rows in registers at a time: the top register bit's terms take the other half's rows ----
    double out[R];
    {
      const dv2 t01 = S.td[0][tid], t23 = S.td[1][tid], t45 = S.td[2][tid];
      const double tdv[1 + kRealRB] = {t01.x, t01.y, t23.x, t23.y, t45.x, t45.y};
      constexpr int TOP = RB - 1;
      // half hh: diagonal and the terms among the other register bits
      auto own_half = [&](int hh) {
        double own[RH];
        rd_pairs<HRP, HRP>(wb, tid, hh, 0, own);
        double* oh = out + hh * RH;
#pragma unroll
        for (int rr = 0; rr < RH; ++rr) {
          const int r = hh * RH + rr;
          double d = tdv[0] + S.zr[r];
#pragma unroll
          for (int i = 0; i < RB; ++i) d += ((r >> i) & 1 ? -0.5 : 0.5) * tdv[1 + i];
          oh[rr] = d * own[rr];
        }
#pragma unroll
        for (int i = 0; i < TOP; ++i) {
          if (!((rfm >> i) & 1)) continue;
          const double c0 = ctab->rflip[i][0], c1 = ctab->rflip[i][1];
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) oh[rr] = fma((rr >> i) & 1 ? c1 : c0, own[rr ^ (1 << i)], oh[rr]);
        }
#pragma unroll
        for (int a = 0; a < TOP; ++a)
#pragma unroll
          for (int b = a + 1; b < TOP; ++b) {
            const double g = ctab->rr_g[real_rr_index(a, b)];
#pragma unroll
            for (int rr = 0; rr < RH; ++rr) {
              if (((rr >> a) ^ (rr >> b)) & 1) continue;
              oh[rr] = fma(g, own[rr ^ ((1 << a) | (1 << b))], oh[rr]);
            }
          }
      };
      // the top bit's terms into half hh from the other half's rows (output top value hh)
      auto cross_half = [&](int hh) {
        double oth[RH];
        rd_pairs<HRP, HRP>(wb, tid, 1 - hh, 0, oth);
        double* oh = out + hh * RH;
        if ((rfm >> TOP) & 1) {
          const double c = ctab->rflip[TOP][hh];
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) oh[rr] = fma(c, oth[rr], oh[rr]);
        }
#pragma unroll
        for (int a = 0; a < TOP; ++a) {  // pair (a, top): rows with r_a == r_top = hh
          const double g = ctab->rr_g[real_rr_index(a, TOP)];
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) {
            if (((rr >> a) & 1) != hh) continue;
            oh[rr] = fma(g, oth[rr ^ (1 << a)], oh[rr]);
          }
        }
      };
      if constexpr (!(ab & 1)) {
        own_half(0);
        own_half(1);
        cross_half(0);
        cross_half(1);
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) out[r] = 0.0;
      }
    }
    __syncthreads();  // (first term: the setup's stores; later: w_{k-1} complete in LDS)

    // ---- fused loop: sweep of thread bit j + its four thread pairs, software-pipelined: the
    // sweep's rows in halves, the pairs' rows in quarters, each next read issued before the FMAs
    // of the current one ----
    const uint32_t itb = lds_u32(&S.it[0][0]);
#pragma unroll 1
    for (int j = 0; j < TB; ++j) {
      const int pt = tid ^ (1 << j);
      double pv[RH];
      rd_pairs<HRP, HRP>(wb, pt, 0, 0, pv);
      uint32_t ia;
      asm("v_mov_b32_e32 %0, %1" : "=v"(ia) : "s"(itb + (uint32_t)j * 6u * 16u));
      const dv2 dc = *(ldv2*)(size_t)ia;              // rotated drive by output value
      const dv2 g01 = *(ldv2*)(size_t)(ia + 16u);     // pairs (j, register bit 0 .. 5)
      const dv2 g23 = *(ldv2*)(size_t)(ia + 32u);
      const dv2 g45 = *(ldv2*)(size_t)(ia + 48u);
      const dv2 gp01 = *(ldv2*)(size_t)(ia + 64u);    // the four thread pairs
      const dv2 gp23 = *(ldv2*)(size_t)(ia + 80u);
      const int bj = (tid >> j) & 1;
      const double c = bj ? dc.y : dc.x;
      // pair (j, register bit i) acts on the rows with r_i == t_j: coefficient g_i there, 0 elsewhere
      auto gsel = [&](int i, int bit) {
        const double g = i == 0 ? g01.x : i == 1 ? g01.y : i == 2 ? g23.x : i == 3 ? g23.y : g45.x;
        return bit == bj ? g : 0.0;
      };
      int tpt[4];
      double ge[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const uint32_t m = real_pair_mask(j, qq);
        tpt[qq] = tid ^ (int)m;
        const double g = qq == 0 ? gp01.x : qq == 1 ? gp01.y : qq == 2 ? gp23.x : gp23.y;
        ge[qq] = par32((uint32_t)tid & m) ? 0.0 : g;  // rows with x_a == x_b
      }
      // sweep of half hh (rows with top register bit = hh) from its partner rows
      auto sweep = [&](int hh, const double* pvh) {
        double* oh = out + hh * RH;
#pragma unroll
        for (int rr = 0; rr < RH; ++rr) oh[rr] = fma(c, pvh[rr], oh[rr]);
#pragma unroll
        for (int i = 0; i < RB - 1; ++i)
#pragma unroll
          for (int rr = 0; rr < RH; ++rr) oh[rr] = fma(gsel(i, (rr >> i) & 1), pvh[rr ^ (1 << i)], oh[rr]);
        // (j, top register bit): rows of the other half, r_top = 1 - hh
        double* oo = out + (1 - hh) * RH;
        const double gt = gsel(RB - 1, 1 - hh);
#pragma unroll
        for (int rr = 0; rr < RH; ++rr) oo[rr] = fma(gt, pvh[rr], oo[rr]);
      };
      constexpr int QP = HRP / 2;  // row pairs per quarter
      double qa[2 * QP], qb[2 * QP];
      if constexpr ((ab & 6) != 0) {  // ablation variants (diagnostics)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          if (hh) rd_pairs<HRP, HRP>(wb, pt, 1, 0, pv);
          if (!(ab & 2)) sweep(hh, pv);
          if (!(ab & 4))
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
              rd_pairs<HRP, HRP>(wb, tpt[qq], hh, 0, qa);
              double* oh = out + hh * RH;
#pragma unroll
              for (int rr = 0; rr < 2 * QP; ++rr) oh[rr] = fma(ge[qq], qa[rr], oh[rr]);
            }
        }
        continue;
      }
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        rd_pairs<HRP, QP>(wb, tpt[0], hh, 0, qa);
        sweep(hh, pv);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          rd_pairs<HRP, QP>(wb, tpt[qq], hh, QP, qb);
          {
            double* oh = out + hh * RH;
#pragma unroll
            for (int rr = 0; rr < 2 * QP; ++rr) oh[rr] = fma(ge[qq], qa[rr], oh[rr]);
          }
          if (qq < 3)
            rd_pairs<HRP, QP>(wb, tpt[qq + 1], hh, 0, qa);
          else if (hh == 0)
            rd_pairs<HRP, HRP>(wb, pt, 1, 0, pv);
          {
            double* oh = out + hh * RH + 2 * QP;
#pragma unroll
            for (int rr = 0; rr < 2 * QP; ++rr) oh[rr] = fma(ge[qq], qb[rr], oh[rr]);
          }
        }
      }
    }

    // ---- phase 5: recurrence, complex propagator sums (every third term), w_k -> LDS.  The sums'
    // global loads run D blocks ahead of their use (the compiler cannot hoist them above the
    // previous blocks' stores to the same arrays), so their latency is exposed once per update ----
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = k == 1 ? s1 * out[r] : fma(2.0 * s1, out[r], -prev[r]);
    static_assert(kMaxOut == 2, "phase 5 dispatch covers one or two outputs per launch");
    int um = 0;
    double2* accp[kMaxOut];
    CoefK cf[kMaxOut];  // a_{k-2}, a_{k-1}, a_k of each output (zero when it does not update)
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      // vector loads of the uniform rows (scalar loads of rows the host rewrites between launches
      // read stale scalar-cache lines, dse_interval.hip at crow)
      const int nt = j < n_out ? coef_nterm(k, dj[j]) : 0;
      const double* cc = crow + j * rstride + 2 * (size_t)(k - 1);  // a_{k-2}, a_{k-1}, a_k
      cf[j].upd = nt > 0;
      cf[j].c[0] = nt >= 3 ? make_double2(cc[0], cc[1]) : make_double2(0.0, 0.0);
      cf[j].c[1] = nt >= 2 ? make_double2(cc[2], cc[3]) : make_double2(0.0, 0.0);
      cf[j].c[2] = nt >= 1 ? make_double2(cc[4], cc[5]) : make_double2(0.0, 0.0);
      um |= cf[j].upd ? 1 << j : 0;
      accp[j] = P.racc + ((size_t)(2 * j + comp) << L);
    }
    // NO outputs of the launch; a term where some output updates loads and stores all NO sums
    // (an output past its degree has zero coefficients: its sums pass through unchanged)
    auto phase5 = [&](auto no_c) {
      constexpr int NO = decltype(no_c)::value;
      constexpr bool ACC = NO > 0 && !(ab & 8);
      constexpr int NB = R / AB, D = 1;
      const bool first = k == 1;
      double2 av[D][kMaxOut][AB];
      auto issue = [&](int b, int slot) {
#pragma unroll
        for (int j = 0; j < NO; ++j)
#pragma unroll
          for (int r = 0; r < AB; ++r) av[slot][j][r] = gld(gptr(accp[j]), (size_t)(b * AB + r) * NT + tid);
      };
      if constexpr (ACC) {
#pragma unroll
        for (int b = 0; b < D; ++b) issue(b, b);
      }
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        double ownb[AB];
#pragma unroll
        for (int r = 0; r < AB; r += 2) {
          const dv2 d = S.w[((b * AB + r) >> 1) * NT + tid];
          ownb[r] = d.x;
          ownb[r + 1] = d.y;
        }
        if constexpr (NO > 0) {
#pragma unroll
          for (int j = 0; j < NO; ++j)
#pragma unroll
            for (int r = 0; r < AB; ++r) {
              double2 a = make_double2(0.0, 0.0);
              if constexpr (ACC) {
                a = first ? make_double2(0.0, 0.0) : av[b % D][j][r];
                a.x = fma(cf[j].c[0].x, prev[b * AB + r], a.x);
                a.y = fma(cf[j].c[0].y, prev[b * AB + r], a.y);
              }
              a.x = fma(cf[j].c[1].x, ownb[r], a.x);
              a.y = fma(cf[j].c[1].y, ownb[r], a.y);
              a.x = fma(cf[j].c[2].x, out[b * AB + r], a.x);
              a.y = fma(cf[j].c[2].y, out[b * AB + r], a.y);
              if constexpr (ACC) gst(gptr(accp[j]), (size_t)(b * AB + r) * NT + tid, a);
            }
          if constexpr (ACC) {
            if (b + D < NB) issue(b + D, b % D);
          }
        }
#pragma unroll
        for (int r = 0; r < AB; ++r) prev[b * AB + r] = ownb[r];
      }
    };
    if (um == 0)
      phase5(std::integral_constant<int, 0>());
    else if (n_out >= 2)
      phase5(std::integral_constant<int, 2>());
    else
      phase5(std::integral_constant<int, 1>());
    __syncthreads();  // every read of w_{k-1} done
    if (!(ab & 16))
#pragma unroll
    for (int p = 0; p < RP; ++p) {
      dv2 d;
      d.x = out[2 * p];
      d.y = out[2 * p + 1];
      S.w[p * NT + tid] = d;
    }
  }
}

template <int ABL>
__global__ void __launch_bounds__(kRealNT)
k_real(const DevProb* __restrict__ probs, const int2* __restrict__ items, int set, int n_out) {
  __shared__ RealShared S;
  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  if (P.n == 14)
    real_body<14, ABL>(S, P, it.y, set, n_out);
  else
    real_body<13, ABL>(S, P, it.y, set, n_out);
}

// psi_j = i^{|x0| - |x|} (acc_a + i acc_b) of output j into the buffer k_obs reads (the last output:
// state role q ? 0 : 2; the others: intermediate output j); from the last output also [a | b].
// grid: (2^n / 256, outputs, problems of the list)
__global__ void __launch_bounds__(256)
k_real_combine(const DevProb* __restrict__ probs, const int2* __restrict__ items, int q, int n_out) {
  const DevProb& P = probs[items[blockIdx.z].x];
  const size_t nn = size_t(1) << P.n;
  const size_t x = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (x >= nn) return;
  const int j = blockIdx.y;
  const double2 aa = gld(gptr(P.racc), ((size_t)(2 * j) << P.n) + x);
  const double2 ab = gld(gptr(P.racc), ((size_t)(2 * j + 1) << P.n) + x);
  const double pr = aa.x - ab.y, pi = aa.y + ab.x;  // phi = acc_a + i acc_b
  const bool last = j == n_out - 1;
  if (last) {
    P.rin[x] = pr;
    P.rin[nn + x] = pi;
  }
  const uint32_t px = (uint32_t)__popcll((unsigned long long)x);
  const int e = ((int)P.rtab->x0pop - (int)px) & 3;
  double2 psi;
  psi.x = e == 0 ? pr : e == 1 ? -pi : e == 2 ? -pr : pi;
  psi.y = e == 0 ? pi : e == 1 ? pr : e == 2 ? -pi : -pr;
  double2* dst = last ? P.buf[q ? 0 : 2] : P.xacc + ((size_t)j << P.n);
  gst(gptr(dst), x, psi);
}

// [a | b] = [e_x0 | 0]
__global__ void __launch_bounds__(256)
k_real_init(const DevProb* __restrict__ probs, const int2* __restrict__ items) {
  const DevProb& P = probs[items[blockIdx.y].x];
  const size_t nn = size_t(1) << P.n;
  for (size_t x = (size_t)blockIdx.x * 256 + threadIdx.x; x < 2 * nn; x += (size_t)gridDim.x * 256)
    P.rin[x] = (x == (size_t)P.rtab->x0) ? 1.0 : 0.0;
}

}  // namespace

hipError_t set_real_ablate(int mask) {
  if (mask != 0 && mask != 1 && mask != 2 && mask != 4 && mask != 6 && mask != 8 && mask != 16)
    return hipErrorInvalidValue;
#ifdef DSE_DIAG
  g_real_ablate = mask;
  return hipSuccess;
#else
  return mask ? hipErrorNotSupported : hipSuccess;
#endif
}

hipError_t real_occupancy(int* blocks_per_cu) {
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_real<0>, kRealNT, 0);
}

hipError_t launch_real(const DevProb* probs, const int2* items, int n_items, int set, int n_out,
                       hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  const dim3 g(n_items), b(kRealNT);
#ifdef DSE_DIAG
  switch (g_real_ablate) {
    case 1: hipLaunchKernelGGL(k_real<1>, g, b, 0, st, probs, items, set, n_out); break;
    case 2: hipLaunchKernelGGL(k_real<2>, g, b, 0, st, probs, items, set, n_out); break;
    case 4: hipLaunchKernelGGL(k_real<4>, g, b, 0, st, probs, items, set, n_out); break;
    case 6: hipLaunchKernelGGL(k_real<6>, g, b, 0, st, probs, items, set, n_out); break;
    case 8: hipLaunchKernelGGL(k_real<8>, g, b, 0, st, probs, items, set, n_out); break;
    case 16: hipLaunchKernelGGL(k_real<16>, g, b, 0, st, probs, items, set, n_out); break;
    default: hipLaunchKernelGGL(k_real<0>, g, b, 0, st, probs, items, set, n_out);
  }
#else
  hipLaunchKernelGGL(k_real<0>, g, b, 0, st, probs, items, set, n_out);
#endif
  return hipGetLastError();
}

hipError_t launch_real_combine(const DevProb* probs, const int2* items, int n_items, int q, int n_out,
                               hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_real_combine, dim3((1u << 14) / 256, n_out, n_items), dim3(256), 0, st, probs, items, q,
                     n_out);
  return hipGetLastError();
}

hipError_t launch_real_init(const DevProb* probs, const int2* items, int n_items, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_real_init, dim3(32, n_items), dim3(256), 0, st, probs, items);
  return hipGetLastError();
}

}  // namespace dse
