// dse_kernels.hip -- gfx950 kernels of libdse (see dse_runtime.hip for the host side).
//
// The hot path of the reference is qt.sesolve (dipolar_ensemble_with_rare.py:653-666): every
// ODE right-hand side is a CSR product -1j H psi with H built at :453-588.  Here H is never
// stored: each kernel applies it matrix-free to 2^L-amplitude tiles staged in LDS.
//
//   k_step_rb<L, MODE>       register-block Chebyshev step (tiles of 2^9 .. 2^13 amplitudes):
//                            8 amplitudes per thread, fused recurrence + propagator accumulation
//   k_step_generic<L, MODE>  the same step for tiny tiles (L < 9)
//   k_obs<L>                 <Ix>, <Iy>, <Iz> sums (sea / rare) and ||psi||^2 per tile
//
// MODE_APPLY: out = H w (test hook)      MODE_FIRST: w1 = Ht w0,  acc = a0 w0 + a1 w1
// MODE_GEN:   w_k = 2 Ht w_{k-1} - w_{k-2} (in place over w_{k-2}),  acc += a_k w_k
// with Ht = (H - beta) / alpha.
#include "dse_internal.h"

namespace dse {

// Diagnostic ablation mask (0 in production): sections of k_step_rb to skip, for timing only.
//   1 thread-bit sweeps   2 thread-thread pairs   4 cross-tile terms   8 epilogue global reads
//   16 diagonal table read   32 tile load from global memory
__device__ int g_dse_ablate = 0;

hipError_t set_ablate(int mask) { return hipMemcpyToSymbol(HIP_SYMBOL(g_dse_ablate), &mask, sizeof(int)); }

namespace {

template <int L>
struct Geo {
  static constexpr int T = 1 << L;
  static constexpr int NT = (L >= 13) ? 512 : (T >= 256 ? 256 : 64);
  static constexpr int LGNT = (L >= 13) ? 9 : (T >= 256 ? 8 : 6);
  static constexpr int R = (T >= NT) ? T / NT : 1;
  static constexpr int TB = (L < LGNT) ? L : LGNT;  // tile bits carried by the thread index
};

__device__ __forceinline__ double2 cmad(double2 acc, double cr, double ci, double2 s) {
  acc.x = fma(cr, s.x, fma(-ci, s.y, acc.x));
  acc.y = fma(cr, s.y, fma(ci, s.x, acc.y));
  return acc;
}

__device__ __forceinline__ int par32(uint32_t v) { return __popc(v) & 1; }

// Global address-space views: loads through them are global_load (vmcnt only) instead of
// flat_load (which also counts against lgkmcnt and serialises LDS work).
typedef double __attribute__((ext_vector_type(2))) dv2;
typedef __attribute__((address_space(1))) dv2 gd2;
typedef __attribute__((address_space(1))) double gdbl;
__device__ __forceinline__ gd2* gptr(double2* p) { return (gd2*)p; }
__device__ __forceinline__ const gdbl* gptr(const double* p) { return (const gdbl*)p; }
__device__ __forceinline__ double2 gld(const gd2* p, size_t i) {
  const dv2 v = p[i];
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void gst(gd2* p, size_t i, double2 a) {
  dv2 v;
  v.x = a.x;
  v.y = a.y;
  p[i] = v;
}

// Cooperative copy of n16 16-byte granules from global memory into LDS.
__device__ __forceinline__ void stage16(void* dst, const void* src, int n16, int tid, int nt) {
  const gd2* s = (const gd2*)src;
  dv2* d = (dv2*)dst;
  for (int i = tid; i < n16; i += nt) d[i] = s[i];
}

// Recurrence + propagator accumulation for one amplitude (see CoefK):
//   MODE_APPLY  wdst = H w
//   MODE_FIRST  w1 = s1 * (H - beta) w0,  acc = c1 w0 + c2 w1
//   MODE_GEN    w_k = s2 * (H - beta) w_{k-1} - w_{k-2} (in place),  acc += c0 w_{k-2} + c1 w_{k-1} + c2 w_k
__device__ __forceinline__ double2 gld(const double2* p, size_t i) { return p[i]; }
__device__ __forceinline__ void gst(double2* p, size_t i, double2 a) { p[i] = a; }

template <int MODE, typename Ptr>
__device__ __forceinline__ void step_epilogue(size_t x, double2 out, double2 own, double scale,
                                              Ptr __restrict__ wdst, Ptr __restrict__ acc_b,
                                              const CoefK& C, int no_reads) {
  if (MODE == MODE_APPLY) {
    gst(wdst, x, out);
  } else if (MODE == MODE_FIRST) {
    double2 w;
    w.x = scale * out.x;
    w.y = scale * out.y;
    gst(wdst, x, w);
    double2 a = make_double2(0.0, 0.0);
    a = cmad(a, C.c[1].x, C.c[1].y, own);
    a = cmad(a, C.c[2].x, C.c[2].y, w);
    gst(acc_b, x, a);
  } else {
    const double2 prev = no_reads ? make_double2(0.0, 0.0) : gld(wdst, x);
    double2 w;
    w.x = fma(scale, out.x, -prev.x);
    w.y = fma(scale, out.y, -prev.y);
    gst(wdst, x, w);
    if (C.upd) {
      double2 a = no_reads ? make_double2(0.0, 0.0) : gld(acc_b, x);
      a = cmad(a, C.c[0].x, C.c[0].y, prev);
      a = cmad(a, C.c[1].x, C.c[1].y, own);
      a = cmad(a, C.c[2].x, C.c[2].y, w);
      gst(acc_b, x, a);
    }
  }
}

// Per-tile diagonal pieces: s_c[i] = F_i(h) for tile bits i < L, s_c[L] = C(h).
//   D(x) = zzlo[x_lo] + C(h) + sum_{i<L} F_i(h) s_i(x_lo)
//   F_i(h) = field_i + sum_{j>=L} zz_ij s_j(h)
//   C(h)   = shift - beta + sum_{j>=L} field_j s_j(h) + sum_{L<=i<j} zz_ij s_i(h) s_j(h)
template <int L>
__device__ __forceinline__ void tile_diag_coeffs(const DevProb& P, uint32_t h, double beta,
                                                 double* s_c, int tid) {
  const int n = P.n;
  if (tid < L) {
    double f = P.field[tid];
    for (int j = L; j < n; ++j) f += P.zz[tid * n + j] * (0.5 - (double)((h >> (j - L)) & 1u));
    s_c[tid] = f;
  } else if (tid == L) {
    double c = P.shift - beta;
    for (int j = L; j < n; ++j) {
      const double sj = 0.5 - (double)((h >> (j - L)) & 1u);
      c += P.field[j] * sj;
      for (int i = L; i < j; ++i) c += P.zz[i * n + j] * ((0.5 - (double)((h >> (i - L)) & 1u)) * sj);
    }
    s_c[L] = c;
  }
}

template <int L, int MODE>
__global__ void __launch_bounds__(Geo<L>::NT)
k_step_generic(const DevProb* __restrict__ probs, const int2* __restrict__ items, int k, int q, int set) {
  using G = Geo<L>;
  constexpr int T = G::T, NT = G::NT, R = G::R;
  __shared__ double2 s_w[T];
  __shared__ double s_c[L + 1];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const int tid = threadIdx.x;
  const bool live = (T >= NT) || (tid < T);
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform: this problem's interval is done

  // buffer roles (see host loop): psi = buf[q?2:0], acc = buf[q?0:2], scratch = buf[1]
  double2* psi_b = P.buf[q ? 2 : 0];
  double2* acc_b = P.buf[q ? 0 : 2];
  double2* scr_b = P.buf[1];
  const double2* win;
  double2* wdst;
  if (MODE == MODE_APPLY) {
    win = P.buf[0];
    wdst = P.buf[1];
  } else if (MODE == MODE_FIRST) {
    win = psi_b;
    wdst = scr_b;
  } else {
    win = ((k - 1) & 1) ? scr_b : psi_b;
    wdst = (k & 1) ? scr_b : psi_b;  // holds w_{k-2}; overwritten in place with w_k
  }
  const size_t base = (size_t)h << L;

  double2 own[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int x = r * NT + tid;
    if (live) {
      own[r] = win[base + x];
      s_w[x] = own[r];
    }
  }
  tile_diag_coeffs<L>(P, h, MODE == MODE_APPLY ? 0.0 : P.beta, s_c, tid);
  __syncthreads();
  if (!live) return;

  // ---- diagonal ----
  double gt = s_c[L];
#pragma unroll
  for (int i = 0; i < G::TB; ++i) gt += s_c[i] * (0.5 - (double)((tid >> i) & 1));
  double2 out[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int x = r * NT + tid;
    double d = P.zzlo[x] + gt;
#pragma unroll
    for (int i = G::TB; i < L; ++i) d += s_c[i] * (((r >> (i - G::TB)) & 1) ? -0.5 : 0.5);
    out[r].x = d * own[r].x;
    out[r].y = d * own[r].y;
  }

  // ---- drive flips inside the tile ----
  for (int f = 0; f < P.n_flips_lo; ++f) {
    const DFlip F = P.flips_lo[f];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t x = (uint32_t)(r * NT + tid);
      const bool v = (x & F.mask_lo) != 0u;
      const double2 s = s_w[x ^ F.mask_lo];
      out[r] = cmad(out[r], v ? F.re1 : F.re0, v ? F.im1 : F.im0, s);
    }
  }
  // ---- pair flips inside the tile ----
  for (int p = 0; p < P.n_pairs_lo; ++p) {
    const DPair Q = P.pairs_lo[p];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t x = (uint32_t)(r * NT + tid);
      if (!(__popc(x & Q.mask_lo) & 1)) {
        const double2 s = s_w[x ^ Q.mask_lo];
        out[r].x = fma(Q.g, s.x, out[r].x);
        out[r].y = fma(Q.g, s.y, out[r].y);
      }
    }
  }
  // ---- terms reaching other tiles (global, L2-served) ----
  for (int f = 0; f < P.n_flips_hi; ++f) {
    const DFlip F = P.flips_hi[f];
    const bool v = par32(h & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
    const double2* src = win + ((size_t)(h ^ F.tile_xor) << L);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t x = (uint32_t)(r * NT + tid);
      out[r] = cmad(out[r], cr, ci, src[x ^ F.mask_lo]);
    }
  }
  for (int p = 0; p < P.n_pairs_hi; ++p) {
    const DPair Q = P.pairs_hi[p];
    const int hp = par32(h & Q.tile_xor);
    const double2* src = win + ((size_t)(h ^ Q.tile_xor) << L);
    if (Q.mask_lo == 0u) {
      if (hp) continue;  // both bits above the tile: uniform condition
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const double2 s = src[r * NT + tid];
        out[r].x = fma(Q.g, s.x, out[r].x);
        out[r].y = fma(Q.g, s.y, out[r].y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t x = (uint32_t)(r * NT + tid);
        if (!((__popc(x & Q.mask_lo) + hp) & 1)) {
          const double2 s = src[x ^ Q.mask_lo];
          out[r].x = fma(Q.g, s.x, out[r].x);
          out[r].y = fma(Q.g, s.y, out[r].y);
        }
      }
    }
  }

  // ---- recurrence + accumulation ----
  CoefK C = {};
  if (MODE != MODE_APPLY) C = P.coef[set * P.kcap1 + (MODE == MODE_FIRST ? 1 : k)];
  const double scale = MODE == MODE_GEN ? 2.0 * P.s1 : P.s1;
#pragma unroll
  for (int r = 0; r < R; ++r)
    step_epilogue<MODE>(base + r * NT + tid, out[r], own[r], scale, wdst, acc_b, C, 0);
}

// Observables of one state: per tile partial sums of
//   0 Ix_sea, 1 Iy_sea, 2 Iz_sea, 3 Iz_R, 4 Ix_R, 5 Iy_R, 6 ||psi||^2
// <Ix_k> = sum_{bit_k(x)=0} Re(conj(psi_x) psi_{x^e_k}),  <Iy_k> = Im(...),  <Iz_k> = sum |psi_x|^2 s_k(x)
template <int L>
__global__ void __launch_bounds__(Geo<L>::NT)
k_obs(const DevProb* __restrict__ probs, const int2* __restrict__ items, int bsel,
      double* __restrict__ partial) {
  using G = Geo<L>;
  constexpr int T = G::T, NT = G::NT, R = G::R;
  __shared__ double2 s_w[T];
  __shared__ double s_red[NT / 64][8];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const int tid = threadIdx.x;
  const bool live = (T >= NT) || (tid < T);
  const double2* psi = P.buf[bsel];
  const size_t base = (size_t)h << L;

  double2 own[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    own[r] = make_double2(0.0, 0.0);
    if (live) {
      own[r] = psi[base + r * NT + tid];
      s_w[r * NT + tid] = own[r];
    }
  }
  __syncthreads();

  double acc[7] = {0, 0, 0, 0, 0, 0, 0};
  if (live) {
    const uint64_t hi = (uint64_t)h << L;
    const double half_sea = 0.5 * (double)P.n_sea;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t x = hi | (uint64_t)(r * NT + tid);
      const double p2 = own[r].x * own[r].x + own[r].y * own[r].y;
      acc[6] += p2;
      acc[2] += p2 * (half_sea - (double)__popcll(x & P.sea_mask));
      if (P.rare_bit >= 0) acc[3] += p2 * (0.5 - (double)((x >> P.rare_bit) & 1ull));
    }
    for (int b = 0; b < P.n; ++b) {
      const bool sea = (P.sea_mask >> b) & 1ull;
      const bool rr = (b == P.rare_bit);
      if (!sea && !rr) continue;
      double ore = 0.0, oim = 0.0;
      if (b < L) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t x = (uint32_t)(r * NT + tid);
          if (!((x >> b) & 1u)) {
            const double2 s = s_w[x ^ (1u << b)];
            ore += own[r].x * s.x + own[r].y * s.y;
            oim += own[r].x * s.y - own[r].y * s.x;
          }
        }
      } else {
        if ((h >> (b - L)) & 1u) continue;
        const double2* src = psi + ((size_t)(h ^ (1u << (b - L))) << L);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double2 s = src[r * NT + tid];
          ore += own[r].x * s.x + own[r].y * s.y;
          oim += own[r].x * s.y - own[r].y * s.x;
        }
      }
      if (sea) {
        acc[0] += ore;
        acc[1] += oim;
      }
      if (rr) {
        acc[4] += ore;
        acc[5] += oim;
      }
    }
  }
  // deterministic block reduction: wave butterfly, then waves in order
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    double v = acc[j];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    acc[j] = v;
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int j = 0; j < 7; ++j) s_red[tid >> 6][j] = acc[j];
  }
  __syncthreads();
  if (tid == 0) {
    double* o = partial + (size_t)blockIdx.x * 8;
#pragma unroll
    for (int j = 0; j < 7; ++j) {
      double v = 0.0;
      for (int w = 0; w < NT / 64; ++w) v += s_red[w][j];
      o[j] = v;
    }
    o[7] = 0.0;
  }
}


// ------------------------------------------------------------------------------------------
// register-block step kernel
// ------------------------------------------------------------------------------------------
template <int L>
struct RB {
  static constexpr int T = 1 << L;
  static constexpr int NT = T >> kRegBits;  // threads per workgroup
  static constexpr int TB = L - kRegBits;    // tile bits carried by the thread index
};

// Upper bounds of the cross-tile term lists for a 34-qubit register (static LDS staging).
template <int L>
struct HiCap {
  static constexpr int HB = DSE_MAX_HIGH_BITS(L);
  static constexpr int PAIRS = HB * L + HB * (HB - 1) / 2 + 1;
  static constexpr int FLIPS = HB + 1;
};

template <int L, int MODE>
__global__ void __launch_bounds__(RB<L>::NT)
k_step_rb(const DevProb* __restrict__ probs, const int2* __restrict__ items, int k, int q, int set) {
  constexpr int NT = RB<L>::NT, TB = RB<L>::TB;
  constexpr int NTT = TB * (TB - 1) / 2;
  __shared__ double2 s_w[RB<L>::T];
  __shared__ double s_c[L + 1];
  // per-problem term tables, staged once per workgroup (vector loads of generic pointers inside
  // the loops would serialise every iteration behind a global-memory round trip)
  __shared__ DSweep s_sw[TB];
  __shared__ DPair s_tt[NTT > 0 ? NTT : 1];
  __shared__ DPair s_ph[HiCap<L>::PAIRS];
  __shared__ DFlip s_fh[HiCap<L>::FLIPS];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const int tid = threadIdx.x;
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform: this problem's interval is done

  const int ab = g_dse_ablate;
  const int n_tt = P.n_pairs_tt, n_ph = P.n_pairs_hi, n_fh = P.n_flips_hi;
  gd2* psi_b = gptr(P.buf[q ? 2 : 0]);
  gd2* acc_b = gptr(P.buf[q ? 0 : 2]);
  gd2* scr_b = gptr(P.buf[1]);
  const gd2* win;
  gd2* wdst;
  if (MODE == MODE_APPLY) {
    win = gptr(P.buf[0]);
    wdst = gptr(P.buf[1]);
  } else if (MODE == MODE_FIRST) {
    win = psi_b;
    wdst = scr_b;
  } else {
    win = ((k - 1) & 1) ? scr_b : psi_b;
    wdst = (k & 1) ? scr_b : psi_b;
  }
  const size_t base = (size_t)h << L;

  stage16(s_sw, P.sweeps, TB * (int)(sizeof(DSweep) / 16), tid, NT);
  stage16(s_tt, P.pairs_tt, n_tt, tid, NT);
  stage16(s_ph, P.pairs_hi, n_ph, tid, NT);
  stage16(s_fh, P.flips_hi, n_fh * (int)(sizeof(DFlip) / 16), tid, NT);
#pragma unroll
  for (int r = 0; r < 8; ++r)
    s_w[r * NT + tid] = (ab & 32) ? make_double2(1.0, 0.0) : gld(win, base + r * NT + tid);
  tile_diag_coeffs<L>(P, h, MODE == MODE_APPLY ? 0.0 : P.beta, s_c, tid);
  const gdbl* zzlo = gptr(P.zzlo);
  double zd[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) zd[r] = (ab & 16) ? 0.0 : zzlo[r * NT + tid];
  __syncthreads();

  // The first cross-tile flip (the rare drive in the center geometry) reads the partner tile
  // elementwise: issue those loads now so their latency hides under the LDS work below.
  const bool pre = (n_fh > 0) && !(ab & 4);
  double2 part[8];
  if (pre) {
    const DFlip F = s_fh[0];
    const gd2* src = win + ((size_t)(h ^ F.tile_xor) << L);
#pragma unroll
    for (int r = 0; r < 8; ++r) part[r] = gld(src, (uint32_t)(r * NT + tid) ^ F.mask_lo);
  }

  // ---- diagonal + register-bit terms (own amplitudes) ----
  double2 out[8];
  {
    double2 own[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) own[r] = s_w[r * NT + tid];
    double gt = s_c[L];
#pragma unroll
    for (int i = 0; i < TB; ++i) gt += s_c[i] * (0.5 - (double)((tid >> i) & 1));
    const double fa = 0.5 * s_c[TB], fb = 0.5 * s_c[TB + 1], fc = 0.5 * s_c[TB + 2];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double d = zd[r] + gt + ((r & 1) ? -fa : fa) + ((r & 2) ? -fb : fb) + ((r & 4) ? -fc : fc);
      out[r].x = d * own[r].x;
      out[r].y = d * own[r].y;
    }
    if (P.rflip_mask) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        if (!((P.rflip_mask >> i) & 1)) continue;
        const double c0r = P.rflip[i][0], c0i = P.rflip[i][1], c1r = P.rflip[i][2], c1i = P.rflip[i][3];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const bool v = (r >> i) & 1;
          out[r] = cmad(out[r], v ? c1r : c0r, v ? c1i : c0i, own[r ^ (1 << i)]);
        }
      }
    }
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
      const int a = (pp == 2) ? 1 : 0, b = (pp == 0) ? 1 : 2;
      const double g = P.rr_g[pp];
      if (g == 0.0) continue;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        if (((r >> a) ^ (r >> b)) & 1) continue;  // compile-time after unrolling
        const double2 sv = own[r ^ ((1 << a) | (1 << b))];
        out[r].x = fma(g, sv.x, out[r].x);
        out[r].y = fma(g, sv.y, out[r].y);
      }
    }
  }

  // ---- thread bits: one LDS sweep of the partner thread per bit j ----
  for (int j = 0; j < ((ab & 1) ? 0 : TB); ++j) {
    const DSweep S = s_sw[j];
    if (!(S.has_flip | S.has_pair)) continue;
    const int bj = (tid >> j) & 1;
    const int pt = tid ^ (1 << j);
    double2 pv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) pv[r] = s_w[r * NT + pt];
    if (S.has_flip) {
      const double cr = bj ? S.re1 : S.re0, ci = bj ? S.im1 : S.im0;
#pragma unroll
      for (int r = 0; r < 8; ++r) out[r] = cmad(out[r], cr, ci, pv[r]);
    }
    if (S.has_pair) {
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double g = S.g[i];
        const double g0 = bj ? 0.0 : g, g1 = bj ? g : 0.0;  // pair applies iff bit_i(r) == bj
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const double gg = ((r >> i) & 1) ? g1 : g0;
          const double2 sv = pv[r ^ (1 << i)];
          out[r].x = fma(gg, sv.x, out[r].x);
          out[r].y = fma(gg, sv.y, out[r].y);
        }
      }
    }
  }
  // ---- the prefetched first cross-tile flip (loads issued before the sweeps) ----
  if (pre) {
    const DFlip F = s_fh[0];
    const bool v = par32(h & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
#pragma unroll
    for (int r = 0; r < 8; ++r) out[r] = cmad(out[r], cr, ci, part[r]);
  }
  // ---- epilogue operand w_{k-2}: issued now, its latency hides under the pair loop ----
  CoefK C = {};
  if (MODE != MODE_APPLY) C = P.coef[set * P.kcap1 + (MODE == MODE_FIRST ? 1 : k)];
  const bool rd = (MODE == MODE_GEN) && !(ab & 8);
  double2 prev[8];
  if (rd) {
#pragma unroll
    for (int r = 0; r < 8; ++r) prev[r] = gld(wdst, base + r * NT + tid);
  }

  // ---- pairs between two thread bits ----
  for (int p = 0; p < ((ab & 2) ? 0 : n_tt); ++p) {
    const DPair Q = s_tt[p];
    if (__popc((uint32_t)tid & Q.mask_lo) & 1) continue;
    const int pt = tid ^ (int)Q.mask_lo;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double2 sv = s_w[r * NT + pt];
      out[r].x = fma(Q.g, sv.x, out[r].x);
      out[r].y = fma(Q.g, sv.y, out[r].y);
    }
  }

  // ---- terms reaching other tiles (global, L2/MALL-served) ----
  // (processed four registers at a time to bound register pressure)
  for (int f = 1; f < ((ab & 4) ? 0 : n_fh); ++f) {
    const DFlip F = s_fh[f];
    const bool v = par32(h & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
    const gd2* src = win + ((size_t)(h ^ F.tile_xor) << L);
#pragma unroll
    for (int hr = 0; hr < 8; hr += 4) {
      double2 sv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = gld(src, (uint32_t)((hr + r) * NT + tid) ^ F.mask_lo);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[hr + r] = cmad(out[hr + r], cr, ci, sv[r]);
    }
  }
  for (int p = 0; p < ((ab & 4) ? 0 : n_ph); ++p) {
    const DPair Q = s_ph[p];
    const int hpar = par32(h & Q.tile_xor);
    if (Q.mask_lo == 0u && hpar) continue;  // both bits above the tile: uniform condition
    const gd2* src = win + ((size_t)(h ^ Q.tile_xor) << L);
#pragma unroll
    for (int hr = 0; hr < 8; hr += 4) {
      double2 sv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = gld(src, (uint32_t)((hr + r) * NT + tid) ^ Q.mask_lo);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t x = (uint32_t)((hr + r) * NT + tid);
        const double g = ((__popc(x & Q.mask_lo) + hpar) & 1) ? 0.0 : Q.g;
        out[hr + r].x = fma(g, sv[r].x, out[hr + r].x);
        out[hr + r].y = fma(g, sv[r].y, out[hr + r].y);
      }
    }
  }

  // ---- recurrence + accumulation ----
  const bool rd_acc = rd && C.upd;
  double2 accv[8];
  if (rd_acc) {
#pragma unroll
    for (int r = 0; r < 8; ++r) accv[r] = gld(acc_b, base + r * NT + tid);
  }
  const double scale = MODE == MODE_GEN ? 2.0 * P.s1 : P.s1;
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const size_t x = base + r * NT + tid;
    const double2 own = s_w[r * NT + tid];
    if (MODE == MODE_APPLY) {
      gst(wdst, x, out[r]);
    } else if (MODE == MODE_FIRST) {
      double2 w;
      w.x = scale * out[r].x;
      w.y = scale * out[r].y;
      gst(wdst, x, w);
      double2 a = make_double2(0.0, 0.0);
      a = cmad(a, C.c[1].x, C.c[1].y, own);
      a = cmad(a, C.c[2].x, C.c[2].y, w);
      gst(acc_b, x, a);
    } else {
      const double2 pr = rd ? prev[r] : make_double2(0.0, 0.0);
      double2 w;
      w.x = fma(scale, out[r].x, -pr.x);
      w.y = fma(scale, out[r].y, -pr.y);
      gst(wdst, x, w);
      if (C.upd) {
        double2 a = rd_acc ? accv[r] : make_double2(0.0, 0.0);
        a = cmad(a, C.c[0].x, C.c[0].y, pr);
        a = cmad(a, C.c[1].x, C.c[1].y, own);
        a = cmad(a, C.c[2].x, C.c[2].y, w);
        gst(acc_b, x, a);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// launch dispatch over the tile size
// ------------------------------------------------------------------------------------------
template <int L>
hipError_t launch_step_L(int mode, const DevProb* probs, const int2* items, int n_items, int k,
                         int q, int set, hipStream_t st) {
  if constexpr (L >= kRegBlockMinTile) {
    dim3 grid(n_items), block(RB<L>::NT);
    if (mode == MODE_APPLY)
      hipLaunchKernelGGL((k_step_rb<L, MODE_APPLY>), grid, block, 0, st, probs, items, k, q, set);
    else if (mode == MODE_FIRST)
      hipLaunchKernelGGL((k_step_rb<L, MODE_FIRST>), grid, block, 0, st, probs, items, k, q, set);
    else
      hipLaunchKernelGGL((k_step_rb<L, MODE_GEN>), grid, block, 0, st, probs, items, k, q, set);
  } else {
    dim3 grid(n_items), block(Geo<L>::NT);
    if (mode == MODE_APPLY)
      hipLaunchKernelGGL((k_step_generic<L, MODE_APPLY>), grid, block, 0, st, probs, items, k, q, set);
    else if (mode == MODE_FIRST)
      hipLaunchKernelGGL((k_step_generic<L, MODE_FIRST>), grid, block, 0, st, probs, items, k, q, set);
    else
      hipLaunchKernelGGL((k_step_generic<L, MODE_GEN>), grid, block, 0, st, probs, items, k, q, set);
  }
  return hipGetLastError();
}

template <int L>
hipError_t launch_obs_L(const DevProb* probs, const int2* items, int n_items, int bsel,
                        double* partial, hipStream_t st) {
  hipLaunchKernelGGL((k_obs<L>), dim3(n_items), dim3(Geo<L>::NT), 0, st, probs, items, bsel, partial);
  return hipGetLastError();
}

}  // namespace

#define DSE_TILE_CASES(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13)

hipError_t launch_step(int L, int mode, const DevProb* probs, const int2* items, int n_items,
                       int k, int q, int set, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  switch (L) {
#define X(l) \
  case l: return launch_step_L<l>(mode, probs, items, n_items, k, q, set, st);
    DSE_TILE_CASES(X)
#undef X
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_obs(int L, const DevProb* probs, const int2* items, int n_items, int bsel,
                      double* partial, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  switch (L) {
#define X(l) \
  case l: return launch_obs_L<l>(probs, items, n_items, bsel, partial, st);
    DSE_TILE_CASES(X)
#undef X
    default: return hipErrorInvalidValue;
  }
}

}  // namespace dse
