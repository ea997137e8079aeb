// dse_device.h -- device helpers shared by the step kernels (dse_kernels.hip) and the
// persistent interval kernel (dse_interval.hip).  Internal to libdse.
#pragma once

#include "dse_internal.h"

namespace dse {

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

// constant address space: uniform loads become scalar loads (SGPRs, scalar cache)
template <typename T>
using cptr = const __attribute__((address_space(4))) T*;
template <typename T>
__device__ __forceinline__ cptr<T> cst(const T* p) {
  return (cptr<T>)p;
}

// Global address-space views: loads through them are global_load (vmcnt only) instead of
// flat_load (which also counts against lgkmcnt and serialises LDS work).
typedef double __attribute__((ext_vector_type(2))) dv2;
typedef __attribute__((address_space(1))) dv2 gd2;
typedef __attribute__((address_space(1))) double gdbl;
__device__ __forceinline__ gd2* gptr(double2* p) { return (gd2*)p; }
__device__ __forceinline__ const gd2* gptr(const double2* p) { return (const gd2*)p; }
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

// A wave-uniform double moved into SGPRs (a vector load of a uniform address leaves it in VGPRs)
__device__ __forceinline__ double uniform_d(double v) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Buffer-resource views of one tile (wave-uniform base, 32-bit byte offsets): per-register
// accesses become buffer ops with the register offset in an SGPR instead of one 64-bit VGPR
// address per register.  aux = kSc1 makes a store write-through to the coherence point and a load
// bypass the non-coherent L1 (cross-workgroup hand-off, MI355X_MICROARCH.md Valid forms row 1).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kSc1 = 16;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const double2* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)bytes,
                                           0x00020000);
}
template <int AUX = 0>
__device__ __forceinline__ double2 bld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, AUX);
  const dv2 d = __builtin_bit_cast(dv2, v);
  return make_double2(d.x, d.y);
}
template <int AUX = 0>
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                    double2 a) {
  dv2 d;
  d.x = a.x;
  d.y = a.y;
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d), r, (int)voff, (int)soff, AUX);
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

// (returns the value stored to wdst: the new vector, for a caller that keeps it)
template <int MODE, typename Ptr>
__device__ __forceinline__ double2 step_epilogue(size_t x, double2 out, double2 own, double scale,
                                                 Ptr __restrict__ wdst, Ptr __restrict__ acc_b,
                                                 const CoefK& C, int no_reads) {
  if (MODE == MODE_APPLY) {
    gst(wdst, x, out);
    return out;
  } else if (MODE == MODE_FIRST) {
    double2 w;
    w.x = scale * out.x;
    w.y = scale * out.y;
    gst(wdst, x, w);
    double2 a = make_double2(0.0, 0.0);
    a = cmad(a, C.c[1].x, C.c[1].y, own);
    a = cmad(a, C.c[2].x, C.c[2].y, w);
    gst(acc_b, x, a);
    return w;
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
    return w;
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

template <int L>
struct RB {
  static constexpr int T = 1 << L;
  static constexpr int R = kRegAmps;         // amplitudes per thread
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


// ------------------------------------------------------------------------------------------
// Register-block application of the in-tile part of H (LDS only)
// ------------------------------------------------------------------------------------------
// Workgroup-shared state of the register-block kernels.  One thread owns the R = 16 amplitudes
// x = r * NT + tid (r = 0..15): the four top tile bits are register bits.
template <int L>
struct RBShared {
  static constexpr int TB = RB<L>::TB;
  static constexpr int NTT = TB * (TB - 1) / 2;
  double2 w[RB<L>::T];               // the tile of w_{k-1}
  double c[L + 1];                   // F_i(h) (i < L) and C(h) of the tile
  double zz[L * L];                  // in-tile zz couplings (row-major, upper triangle)
  double zr[kRegAmps];               // register-bit ZZ part of the diagonal per r
  DSweep sw[TB];                     // thread-bit sweeps
  DPair tt[NTT > 0 ? NTT : 1];       // thread-bit pairs
  DPair ph[HiCap<L>::PAIRS];         // cross-tile pairs
  DFlip fh[HiCap<L>::FLIPS];         // cross-tile drive flips
};

// Stages the term tables of problem P into S (no barrier).  Also the in-tile zz block and the
// per-tile diagonal coefficients (tile_diag_coeffs).
template <int L>
__device__ __forceinline__ void rb_stage_tables(RBShared<L>& S, const DevProb& P, uint32_t h,
                                                double beta, int tid) {
  constexpr int NT = RB<L>::NT, TB = RB<L>::TB;
  stage16(S.sw, P.sweeps, TB * (int)(sizeof(DSweep) / 16), tid, NT);
  stage16(S.tt, P.pairs_tt, P.n_pairs_tt, tid, NT);
  stage16(S.ph, P.pairs_hi, P.n_pairs_hi, tid, NT);
  stage16(S.fh, P.flips_hi, P.n_flips_hi * (int)(sizeof(DFlip) / 16), tid, NT);
  const gdbl* zz = gptr(P.zz);
  const int n = P.n;
  for (int e = tid; e < L * L; e += NT) {
    const int i = e / L, j = e % L;
    S.zz[e] = (j > i) ? zz[i * n + j] : 0.0;
  }
  tile_diag_coeffs<L>(P, h, beta, S.c, tid);
}

// Per-thread diagonal: D(r) = zt + sum_i hr[i] s_i(r) + zr[r]  (needs S.zz, S.c; after a barrier)
//   zt    = C(h) + sum_{j<TB} F_j s_j(tid) + sum_{i<j<TB} zz_ij s_i(tid) s_j(tid)
//   hr[i] = F_{TB+i} + sum_{j<TB} zz_{j,TB+i} s_j(tid)
struct ThreadDiag {
  double zt;
  double hr[kRegBits];
};

template <int L>
__device__ __forceinline__ ThreadDiag rb_thread_diag(const RBShared<L>& S, int tid) {
  constexpr int TB = RB<L>::TB;
  ThreadDiag d;
  d.zt = S.c[L];
#pragma unroll
  for (int i = 0; i < kRegBits; ++i) d.hr[i] = S.c[TB + i];
#pragma unroll 1
  for (int j = 0; j < TB; ++j) {
    const double sj = 0.5 - (double)((tid >> j) & 1);
    double a = S.c[j];
#pragma unroll 1
    for (int i = j + 1; i < TB; ++i) a += S.zz[j * L + i] * (0.5 - (double)((tid >> i) & 1));
    d.zt += a * sj;
#pragma unroll
    for (int i = 0; i < kRegBits; ++i) d.hr[i] += S.zz[j * L + TB + i] * sj;
  }
  return d;
}

// zr[r] for the register patterns (one thread per entry; needs S.zz after a barrier)
template <int L>
__device__ __forceinline__ void rb_register_zz(RBShared<L>& S, int tid) {
  constexpr int TB = RB<L>::TB;
  if (tid < kRegAmps) {
    double v = 0.0;
    for (int a = 0; a < kRegBits; ++a)
      for (int b = a + 1; b < kRegBits; ++b)
        v += S.zz[(TB + a) * L + TB + b] * ((0.5 - ((tid >> a) & 1)) * (0.5 - ((tid >> b) & 1)));
    S.zr[tid] = v;
  }
}

// Pairs (thread bit j, register bit i) of one sweep for a wave-uniform bit value BJ of thread
// bit j: the pair applies iff bit_i(r) == BJ, so only those registers are touched.
template <int BJ>
__device__ __forceinline__ void rb_sweep_pairs_uniform(const DSweep& Sw, const double2* pv,
                                                       double2* out) {
#pragma unroll
  for (int i = 0; i < kRegBits; ++i) {
    const double g = Sw.g[i];
#pragma unroll
    for (int r = 0; r < kRegAmps; ++r) {
      if (((r >> i) & 1) != BJ) continue;  // compile-time
      const double2 sv = pv[r ^ (1 << i)];
      out[r].x = fma(g, sv.x, out[r].x);
      out[r].y = fma(g, sv.y, out[r].y);
    }
  }
}

// out = (H - beta) w on the tile's own terms, part A: diagonal, register-bit drives/pairs and
// thread-bit sweeps (one LDS read of the partner thread per bit, serving its drive and its
// pairs with the register bits).  Part B (rb_apply_tile_b): pairs between two thread bits.
// Cross-tile terms are added by the caller.
template <int L>
__device__ __forceinline__ void rb_apply_tile_a(const RBShared<L>& S, const DevProb& P, int tid,
                                                const ThreadDiag& td, int ab,
                                                double2 out[kRegAmps]) {
  constexpr int NT = RB<L>::NT, TB = RB<L>::TB, R = kRegAmps;
  {
    double2 own[R];
#pragma unroll
    for (int r = 0; r < R; ++r) own[r] = S.w[r * NT + tid];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      double d = td.zt + S.zr[r];
#pragma unroll
      for (int i = 0; i < kRegBits; ++i) d += ((r >> i) & 1 ? -0.5 : 0.5) * td.hr[i];
      out[r].x = d * own[r].x;
      out[r].y = d * own[r].y;
    }
    if (P.rflip_mask) {
#pragma unroll
      for (int i = 0; i < kRegBits; ++i) {
        if (!((P.rflip_mask >> i) & 1)) continue;
        const double c0r = P.rflip[i][0], c0i = P.rflip[i][1], c1r = P.rflip[i][2], c1i = P.rflip[i][3];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const bool v = (r >> i) & 1;
          out[r] = cmad(out[r], v ? c1r : c0r, v ? c1i : c0i, own[r ^ (1 << i)]);
        }
      }
    }
#pragma unroll
    for (int a = 0; a < kRegBits; ++a)
#pragma unroll
      for (int b = a + 1; b < kRegBits; ++b) {
        const double g = P.rr_g[rr_index(a, b)];
        if (g == 0.0) continue;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (((r >> a) ^ (r >> b)) & 1) continue;  // compile-time after unrolling
          const double2 sv = own[r ^ ((1 << a) | (1 << b))];
          out[r].x = fma(g, sv.x, out[r].x);
          out[r].y = fma(g, sv.y, out[r].y);
        }
      }
  }
#pragma unroll 1
  for (int j = 0; j < ((ab & 1) ? 0 : TB); ++j) {
    const DSweep Sw = S.sw[j];
    if (!(Sw.has_flip | Sw.has_pair)) continue;
    const int bj = (tid >> j) & 1;
    const int pt = tid ^ (1 << j);
    double2 pv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) pv[r] = S.w[r * NT + pt];
    if (Sw.has_flip) {
      const double cr = bj ? Sw.re1 : Sw.re0, ci = bj ? Sw.im1 : Sw.im0;
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = cmad(out[r], cr, ci, pv[r]);
    }
    if (Sw.has_pair) {
      if (j >= 6) {  // a wave-index bit: bj is uniform, touch only the registers it pairs
        if (bj)
          rb_sweep_pairs_uniform<1>(Sw, pv, out);
        else
          rb_sweep_pairs_uniform<0>(Sw, pv, out);
      } else {
#pragma unroll
        for (int i = 0; i < kRegBits; ++i) {
          const double g = Sw.g[i];
          const double g0 = bj ? 0.0 : g, g1 = bj ? g : 0.0;  // pair applies iff bit_i(r) == bj
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const double gg = ((r >> i) & 1) ? g1 : g0;
            const double2 sv = pv[r ^ (1 << i)];
            out[r].x = fma(gg, sv.x, out[r].x);
            out[r].y = fma(gg, sv.y, out[r].y);
          }
        }
      }
    }
  }
}

template <int L>
__device__ __forceinline__ void rb_apply_tile_b(const RBShared<L>& S, const DevProb& P, int tid,
                                                int ab, double2 out[kRegAmps]) {
  constexpr int NT = RB<L>::NT;
  const int n_tt = (ab & 2) ? 0 : P.n_pairs_tt;
#pragma unroll 1
  for (int p = 0; p < n_tt; ++p) {
    const DPair Q = S.tt[p];
    if (__popc((uint32_t)tid & Q.mask_lo) & 1) continue;
    const int pt = tid ^ (int)Q.mask_lo;
#pragma unroll
    for (int r = 0; r < kRegAmps; ++r) {
      const double2 sv = S.w[r * NT + pt];
      out[r].x = fma(Q.g, sv.x, out[r].x);
      out[r].y = fma(Q.g, sv.y, out[r].y);
    }
  }
}

}  // namespace
}  // namespace dse
