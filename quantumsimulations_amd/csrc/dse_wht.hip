// dse_wht.hip -- H|w> for registers larger than two tiles, in the X / Y eigenbases (gfx950).
//
// H = D_Z + sum_b (a_b X_b + b_b Y_b) + sum_{i<j} g_ij (X_i X_j - Y_i Y_j) / 2    (drive
// c_1 = a_b + i b_b = <1|H|0> of bit b, <0|H|1> = conj(c_1); pair g_ij on the rows with
// x_i == x_j; D_Z the diagonal) is
//   H = D_Z + W D_X W + V D_Y V^+,   W = H_had^{(x)n} (unnormalised),  V = S^{(x)n} W,  S = diag(1, i),
//   D_X(z) = 2^-n [ sum_b a_b z_b + sum_{i<j} (g_ij / 2) z_i z_j ],
//   D_Y(z) = 2^-n [ sum_b b_b z_b - sum_{i<j} (g_ij / 2) z_i z_j ],       z_b = 1 - 2 x_b,
// because H_had Z H_had = 2 X and S X S^+ = Y.  The same H as the term tables of k_step_rb
// (reference: dipolar_ensemble_with_rare.py:516-560 builds the drive and flip-flop terms), applied
// with ~n^2 diagonal work per amplitude instead of one partner-tile read per cross-tile term.
//
// The 2^n state lives in HBM; one H application is a few streaming passes over LDS tiles of 2^13
// amplitudes.  Tile bits are split into groups (WhtGroup): group 0 = global bits 0..12, high
// groups = up to 11 high bits each, completed to 13 tile bits by the lowest c "carried" global
// bits.  The transform over all bits is the product of the groups' in-tile transforms:
//   FIRST  (group 0)          w -> A = W0 w,  B = W0 S^+ w            read 16, write 32 B/amp
//   FWD    (groups 1..G-2)    A, B -> W_g A, W_g B                    read 32, write 32
//   MID    (group G-1)        A -> W_g D_X W_g A,  B -> W_g D_Y W_g B  read 32, write 32
//   INV    (groups G-2..1)    as FWD
//   FINAL  (group 0)          out = D_Z w + W0 A + S W0 B, then the Chebyshev epilogue
// G = 2 up to 24 qubits (three passes, ~200 B per amplitude and H application), G = 3 up to 35.
//
// In a tile, thread t of 512 owns 16 amplitudes; the 13 tile bits tau are spread over the thread
// index and a register index differently in three layouts, and a layout change is one LDS
// transpose (write, barrier, read).  Butterflies run on register bits, plus tile bit 0 (thread bit
// 0 of layout C) across neighbouring lanes by DPP:
//   A  r = tau[9..12]  t = tau[0..8]            (global loads and stores: coalesced)
//   B  r = tau[5..8]   t = tau[0..4] | tau[9..12] << 5
//   C  r = tau[1..4]   t = tau[0] | tau[5..12] << 1
// LDS slot of tau: tau for A <-> B, tau + 2 (tau >> 5) for transposes to or from C -- both
// conflict-free for ds_write_b128 (8-lane groups) and ds_read_b128 (16-lane groups) there, and
// both additive in the register index (one base address per thread, immediate offsets per r).
#include "dse_device.h"
#include "dse_wht.h"

namespace dse {
namespace {

constexpr int WL = kWhtTile, WT = 1 << WL, WNT = 512, WR = 16;

__device__ __forceinline__ int tau_of(int lay, int r, int t) {
  switch (lay) {
    case 0: return (r << 9) | t;
    case 1: return (t & 31) | (r << 5) | ((t >> 5) << 9);
    default: return (t & 1) | (r << 1) | ((t >> 1) << 5);
  }
}
// tile bit of register bit i / thread bit j in a layout
__device__ __forceinline__ int reg_tbit(int lay, int i) { return lay == 0 ? 9 + i : lay == 1 ? 5 + i : 1 + i; }
__device__ __forceinline__ int thr_tbit(int lay, int j) {
  switch (lay) {
    case 0: return j;
    case 1: return j < 5 ? j : 4 + j;
    default: return j == 0 ? 0 : 4 + j;
  }
}
// register mask of the bits a layout transforms in a group with c carried bits
__device__ __forceinline__ int active_mask(int lay, int c) {
  int m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (reg_tbit(lay, i) >= c) m |= 1 << i;
  return m;
}
// last layout of a forward sweep
__device__ __forceinline__ int last_layout(int c) { return c <= 4 ? 2 : c <= 8 ? 1 : 0; }

// butterflies (a + b, a - b) on the register bits in amask (wave-uniform)
__device__ __forceinline__ void reg_wht(double2* v, int amask) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (!((amask >> i) & 1)) continue;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      if ((r >> i) & 1) continue;
      const int s = r | (1 << i);
      const double2 a = v[r], b = v[s];
      v[r] = make_double2(a.x + b.x, a.y + b.y);
      v[s] = make_double2(a.x - b.x, a.y - b.y);
    }
  }
}

// value of lane ^ 1 (DPP quad_perm [1,0,3,2])
__device__ __forceinline__ double lane_xor1(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, 0xB1, 0xF, 0xF, true);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), 0xB1, 0xF, 0xF, true);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// butterfly on thread bit 0 (tile bit 0 in layout C)
__device__ __forceinline__ void lane0_wht(double2* v, int tid) {
  const double sg = (tid & 1) ? -1.0 : 1.0;
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    const double px = lane_xor1(v[r].x), py = lane_xor1(v[r].y);
    v[r].x = fma(sg, v[r].x, px);
    v[r].y = fma(sg, v[r].y, py);
  }
}

// LDS slot of (layout, r, t) = base(t) + stride * r (tau, or tau + 2 (tau >> 5) when padded)
template <int LAY, bool PAD>
__device__ __forceinline__ int slot_base(int t) {
  if (LAY == 0) return PAD ? t + 2 * (t >> 5) : t;
  if (LAY == 1) return (t & 31) + (t >> 5) * (PAD ? 544 : 512);
  return (t & 1) + (t >> 1) * 34;  // C is always padded
}
template <int LAY, bool PAD>
constexpr int slot_stride() { return LAY == 0 ? (PAD ? 544 : 512) : LAY == 1 ? (PAD ? 34 : 32) : 2; }

template <int FROM, int TO>
__device__ __forceinline__ void transpose(double2* lds, double2* v, int tid) {
  constexpr bool PAD = FROM == 2 || TO == 2;
  __syncthreads();  // the previous transpose's reads are done
  double2* wp = lds + slot_base<FROM, PAD>(tid);
#pragma unroll
  for (int r = 0; r < WR; ++r) wp[r * slot_stride<FROM, PAD>()] = v[r];
  __syncthreads();
  const double2* rp = lds + slot_base<TO, PAD>(tid);
#pragma unroll
  for (int r = 0; r < WR; ++r) v[r] = rp[r * slot_stride<TO, PAD>()];
}

__device__ __forceinline__ void layout_wht(double2* v, int lay, int c, int tid) {
  reg_wht(v, active_mask(lay, c));
  if (lay == 2 && c == 0) lane0_wht(v, tid);
}
// forward sweep from layout A; returns the layout it ends in
__device__ __forceinline__ int tile_fwd(double2* lds, double2* v, int c, int tid) {
  const int last = last_layout(c);
  layout_wht(v, 0, c, tid);
  if (last >= 1) {
    transpose<0, 1>(lds, v, tid);
    layout_wht(v, 1, c, tid);
  }
  if (last >= 2) {
    transpose<1, 2>(lds, v, tid);
    layout_wht(v, 2, c, tid);
  }
  return last;
}
// the same butterflies in reverse layout order, from layout `last` back to A
__device__ __forceinline__ void tile_back(double2* lds, double2* v, int c, int last, int tid) {
  if (last >= 2) {
    layout_wht(v, 2, c, tid);
    transpose<2, 1>(lds, v, tid);
  }
  if (last >= 1) {
    layout_wht(v, 1, c, tid);
    transpose<1, 0>(lds, v, tid);
  }
  layout_wht(v, 0, c, tid);
}
__device__ __forceinline__ void tile_full(double2* lds, double2* v, int c, int tid) {
  const int last = tile_fwd(lds, v, c, tid);
  if (last == 2) transpose<2, 0>(lds, v, tid);
  if (last == 1) transpose<1, 0>(lds, v, tid);
}

struct WhtShared {
  double2 w[WT + 2 * (WT >> 5)];  // padded slots (slot_base)
  double fx[WL + 1], fy[WL + 1];  // per-tile linear coefficients of D_X, D_Y (index WL: constant; xytab)
  double cq[WL * WL];             // in-tile couplings c(q, q'), symmetric (D_X sign)
  double zr[WR];                  // register-register part of D_X in the MID layout
  double cz[WL + 1];              // D_Z of a group-0 tile: F_i(h), C(h) - beta (ztab)
};

__device__ __forceinline__ double zsign(uint64_t v, int b) { return ((v >> b) & 1ull) ? -1.0 : 1.0; }

// In-tile couplings c(pos_q, pos_q') of a group (same for all its tiles).  No barrier.
__device__ __forceinline__ void stage_couplings(const WhtProb& W, const WhtGroup& G, WhtShared& S, int tid) {
  const gdbl* cq = gptr(W.cquad);
  for (int e = tid; e < WL * WL; e += WNT) S.cq[e] = cq[G.pos[e / WL] * W.n + G.pos[e % WL]];
}

// zr[r] of layout lay (needs S.cq after a barrier)
__device__ __forceinline__ void tile_zr(WhtShared& S, int lay, int tid) {
  if (tid < WR) {
    double v = 0.0;
    for (int a = 0; a < 4; ++a)
      for (int b = a + 1; b < 4; ++b)
        v += S.cq[reg_tbit(lay, a) * WL + reg_tbit(lay, b)] * (zsign(tid, a) * zsign(tid, b));
    S.zr[tid] = v;
  }
}

// v *= D_X (xsel) or D_Y in layout lay: per-thread part zt, register-bit fields hr, register
// pairs zr (uniform per r).
__device__ __forceinline__ void apply_xy_diag(const WhtShared& S, int lay, bool xsel, double2* v, int tid) {
  const double sg = xsel ? 1.0 : -1.0;
  const double* f = xsel ? S.fx : S.fy;
  double zt = f[WL];
  double hr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) hr[i] = f[reg_tbit(lay, i)];
#pragma unroll 1
  for (int j = 0; j < 9; ++j) {
    const int qj = thr_tbit(lay, j);
    const double zj = zsign(tid, j);
    double a = f[qj];
#pragma unroll 1
    for (int i = j + 1; i < 9; ++i) a += sg * S.cq[qj * WL + thr_tbit(lay, i)] * zsign(tid, i);
    zt += a * zj;
#pragma unroll
    for (int i = 0; i < 4; ++i) hr[i] += sg * S.cq[qj * WL + reg_tbit(lay, i)] * zj;
  }
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    double d = zt + sg * S.zr[r];
#pragma unroll
    for (int i = 0; i < 4; ++i) d += ((r >> i) & 1 ? -1.0 : 1.0) * hr[i];
    v[r].x *= d;
    v[r].y *= d;
  }
}

// v * i^k
__device__ __forceinline__ double2 mul_ipow(double2 v, int k) {
  switch (k & 3) {
    case 0: return v;
    case 1: return make_double2(-v.y, v.x);
    case 2: return make_double2(-v.x, -v.y);
    default: return make_double2(v.y, -v.x);
  }
}

__device__ __forceinline__ uint64_t outer_bits(const WhtGroup& G, uint64_t o) {
  uint64_t x = 0;
  for (int i = 0; i < G.n_outer; ++i) x |= ((o >> i) & 1ull) << G.opos[i];
  return x;
}

// input vector of term k (buffer roles of k_step_rb)
__device__ __forceinline__ int win_role(int mode, int k, int q) {
  if (mode == MODE_APPLY) return 0;
  if (mode == MODE_FIRST) return q ? 2 : 0;
  return ((k - 1) & 1) ? 1 : (q ? 2 : 0);
}

template <int PASS, int MODE>
__global__ void __launch_bounds__(WNT)
k_wht(const WhtProb* __restrict__ probs, const DevProb* __restrict__ dprobs, const int2* __restrict__ items,
      int g, int k, int q, int set) {
  __shared__ WhtShared S;
  const int2 it = items[blockIdx.x];
  const WhtProb& W = probs[it.x];
  const DevProb& P = dprobs[it.x];
  const int tid = threadIdx.x;
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform
  const WhtGroup& G = W.grp[g];
  const uint64_t o = (uint64_t)(uint32_t)it.y;  // outer index of the tile
  const uint64_t xo = outer_bits(G, o);

  // global indices of this thread's amplitudes in layout A: xo | xt | xr[r]
  uint64_t xt = 0;
  for (int j = 0; j < 9; ++j) xt |= (uint64_t)((tid >> j) & 1) << G.pos[j];
  uint64_t xr[WR];
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    uint64_t a = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) a |= (uint64_t)((r >> i) & 1) << G.pos[9 + i];
    xr[r] = a;
  }
  const uint64_t xb = xo | xt;

  double2 v[WR];
  if (PASS == WHT_FIRST) {
    const gd2* win = gptr((const double2*)P.buf[win_role(MODE, k, q)]);
    double2 u[WR];
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      v[r] = gld(win, xb | xr[r]);
      u[r] = mul_ipow(v[r], -__popcll(xb | xr[r]));  // S^+ of every qubit
    }
    tile_full(S.w, v, 0, tid);
    gd2* A = gptr(W.vec_a);
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(A, xb | xr[r], v[r]);
    tile_full(S.w, u, 0, tid);
    gd2* B = gptr(W.vec_b);
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(B, xb | xr[r], u[r]);
    return;
  }

  if (PASS == WHT_FWD || PASS == WHT_INV || PASS == WHT_MID) {
    const int lm = last_layout(G.c);
    if (PASS == WHT_MID) {
      stage_couplings(W, G, S, tid);
      if (tid < 32) {
        const double c = gptr((const double*)W.xytab)[o * 32 + tid];
        if (tid <= WL) S.fx[tid] = c;
        else if (tid >= 16 && tid <= 16 + WL) S.fy[tid - 16] = c;
      }
      __syncthreads();
      tile_zr(S, lm, tid);  // read after the first transpose's barriers
    }
#pragma unroll 1
    for (int vec = 0; vec < 2; ++vec) {
      gd2* X = gptr(vec == 0 ? W.vec_a : W.vec_b);
#pragma unroll
      for (int r = 0; r < WR; ++r) v[r] = gld(X, xb | xr[r]);
      if (PASS == WHT_MID) {
        if (lm == 0) __syncthreads();  // no transpose before the diagonal: S.zr
        tile_fwd(S.w, v, G.c, tid);
        apply_xy_diag(S, lm, vec == 0, v, tid);
        tile_back(S.w, v, G.c, lm, tid);
      } else {
        tile_full(S.w, v, G.c, tid);
      }
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(X, xb | xr[r], v[r]);
    }
    return;
  }

  // ---- FINAL (group 0 tile = ordinary tile h): out = D_Z w + W0 A + S W0 B, then the recurrence
  if (PASS == WHT_FINAL) {
    const uint32_t h = (uint32_t)o;
    if (tid <= WL) {
      const double c = gptr((const double*)W.ztab)[(uint64_t)h * 16 + tid];
      S.cz[tid] = (tid == WL && MODE != MODE_APPLY) ? c - P.beta : c;
    }
    double2 out[WR];
    const gd2* B = gptr((const double2*)W.vec_b);
#pragma unroll
    for (int r = 0; r < WR; ++r) out[r] = gld(B, xb | xr[r]);
    tile_full(S.w, out, 0, tid);
#pragma unroll
    for (int r = 0; r < WR; ++r) out[r] = mul_ipow(out[r], __popcll(xb | xr[r]));  // S of every qubit
    const gd2* A = gptr((const double2*)W.vec_a);
#pragma unroll
    for (int r = 0; r < WR; ++r) v[r] = gld(A, xb | xr[r]);
    tile_full(S.w, v, 0, tid);
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      out[r].x += v[r].x;
      out[r].y += v[r].y;
    }
    __syncthreads();  // S.cz
    // D_Z(x) = zzlo[x_lo] + C(h) + sum_i F_i(h) s_i(x_lo),  s = 1/2 - bit,  x_lo = r * 512 + tid
    double gt = S.cz[WL];
#pragma unroll
    for (int i = 0; i < 9; ++i) gt += S.cz[i] * (0.5 - (double)((tid >> i) & 1));
    const gd2* win = gptr((const double2*)P.buf[win_role(MODE, k, q)]);
    const gdbl* zzlo = gptr(P.zzlo);
    gd2* psi_b = gptr(P.buf[q ? 2 : 0]);
    gd2* acc_b = gptr(P.buf[q ? 0 : 2]);
    gd2* scr_b = gptr(P.buf[1]);
    CoefK C = {};
    if (MODE != MODE_APPLY) C = P.coef[set * P.kcap1 + (MODE == MODE_FIRST ? 1 : k)];
    gd2* wdst = (MODE == MODE_GEN && !(k & 1)) ? psi_b : scr_b;  // GEN: holds w_{k-2}
    const double scale = MODE == MODE_GEN ? 2.0 * P.s1 : P.s1;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      const double2 own = gld(win, xb | xr[r]);
      double d = zzlo[r * WNT + tid] + gt;
#pragma unroll
      for (int i = 0; i < 4; ++i) d += S.cz[9 + i] * (((r >> i) & 1) ? -0.5 : 0.5);
      out[r].x = fma(d, own.x, out[r].x);
      out[r].y = fma(d, own.y, out[r].y);
      step_epilogue<MODE>(xb | xr[r], out[r], own, scale, wdst, acc_b, C, 0);
    }
  }
}

// One thread per tile o: D_Z pieces of group-0 tile o (tile_diag_coeffs without beta) and the
// D_X / D_Y pieces of MID-group tile o:  F_q = lin(pos_q) + sum_i c(pos_q, opos_i) z_i,
// C = sum_i lin(opos_i) z_i + sum_{i<j} c(opos_i, opos_j) z_i z_j  (D_Y: lin_y, -c).
__global__ void __launch_bounds__(256) k_wht_tables(const WhtProb* __restrict__ wp, const DevProb* __restrict__ dp,
                                                    int64_t tiles) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= tiles) return;
  const WhtProb& W = *wp;
  const DevProb& P = *dp;
  const int n = W.n;
  double* zt = W.ztab + o * 16;
  for (int i = 0; i < WL; ++i) {
    double f = P.field[i];
    for (int j = WL; j < n; ++j) f += P.zz[i * n + j] * (0.5 - (double)((o >> (j - WL)) & 1));
    zt[i] = f;
  }
  double c = P.shift;
  for (int j = WL; j < n; ++j) {
    const double sj = 0.5 - (double)((o >> (j - WL)) & 1);
    c += P.field[j] * sj;
    for (int i = WL; i < j; ++i) c += P.zz[i * n + j] * ((0.5 - (double)((o >> (i - WL)) & 1)) * sj);
  }
  zt[WL] = c;
  zt[WL + 1] = zt[WL + 2] = 0.0;
  const WhtGroup& G = W.grp[W.n_groups - 1];
  const double* cq = W.cquad;
  double* xy = W.xytab + o * 32;
  for (int q = 0; q < WL; ++q) {
    const int b = G.pos[q];
    double fx = W.lin_x[b], fy = W.lin_y[b];
    for (int i = 0; i < G.n_outer; ++i) {
      const double v = cq[b * n + G.opos[i]] * zsign(o, i);
      fx += v;
      fy -= v;
    }
    xy[q] = fx;
    xy[16 + q] = fy;
  }
  double cx = 0.0, cy = 0.0;
  for (int i = 0; i < G.n_outer; ++i) {
    const int bi = G.opos[i];
    const double zi = zsign(o, i);
    cx += W.lin_x[bi] * zi;
    cy += W.lin_y[bi] * zi;
    for (int j = i + 1; j < G.n_outer; ++j) {
      const double v = cq[bi * n + G.opos[j]] * (zi * zsign(o, j));
      cx += v;
      cy -= v;
    }
  }
  xy[WL] = cx;
  xy[16 + WL] = cy;
  xy[14] = xy[15] = xy[30] = xy[31] = 0.0;
}

template <int PASS>
hipError_t launch_pass(int mode, const WhtProb* wp, const DevProb* dp, const int2* items, int n_items,
                       int g, int k, int q, int set, hipStream_t st) {
  const dim3 grid(n_items), block(WNT);
  if (mode == MODE_APPLY)
    hipLaunchKernelGGL((k_wht<PASS, MODE_APPLY>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else if (mode == MODE_FIRST)
    hipLaunchKernelGGL((k_wht<PASS, MODE_FIRST>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else
    hipLaunchKernelGGL((k_wht<PASS, MODE_GEN>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_wht_tables(const WhtProb* wp, const DevProb* dp, int64_t tiles, hipStream_t st) {
  hipLaunchKernelGGL(k_wht_tables, dim3((unsigned)((tiles + 255) / 256)), dim3(256), 0, st, wp, dp, tiles);
  return hipGetLastError();
}

hipError_t launch_wht_step(int mode, int n_groups, const WhtProb* wp, const DevProb* dp,
                           const int2* items, int n_items, int k, int q, int set, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  if (n_groups < 2 || n_groups > kWhtMaxGroups) return hipErrorInvalidValue;
  hipError_t e = launch_pass<WHT_FIRST>(mode, wp, dp, items, n_items, 0, k, q, set, st);
  for (int g = 1; e == hipSuccess && g + 1 < n_groups; ++g)
    e = launch_pass<WHT_FWD>(mode, wp, dp, items, n_items, g, k, q, set, st);
  if (e == hipSuccess) e = launch_pass<WHT_MID>(mode, wp, dp, items, n_items, n_groups - 1, k, q, set, st);
  for (int g = n_groups - 2; e == hipSuccess && g >= 1; --g)
    e = launch_pass<WHT_INV>(mode, wp, dp, items, n_items, g, k, q, set, st);
  if (e == hipSuccess) e = launch_pass<WHT_FINAL>(mode, wp, dp, items, n_items, 0, k, q, set, st);
  return e;
}

}  // namespace dse
