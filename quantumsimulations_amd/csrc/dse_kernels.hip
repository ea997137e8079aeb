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
#include <algorithm>

#include "dse_device.h"

namespace dse {

// Diagnostic ablation mask (diagnostics builds, -DDSE_DIAG; 0 in libdse.so): sections of k_step_rb
// to skip, for timing only.
//   1 thread-bit sweeps   2 thread-thread pairs   4 cross-tile terms   8 epilogue global reads
//   16 diagonal table read   32 tile load from global memory
#ifdef DSE_DIAG
__device__ int g_dse_ablate = 0;
hipError_t set_ablate(int mask) { return hipMemcpyToSymbol(HIP_SYMBOL(g_dse_ablate), &mask, sizeof(int)); }
#else
constexpr int g_dse_ablate = 0;
hipError_t set_ablate(int mask) { return mask ? hipErrorNotSupported : hipSuccess; }
#endif

namespace {

template <int L, int MODE>
__global__ void __launch_bounds__(Geo<L>::NT)
k_step_generic(const DevProb* __restrict__ probs, const int2* __restrict__ items, int k, int q, int set) {
  using G = Geo<L>;
  constexpr int T = G::T, NT = G::NT, R = G::R;
  __shared__ double2 s_w[T];
  __shared__ double s_c[L + 1];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;       // local tile
  const uint32_t hg = P.h_base | h;          // global tile index (partitioned registers)
  const int tid = threadIdx.x;
  const bool live = (T >= NT) || (tid < T);
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform: this problem's interval is done

  // buffer roles (see host loop): psi = buf[q?2:0], acc = buf[q?0:2], scratch = buf[1]
  double2* psi_b = P.buf[q ? 2 : 0];
  double2* acc_b = P.buf[q ? 0 : 2];
  double2* scr_b = P.buf[1];
  int win_role;
  double2* wdst;
  if (MODE == MODE_APPLY) {
    win_role = 0;
    wdst = P.buf[1];
  } else if (MODE == MODE_FIRST) {
    win_role = q ? 2 : 0;
    wdst = scr_b;
  } else {
    win_role = ((k - 1) & 1) ? 1 : (q ? 2 : 0);
    wdst = (k & 1) ? scr_b : psi_b;  // holds w_{k-2}; overwritten in place with w_k
  }
  const double2* win = P.buf[win_role];
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
  tile_diag_coeffs<L>(P, hg, MODE == MODE_APPLY ? 0.0 : P.beta, s_c, tid);
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
    const bool v = par32(hg & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
    const double2* src = tile_ptr(P, win_role, hg ^ F.tile_xor);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t x = (uint32_t)(r * NT + tid);
      out[r] = cmad(out[r], cr, ci, src[x ^ F.mask_lo]);
    }
  }
  for (int p = 0; p < P.n_pairs_hi; ++p) {
    const DPair Q = P.pairs_hi[p];
    const int hp = par32(hg & Q.tile_xor);
    const double2* src = tile_ptr(P, win_role, hg ^ Q.tile_xor);
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
  if (MODE != MODE_APPLY) C = coef_at(coef_row(P, set, 0), MODE == MODE_FIRST ? 1 : k);
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
k_obs(const DevProb* __restrict__ probs, const int2* __restrict__ items, int bsel_last,
      double* __restrict__ partial, size_t out_stride, int xq) {
  using G = Geo<L>;
  constexpr int T = G::T, NT = G::NT, R = G::R;
  __shared__ double2 s_w[T];
  __shared__ double s_red[NT / 64][8];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const uint32_t hg = P.h_base | h;
  const int tid = threadIdx.x;
  const bool live = (T >= NT) || (tid < T);
  // blockIdx.y = output j of the group: the last one in state buffer role bsel_last (< 3), the
  // others in intermediate output j (bsel = 3 + j) of a multi-output launch
  const int bsel = (blockIdx.y == gridDim.y - 1) ? bsel_last : 3 + (int)blockIdx.y;
  partial += (size_t)blockIdx.y * out_stride;
  const double2* psi = bsel < 3 ? P.buf[bsel] : P.xacc + ((size_t)(xq * P.xacc_q + bsel - 3) << (L + P.tbl));
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
    const uint64_t hi = (uint64_t)hg << L;
    const double half_sea = 0.5 * (double)P.n_sea;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t x = hi | (uint64_t)(r * NT + tid);
      const double p2 = own[r].x * own[r].x + own[r].y * own[r].y;
      acc[6] += p2;
      acc[2] += p2 * (half_sea - (double)__popcll(x & P.sea_mask));
      if (P.rare_bit >= 0) acc[3] += p2 * (0.5 - (double)((x >> P.rare_bit) & 1ull));
    }
    // in-tile bits, unrolled: a register bit's partner is another row of this thread (no LDS
    // read, rows chosen at compile time), a thread bit's rows are all this lane's or none; same
    // rows in the same order as a per-row test, so the sums are bitwise unchanged
    constexpr int TB = G::TB;
#pragma unroll
    for (int b = 0; b < L; ++b) {
      if (b >= P.n) break;
      const bool sea = (P.sea_mask >> b) & 1ull;
      const bool rr = (b == P.rare_bit);
      if (!sea && !rr) continue;
      double ore = 0.0, oim = 0.0;
      if (b >= TB) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if ((r >> (b - TB)) & 1) continue;
          const double2 s = own[r ^ (1 << (b - TB))];
          ore += own[r].x * s.x + own[r].y * s.y;
          oim += own[r].x * s.y - own[r].y * s.x;
        }
      } else if (!((tid >> b) & 1)) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const double2 s = s_w[(uint32_t)(r * NT + tid) ^ (1u << b)];
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
    for (int b = L; b < P.n; ++b) {
      const bool sea = (P.sea_mask >> b) & 1ull;
      const bool rr = (b == P.rare_bit);
      if (!sea && !rr) continue;
      double ore = 0.0, oim = 0.0;
      {
        if ((hg >> (b - L)) & 1u) continue;
        const uint32_t hp = hg ^ (1u << (b - L));
        // intermediate outputs (bsel >= 3) live only in this context, unsharded
        const double2* src = bsel < 3 ? tile_ptr(P, bsel, hp)
                                      : psi + ((size_t)(hp & ((1u << P.tbl) - 1u)) << L);
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
template <int L, int MODE>
__global__ void __launch_bounds__(RB<L>::NT)
k_step_rb(const DevProb* __restrict__ probs, const int2* __restrict__ items, int k, int q, int set) {
  constexpr int NT = RB<L>::NT, R = kRegAmps;
  __shared__ RBShared<L> S;

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;       // local tile
  const uint32_t hg = P.h_base | h;          // global tile index (partitioned registers)
  const int tid = threadIdx.x;
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform: this problem's interval is done

  const int ab = g_dse_ablate;
  const int n_ph = P.n_pairs_hi, n_fh = P.n_flips_hi;
  gd2* psi_b = gptr(P.buf[q ? 2 : 0]);
  gd2* acc_b = gptr(P.buf[q ? 0 : 2]);
  gd2* scr_b = gptr(P.buf[1]);
  int win_role;
  gd2* wdst;
  if (MODE == MODE_APPLY) {
    win_role = 0;
    wdst = gptr(P.buf[1]);
  } else if (MODE == MODE_FIRST) {
    win_role = q ? 2 : 0;
    wdst = scr_b;
  } else {
    win_role = ((k - 1) & 1) ? 1 : (q ? 2 : 0);
    wdst = (k & 1) ? scr_b : psi_b;
  }
  const gd2* win = gptr(P.buf[win_role]);
  const size_t base = (size_t)h << L;

  rb_stage_tables<L>(S, P, hg, MODE == MODE_APPLY ? 0.0 : P.beta, tid);
#pragma unroll
  for (int r = 0; r < R; ++r)
    S.w[r * NT + tid] = (ab & 32) ? make_double2(1.0, 0.0) : gld(win, base + r * NT + tid);
  __syncthreads();
  rb_register_zz<L>(S, tid);
  const ThreadDiag td = rb_thread_diag<L>(S, tid);
  __syncthreads();

  // The first cross-tile flip (the rare drive in the center geometry) reads the partner tile
  // elementwise: issue those loads now so their latency hides under the sweeps.
  const bool pre = (n_fh > 0) && !(ab & 4);
  double2 part[R];
  if (pre) {
    const DFlip F = S.fh[0];
    const gd2* src = gptr(tile_ptr(P, win_role, hg ^ F.tile_xor));
#pragma unroll
    for (int r = 0; r < R; ++r) part[r] = gld(src, (uint32_t)(r * NT + tid) ^ F.mask_lo);
  }

  double2 out[R];
  rb_apply_tile_a<L>(S, P, tid, td, ab, out);

  if (pre) {
    const DFlip F = S.fh[0];
    const bool v = par32(hg & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = cmad(out[r], cr, ci, part[r]);
  }
  // epilogue operand w_{k-2}: issued now, its latency hides under the thread-pair loop
  CoefK C = {};
  if (MODE != MODE_APPLY) C = coef_at(coef_row(P, set, 0), MODE == MODE_FIRST ? 1 : k);
  const bool rd = (MODE == MODE_GEN) && !(ab & 8);
  double2 prev[R];
  if (rd) {
#pragma unroll
    for (int r = 0; r < R; ++r) prev[r] = gld(wdst, base + r * NT + tid);
  }

  rb_apply_tile_b<L>(S, P, tid, ab, out);

  // ---- remaining cross-tile terms (global, L2/MALL-served), four registers at a time ----
  for (int f = 1; f < ((ab & 4) ? 0 : n_fh); ++f) {
    const DFlip F = S.fh[f];
    const bool v = par32(hg & F.tile_xor);
    const double cr = v ? F.re1 : F.re0, ci = v ? F.im1 : F.im0;
    const gd2* src = gptr(tile_ptr(P, win_role, hg ^ F.tile_xor));
#pragma unroll
    for (int hr4 = 0; hr4 < R; hr4 += 4) {
      double2 sv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = gld(src, (uint32_t)((hr4 + r) * NT + tid) ^ F.mask_lo);
#pragma unroll
      for (int r = 0; r < 4; ++r) out[hr4 + r] = cmad(out[hr4 + r], cr, ci, sv[r]);
    }
  }
  for (int p = 0; p < ((ab & 4) ? 0 : n_ph); ++p) {
    const DPair Q = S.ph[p];
    const int hpar = par32(hg & Q.tile_xor);
    if (Q.mask_lo == 0u && hpar) continue;  // both bits above the tile: uniform condition
    const gd2* src = gptr(tile_ptr(P, win_role, hg ^ Q.tile_xor));
#pragma unroll
    for (int hr4 = 0; hr4 < R; hr4 += 4) {
      double2 sv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = gld(src, (uint32_t)((hr4 + r) * NT + tid) ^ Q.mask_lo);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t x = (uint32_t)((hr4 + r) * NT + tid);
        const double g = ((__popc(x & Q.mask_lo) + hpar) & 1) ? 0.0 : Q.g;
        out[hr4 + r].x = fma(g, sv[r].x, out[hr4 + r].x);
        out[hr4 + r].y = fma(g, sv[r].y, out[hr4 + r].y);
      }
    }
  }

  // ---- recurrence + accumulation ----
  const bool rd_acc = rd && C.upd;
  double2 accv[R];
  if (rd_acc) {
#pragma unroll
    for (int r = 0; r < R; ++r) accv[r] = gld(acc_b, base + r * NT + tid);
  }
  const double scale = MODE == MODE_GEN ? 2.0 * P.s1 : P.s1;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const size_t x = base + r * NT + tid;
    const double2 own = S.w[r * NT + tid];
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
                        double* partial, hipStream_t st, int n_out, size_t out_stride, int xq) {
  hipLaunchKernelGGL((k_obs<L>), dim3(n_items, n_out), dim3(Geo<L>::NT), 0, st, probs, items, bsel,
                     partial, out_stride, xq);
  return hipGetLastError();
}

// <a|b> pieces for dse_energy: per block sum Re(conj(a) b) and sum |a|^2 over a grid-stride
// range (fixed grid, fixed order: bitwise deterministic).
__global__ void __launch_bounds__(256)
k_dot(const double2* __restrict__ a, const double2* __restrict__ b, size_t n, double* __restrict__ partial) {
  __shared__ double s_red[4][2];
  const gd2* ga = gptr(a);
  const gd2* gb = gptr(b);
  double e = 0.0, q = 0.0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const double2 x = gld(ga, i), y = gld(gb, i);
    e += x.x * y.x + x.y * y.y;
    q += x.x * x.x + x.y * x.y;
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    e += __shfl_xor(e, off, 64);
    q += __shfl_xor(q, off, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_red[threadIdx.x >> 6][0] = e;
    s_red[threadIdx.x >> 6][1] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[2 * blockIdx.x] = s_red[0][0] + s_red[1][0] + s_red[2][0] + s_red[3][0];
    partial[2 * blockIdx.x + 1] = s_red[0][1] + s_red[1][1] + s_red[2][1] + s_red[3][1];
  }
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
                      double* partial, hipStream_t st, int n_out, size_t out_stride, int xq) {
  if (n_items <= 0 || n_out <= 0) return hipSuccess;
  if (n_out > 1 && bsel >= 3) return hipErrorInvalidValue;
  switch (L) {
#define X(l) \
  case l: return launch_obs_L<l>(probs, items, n_items, bsel, partial, st, n_out, out_stride, xq);
    DSE_TILE_CASES(X)
#undef X
    default: return hipErrorInvalidValue;
  }
}

// one basis state per register: grid.y = entry, grid-stride over its amplitudes (16-B stores)
__global__ void __launch_bounds__(256) k_basis_init(const BasisInit* __restrict__ list) {
  const BasisInit e = list[blockIdx.y];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < e.n; i += stride)
    e.ptr[i] = make_double2((int64_t)i == e.one_at ? 1.0 : 0.0, 0.0);
}

hipError_t launch_basis_init(const BasisInit* list, int n_entries, uint64_t max_amps, hipStream_t st) {
  if (n_entries <= 0) return hipSuccess;
  if (n_entries > 65535) return hipErrorInvalidValue;
  const uint64_t blocks = std::min<uint64_t>((max_amps + 255) / 256, 2048);
  hipLaunchKernelGGL(k_basis_init, dim3((unsigned)std::max<uint64_t>(blocks, 1), n_entries), dim3(256), 0, st, list);
  return hipGetLastError();
}

hipError_t launch_dot(const double2* a, const double2* b, size_t n, double* partial, int blocks,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_dot, dim3(blocks), dim3(256), 0, st, a, b, n, partial);
  return hipGetLastError();
}

}  // namespace dse
