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
// The 2^n state lives in HBM; one H application is a few streaming passes over LDS tiles of 2^WL
// amplitudes (WL = 12 or 13).  Tile bits are split into groups (WhtGroup): group 0 = global bits
// 0..WL-1, high groups = up to WL-2 high bits each, completed to WL tile bits by the lowest c
// "carried" global bits.  The transform over all bits is the product of the groups' transforms:
//   FIRST  (group 0)          w -> A = W0 w,  B = W0 S^+ w            read 16, write 32 B/amp
//   FWD    (groups 1..G-2)    A, B -> W_g A, W_g B                    read 32, write 32
//   MID    (group G-1)        A -> W_g D_X W_g A,  B -> W_g D_Y W_g B  read 32, write 32
//   INV    (groups G-2..1)    as FWD
//   FINAL  (group 0)          out = D_Z w + W0 A + S W0 B, then the Chebyshev epilogue
//
// In a tile, thread t of 2^(WL-4) owns 16 amplitudes; the tile bits tau are spread over a
// register index r (4 bits at base b) and the thread index in three layouts,
//   A  b = WL-4   (global loads)      B  b = WL-8   (global stores)      C  b = WL-12
//   tau = (t & (2^b - 1)) | r << b | (t >> b) << (b + 4),
// and a layout change is one LDS transpose (write, barrier, read).  Butterflies run on register
// bits, plus tile bit 0 across neighbouring lanes by DPP in layout C when WL = 13.  A forward
// transform visits A -> C -> B (skipping layouts without active bits) and stores from B, whose
// lanes still cover runs of 16-32 consecutive amplitudes; MID comes back B -> C -> A.  LDS slots:
// tau for A <-> B, tau + K (tau >> S) for transposes touching C (K, S = 2, 5 at WL = 13 and 1, 4
// at WL = 12): conflict-free ds_write_b128 / ds_read_b128 except the C -> A read at WL = 12
// (2-way), and separable, slot = f(t) + g(r): one base address per thread, immediate offsets.
// WL = 12 tiles (64 KiB) fit two workgroups per CU, so one workgroup's loads overlap the other's
// transposes; WL = 13 needs fewer passes below 25 qubits.
#include <algorithm>

#include "dse_device.h"
#include "dse_wht.h"

namespace dse {
namespace {

constexpr int WR = 16;

template <int WL>
struct WG {
  static constexpr int T = 1 << WL;
  static constexpr int NT = 1 << (WL - 4);
  static constexpr int LGNT = WL - 4;
  static constexpr int PK = WL == 13 ? 2 : 1;  // slot pad of transposes touching layout C
  static constexpr int PS = WL == 13 ? 5 : 4;
  static constexpr int SLOTS = T + PK * ((T - 1) >> PS) + 1;
};

template <int WL>
__host__ __device__ constexpr int rbase(int lay) { return WL - 4 - 4 * lay; }
template <int WL>
__host__ __device__ constexpr int tau_of(int lay, int r, int t) {
  return (t & ((1 << rbase<WL>(lay)) - 1)) | (r << rbase<WL>(lay)) | ((t >> rbase<WL>(lay)) << (rbase<WL>(lay) + 4));
}
template <int WL>
__host__ __device__ constexpr int reg_tbit(int lay, int i) { return rbase<WL>(lay) + i; }
template <int WL>
__host__ __device__ constexpr int thr_tbit(int lay, int j) { return j < rbase<WL>(lay) ? j : j + 4; }
template <int WL, bool PAD>
__host__ __device__ constexpr int slot(int tau) { return PAD ? tau + WG<WL>::PK * (tau >> WG<WL>::PS) : tau; }

// register mask of the bits a layout transforms in a group with c carried bits
template <int WL>
__device__ __forceinline__ int active_mask(int lay, int c) {
  int m = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (reg_tbit<WL>(lay, i) >= c) m |= 1 << i;
  return m;
}
// layouts a forward transform visits after A: C holds bits rbase(2).., B bits rbase(1)..
template <int WL>
__device__ __forceinline__ bool has_c(int c) { return c < rbase<WL>(2) + 4; }
template <int WL>
__device__ __forceinline__ bool has_b(int c) { return c < rbase<WL>(1) + 4; }

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
// butterfly on thread bit 0 (tile bit 0 in layout C at WL = 13)
__device__ __forceinline__ void lane0_wht(double2* v, int tid) {
  const double sg = (tid & 1) ? -1.0 : 1.0;
#pragma unroll
  for (int r = 0; r < WR; ++r) {
    const double px = lane_xor1(v[r].x), py = lane_xor1(v[r].y);
    v[r].x = fma(sg, v[r].x, px);
    v[r].y = fma(sg, v[r].y, py);
  }
}

template <int WL, int FROM, int TO>
__device__ __forceinline__ void transpose(double2* lds, double2* v, int tid) {
  constexpr bool PAD = FROM == 2 || TO == 2;
  __syncthreads();  // the previous transpose's reads are done
  double2* wp = lds + slot<WL, PAD>(tau_of<WL>(FROM, 0, tid));
#pragma unroll
  for (int r = 0; r < WR; ++r) wp[slot<WL, PAD>(tau_of<WL>(FROM, r, 0))] = v[r];
  __syncthreads();
  const double2* rp = lds + slot<WL, PAD>(tau_of<WL>(TO, 0, tid));
#pragma unroll
  for (int r = 0; r < WR; ++r) v[r] = rp[slot<WL, PAD>(tau_of<WL>(TO, r, 0))];
}

// The same layout change through half the LDS: the real parts, then the imaginary parts, each a
// ds_write_b64 / ds_read_b64 transpose of 8-byte slots (the slot map is conflict-free for these
// too: 4 LDS-array cycles per write, 2 per read, every transpose at WL = 13).  A 13-bit tile then
// takes 68 KiB, so two workgroups share a CU and one's HBM traffic runs under the other's
// transposes (option wht_half).
template <int WL, int FROM, int TO>
__device__ __forceinline__ void transpose_h(double* lds, double2* v, int tid) {
  constexpr bool PAD = FROM == 2 || TO == 2;
  asm volatile("" : "+v"(tid));  // the LDS bases are computed here, not held from kernel entry
  double* wp = lds + slot<WL, PAD>(tau_of<WL>(FROM, 0, tid));
  const double* rp = lds + slot<WL, PAD>(tau_of<WL>(TO, 0, tid));
  __syncthreads();  // the previous transpose's reads are done
#pragma unroll
  for (int r = 0; r < WR; ++r) wp[slot<WL, PAD>(tau_of<WL>(FROM, r, 0))] = v[r].x;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < WR; ++r) v[r].x = rp[slot<WL, PAD>(tau_of<WL>(TO, r, 0))];
  __syncthreads();
#pragma unroll
  for (int r = 0; r < WR; ++r) wp[slot<WL, PAD>(tau_of<WL>(FROM, r, 0))] = v[r].y;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < WR; ++r) v[r].y = rp[slot<WL, PAD>(tau_of<WL>(TO, r, 0))];
}

template <int WL, bool H, int FROM, int TO>
__device__ __forceinline__ void xpose(void* lds, double2* v, int tid) {
  if constexpr (H)
    transpose_h<WL, FROM, TO>((double*)lds, v, tid);
  else
    transpose<WL, FROM, TO>((double2*)lds, v, tid);
}

template <int WL>
__device__ __forceinline__ void layout_wht(double2* v, int lay, int c, int tid) {
  reg_wht(v, active_mask<WL>(lay, c));
  if (WL == 13 && lay == 2 && c == 0) lane0_wht(v, tid);
}
// forward transform of a group (c carried bits) from layout A; returns the layout it ends in
template <int WL, bool H = false>
__device__ __forceinline__ int tile_fwd(void* lds, double2* v, int c, int tid) {
  layout_wht<WL>(v, 0, c, tid);
  if (!has_b<WL>(c)) return 0;
  if (has_c<WL>(c)) {
    xpose<WL, H, 0, 2>(lds, v, tid);
    layout_wht<WL>(v, 2, c, tid);
    xpose<WL, H, 2, 1>(lds, v, tid);
  } else {
    xpose<WL, H, 0, 1>(lds, v, tid);
  }
  layout_wht<WL>(v, 1, c, tid);
  return 1;
}
// the same butterflies from layout `last` (tile_fwd's result) back to layout A
template <int WL, bool H = false>
__device__ __forceinline__ void tile_back(void* lds, double2* v, int c, int last, int tid) {
  if (last == 1) {
    layout_wht<WL>(v, 1, c, tid);
    if (has_c<WL>(c)) {
      xpose<WL, H, 1, 2>(lds, v, tid);
      layout_wht<WL>(v, 2, c, tid);
      xpose<WL, H, 2, 0>(lds, v, tid);
    } else {
      xpose<WL, H, 1, 0>(lds, v, tid);
    }
  }
  layout_wht<WL>(v, 0, c, tid);
}

template <int WL>
struct WhtShared {
  double2 w[WG<WL>::SLOTS];
  double f[2][WL + 1];  // MID: D_X, D_Y fields per tile bit + constant; FINAL: D_Z (z convention)
};
template <int WL>
struct WhtSharedH {  // half-LDS passes (transpose_h)
  double w[WG<WL>::SLOTS];
  double f[2][WL + 1];
};

// size of one pair form in WhtProb::qtab
template <int WL>
constexpr int kQForm = 5 * WG<WL>::NT + WR;

__device__ __forceinline__ double zsign(uint64_t v, int b) { return ((v >> b) & 1ull) ? -1.0 : 1.0; }

// linear part f[WL] + sum_q f[q] z_q of this thread's amplitudes in layout lay:
// lt + sum_i lh[i] z_i(r)
template <int WL>
__device__ __forceinline__ void lin_parts(const double* f, int lay, int tid, double& lt, double* lh) {
  lt = f[WL];
#pragma unroll
  for (int j = 0; j < WG<WL>::LGNT; ++j) lt += f[thr_tbit<WL>(lay, j)] * zsign(tid, j);
#pragma unroll
  for (int i = 0; i < 4; ++i) lh[i] = f[reg_tbit<WL>(lay, i)];
}
// pair form of this thread from qtab: qt + sum_i qh[i] z_i(r) + zr[r]
template <int WL>
__device__ __forceinline__ void pair_parts(const double* form, int tid, double& qt, double* qh) {
  const gdbl* q = gptr(form);
  qt = q[tid];
#pragma unroll
  for (int i = 0; i < 4; ++i) qh[i] = q[(1 + i) * WG<WL>::NT + tid];
}

__device__ __forceinline__ double quad_at(double zt, const double* hr, double zr_r, double sg, int r) {
  double d = zt + sg * zr_r;
#pragma unroll
  for (int i = 0; i < 4; ++i) d += ((r >> i) & 1 ? -1.0 : 1.0) * hr[i];
  return d;
}

// an opaque copy: values derived from it are recomputed, not kept live across a transform
__device__ __forceinline__ uint64_t launder(uint64_t x) {
  asm volatile("" : "+v"(x));
  return x;
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

// global indices of this thread's amplitudes in layout lay: xo | xt | xr[r]
template <int WL>
struct LayIdx {
  uint64_t xt;
  uint64_t rb[4];  // global index bit of each register bit (wave-uniform: scalar registers)
  __device__ __forceinline__ LayIdx(const WhtGroup& G, int lay, int tid, uint64_t xo) {
    xt = xo;
    for (int j = 0; j < WG<WL>::LGNT; ++j) xt |= (uint64_t)((tid >> j) & 1) << G.pos[thr_tbit<WL>(lay, j)];
#pragma unroll
    for (int i = 0; i < 4; ++i) rb[i] = uint64_t(1) << G.pos[reg_tbit<WL>(lay, i)];
  }
  __device__ __forceinline__ uint64_t operator[](int r) const {
    uint64_t x = xt;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if ((r >> i) & 1) x |= rb[i];
    return x;
  }
};

// group 0 (pos = identity): global index = o << WL | tau, the register part an immediate
template <int WL>
struct LayIdx0 {
  uint64_t xt;
  int lay;
  __device__ __forceinline__ LayIdx0(int lay_, int tid, uint64_t o) : lay(lay_) {
    xt = (o << WL) | (uint64_t)tau_of<WL>(lay, 0, tid);
  }
  __device__ __forceinline__ uint64_t operator[](int r) const { return xt | (uint64_t)tau_of<WL>(lay, r, 0); }
};

// input vector of term k (buffer roles of k_step_rb)
__device__ __forceinline__ int win_role(int mode, int k, int q) {
  if (mode == MODE_APPLY) return 0;
  if (mode == MODE_FIRST) return q ? 2 : 0;
  return ((k - 1) & 1) ? 1 : (q ? 2 : 0);
}

template <int WL, int PASS, int MODE, int VSEL>
__global__ void __launch_bounds__(WG<WL>::NT)
k_wht(const WhtProb* __restrict__ probs, const DevProb* __restrict__ dprobs, const int2* __restrict__ items,
      int g, int k, int q, int set) {
  __shared__ WhtShared<WL> S;
  const int2 it = items[blockIdx.x];
  const WhtProb& W = probs[it.x];
  const DevProb& P = dprobs[it.x];
  const int tid = threadIdx.x;
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform
  const WhtGroup& G = W.grp[g];
  const uint64_t o = (uint64_t)(uint32_t)it.y;  // outer index of the tile
  const uint64_t xo = outer_bits(G, o);
  double2 v[WR];
  if (PASS == WHT_FIRST) {
    const LayIdx0<WL> ia(0, tid, o);
    const gd2* win = gptr((const double2*)P.buf[win_role(MODE, k, q)]);
    double2 u[WR];
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      v[r] = gld(win, ia[r]);
      u[r] = mul_ipow(v[r], -(__popcll(ia[r]) + W.phase0));  // S^+ of every qubit
    }
    tile_fwd<WL>(S.w, v, 0, tid);  // ends in layout B
    const LayIdx0<WL> is(1, tid, o);
    gd2* A = gptr(W.vec_a);
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(A, is[r], v[r]);
    tile_fwd<WL>(S.w, u, 0, tid);
    gd2* B = gptr(W.vec_b);
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(B, is[r], u[r]);
    return;
  }

  const LayIdx<WL> ia(G, 0, tid, xo);  // loads of the FWD / INV / MID passes
  if (PASS == WHT_FWD || PASS == WHT_INV) {
    const int last = has_b<WL>(G.c) ? 1 : 0;
    const LayIdx<WL> is(G, last, tid, xo);
    // both vectors' loads in flight from the start: B's latency hides under A's transposes
    // (VSEL: bit 0 the X-branch vector A, bit 1 the Y-branch vector B -- partitioned registers
    // transform them in separate launches so one vector's index swap overlaps the other's pass;
    // compile-time, so the tile arrays stay in registers)
    double2 vb[WR];
    gd2* XA = gptr(W.vec_a);
    gd2* XB = gptr(W.vec_b);
    if constexpr ((VSEL & 1) != 0) {
#pragma unroll
      for (int r = 0; r < WR; ++r) v[r] = gld(XA, ia[r]);
    }
    if constexpr ((VSEL & 2) != 0) {
#pragma unroll
      for (int r = 0; r < WR; ++r) vb[r] = gld(XB, ia[r]);
    }
    if constexpr ((VSEL & 1) != 0) {
      tile_fwd<WL>(S.w, v, G.c, tid);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(XA, is[r], v[r]);
    }
    if constexpr ((VSEL & 2) != 0) {
      tile_fwd<WL>(S.w, vb, G.c, tid);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(XB, is[r], vb[r]);
    }
    return;
  }

  if (PASS == WHT_MID) {
    const int last = has_b<WL>(G.c) ? 1 : 0;
    // both vectors in flight from the start (the diagonal needs no staged couplings: the pair
    // form is a per-thread table, the linear parts one 256-B row per tile)
    double2 vb[WR];
    gd2* XA = gptr(W.vec_at);
    gd2* XB = gptr(W.vec_bt);
    if constexpr ((VSEL & 1) != 0) {
#pragma unroll
      for (int r = 0; r < WR; ++r) v[r] = gld(XA, ia[r]);
    }
    if constexpr ((VSEL & 2) != 0) {
#pragma unroll
      for (int r = 0; r < WR; ++r) vb[r] = gld(XB, ia[r]);
    }
    if (tid < 32) {
      const double c = gptr((const double*)W.xytab)[o * 32 + tid];
      if (tid <= WL) S.f[0][tid] = c;
      else if (tid >= 16 && tid <= 16 + WL) S.f[1][tid - 16] = c;
    }
    double qt, qh[4];
    pair_parts<WL>(W.qtab, tid, qt, qh);
    const double* zr = W.qtab + 5 * WG<WL>::NT;
    __syncthreads();  // S.f
    // D_X = lin_X + Q, D_Y = lin_Y - Q; each branch's pieces formed when it needs them
    auto diag = [&](double2* x, int vec) {
      const double sg = vec == 0 ? 1.0 : -1.0;
      double lt, lh[4];
      lin_parts<WL>(S.f[vec], last, tid, lt, lh);
      lt += sg * qt;
#pragma unroll
      for (int i = 0; i < 4; ++i) lh[i] += sg * qh[i];
#pragma unroll
      for (int r = 0; r < WR; ++r) {
        const double d = quad_at(lt, lh, zr[r], sg, r);
        x[r].x *= d;
        x[r].y *= d;
      }
    };
    if constexpr ((VSEL & 1) != 0) {
      tile_fwd<WL>(S.w, v, G.c, tid);
      diag(v, 0);
      tile_back<WL>(S.w, v, G.c, last, tid);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(XA, ia[r], v[r]);
    }
    if constexpr ((VSEL & 2) != 0) {
      tile_fwd<WL>(S.w, vb, G.c, tid);
      diag(vb, 1);
      tile_back<WL>(S.w, vb, G.c, last, tid);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(XB, ia[r], vb[r]);
    }
    return;
  }

  // ---- FINAL (group 0 tile = ordinary tile h): out = D_Z w + W0 A + S W0 B, then the recurrence;
  // FINAL_NEXT then runs the next term's FIRST on the new w_k while it is in registers: A = W0 w_k,
  // B = W0 S^+ w_k, transformed from layout B back to A (the butterflies of a transform commute,
  // so the order only changes the rounding), saving FIRST's read of w_k and its launch
  if (PASS == WHT_FINAL || PASS == WHT_FINAL_NEXT) {
    constexpr int last = 1;  // group 0 ends every forward transform in layout B
    const LayIdx0<WL> ia0(0, tid, o);
    // D_Z in the z convention: fields F_i / 2 and constant C(h) - beta per tile (ztab), the in-tile
    // zz / 4 form per thread (qtab form 1)
    if (tid <= WL) {
      const double c = gptr((const double*)W.ztab)[o * 16 + tid];
      S.f[0][tid] = tid == WL ? (MODE == MODE_APPLY ? c : c - P.beta) : 0.5 * c;
    }
    double2 out[WR];
    {
      const gd2* B = gptr((const double2*)W.vec_b);
      const gd2* A = gptr((const double2*)W.vec_a);
#pragma unroll
      for (int r = 0; r < WR; ++r) out[r] = gld(B, ia0[r]);
#pragma unroll
      for (int r = 0; r < WR; ++r) v[r] = gld(A, ia0[r]);
    }
    tile_fwd<WL>(S.w, out, 0, tid);
    tile_fwd<WL>(S.w, v, 0, tid);
    const LayIdx0<WL> is(last, tid, o);
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      const double2 s = mul_ipow(out[r], __popcll(is[r]) + W.phase0);  // S of every qubit
      out[r].x = s.x + v[r].x;
      out[r].y = s.y + v[r].y;
    }
    // D_Z(x) = zt + sum_i hr[i] z_i(r) + zr[r]  (S.f visible: the transposes' barriers)
    double zt, hr[4];
    {
      double lt, lh[4], qt, qh[4];
      lin_parts<WL>(S.f[0], last, tid, lt, lh);
      pair_parts<WL>(W.qtab + kQForm<WL>, tid, qt, qh);
      zt = lt + qt;
#pragma unroll
      for (int i = 0; i < 4; ++i) hr[i] = lh[i] + qh[i];
    }
    const double* zrz = W.qtab + kQForm<WL> + 5 * WG<WL>::NT;
    const gd2* win = gptr((const double2*)P.buf[win_role(MODE, k, q)]);
    gd2* psi_b = gptr(P.buf[q ? 2 : 0]);
    gd2* acc_b = gptr(P.buf[q ? 0 : 2]);
    gd2* scr_b = gptr(P.buf[1]);
    CoefK C = {};
    if (MODE != MODE_APPLY) C = coef_at(coef_row(P, set, 0), MODE == MODE_FIRST ? 1 : k);
    gd2* wdst = (MODE == MODE_GEN && !(k & 1)) ? psi_b : scr_b;  // GEN: holds w_{k-2}
    const double scale = MODE == MODE_GEN ? 2.0 * P.s1 : P.s1;
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      const double2 own = gld(win, is[r]);
      const double d = quad_at(zt, hr, zrz[r], 1.0, r);
      out[r].x = fma(d, own.x, out[r].x);
      out[r].y = fma(d, own.y, out[r].y);
      const double2 w = step_epilogue<MODE>(is[r], out[r], own, scale, wdst, acc_b, C, 0);
      if constexpr (PASS == WHT_FINAL_NEXT) out[r] = w;
    }
    if constexpr (PASS == WHT_FINAL_NEXT && MODE != MODE_APPLY) {
      if (k < P.degree) {  // uniform: the next term exists for this register
        asm volatile("" : : : "memory");  // the epilogue's stores first: its registers free for v
        int t2 = tid;  // indices recomputed from an opaque copy, not held from the kernel's start
        asm volatile("" : "+v"(t2));
        {
          const uint64_t xb = (o << WL) | (uint64_t)tau_of<WL>(last, 0, t2);
#pragma unroll
          for (int r = 0; r < WR; ++r)  // S^+
            v[r] = mul_ipow(out[r], -(__popcll(xb | (uint64_t)tau_of<WL>(last, r, 0)) + W.phase0));
        }
        tile_back<WL>(S.w, out, 0, last, tid);  // B -> C -> A
        {
          const uint64_t xa = (o << WL) | (uint64_t)tau_of<WL>(0, 0, t2);
          gd2* A = gptr(W.vec_a);
#pragma unroll
          for (int r = 0; r < WR; ++r) gst(A, xa | (uint64_t)tau_of<WL>(0, r, 0), out[r]);
        }
        tile_back<WL>(S.w, v, 0, last, tid);
        {
          const uint64_t xa = launder((o << WL) | (uint64_t)tau_of<WL>(0, 0, t2));
          gd2* B = gptr(W.vec_b);
#pragma unroll
          for (int r = 0; r < WR; ++r) gst(B, xa | (uint64_t)tau_of<WL>(0, r, 0), v[r]);
        }
      }
    }
  }
}

// Persistent MID (option wht_persist bit 1): gridDim.x workgroups loop over the items; a vector's
// next tile is loaded as soon as its current tile is stored, so the loads of A(o + grid) land while
// B(o) is transformed and those of B(o + grid) while A(o + grid) is -- one workgroup per CU keeps
// HBM busy through its LDS transposes (the one-tile-per-workgroup form leaves them unoverlapped).
template <int WL, int MODE, int VSEL>
__global__ void __launch_bounds__(WG<WL>::NT)
k_wht_mid_p(const WhtProb* __restrict__ probs, const DevProb* __restrict__ dprobs, const int2* __restrict__ items,
            int n_items, int g, int k) {
  __shared__ WhtShared<WL> S;
  const int tid = threadIdx.x;
  int i = blockIdx.x;
  if (i >= n_items) return;
  auto lidx = [&](int item) {
    const int2 it = items[item];
    const WhtGroup& G = probs[it.x].grp[g];
    return LayIdx<WL>(G, 0, tid, outer_bits(G, (uint64_t)(uint32_t)it.y));
  };
  double2 v[WR], vb[WR];
  auto load_a = [&](int item) {
    const LayIdx<WL> ia = lidx(item);
    const gd2* XA = gptr((const double2*)probs[items[item].x].vec_at);
#pragma unroll
    for (int r = 0; r < WR; ++r) v[r] = gld(XA, ia[r]);
  };
  auto load_b = [&](int item) {
    const LayIdx<WL> ia = lidx(item);
    const gd2* XB = gptr((const double2*)probs[items[item].x].vec_bt);
#pragma unroll
    for (int r = 0; r < WR; ++r) vb[r] = gld(XB, ia[r]);
  };
  if constexpr ((VSEL & 1) != 0) load_a(i);
  if constexpr ((VSEL & 2) != 0) load_b(i);
  for (; i < n_items; i += gridDim.x) {
    const int2 it = items[i];
    const WhtProb& W = probs[it.x];
    const int inext = i + (int)gridDim.x;
    // a problem whose series has ended (k past its degree) is transformed but not stored: one code
    // path, so the next tile's loads stay where they are
    const bool live = !(MODE == MODE_GEN && k > dprobs[it.x].degree);
    const WhtGroup& G = W.grp[g];
    const uint64_t o = (uint64_t)(uint32_t)it.y;
    const int last = has_b<WL>(G.c) ? 1 : 0;
    const LayIdx<WL> ia(G, 0, tid, outer_bits(G, o));
    // S.f of this tile: the previous tile's last reads of S.f came before its back transforms,
    // whose transposes hold workgroup barriers
    if (tid < 32) {
      const double c = gptr((const double*)W.xytab)[o * 32 + tid];
      if (tid <= WL) S.f[0][tid] = c;
      else if (tid >= 16 && tid <= 16 + WL) S.f[1][tid - 16] = c;
    }
    double qt, qh[4];
    pair_parts<WL>(W.qtab, tid, qt, qh);
    const double* zr = W.qtab + 5 * WG<WL>::NT;
    __syncthreads();  // S.f
    auto diag = [&](double2* x, int vec) {
      const double sg = vec == 0 ? 1.0 : -1.0;
      double lt, lh[4];
      lin_parts<WL>(S.f[vec], last, tid, lt, lh);
      lt += sg * qt;
#pragma unroll
      for (int q = 0; q < 4; ++q) lh[q] += sg * qh[q];
#pragma unroll
      for (int r = 0; r < WR; ++r) {
        const double d = quad_at(lt, lh, zr[r], sg, r);
        x[r].x *= d;
        x[r].y *= d;
      }
    };
    if constexpr ((VSEL & 1) != 0) {
      gd2* XA = gptr(W.vec_at);
      tile_fwd<WL>(S.w, v, G.c, tid);
      diag(v, 0);
      tile_back<WL>(S.w, v, G.c, last, tid);
      if (live) {
#pragma unroll
        for (int r = 0; r < WR; ++r) gst(XA, ia[r], v[r]);
      }
      if (inext < n_items) load_a(inext);
    }
    if constexpr ((VSEL & 2) != 0) {
      gd2* XB = gptr(W.vec_bt);
      tile_fwd<WL>(S.w, vb, G.c, tid);
      diag(vb, 1);
      tile_back<WL>(S.w, vb, G.c, last, tid);
      if (live) {
#pragma unroll
        for (int r = 0; r < WR; ++r) gst(XB, ia[r], vb[r]);
      }
      if (inext < n_items) load_b(inext);
    }
  }
}

// Half-LDS passes (option wht_half): FIRST, FWD / INV and MID with one vector in registers at a
// time and the transposes through transpose_h, so two workgroups (at most 128 VGPRs each) share a
// CU and one's loads and stores run under the other's transposes -- the one-workgroup-per-CU form
// leaves each tile's compute unoverlapped apart from the second vector's loads.  FIRST reads the
// tile of w twice (A from it, then B from S^+ w: the second read mostly from the caches) instead
// of holding both vectors.  Same arithmetic, same order: bitwise identical to k_wht.

// tile_fwd / tile_back with the layout path fixed at compile time (PATH 2: A -> C -> B, 1: A -> B,
// 0: no transpose; tile_path(c)), so the register arrays take no copies where paths would merge
__host__ __device__ constexpr int tile_path13(int c) { return c < 5 ? 2 : (c < 9 ? 1 : 0); }
template <int WL, int PATH>
__device__ __forceinline__ void tile_fwd_p(double* lds, double2* v, int c, int tid) {
  layout_wht<WL>(v, 0, c, tid);
  if constexpr (PATH == 2) {
    transpose_h<WL, 0, 2>(lds, v, tid);
    layout_wht<WL>(v, 2, c, tid);
    transpose_h<WL, 2, 1>(lds, v, tid);
  } else if constexpr (PATH == 1) {
    transpose_h<WL, 0, 1>(lds, v, tid);
  }
  if constexpr (PATH > 0) layout_wht<WL>(v, 1, c, tid);
}
template <int WL, int PATH>
__device__ __forceinline__ void tile_back_p(double* lds, double2* v, int c, int tid) {
  if constexpr (PATH > 0) layout_wht<WL>(v, 1, c, tid);
  if constexpr (PATH == 2) {
    transpose_h<WL, 1, 2>(lds, v, tid);
    layout_wht<WL>(v, 2, c, tid);
    transpose_h<WL, 2, 0>(lds, v, tid);
  } else if constexpr (PATH == 1) {
    transpose_h<WL, 1, 0>(lds, v, tid);
  }
  layout_wht<WL>(v, 0, c, tid);
}

// offset of register r from a LayIdx's per-thread part (wave-uniform bits)
template <int WL>
__device__ __forceinline__ uint64_t roff(const LayIdx<WL>& L, int r) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if ((r >> i) & 1) x |= L.rb[i];
  return x;
}

// FWD / INV / MID of one vector through half the LDS (k_wht_h), layout path fixed
template <int WL, int PASS, int PATH>
__device__ __forceinline__ void wht_h_vec(WhtSharedH<WL>& S, const WhtProb& W, const WhtGroup& G, uint64_t o,
                                          int vec, int tid) {
  constexpr int last = PATH > 0 ? 1 : 0;
  double2 v[WR];
  const uint64_t xo = outer_bits(G, o);
  gd2* X = gptr(PASS == WHT_MID ? (vec == 0 ? W.vec_at : W.vec_bt) : (vec == 0 ? W.vec_a : W.vec_b));
  {
    const LayIdx<WL> ia(G, 0, tid, launder(xo));
#pragma unroll
    for (int r = 0; r < WR; ++r) v[r] = gld(X, ia.xt | roff<WL>(ia, r));
  }
  double qt = 0.0, qh[4] = {0.0, 0.0, 0.0, 0.0};
  if constexpr (PASS == WHT_MID) pair_parts<WL>(W.qtab, tid, qt, qh);  // in flight under the transform
  tile_fwd_p<WL, PATH>(S.w, v, G.c, tid);
  if constexpr (PASS == WHT_MID) {
    if constexpr (PATH == 0) __syncthreads();  // no transpose ran: S.f
    const double* zr = W.qtab + 5 * WG<WL>::NT;
    const double sg = vec == 0 ? 1.0 : -1.0;
    double lt, lh[4];
    lin_parts<WL>(S.f[vec], last, tid, lt, lh);
    lt += sg * qt;
#pragma unroll
    for (int i = 0; i < 4; ++i) lh[i] += sg * qh[i];
#pragma unroll
    for (int r = 0; r < WR; ++r) {
      const double d = quad_at(lt, lh, zr[r], sg, r);
      v[r].x *= d;
      v[r].y *= d;
    }
    tile_back_p<WL, PATH>(S.w, v, G.c, tid);
    const LayIdx<WL> is(G, 0, tid, launder(xo));
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(X, is.xt | roff<WL>(is, r), v[r]);
  } else {
    const LayIdx<WL> is(G, last, tid, launder(xo));
#pragma unroll
    for (int r = 0; r < WR; ++r) gst(X, is.xt | roff<WL>(is, r), v[r]);
  }
}

template <int WL, int PASS, int MODE, int VSEL>
__global__ void __launch_bounds__(WG<WL>::NT, 4 * WG<WL>::NT / 512)  // two workgroups per CU: <= 128 VGPRs at WL = 13
k_wht_h(const WhtProb* __restrict__ probs, const DevProb* __restrict__ dprobs, const int2* __restrict__ items,
        int g, int k, int q, int set) {
  static_assert(WL == 13, "half-LDS passes: 13-bit tiles (12-bit tiles already fit two workgroups per CU)");
  __shared__ WhtSharedH<WL> S;
  const int2 it = items[blockIdx.x];
  const WhtProb& W = probs[it.x];
  const DevProb& P = dprobs[it.x];
  const int tid = threadIdx.x;
  if (MODE == MODE_GEN && k > P.degree) return;  // uniform
  const WhtGroup& G = W.grp[g];
  const uint64_t o = (uint64_t)(uint32_t)it.y;
  if constexpr (PASS == WHT_FIRST) {
    double2 v[WR];
    const uint64_t xa = (o << WL) | (uint64_t)tau_of<WL>(0, 0, tid);  // LayIdx0: x = xt | tau(lay, r, 0)
    const gd2* win = gptr((const double2*)P.buf[win_role(MODE, k, q)]);
#pragma unroll
    for (int r = 0; r < WR; ++r) v[r] = gld(win, xa | (uint64_t)tau_of<WL>(0, r, 0));
    tile_fwd_p<WL, 2>(S.w, v, 0, tid);
    {
      const uint64_t xs = launder((o << WL) | (uint64_t)tau_of<WL>(1, 0, tid));
      gd2* A = gptr(W.vec_a);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(A, xs | (uint64_t)tau_of<WL>(1, r, 0), v[r]);
    }
    {
      const uint64_t xb = launder(xa);
#pragma unroll
      for (int r = 0; r < WR; ++r) {
        const uint64_t x = xb | (uint64_t)tau_of<WL>(0, r, 0);
        v[r] = mul_ipow(gld(win, x), -(__popcll(x) + W.phase0));
      }
    }
    tile_fwd_p<WL, 2>(S.w, v, 0, tid);
    {
      const uint64_t xs = launder((o << WL) | (uint64_t)tau_of<WL>(1, 0, tid));
      gd2* B = gptr(W.vec_b);
#pragma unroll
      for (int r = 0; r < WR; ++r) gst(B, xs | (uint64_t)tau_of<WL>(1, r, 0), v[r]);
    }
  } else {
    if constexpr (PASS == WHT_MID) {
      if (tid < 32) {  // read after the first forward transform's barriers
        const double c = gptr((const double*)W.xytab)[o * 32 + tid];
        if (tid <= WL) S.f[0][tid] = c;
        else if (tid >= 16 && tid <= 16 + WL) S.f[1][tid - 16] = c;
      }
    }
    const int path = tile_path13(G.c);  // uniform
#pragma unroll
    for (int vec = 0; vec < 2; ++vec) {
      if (!((VSEL >> vec) & 1)) continue;
      if (path == 2)
        wht_h_vec<WL, PASS, 2>(S, W, G, o, vec, tid);
      else if (path == 1)
        wht_h_vec<WL, PASS, 1>(S, W, G, o, vec, tid);
      else
        wht_h_vec<WL, PASS, 0>(S, W, G, o, vec, tid);
    }
  }
}

// One thread per tile o: D_Z pieces of group-0 tile o (tile_diag_coeffs without beta) and the
// D_X / D_Y pieces of MID-group tile o:  F_q = lin(pos_q) + sum_i c(pos_q, opos_i) z_i,
// C = sum_i lin(opos_i) z_i + sum_{i<j} c(opos_i, opos_j) z_i z_j  (D_Y: lin_y, -c).
template <int WL>
__global__ void __launch_bounds__(256) k_wht_tables(const WhtProb* __restrict__ wp, const DevProb* __restrict__ dp,
                                                    int64_t tiles) {
  const int64_t o = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (o >= tiles) return;
  const WhtProb& W = *wp;
  const DevProb& P = *dp;
  const int n = W.n;
  // D_Z: global tile index (a shard's rank bits above its local tiles)
  const uint64_t hg = (uint64_t)P.h_base | (uint64_t)o;
  double* zt = W.ztab + o * 16;
  for (int i = 0; i < WL; ++i) {
    double f = P.field[i];
    for (int j = WL; j < n; ++j) f += P.zz[i * n + j] * (0.5 - (double)((hg >> (j - WL)) & 1));
    zt[i] = f;
  }
  double c = P.shift;
  for (int j = WL; j < n; ++j) {
    const double sj = 0.5 - (double)((hg >> (j - WL)) & 1);
    c += P.field[j] * sj;
    for (int i = WL; i < j; ++i) c += P.zz[i * n + j] * ((0.5 - (double)((hg >> (i - WL)) & 1)) * sj);
  }
  zt[WL] = c;
  for (int i = WL + 1; i < 16; ++i) zt[i] = 0.0;
  // D_X / D_Y of the MID group: outer bits (through gmap) and the rank-held bits are "outer"
  const WhtGroup& G = W.grp[W.n_groups - 1];
  const double* cq = W.cquad;
  int ob[kWhtMaxQubits];
  double oz[kWhtMaxQubits];
  int no = 0;
  for (int i = 0; i < G.n_outer; ++i) {
    ob[no] = W.gmap[G.opos[i]];
    oz[no++] = zsign(o, i);
  }
  for (int b = 0; b < n; ++b)
    if ((W.fix_mask >> b) & 1ull) {
      ob[no] = b;
      oz[no++] = zsign(W.fix_val, b);
    }
  double* xy = W.xytab + o * 32;
  for (int qb = 0; qb < WL; ++qb) {
    const int b = W.gmap[G.pos[qb]];
    double fx = W.lin_x[b], fy = W.lin_y[b];
    for (int i = 0; i < no; ++i) {
      const double v = cq[b * n + ob[i]] * oz[i];
      fx += v;
      fy -= v;
    }
    xy[qb] = fx;
    xy[16 + qb] = fy;
  }
  double cx = 0.0, cy = 0.0;
  for (int i = 0; i < no; ++i) {
    cx += W.lin_x[ob[i]] * oz[i];
    cy += W.lin_y[ob[i]] * oz[i];
    for (int j = i + 1; j < no; ++j) {
      const double v = cq[ob[i] * n + ob[j]] * (oz[i] * oz[j]);
      cx += v;
      cy -= v;
    }
  }
  xy[WL] = cx;
  xy[16 + WL] = cy;
  for (int i = WL + 1; i < 16; ++i) xy[i] = xy[16 + i] = 0.0;
}

// Tile-independent pair forms (WhtProb::qtab), one block per form, one thread per tile thread.
template <int WL>
__global__ void __launch_bounds__(512) k_wht_qtab(const WhtProb* __restrict__ wp, const DevProb* __restrict__ dp) {
  const WhtProb& W = *wp;
  const DevProb& P = *dp;
  const int form = blockIdx.x, tid = threadIdx.x, n = W.n;
  if (tid >= WG<WL>::NT) return;
  const WhtGroup& G = W.grp[form == 0 ? W.n_groups - 1 : 0];
  const int lay = form == 0 ? (has_b<WL>(G.c) ? 1 : 0) : 1;
  auto cpl = [&](int qa, int qb) -> double {  // coupling of tile bits qa != qb (z convention)
    if (form == 0) return W.cquad[W.gmap[G.pos[qa]] * n + W.gmap[G.pos[qb]]];
    const int a = qa < qb ? qa : qb, b = qa < qb ? qb : qa;
    return 0.25 * P.zz[a * n + b];
  };
  double qt = 0.0, qh[4] = {0.0, 0.0, 0.0, 0.0};
  for (int j = 0; j < WG<WL>::LGNT; ++j) {
    const double zj = zsign(tid, j);
    for (int i = j + 1; i < WG<WL>::LGNT; ++i)
      qt += cpl(thr_tbit<WL>(lay, j), thr_tbit<WL>(lay, i)) * zj * zsign(tid, i);
    for (int i = 0; i < 4; ++i) qh[i] += cpl(reg_tbit<WL>(lay, i), thr_tbit<WL>(lay, j)) * zj;
  }
  double* out = W.qtab + form * kQForm<WL>;
  out[tid] = qt;
  for (int i = 0; i < 4; ++i) out[(1 + i) * WG<WL>::NT + tid] = qh[i];
  if (tid < WR) {
    double v = 0.0;
    for (int a = 0; a < 4; ++a)
      for (int b = a + 1; b < 4; ++b) v += cpl(reg_tbit<WL>(lay, a), reg_tbit<WL>(lay, b)) * zsign(tid, a) * zsign(tid, b);
    out[5 * WG<WL>::NT + tid] = v;
  }
}

template <int WL, int PASS, int VSEL>
hipError_t launch_pass_v(int mode, const WhtProb* wp, const DevProb* dp, const int2* items, int n_items,
                         int g, int k, int q, int set, hipStream_t st) {
  const dim3 grid(n_items), block(WG<WL>::NT);
  if (mode == MODE_APPLY)
    hipLaunchKernelGGL((k_wht<WL, PASS, MODE_APPLY, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else if (mode == MODE_FIRST)
    hipLaunchKernelGGL((k_wht<WL, PASS, MODE_FIRST, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else
    hipLaunchKernelGGL((k_wht<WL, PASS, MODE_GEN, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  return hipGetLastError();
}

template <int WL, int PASS, int VSEL>
hipError_t launch_pass_h(int mode, const WhtProb* wp, const DevProb* dp, const int2* items, int n_items,
                         int g, int k, int q, int set, hipStream_t st) {
  const dim3 grid(n_items), block(WG<WL>::NT);
  if (mode == MODE_APPLY)
    hipLaunchKernelGGL((k_wht_h<WL, PASS, MODE_APPLY, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else if (mode == MODE_FIRST)
    hipLaunchKernelGGL((k_wht_h<WL, PASS, MODE_FIRST, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  else
    hipLaunchKernelGGL((k_wht_h<WL, PASS, MODE_GEN, VSEL>), grid, block, 0, st, wp, dp, items, g, k, q, set);
  return hipGetLastError();
}

// FIRST and FINAL always take both vectors; FWD / MID / INV one (vsel 1, 2) or both (3).  half:
// the half-LDS form (k_wht_h; not FINAL, which holds both transformed vectors)
template <int WL, int PASS>
hipError_t launch_pass(int mode, const WhtProb* wp, const DevProb* dp, const int2* items, int n_items,
                       int g, int k, int q, int set, int vsel, hipStream_t st, bool half = false) {
  if constexpr (PASS != WHT_FINAL && PASS != WHT_FINAL_NEXT && WL == 13) {
    if (half) {
      if constexpr (PASS == WHT_FIRST) {
        return launch_pass_h<WL, PASS, 3>(mode, wp, dp, items, n_items, g, k, q, set, st);
      } else {
        if (vsel == 3) return launch_pass_h<WL, PASS, 3>(mode, wp, dp, items, n_items, g, k, q, set, st);
        if (vsel == 1) return launch_pass_h<WL, PASS, 1>(mode, wp, dp, items, n_items, g, k, q, set, st);
        return launch_pass_h<WL, PASS, 2>(mode, wp, dp, items, n_items, g, k, q, set, st);
      }
    }
  }
  if constexpr (PASS == WHT_FIRST || PASS == WHT_FINAL || PASS == WHT_FINAL_NEXT) {
    return launch_pass_v<WL, PASS, 3>(mode, wp, dp, items, n_items, g, k, q, set, st);
  } else {
    if (vsel == 3) return launch_pass_v<WL, PASS, 3>(mode, wp, dp, items, n_items, g, k, q, set, st);
    if (vsel == 1) return launch_pass_v<WL, PASS, 1>(mode, wp, dp, items, n_items, g, k, q, set, st);
    return launch_pass_v<WL, PASS, 2>(mode, wp, dp, items, n_items, g, k, q, set, st);
  }
}

template <int WL, int VSEL>
hipError_t launch_mid_p(int mode, const WhtProb* wp, const DevProb* dp, const int2* items, int n_items, int g,
                        int k, int grid, hipStream_t st) {
  const dim3 gr(std::min(grid, n_items)), block(WG<WL>::NT);
  if (mode == MODE_APPLY)
    hipLaunchKernelGGL((k_wht_mid_p<WL, MODE_APPLY, VSEL>), gr, block, 0, st, wp, dp, items, n_items, g, k);
  else if (mode == MODE_FIRST)
    hipLaunchKernelGGL((k_wht_mid_p<WL, MODE_FIRST, VSEL>), gr, block, 0, st, wp, dp, items, n_items, g, k);
  else
    hipLaunchKernelGGL((k_wht_mid_p<WL, MODE_GEN, VSEL>), gr, block, 0, st, wp, dp, items, n_items, g, k);
  return hipGetLastError();
}

template <int WL>
hipError_t wht_part(int part, int mode, int n_groups, const WhtProb* wp, const DevProb* dp, const int2* items,
                    int n_items, int k, int q, int set, int vsel, hipStream_t st, int pgrid, int pmask) {
  hipError_t e = hipSuccess;
  // pmask: option wht_persist (bit 1 persistent MID) | option wht_half << 8 (bit 0 FIRST, bit 1
  // FWD / INV, bit 2 MID)
  const int half = (pmask >> 8) & 0xff;
  const bool fuse = (pmask >> 16) & 1;  // option wht_fuse: FINAL_NEXT, and no FIRST past term 1
  if (part == WHT_PART_MID && (half & 4))
    return launch_pass<WL, WHT_MID>(mode, wp, dp, items, n_items, n_groups - 1, k, q, set, vsel, st, true);
  if (part == WHT_PART_MID && pgrid > 0 && (pmask & 2)) {  // persistent MID
    const int g = n_groups - 1;
    if (vsel == 3) return launch_mid_p<WL, 3>(mode, wp, dp, items, n_items, g, k, pgrid, st);
    if (vsel == 1) return launch_mid_p<WL, 1>(mode, wp, dp, items, n_items, g, k, pgrid, st);
    return launch_mid_p<WL, 2>(mode, wp, dp, items, n_items, g, k, pgrid, st);
  }
  if (part == WHT_PART_PRE) {
    if ((vsel & 1) && !(fuse && mode == MODE_GEN))
      e = launch_pass<WL, WHT_FIRST>(mode, wp, dp, items, n_items, 0, k, q, set, 3, st, half & 1);
    for (int g = 1; e == hipSuccess && g + 1 < n_groups; ++g)
      e = launch_pass<WL, WHT_FWD>(mode, wp, dp, items, n_items, g, k, q, set, vsel, st, half & 2);
  } else if (part == WHT_PART_MID) {
    e = launch_pass<WL, WHT_MID>(mode, wp, dp, items, n_items, n_groups - 1, k, q, set, vsel, st);
  } else {
    for (int g = n_groups - 2; e == hipSuccess && g >= 1; --g)
      e = launch_pass<WL, WHT_INV>(mode, wp, dp, items, n_items, g, k, q, set, vsel, st, half & 2);
    if (e == hipSuccess && (vsel & 2)) {
      if (fuse && mode != MODE_APPLY)
        e = launch_pass<WL, WHT_FINAL_NEXT>(mode, wp, dp, items, n_items, 0, k, q, set, 3, st);
      else
        e = launch_pass<WL, WHT_FINAL>(mode, wp, dp, items, n_items, 0, k, q, set, 3, st);
    }
  }
  return e;
}

}  // namespace

hipError_t launch_wht_tables(int wl, const WhtProb* wp, const DevProb* dp, int64_t tiles, hipStream_t st) {
  const dim3 grid((unsigned)((tiles + 255) / 256)), block(256);
  if (wl == 12) {
    hipLaunchKernelGGL(k_wht_tables<12>, grid, block, 0, st, wp, dp, tiles);
    hipLaunchKernelGGL(k_wht_qtab<12>, dim3(2), dim3(512), 0, st, wp, dp);
  } else if (wl == 13) {
    hipLaunchKernelGGL(k_wht_tables<13>, grid, block, 0, st, wp, dp, tiles);
    hipLaunchKernelGGL(k_wht_qtab<13>, dim3(2), dim3(512), 0, st, wp, dp);
  } else {
    return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_wht_part(int part, int wl, int mode, int n_groups, const WhtProb* wp, const DevProb* dp,
                           const int2* items, int n_items, int k, int q, int set, int vsel, hipStream_t st,
                           int pgrid, int pmask) {
  if (n_items <= 0) return hipSuccess;
  if (n_groups < 2 || n_groups > kWhtMaxGroups || vsel < 1 || vsel > 3) return hipErrorInvalidValue;
  if (wl == 12) return wht_part<12>(part, mode, n_groups, wp, dp, items, n_items, k, q, set, vsel, st, pgrid, pmask);
  if (wl == 13) return wht_part<13>(part, mode, n_groups, wp, dp, items, n_items, k, q, set, vsel, st, pgrid, pmask);
  return hipErrorInvalidValue;
}

}  // namespace dse
