// dse_interval.hip -- persistent per-interval Chebyshev kernel (gfx950).
//
// One launch propagates one output interval [t_m, t_{m+1}] of every problem whose register fits
// one or two LDS tiles (n <= L + 1; the N = 14 sweep: center_off has n = 13, center_on and
// shell_off n = 14).  Each workgroup owns one tile for all K Chebyshev terms of the interval:
//   LDS        w_{k-1}, the tile being multiplied (128 KiB at L = 13)
//   registers  w_{k-2} (prev) and the new w_k (out), 16 amplitudes per thread each
//   global     acc (read-modify-write every third term, L2-resident) and, for 2-tile problems,
//              the cross-tile operand exchanged with the partner workgroup every term.
//
// Thread t owns the amplitudes x = r * NT + t, r = 0..15 (the four top tile bits are register
// bits).  One H application is
//   phase 1  diagonal, drives and pairs among register bits      (own amplitudes, registers)
//   phase 2  one LDS sweep per thread bit j: the partner thread t ^ e_j's amplitudes serve the
//            drive flip of j and the pairs (j, register bit i)
//   phase 3  pairs between two thread bits (partner t ^ e_i ^ e_j, rows with x_i == x_j)
//   phase 4  the partner tile's contribution (2-tile problems)
//   phase 5  w_k = 2 (H - beta) w_{k-1} / alpha - w_{k-2}; acc += c0 w_{k-2} + c1 w_{k-1} + c2 w_k
//            every third term; w_k -> LDS
// Partner reads go through registers in halves of 8 amplitudes (split on register bit 3) so the
// kernel stays inside the 256-VGPR budget of 2 waves per SIMD without spilling.  Term tables are
// read through the constant address space (scalar loads into SGPRs).
//
// Cross-tile hand-off (2-tile problems; tiles A/B differ in the top bit L).  What B needs from A
// for term k is u_{A->B}(x) = flip_L(b_B) w_A(x) + sum_{j<L} g_{j,L} [x_j == b_B] w_A(x ^ e_j):
//   * flip-only crossing (center geometry: the top bit is the rare spin, coupled by ZZ only):
//     B applies the flip coefficient itself, so A hands over w_{k-1} raw.  A stores w_k with
//     16-byte sc1 stores at the end of term k (w_0 is A's psi tile, readable as is);
//   * crossing pairs (shell geometry): A computes u in a pre-pass at the start of the term.
// Thread t of one tile reads only the rows of thread t of the other, so the hand-off is per wave:
// after its first tile phase each wave waits for its own stores (s_waitcnt vmcnt(0)) and one lane
// publishes the term index with an sc1 flag store for that wave; the partner's wave of the same
// index polls it with sc1 loads (one lane, s_sleep, bounded) and reads the operand with sc1 loads
// after its tile phases (MI355X_MICROARCH.md "Valid forms", row 1, per wave: one workgroup per CU).
// No workgroup barrier is involved, which lets waves 4..7 run the tile phases in the opposite order
// to their SIMD partners 0..3.  Slots form a ring of kXSlots per tile; a slot is rewritten kXSlots
// terms later, and every term waits for the partner wave's flag of that term, so the partner wave
// has long finished reading it.
//
// Register budget: this kernel must not spill VGPRs.  A build that spilled 12 VGPRs (stored once in
// the prologue, reloaded every term) gave run-to-run differences of ~1e-9 on 2-tile problems;
// tests/test_build.py checks the resource usage and tests/test_gpu_parity.py bitwise determinism.
#include <type_traits>

#include "dse_device.h"

namespace dse {

// Diagnostic ablation mask of k_interval (diagnostics builds, -DDSE_DIAG; 0 in libdse.so).
#ifdef DSE_DIAG
__device__ int g_dse_ablate_iv = 0;
hipError_t set_ablate_interval(int mask) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dse_ablate_iv), &mask, sizeof(int));
}
#else
constexpr int g_dse_ablate_iv = 0;
hipError_t set_ablate_interval(int mask) { return mask ? hipErrorNotSupported : hipSuccess; }
#endif
// Hand-off options (HandoffKnobs, per context, a kernel argument): spin_limit polls of a partner's
// flag before a hand-off is declared failed (the runtime then re-runs on the streaming kernels);
// fences 0 (default) the sc1 form -- sc1 payload stores and loads, per-wave s_waitcnt vmcnt(0) +
// barrier before an sc1 flag store, sc1 poll (MI355X_MICROARCH.md, Valid forms, table row 1); 1
// adds an agent-scope release in front of every flag store and an agent-scope acquire behind every
// poll (the placement-independent Guideline 16 recipe): -2.8% points/h on the bench
// (profiles/r02/ab/handoff_fences.jsonl).

namespace {

typedef __attribute__((address_space(1))) int gint;


// out += c * s for a drive coefficient c = cr + i ci; IMAG: cr == 0 (drive phase pi/2)
template <bool IMAG>
__device__ __forceinline__ double2 dmad(double2 acc, double cr, double ci, double2 s) {
  if (IMAG) {
    acc.x = fma(-ci, s.y, acc.x);
    acc.y = fma(ci, s.x, acc.y);
    return acc;
  }
  return cmad(acc, cr, ci, s);
}

__device__ __forceinline__ void rmad(double2& acc, double g, double2 s) {
  acc.x = fma(g, s.x, acc.x);
  acc.y = fma(g, s.y, acc.y);
}

typedef __attribute__((address_space(3))) const dv2 ldv2;

// LDS byte address of a __shared__ object (for the half-tile row reads below)
template <typename T>
__device__ __forceinline__ uint32_t lds_addr(const T* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) T*)p;
}

// Rows hh * NH + r0 .. hh * NH + r0 + NR - 1 of thread t from the LDS tile w (row r of thread t
// at w[r * NT + t]).  One base address per half and the rows at immediate offsets: the second half
// of a 2^13 tile starts 64 KiB in, past ds_read's 16-bit offset field, and left to itself the
// compiler forms one address per row (8 extra VALU adds per partner half).  The base of the
// second half is made opaque so it is not re-associated into per-row adds.
template <int NT, int NH, int NR>
__device__ __forceinline__ void ld_rows(const double2* w, int t, int hh, int r0, double2* v) {
  uint32_t a = lds_addr(w + t);
  constexpr uint32_t HALF = (uint32_t)NH * NT * 16u;
  if (hh) {
    if (HALF >= 65536u)
      asm("v_add_u32_e32 %0, %1, %2" : "=v"(a) : "i"(HALF), "v"(a));
    else
      a += HALF;
  }
#pragma unroll
  for (int rr = 0; rr < NR; ++rr) {
    const dv2 d = *(ldv2*)(size_t)(a + (uint32_t)(r0 + rr) * NT * 16u);
    v[rr] = make_double2(d.x, d.y);
  }
}

template <int L>
struct IvShared {
  double2 w[RB<L>::T];  // the tile of w_{k-1}
  double c[L + 1];      // F_i(h) (i < L) and C(h) of the tile
  double zz[L * L];     // in-tile zz couplings (upper triangle)
  double zr[kRegAmps];  // register-bit ZZ part of the diagonal per r
  // per-thread diagonal D(r) = td[0] + sum_i td[1 + i] s_i(r) + zr[r], kept here rather than in
  // registers: the kernel is at the 256-VGPR limit and these are read once per term
  // (pairs per thread: {td0, td1}, {td2, td3}, {td4, 0} -- addressed like the tile rows, from the
  // thread's 16-byte index, so no separate address register stays live across the term)
  dv2 td[3][RB<L>::NT];
  double xg[kRegBits];  // cross pairs (register bit i, top bit) of the u pre-pass
  double xq[RB<L>::TB];  // cross pairs (thread bit j, top bit) of the u pre-pass (0: none)
  // per fused-loop iteration j (thread bit j), 8 granules: the first 64 B of P.sweeps[j] (re0 im0 |
  // re1 im1 | g0 g1 | g2 g3) and thread pairs 4j .. 4j + 3 of P.pairs_tt (mask_lo tile_xor | g),
  // zero past the list -- LDS copies (counted waits, no SMEM), one base address per iteration
  dv2 it[RB<L>::TB][8];
};

template <int L, bool IMAG>
__global__ void __launch_bounds__(RB<L>::NT)
k_interval(const DevProb* __restrict__ probs, const int2* __restrict__ items, int q, int set,
           int n_out, int* __restrict__ flags, int* __restrict__ err, HandoffKnobs hk, long colstride) {
  constexpr int NT = RB<L>::NT, R = kRegAmps, TB = RB<L>::TB, NH = R / 2;
  // software-pipelined partner reads in the fused loop (the production IMAG build; the general
  // build keeps the plain order, which fits its larger drive arithmetic without spilling)
  constexpr bool PIPE = DSE_PIPE && IMAG;
  constexpr uint32_t T = 1u << L;
  __shared__ IvShared<L> S;
  __shared__ int s_fail;

  // a hand-off of an earlier launch timed out: this evolve is abandoned (the runtime re-runs it on
  // the streaming kernels), so launches queued behind that one return at once
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  // column mode (colstride > 0, the propagator-matrix build of dse_runtime's matrix_run): a
  // one-tile register, item.y = the column; its state buffers start column * colstride in
  const uint32_t h = colstride ? 0u : (uint32_t)it.y;
  const size_t coff = colstride ? (size_t)it.y * (size_t)colstride : 0;
  const int tid = threadIdx.x;
  const bool pair = (P.n == L + 1);
  const bool xgen = pair && P.n_pairs_hi > 0;  // pairs cross the tile boundary: u pre-pass
  const int K = P.degree;
  const double s1 = P.s1;
  const uint32_t b_me = h & 1u, b_pa = b_me ^ 1u;  // top-bit values of this / the partner tile

  // hand-off slots (AoS double2, sc1): a ring of kXSlots tile-sized regions per tile,
  // P.xslots[(tile * kXSlots + (k - 1) % kXSlots) << L] carries the operand of term k.  The
  // partner's w_0 is read from its psi tile.
  constexpr uint32_t TBYTES = T * 16u;
  const __amdgpu_buffer_rsrc_t psi_me = tile_rsrc(P.buf[q ? 2 : 0] + coff + (h << L), TBYTES);
  const __amdgpu_buffer_rsrc_t psi_pa = tile_rsrc(P.buf[q ? 2 : 0] + ((h ^ 1u) << L), TBYTES);
  double2* const xs_me = P.xslots + ((size_t)h * kXSlots << L);
  double2* const xs_pa = P.xslots + ((size_t)(h ^ 1u) * kXSlots << L);
  const __amdgpu_buffer_rsrc_t acc_t = tile_rsrc(P.buf[q ? 0 : 2] + coff + (h << L), TBYTES);
  const uint32_t voff = (uint32_t)tid * 16u;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // hand-off flags: one per wave, flags[(2 * problem + tile) * kIvWaves + wave]
  gint* flag_me = (gint*)flags + (2 * it.x + (int)h) * kIvWaves + wave;
  const gint* flag_pa = (const gint*)flags + (2 * it.x + (int)(h ^ 1u)) * kIvWaves + wave;

  // term tables (scalar loads)
  const cptr<DPair> cph = cst(P.pairs_hi);
  const cptr<DFlip> cfh = cst(P.flips_hi);
  // coefficient rows of the outputs (coef_row): [j][0].x = degree d_j, [j][1 + k] = a_k
  // (vector loads of uniform addresses: the scalar-load form of these reads, measured, made the
  // 2-tile problems' results vary from run to run at the 1e-10 level; tools/diag_repeat.py)
  const double* crow = (const double*)coef_row(P, set, 0);
  const size_t rstride = 2 * (size_t)(P.kcap1 + 1);  // doubles per row
  int dj[kMaxOut];
#pragma unroll
  for (int j = 0; j < kMaxOut; ++j) dj[j] = j < n_out ? (int)crow[j * rstride] : 0;

  // diagnostics only (0 in production): 4 skip the register-bit terms, 64 skip the hand-off stores
  // and flag, 128 skip the partner wait and read, 256 skip the acc updates, 512 skip the tile terms
  const int ab = g_dse_ablate_iv;
  const bool fences = hk.fences != 0;

  // ---- setup: tables, w_0 tile -> LDS, per-thread diagonal ----
  if (tid == 0) s_fail = 0;
  {
    const gdbl* zz = gptr(P.zz);
    const int n = P.n;
    for (int e = tid; e < L * L; e += NT) {
      const int i = e / L, j = e % L;
      S.zz[e] = (j > i) ? zz[i * n + j] : 0.0;
    }
    tile_diag_coeffs<L>(P, h, P.beta, S.c, tid);
    static_assert(sizeof(DSweep) == 80 && sizeof(DPair) == 16, "iteration table layout");
    const gd2* psw = (const gd2*)P.sweeps;
    const gd2* ptt = (const gd2*)P.pairs_tt;
    for (int e = tid; e < 8 * TB; e += NT) {
      const int j = e >> 3, c = e & 7;
      dv2 v;
      v.x = v.y = 0.0;
      if (c < 4)
        v = psw[j * 5 + c];
      else if (4 * j + c - 4 < P.n_pairs_tt)
        v = ptt[4 * j + c - 4];
      S.it[j][c] = v;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) S.w[r * NT + tid] = bld(psi_me, voff, (uint32_t)(r * NT * 16));
  __syncthreads();
  if (tid < kRegAmps) {
    double v = 0.0;
    for (int a = 0; a < kRegBits; ++a)
      for (int b = a + 1; b < kRegBits; ++b)
        v += S.zz[(TB + a) * L + TB + b] * ((0.5 - ((tid >> a) & 1)) * (0.5 - ((tid >> b) & 1)));
    S.zr[tid] = v;
  }
  // per-thread diagonal: D(r) = zt + sum_i hr[i] s_i(r) + zr[r]
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
  static_assert(kRegBits == 4, "td packing");
  {
    dv2 v;
    v.x = zt, v.y = hr[0];
    S.td[0][tid] = v;
    v.x = hr[1], v.y = hr[2];
    S.td[1][tid] = v;
    v.x = hr[3], v.y = 0.0;
    S.td[2][tid] = v;
  }
  // register-bit cross pairs (register bit i, top bit) for the u pre-pass
  if (tid < kRegBits) {
    double g = 0.0;
    if (xgen)
      for (int p = 0; p < P.n_pairs_hi; ++p)
        if (cph[p].mask_lo == (1u << (TB + tid))) g = cph[p].g;
    S.xg[tid] = g;
  }
  if (tid < TB) {
    double g = 0.0;
    if (xgen)
      for (int p = 0; p < P.n_pairs_hi; ++p)
        if (cph[p].mask_lo == (1u << tid)) g = cph[p].g;
    S.xq[tid] = g;
  }
  __syncthreads();

  double2 prev[R];
#pragma unroll
  for (int r = 0; r < R; ++r) prev[r] = make_double2(0.0, 0.0);

  // The term loop is instantiated twice, for tiles with and without the u pre-pass (crossing pairs),
  // so that the register allocator sees the two phase orders separately (block-uniform dispatch).
  auto term_loop = [&](auto xg_tag) {
  constexpr bool xgen = decltype(xg_tag)::value;
  const bool xraw = pair && !xgen;
  for (int k = 1; k <= K; ++k) {
    // ---- phase 1: diagonal and register-bit terms (the thread's own rows, which it wrote itself).
    // Without a pre-pass it runs before the barrier, while the other threads' stores of w_{k-1}
    // to LDS drain; with one, after the pre-pass, whose u does not fit beside out ----
    double2 out[R];
    auto phase1 = [&]() {
      double2 own[R];
#pragma unroll
      for (int r = 0; r < R; ++r) own[r] = S.w[r * NT + tid];
      if (ab & (512 | 4)) {
#pragma unroll
        for (int r = 0; r < R; ++r) out[r] = own[r];
      } else {
        const dv2 t01 = S.td[0][tid], t23 = S.td[1][tid], t4 = S.td[2][tid];
        const double tdv[1 + kRegBits] = {t01.x, t01.y, t23.x, t23.y, t4.x};
#pragma unroll
        for (int r = 0; r < R; ++r) {
          double d = tdv[0] + S.zr[r];
#pragma unroll
          for (int i = 0; i < kRegBits; ++i) d += ((r >> i) & 1 ? -0.5 : 0.5) * tdv[1 + i];
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
              out[r] = dmad<IMAG>(out[r], v ? c1r : c0r, v ? c1i : c0i, own[r ^ (1 << i)]);
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
              rmad(out[r], g, own[r ^ ((1 << a) | (1 << b))]);
            }
          }
      }
    };
    if constexpr (!xgen) phase1();
    __syncthreads();  // w_{k-1} complete in LDS

    // ---- phase 0 (crossing pairs): u(w_{k-1}) for the partner -> slot (k-1)&1, sc1 ----
    if (xgen && !(ab & 64)) {
      double2 u[R];
#pragma unroll
      for (int r = 0; r < R; ++r) u[r] = make_double2(0.0, 0.0);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        double2 ow[NH];
        ld_rows<NT, NH, NH>(S.w, tid, hh, 0, ow);
        for (int f = 0; f < P.n_flips_hi; ++f) {  // top-bit drive at the partner's bit value
          const double cr = b_pa ? cfh[f].re1 : cfh[f].re0, ci = b_pa ? cfh[f].im1 : cfh[f].im0;
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) u[hh * NH + rr] = cmad(u[hh * NH + rr], cr, ci, ow[rr]);
        }
        // (register bit i, top): output rows with r_i == b_pa, source r ^ e_i
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) {
            const double g = (((rr >> i) & 1u) == b_pa) ? S.xg[i] : 0.0;
            rmad(u[hh * NH + rr], g, ow[rr ^ (1 << i)]);
          }
        {
          const double g = ((uint32_t)(1 - hh) == b_pa) ? S.xg[3] : 0.0;
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) rmad(u[(1 - hh) * NH + rr], g, ow[rr]);
        }
      }
      // (thread bit j, top): applies iff t_j == b_pa, source t ^ e_j.  Lane bits in a software
      // pipeline of 8-row halves (the next half in flight under the current FMAs), the coefficient
      // zero in the lanes where the pair does not act; thread bits j >= 6 index the wave, so the
      // pair acts on a whole wave or not at all: those partner reads are skipped by a scalar branch
      constexpr int JL = TB < 6 ? TB : 6;
      double2 ba[NH], bb[NH];
      ld_rows<NT, NH, NH>(S.w, tid ^ 1, 0, 0, ba);
#pragma unroll
      for (int j = 0; j < JL; ++j) {
        const double gj = ((uint32_t)((tid >> j) & 1) == b_pa) ? S.xq[j] : 0.0;
        ld_rows<NT, NH, NH>(S.w, tid ^ (1 << j), 1, 0, bb);
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(u[rr], gj, ba[rr]);
        if (j + 1 < JL) ld_rows<NT, NH, NH>(S.w, tid ^ (1 << (j + 1)), 0, 0, ba);
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(u[NH + rr], gj, bb[rr]);
      }
#pragma unroll
      for (int j = JL; j < TB; ++j) {
        if ((uint32_t)__builtin_amdgcn_readfirstlane((tid >> j) & 1) != b_pa) continue;  // whole wave
        const double gj = S.xq[j];
        ld_rows<NT, NH, NH>(S.w, tid ^ (1 << j), 0, 0, ba);
        ld_rows<NT, NH, NH>(S.w, tid ^ (1 << j), 1, 0, bb);
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(u[rr], gj, ba[rr]);
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(u[NH + rr], gj, bb[rr]);
      }
      const __amdgpu_buffer_rsrc_t dst = tile_rsrc(xs_me + ((size_t)((k - 1) % kXSlots) << L), TBYTES);
#pragma unroll
      for (int r = 0; r < R; ++r) bst<kSc1>(dst, voff, (uint32_t)(r * NT * 16), u[r]);
    }

    if constexpr (xgen) phase1();

    // ---- publish (per wave): thread t's hand-off rows are read only by thread t of the partner
    // tile, i.e. wave w's stores only by the partner's wave w.  The wave waits for its own stores
    // (s_waitcnt vmcnt(0)) and one lane stores the term index to the wave's flag (sc1); no
    // workgroup barrier, so the two halves of the workgroup can run their phases in either order ----
    auto publish = [&]() {
      if (pair && !(ab & 64) && (xgen || k > 1)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          if (fences) {  // agent-scope release in front of the flag (Guideline 16 form)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
          __hip_atomic_store(flag_me, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    };

    // ---- phases 2 + 3, fused: iteration j = the LDS sweep of thread bit j (its drive and its pairs
    // with the register bits; VALU-heavy) + thread-bit pairs 4j .. 4j + 3 (partner t ^ e_i ^ e_j,
    // coefficient zero in the lanes with x_i != x_j; LDS-heavy), one basic block, so the pairs'
    // partner reads issue under the sweep's FMAs.  The hand-off is published half way. ----
    // ---- phase 4 (after the fused loop below): the partner tile's contribution, read with sc1 loads
    // after one poll of the partner wave's flag ----
    constexpr int J_PUB = TB / 2;  // publish half way through the fused loop

#pragma unroll 1
    for (int j = 0; j < ((ab & 512) ? 0 : TB); ++j) {
      if (j == J_PUB) publish();
      const int pt = tid ^ (1 << j);
      double2 pv[NH];  // partner rows of the sweep (PIPE: the first half, in flight under the tables)
      if constexpr (PIPE) ld_rows<NT, NH, NH>(S.w, pt, 0, 0, pv);
      // the iteration's tables (S.it[j]), eight 16-byte reads issued together
      dv2 swv[4], ttv[4];
      {
        // one VGPR base for the eight reads (immediate offsets); left uniform, the compiler forms
        // each address in an SGPR and moves it into one reused VGPR, serialising the reads
        uint32_t ia;
        asm("v_mov_b32_e32 %0, %1" : "=v"(ia) : "s"(lds_addr(&S.it[j][0])));
#pragma unroll
        for (int e = 0; e < 4; ++e) swv[e] = *(ldv2*)(size_t)(ia + 16u * e);
#pragma unroll
        for (int e = 0; e < 4; ++e) ttv[e] = *(ldv2*)(size_t)(ia + 16u * (4 + e));
      }
      const int bj = (tid >> j) & 1;
      const double cr = bj ? swv[1].x : swv[0].x, ci = bj ? swv[1].y : swv[0].y;
      double g0[kRegBits], g1[kRegBits];  // pair (j, register bit i) on rows with r_i = 0 / 1
#pragma unroll
      for (int i = 0; i < kRegBits; ++i) {
        const double g = (i & 1) ? swv[2 + i / 2].y : swv[2 + i / 2].x;
        g0[i] = bj ? 0.0 : g;
        g1[i] = bj ? g : 0.0;
      }
      int tpt[4];
      double ge[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {  // zero entries beyond the problem's pairs
        const uint32_t m = (uint32_t)__double_as_longlong(ttv[qq].x);  // DPair::mask_lo
        tpt[qq] = tid ^ (int)m;
        ge[qq] = par32((uint32_t)tid & m) ? 0.0 : ttv[qq].y;  // rows with x_i == x_j
      }
      auto gsel = [&](int i, int bit) { return bit ? g1[i] : g0[i]; };
      // the sweep of half hh (rows r_3 = hh) from the partner rows pv, and thread pair qq on half hh
      auto sweep = [&](int hh, const double2* pv) {
        double2* oh = out + hh * NH;
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) oh[rr] = dmad<IMAG>(oh[rr], cr, ci, pv[rr]);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
          for (int rr = 0; rr < NH; ++rr) rmad(oh[rr], gsel(i, (rr >> i) & 1), pv[rr ^ (1 << i)]);
        // (j, register bit 3): rows of the other half, r_3 = 1 - hh
        double2* oo = out + (1 - hh) * NH;
        const double g3 = gsel(3, 1 - hh);
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(oo[rr], g3, pv[rr]);
      };
      auto tpair = [&](int qq, int hh, const double2* tv) {
        double2* oh = out + hh * NH;
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) rmad(oh[rr], ge[qq], tv[rr]);
      };
      if constexpr (PIPE) {
        // software pipeline over the iteration's partner reads: the sweep's 8-row halves and the
        // thread pairs in 4-row quarters, each next read issued before the FMAs of the current one
        // (+2-3% points/h, profiles/r02/ab/pipelined_loop.jsonl)
        constexpr int NQ = NH / 2;
        auto tpair_q = [&](int qq, int hh, int qh, const double2* tv) {
          double2* oh = out + hh * NH + qh * NQ;
#pragma unroll
          for (int rr = 0; rr < NQ; ++rr) rmad(oh[rr], ge[qq], tv[rr]);
        };
        double2 qa[NQ], qb[NQ];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          ld_rows<NT, NH, NQ>(S.w, tpt[0], hh, 0, qa);
          sweep(hh, pv);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            ld_rows<NT, NH, NQ>(S.w, tpt[qq], hh, NQ, qb);
            tpair_q(qq, hh, 0, qa);
            if (qq < 3)
              ld_rows<NT, NH, NQ>(S.w, tpt[qq + 1], hh, 0, qa);
            else if (hh == 0)
              ld_rows<NT, NH, NH>(S.w, pt, 1, 0, pv);
            tpair_q(qq, hh, 1, qb);
          }
        }
      } else {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          ld_rows<NT, NH, NH>(S.w, pt, hh, 0, pv);
          sweep(hh, pv);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            double2 tv[NH];
            ld_rows<NT, NH, NH>(S.w, tpt[qq], hh, 0, tv);
            tpair(qq, hh, tv);
          }
        }
      }
    }
    if (ab & 512) publish();  // diagnostics: no tile terms, the hand-off alone
    if (pair && !(ab & 128)) {
      const __amdgpu_buffer_rsrc_t src =  // operand of term k: partner slot, or (raw, k = 1) its psi
          (xraw && k == 1) ? psi_pa : tile_rsrc(xs_pa + ((size_t)((k - 1) % kXSlots) << L), TBYTES);
      // the top-bit drive (cross flip) at this tile's output bit value (raw exchange; scalar loads
      // here rather than registers held across the term)
      double xr = 0.0, xi = 0.0;
      if (xraw && P.n_flips_hi > 0) {
        xr = b_me ? cfh[0].re1 : cfh[0].re0;
        xi = b_me ? cfh[0].im1 : cfh[0].im0;
      }
        if ((xgen || k > 1) && lane == 0 && !(ab & 64)) {  // w_0 of the partner is its psi tile
          int spins = 0;
          const int limit = hk.spin_limit;
          while (limit < 0 || __hip_atomic_load(flag_pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) {
            __builtin_amdgcn_s_sleep(1);
            // give up at the limit, or as soon as another pair has (its partner may never come)
            if (limit < 0 || ++spins > limit ||
                ((spins & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
              s_fail = 1;
              atomicExch(err, 1);
              break;
            }
          }
          if (fences) {  // agent-scope acquire behind the poll
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          }
        }
      // compiler barrier: the operand loads below stay behind the poll in program order (one wave
      // issues its memory instructions in order, so the hardware keeps them there too)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        double2 uv[NH];
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) uv[rr] = bld<kSc1>(src, voff, (uint32_t)((hh * NH + rr) * NT * 16));
#pragma unroll
        for (int rr = 0; rr < NH; ++rr) {
          double2& o = out[hh * NH + rr];
          if (xgen) {
            o.x += uv[rr].x;
            o.y += uv[rr].y;
          } else {
            o = dmad<IMAG>(o, xr, xi, uv[rr]);
          }
        }
      }
    }

    // ---- phase 5: recurrence, then the propagator sums of the n_out outputs (each updated every
    // third term from w_{k-2}, w_{k-1}, w_k, and at its own last term) in blocks of AB registers,
    // every output's accumulator loads of a block in flight together ----
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (k == 1) {
        out[r].x *= s1;
        out[r].y *= s1;
      } else {
        out[r].x = fma(2.0 * s1, out[r].x, -prev[r].x);
        out[r].y = fma(2.0 * s1, out[r].y, -prev[r].y);
      }
    }
    constexpr int AB = kMaxOut <= 2 ? 4 : (kMaxOut == 3 ? 2 : 1);  // VGPR budget: AB x kMaxOut loads
    const int nj = (ab & 256) ? 0 : n_out;
    bool upd[kMaxOut];
    __amdgpu_buffer_rsrc_t acc_j[kMaxOut];
#pragma unroll
    for (int j = 0; j < kMaxOut; ++j) {
      upd[j] = j < nj && coef_nterm(k, dj[j]) > 0;
      acc_j[j] = (j == n_out - 1) ? acc_t
                                  : tile_rsrc(P.xacc + ((size_t)(q * P.xacc_q + j) << (L + P.tbl)) + (h << L), TBYTES);
    }
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += AB) {
      double2 ownb[AB];
#pragma unroll
      for (int r = 0; r < AB; ++r) ownb[r] = S.w[(r0 + r) * NT + tid];
      double2 accv[kMaxOut][AB];
#pragma unroll
      for (int j = 0; j < kMaxOut; ++j)
        if (upd[j] && k > 1) {
#pragma unroll
          for (int r = 0; r < AB; ++r) accv[j][r] = bld(acc_j[j], voff, (uint32_t)((r0 + r) * NT * 16));
        }
#pragma unroll
      for (int j = 0; j < kMaxOut; ++j) {
        if (!upd[j]) continue;
        const int nt = coef_nterm(k, dj[j]);
        const auto cc = crow + j * rstride + 2 * (size_t)(k - 1);  // a_{k-2}, a_{k-1}, a_k
        const double2 c0 = nt >= 3 ? make_double2(cc[0], cc[1]) : make_double2(0.0, 0.0),
                      c1 = nt >= 2 ? make_double2(cc[2], cc[3]) : make_double2(0.0, 0.0),
                      c2 = make_double2(cc[4], cc[5]);
#pragma unroll
        for (int r = 0; r < AB; ++r) {
          double2 a = make_double2(0.0, 0.0);
          if (k > 1) a = cmad(accv[j][r], c0.x, c0.y, prev[r0 + r]);
          a = cmad(a, c1.x, c1.y, ownb[r]);
          a = cmad(a, c2.x, c2.y, out[r0 + r]);
          bst(acc_j[j], voff, (uint32_t)((r0 + r) * NT * 16), a);
        }
      }
#pragma unroll
      for (int r = 0; r < AB; ++r) prev[r0 + r] = ownb[r];
    }
    __syncthreads();  // every read of w_{k-1} in LDS is done
    if (s_fail) break;  // uniform: a hand-off timed out (error reported to the host)
#pragma unroll
    for (int r = 0; r < R; ++r) S.w[r * NT + tid] = out[r];
    if (xraw && k < K && !(ab & 64)) {  // w_k for the partner's term k + 1
      const __amdgpu_buffer_rsrc_t dst = tile_rsrc(xs_me + ((size_t)(k % kXSlots) << L), TBYTES);
#pragma unroll
      for (int r = 0; r < R; ++r) bst<kSc1>(dst, voff, (uint32_t)(r * NT * 16), out[r]);
    }
  }
  };
  if (xgen)
    term_loop(std::true_type{});
  else
    term_loop(std::false_type{});
}

// hand-off flags of the launched items only (2 per problem: flags[2 * problem + tile]), so the
// launches of another stream, whose problems' flags are in use, are not disturbed
__global__ void k_zero_flags(const int2* __restrict__ items, int n_items, int* __restrict__ flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_items * kIvWaves) {
    const int2 e = items[i / kIvWaves];
    flags[(2 * e.x + e.y) * kIvWaves + i % kIvWaves] = 0;
  }
}

}  // namespace

hipError_t zero_flags(const int2* items, int n_items, int* flags, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_zero_flags, dim3((n_items * kIvWaves + 255) / 256), dim3(256), 0, st, items, n_items, flags);
  return hipGetLastError();
}

bool interval_supported(int L) { return L >= kRegBlockMinTile && L <= kMaxTile; }

hipError_t interval_occupancy(int L, bool imag, int* blocks_per_cu) {
  switch (L) {
#define X(l)                                                                                       \
  case l:                                                                                          \
    return imag ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_interval<l, true>, \
                                                               RB<l>::NT, 0)                       \
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_interval<l, false>,\
                                                               RB<l>::NT, 0);
    X(10) X(11) X(12) X(13)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_interval(int L, bool imag, const DevProb* probs, const int2* items, int n_items,
                           int q, int set, int n_out, int* flags, int* err, HandoffKnobs hk, hipStream_t st,
                           long colstride) {
  if (n_items <= 0) return hipSuccess;
  switch (L) {
#define X(l)                                                                                     \
  case l:                                                                                        \
    if (imag)                                                                                    \
      hipLaunchKernelGGL((k_interval<l, true>), dim3(n_items), dim3(RB<l>::NT), 0, st, probs,  \
                         items, q, set, n_out, flags, err, hk, colstride);                        \
    else                                                                                         \
      hipLaunchKernelGGL((k_interval<l, false>), dim3(n_items), dim3(RB<l>::NT), 0, st, probs, \
                         items, q, set, n_out, flags, err, hk, colstride);                        \
    return hipGetLastError();
    X(10) X(11) X(12) X(13)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace dse
