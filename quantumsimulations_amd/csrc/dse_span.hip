// dse_span.hip -- persistent Chebyshev kernel for a register spread over 2^s compute units
// (gfx950).
//
// k_interval (dse_interval.hip) gives a register of up to two 2^13 tiles one workgroup per tile:
// a lone N = 14 evolution -- the reference's own call pattern, one `simulate_rare` at a time
// (sweep_sea_detuning.py:671-673), or one GPU's shard of a 64-point sweep split over 8 GPUs --
// is then a serial chain of ~20 us terms on 2 of 256 CUs.  k_span cuts the register into 2^s
// tiles of L = n - s bits (s <= 4) and runs one workgroup per tile, each on its own CU, for all
// Chebyshev terms of one launch.  A thread owns only R = 2^RB amplitudes (RB = 2 or 3), so the
// per-thread work of a term -- the chain's latency -- shrinks with the tile.
//
// Per term k (one workgroup = one tile h; w_{k-1} in LDS, double-buffered so one barrier per
// term separates the terms):
//   pre-pass  for every top bit b with crossing pairs, the operand the partner tile h ^ e_b needs
//             from this tile:  u_b(x) = flip_b(c) w(x) + sum_{j<L} g_jb [x_j == c] w(x ^ e_j),
//             c = the partner's bit value (1 - h_b); all u_b of a pass from ONE sweep over the
//             tile bits (one LDS read of the partner thread per bit), stored to slot b (sc1)
//   publish   per wave: s_waitcnt vmcnt(0), then one lane stores the term index to the wave's
//             flag (sc1).  Thread t of a tile reads only the rows of thread t of a partner, so a
//             wave's operands come from the same wave index of every partner (MI355X_MICROARCH.md
//             "Valid forms", row 1, per wave, as dse_interval.hip's 2-tile hand-off)
//   phase 1   diagonal, drives and pairs among register bits (registers)
//   loop      per thread bit j: the partner thread t ^ e_j's rows serve the drive of j and the
//             pairs (j, register bit); then the iteration's share of the thread-bit pairs
//             (partner t ^ e_i ^ e_j, coefficient zero in lanes with x_i != x_j)
//   phase 4   the cross-tile operands (SpanOp): poll the partner wave's flag, read its rows (sc1)
//   phase 5   w_k = 2 (H - beta) w_{k-1} / alpha - w_{k-2}, the propagator sums of the launch's
//             up to kSpanMaxOut outputs (each every third term, output j on phase j % 3 so the
//             read-modify-writes spread over the terms), w_k -> the other LDS buffer and,
//             when some partner reads raw vectors, to this tile's raw slot
// Ring of kXSlots slots per operand kind: slot (k - 1) % kXSlots carries the operand of term k,
// rewritten kXSlots terms later, by when every reader has passed its flag of a later term.
#include <type_traits>

#include "dse_device.h"

namespace dse {

// Diagnostic ablation mask (diagnostics builds, -DDSE_DIAG; 0 in libdse.so; results are wrong
// otherwise): 1 no pre-pass, 2 no publish, 4 no poll, 8 no operand loads, 16 no propagator sums, 32
// no fused loop, 64 no raw store.  The partners' flags are polled HandoffKnobs::spin_limit times
// (a kernel argument, per context) before a hand-off is declared failed; negative: fail at once.
#ifdef DSE_DIAG
__device__ int g_span_ablate = 0;
hipError_t set_span_ablate(int mask) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_span_ablate), &mask, sizeof(int));
}
#else
constexpr int g_span_ablate = 0;
hipError_t set_span_ablate(int mask) { return mask ? hipErrorNotSupported : hipSuccess; }
#endif

namespace {

typedef __attribute__((address_space(1))) int gint;
typedef __attribute__((address_space(3))) const dv2 ldv2;
typedef __attribute__((address_space(3))) dv2 sdv2;

template <int L, int RB>
struct SpanGeo {
  static constexpr int R = 1 << RB;                    // amplitudes per thread
  static constexpr int TB = L - RB;                    // thread bits
  static constexpr int NT = 1 << TB;                   // threads per workgroup
  static constexpr int NW = NT / 64;                   // waves
  static constexpr int NPI = (TB * (TB - 1) / 2 + TB - 1) / TB;  // thread pairs per iteration
  static constexpr int IW = 4 + NPI;                   // dv2 per iteration row
  static constexpr uint32_t TBYTES = (16u << L);
  // u operands built per pre-pass sweep (2^11-amplitude tiles have at most 3 top bits at n <= 14,
  // and 3 keeps the pipelined pre-pass inside the register budget there; 2-row threads hold 4)
  static constexpr int US = R <= 2 ? 4 : (R <= 4 && NT < 1024) ? (TB >= 9 ? 3 : 4) : 2;
};

template <bool IMAG>
__device__ __forceinline__ double2 smad(double2 acc, double cr, double ci, double2 s) {
  if (IMAG) {
    acc.x = fma(-ci, s.y, acc.x);
    acc.y = fma(ci, s.x, acc.y);
    return acc;
  }
  return cmad(acc, cr, ci, s);
}

__device__ __forceinline__ void rfma(double2& acc, double g, double2 s) {
  acc.x = fma(g, s.x, acc.x);
  acc.y = fma(g, s.y, acc.y);
}

template <typename T>
__device__ __forceinline__ uint32_t lds_byte(const T* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) T*)p;
}

// rows r = 0..R-1 of thread tp from the LDS tile starting at byte address base
template <int NT, int R>
__device__ __forceinline__ void rows_lds(uint32_t base, int tp, double2* v) {
  const uint32_t a = base + (uint32_t)tp * 16u;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const dv2 d = *(ldv2*)(size_t)(a + (uint32_t)r * NT * 16u);
    v[r] = make_double2(d.x, d.y);
  }
}

template <int L, int RB>
struct SpanShared {
  using G = SpanGeo<L, RB>;
  dv2 w[2][1 << L];        // w_{k-1} and w_k (double buffer)
  dv2 it[G::TB][G::IW];    // iteration rows
  // the u pre-pass's coefficients by operand slot c (the c-th top bit with a u operand): g_{j,b}
  // of the tile bits, the top bit's drive at the partner's bit value, that value (0 / 1)
  double ug[kSpanMaxTop][16];
  double uf[kSpanMaxTop][2];
  double ucb[kSpanMaxTop];
  int fail;
};

template <int L, int RB, bool IMAG>
__global__ void __launch_bounds__(1 << (L - RB))
k_span(const DevProb* __restrict__ probs, const SpanDesc* __restrict__ sdesc,
       const int2* __restrict__ items, int q, int set, int n_out, int* __restrict__ err, HandoffKnobs hk) {
  using G = SpanGeo<L, RB>;
  constexpr int R = G::R, TB = G::TB, NT = G::NT, IW = G::IW, NPI = G::NPI, US = G::US;
  // 1024-thread tiles run 4 waves per SIMD (<= 128 VGPRs): fewer operands in flight, propagator
  // sums loaded when used
  constexpr bool LEAN = NT >= 1024;
  constexpr int NB = LEAN ? 2 : (R <= 4 ? 4 : 3);  // operands loaded together in phase 4
  constexpr int J_PUB = TB > 2 ? 2 : TB - 1;  // loop iteration that publishes the term
  constexpr uint32_t TBYTES = G::TBYTES;
  __shared__ SpanShared<L, RB> S;

  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
  const int2 item = items[blockIdx.x];
  if (item.x < 0) return;  // padding item (XCD placement of the registers' tiles)
  const DevProb& P = probs[item.x];
  const SpanDesc& D = sdesc[item.x];
  const cptr<SpanTab> tab = cst(D.tab);
  const uint32_t h = (uint32_t)item.y;
  const int s = D.s;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int K = P.degree;
  const double s1 = P.s1;
  const uint32_t voff = (uint32_t)tid * 16u;
  const int nkind = s + 1;
  auto slot_ptr = [&](uint32_t tile, int kind, int ring) {
    return D.slots + ((((size_t)tile * nkind + kind) * kXSlots + ring) << L);
  };
  const __amdgpu_buffer_rsrc_t psi_me = tile_rsrc(P.buf[q ? 2 : 0] + ((size_t)h << L), TBYTES);
  const __amdgpu_buffer_rsrc_t acc_t = tile_rsrc(P.buf[q ? 0 : 2] + ((size_t)h << L), TBYTES);
  gint* const flag_me = (gint*)D.flags + (int)h * kSpanWaves + wave;
  const int ab = g_span_ablate;
  const int u_mask = (ab & 1) ? 0 : tab->u_mask, n_ops = (ab & 8) ? 0 : tab->n_ops;
  const int n_u = __builtin_popcount(u_mask);
  // the c-th top bit with a u operand (uniform; no runtime-indexed array, which would go to scratch)
  auto ubit_of = [&](int c) {
    uint32_t m = (uint32_t)u_mask;
    for (int i = 0; i < c; ++i) m &= m - 1;
    return (int)__builtin_ctz(m);
  };
  const bool need_raw = tab->need_raw != 0;

  const double* crow = (const double*)coef_row(P, set, 0);
  const size_t rstride = 2 * (size_t)(P.kcap1 + 1);
  int dj[kSpanMaxOut];
#pragma unroll
  for (int j = 0; j < kSpanMaxOut; ++j) dj[j] = j < n_out ? (int)crow[j * rstride] : 0;

  // ---- setup: iteration rows -> LDS, w_0 tile -> LDS buffer 0, per-row diagonal ----
  if (tid == 0) S.fail = 0;
  {
    const gd2* src = (const gd2*)D.tab->it;
    for (int e = tid; e < TB * IW; e += NT) (&S.it[0][0])[e] = src[e];
    if (tid < kSpanMaxTop * 16) {  // u operand slots c < n_u (LDS broadcast reads in the pre-pass)
      const int c = tid >> 4, j = tid & 15;
      if (c < n_u) {
        const int b = ubit_of(c);
        const int v = (int)(((h >> b) & 1u) ^ 1u);  // the consumer's (partner's) value of bit b
        S.ug[c][j] = j < L ? tab->ug[b][j] : 0.0;
        if (j < 2) S.uf[c][j] = tab->uflip[b][2 * v + j];
        if (j == 0) S.ucb[c] = (double)v;
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const double2 v = bld(psi_me, voff, (uint32_t)(r * NT * 16));
    dv2 d;
    d.x = v.x, d.y = v.y;
    S.w[0][r * NT + tid] = d;
  }
  // D(x) = shift - beta + sum_b field_b s_b + sum_{a<b} zz_ab s_a s_b over all n bits
  double dg[R];
  {
    const int n = P.n;
    const cptr<double> fld = cst(P.field), zz = cst(P.zz);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t x = ((uint64_t)h << L) | ((uint64_t)r << TB) | (uint64_t)tid;
      double d = P.shift - P.beta;
      for (int a = 0; a < n; ++a) {
        const double sa = 0.5 - (double)((x >> a) & 1);
        double za = fld[a];
        for (int b = a + 1; b < n; ++b) za = fma(zz[a * n + b], 0.5 - (double)((x >> b) & 1), za);
        d = fma(za, sa, d);
      }
      dg[r] = d;
    }
  }
  __syncthreads();

  // lane o < n_ops: the flag of operand o's partner wave (null: the operand does not apply here)
  const gint* pflag = nullptr;
  int pkind = -1;
  if (lane < n_ops) {
    const SpanOp& op = D.tab->ops[lane];
    if (!(op.kind == 2 && (((h >> op.b) ^ (h >> op.b2)) & 1u))) {
      pflag = (const gint*)D.flags + (int)(h ^ op.pmask) * kSpanWaves + wave;
      pkind = op.kind;
    }
  }

  double2 prev[R];
#pragma unroll
  for (int r = 0; r < R; ++r) prev[r] = make_double2(0.0, 0.0);
  const uint32_t wbase = lds_byte(&S.w[0][0]);

  for (int k = 1; k <= K; ++k) {
    const uint32_t cur = wbase + (uint32_t)((k - 1) & 1) * TBYTES;
    const uint32_t nxt = wbase + (uint32_t)(k & 1) * TBYTES;
    double2 own[R];
    rows_lds<NT, R>(cur, tid, own);

    // ---- pre-pass: u_b for the partners across the top bits with crossing pairs, NU of them per
    // sweep over the tile bits (compile-time NU: no work for absent operands) ----
    auto prepass = [&](auto nu_tag, int c0) {
      constexpr int NU = decltype(nu_tag)::value;
      double2 u[NU][R];
      double cb[NU];  // the consumer's value of bit b (the partner's: 1 - h_b)
#pragma unroll
      for (int bb = 0; bb < NU; ++bb) {
        const int c = c0 + bb;
        cb[bb] = S.ucb[c];
        const double fr = S.uf[c][0], fi = S.uf[c][1];
#pragma unroll
        for (int r = 0; r < R; ++r) u[bb][r] = smad<IMAG>(make_double2(0.0, 0.0), fr, fi, own[r]);
        // register bits: output rows with r_i == c, source r ^ e_i
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const double g = S.ug[c][TB + i];
#pragma unroll
          for (int r = 0; r < R; ++r) rfma(u[bb][r], ((double)((r >> i) & 1) == cb[bb]) ? g : 0.0, own[r ^ (1 << i)]);
        }
      }
      // thread bits, software-pipelined (round 5: the rows of bit j + 1 in flight under bit j's
      // FMAs, the coefficients LDS broadcasts staged at setup; the round-4 loop waited on a scalar
      // load and an LDS read every iteration: 2.3 of the 10.0 us term of a lone register)
      auto bit_terms = [&](int j, const double2* pv) {
        const double tj = (double)((tid >> j) & 1);
#pragma unroll
        for (int bb = 0; bb < NU; ++bb) {
          const double gj = (tj == cb[bb]) ? S.ug[c0 + bb][j] : 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r) rfma(u[bb][r], gj, pv[r]);
        }
      };
#pragma unroll 1
      for (int j = 0; j < TB; ++j) {
        double2 pv[R];
        rows_lds<NT, R>(cur, tid ^ (1 << j), pv);
        bit_terms(j, pv);
      }
#pragma unroll
      for (int bb = 0; bb < NU; ++bb) {
        const __amdgpu_buffer_rsrc_t dst = tile_rsrc(slot_ptr(h, ubit_of(c0 + bb), (k - 1) % kXSlots), TBYTES);
#pragma unroll
        for (int r = 0; r < R; ++r) bst<kSc1>(dst, voff, (uint32_t)(r * NT * 16), u[bb][r]);
      }
    };
    for (int c0 = 0; c0 < n_u; c0 += US) {
      const int m = n_u - c0 < US ? n_u - c0 : US;
      if (m == 1) prepass(std::integral_constant<int, 1>{}, c0);
      else if (m == 2) prepass(std::integral_constant<int, 2>{}, c0);
      else if constexpr (US >= 3) {
        if (m == 3) prepass(std::integral_constant<int, (US >= 3 ? 3 : 1)>{}, c0);
        else prepass(std::integral_constant<int, (US >= 4 ? 4 : 1)>{}, c0);
      }
    }
    // ---- phase 1: diagonal, register-bit drives and pairs (own rows re-read: not held across the
    // pre-pass, whose operands and pipelined partner rows take those registers) ----
    if (n_u > 0) rows_lds<NT, R>(cur, tid, own);
    double2 out[R];
#pragma unroll
    for (int r = 0; r < R; ++r) out[r] = make_double2(dg[r] * own[r].x, dg[r] * own[r].y);
    {
      const int rfm = tab->rflip_mask;
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        if (!((rfm >> i) & 1)) continue;
        const double c0r = tab->rflip[i][0], c0i = tab->rflip[i][1], c1r = tab->rflip[i][2], c1i = tab->rflip[i][3];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const bool v = (r >> i) & 1;
          out[r] = smad<IMAG>(out[r], v ? c1r : c0r, v ? c1i : c0i, own[r ^ (1 << i)]);
        }
      }
#pragma unroll
      for (int a = 0; a < RB; ++a)
#pragma unroll
        for (int b = a + 1; b < RB; ++b) {
          const double g = tab->rr_g[rr_index(a, b)];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            if (((r >> a) ^ (r >> b)) & 1) continue;
            rfma(out[r], g, own[r ^ ((1 << a) | (1 << b))]);
          }
        }
    }

    // ---- fused loop over the thread bits: the sweep's partner rows, then the thread pairs one at a
    // time, each next partner's rows in flight under the current one's FMAs ----
    const uint32_t itb = lds_byte(&S.it[0][0]);
    // publish term k -- u(w_{k-1}) stored by the pre-pass, raw w_{k-1} at the end of term k - 1 --
    // after J_PUB iterations, so the stores drain under the loop: per wave, s_waitcnt vmcnt(0)
    // then one lane's flag store
    const bool pub = u_mask || (need_raw && k > 1);
#pragma unroll 1
    for (int j = 0; j < ((ab & 32) ? 0 : TB); ++j) {
      if (j == J_PUB && pub && !(ab & 2)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(flag_me, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      uint32_t ia;  // one VGPR base for the iteration row (broadcast reads)
      asm("v_mov_b32_e32 %0, %1" : "=v"(ia) : "s"(itb + (uint32_t)j * IW * 16u));
      const dv2 d0 = *(ldv2*)(size_t)ia, d1 = *(ldv2*)(size_t)(ia + 16u);
      double2 pv[R];
      rows_lds<NT, R>(cur, tid ^ (1 << j), pv);
      dv2 pr = *(ldv2*)(size_t)(ia + 16u * 4);
      double2 ta[R], tb[R];
      rows_lds<NT, R>(cur, tid ^ (int)(uint32_t)__double_as_longlong(pr.x), ta);
      const int bj = (tid >> j) & 1;
      const double cr = bj ? d1.x : d0.x, ci = bj ? d1.y : d0.y;
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = smad<IMAG>(out[r], cr, ci, pv[r]);
      {
        const dv2 g01 = *(ldv2*)(size_t)(ia + 16u * 2);
        const dv2 g23 = *(ldv2*)(size_t)(ia + 16u * 3);
#pragma unroll
        for (int i = 0; i < RB; ++i) {
          const double g = i == 0 ? g01.x : i == 1 ? g01.y : i == 2 ? g23.x : g23.y;
          const double g0 = bj ? 0.0 : g, g1 = bj ? g : 0.0;
#pragma unroll
          for (int r = 0; r < R; ++r) rfma(out[r], ((r >> i) & 1) ? g1 : g0, pv[r ^ (1 << i)]);
        }
      }
#pragma unroll
      for (int qq = 0; qq < NPI; ++qq) {
        dv2 pn;
        if (qq + 1 < NPI) {
          pn = *(ldv2*)(size_t)(ia + 16u * (5 + qq));
          rows_lds<NT, R>(cur, tid ^ (int)(uint32_t)__double_as_longlong(pn.x), (qq & 1) ? ta : tb);
        }
        const double ge = par32((uint32_t)tid & (uint32_t)__double_as_longlong(pr.x)) ? 0.0 : pr.y;
        const double2* tv = (qq & 1) ? tb : ta;
#pragma unroll
        for (int r = 0; r < R; ++r) rfma(out[r], ge, tv[r]);
        if (qq + 1 < NPI) pr = pn;
      }
    }

    if ((ab & 32) && pub && !(ab & 2)) {  // diagnostics: no loop, publish here
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(flag_me, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- propagator sums updating at term k.  Output j updates on phase j % 3 (coef_nterm), so
    // outside the rare coincidence with an output's last term at most SL of the launch's sums are
    // read-modify-written per term; their rows are loaded now so the latency hides under phase 4 ----
    constexpr int SL = (kSpanMaxOut + 2) / 3;
    uint32_t um = 0, ntp = 0;  // outputs updating at term k; their term counts, 2 bits each (uniform)
#pragma unroll
    for (int j = 0; j < kSpanMaxOut; ++j) {
      const int nt = j < n_out ? coef_nterm(k, dj[j], j % 3) : 0;
      if (nt > 0 && !(ab & 16)) um |= 1u << j;
      ntp |= (uint32_t)nt << (2 * j);
    }
    auto acc_rsrc = [&](int j) {
      return (j == n_out - 1) ? acc_t
                              : tile_rsrc(P.xacc + ((size_t)(q * P.xacc_q + j) << P.n) + ((size_t)h << L), TBYTES);
    };
    double2 av[SL][R];
    auto load_sums = [&](uint32_t m) {  // the first SL outputs of m
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) {
        if (!m) break;
        const __amdgpu_buffer_rsrc_t ar = acc_rsrc(__builtin_ctz(m));
        m &= m - 1;
#pragma unroll
        for (int r = 0; r < R; ++r) av[sl][r] = bld(ar, voff, (uint32_t)(r * NT * 16));
      }
    };
    if (!LEAN && k > 1) load_sums(um);

    // ---- phase 4: cross-tile operands.  Lane o of each wave polls operand o's partner flag, all
    // at once (one round trip when the partners are ahead); then the operands' rows are loaded
    // in batches of NB, every load of a batch in flight together ----
    {
      const bool need = pflag != nullptr && !(pkind != 0 && k == 1) && !(ab & 4);
      int spins = 0;
      for (;;) {
        const bool ok = !need || __hip_atomic_load(pflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= k;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
        __builtin_amdgcn_s_sleep(1);
        if (++spins > hk.spin_limit ||
            ((spins & 1023) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
          if (lane == 0) {
            S.fail = 1;
            atomicExch(err, 1);
          }
          break;
        }
      }
    }
    asm volatile("" ::: "memory");  // the operand loads stay behind the poll
#pragma unroll 1
    for (int o0 = 0; o0 < n_ops; o0 += NB) {
      double2 uv[NB][R];
      bool app[NB];
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) {
        const int o = o0 + bb;
        app[bb] = false;
        if (o >= n_ops) continue;
        const int kind = tab->ops[o].kind;
        app[bb] = !(kind == 2 && (((h >> tab->ops[o].b) ^ (h >> tab->ops[o].b2)) & 1u));
        if (!app[bb]) continue;
        const uint32_t p = h ^ tab->ops[o].pmask;
        const bool raw = kind != 0;
        const double2* sp = (raw && k == 1) ? P.buf[q ? 2 : 0] + ((size_t)p << L)
                                            : slot_ptr(p, raw ? s : tab->ops[o].b, (k - 1) % kXSlots);
        const __amdgpu_buffer_rsrc_t src = tile_rsrc(sp, TBYTES);
#pragma unroll
        for (int r = 0; r < R; ++r) uv[bb][r] = bld<kSc1>(src, voff, (uint32_t)(r * NT * 16));
      }
#pragma unroll
      for (int bb = 0; bb < NB; ++bb) {
        if (!app[bb]) continue;
        const int o = o0 + bb;
        const int kind = tab->ops[o].kind;
        if (kind == 0) {
#pragma unroll
          for (int r = 0; r < R; ++r) out[r].x += uv[bb][r].x, out[r].y += uv[bb][r].y;
        } else if (kind == 1) {
          const int v = (int)((h >> tab->ops[o].b) & 1u);
          const double cr = tab->ops[o].c[2 * v], ci = tab->ops[o].c[2 * v + 1];
#pragma unroll
          for (int r = 0; r < R; ++r) out[r] = smad<IMAG>(out[r], cr, ci, uv[bb][r]);
        } else {
          const double g = tab->ops[o].c[0];
#pragma unroll
          for (int r = 0; r < R; ++r) rfma(out[r], g, uv[bb][r]);
        }
      }
    }

    // ---- phase 5: recurrence, propagator sums, w_k -> LDS (and the raw slot) ----
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
    rows_lds<NT, R>(cur, tid, own);  // w_{k-1} (re-read: not held across the loop)
    for (uint32_t m = um, first = 1; m; first = 0) {  // rounds of SL sums (one round but at rare terms)
      if ((LEAN || !first) && k > 1) load_sums(m);
#pragma unroll
      for (int sl = 0; sl < SL; ++sl) {
        if (!m) break;
        const int j = __builtin_ctz(m);
        m &= m - 1;
        const int nt = (int)((ntp >> (2 * j)) & 3u);
        const __amdgpu_buffer_rsrc_t ar = acc_rsrc(j);
        const auto cc = crow + j * rstride + 2 * (size_t)(k - 1);  // a_{k-2}, a_{k-1}, a_k
        const double2 c0 = nt >= 3 ? make_double2(cc[0], cc[1]) : make_double2(0.0, 0.0),
                      c1 = nt >= 2 ? make_double2(cc[2], cc[3]) : make_double2(0.0, 0.0),
                      c2 = make_double2(cc[4], cc[5]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          double2 a = make_double2(0.0, 0.0);
          if (k > 1) a = cmad(av[sl][r], c0.x, c0.y, prev[r]);
          a = cmad(a, c1.x, c1.y, own[r]);
          a = cmad(a, c2.x, c2.y, out[r]);
          bst(ar, voff, (uint32_t)(r * NT * 16), a);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      prev[r] = own[r];
      dv2 d;
      d.x = out[r].x, d.y = out[r].y;
      *(sdv2*)(size_t)(nxt + ((uint32_t)(r * NT + tid)) * 16u) = d;
    }
    if (need_raw && k < K && !(ab & 64)) {  // w_k for the partners' term k + 1
      const __amdgpu_buffer_rsrc_t dst = tile_rsrc(slot_ptr(h, s, k % kXSlots), TBYTES);
#pragma unroll
      for (int r = 0; r < R; ++r) bst<kSc1>(dst, voff, (uint32_t)(r * NT * 16), out[r]);
    }
    __syncthreads();  // w_k complete; every read of w_{k-1} done
    if (S.fail) break;
  }
}

}  // namespace

// (11, 3) -- 256 threads of 8 rows, one wave per SIMD, 102 AGPRs of spill -- measured 13.5 against
// 11.4 us per term (lone shell_off register, profiles/r05/ab/span_rb3_256thread_dropped.jsonl)
#define DSE_SPAN_CONFIGS(X) X(11, 2) X(10, 2) X(10, 1)

bool span_supported(int L, int RB) {
#define X(l, rb) if (L == l && RB == rb) return true;
  DSE_SPAN_CONFIGS(X)
#undef X
  return false;
}

hipError_t span_occupancy(int L, int RB, bool imag, int* blocks_per_cu) {
#define X(l, rb)                                                                                   \
  if (L == l && RB == rb)                                                                          \
    return imag ? hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_span<l, rb, true>, \
                                                               SpanGeo<l, rb>::NT, 0)              \
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, k_span<l, rb, false>,\
                                                               SpanGeo<l, rb>::NT, 0);
  DSE_SPAN_CONFIGS(X)
#undef X
  return hipErrorInvalidValue;
}

hipError_t launch_span(int L, int RB, bool imag, const DevProb* probs, const SpanDesc* sdesc,
                       const int2* items, int n_items, int q, int set, int n_out, int* err,
                       HandoffKnobs hk, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
#define X(l, rb)                                                                                   \
  if (L == l && RB == rb) {                                                                        \
    if (imag)                                                                                      \
      hipLaunchKernelGGL((k_span<l, rb, true>), dim3(n_items), dim3(SpanGeo<l, rb>::NT), 0, st,   \
                         probs, sdesc, items, q, set, n_out, err, hk);                             \
    else                                                                                           \
      hipLaunchKernelGGL((k_span<l, rb, false>), dim3(n_items), dim3(SpanGeo<l, rb>::NT), 0, st,  \
                         probs, sdesc, items, q, set, n_out, err, hk);                             \
    return hipGetLastError();                                                                      \
  }
  DSE_SPAN_CONFIGS(X)
#undef X
  return hipErrorInvalidValue;
}

}  // namespace dse
