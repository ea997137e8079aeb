// dse_internal.h -- device-side data structures shared by the kernels and the runtime.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace dse {

enum { MODE_APPLY = 0, MODE_FIRST = 1, MODE_GEN = 2 };

constexpr int kMinTile = 1;
constexpr int kMaxTile = 13;
constexpr int kRegBits = 4;                       // amplitudes per thread = 2^kRegBits in that kernel
constexpr int kRegAmps = 1 << kRegBits;
constexpr int kRegPairs = kRegBits * (kRegBits - 1) / 2;
constexpr int kRegBlockMinTile = 6 + kRegBits;    // tiles >= 2^10 (>= one wave) use it
// index of the register-bit pair (a, b), a < b, in DevProb::rr_g: (0,1) (0,2) (0,3) (1,2) ...
__host__ __device__ constexpr int rr_index(int a, int b) {
  return a * (2 * kRegBits - a - 1) / 2 + (b - a - 1);
}
constexpr int kXSlots = 4;                        // hand-off ring of the interval kernel
constexpr int kIvWaves = 8;                       // hand-off flags per tile (one per wave of a 2^13 tile)
#ifndef DSE_PIPE
#define DSE_PIPE 1  // interval kernel: software-pipelined partner reads in the fused loop
#endif
constexpr int kMaxOut = 2;      // output times per launch of k_interval / k_real (sums in registers)
constexpr int kSpanMaxOut = 4;  // output times per k_span launch (staggered sums, coef_nterm)
constexpr int kMaxShardBits = 3;                  // partitioned registers: up to 8 shards
constexpr int kMaxShards = 1 << kMaxShardBits;
// bits above an L-bit tile for the largest register (34 qubits), at least the 32-bit tile index
#define DSE_MAX_HIGH_BITS(L) ((34 - (L)) < 0 ? 0 : (34 - (L)))

// A pair flip or a drive flip, split into its in-tile mask and its tile-index mask.
//   pair : applies iff bit_i(x) == bit_j(x) <=> popc(x_lo & mask_lo) + popc(h & tile_xor) even
//   flip : coefficient index v = parity(x_lo & mask_lo) ^ parity(h & tile_xor) (output bit value)
struct alignas(16) DPair {
  uint32_t mask_lo;
  uint32_t tile_xor;
  double g;
};
struct alignas(16) DFlip {
  uint32_t mask_lo;
  uint32_t tile_xor;
  double re0, im0, re1, im1;
  double pad;
};

// Register-block kernel: one thread owns the 16 amplitudes x = rho * NT + tid (rho = 0..15),
// i.e. the four top tile bits are "register bits".  For every thread bit j a sweep reads the
// partner thread's 16 amplitudes once from LDS and applies (a) the drive flip of bit j and
// (b) the pair flips (j, register bit i) for i = 0..3.
struct alignas(16) DSweep {
  double re0, im0, re1, im1;  // drive flip on thread bit j (zero when absent)
  double g[kRegBits];         // pair coefficient with register bit i
  uint32_t has_flip;
  uint32_t has_pair;
};

// Chebyshev coefficients of one term k for one interval length.  The propagator sum
// acc = sum_k a_k w_k is accumulated every third term (and at the last term) from the three
// vectors the step kernel holds anyway: acc += c[0] w_{k-2} + c[1] w_{k-1} + c[2] w_k.
// MODE_FIRST (k = 1) writes acc = c[1] w_0 + c[2] w_1.
struct alignas(16) CoefK {
  double2 c[3];
  int upd;
  int pad[3];
};

struct RealTab;

struct DevProb {
  double2* buf[3];
  const double* zzlo;     // [2^L]  sum_{i<j<L} zz_ij s_i s_j
  const double* field;    // [n]
  const double* zz;       // [n*n]
  const DPair* pairs_lo;  // generic kernel: both bits inside the tile
  const DPair* pairs_hi;  // at least one bit above the tile (both kernels)
  const DFlip* flips_lo;  // generic kernel
  const DFlip* flips_hi;  // both kernels
  const DSweep* sweeps;   // register-block kernel: [L-kRegBits] thread-bit sweeps
  const DPair* pairs_tt;  // register-block kernel: pairs between two thread bits
  const double2* coef;    // compact Chebyshev rows, see coef_row / coef_at
  uint64_t sea_mask;
  double shift;
  double beta;            // spectral centre
  double s1;              // 1/alpha
  double rr_g[kRegPairs]; // register-block kernel: pairs among register bits (rr_index order)
  double rflip[kRegBits][4];  // register-block kernel: drive flips on register bits (re0 im0 re1 im1)
  int n, L;
  int n_pairs_lo, n_pairs_hi, n_flips_lo, n_flips_hi, n_pairs_tt;
  int kcap1;
  int degree;             // Chebyshev degree K of the current evolve (terms k = 1..K)
  int rare_bit;
  int n_sea;
  int rflip_mask;         // bit i set: register bit i has a drive flip
  // Partitioned registers (dse_add_problem_sharded): this problem holds shard `rank` of a
  // register whose top `shard_bits` qubits are global.  Tile indices in the kernels are global
  // (hg = h_base | h for local tile h); a tile of shard rank ^ m is read through rbuf[m][role]
  // (the partner's own buffers on the same device, or receive buffers filled by an exchange).
  uint32_t h_base;        // rank << tbl (0 for an ordinary problem)
  int tbl;                // local tile-index bits: log2(tiles of this shard)
  double2* rbuf[kMaxShards][3];
  double2* xslots;        // interval kernel, 2-tile problems: [2][kXSlots][2^L] hand-off slots
  // Multi-output launches: one interval-kernel launch propagates n_out <= n_acc consecutive output
  // times from a shared Chebyshev series.  Output j < n_out - 1 is accumulated in
  // xacc[j << n_local], the last in the next psi buffer.  With the observables overlapped
  // (option obs_overlap) the launches of odd groups (q = 1) use the second set,
  // xacc[(xacc_q + j) << n_local], so group g + 1 never writes what group g's observables read.
  double2* xacc;
  int n_acc;
  int xacc_q;             // 0, or n_acc - 1: intermediate outputs per launch-parity set
  // real-component mode (dse_real.hip): the register's tables, its [a | b] input and the
  // per-output, per-component propagator sums
  const struct RealTab* rtab;
  double* rin;
  double2* racc;
};

// ---- spanning registers (dse_span.hip): one register over 2^s cooperating workgroups ----------
// A register of n qubits is cut into 2^s tiles of L = n - s bits (the top s qubits index the
// tile), one workgroup per tile and compute unit, so one register's Chebyshev chain runs on 2^s
// CUs.  In a tile, thread t of NT = 2^(L - RB) owns the R = 2^RB amplitudes x = r * NT + t.
constexpr int kSpanMaxTop = 4;   // top (tile-index) bits: up to 16 workgroups per register
constexpr int kSpanWaves = 16;   // hand-off flags per tile: one per wave (<= 1024 threads)
constexpr int kSpanMaxIt = 160;  // fused-loop iteration rows (dv2): TB x (4 + pairs per iteration)
constexpr int kSpanMaxOps = kSpanMaxTop + kSpanMaxTop * (kSpanMaxTop - 1) / 2;
// One cross-tile operand of every tile's H application (phase 4 of k_span):
//   kind 0  u_b of the partner h ^ e_b (its slot b): flip_b w + sum_j g_jb [x_j == h_b] w(x ^ e_j)
//   kind 1  the partner's raw w_{k-1} under the drive flip of top bit b (no crossing pairs)
//   kind 2  the raw w_{k-1} of the partner h ^ e_b ^ e_b2: pair (b, b2), applies iff h_b == h_b2
struct alignas(16) SpanOp {
  int kind, b, b2;
  uint32_t pmask;  // partner tile = h ^ pmask
  double c[4];     // kind 1: re0 im0 re1 im1 (by this tile's bit b); kind 2: c[0] = g
};
struct alignas(16) SpanTab {
  double rr_g[6];                   // pairs among register bits (rr_index order)
  double rflip[4][4];               // drive flips on register bits (re0 im0 re1 im1)
  double ug[kSpanMaxTop][16];       // u pre-pass: g_{j,b} for tile bits j < L
  double uflip[kSpanMaxTop][4];     // drive flip of top bit b
  SpanOp ops[kSpanMaxOps];
  int rflip_mask, u_mask, n_ops, need_raw;  // need_raw: some operand reads a partner's raw w
  int n_it, pad[3];
  // iteration j (thread bit j): [0] re0 im0, [1] re1 im1 (drive of j by output value t_j),
  // [2] [3] pairs (j, register bit 0..3), [4 + q] thread pair q of the iteration (mask bits, g)
  double2 it[kSpanMaxIt];
};
// Per-context options of the persistent kernels' cross-workgroup hand-offs, passed with every launch
// (kernel arguments: distinct contexts on one process stay independent)
struct HandoffKnobs {
  int spin_limit = 1 << 22;  // polls of a partner's flag before the hand-off is declared failed
                             // (s_sleep 1 between polls; rounds, not time: include/dse.h); < 0: every wait fails at once
                             // (tests: exercises the fallback to the streaming kernels)
  int fences = 0;            // k_interval: 1 adds an agent release / acquire around each flag
};
struct SpanDesc {
  const SpanTab* tab;
  double2* slots;  // [2^s tiles][s + 1 operand kinds: u_0..u_{s-1}, raw][kXSlots][2^L]
  int* flags;      // [2^s tiles][kSpanWaves]: last term each wave of the tile published
  int s, L;
};
hipError_t launch_span(int L, int RB, bool imag, const DevProb* probs, const SpanDesc* sdesc,
                       const int2* items, int n_items, int q, int set, int n_out, int* err,
                       HandoffKnobs hk, hipStream_t st);
bool span_supported(int L, int RB);
hipError_t set_span_ablate(int mask);
hipError_t set_real_ablate(int mask);
hipError_t span_occupancy(int L, int RB, bool imag, int* blocks_per_cu);

// ---- real-component registers (dse_real.hip) ------------------------------------------------
// With every drive purely imaginary (the sweep's phase pi/2) H' = D H D^dagger, D|x> = i^|x| |x>, is
// REAL symmetric, so T_k(H') maps real vectors to real vectors: the rotated state phi = a + i b
// evolves as two independent real Chebyshev recurrences, T_k(H~') a and T_k(H~') b, whose complex
// propagator sums acc_c = sum_k c_k T_k c give phi(t + tau) = acc_a + i acc_b.  One workgroup per
// real component holds the WHOLE register in LDS (2^14 x 8 B = 128 KiB): no cross-workgroup
// hand-off inside a launch.  Thread t of 512 owns rows x = r * 512 + t, r < R = 2^(n - 9).
constexpr int kRealRB = 5;                  // register bits at n = 14 (R = 32 rows per thread)
constexpr int kRealRegPairs = kRealRB * (kRealRB - 1) / 2;
__host__ __device__ constexpr int real_rr_index(int a, int b) {  // a < b < kRealRB
  return a * (2 * kRealRB - a - 1) / 2 + (b - a - 1);
}
struct alignas(16) RealTab {
  double rr_g[kRealRegPairs];  // rotated pair coefficients (-g) among register bits
  double rflip[kRealRB][2];    // rotated drive of register bit i, by output value (0, 1)
  uint64_t x0;                 // psi(t0) = e_x0
  int x0pop;                   // popcount(x0): psi = i^{|x0| - |x|} phi
  int rflip_mask;
  // coefficient row of iteration j (thread bit j), as doubles: the rotated drive of j by output
  // value (2), the rotated pairs (j, register bit 0..5) (6), the iteration's 4 thread pairs in the
  // canonical schedule (span_pair_mask) (4)
  double2 it[9 * 6];
};
// real_c (per problem, real mode): rin = [a | b] (2 x 2^n doubles), racc = [output j][component c]
// blocks of 2^n complex propagator sums
hipError_t launch_real(const DevProb* probs, const int2* items, int n_items, int set, int n_out,
                       hipStream_t st);
// psi = i^{|x0| - |x|} (acc_a + i acc_b) of every output (into the state buffer / intermediate
// outputs k_obs reads) and, from the last output, the next interval's [a | b]
hipError_t launch_real_combine(const DevProb* probs, const int2* items, int n_items, int q, int n_out,
                               hipStream_t st);
hipError_t real_occupancy(int* blocks_per_cu);
hipError_t launch_real_init(const DevProb* probs, const int2* items, int n_items, hipStream_t st);

// Coefficient row of output j of offset set `set`: kcap1 + 1 entries, row[0].x = the degree d of
// that output's series, row[1 + k] = a_k for k = 0..d (zero beyond): 16 B per term.
__host__ __device__ __forceinline__ const double2* coef_row(const DevProb& P, int set, int j) {
  return P.coef + ((size_t)set * P.n_acc + j) * (size_t)(P.kcap1 + 1);
}
// Terms accumulated into a propagator sum at term k (see CoefK), for the update phase ph (0..2):
// 2 at k = 1 (a_0 w_0 + a_1 w_1); then at every k >= 2 with (k - 1 - ph) = 0 mod 3 the terms since
// the previous update (3; at the first update of phase 1 / 2 one / two), and the terms left over at
// k = d; else 0.  A term can reach w_{k-2}, w_{k-1}, w_k, so no gap exceeds 3.  Phase 0 is the
// original schedule (updates at k = 1, 4, 7, ...); k_span staggers output j to phase j % 3, so at
// most ceil(M / 3) of its M sums are read-modify-written in one term.
__host__ __device__ __forceinline__ int coef_nterm(int k, int d, int ph = 0) {
  if (k > d) return 0;
  if (k == 1) return 2;
  const int t = ((k - 1 - ph) % 3 + 3) % 3;
  int last = t == 0 ? k - 3 : k - t;  // the previous update of phase ph at k' >= 2, else 1
  if (last < 2) last = 1;
  return (t == 0 || k == d) ? k - last : 0;
}
// (scalar loads: the row is read-only during a launch and uniform across the workgroup)
__device__ __forceinline__ CoefK coef_at(const double2* row, int k) {
  typedef const __attribute__((address_space(4))) double* kptr;
  const kptr r = (kptr)row;
  const int nt = coef_nterm(k, (int)r[0]);
  CoefK C = {};
  C.upd = nt > 0;
  const size_t o = 2 * (size_t)(k - 1);  // a_{k-2} at row[k - 1]
  C.c[0] = nt >= 3 ? make_double2(r[o], r[o + 1]) : make_double2(0.0, 0.0);
  C.c[1] = nt >= 2 ? make_double2(r[o + 2], r[o + 3]) : make_double2(0.0, 0.0);
  C.c[2] = nt >= 1 ? make_double2(r[o + 4], r[o + 5]) : make_double2(0.0, 0.0);
  return C;
}

// Global tile hp of the role-`role` vector: local buffer or a partner shard's.
__device__ __forceinline__ const double2* tile_ptr(const DevProb& P, int role, uint32_t hp) {
  const uint32_t gm = (hp ^ P.h_base) >> P.tbl;
  const double2* b = gm ? P.rbuf[gm][role] : P.buf[role];
  return b + ((size_t)(hp & ((1u << P.tbl) - 1u)) << P.L);
}

hipError_t launch_step(int L, int mode, const DevProb* probs, const int2* items, int n_items,
                       int k, int q, int set, hipStream_t st);
// diagnostics builds only (-DDSE_DIAG, e.g. DSE_EXTRA_FLAGS for a tools/ variant library): kernel
// section ablation masks; the product library returns hipErrorNotSupported
hipError_t set_ablate(int mask);
hipError_t set_ablate_interval(int mask);
bool interval_supported(int L);
// resident workgroups of k_interval<L> per compute unit (occupancy query)
hipError_t interval_occupancy(int L, bool imag, int* blocks_per_cu);
// imag: every drive coefficient of the launched problems is purely imaginary (HostProblem::imag)
// colstride > 0: column mode (one-tile register, item.y = column, buffers offset by column *
// colstride amplitudes): every column propagated over the interval of coefficient set `set`
hipError_t launch_interval(int L, bool imag, const DevProb* probs, const int2* items, int n_items, int q,
                           int set, int n_out, int* flags, int* err, HandoffKnobs hk, hipStream_t st,
                           long colstride = 0);
// zeroes the interval kernel's hand-off flags of the given items (before a 2-tile launch)
hipError_t zero_flags(const int2* items, int n_items, int* flags, hipStream_t st);
// psi(t0) of many registers in one launch: entry i zeroes ptr[0 .. n) and sets ptr[one_at] = 1
// (one_at < 0: the basis state lies in another shard)
struct BasisInit {
  double2* ptr;
  uint64_t n;
  int64_t one_at;
};
hipError_t launch_basis_init(const BasisInit* list, int n_entries, uint64_t max_amps, hipStream_t st);
// observables of n_out outputs of a group (grid.y): output j < n_out - 1 from intermediate
// accumulator j, the last from state buffer role bsel; output j's partials at partial + j * out_stride
hipError_t launch_obs(int L, const DevProb* probs, const int2* items, int n_items, int bsel,
                      double* partial, hipStream_t st, int n_out = 1, size_t out_stride = 0,
                      int xq = 0);  // xq: launch parity of the intermediate outputs (xacc_q set)
// partial[2 * block + {0, 1}] = block sums of Re(conj(a) b) and |a|^2 over n amplitudes
hipError_t launch_dot(const double2* a, const double2* b, size_t n, double* partial, int blocks,
                      hipStream_t st);

}  // namespace dse
