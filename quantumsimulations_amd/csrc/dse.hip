// dse.hip -- MI355X (gfx950) state-vector engine for the driven heteronuclear dipolar spin
// ensemble of TimHarrelson/QuantumSimulations (dipolar_ensemble_with_rare.py).
//
// Replaces qt.sesolve(H, psi0, t, e_ops) (dipolar_ensemble_with_rare.py:653-666) and the CSR
// operator algebra feeding it (:453-588) for many independent evolutions per device.
//
// Kernels
//   k_step<L, MODE>  one application of H to 2^L-amplitude tiles, matrix-free, fused with the
//                    Chebyshev three-term recurrence and the propagator accumulation
//                    (MODE_APPLY: plain H psi test hook; MODE_FIRST: k = 1; MODE_GEN: k >= 2).
//   k_obs<L>         the six <I> expectations + ||psi||^2 of a state, per-tile partial sums.
//
// Data layout in HBM: every problem owns three state buffers of 2^n double2 (interleaved
// complex, AoS so one lane moves 16 B).  A tile is the 2^L amplitudes sharing the top n-L
// index bits; one workgroup stages one tile of w_{k-1} in LDS.  All H terms among tile bits
// (diagonal, drive flips, pair flips) gather from LDS; terms touching the n-L "high" bits read
// the partner tile straight from global memory (coalesced: the XOR permutes inside aligned
// 1 KiB blocks).  The rare spin is mapped to the top bit by the host, so its only high-bit term
// is its own drive flip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/dse.h"

#define DSE_LIKELY(x) __builtin_expect(!!(x), 1)

namespace {

enum { MODE_APPLY = 0, MODE_FIRST = 1, MODE_GEN = 2 };

// A pair flip or a drive flip, split into the in-tile and tile-index parts of its mask.
//   pair : condition  bit_i(x) == bit_j(x)  <=>  popc(x_lo & mask_lo) + popc(h & tile_xor) even
//   flip : output bit value v = parity(x_lo & mask_lo) ^ parity(h & tile_xor)
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

struct DevProb {
  double2* buf[3];
  const double* zzlo;     // [2^L]  sum_{i<j<L} zz_ij s_i s_j
  const double* field;    // [n]
  const double* zz;       // [n*n]
  const DPair* pairs_lo;  // both bits inside the tile
  const DPair* pairs_hi;  // at least one bit above the tile
  const DFlip* flips_lo;
  const DFlip* flips_hi;
  const double2* coef;    // [n_sets][kcap1] Chebyshev coefficients a_k
  uint64_t sea_mask;
  double shift;
  double beta;            // spectral centre
  double s1;              // 1/alpha
  int n, L;
  int n_pairs_lo, n_pairs_hi, n_flips_lo, n_flips_hi;
  int kcap1;
  int rare_bit;
  int n_sea;
  int pad;
};

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
k_step(const DevProb* __restrict__ probs, const int2* __restrict__ items, int k, int q, int set) {
  using G = Geo<L>;
  constexpr int T = G::T, NT = G::NT, R = G::R;
  __shared__ double2 s_w[T];
  __shared__ double s_c[L + 1];

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const int tid = threadIdx.x;
  const bool live = (T >= NT) || (tid < T);

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
  if (MODE == MODE_APPLY) {
#pragma unroll
    for (int r = 0; r < R; ++r) wdst[base + r * NT + tid] = out[r];
  } else if (MODE == MODE_FIRST) {
    const double s1 = P.s1;
    const double2 a0 = P.coef[set * P.kcap1 + 0];
    const double2 a1 = P.coef[set * P.kcap1 + 1];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t x = base + r * NT + tid;
      double2 w;
      w.x = s1 * out[r].x;
      w.y = s1 * out[r].y;
      wdst[x] = w;
      double2 a = make_double2(0.0, 0.0);
      a = cmad(a, a0.x, a0.y, own[r]);
      a = cmad(a, a1.x, a1.y, w);
      acc_b[x] = a;
    }
  } else {
    const double s2 = 2.0 * P.s1;
    const double2 ak = P.coef[set * P.kcap1 + k];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t x = base + r * NT + tid;
      const double2 prev = wdst[x];
      double2 w;
      w.x = fma(s2, out[r].x, -prev.x);
      w.y = fma(s2, out[r].y, -prev.y);
      wdst[x] = w;
      acc_b[x] = cmad(acc_b[x], ak.x, ak.y, w);
    }
  }
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
// launch dispatch over the tile size
// ------------------------------------------------------------------------------------------
constexpr int kMinTile = 1, kMaxTile = 13;

template <int L>
hipError_t launch_step_L(int mode, const DevProb* probs, const int2* items, int n_items, int k,
                         int q, int set, hipStream_t st) {
  dim3 grid(n_items), block(Geo<L>::NT);
  if (mode == MODE_APPLY)
    hipLaunchKernelGGL((k_step<L, MODE_APPLY>), grid, block, 0, st, probs, items, k, q, set);
  else if (mode == MODE_FIRST)
    hipLaunchKernelGGL((k_step<L, MODE_FIRST>), grid, block, 0, st, probs, items, k, q, set);
  else
    hipLaunchKernelGGL((k_step<L, MODE_GEN>), grid, block, 0, st, probs, items, k, q, set);
  return hipGetLastError();
}

template <int L>
hipError_t launch_obs_L(const DevProb* probs, const int2* items, int n_items, int bsel,
                        double* partial, hipStream_t st) {
  hipLaunchKernelGGL((k_obs<L>), dim3(n_items), dim3(Geo<L>::NT), 0, st, probs, items, bsel, partial);
  return hipGetLastError();
}

#define DSE_TILE_CASES(X) \
  X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13)

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

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
struct HostProblem {
  int n = 0;
  std::vector<double> field, zz, pair, flip;
  double shift = 0.0;
  uint64_t psi0 = 0, sea_mask = 0;
  int rare_bit = -1;
  double rare_z = 0.0;
  double e_min = 0.0, e_max = 0.0;
  // device
  int L = 0;
  int64_t n_tiles = 0;
  double2* buf[3] = {nullptr, nullptr, nullptr};
  void* tables = nullptr;  // zzlo | field | zz | pairs | flips
  double2* coef = nullptr;
  size_t coef_bytes = 0;
  int n_pairs_lo = 0, n_pairs_hi = 0, n_flips_lo = 0, n_flips_hi = 0;
  int degree = 1;  // Chebyshev degree of the current evolve
};

struct Group {  // problems sharing one tile size
  int L = 0;
  std::vector<int> probs;
  std::vector<int2> items_by_prob;  // problem-major, tiles in order
  std::vector<int64_t> item_off;    // offset of each problem's items (indexed by position in probs)
  int2* d_items_by_prob = nullptr;
  int2* d_items_sorted = nullptr;
  std::vector<int> active;          // active[k] = items with degree >= k (sorted list prefix)
};

}  // namespace

struct dse_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::vector<HostProblem> probs;
  std::vector<Group> groups;
  DevProb* d_probs = nullptr;
  std::vector<DevProb> h_desc;  // host mirror of d_probs
  double* d_partial = nullptr;
  size_t partial_slots = 0;
  int64_t total_items = 0;
  bool prepared = false;
  bool evolved = false;
  int last_q = 0;  // parity of the interval after the last evolve
  int tile_bits = 12;
  bool time_kernels = true;
  double max_degree = 2e6;
  std::vector<hipEvent_t> ev[2];
};

namespace {

thread_local std::string g_create_err;

int fail(dse_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIPC(expr)                                                                      \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return fail(ctx, DSE_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

void free_device(dse_ctx* ctx) {
  for (auto& p : ctx->probs) {
    for (auto& b : p.buf)
      if (b) (void)hipFree(b), b = nullptr;
    if (p.tables) (void)hipFree(p.tables), p.tables = nullptr;
    if (p.coef) (void)hipFree(p.coef), p.coef = nullptr;
    p.coef_bytes = 0;
  }
  for (auto& g : ctx->groups) {
    if (g.d_items_by_prob) (void)hipFree(g.d_items_by_prob);
    if (g.d_items_sorted) (void)hipFree(g.d_items_sorted);
  }
  ctx->groups.clear();
  if (ctx->d_probs) (void)hipFree(ctx->d_probs), ctx->d_probs = nullptr;
  if (ctx->d_partial) (void)hipFree(ctx->d_partial), ctx->d_partial = nullptr;
  ctx->partial_slots = 0;
  ctx->prepared = false;
  ctx->evolved = false;
}

size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Builds per-problem device tables and state buffers, the device descriptor array and the
// per-tile-size item lists.
int prepare(dse_ctx* ctx) {
  if (ctx->prepared) return DSE_OK;
  if (ctx->probs.empty()) return fail(ctx, DSE_ERR_STATE, "no problems added");
  std::vector<DevProb> dp(ctx->probs.size());
  std::map<int, int> group_of_L;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    HostProblem& p = ctx->probs[pi];
    const int n = p.n;
    const int L = std::max(std::min(n, ctx->tile_bits), std::max(kMinTile, n - 32));
    if (L > kMaxTile) return fail(ctx, DSE_ERR_ARG, "problem too large for the tile range");
    p.L = L;
    p.n_tiles = int64_t(1) << (n - L);
    const size_t T = size_t(1) << L;
    // tables
    std::vector<double> zzlo(T, 0.0);
    for (size_t x = 0; x < T; ++x) {
      double d = 0.0;
      for (int i = 0; i < L; ++i) {
        const double si = 0.5 - (double)((x >> i) & 1);
        for (int j = i + 1; j < L; ++j) d += p.zz[i * n + j] * (si * (0.5 - (double)((x >> j) & 1)));
      }
      zzlo[x] = d;
    }
    std::vector<DPair> plo, phi;
    for (int i = 0; i < n; ++i)
      for (int j = i + 1; j < n; ++j) {
        const double g = p.pair[i * n + j];
        if (g == 0.0) continue;
        const uint64_t m = (uint64_t(1) << i) | (uint64_t(1) << j);
        DPair q;
        q.mask_lo = (uint32_t)(m & ((uint64_t(1) << L) - 1));
        q.tile_xor = (uint32_t)(m >> L);
        q.g = g;
        (q.tile_xor ? phi : plo).push_back(q);
      }
    std::vector<DFlip> flo, fhi;
    for (int b = 0; b < n; ++b) {
      const double* f = &p.flip[4 * b];
      if (f[0] == 0.0 && f[1] == 0.0 && f[2] == 0.0 && f[3] == 0.0) continue;
      const uint64_t m = uint64_t(1) << b;
      DFlip q;
      q.mask_lo = (uint32_t)(m & ((uint64_t(1) << L) - 1));
      q.tile_xor = (uint32_t)(m >> L);
      q.re0 = f[0];
      q.im0 = f[1];
      q.re1 = f[2];
      q.im1 = f[3];
      q.pad = 0.0;
      (q.tile_xor ? fhi : flo).push_back(q);
    }
    p.n_pairs_lo = (int)plo.size();
    p.n_pairs_hi = (int)phi.size();
    p.n_flips_lo = (int)flo.size();
    p.n_flips_hi = (int)fhi.size();
    const size_t o_zzlo = 0;
    const size_t o_field = align_up(o_zzlo + T * sizeof(double), 256);
    const size_t o_zz = align_up(o_field + n * sizeof(double), 256);
    const size_t o_plo = align_up(o_zz + size_t(n) * n * sizeof(double), 256);
    const size_t o_phi = align_up(o_plo + plo.size() * sizeof(DPair), 256);
    const size_t o_flo = align_up(o_phi + phi.size() * sizeof(DPair), 256);
    const size_t o_fhi = align_up(o_flo + flo.size() * sizeof(DFlip), 256);
    const size_t total = align_up(o_fhi + fhi.size() * sizeof(DFlip), 256);
    std::vector<char> blob(total, 0);
    std::memcpy(blob.data() + o_zzlo, zzlo.data(), T * sizeof(double));
    std::memcpy(blob.data() + o_field, p.field.data(), n * sizeof(double));
    std::memcpy(blob.data() + o_zz, p.zz.data(), size_t(n) * n * sizeof(double));
    if (!plo.empty()) std::memcpy(blob.data() + o_plo, plo.data(), plo.size() * sizeof(DPair));
    if (!phi.empty()) std::memcpy(blob.data() + o_phi, phi.data(), phi.size() * sizeof(DPair));
    if (!flo.empty()) std::memcpy(blob.data() + o_flo, flo.data(), flo.size() * sizeof(DFlip));
    if (!fhi.empty()) std::memcpy(blob.data() + o_fhi, fhi.data(), fhi.size() * sizeof(DFlip));
    if (hipMalloc(&p.tables, total) != hipSuccess) {
      free_device(ctx);
      return fail(ctx, DSE_ERR_OOM, "device allocation of coefficient tables failed");
    }
    HIPC(hipMemcpy(p.tables, blob.data(), total, hipMemcpyHostToDevice));
    const size_t vbytes = (size_t(1) << n) * sizeof(double2);
    for (auto& b : p.buf) {
      if (hipMalloc(&b, vbytes) != hipSuccess) {
        free_device(ctx);
        return fail(ctx, DSE_ERR_OOM, "device allocation of state buffers failed (" +
                                          std::to_string(3 * vbytes) + " bytes per problem)");
      }
      HIPC(hipMemsetAsync(b, 0, vbytes, ctx->stream));
    }
    char* tb = static_cast<char*>(p.tables);
    DevProb& d = dp[pi];
    std::memset(&d, 0, sizeof(d));
    for (int i = 0; i < 3; ++i) d.buf[i] = p.buf[i];
    d.zzlo = reinterpret_cast<const double*>(tb + o_zzlo);
    d.field = reinterpret_cast<const double*>(tb + o_field);
    d.zz = reinterpret_cast<const double*>(tb + o_zz);
    d.pairs_lo = reinterpret_cast<const DPair*>(tb + o_plo);
    d.pairs_hi = reinterpret_cast<const DPair*>(tb + o_phi);
    d.flips_lo = reinterpret_cast<const DFlip*>(tb + o_flo);
    d.flips_hi = reinterpret_cast<const DFlip*>(tb + o_fhi);
    d.coef = nullptr;
    d.sea_mask = p.sea_mask;
    d.shift = p.shift;
    d.beta = 0.0;
    d.s1 = 1.0;
    d.n = n;
    d.L = L;
    d.n_pairs_lo = p.n_pairs_lo;
    d.n_pairs_hi = p.n_pairs_hi;
    d.n_flips_lo = p.n_flips_lo;
    d.n_flips_hi = p.n_flips_hi;
    d.kcap1 = 0;
    d.rare_bit = p.rare_bit;
    d.n_sea = __builtin_popcountll(p.sea_mask);
    auto gi = group_of_L.find(L);
    if (gi == group_of_L.end()) {
      gi = group_of_L.emplace(L, (int)ctx->groups.size()).first;
      ctx->groups.emplace_back();
      ctx->groups.back().L = L;
    }
    ctx->groups[gi->second].probs.push_back((int)pi);
  }
  if (hipMalloc(&ctx->d_probs, dp.size() * sizeof(DevProb)) != hipSuccess) {
    free_device(ctx);
    return fail(ctx, DSE_ERR_OOM, "device allocation of descriptors failed");
  }
  HIPC(hipMemcpy(ctx->d_probs, dp.data(), dp.size() * sizeof(DevProb), hipMemcpyHostToDevice));
  ctx->h_desc = dp;
  ctx->total_items = 0;
  for (auto& g : ctx->groups) {
    g.items_by_prob.clear();
    g.item_off.clear();
    for (int pi : g.probs) {
      g.item_off.push_back((int64_t)g.items_by_prob.size());
      for (int64_t t = 0; t < ctx->probs[pi].n_tiles; ++t) g.items_by_prob.push_back(make_int2(pi, (int)t));
    }
    const size_t bytes = g.items_by_prob.size() * sizeof(int2);
    if (hipMalloc(&g.d_items_by_prob, bytes) != hipSuccess || hipMalloc(&g.d_items_sorted, bytes) != hipSuccess) {
      free_device(ctx);
      return fail(ctx, DSE_ERR_OOM, "device allocation of item lists failed");
    }
    HIPC(hipMemcpy(g.d_items_by_prob, g.items_by_prob.data(), bytes, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(g.d_items_sorted, g.items_by_prob.data(), bytes, hipMemcpyHostToDevice));
    ctx->total_items += (int64_t)g.items_by_prob.size();
  }
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->prepared = true;
  return DSE_OK;
}

int ensure_partial(dse_ctx* ctx, size_t slots) {
  if (ctx->partial_slots >= slots) return DSE_OK;
  if (ctx->d_partial) (void)hipFree(ctx->d_partial), ctx->d_partial = nullptr;
  if (hipMalloc(&ctx->d_partial, slots * ctx->total_items * 8 * sizeof(double)) != hipSuccess)
    return fail(ctx, DSE_ERR_OOM, "device allocation of observable partials failed");
  ctx->partial_slots = slots;
  return DSE_OK;
}

// Launches the observable kernel for every problem on buffer bsel into partial slot `slot`.
int launch_obs_all(dse_ctx* ctx, int bsel, size_t slot) {
  int64_t off = 0;
  for (auto& g : ctx->groups) {
    double* dst = ctx->d_partial + (slot * ctx->total_items + off) * 8;
    HIPC(launch_obs(g.L, ctx->d_probs, g.d_items_by_prob, (int)g.items_by_prob.size(), bsel, dst, ctx->stream));
    off += (int64_t)g.items_by_prob.size();
  }
  return DSE_OK;
}

// Reduces `nslots` partial slots (host copy) into obs_out[p][7][n_t] at time offset t0.
void reduce_partials(dse_ctx* ctx, const std::vector<double>& h, size_t nslots, size_t t0, int n_t,
                     double* obs_out) {
  int64_t off = 0;
  for (auto& g : ctx->groups) {
    for (size_t gp = 0; gp < g.probs.size(); ++gp) {
      const int pi = g.probs[gp];
      const HostProblem& P = ctx->probs[pi];
      const int64_t first = off + g.item_off[gp];
      for (size_t s = 0; s < nslots; ++s) {
        double v[7] = {0, 0, 0, 0, 0, 0, 0};
        const double* row = h.data() + (s * ctx->total_items + first) * 8;
        for (int64_t t = 0; t < P.n_tiles; ++t)
          for (int j = 0; j < 7; ++j) v[j] += row[t * 8 + j];
        const double n2 = v[6];
        const double inv = n2 > 0.0 ? 1.0 / n2 : 0.0;
        double* o = obs_out + (size_t)pi * DSE_N_OBS * n_t + (t0 + s);
        o[0 * (size_t)n_t] = v[0] * inv;
        o[1 * (size_t)n_t] = v[1] * inv;
        o[2 * (size_t)n_t] = v[2] * inv;
        o[3 * (size_t)n_t] = P.rare_bit >= 0 ? v[3] * inv : P.rare_z;
        o[4 * (size_t)n_t] = P.rare_bit >= 0 ? v[4] * inv : 0.0;
        o[5 * (size_t)n_t] = P.rare_bit >= 0 ? v[5] * inv : 0.0;
        o[6 * (size_t)n_t] = std::sqrt(n2);
      }
    }
    off += (int64_t)g.items_by_prob.size();
  }
}

int flush_partials(dse_ctx* ctx, size_t nslots, size_t t0, int n_t, double* obs_out) {
  std::vector<double> h(nslots * ctx->total_items * 8);
  HIPC(hipMemcpyAsync(h.data(), ctx->d_partial, h.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  reduce_partials(ctx, h, nslots, t0, n_t, obs_out);
  return DSE_OK;
}

int ensure_events(dse_ctx* ctx, size_t per_pool) {
  for (int p = 0; p < 2; ++p) {
    while (ctx->ev[p].size() < 2 * per_pool) {
      hipEvent_t e;
      HIPC(hipEventCreate(&e));
      ctx->ev[p].push_back(e);
    }
  }
  return DSE_OK;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------
extern "C" {

int dse_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* dse_create_error(void) { return g_create_err.c_str(); }

dse_ctx* dse_create(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    g_create_err = "no HIP device available";
    return nullptr;
  }
  if (device < 0 || device >= n) {
    g_create_err = "device index out of range";
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    g_create_err = "hipSetDevice failed";
    return nullptr;
  }
  dse_ctx* ctx = new (std::nothrow) dse_ctx();
  if (!ctx) {
    g_create_err = "out of host memory";
    return nullptr;
  }
  ctx->device = device;
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    g_create_err = "hipStreamCreate failed";
    delete ctx;
    return nullptr;
  }
  return ctx;
}

void dse_destroy(dse_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  free_device(ctx);
  for (auto& pool : ctx->ev)
    for (auto e : pool) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* dse_last_error(const dse_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int dse_set_option(dse_ctx* ctx, const char* key, double value) {
  if (!ctx || !key) return DSE_ERR_ARG;
  const std::string k(key);
  if (k == "tile_bits") {
    if (!(value >= 1 && value <= kMaxTile)) return fail(ctx, DSE_ERR_ARG, "tile_bits must be in 1..13");
    (void)hipSetDevice(ctx->device);
    free_device(ctx);
    ctx->tile_bits = (int)value;
  } else if (k == "time_kernels") {
    ctx->time_kernels = value != 0.0;
  } else if (k == "max_degree") {
    if (!(value >= 1)) return fail(ctx, DSE_ERR_ARG, "max_degree must be >= 1");
    ctx->max_degree = value;
  } else {
    return fail(ctx, DSE_ERR_ARG, "unknown option " + k);
  }
  return DSE_OK;
}

int dse_add_problem(dse_ctx* ctx, int n, const double* field, const double* zz, const double* pair,
                    const double* flip, double shift, uint64_t psi0_index, uint64_t sea_mask,
                    int rare_bit, double rare_z_const) {
  if (!ctx) return DSE_ERR_ARG;
  if (n < 1 || n > DSE_MAX_QUBITS) return fail(ctx, DSE_ERR_ARG, "n_qubits out of range 1..34");
  if (!field || !zz || !pair || !flip) return fail(ctx, DSE_ERR_ARG, "null coefficient table");
  const uint64_t dim = uint64_t(1) << n;
  if (psi0_index >= dim) return fail(ctx, DSE_ERR_ARG, "psi0_index >= 2^n");
  if (n < 64 && (sea_mask >> n) != 0) return fail(ctx, DSE_ERR_ARG, "sea_mask has bits >= n");
  if (rare_bit >= n || rare_bit < -1) return fail(ctx, DSE_ERR_ARG, "rare_bit out of range");
  HostProblem p;
  p.n = n;
  p.field.assign(field, field + n);
  p.zz.assign(zz, zz + size_t(n) * n);
  p.pair.assign(pair, pair + size_t(n) * n);
  p.flip.assign(flip, flip + 4 * size_t(n));
  for (double v : p.field)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite field");
  for (double v : p.zz)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite zz");
  for (double v : p.pair)
    if (!std::isfinite(v)) return fail(ctx, DSE_ERR_ARG, "non-finite pair");
  for (int b = 0; b < n; ++b) {
    const double* f = &p.flip[4 * b];
    if (!(std::isfinite(f[0]) && std::isfinite(f[1]) && std::isfinite(f[2]) && std::isfinite(f[3])))
      return fail(ctx, DSE_ERR_ARG, "non-finite flip");
    if (std::fabs(f[0] - f[2]) > 1e-12 * (std::fabs(f[0]) + 1e-300) + 1e-300 ||
        std::fabs(f[1] + f[3]) > 1e-12 * (std::fabs(f[1]) + 1e-300) + 1e-300)
      return fail(ctx, DSE_ERR_ARG, "flip coefficients are not Hermitian (need c1 = conj(c0))");
  }
  if (!std::isfinite(shift)) return fail(ctx, DSE_ERR_ARG, "non-finite shift");
  p.shift = shift;
  p.psi0 = psi0_index;
  p.sea_mask = sea_mask;
  p.rare_bit = rare_bit;
  p.rare_z = rare_z_const;
  dse_spectral_bounds(n, p.field.data(), p.zz.data(), p.pair.data(), p.flip.data(), shift, &p.e_min, &p.e_max);
  (void)hipSetDevice(ctx->device);
  free_device(ctx);  // device layout is rebuilt lazily
  ctx->probs.push_back(std::move(p));
  return (int)ctx->probs.size() - 1;
}

int dse_num_problems(const dse_ctx* ctx) { return ctx ? (int)ctx->probs.size() : DSE_ERR_ARG; }

int dse_clear(dse_ctx* ctx) {
  if (!ctx) return DSE_ERR_ARG;
  (void)hipSetDevice(ctx->device);
  free_device(ctx);
  ctx->probs.clear();
  return DSE_OK;
}

int dse_apply_h(dse_ctx* ctx, int problem, const double* psi_in, double* psi_out) {
  if (!ctx) return DSE_ERR_ARG;
  if (problem < 0 || problem >= (int)ctx->probs.size()) return fail(ctx, DSE_ERR_ARG, "bad problem id");
  if (!psi_in || !psi_out) return fail(ctx, DSE_ERR_ARG, "null state");
  HIPC(hipSetDevice(ctx->device));
  int rc = prepare(ctx);
  if (rc) return rc;
  HostProblem& P = ctx->probs[problem];
  const size_t bytes = (size_t(1) << P.n) * sizeof(double2);
  HIPC(hipMemcpyAsync(P.buf[0], psi_in, bytes, hipMemcpyHostToDevice, ctx->stream));
  for (auto& g : ctx->groups) {
    for (size_t gp = 0; gp < g.probs.size(); ++gp) {
      if (g.probs[gp] != problem) continue;
      HIPC(launch_step(g.L, MODE_APPLY, ctx->d_probs, g.d_items_by_prob + g.item_off[gp],
                       (int)P.n_tiles, 0, 0, 0, ctx->stream));
    }
  }
  HIPC(hipMemcpyAsync(psi_out, P.buf[1], bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->evolved = false;
  return DSE_OK;
}

int dse_observables(dse_ctx* ctx, int problem, const double* psi, double* obs7) {
  if (!ctx) return DSE_ERR_ARG;
  if (problem < 0 || problem >= (int)ctx->probs.size()) return fail(ctx, DSE_ERR_ARG, "bad problem id");
  if (!psi || !obs7) return fail(ctx, DSE_ERR_ARG, "null pointer");
  HIPC(hipSetDevice(ctx->device));
  int rc = prepare(ctx);
  if (rc) return rc;
  if ((rc = ensure_partial(ctx, 1))) return rc;
  HostProblem& P = ctx->probs[problem];
  const size_t bytes = (size_t(1) << P.n) * sizeof(double2);
  HIPC(hipMemcpyAsync(P.buf[0], psi, bytes, hipMemcpyHostToDevice, ctx->stream));
  int64_t off = 0;
  for (auto& g : ctx->groups) {
    for (size_t gp = 0; gp < g.probs.size(); ++gp) {
      if (g.probs[gp] != problem) continue;
      double* dst = ctx->d_partial + (off + g.item_off[gp]) * 8;
      HIPC(launch_obs(g.L, ctx->d_probs, g.d_items_by_prob + g.item_off[gp], (int)P.n_tiles, 0, dst, ctx->stream));
    }
    off += (int64_t)g.items_by_prob.size();
  }
  std::vector<double> h(ctx->total_items * 8);
  HIPC(hipMemcpyAsync(h.data(), ctx->d_partial, h.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  // reduce only this problem
  off = 0;
  for (auto& g : ctx->groups) {
    for (size_t gp = 0; gp < g.probs.size(); ++gp) {
      if (g.probs[gp] != problem) continue;
      double v[7] = {0, 0, 0, 0, 0, 0, 0};
      const double* row = h.data() + (off + g.item_off[gp]) * 8;
      for (int64_t t = 0; t < P.n_tiles; ++t)
        for (int j = 0; j < 7; ++j) v[j] += row[t * 8 + j];
      const double inv = v[6] > 0 ? 1.0 / v[6] : 0.0;
      obs7[0] = v[0] * inv;
      obs7[1] = v[1] * inv;
      obs7[2] = v[2] * inv;
      obs7[3] = P.rare_bit >= 0 ? v[3] * inv : P.rare_z;
      obs7[4] = P.rare_bit >= 0 ? v[4] * inv : 0.0;
      obs7[5] = P.rare_bit >= 0 ? v[5] * inv : 0.0;
      obs7[6] = std::sqrt(v[6]);
    }
    off += (int64_t)g.items_by_prob.size();
  }
  ctx->evolved = false;
  return DSE_OK;
}

int dse_evolve(dse_ctx* ctx, const double* t, int n_t, double tol, double* obs_out, dse_stats* stats) {
  if (!ctx) return DSE_ERR_ARG;
  const auto wall0 = std::chrono::steady_clock::now();
  if (!t || !obs_out) return fail(ctx, DSE_ERR_ARG, "null pointer");
  if (n_t < 1) return fail(ctx, DSE_ERR_ARG, "n_t must be >= 1");
  if (!(tol > 0.0 && tol < 1e-2)) return fail(ctx, DSE_ERR_ARG, "tol must be in (0, 1e-2)");
  for (int i = 0; i < n_t; ++i)
    if (!std::isfinite(t[i])) return fail(ctx, DSE_ERR_ARG, "non-finite time");
  for (int i = 1; i < n_t; ++i)
    if (!(t[i] > t[i - 1])) return fail(ctx, DSE_ERR_ARG, "times must be strictly increasing");
  HIPC(hipSetDevice(ctx->device));
  int rc = prepare(ctx);
  if (rc) return rc;

  // ---- distinct interval lengths -> coefficient sets ----
  std::vector<double> set_dt;
  std::vector<int> set_of(std::max(0, n_t - 1));
  for (int m = 0; m + 1 < n_t; ++m) {
    const double dt = t[m + 1] - t[m];
    int s = -1;
    for (size_t q = 0; q < set_dt.size(); ++q)
      if (set_dt[q] == dt) { s = (int)q; break; }
    if (s < 0) {
      if (set_dt.size() >= 4096) return fail(ctx, DSE_ERR_ARG, "more than 4096 distinct output intervals");
      s = (int)set_dt.size();
      set_dt.push_back(dt);
    }
    set_of[m] = s;
  }
  const int n_sets = std::max<int>(1, (int)set_dt.size());
  if (set_dt.empty()) set_dt.push_back(0.0);

  // ---- Chebyshev coefficients per problem ----
  int max_deg = 1;
  for (size_t pi = 0; pi < ctx->probs.size(); ++pi) {
    HostProblem& P = ctx->probs[pi];
    const double alpha = std::max(0.5 * (P.e_max - P.e_min), 1e-300);
    const double beta = 0.5 * (P.e_max + P.e_min);
    int deg = 1;
    std::vector<std::vector<double>> J(n_sets);
    for (int s = 0; s < n_sets; ++s) {
      const double z = alpha * set_dt[s];
      const int kmax = (int)std::ceil(z + 12.0 * std::cbrt(z + 1.0) + 60.0);
      if (kmax > ctx->max_degree)
        return fail(ctx, DSE_ERR_CONVERGENCE, "Chebyshev degree " + std::to_string(kmax) +
                                                  " exceeds max_degree; use a finer output grid");
      J[s].resize(kmax + 1);
      int d = 1;
      if (dse_bessel_j(z, kmax, J[s].data(), tol, &d) != DSE_OK) return fail(ctx, DSE_ERR_ARG, "bessel failed");
      deg = std::max(deg, d);
    }
    P.degree = deg;
    max_deg = std::max(max_deg, deg);
    const int kcap1 = deg + 1;
    std::vector<double2> coef((size_t)n_sets * kcap1);
    for (int s = 0; s < n_sets; ++s) {
      const double ph = -beta * set_dt[s];
      const std::complex<double> e(std::cos(ph), std::sin(ph));
      std::complex<double> mi(1.0, 0.0);  // (-i)^k
      for (int k = 0; k <= deg; ++k) {
        const double jk = k < (int)J[s].size() ? J[s][k] : 0.0;
        const std::complex<double> a = e * mi * ((k == 0 ? 1.0 : 2.0) * jk);
        coef[(size_t)s * kcap1 + k] = make_double2(a.real(), a.imag());
        mi *= std::complex<double>(0.0, -1.0);
      }
    }
    const size_t cb = coef.size() * sizeof(double2);
    if (cb > P.coef_bytes) {
      if (P.coef) (void)hipFree(P.coef), P.coef = nullptr;
      if (hipMalloc(&P.coef, cb) != hipSuccess) return fail(ctx, DSE_ERR_OOM, "coefficient allocation failed");
      P.coef_bytes = cb;
    }
    HIPC(hipMemcpyAsync(P.coef, coef.data(), cb, hipMemcpyHostToDevice, ctx->stream));
    DevProb& d = ctx->h_desc[pi];
    d.coef = P.coef;
    d.kcap1 = kcap1;
    d.beta = beta;
    d.s1 = 1.0 / alpha;
  }
  HIPC(hipMemcpyAsync(ctx->d_probs, ctx->h_desc.data(), ctx->h_desc.size() * sizeof(DevProb),
                      hipMemcpyHostToDevice, ctx->stream));

  // ---- degree-sorted item lists: items active at step k form a prefix ----
  for (auto& g : ctx->groups) {
    std::vector<int2> sorted = g.items_by_prob;
    std::stable_sort(sorted.begin(), sorted.end(), [&](const int2& a, const int2& b) {
      return ctx->probs[a.x].degree > ctx->probs[b.x].degree;
    });
    HIPC(hipMemcpyAsync(g.d_items_sorted, sorted.data(), sorted.size() * sizeof(int2), hipMemcpyHostToDevice, ctx->stream));
    g.active.assign(max_deg + 2, 0);
    for (int k = 0; k <= max_deg + 1; ++k) {
      int c = 0;
      for (auto& it : sorted)
        if (ctx->probs[it.x].degree >= k) ++c;
      g.active[k] = c;
    }
  }

  // ---- psi(t0) = |psi0> ----
  for (auto& P : ctx->probs) {
    const size_t vbytes = (size_t(1) << P.n) * sizeof(double2);
    HIPC(hipMemsetAsync(P.buf[0], 0, vbytes, ctx->stream));
    static const double2 one = {1.0, 0.0};
    HIPC(hipMemcpyAsync(P.buf[0] + P.psi0, &one, sizeof(double2), hipMemcpyHostToDevice, ctx->stream));
  }

  const size_t chunk = (size_t)std::min<int64_t>(n_t, std::max<int64_t>(1, (int64_t)(256ll << 20) / (ctx->total_items * 64)));
  if ((rc = ensure_partial(ctx, chunk))) return rc;
  size_t max_launch = 0;
  for (auto& g : ctx->groups) (void)g, max_launch += (size_t)max_deg;
  if (ctx->time_kernels && (rc = ensure_events(ctx, max_launch + 1))) return rc;

  double step_ms = 0.0, obs_ms = 0.0, launches = 0.0, amp_updates = 0.0, happl = 0.0;
  std::vector<size_t> pool_used(2, 0);
  auto drain_pool = [&](int pool) -> int {
    if (!ctx->time_kernels || pool_used[pool] == 0) return DSE_OK;
    HIPC(hipEventSynchronize(ctx->ev[pool][2 * pool_used[pool] - 1]));
    for (size_t i = 0; i < pool_used[pool]; ++i) {
      float ms = 0.f;
      HIPC(hipEventElapsedTime(&ms, ctx->ev[pool][2 * i], ctx->ev[pool][2 * i + 1]));
      step_ms += ms;
    }
    pool_used[pool] = 0;
    return DSE_OK;
  };

  size_t slot = 0, t_flushed = 0;
  if ((rc = launch_obs_all(ctx, 0, slot++))) return rc;
  for (int m = 0; m + 1 < n_t; ++m) {
    const int q = m & 1;
    const int set = set_of[m];
    const int pool = m & 1;
    if ((rc = drain_pool(pool))) return rc;
    for (auto& g : ctx->groups) {
      const int T = 1 << g.L;
      HIPC(launch_step(g.L, MODE_FIRST, ctx->d_probs, g.d_items_sorted, g.active[1], 1, q, set, ctx->stream));
      for (int k = 2; k <= max_deg; ++k) {
        const int na = g.active[k];
        if (na <= 0) break;
        if (ctx->time_kernels) {
          const size_t i = pool_used[pool]++;
          HIPC(hipEventRecord(ctx->ev[pool][2 * i], ctx->stream));
          HIPC(launch_step(g.L, MODE_GEN, ctx->d_probs, g.d_items_sorted, na, k, q, set, ctx->stream));
          HIPC(hipEventRecord(ctx->ev[pool][2 * i + 1], ctx->stream));
        } else {
          HIPC(launch_step(g.L, MODE_GEN, ctx->d_probs, g.d_items_sorted, na, k, q, set, ctx->stream));
        }
        launches += 1.0;
        amp_updates += (double)na * T;
      }
    }
    // new psi is in acc(q) = buf[q ? 0 : 2]
    if ((rc = launch_obs_all(ctx, q ? 0 : 2, slot++))) return rc;
    if (slot == chunk) {
      if ((rc = flush_partials(ctx, slot, t_flushed, n_t, obs_out))) return rc;
      t_flushed += slot;
      slot = 0;
    }
  }
  if (slot > 0) {
    if ((rc = flush_partials(ctx, slot, t_flushed, n_t, obs_out))) return rc;
    t_flushed += slot;
  }
  if ((rc = drain_pool(0))) return rc;
  if ((rc = drain_pool(1))) return rc;
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->last_q = (n_t - 1) & 1;
  ctx->evolved = true;

  for (auto& P : ctx->probs) happl += (double)P.degree * (n_t - 1);
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->h_applications = happl;
    stats->amplitude_updates = amp_updates;
    stats->step_bytes = 80.0 * amp_updates;
    stats->step_kernel_ms = ctx->time_kernels ? step_ms : -1.0;
    stats->step_launches = launches;
    stats->obs_kernel_ms = obs_ms;
    stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - wall0).count();
    stats->max_degree = max_deg;
    stats->n_intervals = n_t - 1;
    stats->tile_bits = ctx->groups.empty() ? 0 : ctx->groups.front().L;
  }
  return DSE_OK;
}

int dse_get_state(dse_ctx* ctx, int problem, double* psi_out) {
  if (!ctx) return DSE_ERR_ARG;
  if (problem < 0 || problem >= (int)ctx->probs.size()) return fail(ctx, DSE_ERR_ARG, "bad problem id");
  if (!psi_out) return fail(ctx, DSE_ERR_ARG, "null state");
  if (!ctx->evolved) return fail(ctx, DSE_ERR_STATE, "no evolved state (call dse_evolve first)");
  HIPC(hipSetDevice(ctx->device));
  HostProblem& P = ctx->probs[problem];
  // after the last interval m = n_t-2 the state sits in psi of parity (n_t-1)&1
  const int bsel = ctx->last_q ? 2 : 0;
  const size_t bytes = (size_t(1) << P.n) * sizeof(double2);
  HIPC(hipMemcpyAsync(psi_out, P.buf[bsel], bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return DSE_OK;
}

int dse_time_step_kernel(dse_ctx* ctx, int reps, double* ms_per_launch, double* bytes_per_launch) {
  if (!ctx) return DSE_ERR_ARG;
  if (reps < 1 || !ms_per_launch || !bytes_per_launch) return fail(ctx, DSE_ERR_ARG, "bad arguments");
  if (!ctx->evolved) return fail(ctx, DSE_ERR_STATE, "call dse_evolve first (coefficients needed)");
  HIPC(hipSetDevice(ctx->device));
  int rc = ensure_events(ctx, (size_t)reps * ctx->groups.size());
  if (rc) return rc;
  double bytes = 0.0;
  size_t e = 0;
  for (int r = 0; r < reps; ++r)
    for (auto& g : ctx->groups) {
      const int n_items = (int)g.items_by_prob.size();
      HIPC(hipEventRecord(ctx->ev[0][2 * e], ctx->stream));
      HIPC(launch_step(g.L, MODE_GEN, ctx->d_probs, g.d_items_sorted, n_items, 2, 0, 0, ctx->stream));
      HIPC(hipEventRecord(ctx->ev[0][2 * e + 1], ctx->stream));
      ++e;
      if (r == 0) bytes += 80.0 * (double)n_items * (double)(1 << g.L);
    }
  HIPC(hipStreamSynchronize(ctx->stream));
  double tot = 0.0;
  for (size_t i = 0; i < e; ++i) {
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, ctx->ev[0][2 * i], ctx->ev[0][2 * i + 1]));
    tot += ms;
  }
  *ms_per_launch = tot / reps;
  *bytes_per_launch = bytes;
  ctx->evolved = false;  // buffers now hold timing garbage
  return DSE_OK;
}

}  // extern "C"
