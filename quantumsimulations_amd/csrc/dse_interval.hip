// dse_interval.hip -- persistent per-interval Chebyshev kernel (gfx950).
//
// One launch propagates one output interval [t_m, t_{m+1}] of every problem whose register fits
// one or two LDS tiles (n <= L + 1; the N = 14 sweep: center_off has n = 13, center_on and
// shell_off n = 14).  Each workgroup owns one tile for all K terms of the interval:
//   LDS        w_{k-1} (the tile being multiplied; 128 KiB at L = 13)
//   registers  w_{k-2} (16 amplitudes per thread) and the new w_k
//   global     acc (accumulated every third term, L2-resident) and, for 2-tile problems, the
//              cross-tile contribution u published to the partner workgroup each term.
// This replaces K launches of k_step_rb (each reloading the tile from HBM and writing w_k back)
// by one launch with no per-term HBM traffic for the state.
//
// Cross-tile hand-off (2-tile problems, tiles A/B differ in the top bit L):
//   u_{A->B}(x) = flip_L(b_B) w_A(x) + sum_{j<L} g_{j,L} [x_j == b_B] w_A(x ^ e_j)
// is A's contribution to B's H application of the same term.  A computes it from its LDS tile
// at the start of the term and writes it (real parts, then imaginary parts) with 8-byte
// agent-scope (sc1) stores into a two-slot buffer; after its own tile terms it waits for those
// stores (s_waitcnt vmcnt(0)), barriers, and publishes the term index with an sc1 flag store.
// B polls the flag with sc1 loads (one lane, s_sleep, bounded), barriers and reads u with sc1
// loads (MI355X_MICROARCH.md "Valid forms", row 1: one workgroup per CU).
// Slots alternate with the term parity; a slot is rewritten only after the partner has published
// the next term, i.e. after it finished reading the slot.
#include "dse_device.h"

namespace dse {

// Diagnostic ablation mask of k_interval (0 in production), see set_ablate.
__device__ int g_dse_ablate_iv = 0;

hipError_t set_ablate_interval(int mask) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_dse_ablate_iv), &mask, sizeof(int));
}

namespace {

typedef __attribute__((address_space(1))) int gint;

constexpr int kSpinLimit = 1 << 22;  // ~0.3 s of polling before the hand-off is declared failed

template <int L>
__global__ void __launch_bounds__(RB<L>::NT)
k_interval(const DevProb* __restrict__ probs, const int2* __restrict__ items, int q, int set,
           int* __restrict__ flags, int* __restrict__ err) {
  constexpr int NT = RB<L>::NT, R = kRegAmps;
  constexpr size_t T = size_t(1) << L;
  __shared__ RBShared<L> S;
  __shared__ int s_fail;

  const int2 it = items[blockIdx.x];
  const DevProb& P = probs[it.x];
  const uint32_t h = (uint32_t)it.y;
  const int tid = threadIdx.x;
  const bool pair = (P.n == L + 1);
  const int K = P.degree;
  const double s1 = P.s1;

  // exchange slots (AoS double2, sc1): term parity 0 -> psi region (free once w_0 is in LDS),
  // 1 -> scratch buffer
  constexpr uint32_t TBYTES = uint32_t(T) * 16u;
  const __amdgpu_buffer_rsrc_t slot_me[2] = {tile_rsrc(P.buf[q ? 2 : 0] + (h << L), TBYTES),
                                             tile_rsrc(P.buf[1] + (h << L), TBYTES)};
  const __amdgpu_buffer_rsrc_t slot_pa[2] = {tile_rsrc(P.buf[q ? 2 : 0] + ((h ^ 1u) << L), TBYTES),
                                             tile_rsrc(P.buf[1] + ((h ^ 1u) << L), TBYTES)};
  const __amdgpu_buffer_rsrc_t acc_t = tile_rsrc(P.buf[q ? 0 : 2] + (h << L), TBYTES);
  const uint32_t voff = (uint32_t)tid * 16u;
  gint* flag_me = (gint*)flags + 2 * it.x + h;
  const gint* flag_pa = (const gint*)flags + 2 * it.x + (h ^ 1u);
  const uint32_t b_pa = (h ^ 1u) & 1u;  // top-bit value of the partner tile

  // diagnostics only (0 in production): 64 skip the u publication, 128 skip the partner wait and
  // read, 256 skip the acc updates, 512 skip the own-tile H terms
  const int ab = g_dse_ablate_iv;
  if (tid == 0) s_fail = 0;
  rb_stage_tables<L>(S, P, h, P.beta, tid);
#pragma unroll
  for (int r = 0; r < R; ++r) S.w[r * NT + tid] = bld(slot_me[0], voff, (uint32_t)(r * NT * 16));
  __syncthreads();
  rb_register_zz<L>(S, tid);
  const ThreadDiag td = rb_thread_diag<L>(S, tid);
  __syncthreads();

  double2 prev[R];
  for (int k = 1; k <= K; ++k) {
    // ---- u(w_{k-1}) for the partner: computed and stored (16-byte sc1 stores) before the
    // tile terms, published after them so the write-through drains under the compute ----
    const __amdgpu_buffer_rsrc_t dst = slot_me[(k - 1) & 1];
    if (pair && !(ab & 64)) {
      double2 u[R];
#pragma unroll
      for (int r = 0; r < R; ++r) u[r] = make_double2(0.0, 0.0);
      // cross flip of the top bit: coefficient for the partner's output bit value
      for (int f = 0; f < P.n_flips_hi; ++f) {
        const DFlip F = S.fh[f];
        const double cr = b_pa ? F.re1 : F.re0, ci = b_pa ? F.im1 : F.im0;
#pragma unroll
        for (int r = 0; r < R; ++r) u[r] = cmad(u[r], cr, ci, S.w[r * NT + tid]);
      }
      // cross pairs (j, top): applies iff x_j == b_pa; source w_A(x ^ e_j)
      for (int p = 0; p < P.n_pairs_hi; ++p) {
        const DPair Q = S.ph[p];
        const uint32_t m = Q.mask_lo;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint32_t x = (uint32_t)(r * NT + tid);
          const double g = (((x & m) != 0u) == (b_pa != 0u)) ? Q.g : 0.0;
          const double2 sv = S.w[x ^ m];
          u[r].x = fma(g, sv.x, u[r].x);
          u[r].y = fma(g, sv.y, u[r].y);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) bst<kSc1>(dst, voff, (uint32_t)(r * NT * 16), u[r]);
    }

    // ---- out = (H - beta) w_{k-1}: own-tile terms ----
    double2 out[R];
    if (ab & 512) {
#pragma unroll
      for (int r = 0; r < R; ++r) out[r] = S.w[r * NT + tid];
    } else {
      rb_apply_tile_a<L>(S, P, tid, td, 0, out);
      rb_apply_tile_b<L>(S, P, tid, 0, out);
    }

    // ---- publish, then add the partner's contribution u(w_{k-1}) ----
    if (pair && !(ab & 64)) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(flag_me, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (pair && !(ab & 128)) {
      if (tid == 0 && !(ab & 64)) {
        int spins = 0;
        while (__hip_atomic_load(flag_pa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < k) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kSpinLimit) {
            s_fail = 1;
            atomicExch(err, 1);
            break;
          }
        }
      }
      __syncthreads();
      const __amdgpu_buffer_rsrc_t src = slot_pa[(k - 1) & 1];
      double2 uv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) uv[r] = bld<kSc1>(src, voff, (uint32_t)(r * NT * 16));
#pragma unroll
      for (int r = 0; r < R; ++r) {
        out[r].x += uv[r].x;
        out[r].y += uv[r].y;
      }
    }

    // ---- recurrence + accumulation (in place in out[], acc operands four registers at a time
    // to bound the live registers) ----
    const CoefK C = P.coef[set * P.kcap1 + k];
    const bool upd = C.upd && !(ab & 256);
#pragma unroll
    for (int r0 = 0; r0 < R; r0 += 4) {
      double2 accv[4];
      if (k > 1 && upd) {
#pragma unroll
        for (int r = 0; r < 4; ++r) accv[r] = bld(acc_t, voff, (uint32_t)((r0 + r) * NT * 16));
      }
#pragma unroll
      for (int r = r0; r < r0 + 4; ++r) {
        const double2 own = S.w[r * NT + tid];
        if (k == 1) {
          out[r].x *= s1;
          out[r].y *= s1;
          double2 a = make_double2(0.0, 0.0);
          a = cmad(a, C.c[1].x, C.c[1].y, own);
          a = cmad(a, C.c[2].x, C.c[2].y, out[r]);
          bst(acc_t, voff, (uint32_t)(r * NT * 16), a);
        } else {
          out[r].x = fma(2.0 * s1, out[r].x, -prev[r].x);
          out[r].y = fma(2.0 * s1, out[r].y, -prev[r].y);
          if (upd) {
            double2 a = accv[r - r0];
            a = cmad(a, C.c[0].x, C.c[0].y, prev[r]);
            a = cmad(a, C.c[1].x, C.c[1].y, own);
            a = cmad(a, C.c[2].x, C.c[2].y, out[r]);
            bst(acc_t, voff, (uint32_t)(r * NT * 16), a);
          }
        }
        prev[r] = own;
      }
    }
    __syncthreads();  // every read of w_{k-1} in LDS is done
#pragma unroll
    for (int r = 0; r < R; ++r) S.w[r * NT + tid] = out[r];
    __syncthreads();
    if (s_fail) break;  // uniform: a hand-off timed out (error reported to the host)
  }
}

}  // namespace

bool interval_supported(int L) { return L >= kRegBlockMinTile && L <= kMaxTile; }

hipError_t launch_interval(int L, const DevProb* probs, const int2* items, int n_items, int q,
                           int set, int* flags, int* err, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  switch (L) {
#define X(l)                                                                                  \
  case l:                                                                                     \
    hipLaunchKernelGGL((k_interval<l>), dim3(n_items), dim3(RB<l>::NT), 0, st, probs, items, q, \
                       set, flags, err);                                                      \
    return hipGetLastError();
    X(10) X(11) X(12) X(13)
#undef X
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace dse
