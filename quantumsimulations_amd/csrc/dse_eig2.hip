// dse_eig2.hip -- two-stage symmetric eigendecomposition for the dense engine's large registers
// (gfx950; option eig_impl = 3).
//
// The one-stage tridiagonalisation (dse_sytrd.hip) reads the whole trailing matrix once per column
// (8 n^3 / 6 bytes: 5.9 TB at n = 2^14, 1.76 s at ~5 TB/s).  Two stages move that work into GEMMs
// and a cheap chase (prototype and order proofs: tools/proto_two_stage.py):
//   1. dense -> band b = 32 (sy2sb_lower): panels of b columns; the panel below the band is
//      QR-factorised (k_panel_qr: one row per thread, one grid barrier per column) and the trailing
//      matrix updated two-sided by rocBLAS (dsymm, dtrmm, dgemm, dsyr2k): A22 -= V W^T + W V^T,
//      W = Y - V (T^T V^T Y) / 2, Y = A22 V T.  Reads per panel ~1.5 trailing triangles: 4 n^3 / b
//      bytes in all (0.55 TB at 2^14).
//   2. band -> tridiagonal (k_sb2st): bulge chasing, one reflector of length <= b per task (s, t)
//      (sweep s annihilates column s; task t >= 1 the first column of the bulge block left by task
//      t - 1), each task a 3b-wide strip of the band held in one wave's LDS.  Sweeps are dealt to
//      waves; task (s, t) waits until task t + 3 of sweep s - 1 is done (their strips are then
//      disjoint), so ~n / 4b sweeps run at once.  Band storage: column c, A(c + d, c) at
//      S[c * kLD + d], d <= 2b (the bulge lives below the band).
//   3. rocsolver_dstedc on the tridiagonal.
//   4. Z <- Q2 Z (k_sb_q2): the chase's reflectors in blocks of kQ2NB sweeps (s-blocks last to
//      first, t ascending, s descending inside a block); a wave owns 64 columns and holds the
//      block's 64-row window of each in registers, sliding down by b rows per t.
//   5. Z <- Q1 Z: the panels' reflectors (unit element b rows below their column) by ormtr_lower's
//      blocks of 256 (dse_sytrd.hip).
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "dse_dense.h"

namespace dse {
namespace {

constexpr int kB = 32;              // bandwidth of stage 1 = reflector length of stage 2
constexpr int kLD = 2 * kB + 2;     // band storage per column: d = 0 .. 2b, one pad
// panel QR: rows (threads) per workgroup.  512 against 256: half the workgroups whose partial sums
// every column's exchange gathers, band stage 312 -> 300 ms at 2^14; 1024 spills (329 ms)
// (profiles/r05/ab/panel_qr_rows_ab.txt)
constexpr int kPanelRows = 512;
constexpr int kQ2NB = 32;           // Q2 application: sweeps per group
constexpr int kQ2Win = kQ2NB + kB;  // window rows per column

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LDS writes of other lanes of this wave visible to the reads that follow (no workgroup barrier)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ptr_rsrc(const void* p, size_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)bytes, 0x00020000);
}
constexpr int kBandSc1 = 16;  // aux: sc1 (dse_device.h kSc1)
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, int e) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, e * 8, 0, kBandSc1));
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int e, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), r, e * 8, 0, kBandSc1);
}

// ---- stage 1 ------------------------------------------------------------------------------------

// Householder QR of the m x kB panel P (column-major, ld lda) in place, LAPACK dgeqr2's layout
// (R on and above the diagonal, v below it with v_0 = 1 implied, tau[j]).  Thread = row; the
// workgroups are co-resident (gridDim.x <= CUs).  Column j's partial sums (part[(j G + g)(kB + 1)
// + k]) and pivot row (piv[j kB + k]) are written once each (sc1) into slots that hold the
// all-ones sentinel before the launch; every workgroup polls the values themselves (a slot still
// holding the sentinel is read again), so a column costs one store-to-load round trip and no
// barrier (the mailbox form of the chase).
//
// Every cross-workgroup poll of this file (here and in the chase) is bounded: after `spin` rounds
// (option eig_spin_limit) a poll gives up and sets the solve's device error word *err, and every
// other poll that finds the word set gives up at once, so a launch whose workgroups are not all
// resident (or a NaN input, whose all-ones payload is the sentinel) drains instead of hanging.  The
// host reads the word after the chase (sb2st_lower -> kEig2PollTimeout) and the dense engine
// re-solves that register with rocSOLVER dsyevd.  spin < 0 sets the word at the start (tests).
constexpr unsigned long long kSentinel = ~0ull;
__device__ __forceinline__ bool is_sentinel(double v) {
  return __builtin_bit_cast(unsigned long long, v) == kSentinel;
}
// a poll that has missed `it` times gives up: the limit, or another poll's give-up (checked on the
// first miss and every 64th after); a give-up is recorded in *err (vector atomic)
__device__ __forceinline__ bool poll_give_up(int* err, int spin, int it) {
  bool up = it >= spin;
  if (!up && (it & 63) == 0) up = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  if (up) __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return up;
}
__global__ void __launch_bounds__(kPanelRows)
k_panel_qr(double* __restrict__ P, int lda, int m, double* __restrict__ tau, double* __restrict__ part,
           double* __restrict__ piv, double* __restrict__ Vw, double* __restrict__ Vt, int* __restrict__ err,
           int spin) {
  constexpr int NW = kPanelRows / 64, NG0 = kPanelRows / 32, NQ = 128 / NG0;  // waves; partial sums
  __shared__ double red[NW][kB];
  __shared__ double red8[NG0][kB];
  __shared__ double tot[kB];
  __shared__ double prow[kB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x;
  const __amdgpu_buffer_rsrc_t prs = ptr_rsrc(part, (size_t)kB * G * (kB + 1) * 8);
  const __amdgpu_buffer_rsrc_t vrs = ptr_rsrc(piv, (size_t)kB * kB * 8);
  const int r = blockIdx.x * kPanelRows + tid;
  const bool own = r < m;
  if (spin < 0 && blockIdx.x == 0 && tid == 0) __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  double x[kB];
#pragma unroll
  for (int k = 0; k < kB; ++k) x[k] = own ? P[(size_t)k * lda + r] : 0.0;
  const int kmax = min(m, kB);
  for (int j = 0; j < kmax; ++j) {
    const int pj = (j * G + blockIdx.x) * (kB + 1);
    // slot j: sum of squares of x_j below row j; slot k > j: sum of x_j x_k below row j
    const bool below = own && r > j;
    double xj = 0.0;
#pragma unroll
    for (int k = 0; k < kB; ++k) xj = k == j ? x[k] : xj;
    if (!below) xj = 0.0;
    {  // the wave's 32 sums x_j . x_k by a butterfly reduce-scatter (31 exchanges instead of 32 x 6):
       // after the steps over lane bits 5 .. 1 lane l holds k = l >> 1 over its half, bit 0 adds the pair
      double pk[kB];
#pragma unroll
      for (int k = 0; k < kB; ++k) pk[k] = xj * x[k];
#pragma unroll
      for (int o = 32, h = 16; o >= 2; o >>= 1, h >>= 1) {
        const bool up = (lane & o) != 0;
#pragma unroll
        for (int q = 0; q < h; ++q) {
          const double send = up ? pk[q] : pk[q + h];
          const double keep = up ? pk[q + h] : pk[q];
          pk[q] = keep + __shfl_xor(send, o, 64);
        }
      }
      const double sk = pk[0] + __shfl_xor(pk[0], 1, 64);
      if ((lane & 1) == 0) red[wave][lane >> 1] = sk;
    }
    if (own && r == j) {
#pragma unroll
      for (int k = 0; k < kB; ++k)
        if (k >= j) bstore(vrs, j * kB + k, x[k]);
    }
    __syncthreads();
    if (tid < kB && tid >= j) {
      double a = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) a += red[w][tid];
      bstore(prs, pj + tid, a);
    }
    {  // the G partials: thread (k, g0) sums g = g0, g0 + NG0, ... (G <= 128), then the NG0 in fixed order
      const int k = tid & 31, g0 = tid >> 5;
      double pv[NQ];
      auto slot = [&](int q) { return (j * G + g0 + NG0 * q) * (kB + 1) + k; };
      auto live = [&](int q) { return k >= j && g0 + NG0 * q < G; };
#pragma unroll
      for (int q = 0; q < NQ; ++q) pv[q] = live(q) ? bload(prs, slot(q)) : 0.0;
      double pr = tid < kB && tid >= j ? bload(vrs, j * kB + tid) : 0.0;
      for (int it = 0;; ++it) {
        bool miss = is_sentinel(pr);
#pragma unroll
        for (int q = 0; q < NQ; ++q) miss |= is_sentinel(pv[q]);
        if (!miss || poll_give_up(err, spin, it)) break;
        __builtin_amdgcn_s_sleep(1);
#pragma unroll
        for (int q = 0; q < NQ; ++q)
          if (is_sentinel(pv[q])) pv[q] = bload(prs, slot(q));
        if (is_sentinel(pr)) pr = bload(vrs, j * kB + tid);
      }
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) s += pv[q];
      red8[g0][k] = s;
      if (tid < kB) prow[tid] = pr;
    }
    __syncthreads();
    if (tid < kB) {
      double s = 0.0;
#pragma unroll
      for (int g = 0; g < NG0; ++g) s += red8[g][tid];
      tot[tid] = s;
    }
    __syncthreads();
    const double alpha = prow[j], s2 = tot[j];
    double beta = alpha, t = 0.0, sc = 0.0;
    if (s2 != 0.0) {
      beta = -copysign(sqrt(alpha * alpha + s2), alpha);
      t = (beta - alpha) / beta;
      sc = 1.0 / (alpha - beta);
    }
    if (blockIdx.x == 0 && tid == 0) tau[j] = t;
    if (t != 0.0) {
      if (below) {
        const double v = xj * sc;
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          if (k < j) continue;
          if (k == j) {
            x[k] = v;
          } else {
            const double w = t * (prow[k] + sc * tot[k]);
            x[k] = fma(-v, w, x[k]);
          }
        }
      } else if (own && r == j) {
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          if (k < j) continue;
          if (k == j) {
            x[k] = beta;
          } else {
            const double w = t * (prow[k] + sc * tot[k]);
            x[k] -= w;
          }
        }
      }
    }
  }
  if (own) {
    // the panel in place, and Vw (m x kB, ld m) / Vt (row-major) of the reflectors with their unit
    // diagonal, zeros above it and past kmax (written here from the registers)
#pragma unroll
    for (int k = 0; k < kB; ++k) {
      P[(size_t)k * lda + r] = x[k];
      const double v = k >= kmax ? 0.0 : r > k ? x[k] : (r == k ? 1.0 : 0.0);
      Vw[(size_t)k * m + r] = v;
      Vt[(size_t)r * kB + k] = v;
    }
  }
}

// sum over g < ng of part[g kB^2 + e] in a fixed order: eight interleaved partial sums (g mod 8),
// so eight loads are in flight per thread instead of one dependent add per load
__device__ __forceinline__ double sum_partials(const double* __restrict__ part, int ng, int e) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = 0.0;
  int g = 0;
  for (; g + 8 <= ng; g += 8) {
    double x[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = part[(size_t)(g + i) * kB * kB + e];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += x[i];
  }
  for (int i = 0; g + i < ng; ++i) a[i] += part[(size_t)(g + i) * kB * kB + e];
  return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// T (kB x kB upper, ld kB) of the panel's block reflector I - V T V^T (LAPACK dlarft, forward,
// columnwise): T(j, j) = tau_j, T(0:j, j) = -tau_j T(0:j, 0:j) (V^T V)(0:j, j), with V^T V the sum
// of k_sb_vty's partials (fixed order); one workgroup
__global__ void __launch_bounds__(kB * kB)
k_sb_tmat(const double* __restrict__ part, int ng, int k, const double* __restrict__ tau, double* __restrict__ T) {
  __shared__ double G[kB][kB + 1];
  __shared__ double Ts[kB][kB + 1];
  const int e = threadIdx.x, p = e % kB, q = e / kB;
  G[p][q] = sum_partials(part, ng, e);
  Ts[p][q] = 0.0;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    const double tj = tau[j];
    if (e < j) {
      double sum = 0.0;
      for (int c = e; c < j; ++c) sum = fma(Ts[e][c], G[c][j], sum);
      Ts[e][j] = -tj * sum;
    } else if (e == j) {
      Ts[j][j] = tj;
    }
    __syncthreads();
  }
  T[(size_t)q * kB + p] = (p < k && q < k) ? Ts[p][q] : 0.0;
}

// ---- stage 1's trailing update on the matrix cores (v_mfma_f64_16x16x4_f64: lane l holds A(l & 15,
// l >> 4) and B(l >> 4, l & 15) of a 16 x 4 / 4 x 16 step; D(row (l >> 4) + 4 r, col l & 15), r < 4,
// cdna_hip_programming.md) ----
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int kT = 64;       // tile of the trailing matrix


__device__ __forceinline__ f64x4 mfma64(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Partial Y_I = sum over the column tiles J of chunk blockIdx.y of A22_IJ V_J for the symmetric
// A22 (lower triangle stored, ld lda): tiles J < I as stored, J > I from the stored A_JI (their
// columns are contiguous: one 16-B load = two k-steps), J = I and ragged edge tiles element-wise.
// Wave w takes the chunk's tiles w, w + 4, ..., all 64 x 32 outputs of a tile in its registers;
// the k-steps of an MFMA pair are columns c = 8 u + 2 (lane >> 4) + e, e = 0, 1, of the tile (any
// order of the 4 k-slots works when both operands use it).  The waves' sums meet in LDS (fixed
// order); Yp[(ch kB + q) m + r] holds chunk ch's partial.
constexpr int kSymmCh = 16;  // column tiles per workgroup
__global__ void __launch_bounds__(256, 2)
k_sb_symm(const double* __restrict__ A, int lda, int m, const double* __restrict__ Vt, double* __restrict__ Yp) {
  __shared__ double red[kB][kT + 1];
  const int I = blockIdx.x, ch = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nbk = (m + kT - 1) / kT;
  const int r0 = I * kT;
  f64x4 acc[4][2];
#pragma unroll
  for (int rs = 0; rs < 4; ++rs) acc[rs][0] = acc[rs][1] = f64x4{0.0, 0.0, 0.0, 0.0};
  const int jb = ch * kSymmCh, je = min(nbk, jb + kSymmCh);
  for (int J = jb + w; J < je; J += 4) {
    const int c0 = J * kT;
    const bool full = J != I && r0 + kT <= m && c0 + kT <= m;
    // the tile in two halves of 32 columns (registers for two workgroups per CU)
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      double a[4][8], b[2][8];
      if (full && J < I) {
#pragma unroll
        for (int uu = 0; uu < 4; ++uu)
#pragma unroll
          for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int rs = 0; rs < 4; ++rs)
              a[rs][2 * uu + e] = A[(size_t)(c0 + 8 * (4 * hf + uu) + 2 * lq + e) * lda + r0 + 16 * rs + li];
      } else if (full) {
#pragma unroll
        for (int uu = 0; uu < 4; ++uu)
#pragma unroll
          for (int rs = 0; rs < 4; ++rs) {
            const double2 v = *reinterpret_cast<const double2*>(A + (size_t)(r0 + 16 * rs + li) * lda + c0 +
                                                                8 * (4 * hf + uu) + 2 * lq);
            a[rs][2 * uu] = v.x;
            a[rs][2 * uu + 1] = v.y;
          }
      } else {
#pragma unroll
        for (int uu = 0; uu < 4; ++uu)
#pragma unroll
          for (int e = 0; e < 2; ++e)
#pragma unroll
            for (int rs = 0; rs < 4; ++rs) {
              const int gr = r0 + 16 * rs + li, gc = c0 + 8 * (4 * hf + uu) + 2 * lq + e;
              a[rs][2 * uu + e] =
                  (gr < m && gc < m) ? (gr >= gc ? A[(size_t)gc * lda + gr] : A[(size_t)gr * lda + gc]) : 0.0;
            }
      }
#pragma unroll
      for (int uu = 0; uu < 4; ++uu)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const int gc = c0 + 8 * (4 * hf + uu) + 2 * lq + e;
#pragma unroll
          for (int cs = 0; cs < 2; ++cs) b[cs][2 * uu + e] = gc < m ? Vt[(size_t)gc * kB + 16 * cs + li] : 0.0;
        }
#pragma unroll
      for (int st = 0; st < 8; ++st)
#pragma unroll
        for (int rs = 0; rs < 4; ++rs)
#pragma unroll
          for (int cs = 0; cs < 2; ++cs) acc[rs][cs] = mfma64(a[rs][st], b[cs][st], acc[rs][cs]);
    }
  }
  // D(row (lane >> 4) + 4 x, col lane & 15) of output tile (rs, cs) = Y(16 rs + row, 16 cs + col)
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int rs = 0; rs < 4; ++rs)
#pragma unroll
        for (int cs = 0; cs < 2; ++cs)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            double& d = red[16 * cs + li][16 * rs + lq + 4 * x];
            d = ww == 0 ? acc[rs][cs][x] : d + acc[rs][cs][x];
          }
    }
    __syncthreads();
  }
  for (int e = tid; e < kB * kT; e += 256) {
    const int r = e & 63, q = e >> 6;
    if (r0 + r < m) Yp[((size_t)ch * kB + q) * m + r0 + r] = red[q][r];
  }
}

// A22 (lower, ld lda) -= V W^T + W V^T on the 64 x 64 tiles on and below the diagonal: D' = Q P^T
// with P = [V_I | W_I], Q = [W_J | V_J] (64 x 2 kB each), D'(c, r) -= into A(I 64 + r, J 64 + c)
// for the columns cmin <= c < cmax of A22.
// Operands straight from the row-major copies Vt, Wt (16-B loads: k = 8 u + 2 (lane >> 4) + e, as
// k_sb_symm); wave w takes columns c of subtile w, the A tile's loads issued first.
__global__ void __launch_bounds__(256)
k_sb_syr2k(double* __restrict__ A, int lda, int m, const double* __restrict__ Vt, const double* __restrict__ Wt,
           int cmin, int cmax, int ntiles) {
  // ntiles > 0: a 1-D grid over the tiles on and below the diagonal, e = I (I + 1) / 2 + J; else a
  // 2-D grid (I, J) with the tiles above the diagonal idle
  int I = blockIdx.x, J = blockIdx.y;
  if (ntiles > 0) {
    const int e = (int)blockIdx.x;
    I = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    while ((I + 1) * (I + 2) / 2 <= e) ++I;
    while (I * (I + 1) / 2 > e) --I;
    J = e - I * (I + 1) / 2;
  }
  if (J > I) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lq = lane >> 4;
  const int r0 = I * kT, c0 = J * kT;
  double old[4][4];
#pragma unroll
  for (int sc = 0; sc < 4; ++sc)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int gc = c0 + 16 * w + lq + 4 * x, gr = r0 + 16 * sc + li;
      old[sc][x] = (gr < m && gc < cmax && gc >= cmin && gr >= gc) ? A[(size_t)gc * lda + gr] : 0.0;
    }
  const int qc = c0 + 16 * w + li;
  double qa[16];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const double* src = u < 4 ? Wt : Vt;
    double2 v = double2{0.0, 0.0};
    if (qc < m) v = *reinterpret_cast<const double2*>(src + (size_t)qc * kB + (u & 3) * 8 + 2 * lq);
    qa[2 * u] = v.x;
    qa[2 * u + 1] = v.y;
  }
  f64x4 acc[4];
#pragma unroll
  for (int sc = 0; sc < 4; ++sc) {
    const int pr = r0 + 16 * sc + li;
    double pb[16];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double* src = u < 4 ? Vt : Wt;
      double2 v = double2{0.0, 0.0};
      if (pr < m) v = *reinterpret_cast<const double2*>(src + (size_t)pr * kB + (u & 3) * 8 + 2 * lq);
      pb[2 * u] = v.x;
      pb[2 * u + 1] = v.y;
    }
    acc[sc] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int st = 0; st < 16; ++st) acc[sc] = mfma64(qa[st], pb[st], acc[sc]);
  }
#pragma unroll
  for (int sc = 0; sc < 4; ++sc)
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const int gc = c0 + 16 * w + lq + 4 * x, gr = r0 + 16 * sc + li;
      if (gr < m && gc < cmax && gc >= cmin && gr >= gc) A[(size_t)gc * lda + gr] = old[sc][x] - acc[sc][x];
    }
}

// The same update, kSyr2kNJ column tiles J per workgroup (one row block I): P = [V_I | W_I] is shared
// by the tiles and the four waves, staged once in LDS; each lane holds rows (2 li, 2 li + 1) of
// an output pair (the MFMAs of row halves sc = 2 sp + par take P rows 32 sp + 2 li + par), so A is
// read and written with 16-B accesses.  Column tiles jlo .. jhi (the launch's cmin .. cmax range);
// tiles above the diagonal idle.  A's offsets are 32-bit buffer offsets from A22 (and the buffer
// descriptor's size is 32-bit): valid while lda * m * 8 < 2^32, which every dense register
// (n <= kDenseMaxQubits = 14: 2^31 bytes) meets; sy2sb_lower takes k_sb_syr2k (64-bit pointer
// arithmetic) for anything larger.
static_assert(kDenseMaxQubits <= 14, "k_sb_syr2k2: 32-bit offsets into a 2^n x 2^n matrix");
constexpr int kSyr2kNJ = 4;
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256)
k_sb_syr2k2(double* __restrict__ A, int lda, int m, const double* __restrict__ Vt, const double* __restrict__ Wt,
            int cmin, int cmax) {
  constexpr int PLD = 2 * kB + 2;  // LDS row stride (doubles)
  __shared__ __attribute__((aligned(16))) double Ps[kT][PLD];
  const int I = blockIdx.x;
  const int jlo = cmin / kT + (int)blockIdx.y * kSyr2kNJ;
  const int jhi = min(min(I, (cmax - 1) / kT), jlo + kSyr2kNJ - 1);
  if (jlo > jhi) return;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15, lq = lane >> 4;
  const int r0 = I * kT;
  // A22 through a buffer resource: an element outside the update (column outside cmin .. cmax, row
  // >= m) takes an out-of-range offset (load 0, store dropped).  Elements above the diagonal inside
  // the diagonal tiles are updated too: nothing reads A22's upper triangle (k_sb_symm and the panel
  // QR read the lower one), so no row is a branch
  const __amdgpu_buffer_rsrc_t ar = ptr_rsrc(A, ((size_t)(m - 1) * lda + m) * 8);
  const __amdgpu_buffer_rsrc_t vr = ptr_rsrc(Vt, (size_t)m * kB * 8), wr = ptr_rsrc(Wt, (size_t)m * kB * 8);
  constexpr uint32_t kOOB = 0xffffffffu;
  for (int e = tid; e < kT * kB; e += 256) {  // 16-B pieces: row r, k pair (Vt | Wt)
    const int r = e / kB, kk = 2 * (e % kB);
    const uint32_t off = r0 + r < m ? (uint32_t)(((r0 + r) * kB + (kk & (kB - 1))) * 8) : kOOB;
    const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(kk < kB ? vr : wr, (int)off, 0, 0);
    *reinterpret_cast<u32x4_t*>(&Ps[r][kk]) = v;
  }
  __syncthreads();
#pragma unroll 1
  for (int J = jlo; J <= jhi; ++J) {
    const int c0 = J * kT;
    // A row pairs (sp, x): rows gr, gr + 1 of column gc; a pair cut by row m (m odd) takes the
    // single-element path
    uint32_t aoff[2][4];
    bool split[2][4];
    u32x4_t old[2][4];
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int gc = c0 + 16 * w + lq + 4 * x, gr = r0 + 32 * sp + 2 * li;
        const bool col = gc >= cmin && gc < cmax;
        aoff[sp][x] = (col && gr + 1 < m) ? (uint32_t)(((size_t)gc * lda + gr) * 8) : kOOB;
        split[sp][x] = col && gr + 1 == m;
        old[sp][x] = __builtin_amdgcn_raw_buffer_load_b128(ar, (int)aoff[sp][x], 0, 0);
        if (split[sp][x]) {
          const u32x2_t h = __builtin_amdgcn_raw_buffer_load_b64(ar, (int)(((size_t)gc * lda + gr) * 8), 0, 0);
          old[sp][x].x = h.x;
          old[sp][x].y = h.y;
        }
      }
    double qa[16];
    {
      const int qc = c0 + 16 * w + li;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t off = qc < m ? (uint32_t)((qc * kB + (u & 3) * 8 + 2 * lq) * 8) : kOOB;
        const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(u < 4 ? wr : vr, (int)off, 0, 0);
        const double2 d = __builtin_bit_cast(double2, v);
        qa[2 * u] = d.x;
        qa[2 * u + 1] = d.y;
      }
    }
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {  // row half sp: the two MFMA row sets par = 0, 1, then its stores
      f64x4 acc[2];
#pragma unroll
      for (int par = 0; par < 2; ++par) {
        const double* prow = &Ps[32 * sp + 2 * li + par][0];
        acc[par] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double2 pb = *reinterpret_cast<const double2*>(prow + (u >> 2) * kB + (u & 3) * 8 + 2 * lq);
          acc[par] = mfma64(qa[2 * u], pb.x, acc[par]);
          acc[par] = mfma64(qa[2 * u + 1], pb.y, acc[par]);
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const double2 o = __builtin_bit_cast(double2, old[sp][x]);
        const double2 nv = double2{o.x - acc[0][x], o.y - acc[1][x]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, nv), ar, (int)aoff[sp][x], 0, 0);
        if (split[sp][x]) {
          const int gc = c0 + 16 * w + lq + 4 * x, gr = r0 + 32 * sp + 2 * li;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, nv.x), ar, (int)(((size_t)gc * lda + gr) * 8), 0, 0);
        }
      }
    }
  }
}

// Y <- Y T (T kB x kB upper, ld kB): one thread per output Y(r, q) (32 per row, the row's Y in
// L1), T in LDS
__global__ void __launch_bounds__(256)
k_sb_yt2(const double* __restrict__ Y, double* __restrict__ Yo, int m, int k, const double* __restrict__ T) {
  __shared__ double Ts[kB][kB + 1];
  const int tid = threadIdx.x;
  for (int e = tid; e < kB * kB; e += 256) {
    const int i = e % kB, j = e / kB;
    Ts[i][j] = (i < k && j < k && i <= j) ? T[(size_t)j * kB + i] : 0.0;
  }
  __syncthreads();
  const int r = blockIdx.x * 8 + (tid >> 5), q = tid & 31;  // lanes: q fast within a row
  if (r >= m) return;
  double a = 0.0;
#pragma unroll 8
  for (int p = 0; p < kB; ++p) a = fma(Y[(size_t)p * m + r], Ts[p][q], a);
  Yo[(size_t)q * m + r] = q < k ? a : 0.0;
}

// Y (m x kB, ld m) = the sum of k_sb_symm's nch partials (fixed order), one thread per element
__global__ void __launch_bounds__(256)
k_sb_ysum(double* __restrict__ Y, const double* __restrict__ Yp, int nch, int m) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x, mk = (size_t)m * kB;
  if (e >= mk) return;
  double a = 0.0;
  int c = 0;
  for (; c + 4 <= nch; c += 4) {
    const double x0 = Yp[(size_t)c * mk + e], x1 = Yp[(size_t)(c + 1) * mk + e];
    const double x2 = Yp[(size_t)(c + 2) * mk + e], x3 = Yp[(size_t)(c + 3) * mk + e];
    a += x0;
    a += x1;
    a += x2;
    a += x3;
  }
  for (; c < nch; ++c) a += Yp[(size_t)c * mk + e];
  Y[e] = a;
}

// part[g] (kB x kB, column-major) = V_g^T Y_g over the kVtyRows-row chunk g, on the matrix cores
// (4 waves: wave w takes a quarter of the chunk's rows, the four 16 x 16 output tiles; the waves'
// sums are added in fixed order).  128-row chunks: 74 KB of LDS, two workgroups per CU.
constexpr int kVtyRows = 128;
__global__ void __launch_bounds__(256)
k_sb_vty(const double* __restrict__ V, const double* __restrict__ Y, int m, double* __restrict__ part) {
  __shared__ double Vs[kVtyRows][kB + 4];
  __shared__ double Ys[kVtyRows][kB + 4];
  double(*red)[kB * kB] = reinterpret_cast<double(*)[kB * kB]>(&Vs[0][0]);  // after the products
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int rb = blockIdx.x * kVtyRows;
  for (int e = tid; e < kVtyRows * kB; e += 256) {
    const int r = e % kVtyRows, q = e / kVtyRows;
    const bool ok = rb + r < m;
    Vs[r][q] = ok ? V[(size_t)q * m + rb + r] : 0.0;
    Ys[r][q] = ok ? Y[(size_t)q * m + rb + r] : 0.0;
  }
  __syncthreads();
  // D(p, q) = sum_r V(r, p) Y(r, q): A(i = p, kk = r) = V(r, p), B(kk = r, j = q) = Y(r, q)
  f64x4 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < kVtyRows / 16; ++kk) {
    const int r = (kVtyRows / 4) * w + 4 * kk + (lane >> 4);
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const double va = Vs[r][16 * a + (lane & 15)];
#pragma unroll
      for (int b = 0; b < 2; ++b) acc[a][b] = mfma64(va, Ys[r][16 * b + (lane & 15)], acc[a][b]);
    }
  }
  __syncthreads();  // every wave's reads of Vs done before red overwrites it
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int p = 16 * a + (lane >> 4) + 4 * rr, q = 16 * b + (lane & 15);
        red[w][q * kB + p] = acc[a][b][rr];
      }
  __syncthreads();
  for (int e = tid; e < kB * kB; e += 256)
    part[(size_t)blockIdx.x * kB * kB + e] = (red[0][e] + red[1][e]) + (red[2][e] + red[3][e]);
}

// Gm = T^T M, M = sum of the partials (fixed order); one workgroup
__global__ void __launch_bounds__(kB * kB)
k_sb_gm(const double* __restrict__ part, int ng, int k, const double* __restrict__ T, double* __restrict__ Gm) {
  __shared__ double M[kB][kB];
  const int e = threadIdx.x, p = e % kB, q = e / kB;
  M[p][q] = sum_partials(part, ng, e);
  __syncthreads();
  double gsum = 0.0;
  for (int i = 0; i <= p; ++i) gsum = fma(T[(size_t)p * kB + i], M[i][q], gsum);  // T^T(p, i) = T(i, p)
  Gm[(size_t)q * kB + p] = (p < k && q < k) ? gsum : 0.0;
}

// Wt (row-major m x kB) = Y2 - V Gm / 2; 64 rows per workgroup: thread (r, 8 of the 32 q) from the
// column-major V and Y (coalesced along r), the 64 x 32 result through LDS to whole Wt rows
__global__ void __launch_bounds__(256)
k_sb_w(const double* __restrict__ Y, const double* __restrict__ V, int m, int k, const double* __restrict__ Gm,
       double* __restrict__ Wt) {
  __shared__ double Gs[kB][kB];
  __shared__ double Ws[64][kB + 1];
  const int tid = threadIdx.x, rl = tid & 63, qg = tid >> 6, r0 = blockIdx.x * 64, r = r0 + rl;
  for (int e = tid; e < kB * kB; e += 256) Gs[e % kB][e / kB] = Gm[e];
  __syncthreads();
  if (r < m) {
    double v[kB];
#pragma unroll
    for (int p = 0; p < kB; ++p) v[p] = p < k ? V[(size_t)p * m + r] : 0.0;
#pragma unroll
    for (int qq = 0; qq < 8; ++qq) {
      const int q = 8 * qg + qq;
      double a = 0.0;
#pragma unroll
      for (int p = 0; p < kB; ++p) a = fma(v[p], Gs[p][q], a);
      Ws[rl][q] = q < k ? Y[(size_t)q * m + r] - 0.5 * a : 0.0;
    }
  }
  __syncthreads();
  for (int e = tid; e < 64 * kB; e += 256) {
    const int rr = e >> 5, q = e & 31;
    if (r0 + rr < m) Wt[(size_t)(r0 + rr) * kB + q] = Ws[rr][q];
  }
}

// band storage S[c * kLD + d] = A(c + d, c) for d <= kB (0 beyond, room for the bulge)
__global__ void __launch_bounds__(256)
k_sb_band(const double* __restrict__ A, int lda, int n, double* __restrict__ S) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (size_t)n * kLD) return;
  const int c = (int)(e / kLD), d = (int)(e % kLD);
  S[e] = (d <= kB && c + d < n) ? A[(size_t)c * lda + c + d] : 0.0;
}

// ---- stage 2 ------------------------------------------------------------------------------------

__host__ __device__ __forceinline__ int chase_tasks(int n, int s) { return 1 + (n - 2 - s) / kB; }

// Reflector (s, t) of the chase in group-major order for the Q2 application: group (block, t) of
// sweeps s in [block kQ2NB, block kQ2NB + kQ2NB) is kQ2NB consecutive records (v[kB], tau, pad:
// kRec doubles, v 16-B aligned) starting at goff[block] + t kQ2NB kRec; absent reflectors stay
// zero (tau = 0).
constexpr int kRec = kB + 2;
__device__ __forceinline__ double* refl_at(double* refl, const long long* goff, int s, int t) {
  return refl + goff[s / kQ2NB] + ((size_t)t * kQ2NB + (s % kQ2NB)) * kRec;
}

// One task (s, t) by one wave, the three 32 x 32 blocks in registers: lane = column j (L, D) or row
// i (R) of a 16-row / 16-column half h = lane >> 5.  v, w and the annihilated column in LDS.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t band_rsrc(double* S, int n) {
  const uint64_t a = (uint64_t)S;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)((size_t)n * kLD * 8),
                                           0x00020000);
}
// band element e (32-bit index) with sc1 loads and stores: the chase hands the band between CUs in
// the guide's valid form (MI355X_MICROARCH.md "Valid forms", row 1, per wave: every load and
// store of the band sc1, each storing wave's s_waitcnt vmcnt(0) before its sc1 flag store, the
// consumer wave polls the flag with sc1 loads and then loads)

constexpr int kChaseWG = 4;  // waves per chase workgroup

struct ChaseVec {
  double x[kB];
  double v[kB];
  double w[kB];
  double Lt[kB][kB + 1];  // L and D between the memory layout (lane = row) and the compute layout
  double Dt[kB][kB + 1];  // (lane = column); pitch kB + 1: both conflict-free
};

#ifdef DSE_EIG2_VARIANTS
// ---- A/B record (tools/probe_eig2.cpp builds with -DDSE_EIG2_VARIANTS; not in libdse.so): the
// round-4 chase that waits for task (s - 1, t + 2) complete (variant 0, 336 ms at 2^14) and its
// per-task timing build (DBG, option EIG2_CHASE_DBG of the probe).  Its polls are unbounded.
__device__ __forceinline__ long long rt_now() { return (long long)__builtin_amdgcn_s_memrealtime(); }

template <bool DBG>
__device__ void chase_task(double* __restrict__ S, int n, int s, int t, ChaseVec& B, double* __restrict__ rf,
                           long long* tl) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 31, h = lane >> 5, i0 = 16 * h;
  const int col = t == 0 ? s : s + (t - 1) * kB + 1;
  const int r0 = t == 0 ? s + 1 : s + t * kB + 1;
  const int m = min(kB, n - r0);
  const int nL = t == 0 ? 1 : kB;
  const int mr = max(0, min(kB, n - r0 - m));
  const __amdgpu_buffer_rsrc_t rs = band_rsrc(S, n);
  double Lc[16], Dc[16], Rr[16];
  // L(i, j) = A(r0 + i, col + j); D(i, j) = A(r0 + i, r0 + j) (i >= j stored); R(i, jj) =
  // A(r0 + m + i, r0 + jj).  Memory layout: lane = row i (band column contiguous), load q takes
  // columns 2 q + h; R is read in its compute layout (lane = row, contiguous already).
  const int eR = (r0 + i0) * kLD + (m + j - i0);  // + q (kLD - 1)
  {
    double Lm[16], Dm[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = 2 * q + h;
      Lm[q] = (j < m && c < nL) ? bload(rs, (col + c) * kLD + (r0 - col - c) + j) : 0.0;
      Dm[q] = (j < m && c < m && j >= c) ? bload(rs, (r0 + c) * kLD + j - c) : 0.0;
      const int jj = i0 + q;
      Rr[q] = (j < mr && jj < m) ? bload(rs, eR + q * (kLD - 1)) : 0.0;
    }
    if constexpr (DBG) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tl[0] = rt_now();
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      B.Lt[j][2 * q + h] = Lm[q];
      B.Dt[j][2 * q + h] = Dm[q];
    }
  }
  wave_sync();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int i = i0 + q;
    Lc[q] = B.Lt[i][j];
    Dc[q] = i >= j ? B.Dt[i][j] : B.Dt[j][i];
  }
  // the reflector of L(:, 0)
  if (lane < kB) B.x[lane] = B.Lt[lane][0];
  wave_sync();
  const double xi = lane < kB ? B.x[lane] : 0.0;
  const double alpha = B.x[0];
  const double s2 = wave_sum((lane >= 1 && lane < m) ? xi * xi : 0.0);
  double beta = alpha, tau = 0.0, sc = 0.0;
  if (s2 != 0.0) {
    beta = -copysign(sqrt(alpha * alpha + s2), alpha);
    tau = (beta - alpha) / beta;
    sc = 1.0 / (alpha - beta);
  }
  if (lane < kB) B.v[lane] = lane == 0 ? 1.0 : (lane < m ? xi * sc : 0.0);
  wave_sync();
  if constexpr (DBG) tl[1] = rt_now();
  if (tau != 0.0) {
    double vh[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) vh[q] = B.v[i0 + q];
    const double vj = B.v[j];
    // L <- H L (columns 1 ..; column 0 becomes beta e1)
    {
      double p = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) p = fma(vh[q], Lc[q], p);
      const double wl = tau * (p + __shfl_xor(p, 32, 64));
      if (j == 0) {
#pragma unroll
        for (int q = 0; q < 16; ++q) Lc[q] = (h == 0 && q == 0) ? beta : 0.0;
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) Lc[q] = fma(-wl, vh[q], Lc[q]);
      }
    }
    // D <- H D H: y_j = D(:, j) . v (symmetric), w = tau y - tau^2 (v . y) v / 2,
    // D -= v w^T + w v^T
    {
      double p = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) p = fma(vh[q], Dc[q], p);
      const double y = p + __shfl_xor(p, 32, 64);
      const double K = wave_sum(lane < kB ? vj * y : 0.0);
      const double wj = tau * y - 0.5 * tau * tau * K * vj;
      if (lane < kB) B.w[lane] = wj;
      wave_sync();
#pragma unroll
      for (int q = 0; q < 16; ++q) Dc[q] -= vh[q] * wj + B.w[i0 + q] * vj;
    }
    // R <- R H (lane = row j, columns of half h): z = R(j, :) . v, R(j, :) -= tau z v^T
    {
      double p = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) p = fma(vh[q], Rr[q], p);
      const double z = tau * (p + __shfl_xor(p, 32, 64));
#pragma unroll
      for (int q = 0; q < 16; ++q) Rr[q] = fma(-z, vh[q], Rr[q]);
    }
    if constexpr (DBG) tl[2] = rt_now();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int jj = i0 + q;
      if (j < mr && jj < m) bstore(rs, eR + q * (kLD - 1), Rr[q]);
    }
    wave_sync();  // every lane's reads of Lt / Dt above are done
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      B.Lt[i0 + q][j] = Lc[q];
      B.Dt[i0 + q][j] = Dc[q];
    }
    wave_sync();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int c = 2 * q + h;
      if (j < m && c < nL) bstore(rs, (col + c) * kLD + (r0 - col - c) + j, B.Lt[j][c]);
      if (j < m && c < m && j >= c) bstore(rs, (r0 + c) * kLD + j - c, B.Dt[j][c]);
    }
  }
  if (lane == 0) rf[kB] = tau;
  if (lane < kB) rf[lane] = B.v[lane];
  wave_sync();
}

// Workers = waves (kChaseWG per workgroup, the workgroups spread over the chip); worker w takes
// sweeps w, w + W, ...; task (s, t) waits until sweep s - 1 has finished task t + 2 (or all its
// tasks): the strips of (s, t) and (s - 1, t + 3) share no entry (tools/proto_two_stage.py).
// prog[s] = tasks of sweep s done (zeroed before); relaxed agent-scope (sc1) flag stores and polls.
// DBG: per worker, the sums of the poll wait, load, compute + store issue and store drain times
// (100 MHz ticks) and the task count into dbg[5 w ..].
template <bool DBG>
__global__ void __launch_bounds__(64 * kChaseWG)
k_sb2st(double* __restrict__ S, int n, double* __restrict__ refl, const long long* __restrict__ goff,
        int* __restrict__ prog, long long* __restrict__ dbg) {
  __shared__ ChaseVec lds[kChaseWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int W = gridDim.x * kChaseWG, w = blockIdx.x * kChaseWG + wv;
  ChaseVec& B = lds[wv];
  long long sw = 0, sl = 0, sc = 0, sd = 0, cnt = 0;
  for (int s = w; s < n - 1; s += W) {
    const int nt = chase_tasks(n, s);
    const int ntp = s > 0 ? chase_tasks(n, s - 1) : 0;
    for (int t = 0; t < nt; ++t) {
      long long t0 = 0, t1 = 0, tls[3] = {0, 0, 0}, t2 = 0;
      if constexpr (DBG) t0 = rt_now();
      if (s > 0) {
        const int need = min(ntp, t + 3);
        while (__hip_atomic_load(prog + s - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need)
          __builtin_amdgcn_s_sleep(1);
      }
      if constexpr (DBG) t1 = rt_now();
      chase_task<DBG>(S, n, s, t, B, refl_at(refl, goff, s, t), tls);
      const long long tl = tls[0];
      if constexpr (DBG) t2 = rt_now();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(prog + s, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (DBG) {
        const long long t3 = rt_now();
        sw += t1 - t0, sl += tl - t1, sc += t2 - tl, sd += t3 - t2, ++cnt;
        // per sweep: start (after the wait) and flag times of tasks 0, 1, 2
        if (lane == 0 && t < 3) dbg[5 * 4096 + 6 * s + 2 * t] = t1, dbg[5 * 4096 + 6 * s + 2 * t + 1] = t3;
        // every task (n <= 4096): wait start, start, load done, flag at (s nt(0) + t) 4
        if (lane == 0 && n <= 4096) {
          long long* q = dbg + 5 * 4096 + 6 * (size_t)n + ((size_t)s * chase_tasks(n, 0) + t) * 4;
          q[0] = tls[1], q[1] = t1, q[2] = tl, q[3] = t3;
          q[4 * chase_tasks(n, 0) * (size_t)n] = tls[2];  // second plane: after the updates
          q[4 * chase_tasks(n, 0) * (size_t)n + 1] = t2;
        }
      }
    }
  }
  if constexpr (DBG) {
    if (lane == 0) {
      dbg[5 * w] = sw, dbg[5 * w + 1] = sl, dbg[5 * w + 2] = sc, dbg[5 * w + 3] = sd, dbg[5 * w + 4] = cnt;
    }
  }
}
#endif  // DSE_EIG2_VARIANTS

// The chase with the next task's operands prefetched (round 4, default).  Task (s, t)'s R block is
// its next task's L block: it stays in registers (stored there, as L), so a task loads only D and R,
// and it loads them during the previous task, once sweep s - 1's task t + 1 is done (prog[s - 1] >=
// t + 2: D_t and R_t are then final but for R_t(b-1, b-1)).  That one element is the annihilated
// column's head of task (s - 1, t + 2) (its L(0, 0) = beta): the producer publishes beta in the
// mailbox mb[(s - 1) MT + t + 2] as soon as it has it and never stores the element; the consumer
// polls the mailbox (8-B sc1, sentinel all-ones) instead of waiting for the whole task.  So task
// (s, t) waits for (s - 1, t + 1) complete + beta of (s - 1, t + 2) (was: (s - 1, t + 2) complete).
// EARLY: the next task's D / R loads are issued before this task's stores (their blocks are
// disjoint), so the store drain before the progress flag also lands them.
template <bool EARLY>
__global__ void __launch_bounds__(64 * kChaseWG)
k_sb2st_pf(double* __restrict__ S, int n, double* __restrict__ refl, const long long* __restrict__ goff,
           int* __restrict__ prog, unsigned long long* __restrict__ mb, int MT, int* __restrict__ err, int spin) {
  __shared__ ChaseVec lds[kChaseWG];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int W = gridDim.x * kChaseWG, w = blockIdx.x * kChaseWG + wv;
  const int j = lane & 31, h = lane >> 5, i0 = 16 * h;
  ChaseVec& B = lds[wv];
  const __amdgpu_buffer_rsrc_t rs = band_rsrc(S, n);
  for (int s = w; s < n - 1; s += W) {
    const int nt = chase_tasks(n, s);
    const int ntp = s > 0 ? chase_tasks(n, s - 1) : 0;
    auto wait_prog = [&](int need) {  // bounded (poll_give_up): a give-up drains the launch
      if (s > 0)
        for (int it = 0; __hip_atomic_load(prog + s - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need; ++it) {
          if (poll_give_up(err, spin, it)) break;
          __builtin_amdgcn_s_sleep(1);
        }
    };
    double Lcar[16], Dm[16], Rm[16];  // carried L (R layout: lane = row), D (memory layout), R
    auto load_dr = [&](int t) {
      const int r0 = t == 0 ? s + 1 : s + t * kB + 1;
      const int m = min(kB, n - r0), mr = max(0, min(kB, n - r0 - m));
      const int eR = (r0 + i0) * kLD + (m + j - i0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = 2 * q + h, jj = i0 + q;
        Dm[q] = (j < m && c < m && j >= c) ? bload(rs, (r0 + c) * kLD + j - c) : 0.0;
        Rm[q] = (j < mr && jj < m) ? bload(rs, eR + q * (kLD - 1)) : 0.0;
      }
    };
    wait_prog(min(ntp, 2));
#pragma unroll
    for (int q = 0; q < 16; ++q) Lcar[q] = 0.0;
    double L0 = (j < min(kB, n - s - 1) && h == 0) ? bload(rs, s * kLD + 1 + j) : 0.0;  // L_0 = A(s + 1 + j, s)
    load_dr(0);
    for (int t = 0; t < nt; ++t) {
      const int col = t == 0 ? s : s + (t - 1) * kB + 1;
      const int r0 = t == 0 ? s + 1 : s + t * kB + 1;
      const int m = min(kB, n - r0);
      const int nL = t == 0 ? 1 : kB;
      const int mr = max(0, min(kB, n - r0 - m));
      double* rf = refl_at(refl, goff, s, t);
      // L and D into LDS (memory layout: lane = row j)
      if (t == 0) {
        if (h == 0) B.Lt[j][0] = L0;
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) B.Lt[j][i0 + q] = Lcar[q];
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) B.Dt[j][2 * q + h] = Dm[q];
      // R(b-1, b-1) from task (s - 1, t + 2)
      if (s > 0 && mr == kB) {
        unsigned long long bits;
        for (int it = 0;; ++it) {  // bounded: a NaN beta is the sentinel; a give-up drains the launch
          bits = __hip_atomic_load(mb + (size_t)(s - 1) * MT + t + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (bits != ~0ull || poll_give_up(err, spin, it)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        if (j == kB - 1 && h == 1) Rm[15] = __builtin_bit_cast(double, bits);
      }
      wave_sync();
      double Lc[16], Dc[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int i = i0 + q;
        Lc[q] = (t == 0 && j > 0) ? 0.0 : B.Lt[i][j];
        Dc[q] = i >= j ? B.Dt[i][j] : B.Dt[j][i];
      }
      if (lane < kB) B.x[lane] = B.Lt[lane][0];
      wave_sync();
      const double xi = lane < kB ? B.x[lane] : 0.0;
      const double alpha = B.x[0];
      const double s2 = wave_sum((lane >= 1 && lane < m) ? xi * xi : 0.0);
      double beta = alpha, tau = 0.0, sc = 0.0;
      if (s2 != 0.0) {
        beta = -copysign(sqrt(alpha * alpha + s2), alpha);
        tau = (beta - alpha) / beta;
        sc = 1.0 / (alpha - beta);
      }
      // L(0, 0)'s new value goes to the consumer (s + 1, t - 2) now
      if (t >= 2 && lane == 0)
        __hip_atomic_store(mb + (size_t)s * MT + t, __builtin_bit_cast(unsigned long long, beta), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      if (lane < kB) B.v[lane] = lane == 0 ? 1.0 : (lane < m ? xi * sc : 0.0);
      wave_sync();
      if (tau != 0.0) {
        double vh[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) vh[q] = B.v[i0 + q];
        const double vj = B.v[j];
        {  // L <- H L (column 0 becomes beta e1)
          double p = 0.0;
#pragma unroll
          for (int q = 0; q < 16; ++q) p = fma(vh[q], Lc[q], p);
          const double wl = tau * (p + __shfl_xor(p, 32, 64));
          if (j == 0) {
#pragma unroll
            for (int q = 0; q < 16; ++q) Lc[q] = (h == 0 && q == 0) ? beta : 0.0;
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) Lc[q] = fma(-wl, vh[q], Lc[q]);
          }
        }
        {  // D <- H D H
          double p = 0.0;
#pragma unroll
          for (int q = 0; q < 16; ++q) p = fma(vh[q], Dc[q], p);
          const double y = p + __shfl_xor(p, 32, 64);
          const double K = wave_sum(lane < kB ? vj * y : 0.0);
          const double wj = tau * y - 0.5 * tau * tau * K * vj;
          if (lane < kB) B.w[lane] = wj;
          wave_sync();
#pragma unroll
          for (int q = 0; q < 16; ++q) Dc[q] -= vh[q] * wj + B.w[i0 + q] * vj;
        }
        {  // R <- R H (lane = row j)
          double p = 0.0;
#pragma unroll
          for (int q = 0; q < 16; ++q) p = fma(vh[q], Rm[q], p);
          const double z = tau * (p + __shfl_xor(p, 32, 64));
#pragma unroll
          for (int q = 0; q < 16; ++q) Rm[q] = fma(-z, vh[q], Rm[q]);
        }
      }
      if (EARLY && t + 1 < nt) {
#pragma unroll
        for (int q = 0; q < 16; ++q) Lcar[q] = Rm[q];
        wait_prog(min(ntp, t + 3));
        load_dr(t + 1);
      }
      // stores: L always (a carried L is only in registers), but L(0, 0) from t = 2 on (the
      // consumer's); D when changed; R stays in registers (the next task's L)
      wave_sync();  // every lane's reads of Lt / Dt above are done
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        B.Lt[i0 + q][j] = Lc[q];
        B.Dt[i0 + q][j] = Dc[q];
      }
      wave_sync();
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int c = 2 * q + h;
        if (j < m && c < nL && !(t >= 2 && j == 0 && c == 0))
          bstore(rs, (col + c) * kLD + (r0 - col - c) + j, B.Lt[j][c]);
        if (tau != 0.0 && j < m && c < m && j >= c) bstore(rs, (r0 + c) * kLD + j - c, B.Dt[j][c]);
      }
      if (lane == 0) rf[kB] = tau;
      if (lane < kB) rf[lane] = B.v[lane];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(prog + s, t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!EARLY && t + 1 < nt) {
#pragma unroll
        for (int q = 0; q < 16; ++q) Lcar[q] = Rm[q];
        wait_prog(min(ntp, t + 3));
        load_dr(t + 1);
      }
      wave_sync();
    }
  }
}

// d, e of the tridiagonal from the band
__global__ void k_sb_tridiag(const double* __restrict__ S, int n, double* __restrict__ d, double* __restrict__ e) {
  const int c = (int)(blockIdx.x * 256 + threadIdx.x);
  if (c >= n) return;
  d[c] = S[(size_t)c * kLD];
  e[c] = c + 1 < n ? S[(size_t)c * kLD + 1] : 0.0;
}

// ---- Z <- Q2 Z ----------------------------------------------------------------------------------

// 64 columns (lane = column) per workgroup of kQ2Waves waves.  Blocks of kQ2NB sweeps are applied
// from the last to the first; block i of that order (i = 0, 1, ...) goes to wave i % kQ2Waves, which
// trails the wave of block i - 1 by one group: group t of block i needs block i - 1's group t done
// (its window has then moved below every row group t touches; tools/proto_two_stage.py's order).
// In a block, t ascending; the group (block, t)'s reflectors (s descending) act on window rows
// lo .. lo + 62, lo = s0 + t b + 1, reflector s at window offset s - s0 (compile time).  The next
// group's records (contiguous, refl_at) are loaded into registers while this group is applied.
// Z is row-major here (Zt, row stride ldt: a window row of the 64 columns is one 512-B load).  Waves
// of one workgroup hand rows over with a workgroup-scope release fence before the LDS progress
// word and an acquire fence after the poll (the memory model's own workgroup hand-off).
constexpr int kQ2Rec = kQ2NB * kRec;             // doubles per group
constexpr int kQ2PerLane = (kQ2Rec + 63) / 64;    // staging loads per lane
[[maybe_unused]] constexpr int kQ2Waves = 4;  // (probe variants)
// NC columns per lane (64 NC per workgroup): each reflector value read from LDS serves 2 NC FMAs.
// PF: group t + 1's new rows are loaded under group t (and released one group late); PAIR: two
// reflectors per step (both dot products on one window).
// DMA: the group records go global -> LDS directly (global_load_lds, 16 B per lane, double-buffered,
// no staging registers); W waves per workgroup.
constexpr int kQ2Dma = (kQ2Rec * 8 + 1023) / 1024;  // 1-KiB copies per group
// SC: the reflector values are read with scalar loads straight from the records (uniform across the
// wave: SGPR operands of the FMAs, no LDS traffic); the records are written by earlier launches.
template <int NC, bool PF, bool PAIR, bool DMA, int W, bool SC = false, bool NL = false>
__global__ void __launch_bounds__(64 * W)
k_sb_q2(double* __restrict__ Zt, int ldt, int n, const double* __restrict__ refl, const long long* __restrict__ goff) {
  constexpr int kBuf = SC ? 2 : DMA ? 2 * kQ2Dma * 128 : kQ2PerLane * 64;  // doubles per wave
  __shared__ __attribute__((aligned(16))) double rvs[W][kBuf];
  __shared__ int state[W];  // (block order index) * 65536 + groups done (65535: block done)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double* rv = rvs[wv];
  const int col0 = blockIdx.x * 64 * NC;
  // Zt through a buffer resource at the workgroup's first column: rows past n and columns past n
  // take an out-of-range offset (loads read 0, stores are dropped), so no row is a branch
  const size_t zbytes = ((size_t)n * ldt - (size_t)col0) * 8;
  const __amdgpu_buffer_rsrc_t zr = ptr_rsrc(Zt + (size_t)col0, std::min<size_t>(zbytes, 0xfffffff0u));
  auto zoff = [&](int row, int c) -> uint32_t {
    const int cl = lane + 64 * c;
    return (col0 + cl < n && row < n) ? ((uint32_t)row * (uint32_t)ldt + (uint32_t)cl) * 8u : 0xffffffffu;
  };
  auto zld = [&](int row, int c) -> double {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zr, zoff(row, c), 0, 0));
  };
  auto zst = [&](int row, int c, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), zr, zoff(row, c), 0, 0);
  };
  if (lane == 0) state[wv] = -1;
  __syncthreads();
  const int ns = n - 1;
  const int nblk = (ns + kQ2NB - 1) / kQ2NB;
  const int pw = (wv + W - 1) % W;  // the wave of the previous block
  for (int i = wv; i < nblk; i += W) {
    const int blk = nblk - 1 - i;
    const int s0 = blk * kQ2NB;
    const int T0 = chase_tasks(n, s0);
    auto wait_prev = [&](int t) {  // block i - 1 has finished group t (or the whole block)
      if (i == 0) return;
      const int need = (i - 1) * 65536 + min(t + 1, 65535);
      while (__hip_atomic_load(&state[pw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
        __builtin_amdgcn_s_sleep(1);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    };
    const double* gb = refl + goff[blk];
    double pre[DMA ? 1 : kQ2PerLane];
    auto dma = [&](int t) {  // group t's records into buffer t & 1
      const char* src = reinterpret_cast<const char*>(gb + (size_t)t * kQ2Rec) + lane * 16;
      double* dst = rv + (t & 1) * kQ2Dma * 128;
#pragma unroll
      for (int q = 0; q < kQ2Dma; ++q)
        __builtin_amdgcn_global_load_lds(src + q * 1024, (__attribute__((address_space(3))) void*)(dst + q * 128), 16, 0, 0);
    };
    if constexpr (SC) {
    } else if constexpr (DMA) {
      dma(0);
    } else {
#pragma unroll
      for (int q = 0; q < kQ2PerLane; ++q) {
        const int e = q * 64 + lane;
        pre[q] = e < kQ2Rec ? gb[e] : 0.0;
      }
    }
    double win[NC][kQ2Win];
    int lo = s0 + 1;
    wait_prev(0);
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = 0; r < kQ2Win; ++r) win[c][r] = zld(lo + r, c);
    for (int t = 0; t < T0; ++t) {
      // NC = 1: the rows group t + 1 adds (lo + kQ2Win ..), loaded while group t is applied: block
      // i - 1 has stored them once its group t + 1 is flagged
      double nxt[kB];
      auto prefetch_rows = [&]() {
        if constexpr (PF) {
          if (t + 1 < T0) {
            wait_prev(t + 1);
#pragma unroll
            for (int r = 0; r < kB; ++r) nxt[r] = zld(lo + kQ2Win + r, 0);
          }
        }
      };
      if constexpr (!DMA) prefetch_rows();
      const double* rg = rv;  // this group's records
      if constexpr (SC) {
        const uint64_t ga = (uint64_t)(gb + (size_t)t * kQ2Rec);
        const uint32_t ghi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(ga >> 32));
        const uint32_t glo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)ga);  // unsigned: no sign extension
        rg = (const double*)(((uint64_t)ghi << 32) | (uint64_t)glo);
      } else if constexpr (DMA) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // group t's copy (and the window rows) landed
        __builtin_amdgcn_wave_barrier();
        rg = rv + (t & 1) * kQ2Dma * 128;
        if (t + 1 < T0) dma(t + 1);
        prefetch_rows();  // after the wait: the next rows load under this group
      } else {
#pragma unroll
        for (int q = 0; q < kQ2PerLane; ++q) rv[q * 64 + lane] = pre[q];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (t + 1 < T0) {
          const double* g = gb + (size_t)(t + 1) * kQ2Rec;
#pragma unroll
          for (int q = 0; q < kQ2PerLane; ++q) {
            const int e = q * 64 + lane;
            pre[q] = e < kQ2Rec ? g[e] : 0.0;
          }
        }
      }
      if constexpr (!PAIR) {  // one reflector at a time
#pragma unroll
        for (int u = kQ2NB - 1; u >= 0; --u) {
          typedef const __attribute__((address_space(4))) double* kptr;
          const kptr r = SC ? (kptr)(rg + u * kRec) : (kptr) nullptr;
          const double* rl = rg + u * kRec;
          auto rval = [&](int k) -> double { return SC ? r[k] : rl[k]; };
          const double tau = rval(kB);
          if (tau == 0.0) continue;  // uniform
          double d[NC][4];
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int x = 0; x < 4; ++x) d[c][x] = 0.0;
#pragma unroll
          for (int k = 0; k < kB; k += 4)
#pragma unroll
            for (int x = 0; x < 4; ++x) {
              const double p = rval(k + x);
#pragma unroll
              for (int c = 0; c < NC; ++c) d[c][x] = fma(p, win[c][u + k + x], d[c][x]);
            }
          double g[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) g[c] = tau * ((d[c][0] + d[c][1]) + (d[c][2] + d[c][3]));
#pragma unroll
          for (int k = 0; k < kB; ++k) {
            const double p = rval(k);
#pragma unroll
            for (int c = 0; c < NC; ++c) win[c][u + k] = fma(-g[c], p, win[c][u + k]);
          }
        }
      } else {
      // reflectors u and u - 1 together: both dot products on the same window, then
      // g2 = tau2 (d2 - g1 c) with c = v_{u-1}[1:] . v_u[:-1] (record slot kB + 1, k_sb_q2c)
#pragma unroll
      for (int u = kQ2NB - 1; u >= 1; u -= 2) {
        const double* r1 = rg + u * kRec;
        const double* r2 = rg + (u - 1) * kRec;
        const double tau1 = r1[kB], tau2 = r2[kB];
        if (tau1 == 0.0 && tau2 == 0.0) continue;  // uniform
        double a[NC][4], b[NC][4];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int x = 0; x < 4; ++x) a[c][x] = b[c][x] = 0.0;
#pragma unroll
        for (int k = 0; k < kB; k += 4)
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const double p1 = r1[k + x], p2 = r2[k + x];
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              a[c][x] = fma(p1, win[c][u + k + x], a[c][x]);
              b[c][x] = fma(p2, win[c][u - 1 + k + x], b[c][x]);
            }
          }
        const double cpl = r1[kB + 1];
        double g1[NC], g2[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          g1[c] = tau1 * ((a[c][0] + a[c][1]) + (a[c][2] + a[c][3]));
          g2[c] = tau2 * (((b[c][0] + b[c][1]) + (b[c][2] + b[c][3])) - g1[c] * cpl);
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          const double p1 = r1[k];
#pragma unroll
          for (int c = 0; c < NC; ++c) win[c][u + k] = fma(-g1[c], p1, win[c][u + k]);
        }
#pragma unroll
        for (int k = 0; k < kB; ++k) {
          const double p2 = r2[k];
#pragma unroll
          for (int c = 0; c < NC; ++c) win[c][u - 1 + k] = fma(-g2[c], p2, win[c][u - 1 + k]);
        }
      }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if constexpr (PF) {
        // group t - 1's rows (stored one group ago) are released now, their stores long complete
        if (t > 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0)
            __hip_atomic_store(&state[wv], i * 65536 + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      }
      // rows lo .. lo + b - 1 are final for this block
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int r = 0; r < kB; ++r) zst(lo + r, c, win[c][r]);
      if constexpr (!PF) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0)
          __hip_atomic_store(&state[wv], i * 65536 + t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (t + 1 < T0) {
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int r = 0; r < kQ2Win - kB; ++r) win[c][r] = win[c][r + kB];
        if constexpr (PF) {
#pragma unroll
          for (int r = 0; r < kB; ++r) win[0][kQ2Win - kB + r] = nxt[r];
        } else {
          wait_prev(t + 1);
          if constexpr (!NL) {  // NL (probe ablation only, wrong results): the new rows not loaded
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
              for (int r = 0; r < kB; ++r) win[c][kQ2Win - kB + r] = zld(lo + kQ2Win + r, c);
          }
        }
        lo += kB;
      }
    }
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int r = kB; r < kQ2Win; ++r) zst(lo + r, c, win[c][r]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_store(&state[wv], i * 65536 + 65535, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
}

// slot kB + 1 of record u >= 1 of each group: c = v_{u-1}[1:kB] . v_u[0:kB-1] (the coupling of the
// pair k_sb_q2 applies together; 0 for u = 0)
__global__ void __launch_bounds__(256)
k_sb_q2c(double* __restrict__ refl, size_t nrec) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= nrec) return;
  double c = 0.0;
  if (e % kQ2NB != 0) {
    const double* a = refl + e * kRec;
    const double* p = a - kRec;
#pragma unroll
    for (int k = 0; k < kB - 1; ++k) c = fma(p[k + 1], a[k], c);
  }
  refl[e * kRec + kB + 1] = c;
}

// B (row-major, ld ldb) = A (column-major, ld lda), n x n; or back (the same map with the roles of
// the two layouts swapped): 64 x 64 tiles through LDS, reads and writes along contiguous rows
__global__ void __launch_bounds__(256)
k_sb_transpose(const double* __restrict__ A, int lda, double* __restrict__ B, int ldb, int n) {
  __shared__ double tile[64][65];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 64, tid = threadIdx.x;
  const int a = tid & 63, b0 = tid >> 6;
  for (int b = b0; b < 64; b += 4) {  // column c0 + b of A, rows r0 + a
    const int r = r0 + a, c = c0 + b;
    tile[b][a] = (r < n && c < n) ? A[(size_t)c * lda + r] : 0.0;
  }
  __syncthreads();
  for (int b = b0; b < 64; b += 4) {  // row r0 + b of B, columns c0 + a
    const int r = r0 + b, c = c0 + a;
    if (r < n && c < n) B[(size_t)r * ldb + c] = tile[a][b];
  }
}

#ifdef DSE_EIG2_VARIANTS
// A/B record, probe builds only (tools/probe_eig2.cpp, -DDSE_EIG2_VARIANTS); libdse.so runs the
// defaults as constants.  k_sb_q2 variant (2^14, profiles/r04/eig2_q2_variants.txt): 0 one
// reflector at a time, rows loaded after each group (346 ms); 1 pairs + the next rows under the
// group (361); 2 two columns per lane (649); 3 pairs (357); 4 = 0 with the records copied global ->
// LDS (371); 5 = 4 with 8 waves per workgroup, 2 per SIMD (296, default); 6 / 7 the reflector values
// as scalar-load SGPR operands, 8 / 4 waves (512 / 921: each reflector waits on its s_loads); 8 =
// 5 with the next rows loaded under the group (354 vs 296 ms, round 5: 25 VGPRs of spill; issued
// late in the group the same, 378 ms); 9 = 5 without the new window rows (ablation, wrong results:
// 249 ms, so their exposed load is ~47 ms).  Round 5 also measured the update pass re-reading the
// reflector from LDS instead of holding it (405 ms; with the prefetch 432): the broadcast LDS reads
// are part of the bound (profiles/r05/ab/eig2_q2_variants_r05.txt)
int g_q2_variant = 5;
// the chase: 0 k_sb2st (waits for (s - 1, t + 2) complete: 336 ms at 2^14), 1 k_sb2st_pf (243 ms,
// default), 2 k_sb2st_pf with the next task's loads issued before the stores (280 ms: the progress
// flag then waits for sweep s - 1 too)
int g_chase_variant = 1;
// the trailing update's grid: 0 2-D (nbk x nbk, the upper tiles idle), 1 1-D over the lower tiles
// (band 413-425 vs 377 ms at 2^14: the 2-D order, I fastest, keeps a column's V/W rows warm), 2
// k_sb_syr2k2 (P in LDS, kSyr2kNJ tiles per workgroup, 16-B row pairs; default)
int g_syr2k_tri = 2;
#else
constexpr int g_q2_variant = 5, g_chase_variant = 1, g_syr2k_tri = 2;
#endif

struct Eig2Ws {
  double* tau1;     // n: stage-1 reflectors (zero where none)
  double* T;        // panels x b x b
  double* Vw2[2];   // n x b, by panel parity
  double* Vt2[2];   // n x b, row-major, by panel parity
  double* part2v;   // V^T V partials (the side stream's)
  double* Y;        // n x b
  double* Wt;       // n x b, row-major
  double* Yp;       // symm partials: chunks x b x n
  double* Zt;       // n x n: Z row-major for the Q2 application
  double* M;        // b x b
  double* Gm;       // b x b
  double* part;     // 2 x 128 x (b + 1)
  double* part2;    // (n / kVtyRows + 2) x b x b: V^T Y partials
  double* piv;      // 2 x b
  double* S;        // n x kLD band
  double* refl;     // chase reflectors x (b + 1)
  double* orm;      // ormtr_lower workspace
  long long* goff;  // n / kQ2NB + 1: group-major reflector offsets per block of sweeps
  int* prog;        // n
  unsigned long long* mb;  // n x (chase_tasks(n, 0) + 1): the chase's mailboxes
  int* cnt;         // 1
  int* err;         // 1: a bounded poll gave up (poll_give_up)
};

// doubles of the group-major reflector records: per block of kQ2NB sweeps, chase_tasks(first
// sweep) groups of kQ2NB records
size_t chase_refl_doubles(int n, std::vector<long long>* goff = nullptr) {
  const int ns = n - 1, nblk = (ns + kQ2NB - 1) / kQ2NB;
  size_t k = 0;
  if (goff) goff->assign(nblk + 1, 0);
  for (int b = 0; b < nblk; ++b) {
    if (goff) (*goff)[b] = (long long)k;
    k += (size_t)chase_tasks(n, b * kQ2NB) * kQ2NB * kRec;
  }
  if (goff) (*goff)[nblk] = (long long)k;
  return k;
}

// the workspace's arrays from base (nullptr: offsets only, for the size)
Eig2Ws carve2(void* work, int n, size_t* bytes = nullptr) {
  const int panels = n / kB + 1;
  size_t off = 0;
  const uintptr_t base = reinterpret_cast<uintptr_t>(work);
  auto take = [&](size_t b) {
    const size_t o = off;
    off += (b + 255) / 256 * 256;
    return reinterpret_cast<void*>(base + o);
  };
  Eig2Ws w;
  w.tau1 = (double*)take((size_t)n * 8);
  w.T = (double*)take((size_t)panels * kB * kB * 8);
  for (int q = 0; q < 2; ++q) {
    w.Vw2[q] = (double*)take((size_t)n * kB * 8);
    w.Vt2[q] = (double*)take((size_t)n * kB * 8);
  }
  w.part2v = (double*)take(((size_t)n / kVtyRows + 2) * kB * kB * 8);
  w.Y = (double*)take((size_t)n * kB * 8);
  w.Wt = (double*)take((size_t)n * kB * 8);
  w.Zt = (double*)take((size_t)n * n * 8);
  w.Yp = (double*)take((size_t)((n / kT + 1 + kSymmCh - 1) / kSymmCh) * kB * n * 8);
  w.M = (double*)take((size_t)kB * kB * 8);
  w.Gm = (double*)take((size_t)kB * kB * 8);
  w.part = (double*)take(((size_t)kB * 128 * (kB + 1) + (size_t)kB * kB) * 8);  // + the pivot rows
  w.piv = (double*)take((size_t)2 * kB * 8);
  w.part2 = (double*)take(((size_t)n / kVtyRows + 2) * kB * kB * 8);
  w.S = (double*)take((size_t)n * kLD * 8);
  w.refl = (double*)take(chase_refl_doubles(n) * 8);
  w.orm = (double*)take(sytrd_workspace(n));
  w.goff = (long long*)take(((size_t)n / kQ2NB + 2) * 8);
  w.prog = (int*)take((size_t)n * 4);
  w.mb = (unsigned long long*)take((size_t)n * (chase_tasks(n, 0) + 1) * 8);
  w.cnt = (int*)take(256);
  w.err = (int*)take(256);
  if (bytes) *bytes = off;
  return w;
}

}  // namespace

#ifdef DSE_EIG2_VARIANTS
void set_eig2_q2_variant(int v) { g_q2_variant = v; }
void set_eig2_chase_variant(int v) { g_chase_variant = v; }
void set_eig2_syr2k_tri(int v) { g_syr2k_tri = v; }
#endif

size_t eig2_workspace(int n) {
  size_t b = 0;
  carve2(nullptr, n, &b);
  return b;
}

// Panel p + 1's QR (and its V copies, V^T V, T) runs on a second stream under panel p's trailing
// update: the update first rewrites A22's first kB columns (the next panel and its diagonal block),
// then the rest while the panel is factored; V, its copies and the V^T V partials are double-buffered
// by panel parity.
int sy2sb_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, void* work, int spin) {
  (void)h;
  Eig2Ws ws = carve2(work, n);
  if (hipMemsetAsync(ws.tau1, 0, (size_t)n * 8, st) != hipSuccess) return -1;
  if (hipMemsetAsync(ws.cnt, 0, sizeof(int), st) != hipSuccess) return -1;
  if (hipMemsetAsync(ws.err, 0, sizeof(int), st) != hipSuccess) return -1;
  hipStream_t s2 = nullptr;
  hipEvent_t evS = nullptr, evP = nullptr;
  if (hipStreamCreateWithFlags(&s2, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&evS, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&evP, hipEventDisableTiming) != hipSuccess)
    return -1;
  // the panel at column i: QR, V copies, V^T V partials, T, on stream q
  auto factor = [&](int i, int p, hipStream_t q) -> int {
    const int m = n - i - kB, par = p & 1;
    double* P = A + (size_t)i * lda + i + kB;
    const int G = (m + kPanelRows - 1) / kPanelRows, ng = (m + kVtyRows - 1) / kVtyRows, k = std::min(m, kB);
    if (G > 128) return -2;
    if (hipMemsetAsync(ws.part, 0xff, ((size_t)kB * G * (kB + 1) + (size_t)kB * kB) * 8, q) != hipSuccess) return -1;
    hipLaunchKernelGGL(k_panel_qr, dim3(G), dim3(kPanelRows), 0, q, P, lda, m, ws.tau1 + i, ws.part,
                       ws.part + (size_t)kB * G * (kB + 1), ws.Vw2[par], ws.Vt2[par], ws.err, spin);
    hipLaunchKernelGGL(k_sb_vty, dim3(ng), dim3(256), 0, q, ws.Vw2[par], ws.Vw2[par], m, ws.part2v);
    hipLaunchKernelGGL(k_sb_tmat, dim3(1), dim3(kB * kB), 0, q, ws.part2v, ng, k, ws.tau1 + i,
                       ws.T + (size_t)p * kB * kB);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  };
  // A22 -= V W^T + W V^T on the columns cmin .. cmax - 1 (k_sb_syr2k2 addresses A22 with 32-bit
  // buffer offsets: only while the whole matrix spans < 4 GiB)
  const bool wide_ok = (size_t)n * (size_t)lda * 8u < ((size_t)1 << 32);
  auto launch_syr2k = [&](double* A22, int m, const double* Vt, int cmin, int cmax) {
    const int nbk = (m + kT - 1) / kT;
    if (g_syr2k_tri == 2 && wide_ok) {
      const int nj = ((cmax - 1) / kT - cmin / kT) / kSyr2kNJ + 1;
      hipLaunchKernelGGL(k_sb_syr2k2, dim3(nbk, nj), dim3(256), 0, st, A22, lda, m, Vt, ws.Wt, cmin, cmax);
    } else if (g_syr2k_tri == 1) {
      const int ntri = nbk * (nbk + 1) / 2;
      hipLaunchKernelGGL(k_sb_syr2k, dim3(ntri), dim3(256), 0, st, A22, lda, m, Vt, ws.Wt, cmin, cmax, ntri);
    } else {
      hipLaunchKernelGGL(k_sb_syr2k, dim3(nbk, cmax <= kB ? 1 : nbk), dim3(256), 0, st, A22, lda, m, Vt, ws.Wt,
                         cmin, cmax, 0);
    }
  };
  int rc = 0, p = 0;
  const int last = n - kB - 1;  // panels at i < last
  if (last > 0) rc = factor(0, 0, st);
  for (int i = 0; i < last && rc == 0; i += kB, ++p) {
    const int m = n - i - kB, par = p & 1;
    const int k = std::min(m, kB);
    const double* T = ws.T + (size_t)p * kB * kB;
    const double* Vw = ws.Vw2[par];
    const double* Vt = ws.Vt2[par];
    const int nbk = (m + kT - 1) / kT, ng = (m + kVtyRows - 1) / kVtyRows, nch = (nbk + kSymmCh - 1) / kSymmCh;
    if (p > 0 && hipStreamWaitEvent(st, evP, 0) != hipSuccess) rc = -1;
    double* A22 = A + (size_t)(i + kB) * lda + i + kB;
    // Y = A22 Vw T; W = Y - Vw (T^T (Vw^T Y)) / 2; A22 -= Vw W^T + W Vw^T
    hipLaunchKernelGGL(k_sb_symm, dim3(nbk, nch), dim3(256), 0, st, A22, lda, m, Vt, ws.Yp);
    hipLaunchKernelGGL(k_sb_ysum, dim3((unsigned)(((size_t)m * kB + 255) / 256)), dim3(256), 0, st, ws.Y, ws.Yp, nch, m);
    hipLaunchKernelGGL(k_sb_yt2, dim3((m + 7) / 8), dim3(256), 0, st, ws.Y, ws.Yp, m, k, T);
    hipLaunchKernelGGL(k_sb_vty, dim3(ng), dim3(256), 0, st, Vw, ws.Yp, m, ws.part2);
    hipLaunchKernelGGL(k_sb_gm, dim3(1), dim3(kB * kB), 0, st, ws.part2, ng, k, T, ws.Gm);
    hipLaunchKernelGGL(k_sb_w, dim3((m + 63) / 64), dim3(256), 0, st, ws.Yp, Vw, m, k, ws.Gm, ws.Wt);
    if (i + kB < last) {
      launch_syr2k(A22, m, Vt, 0, kB);
      if (hipEventRecord(evS, st) != hipSuccess || hipStreamWaitEvent(s2, evS, 0) != hipSuccess) rc = -1;
      if (rc == 0) rc = factor(i + kB, p + 1, s2);
      if (rc == 0 && hipEventRecord(evP, s2) != hipSuccess) rc = -1;
      launch_syr2k(A22, m, Vt, kB, m);
    } else {
      launch_syr2k(A22, m, Vt, 0, m);
    }
  }
  if (hipGetLastError() != hipSuccess && rc == 0) rc = -1;
  (void)hipStreamSynchronize(s2);
  (void)hipEventDestroy(evS);
  (void)hipEventDestroy(evP);
  (void)hipStreamDestroy(s2);
  return rc;
}

int sb2st_lower(hipStream_t st, int n, const double* A, int lda, double* d, double* e, void* work, int n_cu,
                int spin, long long* dbg) {
  Eig2Ws ws = carve2(work, n);
  std::vector<long long> goff;
  const size_t nrefl = chase_refl_doubles(n, &goff);
  if (hipMemcpyAsync(ws.goff, goff.data(), goff.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
  if (hipMemsetAsync(ws.refl, 0, nrefl * 8, st) != hipSuccess) return -1;
  if (hipMemsetAsync(ws.prog, 0, (size_t)n * 4, st) != hipSuccess) return -1;
  hipLaunchKernelGGL(k_sb_band, dim3((unsigned)(((size_t)n * kLD + 255) / 256)), dim3(256), 0, st, A, lda, n, ws.S);
  // ~n / (3 b) sweeps run at once: one worker per 2 b columns, at most one workgroup per CU
  const int nwg = std::max(1, std::min(n_cu, (n + 2 * kB * kChaseWG - 1) / (2 * kB * kChaseWG)));
#ifdef DSE_EIG2_VARIANTS
  if (dbg)
    hipLaunchKernelGGL(k_sb2st<true>, dim3(nwg), dim3(64 * kChaseWG), 0, st, ws.S, n, ws.refl, ws.goff, ws.prog, dbg);
  else if (g_chase_variant == 0)
    hipLaunchKernelGGL(k_sb2st<false>, dim3(nwg), dim3(64 * kChaseWG), 0, st, ws.S, n, ws.refl, ws.goff, ws.prog, dbg);
  else
#else
  (void)dbg;
#endif
  {
    const int MT = chase_tasks(n, 0) + 1;
    if (hipMemsetAsync(ws.mb, 0xff, (size_t)n * MT * 8, st) != hipSuccess) return -1;
    if (g_chase_variant == 2)
      hipLaunchKernelGGL(k_sb2st_pf<true>, dim3(nwg), dim3(64 * kChaseWG), 0, st, ws.S, n, ws.refl, ws.goff, ws.prog, ws.mb,
                         MT, ws.err, spin);
    else
      hipLaunchKernelGGL(k_sb2st_pf<false>, dim3(nwg), dim3(64 * kChaseWG), 0, st, ws.S, n, ws.refl, ws.goff, ws.prog, ws.mb,
                         MT, ws.err, spin);
  }
  hipLaunchKernelGGL(k_sb_tridiag, dim3((n + 255) / 256), dim3(256), 0, st, ws.S, n, d, e);
  if (hipStreamSynchronize(st) != hipSuccess) return -1;  // goff is host memory until here
  if (hipGetLastError() != hipSuccess) return -1;
  int herr = 0;  // a bounded poll of the panel QR or of the chase gave up: the band / tridiagonal is void
  if (hipMemcpy(&herr, ws.err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return herr ? kEig2PollTimeout : 0;
}

int q2_apply(hipStream_t st, int n, double* Z, int ldz, void* work) {
#ifndef DSE_EIG2_VARIANTS
  static_assert(g_q2_variant == 5, "libdse.so: k_sb_q2<1, false, false, true, 8> only");
#endif
  Eig2Ws ws = carve2(work, n);
  const dim3 tg((n + 63) / 64, (n + 63) / 64);
  const size_t nrec = chase_refl_doubles(n) / kRec;
  hipLaunchKernelGGL(k_sb_q2c, dim3((unsigned)((nrec + 255) / 256)), dim3(256), 0, st, ws.refl, nrec);
  hipLaunchKernelGGL(k_sb_transpose, tg, dim3(256), 0, st, Z, ldz, ws.Zt, n, n);
  const dim3 g1((n + 63) / 64);
#ifndef DSE_EIG2_VARIANTS
  hipLaunchKernelGGL((k_sb_q2<1, false, false, true, 8>), g1, dim3(512), 0, st, ws.Zt, n, n, ws.refl, ws.goff);
#else
  const dim3 blk(64 * kQ2Waves);
  switch (g_q2_variant) {
    case 1: hipLaunchKernelGGL((k_sb_q2<1, true, true, false, 4>), g1, blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 2: hipLaunchKernelGGL((k_sb_q2<2, false, false, false, 4>), dim3((n + 127) / 128), blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 3: hipLaunchKernelGGL((k_sb_q2<1, false, true, false, 4>), g1, blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 4: hipLaunchKernelGGL((k_sb_q2<1, false, false, true, 4>), g1, blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 5: hipLaunchKernelGGL((k_sb_q2<1, false, false, true, 8>), g1, dim3(512), 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 6: hipLaunchKernelGGL((k_sb_q2<1, false, false, false, 8, true>), g1, dim3(512), 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 7: hipLaunchKernelGGL((k_sb_q2<1, false, false, false, 4, true>), g1, blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 8: hipLaunchKernelGGL((k_sb_q2<1, true, false, true, 8>), g1, dim3(512), 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    case 9: hipLaunchKernelGGL((k_sb_q2<1, false, false, true, 8, false, true>), g1, dim3(512), 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
    default: hipLaunchKernelGGL((k_sb_q2<1, false, false, false, 4>), g1, blk, 0, st, ws.Zt, n, n, ws.refl, ws.goff); break;
  }
#endif
  // back: Z(r, c) = Zt[r n + c], i.e. the column-major read of Zt^T
  hipLaunchKernelGGL(k_sb_transpose, tg, dim3(256), 0, st, ws.Zt, n, Z, ldz, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int eig2_q1(rocblas_handle h, hipStream_t st, int n, const double* A, int lda, double* Z, int ldz, void* work) {
  Eig2Ws ws = carve2(work, n);
  return ormtr_lower(h, st, n, A, lda, ws.tau1, Z, ldz, ws.orm, kB);
}

int eig_sym_2stage(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* lam, double* V, int ldv,
                   double* e, void* work, int* info, int n_cu, int spin) {
  int rc = sy2sb_lower(h, st, n, A, lda, work, spin);
  if (rc) return rc;
  if ((rc = sb2st_lower(st, n, A, lda, lam, e, work, n_cu, spin, nullptr))) return rc;
  if (rocsolver_dstedc(h, rocblas_evect_tridiagonal, n, lam, e, V, ldv, info) != rocblas_status_success) return -8;
  if ((rc = q2_apply(st, n, V, ldv, work))) return rc;
  return eig2_q1(h, st, n, A, lda, V, ldv, work);
}

}  // namespace dse
