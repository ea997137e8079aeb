// dse_sytrd.hip -- symmetric eigendecomposition for the dense engine (dse_dense.h, option
// "eig_impl" = 1): a blocked Householder tridiagonalisation of the lower triangle written for
// gfx950, rocSOLVER's tridiagonal divide and conquer (dstedc) and a blocked back-transformation.
//
// Why: rocSOLVER dsyevd spends ~73% of a 2^14 solve in its tridiagonalisation (dsytrd 2.94 of
// 4.04 s, profiles/r03/eig_concurrency_16384.jsonl), most of it in one matrix-vector product per
// column against the trailing matrix, which it reads whole (latrd_lower_computeW_gemvt_kernel:
// 152 us per column on average at 2^14, the trailing block's full bytes at ~4.7 TB/s).  The
// product is symmetric, so reading only the tiles on and below the diagonal and using each twice
// halves those bytes.
//
// Algorithm (LAPACK dsytrd / dlatrd, lower): panels of NB columns; for column c of a panel starting
// at column i (local j = c - i; W the panel's n x NB block, row r of W at r - i; v_p = A(:, i+p)):
//   1. A(c:n, c) -= A(c:n, i:c) W(c, 0:j)^T + W(c:n, 0:j) A(c, i:c)^T
//   2. reflector of A(c+1:n, c): beta, tau, v (v_0 = 1 at A(c+1, c)); u2' = W'(c+1:n, 0:j)^T v,
//      u3 = A(c+1:n, i:c)^T v                                                     (k_trd_colref)
//   3. y = A(c+1:n, c+1:n) v over the lower-triangle tiles, partials per block  (k_trd_symv)
//   4. W(c+1:n, j) = tau (y - A(c+1:n, i:c) u2 - W(c+1:n, 0:j) u3)              (k_trd_wfin)
//   5. W(:, j) += alpha_j v, alpha_j = -tau/2 W(:, j).v
// k_trd_colref's workgroups each update 256 rows of the column and leave their rows' share of
// ||x||^2 and of the dot products of x with the panel's W' and V columns; the last workgroup to
// finish (agent-scope counter) forms beta, tau, the reflector's scale and u2', u3 (v = scale x
// below its leading 1, so the dots are the scaled sums plus the leading row).  The scale is applied
// lazily: k_trd_symv scales v as it loads it, k_trd_wfin stores it.  Step 5 is never a pass of its
// own: k_trd_wfin leaves W' = W - alpha v and per-block partial dots of W'.v, the next column's
// k_trd_colref sums them into alpha_j, and every reader of W forms W' + alpha v from the W' and v
// entries it loads anyway (k_trd_wfix finalises the panel for the update).  Then A(i+NB:n,
// i+NB:n) -= V W^T + W V^T (rocBLAS dsyr2k); the last columns by rocsolver_dsytd2.  Three launches
// per column, every reduction in fixed order (deterministic).  d, e, tau and the reflectors below
// the subdiagonal follow LAPACK's layout: rocsolver_dstedc gives the tridiagonal eigenvectors Z,
// ormtr_lower (blocks of 256 reflectors) V = Q Z.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "dse_dense.h"

namespace dse {
namespace {

constexpr int kTrdNB = 32;   // panel width
constexpr int kTrdBS = 64;   // symv tile, rows per k_trd_wfin workgroup
constexpr int kTrdRem = 64;  // columns left to rocsolver_dsytd2
constexpr int kTrdRows = 256;  // rows per k_trd_colref workgroup

struct TrdWs {
  double* W;        // n x NB, ldw = n
  double* partial;  // nbk x nbk x BS: symv partials
  double* upart;    // ceil(n / 256) x 2 NB: k_trd_colref's partial x.W'(:, p) (slots < NB), x.v_p (>= NB)
  double* u;        // 2 NB: u2' (slots < NB), u3 (slots >= NB) of the current column
  double* apart;    // nbk: partial W'(:, j).v
  double* alpha;    // NB
  double* sspart;   // ceil(n / 256): k_trd_colref's partial sums of squares
  double* scale;    // 1: the reflector's 1 / (alpha - beta) until k_trd_wfin applies it (1 when applied)
  int* cnt;         // 1: k_trd_colref's workgroups done (zero between launches)
};

// v(r) of the current reflector: A(c+1, c) stands for 1, the rows below are scaled lazily
__device__ __forceinline__ double refl_v(const double* col, int r, int c, double scale) {
  return r == c + 1 ? 1.0 : scale * col[r];
}

// wave sum in fixed order, lane 0's value
__device__ __forceinline__ double wave_sum0(double v) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return __shfl(v, 0, 64);
}

// the wave sums of 8 values per lane: xor 32 / 16 / 8 halve the set, xor 4 / 2 / 1 finish it; the
// lanes of an aligned group of 8 hold the sum of p[4 b5 + 2 b4 + b3] (b = lane bits 5, 4, 3)
__device__ __forceinline__ double reduce_scatter8(const double (&p)[8], int b5, int b4, int b3) {
  double k4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) k4[q] = (b5 ? p[4 + q] : p[q]) + __shfl_xor(b5 ? p[q] : p[4 + q], 32, 64);
  double k2[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) k2[q] = (b4 ? k4[2 + q] : k4[q]) + __shfl_xor(b4 ? k4[q] : k4[2 + q], 16, 64);
  double s = (b3 ? k2[1] : k2[0]) + __shfl_xor(b3 ? k2[0] : k2[1], 8, 64);
#pragma unroll
  for (int of = 4; of > 0; of >>= 1) s += __shfl_xor(s, of, 64);
  return s;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum0(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int q = 0; q < nw; ++q) s += red[q];
  return s;
}

// alpha_{j-1} from k_trd_wfin's partials (every workgroup the same sum), alpha_p for p < j - 1
// from memory, into s_al[0 .. j)
__device__ __forceinline__ void load_alpha(const TrdWs& ws, const double* tau, int c, int j, int nbk_prev,
                                           double* s_al) {
  if (threadIdx.x < 64) {
    double s = 0.0;
    for (int k = threadIdx.x; k < nbk_prev; k += 64) s += ws.apart[k];
    s = wave_sum0(s);
    if (threadIdx.x == 0) s_al[j - 1] = -0.5 * tau[c - 1] * s;
  } else if (threadIdx.x - 64 < j - 1) {
    s_al[threadIdx.x - 64] = ws.alpha[threadIdx.x - 64];
  }
  __syncthreads();
}

// 1 + 2: the column update (j > 0), and per workgroup of 256 rows the sum of squares of x =
// A(c+2:n, c) and the dots x.W'(:, p), x.v_p; the last workgroup forms the reflector and u2', u3.
__global__ void __launch_bounds__(kTrdRows)
k_trd_colref(double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, int c, int j,
             double* __restrict__ d, double* __restrict__ e, double* __restrict__ tau, int nbk_prev) {
  __shared__ double s_al[kTrdNB];
  __shared__ double s_vc[kTrdNB], s_wc[kTrdNB];  // row c of the panel: A(c, i+p), W(c-i, p) final
  __shared__ double red[4];
  __shared__ double ured[4][2 * kTrdNB];
  __shared__ int s_last;
  const int tid = (int)threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = c + (int)blockIdx.x * kTrdRows + tid;
  const double* W = ws.W;
  double s = r < n ? A[(size_t)c * lda + r] : 0.0;
  if (j > 0) {
    // alpha (wave 0 sums, threads 64.. load), row c of V and W' (threads 128.., 192..)
    const int tq = tid - 128, tw = tid - 192;
    if (tq >= 0 && tq < j) s_vc[tq] = A[(size_t)(i + tq) * lda + c];
    if (tw >= 0 && tw < j) s_wc[tw] = W[(size_t)tw * ldw + (c - i)];
    // all of the row's panel loads at once, in flight under the alpha prologue (p >= j: column i
    // again, dropped by the selects)
    double vr[kTrdNB], wr[kTrdNB];
#pragma unroll
    for (int p = 0; p < kTrdNB; ++p) {
      const int pp = p < j ? p : 0;
      vr[p] = r < n ? A[(size_t)(i + pp) * lda + r] : 0.0;
      wr[p] = r < n ? W[(size_t)pp * ldw + (r - i)] : 0.0;
    }
    load_alpha(ws, tau, c, j, nbk_prev, s_al);
    if (tid < j) s_wc[tid] = fma(s_al[tid], s_vc[tid], s_wc[tid]);
    if (blockIdx.x == 0 && tid == 0) ws.alpha[j - 1] = s_al[j - 1];
    __syncthreads();
#pragma unroll
    for (int p = 0; p < kTrdNB; ++p) {
      const int pp = p < j ? p : 0;
      const double wf = fma(s_al[pp], vr[p], wr[p]);
      const double dd = vr[p] * s_wc[pp] + wf * s_vc[pp];
      s -= p < j ? dd : 0.0;
    }
    if (r < n) A[(size_t)c * lda + r] = s;
    // this workgroup's x.W'(:, p) and x.v_p (rows c+2 and below), slots p and NB + p
    const double x = r >= c + 2 && r < n ? s : 0.0;
    const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1, b3 = (lane >> 3) & 1;
#pragma unroll
    for (int g = 0; g < 2 * kTrdNB / 8; ++g) {
      if (8 * (g % (kTrdNB / 8)) >= j) continue;  // slots of panel columns not yet reduced
      double pv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int slot = 8 * g + q;
        const int p = slot < kTrdNB ? slot : slot - kTrdNB;
        pv[q] = p < j ? x * (slot < kTrdNB ? wr[p] : vr[p]) : 0.0;
      }
      const double t = reduce_scatter8(pv, b5, b4, b3);
      if ((lane & 7) == 0) ured[w][8 * g + 4 * b5 + 2 * b4 + b3] = t;
    }
  }
  const double ss = block_sum(r >= c + 2 && r < n ? s * s : 0.0, red);  // (its barriers order ured)
  if (tid == 0) ws.sspart[blockIdx.x] = ss;
  if (j > 0 && tid < 2 * kTrdNB)
    ws.upart[(size_t)blockIdx.x * 2 * kTrdNB + tid] = ured[0][tid] + ured[1][tid] + ured[2][tid] + ured[3][tid];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int last = __hip_atomic_fetch_add(ws.cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  // the last workgroup: its four waves sum the dot products' partials (slot = lane, a quarter of
  // the workgroups each), wave 0 forms beta, tau, scale (every lane the same) and u2', u3
  const int G = (int)gridDim.x;
  const double* col = A + (size_t)c * lda;
  const int p = lane < kTrdNB ? lane : lane - kTrdNB;
  // wave 0's own operands first, in flight under the partial sums
  double xn2 = 0.0, alpha = 0.0, dcc = 0.0, lead = 0.0;
  if (w == 0) {
    for (int b = lane; b < G; b += 64) xn2 += __builtin_nontemporal_load(ws.sspart + b);
    alpha = __builtin_nontemporal_load(col + c + 1);
    dcc = __builtin_nontemporal_load(col + c);
    if (p < j) lead = lane < kTrdNB ? W[(size_t)p * ldw + (c + 1 - i)] : A[(size_t)(i + p) * lda + c + 1];
  }
  if (j > 0) {
    double us = 0.0;
    for (int b0 = w; b0 < G; b0 += 4 * 16) {
      double xs[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int b = b0 + 4 * q;
        xs[q] = b < G ? __builtin_nontemporal_load(ws.upart + (size_t)b * 2 * kTrdNB + lane) : 0.0;
      }
#pragma unroll
      for (int q = 0; q < 16; ++q) us += xs[q];
    }
    ured[w][lane] = us;
  }
  __syncthreads();
  if (tid >= 64) return;
  xn2 = wave_sum0(xn2);
  double t = 0.0, beta = alpha, scale = 1.0;
  if (xn2 > 0.0) {
    beta = -std::copysign(std::sqrt(alpha * alpha + xn2), alpha);
    t = (beta - alpha) / beta;
    scale = 1.0 / (alpha - beta);
  }
  // lane = slot: u2'[p] = scale sum x.W'(:, p) + W'(c+1-i, p), u3[p] = scale sum x.v_p + A(c+1, i+p)
  if (p < j) {
    const double us = ured[0][lane] + ured[1][lane] + ured[2][lane] + ured[3][lane];
    ws.u[lane] = fma(scale, us, lead);
  }
  if (lane == 0) {
    d[c] = dcc;
    e[c] = beta;
    tau[c] = t;
    *ws.scale = scale;
    *ws.cnt = 0;
  }
}

// 3. y = S v for the trailing block S = A(o:o+m, o:o+m) (lower triangle valid), v = A(o:o+m, c):
// one workgroup per tile (I, J), I >= J, of 64 x 64; wave w takes columns 16 w .. 16 w + 15, lane l
// row l.  Direct part -> partial[I][J], transposed part (I > J) -> partial[J][I]; the diagonal
// tile's two halves are summed in the workgroup.  Transposed column sums by a butterfly reduce-
// scatter over the wave (as k_symv).
__global__ void __launch_bounds__(256)
k_trd_symv(const double* __restrict__ A, int lda, TrdWs ws, int o, int m, int c, int nbk) {
  constexpr int BS = kTrdBS, CW = BS / 4;
  // blockIdx.x -> (I, J), J <= I, row-major over the lower triangle
  const int t = (int)blockIdx.x;
  int I = (int)((std::sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
  while ((I + 1) * (I + 2) / 2 <= t) ++I;
  while (I * (I + 1) / 2 > t) --I;
  const int J = t - I * (I + 1) / 2;
  __shared__ double vs[2][BS];  // v_J (columns), v_I (rows)
  __shared__ double red[4][BS];
  __shared__ double tr[BS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int row = I * BS + lane;
  const bool rv = row < m;
  const bool diag = I == J;
  const double* base = A + (size_t)(o + J * BS) * lda + o + I * BS + lane;
  const double* col = A + (size_t)c * lda;
  if (tid < BS) {
    const double scale = *ws.scale;
    const int cj = J * BS + tid, ri = I * BS + tid;
    vs[0][tid] = cj < m ? refl_v(col, o + cj, c, scale) : 0.0;
    vs[1][tid] = ri < m ? refl_v(col, o + ri, c, scale) : 0.0;
  }
  __syncthreads();
  const double vi = vs[1][lane];
  double a = 0.0;
  const int b5 = (lane >> 5) & 1, b4 = (lane >> 4) & 1, b3 = (lane >> 3) & 1;
#pragma unroll 1
  for (int c0 = 0; c0 < CW; c0 += 8) {
    double u[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cc = w * CW + c0 + q;
      u[q] = (rv && J * BS + cc < m) ? base[(size_t)cc * lda] : 0.0;
    }
    double p[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int cc = w * CW + c0 + q;
      const double ud = (!diag || lane >= cc) ? u[q] : 0.0;  // lower triangle of a diagonal tile
      const double ut = (!diag || lane > cc) ? u[q] : 0.0;
      a = fma(ud, vs[0][cc], a);
      p[q] = ut * vi;
    }
    const double s = reduce_scatter8(p, b5, b4, b3);
    if ((lane & 7) == 0) tr[w * CW + c0 + 4 * b5 + 2 * b4 + b3] = s;
  }
  red[w][lane] = a;
  __syncthreads();
  if (tid < BS) {
    double s = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    double* partial = ws.partial;
    if (diag) {
      s += tr[tid];
      partial[((size_t)I * nbk + I) * BS + tid] = s;
    } else {
      partial[((size_t)I * nbk + J) * BS + tid] = s;
      partial[((size_t)J * nbk + I) * BS + tid] = tr[tid];
    }
  }
}

// 4. W'(r - i, j) = tau (y(r) - sum_p A(r, i+p) u2[p] + W(r - i, p) u3[p]), rows of block B =
// blockIdx.x; y from the symv partials, u2 = u2' + alpha u3.  Leaves the block's W'(:, j).v in
// apart[B].  1024 threads: 16 waves split the partials (16 loads per lane in flight at 2^14) and
// the panel.
__global__ void __launch_bounds__(1024)
k_trd_wfin(double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, int c, int j, int nbk,
           const double* __restrict__ tau) {
  constexpr int BS = kTrdBS, NW = 16;
  __shared__ double su[2 * kTrdNB];
  __shared__ double s_al[kTrdNB];
  __shared__ double red[NW][BS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int o = c + 1;
  const int B = blockIdx.x;
  const int r = o + B * BS + lane;
  const bool live = r < n;
  double* col = A + (size_t)c * lda;
  // the epilogue's operands, early
  double t_c = 0.0, vr_c = 0.0;
  if (tid < BS) {
    t_c = tau[c];
    vr_c = live ? refl_v(col, r, c, *ws.scale) : 0.0;
  }
  if (j > 0) {
    if (tid < j) {
      const double al = ws.alpha[tid], u3 = ws.u[kTrdNB + tid];
      s_al[tid] = al;
      su[tid] = fma(al, u3, ws.u[tid]);
      su[j + tid] = u3;
    }
    __syncthreads();
  }
  double y = 0.0;
  if (live) {
    const double* pp = ws.partial + (size_t)B * nbk * BS + lane;
    for (int k0 = 0; k0 < nbk; k0 += NW * 16) {
      double x[16];
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int k = k0 + w + NW * t;
        x[t] = k < nbk ? pp[(size_t)k * BS] : 0.0;
      }
#pragma unroll
      for (int t = 0; t < 16; ++t) y += x[t];
    }
#pragma unroll 2
    for (int p = w; p < j; p += NW) {
      const double vr = A[(size_t)(i + p) * lda + r];
      const double wr = fma(s_al[p], vr, ws.W[(size_t)p * ldw + (r - i)]);
      y -= vr * su[p] + wr * su[j + p];
    }
  }
  red[w][lane] = y;
  __syncthreads();
  if (tid < BS) {
    double s = red[0][tid];
#pragma unroll
    for (int q = 1; q < NW; ++q) s += red[q][tid];
    const double wv = t_c * s;
    double prod = 0.0;
    if (live) {
      ws.W[(size_t)j * ldw + (r - i)] = wv;
      col[r] = vr_c;
      prod = wv * vr_c;
    }
    prod = wave_sum0(prod);
    if (tid == 0) ws.apart[B] = prod;
  }
}

// W(r - i, p) += alpha_p A(r, i + p) for rows r >= i + NB (the rows dsyr2k reads), all p < NB
__global__ void __launch_bounds__(256)
k_trd_wfix(const double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, const double* tau, int nbk_prev) {
  __shared__ double s_al[kTrdNB];
  load_alpha(ws, tau, i + kTrdNB, kTrdNB, nbk_prev, s_al);
  const int r = i + kTrdNB + (int)(blockIdx.x * 256 + threadIdx.x);
  if (r >= n) return;
#pragma unroll 4
  for (int p = 0; p < kTrdNB; ++p) {
    double* wp = ws.W + (size_t)p * ldw + (r - i);
    *wp = fma(s_al[p], A[(size_t)(i + p) * lda + r], *wp);
  }
}

// ---- back-transformation V = Q Z, Q = H(0) H(1) ... H(n-2) (LAPACK dormtr, left, lower) ----
// Blocks of orm_kb(n) reflectors from the last to the first, each applied as I - Vb T Vb^T in the
// "UT" form T = S^{-1}, S = diag(1 / tau) + striu(Vb^T Vb): Wt = Vb^T Z_b (GEMM), Wt = S^{-1} Wt
// (TRSM), Z_b -= Vb Wt (GEMM), where Z_b = the rows i+1 .. n-1 the block acts on.  A block of k
// reflectors reads Z_b three times (rocSOLVER dormtr's blocks of 32: ~24 passes over the same
// rows; measured 769 ms at 2^14, 11 TF/s).  A reflector with tau = 0 (H = I: its column was zero
// already) gets a zero column in Vb and 1 on S's diagonal, so it changes nothing.  Block size
// (round 4, probe_eig2's Q1 at 2^14 / 2^13, profiles/r04/orm_block_ab.txt): 256 -> 235 / -, 512 ->
// 204, 1024 -> 169 / 24, 2048 -> 160 / 28, 4096 -> 190 / 38 ms.
#ifndef DSE_ORM_KB
#define DSE_ORM_KB 0
#endif
inline int orm_kb(int n) { return DSE_ORM_KB > 0 ? DSE_ORM_KB : n >= 16384 ? 2048 : 1024; }
constexpr int kHalfTrdMinDim = 8192;

// Vb (m_b x k, column-major): unit lower trapezoid of the reflectors i .. i+k-1 (reflector q of
// column i + q starts at row i + q + off: rows i + off .. n-1)
__global__ void __launch_bounds__(256)
k_orm_vb(const double* __restrict__ A, int lda, const double* __restrict__ tau, int i, int k, int m_b, int off,
         double* __restrict__ Vb) {
  const int r = (int)(blockIdx.x * 256 + threadIdx.x), q = (int)blockIdx.y;
  if (r >= m_b) return;
  double v = 0.0;
  if (tau[i + q] != 0.0) v = r > q ? A[(size_t)(i + q) * lda + (i + off + r)] : r == q ? 1.0 : 0.0;
  Vb[(size_t)q * m_b + r] = v;
}

__global__ void k_orm_sdiag(double* __restrict__ S, int k, const double* __restrict__ tau, int i) {
  const int q = (int)threadIdx.x + (int)blockIdx.x * 256;
  if (q >= k) return;
  const double t = tau[i + q];
  S[(size_t)q * k + q] = t != 0.0 ? 1.0 / t : 1.0;
}

TrdWs carve(double* work, int n) {
  const size_t nbk = ((size_t)n + kTrdBS - 1) / kTrdBS, ng = ((size_t)n + kTrdRows - 1) / kTrdRows;
  TrdWs ws;
  ws.W = work;
  ws.partial = ws.W + (size_t)n * kTrdNB;
  ws.upart = ws.partial + nbk * nbk * kTrdBS;
  ws.u = ws.upart + ng * 2 * kTrdNB;
  ws.apart = ws.u + 2 * kTrdNB;
  ws.alpha = ws.apart + nbk;
  ws.sspart = ws.alpha + kTrdNB;
  ws.scale = ws.sspart + ng;
  ws.cnt = reinterpret_cast<int*>(ws.scale + 1);
  return ws;
}

}  // namespace

size_t sytrd_workspace(int n) {
  const size_t nbk = ((size_t)n + kTrdBS - 1) / kTrdBS, ng = ((size_t)n + kTrdRows - 1) / kTrdRows;
  const size_t trd = (size_t)n * kTrdNB + nbk * nbk * kTrdBS + ng * 2 * kTrdNB + 2 * kTrdNB + nbk + kTrdNB + ng + 2;
  const size_t kb = (size_t)orm_kb(n);
  const size_t orm = 2 * (size_t)n * kb + kb * kb;  // Vb, Wt, S
  return std::max(trd, orm) * sizeof(double);
}

int ormtr_lower(rocblas_handle h, hipStream_t st, int n, const double* A, int lda, const double* tau, double* Z,
                int ldz, double* work, int off) {
  const int nref = n - off;
  if (nref <= 0) return 0;
  const int kOrmKB = orm_kb(n);
  double* Vb = work;
  double* Wt = Vb + (size_t)n * kOrmKB;
  double* S = Wt + (size_t)n * kOrmKB;
  const double one = 1.0, zero = 0.0, minus_one = -1.0;
  const int nblk = (nref + kOrmKB - 1) / kOrmKB;
  for (int b = nblk - 1; b >= 0; --b) {
    const int i = b * kOrmKB, k = std::min(kOrmKB, nref - i), m_b = n - i - off;
    hipLaunchKernelGGL(k_orm_vb, dim3((m_b + 255) / 256, k), dim3(256), 0, st, A, lda, tau, i, k, m_b, off, Vb);
    if (hipGetLastError() != hipSuccess) return -6;
    if (rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, k, k, m_b, &one, Vb, m_b, Vb, m_b, &zero,
                      S, k) != rocblas_status_success)
      return -7;
    hipLaunchKernelGGL(k_orm_sdiag, dim3((k + 255) / 256), dim3(256), 0, st, S, k, tau, i);
    if (rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, k, n, m_b, &one, Vb, m_b, Z + i + off,
                      ldz, &zero, Wt, k) != rocblas_status_success)
      return -7;
    if (rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_upper, rocblas_operation_none, rocblas_diagonal_non_unit, k,
                      n, &one, S, k, Wt, k) != rocblas_status_success)
      return -8;
    if (rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, m_b, n, k, &minus_one, Vb, m_b, Wt, k, &one,
                      Z + i + off, ldz) != rocblas_status_success)
      return -7;
  }
  return hipGetLastError() == hipSuccess ? 0 : -6;
}

int sytrd_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* d, double* e, double* tau,
                double* work) {
  const TrdWs ws = carve(work, n);
  const int ldw = n;
  if (hipMemsetAsync(ws.cnt, 0, sizeof(int), st) != hipSuccess) return -1;
  int i = 0;
  for (; n - i > kTrdRem + kTrdNB; i += kTrdNB) {
    int nbk_prev = 0;
    for (int j = 0; j < kTrdNB; ++j) {
      const int c = i + j;
      hipLaunchKernelGGL(k_trd_colref, dim3((n - c + kTrdRows - 1) / kTrdRows), dim3(kTrdRows), 0, st, A, lda, ws,
                         ldw, n, i, c, j, d, e, tau, nbk_prev);
      const int o = c + 1, m = n - o;
      const int nbk = (m + kTrdBS - 1) / kTrdBS;
      hipLaunchKernelGGL(k_trd_symv, dim3(nbk * (nbk + 1) / 2), dim3(256), 0, st, A, lda, ws, o, m, c, nbk);
      hipLaunchKernelGGL(k_trd_wfin, dim3(nbk), dim3(1024), 0, st, A, lda, ws, ldw, n, i, c, j, nbk, tau);
      nbk_prev = nbk;
    }
    const int nt = n - i - kTrdNB;
    hipLaunchKernelGGL(k_trd_wfix, dim3((nt + 255) / 256), dim3(256), 0, st, A, lda, ws, ldw, n, i, tau, nbk_prev);
    if (hipGetLastError() != hipSuccess) return -1;
    // A(i+NB:n, i+NB:n) -= V W^T + W V^T
    const double minus_one = -1.0, one = 1.0;
    if (rocblas_dsyr2k(h, rocblas_fill_lower, rocblas_operation_none, nt, kTrdNB, &minus_one,
                       A + (size_t)i * lda + i + kTrdNB, lda, ws.W + kTrdNB, ldw, &one,
                       A + (size_t)(i + kTrdNB) * lda + i + kTrdNB, lda) != rocblas_status_success)
      return -2;
  }
  // the last columns unblocked
  if (rocsolver_dsytd2(h, rocblas_fill_lower, n - i, A + (size_t)i * lda + i, lda, d + i, e + i, tau + i) !=
      rocblas_status_success)
    return -3;
  return 0;
}

int eig_sym_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* lam, double* V, int ldv,
                  double* e, double* tau, double* work, int* info) {
  // below 2^13 rocSOLVER's tridiagonalisation is the faster one (per-column launch latency
  // outweighs the halved reads: 101 vs 112 ms at 2^12, profiles/r03/sytrd_probe.jsonl)
  if (n >= kHalfTrdMinDim) {
    const int rc = sytrd_lower(h, st, n, A, lda, lam, e, tau, work);
    if (rc) return rc;
  } else if (rocsolver_dsytrd(h, rocblas_fill_lower, n, A, lda, lam, e, tau) != rocblas_status_success) {
    return -3;
  }
  if (rocsolver_dstedc(h, rocblas_evect_tridiagonal, n, lam, e, V, ldv, info) != rocblas_status_success) return -4;
  return ormtr_lower(h, st, n, A, lda, tau, V, ldv, work);
}

}  // namespace dse
