// dse_sytrd.hip -- symmetric eigendecomposition for the dense engine (dse_dense.h, option
// "eig_impl" = 1): a blocked Householder tridiagonalisation of the lower triangle written for
// gfx950, then rocSOLVER's tridiagonal divide and conquer (dstedc) and back-transformation
// (dormtr).
//
// Why: rocSOLVER dsyevd spends ~73% of a 2^14 solve in its tridiagonalisation (dsytrd 2.94 of
// 4.04 s, profiles/r03/eig_concurrency_16384.jsonl), most of it in one matrix-vector product per
// column against the trailing matrix, which it reads whole (latrd_lower_computeW_gemvt_kernel:
// 38.5 us per column on average at 2^13, the trailing block's full bytes at ~4.7 TB/s).  The
// product is symmetric, so reading only the tiles on and below the diagonal and using each twice
// halves those bytes.
//
// Algorithm (LAPACK dsytrd / dlatrd, lower): panels of NB columns; for column c of a panel starting
// at column i (local j = c - i; W the panel's n x NB block, row r of W at r - i; v_p = A(:, i+p)):
//   1. A(c:n, c) -= A(c:n, i:c) W(c, 0:j)^T + W(c:n, 0:j) A(c, i:c)^T          (k_trd_colupd)
//   2. reflector of A(c+1:n, c): beta, tau, v (v_0 = 1 stored in A(c+1, c))     (k_trd_larfg)
//   3. y = A(c+1:n, c+1:n) v over the lower-triangle tiles, partials per block;
//      u2 = W(c+1:n, 0:j)^T v, u3 = A(c+1:n, i:c)^T v by the diagonal tiles     (k_trd_symv)
//   4. W(c+1:n, j) = tau (y - A(c+1:n, i:c) u2 - W(c+1:n, 0:j) u3)              (k_trd_wfin)
//   5. W(:, j) += alpha_j v, alpha_j = -tau/2 W(:, j).v
// Step 5 is never a pass of its own: k_trd_wfin leaves W' = W - alpha v and per-block partial dots
// of W'.v, the next column's k_trd_colupd sums them into alpha_j, and every reader of W forms
// W' + alpha v from the W' and v entries it loads anyway (k_trd_wfix finalises the panel for the
// update).  Then A(i+NB:n, i+NB:n) -= V W^T + W V^T (rocBLAS dsyr2k); the last columns by
// rocsolver_dsytd2.  Per column: 4 launches, all reductions in fixed order (deterministic).
// d, e, tau and the reflectors below the subdiagonal follow LAPACK's layout: rocsolver_dstedc gives
// the tridiagonal eigenvectors Z, ormtr_lower (blocks of 256 reflectors) V = Q Z.
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

struct TrdWs {
  double* W;        // n x NB, ldw = n
  double* partial;  // nbk x nbk x BS: symv partials
  double* dpart;    // nbk x 2 NB: partial u2', u3
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

// 1. column update, rows r in [c, n); j > 0.  Also alpha_{j-1} (workgroup 0 stores it).
__global__ void __launch_bounds__(256)
k_trd_colupd(double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, int c, int j, const double* tau,
             int nbk_prev) {
  __shared__ double s_al[kTrdNB];
  load_alpha(ws, tau, c, j, nbk_prev, s_al);
  if (blockIdx.x == 0 && threadIdx.x == 0) ws.alpha[j - 1] = s_al[j - 1];
  const int r = c + (int)(blockIdx.x * 256 + threadIdx.x);
  if (r >= n) return;
  const double* W = ws.W;
  double s = A[(size_t)c * lda + r];
  for (int p = 0; p < j; ++p) {
    const double vr = A[(size_t)(i + p) * lda + r], vc = A[(size_t)(i + p) * lda + c];
    const double wr = fma(s_al[p], vr, W[(size_t)p * ldw + (r - i)]);
    const double wc = fma(s_al[p], vc, W[(size_t)p * ldw + (c - i)]);
    s -= vr * wc + wr * vc;
  }
  A[(size_t)c * lda + r] = s;
}

// 1 + 2 in one launch: the column update (j > 0) and the sums of squares of A(c+2:n, c) by block;
// the last workgroup to finish (agent-scope counter) forms beta, tau and the scale of the reflector,
// which k_trd_symv and k_trd_wfin apply as they read it (k_trd_wfin stores v).
__global__ void __launch_bounds__(256)
k_trd_colref(double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, int c, int j,
             double* __restrict__ d, double* __restrict__ e, double* __restrict__ tau, int nbk_prev) {
  __shared__ double s_al[kTrdNB];
  __shared__ double red[4];
  __shared__ int s_last;
  if (j > 0) {
    load_alpha(ws, tau, c, j, nbk_prev, s_al);
    if (blockIdx.x == 0 && threadIdx.x == 0) ws.alpha[j - 1] = s_al[j - 1];
  }
  const int r = c + (int)(blockIdx.x * 256 + threadIdx.x);
  double s = 0.0;
  if (r < n) {
    s = A[(size_t)c * lda + r];
    if (j > 0) {
      const double* W = ws.W;
#pragma unroll 8
      for (int p = 0; p < j; ++p) {
        const double vr = A[(size_t)(i + p) * lda + r], vc = A[(size_t)(i + p) * lda + c];
        const double wr = fma(s_al[p], vr, W[(size_t)p * ldw + (r - i)]);
        const double wc = fma(s_al[p], vc, W[(size_t)p * ldw + (c - i)]);
        s -= vr * wc + wr * vc;
      }
      A[(size_t)c * lda + r] = s;
    }
  }
  const double ss = block_sum(r >= c + 2 && r < n ? s * s : 0.0, red);
  if (threadIdx.x == 0) ws.sspart[blockIdx.x] = ss;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
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
  if (!s_last || threadIdx.x >= 64) return;
  double xn2 = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += 64) xn2 += __builtin_nontemporal_load(ws.sspart + b);
  xn2 = wave_sum0(xn2);
  if (threadIdx.x != 0) return;
  const double* col = A + (size_t)c * lda;
  const double alpha = __builtin_nontemporal_load(col + c + 1);
  double t = 0.0, beta = alpha, scale = 1.0;
  if (xn2 > 0.0) {
    beta = -std::copysign(std::sqrt(alpha * alpha + xn2), alpha);
    t = (beta - alpha) / beta;
    scale = 1.0 / (alpha - beta);
  }
  d[c] = __builtin_nontemporal_load(col + c);
  e[c] = beta;
  tau[c] = t;
  *ws.scale = scale;
  *ws.cnt = 0;
}

// 2. reflector H = I - tau v v^T with H (alpha, x)^T = (beta, 0); alpha = A(c+1, c), x = A(c+2:n, c)
__global__ void __launch_bounds__(1024)
k_trd_larfg(double* __restrict__ A, int lda, int n, int c, double* __restrict__ d, double* __restrict__ e,
            double* __restrict__ tau, double* __restrict__ ws_scale) {
  __shared__ double red[16];
  __shared__ double s_scale;
  double* col = A + (size_t)c * lda;
  double ss = 0.0;
  for (int r = c + 2 + (int)threadIdx.x; r < n; r += 1024) ss = fma(col[r], col[r], ss);
  const double xn2 = block_sum(ss, red);
  if (threadIdx.x == 0) {
    const double alpha = col[c + 1];
    double t = 0.0, beta = alpha, scale = 1.0;
    if (xn2 > 0.0) {
      beta = -std::copysign(std::sqrt(alpha * alpha + xn2), alpha);
      t = (beta - alpha) / beta;
      scale = 1.0 / (alpha - beta);
    }
    d[c] = col[c];
    e[c] = beta;
    tau[c] = t;
    col[c + 1] = 1.0;
    s_scale = scale;
  }
  __syncthreads();
  const double scale = s_scale;
  for (int r = c + 2 + (int)threadIdx.x; r < n; r += 1024) col[r] *= scale;
  if (threadIdx.x == 0) *ws_scale = 1.0;
}

// 3. y = S v for the trailing block S = A(o:o+m, o:o+m) (lower triangle valid), v = A(o:o+m, c):
// one workgroup per tile (I, J), I >= J, of 64 x 64; wave w takes columns 16 w .. 16 w + 15, lane l
// row l.  Direct part -> partial[I][J], transposed part (I > J) -> partial[J][I]; the diagonal
// tile's two halves are summed in the workgroup.  Transposed column sums by a butterfly reduce-
// scatter over the wave (as k_symv).  The diagonal tiles also leave the block's share of the
// dot products u2' = W'^T v and u3 = V^T v (panel columns 0 .. j) in dpart[I].
__global__ void __launch_bounds__(256)
k_trd_symv(const double* __restrict__ A, int lda, TrdWs ws, int ldw, int i, int j, int o, int m, int c, int nbk) {
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
  const double* col = A + (size_t)c * lda;
  if (tid < BS) {
    const double scale = *ws.scale;
    const int cj = J * BS + tid, ri = I * BS + tid;
    vs[0][tid] = cj < m ? refl_v(col, o + cj, c, scale) : 0.0;
    vs[1][tid] = ri < m ? refl_v(col, o + ri, c, scale) : 0.0;
  }
  __syncthreads();
  const int row = I * BS + lane;
  const bool rv = row < m;
  const bool diag = I == J;
  const double vi = vs[1][lane];
  const double* base = A + (size_t)(o + J * BS) * lda + o + I * BS + lane;
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
  if (diag && j > 0) {
    // wave w: dots q = 16 w .. 16 w + 15 (q < j: W', else V), loads first, then two reduce-scatters
    const int r = o + row;  // global row
    double x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int q = w * 16 + k;
      x[k] = (!rv || q >= 2 * j) ? 0.0
             : q < j             ? ws.W[(size_t)q * ldw + (r - i)]
                                 : A[(size_t)(i + q - j) * lda + r];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      double p[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) p[q] = x[8 * h + q] * vi;
      const double s = reduce_scatter8(p, b5, b4, b3);
      const int q = w * 16 + 8 * h + 4 * b5 + 2 * b4 + b3;
      if ((lane & 7) == 0 && q < 2 * j) ws.dpart[(size_t)I * 2 * kTrdNB + q] = s;
    }
  }
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
// blockIdx.x; y from the symv partials, u2 = u2' + alpha u3 from the diagonal tiles' partials.
// Leaves the block's W'(:, j).v in apart[B].  512 threads: 8 waves split the partials and the panel.
__global__ void __launch_bounds__(512)
k_trd_wfin(double* __restrict__ A, int lda, TrdWs ws, int ldw, int n, int i, int c, int j, int nbk,
           const double* __restrict__ tau) {
  constexpr int BS = kTrdBS;
  __shared__ double su[2 * kTrdNB];
  __shared__ double s_al[kTrdNB];
  __shared__ double red[8][BS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (j > 0) {
    const int q = tid >> 3, sub = tid & 7;
    double s = 0.0;
    if (q < 2 * j)
#pragma unroll 8
      for (int k = sub; k < nbk; k += 8) s += ws.dpart[(size_t)k * 2 * kTrdNB + q];
    s += __shfl_xor(s, 4, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 1, 64);
    if (sub == 0 && q < 2 * j) su[q] = s;
    if (tid < j) s_al[tid] = ws.alpha[tid];
    __syncthreads();
    if (tid < j) su[tid] = fma(s_al[tid], su[j + tid], su[tid]);
    __syncthreads();
  }
  const int o = c + 1;
  const int B = blockIdx.x;
  const int r = o + B * BS + lane;
  const bool live = r < n;
  double y = 0.0;
  if (live) {
    const double* pp = ws.partial + (size_t)B * nbk * BS + lane;
    int k = w;
    for (; k + 24 < nbk; k += 32) {
      const double p0 = pp[(size_t)k * BS], p1 = pp[(size_t)(k + 8) * BS], p2 = pp[(size_t)(k + 16) * BS],
                   p3 = pp[(size_t)(k + 24) * BS];
      y += p0;
      y += p1;
      y += p2;
      y += p3;
    }
    for (; k < nbk; k += 8) y += pp[(size_t)k * BS];
#pragma unroll 4
    for (int p = w; p < j; p += 8) {
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
    for (int q = 1; q < 8; ++q) s += red[q][tid];
    const double wv = tau[c] * s;
    double prod = 0.0;
    if (live) {
      ws.W[(size_t)j * ldw + (r - i)] = wv;
      double* col = A + (size_t)c * lda;
      const double v = refl_v(col, r, c, *ws.scale);
      col[r] = v;
      prod = wv * v;
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
// Blocks of kOrmKB reflectors from the last to the first, each applied as I - Vb T Vb^T in the
// "UT" form T = S^{-1}, S = diag(1 / tau) + striu(Vb^T Vb): Wt = Vb^T Z_b (GEMM), Wt = S^{-1} Wt
// (TRSM), Z_b -= Vb Wt (GEMM), where Z_b = the rows i+1 .. n-1 the block acts on.  A block of 256
// reflectors reads Z_b three times (rocSOLVER dormtr's blocks of 32: ~24 passes over the same
// rows; measured 769 ms at 2^14, 11 TF/s).  A reflector with tau = 0 (H = I: its column was zero
// already) gets a zero column in Vb and 1 on S's diagonal, so it changes nothing.
constexpr int kOrmKB = 256;
constexpr int kHalfTrdMinDim = 8192;

// Vb (m_b x k, column-major): unit lower trapezoid of the reflectors i .. i+k-1 (rows i+1 .. n-1)
__global__ void __launch_bounds__(256)
k_orm_vb(const double* __restrict__ A, int lda, const double* __restrict__ tau, int i, int k, int m_b,
         double* __restrict__ Vb) {
  const int r = (int)(blockIdx.x * 256 + threadIdx.x), q = (int)blockIdx.y;
  if (r >= m_b) return;
  double v = 0.0;
  if (tau[i + q] != 0.0) v = r > q ? A[(size_t)(i + q) * lda + (i + 1 + r)] : r == q ? 1.0 : 0.0;
  Vb[(size_t)q * m_b + r] = v;
}

__global__ void k_orm_sdiag(double* __restrict__ S, int k, const double* __restrict__ tau, int i) {
  const int q = (int)threadIdx.x + (int)blockIdx.x * 256;
  if (q >= k) return;
  const double t = tau[i + q];
  S[(size_t)q * k + q] = t != 0.0 ? 1.0 / t : 1.0;
}

TrdWs carve(double* work, int n) {
  const size_t nbk = ((size_t)n + kTrdBS - 1) / kTrdBS;
  TrdWs ws;
  ws.W = work;
  ws.partial = ws.W + (size_t)n * kTrdNB;
  ws.dpart = ws.partial + nbk * nbk * kTrdBS;
  ws.apart = ws.dpart + nbk * 2 * kTrdNB;
  ws.alpha = ws.apart + nbk;
  ws.sspart = ws.alpha + kTrdNB;
  ws.scale = ws.sspart + (n + 255) / 256;
  ws.cnt = reinterpret_cast<int*>(ws.scale + 1);
  return ws;
}

}  // namespace

size_t sytrd_workspace(int n) {
  const size_t nbk = ((size_t)n + kTrdBS - 1) / kTrdBS;
  const size_t trd =
      (size_t)n * kTrdNB + nbk * nbk * kTrdBS + nbk * 2 * kTrdNB + nbk + kTrdNB + ((size_t)n + 255) / 256 + 2;
  const size_t orm = 2 * (size_t)n * kOrmKB + (size_t)kOrmKB * kOrmKB;  // Vb, Wt, S
  return std::max(trd, orm) * sizeof(double);
}

int ormtr_lower(rocblas_handle h, hipStream_t st, int n, const double* A, int lda, const double* tau, double* Z,
                int ldz, double* work) {
  const int nref = n - 1;
  if (nref <= 0) return 0;
  double* Vb = work;
  double* Wt = Vb + (size_t)n * kOrmKB;
  double* S = Wt + (size_t)n * kOrmKB;
  const double one = 1.0, zero = 0.0, minus_one = -1.0;
  const int nblk = (nref + kOrmKB - 1) / kOrmKB;
  for (int b = nblk - 1; b >= 0; --b) {
    const int i = b * kOrmKB, k = std::min(kOrmKB, nref - i), m_b = n - i - 1;
    hipLaunchKernelGGL(k_orm_vb, dim3((m_b + 255) / 256, k), dim3(256), 0, st, A, lda, tau, i, k, m_b, Vb);
    if (hipGetLastError() != hipSuccess) return -6;
    if (rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, k, k, m_b, &one, Vb, m_b, Vb, m_b, &zero,
                      S, k) != rocblas_status_success)
      return -7;
    hipLaunchKernelGGL(k_orm_sdiag, dim3((k + 255) / 256), dim3(256), 0, st, S, k, tau, i);
    if (rocblas_dgemm(h, rocblas_operation_transpose, rocblas_operation_none, k, n, m_b, &one, Vb, m_b, Z + i + 1, ldz,
                      &zero, Wt, k) != rocblas_status_success)
      return -7;
    if (rocblas_dtrsm(h, rocblas_side_left, rocblas_fill_upper, rocblas_operation_none, rocblas_diagonal_non_unit, k,
                      n, &one, S, k, Wt, k) != rocblas_status_success)
      return -8;
    if (rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, m_b, n, k, &minus_one, Vb, m_b, Wt, k, &one,
                      Z + i + 1, ldz) != rocblas_status_success)
      return -7;
  }
  return hipGetLastError() == hipSuccess ? 0 : -6;
}

int sytrd_lower(rocblas_handle h, hipStream_t st, int n, double* A, int lda, double* d, double* e, double* tau,
                double* work, int fused) {
  const TrdWs ws = carve(work, n);
  const int ldw = n;
  if (hipMemsetAsync(ws.cnt, 0, sizeof(int), st) != hipSuccess) return -1;
  int i = 0;
  for (; n - i > kTrdRem + kTrdNB; i += kTrdNB) {
    int nbk_prev = 0;
    for (int j = 0; j < kTrdNB; ++j) {
      const int c = i + j;
      if (fused) {
        hipLaunchKernelGGL(k_trd_colref, dim3((n - c + 255) / 256), dim3(256), 0, st, A, lda, ws, ldw, n, i, c, j, d,
                           e, tau, nbk_prev);
      } else {
        if (j > 0)
          hipLaunchKernelGGL(k_trd_colupd, dim3((n - c + 255) / 256), dim3(256), 0, st, A, lda, ws, ldw, n, i, c, j,
                             tau, nbk_prev);
        hipLaunchKernelGGL(k_trd_larfg, dim3(1), dim3(1024), 0, st, A, lda, n, c, d, e, tau, ws.scale);
      }
      const int o = c + 1, m = n - o;
      const int nbk = (m + kTrdBS - 1) / kTrdBS;
      hipLaunchKernelGGL(k_trd_symv, dim3(nbk * (nbk + 1) / 2), dim3(256), 0, st, A, lda, ws, ldw, i, j, o, m, c,
                         nbk);
      hipLaunchKernelGGL(k_trd_wfin, dim3(nbk), dim3(512), 0, st, A, lda, ws, ldw, n, i, c, j, nbk, tau);
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
  // outweighs the halved reads: 101 vs 112 ms at 2^12, profiles/r03/sytrd_probe.jsonl); the
  // fused column kernel pays its cross-XCD release only where the columns are long
  if (n >= kHalfTrdMinDim) {
    const int rc = sytrd_lower(h, st, n, A, lda, lam, e, tau, work, n >= 16384 ? 1 : 0);
    if (rc) return rc;
  } else if (rocsolver_dsytrd(h, rocblas_fill_lower, n, A, lda, lam, e, tau) != rocblas_status_success) {
    return -3;
  }
  if (rocsolver_dstedc(h, rocblas_evect_tridiagonal, n, lam, e, V, ldv, info) != rocblas_status_success) return -4;
  return ormtr_lower(h, st, n, A, lda, tau, V, ldv, work);
}

}  // namespace dse
