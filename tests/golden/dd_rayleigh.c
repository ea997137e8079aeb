/* Double-double Rayleigh quotients of the columns of a dense eigenvector matrix (fixture tooling
 * for make_golden_grid30_n14.py; build container only, never shipped or loaded on the GPU box).
 *
 *   lambda_j = (v_j^T A v_j) / (v_j^T v_j),   A = diag(d_hi + d_lo) + offdiag (CSR, fp64 entries)
 *
 * Every product is split exactly (TwoProd by fma), every sum error-free (TwoSum), so each quotient
 * carries ~1e-30 relative rounding: what is left is the eigenvector's own error, which enters
 * the Rayleigh quotient at second order.  Built by the generator as
 *     gcc -O2 -march=native -ffp-contract=off -fopenmp -shared -fPIC dd_rayleigh.c
 * (contraction OFF: a contracted hi + lo of a split product would count its rounding twice).
 * V is row-major n x n (numpy eigh output: column j = eigenvector j).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct { double hi, lo; } dd;

static inline void two_sum(double a, double b, double *s, double *e) {
    double x = a + b, bb = x - a;
    *s = x;
    *e = (a - (x - bb)) + (b - bb);
}

/* acc += a * b, exactly split */
static inline void dd_fma(double *hi, double *lo, double a, double b) {
    double p = a * b, pe = fma(a, b, -p), s, e;
    two_sum(*hi, p, &s, &e);
    *hi = s;
    *lo += e + pe;
}

static inline void dd_norm(double *hi, double *lo) {
    double s = *hi + *lo;
    *lo = *lo - (s - *hi);
    *hi = s;
}

#define CHUNK 128

void dd_rayleigh(int64_t n, const int64_t *rowptr, const int64_t *col, const double *val,
                 const double *d_hi, const double *d_lo, const double *V,
                 double *lam_hi, double *lam_lo) {
    int64_t nchunk = (n + CHUNK - 1) / CHUNK;
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t c = 0; c < nchunk; ++c) {
        int64_t j0 = c * CHUNK, nj = (n - j0 < CHUNK) ? n - j0 : CHUNK;
        double q_hi[CHUNK], q_lo[CHUNK], m_hi[CHUNK], m_lo[CHUNK], a_hi[CHUNK], a_lo[CHUNK];
        for (int j = 0; j < nj; ++j) q_hi[j] = q_lo[j] = m_hi[j] = m_lo[j] = 0.0;
        for (int64_t x = 0; x < n; ++x) {
            const double *vx = V + x * n + j0;
            for (int j = 0; j < nj; ++j) {          /* (A v)_x: exact diagonal d_hi + d_lo */
                a_hi[j] = 0.0;
                a_lo[j] = 0.0;
                dd_fma(&a_hi[j], &a_lo[j], d_hi[x], vx[j]);
                a_lo[j] += d_lo[x] * vx[j];
            }
            for (int64_t k = rowptr[x]; k < rowptr[x + 1]; ++k) {
                const double h = val[k];
                const double *vy = V + col[k] * n + j0;
                for (int j = 0; j < nj; ++j) dd_fma(&a_hi[j], &a_lo[j], h, vy[j]);
            }
            for (int j = 0; j < nj; ++j) {
                dd_norm(&a_hi[j], &a_lo[j]);
                double v = vx[j];
                dd_fma(&q_hi[j], &q_lo[j], v, a_hi[j]);   /* v_x (A v)_x */
                q_lo[j] += v * a_lo[j];
                dd_fma(&m_hi[j], &m_lo[j], v, v);         /* v_x^2 */
            }
            if ((x & 63) == 63)
                for (int j = 0; j < nj; ++j) { dd_norm(&q_hi[j], &q_lo[j]); dd_norm(&m_hi[j], &m_lo[j]); }
        }
        for (int j = 0; j < nj; ++j) {
            dd_norm(&q_hi[j], &q_lo[j]);
            dd_norm(&m_hi[j], &m_lo[j]);
            /* dd division q / m: one Newton correction of the fp64 quotient */
            double r = q_hi[j] / m_hi[j];
            double p_hi = r * m_hi[j], p_lo = fma(r, m_hi[j], -p_hi) + r * m_lo[j];
            double rem = ((q_hi[j] - p_hi) - p_lo) + q_lo[j];
            double r2 = rem / m_hi[j];
            double s = r + r2;
            lam_hi[j0 + j] = s;
            lam_lo[j0 + j] = r2 - (s - r);
        }
    }
}
