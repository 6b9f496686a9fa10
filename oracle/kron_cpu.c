/*
 * CPU ORACLE (test infrastructure / CPU baseline only -- never linked into the
 * product).  A C restatement of the loop nest pyccel would emit for
 * `kron_dot_pyccel_2d` (pyccel/pyccel_functions.py:4-21), generalised to the
 * 3D Kronecker-sum operator of the -Δu+u problem, plus the damped-Jacobi sweep
 * (sources/solvers.py:207-219) and the vector algebra of sources/solvers.py.
 *
 * Same padded layout as the device path (spl StencilVector._data): local
 * extent n_d plus p ghost cells per side per axis, C order, zero ghosts.
 * Pass structure follows the reference kernel: pass 1 along the LAST axis
 * over every leading row INCLUDING ghost rows (:12-15), then the middle axis,
 * then the first axis over owned rows only (:17-19).  OpenMP over the
 * outermost loop of each pass; temporaries are caller-allocated (as X_tmp).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX3(i0, i1, i2, s0, s1) ((int64_t)(i0) * (s0) + (int64_t)(i1) * (s1) + (int64_t)(i2))

/* ---- 2D: literal pyccel kernel (pyccel/pyccel_functions.py:4-21) ---------- */
void oracle_kron_dot_pyccel_2d(const int64_t* starts, const int64_t* ends, const int64_t* pads,
                               const double* X, double* X_tmp, double* Y,
                               const double* A, const double* B) {
    const int64_t s1 = starts[0], s2 = starts[1], e1 = ends[0], e2 = ends[1];
    const int64_t p1 = pads[0], p2 = pads[1];
    const int64_t ld = (e2 - s2 + 1) + 2 * p2;   /* padded row length */
    const int64_t wb = 2 * p2 + 1, wa = 2 * p1 + 1;
#pragma omp parallel for schedule(static)
    for (int64_t j1 = s1 - p1; j1 <= e1 + p1; ++j1)
        for (int64_t i2 = s2; i2 <= e2; ++i2) {
            double acc = 0.0;
            for (int64_t k = 0; k < wb; ++k)
                acc += X[(j1 + p1 - s1) * ld + (i2 - s2 + k)] * B[i2 * wb + k];
            X_tmp[(j1 + p1 - s1) * ld + (i2 - s2 + p2)] = acc;
        }
#pragma omp parallel for schedule(static)
    for (int64_t i1 = s1; i1 <= e1; ++i1)
        for (int64_t i2 = s2; i2 <= e2; ++i2) {
            double acc = 0.0;
            for (int64_t k = 0; k < wa; ++k)
                acc += A[i1 * wa + k] * X_tmp[(i1 - s1 + k) * ld + (i2 - s2 + p2)];
            Y[(i1 - s1 + p1) * ld + (i2 - s2 + p2)] = acc;
        }
}

/*
 * 3D Kronecker-sum operator  y = A0 (x) M1 (x) M2 x + M0 (x) (K1 (x) M2 + M1 (x) K2) x
 * (A0 = c M0 + K0), all factors square banded of width W = 2p+1, global = local.
 * mode 0: y = A x; mode 1: y = b - A x; mode 2: y = x + omega (b - A x) / diag,
 * returns sum(dr^2) for mode 2.
 * Work arrays: ta, tb of (n0+2p)*(n1+2p)*n2 doubles; tc, td of (n0+2p)*n1*n2.
 */
/* b0: half-width of the axis-0 bands actually used (p for 3D; 0 when a 2D
 * operator runs as one axis-0 plane with scalar A0 = c, M0 = 1): passes 1 and 2
 * then skip the ghost planes no band reaches. */
double oracle_kron_sum_3d_b0(int64_t n0, int64_t n1, int64_t n2, int64_t p, int64_t b0,
                             const double* A0, const double* M0, const double* M1, const double* K1,
                             const double* M2, const double* K2, const double* x, const double* b,
                             double* y, int mode, double omega,
                             double* ta, double* tb, double* tc, double* td) {
    const int64_t W = 2 * p + 1;
    const int64_t P0 = n0 + 2 * p, P1 = n1 + 2 * p, P2 = n2 + 2 * p;
    const int64_t xs1 = P2, xs0 = P1 * P2;            /* padded x / y / b */
    const int64_t as1 = n2, as0 = P1 * n2;             /* ta, tb */
    const int64_t cs1 = n2, cs0 = n1 * n2;             /* tc, td */
    const int64_t jlo = p - b0, jhi = P0 - (p - b0); /* planes the axis-0 bands reach */
    /* pass 1: last axis, all planes and rows incl. ghosts */
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t j0 = jlo; j0 < jhi; ++j0)
        for (int64_t j1 = 0; j1 < P1; ++j1)
            for (int64_t i2 = 0; i2 < n2; ++i2) {
                double sa = 0.0, sb = 0.0;
                for (int64_t k = 0; k < W; ++k) {
                    const double v = x[IDX3(j0, j1, i2 + k, xs0, xs1)];
                    sa += M2[i2 * W + k] * v;
                    sb += K2[i2 * W + k] * v;
                }
                ta[IDX3(j0, j1, i2, as0, as1)] = sa;
                tb[IDX3(j0, j1, i2, as0, as1)] = sb;
            }
    /* pass 2: middle axis, all planes incl. ghosts, owned rows */
#pragma omp parallel for collapse(2) schedule(static)
    for (int64_t j0 = jlo; j0 < jhi; ++j0)
        for (int64_t i1 = 0; i1 < n1; ++i1)
            for (int64_t i2 = 0; i2 < n2; ++i2) {
                double sc = 0.0, sd = 0.0;
                for (int64_t k = 0; k < W; ++k) {
                    const double va = ta[IDX3(j0, i1 + k, i2, as0, as1)];
                    const double vb = tb[IDX3(j0, i1 + k, i2, as0, as1)];
                    sc += M1[i1 * W + k] * va;
                    sd += K1[i1 * W + k] * va + M1[i1 * W + k] * vb;
                }
                tc[IDX3(j0, i1, i2, cs0, cs1)] = sc;
                td[IDX3(j0, i1, i2, cs0, cs1)] = sd;
            }
    /* pass 3: first axis, owned planes */
    double nrm = 0.0;
#pragma omp parallel for collapse(2) schedule(static) reduction(+ : nrm)
    for (int64_t i0 = 0; i0 < n0; ++i0)
        for (int64_t i1 = 0; i1 < n1; ++i1)
            for (int64_t i2 = 0; i2 < n2; ++i2) {
                double s = 0.0;
                for (int64_t k = p - b0; k <= p + b0; ++k)
                    s += A0[i0 * W + k] * tc[IDX3(i0 + k, i1, i2, cs0, cs1)]
                       + M0[i0 * W + k] * td[IDX3(i0 + k, i1, i2, cs0, cs1)];
                const int64_t o = IDX3(i0 + p, i1 + p, i2 + p, xs0, xs1);
                if (mode == 0) {
                    y[o] = s;
                } else if (mode == 1) {
                    y[o] = b[o] - s;
                } else {
                    const double d = A0[i0 * W + p] * M1[i1 * W + p] * M2[i2 * W + p]
                                   + M0[i0 * W + p] * (K1[i1 * W + p] * M2[i2 * W + p]
                                                       + M1[i1 * W + p] * K2[i2 * W + p]);
                    const double dr = omega * (b[o] - s) / d;
                    y[o] = x[o] + dr;
                    nrm += dr * dr;
                }
            }
    return nrm;
}

double oracle_kron_sum_3d(int64_t n0, int64_t n1, int64_t n2, int64_t p,
                          const double* A0, const double* M0, const double* M1, const double* K1,
                          const double* M2, const double* K2, const double* x, const double* b,
                          double* y, int mode, double omega,
                          double* ta, double* tb, double* tc, double* td) {
    return oracle_kron_sum_3d_b0(n0, n1, n2, p, p, A0, M0, M1, K1, M2, K2, x, b, y, mode, omega, ta, tb, tc, td);
}

/* ---- vector algebra on the padded interior -------------------------------- */
static inline int64_t row_off(int64_t r, int64_t n1, int64_t p, int64_t s0, int64_t s1) {
    const int64_t i0 = r / n1, i1 = r % n1;
    return (i0 + p) * s0 + (i1 + p) * s1 + p;
}

/* z = a x + b y (interior of 3D padded arrays) */
void oracle_axpby_3d(int64_t n0, int64_t n1, int64_t n2, int64_t p, double a, const double* x,
                     double b, const double* y, double* z) {
    const int64_t s1 = n2 + 2 * p, s0 = (n1 + 2 * p) * s1;
#pragma omp parallel for schedule(static)
    for (int64_t r = 0; r < n0 * n1; ++r) {
        const int64_t o = row_off(r, n1, p, s0, s1);
        for (int64_t c = 0; c < n2; ++c) z[o + c] = a * x[o + c] + b * y[o + c];
    }
}

double oracle_dot_3d(int64_t n0, int64_t n1, int64_t n2, int64_t p, const double* x, const double* y) {
    const int64_t s1 = n2 + 2 * p, s0 = (n1 + 2 * p) * s1;
    double s = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (int64_t r = 0; r < n0 * n1; ++r) {
        const int64_t o = row_off(r, n1, p, s0, s1);
        for (int64_t c = 0; c < n2; ++c) s += x[o + c] * y[o + c];
    }
    return s;
}

int oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

void oracle_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}
