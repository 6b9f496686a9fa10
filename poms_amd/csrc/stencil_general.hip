// General stencil operator: spl `StencilMatrix.dot` with its own coefficients per
// row (`slides/content.tex:285-290`),
//     v[i] = sum_k M[i, k] u[i + k - p],   k in [0, 2p_d] per axis,
// the operator the reference assembles with `assembly_2d`
// (`sources/matrix_assembler.py:84-179`) and applies at `sources/solvers.py:85,
// 103, 109, 209`.  Variable-coefficient operators that are not Kronecker sums
//  run here.
//
// Coefficients live on the device as structure-of-arrays planes: plane k holds
// M[., k] for every owned row in dense C order, so each of the (2p+1)^d
// coefficient streams is read coalesced once (8 (2p+1)^d B/DOF: 392 B/DOF in 2D
// at p = 3) while x comes through L1/L2 (the (2p+1)^d neighbours of a row are
// shared with its neighbours).  One thread per output row, grid-stride, per-block
// partial sums for the Jacobi norm and the fused dots.
#include "common.hpp"

namespace poms {

template <int EPI>
__global__ void __launch_bounds__(256)
stencil_kernel(const StencilGeom g, const double* __restrict__ coef, const double* __restrict__ x,
               double* __restrict__ y, const double* __restrict__ b, double omega,
               double* __restrict__ partial, double* __restrict__ partial2) {
    __shared__ double red[4];
    const int64_t npl = (int64_t)g.n1 * g.n2;
    const int64_t nr1 = (int64_t)(g.z_end - g.z_begin) * npl;
    const int64_t total = nr1 + (int64_t)(g.z2_end - g.z2_begin) * npl;
    const int W = g.w0 * g.w1 * g.w2;
    const int kc = ((g.w0 / 2) * g.w1 + g.w1 / 2) * g.w2 + g.w2 / 2;   // centre offset (diagonal)
    double nrm = 0.0, dot = 0.0;
    for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
        int64_t z, rem;
        if (idx < nr1) {
            z = g.z_begin + idx / npl;
            rem = idx % npl;
        } else {
            z = g.z2_begin + (idx - nr1) / npl;
            rem = (idx - nr1) % npl;
        }
        const int64_t i1 = rem / g.n2, i2 = rem % g.n2;
        const int64_t lin = z * npl + rem;
        const int64_t xo = (z + g.pd0) * g.s0 + (i1 + g.pd1) * g.s1 + (i2 + g.pd2);
        if constexpr (EPI == EPI_DIAG) {
            const double v = omega * b[xo] / coef[kc * g.cstride + lin];
            y[xo] = v;
            nrm = fma(v, v, nrm);
            continue;
        }
        double s = 0.0;
        int k = 0;
        for (int k0 = 0; k0 < g.w0; ++k0) {
            const double* xr0 = x + xo + (int64_t)(k0 - g.p0) * g.s0;
            for (int k1 = 0; k1 < g.w1; ++k1) {
                const double* xr = xr0 + (int64_t)(k1 - g.p1) * g.s1 - g.p2;
                for (int k2 = 0; k2 < g.w2; ++k2, ++k) s = fma(coef[k * g.cstride + lin], xr[k2], s);
            }
        }
        if constexpr (EPI == EPI_APPLY) {
            y[xo] = s;
        } else if constexpr (EPI == EPI_RESID) {
            y[xo] = b[xo] - s;
        } else if constexpr (EPI == EPI_JACOBI) {
            const double bv = b[xo];
            const double dr = omega * (bv - s) / coef[kc * g.cstride + lin];
            const double xn = x[xo] + dr;
            y[xo] = xn;
            nrm = fma(dr, dr, nrm);
            dot = fma(xn, bv, dot);
        } else {   // EPI_APPLYDOT
            y[xo] = s;
            dot = fma(x[xo], s, dot);
        }
        (void)W;
    }
    if (partial) {
        const double t = block_sum_256(nrm, red);
        if (threadIdx.x == 0) partial[blockIdx.x] = t;
        __syncthreads();
    }
    if (partial2) {
        const double t = block_sum_256(dot, red);
        if (threadIdx.x == 0) partial2[blockIdx.x] = t;
    }
}

// On-device assembly of -div(a grad u) + c u (`sources/matrix_assembler.py:84-179`,
// where a = c = 1): one thread per (owned row, stencil offset), writing coefficient
// plane k of row `lin`.  The row pair (i, j) meets on the elements both supports
// share; per element the quadrature sum is formed first and then added, as the
// reference's element loop does.  a_q / c_q: coefficients at every quadrature
// point (index ((e0 nq0 + g0) NQ1 + e1 nq1 + g1) NQ2 + e2 nq2 + g2), or null for
// a = 1, c = mass_coef.
__global__ void __launch_bounds__(256)
assemble_kernel(const AssembleAxis A0, const AssembleAxis A1, const AssembleAxis A2, int g0, int nl0,
                const double* __restrict__ a_q, const double* __restrict__ c_q, double mass_coef,
                double* __restrict__ coef) {
    const int64_t cst = (int64_t)nl0 * A1.n * A2.n;
    const int W1 = 2 * A1.p + 1, W2 = 2 * A2.p + 1;
    const int64_t total = cst * (int64_t)(2 * A0.p + 1) * W1 * W2;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= total) return;
    const int64_t lin = tid % cst;
    const int k = (int)(tid / cst);
    const int k2 = k % W2, k1 = (k / W2) % W1, k0 = k / (W2 * W1);
    const int i2 = (int)(lin % A2.n), i1 = (int)((lin / A2.n) % A1.n), i0 = g0 + (int)(lin / ((int64_t)A2.n * A1.n));
    const int j0 = i0 + k0 - A0.p, j1 = i1 + k1 - A1.p, j2 = i2 + k2 - A2.p;
    double tot = 0.0;
    if (j0 >= 0 && j0 < A0.n && j1 >= 0 && j1 < A1.n && j2 >= 0 && j2 < A2.n) {
        const int ea0 = max(A0.es[i0], A0.es[j0]), eb0 = min(A0.ee[i0], A0.ee[j0]);
        const int ea1 = max(A1.es[i1], A1.es[j1]), eb1 = min(A1.ee[i1], A1.ee[j1]);
        const int ea2 = max(A2.es[i2], A2.es[j2]), eb2 = min(A2.ee[i2], A2.ee[j2]);
        const int NQ1 = A1.nel * A1.nq, NQ2 = A2.nel * A2.nq;
        for (int e0 = ea0; e0 <= eb0; ++e0) {
            const int li0 = i0 - A0.first[e0], lj0 = j0 - A0.first[e0];
            for (int e1 = ea1; e1 <= eb1; ++e1) {
                const int li1 = i1 - A1.first[e1], lj1 = j1 - A1.first[e1];
                for (int e2 = ea2; e2 <= eb2; ++e2) {
                    const int li2 = i2 - A2.first[e2], lj2 = j2 - A2.first[e2];
                    double v = 0.0;
                    for (int q0 = 0; q0 < A0.nq; ++q0) {
                        const double* B0 = A0.basis + (int64_t)(e0 * A0.nq + q0) * (A0.p + 1) * 2;
                        const double w0 = A0.w[e0 * A0.nq + q0];
                        const double bi0 = B0[2 * li0], di0 = B0[2 * li0 + 1];
                        const double bj0 = B0[2 * lj0], dj0 = B0[2 * lj0 + 1];
                        for (int q1 = 0; q1 < A1.nq; ++q1) {
                            const double* B1 = A1.basis + (int64_t)(e1 * A1.nq + q1) * (A1.p + 1) * 2;
                            const double w1 = A1.w[e1 * A1.nq + q1];
                            const double bi1 = B1[2 * li1], di1 = B1[2 * li1 + 1];
                            const double bj1 = B1[2 * lj1], dj1 = B1[2 * lj1 + 1];
                            for (int q2 = 0; q2 < A2.nq; ++q2) {
                                const double* B2 = A2.basis + (int64_t)(e2 * A2.nq + q2) * (A2.p + 1) * 2;
                                const double w2 = A2.w[e2 * A2.nq + q2];
                                const double bi2 = B2[2 * li2], di2 = B2[2 * li2 + 1];
                                const double bj2 = B2[2 * lj2], dj2 = B2[2 * lj2 + 1];
                                // bi_0 bj_0 + bi_x bj_x + bi_y bj_y (+ bi_z bj_z), times wvol
                                const double i_0 = bi0 * (bi1 * bi2), j_0 = bj0 * (bj1 * bj2);
                                const double gx = (di0 * (bi1 * bi2)) * (dj0 * (bj1 * bj2));
                                const double gy = (bi0 * (di1 * bi2)) * (bj0 * (dj1 * bj2));
                                const double gz = (bi0 * (bi1 * di2)) * (bj0 * (bj1 * dj2));
                                const int64_t qi = ((int64_t)(e0 * A0.nq + q0) * NQ1 + (e1 * A1.nq + q1)) * NQ2 +
                                                   (e2 * A2.nq + q2);
                                const double ca = a_q ? a_q[qi] : 1.0;
                                const double cc = c_q ? c_q[qi] : mass_coef;
                                v = fma(cc * i_0 * j_0 + ca * (gx + gy + gz), w0 * (w1 * w2), v);
                            }
                        }
                    }
                    tot += v;
                }
            }
        }
    }
    coef[k * cst + lin] = tot;
}

int assemble_launch(const AssembleAxis* ax, int g0, int nl0, const double* a_q, const double* c_q, double mass_coef,
                    double* coef, hipStream_t st) {
    const int64_t total = (int64_t)nl0 * ax[1].n * ax[2].n * (2 * ax[0].p + 1) * (2 * ax[1].p + 1) * (2 * ax[2].p + 1);
    if (total == 0) return 0;
    hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, ax[0], ax[1], ax[2],
                       g0, nl0, a_q, c_q, mass_coef, coef);
    return 0;
}

// Coefficient planes -> the spl StencilMatrix._data layout (padded rows, offsets last).
__global__ void __launch_bounds__(256)
stencil_to_spl_kernel(const StencilGeom g, const double* __restrict__ coef, double* __restrict__ out) {
    const int W = g.w0 * g.w1 * g.w2;
    const int64_t total = g.cstride * W;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= total) return;
    const int64_t lin = tid / W;
    const int k = (int)(tid % W);
    const int64_t i2 = lin % g.n2, i1 = (lin / g.n2) % g.n1, i0 = lin / ((int64_t)g.n2 * g.n1);
    const int64_t P1 = g.n1 + 2 * g.p1, P2 = g.n2 + 2 * g.p2;
    const int64_t row = ((i0 + g.p0) * P1 + (i1 + g.p1)) * P2 + (i2 + g.p2);
    out[row * W + k] = coef[k * g.cstride + lin];
}

int stencil_to_spl_launch(const StencilGeom& g, const double* coef, double* out, hipStream_t st) {
    const int64_t total = g.cstride * g.w0 * g.w1 * g.w2;
    if (total == 0) return 0;
    hipLaunchKernelGGL(stencil_to_spl_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, g, coef, out);
    return 0;
}

// Blocks of the grid-stride launch (<= max_blocks so the partials fit the scratch).
int stencil_launch(int epi, const StencilGeom& g, const double* coef, const double* x, double* y,
                   const double* b, double omega, double* partial, double* partial2, int max_blocks,
                   hipStream_t st, int* nblk_out) {
    const int64_t total = (int64_t)((g.z_end - g.z_begin) + (g.z2_end - g.z2_begin)) * g.n1 * g.n2;
    const int64_t want = (total + 255) / 256;
    const int nb = (int)std::min<int64_t>(std::max<int64_t>(want, 1), max_blocks);
    *nblk_out = total > 0 ? nb : 0;
    if (total == 0) return 0;
    switch (epi) {
        case EPI_APPLY:
            hipLaunchKernelGGL(stencil_kernel<EPI_APPLY>, dim3(nb), dim3(256), 0, st, g, coef, x, y, b, omega,
                               partial, partial2);
            break;
        case EPI_RESID:
            hipLaunchKernelGGL(stencil_kernel<EPI_RESID>, dim3(nb), dim3(256), 0, st, g, coef, x, y, b, omega,
                               partial, partial2);
            break;
        case EPI_JACOBI:
            hipLaunchKernelGGL(stencil_kernel<EPI_JACOBI>, dim3(nb), dim3(256), 0, st, g, coef, x, y, b, omega,
                               partial, partial2);
            break;
        case EPI_APPLYDOT:
            hipLaunchKernelGGL(stencil_kernel<EPI_APPLYDOT>, dim3(nb), dim3(256), 0, st, g, coef, x, y, b, omega,
                               partial, partial2);
            break;
        case EPI_DIAG:
            hipLaunchKernelGGL(stencil_kernel<EPI_DIAG>, dim3(nb), dim3(256), 0, st, g, coef, x, y, b, omega,
                               partial, partial2);
            break;
        default:
            set_error("general stencil: unsupported epilogue");
            return 1;
    }
    return 0;
}

}  // namespace poms
