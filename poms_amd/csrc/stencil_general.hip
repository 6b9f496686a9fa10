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
