// Knot-insertion restriction / prolongation as a sequence of 1D Kronecker
// axis passes (R = P^T with P = P0 (x) P1 (x) P2, sources/mg_jac.py:67-70).
//
// restrict pass:  out[a][J][b] = sum_i P[goff+i][J] * in[a][i][b]
// prolong  pass:  out[a][i][b] (+)= sum_J P[goff+i][J] * in[a][J][b]
//
// One thread per independent (a, b1, b2) line; the thread marches along the
// contracted axis with the NCM coarse values / accumulators in registers and
// wave-uniform (scalar) rows of P (P is stored fine-row-major, padded to NCM
// columns with zeros).  The dominant pass (axis 0 of the fine slab) streams the
// fine vector once: 8 B/DOF for restriction, 16 B/DOF for prolong-add.
// Coarse extents > 32 (multilevel hierarchies) use the banded gather kernels.
#include "common.hpp"

#include <algorithm>

namespace poms {

// Few lines (a 2D grid's passes: ~10^3 lines of ~10^3 points, or the coarse
// axis' ~10 lines) leave the one-thread-per-line march latency-bound: the
// contracted axis is then split in KS chunks (blockIdx.y), each thread writing its
// NCM partial sums to `part`, and restrict_sum_kernel adds the KS partials of each
// output in chunk order (deterministic).
template <int NCM>
__global__ void __launch_bounds__(256)
restrict_pass_kernel(const AxisPass ps, const double* __restrict__ Pm,
                     const double* __restrict__ in, double* __restrict__ out, double* __restrict__ part) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    if (tid >= nline) return;
    const int ks = gridDim.y, kc = (ps.nI + ks - 1) / ks;
    const int i_begin = blockIdx.y * kc, i_end = min(ps.nI, i_begin + kc);
    const int64_t b2 = tid % ps.nB2;
    const int64_t t1 = tid / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double acc[NCM];
#pragma unroll
    for (int j = 0; j < NCM; ++j) acc[j] = 0.0;
    for (int i = i_begin; i < i_end; ++i) {
        const double v = src[(int64_t)i * ps.in_si];
        const double* prow = Pm + (int64_t)(ps.goff + i) * NCM;
#pragma unroll
        for (int j = 0; j < NCM; ++j) acc[j] = fma(prow[j], v, acc[j]);
    }
    if (ks > 1) {   // partials [chunk][j][line]: coalesced over lines
#pragma unroll
        for (int j = 0; j < NCM; ++j)
            if (j < ps.nJ) part[((int64_t)blockIdx.y * NCM + j) * nline + tid] = acc[j];
        return;
    }
    double* dst = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2;
#pragma unroll
    for (int j = 0; j < NCM; ++j)
        if (j < ps.nJ) dst[(int64_t)j * ps.out_si] = acc[j];
}

__global__ void __launch_bounds__(256)
restrict_sum_kernel(const AxisPass ps, int ncm, int ks, const double* __restrict__ part, double* __restrict__ out) {
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= nline * ps.nJ) return;
    const int j = (int)(tid / nline);
    const int64_t line = tid - (int64_t)j * nline;
    double s = 0.0;
    for (int k = 0; k < ks; ++k) s += part[((int64_t)k * ncm + j) * nline + line];
    const int64_t b2 = line % ps.nB2;
    const int64_t t1 = line / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    out[ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)j * ps.out_si] = s;
}

template <int NCM>
__global__ void __launch_bounds__(256)
prolong_pass_kernel(const AxisPass ps, const double* __restrict__ Pm,
                    const double* __restrict__ in, double* __restrict__ out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    if (tid >= nline) return;
    const int64_t b2 = tid % ps.nB2;
    const int64_t t1 = tid / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double cv[NCM];
#pragma unroll
    for (int j = 0; j < NCM; ++j) cv[j] = (j < ps.nJ) ? src[(int64_t)j * ps.in_si] : 0.0;
    double* dst = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2;
    // outputs are independent: few lines split the expanded axis over blockIdx.y
    const int ks = gridDim.y, kc = (ps.nI + ks - 1) / ks;
    const int i_end = min(ps.nI, (int)blockIdx.y * kc + kc);
    for (int i = blockIdx.y * kc; i < i_end; ++i) {
        const double* prow = Pm + (int64_t)(ps.goff + i) * NCM;
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < NCM; ++j) s = fma(prow[j], cv[j], s);
        double* o = dst + (int64_t)i * ps.out_si;
        if (ps.accumulate) *o += s;
        else *o = s;
    }
}

// Banded gather form for large coarse extents (multilevel hierarchies, where P
// is the dyadic knot-insertion matrix with a few non-zeros per row / column):
// one thread per OUTPUT element, the fastest index (b2) on consecutive lanes.
//   restrict: out[a][J][b] = sum_k Rb[J][k] in[a][ilo[J] + k - goff][b]  (local rows only)
//   prolong : out[a][i][b] (+)= sum_k Pb[goff+i][k] in[a][jlo[goff+i] + k][b]
__global__ void __launch_bounds__(256)
restrict_band_kernel(const AxisPass ps, const double* __restrict__ Rb, const int* __restrict__ ilo, int wR,
                     const double* __restrict__ in, double* __restrict__ out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nout = ps.nA * ps.nJ * ps.nB1 * ps.nB2;
    if (tid >= nout) return;
    const int64_t b2 = tid % ps.nB2;
    int64_t t = tid / ps.nB2;
    const int64_t b1 = t % ps.nB1;
    t /= ps.nB1;
    const int J = (int)(t % ps.nJ);
    const int64_t a = t / ps.nJ;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double s = 0.0;
    const int i0 = ilo[J] - ps.goff;
    for (int k = 0; k < wR; ++k) {
        const int i = i0 + k;
        if (i >= 0 && i < ps.nI) s = fma(Rb[(int64_t)J * wR + k], src[(int64_t)i * ps.in_si], s);
    }
    out[ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)J * ps.out_si] = s;
}

__global__ void __launch_bounds__(256)
prolong_band_kernel(const AxisPass ps, const double* __restrict__ Pb, const int* __restrict__ jlo, int wP,
                    const double* __restrict__ in, double* __restrict__ out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nout = ps.nA * (int64_t)ps.nI * ps.nB1 * ps.nB2;
    if (tid >= nout) return;
    const int64_t b2 = tid % ps.nB2;
    int64_t t = tid / ps.nB2;
    const int64_t b1 = t % ps.nB1;
    t /= ps.nB1;
    const int i = (int)(t % ps.nI);
    const int64_t a = t / ps.nI;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    const int gi = ps.goff + i;
    const int j0 = jlo[gi];
    double s = 0.0;
    for (int k = 0; k < wP; ++k) {
        const int j = j0 + k;
        if (j < ps.nJ) s = fma(Pb[(int64_t)gi * wP + k], src[(int64_t)j * ps.in_si], s);
    }
    double* o = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)i * ps.out_si;
    if (ps.accumulate) *o += s;
    else *o = s;
}

int transfer_band_launch(bool restrict_dir, const AxisPass& ps, const double* band, const int* lo, int w,
                         const double* in, double* out, hipStream_t st) {
    const int64_t nout = ps.nA * (int64_t)(restrict_dir ? ps.nJ : ps.nI) * ps.nB1 * ps.nB2;
    const int64_t nb = (nout + 255) / 256;
    if (nb == 0) return 0;
    if (restrict_dir)
        hipLaunchKernelGGL(restrict_band_kernel, dim3((unsigned)nb), dim3(256), 0, st, ps, band, lo, w, in, out);
    else
        hipLaunchKernelGGL(prolong_band_kernel, dim3((unsigned)nb), dim3(256), 0, st, ps, band, lo, w, in, out);
    return 0;
}

// chunks of the contracted / expanded axis: enough threads for the GPU when the
// lines are few, chunks of at least 16 points
static int transfer_split(int64_t nline, int nI) {
    if (nline >= 32768 || nI < 64) return 1;
    const int64_t want = (65536 + nline - 1) / nline;
    return (int)std::max<int64_t>(1, std::min<int64_t>({want, (int64_t)nI / 16, 256}));
}

int transfer_split_scratch(int ncm, const AxisPass& ps) {   // doubles of partials a restrict pass needs
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int ks = transfer_split(nline, ps.nI);
    return ks > 1 ? (int)(ks * (int64_t)ncm * nline) : 0;
}

int transfer_pass_launch(bool restrict_dir, int ncm, const AxisPass& ps, const double* Pm,
                         const double* in, double* out, hipStream_t st, double* part) {
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int nb = (int)((nline + 255) / 256);
    if (nb == 0) return 0;
    int ks = transfer_split(nline, ps.nI);
    if (restrict_dir && ks > 1 && part == nullptr) ks = 1;
    const dim3 grid(nb, ks);
    if (ncm == 16) {
        if (restrict_dir)
            hipLaunchKernelGGL(restrict_pass_kernel<16>, grid, dim3(256), 0, st, ps, Pm, in, out, part);
        else
            hipLaunchKernelGGL(prolong_pass_kernel<16>, grid, dim3(256), 0, st, ps, Pm, in, out);
    } else if (ncm == 32) {
        if (restrict_dir)
            hipLaunchKernelGGL(restrict_pass_kernel<32>, grid, dim3(256), 0, st, ps, Pm, in, out, part);
        else
            hipLaunchKernelGGL(prolong_pass_kernel<32>, grid, dim3(256), 0, st, ps, Pm, in, out);
    } else {
        set_error("transfer: coarse extent must be <= 32");
        return 1;
    }
    if (restrict_dir && ks > 1) {
        const int64_t nsum = nline * ps.nJ;
        hipLaunchKernelGGL(restrict_sum_kernel, dim3((unsigned)((nsum + 255) / 256)), dim3(256), 0, st, ps, ncm, ks,
                           part, out);
    }
    return 0;
}

}  // namespace poms
