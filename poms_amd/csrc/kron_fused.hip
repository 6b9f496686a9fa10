// Fused, sum-factorised Kronecker(-sum) banded operator for gfx950.
//
// Computes, on a padded C-order slab (axis 2 unit-stride):
//   FORM_SUM    3D: y = A0(x)M1(x)M2 x + M0(x)(K1(x)M2 + M1(x)K2) x
//               2D: y = A1(x)M2 x + M1(x)K2 x
//   FORM_SINGLE 3D: y = F0(x)F1(x)F2 x,   2D: y = F1(x)F2 x
// with an epilogue that either stores y (APPLY), b - y (RESID) or performs a
// damped-Jacobi update x + w (b - y)/diag (JACOBI, with ||dr||^2 partials).
//
// Reference semantics: `kron_dot_pyccel_2d` (pyccel/pyccel_functions.py:4-21)
// does pass 1 along the last axis over the first-axis rows INCLUDING ghosts,
// then pass 2 along the first axis; the 3D -Δu+u operator is the Kronecker sum
// of the 1D mass/stiffness factors assembled by sources/matrix_assembler.py:173.
//
// Structure (one 256-thread workgroup = 4 wave64s):
//   * tile of T1 = 4*R rows (axis 1) x 64 columns (axis 2); lane = column,
//     wave w owns R consecutive rows; the workgroup marches along axis 0 over
//     `chunk` output planes (+2P halo planes);
//   * per input plane: the (T1+2P) x (64+2P) input tile goes global -> VGPR ->
//     LDS (the next plane's global loads are issued before this plane's math);
//     axis-2 pass from LDS (per-lane band coefficients held in VGPRs) -> LDS;
//     axis-1 pass from LDS with wave-uniform (scalar) coefficients;
//   * axis-0 pass: each input plane's axis-1 results are scattered into
//     2P+1 rotating accumulator slots held in VGPRs (static slot indices via
//     a (2P+1)-way unrolled plane loop) with wave-uniform coefficients; the
//     oldest slot completes one output plane per input plane.
// No MFMA: 49 FMA per DOF at p=3 against 16 B/DOF of HBM traffic.
#include "common.hpp"

namespace poms {

template <int P, int R, bool IS3D, int FORM, int EPI>
__global__ void __launch_bounds__(256)
kron_fused_kernel(const double* __restrict__ x, double* __restrict__ y,
                  const double* __restrict__ bvec,
                  const double* __restrict__ a0t, const double* __restrict__ b0t,
                  const double* __restrict__ a1, const double* __restrict__ b1,
                  const double* __restrict__ a2, const double* __restrict__ b2,
                  double* __restrict__ partial, const KronGeom g, const double omega) {
    constexpr int W = 2 * P + 1;
    constexpr int NW = 4;
    constexpr int T2 = 64;
    constexpr int T1 = NW * R;
    constexpr int XR = T1 + 2 * P;
    constexpr int XC = T2 + 2 * P;
    constexpr int NX = XR * XC;
    constexpr int NLD = (NX + kBlock - 1) / kBlock;
    constexpr bool SUM = (FORM == FORM_SUM);
    constexpr int NS = IS3D ? W : 1;

    __shared__ double xs[NX];
    __shared__ double as_[XR * T2];
    __shared__ double bs_[SUM ? XR * T2 : 1];
    __shared__ double red[NW];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);

    int bid = blockIdx.x;
    const int t2 = bid % g.tiles2;
    bid /= g.tiles2;
    const int t1 = bid % g.tiles1;
    const int ch = bid / g.tiles1;
    const int c0 = t2 * T2;
    const int r0 = t1 * T1;
    const int i2 = c0 + lane;
    const bool col_ok = i2 < g.n2;

    // Per-lane axis-2 band coefficients (constant for the whole march).
    double ca2[W], cb2[W];
    {
        const int ic = col_ok ? i2 : 0;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            ca2[k] = col_ok ? a2[ic * W + k] : 0.0;
            if constexpr (SUM) cb2[k] = col_ok ? b2[ic * W + k] : 0.0;
            else cb2[k] = 0.0;
        }
    }

    int z0 = 0, z1 = 1;
    if constexpr (IS3D) {
        chunk_planes(g, ch, z0, z1);
    }
    const int nplanes = IS3D ? (z1 - z0) + 2 * P : 1;

    // Per-thread tile-load offsets inside one plane (plane-invariant).
    int xoff[NLD];
    unsigned okmask = 0;
    {
        const int rows = g.n1 + 2 * g.pd1, cols = g.n2 + 2 * g.pd2;
#pragma unroll
        for (int l = 0; l < NLD; ++l) {
            const int e = tid + l * kBlock;
            const int rr = e / XC, cc = e - (e / XC) * XC;
            const int si1 = r0 + rr - P + g.pd1;
            const int si2 = c0 + cc - P + g.pd2;
            const bool ok = (e < NX) && si1 >= 0 && si1 < rows && si2 >= 0 && si2 < cols;
            xoff[l] = ok ? (int)(si1 * g.s1 + si2) : 0;
            okmask |= (ok ? 1u : 0u) << l;
        }
    }
    double xr[NLD];
    auto load_plane = [&](int jj) {
        const int sp = IS3D ? jj + g.pd0 : 0;
        const bool pl_ok = !IS3D || (sp >= 0 && sp < g.n0 + 2 * g.pd0);
        const double* base = x + (int64_t)(pl_ok ? sp : 0) * g.s0;
#pragma unroll
        for (int l = 0; l < NLD; ++l)
            xr[l] = (pl_ok && ((okmask >> l) & 1u)) ? base[xoff[l]] : 0.0;
    };
    auto store_plane = [&]() {
#pragma unroll
        for (int l = 0; l < NLD; ++l) {
            const int e = tid + l * kBlock;
            if (NX % kBlock == 0 || e < NX) xs[e] = xr[l];
        }
    };

    double acc[R][NS];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int s = 0; s < NS; ++s) acc[r][s] = 0.0;
    double nrm = 0.0;

    auto epilogue = [&](int zo, int r, double v) {
        const int i1 = r0 + wv * R + r;
        if (!(col_ok && i1 < g.n1)) return;
        const int64_t off = (int64_t)(zo + g.pd0) * g.s0 + (int64_t)(i1 + g.pd1) * g.s1 + (i2 + g.pd2);
        if constexpr (EPI == EPI_APPLY) {
            y[off] = v;
        } else if constexpr (EPI == EPI_RESID) {
            y[off] = bvec[off] - v;
        } else {
            const double d1a = a1[i1 * W + P];
            const double d2a = ca2[P];
            double diag;
            if constexpr (IS3D) {
                const int i0g = g.g0 + zo;
                const double d0a = a0t[(i0g + P) * W + P];
                if constexpr (SUM) {
                    const double d0b = b0t[(i0g + P) * W + P];
                    const double d1b = b1[i1 * W + P];
                    diag = d0a * (d1a * d2a) + d0b * (d1b * d2a + d1a * cb2[P]);
                } else {
                    diag = d0a * d1a * d2a;
                }
            } else {
                if constexpr (SUM) diag = d1a * d2a + b1[i1 * W + P] * cb2[P];
                else diag = d1a * d2a;
            }
            const double dr = omega * (bvec[off] - v) / diag;
            y[off] = x[off] + dr;
            nrm = fma(dr, dr, nrm);
        }
    };

    load_plane(IS3D ? z0 - P : 0);
    for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nplanes) {
                store_plane();
                __syncthreads();
                if (IS3D && t + 1 < nplanes) load_plane(z0 - P + t + 1);

                // ---- axis-2 pass: (T1+2P) rows x 64 columns, LDS -> LDS
#pragma unroll
                for (int it = 0; it < (XR + NW - 1) / NW; ++it) {
                    const int rr = wv + it * NW;
                    if (rr < XR) {
                        double sa = 0.0, sb = 0.0;
#pragma unroll
                        for (int k = 0; k < W; ++k) {
                            const double v = xs[rr * XC + lane + k];
                            sa = fma(ca2[k], v, sa);
                            if constexpr (SUM) sb = fma(cb2[k], v, sb);
                        }
                        as_[rr * T2 + lane] = sa;
                        if constexpr (SUM) bs_[rr * T2 + lane] = sb;
                    }
                }
                __syncthreads();

                // ---- axis-1 pass: R rows per lane, wave-uniform coefficients
                double cv[R], dv[R];
#pragma unroll
                for (int r = 0; r < R; ++r) { cv[r] = 0.0; dv[r] = 0.0; }
#pragma unroll
                for (int qq = 0; qq < R + 2 * P; ++qq) {
                    const int rr = wv * R + qq;
                    const double va = as_[rr * T2 + lane];
                    const double vb = SUM ? bs_[rr * T2 + lane] : 0.0;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int k = qq - r;
                        if (k >= 0 && k < W) {
                            const int i1 = min(r0 + wv * R + r, g.n1 - 1);
                            const double ca = a1[i1 * W + k];
                            cv[r] = fma(ca, va, cv[r]);
                            if constexpr (SUM) {
                                const double cb = b1[i1 * W + k];
                                if constexpr (IS3D) dv[r] = fma(cb, va, fma(ca, vb, dv[r]));
                                else cv[r] = fma(cb, vb, cv[r]);
                            }
                        }
                    }
                }

                if constexpr (IS3D) {
                    // ---- axis-0 pass: scatter into rotating accumulator slots
                    const int jrow = (g.g0 + z0 - P + t + P) * W;  // padded transposed-band row
#pragma unroll
                    for (int s = 0; s < W; ++s) {
                        const int slot = (q - P + s + NS) % NS;
                        const double ka = a0t[jrow + s];
#pragma unroll
                        for (int r = 0; r < R; ++r) acc[r][slot] = fma(ka, cv[r], acc[r][slot]);
                        if constexpr (SUM) {
                            const double kb = b0t[jrow + s];
#pragma unroll
                            for (int r = 0; r < R; ++r) acc[r][slot] = fma(kb, dv[r], acc[r][slot]);
                        }
                    }
                    const int done = (q + P + 1) % NS;
                    if (t >= 2 * P) {
                        const int zo = z0 - 2 * P + t;
#pragma unroll
                        for (int r = 0; r < R; ++r) epilogue(zo, r, acc[r][done]);
                    }
#pragma unroll
                    for (int r = 0; r < R; ++r) acc[r][done] = 0.0;
                } else {
#pragma unroll
                    for (int r = 0; r < R; ++r) epilogue(0, r, cv[r]);
                }
            }
        }
    }

    if constexpr (EPI == EPI_JACOBI) {
        if (partial != nullptr) {
            const double s = block_sum_256(nrm, red);
            if (tid == 0) partial[blockIdx.x] = s;
        }
    }
}

// ---------------------------------------------------------------------------
// Launch helpers
// ---------------------------------------------------------------------------

constexpr int kRowsPerWave = 4;  // R
constexpr int kTileRows = 4 * kRowsPerWave;
constexpr int kTileCols = 64;

template <int P, bool IS3D, int FORM, int EPI>
static void launch_t(const KronPtrs& p, const KronGeom& g, double omega, hipStream_t st) {
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    hipLaunchKernelGGL((kron_fused_kernel<P, kRowsPerWave, IS3D, FORM, EPI>), dim3(nblk),
                       dim3(kBlock), 0, st, p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2,
                       p.b2, p.partial, g, omega);
}

template <int P, bool IS3D, int FORM>
static int launch_e(int epi, const KronPtrs& p, const KronGeom& g, double omega, hipStream_t st) {
    switch (epi) {
        case EPI_APPLY: launch_t<P, IS3D, FORM, EPI_APPLY>(p, g, omega, st); return 0;
        case EPI_RESID: launch_t<P, IS3D, FORM, EPI_RESID>(p, g, omega, st); return 0;
        case EPI_JACOBI: launch_t<P, IS3D, FORM, EPI_JACOBI>(p, g, omega, st); return 0;
    }
    return 1;
}

template <int P>
static int launch_p(bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                    double omega, hipStream_t st) {
    if (is3d) {
        return form == FORM_SUM ? launch_e<P, true, FORM_SUM>(epi, p, g, omega, st)
                                : launch_e<P, true, FORM_SINGLE>(epi, p, g, omega, st);
    }
    return form == FORM_SUM ? launch_e<P, false, FORM_SUM>(epi, p, g, omega, st)
                            : launch_e<P, false, FORM_SINGLE>(epi, p, g, omega, st);
}

int kron_launch(int pmax, bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                double omega, hipStream_t st) {
    switch (pmax) {
        case 1: return launch_p<1>(is3d, form, epi, p, g, omega, st);
        case 2: return launch_p<2>(is3d, form, epi, p, g, omega, st);
        case 3: return launch_p<3>(is3d, form, epi, p, g, omega, st);
        case 4: return launch_p<4>(is3d, form, epi, p, g, omega, st);
        case 5: return launch_p<5>(is3d, form, epi, p, g, omega, st);
    }
    set_error("pmax must be in 1..5");
    return 1;
}

int kron_tile_rows() { return kTileRows; }
int kron_tile_cols() { return kTileCols; }

}  // namespace poms
