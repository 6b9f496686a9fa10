// Kronecker direct solve  X = (A0^-1 (x) A1^-1 (x) A2^-1) Y  by banded LU line
// solves along each axis: the GLT post-smoother's preconditioner
// (`kron_solve_par` / `kron_solve_par_bnd_pyccel_2d|3d`,
// `sources/kron_product.py:93-238`, `pyccel/pyccel_functions.py:114-248`).
//
// Host: each 1D band matrix is factorised once with partial pivoting, the
// LAPACK dgbtf2 algorithm that scipy's dgbtrf runs for kl < 32 (restated in
// `band_lu` below).  Device: every line of an axis is one independent
// dgbtrs: forward sweep (row interchanges + unit-lower L, column form) then
// backward sweep (non-unit upper U with kl+ku super-diagonals, column form as
// dtbsv), each a sliding window of <= MW+1 pending values in registers.  The
// interchanges and coefficients are the same for every line, so all branches
// and coefficient loads are wave-uniform (scalar).
//
// Two kernels, both HBM-bound (32 B/DOF per axis: read b, write y, read y,
// write x):
//  * ksolve_strided_kernel: lines along a strided axis (axis 0 / axis 1, or the
//    transposed axis-0 buffer of a distributed solve); one thread per line, the
//    unit-stride index on consecutive lanes, 8 loads in flight per thread.
//  * ksolve_rows_kernel: lines along the unit-stride axis 2; each wave owns 64
//    rows, stages 16-column chunks through LDS with coalesced 128-B row
//    segments, and each lane then marches its own row through the chunk.  The
//    forward and backward sweeps are separate launches (the backward re-reads
//    the forward's output written by other lanes).
#include "common.hpp"

#include <algorithm>
#include <cmath>
#include <vector>

namespace poms {

// window shift: w[0..S-1] <- w[1..S], w[S] <- v   (S <= MW, wave-uniform)
template <int MW>
__device__ __forceinline__ void feed(double (&w)[MW + 1], int S, double v) {
#pragma unroll
    for (int t = 0; t < MW; ++t)
        if (t < S) w[t] = w[t + 1];
#pragma unroll
    for (int t = 0; t <= MW; ++t)
        if (t == S) w[t] = v;
}

// dgbtrs forward step j: w[t] = b(j + t).  Interchange b(j) <-> b(ipiv(j)),
// then b(j+t) -= l(j+t, j) b(j) (the DGER of dgbtrs, column form).
// CKL / CK >= 0: kl / K known at compile time (the predicates fold away).
template <int MW, int CKL = -1>
__device__ __forceinline__ double step_fwd(double (&w)[MW + 1], const BandLU& f, int j) {
    const int kl = CKL >= 0 ? CKL : f.kl;
    const int l = f.piv[j];
    if (l != 0) {
#pragma unroll
        for (int t = 1; t <= MW; ++t)
            if (t == l) {
                const double s = w[0];
                w[0] = w[t];
                w[t] = s;
            }
    }
    const double b0 = w[0];
    const double* Lj = f.L + (int64_t)j * kl;
#pragma unroll
    for (int t = 1; t <= MW; ++t)
        if (t <= kl) w[t] = fma(-Lj[t - 1], b0, w[t]);
    return b0;
}

// dtbsv (upper, no transpose, non-unit) step j: w[t] = b(j - t).
// x(j) = b(j) / u(j,j), then b(j-t) -= x(j) u(j-t, j).
template <int MW, int CK = -1>
__device__ __forceinline__ double step_bwd(double (&w)[MW + 1], const BandLU& f, int j) {
    const int K = CK >= 0 ? CK : f.K;
    const double* Uj = f.U + (int64_t)j * (K + 1);
    const double x = w[0] / Uj[0];
#pragma unroll
    for (int t = 1; t <= MW; ++t)
        if (t <= K) w[t] = fma(-Uj[t], x, w[t]);
    return x;
}

// One line per thread.  `in` may alias `out`: every position is loaded before
// it is stored (forward: stores trail the loads by kl; backward runs downward
// and stores trail by K), and the backward re-reads only this thread's stores.
template <int MW, int CKL, int CK>
__global__ void __launch_bounds__(256)
ksolve_strided_kernel(const LineGeom g, const BandLU f, const double* in, double* out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= g.no * g.n2) return;
    const int64_t i2 = tid % g.n2, io = tid / g.n2;
    const int64_t off = g.base + io * g.so + i2;
    const double* src = in + off;
    double* dst = out + off;
    const int n = f.n, kl = CKL >= 0 ? CKL : f.kl, K = CK >= 0 ? CK : f.K;
    constexpr int D = MW <= 4 ? 16 : 8;   // loads in flight per thread
    double w[MW + 1];
#pragma unroll
    for (int t = 0; t <= MW; ++t) w[t] = 0.0;
    for (int m0 = 0; m0 < n + kl; m0 += D) {
        double v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int m = m0 + d;
            v[d] = (m < n) ? src[(int64_t)m * g.sa] : 0.0;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int m = m0 + d;
            if (m >= n + kl) break;
            feed<MW>(w, kl, v[d]);
            const int j = m - kl;
            if (j >= 0) dst[(int64_t)j * g.sa] = step_fwd<MW, CKL>(w, f, j);
        }
    }
#pragma unroll
    for (int t = 0; t <= MW; ++t) w[t] = 0.0;
    for (int m0 = n - 1; m0 >= -K; m0 -= D) {
        double v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int m = m0 - d;
            v[d] = (m >= 0) ? dst[(int64_t)m * g.sa] : 0.0;
        }
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int m = m0 - d;
            if (m < -K) break;
            feed<MW>(w, K, v[d]);
            const int j = m + K;
            if (j <= n - 1) dst[(int64_t)j * g.sa] = step_bwd<MW, CK>(w, f, j);
        }
    }
}

constexpr int kRowWaves = 2;   // waves per workgroup (each wave is independent)
constexpr int kChunk = 16;     // columns per LDS chunk (one 128-B line per row segment)

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One sweep (BWD = 0 forward, 1 backward) over rows along the unit-stride axis.
// Forward feeds columns m = 0, 1, ... and emits y(m - kl); backward feeds
// m = n-1, n-2, ... and emits x(m + K).  in may alias out.
template <int MW, int BWD, int CKL, int CK>
__global__ void __launch_bounds__(64 * kRowWaves)
ksolve_rows_kernel(const RowLines g, const BandLU f, const double* in, double* out) {
    constexpr int C = kChunk, RPI = 64 / C;
    // one tile: a lane reads column c of its own row before it writes its output there
    __shared__ double s_in[kRowWaves][64][C + 1];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t row0 = ((int64_t)blockIdx.x * kRowWaves + wv) * 64;
    if (row0 >= g.nrows) return;  // the whole wave leaves; no block barriers below
    const int n = f.n, S = BWD ? (CK >= 0 ? CK : f.K) : (CKL >= 0 ? CKL : f.kl);
    const int ccol = lane % C, crow0 = lane / C;
    int64_t ra[C];   // row start of coop element i (row crow0 + i*RPI of the wave)
    bool rv[C];
#pragma unroll
    for (int i = 0; i < C; ++i) {
        const int64_t r = row0 + i * RPI + crow0;
        rv[i] = r < g.nrows;
        const int64_t rr = rv[i] ? r : 0;
        ra[i] = g.base + (rr / g.n1) * g.s0 + (rr % g.n1) * g.s1;
    }
    const int nch = (n + S + C - 1) / C;
    double pre[C];
    auto gload = [&](int q) {
        const int m = BWD ? (n - 1) - q * C - ccol : q * C + ccol;
        const bool ok = m >= 0 && m < n;
#pragma unroll
        for (int i = 0; i < C; ++i) pre[i] = (ok && rv[i]) ? in[ra[i] + m] : 0.0;
    };
    gload(0);
#pragma unroll
    for (int i = 0; i < C; ++i) s_in[wv][i * RPI + crow0][ccol] = pre[i];
    wave_sync();
    double w[MW + 1];
#pragma unroll
    for (int t = 0; t <= MW; ++t) w[t] = 0.0;
    for (int q = 0; q < nch; ++q) {
        if (q + 1 < nch) gload(q + 1);
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int m = BWD ? (n - 1) - q * C - c : q * C + c;
            feed<MW>(w, S, s_in[wv][lane][c]);
            const int j = BWD ? m + S : m - S;
            double o = 0.0;
            if (j >= 0 && j < n) o = BWD ? step_bwd<MW, CK>(w, f, j) : step_fwd<MW, CKL>(w, f, j);
            s_in[wv][lane][c] = o;
        }
        wave_sync();
        {
            const int j = BWD ? (n - 1) - q * C - ccol + S : q * C + ccol - S;
            if (j >= 0 && j < n) {
#pragma unroll
                for (int i = 0; i < C; ++i)
                    if (rv[i]) out[ra[i] + j] = s_in[wv][i * RPI + crow0][ccol];
            }
        }
        wave_sync();   // every lane has read its outputs before the tile is refilled
        if (q + 1 < nch) {
#pragma unroll
            for (int i = 0; i < C; ++i) s_in[wv][i * RPI + crow0][ccol] = pre[i];
        }
        wave_sync();
    }
}

static int mw_for(int w) {
    if (w <= 2) return 2;
    if (w <= 4) return 4;
    if (w <= 8) return 8;
    if (w <= 16) return 16;
    return 0;
}

// (kl, K) pairs with compiled-in bandwidths: GLT collocation p = 2, 3 (1, 2) and
// p = 4, 5 (2, 4), the symmetric p = 3 recipe (3, 6); anything else runs the
// run-time-bandwidth kernels with a window of MW >= max(kl, K).
template <template <int, int, int> class L, typename... A>
static int dispatch(const BandLU& f, A&&... a) {
    if (f.kl == 1 && f.K == 2) return L<2, 1, 2>::run(a...);
    if (f.kl == 2 && f.K == 4) return L<4, 2, 4>::run(a...);
    if (f.kl == 3 && f.K == 6) return L<8, 3, 6>::run(a...);
    switch (mw_for(std::max(f.kl, f.K))) {
        case 2: return L<2, -1, -1>::run(a...);
        case 4: return L<4, -1, -1>::run(a...);
        case 8: return L<8, -1, -1>::run(a...);
        case 16: return L<16, -1, -1>::run(a...);
        default: set_error("kron solve: kl + ku must be <= 16"); return 1;
    }
}

template <int MW, int CKL, int CK>
struct StridedL {
    static int run(const LineGeom& g, const BandLU& f, const double* in, double* out, hipStream_t st) {
        const int64_t nt = g.no * g.n2;
        hipLaunchKernelGGL((ksolve_strided_kernel<MW, CKL, CK>), dim3((unsigned)((nt + 255) / 256)), dim3(256), 0,
                           st, g, f, in, out);
        return 0;
    }
};

template <int MW, int CKL, int CK>
struct RowsL {
    static int run(const RowLines& g, const BandLU& f, const double* in, double* out, hipStream_t st) {
        const dim3 grid((unsigned)((g.nrows + 64 * kRowWaves - 1) / (64 * kRowWaves)));
        hipLaunchKernelGGL((ksolve_rows_kernel<MW, 0, CKL, CK>), grid, dim3(64 * kRowWaves), 0, st, g, f, in, out);
        hipLaunchKernelGGL((ksolve_rows_kernel<MW, 1, CKL, CK>), grid, dim3(64 * kRowWaves), 0, st, g, f,
                           (const double*)out, out);
        return 0;
    }
};

int ksolve_strided_launch(const LineGeom& g, const BandLU& f, const double* in, double* out, hipStream_t st) {
    if (g.no * g.n2 == 0 || f.n == 0) return 0;
    return dispatch<StridedL>(f, g, f, in, out, st);
}

int ksolve_rows_launch(const RowLines& g, const BandLU& f, const double* in, double* out, hipStream_t st) {
    if (g.nrows == 0 || f.n == 0) return 0;
    return dispatch<RowsL>(f, g, f, in, out, st);
}

// ---- host: banded LU with partial pivoting (LAPACK dgbtf2, 0-based) --------
// ab: column-major (ldab, n), ldab >= 2 kl + ku + 1, a(i, j) at
// ab[(kl + ku + i - j) + j*ldab] (the layout `to_bnd` builds,
// `sources/kron_product.py:179-191`).  Factorised in place; ipiv absolute
// 0-based rows.  Returns 0, or j+1 if u(j, j) is exactly zero (LAPACK info).
int band_lu(int64_t n, int kl, int ku, double* ab, int64_t ldab, int* ipiv) {
    const int kv = ku + kl;
    auto AB = [&](int64_t r, int64_t c) -> double& { return ab[r + c * ldab]; };
    // fill-in rows of columns ku+1 .. min(kv, n)-1 start at zero
    for (int64_t j = ku + 1; j < std::min<int64_t>(kv, n); ++j)
        for (int64_t i = kv - j; i < kl; ++i) AB(i, j) = 0.0;
    int64_t ju = 0;
    int info = 0;
    for (int64_t j = 0; j < n; ++j) {
        if (j + kv < n)
            for (int i = 0; i < kl; ++i) AB(i, j + kv) = 0.0;
        const int km = (int)std::min<int64_t>(kl, n - 1 - j);
        int jp = 0;
        double amax = std::fabs(AB(kv, j));
        for (int i = 1; i <= km; ++i)
            if (std::fabs(AB(kv + i, j)) > amax) { amax = std::fabs(AB(kv + i, j)); jp = i; }
        ipiv[j] = (int)(j + jp);
        if (AB(kv + jp, j) != 0.0) {
            ju = std::max<int64_t>(ju, std::min<int64_t>(j + ku + jp, n - 1));
            if (jp != 0)
                for (int64_t c = 0; c <= ju - j; ++c) std::swap(AB(kv + jp - c, j + c), AB(kv - c, j + c));
            if (km > 0) {
                const double r = 1.0 / AB(kv, j);
                for (int i = 1; i <= km; ++i) AB(kv + i, j) *= r;
                for (int64_t k = 1; k <= ju - j; ++k) {
                    const double y = AB(kv - k, j + k);
                    if (y == 0.0) continue;
                    const double tmp = -y;
                    for (int i = 1; i <= km; ++i) AB(kv + i - k, j + k) += AB(kv + i, j) * tmp;
                }
            }
        } else if (info == 0) {
            info = (int)(j + 1);
        }
    }
    return info;
}

// Factor tables of one axis from a factorised band (see BandLU).
void band_lu_tables(int64_t n, int kl, int ku, const double* ab, int64_t ldab, const int* ipiv,
                    std::vector<double>& L, std::vector<double>& U, std::vector<int>& piv) {
    const int kv = kl + ku, K = kv;
    L.assign((size_t)std::max<int64_t>(n * kl, 1), 0.0);
    U.assign((size_t)n * (K + 1), 0.0);
    piv.assign((size_t)n, 0);
    for (int64_t j = 0; j < n; ++j) {
        piv[j] = (int)(ipiv[j] - j);
        for (int t = 1; t <= kl; ++t)
            if (j + t < n) L[j * kl + t - 1] = ab[(kv + t) + j * ldab];
        for (int t = 0; t <= K; ++t)
            if (j - t >= 0) U[j * (K + 1) + t] = ab[(kv - t) + j * ldab];
    }
}

}  // namespace poms
