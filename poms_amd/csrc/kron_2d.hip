// Two damped-Jacobi sweeps of a 2D Kronecker(-sum) operator in one launch (round 6).
//
// The V-cycle's smoother (`sources/solvers.py:167-235`, damped_jacobi) runs its
// sweeps one after the other; at 2D sizes (1024^2: 8 MB per vector) a sweep is a
// few microseconds of work behind a ~2 us launch boundary, so the 2D cycle is
// bound by launches, not by HBM.  This kernel runs sweeps k and k+1 of the same
// loop in one launch: each workgroup computes sweep k on its output tile plus a
// P-wide halo (recomputed by the neighbouring tiles -- the same expressions on the
// same operands, so the same bits), keeps x_k in registers and finishes sweep k+1
// on the tile.  Only x_{k+1} is stored; the caller recomputes x_k with a single
// sweep in the rare case that sweep k's stop test fires (poms_pcg_jacobi).
//
// Tile: 8 waves, T = 2 RE + 6 R = 44 output rows x (64 - 4P) output columns; lane l is
// column c0 - 2P + l (both sweeps' halos in one 64-lane row).  Tile row q in
// [0, T + 4P) is interior row r0 - 2P + q:
//   phase A  axis 2 of x (DPP lane shifts, as kron_v3_kernel) for rows [0, T+4P)
//            -> (M2 x, K2 x) pairs in LDS
//   phase B  axis 1 from LDS + the Jacobi update for rows [P, T+3P): x_k, masked
//            to zero outside the domain (x's ghosts), kept in registers
//   phase C  axis 2 of x_k for the same rows -> LDS
//   phase D  axis 1 + the update for rows [2P, T+2P): x_{k+1}, stored
// Each wave's rows are contiguous (one LDS row read per row plus 2P per block), and
// x and b of a row stay in the registers of the wave that updates it: waves 1..6 own
// R output rows, waves 0 and 7 own RE and also carry the P halo rows of phase B and
// the 2P of phase A on their side (RE < R evens out the phases' critical path:
// 14.5 against 15.5 us at 1027^2 for RE = R = 6).  Where the tile lies in the
// Toeplitz interior of both axes the band rows and 1/diag(A) are constants.
//
// Bits: every sweep-k value is the kron_v3_kernel (variant 9) single sweep's --
// the same axis-2 product order (k = 0..2P, per-lane band rows), the same axis-1
// order, the same diag / reciprocal / update expressions; test_gpu_kernels.py
// compares x_{k+1} with two single sweeps bitwise.  The norms' partial sums group
// the points by this kernel's tiles (their rounding differs from the single sweeps').
// Preconditions (host): storage pads == P, one rank (zero ghost rows and columns),
// array < 2 GiB.
#include "common.hpp"

#include <cstdio>
#include <cstdlib>
#include <type_traits>

namespace poms {

namespace {
__device__ __forceinline__ double j2_shr1(double v) {   // lane l <- lane l-1 (lane 0 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double j2_shl1(double v) {   // lane l <- lane l+1 (lane 63 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
}  // namespace

constexpr int kJ2Waves = 8;
constexpr int kJ2Rows = 6;       // output rows of waves 1..6
constexpr int kJ2EdgeRows = 4;   // output rows of waves 0 and 7, which also carry the tile's halo rows
// (44-row tiles: 1027^2 is 24 x 20 = 480 workgroups, one round of the 512 slots)
constexpr int kJ2Tile = 2 * kJ2EdgeRows + (kJ2Waves - 2) * kJ2Rows;

template <int P, int R, int RE, int FORM, bool FZ = false>
__global__ void __launch_bounds__(kJ2Waves * 64, 4)   // 2 workgroups (16 waves) per CU
kron2d_j2_kernel(const double* __restrict__ x, double* __restrict__ y, const double* __restrict__ bvec,
                 const double* __restrict__ a1, const double* __restrict__ b1,
                 const double* __restrict__ a2, const double* __restrict__ b2,
                 double* __restrict__ part_k1, double* __restrict__ part_k, double* __restrict__ part_0,
                 const KronGeom g,
                 const ToepConst tc, const double omega) {
    constexpr int NW = kJ2Waves;
    constexpr int W = 2 * P + 1;
    constexpr int T = 2 * RE + (NW - 2) * R;
    constexpr int XR = T + 4 * P;    // tile rows
    constexpr int TO = 64 - 4 * P;   // output columns
    constexpr bool SUM = (FORM == FORM_SUM);
    typedef double d2 __attribute__((ext_vector_type(2)));
    __shared__ d2 ab_[SUM ? XR * 64 : 1];
    __shared__ double as_[SUM ? 1 : XR * 64];
    __shared__ double red[3 * NW];
    __shared__ double c2t[(SUM ? 2 : 1) * W * 64];   // [a|b][k][lane] boundary-tile axis-2 rows

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    int bid;
    {   // consecutive tiles on one XCD (blocks are dealt to the 8 XCDs round robin)
        const int nblk = gridDim.x, b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
        bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
    }
    const int t2 = bid % g.tiles2;
    const int t1 = bid / g.tiles2;
    const int c0 = t2 * TO;   // first output column
    const int r0 = t1 * T;    // first output row
    const int ic = c0 - 2 * P + lane;
    const bool col_in = ic >= 0 && ic < g.n2;
    const bool col_own = col_in && lane >= 2 * P && lane < 2 * P + TO;

    // axis-2 band rows: in column tiles inside the axis-2 Toeplitz interior from tc (the
    // same values as the per-lane rows, bitwise; no registers), in the two boundary
    // tiles per lane from an LDS table, one row at a time (sched_barrier: per-lane
    // registers for the 2(2P+1) values, or LDS reads hoisted over rows, spill at
    // 4 waves / SIMD)
    const bool fast2 = (max(c0 - 2 * P, 0) >= tc.lo2) && (min(c0 - 2 * P + 64, g.n2) <= tc.hi2);
    if (!fast2) {
        const int icc = min(max(ic, 0), g.n2 - 1);
        for (int k = wv; k < W; k += NW) {
            c2t[k * 64 + lane] = a2[icc * W + k];
            if constexpr (SUM) c2t[(W + k) * 64 + lane] = b2[icc * W + k];
        }
    }
    // phase-B rows (interior rows r0 - P .. r0 + T + P - 1) inside the axis-1 Toeplitz
    // interior: the band rows from tc (the same values bitwise); in the first and last
    // tile rows by scalar loads of the band table (the rows are wave-uniform)
    // (FZ scales every x-tile row by 1/diag: all of them in the interior)
    const bool fast1 = FZ ? (r0 - 2 * P >= tc.lo1) && (r0 + T + 2 * P <= tc.hi1)
                          : (r0 - P >= tc.lo1) && (r0 + T + P <= tc.hi1);

    const uint32_t arr_bytes = (uint32_t)((int64_t)(g.n0 + 2 * g.pd0) * g.s0 * 8);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, arr_bytes);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(bvec, arr_bytes);
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, arr_bytes);
    // storage (row, column) of tile row q, lane: (r0 - P + q, c0 - P + lane); before the
    // array's start the offset is negative, i.e. past num_records as an unsigned
    // voffset: the load returns 0
    auto off_of = [&](int q) { return ((r0 - P + q) * (int)g.s1 + (c0 - P + lane)) * 8; };

    double n_k = 0.0, n_k1 = 0.0, n_0 = 0.0;
    // axis 2 of one row held by this lane's column: (sum_k F2a[k] v[c+k-P], sum_k F2b[k] v[c+k-P])
    auto axis2 = [&](double v, double& sa, double& sb, auto c2) {
        double sh[W];
        sh[P] = v;
#pragma unroll
        for (int d = 1; d <= P; ++d) {
            sh[P - d] = j2_shr1(sh[P - d + 1]);
            sh[P + d] = j2_shl1(sh[P + d - 1]);
        }
        double ca, cb;
        c2(0, ca, cb);
        sa = ca * sh[0];
        sb = SUM ? cb * sh[0] : 0.0;
#pragma unroll
        for (int k = 1; k < W; ++k) {
            c2(k, ca, cb);
            sa = fma(ca, sh[k], sa);
            if constexpr (SUM) sb = fma(cb, sh[k], sb);
        }
    };
    auto c2_t = [&](int k, double& ca, double& cb) {
        const int jj = k < P ? P - k : k - P;
        ca = tc.t2a[jj];
        cb = SUM ? tc.t2b[jj] : 0.0;
    };
    auto c2_l = [&](int k, double& ca, double& cb) {
        ca = c2t[k * 64 + lane];
        cb = SUM ? c2t[(W + k) * 64 + lane] : 0.0;
    };
    auto put = [&](int q, double sa, double sb) {
        if constexpr (SUM) {
            d2 pr;
            pr.x = sa;
            pr.y = sb;
            ab_[q * 64 + lane] = pr;
        } else {
            as_[q * 64 + lane] = sa;
        }
    };
    // axis 1 for NR consecutive tile rows from q0 (LDS rows q0 - P .. q0 + NR + P - 1)
    // into cv[], in kron_v3_kernel's order (k = 0..2P, a then b per k)
    auto axis1 = [&](auto nr_c, int q0, double* cv, auto coef) {
        constexpr int NR = decltype(nr_c)::value;
#pragma unroll
        for (int r = 0; r < NR; ++r) cv[r] = 0.0;
#pragma unroll
        for (int qq = 0; qq < NR + 2 * P; ++qq) {
            const int rr = q0 - P + qq;
            double va, vb = 0.0;
            if constexpr (SUM) {
                const d2 pr = ab_[rr * 64 + lane];
                va = pr.x;
                vb = pr.y;
            } else {
                va = as_[rr * 64 + lane];
            }
#pragma unroll
            for (int r = 0; r < NR; ++r) {
                const int k = qq - r;
                if (k >= 0 && k < W) {
                    double ca, cb;
                    coef(q0 + r, k, ca, cb);
                    cv[r] = fma(ca, va, cv[r]);
                    if constexpr (SUM) cv[r] = fma(cb, vb, cv[r]);
                }
            }
        }
    };
    // band row of tile row q (phase-B rows): a separate unrolled body per source
    auto coef_t = [&](int, int k, double& ca, double& cb) {
        const int jj = k < P ? P - k : k - P;
        ca = tc.t1a[jj];
        cb = SUM ? tc.t1b[jj] : 0.0;
    };
    auto coef_l = [&](int q, int k, double& ca, double& cb) {
        const int row = min(max(r0 - 2 * P + q, 0), g.n1 - 1);
        ca = a1[row * W + k];
        cb = SUM ? b1[row * W + k] : 0.0;
    };
    // 1/diag(A) at tile row q (phase-B rows), this lane's column: kron_v3_kernel's
    // diag_parts expression and reciprocal
    auto rdiag = [&](int q, double d2a, double d2b, auto f1_c) {
        constexpr bool F1 = decltype(f1_c)::value;
        const int row = min(max(r0 - 2 * P + q, 0), g.n1 - 1);
        const double d1a = F1 ? tc.t1a[0] : a1[row * W + P];
        const double d1b = SUM ? (F1 ? tc.t1b[0] : b1[row * W + P]) : 0.0;
        const double dX = SUM ? diag2d_sum(d1a, d2a, d1b, d2b) : d1a * d2a;
        double rc = __builtin_amdgcn_rcp(dX);
        double e = fma(-dX, rc, 1.0);
        rc = fma(rc, e, rc);
        e = fma(-dX, rc, 1.0);
        rc = fma(rc, e, rc);
        return rc;
    };

    // the wave's rows: ROLE 0 (wave 0) and 2 (wave NW-1) own RE output rows and carry
    // the tile's halo rows on their side, the others own R; every register index below
    // is a compile-time constant.  F1: the phase-B rows in the axis-1 Toeplitz interior
    // (band rows from tc); with the axis-2 constants too, 1/diag(A) is one value for the
    // whole tile (the same expression on the same constants, so the same bits)
    auto body = [&](auto role_c, auto c2, auto f1_c) {
        constexpr int ROLE = decltype(role_c)::value;
        constexpr bool F1 = decltype(f1_c)::value;
        constexpr bool SLOW2 = !std::is_same_v<decltype(c2), decltype(c2_t)>;
        constexpr bool EDGE = ROLE != 1;
        constexpr int ND = EDGE ? RE : R;          // phase-D (output) rows
        constexpr int NA = EDGE ? ND + 2 * P : R;  // phase-A rows
        constexpr int NB = EDGE ? ND + P : R;      // phase-B / C rows
        constexpr int BA = ROLE == 0 ? P : 0;      // b_lo - a_lo
        constexpr int DA = ROLE == 0 ? 2 * P : 0;  // d_lo - a_lo
        const int d_lo = 2 * P + (ROLE == 0 ? 0 : ROLE == 2 ? RE + (NW - 2) * R : RE + (wv - 1) * R);
        const int a_lo = d_lo - DA;
        const int b_lo = a_lo + BA;
        double X[NA], Bv[NB];
#pragma unroll
        for (int j = 0; j < NA; ++j) X[j] = bload(rx, off_of(a_lo + j));
        __syncthreads();   // c2t
        double d2a, d2b, dummy;   // this lane's axis-2 band diagonal (after the barrier: c2t)
        c2(P, d2a, dummy);
        d2b = 0.0;
        if constexpr (SUM) c2(P, dummy, d2b);
        auto coef = [&](int q, int k, double& ca, double& cb) {
            if constexpr (F1) coef_t(q, k, ca, cb);
            else coef_l(q, k, ca, cb);
        };
        constexpr bool RC1 = F1 && !SLOW2;
        const double rc1 = RC1 ? rdiag(P, d2a, d2b, f1_c) : 0.0;
        if constexpr (FZ) {
            // x is b: keep b of the phase-B rows, then x1 = (omega b) / diag(A) at every
            // x-tile point (poms_op_diag_scale's expression; zero outside the domain)
#pragma unroll
            for (int r = 0; r < NB; ++r) Bv[r] = X[BA + r];
#pragma unroll
            for (int j = 0; j < NA; ++j) {
                const int q = a_lo + j;
                const int ir = r0 - 2 * P + q;
                const bool ok = col_in && ir >= 0 && ir < g.n1;
                const double rc = RC1 ? rc1 : rdiag(q, d2a, d2b, f1_c);
                const double v = omega * X[j] * rc;
                X[j] = ok ? v : 0.0;
                const bool own = ok && lane >= 2 * P && lane < 2 * P + TO && q >= 2 * P && q < T + 2 * P;
                n_0 = own ? fma(v, v, n_0) : n_0;   // ||x1||^2 = ||dr_1||^2
            }
        }
        // ---- phase A: axis 2 of x
#pragma unroll
        for (int j = 0; j < NA; ++j) {
            double sa, sb;
            axis2(X[j], sa, sb, c2);
            put(a_lo + j, sa, sb);
            if constexpr (SLOW2) __builtin_amdgcn_sched_barrier(0);
        }
        // b of the phase-B rows (not live during phase A)
        if constexpr (!FZ) {
#pragma unroll
            for (int j = 0; j < NB; ++j) Bv[j] = bload(rb, off_of(b_lo + j));
        }
        __syncthreads();
        // ---- phase B: sweep k on rows [b_lo, b_lo + NB)
        {
            double cv[NB];
            axis1(std::integral_constant<int, NB>{}, b_lo, cv, coef);
#pragma unroll
            for (int r = 0; r < NB; ++r) {
                const int q = b_lo + r;
                const int ir = r0 - 2 * P + q;
                const bool ok = col_in && ir >= 0 && ir < g.n1;
                const double rc = RC1 ? rc1 : rdiag(q, d2a, d2b, f1_c);
                const double dr = omega * (Bv[r] - cv[r]) * rc;
                const double xk = add_nc(X[BA + r], dr);
                X[BA + r] = ok ? xk : 0.0;   // x_k's zero ghosts outside the domain
                const bool own = ok && lane >= 2 * P && lane < 2 * P + TO && q >= 2 * P && q < T + 2 * P;
                n_k = own ? fma(dr, dr, n_k) : n_k;
            }
        }
        double Bd[ND];   // b of the phase-D rows, again (L2): Bv is not kept live past phase B
#pragma unroll
        for (int r = 0; r < ND; ++r) Bd[r] = FZ ? Bv[DA - BA + r] : bload(rb, off_of(d_lo + r));
        __syncthreads();   // every wave's phase-B reads of the LDS tile are done
        // ---- phase C: axis 2 of x_k
#pragma unroll
        for (int r = 0; r < NB; ++r) {
            double sa, sb;
            axis2(X[BA + r], sa, sb, c2);
            put(b_lo + r, sa, sb);
            if constexpr (SLOW2) __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        // ---- phase D: sweep k + 1 on rows [d_lo, d_lo + ND), stored
        {
            double cv[ND];
            axis1(std::integral_constant<int, ND>{}, d_lo, cv, coef);
#pragma unroll
            for (int r = 0; r < ND; ++r) {
                const int q = d_lo + r;
                const int ir = r0 - 2 * P + q;
                const bool own = col_own && ir < g.n1;
                const double rc = RC1 ? rc1 : rdiag(q, d2a, d2b, f1_c);
                const double dr = omega * (Bd[r] - cv[r]) * rc;
                const double xk1 = add_nc(X[DA + r], dr);
                n_k1 = own ? fma(dr, dr, n_k1) : n_k1;
                bstore(ry, own ? off_of(q) : 0x7ffffff0, xk1);
            }
        }
    };
    auto roles = [&](auto c2, auto f1_c) {
        if (wv == 0) body(std::integral_constant<int, 0>{}, c2, f1_c);
        else if (wv == NW - 1) body(std::integral_constant<int, 2>{}, c2, f1_c);
        else body(std::integral_constant<int, 1>{}, c2, f1_c);
    };
    if (fast2) {
        if (fast1) roles(c2_t, std::true_type{});
        else roles(c2_t, std::false_type{});
    } else {
        if (fast1) roles(c2_l, std::true_type{});
        else roles(c2_l, std::false_type{});
    }

    if (part_k1 != nullptr || part_k != nullptr || part_0 != nullptr) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            n_k += __shfl_xor(n_k, off, 64);
            n_k1 += __shfl_xor(n_k1, off, 64);
            if constexpr (FZ) n_0 += __shfl_xor(n_0, off, 64);
        }
        if (lane == 0) {
            red[wv] = n_k;
            red[NW + wv] = n_k1;
            red[2 * NW + wv] = n_0;
        }
        __syncthreads();
        if (tid == 0) {
            double s = 0.0, s1 = 0.0, s0 = 0.0;
            for (int w = 0; w < NW; ++w) {
                s += red[w];
                s1 += red[NW + w];
                s0 += red[2 * NW + w];
            }
            if (part_k != nullptr) part_k[blockIdx.x] = s;
            if (part_k1 != nullptr) part_k1[blockIdx.x] = s1;
            if (FZ && part_0 != nullptr) part_0[blockIdx.x] = s0;
        }
    }
}

// tile shape (R, RE): POMS_J2_TILE=r,re (tuning: 6,4 default; 7,5; 6,5; 5,4; 5,3)
static void j2_tile(int* r, int* re) {
    static int R = -1, RE = -1;
    if (R < 0) {
        R = kJ2Rows;
        RE = kJ2EdgeRows;
        if (const char* e = getenv("POMS_J2_TILE")) {
            int a = 0, b = 0;
            if (sscanf(e, "%d,%d", &a, &b) == 2 &&
                ((a == 7 && b == 5) || (a == 6 && b == 5) || (a == 5 && b == 4) || (a == 5 && b == 3))) {
                R = a;
                RE = b;
            }
        }
    }
    *r = R;
    *re = RE;
}
int kron2d_j2_rows() {
    int r, re;
    j2_tile(&r, &re);
    return 2 * re + (kJ2Waves - 2) * r;
}
int kron2d_j2_rows_default() { return kJ2Tile; }
int kron2d_j2_cols(int pmax) { return 64 - 4 * pmax; }

template <int R, int RE, bool FZ = false>
static void j2_launch_t(int form, const KronPtrs& p, double* part0, const KronGeom& g, const ToepConst& tc,
                        double omega, hipStream_t st, int nblk) {
    if (form == FORM_SUM)
        hipLaunchKernelGGL((kron2d_j2_kernel<3, R, RE, FORM_SUM, FZ>), dim3(nblk), dim3(kJ2Waves * 64), 0, st, p.x,
                           p.y, p.b, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, part0, g, tc, omega);
    else
        hipLaunchKernelGGL((kron2d_j2_kernel<3, R, RE, FORM_SINGLE, FZ>), dim3(nblk), dim3(kJ2Waves * 64), 0, st, p.x,
                           p.y, p.b, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, part0, g, tc, omega);
}

// Two sweeps x -> y; p.partial: sweep k+1's ||dr||^2 per block, p.partial2: sweep k's.
// from_zero: sweeps 1-3 from x = 0 (p.x = p.b), part0: ||x1||^2 per block (p.partial2:
// sweep 2, p.partial: sweep 3).
// g: the operator's 2D geometry with tiles1 / tiles2 for kron2d_j2_rows / _cols.
int kron2d_j2_launch(int pmax, int form, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, double omega,
                     hipStream_t st, bool from_zero, double* part0) {
    if (pmax != 3 || (form != FORM_SUM && form != FORM_SINGLE)) {
        set_error("two sweeps per launch: 2D p = 3 Kronecker operators only");
        return 1;
    }
    if (g.pd1 != 3 || g.pd2 != 3 || g.tiles1 * kron2d_j2_rows() < g.n1 || g.tiles2 * kron2d_j2_cols(3) < g.n2 ||
        (int64_t)(g.n0 + 2 * g.pd0) * g.s0 * 8 >= 0x7ffffff0LL) {
        set_error("two sweeps per launch: bad geometry");
        return 1;
    }
    const int nblk = g.tiles1 * g.tiles2;
    int r, re;
    j2_tile(&r, &re);
    if (from_zero) {   // (the default tile only)
        if (r != kJ2Rows || re != kJ2EdgeRows) { set_error("three sweeps from zero: default tile only"); return 1; }
        j2_launch_t<kJ2Rows, kJ2EdgeRows, true>(form, p, part0, g, tc, omega, st, nblk);
        return 0;
    }
    if (r == 7) j2_launch_t<7, 5>(form, p, nullptr, g, tc, omega, st, nblk);
    else if (r == 6 && re == 5) j2_launch_t<6, 5>(form, p, nullptr, g, tc, omega, st, nblk);
    else if (r == 5 && re == 4) j2_launch_t<5, 4>(form, p, nullptr, g, tc, omega, st, nblk);
    else if (r == 5 && re == 3) j2_launch_t<5, 3>(form, p, nullptr, g, tc, omega, st, nblk);
    else j2_launch_t<kJ2Rows, kJ2EdgeRows>(form, p, nullptr, g, tc, omega, st, nblk);
    return 0;
}

}  // namespace poms
