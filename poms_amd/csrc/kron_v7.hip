// Fused Kronecker-sum operator, v7 (variant 11): flat lane mapping, axis 1 then
// axis 2 through LDS windows, one barrier per plane.
//
// Why (round 4).  v5 (kron_v5.hip) gives each wave one output row of a 128-column
// tile: 16 of its 128 lane-columns are halo, the last tile column of a 515-wide grid
// holds 67 output columns in 128 lanes, and the axis-2 neighbours come in by 24 DPP
// lane shifts per lane and plane -- 121 VALU instructions per lane and plane for
// ~1.65 output points on average (profiles/r03/pmc_sq_v5_apply_jacobi.txt).  The
// VALU is busy ~68 % of the kernel while the access pattern alone needs ~80 % of
// its time, and at 4 waves per SIMD the two do not overlap better than that.
//
// v7 separates the two passes and lets the lanes of a workgroup map onto the tile
// freely ("flat" pairs: lane L of wave W handles pair W*64+L in row-major order):
//   * tile: R output rows x C output columns (C = 112 for the wide tile columns:
//     7 whole 128-B lines of output per row on the aligned layout; the last tile
//     column, when the grid is not a multiple of 112 wide, is CN < 112 columns wide
//     and has more rows);
//   * x tile: R+2P rows x XP pairs (XP = C/2 + 2 HP, HP = ceil(P/2) halo pairs a
//     side), packed flat in LDS (pair q*XP + k) and DMA'd by buffer_load ... lds,
//     64 pairs per instruction, into a D-deep ring, D-1 planes ahead;
//   * stage 1, plane t: lane -> (row r, x pair k), R*XP <= 1024: u = F1a x and
//     v = F1b x from the 2P+1 x-tile rows around r (one ds_read_b128 per tap at a
//     constant offset), written into the u/v buffer of plane t (two slots);
//   * stage 2, plane t-1: lane -> (row r, output pair j): the axis-2 window (2HP+1
//     pairs of u and of v, read from LDS: no lane shifts), c = F2a u and
//     d = F2a v + F2b u, then the axis-0 scatter into 2P+1 rotating accumulators and
//     the epilogue of the finished plane;
//   * one barrier per plane: after it x(t) has landed, u/v(t-1) is complete, and
//     every wave has finished reading u/v(t-2) and x(t-1), whose slots the
//     iteration then refills.
//
// Preconditions (host, v7_ok in poms_abi.hip): 3D FORM_SUM, P == 3, storage pads ==
// P, line-aligned layout (row pitch a multiple of 16 doubles, interior column 0 on a
// 128-B line), array < 2 GiB, every non-Toeplitz row / column of the axis-1 / axis-2
// factors among the first or last 2P (open uniform knots: rows 0 .. 2p-1 touch a
// non-uniform basis function), and no data in the corner ghosts (as v5 at odd P).
#include "common.hpp"

#include <algorithm>
#include <cstdlib>

namespace poms {

#ifndef POMS_V7_STUB   // (the product build compiles this file with POMS_V7_STUB: v7 is an
                       // experimental variant, slower than v5; POMS_WITH_V7=1 builds it)

typedef __attribute__((address_space(3))) void lds7_void_t;

struct V7Geom {
    int nw2;        // wide tile columns (112 output columns each)
    int cn;         // narrow last tile column: template width (0: none)
    int rw, rn;     // output rows per wide / narrow tile
    int t1w, t1n;   // tile rows of each type
    int ntiles;     // nw2 * t1w + (cn ? t1n : 0)
};

constexpr int V7_NW = 16;           // waves per workgroup
constexpr int V7_CW = 112;          // output columns of a wide tile
constexpr int v7_hp(int P) { return (P + 1) / 2; }
constexpr int v7_xp(int P, int C) { return C / 2 + 2 * v7_hp(P); }
constexpr int v7_rmax(int P, int C) { return 1024 / v7_xp(P, C); }
// x-tile DMAs per plane at the largest R the lanes allow (R * XP <= 1024)
constexpr int v7_ndma(int P, int C) { return ((v7_rmax(P, C) + 2 * P) * v7_xp(P, C) + 63) / 64; }
constexpr int v7_max(int a, int b) { return a > b ? a : b; }
// Entry of boundary-table row / column i of an n-long factor: the first and last NE
// rows have their own entries (B-spline factors on open knots: rows 0 .. 2p-1 and
// n-2p .. n-1 touch a non-uniform basis function), every other row the Toeplitz one
// (entry 2 NE).  Host precondition (v7_ok): the Toeplitz range covers [NE, n - NE).
__device__ __forceinline__ int v7_bidx(int i, int n, int NE) {
    return i < NE ? i : (i >= n - NE ? NE + i - (n - NE) : 2 * NE);
}

template <int AUX = 0>
__device__ __forceinline__ void v7_dma16(__amdgpu_buffer_rsrc_t r, double* lds_dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds7_void_t*)lds_dst, 16, voff, (int)soff, 0, AUX);
}
template <int AUX>
__device__ __forceinline__ void v7_store16(__amdgpu_buffer_rsrc_t r, int voff, double d0, double d1) {
    u32x4 v;
    const u32x2 a = __builtin_bit_cast(u32x2, d0), b = __builtin_bit_cast(u32x2, d1);
    v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, AUX);
}
template <int N>
__device__ __forceinline__ void v7_wait_vm() {  // s_waitcnt vmcnt(N) (gfx9 encoding)
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void v7_barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}

// LDS layout (doubles), shared by the two tile shapes of one launch
template <int P, int D, int CN>
struct V7Lds {
    static constexpr int W = 2 * P + 1;
    static constexpr int NDMA = v7_max(v7_ndma(P, V7_CW), CN ? v7_ndma(P, CN) : 0);
    static constexpr int SLOT = 128 * NDMA;        // one x plane tile
    static constexpr int XS = 0;
    static constexpr int UVQ = 2048;               // one quantity (u or v) of one slot: 1024 pairs
    static constexpr int UV = XS + D * SLOT;       // 2 slots x (u, v); the two-barrier schedule
                                                   // uses one and puts its b ring in the other
    static constexpr int BRING = UV + 2 * UVQ;
    static constexpr int NE = 2 * P;               // edge rows of a factor kept in the boundary tables
    static constexpr int NBT = (2 * NE + 1) * W * 2;  // rows 0..NE-1, n-NE..n-1, the Toeplitz row
    static constexpr int BT1 = UV + 4 * UVQ;
    static constexpr int BT2 = BT1 + NBT;
    static constexpr int RED = BT2 + NBT;
    static constexpr int N = RED + V7_NW;
};

// One workgroup's march over its tile (R rows x C output columns) and axis-0 chunk.
// EPI: APPLY (y = A x), RESID (r = b - A x), JACOBI (x_out = x + omega (b - A x) / diag,
// ||dr||^2 and with JDOT x_out . b per block), APPLYDOT (y = A x, x . y per block).
template <int P, int EPI, int D, int C, int CN, int CP, bool SAME12, bool JDOT>
__device__ __forceinline__ void v7_body(double* __restrict__ lds, const double* __restrict__ x,
                                        double* __restrict__ y, const double* __restrict__ bvec,
                                        const double* __restrict__ a0t, const double* __restrict__ b0t,
                                        const double* __restrict__ rdiag0, const KronGeom& g, const ToepConst& tc,
                                        const double omega, const int R, const int r0, const int c0, const int ch,
                                        double& nrm, double& dotp) {
    typedef V7Lds<P, D, CN> L;
    constexpr int W = L::W;
    // Residual, Jacobi and apply-dot (b read, or an x history) run the two-barrier
    // schedule (TB2, below); the apply the pipelined one.  Rotating axis-0 accumulators: the pipelined march
    // keeps 8 (>= 2P+1) so that its ring indices (x slot t % 4, x history t % 4) fold
    // at compile time over the 8-plane unroll; TB2 keeps 2P+1 (its slots are indexed at
    // run time, its x history is a shift register).
    constexpr bool HASB = EPI == EPI_RESID || EPI == EPI_JACOBI;
    constexpr bool J0 = EPI == EPI_JACOBI0;   // sweeps 1 and 2 from x = 0 (the x ring holds b)
    constexpr bool TB2 = HASB || J0 || EPI == EPI_APPLYDOT;   // (apply-dot: its x history)
    constexpr int NS = TB2 ? W : 8;
    static_assert(NS >= W && (TB2 || (NS % D == 0 && D == 4)), "ring indices fold over the 8-plane unroll");
    constexpr int HP = v7_hp(P);
    constexpr int XP = v7_xp(P, C);     // x pairs per x-tile row
    constexpr int OP = C / 2;           // output pairs per row
    constexpr int NWIN = 2 * HP + 1;    // window pairs of one quantity
    constexpr int PFX = D - 1;          // x prefetch distance (planes)
    constexpr int YAUX = (CP & 4) ? 2 : 0;
    constexpr int BAUX = (CP & 2) ? 2 : 0;
    constexpr int XAUX = (CP & 1) ? 2 : 0;   // x DMAs non-temporal (tuning; the halo rows are re-read)
    constexpr bool JAC = EPI == EPI_JACOBI;
    constexpr bool APD = EPI == EPI_APPLYDOT;
    constexpr bool HIST = JAC || APD || J0;   // x (J0: x1) at the output point (a register history)
    // diagnostic builds (apply, timing only): CP bit 256 = memory only (the DMAs and
    // stores, no LDS reads or arithmetic), bit 512 = arithmetic only (no DMA, no bytes
    // stored)
    constexpr bool MEMONLY = (CP & 256) != 0, ARITHONLY = (CP & 512) != 0;
    typedef double d2 __attribute__((ext_vector_type(2)));
    static_assert(v7_ndma(P, C) <= 2 * V7_NW, "at most two x DMAs per wave and plane");
#define T2A(k) (SAME12 ? tc.t1a[k] : tc.t2a[k])
#define T2B(k) (SAME12 ? tc.t1b[k] : tc.t2b[k])

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fl = wv * 64 + lane;      // this lane's flat pair index

    // One mapping for both stages: lane -> (row ru, x pair ku), R*XP <= 1024.  Stage 1
    // computes u, v of that pair; stage 2 the output pair jo = ku - HP of the same row
    // (lanes on the 2 HP halo pairs of a row have no output), so the stage-1 centre
    // tap is the x at the lane's own output point (the Jacobi / apply-dot history).
    // Idle lanes read pair 0 (in range) and write nothing.
    // (idle lanes keep their own, distinct addresses: a shared dummy address puts a
    // second address on some bank of almost every lane group -- 2-way LDS conflicts)
    const int ru = fl / XP, ku = fl - ru * XP;
    const bool act1 = ru < R;
    const int fu = act1 ? fl : fl - R * XP;   // (idle lanes: pairs 0.. of the tile, in range)
    const int jo = ku - HP;
    const bool act2 = act1 && jo >= 0 && jo < OP;
    const int fo = max(fu - HP, 0);     // first window pair (row ru, x pair jo) in the u/v buffer
    const int orow = r0 + ru;           // output row (stage 2)
    const int ocol = c0 + 2 * jo;       // output column of element 0

    // fast paths: axis 1 per lane (its row inside the Toeplitz interior: the same choice
    // per output row as v5, whose waves are rows, so the two agree bitwise), axis 2 per
    // tile (every column of the tile Toeplitz: v5's per-workgroup choice, on the same
    // 112-column tile boundaries)
    const bool fast1 = orow >= tc.lo1 && orow < tc.hi1;
    const bool fast2 = c0 >= tc.lo2 && min(c0 + C, g.n2) <= tc.hi2;

    int z0, z1;
    chunk_planes(g, ch, z0, z1);
    const int nplanes = (z1 - z0) + 2 * P;
    const int nsp = g.n0 + 2 * g.pd0;
    const int s1 = (int)g.s1;
    const uint32_t arr_bytes = (uint32_t)((int64_t)nsp * g.s0 * 8);
    const uint32_t plane8 = (uint32_t)(g.s0 * 8);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, arr_bytes);
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, arr_bytes);
    const __amdgpu_buffer_rsrc_t rb = make_rsrc(bvec, HASB ? arr_bytes : 0u);

    // ---- per-lane DMA voffsets (the plane goes into soffset): DMA i of a plane moves
    // flat x pairs 64 i .. 64 i + 63; this wave issues i = wv and, if dma2, wv + 16.
    // Pairs past the tile, rows past the padded rows and columns past the row pitch
    // get a voffset out of the buffer range (+2^31, arrays < 2 GiB): no bytes move.
    const int nxp = (R + 2 * P) * XP;
    const bool dma2 = wv + V7_NW < (nxp + 63) / 64;
    uint32_t xvo[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int f = (wv + s * V7_NW) * 64 + lane;
        const int q = f / XP, k = f - q * XP;
        const int srow = r0 + q;        // x-tile row q = interior row r0 - P + q = storage row r0 + q
        const int scol = g.pd2 + c0 - 2 * HP + 2 * k;
        // (the pair at storage column -1 of storage row 0 -- the corner ghost -- is dropped,
        // as in v5: zero unless the layout holds corner data, which v7_ok excludes)
        const bool ok = f < nxp && srow < g.n1 + 2 * g.pd1 && srow * s1 + scol >= 0 && scol + 1 < s1;
        xvo[s] = ok ? (uint32_t)((srow * s1 + scol) * 8) : 0x80000000u;
    }
    auto dma_x = [&](int t, int slot) {   // x plane t of the march (dummy past its end)
        if constexpr (ARITHONLY) return;
        const int sp = z0 - P + t + g.pd0;
        const bool ok = t < nplanes && sp >= 0 && sp < nsp;
        const uint32_t so = ok ? (uint32_t)sp * plane8 : 0u;
        double* dst = lds + L::XS + slot * L::SLOT + wv * 128;
        v7_dma16<XAUX>(rx, dst, ok ? (int)xvo[0] : (int)0x80000000u, so);
        if (dma2) v7_dma16<XAUX>(rx, dst + V7_NW * 128, ok ? (int)xvo[1] : (int)0x80000000u, so);
    };
    // output point of stage 2 (row-and-column part; the plane goes in separately)
    const bool okrc0 = act2 && orow < g.n1 && ocol < g.n2;
    const bool okrc1 = act2 && orow < g.n1 && ocol + 1 < g.n2;
    const int vrc = ((orow + g.pd1) * s1 + g.pd2 + ocol) * 8;
    auto zo_of = [&](int t2) { return max(z0 - 2 * P + t2, z0); };
    // ---- Jacobi: omega / diag(A) at this lane's two output points on the planes of the
    // axis-0 Toeplitz interior (plane-invariant there: computed once), and the
    // plane-invariant factors X = d1a d2a, Y = d1b d2a + d1a d2b of diag(A) = d0a X + d0b Y
    auto rcp_nr = [](double dg) {   // 1/dg: v_rcp_f64 + two Newton steps
        double r = __builtin_amdgcn_rcp(dg);
        double ee = fma(-dg, r, 1.0);
        r = fma(r, ee, r);
        ee = fma(-dg, r, 1.0);
        return fma(r, ee, r);
    };
    auto diag_xy = [&](int e, double& X, double& Y) {
        const int col = ocol + e;
        const int b1 = v7_bidx(orow, g.n1, L::NE), b2 = v7_bidx(col, g.n2, L::NE);
        const d2 f1 = *(const d2*)(lds + L::BT1 + 2 * (W * (act2 ? b1 : 2 * L::NE) + P));
        const d2 f2 = *(const d2*)(lds + L::BT2 + 2 * (W * (act2 ? b2 : 2 * L::NE) + P));
        X = f1[0] * f2[0];
        Y = fma(f1[1], f2[0], f1[0] * f2[1]);
    };
    const bool rfast = fast1 && fast2 && rdiag0 != nullptr;
    double rci[2] = {0.0, 0.0};
    if constexpr (JAC) {
        if (!rfast) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                double X, Y;
                diag_xy(e, X, Y);
                const double dg = fma(tc.t0a[0], X, tc.t0b[0] * Y);
                rci[e] = dg != 0.0 ? omega * rcp_nr(dg) : 0.0;
            }
        }
    }

    // ---- two sweeps from zero: s = omega / diag(A) (x1 = s b, x2 = x1 + s (b - A x1)).
    // s at (plane with axis-0 diagonal d0a, d0b; row; column), as v5's j0_scale; and
    // sc[e] at this lane's columns on Toeplitz rows and planes, where s depends on the
    // column only (the stage-1 columns of the lane are its output columns)
    auto s_at = [&](double d0a, double d0b, int row, int col) {
        row = min(max(row, 0), g.n1 - 1);
        col = min(max(col, 0), g.n2 - 1);
        const d2 f1 = *(const d2*)(lds + L::BT1 + 2 * (W * v7_bidx(row, g.n1, L::NE) + P));
        const d2 f2 = *(const d2*)(lds + L::BT2 + 2 * (W * v7_bidx(col, g.n2, L::NE) + P));
        const double dg = fma(d0a, f1[0] * f2[0], d0b * fma(f1[1], f2[0], f1[0] * f2[1]));
        return dg != 0.0 ? omega * rcp_nr(dg) : 0.0;   // zero diagonal: a ghost plane (b = 0)
    };
    // J0: every x-tile row (the 2P halo rows too) has the Toeplitz axis-1 band: on such a
    // tile and a Toeplitz plane x1 = sc(col) b, and the scaling commutes with the axis-1
    // pass (applied to u, v after it, as v5 does on its row-Toeplitz tiles)
    const bool jrf = J0 && r0 - P >= tc.lo1 && r0 + R + P <= tc.hi1;
    double sc[2] = {0.0, 0.0};
    auto j0_sc_after = [&](int tt) {   // (tile-uniform)
        const int m = g.g0 + z0 - P + tt;   // global plane of x(tt)
        return jrf && m >= tc.lo0 && m < tc.hi0;
    };
    // Otherwise (boundary tile rows, the P planes next to each global end of axis 0) the
    // ring slot of x(tt) = b is scaled to x1 = s b in place, each wave the pairs it
    // DMA'd, between the plane's barrier and one more (rare: a few % of the work)
    auto j0_scale_slot = [&](double* slot, int tt) {
        const int m = g.g0 + z0 - P + tt;
        const bool tp = m >= tc.lo0 && m < tc.hi0;
        const int i0 = (m + P) * W + P;   // (a0t is padded by P planes on each side)
        const double d0a = tp ? tc.t0a[0] : a0t[i0], d0b = tp ? tc.t0b[0] : b0t[i0];
        const int nxp2 = (R + 2 * P) * XP;
#pragma unroll
        for (int sdma = 0; sdma < 2; ++sdma) {
            const int f = (wv + sdma * V7_NW) * 64 + lane;
            if (f < nxp2) {
                const int qq = f / XP, kk = f - qq * XP;
                d2* pr = (d2*)(slot + 2 * f);
                d2 vv = *pr;
#pragma unroll
                for (int e = 0; e < 2; ++e) vv[e] *= s_at(d0a, d0b, r0 - P + qq, c0 - 2 * HP + 2 * kk + e);
                *pr = vv;
            }
        }
    };

    double acc[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) { acc[s][0] = 0.0; acc[s][1] = 0.0; }

    // ---- stage 1 of one x plane tile (xsl): u = F1a x, v = F1b x of the lane's pair into
    // the u/v buffer at uvb; returns the x tap at the lane's output point
    auto stage1 = [&](const double* xsl, double* uvb, int tt) -> d2 {
        const double* xs = xsl + 2 * fu;
        d2 xv[W];
#pragma unroll
        for (int k = 0; k < W; ++k) xv[k] = *(const d2*)(xs + 2 * k * XP);
        // J0: scale u, v (and the centre) after the axis-1 pass; elsewhere the ring slot was
        // scaled in place before this pass (j0_scale_slot)
        const bool jsc = J0 && j0_sc_after(tt);
        double u[2], v[2];
        if (fast1) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                double pr[P + 1];
                pr[0] = xv[P][e];
#pragma unroll
                for (int k = 1; k <= P; ++k) pr[k] = xv[P - k][e] + xv[P + k][e];
                double su = tc.t1a[0] * pr[0], sv = tc.t1b[0] * pr[0];
#pragma unroll
                for (int k = 1; k <= P; ++k) {
                    su = fma(tc.t1a[k], pr[k], su);
                    sv = fma(tc.t1b[k], pr[k], sv);
                }
                u[e] = su;
                v[e] = sv;
            }
        } else {
            const int row = r0 + ru;
            const double* bt = lds + L::BT1 + 2 * W * (act1 ? v7_bidx(row, g.n1, L::NE) : 2 * L::NE);
            u[0] = u[1] = v[0] = v[1] = 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                const d2 f = *(const d2*)(bt + 2 * k);
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    u[e] = fma(f[0], xv[k][e], u[e]);
                    v[e] = fma(f[1], xv[k][e], v[e]);
                }
            }
        }
        if constexpr (J0) {
            if (jsc) {
                const d2 scl = *(const d2*)(lds + L::BRING + L::UVQ + 2 * fl);
                double sc[2] = {scl[0], scl[1]};
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    u[e] *= sc[e];
                    v[e] *= sc[e];
                    xv[P][e] *= sc[e];   // the centre tap the x1 history keeps
                }
            }
        }
        if (act1) {
            double* uv = uvb + 2 * fl;
            *(d2*)uv = d2{u[0], u[1]};
            *(d2*)(uv + L::UVQ) = d2{v[0], v[1]};
        }
        return xv[P];
    };
    // ---- stage 2, axis 2: c = F2a u, d = F2a v + F2b u at the lane's output pair from
    // the u/v buffer at uvb
    auto axis2 = [&](const double* uvb, double cc[2], double dd[2]) {
        const double* us = uvb + 2 * fo;
        // window values 2HP - P .. 2HP + 1 + P (columns ocol - P .. ocol + 1 + P): whole
        // pairs inside, single doubles at odd-P edges
        constexpr int W0 = 2 * HP - P, W1 = 2 * HP + 1 + P;
        double wu[2 * NWIN], wvv[2 * NWIN];
#pragma unroll
        for (int m = 0; m < NWIN; ++m) {
            if (2 * m + 1 < W0 || 2 * m > W1) continue;
            // whole pairs (ds_read_b128) even where one value is used: single doubles at a
            // 16-B lane stride (ds_read_b64) conflict 2-way on every lane group.  (The
            // Jacobi build with the fused dot lacks the 4 VGPRs: single doubles there.)
            if constexpr (JAC && JDOT) {
                if (2 * m < W0) {
                    wu[2 * m + 1] = us[2 * m + 1];
                    wvv[2 * m + 1] = us[L::UVQ + 2 * m + 1];
                    continue;
                }
                if (2 * m + 1 > W1) {
                    wu[2 * m] = us[2 * m];
                    wvv[2 * m] = us[L::UVQ + 2 * m];
                    continue;
                }
            }
            const d2 a = *(const d2*)(us + 2 * m);
            const d2 b = *(const d2*)(us + L::UVQ + 2 * m);
            wu[2 * m] = a[0];
            wu[2 * m + 1] = a[1];
            wvv[2 * m] = b[0];
            wvv[2 * m + 1] = b[1];
        }
        if (fast2) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int cen = 2 * HP + e;
                double pu[P + 1], pv[P + 1];
                pu[0] = wu[cen];
                pv[0] = wvv[cen];
#pragma unroll
                for (int k = 1; k <= P; ++k) {
                    pu[k] = wu[cen - k] + wu[cen + k];
                    pv[k] = wvv[cen - k] + wvv[cen + k];
                }
                double c = T2A(0) * pu[0];
                double d = fma(T2A(0), pv[0], T2B(0) * pu[0]);
#pragma unroll
                for (int k = 1; k <= P; ++k) {
                    c = fma(T2A(k), pu[k], c);
                    d = fma(T2A(k), pv[k], fma(T2B(k), pu[k], d));
                }
                cc[e] = c;
                dd[e] = d;
            }
        } else {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int col = ocol + e;
                const double* bt = lds + L::BT2 + 2 * W * (act2 ? v7_bidx(col, g.n2, L::NE) : 2 * L::NE);
                double c = 0.0, d = 0.0;
#pragma unroll
                for (int k = 0; k < W; ++k) {
                    const d2 f = *(const d2*)(bt + 2 * k);
                    const int wi = 2 * HP - P + e + k;
                    c = fma(f[0], wu[wi], c);
                    d = fma(f[0], wvv[wi], fma(f[1], wu[wi], d));
                }
                cc[e] = c;
                dd[e] = d;
            }
        }
    };
    // ---- axis 0: scatter march plane tt's (c, d) into the rotating slots (qq = tt mod
    // NS, folded by the unroll); returns the finished output plane's A x (plane tt - P)
    auto axis0 = [&](int qq, int tt, const double cc[2], const double dd[2], double vo[2]) {
        const int jrow = (g.g0 + z0 - P + tt + P) * W;
#pragma unroll
        for (int s = 0; s < W; ++s) {
            const int slot = (qq - P + s + NS) % NS;
            const double ka = a0t[jrow + s];
            const double kb = b0t[jrow + s];
#pragma unroll
            for (int e = 0; e < 2; ++e) acc[slot][e] = fma(ka, cc[e], fma(kb, dd[e], acc[slot][e]));
        }
        const int done = (qq - P + NS) % NS;
        vo[0] = acc[done][0];
        vo[1] = acc[done][1];
        acc[done][0] = 0.0;
        acc[done][1] = 0.0;
    };
    // ---- epilogue of output plane zo (march plane tt = zo - z0 + 2P): x_in the x at the
    // output point, bv b there
    auto epilogue = [&](int tt, const double vo[2], const d2 xin, const d2 bv) {
        const bool en = tt >= 2 * P;
        const int zo = zo_of(tt);
        const bool ok0 = en && okrc0, ok1 = en && okrc1;
        double outv[2];
        if constexpr (EPI == EPI_APPLY) {
            outv[0] = vo[0];
            outv[1] = vo[1];
        } else if constexpr (APD) {
            outv[0] = vo[0];
            outv[1] = vo[1];
            dotp = ok0 ? fma(xin[0], vo[0], dotp) : dotp;
            dotp = ok1 ? fma(xin[1], vo[1], dotp) : dotp;
        } else if constexpr (EPI == EPI_RESID) {
            outv[0] = bv[0] - vo[0];
            outv[1] = bv[1] - vo[1];
        } else if constexpr (J0) {
            // x1 = s b, x2 = x1 + s (b - A x1) = x1 + (x1 - s A x1); xin = x1 at the output point
            const int m = g.g0 + zo;
            const bool tp = m >= tc.lo0 && m < tc.hi0;
            double so[2];
            if (fast1 && tp) {
                const d2 scl = *(const d2*)(lds + L::BRING + L::UVQ + 2 * fl);
                so[0] = scl[0];
                so[1] = scl[1];
            } else {
                const int i0 = (m + P) * W + P;
                const double d0a = tp ? tc.t0a[0] : a0t[i0], d0b = tp ? tc.t0b[0] : b0t[i0];
                so[0] = s_at(d0a, d0b, orow, ocol);
                so[1] = s_at(d0a, d0b, orow, ocol + 1);
            }
            // the two running sums live in LDS (this lane's slot in the unused b ring): the 4
            // VGPRs they would pin across the march are what the build lacks at 128
            d2* jsum = (d2*)(lds + L::BRING + 2 * fl);
            d2 js = *jsum;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const double x1 = xin[e];
                const double dr = fma(-vo[e], so[e], x1);
                outv[e] = x1 + dr;
                const bool oke = e ? ok1 : ok0;
                js[0] = oke ? fma(dr, dr, js[0]) : js[0];   // ||dr_2||^2
                js[1] = oke ? fma(x1, x1, js[1]) : js[1];   // ||x1||^2 = ||dr_1||^2
            }
            *jsum = js;
        } else {
            double rc[2];
            const int gz = g.g0 + zo;
            if (rfast) {
                rc[0] = rc[1] = omega * rdiag0[gz];   // one multiply per plane
            } else if (gz >= tc.lo0 && gz < tc.hi0) {
                rc[0] = rci[0];
                rc[1] = rci[1];
            } else {   // the P planes next to each global end of axis 0
                const int i0 = (gz + P) * W + P;
                const double d0a = a0t[i0], d0b = b0t[i0];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    double X, Y;
                    diag_xy(e, X, Y);
                    rc[e] = omega * rcp_nr(fma(d0a, X, d0b * Y));
                }
            }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const double dr = (bv[e] - vo[e]) * rc[e];   // rc = omega / diag
                outv[e] = xin[e] + dr;
                const bool oke = e ? ok1 : ok0;
                nrm = oke ? fma(dr, dr, nrm) : nrm;
                if constexpr (JDOT) dotp = oke ? fma(outv[e], bv[e], dotp) : dotp;
            }
        }
        // one 16-B store per lane; a second column past n2 (ghost or dead pitch column) is
        // written 0.  The plane offset goes into voffset (gfx950 wait state before a VALU
        // overwrites a >8-B store's data VGPRs; see v5).
        const double o1 = ok1 ? outv[1] : 0.0;
        const int voy = vrc + (zo + g.pd0) * (int)plane8;
        v7_store16<YAUX>(ry, (ok0 || ok1) && (!ARITHONLY || outv[0] == 12345.678) ? voy : (int)0x80000000u,
                         outv[0], o1);
    };

    if constexpr (TB2) {
        // ---- residual / Jacobi: two barriers per plane, b DMA'd into LDS one plane ahead.
        // Iteration t: [wait, barrier] DMA b(t+1), DMA x(t+PFX); stage 1 of x(t) into the
        // single u/v slot; [barrier] stage 2 of plane t, output plane t - P.
        // b: flat output pairs r*OP + j, DMA i moves pairs 64 i .. 64 i + 63 (one per
        // wave, waves < ndb)
        const int nbp = R * OP;
        const bool hasb = wv * 64 < nbp;
        uint32_t bvo;
        {
            const int f = wv * 64 + lane;
            const int r = f / OP, j = f - r * OP;
            const bool ok = f < nbp && r0 + r < g.n1 && c0 + 2 * j < g.n2;
            bvo = ok ? (uint32_t)(((r0 + r + g.pd1) * s1 + g.pd2 + c0 + 2 * j) * 8) : 0x80000000u;
        }
        const int fb = act2 ? ru * OP + jo : 0;   // this lane's output pair in a b slot
        auto dma_b = [&](int tt) {   // b of the output plane of march plane tt (dummy past the march)
            if (!hasb) return;
            const uint32_t so = (uint32_t)(zo_of(tt) + g.pd0) * plane8;
            double* dst = lds + L::BRING + (tt & 1) * L::UVQ + wv * 128;
            v7_dma16<BAUX>(rb, dst, tt < nplanes ? (int)bvo : (int)0x80000000u, so);
        };
        d2 hs[HIST ? P : 1];   // x at the output point, planes t-P .. t-1 (shift register)
#pragma unroll
        for (int i = 0; i < (HIST ? P : 1); ++i) hs[i] = d2{0.0, 0.0};
        __syncthreads();   // boundary tables visible; no DMA in flight yet
        if constexpr (J0) {
#pragma unroll
            for (int e = 0; e < 2; ++e) sc[e] = s_at(tc.t0a[0], tc.t0b[0], max(tc.lo1, 0), ocol + e);
            *(d2*)(lds + L::BRING + 2 * fl) = d2{0.0, 0.0};   // the lane's running sums
            *(d2*)(lds + L::BRING + L::UVQ + 2 * fl) = d2{sc[0], sc[1]};   // and its sc (re-read per plane)
        }
        dma_b(0);
#pragma unroll
        for (int i = 0; i < PFX; ++i) dma_x(i, i);
        for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const int t = tb + q;
                if (t < nplanes) {
                    // x(t) and b(t) landed.  Loads after b(t) (issued first in iteration t-1):
                    // that iteration's x DMAs; after x(t): PFX-1 iterations of b + x DMAs
                    if (hasb) {
                        if (dma2) v7_wait_vm<2>();
                        else v7_wait_vm<1>();
                    } else {
                        if (dma2) v7_wait_vm<2 * (PFX - 1)>();
                        else v7_wait_vm<PFX - 1>();
                    }
                    v7_barrier();
                    dma_b(t + 1);
                    dma_x(t + PFX, (t + PFX) % D);
                    if constexpr (J0) {
                        if (!j0_sc_after(t)) {
                            j0_scale_slot(lds + L::XS + (t % D) * L::SLOT, t);
                            v7_barrier();
                        }
                    }
                    const d2 xc = stage1(lds + L::XS + (t % D) * L::SLOT, lds + L::UV, t);
                    d2 xin = {0.0, 0.0};
                    if constexpr (HIST) {
                        xin = hs[0];
#pragma unroll
                        for (int i = 0; i + 1 < P; ++i) hs[i] = hs[i + 1];
                        hs[P - 1] = xc;
                    }
                    v7_barrier();
                    double cc[2], dd[2], vo[2];
                    axis2(lds + L::UV, cc, dd);
                    axis0(q, t, cc, dd, vo);
                    d2 bv = {0.0, 0.0};
                    if constexpr (HASB) bv = *(const d2*)(lds + L::BRING + (t & 1) * L::UVQ + 2 * fb);
                    epilogue(t, vo, xin, bv);
                }
            }
        }
        if constexpr (J0) {
            const d2 js = *(const d2*)(lds + L::BRING + 2 * fl);
            nrm = js[0];
            dotp = js[1];
        }
    } else {
        d2 hx[HIST ? 4 : 1];                // x at the output point, planes t-3 .. t (ring t % 4)
#pragma unroll
        for (int i = 0; i < (HIST ? 4 : 1); ++i) hx[i] = d2{0.0, 0.0};
        __syncthreads();   // boundary tables visible; no DMA in flight yet
#pragma unroll
        for (int i = 0; i < PFX; ++i) dma_x(i, i);

        for (int tb = 0; tb <= nplanes; tb += NS) {
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const int t = tb + q;
                if (t <= nplanes) {
                    // ---- x(t) landed: own DMAs by vmcnt (the loads issued after x(t)'s are
                    // the DMAs of planes t+1 .. t+PFX-1), everyone's by the barrier.  Stores
                    // never count (one may be acknowledged before an older load returns):
                    // vmcnt <= N implies the load has landed.
                    if (dma2) v7_wait_vm<2 * (PFX - 1)>();
                    else v7_wait_vm<PFX - 1>();
                    v7_barrier();
                    dma_x(t + PFX, (q + PFX) % D);

                    // ---- stage 1: u, v of plane t
                    d2 xnew = {0.0, 0.0};
                    if (t < nplanes && !MEMONLY) xnew = stage1(lds + L::XS + (q % D) * L::SLOT, lds + L::UV + (q & 1) * 2 * L::UVQ, t);
                    // the x history: x(t - 4) is the output plane of stage-2 plane t - 1
                    d2 xin = {0.0, 0.0};
                    if constexpr (HIST) {
                        xin = hx[q % 4];
                        hx[q % 4] = xnew;
                    }
                    // (no instruction moves across: stage 1's and stage 2's transients must
                    // not be live at once -- 128 VGPRs at 4 waves per SIMD)
                    __builtin_amdgcn_sched_barrier(0);
                    // ---- stage 2: plane t-1 -- axis 2 from the u/v windows, axis 0, epilogue
                    if constexpr (MEMONLY) {
                        if (t >= 1) {
                            const int zo = zo_of(t - 1);
                            const bool any = t - 1 >= 2 * P && okrc0;
                            v7_store16<YAUX>(ry, any ? vrc + (zo + g.pd0) * (int)plane8 : (int)0x80000000u, 1.0,
                                             okrc1 ? 1.0 : 0.0);
                        }
                    } else if (t >= 1) {
                        const int q2 = (q + NS - 1) % NS;   // (t - 1) mod NS (folded by the unroll)
                        double cc[2], dd[2], vo[2];
                        axis2(lds + L::UV + (q2 & 1) * 2 * L::UVQ, cc, dd);
                        axis0(q2, t - 1, cc, dd, vo);
                        epilogue(t - 1, vo, xin, d2{0.0, 0.0});
                    }
                }
            }
        }
    }
    v7_wait_vm<0>();  // no DMA or load may outlive the workgroup
#undef T2A
#undef T2B
}

template <int P, int EPI, int D, int CN, int CP, bool SAME12, bool JDOT>
__global__ void __launch_bounds__(64 * V7_NW, 1)
kron_v7_kernel(const double* __restrict__ x, double* __restrict__ y, const double* __restrict__ bvec,
               const double* __restrict__ a0t, const double* __restrict__ b0t, const double* __restrict__ a1,
               const double* __restrict__ b1, const double* __restrict__ a2, const double* __restrict__ b2,
               double* __restrict__ partial, double* __restrict__ partial2, const double* __restrict__ rdiag0,
               const KronGeom g, const ToepConst tc, const V7Geom vg, const double omega) {
    typedef V7Lds<P, D, CN> L;
    constexpr int W = L::W;
    __shared__ __attribute__((aligned(16))) double lds[L::N];

    int bid;
    {   // consecutive work items on one XCD (round-robin dispatch over the 8 XCDs)
        const int nblk = gridDim.x;
        const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
        bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
    }
    const int tile = bid % vg.ntiles;
    const int ch = bid / vg.ntiles;

    // boundary coefficient tables (a, b interleaved) of both axes; entry 2P = the
    // Toeplitz row (lanes on interior rows / columns of a boundary tile read it)
    constexpr int NE = L::NE;
    for (int e = threadIdx.x; e < (2 * NE + 1) * W; e += V7_NW * 64) {
        const int i = e / W, k = e - i * W;
        const int r1 = i < NE ? i : g.n1 - 2 * NE + i;
        const int r2 = i < NE ? i : g.n2 - 2 * NE + i;
        const int ct = k < P ? P - k : k - P;
        const bool toe = i == 2 * NE;
        lds[L::BT1 + 2 * e] = toe ? tc.t1a[ct] : a1[(int64_t)r1 * W + k];
        lds[L::BT1 + 2 * e + 1] = toe ? tc.t1b[ct] : b1[(int64_t)r1 * W + k];
        lds[L::BT2 + 2 * e] = toe ? (SAME12 ? tc.t1a[ct] : tc.t2a[ct]) : a2[(int64_t)r2 * W + k];
        lds[L::BT2 + 2 * e + 1] = toe ? (SAME12 ? tc.t1b[ct] : tc.t2b[ct]) : b2[(int64_t)r2 * W + k];
    }
    __syncthreads();   // the tables are read from the body's set-up on (Jacobi's omega/diag)

    double nrm = 0.0, dotp = 0.0;
    const int nwide = vg.nw2 * vg.t1w;
    bool narrow = false;
    if constexpr (CN > 0) narrow = tile >= nwide;
    if (narrow) {
        const int t1 = tile - nwide;
        v7_body<P, EPI, D, (CN > 0 ? CN : V7_CW), CN, CP, SAME12, JDOT>(lds, x, y, bvec, a0t, b0t, rdiag0, g, tc, omega,
                                                                     vg.rn, t1 * vg.rn, vg.nw2 * V7_CW, ch, nrm, dotp);
    } else {
        const int t1 = tile / vg.nw2, t2 = tile - t1 * vg.nw2;
        v7_body<P, EPI, D, V7_CW, CN, CP, SAME12, JDOT>(lds, x, y, bvec, a0t, b0t, rdiag0, g, tc, omega, vg.rw,
                                                      t1 * vg.rw, t2 * V7_CW, ch, nrm, dotp);
    }

    // per-block partial sums (wave butterflies, then the waves in order)
    if constexpr (EPI == EPI_JACOBI || EPI == EPI_APPLYDOT || EPI == EPI_JACOBI0) {
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
        double* red = lds + L::RED;
        if (partial != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nrm += __shfl_xor(nrm, off, 64);
            __syncthreads();
            if (lane == 0) red[wv] = nrm;
            __syncthreads();
            if (threadIdx.x == 0) {
                double s = 0.0;
                for (int w = 0; w < V7_NW; ++w) s += red[w];
                partial[blockIdx.x] = s;
            }
        }
        if (partial2 != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) dotp += __shfl_xor(dotp, off, 64);
            __syncthreads();
            if (lane == 0) red[wv] = dotp;
            __syncthreads();
            if (threadIdx.x == 0) {
                double s = 0.0;
                for (int w = 0; w < V7_NW; ++w) s += red[w];
                partial2[blockIdx.x] = s;
            }
        }
    }
}

// Tile plan for an n1 x n2 plane at degree P: wide tiles of 112 columns, the rest
// (if any) in one narrow column of width CN (a multiple of 16 below 112), rows
// balanced over the tile rows of each type.
static int v7_cn_of(int n2, int* nw2) {
    int w = n2 / V7_CW, rem = n2 - w * V7_CW;
    int cn = rem == 0 ? 0 : ((rem + 15) / 16) * 16;
    if (cn > 96) { ++w; cn = 0; }   // the remainder takes a whole wide tile
    *nw2 = w;
    return cn;
}

static int v7_rows(int n1, int rmax) {
    rmax = std::max(1, std::min(rmax, n1));
    const int nt = (n1 + rmax - 1) / rmax;
    return (n1 + nt - 1) / nt;
}

template <int P>
static int v7_plan_p(int n1, int n2, V7Geom* vg) {
    int nw2 = 0;
    const int cn = v7_cn_of(n2, &nw2);
    vg->nw2 = nw2;
    vg->cn = cn;
    vg->rw = v7_rows(n1, v7_rmax(P, V7_CW));
    vg->t1w = (n1 + vg->rw - 1) / vg->rw;
    if (cn) {
        vg->rn = v7_rows(n1, v7_rmax(P, cn));
        vg->t1n = (n1 + vg->rn - 1) / vg->rn;
    } else {
        vg->rn = vg->t1n = 0;
    }
    vg->ntiles = nw2 * vg->t1w + (cn ? vg->t1n : 0);
    return 0;
}

// Number of (tile, chunk)-independent tiles of a v7 launch over an n1 x n2 plane.
int kron_v7_tiles(int pmax, int n1, int n2) {
    V7Geom vg{};
    if (pmax != 3) return 0;
    v7_plan_p<3>(n1, n2, &vg);
    return vg.ntiles;
}

// dry: only check that the build exists and does not spill (0), else 2 -- the caller
// then runs v5 instead (op_run), as for every other unmet v7 precondition
template <int P, int EPI, int D, int CN, int CP, bool SAME12, bool JDOT>
static int v7_launch_t(const KronPtrs& p, const KronGeom& g, const V7Geom& vg, const ToepConst& tc, double omega,
                       hipStream_t st, bool dry) {
    // hand-counted vmcnt waits: a build that spills to scratch would break them
    static int scratch = -1;
    if (scratch < 0) {
        hipFuncAttributes at{};
        scratch = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&kron_v7_kernel<P, EPI, D, CN, CP, SAME12, JDOT>)) ==
                          hipSuccess
                      ? (int)at.localSizeBytes
                      : (1 << 30);
    }
    if (dry) return scratch > 0 ? 2 : 0;
    if (scratch > 0) {
        set_error("v7: kernel build spills to scratch (vmcnt counting invalid)");
        return 1;
    }
    const int nblk = vg.ntiles * g.nchunks;
    hipLaunchKernelGGL((kron_v7_kernel<P, EPI, D, CN, CP, SAME12, JDOT>), dim3(nblk), dim3(64 * V7_NW), 0, st, p.x,
                       p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, p.rdiag0, g, tc, vg,
                       omega);
    return 0;
}

template <int P, int EPI, int D, int CP, bool SAME12, bool JDOT>
static int v7_launch_cn(const KronPtrs& p, const KronGeom& g, const V7Geom& vg, const ToepConst& tc, double omega,
                        hipStream_t st, bool dry) {
    switch (vg.cn) {
        case 0: return v7_launch_t<P, EPI, D, 0, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 16: return v7_launch_t<P, EPI, D, 16, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 32: return v7_launch_t<P, EPI, D, 32, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 48: return v7_launch_t<P, EPI, D, 48, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 64: return v7_launch_t<P, EPI, D, 64, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 80: return v7_launch_t<P, EPI, D, 80, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
        case 96: return v7_launch_t<P, EPI, D, 96, CP, SAME12, JDOT>(p, g, vg, tc, omega, st, dry);
    }
    set_error("v7: bad narrow tile width");
    return 1;
}

template <int EPI, int CP, bool JDOT>
static int v7_launch_e(bool same, const KronPtrs& p, const KronGeom& g, const V7Geom& vg, const ToepConst& tc,
                       double omega, hipStream_t st, bool dry) {
    return same ? v7_launch_cn<3, EPI, 4, CP, true, JDOT>(p, g, vg, tc, omega, st, dry)
                : v7_launch_cn<3, EPI, 4, CP, false, JDOT>(p, g, vg, tc, omega, st, dry);
}

// Epilogues built: APPLY, RESID, JACOBI (with / without the fused x_out . b), APPLYDOT.
// Cache policy (CP): 4 = non-temporal y stores, 2 = non-temporal b loads (both streamed).
int kron_v7_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, double omega,
                   hipStream_t st, int diag, bool dry) {
    if (pmax != 3) { if (dry) return 2; set_error("v7: p = 3 only"); return 1; }
    V7Geom vg{};
    v7_plan_p<3>(g.n1, g.n2, &vg);
    if (vg.ntiles <= 0) return 0;
    bool same = true;   // axis-1 / axis-2 Toeplitz rows, bitwise
    for (int k = 0; k <= 3; ++k) same = same && tc.t1a[k] == tc.t2a[k] && tc.t1b[k] == tc.t2b[k];
    if (diag) {   // diagnostic / tuning builds (apply): 1 memory only, 2 arithmetic only,
                  // 3 non-temporal x DMAs, 4 y stores with the default policy
        if (epi != EPI_APPLY || diag > 4) { if (dry) return 2; set_error("v7 diag: apply, modes 1-4"); return 1; }
        switch (diag) {
            case 1: return v7_launch_e<EPI_APPLY, 4 | 256, false>(same, p, g, vg, tc, omega, st, dry);
            case 2: return v7_launch_e<EPI_APPLY, 4 | 512, false>(same, p, g, vg, tc, omega, st, dry);
            case 3: return v7_launch_e<EPI_APPLY, 4 | 1, false>(same, p, g, vg, tc, omega, st, dry);
            default: return v7_launch_e<EPI_APPLY, 0, false>(same, p, g, vg, tc, omega, st, dry);
        }
    }
    switch (epi) {
        case EPI_APPLY: return v7_launch_e<EPI_APPLY, 4, false>(same, p, g, vg, tc, omega, st, dry);
        case EPI_RESID: return v7_launch_e<EPI_RESID, 6, false>(same, p, g, vg, tc, omega, st, dry);
        case EPI_JACOBI:
            return p.partial2 ? v7_launch_e<EPI_JACOBI, 6, true>(same, p, g, vg, tc, omega, st)
                              : v7_launch_e<EPI_JACOBI, 6, false>(same, p, g, vg, tc, omega, st, dry);
        case EPI_APPLYDOT: return v7_launch_e<EPI_APPLYDOT, 4, false>(same, p, g, vg, tc, omega, st, dry);
        // (EPI_JACOBI0 compiles -- the body has it -- but spills a few VGPRs in the
        // epilogue of the P planes next to each global end; not built until it fits)
    }
    if (dry) return 2;
    set_error("v7: epilogue not built");
    return 1;
}

int kron_v7_built() { return 1; }

#else   // POMS_V7_STUB: the product library without the v7 kernels

int kron_v7_tiles(int, int, int) { return 0; }

int kron_v7_launch(int, int, const KronPtrs&, const KronGeom&, const ToepConst&, double, hipStream_t, int, bool dry) {
    if (dry) return 2;
    set_error("v7 (variant 11) is not in this build: rebuild with POMS_WITH_V7=1");
    return 1;
}

int kron_v7_built() { return 0; }

#endif

}  // namespace poms
