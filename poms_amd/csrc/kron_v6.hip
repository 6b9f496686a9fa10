// Fused Kronecker-sum operator, v6 (variant 11): 8 waves x R output rows per
// wave, 128-column tiles, x planes DMA'd into an LDS ring, axis 1 first.
//
// What changed against v5 (kron_v5.hip, 16 waves x 1 row) and why
// (profiles/r02/, tools/kernel_bench.py at 515^3 p = 3):
//   * taller tiles: T1 = 8 R rows (24 or 32) instead of 16, so the 2P halo rows
//     every tile re-reads are 6/32 of the tile instead of 6/16 -- the apply's
//     HBM reads were 1.27x the x bytes (PMC) and its memory-only build ran
//     484 us, slower than the 6 TB/s the copy micro-benchmarks reach;
//   * R rows per wave: one barrier per plane for 8 R rows instead of 16, R
//     independent dependency chains per wave, and R + 2P LDS row reads per wave
//     for R rows (v5: 2P + 1 per row).  The arithmetic-only v5 build ran 416 us
//     against ~250 us of issued VALU work: the waves of a workgroup reached
//     their LDS reads, scalar loads and barrier at the same moment;
//   * 512-thread workgroups, 256 VGPRs per lane (two waves per SIMD), one
//     workgroup per CU;
//   * deferred stores: the outputs finished at plane t are stored after the
//     barrier of plane t + 1.  gfx9 counts stores in vmcnt, so a store issued
//     right before the next plane's vmcnt wait is waited for (its ack takes
//     hundreds of cycles); one plane later it has long retired;
//   * b (residual / Jacobi) goes through one slot per wave: each wave DMAs only
//     the rows it consumes, at the end of the previous plane, and waits for them
//     with its own vmcnt (no barrier involved).
// Unchanged from v5: each lane owns two adjacent columns (16-B DMAs / stores),
// the first H and last 128 - H - TO lane-columns are halo, axis 2 windows by
// DPP whole-wave lane shifts, axis 0 scattered into 2P + 1 rotating register
// accumulators, symmetric Toeplitz pair sums inside the interior, per-row /
// per-column band rows outside it, whole-array buffer resources (< 2 GiB),
// out-of-range dummies through voffset, hand-counted vmcnt on LOADS only.
// Preconditions (host): 3D, FORM_SUM, P <= 3, storage pads == P.
#include "common.hpp"

#include <cstdio>
#include <cstdlib>

namespace poms {
namespace v6 {

typedef __attribute__((address_space(3))) void lds_void_t;

template <int AUX = 0>   // cache policy (gfx950: bit 1 = nt, streaming)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, double* lds_dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_dst, 16, voff, (int)soff, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void store16(__amdgpu_buffer_rsrc_t r, int voff, double d0, double d1) {
    u32x4 v;
    const u32x2 a = __builtin_bit_cast(u32x2, d0), b = __builtin_bit_cast(u32x2, d1);
    v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    // plane offset inside voffset, soffset = 0: gfx950 needs a wait state before a
    // VALU overwrites the data VGPRs of a > 8-B store, inserted only with a
    // non-register soffset (kron_v5.hip, tools/diag_v5_fullsize.py)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, AUX);
}
__device__ __forceinline__ double shr1(double v) {  // lane l <- lane l-1 (lane 0 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double shl1(double v) {  // lane l <- lane l+1 (lane 63 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
template <int N>
__device__ __forceinline__ void wait_vm() {  // s_waitcnt vmcnt(N) (gfx9 encoding)
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xc07f); }  // lgkmcnt(0) only
__device__ __forceinline__ void barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}
__device__ __forceinline__ double rcp_nr(double dg) {  // 1/dg: v_rcp_f64 + two Newton steps
    double r = __builtin_amdgcn_rcp(dg);
    double e = fma(-dg, r, 1.0);
    r = fma(r, e, r);
    e = fma(-dg, r, 1.0);
    return fma(r, e, r);
}

}  // namespace v6

// MODE (diagnostic builds, apply only): 1 = memory only (no arithmetic), 2 =
// arithmetic only (no DMA).
// CP: cache policy bits -- 2: b DMAs nt, 4: y stores nt, 8: nt on the x rows no
// other tile reads (x-tile rows 2P .. T1 - 1).
// JDOT: the Jacobi sweep also accumulates x_out . b.
template <int P, int EPI, int NW, int R, int D, int MODE = 0, int CP = 14, bool JDOT = true>
__global__ void __launch_bounds__(NW * 64, 1)
kron_v6_kernel(const double* __restrict__ x, double* __restrict__ y, const double* __restrict__ bvec,
               const double* __restrict__ a0t, const double* __restrict__ b0t,
               const double* __restrict__ a1, const double* __restrict__ b1,
               const double* __restrict__ a2, const double* __restrict__ b2,
               double* __restrict__ partial, double* __restrict__ partial2,
               const double* __restrict__ rdiag0, const double* __restrict__ ab0,
               const KronGeom g, const ToepConst tc, const int H, const double omega) {
    using namespace v6;
    constexpr int W = 2 * P + 1;
    static_assert(NW == 8 || NW == 16, "8 or 16 waves per workgroup");
    constexpr int T1 = NW * R;          // output rows per tile
    constexpr int XR = T1 + 2 * P;      // x rows per plane tile
    // DMA groups per plane: wave w issues rows q = w + NW i, i < NXW; groups i < NXW - 1
    // are all real rows, in the last one row XR carries the plane's axis-0 (A0, M0)
    // pairs and waves past it issue nothing (NXW - 1 DMAs)
    constexpr int NXW = XR / NW + 1;
    constexpr int XRP = XR + 1;         // LDS rows per ring slot (x rows + the coefficient row)
    constexpr int TC = 128;             // columns per tile (2 per lane)
    constexpr int NS = W;               // rotating axis-0 accumulators
    constexpr int PFX = D - 1;          // x prefetch distance (planes)
    constexpr bool HASB = (EPI == EPI_RESID) || (EPI == EPI_JACOBI);
    constexpr bool JAC = (EPI == EPI_JACOBI);
    constexpr bool APD = (EPI == EPI_APPLYDOT);
    constexpr bool HIST = APD || JAC;   // x at the output point from a register history
    constexpr int BAUX = (CP & 2) ? 2 : 0, YAUX = (CP & 4) ? 2 : 0;
    constexpr int NWIN = 2 * P + 2;     // columns 2j-P .. 2j+1+P of a lane's pair
    // loads a wave issues after its x(t) DMAs, before the wait at plane t >= PFX:
    // b rows of planes t-PFX+1 .. t (R each) and x(t+1) .. x(t+PFX-1) (NXW or NXW - 1 each)
    constexpr int WAIT_XF = (HASB ? PFX * R : 0) + (PFX - 1) * NXW;
    constexpr int WAIT_XS = (HASB ? PFX * R : 0) + (PFX - 1) * (NXW - 1);
    static_assert(D >= 2 && WAIT_XF < 64, "ring depth / vmcnt range");
    typedef double d2 __attribute__((ext_vector_type(2)));

    constexpr int XS_OFF = 0;
    constexpr int BS_OFF = XS_OFF + D * XRP * TC;
    constexpr int C2_OFF = BS_OFF + (HASB ? T1 * TC : 0);
    constexpr int RC_OFF = C2_OFF + 2 * W * TC;          // Jacobi: omega/diag per column (Toeplitz rows, planes)
    constexpr int R1_OFF = RC_OFF + (JAC ? TC : 0);      // axis-1 band rows (a, b pairs) of the tile's output rows
    constexpr int RED_OFF = R1_OFF + T1 * W * 2;
    constexpr int LDS_N = RED_OFF + 2 * NW;
    static_assert(LDS_N * 8 <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(16))) double lds[LDS_N];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int nblk = gridDim.x;
    int bid;
    {   // consecutive tiles on one XCD (round-robin dispatch over the 8 XCDs)
        const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
        bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
    }
    const int TO = g.tout;
    // tile order within an XCD's contiguous range: t1 fastest (g.order = 1: the
    // tiles above and below, which read each other's halo rows, run together on one
    // L2) or t2 fastest (0)
    int t1, t2;
    if (g.order) {
        t1 = bid % g.tiles1;
        bid /= g.tiles1;
        t2 = bid % g.tiles2;
        bid /= g.tiles2;
    } else {
        t2 = bid % g.tiles2;
        bid /= g.tiles2;
        t1 = bid % g.tiles1;
        bid /= g.tiles1;
    }
    const int ch = bid;
    const int c0 = t2 * TO;             // lane-column ci <-> interior column c0 - H + ci
    const int r0 = t1 * T1;
    const int orow0 = r0 + wv * R;      // this wave's first output row
    const int cg0 = c0 - H + 2 * lane;  // interior column of this lane's element 0
    // output columns of this lane as a VGPR bit mask (bit e: column e is stored);
    // lane-dependent flags kept as bools would pin two SGPRs each for the whole march
    int cok = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int ci = 2 * lane + e;
        cok |= (ci >= H && ci < H + TO && cg0 + e < g.n2) ? (1 << e) : 0;
    }
    const bool fast2 = (c0 >= tc.lo2) && (min(c0 + TO, g.n2) <= tc.hi2);   // per workgroup

    // axis-1 band rows of the tile's output rows as (a, b) pairs: read by the
    // non-Toeplitz rows with broadcast LDS reads (no SGPRs held across the march)
    for (int e = tid; e < T1 * W; e += NW * 64) {
        const int r = e / W, k = e - r * W;
        const int row = min(r0 + r, g.n1 - 1);
        lds[R1_OFF + 2 * e] = a1[row * W + k];
        lds[R1_OFF + 2 * e + 1] = b1[row * W + k];
    }
    // axis-2 band rows of the tile's columns (only outside the Toeplitz interior)
    if (!fast2) {
        for (int e = tid; e < W * TC; e += NW * 64) {
            const int k = e / TC, ci = e - k * TC;
            const int col = min(max(c0 - H + ci, 0), g.n2 - 1);
            lds[C2_OFF + e] = a2[col * W + k];
            lds[C2_OFF + W * TC + e] = b2[col * W + k];
        }
        if constexpr (JAC) {   // omega / diag(A) on Toeplitz rows and planes, per column
            if (tid < TC) {
                const int col = min(max(c0 - H + tid, 0), g.n2 - 1);
                const double d2a = a2[col * W + P], d2b = b2[col * W + P];
                const double X = tc.t1a[0] * d2a, Y = fma(tc.t1b[0], d2a, tc.t1a[0] * d2b);
                lds[RC_OFF + tid] = omega * rcp_nr(fma(tc.t0a[0], X, tc.t0b[0] * Y));
            }
        }
    }

    int z0, z1;
    chunk_planes(g, ch, z0, z1);
    const int nplanes = (z1 - z0) + 2 * P;
    const int nsp = g.n0 + 2 * g.pd0;
    const int s1 = (int)g.s1;
    const uint32_t arr_bytes = (uint32_t)((int64_t)nsp * g.s0 * 8);
    const uint32_t plane8 = (uint32_t)(g.s0 * 8);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, arr_bytes);
    const __amdgpu_buffer_rsrc_t rbv = make_rsrc(bvec, HASB ? arr_bytes : 0u);
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, arr_bytes);
    // axis-0 band coefficients, (A0, M0) pairs per global plane j at pair row j + 2P
    const __amdgpu_buffer_rsrc_t rab = make_rsrc(ab0, (uint32_t)((g.g0 + g.n0 + 3 * P) * W * 16));
    auto zo_of = [&](int t) { return max(z0 - 2 * P + t, z0); };
    const int colb = (c0 - H + P) * 8 + 16 * lane;   // storage column byte offset (pads == P)

    // ---- LDS-DMA issue.  x-tile row q = storage row r0 + q; wave w issues rows
    // q = w + NW i (i < NXW; see NXW).  Everything wave-dependent is recomputed from
    // an opaque copy of the wave index per plane, so no per-row flags or LDS
    // addresses stay live in SGPRs across the march.
    static_assert(NW * (NXW - 1) <= XR && XR < NW * NXW, "DMA groups");
    const bool full = wv + NW * (NXW - 1) <= XR;   // this wave issues NXW DMAs per plane
    auto dma_x = [&](int m, int slot) {
        if constexpr (MODE == 2) return;
        int w = wv;
        __asm__ volatile("" : "+s"(w));
        const int sp = m + g.pd0;
        const bool ok = sp >= 0 && sp < nsp;
        const uint32_t so = ok ? (uint32_t)sp * plane8 : 0u;
        const int vx = (r0 + w) * s1 * 8 + colb;
#pragma unroll
        for (int i = 0; i < NXW - 1; ++i) {
            double* dst = lds + XS_OFF + (slot * XRP + w + NW * i) * TC;
            const int vo = ok ? vx + NW * i * s1 * 8 : 0x7ffffff0;
            // rows 1 <= i < NXW - 1 lie in [NW, T1): no neighbouring tile reads them
            if ((CP & 8) && i >= 1) dma16<2>(rx, dst, vo, so);
            else dma16<0>(rx, dst, vo, so);
        }
        const int q = w + NW * (NXW - 1);
        double* dst = lds + XS_OFF + (slot * XRP + q) * TC;
        if (q > XR) return;
        const bool real = q < XR, coef = q == XR;
        const int vo = !ok ? 0x7ffffff0 : real ? vx + NW * (NXW - 1) * s1 * 8 : coef ? 16 * lane : 0x7ffffff0;
        // (soffset is not range-checked: 0 for the out-of-range dummies)
        // the coefficient window starts at plane m - P (pair row g0 + m + P): plane m's pairs
        // at pair P W, the output plane m - P's at pair 0 (its diagonal at pair P)
        const uint32_t sl = !ok ? 0u : real ? so : coef ? (uint32_t)((g.g0 + m + P) * W * 16) : 0u;
        dma16<0>(coef ? rab : rx, dst, vo, sl);
    };
    auto dma_b = [&](int zo) {   // this wave's R output rows of b at plane zo
        const uint32_t so = (uint32_t)(zo + g.pd0) * plane8;
#pragma unroll
        for (int j = 0; j < R; ++j)
            dma16<BAUX>(rbv, lds + BS_OFF + (wv * R + j) * TC, (orow0 + j + P) * s1 * 8 + colb, so);
    };

    double acc[NS][R][2];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < R; ++j) { acc[s][j][0] = 0.0; acc[s][j][1] = 0.0; }
    double hist[HIST ? P : 1][R][2];
#pragma unroll
    for (int i = 0; i < (HIST ? P : 1); ++i)
#pragma unroll
        for (int j = 0; j < R; ++j) { hist[i][j][0] = 0.0; hist[i][j][1] = 0.0; }
    double pend[R][2];       // outputs of the last finished plane, stored after the next barrier
    int pend_off[R];
    bool pend_on = false;
#pragma unroll
    for (int j = 0; j < R; ++j) { pend[j][0] = pend[j][1] = 0.0; pend_off[j] = 0x7ffffff0; }
    double nrm = 0.0, dotp = 0.0;

    __syncthreads();  // C2 / RC tables visible; no DMA in flight yet

#pragma unroll
    for (int i = 0; i < PFX; ++i) dma_x(i < nplanes ? z0 - P + i : -(1 << 20), i);
    if constexpr (HASB) dma_b(zo_of(0));

    for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nplanes) {
                // ---- x(t) landed: own DMAs by vmcnt (loads only), everyone's by the barrier
                if (t < PFX) wait_vm<0>();
                else if (full) wait_vm<WAIT_XF>();
                else wait_vm<WAIT_XS>();
                barrier();
                dma_x(t + PFX < nplanes ? z0 - P + t + PFX : -(1 << 20), (t + PFX) % D);
                if (pend_on) {   // deferred stores of the plane finished last iteration
#pragma unroll
                    for (int j = 0; j < R; ++j) store16<YAUX>(ry, pend_off[j], pend[j][0], pend[j][1]);
                }

                // row flags of this wave, recomputed per plane from an opaque row index
                int orw = orow0;
                __asm__ volatile("" : "+s"(orw));
                bool allfast1 = true;
#pragma unroll
                for (int j = 0; j < R; ++j)
                    allfast1 = allfast1 && ((orw + j >= tc.lo1 && orw + j < tc.hi1) || orw + j >= g.n1);
                // ---- x rows of this wave's R output rows (R + 2P LDS rows, 2 columns per lane)
                const double* xs = lds + XS_OFF + (t % D) * XRP * TC + 2 * lane + wv * R * TC;
                d2 xv[R + 2 * P];
#pragma unroll
                for (int k = 0; k < R + 2 * P; ++k) xv[k] = *(const d2*)(xs + k * TC);
                // axis-0 coefficients of x plane m: broadcast reads of the slot's coefficient row
                const double* kab = lds + XS_OFF + ((t % D) * XRP + XR) * TC;
                double ka[W], kb[W];
#pragma unroll
                for (int s = 0; s < W; ++s) {
                    const d2 kk = *(const d2*)(kab + 2 * (P * W + s));
                    ka[s] = kk[0];
                    kb[s] = kk[1];
                }
                if constexpr (MODE == 1) {   // memory only: forward the centre taps
#pragma unroll
                    for (int j = 0; j < R; ++j) { acc[q][j][0] = xv[j + P][0]; acc[q][j][1] = xv[j + P][1]; }
                }

#pragma unroll
                for (int j = 0; j < R; ++j) {
                    if constexpr (MODE == 1) continue;
                    // ---- axis 1: u = F1a x, v = F1b x on row orow0 + j
                    double u[2], v[2];
                    if (allfast1 || (orw + j >= tc.lo1 && orw + j < tc.hi1)) {
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            double pr[P + 1];
                            pr[0] = xv[j + P][e];
#pragma unroll
                            for (int k = 1; k <= P; ++k) pr[k] = xv[j + P - k][e] + xv[j + P + k][e];
                            double su = tc.t1a[0] * pr[0], sv = tc.t1b[0] * pr[0];
#pragma unroll
                            for (int k = 1; k <= P; ++k) {
                                su = fma(tc.t1a[k], pr[k], su);
                                sv = fma(tc.t1b[k], pr[k], sv);
                            }
                            u[e] = su;
                            v[e] = sv;
                        }
                    } else {   // band row from LDS (broadcast reads)
                        const double* rw = lds + R1_OFF + (wv * R + j) * W * 2;
                        d2 f = *(const d2*)rw;
                        double su[2], sv[2];
#pragma unroll
                        for (int e = 0; e < 2; ++e) { su[e] = f[0] * xv[j][e]; sv[e] = f[1] * xv[j][e]; }
#pragma unroll
                        for (int k = 1; k < W; ++k) {
                            f = *(const d2*)(rw + 2 * k);
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                su[e] = fma(f[0], xv[j + k][e], su[e]);
                                sv[e] = fma(f[1], xv[j + k][e], sv[e]);
                            }
                        }
                        u[0] = su[0]; u[1] = su[1];
                        v[0] = sv[0]; v[1] = sv[1];
                    }
                    // ---- axis 2: column windows by whole-lane DPP shifts (2 columns per lane)
                    double wu[NWIN], wvv[NWIN];
                    wu[P] = u[0];
                    wu[P + 1] = u[1];
                    wvv[P] = v[0];
                    wvv[P + 1] = v[1];
#pragma unroll
                    for (int i = P - 1; i >= 0; --i) {
                        wu[i] = shr1(wu[i + 2]);
                        wvv[i] = shr1(wvv[i + 2]);
                    }
#pragma unroll
                    for (int i = P + 2; i <= 2 * P + 1; ++i) {
                        wu[i] = shl1(wu[i - 2]);
                        wvv[i] = shl1(wvv[i - 2]);
                    }
                    double cc[2], dd[2];
                    if (fast2) {
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            double pu[P + 1], pv[P + 1];
                            pu[0] = wu[e + P];
                            pv[0] = wvv[e + P];
#pragma unroll
                            for (int k = 1; k <= P; ++k) {
                                pu[k] = wu[e + P - k] + wu[e + P + k];
                                pv[k] = wvv[e + P - k] + wvv[e + P + k];
                            }
                            double c = tc.t2a[0] * pu[0];
                            double d = fma(tc.t2a[0], pv[0], tc.t2b[0] * pu[0]);
#pragma unroll
                            for (int k = 1; k <= P; ++k) {
                                c = fma(tc.t2a[k], pu[k], c);
                                d = fma(tc.t2a[k], pv[k], fma(tc.t2b[k], pu[k], d));
                            }
                            cc[e] = c;
                            dd[e] = d;
                        }
                    } else {
                        double c[2] = {0.0, 0.0}, d[2] = {0.0, 0.0};
#pragma unroll
                        for (int k = 0; k < W; ++k) {
                            const d2 fa = *(const d2*)(lds + C2_OFF + k * TC + 2 * lane);
                            const d2 fb = *(const d2*)(lds + C2_OFF + (W + k) * TC + 2 * lane);
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                c[e] = fma(fa[e], wu[e + k], c[e]);
                                d[e] = fma(fa[e], wvv[e + k], fma(fb[e], wu[e + k], d[e]));
                            }
                        }
                        cc[0] = c[0]; cc[1] = c[1];
                        dd[0] = d[0]; dd[1] = d[1];
                    }
                    // ---- axis 0: scatter into the rotating slots
#pragma unroll
                    for (int s = 0; s < W; ++s) {
                        const int slot = (q - P + s + NS) % NS;
#pragma unroll
                        for (int e = 0; e < 2; ++e)
                            acc[slot][j][e] = fma(ka[s], cc[e], fma(kb[s], dd[e], acc[slot][j][e]));
                    }
                }

                const int done = (MODE == 1) ? q : (q + P + 1) % NS;
                const bool en = t >= 2 * P;
                const int zo = zo_of(t);
                const int m_out = g.g0 + zo;   // global plane of the finished output plane

                // ---- epilogue of the finished plane zo (R rows)
                d2 bv[R];
                if constexpr (HASB) {
                    // b(zo): only x(t+PFX) was issued after it
                    if (full) wait_vm<NXW>();
                    else wait_vm<NXW - 1>();
#pragma unroll
                    for (int j = 0; j < R; ++j) bv[j] = *(const d2*)(lds + BS_OFF + (wv * R + j) * TC + 2 * lane);
                }
                pend_on = en;
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    double vo[2] = {acc[done][j][0], acc[done][j][1]};
                    acc[done][j][0] = 0.0;
                    acc[done][j][1] = 0.0;
                    double xin[2] = {0.0, 0.0};
                    if constexpr (HIST) {
                        xin[0] = hist[0][j][0];
                        xin[1] = hist[0][j][1];
#pragma unroll
                        for (int i = 0; i + 1 < P; ++i) { hist[i][j][0] = hist[i + 1][j][0]; hist[i][j][1] = hist[i + 1][j][1]; }
                        hist[P - 1][j][0] = xv[j + P][0];
                        hist[P - 1][j][1] = xv[j + P][1];
                    }
                    bool ok[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) ok[e] = en && (orw + j < g.n1) && ((cok >> e) & 1);
                    double outv[2];
                    if constexpr (EPI == EPI_APPLY) {
                        outv[0] = vo[0];
                        outv[1] = vo[1];
                    } else if constexpr (APD) {
                        outv[0] = vo[0];
                        outv[1] = vo[1];
#pragma unroll
                        for (int e = 0; e < 2; ++e) dotp = ok[e] ? fma(xin[e], outv[e], dotp) : dotp;
                    } else if constexpr (EPI == EPI_RESID) {
                        outv[0] = bv[j][0] - vo[0];
                        outv[1] = bv[j][1] - vo[1];
                    } else {   // Jacobi: x_out = x_in + (b - A x) omega / diag
                        double rc[2];
                        const bool tp0 = m_out >= tc.lo0 && m_out < tc.hi0;
                        const bool f1 = allfast1 || (orw + j >= tc.lo1 && orw + j < tc.hi1);
                        if (f1 && fast2 && rdiag0 != nullptr) {
                            rc[0] = rc[1] = omega * rdiag0[m_out];   // one multiply per plane
                        } else if (f1 && tp0 && !fast2) {
                            const d2 rr = *(const d2*)(lds + RC_OFF + 2 * lane);
                            rc[0] = rr[0];
                            rc[1] = rr[1];
                        } else {   // boundary rows / planes: the diagonal from the band centres
                            const d2 d0 = *(const d2*)(kab + 2 * P);   // output plane's axis-0 centre pair
                            const d2 d1 = *(const d2*)(lds + R1_OFF + ((wv * R + j) * W + P) * 2);
                            const double d0a = d0[0], d0b = d0[1], d1a = d1[0], d1b = d1[1];
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                const double d2a = fast2 ? tc.t2a[0] : lds[C2_OFF + P * TC + 2 * lane + e];
                                const double d2b = fast2 ? tc.t2b[0] : lds[C2_OFF + (W + P) * TC + 2 * lane + e];
                                const double X = d1a * d2a, Y = fma(d1b, d2a, d1a * d2b);
                                rc[e] = omega * rcp_nr(fma(d0a, X, d0b * Y));
                            }
                        }
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const double dr = (bv[j][e] - vo[e]) * rc[e];
                            outv[e] = xin[e] + dr;
                            nrm = ok[e] ? fma(dr, dr, nrm) : nrm;
                            if constexpr (JDOT) dotp = ok[e] ? fma(outv[e], bv[j][e], dotp) : dotp;
                        }
                    }
                    // a lane whose second column lies past n2 (ghost / dead pitch column)
                    // writes 0 there, which keeps ghosts zero
                    const bool any = (ok[0] || ok[1]) && (MODE != 2 || outv[0] == 12345.678);
                    pend[j][0] = outv[0];
                    pend[j][1] = ok[1] ? outv[1] : 0.0;
                    pend_off[j] = any ? (orw + j + P) * s1 * 8 + colb + (zo + g.pd0) * (int)plane8 : 0x7ffffff0;
                }
                if constexpr (HASB) {
                    wait_lgkm0();   // this wave's b rows read before they are overwritten
                    dma_b(zo_of(t + 1));
                }
            }
        }
    }
    if (pend_on) {
#pragma unroll
        for (int j = 0; j < R; ++j) store16<YAUX>(ry, pend_off[j], pend[j][0], pend[j][1]);
    }
    wait_vm<0>();  // no LDS-DMA may outlive the workgroup

    if constexpr (JAC || APD) {
        if (partial != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nrm += __shfl_xor(nrm, off, 64);
            __syncthreads();
            if (lane == 0) lds[RED_OFF + wv] = nrm;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < NW; ++w) s += lds[RED_OFF + w];
                partial[blockIdx.x] = s;
            }
        }
        if (partial2 != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) dotp += __shfl_xor(dotp, off, 64);
            __syncthreads();
            if (lane == 0) lds[RED_OFF + NW + wv] = dotp;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < NW; ++w) s += lds[RED_OFF + NW + w];
                partial2[blockIdx.x] = s;
            }
        }
    }
}

template <int P, int EPI, int NW, int R, int D, int MODE = 0, int CP = 14, bool JDOT = true>
static int v6_launch_t(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    // the hand-counted vmcnt waits assume the only VMEM ops in the loop are the
    // DMAs and the stores: a build that spills to scratch would break them
    static int scratch = -1;
    if (scratch < 0) {
        hipFuncAttributes at{};
        if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&kron_v6_kernel<P, EPI, NW, R, D, MODE, CP, JDOT>)) != hipSuccess) {
            set_error("v6: hipFuncGetAttributes failed");
            return 1;
        }
        scratch = (int)at.localSizeBytes;
    }
    if (scratch > 0) {
        set_error("v6: kernel build spills to scratch (vmcnt counting invalid)");
        return 1;
    }
    if (!p.ab0) { set_error("v6: no interleaved axis-0 coefficients"); return 1; }
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    hipLaunchKernelGGL((kron_v6_kernel<P, EPI, NW, R, D, MODE, CP, JDOT>), dim3(nblk), dim3(NW * 64), 0, st, p.x, p.y,
                       p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, p.rdiag0, p.ab0, g, tc, H,
                       omega);
    return 0;
}

// Workgroup shape (waves NW x rows per wave R; the tile height is NW R) of each
// epilogue.  POMS_V6_CFG<epi>=<NW>x<R> overrides it for tuning runs.
struct V6Cfg { int nw, r; };
static V6Cfg v6_cfg_default(int epi) {
    switch (epi) {
        case EPI_APPLY: return {8, 4};
        default: return {8, 2};
    }
}
static V6Cfg v6_cfg(int epi) {
    static V6Cfg cfg[8] = {};
    if (epi < 0 || epi > 7) return {8, 2};
    if (!cfg[epi].nw) {
        char name[32];
        snprintf(name, sizeof name, "POMS_V6_CFG%d", epi);
        const char* e = getenv(name);
        int nw = 0, r = 0;
        if (e && sscanf(e, "%dx%d", &nw, &r) == 2 && (nw == 8 || nw == 16) && r >= 1 && r <= 4)
            cfg[epi] = {nw, r};
        else
            cfg[epi] = v6_cfg_default(epi);
    }
    return cfg[epi];
}
int kron_v6_rows(int pmax, int epi) {
    (void)pmax;
    const V6Cfg c = v6_cfg(epi);
    return c.nw * c.r;   // the tile height
}

template <int P, int EPI, int MODE = 0, int CP = 14, bool JDOT = true>
static int v6_launch_c(V6Cfg c, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    constexpr bool HASB = EPI == EPI_RESID || EPI == EPI_JACOBI;
    if (c.nw == 16 && c.r == 2) return v6_launch_t<P, EPI, 16, 2, HASB ? 2 : 3, MODE, CP, JDOT>(p, g, tc, H, omega, st);
    if (c.nw == 16 && c.r == 1) return v6_launch_t<P, EPI, 16, 1, 3, MODE, CP, JDOT>(p, g, tc, H, omega, st);
    if (c.nw == 8 && c.r == 2) return v6_launch_t<P, EPI, 8, 2, 3, MODE, CP, JDOT>(p, g, tc, H, omega, st);
    if (c.nw == 8 && c.r == 3) return v6_launch_t<P, EPI, 8, 3, 3, MODE, CP, JDOT>(p, g, tc, H, omega, st);
    if constexpr (!HASB)   // the b slot beside a 4-row ring exceeds the LDS
        if (c.nw == 8 && c.r == 4) return v6_launch_t<P, EPI, 8, 4, 3, MODE, CP, JDOT>(p, g, tc, H, omega, st);
    set_error("v6: workgroup shape not built");
    return 1;
}

template <int P>
static int v6_launch_p(int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    const V6Cfg c = v6_cfg(epi);
    switch (epi) {
        case EPI_APPLY: return v6_launch_c<P, EPI_APPLY>(c, p, g, tc, H, omega, st);
        case EPI_RESID: return v6_launch_c<P, EPI_RESID>(c, p, g, tc, H, omega, st);
        case EPI_JACOBI:
            return p.partial2 == nullptr ? v6_launch_c<P, EPI_JACOBI, 0, 14, false>(c, p, g, tc, H, omega, st)
                                         : v6_launch_c<P, EPI_JACOBI>(c, p, g, tc, H, omega, st);
        case EPI_APPLYDOT: return v6_launch_c<P, EPI_APPLYDOT>(c, p, g, tc, H, omega, st);
    }
    set_error("v6: epilogue not built");
    return 1;
}

int kron_v6_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H,
                   double omega, hipStream_t st, int diag_mode) {
    if (H < pmax || (H & 1) || (g.tout & 1) || H + g.tout + pmax > 128) {
        set_error("v6: bad tile geometry");
        return 1;
    }
    if (g.tiles1 * kron_v6_rows(pmax, epi) < g.n1) {
        set_error("v6: row tiles do not cover the rows");
        return 1;
    }
    if (diag_mode) {   // DIAGNOSTIC builds (apply, p = 3): 1 = memory only, 2 = arithmetic only
        if (pmax != 3 || epi != EPI_APPLY || diag_mode > 2) { set_error("v6 diag mode: apply, p = 3, mode 1/2"); return 1; }
        const V6Cfg c = v6_cfg(epi);
        return diag_mode == 1 ? v6_launch_c<3, EPI_APPLY, 1>(c, p, g, tc, H, omega, st)
                              : v6_launch_c<3, EPI_APPLY, 2>(c, p, g, tc, H, omega, st);
    }
    switch (pmax) {
        case 1: return v6_launch_p<1>(epi, p, g, tc, H, omega, st);
        case 2: return v6_launch_p<2>(epi, p, g, tc, H, omega, st);
        case 3: return v6_launch_p<3>(epi, p, g, tc, H, omega, st);
    }
    set_error("v6: pmax must be in 1..3");
    return 1;
}

}  // namespace poms
