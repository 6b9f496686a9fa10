// Fused Kronecker(-sum) operator, v4 (variant 7): axis-1-first sum
// factorisation over x planes staged in LDS by buffer_load ... lds.
//
// Why this shape (measured on v3 at 515^3, p = 3): a copy of v3's access
// pattern without arithmetic ran 558 us and its arithmetic without memory
// 548 us -- both halves had to shrink.
//   * memory: each x plane tile (rows r0-P .. r0+T1+P, 64 columns) is DMA'd
//     straight into a 3-deep LDS ring two planes ahead (no VGPR staging, ~2x
//     the bytes in flight of v3's register prefetch); b (residual / Jacobi)
//     goes through a 2-deep ring the same way.  All loads in the loop are
//     LDS-DMA, so the vmcnt waits are counted by hand (one barrier per plane).
//   * arithmetic: axis 1 goes FIRST (u = F1a x, v = F1b x) on the lane's own
//     output row only -- the 2P halo rows are read from LDS but never
//     computed on -- then axis 2 (c = F2a u, d = F2a v + F2b u) with the
//     column neighbours exchanged through a wave-private LDS slot (no DPP,
//     no barrier), then the axis-0 march into 2P+1 rotating accumulators.
//     Each lane holds TWO adjacent columns (a wave = 2 rows x 64 columns),
//     and the uniform-knot interior uses symmetric Toeplitz pair sums
//     (p + 1 multiplies instead of 2p + 1).  Boundary rows / columns of the
//     1D factors take a per-lane coefficient path chosen per workgroup.
//   * Jacobi: inside the Toeplitz interior diag(A) is constant on a plane,
//     so 1/diag is formed once per plane; x_in of the output plane is kept
//     in a P+1 deep register history of the lane's centre tap.
// Preconditions (checked by the host): storage pads == P on every used axis.
#include "common.hpp"

namespace poms {

typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, double* lds_dst, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds_dst, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ double v4_shr1(double v) {  // lane l <- lane l-1
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double v4_shl1(double v) {  // lane l <- lane l+1
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}

// s_waitcnt vmcnt(N) only (gfx9 encoding: vmcnt[3:0], expcnt[6:4], lgkmcnt[11:8], vmcnt[5:4] at [15:14])
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int P, int NW, bool IS3D, int FORM, int EPI, int MODE = 0, bool EXDPP = true, int MINW = (2 * NW * 64) / 256, int DFORCE = 0>
__global__ void __launch_bounds__(NW * 64, MINW)
kron_v4_kernel(const double* __restrict__ x, double* __restrict__ y,
               const double* __restrict__ bvec,
               const double* __restrict__ a0t, const double* __restrict__ b0t,
               const double* __restrict__ a1, const double* __restrict__ b1,
               const double* __restrict__ a2, const double* __restrict__ b2,
               double* __restrict__ partial, double* __restrict__ partial2, const KronGeom g,
               const ToepConst tc, const double omega) {
    constexpr int W = 2 * P + 1;
    constexpr int NT = NW * 64;
    const int TO = g.tout;                 // output columns per tile
    constexpr int T1 = 2 * NW;          // output rows per tile (one per half-wave)
    constexpr int XR = T1 + 2 * P;      // x rows per plane tile
    constexpr bool SUM = (FORM == FORM_SUM);
    constexpr bool HASB = (EPI != EPI_APPLY);
    // Jacobi (3D) also DMAs x_in of the output plane next to b (no register
    // history) and pays for that LDS with a 2-deep x ring.
    constexpr bool XIN = (EPI == EPI_JACOBI) && IS3D;
    // x ring depth: apply 4 (3 planes in flight); with a b ring the b DMA of the
    // next plane anchors the wait, so 3 is all the depth that can be used
    constexpr int D = IS3D ? (DFORCE ? DFORCE : (HASB ? 3 : 4)) : 1;
    constexpr int PFX = D - 1;                      // x prefetch distance (planes)
    constexpr int DB = IS3D ? 2 : 1;               // b ring depth
    constexpr int BSLOT = (XIN ? 2 : 1) * T1 * 64; // b rows (+ x_in rows)
    constexpr int NS = IS3D ? W : 1;
    constexpr int NWIN = 2 * P + 2;     // columns 2j-P .. 2j+1+P of a lane's pair
    static_assert(P <= NW, "extra DMA pairs are issued by waves 0..P-1");
    typedef double d2 __attribute__((ext_vector_type(2)));

    // one LDS object, carved by hand (LDS-DMA destinations must be exact)
    constexpr int XS_OFF = 0;
    constexpr int BS_OFF = XS_OFF + D * XR * 64;
    constexpr int EX_OFF = BS_OFF + (HASB ? DB * BSLOT : 0) + (EXDPP ? 0 : 8);   // guard for lane-a reads
    constexpr int C1_OFF = EX_OFF + (EXDPP ? 0 : NW * 128 + 8);
    constexpr int C2_OFF = C1_OFF + 2 * T1 * W;
    constexpr int RED_OFF = C2_OFF + 2 * 64 * W;
    constexpr int LDS_N = RED_OFF + NW;
    __shared__ double lds[LDS_N];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int h = lane >> 5;
    const int j = lane & 31;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int nblk = gridDim.x;
    int bid;
    {
        const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
        bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
    }
    const int t2 = bid % g.tiles2;
    bid /= g.tiles2;
    const int t1 = bid % g.tiles1;
    const int ch = bid / g.tiles1;
    const int c0 = t2 * TO;            // tile column ci <-> global column c0 - P + ci
    const int r0 = t1 * T1;
    const int rl = 2 * wv + h;         // this lane's output row in the tile
    const int orow = r0 + rl;
    const bool row_ok = orow < g.n1;
    const int cg0 = c0 - P + 2 * j;    // global column of element 0
    bool col_ok[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int ci = 2 * j + e;
        col_ok[e] = ci >= P && ci < P + TO && cg0 + e < g.n2;
    }
    const bool fast1 = (r0 >= tc.lo1) && (min(r0 + T1, g.n1) <= tc.hi1);
    const bool fast2 = (c0 >= tc.lo2) && (min(c0 + TO, g.n2) <= tc.hi2);

    // boundary tables (indexed through `lds` directly so every access stays a ds_* op):
    // C1: [T1][W] F1a rows, then [T1][W] F1b rows; C2: [64][W] F2a rows, then [64][W] F2b rows
    if (!fast1) {
        for (int e = tid; e < T1 * W; e += NT) {
            const int r = e / W, k = e - r * W;
            const int row = min(r0 + r, g.n1 - 1);
            lds[C1_OFF + e] = a1[row * W + k];
            lds[C1_OFF + T1 * W + e] = SUM ? b1[row * W + k] : 0.0;
        }
    }
    if (!fast2) {
        for (int e = tid; e < 64 * W; e += NT) {
            const int ci = e / W, k = e - ci * W;
            const int col = min(max(c0 - P + ci, 0), g.n2 - 1);
            lds[C2_OFF + e] = a2[col * W + k];
            lds[C2_OFF + 64 * W + e] = SUM ? b2[col * W + k] : 0.0;
        }
    }

    int z0 = 0, z1 = 1;
    if constexpr (IS3D) {
        chunk_planes(g, ch, z0, z1);
    }
    const int nplanes = IS3D ? (z1 - z0) + 2 * P : 1;
    const int nsp = g.n0 + 2 * g.pd0;
    const int s1 = (int)g.s1;
    auto zo_of = [&](int t) { return IS3D ? max(z0 - 2 * P + t, z0) : 0; };

    // ---- LDS-DMA issue (counts per wave: x 1 or 2 (waves < P), b 1) ----
    auto dma_x = [&](int m, int slot) {
        if constexpr (MODE == 2 || MODE == 7) return;
        const int sp = IS3D ? m + g.pd0 : 0;
        const bool ok = (sp >= 0) && (sp < nsp);
        const __amdgpu_buffer_rsrc_t rs =
            make_rsrc(x + (int64_t)(ok ? sp : 0) * g.s0, ok ? plane_bytes(nsp - sp, g.s0) : 0u);
        // x-row 2q+h of the tile = storage row r0 + 2q + h (pads == P)
        {
            const int q = wv;
            dma16(rs, lds + XS_OFF + (slot * XR + 2 * q) * 64, ((r0 + 2 * q + h) * s1 + c0 + 2 * j) * 8);
        }
        if (wv < P) {
            const int q = wv + NW;
            dma16(rs, lds + XS_OFF + (slot * XR + 2 * q) * 64, ((r0 + 2 * q + h) * s1 + c0 + 2 * j) * 8);
        }
    };
    auto dma_b = [&](int zo, int slot) {
        if constexpr (MODE == 2 || MODE == 7) return;
        const int sp = zo + g.pd0;
        const bool ok = (sp >= 0) && (sp < nsp);
        const __amdgpu_buffer_rsrc_t rs =
            make_rsrc(bvec + (int64_t)(ok ? sp : 0) * g.s0, ok ? plane_bytes(nsp - sp, g.s0) : 0u);
        dma16(rs, lds + BS_OFF + slot * BSLOT + 2 * wv * 64, ((r0 + rl + P) * s1 + c0 + 2 * j) * 8);
        if constexpr (XIN) {
            const __amdgpu_buffer_rsrc_t rx =
                make_rsrc(x + (int64_t)(ok ? sp : 0) * g.s0, ok ? plane_bytes(nsp - sp, g.s0) : 0u);
            dma16(rx, lds + BS_OFF + slot * BSLOT + (T1 + 2 * wv) * 64, ((r0 + rl + P) * s1 + c0 + 2 * j) * 8);
        }
    };

    // coefficients and diagonal pieces
    auto t1c = [&](int k, bool bb) { return bb ? tc.t1b[k] : tc.t1a[k]; };
    auto t2c = [&](int k, bool bb) { return bb ? tc.t2b[k] : tc.t2a[k]; };

    double acc[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) { acc[s][0] = 0.0; acc[s][1] = 0.0; }
    double nrm = 0.0, dotp = 0.0;

    const int exo = EX_OFF + wv * 128;   // this wave's exchange slot

    __syncthreads();  // c1 / c2 tables visible; no DMA in flight yet

    dma_x(IS3D ? z0 - P : 0, 0);
#pragma unroll
    for (int i = 1; i < PFX; ++i) dma_x(i < nplanes ? z0 - P + i : -(1 << 20), i);
    if constexpr (HASB) dma_b(zo_of(0), 0);

    for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nplanes) {
                // ---- x(t) and b(t) landed (own DMA), then everyone's
                // issue order per iteration: b(t+1) [x_in(t+1)], x(t+PFX), 2 stores
                if constexpr (MODE == 2 || MODE == 7) {
                } else if constexpr (!IS3D) {
                    wait_vm<0>();
                } else if constexpr (HASB) {
                    // Loads return in order but a store may be acknowledged before an
                    // older load returns: count only the LOADS issued after the one
                    // waited for.  After b(t) (issued in iteration t-1): that iteration's x DMAs
                    if (t == 0) wait_vm<0>();
                    else if (wv < P) wait_vm<2>();
                    else wait_vm<1>();
                } else {
                    // after x(t) (issued in iteration t-PFX): (PFX-1) iterations' x DMAs
                    if (t < PFX) wait_vm<0>();
                    else if (wv < P) wait_vm<(PFX - 1) * 2>();
                    else wait_vm<(PFX - 1) * 1>();
                }
                if constexpr (MODE != 4 && MODE != 7) __builtin_amdgcn_s_barrier();
                // ---- prefetch (dummies past the end keep the counts fixed)
                if constexpr (IS3D) {
                    if constexpr (HASB) dma_b(zo_of(t + 1), (t + 1) & 1);
                    dma_x(t + PFX < nplanes ? z0 - P + t + PFX : -(1 << 20), (t + PFX) % D);
                }

                // ---- axis 1 (first): u = F1a x, v = F1b x on this lane's row, 2 columns
                const double* xs = lds + XS_OFF + (IS3D ? (t % D) : 0) * XR * 64 + 2 * j;
                d2 xv[W];
#pragma unroll
                for (int k = 0; k < W; ++k) xv[k] = *(const d2*)(xs + (rl + k) * 64);
                double u[2], v[2];
                if constexpr (MODE == 1 || MODE == 3 || MODE == 4 || MODE == 5 || MODE == 6) {
                    double vo1[2] = {xv[P][0] + xv[0][0] + xv[W - 1][0], xv[P][1] + xv[0][1] + xv[W - 1][1]};
                    const int zo = zo_of(t);
                    const int sp = zo + g.pd0;
                    const __amdgpu_buffer_rsrc_t ys = make_rsrc(y + (int64_t)sp * g.s0, plane_bytes(nsp - sp, g.s0));
                    const int obase = ((orow + P) * s1 + c0 + 2 * j) * 8;
                    const bool en = !IS3D || t >= 2 * P;
                    if constexpr (MODE == 6) {
                        bstore2_p<0>(ys, (en && row_ok && col_ok[1]) ? obase : 0x7ffffff0, vo1[0], vo1[1]);
                        continue;
                    }
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        if constexpr (MODE == 5) {
                            bstore_p<2>(ys, (en && row_ok && col_ok[e]) ? obase + 8 * e : 0x7ffffff0, vo1[e]);
                        } else if (MODE != 3 || vo1[e] == 12345.678) {
                            bstore(ys, (en && row_ok && col_ok[e]) ? obase + 8 * e : 0x7ffffff0, vo1[e]);
                        }
                    }
                    continue;
                }
                if (fast1) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        double pr[P + 1];
                        pr[0] = xv[P][e];
#pragma unroll
                        for (int k = 1; k <= P; ++k) pr[k] = xv[P - k][e] + xv[P + k][e];
                        double su = t1c(0, false) * pr[0];
                        double sv = SUM ? t1c(0, true) * pr[0] : 0.0;
#pragma unroll
                        for (int k = 1; k <= P; ++k) {
                            su = fma(t1c(k, false), pr[k], su);
                            if constexpr (SUM) sv = fma(t1c(k, true), pr[k], sv);
                        }
                        u[e] = su;
                        v[e] = sv;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 2; ++e) { u[e] = 0.0; v[e] = 0.0; }
#pragma unroll
                    for (int k = 0; k < W; ++k) {
                        const double ca = lds[C1_OFF + rl * W + k];
                        const double cb = SUM ? lds[C1_OFF + T1 * W + rl * W + k] : 0.0;
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            u[e] = fma(ca, xv[k][e], u[e]);
                            if constexpr (SUM) v[e] = fma(cb, xv[k][e], v[e]);
                        }
                    }
                }

                // ---- axis 2: column neighbours through the wave-private LDS slot
                auto exchange = [&](double f0, double f1, double* win) {
                    if constexpr (EXDPP) {
                        // wave-wide lane shifts; across the half-wave seam only halo
                        // (non-output) lanes receive the other row's values
                        win[P] = f0;
                        win[P + 1] = f1;
#pragma unroll
                        for (int i = P - 1; i >= 0; --i) win[i] = v4_shr1(win[i + 2]);
#pragma unroll
                        for (int i = P + 2; i <= 2 * P + 1; ++i) win[i] = v4_shl1(win[i - 2]);
                        return;
                    }
                    __builtin_amdgcn_wave_barrier();
                    d2 own;
                    own.x = f0;
                    own.y = f1;
                    *(d2*)(lds + exo + 2 * lane) = own;
                    __builtin_amdgcn_wave_barrier();
                    win[P] = f0;
                    win[P + 1] = f1;
#pragma unroll
                    for (int a = 1; 2 * a - 1 <= P; ++a) {
                        if (P - 2 * a >= 0) {
                            const d2 lv = *(const d2*)(lds + exo + 2 * (lane - a));
                            win[P - 2 * a] = lv.x;
                            win[P - 2 * a + 1] = lv.y;
                        } else {
                            win[P - 2 * a + 1] = lds[exo + 2 * (lane - a) + 1];
                        }
                        if (P + 2 * a + 1 <= 2 * P + 1) {
                            const d2 rv = *(const d2*)(lds + exo + 2 * (lane + a));
                            win[P + 2 * a] = rv.x;
                            win[P + 2 * a + 1] = rv.y;
                        } else {
                            win[P + 2 * a] = lds[exo + 2 * (lane + a)];
                        }
                    }
                };
                double wu[NWIN], wvv[NWIN];
                exchange(u[0], u[1], wu);
                if constexpr (SUM) exchange(v[0], v[1], wvv);
                double cc[2], dd[2];
                if (fast2) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        double pu[P + 1], pv[P + 1];
                        pu[0] = wu[e + P];
                        pv[0] = SUM ? wvv[e + P] : 0.0;
#pragma unroll
                        for (int k = 1; k <= P; ++k) {
                            pu[k] = wu[e + P - k] + wu[e + P + k];
                            if constexpr (SUM) pv[k] = wvv[e + P - k] + wvv[e + P + k];
                        }
                        double c = t2c(0, false) * pu[0];
                        double d = 0.0;
                        if constexpr (SUM) d = IS3D ? fma(t2c(0, false), pv[0], t2c(0, true) * pu[0])
                                                    : t2c(0, true) * pv[0];
#pragma unroll
                        for (int k = 1; k <= P; ++k) {
                            c = fma(t2c(k, false), pu[k], c);
                            if constexpr (SUM) {
                                if constexpr (IS3D) d = fma(t2c(k, false), pv[k], fma(t2c(k, true), pu[k], d));
                                else d = fma(t2c(k, true), pv[k], d);
                            }
                        }
                        cc[e] = c;
                        dd[e] = d;
                    }
                } else {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int cbase = C2_OFF + (2 * j + e) * W;
                        double c = 0.0, d = 0.0;
#pragma unroll
                        for (int k = 0; k < W; ++k) {
                            const double fa = lds[cbase + k];
                            c = fma(fa, wu[e + k], c);
                            if constexpr (SUM) {
                                const double fb = lds[cbase + 64 * W + k];
                                if constexpr (IS3D) d = fma(fa, wvv[e + k], fma(fb, wu[e + k], d));
                                else d = fma(fb, wvv[e + k], d);
                            }
                        }
                        cc[e] = c;
                        dd[e] = d;
                    }
                }

                // ---- axis 0: scatter into the rotating slots; epilogue of the finished plane
                double vo[2];
                bool en = true;
                if constexpr (IS3D) {
                    const int jrow = (g.g0 + z0 - P + t + P) * W;
#pragma unroll
                    for (int s = 0; s < W; ++s) {
                        const int slot = (q - P + s + NS) % NS;
                        const double ka = a0t[jrow + s];
                        const double kb = SUM ? b0t[jrow + s] : 0.0;
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            acc[slot][e] = fma(ka, cc[e], acc[slot][e]);
                            if constexpr (SUM) acc[slot][e] = fma(kb, dd[e], acc[slot][e]);
                        }
                    }
                    const int done = (q + P + 1) % NS;
                    vo[0] = acc[done][0];
                    vo[1] = acc[done][1];
                    acc[done][0] = 0.0;
                    acc[done][1] = 0.0;
                    en = t >= 2 * P;
                } else {
                    vo[0] = SUM ? cc[0] + dd[0] : cc[0];
                    vo[1] = SUM ? cc[1] + dd[1] : cc[1];
                }

                const int zo = zo_of(t);
                const int sp = zo + g.pd0;
                double outv[2];
                if constexpr (EPI == EPI_APPLY) {
                    outv[0] = vo[0];
                    outv[1] = vo[1];
                } else {
                    const int bso = BS_OFF + (IS3D ? (t & 1) : 0) * BSLOT + rl * 64 + 2 * j;
                    const d2 bv = *(const d2*)(lds + bso);
                    if constexpr (EPI == EPI_RESID) {
                        outv[0] = bv.x - vo[0];
                        outv[1] = bv.y - vo[1];
                    } else {
                        double d0a = 1.0, d0b = 0.0;
                        if constexpr (IS3D) {
                            d0a = a0t[(g.g0 + zo + P) * W + P];
                            if constexpr (SUM) d0b = b0t[(g.g0 + zo + P) * W + P];
                        }
                        auto diag_of = [&](double f1a, double f1b, double f2a, double f2b) {
                            if constexpr (SUM) {
                                if constexpr (IS3D) return fma(d0a, f1a * f2a, d0b * fma(f1b, f2a, f1a * f2b));
                                else return fma(f1a, f2a, f1b * f2b);
                            } else {
                                return d0a * f1a * f2a;
                            }
                        };
                        auto recip = [&](double dg) {
                            double rc = __builtin_amdgcn_rcp(dg);
                            double ee = fma(-dg, rc, 1.0);
                            rc = fma(rc, ee, rc);
                            ee = fma(-dg, rc, 1.0);
                            return fma(rc, ee, rc);
                        };
                        double rc[2];
                        if (fast1 && fast2) {
                            const double r = recip(diag_of(tc.t1a[0], tc.t1b[0], tc.t2a[0], tc.t2b[0]));
                            rc[0] = r;
                            rc[1] = r;
                        } else {
                            // tables are read unconditionally (garbage when unused) so that
                            // the selects are on values, not on LDS / kernarg pointers
                            const double l1a = lds[C1_OFF + rl * W + P];
                            const double l1b = lds[C1_OFF + T1 * W + rl * W + P];
                            const double f1a = fast1 ? tc.t1a[0] : l1a;
                            const double f1b = SUM ? (fast1 ? tc.t1b[0] : l1b) : 0.0;
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                const double l2a = lds[C2_OFF + (2 * j + e) * W + P];
                                const double l2b = lds[C2_OFF + 64 * W + (2 * j + e) * W + P];
                                const double f2a = fast2 ? tc.t2a[0] : l2a;
                                const double f2b = SUM ? (fast2 ? tc.t2b[0] : l2b) : 0.0;
                                rc[e] = recip(diag_of(f1a, f1b, f2a, f2b));
                            }
                        }
                        double xin0 = xv[P][0], xin1 = xv[P][1];
                        if constexpr (XIN) {
                            const d2 xi = *(const d2*)(lds + bso + T1 * 64);
                            xin0 = xi.x;
                            xin1 = xi.y;
                        }
                        const double dr0 = omega * (bv.x - vo[0]) * rc[0];
                        const double dr1 = omega * (bv.y - vo[1]) * rc[1];
                        outv[0] = xin0 + dr0;
                        outv[1] = xin1 + dr1;
                        nrm = (en && row_ok && col_ok[0]) ? fma(dr0, dr0, nrm) : nrm;
                        nrm = (en && row_ok && col_ok[1]) ? fma(dr1, dr1, nrm) : nrm;
                        dotp = (en && row_ok && col_ok[0]) ? fma(outv[0], bv.x, dotp) : dotp;
                        dotp = (en && row_ok && col_ok[1]) ? fma(outv[1], bv.y, dotp) : dotp;
                    }
                }
                const __amdgpu_buffer_rsrc_t ys = make_rsrc(y + (int64_t)sp * g.s0, plane_bytes(nsp - sp, g.s0));
                const int obase = ((orow + P) * s1 + c0 + 2 * j) * 8;
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const bool ok = en && row_ok && col_ok[e];
                    if constexpr (MODE == 2 || MODE == 7) {
                        if (outv[e] == 12345.678) bstore(ys, ok ? obase + 8 * e : 0x7ffffff0, outv[e]);
                    } else {
                        bstore(ys, ok ? obase + 8 * e : 0x7ffffff0, outv[e]);
                    }
                }
            }
        }
    }
    wait_vm<0>();  // no LDS-DMA may outlive the workgroup

    if constexpr (EPI == EPI_JACOBI) {
        if (partial != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nrm += __shfl_xor(nrm, off, 64);
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
            if (lane == 0) lds[RED_OFF + wv] = dotp;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < NW; ++w) s += lds[RED_OFF + w];
                partial2[blockIdx.x] = s;
            }
        }
    }
}

template <int P, int NW, bool IS3D, int FORM, int EPI>
static void v4_launch_t(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, double omega,
                        hipStream_t st) {
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    hipLaunchKernelGGL((kron_v4_kernel<P, NW, IS3D, FORM, EPI>), dim3(nblk), dim3(NW * 64), 0, st,
                       p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
}

template <int P, bool IS3D, int FORM>
static int v4_launch_e(int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc,
                       double omega, hipStream_t st) {
    switch (epi) {
        case EPI_APPLY: v4_launch_t<P, 8, IS3D, FORM, EPI_APPLY>(p, g, tc, omega, st); return 0;
        case EPI_RESID: v4_launch_t<P, 8, IS3D, FORM, EPI_RESID>(p, g, tc, omega, st); return 0;
        case EPI_JACOBI: v4_launch_t<P, 8, IS3D, FORM, EPI_JACOBI>(p, g, tc, omega, st); return 0;
    }
    set_error("bad epilogue");
    return 1;
}

template <int P>
static int v4_launch_p(bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                       const ToepConst& tc, double omega, hipStream_t st) {
    if (is3d)
        return form == FORM_SUM ? v4_launch_e<P, true, FORM_SUM>(epi, p, g, tc, omega, st)
                                : v4_launch_e<P, true, FORM_SINGLE>(epi, p, g, tc, omega, st);
    return form == FORM_SUM ? v4_launch_e<P, false, FORM_SUM>(epi, p, g, tc, omega, st)
                            : v4_launch_e<P, false, FORM_SINGLE>(epi, p, g, tc, omega, st);
}

// Tile: 16 rows x (64 - 2P) output columns, 8 waves (2 workgroups per CU).
int kron_v4_launch(int pmax, bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                   const ToepConst& tc, double omega, hipStream_t st, int diag_mode) {
    if (diag_mode) {  // DIAGNOSTIC: 1 = memory only, 2 = arithmetic only (3D SUM P=3 apply)
        if (pmax != 3 || !is3d || form != FORM_SUM || epi != EPI_APPLY) { set_error("diag mode: 3D SUM P=3 apply only"); return 1; }
        const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
        if (diag_mode == 1)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 1>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 3)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 3>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 4)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 4>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 5)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 5>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 8)   // 3 workgroups per CU: 6 waves/SIMD, 3-deep ring
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 0, true, 6, 3>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 9)   // 5 waves/SIMD
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 0, true, 5, 3>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 7)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 7>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else if (diag_mode == 6)
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 6>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        else
            hipLaunchKernelGGL((kron_v4_kernel<3, 8, true, FORM_SUM, EPI_APPLY, 2>), dim3(nblk), dim3(512), 0, st,
                               p.x, p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, g, tc, omega);
        return 0;
    }
    switch (pmax) {
        case 1: return v4_launch_p<1>(is3d, form, epi, p, g, tc, omega, st);
        case 2: return v4_launch_p<2>(is3d, form, epi, p, g, tc, omega, st);
        case 3: return v4_launch_p<3>(is3d, form, epi, p, g, tc, omega, st);
        case 4: return v4_launch_p<4>(is3d, form, epi, p, g, tc, omega, st);
        case 5: return v4_launch_p<5>(is3d, form, epi, p, g, tc, omega, st);
    }
    set_error("pmax must be in 1..5");
    return 1;
}

}  // namespace poms
