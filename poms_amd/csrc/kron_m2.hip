// 2D Kronecker-sum operator, m2 (variant 12): one wave per (column tile, row chunk),
// rows marched through 2P+1 rotating accumulators, columns by DPP lane shifts.
//
// Why (round 5).  The 2D p = 3 1024^2 V-cycle is kernel-bound, not host-bound: its
// rocprofv3 trace sums to 3.04 ms of kernel time per 3.21 ms cycle, 64 % of it in
// 198 damped-Jacobi sweeps of 9.8 us each (profiles/r04/final6/).  A sweep moves
// 25 MB, which the L2s and the MALL hold: the v3 kernel (64-column tiles of 16 rows,
// 1170 workgroups in 2.3 rounds, every tile loading its 6 halo rows, one LDS round
// trip and barrier per tile) is bound by its rounds of short-lived workgroups.
//
// m2 gives each wave a 128-column tile (two columns per lane, 16-B loads and stores:
// v5's tile, 112 line-aligned output columns on the aligned layout) and a chunk of
// rows, marched like v5's axis 0:
//   * no LDS ring and no barrier: a wave loads its own x rows straight into a
//     (2P+1)-deep register ring, PF = P+1 rows ahead, and reads x at the output row
//     (Jacobi, apply + dot) back from the same ring, P rows late -- the ring and the
//     accumulators rotate with one period (the loop is unrolled by 2P+1), so no
//     register moves;
//   * axis 2 (columns) first: a = F2a x, b = F2b x with the column neighbours by
//     wave_shr / wave_shl DPP (symmetric Toeplitz pair sums inside the interior
//     column tiles, per-column rows from an LDS table in the boundary tiles);
//   * axis 1 (rows): y = F1a a + F1b b scattered into 2P+1 rotating accumulators
//     (the Toeplitz row constants inside the interior, the band rows by scalar loads
//     next to the row ends); b (residual, Jacobi) through a second register ring;
//   * epilogues APPLY, RESID, JACOBI (||dr||^2 and optionally x_out . b), APPLYDOT
//     (x . Ax); per-block partials summed in wave order.
// Preconditions (host, m2_ok): 2D FORM_SUM, P <= 3, storage pads == P, array < 2 GiB.
#include "common.hpp"

namespace poms {

namespace {

__device__ __forceinline__ double m2_shr1(double v) {   // lane l <- lane l-1 (lane 0 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double m2_shl1(double v) {   // lane l <- lane l+1 (lane 63 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}

typedef double m2d2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ m2d2 m2_load(__amdgpu_buffer_rsrc_t r, int voff) {   // 16 B, non-temporal off
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    return m2d2{__builtin_bit_cast(double, u32x2{v.x, v.y}), __builtin_bit_cast(double, u32x2{v.z, v.w})};
}

}  // namespace

// Waves per workgroup: one.  A 2D sweep runs only ~650-1300 waves (one per tile and
// row chunk), fewer than the chip's 1024 SIMDs hold at 4 waves each, so occupancy is
// not what bounds it; one-wave workgroups spread over every CU, and 256 VGPRs keep the
// p = 3 rings and accumulators out of scratch.
constexpr int kM2Waves = 1;

template <int P, int EPI, bool ST16, bool JDOT>
__global__ void __launch_bounds__(64 * kM2Waves, 2)
kron_m2_kernel(const double* __restrict__ x, double* __restrict__ y, const double* __restrict__ bvec,
               const double* __restrict__ a1, const double* __restrict__ b1,
               const double* __restrict__ a2, const double* __restrict__ b2,
               double* __restrict__ partial, double* __restrict__ partial2,
               const double* __restrict__ rdiag0, const KronGeom g, const ToepConst tc, const int H,
               const double omega) {
    constexpr int W = 2 * P + 1;
    constexpr int NS = W;           // accumulators, x ring and b ring: one rotation period
    constexpr int PF = NS - P;      // x rows in flight ahead of the one being used
    constexpr bool HASB = EPI == EPI_RESID || EPI == EPI_JACOBI;
    constexpr bool JAC = EPI == EPI_JACOBI;
    constexpr bool APD = EPI == EPI_APPLYDOT;
    constexpr int NWIN = 2 * P + 2;   // columns 2j-P .. 2j+1+P of a lane's pair

    // the workgroup's waves share one column tile (consecutive row chunks): one LDS
    // table of the boundary tiles' column rows, built before the march
    __shared__ __attribute__((aligned(16))) double ct[2 * W * 128];
    __shared__ double red[kM2Waves];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int TO = g.tout;
    const int t2 = blockIdx.x % g.tiles2;
    const int ch = (blockIdx.x / g.tiles2) * kM2Waves + wv;
    const bool live = ch < g.nchunks;      // (the last workgroups of a column may hold idle waves)
    const int c0 = t2 * TO;
    const int r0 = ch * g.chunk;
    const int r1 = min(r0 + g.chunk, g.n1);
    const int nsteps = live ? (r1 - r0) + 2 * P : 0;
    const int cg0 = c0 - H + 2 * lane;     // interior column of this lane's element 0
    int cok = 0;                           // output columns of this lane (bit e)
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int ci = 2 * lane + e;
        cok |= (ci >= H && ci < H + TO && cg0 + e < g.n2) ? (1 << e) : 0;
    }
    const bool fast2 = c0 >= tc.lo2 && min(c0 + TO, g.n2) <= tc.hi2;
    if (!fast2) {
        for (int e = tid; e < W * 128; e += 64 * kM2Waves) {
            const int k = e / 128, ci = e - k * 128;
            const int col = min(max(c0 - H + ci, 0), g.n2 - 1);
            ct[e] = a2[col * W + k];
            ct[W * 128 + e] = b2[col * W + k];
        }
    }
    __syncthreads();
    const int s1 = (int)g.s1;
    const uint32_t arr_bytes = (uint32_t)((int64_t)(g.n1 + 2 * g.pd1) * g.s1 * 8);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, arr_bytes);
    const __amdgpu_buffer_rsrc_t rbv = make_rsrc(bvec, HASB ? arr_bytes : 0u);
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, arr_bytes);
    const uint32_t colb = (uint32_t)((c0 - H + g.pd2) * 8 + 16 * lane);   // this lane's pair in a row (bytes)
    // lane-columns no output point reads are not fetched: pushed out of the buffer range
    // (+2^31; arrays < 2 GiB), so the load moves no bytes and returns zeros
    const uint32_t colx = colb + ((2 * lane + 1 >= H - P && 2 * lane < H + TO + P) ? 0u : 0x80000000u);
    const uint32_t colo = colb + ((2 * lane + 1 >= H && 2 * lane < H + TO) ? 0u : 0x80000000u);
    auto xoff = [&](int m) {   // storage row of interior row m (out of the array: no bytes)
        return (m >= -g.pd1 && m < g.n1 + g.pd1) ? (int)((uint32_t)((m + g.pd1) * s1 * 8) + colx) : (int)0x7ffffff0;
    };
    auto ooff = [&](int m) {
        return (m >= 0 && m < g.n1) ? (int)((uint32_t)((m + g.pd1) * s1 * 8) + colo) : (int)0x7ffffff0;
    };

    m2d2 xr[NS], br[NS];
    double acc[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        acc[s][0] = acc[s][1] = 0.0;
        xr[s] = m2d2{0.0, 0.0};
        br[s] = m2d2{0.0, 0.0};
    }
    // x rows of steps 0 .. PF-1 (b of step t's output row is loaded at step t - PF >= 0:
    // outputs start at step 2P >= PF)
#pragma unroll
    for (int i = 0; i < PF; ++i) xr[i] = m2_load(rx, i < nsteps ? xoff(r0 - P + i) : (int)0x7ffffff0);
    double nrm = 0.0, dotp = 0.0;

    for (int tb = 0; tb < nsteps; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nsteps) {
                const int m = r0 - P + t;   // interior row of x(t)
                // ---- axis 2 (columns) on row m: a = F2a x, b = F2b x
                const m2d2 xv = xr[q];
                double w[NWIN];
                w[P] = xv[0];
                w[P + 1] = xv[1];
#pragma unroll
                for (int i = P - 1; i >= 0; --i) w[i] = m2_shr1(w[i + 2]);
#pragma unroll
                for (int i = P + 2; i <= 2 * P + 1; ++i) w[i] = m2_shl1(w[i - 2]);
                double ua[2], ub[2];
                if (fast2) {
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        double pr[P + 1];
                        pr[0] = w[e + P];
#pragma unroll
                        for (int k = 1; k <= P; ++k) pr[k] = w[e + P - k] + w[e + P + k];
                        double sa = tc.t2a[0] * pr[0], sb = tc.t2b[0] * pr[0];
#pragma unroll
                        for (int k = 1; k <= P; ++k) {
                            sa = fma(tc.t2a[k], pr[k], sa);
                            sb = fma(tc.t2b[k], pr[k], sb);
                        }
                        ua[e] = sa;
                        ub[e] = sb;
                    }
                } else {
                    double sa[2] = {0.0, 0.0}, sb[2] = {0.0, 0.0};
#pragma unroll
                    for (int k = 0; k < W; ++k) {
                        const m2d2 fa = *(const m2d2*)(ct + k * 128 + 2 * lane);
                        const m2d2 fb = *(const m2d2*)(ct + (W + k) * 128 + 2 * lane);
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            sa[e] = fma(fa[e], w[e + k], sa[e]);
                            sb[e] = fma(fb[e], w[e + k], sb[e]);
                        }
                    }
                    ua[0] = sa[0]; ua[1] = sa[1];
                    ub[0] = sb[0]; ub[1] = sb[1];
                }
                // ---- axis 1 (rows): row m contributes to output rows m - P + s
                if (m - P >= tc.lo1 && m + P < tc.hi1) {   // every target row Toeplitz
#pragma unroll
                    for (int s = 0; s < W; ++s) {
                        const int slot = (q - P + s + NS) % NS;
                        const int k = s < P ? P - s : s - P;
#pragma unroll
                        for (int e = 0; e < 2; ++e) acc[slot][e] = fma(tc.t1a[k], ua[e], fma(tc.t1b[k], ub[e], acc[slot][e]));
                    }
                } else {
#pragma unroll
                    for (int s = 0; s < W; ++s) {
                        const int slot = (q - P + s + NS) % NS;
                        const int row = min(max(m - P + s, 0), g.n1 - 1);   // (rows past the ends are not output)
                        const double ka = a1[row * W + (2 * P - s)];
                        const double kb = b1[row * W + (2 * P - s)];
#pragma unroll
                        for (int e = 0; e < 2; ++e) acc[slot][e] = fma(ka, ua[e], fma(kb, ub[e], acc[slot][e]));
                    }
                }
                const int done = (q + P + 1) % NS;
                const double vo[2] = {acc[done][0], acc[done][1]};
                acc[done][0] = acc[done][1] = 0.0;
                // x(t + PF): into the slot of x(t - P), read by this step's epilogue below
                // ... issued after it (the slot is free only then)
                const bool en = t >= 2 * P;
                const int zo = m - P;          // output row of this step
                if (en) {
                    const m2d2 xin = xr[(q - P + NS) % NS];   // x at the output row (Jacobi, apply + dot)
                    const m2d2 bv = br[q];
                    bool ok[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) ok[e] = (cok >> e) & 1;
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
                        outv[0] = bv[0] - vo[0];
                        outv[1] = bv[1] - vo[1];
                    } else {
                        double rc[2];
                        const bool frow = zo >= tc.lo1 && zo < tc.hi1;
                        if (fast2 && frow && rdiag0 != nullptr) {
                            rc[0] = rc[1] = omega * rdiag0[0];
                        } else {
                            const double d1a = a1[zo * W + P], d1b = b1[zo * W + P];
#pragma unroll
                            for (int e = 0; e < 2; ++e) {
                                const double d2a = fast2 ? tc.t2a[0] : ct[P * 128 + 2 * lane + e];
                                const double d2b = fast2 ? tc.t2b[0] : ct[(W + P) * 128 + 2 * lane + e];
                                const double dg = fma(d1a, d2a, d1b * d2b);
                                double r = __builtin_amdgcn_rcp(dg);
                                double ee = fma(-dg, r, 1.0);
                                r = fma(r, ee, r);
                                ee = fma(-dg, r, 1.0);
                                r = fma(r, ee, r);
                                rc[e] = omega * r;
                            }
                        }
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const double dr = (bv[e] - vo[e]) * rc[e];
                            outv[e] = xin[e] + dr;
                            const double drm = ok[e] ? dr : 0.0;   // (nrm >= 0: + 0 * 0 is exact)
                            nrm = fma(drm, drm, nrm);
                            if constexpr (JDOT) dotp = ok[e] ? fma(outv[e], bv[e], dotp) : dotp;
                        }
                    }
                    const int voy = ooff(zo);
                    const double o1 = ok[1] ? outv[1] : 0.0;   // (a column past n2 is a ghost: keep it 0)
                    if constexpr (ST16) {
                        u32x4 v;
                        const u32x2 a = __builtin_bit_cast(u32x2, outv[0]), b = __builtin_bit_cast(u32x2, o1);
                        v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
                        __builtin_amdgcn_raw_buffer_store_b128(v, ry, (ok[0] || ok[1]) ? voy : (int)0x7ffffff0, 0, 2);
                    } else {
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, outv[0]), ry,
                                                              ok[0] ? voy : (int)0x7ffffff0, 0, 2);
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o1), ry,
                                                              (ok[0] || ok[1]) ? voy + 8 : (int)0x7ffffff0, 0, 2);
                    }
                }
                // prefetch: x(t + PF) into x(t - P)'s slot, b of step t + PF's output row
                xr[(q + PF) % NS] = m2_load(rx, t + PF < nsteps ? xoff(m + PF) : (int)0x7ffffff0);
                if constexpr (HASB)
                    br[(q + PF) % NS] = m2_load(rbv, (t + PF >= 2 * P && t + PF < nsteps) ? ooff(m + PF - P) : (int)0x7ffffff0);
            }
        }
    }
    if constexpr (JAC || APD) {
        if (partial != nullptr || partial2 != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
                nrm += __shfl_xor(nrm, off, 64);
                dotp += __shfl_xor(dotp, off, 64);
            }
            if (partial != nullptr) {
                if (lane == 0) red[wv] = nrm;
                __syncthreads();
                if (tid == 0) {
                    double s = 0.0;
                    for (int i = 0; i < kM2Waves; ++i) s += red[i];
                    partial[blockIdx.x] = s;
                }
                __syncthreads();
            }
            if (partial2 != nullptr) {
                if (lane == 0) red[wv] = dotp;
                __syncthreads();
                if (tid == 0) {
                    double s = 0.0;
                    for (int i = 0; i < kM2Waves; ++i) s += red[i];
                    partial2[blockIdx.x] = s;
                }
            }
        }
    }
}

template <int P, int EPI, bool ST16, bool JDOT>
static int m2_launch_t(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega, hipStream_t st) {
    const int nblk = g.tiles2 * ((g.nchunks + kM2Waves - 1) / kM2Waves);
    hipLaunchKernelGGL((kron_m2_kernel<P, EPI, ST16, JDOT>), dim3(nblk), dim3(64 * kM2Waves), 0, st, p.x, p.y, p.b,
                       p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, p.rdiag0, g, tc, H, omega);
    return 0;
}

template <int P, int EPI>
static int m2_launch_e(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega, hipStream_t st) {
    const bool st16 = ((reinterpret_cast<uintptr_t>(p.y) + 8 * (int64_t)(g.pd2 - H)) & 15) == 0 && g.s1 % 2 == 0 &&
                      ((reinterpret_cast<uintptr_t>(p.x) + 8 * (int64_t)(g.pd2 - H)) & 15) == 0 &&
                      (p.b == nullptr || ((reinterpret_cast<uintptr_t>(p.b) + 8 * (int64_t)(g.pd2 - H)) & 15) == 0);
    if (!st16) {   // 16-B loads need 16-B aligned rows too
        set_error("m2: rows not 16-B aligned");
        return 1;
    }
    if (EPI == EPI_JACOBI && p.partial2 != nullptr) return m2_launch_t<P, EPI, true, true>(p, g, tc, H, omega, st);
    return m2_launch_t<P, EPI, true, false>(p, g, tc, H, omega, st);
}

template <int P>
static int m2_launch_p(int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    switch (epi) {
        case EPI_APPLY: return m2_launch_e<P, EPI_APPLY>(p, g, tc, H, omega, st);
        case EPI_RESID: return m2_launch_e<P, EPI_RESID>(p, g, tc, H, omega, st);
        case EPI_JACOBI: return m2_launch_e<P, EPI_JACOBI>(p, g, tc, H, omega, st);
        case EPI_APPLYDOT: return m2_launch_e<P, EPI_APPLYDOT>(p, g, tc, H, omega, st);
    }
    set_error("m2: epilogue not built");
    return 1;
}

// 16-B aligned rows of x, y (and b) at the tile's first lane-column: m2 needs them
bool kron_m2_aligned(const double* x, const double* y, const double* b, int pd2, int H, int64_t s1) {
    auto al = [&](const double* v) { return v == nullptr || ((reinterpret_cast<uintptr_t>(v) + 8 * (int64_t)(pd2 - H)) & 15) == 0; };
    return s1 % 2 == 0 && al(x) && al(y) && al(b);
}

int kron_m2_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                   hipStream_t st) {
    if (H < pmax || (H & 1) || (g.tout & 1) || H + g.tout + pmax > 128 || g.chunk < 1) {
        set_error("m2: bad tile geometry");
        return 1;
    }
    switch (pmax) {
        case 1: return m2_launch_p<1>(epi, p, g, tc, H, omega, st);
        case 2: return m2_launch_p<2>(epi, p, g, tc, H, omega, st);
        case 3: return m2_launch_p<3>(epi, p, g, tc, H, omega, st);
    }
    set_error("m2: pmax must be in 1..3");
    return 1;
}

}  // namespace poms
