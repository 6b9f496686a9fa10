// Fused Kronecker-sum operator, v6 (variant 11): THREE columns per lane.
//
// Why (tools/ubench_valu.hip, SQ counters in profiles/r03/): on gfx950 an FP64
// FMA and a 32-bit DPP lane shift both cost ~4 cycles per wave instruction, and
// the v5 apply keeps the VALU busy ~70 % of its time -- memory alone (v5's own
// access pattern, no arithmetic) runs in ~440 us at 515^3, the full kernel in
// 520-590 us.  The arithmetic per OUTPUT point is what has to shrink, and v5
// spends a fifth of it on lanes and shifts that produce nothing:
//   * v5 tiles are 128 lane-columns (two per lane) for 112 outputs, five tiles per
//     515-column row (640 lane-columns: 80 % useful);
//   * v5 shifts 12 doubles per lane and plane by DPP (6 per output column).
// With three columns per lane the +-3 window of a lane is exactly its two
// neighbour lanes: ONE DPP shift per neighbour double (24 DPP movs per three
// columns, 4 per column), one halo lane per side, and three 192-lane-column tiles
// per row (576 lane-columns: 89 % useful).  Same 43 FP64 operations per column.
//
//   * workgroup: 16 waves = 16 output rows (axis 1) x 192 lane-columns; lane l owns
//     lane-columns 3l, 3l+1, 3l+2 <-> interior columns c0 - 3 + 3l + e.  Output
//     columns c0 .. c0+TO-1 (TO = 176 = 11 whole lines on the aligned layout);
//   * x planes DMA'd into a D-deep LDS ring (22 rows x 192 doubles; LDS column j
//     <-> interior column c0 - 4 + j, so every 16-B DMA piece starts 16-B aligned),
//     read back by ds_read_b64 (lane l reads 8 (3l + 1 + e): conflict-free);
//   * axis 1 (first) on the wave's own row, axis 2 by one DPP shift per neighbour
//     double, axis 0 scattered into 2P+1 rotating accumulators (as v5);
//   * non-Toeplitz columns (the boundary tiles): per-lane-column band rows from an
//     LDS table; non-Toeplitz rows: the wave's band row by scalar loads.
// Preconditions (host): 3D, FORM_SUM, P <= 3, pads == P, line-aligned layout
// (pitch a multiple of 16 doubles, interior column 0 on a 128-B line), array < 2 GiB.
// Epilogue: APPLY (the Kron SpMV, sources/kron_product.py:80-86).
#include "common.hpp"

namespace poms {

typedef __attribute__((address_space(3))) void lds6_void_t;

template <int AUX = 0>
__device__ __forceinline__ void v6_dma16(__amdgpu_buffer_rsrc_t r, double* lds_dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds6_void_t*)lds_dst, 16, voff, (int)soff, 0, AUX);
}
__device__ __forceinline__ double v6_shr1(double v) {  // lane l <- lane l-1 (lane 0 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double v6_shl1(double v) {  // lane l <- lane l+1 (lane 63 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
template <int N>
__device__ __forceinline__ void v6_wait_vm() {  // s_waitcnt vmcnt(N) (gfx9 encoding)
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
__device__ __forceinline__ void v6_barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}

constexpr int V6_NW = 16;    // waves = output rows per tile
constexpr int V6_XP = 192;   // LDS row pitch of the x image (doubles)

template <int P, int EPI, int D, int YAUX, bool SAME12>
__global__ void __launch_bounds__(64 * V6_NW, 1)
kron_v6_kernel(const double* __restrict__ x, double* __restrict__ y,
               const double* __restrict__ a0t, const double* __restrict__ b0t,
               const double* __restrict__ a1, const double* __restrict__ b1,
               const double* __restrict__ a2, const double* __restrict__ b2,
               const KronGeom g, const ToepConst tc) {
    static_assert(P >= 1 && P <= 3, "v6: P <= 3 (the +-P window is the two neighbour lanes)");
    static_assert(EPI == EPI_APPLY, "v6: apply epilogue");
    constexpr int W = 2 * P + 1;
    constexpr int NW = V6_NW, T1 = NW, XR = T1 + 2 * P, XP = V6_XP, NS = W;
    constexpr int PFX = D - 1;
    // [a|b][k][e][lane] band rows of the tile's columns, first: its reads then fit the
    // 16-bit ds_read offset from one lane base (at the end of the 135-KB ring every
    // read needed its own address VGPR, and the p = 3 build spilled them)
    constexpr int C2_OFF = 0;
    constexpr int XS_OFF = C2_OFF + 2 * W * 3 * 64;
    constexpr int LDS_N = XS_OFF + D * XR * XP;
    __shared__ __attribute__((aligned(16))) double lds[LDS_N];
#define T2A(k) (SAME12 ? tc.t1a[k] : tc.t2a[k])
#define T2B(k) (SAME12 ? tc.t1b[k] : tc.t2b[k])

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
    int t1, t2;
    if (g.order) {
        t1 = bid % g.tiles1; bid /= g.tiles1;
        t2 = bid % g.tiles2; bid /= g.tiles2;
    } else {
        t2 = bid % g.tiles2; bid /= g.tiles2;
        t1 = bid % g.tiles1; bid /= g.tiles1;
    }
    const int ch = bid;
    const int c0 = t2 * TO;
    const int r0 = t1 * T1;
    const int orow = r0 + wv;
    const bool row_ok = orow < g.n1;
    const int cg0 = c0 - 3 + 3 * lane;   // interior column of this lane's element 0
    const int cend = min(c0 + TO, g.n2);
    int cok = 0;   // output columns of this lane (VGPR bit mask)
#pragma unroll
    for (int e = 0; e < 3; ++e) cok |= (cg0 + e >= c0 && cg0 + e < cend) ? (1 << e) : 0;
    const bool fast1 = orow >= tc.lo1 && orow < tc.hi1;
    const bool fast2 = c0 >= tc.lo2 && cend <= tc.hi2;

    if (!fast2) {   // band rows of every lane-column (clamped: lanes past the grid are never stored)
        for (int i = tid; i < W * 3 * 64; i += NW * 64) {
            const int k = i / 192, e = (i / 64) % 3, l = i % 64;
            const int col = min(max(c0 - 3 + 3 * l + e, 0), g.n2 - 1);
            lds[C2_OFF + i] = a2[col * W + k];
            lds[C2_OFF + W * 192 + i] = b2[col * W + k];
        }
    }
    const int orc = min(orow, g.n1 - 1);
    const double* __restrict__ ra = a1 + orc * W;
    const double* __restrict__ rb = b1 + orc * W;

    int z0, z1;
    chunk_planes(g, ch, z0, z1);
    const int nplanes = (z1 - z0) + 2 * P;
    const int nsp = g.n0 + 2 * g.pd0;
    const int s1 = (int)g.s1;
    const uint32_t arr_bytes = (uint32_t)((int64_t)nsp * g.s0 * 8);
    const uint32_t plane8 = (uint32_t)(g.s0 * 8);
    const __amdgpu_buffer_rsrc_t rx = make_rsrc(x, arr_bytes);
    const __amdgpu_buffer_rsrc_t ry = make_rsrc(y, arr_bytes);
    // x DMA pieces: piece m (16 B) = LDS columns 2m, 2m+1 <-> interior columns
    // c0 - 4 + 2m, +1 (storage c0 - 4 + P + 2m): pieces 0..63 by one DMA, pieces
    // 64 .. 63 + nB by a second one (1024 bytes further: the instruction's offset
    // field) on lanes < nB, which covers interior columns up to cend - 1 + P.
    const uint32_t offA = (uint32_t)((c0 - 4 + P) * 8 + 16 * lane);
    const int nB = min(32, (cend + P - (c0 - 4) + 1) / 2 - 64);
    auto dma_x = [&](int m, int slot) {   // x plane m (local interior index), rows r0 - P .. r0 + T1 + P - 1
        const int sp = m + g.pd0;
        const bool ok = sp >= 0 && sp < nsp;
        const uint32_t so = ok ? (uint32_t)sp * plane8 : 0u;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = wv + i * NW;   // x-tile row q = storage row r0 + q
            if (i == 0 || q < XR) {
                const uint32_t rowb = (uint32_t)((r0 + q) * s1 * 8);
                double* dst = lds + XS_OFF + (slot * XR + q) * XP;
                const int vo = ok ? (int)(rowb + offA) : 0x7ffffff0;
                v6_dma16<0>(rx, dst, vo, so);
                // second piece: LDS columns 128 .. 127 + 2 nB (exec-masked: an out-of-range
                // lane would still write zeros into LDS, past the row).  The instruction
                // offset moves the LDS address too: both 1024 bytes on from the first piece.
                if (lane < nB) __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds6_void_t*)dst, 16, vo, (int)so, 1024, 0);
            }
        }
    };
    const bool xtra = wv < XR - NW;   // this wave DMAs two x rows per plane (4 pieces), else one (2)

    double acc[NS][3];
#pragma unroll
    for (int s = 0; s < NS; ++s) { acc[s][0] = 0.0; acc[s][1] = 0.0; acc[s][2] = 0.0; }
    auto zo_of = [&](int t) { return max(z0 - 2 * P + t, z0); };
    const int colst = (cg0 + P) * 8;   // storage byte column of this lane's element 0

    __syncthreads();   // C2 table visible; no DMA in flight yet
#pragma unroll
    for (int i = 0; i < PFX; ++i) dma_x(i < nplanes ? z0 - P + i : -(1 << 20), i);

    for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nplanes) {
                // x(t) landed: own DMAs by vmcnt (loads issued after it: planes t+1 ..
                // t+PFX-1, 4 or 2 pieces each; stores never counted), everyone's by the barrier
                if (t < PFX) v6_wait_vm<0>();
                else if (xtra) v6_wait_vm<(PFX - 1) * 4>();
                else v6_wait_vm<(PFX - 1) * 2>();
                v6_barrier();
                dma_x(t + PFX < nplanes ? z0 - P + t + PFX : -(1 << 20), (t + PFX) % D);

                // ---- axis 1 on this wave's row, three columns per lane
                const double* xs = lds + XS_OFF + (t % D) * XR * XP + 3 * lane + 1;
                double u[3], v[3];
                if (fast1) {
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        double pr[P + 1];
                        pr[0] = xs[(wv + P) * XP + e];
#pragma unroll
                        for (int k = 1; k <= P; ++k) pr[k] = xs[(wv + P - k) * XP + e] + xs[(wv + P + k) * XP + e];
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
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        const double x0v = xs[wv * XP + e];
                        double su = ra[0] * x0v, sv = rb[0] * x0v;
#pragma unroll
                        for (int k = 1; k < W; ++k) {
                            const double xk = xs[(wv + k) * XP + e];
                            su = fma(ra[k], xk, su);
                            sv = fma(rb[k], xk, sv);
                        }
                        u[e] = su;
                        v[e] = sv;
                    }
                }

                // ---- axis 2: window columns 3l-3 .. 3l+5 = [left lane | own | right lane]
                double cc[3], dd[3];
                if (fast2) {
                    double wu[9], wvv[9];
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        wu[3 + e] = u[e];
                        wvv[3 + e] = v[e];
                    }
#pragma unroll
                    for (int e = 3 - P; e < 3; ++e) {   // left: lane l-1's columns 3l-3+e
                        wu[e] = v6_shr1(u[e]);
                        wvv[e] = v6_shr1(v[e]);
                    }
#pragma unroll
                    for (int e = 0; e < P; ++e) {       // right: lane l+1's columns 3l+3+e
                        wu[6 + e] = v6_shl1(u[e]);
                        wvv[6 + e] = v6_shl1(v[e]);
                    }
#pragma unroll
                    for (int e = 0; e < 3; ++e) {
                        double pu[P + 1], pv[P + 1];
                        pu[0] = wu[3 + e];
                        pv[0] = wvv[3 + e];
#pragma unroll
                        for (int k = 1; k <= P; ++k) {
                            pu[k] = wu[3 + e - k] + wu[3 + e + k];
                            pv[k] = wvv[3 + e - k] + wvv[3 + e + k];
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
                    // per-lane-column band rows: window column i (0..8) is formed, added
                    // into every output column it reaches (band index k = i - 3 - e + P)
                    // and dropped -- all nine windows live at once spilled the p = 3 build
#pragma unroll
                    for (int e = 0; e < 3; ++e) { cc[e] = 0.0; dd[e] = 0.0; }
#pragma unroll
                    for (int i = 3 - P; i < 6 + P; ++i) {
                        const double wi = i < 3 ? v6_shr1(u[i]) : i < 6 ? u[i - 3] : v6_shl1(u[i - 6]);
                        const double vi = i < 3 ? v6_shr1(v[i]) : i < 6 ? v[i - 3] : v6_shl1(v[i - 6]);
#pragma unroll
                        for (int e = 0; e < 3; ++e) {
                            const int k = i - 3 - e + P;
                            if (k >= 0 && k < W) {
                                const double fa = lds[C2_OFF + (k * 3 + e) * 64 + lane];
                                const double fb = lds[C2_OFF + W * 192 + (k * 3 + e) * 64 + lane];
                                cc[e] = fma(fa, wi, cc[e]);
                                dd[e] = fma(fa, vi, fma(fb, wi, dd[e]));
                            }
                        }
                    }
                }

                // ---- axis 0: scatter into the rotating slots
                const int jrow = (g.g0 + z0 - P + t + P) * W;
#pragma unroll
                for (int s = 0; s < W; ++s) {
                    const int slot = (q - P + s + NS) % NS;
                    const double ka = a0t[jrow + s];
                    const double kb = b0t[jrow + s];
#pragma unroll
                    for (int e = 0; e < 3; ++e) acc[slot][e] = fma(ka, cc[e], fma(kb, dd[e], acc[slot][e]));
                }
                const int done = (q + P + 1) % NS;
                double vo[3];
#pragma unroll
                for (int e = 0; e < 3; ++e) {
                    vo[e] = acc[done][e];
                    acc[done][e] = 0.0;
                }
                const bool en = t >= 2 * P && row_ok;
                const int zo = zo_of(t);
                // three 8-B stores (lane stride 24 B: the three instructions together
                // write whole lines, merged in L2); plane offset in voffset, soffset 0
                const int voy = (orow + P) * s1 * 8 + colst + (zo + g.pd0) * (int)plane8;
#pragma unroll
                for (int e = 0; e < 3; ++e)
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, vo[e]), ry,
                                                          (en && ((cok >> e) & 1)) ? voy + 8 * e : 0x7ffffff0, 0, YAUX);
            }
        }
    }
    v6_wait_vm<0>();   // no LDS-DMA may outlive the workgroup
#undef T2A
#undef T2B
}

template <int P, int EPI, int D, int YAUX, bool SAME12>
static int v6_launch_t(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, hipStream_t st) {
    // the hand-counted vmcnt waits assume the only VMEM ops in the loop are the
    // DMAs and the stores: a build that spills to scratch would break them
    static int scratch = -1;
    if (scratch < 0) {
        hipFuncAttributes at{};
        if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&kron_v6_kernel<P, EPI, D, YAUX, SAME12>)) != hipSuccess) {
            set_error("v6: hipFuncGetAttributes failed");
            return 1;
        }
        scratch = (int)at.localSizeBytes;
    }
    if (scratch > 0) {
        set_error("v6: kernel build spills to scratch (vmcnt counting invalid)");
        return 1;
    }
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    hipLaunchKernelGGL((kron_v6_kernel<P, EPI, D, YAUX, SAME12>), dim3(nblk), dim3(64 * V6_NW), 0, st, p.x, p.y,
                       p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, g, tc);
    return 0;
}

template <int P>
static int v6_launch_p(int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, hipStream_t st) {
    bool same = true;   // the axis-1 / axis-2 Toeplitz rows, bitwise (one set of SGPR constants)
    for (int k = 0; k <= P; ++k) same = same && tc.t1a[k] == tc.t2a[k] && tc.t1b[k] == tc.t2b[k];
    if (epi != EPI_APPLY) {
        set_error("v6: apply epilogue only");
        return 1;
    }
    // y stores non-temporal (streamed once), x DMAs default (halo rows re-read)
    return same ? v6_launch_t<P, EPI_APPLY, 4, 2, true>(p, g, tc, st) : v6_launch_t<P, EPI_APPLY, 4, 2, false>(p, g, tc, st);
}

// v6 tiles: 192 lane-columns, one halo lane per side; output columns per tile
// (whole lines on the aligned layout: 176)
int kron_v6_tile_cols() { return 176; }
int kron_v6_rows() { return V6_NW; }

int kron_v6_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, hipStream_t st) {
    // the last output lane's right neighbour lane exists, and the x image (output
    // columns + P on each side, from interior column c0 - 4) fits the 192-column row
    if (g.tout <= 0 || g.tout > 184 || (g.tout & 1)) {
        set_error("v6: bad tile geometry");
        return 1;
    }
    switch (pmax) {
        case 1: return v6_launch_p<1>(epi, p, g, tc, st);
        case 2: return v6_launch_p<2>(epi, p, g, tc, st);
        case 3: return v6_launch_p<3>(epi, p, g, tc, st);
    }
    set_error("v6: pmax must be in 1..3");
    return 1;
}

}  // namespace poms
