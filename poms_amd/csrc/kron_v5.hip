// Fused Kronecker-sum operator, v5 (variant 10): 128-column tiles, one row per
// wave, x planes DMA'd into an LDS ring, axis 1 first.
//
// Why this shape (tools/ubench_copy.hip, tools/ubench_rowtile.hip at 515^3):
// the 64-column tiles of v3/v4 store 58-column row segments that start anywhere
// in a 128-B line, so two workgroups write parts of the same line at different
// times; the access pattern alone (no arithmetic) ran 621-681 us against
// 436 us for a plain copy of the same bytes.  128-column tiles whose 112 output
// columns start on a line (the aligned layout: row pitch a multiple of 16
// doubles, interior column 0 on a line) write whole lines only, and ran 513 us.
//
//   * workgroup: 16 waves = 16 output rows (axis 1) x 128 lane-columns (each
//     lane owns two adjacent columns: 16-B loads / stores), marching a chunk of
//     axis-0 planes.  The first H and last 128-H-TO lane-columns are halo
//     (H = 8, TO = 112 on the aligned layout; H = P rounded up to even,
//     TO = 128 - 2H otherwise);
//   * memory: each x plane tile (T1 + 2P rows x 128 columns) is DMA'd by
//     buffer_load ... lds straight into a D-deep LDS ring, D-1 planes ahead
//     (D = 4 for apply and Jacobi, 3 for the residual); b (residual / Jacobi)
//     through a 3-deep ring two planes ahead (residual) or a 2-deep ring one
//     plane ahead (Jacobi: its 4th x plane leaves no LDS for a 3rd b plane).
//     vmcnt is counted by hand, one barrier per plane;
//   * axis 1 (first) on the wave's own row: u = F1a x, v = F1b x (symmetric
//     Toeplitz pair sums inside the interior, per-row scalar coefficients
//     outside); axis 2 with the column neighbours shifted in by DPP
//     (c = F2a u, d = F2a v + F2b u); axis 0 scattered into 2P+1 rotating
//     accumulators;
//   * epilogues: APPLY, RESID, JACOBI (1/diag from the host table inside the
//     Toeplitz interior, else from the plane-invariant pieces of the diagonal),
//     APPLYDOT (x . Ax).  x at the output point (Jacobi's x_in, APPLYDOT's x)
//     comes from a P-deep register history of the lane's centre tap -- no
//     re-read (the x_in DMA next to b, kept as a tuning build, costs 8 B/DOF);
//   * y stores and b DMAs are non-temporal (streamed once); x DMAs are not
//     (the halo rows are re-read by the neighbouring tiles).
// Preconditions (host, v5_ok): 3D, FORM_SUM, P <= 5 (16-wave tiles at P <= 3, 8-wave
// tiles at P >= 4 and for the p <= 2 sweeps from zero: v5_waves), storage pads == P,
// array < 2 GiB, and no odd P on layouts with data in the corner ghosts (the x-row
// DMA pair holding storage column 0 of storage row 0 fails the range check there).
#include "common.hpp"

#include <hip/hip_ext.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <map>
#include <mutex>
#include <vector>

namespace poms {

typedef __attribute__((address_space(3))) void lds5_void_t;

// MODE 6 (diagnostic, apply / Jacobi): per-wave clock stamps of the march.  Per wave,
// 8 u64: [0] cycles waiting for its own DMAs (s_waitcnt vmcnt), [1] in the plane
// barrier, [2] the rest (DMA issue, arithmetic, store), [3] planes, [4] start and
// [5] end (s_memrealtime, 100 MHz), [6] XCC id, [7] CU id.  s_memtime reads the
// shader clock (a scalar READ; nothing is stored through the scalar cache); the
// stamps go out by vector stores.
constexpr int kV5Stamps = 1 << 19;   // u64 entries: 65536 waves
__device__ unsigned long long g_v5_stamps[kV5Stamps];

template <int AUX = 0>   // cache policy (gfx950: bit 1 = nt, streaming)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, double* lds_dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds5_void_t*)lds_dst, 16, voff, (int)soff, 0, AUX);
}
template <int AUX = 0>
__device__ __forceinline__ void bstore2_sp(__amdgpu_buffer_rsrc_t r, int voff, unsigned soff, double d0, double d1) {
    u32x4 v;
    const u32x2 a = __builtin_bit_cast(u32x2, d0), b = __builtin_bit_cast(u32x2, d1);
    v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, (int)soff, AUX);
}

__device__ __forceinline__ double v5_shr1(double v) {  // lane l <- lane l-1 (lane 0 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}
__device__ __forceinline__ double v5_shl1(double v) {  // lane l <- lane l+1 (lane 63 <- 0)
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}

template <int N>
__device__ __forceinline__ void v5_wait_vm() {  // s_waitcnt vmcnt(N) (gfx9 encoding)
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

__device__ __forceinline__ void v5_barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}

// A barrier after this wave's own LDS stores (s_waitcnt lgkmcnt(0), then s_barrier).
// __syncthreads() here would also wait vmcnt(0): every DMA in flight, the prefetched
// planes included, drained at each plane.
__device__ __forceinline__ void v5_lds_barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(15 | (7 << 4) | (0 << 8) | (3 << 14));
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}

// MODE (diagnostic builds, apply only): 1 = memory only (the centre tap is stored,
// no arithmetic), 2 = arithmetic only (no DMA; the LDS ring is never filled).
// CP: cache policy bits -- 1: x DMAs nt, 2: b / x_in DMAs nt, 4: y stores nt,
// 8: nt on the x rows no other tile reads (x-tile rows 2P .. T1-1; the first and
// last 2P rows are the neighbouring tiles' halo and keep the default policy).
// XH: Jacobi x_in from the register history instead of a DMA next to b.
// ST16: every lane's store address is 16-B aligned (host-checked; always on the
// aligned layout): one 16-B store per lane, else two 8-B stores.
// JDOT: the Jacobi sweep also accumulates x_out . b (only the last sweep of a
// preconditioner call asks for it).
// Waves per workgroup (= output rows per tile): 16 at p <= 3 (4 waves per SIMD,
// 128 VGPRs).  p >= 4 needs more registers for its 2p+1 wide windows: 8 waves (2
// per SIMD, up to 256 VGPRs); the x tile is then 8 + 2p rows, up to 3 DMAs per
// wave.  The two-sweeps-from-zero build fits 16 waves at p = 3 with its two sums in
// LDS and x1 = s b scaled as the rows are read (round 3: on the row-Toeplitz tiles
// after the axis-1 pass; round 2 scaled the ring in place before each plane's
// barrier, 917 us at 515^3); at p <= 2 it keeps 8 waves (256^3 p = 2: 16 waves
// 154 us, 8 waves 136, v3 135-146; profiles/r02/j0_16wave/).
// (12 waves at 168 VGPRs fit the p = 5 apply but ran 254 us against 185 at 256^3,
// profiles/r02/configs/kb_p5_waves12.log vs kb_p5_waves8.log.)
// (Round 6: the p = 3 two-sweeps-from-zero build whose axis-1 / axis-2 Toeplitz rows
// differ -- two sets of constants -- spills at 16 waves; it runs 8-wave tiles, with its
// two running sums back in VGPRs, instead of falling back to v3.)
constexpr int v5_waves(int P, int EPI, bool SAME12 = true) {
    return ((P == 3 && (EPI != EPI_JACOBI0 || SAME12)) || (P < 3 && EPI != EPI_JACOBI0)) ? 16 : 8;
}

// Waves per SIMD the build must leave room for (__launch_bounds__): the p >= 4 apply
// with a 3-deep x ring runs two 8-wave workgroups per CU (78 KB of LDS, <= 128 VGPRs,
// no scratch) instead of one with a 4-deep ring: at 261^3 p = 5 183.8 -> 132.4 us,
// p = 4 146.2 -> 101.8 us (MALL-flushed kernel_bench medians, profiles/r06/p45/).  The
// p = 5 apply + dot spills at 128 VGPRs and keeps one workgroup per CU.
constexpr int v5_min_waves(int P, int EPI, int D) { return (P >= 4 && EPI == EPI_APPLY && D == 3) ? 4 : 1; }

template <int P, int EPI, int D, int MODE = 0, int CP = 0, bool XH = false, bool ST16 = true, bool JDOT = true,
          bool SAME12 = false>
__global__ void __launch_bounds__(64 * v5_waves(P, EPI, SAME12), v5_min_waves(P, EPI, D))
kron_v5_kernel(const double* __restrict__ x, double* __restrict__ y, const double* __restrict__ bvec,
               const double* __restrict__ a0t, const double* __restrict__ b0t,
               const double* __restrict__ a1, const double* __restrict__ b1,
               const double* __restrict__ a2, const double* __restrict__ b2,
               double* __restrict__ partial, double* __restrict__ partial2,
               const double* __restrict__ rdiag0, const KronGeom g, const ToepConst tc,
               const int H, const double omega) {
    constexpr int W = 2 * P + 1;
    constexpr int NW = v5_waves(P, EPI, SAME12);
    constexpr int T1 = NW;              // output rows per tile: one per wave
    constexpr int XR = T1 + 2 * P;      // x rows per plane tile
    constexpr int TC = 128;             // lane-columns per tile
    constexpr int NS = W;               // rotating axis-0 accumulators
    constexpr int PFX = D - 1;          // x prefetch distance (planes)
    constexpr bool HASB = (EPI == EPI_RESID) || (EPI == EPI_JACOBI);
    constexpr bool JAC = (EPI == EPI_JACOBI);
    constexpr bool APD = (EPI == EPI_APPLYDOT);
    // two sweeps from x = 0: the x ring holds b, scaled on the fly to x1 = omega b / diag
    constexpr bool J0 = (EPI == EPI_JACOBI0);
    constexpr bool HIST = APD || (JAC && XH) || J0;   // x (J0: x1) at the output point from a register history
    constexpr bool XIN = JAC && !XH;            // ... or DMA'd next to b (fewer VGPRs, 8 B/DOF more reads)
    constexpr bool ZR = J0;                     // zeroed rings + every-lane sums (see below)
    // Finished accumulator slots are not reset (the next plane's newest term starts
    // them) -- except in the plain Jacobi sweep, whose build then spills at 128 VGPRs
    // (round 5: 12 B of scratch; the hand-counted vmcnt waits forbid any)
    constexpr bool NORESET = !(JAC && !JDOT);
    // y stores: nt (bit 4), or sc1 (bit 16: written through, the line is dropped from
    // the XCD's L2 instead of kept -- leaves the L2 to the x halo rows the neighbouring
    // tiles re-read), or sc0 sc1 (bit 32)
    constexpr int XAUX = (CP & 1) ? 2 : 0, BAUX = (CP & 2) ? 2 : 0;
    constexpr int YAUX = (CP & 16) ? 16 : (CP & 32) ? 17 : (CP & 4) ? 2 : 0;
    constexpr int NWIN = 2 * P + 2;     // columns 2j-P .. 2j+1+P of a lane's pair
    constexpr int NXM = (XR + NW - 1) / NW;   // most x-row DMAs one wave issues per plane
    static_assert(NXM >= 2 && (NXM - 1) * NW < XR, "x tile rows vs waves");
    static_assert(D >= 3 || !HASB, "the b ring's wait count assumes x(t) was issued before b(t)");
    typedef double d2 __attribute__((ext_vector_type(2)));

    constexpr int XS_OFF = 0;
    // CP bit 64 (B3): b DMA'd two planes ahead through a 3-deep ring, each iteration
    // issuing x before b (so that b(t) landing still implies x(t), PFX = 2)
    constexpr bool B3 = HASB && (CP & 64) && !XIN && D == 3;   // (x_in DMA builds and deeper x rings keep the 2-deep b ring)
    constexpr int NB = B3 ? 3 : 2;      // b ring depth
    constexpr int BS_OFF = XS_OFF + D * XR * TC;
    constexpr int XI_OFF = BS_OFF + (HASB ? NB * T1 * TC : 0);
    constexpr int C2_OFF = XI_OFF + (XIN ? 2 * T1 * TC : 0);
    constexpr int RED_OFF = C2_OFF + 2 * W * TC;
    // Jacobi (register-history builds; the x_in ring leaves no room): 1/diag on the
    // axis-0 Toeplitz interior planes, one row per wave
    constexpr bool RCIL = JAC && XH;
    constexpr int RCI_OFF = RED_OFF + NW;
    // J0: omega/diag of every x-tile point on the axis-0 Toeplitz planes (XR rows) and
    // the axis-2 diagonal entries of the tile's columns
    constexpr int RS_OFF = RCI_OFF + (RCIL ? T1 * TC : 0);
    constexpr int D2_OFF = RS_OFF + (J0 ? XR * TC : 0);
    constexpr int D1_OFF = D2_OFF + (J0 ? 2 * TC : 0);   // J0: axis-1 diagonal entries of the x-tile rows
    // J0: per-lane running sums (||dr_2||^2, ||x1||^2) in LDS, not VGPRs: the 4
    // VGPRs they would pin for the whole march are what p = 3 lacks at 16 waves
    // (p = 3 only: the 8-wave builds of p <= 2 keep them in VGPRs, which they have)
    constexpr bool JSL = J0 && P == 3 && NW == 16;
    // J0 diagnostic builds (MODE 3: no sums, 4: no x1 scaling of the rows, 5: both;
    // results wrong by design -- timing only)
    constexpr bool J0NS = J0 && (MODE == 3 || MODE == 5);
    constexpr bool J0NX = J0 && (MODE == 4 || MODE == 5);
    constexpr int JS_OFF = (D1_OFF + (J0 ? 2 * XR : 0) + 1) & ~1;
    // J0: a row of ones, the post-axis-1 scale of the planes / tiles scaled in the ring
    constexpr int ONE_OFF = JS_OFF + (JSL ? 2 * NW * 64 : 0);
    constexpr int LDS_N = ONE_OFF + (J0 ? TC : 0);
    __shared__ __attribute__((aligned(16))) double lds[LDS_N];

    // SAME12: axis 2's Toeplitz rows equal axis 1's bitwise (one knot vector on both
    // axes): one set of constants held in SGPRs instead of two (the set the
    // compiler otherwise spilled into VGPR lanes, read back by v_readlane per plane)
#define T2A(k) (SAME12 ? tc.t1a[k] : tc.t2a[k])
#define T2B(k) (SAME12 ? tc.t1b[k] : tc.t2b[k])
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);

    const int nblk = gridDim.x;
    // tile of this workgroup: consecutive tiles on one XCD (round-robin dispatch over
    // the 8 XCDs), taken in the host's order within each XCD's range when g.sched is
    // set (longest tiles first, kron_v5_sched)
    // (g.sched holds the tile of each workgroup, then the tile's slot in the default
    // order: the partial sums keep that slot, so the reductions add in the same order
    // whatever the dispatch order.  Both are scalar loads where they are used, not
    // SGPRs held through the march.)
    auto tile_of = [&]() -> int {
        const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, x = b & 7;
        return g.sched != nullptr ? __builtin_amdgcn_readfirstlane(g.sched[b])
                                  : (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
    };
    auto slot_of = [&]() -> int {
        return g.sched != nullptr ? __builtin_amdgcn_readfirstlane(g.sched[gridDim.x + blockIdx.x]) : (int)blockIdx.x;
    };
    int bid = tile_of();
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
    const int orow = r0 + wv;           // this wave's output row
    const bool row_ok = orow < g.n1;
    const int cg0 = c0 - H + 2 * lane;  // interior column of this lane's element 0
    // output columns of this lane as a VGPR bit mask (lane-dependent bools would pin
    // two SGPRs each for the whole march; SGPR spills cost VGPR lanes)
    int cok = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const int ci = 2 * lane + e;
        cok |= (ci >= H && ci < H + TO && cg0 + e < g.n2) ? (1 << e) : 0;
    }
    const bool fast1 = orow >= tc.lo1 && orow < tc.hi1;                          // per wave
    const bool fast2 = (c0 >= tc.lo2) && (min(c0 + TO, g.n2) <= tc.hi2);         // per workgroup
    // J0 row-Toeplitz tile (per workgroup): every x-tile row has the Toeplitz axis-1
    // band, so omega/diag depends on the plane and the column only.  Such a tile (31
    // of 33 tile rows at 515^3) scales x1 = s b AFTER the axis-1 pass -- 4 multiplies
    // of u, v per lane and plane -- instead of scaling its x rows in the LDS ring in
    // place before the plane's barrier (a read-modify-write of the ring on the
    // critical path of every plane).
    const bool jrf = J0 && r0 - P >= tc.lo1 && r0 + T1 + P <= tc.hi1;

    // axis-2 band rows of the tile's columns (only outside the Toeplitz interior)
    if (!fast2) {
        for (int e = tid; e < W * TC; e += NW * 64) {
            const int k = e / TC, ci = e - k * TC;
            const int col = min(max(c0 - H + ci, 0), g.n2 - 1);
            lds[C2_OFF + e] = a2[col * W + k];
            lds[C2_OFF + W * TC + e] = b2[col * W + k];
        }
    }
    if constexpr (J0) {
        if (tid < TC) {
            const int col = min(max(c0 - H + tid, 0), g.n2 - 1);
            lds[D2_OFF + tid] = a2[col * W + P];
            lds[D2_OFF + TC + tid] = b2[col * W + P];
        }
        if (tid < XR) {   // x-tile row q = interior row r0 - P + q (clamped: ghost rows hold b = 0)
            const int row = min(max(r0 - P + tid, 0), g.n1 - 1);
            lds[D1_OFF + 2 * tid] = a1[row * W + P];
            lds[D1_OFF + 2 * tid + 1] = b1[row * W + P];
        }
    }
    // this wave's axis-1 band row (read by scalar loads where used: kept out of
    // SGPRs, which the per-plane axis-0 coefficients and Toeplitz constants fill)
    const int orc = min(orow, g.n1 - 1);
    const double* __restrict__ ra = a1 + orc * W;
    const double* __restrict__ rb = b1 + orc * W;
    auto rcp_nr = [](double dg) {   // 1/dg: v_rcp_f64 + two Newton steps
        double r = __builtin_amdgcn_rcp(dg);
        double ee = fma(-dg, r, 1.0);
        r = fma(r, ee, r);
        ee = fma(-dg, r, 1.0);
        return fma(r, ee, r);
    };
    // plane-invariant parts of diag(A) = d0a X + d0b Y at this lane's column e: the
    // wave's row by scalar loads, the column from the Toeplitz centre (fast2: every
    // output column is Toeplitz; other lanes are never stored) or the C2 table.
    // Recomputed where needed rather than held in 8 VGPRs across the march.
    auto diag_xy = [&](int e, double& X, double& Y) {
        const double d1a = ra[P], d1b = rb[P];
        const double d2a = fast2 ? T2A(0) : lds[C2_OFF + P * TC + 2 * lane + e];
        const double d2b = fast2 ? T2B(0) : lds[C2_OFF + (W + P) * TC + 2 * lane + e];
        X = d1a * d2a;
        Y = fma(d1b, d2a, d1a * d2b);
    };

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
    auto zo_of = [&](int t) { return max(z0 - 2 * P + t, z0); };
    // storage column of lane-column 0 (pads == P): c0 - H + P
    const int colb = (c0 - H + P) * 8 + 16 * lane;
    // Lane-columns no output point reads are not fetched: their voffset is pushed out
    // of the buffer range (+2^31; arrays are < 2 GiB), so the DMA moves no bytes.  x
    // needs the tile's columns H-P .. H+TO+P-1, b (and x_in, and the y stores) only
    // the output columns H .. H+TO-1: on the aligned layout that drops the two
    // half-lines of halo each b row fetched (8 of 64 lanes) and a quarter-line at
    // each end of every x row.
    // Past the last interior column the same holds (round 6): the last tile column's
    // lanes beyond n2 - 1 + P (x) or n2 - 1 (b) read only pitch padding and the next
    // row's first columns -- 25 of 64 lanes at 515^3 -- so they are not fetched either.
    // Their LDS slots keep an older plane's values; only lanes that are never stored
    // (and whose sums are masked) read them.
    const uint32_t colbx = (uint32_t)colb + ((2 * lane + 1 >= H - P && 2 * lane < H + TO + P && cg0 < g.n2 + P)
                                                 ? 0u : 0x80000000u);
    const uint32_t colbb = (uint32_t)colb + ((2 * lane + 1 >= H && 2 * lane < H + TO && cg0 < g.n2) ? 0u : 0x80000000u);
    // x-tile rows past the last storage row any output reads (n1 - 1 + 2P; the partial
    // last tile row at 515^3: 9 of its 22 rows) are not fetched either
    const int xrows_ok = g.n1 + 2 * P - r0;

    // ---- LDS-DMA issue (per wave per plane: x NXM - 1 or NXM rows, b 1 row) ----
    auto dma_x = [&](int m, int slot) {
        if constexpr (MODE == 2) return;
        const int sp = m + g.pd0;
        // planes outside the array (the dummies past the march) are out of range by
        // voffset: the soffset field is not covered by the buffer range check
        const bool ok = sp >= 0 && sp < nsp;
        const uint32_t so = ok ? (uint32_t)sp * plane8 : 0u;
        // x-tile row q = storage row r0 + q (rows q >= xrows_ok: out of range by voffset)
        const bool ok0 = ok && wv < xrows_ok;
        if ((CP & 8) && wv >= 2 * P)   // a row only this tile reads: stream it
            dma16s<2>(rx, lds + XS_OFF + (slot * XR + wv) * TC, ok0 ? (int)((uint32_t)((r0 + wv) * s1 * 8) + colbx) : 0x7ffffff0, so);
        else
            dma16s<XAUX>(rx, lds + XS_OFF + (slot * XR + wv) * TC, ok0 ? (int)((uint32_t)((r0 + wv) * s1 * 8) + colbx) : 0x7ffffff0, so);
#pragma unroll
        for (int i = 1; i < NXM; ++i)   // rows wv + i NW: every wave but the last on the tile's x rows
            if (i < NXM - 1 || wv < XR - (NXM - 1) * NW)
                dma16s<XAUX>(rx, lds + XS_OFF + (slot * XR + i * NW + wv) * TC,
                             (ok && i * NW + wv < xrows_ok) ? (int)((uint32_t)((r0 + i * NW + wv) * s1 * 8) + colbx)
                                                            : 0x7ffffff0, so);
    };
    auto dma_b = [&](int zo, int slot) {
        const uint32_t so = (uint32_t)(zo + g.pd0) * plane8;
        const int vob = row_ok ? (int)((uint32_t)((orow + P) * s1 * 8) + colbb) : 0x7ffffff0;   // (no output row: no b)
        dma16s<BAUX>(rbv, lds + BS_OFF + (slot * T1 + wv) * TC, vob, so);
        if constexpr (XIN) dma16s<BAUX>(rx, lds + XI_OFF + (slot * T1 + wv) * TC, vob, so);
    };

    double acc[NS][2];
#pragma unroll
    for (int s = 0; s < NS; ++s) { acc[s][0] = 0.0; acc[s][1] = 0.0; }
    double hist[HIST ? P : 1][2];
#pragma unroll
    for (int i = 0; i < (HIST ? P : 1); ++i) { hist[i][0] = 0.0; hist[i][1] = 0.0; }
    double nrm = 0.0, dotp = 0.0;
    constexpr bool STAMP = MODE == 6;
    unsigned long long st_wait = 0, st_bar = 0, st_rest = 0, st_prev = 0, st_t0 = 0;
    if constexpr (STAMP) {
        st_t0 = __builtin_amdgcn_s_memrealtime();
        st_prev = __builtin_amdgcn_s_memtime();
    }

    // J0 (ZR): the rings start zeroed, so lane-columns and rows no DMA fills hold
    // zeros, every lane's epilogue terms are finite, and the two running sums take
    // every lane of the wave, the lanes that are not output points being zeroed once
    // after the march (J0 829 -> 816 us, round 4).  The Jacobi sweep and apply + dot
    // keep the round-3 masked sums: with the zeroed rings the Jacobi build issued 3 %
    // more VALU and 10.6 % more wave cycles (SQ counters, r03 vs r04), 694.6 -> 709.5 us
    // in the driver's bench line (round-4 verdict).
    if constexpr (ZR && (MODE == 0 || MODE == 6)) {
        // (x ring, then b and x_in rings: contiguous from XS_OFF)
        static_assert(BS_OFF == XS_OFF + D * XR * TC && XI_OFF == BS_OFF + (HASB ? NB * T1 * TC : 0), "ring layout");
        constexpr int NZ = (XI_OFF + (XIN ? 2 * T1 * TC : 0) - XS_OFF) / 2;
#pragma unroll 1
        for (int e = tid; e < NZ; e += NW * 64) *(d2*)(lds + XS_OFF + 2 * e) = d2{0.0, 0.0};
    }
    __syncthreads();  // C2 table visible, rings zeroed; no DMA in flight yet
    // J0: omega/diag at x-tile row q, lane-column ci, of a plane with axis-0 diagonal
    // entries d0a, d0b (LDS tables only: no VMEM inside the march)
    auto j0_scale = [&](int q, int ci, double d0a, double d0b) {
        const double d1a = lds[D1_OFF + 2 * q], d1b = lds[D1_OFF + 2 * q + 1];
        const double d2a = lds[D2_OFF + ci], d2b = lds[D2_OFF + TC + ci];
        const double dg = fma(d0a, d1a * d2a, d0b * fma(d1b, d2a, d1a * d2b));
        return dg != 0.0 ? omega * rcp_nr(dg) : 0.0;   // zero diagonal: a ghost plane (b = 0)
    };
    if constexpr (J0) {
        for (int e = tid; e < XR * TC; e += NW * 64)
            lds[RS_OFF + e] = j0_scale(e / TC, e % TC, tc.t0a[0], tc.t0b[0]);
        if constexpr (JSL) *(d2*)(lds + JS_OFF + 2 * tid) = d2{0.0, 0.0};
        if (tid < TC) lds[ONE_OFF + tid] = 1.0;
        __syncthreads();
    }
    if constexpr (RCIL) {
        // on the axis-0 Toeplitz interior planes d0a, d0b are the Toeplitz centre
        // (bitwise), so omega/diag there is plane-invariant: computed once into LDS (two
        // more VGPRs would spill); each wave reads back only its own row
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            double X, Y;
            diag_xy(e, X, Y);
            lds[RCI_OFF + wv * TC + 2 * lane + e] = omega * rcp_nr(fma(tc.t0a[0], X, tc.t0b[0] * Y));
        }
    }

#pragma unroll
    for (int i = 0; i < PFX; ++i) dma_x(i < nplanes ? z0 - P + i : -(1 << 20), i);
    if constexpr (HASB) dma_b(zo_of(0), 0);
    if constexpr (B3) dma_b(zo_of(1), 1);

    const bool xtra = wv < XR - (NXM - 1) * NW;   // this wave issues NXM x DMAs per plane (else NXM - 1)
    for (int tb = 0; tb < nplanes; tb += NS) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int t = tb + q;
            if (t < nplanes) {
                unsigned long long st_a = 0;
                if constexpr (STAMP) {
                    st_a = __builtin_amdgcn_s_memtime();
                    st_rest += st_a - st_prev;
                }
                // ---- x(t) (and b(t)) landed: own DMAs by vmcnt, everyone's by the barrier.
                // Per iteration each wave issues, in order: b(t+1) [x_in(t+1)], x(t+PFX) (1 or
                // 2), 1 store.  Loads return in order, but a store may be acknowledged
                // before an older load returns, so the counts below are the LOADS issued
                // after the one waited for (stores never count): vmcnt <= that number
                // implies the load has landed.  Waiting for b(t) also covers x(t) (issued
                // before it, PFX >= 2).
                if constexpr (B3) {
                    // after b(t): x(t+1) and b(t+1) (the previous iteration's DMAs)
                    if (t == 0) v5_wait_vm<0>();
                    else if (xtra) v5_wait_vm<NXM + 1>();
                    else v5_wait_vm<NXM>();
                } else if constexpr (HASB) {
                    if (t == 0) v5_wait_vm<0>();
                    else if (xtra) v5_wait_vm<NXM>();
                    else v5_wait_vm<NXM - 1>();
                } else {
                    if (t < PFX) v5_wait_vm<0>();
                    else if (xtra) v5_wait_vm<(PFX - 1) * NXM>();
                    else v5_wait_vm<(PFX - 1) * (NXM - 1)>();
                }
                unsigned long long st_b = 0;
                if constexpr (STAMP) {
                    st_b = __builtin_amdgcn_s_memtime();
                    st_wait += st_b - st_a;
                }
                v5_barrier();
                // Every wave starts the plane at a high issue priority and drops it for
                // the plane's axis-0 scatter and epilogue.  A SIMD's four waves otherwise
                // run in age order: the oldest finishes each plane first and then waits
                // ~41 % of its cycles in the barrier, the youngest ~5 % (stamps), and the
                // end of every plane runs on one wave, its latencies exposed.
                __builtin_amdgcn_s_setprio(3);
                if constexpr (STAMP) {
                    st_prev = __builtin_amdgcn_s_memtime();
                    st_bar += st_prev - st_b;
                }
                if constexpr (B3) {
                    dma_x(t + PFX < nplanes ? z0 - P + t + PFX : -(1 << 20), (t + PFX) % D);
                    dma_b(min(zo_of(t + 2), z1), (t + 2) % 3);   // (clamped: the plane past the chunk is a dummy)
                } else {
                    if constexpr (HASB) dma_b(zo_of(t + 1), (t + 1) & 1);
                    dma_x(t + PFX < nplanes ? z0 - P + t + PFX : -(1 << 20), (t + PFX) % D);
                }

                // J0: the ring holds b; x1 = s b with s = omega / diag.  On a row-Toeplitz tile
                // (jrf) and a plane of the axis-0 Toeplitz interior s depends on the column only
                // and is applied after the axis-1 pass (below).  Elsewhere -- the two tile rows
                // at the axis-1 ends, and every tile on the P planes next to each global end --
                // the plane's rows are scaled in the ring in place (s from the LDS table, or
                // formed from the plane's axis-0 diagonal entries), behind a second barrier, and
                // the post-axis-1 scale is a row of ones.  (Scaling those rows in registers
                // instead made the compiler merge three versions of the 2P+1 rows at every
                // plane: 14 64-bit moves on the hot path, round 4.)
                bool jsc = false;
                if constexpr (J0 && !J0NX) {
                    const int m = g.g0 + z0 - P + t;   // global plane of x(t)
                    const bool tp = m >= tc.lo0 && m < tc.hi0;
                    jsc = jrf && tp;
                    if (!jsc) {
                        double* xsl = lds + XS_OFF + (t % D) * XR * TC;
                        if (tp) {
#pragma unroll 1
                            for (int e = tid; e < XR * TC / 2; e += NW * 64) {
                                d2 v = *(const d2*)(xsl + 2 * e);
                                const d2 s = *(const d2*)(lds + RS_OFF + 2 * e);
                                v[0] *= s[0];
                                v[1] *= s[1];
                                *(d2*)(xsl + 2 * e) = v;
                            }
                        } else {
                            const int i0 = (m + P) * W + P;
                            const double d0a = a0t[i0], d0b = b0t[i0];
#pragma unroll 1
                            for (int q = wv; q < XR; q += NW) {   // (row q uniform per wave)
                                d2 v = *(const d2*)(xsl + q * TC + 2 * lane);
                                v[0] *= j0_scale(q, 2 * lane, d0a, d0b);
                                v[1] *= j0_scale(q, 2 * lane + 1, d0a, d0b);
                                *(d2*)(xsl + q * TC + 2 * lane) = v;
                            }
                        }
                        v5_lds_barrier();   // (not __syncthreads: that drained the DMAs in flight)
                    }
                }
                // A wave whose output row lies past the slab's last row (13 of the 16 in
                // the partial last tile row at 515^3) only issues its DMAs and takes the
                // barriers: its points are never stored, and its sums are not kept.
                if (MODE != 2 && !row_ok) continue;
                // ---- axis 1: u = F1a x, v = F1b x on this wave's row, 2 columns per lane
                const double* xs = lds + XS_OFF + (t % D) * XR * TC + 2 * lane;
                d2 xv[W];
#pragma unroll
                for (int k = 0; k < W; ++k) xv[k] = *(const d2*)(xs + (wv + k) * TC);
                if constexpr (MODE == 1) {
                    const bool ok0 = t >= 2 * P && row_ok && (cok & 1);
                    bstore2_sp<YAUX>(ry, ok0 ? (orow + P) * s1 * 8 + colb + (zo_of(t) + g.pd0) * (int)plane8 : 0x7ffffff0,
                                     0u, xv[P][0] + xv[0][0], xv[P][1] + xv[W - 1][1]);
                    continue;
                }
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
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        double su = ra[0] * xv[0][e], sv = rb[0] * xv[0][e];
#pragma unroll
                        for (int k = 1; k < W; ++k) {
                            su = fma(ra[k], xv[k][e], su);
                            sv = fma(rb[k], xv[k][e], sv);
                        }
                        u[e] = su;
                        v[e] = sv;
                    }
                }
                if constexpr (J0 && !J0NX) {
                    // x1 = s(column) b: the scaling commutes with the axis-1 pass (every table
                    // row is equal on a jsc plane); ones where the ring holds x1 already (x 1.0
                    // is exact), so that no path merges register copies
                    static_assert(RS_OFF % 2 == 0 && ONE_OFF % 2 == 0, "16-B aligned scale rows");
                    const int so = __builtin_amdgcn_readfirstlane(jsc ? RS_OFF / 2 : ONE_OFF / 2);
                    const d2 sc = reinterpret_cast<const d2*>(lds)[so + lane];   // (one 16-B read)
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        u[e] *= sc[e];
                        v[e] *= sc[e];
                        xv[P][e] *= sc[e];   // the centre tap the x1 history keeps
                    }
                }

                // ---- axis 2: column windows by whole-lane DPP shifts (2 columns per lane)
                double wu[NWIN], wvv[NWIN];
                wu[P] = u[0];
                wu[P + 1] = u[1];
                wvv[P] = v[0];
                wvv[P + 1] = v[1];
#pragma unroll
                for (int i = P - 1; i >= 0; --i) {
                    wu[i] = v5_shr1(wu[i + 2]);
                    wvv[i] = v5_shr1(wvv[i + 2]);
                }
#pragma unroll
                for (int i = P + 2; i <= 2 * P + 1; ++i) {
                    wu[i] = v5_shl1(wu[i - 2]);
                    wvv[i] = v5_shl1(wvv[i - 2]);
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

                __builtin_amdgcn_s_setprio(0);
                // ---- axis 0: scatter into the rotating slots (column gm of the factors;
                // scalar loads -- taking the Toeplitz constants from the kernel arguments
                // instead ran slower: they no longer fit the SGPRs and are re-loaded)
                const int jrow = (g.g0 + z0 - P + t + P) * W;
#pragma unroll
                for (int s = 0; s < W; ++s) {
                    const int slot = (q - P + s + NS) % NS;
                    const double ka = a0t[jrow + s];
                    const double kb = b0t[jrow + s];
                    // the newest slot (s = 2P) is the one finished at the previous plane: its
                    // first term starts it (kb dd == fma(kb, dd, +0) up to the sign of a zero),
                    // so finished slots need no reset (NORESET: 2 64-bit moves less per plane)
                    if (NORESET && s == 2 * P) {
#pragma unroll
                        for (int e = 0; e < 2; ++e) acc[slot][e] = fma(ka, cc[e], kb * dd[e]);
                    } else {
#pragma unroll
                        for (int e = 0; e < 2; ++e) acc[slot][e] = fma(ka, cc[e], fma(kb, dd[e], acc[slot][e]));
                    }
                }
                const int done = (q + P + 1) % NS;
                double vo[2] = {acc[done][0], acc[done][1]};
                if constexpr (!NORESET) {
                    acc[done][0] = 0.0;
                    acc[done][1] = 0.0;
                }
                const bool en = t >= 2 * P;
                const int zo = zo_of(t);

                // ---- epilogue of the finished plane zo
                double xin[2] = {0.0, 0.0};
                if constexpr (HIST) {
                    xin[0] = hist[0][0];
                    xin[1] = hist[0][1];
#pragma unroll
                    for (int i = 0; i + 1 < P; ++i) { hist[i][0] = hist[i + 1][0]; hist[i][1] = hist[i + 1][1]; }
                    hist[P - 1][0] = xv[P][0];
                    hist[P - 1][1] = xv[P][1];
                }
                bool ok[2];
#pragma unroll
                for (int e = 0; e < 2; ++e) ok[e] = en && row_ok && ((cok >> e) & 1);
                double outv[2];
                if constexpr (EPI == EPI_APPLY) {
                    outv[0] = vo[0];
                    outv[1] = vo[1];
                } else if constexpr (APD) {
                    outv[0] = vo[0];
                    outv[1] = vo[1];
#pragma unroll
                    for (int e = 0; e < 2; ++e) dotp = ok[e] ? fma(xin[e], outv[e], dotp) : dotp;
                } else if constexpr (J0) {
                    // x1 = s b, x2 = x1 + s (b - A x1) = x1 + (x1 - s A x1), s = omega/diag;
                    // xin = x1 at the output point (the scaled centre tap)
                    const int m = g.g0 + zo;
                    double sc[2];
                    if (m >= tc.lo0 && m < tc.hi0) {
                        const d2 r = *(const d2*)(lds + RS_OFF + (wv + P) * TC + 2 * lane);
                        sc[0] = r[0];
                        sc[1] = r[1];
                    } else {
                        const int i0 = (m + P) * W + P;
                        const double d0a = a0t[i0], d0b = b0t[i0];
                        sc[0] = j0_scale(wv + P, 2 * lane, d0a, d0b);
                        sc[1] = j0_scale(wv + P, 2 * lane + 1, d0a, d0b);
                    }
                    double dr[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        dr[e] = fma(-vo[e], sc[e], xin[e]);
                        outv[e] = xin[e] + dr[e];
                    }
                    // The running sums (||dr_2||^2, ||x1||^2 = ||dr_1||^2) take every lane of the
                    // wave on the output planes (en: uniform) and the lanes that are not output
                    // columns, or whose wave's row is past n1, are zeroed once after the march.
                    // Their terms are finite: the x ring starts zeroed, so the lane-columns no DMA
                    // fills hold zeros.  Only a lane whose second column lies past n2 (odd n2, the
                    // last tile column) masks its second terms, as 0 * 0 (the sums are >= 0, so
                    // + 0 is exact): the same sums, term for term, as masking every term.
                    if constexpr (!J0NS) {
                        if (en) {
                            d2 js = {nrm, dotp};
                            if constexpr (JSL) js = *(const d2*)(lds + JS_OFF + 2 * tid);   // this lane's own slot
                            js[0] = fma(dr[0], dr[0], js[0]);
                            js[1] = fma(xin[0], xin[0], js[1]);
                            const double dr1 = (cok & 2) ? dr[1] : 0.0, x11 = (cok & 2) ? xin[1] : 0.0;
                            js[0] = fma(dr1, dr1, js[0]);
                            js[1] = fma(x11, x11, js[1]);
                            if constexpr (JSL) {
                                *(d2*)(lds + JS_OFF + 2 * tid) = js;
                            } else {
                                nrm = js[0];
                                dotp = js[1];
                            }
                        }
                    }
                } else {
                    const d2 bv = *(const d2*)(lds + BS_OFF + ((t % NB) * T1 + wv) * TC + 2 * lane);
                    if constexpr (EPI == EPI_RESID) {
                        outv[0] = bv[0] - vo[0];
                        outv[1] = bv[1] - vo[1];
                    } else {
                        if constexpr (XIN) {
                            const d2 xi = *(const d2*)(lds + XI_OFF + ((t & 1) * T1 + wv) * TC + 2 * lane);
                            xin[0] = xi[0];
                            xin[1] = xi[1];
                        }
                        double rc[2];
                        if (fast1 && fast2 && rdiag0 != nullptr) {
                            rc[0] = rc[1] = omega * rdiag0[g.g0 + zo];   // one multiply per plane
                        } else if (RCIL && g.g0 + zo >= tc.lo0 && g.g0 + zo < tc.hi0) {
                            const d2 ri = *(const d2*)(lds + RCI_OFF + wv * TC + 2 * lane);
                            rc[0] = ri[0];
                            rc[1] = ri[1];
                        } else {
                            const int i0 = (g.g0 + zo + P) * W + P;
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
                            const double drm = ok[e] ? dr : 0.0;   // (nrm >= 0: + 0 * 0 is exact)
                            nrm = fma(drm, drm, nrm);
                            if constexpr (JDOT) dotp = ok[e] ? fma(outv[e], bv[e], dotp) : dotp;
                        }
                    }
                }
                // one 16-B store per lane when 16-B aligned (ST16: the aligned layout); a
                // lane whose second column lies past n2 (a ghost or dead pitch column)
                // writes 0 there, which keeps ghosts zero.  Otherwise two 8-B stores.
                // The plane offset goes into voffset with soffset = 0: gfx950 needs a wait
                // state before a VALU overwrites the data VGPRs of a >8-B store, and the
                // compiler only inserts it when soffset is not a register (with an SGPR
                // soffset the next plane's accumulator reset raced the store and zeroed
                // lanes 12-15 of each row: tools/diag_v5_fullsize.py).
                const bool any = (ok[0] || ok[1]) && (MODE != 2 || outv[0] == 12345.678);
                const double o1 = ok[1] ? outv[1] : 0.0;
                const int voy = (orow + P) * s1 * 8 + colb + (zo + g.pd0) * (int)plane8;
                if constexpr (ST16) {
                    bstore2_sp<YAUX>(ry, any ? voy : 0x7ffffff0, 0u, outv[0], o1);
                } else {
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, outv[0]), ry,
                                                          ok[0] ? voy : 0x7ffffff0, 0, YAUX);
                    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o1), ry,
                                                          any ? voy + 8 : 0x7ffffff0, 0, YAUX);
                }
            }
        }
    }
    v5_wait_vm<0>();  // no LDS-DMA may outlive the workgroup
    if constexpr (STAMP) {
        st_rest += __builtin_amdgcn_s_memtime() - st_prev;
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        const int slot = (blockIdx.x * NW + wv) * 8;
        if (lane < 8 && slot + 8 <= kV5Stamps) {
            unsigned hw;
            __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            unsigned xcc;
            __asm__ volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            const unsigned long long v = lane == 0 ? st_wait : lane == 1 ? st_bar : lane == 2 ? st_rest
                                       : lane == 3 ? (unsigned long long)nplanes : lane == 4 ? st_t0
                                       : lane == 5 ? t1 : lane == 6 ? ((unsigned long long)(xcc & 15) | ((unsigned long long)tile_of() << 8))
                                       : (unsigned long long)(((hw >> 8) & 15) | (((hw >> 13) & 7) << 4));
            g_v5_stamps[slot + lane] = v;
        }
    }
    if constexpr (JSL) {
        const d2 js = *(const d2*)(lds + JS_OFF + 2 * tid);
        nrm = js[0];
        dotp = js[1];
    }
    if constexpr (ZR && !J0NS) {   // the lanes whose terms are not output points
        if (!(row_ok && (cok & 1))) {
            nrm = 0.0;
            dotp = 0.0;
        }
    }

    if constexpr (JAC || APD || J0) {
        if (partial != nullptr) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nrm += __shfl_xor(nrm, off, 64);
            __syncthreads();
            if (lane == 0) lds[RED_OFF + wv] = nrm;
            __syncthreads();
            if (tid == 0) {
                double s = 0.0;
                for (int w = 0; w < NW; ++w) s += lds[RED_OFF + w];
                partial[slot_of()] = s;
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
                partial2[slot_of()] = s;
            }
        }
    }
}

#undef T2A
#undef T2B

// Timing events for the next v5 launch of this thread (op_run's sampled timing):
// passed to hipExtLaunchKernel, which stamps the dispatch's own start and end.
static thread_local hipEvent_t t_v5_ev0 = nullptr, t_v5_ev1 = nullptr;
static thread_local bool t_v5_ev_used = false;

void kron_v5_set_launch_events(hipEvent_t e0, hipEvent_t e1) {
    t_v5_ev0 = e0;
    t_v5_ev1 = e1;
    t_v5_ev_used = false;
}

bool kron_v5_launch_events_used() { return t_v5_ev_used; }

template <int P, int EPI, int D, int MODE, int CP, bool XH, bool ST16, bool JDOT, bool SAME12>
static int v5_launch_t2(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                        hipStream_t st) {
    // the hand-counted vmcnt waits assume the only VMEM ops in the loop are the
    // DMAs and the store: a build that spills to scratch would break them
    static int scratch = -1;
    if (scratch < 0) {
        hipFuncAttributes at{};
        if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&kron_v5_kernel<P, EPI, D, MODE, CP, XH, ST16, JDOT, SAME12>)) != hipSuccess) {
            set_error("v5: hipFuncGetAttributes failed");
            return 1;
        }
        scratch = (int)at.localSizeBytes;
    }
    if (scratch > 0) {
        set_error("v5: kernel build spills to scratch (vmcnt counting invalid)");
        return 1;
    }
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    if (t_v5_ev0 != nullptr) {   // a timed launch: the events on the dispatch itself
        hipExtLaunchKernelGGL((kron_v5_kernel<P, EPI, D, MODE, CP, XH, ST16, JDOT, SAME12>), dim3(nblk),
                              dim3(64 * v5_waves(P, EPI, SAME12)), 0, st, t_v5_ev0, t_v5_ev1, 0, p.x, p.y, p.b, p.a0t,
                              p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, p.rdiag0, g, tc, H, omega);
        t_v5_ev0 = t_v5_ev1 = nullptr;
        t_v5_ev_used = true;
        return 0;
    }
    hipLaunchKernelGGL((kron_v5_kernel<P, EPI, D, MODE, CP, XH, ST16, JDOT, SAME12>), dim3(nblk), dim3(64 * v5_waves(P, EPI, SAME12)), 0, st, p.x,
                       p.y, p.b, p.a0t, p.b0t, p.a1, p.b1, p.a2, p.b2, p.partial, p.partial2, p.rdiag0, g, tc, H, omega);
    return 0;
}

template <int P, int EPI, int D, int MODE = 0, int CP = 0, bool XH = false, bool ST16 = true, bool JDOT = true>
static int v5_launch_t1(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                        hipStream_t st) {
    bool same = true;   // the axis-1 / axis-2 Toeplitz rows, bitwise
    for (int k = 0; k <= P; ++k)
        same = same && tc.t1a[k] == tc.t2a[k] && tc.t1b[k] == tc.t2b[k];
    if constexpr (MODE != 0) {   // diagnostic builds: the cubic headline grid only
        if (!same) { set_error("v5 diag mode: needs equal axis-1 / axis-2 Toeplitz rows"); return 1; }
        return v5_launch_t2<P, EPI, D, MODE, CP, XH, ST16, JDOT, true>(p, g, tc, H, omega, st);
    }
    return same ? v5_launch_t2<P, EPI, D, MODE, CP, XH, ST16, JDOT, true>(p, g, tc, H, omega, st)
                : v5_launch_t2<P, EPI, D, MODE, CP, XH, ST16, JDOT, false>(p, g, tc, H, omega, st);
}

// 16-B stores only where every lane's store address is 16-B aligned
template <int P, int EPI, int D, int MODE = 0, int CP = 0, bool XH = false>
static int v5_launch_t(const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    // (the p = 3 two-sweeps-from-zero build with distinct axis-1 / axis-2 Toeplitz
    // rows spills at 16 waves; resolve_variant leaves that case to v3)
    const bool st16 = ((reinterpret_cast<uintptr_t>(p.y) + 8 * (int64_t)(g.pd2 - H)) & 15) == 0 &&
                      g.s1 % 2 == 0 && g.s0 % 2 == 0;
    // the Jacobi x_in history does not fit the VGPRs beside the split stores: the
    // unaligned build DMAs x_in next to b instead
    constexpr bool XHU = (EPI == EPI_JACOBI) ? false : XH;
    // (the x_in DMA build has no LDS room for a 4th x plane at p = 3)
    constexpr int DU = (EPI == EPI_JACOBI && D > 3) ? 3 : D;
    if (EPI == EPI_JACOBI && p.partial2 == nullptr)
        return st16 ? v5_launch_t1<P, EPI, D, MODE, CP, XH, true, false>(p, g, tc, H, omega, st)
                    : v5_launch_t1<P, EPI, DU, MODE, CP, XHU, false, false>(p, g, tc, H, omega, st);
    return st16 ? v5_launch_t1<P, EPI, D, MODE, CP, XH, true>(p, g, tc, H, omega, st)
                : v5_launch_t1<P, EPI, DU, MODE, CP, XHU, false>(p, g, tc, H, omega, st);
}

// y-store cache policy of the apply / Jacobi builds (tuning: POMS_V5_STORE = 0 nt,
// 1 sc1, 2 sc0 sc1)
static int store_policy() {
    static int sp = -1;
    if (sp < 0) {
        const char* e = getenv("POMS_V5_STORE");
        sp = e ? atoi(e) : 0;
        if (sp < 0 || sp > 2) sp = 0;
    }
    return sp;
}

template <int P>
static int v5_launch_p(int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H, double omega,
                       hipStream_t st) {
    switch (epi) {
        // non-temporal y stores and b DMAs; Jacobi x_in from the register history
        // (tools/kernel_bench.py, variants 103-106 at 515^3: apply 555 -> 534 us,
        // residual 713 -> 672, Jacobi 886 -> 777; nt x DMAs cost 15 %: the halo rows
        // are re-read by the neighbouring tiles)
        // apply: also nt on the x rows no other tile reads (variant 109: 568 -> 539 us)
        // residual: b two planes ahead through a 3-deep ring (CP bit 64; on the Jacobi
        // sweep 749 -> 739 us in kernel_bench, 731 -> 716 us inside the V-cycle at 515^3,
        // profiles/r02/b3/).  Jacobi: a 4-deep x ring (x three planes ahead) with the
        // 2-deep b ring instead -- both do not fit the LDS -- 737-748 -> 729-735 us
        // against the 3-deep b ring on one box (profiles/r02/ring_depth/); the unaligned
        // x_in build keeps 3 x planes and the 3-deep b ring.
        // (round 2 closing: the default policy on those rows after all -- variant 104
        // vs 10 interleaved on one box, median 548-550 vs 583-621 us, equal minima;
        // the streamed rows made the apply's time scatter, profiles/r02/j0ab/)
        case EPI_APPLY:
            // p >= 4: a 3-deep x ring, two workgroups per CU (v5_min_waves)
            if constexpr (P >= 4) return v5_launch_t<P, EPI_APPLY, 3, 0, 6>(p, g, tc, H, omega, st);
            if (store_policy() == 1) return v5_launch_t<P, EPI_APPLY, 4, 0, 2 | 16>(p, g, tc, H, omega, st);
            if (store_policy() == 2) return v5_launch_t<P, EPI_APPLY, 4, 0, 2 | 32>(p, g, tc, H, omega, st);
            return v5_launch_t<P, EPI_APPLY, 4, 0, 6>(p, g, tc, H, omega, st);
        case EPI_RESID: return v5_launch_t<P, EPI_RESID, 3, 0, 6 | 64>(p, g, tc, H, omega, st);
        case EPI_JACOBI:   // (the sc1 / sc0 sc1 store builds of round 2 no longer fit 128 VGPRs with the
                           // zeroed rings: POMS_V5_STORE applies to the apply only)
            return v5_launch_t<P, EPI_JACOBI, 4, 0, 6 | 64, true>(p, g, tc, H, omega, st);
        case EPI_APPLYDOT: return v5_launch_t<P, EPI_APPLYDOT, 4, 0, 6>(p, g, tc, H, omega, st);
        // x ring = b (read once, apply's policy), scaled to x1 as it is read; y = x2
        // streamed
        case EPI_JACOBI0: return v5_launch_t<P, EPI_JACOBI0, 4, 0, 14>(p, g, tc, H, omega, st);
    }
    set_error("v5: epilogue not built");
    return 1;
}

// Tile geometry for the v5 kernel: halo lane-columns H on the left and output
// columns TO per tile.  Line-aligned (interior column 0 of every row on a 128-B
// line, pitch a multiple of 16): H = 8, TO = 112, so every stored row segment is
// whole lines.  Otherwise H = P rounded up to even, TO = 128 - 2H.
void kron_v5_tile(int pmax, bool aligned, int* H, int* TO) {
    if (aligned && pmax <= 8) {
        *H = 8;
        *TO = 112;
    } else {
        *H = (pmax + 1) & ~1;
        *TO = 128 - 2 * *H;
    }
}

// Dispatch order of a launch's tiles (KronGeom::sched).  The hardware hands
// workgroup b to XCD b % 8, and each XCD starts its workgroups in order, one per CU
// as CUs free up (round-robin over its 4 shader engines; r05 stamps,
// tools/v5_stamps.py --raw).  The default order gives each XCD a contiguous range
// of tiles; a range that ends on its slowest tiles -- at 515^3 the two-sweeps-from-
// zero tile rows off the axis-1 Toeplitz interior, 1.2-1.5x the others -- runs them
// in the grid's last round and stretches its tail.  This table keeps each XCD's
// range and starts its tiles in order of decreasing estimated duration (stable:
// equal tiles keep the default order, neighbours together on the XCD's L2).  The
// estimate is the tile's planes (halo included) times the measured factors of its
// slow paths.  Built once per geometry and device, outside any graph capture (a
// launch during a capture that has no table yet keeps the default order).
// POMS_V5_SCHED=0 turns it off.
int kron_v5_rows(int pmax, int epi, int same12);

static std::atomic<int> g_v5_sched{-1};

int kron_v5_set_sched(int mode) {   // poms_diag_v5_sched
    if (g_v5_sched.load() < 0) {
        const char* e = getenv("POMS_V5_SCHED");
        g_v5_sched = e ? (atoi(e) ? 1 : 0) : 1;
    }
    const int prev = g_v5_sched.load();
    if (mode >= 0) g_v5_sched = mode ? 1 : 0;
    return prev;
}

static const int* v5_sched(int P, int epi, const KronGeom& g, const ToepConst& tc, hipStream_t st) {
    const int mode = kron_v5_set_sched(-1);
    const int nblk = g.tiles2 * g.tiles1 * g.nchunks;
    if (mode == 0 || nblk < 16) return nullptr;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    const std::vector<int> key = {dev, P, epi, g.n0, g.n1, g.n2, g.g0, g.z_begin, g.z_end, g.z2_begin, g.z2_end,
                                  g.chunk, g.nch1, g.nchunks, g.tiles1, g.tiles2, g.tout, g.order,
                                  tc.lo0, tc.hi0, tc.lo1, tc.hi1, tc.lo2, tc.hi2};
    // a table is uploaded on the stream of the launch that built it; a launch on another
    // stream waits for the upload's event (advisor, round 5: it could otherwise read the
    // table before the copy landed) until the event is seen complete
    struct Table {
        int* d = nullptr;
        hipEvent_t ev = nullptr;
        hipStream_t st = nullptr;
        bool landed = false;
    };
    static std::mutex mu;
    static std::map<std::vector<int>, Table> cache;
    std::lock_guard<std::mutex> lk(mu);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess) return nullptr;
    auto it = cache.find(key);
    if (it != cache.end()) {
        Table& tb = it->second;
        if (!tb.landed) {
            // inside a capture no event may be queried or waited on (that invalidates
            // the capture): a table not yet seen landed is not used there -- the default
            // order gives the same results bitwise (the partial sums keep their slots)
            if (cs != hipStreamCaptureStatusNone) return nullptr;
            if (hipEventQuery(tb.ev) == hipSuccess) {
                tb.landed = true;
            } else {
                (void)hipGetLastError();
                if (st != tb.st && hipStreamWaitEvent(st, tb.ev, 0) != hipSuccess) {
                    (void)hipGetLastError();
                    return nullptr;
                }
            }
        }
        return tb.d;
    }
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    bool same12 = true;
    for (int k = 0; k <= P; ++k) same12 = same12 && tc.t1a[k] == tc.t2a[k] && tc.t1b[k] == tc.t2b[k];
    const int T1 = kron_v5_rows(P, epi, same12 ? 1 : 0), TO = g.tout;
    const bool j0 = epi == EPI_JACOBI0;
    std::vector<double> w(nblk);
    for (int b = 0; b < nblk; ++b) {
        int r = b, t1, t2;
        if (g.order) { t1 = r % g.tiles1; r /= g.tiles1; t2 = r % g.tiles2; r /= g.tiles2; }
        else { t2 = r % g.tiles2; r /= g.tiles2; t1 = r % g.tiles1; r /= g.tiles1; }
        const int ch = r;
        int z0, z1;   // (chunk_planes)
        if (ch < g.nch1) { z0 = g.z_begin + ch * g.chunk; z1 = std::min(z0 + g.chunk, g.z_end); }
        else { z0 = g.z2_begin + (ch - g.nch1) * g.chunk; z1 = std::min(z0 + g.chunk, g.z2_end); }
        const int r0 = t1 * T1, c0 = t2 * TO;
        double f = 1.0;
        // measured (r05 stamps, 515^3 p = 3): general axis-2 column tiles +11 % (J0) / +5 %;
        // J0 tiles that scale the ring in place +20 %, the partial last tile row +50 %
        if (!(c0 >= tc.lo2 && std::min(c0 + TO, g.n2) <= tc.hi2)) f += j0 ? 0.11 : 0.05;
        if (j0 && !(r0 - P >= tc.lo1 && r0 + T1 + P <= tc.hi1)) f += 0.2;
        if (j0 && r0 + T1 > g.n1) f += 0.3;
        w[b] = (double)(z1 - z0 + 2 * P) * f;
    }
    // [0, nblk): the tile of workgroup b; [nblk, 2 nblk): that tile's slot in the
    // default order (workgroup k * 8 + x runs tile lo(x) + k)
    std::vector<int> h(2 * (size_t)nblk);
    const int q = nblk >> 3, rr = nblk & 7;
    for (int x = 0; x < 8; ++x) {
        const int lo = x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q, cnt = x < rr ? q + 1 : q;
        std::vector<int> idx(cnt);
        for (int k = 0; k < cnt; ++k) idx[k] = lo + k;
        std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return w[a] > w[b]; });
        for (int k = 0; k < cnt; ++k) {
            h[k * 8 + x] = idx[k];
            h[nblk + k * 8 + x] = (idx[k] - lo) * 8 + x;
        }
    }
    // stream-ordered allocation and upload on the launch's stream (no device-wide
    // synchronisation: another stream may hold a peer exchange waiting on a
    // neighbour); the host copy stays alive with the table
    static std::map<std::vector<int>, std::vector<int>> host;
    int* d = nullptr;
    if (hipMallocAsync(reinterpret_cast<void**>(&d), h.size() * sizeof(int), st) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    std::vector<int>& hk = host[key];
    hk = std::move(h);
    if (hipMemcpyAsync(d, hk.data(), hk.size() * sizeof(int), hipMemcpyHostToDevice, st) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipFreeAsync(d, st);
        host.erase(key);
        return nullptr;
    }
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess || hipEventRecord(ev, st) != hipSuccess) {
        (void)hipGetLastError();
        if (ev) (void)hipEventDestroy(ev);
        (void)hipFreeAsync(d, st);
        host.erase(key);
        return nullptr;
    }
    cache[key] = Table{d, ev, st, false};
    return d;
}

int kron_v5_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g_in, const ToepConst& tc, int H,
                   double omega, hipStream_t st, int diag_mode) {
    KronGeom g = g_in;
    g.sched = v5_sched(pmax, epi, g_in, tc, st);
    if (H < pmax || (H & 1) || (g.tout & 1) || H + g.tout + pmax > 128) {
        set_error("v5: bad tile geometry");
        return 1;
    }
#ifndef POMS_V5_QUICK   // (POMS_V5_QUICK: p = 3 production builds only, for quick tuning builds)
    if (diag_mode) {   // DIAGNOSTIC / tuning builds (p = 3)
        if (pmax != 3) { set_error("v5 diag mode: p = 3 only"); return 1; }
        if (diag_mode == 13) {   // Jacobi sweep (production ring depths) + nt on the x rows no other tile reads
            if (epi != EPI_JACOBI) { set_error("v5 diag mode 13: Jacobi only"); return 1; }
            return v5_launch_t<3, EPI_JACOBI, 4, 0, 14 | 64, true>(p, g, tc, H, omega, st);
        }
        if (diag_mode >= 10 && diag_mode <= 12) {   // two sweeps from zero: 10 no sums, 11 no x1 scaling, 12 both
            if (epi != EPI_JACOBI0) { set_error("v5 diag mode 10-12: two sweeps from zero only"); return 1; }
            return diag_mode == 10 ? v5_launch_t<3, EPI_JACOBI0, 4, 3, 14>(p, g, tc, H, omega, st)
                 : diag_mode == 11 ? v5_launch_t<3, EPI_JACOBI0, 4, 4, 14>(p, g, tc, H, omega, st)
                                   : v5_launch_t<3, EPI_JACOBI0, 4, 5, 14>(p, g, tc, H, omega, st);
        }
        if (diag_mode == 14) {   // stamped march (MODE 6): apply, or the Jacobi sweep's / J0's production build
            if (epi == EPI_APPLY) return v5_launch_t<3, EPI_APPLY, 4, 6, 6>(p, g, tc, H, omega, st);
            if (epi == EPI_JACOBI) return v5_launch_t<3, EPI_JACOBI, 4, 6, 6 | 64, true>(p, g, tc, H, omega, st);
            if (epi == EPI_JACOBI0) return v5_launch_t<3, EPI_JACOBI0, 4, 6, 14>(p, g, tc, H, omega, st);
            set_error("v5 diag mode 14: apply / Jacobi / two sweeps from zero only");
            return 1;
        }
        if (diag_mode <= 2) {   // 1 = memory only, 2 = arithmetic only (apply)
            if (epi != EPI_APPLY) { set_error("v5 diag mode 1/2: apply only"); return 1; }
            return diag_mode == 1 ? v5_launch_t<3, EPI_APPLY, 4, 1, 6>(p, g, tc, H, omega, st)   // (the apply's cache policy)
                                  : v5_launch_t<3, EPI_APPLY, 4, 2>(p, g, tc, H, omega, st);
        }
#define V5CP(CP, XH)                                                                               \
        switch (epi) {                                                                             \
            case EPI_APPLY: return v5_launch_t<3, EPI_APPLY, 4, 0, CP, XH>(p, g, tc, H, omega, st);   \
            case EPI_RESID: return v5_launch_t<3, EPI_RESID, 3, 0, CP, XH>(p, g, tc, H, omega, st);   \
            case EPI_JACOBI: return v5_launch_t<3, EPI_JACOBI, 3, 0, CP, XH>(p, g, tc, H, omega, st); \
        }                                                                                          \
        break;
        switch (diag_mode) {   // 3: nt y stores; 4: + nt b / x_in; 5: + nt x; 6: 3 + Jacobi x_in history;
                               // 7: default policy everywhere; 8: nt b only
            case 3: V5CP(4, false)
            case 4: V5CP(6, false)
            case 5: V5CP(7, false)
            case 6: V5CP(4, true)
            case 7: V5CP(0, false)
            case 8: V5CP(2, false)
            case 9: V5CP(14, true)   // default + nt on the rows no other tile reads
        }
#undef V5CP
        set_error("v5 diag mode: bad mode / epilogue");
        return 1;
    }
#endif
    switch (pmax) {
#ifndef POMS_V5_QUICK
        case 1: return v5_launch_p<1>(epi, p, g, tc, H, omega, st);
        case 2: return v5_launch_p<2>(epi, p, g, tc, H, omega, st);
        case 4: return v5_launch_p<4>(epi, p, g, tc, H, omega, st);   // 8-wave tiles
        case 5: return v5_launch_p<5>(epi, p, g, tc, H, omega, st);
#endif
        case 3: return v5_launch_p<3>(epi, p, g, tc, H, omega, st);
    }
    set_error("v5: pmax must be in 1..5");
    return 1;
}

int kron_v5_rows(int pmax, int epi, int same12) { return v5_waves(pmax, epi, same12 != 0); }

// MODE 6 stamps: copy n u64 (<= kV5Stamps) to host (zeroed after the copy)
int kron_v5_stamps(unsigned long long* host, int64_t n) {
    if (n < 0 || n > kV5Stamps) { set_error("v5 stamps: bad count"); return 1; }
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_v5_stamps), n * sizeof(unsigned long long)) != hipSuccess) {
        set_error("v5 stamps: copy failed");
        return 1;
    }
    std::vector<unsigned long long> z((size_t)n, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_v5_stamps), z.data(), n * sizeof(unsigned long long)) != hipSuccess) {
        set_error("v5 stamps: clear failed");
        return 1;
    }
    return 0;
}

}  // namespace poms
