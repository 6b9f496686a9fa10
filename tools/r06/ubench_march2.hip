// Build: hipcc --offload-arch=gfx950 -O3 tools/r06/ubench_march2.hip -o tools/r06/ubench_march2.bin;
// run: tools/r06/ubench_march2.bin [case] [fill]  (case: one measurement, else all; fill 1: non-zero x).
// Round 6: memory-only models of the p = 3 apply's march at 515^3 (line-aligned
// layout: pitch 528, interior column 0 on a 128-B line), as tools/ubench_march.hip,
// with two additions:
//   * trims: x lanes past interior column n2 - 1 + P and x rows past storage row
//     n1 - 1 + 2P are not fetched (the last tile column / tile row);
//   * the 32-row tile of a candidate kernel: 8 waves x 4 rows, each wave two rows
//     at a time (lanes 0-31 one row, lanes 32-63 the next-but-one), 4 columns per
//     lane; each x row DMA'd by one instruction whose lanes 0-31 fetch the column
//     pairs (4i, 4i+1) and lanes 32-63 the pairs (4i+2, 4i+3), so that a lane's two
//     16-B LDS reads are contiguous across the lanes (conflict-free ds_read_b128);
//     y stored as two 16-B stores per lane and row (32-B lane stride).
// 3 axis-0 chunks: 255 workgroups of 32-row tiles (one round of the 256 CUs), 495 of
// 16-row tiles (1.93 rounds).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/r06/ubench_march2.hip -o tools/r06/ubench_march2.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int N = 515, P = 3, NP = N + 2 * P, PITCH = 528, SHIFT = 13;
constexpr int64_t S0 = (int64_t)NP * PITCH;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, double* dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)dst, 16, voff, (int)soff, 0, 0);
}
template <int N_>
__device__ __forceinline__ void wait_vm() {
    __builtin_amdgcn_s_waitcnt((N_ & 15) | (7 << 4) | (15 << 8) | ((N_ >> 4) << 14));
}
__device__ __forceinline__ void barrier() {
    __asm__ volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __asm__ volatile("" ::: "memory");
}
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int voff, double a, double b) {
    const u32x2 pa = __builtin_bit_cast(u32x2, a), pb = __builtin_bit_cast(u32x2, b);
    u32x4 v;
    v.x = pa.x; v.y = pa.y; v.z = pb.x; v.w = pb.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, 2);   // nt
}
__device__ __forceinline__ int xcd_bid(int nblk) {
    const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
}

// ---- v5 shape: 16 waves x 1 row, 2 columns per lane (TRIM: n2 / row trims) ----------
template <int D, bool TRIM>
__global__ void __launch_bounds__(1024, 1)
t16_k(const double* __restrict__ x, double* __restrict__ y, int chunk, int tiles2, int fma, int extra) {
    constexpr int NW = 16, T1 = 16, XR = T1 + 2 * P, TC = 128, PFX = D - 1, NXM = 2;
    __shared__ __attribute__((aligned(16))) double lds[D * XR * TC];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_bid(gridDim.x);
    const auto rx = rsrc(x, (uint32_t)(NP * S0 * 8)), ry = rsrc(y, (uint32_t)(NP * S0 * 8));
    const uint32_t plane8 = (uint32_t)(S0 * 8);
    const bool xtra = wv < XR - NW;
    const int ntiles = tiles2 * ((N + T1 - 1) / T1);
    const int tile = bid % ntiles, ch = bid / ntiles;
    const int z0 = ch * chunk, z1 = min(z0 + chunk, N);
    const int t2 = tile % tiles2, t1 = tile / tiles2;
    const int c0 = t2 * 112, r0 = t1 * T1;
    const int colb = (SHIFT + c0 - 8 + P) * 8 + 16 * lane;
    const int cg0 = c0 - 8 + 2 * lane;
    const uint32_t colbx = (uint32_t)colb + ((2 * lane + 1 >= 8 - P && 2 * lane < 120 + P && (!TRIM || cg0 < N + P)) ? 0u : 0x80000000u);
    const int xrows_ok = TRIM ? N + 2 * P - r0 : 1 << 20;
    const int nplanes = (z1 - z0) + 2 * P;
    auto dma_x = [&](int t, int slot) {
        const bool ok = t < nplanes;
        const uint32_t so = ok ? (uint32_t)(z0 + t) * plane8 : 0u;
#pragma unroll
        for (int i = 0; i < NXM; ++i)
            if (i < NXM - 1 || xtra) {
                const int q = wv + i * NW;
                dma16(rx, lds + (slot * XR + q) * TC, (ok && q < xrows_ok) ? (int)((uint32_t)((r0 + q) * PITCH * 8) + colbx) : 0x7ffffff0, so);
            }
    };
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PFX; ++i) dma_x(i, i);
    for (int t = 0; t < nplanes; ++t) {
        if (t < PFX) wait_vm<0>();
        else if (xtra) wait_vm<(PFX - 1) * NXM>();
        else wait_vm<(PFX - 1) * (NXM - 1)>();
        barrier();
        dma_x(t + PFX, (t + PFX) % D);
        const double* xs = lds + (t % D) * XR * TC + 2 * lane;
        d2 a = *(const d2*)(xs + wv * TC);
#pragma unroll
        for (int k = 1; k <= 2 * P; ++k) a += *(const d2*)(xs + (wv + k) * TC);
        // fake arithmetic: fma dependent multiply-adds per lane (4 independent chains),
        // `extra` % more on the boundary tile columns (the real kernel's general paths)
        {
            const int nf = (t2 == 0 || t2 == tiles2 - 1) ? fma + fma * extra / 100 : fma;
            d2 c0 = a, c1 = a * 0.5;
            for (int f = 0; f < nf; f += 4) {
                c0 = c0 * 0.999 + 1e-3;
                c1 = c1 * 0.999 + 1e-3;
            }
            a = c0 + c1;
        }
        const int orow = r0 + wv;
        const bool ok = t >= 2 * P && orow < N && 2 * lane >= 8 && 2 * lane < 120 && cg0 < N;
        const int voy = (orow + P) * PITCH * 8 + colb + (z0 + t - P) * (int)plane8;
        st16(ry, ok ? voy : 0x7ffffff0, a[0], a[1]);
    }
    wait_vm<0>();
}

// ---- 32-row tile: 8 waves x 4 rows, 4 columns per lane -----------------------------
// SP: store pattern 0 = each lane's own 4 columns (two 16-B stores, 32-B lane stride),
// 1 = contiguous 16-B lane stride (wrong placement; the store pattern's cost only)
template <int D, int SP>
__global__ void __launch_bounds__(512, 1)
t32_k(const double* __restrict__ x, double* __restrict__ y, int chunk, int tiles2) {
    constexpr int NW = 8, T1 = 32, XR = T1 + 2 * P, TC = 128, PFX = D - 1;
    constexpr int NXM = (XR + NW - 1) / NW;   // 5
    __shared__ __attribute__((aligned(16))) double lds[D * XR * TC];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_bid(gridDim.x);
    const auto rx = rsrc(x, (uint32_t)(NP * S0 * 8)), ry = rsrc(y, (uint32_t)(NP * S0 * 8));
    const uint32_t plane8 = (uint32_t)(S0 * 8);
    const bool xtra = wv < XR - (NXM - 1) * NW;
    const int ntiles = tiles2 * ((N + T1 - 1) / T1);
    const int tile = bid % ntiles, ch = bid / ntiles;
    const int z0 = ch * chunk, z1 = min(z0 + chunk, N);
    const int t2 = tile % tiles2, t1 = tile / tiles2;
    const int c0 = t2 * 112, r0 = t1 * T1;
    // DMA lane -> lane-column pair: lanes 0-31 (4i, 4i+1), lanes 32-63 (4i+2, 4i+3)
    const int dlc = 4 * (lane & 31) + 2 * (lane >> 5);
    const int dcg = c0 - 8 + dlc;
    const uint32_t colbx = (uint32_t)((SHIFT + P + dcg) * 8) + ((dlc + 1 >= 8 - P && dlc < 120 + P && dcg < N + P) ? 0u : 0x80000000u);
    const int xrows_ok = N + 2 * P - r0;
    // compute lane: half h = lane >> 5 takes rows 4 wv + 2 h + {0, 1}; columns 4 (lane & 31) + 0..3
    const int h = lane >> 5, ll = lane & 31;
    const int lc = 4 * ll, cg = c0 - 8 + lc;
    const int nplanes = (z1 - z0) + 2 * P;
    auto dma_x = [&](int t, int slot) {
        const bool ok = t < nplanes;
        const uint32_t so = ok ? (uint32_t)(z0 + t) * plane8 : 0u;
#pragma unroll
        for (int i = 0; i < NXM; ++i)
            if (i < NXM - 1 || xtra) {
                const int q = wv + i * NW;
                dma16(rx, lds + (slot * XR + q) * TC, (ok && q < xrows_ok) ? (int)((uint32_t)((r0 + q) * PITCH * 8) + colbx) : 0x7ffffff0, so);
            }
    };
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PFX; ++i) dma_x(i, i);
    for (int t = 0; t < nplanes; ++t) {
        if (t < PFX) wait_vm<0>();
        else if (xtra) wait_vm<(PFX - 1) * NXM>();
        else wait_vm<(PFX - 1) * (NXM - 1)>();
        barrier();
        dma_x(t + PFX, (t + PFX) % D);
        // this lane's rows q0 = 4 wv + 2 h and q0 + 1; x rows q0 .. q0 + 2P + 1
        const int q0 = 4 * wv + 2 * h;
        const double* xs = lds + (t % D) * XR * TC + 2 * ll;
        d2 a0 = {0, 0}, a1 = {0, 0}, b0 = {0, 0}, b1 = {0, 0};
#pragma unroll
        for (int k = 0; k <= 2 * P + 1; ++k) {
            const d2 lo = *(const d2*)(xs + (q0 + k) * TC);        // columns lc, lc + 1
            const d2 hi = *(const d2*)(xs + (q0 + k) * TC + 64);   // columns lc + 2, lc + 3
            if (k <= 2 * P) { a0 += lo; a1 += hi; }
            if (k >= 1) { b0 += lo; b1 += hi; }
        }
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int orow = r0 + q0 + rr;
            const d2 v0 = rr ? b0 : a0, v1 = rr ? b1 : a1;
            const bool ok = t >= 2 * P && orow < N && lc >= 8 && lc < 120 && cg < N;
            const int rowb = (orow + P) * PITCH * 8 + (z0 + t - P) * (int)plane8;
            if (SP == 0) {
                const int voy = rowb + (SHIFT + P + cg) * 8;
                st16(ry, ok ? voy : 0x7ffffff0, v0[0], v0[1]);
                st16(ry, ok ? voy + 16 : 0x7ffffff0, v1[0], v1[1]);
            } else {
                const int voy = rowb + (SHIFT + P + c0 - 8) * 8 + 16 * ll;
                st16(ry, ok ? voy : 0x7ffffff0, v0[0], v0[1]);
                st16(ry, ok ? voy + 512 : 0x7ffffff0, v1[0], v1[1]);
            }
        }
    }
    wait_vm<0>();
}

__global__ void __launch_bounds__(256) copy_k(const double* __restrict__ x, double* __restrict__ y, int64_t n2) {
    const int64_t per = 4;
    const int64_t stride = (int64_t)gridDim.x * 256 * 2 * per;
    for (int64_t b = ((int64_t)blockIdx.x * 256) * 2 * per + 2 * (threadIdx.x & 63) + (threadIdx.x >> 6) * 128 * per; b < n2; b += stride) {
        d2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load((const d2*)(x + b + u * 128));
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], (d2*)(y + b + u * 128));
    }
}

template <typename F>
static float time_it(F f, int reps = 9) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    f();
    CK(hipDeviceSynchronize());
    std::vector<float> v;
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        f();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        v.push_back(ms);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static void report(const char* tag, int nwg, float ms) {
    const double bytes = 16.0 * N * N * (double)N;
    printf("%-28s %5d WGs: %7.1f us  %.2f TB/s (16 B/DOF)\n", tag, nwg, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
}

template <int D, bool TRIM>
static void run16(double* x, double* y, int nch, const char* tag, int fma = 0, int extra = 0) {
    const int tiles2 = 5, ntiles = tiles2 * ((N + 15) / 16), chunk = (N + nch - 1) / nch, nwg = ntiles * nch;
    report(tag, nwg, time_it([&] { hipLaunchKernelGGL((t16_k<D, TRIM>), dim3(nwg), dim3(1024), 0, 0, x, y, chunk, tiles2, fma, extra); }));
}
template <int D, int SP>
static void run32(double* x, double* y, int nch, const char* tag) {
    const int tiles2 = 5, ntiles = tiles2 * ((N + 31) / 32), chunk = (N + nch - 1) / nch, nwg = ntiles * nch;
    report(tag, nwg, time_it([&] { hipLaunchKernelGGL((t32_k<D, SP>), dim3(nwg), dim3(512), 0, 0, x, y, chunk, tiles2); }));
}

int main(int argc, char** argv) {
    const int64_t alloc = NP * S0 + 64;
    double *x, *y;
    CK(hipMalloc(&x, alloc * 8));
    CK(hipMalloc(&y, alloc * 8));
    const int which = argc > 1 ? atoi(argv[1]) : -1;   // one case only (for --pmc passes), or all
    // argv[2] = 1: x filled with non-zero bytes (0x3f3f... = 3.7e-4 in every double), else zeros
    const int fill = argc > 2 ? atoi(argv[2]) : 0;
    CK(hipMemset(x, fill ? 0x3f : 0, alloc * 8));
    CK(hipMemset(y, 0, alloc * 8));
    for (int rep = 0; rep < (which < 0 ? 2 : 1); ++rep) {
        if (which < 0 || which == 0) {
            const int64_t n2 = (int64_t)N * N * N / 2048 * 2048;
            report("copy nt", 4096, time_it([&] { hipLaunchKernelGGL(copy_k, dim3(4096), dim3(256), 0, 0, x + 16, y + 16, n2); }));
        }
        if (which < 0 || which == 1) run16<4, false>(x, y, 3, "t16 D4 chunks3");
        if (which < 0 || which == 2) run16<4, true>(x, y, 3, "t16 D4 chunks3 trim");
        if (which < 0 || which == 3) run16<4, true>(x, y, 3, "t16 trim fma64", 64, 0);
        if (which < 0 || which == 4) run16<4, true>(x, y, 3, "t16 trim fma128", 128, 0);
        if (which < 0 || which == 5) run16<4, true>(x, y, 3, "t16 trim fma128 +10%", 128, 10);
        if (which < 0 || which == 6) run16<4, true>(x, y, 3, "t16 trim fma192", 192, 0);
        if (which < 0 || which == 7) run16<4, true>(x, y, 3, "t16 trim fma192 +10%", 192, 10);
        if (which == 8) run32<4, 1>(x, y, 3, "t32 D4 chunks3 sp1");
    }
    return 0;
}
