// Build (CPU side, in-tree): hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/r06/ublib.hip -o tools/r06/ublib.so
// (loaded by tools/r06/ublib_bench.py and ublib_offsets.py).
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
//   (generated from ubench_march2.hip: the t16 kernel as a shared library, tools/r06/ublib_bench.py)
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

constexpr int N = 515, P = 3, NP = N + 2 * P, PITCH = 528, SHIFT = 0;
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


// x, y: element (0,0,0) of the padded 521 x 521 x 528 arrays (interior column 0 on a 128-B line)
extern "C" int ub_t16(const double* x, double* y, int trim, int fma, hipStream_t st) {
    const int tiles2 = 5, ntiles = tiles2 * ((N + 15) / 16), nch = 3, chunk = (N + nch - 1) / nch, nwg = ntiles * nch;
    if (trim) hipLaunchKernelGGL((t16_k<4, true>), dim3(nwg), dim3(1024), 0, st, x, y, chunk, tiles2, fma, 0);
    else hipLaunchKernelGGL((t16_k<4, false>), dim3(nwg), dim3(1024), 0, st, x, y, chunk, tiles2, fma, 0);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
