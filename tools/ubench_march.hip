// Memory-only models of candidate operator tilings at 515^3, p = 3, on the
// line-aligned layout (pitch 528, interior column 0 on a 128-B line), with the
// real kernels' machinery: x planes DMA'd by buffer_load ... lds into a D-deep
// ring, hand-counted vmcnt, one barrier per plane, the wave's 2P+1 x rows read
// back from LDS, 16-B stores.  Apply mix: x read (with the tile's halo), y written.
//
//   tile<NW,RPW,D>: 128 lane-columns (112 output columns) x NW*RPW output rows,
//                   the v5 shape (NW = 16, RPW = 1) and taller tiles (RPW = 2)
//   full<R,D>     : R output rows x the full row width; 5 waves per row, each a
//                   128-lane-column window (112 output columns, whole lines); the
//                   x region of a plane is (R + 2P) whole storage rows, ONE
//                   contiguous block, DMA'd as 1-KiB pieces
// Work decomposition: a chunk grid (tile x axis-0 chunk per workgroup), or a
// persistent grid of G workgroups each taking an equal share of the tile-planes
// (tile-major, planes fastest; a share spans at most a few tiles).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_march.hip -o tools/ubench_march.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int N = 515, P = 3, NP = N + 2 * P, PITCH = 528, SHIFT = 13;
constexpr int64_t S0 = (int64_t)NP * PITCH;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, double* dst, int voff, unsigned soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)dst, 16, voff, (int)soff, 0, AUX);
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
template <int AUX>
__device__ __forceinline__ void st16(__amdgpu_buffer_rsrc_t r, int voff, double a, double b) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 pa = __builtin_bit_cast(u32x2, a), pb = __builtin_bit_cast(u32x2, b);
    u32x4 v;
    v.x = pa.x; v.y = pa.y; v.z = pb.x; v.w = pb.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, 0, AUX);
}

struct Sched {
    int ntiles;   // tiles per plane
    int chunk;    // chunk grid: planes per chunk (0: persistent)
    int64_t total;   // persistent: tile-planes
    int nwg;      // grid size
};

// next work item of this workgroup: tile and output planes [z0, z1); false when done
__device__ __forceinline__ bool next_work(const Sched& s, int bid, int& it, int& tile, int& z0, int& z1) {
    if (s.chunk > 0) {
        if (it++) return false;
        tile = bid % s.ntiles;
        const int ch = bid / s.ntiles;
        z0 = ch * s.chunk;
        z1 = min(z0 + s.chunk, N);
        return z0 < z1;
    }
    const int64_t lo = s.total * bid / s.nwg, hi = s.total * (bid + 1) / s.nwg;
    // it = tile-planes of this share already done
    const int64_t w = lo + it;
    if (w >= hi) return false;
    tile = (int)(w / N);
    z0 = (int)(w % N);
    z1 = (int)min<int64_t>(N, z0 + (hi - w));
    it += z1 - z0;
    return true;
}

// logical workgroup index: consecutive indices on one XCD (round-robin dispatch)
__device__ __forceinline__ int xcd_bid(int nblk) {
    const int b = blockIdx.x, q = nblk >> 3, rr = nblk & 7, xcd = b & 7, k = b >> 3;
    return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + k;
}

// ---- 128-lane-column tiles (v5 shape): T1 = NW * RPW output rows ------------------
template <int NW, int RPW, int D, int YAUX>
__global__ void __launch_bounds__(64 * NW, 1)
tile_k(const double* __restrict__ x, double* __restrict__ y, Sched s, int tiles2) {
    constexpr int T1 = NW * RPW, XR = T1 + 2 * P, TC = 128, PFX = D - 1;
    constexpr int NXM = (XR + NW - 1) / NW;
    __shared__ __attribute__((aligned(16))) double lds[D * XR * TC];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_bid(gridDim.x);
    const uint32_t arr = (uint32_t)(NP * S0 * 8);
    const auto rx = rsrc(x, arr), ry = rsrc(y, arr);
    const uint32_t plane8 = (uint32_t)(S0 * 8);
    const bool xtra = wv < XR - (NXM - 1) * NW;
    int it = 0, tile, z0, z1;
    double sink = 0.0;
    while (next_work(s, bid, it, tile, z0, z1)) {
        const int t2 = tile % tiles2, t1 = tile / tiles2;
        const int c0 = t2 * 112, r0 = t1 * T1;
        // storage column of lane-column 0 = c0 - 8 + P (+SHIFT in elements of the buffer)
        const int colb = (SHIFT + c0 - 8 + P) * 8 + 16 * lane;
        const uint32_t colbx = (uint32_t)colb + ((2 * lane + 1 >= 8 - P && 2 * lane < 120 + P) ? 0u : 0x80000000u);
        const int nplanes = (z1 - z0) + 2 * P;
        auto dma_x = [&](int t, int slot) {
            const int sp = z0 + t;   // storage plane
            const bool ok = t < nplanes;
            const uint32_t so = ok ? (uint32_t)sp * plane8 : 0u;
#pragma unroll
            for (int i = 0; i < NXM; ++i)
                if (i < NXM - 1 || xtra) {
                    const int q = wv + i * NW;
                    dma16<0>(rx, lds + (slot * XR + q) * TC, ok ? (int)((uint32_t)((r0 + q) * PITCH * 8) + colbx) : 0x7ffffff0, so);
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
#pragma unroll
            for (int rr = 0; rr < RPW; ++rr) {
                const int q = wv * RPW + rr;
                d2 a = *(const d2*)(xs + q * TC);
#pragma unroll
                for (int k = 1; k <= 2 * P; ++k) a += *(const d2*)(xs + (q + k) * TC);
                const int orow = r0 + q;
                const bool ok = t >= 2 * P && orow < N && 2 * lane >= 8 && 2 * lane < 120 && c0 + 2 * lane - 8 < N;
                const int voy = (orow + P) * PITCH * 8 + colb + (z0 + t - P) * (int)plane8;
                st16<YAUX>(ry, ok ? voy : 0x7ffffff0, a[0], a[1]);
            }
        }
        wait_vm<0>();
    }
    if (sink == 1.2345) y[0] = sink;
}

// ---- full-width tiles: R rows x 5 windows of 128 lane-columns ----------------------
template <int R, int D, int YAUX>
__global__ void __launch_bounds__(64 * 5 * R, 1)
full_k(const double* __restrict__ x, double* __restrict__ y, Sched s) {
    constexpr int NW = 5 * R, XR = R + 2 * P, ROWB = PITCH * 8;
    constexpr int PIECES = (XR * ROWB + 1023) / 1024;       // 1-KiB DMA pieces per plane
    constexpr int SLOT = PIECES * 128;                       // doubles per ring slot
    constexpr int NPM = (PIECES + NW - 1) / NW;              // most pieces one wave issues
    __shared__ __attribute__((aligned(16))) double lds[D * SLOT + 128];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bid = xcd_bid(gridDim.x);
    const uint32_t arr = (uint32_t)(NP * S0 * 8);
    const auto rx = rsrc(x, arr), ry = rsrc(y, arr);
    const uint32_t plane8 = (uint32_t)(S0 * 8);
    const bool xtra = wv < PIECES - (NPM - 1) * NW;
    const int wrow = wv / 5, seg = wv % 5;
    int it = 0, tile, z0, z1;
    while (next_work(s, bid, it, tile, z0, z1)) {
        const int r0 = tile * R;
        // region: storage rows r0 .. r0 + XR - 1 from interior column -8 (a 64-B boundary)
        const int regb = (r0 * PITCH + SHIFT + P - 8) * 8;
        const int nplanes = (z1 - z0) + 2 * P;
        auto dma_x = [&](int t, int slot) {
            const bool ok = t < nplanes;
            const uint32_t so = ok ? (uint32_t)(z0 + t) * plane8 : 0u;
#pragma unroll
            for (int i = 0; i < NPM; ++i)
                if (i < NPM - 1 || xtra) {
                    const int pc = wv + i * NW;
                    dma16<0>(rx, lds + slot * SLOT + pc * 128, ok ? regb + pc * 1024 + 16 * lane : 0x7ffffff0, so);
                }
        };
        __syncthreads();
#pragma unroll
        for (int i = 0; i < D - 1; ++i) dma_x(i, i);
        for (int t = 0; t < nplanes; ++t) {
            if (t < D - 1) wait_vm<0>();
            else if (xtra) wait_vm<(D - 2) * NPM>();
            else wait_vm<(D - 2) * (NPM - 1)>();
            barrier();
            dma_x(t + D - 1, (t + D - 1) % D);
            // window of lane-columns: interior columns 112 seg - 8 + 2 lane, +1 = LDS column
            const double* xs = lds + (t % D) * SLOT + 112 * seg + 2 * lane;
            d2 a = *(const d2*)(xs + wrow * PITCH);
#pragma unroll
            for (int k = 1; k <= 2 * P; ++k) a += *(const d2*)(xs + (wrow + k) * PITCH);
            const int orow = r0 + wrow;
            const int col = 112 * seg + 2 * lane - 8;
            const bool ok = t >= 2 * P && orow < N && 2 * lane >= 8 && 2 * lane < 120 && col < N;
            const int voy = ((orow + P) * PITCH + SHIFT + P + col) * 8 + (z0 + t - P) * (int)plane8;
            st16<YAUX>(ry, ok ? voy : 0x7ffffff0, a[0], a[1]);
        }
        wait_vm<0>();
    }
}

// ---- reference: streaming copy, each wave moving contiguous 1-KiB pieces (nt) -------
__global__ void __launch_bounds__(256) copy_k(const double* __restrict__ x, double* __restrict__ y, int64_t n2) {
    const int64_t per = 4;   // 16-B pieces in flight per lane
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
static float time_it(F f, int reps = 7) {
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

static int g_cus = 256;

template <int NW, int RPW, int D, int YAUX>
static void run_tile(double* x, double* y, int persist_per_cu, int nchunks, const char* tag) {
    constexpr int T1 = NW * RPW;
    const int tiles2 = (N + 111) / 112, tiles1 = (N + T1 - 1) / T1, ntiles = tiles2 * tiles1;
    Sched s{};
    s.ntiles = ntiles;
    if (persist_per_cu) {
        s.chunk = 0;
        s.total = (int64_t)ntiles * N;
        s.nwg = g_cus * persist_per_cu;
    } else {
        s.chunk = (N + nchunks - 1) / nchunks;
        s.nwg = ntiles * nchunks;
    }
    const float ms = time_it([&] { hipLaunchKernelGGL((tile_k<NW, RPW, D, YAUX>), dim3(s.nwg), dim3(64 * NW), 0, 0, x, y, s, tiles2); });
    const double bytes = 16.0 * N * N * (double)N;
    printf("tile NW %2d RPW %d D %d Y%-2d %-12s %5d WGs: %7.1f us  %.2f TB/s (16 B/DOF)\n", NW, RPW, D, YAUX, tag, s.nwg,
           ms * 1e3, bytes / (ms * 1e-3) / 1e12);
}

template <int R, int D, int YAUX>
static void run_full(double* x, double* y, int persist_per_cu, int nchunks, const char* tag) {
    const int ntiles = (N + R - 1) / R;
    Sched s{};
    s.ntiles = ntiles;
    if (persist_per_cu) {
        s.chunk = 0;
        s.total = (int64_t)ntiles * N;
        s.nwg = g_cus * persist_per_cu;
    } else {
        s.chunk = (N + nchunks - 1) / nchunks;
        s.nwg = ntiles * nchunks;
    }
    const float ms = time_it([&] { hipLaunchKernelGGL((full_k<R, D, YAUX>), dim3(s.nwg), dim3(64 * 5 * R), 0, 0, x, y, s); });
    const double bytes = 16.0 * N * N * (double)N;
    printf("full R %d D %d Y%-2d %-12s %5d WGs: %7.1f us  %.2f TB/s (16 B/DOF)\n", R, D, YAUX, tag, s.nwg, ms * 1e3,
           bytes / (ms * 1e-3) / 1e12);
}

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    g_cus = prop.multiProcessorCount;
    printf("device %s, %d CUs\n", prop.name, g_cus);
    const int64_t alloc = NP * S0 + 64;
    double *x, *y;
    CK(hipMalloc(&x, alloc * 8));
    CK(hipMalloc(&y, alloc * 8));
    CK(hipMemset(x, 0, alloc * 8));
    CK(hipMemset(y, 0, alloc * 8));
    {
        const int64_t n2 = (int64_t)N * N * N / 2048 * 2048;
        const float ms = time_it([&] { hipLaunchKernelGGL(copy_k, dim3(4096), dim3(256), 0, 0, x + 16, y + 16, n2); });
        printf("copy nt (same DOF count)          : %7.1f us  %.2f TB/s\n", ms * 1e3, 16.0 * n2 / (ms * 1e-3) / 1e12);
    }
    for (int rep = 0; rep < 2; ++rep) {
        run_tile<16, 1, 4, 2>(x, y, 0, 3, "chunks3");
        run_tile<16, 1, 4, 16>(x, y, 0, 3, "chunks3");
        run_tile<16, 1, 4, 2>(x, y, 1, 0, "persist1");
        run_tile<16, 1, 4, 16>(x, y, 1, 0, "persist1");
        run_tile<16, 2, 3, 2>(x, y, 0, 6, "chunks6");
        run_tile<16, 2, 3, 2>(x, y, 1, 0, "persist1");
        run_tile<16, 2, 3, 16>(x, y, 1, 0, "persist1");
        run_tile<8, 1, 4, 2>(x, y, 2, 0, "persist2");
        run_full<3, 4, 2>(x, y, 0, 3, "chunks3");
        run_full<3, 4, 2>(x, y, 1, 0, "persist1");
        run_full<3, 4, 16>(x, y, 1, 0, "persist1");
        run_full<3, 3, 2>(x, y, 1, 0, "persist1");
        run_full<2, 4, 2>(x, y, 1, 0, "persist1");
        run_full<2, 4, 16>(x, y, 1, 0, "persist1");
        run_full<1, 4, 2>(x, y, 1, 0, "persist1");
        run_full<1, 2, 2>(x, y, 2, 0, "persist2");
    }
    return 0;
}
