// Memory-only access patterns for candidate operator tilings at 515^3, p = 3
// (padded 521^3 grid; pitch 521 or a 16-multiple pitch 528).  Each pattern
// reads x with the tile's halo and writes y once per output point (apply mix):
//   col64  : current shape -- 16 rows x 58 output columns, 64-column loads
//   rowT   : full-row tiles -- T1 whole rows per workgroup and plane, loads of
//            T1 + 2P whole rows (one contiguous region), stores of T1 whole rows
//            (one contiguous region, ghost columns included)
// The axis-0 march is a chunk of planes per workgroup (as in the kernels).
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_rowtile.hip -o tools/ubench_rowtile.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
typedef double d2 __attribute__((ext_vector_type(2)));

// full-row tile: rows [r0, r0+T1) of the padded plane (interior rows r0 >= P), 16 B per lane
template <int T1, int NT>
__global__ void __launch_bounds__(NT) rowtile(const double* __restrict__ x, double* __restrict__ y, int n, int S, long s0,
                                                int tiles1, int chunk, int P) {
    const int t1 = blockIdx.x % tiles1, ch = blockIdx.x / tiles1;
    const int r0 = P + t1 * T1;
    const int r1 = min(r0 + T1, n + P);
    const int z0 = P + ch * chunk, z1 = min(z0 + chunk, n + P);
    const long lo = (long)(r0 - P) * S, hi = (long)(r1 + P) * S;   // x region (elements of a plane)
    const long olo = (long)r0 * S, ohi = (long)r1 * S;
    for (int z = z0; z < z1; ++z) {
        const double* xp = x + (long)z * s0;
        double* yp = y + (long)z * s0;
        d2 acc = {0.0, 0.0};
        for (long e = lo + 2 * threadIdx.x; e + 1 < hi; e += 2 * NT) acc += *(const d2*)(xp + e);
        for (long e = olo + 2 * threadIdx.x; e + 1 < ohi; e += 2 * NT) *(d2*)(yp + e) = acc;
    }
}

// current shape: 64-column loads (22 rows), 58-column stores (16 rows), 8 B per lane
__global__ void __launch_bounds__(512) col64(const double* __restrict__ x, double* __restrict__ y, int n, int S, long s0,
                                             int tiles2, int tiles1, int chunk) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int bid = blockIdx.x;
    const int t2 = bid % tiles2; bid /= tiles2;
    const int t1 = bid % tiles1;
    const int ch = bid / tiles1;
    const int z0 = 3 + ch * chunk, z1 = min(z0 + chunk, n + 3);
    const int c = t2 * 58 + lane;   // padded column of this lane's x (tile cols c0-3 .. c0+60)
    for (int z = z0; z < z1; ++z) {
        const double* xp = x + (long)z * s0;
        double* yp = y + (long)z * s0;
        double acc = 0.0;
        for (int r = wv; r < 22; r += 8) {
            const int row = min(t1 * 16 + r, n + 5);
            if (c < n + 6) acc += xp[(long)row * S + c];
        }
        for (int r = 0; r < 2; ++r) {
            const int row = t1 * 16 + wv * 2 + r;
            if (row < n && lane >= 3 && lane < 61 && c < n + 3) yp[(long)(row + 3) * S + c] = acc;
        }
    }
}


// 2 columns per lane: 22 rows x 128 columns loaded (16 B / lane, line-aligned with
// pitch 528 and the interior shifted to a line start), 16 rows x TO columns stored
// (TO = 112: whole lines only; TO = 122: the unaligned maximum)
template <int TO>
__global__ void __launch_bounds__(512) col128(const double* __restrict__ x, double* __restrict__ y, int n, int S, long s0,
                                              int tiles2, int tiles1, int chunk, int shift) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int bid = blockIdx.x;
    const int t2 = bid % tiles2; bid /= tiles2;
    const int t1 = bid % tiles1;
    const int ch = bid / tiles1;
    const int z0 = 3 + ch * chunk, z1 = min(z0 + chunk, n + 3);
    const int h = (128 - TO) / 2;
    const int c = shift + t2 * TO - h + 3 + 2 * lane;   // padded column (+shift) of this lane's first x element
    const bool cin = c >= 0 && c + 1 < S;
    const bool oin = 2 * lane >= h && 2 * lane < h + TO && (c - shift - 3) + 1 < n;
    for (int z = z0; z < z1; ++z) {
        const double* xp = x + (long)z * s0;
        double* yp = y + (long)z * s0;
        d2 acc = {0.0, 0.0};
#pragma unroll
        for (int r = wv; r < 22 + 8; r += 8) {
            const int row = min(t1 * 16 + r, n + 5);
            if (r < 22 && cin) acc += *(const d2*)(xp + (long)row * S + c);
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int row = t1 * 16 + wv * 2 + r;
            if (row < n && oin) *(d2*)(yp + (long)(row + 3) * S + c) = acc;
        }
    }
}

template <typename F>
static float time_it(F f) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f();
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        f();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        best = ms < best ? ms : best;
    }
    return best;
}

int main() {
    const int n = 515, P = 3, R = n + 2 * P;
    const long alloc = (long)R * R * 528 + 64;
    double *x, *y;
    CK(hipMalloc(&x, alloc * 8));
    CK(hipMalloc(&y, alloc * 8));
    CK(hipMemset(x, 0, alloc * 8));
    CK(hipMemset(y, 0, alloc * 8));
    const double bytes = 16.0 * n * n * (double)n;
    for (int chunk : {64, 103, 172}) {
        const int nch = (n + chunk - 1) / chunk;
        const int tiles2 = 9, tiles1 = (n + 15) / 16;
        float ms = time_it([&] { hipLaunchKernelGGL(col64, dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, y, n, R, (long)R * R, tiles2, tiles1, chunk); });
        printf("col64 chunk %3d (%5d WGs): %7.1f us  %.2f TB/s (16 B/DOF)\n", chunk, tiles2 * tiles1 * nch, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
    for (int S : {522, 528}) {   // even pitches: 16-B aligned rows and planes
        const long s0 = (long)S * R;
        for (int chunk : {32, 64, 103, 172}) {
            const int nch = (n + chunk - 1) / chunk;
#define RT(T1, NT)                                                                                                   \
            {                                                                                                        \
                const int tiles1 = (n + T1 - 1) / T1;                                                                \
                float ms = time_it([&] { hipLaunchKernelGGL((rowtile<T1, NT>), dim3(tiles1 * nch), dim3(NT), 0, 0, x, y, n, S, s0, tiles1, chunk, P); }); \
                printf("row pitch %d T1 %2d NT %d chunk %3d (%5d WGs): %7.1f us  %.2f TB/s\n", S, T1, NT, chunk, tiles1 * nch, ms * 1e3, bytes / (ms * 1e-3) / 1e12); \
            }
            RT(8, 256) RT(8, 512) RT(16, 512) RT(16, 1024) RT(32, 1024)
#undef RT
        }
    }
    for (int chunk : {32, 64, 103}) {
        const int nch = (n + chunk - 1) / chunk, tiles1 = (n + 15) / 16;
        {   // 112 aligned outputs per tile, pitch 528, interior column 0 on a line start (shift 13)
            const int S = 528, tiles2 = (n + 111) / 112;
            float ms = time_it([&] { hipLaunchKernelGGL((col128<112>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, y, n, S, (long)S * R, tiles2, tiles1, chunk, 13); });
            printf("col128 TO 112 aligned chunk %3d (%5d WGs): %7.1f us  %.2f TB/s\n", chunk, tiles2 * tiles1 * nch, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        }
        {   // 122 outputs per tile, pitch 522 (16-B aligned rows only)
            const int S = 522, tiles2 = (n + 121) / 122;
            float ms = time_it([&] { hipLaunchKernelGGL((col128<122>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, y, n, S, (long)S * R, tiles2, tiles1, chunk, 0); });
            printf("col128 TO 122 pitch 522 chunk %3d (%5d WGs): %7.1f us  %.2f TB/s\n", chunk, tiles2 * tiles1 * nch, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
