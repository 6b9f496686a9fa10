// HBM write / copy micro-benchmark for the Kronecker kernels' access pattern
// (gfx950).  Geometry of the 515^3 p=3 padded grid (521^3 doubles):
//   w1  contiguous stream writes, 16 B per lane
//   c1  contiguous copy (read + write), 16 B per lane
//   w2  the fused kernel's tile pattern: per workgroup 16 rows x 58 columns of a
//       plane, 74 planes per chunk, 8 B per lane (one column per lane)
//   w3  same tile pattern, rows of 64 columns (full 512 B), 8 B per lane
//   w4  tile pattern with 122-column rows (2 columns per lane, 16 B stores)
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_mem.hip -o tools/ubench_mem.bin && tools/ubench_mem.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void __launch_bounds__(256) stream_write(double2* y, long n2) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) y[i] = make_double2(1.0, 2.0);
}
__global__ void __launch_bounds__(256) stream_copy(const double2* x, double2* y, long n2) {
    const long stride = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) y[i] = x[i];
}

// one workgroup of 8 waves = 16 rows (2 rows per wave) x COLS columns, chunk of planes
// contiguous copy with 4 independent 16-B loads in flight per thread before the stores
template <int AUX>
__global__ void __launch_bounds__(256) stream_copy4(const double2* x, double2* y, long n2) {
    const long stride = (long)gridDim.x * blockDim.x;
    long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n2; i += 4 * stride) {
        double2 a = x[i], b = x[i + stride], c = x[i + 2 * stride], d = x[i + 3 * stride];
        if (AUX) {
            typedef double dv2 __attribute__((ext_vector_type(2)));
            dv2* yy = (dv2*)y;
            __builtin_nontemporal_store(dv2{a.x, a.y}, yy + i); __builtin_nontemporal_store(dv2{b.x, b.y}, yy + i + stride);
            __builtin_nontemporal_store(dv2{c.x, c.y}, yy + i + 2 * stride); __builtin_nontemporal_store(dv2{d.x, d.y}, yy + i + 3 * stride);
        } else {
            y[i] = a; y[i + stride] = b; y[i + 2 * stride] = c; y[i + 3 * stride] = d;
        }
    }
    for (; i < n2; i += stride) y[i] = x[i];
}

template <int COLS, int CPL>
__global__ void __launch_bounds__(512) tile_write(double* y, int n, int s1, long s0, int tiles2, int tiles1, int chunk, int coff = 3) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int bid = blockIdx.x;
    const int t2 = bid % tiles2; bid /= tiles2;
    const int t1 = bid % tiles1;
    const int ch = bid / tiles1;
    const int z0 = ch * chunk, z1 = min(z0 + chunk, n);
    for (int z = z0; z < z1; ++z) {
        for (int r = 0; r < 2; ++r) {
            const int row = t1 * 16 + wv * 2 + r;
            if (CPL == 1) {
                const int col = t2 * COLS + lane;
                if (row < n && col < n && lane < COLS) y[(long)(z + 3) * s0 + (long)(row + 3) * s1 + col + coff] = 1.0;
            } else {
                const int col = t2 * COLS + 2 * lane;
                if (row < n && col + 1 < n && 2 * lane < COLS) {
                    double* p = y + (long)(z + 3) * s0 + (long)(row + 3) * s1 + col + 3;
                    p[0] = 1.0;
                    p[1] = 2.0;
                }
            }
        }
    }
}

// Jacobi-like traffic: per plane and workgroup read x (16 + 6 rows x 64 columns),
// read b and write y (16 rows x OUTC columns).  `shift` moves the whole grid inside
// the row (pitch > 521) so that output segments can start on a 128-B line.
template <int OUTC>
__global__ void __launch_bounds__(512) tile_jac(const double* x, const double* b, double* y, int n, int s1, long s0,
                                                int tiles2, int tiles1, int chunk, int shift) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    int bid = blockIdx.x;
    const int t2 = bid % tiles2; bid /= tiles2;
    const int t1 = bid % tiles1;
    const int ch = bid / tiles1;
    const int z0 = ch * chunk, z1 = min(z0 + chunk, n);
    const int c0 = t2 * OUTC;
    const int halo = (64 - OUTC) / 2;
    const int xc = min(max(c0 - halo + lane, -3), n + 2) + 3 + shift;   // padded column of this lane's x
    const int oc = c0 + lane;                                         // interior output column
    for (int z = z0; z < z1; ++z) {
        double acc = 0.0;
        const long pl = (long)(z + 3) * s0;
        for (int r = wv; r < 22; r += 8) {
            const int row = min(t1 * 16 + r - 3, n + 2) + 3;
            acc += x[pl + (long)row * s1 + xc];
        }
        for (int r = 0; r < 2; ++r) {
            const int row = t1 * 16 + wv * 2 + r;
            if (row < n && oc < n && lane < OUTC) {
                const long o = pl + (long)(row + 3) * s1 + oc + 3 + shift;
                y[o] = b[o] + 0.1 * acc;
            }
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
    const int n = 515, S = 521;
    const long s0 = (long)S * S, tot = s0 * S;
    const long alloc = 528L * 528L * 528L;   // covers the 528-pitch layouts below
    // host-side bound check of the largest index any tile_write launch below can touch
    auto max_index = [&](long pitch, long plane, int coff) { return (long)(n - 1 + 3) * plane + (long)(n - 1 + 3) * pitch + (n - 1) + coff + 1; };
    if (max_index(528, 528L * S, 3) >= alloc || max_index(S, s0, 3) >= alloc) { printf("bad bounds\n"); return 1; }
    double *x, *y, *bb;
    CK(hipMalloc(&bb, alloc * 8));
    CK(hipMemset(bb, 0, alloc * 8));
    CK(hipMalloc(&x, alloc * 8));
    CK(hipMalloc(&y, alloc * 8));
    CK(hipMemset(x, 0, alloc * 8));
    CK(hipMemset(y, 0, alloc * 8));
    const double dof = (double)n * n * n;
    const long n2 = tot / 2;
    float ms = time_it([&] { hipLaunchKernelGGL(stream_write, dim3(8192), dim3(256), 0, 0, (double2*)y, n2); });
    printf("w1 stream write 16B/lane: %.1f us  %.2f TB/s\n", ms * 1e3, tot * 8 / (ms * 1e-3) / 1e12);
    ms = time_it([&] { hipLaunchKernelGGL(stream_copy, dim3(8192), dim3(256), 0, 0, (const double2*)x, (double2*)y, n2); });
    printf("c1 stream copy 16B/lane: %.1f us  %.2f TB/s (read+write)\n", ms * 1e3, 2.0 * tot * 8 / (ms * 1e-3) / 1e12);
    {
        const int cols = 58, tiles2 = (n + cols - 1) / cols, tiles1 = (n + 15) / 16, chunk = 74, nch = (n + chunk - 1) / chunk;
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<58, 1>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S, s0, tiles2, tiles1, chunk); });
        printf("w2 tile 16x58, 8B/lane: %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
    }
    {
        const int cols = 64, tiles2 = (n + cols - 1) / cols, tiles1 = (n + 15) / 16, chunk = 74, nch = (n + chunk - 1) / chunk;
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<64, 1>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S, s0, tiles2, tiles1, chunk); });
        printf("w3 tile 16x64, 8B/lane: %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
    }
    {
        const int cols = 122, tiles2 = (n + cols - 1) / cols, tiles1 = (n + 15) / 16, chunk = 74, nch = (n + chunk - 1) / chunk;
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<122, 2>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S, s0, tiles2, tiles1, chunk); });
        printf("w4 tile 16x122, 2 cols/lane: %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
    }
    {
        const int cols = 58, tiles2 = (n + cols - 1) / cols, tiles1 = (n + 15) / 16, chunk = 515, nch = 1;
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<58, 1>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S, s0, tiles2, tiles1, chunk); });
        printf("w5 tile 16x58, full-depth chunks (297 WGs): %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
    }
    ms = time_it([&] { hipLaunchKernelGGL(stream_copy4<0>, dim3(4096), dim3(256), 0, 0, (const double2*)x, (double2*)y, n2); });
    printf("c2 stream copy, 4 loads in flight: %.1f us  %.2f TB/s (read+write)\n", ms * 1e3, 2.0 * tot * 8 / (ms * 1e-3) / 1e12);
    ms = time_it([&] { hipLaunchKernelGGL(stream_copy4<1>, dim3(4096), dim3(256), 0, 0, (const double2*)x, (double2*)y, n2); });
    printf("c3 stream copy, 4 in flight, nt stores: %.1f us  %.2f TB/s (read+write)\n", ms * 1e3, 2.0 * tot * 8 / (ms * 1e-3) / 1e12);
    {   // rows padded to a 128-B multiple (528 doubles), 64-column tiles starting on a line
        const int S2 = 528;
        const long s02 = (long)S2 * S;
        const int cols = 64, tiles2 = (n + cols - 1) / cols, tiles1 = (n + 15) / 16, chunk = 74, nch = (n + chunk - 1) / chunk;
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<64, 1>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S2, s02, tiles2, tiles1, chunk, 0); });
        printf("w6 tile 16x64, 128-B aligned rows: %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
        ms = time_it([&] { hipLaunchKernelGGL((tile_write<64, 1>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, y, n, S2, s02, tiles2, tiles1, chunk, 3); });
        printf("w7 tile 16x64, aligned pitch, 24-B offset: %.1f us  %.2f TB/s of y\n", ms * 1e3, dof * 8 / (ms * 1e-3) / 1e12);
    }
    {   // Jacobi-like mixes (24 algorithmic B/DOF); shift 13 puts padded column 3 on a 128-B line
        const int tiles1 = (n + 15) / 16, chunk = 103, nch = (n + chunk - 1) / chunk;
        const long need = (long)(n + 6) * 528L * S + 16;
        if (need > alloc || (long)(n + 6) * s0 + 16 > alloc) { printf("bad bounds\n"); return 1; }
        struct Cfg { const char* name; int outc; int pitch; int shift; };
        const Cfg cfgs[] = {{"j1 58 cols, pitch 521 (current)", 58, S, 0},
                            {"j2 58 cols, pitch 528, unaligned", 58, 528, 0},
                            {"j3 48 cols, pitch 528, 128-B aligned", 48, 528, 13},
                            {"j4 48 cols, pitch 528, unaligned", 48, 528, 0},
                            {"j5 56 cols, pitch 528, start aligned", 56, 528, 13}};
        for (const Cfg& c : cfgs) {
            const long pl = (long)c.pitch * S;
            const int tiles2 = (n + c.outc - 1) / c.outc;
            if (c.outc == 58)
                ms = time_it([&] { hipLaunchKernelGGL((tile_jac<58>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, bb, y, n, c.pitch, pl, tiles2, tiles1, chunk, c.shift); });
            else if (c.outc == 56)
                ms = time_it([&] { hipLaunchKernelGGL((tile_jac<56>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, bb, y, n, c.pitch, pl, tiles2, tiles1, chunk, c.shift); });
            else
                ms = time_it([&] { hipLaunchKernelGGL((tile_jac<48>), dim3(tiles2 * tiles1 * nch), dim3(512), 0, 0, x, bb, y, n, c.pitch, pl, tiles2, tiles1, chunk, c.shift); });
            printf("%s: %.1f us  %.2f TB/s (24 B/DOF)\n", c.name, ms * 1e3, dof * 24 / (ms * 1e-3) / 1e12);
        }
    }
    return 0;
}
