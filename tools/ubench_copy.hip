// HBM streaming ceilings on gfx950 for the shapes the operator kernels could
// take: copy (1 read : 1 write, the Kron apply's mix), 2 reads : 1 write (the
// Jacobi sweep's mix), read-only and write-only, each as (a) a grid-stride
// loop and (b) block-contiguous segments with several 16-B loads in flight.
// Arrays: 521^3 doubles (the 515^3 p=3 padded vector, 1.13 GB).
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_copy.hip -o tools/ubench_copy.bin && tools/ubench_copy.bin
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) gs_copy(const d2* x, d2* y, long n) {
    const long st = (long)gridDim.x * blockDim.x;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += st) y[i] = x[i];
}

// block-contiguous: block b owns [b*seg, (b+1)*seg) d2 elements; U loads in flight per thread
template <int U, int MIX>   // MIX 0 copy, 1 y = x + b, 2 read-only, 3 write-only
__global__ void __launch_bounds__(256) seg_kernel(const d2* x, const d2* b, d2* y, long n, long seg, double* out) {
    const long s0 = (long)blockIdx.x * seg;
    const long s1 = s0 + seg < n ? s0 + seg : n;
    d2 acc = {0.0, 0.0};
    for (long i = s0 + threadIdx.x; i < s1; i += 256L * U) {
        d2 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long j = i + 256L * u;
            if (MIX != 3) v[u] = j < s1 ? x[j] : d2{0.0, 0.0};
            if (MIX == 1) w[u] = j < s1 ? b[j] : d2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long j = i + 256L * u;
            if (j < s1) {
                if (MIX == 0) y[j] = v[u];
                else if (MIX == 1) y[j] = v[u] + w[u];
                else if (MIX == 2) acc += v[u];
                else y[j] = d2{1.0, (double)j};
            }
        }
    }
    if (MIX == 2 && acc.x == 1234.5) out[0] = acc.y;
}


// each thread moves 16*V contiguous bytes per step (V x 16-B loads in flight, consecutive)
template <int V, bool NT>
__global__ void __launch_bounds__(256) wide_copy(const d2* __restrict__ x, d2* __restrict__ y, long n) {
    const long st = (long)gridDim.x * blockDim.x * V;
    for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * V; i + V <= n; i += st) {
        d2 v[V];
#pragma unroll
        for (int u = 0; u < V; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u) : x[i + u];
#pragma unroll
        for (int u = 0; u < V; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], y + i + u);
            else y[i + u] = v[u];
        }
    }
}
// wave-contiguous: each wave moves U consecutive 1-KiB pieces per step
template <int U, bool NT>
__global__ void __launch_bounds__(256) wave_copy(const d2* __restrict__ x, d2* __restrict__ y, long n) {
    const int lane = threadIdx.x & 63;
    const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const long nw = ((long)gridDim.x * blockDim.x) >> 6;
    for (long base = wave * 64 * U; base + 64 * U <= n; base += nw * 64 * U) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(x + base + u * 64 + lane) : x[base + u * 64 + lane];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], y + base + u * 64 + lane);
            else y[base + u * 64 + lane] = v[u];
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
    const long S = 521, tot = S * S * S, n = tot / 2;   // d2 elements
    double *x, *b, *y, *out;
    CK(hipMalloc(&x, tot * 8));
    CK(hipMalloc(&b, tot * 8));
    CK(hipMalloc(&y, tot * 8));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(x, 0, tot * 8));
    CK(hipMemset(b, 0, tot * 8));
    CK(hipMemset(y, 0, tot * 8));
    const double B = tot * 8.0;
    float ms = time_it([&] { hipLaunchKernelGGL(gs_copy, dim3(8192), dim3(256), 0, 0, (const d2*)x, (d2*)y, n); });
    printf("gs copy 8192x256: %.1f us %.2f TB/s\n", ms * 1e3, 2 * B / (ms * 1e-3) / 1e12);
    const char* mixn[] = {"copy", "x+b", "read", "write"};
    const double mixb[] = {2, 3, 1, 1};
    for (int blocks : {8192}) {
        const long seg = (n + blocks - 1) / blocks;
        for (int mix = 0; mix < 4; ++mix) {
            for (int u : {2, 4, 8}) {
                auto go = [&] {
                    const d2 *xx = (const d2*)x, *bb = (const d2*)b;
                    d2* yy = (d2*)y;
#define L(U, M) if (u == U && mix == M) hipLaunchKernelGGL((seg_kernel<U, M>), dim3(blocks), dim3(256), 0, 0, xx, bb, yy, n, seg, out)
                    L(2, 0); L(2, 1); L(2, 2); L(2, 3); L(4, 0); L(4, 1); L(4, 2); L(4, 3); L(8, 0); L(8, 1); L(8, 2); L(8, 3);
#undef L
                };
                ms = time_it(go);
                printf("seg %5d blocks U=%d %-5s: %8.1f us %.2f TB/s\n", blocks, u, mixn[mix], ms * 1e3, mixb[mix] * B / (ms * 1e-3) / 1e12);
            }
        }
    }
    for (int blocks : {1024, 2048, 4096, 8192}) {
#define WC(V, NT) { float m2 = time_it([&] { hipLaunchKernelGGL((wide_copy<V, NT>), dim3(blocks), dim3(256), 0, 0, (const d2*)x, (d2*)y, n); }); \
        printf("wide  %5d blocks V=%d nt=%d: %8.1f us %.2f TB/s\n", blocks, V, (int)NT, m2 * 1e3, 2 * B / (m2 * 1e-3) / 1e12); }
#define WV(U, NT) { float m2 = time_it([&] { hipLaunchKernelGGL((wave_copy<U, NT>), dim3(blocks), dim3(256), 0, 0, (const d2*)x, (d2*)y, n); }); \
        printf("wave  %5d blocks U=%d nt=%d: %8.1f us %.2f TB/s\n", blocks, U, (int)NT, m2 * 1e3, 2 * B / (m2 * 1e-3) / 1e12); }
        WC(2, false) WC(4, false) WC(4, true) WV(4, false) WV(8, false) WV(4, true) WV(8, true)
#undef WC
#undef WV
    }
    return 0;
}
