// Micro-benchmark of the VALU operations the Kronecker kernels are built from
// (gfx950): FP64 FMA throughput / dependent latency, 32-bit DPP lane shifts,
// ds_read_b128.  Prints per-wave-instruction costs in shader-clock cycles
// (s_memtime counts the constant 100 MHz reference clock on gfx9x, so clocks
// are derived from the wall time and the known instruction count instead).
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench && /tmp/ubench
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int CHAINS>
__global__ void __launch_bounds__(256) fma_kernel(double* out, int iters, double a, double b) {
    double v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) v[c] = fma(v[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += v[c];
    if (s == 1234.5) out[threadIdx.x] = s;
}

__device__ __forceinline__ double dshr(double v) {
    const int2 w = __builtin_bit_cast(int2, v);
    const int lo = __builtin_amdgcn_update_dpp(0, w.x, 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, w.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, make_int2(lo, hi));
}

template <int CHAINS>
__global__ void __launch_bounds__(256) dpp_kernel(double* out, int iters) {
    double v[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) v[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) v[c] = dshr(v[c]);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += v[c];
    if (s == 1234.5) out[threadIdx.x] = s;
}

// 7-tap stencil along lanes: 6 DPP shifts + 7 FMA per output, 4 independent rows
__global__ void __launch_bounds__(256) stencil_kernel(double* out, int iters, double c0, double c1, double c2,
                                                      double c3) {
    double x[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = threadIdx.x * 1e-3 + r;
    double acc = 0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double sh[7];
            sh[3] = x[r];
#pragma unroll
            for (int d = 1; d <= 3; ++d) { sh[3 - d] = dshr(sh[4 - d]); sh[3 + d] = dshr(sh[2 + d] * 1.0000001); }
            double a = c0 * sh[3];
            a = fma(c1, sh[2], a); a = fma(c1, sh[4], a);
            a = fma(c2, sh[1], a); a = fma(c2, sh[5], a);
            a = fma(c3, sh[0], a); a = fma(c3, sh[6], a);
            x[r] = a;
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) acc += x[r];
    if (acc == 1234.5) out[threadIdx.x] = acc;
}

template <typename F>
static float time_it(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    f();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    double* out;
    CK(hipMalloc(&out, 4096 * sizeof(double)));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double clk = prop.clockRate * 1e3;  // Hz (max)
    printf("CUs %d max clock %.0f MHz\n", cus, clk / 1e6);
    const int iters = 4096;
    // throughput: waves/SIMD = blocks*4/(cus*4)
    for (int wps : {1, 2, 4, 8}) {
        const int blocks = cus * wps;   // 256 threads = 4 waves -> wps waves per SIMD
        float ms = time_it([&] { hipLaunchKernelGGL(fma_kernel<8>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999, 1e-3); });
        const double winstr = (double)blocks * 4 * iters * 16 * 8;        // wave-instructions
        const double per_simd = winstr / (cus * 4);
        printf("fma f64 8 chains, %d waves/SIMD: %.3f ms -> %.2f clk/wave-instr @max clock, %.1f TFLOP/s\n", wps, ms,
               ms * 1e-3 * clk / per_simd, winstr * 64 * 2 / (ms * 1e-3) / 1e12);
    }
    for (int wps : {1, 4}) {
        const int blocks = cus * wps;
        float ms = time_it([&] { hipLaunchKernelGGL(fma_kernel<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999, 1e-3); });
        const double per_simd = (double)blocks * 4 * iters * 16 / (cus * 4);
        printf("fma f64 1 chain (latency), %d waves/SIMD: %.2f clk/instr\n", wps, ms * 1e-3 * clk / per_simd);
    }
    for (int wps : {1, 4}) {
        const int blocks = cus * wps;
        float ms = time_it([&] { hipLaunchKernelGGL(dpp_kernel<8>, dim3(blocks), dim3(256), 0, 0, out, iters); });
        const double per_simd = (double)blocks * 4 * iters * 16 * 8 * 2 / (cus * 4);  // 2 dpp per double
        printf("dpp b32 wave_shr, 8 chains, %d waves/SIMD: %.2f clk/dpp-instr\n", wps, ms * 1e-3 * clk / per_simd);
        float ms1 = time_it([&] { hipLaunchKernelGGL(dpp_kernel<1>, dim3(blocks), dim3(256), 0, 0, out, iters); });
        const double per1 = (double)blocks * 4 * iters * 16 * 2 / (cus * 4);
        printf("dpp b32 wave_shr, 1 chain, %d waves/SIMD: %.2f clk/dpp-instr\n", wps, ms1 * 1e-3 * clk / per1);
    }
    for (int wps : {2, 4, 8}) {
        const int blocks = cus * wps;
        float ms = time_it([&] { hipLaunchKernelGGL(stencil_kernel, dim3(blocks), dim3(256), 0, 0, out, iters, 0.5, 0.1, 0.05, 0.01); });
        const double outs = (double)blocks * 4 * iters * 4;   // wave-outputs (64 lanes)
        printf("7-tap DPP stencil, %d waves/SIMD: %.2f clk per wave-output (12 dpp + 3 mul + 7 fma)\n", wps,
               ms * 1e-3 * clk / (outs / (cus * 4)));
    }
    return 0;
}
