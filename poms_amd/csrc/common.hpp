// Shared definitions for the gfx950 kernels of libpoms_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace poms {

constexpr int kBlock = 256;  // 4 wave64s per workgroup
// doubles of the per-context partial-sum scratch (poms_ctx::scratch); every kernel
// that writes per-block partials there caps its grid at this (vec_ops.hip asserts it)
constexpr int64_t kScratch = 1 << 16;

enum Form : int { FORM_SINGLE = 0, FORM_SUM = 1, FORM_STENCIL = 2 };
enum Epi : int { EPI_APPLY = 0, EPI_RESID = 1, EPI_JACOBI = 2,
                 EPI_JACOBI0 = 3,   /* two damped-Jacobi sweeps from x0 = 0 (x planes = b) */
                 EPI_APPLYDOT = 4,  /* y = A x and per-block sums of x . y              */
                 EPI_DIAG = 5,      /* x = scale b / diag(A) (general stencil form)    */
                 EPI_JACOBI2 = 6,   /* two sweeps from x in one launch (2D, kron_2d.hip) */
                 EPI_JACOBI3Z = 7   /* sweeps 1-3 from x = 0 in one launch (2D, kron_2d.hip) */ };

// Geometry of one fused Kronecker launch (all extents local to this rank's slab).
struct KronGeom {
    int64_t s0, s1;      // plane / row strides of the padded layout (doubles)
    int n0, n1, n2;      // interior extents
    int pd0, pd1, pd2;   // storage pads (ghost widths)
    int g0;              // global index of local plane 0 (axis-0 coefficient rows)
    int z_begin, z_end;  // output planes [z_begin, z_end)
    int chunk;           // output planes per workgroup (3D)
    int tiles2, tiles1, nchunks;
    int nch1;            // chunks of [z_begin, z_end); chunks nch1.. cover [z2_begin, z2_end)
    int z2_begin, z2_end;  // optional second plane range of the same launch (the other slab boundary)
    int tout;            // output columns per 64-column tile (v3 / v4 kernels; <= 64 - 2P)
    int order = 0;       // v5 / v6 tile order within an XCD: 0 = axis-2 tiles fastest, 1 = axis-1 tiles fastest
    const int* sched = nullptr;   // v5: tile of each workgroup (kron_v5_sched), or null: the XCD-contiguous order
};

// Output planes [z0, z1) of axis-0 chunk `ch` (3D launches may cover two ranges).
__device__ __forceinline__ void chunk_planes(const KronGeom& g, int ch, int& z0, int& z1) {
    if (ch < g.nch1) {
        z0 = g.z_begin + ch * g.chunk;
        z1 = min(z0 + g.chunk, g.z_end);
    } else {
        z0 = g.z2_begin + (ch - g.nch1) * g.chunk;
        z1 = min(z0 + g.chunk, g.z2_end);
    }
}

// One launch of the general-stencil kernel (stencil_general.hip): owned planes
// [z_begin, z_end) u [z2_begin, z2_end) of the local slab.
struct StencilGeom {
    int64_t s0, s1;          // plane / row strides of the padded vectors
    int n0, n1, n2;          // local interior extents
    int pd0, pd1, pd2;       // storage pads
    int p0, p1, p2;          // stencil half-widths
    int w0, w1, w2;          // 2 p_d + 1 (1 on unused axes)
    int64_t cstride;         // doubles per coefficient plane (n0 n1 n2)
    int z_begin, z_end, z2_begin, z2_end;
};

// One axis of an on-device quadrature assembly (stencil_general.hip): elements
// (non-empty knot spans), nq Gauss points each, the p+1 local B-splines.
struct AssembleAxis {
    const int* first;      // nel: global index of the element's first basis function
    const int* es;         // n  : first element of basis function i's support
    const int* ee;         // n  : last element of basis function i's support
    const double* basis;   // nel*nq*(p+1)*2: value, derivative
    const double* w;       // nel*nq: quadrature weights (with the element Jacobian)
    int nel, nq, p, n;
};

// pcg's scalars folded into the flat vector updates (one rank, round 6): every block
// reduces `n` per-block partials in reduce_partials_kernel's order (the same bits as
// the one-block kernels they replace) and forms the scalar itself; block 0 stores it.
//  * V_RUPD (alpha): p.q from the apply + dot partials, alpha = sc[sr] / p.q; block 0
//    stores p.q, 1, alpha, alpha at sc[1..4] (pcg_alpha_kernel's slots) and, with
//    copy_sr, sc[0] = sc[sr] (the s.r_old update a folded beta left pending);
//  * V_XPUPD (beta): s.r_new from the last sweep's x . rhs partials, beta = s.r_new /
//    sc[0]; block 0 stores s.r_new at sc[6] and beta at sc[5] -- NOT sc[0], which the
//    other blocks are reading (the next r update's copy_sr does that).
struct AlphaFold {
    const double* part = nullptr;   // null: no fold, the coefficients as before
    int n = 0;
    double* sc = nullptr;
    int sr = 0;                     // V_RUPD: slot of s.r
    int copy_sr = 0;
};

// 2D Jacobi expressions shared by kron_v3_kernel and kron2d_j2_kernel, written with
// contraction off so that both kernels form the same bits whatever the compiler
// fuses around them (the two-sweep launch must reproduce two single sweeps):
// diag(A) = d1a d2a + d1b d2b, and x_out = x + dr with dr rounded.
__device__ __forceinline__ double diag2d_sum(double d1a, double d2a, double d1b, double d2b) {
#pragma clang fp contract(off)
    return d1a * d2a + d1b * d2b;
}
__device__ __forceinline__ double add_nc(double a, double b) {
#pragma clang fp contract(off)
    return a + b;
}

// Padded row layout used by the row-wise vector kernels.
struct RowGeom {
    int64_t s0, s1;
    int n0, n1, n2;
    int pd0, pd1, pd2;
};

// One axis of a Kronecker transfer (restriction / prolongation), see transfer.hip.
struct AxisPass {
    int64_t nA, nB1, nB2;                     // independent thread space
    int64_t in_base, in_sa, in_sb1, in_sb2, in_si;
    int64_t out_base, out_sa, out_sb1, out_sb2, out_si;
    int nI;          // fine extent of the contracted / expanded axis (local)
    int nJ;          // coarse extent
    int goff;        // global fine row of local i = 0
    int accumulate;  // prolongation: out += (1) or out = (0)
};

// Symmetric-Toeplitz interior of the band factors (v2 fast path): rows
// [lo, hi) of an axis equal one symmetric row; t?[j] = row[P + j] = row[P - j].
struct ToepConst {
    double t1a[6], t1b[6];   // axis 1 (A1, B1)
    double t0a[6], t0b[6];   // axis 0 (A0, M0), global rows
    double t2a[6], t2b[6];   // axis 2 (M2, K2)
    int lo1, hi1, lo0, hi0, lo2, hi2;
    double rdi;              // 1/diag(A) inside the Toeplitz interior of every axis (3D; 0 if empty)
};

// Device pointers of one fused Kronecker launch.
struct KronPtrs {
    const double* x;
    double* y;
    const double* b;
    const double *a0t, *b0t, *a1, *b1, *a2, *b2;
    double* partial;    // Jacobi: per-block sums of dr.dr (or null)
    double* partial2;   // Jacobi: per-block sums of x_out.b (or null)
    const double* rdiag0 = nullptr;  // 1/diag(A) per global plane inside the axis-1/2 Toeplitz interior
};

// Banded LU factors of one axis of a Kronecker solve (kron_solve.hip).
struct BandLU {
    const double* L;  // n * kl   : L[j*kl + t-1] = l(j+t, j), t = 1..kl (0 past the end)
    const double* U;  // n * (K+1): U[j*(K+1) + t] = u(j-t, j), t = 0..K (0 before the start)
    const int* piv;   // n        : ipiv(j) - j in [0, kl]
    int n, kl, K;     // K = kl + ku (fill-in widens U by kl)
};

// element (io, i2, j) of a line set at base + io*so + i2 + j*sa
struct LineGeom {
    int64_t base, so, sa;
    int64_t no, n2;
};

// rows r in [0, nrows): row start base + (r / n1)*s0 + (r % n1)*s1, line along +1
struct RowLines {
    int64_t base, s0, s1;
    int64_t n1, nrows;
};

void set_error(const std::string& msg);

// Block-wide (256 threads) sum; result valid in thread 0.
__device__ inline double block_sum_256(double v, double* red4) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) red4[wv] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) s = (red4[0] + red4[1]) + (red4[2] + red4[3]);
    return s;
}

// ---- raw buffer access (hardware range check: loads past num_records return
// 0, stores past it are dropped) ------------------------------------------------
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ double bload(__amdgpu_buffer_rsrc_t r, int off_bytes) {
    u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, off_bytes, 0, 0);
    return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void bstore(__amdgpu_buffer_rsrc_t r, int off_bytes, double d) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, d), r, off_bytes, 0, 0);
}
// loads / stores with a scalar (per-plane) offset on a whole-array resource
__device__ __forceinline__ double bload_s(__amdgpu_buffer_rsrc_t r, int voff, unsigned soff) {
    u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, (int)soff, 0);
    return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void bstore_s(__amdgpu_buffer_rsrc_t r, int voff, unsigned soff, double d) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, d), r, voff, (int)soff, 0);
}
// store with an explicit cache-policy field (gfx950 aux: bit0 sc0, bit1 nt, bit4 sc1)
template <int AUX>
__device__ __forceinline__ void bstore_p(__amdgpu_buffer_rsrc_t r, int off_bytes, double d) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, d), r, off_bytes, 0, AUX);
}
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <int AUX>
__device__ __forceinline__ void bstore2_p(__amdgpu_buffer_rsrc_t r, int off_bytes, double d0, double d1) {
    u32x4 v;
    const u32x2 a = __builtin_bit_cast(u32x2, d0), b = __builtin_bit_cast(u32x2, d1);
    v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off_bytes, 0, AUX);
}

// 16-B store of two doubles with a scalar (per-plane) offset on a whole-array resource
__device__ __forceinline__ void bstore2_s(__amdgpu_buffer_rsrc_t r, int voff, unsigned soff, double d0, double d1) {
    u32x4 v;
    const u32x2 a = __builtin_bit_cast(u32x2, d0), b = __builtin_bit_cast(u32x2, d1);
    v.x = a.x; v.y = a.y; v.z = b.x; v.w = b.y;
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, (int)soff, 0);
}

// bytes of `planes_left` padded planes of s0 doubles, clamped to 2^31-1
__device__ __forceinline__ uint32_t plane_bytes(int64_t planes_left, int64_t s0) {
    if (planes_left <= 0) return 0u;
    const int64_t b = planes_left * s0 * 8;
    return b > 0x7fffffffLL ? 0x7fffffffu : (uint32_t)b;
}

}  // namespace poms

#define POMS_HIP_CHECK(expr)                                                   \
    do {                                                                       \
        hipError_t _e = (expr);                                                \
        if (_e != hipSuccess) {                                                \
            ::poms::set_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)
