// Interior-only vector kernels on the padded stencil layout (spl StencilVector
// algebra used by sources/solvers.py) plus deterministic reductions and the
// dense coarse-grid mat-vec.
//
// Layout walk: one wave64 per interior row (i0, i1); lanes stride the
// unit-stride axis i2 (coalesced 8-B accesses); grid-stride over rows.
// HBM-bound: 16-32 B per DOF, no reuse.
#include "common.hpp"

#include <cstdlib>

namespace poms {

enum VecOp : int { V_AXPBY = 0, V_SCALE = 1, V_FILL = 2, V_DOT = 3, V_PCGUPD = 4, V_RUPD = 5, V_XPUPD = 6,
                  V_SCALEDOT = 7 /* z = a x and z.z (flat kernel only) */ };

// grid caps (= partial sums per launch): the flat vector kernels run one pass per
// thread up to 65536 blocks of 256 (grid-stride beyond): at 515^3 the r update
// took 720 us with 4096 grid-stride blocks and 640 with 65536 (x/p update 1221 ->
// 1042 us; profiles/r03/s3/vec_blocks_16k_64k.log); the per-row kernels keep 4096
constexpr int kMaxPartials = 65536;
constexpr int kMaxRowPartials = 4096;
static_assert(kMaxPartials <= kScratch && kMaxRowPartials <= kScratch,
              "vector-kernel partials must fit the context scratch (advisor, round 3)");

template <int OP>
__global__ void __launch_bounds__(256)
vec_rows_kernel(const RowGeom g, double a, double b,
                const double* __restrict__ x, const double* __restrict__ yv,
                double* __restrict__ z, double* __restrict__ w, const double* __restrict__ q,
                double* __restrict__ partial, const double* __restrict__ ab) {
    __shared__ double red[4];
    if (ab != nullptr) { a = ab[0]; b = ab[1]; }   // coefficients from device memory
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t nrows = (int64_t)g.n0 * g.n1;
    double s = 0.0;
    for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < nrows; row += (int64_t)gridDim.x * 4) {
        const int i0 = (int)(row / g.n1);
        const int i1 = (int)(row - (int64_t)i0 * g.n1);
        const int64_t base = (int64_t)(i0 + g.pd0) * g.s0 + (int64_t)(i1 + g.pd1) * g.s1 + g.pd2;
        for (int c = lane; c < g.n2; c += 64) {
            const int64_t o = base + c;
            if constexpr (OP == V_AXPBY) {
                z[o] = a * x[o] + b * yv[o];
            } else if constexpr (OP == V_SCALE) {
                z[o] = a * x[o];
            } else if constexpr (OP == V_FILL) {
                z[o] = a;
            } else if constexpr (OP == V_DOT) {
                s = fma(x[o], yv[o], s);
            } else if constexpr (OP == V_PCGUPD) {  // z = x += a*p (yv = p), w = r -= a*q
                z[o] = fma(a, yv[o], z[o]);
                const double rn = fma(-a, q[o], w[o]);
                w[o] = rn;
                s = fma(rn, rn, s);
            } else if constexpr (OP == V_RUPD) {    // w = r -= a*q, r.r
                const double rn = fma(-a, q[o], w[o]);
                w[o] = rn;
                s = fma(rn, rn, s);
            } else {                                 // V_XPUPD: z = x += a*p_old; w = p = s + b*p_old (x = s)
                const double po = w[o];
                z[o] = fma(a, po, z[o]);
                w[o] = x[o] + b * po;
            }
        }
    }
    if constexpr (OP == V_DOT || OP == V_PCGUPD || OP == V_RUPD) {
        const double t = block_sum_256(s, red);
        if (threadIdx.x == 0) partial[blockIdx.x] = t;
    }
}

// The same element-wise ops over a flat range of whole padded planes (interior
// planes only): 16-B accesses, U of them in flight per thread, non-temporal
// stores.  Valid because the ghost rows / columns (and dead pitch columns) of
// every vector are zero and every op maps zeros to zeros: results there stay
// zero and add nothing to the reductions.  `head` / `tail` are single leading /
// trailing elements outside the 16-B aligned middle (done by thread 0).
template <int OP>
__device__ __forceinline__ void vec_elem(double a, double b, const double* x, const double* yv, double* z,
                                         double* w, const double* q, int64_t o, double& s) {
    if constexpr (OP == V_AXPBY) {
        z[o] = a * x[o] + b * yv[o];
    } else if constexpr (OP == V_SCALE) {
        z[o] = a * x[o];
    } else if constexpr (OP == V_DOT) {
        s = fma(x[o], yv[o], s);
    } else if constexpr (OP == V_PCGUPD) {
        z[o] = fma(a, yv[o], z[o]);
        const double rn = fma(-a, q[o], w[o]);
        w[o] = rn;
        s = fma(rn, rn, s);
    } else if constexpr (OP == V_RUPD) {
        const double rn = fma(-a, q[o], w[o]);
        w[o] = rn;
        s = fma(rn, rn, s);
    } else if constexpr (OP == V_XPUPD) {
        const double po = w[o];
        z[o] = fma(a, po, z[o]);
        w[o] = x[o] + b * po;
    } else if constexpr (OP == V_SCALEDOT) {
        const double zo = a * x[o];
        z[o] = zo;
        s = fma(zo, zo, s);
    }
}

template <int OP, bool NTL = true>   // NTL: non-temporal loads (tuning: POMS_VEC_LOADS=plain)
__global__ void __launch_bounds__(256)
vec_flat_kernel(const int head, const int64_t nd2, const int tail, double a, double b,
                const double* __restrict__ x, const double* __restrict__ yv, double* __restrict__ z,
                double* __restrict__ w, const double* __restrict__ q, double* __restrict__ partial,
                const double* __restrict__ ab, const AlphaFold af) {
    if (ab != nullptr) { a = ab[0]; b = ab[1]; }   // coefficients from device memory
    typedef double d2 __attribute__((ext_vector_type(2)));
    constexpr int U = 4;
    __shared__ double red[4];
    if constexpr (OP == V_RUPD || OP == V_XPUPD) {
        if (af.part != nullptr) {   // alpha / beta from partials (see AlphaFold)
            double sp = 0.0;
            for (int i = threadIdx.x; i < af.n; i += 256) sp += af.part[i];
            const double t = block_sum_256(sp, red);
            if (threadIdx.x == 0) {
                double v;
                if constexpr (OP == V_RUPD) {   // t = p.q
                    v = af.sc[af.sr] / t;
                    if (blockIdx.x == 0) {
                        af.sc[1] = t;
                        af.sc[2] = 1.0;
                        af.sc[3] = v;
                        af.sc[4] = v;
                        if (af.copy_sr) af.sc[0] = af.sc[af.sr];
                    }
                } else {                        // t = s.r_new
                    v = t / af.sc[0];
                    if (blockIdx.x == 0) {
                        af.sc[6] = t;
                        af.sc[5] = v;
                    }
                }
                red[0] = v;
            }
            __syncthreads();
            if constexpr (OP == V_RUPD) a = red[0];
            else b = red[0];
            __syncthreads();   // (red is the final reduction's again)
        }
    }
    double s = 0.0;
    const d2* X = (const d2*)(x + head);
    const d2* Y = (const d2*)(yv + head);
    d2* Z = (d2*)(z + head);
    d2* Wv = (d2*)(w + head);
    const d2* Q = (const d2*)(q + head);
    const int64_t step = (int64_t)gridDim.x * 256 * U;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < nd2; base += step) {
        d2 xa[U], ya[U], za[U], wa[U], qa[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < nd2) {
                // non-temporal loads as well as stores: each operand is streamed once
                // (tools/ubench_copy.hip: 1 KiB per wave and load, nt loads + nt stores
                // 6.1-6.2 TB/s against 5.7 with plain loads)
                auto ld = [](const d2* ptr) { if constexpr (NTL) return __builtin_nontemporal_load(ptr); else return *ptr; };
                if constexpr (OP == V_AXPBY || OP == V_SCALE || OP == V_DOT || OP == V_XPUPD || OP == V_SCALEDOT)
                    xa[u] = ld(X + i);
                if constexpr (OP == V_AXPBY || OP == V_DOT || OP == V_PCGUPD) ya[u] = ld(Y + i);
                if constexpr (OP == V_PCGUPD || OP == V_XPUPD) za[u] = ld(Z + i);
                if constexpr (OP == V_PCGUPD || OP == V_RUPD || OP == V_XPUPD) wa[u] = ld(Wv + i);
                if constexpr (OP == V_PCGUPD || OP == V_RUPD) qa[u] = ld(Q + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < nd2) {
                if constexpr (OP == V_AXPBY) {
                    __builtin_nontemporal_store(a * xa[u] + b * ya[u], Z + i);
                } else if constexpr (OP == V_SCALE) {
                    __builtin_nontemporal_store(a * xa[u], Z + i);
                } else if constexpr (OP == V_SCALEDOT) {   // (with a = 1: the bits of V_SCALE + V_DOT(z, z))
                    const d2 zn = a * xa[u];
                    __builtin_nontemporal_store(zn, Z + i);
                    s = fma(zn.x, zn.x, s);
                    s = fma(zn.y, zn.y, s);
                } else if constexpr (OP == V_DOT) {
                    s = fma(xa[u].x, ya[u].x, s);
                    s = fma(xa[u].y, ya[u].y, s);
                } else if constexpr (OP == V_PCGUPD) {
                    __builtin_nontemporal_store(a * ya[u] + za[u], Z + i);
                    d2 rn;
                    rn.x = fma(-a, qa[u].x, wa[u].x);
                    rn.y = fma(-a, qa[u].y, wa[u].y);
                    __builtin_nontemporal_store(rn, Wv + i);
                    s = fma(rn.x, rn.x, s);
                    s = fma(rn.y, rn.y, s);
                } else if constexpr (OP == V_RUPD) {
                    d2 rn;
                    rn.x = fma(-a, qa[u].x, wa[u].x);
                    rn.y = fma(-a, qa[u].y, wa[u].y);
                    __builtin_nontemporal_store(rn, Wv + i);
                    s = fma(rn.x, rn.x, s);
                    s = fma(rn.y, rn.y, s);
                } else {   // V_XPUPD
                    d2 zn, wn;
                    zn.x = fma(a, wa[u].x, za[u].x);
                    zn.y = fma(a, wa[u].y, za[u].y);
                    wn.x = xa[u].x + b * wa[u].x;
                    wn.y = xa[u].y + b * wa[u].y;
                    __builtin_nontemporal_store(zn, Z + i);
                    __builtin_nontemporal_store(wn, Wv + i);
                }
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (head) vec_elem<OP>(a, b, x, yv, z, w, q, 0, s);
        if (tail) vec_elem<OP>(a, b, x, yv, z, w, q, head + 2 * nd2, s);
    }
    if constexpr (OP == V_DOT || OP == V_PCGUPD || OP == V_RUPD || OP == V_SCALEDOT) {
        const double t = block_sum_256(s, red);
        if (threadIdx.x == 0) partial[blockIdx.x] = t;
    }
}

// Deterministic single-block reduction of `count` partials.
__global__ void __launch_bounds__(256)
reduce_partials_kernel(const double* __restrict__ partial, int count, double* __restrict__ out, int accumulate) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < count; i += 256) s += partial[i];
    const double t = block_sum_256(s, red);
    if (threadIdx.x == 0) out[0] = accumulate ? out[0] + t : t;
}

// Deterministic single-block reduction of many partials (the flat vector kernels'
// up to kMaxPartials blocks): 1024 threads, each a strided running sum with four
// independent accumulators, then the wave butterflies and the 16 wave sums in order.
// (reduce_partials_kernel keeps its 256-thread order: the native loop's host-side
// sums of the operator launches' partials reproduce it bit for bit.)
__global__ void __launch_bounds__(1024)
reduce_partials_wide_kernel(const double* __restrict__ partial, int count, double* __restrict__ out, int accumulate) {
    __shared__ double red[16];
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int i = threadIdx.x;
    for (; i + 3 * 1024 < count; i += 4 * 1024) {
        s0 += partial[i];
        s1 += partial[i + 1024];
        s2 += partial[i + 2 * 1024];
        s3 += partial[i + 3 * 1024];
    }
    for (; i < count; i += 1024) s0 += partial[i];
    double s = (s0 + s1) + (s2 + s3);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < 16; ++w) t += red[w];
        out[0] = accumulate ? out[0] + t : t;
    }
}

// x = scale * b / diag(A), optional ||x||^2 partials.  diag(A) from the 1D
// band diagonals exactly as in the fused kernels' JACOBI epilogue; the
// axis-2 diagonals come as contiguous arrays (dg2a, dg2b) so the loads are
// coalesced, and 1/diag is v_rcp_f64 + two Newton steps.
// ROWBLK: one row per workgroup, its columns over all 256 threads (2D operators: a
// wave per row over 256 rows left each lane a latency-bound march of n2 / 64 steps,
// 13.3 us for 1027^2 against 9.7 us for a whole Jacobi sweep)
template <bool IS3D, int FORM, bool ROWBLK = false>
__global__ void __launch_bounds__(256)
diag_scale_kernel(const RowGeom g, const int P, const int g0, const double scale,
                  const double* __restrict__ bvec, double* __restrict__ xout,
                  const double* __restrict__ a0t, const double* __restrict__ b0t,
                  const double* __restrict__ a1, const double* __restrict__ b1,
                  const double* __restrict__ dg2a, const double* __restrict__ dg2b,
                  double* __restrict__ partial) {
    __shared__ double red[4];
    const int W = 2 * P + 1;
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    const int64_t nrows = (int64_t)g.n0 * g.n1;
    double s = 0.0;
    const int64_t row0 = ROWBLK ? blockIdx.x : (int64_t)blockIdx.x * 4 + wv;
    const int64_t rstep = ROWBLK ? nrows : (int64_t)gridDim.x * 4;
    const int cl = ROWBLK ? (int)threadIdx.x : lane, cstep = ROWBLK ? 256 : 64;
    for (int64_t row = row0; row < nrows; row += rstep) {
        const int i0 = (int)(row / g.n1);
        const int i1 = (int)(row - (int64_t)i0 * g.n1);
        const int64_t base = (int64_t)(i0 + g.pd0) * g.s0 + (int64_t)(i1 + g.pd1) * g.s1 + g.pd2;
        const double d1a = a1[i1 * W + P];
        const double d1b = (FORM == FORM_SUM) ? b1[i1 * W + P] : 0.0;
        double d0a = 1.0, d0b = 0.0;
        if constexpr (IS3D) {
            d0a = a0t[(g0 + i0 + P) * W + P];
            if constexpr (FORM == FORM_SUM) d0b = b0t[(g0 + i0 + P) * W + P];
        }
        for (int c = cl; c < g.n2; c += cstep) {
            const double d2a = dg2a[c];
            double diag;
            if constexpr (FORM == FORM_SUM) {
                const double d2b = dg2b[c];
                if constexpr (IS3D) diag = d0a * (d1a * d2a) + d0b * (d1b * d2a + d1a * d2b);
                else diag = diag2d_sum(d1a, d2a, d1b, d2b);   // (the 2D sweeps' diag bits)
            } else {
                diag = d0a * d1a * d2a;
            }
            double rc = __builtin_amdgcn_rcp(diag);
            double e = fma(-diag, rc, 1.0);
            rc = fma(rc, e, rc);
            e = fma(-diag, rc, 1.0);
            rc = fma(rc, e, rc);
            const double v = scale * bvec[base + c] * rc;
            xout[base + c] = v;
            s = fma(v, v, s);
        }
    }
    if (partial != nullptr) {
        const double t = block_sum_256(s, red);
        if (threadIdx.x == 0) partial[blockIdx.x] = t;
    }
}

// y = M x, dense row-major n x n; one wave per row.
__global__ void __launch_bounds__(256)
dense_matvec_kernel(const int n, const double* __restrict__ M, const double* __restrict__ x,
                    double* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n) return;
    const double* mr = M + (int64_t)row * n;
    double s = 0.0;
    for (int j = lane; j < n; j += 64) s = fma(mr[j], x[j], s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) y[row] = s;
}

static int row_blocks(const RowGeom& g) {
    const int64_t nrows = (int64_t)g.n0 * g.n1;
    int64_t nb = (nrows + 3) / 4;
    if (nb > kMaxRowPartials) nb = kMaxRowPartials;
    if (nb < 1) nb = 1;
    return (int)nb;
}

int vec_launch(int op, const RowGeom& g, double a, double b, const double* x, const double* y,
               double* z, double* w, const double* q, double* partial, hipStream_t st,
               int* nblk_out, const double* ab) {
    const int nb = row_blocks(g);
    if (nblk_out) *nblk_out = nb;
    switch (op) {
#define POMS_VL(OPV)                                                                        \
    case OPV:                                                                               \
        hipLaunchKernelGGL(vec_rows_kernel<OPV>, dim3(nb), dim3(256), 0, st, g, a, b, x, y, z, \
                           w, q, partial, ab);                                              \
        return 0;
        POMS_VL(V_AXPBY)
        POMS_VL(V_SCALE)
        POMS_VL(V_FILL)
        POMS_VL(V_DOT)
        POMS_VL(V_PCGUPD)
        POMS_VL(V_RUPD)
        POMS_VL(V_XPUPD)
#undef POMS_VL
    }
    set_error("unknown vector op");
    return 1;
}

// Zero every padded entry outside the interior -- ghost planes, ghost rows, ghost
// columns and dead pitch columns -- in one launch (a fresh vector's ghosts; the
// interior is left as it is).  One wave per padded row, four rows per block.
__global__ void __launch_bounds__(256)
zero_ghosts_kernel(const RowGeom g, int64_t nrows, int nr1, double* __restrict__ z) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= nrows) return;
    const int lane = threadIdx.x & 63;
    const int64_t i0 = row / nr1;
    const int i1 = (int)(row - i0 * nr1);
    double* __restrict__ zr = z + i0 * g.s0 + (int64_t)i1 * g.s1;
    const bool ghost = i0 < g.pd0 || i0 >= g.pd0 + g.n0 || i1 < g.pd1 || i1 >= g.pd1 + g.n1;
    if (ghost) {
        for (int64_t c = lane; c < g.s1; c += 64) zr[c] = 0.0;
    } else {
        if (lane < g.pd2) zr[lane] = 0.0;
        for (int64_t c = g.pd2 + g.n2 + lane; c < g.s1; c += 64) zr[c] = 0.0;
    }
}

int zero_ghosts_launch(const RowGeom& g, double* z, hipStream_t st) {
    const int nr1 = g.n1 + 2 * g.pd1;
    const int64_t nrows = (int64_t)(g.n0 + 2 * g.pd0) * nr1;
    if (nrows < 1) return 0;
    hipLaunchKernelGGL(zero_ghosts_kernel, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, st, g, nrows, nr1, z);
    return 0;
}

// Flat form over `count` doubles starting at each pointer (whole interior planes).
// The pointers must share their alignment modulo 16 B (same layout): returns 1
// (nothing launched) otherwise, and for ops without a flat form (V_FILL).
int vec_flat_launch(int op, int64_t count, double a, double b, const double* x, const double* y,
                    double* z, double* w, const double* q, double* partial, hipStream_t st,
                    int* nblk_out, const double* ab, const AlphaFold* af) {
    const AlphaFold afv = (af != nullptr && (op == V_RUPD || op == V_XPUPD)) ? *af : AlphaFold{};
    if (op == V_FILL || count < 4) return 1;
    int mis = -1;
    for (const void* ptr : {(const void*)x, (const void*)y, (const void*)z, (const void*)w, (const void*)q}) {
        if (!ptr) continue;
        const int m = (int)(reinterpret_cast<uintptr_t>(ptr) & 15);
        if (m & 7) return 1;
        if (mis >= 0 && m != mis) return 1;
        mis = m;
    }
    if (mis < 0) return 1;
    const int head = mis ? 1 : 0;
    const int64_t nd2 = (count - head) / 2;
    const int tail = (int)((count - head) - 2 * nd2);
    int64_t nb = (nd2 + 256 * 4 - 1) / (256 * 4);
    static const int cap = [] {   // grid cap (tuning: POMS_VEC_BLOCKS, at most kMaxPartials)
        const char* e = getenv("POMS_VEC_BLOCKS");
        const int v = e ? atoi(e) : kMaxPartials;
        return v < 64 ? 64 : v > kMaxPartials ? kMaxPartials : v;
    }();
    if (nb > cap) nb = cap;
    if (nb < 1) nb = 1;
    if (nblk_out) *nblk_out = (int)nb;
    static const bool plain = [] {
        const char* e = getenv("POMS_VEC_LOADS");
        return e && e[0] == 'p';
    }();
    switch (op) {
#define POMS_VF(OPV)                                                                                  \
    case OPV:                                                                                         \
        if (plain)                                                                                    \
            hipLaunchKernelGGL((vec_flat_kernel<OPV, false>), dim3((int)nb), dim3(256), 0, st, head, nd2, tail, a, b, \
                               x, y, z, w, q, partial, ab, afv);                                      \
        else                                                                                          \
            hipLaunchKernelGGL((vec_flat_kernel<OPV, true>), dim3((int)nb), dim3(256), 0, st, head, nd2, tail, a, b, \
                               x, y, z, w, q, partial, ab, afv);                                      \
        return 0;
        POMS_VF(V_AXPBY)
        POMS_VF(V_SCALE)
        POMS_VF(V_DOT)
        POMS_VF(V_PCGUPD)
        POMS_VF(V_RUPD)
        POMS_VF(V_XPUPD)
        POMS_VF(V_SCALEDOT)
#undef POMS_VF
    }
    return 1;
}

int reduce_launch(const double* partial, int count, double* out, hipStream_t st, int accumulate) {
    hipLaunchKernelGGL(reduce_partials_kernel, dim3(1), dim3(256), 0, st, partial, count, out, accumulate);
    return 0;
}

int reduce_wide_launch(const double* partial, int count, double* out, hipStream_t st, int accumulate) {
    if (count <= 4096) return reduce_launch(partial, count, out, st, accumulate);
    hipLaunchKernelGGL(reduce_partials_wide_kernel, dim3(1), dim3(1024), 0, st, partial, count, out, accumulate);
    return 0;
}

// Workgroups (= partial sums) of one diag_scale_launch
int diag_scale_blocks(bool is3d, const RowGeom& g) {
    const int64_t nrows = (int64_t)g.n0 * g.n1;
    return (!is3d && nrows <= 4096) ? (int)nrows : row_blocks(g);
}

int diag_scale_launch(bool is3d, int form, const RowGeom& g, int P, int g0, double scale,
                      const double* b, double* x, const double* a0t, const double* b0t,
                      const double* a1, const double* b1, const double* a2, const double* b2,
                      double* partial, hipStream_t st, int* nblk_out) {
    // a2 / b2 here are the contiguous axis-2 diagonals (poms_op keeps them)
    const int64_t nrows = (int64_t)g.n0 * g.n1;
    if (!is3d && nrows <= 4096) {   // a row per workgroup (see diag_scale_kernel)
        if (nblk_out) *nblk_out = (int)nrows;
        if (form == FORM_SUM)
            hipLaunchKernelGGL((diag_scale_kernel<false, FORM_SUM, true>), dim3(nrows), dim3(256), 0, st, g, P, g0,
                               scale, b, x, a0t, b0t, a1, b1, a2, b2, partial);
        else
            hipLaunchKernelGGL((diag_scale_kernel<false, FORM_SINGLE, true>), dim3(nrows), dim3(256), 0, st, g, P,
                               g0, scale, b, x, a0t, b0t, a1, b1, a2, b2, partial);
        return 0;
    }
    const int nb = row_blocks(g);
    if (nblk_out) *nblk_out = nb;
#define POMS_DS(I3, F)                                                                          \
    hipLaunchKernelGGL((diag_scale_kernel<I3, F>), dim3(nb), dim3(256), 0, st, g, P, g0, scale, b, \
                       x, a0t, b0t, a1, b1, a2, b2, partial)
    if (is3d) {
        if (form == FORM_SUM) POMS_DS(true, FORM_SUM); else POMS_DS(true, FORM_SINGLE);
    } else {
        if (form == FORM_SUM) POMS_DS(false, FORM_SUM); else POMS_DS(false, FORM_SINGLE);
    }
#undef POMS_DS
    return 0;
}

int dense_matvec_launch(int n, const double* M, const double* x, double* y, hipStream_t st) {
    hipLaunchKernelGGL(dense_matvec_kernel, dim3((n + 3) / 4), dim3(256), 0, st, n, M, x, y);
    return 0;
}

int max_partials() { return kMaxPartials; }

}  // namespace poms
