// Knot-insertion restriction / prolongation as a sequence of 1D Kronecker
// axis passes (R = P^T with P = P0 (x) P1 (x) P2, sources/mg_jac.py:67-70).
//
// restrict pass:  out[a][J][b] = sum_i P[goff+i][J] * in[a][i][b]
// prolong  pass:  out[a][i][b] (+)= sum_J P[goff+i][J] * in[a][J][b]
//
// One thread per independent (a, b1, b2) line; the thread marches along the
// contracted axis with the NCM coarse values / accumulators in registers and
// wave-uniform (scalar) rows of P (P is stored fine-row-major, padded to NCM
// columns with zeros).  The dominant pass (axis 0 of the fine slab) streams the
// fine vector once: 8 B/DOF for restriction, 16 B/DOF for prolong-add.
// Coarse extents > 32 (multilevel hierarchies) use the banded gather kernels.
#include "transfer.hpp"

#include <algorithm>
#include <cstdlib>

namespace poms {

// Few lines (a 2D grid's passes: ~10^3 lines of ~10^3 points, or the coarse
// axis' ~10 lines) leave the one-thread-per-line march latency-bound: the
// contracted axis is then split in KS chunks (blockIdx.y), each thread writing its
// NCM partial sums to `part`, and restrict_sum_kernel adds the KS partials of each
// output in chunk order (deterministic).
template <int NCM>
__global__ void __launch_bounds__(256)
restrict_pass_kernel(const AxisPass ps, const double* __restrict__ Pm,
                     const double* __restrict__ in, double* __restrict__ out, double* __restrict__ part) {
    // Rows of P are staged through LDS, RB at a time, and read back as broadcasts; the
    // inputs of BT rows are loaded before any is used (round 6: per-row scalar loads of
    // P, each waited for, and one input load per wave in flight left the 515^3 axis-0
    // pass latency-bound).  The FMAs keep their order: the same bits.  (16 rows and
    // non-temporal loads, as the fused pass takes them: 249-251 -> 257-258 us; the
    // prolong-add with nt loads and stores 575-578 -> 634-638 us; not kept.)
    constexpr int BT = 8, RB = 64;
    __shared__ double sp[RB * NCM];
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const bool live = tid < nline;
    const int ks = gridDim.y, kc = (ps.nI + ks - 1) / ks;
    const int i_begin = blockIdx.y * kc, i_end = min(ps.nI, i_begin + kc);
    const int64_t ln = live ? tid : 0;
    const int64_t b2 = ln % ps.nB2;
    const int64_t t1 = ln / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double acc[NCM];
#pragma unroll
    for (int j = 0; j < NCM; ++j) acc[j] = 0.0;
    for (int c0 = i_begin; c0 < i_end; c0 += RB) {
        const int nr = min(RB, i_end - c0);
        __syncthreads();
        for (int e = threadIdx.x; e < nr * NCM; e += 256) sp[e] = Pm[(int64_t)(ps.goff + c0) * NCM + e];
        __syncthreads();
        if (!live) continue;
        for (int r0 = 0; r0 < nr; r0 += BT) {
            double v[BT];
#pragma unroll
            for (int u = 0; u < BT; ++u) v[u] = (r0 + u < nr) ? src[(int64_t)(c0 + r0 + u) * ps.in_si] : 0.0;
#pragma unroll
            for (int u = 0; u < BT; ++u) {
                if (r0 + u >= nr) break;
#pragma unroll
                for (int j = 0; j < NCM; ++j) acc[j] = fma(sp[(r0 + u) * NCM + j], v[u], acc[j]);
            }
        }
    }
    if (!live) return;
    if (ks > 1) {   // partials [chunk][j][line]: coalesced over lines
#pragma unroll
        for (int j = 0; j < NCM; ++j)
            if (j < ps.nJ) part[((int64_t)blockIdx.y * NCM + j) * nline + tid] = acc[j];
        return;
    }
    double* dst = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2;
#pragma unroll
    for (int j = 0; j < NCM; ++j)
        if (j < ps.nJ) dst[(int64_t)j * ps.out_si] = acc[j];
}

__global__ void __launch_bounds__(256)
restrict_sum_kernel(const AxisPass ps, int ncm, int ks, const double* __restrict__ part, double* __restrict__ out) {
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= nline * ps.nJ) return;
    const int j = (int)(tid / nline);
    const int64_t line = tid - (int64_t)j * nline;
    double s = 0.0;
    int k = 0;
    for (; k + 8 <= ks; k += 8) {   // 8 loads in flight, added in chunk order
        double w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = part[((int64_t)(k + u) * ncm + j) * nline + line];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += w[u];
    }
    for (; k < ks; ++k) s += part[((int64_t)k * ncm + j) * nline + line];
    const int64_t b2 = line % ps.nB2;
    const int64_t t1 = line / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    out[ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)j * ps.out_si] = s;
}

template <int NCM>
__global__ void __launch_bounds__(256)
prolong_pass_kernel(const AxisPass ps, const double* __restrict__ Pm,
                    const double* __restrict__ in, double* __restrict__ out) {
    // P rows through LDS and BT rows per step, as restrict_pass_kernel (the accumulated
    // rows' loads are issued together, before the stores)
    constexpr int BT = 8, RB = 64;
    __shared__ double sp[RB * NCM];
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const bool live = tid < nline;
    const int64_t ln = live ? tid : 0;
    const int64_t b2 = ln % ps.nB2;
    const int64_t t1 = ln / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double cv[NCM];
#pragma unroll
    for (int j = 0; j < NCM; ++j) cv[j] = (live && j < ps.nJ) ? src[(int64_t)j * ps.in_si] : 0.0;
    double* dst = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2;
    // outputs are independent: few lines split the expanded axis over blockIdx.y
    const int ks = gridDim.y, kc = (ps.nI + ks - 1) / ks;
    const int i_begin = blockIdx.y * kc, i_end = min(ps.nI, i_begin + kc);
    for (int c0 = i_begin; c0 < i_end; c0 += RB) {
        const int nr = min(RB, i_end - c0);
        __syncthreads();
        for (int e = threadIdx.x; e < nr * NCM; e += 256) sp[e] = Pm[(int64_t)(ps.goff + c0) * NCM + e];
        __syncthreads();
        if (!live) continue;
        for (int r0 = 0; r0 < nr; r0 += BT) {
            double old[BT];
#pragma unroll
            for (int u = 0; u < BT; ++u)
                old[u] = (ps.accumulate && r0 + u < nr) ? dst[(int64_t)(c0 + r0 + u) * ps.out_si] : 0.0;
#pragma unroll
            for (int u = 0; u < BT; ++u) {
                if (r0 + u >= nr) break;
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < NCM; ++j) s = fma(sp[(r0 + u) * NCM + j], cv[j], s);
                dst[(int64_t)(c0 + r0 + u) * ps.out_si] = ps.accumulate ? old[u] + s : s;
            }
        }
    }
}

// Banded gather form for large coarse extents (multilevel hierarchies, where P
// is the dyadic knot-insertion matrix with a few non-zeros per row / column):
// one thread per OUTPUT element, the fastest index (b2) on consecutive lanes.
//   restrict: out[a][J][b] = sum_k Rb[J][k] in[a][ilo[J] + k - goff][b]  (local rows only)
//   prolong : out[a][i][b] (+)= sum_k Pb[goff+i][k] in[a][jlo[goff+i] + k][b]
__global__ void __launch_bounds__(256)
restrict_band_kernel(const AxisPass ps, const double* __restrict__ Rb, const int* __restrict__ ilo, int wR,
                     const double* __restrict__ in, double* __restrict__ out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nout = ps.nA * ps.nJ * ps.nB1 * ps.nB2;
    if (tid >= nout) return;
    const int64_t b2 = tid % ps.nB2;
    int64_t t = tid / ps.nB2;
    const int64_t b1 = t % ps.nB1;
    t /= ps.nB1;
    const int J = (int)(t % ps.nJ);
    const int64_t a = t / ps.nJ;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double s = 0.0;
    const int i0 = ilo[J] - ps.goff;
    for (int k = 0; k < wR; ++k) {
        const int i = i0 + k;
        if (i >= 0 && i < ps.nI) s = fma(Rb[(int64_t)J * wR + k], src[(int64_t)i * ps.in_si], s);
    }
    out[ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)J * ps.out_si] = s;
}

__global__ void __launch_bounds__(256)
prolong_band_kernel(const AxisPass ps, const double* __restrict__ Pb, const int* __restrict__ jlo, int wP,
                    const double* __restrict__ in, double* __restrict__ out) {
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nout = ps.nA * (int64_t)ps.nI * ps.nB1 * ps.nB2;
    if (tid >= nout) return;
    const int64_t b2 = tid % ps.nB2;
    int64_t t = tid / ps.nB2;
    const int64_t b1 = t % ps.nB1;
    t /= ps.nB1;
    const int i = (int)(t % ps.nI);
    const int64_t a = t / ps.nI;
    const double* src = in + ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    const int gi = ps.goff + i;
    const int j0 = jlo[gi];
    double s = 0.0;
    for (int k = 0; k < wP; ++k) {
        const int j = j0 + k;
        if (j < ps.nJ) s = fma(Pb[(int64_t)gi * wP + k], src[(int64_t)j * ps.in_si], s);
    }
    double* o = out + ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)i * ps.out_si;
    if (ps.accumulate) *o += s;
    else *o = s;
}

// ---- fused residual -> restriction (sources/mg_jac.py:93-94) ----------------------
// rc = R (b - A x) = R b - (R A) x with A = sum_t (x)_d F_{t,d}: every factor of R A
// is a (nf x nc) matrix G = F^T P (host, poms_transfer_set_operator), so R A x is
// sum-factorised like R itself and neither r = b - A x nor A x is ever stored.  One
// pass over axis d reads up to 3 inputs and forms up to 3 outputs
//     out[o][.. J ..] = sum_i sum_k M[o][k][goff + i][J] in[k][.. i ..]
// (rows padded to NCM columns with zeros; a null M[o][k] is no term).  The first pass
// streams x and b once: 16 B per fine DOF, against 24 (residual) + 8 (restriction).
// Every thread marches one line; the inputs of BT consecutive rows are loaded before
// any of them is used.  The (o, k) terms of a pass are a compile-time MASK (bit
// 3 o + k), and the workgroup stages the matrix rows of RB rows at a time into LDS,
// read back as broadcasts.  Measured at 515^3 (the three passes, round 6): scalar
// loads of the rows, each waited for before its FMAs, 1.52-1.55 ms; LDS-staged rows
// 0.69-0.70 ms; the same with two lines per thread (half the LDS reads per line, two
// waves per SIMD) 0.83 ms.  The residual + restriction pair it replaces: 0.92 ms.
constexpr int mask_np(int m) { int c = 0; for (int b = 0; b < 9; ++b) c += (m >> b) & 1; return c; }
constexpr int mask_bit(int m, int p) {   // bit of the p-th term
    for (int b = 0, c = 0; b < 9; ++b)
        if ((m >> b) & 1) { if (c == p) return b; ++c; }
    return 0;
}
constexpr int mask_no(int m) { int n = 0; for (int b = 0; b < 9; ++b) if ((m >> b) & 1) n = b / 3 + 1 > n ? b / 3 + 1 : n; return n; }
constexpr int mask_ni(int m) { int n = 0; for (int b = 0; b < 9; ++b) if ((m >> b) & 1) n = b % 3 + 1 > n ? b % 3 + 1 : n; return n; }

template <int NCM, int MASK, int BT = 4, int RB = 32, bool NT = false>
__global__ void __launch_bounds__(256)
mrestrict_kernel(const MultiPass mp, double* __restrict__ part) {
    constexpr int NP = mask_np(MASK), NO = mask_no(MASK), NI = mask_ni(MASK);
    __shared__ double smat[RB * NP * NCM];
    const AxisPass& ps = mp.ps;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const bool live = tid < nline;   // (every thread stages rows and takes the barriers)
    const int ks = gridDim.y, kc = (ps.nI + ks - 1) / ks;
    const int i_begin = blockIdx.y * kc, i_end = min(ps.nI, i_begin + kc);
    const int64_t ln = live ? tid : 0;
    const int64_t b2 = ln % ps.nB2;
    const int64_t t1 = ln / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    const int64_t ioff = ps.in_base + a * ps.in_sa + b1 * ps.in_sb1 + b2 * ps.in_sb2;
    double acc[NO][NCM];
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
        for (int j = 0; j < NCM; ++j) acc[o][j] = 0.0;
    for (int c0 = i_begin; c0 < i_end; c0 += RB) {
        const int nr = min(RB, i_end - c0);
        __syncthreads();   // the previous stage's rows are read
        for (int e = threadIdx.x; e < nr * NP * NCM; e += 256) {
            const int r = e / (NP * NCM), q = e - r * (NP * NCM), pp = q / NCM, j = q - pp * NCM;
            const double* m = nullptr;
#pragma unroll
            for (int t = 0; t < NP; ++t)
                if (t == pp) m = mp.m[mask_bit(MASK, t) / 3][mask_bit(MASK, t) % 3];
            smat[e] = m[(int64_t)(ps.goff + c0 + r) * NCM + j];
        }
        __syncthreads();
        if (!live) continue;
        for (int r0 = 0; r0 < nr; r0 += BT) {
            double v[BT][NI];
#pragma unroll
            for (int u = 0; u < BT; ++u)
#pragma unroll
                for (int k = 0; k < NI; ++k)
                    v[u][k] = (r0 + u < nr) ? (NT ? __builtin_nontemporal_load(mp.in[k] + ioff + (int64_t)(c0 + r0 + u) * ps.in_si)
                                                  : mp.in[k][ioff + (int64_t)(c0 + r0 + u) * ps.in_si]) : 0.0;
#pragma unroll
            for (int u = 0; u < BT; ++u) {
                if (r0 + u >= nr) break;
                const double* sm = smat + (r0 + u) * NP * NCM;
#pragma unroll
                for (int t = 0; t < NP; ++t) {
                    const int o = mask_bit(MASK, t) / 3, k = mask_bit(MASK, t) % 3;
#pragma unroll
                    for (int j = 0; j < NCM; ++j) acc[o][j] = fma(sm[t * NCM + j], v[u][k], acc[o][j]);
                }
            }
        }
    }
    if (!live) return;
    if (ks > 1) {   // partials [chunk][o][j][line]: coalesced over lines
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
            for (int j = 0; j < NCM; ++j)
                if (j < ps.nJ) part[(((int64_t)blockIdx.y * NO + o) * NCM + j) * nline + tid] = acc[o][j];
        return;
    }
    const int64_t doff = ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2;
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
        for (int j = 0; j < NCM; ++j)
            if (j < ps.nJ) mp.out[o][doff + (int64_t)j * ps.out_si] = acc[o][j];
}

// Sum of the ks chunk partials of every output, in chunk order (deterministic); the
// loads of 8 chunks are issued before they are added.
__global__ void __launch_bounds__(256)
mrestrict_sum_kernel(const MultiPass mp, int ncm, int no, int ks, const double* __restrict__ part) {
    const AxisPass& ps = mp.ps;
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (tid >= nline * ps.nJ * no) return;
    const int64_t line = tid % nline;
    const int oj = (int)(tid / nline);
    const int j = oj % ps.nJ, o = oj / ps.nJ;
    const double* pp = part + ((int64_t)o * ncm + j) * nline + line;
    const int64_t cs = (int64_t)no * ncm * nline;   // one chunk's partials
    double s = 0.0;
    int k = 0;
    for (; k + 8 <= ks; k += 8) {
        double w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) w[u] = pp[(int64_t)(k + u) * cs];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += w[u];
    }
    for (; k < ks; ++k) s += pp[(int64_t)k * cs];
    const int64_t b2 = line % ps.nB2;
    const int64_t t1 = line / ps.nB2;
    const int64_t b1 = t1 % ps.nB1;
    const int64_t a = t1 / ps.nB1;
    mp.out[o][ps.out_base + a * ps.out_sa + b1 * ps.out_sb1 + b2 * ps.out_sb2 + (int64_t)j * ps.out_si] = s;
}

// chunks of a multi-output pass: at least 32768 threads where the lines are few, the
// chunk partials (no x ncm per line and chunk) kept below the pass's input reads
static int mrestrict_split(int64_t nline, int nI, int ni, int no, int ncm) {
    if (nline >= 32768 || nI < 64) return 1;
    const int64_t want = (32768 + nline - 1) / nline;
    const int64_t cap = std::max<int64_t>(1, (int64_t)nI * ni / ((int64_t)no * ncm));
    return (int)std::max<int64_t>(1, std::min<int64_t>({want, cap, (int64_t)nI / 16, 256}));
}

int64_t mrestrict_scratch(const MultiPass& mp, int ncm) {   // doubles of partials a pass needs
    const int64_t nline = mp.ps.nA * mp.ps.nB1 * mp.ps.nB2;
    const int ks = mrestrict_split(nline, mp.ps.nI, mp.ni, mp.no, ncm);
    return ks > 1 ? ks * (int64_t)mp.no * ncm * nline : 0;
}

// the term patterns poms_resid_restrict issues (bit 3 o + k): FORM_SUM axis 0 (and
// 2D's first pass), axis 1, last pass; FORM_SINGLE the same three.  The first passes
// (x and b streamed once) load 16 rows per batch with non-temporal loads and stage 64
// rows: 515^3, interleaved A/B on one box (profiles/r06/resid_restrict/ab_axis0.txt):
// 4 / 32 / plain 705-710 us, 8 / 64 / nt 633-641, 8 / 128 / nt 632-633, 16 / 64 / nt
// 622-623, 16 / 128 / nt 623-628.
constexpr int kMasks[6] = {(1 << 1) | (1 << 3) | (1 << 6), 1 | (1 << 4) | (1 << 5) | (1 << 8), 7,
                           (1 << 1) | (1 << 3), 1 | (1 << 4), 3};

template <int NCM>
static int mrestrict_go(int mask, const MultiPass& mp, dim3 grid, double* part, hipStream_t st) {
    switch (mask) {
        case kMasks[0]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[0], 16, 64, true>), grid, dim3(256), 0, st, mp, part); return 0;
        case kMasks[1]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[1]>), grid, dim3(256), 0, st, mp, part); return 0;
        case kMasks[2]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[2]>), grid, dim3(256), 0, st, mp, part); return 0;
        case kMasks[3]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[3], 16, 64, true>), grid, dim3(256), 0, st, mp, part); return 0;
        case kMasks[4]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[4]>), grid, dim3(256), 0, st, mp, part); return 0;
        case kMasks[5]: hipLaunchKernelGGL((mrestrict_kernel<NCM, kMasks[5]>), grid, dim3(256), 0, st, mp, part); return 0;
        default: set_error("resid_restrict: unsupported term pattern"); return 1;
    }
}

int mrestrict_launch(int ncm, const MultiPass& mp, double* part, hipStream_t st) {
    const int64_t nline = mp.ps.nA * mp.ps.nB1 * mp.ps.nB2;
    const int nb = (int)((nline + 255) / 256);
    if (nb == 0) return 0;
    if (mp.no < 1 || mp.no > 3 || mp.ni < 1 || mp.ni > 3) { set_error("resid_restrict: 1..3 inputs / outputs"); return 1; }
    int mask = 0;
    for (int o = 0; o < 3; ++o)
        for (int k = 0; k < 3; ++k)
            if (mp.m[o][k]) mask |= 1 << (3 * o + k);
    if (mask_no(mask) != mp.no || mask_ni(mask) != mp.ni) { set_error("resid_restrict: term pattern vs counts"); return 1; }
    const int ks = part ? mrestrict_split(nline, mp.ps.nI, mp.ni, mp.no, ncm) : 1;
    const dim3 grid(nb, ks);
    double* pk = ks > 1 ? part : nullptr;
    int rc = 1;
    switch (ncm) {
        case 8: rc = mrestrict_go<8>(mask, mp, grid, pk, st); break;
        case 12: rc = mrestrict_go<12>(mask, mp, grid, pk, st); break;
        case 16: rc = mrestrict_go<16>(mask, mp, grid, pk, st); break;
        case 32: rc = mrestrict_go<32>(mask, mp, grid, pk, st); break;
        default: set_error("resid_restrict: coarse extent must be <= 32"); return 1;
    }
    if (rc) return 1;
    if (ks > 1) {
        const int64_t nsum = nline * mp.ps.nJ * mp.no;
        hipLaunchKernelGGL(mrestrict_sum_kernel, dim3((unsigned)((nsum + 255) / 256)), dim3(256), 0, st, mp, ncm,
                           mp.no, ks, part);
    }
    return 0;
}

int transfer_band_launch(bool restrict_dir, const AxisPass& ps, const double* band, const int* lo, int w,
                         const double* in, double* out, hipStream_t st) {
    const int64_t nout = ps.nA * (int64_t)(restrict_dir ? ps.nJ : ps.nI) * ps.nB1 * ps.nB2;
    const int64_t nb = (nout + 255) / 256;
    if (nb == 0) return 0;
    if (restrict_dir)
        hipLaunchKernelGGL(restrict_band_kernel, dim3((unsigned)nb), dim3(256), 0, st, ps, band, lo, w, in, out);
    else
        hipLaunchKernelGGL(prolong_band_kernel, dim3((unsigned)nb), dim3(256), 0, st, ps, band, lo, w, in, out);
    return 0;
}

// chunks of the contracted / expanded axis: enough threads for the GPU when the
// lines are few, chunks of at least 16 points
static int transfer_split(int64_t nline, int nI) {
    if (nline >= 32768 || nI < 64) return 1;
    const int64_t want = (65536 + nline - 1) / nline;
    return (int)std::max<int64_t>(1, std::min<int64_t>({want, (int64_t)nI / 16, 256}));
}

int transfer_split_scratch(int ncm, const AxisPass& ps) {   // doubles of partials a restrict pass needs
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int ks = transfer_split(nline, ps.nI);
    return ks > 1 ? (int)(ks * (int64_t)ncm * nline) : 0;
}

int transfer_pass_launch(bool restrict_dir, int ncm, const AxisPass& ps, const double* Pm,
                         const double* in, double* out, hipStream_t st, double* part) {
    const int64_t nline = ps.nA * ps.nB1 * ps.nB2;
    const int nb = (int)((nline + 255) / 256);
    if (nb == 0) return 0;
    int ks = transfer_split(nline, ps.nI);
    if (restrict_dir && ks > 1 && part == nullptr) ks = 1;
    const dim3 grid(nb, ks);
    if (ncm == 16) {
        if (restrict_dir)
            hipLaunchKernelGGL(restrict_pass_kernel<16>, grid, dim3(256), 0, st, ps, Pm, in, out, part);
        else
            hipLaunchKernelGGL(prolong_pass_kernel<16>, grid, dim3(256), 0, st, ps, Pm, in, out);
    } else if (ncm == 32) {
        if (restrict_dir)
            hipLaunchKernelGGL(restrict_pass_kernel<32>, grid, dim3(256), 0, st, ps, Pm, in, out, part);
        else
            hipLaunchKernelGGL(prolong_pass_kernel<32>, grid, dim3(256), 0, st, ps, Pm, in, out);
    } else {
        set_error("transfer: coarse extent must be <= 32");
        return 1;
    }
    if (restrict_dir && ks > 1) {
        const int64_t nsum = nline * ps.nJ;
        hipLaunchKernelGGL(restrict_sum_kernel, dim3((unsigned)((nsum + 255) / 256)), dim3(256), 0, st, ps, ncm, ks,
                           part, out);
    }
    return 0;
}

}  // namespace poms
