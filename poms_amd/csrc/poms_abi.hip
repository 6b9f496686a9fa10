// extern "C" boundary of libpoms_hip.so (declared in include/poms_hip.h).
#include "common.hpp"
#include "transfer.hpp"
#include "split_hooks.hpp"
#include "../../include/poms_hip.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace poms {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

int kron_launch(int pmax, bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                double omega, hipStream_t st);
int kron_v3_launch(int variant, int pmax, bool is3d, int form, int epi, const KronPtrs& p,
                   const KronGeom& g, const ToepConst& tc, double omega, hipStream_t st);
int kron_v4_launch(int pmax, bool is3d, int form, int epi, const KronPtrs& p, const KronGeom& g,
                   const ToepConst& tc, double omega, hipStream_t st, int diag_mode);
int kron_v5_launch(int pmax, int epi, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, int H,
                   double omega, hipStream_t st, int diag_mode);
void kron_v5_tile(int pmax, bool aligned, int* H, int* TO);
int kron_v5_rows(int pmax, int epi, int same12);
int kron_v5_stamps(unsigned long long* host, int64_t n);
int kron_v5_set_sched(int mode);
void kron_v5_set_launch_events(hipEvent_t e0, hipEvent_t e1);
bool kron_v5_launch_events_used();
int kron_tile_rows();
int kron_v3_rows_2d();
int kron2d_j2_rows();
int kron2d_j2_cols(int pmax);
int kron2d_j2_launch(int pmax, int form, const KronPtrs& p, const KronGeom& g, const ToepConst& tc, double omega,
                     hipStream_t st, bool from_zero, double* part0);
int kron2d_j2_rows_default();
int kron_tile_cols();
int vec_launch(int op, const RowGeom& g, double a, double b, const double* x, const double* y,
               double* z, double* w, const double* q, double* partial, hipStream_t st,
               int* nblk_out, const double* ab = nullptr);
int reduce_launch(const double* partial, int count, double* out, hipStream_t st, int accumulate = 0);
int reduce_wide_launch(const double* partial, int count, double* out, hipStream_t st, int accumulate = 0);
int vec_flat_launch(int op, int64_t count, double a, double b, const double* x, const double* y,
                    double* z, double* w, const double* q, double* partial, hipStream_t st,
                    int* nblk_out, const double* ab = nullptr, const AlphaFold* af = nullptr);
int zero_ghosts_launch(const RowGeom& g, double* z, hipStream_t st);
int diag_scale_blocks(bool is3d, const RowGeom& g);
int diag_scale_launch(bool is3d, int form, const RowGeom& g, int P, int g0, double scale,
                      const double* b, double* x, const double* a0t, const double* b0t,
                      const double* a1, const double* b1, const double* a2, const double* b2,
                      double* partial, hipStream_t st, int* nblk_out);
int dense_matvec_launch(int n, const double* M, const double* x, double* y, hipStream_t st);
int assemble_launch(const AssembleAxis* ax, int g0, int nl0, const double* a_q, const double* c_q, double mass_coef,
                    double* coef, hipStream_t st);
int stencil_to_spl_launch(const StencilGeom& g, const double* coef, double* out, hipStream_t st);
int stencil_launch(int epi, const StencilGeom& g, const double* coef, const double* x, double* y,
                   const double* b, double omega, double* partial, double* partial2, int max_blocks,
                   hipStream_t st, int* nblk_out);
int transfer_pass_launch(bool restrict_dir, int ncm, const AxisPass& ps, const double* Pm,
                         const double* in, double* out, hipStream_t st, double* part);
int transfer_split_scratch(int ncm, const AxisPass& ps);
int transfer_band_launch(bool restrict_dir, const AxisPass& ps, const double* band, const int* lo, int w,
                         const double* in, double* out, hipStream_t st);

int ksolve_strided_launch(const LineGeom& g, const BandLU& f, const double* in, double* out, hipStream_t st);
int ksolve_rows_launch(const RowLines& g, const BandLU& f, const double* in, double* out, hipStream_t st);
int band_lu(int64_t n, int kl, int ku, double* ab, int64_t ldab, int* ipiv);
void band_lu_tables(int64_t n, int kl, int ku, const double* ab, int64_t ldab, const int* ipiv,
                    std::vector<double>& L, std::vector<double>& U, std::vector<int>& piv);

enum { V_AXPBY = 0, V_SCALE = 1, V_FILL = 2, V_DOT = 3, V_PCGUPD = 4, V_RUPD = 5, V_XPUPD = 6, V_SCALEDOT = 7 };   // (vec_ops.hip's VecOp)

}  // namespace poms

using namespace poms;

struct poms_ctx {
    int device = 0;
    double* scratch = nullptr;  // reduction partials
};

// A launch-timing event; under stream capture it becomes an event-record node of the
// graph (every replay records it again), not a capture-ordering marker.
static hipError_t timing_record(hipEvent_t e, hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    const hipError_t q = hipStreamIsCapturing(s, &cs);
    if (q != hipSuccess) return q;
    if (cs != hipStreamCaptureStatusActive) return hipEventRecord(e, s);
    // an event-record node after the capture's current frontier, which it then replaces
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    hipError_t r = hipStreamGetCaptureInfo_v2(s, &cs, nullptr, &g, &deps, &nd);
    if (r != hipSuccess) return r;
    hipGraphNode_t node = nullptr;
    r = hipGraphAddEventRecordNode(&node, g, deps, nd, e);
    if (r != hipSuccess) return r;
    return hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies);
}

// Host-reduced partials of one speculative launch: blocks n at offset off of the pinned
// region, kind bit 0 norm / bit 1 dot, into value index vi (+1 when both).
struct SpecPart { int64_t off; int n; int kind; int vi; };

struct poms_op {
    poms_ctx* ctx = nullptr;
    // where a launch writes its per-block partials: norms at scratch + part_off, dots
    // at scratch + (dot_base < 0 ? nblk : dot_base) + part_off (op_run_split puts two
    // launches' partials side by side and reduces them once)
    int64_t part_off = 0, dot_base = -1;
    // op_run_split's interior launch: the communication stream's exchange and boundary
    // launch run beside it (the automatic chunking leaves them CUs, op_geom)
    bool split_interior = false;
    int ndim = 3, form = FORM_SUM, pmax = 1, chunk = 0, tout = 0;
    poms_layout L{};
    int64_t g0 = 0, n0g = 1;
    double *a0t = nullptr, *b0t = nullptr, *a1 = nullptr, *b1 = nullptr, *a2 = nullptr, *b2 = nullptr;
    int64_t last_partials = 0;
    double *dg2a = nullptr, *dg2b = nullptr;  // contiguous axis-2 band diagonals
    double* rdiag0 = nullptr;                  // 1/diag(A) per global plane (Toeplitz interior of axes 1, 2)
    int variant = 0;
    int last_variant = -1;    // the kernel variant the last operator launch ran (after per-call fall-backs)
    bool v2_ok = false;       // storage pads == pmax on every used axis (the Toeplitz kernels' precondition)
    bool ghost_corners = false;   // ghost edges / corners of axes 1 and 2 may be non-zero (a Cart block)
    ToepConst tc{};
    double* coef = nullptr;   // FORM_STENCIL: (2p+1)^d coefficient planes of the owned rows
    int sp[3]{};              // FORM_STENCIL: stencil half-widths per axis
    // native pcg loop (poms_pcg_jacobi): device scalars and the pinned host slots
    double* sv_dev = nullptr;
    double* sv_host = nullptr;
    // poms_pcg_jacobi, one rank: ring of pinned host slots the reduction kernels
    // write the host-read norms into.  sv_seq[i] = launch sequence number that armed
    // slot i (-1: never); every launch numbered below sv_done is known complete (a
    // value written by a later launch of the same stream has been read), so its slot
    // can be re-armed without a stale write landing after the sentinel.
    static constexpr int kSvRing = 48;
    int sv_next = 0;
    int64_t sv_seq_next = 0, sv_done = 0;
    int64_t sv_seq[kSvRing];
    // ... and per slot a region of kSvPart doubles the operator launch writes its
    // per-block partial sums into (no reduction launch: the host adds them in the
    // reduction kernel's order when it reads the slot).  sv_npart[i] = blocks of the
    // launch that last used region i (0: none pending), sv_pkind[i] bit 0 norm
    // partials at [0, n), bit 1 dot partials after them.
    static constexpr int kSvPart = 4096;
    double* sv_part = nullptr;   // kSvRing x kSvPart, pinned, device-mapped, armed unset
    // poms_pcg_jacobi, speculative mode: the sweeps' per-block partials (pinned,
    // device-mapped; kSpecPart doubles), the device array of the other host-read sums,
    // and the backup of x0
    static constexpr int64_t kSpecPart = 1 << 19;
    static constexpr int kSpecVals = 4096;
    double* spec_part = nullptr;
    double* spec_dev = nullptr;
    double* spec_host = nullptr;    // kSpecVals, pinned
    double* la_buf = nullptr;   // the two-sweep lookahead's fourth preconditioner buffer (zero ghosts)
    double* la_raw = nullptr;   // its allocation: la_buf sits la_off doubles in, on the work vectors' 128-B phase
    int64_t la_off = -1;
    int64_t la_n = 0;
    double* spec_bak = nullptr;
    int64_t spec_bak_n = 0;
    struct SpecGraph {   // a captured speculative call (see pcg_speculative)
        uint64_t key[16] = {};
        hipGraphExec_t exec = nullptr;
        std::vector<SpecPart> parts;
        std::vector<int> chk, rr;
        int sn = 0, vrr0 = 0;
        int64_t use = 0;
    };
    static constexpr int kSpecGraphs = 4;
    SpecGraph spec_graphs[kSpecGraphs];
    int64_t spec_graph_clock = 0;
    uint64_t gen = 0;   // bumped by every setter that changes the launches a graph would capture
    int spec_graph_hits = 0, spec_graph_caps = 0;   // graphs stop when captures outnumber hits
    int spec_calls = 0, spec_repeats = 0;            // speculative calls, and those repeated step by step
    hipStream_t cap_stream = nullptr;                 // private non-blocking capture stream
    int sv_npart[kSvRing] = {};
    int sv_pkind[kSvRing] = {};
    // op_run: write the partials to part_dst instead of the scratch when they fit
    // in part_cap doubles (last_part_host says whether they went there)
    double* part_dst = nullptr;
    int64_t part_cap = 0;
    bool last_part_host = false;
    // launch timing (poms_op_timing): HIP events around every operator launch
    struct TimedLaunch { int epi; int64_t ndof; hipEvent_t e0, e1; };
    bool timing = false;
    int t_epi = -1, t_every = 1;   // record launches of this epilogue only (-1: all), every n-th
    int64_t t_seen = 0;
    std::vector<TimedLaunch> tl;
    size_t tl_used = 0;
};

static int resolve_variant(const poms_op* o, int epi);

// Largest row range [lo, hi) around the middle whose band rows equal one
// symmetric row (bitwise), for the pair (fa, fb) (fb may be null).
static void toeplitz_range(const double* fa, const double* fb, int64_t n, int P, int* lo, int* hi,
                           double* ta, double* tb) {
    const int W = 2 * P + 1;
    *lo = *hi = 0;
    for (int j = 0; j < 6; ++j) { ta[j] = 0.0; tb[j] = 0.0; }
    if (n < 1) return;
    const int64_t m = n / 2;
    auto sym = [&](const double* f) {
        if (!f) return true;
        for (int j = 1; j <= P; ++j)
            if (f[m * W + P + j] != f[m * W + P - j]) return false;
        return true;
    };
    if (!sym(fa) || !sym(fb)) return;
    auto same = [&](int64_t i) {
        for (int k = 0; k < W; ++k) {
            if (fa[i * W + k] != fa[m * W + k]) return false;
            if (fb && fb[i * W + k] != fb[m * W + k]) return false;
        }
        return true;
    };
    int64_t a = m, b = m + 1;
    while (a > 0 && same(a - 1)) --a;
    while (b < n && same(b)) ++b;
    *lo = (int)a;
    *hi = (int)b;
    for (int j = 0; j <= P; ++j) {
        ta[j] = fa[m * W + P + j];
        tb[j] = fb ? fb[m * W + P + j] : 0.0;
    }
}

struct poms_transfer {
    poms_ctx* ctx = nullptr;
    int ndim = 3, ncm = 16;
    poms_layout L{};
    int64_t g0 = 0;
    int64_t nf[3]{}, nc[3]{};
    double* Pm[3]{};
    // banded form (coarse extent > 32): rows of P (Pb, jlo, wP) and of P^T (Rb, ilo, wR)
    bool banded = false;
    double *Pb[3]{}, *Rb[3]{};
    int *jlo[3]{}, *ilo[3]{};
    int wP[3]{}, wR[3]{};
    double *t0 = nullptr, *t1 = nullptr;
    double* part = nullptr;   // split-axis restriction partials (few lines)
    int64_t part_n = 0;
    // fused residual -> restriction (poms_transfer_set_operator / poms_resid_restrict)
    int rform = -1;           // POMS_FORM_SUM / POMS_FORM_SINGLE; -1: no operator set
    int ncf = 0;              // columns of the fused passes' matrices (8, 12, 16, 32)
    double* Gf[6]{};          // F^T P per operator role (last axis negated), ncf columns
    double* Pf[3]{};          // P, ncf columns
    double* ru = nullptr;     // axis-0 outputs: 3 x [c0][n1][n2]
    double* rv = nullptr;     // axis-1 outputs: 3 x [c0][c1][n2]
    double* mpart = nullptr;  // chunk partials of the fused passes
    int64_t mpart_n = 0;
};

struct poms_ksolve {
    poms_ctx* ctx = nullptr;
    int ndim = 3;
    poms_layout L{};
    int64_t n0g = 1;
    int64_t ng[3]{1, 1, 1};     // global extent of every axis (the factor sizes)
    int info[3]{};
    int kl[3]{}, ku[3]{};
    std::vector<int> ipiv[3];   // absolute 0-based pivot rows (host copy, for callers)
    double *Ld[3]{}, *Ud[3]{};
    int* pivd[3]{};
    BandLU f[3]{};
};

static hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static bool layout_ok(const poms_layout* L) {
    if (!L) return false;
    for (int d = 0; d < 3; ++d)
        if (L->n[d] < 1 || L->pads[d] < 0) return false;
    return L->pitch == 0 || L->pitch >= L->n[2] + 2 * L->pads[2];
}

static RowGeom row_geom(const poms_layout* L) {
    RowGeom g;
    const int64_t c2 = L->pitch > 0 ? L->pitch : L->n[2] + 2 * L->pads[2];
    const int64_t c1 = L->n[1] + 2 * L->pads[1];
    g.s1 = c2;
    g.s0 = c1 * c2;
    g.n0 = (int)L->n[0];
    g.n1 = (int)L->n[1];
    g.n2 = (int)L->n[2];
    g.pd0 = (int)L->pads[0];
    g.pd1 = (int)L->pads[1];
    g.pd2 = (int)L->pads[2];
    return g;
}

static int upload(const double* host, size_t n, double** dev) {
    POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dev), std::max<size_t>(n, 1) * sizeof(double)));
    if (n) POMS_HIP_CHECK(hipMemcpy(*dev, host, n * sizeof(double), hipMemcpyHostToDevice));
    return 0;
}

extern "C" {

int poms_abi_version(void) { return POMS_ABI_VERSION; }

const char* poms_last_error(void) { return g_err.c_str(); }

int poms_device_count(int* count) {
    if (!count) { set_error("null count"); return 1; }
    POMS_HIP_CHECK(hipGetDeviceCount(count));
    return 0;
}

int poms_ctx_create(int device, poms_ctx** ctx) {
    if (!ctx) { set_error("null ctx out"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(device));
    auto* c = new poms_ctx();
    c->device = device;
    if (hipMalloc(reinterpret_cast<void**>(&c->scratch), kScratch * sizeof(double)) != hipSuccess) {
        delete c;
        set_error("hipMalloc scratch failed");
        return 1;
    }
    *ctx = c;
    return 0;
}

int poms_ctx_destroy(poms_ctx* ctx) {
    if (!ctx) return 0;
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    delete ctx;
    return 0;
}

int poms_synchronize(poms_ctx* ctx, void* stream) {
    (void)ctx;
    POMS_HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
    return 0;
}

int poms_op_create(poms_ctx* ctx, int ndim, const poms_layout* layout, int form, int pmax,
                   const double* const* f, int64_t g0, int64_t n0_global, poms_op** op) {
    if (!ctx || !op || !f) { set_error("poms_op_create: null argument"); return 1; }
    if (ndim < 1 || ndim > 3) { set_error("poms_op_create: ndim must be 1..3"); return 1; }
    if (pmax < 1 || pmax > 5) { set_error("poms_op_create: pmax must be 1..5"); return 1; }
    if (form != FORM_SUM && form != FORM_SINGLE) { set_error("poms_op_create: bad form"); return 1; }
    if (!layout_ok(layout)) { set_error("poms_op_create: bad layout"); return 1; }
    const bool is3d = ndim == 3;
    if (!is3d && (layout->n[0] != 1 || layout->pads[0] != 0)) {
        set_error("poms_op_create: 1D/2D layouts need n[0]=1, pads[0]=0");
        return 1;
    }
    for (int d = 0; d < 3; ++d)
        if (layout->pads[d] > pmax) { set_error("poms_op_create: storage pad exceeds pmax"); return 1; }
    if (is3d && (g0 < 0 || g0 + layout->n[0] > n0_global)) {
        set_error("poms_op_create: slab [g0, g0+n0) outside [0, n0_global)");
        return 1;
    }
    const bool sum = form == FORM_SUM;
    if (!f[2] || !f[4] || (sum && (!f[3] || !f[5])) || (is3d && (!f[0] || (sum && !f[1])))) {
        set_error("poms_op_create: missing factor array");
        return 1;
    }
    POMS_HIP_CHECK(hipSetDevice(ctx->device));
    const int W = 2 * pmax + 1;
    auto* o = new poms_op();
    o->ctx = ctx;
    o->ndim = ndim;
    o->form = form;
    o->pmax = pmax;
    o->L = *layout;
    o->g0 = is3d ? g0 : 0;
    o->n0g = is3d ? n0_global : 1;
    o->ghost_corners = (layout->flags & POMS_LAYOUT_GHOST_DATA) != 0;
    int rc = 0;
    if (is3d) {
        // Transposed (column) bands of the axis-0 factors, padded by pmax rows on
        // both sides: at[(j+P)*W + s] = F[j-P+s][2P-s].
        const int64_t nrow = n0_global + 2 * pmax;
        std::vector<double> ta(nrow * W, 0.0), tb(nrow * W, 0.0);
        for (int64_t j = -pmax; j < n0_global + pmax; ++j)
            for (int s = 0; s < W; ++s) {
                const int64_t i = j - pmax + s;
                if (i < 0 || i >= n0_global) continue;
                ta[(j + pmax) * W + s] = f[0][i * W + (2 * pmax - s)];
                if (sum) tb[(j + pmax) * W + s] = f[1][i * W + (2 * pmax - s)];
            }
        rc |= upload(ta.data(), ta.size(), &o->a0t);
        if (sum) rc |= upload(tb.data(), tb.size(), &o->b0t);
    }
    rc |= upload(f[2], (size_t)layout->n[1] * W, &o->a1);
    rc |= upload(f[4], (size_t)layout->n[2] * W, &o->a2);
    if (sum) {
        rc |= upload(f[3], (size_t)layout->n[1] * W, &o->b1);
        rc |= upload(f[5], (size_t)layout->n[2] * W, &o->b2);
    }
    {
        std::vector<double> da(layout->n[2]), db(layout->n[2], 0.0);
        for (int64_t c = 0; c < layout->n[2]; ++c) {
            da[c] = f[4][c * W + pmax];
            if (sum) db[c] = f[5][c * W + pmax];
        }
        rc |= upload(da.data(), da.size(), &o->dg2a);
        rc |= upload(db.data(), db.size(), &o->dg2b);
    }
    if (rc) { poms_op_destroy(o); return 1; }
    // v2 preconditions: storage pads == pmax on the used axes
    o->v2_ok = layout->pads[1] == pmax && layout->pads[2] == pmax && (!is3d || layout->pads[0] == pmax);
    if (is3d)
        toeplitz_range(f[0], sum ? f[1] : nullptr, n0_global, pmax, &o->tc.lo0, &o->tc.hi0, o->tc.t0a, o->tc.t0b);
    toeplitz_range(f[2], sum ? f[3] : nullptr, layout->n[1], pmax, &o->tc.lo1, &o->tc.hi1, o->tc.t1a, o->tc.t1b);
    toeplitz_range(f[4], sum ? f[5] : nullptr, layout->n[2], pmax, &o->tc.lo2, &o->tc.hi2, o->tc.t2a, o->tc.t2b);
    o->variant = o->v2_ok ? 8 : 0;
    // 1/diag(A) on each global plane for points in the Toeplitz interior of axes 1
    // and 2 (same expression as the kernels' per-point diagonal)
    if (o->tc.lo1 < o->tc.hi1 && o->tc.lo2 < o->tc.hi2) {
        const double d1a = o->tc.t1a[0], d1b = sum ? o->tc.t1b[0] : 0.0;
        const double d2a = o->tc.t2a[0], d2b = sum ? o->tc.t2b[0] : 0.0;
        const int64_t np = is3d ? n0_global : 1;
        std::vector<double> rd(np);
        for (int64_t i = 0; i < np; ++i) {
            double dg;
            if (is3d) {
                const double d0a = f[0][i * W + pmax], d0b = sum ? f[1][i * W + pmax] : 0.0;
                dg = sum ? d0a * (d1a * d2a) + d0b * (d1b * d2a + d1a * d2b) : d0a * (d1a * d2a);
            } else {
                dg = sum ? d1a * d2a + d1b * d2b : d1a * d2a;
            }
            rd[i] = dg != 0.0 ? 1.0 / dg : 0.0;
        }
        if (upload(rd.data(), rd.size(), &o->rdiag0)) { poms_op_destroy(o); return 1; }
        // the same value on every plane of the axis-0 Toeplitz interior (bitwise: those
        // rows equal the middle row)
        if (is3d && o->tc.lo0 < o->tc.hi0) o->tc.rdi = rd[(o->tc.lo0 + o->tc.hi0) / 2];
    }
    *op = o;
    return 0;
}

int poms_op_create_stencil(poms_ctx* ctx, int ndim, const poms_layout* layout, const double* data,
                           int64_t g0, int64_t n0_global, poms_op** op) {
    if (!ctx || !op || !data || !layout_ok(layout)) { set_error("poms_op_create_stencil: bad argument"); return 1; }
    if (ndim < 1 || ndim > 3) { set_error("poms_op_create_stencil: ndim 1..3"); return 1; }
    for (int d = 0; d < 3 - ndim; ++d)
        if (layout->n[d] != 1 || layout->pads[d] != 0) {
            set_error("poms_op_create_stencil: unused leading axes need n = 1, pads = 0");
            return 1;
        }
    const RowGeom r = row_geom(layout);
    const int p[3] = {r.pd0, r.pd1, r.pd2};
    const int w[3] = {2 * p[0] + 1, 2 * p[1] + 1, 2 * p[2] + 1};
    const int64_t W = (int64_t)w[0] * w[1] * w[2];
    const int64_t cst = (int64_t)r.n0 * r.n1 * r.n2;
    if (W * cst * 8 > ((int64_t)1 << 40)) { set_error("poms_op_create_stencil: coefficients too large"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(ctx->device));
    // spl layout: rows over the padded local extents, then the W offsets of each row
    const int64_t P1 = r.n1 + 2 * p[1], P2 = r.n2 + 2 * p[2];
    std::vector<double> soa((size_t)(W * cst));
    for (int64_t i0 = 0; i0 < r.n0; ++i0)
        for (int64_t i1 = 0; i1 < r.n1; ++i1)
            for (int64_t i2 = 0; i2 < r.n2; ++i2) {
                const int64_t row = ((i0 + p[0]) * P1 + (i1 + p[1])) * P2 + (i2 + p[2]);
                const int64_t lin = (i0 * r.n1 + i1) * r.n2 + i2;
                const double* src = data + row * W;
                for (int64_t k = 0; k < W; ++k) soa[(size_t)(k * cst + lin)] = src[k];
            }
    auto* o = new poms_op();
    o->ctx = ctx;
    o->ndim = ndim;
    o->form = FORM_STENCIL;
    o->pmax = std::max(p[0], std::max(p[1], p[2]));
    o->L = *layout;
    o->g0 = ndim == 3 ? g0 : 0;
    o->n0g = ndim == 3 ? n0_global : 1;
    for (int d = 0; d < 3; ++d) o->sp[d] = p[d];
    if (upload(soa.data(), soa.size(), &o->coef)) { poms_op_destroy(o); return 1; }
    *op = o;
    return 0;
}

// On-device assembly of -div(a grad u) + c u into a FORM_STENCIL operator.
int poms_op_assemble_stencil(poms_ctx* ctx, int ndim, const poms_layout* layout, const int* nel, const int* nq,
                             const int* p, const int* const* first, const int* const* es, const int* const* ee,
                             const double* const* basis, const double* const* weights, const int64_t* nglob,
                             const double* a_q, const double* c_q, double mass_coef, int64_t g0, poms_op** op) {
    if (!ctx || !op || !layout_ok(layout) || !nel || !nq || !p || !first || !es || !ee || !basis || !weights || !nglob) {
        set_error("poms_op_assemble_stencil: bad argument");
        return 1;
    }
    if (ndim < 1 || ndim > 3) { set_error("poms_op_assemble_stencil: ndim 1..3"); return 1; }
    const int d0 = 3 - ndim;
    for (int d = 0; d < d0; ++d)
        if (layout->n[d] != 1 || layout->pads[d] != 0) {
            set_error("poms_op_assemble_stencil: unused leading axes need n = 1, pads = 0");
            return 1;
        }
    for (int d = d0; d < 3; ++d) {
        if (p[d] != layout->pads[d] || nel[d] < 1 || nq[d] < 1 || !first[d] || !es[d] || !ee[d] || !basis[d] ||
            !weights[d]) {
            set_error("poms_op_assemble_stencil: axis " + std::to_string(d) + " (degree must equal the pad)");
            return 1;
        }
        if (d > 0 && nglob[d] != layout->n[d]) { set_error("poms_op_assemble_stencil: only axis 0 may be sliced"); return 1; }
    }
    if (ndim == 3 && (g0 < 0 || g0 + layout->n[0] > nglob[0])) { set_error("poms_op_assemble_stencil: bad slab"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(ctx->device));
    const RowGeom r = row_geom(layout);
    const int64_t W = (int64_t)(2 * r.pd0 + 1) * (2 * r.pd1 + 1) * (2 * r.pd2 + 1);
    const int64_t cst = (int64_t)r.n0 * r.n1 * r.n2;
    auto* o = new poms_op();
    o->ctx = ctx;
    o->ndim = ndim;
    o->form = FORM_STENCIL;
    o->pmax = std::max(r.pd0, std::max(r.pd1, r.pd2));
    o->L = *layout;
    o->g0 = ndim == 3 ? g0 : 0;
    o->n0g = ndim == 3 ? nglob[0] : 1;
    o->sp[0] = r.pd0; o->sp[1] = r.pd1; o->sp[2] = r.pd2;
    std::vector<void*> tmp;
    auto up_i = [&](const int* h, int64_t n) -> const int* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<int64_t>(n, 1) * sizeof(int)) != hipSuccess) return nullptr;
        tmp.push_back(d);
        if (hipMemcpy(d, h, n * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return static_cast<const int*>(d);
    };
    auto up_d = [&](const double* h, int64_t n) -> const double* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<int64_t>(n, 1) * sizeof(double)) != hipSuccess) return nullptr;
        tmp.push_back(d);
        if (hipMemcpy(d, h, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return static_cast<const double*>(d);
    };
    static const int zero_i = 0;
    static const double unit_b[2] = {1.0, 0.0}, unit_w = 1.0;
    AssembleAxis ax[3];
    int rc = 0;
    for (int d = 0; d < 3 && !rc; ++d) {
        const bool used = d >= d0;
        const int ne = used ? nel[d] : 1, q = used ? nq[d] : 1, pp = used ? p[d] : 0;
        const int64_t n = used ? nglob[d] : 1;
        ax[d].first = up_i(used ? first[d] : &zero_i, ne);
        ax[d].es = up_i(used ? es[d] : &zero_i, n);
        ax[d].ee = up_i(used ? ee[d] : &zero_i, n);
        ax[d].basis = up_d(used ? basis[d] : unit_b, (int64_t)ne * q * (pp + 1) * 2);
        ax[d].w = up_d(used ? weights[d] : &unit_w, (int64_t)ne * q);
        ax[d].nel = ne; ax[d].nq = q; ax[d].p = pp; ax[d].n = (int)n;
        if (!ax[d].first || !ax[d].es || !ax[d].ee || !ax[d].basis || !ax[d].w) rc = 1;
    }
    if (!rc && hipMalloc(reinterpret_cast<void**>(&o->coef), std::max<int64_t>(W * cst, 1) * sizeof(double)) != hipSuccess)
        rc = 1;
    if (!rc) {
        assemble_launch(ax, (int)o->g0, r.n0, a_q, c_q, mass_coef, o->coef, nullptr);
        if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = 1;
    }
    for (void* d : tmp) (void)hipFree(d);
    if (rc) {
        set_error("poms_op_assemble_stencil: allocation, upload or launch failed");
        poms_op_destroy(o);
        return 1;
    }
    *op = o;
    return 0;
}

int poms_op_stencil_data(poms_op* o, double* data_host) {
    if (!o || !data_host || o->form != FORM_STENCIL) { set_error("poms_op_stencil_data: needs a general-stencil operator"); return 1; }
    const RowGeom r = row_geom(&o->L);
    StencilGeom g{r.s0, r.s1, r.n0, r.n1, r.n2, r.pd0, r.pd1, r.pd2, o->sp[0], o->sp[1], o->sp[2],
                  2 * o->sp[0] + 1, 2 * o->sp[1] + 1, 2 * o->sp[2] + 1, (int64_t)r.n0 * r.n1 * r.n2, 0, 0, 0, 0};
    const int64_t W = (int64_t)g.w0 * g.w1 * g.w2;
    const int64_t rows = (int64_t)(r.n0 + 2 * o->sp[0]) * (r.n1 + 2 * o->sp[1]) * (r.n2 + 2 * o->sp[2]);
    double* d = nullptr;
    POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&d), rows * W * sizeof(double)));
    int rc = 0;
    if (hipMemset(d, 0, rows * W * sizeof(double)) != hipSuccess) rc = 1;
    if (!rc) stencil_to_spl_launch(g, o->coef, d, nullptr);
    if (!rc && (hipGetLastError() != hipSuccess ||
                hipMemcpy(data_host, d, rows * W * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess))
        rc = 1;
    (void)hipFree(d);
    if (rc) { set_error("poms_op_stencil_data: copy failed"); return 1; }
    return 0;
}

int poms_op_destroy(poms_op* o) {
    if (!o) return 0;
    for (double* p : {o->a0t, o->b0t, o->a1, o->b1, o->a2, o->b2, o->dg2a, o->dg2b, o->rdiag0, o->coef, o->sv_dev,
                      o->spec_dev, o->spec_bak, o->la_raw})
        if (p) (void)hipFree(p);
    for (double* p : {o->sv_host, o->sv_part, o->spec_part, o->spec_host})
        if (p) (void)hipHostFree(p);
    for (auto& g : o->spec_graphs)
        if (g.exec) (void)hipGraphExecDestroy(g.exec);
    if (o->cap_stream) (void)hipStreamDestroy(o->cap_stream);
    for (auto& t : o->tl) {
        (void)hipEventDestroy(t.e0);
        (void)hipEventDestroy(t.e1);
    }
    delete o;
    return 0;
}

int poms_op_set_variant(poms_op* op, int variant) {
    // 90/91, 92-100, 101-113: diagnostic / tuning builds of v3, v4, v5 (110-112: v5
    // two sweeps from zero without sums / x1 scaling, timing only; 113: the Jacobi
    // sweep streaming the x rows no other tile reads)
    // (11, v7, was removed in round 6: an experimental kernel slower than v5)
    const bool known = variant == 0 || variant == 4 || (variant >= 7 && variant <= 10) ||
                       (variant >= 90 && variant <= 114);
    if (!op || !known) {
        set_error("poms_op_set_variant: bad argument (0, 4, 7, 8, 9, 10; 90-114 diagnostic)");
        return 1;
    }
    if (variant > 0 && !op->v2_ok) { set_error("poms_op_set_variant: variant needs pads == pmax"); return 1; }
    op->variant = variant;
    ++op->gen;
    return 0;
}

int poms_diag_v5_stamps(uint64_t* host_out, int64_t n) {
    if (!host_out) { set_error("poms_diag_v5_stamps: null argument"); return 1; }
    return kron_v5_stamps(reinterpret_cast<unsigned long long*>(host_out), n);
}

int poms_diag_v5_sched(int mode) { return kron_v5_set_sched(mode); }

int poms_variant_built(int variant) {
    return (variant == 0 || variant == 4 || (variant >= 7 && variant <= 10) || (variant >= 90 && variant <= 114)) ? 1 : 0;
}

int poms_op_kernel_variant(poms_op* op, int epilogue, int* variant) {
    if (!op || !variant || epilogue < EPI_APPLY || epilogue > EPI_APPLYDOT) {
        set_error("poms_op_kernel_variant: bad argument");
        return 1;
    }
    *variant = resolve_variant(op, epilogue);
    return 0;
}

int poms_op_last_variant(poms_op* op, int* variant) {
    if (!op || !variant) { set_error("poms_op_last_variant: null argument"); return 1; }
    *variant = op->last_variant;
    return 0;
}

int poms_op_spec_stats(poms_op* op, int* stats) {
    if (!op || !stats) { set_error("poms_op_spec_stats: null argument"); return 1; }
    stats[0] = op->spec_calls;
    stats[1] = op->spec_repeats;
    stats[2] = op->spec_graph_caps;
    stats[3] = op->spec_graph_hits;
    return 0;
}

int poms_op_get_variant(poms_op* op, int* variant) {
    if (!op || !variant) { set_error("poms_op_get_variant: null argument"); return 1; }
    *variant = op->variant;
    return 0;
}

int poms_op_set_tile_cols(poms_op* op, int cols) {
    if (!op || cols < 0 || cols > 64 - 2 * op->pmax) { set_error("poms_op_set_tile_cols: bad argument"); return 1; }
    op->tout = cols;
    ++op->gen;
    return 0;
}

int poms_op_set_chunk(poms_op* op, int chunk) {
    if (!op || chunk < 0) { set_error("poms_op_set_chunk: bad argument"); return 1; }
    op->chunk = chunk;
    ++op->gen;
    return 0;
}

// Axis-0 chunk length.  A workgroup streams `chunk` planes plus 2p halo planes, so
// long chunks save re-reads but leave a ragged last round of workgroups on the
// 256 CUs (512 resident workgroups at p <= 3).  Cost of nc chunks ~ rounds(nc) *
// (chunk + 2p), the partial last round weighted 5x its fill (fit to the chunk sweeps
// in profiles/r01/chunks/*.log; picks 103 at 515^3 p=3, 43 at 258^3 p=2).  For
// p >= 4 the kernels are VALU-bound and want >= 3 workgroups per CU instead.
static int auto_chunk(int nz, int tiles, int p, double slots = 512.0) {
    if (nz <= 0) return 1;
    tiles = std::max(tiles, 1);
    if (p >= 4 && slots > 256.0) {
        const int nc = std::max(1, std::min(nz / 8, (768 + tiles - 1) / tiles));
        return (nz + nc - 1) / nc;
    }
    double best = 1e300;
    int best_chunk = nz;
    for (int nc = 1; nc <= std::max(1, nz / 8); ++nc) {
        const int ch = (nz + nc - 1) / nc;
        const double r = (double)nc * tiles / slots;
        const double fr = std::floor(r);
        const double rounds = r > 1.0 ? fr + std::min(1.0, (r - fr) * 5.0) : 1.0;
        const double cost = rounds * (ch + 2 * p);
        if (cost < best - 1e-9) { best = cost; best_chunk = ch; }
    }
    return best_chunk;
}

// v5 (variant 10) runs 3D FORM_SUM operators, p <= 3, pads == pmax, arrays < 2 GiB.
// At odd p its x-row DMA pairs straddle storage column 0, and the pair holding
// column 0 of storage row 0 (the corner ghost of each plane) fails the buffer range
// check: zero, as the ghost always is unless axes 1 and 2 both have a lower
// neighbour -- then (ghost_corners) the operator runs v3.
static bool v5_ok(const poms_op* o) {
    const int64_t bytes = (int64_t)(o->L.n[0] + 2 * o->L.pads[0]) * row_geom(&o->L).s0 * 8;
    return o->ndim == 3 && o->form == FORM_SUM && o->v2_ok && o->pmax <= 5 && bytes < 0x7ffffff0LL &&
           !(o->ghost_corners && (o->pmax & 1));
}

// v5 tiles are line-aligned when the row pitch is a multiple of 16 doubles and
// interior column 0 of x starts a 128-B line
static bool v5_aligned(const poms_op* o, const double* x) {
    const int64_t pitch = row_geom(&o->L).s1;
    return pitch % 16 == 0 && (reinterpret_cast<uintptr_t>(x + o->L.pads[2]) & 127) == 0;
}

static bool same_toeplitz12(const poms_op* o);

static int op_geom(poms_op* o, int64_t zb, int64_t ze, KronGeom& g, int v = -1, int v5_to = 0,
                   int64_t zb2 = 0, int64_t ze2 = 0, int epi = EPI_APPLY) {
    if (v < 0) v = o->variant;
    const bool is3d = o->ndim == 3;
    const RowGeom r = row_geom(&o->L);
    g.s0 = r.s0;
    g.s1 = r.s1;
    g.n0 = r.n0; g.n1 = r.n1; g.n2 = r.n2;
    g.pd0 = r.pd0; g.pd1 = r.pd1; g.pd2 = r.pd2;
    g.g0 = (int)o->g0;
    g.tiles2 = (int)((o->L.n[2] + kron_tile_cols() - 1) / kron_tile_cols());
    const int trows = v == 10 ? kron_v5_rows(o->pmax, epi, same_toeplitz12(o) ? 1 : 0)
                    : (!is3d && v == 9 && o->pmax == 3) ? kron_v3_rows_2d() : kron_tile_rows();
    g.tiles1 = (int)((o->L.n[1] + trows - 1) / trows);
    g.tout = v == 10 ? v5_to : (o->tout > 0 ? o->tout : 64 - 2 * o->pmax);
    if (v >= 4) g.tiles2 = (int)((o->L.n[2] + g.tout - 1) / g.tout);
    if (!is3d) {
        g.z_begin = 0; g.z_end = 1; g.chunk = 1; g.nchunks = 1; g.nch1 = 1; g.z2_begin = g.z2_end = 0;
        return 0;
    }
    if (zb < 0 || ze > o->L.n[0] || zb > ze) { set_error("plane range outside the slab"); return 1; }
    if (zb2 < 0 || ze2 > o->L.n[0] || zb2 > ze2 || (ze2 > zb2 && zb2 < ze && ze2 > zb)) {
        set_error("second plane range outside the slab or overlapping the first");
        return 1;
    }
    {   // tile order (tuning: POMS_TILE_ORDER=0/1)
        static int ord = -1;
        if (ord < 0) {
            const char* e = getenv("POMS_TILE_ORDER");
            ord = e ? (atoi(e) ? 1 : 0) : 0;
        }
        g.order = ord;
    }
    g.z_begin = (int)zb;
    g.z_end = (int)ze;
    g.z2_begin = (int)zb2;
    g.z2_end = (int)ze2;
    const int nz = (int)(ze - zb) + (int)(ze2 - zb2);
    int chunk = o->chunk;
    if (chunk <= 0) {
        const double slots = v == 10 ? 256.0 : 512.0;
        const int tiles = g.tiles2 * g.tiles1;
        chunk = auto_chunk(nz, tiles, o->pmax, slots);
        // The interior launch of a distributed call shares the GPU with the exchange and
        // the boundary launch on the communication stream: one chunk (one short round
        // that leaves CUs to them) where it fits 3/4 of the slots and costs at most 1.4x
        // the plane steps of the chunked grid (POMS_SPLIT_ONE=0: off).  Loopback proxy,
        // rank 1, interleaved (profiles/r06/split_chunk/): 8 ranks (59 interior planes)
        // 41.7-41.8 -> 38.7-38.9 ms per cycle, 4 ranks (123) 60.6-60.8 -> 58.8-59.1 ms;
        // at 2 ranks (252 planes, 1.43x) one chunk was slower (103.7 -> 111.1 ms) and
        // the rule keeps the chunks there
        static const bool split_one = !(getenv("POMS_SPLIT_ONE") && getenv("POMS_SPLIT_ONE")[0] == '0');
        bool one = false;
        if (o->split_interior && split_one && tiles <= 0.75 * slots && chunk < nz) {
            const int nc = (nz + chunk - 1) / chunk;
            const double r = (double)nc * tiles / slots;
            const double fr = std::floor(r);
            const double rounds = r > 1.0 ? fr + std::min(1.0, (r - fr) * 5.0) : 1.0;
            one = nz + 2 * o->pmax <= 1.4 * rounds * (chunk + 2 * o->pmax);
            if (one) chunk = nz;
        }
        // the v5 two-sweeps-from-zero launch (VALU-bound) balances better over twice
        // as many chunks: 515^3 p = 3, 86 instead of 172 planes, 836-838 against
        // 865-882 us in two interleaved sweeps, equal medians (833 us) in a third
        // (profiles/r03/chunks/); the other epilogues keep the model's pick (Jacobi
        // 715 us at 172 against 729 at 86)
        if (!one && v == 10 && epi == EPI_JACOBI0 && o->pmax == 3 && same_toeplitz12(o) && chunk / 2 >= 8 * o->pmax)
            chunk = (chunk + 1) / 2;   // (the 16-wave build only)
    }
    chunk = std::max(1, std::min(chunk, std::max(nz, 1)));
    g.chunk = chunk;
    g.nch1 = (int)((ze - zb + chunk - 1) / chunk);
    g.nchunks = g.nch1 + (int)((ze2 - zb2 + chunk - 1) / chunk);
    return 0;
}

// variants whose Jacobi epilogue also accumulates x_out . b (v3 and v4 kernels)
static bool fused_dot_ok(const poms_op* o) {
    return o->form == FORM_STENCIL || (o->variant >= 4 && o->variant <= 10) || o->variant == 114;
}


// General-stencil launch (FORM_STENCIL): the epilogues of op_run plus EPI_DIAG.
static int stencil_run(poms_op* o, int epi, double omega, const double* x, double* y, const double* b,
                       int64_t zb, int64_t ze, int want_norm, void* stream, int want_dot, int64_t zb2,
                       int64_t ze2) {
    if (epi == EPI_JACOBI0) { set_error("general stencil: no two-sweeps-from-zero epilogue"); return 1; }
    if (want_dot && epi != EPI_JACOBI && epi != EPI_APPLYDOT) { set_error("general stencil: dot needs Jacobi / apply+dot"); return 1; }
    const RowGeom r = row_geom(&o->L);
    if (zb < 0 || ze > r.n0 || zb > ze || zb2 < 0 || ze2 > r.n0 || zb2 > ze2) { set_error("general stencil: bad plane range"); return 1; }
    StencilGeom g{r.s0, r.s1, r.n0, r.n1, r.n2, r.pd0, r.pd1, r.pd2, o->sp[0], o->sp[1], o->sp[2],
                  2 * o->sp[0] + 1, 2 * o->sp[1] + 1, 2 * o->sp[2] + 1, (int64_t)r.n0 * r.n1 * r.n2,
                  (int)zb, (int)ze, (int)zb2, (int)ze2};
    const int maxb = (int)(kScratch / 2);
    int nb = 0;
    double* scr = o->ctx->scratch;
    const bool red = want_norm || want_dot || epi == EPI_APPLYDOT;
    if (stencil_launch(epi, g, o->coef, x, y, b, omega, want_norm ? scr : nullptr,
                       (want_dot || epi == EPI_APPLYDOT) ? scr + std::min<int64_t>(maxb, std::max<int64_t>(1, ((int64_t)(ze - zb + ze2 - zb2) * r.n1 * r.n2 + 255) / 256)) : nullptr,
                       maxb, as_stream(stream), &nb))
        return 1;
    POMS_HIP_CHECK(hipGetLastError());
    o->last_partials = red ? nb : 0;
    return 0;
}

// axis 1 and axis 2 share their Toeplitz rows bitwise (v5's SAME12 builds)
static bool same_toeplitz12(const poms_op* o) {
    for (int k = 0; k <= o->pmax; ++k)
        if (o->tc.t1a[k] != o->tc.t2a[k] || o->tc.t1b[k] != o->tc.t2b[k]) return false;
    return true;
}

// 2D Jacobi sweeps at p <= 3: v3 (9) by default; POMS_JAC2D_VARIANT=7 selects v4
// (tuning knob)
static int jacobi2d_variant() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("POMS_JAC2D_VARIANT");
        v = (e && atoi(e) == 7) ? 7 : 9;
    }
    return v;
}

// The kernel variant one launch of epilogue `epi` runs (see op_run).
static int resolve_variant(const poms_op* o, int epi) {
    int v = o->variant;
    if (v == 8) {
        const bool plain = epi == EPI_APPLY || epi == EPI_RESID || epi == EPI_JACOBI;
        if (o->ndim == 3 && v5_ok(o))
            v = 10;   // v5: kernel_bench at 515^3 p = 3; 8-wave tiles at 256^3 p = 4, 5
                      // (profiles/r02/configs/kb_p5_waves8.log: apply 231 -> 185 us at p = 5);
                      // sweeps from zero at p <= 2 and p = 4, 5 (8-wave tiles; at 256^3
                      // p = 4 208 vs 291 us for v3, p = 5 261 vs 428 us,
                      // profiles/r05/late/kb_p45_j0.log) and at p = 3 (16-wave tiles, 930 vs
                      // 945 us for v3 at 515^3, profiles/r02/j0_16wave/) where axes 1 and 2
                      // share their rows, 8-wave tiles where they do not (round 6; the
                      // 16-wave build of that case spills)
        else if (o->ndim == 3)
            v = ((epi == EPI_APPLY && o->pmax >= 3) || (plain && o->pmax >= 4)) ? 7 : 9;
        else if (epi == EPI_JACOBI && o->pmax <= 3)
            v = jacobi2d_variant();
        else
            v = ((epi == EPI_APPLY || epi == EPI_RESID) && o->pmax <= 3) ? 7 : 9;
    }
    if (v == 10 && !v5_ok(o)) v = 9;
    return v;
}

// Two Jacobi sweeps per launch (EPI_JACOBI2, kron_2d.hip): one-rank 2D p = 3
// Kronecker operators whose single sweep runs the v3 whole-array kernel (variant 9),
// whose bits the two-sweep kernel reproduces
static bool sweep2_ok(const poms_op* o) {
    if (o->ndim != 2 || o->pmax != 3 || o->form == FORM_STENCIL || o->ghost_corners) return false;
    if (o->L.pads[1] != 3 || o->L.pads[2] != 3 || resolve_variant(o, EPI_JACOBI) != 9) return false;
    const int64_t bytes = (int64_t)(o->L.n[0] + 2 * o->L.pads[0]) * row_geom(&o->L).s0 * 8;
    return bytes < 0x7ffffff0LL;
}

// partials as op_run: norm (sweep k+1) and dot (sweep k) at part_dst / the scratch.
// EPI_JACOBI3Z (x = b): all three sums or none, ||x1||^2, ||dr_2||^2, ||dr_3||^2 side by
// side (part_dst, or scratch[0, 3n))
static int op_run_j2(poms_op* o, int epi, double omega, const double* x, double* y, const double* b, int want_norm,
                     int want_dot, void* stream) {
    if (!sweep2_ok(o)) { set_error("two sweeps per launch: one-rank 2D p = 3 Kronecker operators (variant 9) only"); return 1; }
    if (x == y || b == y) { set_error("two sweeps per launch: x_out must not alias x_in or b"); return 1; }
    const bool fz = epi == EPI_JACOBI3Z;
    if (fz && (x != b || want_norm != want_dot)) { set_error("three sweeps from zero: x = b, all three sums or none"); return 1; }
    KronGeom g;
    if (op_geom(o, 0, 1, g, 9, 0, 0, 0, EPI_JACOBI)) return 1;
    const int trows = fz ? kron2d_j2_rows_default() : kron2d_j2_rows();
    g.tout = kron2d_j2_cols(o->pmax);
    g.tiles2 = (int)((o->L.n[2] + g.tout - 1) / g.tout);
    g.tiles1 = (int)((o->L.n[1] + trows - 1) / trows);
    const int64_t nblk = (int64_t)g.tiles2 * g.tiles1;
    o->last_variant = 9;
    if (nblk == 0) { o->last_partials = 0; return 0; }
    if (fz) {
        double* s0 = nullptr;
        o->last_part_host = false;
        if (want_norm) {
            if (o->part_dst && 3 * nblk <= o->part_cap) {
                s0 = o->part_dst;
                o->last_part_host = true;
            } else if (o->part_off == 0 && o->dot_base < 0 && 3 * nblk <= kScratch) {
                s0 = o->ctx->scratch;
            } else {
                set_error("too many blocks for the partial-sum scratch");
                return 1;
            }
        }
        KronPtrs p{b, y, b, o->a0t, o->b0t, o->a1, o->b1, o->a2, o->b2, s0 ? s0 + 2 * nblk : nullptr,
                   s0 ? s0 + nblk : nullptr, nullptr};
        if (kron2d_j2_launch(o->pmax, o->form, p, g, o->tc, omega, as_stream(stream), true, s0)) return 1;
        POMS_HIP_CHECK(hipGetLastError());
        o->last_partials = want_norm ? nblk : 0;
        return 0;
    }
    const int64_t dbase = o->dot_base < 0 ? nblk : o->dot_base;
    if ((want_norm || want_dot) && (o->part_off + nblk > dbase || dbase + o->part_off + nblk > kScratch)) {
        set_error("too many blocks for the partial-sum scratch");
        return 1;
    }
    double* pn = o->ctx->scratch + o->part_off;
    double* pd = o->ctx->scratch + dbase + o->part_off;
    o->last_part_host = false;
    if (o->part_dst && ((want_norm ? 1 : 0) + (want_dot ? 1 : 0)) * nblk <= o->part_cap) {
        pn = o->part_dst;
        pd = o->part_dst + (want_norm ? nblk : 0);
        o->last_part_host = true;
    }
    KronPtrs p{x, y, b, o->a0t, o->b0t, o->a1, o->b1, o->a2, o->b2, want_norm ? pn : nullptr,
               want_dot ? pd : nullptr, nullptr};
    if (kron2d_j2_launch(o->pmax, o->form, p, g, o->tc, omega, as_stream(stream), false, nullptr)) return 1;
    POMS_HIP_CHECK(hipGetLastError());
    o->last_partials = (want_norm || want_dot) ? nblk : 0;
    return 0;
}

static int op_run(poms_op* o, int epi, double omega, const double* x, double* y, const double* b,
                  int64_t zb, int64_t ze, int want_norm, void* stream, int want_dot = 0,
                  int64_t zb2 = 0, int64_t ze2 = 0) {
    if (!o || !x || !y) { set_error("null operator or vector"); return 1; }
    if (epi != EPI_APPLY && !b) { set_error("null right-hand side"); return 1; }
    if (epi == EPI_JACOBI2 || epi == EPI_JACOBI3Z) return op_run_j2(o, epi, omega, x, y, b, want_norm, want_dot, stream);
    if (o->form == FORM_STENCIL)
        return stencil_run(o, epi, omega, x, y, b, zb, ze, want_norm, stream, want_dot, zb2, ze2);
    if (epi == EPI_APPLYDOT && !(o->variant == 4 || o->variant == 8 || o->variant == 9 || o->variant == 10)) {
        set_error("apply + x.y: kernel variants 4, 8, 9, 10 only");
        return 1;
    }
    if (want_dot && ((epi != EPI_JACOBI && epi != EPI_JACOBI0 && epi != EPI_APPLYDOT) || !fused_dot_ok(o))) {
        set_error("fused x_out.b needs a Jacobi sweep on kernel variants 4-10");
        return 1;
    }
    if (epi == EPI_JACOBI0 && !(o->variant == 8 || o->variant == 9 || o->variant == 10 ||
                                (o->variant >= 110 && o->variant <= 112) || o->variant == 114)) {
        set_error("two sweeps from zero: kernel variant 8, 9 or 10 only");
        return 1;
    }
    // variant 8 (default when pads == pmax): the fastest measured kernel per
    // epilogue (profiles/r01/chunks/*.log) -- in 3D v4 (7) for apply at p >= 3 and
    // for every plain epilogue at p >= 4 (VALU-bound there), v3 with whole-array
    // buffer resources (9; falls back to 4 for arrays >= 2 GiB) otherwise; in 2D
    // v4 for apply / residual at p <= 3.  Fused dots and two-sweeps-from-zero: 9.
    // Variant 10 (v5) runs apply / residual / Jacobi / apply+dot of 3D p <= 3
    // operators, and is what 8 picks for them; 9 otherwise.
    int v = resolve_variant(o, epi);
    const int v5_diag = (v >= 101 && v <= 114) ? v - 100 : 0;   // v5 diagnostic / tuning builds
    if (v5_diag) v = 10;
    o->last_variant = v5_diag ? 100 + v5_diag : v;
    int v5_h = 0, v5_to = 0;
    if (v == 10) kron_v5_tile(o->pmax, v5_aligned(o, x), &v5_h, &v5_to);
    KronGeom g;
    if (op_geom(o, zb, ze, g, v, v5_to, zb2, ze2, epi)) return 1;
    const int64_t nblk = (int64_t)g.tiles2 * g.tiles1 * g.nchunks;
    if (nblk == 0) { o->last_partials = 0; return 0; }
    const int64_t dbase = o->dot_base < 0 ? nblk : o->dot_base;
    if ((want_norm || want_dot) &&
        (o->part_off + nblk > dbase || dbase + o->part_off + nblk > kScratch)) {
        set_error("too many blocks for the partial-sum scratch");
        return 1;
    }
    double* pn = o->ctx->scratch + o->part_off;
    double* pd = o->ctx->scratch + dbase + o->part_off;
    o->last_part_host = false;
    if (o->part_dst && ((want_norm ? 1 : 0) + (want_dot ? 1 : 0)) * nblk <= o->part_cap) {
        pn = o->part_dst;
        pd = o->part_dst + (want_norm ? nblk : 0);
        o->last_part_host = true;
    }
    KronPtrs p{x, y, b, o->a0t, o->b0t, o->a1, o->b1, o->a2, o->b2, want_norm ? pn : nullptr,
               want_dot ? pd : nullptr, o->rdiag0};
    poms_op::TimedLaunch* tlh = nullptr;
    bool tl_ext = false;
    if (o->timing && (o->t_epi < 0 || o->t_epi == epi) && (o->t_seen++ % o->t_every) == 0) {
        // events on the launch stream around this launch (a sample: every t_every-th)
        if (o->tl_used == o->tl.size()) {
            poms_op::TimedLaunch t{};
            POMS_HIP_CHECK(hipEventCreate(&t.e0));
            POMS_HIP_CHECK(hipEventCreate(&t.e1));
            o->tl.push_back(t);
        }
        tlh = &o->tl[o->tl_used++];
        tlh->epi = epi;
        tlh->ndof = (int64_t)((ze - zb) + (ze2 - zb2)) * g.n1 * g.n2;
        // v5 outside a capture: the events ride on the kernel's own dispatch
        // (hipExtLaunchKernel start / stop), i.e. the kernel's execution time as
        // rocprofv3 reports it; otherwise event records before and after the launch
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        POMS_HIP_CHECK(hipStreamIsCapturing(as_stream(stream), &cs));
        if (v == 10 && cs == hipStreamCaptureStatusNone) {
            kron_v5_set_launch_events(tlh->e0, tlh->e1);
            tl_ext = true;
        } else {
            POMS_HIP_CHECK(timing_record(tlh->e0, as_stream(stream)));
        }
    }
    const int rc = v == 10
        ? kron_v5_launch(o->pmax, epi, p, g, o->tc, v5_h, omega, as_stream(stream), v5_diag)
        : v == 0
        ? kron_launch(o->pmax, o->ndim == 3, o->form, epi, p, g, omega, as_stream(stream))
        : (v == 7 || (v >= 92 && v <= 100))
        ? kron_v4_launch(o->pmax, o->ndim == 3, o->form, epi, p, g, o->tc, omega, as_stream(stream),
                         v == 7 ? 0 : v - 91)
        : kron_v3_launch(v, o->pmax, o->ndim == 3, o->form, epi, p, g, o->tc, omega, as_stream(stream));
    if (tl_ext && !kron_v5_launch_events_used()) {   // (the v5 launch failed before its dispatch)
        kron_v5_set_launch_events(nullptr, nullptr);
        if (!rc) { set_error("v5: timed launch did not take its events"); return 1; }
    }
    if (tlh && !tl_ext) POMS_HIP_CHECK(timing_record(tlh->e1, as_stream(stream)));
    if (rc) return 1;
    POMS_HIP_CHECK(hipGetLastError());
    o->last_partials = (want_norm || want_dot) ? nblk : 0;
    return 0;
}

int poms_op_apply(poms_op* op, const double* x, double* y, int64_t zb, int64_t ze, void* stream) {
    return op_run(op, EPI_APPLY, 0.0, x, y, nullptr, zb, ze, 0, stream);
}

int poms_op_residual(poms_op* op, const double* b, const double* x, double* r, int64_t zb,
                     int64_t ze, void* stream) {
    return op_run(op, EPI_RESID, 0.0, x, r, b, zb, ze, 0, stream);
}

int poms_op_jacobi_sweep(poms_op* op, double omega, const double* b, const double* x_in,
                         double* x_out, int64_t zb, int64_t ze, int want_norm, void* stream) {
    if (x_in == x_out) { set_error("jacobi sweep: x_out must not alias x_in"); return 1; }
    return op_run(op, EPI_JACOBI, omega, x_in, x_out, b, zb, ze, want_norm, stream);
}

int poms_op_jacobi_sweep_dot(poms_op* op, double omega, const double* b, const double* x_in,
                             double* x_out, int64_t zb, int64_t ze, int want_norm, void* stream) {
    if (x_in == x_out) { set_error("jacobi sweep: x_out must not alias x_in"); return 1; }
    return op_run(op, EPI_JACOBI, omega, x_in, x_out, b, zb, ze, want_norm, stream, 1);
}

int poms_op_apply_dot(poms_op* op, const double* x, double* y, int64_t zb, int64_t ze, void* stream) {
    if (x == y) { set_error("apply: y must not alias x"); return 1; }
    return op_run(op, EPI_APPLYDOT, 0.0, x, y, x, zb, ze, 0, stream, 1);
}

int poms_op_apply_dot_supported(poms_op* op, int* yes) {
    if (!op || !yes) { set_error("poms_op_apply_dot_supported: null argument"); return 1; }
    const int v = op->variant;
    *yes = (op->form == FORM_STENCIL || v == 4 || v == 8 || v == 9 || v == 10) ? 1 : 0;
    return 0;
}

int poms_op_jacobi_from_zero(poms_op* op, double omega, const double* b, double* x_out,
                             int64_t zb, int64_t ze, int want_norm, void* stream) {
    if (!op || !b || !x_out) { set_error("jacobi from zero: null argument"); return 1; }
    if (b == x_out) { set_error("jacobi from zero: x_out must not alias b"); return 1; }
    int yes = 0;
    if (poms_op_from_zero_supported(op, &yes)) return 1;
    if (!yes) { set_error("jacobi from zero: not supported by this operator (poms_op_from_zero_supported)"); return 1; }
    return op_run(op, EPI_JACOBI0, omega, b, x_out, b, zb, ze, want_norm, stream, want_norm);
}

int poms_op_from_zero_supported(poms_op* op, int* yes) {
    if (!op || !yes) { set_error("poms_op_from_zero_supported: null argument"); return 1; }
    const int64_t bytes = (int64_t)(op->L.n[0] + 2 * op->L.pads[0]) * row_geom(&op->L).s0 * 8;
    // 2D (round 6, v3): not on a block of a decomposition (its ghost rows' x1 would need
    // the neighbours' diagonal)
    *yes = ((op->ndim == 3 || (op->ndim == 2 && !op->ghost_corners)) && op->form != FORM_STENCIL &&
            (op->variant == 8 || op->variant == 9 || op->variant == 10 ||
             (op->variant >= 110 && op->variant <= 112) || op->variant == 114) &&
            bytes < 0x7ffffff0LL) ? 1 : 0;
    return 0;
}

int poms_op_sweep2_supported(poms_op* op, int* yes) {
    if (!op || !yes) { set_error("poms_op_sweep2_supported: null argument"); return 1; }
    *yes = sweep2_ok(op) ? 1 : 0;
    return 0;
}

int poms_op_jacobi3_from_zero(poms_op* op, double omega, const double* b, double* x_out, double* norms_out,
                              void* stream) {
    if (!op || !b || !x_out) { set_error("jacobi3 from zero: null argument"); return 1; }
    const bool wn = norms_out != nullptr;
    if (op_run(op, EPI_JACOBI3Z, omega, b, x_out, b, 0, 1, wn ? 1 : 0, stream, wn ? 1 : 0)) return 1;
    const int64_t n = op->last_partials;
    if (wn)
        for (int i = 0; i < 3; ++i) reduce_launch(op->ctx->scratch + i * n, (int)n, norms_out + i, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_op_fused_dot_supported(poms_op* op, int* yes) {
    if (!op || !yes) { set_error("poms_op_fused_dot_supported: null argument"); return 1; }
    *yes = fused_dot_ok(op) ? 1 : 0;
    return 0;
}

int poms_op_diag_scale(poms_op* o, double scale, const double* b, double* x, int want_norm,
                       void* stream) {
    if (!o || !b || !x) { set_error("poms_op_diag_scale: null argument"); return 1; }
    if (o->form == FORM_STENCIL)
        return stencil_run(o, EPI_DIAG, scale, b, x, b, 0, o->L.n[0], want_norm, stream, 0, 0, 0);
    const RowGeom g = row_geom(&o->L);
    int nb = 0;
    diag_scale_launch(o->ndim == 3, o->form, g, o->pmax, (int)o->g0, scale, b, x, o->a0t, o->b0t,
                      o->a1, o->b1, o->dg2a, o->dg2b, want_norm ? o->ctx->scratch : nullptr,
                      as_stream(stream), &nb);
    POMS_HIP_CHECK(hipGetLastError());
    o->last_partials = want_norm ? nb : 0;
    return 0;
}

int poms_op_set_ghost_corners(poms_op* op, int yes) {
    if (!op) { set_error("poms_op_set_ghost_corners: null operator"); return 1; }
    op->ghost_corners = yes != 0;
    ++op->gen;
    return 0;
}

// One launch plus its reductions (one host call instead of three); the launch
// may cover a second plane range [zb2, ze2) (the slab's other boundary).
}  // extern "C"

// One launch of `epilogue` over planes [zb, ze) + [zb2, ze2), its partials written
// where op->part_off / dot_base say; the argument checks of poms_op_run_reduce2.
static int op_run_epi(poms_op* op, int epilogue, double omega, const double* x, double* y, const double* b,
                      int64_t zb, int64_t ze, int64_t zb2, int64_t ze2, bool wn, bool wd, void* stream) {
    switch (epilogue) {
        case EPI_APPLY:
            if (wn || wd) { set_error("poms_op_run_reduce: apply has no reductions"); return 1; }
            if (op_run(op, EPI_APPLY, 0.0, x, y, nullptr, zb, ze, 0, stream, 0, zb2, ze2)) return 1;
            break;
        case EPI_RESID:
            if (wn || wd) { set_error("poms_op_run_reduce: residual has no reductions"); return 1; }
            if (op_run(op, EPI_RESID, 0.0, x, y, b, zb, ze, 0, stream, 0, zb2, ze2)) return 1;
            break;
        case EPI_JACOBI:
            if (x == y) { set_error("jacobi sweep: x_out must not alias x_in"); return 1; }
            if (op_run(op, EPI_JACOBI, omega, x, y, b, zb, ze, wn ? 1 : 0, stream, wd ? 1 : 0, zb2, ze2)) return 1;
            break;
        case EPI_JACOBI0:   // x = b: norm_out <- ||dr_2||^2, dot_out <- ||x1||^2
            {
                int fz = 0;
                if (poms_op_from_zero_supported(op, &fz)) return 1;
                if (!fz) { set_error("jacobi from zero: not supported by this operator"); return 1; }
            }
            if (b == y) { set_error("jacobi from zero: x_out must not alias b"); return 1; }
            if (wn != wd) { set_error("jacobi from zero: both norms or neither"); return 1; }
            if (op_run(op, EPI_JACOBI0, omega, b, y, b, zb, ze, wn ? 1 : 0, stream, wn ? 1 : 0, zb2, ze2)) return 1;
            break;
        case EPI_JACOBI2:   // two sweeps from x: norm_out <- ||dr_{k+1}||^2, dot_out <- ||dr_k||^2
            if (zb != 0 || ze != 1 || zb2 != ze2) { set_error("two sweeps per launch: 2D (planes [0, 1))"); return 1; }
            if (op_run(op, EPI_JACOBI2, omega, x, y, b, 0, 1, wn ? 1 : 0, stream, wd ? 1 : 0)) return 1;
            break;
        case EPI_JACOBI3Z:   // sweeps 1-3 from x = 0 (x = b): norm_out <- ||dr_3||^2, dot_out <- ||dr_2||^2
            // (poms_op_run_reduce2 cannot return the third sum: poms_op_jacobi3_from_zero)
            if (zb != 0 || ze != 1 || zb2 != ze2) { set_error("three sweeps from zero: 2D (planes [0, 1))"); return 1; }
            if (op_run(op, EPI_JACOBI3Z, omega, b, y, b, 0, 1, wn ? 1 : 0, stream, wd ? 1 : 0)) return 1;
            break;
        case EPI_APPLYDOT:
            if (x == y) { set_error("apply: y must not alias x"); return 1; }
            if (wn || !wd) { set_error("apply + dot: dot_out only"); return 1; }
            if (op_run(op, EPI_APPLYDOT, 0.0, x, y, x, zb, ze, 0, stream, 1, zb2, ze2)) return 1;
            break;
        default:
            set_error("poms_op_run_reduce: bad epilogue");
            return 1;
    }
    return 0;
}

namespace poms {
// The distributed operator call's two launches -- planes [ib, ie) on `stream`, then
// the boundary ranges [b1s, b1e) + [b2s, b2e) once the ghost exchange is done --
// with both launches' partials side by side in the scratch and ONE reduction per
// requested sum after both (one launch fewer per sum than reducing each launch;
// poms_op_run_dist).  The boundary launch goes to h.bstream when given (the
// communication stream, right behind the exchange): it depends on the exchange
// only, not on the interior launch, so its workgroups fill the CUs the interior
// launch's last round leaves idle instead of running as a separate, mostly empty
// round of its own; `stream` then waits for it (h.join) before the reductions.
int op_run_split(poms_op* op, int epilogue, double omega, const double* x, double* y, const double* b,
                 int64_t ib, int64_t ie, int64_t b1s, int64_t b1e, int64_t b2s, int64_t b2e, double* norm_out,
                 double* dot_out, const SplitHooks& h, void* stream) {
    if (!op) { set_error("op_run_split: null operator"); return 1; }
    if (op->form == FORM_STENCIL) {   // its own partials layout: reduce each launch, both on `stream`
        if (poms_op_run_reduce2(op, epilogue, omega, x, y, b, ib, ie, 0, 0, norm_out, dot_out, 0, stream)) return 1;
        if (h.ghosts_on(h.arg, stream)) return 1;
        return poms_op_run_reduce2(op, epilogue, omega, x, y, b, b1s, b1e, b2s, b2e, norm_out, dot_out, 1, stream);
    }
    const bool wn = norm_out != nullptr, wd = dot_out != nullptr;
    struct Reset {
        poms_op* o;
        ~Reset() { o->part_off = 0; o->dot_base = -1; }
    } reset{op};
    op->part_off = 0;
    op->dot_base = kScratch / 2;
    op->split_interior = true;
    const int rci = op_run_epi(op, epilogue, omega, x, y, b, ib, ie, 0, 0, wn, wd, stream);
    op->split_interior = false;
    if (rci) return 1;
    const int64_t n1 = op->last_partials;
    void* bs = h.bstream ? h.bstream : stream;
    if (h.ghosts_on(h.arg, bs)) return 1;
    op->part_off = n1;
    if (op_run_epi(op, epilogue, omega, x, y, b, b1s, b1e, b2s, b2e, wn, wd, bs)) return 1;
    if (bs != stream && h.join(h.arg, bs, stream)) return 1;
    const int64_t n = n1 + op->last_partials;
    op->last_partials = 0;   // not in the layout poms_op_last_partials describes
    // (the reductions stay on `stream`: queued on the boundary stream behind the
    // boundary launch they added a second cross-queue wait per call -- loopback proxy
    // 41.7 -> 43.5 ms, profiles/r03/proxy/reductions_on_cs_REVERTED/)
    if (wn) reduce_launch(op->ctx->scratch, (int)n, norm_out, as_stream(stream));
    if (wd) reduce_launch(op->ctx->scratch + kScratch / 2, (int)n, dot_out, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}
}  // namespace poms

extern "C" {

int poms_op_run_reduce2(poms_op* op, int epilogue, double omega, const double* x, double* y,
                        const double* b, int64_t zb, int64_t ze, int64_t zb2, int64_t ze2,
                        double* norm_out, double* dot_out, int accumulate, void* stream) {
    if (!op) { set_error("poms_op_run_reduce: null operator"); return 1; }
    const bool wn = norm_out != nullptr, wd = dot_out != nullptr;
    if (op_run_epi(op, epilogue, omega, x, y, b, zb, ze, zb2, ze2, wn, wd, stream)) return 1;
    const int64_t n = op->last_partials;
    if (wn) reduce_launch(op->ctx->scratch, (int)n, norm_out, as_stream(stream), accumulate);
    if (wd) reduce_launch(op->ctx->scratch + n, (int)n, dot_out, as_stream(stream), accumulate);
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_op_run_reduce(poms_op* op, int epilogue, double omega, const double* x, double* y,
                       const double* b, int64_t zb, int64_t ze, double* norm_out, double* dot_out,
                       int accumulate, void* stream) {
    return poms_op_run_reduce2(op, epilogue, omega, x, y, b, zb, ze, 0, 0, norm_out, dot_out, accumulate, stream);
}

// Async copy of `count` doubles from device memory to (pinned) host memory.
int poms_copy_to_host_async(poms_ctx* ctx, const double* src_dev, double* dst_host, int64_t count, void* stream) {
    if (!ctx || !src_dev || !dst_host || count < 0) { set_error("poms_copy_to_host_async: bad argument"); return 1; }
    POMS_HIP_CHECK(hipMemcpyAsync(dst_host, src_dev, count * sizeof(double), hipMemcpyDeviceToHost,
                                  as_stream(stream)));
    return 0;
}

int poms_op_last_partials(poms_op* op, int64_t* count) {
    if (!op || !count) { set_error("null argument"); return 1; }
    *count = op->last_partials;
    return 0;
}

int poms_kron_dot_2d(poms_ctx* ctx, const int64_t* starts, const int64_t* ends,
                     const int64_t* pads, const double* X, double* X_tmp, double* Y,
                     const double* A, int64_t a_rows, const double* B, int64_t b_rows) {
    (void)X_tmp;
    if (!ctx || !starts || !ends || !pads || !X || !Y || !A || !B) {
        set_error("poms_kron_dot_2d: null argument");
        return 1;
    }
    const int64_t n1 = ends[0] - starts[0] + 1, n2 = ends[1] - starts[1] + 1;
    const int p1 = (int)pads[0], p2 = (int)pads[1];
    if (n1 < 1 || n2 < 1 || p1 < 1 || p2 < 1 || p1 > 5 || p2 > 5) {
        set_error("poms_kron_dot_2d: bad extents or pads (1..5)");
        return 1;
    }
    if (starts[0] < 0 || ends[0] >= a_rows || starts[1] < 0 || ends[1] >= b_rows) {
        set_error("poms_kron_dot_2d: starts/ends outside the band arrays");
        return 1;
    }
    const int pm = std::max(p1, p2), W = 2 * pm + 1;
    // local, re-centred band rows of width 2*pm+1
    std::vector<double> fa(n1 * W, 0.0), fb(n2 * W, 0.0);
    for (int64_t i = 0; i < n1; ++i)
        for (int k = 0; k < 2 * p1 + 1; ++k) fa[i * W + k + pm - p1] = A[(starts[0] + i) * (2 * p1 + 1) + k];
    for (int64_t i = 0; i < n2; ++i)
        for (int k = 0; k < 2 * p2 + 1; ++k) fb[i * W + k + pm - p2] = B[(starts[1] + i) * (2 * p2 + 1) + k];
    poms_layout L{{1, n1, n2}, {0, p1, p2}};
    const double* f[6] = {nullptr, nullptr, fa.data(), nullptr, fb.data(), nullptr};
    poms_op* op = nullptr;
    if (poms_op_create(ctx, 2, &L, FORM_SINGLE, pm, f, 0, 1, &op)) return 1;
    const size_t nel = (size_t)(n1 + 2 * p1) * (n2 + 2 * p2);
    double *dx = nullptr, *dy = nullptr;
    int rc = 0;
    if (hipMalloc(reinterpret_cast<void**>(&dx), nel * sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dy), nel * sizeof(double)) != hipSuccess) {
        set_error("poms_kron_dot_2d: hipMalloc failed");
        rc = 1;
    }
    if (!rc && (hipMemcpy(dx, X, nel * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(dy, Y, nel * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)) {
        set_error("poms_kron_dot_2d: upload failed");
        rc = 1;
    }
    if (!rc) rc = poms_op_apply(op, dx, dy, 0, 1, nullptr);
    if (!rc && hipMemcpy(Y, dy, nel * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("poms_kron_dot_2d: download failed");
        rc = 1;
    }
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    poms_op_destroy(op);
    return rc;
}

// ---- vector kernels -----------------------------------------------------------
static int vec_common(poms_ctx* ctx, const poms_layout* L, int op, double a, double b,
                      const double* x, const double* y, double* z, double* w, const double* q,
                      double* out_dev, void* stream, const double* ab_dev = nullptr) {
    if (!ctx || !layout_ok(L)) { set_error("vector op: bad context or layout"); return 1; }
    const RowGeom g = row_geom(L);
    int nb = 0;
    const bool red = (op == V_DOT || op == V_PCGUPD || op == V_RUPD);
    // whole interior planes as one flat range (ghost rows / columns are zero in every
    // vector and stay zero -- unless the layout says they hold a neighbour's data);
    // the per-row kernel for fills, mixed alignments and ghost data
    const int64_t off = (int64_t)g.pd0 * g.s0, count = (int64_t)g.n0 * g.s0;
    auto at = [&](const double* v) { return v ? v + off : nullptr; };
    const bool flat = !(L->flags & POMS_LAYOUT_GHOST_DATA) &&
                      vec_flat_launch(op, count, a, b, at(x), at(y), const_cast<double*>(at(z)),
                                      const_cast<double*>(at(w)), at(q), red ? ctx->scratch : nullptr,
                                      as_stream(stream), &nb, ab_dev) == 0;
    if (!flat && vec_launch(op, g, a, b, x, y, z, w, q, red ? ctx->scratch : nullptr, as_stream(stream), &nb,
                            ab_dev))
        return 1;
    if (red) reduce_wide_launch(ctx->scratch, nb, out_dev, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_vec_axpby(poms_ctx* ctx, const poms_layout* L, double a, const double* x, double b,
                   const double* y, double* z, void* stream) {
    if (!x || !y || !z) { set_error("axpby: null vector"); return 1; }
    return vec_common(ctx, L, V_AXPBY, a, b, x, y, z, nullptr, nullptr, nullptr, stream);
}

int poms_vec_scale(poms_ctx* ctx, const poms_layout* L, double a, const double* x, double* z,
                   void* stream) {
    if (!x || !z) { set_error("scale: null vector"); return 1; }
    return vec_common(ctx, L, V_SCALE, a, 0.0, x, nullptr, z, nullptr, nullptr, nullptr, stream);
}

// z = x and z.z into out_dev in one pass (pcg from x0 = None: r = b, ||r||^2), with the
// bits of poms_vec_scale(1.0) + poms_vec_dot(z, z): the same flat grid, the same
// per-thread order.  Where the flat kernel does not apply (mixed alignment, ghost
// data) the two calls.
static int vec_copy_dot(poms_ctx* ctx, const poms_layout* L, const double* x, double* z, double* out_dev,
                        void* stream) {
    if (!ctx || !layout_ok(L) || !x || !z || !out_dev) { set_error("copy_dot: bad argument"); return 1; }
    const RowGeom g = row_geom(L);
    const int64_t off = (int64_t)g.pd0 * g.s0, count = (int64_t)g.n0 * g.s0;
    int nb = 0;
    static const bool cd_off = [] { const char* e = getenv("POMS_COPY_DOT"); return e && e[0] == '0'; }();
    if (!cd_off && !(L->flags & POMS_LAYOUT_GHOST_DATA) &&
        vec_flat_launch(V_SCALEDOT, count, 1.0, 0.0, x + off, nullptr, z + off, nullptr, nullptr, ctx->scratch,
                        as_stream(stream), &nb) == 0) {
        reduce_wide_launch(ctx->scratch, nb, out_dev, as_stream(stream));
        POMS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    return poms_vec_scale(ctx, L, 1.0, x, z, stream) || poms_vec_dot(ctx, L, z, z, out_dev, stream);
}

int poms_vec_fill(poms_ctx* ctx, const poms_layout* L, double v, double* z, void* stream) {
    if (!z) { set_error("fill: null vector"); return 1; }
    return vec_common(ctx, L, V_FILL, v, 0.0, nullptr, nullptr, z, nullptr, nullptr, nullptr, stream);
}

int poms_vec_zero_ghosts(poms_ctx* ctx, const poms_layout* L, double* z, void* stream) {
    if (!ctx || !layout_ok(L) || !z) { set_error("zero_ghosts: bad argument"); return 1; }
    zero_ghosts_launch(row_geom(L), z, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_vec_dot(poms_ctx* ctx, const poms_layout* L, const double* x, const double* y,
                 double* out_dev, void* stream) {
    if (!x || !y || !out_dev) { set_error("dot: null argument"); return 1; }
    return vec_common(ctx, L, V_DOT, 0.0, 0.0, x, y, nullptr, nullptr, nullptr, out_dev, stream);
}

int poms_pcg_update(poms_ctx* ctx, const poms_layout* L, double alpha, double* x, const double* p,
                    double* r, const double* q, double* out_dev, void* stream) {
    if (!x || !p || !r || !q || !out_dev) { set_error("pcg_update: null argument"); return 1; }
    return vec_common(ctx, L, V_PCGUPD, alpha, 0.0, nullptr, p, x, r, q, out_dev, stream);
}

int poms_pcg_r_update(poms_ctx* ctx, const poms_layout* L, double alpha, double* r, const double* q,
                      double* out_dev, void* stream) {
    if (!r || !q || !out_dev) { set_error("pcg_r_update: null argument"); return 1; }
    return vec_common(ctx, L, V_RUPD, alpha, 0.0, nullptr, nullptr, nullptr, r, q, out_dev, stream);
}

int poms_pcg_xp_update(poms_ctx* ctx, const poms_layout* L, double alpha, double beta, double* x,
                       double* p, const double* s, void* stream) {
    if (!x || !p || !s) { set_error("pcg_xp_update: null argument"); return 1; }
    return vec_common(ctx, L, V_XPUPD, alpha, beta, s, nullptr, x, p, nullptr, nullptr, stream);
}

// Device-coefficient forms: the scalars are read by the kernel from device memory
// (ab_dev[0], ab_dev[1]), so pcg's alpha / beta never visit the host.
int poms_vec_axpby_dev(poms_ctx* ctx, const poms_layout* L, const double* ab_dev, const double* x,
                       const double* y, double* z, void* stream) {
    if (!x || !y || !z || !ab_dev) { set_error("axpby_dev: null argument"); return 1; }
    return vec_common(ctx, L, V_AXPBY, 0.0, 0.0, x, y, z, nullptr, nullptr, nullptr, stream, ab_dev);
}

int poms_pcg_r_update_dev(poms_ctx* ctx, const poms_layout* L, const double* alpha_dev, double* r,
                          const double* q, double* out_dev, void* stream) {
    if (!r || !q || !out_dev || !alpha_dev) { set_error("pcg_r_update_dev: null argument"); return 1; }
    return vec_common(ctx, L, V_RUPD, 0.0, 0.0, nullptr, nullptr, nullptr, r, q, out_dev, stream, alpha_dev);
}

int poms_pcg_xp_update_dev(poms_ctx* ctx, const poms_layout* L, const double* ab_dev, double* x, double* p,
                           const double* s, void* stream) {
    if (!x || !p || !s || !ab_dev) { set_error("pcg_xp_update_dev: null argument"); return 1; }
    return vec_common(ctx, L, V_XPUPD, 0.0, 0.0, s, nullptr, x, p, nullptr, nullptr, stream, ab_dev);
}

int poms_reduce_partials(poms_ctx* ctx, int64_t count, double* out_dev, void* stream) {
    return poms_reduce_partials_at(ctx, 0, count, out_dev, stream);
}

int poms_reduce_partials_at(poms_ctx* ctx, int64_t offset, int64_t count, double* out_dev, void* stream) {
    if (!ctx || !out_dev || count < 0 || offset < 0 || offset + count > kScratch) {
        set_error("reduce: bad argument");
        return 1;
    }
    reduce_launch(ctx->scratch + offset, (int)count, out_dev, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- transfer -------------------------------------------------------------------
int poms_transfer_create(poms_ctx* ctx, int ndim, const poms_layout* fine, int64_t g0,
                         const int64_t* nf_global, const int64_t* nc, const double* const* P,
                         poms_transfer** tr) {
    if (!ctx || !tr || !nf_global || !nc || !P || !layout_ok(fine)) {
        set_error("poms_transfer_create: bad argument");
        return 1;
    }
    if (ndim < 1 || ndim > 3) { set_error("poms_transfer_create: ndim 1..3"); return 1; }
    const bool is3d = ndim == 3;
    const int d0 = is3d ? 0 : 1;
    int64_t ncmax = 0;
    for (int d = d0; d < 3; ++d) {
        if (!P[d] || nc[d] < 1 || nf_global[d] < 1) { set_error("poms_transfer_create: bad axis"); return 1; }
        ncmax = std::max(ncmax, nc[d]);
    }
    if (!is3d && (fine->n[0] != 1 || fine->pads[0] != 0)) {
        set_error("poms_transfer_create: 1D/2D layouts need n[0]=1, pads[0]=0");
        return 1;
    }
    for (int d = 1; d < 3; ++d)
        if (nf_global[d] != fine->n[d]) { set_error("poms_transfer_create: only axis 0 may be sliced"); return 1; }
    if (is3d && (g0 < 0 || g0 + fine->n[0] > nf_global[0])) { set_error("poms_transfer_create: bad slab"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(ctx->device));
    auto* t = new poms_transfer();
    t->ctx = ctx;
    t->ndim = ndim;
    t->ncm = ncmax <= 16 ? 16 : 32;
    t->banded = ncmax > 32;
    t->L = *fine;
    t->g0 = is3d ? g0 : 0;
    int rc = 0;
    for (int d = 0; d < 3; ++d) {
        t->nf[d] = (d < d0) ? 1 : nf_global[d];
        t->nc[d] = (d < d0) ? 1 : nc[d];
        if (d < d0) continue;
        if (!t->banded) {
            std::vector<double> pm(t->nf[d] * t->ncm, 0.0);
            for (int64_t i = 0; i < t->nf[d]; ++i)
                for (int64_t j = 0; j < t->nc[d]; ++j) pm[i * t->ncm + j] = P[d][i * t->nc[d] + j];
            rc |= upload(pm.data(), pm.size(), &t->Pm[d]);
            continue;
        }
        // banded: non-zero span of every row of P and of every column
        const int64_t nfd = t->nf[d], ncd = t->nc[d];
        const double* Pd = P[d];
        std::vector<int> jl(nfd, 0), il(ncd, 0);
        int wp = 1, wr = 1;
        for (int64_t i = 0; i < nfd; ++i) {
            int64_t a = -1, b = -1;
            for (int64_t j = 0; j < ncd; ++j)
                if (Pd[i * ncd + j] != 0.0) { if (a < 0) a = j; b = j; }
            jl[i] = a < 0 ? 0 : (int)a;
            wp = std::max(wp, a < 0 ? 1 : (int)(b - a + 1));
        }
        for (int64_t j = 0; j < ncd; ++j) {
            int64_t a = -1, b = -1;
            for (int64_t i = 0; i < nfd; ++i)
                if (Pd[i * ncd + j] != 0.0) { if (a < 0) a = i; b = i; }
            il[j] = a < 0 ? 0 : (int)a;
            wr = std::max(wr, a < 0 ? 1 : (int)(b - a + 1));
        }
        if (wp > 64 || wr > 256) { set_error("poms_transfer_create: prolongation is not banded"); rc = 1; break; }
        std::vector<double> pb(nfd * wp, 0.0), rb(ncd * wr, 0.0);
        for (int64_t i = 0; i < nfd; ++i)
            for (int k = 0; k < wp && jl[i] + k < ncd; ++k) pb[i * wp + k] = Pd[i * ncd + jl[i] + k];
        for (int64_t j = 0; j < ncd; ++j)
            for (int k = 0; k < wr && il[j] + k < nfd; ++k) rb[j * wr + k] = Pd[(il[j] + k) * ncd + j];
        t->wP[d] = wp;
        t->wR[d] = wr;
        rc |= upload(pb.data(), pb.size(), &t->Pb[d]);
        rc |= upload(rb.data(), rb.size(), &t->Rb[d]);
        if (!rc && hipMalloc(reinterpret_cast<void**>(&t->jlo[d]), nfd * sizeof(int)) != hipSuccess) rc = 1;
        if (!rc && hipMalloc(reinterpret_cast<void**>(&t->ilo[d]), ncd * sizeof(int)) != hipSuccess) rc = 1;
        if (!rc && hipMemcpy(t->jlo[d], jl.data(), nfd * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) rc = 1;
        if (!rc && hipMemcpy(t->ilo[d], il.data(), ncd * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) rc = 1;
    }
    const int64_t n1 = fine->n[1], n2 = fine->n[2];
    const size_t sz0 = (size_t)t->nc[0] * n1 * n2;
    const size_t sz1 = (size_t)t->nc[0] * t->nc[1] * n2;
    if (!rc && hipMalloc(reinterpret_cast<void**>(&t->t0), std::max<size_t>(sz0, 1) * sizeof(double)) != hipSuccess) rc = 1;
    if (!rc && hipMalloc(reinterpret_cast<void**>(&t->t1), std::max<size_t>(sz1, 1) * sizeof(double)) != hipSuccess) rc = 1;
    if (rc) {
        if (g_err.empty()) set_error("poms_transfer_create: allocation failed");
        poms_transfer_destroy(t);
        return 1;
    }
    *tr = t;
    return 0;
}

int poms_transfer_destroy(poms_transfer* t) {
    if (!t) return 0;
    for (double* p : {t->Pm[0], t->Pm[1], t->Pm[2], t->t0, t->t1, t->Pb[0], t->Pb[1], t->Pb[2], t->Rb[0],
                      t->Rb[1], t->Rb[2], t->part, t->Gf[0], t->Gf[1], t->Gf[2], t->Gf[3], t->Gf[4], t->Gf[5],
                      t->Pf[0], t->Pf[1], t->Pf[2], t->ru, t->rv, t->mpart})
        if (p) (void)hipFree(p);
    for (int* p : {t->jlo[0], t->jlo[1], t->jlo[2], t->ilo[0], t->ilo[1], t->ilo[2]})
        if (p) (void)hipFree(p);
    delete t;
    return 0;
}

// one axis pass of a transfer: dense-P kernels for small coarse extents, banded
// gather kernels otherwise
static int tpass(poms_transfer* t, bool restrict_dir, int d, const AxisPass& ps, const double* in,
                 double* out, hipStream_t st) {
    if (!t->banded) {
        double* part = nullptr;
        if (restrict_dir) {   // split-axis partials (few lines): a buffer grown on first use
            const int64_t need = transfer_split_scratch(t->ncm, ps);
            if (need > t->part_n) {
                if (t->part) (void)hipFree(t->part);
                t->part = nullptr;
                t->part_n = 0;
                if (hipMalloc(reinterpret_cast<void**>(&t->part), need * sizeof(double)) != hipSuccess) {
                    set_error("transfer: partial-sum buffer allocation failed");
                    return 1;
                }
                t->part_n = need;
            }
            part = t->part;
        }
        return transfer_pass_launch(restrict_dir, t->ncm, ps, t->Pm[d], in, out, st, part);
    }
    return restrict_dir ? transfer_band_launch(true, ps, t->Rb[d], t->ilo[d], t->wR[d], in, out, st)
                        : transfer_band_launch(false, ps, t->Pb[d], t->jlo[d], t->wP[d], in, out, st);
}

int poms_restrict(poms_transfer* t, const double* fine, double* coarse, void* stream) {
    if (!t || !fine || !coarse) { set_error("poms_restrict: null argument"); return 1; }
    const RowGeom g = row_geom(&t->L);
    const int64_t n0 = g.n0, n1 = g.n1, n2 = g.n2;
    const int64_t c0 = t->nc[0], c1 = t->nc[1], c2 = t->nc[2];
    hipStream_t st = as_stream(stream);
    const int64_t fbase = (int64_t)g.pd0 * g.s0 + (int64_t)g.pd1 * g.s1 + g.pd2;
    const double* src1;  // input of the axis-1 pass (dense [c0][n1][n2] or the fine vector)
    AxisPass a1{};
    if (t->ndim == 3) {
        AxisPass a0{};
        a0.nA = 1; a0.nB1 = n1; a0.nB2 = n2;
        a0.in_base = fbase; a0.in_sb1 = g.s1; a0.in_sb2 = 1; a0.in_si = g.s0;
        a0.out_sb1 = n2; a0.out_sb2 = 1; a0.out_si = n1 * n2;
        a0.nI = (int)n0; a0.nJ = (int)c0; a0.goff = (int)t->g0;
        if (tpass(t, true, 0, a0, fine, t->t0, st)) return 1;
        src1 = t->t0;
        a1.nA = c0; a1.nB1 = 1; a1.nB2 = n2;
        a1.in_base = 0; a1.in_sa = n1 * n2; a1.in_sb2 = 1; a1.in_si = n2;
    } else {
        src1 = fine;
        a1.nA = 1; a1.nB1 = 1; a1.nB2 = n2;
        a1.in_base = fbase; a1.in_sb2 = 1; a1.in_si = g.s1;
    }
    a1.out_sa = c1 * n2; a1.out_sb2 = 1; a1.out_si = n2;
    a1.nI = (int)n1; a1.nJ = (int)c1; a1.goff = 0;
    if (tpass(t, true, 1, a1, src1, t->t1, st)) return 1;
    AxisPass a2{};
    a2.nA = c0 * c1; a2.nB1 = 1; a2.nB2 = 1;
    a2.in_sa = n2; a2.in_si = 1;
    a2.out_sa = c2; a2.out_si = 1;
    a2.nI = (int)n2; a2.nJ = (int)c2; a2.goff = 0;
    if (tpass(t, true, 2, a2, t->t1, coarse, st)) return 1;
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_prolong_add(poms_transfer* t, const double* coarse, double* fine, void* stream) {
    if (!t || !fine || !coarse) { set_error("poms_prolong_add: null argument"); return 1; }
    const RowGeom g = row_geom(&t->L);
    const int64_t n0 = g.n0, n1 = g.n1, n2 = g.n2;
    const int64_t c0 = t->nc[0], c1 = t->nc[1], c2 = t->nc[2];
    hipStream_t st = as_stream(stream);
    const int64_t fbase = (int64_t)g.pd0 * g.s0 + (int64_t)g.pd1 * g.s1 + g.pd2;
    // axis 2: coarse [c0*c1][c2] -> t1 [c0*c1][n2]
    AxisPass a2{};
    a2.nA = c0 * c1; a2.nB1 = 1; a2.nB2 = 1;
    a2.in_sa = c2; a2.in_si = 1; a2.nJ = (int)c2;
    a2.out_sa = n2; a2.out_si = 1; a2.nI = (int)n2; a2.goff = 0; a2.accumulate = 0;
    if (tpass(t, false, 2, a2, coarse, t->t1, st)) return 1;
    // axis 1: t1 [c0][c1][n2] -> t0 [c0][n1][n2] (3D) or fine (2D, accumulate)
    AxisPass a1{};
    a1.nA = c0; a1.nB1 = 1; a1.nB2 = n2;
    a1.in_sa = c1 * n2; a1.in_sb2 = 1; a1.in_si = n2; a1.nJ = (int)c1;
    a1.nI = (int)n1; a1.goff = 0;
    if (t->ndim == 3) {
        a1.out_sa = n1 * n2; a1.out_sb2 = 1; a1.out_si = n2; a1.accumulate = 0;
        if (tpass(t, false, 1, a1, t->t1, t->t0, st)) return 1;
        AxisPass a0{};
        a0.nA = 1; a0.nB1 = n1; a0.nB2 = n2;
        a0.in_sb1 = n2; a0.in_sb2 = 1; a0.in_si = n1 * n2; a0.nJ = (int)c0;
        a0.out_base = fbase; a0.out_sb1 = g.s1; a0.out_sb2 = 1; a0.out_si = g.s0;
        a0.nI = (int)n0; a0.goff = (int)t->g0; a0.accumulate = 1;
        if (tpass(t, false, 0, a0, t->t0, fine, st)) return 1;
    } else {
        a1.out_base = fbase; a1.out_sb2 = 1; a1.out_si = g.s1; a1.accumulate = 1;
        if (tpass(t, false, 1, a1, t->t1, fine, st)) return 1;
    }
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- fused residual -> restriction ------------------------------------------------
// G[r] are HOST dense row-major (rows of axis d x nc_d) matrices F_r^T P_d, one per
// operator role in poms_op_create's factor order (A0 M0 A1 B1 M2 K2 for FORM_SUM,
// F0 - F1 - F2 - for FORM_SINGLE; 2D: roles 0, 1 unused).  Rows as P's: axis 0 global
// (3D), axes 1 and 2 the transfer's own.
int poms_transfer_set_operator(poms_transfer* t, int form, const double* const* G) {
    if (!t || !G || (form != FORM_SUM && form != FORM_SINGLE)) {
        set_error("poms_transfer_set_operator: bad argument");
        return 1;
    }
    if (t->banded) { set_error("poms_transfer_set_operator: coarse extents > 32 (banded transfer)"); return 1; }
    const bool is3d = t->ndim == 3;
    const bool sum = form == FORM_SUM;
    int64_t ncmax = 1;
    for (int d = 0; d < 3; ++d) ncmax = std::max(ncmax, t->nc[d]);
    const int ncf = ncmax <= 8 ? 8 : ncmax <= 12 ? 12 : ncmax <= 16 ? 16 : 32;
    for (int r = 0; r < 6; ++r) {
        const bool need = (r / 2 > 0 || is3d) && (sum || r % 2 == 0);
        if (need && !G[r]) { set_error("poms_transfer_set_operator: missing factor"); return 1; }
    }
    POMS_HIP_CHECK(hipSetDevice(t->ctx->device));
    for (double*& p : t->Gf) { if (p) (void)hipFree(p); p = nullptr; }
    for (double*& p : t->Pf) { if (p) (void)hipFree(p); p = nullptr; }
    if (t->ru) (void)hipFree(t->ru);
    if (t->rv) (void)hipFree(t->rv);
    t->ru = t->rv = nullptr;
    t->rform = -1;
    int rc = 0;
    auto pad = [&](const double* src, int d, double sign, double** dev) {
        std::vector<double> m(t->nf[d] * ncf, 0.0);
        for (int64_t i = 0; i < t->nf[d]; ++i)
            for (int64_t j = 0; j < t->nc[d]; ++j) m[i * ncf + j] = sign * src[i * t->nc[d] + j];
        return upload(m.data(), m.size(), dev);
    };
    for (int r = 0; r < 6 && !rc; ++r) {
        const int d = r / 2;
        if ((d == 0 && !is3d) || !G[r] || (!sum && r % 2)) continue;
        rc |= pad(G[r], d, d == 2 ? -1.0 : 1.0, &t->Gf[r]);
    }
    // P padded to ncf: the transfer keeps only its own (16 / 32-column) copy on the device
    for (int d = is3d ? 0 : 1; d < 3 && !rc; ++d) {
        std::vector<double> pm(t->nf[d] * t->ncm);
        if (hipMemcpy(pm.data(), t->Pm[d], pm.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
            rc = 1;
            break;
        }
        std::vector<double> pc(t->nf[d] * t->nc[d]);
        for (int64_t i = 0; i < t->nf[d]; ++i)
            for (int64_t j = 0; j < t->nc[d]; ++j) pc[i * t->nc[d] + j] = pm[i * t->ncm + j];
        rc |= pad(pc.data(), d, 1.0, &t->Pf[d]);
    }
    const int64_t n1 = t->L.n[1], n2 = t->L.n[2];
    const size_t su = (size_t)t->nc[0] * n1 * n2, sv = (size_t)t->nc[0] * t->nc[1] * n2;
    if (!rc && hipMalloc(reinterpret_cast<void**>(&t->ru), 3 * std::max<size_t>(su, 1) * sizeof(double)) != hipSuccess) rc = 1;
    if (!rc && hipMalloc(reinterpret_cast<void**>(&t->rv), 3 * std::max<size_t>(sv, 1) * sizeof(double)) != hipSuccess) rc = 1;
    if (rc) {
        if (g_err.empty()) set_error("poms_transfer_set_operator: allocation failed");
        return 1;
    }
    t->ncf = ncf;
    t->rform = form;
    return 0;
}

static int mpass(poms_transfer* t, const MultiPass& mp, hipStream_t st) {
    const int64_t need = mrestrict_scratch(mp, t->ncf);
    if (need > t->mpart_n) {
        if (t->mpart) (void)hipFree(t->mpart);
        t->mpart = nullptr;
        t->mpart_n = 0;
        if (hipMalloc(reinterpret_cast<void**>(&t->mpart), need * sizeof(double)) != hipSuccess) {
            set_error("resid_restrict: partial-sum buffer allocation failed");
            return 1;
        }
        t->mpart_n = need;
    }
    return mrestrict_launch(t->ncf, mp, t->mpart, st);
}

// coarse = R (b - A x), local slab contribution (the caller all-reduces).  Three
// passes (2D: two); the FORM_SUM factorisation shares its axis-0 and axis-1 outputs:
//   u_a = G_A0 x, u_m = G_M0 x, u_c = P0 b                          (axis 0)
//   v_1 = G_A1 u_a + G_B1 u_m, v_2 = G_A1 u_m, v_3 = P1 u_c           (axis 1)
//   coarse = P2 v_3 - G_M2 v_1 - G_K2 v_2                            (axis 2)
// since A = A0 (x) A1 (x) M2 + M0 (x) B1 (x) M2 + M0 (x) A1 (x) K2 (2D: A1 (x) M2 +
// B1 (x) K2; FORM_SINGLE: F0 (x) F1 (x) F2).  x needs no ghost planes: each fine
// row enters through its own row of G.
int poms_resid_restrict(poms_transfer* t, const double* b, const double* x, double* coarse, void* stream) {
    if (!t || !b || !x || !coarse) { set_error("poms_resid_restrict: null argument"); return 1; }
    if (t->rform < 0) { set_error("poms_resid_restrict: no operator set (poms_transfer_set_operator)"); return 1; }
    const RowGeom g = row_geom(&t->L);
    const int64_t n0 = g.n0, n1 = g.n1, n2 = g.n2;
    const int64_t c0 = t->nc[0], c1 = t->nc[1], c2 = t->nc[2];
    hipStream_t st = as_stream(stream);
    const int64_t fbase = (int64_t)g.pd0 * g.s0 + (int64_t)g.pd1 * g.s1 + g.pd2;
    const bool sum = t->rform == FORM_SUM;
    const size_t su = (size_t)c0 * n1 * n2, sv = (size_t)c0 * c1 * n2;
    double* u[3] = {t->ru, t->ru + su, t->ru + 2 * su};
    double* v[3] = {t->rv, t->rv + sv, t->rv + 2 * sv};
    double* const* G = t->Gf;
    auto clear = [](MultiPass& mp) {
        mp = MultiPass{};
    };
    // the axis-2 pass (the last) reads w[0..2] with w[0] = the P-chain of b
    auto last = [&](const double* wb, const double* w1, const double* w2, const AxisPass& a2) {
        MultiPass mp;
        clear(mp);
        mp.ps = a2;
        mp.ni = sum ? 3 : 2;
        mp.no = 1;
        mp.in[0] = wb; mp.in[1] = w1; mp.in[2] = sum ? w2 : nullptr;
        mp.out[0] = coarse;
        mp.m[0][0] = t->Pf[2];
        mp.m[0][1] = G[4];
        mp.m[0][2] = sum ? G[5] : nullptr;
        return mpass(t, mp, st);
    };
    AxisPass a2{};
    a2.nA = c0 * c1; a2.nB1 = 1; a2.nB2 = 1;
    a2.in_sa = n2; a2.in_si = 1;
    a2.out_sa = c2; a2.out_si = 1;
    a2.nI = (int)n2; a2.nJ = (int)c2; a2.goff = 0;
    if (t->ndim == 3) {
        MultiPass mp;
        clear(mp);
        AxisPass& a0 = mp.ps;
        a0.nA = 1; a0.nB1 = n1; a0.nB2 = n2;
        a0.in_base = fbase; a0.in_sb1 = g.s1; a0.in_sb2 = 1; a0.in_si = g.s0;
        a0.out_sb1 = n2; a0.out_sb2 = 1; a0.out_si = n1 * n2;
        a0.nI = (int)n0; a0.nJ = (int)c0; a0.goff = (int)t->g0;
        mp.ni = 2;
        mp.in[0] = x; mp.in[1] = b;
        // outputs: u_c (b), u_a, [u_m]
        mp.no = sum ? 3 : 2;
        mp.out[0] = u[0]; mp.out[1] = u[1]; mp.out[2] = u[2];
        mp.m[0][1] = t->Pf[0];
        mp.m[1][0] = G[0];
        if (sum) mp.m[2][0] = G[1];
        if (mpass(t, mp, st)) return 1;
        MultiPass m1;
        clear(m1);
        AxisPass& a1 = m1.ps;
        a1.nA = c0; a1.nB1 = 1; a1.nB2 = n2;
        a1.in_base = 0; a1.in_sa = n1 * n2; a1.in_sb2 = 1; a1.in_si = n2;
        a1.out_sa = c1 * n2; a1.out_sb2 = 1; a1.out_si = n2;
        a1.nI = (int)n1; a1.nJ = (int)c1; a1.goff = 0;
        m1.ni = sum ? 3 : 2;
        m1.in[0] = u[0]; m1.in[1] = u[1]; m1.in[2] = u[2];
        m1.no = sum ? 3 : 2;
        m1.out[0] = v[0]; m1.out[1] = v[1]; m1.out[2] = v[2];
        m1.m[0][0] = t->Pf[1];              // v_3 (here v[0]) = P1 u_c
        m1.m[1][1] = G[2];                  // v_1 = G_A1 u_a + G_B1 u_m
        if (sum) {
            m1.m[1][2] = G[3];
            m1.m[2][2] = G[2];              // v_2 = G_A1 u_m
        }
        if (mpass(t, m1, st)) return 1;
        if (last(v[0], v[1], v[2], a2)) return 1;
    } else {
        MultiPass mp;
        clear(mp);
        AxisPass& a1 = mp.ps;
        a1.nA = 1; a1.nB1 = 1; a1.nB2 = n2;
        a1.in_base = fbase; a1.in_sb2 = 1; a1.in_si = g.s1;
        a1.out_sa = c1 * n2; a1.out_sb2 = 1; a1.out_si = n2;
        a1.nI = (int)n1; a1.nJ = (int)c1; a1.goff = 0;
        mp.ni = 2;
        mp.in[0] = x; mp.in[1] = b;
        mp.no = sum ? 3 : 2;
        mp.out[0] = v[0]; mp.out[1] = v[1]; mp.out[2] = v[2];
        mp.m[0][1] = t->Pf[1];              // P1 b
        mp.m[1][0] = G[2];                  // G_A1 x (-> M2)
        if (sum) mp.m[2][0] = G[3];         // G_B1 x (-> K2)
        if (mpass(t, mp, st)) return 1;
        if (last(v[0], v[1], v[2], a2)) return 1;
    }
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_dense_matvec(poms_ctx* ctx, int64_t n, const double* Minv, const double* x, double* y,
                      void* stream) {
    if (!ctx || !Minv || !x || !y || n < 1 || n > (1 << 20)) { set_error("dense_matvec: bad argument"); return 1; }
    dense_matvec_launch((int)n, Minv, x, y, as_stream(stream));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

// ---- Kronecker direct solve (banded LU line solves) ---------------------------
int poms_ksolve_destroy(poms_ksolve* ks) {
    if (!ks) return 0;
    for (int d = 0; d < 3; ++d) {
        if (ks->Ld[d]) (void)hipFree(ks->Ld[d]);
        if (ks->Ud[d]) (void)hipFree(ks->Ud[d]);
        if (ks->pivd[d]) (void)hipFree(ks->pivd[d]);
    }
    delete ks;
    return 0;
}

int poms_ksolve_create(poms_ctx* ctx, int ndim, const poms_layout* layout, int64_t n0_global,
                       const double* const* ab, const int64_t* ldab, const int* kl, const int* ku,
                       poms_ksolve** out) {
    if (!layout) { set_error("poms_ksolve_create: bad argument"); return 1; }
    const int64_t ng[3] = {n0_global, layout->n[1], layout->n[2]};
    return poms_ksolve_create_global(ctx, ndim, layout, ng, ab, ldab, kl, ku, out);
}

int poms_ksolve_create_global(poms_ctx* ctx, int ndim, const poms_layout* layout, const int64_t* n_global,
                              const double* const* ab, const int64_t* ldab, const int* kl, const int* ku,
                              poms_ksolve** out) {
    if (!ctx || !out || !ab || !ldab || !kl || !ku || !n_global || !layout_ok(layout)) {
        set_error("poms_ksolve_create: bad argument");
        return 1;
    }
    const int64_t n0_global = n_global[0];
    if (ndim < 1 || ndim > 3) { set_error("poms_ksolve_create: ndim 1..3"); return 1; }
    const int d0 = 3 - ndim;
    for (int d = 0; d < d0; ++d)
        if (layout->n[d] != 1 || layout->pads[d] != 0) {
            set_error("poms_ksolve_create: unused leading axes need n = 1, pads = 0");
            return 1;
        }
    if (ndim == 3 && n0_global < layout->n[0]) { set_error("poms_ksolve_create: n0_global < local n0"); return 1; }
    for (int d = 1; d < 3; ++d)
        if (d >= d0 && n_global[d] < layout->n[d]) { set_error("poms_ksolve_create: global extent < local extent"); return 1; }
    for (int d = d0; d < 3; ++d) {
        if (!ab[d] || kl[d] < 0 || ku[d] < 0 || ldab[d] < 2 * kl[d] + ku[d] + 1) {
            set_error("poms_ksolve_create: bad band of axis " + std::to_string(d));
            return 1;
        }
        if (kl[d] + ku[d] > 16) { set_error("poms_ksolve_create: kl + ku must be <= 16"); return 1; }
    }
    POMS_HIP_CHECK(hipSetDevice(ctx->device));
    auto* ks = new poms_ksolve();
    ks->ctx = ctx;
    ks->ndim = ndim;
    ks->L = *layout;
    ks->n0g = ndim == 3 ? n0_global : 1;
    for (int d = 0; d < 3; ++d) ks->ng[d] = d < d0 ? 1 : d == 0 ? ks->n0g : n_global[d];
    int rc = 0;
    for (int d = d0; d < 3 && !rc; ++d) {
        const int64_t n = ks->ng[d];
        std::vector<double> band(ab[d], ab[d] + ldab[d] * n);
        ks->ipiv[d].assign((size_t)n, 0);
        ks->info[d] = band_lu(n, kl[d], ku[d], band.data(), ldab[d], ks->ipiv[d].data());
        ks->kl[d] = kl[d];
        ks->ku[d] = ku[d];
        std::vector<double> Lt, Ut;
        std::vector<int> pt;
        band_lu_tables(n, kl[d], ku[d], band.data(), ldab[d], ks->ipiv[d].data(), Lt, Ut, pt);
        rc |= upload(Lt.data(), Lt.size(), &ks->Ld[d]);
        rc |= upload(Ut.data(), Ut.size(), &ks->Ud[d]);
        if (!rc && hipMalloc(reinterpret_cast<void**>(&ks->pivd[d]), pt.size() * sizeof(int)) != hipSuccess) rc = 1;
        if (!rc && hipMemcpy(ks->pivd[d], pt.data(), pt.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
            rc = 1;
        ks->f[d] = BandLU{ks->Ld[d], ks->Ud[d], ks->pivd[d], (int)n, kl[d], kl[d] + ku[d]};
    }
    if (rc) {
        if (g_err.empty()) set_error("poms_ksolve_create: allocation failed");
        poms_ksolve_destroy(ks);
        return 1;
    }
    *out = ks;
    return 0;
}

int poms_ksolve_info(poms_ksolve* ks, int* info) {
    if (!ks || !info) { set_error("poms_ksolve_info: bad argument"); return 1; }
    for (int d = 0; d < 3; ++d) info[d] = ks->info[d];
    return 0;
}

int poms_ksolve_pivots(poms_ksolve* ks, int axis, int* ipiv) {
    if (!ks || !ipiv || axis < 3 - ks->ndim || axis > 2) { set_error("poms_ksolve_pivots: bad argument"); return 1; }
    std::copy(ks->ipiv[axis].begin(), ks->ipiv[axis].end(), ipiv);
    return 0;
}

static int ksolve_axis(poms_ksolve* ks, int axis, const double* in, double* out, hipStream_t st) {
    if (ks->info[axis] != 0) {
        set_error("kron solve: factor of axis " + std::to_string(axis) + " is singular (info " +
                  std::to_string(ks->info[axis]) + ")");
        return 1;
    }
    if (ks->L.n[axis] != ks->ng[axis]) {
        set_error("kron solve: axis " + std::to_string(axis) +
                  " is distributed; solve its transposed lines with poms_kron_solve_lines_dense");
        return 1;
    }
    const RowGeom g = row_geom(&ks->L);
    const int64_t base = g.pd0 * g.s0 + g.pd1 * g.s1 + g.pd2;
    int rc = 0;
    if (axis == 2) {
        RowLines r{base, g.s0, g.s1, g.n1, (int64_t)g.n0 * g.n1};
        rc = ksolve_rows_launch(r, ks->f[2], in, out, st);
    } else if (axis == 1) {
        LineGeom lg{base, g.s0, g.s1, g.n0, g.n2};
        rc = ksolve_strided_launch(lg, ks->f[1], in, out, st);
    } else {
        if (ks->L.n[0] != ks->n0g) {
            set_error("kron solve: axis 0 is distributed; use poms_kron_solve_axis0_dense on transposed data");
            return 1;
        }
        LineGeom lg{base, g.s1, g.s0, g.n1, g.n2};
        rc = ksolve_strided_launch(lg, ks->f[0], in, out, st);
    }
    if (rc) return rc;
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_kron_solve_axis(poms_ksolve* ks, int axis, const double* in, double* out, void* stream) {
    if (!ks || !in || !out || axis < 3 - ks->ndim || axis > 2) { set_error("poms_kron_solve_axis: bad argument"); return 1; }
    return ksolve_axis(ks, axis, in, out, as_stream(stream));
}

int poms_kron_solve(poms_ksolve* ks, const double* y, double* x, void* stream) {
    if (!ks || !y || !x) { set_error("poms_kron_solve: bad argument"); return 1; }
    const double* src = y;
    for (int d = 3 - ks->ndim; d < 3; ++d) {
        if (ksolve_axis(ks, d, src, x, as_stream(stream))) return 1;
        src = x;
    }
    return 0;
}

int poms_kron_solve_axis0_dense(poms_ksolve* ks, const double* in, double* out, int64_t m, void* stream) {
    if (!ks || ks->ndim != 3) { set_error("poms_kron_solve_axis0_dense: bad argument"); return 1; }
    return poms_kron_solve_lines_dense(ks, 0, in, out, m, stream);
}

int poms_kron_solve_lines_dense(poms_ksolve* ks, int axis, const double* in, double* out, int64_t m, void* stream) {
    if (!ks || !in || !out || m < 0 || axis < 3 - ks->ndim || axis > 2) {
        set_error("poms_kron_solve_lines_dense: bad argument");
        return 1;
    }
    if (ks->info[axis] != 0) { set_error("kron solve: factor of axis " + std::to_string(axis) + " is singular"); return 1; }
    if (m == 0) return 0;
    // m lines of ng[axis] points, line j at column j of a dense C-order (ng, m) buffer
    LineGeom lg{0, 0, m, 1, m};
    if (ksolve_strided_launch(lg, ks->f[axis], in, out, as_stream(stream))) return 1;
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

// host drop-in of kron_solve_par_bnd_pyccel_2d / _3d on one rank
static int kron_solve_bnd_host(poms_ctx* ctx, int ndim, const double* const* bands, const int64_t* ld,
                               const int* kl, const int* ku, double* X, const double* Y,
                               const int64_t* points, const int64_t* pads) {
    if (!ctx || !X || !Y || !points || !pads) { set_error("poms_kron_solve_bnd: null argument"); return 1; }
    const int d0 = 3 - ndim;
    poms_layout L{{1, 1, 1}, {0, 0, 0}, 0};
    for (int d = d0; d < 3; ++d) {
        L.n[d] = points[d - d0];
        L.pads[d] = pads[d - d0];
        if (!bands[d]) { set_error("poms_kron_solve_bnd: null band"); return 1; }
    }
    poms_ksolve* ks = nullptr;
    if (poms_ksolve_create(ctx, ndim, &L, L.n[0], bands, ld, kl, ku, &ks)) return 1;
    const RowGeom g = row_geom(&L);
    const size_t nel = (size_t)(L.n[0] + 2 * L.pads[0]) * g.s0;
    double *dx = nullptr, *dy = nullptr;
    int rc = 0;
    if (hipMalloc(reinterpret_cast<void**>(&dx), nel * sizeof(double)) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&dy), nel * sizeof(double)) != hipSuccess) {
        set_error("poms_kron_solve_bnd: hipMalloc failed");
        rc = 1;
    }
    if (!rc && (hipMemcpy(dx, X, nel * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(dy, Y, nel * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)) {
        set_error("poms_kron_solve_bnd: upload failed");
        rc = 1;
    }
    if (!rc) rc = poms_kron_solve(ks, dy, dx, nullptr);
    if (!rc && hipMemcpy(X, dx, nel * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
        set_error("poms_kron_solve_bnd: download failed");
        rc = 1;
    }
    if (dx) (void)hipFree(dx);
    if (dy) (void)hipFree(dy);
    poms_ksolve_destroy(ks);
    return rc;
}

int poms_kron_solve_bnd_2d(poms_ctx* ctx, const double* A_bnd, int64_t lda, int la, int ua,
                           const double* B_bnd, int64_t ldb, int lb, int ub, double* X, const double* Y,
                           const int64_t* points, const int64_t* pads) {
    const double* bands[3] = {nullptr, A_bnd, B_bnd};
    const int64_t ld[3] = {1, lda, ldb};
    const int kl[3] = {0, la, lb}, ku[3] = {0, ua, ub};
    return kron_solve_bnd_host(ctx, 2, bands, ld, kl, ku, X, Y, points, pads);
}

int poms_kron_solve_bnd_3d(poms_ctx* ctx, const double* A_bnd, int64_t lda, int la, int ua,
                           const double* B_bnd, int64_t ldb, int lb, int ub, const double* C_bnd,
                           int64_t ldc, int lc, int uc, double* X, const double* Y,
                           const int64_t* points, const int64_t* pads) {
    const double* bands[3] = {A_bnd, B_bnd, C_bnd};
    const int64_t ld[3] = {lda, ldb, ldc};
    const int kl[3] = {la, lb, lc}, ku[3] = {ua, ub, uc};
    return kron_solve_bnd_host(ctx, 3, bands, ld, kl, ku, X, Y, points, pads);
}

}  // extern "C"

// ---- native pcg + damped-Jacobi loop (poms_pcg_jacobi) ------------------------
// The V-cycle's smoother (`sources/mg_jac.py:88,104` -> `sources/solvers.py:69-135`
// with psolve = damped_jacobi, :167-235) as one C call: the same launches, device
// scalars and stop tests as poms_amd.solvers._pcg_device, without a Python round
// trip per launch.  The host reads a norm one launch after queuing the next one
// (the GPU never waits for the host while the host waits for that norm).
namespace {

// device scalars (the sums only the host reads live in host slots / comm ring slots)
enum { SC_SR = 0, SC_PQ = 1, SC_ONE = 2, SC_ALPHA = 3, SC_ALPHA2 = 4, SC_BETA = 5, SC_SRN = 6, SC_N = 16 };
enum { H_RR0 = 0, H_RR = 1, H_J0 = 2 /* 2 slots */, H_JN = 4 /* 2 slots */ };
// an unwritten partial in a host region: a NaN payload no reduction produces
constexpr uint64_t kPartUnset = 0x7ff8dead0000beefull;

__global__ void pcg_scalars_kernel(double* sc, int mode) {
    if (threadIdx.x != 0) return;
    if (mode == 0) {            // alpha = s.r / p.q; pairs [1, alpha] and [alpha, beta]
        const double a = sc[SC_SR] / sc[SC_PQ];
        sc[SC_ONE] = 1.0;
        sc[SC_ALPHA] = a;
        sc[SC_ALPHA2] = a;
    } else {                    // beta = s.r / s.r_old; s.r_old <- s.r
        sc[SC_BETA] = sc[SC_SRN] / sc[SC_SR];
        sc[SC_SR] = sc[SC_SRN];
    }
}

// p.q from the apply + dot launch's per-block partials -- reduce_partials_kernel's
// order, so the same bits -- and alpha from it, in one launch (one rank: saves the
// one-block reduction launch per pcg iteration)
__global__ void __launch_bounds__(256) pcg_alpha_kernel(const double* __restrict__ part, int count, double* sc) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < count; i += 256) s += part[i];
    const double pq = block_sum_256(s, red);
    if (threadIdx.x != 0) return;
    sc[SC_PQ] = pq;
    const double a = sc[SC_SR] / pq;
    sc[SC_ONE] = 1.0;
    sc[SC_ALPHA] = a;
    sc[SC_ALPHA2] = a;
}

// s.r_new from the last damped-Jacobi sweep's per-block partials (reduce_partials_kernel's
// order: the same bits), then beta = s.r_new / s.r_old and s.r_old <- s.r_new, in one
// launch (one rank: saves the one-block reduction launch per pcg iteration)
// s.r_old <- s.r_new, where a beta folded into the x/p update left it pending and no
// folded r update follows (AlphaFold)
__global__ void pcg_sr_fix_kernel(double* sc) {
    if (threadIdx.x == 0) sc[SC_SR] = sc[SC_SRN];
}

__global__ void __launch_bounds__(256) pcg_beta_kernel(const double* __restrict__ part, int count, double* sc) {
    __shared__ double red[4];
    double s = 0.0;
    for (int i = threadIdx.x; i < count; i += 256) s += part[i];
    const double srn = block_sum_256(s, red);
    if (threadIdx.x != 0) return;
    sc[SC_SRN] = srn;
    sc[SC_BETA] = srn / sc[SC_SR];
    sc[SC_SR] = srn;
}

struct PcgRun {
    poms_op* op;
    poms_comm* comm;
    const poms_pcg_opts* o;
    hipStream_t st;
    void* stv;
    double* sc;
    double* host;
    int64_t n0 = 1;

    int run(int epi, const double* x, double* y, const double* b, double* nrm, double* dot) {
        if (comm) {
            const RowGeom g = row_geom(&op->L);
            int tk = -1;
            return poms_op_run_dist(op, comm, epi, o->omega, x, y, b, const_cast<double*>(x), g.s0, op->L.n[0],
                                    (int)op->L.pads[0], op->pmax, o->prev, o->next, 1, nrm ? 1 : 0, dot ? 1 : 0, nrm,
                                    dot, 0, nullptr, &tk, stv);
        }
        return poms_op_run_reduce2(op, epi, o->omega, x, y, b, 0, n0, 0, 0, nrm, dot, 0, stv);
    }
    // q = A p, p.q and alpha: one rank folds p.q's reduction into the alpha kernel
    int apd_alpha(const double* p, double* q) {
        if (comm || op->dot_base >= 0 || op->part_off != 0 || op->part_dst || op->form == FORM_STENCIL) {
            if (run(EPI_APPLYDOT, p, q, p, nullptr, sc + SC_PQ) || allsum(sc + SC_PQ, 1)) return 1;
            hipLaunchKernelGGL(pcg_scalars_kernel, dim3(1), dim3(64), 0, st, sc, 0);
            POMS_HIP_CHECK(hipGetLastError());
            return 0;
        }
        if (op_run_epi(op, EPI_APPLYDOT, o->omega, p, q, p, 0, n0, 0, 0, false, true, stv)) return 1;
        const int64_t n = op->last_partials;   // (the dot's partials at scratch + n, as poms_op_run_reduce2 reads them)
        // alpha is formed by the r update that follows (rupd: AlphaFold), or by
        // pcg_alpha_kernel when that cannot take it (flush_alpha)
        alpha_part = op->ctx->scratch + n;
        alpha_n = n;
        return 0;
    }
    const double* alpha_part = nullptr;   // p.q's partials awaiting alpha (apd_alpha)
    int64_t alpha_n = 0;
    bool sr_stale = false;                // a folded beta left s.r_old <- s.r_new pending
    int fix_sr() {
        if (!sr_stale) return 0;
        hipLaunchKernelGGL(pcg_sr_fix_kernel, dim3(1), dim3(64), 0, st, sc);
        sr_stale = false;
        POMS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    static bool fold_on() {   // POMS_ALPHA_FOLD=0: the one-block scalar kernels (tuning / A-B)
        static const bool f = !(getenv("POMS_ALPHA_FOLD") && getenv("POMS_ALPHA_FOLD")[0] == '0');
        return f;
    }
    // beta folded into the x/p update: x += alpha p, p = s + beta p with beta from the
    // last sweep's x . rhs partials (dot_part); 1 if it cannot (the caller runs
    // pcg_beta_kernel and the plain update), -1 on error
    int xpupd_beta(double* x, double* p, const double* s) {
        if (!fold_on() || !direct() || (op->L.flags & POMS_LAYOUT_GHOST_DATA) || dot_part_n < 0) return 1;
        const RowGeom g = row_geom(&op->L);
        const int64_t off = (int64_t)g.pd0 * g.s0, count = (int64_t)g.n0 * g.s0;
        const int head = (reinterpret_cast<uintptr_t>(x + off) & 15) ? 1 : 0;
        const int64_t nbp = std::max<int64_t>(1, ((count - head) / 2 + 1023) / 1024);
        if (dot_part_n * nbp > (int64_t)1 << 20) return 1;
        if (fix_sr()) return -1;   // (beta reads s.r_old at sc[SC_SR])
        AlphaFold bf;
        bf.part = dot_part;
        bf.n = (int)dot_part_n;
        bf.sc = sc;
        static_assert(SC_SR == 0 && SC_BETA == 5 && SC_SRN == 6, "AlphaFold's beta slots");
        int nb = 0;
        if (vec_flat_launch(V_XPUPD, count, 0.0, 0.0, s + off, nullptr, x + off, p + off, nullptr, nullptr, st, &nb,
                            sc + SC_ALPHA2, &bf) != 0)
            return 1;
        if (hipGetLastError() != hipSuccess) { set_error("x/p update with beta: launch failed"); return -1; }
        sr_stale = true;
        return 0;
    }
    int flush_alpha() {
        if (fix_sr()) return 1;
        if (!alpha_part) return 0;
        hipLaunchKernelGGL(pcg_alpha_kernel, dim3(1), dim3(256), 0, st, alpha_part, (int)alpha_n, sc);
        alpha_part = nullptr;
        POMS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    // the last sweep of a psolve left x . rhs as per-block partials (dot_part, dot_part_n
    // blocks) for pcg_beta_kernel instead of reducing them itself (-1: it did not)
    const double* dot_part = nullptr;
    int64_t dot_part_n = -1;
    int tk[poms_op::kSvRing] = {};   // with a communicator: the ring ticket of host slot h
    // a sum the device needs (alpha, beta): all-reduced, the compute stream waits
    int allsum(double* d, int cnt) { return comm ? poms_allreduce_sum(comm, d, cnt, stv, 1) : 0; }
    // A value only the host reads: one rank -- the reduction kernel writes it straight
    // into the pinned (coherent, device-mapped) host slot, armed with a sentinel the
    // host spins on (~1-2 us after the kernel instead of an event wake-up, ~15 us:
    // profiles/r02/sync_probe.log); with a communicator -- a ring slot of the
    // communicator, all-reduced and copied to the host slot on the communication
    // stream while the compute stream goes on (lazy_post; the compute stream used to
    // wait for that all-reduce and copy, ~40 us per sweep in profiles/r03/proxy/).
    bool direct() const { return comm == nullptr; }
    double* hslot(int h) {
        if (direct()) return host + h;
        double* d = nullptr;
        if (poms_comm_slot(comm, &d, &tk[h])) return nullptr;
        return d;
    }
    int lazy_post(int h, int cnt) { return direct() ? 0 : poms_allreduce_to_host(comm, tk[h], cnt, host + h, stv); }
    // an operator launch whose sums only the host reads: [dot, norm] from host slot h
    int jrun(int epi, const double* x, double* y, const double* b, bool wn, bool wd, int h) {
        if (direct()) {   // the launch writes its partials into slot h's host region
            // (up to host_partials_max() blocks).  A/B on one box
            // (profiles/r03/host_partials/): 2D 1027^2 cycle 4.5-5.2 -> 3.6-3.7 ms,
            // 3D 515^3 195.0-195.5 -> 194.9-195.3 ms
            op->part_dst = op->sv_part + (size_t)h * poms_op::kSvPart;
            op->part_cap = ((wn ? 1 : 0) + (wd ? 1 : 0)) * host_partials_max();
            const int rc = op_run_epi(op, epi, o->omega, x, y, b, 0, n0, 0, 0, wn, wd, stv);
            op->part_dst = nullptr;
            if (rc) return 1;
            const int64_t n = op->last_partials;
            if (op->last_part_host) {
                op->sv_npart[h] = (int)n;
                op->sv_pkind[h] = (wn ? 1 : 0) | (wd ? 2 : 0);
                return 0;
            }
            // too many blocks for the region: reduce on the device into the slots
            double* pdot = op->ctx->scratch + (op->dot_base < 0 ? n : op->dot_base);
            if (wn) reduce_launch(op->ctx->scratch, (int)n, host + h + (wd ? 1 : 0), st);
            if (wd) reduce_launch(pdot, (int)n, host + h, st);
            POMS_HIP_CHECK(hipGetLastError());
            return 0;
        }
        const RowGeom g = row_geom(&op->L);
        return poms_op_run_dist(op, comm, epi, o->omega, x, y, b, const_cast<double*>(x), g.s0, op->L.n[0],
                                (int)op->L.pads[0], op->pmax, o->prev, o->next, 1, wn ? 1 : 0, wd ? 1 : 0, nullptr,
                                nullptr, (wn ? 1 : 0) + (wd ? 1 : 0), host + h, &tk[h], stv);
    }
    // sweeps 1-3 from x = 0 (one rank): [||x1||^2, ||dr_2||^2, ||dr_3||^2] into slots h .. h+2
    int jrun3(const double* rhs, double* y, int h) {
        op->part_dst = op->sv_part + (size_t)h * poms_op::kSvPart;
        op->part_cap = 3 * host_partials_max();
        const int rc = op_run_epi(op, EPI_JACOBI3Z, o->omega, rhs, y, rhs, 0, n0, 0, 0, true, true, stv);
        op->part_dst = nullptr;
        if (rc) return 1;
        const int64_t n = op->last_partials;
        if (op->last_part_host) {
            op->sv_npart[h] = (int)n;
            op->sv_pkind[h] = 4;
            return 0;
        }
        for (int i = 0; i < 3; ++i) reduce_launch(op->ctx->scratch + i * n, (int)n, host + h + i, st);
        POMS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    // Arm `cnt` consecutive host slots for the next launch and return the first.
    // Direct mode takes fresh slots from a ring: a launch the loop abandoned (an
    // early damped-Jacobi stop leaves the next sweep queued) still writes ITS slot
    // later, so a slot is re-armed only once that launch is known complete -- a value
    // of a later launch has been read (launches of one stream finish in order) --
    // else the stream is drained first (advisor finding, round 2).
    int arm(int fixed_h, int cnt) {
        if (!direct()) return fixed_h;
        if (op->sv_next + cnt > poms_op::kSvRing) op->sv_next = 0;
        const int h = op->sv_next;
        op->sv_next += cnt;
        for (int i = 0; i < cnt; ++i)
            if (op->sv_seq[h + i] >= op->sv_done) {
                (void)hipStreamSynchronize(st);
                op->sv_done = op->sv_seq_next;
                break;
            }
        for (int i = 0; i < cnt; ++i) {
            reinterpret_cast<volatile double*>(host)[h + i] = -1.0;   // norms are >= 0
            op->sv_seq[h + i] = op->sv_seq_next;
            if (op->sv_npart[h + i] > 0) {   // an abandoned launch's partials (complete by now): re-arm
                part_arm(op->sv_part + (size_t)(h + i) * poms_op::kSvPart, pk_nsum(op->sv_pkind[h + i]) * op->sv_npart[h + i]);
                op->sv_npart[h + i] = 0;
                op->sv_pkind[h + i] = 0;
            }
        }
        ++op->sv_seq_next;
        return h;
    }
    static int64_t host_partials_max() {   // tuning: POMS_HOST_PARTIALS (0: always reduce on the device)
        // read per launch (a getenv against a kernel launch): the parity tests switch it
        // inside one process to run the device-reduction fall-back
        const char* e = getenv("POMS_HOST_PARTIALS");
        const int64_t m = e ? std::max<int64_t>(0, atoll(e)) : poms_op::kSvPart / 2;
        return std::min<int64_t>(m, poms_op::kSvPart / 2);
    }
    // Wait for every partial of slot h's region and add them on the host in the
    // order of reduce_partials_kernel (256 strided running sums, the 64-lane xor
    // butterfly, then (w0 + w1) + (w2 + w3)): the same bits as the device reduction.
    static double host_reduce(const double* p, int n) {
        double sv[256];
        for (int t = 0; t < 256; ++t) {
            double a = 0.0;
            for (int i = t; i < n; i += 256) a += p[i];
            sv[t] = a;
        }
        double red[4];
        for (int w = 0; w < 4; ++w) {
            double v[64], nv[64];
            for (int l = 0; l < 64; ++l) v[l] = sv[64 * w + l];
            for (int off = 32; off > 0; off >>= 1) {
                for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
                for (int l = 0; l < 64; ++l) v[l] = nv[l];
            }
            red[w] = v[0];
        }
        return (red[0] + red[1]) + (red[2] + red[3]);
    }
    int settle_partials(int h) {
        const int n = op->sv_npart[h];
        double* reg = op->sv_part + (size_t)h * poms_op::kSvPart;
        const int nsum = pk_nsum(op->sv_pkind[h]);
        for (int i = 0; i < nsum * n; ++i) {
            for (long k = 1; part_unset(reg + i); ++k) {
                __builtin_ia32_pause();
                if ((k & 4095) == 0 && hipStreamQuery(st) != hipErrorNotReady) {
                    std::atomic_thread_fence(std::memory_order_seq_cst);
                    if (part_unset(reg + i)) return 1;   // never written: the launch failed
                }
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        const bool wn = op->sv_pkind[h] & 1, wd = op->sv_pkind[h] & 2;
        if (op->sv_pkind[h] & 4) {   // three sums, slots h .. h+2 (EPI_JACOBI3Z)
            for (int i = 0; i < 3; ++i) host[h + i] = host_reduce(reg + (size_t)i * n, n);
        } else {
            if (wn) host[h + (wd ? 1 : 0)] = host_reduce(reg, n);
            if (wd) host[h] = host_reduce(reg + (wn ? n : 0), n);
        }
        part_arm(reg, nsum * n);
        op->sv_npart[h] = 0;
        op->sv_pkind[h] = 0;
        return 0;
    }
    // sums in a slot region: bit 0 a norm, bit 1 a dot, bit 2 three sums (EPI_JACOBI3Z)
    static int pk_nsum(int pk) { return (pk & 4) ? 3 : ((pk & 1) ? 1 : 0) + ((pk & 2) ? 1 : 0); }
    static bool part_unset(const double* v) {
        uint64_t u;
        const volatile uint64_t* q = reinterpret_cast<const volatile uint64_t*>(v);
        u = *q;
        return u == kPartUnset;
    }
    static void part_arm(double* v, int n) {
        volatile uint64_t* q = reinterpret_cast<volatile uint64_t*>(v);
        for (int i = 0; i < n; ++i) q[i] = kPartUnset;
    }
    // A failed wait (the shm sum timed out, a launch never wrote its sum) sets
    // `failed` and keeps poms_comm_wait's message: the loop returns 1 at its next
    // check instead of carrying a NaN into the stop tests (advisor, round 3).
    bool failed = false;
    double fail() {
        failed = true;
        return std::nan("");
    }
    double get(int h, int i = 0) {
        if (!direct()) {
            if (poms_comm_wait(comm, tk[h])) return fail();
            return host[h + i];
        }
        if (op->sv_npart[h] > 0) {
            if (settle_partials(h)) {
                set_error("poms_pcg_jacobi: a launch did not write its partial sums");
                return fail();
            }
            op->sv_done = std::max(op->sv_done, op->sv_seq[h] + 1);
            return host[h + i];
        }
        const volatile double* v = reinterpret_cast<const volatile double*>(host) + h + i;
        for (long n = 1; *v == -1.0; ++n) {
            __builtin_ia32_pause();
            if ((n & 4095) == 0 && hipStreamQuery(st) != hipErrorNotReady) {   // stream drained (or failed)
                std::atomic_thread_fence(std::memory_order_seq_cst);
                if (*v == -1.0) {   // never written: the launch failed
                    set_error("poms_pcg_jacobi: a launch did not write its sum");
                    return fail();
                }
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        op->sv_done = std::max(op->sv_done, op->sv_seq[h + i] + 1);   // that launch and all before it are done
        return *v;
    }
    int dot(const double* a, const double* b, double* dst) {
        if (poms_vec_dot(op->ctx, &op->L, a, b, dst, stv)) return 1;
        return allsum(dst, 1);
    }
    // r -= alpha q, r.r -> host slot h.  One rank: the flat kernel writes its per-block
    // partials straight into the slot's host region (the host adds them in the order
    // of the device reduction it replaces, so the same bits) -- one launch less per
    // pcg iteration
    int rupd(double* r, const double* q, int h) {
        if (direct() && !(op->L.flags & POMS_LAYOUT_GHOST_DATA)) {
            const RowGeom g = row_geom(&op->L);
            const int64_t off = (int64_t)g.pd0 * g.s0, count = (int64_t)g.n0 * g.s0;
            const int head = (reinterpret_cast<uintptr_t>(r + off) & 15) ? 1 : 0;
            const int64_t nbp = std::max<int64_t>(1, ((count - head) / 2 + 1023) / 1024);   // (vec_flat_launch's grid, before its cap)
            if (nbp <= host_partials_max()) {
                int nb = 0;
                double* reg = op->sv_part + (size_t)h * poms_op::kSvPart;
                // alpha folded into this launch where its blocks' extra reads of the
                // partials are small (2D: 468 partials x ~515 blocks; not the 3D grid's
                // 495 x 65536): one launch less per pcg iteration (round 6)
                AlphaFold af;
                static const bool fold = !(getenv("POMS_ALPHA_FOLD") && getenv("POMS_ALPHA_FOLD")[0] == '0');
                if (fold && alpha_part && alpha_n * nbp <= (int64_t)1 << 20) {
                    af.part = alpha_part;
                    af.n = (int)alpha_n;
                    af.sc = sc;
                    af.sr = sr_stale ? SC_SRN : SC_SR;   // (a folded beta's s.r_new, copied to SC_SR by block 0)
                    af.copy_sr = sr_stale ? 1 : 0;
                    static_assert(SC_SR == 0 && SC_PQ == 1 && SC_ONE == 2 && SC_ALPHA == 3 && SC_ALPHA2 == 4,
                                  "AlphaFold's slots");
                } else if (flush_alpha()) {
                    return 1;
                }
                if (vec_flat_launch(V_RUPD, count, 0.0, 0.0, nullptr, nullptr, nullptr, r + off, q + off, reg, st, &nb,
                                    sc + SC_ALPHA, af.part ? &af : nullptr) == 0) {
                    if (af.part) sr_stale = false;
                    alpha_part = nullptr;
                    POMS_HIP_CHECK(hipGetLastError());
                    op->sv_npart[h] = nb;
                    op->sv_pkind[h] = 1;
                    return 0;
                }
            }
        }
        if (flush_alpha()) return 1;
        double* d = hslot(h);
        if (!d || poms_pcg_r_update_dev(op->ctx, &op->L, sc + SC_ALPHA, r, q, d, stv) || lazy_post(h, 1)) return 1;
        return 0;
    }
    int diag_scale_norm(const double* b, double* x, int h) {   // x = omega b / diag, ||x||^2 -> host slot h
        if (direct() && op->form != FORM_STENCIL) {   // partials straight into slot h's host region
            const RowGeom g = row_geom(&op->L);
            const int nb = diag_scale_blocks(op->ndim == 3, g);
            if (nb <= host_partials_max()) {
                int nl = 0;
                diag_scale_launch(op->ndim == 3, op->form, g, op->pmax, (int)op->g0, o->omega, b, x, op->a0t,
                                  op->b0t, op->a1, op->b1, op->dg2a, op->dg2b,
                                  op->sv_part + (size_t)h * poms_op::kSvPart, st, &nl);
                POMS_HIP_CHECK(hipGetLastError());
                if (nl != nb) { set_error("diag scale: block count mismatch"); return 1; }
                op->last_partials = nb;
                op->sv_npart[h] = nb;
                op->sv_pkind[h] = 1;
                return 0;
            }
        }
        if (poms_op_diag_scale(op, o->omega, b, x, 1, stv)) return 1;
        double* d = hslot(h);
        if (!d) return 1;
        reduce_launch(op->ctx->scratch, (int)op->last_partials, d, st);
        return lazy_post(h, 1);
    }

    // ---- speculative mode (spec_*): the whole smoother call is queued without reading a
    // single stop test; every host-read sum goes to its own place (a partials region of
    // op->spec_part, or op->spec_dev[i]) and the tests are evaluated once the stream has
    // drained.  If one of them fires, the call is repeated step by step (x0 restored).
    // The launches and their order are those of the step-by-step loop when no test
    // fires, so the result is the same bits (tests/test_gpu_solvers.py).
    using SPart = SpecPart;
    std::vector<SPart> sparts;
    int64_t scur = 0;       // next free double of op->spec_part
    int sn = 0;             // next free value index
    std::vector<int> schk;  // value indices tested against jtol^2 (< fires)
    std::vector<int> srr;   // pcg r.r value index per iteration (k = 1..)
    int svals(int cnt) {
        const int i = sn;
        sn += cnt;
        return i;
    }
    // an operator launch whose sums are tested at the end: [dot, norm] at value vi
    int sjrun(int epi, const double* x, double* y, const double* b, bool wn, bool wd, int* vi_out) {
        const int cnt = (wn ? 1 : 0) + (wd ? 1 : 0);
        const int vi = svals(cnt);
        *vi_out = vi;
        double* dn = wn ? op->spec_dev + vi + (wd ? 1 : 0) : nullptr;
        double* dd = wd ? op->spec_dev + vi : nullptr;
        if (!direct()) return run(epi, x, y, b, dn, dd);
        op->part_dst = op->spec_part + scur;
        op->part_cap = poms_op::kSpecPart - scur;
        const int rc = op_run_epi(op, epi, o->omega, x, y, b, 0, n0, 0, 0, wn, wd, stv);
        op->part_dst = nullptr;
        if (rc) return 1;
        const int64_t n = op->last_partials;
        if (op->last_part_host) {
            sparts.push_back(SPart{scur, (int)n, (wn ? 1 : 0) | (wd ? 2 : 0), vi});
            scur += cnt * n;
            return 0;
        }
        double* pdot = op->ctx->scratch + (op->dot_base < 0 ? n : op->dot_base);
        if (wn) reduce_launch(op->ctx->scratch, (int)n, dn, st);
        if (wd) reduce_launch(pdot, (int)n, dd, st);
        POMS_HIP_CHECK(hipGetLastError());
        return 0;
    }
    // damped_jacobi with every sweep queued (no stop test read); as damped_jacobi below
    int spec_damped_jacobi(const double* rhs, double* A, double* B, int dot_idx, double** out) {
        const int maxit = o->jmaxiter;
        double *x = A, *xn = B;
        int fz = 0, k0;
        if (maxit >= 2 && maxit != 2 && op->form != FORM_STENCIL) (void)poms_op_from_zero_supported(op, &fz);
        if (fz) {   // sweeps 1, 2 from x = 0: [||x1||^2, ||dr2||^2]
            int vi;
            if (sjrun(EPI_JACOBI0, rhs, A, rhs, true, true, &vi)) return 1;
            schk.push_back(vi);
            schk.push_back(vi + 1);
            k0 = 3;
        } else {
            const int vi = svals(1);
            if (poms_op_diag_scale(op, o->omega, rhs, A, 1, stv)) return 1;
            reduce_launch(op->ctx->scratch, (int)op->last_partials, op->spec_dev + vi, st);   // (rank sums at the end)
            schk.push_back(vi);
            k0 = 2;
        }
        for (int k = k0; k <= maxit; ++k) {
            if (k == maxit) {   // the last sweep's norm cannot change the result: x . rhs instead
                if (run(EPI_JACOBI, x, xn, rhs, nullptr, sc + dot_idx) || allsum(sc + dot_idx, 1)) return 1;
            } else {
                int vi;
                if (sjrun(EPI_JACOBI, x, xn, rhs, true, false, &vi)) return 1;
                schk.push_back(vi);
            }
            std::swap(x, xn);
        }
        *out = x;
        return 0;
    }
    // damped_jacobi(A, rhs) with x0 = None into buffers {A, B} (and C: see below); the
    // last sweep also forms x . rhs into sc[dot_idx] (*dot_done = 1), else the caller
    // forms it.  Each sweep's stop test is read after the next sweep is queued -- or,
    // with a third buffer C (one rank), after the next TWO are queued: the sweeps rotate
    // over three buffers, so the two queued past a stop that fires (abandoned) cannot
    // overwrite the result, and the host's turn-around per sweep can take up to two
    // sweeps' time before the GPU waits.  The same launches and bits either way.
    int damped_jacobi(const double* rhs, double* A, double* B, int dot_idx, double** out, int* dot_done,
                      double* C = nullptr) {
        const double tol2 = o->jtol * o->jtol;
        const int maxit = o->jmaxiter;
        *dot_done = 0;
        double* bufs[3] = {A, B, C};
        const int nb = C ? 3 : 2, depth = C ? 2 : 1;
        // two sweeps per launch (one rank, 2D p = 3, three buffers; POMS_J2=0: off):
        // sweeps k, k+1 from bufs[cur] into bufs[nxt]; x_k is not stored
        static const bool j2_env = !(getenv("POMS_J2") && getenv("POMS_J2")[0] == '0');
        const bool j2 = j2_env && C && direct() && sweep2_ok(op);
        int cur = 0;                              // buffer of the latest queued x
        struct Pend { int kind, h, buf, in; };    // 1: sweep norm in slot h; 2: the from-zero
        Pend q[2];                                // pair; 3: a two-sweep launch from bufs[in];
                                                  // 5: sweeps 1-3 from zero
        int nq = 0, ring = 0, k0;
        int fz = 0;
        if (maxit >= 2 && maxit != 2 && op->form != FORM_STENCIL) (void)poms_op_from_zero_supported(op, &fz);
        // sweeps 1-3 from x = 0 in one launch where the two-sweep launches run (POMS_J2FZ=0: off)
        static const bool j3_env = !(getenv("POMS_J2FZ") && getenv("POMS_J2FZ")[0] == '0');
        if (fz && j2 && j3_env && maxit >= 4) {   // [||x1||^2, ||dr2||^2, ||dr3||^2]
            const int h0 = arm(H_J0, 3);
            if (jrun3(rhs, A, h0)) return 1;
            q[nq++] = Pend{5, h0, 0, -1};
            k0 = 4;
        } else if (fz) {   // sweeps 1, 2 from x = 0 in one pass over rhs: [||x1||^2, ||dr2||^2]
            const int h0 = arm(H_J0, 2);
            if (jrun(EPI_JACOBI0, rhs, A, rhs, true, true, h0)) return 1;
            q[nq++] = Pend{2, h0, 0, -1};
            k0 = 3;
        } else {
            if (maxit < 1) { set_error("pcg: jacobi maxiter < 1"); return 1; }
            const int h = arm(H_JN, 1);
            if (diag_scale_norm(rhs, A, h)) return 1;
            q[nq++] = Pend{1, h, 0, -1};
            ring = 1;
            k0 = 2;
        }
        // the oldest open stop test: done with *res when it fires
        auto settle = [&](bool& done, double*& res) {
            done = false;
            const Pend f = q[0];
            q[0] = q[1];
            --nq;
            if (f.kind == 2) {
                if (get(f.h, 0) < tol2) {   // the reference stops after sweep 1: x1 itself
                    // (into the buffer the abandoned sweep 3 wrote; queued after every sweep
                    // that reads it)
                    double* x1 = bufs[(f.buf + 1) % nb];
                    if (poms_op_diag_scale(op, o->omega, rhs, x1, 0, stv)) return 1;
                    done = true;
                    res = x1;
                } else if (get(f.h, 1) < tol2) {
                    done = true;
                    res = bufs[f.buf];
                }
            } else if (f.kind == 5) {   // sweeps 1-3 from zero; x1 and x2 re-formed into the
                double* xr = bufs[(f.buf + 1) % nb];   // buffer the abandoned next launch wrote
                if (get(f.h, 0) < tol2) {
                    if (poms_op_diag_scale(op, o->omega, rhs, xr, 0, stv)) return 1;
                    done = true;
                    res = xr;
                } else if (get(f.h, 1) < tol2) {
                    if (op_run_epi(op, EPI_JACOBI0, o->omega, rhs, xr, rhs, 0, n0, 0, 0, false, false, stv)) return 1;
                    done = true;
                    res = xr;
                } else if (get(f.h, 2) < tol2) {
                    done = true;
                    res = bufs[f.buf];
                }
            } else if (f.kind == 3) {
                if (get(f.h, 0) < tol2) {   // stopped after sweep k: x_k, one sweep from the
                    // launch's input (intact: only one launch was queued after it) into the
                    // buffer that launch wrote (abandoned)
                    double* xk = bufs[(f.buf + 1) % nb];
                    if (op_run_epi(op, EPI_JACOBI, o->omega, bufs[f.in], xk, rhs, 0, n0, 0, 0, false, false, stv))
                        return 1;
                    done = true;
                    res = xk;
                } else if (get(f.h, 1) < tol2) {
                    done = true;
                    res = bufs[f.buf];
                }
            } else if (get(f.h) < tol2) {
                done = true;
                res = bufs[f.buf];
            }
            return failed ? 1 : 0;
        };
        for (int k = k0; k <= maxit; ++k) {
            const bool last = k == maxit;
            const int nxt = (cur + 1) % nb;
            int h = -1;
            if (j2 && k + 1 < maxit) {   // sweeps k, k+1: [||dr_k||^2, ||dr_{k+1}||^2]
                h = arm(H_J0, 2);
                if (jrun(EPI_JACOBI2, bufs[cur], bufs[nxt], rhs, true, true, h)) return 1;
                // every open test is read now: a two-sweep launch's own (below) after the
                // next launch, because the one after that would overwrite its input
                while (nq > 0) {
                    bool done;
                    double* res = nullptr;
                    if (settle(done, res)) return 1;
                    if (done) { *out = res; return 0; }
                }
                q[nq++] = Pend{3, h, nxt, cur};
                cur = nxt;
                ++k;
                continue;
            }
            if (last) {   // the last sweep's norm cannot change the result: x . rhs instead
                dot_part_n = -1;
                if (direct() && dot_idx == SC_SRN && op->dot_base < 0 && op->part_off == 0 && !op->part_dst &&
                    op->form != FORM_STENCIL) {   // its partials wait for pcg_beta_kernel
                    if (op_run_epi(op, EPI_JACOBI, o->omega, bufs[cur], bufs[nxt], rhs, 0, n0, 0, 0, false, true, stv))
                        return 1;
                    dot_part_n = op->last_partials;
                    dot_part = op->ctx->scratch + dot_part_n;   // (where poms_op_run_reduce2 reads a dot's partials)
                } else if (run(EPI_JACOBI, bufs[cur], bufs[nxt], rhs, nullptr, sc + dot_idx) || allsum(sc + dot_idx, 1)) {
                    return 1;
                }
            } else {
                h = arm(H_JN + ring, 1);
                if (jrun(EPI_JACOBI, bufs[cur], bufs[nxt], rhs, true, false, h)) return 1;
                ring ^= 1;
            }
            cur = nxt;
            if (nq == depth || (nq > 0 && (q[0].kind == 3 || q[0].kind == 5))) {   // the test of the sweep `depth`
                bool done;                                      // back, read after this one is queued
                double* res = nullptr;
                if (settle(done, res)) return 1;
                if (done) { *out = res; return 0; }
            }
            if (!last) q[nq++] = Pend{1, h, cur, -1};
        }
        while (nq > 0) {   // tests still open after the last sweep (its own has none)
            bool done;
            double* res = nullptr;
            if (settle(done, res)) return 1;
            if (done) { *out = res; return 0; }
        }
        *dot_done = k0 <= maxit ? 1 : 0;
        *out = bufs[cur];
        return 0;
    }
};

}  // namespace

// Speculative smoother call (see PcgRun::spec_*), in two halves: spec_issue queues every
// launch of the call (and, last, the copy of the device-held sums to the host); the
// values it needs later are described by R.sparts / schk / srr / sn / vrr0.
// spec_finish waits for the stream and evaluates the stop tests: 0 done, 1 error, 2 a
// stop test fired (the caller repeats the call step by step).
static int spec_issue(PcgRun& R, const double* b, double* x, int has_x0, double* const* work, int* vrr0_out) {
    poms_op* op = R.op;
    const poms_pcg_opts* o = R.o;
    poms_ctx* ctx = op->ctx;
    const poms_layout* L = &op->L;
    void* stream = R.stv;
    double *r = work[0], *q = work[1];
    double* z[3] = {work[2], work[3], work[4]};
    if (has_x0) {   // x0 is kept for the step-by-step repeat
        const int64_t nbak = (int64_t)(op->L.n[0] + 2 * op->L.pads[0]) * row_geom(&op->L).s0;
        POMS_HIP_CHECK(hipMemcpyAsync(op->spec_bak, x, nbak * sizeof(double), hipMemcpyDeviceToDevice, R.st));
    }
    if (!has_x0) {
        if (poms_vec_fill(ctx, L, 0.0, x, stream)) return 1;
    } else if (R.run(EPI_RESID, x, r, b, nullptr, nullptr)) {
        return 1;
    }
    const int vrr0 = R.svals(1);
    *vrr0_out = vrr0;
    if (!has_x0 ? vec_copy_dot(ctx, L, b, r, op->spec_dev + vrr0, stream)   // r = b and r.r
                : poms_vec_dot(ctx, L, r, r, op->spec_dev + vrr0, stream))
        return 1;
    double* s = nullptr;
    if (R.spec_damped_jacobi(r, z[0], z[1], SC_SR, &s)) return 1;
    double* p = s;   // p keeps this buffer; the later psolves use the other two
    double* fa = nullptr;
    double* fb = nullptr;
    for (double* c : z)
        if (c != p) (fa ? fb : fa) = c;
    for (int k = 1; k <= o->maxiter; ++k) {
        if (R.run(EPI_APPLYDOT, p, q, p, nullptr, R.sc + SC_PQ) || R.allsum(R.sc + SC_PQ, 1)) return 1;
        hipLaunchKernelGGL(pcg_scalars_kernel, dim3(1), dim3(64), 0, R.st, R.sc, 0);
        const int vrr = R.svals(1);
        R.srr.push_back(vrr);
        if (poms_pcg_r_update_dev(ctx, L, R.sc + SC_ALPHA, r, q, op->spec_dev + vrr, stream)) return 1;
        double* sn = nullptr;
        if (R.spec_damped_jacobi(r, fa, fb, SC_SRN, &sn)) return 1;
        hipLaunchKernelGGL(pcg_scalars_kernel, dim3(1), dim3(64), 0, R.st, R.sc, 1);
        if (poms_pcg_xp_update_dev(ctx, L, R.sc + SC_ALPHA2, x, p, sn, stream)) return 1;
    }
    if (R.sn > poms_op::kSpecVals) { set_error("pcg speculative: too many values"); return 1; }
    if (R.comm && R.sn > 0 && poms_allreduce_sum(R.comm, op->spec_dev, R.sn, stream, 1)) return 1;
    if (R.sn > 0)
        POMS_HIP_CHECK(hipMemcpyAsync(op->spec_host, op->spec_dev, R.sn * sizeof(double), hipMemcpyDeviceToHost, R.st));
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

static int spec_finish(PcgRun& R, int vrr0, poms_pcg_info* info) {
    const poms_pcg_opts* o = R.o;
    POMS_HIP_CHECK(hipStreamSynchronize(R.st));
    std::vector<double> v(R.op->spec_host, R.op->spec_host + R.sn);
    for (const PcgRun::SPart& s : R.sparts) {
        const bool wn = s.kind & 1, wd = s.kind & 2;
        const double* reg = R.op->spec_part + s.off;
        if (wn) v[s.vi + (wd ? 1 : 0)] = PcgRun::host_reduce(reg, s.n);
        if (wd) v[s.vi] = PcgRun::host_reduce(reg + (wn ? s.n : 0), s.n);
    }
    const double tol2 = o->jtol * o->jtol;
    for (int i : R.schk)
        if (v[i] < tol2) return 2;
    const double nrmr0 = std::sqrt(v[vrr0]);
    for (int i : R.srr)
        if (v[i] < o->tol * nrmr0) return 2;
    const double nrmr = R.srr.empty() ? nrmr0 * nrmr0 : v[R.srr.back()];
    info->niter = o->maxiter;
    info->success = 0;
    info->res_norm = std::sqrt(nrmr);
    return 0;
}

// One speculative call, through a captured graph of its launches when POMS_PCG_GRAPH
// is not 0 and there is no host-transport communicator (its callbacks synchronise).
// Graphs are cached per operator by the call's buffers, options and launch-timing
// state (kSpecGraphs entries, least recently used replaced).
static int pcg_speculative(PcgRun& R, const double* b, double* x, int has_x0, double* const* work,
                           poms_pcg_info* info) {
    poms_op* op = R.op;
    const poms_pcg_opts* o = R.o;
    // POMS_PCG_GRAPH=0: never.  Not with a communicator: the distributed operator call's
    // ring-slot and exchange bookkeeping is host-side per call (a captured RCCL
    // loopback call crashed in the attempt, r04graph logs).  A caller whose buffers
    // never repeat would capture every call: after 8 more captures than hits the
    // operator stops using graphs.
    // POMS_PCG_GRAPH=2 (opt-in, tools/graph_rccl_probe.py): graphs with a communicator
    // too -- every exchange and all-reduce of the call captured; RCCL's point-to-point
    // exchange does not survive capture, the peer transport's does (POMS_COMM_PEER=1)
    const char* ge = getenv("POMS_PCG_GRAPH");
    int host_comm = 0;
    if (R.comm && poms_comm_is_host(R.comm, &host_comm)) return 1;
    const bool comm_ok = !R.comm || (ge && ge[0] == '2' && !host_comm);
    const bool graph = !(ge && ge[0] == '0') && comm_ok && op->spec_graph_caps <= op->spec_graph_hits + 8;
    if (!graph) {
        int vrr0 = 0;
        if (spec_issue(R, b, x, has_x0, work, &vrr0)) return 1;
        return spec_finish(R, vrr0, info);
    }
    uint64_t key[16] = {};
    auto bits = [](double d) { uint64_t u; std::memcpy(&u, &d, 8); return u; };
    key[0] = (uint64_t)(uintptr_t)b;
    key[1] = (uint64_t)(uintptr_t)x;
    for (int i = 0; i < 5; ++i) key[2 + i] = (uint64_t)(uintptr_t)work[i];
    key[7] = (uint64_t)has_x0 | ((uint64_t)(uint32_t)o->maxiter << 8) | ((uint64_t)(uint32_t)o->jmaxiter << 40);
    key[8] = bits(o->tol);
    key[9] = bits(o->jtol);
    key[10] = bits(o->omega);
    key[11] = (uint64_t)(uint32_t)op->variant | ((uint64_t)(uint32_t)op->chunk << 32);
    key[12] = (uint64_t)(op->timing ? 1 : 0) | ((uint64_t)(uint32_t)op->t_epi << 8) | ((uint64_t)(uint32_t)op->t_every << 32);
    key[13] = (uint64_t)(uintptr_t)R.comm | ((uint64_t)(uint32_t)(o->prev + 1) << 48) | ((uint64_t)(uint32_t)(o->next + 1) << 56);
    {   // whatever else changes the captured launches: the setters' generation, the tile
        // geometry and ghost corners, the partials layout, and the env knobs read per launch
        const char* hp = getenv("POMS_HOST_PARTIALS");
        const char* la = getenv("POMS_PCG_LOOKAHEAD");
        key[14] = op->gen ^ ((uint64_t)(uint32_t)op->tout << 20) ^ ((uint64_t)(op->ghost_corners ? 1 : 0) << 52) ^
                  ((uint64_t)(uint32_t)(hp ? atoi(hp) + 1 : 0) << 40);
        key[15] = (uint64_t)(uint32_t)(op->dot_base + 1) ^ ((uint64_t)(uint32_t)op->part_off << 32) ^
                  ((uint64_t)(la && la[0] ? la[0] : 0) << 56);
    }
    poms_op::SpecGraph* hit = nullptr;
    for (auto& g : op->spec_graphs)
        if (g.exec && std::memcmp(g.key, key, sizeof(key)) == 0) hit = &g;
    if (!hit) {   // capture the call's launches once
        poms_op::SpecGraph* slot = &op->spec_graphs[0];
        for (auto& g : op->spec_graphs)
            if (!g.exec || g.use < slot->use) slot = &g;
        if (slot->exec) {
            (void)hipGraphExecDestroy(slot->exec);
            slot->exec = nullptr;
        }
        // captured on a private stream (torch's default stream is the null stream, which
        // cannot be captured); nothing runs until the graph is launched on the caller's
        if (!op->cap_stream) POMS_HIP_CHECK(hipStreamCreateWithFlags(&op->cap_stream, hipStreamNonBlocking));
        const hipStream_t cst = R.st;
        void* const cstv = R.stv;
        R.st = op->cap_stream;
        R.stv = op->cap_stream;
        POMS_HIP_CHECK(hipStreamBeginCapture(R.st, hipStreamCaptureModeRelaxed));
        int vrr0 = 0;
        const int rc = spec_issue(R, b, x, has_x0, work, &vrr0);
        hipGraph_t gr = nullptr;
        const hipError_t ce = hipStreamEndCapture(R.st, &gr);
        R.st = cst;
        R.stv = cstv;
        ++op->spec_graph_caps;
        hipGraphExec_t ex = nullptr;
        hipError_t ie = hipSuccess;
        if (!rc && ce == hipSuccess) ie = hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0);
        if (gr) (void)hipGraphDestroy(gr);
        if (rc || ce != hipSuccess || ie != hipSuccess) {
            // Nothing captured ran.  Clear the sticky error and run the call uncaptured on
            // the caller's stream (advisor, round 4: a capture or instantiate failure used
            // to fail the whole poms_pcg_jacobi call); graphs are off for this operator
            // from now on.
            (void)hipGetLastError();
            op->spec_graph_caps += 1 << 20;
            R.sparts.clear();
            R.schk.clear();
            R.srr.clear();
            R.scur = 0;
            R.sn = 0;
            int vrr0u = 0;
            if (spec_issue(R, b, x, has_x0, work, &vrr0u)) return 1;
            return spec_finish(R, vrr0u, info);
        }
        std::memcpy(slot->key, key, sizeof(key));
        slot->exec = ex;
        slot->parts = R.sparts;
        slot->chk = R.schk;
        slot->rr = R.srr;
        slot->sn = R.sn;
        slot->vrr0 = vrr0;
        hit = slot;
    } else {
        ++op->spec_graph_hits;
    }
    hit->use = ++op->spec_graph_clock;
    POMS_HIP_CHECK(hipGraphLaunch(hit->exec, R.st));
    R.sparts = hit->parts;
    R.schk = hit->chk;
    R.srr = hit->rr;
    R.sn = hit->sn;
    return spec_finish(R, hit->vrr0, info);
}

// Speculative mode is opt-in (POMS_PCG_SPEC=1): on the 2D 1024^2 cycle, measured in one
// process against the step-by-step loop, it costs 3.8 ms per cycle vs 3.1 (graph replay
// included; profiles/r04/graph): the stream drain it needs at the end of every call
// exposes the host's issue of the next phase, and the step-by-step loop's lazy reads
// already keep the queue ahead of the GPU.
static bool pcg_spec_wanted(const poms_op*, const poms_pcg_opts* o) {
    const char* e = getenv("POMS_PCG_SPEC");
    return e && e[0] == '1' && o->maxiter >= 1 && o->jmaxiter >= 3;
}

static int pcg_jacobi_impl(poms_op* op, poms_comm* comm, const poms_pcg_opts* o, const double* b, double* x,
                           int has_x0, double* const* work, poms_pcg_info* info, void* stream);

// (a peer exchange that timed out during the call fails it: poms_comm_check)
int poms_pcg_jacobi(poms_op* op, poms_comm* comm, const poms_pcg_opts* o, const double* b, double* x, int has_x0,
                    double* const* work, poms_pcg_info* info, void* stream) {
    if (pcg_jacobi_impl(op, comm, o, b, x, has_x0, work, info, stream)) return 1;
    return comm ? poms_comm_check(comm) : 0;
}

static int pcg_jacobi_impl(poms_op* op, poms_comm* comm, const poms_pcg_opts* o, const double* b, double* x,
                           int has_x0, double* const* work, poms_pcg_info* info, void* stream) {
    if (!op || !o || !b || !x || !work || !info) { set_error("poms_pcg_jacobi: null argument"); return 1; }
    for (int i = 0; i < 5; ++i)
        if (!work[i]) { set_error("poms_pcg_jacobi: null work vector"); return 1; }
    if (o->maxiter < 0 || o->jmaxiter < 1) { set_error("poms_pcg_jacobi: bad iteration counts"); return 1; }
    POMS_HIP_CHECK(hipSetDevice(op->ctx->device));
    if (!op->sv_dev) {
        POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&op->sv_dev), SC_N * sizeof(double)));
        POMS_HIP_CHECK(hipMemset(op->sv_dev, 0, SC_N * sizeof(double)));
        // coherent (fine-grained) and device-mapped: reduction kernels write the
        // host-read norms straight into it
        POMS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&op->sv_host), poms_op::kSvRing * sizeof(double),
                                     hipHostMallocMapped | hipHostMallocCoherent));
        POMS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&op->sv_part),
                                     (size_t)poms_op::kSvRing * poms_op::kSvPart * sizeof(double),
                                     hipHostMallocMapped | hipHostMallocCoherent));
        PcgRun::part_arm(op->sv_part, poms_op::kSvRing * poms_op::kSvPart);
        for (int64_t& q : op->sv_seq) q = -1;
    }
    if (pcg_spec_wanted(op, o)) {
        const int64_t nbak = (int64_t)(op->L.n[0] + 2 * op->L.pads[0]) * row_geom(&op->L).s0;
        if (!op->spec_dev) {
            POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&op->spec_dev), poms_op::kSpecVals * sizeof(double)));
            POMS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&op->spec_host), poms_op::kSpecVals * sizeof(double),
                                         hipHostMallocDefault));
            POMS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&op->spec_part), poms_op::kSpecPart * sizeof(double),
                                         hipHostMallocMapped | hipHostMallocCoherent));
        }
        if (has_x0 && op->spec_bak_n < nbak) {
            if (op->spec_bak) POMS_HIP_CHECK(hipFree(op->spec_bak));
            op->spec_bak = nullptr;
            op->spec_bak_n = 0;
            POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&op->spec_bak), nbak * sizeof(double)));
            op->spec_bak_n = nbak;
        }
        PcgRun RS{op, comm, o, as_stream(stream), stream, op->sv_dev, op->sv_host};
        RS.n0 = op->ndim == 3 ? op->L.n[0] : 1;
        ++op->spec_calls;
        const int rc = pcg_speculative(RS, b, x, has_x0, work, info);
        if (rc != 2) return rc;
        ++op->spec_repeats;
        // a stop test fired: the step-by-step loop from the same inputs
        if (has_x0)
            POMS_HIP_CHECK(hipMemcpyAsync(x, op->spec_bak, nbak * sizeof(double), hipMemcpyDeviceToDevice, as_stream(stream)));
    }
    PcgRun R{op, comm, o, as_stream(stream), stream, op->sv_dev, op->sv_host};
    R.n0 = op->ndim == 3 ? op->L.n[0] : 1;
    poms_ctx* ctx = op->ctx;
    const poms_layout* L = &op->L;
    double *r = work[0], *q = work[1];
    double* z[3] = {work[2], work[3], work[4]};
    // x0 = None: x = 0, r = b - A.0 = b exactly; else r = b - A x0
    if (!has_x0) {
        if (poms_vec_fill(ctx, L, 0.0, x, stream)) return 1;
    } else if (R.run(EPI_RESID, x, r, b, nullptr, nullptr)) {
        return 1;
    }
    const int hrr0 = R.arm(H_RR0, 1);
    {
        double* d = R.hslot(hrr0);
        if (!d) return 1;
        if (!has_x0 ? vec_copy_dot(ctx, L, b, r, d, stream)   // r = b and r.r in one pass
                    : poms_vec_dot(ctx, L, r, r, d, stream))
            return 1;
        if (R.lazy_post(hrr0, 1)) return 1;
    }
    const double nrmr0 = std::sqrt(R.get(hrr0));
    if (R.failed) return 1;
    // Two-sweep lookahead in the damped-Jacobi calls (one rank; POMS_PCG_LOOKAHEAD=1 /
    // 0 forces it on / off, default on for 2D operators, where the host's turn-around
    // per sweep is close to a sweep's GPU time): a fourth preconditioner buffer
    double* e4 = nullptr;
    {
        const char* le = getenv("POMS_PCG_LOOKAHEAD");
        const bool la = R.direct() && (le && le[0] ? le[0] == '1' : op->ndim == 2);
        if (la) {
            // The buffer takes the work vectors' 16-B / 128-B phase (they start `shift`
            // doubles into their allocation on the line-aligned layout): the flat vector
            // kernels and v5's aligned tiles then run on it exactly as on the other three
            // buffers, with the same block split of the sums (advisor, round 4).
            const int64_t nbuf = (int64_t)(op->L.n[0] + 2 * op->L.pads[0]) * row_geom(&op->L).s0;
            const int64_t off = (int64_t)((reinterpret_cast<uintptr_t>(work[2]) & 127) / sizeof(double));
            if (op->la_n < nbuf) {
                if (op->la_raw) POMS_HIP_CHECK(hipFree(op->la_raw));
                op->la_raw = op->la_buf = nullptr;
                op->la_n = 0;
                POMS_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&op->la_raw), (nbuf + 16) * sizeof(double)));
                op->la_n = nbuf;
                op->la_off = -1;
            }
            if (op->la_off != off) {   // (re-)placed: zero ghosts
                POMS_HIP_CHECK(hipMemsetAsync(op->la_raw, 0, (nbuf + 16) * sizeof(double), R.st));
                op->la_off = off;
                op->la_buf = op->la_raw + off;
            }
            e4 = op->la_buf;
        }
    }
    double* s = nullptr;
    int dd = 0;
    if (R.damped_jacobi(r, z[0], z[1], SC_SR, &s, &dd, e4)) return 1;
    if (!dd && R.dot(s, r, R.sc + SC_SR)) return 1;
    double* p = s;   // p keeps this buffer; later psolves use the others
    double* fp[3] = {nullptr, nullptr, nullptr};
    {
        int nf = 0;
        for (double* c : {z[0], z[1], z[2], e4})
            if (c && c != p) fp[nf++] = c;
    }
    double* fa = fp[0];
    double* fb = fp[1];
    double* fc = fp[2];   // (nullptr without the lookahead)
    int k = 0;
    double nrmr = nrmr0 * nrmr0;
    for (k = 1; k <= o->maxiter; ++k) {
        if (R.apd_alpha(p, q)) return 1;
        const int hrr = R.arm(H_RR, 1);
        if (R.rupd(r, q, hrr)) return 1;
        double* sn = nullptr;
        if (R.damped_jacobi(r, fa, fb, SC_SRN, &sn, &dd, fc)) return 1;   // queued before the read
        if (!dd && R.dot(sn, r, R.sc + SC_SRN)) return 1;
        nrmr = R.get(hrr);
        if (R.failed) return 1;
        if (nrmr < o->tol * nrmr0) {   // the reference stops before psolve: that one is discarded
            if (poms_vec_axpby_dev(ctx, L, R.sc + SC_ONE, x, p, x, stream)) return 1;
            k -= 1;
            break;
        }
        // beta folded into the x/p update where it can be (one rank, small grids)
        const int fb = (dd && R.dot_part_n >= 0) ? R.xpupd_beta(x, p, sn) : 1;
        if (fb < 0) return 1;
        if (fb > 0) {
            if (R.fix_sr()) return 1;
            if (dd && R.dot_part_n >= 0)   // x . rhs's partials from the last sweep, reduced here
                hipLaunchKernelGGL(pcg_beta_kernel, dim3(1), dim3(256), 0, R.st, R.dot_part, (int)R.dot_part_n, R.sc);
            else
                hipLaunchKernelGGL(pcg_scalars_kernel, dim3(1), dim3(64), 0, R.st, R.sc, 1);
            if (poms_pcg_xp_update_dev(ctx, L, R.sc + SC_ALPHA2, x, p, sn, stream)) return 1;
        }
    }
    // (a folded beta's pending s.r_old <- s.r_new is dropped: the next call's first
    // psolve writes s.r before anything reads it)
    R.sr_stale = false;
    if (R.flush_alpha()) return 1;
    if (k > o->maxiter) k = o->maxiter;
    info->niter = k;
    info->success = nrmr < o->tol * nrmr0 ? 1 : 0;
    info->res_norm = std::sqrt(nrmr);
    POMS_HIP_CHECK(hipGetLastError());
    return 0;
}

int poms_op_timing(poms_op* op, int enable, int epilogue, int every, int reserve) {
    if (!op || every < 1 || reserve < 0) { set_error("poms_op_timing: bad argument"); return 1; }
    op->timing = enable != 0;
    if (!op->timing) return 0;   // disabling keeps the record for poms_op_timing_read
    op->tl_used = 0;
    op->t_epi = epilogue;
    op->t_every = every;
    op->t_seen = 0;
    POMS_HIP_CHECK(hipSetDevice(op->ctx->device));
    while (op->tl.size() < (size_t)reserve) {   // create the events now, not inside the timed work
        poms_op::TimedLaunch t{};
        POMS_HIP_CHECK(hipEventCreate(&t.e0));
        POMS_HIP_CHECK(hipEventCreate(&t.e1));
        op->tl.push_back(t);
    }
    return 0;
}

int poms_op_timing_read(poms_op* op, int epilogue, double* total_ms, int64_t* launches, int64_t* dofs) {
    if (!op || !total_ms || !launches || !dofs) { set_error("poms_op_timing_read: null argument"); return 1; }
    double tot = 0.0;
    int64_t n = 0, d = 0;
    for (size_t i = 0; i < op->tl_used; ++i) {
        const auto& t = op->tl[i];
        if (t.epi != epilogue) continue;
        POMS_HIP_CHECK(hipEventSynchronize(t.e1));
        float ms = 0.0f;
        POMS_HIP_CHECK(hipEventElapsedTime(&ms, t.e0, t.e1));
        tot += ms;
        ++n;
        d += t.ndof;
    }
    *total_ms = tot;
    *launches = n;
    *dofs = d;
    return 0;
}
