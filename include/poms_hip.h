/*
 * poms_hip.h -- C ABI of libpoms_hip.so, the MI355X (gfx950) hot path of the
 * POMS tensor-product B-spline multigrid.
 *
 * Every entry point is plain C: integers, doubles, raw pointers, an opaque
 * handle and a hipStream_t passed as `void*`.  No torch or C++ types cross
 * this boundary.  Each function returns 0 on success and a non-zero status
 * otherwise; `poms_last_error()` then returns a thread-local message.
 *
 * Memory: the caller owns every vector buffer.  Vector arguments are DEVICE
 * pointers to padded C-order arrays with the spl `StencilVector._data`
 * layout (`slides/content.tex:256-264`): local extent n_d plus `pads[d]`
 * ghost cells on each side of every axis (2D: n0 = 1, pads[0] = 0;
 * 1D additionally n1 = 1, pads[1] = 0).  Kernels read ghost cells and never
 * write them; halo transport of the axis-0 ghost planes is the caller's
 * (RCCL send/recv via torch.distributed), see INTEGRATION.md.
 *
 * Band convention for every 1D factor: row-major (n, 2*pmax+1) doubles,
 * F_band[i*(2*pmax+1) + k] = F[i, i + k - pmax] -- the 1D StencilMatrix
 * layout `A[i1, k]` of `pyccel/pyccel_functions.py:4-21`.
 *
 * Streams: every kernel is enqueued on the given stream (NULL = default);
 * nothing synchronises the host except `poms_kron_dot_2d` (host-pointer
 * drop-in) and the `*_host` getters.  Handles are not thread-safe; one
 * context per device per host thread.
 */
#ifndef POMS_HIP_H
#define POMS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POMS_ABI_VERSION 3

/* operator forms (see poms_op_create) */
#define POMS_FORM_SINGLE 0 /* y = F0 (x) F1 (x) F2 x                                  */
#define POMS_FORM_SUM    1 /* y = A0(x)M1(x)M2 x + M0(x)(K1(x)M2 + M1(x)K2) x (3D)   */
                           /* y = A1(x)M2 x + M1(x)K2 x                      (2D/1D)  */

typedef struct poms_ctx poms_ctx;           /* per-device context + scratch      */
typedef struct poms_op poms_op;             /* Kronecker(-sum) banded operator   */
typedef struct poms_transfer poms_transfer; /* knot-insertion R = P^T / P        */
typedef struct poms_comm poms_comm;         /* RCCL communicator of the slabs    */
typedef struct poms_ksolve poms_ksolve;     /* factorised Kronecker direct solve */

/* Grid layout of a (local) padded vector.  ndim in {1,2,3}; unused leading
 * axes have n = 1 and pad = 0.  Axis order is C order: axis 2 is unit-stride. */
typedef struct poms_layout {
    int64_t n[3];    /* local interior extent per axis                       */
    int64_t pads[3]; /* ghost width per axis (storage pad)                   */
    int64_t pitch;   /* row stride (doubles) of axis 2; 0 = n[2] + 2 pads[2].
                      * A pitch that is a multiple of 16 together with a base
                      * pointer whose column pads[2] sits on a 128-B line makes
                      * every row segment of a 16k-column tile start on a line. */
    int64_t flags;   /* bit 0 (POMS_LAYOUT_GHOST_DATA): the ghost rows / columns
                      * of axes 1 and 2 may hold data (a block of a decomposition
                      * of those axes, spl Cart): vector operations then touch
                      * the interior only instead of whole interior planes.   */
} poms_layout;
#define POMS_LAYOUT_GHOST_DATA 1

/* ---- library / context ---------------------------------------------------- */
int         poms_abi_version(void);
const char* poms_last_error(void);
int         poms_device_count(int* count);
/* Creates a context on `device` (hipSetDevice) with reduction scratch.
 * Replaces: the per-process MPI/spl setup of `sources/mg_jac.py:19-46`.       */
int         poms_ctx_create(int device, poms_ctx** ctx);
int         poms_ctx_destroy(poms_ctx* ctx);
int         poms_synchronize(poms_ctx* ctx, void* stream);

/* ---- banded Kronecker operator ------------------------------------------- */
/* Create an operator on a local slab.  `layout` is the vector layout.  Axis-0
 * rows are global: local plane z is global plane g0 + z, n0_global planes.
 * Factor arrays are HOST pointers, band rows of width 2*pmax+1, copied to the
 * device:
 *   POMS_FORM_SINGLE (3D): f[0]=F0 (n0_global rows), f[2]=F1, f[4]=F2
 *   POMS_FORM_SUM    (3D): f[0]=A0 (= M0+K0), f[1]=M0, f[2]=M1, f[3]=K1,
 *                          f[4]=M2, f[5]=K2
 *   2D/1D: axis-0 factors are ignored (pass NULL); SINGLE: f[2]=F1, f[4]=F2;
 *          SUM: f[2]=A1 (= M1+K1), f[3]=M1, f[4]=M2, f[5]=K2
 * Replaces: the operator built by `assembly_2d` (`sources/matrix_assembler.py:84-179`)
 * whose `StencilMatrix.dot` is called at `sources/solvers.py:85,103,109,209`
 * and `sources/mg_jac.py:93`; and the (A, B) pair of `kron_dot_v2`
 * (`sources/kron_product.py:56`).  pmax in 1..5.                               */
int poms_op_create(poms_ctx* ctx, int ndim, const poms_layout* layout, int form,
                   int pmax, const double* const* factors, int64_t g0,
                   int64_t n0_global, poms_op** op);
/* General stencil operator (spl StencilMatrix with its own coefficients per row,
 * `slides/content.tex:285-290`): v[i] = sum_k M[i, k] u[i + k - p].  `data` is a
 * HOST array in the spl `StencilMatrix._data` layout of the local slab: the padded
 * local extents (n_d + 2 pads_d, C order), then 2 pads_d + 1 offsets per axis
 * (2D: (n1+2p1, n2+2p2, 2p1+1, 2p2+1)); the stencil half-widths are the layout's
 * pads.  Coefficients are copied to the device once as one plane per offset.
 * Every poms_op_* entry point works on it (apply, residual, Jacobi sweep with norm
 * and x_out.b, apply + x.y, diag_scale, run_reduce, run_dist) except the
 * two-sweeps-from-zero epilogue.
 * Replaces: `StencilMatrix.dot` of the operator `assembly_2d` builds
 * (`sources/matrix_assembler.py:84-179`), called at `sources/solvers.py:85,103,
 * 109,209` and `sources/mg_jac.py:93`.                                         */
int poms_op_create_stencil(poms_ctx* ctx, int ndim, const poms_layout* layout, const double* data,
                           int64_t g0, int64_t n0_global, poms_op** op);
/* On-device assembly of the variable-coefficient operator
 * -div(a grad u) + c u on a tensor B-spline space into a general-stencil operator:
 *   M[i, j] = sum_elements sum_quadrature w (c phi_i phi_j + a grad phi_i . grad phi_j),
 * per element the quadrature sum first, as `assembly_2d` (`sources/matrix_assembler.py:
 * 84-179`, a = c = 1, which this reproduces).  Per used axis d (HOST arrays): nel[d]
 * elements (non-empty knot spans) with nq[d] Gauss points; first[d][e] = global index
 * of element e's first basis function (span - p); es[d][i] / ee[d][i] = first / last
 * element of basis function i's support (nglob[d] entries); basis[d] =
 * (nel, nq, p+1, 2) values and first derivatives; weights[d] = (nel, nq) weights with
 * the element Jacobian.  p[d] must equal layout->pads[d].  a_q, c_q: DEVICE arrays of
 * the coefficients at every quadrature point, C order over (e0 q0, e1 q1, e2 q2) of
 * the GLOBAL grid, or NULL for a = 1, c = mass_coef.  Axis 0 may be a slab (g0).    */
int poms_op_assemble_stencil(poms_ctx* ctx, int ndim, const poms_layout* layout, const int* nel, const int* nq,
                             const int* p, const int* const* first, const int* const* es, const int* const* ee,
                             const double* const* basis, const double* const* weights, const int64_t* nglob,
                             const double* a_q, const double* c_q, double mass_coef, int64_t g0, poms_op** op);
/* The coefficients of a general-stencil operator in the spl StencilMatrix._data
 * layout (the layout poms_op_create_stencil takes), HOST output.               */
int poms_op_stencil_data(poms_op* op, double* data_host);
int poms_op_destroy(poms_op* op);
/* Planes per workgroup along axis 0 (3D); 0 = automatic. */
int poms_op_set_chunk(poms_op* op, int chunk);
/* Output columns per 64-lane tile of the v3 / v4 kernels (variants 4-9):
 * 0 = 64 - 2 pmax (default); a multiple of 16 keeps stores line-aligned on an
 * aligned layout (see poms_layout.pitch).  Must be <= 64 - 2 pmax.            */
int poms_op_set_tile_cols(poms_op* op, int cols);
/* Kernel variant.  All variants compute the same operator:
 *   0 = general (any band rows, any pads);
 *   4 = v3: axis-2 pass by DPP lane shifts, (a, b) tile in LDS, one barrier per plane;
 *   7 = v4: axis-1-first, x planes DMA'd into an LDS ring (buffer_load ... lds),
 *       two columns per lane, symmetric Toeplitz pair sums;
 *   8 = auto (default when pads == pmax): the fastest measured kernel per epilogue;
 *   9 = v3 addressing each array through one buffer resource (arrays < 2 GiB);
 *  10 = v5: 128-column tiles (112 line-aligned output columns on an aligned
 *       layout), one row per wave, x DMA'd into an LDS ring, axis-1-first
 *       (3D FORM_SUM, arrays < 2 GiB, not at odd p with ghost corners; other
 *       operators, and two-sweeps-from-zero at p = 3 with distinct axis-1 /
 *       axis-2 Toeplitz rows, run variant 9);
 *  90-114 = diagnostic / tuning builds (memory-only, compute-only, cache policies;
 *  110-112: two sweeps from zero without sums / x1 scaling, timing only; 114:
 *  clock-stamped apply / Jacobi sweep, poms_diag_v5_stamps).
 * (11, the experimental v7 kernel, was removed in round 6.)
 * Variants 4-10 need storage pads == pmax on every used axis.                  */
int poms_op_set_variant(poms_op* op, int variant);
/* 1 if the kernels of `variant` are compiled into this library, else 0. */
int poms_variant_built(int variant);
/* Diagnostic: the per-wave clock stamps of the last v5 stamped launches (variant
 * 114, p = 3 apply / Jacobi sweep): n u64, 8 per wave in launch order (block x
 * waves + wave): cycles waiting for the wave's DMAs, in the plane barrier, the
 * rest; planes; start / end (100 MHz); XCC | tile << 8 (the tile's index in the
 * default order); CU.  The buffer is cleared after.                            */
int poms_diag_v5_stamps(uint64_t* host_out, int64_t n);
/* Tuning: the order in which v5 launches start their tiles within each XCD's
 * range -- 1 longest estimated first (default; POMS_V5_SCHED=0 in the environment
 * starts with 0), 0 the default order.  Results are bitwise the same either way
 * (the partial sums keep their slots).  mode < 0 only queries.  Returns the
 * previous mode.                                                                */
int poms_diag_v5_sched(int mode);
/* Declare that the ghost edges / corners of axes 1 and 2 may hold non-zero data:
 * the vector is a block of a decomposition of axes 1 and 2 (spl Cart,
 * `sources/tests/test_kron_dot.py:51-55`), not an axis-0 slab whose ghosts off
 * axis 0 are zero.  Kernels that rely on zero corner ghosts are not selected.   */
int poms_op_set_ghost_corners(poms_op* op, int yes);
int poms_op_get_variant(poms_op* op, int* variant);
/* The variant one launch of `epilogue` runs after automatic selection and
 * fall-backs: 0 apply, 1 residual, 2 Jacobi sweep, 3 two sweeps from zero,
 * 4 apply + x.y.                                                              */
int poms_op_kernel_variant(poms_op* op, int epilogue, int* variant);
/* The kernel variant the operator's last launch actually ran, after the per-call
 * fall-backs (layout alignment, Toeplitz ranges) that poms_op_kernel_variant cannot
 * see; -1 before the first launch.                                               */
int poms_op_last_variant(poms_op* op, int* variant);
/* One operator launch on planes [z_begin, z_end) and its reductions, in one
 * call: epilogue as in poms_op_kernel_variant (0 apply y = A x; 1 residual
 * y = b - A x; 2 Jacobi sweep y = x + omega (b - A x)/diag; 3 sweeps 1-2 from
 * zero, x = b; 4 apply + x.y; 6 two sweeps from x, poms_op_sweep2_supported).
 * If norm_out / dot_out (device) are non-null the
 * per-block partials are reduced into them (accumulate: added to their value),
 * as poms_op_jacobi_sweep_dot / poms_op_apply_dot + poms_reduce_partials_at
 * would: Jacobi: norm = ||dr||^2, dot = x_out . b; from zero: norm = ||dr_2||^2,
 * dot = ||x1||^2; apply + dot: dot = x . y.                                   */
int poms_op_run_reduce(poms_op* op, int epilogue, double omega, const double* x, double* y,
                       const double* b, int64_t z_begin, int64_t z_end, double* norm_out,
                       double* dot_out, int accumulate, void* stream);
/* The same with a second plane range [z2_begin, z2_end) in the same launch (a
 * slab's two p-plane boundaries after the ghost exchange: one launch).       */
int poms_op_run_reduce2(poms_op* op, int epilogue, double omega, const double* x, double* y,
                        const double* b, int64_t z_begin, int64_t z_end, int64_t z2_begin,
                        int64_t z2_end, double* norm_out, double* dot_out, int accumulate,
                        void* stream);
/* hipMemcpyAsync of `count` doubles, device -> (pinned) host, on `stream`. */
int poms_copy_to_host_async(poms_ctx* ctx, const double* src_dev, double* dst_host, int64_t count,
                            void* stream);

/* y = A x on output planes [z_begin, z_end) (local axis-0 indices; 2D/1D: 0,1).
 * x must have current ghosts on the planes the range touches.
 * Replaces: `kron_dot_pyccel_2d` (`pyccel/pyccel_functions.py:4-21`) and
 * spl `StencilMatrix.dot` (`sources/solvers.py:103`).                         */
int poms_op_apply(poms_op* op, const double* x, double* y, int64_t z_begin,
                  int64_t z_end, void* stream);
/* y = A x, also accumulating x . y per block into scratch[count, 2 count)
 * (count from poms_op_last_partials; reduce with poms_reduce_partials_at).
 * pcg's `q = A.dot(p)` + `p.dot(q)` (`sources/solvers.py:103-104`) in one
 * pass.  Kernel variants 4, 5, 6, 8, 9, 10 (poms_op_apply_dot_supported).    */
int poms_op_apply_dot(poms_op* op, const double* x, double* y, int64_t z_begin,
                      int64_t z_end, void* stream);
int poms_op_apply_dot_supported(poms_op* op, int* yes);
/* r = b - A x (fused).  Replaces: `r = b - A.dot(x)` at `sources/solvers.py:85`,
 * `sources/solvers.py:209`, `sources/mg_jac.py:93`.                           */
int poms_op_residual(poms_op* op, const double* b, const double* x, double* r,
                     int64_t z_begin, int64_t z_end, void* stream);
/* One damped-Jacobi sweep, fused:  dr = omega (b - A x_in) / diag(A);
 * x_out = x_in + dr;  if norm_dev != NULL, per-block partial sums of dr.dr are
 * written to the context scratch and reduced into norm_dev[0] (device double)
 * by poms_reduce_partials.  x_out must not alias x_in.
 * Replaces: the body of `damped_jacobi`, `sources/solvers.py:207-219`.        */
int poms_op_jacobi_sweep(poms_op* op, double omega, const double* b,
                         const double* x_in, double* x_out, int64_t z_begin,
                         int64_t z_end, int want_norm, void* stream);
/* The same sweep, also accumulating x_out . b per block: the dr.dr partials
 * (if want_norm) go to scratch[0, count), the x_out . b partials to
 * scratch[count, 2 count) with count from poms_op_last_partials; reduce them
 * with poms_reduce_partials_at.  With b = r this is pcg's `sr = s.dot(r)`
 * (`sources/solvers.py:91,120`) fused into the last smoothing sweep.
 * Kernel variants 4-10 only (poms_op_fused_dot_supported).                   */
int poms_op_jacobi_sweep_dot(poms_op* op, double omega, const double* b,
                             const double* x_in, double* x_out, int64_t z_begin,
                             int64_t z_end, int want_norm, void* stream);
int poms_op_fused_dot_supported(poms_op* op, int* yes);
/* Sweeps 1 and 2 of damped_jacobi from x0 = 0 in one pass over b:
 * x1 = omega b / diag(A) (poms_op_diag_scale) formed as the planes are read,
 * x_out = x1 + omega (b - A x1) / diag(A).  With want_norm, ||dr_2||^2 partials
 * go to scratch[0, count) and ||x1||^2 = ||dr_1||^2 partials to
 * scratch[count, 2 count).  Replaces the first two iterations of
 * `sources/solvers.py:207-219` (x0 = None).  3D, and 2D without ghost corners;
 * variants 8-10, arrays < 2 GiB (poms_op_from_zero_supported).               */
int poms_op_jacobi_from_zero(poms_op* op, double omega, const double* b, double* x_out,
                             int64_t z_begin, int64_t z_end, int want_norm, void* stream);
int poms_op_from_zero_supported(poms_op* op, int* yes);
/* Two damped-Jacobi sweeps k, k+1 of `sources/solvers.py:207-219` in one launch:
 * poms_op_run_reduce2 with epilogue 6 (x -> y; plane range [0, 1)): norm_out <-
 * ||dr_{k+1}||^2, dot_out <- ||dr_k||^2; x_k is not stored.  y is bitwise the
 * result of two poms_op_jacobi_sweep calls (variant 9).  One-rank 2D p = 3
 * Kronecker operators whose sweeps run variant 9, arrays < 2 GiB (1 in *yes);
 * poms_pcg_jacobi uses it for the smoother's middle sweeps (POMS_J2=0: off).    */
int poms_op_sweep2_supported(poms_op* op, int* yes);
/* Damped-Jacobi sweeps 1-3 of `sources/solvers.py:207-219` from x0 = 0 in one launch
 * (operators of poms_op_sweep2_supported): x1 = omega b / diag(A) formed as b is
 * read, then two sweeps; x_out = x3, bitwise poms_op_jacobi_from_zero followed by
 * poms_op_jacobi_sweep.  norms_out (device, 3 doubles, or NULL) <- ||x1||^2,
 * ||dr_2||^2, ||dr_3||^2.  poms_pcg_jacobi starts the smoother with it where it runs
 * the two-sweep launches (POMS_J2FZ=0: off).                                      */
int poms_op_jacobi3_from_zero(poms_op* op, double omega, const double* b, double* x_out, double* norms_out,
                              void* stream);
/* x = scale * b / diag(A) on the interior.  With scale = 1 this is
 * `jacobi(A, b)` (`sources/solvers.py:139-163`); with scale = omega it is the
 * first damped-Jacobi sweep from x0 = 0 (A.0 = 0 exactly).                    */
int poms_op_diag_scale(poms_op* op, double scale, const double* b, double* x,
                       int want_norm, void* stream);
/* Number of norm partials the last want_norm launch on this op produced. */
int poms_op_last_partials(poms_op* op, int64_t* count);

/* Host-pointer drop-in for the pyccel kernel `kron_dot_pyccel_2d(starts, ends,
 * pads, X, X_tmp, Y, A, B)` (`pyccel/pyccel_functions.py:3-21`).  X, X_tmp, Y
 * are the local padded arrays ((e0-s0+1+2p0) x (e1-s1+1+2p1), C order); A, B
 * are GLOBAL band arrays ((n_global_d) x (2p_d+1)).  X_tmp is accepted for
 * signature parity and left untouched (the intermediate lives in LDS).
 * Synchronous.  starts/ends are global indices as in spl.                     */
int poms_kron_dot_2d(poms_ctx* ctx, const int64_t* starts, const int64_t* ends,
                     const int64_t* pads, const double* X, double* X_tmp,
                     double* Y, const double* A, int64_t a_rows,
                     const double* B, int64_t b_rows);

/* ---- vector kernels (interior only; ghosts untouched) --------------------- */
/* z = a*x + b*y.  Replaces spl StencilVector `a*v + w` algebra used at
 * `sources/solvers.py:106,107,124,217`.  z may alias x or y.                  */
int poms_vec_axpby(poms_ctx* ctx, const poms_layout* L, double a, const double* x,
                   double b, const double* y, double* z, void* stream);
/* z = a*x (b-free form, safe on uninitialised z) */
int poms_vec_scale(poms_ctx* ctx, const poms_layout* L, double a, const double* x,
                   double* z, void* stream);
int poms_vec_fill(poms_ctx* ctx, const poms_layout* L, double v, double* z, void* stream);
/* Zero everything OUTSIDE the interior (ghost planes / rows / columns and dead
 * pitch columns; the interior is untouched): the zero ghost regions a new spl
 * `StencilVector(V)` has (`sources/solvers.py:71,169`), one launch.            */
int poms_vec_zero_ghosts(poms_ctx* ctx, const poms_layout* L, double* z, void* stream);
/* Local (un-reduced across ranks) inner product over the interior; result to
 * out_dev[0].  Replaces `StencilVector.dot` (`sources/solvers.py:87,91,104,111`). */
int poms_vec_dot(poms_ctx* ctx, const poms_layout* L, const double* x,
                 const double* y, double* out_dev, void* stream);
/* PCG update, fused: x += alpha p; r -= alpha q; out_dev[0] = r.r (local).
 * Replaces `sources/solvers.py:106-111` (minus the discarded A.dot(r) at :109). */
int poms_pcg_update(poms_ctx* ctx, const poms_layout* L, double alpha, double* x,
                    const double* p, double* r, const double* q, double* out_dev,
                    void* stream);
/* r -= alpha q; out_dev[0] = r.r (local).  With poms_pcg_xp_update this splits
 * poms_pcg_update so that x's update can ride on the p update one psolve later. */
int poms_pcg_r_update(poms_ctx* ctx, const poms_layout* L, double alpha, double* r,
                      const double* q, double* out_dev, void* stream);
/* x += alpha p; p = s + beta p (both from the old p, one pass):
 * `sources/solvers.py:106` of iteration k and :124 of the same iteration.    */
int poms_pcg_xp_update(poms_ctx* ctx, const poms_layout* L, double alpha, double beta,
                       double* x, double* p, const double* s, void* stream);
/* Device-coefficient forms of axpby / pcg_r_update / pcg_xp_update: the kernel
 * reads (a, b) = ab_dev[0..1] (alpha = alpha_dev[0]) from device memory, so
 * pcg's alpha = s.r / p.q and beta = s.r / s.r_old are formed on the device and
 * never synchronise the host (`sources/solvers.py:105,107,123-124`).         */
int poms_vec_axpby_dev(poms_ctx* ctx, const poms_layout* L, const double* ab_dev, const double* x,
                       const double* y, double* z, void* stream);
int poms_pcg_r_update_dev(poms_ctx* ctx, const poms_layout* L, const double* alpha_dev, double* r,
                          const double* q, double* out_dev, void* stream);
int poms_pcg_xp_update_dev(poms_ctx* ctx, const poms_layout* L, const double* ab_dev, double* x, double* p,
                           const double* s, void* stream);
/* Reduce `count` partials from the context scratch into out_dev[0]. */
int poms_reduce_partials(poms_ctx* ctx, int64_t count, double* out_dev, void* stream);
/* Same, starting at scratch[offset]. */
int poms_reduce_partials_at(poms_ctx* ctx, int64_t offset, int64_t count, double* out_dev,
                            void* stream);

/* ---- inter-grid transfer (knot insertion) --------------------------------- */
/* P_d are HOST dense row-major (nf_global_d x nc_d) prolongation factors
 * (`P1 = matrix_multi_stages(Ts, nc, p, Tc)`, `sources/mg_jac.py:67-70`).
 * Fine vectors use `fine` layout (local slab, axis-0 global offset g0);
 * coarse vectors are dense (no ghosts) C-order nc0*nc1*nc2 (2D: nc0 = 1).
 * nc_d <= 32.                                                                 */
int poms_transfer_create(poms_ctx* ctx, int ndim, const poms_layout* fine,
                         int64_t g0, const int64_t* nf_global, const int64_t* nc,
                         const double* const* P, poms_transfer** tr);
int poms_transfer_destroy(poms_transfer* tr);
/* coarse = (P0 (x) P1 (x) P2)^T fine  (local slab contribution; the caller
 * all-reduces across ranks).  Replaces `rc = R.dot(rf.toarray())`,
 * `sources/mg_jac.py:94`.                                                     */
int poms_restrict(poms_transfer* tr, const double* fine, double* coarse, void* stream);
/* fine += (P0 (x) P1 (x) P2) coarse on the local slab.
 * Replaces `xc_p = P.dot(xc)` + `xf = xf + rf` (`sources/mg_jac.py:102-112`). */
int poms_prolong_add(poms_transfer* tr, const double* coarse, double* fine, void* stream);
/* Fused residual -> restriction (`sources/mg_jac.py:93-94`, `rf = bf - Af.dot(xf)`
 * then `rc = R.dot(rf)`): set once per operator, then
 *   coarse = R (b - A x)   (local slab contribution; the caller all-reduces)
 * with r = b - A x never stored.  G[r] are HOST dense row-major (rows_d x nc_d)
 * matrices F_r^T P_d, one per role of poms_op_create's factor list (FORM_SUM: A0 M0
 * A1 B1 M2 K2; FORM_SINGLE: F0 - F1 - F2 -; 2D: roles 0 and 1 unused), rows as the
 * P_d given to poms_transfer_create.  x needs no up-to-date ghost regions.
 * Results equal poms_op_residual + poms_restrict to rounding (R b - (R A) x is
 * summed in another order).  Dense-P transfers only (nc_d <= 32).              */
int poms_transfer_set_operator(poms_transfer* tr, int form, const double* const* G);
int poms_resid_restrict(poms_transfer* tr, const double* b, const double* x, double* coarse,
                        void* stream);

/* ---- coarse solve ---------------------------------------------------------- */
/* y = Minv x with a dense (n x n) row-major DEVICE matrix (the factorised
 * Galerkin coarse operator).  Replaces `splu(Ac).solve(rc)`,
 * `sources/mg_jac.py:98-99`.                                                  */
int poms_dense_matvec(poms_ctx* ctx, int64_t n, const double* Minv, const double* x,
                      double* y, void* stream);

/* ---- Kronecker direct solve (GLT post-smoother preconditioner) --------------- */
/* X = (A0^-1 (x) A1^-1 (x) A2^-1) Y by banded LU line solves along each axis
 * (axis 0 first, as the reference).  ab[d] is a HOST column-major (ldab[d] x n_d)
 * array in LAPACK band storage of the UNFACTORED matrix of axis d, with kl[d]
 * spare rows for fill-in: a(i, j) at ab[(kl+ku+i-j) + j*ldab], ldab >= 2kl+ku+1
 * -- the layout `to_bnd` builds (`sources/kron_product.py:179-191`,
 * `pyccel/test_kron_solve.py:37-44`).  Each is factorised once on the host with
 * partial pivoting (LAPACK dgbtf2, as scipy's dgbtrf for kl < 32); axis-0 rows are
 * global (n0_global).  2D/1D: leading unused axes have n = 1, pads = 0 and a NULL
 * band.  kl + ku <= 16.
 * Replaces: `dgbtrf` + the per-line `dgbtrs` loops of `kron_solve_par_bnd_pyccel_2d`
 * / `_3d` (`pyccel/pyccel_functions.py:114-248`) and `kron_solve_par` /
 * `kron_solve_serial` (`sources/kron_product.py:93-158`, dense dgetrf there).     */
int poms_ksolve_create(poms_ctx* ctx, int ndim, const poms_layout* layout, int64_t n0_global,
                       const double* const* ab, const int64_t* ldab, const int* kl, const int* ku,
                       poms_ksolve** ks);
/* As poms_ksolve_create with the global extent of EVERY axis (n_global[3]; the
 * factor of axis d is n_global[d] x n_global[d]): the block layouts of a Cart
 * decomposition, whose distributed axes are solved on transposed lines with
 * poms_kron_solve_lines_dense (replaces the per-line `Allgatherv` over the axis
 * sub-communicators of `kron_solve_par` / `kron_solve_bnd_par`,
 * `sources/kron_product.py:119-170, 191-238`).                                  */
int poms_ksolve_create_global(poms_ctx* ctx, int ndim, const poms_layout* layout, const int64_t* n_global,
                              const double* const* ab, const int64_t* ldab, const int* kl, const int* ku,
                              poms_ksolve** ks);
int poms_ksolve_destroy(poms_ksolve* ks);
/* dgbtrf info per axis (0 = ok, j+1 = u(j,j) is exactly zero; solves then fail). */
int poms_ksolve_info(poms_ksolve* ks, int* info3);
/* Absolute 0-based pivot rows of axis `axis` (n_d ints, host). */
int poms_ksolve_pivots(poms_ksolve* ks, int axis, int* ipiv);
/* x = solve(y) on the interior of padded device arrays (x may alias y; ghosts
 * untouched).  All axes must be local (n == n_global).                        */
int poms_kron_solve(poms_ksolve* ks, const double* y, double* x, void* stream);
/* One axis only (it must be local: n[axis] == n_global[axis]). */
int poms_kron_solve_axis(poms_ksolve* ks, int axis, const double* in, double* out, void* stream);
/* Axis-0 solve of a dense C-order (n0_global, m) device buffer (the all-to-all
 * transposed slab of a distributed solve; replaces the per-line `Allgatherv` +
 * `dgbtrs` of `pyccel/pyccel_functions.py:150-155`).  out may alias in.         */
int poms_kron_solve_axis0_dense(poms_ksolve* ks, const double* in, double* out, int64_t m, void* stream);
/* Lines of axis `axis` (any axis): a dense C-order (n_global[axis], m) device
 * buffer, column j = one line.  out may alias in.                               */
int poms_kron_solve_lines_dense(poms_ksolve* ks, int axis, const double* in, double* out, int64_t m, void* stream);
/* Host-pointer drop-ins of `kron_solve_par_bnd_pyccel_2d(A_bnd, la, ua, B_bnd, lb,
 * ub, X, Y, points, pads, ...)` / `_3d` on one rank: X, Y are padded C-order
 * host arrays ((n_d + 2 pads_d) per axis); X's interior is overwritten, its
 * ghosts are kept.  Synchronous.                                               */
int poms_kron_solve_bnd_2d(poms_ctx* ctx, const double* A_bnd, int64_t lda, int la, int ua,
                           const double* B_bnd, int64_t ldb, int lb, int ub, double* X, const double* Y,
                           const int64_t* points, const int64_t* pads);
int poms_kron_solve_bnd_3d(poms_ctx* ctx, const double* A_bnd, int64_t lda, int la, int ua,
                           const double* B_bnd, int64_t ldb, int lb, int ub, const double* C_bnd,
                           int64_t ldc, int lc, int uc, double* X, const double* Y,
                           const int64_t* points, const int64_t* pads);

/* ---- native RCCL communicator (slab ghost exchange, scalar all-reduces) ------ */
/* Replaces `_update_ghost_regions_parallel` (`pyccel/kron_product.py:21-41`) and
 * the solvers' `comm.allreduce` (`sources/solvers.py:87-124`, `sources/mg_jac.py:95`).
 * All RCCL work goes to one communication stream in host issue order, ordered
 * against the caller's stream with events.                                    */
int poms_comm_id_bytes(void);
int poms_comm_unique_id(char* out, int len);          /* rank 0; broadcast it */
int poms_comm_create(int device, const char* id, int rank, int nranks, poms_comm** out);
int poms_comm_destroy(poms_comm* comm);
int poms_comm_stream(poms_comm* comm, void** stream);
/* Host transport: the same communicator API and schedule (poms_op_run_dist,
 * lazy ring slots) with the data moved by host callbacks instead of RCCL, for
 * process groups without RCCL peers (e.g. gloo ranks sharing one GPU in the
 * tests).  Each call synchronises the caller's stream and stages through host
 * memory.  exchange: send_lo (cnt doubles) to prev and recv_lo from it, send_hi
 * to next and recv_hi from it (prev / next = -1: none); allreduce: in-place sum
 * of cnt doubles over the ranks.  Callbacks return 0 on success.              */
typedef int (*poms_host_exchange_fn)(void* user, const double* send_lo, double* recv_lo, const double* send_hi,
                                     double* recv_hi, int64_t cnt, int prev, int next);
typedef int (*poms_host_allreduce_fn)(void* user, double* buf, int64_t cnt);
int poms_comm_create_host(int device, int rank, int nranks, poms_host_exchange_fn exchange,
                          poms_host_allreduce_fn allreduce, void* user, poms_comm** out);
int poms_comm_is_host(poms_comm* comm, int* yes);
/* Host transport on one node: attach the node-local shared-memory block named by
 * `id` (id_len bytes, identical on every rank; collective over the ranks through
 * the all-reduce callback) so that the lazily read sums (poms_comm_wait) are added
 * in shared memory as on the RCCL path.  *attached = 0 when not every rank found
 * all the others (the callback then keeps doing the sums).                     */
int poms_comm_host_attach_shm(poms_comm* comm, const char* id, int id_len, int* attached);
/* 1 when poms_comm_wait sums through the node-local shared-memory block.       */
int poms_comm_uses_shm(poms_comm* comm, int* yes);
/* data -> plane 0 of the padded local array (first ghost plane); the first /
 * last `width` owned planes go to prev / next (-1: none), the neighbours'
 * planes land in the ghost planes.  Starts after the work queued on `stream`;
 * poms_halo_finish makes `stream` wait for the exchange.                       */
int poms_halo_start(poms_comm* comm, double* data, int64_t plane_elems, int64_t n_local, int pad,
                    int width, int prev, int next, void* stream);
int poms_halo_finish(poms_comm* comm, void* stream);
/* Peer transport for poms_halo_start (every rank the same enable / wgs): the
 * exchange becomes ONE kernel of `wgs` workgroups (1..256) on the communication
 * stream that stores the boundary planes straight into the neighbours' mailboxes
 * (IPC-mapped device memory; xGMI peer stores between GPUs) and copies its own
 * mailboxes into the ghost planes, ordered by per-workgroup flag slots -- no RCCL
 * call and no host step, so it can be captured into a graph.  The mailboxes are
 * (re)built, collectively with the two neighbours, at the first exchange of a
 * larger size or poms_comm_peer_reserve (never inside a capture).  A wait that
 * exceeds 20 s gives up and sets the timed-out flag (poms_comm_peer_status)
 * instead of hanging the GPU.  Replaces the same `_update_ghost_regions_parallel`
 * (`pyccel/kron_product.py:21-41`).                                            */
int poms_comm_set_peer(poms_comm* comm, int enable, int wgs);
int poms_comm_peer_reserve(poms_comm* comm, int64_t cnt, int prev, int next);
int poms_comm_peer_status(poms_comm* comm, int* active, int* fine_grained, int* timed_out);
/* Fails (returns 1, poms_last_error says why) if a peer exchange of this
 * communicator has timed out: its ghost planes, and every result computed from
 * them, are invalid.  No synchronisation (reads a host-mapped flag the exchange
 * kernel sets); poms_comm_wait and poms_pcg_jacobi run it themselves.  The peer
 * mailboxes cannot be rebuilt (a larger exchange, other neighbours, set_peer off or
 * another wgs) once an exchange was captured into a graph: that call fails too.
 * Neighbours must use the same wgs (checked when the mailboxes are built).      */
int poms_comm_check(poms_comm* comm);
/* In-place global sum of `count` doubles after the work queued on `stream`;
 * wait_back: `stream` waits for the result, else it is ready on the
 * communication stream only.                                                  */
int poms_allreduce_sum(poms_comm* comm, double* buf, int64_t count, void* stream, int wait_back);
/* Lazily read global sums (values only the host reads: stop tests).  A ring of
 * slots of 2 doubles in pinned, device-mapped host memory: a launch reduces the
 * rank's local sum into poms_comm_slot's slot; poms_allreduce_to_host records the
 * launch (queued on `stream`) and where the result goes; poms_comm_wait spins
 * until the slot is written, sums it over the ranks ON THE HOST (node-local
 * shared memory; the host transport's callback; RCCL synchronously when the
 * ranks span nodes) and leaves the sums in host_dst.  Nothing is queued on the
 * communication stream.  Every rank must wait on the same tickets in the same
 * order (the sums are collective).                                            */
int poms_comm_slot(poms_comm* comm, double** dev_slot, int* ticket);
int poms_allreduce_to_host(poms_comm* comm, int ticket, int count, double* host_dst, void* stream);
int poms_comm_wait(poms_comm* comm, int ticket);
/* One distributed operator call (epilogue as poms_op_run_reduce2) from one host
 * call: with `exchange` the p-plane ghost exchange of x (xplanes = plane 0 of its
 * padded array) overlaps the interior planes and both boundaries follow in one
 * launch.  Reductions go to norm_dev / dot_dev (device, local sums), or with
 * lazy_count > 0 to a ring slot all-reduced and copied to host_dst on the
 * communication stream ([dot, norm] with both; *ticket for poms_comm_wait).   */
int poms_op_run_dist(poms_op* op, poms_comm* comm, int epilogue, double omega, const double* x,
                     double* y, const double* b, double* xplanes, int64_t plane_elems,
                     int64_t n_local, int pad, int pmax, int prev, int next, int exchange,
                     int want_norm, int want_dot, double* norm_dev, double* dot_dev,
                     int lazy_count, double* host_dst, int* ticket, void* stream);

/* ---- native smoother loop ----------------------------------------------------- */
/* pcg(A, damped_jacobi, b, x0, tol, maxiter) of `sources/solvers.py:69-135` with the
 * damped-Jacobi preconditioner of :167-235 (omega, jtol, jmaxiter), as ONE host call:
 * the launches, device-side scalars (alpha = s.r / p.q, beta = s.r / s.r_old) and stop
 * tests of poms_amd.solvers.pcg -- bitwise the same iterates -- without a Python round
 * trip per launch; each norm is read one launch after the next one is queued.  The
 * V-cycle's pre/post smoothing (`sources/mg_jac.py:88,104`).
 * comm != NULL: the slab-distributed form (ghost exchange per operator call through
 * poms_op_run_dist with neighbours prev / next, sums all-reduced).
 * x: in = x0 when has_x0, out = the solution (current ghosts not required).
 * work: 5 vectors of the operator's layout with zero ghosts (r, q and three
 * preconditioner buffers), not aliasing b or x.
 * Speculative mode (opt-in, POMS_PCG_SPEC=1; slower on the measured cycles): the whole
 * call is queued without reading a stop test, the tests are evaluated once the stream
 * drains, and if one fires the call is repeated step by step from the restored x0 --
 * the same bits either way.  Its launches are captured once into a hipGraph per
 * (buffers, options, timing) and replayed when there is no communicator
 * (POMS_PCG_GRAPH=0: never).                                                      */
typedef struct poms_pcg_opts {
    double tol;      /* pcg: stop when r.r < tol * ||r0|| (the reference's mixed norms) */
    int maxiter;
    double jtol;     /* damped Jacobi: stop when dr.dr < jtol^2                         */
    int jmaxiter;
    double omega;    /* 2/3                                                             */
    int prev, next;  /* slab neighbours (comm != NULL), -1: none                        */
} poms_pcg_opts;
typedef struct poms_pcg_info {
    int niter;
    int success;
    double res_norm;
} poms_pcg_info;
int poms_pcg_jacobi(poms_op* op, poms_comm* comm, const poms_pcg_opts* opts, const double* b, double* x,
                    int has_x0, double* const* work, poms_pcg_info* info, void* stream);
/* Launch timing: with enable, operator launches on this op (any caller, including
 * poms_pcg_jacobi) of `epilogue` (-1: all; see poms_op_kernel_variant), every
 * `every`-th one, are bracketed by HIP events on their stream; enabling clears the
 * record and pre-creates `reserve` event pairs (an event record costs the host a
 * few microseconds: sample to keep the timed work unperturbed).
 * poms_op_timing_read sums the recorded launches of one epilogue: total
 * milliseconds, launch count and output DOFs (synchronises on the events).      */
int poms_op_timing(poms_op* op, int enable, int epilogue, int every, int reserve);
/* Speculative smoother calls of this operator: stats[0] calls, [1] calls repeated
 * step by step (a stop test fired), [2] graph captures, [3] graph replays of an
 * earlier capture.                                                                */
int poms_op_spec_stats(poms_op* op, int* stats);
int poms_op_timing_read(poms_op* op, int epilogue, double* total_ms, int64_t* launches, int64_t* dofs);

#ifdef __cplusplus
}
#endif
#endif /* POMS_HIP_H */
