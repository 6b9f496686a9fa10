"""CPU restatement of the parts of the (absent) third-party ``spl`` library the
reference uses -- TEST INFRASTRUCTURE ONLY (golden-fixture generation).

The reference imports ``spl`` (`requirements.txt:4`, no version pin) for its
stencil linear algebra and B-spline spaces; the package is not installed and
not vendored.  To run the reference's own ``assembly_2d``, ``solvers.pcg`` /
``damped_jacobi``, ``utils.kron_dot_ref`` and the ``mg_jac.py`` driver in this
container, ``install()`` places NumPy stand-ins with spl's documented semantics
in ``sys.modules``:

* ``spl.linalg.stencil``: ``StencilVectorSpace(npts, pads, periods)``,
  ``StencilVector`` (padded ``_data``, global-index ``[]``, algebra, ``dot``,
  ``toarray``, ``update_ghost_regions`` = no-op on one rank),
  ``StencilMatrix`` (``M[i, k]`` / ``M[i1, i2, k1, k2]`` with offsets
  ``k in [-p, p]``, ``dot``, ``tocoo/tocsr/toarray``, ``remove_spurious_entries``)
  -- `slides/content.tex:256-290`;
* ``spl.fem.splines.SplineSpace`` / ``spl.fem.tensor.TensorFemSpace``: spans
  (1-based, as `sources/matrix_assembler.py:147` ``i1 = span - p - 1 + il``),
  basis values/derivatives at ``p+1`` Gauss points per element, weights;
* ``spl.core.interface``: ``make_open_knots``, ``matrix_multi_stages``;
* ``mpi4py.MPI``: a one-rank ``COMM_WORLD``.

Everything here is the build's own restatement; goldens produced through it pin
the reference's *code* (assembly, solvers, driver) on top of these semantics.
"""
from __future__ import annotations

import sys
import types

import numpy as np
import scipy.sparse as sp


# ---------------------------------------------------------------------------
class _SubComm:
    """Single-rank sub-communicator: ``Allgatherv`` copies the local block into the
    receive buffer (``recv`` or ``[recv, sizes, displs(, type)]``)."""

    def Allgatherv(self, send, recv):
        buf = recv[0] if isinstance(recv, (list, tuple)) else recv
        send = np.asarray(send)
        buf[:send.size] = send.reshape(-1)

    def py2f(self):
        return 0


class _Cart:
    def __init__(self, ndim):
        self._rank = 0
        self._size = 1
        self.nprocs = [1] * ndim
        self.coords = [0] * ndim
        self.subcomm = [_SubComm() for _ in range(ndim)]


class StencilVectorSpace:
    def __init__(self, npts, pads, periods=None):
        self.npts = tuple(int(n) for n in npts)
        self.pads = tuple(int(p) for p in pads)
        self.ndim = len(self.npts)
        self.periods = tuple(periods) if periods is not None else (False,) * self.ndim
        self.starts = tuple(0 for _ in self.npts)
        self.ends = tuple(n - 1 for n in self.npts)
        self.cart = _Cart(self.ndim)
        self.dimension = int(np.prod(self.npts))
        self.shape = tuple(n + 2 * p for n, p in zip(self.npts, self.pads))


class StencilVector:
    def __init__(self, V):
        self._space = V
        self._data = np.zeros(V.shape)

    space = property(lambda self: self._space)
    starts = property(lambda self: self._space.starts)
    ends = property(lambda self: self._space.ends)
    pads = property(lambda self: self._space.pads)
    shape = property(lambda self: (self._space.dimension,))

    def _idx(self, key):
        if not isinstance(key, tuple):
            key = (key,)
        out = []
        for k, s, p in zip(key, self._space.starts, self._space.pads):
            if isinstance(k, slice):
                if k == slice(None):
                    out.append(slice(p, p + self._space.npts[len(out)]))
                else:
                    a = s if k.start is None else k.start
                    b = self._space.ends[len(out)] + 1 if k.stop is None else k.stop
                    out.append(slice(a - s + p, b - s + p))
            else:
                out.append(int(k) - s + p)
        return tuple(out)

    def __getitem__(self, key):
        return self._data[self._idx(key)]

    def __setitem__(self, key, value):
        self._data[self._idx(key)] = value

    def copy(self):
        v = StencilVector(self._space)
        v._data[...] = self._data
        return v

    def _new(self, data):
        v = StencilVector(self._space)
        v._data[...] = data
        return v

    def __add__(self, o):
        return self._new(self._data + o._data)

    def __sub__(self, o):
        return self._new(self._data - o._data)

    def __mul__(self, a):
        return self._new(self._data * a)

    __rmul__ = __mul__

    def __neg__(self):
        return self._new(-self._data)

    def _interior(self):
        return self._data[tuple(slice(p, p + n) for p, n in zip(self._space.pads, self._space.npts))]

    def dot(self, o):
        return float(np.vdot(self._interior(), o._interior()))

    def update_ghost_regions(self, direction=None):
        pass  # one rank, non-periodic: ghosts stay zero

    def toarray(self):
        return self._interior().reshape(-1).copy()


class StencilMatrix:
    def __init__(self, V, W=None):
        self._domain = V
        self._codomain = W if W is not None else V
        nd = V.ndim
        self.pads = V.pads
        self.starts, self.ends = V.starts, V.ends
        self._data = np.zeros(V.shape + tuple(2 * p + 1 for p in V.pads))
        self._nd = nd

    shape = property(lambda self: (self._domain.dimension, self._domain.dimension))

    def _idx(self, key):
        nd = self._nd
        ii, kk = key[:nd], key[nd:]
        out = []
        for i, p, s in zip(ii, self.pads, self.starts):
            out.append(slice(p, p + self._domain.npts[len(out)]) if isinstance(i, slice) and i == slice(None)
                       else int(i) - s + p)
        for k, p in zip(kk, self.pads):
            out.append(int(k) + p)
        return tuple(out)

    def __getitem__(self, key):
        return self._data[self._idx(key)]

    def __setitem__(self, key, value):
        self._data[self._idx(key)] = value

    def remove_spurious_entries(self):
        nd = self._nd
        for idx in np.ndindex(*self._domain.npts):
            for kk in np.ndindex(*[2 * p + 1 for p in self.pads]):
                ks = [k - p for k, p in zip(kk, self.pads)]
                if any(not 0 <= i + k < n for i, k, n in zip(idx, ks, self._domain.npts)):
                    self._data[tuple(i + p for i, p in zip(idx, self.pads)) + kk] = 0.0

    def tocoo(self):
        nd = self._nd
        npts = self._domain.npts
        rows, cols, vals = [], [], []
        for idx in np.ndindex(*npts):
            r = np.ravel_multi_index(idx, npts)
            for kk in np.ndindex(*[2 * p + 1 for p in self.pads]):
                j = tuple(i + k - p for i, k, p in zip(idx, kk, self.pads))
                if all(0 <= jj < n for jj, n in zip(j, npts)):
                    v = self._data[tuple(i + p for i, p in zip(idx, self.pads)) + kk]
                    if v != 0.0:
                        rows.append(r)
                        cols.append(np.ravel_multi_index(j, npts))
                        vals.append(v)
        n = int(np.prod(npts))
        return sp.coo_matrix((vals, (rows, cols)), shape=(n, n))

    def tocsr(self):
        return self.tocoo().tocsr()

    def toarray(self):
        return self.tocoo().toarray()

    def dot(self, x):
        """v[i] = Σ_k M[i, k] x[i + k] (`slides/content.tex:285-290`)."""
        V = self._domain
        y = StencilVector(V)
        xd = x._data
        nd = self._nd
        out = np.zeros(V.npts)
        for kk in np.ndindex(*[2 * p + 1 for p in self.pads]):
            ks = [k - p for k, p in zip(kk, self.pads)]
            coef = self._data[tuple(slice(p, p + n) for p, n in zip(self.pads, V.npts)) + kk]
            xs = xd[tuple(slice(p + k, p + k + n) for p, k, n in zip(self.pads, ks, V.npts))]
            out += coef * xs
        y._data[tuple(slice(p, p + n) for p, n in zip(self.pads, V.npts))] = out
        return y


# ---------------------------------------------------------------------------
def make_open_knots(p, n):
    ncells = n - p
    return np.concatenate([np.zeros(p + 1), np.arange(1, ncells) / ncells, np.ones(p + 1)])


def _basis_ders(T, p, x, span):
    """Non-zero B-splines and first derivatives at x (direct Cox-de Boor)."""
    # degree-0 .. p triangle of values
    N = np.zeros(p + 1)
    N[0] = 1.0
    left, right = np.zeros(p + 1), np.zeros(p + 1)
    Nlow = None
    for j in range(1, p + 1):
        left[j] = x - T[span + 1 - j]
        right[j] = T[span + j] - x
        saved = 0.0
        Nnew = np.zeros(p + 1)
        for r in range(j):
            tmp = N[r] / (right[r + 1] + left[j - r])
            Nnew[r] = saved + right[r + 1] * tmp
            saved = left[j - r] * tmp
        Nnew[j] = saved
        if j == p:
            Nlow = N[:p].copy()
        N = Nnew
    D = np.zeros(p + 1)
    if p > 0:
        # B'_{i,p} = p/(t_{i+p}-t_i) B_{i,p-1} - p/(t_{i+p+1}-t_{i+1}) B_{i+1,p-1}
        for r in range(p + 1):
            i = span - p + r
            a = Nlow[r - 1] if r - 1 >= 0 else 0.0   # B_{i, p-1} lives at index r-1 of degree p-1
            bb = Nlow[r] if r < p else 0.0            # B_{i+1, p-1}
            d1 = T[i + p] - T[i]
            d2 = T[i + p + 1] - T[i + 1]
            D[r] = (p * a / d1 if d1 > 0 else 0.0) - (p * bb / d2 if d2 > 0 else 0.0)
    return N, D


class SplineSpace:
    def __init__(self, degree, knots=None, grid=None, nquad=None):
        p = int(degree)
        if knots is None:
            grid = np.asarray(grid, dtype=float)
            knots = np.concatenate([[grid[0]] * (p + 1), grid[1:-1], [grid[-1]] * (p + 1)])
        T = np.asarray(knots, dtype=float)
        self.degree = p
        self.knots = T
        self.nbasis = len(T) - p - 1
        self.quad_order = p + 1 if nquad is None else nquad
        spans0 = [i for i in range(p, self.nbasis) if T[i + 1] > T[i]]
        self.ne = len(spans0)
        self.spans = np.array([s + 1 for s in spans0])   # 1-based as spl
        xg, wg = np.polynomial.legendre.leggauss(self.quad_order)
        nq = self.quad_order
        self.points = np.zeros((nq, self.ne))
        self.weights = np.zeros((nq, self.ne))
        self.basis = np.zeros((p + 1, 2, nq, self.ne))
        for e, s in enumerate(spans0):
            a, b = T[s], T[s + 1]
            for g in range(nq):
                x = a + 0.5 * (b - a) * (xg[g] + 1)
                self.points[g, e] = x
                self.weights[g, e] = 0.5 * (b - a) * wg[g]
                N, D = _basis_ders(T, p, x, s)
                self.basis[:, 0, g, e] = N
                self.basis[:, 1, g, e] = D
        self.vector_space = StencilVectorSpace([self.nbasis], [p], [False])


class TensorFemSpace:
    def __init__(self, *spaces, comm=None):
        self.spaces = list(spaces)
        self.vector_space = StencilVectorSpace([s.nbasis for s in spaces], [s.degree for s in spaces],
                                               [False] * len(spaces))


def matrix_multi_stages(ts, nc, p, knots):
    """Sequential Boehm insertion of ``ts`` into ``knots`` -> (n_f x n_c) prolongation."""
    T = np.asarray(knots, dtype=float)
    P = np.eye(nc)
    for t in sorted(ts):
        n = len(T) - p - 1
        k = max(i for i in range(p, n) if T[i] <= t)
        A = np.zeros((n + 1, n))
        for i in range(n + 1):
            if i <= k - p:
                al = 1.0
            elif i >= k + 1:
                al = 0.0
            else:
                al = (t - T[i]) / (T[i + p] - T[i])
            if i < n:
                A[i, i] += al
            if i >= 1:
                A[i, i - 1] += 1 - al
        T = np.sort(np.concatenate([T, [t]]))
        P = A @ P
    return sp.csr_matrix(P)


# ---------------------------------------------------------------------------
class _Comm:
    def Get_rank(self):
        return 0

    def Get_size(self):
        return 1

    def Barrier(self):
        pass

    def allreduce(self, x, op=None):
        return x


def install():
    """Register the stand-ins under the module names the reference imports."""
    spl = types.ModuleType("spl")
    linalg = types.ModuleType("spl.linalg")
    stencil = types.ModuleType("spl.linalg.stencil")
    stencil.StencilVectorSpace = StencilVectorSpace
    stencil.StencilVector = StencilVector
    stencil.StencilMatrix = StencilMatrix
    fem = types.ModuleType("spl.fem")
    splines = types.ModuleType("spl.fem.splines")
    splines.SplineSpace = SplineSpace
    tensor = types.ModuleType("spl.fem.tensor")
    tensor.TensorFemSpace = TensorFemSpace
    core = types.ModuleType("spl.core")
    interface = types.ModuleType("spl.core.interface")
    interface.make_open_knots = make_open_knots
    interface.matrix_multi_stages = matrix_multi_stages
    ddm = types.ModuleType("spl.ddm")
    cart = types.ModuleType("spl.ddm.cart")
    cart.Cart = object
    mpi4py = types.ModuleType("mpi4py")
    MPI = types.ModuleType("mpi4py.MPI")
    MPI.COMM_WORLD = _Comm()
    MPI.SUM = "sum"
    MPI.DOUBLE = "double"
    import time as _t
    MPI.Wtime = _t.perf_counter
    mpi4py.MPI = MPI
    for name, mod in {
        "spl": spl, "spl.linalg": linalg, "spl.linalg.stencil": stencil, "spl.fem": fem,
        "spl.fem.splines": splines, "spl.fem.tensor": tensor, "spl.core": core,
        "spl.core.interface": interface, "spl.ddm": ddm, "spl.ddm.cart": cart,
        "mpi4py": mpi4py, "mpi4py.MPI": MPI,
    }.items():
        sys.modules[name] = mod
