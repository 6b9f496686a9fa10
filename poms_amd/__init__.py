"""poms_amd -- MI355X (gfx950) hot path of the pyccel/poms B-spline multigrid.

Public surface mirrors the reference (`sources/solvers.py`,
`sources/kron_product.py`, `sources/multilevels.py`, `sources/mg_jac.py`):

    from poms_amd import StencilVectorSpace, StencilVector, KronOperator
    from poms_amd import pcg, damped_jacobi, jacobi, kron_dot_v2, TwoLevelVCycle

Importing the package loads ``libpoms_hip.so``; it raises if the library is
missing (there is no CPU fallback).  Device objects additionally need a GPU.
"""
from . import _lib  # noqa: F401  (fails loudly without the HIP library)
from .splines import (assemble_1d, collocation_cardinal_splines, make_open_knots,  # noqa: F401
                      matrix_multi_stages, uniform_knots)

__all__ = [
    "StencilVectorSpace", "StencilVector", "StencilMatrix1D", "KronOperator", "StencilMatrix",
    "pcg", "damped_jacobi", "jacobi", "kron_dot_v2", "kron_dot_pyccel_2d",
    "knots_to_insert", "KronTransfer", "TwoLevelVCycle", "SlabDistribution",
    "assemble_1d", "make_open_knots", "uniform_knots", "matrix_multi_stages",
    "pcg_glt", "pcg_kron", "KronSolver", "kron_solve_serial", "kron_solve_par", "to_bnd",
    "collocation_cardinal_splines", "MultilevelVCycle", "crl", "assemble_stencil",
]


def __getattr__(name):
    # Lazy: torch-dependent modules load on first use.
    if name in ("StencilVectorSpace", "StencilVector", "StencilMatrix1D", "KronOperator", "StencilMatrix"):
        from . import stencil
        return getattr(stencil, name)
    if name == "assemble_stencil":
        from .assembly import assemble_stencil
        return assemble_stencil
    if name in ("KronSolver", "kron_solve_serial", "kron_solve_par", "to_bnd"):
        from . import kron_solve
        return getattr(kron_solve, name)
    if name in ("pcg", "damped_jacobi", "jacobi", "pcg_glt", "pcg_kron", "crl"):
        from . import solvers
        return getattr(solvers, name)
    if name in ("kron_dot_v2", "kron_dot_pyccel_2d"):
        from . import kron_product
        return getattr(kron_product, name)
    if name in ("knots_to_insert", "KronTransfer"):
        from . import multilevels
        return getattr(multilevels, name)
    if name in ("TwoLevelVCycle", "MultilevelVCycle"):
        from . import mg
        return getattr(mg, name)
    if name == "SlabDistribution":
        from .dist import SlabDistribution
        return SlabDistribution
    raise AttributeError(name)
