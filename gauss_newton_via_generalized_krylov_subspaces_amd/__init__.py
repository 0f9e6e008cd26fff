"""MI355X-native generalized-Krylov Gauss-Newton (drop-in for the reference's
``gauss_newton_krylow`` / ``gauss_newton`` on the Bratu problem).

Public surface (mirrors mariusbaehr/gauss_newton_via_generalized_krylov_subspaces):
  gauss_newton_krylow, gauss_newton, cg_least_squares, BratuPdeProblem,
  RegressionResult, StepLengthConvergenceError, benchmark_method, Problem,
  GeneralizedKrylowSubspaceBreakdown, GeneralizedKrylowSubspaceSpansEntireSpace.
Hot path: libgnk.so (HIP, gfx950) via ctypes -- see include/gnk.h.
"""
from .armijo_goldstein import StepLengthConvergenceError
from .benchmark import benchmark_method, reverse_accumulation
from .bratu_pde_problem import BratuJacobian, BratuPdeProblem, default_u
from .gauss_newton import GNSolver, cg_least_squares, gauss_newton
from .gauss_newton_krylow import GNKSolver, gauss_newton_krylow
from .problem import Problem, ProblemJacobian
from .krylow import GeneralizedKrylowSubspaceBreakdown, GeneralizedKrylowSubspaceSpansEntireSpace
from .regression_result import RegressionResult
from .slab import Comm, SlabVector, row_partition

__all__ = [
    "gauss_newton_krylow", "gauss_newton", "cg_least_squares", "BratuPdeProblem", "BratuJacobian",
    "default_u", "RegressionResult", "StepLengthConvergenceError", "GeneralizedKrylowSubspaceBreakdown",
    "GeneralizedKrylowSubspaceSpansEntireSpace", "GNKSolver", "GNSolver", "Comm", "row_partition", "benchmark_method", "reverse_accumulation",
    "Problem", "ProblemJacobian",
]
