"""Solver return record (ref:regression_result.py:4-49)."""
from __future__ import annotations


class RegressionResult:
    """Fields: method_name, x, success, nrev (residual evaluations), njev, nit."""

    def __init__(self, method_name, x, success, nrev, njev, nit):
        self.method_name = method_name
        self.x = x
        self.success = success
        self.nrev = nrev
        self.njev = njev
        self.nit = nit

    @property
    def nfev(self):
        return self.nrev

    def __str__(self):
        state = "converged successfuly to" if self.success else "failed to terminate and stopped at"
        return (f"{self.method_name} {state} {self.x}. After {self.nit} iterations using {self.nrev} "
                "evaluations of the residual, ")
