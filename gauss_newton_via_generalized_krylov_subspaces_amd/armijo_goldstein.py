"""Armijo-Goldstein backtracking (ref:armijo_goldstein.py:1-72).

``armijo_device`` is the form the device solvers use: every trial point
x_t = x + t d is evaluated by a caller-supplied ``trial(t) -> sum(res(x_t)**2)``
that runs on the GPU (basis GEMV + fused residual/norm kernel for GNK, axpy +
residual for GN), and only the scalar loss comes back to the host.
The constants are the reference's: t0 = 1, halve up to 100 times, accept when
prev - cur >= 0.5 * t * ||J d||^2.
"""
from __future__ import annotations

import numpy as np


class StepLengthConvergenceError(RuntimeError):
    """ref:armijo_goldstein.py:8-13"""

    message: str

    def __init__(self, message: str):
        super().__init__(message)
        self.message = message


def failure_message(d_norm: float) -> str:
    return ("The armijio_goldstein subroutine reached maximum iteration bound before principle was satisfied! "
            "Possible reasons:"
            + "\n- The max iteration count is not big enough to allow for a sufficiently small step size"
            + "\n- Or the descent direction is invalid."
            + f"Norm of descent_direction ={d_norm}.")


def armijo_device(trial, prev_loss: float, jdd: float, d: np.ndarray, max_iter: int = 100,
                  initial_step_length: float = 1.0):
    """Returns (step_length, number_of_trials); the last trial's state is the accepted one."""
    t = initial_step_length
    for it in range(max_iter):
        cur = trial(t)
        if prev_loss - cur >= 0.5 * t * jdd:
            return t, it + 1
        t /= 2
    raise StepLengthConvergenceError(failure_message(np.linalg.norm(d)))
