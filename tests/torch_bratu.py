"""The Bratu problem written as a user would write a ``Problem``: torch operations on flat device tensors.

Test helper only (the product's Bratu path is the matrix-free HIP stencil).  Same operator as
ref:bratu_pde_problem.py:76-96 on the flat index jx * N + iy (SURVEY.md §8 grid layout):
F(u) = L u + ALPHA D_x u + LAMBDA e^u with zero Dirichlet ghosts, res = y - F, J = d res / du.
"""
import torch
import torch.nn.functional as tF


def make_torch_bratu(N, alpha, lam, y, grid_resolution=None, with_jvp=True, with_diag=True):
    """(residual, jvp, vjp, diag_jtj) callables; jvp / vjp / diag_jtj None when not requested."""
    h = 6.0 / (N + 1) if grid_resolution is None else grid_resolution
    hm2, hm1 = h ** -2, h ** -1
    yt = {}

    def y_on(dev):
        if dev not in yt:
            yt[dev] = torch.as_tensor(y, dtype=torch.float64, device=dev)
        return yt[dev]

    def lin(v, transpose=False):
        U = v.reshape(N, N)
        P = tF.pad(U, (1, 1, 1, 1))
        Lv = (4.0 * U - P[:-2, 1:-1] - P[2:, 1:-1] - P[1:-1, :-2] - P[1:-1, 2:]) * hm2
        Dv = (P[:-2, 1:-1] - U) * hm1 if transpose else (P[2:, 1:-1] - U) * hm1
        return (Lv + alpha * Dv).reshape(-1)

    def residual(u):
        F = lin(u) if lam == 0 else lin(u) + lam * torch.exp(u)
        return y_on(u.device) - F

    def jvp(u, v):
        return -(lin(v) + lam * torch.exp(u) * v)

    def vjp(u, w):
        return -(lin(w, transpose=True) + lam * torch.exp(u) * w)

    def diag_jtj(u):
        c = (4.0 * hm2 - alpha * hm1) + lam * torch.exp(u)
        d = (c * c).reshape(N, N).clone()
        d[1:, :] += (-hm2 + alpha * hm1) ** 2          # the jx - 1 neighbour's row
        d[:-1, :] += hm2 * hm2                          # jx + 1
        d[:, 1:] += hm2 * hm2                           # iy - 1
        d[:, :-1] += hm2 * hm2                          # iy + 1
        return d.reshape(-1)

    return (residual, jvp if with_jvp else None, vjp if with_jvp else None, diag_jtj if with_diag else None)
