"""Bit-level fingerprint of the Bratu operator, basis and Gram kernels on fixed random inputs, for comparing two
library builds (GNK_LIB) kernel by kernel:  python tools/kernel_bits.py OUT.npz [--grid N] ;
python tools/kernel_bits.py --compare A.npz B.npz"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out, N, K):
    from gauss_newton_via_generalized_krylov_subspaces_amd import BratuPdeProblem
    from gauss_newton_via_generalized_krylov_subspaces_amd._device import BratuDevice
    from gauss_newton_via_generalized_krylov_subspaces_amd.slab import Comm
    torch.cuda.set_device(0)
    dev = BratuDevice(BratuPdeProblem(N + 1, 5, 10), Comm(single=True))
    be, sl = dev.backend, dev.slab
    g = torch.Generator(device=be.device).manual_seed(1)
    n = N * N

    def rnd(scale=1.0):
        v = dev.vec()
        v[sl.own] = scale * torch.randn(n, generator=g, device=be.device, dtype=torch.float64)
        return v

    u, v, w, y, r = rnd(0.1), rnd(), rnd(), rnd(), rnd()
    V = be.zeros(max(K, 20) + 1, sl.length)
    V[:, sl.own] = torch.randn(V.shape[0], n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    res = {}

    def keep(name, t):
        torch.cuda.synchronize()
        res[name] = t.detach().cpu().numpy().copy()

    o = dev.vec(); be.jvp(u, v, o); keep("jvp", o)
    o = dev.vec(); be.vjp(u, w, o); keep("vjp", o)
    o = dev.vec(); be.forward(u, o); keep("forward", o)
    o = dev.vec(); nr = be.zeros(64); be.residual(u, y, o, nr); keep("residual", o); keep("residual_n2", nr)
    for k in (1, 5, 12):
        c = be.to_device(np.linspace(0.5, 1.5, 64))
        hh = be.to_device(np.linspace(-0.1, 0.1, 64))
        gg, h, x = dev.vec(), be.zeros(256), dev.vec()
        be.vjp_gemv_t(u, r, V, k, gg, h); keep(f"vjp_gemv_t{k}_g", gg); keep(f"vjp_gemv_t{k}_h", h)
        gg, h, x = dev.vec(), be.zeros(256), dev.vec()
        be.gemv_vjp_gemv_t(V, k, c, r, x, gg, h); keep(f"trial{k}_x", x); keep(f"trial{k}_g", gg); keep(f"trial{k}_h", h)
        Vp = V.clone()
        gg, h, x, st = dev.vec(), be.zeros(256), dev.vec(), be.zeros(64)
        be.gemv_vjp_gemv_t_pending(Vp, k, c, hh, r, x, gg, h, st)
        keep(f"trialp{k}_x", x); keep(f"trialp{k}_g", gg); keep(f"trialp{k}_h", h); keep(f"trialp{k}_w", Vp[k])
    Vw = be.zeros(101, sl.length)                     # wide bases: the split gnk_vjp_gemv_t (k > 24)
    Vw[:, sl.own] = torch.randn(101, n, generator=g, device=be.device, dtype=torch.float64) / np.sqrt(n)
    for k in (25, 40, 57, 100):
        gg, h = dev.vec(), be.zeros(128)
        be.vjp_gemv_t(u, r, Vw, k, gg, h); keep(f"vjp_gemv_t{k}_g", gg); keep(f"vjp_gemv_t{k}_h", h)
    del Vw
    for k in (1, 5, 12, 20):
        c = be.to_device(np.linspace(0.5, 1.5, 64))
        hh = be.to_device(np.linspace(-0.1, 0.1, 64))
        Vp, x, st = V.clone(), dev.vec(), be.zeros(64)
        be.gemv_pending(Vp, k, c, hh, x, st)
        keep(f"gemvp{k}_x", x); keep(f"gemvp{k}_w", Vp[k]); keep(f"gemvp{k}_max", st[1:2])
    # CG: the normal matvec, the fused step matvec (direction update + lagged x) and the x / r update
    d = dev.vec(); be.jdiag(u, d)
    q, pq = dev.vec(), be.zeros(8)
    be.cg_matvec(d, v, q, pq, pairs=True); keep("cg_matvec_q", q); keep("cg_matvec_pq", pq)
    p_out, q2, x2, pq2 = dev.vec(), dev.vec(), w.clone(), be.zeros(8)
    be.cg_step_matvec(d, y, v, p_out, q2, 0.7, False, x2, 0.3, pq2, pairs=True)
    keep("cg_step_p", p_out); keep("cg_step_q", q2); keep("cg_step_x", x2); keep("cg_step_pq", pq2)
    x3, r3, z3, o3 = w.clone(), r.clone(), dev.vec(), be.zeros(8)
    dinv = dev.vec(); dinv[sl.own] = 1.0 / (1.0 + u[sl.own] ** 2)
    be.cg_update_xr(0.45, v, q, x3, r3, dinv, z3, o3, pairs=True)
    keep("cg_xr_x", x3); keep("cg_xr_r", r3); keep("cg_xr_z", z3); keep("cg_xr_dots", o3)
    # single-reduction CG update and the plain direction update
    sp, ss_, sx, sr, su, so = v.clone(), w.clone(), u.clone(), r.clone(), y.clone(), be.zeros(8)
    be.cg_sr_update(0.3, 0.6, False, r, sp, ss_, sx, sr, dinv, su, so)
    keep("cg_sr_p", sp); keep("cg_sr_s", ss_); keep("cg_sr_x", sx); keep("cg_sr_r", sr); keep("cg_sr_u", su)
    keep("cg_sr_dots", so)
    pp = v.clone(); be.cg_update_p(0.6, False, w, pp); keep("cg_p", pp)
    # small streaming kernels (slab and flat forms)
    st = be.zeros(8); be.vec_stats(r, st); keep("vec_stats", st)
    o = dev.vec(); be.vec_div(r, 3.7, o, True); keep("vec_div", o)
    o = dev.vec(); be.vec_axpy(w, 0.37, r, o, True); keep("vec_axpy", o)
    o = dev.vec(); be.jdiag(u, o); keep("jdiag", o)
    fl = r[sl.own].clone()
    st = be.zeros(8); be.flat_stats(fl, st); keep("flat_stats", st)
    o = torch.empty_like(fl); be.flat_div(fl, 3.7, o); keep("flat_div", o)
    o = torch.empty_like(fl); be.flat_axpy(fl, 0.37, fl.flip(0).contiguous(), o); keep("flat_axpy", o)
    fx, frr, fz, fo = fl.clone(), fl.flip(0).contiguous(), torch.empty_like(fl), be.zeros(8)
    be.flat_cg_update_xr(0.45, fl, fl * 0.5, fx, frr, torch.ones_like(fl) * 0.9, fz, fo, pairs=True)
    keep("flat_xr_x", fx); keep("flat_xr_r", frr); keep("flat_xr_z", fz); keep("flat_xr_dots", fo)
    o, jn = dev.vec(), be.zeros(64)
    be.normalize_jnorm(u, w, 3.0, o, jn); keep("normalize", o); keep("normalize_jn", jn)
    for k in range(1, K + 1):
        kp = be.gram_dim(k, True)
        rinv = np.zeros((kp, kp))
        rinv[:k + 1, :k + 1] = np.triu(np.ones((k + 1, k + 1))) * 0.1 + np.eye(k + 1)
        G = be.zeros(kp * kp)
        be.gram(u, V[:k], k, be.to_device(rinv.reshape(-1)), r, G); keep(f"gram{k}", G)
    np.savez(out, **res)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    for key in A.files:
        x, z = A[key], B[key]
        same = np.array_equal(x.view(np.int64), z.view(np.int64))
        d = float(np.max(np.abs(x - z))) if not same else 0.0
        print(f"{key:24s} {'identical' if same else 'DIFFERS'} {d:.3e}")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--grid", type=int, default=1024)
    ap.add_argument("--k", type=int, default=12)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        compare(*a.compare)
    else:
        run(a.out, a.grid, a.k)
