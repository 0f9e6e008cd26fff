"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

This script is the only thing in the repository that imports the reference
(mariusbaehr/gauss_newton_via_generalized_krylov_subspaces, mounted read-only at
/root/reference in the build container).  It is run once, in the build
container, with OPENBLAS_NUM_THREADS=1 (bookkeeping is
thread-count independent, fp64 norms drift by ~1e-15 across thread counts).
Its outputs -- inputs plus expected outputs, nothing else -- are committed as
``*.npz`` + ``golden.json``; the reference source itself never travels.

Usage:  OPENBLAS_NUM_THREADS=1 PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import contextlib
import io
import json
import os
import sys

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.dont_write_bytecode = True
REF = os.environ.get("GNK_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import scipy  # noqa: E402

import armijo_goldstein as ref_ag  # noqa: E402
import bratu_pde_problem as ref_bratu  # noqa: E402
import gauss_newton as ref_gn  # noqa: E402
import gauss_newton_krylow as ref_gnk  # noqa: E402
import krylow as ref_krylow  # noqa: E402
import rosenbrock_problem as ref_rosen  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
META = {
    "generator": "tests/golden/make_golden.py",
    "numpy": np.__version__,
    "scipy": scipy.__version__,
    "openblas_threads": os.environ.get("OPENBLAS_NUM_THREADS"),
    "cases": {},
}
ARRAYS = {}


def run_recorded(method, res, x0, jac, **kwargs):
    """Run a reference solver; record per-iteration (||x||, ||res(x)||, nfev, cg_iter)."""
    rec = {"xnorm": [], "rnorm": [], "nfev": [], "cg_iter": []}
    xs = []

    def callback(x, nfev, cg_iter):
        rec["xnorm"].append(float(np.linalg.norm(x)))
        rec["rnorm"].append(float(np.linalg.norm(res(x))))
        rec["nfev"].append(None if nfev is None else int(nfev))
        rec["cg_iter"].append(None if cg_iter is None else int(cg_iter))
        xs.append(np.array(x, copy=True))

    buf = io.StringIO()
    exc = None
    result = None
    with contextlib.redirect_stdout(buf):
        try:
            result = method(res, x0, jac, callback=callback, **kwargs)
        except ref_ag.StepLengthConvergenceError as e:
            exc = ("StepLengthConvergenceError", e.message)
    out = {
        "per_iter": rec,
        "stdout": buf.getvalue().splitlines(),
        "exception": exc,
    }
    if result is not None:
        out.update(
            method_name=result.method_name,
            success=bool(result.success),
            nrev=int(result.nrev),
            njev=int(result.njev),
            nit=int(result.nit),
            xnorm_final=float(np.linalg.norm(result.x)),
            rnorm_final=float(np.linalg.norm(res(result.x))),
            str=str(result),
        )
    return out, (None if result is None else result.x), xs


def bratu_setup(grid_nodes, alpha, lam, grid_resolution=None, seed=42, linear_u0=False):
    """Workload of ref:bratu_pde_test.py:22-36 (and :193-219 for the linear case)."""
    prob = ref_bratu.BratuPdeProblem(grid_nodes, alpha, lam, grid_resolution=grid_resolution)
    y = prob.pde_operator(prob.u_true)
    res = prob.make_res(y)
    jac = prob.make_jac()
    if linear_u0:
        u0 = -1 * jac(np.zeros((grid_nodes - 1) ** 2)).T @ y
    else:
        np.random.seed(seed)
        u0 = prob.u_true + 0.1 * np.random.normal(loc=0, scale=1, size=len(prob.u_true))
    return prob, y, res, jac, u0


def add_gnk_case(name, res, x0, jac, keep_iterates=False, **kwargs):
    print("case", name, flush=True)
    out, x, xs = run_recorded(ref_gnk.gauss_newton_krylow, res, x0, jac, **kwargs)
    out["kwargs"] = {k: v for k, v in kwargs.items()}
    META["cases"][name] = out
    if x is not None:
        ARRAYS[name + "__x"] = x
    if keep_iterates and xs:
        ARRAYS[name + "__iterates"] = np.stack(xs)


def add_gn_case(name, res, x0, jac, **kwargs):
    print("case", name, flush=True)
    out, x, _ = run_recorded(ref_gn.gauss_newton, res, x0, jac, **kwargs)
    out["kwargs"] = dict(kwargs)
    META["cases"][name] = out
    if x is not None:
        ARRAYS[name + "__x"] = x


# ---------------------------------------------------------------- F1: Rosenbrock p = 2
ref_rosen.parameter_count = 2  # jac reads the module global at call time (ref:rosenbrock_problem.py:15-18)
for x0name, x0 in (("m1_1", [-1.0, 1.0]), ("2_2", [2.0, 2.0])):
    for version in ("res_old", "res_new"):
        add_gnk_case(f"rosen2_{x0name}_{version}", ref_rosen.res, np.array(x0), ref_rosen.jac,
                     version=version, keep_iterates=True)
    add_gn_case(f"rosen2_{x0name}_gn", ref_rosen.res, np.array(x0), ref_rosen.jac)

# ---------------------------------------------------------------- F5: Rosenbrock p = 1000
ref_rosen.parameter_count = 1000
x_exact = np.ones(1000)
np.random.seed(42)
r_x0_i = x_exact + 0.1 * np.random.normal(loc=0, scale=1, size=1000)   # ref:rosenbrock_test.py:20-22
r_x0_ii = 2 * x_exact                                                   # :70
r_x0_iii = 2 * x_exact
r_x0_iii[2] = 1.99                                                      # :93-94
ARRAYS["rosen1000_x0_i"] = r_x0_i
for x0name, x0 in (("i", r_x0_i), ("ii", r_x0_ii), ("iii", r_x0_iii)):
    for version in ("res_old", "res_new"):
        add_gnk_case(f"rosen1000_{x0name}_{version}", ref_rosen.res, x0.copy(), ref_rosen.jac, version=version)
    add_gn_case(f"rosen1000_{x0name}_gn", ref_rosen.res, x0.copy(), ref_rosen.jac)

# ---------------------------------------------------------------- F2: Bratu grid 25 (N = 24)
prob, y, res, jac, u0 = bratu_setup(25, 5, 10)
ARRAYS["bratu24_u0"] = u0
ARRAYS["bratu24_y"] = y
for version in ("res_old", "res_new", "jac_old_res_old", "jac_old_res_new"):
    for restart in (None, 20):
        add_gnk_case(f"bratu24_{version}_r{restart}", res, u0, jac, version=version,
                     krylow_restart=restart, max_iter=100, keep_iterates=(restart is None))
add_gn_case("bratu24_gn", res, u0, jac)
add_gn_case("bratu24_gn_precond", res, u0, jac, cg_preconditioner=True)

# without scaling (ref:bratu_pde_test.py:76-104), grid 25
prob_ns, y_ns, res_ns, jac_ns, u0_ns = bratu_setup(25, 5, 10, grid_resolution=1)
for version in ("res_old", "res_new"):
    add_gnk_case(f"bratu24_noscale_{version}", res_ns, u0_ns, jac_ns, version=version, max_iter=100)
add_gn_case("bratu24_noscale_gn", res_ns, u0_ns, jac_ns)

# ---------------------------------------------------------------- F4: linear Bratu (lambda = 0), grid 25
prob_l, y_l, res_l, jac_l, u0_l = bratu_setup(25, 5, 0, linear_u0=True)
ARRAYS["bratu24_linear_u0"] = u0_l
add_gnk_case("bratu24_linear_res_old", res_l, u0_l, jac_l, max_iter=100)
add_gnk_case("bratu24_linear_res_new", res_l, u0_l, jac_l, version="res_new", max_iter=200)
add_gn_case("bratu24_linear_gn", res_l, u0_l, jac_l)

# ---------------------------------------------------------------- F3: Bratu grid 101 (N = 100)
prob, y, res, jac, u0 = bratu_setup(101, 5, 10)
ARRAYS["bratu100_u0"] = u0
for version in ("res_old", "res_new"):
    for restart in (None, 20):
        add_gnk_case(f"bratu100_{version}_r{restart}", res, u0, jac, version=version,
                     krylow_restart=restart, max_iter=100)
add_gn_case("bratu100_gn", res, u0, jac)

# ---------------------------------------------------------------- F7: cg_least_squares, first GN step
for N, gn in ((24, 25), (100, 101)):
    prob, y, res, jac, u0 = bratu_setup(gn, 5, 10)
    r0 = res(u0)
    J0 = jac(u0)
    for pre in (False, True):
        x, cg_iter = ref_gn.cg_least_squares(-1 * J0, r0, preconditioner=pre)
        ARRAYS[f"cgls{N}_pre{int(pre)}__x"] = x
        META["cases"][f"cgls{N}_pre{int(pre)}"] = {"cg_iter": int(cg_iter)}
    for rtol in (1e-8,):
        x, cg_iter = ref_gn.cg_least_squares(-1 * J0, r0, preconditioner=True, cg_rtol=rtol)
        ARRAYS[f"cgls{N}_pre1_rtol1e-8__x"] = x
        META["cases"][f"cgls{N}_pre1_rtol1e-8"] = {"cg_iter": int(cg_iter)}

# ---------------------------------------------------------------- F6: single-operator vectors
for N in (8, 64):
    gn = N + 1
    prob = ref_bratu.BratuPdeProblem(gn, 5, 10)
    rng = np.random.default_rng(1234 + N)
    n = N * N
    u = prob.u_true + 0.1 * rng.standard_normal(n)
    v = rng.standard_normal(n)
    w = rng.standard_normal(n)
    y = prob.pde_operator(prob.u_true)
    J = prob.make_jac()(u)
    ARRAYS[f"ops{N}_u"] = u
    ARRAYS[f"ops{N}_v"] = v
    ARRAYS[f"ops{N}_w"] = w
    ARRAYS[f"ops{N}_y"] = y
    ARRAYS[f"ops{N}_utrue"] = prob.u_true
    ARRAYS[f"ops{N}_Jv"] = J @ v
    ARRAYS[f"ops{N}_JTw"] = J.T @ w
    ARRAYS[f"ops{N}_F"] = prob.pde_operator(u)
    ARRAYS[f"ops{N}_res"] = prob.make_res(y)(u)
    ARRAYS[f"ops{N}_diagJTJ"] = np.asarray((J.T @ J).diagonal())
    # one Krylov start + 3 updates (ref:krylow.py:30-73)
    kr = ref_krylow.GeneralizedKrylowSubspace()
    c = kr.start(u)
    upd = rng.standard_normal((3, n))
    ARRAYS[f"ops{N}_update_res"] = upd
    for step in range(3):
        kr.update(J, upd[step])
        c = np.append(c, 0)
    ARRAYS[f"ops{N}_basis"] = kr.basis
    # one linear least squares solve on -J V (ref:gauss_newton_krylow.py:16-36)
    JV = J @ kr.basis
    r = prob.make_res(y)(u)
    ARRAYS[f"ops{N}_lls_d"] = ref_gnk.linear_least_squares(-1 * JV, r)
    ARRAYS[f"ops{N}_lls_r"] = r
    # parameter metadata
    META["cases"][f"ops{N}"] = {"grid_nodes": gn, "h": prob.grid_resolution}

with open(os.path.join(OUT, "golden.json"), "w") as f:
    json.dump(META, f, indent=1, sort_keys=True)
np.savez_compressed(os.path.join(OUT, "golden.npz"), **ARRAYS)
print("wrote", len(META["cases"]), "cases,", len(ARRAYS), "arrays")
