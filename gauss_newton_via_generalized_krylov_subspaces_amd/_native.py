"""ctypes binding of libgnk.so (include/gnk.h) and the HIP kernel backend.

The solver talks to a *backend* object whose methods mirror the C-ABI one to one
and take torch tensors.  ``HipBackend`` is the only backend the product uses; if
the library is missing or no GPU is visible it raises -- there is no CPU
fallback anywhere in the package.  (The test suite injects its own NumPy
backend to exercise the multi-rank host logic on CPU with gloo; that backend
lives in tests/ and is never importable from here.)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GNK_LIB", os.path.join(_HERE, "libgnk.so"))
GHOST = 2  # GNK_GHOST_ROWS
TIMER_GRAM, TIMER_JVP, TIMER_CG_MATVEC, TIMER_TRIAL, TIMER_PROBE, TIMER_CG_XR, TIMER_CG_AUX = 1, 2, 3, 4, 5, 6, 7  # GNK_TIMER_*
ABI_VERSION = 6  # GNK_ABI_VERSION
# GNK_TUNE_* keys of gnk_set_tuning (tests / A/B tooling only; the solver never sets them)
TUNE = {"gram_path": 0, "gram_ring": 1, "gram_v1min": 2, "cg_matvec": 3, "vjpg_blocks": 4, "gram_wide": 5, "gram_rpr": 6, "lls": 7, "vjpg_zmax": 8,
        "decomp_lds": 9, "trialw": 10, "gram_tm": 11, "gram_q": 12}

_c_int, _c_i64, _c_dbl, _c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p

# name -> (restype, argtypes); exactly the declarations of include/gnk.h
SIGNATURES = {
    "gnk_abi_version": (_c_int, []),
    "gnk_ctx_create": (_c_int, [_c_int, ctypes.POINTER(_c_vp)]),
    "gnk_ctx_destroy": (None, [_c_vp]),
    "gnk_last_error": (ctypes.c_char_p, [_c_vp]),
    "gnk_set_stream": (_c_int, [_c_vp, _c_vp]),
    "gnk_set_reduce_pairs": (_c_int, [_c_vp, _c_int]),
    "gnk_set_segments": (_c_int, [_c_vp, _c_i64]),
    "gnk_segment_fallbacks": (_c_i64, [_c_vp]),
    "gnk_set_tuning": (_c_int, [_c_vp, _c_int, _c_int]),
    "gnk_scratch_doubles": (_c_i64, []),
    "gnk_set_bratu": (_c_int, [_c_vp, _c_i64, _c_i64, _c_i64, _c_dbl, _c_dbl, _c_dbl]),
    "gnk_slab_len": (_c_i64, [_c_vp]),
    "gnk_bratu_jvp": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_bratu_vjp": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_bratu_forward": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "gnk_bratu_residual": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_bratu_diag_jtj": (_c_int, [_c_vp, _c_vp, _c_vp, _c_int]),
    "gnk_bratu_jdiag": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "gnk_basis_gemv": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp]),
    "gnk_vjp_gemv_t": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp]),
    "gnk_cgs_update": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp]),
    "gnk_vec_stats": (_c_int, [_c_vp, _c_vp, _c_vp]),
    "gnk_vec_div": (_c_int, [_c_vp, _c_vp, _c_dbl, _c_vp, _c_int]),
    "gnk_flat_gemv": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_i64]),
    "gnk_flat_gemv_t": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_i64, _c_vp]),
    "gnk_flat_cgs_update": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_i64, _c_vp]),
    "gnk_flat_stats": (_c_int, [_c_vp, _c_vp, _c_i64, _c_vp]),
    "gnk_flat_dot": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "gnk_flat_div": (_c_int, [_c_vp, _c_vp, _c_dbl, _c_vp, _c_i64]),
    "gnk_flat_axpy": (_c_int, [_c_vp, _c_vp, _c_dbl, _c_vp, _c_vp, _c_i64]),
    "gnk_flat_cg_update_xr": (_c_int, [_c_vp, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_i64, _c_vp]),
    "gnk_flat_cg_update_p": (_c_int, [_c_vp, _c_dbl, _c_int, _c_vp, _c_vp, _c_i64]),
    "gnk_csr_spmv": (_c_int, [_c_vp, _c_i64, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int]),
    "gnk_flat_gram": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_i64, _c_vp, _c_i64, _c_vp]),
    "gnk_basis_gemv_vjp_gemv_t": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_basis_gemv_pending": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_basis_gemv_vjp_gemv_t_pending": (_c_int, [_c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                                   _c_vp, _c_vp]),
    "gnk_normalize_jnorm": (_c_int, [_c_vp, _c_vp, _c_vp, _c_dbl, _c_vp, _c_vp]),
    "gnk_vec_axpy": (_c_int, [_c_vp, _c_vp, _c_dbl, _c_vp, _c_vp, _c_int]),
    "gnk_gram_padded_dim": (_c_int, [_c_int, _c_int]),
    "gnk_gram": (_c_int, [_c_vp, _c_vp, _c_vp, _c_i64, _c_int, _c_vp, _c_i64, _c_vp, _c_vp]),
    "gnk_cg_normal_matvec": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_cg_update_xr": (_c_int, [_c_vp, _c_dbl, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_cg_step_matvec": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_dbl, _c_int, _c_vp, _c_dbl,
                                    _c_vp]),
    "gnk_cg_step_matvec_dev": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp]),
    "gnk_cg_update_xr_dev": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_cg_scalars": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_vp]),
    "gnk_cg_update_p": (_c_int, [_c_vp, _c_dbl, _c_int, _c_vp, _c_vp]),
    "gnk_cg_sr_update": (_c_int, [_c_vp, _c_dbl, _c_dbl, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp, _c_vp,
                                  _c_vp]),
    "gnk_rank_sum": (_c_int, [_c_vp, _c_vp, _c_int, _c_i64, _c_vp]),
    "gnk_lls_max_k": (_c_int, []),
    "gnk_lls_solve": (_c_int, [_c_vp, _c_vp, _c_int, _c_int, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp]),
    "gnk_lls_next": (_c_int, [_c_vp, _c_int, _c_int, _c_vp, _c_vp, _c_vp, _c_vp, _c_int, _c_vp, _c_vp, _c_vp, _c_vp,
                              _c_vp, _c_vp]),
    "gnk_probe_mfma_f64": (_c_int, [_c_vp, _c_vp, _c_int, _c_int]),
    "gnk_decomp_check": (_c_int, [_c_vp, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int), _c_int]),
    "gnk_probe_stream": (_c_int, [_c_vp, _c_vp, _c_vp, _c_vp, _c_dbl, _c_i64, _c_int]),
    "gnk_timer_start": (_c_int, [_c_vp, _c_int, _c_int]),
    "gnk_timer_add": (_c_int, [_c_vp, _c_int]),
    "gnk_timer_collect": (_c_int, [_c_vp, ctypes.POINTER(_c_dbl), ctypes.POINTER(_c_dbl), _c_int]),
    "gnk_timer_collect_ids": (_c_int, [_c_vp, ctypes.POINTER(_c_dbl), ctypes.POINTER(_c_dbl),
                                       ctypes.POINTER(ctypes.c_int), _c_int]),
}

_LIB = None


# tooling exports (not on the solver path) an A/B variant build (GNK_LIB) may lack
TOOLING_SYMBOLS = {"gnk_decomp_check"}


class NativeLibraryError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load libgnk.so and bind every symbol of include/gnk.h (raises if any is missing)."""
    global _LIB
    if _LIB is not None and path == LIB_PATH:
        return _LIB
    if not os.path.exists(path):
        raise NativeLibraryError(
            f"libgnk.so not found at {path}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C gauss_newton_via_generalized_krylov_subspaces_amd/csrc`")
    lib = ctypes.CDLL(path)
    variant = "GNK_LIB" in os.environ          # tooling A/B against an older build (tools/lib_ab.sh)
    for name, (res, args) in SIGNATURES.items():
        if variant and name in TOOLING_SYMBOLS and not hasattr(lib, name):
            continue                           # an older variant build may predate a tooling export
        fn = getattr(lib, name)  # AttributeError = missing export
        fn.restype = res
        fn.argtypes = args
    if lib.gnk_abi_version() != ABI_VERSION:
        raise NativeLibraryError("libgnk.so ABI version mismatch")
    if path == LIB_PATH:
        _LIB = lib
    return lib


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class HipBackend:
    """One gnk_ctx on one GPU; every method enqueues on torch's current stream."""

    def __init__(self, device: torch.device):
        if not torch.cuda.is_available():
            raise NativeLibraryError("no ROCm GPU visible: the GNK hot path runs only on MI355X (gfx950)")
        self.lib = load_library()
        self.device = torch.device(device)
        idx = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self.device = torch.device("cuda", idx)
        ctx = ctypes.c_void_p()
        with torch.cuda.device(idx):
            rc = self.lib.gnk_ctx_create(idx, ctypes.byref(ctx))
        if rc != 0:
            raise NativeLibraryError(f"gnk_ctx_create failed ({rc})")
        self.ctx = ctx
        self._stream = None
        self.pairs = False

    def __del__(self):
        try:
            if getattr(self, "ctx", None) and self.lib is not None:
                self.lib.gnk_ctx_destroy(self.ctx)
                self.ctx = None
        except Exception:
            pass

    def _sync_stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream:
            self._chk(self.lib.gnk_set_stream(self.ctx, ctypes.c_void_p(s)), "set_stream")
            self._stream = s

    def _chk(self, rc, what):
        if rc != 0:
            msg = self.lib.gnk_last_error(self.ctx)
            raise RuntimeError(f"libgnk {what} failed ({rc}): {msg.decode() if msg else ''}")

    def _call(self, name, *args):
        self._sync_stream()
        self._chk(getattr(self.lib, name)(self.ctx, *args), name)

    def set_reduce_pairs(self, on: bool):
        """Compensated reductions return unevaluated (s, c) pairs (gnk_set_reduce_pairs).  The
        methods below that reduce take the mode per call (``pairs=``) and switch the context only
        when it differs, so one backend can serve a pair-mode solver (Bratu GN / CGLS) and a plain one
        (GNK, generic problems) in any order."""
        self._chk(self.lib.gnk_set_reduce_pairs(self.ctx, int(bool(on))), "set_reduce_pairs")
        self.pairs = bool(on)

    def _mode(self, pairs, out, plain_len, pair_len, what):
        """Set the context's reduction mode for one call and check the output buffer holds what that
        mode writes (plain_len / pair_len doubles): a too-small buffer would be a device OOB write."""
        need = pair_len if pairs else plain_len
        if out is None or out.numel() < need:
            raise ValueError(f"{what}: output buffer holds {0 if out is None else out.numel()} doubles, "
                             f"{'pair' if pairs else 'plain'} mode writes {need}")
        if bool(pairs) != self.pairs:
            self.set_reduce_pairs(pairs)

    def set_tuning(self, key: str, value: int):
        """Kernel-choice override for tests / A/B tooling (gnk_set_tuning; 0 restores the default)."""
        self._chk(self.lib.gnk_set_tuning(self.ctx, TUNE[key], int(value)), "set_tuning")

    def scratch_doubles(self) -> int:
        return int(self.lib.gnk_scratch_doubles())

    # --- problem ---------------------------------------------------------------
    def set_bratu(self, N, row0, nrows, h, alpha, lam):
        self._chk(self.lib.gnk_set_bratu(self.ctx, N, row0, nrows, float(h), float(alpha), float(lam)), "set_bratu")

    def set_segments(self, seg_rows: int):
        """Rank-count-independent reductions over fixed global row segments of ``seg_rows`` rows
        (gnk_set_segments; 0 = off).  Call after set_bratu, which resets it."""
        self._chk(self.lib.gnk_set_segments(self.ctx, int(seg_rows)), "set_segments")
        self.seg_rows = int(seg_rows)

    def segment_fallbacks(self) -> int:
        """Reductions that ran on the per-slab decomposition while segments were on (the wide Gram
        passes, k > 20): rank-count dependent in rounding (gnk_segment_fallbacks)."""
        return int(self.lib.gnk_segment_fallbacks(self.ctx))

    def slab_len(self):
        return int(self.lib.gnk_slab_len(self.ctx))

    def empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float64, device=self.device)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=torch.float64, device=self.device)

    def to_device(self, a):
        return torch.as_tensor(a, dtype=torch.float64).to(self.device)

    _PIN_SLOTS, _PIN_LEN = 16, 64 * 64

    def upload(self, dst, a):
        """dst[:len(a)] = a for a small host array, without stalling the host: through a ring of
        pinned staging buffers and a stream-ordered copy (a pageable copy would wait for the
        queue to drain).  Each slot is reused only after its previous copy completed."""
        a = np.asarray(a, dtype=np.float64).reshape(-1)
        n = a.size
        if n > self._PIN_LEN:
            dst[:n].copy_(self.to_device(a))
            return dst
        if not hasattr(self, "_pin"):
            self._pin = [torch.empty(self._PIN_LEN, dtype=torch.float64, pin_memory=True)
                         for _ in range(self._PIN_SLOTS)]
            self._pin_ev = [None] * self._PIN_SLOTS
            self._pin_i = 0
        i = self._pin_i
        self._pin_i = (i + 1) % self._PIN_SLOTS
        if self._pin_ev[i] is not None:
            self._pin_ev[i].synchronize()
        buf = self._pin[i]
        buf.numpy()[:n] = a
        dst[:n].copy_(buf[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._pin_ev[i] = ev
        return dst

    # --- operator ----------------------------------------------------------------
    def jvp(self, u, v, out):
        self._call("gnk_bratu_jvp", _p(u), _p(v), _p(out))

    def vjp(self, u, w, out):
        self._call("gnk_bratu_vjp", _p(u), _p(w), _p(out))

    def forward(self, x, F):
        self._call("gnk_bratu_forward", _p(x), _p(F))

    def residual(self, x, y, r, norm2):
        self._call("gnk_bratu_residual", _p(x), _p(y), _p(r), _p(norm2))

    def diag_jtj(self, u, out, reciprocal=False):
        self._call("gnk_bratu_diag_jtj", _p(u), _p(out), int(bool(reciprocal)))

    def jdiag(self, u, d):
        self._call("gnk_bratu_jdiag", _p(u), _p(d))

    # --- basis -------------------------------------------------------------------
    def gemv(self, V, k, c, x):
        self._call("gnk_basis_gemv", _p(V), V.stride(0), int(k), _p(c), _p(x))

    def vjp_gemv_t(self, u, r, V, k, g, h):
        ldv = V.stride(0) if V is not None else 0
        self._call("gnk_vjp_gemv_t", _p(u), _p(r), _p(V), ldv, int(k), _p(g), _p(h))

    def gemv_vjp_gemv_t(self, V, k, c, r, x, g, h):
        self._call("gnk_basis_gemv_vjp_gemv_t", _p(V), V.stride(0), int(k), _p(c), _p(r), _p(x), _p(g), _p(h))

    def gemv_pending(self, V, k, c, hh, x, stats):
        """column k of V is the pending raw column: materialised in place (see gnk.h)"""
        self._call("gnk_basis_gemv_pending", _p(V), V.stride(0), int(k), _p(c), _p(hh), _p(x), _p(stats))

    def gemv_vjp_gemv_t_pending(self, V, k, c, hh, r, x, g, h, stats):
        self._call("gnk_basis_gemv_vjp_gemv_t_pending", _p(V), V.stride(0), int(k), _p(c), _p(hh), _p(r), _p(x),
                   _p(g), _p(h), _p(stats))

    # -- flat vectors (generic problems) --------------------------------------------------
    def flat_gemv(self, V, k, c, x):
        self._call("gnk_flat_gemv", _p(V), V.stride(0), int(k), _p(c), _p(x), x.numel())

    def flat_gemv_t(self, V, k, g, h):
        self._call("gnk_flat_gemv_t", _p(V), V.stride(0), int(k), _p(g), g.numel(), _p(h))

    def flat_cgs_update(self, V, k, h, g, stats):
        self._call("gnk_flat_cgs_update", _p(V), V.stride(0), int(k), _p(h), _p(g), g.numel(), _p(stats))

    def flat_stats(self, x, stats, pairs=False):
        self._mode(pairs, stats, 2, 3, "flat_stats")
        self._call("gnk_flat_stats", _p(x), x.numel(), _p(stats))

    def flat_dot(self, a, b, out, pairs=False):
        self._mode(pairs, out, 1, 2, "flat_dot")
        self._call("gnk_flat_dot", _p(a), _p(b), a.numel(), _p(out))

    def flat_div(self, src, denom, dst):
        self._call("gnk_flat_div", _p(src), float(denom), _p(dst), src.numel())

    def flat_axpy(self, x, alpha, d, out):
        self._call("gnk_flat_axpy", _p(x), float(alpha), _p(d), _p(out), x.numel())

    def flat_cg_update_xr(self, alpha, p, q, x, r, dinv, z, out, pairs=False):
        self._mode(pairs, out, 2, 4, "flat_cg_update_xr")
        self._call("gnk_flat_cg_update_xr", float(alpha), _p(p), _p(q), _p(x), _p(r), _p(dinv), _p(z), x.numel(),
                   _p(out))

    def flat_cg_update_p(self, beta, first, z, p):
        self._call("gnk_flat_cg_update_p", float(beta), int(bool(first)), _p(z), _p(p), p.numel())

    def csr_spmv(self, nrows, indptr, indices, data, x, y, negate=False, reciprocal=False):
        mode = 2 if reciprocal else (1 if negate else 0)
        self._call("gnk_csr_spmv", int(nrows), _p(indptr), _p(indices), _p(data), _p(x), _p(y), mode)

    def flat_gram(self, W, k, rinv, r, m, G):
        kp = self.gram_dim(k, r is not None)
        self._call("gnk_flat_gram", _p(W), W.stride(0), int(k), _p(rinv), kp, _p(r), int(m), _p(G))

    def cgs_update(self, V, k, h, g, stats):
        self._call("gnk_cgs_update", _p(V), V.stride(0), int(k), _p(h), _p(g), _p(stats))

    def vec_stats(self, x, stats, pairs=False):
        self._mode(pairs, stats, 2, 3, "vec_stats")
        self._call("gnk_vec_stats", _p(x), _p(stats))

    def vec_div(self, src, denom, dst, full_slab):
        self._call("gnk_vec_div", _p(src), float(denom), _p(dst), int(bool(full_slab)))

    def normalize_jnorm(self, u, g, denom, v, jn2):
        self._call("gnk_normalize_jnorm", _p(u), _p(g), float(denom), _p(v), _p(jn2))

    def vec_axpy(self, x, alpha, d, out, full_slab):
        self._call("gnk_vec_axpy", _p(x), float(alpha), _p(d), _p(out), int(bool(full_slab)))

    def cg_sr_update(self, alpha, beta, first, w, p, s, x, r, dinv, u, out):
        self._call("gnk_cg_sr_update", float(alpha), float(beta), int(bool(first)), _p(w), _p(p), _p(s), _p(x), _p(r),
                   _p(dinv), _p(u), _p(out))

    def rank_sum(self, parts, world, out):
        """out = the ranks' parts (world x n, contiguous) summed on the device in slab.tree_sum's order
        (pairwise, fixed), one launch."""
        n = out.numel()
        self._call("gnk_rank_sum", _p(parts), int(world), int(n), _p(out))
        return out

    def lls_max_k(self):
        return int(self.lib.gnk_lls_max_k())

    def lls_solve(self, G, kp, k, P, rescale, sdd, e, out, e_try):
        self._call("gnk_lls_solve", _p(G), int(kp), int(k), _p(P), int(bool(rescale)), _p(sdd), _p(e), _p(out),
                   _p(e_try))

    def lls_next(self, k, pending, out, e_try, pack, sc, kp_next, T, P, sdd, e, hh, scn):
        self._call("gnk_lls_next", int(k), int(bool(pending)), _p(out), _p(e_try), _p(pack), _p(sc), int(kp_next),
                   _p(T), _p(P), _p(sdd), _p(e), _p(hh), _p(scn))

    def gram_dim(self, k, with_r):
        return int(self.lib.gnk_gram_padded_dim(int(k), int(bool(with_r))))

    def gram(self, u, V, k, rinv, r, G):
        kp = self.gram_dim(k, r is not None)
        self._call("gnk_gram", _p(u), _p(V), V.stride(0), int(k), _p(rinv), kp, _p(r), _p(G))

    # --- CG ------------------------------------------------------------------------
    def cg_matvec(self, d, p, q, pq, pairs=False):
        self._mode(pairs, pq, 1, 2, "cg_matvec")
        self._call("gnk_cg_normal_matvec", _p(d), _p(p), _p(q), _p(pq))

    def cg_step_matvec(self, d, z, p_in, p_out, q, beta, first, x, xalpha, pq, pairs=False):
        self._mode(pairs, pq, 1, 2, "cg_step_matvec")
        self._call("gnk_cg_step_matvec", _p(d), _p(z), _p(p_in), _p(p_out), _p(q), float(beta), int(bool(first)),
                   _p(x), float(xalpha), _p(pq))

    def cg_update_xr(self, alpha, p, q, x, r, dinv, z, out, pairs=False):
        self._mode(pairs, out, 2, 4, "cg_update_xr")
        self._call("gnk_cg_update_xr", float(alpha), _p(p), _p(q), _p(x), _p(r), _p(dinv), _p(z), _p(out))

    def cg_update_p(self, beta, first, z, p):
        self._call("gnk_cg_update_p", float(beta), int(bool(first)), _p(z), _p(p))

    def cg_step_matvec_dev(self, d, z, p_in, p_out, q, first, x, state, pq):
        """gnk_cg_step_matvec with beta / the lagged alpha from the device CG state (pairs out)."""
        self._mode(True, pq, 1, 2, "cg_step_matvec_dev")
        self._call("gnk_cg_step_matvec_dev", _p(d), _p(z), _p(p_in), _p(p_out), _p(q), int(bool(first)), _p(x),
                   _p(state), _p(pq))

    def cg_update_xr_dev(self, state, p, q, x, r, dinv, z, out):
        """gnk_cg_update_xr with alpha from the device CG state (pairs out)."""
        self._mode(True, out, 2, 4, "cg_update_xr_dev")
        self._call("gnk_cg_update_xr_dev", _p(state), _p(p), _p(q), _p(x), _p(r), _p(dinv), _p(z), _p(out))

    def cg_scalars(self, parts, world, stage, state):
        """The fused CG iteration's scalar recurrence on the device (gnk_cg_scalars)."""
        self._call("gnk_cg_scalars", _p(parts), int(world), int(stage), _p(state))

    def timer_start(self, kernel_id, capacity):
        self._chk(self.lib.gnk_timer_start(self.ctx, int(kernel_id), int(capacity)), "timer_start")

    def timer_collect(self, capacity):
        """-> list of (ms, algorithmic bytes) for each timed launch."""
        ms = (_c_dbl * capacity)()
        by = (_c_dbl * capacity)()
        n = self.lib.gnk_timer_collect(self.ctx, ms, by, int(capacity))
        if n < 0:
            self._chk(n, "timer_collect")
        return [(ms[i], by[i]) for i in range(n)]

    def timer_add(self, kernel_id):
        """Also time the launches of another kernel class in the window timer_start opened."""
        self._chk(self.lib.gnk_timer_add(self.ctx, int(kernel_id)), "timer_add")

    def timer_collect_ids(self, capacity):
        """-> list of (kernel class id, ms, algorithmic bytes) for each timed launch, in launch order."""
        ms = (_c_dbl * capacity)()
        by = (_c_dbl * capacity)()
        ids = (ctypes.c_int * capacity)()
        n = self.lib.gnk_timer_collect_ids(self.ctx, ms, by, ids, int(capacity))
        if n < 0:
            self._chk(n, "timer_collect_ids")
        return [(ids[i], ms[i], by[i]) for i in range(n)]

    def probe_stream(self, a, b, c, s, n, mode):
        self._call("gnk_probe_stream", _p(a), _p(b), _p(c), float(s), int(n), int(mode))

    def decomp_check(self):
        """[(table workgroups per CU, live occupancy)] of the persistent kernels' fixed grids (gnk_decomp_check)."""
        cap = 256
        t, l = (ctypes.c_int * cap)(), (ctypes.c_int * cap)()
        n = self.lib.gnk_decomp_check(self.ctx, t, l, cap)
        if n < 0:
            self._chk(n, "decomp_check")
        return [(t[i], l[i]) for i in range(min(n, cap))]

    def probe_mfma(self, out, blocks, iters):
        self._call("gnk_probe_mfma_f64", _p(out), int(blocks), int(iters))
