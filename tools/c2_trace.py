"""C2 (N = 1024, restart 20) step trace of the GNK solver: k, step length, trials and loss per iteration, as JSON
lines -- for comparing two library builds (GNK_LIB) step by step.  python tools/c2_trace.py [version] [max_iter]"""
import io
import contextlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gauss_newton_via_generalized_krylov_subspaces_amd as gnk  # noqa: E402
from oracle import gnk_oracle as O  # noqa: E402


def main():
    version = sys.argv[1] if len(sys.argv) > 1 else "res_old"
    max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    N = 1024
    _, y, u0 = O.bratu_workload(N)
    prob = gnk.BratuPdeProblem(N + 1, 5, 10)
    s = gnk.GNKSolver(prob, y, krylow_restart=20, max_iter=max_iter, version=version)
    buf = io.StringIO()
    err = None
    with contextlib.redirect_stdout(buf):
        s.setup(u0)
        try:
            while not s.step():
                pass
        except Exception as e:          # noqa: BLE001 -- reported below
            err = repr(e)[:200]
    for i, t in enumerate(s.trace):
        print(json.dumps({"it": i + 1, "k": t["k"], "t": t["t"], "trials": t["trials"], "prev_loss": t["prev_loss"],
                          "jdd": t["jdd"], "losses": t["losses"][:3]}))
    print(json.dumps({"error": err, "lib": os.environ.get("GNK_LIB", "product"),
                      "first_loss": float(np.float64(s.trace[0]["prev_loss"])) if s.trace else None}))


if __name__ == "__main__":
    main()
