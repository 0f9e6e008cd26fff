"""Oracle trajectories of the multi-rank GPU cases (tests/multislab_worker.py), precomputed.

The oracle side of test_gpu_multislab does not depend on the rank count or the transport, and its
exactly-rounded-dot GN runs take minutes of host time (unpreconditioned CGLS at 256^2: ~20 k CG
iterations with math.fsum dots), so it is computed once here -- with the same run_oracle the worker
would call -- and committed as tests/golden/multislab_oracle.json; the worker reads it and recomputes
only a case the fixture lacks.

  OMP_NUM_THREADS=1 python tests/golden/make_multislab_oracle.py   (~10 min on 6 processes)
"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "multislab_oracle.json")


def job(args):
    grid, kind, kw = args
    sys.argv = ["x"]
    from tests import multislab_worker as W
    return grid, W.case_key(kind, kw), W.run_oracle(kind, grid, **kw)


def main():
    from tests import multislab_worker as W
    jobs = [(grid, kind, kw) for grid in (256, 384) for kind, kw in W.cases_for(grid, W.DEFAULT_ITERS)]
    out = {}
    with ProcessPoolExecutor(max_workers=6) as ex:
        for grid, key, res in ex.map(job, jobs):
            out.setdefault(str(grid), {})[key] = res
            print(grid, key, res["nit"], res["cg_iter"][-1:], flush=True)
    with open(OUT, "w") as f:
        json.dump({"note": "oracle/gnk_oracle.py trajectories of the multislab cases (tests/golden/make_multislab_oracle.py); "
                           "GN with exactly rounded CG dot products (tests/multislab_worker.py exact_cg)", "grids": out}, f)


if __name__ == "__main__":
    main()
