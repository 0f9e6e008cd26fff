"""The committed oracle trajectories of the multi-rank GPU cases (tests/golden/multislab_oracle.json,
made by tests/golden/make_multislab_oracle.py) equal a fresh oracle run: checked on the cheap GNK
case at grid 256 (the GN cases take minutes of exactly rounded CG dots; same code path)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_multislab_oracle_fixture_matches_fresh_oracle():
    sys.argv = ["x"]
    from tests import multislab_worker as W
    with open(W.ORACLE_FIXTURE) as f:
        grids = json.load(f)["grids"]
    for grid in ("256", "384"):
        assert sorted(grids[grid]) == sorted(W.case_key(k, kw) for k, kw in W.cases_for(int(grid), W.DEFAULT_ITERS))
    kind, kw = W.cases_for(256, W.DEFAULT_ITERS)[0]
    fresh = json.loads(json.dumps(W.run_oracle(kind, 256, **kw)))
    assert fresh == grids["256"][W.case_key(kind, kw)]
