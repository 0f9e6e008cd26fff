"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into HBM bytes per launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per 128-B request of a
wide (16 B/lane) coalesced read, i.e. reports half the bytes -> x2; WRITE_SIZE is exact for
16-B stores.  Both counters are in KiB.  The Gram kernel's loads are 16 B per lane.

  python tools/pmc_summary.py <pmc dir> <config key> [<bench window json>]

With the window file that bench.py wrote in the same run (GNK_BENCH_WINDOW_OUT: the number of
bench-grid Gram launches before the timed regions and their count), the Gram traffic is taken over
exactly the timed regions' launches (in dispatch order) and the summary records that window and
its algorithmic bytes, which bench.py matches before it reports the traffic.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

GRAM = re.compile(r"k_gram_(?:[smwqx]p?|v1?)<")    # every Gram-pass kernel (staged / marching / chunked / VALU)
TRIAL = re.compile(r"k_gemv_vjpg<")                # the first Armijo trial + update products
BENCH_GRID_MIN = 50e6                              # bytes: launches on the bench grid (not the 256^2 pre-warm)


def load(d, counter):
    """kernel -> [(dispatch id, bytes)] in dispatch order."""
    vals = defaultdict(list)
    for p in glob.glob(os.path.join(d, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            if row["Counter_Name"] == counter:
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                did = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
                vals[name].append((did, float(row["Counter_Value"]) * 1024.0))
    for v in vals.values():
        v.sort()
    return vals


def section(f, w, pat, win, off_key, cnt_key):
    """Launches of the kernels matching pat on the bench grid, in dispatch order across those kernels;
    with a window: exactly the timed regions' launches, their traffic and the window's algorithmic bytes."""
    gf = sorted((did, v) for name, lst in f.items() if pat.search(name) for did, v in lst if v > BENCH_GRID_MIN)
    gw = dict((did, v) for name, lst in w.items() if pat.search(name) for did, v in lst)
    seq = [(did, 2 * v + gw.get(did, 0.0)) for did, v in gf]
    out = {}
    if win:
        lo, cnt = win[off_key], win[cnt_key]
        sel = seq[lo:lo + cnt]
        if len(sel) != cnt:
            raise SystemExit(f"window {lo}+{cnt} outside the {len(seq)} bench-grid launches of {pat.pattern}")
        alg = win["launch_bytes"]
        out["window"] = {k: win[k] for k in ("warmup", "steps", "repeats", off_key, cnt_key,
                                             "algorithmic_bytes_per_launch")}
        out["traffic_bytes_per_launch"] = sum(t for _, t in sel) / cnt
        out["traffic_over_algorithmic"] = sum(t for _, t in sel) / sum(alg)
        out["per_launch"] = [{"algorithmic": a, "traffic": t} for a, (_, t) in zip(alg, sel)]
    elif seq:
        out["traffic_bytes_per_launch"] = sum(t for _, t in seq) / len(seq)
    return out


def main(d, config=None, window_path=None):
    f = load(d, "FETCH_SIZE")
    w = load(d, "WRITE_SIZE")
    out = {"correction": "FETCH_SIZE x2 (16-B/lane reads on gfx950), WRITE_SIZE x1; KiB -> bytes", "kernels": {}}
    for name in sorted(set(f) | set(w)):
        fa = [v for _, v in f.get(name, [])]
        wa = [v for _, v in w.get(name, [])]
        keep = [i for i, v in enumerate(fa) if v > BENCH_GRID_MIN]
        fv = [fa[i] for i in keep]
        wv = [wa[i] for i in keep if i < len(wa)]
        if not fv:
            continue
        fm = sum(fv) / len(fv)
        wm = sum(wv) / len(wv) if wv else 0.0
        out["kernels"][name] = {"launches": len(fv), "fetch_bytes_raw": fm, "fetch_bytes_corrected": 2 * fm,
                                "write_bytes": wm, "traffic_bytes_per_launch": 2 * fm + wm}
    if config:
        out["config"] = config
    win = None
    if window_path:
        with open(window_path) as fh:
            win = json.load(fh)
    out["gram_kernels"] = sorted(k for k in out["kernels"] if GRAM.search(k))
    out.update(section(f, w, GRAM, win, "gram_launch_offset", "gram_launches"))
    if win and "trial" in win:
        out["trial"] = section(f, w, TRIAL, win["trial"], "trial_launch_offset", "trial_launches")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None, sys.argv[3] if len(sys.argv) > 3 else None)
