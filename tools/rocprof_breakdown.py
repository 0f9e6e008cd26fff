"""Per-cycle kernel-time breakdown of the bench's timed window from a rocprofv3 kernel trace.

  python tools/rocprof_breakdown.py <run_kernel_trace.csv> <bench window json (GNK_BENCH_WINDOW_OUT)> [cycles] [min_ns]

The window runs from the first timed Gram launch to the launch after the last one (tools/rocprof_window.py's
selection of the bench-grid Gram launches: longer than min_ns, default 10 us, which drops the 256^2
pre-warm's); every kernel that starts inside it is summed per name, and
the totals are divided by the number of restart cycles timed (``cycles``, default: the bench's repeats).
Also reports the GPU-busy fraction (union of kernel intervals over the window span) and launches per cycle.
"""
import csv
import json
import re
import sys
from collections import defaultdict

GRAM = re.compile(r"k_gram_(?:[smwqx]p?|v1?)<")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].split("<")[0]


def main(trace, window, cycles=None, min_ns=10_000):
    win = json.load(open(window))
    rows = []
    for r in csv.DictReader(open(trace)):
        rows.append((int(r.get("Dispatch_Id") or r["Correlation_Id"]), int(r["Start_Timestamp"]),
                     int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    grams = [r for r in rows if GRAM.search(r[3]) and r[2] - r[1] > int(min_ns)]
    lo, cnt = win["gram_launch_offset"], win["gram_launches"]
    t0 = grams[lo][1]
    if lo + cnt < len(grams) and "trial" not in win:
        t1 = grams[lo + cnt][1]
    else:
        # the window's last step: its first trial, then the residual and the reductions that follow it
        TRIAL = re.compile(r"k_gemv_vjpg<")
        t = win.get("trial") or {}
        trials = [r for r in rows if TRIAL.search(r[3]) and r[2] - r[1] > int(min_ns)]
        last = trials[t["trial_launch_offset"] + t["trial_launches"] - 1] if t else grams[lo + cnt - 1]
        after = [r for r in rows if r[0] > last[0]]
        res = next((i for i, r in enumerate(after) if "k_forward" in r[3]), None)
        t1 = last[2]
        if res is not None:
            t1 = after[res][2]
            for r in after[res + 1:]:
                if "reduce" not in r[3]:
                    break
                t1 = r[2]
    sel = [r for r in rows if t0 <= r[1] < t1]
    ncyc = float(cycles) if cycles else float(win.get("repeats", 1))
    per = defaultdict(float)
    calls = defaultdict(int)
    for _, s, e, n in sel:
        per[short(n)] += (e - s) / 1e6
        calls[short(n)] += 1
    iv = sorted((s, e) for _, s, e, _ in sel)
    busy, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    out = {"window_span_ms": (t1 - t0) / 1e6, "kernels_busy_ms": busy / 1e6, "busy_frac": busy / (t1 - t0),
           "cycles": ncyc, "launches_per_cycle": len(sel) / ncyc,
           "ms_per_cycle": {k: round(v / ncyc, 4) for k, v in sorted(per.items(), key=lambda t: -t[1])},
           "calls_per_cycle": {k: round(calls[k] / ncyc, 2) for k in sorted(per, key=lambda t: -per[t])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
