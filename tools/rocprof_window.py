"""Average duration of the bench's timed-window Gram launches from a rocprofv3 kernel trace.

  python tools/rocprof_window.py <run_kernel_trace.csv> <bench window json (GNK_BENCH_WINDOW_OUT)>

Keeps the Gram-pass kernels on the bench grid (launches longer than the 256^2 pre-warm's), in dispatch
order, and averages the window's launches -- the number bench.py's HIP-event timing reports as
roofline.avg_launch_ms for the same run.
"""
import csv
import json
import re
import sys

GRAM = re.compile(r"k_gram_(?:[smwqx]p?|v1?)<")
TRIAL = re.compile(r"k_gemv_vjpg<")


def window_avg(trace, pat, lo, cnt):
    rows = []
    for r in csv.DictReader(open(trace)):
        if pat.search(r["Kernel_Name"]):
            rows.append((int(r.get("Dispatch_Id") or r["Correlation_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         r["Kernel_Name"]))
    rows.sort()
    # the pre-warm cycle runs the same kernels on a 256^2 grid first: its launches are ~100x shorter
    big = [r for r in rows if r[1] > 50_000]
    sel = big[lo:lo + cnt]
    return {"launches": len(sel), "avg_launch_ms": sum(d for _, d, _ in sel) / len(sel) / 1e6,
            "first": sel[0][2].split("(")[0]}


def main(trace, window):
    win = json.load(open(window))
    g = window_avg(trace, GRAM, win["gram_launch_offset"], win["gram_launches"])
    out = {"gram_launches": g["launches"], "avg_launch_ms": g["avg_launch_ms"], "first": g["first"]}
    if "trial" in win:
        t = win["trial"]
        out["trial"] = window_avg(trace, TRIAL, t["trial_launch_offset"], t["trial_launches"])
        win = {k: v for k, v in win.items() if k != "trial"} | {"trial": {k: v for k, v in t.items() if k != "launch_bytes"}}
    out["bench_window"] = {k: v for k, v in win.items() if k != "launch_bytes"}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
