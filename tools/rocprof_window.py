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

GRAM = re.compile(r"k_gram_(?:[smw]p?|v1?)<")


def main(trace, window):
    win = json.load(open(window))
    rows = []
    for r in csv.DictReader(open(trace)):
        if GRAM.search(r["Kernel_Name"]):
            rows.append((int(r.get("Dispatch_Id") or r["Correlation_Id"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         r["Kernel_Name"]))
    rows.sort()
    # the pre-warm cycle runs the same kernels on a 256^2 grid first: its launches are ~100x shorter
    big = [r for r in rows if r[1] > 50_000]
    lo, cnt = win["gram_launch_offset"], win["gram_launches"]
    sel = big[lo:lo + cnt]
    avg_ms = sum(d for _, d, _ in sel) / len(sel) / 1e6
    print(json.dumps({"gram_launches": len(sel), "avg_launch_ms": avg_ms, "first": sel[0][2].split("(")[0],
                      "bench_window": win}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
