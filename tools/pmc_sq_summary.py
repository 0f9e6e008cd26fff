"""Summarise a rocprofv3 SQ counter pass over the bench command (tools/pmc_bench_sq.sh) into the fp64
pipe use of the Gram passes of exactly the timed window, per basis size k.

  python tools/pmc_sq_summary.py <pmc dir> <config key> <bench window json>

Counters (MI355X_MICROARCH.md, PMC units): SQ_VALU_MFMA_BUSY_CYCLES counts MFMA pipe cycles summed over
all SIMDs; GRBM_GUI_ACTIVE counts GPU cycles summed over the 8 XCDs, so the SIMD-cycles available to a
dispatch are 128 x GRBM_GUI_ACTIVE (32 CUs x 4 SIMDs per XCD) and
  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (128 GRBM_GUI_ACTIVE).
SQ_WAVE_CYCLES / SQ_WAIT_INST_ANY are quad-cycles per wave (their ratio is the share of a wave's life
spent waiting for an instruction's operands: memory, LDS or the fp64 pipe).  SQ_INSTS_* are wave
instructions.  Per k: the window's launches at that basis size (the algorithmic bytes per launch
8 n (k + 2) give k), averaged.  Also the effective clock GRBM_GUI_ACTIVE / 8 / duration.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

GRAM = re.compile(r"k_gram_(?:[smwqx]p?|v1?)<")
MIN_NS = 100e3                       # bench-grid Gram launches take >= 0.28 ms; the 256^2 pre-warm's a few us
CTRS = ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY",
        "SQ_WAVE_CYCLES", "SQ_INSTS_LDS", "GRBM_GUI_ACTIVE")


def load(d):
    """dispatch id -> {kernel, ns, counters}"""
    disp = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(p)):
            did = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
            e = disp.setdefault(did, {"kernel": row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0],
                                      "ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), "c": {}})
            e["c"][row["Counter_Name"]] = e["c"].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    return disp


def main(d, config, window_path):
    disp = load(d)
    with open(window_path) as fh:
        win = json.load(fh)
    seq = [disp[i] for i in sorted(disp) if GRAM.search(disp[i]["kernel"]) and disp[i]["ns"] > MIN_NS]
    lo, cnt = win["gram_launch_offset"], win["gram_launches"]
    sel = seq[lo:lo + cnt]
    if len(sel) != cnt:
        raise SystemExit(f"window {lo}+{cnt} outside the {len(seq)} bench-grid Gram launches")
    n = win["grid"] ** 2
    byk = defaultdict(list)
    for e, b in zip(sel, win["launch_bytes"]):
        byk[int(round(b / (8.0 * n))) - 2].append(e)
    per_k = {}
    tot_busy = tot_avail = 0.0
    for k, es in sorted(byk.items()):
        c = {name: sum(e["c"].get(name, 0.0) for e in es) / len(es) for name in CTRS}
        ms = sum(e["ns"] for e in es) / len(es) / 1e6
        avail = 128.0 * c["GRBM_GUI_ACTIVE"]
        tot_busy += c["SQ_VALU_MFMA_BUSY_CYCLES"] * len(es)
        tot_avail += avail * len(es)
        per_k[str(k)] = {"kernel": es[0]["kernel"], "launches": len(es), "ms_under_pmc": ms,
                         "mfma_busy": c["SQ_VALU_MFMA_BUSY_CYCLES"] / avail if avail else None,
                         "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"] if c["SQ_WAVE_CYCLES"] else None,
                         "insts_valu": c["SQ_INSTS_VALU"], "insts_mfma": c["SQ_INSTS_MFMA"], "insts_lds": c["SQ_INSTS_LDS"],
                         "clock_ghz": c["GRBM_GUI_ACTIVE"] / 8.0 / (ms * 1e6) if ms else None,
                         "counters": c}
    out = {"note": __doc__.strip().splitlines()[0], "config": config,
           "window": {k: win[k] for k in ("warmup", "steps", "repeats", "gram_launch_offset", "gram_launches",
                                          "algorithmic_bytes_per_launch")},
           "mfma_busy": tot_busy / tot_avail if tot_avail else None, "per_k": per_k}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
