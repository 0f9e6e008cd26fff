"""Summarise tools/pmc.sh passes over kbench gram2 runs of the wide Gram kernels into
profiles/<round>/pmc_wide_gram.json: HBM fetch vs algorithmic bytes, L2 hit rate, SQ instruction
mix, and the useful fp64 rate against the MI355X fp64 MFMA peak (78.6 TF/s).

  python tools/pmc_wide_summary.py OUT.json grid k1=DIR1 k2=DIR2 ...
Useful flops per grid point: the triangular transform Y = W P^-1 and the symmetric Gram of the
K = k + 1 columns (with r): 2 * K (K + 1) / 2 each.  FETCH_SIZE x2 (16-B/lane reads, MI355X_MICROARCH.md
HBM section; the pass's stencil loads are 16 B/lane, its in-row neighbours 8-B loads of lines the
centre load fetched).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

PEAK_TF = 78.6
WIDE = re.compile(r"k_gram(?:_x|_w|_wp)?<")


def rows(d, counter):
    out = defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == counter:
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                out[name].append((float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    return out


def main(outp, grid, cases):
    n = grid * grid
    res = {"note": __doc__.strip().splitlines()[0], "grid": grid, "peak_fp64_tflops": PEAK_TF, "cases": {}}
    for case in cases:
        k, d = case.split("=")
        k = int(k)
        c = {}
        for counter, key in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write"), ("TCC_HIT_sum", "tcc_hit"),
                             ("TCC_MISS_sum", "tcc_miss"), ("SQ_WAVE_CYCLES", "sq_wave_cycles"),
                             ("SQ_WAIT_ANY", "sq_wait_any"), ("SQ_BUSY_CYCLES", "sq_busy"),
                             ("SQ_INSTS_VMEM", "sq_insts_vmem"), ("SQ_INSTS_LDS", "sq_insts_lds"),
                             ("SQ_INSTS_VALU", "sq_insts_valu"), ("SQ_VALU_MFMA_BUSY_CYCLES", "sq_mfma_busy")):
            for p in sorted(glob.glob(os.path.join(d, "p*"))):
                vals = rows(p, counter)
                for name, lst in vals.items():
                    if WIDE.search(name):
                        big = [v for v in lst if v[1] > 1e6]          # bench-grid launches (> 1 ms)
                        if big:
                            c["kernel"] = name
                            c[key] = sum(v for v, _ in big) / len(big)
                            c.setdefault("ms", sum(t for _, t in big) / len(big) / 1e6)
        if "fetch" not in c:
            continue
        K = k + 1
        alg = 8.0 * n * (k + 2)
        flops = n * 2.0 * K * (K + 1)          # transform + Gram, FMA = 2 flops
        c["fetch_bytes_corrected"] = 2 * c.pop("fetch") * 1024
        c["write_bytes"] = c.pop("write") * 1024
        c["algorithmic_bytes"] = alg
        c["fetch_over_algorithmic"] = c["fetch_bytes_corrected"] / alg
        c["tcc_hit_rate"] = c["tcc_hit"] / (c["tcc_hit"] + c["tcc_miss"]) if "tcc_miss" in c else None
        c["useful_tflops"] = flops / (c["ms"] * 1e-3) / 1e12
        c["frac_of_fp64_mfma_peak"] = c["useful_tflops"] / PEAK_TF
        if "sq_wave_cycles" in c:
            c["sq_wait_any_frac"] = c["sq_wait_any"] / c["sq_wave_cycles"]
        res["cases"][f"k={k}"] = c
    json.dump(res, open(outp, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3:])
