"""Hardware probes for the roofline numbers in DESIGN.md: fp64 MFMA issue rate and
achievable HBM copy bandwidth (torch copy kernel), on cuda:0."""
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gauss_newton_via_generalized_krylov_subspaces_amd._native import HipBackend  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    be = HipBackend(dev)
    out = torch.zeros(256, dtype=torch.float64, device=dev)
    res = {}
    for blocks, iters in ((1024, 2000), (2048, 2000)):
        be.probe_mfma(out, blocks, 10)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        be.probe_mfma(out, blocks, iters)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e)
        n_mfma = blocks * 4 * iters * 4          # blocks x 4 waves x iters x 4 MFMAs
        flops = n_mfma * 2 * 16 * 16 * 4
        res[f"mfma_f64_blocks{blocks}"] = {"ms": ms, "TFLOPs": flops / ms / 1e9,
                                           "cycles_per_mfma_per_simd_at_2.4GHz": (ms * 1e-3 * 2.4e9) / (n_mfma / 1024)}
    for mb in (512, 2048):
        n = mb * 1024 * 1024 // 8
        a = torch.randn(n, dtype=torch.float64, device=dev)
        b = torch.empty_like(a)
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            b.copy_(a)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 10
        res[f"copy_{mb}MiB"] = {"ms": ms, "GBs": 2 * n * 8 / ms / 1e6}
    props = torch.cuda.get_device_properties(0)
    res["device"] = {"name": props.name, "cus": props.multi_processor_count, "mem_GB": props.total_memory / 1e9}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
