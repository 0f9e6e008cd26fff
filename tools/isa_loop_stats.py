"""Instruction mix of a kernel's hot loop, from the gfx950 assembly hipcc writes with -save-temps.

    cd gauss_newton_via_generalized_krylov_subspaces_amd/csrc && hipcc <Makefile flags> -save-temps=obj \
        -o /tmp/isa/libgnk.so gnk_kernels.hip
    python tools/isa_loop_stats.py /tmp/isa/gnk_kernels-hip-amdgcn-amd-amdhsa-gfx950.s 'k_gram_sILi2ELi3ELi1ELi1E'

For every function whose symbol contains the pattern: VGPR/AGPR counts and, for the largest loop body
(the instructions between a loop label and the backward branch to it), the counts per class -- fp64 VALU
(v_*_f64 / v_fma_f64 / DPP moves of 64 bits), other VALU, MFMA, LDS, VMEM/DMA, SALU, waitcnt/barrier.
Static counts: an unrolled loop body of R row steps is divided by the `--steps` argument.
"""
import argparse
import re
import sys
from collections import Counter


def functions(text, pattern):
    for m in re.finditer(r"^(\S*%s\S*):\s*;\s*@" % re.escape(pattern), text, re.M):
        name = m.group(1)
        end = text.find(".Lfunc_end", m.end())
        yield name, text[m.end():end], text


def classify(op, line):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_barrier")):
        return "sync"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        if "f64" in op or op.startswith("v_mov_b64") or op.startswith("v_lshl_add_u64") or op.startswith("v_pk_mov_b32"):
            return "valu64" if "f64" in op else "valu_mov64"
        return "valu32"
    return "other"


def loops(body):
    """(label, [instruction lines]) for every backward branch target."""
    lines = body.split("\n")
    labels = {}
    out = []
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.match(r"^\s+s_cbranch_\w+\s+(\.LBB\w+)|^\s+s_branch\s+(\.LBB\w+)", ln)
        if m:
            tgt = m.group(1) or m.group(2)
            if tgt in labels and labels[tgt] < i:
                out.append((tgt, lines[labels[tgt]:i + 1]))
    return out


def stats(lines):
    c = Counter()
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c[classify(op, s)] += 1
        if "dpp" in s or "row_newbcast" in s:
            c["dpp"] += 1
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("pattern")
    ap.add_argument("--steps", type=int, default=1, help="row steps in the unrolled loop body")
    a = ap.parse_args()
    text = open(a.asm).read()
    found = False
    for name, body, _ in functions(text, a.pattern):
        found = True
        vg = re.search(r"\.set %s\.num_vgpr, (\d+)" % re.escape(name), text)
        ag = re.search(r"\.set %s\.num_agpr, (\d+)" % re.escape(name), text)
        sp = re.search(r"\.set %s\.private_seg_size, (\d+)" % re.escape(name), text)
        print(name)
        print("  vgpr %s agpr %s scratch %s" % (vg and vg.group(1), ag and ag.group(1), sp and sp.group(1)))
        ls = loops(body)
        if not ls:
            print("  no loop")
            continue
        lab, lines = max(ls, key=lambda t: len(t[1]))
        c = stats(lines)
        print("  largest loop %s: %d lines" % (lab, len(lines)))
        print("  " + "  ".join("%s %.1f" % (k, v / a.steps) for k, v in sorted(c.items())))
    if not found:
        sys.exit("no function matches %r" % a.pattern)


if __name__ == "__main__":
    main()
