"""Static instruction counts of one kernel in a device assembly file (hipcc
--offload-device-only -S): totals by class, and the same for its hottest loop
(the basic blocks between the loop header and its back-edge with the most
VALU instructions).  Development aid: compares builds before a GPU A/B.

    python tools/isa_stats.py file.s 'k_blind_rotateILi3ELb1ELb1ELb1ELb1E'
"""
import re
import sys
from collections import Counter


def kernel_body(lines, pat):
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\w*" + pat + r"\w*:", l):
            start = i
        elif start is not None and (l.startswith("\t.end_amdhsa") or re.match(r"^\.Lfunc_end", l)):
            return lines[start:i]
    raise SystemExit(f"kernel {pat} not found")


def klass(op):
    if op.startswith("v_") and "f64" in op:
        return "valu_f64"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    return "other"


def stats(body):
    c = Counter()
    ops = Counter()
    for l in body:
        t = l.strip()
        if not t or t.startswith((".", ";", "//")) or re.match(r"^[\w.]+:", t):
            continue
        op = t.split()[0]
        c[klass(op)] += 1
        ops[op] += 1
    return c, ops


def loops(body):
    """(label, first line, back-edge line) of every backward branch."""
    labels = {}
    out = []
    for i, l in enumerate(body):
        t = l.strip()
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            labels[m.group(1)] = i
        m = re.match(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", t)
        if m:
            lab = m.group(1) or m.group(2)
            if lab in labels:
                out.append((lab, labels[lab], i))
    return out


def main():
    lines = open(sys.argv[1]).read().splitlines()
    body = kernel_body(lines, sys.argv[2])
    c, ops = stats(body)
    print("kernel total:", dict(c))
    best = None
    for lab, a, b in loops(body):
        lc, _ = stats(body[a:b + 1])
        v = lc["valu_f64"] + lc["valu_other"]
        if best is None or v > best[0]:
            best = (v, lab, lc, body[a:b + 1])
    if best:
        v, lab, lc, seg = best
        print(f"hottest loop {lab} ({len(seg)} lines):", dict(lc), "valu", v)
        _, lops = stats(seg)
        print("  top ops:", lops.most_common(25))


if __name__ == "__main__":
    main()
