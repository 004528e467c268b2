"""Communication / compute overlap from a rocprofv3 ``--kernel-trace`` CSV.

Usage: python tools/prof_overlap.py <kernel_trace.csv> [--comm-regex REGEX] [--steps 3] [--marker sgd]

For the last ``--steps`` training steps (delimited by the fused optimizer kernel, as in
``prof_summary.py``) reports the number and total time of communication kernels (RCCL by
default), how much of that time overlapped with compute kernels on other streams, and the
step's wall time.  Output is markdown for ``profiles/``.
"""
from __future__ import annotations

import argparse
import csv
import re


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def _union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Total length of the intersection of two sorted, disjoint interval lists."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--comm-regex", default=r"ncclDevKernel|rccl|oneRank|nccl")
    ap.add_argument("--marker", default="sgd")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--copies", default=None, help="rocprofv3 --memory-copy-trace CSV: count copies as comm")
    a = ap.parse_args()
    ks = []
    with open(a.trace) as f:
        for row in csv.DictReader(f):
            name = _col(row, "Kernel_Name", "KernelName", "Name")
            s = int(_col(row, "Start_Timestamp", "BeginNs", "Start"))
            e = int(_col(row, "End_Timestamp", "EndNs", "End"))
            q = row.get("Stream_Id") or row.get("Queue_Id") or row.get("Queue_ID") or "?"
            ks.append((s, e, name, q))
    if a.copies:
        with open(a.copies) as f:
            for row in csv.DictReader(f):
                s = int(_col(row, "Start_Timestamp", "BeginNs", "Start"))
                e = int(_col(row, "End_Timestamp", "EndNs", "End"))
                d = row.get("Direction") or row.get("Operation") or "copy"
                ks.append((s, e, "memcpy:%s" % d, "copy"))
    ks.sort()
    marks = [s for s, e, n, q in ks if re.search(a.marker, n)]
    if len(marks) < a.steps + 1:
        print("not enough steps (%d markers)" % len(marks))
        return
    lo, hi = marks[-a.steps - 1], marks[-1]
    comm_re = re.compile(a.comm_regex)
    comm = [(s, e) for s, e, n, q in ks if lo <= s < hi and comm_re.search(n)]
    comp = [(s, e) for s, e, n, q in ks if lo <= s < hi and not comm_re.search(n)]
    cu, pu = _union(comm), _union(comp)
    ct = sum(e - s for s, e in cu)
    ov = _overlap(cu, pu)
    wall = (hi - lo) / a.steps
    print("| steps | wall ms/step | comm kernels/step | comm busy ms/step | overlapped with compute | exposed comm ms/step |")
    print("|---:|---:|---:|---:|---:|---:|")
    print("| %d | %.3f | %.1f | %.3f | %.1f %% | %.3f |" % (
        a.steps, wall / 1e6, len(comm) / a.steps, ct / a.steps / 1e6, 100.0 * ov / ct if ct else 0.0,
        (ct - ov) / a.steps / 1e6))
    names = {}
    for s, e, n, q in ks:
        if lo <= s < hi and comm_re.search(n):
            k = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", "").replace("void ", "", 1))[:90]
            names[k] = names.get(k, 0) + (e - s)
    for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:8]:
        print("| `%s` | %.3f ms/step |" % (k, v / a.steps / 1e6))


if __name__ == "__main__":
    main()
