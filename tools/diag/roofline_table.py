"""Per-kernel HBM roofline of one training step from two rocprofv3 --pmc passes over the same
bench.py run (tools/runs/gpu_r5_t15.sh): pass 1 FETCH_SIZE, pass 2 WRITE_SIZE (KB per dispatch),
each with --kernel-trace.  The step = the dispatches between the last two launches of the
optimizer kernel (--marker); the two passes are aligned by dispatch order within that step (the
same program, so the same kernel sequence -- checked by name).  Per kernel family (name + grid):
launches, us (pass-1 kernel trace), MB read + written, achieved TB/s and its share of a 5.3 TB/s
streaming roofline (the copy rate measured on the box, tools/stream_bw.hip); the family's
roofline time bytes / 5.3 TB/s and the excess over it, sorted by excess."""
import argparse
import collections
import csv
import glob
import os
import re

BW = 5.3e12  # B/s


def load(d, counter):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = int(r["Dispatch_Id"])
            e = rows.setdefault(k, {"name": r["Kernel_Name"], "v": 0.0, "grid": r.get("Grid_Size", "")})
            e["v"] += float(r["Counter_Value"])
    durs = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    seq = [(k, rows[k]) for k in sorted(rows)]
    return seq, durs


def last_step(seq, marker):
    marks = [i for i, (_, e) in enumerate(seq) if re.search(marker, e["name"], re.I)]
    if len(marks) < 2:
        raise SystemExit("need >= 2 marker kernels, found %d" % len(marks))
    return seq[marks[-2] + 1:marks[-1] + 1]


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0][:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--marker", default="sgd")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    s1, d1 = load(a.fetch_dir, "FETCH_SIZE")
    s2, _ = load(a.write_dir, "WRITE_SIZE")
    st1, st2 = last_step(s1, a.marker), last_step(s2, a.marker)
    if [e["name"] for _, e in st1] != [e["name"] for _, e in st2]:
        raise SystemExit("the two passes' steps differ in kernel sequence")
    fam = collections.OrderedDict()
    tot_us = tot_b = 0.0
    for (k1, e1), (_, e2) in zip(st1, st2):
        key = (short(e1["name"]), e1["grid"])
        f = fam.setdefault(key, [0, 0.0, 0.0, 0.0])
        us = d1.get(k1, 0.0)
        f[0] += 1
        f[1] += us
        f[2] += e1["v"] * 1024
        f[3] += e2["v"] * 1024
        tot_us += us
        tot_b += (e1["v"] + e2["v"]) * 1024
    rows = []
    for (name, grid), (n, us, rb, wb) in fam.items():
        roof = (rb + wb) / BW * 1e6
        rows.append((us - roof, name, grid, n, us, rb, wb, roof))
    rows.sort(reverse=True)
    print("# Per-kernel HBM roofline, one training step (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE)\n")
    print("step: %d dispatches, %.2f ms of kernel time (counter-collection run: kernels serialised), %.2f GB moved"
          " -> %.2f TB/s mean; the step's bytes at %.1f TB/s take %.2f ms\n" % (
              len(st1), tot_us / 1e3, tot_b / 1e9, tot_b / (tot_us * 1e-6) / 1e12 if tot_us else 0, BW / 1e12,
              tot_b / BW * 1e3))
    print("| kernel | grid | launches | us | MB read | MB written | TB/s | % of roofline BW | roofline us | excess us |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for ex, name, grid, n, us, rb, wb, roof in rows[:a.top]:
        tbs = (rb + wb) / (us * 1e-6) / 1e12 if us else 0.0
        print("| `%s` | %s | %d | %.1f | %.1f | %.1f | %.2f | %.0f | %.1f | %.1f |" % (
            name, grid, n, us, rb / 1e6, wb / 1e6, tbs, 100 * tbs * 1e12 / BW, roof, ex))


if __name__ == "__main__":
    main()
