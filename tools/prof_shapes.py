"""Per-launch-shape kernel table from a rocprofv3 --kernel-trace CSV: time per step of every
(kernel, grid, workgroup) combination, so two launches of one template on different layers are
told apart.  Steps are counted by a once-per-step marker kernel.

Usage: python tools/prof_shapes.py <kernel_trace.csv> [--marker conv_flip_multi] [--top 60]
"""
import argparse
import collections
import csv
import re

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--marker", default="sgd_f32x4|conv_flip_multi")
ap.add_argument("--top", type=int, default=60)
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
mk = re.compile(a.marker)
marks = collections.Counter(r["Kernel_Name"] for r in rows if mk.search(r["Kernel_Name"]))
steps = max(marks.values()) if marks else 1
agg = collections.defaultdict(list)
for r in rows:
    n = re.sub(r"^void ", "", r["Kernel_Name"]).replace("(anonymous namespace)::", "").split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
    agg[(n[:80], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Workgroup_Size_X"])].append(d)
total = sum(sum(v) for v in agg.values()) / steps
print("steps %d, kernel time %.1f us/step\n" % (steps, total))
print("| us/step | launches/step | us/launch | kernel | blocks | threads |")
print("|---:|---:|---:|---|---:|---:|")
for (n, g, b), v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
    print("| %.1f | %.1f | %.1f | `%s` | %d | %s |" % (sum(v) / steps, len(v) / steps, sum(v) / len(v), n, g, b))
