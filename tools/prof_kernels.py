"""Per-kernel table (one step, between the last two marker kernels) with grid / VGPR / duration.
Usage: python tools/prof_kernels.py trace.csv [--match REGEX] [--marker sgd]"""
import argparse, csv, re

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--match", default="")
ap.add_argument("--marker", default="sgd")
ap.add_argument("--agg", action="store_true", help="aggregate by kernel name")
a = ap.parse_args()
r = list(csv.DictReader(open(a.trace)))
r.sort(key=lambda x: int(x["Start_Timestamp"]))
idx = [i for i, x in enumerate(r) if re.search(a.marker, x["Kernel_Name"], re.I)]
seg = r[idx[-2] + 1: idx[-1] + 1]


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"kfk::", "", n)
    return re.sub(r"\(.*", "", n)[:100]


agg = {}
for i, x in enumerate(seg):
    if a.match and not re.search(a.match, x["Kernel_Name"]):
        continue
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e3
    if a.agg:
        k = short(x["Kernel_Name"])
        t = agg.setdefault(k, [0.0, 0])
        t[0] += d
        t[1] += 1
    else:
        print("%4d %8.1f us grid %8s vgpr %3s  %s" % (i, d, x["Grid_Size_X"], x["VGPR_Count"], short(x["Kernel_Name"])))
for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print("%9.1f us %4d  %s" % (t, n, k))
