"""How much of the emulated all-reduce kernels' time overlaps other kernels (rocprofv3 kernel trace)?
Usage: python tools/diag/emu_overlap.py <prof_kernel_trace.csv> [--last-frac 0.5]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--last-frac", type=float, default=0.5, help="analyse only the last fraction of the trace (timed steps)")
a = ap.parse_args()
rows = []
with open(a.csv) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
t0, t1 = rows[0][0], max(e for _, e, _ in rows)
cut = t1 - (t1 - t0) * a.last_frac
rows = [r for r in rows if r[0] >= cut]
emu = [(s, e) for s, e, n in rows if "comm_emu" in n]
other = sorted((s, e) for s, e, n in rows if "comm_emu" not in n)
merged = []
for s, e in other:  # union of the other kernels' intervals
    if merged and s <= merged[-1][1]:
        merged[-1][1] = max(merged[-1][1], e)
    else:
        merged.append([s, e])
tot = sum(e - s for s, e in emu)
ov = 0
for s, e in emu:
    for ms, me in merged:
        if me <= s:
            continue
        if ms >= e:
            break
        ov += min(e, me) - max(s, ms)
span = rows[-1][1] - rows[0][0]
busy = sum(e - s for s, e in merged)
print("window %.2f ms: comm_emu kernels %d, %.2f ms, overlapped with other kernels %.2f ms (%.0f %%); "
      "other kernels busy %.2f ms" % (span / 1e6, len(emu), tot / 1e6, ov / 1e6, 100.0 * ov / max(tot, 1), busy / 1e6))
