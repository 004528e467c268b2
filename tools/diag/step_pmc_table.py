"""Per-kernel-family PMC table of one training step from several rocprofv3 --pmc passes over the
same bench.py run (one counter group per pass, tools/runs/gpu_r6_pmc.sh).  Like roofline_table.py
the step is the dispatches between the last two optimizer kernels (--marker); passes are aligned
by dispatch order inside that step and checked by kernel name.  Per family (name + grid): launches,
us, and per-launch-summed counters, then derived columns:

  MFMA busy % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
                (GRBM_GUI_ACTIVE is summed over the 8 XCDs, the MFMA busy cycles over the SIMDs;
                checked: the 3x3 256x256 tile at 826 TF/s by MOPS reads 32 %)
  TF/s        = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / us
  occupancy   = SQ_WAVE_CYCLES / SQ_BUSY_CYCLES                      (waves resident per busy SE-cycle)
  wait %      = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  LDS wait %  = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES
  TB/s        = (FETCH_SIZE + WRITE_SIZE) / us
"""
import argparse
import collections
import csv
import glob
import os
import re

BW = 5.3e12
CUS = 256


def load(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            e = rows.setdefault(k, {"name": r["Kernel_Name"], "grid": r.get("Grid_Size", ""), "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    durs = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return [(k, rows[k]) for k in sorted(rows)], durs


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
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--marker", default="sgd")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    steps, durs = [], None
    for d in a.dirs:
        s, du = load(d)
        steps.append(last_step(s, a.marker))
        if durs is None:
            durs = du
    names = [e["name"] for _, e in steps[0]]
    for s in steps[1:]:
        if [e["name"] for _, e in s] != names:
            raise SystemExit("passes differ in kernel sequence")
    fam = collections.OrderedDict()
    for i, (k0, e0) in enumerate(steps[0]):
        key = (short(e0["name"]), e0["grid"])
        f = fam.setdefault(key, {"n": 0, "us": 0.0, "c": collections.defaultdict(float)})
        f["n"] += 1
        f["us"] += durs.get(k0, 0.0)
        for s in steps:
            for c, v in s[i][1]["c"].items():
                f["c"][c] += v
    rows = sorted(fam.items(), key=lambda kv: -kv[1]["us"])
    if a.filter:
        rows = [r for r in rows if re.search(a.filter, r[0][0])]
    cols = sorted({c for _, f in rows for c in f["c"]})

    def g(f, c):
        return f["c"].get(c)

    print("| kernel | grid | n | us | TF/s | MFMA busy % | occ | wait % | LDS wait % | TB/s | % of 5.3 TB/s | "
          + " | ".join(cols) + " |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|" + "---:|" * len(cols))
    for (name, grid), f in rows[:a.top]:
        mb, ga = g(f, "SQ_VALU_MFMA_BUSY_CYCLES"), g(f, "GRBM_GUI_ACTIVE")
        mfma = "%.1f" % (100 * mb * 8 / (ga * 1024)) if mb is not None and ga else "-"
        wc, bc = g(f, "SQ_WAVE_CYCLES"), g(f, "SQ_BUSY_CYCLES")
        occ = "%.1f" % (wc / bc) if wc and bc else "-"
        wa = "%.0f" % (100 * g(f, "SQ_WAIT_ANY") / wc) if wc and g(f, "SQ_WAIT_ANY") is not None else "-"
        wl = "%.0f" % (100 * g(f, "SQ_WAIT_INST_LDS") / wc) if wc and g(f, "SQ_WAIT_INST_LDS") is not None else "-"
        fs, ws = g(f, "FETCH_SIZE"), g(f, "WRITE_SIZE")
        bw = (fs + ws) * 1024 / (f["us"] * 1e-6) if fs is not None and ws is not None and f["us"] else None
        tbs = "%.2f" % (bw / 1e12) if bw else "-"
        pct = "%.0f" % (100 * bw / BW) if bw else "-"
        mo = g(f, "SQ_INSTS_VALU_MFMA_MOPS_BF16")
        tf = "%.0f" % (mo * 512 / (f["us"] * 1e-6) / 1e12) if mo and f["us"] else "-"
        print("| `%s` | %s | %d | %.1f | %s | %s | %s | %s | %s | %s | %s | " % (
            name, grid, f["n"], f["us"], tf, mfma, occ, wa, wl, tbs, pct)
              + " | ".join("%.3g" % f["c"][c] if c in f["c"] else "-" for c in cols) + " |")


if __name__ == "__main__":
    main()
