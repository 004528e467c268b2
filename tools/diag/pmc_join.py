"""Join rocprofv3 --pmc passes of the same program dispatch-by-dispatch and print per-kernel-shape
ratios (MFMA busy, wait / issue-stall / active shares, TA / TD busy, VALU per MFMA ...).
    python tools/diag/pmc_join.py DIR_PASS1 DIR_PASS2 ... [--match conv]"""
import argparse
import collections
import csv
import glob
import os
import re


def load(d, match):
    rows = collections.defaultdict(dict)
    meta = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if match not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
            m = re.search(r"(\w+_kernel)<([^>]*)>", r["Kernel_Name"])
            meta[k] = "%s<%s> g%s" % (m.group(1), m.group(2), r.get("Grid_Size", "")) if m else r["Kernel_Name"][:60]
    return [(meta[k], rows[k]) for k in sorted(rows)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="kernel")
    a = ap.parse_args()
    passes = [load(d, a.match) for d in a.dirs]
    n = min(len(p) for p in passes)
    groups = collections.OrderedDict()
    for j in range(n):
        d = {}
        for p in passes:
            d.update(p[j][1])
        groups.setdefault(passes[0][j][0], []).append(d)
    for name, lst in groups.items():
        a_ = {c: sum(x.get(c, 0.0) for x in lst) / len(lst) for c in lst[0]}
        out = []
        cyc = a_.get("GRBM_GUI_ACTIVE", 0) / 8
        wc = a_.get("SQ_WAVE_CYCLES")
        if cyc and "SQ_VALU_MFMA_BUSY_CYCLES" in a_:
            out.append("mfma %.1f%%" % (100 * a_["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024)))
        if wc:
            for c, t in (("SQ_WAIT_ANY", "wait"), ("SQ_WAIT_INST_ANY", "stall"), ("SQ_ACTIVE_INST_ANY", "active"),
                         ("SQ_WAIT_INST_LDS", "ldsstall")):
                if c in a_:
                    out.append("%s %.1f%%" % (t, 100 * a_[c] / wc))
        for c, t in (("TA_TA_BUSY_sum", "ta"), ("TD_TD_BUSY_sum", "td")):
            if c in a_ and cyc:
                out.append("%s %.1f%%" % (t, 100 * a_[c] / 256 / cyc))
        if "SQ_INSTS_VALU" in a_ and a_.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) > 0:
            nm = a_["SQ_VALU_MFMA_BUSY_CYCLES"] / 16  # 16x16x32 bf16: 16 busy cycles each
            out.append("valu/mfma %.2f salu/mfma %.2f lds/mfma %.2f" % (
                a_["SQ_INSTS_VALU"] / nm, a_.get("SQ_INSTS_SALU", 0) / nm, a_.get("SQ_INSTS_LDS", 0) / nm))
        if "SQ_LDS_BANK_CONFLICT" in a_:
            out.append("bankconf %.3g" % a_["SQ_LDS_BANK_CONFLICT"])
        if "FETCH_SIZE" in a_:
            out.append("fetch %.1f MB" % (a_["FETCH_SIZE"] / 1e3))
        if "SQ_WAVES" in a_:
            out.append("waves %d" % a_["SQ_WAVES"])
        if cyc:
            out.append("%.1f us@2.1GHz" % (cyc / 2.1e3))
        print("%-50s n=%d  %s" % (name[:50], len(lst), "  ".join(out)))


if __name__ == "__main__":
    main()
