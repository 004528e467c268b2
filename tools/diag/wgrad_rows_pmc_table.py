"""Table of tools/runs/gpu_r5_t12.sh's rocprofv3 --pmc passes over the row-image weight gradient
(wgrad_rows_pmc.py): per shape and variant, the median kernel time and the mean of each counter
over the 5 dispatches of wgrad_rows_rect_kernel (the reduce kernel excluded)."""
import collections
import csv
import glob
import os
import sys

NAMES = {0: "Conv2d_2a 111x111 32->32 3x3", 1: "Conv2d_2b 109x109 32->64 3x3 p1", 2: "Conv2d_4a 54x54 80->192 3x3",
         3: "Mixed_5 25x25 96->96 3x3 p1", 4: "Mixed_6 12x12 160->160 1x7"}


def main():
    out = sys.argv[1]
    rows = []
    for d in sorted(glob.glob(os.path.join(out, "r5wr_s*_v*_p1"))):
        tag = os.path.basename(d)[len("r5wr_"):-3]
        s, v = tag.split("_")
        vals = collections.defaultdict(list)
        us = []
        for p in (1, 2, 3):
            for f in glob.glob(os.path.join(out, "r5wr_%s_p%d" % (tag, p), "**", "*counter_collection.csv"), recursive=True):
                per = collections.defaultdict(dict)
                for r in csv.DictReader(open(f)):
                    if "wgrad_rows_rect_kernel" not in r["Kernel_Name"]:
                        continue
                    c = per[r["Dispatch_Id"]]
                    c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                for c in per.values():
                    for k, x in c.items():
                        vals[k].append(x)
            if p == 1:
                for f in glob.glob(os.path.join(out, "r5wr_%s_p1" % tag, "**", "*kernel_trace.csv"), recursive=True):
                    for r in csv.DictReader(open(f)):
                        if "wgrad_rows_rect_kernel" in r["Kernel_Name"]:
                            us.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        m = {k: sum(x) / len(x) for k, x in vals.items()}
        us.sort()
        rows.append((NAMES[int(s[1:])], v[1:], us[len(us) // 2] if us else 0.0, m))
    cols = ["SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
            "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "TCP_TCC_READ_REQ_sum", "TCC_HIT_sum",
            "TCC_MISS_sum"]
    print("| shape | variant | us | MFMA busy % | " + " | ".join(cols) + " |")
    print("|---|---|---:|---:|" + "---:|" * len(cols))
    for name, v, us, m in rows:
        b = m.get("SQ_BUSY_CYCLES", 0)
        mb = "%.1f" % (100 * m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / b) if b else "-"
        print("| %s | %s | %.1f | %s | " % (name, v, us, mb) + " | ".join("%.4g" % m.get(c, 0) for c in cols) + " |")


if __name__ == "__main__":
    main()
