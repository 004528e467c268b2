"""Table of the rocprofv3 passes of tools/runs/gpu_r5_pmc.sh (gemm_pmc.py per BERT shape): per shape,
direction (forward / data gradient) and kernel family (hipBLASLt `Cijk_*` vs gemm.hip `gemm_nt*`), the
mean duration and every counter per 10^9 bf16 MFMA MOPs (so the two families doing the same math
compare directly), plus the derived MFMA-busy share of the busy cycles."""
import collections
import csv
import glob
import os
import sys

SHAPES = ["qkv 768->2304", "out 768->768", "fc1 768->3072", "fc2 3072->768"]


def family(name):
    if "Cijk" in name:
        return "hipBLASLt"
    if "gemm_nt" in name:
        return "gemm_nt"
    return None


def load(out, s):
    """{(family, dir): {counter: mean}} and {(family, dir): mean us} for shape s."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for p in (1, 2, 3):
        files = glob.glob(os.path.join(out, "r5pmc_s%d_p%d" % (s, p), "**", "*counter_collection.csv"), recursive=True)
        for f in files:
            per = collections.OrderedDict()
            for r in csv.DictReader(open(f)):
                fam = family(r.get("Kernel_Name", ""))
                if fam is None:
                    continue
                d = per.setdefault(int(r["Dispatch_Id"]), {"fam": fam, "c": {}})
                d["c"][r["Counter_Name"]] = d["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            seen = collections.Counter()
            for did in sorted(per):
                d = per[did]
                k = seen[d["fam"]]
                seen[d["fam"]] += 1
                direction = "fwd" if k < 5 else "dgrad"
                for c, v in d["c"].items():
                    vals[(d["fam"], direction)][c].append(v)
        for f in glob.glob(os.path.join(out, "r5pmc_s%d_p%d" % (s, p), "**", "*kernel_trace.csv"), recursive=True):
            seen = collections.Counter()
            rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
            for r in rows:
                fam = family(r.get("Kernel_Name", ""))
                if fam is None:
                    continue
                k = seen[fam]
                seen[fam] += 1
                durs[(fam, "fwd" if k < 5 else "dgrad")].append(
                    (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return ({k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()},
            {k: sorted(v)[len(v) // 2] for k, v in durs.items()})


def main():
    out = sys.argv[1]
    cols = ["us", "TF/s", "MFMA busy %", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
            "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
            "SQ_INSTS_VMEM", "TCP_TCC_READ_REQ_sum", "TCC_HIT_sum", "TCC_MISS_sum", "SQ_WAVES"]
    print("# Round 5: BERT-base GEMMs, hipBLASLt vs gemm.hip (rocprofv3 --pmc, 1 MI355X)\n")
    print("Counters are per 10^9 bf16 MFMA MOPs (`SQ_INSTS_VALU_MFMA_MOPS_BF16`, the same for both families "
          "doing the same product); `MFMA busy %` = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES; us = median "
          "kernel duration (kernel trace of the counter runs).  16,384 tokens.\n")
    for s, sname in enumerate(SHAPES):
        v, d = load(out, s)
        K, N = (int(t) for t in sname.split()[1].split("->"))
        print("## %s\n" % sname)
        print("| kernel | " + " | ".join(cols) + " |")
        print("|---|" + "---:|" * len(cols))
        for direction in ("fwd", "dgrad"):
            for fam in ("hipBLASLt", "gemm_nt"):
                c = v.get((fam, direction))
                if not c:
                    continue
                mops = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) or 1.0
                row = []
                us = d.get((fam, direction))
                flops = 2.0 * 16384 * K * N
                for col in cols:
                    if col == "us":
                        row.append("%.1f" % us if us else "-")
                    elif col == "TF/s":
                        row.append("%.0f" % (flops / us / 1e6) if us else "-")
                    elif col == "MFMA busy %":
                        b = c.get("SQ_BUSY_CYCLES")
                        row.append("%.1f" % (100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / b) if b else "-")
                    elif col == "SQ_WAVES":
                        row.append("%.0f" % c.get(col, 0))
                    elif col in c:
                        row.append("%.3g" % (c[col] / mops * 1e9))
                    else:
                        row.append("-")
                print("| %s %s | " % (fam, direction) + " | ".join(row) + " |")
        print()


if __name__ == "__main__":
    main()
