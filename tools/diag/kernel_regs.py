"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (make hip EXTRA_HIPFLAGS=... 2> log):
one line per kernel matching a regex -- VGPRs, AGPRs, spills, LDS, occupancy.
Usage: python tools/diag/kernel_regs.py build_err.log [regex]"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
cur, rows = None, {}
for line in open(sys.argv[1]):
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
names = list(rows)
dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
for n, d in zip(names, dem):
    d = d.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    if not pat.search(d):
        continue
    r = rows[n]
    print("%-60s V %3s A %3s occ %s sgprspill %s vgprspill %s scratch %s lds %s" % (
        d[:60], r.get("VGPRs"), r.get("AGPRs"), r.get("Occupancy [waves/SIMD]"), r.get("SGPRs Spill"),
        r.get("VGPRs Spill"), r.get("ScratchSize [bytes/lane]"), r.get("LDS Size [bytes/block]")))
