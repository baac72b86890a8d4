"""Summarise rocprofv3 --pmc CSVs (one dir per pass) for the fused trial kernel.

    python tools/pmc_summary.py gpurun_out/pmc [kernel-substring]
Prints per-dispatch averages of every counter and a few derived ratios.
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "trial_kernel"
vals = collections.defaultdict(list)
for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(float)
    with open(path) as f:
        for row in csv.DictReader(f):
            if pat not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
for c in sorted(avg):
    print(f"{c:32s} {avg[c]:16.4g}  (n={len(vals[c])})")


def ratio(a, b):
    return avg[a] / avg[b] if a in avg and b in avg and avg[b] else None


print("--- derived")
for name, a, b in [("VALU active / wave cycles", "SQ_ACTIVE_INST_VALU", "SQ_WAVE_CYCLES"),
                   ("any-inst active / wave cycles", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES"),
                   ("waiting (any) / wave cycles", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES"),
                   ("waiting for inst / wave cycles", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES"),
                   ("LDS bank conflicts / LDS active", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS"),
                   # MI355X_MICROARCH §LDS: SQ_LDS_IDX_ACTIVE = all LDS-array cycles (conflict cycles included)
                   ("LDS bank conflicts / LDS-array cycles", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"),
                   ("VALU insts per wave", "SQ_INSTS_VALU", "SQ_WAVES")]:
    r = ratio(a, b)
    print(f"{name:34s} {r:.4f}" if r is not None else f"{name:34s} n/a")
