#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh): per kernel, the mean of each counter per dispatch.

  python tools/pmc_summary.py gpurun_out/<tag> [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))
    meta = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {x: r[x] for x in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                         "Accum_VGPR_Count", "SGPR_Count")}
    return acc, meta


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc, meta = load(root)
    for k in sorted(acc):
        if filt not in k:
            continue
        print(k, meta[k])
        for c in sorted(acc[k]):
            v = acc[k][c]
            print("   %-24s %16.1f  (n=%d)" % (c, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main()
