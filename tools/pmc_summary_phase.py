"""Summarises tools/pmc_phase.sh: instructions per k_doc_fast wave after each phase and per phase."""
import csv
import glob
import os
import sys

out = sys.argv[1]
rows = []
for k in [str(i) for i in range(15)] + ["full"]:
    f = glob.glob(os.path.join(out, "s%s" % k, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    tot = {}
    for r in csv.DictReader(open(f[0])):
        if "k_doc_fast" not in r.get("Kernel_Name", ""):
            continue
        tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    w = tot.get("SQ_WAVES", 0) or 1
    rows.append((k, tot.get("SQ_INSTS_VALU", 0) / w, tot.get("SQ_INSTS_SALU", 0) / w, tot.get("SQ_INSTS_LDS", 0) / w))
prev = (0, 0, 0)
print("%-6s %10s %10s %10s   %8s %8s %8s" % ("stop", "VALU/wave", "SALU/wave", "LDS/wave", "dVALU", "dSALU", "dLDS"))
for k, v, s_, l in rows:
    print("%-6s %10.0f %10.0f %10.0f   %8.0f %8.0f %8.0f" % (k, v, s_, l, v - prev[0], s_ - prev[1], l - prev[2]))
    prev = (v, s_, l)
