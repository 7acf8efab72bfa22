"""Summarise tools/pmc_detail.sh output (csv): per kernel, each counter
averaged per dispatch.  usage: pmc_csv.py gpurun_out/pmcd_TAG"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kmz::", "").replace("void ", "")
        acc[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for k in sorted(acc):
    d = acc[k]
    vals = {c: sum(v.values()) / len(v) for c, v in d.items()}
    print(k)
    for c in sorted(vals):
        print(f"  {c:26s} {vals[c]:16.5g}")
    if "SQ_WAVE_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals:
        wc = vals["SQ_WAVE_CYCLES"]
        print("  -> wait_any %.2f  wait_inst %.2f  active %.2f" % (vals.get("SQ_WAIT_ANY", 0) / wc,
              vals.get("SQ_WAIT_INST_ANY", 0) / wc, vals.get("SQ_ACTIVE_INST_ANY", 0) / wc))
