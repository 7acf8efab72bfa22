"""FETCH_SIZE calibration (tools/calib/calib_fetch.hip): per launch, the
counter's bytes (KiB x 1024, before pmc_traffic.py's doubling) against the
bytes the launch is known to read.

usage: calib_fetch.py PMC_DIR
"""
import collections
import csv
import glob
import json
import os
import sys

acc = collections.defaultdict(float)
names = {}
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "FETCH_SIZE":
            d = int(r["Dispatch_Id"])
            acc[d] += float(r["Counter_Value"]) * 1024
            names[d] = r["Kernel_Name"].split("(")[0]
known = {"k_stream": 1 << 30, "k_rand": 50000000 * 16}
rows = []
nrand = 0
for d in sorted(acc):
    k = names[d]
    if k.startswith("__amd"):
        continue  # (the buffers' fills)
    if "stream" in k:
        access, base = "stream (1 GiB, coalesced 16-B words)", known["k_stream"]
    else:
        access = ["random 16-B reads, 64 MiB table", "random 16-B reads, 1 GiB table"][nrand % 2]
        base = known["k_rand"]
        nrand += 1
    rows.append({"dispatch": d, "kernel": k, "access": access, "fetch_size_bytes": acc[d], "known_bytes": base,
                 "ratio": round(acc[d] / base, 3), "bytes_per_16B_read": round(acc[d] / (base / 16), 1)})
print(json.dumps(rows, indent=1))
