"""HBM traffic per kernel launch from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, one pass each: they do not fit one pass together), stamped with
the build it was measured on (bench.py only quotes a traffic figure whose
build stamp equals the running build).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide coalesced reads
(128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is taken as is.
Other access widths are uncalibrated there, so for kernels dominated by narrow
random reads the doubled figure is an upper estimate.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG N_SPANS OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def per_launch(d, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                k = r["Kernel_Name"].split("(")[0].replace("kmz::", "").replace("void ", "")
                acc[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


fetch = per_launch(sys.argv[1], "FETCH_SIZE")
write = per_launch(sys.argv[2], "WRITE_SIZE")
out = {"build": bench.build_id(), "config": int(sys.argv[3]), "n_spans": int(sys.argv[4]),
       "unit": "bytes per launch", "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f = 2 * 1024 * fetch.get(k, 0.0)
    w = 1024 * write.get(k, 0.0)
    out["kernels"][k] = {"fetch_bytes": round(f), "write_bytes": round(w), "traffic_bytes": round(f + w)}
json.dump(out, open(sys.argv[5], "w"), indent=1)
print(json.dumps(out, indent=1))
