"""HBM traffic per kernel launch from two rocprofv3 --pmc passes (FETCH_SIZE and
WRITE_SIZE, one pass each: they do not fit one pass together), stamped with
the build it was measured on (bench.py only quotes a traffic figure whose
build stamp equals the running build).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports half of the bytes of wide coalesced reads
(128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is taken as is.
Other access widths are uncalibrated there, so for kernels dominated by narrow
random reads the doubled figure is an upper estimate.

Two figures per kernel (round 5): `traffic_bytes` = 2 x FETCH_SIZE +
WRITE_SIZE (every read request counted as the 128 B a coalesced stream moves:
the upper figure) and `traffic_lower_bytes` = FETCH_SIZE + WRITE_SIZE (every
request 64 B: a random 16-B read registers one 64-B request,
profiles/r04/calib_fetch.json, and moves at least that).  With a third pass
of TCC_HIT_sum / TCC_MISS_sum the L2 hit rate of each kernel's requests.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG N_SPANS OUT_JSON [TCC_DIR]
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
hit = per_launch(sys.argv[6], "TCC_HIT_sum") if len(sys.argv) > 6 else {}
miss = per_launch(sys.argv[6], "TCC_MISS_sum") if len(sys.argv) > 6 else {}
out = {"build": bench.build_id(), "config": int(sys.argv[3]), "n_spans": int(sys.argv[4]),
       "unit": "bytes per launch", "kernels": {}}
for k in sorted(set(fetch) | set(write)):
    f = 2 * 1024 * fetch.get(k, 0.0)
    w = 1024 * write.get(k, 0.0)
    out["kernels"][k] = {"fetch_bytes": round(f), "write_bytes": round(w), "traffic_bytes": round(f + w),
                         "traffic_lower_bytes": round(f / 2 + w)}
    if k in hit and k in miss and hit[k] + miss[k] > 0:
        out["kernels"][k]["l2_hit_rate"] = round(hit[k] / (hit[k] + miss[k]), 4)
json.dump(out, open(sys.argv[5], "w"), indent=1)
print(json.dumps(out, indent=1))
