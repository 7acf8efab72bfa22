"""Which unit bounds each kernel: from tools/pmc_detail.sh output (csv), per
kernel the average duration, the effective clock (SQ_BUSY_CYCLES per shader
engine over the duration), the VALU issue share of every SIMD's cycles
(SQ_ACTIVE_INST_VALU is in quad-cycles summed over the waves; a SIMD issues
one wave64 VALU instruction per quad-cycle), the share of LDS cycles lost to
bank conflicts, and the wave-cycle split (waiting on memory / waiting to
issue / issuing).  usage: pmc_bound.py gpurun_out/pmcd_TAG [n_se] [n_simd]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
N_SE = int(sys.argv[2]) if len(sys.argv) > 2 else 32      # 8 XCDs x 4 shader engines
N_SIMD = int(sys.argv[3]) if len(sys.argv) > 3 else 1024  # 256 CUs x 4 SIMDs


def kname(s):
    return s.split("(")[0].replace("kmz::", "").replace("void ", "")


ctr = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
dur = collections.defaultdict(list)
for d in sorted(glob.glob(os.path.join(root, "*", ""))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ctr[kname(r["Kernel_Name"])][r["Counter_Name"]][(d, r["Dispatch_Id"])] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[kname(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)

rows = []
for k, d in ctr.items():
    v = {c: sum(x.values()) / len(x) for c, x in d.items()}
    if k not in dur or "SQ_BUSY_CYCLES" not in v or "SQ_ACTIVE_INST_VALU" not in v:
        continue
    t = sum(dur[k]) / len(dur[k])
    cyc = v["SQ_BUSY_CYCLES"] / N_SE
    valu = v["SQ_ACTIVE_INST_VALU"] * 4 / N_SIMD / cyc
    lds = v.get("SQ_LDS_BANK_CONFLICT", 0) / v["SQ_LDS_IDX_ACTIVE"] if v.get("SQ_LDS_IDX_ACTIVE") else 0.0
    wc = v["SQ_WAVE_CYCLES"]
    rows.append((t, k, cyc / t / 1e9, valu, v.get("SQ_INSTS_SALU", 0) / max(v["SQ_INSTS_VALU"], 1), lds,
                 v.get("SQ_WAIT_ANY", 0) / wc, v.get("SQ_WAIT_INST_ANY", 0) / wc, v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
print(f"{'kernel':34s} {'ms':>7s} {'GHz':>5s} {'VALU':>5s} {'S/V':>5s} {'LDSc':>5s} {'wait':>5s} {'winst':>5s} {'act':>5s}")
for t, k, ghz, valu, sv, lds, wa, wi, ac in sorted(rows, reverse=True):
    if t < 2e-5:
        continue
    print(f"{k[:34]:34s} {t * 1e3:7.3f} {ghz:5.2f} {valu:5.2f} {sv:5.2f} {lds:5.2f} {wa:5.2f} {wi:5.2f} {ac:5.2f}")
