#!/bin/bash
# Per-kernel SQ / TCC counters of the mesh bench on the current build (one
# counter set per rocprofv3 pass), summarised to gpurun_out/ctr_TAG.json.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
D=gpurun_out/ctr_$TAG
mkdir -p $D
KR="k4_tile|k3_reduce_bal|k3_produce|k_cert_split|k_cert_check|k_join_window"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/$name -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-h2d > $D/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
python3 - "$D" "$TAG" <<'P'
import collections, csv, glob, json, os, sys
root, tag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("kmz::", "").replace("void ", "")
        acc[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
out = {"tag": tag, "workload": "config 3 mesh 1e8 spans, bench.py --steps 2 --warmup 1", "unit": "per dispatch (mean)",
       "kernels": {k: {c: round(sum(v.values()) / len(v), 1) for c, v in d.items()} for k, d in acc.items()}}
for k, d in out["kernels"].items():
    if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
        d["wait_any_frac"] = round(d.get("SQ_WAIT_ANY", 0) / d["SQ_WAVE_CYCLES"], 3)
    if "SQ_BUSY_CYCLES" in d and d.get("SQ_ACTIVE_INST_VALU"):
        pass
    if d.get("SQ_LDS_IDX_ACTIVE"):
        d["lds_conflict_frac"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0) / d["SQ_LDS_IDX_ACTIVE"], 3)
json.dump(out, open(f"gpurun_out/ctr_{tag}.json", "w"), indent=1)
print(json.dumps({k: {c: d.get(c) for c in ("wait_any_frac", "lds_conflict_frac", "SQ_INSTS_VALU", "SQ_WAVES")} for k, d in out["kernels"].items()}))
P
echo CTR_DONE
