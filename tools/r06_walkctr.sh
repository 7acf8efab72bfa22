#!/bin/bash
# Walk counters of two builds side by side (KMZ_LIB_VARIANT values, "base" =
# libkmz.so): instruction mix, waits, L2 traffic of k4_tile9, config 3 at 10^8.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06walkctr
mkdir -p $D
for v in "$@"; do
  if [ $v = base ]; then unset KMZ_LIB_VARIANT; else export KMZ_LIB_VARIANT=$v; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_LDS \
    --kernel-include-regex "k4_tile" --kernel-trace --output-format csv -d $D/${v}_sq -o walk -- \
    python3 tools/ab/ablate.py child 3650000 > $D/${v}_sq.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum \
    --kernel-include-regex "k4_tile" --kernel-trace --output-format csv -d $D/${v}_tcc -o walk -- \
    python3 tools/ab/ablate.py child 3650000 > $D/${v}_tcc.log 2>&1 || exit 1
done
python3 - "$D" <<'P'
import csv, glob, collections, sys
root = sys.argv[1]
for d in sorted(glob.glob(root + "/*_sq")) + sorted(glob.glob(root + "/*_tcc")):
    acc = collections.defaultdict(float); disp = set()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    nd = max(1, len(disp))
    print(d.split("/")[-1], {k: round(v / nd) for k, v in sorted(acc.items())})
P
echo CTR_DONE
