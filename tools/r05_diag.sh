#!/bin/bash
# Round-5 diagnostics on the box (via gpurun): the probe-rate calibration,
# then per-kernel PMC passes of the mesh bench (one counter set per pass).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
D=gpurun_out/diag_$TAG
mkdir -p $D
timeout -k 10 120 ./tools/calib/calib_probe > $D/calib_probe.json 2> $D/calib_probe.err || exit 1
timeout -s KILL 60 rocprofv3 -L > $D/counters.txt 2>&1 || true
KR="k4_tile|k3_reduce_bal|k3_produce|k_cert_split|k_cert_check|k_join_window"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/$name -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $D/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
run ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum || echo "ea pass failed" >> $D/notes.txt
echo DIAG_DONE
