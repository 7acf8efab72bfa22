#!/bin/bash
# Diagnostic GPU call (via gpurun): config 5 bench with progress on stderr,
# then SQ counter passes of the mesh bench (one rocprofv3 run per counter set).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
mkdir -p gpurun_out/diag_$TAG
if [ -n "$POWER" ]; then
  KMZ_BENCH_TRACE=1 timeout -k 10 240 python -u bench.py --config power --steps 5 --warmup 3 --cpu-seconds 0 \
    > gpurun_out/diag_$TAG/power.json 2> gpurun_out/diag_$TAG/power.err || exit 1
fi
KR="k4_chain|k_join_window|k3_produce|k3_reduce|k_cert_split|k_cert_check"
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$KR" --output-format csv -d gpurun_out/diag_$TAG/$name -o run -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --no-h2d > gpurun_out/diag_$TAG/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
echo DONE
