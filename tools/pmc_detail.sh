#!/bin/bash
# Per-kernel PMC passes over one bench config (run on the box via gpurun):
# one counter set per rocprofv3 invocation (the per-block slot limits of
# MI355X_MICROARCH.md), kernel trace only.  usage: pmc_detail.sh TAG [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
shift
ARGS=${*:---steps 2 --warmup 1}
mkdir -p gpurun_out/pmcd_$TAG
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcd_$TAG/counters.txt 2>&1 || true
run() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmcd_$TAG/$name -o run -- \
    python3 bench.py $ARGS --cpu-seconds 0 > gpurun_out/pmcd_$TAG/$name.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run sq2 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
run tcc TCC_HIT_sum TCC_MISS_sum || exit 1
echo DONE
