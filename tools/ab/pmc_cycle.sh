#!/bin/bash
# PMC passes over the mesh bench (run on the box via gpurun): one counter set
# per rocprofv3 invocation, kernel trace only (no runtime/sys traces).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-x}
STEPS=${2:-2}
run() {  # name, counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/$name -o mesh -- \
    python3 bench.py --steps $STEPS --warmup 1 --cpu-seconds 0 > gpurun_out/pmc_${TAG}_$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS || exit 1
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 1
echo DONE
