#!/bin/bash
# End-of-round check on the box: the GPU suite, smoke(), then both measurement parts.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-fin}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$TAG/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
bash tools/r05_measure.sh $TAG || exit 1
bash tools/r05_measure2.sh $TAG || exit 1
echo FINAL_DONE
