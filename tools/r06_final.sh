#!/bin/bash
# End-of-round set, round 6 (on the box via gpurun), in two calls:
#   tools/r06_final.sh TAG 1   GPU suite, smoke(), rocprofv3 stats + stamped PMC traffic + the default bench line
#   tools/r06_final.sh TAG 2   configs 2 and 5, tick latency, 2-rank rehearsal, 10^9 spans, guard cost
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r06f}
PART=${2:-1}
mkdir -p gpurun_out/$TAG
if [ "$PART" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
  tail -2 gpurun_out/$TAG/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
  tail -1 gpurun_out/$TAG/smoke.log
  bash tools/r05_measure.sh $TAG || exit 1
else
  bash tools/r05_measure2.sh $TAG || exit 1
fi
echo "PART${PART}_DONE"
