#!/bin/bash
# fused-kernel threshold: parity tests of the fused path, the tick latency
# (fused / separate / graph / serial) and its kernel trace, the bench at
# 1e6 / 4e6 / 1e7 mesh spans fused vs separate.  usage: tools/r03_tick2.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-tick2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "fused or far or messy or chain_waits or spin or window_join or sig or graph" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_tick.py > $O/tick.json 2> $O/tick.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o tick -- python3 tools/bench_tick.py --ticks 50 > $O/tick_prof.json 2> $O/tick_prof.err || exit 1
for sp in 1e6 4e6 1e7; do for ab in 0 16; do
  KMZ_ABLATE2=$ab timeout -k 10 300 python -u bench.py --spans $sp --steps 20 --warmup 5 --cpu-seconds 0 --no-h2d > $O/mesh_${sp}_$ab.json 2> $O/mesh_${sp}_$ab.err || exit 1
done; done
echo TICK2_DONE
