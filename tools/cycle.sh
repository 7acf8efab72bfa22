#!/bin/bash
# One build-measure cycle on the box (via gpurun): GPU tests (messy batches
# deselected unless FULL=1), the mesh bench, optional extra benches.
# usage: tools/cycle.sh TAG [extra bench args for a second line...]
export TMPDIR=/tmp
TAG=${1:-x}
DES="--deselect tests/test_gpu_parity.py::test_messy_batches_vs_oracle"
[ -n "$FULL" ] && DES=""
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider $DES > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
if [ -n "$BOOK" ]; then
  timeout -k 10 200 python bench.py --config bookinfo --steps 20 --warmup 5 --cpu-seconds 0 > gpurun_out/${TAG}_book.json 2> gpurun_out/${TAG}_book.err || exit 1
fi
if [ -n "$POWER" ]; then
  timeout -k 10 300 python bench.py --config power --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/${TAG}_power.json 2> gpurun_out/${TAG}_power.err || exit 1
fi
if [ -n "$DIAG" ]; then
  timeout -k 10 300 python tools/diag_phase_join.py > gpurun_out/${TAG}_diag.txt 2>&1 || exit 1
fi
echo CYCLE_DONE
