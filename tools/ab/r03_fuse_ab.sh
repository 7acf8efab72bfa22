#!/bin/bash
# quick fused-kernel iteration: its parity tests, the mesh bench fused vs
# separate, the phase split.  usage: tools/r03_fuse_ab.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-fab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
  -k "fused or far or messy_batches_vs or chain_waits or spin or window_join or sig" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
for ab in 0 16; do
  KMZ_ABLATE2=$ab timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_$ab.json 2> $O/mesh_$ab.err || exit 1
done
timeout -k 10 300 python -u tools/diag_fuse.py > $O/diag.txt 2>&1 || exit 1
echo FAB_DONE
