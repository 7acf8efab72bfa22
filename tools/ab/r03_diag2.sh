#!/bin/bash
# Bookinfo 1e6 with a long timed region (200 steps, twice), the mesh phase
# clocks of k_join_window / k4_chain, and the fused kernel's phases at 4e6
# mesh spans.  usage: tools/r03_diag2.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-diag2}
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 --cpu-seconds 0 --no-h2d > $O/book_$rep.json 2> $O/book_$rep.err || exit 1
done
timeout -k 10 300 python -u tools/diag_phase_join.py > $O/phase_mesh.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/diag_fuse.py 146000 > $O/phase_fused_4e6.txt 2>&1 || exit 1
echo DIAG2_DONE
