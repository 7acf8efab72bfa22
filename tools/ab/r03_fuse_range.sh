#!/bin/bash
# Is the fused join + walk still the faster form at the edges of its range
# (2^19..2^23 spans) after the pass-1 rank change?  Fused vs separate
# (KMZ_ABLATE2 bit 4: never fused; bit 5: fused at any size), two runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fuse_range
mkdir -p $O
for rep in 1 2; do
  for sp in 6e5 4e6 8e6; do
    timeout -k 10 300 python -u bench.py --spans $sp --steps 50 --warmup 10 --cpu-seconds 0 --no-h2d > $O/mesh${sp}_fused_$rep.json 2> $O/e.err || exit 1
    KMZ_ABLATE2=16 timeout -k 10 300 python -u bench.py --spans $sp --steps 50 --warmup 10 --cpu-seconds 0 --no-h2d > $O/mesh${sp}_sep_$rep.json 2> $O/e.err || exit 1
  done
  for sp in 1.2e7 2e7; do
    timeout -k 10 300 python -u bench.py --spans $sp --steps 20 --warmup 5 --cpu-seconds 0 --no-h2d > $O/mesh${sp}_sep_$rep.json 2> $O/e.err || exit 1
    KMZ_ABLATE2=32 timeout -k 10 300 python -u bench.py --spans $sp --steps 20 --warmup 5 --cpu-seconds 0 --no-h2d > $O/mesh${sp}_fused_$rep.json 2> $O/e.err || exit 1
  done
done
echo RANGE_DONE
