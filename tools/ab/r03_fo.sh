#!/bin/bash
# Fused join + walk with certificate pass-1 ranks from LDS atomics (default
# build) against wave ballots (libkmz_fo.so): the fused-kernel parity tests,
# then Bookinfo 1e6 and the mesh at 4e6 spans, two runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fo
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fused or wide or headline or cert" --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2; do
for v in - fo; do
  if [ "$v" = "-" ]; then unset KMZ_LIB_VARIANT; else export KMZ_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u bench.py --config bookinfo --steps 200 --warmup 50 --cpu-seconds 0 --no-h2d > $O/book_${v}_$rep.json 2> $O/book_${v}_$rep.err || exit 1
  timeout -k 10 300 python -u bench.py --spans 4e6 --steps 50 --warmup 10 --cpu-seconds 0 --no-h2d > $O/mesh4M_${v}_$rep.json 2> $O/mesh4M_${v}_$rep.err || exit 1
done
done
echo FO_DONE
