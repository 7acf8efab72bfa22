#!/bin/bash
# A/B of engine build variants (tools/variant.sh) on the mesh bench, plus the
# default build with the side stream forced on (KMZ_ABLATE bit 27: K3 beside
# the join, the certificate beside the walk).
# usage: tools/r03_var.sh TAG VARIANT...   ("-" = the default libkmz.so)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = "-" ]; then unset KMZ_LIB_VARIANT; else export KMZ_LIB_VARIANT=$v; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_${v}_$rep.json 2> $O/mesh_${v}_$rep.err || exit 1
done
unset KMZ_LIB_VARIANT
KMZ_ABLATE=134217728 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/mesh_overlap_$rep.json 2> $O/mesh_overlap_$rep.err || exit 1
done
echo VAR_DONE
