#!/bin/bash
# A/B of engine variants (tools/variant.sh builds) on one bench config.
# usage: ab_variants.sh TAG "ARGS" v1 v2 ... ("base" = libkmz.so)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/ab_$TAG
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = base ]; then unset KMZ_LIB_VARIANT; else export KMZ_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py $ARGS --cpu-seconds 0 > gpurun_out/ab_$TAG/${v}_$rep.json 2>>gpurun_out/ab_$TAG/err.log || exit 1
  done
done
echo AB_DONE
