#!/bin/bash
# A/B of engine variants on one bench config; a variant is NAME=LIB[:ENV=VAL[:ENV=VAL]]
# (LIB "base" = libkmz.so, else kmamiz_amd/libkmz_LIB.so).
# usage: ab_env.sh TAG "BENCH ARGS" REPS v1 v2 ...
set -o pipefail
TAG=$1; ARGS=$2; REPS=$3; shift 3
mkdir -p gpurun_out/ab_$TAG
for rep in $(seq 1 $REPS); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}
    IFS=':' read -ra parts <<< "$rest"
    lib=${parts[0]}
    envs=()
    [ "$lib" != base ] && envs+=("KMZ_LIB_VARIANT=$lib")
    for e in "${parts[@]:1}"; do envs+=("$e"); done
    env "${envs[@]}" timeout -k 10 200 python bench.py $ARGS --cpu-seconds 0 > gpurun_out/ab_$TAG/${name}_$rep.json 2>>gpurun_out/ab_$TAG/err.log || exit 1
  done
done
echo AB_DONE
