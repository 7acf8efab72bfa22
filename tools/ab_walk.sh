#!/bin/bash
# A/B of K4 chain-walk variants on the mesh (config 3, 1e8 spans), two runs
# each: default build, runtime knobs (KMZ_ABLATE2) and variant builds
# (tools/variant.sh -> KMZ_LIB_VARIANT).  usage: tools/ab_walk.sh TAG "name:env ..."
# (AB_CONFIG=power|book|... picks another bench config)
export TMPDIR=/tmp
TAG=${1:-ab}; shift
O=gpurun_out/$TAG
mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for rep in 1 2; do
    env $envs timeout -k 10 240 python -u bench.py --config ${AB_CONFIG:-mesh} --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d > $O/${name}_$rep.json 2> $O/${name}_$rep.err || exit 1
    python3 -c "
import json;d=json.load(open('$O/${name}_$rep.json'));k=d['roofline']['kernels']
print('$name', $rep, d['ms_per_step'], {x: k[x]['ms_per_step'] for x in k if k[x]['ms_per_step'] > 0.04})"
  done
done
echo AB_DONE
