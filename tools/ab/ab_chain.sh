#!/bin/bash
# A/B of engine builds on the mesh bench (run on the box via gpurun).
# usage: tools/ab_chain.sh VARIANT... ("base" = kmamiz_amd/libkmz.so; others
# are tools/variant.sh builds); prints step / walk / join / K3 ms per variant
export TMPDIR=/tmp
ARGS=${AB_ARGS:---steps 20 --warmup 3}
for v in "$@"; do
  [ "$v" = base ] && vv="" || vv=$v
  KMZ_LIB_VARIANT=$vv timeout -k 10 120 python bench.py $ARGS --cpu-seconds 0 --no-h2d > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || { echo "$v failed"; exit 1; }
  python -c "
import json;d=json.load(open('gpurun_out/ab_$v.json'));k=d['roofline']['kernels'];print('$v', d['ms_per_step'], {x: k[x]['ms_per_step'] for x in k if k[x]['ms_per_step'] > 0.05})"
done
