#!/bin/bash
# A/B of the side-stream overlap (run on the box via gpurun): serial (KMZ_ABLATE
# bit 25), K3 on the side stream only (bit 26), K3 + certificate on the side
# stream (default), for the mesh, power and Bookinfo configs.
set -o pipefail
for cfg in mesh power bookinfo; do
  for v in 33554432 67108864 0; do
    KMZ_ABLATE=$v timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --cpu-seconds 0 --tail off > gpurun_out/ab_${cfg}_$v.json 2>gpurun_out/ab_${cfg}_$v.err || exit 1
  done
done
echo DONE
