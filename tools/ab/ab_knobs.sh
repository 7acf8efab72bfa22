#!/bin/bash
# k4_chain cost split by diagnostic knobs (KMZ_ABLATE bits: 16 no walk/probe,
# 17 hash only, 18 probe without inserts); results are wrong under the knobs,
# only the kernel times matter.  usage: tools/ab_knobs.sh [bench args]
export TMPDIR=/tmp
for k in 0 $((1<<16)) $((1<<17)) $((1<<18)); do
  KMZ_ABLATE=$k timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-h2d "$@" > gpurun_out/knob_$k.json 2>gpurun_out/knob_$k.err || { echo "knob $k failed"; tail -3 gpurun_out/knob_$k.err; continue; }
  python -c "
import json;d=json.load(open('gpurun_out/knob_$k.json'));k=d['roofline']['kernels'];print('knob $k', d['ms_per_step'], {x: k[x]['ms_per_step'] for x in ('walk','settle','join')})"
done
