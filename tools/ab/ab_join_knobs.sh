#!/bin/bash
# k_join_window cost split by diagnostic knobs (KMZ_ABLATE bits: 256 no window
# insert, 512 no parent lookup, 64 no certificate pass 1); results are wrong
# under the knobs, only the kernel times matter
export TMPDIR=/tmp
for k in 0 256 512 64 $((256|512)) $((256|512|64)); do
  KMZ_ABLATE=$k timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-h2d "$@" > gpurun_out/jknob_$k.json 2>gpurun_out/jknob_$k.err || { echo "knob $k failed"; tail -2 gpurun_out/jknob_$k.err; continue; }
  python -c "
import json;d=json.load(open('gpurun_out/jknob_$k.json'));k=d['roofline']['kernels'];print('knob $k', {x: k[x]['ms_per_step'] for x in ('join','walk') if x in k})"
done
