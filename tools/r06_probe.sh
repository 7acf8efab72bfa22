#!/bin/bash
# Round-6 first probe on the box: (a) k4_tile8's VALU / SALU / LDS instructions
# per wave under the phase knobs (KMZ_ABLATE bit 16: window + row counts only;
# bit 17: + walk and sigs; bit 18: + probes, no inserts; 0: all), config 3 at
# 10^8 spans; (b) rocprofv3 kernel traces of the realtime tick (Bookinfo and
# mesh, direct and graphed); (c) tools/bench_tick.py.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06probe
mkdir -p $D
for a in 0 65536 131072 262144; do
  KMZ_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex "k4_tile8" --kernel-trace --output-format csv -d $D/knob_$a -o walk -- \
    python3 tools/ab/ablate.py child 3650000 > $D/knob_$a.log 2>&1 || exit 1
done
for c in bookinfo mesh; do
  for m in direct graph; do
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/tick_${c}_$m -o tick -- \
      python3 tools/tick_trace.py $c $m 60 > $D/tick_${c}_$m.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u tools/bench_tick.py > $D/tick.json 2> $D/tick.err || exit 1
echo PROBE_DONE
