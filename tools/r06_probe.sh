#!/bin/bash
# Round-6 GPU cycle: (1) the GPU suite (messy batches deselected); (2) mesh
# bench A/B, k4_tile9 (default, 7 workgroups per CU), the 8-per-CU build
# (libkmz_t9w8.so) and k4_tile8 (KMZ_ABLATE2 bit 22); config 5 once each;
# (3) the walk's instruction counters per wave under the phase knobs (KMZ_ABLATE
# bit 16: window + row counts only; bit 17: + walk and sigs; 0: all), config 3
# at 10^8 spans; (4) rocprofv3 kernel traces of the realtime tick (Bookinfo and
# mesh, graphed and direct) and tools/bench_tick.py.
# usage: tools/r06_probe.sh [skip-tests]
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06probe
mkdir -p $D
if [ "$1" != skip-tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    --deselect tests/test_gpu_parity.py::test_messy_batches_vs_oracle > $D/tests.log 2>&1
  rc=$?
  tail -3 $D/tests.log
  [ $rc -eq 0 ] || exit 1
fi
bash tools/ab/ab_env.sh w9 "--steps 10 --warmup 3" 2 t9=base t9w8=t9w8 t8=base:KMZ_ABLATE2=4194304 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_w9
bash tools/ab/ab_env.sh w9p "--config power --steps 10 --warmup 3" 1 t9=base t8=base:KMZ_ABLATE2=4194304 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_w9p
bash tools/ab/ab_env.sh w9b "--config bookinfo --steps 200 --warmup 50" 2 graph=base direct=base:KMZ_HIPGRAPH=0 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_w9b
for v in 0; do
  for a in 0 65536 131072; do
    KMZ_ABLATE=$a KMZ_ABLATE2=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      --kernel-include-regex "k4_tile" --kernel-trace --output-format csv -d $D/knobB_${v}_$a -o walk -- \
      python3 tools/ab/ablate.py child 3650000 > $D/knobB_${v}_$a.log 2>&1 || exit 1
  done
done
for c in bookinfo mesh; do
  for m in direct graph; do
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/tick_${c}_$m -o tick -- \
      python3 tools/tick_trace.py $c $m 60 > $D/tick_${c}_$m.log 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u tools/bench_tick.py > $D/tick.json 2> $D/tick.err || exit 1
echo PROBE_DONE
