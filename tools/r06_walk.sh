#!/bin/bash
# Round-6 walk cycle: the walk's parity tests (k4_tile9 against k4_tile8 and
# the C oracle, every chain-interning test, the deprecation and cache tests),
# then the mesh A/B k4_tile9 / k4_tile8, and the walk's counters per wave under
# the phase knobs.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r06walk
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_deprecation.py tests/test_gpu_cache.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_parity.py::test_messy_batches_vs_oracle \
  -k "tile9 or synthetic or chain or sig_collision or spin or deep or gather or graph or headline or full_size or filter or cache or entries or reduced or fixture or far or mock" > $D/tests.log 2>&1
rc=$?
tail -2 $D/tests.log
[ $rc -eq 0 ] || exit 1
bash tools/ab/ab_env.sh ${1:-w9r} "--steps 10 --warmup 3" 2 t9=base t8=base:KMZ_ABLATE2=4194304 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_${1:-w9r}
for a in 0 131072; do
  KMZ_ABLATE=$a timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex "k4_tile" --kernel-trace --output-format csv -d $D/knob_$a -o walk -- \
    python3 tools/ab/ablate.py child 3650000 > $D/knob_$a.log 2>&1 || exit 1
done
echo WALK_DONE
