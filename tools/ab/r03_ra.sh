#!/bin/bash
# Parity of the atomic-rank certificate pass-1 variant (libkmz_ra.so) on the
# GPU parity tests, then the mesh A/B against the default build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ra
KMZ_LIB_VARIANT=ra timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ra/tests.txt 2>&1 || { tail -30 gpurun_out/ra/tests.txt; exit 1; }
tail -3 gpurun_out/ra/tests.txt
bash tools/r03_var.sh ra_ab - ra
