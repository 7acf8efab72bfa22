#!/bin/bash
# balanced K3 reduce + device service sums: tests, then A/B bench lines
# (config 5 and the mesh, default vs KMZ_ABLATE bit 14 = fixed slices) and
# the tail's diagnostic knobs (bit 7: no link keys, bit 12: no pairs).
# usage: tools/r03_k3.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-k3}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -m gpu \
  tests/test_tail.py "tests/test_gpu_parity.py::test_k3_reduce_variants_equal" \
  "tests/test_gpu_parity.py::test_synthetic_vs_c_oracle" "tests/test_gpu_parity.py::test_compact_key_staging_equals_wide_keys" \
  "tests/test_gpu_parity.py::test_compact_staging_with_distances_past_32" "tests/test_gpu_parity.py::test_key_staging_paths_equal" \
  > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
b() {  # name, ablate, bench args...  (KMZ_ABLATE2 from the environment)
  local name=$1 ab=$2; shift 2
  KMZ_ABLATE=$ab timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d "$@" \
    > $O/$name.json 2> $O/$name.err || exit 1
}
b power 0 --config power
b power_fixed 16384 --config power
KMZ_ABLATE2=1 b power_wide 0 --config power
b mesh 0
b mesh_fixed 16384
KMZ_ABLATE2=4 b mesh_lf2 0
KMZ_ABLATE2=8 b mesh_lf4 0
b power_nolinks 128 --config power
b power_nopairs 4096 --config power
echo K3_DONE
