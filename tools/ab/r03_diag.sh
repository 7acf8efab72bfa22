#!/bin/bash
# diagnostics on the mesh at 1e8: k_join_window / k4_chain phase clocks, the
# k4_chain knob split, the K3 reduce balanced vs fixed slices (KMZ_ABLATE bit 14).
# usage: tools/r03_diag.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-diag}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u tools/diag_phase_join.py > $O/phase.txt 2>&1 || exit 1
b() {  # name, ablate, bench args...
  local name=$1 ab=$2; shift 2
  KMZ_ABLATE=$ab timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d "$@" \
    > $O/$name.json 2> $O/$name.err || exit 1
}
b mesh 0
b mesh_k3fixed 16384
b knob16 65536
b knob17 131072
b knob18 262144
echo DIAG_DONE
