#!/bin/bash
# fused join + chain walk: every GPU test (the fused kernel is the default
# chain-interning path), then A/B bench lines: fused vs the two kernels
# (KMZ_ABLATE2 bit 4) on the mesh, Bookinfo and config 5, and the phase split.
# usage: tools/r03_fuse.sh TAG [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-fuse}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then K=(-k "$2"); else K=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread "${K[@]}" > $O/tests.log 2>&1
rc=$?; echo "tests exit $rc" >> $O/tests.log; [ $rc -eq 0 ] || exit 1
[ -n "$NOBENCH" ] && exit 0
b() {  # name, ablate2, bench args...
  local name=$1 ab=$2; shift 2
  KMZ_ABLATE2=$ab timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-h2d "$@" \
    > $O/$name.json 2> $O/$name.err || exit 1
}
b mesh 0
b mesh_sep 16
b book 0 --config bookinfo --steps 20 --warmup 5
b book_sep 16 --config bookinfo --steps 20 --warmup 5
b power 0 --config power
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o mesh -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d > $O/prof.log 2>&1 || exit 1
echo FUSE_DONE
