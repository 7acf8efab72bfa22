#!/bin/bash
# One parameterised GPU A/B (replaces round 5's one-shot tools/ab/g_*.sh
# launchers): optionally a GPU test selection first (under the variant's env),
# then tools/ab/ab_env.sh over one or more bench configs, summarised by
# tools/ab/abread.py.
#
# usage: tools/ab/gab.sh TAG REPS "TESTS" "VARIANTS" "BENCH ARGS" ["BENCH ARGS" ...]
#   TESTS     pytest arguments ("-" for none), e.g.
#             "tests/test_gpu_parity.py -k synthetic_vs_c_oracle"; run once per
#             variant whose spec sets env (NAME=LIB:ENV=VAL...), once plain otherwise
#   VARIANTS  ab_env.sh specs, e.g. "new=base old=base:KMZ_ABLATE2=4194304"
#   each BENCH ARGS is one bench.py configuration ("--config power --steps 20 --warmup 3")
# e.g. round 5's g_k3walk.sh:
#   tools/ab/gab.sh k3walk 2 "tests/test_gpu_parity.py -k 'power or config5 or direct or tail'" \
#       "join=base walk=base:KMZ_ABLATE2=524288" "--config power --steps 20 --warmup 3"
set -o pipefail
export TMPDIR=/tmp
TAG=$1; REPS=$2; TESTS=$3; VARIANTS=$4; shift 4
D=gpurun_out/$TAG
mkdir -p $D
if [ "$TESTS" != "-" ]; then
  for spec in $VARIANTS; do
    rest=${spec#*=}
    IFS=':' read -ra parts <<< "$rest"
    envs=()
    [ "${parts[0]}" != base ] && envs+=("KMZ_LIB_VARIANT=${parts[0]}")
    for e in "${parts[@]:1}"; do envs+=("$e"); done
    eval env "${envs[@]}" timeout -k 10 900 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider $TESTS > $D/tests_${spec%%=*}.log 2>&1 || { tail -40 $D/tests_${spec%%=*}.log; exit 1; }
    tail -1 $D/tests_${spec%%=*}.log
  done
fi
k=0
for args in "$@"; do
  k=$((k + 1))
  bash tools/ab/ab_env.sh ${TAG}_$k "$args" $REPS $VARIANTS || exit 1
  python3 tools/ab/abread.py gpurun_out/ab_${TAG}_$k
done
echo GAB_DONE
