#!/bin/bash
# rocprofv3 kernel stats of one bench config: tools/prof_stats.sh TAG CONFIG [extra bench args]
export TMPDIR=/tmp
TAG=${1:-r04}; CFG=${2:-mesh}; shift 2
mkdir -p gpurun_out/${TAG}_prof_${CFG}
if [ -n "$PROF_TESTS" ]; then  # parity tests first (e.g. PROF_TESTS=tests/test_tail.py)
  timeout -k 10 400 python -u -m pytest $PROF_TESTS -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_prof_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_prof_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_prof_tests.log
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_${CFG} -o run -- python3 bench.py --config $CFG --steps 5 --warmup 2 --cpu-seconds 0 --no-h2d "$@" > gpurun_out/${TAG}_prof_${CFG}.json 2> gpurun_out/${TAG}_prof_${CFG}.err || exit 1
f=$(find gpurun_out/${TAG}_prof_${CFG} -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print("%-60s %6s calls %9.3f ms avg %8.4f ms" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e6, float(r["AverageNs"]) / 1e6))
PY
