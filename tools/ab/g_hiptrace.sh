# HIP API trace of a few mesh steps (host calls between a run's first memset and its first kernel)
set -o pipefail
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/ht -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/ht.log 2>&1 || exit 1
ls gpurun_out/ht/
