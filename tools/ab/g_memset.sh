# the run's counters zeroed by k_fill (base) against hipMemsetAsync (bit 20); HIP trace of the new build
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh memset "--steps 20 --warmup 3 --no-h2d" 2 kfill=base blit=base:KMZ_ABLATE2=1048576 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_memset
timeout -s KILL 200 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/ht2 -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-h2d > gpurun_out/ht2.log 2>&1 || exit 1
