# Bookinfo: HIP's 4 hardware queues against 8 (stream-to-queue sharing)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh bookq "--config bookinfo --steps 200 --warmup 50 --no-h2d" 2 q4=base q8=base:GPU_MAX_HW_QUEUES=8 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_bookq
