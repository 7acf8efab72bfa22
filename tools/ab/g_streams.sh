# the certificate on the idle side stream, no fifth stream (base) against HEAD (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/streams
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/streams/tests.log 2>&1 || { tail -40 gpurun_out/streams/tests.log; exit 1; }
tail -2 gpurun_out/streams/tests.log
bash tools/ab/ab_env.sh strb "--config bookinfo --steps 200 --warmup 50 --no-h2d" 2 new=base old=old || exit 1
bash tools/ab/ab_env.sh strm "--steps 20 --warmup 3 --no-h2d" 2 new=base old=old || exit 1
bash tools/ab/ab_env.sh strp "--config power --steps 10 --warmup 3 --no-h2d" 1 new=base old=old || exit 1
for d in strb strm strp; do python3 tools/ab/abread.py gpurun_out/ab_$d; done
