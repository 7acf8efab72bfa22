# the join's 8-bit-fingerprint window hash (base) against the 16-entry SWAR one (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fp8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fp8/tests.log 2>&1 || { tail -40 gpurun_out/fp8/tests.log; exit 1; }
tail -2 gpurun_out/fp8/tests.log
bash tools/ab/ab_env.sh fp8 "--steps 20 --warmup 3" 2 fp8=base old=old || exit 1
bash tools/ab/ab_env.sh fp8p "--config power --steps 20 --warmup 3" 1 fp8=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_fp8
python3 tools/ab/abread.py gpurun_out/ab_fp8p
