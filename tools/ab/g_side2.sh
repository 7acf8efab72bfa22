# the certificate on a stream of its own (default) against behind K3 (KMZ_ABLATE2 bit 14)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/s2/tests.log 2>&1 || { tail -40 gpurun_out/s2/tests.log; exit 1; }
tail -2 gpurun_out/s2/tests.log
bash tools/ab/ab_env.sh side2 "--steps 20 --warmup 3" 3 side2=base side=base:KMZ_ABLATE2=16384 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_side2
