# config 5: the certificate deferred beside the settle with K3 (KMZ_ABLATE2 bit 15) against on the main stream before it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cdf
KMZ_ABLATE2=32768 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "synthetic_vs_c_oracle or headline_config5 or direct_enumeration_vs" --timeout 120 --timeout-method thread > gpurun_out/cdf/tests.log 2>&1 || { tail -40 gpurun_out/cdf/tests.log; exit 1; }
tail -1 gpurun_out/cdf/tests.log
bash tools/ab/ab_env.sh cdf "--config power --steps 20 --warmup 3 --no-h2d" 3 new=base:KMZ_ABLATE2=32768 old=base || exit 1
python3 tools/ab/abread.py gpurun_out/ab_cdf
