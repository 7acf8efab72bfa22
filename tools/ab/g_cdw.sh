# config 5: the certificate beside the direct walk (KMZ_ABLATE2 bit 22) against on the main stream before it
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cdw
KMZ_ABLATE2=4194304 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "synthetic_vs_c_oracle or headline_config5 or direct_enumeration_vs" --timeout 120 --timeout-method thread > gpurun_out/cdw/tests.log 2>&1 || { tail -40 gpurun_out/cdw/tests.log; exit 1; }
tail -1 gpurun_out/cdw/tests.log
bash tools/ab/ab_env.sh cdw "--config power --steps 20 --warmup 3 --no-h2d" 3 new=base:KMZ_ABLATE2=4194304 old=base || exit 1
python3 tools/ab/abread.py gpurun_out/ab_cdw
