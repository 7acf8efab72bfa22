# config 5: k_key_part's LDS key cache (default) against none (KMZ_ABLATE2 bit 16)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/kc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_deprecation.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kc/tests.log 2>&1 || { tail -40 gpurun_out/kc/tests.log; exit 1; }
tail -2 gpurun_out/kc/tests.log
bash tools/ab/ab_env.sh kc "--config power --steps 20 --warmup 3" 2 kc=base none=base:KMZ_ABLATE2=65536 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_kc
