# CU-masked certificate split beside the walk (KMZ_CERT_CUS) against the default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cus
KMZ_CERT_CUS=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cus/tests.log 2>&1 || { tail -30 gpurun_out/cus/tests.log; exit 1; }
tail -2 gpurun_out/cus/tests.log
bash tools/ab/ab_env.sh cus "--steps 20 --warmup 3" 2 base=base c32=base:KMZ_CERT_CUS=32 c64=base:KMZ_CERT_CUS=64 c16=base:KMZ_CERT_CUS=16 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_cus
