# K3 beside config 5's settle (KMZ_ABLATE2 bit 21) against beside the join: parity with the knob, then A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/k3s
KMZ_ABLATE2=2097152 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "synthetic_vs_c_oracle or headline_config5 or k3_reduce_variants or direct_enumeration_vs" --timeout 120 --timeout-method thread > gpurun_out/k3s/tests.log 2>&1 || { tail -40 gpurun_out/k3s/tests.log; exit 1; }
tail -1 gpurun_out/k3s/tests.log
bash tools/ab/ab_env.sh k3s "--config power --steps 20 --warmup 3 --no-h2d" 3 new=base:KMZ_ABLATE2=2097152 old=base || exit 1
python3 tools/ab/abread.py gpurun_out/ab_k3s
