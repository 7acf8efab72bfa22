set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t_parity7.log 2>&1 || exit 1
tools/ab/ab_env.sh s7 "--steps 10 --warmup 3" 2 old=base:KMZ_ABLATE2=1024 s7=base s8=s8 s6=s6 g7=base:KMZ_ABLATE2=2048
