# k_join_window's halo: 128 (base) against 256 (h256), mesh and config 5
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/halo
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/halo/tests.log 2>&1 || { tail -40 gpurun_out/halo/tests.log; exit 1; }
tail -2 gpurun_out/halo/tests.log
bash tools/ab/ab_env.sh halo "--steps 20 --warmup 3 --no-h2d" 2 h128=base h256=h256 || exit 1
bash tools/ab/ab_env.sh halop "--config power --steps 10 --warmup 3 --no-h2d" 2 h128=base h256=h256 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_halo
python3 tools/ab/abread.py gpurun_out/ab_halop
