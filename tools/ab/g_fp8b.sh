# the join's 8-bit-fingerprint hash, 51.5 KB LDS (base) against the 16-entry SWAR hash (old)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fp8b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fp8b/tests.log 2>&1 || { tail -40 gpurun_out/fp8b/tests.log; exit 1; }
tail -2 gpurun_out/fp8b/tests.log
bash tools/ab/ab_env.sh fp8b "--steps 20 --warmup 3" 2 fp8=base old=old || exit 1
python3 tools/ab/abread.py gpurun_out/ab_fp8b
timeout -k 10 200 python -u tools/diag_phase_join.py | grep debug_join
