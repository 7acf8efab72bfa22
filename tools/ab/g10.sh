set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t_parity10.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_guard.py tests/test_dist_engine.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu > gpurun_out/t_guard10.log 2>&1 || exit 1
tools/ab/ab_env.sh s10 "--steps 10 --warmup 3" 2 old=base:KMZ_ABLATE2=1024 new=base s8=s8 k3s=k3s k3r512=k3r512 fused=base:KMZ_ABLATE2=32 || exit 1
tools/ab/ab_env.sh k10 "--steps 10 --warmup 3" 1 nohash=base:KMZ_ABLATE=65536 hashonly=base:KMZ_ABLATE=131072 || exit 1
D=gpurun_out/pmc10; mkdir -p $D
KR="k4_tile8|k_join_window|k3_reduce_bal"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/sq1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $D/sq1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $D/sq2.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_guard.py > gpurun_out/guard_cost10.json 2> gpurun_out/guard_cost10.err || exit 1
echo G10_DONE
