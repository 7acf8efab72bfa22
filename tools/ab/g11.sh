set -o pipefail
export TMPDIR=/tmp
tools/ab/ab_env.sh k11 "--steps 10 --warmup 3" 1 base=base nohash=base:KMZ_ABLATE=65536 hashonly=base:KMZ_ABLATE=131072 || exit 1
D=gpurun_out/pmc11; mkdir -p $D
KR="k4_tile8|k_join_window|k3_reduce_bal|k3_produce|k_cert_split|k_cert_check"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/sq1 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $D/sq1.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-include-regex "$KR" --kernel-trace --output-format csv -d $D/sq2 -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 > $D/sq2.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl11 -o tl -- python3 bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/tl11.log 2>&1 || exit 1
echo G11_TL_DONE
