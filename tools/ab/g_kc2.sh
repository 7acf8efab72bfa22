# config 5: k_key_part's key cache size 1024 / 2048 (default) / 4096
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh kc2 "--config power --steps 20 --warmup 3" 2 kc2048=base kc4096=kc4 kc1024=kc1 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_kc2
