# certificate pass 1 with 2^8 bins at 10^8 (KMZ_ABLATE2 bit 6) against 2^6; with K3 after the walk (bit 18)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab/ab_env.sh wide "--steps 20 --warmup 3" 2 b6=base b8=base:KMZ_ABLATE2=64 late=base:KMZ_ABLATE2=262144 lateb8=base:KMZ_ABLATE2=262208 || exit 1
python3 tools/ab/abread.py gpurun_out/ab_wide
