export TMPDIR=/tmp
for a in 0 64 256 832 65536 131072 262144; do
  KMZ_ABLATE=$a timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/abl_$a.json 2> gpurun_out/abl_$a.err || exit 1
done
