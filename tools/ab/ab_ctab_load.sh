set -o pipefail
mkdir -p gpurun_out/ab1
for v in 0 4 8 0 4; do
  KMZ_ABLATE2=$v timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/ab1/mesh_$v.$RANDOM.json 2>>gpurun_out/ab1/err.log || exit 1
done
echo AB_DONE
