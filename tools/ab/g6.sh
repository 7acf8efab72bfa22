set -o pipefail
tools/ab/ab_env.sh w8g "--steps 10 --warmup 3" 2 old=base:KMZ_ABLATE2=1024 w8g=base:KMZ_ABLATE2=2048 w7g=w7:KMZ_ABLATE2=2048 w6g=w6:KMZ_ABLATE2=2048 w7=w7
