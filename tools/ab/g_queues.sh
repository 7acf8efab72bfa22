# bench_guard with HIP's default 4 hardware queues and with 8
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/q1
timeout -k 10 400 python -u tools/bench_guard.py > gpurun_out/q1/q4.json 2> gpurun_out/q1/q4.err || exit 1
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u tools/bench_guard.py > gpurun_out/q1/q8.json 2> gpurun_out/q1/q8.err || exit 1
python3 - <<'P'
import json
for q in ("q4", "q8"):
    d = json.load(open(f"gpurun_out/q1/{q}.json"))
    for w, x in d["worlds"].items():
        print(q, w, "step", x["step_ms"], "nocert", x["step_nocert_ms"], "cert", x["seg_certificate_ms"], "guarded", x["guarded_step_ms"])
P
