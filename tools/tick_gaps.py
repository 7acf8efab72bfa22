"""Summarise a rocprofv3 kernel trace of tools/tick_trace.py: per realtime
tick (one kmz_load + kmz_run + kmz_fetch), the kernels launched, their summed
time, the span from the tick's first kernel start to its last kernel end, and
the idle gaps in between (median over the ticks after the first ten).

    python tools/tick_gaps.py gpurun_out/r06probe/tick_mesh_direct
"""
import csv
import glob
import os
import statistics
import sys


def ticks(path):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    # a tick starts with kmz_load's copies (the runtime's copy kernels) after
    # the previous tick's run kernels; the fetch's copies end a tick
    out, cur = [], []
    for s, e, k in rows:
        if cur and "copyBuffer" in k and "copyBuffer" not in cur[-1][2] and any("copyBuffer" in x[2] for x in cur[-3:]) is False \
                and len(cur) > 8:
            out.append(cur)
            cur = []
        cur.append((s, e, k))
    if cur:
        out.append(cur)
    return out


def main():
    for path in sys.argv[1:]:
        ts = ticks(path)[10:]
        if not ts:
            print(path, "no ticks")
            continue
        n = [len(t) for t in ts]
        busy = [sum(e - s for s, e, _ in t) / 1000 for t in ts]
        span = [(t[-1][1] - t[0][0]) / 1000 for t in ts]
        gaps = [sum(max(0, t[i + 1][0] - t[i][1]) for i in range(len(t) - 1)) / 1000 for t in ts]
        med = statistics.median
        print(f"{os.path.basename(path.rstrip('/'))}: {len(ts)} ticks, kernels/tick {med(n)}, "
              f"kernel us {med(busy):.1f}, first->last us {med(span):.1f}, gaps us {med(gaps):.1f}")
        t = ts[len(ts) // 2]
        names = {}
        for s, e, k in t:
            names.setdefault(k, []).append((e - s) / 1000)
        for k, v in sorted(names.items(), key=lambda x: -sum(x[1])):
            print(f"   {sum(v):7.1f} us  x{len(v):2d}  {k[:90]}")


if __name__ == "__main__":
    main()
