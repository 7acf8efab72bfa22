"""One step's kernel timeline from a rocprofv3 --kernel-trace CSV: the
kernels of the last complete step, each with start / end relative to the
step's first kernel and its queue.  usage: timeline.py kernel_trace.csv [marker_kernel [lead_us]]"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_join_window"
    lead = float(sys.argv[3]) if len(sys.argv) > 3 else 300.0  # us before the marker that still belong to its step
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", r.get("Stream_Id", "?")),
                         r["Kernel_Name"].split("(")[0][:60]))
    rows.sort()
    marks = [r[0] for r in rows if marker in r[3]]
    # a step: from `lead` us before one marker launch to `lead` us before the
    # next (the last complete one: the second to last marker)
    lo, hi = (marks[-2] - lead * 1e3, marks[-1] - lead * 1e3) if len(marks) >= 2 else (rows[0][0], rows[-1][1])
    step = [r for r in rows if lo <= r[0] < hi]
    t0 = step[0][0]
    tend = max(r[1] for r in step)
    print(f"step span {(tend - t0) / 1e3:.1f} us, {len(step)} kernels")
    for s, e, q, k in step:
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {k}")


if __name__ == "__main__":
    main()
