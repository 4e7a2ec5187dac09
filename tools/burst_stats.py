"""Per-launch statistics of the timed headline burst from a rocprofv3 kernel trace.

bench.py --headline-only runs settle steps, W warmup steps and K timed steps of the
headline kernel and nothing else; the timed burst is the last 3 K dispatches of that
kernel.  This prints (and writes as JSON) their mean / min / max duration, the mean x 3
per step, and the burst's wall span per step, to compare with bench's ms_per_step.

  python tools/burst_stats.py <kernel_trace.csv> <kernel name> <timed steps> <out.json> [launches per step]
"""
import csv
import json
import sys


def main():
    path, name, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    per_step = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Kernel_Name"].startswith(name):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    k = steps * per_step
    if len(rows) < k:
        raise SystemExit(f"only {len(rows)} dispatches of {name}, expected >= {k}")
    burst = rows[-k:]
    dur = [(e - s) * 1e-3 for s, e in burst]          # us
    span_us = (burst[-1][1] - burst[0][0]) * 1e-3
    res = {"kernel": name, "source": path, "dispatches_total": len(rows), "burst_dispatches": k,
           "mean_us": sum(dur) / k, "min_us": min(dur), "max_us": max(dur),
           "mean_x_per_step_ms": sum(dur) / k * per_step * 1e-3,
           "burst_span_per_step_ms": span_us / steps * 1e-3,
           "first_launch_of_step_mean_us": sum(dur[0::per_step]) / steps,
           "other_launches_mean_us": (sum(dur) - sum(dur[0::per_step])) / (k - steps) if per_step > 1 else None}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
