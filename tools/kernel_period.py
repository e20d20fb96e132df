"""Launch durations and the spacing of consecutive ends of one kernel in a rocprofv3
kernel trace (run_kernel_trace.csv).  With several frames in flight a launch's duration
overlaps its neighbours', so the device time per frame is the spacing of the ends (bench.py
--inflight).  Usage: kernel_period.py TRACE.csv [NAME_SUBSTRING] [LAST_K]
Prints one JSON line: every launch's start/end (ms from the first start), duration, and the
mean end spacing over the last K launches (K - 1 spacings plus the first of them measured from
the end of the launch before)."""
import csv
import json
import sys

path = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "integrate_kernel<1, false>"
last_k = int(sys.argv[3]) if len(sys.argv) > 3 else 0
rows = [r for r in csv.DictReader(open(path)) if name in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
if not rows:
    sys.exit(f"no launch of {name!r} in {path}")
t0 = int(rows[0]["Start_Timestamp"])
starts = [(int(r["Start_Timestamp"]) - t0) / 1e6 for r in rows]
ends = [(int(r["End_Timestamp"]) - t0) / 1e6 for r in rows]
durs = [e - s for s, e in zip(starts, ends)]
ends_sorted = sorted(ends)
spacing = [b - a for a, b in zip(ends_sorted, ends_sorted[1:])]
k = last_k if 0 < last_k < len(rows) else len(rows) - 1
out = {"kernel": name, "launches": len(rows), "start_ms": [round(x, 3) for x in starts],
       "end_ms": [round(x, 3) for x in ends], "duration_ms": [round(x, 3) for x in durs],
       "mean_duration_ms": sum(durs) / len(durs), "end_spacing_ms": [round(x, 3) for x in spacing],
       f"mean_end_spacing_last_{k}_ms": sum(spacing[-k:]) / k}
print(json.dumps(out))
