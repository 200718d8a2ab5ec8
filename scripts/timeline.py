#!/usr/bin/env python3
"""Print the last ~3 sweeps of a rocprofv3 kernel trace as a timeline (start / duration / gap to the
previous kernel, per queue), with the kernel names shortened.

    python scripts/timeline.py <run_kernel_trace.csv> [n_kernels]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n - 40:-40] if len(rows) > n + 40 else rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void mdfx::dev::", "")[:70]
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print("%9.1f us  dur %8.1f  gap %7.1f  q%-3s %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r.get("Queue_Id", "?"), name))
    prev_end = max(prev_end or 0, e)
