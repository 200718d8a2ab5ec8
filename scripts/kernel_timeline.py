#!/usr/bin/env python3
"""Stream timeline of a rocprofv3 --kernel-trace run: where the wall time of a step goes.

Usage: kernel_timeline.py <run_kernel_trace.csv | dir containing one> [--skip N] [--match SUBSTR]

Per stream: kernels, busy time; for the whole device: wall span of the traced window, union of busy
intervals, time with >= 2 streams busy (overlap), and the idle gaps (nothing running) binned by
length. --skip drops the first N dispatches (warm-up, init fills). Used on the rank proxies to see
whether the halo stream's boundary/copy work hides under the interior sweep or serialises with it.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    if os.path.isdir(path):
        hits = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
        if not hits:
            sys.exit(f"no kernel_trace.csv under {path}")
        path = sorted(hits)[0]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]),
                         int(r["Queue_Id"]), r["Kernel_Name"]))
    rows.sort()
    return path, rows


def short(name, n=60):
    name = name.split("(")[0]
    return name if len(name) <= n else name[: n - 3] + "..."


def main(argv):
    if not argv:
        sys.exit(__doc__)
    skip, match = 0, None
    args = list(argv)
    if "--skip" in args:
        i = args.index("--skip"); skip = int(args[i + 1]); del args[i:i + 2]
    if "--match" in args:
        i = args.index("--match"); match = args[i + 1]; del args[i:i + 2]
    path, rows = load(args[0])
    rows = rows[skip:]
    if match:
        first = next((k for k, r in enumerate(rows) if match in r[4]), None)
        rows = rows[first:] if first is not None else []
    if not rows:
        sys.exit("no dispatches")
    t0 = rows[0][0]
    t1 = max(r[1] for r in rows)
    span = t1 - t0
    print(f"trace: {path}\ndispatches: {len(rows)}   window: {span / 1e6:.3f} ms")
    by_stream = defaultdict(list)
    for r in rows:
        by_stream[(r[2], r[3])].append(r)
    for (s, q), rs in sorted(by_stream.items()):
        busy = sum(e - b for b, e, *_ in rs)
        names = defaultdict(lambda: [0, 0])
        for b, e, _, _, n in rs:
            names[short(n)][0] += 1
            names[short(n)][1] += e - b
        print(f"\nstream {s} queue {q}: {len(rs)} kernels, busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f}% of window)")
        for n, (c, t) in sorted(names.items(), key=lambda kv: -kv[1][1])[:8]:
            print(f"   {c:6d} x {t / c / 1e3:9.1f} us  {t / 1e6:8.3f} ms  {n}")
    # sweep: union busy, overlap (>=2 streams), idle gaps
    ev = []
    for b, e, s, q, _ in rows:
        ev.append((b, 1)); ev.append((e, -1))
    ev.sort(key=lambda x: (x[0], x[1]))
    active, last, busy1, busy2 = 0, ev[0][0], 0, 0
    gaps = []
    for t, d in ev:
        if active >= 1:
            busy1 += t - last
        if active >= 2:
            busy2 += t - last
        if active == 0 and t > last:
            gaps.append(t - last)
        active += d
        last = t
    print(f"\ndevice busy (any stream): {busy1 / 1e6:.3f} ms ({100 * busy1 / span:.1f}%)")
    print(f"overlap (>=2 kernels):     {busy2 / 1e6:.3f} ms ({100 * busy2 / span:.1f}%)")
    idle = sum(gaps)
    print(f"idle gaps: {len(gaps)}  total {idle / 1e6:.3f} ms ({100 * idle / span:.1f}%)")
    bins = [(0, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e12)]
    for lo, hi in bins:
        g = [x for x in gaps if lo <= x < hi]
        if g:
            print(f"   {lo / 1e3:6.0f}-{hi / 1e3 if hi < 1e12 else float('inf'):6.0f} us: {len(g):5d} gaps, {sum(g) / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1:])
