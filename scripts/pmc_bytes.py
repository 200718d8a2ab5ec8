#!/usr/bin/env python3
"""Per-kernel DRAM-side bytes and achieved bandwidth from separate rocprofv3 FETCH_SIZE and
WRITE_SIZE passes (scripts/gpu_session.sh pmc_fetch / pmc_write, optional PMC_TAG suffix).

    python scripts/pmc_bytes.py gpurun_out [tag] [--field-bytes B]

FETCH_SIZE / WRITE_SIZE are KB per dispatch. On gfx950 FETCH_SIZE counts half the bytes of a
wide coalesced streaming read (MI355X_MICROARCH.md, HBM section), so it is doubled here. Only the
large dispatches of each kernel (>= 25% of its largest byte count) are averaged: the engine's
boundary-plane launches of the same kernel are tiny and would mix two populations. The rate is
(fetch + write) / kernel time; field/step columns divide by one field's bytes.
"""
import argparse
import collections
import csv
import os

ROOF_TBPS = 6.29  # float4 copy, MI355X_MICROARCH.md


def load(path, counter):
    rows = collections.defaultdict(list)
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return rows
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter or "mdfx" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void mdfx::dev::", "")
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        rows[name].append((float(r["Counter_Value"]) * 1024.0, ns))
    return rows


def big(vals):
    top = max(v for v, _ in vals)
    sel = [(v, ns) for v, ns in vals if v >= 0.25 * top]
    return sum(v for v, _ in sel) / len(sel), sum(ns for _, ns in sel) / len(sel), len(sel)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root", nargs="?", default="gpurun_out")
    ap.add_argument("tag", nargs="?", default="")
    ap.add_argument("--field-bytes", type=float, default=0.0, help="bytes of one field (0: no per-field column)")
    a = ap.parse_args()
    sfx = "_" + a.tag if a.tag else ""
    fetch = load(os.path.join(a.root, "pmc_fetch" + sfx), "FETCH_SIZE")
    write = load(os.path.join(a.root, "pmc_write" + sfx), "WRITE_SIZE")
    print("pass: %s  (FETCH_SIZE x2 corrected; large dispatches only)" % (a.tag or "default bench"))
    print("%-52s %5s %9s %10s %10s %8s %7s %s" % ("kernel", "n", "ms", "fetch GB", "write GB", "TB/s", "%roof",
                                                  "fetch+write / field" if a.field_bytes else ""))
    for k in sorted(set(fetch) | set(write)):
        if k not in fetch:
            continue
        if k not in write:  # a fetch-only pass: bytes fetched per dispatch and the kernel time
            fb, fns, n = big(fetch[k])
            extra = "%.3f fetched" % (2.0 * fb / a.field_bytes) if a.field_bytes else ""
            print("%-52s %5d %9.3f %10.3f %10s %8s %7s %s" % (k[:52], n, fns / 1e6, 2.0 * fb / 1e9, "-", "-", "-", extra))
            continue
        fb, fns, n = big(fetch[k])
        wb, wns, _ = big(write[k])
        fb *= 2.0
        ms = min(fns, wns) / 1e6
        tbps = (fb + wb) / (ms * 1e-3) / 1e12
        extra = "%.3f + %.3f" % (fb / a.field_bytes, wb / a.field_bytes) if a.field_bytes else ""
        print("%-52s %5d %9.3f %10.3f %10.3f %8.2f %6.1f%% %s" % (k[:52], n, ms, fb / 1e9, wb / 1e9, tbps,
                                                                100 * tbps / ROOF_TBPS, extra))


if __name__ == "__main__":
    main()
