#!/usr/bin/env python3
"""Sum the counters of one rocprofv3 --pmc pass per kernel (large dispatches of the named kernel) and
print them per SQ_WAVE_CYCLES / per wave (scripts/gpu_r05m.sh).

    python scripts/pmc_sq.py <pass dir> <kernel substring>
"""
import collections
import csv
import os
import sys

d, sub = sys.argv[1], sys.argv[2]
f = os.path.join(d, "run_counter_collection.csv")
disp = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(f)):
    if sub not in r["Kernel_Name"]:
        continue
    k = int(r["Dispatch_Id"])
    disp[k][r["Counter_Name"]] = float(r["Counter_Value"])
    disp[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    names[k] = r["Kernel_Name"].split("(")[0].replace("void mdfx::dev::", "")
if not disp:
    sys.exit("no dispatch of %s" % sub)
big = max(v.get("SQ_WAVE_CYCLES", 0) for v in disp.values())
tot = collections.Counter()
n = 0
for k, v in disp.items():
    if v.get("SQ_WAVE_CYCLES", 0) < 0.25 * big:
        continue
    n += 1
    for c, x in v.items():
        tot[c] += x
print("%s: %d dispatches, %.3f ms each" % (names[next(iter(disp))], n, tot["_ns"] / n / 1e6))
wc = tot.get("SQ_WAVE_CYCLES", 0) or 1
waves = tot.get("SQ_WAVES", 0) or 1
for c in sorted(tot):
    if c.startswith("_"):
        continue
    extra = ""
    if c.startswith("SQ_") and c not in ("SQ_WAVES", "SQ_WAVE_CYCLES"):
        extra = "  %.3f per wave cycle  %.1f per wave" % (tot[c] / wc, tot[c] / waves)
    print("  %-24s %16.0f%s" % (c, tot[c], extra))
if "GRBM_GUI_ACTIVE" in tot:
    print("  effective clock %.3f GHz" % (tot["GRBM_GUI_ACTIVE"] / 8 / tot["_ns"]))
