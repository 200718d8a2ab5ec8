#!/usr/bin/env python3
"""Per-dispatch effective shader clock and SQ ratios of the headline kernel from a rocprofv3 --pmc
pass with GRBM_GUI_ACTIVE (scripts/gpu_r05d.sh). GRBM_GUI_ACTIVE sums the busy cycles of the 8
XCDs (MI355X_MICROARCH.md, DVFS give-back), so the clock is GUI_ACTIVE / 8 / dispatch time. The
dispatches are listed in launch order, so the sweeps right after a random init (rough data) can be
compared with later ones.

    python scripts/pmc_clock.py gpurun_out/r05d/clock [kernel-substring]
"""
import collections
import csv
import os
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "heat7_wxk"
f = [os.path.join(d, x) for x in os.listdir(d) if x.endswith("counter_collection.csv")]
assert f, "no counter_collection.csv under %s" % d
disp = collections.OrderedDict()
for r in csv.DictReader(open(f[0])):
    if sub not in r["Kernel_Name"]:
        continue
    k = int(r["Dispatch_Id"])
    e = disp.setdefault(k, {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
print("%5s %9s %8s %8s %8s %8s" % ("disp", "ms", "GHz", "valu", "wait", "waitI"))
for k, e in disp.items():
    ms = e["ns"] / 1e6
    ghz = e.get("GRBM_GUI_ACTIVE", 0) / 8 / e["ns"] if e["ns"] else 0
    wc = e.get("SQ_WAVE_CYCLES", 0) or 1
    print("%5d %9.4f %8.3f %8.3f %8.3f %8.3f" % (k, ms, ghz, e.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                                               e.get("SQ_WAIT_ANY", 0) / wc, e.get("SQ_WAIT_INST_ANY", 0) / wc))
