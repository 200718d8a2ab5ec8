#!/usr/bin/env python3
"""Summarise scripts/pmc_tbk.sh output: per fused kernel (tbk / tb2), counters averaged over its
dispatches (timed launches only, the bitwise-check launch included), plus derived ratios."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_tbk"
field = 4 * 1024 ** 3  # 1024^3 fp32 field bytes
rows = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "*_p*", "run_counter_collection.csv"))):
    tag = os.path.basename(os.path.dirname(f)).rsplit("_p", 1)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "heat7_tb" not in k:
            continue
        rows[(tag, k.split("(")[0].replace("void ", ""))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (tag, k), c in sorted(rows.items()):
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(f"## {tag}: {k}")
    for n in sorted(m):
        print(f"   {n:24s} {m[n]:16.4g}")
    if "SQ_WAVE_CYCLES" in m and "SQ_INSTS_VALU" in m:
        print(f"   VALU insts / wave        {m['SQ_INSTS_VALU'] / max(1, m.get('SQ_WAVES', 1)):16.4g}")
        print(f"   busy frac VALU (act/wave_cyc) {m['SQ_ACTIVE_INST_VALU'] / m['SQ_WAVE_CYCLES']:.3f}")
        print(f"   wait_any / wave_cycles   {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
        print(f"   wait_inst_any / wave_cyc {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
    if "FETCH_SIZE" in m:
        print(f"   fetch/field (x2 corr.)   {2 * m['FETCH_SIZE'] * 1024 / field:.3f}")
