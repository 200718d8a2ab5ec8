#!/usr/bin/env python3
"""Summarise scripts/pmc_sq.sh passes: per kernel (largest dispatches), mean duration and the SQ
ratios that say what bounds a streaming stencil kernel.

    python scripts/pmc_sq_summary.py gpurun_out/sq_k2 [gpurun_out/sq_k3 ...]

VALU issue utilisation = SQ_ACTIVE_INST_VALU * 4 / (SQ_BUSY_CYCLES * SIMDs-per-SE-sampled) is not
portable, so the table reports per-wave ratios instead: VALU instructions per wave, the fraction of
wave-cycles spent issuing VALU (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES) and waiting
(SQ_WAIT_INST_ANY, SQ_WAIT_ANY over SQ_WAVE_CYCLES)."""
import collections
import csv
import sys

for root in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(root + "/run_counter_collection.csv")):
        if "mdfx::dev" not in r["Kernel_Name"] or "init_kernel" in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void mdfx::dev::", "")
        agg[k][r["Counter_Name"]].append((float(r["Counter_Value"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    for k, d in agg.items():
        waves = d["SQ_WAVES"]
        top = max(v for v, _ in waves)
        idx = [i for i, (v, _) in enumerate(waves) if v >= 0.5 * top]
        m = lambda c: sum(d[c][i][0] for i in idx) / len(idx)
        ms = sum(d["SQ_WAVES"][i][1] for i in idx) / len(idx) / 1e6
        wc = m("SQ_WAVE_CYCLES")
        print("%-40s %s  ms %.3f  waves %.0f  valu/wave %.0f  lds/wave %.0f  valu-issue %.3f  wait_inst %.3f  wait_any %.3f"
              % (k[:40], root.split("/")[-1], ms, m("SQ_WAVES"), m("SQ_INSTS_VALU") / m("SQ_WAVES"),
                 m("SQ_INSTS_LDS") / m("SQ_WAVES"), m("SQ_ACTIVE_INST_VALU") / wc, m("SQ_WAIT_INST_ANY") / wc,
                 m("SQ_WAIT_ANY") / wc))
