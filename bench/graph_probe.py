#!/usr/bin/env python3
"""Graph replay vs eager steps of the N = 8 rank proxy under HIP runtime settings (one child process
per setting, since the runtime reads them at start-up). Question answered: does hipGraphLaunch keep
the captured cycle's two branches (interior sweep on the compute stream || boundary sweep +
exchange on the halo stream) concurrent, or run them one after the other?

    python bench/graph_probe.py [--temporal 2] [--rounds 2]
"""

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (the package defaults DEBUG_HIP_FORCE_GRAPH_QUEUES to 1; "0" restores the runtime's own choice)
SETTINGS = [{"DEBUG_HIP_FORCE_GRAPH_QUEUES": "0"}, {"DEBUG_CLR_GRAPH_PACKET_CAPTURE": "0", "DEBUG_HIP_FORCE_GRAPH_QUEUES": "0"},
            {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "4"}, {"DEBUG_HIP_FORCE_GRAPH_QUEUES": "1"}]


def child(a):
    sys.path.insert(0, ROOT)
    import torch

    import mpi_cuda_process_amd as m

    prob = m.heat3d(n=1024)
    out = {"env": {k: os.environ.get(k) for s in SETTINGS for k in s}}
    with m.Simulation(prob, device="hip", ranks=8, proxy_rank=4, temporal=a.temporal, graph=False) as sim:
        def ms(steps=48):
            sim.synchronize()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sim.run(steps)
            sim.synchronize()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / steps * 1e3
        for ov in (True, False):
            for g in (False, True):
                sim.set_options(graph=g, min_rounds=a.rounds, overlap=ov)
                sim.init()
                sim.prepare_graphs()
                sim.run(12)
                out["%s_%s" % ("overlap" if ov else "serial", "graph" if g else "eager")] = round(
                    min(ms() for _ in range(3)), 4)
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--temporal", type=int, default=2)
    p.add_argument("--rounds", type=int, default=2)
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        return child(a)
    rc = 0
    for s in SETTINGS:
        env = dict(os.environ, **s)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--temporal", str(a.temporal),
                            "--rounds", str(a.rounds)], env=env, capture_output=True, timeout=240)
        line = [l for l in r.stdout.decode().splitlines() if l.startswith("{")]
        print(json.dumps(s), line[0] if line else "FAILED rc=%d %s" % (r.returncode, r.stderr.decode()[-400:]),
              flush=True)
        if r.returncode != 0:
            rc = r.returncode
            if r.returncode < 0 or r.returncode > 1:
                break  # a crash: no further GPU work in this call
    return rc


if __name__ == "__main__":
    sys.exit(main())
