#!/usr/bin/env python3
"""Is the N = 8 rank proxy host-bound? Times the host's enqueue of `steps` steps (run() returns once
every launch is queued) against the wall time to their completion, eager and graph-replayed.

    python bench/host_probe.py [--ranks 8] [--py 1] [--steps 48]
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mpi_cuda_process_amd as m  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--py", type=int, default=1)
    p.add_argument("--steps", type=int, default=48)
    p.add_argument("--n", type=int, default=1024)
    a = p.parse_args()
    prob = m.heat3d(n=a.n)
    out = {}
    with m.Simulation(prob, device="hip", ranks=a.ranks, proxy_rank=a.ranks // 2, temporal=4, py=a.py) as sim:
        for g in (False, True):
            sim.set_options(graph=g, min_rounds=1, overlap=True)
            sim.init()
            sim.prepare_graphs()
            sim.run(8)
            best = None
            for _ in range(3):
                sim.synchronize()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                sim.run(a.steps)
                t1 = time.perf_counter()
                sim.synchronize()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                rec = (round((t1 - t0) / a.steps * 1e3, 4), round((t2 - t0) / a.steps * 1e3, 4))
                best = rec if best is None or rec[1] < best[1] else best
            out["graph" if g else "eager"] = {"enqueue_ms_per_step": best[0], "total_ms_per_step": best[1]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
