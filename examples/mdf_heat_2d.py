#!/usr/bin/env python3
"""2D finite-difference heat diffusion (the reference's MDF program, MDF_kernel.cu) to convergence.

Edges held at 100, interior starting at 0; runs until the global L2 norm of the update falls
below --tol, printing the residual every --report steps. Runs on the GPU when one is visible
(fused multi-step sweeps), else on the CPU; add --ranks P to split the rows into P slabs.

    python examples/mdf_heat_2d.py --h 512 --w 512 --tol 1e-3
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import mpi_cuda_process_amd as m  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--h", type=int, default=256)
    p.add_argument("--w", type=int, default=256)
    p.add_argument("--tol", type=float, default=1e-2)
    p.add_argument("--report", type=int, default=500)
    p.add_argument("--max-steps", type=int, default=200000)
    p.add_argument("--ranks", type=int, default=None)
    p.add_argument("--device", default="auto")
    a = p.parse_args(argv)
    prob = m.mdf2d(h=a.h, w=a.w)  # Dirichlet: edges 100, interior 0
    t0 = time.perf_counter()
    with m.Simulation(prob, device=a.device, ranks=a.ranks, residual_every=a.report, temporal=0) as sim:
        sim.init()
        while sim.steps < a.max_steps:
            sim.run(a.report)
            print("step %7d  residual %.6e" % (sim.steps, sim.residual))
            if sim.residual < a.tol:
                break
        grid = sim.gather()
        steps, res, dev, depth = sim.steps, sim.residual, sim.device, sim.temporal
    dt = time.perf_counter() - t0
    centre = float(grid[a.h // 2, 0, a.w // 2])
    print("%s after %d steps in %.2f s (%s, %d fused steps per sweep): centre temperature %.4f" %
          ("converged" if res < a.tol else "stopped", steps, dt, dev, depth, centre))
    return 0 if res < a.tol else 1


if __name__ == "__main__":
    sys.exit(main())
