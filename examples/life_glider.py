#!/usr/bin/env python3
"""Game of Life (the reference's kernel.cu) with a glider: print the board before and after.

The glider moves one cell diagonally every 4 generations; after 4*k generations the same shape
reappears k cells down and right. The board is split into row slabs (--ranks) exactly like the
reference's two MPI ranks, and printed with the reference's print_array format.

    python examples/life_glider.py --h 20 --w 40 --generations 16 --ranks 3
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import mpi_cuda_process_amd as m  # noqa: E402
from mpi_cuda_process_amd.utils import format_array  # noqa: E402

GLIDER = np.array([[0, 1, 0], [0, 0, 1], [1, 1, 1]], dtype=np.uint8)


def run(h, w, generations, ranks=None, device="auto"):
    board = np.zeros((h, 1, w), dtype=np.uint8)
    board[2:5, 0, 2:5] = GLIDER
    prob = m.life2d(h=h, w=w)
    with m.Simulation(prob, device=device, ranks=ranks) as sim:
        sim.init(m.InitCondition(kind="constant", value=0))
        for i in range(sim.num_local):
            lay = sim.layout(i)
            sim.write_local(i, board[lay["z0"]:lay["z1"]])
        sim.run(generations)
        return board, sim.gather()


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--h", type=int, default=20)
    p.add_argument("--w", type=int, default=40)
    p.add_argument("--generations", type=int, default=16)
    p.add_argument("--ranks", type=int, default=None)
    p.add_argument("--device", default="auto")
    a = p.parse_args(argv)
    before, after = run(a.h, a.w, a.generations, a.ranks, a.device)
    sys.stdout.write(format_array(before))
    sys.stdout.write(format_array(after))
    k = a.generations // 4
    expected = np.zeros_like(before)
    expected[2 + k:5 + k, 0, 2 + k:5 + k] = GLIDER
    ok = a.generations % 4 == 0 and np.array_equal(after, expected)
    print("glider moved %d cells diagonally: %s" % (k, "yes" if ok else "no"))
    return 0 if ok or a.generations % 4 else 1


if __name__ == "__main__":
    sys.exit(main())
