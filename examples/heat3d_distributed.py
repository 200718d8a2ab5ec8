#!/usr/bin/env python3
"""3D heat diffusion across GPUs: one process per GPU under torchrun, slabs along z, RCCL halos
(or --transport ipc: device-resident faces through HIP IPC mailboxes, copy engines, no CUs).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/heat3d_distributed.py --n 1024 --steps 200
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/heat3d_distributed.py --transport ipc --share-gpu
        (on a one-GPU machine both ranks share cuda:0: only the ipc transport allows that, and only with
        --share-gpu, a test mode)
    python examples/heat3d_distributed.py --n 128 --steps 20 --device cpu      # single process

Prints the global residual every --report steps and the throughput at the end (rank 0). With
--checkpoint DIR it saves a checkpoint at the end that any other decomposition can resume.
"""

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpi_cuda_process_amd as m  # noqa: E402
from mpi_cuda_process_amd.parallel.dist import detect_env, init_distributed  # noqa: E402
from mpi_cuda_process_amd.utils import metrics_record  # noqa: E402


def main(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--report", type=int, default=50)
    p.add_argument("--dtype", default="f32")
    p.add_argument("--device", default="auto")
    p.add_argument("--checkpoint", default="")
    p.add_argument("--transport", default="auto", help="auto (rccl on GPUs, torch on CPUs) | rccl | ipc | torch")
    p.add_argument("--share-gpu", action="store_true",
                   help="ipc: allow several ranks on one GPU (tests; the exchange assumes one process per GPU)")
    a = p.parse_args(argv)
    distributed = detect_env().world > 1
    if distributed:
        init_distributed()
    rank = dist.get_rank() if distributed else 0
    prob = m.heat3d(n=a.n, dtype=a.dtype)
    kw = dict(transport=a.transport, share_gpu=a.share_gpu) if distributed else {}
    with m.Simulation(prob, device=a.device, distributed=distributed, residual_every=a.report, temporal=0,
                      **kw) as sim:
        sim.init()
        sim.synchronize()
        t0 = time.perf_counter()
        while sim.steps < a.steps:
            sim.run(min(a.report, a.steps - sim.steps))
            if rank == 0:
                print("step %6d  residual %.6e" % (sim.steps, sim.residual), flush=True)
        sim.synchronize()
        dt = time.perf_counter() - t0
        if a.checkpoint:
            sim.save_checkpoint(a.checkpoint)
        n = dist.get_world_size() if distributed else 1
        if rank == 0:
            rec = metrics_record(prob, a.steps, dt, n if sim.device == "hip" else 0,
                                 {"slabs": sim.nranks, "transport": sim.transport, "temporal": sim.temporal})
            print(rec)
    if distributed:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
