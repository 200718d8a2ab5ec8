"""Python command line over :class:`mpi_cuda_process_amd.Simulation`.

    python -m mpi_cuda_process_amd --stencil 7 --n 256 --steps 100 --json
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 -m mpi_cuda_process_amd --stencil 7 --n 512

The native executables (build/bin/mdfx, mdf, life) are the reference-compatible entry points
(stdin dialogue). This module is the same engine driven from Python, for launches
through torchrun and for scripting; it prints the same JSON metrics line (--json) and the same
print_array dump (--print, reference kernel.cu:115-129).
"""

from __future__ import annotations

import argparse
import json
import sys
import time

from .utils import metrics_record, print_array


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="python -m mpi_cuda_process_amd", description=__doc__.split("\n\n")[0])
    p.add_argument("--stencil", default="7", help="5 | 7 | 27 | life (aliases: mdf, heat7, box27, gol)")
    p.add_argument("--n", type=int, default=0)
    p.add_argument("--nx", type=int, default=0)
    p.add_argument("--ny", type=int, default=0)
    p.add_argument("--nz", type=int, default=0)
    p.add_argument("--h", type=int, default=0, help="2D rows")
    p.add_argument("--w", type=int, default=0, help="2D columns")
    p.add_argument("--steps", "--iters", type=int, default=100)
    p.add_argument("--warmup", type=int, default=0)
    p.add_argument("--dtype", default="f32")
    p.add_argument("--device", default="auto", help="auto | hip | cpu")
    p.add_argument("--ranks", type=int, default=None, help="P virtual slabs in this process")
    p.add_argument("--py", type=int, default=1, help="(z, y) pencils: ranks along y (3D stencils)")
    p.add_argument("--transport", default="auto",
                   help="auto | rccl | ipc | ipc_sdma | torch | staged (one process per rank) | loopback | host "
                        "(one process); ipc pulls faces with blit kernels, ipc_sdma with the SDMA engines")
    p.add_argument("--residual-every", type=int, default=0)
    p.add_argument("--temporal", type=int, default=0,
                   help="time steps fused per sweep: 0 = auto (as mdfx and bench.py: 5 for the fp32 3D 7-point (fp64: 5 from 2048-cell rows, else 4) on "
                        "the GPU, 3 for the 27-point at 1024-cell rows and in fp64, else 2; 8 for the 2D MDF, 12 "
                        "for Life), 1 = one step per sweep")
    p.add_argument("--graph", action="store_true")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--sync-debug", action="store_true")
    p.add_argument("--timeout", type=float, default=0.0)
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--resume", default="")
    p.add_argument("--dump", default="", help="write the final grid (checkpoint format) to this directory")
    p.add_argument("--print", action="store_true", help="print_array dump of the final grid (rank 0)")
    p.add_argument("--json", action="store_true")
    return p


def _problem(a):
    from .models import from_name

    kind = from_name(a.stencil).kind  # resolve aliases
    if kind in ("jacobi5", "life"):
        h = a.h or a.nz or a.n or 256
        w = a.w or a.nx or a.n or 256
        kw = dict(h=h, w=w)
        if kind == "jacobi5":
            kw["dtype"] = a.dtype
        else:
            kw["seed"] = a.seed
        return from_name(kind, **kw)
    n = a.n or 256
    return from_name(kind, nx=a.nx or n, ny=a.ny or n, nz=a.nz or n, dtype=a.dtype).with_init(seed=a.seed)


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    import torch
    import torch.distributed as dist

    from . import Simulation
    from .parallel.dist import detect_env, init_distributed

    distributed = detect_env().world > 1 and a.ranks is None
    if distributed:
        init_distributed()
    prob = _problem(a)
    sim = Simulation(prob, device=a.device, ranks=a.ranks, transport=a.transport, distributed=distributed,
                     overlap=not a.no_overlap, sync_debug=a.sync_debug, residual_every=a.residual_every,
                     graph=a.graph, timeout_s=a.timeout, temporal=a.temporal, py=a.py)
    with sim:
        if a.resume:
            sim.load_checkpoint(a.resume)
        else:
            sim.init()
        sim.run(a.warmup)
        sim.synchronize()
        if distributed:
            dist.barrier()
        t0 = time.perf_counter()
        sim.run(a.steps)
        sim.synchronize()
        dt = time.perf_counter() - t0
        if distributed:  # the slowest rank defines the step time
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        rank0 = not distributed or dist.get_rank() == 0
        if a.dump:
            sim.save_checkpoint(a.dump)
        if a.print:
            g = sim.gather()
            if rank0:
                print_array(g.reshape(prob.nz, prob.ny, prob.nx))
        ngpu = (dist.get_world_size() if distributed else 1) if sim.device == "hip" else 0
        rec = metrics_record(prob, a.steps, dt, ngpu, {"device": sim.device, "temporal": sim.temporal,
                                                       "residual": sim.residual})
        if rank0 and a.json:
            print(json.dumps(rec))
        elif rank0 and not a.print:
            print("%s %dx%dx%d %s | %d steps in %.4f s | %.2f GCells/s" % (prob.kind, prob.nx, prob.ny, prob.nz,
                                                                          prob.dtype, a.steps, dt, rec["value"]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
