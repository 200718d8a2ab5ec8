#!/usr/bin/env python3
"""Headline benchmark: GCells/s of the 3D 7-point Jacobi stencil on a 1024^3 fp32 grid,
slab-decomposed over N MI355X GPUs (one process per GPU, RCCL halo exchange over xGMI).

    python bench.py                         # N = 1
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

The grid is fixed as N grows (strong scaling, the BASELINE.json config "3D 7-pt Jacobi 1024^3 fp32
slab-decomposed across 8xMI355X"). Data is synthetic: a uniform random initial grid generated on
the device from a counter-based hash of the global cell index (seed 1). Every timed step is a full
Jacobi update of every cell (boundary planes + halo exchange + interior), nothing is skipped or
cached. By default two consecutive Jacobi steps are fused into one pass over memory (temporal
blocking, --temporal 2; bitwise identical to two single steps, tests/test_gpu_temporal.py): every
step is still computed in full, the fused kernel just keeps u^{t+1} on chip. --temporal 1 measures
one sweep per step. Timing: W untimed warmup steps, then exactly K steps bracketed by barrier +
torch.cuda.synchronize() on both sides; the slowest rank's time is reported. GCells/s =
nx*ny*nz*K / t / 1e9 for the whole job. Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "GCells/s (whole node), 3D 7-pt Jacobi 1024^3 fp32 at 1/2/4/8 MI355X"
HBM_MEASURED_TBPS = 6.29  # float4 copy, MI355X_MICROARCH.md (8.0 spec)


def parse():
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n", type=int, default=1024, help="cube edge (default 1024)")
    p.add_argument("--nx", type=int, default=0)
    p.add_argument("--ny", type=int, default=0)
    p.add_argument("--nz", type=int, default=0)
    p.add_argument("--stencil", default="heat7", choices=["heat7", "box27", "jacobi5", "life"])
    p.add_argument("--dtype", default="f32", choices=["f32", "f64", "u8"])
    p.add_argument("--transport", default="auto",
                   help="auto|rccl|torch|staged (distributed), loopback (1 process)")
    p.add_argument("--virtual-ranks", type=int, default=0,
                   help="split the grid into P slabs inside ONE process (loopback transport)")
    p.add_argument("--graph", action="store_true", help="replay 2-step cycles as hipGraphs")
    p.add_argument("--temporal", type=int, default=0,
                   help="time steps fused per memory sweep (temporal blocking); 0 = auto: 2 for the 3D "
                        "stencils, 8 (2D MDF) / 4 (Life) for the 2D ones, where a fused kernel exists")
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--residual-every", type=int, default=0)
    p.add_argument("--variant", default="auto", choices=["auto", "tuned", "naive"])
    p.add_argument("--device", default="auto", choices=["auto", "hip", "cpu"])
    p.add_argument("--repeats", type=int, default=1, help="timed repetitions; the best is reported")
    return p.parse_args()


def main():
    a = parse()
    from mpi_cuda_process_amd import Simulation, heat3d, box27, mdf2d, life2d, native
    from mpi_cuda_process_amd.parallel.dist import init_distributed

    force = os.environ.get("MDFX_FORCE_DIST", "") == "1"  # distributed path even at WORLD_SIZE 1 (tests)
    env = init_distributed("gloo", force=force) if (int(os.environ.get("WORLD_SIZE", "1")) > 1 or force) else None
    world = dist.get_world_size() if env else 1
    rank = dist.get_rank() if env else 0
    if env and a.gpus != world:
        print("warning: --gpus %d but WORLD_SIZE %d; using WORLD_SIZE" % (a.gpus, world), file=sys.stderr)
    hip = torch.cuda.is_available() and a.device != "cpu"
    if hip:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local % torch.cuda.device_count())
    native().set_kernel_variant(a.variant)

    nx, ny, nz = a.nx or a.n, a.ny or a.n, a.nz or a.n
    if a.stencil in ("jacobi5", "life"):
        ny = 1  # 2D grids: nx = width, nz = height
    if a.stencil == "heat7":
        prob = heat3d(nx=nx, ny=ny, nz=nz, dtype=a.dtype)
    elif a.stencil == "box27":
        prob = box27(nx=nx, ny=ny, nz=nz, dtype=a.dtype)
    elif a.stencil == "jacobi5":
        prob = mdf2d(h=nz, w=nx, dtype=a.dtype)
    else:
        prob = life2d(h=nz, w=nx)

    temporal = a.temporal
    if temporal <= 0:
        # fused depth where a kernel exists: 2 for the 3D stencils, 8 (MDF) / 4 (Life) for the 2D
        # ones (profiles/r01_deep_temporal_2d.txt), capped so every slab is at least 4 sweeps deep
        want = {"jacobi5": 8, "life": 4}.get(a.stencil, 2)
        nslab = max(1, int(os.environ.get("WORLD_SIZE", "1")), a.virtual_ranks)
        while want > 1 and prob.nz < 4 * want * nslab:
            want //= 2
        temporal = 1
        if want > 1 and (not hip or native().hip_supports_steps(prob.kind, prob.dtype, prob.nx, prob.ny,
                                                                prob.nz, want, want)):
            temporal = want
    kw = dict(device="hip" if hip else "cpu", overlap=not a.no_overlap, graph=a.graph,
              residual_every=a.residual_every, timeout_s=900.0 if hip else 0.0, temporal=temporal)
    if env:
        sim = Simulation(prob, distributed=True, transport=a.transport, **kw)
    else:
        vr = a.virtual_ranks or 1
        sim = Simulation(prob, ranks=vr, distributed=False,
                         transport="auto" if a.transport in ("auto", "rccl", "torch", "staged") else a.transport,
                         **kw)
    sim.init()

    def barrier():
        if env:
            dist.barrier()

    def sync():
        sim.synchronize()
        if hip:
            torch.cuda.synchronize()

    sim.run(a.warmup)
    sync()
    best = None
    for _ in range(max(1, a.repeats)):
        barrier()
        sync()
        t0 = time.perf_counter()
        sim.run(a.steps)
        sync()
        t1 = time.perf_counter()
        barrier()
        dt = t1 - t0
        if env:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        best = dt if best is None else min(best, dt)

    cells = prob.cells
    gcells = cells * a.steps / best / 1e9
    ms = best / a.steps * 1e3
    nproc = world if env else 1
    bpc = prob.bytes_per_cell_per_step
    roof = HBM_MEASURED_TBPS * 1e12 / bpc / 1e9 * (nproc if hip else 0)
    if rank == 0:
        par = ("slab-z%d (1 process/GPU, %s halo over xGMI, interior||boundary streams)" % (world, sim.transport)
               if env else ("slab-z%d virtual in 1 process (%s)" % (a.virtual_ranks, sim.transport)
                            if a.virtual_ranks > 1 else "single GPU" if hip else "cpu"))
        model = {"heat7": "3D 7-pt Jacobi", "box27": "3D 27-pt", "jacobi5": "2D 5-pt MDF",
                 "life": "2D Game of Life"}[a.stencil]
        rec = {
            "metric": METRIC if (a.stencil == "heat7" and a.dtype == "f32" and (nx, ny, nz) == (1024,) * 3)
            else "GCells/s (whole node), %s %dx%dx%d %s" % (model, nx, ny, nz, a.dtype),
            "value": round(gcells, 3),
            "unit": "GCells/s",
            "n_gpus": nproc if hip else 0,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": {"f32": "fp32", "f64": "fp64", "u8": "u8"}[a.dtype],
            "data": "synthetic (uniform random grid from a counter hash of the global index, seed 1)",
            "config": {
                "model": "%s %dx%dx%d %s" % (model, nx, ny, nz, a.dtype),
                "global_batch": 1,
                "seq_len": nz,
                "grid": [nx, ny, nz],
                "parallelism": par,
                "kernel_variant": native().kernel_variant(),
                "graph": a.graph,
                "overlap": not a.no_overlap,
                "temporal_block": temporal,
            },
            "per_gpu_gcells": round(gcells / max(nproc, 1), 3),
            "effective_hbm_TBps_per_gpu": round(gcells * bpc / 1e3 / max(nproc, 1), 3),
            "pct_of_measured_hbm_roof": round(100.0 * gcells / roof, 1) if roof else None,
        }
        print(json.dumps(rec), flush=True)
    sim.close()
    if env:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
