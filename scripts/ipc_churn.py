#!/usr/bin/env python3
"""Repeated ipc engine construction / teardown in W processes sharing one GPU, in bench.py's trial
order ((ipc, slabs), (ipc, pencils), (ipc_sdma, slabs), (ipc_sdma, pencils), twice). Reproduces and
checks the fix for "hipIpcGetMemHandle -> invalid argument" on the 4th-11th engine of a process
(round-4 share-GPU rehearsal of the N = 8 bench).

    python scripts/ipc_churn.py --world 8 [--n 1024] [--passes 2]
"""

import argparse
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    import mpi_cuda_process_amd as m
    from mpi_cuda_process_amd.parallel.dist import init_distributed

    env = init_distributed("gloo")
    torch.cuda.set_device(0)
    prob = m.heat3d(n=a.n)
    combos = [("ipc", 1), ("ipc", 2), ("ipc_sdma", 1), ("ipc_sdma", 2)] * a.passes
    t0 = time.time()
    for i, (t, py) in enumerate(combos):
        try:
            sim = m.Simulation(prob, device="hip", distributed=True, transport=t, py=py, temporal=4, devices=[0],
                               timeout_s=60.0, share_gpu=True)
            sim.init()
            sim.run(8)
            sim.synchronize()
            sim.close()
        except Exception as e:  # noqa: BLE001 - name the rank and engine, then fail
            print("CHURN rank %d engine %d %s py=%d FAILED: %s: %s" % (env.rank, i, t, py, type(e).__name__, e),
                  file=sys.stderr, flush=True)
            raise
        if env.rank == 0:
            print("engine %d %s py=%d ok (+%.1fs)" % (i, t, py, time.time() - t0), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--world", type=int, default=8)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--passes", type=int, default=2)
    p.add_argument("--child", action="store_true")
    a = p.parse_args()
    if a.child:
        return child(a)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(a.world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", "--n", str(a.n),
                                       "--passes", str(a.passes)], env=env))
    rc = 0
    for r, q in enumerate(procs):
        q.wait()
        if q.returncode != 0:
            print("ipc_churn rank %d exit status %d" % (r, q.returncode), flush=True)
        rc = rc or q.returncode
    print("ipc_churn world=%d rc=%d" % (a.world, rc), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main())
