"""Process bootstrap over torch.distributed and the torch point-to-point halo transport.

One process per GPU (``torchrun --nproc-per-node N`` or ``mpirun -np N``): the process's rank is
its slab index, its device is ``LOCAL_RANK % device_count``. The control plane (unique-id
broadcast, barriers, max-over-ranks timing) runs on a gloo process group; the data plane is either
the native RCCL transport (ncclSend/ncclRecv over xGMI on the engine's halo stream) or
:class:`TorchP2PTransport` (torch.distributed isend/irecv, e.g. gloo for CPU tests).
"""

from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    launched: bool = False  # started by torchrun / mpirun


def detect_env() -> DistEnv:
    """Rank / size from torchrun (RANK/WORLD_SIZE), MPICH hydra (PMI_*) or Open MPI (OMPI_*)."""
    e = os.environ
    for rk, ws, lr in (("RANK", "WORLD_SIZE", "LOCAL_RANK"),
                       ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"),
                       ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID")):
        if rk in e and ws in e:
            rank, world = int(e[rk]), int(e[ws])
            local = int(e.get(lr, rank))
            return DistEnv(rank, world, local, True)
    return DistEnv()


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def init_distributed(backend: str = "gloo", timeout_s: float = 600.0, force: bool = False) -> DistEnv:
    """Initialise the default process group from the launcher environment (idempotent).

    ``force`` initialises it even for a single process (exercises the distributed code path)."""
    env = detect_env()
    if not dist.is_initialized() and (env.world > 1 or force):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", str(env.rank))
        os.environ.setdefault("WORLD_SIZE", str(env.world))
        dist.init_process_group(backend=backend, rank=env.rank, world_size=env.world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    if dist.is_initialized():
        env.rank, env.world = dist.get_rank(), dist.get_world_size()
    return env


def broadcast_bytes(data: Optional[bytes], src: int = 0, group=None) -> bytes:
    """Broadcast a byte string (e.g. the 128-byte ncclUniqueId) from ``src`` over a CPU group."""
    obj = [data]
    dist.broadcast_object_list(obj, src=src, group=group)
    return obj[0]


# groups made for engines on a default group of another backend, one per (backend, rank set) and
# process: dist.new_group is a collective every default-group rank must join in the same order, so
# building one per engine would leak groups and hang any rank that builds an engine its peers do not
_GROUPS: dict = {}


def group_for(backend: str, group=None, timeout_s: float = 300.0):
    """A ``backend`` group over the ranks of ``group`` (the default group if None): ``group`` itself
    if it already uses that backend, else one created once per process and rank set (with the given
    timeout) and reused by every later engine."""
    if dist.get_backend(group) == backend:
        return group
    ranks = tuple(range(dist.get_world_size())) if group is None else tuple(dist.get_process_group_ranks(group))
    g = _GROUPS.get((backend, ranks))
    if g is None:
        g = dist.new_group(ranks=list(ranks), backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        _GROUPS[(backend, ranks)] = g
    return g


def gloo_group_for(group=None, timeout_s: float = 300.0):
    """The CPU (gloo) group a control plane over ``group``'s ranks uses (see :func:`group_for`)."""
    return group_for("gloo", group, timeout_s)


class ControlPlane:
    """Host-side collectives for the native transports that move data on the device themselves
    (``ipc``): the handle swap (allgather of byte strings), the residual all-reduce and barriers,
    over a CPU (gloo) process group."""

    def __init__(self, group=None, timeout_s: float = 300.0):
        # the control plane moves CPU tensors: on a non-gloo group (e.g. a torchrun default NCCL
        # group) it uses a gloo group over the same ranks (made once per process, gloo_group_for)
        self.group = gloo_group_for(group, timeout_s)
        self.timeout_s = timeout_s

    def callbacks(self) -> dict:
        return {"allgather": self.allgather, "allreduce_sum": self.allreduce_sum,
                "allreduce_max": self.allreduce_max, "barrier": self.barrier}

    def allgather(self, mine: bytes) -> list:
        out = [None] * dist.get_world_size(self.group)
        dist.all_gather_object(out, bytes(mine), group=self.group)
        return out

    def allreduce_sum(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return float(t.item())

    def allreduce_max(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def barrier(self) -> None:
        # bounded (gloo): a dead peer raises after timeout_s instead of blocking for the group timeout
        if dist.get_backend(self.group) == "gloo":
            dist.monitored_barrier(group=self.group, timeout=datetime.timedelta(seconds=self.timeout_s))
        else:
            dist.barrier(group=self.group)


class TorchP2PTransport:
    """Halo exchange through torch.distributed point-to-point ops (callback transport).

    The native engine calls :meth:`exchange` with the index of the buffer just written; faces are
    exported zero-copy from the engine (DLPack) and exchanged with ``isend``/``irecv``. On a HIP
    field the ops are issued on the slab's halo stream, so they stay ordered with the engine's
    kernels exactly like the native transports.
    """

    def __init__(self, group=None, staged: bool = False):
        self.group = group
        # staged: device faces travel through host memory over a CPU (gloo) group. Slow, but it
        # lets several processes share ONE GPU and still run the real multi-process engine path
        # (RCCL refuses two ranks on one device) — tests/test_gpu_multiprocess.py.
        self.staged = staged
        self.solver = None  # set by the Simulation once the native solver exists

    def callbacks(self) -> dict:
        return {"exchange": self.exchange, "allreduce_sum": self.allreduce_sum,
                "allreduce_max": self.allreduce_max, "barrier": self.barrier}

    def _bytes(self, ptr: int, n: int) -> torch.Tensor:
        return torch.from_dlpack(self.solver.bytes_view(0, ptr, n))

    def _face(self, sp: dict, key: str) -> torch.Tensor:
        """The span's send or recv cells as a (height, width) byte view: z faces are one
        contiguous piece, pencil y faces `height` rows of planes `stride` bytes apart."""
        h, w, st = sp.get("height", 1), sp.get("width", sp["bytes"]), sp.get("stride", sp["bytes"])
        flat = self._bytes(sp[key], (h - 1) * st + w)
        return flat.as_strided((h, w), (st, 1))

    def exchange(self, b: int) -> None:
        s = self.solver
        spans = [sp for sp in s.halo_spans(0, b) if sp["peer"] >= 0]
        if not spans:
            return
        # pencils: the y faces first, then the z faces, which carry the y ghost rows just received
        # (the edge / corner cells of the 27-point stencil)
        for ph in ([sp for sp in spans if sp["side"] >= 2], [sp for sp in spans if sp["side"] < 2]):
            if ph:
                self._exchange_phase(ph)

    def _exchange_phase(self, spans) -> None:
        s = self.solver
        dev = s.device(0)
        if dev >= 0 and self.staged:
            self._exchange_staged(spans)
            return
        ctx = torch.cuda.stream(torch.cuda.ExternalStream(s.halo_stream(0))) if dev >= 0 else _null()
        with ctx:
            ops, unpack = [], []
            for sp in spans:
                send, recv = self._face(sp, "send"), self._face(sp, "recv")
                if not recv.is_contiguous():
                    tmp = torch.empty(recv.shape, dtype=recv.dtype, device=recv.device)
                    unpack.append((recv, tmp))
                    recv = tmp
                ops.append(dist.P2POp(dist.irecv, recv, sp["peer"], self.group))
                ops.append(dist.P2POp(dist.isend, send.contiguous(), sp["peer"], self.group))
            if dev >= 0:
                # one NCCL (= RCCL) group for all faces: no pairwise ordering hazards
                reqs = dist.batch_isend_irecv(ops)
            else:
                reqs = [op.op(op.tensor, op.peer, op.group) for op in ops]
            for r in reqs:
                r.wait()
            for dst, tmp in unpack:
                dst.copy_(tmp)

    def _exchange_staged(self, spans) -> None:
        s = self.solver
        hs = torch.cuda.ExternalStream(s.halo_stream(0))
        hs.synchronize()  # the boundary kernels that produced the faces are done
        sends, recvs, reqs = [], [], []
        for sp in spans:
            sends.append(self._face(sp, "send").cpu().contiguous())
            recvs.append(torch.empty((sp.get("height", 1), sp.get("width", sp["bytes"])), dtype=torch.uint8))
        for sp, snd, rcv in zip(spans, sends, recvs):
            reqs.append(dist.irecv(rcv, src=sp["peer"], group=self.group))
            reqs.append(dist.isend(snd, dst=sp["peer"], group=self.group))
        for r in reqs:
            r.wait()
        with torch.cuda.stream(hs):
            for sp, rcv in zip(spans, recvs):
                self._face(sp, "recv").copy_(rcv, non_blocking=False)
        hs.synchronize()

    def allreduce_sum(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return float(t.item())

    def allreduce_max(self, v: float) -> float:
        t = torch.tensor([v], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def barrier(self) -> None:
        dist.barrier(group=self.group)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
