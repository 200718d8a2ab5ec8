"""High-level simulation API over the native engine (``mdfx::Solver``).

:class:`Simulation` owns one native solver and picks the device backend and the halo transport:

=================  ==============================================================================
mode               slabs / transport
=================  ==============================================================================
single             1 slab (P = 1), no exchange
virtual            P slabs in this process: ``host`` (CPU memcpy) or ``loopback`` (HIP D2D / peer
                   copies, possibly over several GPUs) — how multi-rank runs are tested on one GPU
distributed        one slab per torch.distributed rank (torchrun / mpirun): ``rccl`` (native
                   ncclSend/ncclRecv on the engine's halo stream, unique id broadcast over the
                   control group), ``ipc`` (native: faces pulled from the neighbours' buffers
                   mapped through HIP IPC, ordered by device counters; any number of processes
                   per GPU), or ``torch`` / ``staged`` (torch.distributed p2p through a callback:
                   gloo on CPU, nccl = RCCL on GPU, or host-staged gloo)
=================  ==============================================================================

Reference parity: the reference's ``main`` (MDF_kernel.cu:101-236 / kernel.cu:148-283) is this
object with P = 2 fixed, MPI host-staged halos, and no swap.
"""

from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from ._native import hip_available, native
from .models import InitCondition, Problem
from .ops import TORCH_DTYPE
from .parallel.decomp import slab_bounds
from .parallel.dist import ControlPlane, TorchP2PTransport, broadcast_bytes, group_for, is_distributed


def auto_temporal(problem: Problem, nranks: int, device: str, py: int = 1, residual_every: int = 0) -> int:
    """Fused steps per sweep chosen like the CLIs' auto mode: the deepest fused kernel that exists on
    this device (``hip_fused_depth``: 5 for the fp32 3D 7-point through heat7_wxk, fp64 5 from rows of 2048 cells and 4 below, 3 for the 27-point in fp64 or at rows of 1024+ cells, else 2 for the 3D stencils,
    8 for the 2D MDF, 12 for Life), made shallower until every slab is at least 4 sweeps
    deep; 1 on the CPU, where fused sweeps bring nothing."""
    if device != "hip":
        return 1
    if py > 1:
        # pencils: the fused 7-point sweep (heat7_wxk, K = 4) is the one that takes y ghost rows;
        # the other stencils step singly
        if problem.kind != "heat7":
            return 1
        want = 4
        pz = nranks // py
        return want if problem.nz >= 4 * want * pz and problem.ny >= 4 * want * py else 1
    want = native().hip_fused_depth(problem.kind, problem.dtype, problem.nx, problem.ref_precision)
    while want > 1 and problem.nz < 4 * want * nranks:
        want = {5: 4, 3: 2}.get(want, want // 2)
    if want > 1 and native().hip_supports_steps(problem.kind, problem.dtype, problem.nx, problem.ny, problem.nz,
                                                want, want, problem.ref_precision):
        # the depth for the residual interval (native interval_depth: least plan cost on one rank,
        # whole sweeps of the depth with several)
        return native().hip_auto_depth(problem.kind, problem.dtype, problem.nx, problem.ny, problem.nz, want,
                                       residual_every, problem.ref_precision, nranks)
    return 1


class Simulation:
    """One decomposed stencil simulation driven by the native engine.

    Parameters: ``device`` hip | cpu | auto; ``ranks`` P virtual slabs in this process (default:
    one per distributed rank, or 1); ``devices`` GPU ids for the local slabs; ``transport`` auto |
    rccl | rccl_fold (rccl with the folded lower boundary) | ipc | ipc_sdma | torch | staged |
    loopback | host; ``overlap`` interior sweep concurrent with boundary
    planes + exchange; ``sync_debug`` serialise every phase (race screen); ``residual_every`` k:
    global L2 norm of the update every k steps (NaN/Inf guard); ``graph`` replay two-sweep cycles
    as hipGraphs; ``timeout_s`` watchdog; ``temporal`` fused steps per sweep (1 = none, 0 = auto,
    see :func:`auto_temporal`; halo planes = temporal); ``share_gpu`` let several engine processes
    use one GPU with the ipc transport (tests only: its device spin waits assume one process per
    GPU, native ipc_shared_gpu_problem).
    """

    def __init__(self, problem: Problem, *, device: str = "auto", ranks: Optional[int] = None,
                 devices: Optional[Sequence[int]] = None, transport: str = "auto",
                 distributed: Optional[bool] = None, overlap: bool = True, sync_debug: bool = False,
                 residual_every: int = 0, graph: bool = False, timeout_s: float = 0.0,
                 temporal: int = 1, group=None, proxy_rank: Optional[int] = None, py: int = 1,
                 share_gpu: bool = False):
        self.problem = problem
        if device == "auto":
            device = "hip" if hip_available() else "cpu"
        if device not in ("hip", "cpu"):
            raise ValueError("device must be 'hip', 'cpu' or 'auto'")
        self.device = device
        if distributed is None:
            distributed = is_distributed() and ranks is None
        self.distributed = bool(distributed)
        self._torch_transport = None
        self._control = None  # host control plane of the ipc transport (teardown barrier)
        self.group = group

        fold_req = None
        if transport == "rccl_fold":
            # rccl with the folded lower boundary (not rccl's default: Transport::fold_by_default)
            transport, fold_req = "rccl", 1
        if self.distributed:
            if transport in ("rccl", "ipc", "ipc_sdma") and device != "hip":
                raise ValueError("%s transport needs HIP devices" % transport)
            world = dist.get_world_size(group)
            rank = dist.get_rank(group)
            nranks, local_ranks = world, [rank]
            if device == "hip":
                ndev = torch.cuda.device_count()
                local = int(__import__("os").environ.get("LOCAL_RANK", rank))
                dev_list = [devices[0] if devices else local % ndev]
            else:
                dev_list = [-1]
            if transport == "auto":
                transport = "rccl" if device == "hip" else "torch"
            if transport == "rccl":
                if device != "hip":
                    raise ValueError("rccl transport needs HIP devices")
                torch.cuda.set_device(dev_list[0])
                uid = native().rccl_unique_id() if rank == 0 else None
                uid = broadcast_bytes(uid, src=0, group=group)
                args = dict(transport="rccl", unique_id=uid)
            elif transport in ("ipc", "ipc_sdma"):
                # ipc: faces pulled by the runtime's blit kernels; ipc_sdma: by the SDMA engines
                if device != "hip":
                    raise ValueError("ipc transport needs HIP devices")
                torch.cuda.set_device(dev_list[0])
                self._control = ControlPlane(group, timeout_s=max(60.0, 2 * timeout_s))
                args = dict(transport=transport, callbacks=self._control.callbacks())
            elif transport in ("torch", "staged"):
                p2p_group = group
                staged = transport == "staged" and device == "hip"
                if device == "hip":
                    torch.cuda.set_device(dev_list[0])
                    if not staged:
                        p2p_group = group_for("nccl", group, max(60.0, 2 * timeout_s)) if group is None else group
                self._torch_transport = TorchP2PTransport(p2p_group, staged=staged)
                args = dict(transport="callback", callbacks=self._torch_transport.callbacks())
            else:
                raise ValueError("distributed transport must be rccl|ipc|ipc_sdma|torch|staged|auto")
        elif proxy_rank is not None:
            # rank proxy: only slab `proxy_rank` of a `ranks`-way split, on one GPU, its halo
            # exchange looped back through the ipc mailbox machinery (proxy_transport.cpp)
            if device != "hip":
                raise ValueError("the rank proxy needs a HIP device")
            nranks = int(ranks or 1)
            if not 0 <= proxy_rank < nranks:
                raise ValueError("proxy_rank must be in [0, ranks)")
            local_ranks = [int(proxy_rank)]
            dev_list = [devices[0] if devices else torch.cuda.current_device()]
            # proxy_sdma: the face copies on the SDMA engines (the ipc_sdma transport's exchange)
            if transport not in ("auto", "proxy", "proxy_sdma"):
                raise ValueError("the rank proxy's transport is proxy or proxy_sdma")
            args = dict(transport="proxy_sdma" if transport == "proxy_sdma" else "proxy")
        else:
            nranks = ranks or 1
            local_ranks = list(range(nranks))
            if device == "hip":
                dev_list = list(devices) if devices else [torch.cuda.current_device()]
                if len(dev_list) == 1:
                    dev_list = dev_list * nranks
                if len(dev_list) != nranks:
                    raise ValueError("devices must list one device per rank")
            else:
                dev_list = [-1] * nranks
            if transport == "auto":
                transport = "loopback" if device == "hip" else "host"
            if transport not in ("loopback", "host", "rccl"):
                raise ValueError("in-process transport must be loopback|host|rccl")
            args = dict(transport=transport)
            if transport == "rccl":  # one process driving several GPUs
                args["unique_id"] = native().rccl_unique_id()

        self.nranks = nranks
        self.py = int(py)
        if temporal <= 0:
            temporal = auto_temporal(problem, nranks, device, int(py), int(residual_every))
        self._s = native().Solver(problem.kind, problem.dtype, problem.nx, problem.ny, problem.nz,
                                  nranks, local_ranks, dev_list, overlap=overlap,
                                  sync_debug=sync_debug, residual_every=residual_every, graph=graph,
                                  timeout_s=timeout_s, temporal=temporal, py=int(py), share_gpu=bool(share_gpu),
                                  **problem.coef_kwargs(), **args)
        if self._torch_transport is not None:
            self._torch_transport.solver = self._s
        self.transport = self._s.transport_name if self._torch_transport is None else "torch"
        if fold_req is not None:
            self._s.set_options(fold=fold_req)
            self.transport = "rccl_fold"
        self.bounds = slab_bounds(problem.nz, nranks // max(1, self.py))

    # ---- lifecycle -------------------------------------------------------------------------
    def close(self):
        if self._s is not None:
            if self._control is not None:
                # ipc: a neighbour may still be pulling this process's last faces out of its
                # exported mailbox; every rank drains its own streams, then all meet, then free
                try:
                    self._s.synchronize()
                    self._control.barrier()
                except Exception:  # noqa: BLE001 - a failed peer / poisoned engine: free anyway
                    pass
            self._s.close()
            self._s = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
        return False

    @property
    def native(self):
        return self._s

    # ---- state -----------------------------------------------------------------------------
    def init(self, init: Optional[InitCondition] = None) -> "Simulation":
        ic = init or self.problem.init
        if ic.kind == "compat":
            # reference GoL grid: glibc rand() Bernoulli(density) in global row-major order
            g = native().life_compat_init(self.problem.nz, self.problem.nx, ic.density, ic.seed)
            self._s.init("constant", value=0.0)
            for i in range(self._s.num_local):
                lay = self._s.layout(i)
                self._s.write_owned(i, np.ascontiguousarray(g[lay["z0"]:lay["z1"]]).reshape(-1, 1, self.problem.nx))
            return self
        self._s.init(ic.kind, seed=ic.seed, lo=ic.lo, hi=ic.hi, value=ic.value, edge=ic.edge,
                     interior=ic.interior, density=ic.density)
        return self

    def run(self, steps: int) -> "Simulation":
        self._s.run(int(steps))
        return self

    def synchronize(self):
        self._s.synchronize()

    def set_options(self, **kw):
        """Change run options (overlap, sync_debug, residual_every, graph, timeout_s, profile,
        min_rounds, fold: -1 the transport's default, 0 never, 1 where possible); options not named
        keep their values."""
        self._s.set_options(**kw)

    def warm_kernels(self, steps: int) -> None:
        """Launch every kernel instance that run(steps) would use once (each fused depth, the
        residual copy included) into the scratch buffer, without exchanges, and synchronize: the
        one-time costs of a first launch stay out of a timed run. The field state is unchanged."""
        self._s.warm_kernels(int(steps))

    def sweep_plan(self, steps: int) -> list:
        """The sweeps run(steps) would issue from the current step: a list of (fused depth,
        residual sweep). Each stretch up to a residual step (or the end) runs sweeps of the full
        depth and a tail cut by the measured cost of each fused depth (on the GPU, 10 steps at
        temporal 4 on 1024-cell rows: 4, 3, 3); the residual is evaluated by the last sweep."""
        return [(int(k), bool(r)) for k, r in self._s.sweep_plan(int(steps))]

    def prepare_graphs(self) -> int:
        """Capture the hipGraph cycles of both buffer parities now (graph=True and capturable), so
        that later run() calls only replay them: benchmarks call this before their warmup so no
        capture or instantiation lands in a timed region. init() keeps the captured cycles. Returns
        the number of cycles held (0: graphs off or not capturable in this configuration)."""
        return int(self._s.prepare_graphs())

    @property
    def graph_captures(self) -> int:
        """hipGraph cycles captured and instantiated so far (prepare_graphs() or on demand in run())."""
        return int(self._s.graph_captures)

    @property
    def folded_sweeps(self) -> int:
        """Eager sweeps whose lower boundary region ran inside the interior sweep (schedule 'folded')."""
        return int(self._s.folded_sweeps)

    @property
    def graph_wait_nodes(self) -> tuple:
        """(device spin-wait nodes in the captured graphs, those among them waiting on a slab's own
        fold counters). The second is 0 by construction: captured cycles never fold."""
        return int(self._s.graph_wait_nodes), int(self._s.graph_fold_waits)

    @property
    def graph_eligible(self) -> bool:
        """Whether run() replays captured cycles in the current configuration."""
        return bool(self._s.graph_eligible)

    @property
    def schedule(self) -> str:
        """The per-step schedule eager steps run: 'serialised', 'two-stream', 'boundary-on-compute'
        or 'folded' (native step_schedule; docs/DESIGN.md §3)."""
        return str(self._s.schedule)

    @property
    def graph_replays(self) -> int:
        """2-sweep cycles replayed from a captured hipGraph so far (0: every step ran eagerly, e.g.
        graph replay off or not capturable under this HIP runtime)."""
        return self._s.graph_replays

    @property
    def options(self) -> dict:
        from . import GRAPH_QUEUES

        d = dict(self._s.options())
        d["graph_queues"] = GRAPH_QUEUES  # whether hipGraph replay runs on one hardware queue (__init__.py)
        return d

    @property
    def temporal(self) -> int:
        return self._s.temporal

    @property
    def steps(self) -> int:
        return self._s.steps

    @property
    def residual(self) -> float:
        return self._s.residual

    @property
    def num_local(self) -> int:
        return self._s.num_local

    def layout(self, i: int = 0) -> dict:
        return self._s.layout(i)

    def read_local(self, i: int = 0) -> np.ndarray:
        """Owned cells of local part i as a dense (nzl, nyl, nx) numpy array (nyl = ny for slabs)."""
        return self._s.read_owned(i)

    def write_local(self, i: int, a: np.ndarray):
        self._s.write_owned(i, np.ascontiguousarray(a))

    def view(self, i: int = 0, current: bool = True) -> torch.Tensor:
        """Zero-copy torch view (planes, rows, pitch) of a part's buffer (ghost planes and, for
        pencils, ghost rows included)."""
        b = self._s.current_index if current else 1 - self._s.current_index
        t = torch.from_dlpack(self._s.view(i, b))
        t._mdfx_owner = self  # keep the engine alive while the view is
        return t

    def gather(self) -> np.ndarray:
        """The whole global grid (nz, ny, nx) as numpy, on every caller.

        Each part lands at its (z0:z1, y0:y1) block, so slabs and pencils gather alike. In-process:
        the local parts; distributed: all_gather_object over the control group (debug / test sized
        grids only).
        """
        parts = []
        for i in range(self.num_local):
            lay = self._s.layout(i)
            parts.append((lay["z0"], lay["z1"], lay["y0"], lay["y1"], self.read_local(i)))
        if self.distributed:
            allp: List = [None] * dist.get_world_size(self.group)
            dist.all_gather_object(allp, parts[0], group=self.group)
            parts = allp
        p = self.problem
        out = np.empty((p.nz, p.ny, p.nx), dtype=parts[0][4].dtype)
        for z0, z1, y0, y1, a in parts:
            out[z0:z1, y0:y1] = a
        return out

    def save_checkpoint(self, path: str):
        self._s.save_checkpoint(path)

    def load_checkpoint(self, path: str):
        self._s.load_checkpoint(path)

    @property
    def torch_dtype(self):
        return TORCH_DTYPE[self.problem.dtype]


__all__ = ["Simulation"]
