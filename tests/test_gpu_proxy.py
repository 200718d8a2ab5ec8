"""Rank proxy on ONE MI355X (bench.py --rank-proxy, csrc/comm/proxy_transport.cpp): one slab of an
N-way split runs the engine's real per-rank schedule with its halo exchange looped back through the
ipc mailbox copies and device counters. Its ghosts hold the slab's own faces instead of the
neighbours', so a plane is exact only if no wrong ghost value can reach it: after S steps, the
planes more than S away from a proxied boundary equal the full-grid run bitwise."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import mpi_cuda_process_amd as m  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _full(prob, steps, temporal):
    with m.Simulation(prob, device="hip", temporal=temporal) as sim:
        sim.init()
        sim.run(steps)
        return sim.gather()


@pytest.mark.parametrize("n,r,temporal,graph,transport,direct", [
    (2, 0, 1, False, "proxy", "1"), (2, 1, 3, True, "proxy", "1"), (4, 1, 3, False, "proxy", "1"),
    (4, 2, 2, True, "proxy", "1"), (8, 3, 3, True, "proxy", "1"), (8, 7, 3, False, "proxy", "1"),
    (8, 3, 4, True, "proxy", "0"), (4, 2, 4, True, "proxy_sdma", "1"), (4, 1, 2, False, "proxy_sdma", "0")])
def test_proxy_slab_matches_full_grid_away_from_boundaries(hip, monkeypatch, n, r, temporal, graph, transport,
                                                           direct):
    """(both ipc protocols: direct pulls / mailboxes; both copy engines: blit / SDMA)"""
    monkeypatch.setenv("MDFX_IPC_DIRECT", direct)
    prob = m.heat3d(nx=1024 if temporal >= 3 else 256, ny=24, nz=36 * n)
    steps = 2 * temporal  # at least one replayed 2-sweep cycle at the full depth
    full = _full(prob, steps, temporal)
    with m.Simulation(prob, device="hip", ranks=n, proxy_rank=r, temporal=temporal, graph=graph,
                      transport=transport) as sim:
        assert sim.transport == "proxy"
        sim.init()
        sim.prepare_graphs()
        sim.run(steps)
        got = sim.read_local(0)
        lay = sim.layout(0)
        if graph:
            assert sim.graph_replays >= 1
    z0, z1 = lay["z0"], lay["z1"]
    lo = steps if r > 0 else 0          # planes a wrong lo ghost may have reached
    hi = steps if r < n - 1 else 0
    assert np.array_equal(got[lo:(z1 - z0) - hi], full[z0 + lo:z1 - hi])


@pytest.mark.parametrize("n,py,r,temporal,graph", [(8, 2, 3, 4, True), (8, 2, 4, 3, False), (8, 4, 5, 4, True),
                                                    (4, 2, 0, 3, False)])
def test_proxy_pencil_matches_full_grid_away_from_boundaries(hip, n, py, r, temporal, graph):
    """A (z, y) pencil of a pz x py split (4 x 2, 2 x 4, 2 x 2) looped back: the y faces as 2-D
    copies, then the z faces after the readyZ signal; exact wherever no proxied ghost can reach."""
    from mpi_cuda_process_amd.parallel.decomp import pencil_neighbors

    prob = m.heat3d(nx=1024 if temporal >= 3 else 256, ny=40 * py, nz=36 * (n // py))
    steps = 2 * temporal  # one replayed 2-sweep cycle at the full depth
    full = _full(prob, steps, temporal)
    with m.Simulation(prob, device="hip", ranks=n, proxy_rank=r, temporal=temporal, graph=graph, py=py) as sim:
        sim.init()
        sim.prepare_graphs()
        sim.run(steps)
        got = sim.read_local(0)
        lay = sim.layout(0)
        if graph:
            assert sim.graph_replays >= 1
    zl, zh, yl, yh = (steps if q >= 0 else 0 for q in pencil_neighbors(r, n // py, py))
    z0, z1, y0, y1 = lay["z0"], lay["z1"], lay["y0"], lay["y1"]
    assert got.shape == (z1 - z0, y1 - y0, prob.nx)
    assert np.array_equal(got[zl:(z1 - z0) - zh, yl:(y1 - y0) - yh], full[z0 + zl:z1 - zh, y0 + yl:y1 - yh])


def test_bench_rank_proxy_json(hip):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rank-proxy", "4", "--n", "256",
                        "--steps", "6", "--warmup", "3"], capture_output=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr.decode()
    rec = json.loads([l for l in p.stdout.decode().splitlines() if l.startswith("{")][0])
    assert rec["proxy"] is True and "PROXY" in rec["metric"] and rec["proxied_n_gpus"] == 4
    assert rec["proxy_rank"] == 2 and rec["config"]["slab_planes"] == [128, 192]
    assert rec["implied_node_gcells"] == pytest.approx(4 * rec["value"], rel=1e-3)
    assert rec["config"]["graph_captures_timed"] == 0


def test_replayed_cycles_run_as_fast_as_eager_steps_after_reinit(hip):
    """Round 3's slow graph replay (N = 8 proxy, K = 2, 2 rounds: 2.5x the eager time per step
    after init() on a used engine and three replayed warm-up cycles). Its cause: the block-round
    count was a process-wide setting that only run() updated, so cycles captured by
    prepare_graphs() after set_options(min_rounds=...) replayed the previous configuration's
    launch geometry (1-round sweeps under the overlapped schedule). The round count now travels
    with every launch (RegionArgs::min_rounds): the replay must stay within 1.2x the eager steps."""
    import time

    import torch

    prob = m.heat3d(n=1024)
    steps = 48

    def ms_per_step(sim):
        sim.synchronize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.run(steps)
        sim.synchronize()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    with m.Simulation(prob, device="hip", ranks=8, proxy_rank=4, temporal=2, graph=True) as sim:
        # a used engine: other round counts captured and run first (the trial loop's history)
        for rr in (1, 2, 1):
            sim.set_options(graph=True, min_rounds=rr, overlap=True)
            sim.init()
            sim.prepare_graphs()
            sim.run(12)
        sim.set_options(graph=False, min_rounds=2, overlap=True)
        sim.init()
        sim.run(12)
        eager = min(ms_per_step(sim) for _ in range(2))
        sim.set_options(graph=True, min_rounds=2, overlap=True)
        sim.init()
        sim.prepare_graphs()
        sim.run(12)  # three replayed warm-up cycles (2 sweeps of 2 steps each)
        r0 = sim.graph_replays
        replay = min(ms_per_step(sim) for _ in range(2))
        assert sim.graph_replays > r0
    assert replay <= 1.2 * eager, (replay, eager)
