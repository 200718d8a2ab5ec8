#!/usr/bin/env python3
"""A/B harness for the stencil kernels on one MI355X (cdna_hip_programming.md §5.4 rule 24:
variants interleaved in ONE process, several rounds, best and median reported).

Variants are the native dispatcher's kernel-family selectors (MDFX_TB_RY, MDFX_WTK_WB, MDFX_H7_WXK,
and MDFX_B27_WXK; cached by the native layer and re-read per variant) plus the kernel family (tuned / naive) and the fused depth. Every variant's output is first checked
bitwise against the naive kernel.

    python bench/kernel_ab.py --kind heat7 --n 1024 --variants "STEPS=4;STEPS=3;STEPS=3,WXK=0;STEPS=2"
"""

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import mpi_cuda_process_amd as m  # noqa: E402
from mpi_cuda_process_amd.ops import (FieldLayout, alloc_field, apply_stencil, init_field,  # noqa: E402
                                      set_kernel_variant)

KEYS = {"TBRY": "MDFX_TB_RY", "WB": "MDFX_WTK_WB", "WXK": "MDFX_H7_WXK", "B27WXK": "MDFX_B27_WXK"}


def parse_variant(s):
    fam, env, steps = "tuned", {}, 1
    for part in filter(None, s.split(",")):
        k, v = part.split("=")
        if k == "FAM":
            fam = v
        elif k == "STEPS":
            steps = int(v)
        else:
            env[KEYS[k]] = v
    return fam, env, steps


def apply_env(env):
    for k in KEYS.values():
        os.environ.pop(k, None)
    os.environ.update(env)
    m.native().reload_knobs()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--kind", default="heat7")
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--nx", type=int, default=0)
    p.add_argument("--ny", type=int, default=0)
    p.add_argument("--nz", type=int, default=0)
    p.add_argument("--dtype", default="f32")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--variants", default="FAM=naive;RY=4,PF=2")
    p.add_argument("--json", default="")
    p.add_argument("--thief", type=int, default=0,
                   help="launch this many single-block spin kernels (torch.cuda._sleep, ~--thief-us) on "
                        "side streams next to every timed launch: emulates the CUs RCCL's send/recv "
                        "kernels hold during an overlapped halo exchange")
    p.add_argument("--thief-us", type=float, default=100.0)
    a = p.parse_args()
    nx, ny, nz = a.nx or a.n, a.ny or a.n, a.nz or a.n
    if a.kind == "heat7":
        prob = m.heat3d(nx=nx, ny=ny, nz=nz, dtype=a.dtype)
    elif a.kind == "box27":
        prob = m.box27(nx=nx, ny=ny, nz=nz, dtype=a.dtype)
    elif a.kind == "jacobi5":
        prob = m.mdf2d(h=nz, w=nx, dtype=a.dtype)
    else:
        prob = m.life2d(h=nz, w=nx)
    variants = [v for v in a.variants.split(";") if v]
    max_steps = max(parse_variant(v)[2] for v in variants)
    lay = FieldLayout.make(prob, halo=max_steps)
    A = alloc_field(lay, "cuda")
    B = alloc_field(lay, "cuda")
    R = alloc_field(lay, "cuda")
    init_field(prob, lay, A)
    init_field(prob, lay, B)
    set_kernel_variant("naive")
    refs = {1: R}
    apply_stencil(prob, lay, A, R)
    if max_steps > 1:  # k naive single steps; the fused sweep must match them bitwise
        R2 = alloc_field(lay, "cuda")
        cur = R
        for k in range(2, max_steps + 1):
            nxt = alloc_field(lay, "cuda")
            nxt.copy_(cur)
            apply_stencil(prob, lay, cur, nxt)
            refs[k] = nxt
            cur = nxt
        del R2
    torch.cuda.synchronize()
    ok = {}
    for v in variants:
        fam, env, steps = parse_variant(v)
        apply_env(env)
        set_kernel_variant(fam)
        B.zero_()
        apply_stencil(prob, lay, A, B, steps=steps)
        torch.cuda.synchronize()
        ok[v] = bool(torch.equal(B[lay.owned, :, :nx], refs[steps][lay.owned, :, :nx]))
    thieves = [torch.cuda.Stream() for _ in range(a.thief)]
    thief_cycles = int(a.thief_us * 2.4e3)  # gfx950 shader clock ~2.4 GHz
    # copy roof with the same bytes (one read + one write of the field)
    times = {v: [] for v in variants}
    copy_t = []
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        e0.record()
        for i in range(a.iters):
            (B if i % 2 == 0 else A).copy_(A if i % 2 == 0 else B)
        e1.record()
        torch.cuda.synchronize()
        copy_t.append(e0.elapsed_time(e1) / a.iters)
        for v in variants:
            fam, env, steps = parse_variant(v)
            apply_env(env)
            set_kernel_variant(fam)
            # every variant starts from the same fresh grid: the sweeps run measurably slower on the
            # rough data of the first ~40 steps after a random init (a data-dependent clock), so a
            # variant timed right after the init would be penalised against the ones timed later
            init_field(prob, lay, A)
            apply_stencil(prob, lay, A, B, steps=steps)
            e0.record()
            for i in range(a.iters):
                if thieves:
                    ev = torch.cuda.Event()
                    ev.record()
                    for st in thieves:
                        st.wait_event(ev)
                        with torch.cuda.stream(st):
                            torch.cuda._sleep(thief_cycles)
                apply_stencil(prob, lay, A if i % 2 == 0 else B, B if i % 2 == 0 else A, steps=steps)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters / steps)  # per time step
    set_kernel_variant("auto")
    apply_env({})
    cells = prob.cells
    bpc = prob.bytes_per_cell_per_step
    cbest = min(copy_t)
    out = {"problem": prob.describe(), "copy_ms": cbest, "copy_TBps": lay.planes * lay.plane * (bpc // 2) * 2 / cbest / 1e9,
           "variants": []}
    print("(times are per time step; fused variants divide the sweep time by STEPS)")
    print("%-28s %9s %9s %10s %8s %s" % ("variant", "best ms", "med ms", "GCells/s", "%copy", "bitwise"))
    print("%-28s %9.4f %9s %10.1f %8s" % ("torch copy_ (roof)", cbest, "", cells / cbest / 1e6, "100"))
    for v in variants:
        b, md = min(times[v]), statistics.median(times[v])
        rec = {"variant": v, "best_ms": b, "median_ms": md, "gcells": cells / b / 1e6, "pct_copy": 100 * cbest / b,
               "bitwise_vs_naive": ok[v]}
        out["variants"].append(rec)
        print("%-28s %9.4f %9.4f %10.1f %8.1f %s" % (v, b, md, rec["gcells"], rec["pct_copy"], ok[v]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
