#!/usr/bin/env python3
"""Per-kernel register / LDS / scratch table of the gfx950 code objects inside libmdfx.so.

The code objects are unbundled with llvm-objdump --offloading (in a scratch directory) and their
AMDHSA metadata notes are parsed with llvm-readelf --notes. No GPU is needed.

    python scripts/kernel_resources.py [--lib PATH] [--json OUT]

Occupancy (waves per SIMD) follows the gfx950 rule: 512 VGPRs (arch + acc) per SIMD lane,
allocated in granules of 8, at most 8 waves.
"""

import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "private_segment_fixed_size", "group_segment_fixed_size", "max_flat_workgroup_size")


def _demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), stdout=subprocess.PIPE, text=True,
                             check=True).stdout.splitlines()
        return out if len(out) == len(names) else names
    except (OSError, subprocess.CalledProcessError):
        return names


def occupancy(vgpr, agpr):
    regs = max(8, ((vgpr + 7) // 8) * 8 + ((agpr + 7) // 8) * 8)
    return min(8, 512 // regs)


def kernel_resources(lib=None):
    """List of dicts, one per kernel in every gfx950 code object of `lib`."""
    lib = lib or os.path.join(ROOT, "mpi_cuda_process_amd", "lib", "libmdfx.so")
    tmp = tempfile.mkdtemp(prefix="mdfx_co_")
    try:
        local = os.path.join(tmp, os.path.basename(lib))
        shutil.copy(lib, local)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        kernels = {}
        for f in sorted(os.listdir(tmp)):
            if "gfx950" not in f:
                continue
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", os.path.join(tmp, f)],
                                   stdout=subprocess.PIPE, text=True, check=True).stdout
            # one kernel per "  - .agpr_count:" item of amdhsa.kernels; keys at 4 spaces of indent
            for block in re.split(r"\n  - (?=\.agpr_count:)", notes)[1:]:
                rec = {"agpr_count": int(re.match(r"\.agpr_count:\s+(\d+)", block).group(1))}
                for m in re.finditer(r"^    \.([a-z_]+):\s+(\S+)$", block, re.M):
                    k, v = m.group(1), m.group(2)
                    if k in FIELDS:
                        rec[k] = int(v)
                    elif k == "name":
                        rec["mangled"] = v
                if "mangled" in rec:
                    kernels[rec["mangled"]] = rec
        recs = list(kernels.values())
        for r, d in zip(recs, _demangle([r["mangled"] for r in recs])):
            r["name"] = d
            r["waves_per_simd"] = occupancy(r.get("vgpr_count", 0), r.get("agpr_count", 0))
        return sorted(recs, key=lambda r: r["name"])
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def kernel_isa(lib, mangled_prefix):
    """Disassembly lines (instructions only) of the kernels whose mangled name starts with
    `mangled_prefix`, keyed by mangled name."""
    tmp = tempfile.mkdtemp(prefix="mdfx_isa_")
    try:
        local = os.path.join(tmp, os.path.basename(lib))
        shutil.copy(lib, local)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=tmp, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        out = {}
        for f in sorted(os.listdir(tmp)):
            if "gfx950" not in f:
                continue
            path = os.path.join(tmp, f)
            syms = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-s", path], stdout=subprocess.PIPE,
                                  text=True, check=True).stdout
            if mangled_prefix not in syms:
                continue
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", path], stdout=subprocess.PIPE,
                                 text=True, check=True).stdout
            cur = None
            for line in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
                if m:
                    cur = m.group(1) if m.group(1).startswith(mangled_prefix) else None
                    if cur:
                        out[cur] = []
                    continue
                if cur and line.strip():
                    out[cur].append(line.split("//")[0].strip())
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--lib", default=None)
    p.add_argument("--json", default="")
    a = p.parse_args()
    recs = kernel_resources(a.lib)
    print("%-6s %-6s %-6s %-6s %-8s %-6s %-5s  %s" % ("VGPR", "AGPR", "SGPR", "sspill", "scratch", "LDS", "occ",
                                                    "kernel"))
    for r in recs:
        print("%-6d %-6d %-6d %-6d %-8d %-6d %-5d  %s" % (r.get("vgpr_count", 0), r.get("agpr_count", 0),
                                                   r.get("sgpr_count", 0), r.get("sgpr_spill_count", 0),
                                                   r.get("private_segment_fixed_size", 0),
                                                   r.get("group_segment_fixed_size", 0), r["waves_per_simd"],
                                                   r["name"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(recs, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
