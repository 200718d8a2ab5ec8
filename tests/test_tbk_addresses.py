"""Host emulation of the streaming 3D kernel's global address arithmetic (scripts/
check_tbk_addresses.py): every DMA row / seam / store of every block, lane and plane stays inside
the allocation, for the GPU test shapes and every fused depth / tile height. Runs on the CPU, so an
addressing change is caught before it can fault a GPU."""

import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))

import check_tbk_addresses as c  # noqa: E402


def test_all_tbk_accesses_in_bounds():
    assert c.main() == 0


def test_checker_sees_a_wrapped_offset():
    # the bug this guards against: a negative per-lane column for a wave beyond the row pitch
    bad, info = c.check(700, 19, 15, "f32", 2, 2)
    assert bad == 0 and info["WXN"] == 4 and info["pitch"] < 4 * 256
