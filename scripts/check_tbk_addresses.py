#!/usr/bin/env python3
"""Host-side emulation of heat7_tbk's global address arithmetic (DMA rows, DMA seams, stores) for
every block, lane, row and plane of a launch, checked against the allocation. box27_tbk uses the
same addressing (K = 2, RY 1 / 2 / 4), so its GPU test shapes are checked here too. Run before taking a
changed kernel to the GPU: an out-of-bounds index here would be an illegal access there.

    python scripts/check_tbk_addresses.py      # the GPU test shapes + the bench shapes
"""
import sys

import numpy as np

SLACK_BYTES = 1024


def layout(nx, ny, nz, esize, halo):
    align = 256 // esize
    pitch = (nx + align - 1) // align * align
    plane = pitch * ny
    lz_max = nz + 2 * halo
    return pitch, plane, lz_max, lz_max * plane + SLACK_BYTES // esize


def tbk_zc(planes, tiles, resident):
    per_slot = planes * tiles / resident
    rounds = max(1, min(4, int(per_slot / 128.0 + 0.5)))
    zt = max(1, min(planes, (rounds * resident + tiles // 2) // tiles))
    return (planes + zt - 1) // zt


def check(nx, ny, nz, dtype, K, RY, lz_begin=None, lz_end=None, resident=512):
    esize = 4 if dtype == "f32" else 8
    N = 16 // esize
    WX = 64 * N
    pitch, plane, lz_max, alloc = layout(nx, ny, nz, esize, K)
    lzb = K if lz_begin is None else lz_begin
    lze = K + nz if lz_end is None else lz_end
    XT = pitch > 4 * WX  # x tiles of 4 waves (two fused steps only)
    assert not XT or K == 2, "rows wider than one block need two fused steps"
    WXN = 4 if pitch > 2 * WX else 2 if pitch > WX else 1
    WYN = 4 // WXN
    XTn = (pitch + 4 * WX - 1) // (4 * WX) if XT else 1
    if ny < 8:
        RY = 1
    R0 = RY + 2 * K
    planes = lze - lzb
    YT = (ny + WYN * RY - 1) // (WYN * RY)
    zc = tbk_zc(planes, XTn * YT, resident)
    ZT = (planes + zc - 1) // zc
    lane = np.arange(64)
    bad = 0
    for xt, yt in ((a, b) for a in range(XTn) for b in range(YT)):
        for zt in range(ZT):
            zs = lzb + zt * zc
            ze = min(lze, zs + zc)
            for w in range(4):
                wx, wy = w % WXN, w // WXN
                xw = xt * WXN * WX + wx * WX
                x = xw + lane * N
                xin = x < pitch
                y0 = (yt * WYN + wy) * RY
                xcol = np.where(xin, x, pitch - N)                      # xcb / esize
                has_l, has_r = 0 < xw < pitch, xw + WX < pitch
                srow = lane & 31
                son = np.where(lane < 32, has_l & (srow < R0), (WXN > 1) & has_r & (srow < R0))
                scol = np.where(son, np.where(lane < 32, xw - N, xw + WX), xcol)
                assert (xcol >= 0).all() and (scol >= 0).all(), "negative 32-bit lane offset"
                assert (xcol * esize < 2 ** 32).all()

                def rowc(k):
                    y = y0 - K + k
                    return min(max(y, 0), ny - 1)
                # addresses are lz * plane + (row, lane) terms: the extreme planes bound them all
                for lz in sorted({zs - K, ze + K - 1}):
                    if lz < 0 or lz >= lz_max:
                        bad += 1
                        continue
                    for k in range(R0):
                        a = lz * plane + rowc(k) * pitch + xcol
                        bad += int(((a < 0) | (a + N > alloc)).sum())
                    if WXN > 1:
                        sr = np.array([rowc(int(r)) if r < R0 else rowc(0) for r in srow])
                        a = lz * plane + sr * pitch + scol
                        bad += int(((a < 0) | (a + N > alloc)).sum())
                for lz in sorted({zs, ze - 1}):
                    for i in range(RY):
                        if y0 + i < ny:
                            a = lz * plane + (y0 + i) * pitch + x[xin]
                            bad += int(((a < 0) | (a + N > alloc)).sum())
    return bad, dict(pitch=pitch, WXN=WXN, XTn=XTn, YT=YT, zc=zc, ZT=ZT)


SHAPES = [(1024, 37, 23, "f32"), (700, 19, 15, "f32"), (256, 9, 12, "f32"), (500, 21, 11, "f64"),
          (64, 64, 9, "f32"), (1000, 5, 14, "f32"), (300, 40, 10, "f64"), (1024, 20, 40, "f32"),
          (512, 32, 33, "f64")]
# box27_tbk's GPU test shapes (two fused steps only)
BOX27 = [(1024, 11, 9, "f32"), (512, 21, 15, "f32"), (300, 9, 12, "f64"), (64, 40, 10, "f32"),
         (500, 30, 13, "f64"), (200, 5, 9, "f32"), (512, 512, 512, "f64")]
# rows wider than one block (x tiles, K = 2): the GPU test shapes
WIDE = [(2048, 13, 11, "f32"), (1100, 9, 9, "f64"), (1030, 7, 8, "f32"), (2048, 21, 12, "f64"),
        (1300, 17, 10, "f32")]


def main():
    fails = 0
    cases = [(s, K, RY) for s in SHAPES for K, rys in ((2, (1, 2, 3, 4)), (3, (1, 2, 3)), (4, (1, 2)))
             for RY in rys]
    cases += [(s, 2, RY) for s in WIDE for RY in (1, 2, 3, 4)]
    cases += [(s, 2, RY) for s in BOX27 for RY in (1, 2, 4)]
    for (nx, ny, nz, dt), K, RY in cases:
        bad, info = check(nx, ny, nz, dt, K, RY)
        fails += bad > 0
        if bad:
            print("OUT OF BOUNDS", nx, ny, nz, dt, "K", K, "RY", RY, bad, info)
    print("checked %d shapes x depths: %s" % (len(SHAPES) + len(WIDE) + len(BOX27),
                                              "FAIL" if fails else "all accesses in bounds"))
    return 1 if fails else 0


if __name__ == "__main__":
    sys.exit(main())
