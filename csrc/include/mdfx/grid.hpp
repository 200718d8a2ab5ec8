// mdfx — field layout, 1-D slab and 2-D (z, y) pencil decompositions.
//
// Reference parity: the reference replicates the whole h*w grid on every rank, host and device
// (MDF_kernel.cu:137-144), indexes it with 32-bit ints and __mul24 (D16) and splits it
// at exactly size/2 between two hard-coded ranks (MDF_kernel.cu:30,38,54,62, D15). Here each rank
// stores only its subdomain plus `halo` ghost planes per side (and, split in y as well, `hy` ghost
// rows per side), every index is 64-bit, and the split works for any P <= nz with an uneven
// remainder.
#pragma once

#include <vector>

#include "mdfx/common.hpp"

namespace mdfx {

// Row pitch alignment in bytes: rows start 256-B aligned so every lane's 16-B vector access is
// naturally aligned and a wave's 1 KiB row segment never splits a 128-B line unevenly.
constexpr int64_t kRowAlignBytes = 256;
// Extra bytes after the last plane so a vector kernel's right-neighbour read of the final row
// never leaves the allocation.
constexpr int64_t kSlackBytes = 1024;

struct FieldLayout {
  Extent3 global;      // global grid (2D kinds: nx = w, ny = 1, nz = h)
  int64_t z0 = 0;      // first owned global plane
  int64_t z1 = 0;      // one past the last owned global plane
  int halo = 1;        // ghost planes on each side
  int64_t y0 = 0;      // first owned global row (a pencil decomposition splits y as well)
  int64_t y1 = 0;      // one past the last owned global row
  int hy = 0;          // ghost rows on each side (0 for slabs: every row is owned)
  DType dtype = DType::F32;
  int64_t pitch = 0;   // elements per row (>= nx)
  int64_t plane = 0;   // elements per plane = pitch * rows()

  // y1 < 0: every row (a slab)
  static FieldLayout make(Extent3 g, int64_t z0, int64_t z1, int halo, DType dt, int64_t y0 = 0, int64_t y1 = -1,
                          int hy = 0);

  size_t esize() const { return dtype_size(dtype); }
  int64_t nzl() const { return z1 - z0; }
  int64_t nyl() const { return y1 - y0; }
  int64_t rows() const { return nyl() + 2 * hy; }  // storage rows per plane
  bool pencil() const { return hy > 0 || nyl() != global.ny; }
  int64_t planes() const { return nzl() + 2 * halo; }
  int64_t elems() const { return planes() * plane; }
  size_t bytes() const { return (size_t)elems() * esize() + kSlackBytes; }
  // storage plane index of a global plane
  int64_t lz(int64_t gz) const { return gz - z0 + halo; }
  // global plane of a storage plane index
  int64_t gz(int64_t lz) const { return lz - halo + z0; }
  // storage row of a global row, and back
  int64_t ly(int64_t gy) const { return gy - y0 + hy; }
  int64_t gy(int64_t ly) const { return ly - hy + y0; }
  int64_t offset(int64_t x, int64_t y, int64_t lzi) const { return lzi * plane + y * pitch + x; }
  size_t plane_bytes() const { return (size_t)plane * esize(); }
  // owned cells (what a rank contributes to GCells/s)
  int64_t owned_cells() const { return global.nx * nyl() * nzl(); }
};

// 1-D slab decomposition along the slowest axis (z; rows for 2D grids).
struct SlabDecomposition {
  int64_t nz = 0;
  int parts = 1;

  SlabDecomposition() = default;
  SlabDecomposition(int64_t nz_, int parts_);
  int64_t z0(int p) const;
  int64_t z1(int p) const { return z0(p + 1); }
  int64_t size(int p) const { return z1(p) - z0(p); }
  int lo_neighbor(int p) const { return p > 0 ? p - 1 : -1; }
  int hi_neighbor(int p) const { return p + 1 < parts ? p + 1 : -1; }
  int owner(int64_t gz) const;
};

// 2-D (z, y) pencil decomposition: pz slabs along z, each split into py pencils along y. Rank
// r = rz * py + ry owns planes [z0(rz), z1(rz)) and rows [y0(ry), y1(ry)). Its z neighbours are
// r -+ py, its y neighbours r -+ 1 inside the same slab. py = 1 is the slab decomposition.
// (MI355X: a slab's halo traffic rides the two xGMI links to its z neighbours only; a pencil's
// spreads over up to four links with half the z-face bytes at py = 2, docs/DESIGN.md §3.)
struct PencilDecomposition {
  SlabDecomposition z, y;
  PencilDecomposition() = default;
  PencilDecomposition(Extent3 g, int pz, int py) : z(g.nz, pz), y(g.ny, py) {}
  int pz() const { return z.parts; }
  int py() const { return y.parts; }
  int ranks() const { return pz() * py(); }
  int rz(int r) const { return r / py(); }
  int ry(int r) const { return r % py(); }
  // neighbour of rank r across face `side` (0 z-lo, 1 z-hi, 2 y-lo, 3 y-hi), -1 at the grid boundary
  int neighbor(int r, int side) const {
    const int a = rz(r), b = ry(r);
    switch (side) {
      case 0: return a > 0 ? r - py() : -1;
      case 1: return a + 1 < pz() ? r + py() : -1;
      case 2: return b > 0 ? r - 1 : -1;
      default: return b + 1 < py() ? r + 1 : -1;
    }
  }
};

}  // namespace mdfx
