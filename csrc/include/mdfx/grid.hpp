// mdfx — field layout and 1-D slab decomposition.
//
// Reference parity: the reference replicates the whole h*w grid on every rank, host and device
// (MDF_kernel.cu:137-144), indexes it with 32-bit ints and __mul24 (D16) and splits it
// at exactly size/2 between two hard-coded ranks (MDF_kernel.cu:30,38,54,62, D15). Here each rank
// stores only its slab plus `halo` ghost planes per side, every index is 64-bit, and the split
// works for any P <= nz with an uneven remainder.
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
  DType dtype = DType::F32;
  int64_t pitch = 0;   // elements per row (>= nx)
  int64_t plane = 0;   // elements per plane = pitch * ny

  static FieldLayout make(Extent3 g, int64_t z0, int64_t z1, int halo, DType dt);

  size_t esize() const { return dtype_size(dtype); }
  int64_t nzl() const { return z1 - z0; }
  int64_t planes() const { return nzl() + 2 * halo; }
  int64_t elems() const { return planes() * plane; }
  size_t bytes() const { return (size_t)elems() * esize() + kSlackBytes; }
  // storage plane index of a global plane
  int64_t lz(int64_t gz) const { return gz - z0 + halo; }
  // global plane of a storage plane index
  int64_t gz(int64_t lz) const { return lz - halo + z0; }
  int64_t offset(int64_t x, int64_t y, int64_t lzi) const { return lzi * plane + y * pitch + x; }
  size_t plane_bytes() const { return (size_t)plane * esize(); }
  // owned cells (what a rank contributes to GCells/s)
  int64_t owned_cells() const { return global.nx * global.ny * nzl(); }
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

}  // namespace mdfx
