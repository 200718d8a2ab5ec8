// Device-side helpers shared by the gfx950 stencil kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mdfx {
namespace dev {

// 16-byte per-lane vectors: one global_load_dwordx4 / global_store_dwordx4 per lane, a wave moves
// 1 KiB per instruction (cdna_hip_programming.md Guideline 13).
template <class T>
struct VT;
template <>
struct VT<float> {
  typedef float type __attribute__((ext_vector_type(4)));
  static constexpr int N = 4;
};
template <>
struct VT<double> {
  typedef double type __attribute__((ext_vector_type(2)));
  static constexpr int N = 2;
};

// Geometry of one region launch (all in elements; storage plane index "lz").
struct Geo {
  int64_t pitch;     // elements per row
  int64_t plane;     // elements per plane
  int64_t nx, ny;    // global x / y extents
  int64_t gnz;       // global z extent
  int64_t lz_begin;  // first storage plane to write
  int64_t lz_end;    // one past the last storage plane to write
  int64_t gz_off;    // global z = lz + gz_off
  int64_t lz_max;    // storage planes allocated (loads outside [0,lz_max) return 0)
};

// Bijective XCD-aware block remap (cdna_hip_programming.md §5, T1): blocks b and b+8 share an
// XCD, so consecutive *tiles* are handed to the same XCD and their shared halo rows hit that
// XCD's L2. Placement only affects speed, never correctness.
__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nwg) {
  const unsigned q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

template <class V>
__device__ __forceinline__ void store_nt(V* p, V v) {
  __builtin_nontemporal_store(v, p);
}

// Wave-wide sum then one device-scope atomic per wave (Guideline 12: one atomic per wave/block).
__device__ __forceinline__ void wave_atomic_add(double* dst, double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(dst, v);
}

}  // namespace dev
}  // namespace mdfx
