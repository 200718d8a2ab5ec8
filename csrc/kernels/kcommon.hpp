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
  int64_t nx, ny;    // global x extent; y: storage rows per plane (the global extent for slabs)
  int64_t gnz;       // global z extent
  int64_t lz_begin;  // first storage plane to write
  int64_t lz_end;    // one past the last storage plane to write
  int64_t gz_off;    // global z = lz + gz_off
  int64_t lz_max;    // storage planes allocated (loads outside [0,lz_max) return 0)
  int64_t lz2_begin = 0, lz2_end = 0;  // optional second region of the same launch (heat7_wtk)
  int64_t alloc = 0;                 // elements allocated (planes + slack), for device checks
  int min_rounds = 1;                // whole rounds of resident blocks a streaming sweep spans at least (RegionArgs)
  // pencil layouts (a y split with ghost rows): global rows, global y = storage row + gy_off, and the
  // storage rows [ly_begin, ly_end) to write (slabs: gny = ny, gy_off = 0, every row). Kernels
  // without pencil support only ever see slab geometry (hip_stencil routes pencils to naive / wxk)
  int64_t gny = 0, gy_off = 0, ly_begin = 0, ly_end = 0;
  // folded lower boundary (heat7_wxk SIG copy, RegionArgs::sig): every block of the chunks that start
  // at lz_begin signals once its output planes [lz_begin, sig_z) are stored; the last of them bumps
  // sig[16] (sig[0] counts arrivals)
  unsigned long long* sig = nullptr;
  int64_t sig_z = 0;
  int fold_release = 0;  // the signalling blocks write their XCD's L2 back first (Knobs::fold_release)
  unsigned long long* oob = nullptr;  // device-check violation counter (debug builds only)
};

// Debug builds (-DMDFX_DEVICE_CHECKS: make devcheck) check the element range of every tuned-kernel
// load and store against the allocation and COUNT violations in g.oob, which the host reads back
// (hip_device_check_violations). Counting instead of trapping keeps a bad index from faulting the
// GPU. Release builds compile the checks out.
template <class T>
__device__ __forceinline__ void dcheck(const Geo& g, const T* base, const T* p, int n) {
#ifdef MDFX_DEVICE_CHECKS
  const int64_t i = p - base;
  if (g.oob && (i < 0 || i + n > g.alloc)) atomicAdd(g.oob, 1ull);
#else
  (void)g;
  (void)base;
  (void)p;
  (void)n;
#endif
}

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

namespace mdfx {
namespace dev {

// LDS DMA: each active lane loads 16 bytes from its own global address into LDS at
// `l` + 16 * lane (global_load_lds_dwordx4, gfx950), without a VGPR destination. `l` must be
// wave-uniform. hipcc does not track these LDS writes: wait with vmcnt(0) before reading them.
__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// The same with 4 bytes per lane (global_load_lds_dword): LDS at `l` + 4 * lane.
__device__ __forceinline__ void glds4(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 4, 0, 0);
}

// The same copies through a buffer descriptor (buffer_load_dword{,x4} ... lds) whose base is a
// wave-uniform row address in SGPRs, `off` the lane's byte offset from it. hipcc's waitcnt pass
// counts a global_load_lds in flight as a possible LDS access by a flat instruction, whose lgkm
// completion is out of order, so every LDS read issued while one is in flight waits for ALL
// outstanding LDS reads (lgkmcnt(0)) at its first use; a buffer DMA leaves those waits partial
// (lgkmcnt(n): the reads return in order). Offsets past the descriptor's range read 0, never fault.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t off, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, off, 0, 0, 0);
}
// (`soff`: a wave-uniform byte offset added in the instruction's SGPR offset field)
__device__ __forceinline__ void blds16s(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t soff, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 16, off, (int)soff, 0, 0);
}
__device__ __forceinline__ void blds4(__amdgpu_buffer_rsrc_t r, uint32_t off, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)l, 4, off, 0, 0, 0);
}

// Raw waits: s_waitcnt encodings for gfx9 (vmcnt [3:0]+[15:14], expcnt [6:4], lgkmcnt [11:8]).
__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// vmcnt(n) for a wave-uniform n in 0..15 (an immediate per case): wait until at most the wave's n
// youngest vector-memory operations are outstanding. The streaming kernels issue the next plane's
// LDS DMA first and the output stores of the plane after it; waiting with n = the stores issued
// since the DMA leaves those stores in flight across the next plane's barrier instead of
// exposing a full store round trip per plane (an out-of-range n waits for everything).
__device__ __forceinline__ void wait_vm_le(int n) {
  switch (n) {
    case 1: __builtin_amdgcn_s_waitcnt(0x0F71); break;
    case 2: __builtin_amdgcn_s_waitcnt(0x0F72); break;
    case 3: __builtin_amdgcn_s_waitcnt(0x0F73); break;
    case 4: __builtin_amdgcn_s_waitcnt(0x0F74); break;
    case 5: __builtin_amdgcn_s_waitcnt(0x0F75); break;
    case 6: __builtin_amdgcn_s_waitcnt(0x0F76); break;
    case 7: __builtin_amdgcn_s_waitcnt(0x0F77); break;
    case 8: __builtin_amdgcn_s_waitcnt(0x0F78); break;
    case 9: __builtin_amdgcn_s_waitcnt(0x0F79); break;
    case 10: __builtin_amdgcn_s_waitcnt(0x0F7A); break;
    case 11: __builtin_amdgcn_s_waitcnt(0x0F7B); break;
    case 12: __builtin_amdgcn_s_waitcnt(0x0F7C); break;
    case 13: __builtin_amdgcn_s_waitcnt(0x0F7D); break;
    case 14: __builtin_amdgcn_s_waitcnt(0x0F7E); break;
    case 15: __builtin_amdgcn_s_waitcnt(0x0F7F); break;
    default: __builtin_amdgcn_s_waitcnt(0x0F70); break;
  }
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }
// An LDS pointer whose (wave-uniform) address is pinned in a VGPR: ds_read / ds_write take a VGPR
// address, and a uniform address kept in an SGPR is otherwise copied into a VGPR at every access
// (v_mov + access). Accesses through the result at compile-time indices use the instruction's
// offset field.
template <class T>
__device__ __forceinline__ __attribute__((address_space(3))) T* lds_vptr(T* p) {
  unsigned a = (unsigned)(uintptr_t)((__attribute__((address_space(3))) T*)p);
  asm volatile("" : "+v"(a));
  return (__attribute__((address_space(3))) T*)(uintptr_t)a;
}

// Workgroup barrier that does NOT drain outstanding vector-memory operations (a __syncthreads
// makes hipcc wait for vmcnt(0), which would also wait for an in-flight LDS DMA). LDS writes are
// completed first; the empty asm statements keep the compiler from moving memory accesses across.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS store outside the compiler's view. hipcc's wait-count pass treats a compiler-visible LDS
// store as a possible alias of an in-flight LDS DMA (global_load_lds) and puts s_waitcnt vmcnt(0)
// in front of it, which drains the next plane's DMA in the middle of the plane's compute. The
// stores below go to tables no DMA writes; lds_barrier()'s lgkmcnt(0) completes them.
template <class V>
__device__ __forceinline__ void lds_store(void* p, const V& v) {
  const unsigned a = (unsigned)(uintptr_t)((__attribute__((address_space(3))) void*)p);
  static_assert(sizeof(V) == 8 || sizeof(V) == 16, "8- or 16-byte LDS stores");
  if constexpr (sizeof(V) == 8)
    asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
  else
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}

// Whole-wave lane shifts by one (lane i <- lane i-1 / lane i+1) with DPP wave_shr:1 / wave_shl:1:
// a VALU move with a DPP modifier instead of a ds_bpermute through the LDS crossbar. The lane that
// has no source (0 or 63) receives 0; callers overwrite it with the seam value.
// bound_ctrl on: the lane without a source reads 0 with no `old` operand to materialise first
__device__ __forceinline__ int dpp_shr1_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int dpp_shl1_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xF, 0xF, true); }
__device__ __forceinline__ int lane_up1(int v) { return dpp_shr1_i(v); }
__device__ __forceinline__ int lane_down1(int v) { return dpp_shl1_i(v); }
__device__ __forceinline__ float lane_up1(float v) { return __int_as_float(dpp_shr1_i(__float_as_int(v))); }
__device__ __forceinline__ float lane_down1(float v) { return __int_as_float(dpp_shl1_i(__float_as_int(v))); }
__device__ __forceinline__ double lane_up1(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_shr1_i((int)(b & 0xffffffffll)), hi = dpp_shr1_i((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_down1(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = dpp_shl1_i((int)(b & 0xffffffffll)), hi = dpp_shl1_i((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// lane i <- lane i-1 (up) / lane i+1 (down); the lane without a source (0 / 63) keeps `edge`.
// DPP with bound_ctrl off leaves that lane's destination at the `old` operand, so the seam value
// costs no extra instruction.
__device__ __forceinline__ float lane_up1_or(float edge, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x138, 0xF, 0xF, false));
}
__device__ __forceinline__ float lane_down1_or(float edge, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(edge), __float_as_int(v), 0x130, 0xF, 0xF, false));
}
__device__ __forceinline__ double lane_up1_or(double edge, double v) {
  const long long b = __double_as_longlong(v), o = __double_as_longlong(edge);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffll), (int)(b & 0xffffffffll), 0x138, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x138, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double lane_down1_or(double edge, double v) {
  const long long b = __double_as_longlong(v), o = __double_as_longlong(edge);
  const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffffll), (int)(b & 0xffffffffll), 0x130, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), 0x130, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Host-side kernel tuning knobs (MDFX_* environment variables), read once per process and cached:
// the dispatchers run on every launch and never call getenv there. hip_reload_knobs() re-reads
// them (tests that change a knob in-process; Python: native().reload_knobs()).
struct Knobs {
  // kernel-family selectors the GPU tests use to reach every shipped instance (each is the default
  // somewhere: a dtype, a row width, a region depth); the round-2..4 tuning switches whose
  // non-default settings measured slower were removed in round 5 (their numbers: docs/DESIGN.md)
  int tb_ry = 0;       // MDFX_TB_RY: rows per tile of heat7_tb2 (x-tiled rows) / box27_tb2 (1; 0: 2, 1 on short columns)
  int wtk_wb = 0;      // MDFX_WTK_WB: heat7_wtk waves per y band (4 or 8; 0: by region depth)
  int h7_wxk = -1;     // MDFX_H7_WXK: K >= 3 sweeps of the 3D 7-point through heat7_wxk (-1: by dtype / width, 0: never, 1: always)
  int b27_wxk = -1;    // MDFX_B27_WXK: the 27-point's fused depth 3 through box27_wxk (-1: fp64, fp32 rows of 257..512 or >= 1024 cells; 0 / 1)
  int devcheck_selftest = 0;  // MDFX_DEVCHECK_SELFTEST (make devcheck builds)
  int fold_release = 0;       // MDFX_FOLD_RELEASE: folded-boundary blocks release (L2 writeback) before they signal
};
const Knobs& knobs();

}  // namespace dev
}  // namespace mdfx
