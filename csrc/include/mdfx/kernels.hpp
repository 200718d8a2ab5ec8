// mdfx — stencil / init / reduction kernels: one interface, two implementations
// (hand-written gfx950 HIP in csrc/kernels/*.hip, and the CPU oracle in csrc/cpu/cpu_kernels.cpp).
//
// Reference parity:
//   run_mdf      MDF_kernel.cu:10-22   -> StencilKind::Jacobi5
//   game_of_life kernel.cu:10-68       -> StencilKind::Life
//   middle_kernel / border_kernel (MDF_kernel.cu:24-70, kernel.cu:70-113) -> a *region* launch:
//   one kernel computes a plane range [lz_begin, lz_end) of the slab. Unlike the reference, a
//   region launch writes only its own planes (fixes the cross-stream write race D6) and every
//   boundary cell is handled explicitly (fixes the unsigned-wrap OOB reads D8 and the floored
//   grid D10).
//   create_universe MDF_kernel.cu:88-99 / kernel.cu:131-146 -> InitSpec.
#pragma once

#include "mdfx/grid.hpp"

namespace mdfx {

// One region update: out[planes lz_begin..lz_end) = stencil(in). Cells on the global boundary
// (x, y or z equal to 0 or n-1) are Dirichlet: copied through unchanged.
struct RegionArgs {
  const void* in = nullptr;
  void* out = nullptr;
  FieldLayout lay;
  int64_t lz_begin = 0, lz_end = 0;  // storage planes to write
  // optional second region written by the same call (the engine passes both K-plane boundary
  // regions of a slab at once; heat7_wtk runs them as one launch, other kernels as two)
  int64_t lz2_begin = 0, lz2_end = 0;
  // storage rows to write (pencil layouts: the y-boundary strips); empty = every owned row
  int64_t ly_begin = 0, ly_end = 0;
  double* resid = nullptr;           // optional accumulator of sum((out-in)^2) over the region
  // Time steps fused into this sweep (temporal blocking). 2 needs lay.halo >= 2 and reads
  // in[lz_begin-2, lz_end+2); the residual then covers the second step only.
  int steps = 1;
  // Minimum whole rounds of resident blocks per streaming fused sweep (0 = 1, at most 4). The engine
  // asks for 2 when slabs exchange halos: the exchange's RCCL / copy kernels then find CUs freed
  // after half the interior sweep. It is part of the launch, so a captured hipGraph replays exactly
  // the geometry the engine asked for when it captured.
  int min_rounds = 0;
  // Folded boundary (slabs, fused 7-point sweeps through heat7_wxk: hip_region_signals): the region
  // starts at the lower boundary planes [lz_begin, sig_z), and once every block has stored them the
  // kernel bumps the device counter sig[16] by one (sig[0] counts the blocks' arrivals; both in
  // memory from hip_alloc_uncached, one counter block per signalling launch). The halo stream waits for that counter instead of a separate
  // boundary launch, so the lower face is sent while the same sweep continues upward.
  unsigned long long* sig = nullptr;
  int64_t sig_z = 0;
};

// Whether a slab sweep of `steps` fused steps runs through a kernel that honours RegionArgs::sig.
//
// Visibility assumption of the folded boundary (measured, not specified): a signalling block only
// waits until its stores are acknowledged by its XCD's L2 (vmcnt 0) before counting its arrival; it
// issues no release, so the face may still sit dirty in up to 8 XCD L2s when the count completes.
// What makes it visible to the exchange is the halo stream's counter-wait kernel: the exchange is
// the next operation on that stream, and the runtime ends every kernel dispatch with a system-scope
// release that writes back each XCD's L2 before a dependent operation (blit kernel, SDMA copy, RCCL
// kernel, peer read over xGMI) starts. Per-block agent-scope releases instead (an L2 writeback by
// each of 235 blocks) made the whole sweep ~25 % slower (round 4). The ipc / proxy tests run this
// bitwise with both readers on one device; a cross-device reader relies on the same end-of-dispatch
// release.
bool hip_region_signals(const StencilSpec& spec, const FieldLayout& lay, int steps);

// Whether a fused multi-step sweep is implemented for this stencil / grid on the device.
bool hip_supports_steps(const StencilSpec& spec, const FieldLayout& lay, int steps);
// The deepest fused sweep that is a measured win for this stencil at row width nx (before any
// cap by slab depth): 8 for the 2D MDF, 12 for Life, 4 for the 3D 7-point where heat7_wxk's x
// segments cover the row efficiently, else 2
// (profiles/archive/r02_wtk/README.txt, r02_mdf2d/, r02_life.txt, r04_session_o/).
int hip_fused_depth(const StencilSpec& spec, int64_t nx);
// Relative time of one `steps`-step sweep on the device, in single-step sweeps of the same grid
// (the engine's sweep plan minimises the sum over a residual stretch).
double hip_sweep_cost(const StencilSpec& spec, int64_t nx, int steps);
// One step shallower than `steps` among the fused depths (12 -> 6 -> 3 -> 2 -> 1).
inline int shallower_depth(int steps) { return steps == 5 ? 4 : steps == 3 ? 2 : steps / 2; }

enum class InitKind : int {
  Constant = 0,   // every cell = value
  Dirichlet = 1,  // global-boundary cells = edge, interior = interior (MDF_kernel.cu:88-99)
  Random = 2,     // uniform [lo, hi) from a counter-based hash of (seed, global index)
  LifeRandom = 3, // U8: alive with probability `density` off the frame, frame dead (kernel.cu:131-146)
};

struct InitSpec {
  InitKind kind = InitKind::Random;
  uint64_t seed = 1;
  double lo = 0.0, hi = 1.0;
  double value = 0.0;
  double edge = 100.0, interior = 0.0;
  double density = 0.15;
};

// Counter-based generator shared by host and device: value depends only on (seed, global linear
// index gx + nx*(gy + ny*gz)), so any decomposition produces the same grid.
#if defined(__HIPCC__)
#define MDFX_HD __host__ __device__
#else
#define MDFX_HD
#endif
MDFX_HD inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}
MDFX_HD inline double hash_unit(uint64_t seed, uint64_t gidx) {
  const uint64_t h = mix64(gidx * 0x9E3779B97F4A7C15ull + mix64(seed + 0x632BE59BD9B4E019ull));
  return (double)(h >> 11) * (1.0 / 9007199254740992.0);  // [0,1) with 53 bits
}

// ---- HIP (gfx950) -------------------------------------------------------------------------
// `stream` is a hipStream_t. All launches are asynchronous.
void hip_stencil(const StencilSpec& spec, const RegionArgs& a, void* stream);
void hip_init(const InitSpec& init, const FieldLayout& lay, void* buf, void* stream);
// Variant selection for kernel A/B benchmarking and tests: "auto", "naive", "tuned".
// Out-of-allocation accesses counted by the device checks of a `make devcheck` build (-1 when
// the checks are compiled out, as in release builds).
int64_t hip_device_check_violations();
void hip_set_kernel_variant(const char* name);
// hipRuntimeGetVersion of the HIP runtime in this process (e.g. 70051831 for PyTorch's bundled
// 7.0, 70226015 for /opt/rocm 7.2); 0 when no runtime answers.
int hip_runtime_version();
// Re-read the MDFX_* kernel tuning knobs from the environment (they are cached at first use).
void hip_reload_knobs();
const char* hip_kernel_variant();

// ---- CPU oracle / CPU backend ----------------------------------------------------------------
void cpu_stencil(const StencilSpec& spec, const RegionArgs& a);
void cpu_init(const InitSpec& init, const FieldLayout& lay, void* buf);
// Reproduce the reference's intended GoL initial grid with glibc rand() seeded by `seed` (the
// reference never seeds: seed 1). Fills a dense h*w int8 host array in global row-major order.
void cpu_life_compat_init(uint8_t* grid, int64_t h, int64_t w, double density, unsigned seed);

}  // namespace mdfx
