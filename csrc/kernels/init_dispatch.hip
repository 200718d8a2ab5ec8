// Device-side field initialisation and the stencil dispatcher (variant selection + geometry).
//
// Reference parity: create_universe (MDF_kernel.cu:88-99, kernel.cu:131-146) built the grid on the
// host and shipped it over PCIe every generation (D12); here the initial condition is generated
// in place on the device from the *global* cell index, so every decomposition yields the same grid
// and no host copy is needed.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "kcommon.hpp"
#include "mdfx/kernels.hpp"

namespace mdfx {
namespace dev {

void naive_launch(const StencilSpec& spec, const Geo& g, const void* in, void* out, double* resid,
                  hipStream_t s);
template <class T>
void launch_heat7(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s);
template <class T>
void launch_jacobi5(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s, bool ref);
template <class T>
void launch_jacobi5_tb2(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s);
template <class T>
void launch_jacobi5_tbk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s,
                        bool ref_precision);
template <class T>
void launch_box27_tb2(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid, hipStream_t s);
template <class T>
bool box27_tb2_supported(const Geo& g);
template <class T>
void launch_box27(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                  hipStream_t s);
void launch_life(const Geo& g, const uint8_t* in, uint8_t* out, double* resid, hipStream_t s);
void launch_life_tb2(const Geo& g, const uint8_t* in, uint8_t* out, double* resid, hipStream_t s);
void launch_life_tbk(const Geo& g, const uint8_t* in, uint8_t* out, int steps, double* resid, hipStream_t s);
template <class T>
void launch_heat7_tb2(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s);
template <class T>
bool heat7_tb2_supported(const Geo& g);
template <class T>
void launch_heat7_tbk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s);
template <class T>
bool heat7_tbk_supported(const Geo& g, int steps);
template <class T>
void launch_heat7_wtk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s);
bool heat7_wtk_supported(int steps);
bool heat7_wxk_supported(int steps);
template <class T>
void launch_heat7_wxk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s);
template <class T>
void launch_box27_wxk(const Geo& g, const T* in, T* out, const StencilCoef& cf, int steps, double* resid,
                      hipStream_t s);
double heat7_wtk_xeff(int64_t nx, int esize, int steps);
// 3D 7-point sweeps of K >= 3 steps run heat7_wtk (wave-independent tiles; 1024^3 fp32 K = 3:
// 1443 vs 1081 GCells/s for heat7_tbk, profiles/archive/r02_wtk/README.txt; heat7_tbk's K = 3 / 4 were
// removed in round 5)
static bool use_wxk(DType dt, int64_t nx, int steps);
// (fp32 K = 5: heat7_wxk only, in rows of 2 cells per lane)
static bool use_wtk(int steps, DType dt) {
  return heat7_wtk_supported(steps) || ((dt == DType::F32 || dt == DType::F64) && steps == 5);
}
// ... and among them heat7_wxk (y halo exchanged inside the band, stencil_heat_wxk.hip) for fp32:
// 1024^3 K = 4 2262 GCells/s vs heat7_wtk K = 3 1868 on one box (profiles/archive/r03_wxk/); since
// round 6 heat7_wtk is fp64 only (its fp32 instances ran only under MDFX_H7_WXK=0: 12 kernels,
// ~290 KB of code object, removed). MDFX_H7_WXK = 0 / 1 forces fp64's choice off / on. fp64 K = 3
// takes it from 2048-cell rows on, in 3 + 1-row bands: 2048^3
// fp64 + residual every 12 897 vs 796 GCells/s for heat7_wtk, while at 1024-cell rows heat7_wtk's
// 3-row waves stay ahead (907 vs 874) (profiles/archive/r03_session_p/). fp64 K = 4 always runs it, in
// 2 + 1-row bands (heat7_wtk's K = 4 needs 1-row waves: 1024^3 1112-1124 vs 418 GCells/s,
// profiles/r04_session_o/)
static bool use_wxk(DType dt, int64_t nx, int steps) {
  return steps >= 5 || dt == DType::F32 || knobs().h7_wxk == 1 || (knobs().h7_wxk < 0 && (nx >= 2048 || steps == 4));
}

static int env_int(const char* name, int dflt) {
  const char* v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atoi(v);
}

static Knobs read_knobs() {
  Knobs k;
  k.tb_ry = env_int("MDFX_TB_RY", 0);
  k.wtk_wb = env_int("MDFX_WTK_WB", 0);
  k.h7_wxk = env_int("MDFX_H7_WXK", -1);
  k.b27_wxk = env_int("MDFX_B27_WXK", -1);
  k.devcheck_selftest = env_int("MDFX_DEVCHECK_SELFTEST", 0);
  k.fold_release = env_int("MDFX_FOLD_RELEASE", 0);
  return k;
}

// Published snapshots are never freed (a launch on another thread may still read the previous
// one); a reload allocates a few dozen bytes.
static std::atomic<const Knobs*> g_knobs{nullptr};

const Knobs& knobs() {
  const Knobs* k = g_knobs.load(std::memory_order_acquire);
  if (!k) {
    hip_reload_knobs();
    k = g_knobs.load(std::memory_order_acquire);
  }
  return *k;
}

struct InitArgs {
  int kind;
  uint64_t seed;
  double lo, hi, value, edge, interior, density;
  int dims;
};

template <class T>
__global__ __launch_bounds__(256) void init_kernel(T* __restrict__ buf, Geo g, InitArgs a) {
  const int64_t n = g.pitch * g.ny * g.lz_max;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % g.pitch, t = i / g.pitch, y = t % g.ny, lz = t / g.ny;
    const int64_t gz = lz + g.gz_off, gy = y + g.gy_off;  // (a pencil's ghost rows beyond the grid stay 0)
    double v = 0.0;
    if (x < g.nx && gz >= 0 && gz < g.gnz && gy >= 0 && gy < g.gny) {
      const bool bnd = x == 0 || x == g.nx - 1 || gz == 0 || gz == g.gnz - 1 ||
                       (a.dims == 3 && (gy == 0 || gy == g.gny - 1));
      const uint64_t gidx = (uint64_t)x + (uint64_t)g.nx * ((uint64_t)gy + (uint64_t)g.gny * (uint64_t)gz);
      switch (a.kind) {
        case 0: v = a.value; break;
        case 1: v = bnd ? a.edge : a.interior; break;
        case 2: v = fma(a.hi - a.lo, hash_unit(a.seed, gidx), a.lo); break;
        default: v = (!bnd && hash_unit(a.seed, gidx) < a.density) ? 1.0 : 0.0; break;
      }
    }
    buf[lz * g.plane + y * g.pitch + x] = (T)v;
  }
}

#ifdef MDFX_DEVICE_CHECKS
// one violation counter per device (make devcheck builds only)
static std::mutex g_oob_mu;
static std::map<int, unsigned long long*> g_oob;
static unsigned long long* oob_counter() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_oob_mu);
  auto it = g_oob.find(dev);
  if (it != g_oob.end()) return it->second;
  void* p = nullptr;
  if (hipMalloc(&p, sizeof(unsigned long long)) != hipSuccess) return nullptr;
  if (hipMemset(p, 0, sizeof(unsigned long long)) != hipSuccess) return nullptr;
  return g_oob[dev] = (unsigned long long*)p;
}
#endif

static Geo make_geo(const FieldLayout& lay, int64_t lz_begin, int64_t lz_end) {
  Geo g;
  g.alloc = lay.elems() + kSlackBytes / (int64_t)lay.esize();
#ifdef MDFX_DEVICE_CHECKS
  g.oob = oob_counter();
  // self-test of the checking machinery: pretend the allocation is half its size so in-bounds
  // accesses beyond that count as violations (nothing is accessed out of bounds)
  if (knobs().devcheck_selftest) g.alloc = lay.elems() / 2;
#endif
  g.pitch = lay.pitch;
  g.plane = lay.plane;
  g.nx = lay.global.nx;
  g.ny = lay.rows();
  g.gny = lay.global.ny;
  g.gy_off = lay.y0 - lay.hy;
  g.ly_begin = lay.hy;
  g.ly_end = lay.hy + lay.nyl();
  g.gnz = lay.global.nz;
  g.lz_begin = lz_begin;
  g.lz_end = lz_end;
  g.gz_off = lay.z0 - lay.halo;
  g.lz_max = lay.planes();
  return g;
}

static std::mutex g_variant_mu;
static std::string g_variant = "auto";

}  // namespace dev

int64_t hip_device_check_violations() {
#ifdef MDFX_DEVICE_CHECKS
  int64_t total = 0;
  std::lock_guard<std::mutex> lk(dev::g_oob_mu);
  for (auto& kv : dev::g_oob) {
    unsigned long long h = 0;
    if (hipSetDevice(kv.first) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(&h, kv.second, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
      MDFX_FAIL("reading the device-check counter failed");
    total += (int64_t)h;
  }
  return total;
#else
  return -1;
#endif
}

int hip_runtime_version() {
  int v = 0;
  return hipRuntimeGetVersion(&v) == hipSuccess ? v : 0;
}

void hip_reload_knobs() {
  dev::g_knobs.store(new dev::Knobs(dev::read_knobs()), std::memory_order_release);
}

void hip_set_kernel_variant(const char* name) {
  std::lock_guard<std::mutex> lk(dev::g_variant_mu);
  const std::string v = name ? name : "auto";
  MDFX_CHECK(v == "auto" || v == "naive" || v == "tuned", "unknown kernel variant " + v);
  dev::g_variant = v;
}

const char* hip_kernel_variant() {
  std::lock_guard<std::mutex> lk(dev::g_variant_mu);
  return dev::g_variant.c_str();
}

void hip_init(const InitSpec& init, const FieldLayout& lay, void* buf, void* stream) {
  const dev::Geo g = dev::make_geo(lay, 0, lay.planes());
  dev::InitArgs a{(int)init.kind, init.seed, init.lo,       init.hi,  init.value,
                  init.edge,      init.interior, init.density, lay.global.ny == 1 ? 2 : 3};
  const int64_t n = lay.pitch * lay.rows() * lay.planes();
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 256 * 64);
  hipStream_t s = (hipStream_t)stream;
  switch (lay.dtype) {
    case DType::F32:
      hipLaunchKernelGGL(dev::init_kernel<float>, dim3(grid), dim3(256), 0, s, (float*)buf, g, a);
      break;
    case DType::F64:
      hipLaunchKernelGGL(dev::init_kernel<double>, dim3(grid), dim3(256), 0, s, (double*)buf, g, a);
      break;
    case DType::U8:
      hipLaunchKernelGGL(dev::init_kernel<uint8_t>, dim3(grid), dim3(256), 0, s, (uint8_t*)buf, g, a);
      break;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) MDFX_FAIL(std::string("init launch failed: ") + hipGetErrorString(e));
}

bool hip_supports_steps(const StencilSpec& spec, const FieldLayout& lay, int steps) {
  if (steps == 1) return true;
  if (steps < 2 || lay.halo < steps) return false;
  if (lay.pencil())  // pencils (y ghost rows): the fused 7-point sweep of heat7_wxk only
    return spec.kind == StencilKind::Heat7 && dev::heat7_wxk_supported(steps) && lay.hy >= steps &&
           dev::knobs().h7_wxk != 0;
  const bool k2d = steps == 2 || steps == 3 || steps == 4 || steps == 6 || steps == 8;
  if (spec.kind == StencilKind::Jacobi5)  // deep temporal blocking of the 2D problems
    return (spec.dtype == DType::F32 || spec.dtype == DType::F64) && k2d;  // ref precision too (jacobi5_tbk REF)
  if (spec.kind == StencilKind::Life) return k2d || steps == 12 || steps == 16;  // 12 / 16: life_bits
  if (spec.kind == StencilKind::Heat7 && steps > 2) {  // deep temporal blocking (rows within one block)
    if (dev::use_wtk(steps, spec.dtype)) return true;
    const dev::Geo g = dev::make_geo(lay, lay.halo, lay.halo + lay.nzl());
    return spec.dtype == DType::F32 ? dev::heat7_tbk_supported<float>(g, steps)
                                    : dev::heat7_tbk_supported<double>(g, steps);
  }
  if (spec.kind == StencilKind::Box27 && steps == 3) return true;  // box27_wxk (any row width)
  if (steps != 2) return false;
  if (spec.kind == StencilKind::Box27) {
    const dev::Geo g = dev::make_geo(lay, lay.halo, lay.halo + lay.nzl());
    return spec.dtype == DType::F32 ? dev::box27_tb2_supported<float>(g) : dev::box27_tb2_supported<double>(g);
  }
  if (spec.kind != StencilKind::Heat7) return false;
  const dev::Geo g = dev::make_geo(lay, lay.halo, lay.halo + lay.nzl());
  return spec.dtype == DType::F32 ? dev::heat7_tb2_supported<float>(g) : dev::heat7_tb2_supported<double>(g);
}

bool hip_region_signals(const StencilSpec& spec, const FieldLayout& lay, int steps) {
  return !lay.pencil() && spec.kind == StencilKind::Heat7 &&
         (steps == 3 || steps == 4 || steps == 5) && lay.halo >= steps &&
         dev::use_wtk(steps, spec.dtype) && dev::use_wxk(spec.dtype, lay.global.nx, steps);
}

int hip_fused_depth(const StencilSpec& spec, int64_t nx) {
  switch (spec.kind) {
    case StencilKind::Jacobi5: return 8;
    case StencilKind::Life: return 12;
    case StencilKind::Box27:
      // K = 3 through box27_wxk for fp64 (512^3: 663 vs 527 GCells/s for box27_tbk K = 2), for fp32
      // rows of 1024 cells and more (1024^3: 1291 vs 1102, profiles/archive/r03_wxk/) and, since round 5's
      // whole-row blocks, for fp32 rows of 257..512 cells (512^3: 1332 vs 1092 for box27_tb2n K = 2,
      // profiles/r05_session_f/). MDFX_B27_WXK = 0 / 1 forces K = 2 / 3
      if (dev::knobs().b27_wxk == 1) return 3;
      if (dev::knobs().b27_wxk == 0) return 2;
      return (spec.dtype == DType::F64 || nx >= 1024 || (nx > 256 && nx <= 512)) ? 3 : 2;
    case StencilKind::Heat7:
      // K = 3 through heat7_wtk wherever its x segments cover at least 2/3 of the lane cells:
      // 1024^3 fp32 1617-1679 vs 1221-1232 GCells/s at K = 2 (round 2), 2048^3 fp32 1666 vs 1136,
      // 1024^3 fp64 823-825 vs 546, 2048^3 fp64 818 vs 556; since the natural-layout rows also
      // 512^3 fp32 (3 segments of 256 for 512 cells): 1311 vs 1230 (profiles/archive/r03_wtk/). K = 4
      // where heat7_wxk runs: its per-wave rows no longer grow with K, so the fourth step per pass
      // costs less than the HBM pass it saves (fp32; fp64 in round 4: 512^3 983 vs 740 GCells/s at
      // K = 3, 1024^3 1121 vs 885, 2048^3 + residual every 12 953 vs 890, profiles/r04_session_{o,p}/)
      // fp32 K = 5 (round 5): heat7_wxk in rows of 2 cells per lane (RowOps2f), whose half-size
      // rows leave room for the fifth level: 1024^3 2689 vs 2426 GCells/s at K = 4 in one process,
      // 1024^2 x 256 2639 vs 2399, x 128 2536 vs 2384, 768^3 2349 vs 1954, 512^3 2187 vs 2039,
      // 2048^2 x 512 2166 vs 2144 (profiles/r05_session_t/, r05_session_u/)
      // fp64 K = 5 (round 6): heat7_wxk in rows of 1 cell per lane (RowOps1d, the 2-cell fp32 rows'
      // register footprint; 54 of 64 lanes own a column), from rows of 2048 cells: 2048^3 + residual
      // every 20 1120 vs 1058 GCells/s at K = 4, while at 1024-cell rows its 19 x segments x 27 bands
      // (513 tiles on 256 CUs) lose to K = 4 (1011-1035 vs 1062-1080) (profiles/r06_session_b/)
      if (nx >= 512 && dev::heat7_wtk_xeff(nx, (int)dtype_size(spec.dtype), 3) >= 0.66) {
        if (spec.dtype == DType::F32 && dev::knobs().h7_wxk != 0) return 5;
        if (spec.dtype == DType::F64 && nx >= 2048 && dev::knobs().h7_wxk != 0) return 5;
        return dev::use_wxk(spec.dtype, nx, 4) ? 4 : 3;
      }
      return 2;
  }
  return 1;
}

// From the per-step rates of each fused depth on one MI355X (GCells/s; the time of a k-step sweep
// is k / rate_k): 3D 7-point fp32 1024^3 694 / 1300 / 1896 / 2350 for K = 1..4, fp64 347 / 546 /
// 885 / 1110 (profiles/archive/r03_wxk/first_ab.txt, r04_session_o/). Elsewhere a
// deeper sweep is taken to cost 5 % more per pass than a single step, which makes the plan the
// fewest sweeps with the deepest first.
double hip_sweep_cost(const StencilSpec& spec, int64_t nx, int steps) {
  if (steps <= 1) return 1.0;
  if (spec.kind == StencilKind::Heat7 && steps <= 5 && nx >= 1024) {
    // (fp32 K = 5 from the round-5 rates 1929 / 2399 / 2639 GCells/s for K = 3 / 4 / 5 at 1024^2 x
    // 256, scaled to the K = 4 entry; fp64 K = 5 from round 6's per-sweep times against K = 4: 2048^3
    // 38.4 vs 32.5 ms (x 1.18), 1024^3 x 1.31, profiles/r06_session_b/)
    // fp64 rows of 2048+ cells have their own row (round 6, per-sweep times at 2048^3: K = 3 28.8 ms
    // (heat7_wxk 3 + 1 rows, round 3's 897 GCells/s), K = 4 34.9, K = 5 38.4, against ~24.8 ms for a
    // single step; a residual every 12 steps then plans 5 + 4 + 3, which measured 1022 vs 961-985
    // GCells/s for depth 4's 4 + 4 + 4 on one box, profiles/r06_session_g/)
    static const double f32[6] = {0.0, 1.0, 1.07, 1.10, 1.18, 1.34};
    static const double f64[6] = {0.0, 1.0, 1.27, 1.18, 1.25, 1.64};
    static const double f64w[6] = {0.0, 1.0, 1.27, 1.16, 1.41, 1.55};
    if (spec.dtype == DType::F64) return (nx >= 2048 ? f64w : f64)[steps];
    return f32[steps];
  }
  return 1.0 + 0.05 * (steps - 1);
}

void hip_stencil(const StencilSpec& spec, const RegionArgs& a, void* stream) {
  if (a.lz2_end > a.lz2_begin) {
    // two regions in one call: heat7_wtk sweeps them in ONE launch (both boundary regions of a
    // slab: one fill of the device, one launch gap); every other kernel runs them one after the other
    const bool fuse = a.lz_end > a.lz_begin &&
                      ((a.steps > 1 && spec.kind == StencilKind::Heat7 && dev::use_wtk(a.steps, spec.dtype) &&
                        dev::use_wxk(spec.dtype, a.lay.global.nx, a.steps)) ||
                       (spec.kind == StencilKind::Box27 && a.steps == 3));
    if (!fuse) {
      RegionArgs r1 = a, r2 = a;
      r1.lz2_begin = r1.lz2_end = r2.lz2_begin = r2.lz2_end = 0;
      r2.lz_begin = a.lz2_begin;
      r2.lz_end = a.lz2_end;
      hip_stencil(spec, r1, stream);
      hip_stencil(spec, r2, stream);
      return;
    }
    MDFX_CHECK(a.lz2_begin >= a.lay.halo && a.lz2_end <= a.lay.halo + a.lay.nzl() && a.lz2_begin >= a.lz_end,
               "second region must lie inside the owned planes, after the first");
  }
  if (a.lz_end <= a.lz_begin) return;
  MDFX_CHECK(a.lz_begin >= a.lay.halo && a.lz_end <= a.lay.halo + a.lay.nzl(),
             "region must lie inside the owned planes");
  dev::Geo g = dev::make_geo(a.lay, a.lz_begin, a.lz_end);
  g.lz2_begin = a.lz2_begin;
  g.lz2_end = a.lz2_end;
  g.min_rounds = std::max(1, std::min(4, a.min_rounds));
  if (a.sig) {
    MDFX_CHECK(hip_region_signals(spec, a.lay, a.steps) && a.lz2_end <= a.lz2_begin && a.sig_z > a.lz_begin &&
                   a.sig_z <= a.lz_end,
               "a folded boundary (RegionArgs::sig) needs a one-region slab sweep through heat7_wxk");
    g.sig = a.sig;
    g.sig_z = a.sig_z;
    g.fold_release = dev::knobs().fold_release;
  }
  if (a.ly_end > a.ly_begin) {
    MDFX_CHECK(a.ly_begin >= a.lay.hy && a.ly_end <= a.lay.hy + a.lay.nyl(), "row range must lie inside the owned rows");
    g.ly_begin = a.ly_begin;
    g.ly_end = a.ly_end;
  }
  hipStream_t s = (hipStream_t)stream;
  if (a.lay.pencil()) {
    // pencil layouts: the fused 7-point sweeps through heat7_wxk, single steps through the
    // one-cell-per-lane kernels (every stencil); the other tuned kernels assume slab geometry
    if (a.steps != 1) {
      MDFX_CHECK(hip_supports_steps(spec, a.lay, a.steps),
                 format("no fused %d-step kernel for %s %s on a pencil layout (heat7_wxk: the 3D 7-point, K = 3 / 4)",
                        a.steps, stencil_name(spec.kind), dtype_name(spec.dtype)));
      if (spec.dtype == DType::F32)
        dev::launch_heat7_wxk<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.steps, a.resid, s);
      else
        dev::launch_heat7_wxk<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.steps, a.resid, s);
    } else {
      MDFX_CHECK(a.lz2_end <= a.lz2_begin, "single pencil steps take one region per call");
      dev::naive_launch(spec, g, a.in, a.out, a.resid, s);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) MDFX_FAIL(std::string("stencil launch failed: ") + hipGetErrorString(e));
    return;
  }
  if (a.steps != 1) {
    MDFX_CHECK(hip_supports_steps(spec, a.lay, a.steps),
               format("no fused %d-step kernel for %s %s at nx=%lld (halo %d)", a.steps, stencil_name(spec.kind),
                      dtype_name(spec.dtype), (long long)a.lay.global.nx, a.lay.halo));
    if (spec.kind == StencilKind::Box27 && a.steps == 3) {
      if (spec.dtype == DType::F32)
        dev::launch_box27_wxk<float>(g, (const float*)a.in, (float*)a.out, spec.coef, 3, a.resid, s);
      else
        dev::launch_box27_wxk<double>(g, (const double*)a.in, (double*)a.out, spec.coef, 3, a.resid, s);
    } else if (spec.kind == StencilKind::Box27) {
      if (spec.dtype == DType::F32)
        dev::launch_box27_tb2<float>(g, (const float*)a.in, (float*)a.out, spec.coef, a.resid, s);
      else
        dev::launch_box27_tb2<double>(g, (const double*)a.in, (double*)a.out, spec.coef, a.resid, s);
    } else if (spec.kind == StencilKind::Life) {
      if (a.steps > 2)
        dev::launch_life_tbk(g, (const uint8_t*)a.in, (uint8_t*)a.out, a.steps, a.resid, s);
      else
        dev::launch_life_tb2(g, (const uint8_t*)a.in, (uint8_t*)a.out, a.resid, s);
    } else if (spec.kind == StencilKind::Jacobi5) {
      // ref_precision takes the mixed kernels only where it can change a bit (mixed_update())
      const bool mixed = spec.mixed_update();
      if (a.steps > 2 || mixed) {
        if (spec.dtype == DType::F32)
          dev::launch_jacobi5_tbk<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.steps, a.resid, s,
                                         mixed);
        else
          dev::launch_jacobi5_tbk<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.steps, a.resid, s,
                                          false);
      } else if (spec.dtype == DType::F32) {
        dev::launch_jacobi5_tb2<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.resid, s);
      } else {
        dev::launch_jacobi5_tb2<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.resid, s);
      }
    } else if (dev::use_wtk(a.steps, spec.dtype) && dev::use_wxk(spec.dtype, a.lay.global.nx, a.steps)) {
      if (spec.dtype == DType::F32)
        dev::launch_heat7_wxk<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.steps, a.resid, s);
      else
        dev::launch_heat7_wxk<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.steps, a.resid, s);
    } else if (dev::use_wtk(a.steps, spec.dtype)) {  // (fp64 only: use_wxk holds for every fp32 sweep)
      dev::launch_heat7_wtk<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.steps, a.resid, s);
    } else if (a.steps > 2 || (spec.dtype == DType::F32 ? dev::heat7_tbk_supported<float>(g, 2)
                                                        : dev::heat7_tbk_supported<double>(g, 2))) {
      // rows within one block: the streaming K-step kernel; wider rows (K = 2): heat7_tb2 x tiles
      if (spec.dtype == DType::F32)
        dev::launch_heat7_tbk<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.steps, a.resid, s);
      else
        dev::launch_heat7_tbk<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.steps, a.resid, s);
    } else if (spec.dtype == DType::F32) {
      dev::launch_heat7_tb2<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.resid, s);
    } else {
      dev::launch_heat7_tb2<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.resid, s);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) MDFX_FAIL(std::string("stencil launch failed: ") + hipGetErrorString(e));
    return;
  }
  std::string variant;
  {
    std::lock_guard<std::mutex> lk(dev::g_variant_mu);
    variant = dev::g_variant;
  }
  if (variant == "naive") {
    dev::naive_launch(spec, g, a.in, a.out, a.resid, s);
  } else {
    switch (spec.kind) {
      case StencilKind::Heat7:
        if (spec.dtype == DType::F32)
          dev::launch_heat7<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.resid, s);
        else
          dev::launch_heat7<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.resid, s);
        break;
      case StencilKind::Jacobi5:
        if (spec.dtype == DType::F32)
          dev::launch_jacobi5<float>(g, (const float*)a.in, (float*)a.out, (float)spec.rate(), a.resid, s,
                                     spec.mixed_update());
        else
          dev::launch_jacobi5<double>(g, (const double*)a.in, (double*)a.out, spec.rate(), a.resid, s, false);
        break;
      case StencilKind::Box27:
        if (spec.dtype == DType::F32)
          dev::launch_box27<float>(g, (const float*)a.in, (float*)a.out, spec.coef, a.resid, s);
        else
          dev::launch_box27<double>(g, (const double*)a.in, (double*)a.out, spec.coef, a.resid, s);
        break;
      case StencilKind::Life:
        dev::launch_life(g, (const uint8_t*)a.in, (uint8_t*)a.out, a.resid, s);
        break;
    }
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) MDFX_FAIL(std::string("stencil launch failed: ") + hipGetErrorString(e));
}

}  // namespace mdfx
