// CPU oracle and CPU backend kernels. Same point arithmetic as the device (stencil_math.hpp);
// std::fma is exact, so fp32/fp64 results are bitwise identical to the gfx950 kernels.
//
// Reference parity: MDF_kernel.cu:10-22 / kernel.cu:10-68 (point updates), create_universe
// MDF_kernel.cu:88-99 / kernel.cu:131-146 (initial grids). This is also the CPU reference path
// of BASELINE.json config 1 (2D 5-pt Laplace 256x256 fp32, single rank).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

#define MDFX_CPU_NS cpu_base
#include "cpu_stencils.inc"

namespace mdfx {
namespace cpu_avx2 {
void region(const StencilSpec& spec, const RegionArgs& a);
}

namespace {
using cpu_base::Pl;
using cpu_base::pl_of;
}  // namespace

static void cpu_region(const StencilSpec& spec, const RegionArgs& a);

void cpu_stencil(const StencilSpec& spec, const RegionArgs& a) {
  if (a.lz2_end > a.lz2_begin) {  // two regions: one after the other
    RegionArgs r1 = a, r2 = a;
    r1.lz2_begin = r1.lz2_end = r2.lz2_begin = r2.lz2_end = 0;
    r2.lz_begin = a.lz2_begin;
    r2.lz_end = a.lz2_end;
    cpu_stencil(spec, r1);
    cpu_stencil(spec, r2);
    return;
  }
  if (a.lz_end <= a.lz_begin) return;
  MDFX_CHECK(a.lz_begin >= a.lay.halo && a.lz_end <= a.lay.halo + a.lay.nzl(),
             "region must lie inside the owned planes");
  MDFX_CHECK(a.ly_end <= a.ly_begin || (a.ly_begin >= a.lay.hy && a.ly_end <= a.lay.hy + a.lay.nyl()),
             "row range must lie inside the owned rows");
  if (a.steps == 1) {
    cpu_region(spec, a);
    return;
  }
  // fused k-step sweep = k single steps through a scratch copy, widening the first steps by the
  // planes the later ones read (the device kernel computes exactly these values on chip)
  const int k = a.steps;
  MDFX_CHECK(k >= 1 && a.lay.halo >= k, "fused steps need halo >= steps");
  std::vector<char> tmp[2];
  tmp[0].assign(a.lay.bytes(), 0);
  tmp[1].assign(a.lay.bytes(), 0);
  std::memcpy(tmp[0].data(), a.in, a.lay.bytes());
  const int64_t yb = a.ly_end > a.ly_begin ? a.ly_begin : a.lay.hy, ye = a.ly_end > a.ly_begin ? a.ly_end : a.lay.hy + a.lay.nyl();
  for (int s = 1; s <= k; ++s) {
    RegionArgs b = a;
    b.in = tmp[(s - 1) & 1].data();
    b.out = s == k ? a.out : (void*)tmp[s & 1].data();
    b.lz_begin = a.lz_begin - (k - s);
    b.lz_end = a.lz_end + (k - s);
    // the rows the later steps read, as far as the layout holds them (a pencil's ghost rows;
    // global boundary rows are held, so a slab needs no widening)
    b.ly_begin = std::max<int64_t>(yb - (k - s), a.lay.hy > 0 ? 1 : 0);
    b.ly_end = std::min<int64_t>(ye + (k - s), a.lay.hy > 0 ? a.lay.rows() - 1 : a.lay.rows());
    b.resid = s == k ? a.resid : nullptr;
    if (s < k) std::memcpy(tmp[s & 1].data(), tmp[(s - 1) & 1].data(), a.lay.bytes());
    cpu_region(spec, b);
  }
}

// AVX2 + FMA build when the host supports it (hardware fma instead of libm's software fmaf on
// baseline x86-64); both are exact, so the choice never changes a result
static void cpu_region(const StencilSpec& spec, const RegionArgs& a) {
  static const bool avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") &&
                           !std::getenv("MDFX_CPU_BASELINE");
  if (avx2)
    cpu_avx2::region(spec, a);
  else
    cpu_base::region(spec, a);
}

template <class T>
static void init_cpu_t(const InitSpec& s, const FieldLayout& l, T* buf) {
  const Pl g = pl_of(l);
  const int dims = l.global.ny == 1 ? 2 : 3;
  const int64_t planes = l.planes();
#pragma omp parallel for schedule(static) if (planes * g.plane > 65536)
  for (int64_t lz = 0; lz < planes; ++lz) {
    const int64_t gz = lz + g.gz_off;
    for (int64_t y = 0; y < g.ny; ++y)
      for (int64_t x = 0; x < g.pitch; ++x) {
        double v = 0.0;
        const int64_t gy = y + g.gy_off;  // (ghost rows beyond the grid stay 0, as ghost planes)
        if (x < g.nx && gz >= 0 && gz < g.gnz && gy >= 0 && gy < g.gny) {
          const bool bnd = x == 0 || x == g.nx - 1 || gz == 0 || gz == g.gnz - 1 ||
                           (dims == 3 && (gy == 0 || gy == g.gny - 1));
          const uint64_t gidx =
              (uint64_t)x + (uint64_t)g.nx * ((uint64_t)gy + (uint64_t)g.gny * (uint64_t)gz);
          switch (s.kind) {
            case InitKind::Constant: v = s.value; break;
            case InitKind::Dirichlet: v = bnd ? s.edge : s.interior; break;
            case InitKind::Random: v = std::fma(s.hi - s.lo, hash_unit(s.seed, gidx), s.lo); break;
            case InitKind::LifeRandom:
              v = (!bnd && hash_unit(s.seed, gidx) < s.density) ? 1.0 : 0.0;
              break;
          }
        }
        buf[lz * g.plane + y * g.pitch + x] = (T)v;
      }
  }
}

void cpu_init(const InitSpec& init, const FieldLayout& lay, void* buf) {
  switch (lay.dtype) {
    case DType::F32: init_cpu_t<float>(init, lay, (float*)buf); break;
    case DType::F64: init_cpu_t<double>(init, lay, (double*)buf); break;
    case DType::U8: init_cpu_t<uint8_t>(init, lay, (uint8_t*)buf); break;
  }
}

void cpu_life_compat_init(uint8_t* grid, int64_t h, int64_t w, double density, unsigned seed) {
  // kernel.cu:131-146: rand() is drawn only for non-frame cells, in row-major order;
  // alive iff (float)rand()/RAND_MAX <= prob (the reference writes `rand_prob > prob ? 0 : 1`).
  srand(seed);
  const float prob = (float)density;
  for (int64_t i = 0; i < h; ++i)
    for (int64_t j = 0; j < w; ++j) {
      const int64_t k = i * w + j;
      if (i == 0 || j == 0 || i == h - 1 || j == w - 1) {
        grid[k] = 0;
      } else {
        const float rp = (float)rand() / (float)RAND_MAX;
        grid[k] = rp > prob ? 0 : 1;
      }
    }
}

}  // namespace mdfx
