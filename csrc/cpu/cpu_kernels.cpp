// CPU oracle and CPU backend kernels. Same point arithmetic as the device (stencil_math.hpp);
// std::fma is exact, so fp32/fp64 results are bitwise identical to the gfx950 kernels.
//
// Reference parity: MDF_kernel.cu:10-22 / kernel.cu:10-68 (point updates), create_universe
// MDF_kernel.cu:88-99 / kernel.cu:131-146 (initial grids). This is also the CPU reference path
// of BASELINE.json config 1 (2D 5-pt Laplace 256x256 fp32, single rank).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {

namespace {

struct Pl {
  int64_t pitch, plane, nx, ny, gnz, gz_off;
};

Pl pl_of(const FieldLayout& l) {
  return Pl{l.pitch, l.plane, l.global.nx, l.global.ny, l.global.nz, l.z0 - l.halo};
}

template <class T>
void heat7_cpu(const T* in, T* out, const Pl& g, int64_t lb, int64_t le, T r, double* resid) {
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) if ((le - lb) * g.ny * g.nx > 65536)
  for (int64_t lz = lb; lz < le; ++lz) {
    const int64_t gz = lz + g.gz_off;
    for (int64_t y = 0; y < g.ny; ++y) {
      const int64_t row = lz * g.plane + y * g.pitch;
      const bool inner = gz > 0 && gz < g.gnz - 1 && y > 0 && y < g.ny - 1;
      for (int64_t x = 0; x < g.nx; ++x) {
        const int64_t i = row + x;
        const T c = in[i];
        T o = c;
        if (inner && x > 0 && x < g.nx - 1)
          o = sm::heat7<T>(c, in[i - 1], in[i + 1], in[i - g.pitch], in[i + g.pitch], in[i - g.plane],
                           in[i + g.plane], r);
        out[i] = o;
        const double d = (double)o - (double)c;
        acc += d * d;
      }
    }
  }
  if (resid) *resid += acc;
}

template <class T>
void jacobi5_cpu(const T* in, T* out, const Pl& g, int64_t lb, int64_t le, T r, double* resid) {
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) if ((le - lb) * g.nx > 65536)
  for (int64_t lz = lb; lz < le; ++lz) {
    const int64_t gz = lz + g.gz_off;
    const int64_t row = lz * g.plane;
    const bool inner = gz > 0 && gz < g.gnz - 1;
    for (int64_t x = 0; x < g.nx; ++x) {
      const int64_t i = row + x;
      const T c = in[i];
      T o = c;
      if (inner && x > 0 && x < g.nx - 1)
        o = sm::jacobi5<T>(c, in[i - 1], in[i + 1], in[i - g.plane], in[i + g.plane], r);
      out[i] = o;
      const double d = (double)o - (double)c;
      acc += d * d;
    }
  }
  if (resid) *resid += acc;
}

template <class T>
inline void box27_partials(const T* p, int64_t pitch, T& center, T& cross, T& diag) {
  const T hm = p[-pitch - 1] + p[-pitch + 1];
  const T h0 = p[-1] + p[1];
  const T hp = p[pitch - 1] + p[pitch + 1];
  center = p[0];
  cross = h0 + (p[-pitch] + p[pitch]);
  diag = hm + hp;
}

template <class T>
void box27_cpu(const T* in, T* out, const Pl& g, int64_t lb, int64_t le, const StencilCoef& cf,
               double* resid) {
  const T c0 = (T)cf.c0, c1 = (T)cf.c1, c2 = (T)cf.c2, c3 = (T)cf.c3;
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) if ((le - lb) * g.ny * g.nx > 65536)
  for (int64_t lz = lb; lz < le; ++lz) {
    const int64_t gz = lz + g.gz_off;
    for (int64_t y = 0; y < g.ny; ++y) {
      const int64_t row = lz * g.plane + y * g.pitch;
      const bool inner = gz > 0 && gz < g.gnz - 1 && y > 0 && y < g.ny - 1;
      for (int64_t x = 0; x < g.nx; ++x) {
        const int64_t i = row + x;
        const T c = in[i];
        T o = c;
        if (inner && x > 0 && x < g.nx - 1) {
          T ce, cr, dg;
          box27_partials(in + i - g.plane, g.pitch, ce, cr, dg);
          const T am = sm::box27_A(ce, cr, dg, c1, c2, c3);
          box27_partials(in + i, g.pitch, ce, cr, dg);
          const T bc = sm::box27_B(ce, cr, dg, c0, c1, c2);
          box27_partials(in + i + g.plane, g.pitch, ce, cr, dg);
          const T ap = sm::box27_A(ce, cr, dg, c1, c2, c3);
          o = sm::box27_combine(am, bc, ap);
        }
        out[i] = o;
        const double d = (double)o - (double)c;
        acc += d * d;
      }
    }
  }
  if (resid) *resid += acc;
}

void life_cpu(const uint8_t* in, uint8_t* out, const Pl& g, int64_t lb, int64_t le, double* resid) {
  double acc = 0.0;
#pragma omp parallel for schedule(static) reduction(+ : acc) if ((le - lb) * g.nx > 65536)
  for (int64_t lz = lb; lz < le; ++lz) {
    const int64_t gz = lz + g.gz_off;
    const int64_t row = lz * g.plane;
    const bool inner = gz > 0 && gz < g.gnz - 1;
    for (int64_t x = 0; x < g.nx; ++x) {
      const int64_t i = row + x;
      const uint8_t c = in[i];
      uint8_t o = c;
      if (inner && x > 0 && x < g.nx - 1) {
        unsigned t = 0;
        for (int dz = -1; dz <= 1; ++dz)
          for (int dx = -1; dx <= 1; ++dx) t += in[i + dz * g.plane + dx];
        o = sm::life_rule(t, c);
      }
      out[i] = o;
      acc += (o != c) ? 1.0 : 0.0;
    }
  }
  if (resid) *resid += acc;
}

}  // namespace

static void cpu_region(const StencilSpec& spec, const RegionArgs& a);

void cpu_stencil(const StencilSpec& spec, const RegionArgs& a) {
  if (a.lz_end <= a.lz_begin) return;
  MDFX_CHECK(a.lz_begin >= a.lay.halo && a.lz_end <= a.lay.halo + a.lay.nzl(),
             "region must lie inside the owned planes");
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
  for (int s = 1; s <= k; ++s) {
    RegionArgs b = a;
    b.in = tmp[(s - 1) & 1].data();
    b.out = s == k ? a.out : (void*)tmp[s & 1].data();
    b.lz_begin = a.lz_begin - (k - s);
    b.lz_end = a.lz_end + (k - s);
    b.resid = s == k ? a.resid : nullptr;
    if (s < k) std::memcpy(tmp[s & 1].data(), tmp[(s - 1) & 1].data(), a.lay.bytes());
    cpu_region(spec, b);
  }
}

static void cpu_region(const StencilSpec& spec, const RegionArgs& a) {
  const Pl g = pl_of(a.lay);
  switch (spec.kind) {
    case StencilKind::Heat7:
      if (spec.dtype == DType::F32)
        heat7_cpu<float>((const float*)a.in, (float*)a.out, g, a.lz_begin, a.lz_end, (float)spec.rate(), a.resid);
      else
        heat7_cpu<double>((const double*)a.in, (double*)a.out, g, a.lz_begin, a.lz_end, spec.rate(), a.resid);
      break;
    case StencilKind::Jacobi5:
      if (spec.dtype == DType::F32)
        jacobi5_cpu<float>((const float*)a.in, (float*)a.out, g, a.lz_begin, a.lz_end, (float)spec.rate(), a.resid);
      else
        jacobi5_cpu<double>((const double*)a.in, (double*)a.out, g, a.lz_begin, a.lz_end, spec.rate(), a.resid);
      break;
    case StencilKind::Box27:
      if (spec.dtype == DType::F32)
        box27_cpu<float>((const float*)a.in, (float*)a.out, g, a.lz_begin, a.lz_end, spec.coef, a.resid);
      else
        box27_cpu<double>((const double*)a.in, (double*)a.out, g, a.lz_begin, a.lz_end, spec.coef, a.resid);
      break;
    case StencilKind::Life:
      life_cpu((const uint8_t*)a.in, (uint8_t*)a.out, g, a.lz_begin, a.lz_end, a.resid);
      break;
  }
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
        if (x < g.nx && gz >= 0 && gz < g.gnz) {
          const bool bnd = x == 0 || x == g.nx - 1 || gz == 0 || gz == g.gnz - 1 ||
                           (dims == 3 && (y == 0 || y == g.ny - 1));
          const uint64_t gidx =
              (uint64_t)x + (uint64_t)g.nx * ((uint64_t)y + (uint64_t)g.ny * (uint64_t)gz);
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
