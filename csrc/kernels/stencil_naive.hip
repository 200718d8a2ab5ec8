// One-cell-per-lane gfx950 kernels for every stencil family. They are the "naive" variant: the
// on-device oracle the tuned kernels are checked against bitwise, and the A/B baseline in
// bench/micro. They use the same point arithmetic (stencil_math.hpp) as every other path.
//
// Reference parity: this is what run_mdf/game_of_life (MDF_kernel.cu:10-22, kernel.cu:10-68)
// compute per thread, minus their defects: 64-bit grid-stride indexing (no __mul24, no floored
// grid — SURVEY D10, D16) and explicit boundary handling (D8, D9).
#include "kcommon.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

// (3D kernels: rows [ly_begin, ly_end) of a pencil's storage, held at the GLOBAL y boundary)
template <class T, bool RES>
__global__ __launch_bounds__(256) void naive_heat7(const T* __restrict__ in, T* __restrict__ out,
                                                   Geo g, T r, double* __restrict__ resid) {
  const int64_t nr = g.ly_end - g.ly_begin;
  const int64_t n = g.nx * nr * (g.lz_end - g.lz_begin);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % g.nx, t = i / g.nx, y = g.ly_begin + t % nr, lz = g.lz_begin + t / nr;
    const int64_t gz = lz + g.gz_off, gy = y + g.gy_off;
    const int64_t idx = lz * g.plane + y * g.pitch + x;
    const T c = in[idx];
    T o = c;
    if (x > 0 && x < g.nx - 1 && gy > 0 && gy < g.gny - 1 && gz > 0 && gz < g.gnz - 1)
      o = sm::heat7<T>(c, in[idx - 1], in[idx + 1], in[idx - g.pitch], in[idx + g.pitch],
                       in[idx - g.plane], in[idx + g.plane], r);
    out[idx] = o;
    if (RES) {
      const double d = (double)o - (double)c;
      acc += d * d;
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, bool RES>
__global__ __launch_bounds__(256) void naive_jacobi5(const T* __restrict__ in, T* __restrict__ out,
                                                     Geo g, T r, int ref, double* __restrict__ resid) {
  const int64_t n = g.nx * (g.lz_end - g.lz_begin);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % g.nx, lz = g.lz_begin + i / g.nx;
    const int64_t gz = lz + g.gz_off;
    const int64_t idx = lz * g.plane + x;
    const T c = in[idx];
    T o = c;
    if (x > 0 && x < g.nx - 1 && gz > 0 && gz < g.gnz - 1)
      o = ref ? sm::jacobi5_ref<T>(c, in[idx - 1], in[idx + 1], in[idx - g.plane], in[idx + g.plane], r)
              : sm::jacobi5<T>(c, in[idx - 1], in[idx + 1], in[idx - g.plane], in[idx + g.plane], r);
    out[idx] = o;
    if (RES) {
      const double d = (double)o - (double)c;
      acc += d * d;
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T>
__device__ __forceinline__ void box27_plane_partials(const T* p, int64_t pitch, T& center, T& cross,
                                                     T& diag) {
  // p points at (x, y) of one plane
  const T hm = p[-pitch - 1] + p[-pitch + 1];
  const T h0 = p[-1] + p[1];
  const T hp = p[pitch - 1] + p[pitch + 1];
  center = p[0];
  cross = h0 + (p[-pitch] + p[pitch]);
  diag = hm + hp;
}

template <class T, bool RES>
__global__ __launch_bounds__(256) void naive_box27(const T* __restrict__ in, T* __restrict__ out,
                                                   Geo g, T c0, T c1, T c2, T c3,
                                                   double* __restrict__ resid) {
  const int64_t nr = g.ly_end - g.ly_begin;
  const int64_t n = g.nx * nr * (g.lz_end - g.lz_begin);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % g.nx, t = i / g.nx, y = g.ly_begin + t % nr, lz = g.lz_begin + t / nr;
    const int64_t gz = lz + g.gz_off, gy = y + g.gy_off;
    const int64_t idx = lz * g.plane + y * g.pitch + x;
    const T c = in[idx];
    T o = c;
    if (x > 0 && x < g.nx - 1 && gy > 0 && gy < g.gny - 1 && gz > 0 && gz < g.gnz - 1) {
      T ce, cr, dg;
      box27_plane_partials(in + idx - g.plane, g.pitch, ce, cr, dg);
      const T am = sm::box27_A(ce, cr, dg, c1, c2, c3);
      box27_plane_partials(in + idx, g.pitch, ce, cr, dg);
      const T bc = sm::box27_B(ce, cr, dg, c0, c1, c2);
      box27_plane_partials(in + idx + g.plane, g.pitch, ce, cr, dg);
      const T ap = sm::box27_A(ce, cr, dg, c1, c2, c3);
      o = sm::box27_combine(am, bc, ap);
    }
    out[idx] = o;
    if (RES) {
      const double d = (double)o - (double)c;
      acc += d * d;
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <bool RES>
__global__ __launch_bounds__(256) void naive_life(const uint8_t* __restrict__ in,
                                                  uint8_t* __restrict__ out, Geo g,
                                                  double* __restrict__ resid) {
  const int64_t n = g.nx * (g.lz_end - g.lz_begin);
  double acc = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i % g.nx, lz = g.lz_begin + i / g.nx;
    const int64_t gz = lz + g.gz_off;
    const int64_t idx = lz * g.plane + x;
    const uint8_t c = in[idx];
    uint8_t o = c;
    if (x > 0 && x < g.nx - 1 && gz > 0 && gz < g.gnz - 1) {
      unsigned t = 0;
#pragma unroll
      for (int dz = -1; dz <= 1; ++dz)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) t += in[idx + dz * g.plane + dx];
      o = sm::life_rule(t, c);
    }
    out[idx] = o;
    if (RES) acc += (o != c) ? 1.0 : 0.0;
  }
  if (RES) wave_atomic_add(resid, acc);
}

static int naive_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  return (int)std::min<int64_t>(std::max<int64_t>(b, 1), 256 * 32);
}

void naive_launch(const StencilSpec& spec, const Geo& g, const void* in, void* out, double* resid,
                  hipStream_t s) {
  const int64_t n = g.nx * (g.ly_end - g.ly_begin) * (g.lz_end - g.lz_begin);
  if (n <= 0) return;
  const dim3 grd(naive_grid(n)), blk(256);
  const bool res = resid != nullptr;
#define MDFX_NAIVE(KERNEL, T, ...)                                                              \
  do {                                                                                          \
    if (res)                                                                                    \
      hipLaunchKernelGGL((KERNEL<T, true>), grd, blk, 0, s, (const T*)in, (T*)out, g, __VA_ARGS__, resid); \
    else                                                                                        \
      hipLaunchKernelGGL((KERNEL<T, false>), grd, blk, 0, s, (const T*)in, (T*)out, g, __VA_ARGS__, resid); \
  } while (0)
  switch (spec.kind) {
    case StencilKind::Heat7:
      if (spec.dtype == DType::F32)
        MDFX_NAIVE(naive_heat7, float, (float)spec.rate());
      else
        MDFX_NAIVE(naive_heat7, double, spec.rate());
      break;
    case StencilKind::Jacobi5:
      if (spec.dtype == DType::F32)
        MDFX_NAIVE(naive_jacobi5, float, (float)spec.rate(), (int)spec.coef.ref_precision);
      else
        MDFX_NAIVE(naive_jacobi5, double, spec.rate(), (int)spec.coef.ref_precision);
      break;
    case StencilKind::Box27: {
      const auto& c = spec.coef;
      if (spec.dtype == DType::F32)
        MDFX_NAIVE(naive_box27, float, (float)c.c0, (float)c.c1, (float)c.c2, (float)c.c3);
      else
        MDFX_NAIVE(naive_box27, double, c.c0, c.c1, c.c2, c.c3);
      break;
    }
    case StencilKind::Life:
      if (res)
        hipLaunchKernelGGL(naive_life<true>, grd, blk, 0, s, (const uint8_t*)in, (uint8_t*)out, g, resid);
      else
        hipLaunchKernelGGL(naive_life<false>, grd, blk, 0, s, (const uint8_t*)in, (uint8_t*)out, g, resid);
      break;
  }
#undef MDFX_NAIVE
}

}  // namespace dev
}  // namespace mdfx
