// Tuned gfx950 kernel for the 3D 27-point stencil (BASELINE.json config 4).
//
// Same 2.5D z-march as heat7_zw, but the 27 taps are factored into per-plane partial sums
// (stencil_math.hpp): when plane k enters the window each lane computes, for its RY rows,
//   A(k) = c3*diag + c2*cross + c1*center   (what plane k contributes to outputs k-1 and k+1)
//   B(k) = c2*diag + c1*cross + c0*center   (what plane k contributes to output k)
// once, from its own rows plus one halo row above and below, so output k = (A(k-1)+B(k))+A(k+1)
// costs 2 adds, and each input plane is loaded once per chunk (27 taps, 1 read + 1 write per
// cell from HBM). x-neighbours: lane shuffles + LDS for wave edges + one scalar load at the block
// edge, as in heat7_zw.
#include <algorithm>

#include "kcommon.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target);
int env_int(const char* name, int dflt);

template <class V, class T>
__device__ __forceinline__ V vsplat27(T v) {
  V r;
#pragma unroll
  for (int e = 0; e < (int)(sizeof(V) / sizeof(T)); ++e) r[e] = v;
  return r;
}

template <class T, int RY, int WXN, bool RES>
__global__ __launch_bounds__(256) void box27_zw(const T* __restrict__ in, T* __restrict__ out,
                                                Geo g, T c0, T c1, T c2, T c3, int zc, int XT,
                                                int YT, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  constexpr int N = VT<T>::N;
  constexpr int WYN = 4 / WXN;
  constexpr int WX = 64 * N;
  constexpr int RR = RY + 2;  // rows loaded per plane (with the y halo)
  __shared__ T edge[2][4][RR][2];
  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);
  const int xt = t % XT;
  const int yt = (t / XT) % YT;
  const int zt = t / (XT * YT);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wx = w % WXN, wy = w / WXN;
  const int64_t x = ((int64_t)xt * WXN + wx) * WX + (int64_t)lane * N;
  const int64_t y0 = ((int64_t)yt * WYN + wy) * RY;
  const int64_t lzs = g.lz_begin + (int64_t)zt * zc;
  const int64_t lze = min(g.lz_end, lzs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  const T* ib = in + (y0 - 1) * pitch + x;  // row j of the window = y0 - 1 + j
  T* ob = out + y0 * pitch + x;

  auto ld = [&](int64_t lz, int j) -> V {
    V v = vsplat27<V>(T(0));
    const int64_t y = y0 - 1 + j;
    if (xin && lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny)
      v = *(const V*)(ib + lz * plane + (int64_t)j * pitch);
    return v;
  };
  auto ldl = [&](int64_t lz, int j) -> T {
    const int64_t y = y0 - 1 + j;
    if (wx == 0 && lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny)
      return ib[lz * plane + (int64_t)j * pitch - 1];
    return T(0);
  };
  auto ldr = [&](int64_t lz, int j) -> T {
    const int64_t y = y0 - 1 + j;
    if (wx == WXN - 1 && lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max && y >= 0 &&
        y < g.ny)
      return ib[lz * plane + (int64_t)j * pitch + N];
    return T(0);
  };

  V R[RR];
  T EL[RR], ER[RR];
  auto load_plane = [&](int64_t lz) {
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      R[j] = ld(lz, j);
      EL[j] = ldl(lz, j);
      ER[j] = ldr(lz, j);
    }
  };
  int buf = 0;
  // Partials of the plane currently in R[] -> A[], B[] for the RY owned rows; center kept in Cn.
  auto partials = [&](V* A, V* B, V* Cn) {
    if (WXN > 1) {
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < RR; ++j) edge[buf][w][j][0] = R[j][0];
      }
      if (lane == 63) {
#pragma unroll
        for (int j = 0; j < RR; ++j) edge[buf][w][j][1] = R[j][N - 1];
      }
      __syncthreads();
    }
    V H[RR];
#pragma unroll
    for (int j = 0; j < RR; ++j) {
      T l = lane_up1(R[j][N - 1]);
      T rr = lane_down1(R[j][0]);
      if (lane == 0) l = (WXN > 1 && wx > 0) ? edge[buf][w - 1][j][1] : EL[j];
      if (lane == 63) rr = (WXN > 1 && wx < WXN - 1) ? edge[buf][w + 1][j][0] : ER[j];
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const T xm = e == 0 ? l : R[j][e - 1];
        const T xp = e == N - 1 ? rr : R[j][e + 1];
        H[j][e] = xm + xp;
      }
    }
    buf ^= 1;
#pragma unroll
    for (int i = 0; i < RY; ++i) {
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const T center = R[i + 1][e];
        const T cross = H[i + 1][e] + (R[i][e] + R[i + 2][e]);
        const T diag = H[i][e] + H[i + 2][e];
        A[i][e] = sm::box27_A<T>(center, cross, diag, c1, c2, c3);
        if (B) B[i][e] = sm::box27_B<T>(center, cross, diag, c0, c1, c2);
      }
      if (Cn) Cn[i] = R[i + 1];
    }
  };

  V Am[RY], Ac[RY], Bc[RY], Cc[RY];
  load_plane(lzs - 1);
  partials(Am, nullptr, nullptr);
  load_plane(lzs);
  partials(Ac, Bc, Cc);
  load_plane(lzs + 1);
  double acc = 0.0;
  for (int64_t lz = lzs; lz < lze; ++lz) {
    V Ap[RY], Bp[RY], Cp[RY];
    partials(Ap, Bp, Cp);  // plane lz+1 (in R)
    load_plane(lz + 2);    // prefetch; consumed next iteration
    const int64_t gz = lz + g.gz_off;
    const bool zb = (gz == 0 || gz == g.gnz - 1);
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      const int64_t y = y0 + i;
      if (y >= g.ny) break;
      const V c = Cc[i];
      V o = c;
      if (!zb && y != 0 && y != g.ny - 1) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const T v = sm::box27_combine<T>(Am[i][e], Bc[i][e], Ap[i][e]);
          const int64_t xe = x + e;
          o[e] = (xe == 0 || xe >= g.nx - 1) ? c[e] : v;
        }
      }
      if (xin) {
        store_nt((V*)(ob + lz * plane + (int64_t)i * pitch), o);
        if (RES) {
#pragma unroll
          for (int e = 0; e < N; ++e)
            if (x + e < g.nx) {
              const double d = (double)o[e] - (double)c[e];
              acc += d * d;
            }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      Am[i] = Ac[i];
      Ac[i] = Ap[i];
      Bc[i] = Bp[i];
      Cc[i] = Cp[i];
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, int RY, int WXN>
static void launch_box27_t(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                           hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  constexpr int WYN = 4 / WXN;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int XT = (int)((g.nx + WXN * WX - 1) / (WXN * WX));
  const int YT = (int)((g.ny + WYN * RY - 1) / (WYN * RY));
  int zc = env_int("MDFX_ZC", 0);
  if (zc <= 0) zc = pick_zc(planes, (int64_t)XT * YT, 128, 2048);
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)XT * YT * ZT)), blk(256);
  const T c0 = (T)c.c0, c1 = (T)c.c1, c2 = (T)c.c2, c3 = (T)c.c3;
  if (resid)
    hipLaunchKernelGGL((box27_zw<T, RY, WXN, true>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc,
                       XT, YT, resid);
  else
    hipLaunchKernelGGL((box27_zw<T, RY, WXN, false>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3,
                       zc, XT, YT, resid);
}

template <class T, int RY>
static void launch_box27_ry(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                            hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  if (g.nx > 2 * WX)
    launch_box27_t<T, RY, 4>(g, in, out, c, resid, s);
  else if (g.nx > WX)
    launch_box27_t<T, RY, 2>(g, in, out, c, resid, s);
  else
    launch_box27_t<T, RY, 1>(g, in, out, c, resid, s);
}

template <class T>
void launch_box27(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                  hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  int ry = env_int("MDFX_RY", 0);
  if (ry <= 0) ry = 2;
  if (g.ny < 8) ry = 1;
  switch (ry) {
    case 1: launch_box27_ry<T, 1>(g, in, out, c, resid, s); break;
    case 4: launch_box27_ry<T, 4>(g, in, out, c, resid, s); break;
    default: launch_box27_ry<T, 2>(g, in, out, c, resid, s); break;
  }
}
template void launch_box27<float>(const Geo&, const float*, float*, const StencilCoef&, double*,
                                  hipStream_t);
template void launch_box27<double>(const Geo&, const double*, double*, const StencilCoef&, double*,
                                   hipStream_t);

}  // namespace dev
}  // namespace mdfx
