// Temporally blocked 3D 7-point heat/Jacobi: TWO time steps per sweep over memory.
//
// The single-step kernels (stencil_heat.hip) already run at the HBM copy roof (1 read + 1 write
// per cell per step). This kernel reads u^t once and writes u^{t+2} once, computing u^{t+1} on
// chip, so a sweep advances two steps for the same HBM bytes.
//
// Geometry: one block = 4 waves along x; RY rows per lane; the block marches along z over `zc`
// output planes. Rows up to 4 * 64 * N wide (1024 fp32 / 512 fp64) are covered by ONE block, whose
// x edges are then the Dirichlet boundary. Wider rows are cut into aligned x tiles of 4 * 64 * N
// cells (2048^2 rows: exactly 2 tiles). A tile needs two u0 columns of each x neighbour: the edge
// wave streams them (one 16-B vector per row, prefetched a plane ahead, L2 hits) through a small
// LDS plane ring, and its seam lane recomputes the neighbour's u1 column from that ring. Per z-iteration with u1 plane c:
//   u1(c)   rows y0-1 .. y0+RY   from u0 planes c-1, c, c+1 (rows y0-2 .. y0+RY+1 of plane c)
//   u2(c-1) rows y0   .. y0+RY-1 from u1 planes c-2, c-1, c
// u0 planes are loaded once (RY+4 rows each: the y halo rows are L2 hits shared with the
// neighbouring tiles, which the XCD-aware block order keeps on the same XCD); the one redundant u1
// row above and below the tile is recomputed instead of exchanged. x neighbours come from lane
// shuffles plus a 2-deep LDS ring for the 4 wave seams (one barrier per z-iteration).
// The arithmetic is exactly two applications of sm::heat7 with the boundary held, so the result
// is bitwise identical to two single steps (tests/test_gpu_temporal.py).
//
// Region contract: output storage planes [lz_begin, lz_end) need u0 valid on
// [lz_begin - 2, lz_end + 2): the engine keeps 2 ghost planes (halo = 2) when temporal blocking is on.
#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <map>
#include <mutex>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target);

template <class V, class T>
__device__ __forceinline__ V vsplat_tb(T v) {
  V r;
#pragma unroll
  for (int e = 0; e < (int)(sizeof(V) / sizeof(T)); ++e) r[e] = v;
  return r;
}

template <class T, int RY, int WXN, bool RES, int PF, bool XT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(XT && RY <= 2 ? 3 : 1))) void heat7_tb2(const T* __restrict__ in, T* __restrict__ out, Geo g,
                                                 T r, int zc, int YT, int XTn, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  constexpr int N = VT<T>::N;
  constexpr int WX = 64 * N;
  constexpr int WYN = 4 / WXN;  // narrow rows: wave groups stacked along y, each its own RY-row tile
  constexpr int R0 = RY + 4;  // u0 rows y0-2 .. y0+RY+1
  constexpr int R1 = RY + 2;  // u1 rows y0-1 .. y0+RY
  __shared__ T edge[2][4][R1 + RY][2];
  const unsigned t0 = xcd_remap(blockIdx.x, gridDim.x);
  const int xt = XT ? t0 % XTn : 0;  // x tiles fastest: neighbours share their overlap vectors in L2
  const unsigned t = XT ? t0 / XTn : t0;
  const int yt = t % YT;
  const int zt = t / YT;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wx = w % WXN, wy = w / WXN;
  constexpr int TW = WXN * WX;  // x tile width (XT implies WXN == 4)
  const int64_t X0 = (int64_t)xt * TW;
  const int64_t xw = X0 + (int64_t)wx * WX;
  const uint32_t xo = (uint32_t)lane * N;
  const int64_t x = xw + xo;
  const bool hl = XT && X0 > 0, hr = XT && X0 + TW < g.pitch;  // neighbour tiles
  const int64_t y0 = ((int64_t)yt * WYN + wy) * RY;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  const T* ib = in + (y0 - 2) * pitch + xw;  // u0 row r of the window = y0 - 2 + r
  T* ob = out + y0 * pitch + xw;
  // x-held cells (x = 0, x >= nx - 1) get coefficient 0: u' = fma(0, t, u) = u for finite data,
  // no per-cell select (y / z holds are whole rows / planes and branch uniformly)
  T rxe[N];
#pragma unroll
  for (int e = 0; e < N; ++e) rxe[e] = (x + e == 0 || x + e >= g.nx - 1) ? T(0) : r;

  auto ld = [&](int64_t lz, int rr) -> V {
    V v = vsplat_tb<V>(T(0));
    const int64_t y = y0 - 2 + rr;
    if (lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny) {
      const T* p = ib + lz * plane + (int64_t)rr * pitch;
      if (xin) {
        dcheck(g, in, p + xo, N);
        v = *(const V*)(p + xo);
      }
    }
    return v;
  };

  // x-tiled rows: lanes 0..R0-1 of the edge wave stream the two u0 columns beyond the tile edge
  // (one 16-B vector per row) into a 4-plane LDS ring; the seam lane computes the neighbour
  // tile's u1 column from it. Only that one wave writes and reads its side of the ring.
  __shared__ T hx[4][2][R0][2];  // [plane & 3][left/right][window row][adjacent column, next]
  const bool hw = (hl && wx == 0) || (hr && wx == WXN - 1);
  const int side = wx == 0 ? 0 : 1;
  auto ldhv = [&](int64_t lz) -> V {
    V v = vsplat_tb<V>(T(0));
    const int64_t y = y0 - 2 + lane;
    if (lane < R0 && lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny) {
      const T* hp = ib + lz * plane + (int64_t)lane * pitch + (side == 0 ? -N : WX);
      dcheck(g, in, hp, N);
      v = *(const V*)hp;
    }
    return v;
  };
  auto puthv = [&](int64_t lz, V v) {
    if (lane < R0) {
      hx[lz & 3][side][lane][0] = side == 0 ? v[N - 1] : v[0];
      hx[lz & 3][side][lane][1] = side == 0 ? v[N - 2] : v[1];
    }
  };
  // u1 at the neighbour column of side sd, plane p, row y0 + i; `inner` = u0 of this tile's edge cell
  auto u1h = [&](int64_t p, int sd, int i, T inner) -> T {
    const int k = i + 2, sp = (int)(p & 3);
    const T cc = hx[sp][sd][k][0];
    const int64_t y = y0 + i, gz = p + g.gz_off, xh = sd == 0 ? X0 - 1 : X0 + TW;
    if (gz <= 0 || gz >= g.gnz - 1 || y <= 0 || y >= g.ny - 1 || xh >= g.nx - 1) return cc;
    const T out_ = hx[sp][sd][k][1];
    return sm::heat7<T>(cc, sd == 0 ? out_ : inner, sd == 0 ? inner : out_, hx[sp][sd][k - 1][0],
                        hx[sp][sd][k + 1][0], hx[(p - 1) & 3][sd][k][0], hx[(p + 1) & 3][sd][k][0], r);
  };
  V HV;
  if (XT && hw) {
    puthv(zs - 1, ldhv(zs - 1));
    HV = ldhv(zs);
  }

  V L0[R0], M0[R0], H0[R0];  // u0 planes c-1, c, c+1
  V U1a[R1], U1b[R1];        // u1 planes c-2, c-1
#pragma unroll
  for (int k = 0; k < R0; ++k) {
    L0[k] = ld(zs - 2, k);
    M0[k] = ld(zs - 1, k);
    H0[k] = ld(zs, k);
  }
#pragma unroll
  for (int k = 0; k < R1; ++k) {
    U1a[k] = vsplat_tb<V>(T(0));
    U1b[k] = vsplat_tb<V>(T(0));
  }
  double acc = 0.0;
  int buf = 0;
  // c = u1 plane computed this iteration; u2 plane c-1 is produced from c >= zs + 1
  for (int64_t c = zs - 1; c <= ze; ++c) {
    V NX[R0];
    if (PF) {
#pragma unroll
      for (int k = 0; k < R0; ++k) NX[k] = ld(c + 2, k);
    }
    // publish the wave-seam values: u0 plane c rows used for u1, u1 plane c-1 own rows for u2
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < R1; ++j) edge[buf][w][j][0] = M0[j + 1][0];
#pragma unroll
      for (int i = 0; i < RY; ++i) edge[buf][w][R1 + i][0] = U1b[i + 1][0];
    }
    if (lane == 63) {
#pragma unroll
      for (int j = 0; j < R1; ++j) edge[buf][w][j][1] = M0[j + 1][N - 1];
#pragma unroll
      for (int i = 0; i < RY; ++i) edge[buf][w][R1 + i][1] = U1b[i + 1][N - 1];
    }
    if (XT && hw) {  // stream the next u0 halo columns into the ring (plane c+1 now, c+2 prefetched)
      puthv(c + 1, HV);
      HV = ldhv(c + 2);
    }
    lds_barrier();  // s_barrier after the LDS writes only: the register prefetch stays in flight

    // ---- u1 at plane c ------------------------------------------------------------------
    V U1c[R1];
    {
      const int64_t gz = c + g.gz_off;
      const bool zb = (gz <= 0 || gz >= g.gnz - 1);
#pragma unroll
      for (int j = 0; j < R1; ++j) {
        const int64_t y = y0 - 1 + j;
        const V cc = M0[j + 1];
        V o = cc;
        T l = lane_up1(cc[N - 1]);
        T rr = lane_down1(cc[0]);
        if (lane == 0) l = wx > 0 ? edge[buf][w - 1][j][1] : (hl ? hx[c & 3][0][j + 1][0] : T(0));
        if (lane == 63) rr = wx < WXN - 1 ? edge[buf][w + 1][j][0] : (hr ? hx[c & 3][1][j + 1][0] : T(0));
        if (!zb && y > 0 && y < g.ny - 1) {
          const V ym = M0[j], yp = M0[j + 2], zm = L0[j + 1], zp = H0[j + 1];
#pragma unroll
          for (int e = 0; e < N; ++e) {
            const T xm = e == 0 ? l : cc[e - 1];
            const T xp = e == N - 1 ? rr : cc[e + 1];
            o[e] = sm::heat7<T>(cc[e], xm, xp, ym[e], yp[e], zm[e], zp[e], rxe[e]);
          }
        }
        U1c[j] = o;
      }
    }
    // ---- u2 at plane c-1 ----------------------------------------------------------------
    if (c >= zs + 1) {
      const int64_t lz = c - 1;
      const int64_t gz = lz + g.gz_off;
      const bool zb = (gz == 0 || gz == g.gnz - 1);
#pragma unroll
      for (int i = 0; i < RY; ++i) {
        const int64_t y = y0 + i;
        if (y >= g.ny) break;
        const V cc = U1b[i + 1];
        V o = cc;
        T l = lane_up1(cc[N - 1]);
        T rr = lane_down1(cc[0]);
        if (lane == 0) l = wx > 0 ? edge[buf][w - 1][R1 + i][1] : (hl ? u1h(lz, 0, i, L0[i + 2][0]) : T(0));
        if (lane == 63) rr = wx < WXN - 1 ? edge[buf][w + 1][R1 + i][0] : (hr ? u1h(lz, 1, i, L0[i + 2][N - 1]) : T(0));
        if (!zb && y != 0 && y != g.ny - 1) {
          const V ym = U1b[i], yp = U1b[i + 2], zm = U1a[i + 1], zp = U1c[i + 1];
#pragma unroll
          for (int e = 0; e < N; ++e) {
            const T xm = e == 0 ? l : cc[e - 1];
            const T xp = e == N - 1 ? rr : cc[e + 1];
            o[e] = sm::heat7<T>(cc[e], xm, xp, ym[e], yp[e], zm[e], zp[e], rxe[e]);
          }
        }
        if (xin) {
          dcheck(g, (const T*)out, ob + lz * plane + (int64_t)i * pitch + xo, N);
          store_nt((V*)(ob + lz * plane + (int64_t)i * pitch + xo), o);
          if (RES) {
#pragma unroll
            for (int e = 0; e < N; ++e)
              if (x + e < g.nx) {
                const double d = (double)o[e] - (double)cc[e];
                acc += d * d;
              }
          }
        }
      }
    }
    buf ^= 1;
#pragma unroll
    for (int k = 0; k < R1; ++k) {
      U1a[k] = U1b[k];
      U1b[k] = U1c[k];
    }
#pragma unroll
    for (int k = 0; k < R0; ++k) {
      L0[k] = M0[k];
      M0[k] = H0[k];
      H0[k] = PF ? NX[k] : ld(c + 2, k);
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T>
bool heat7_tb2_supported(const Geo& g) {
  constexpr int WX = 64 * VT<T>::N;
  (void)WX;  // any row width: rows wider than one block are x-tiled
  return g.nx >= 1 && g.ny >= 1;
}
template bool heat7_tb2_supported<float>(const Geo&);
template bool heat7_tb2_supported<double>(const Geo&);

// Blocks of kernel `kfn` (of `block` threads, default 256) the whole device holds at once, cached
// per kernel and block size.
int64_t resident_blocks(const void* kfn, int block) {
  static std::mutex mu;
  static std::map<std::pair<int, std::pair<const void*, int>>, int64_t> cache;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({dev, {kfn, block}});
  if (it != cache.end()) return it->second;
  int cus = 0, nb = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kfn, block, 0) != hipSuccess || nb <= 0) nb = block > 256 ? 1 : 2;
  return cache[{dev, {kfn, block}}] = (int64_t)cus * nb;
}
int64_t resident_blocks(const void* kfn) { return resident_blocks(kfn, 256); }

// z-chunk of a fused sweep over `planes` planes and `tiles` xy tiles: balanced chunks of about 43
// planes (equal up to one plane), shortened while the grid would not fill the device once.
// Short chunks keep y-neighbour tiles at nearly the same z, so they share their halo rows in the
// XCD's L2 (zc 128 fetched 2.00x the field, zc 32 1.25x: profiles/archive/r01_tb2_zc_sweep.txt); balanced
// ~43-plane chunks were the best or within 1% of it at every slab depth of the 1024^2 strong-
// scaling shapes, e.g. 1024 x 1024 x 128 (the N = 8 slab): 876 GCells/s at zc 64 vs 1043 at zc 43
// (profiles/archive/r01_tb2_zc_slabs.txt).
int tb2_zc(int64_t planes, int64_t tiles, int64_t resident) {
  if (planes <= 16) return (int)std::max<int64_t>(planes, 1);
  int64_t zt = (planes + 43) / 44;
  int64_t zc = (planes + zt - 1) / zt;
  while (zt * tiles < resident && zc > 16) {
    ++zt;
    zc = (planes + zt - 1) / zt;
  }
  return (int)zc;
}

// Rows wider than one block (the streaming heat7_tbk covers rows within one block): aligned x
// tiles of 4 * 64 * N cells, RY rows each, the next u0 plane prefetched into registers.
template <class T, int RY>
static void launch_tb2_xt(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int N = VT<T>::N, WX = 64 * N;
  const int XTn = (int)((g.pitch + 4 * WX - 1) / (4 * WX));
  const int64_t planes = g.lz_end - g.lz_begin;
  const int YT = (int)((g.ny + RY - 1) / RY);
  const void* kfn = (const void*)&heat7_tb2<T, RY, 4, false, 1, true>;
  const int zc = tb2_zc(planes, (int64_t)XTn * YT, resident_blocks(kfn));
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)XTn * YT * ZT)), blk(256);
  if (resid)
    hipLaunchKernelGGL((heat7_tb2<T, RY, 4, true, 1, true>), grd, blk, 0, s, in, out, g, r, zc, YT, XTn, resid);
  else
    hipLaunchKernelGGL((heat7_tb2<T, RY, 4, false, 1, true>), grd, blk, 0, s, in, out, g, r, zc, YT, XTn, resid);
}

template <class T>
void launch_heat7_tb2(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  MDFX_CHECK(g.pitch > 4 * 64 * VT<T>::N, "heat7_tb2 serves rows wider than one block (heat7_tbk covers the rest)");
  // RY = 2 (MDFX_TB_RY=1 for one row per tile): f64 2048^3 533 GCells/s vs 505 at RY = 4 and 429 at
  // RY = 1, and the x-tiled heat7_tbk at 483 (profiles/archive/r02_ab_f64_2048.txt)
  if (knobs().tb_ry == 1 || g.ny < 8)
    launch_tb2_xt<T, 1>(g, in, out, r, resid, s);
  else
    launch_tb2_xt<T, 2>(g, in, out, r, resid, s);
}
template void launch_heat7_tb2<float>(const Geo&, const float*, float*, float, double*, hipStream_t);
template void launch_heat7_tb2<double>(const Geo&, const double*, double*, double, double*, hipStream_t);

// ---- 2D 5-point, two steps per sweep ----------------------------------------------------------
//
// The reference's own program (MDF_kernel.cu:10-22) fused like heat7_tb2: rows are planes
// (ny == 1) and each wave is an independent task (x segment of 64*N values, zc rows), so there is
// no block barrier. Per row c the wave computes u1(c) for its segment and, in lanes 0 / 63, u1 at
// the one column beyond each segment edge (from a 16-B halo vector those lanes load), then
// u2(c-1) for the segment. u0 is read once (+ 2 halo vectors per 64 lanes, L2 hits), u2 written
// once; bitwise equal to two sm::jacobi5 steps.
template <class T, bool RES>
__global__ __launch_bounds__(256) void jacobi5_tb2(const T* __restrict__ in, T* __restrict__ out, Geo g, T r,
                                                   int zc, int XT, int ntasks, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  constexpr int N = VT<T>::N;
  constexpr int WX = 64 * N;
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform; no block barriers in this kernel
  const int xt = task % XT, zt = task / XT;
  const int64_t x0 = (int64_t)xt * WX;
  const int64_t x = x0 + (int64_t)lane * N;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t plane = g.plane;
  // halo column of this lane: lane 0 -> x0-1 (vector [x0-N, x0)), lane 63 -> x0+WX (vector at x0+WX)
  const int64_t hcol = lane == 0 ? x0 - 1 : x0 + WX;
  const int64_t hvec = lane == 0 ? x0 - N : x0 + WX;
  const bool hin = (lane == 0 && x0 > 0) || (lane == 63 && x0 + WX < g.pitch);
  const int ha = lane == 0 ? N - 1 : 0;  // element of the halo vector at hcol
  const int hb = lane == 0 ? N - 2 : 1;  // element one further out
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);
  const bool hbnd = hcol <= 0 || hcol >= g.nx - 1;

  auto ld = [&](int64_t lz) -> V {
    V v = vsplat_tb<V>(T(0));
    if (xin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x, N);
      v = *(const V*)(in + lz * plane + x);
    }
    return v;
  };
  auto ldh = [&](int64_t lz) -> V {
    V v = vsplat_tb<V>(T(0));
    if (hin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + hvec, N);
      v = *(const V*)(in + lz * plane + hvec);
    }
    return v;
  };
  V L = ld(zs - 2), M = ld(zs - 1), H = ld(zs);
  V HL = ldh(zs - 2), HM = ldh(zs - 1), HH = ldh(zs);
  V Ua = vsplat_tb<V>(T(0)), Ub = Ua;
  T ub = T(0);  // u1 at the halo column, row c-1
  double acc = 0.0;
  for (int64_t c = zs - 1; c <= ze; ++c) {
    const V NX = ld(c + 2), NXH = ldh(c + 2);
    // ---- u1 at row c: the segment, then the halo column (lanes 0 / 63)
    const int64_t gz = c + g.gz_off;
    const bool zb = gz <= 0 || gz >= g.gnz - 1;
    V Uc = M;
    T uc = HM[ha];
    {
      T l = lane_up1(M[N - 1]);
      T rr = lane_down1(M[0]);
      if (lane == 0) l = HM[N - 1];
      if (lane == 63) rr = HM[0];
      if (!zb) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const T xm = e == 0 ? l : M[e - 1];
          const T xp = e == N - 1 ? rr : M[e + 1];
          const T v = sm::jacobi5<T>(M[e], xm, xp, L[e], H[e], r);
          Uc[e] = xb[e] ? M[e] : v;
        }
        if (!hbnd) {  // lane 0: neighbours x0-2 | x0 ; lane 63: x0+WX-1 | x0+WX+1
          const T xm = lane == 0 ? HM[hb] : M[N - 1];
          const T xp = lane == 0 ? M[0] : HM[hb];
          uc = sm::jacobi5<T>(HM[ha], xm, xp, HL[ha], HH[ha], r);
        }
      }
    }
    // ---- u2 at row c-1
    if (c >= zs + 1) {
      const int64_t lz = c - 1;
      const int64_t gz2 = lz + g.gz_off;
      V o = Ub;
      T l = lane_up1(Ub[N - 1]);
      T rr = lane_down1(Ub[0]);
      if (lane == 0) l = ub;
      if (lane == 63) rr = ub;
      if (gz2 != 0 && gz2 != g.gnz - 1) {
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const T xm = e == 0 ? l : Ub[e - 1];
          const T xp = e == N - 1 ? rr : Ub[e + 1];
          const T v = sm::jacobi5<T>(Ub[e], xm, xp, Ua[e], Uc[e], r);
          o[e] = xb[e] ? Ub[e] : v;
        }
      }
      if (xin) {
        dcheck(g, (const T*)out, out + lz * plane + x, N);
        store_nt((V*)(out + lz * plane + x), o);
        if (RES) {
#pragma unroll
          for (int e = 0; e < N; ++e)
            if (x + e < g.nx) {
              const double d = (double)o[e] - (double)Ub[e];
              acc += d * d;
            }
        }
      }
    }
    L = M;
    M = H;
    H = NX;
    HL = HM;
    HM = HH;
    HH = NXH;
    Ua = Ub;
    Ub = Uc;
    ub = uc;
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T>
void launch_jacobi5_tb2(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int WX = 64 * VT<T>::N;
  const int XT = (int)((g.nx + WX - 1) / WX);
  const int zc = pick_zc(planes, XT, 256, 4 * 2048);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL((jacobi5_tb2<T, true>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL((jacobi5_tb2<T, false>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
}
template void launch_jacobi5_tb2<float>(const Geo&, const float*, float*, float, double*, hipStream_t);
template void launch_jacobi5_tb2<double>(const Geo&, const double*, double*, double, double*, hipStream_t);

// ---- 2D 5-point, K steps per sweep ------------------------------------------------------------
//
// Deep temporal blocking for the 2D problem. Wave segments OVERLAP by OV = ceil(K / N) lanes on each
// side: a wave covers 64 lanes x N columns but owns only lanes OV..63-OV, so the outer lanes carry
// the neighbour segments' edge columns through the same SIMD instructions. Each level of the
// pipeline corrupts one more column from the outside in (the outermost neighbour is unknown), so
// after K <= OV * N levels the owned lanes are still exact and are the only ones stored.
// Each level is a streaming recurrence over rows, as in heat7_tbk: its only state between rows is
// the partial sum S = (xm + xp) + zm of row p and the centre C = u_{l-1}(p). When u_{l-1}(p+1)
// arrives it finishes u_l(p) = fma(r, fma(-4, C, S + zp), C) -- sm::jacobi5's operation order, so
// bitwise equal to K single steps -- and replaces S / C with row p+1's. No register rotation, and
// held cells take a zero coefficient (fma(0, t, u) = u for finite t; every lane, inside the grid or
// not, holds finite data) instead of a select. One read and one write of the field per K steps.
// REF: the reference program's own evaluation of every level (sm::jacobi5_ref, MDF_kernel.cu:20,
// SURVEY D17): the fp32 sum and -4u term as usual, then r * t + u as ONE fp64 fma of the widened
// values, rounded back to fp32. Held cells stay exact (fma(0, t, u) = u). fp64 fields: identical.
// MODE (fp32): 2 = rows in the natural pair layout (RowOpsN: no regrouping after a 16-B load, x
// sums as scalar adds with DPP-folded lane shifts) and the row loop unrolled by two with the
// loop-carried centres ping-ponged between two arrays (no per-row centre copies); 0 = round 2's
// pair layout (RowOps<float>). fp64 runs mode 0.
template <class T, int K, bool RES, bool REF, int MODE>
__global__ __launch_bounds__(256) void jacobi5_tbk(const T* __restrict__ in, T* __restrict__ out, Geo g, T r,
                                                   int zc, int XT, int ntasks, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  using RO = typename std::conditional<sizeof(T) == 4 && MODE >= 1, RowOpsN, RowOps<T>>::type;
  using Row = typename RO::Row;
  constexpr int N = VT<T>::N;
  constexpr int OV = (K + N - 1) / N;  // overlap lanes per side
  constexpr int SEG = (64 - 2 * OV) * N;  // owned columns per wave
  // u0 rows in flight: MODE 2 two, MODE 3 four (the row loop unrolled by as many); modes 0 / 1 one
  constexpr int PD = MODE == 3 ? 4 : MODE == 2 ? 2 : 1;
  const int lane = threadIdx.x & 63;
  // wave-uniform task index in an SGPR, so every row index and row test below is scalar
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform; no block barriers in this kernel
  const int xt = task % XT, zt = task / XT;
  const int64_t x = (int64_t)xt * SEG - OV * N + (int64_t)lane * N;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x >= 0 && x < g.pitch;
  const bool own = lane >= OV && lane <= 63 - OV && xin;
  const int64_t plane = g.plane;
  // per-cell coefficient 0 on the held columns x = 0, x >= nx - 1
  bool held[N];
#pragma unroll
  for (int e = 0; e < N; ++e) held[e] = (x + e == 0) || (x + e >= g.nx - 1);
  const Row rx = RO::coef(r, held);
  // Loads without lane predication: lanes outside the row read the nearest in-row vector and rows
  // past the storage read its last row. Those values are finite and only ever meet held or unowned
  // cells (the left halo lane of the first segment feeds only x = 0, which is held; lanes beyond
  // the row feed only x >= nx - 1 and themselves).
  const T* ib = in + (x < 0 ? 0 : x >= g.pitch ? g.pitch - N : x);
  auto ld = [&](int64_t lz) -> Row {
    const int64_t lzc = lz < 0 ? 0 : lz >= g.lz_max ? g.lz_max - 1 : lz;
    dcheck(g, in, ib + lzc * plane, N);
    return RO::lds(ib + lzc * plane);  // one 16-B vector
  };
  Row S[K], CA[K], CB[K];  // level l = 1..K at index l - 1
#pragma unroll
  for (int l = 0; l < K; ++l) {
    S[l] = RO::zero();
    CA[l] = RO::zero();
    CB[l] = RO::zero();
  }
  Row nx = ld(zs - K);
  double acc = 0.0;
  const int64_t qlast = ze - 1 + K;
  // newest u0 row q; level l finishes row q - l (each level's first two rows are priming garbage
  // that no level needs). Rows of the chunk's pipeline (zs - K - 1 .. ze + K - 1) that are all
  // interior in z need no z test: one loop copy without it, one with the per-level test for chunks
  // at the z boundary.
  const bool zint = zs - K - 1 + g.gz_off >= 1 && ze + K - 1 + g.gz_off <= g.gnz - 2;
  // MODE 2 / 3 keep PD rows in flight (u0 rows q + 1 .. q + PD load while row q is consumed): one
  // row of K-level work is far shorter than a loaded global-load round trip at 2-3 waves per SIMD
  // (16384^2 fp32 K = 8: 4487-4515 GCells/s with two rows in flight vs 4202-4208 with one,
  // profiles/archive/r03_session_aa/)
  Row nxr[PD];
  nxr[0] = nx;
#pragma unroll
  for (int i = 1; i < PD; ++i) nxr[i] = ld(zs - K + i);
  auto row_step = [&](int64_t q, Row(&Cin)[K], Row(&Cout)[K], auto ztest, auto slot) __attribute__((always_inline)) {
    constexpr bool ZT = decltype(ztest)::value;
    constexpr int SL = decltype(slot)::value;  // which in-flight row is row q
    Row X = nxr[SL];
    nxr[SL] = ld(q + PD);
#pragma unroll
    for (int l = 1; l <= K; ++l) {
      const int64_t row = q - l;
      const int64_t gz = row + g.gz_off;
      // z-held rows through a wave-uniform 0 / 1 factor (r * 1 = r, r * 0 = +0; a Row-valued select
      // here was lowered to a scratch-memory table)
      const Row rc = ZT ? RO::scale(rx, (gz <= 0 || gz >= g.gnz - 1) ? T(0) : T(1)) : rx;
      const Row c = Cin[l - 1];
      const Row o = REF ? RO::fin4_ref(S[l - 1], X, c, rc) : RO::fin4(S[l - 1], X, c, rc);
      // row + 1's partial from the arriving row X: (xm + xp) + zm
      const T lft = lane_up1(RO::last(X));
      const T rgt = lane_down1(RO::first(X));
      S[l - 1] = RO::partial5(X, lft, rgt, c);
      RO::pin(S[l - 1]);
      Cout[l - 1] = X;
      if (l < K) {
        X = o;
      } else if (row >= zs && q <= qlast && own) {
        dcheck(g, (const T*)out, out + row * plane + x, N);
        store_nt((V*)(out + row * plane + x), RO::vec(o));
        if (RES) {
#pragma unroll
          for (int e = 0; e < N; ++e)
            if (x + e < g.nx) {
              const double d = (double)RO::get(o, e) - (double)RO::get(c, e);
              acc += d * d;
            }
        }
      }
    }
  };
  auto march = [&](auto ztest) __attribute__((always_inline)) {
    if constexpr (MODE == 2) {
      // an odd row count ends with one extra row (q = qlast + 1): loads clamp, nothing is stored
      for (int64_t q = zs - K; q <= qlast; q += 2) {
        row_step(q, CA, CB, ztest, std::integral_constant<int, 0>{});
        row_step(q + 1, CB, CA, ztest, std::integral_constant<int, 1>{});
      }
    } else {
      for (int64_t q = zs - K; q <= qlast; ++q) row_step(q, CA, CA, ztest, std::integral_constant<int, 0>{});
    }
  };
  // (fp64: one loop copy with the test; the second copy costs the VGPRs of occupancy 4 at K = 8)
  if (zint && sizeof(T) == 4)
    march(std::integral_constant<bool, false>{});
  else
    march(std::integral_constant<bool, true>{});
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, int K, bool REF, int MODE>
static void launch_jacobi5_tbk_km(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int N = VT<T>::N, OV = (K + N - 1) / N, SEG = (64 - 2 * OV) * N;
  const int XT = (int)((g.nx + SEG - 1) / SEG);
  const int zc = pick_zc(planes, XT, 256, 4 * 2048);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL((jacobi5_tbk<T, K, true, REF, MODE>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL((jacobi5_tbk<T, K, false, REF, MODE>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
}

// fp32: the natural layout with the 2-row unroll (mode 2); the reference-precision instance keeps
// 4 waves per SIMD without the unroll (mode 1; 16384^2 K = 8: 3346-3368 GCells/s vs 3131-3145
// unrolled at 2 waves per SIMD). fp64: the pair rows (RowOps<double>) with the 2-row unroll and two
// u0 rows in flight (mode 2; 16384^2 K = 8: 2216-2219 vs 2005 GCells/s for mode 0,
// profiles/archive/r03_session_ac/). Round 2's fp32 pair layout and fp64 mode 0, and a 4-row unroll
// (mode 3), measured slower and were removed in round 4 (profiles/archive/r03_mdf2d/, r03_session_ac/).
template <class T, int K, bool REF>
static void launch_jacobi5_tbk_k(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  if constexpr (sizeof(T) == 4 && REF)
    launch_jacobi5_tbk_km<T, K, REF, 1>(g, in, out, r, resid, s);
  else
    launch_jacobi5_tbk_km<T, K, REF, 2>(g, in, out, r, resid, s);
}

template <class T, bool REF>
static void launch_jacobi5_tbk_r(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s) {
  switch (steps) {
    case 2: launch_jacobi5_tbk_k<T, 2, REF>(g, in, out, r, resid, s); break;
    case 3: launch_jacobi5_tbk_k<T, 3, REF>(g, in, out, r, resid, s); break;
    case 4: launch_jacobi5_tbk_k<T, 4, REF>(g, in, out, r, resid, s); break;
    case 6: launch_jacobi5_tbk_k<T, 6, REF>(g, in, out, r, resid, s); break;
    case 8: launch_jacobi5_tbk_k<T, 8, REF>(g, in, out, r, resid, s); break;
    default: break;
  }
}

// ref_precision (fp32 only; an fp64 field evaluates the reference's update exactly as sm::jacobi5)
template <class T>
void launch_jacobi5_tbk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s,
                        bool ref_precision) {
  if constexpr (sizeof(T) == 4) {
    if (ref_precision) return launch_jacobi5_tbk_r<T, true>(g, in, out, r, steps, resid, s);
  }
  launch_jacobi5_tbk_r<T, false>(g, in, out, r, steps, resid, s);
}
template void launch_jacobi5_tbk<float>(const Geo&, const float*, float*, float, int, double*, hipStream_t, bool);
template void launch_jacobi5_tbk<double>(const Geo&, const double*, double*, double, int, double*, hipStream_t, bool);

}  // namespace dev
}  // namespace mdfx
