// Tuned gfx950 kernels for the 3D 7-point heat/Jacobi stencil (headline benchmark) and the 2D
// 5-point MDF stencil.
//
// heat7_zw: 2.5D blocking. A 256-thread block = 4 waves arranged WXN (along x) x WYN (along y).
// Every lane owns one 16-byte vector (4 fp32 / 2 fp64) of RY consecutive rows and marches along z
// through `zc` planes, keeping planes z-1, z, z+1 of its rows in registers (no re-read of the
// z-neighbours: each input byte crosses HBM once per chunk). In-plane neighbours:
//   x +-1   : lane shuffles (ds_bpermute), the wave-segment edge from the neighbouring wave
//             through a 2-deep LDS ring, and the block edge from one scalar global load;
//   y +-1   : the lane's own registers except the top / bottom halo row (2 vector loads / plane).
// Plane z+2 (own rows) and the halo rows / edges of z+1 are prefetched one iteration ahead so a
// wave keeps ~RY+2 KiB of loads in flight. Stores are non-temporal (the next sweep reads the
// output after ~8 GiB of other traffic: keeping it in L2/MALL only evicts useful lines).
// Block->tile order is XCD-aware so vertically adjacent tiles (sharing halo rows) share an L2.
//
// Measured (bench/kernel_ab.py, 1024^3 fp32, one MI355X): RY=2 rows per lane, 4 waves along x
// (one block spans the 1024-wide row, so no block-edge loads), prefetch depth 1: 1.546 ms per
// sweep = 694.5 GCells/s = 5.56 TB/s at 8 B/cell, vs 3.18 ms for the one-cell-per-lane kernel and
// 1.63 ms for torch's copy_ of the same bytes.
//
// Reference parity: replaces run_mdf + middle_kernel/border_kernel (MDF_kernel.cu:10-70): the
// "region" is [lz_begin, lz_end), so the same kernel serves the interior and the boundary planes.
#include <algorithm>

#include "kcommon.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

template <class V, class T>
__device__ __forceinline__ V vsplat(T v) {
  V r;
#pragma unroll
  for (int e = 0; e < (int)(sizeof(V) / sizeof(T)); ++e) r[e] = v;
  return r;
}

template <class T, int RY, int WXN, bool RES, bool EDGE, int PF>
__global__ __launch_bounds__(256) void heat7_zw(const T* __restrict__ in, T* __restrict__ out, Geo g,
                                                T r, int zc, int XT, int YT,
                                                double* __restrict__ resid) {
  using V = typename VT<T>::type;
  constexpr int N = VT<T>::N;
  constexpr int WYN = 4 / WXN;
  constexpr int WX = 64 * N;
  __shared__ T edge[2][4][RY][2];
  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);
  const int xt = t % XT;
  const int yt = (t / XT) % YT;
  const int zt = t / (XT * YT);
  const int lane = threadIdx.x & 63;
  // wave index made provably uniform: every row / plane address below is an SGPR base plus ONE
  // per-lane 32-bit offset (global_load saddr form), which keeps the register file for data.
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wx = w % WXN, wy = w / WXN;
  const int64_t xw = ((int64_t)xt * WXN + wx) * WX;
  const uint32_t xo = (uint32_t)lane * N;
  const int64_t x = xw + xo;
  const int64_t y0 = ((int64_t)yt * WYN + wy) * RY;
  const int64_t lzs = g.lz_begin + (int64_t)zt * zc;
  const int64_t lze = min(g.lz_end, lzs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  const T* ib = in + y0 * pitch + xw;
  T* ob = out + y0 * pitch + xw;

  auto ld = [&](int64_t lz, int i) -> V {
    V v = vsplat<V>(T(0));
    const int64_t y = y0 + i;
    if (lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny) {
      const T* p = ib + lz * plane + (int64_t)i * pitch;
      if (xin) {
        dcheck(g, in, p + xo, N);
        v = *(const V*)(p + xo);
      }
    }
    return v;
  };
  auto ldl = [&](int64_t lz, int i) -> T {
    if (!EDGE) return T(0);
    const int64_t y = y0 + i;
    if (wx == 0 && lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max && y < g.ny) {
      dcheck(g, in, ib + lz * plane + (int64_t)i * pitch - 1, 1);
      return ib[lz * plane + (int64_t)i * pitch - 1];
    }
    return T(0);
  };
  auto ldr = [&](int64_t lz, int i) -> T {
    if (!EDGE) return T(0);
    const int64_t y = y0 + i;
    if (wx == WXN - 1 && lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max && y < g.ny) {
      dcheck(g, in, ib + lz * plane + (int64_t)i * pitch + WX, 1);
      return ib[lz * plane + (int64_t)i * pitch + WX];
    }
    return T(0);
  };

  V P[RY], C[RY], Nx[RY];
  T EL[RY], ER[RY];
#pragma unroll
  for (int i = 0; i < RY; ++i) {
    P[i] = ld(lzs - 1, i);
    C[i] = ld(lzs, i);
    if (PF == 2) Nx[i] = ld(lzs + 1, i);
    EL[i] = ldl(lzs, i);
    ER[i] = ldr(lzs, i);
  }
  V HL = ld(lzs, -1), HH = ld(lzs, RY);
  double acc = 0.0;
  int buf = 0;
  for (int64_t lz = lzs; lz < lze; ++lz) {
    // PF == 2: the own rows of plane z+2 and the halo/edges of z+1 are in flight during plane z.
    // PF == 1: only plane z+1 is loaded here (fewer registers, more waves hide the latency).
    V NN[RY];
    T ELN[RY], ERN[RY];
    V HLN, HHN;
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      if (PF == 2)
        NN[i] = ld(lz + 2, i);
      else
        Nx[i] = ld(lz + 1, i);
      if (PF == 2) {
        ELN[i] = ldl(lz + 1, i);
        ERN[i] = ldr(lz + 1, i);
      }
    }
    if (PF == 2) {
      HLN = ld(lz + 1, -1);
      HHN = ld(lz + 1, RY);
    }
    if (WXN > 1) {
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < RY; ++i) edge[buf][w][i][0] = C[i][0];
      }
      if (lane == 63) {
#pragma unroll
        for (int i = 0; i < RY; ++i) edge[buf][w][i][1] = C[i][N - 1];
      }
      lds_barrier();  // s_barrier after the LDS writes only: the register prefetch stays in flight
    }
    const int64_t gz = lz + g.gz_off;
    const bool zb = (gz == 0 || gz == g.gnz - 1);
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      const int64_t y = y0 + i;
      if (y >= g.ny) break;
      const V c = C[i];
      V o = c;
      T l = lane_up1(c[N - 1]);
      T rr = lane_down1(c[0]);
      if (lane == 0) l = (WXN > 1 && wx > 0) ? edge[buf][w - 1][i][1] : EL[i];
      if (lane == 63) rr = (WXN > 1 && wx < WXN - 1) ? edge[buf][w + 1][i][0] : ER[i];
      if (!zb && y != 0 && y != g.ny - 1) {
        const V ym = i > 0 ? C[i - 1] : HL;
        const V yp = i < RY - 1 ? C[i + 1] : HH;
        const V zm = P[i], zp = Nx[i];
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const T xm = e == 0 ? l : c[e - 1];
          const T xp = e == N - 1 ? rr : c[e + 1];
          const T v = sm::heat7<T>(c[e], xm, xp, ym[e], yp[e], zm[e], zp[e], r);
          const int64_t xe = x + e;
          o[e] = (xe == 0 || xe >= g.nx - 1) ? c[e] : v;
        }
      }
      if (xin) {
        dcheck(g, (const T*)out, ob + lz * plane + (int64_t)i * pitch + xo, N);
        store_nt((V*)(ob + lz * plane + (int64_t)i * pitch + xo), o);
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
    buf ^= 1;
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      P[i] = C[i];
      C[i] = Nx[i];
      if (PF == 2) {
        Nx[i] = NN[i];
        EL[i] = ELN[i];
        ER[i] = ERN[i];
      } else {
        EL[i] = ldl(lz + 1, i);
        ER[i] = ldr(lz + 1, i);
      }
    }
    if (PF == 2) {
      HL = HLN;
      HH = HHN;
    } else {
      HL = ld(lz + 1, -1);
      HH = ld(lz + 1, RY);
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

// 2D 5-point: rows are planes (ny == 1). Each wave is an independent task (x segment of 64*N
// values, zc rows); block = 4 tasks. Wave-edge x neighbours come from scalar global loads.
template <class T, bool RES, bool REF>
__global__ __launch_bounds__(256) void jacobi5_wave(const T* __restrict__ in, T* __restrict__ out,
                                                    Geo g, T r, int zc, int XT, int ntasks,
                                                    double* __restrict__ resid) {
  using V = typename VT<T>::type;
  constexpr int N = VT<T>::N;
  constexpr int WX = 64 * N;
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform; no block barriers in this kernel
  const int xt = task % XT, zt = task / XT;
  const int64_t x = (int64_t)xt * WX + (int64_t)lane * N;
  const int64_t lzs = g.lz_begin + (int64_t)zt * zc;
  const int64_t lze = min(g.lz_end, lzs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t plane = g.plane;
  auto ld = [&](int64_t lz) -> V {
    V v = vsplat<V>(T(0));
    if (xin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x, N);
      v = *(const V*)(in + lz * plane + x);
    }
    return v;
  };
  auto ldl = [&](int64_t lz) -> T {
    if (lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x - 1, 1);
      return in[lz * plane + x - 1];
    }
    return T(0);
  };
  auto ldr = [&](int64_t lz) -> T {
    if (lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x + N, 1);
      return in[lz * plane + x + N];
    }
    return T(0);
  };
  V P = ld(lzs - 1), C = ld(lzs), Nx = ld(lzs + 1);
  T EL = ldl(lzs), ER = ldr(lzs);
  double acc = 0.0;
  for (int64_t lz = lzs; lz < lze; ++lz) {
    const V NN = ld(lz + 2);
    const T ELN = ldl(lz + 1), ERN = ldr(lz + 1);
    const int64_t gz = lz + g.gz_off;
    const V c = C;
    V o = c;
    T l = lane_up1(c[N - 1]);
    T rr = lane_down1(c[0]);
    if (lane == 0) l = EL;
    if (lane == 63) rr = ER;
    if (gz != 0 && gz != g.gnz - 1) {
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const T xm = e == 0 ? l : c[e - 1];
        const T xp = e == N - 1 ? rr : c[e + 1];
        const T v = REF ? sm::jacobi5_ref<T>(c[e], xm, xp, P[e], Nx[e], r)
                        : sm::jacobi5<T>(c[e], xm, xp, P[e], Nx[e], r);
        const int64_t xe = x + e;
        o[e] = (xe == 0 || xe >= g.nx - 1) ? c[e] : v;
      }
    }
    if (xin) {
      dcheck(g, (const T*)out, out + lz * plane + x, N);
      store_nt((V*)(out + lz * plane + x), o);
      if (RES) {
#pragma unroll
        for (int e = 0; e < N; ++e)
          if (x + e < g.nx) {
            const double d = (double)o[e] - (double)c[e];
            acc += d * d;
          }
      }
    }
    P = C;
    C = Nx;
    Nx = NN;
    EL = ELN;
    ER = ERN;
  }
  if (RES) wave_atomic_add(resid, acc);
}

// ---- launch helpers ---------------------------------------------------------------------------

// Pick the z-chunk so the grid has >= ~8 blocks per CU (2048) without chunks so short that the
// 2 extra planes each chunk re-reads dominate.
int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target) {
  if (planes <= 0) return 1;
  int64_t chunks = (blocks_target + columns - 1) / std::max<int64_t>(columns, 1);
  chunks = std::max<int64_t>(chunks, 1);
  int64_t zc = (planes + chunks - 1) / chunks;
  zc = std::max<int64_t>(zc, 8);
  zc = std::min<int64_t>(zc, zc_max);
  return (int)std::max<int64_t>(zc, 1);
}

template <class T, int RY, int WXN, bool EDGE, int PF>
static void launch_heat7_t(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int N = VT<T>::N;
  constexpr int WX = 64 * N;
  constexpr int WYN = 4 / WXN;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int XT = (int)((g.nx + WXN * WX - 1) / (WXN * WX));
  const int YT = (int)((g.ny + WYN * RY - 1) / (WYN * RY));
  // ~16 blocks per CU: 512^3 fp32 ran 0.2018 ms at 4096 blocks vs 0.2296 ms at 2048
  const int zc = pick_zc(planes, (int64_t)XT * YT, 128, 4096);
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)XT * YT * ZT)), blk(256);
  if (resid)
    hipLaunchKernelGGL((heat7_zw<T, RY, WXN, true, EDGE, PF>), grd, blk, 0, s, in, out, g, r, zc, XT, YT, resid);
  else
    hipLaunchKernelGGL((heat7_zw<T, RY, WXN, false, EDGE, PF>), grd, blk, 0, s, in, out, g, r, zc, XT, YT, resid);
}

template <class T, int RY, int WXN>
static void launch_heat7_e(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  // planes of prefetch: 1 for fp32, 2 for fp64 (bench/kernel_ab.py, see launch_heat7)
  constexpr int PF = sizeof(T) == 4 ? 1 : 2;
  // one block spans the whole row: the x neighbours at the block edge are the Dirichlet
  // boundary, so the block-edge loads vanish from the kernel.
  // (launch_heat7_ry picks fewer x waves only for rows that fit them: only 4-wave rows have edges)
  if constexpr (WXN == 4) {
    if (g.nx > (int64_t)WXN * WX) return launch_heat7_t<T, RY, WXN, true, PF>(g, in, out, r, resid, s);
  }
  launch_heat7_t<T, RY, WXN, false, PF>(g, in, out, r, resid, s);
}

template <class T, int RY>
static void launch_heat7_ry(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  // waves along x only as far as the row is wide; the rest stack along y.
  if (g.nx > 2 * WX)
    launch_heat7_e<T, RY, 4>(g, in, out, r, resid, s);
  else if (g.nx > WX)
    launch_heat7_e<T, RY, 2>(g, in, out, r, resid, s);
  else
    launch_heat7_e<T, RY, 1>(g, in, out, r, resid, s);
}

template <class T>
void launch_heat7(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  // defaults from bench/kernel_ab.py on MI355X, 1024^3 fp32 (profiles/archive/r01_ab_heat7_f32.json):
  // RY=2 PF=1 1.546 ms (694.5 GCells/s) > RY=4 PF=1 1.584 > RY=4 PF=2 1.603 > RY=2 PF=2 1.662
  // fp64 1024^3: RY=4 PF=2 3.395 ms (316 GCells/s) > RY=4 PF=1 3.415 > RY=2 PF=1 3.479
  // (profiles/archive/r01_ab_heat7_f64.json).
  // (short columns take the same tiles: a 1-row copy for ny < 8 was dropped in round 5 with the other
  // rarely reached instances, libmdfx.so size)
  constexpr int RY = sizeof(T) == 4 ? 2 : 4;
  launch_heat7_ry<T, RY>(g, in, out, r, resid, s);
}
template void launch_heat7<float>(const Geo&, const float*, float*, float, double*, hipStream_t);
template void launch_heat7<double>(const Geo&, const double*, double*, double, double*, hipStream_t);

template <class T>
void launch_jacobi5(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s, bool ref) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int WX = 64 * VT<T>::N;
  const int XT = (int)((g.nx + WX - 1) / WX);
  const int zc = pick_zc(planes, XT, 256, 4 * 2048);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (ref) {
    if (resid)
      hipLaunchKernelGGL((jacobi5_wave<T, true, true>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
    else
      hipLaunchKernelGGL((jacobi5_wave<T, false, true>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
  } else if (resid) {
    hipLaunchKernelGGL((jacobi5_wave<T, true, false>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
  } else {
    hipLaunchKernelGGL((jacobi5_wave<T, false, false>), grd, blk, 0, s, in, out, g, r, zc, XT, ntasks, resid);
  }
}
template void launch_jacobi5<float>(const Geo&, const float*, float*, float, double*, hipStream_t, bool);
template void launch_jacobi5<double>(const Geo&, const double*, double*, double, double*, hipStream_t, bool);

}  // namespace dev
}  // namespace mdfx
