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
#include <type_traits>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target);
int64_t resident_blocks(const void* kfn);
int tbk_zc(int64_t planes, int64_t tiles, int64_t resident, int K, int min_rounds);

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
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
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
    if (xin && lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny) {
      dcheck(g, in, ib + lz * plane + (int64_t)j * pitch, N);
      v = *(const V*)(ib + lz * plane + (int64_t)j * pitch);
    }
    return v;
  };
  auto ldl = [&](int64_t lz, int j) -> T {
    const int64_t y = y0 - 1 + j;
    if (wx == 0 && lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max && y >= 0 && y < g.ny) {
      dcheck(g, in, ib + lz * plane + (int64_t)j * pitch - 1, 1);
      return ib[lz * plane + (int64_t)j * pitch - 1];
    }
    return T(0);
  };
  auto ldr = [&](int64_t lz, int j) -> T {
    const int64_t y = y0 - 1 + j;
    if (wx == WXN - 1 && lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max && y >= 0 &&
        y < g.ny) {
      dcheck(g, in, ib + lz * plane + (int64_t)j * pitch + N, 1);
      return ib[lz * plane + (int64_t)j * pitch + N];
    }
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
      lds_barrier();  // s_barrier after the LDS writes only: the register prefetch stays in flight
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
        dcheck(g, (const T*)out, ob + lz * plane + (int64_t)i * pitch, N);
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
  const int zc = pick_zc(planes, (int64_t)XT * YT, 128, 2048);
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
  // 2 rows per tile (short columns too: a 1-row copy for ny < 8 was dropped in round 5 with the
  // other rarely reached instances, libmdfx.so size)
  launch_box27_ry<T, 2>(g, in, out, c, resid, s);
}
template void launch_box27<float>(const Geo&, const float*, float*, const StencilCoef&, double*,
                                  hipStream_t);
template void launch_box27<double>(const Geo&, const double*, double*, const StencilCoef&, double*,
                                   hipStream_t);

// ---- two steps per sweep ----------------------------------------------------------------------
//
// The 27-point update fused over two time steps, with the partial-sum factorisation carried
// through both levels. When u0 plane k enters, each lane forms A0(k), B0(k) for the RY+2 rows of
// the tile's u1 window and finishes u1(k-1) = (A0(k-2) + B0(k-1)) + A0(k) from a running sum; the
// u1 plane produced the previous iteration then gets its partials A1, B1 for the RY owned rows and
// finishes u2(k-3) the same way. Only the running sums, the last A and the centres are carried
// between planes, so the registers stay close to the 7-point fused kernel. One barrier per plane
// publishes the wave-seam values of the new u0 plane and of the pending u1 plane together. Rows
// must fit one block (nx <= 4 * 64 * N); the result is bitwise equal to two box27_zw steps.
//
// box27_tb2n: that scheme for fp32 in the natural pair layout (RowOpsN: (e0,e1),(e2,e3) straight from a 16-B
// load, x sums as scalar adds) with the plane loop unrolled by two: every loop-carried row (the
// running sums, the last A, the centres, the pending u1 plane and the prefetched u0 plane) lives in
// two copies that swap roles between the planes of a trip, so no carried row is ever copied (the
// pair-layout kernel, removed in round 5 with its last fp64 use, spent 161 of its 400 VALU
// instructions per plane on register moves). Bitwise equal to two box27_zw steps. An odd plane
// count ends with one extra plane that stores nothing.
// (Reading the plane's seam cells into registers right after the barrier, instead of one LDS round
// trip per row inside hsum, measured 1091 vs 1099 GCells/s at 512^3: profiles/r05_session_c/.)
template <int RY, int WXN, bool RES>
__global__ __launch_bounds__(256) void box27_tb2n(const float* __restrict__ in, float* __restrict__ out, Geo g,
                                                  float c0, float c1, float c2, float c3, int zc, int YT,
                                                  double* __restrict__ resid) {
  using T = float;
  using V = typename VT<T>::type;
  using RO = RowOpsN;
  using Row = RO::Row;
  constexpr int N = 4;
  constexpr int WX = 64 * N;
  constexpr int WYN = 4 / WXN;
  constexpr int R0 = RY + 4;  // u0 rows y0-2 .. y0+RY+1
  constexpr int R1 = RY + 2;  // u1 rows y0-1 .. y0+RY
  __shared__ T edge[2][4][R0 + R1][2];
  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);
  const int yt = t % YT;
  const int zt = t / YT;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wx = w % WXN, wy = w / WXN;
  const int64_t xw = (int64_t)wx * WX;
  const uint32_t xo = (uint32_t)lane * N;
  const int64_t x = xw + xo;
  const int64_t y0 = ((int64_t)yt * WYN + wy) * RY;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  T* ob = out + y0 * pitch + xw;
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);

  // Unpredicated loads from clamped addresses (rows outside [0, ny), planes outside the storage and
  // lanes beyond the row read the nearest valid vector): those values are finite and only ever
  // feed held cells (the selects keep the centre there) or unstored lanes. The plane / row part of
  // the address is wave-uniform, the lane part a 32-bit byte offset.
  const int ny32 = (int)g.ny;
  const uint32_t xcb = (uint32_t)((xin ? x : pitch - N) * (int64_t)sizeof(T));
  auto ld = [&](int64_t lz, int k) -> Row {
    const int y = (int)y0 - 2 + k;
    const int yc = y < 0 ? 0 : y >= ny32 ? ny32 - 1 : y;
    const int64_t lzc = lz < 0 ? 0 : lz >= g.lz_max ? g.lz_max - 1 : lz;
    const T* a = (const T*)((const char*)(in + lzc * plane + (int64_t)yc * pitch) + xcb);
    dcheck(g, in, a, N);
    return RO::lds(a);
  };
  // Seam cells of the neighbouring waves in the row, read by every lane (broadcast) from VGPR-held
  // LDS bases. A wave at the row's left / right end reads its own entry instead of a neighbour's:
  // that value only reaches the x = 0 / x >= nx - 1 cells, which the selects hold, so any finite
  // value serves (round 2 branched to substitute 0).
  constexpr int SL = R0 + R1;  // seam slots per wave and parity
  const int wl = wx > 0 ? w - 1 : w, wr = wx < WXN - 1 ? w + 1 : w;
  const auto eL = lds_vptr(&edge[0][wl][0][1]);
  const auto eR = lds_vptr(&edge[0][wr][0][0]);
  const auto eW = lds_vptr(&edge[0][w][0][lane == 0 ? 0 : 1]);
  auto hsum = [&](const Row& v, int buf, int slot) -> Row {
    const T le = eL[(buf * 4 * SL + slot) * 2];
    const T re = eR[(buf * 4 * SL + slot) * 2];
    return RO::hsum(v, lane_up1_or(le, RO::last(v)), lane_down1_or(re, RO::first(v)));
  };
  struct St {
    Row Rw[R0];                   // u0 plane k
    Row A0p[R1], S0[R1], C0[R1];  // A0(k-1); A0(k-2) + B0(k-1); u0 plane k-1 (u1 window rows)
    Row U1[R1];                   // u1 plane k-2
    Row A1p[RY], S1[RY], C1[RY];  // A1(k-3); A1(k-4) + B1(k-3); u1 plane k-3 (owned rows)
  };
  St sa, sb;
#pragma unroll
  for (int j = 0; j < R0; ++j) {
    sa.Rw[j] = ld(zs - 2, j);
    sb.Rw[j] = RO::zero();
  }
#pragma unroll
  for (int j = 0; j < R1; ++j) sa.A0p[j] = sa.S0[j] = sa.C0[j] = sa.U1[j] = sb.A0p[j] = sb.S0[j] = sb.C0[j] = sb.U1[j] = RO::zero();
#pragma unroll
  for (int i = 0; i < RY; ++i) sa.A1p[i] = sa.S1[i] = sa.C1[i] = sb.A1p[i] = sb.S1[i] = sb.C1[i] = RO::zero();
  double acc = 0.0;
  const int64_t klast = ze + 2;

  auto plane_step = [&](int64_t k, int buf, St& si, St& so) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < R0; ++j) so.Rw[j] = ld(k + 1, j);  // next plane, in flight over this one
    if (lane == 0 || lane == 63) {  // lane 0 publishes each row's first cell, lane 63 its last
#pragma unroll
      for (int j = 0; j < R0; ++j) eW[(buf * 4 * SL + j) * 2] = lane == 0 ? RO::first(si.Rw[j]) : RO::last(si.Rw[j]);
#pragma unroll
      for (int j = 0; j < R1; ++j)
        eW[(buf * 4 * SL + R0 + j) * 2] = lane == 0 ? RO::first(si.U1[j]) : RO::last(si.U1[j]);
    }
    lds_barrier();  // s_barrier after the LDS writes only: the register prefetch stays in flight

    // ---- level 1: partials of u1 plane k-2, u2(k-3) ------------------------------------------
    if (k >= zs + 1) {
      Row Hm = hsum(si.U1[0], buf, R0), Hc = hsum(si.U1[1], buf, R0 + 1);
      const int64_t lz = k - 3;
      const int64_t gz = lz + g.gz_off;
      const bool zb = gz == 0 || gz == g.gnz - 1;
#pragma unroll
      for (int i = 0; i < RY; ++i) {
        const int j = i + 1;
        const Row Hp = hsum(si.U1[j + 1], buf, R0 + j + 1);
        const Row cross = RO::add(Hc, RO::add(si.U1[j - 1], si.U1[j + 1]));
        const Row diag = RO::add(Hm, Hp);
        const Row A = RO::lin3(si.U1[j], cross, diag, c1, c2, c3);  // sm::box27_A
        const Row B = RO::lin3(si.U1[j], cross, diag, c0, c1, c2);  // sm::box27_B
        Hm = Hc;
        Hc = Hp;
        const int64_t y = y0 + i;
        if (k >= zs + 3 && k <= klast && y < g.ny) {
          Row o = si.C1[i];
          if (!zb && y != 0 && y != g.ny - 1) o = RO::sel(xb, si.C1[i], RO::add(si.S1[i], A));
          if (xin) {
            dcheck(g, (const T*)out, ob + lz * plane + (int64_t)i * pitch + xo, N);
            store_nt((V*)(ob + lz * plane + (int64_t)i * pitch + xo), RO::vec(o));
            if (RES) {
#pragma unroll
              for (int e = 0; e < N; ++e)
                if (x + e < g.nx) {
                  const double d = (double)RO::get(o, e) - (double)RO::get(si.C1[i], e);
                  acc += d * d;
                }
            }
          }
        }
        so.S1[i] = RO::add(si.A1p[i], B);
        so.A1p[i] = A;
        so.C1[i] = si.U1[j];
      }
    }
    // ---- level 0: partials of u0 plane k, u1(k-1) ----------------------------------------------
    {
      const int64_t gz = k - 1 + g.gz_off;
      const bool zb = gz <= 0 || gz >= g.gnz - 1;
      Row Hm = hsum(si.Rw[0], buf, 0), Hc = hsum(si.Rw[1], buf, 1);
#pragma unroll
      for (int jj = 0; jj < R1; ++jj) {
        const int j = jj + 1;
        const Row Hp = hsum(si.Rw[j + 1], buf, j + 1);
        const Row cross = RO::add(Hc, RO::add(si.Rw[j - 1], si.Rw[j + 1]));
        const Row diag = RO::add(Hm, Hp);
        const Row A = RO::lin3(si.Rw[j], cross, diag, c1, c2, c3);
        const Row B = RO::lin3(si.Rw[j], cross, diag, c0, c1, c2);
        Hm = Hc;
        Hc = Hp;
        const int64_t y = y0 - 1 + jj;
        Row u = si.C0[jj];
        if (!zb && y > 0 && y < g.ny - 1) u = RO::sel(xb, si.C0[jj], RO::add(si.S0[jj], A));
        so.U1[jj] = u;
        so.S0[jj] = RO::add(si.A0p[jj], B);
        so.A0p[jj] = A;
        so.C0[jj] = si.Rw[j];
      }
    }
  };
  for (int64_t k = zs - 2; k <= klast; k += 2) {
    plane_step(k, 0, sa, sb);
    plane_step(k + 1, 1, sb, sa);
  }
  if (RES) wave_atomic_add(resid, acc);
}

// ---- K steps per sweep, streaming levels (box27_tbk) ---------------------------------------------
//
// heat7_tbk's organisation applied to the 27-point update: u0 planes arrive by LDS DMA (each wave
// its own RY + 2K rows plus the x-seam vectors, one plane ahead), and every level k = 1..K is a
// streaming z-march over RY + 2(K-k) rows whose state per row is the partial-sum pipeline of
// box27_zw: A = A(p-1), S = A(p-2) + B(p-1) and the centre C = u(p-1). When plane p of u_{k-1}
// arrives, the level forms its x sums H = xm + xp (DPP shifts, seams from LDS), then per row
//   cross = H + (ym + yp), diag = Hm + Hp, a = box27_A, b = box27_B
//   u_k(p-1) = S + a;  S = A + b;  A = a;  C = centre
// -- box27_combine's order, so the result is bitwise equal to K single box27_zw steps. Rows sit in
// the pair layout of RowOps (fp32: every operation a packed v_pk op, the x sums without moves).
// Held cells (x / y / z boundary) keep their centre through a select that only the waves and
// levels that contain such cells execute. Seams of levels 1..K-1: double-buffered LDS edge table,
// one barrier per level and plane. Region contract as heat7_tbk: u0 valid on [lz_begin - K, lz_end + K).
template <class T, int RY, int K, int WXN, bool RES>
__global__ __launch_bounds__(256) void box27_tbk(const T* __restrict__ in, T* __restrict__ out, Geo g, T c0, T c1,
                                                 T c2, T c3, int zc, int YT, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  using RO = RowOps<T>;
  using Row = typename RO::Row;
  constexpr int N = VT<T>::N;
  constexpr int WX = 64 * N;
  constexpr int WYN = 4 / WXN;
  constexpr int R0 = RY + 2 * K;              // u0 window rows y0-K .. y0+RY+K-1
  constexpr int TOT = tbk_off<RY, K>(K + 1);  // state rows over all levels
  constexpr int NLV = K > 1 ? K - 1 : 1;
  static_assert(R0 <= 32, "seam DMA uses lanes 0..R0-1 and 32..32+R0-1");
  __shared__ V slot[4][R0 + 1][64];  // per-wave u0 plane; row R0 holds the seam vectors
  constexpr int TB_ROW = 4, TB_W = R0 * TB_ROW, TB_PAR = 4 * TB_W, TB_LV = 2 * TB_PAR;
  __shared__ __attribute__((aligned(16))) T tb[NLV * TB_LV + 4];

  const unsigned t = xcd_remap(blockIdx.x, gridDim.x);
  const int yt = t % YT;
  const int zt = t / YT;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wx = w % WXN, wy = w / WXN;
  const int64_t xw = (int64_t)wx * WX;
  const uint32_t xo = (uint32_t)lane * N;
  const int64_t x = xw + xo;
  const int64_t y0 = ((int64_t)yt * WYN + wy) * RY;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  T* ob = out + y0 * pitch + xw;

  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);
  // wave-uniform: does this wave hold any x-boundary cell, are all computed rows y-interior
  const bool xedge = xw == 0 || xw + WX >= g.nx;
  const bool yint = y0 - (K - 1) >= 1 && y0 + RY + K - 2 <= g.ny - 2;

  // ---- u0 streaming (heat7_tbk's DMA: clamped in-bounds addresses, 32-bit lane offsets) ---------
  const bool has_l = xw > 0 && xw < pitch, has_r = xw + WX < pitch;
  const int srow = lane & 31;
  const bool son = lane < 32 ? (has_l && srow < R0) : (WXN > 1 && has_r && srow < R0);
  const uint32_t xcb = (uint32_t)((xin ? x : pitch - N) * (int64_t)sizeof(T));
  const uint32_t socb = son ? (uint32_t)((lane < 32 ? xw - N : xw + WX) * (int64_t)sizeof(T)) : xcb;
  const T* ib0 = in + (y0 - K) * pitch;
  auto rowc = [&](int k) -> int64_t {
    const int64_t y = y0 - K + k;
    return (y < 0 ? 0 : y >= g.ny ? g.ny - 1 : y) - (y0 - K);
  };
  const int64_t srowc = rowc(srow < R0 ? srow : 0);
  // (buffer-descriptor DMAs as heat7_tbk's: partial lgkmcnt waits for the LDS reads that follow)
  auto issue = [&](int64_t lz) {
    uint64_t pbs = (uint64_t)(uintptr_t)(ib0 + lz * plane);
    asm volatile("" : "+s"(pbs));
    const char* pb = (const char*)(uintptr_t)pbs;
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(pb);
#pragma unroll
    for (int k = 0; k < R0; ++k) {
      const uint32_t ro = (uint32_t)(rowc(k) * pitch * (int64_t)sizeof(T));
      dcheck(g, in, (const T*)(pb + ro + xcb), N);
      blds16s(rs, xcb, ro, &slot[w][k][0]);
    }
    if (WXN > 1) {
      const uint32_t o = (uint32_t)(srowc * pitch * (int64_t)sizeof(T)) + socb;
      dcheck(g, in, (const T*)(pb + o), N);
      blds16(rs, o, &slot[w][R0][0]);
    }
  };
  const int wl = wx > 0 ? w - 1 : w, wr = wx < WXN - 1 ? w + 1 : w;
  const T* base1 = lane < 32 ? &tb[2 + wl * TB_W + 2 + 1] : &tb[2 + wr * TB_W + 0 - 1];
  T* wrp = &tb[2 + w * TB_W + (lane == 0 ? 0 : 2)];

  Row A[TOT], S[TOT], C[TOT];
#pragma unroll
  for (int i = 0; i < TOT; ++i) {
    A[i] = RO::zero();
    S[i] = RO::zero();
    C[i] = RO::zero();
  }
  // output stores per stored plane (wave-uniform; a wave with no lane in the row issues none)
  const int nsto = __builtin_amdgcn_ballot_w64(xin) != 0 ? (int)max((int64_t)0, min((int64_t)RY, g.ny - y0)) : 0;
  int nst = 0;  // stores issued since this wave's last DMA
  double acc = 0.0;
  const int64_t cend = ze + K;
  const T* base0 = (const T*)&slot[w][R0][0] + (lane < 32 ? N - 1 : 0);
  issue(zs - K);
  for (int64_t c = zs - K; c < cend; ++c) {
    const int par = (int)(c & 1);
    wait_vm_le(nst);  // this wave's DMA of plane c has landed (its later stores may not have)
    Row X[R0];
    T LO[R0], HI[R0];
#pragma unroll
    for (int k = 0; k < R0; ++k) {
      X[k] = RO::lds_pairs((const T*)&slot[w][k][lane]);
      // a wave edge without a neighbouring wave has no DMA'd seam (stale LDS): 0 instead
      LO[k] = has_l ? base0[k * N] : T(0);
      HI[k] = (WXN > 1 && has_r) ? base0[k * N + 32 * N] : T(0);
    }
    wait_lgkm0();  // slot consumed: refill it with the next plane while the levels compute
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < R0; ++k) RO::fence(X[k]);
    if (c + 1 < cend) issue(c + 1);

#pragma unroll
    for (int k = 1; k <= K; ++k) {
      const int ROUT = RY + 2 * (K - k);
      const int off = tbk_off<RY, K>(k);
      if (c >= zs - K + 2 * k - 2) {  // block-uniform pipeline fill
        if (k >= 2 && WXN > 1) {
          const T* b1 = base1 + (k - 2) * TB_LV + par * TB_PAR;
#pragma unroll
          for (int j = 0; j < ROUT + 2; ++j) {
            LO[j] = b1[j * TB_ROW];
            HI[j] = b1[j * TB_ROW + 1];
          }
        }
        const int64_t gz = c - k + g.gz_off;  // plane finished by this level: c - k
        const bool zh = gz <= 0 || gz >= g.gnz - 1;
        Row H[R0], Y[R0];
#pragma unroll
        for (int j = 0; j < ROUT + 2; ++j) {
          const T l = lane_up1_or(LO[j], RO::last(X[j]));
          const T rr = lane_down1_or(HI[j], RO::first(X[j]));
          H[j] = RO::hsum(X[j], l, rr);
        }
        auto rows = [&](auto hold) __attribute__((always_inline)) {
          constexpr bool HOLD = decltype(hold)::value;
#pragma unroll
          for (int i = 0; i < ROUT; ++i) {
            const Row cen = X[i + 1];
            const Row cross = RO::add(H[i + 1], RO::add(X[i], X[i + 2]));
            const Row diag = RO::add(H[i], H[i + 2]);
            const Row a = RO::lin3(cen, cross, diag, c1, c2, c3);
            const Row b = RO::lin3(cen, cross, diag, c0, c1, c2);
            const Row cold = C[off + i];
            Row o = RO::add(S[off + i], a);
            if (HOLD) {
              const int64_t y = y0 - (K - k) + i;
              const bool rh = zh || y <= 0 || y >= g.ny - 1;
              bool h[N];
#pragma unroll
              for (int e = 0; e < N; ++e) h[e] = rh || xb[e];
              o = RO::sel(h, cold, o);
            }
            S[off + i] = RO::add(A[off + i], b);
            A[off + i] = a;
            C[off + i] = cen;
            Y[i] = o;
            if (RES && k == K && c >= zs + K && y0 + i < g.ny && xin) {
#pragma unroll
              for (int e = 0; e < N; ++e)
                if (x + e < g.nx) {
                  const double d = (double)RO::get(o, e) - (double)RO::get(cold, e);
                  acc += d * d;
                }
            }
          }
        };
        if (zh || xedge || !yint)
          rows(std::integral_constant<bool, true>{});
        else
          rows(std::integral_constant<bool, false>{});
        if (k < K) {
          if (WXN > 1) {  // publish the edge pairs of every row: the next level's whole window
            if (lane == 0 || lane == 63) {
              T* wp = wrp + (k - 1) * TB_LV + par * TB_PAR;
#pragma unroll
              for (int j = 0; j < ROUT; ++j) lds_store(wp + j * TB_ROW, RO::edges(Y[j]));
            }
            lds_barrier();
          }
#pragma unroll
          for (int j = 0; j < ROUT; ++j) X[j] = Y[j];
        } else if (c >= zs + K) {  // u_K(c - K) is an owned output plane
          nst = nsto;
          const int64_t lz = c - K;
#pragma unroll
          for (int i = 0; i < RY; ++i) {
            if (y0 + i < g.ny && xin) {
              T* a = (T*)((char*)(ob + lz * plane + (int64_t)i * pitch) + xo * (uint32_t)sizeof(T));
              dcheck(g, (const T*)out, a, N);
              store_nt((V*)a, RO::vec(Y[i]));
            }
          }
        }
      }
    }
  }
  wait_vm0();  // no DMA may outlive the wave
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, int RY, int K, int WXN>
static void launch_box27_tbk_w(const Geo& g, const T* in, T* out, const StencilCoef& cf, double* resid,
                               hipStream_t s) {
  constexpr int WYN = 4 / WXN;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int YT = (int)((g.ny + WYN * RY - 1) / (WYN * RY));
  const int zc = tbk_zc(planes, YT, resident_blocks((const void*)&box27_tbk<T, RY, K, WXN, false>), K, g.min_rounds);
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)YT * ZT)), blk(256);
  const T c0 = (T)cf.c0, c1 = (T)cf.c1, c2 = (T)cf.c2, c3 = (T)cf.c3;
  if (resid)
    hipLaunchKernelGGL((box27_tbk<T, RY, K, WXN, true>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT, resid);
  else
    hipLaunchKernelGGL((box27_tbk<T, RY, K, WXN, false>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT, resid);
}

template <class T, int RY, int K>
static void launch_box27_tbk_ry(const Geo& g, const T* in, T* out, const StencilCoef& cf, double* resid,
                                hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  if (g.pitch > 2 * WX)
    launch_box27_tbk_w<T, RY, K, 4>(g, in, out, cf, resid, s);
  else if (g.pitch > WX)
    launch_box27_tbk_w<T, RY, K, 2>(g, in, out, cf, resid, s);
  else
    launch_box27_tbk_w<T, RY, K, 1>(g, in, out, cf, resid, s);
}

template <class T>
bool box27_tb2_supported(const Geo& g) {
  return g.pitch <= 4 * 64 * VT<T>::N && g.ny >= 1;
}
template bool box27_tb2_supported<float>(const Geo&);
template bool box27_tb2_supported<double>(const Geo&);

template <class T, int RY, int WXN>
static void launch_box27_tb2_w(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                               hipStream_t s) {
  constexpr int WYN = 4 / WXN;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int YT = (int)((g.ny + WYN * RY - 1) / (WYN * RY));
  // balanced ~43-plane chunks, as the 7-point fused kernel (5 pipeline planes here)
  int64_t zt = (planes + 43) / 44;
  int zc = (int)((planes + zt - 1) / zt);
  while ((int64_t)YT * zt < 1024 && zc > 16) {
    ++zt;
    zc = (int)((planes + zt - 1) / zt);
  }
  zc = std::max(zc, 1);
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)YT * ZT)), blk(256);
  const T c0 = (T)c.c0, c1 = (T)c.c1, c2 = (T)c.c2, c3 = (T)c.c3;
  // the natural-layout kernel with the 2-plane unroll (box27_tb2n; round 2's pair-layout fp32
  // box27_tb2, 937-944 vs 1005-1013 GCells/s at 512^3, was removed in round 4,
  // profiles/archive/r03_wtk/b27f32_*; its fp64 instance, 491.8 GCells/s against box27_tbk's 553, in round 5)
  static_assert(std::is_same<T, float>::value, "box27_tb2n: fp32 rows (fp64 runs box27_tbk)");
  if (resid)
    hipLaunchKernelGGL((box27_tb2n<RY, WXN, true>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT, resid);
  else
    hipLaunchKernelGGL((box27_tb2n<RY, WXN, false>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT, resid);
}

template <class T, int RY>
static void launch_box27_tb2_ry(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid,
                                hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  if (g.pitch > 2 * WX)
    launch_box27_tb2_w<T, RY, 4>(g, in, out, c, resid, s);
  else if (g.pitch > WX)
    launch_box27_tb2_w<T, RY, 2>(g, in, out, c, resid, s);
  else
    launch_box27_tb2_w<T, RY, 1>(g, in, out, c, resid, s);
}

template <class T>
void launch_box27_tb2(const Geo& g, const T* in, T* out, const StencilCoef& c, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  // fp64: box27_tbk with 4 rows per tile, fp32: box27_tb2 (interleaved A/B on one MI355X, GCells/s,
  // tb2 / tbk RY 2 / tbk RY 4: 512^3 fp32 987 / 942 / 884, 1024^3 fp32 995 / 873 / 985, 512^3 fp64
  // 492 / 468 / 553; profiles/archive/r02_box27_tbk.txt). box27_tb2 exists for fp32 only (its pair-layout
  // rows cost the fp64 instance occupancy: 489 -> 341). One row per tile on short columns. (The
  // switch to the other combinations, measured slower, was removed in round 5.)
  if constexpr (std::is_same<T, double>::value) {
    if (g.ny < 8)
      launch_box27_tbk_ry<T, 1, 2>(g, in, out, c, resid, s);
    else
      launch_box27_tbk_ry<T, 4, 2>(g, in, out, c, resid, s);
  } else {
    if (knobs().tb_ry == 1 || g.ny < 8)
      launch_box27_tb2_ry<T, 1>(g, in, out, c, resid, s);
    else
      launch_box27_tb2_ry<T, 2>(g, in, out, c, resid, s);
  }
}
template void launch_box27_tb2<float>(const Geo&, const float*, float*, const StencilCoef&, double*, hipStream_t);
template void launch_box27_tb2<double>(const Geo&, const double*, double*, const StencilCoef&, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
