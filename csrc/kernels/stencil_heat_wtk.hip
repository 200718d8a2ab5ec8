// Deep temporal blocking for the 3D 7-point stencil in y bands of wave tiles (heat7_wtk):
// K = 3 or 4 fused steps per sweep, rows of any width, one block barrier per plane.
//
// heat7_tbk (stencil_heat_tbk.hip) spreads one row over the 4 waves of a block and hands the x
// seams of every level between them through LDS: K-1 block barriers per plane, and at K >= 3 the
// barrier-coupled waves are latency-bound at two waves per SIMD. Here no level seam
// crosses a wave -- jacobi5_tbk's overlapping wave segments carried into 3D:
//   x: a wave covers 64 lanes x N cells but owns only lanes OV..63-OV (OV = ceil(K / N)); the
//      outer lanes carry the neighbouring segments' edge columns through the same instructions and
//      go wrong one cell per level from the outside, so after K levels the owned lanes are exact.
//      x neighbours inside the wave are DPP lane shifts.
//   y: the wave owns RY output rows; level k computes the RY + 2(K-k) rows the levels above it
//      need (the y halo is recomputed, as in heat7_tbk).
//   z: every level is heat7_tbk's streaming recurrence: per row only the partial sum
//      S_k = (((xm + xp) + ym) + yp) + zm of plane p and the centre C_k = u_{k-1}(p) live between
//      planes; when u_{k-1}(p+1) arrives the level finishes u_k(p) = fma(r, fma(-6, C, S + zp), C),
//      sm::heat7's operation order, so the sweep is bitwise equal to K single steps.
//   u0: the waves of a block form a y band; the band's rows of the next plane stream by LDS DMA into
//      a shared double-buffered window one plane ahead (no VGPRs held by the prefetch), and the one
//      barrier per plane both publishes a plane and frees the other buffer (below).
//   Boundaries: held cells get a zero coefficient (fma(0, t, u) = u for finite t): per lane for x,
//   per level and plane for z, per row only in tiles that reach y = 0 / ny-1. Loads outside the
//   grid read the nearest valid row / vector, so every value a lane carries is finite.
//
// Region contract (as heat7_tbk): output storage planes [lz_begin, lz_end) need u0 valid on
// [lz_begin - K, lz_end + K) (the engine keeps K ghost planes per side).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <type_traits>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int64_t resident_blocks(const void* kfn, int block);

// Schedule of one streaming sweep over `planes` planes of `tiles` tiles on `resident` block slots:
// z chunks of zc planes, tiles x chunks blocks, dealt in rounds of `resident`; every chunk pays 2K
// planes of pipeline fill, so the chunk count minimises rounds x (zc + 2K) (chunks of at least 4K
// planes; at least `min_rounds` rounds when several slabs leave CUs for exchange kernels). 1024^3
// fp32 in 8-wave bands: 7 chunks of 147 planes (5.9 rounds), the measured optimum of round 2's zc
// sweep, where 6 or 4 chunks (171, 256 planes) end on a nearly empty round. (A balanced one-round
// "split" schedule, block b marching the b-th equal share of the tile-major work, measured slower:
// neighbouring y bands stop marching in lockstep and lose their L2 sharing of the y-halo rows, 1.59
// instead of 1.20 fields fetched; removed in round 4, numbers in profiles/archive/r03_wtk/.)
static int wtk_zc(int64_t planes, int64_t tiles, int64_t resident, int K, int min_rounds) {
  const int64_t fill = 2 * K;
  const int64_t zmax = std::max<int64_t>(1, planes / (4 * K));
  double best = 1e300;
  int64_t bz = 1;
  for (int64_t zt = 1; zt <= zmax; ++zt) {
    const int64_t rounds = (tiles * zt + resident - 1) / resident;
    if (rounds < min_rounds && zt < zmax) continue;
    const double t = (double)rounds * (double)((planes + zt - 1) / zt + fill);
    if (t < best * 0.999) {
      best = t;
      bz = zt;
    }
  }
  return (int)((planes + bz - 1) / bz);
}

// A block is one task: WB = 4 or 8 waves stacked along y on one x segment (a y band of WB * RY
// rows). The band's u0 window (WB * RY + 2K rows) streams into a shared double-buffered LDS
// window, each row fetched once for the band instead of once per wave (9 rows per 3 output rows
// -> 18 per 12 / 30 per 24), at one block barrier per plane. (The first version ran every wave as
// an independent task with a private LDS slot and no barrier: 1.565 fields fetched per sweep
// against 1.444 / 1.108 for bands of 4 / 8, and slower on every shape, profiles/archive/r02_wtk/README.txt.)
template <class T, int RY, int K, int WB, bool RES, int MODE>
__global__ __launch_bounds__(WB == 8 ? 512 : 256) void heat7_wtk(const T* __restrict__ in, T* __restrict__ out, Geo g, T r,
                                                 int zc, int XT, int YT, int ntasks, double* __restrict__ resid) {
  using V = typename VT<T>::type;
  using RO = typename std::conditional<sizeof(T) == 4 && MODE >= 1, RowOpsN, RowOps<T>>::type;
  using Row = typename RO::Row;
  constexpr int N = VT<T>::N;
  constexpr int OV = (K + N - 1) / N;         // overlap lanes per side
  constexpr int SEG = (64 - 2 * OV) * N;      // owned columns per wave
  constexpr int R0 = RY + 2 * K;              // u0 window rows y0-K .. y0+RY+K-1
  constexpr int TOT = tbk_off<RY, K>(K + 1);  // state rows over all levels
  constexpr int RB = WB * RY + 2 * K;         // shared window rows of a band
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // Work: block-uniform task = one z chunk of one tile (x segment, y band); order x segments
  // fastest, then y bands, then z chunks. A second region (g.lz2_*: the other boundary region of a
  // slab) adds its own z chunks after the first region's.
  const int b = (int)xcd_remap(blockIdx.x, gridDim.x);
  const int P = (int)(g.lz_end - g.lz_begin);
  if (b >= ntasks) return;  // block-uniform (the grid has exactly ntasks blocks)
  __shared__ V slot[2][RB][64];
  double acc = 0.0;
  // one segment: storage planes [zs, ze) for tile `tile`
  auto segment = [&](const int tile, const int zs, const int ze) __attribute__((always_inline)) {
  const int xt = tile % XT;
  const int yt = tile / XT;
  const int64_t xs = (int64_t)xt * SEG - OV * N;  // column of lane 0
  const int64_t x = xs + (int64_t)lane * N;
  // row / plane indices in 32 bits (extents < 2^31; the launcher checks): fewer SGPRs, so the
  // scalar tests stay scalar
  const int ny = (int)g.ny, lzmax = (int)g.lz_max, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  const int yb = yt * RY * WB;  // first row of the band
  const int y0 = yb + w * RY;   // first row of this wave
  const int64_t pitch = g.pitch, plane = g.plane;
  const bool xin = x >= 0 && x < pitch;
  const bool own = lane >= OV && lane <= 63 - OV && xin;

  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);
  const Row rx = RO::coef(r, xb);
  const Row r0 = RO::zero();
  // block-uniform: all rows the band computes at any level are y-interior. Every wave of the block
  // then runs the same march() copy, so all of them reach the per-plane barrier from one code path
  // (bands at y = 0 / ny-1 take the per-row tested copy as a whole)
  const bool yint = yb - (K - 1) >= 1 && yb + WB * RY + K - 2 <= ny - 2;
  // output stores this wave issues per stored plane (wave-uniform; a store whose lanes are all
  // masked may be skipped by the compiler, so a wave without owned lanes counts none)
  const int nsto = __builtin_amdgcn_ballot_w64(own) != 0 ? max(0, min(RY, ny - y0)) : 0;
  int nst = 0;  // stores issued since this wave's last DMA

  // u0 plane lz -> LDS by LDS DMA (global_load_lds, no VGPR destination): rows outside [0, ny) and
  // lanes outside the row read the nearest valid row / vector (finite values that only meet held
  // or unowned cells). Per lane a 32-bit byte offset from the wave-uniform row start. Wave w
  // fetches rows w, w + WB, ... of the band's window.
  const uint32_t xcb = (uint32_t)((x < 0 ? 0 : x >= pitch ? pitch - N : x) * (int64_t)sizeof(T));
  auto issue = [&](int lz, int buf) {
    const int lzc = lz < 0 ? 0 : lz >= lzmax ? lzmax - 1 : lz;
#pragma unroll
      for (int j = 0; j < (RB + WB - 1) / WB; ++j) {
        const int k = w + j * WB;
        if (k < RB) {
          const int y = yb - K + k;
          const int yc = y < 0 ? 0 : y >= ny ? ny - 1 : y;
          // buffer-descriptor DMA on the wave-uniform row base: partial lgkmcnt waits for the LDS
          // reads that follow (blds16)
          uint64_t rb = (uint64_t)(uintptr_t)(in + (int64_t)lzc * plane + (int64_t)yc * pitch);
          asm volatile("" : "+s"(rb));
          dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + xcb), N);
          blds16(row_rsrc((const void*)(uintptr_t)rb), xcb, &slot[buf][k][0]);
        }
      }
  };

  // MODE 2 unrolls the plane loop by two with the loop-carried centres in two arrays that swap
  // roles (plane q reads CA and writes CB, plane q+1 the reverse), so a new centre is produced
  // straight into the register the next plane reads instead of being copied there every plane
  Row S[TOT], CA[TOT], CB[TOT];
#pragma unroll
  for (int i = 0; i < TOT; ++i) {
    S[i] = RO::zero();
    CA[i] = RO::zero();
    CB[i] = RO::zero();
  }
  const int qlast = ze - 1 + K;  // last u0 plane of the march
  issue(zs - K, 0);
  T* ob = out + (int64_t)y0 * pitch;
  const uint32_t xob = (uint32_t)((xin ? x : 0) * (int64_t)sizeof(T));

  // one u0 plane q: level k finishes plane q - k (its first planes are priming garbage that no
  // stored plane depends on); centres of the previous plane come from Cin, this plane's go to Cout
  auto plane_step = [&](int q, Row(&Cin)[TOT], Row(&Cout)[TOT], auto edge) __attribute__((always_inline)) {
    constexpr bool EDGE = decltype(edge)::value;
    // the DMA of plane q has landed: every wave waits for its own rows (the stores it issued
    // after that DMA stay in flight), then one barrier publishes them and also certifies that
    // every wave has finished reading the other buffer (plane q-1), which the next DMA overwrites
    // no instruction moves across a plane boundary: the two planes of an unrolled trip would
    // otherwise be interleaved by the scheduler, with both planes' rows live at once
    if constexpr (MODE == 2) __builtin_amdgcn_sched_barrier(0);
    wait_vm_le(nst);
    const int buf = (int)((q - (zs - K)) & 1);
    lds_barrier();
    if (q < qlast) issue(q + 1, buf ^ 1);
    // level 1 reads its u0 rows from the window as it goes (three rows live, not R0; plane q
    // stays in its buffer for the whole iteration)
    const T* xw = (const T*)&slot[buf][w * RY][lane];
    auto u0row = [&](int k) -> Row { return RO::lds(xw + k * 64 * N); };
    Row X[R0];
#pragma unroll
    for (int l = 1; l <= K; ++l) {
      const int ROUT = RY + 2 * (K - l);
      const int off = tbk_off<RY, K>(l);
      const int gz = q - l + gzoff;
      // z-held planes: coefficient 0 through a wave-uniform 0 / 1 factor (exact: r * 1 = r,
      // r * 0 = +0 for r >= 0)
      const Row rl = RO::scale(rx, (gz <= 0 || gz >= gnz - 1) ? T(0) : T(1));
      Row Y[R0];
#pragma unroll
      for (int i = 0; i < ROUT; ++i) {
        Row ri = rl;
        if (EDGE) {
          const int y = y0 - (K - l) + i;
          if (y == 0 || y == ny - 1) ri = r0;
        }
        if (l == 1) {  // sliding three-row window over the u0 rows in LDS
          if (i == 0) {
            X[0] = u0row(0);
            X[1] = u0row(1);
          }
          X[i + 2] = u0row(i + 2);
        }
        const Row cen = X[i + 1];
        const Row cold = Cin[off + i];
        const Row o = RO::fin(S[off + i], cen, cold, ri);
        const T lft = lane_up1(RO::last(cen));
        const T rgt = lane_down1(RO::first(cen));
        S[off + i] = RO::partial(cen, lft, rgt, X[i], X[i + 2], cold);
        RO::pin(S[off + i]);
        Cout[off + i] = cen;
        Y[i] = o;
        if (RES && l == K && q - K >= zs && q <= qlast && y0 + i < ny && own) {
#pragma unroll
          for (int e = 0; e < N; ++e)
            if (x + e < g.nx) {
              const double d = (double)RO::get(o, e) - (double)RO::get(cold, e);
              acc += d * d;
            }
        }
      }
      if (l < K) {
#pragma unroll
        for (int j = 0; j < ROUT; ++j) X[j] = Y[j];
      } else if (q - K >= zs && q <= qlast) {  // u_K(q - K) is an owned output plane
        const int lz = q - K;
        nst = nsto;
#pragma unroll
        for (int i = 0; i < RY; ++i) {
          if (y0 + i < ny && own) {
            T* a = (T*)((char*)(ob + (int64_t)lz * plane + (int64_t)i * pitch) + xob);
            dcheck(g, (const T*)out, a, N);
            store_nt((V*)a, RO::vec(Y[i]));
          }
        }
      }
    }
  };
  auto march = [&](auto edge) __attribute__((always_inline)) {
    if constexpr (MODE == 2) {
      // an odd plane count ends with one extra plane (q = qlast + 1): no DMA, nothing stored
      for (int q = zs - K; q <= qlast; q += 2) {
        plane_step(q, CA, CB, edge);
        plane_step(q + 1, CB, CA, edge);
      }
    } else {
      for (int q = zs - K; q <= qlast; ++q) plane_step(q, CA, CA, edge);
    }
  };
  // (fp64: only the copy with the per-row y test; a second copy costs the registers that keep
  // the 8-wave bands at two waves per SIMD without spilling)
  if (yint && sizeof(T) == 4)
    march(std::integral_constant<bool, false>{});
  else
    march(std::integral_constant<bool, true>{});
  wait_vm0();  // no DMA may outlive the wave (or the segment)
  };
  const int t = b % (XT * YT), zt = b / (XT * YT);
  const int zt1 = (P + zc - 1) / zc;  // chunks of the first region
  if (zt < zt1) {
    const int zs = (int)g.lz_begin + zt * zc;
    segment(t, zs, min((int)g.lz_end, zs + zc));
  } else {
    const int zs = (int)g.lz2_begin + (zt - zt1) * zc;
    segment(t, zs, min((int)g.lz2_end, zs + zc));
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, int RY, int K, int WB, int MODE>
static void launch_wtk_kn(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int N = VT<T>::N, OV = (K + N - 1) / N, SEG = (64 - 2 * OV) * N;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int XT = (int)((g.nx + SEG - 1) / SEG);
  const int YT = (int)((g.ny + RY * WB - 1) / (RY * WB));  // y bands
  const void* kfn = (const void*)&heat7_wtk<T, RY, K, WB, false, MODE>;
  const int64_t tiles = (int64_t)XT * YT;  // blocks per z chunk
  const int64_t resident = resident_blocks(kfn, 64 * WB);
  int zc = wtk_zc(planes, tiles, resident, K, g.min_rounds);
  const int64_t planes2 = g.lz2_end - g.lz2_begin;  // a second region (boundary pair): one chunk each
  if (planes2 > 0) zc = (int)std::max(planes, planes2);
  const int ZT = (int)((planes + zc - 1) / zc) + (planes2 > 0 ? (int)((planes2 + zc - 1) / zc) : 0);
  const int64_t ntasks = (int64_t)XT * YT * ZT;
  MDFX_CHECK(ntasks < (int64_t)1 << 31, "heat7_wtk: too many tasks");
  const dim3 grd((unsigned)ntasks), blk(64 * WB);
  // residual instances exist where they fit 256 VGPRs without spills: every fp64 shape, fp32 in
  // mode 1 (the fp32 mode-2 3-row residual instance spills), and 2-row waves
  constexpr bool kRes = sizeof(T) == 8 || MODE == 1 || RY <= 2;
  if constexpr (!kRes) {
    MDFX_CHECK(!resid, "heat7_wtk: no residual variant of this shape");
  } else if (resid) {
    hipLaunchKernelGGL((heat7_wtk<T, RY, K, WB, true, MODE>), grd, blk, 0, s, in, out, g, r, zc, XT, YT, (int)ntasks,
                       resid);
    return;
  }
  hipLaunchKernelGGL((heat7_wtk<T, RY, K, WB, false, MODE>), grd, blk, 0, s, in, out, g, r, zc, XT, YT, (int)ntasks,
                     resid);
}

// fp32 rows: the natural pair layout (RowOpsN) with the plane loop unrolled by two (mode 2); the
// 3-row residual sweeps without the unroll (mode 1: the unrolled residual instance spills). fp64:
// one layout (mode 0). (Round 2's regrouped fp32 layout, mode 0, measured slower and was removed
// in round 4: 1.985 vs 1.736 ms per 3-step sweep, profiles/archive/r03_pmc/.)
// (Round 6: only the fp64 instances ship. Every fp32 3D 7-point sweep runs heat7_wxk, so the fp32
// layouts of this kernel, modes 1 and 2, were reachable only through MDFX_H7_WXK=0; their 12
// instances are no longer compiled. The numbers above stay as the record of why heat7_wxk won.)
template <class T, int RY, int K, int WB>
static void launch_wtk_k(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  static_assert(sizeof(T) == 8, "heat7_wtk ships fp64 instances only");
  launch_wtk_kn<T, RY, K, WB, 0>(g, in, out, r, resid, s);
}

bool heat7_wtk_supported(int steps) { return steps == 3 || steps == 4; }

// fraction of the lanes' cells inside the row: x segments overlap by OV lanes per side, and the
// last one is ragged (1024 fp32: 5 segments of 256 cells, 0.8)
double heat7_wtk_xeff(int64_t nx, int esize, int steps) {
  const int N = 16 / esize, OV = (steps + N - 1) / N, SEG = (64 - 2 * OV) * N;
  const int64_t XT = (nx + SEG - 1) / SEG;
  return (double)nx / (double)(XT * 64 * N);
}

// K = 4: 1 row per wave (2 rows need > 256 VGPRs)
template <class T>
void launch_heat7_wtk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  MDFX_CHECK((steps == 3 || steps == 4) && g.lz_begin >= steps && g.lz_end + steps <= g.lz_max,
             format("heat7_wtk: %d fused steps need %d valid planes around [%lld, %lld) of %lld", steps, steps,
                    (long long)g.lz_begin, (long long)g.lz_end, (long long)g.lz_max));
  MDFX_CHECK(g.lz2_end <= g.lz2_begin || (g.lz2_begin >= g.lz_end && g.lz2_end + steps <= g.lz_max),
             "heat7_wtk: the second region must follow the first and have its planes + ghosts allocated");
  MDFX_CHECK(g.pitch % VT<T>::N == 0, "heat7_wtk: the row pitch must be a whole number of vectors");
  MDFX_CHECK(g.ny < ((int64_t)1 << 30) && g.lz_max < ((int64_t)1 << 30) && g.gnz < ((int64_t)1 << 30) &&
                 g.gz_off > -((int64_t)1 << 30) && g.gz_off < ((int64_t)1 << 30),
             "heat7_wtk: row / plane counts must fit 32-bit indices");
  // bands of 8 waves (one 512-thread block per CU) only for deep regions: 1024^3 1632-1674 vs
  // 1593-1612 GCells/s for bands of 4, but on 128..512-plane slabs the few large blocks leave CUs
  // idle (8 slabs of 128 planes: 1188-1223 vs 1347-1385); MDFX_WTK_WB = 4 / 8 forces one
  int wb = knobs().wtk_wb;
  if (wb != 4 && wb != 8) wb = g.lz_end - g.lz_begin >= 768 ? 8 : 4;
  // rows per wave at K = 3: fp32 3 (1024^3: 1679 vs 1447 GCells/s for 2 rows); fp64 2 in bands of
  // 4 (3 rows need more than 256 VGPRs there), see below for bands of 8
  constexpr int RY3 = sizeof(T) == 4 ? 3 : 2;
  if (steps == 3) {
    if (wb == 8) {
      // fp64 8-wave bands: 3 rows per wave at rows up to 1024 cells (1024^3 923-925 vs 849-852
      // GCells/s), 2 rows on wider rows (2048^3 835 vs 802)
      if constexpr (sizeof(T) == 8) {
        if (g.nx > 1024) launch_wtk_k<T, 2, 3, 8>(g, in, out, r, resid, s);
        else launch_wtk_k<T, 3, 3, 8>(g, in, out, r, resid, s);
      } else {
        launch_wtk_k<T, 3, 3, 8>(g, in, out, r, resid, s);
      }
    }
    else launch_wtk_k<T, RY3, 3, 4>(g, in, out, r, resid, s);
  } else {
    launch_wtk_k<T, 1, 4, 4>(g, in, out, r, resid, s);
  }
}
template void launch_heat7_wtk<double>(const Geo&, const double*, double*, double, int, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
