// Deep temporal blocking for the 3D 7-point heat/Jacobi stencil: K time steps per sweep over
// memory (K = 2, 3, 4), for rows that fit one block (up to 1024 fp32 / 512 fp64 cells).
//
// heat7_tb2 keeps whole planes of every level in registers and rotates them each z-iteration;
// at K = 2 that is already ~100 VGPRs and most of its VALU work is register moves. Here every
// level k = 1..K is a *streaming* z-march whose only state between planes is two row vectors per
// row it owns:
//   C_k = u_{k-1}(p)       (the centre of plane p, and the z- neighbour of plane p+1)
//   S_k = partial sum of plane p: (((xm + xp) + ym) + yp) + zm, all from u_{k-1}
// When u_{k-1}(p+1) arrives, level k finishes u_k(p) = fma(r, fma(-6, C_k, S_k + zp), C_k) --
// exactly sm::heat7's operation order, so the result is bitwise identical to K single steps --
// then replaces S_k / C_k with plane p+1's partial and centre. The levels are staggered by one
// plane: in the z-iteration that brings u0(c), level k turns u_{k-1}(c-k+1) into u_k(c-k), and
// level K writes u_K(c-K) to memory. Each u0 byte is read from HBM once per chunk and each output
// byte written once, so a sweep moves the bytes of ONE step for K steps of work.
//
// Geometry: a 256-thread block is 4 waves along x (a 1024-cell fp32 row; narrower rows stack wave
// groups along y). A group owns RY output rows; level k computes the RY + 2(K-k) rows that the
// levels above it need (the redundant y halo is recomputed instead of exchanged). Per lane one
// 16-B vector per row.
//   u0 arrives by LDS DMA: each wave streams its own RY + 2K rows of the next plane, plus one
//   16-B vector per row beyond each wave edge (the x seams), into its private LDS slot
//   (global_load_lds, no VGPR destination), one plane ahead. No other wave reads the slot, so
//   level 1 needs no barrier.
//   x neighbours: DPP wave shifts whose edge lane takes the seam value as DPP's `old` operand.
//   Seams of levels 1..K-1 go through a small double-buffered LDS table: K-1 barriers per plane.
//   Boundaries: held cells (x, y or z on the global boundary) get a zero coefficient,
//   u' = fma(0, t, u) = u, instead of a select or a branch per row: x through a per-lane
//   coefficient vector, z once per level and plane, y only in the tiles that touch y = 0 / ny-1
//   (a second, specialised copy of the level code). Exact for finite data; the one difference
//   from a copy is that a held -0.0 becomes +0.0.
//
// Region contract: output storage planes [lz_begin, lz_end) need u0 valid on
// [lz_begin - K, lz_end + K) (the engine keeps K ghost planes per side: halo = K).
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <type_traits>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int64_t resident_blocks(const void* kfn);

template <class T, int RY, int K, int WXN, bool RES>
__global__ __launch_bounds__(256) void heat7_tbk(const T* __restrict__ in, T* __restrict__ out, Geo g, T r,
                                                 int zc, int YT, double* __restrict__ resid) {
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
  // level seam table [level][parity][wave][row][side] of edge pairs (e0, e_{N-1}) written by lanes
  // 0 (side 0) and 63 (side 1), with one pair of padding at each end for the junk half of the reads
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
  // row / plane indices in 32 bits (the launcher checks the extents): fewer SGPRs
  const int ny = (int)g.ny, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  const int y0 = (yt * WYN + wy) * RY;
  const int zs = (int)g.lz_begin + zt * zc;
  const int ze = min((int)g.lz_end, zs + zc);
  const bool xin = x < g.pitch;
  const int64_t pitch = g.pitch, plane = g.plane;
  T* ob = out + y0 * pitch + xw;

  // held cells get coefficient 0: per lane for x = 0 / x >= nx-1, whole levels for z, whole rows
  // for y (only in tiles whose computed rows reach y = 0 or y = ny-1)
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);
  const Row rx = RO::coef(r, xb);
  const Row r0 = RO::zero();
  const bool yint = y0 - (K - 1) >= 1 && y0 + RY + K - 2 <= ny - 2;

  // ---- u0 streaming: rows + seam vectors of plane lz into this wave's slot ----------------------
  // All lanes of every DMA are active: rows outside [0, ny) and lanes beyond the row read a
  // clamped in-bounds address (those window cells never feed a valid output, and stay finite).
  // (a wave wholly beyond the row, e.g. in the last x tile, reads no seam: it stores nothing)
  const bool has_l = xw > 0 && xw < pitch, has_r = xw + WX < pitch;
  const int srow = lane & 31;
  const bool son = lane < 32 ? (has_l && srow < R0) : (WXN > 1 && has_r && srow < R0);
  // per-lane parts of the DMA addresses as 32-bit byte offsets from the wave-uniform start of the
  // row (x = 0), so the loads use the SGPR-base + VGPR-offset form (one VGPR per address instead
  // of a 64-bit pair per row). Every offset is a clamped column in [0, pitch - N], never negative:
  // lanes beyond the row (possibly a whole wave) read the row's last vector.
  const uint32_t xcb = (uint32_t)((xin ? x : pitch - N) * (int64_t)sizeof(T));
  const uint32_t socb = son ? (uint32_t)((lane < 32 ? xw - N : xw + WX) * (int64_t)sizeof(T)) : xcb;
  const T* ib0 = in + (y0 - K) * pitch;  // u0 window row k, column 0
  auto rowc = [&](int k) -> int {  // window row k, clamped into [0, ny)
    const int y = y0 - K + k;
    return (y < 0 ? 0 : y >= ny ? ny - 1 : y) - (y0 - K);
  };
  const int srowc = rowc(srow < R0 ? srow : 0);
  // buffer-descriptor DMAs on the wave-uniform plane base (blds16s: row offset in the SGPR field,
  // the lane's column in the VGPR one), so the LDS reads that follow get partial lgkmcnt waits
  auto issue = [&](int lz) {
    uint64_t pbs = (uint64_t)(uintptr_t)(ib0 + (int64_t)lz * plane);
    asm volatile("" : "+s"(pbs));
    const char* pb = (const char*)(uintptr_t)pbs;
    const __amdgpu_buffer_rsrc_t rs = row_rsrc(pb);
#pragma unroll
    for (int k = 0; k < R0; ++k) {
      const uint32_t ro = (uint32_t)((int64_t)rowc(k) * pitch * (int64_t)sizeof(T));
      dcheck(g, in, (const T*)(pb + ro + xcb), N);
      blds16s(rs, xcb, ro, &slot[w][k][0]);
    }
    if (WXN > 1) {  // srowc is per lane: its row term goes in the VGPR offset
      const uint32_t o = (uint32_t)((int64_t)srowc * pitch * (int64_t)sizeof(T)) + socb;
      dcheck(g, in, (const T*)(pb + o), N);
      blds16(rs, o, &slot[w][R0][0]);
    }
  };
  // Seam reads: ONE ds_read2 per row gives lane 0 the left neighbour's last cell in `lo` and lane
  // 63 the right neighbour's first cell in `hi` (per-lane base, the other half is junk).
  //   level 0 (DMA'd seam vectors): lo = base0[j*N], hi = base0[j*N + 32*N]
  //   levels 1.. (edge pair table):  lo = base1[j*4], hi = base1[j*4 + 1]
  const T* base0 = (const T*)&slot[w][R0][0] + (lane < 32 ? N - 1 : 0);
  const int wl = wx > 0 ? w - 1 : w, wr = wx < WXN - 1 ? w + 1 : w;
  const T* base1 = lane < 32 ? &tb[2 + wl * TB_W + 2 + 1] : &tb[2 + wr * TB_W + 0 - 1];
  T* wrp = &tb[2 + w * TB_W + (lane == 0 ? 0 : 2)];  // this lane's edge-pair slot (lanes 0 / 63)

  Row S[TOT], C[TOT];
#pragma unroll
  for (int i = 0; i < TOT; ++i) {
    S[i] = RO::zero();
    C[i] = RO::zero();
  }
  // output stores per stored plane (wave-uniform; a wave with no lane in the row issues none)
  const int nsto = __builtin_amdgcn_ballot_w64(xin) != 0 ? max(0, min(RY, ny - y0)) : 0;
  int nst = 0;  // stores issued since this wave's last DMA
  double acc = 0.0;
  const int cend = ze + K;
  issue(zs - K);
  for (int c = zs - K; c < cend; ++c) {
    const int par = (int)(c & 1);
    wait_vm_le(nst);  // this wave's DMA of plane c has landed (its later stores may not have)
    Row X[R0];
    T LO[R0], HI[R0];
    auto ld0 = [&](int k) __attribute__((always_inline)) {
      X[k] = RO::lds((const T*)&slot[w][k][lane]);
      if (k >= 1 && k < R0 - 1) {
        // a wave edge without a neighbouring wave (the global x boundary, or a narrow row's only
        // wave) has no DMA'd seam: its slot row holds stale LDS, possibly a NaN pattern, which
        // the held edge cell's zero coefficient would not cancel (0 * NaN): use 0 instead
        LO[k] = has_l ? base0[k * N] : T(0);
        HI[k] = (WXN > 1 && has_r) ? base0[k * N + 32 * N] : T(0);
      }
    };
#pragma unroll
    for (int k = 0; k < R0; ++k) ld0(k);
    wait_lgkm0();  // slot consumed: refill it with the next plane while the levels compute
    asm volatile("" ::: "memory");
    if (c + 1 < cend) issue(c + 1);

#pragma unroll
    for (int k = 1; k <= K; ++k) {
      const int ROUT = RY + 2 * (K - k);
      const int off = tbk_off<RY, K>(k);
      // block-uniform: level k starts once its inputs are valid planes (the first 2K iterations
      // fill the pipeline)
      if (c >= zs - K + 2 * k - 2) {
        if (k >= 2 && WXN > 1) {
          const T* b1 = base1 + (k - 2) * TB_LV + par * TB_PAR;
#pragma unroll
          for (int j = 1; j <= ROUT; ++j) {
            LO[j] = b1[j * TB_ROW];
            HI[j] = b1[j * TB_ROW + 1];
          }
        }
        const int gz = c - k + gzoff;  // plane finished by this level: c - k
        // z-held planes through a wave-uniform 0 / 1 factor (2 packed multiplies, not 8 selects)
        const Row rl = RO::scale(rx, (gz <= 0 || gz >= gnz - 1) ? T(0) : T(1));
        Row Y[R0];
        auto rows = [&](auto edge) __attribute__((always_inline)) {
          constexpr bool EDGE = decltype(edge)::value;
#pragma unroll
          for (int i = 0; i < ROUT; ++i) {
            Row ri = rl;
            if (EDGE) {
              const int y = y0 - (K - k) + i;
              if (y == 0 || y == ny - 1) ri = r0;
            }
            const Row cen = X[i + 1];
            const Row cold = C[off + i];
            const Row o = RO::fin(S[off + i], cen, cold, ri);
            const T l = lane_up1_or(LO[i + 1], RO::last(cen));
            const T rr = lane_down1_or(HI[i + 1], RO::first(cen));
            S[off + i] = RO::partial(cen, l, rr, X[i], X[i + 2], cold);
            C[off + i] = cen;
            Y[i] = o;
            if (RES && k == K && c >= zs + K && y0 + i < ny && xin) {
#pragma unroll
              for (int e = 0; e < N; ++e)
                if (x + e < g.nx) {
                  const double d = (double)RO::get(o, e) - (double)RO::get(cold, e);
                  acc += d * d;
                }
            }
          }
        };
        if (yint)
          rows(std::integral_constant<bool, false>{});
        else
          rows(std::integral_constant<bool, true>{});
        if (k < K) {
          if (WXN > 1) {  // publish the edge pairs of the rows the next level uses as centres
            if (lane == 0 || lane == 63) {
              T* wp = wrp + (k - 1) * TB_LV + par * TB_PAR;
#pragma unroll
              // a compiler-visible store: hipcc drains this wave's in-flight DMA (vmcnt(0)) before
              // it. Measured faster here than lds_store() without the drain (1024^3 fp32 K=2 1274
              // vs 1125 GCells/s, K=3 1121 vs 1071); the occupancy-1 kernels (K=4, box27_tbk)
              // gain from lds_store() instead (profiles/archive/r02_lds_store_drain.txt)
              for (int j = 1; j < ROUT - 1; ++j) *(typename RO::T2*)(wp + j * TB_ROW) = RO::edges(Y[j]);
            }
            lds_barrier();
          }
#pragma unroll
          for (int j = 0; j < ROUT; ++j) X[j] = Y[j];
        } else if (c >= zs + K) {  // u_K(c - K) is an owned output plane
          nst = nsto;
          const int lz = c - K;
#pragma unroll
          for (int i = 0; i < RY; ++i) {
            if (y0 + i < ny && xin) {
              T* a = (T*)((char*)(ob + (int64_t)lz * plane + (int64_t)i * pitch) + xo * (uint32_t)sizeof(T));
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

}  // namespace dev
}  // namespace mdfx

namespace mdfx {
namespace dev {

// z-chunk of a streaming sweep. Each chunk pays 2K planes of pipeline fill, and the z-march
// needs no short chunks for L2 sharing (y-neighbour tiles are co-resident and march in lockstep),
// so chunks are long: R whole rounds of resident blocks, R = planes-per-slot / 128 clamped to
// [1, 4]. One single round has the best minimum but the worst mean sweep time (slow blocks are
// never rebalanced); about 4 rounds are as fast on average with a small spread. Per-dispatch
// means on 1024^3 fp32, K = 2 (profiles/archive/r01_tbk/zc_dispatch_stats.txt): zc 512 / 256 / 171 /
// 128 / 86 -> 1.768 / 1.770 / 1.646 / 1.671 / 1.646 ms per sweep; the N = 8 slab (128 planes,
// best of 3 x 20): zc 128 / 64 / 43 -> 1025 / 1358 / 1082 GCells/s.
// Every chunk also pays 2K planes of pipeline fill, so a region is never split into chunks shorter
// than 4K planes: under the 2-round policy of multi-slab runs the K-plane boundary regions were
// split in two (8 slabs of 1024^2 x 128 at K = 3: 1369 vs 1491 GCells/s, profiles/archive/r02_wtk/README.txt).
int tbk_zc(int64_t planes, int64_t tiles, int64_t resident, int K, int min_rounds) {
  const double per_slot = (double)planes * (double)tiles / (double)resident;
  const int64_t rounds = std::max<int64_t>(min_rounds,
                                           std::min<int64_t>(4, (int64_t)(per_slot / 128.0 + 0.5)));
  const int64_t zt = std::max<int64_t>(1, std::min<int64_t>(planes, (rounds * resident + tiles / 2) / tiles));
  const int64_t zc = (planes + zt - 1) / zt;
  return (int)std::max<int64_t>(zc, std::min<int64_t>(planes, 4 * (int64_t)K));
}

template <class T>
bool heat7_tbk_supported(const Geo& g, int steps) {
  constexpr int WX = 64 * VT<T>::N;
  // the row in one block (wider rows at K = 2: heat7_tb2 x tiles, 533 vs 483 GCells/s for these
  // kernels' x tiles at 2048^3 fp64, profiles/archive/r02_ab_f64_2048.txt)
  // (K = 3 / 4 run heat7_wtk / heat7_wxk: this kernel's deeper sweeps measured slower and were
  // removed in round 5 with the switch that reached them, profiles/archive/r01_tbk/, r02_wtk/README.txt)
  return steps == 2 && g.pitch <= 4 * WX && g.nx >= 1 && g.ny >= 1;
}
template bool heat7_tbk_supported<float>(const Geo&, int);
template bool heat7_tbk_supported<double>(const Geo&, int);

template <class T, int RY, int K, int WXN>
static void launch_tbk_w(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int WYN = 4 / WXN;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int YT = (int)((g.ny + WYN * RY - 1) / (WYN * RY));
  const void* kfn = (const void*)&heat7_tbk<T, RY, K, WXN, false>;
  const int zc = tbk_zc(planes, YT, resident_blocks(kfn), K, g.min_rounds);
  const int ZT = (int)((planes + zc - 1) / zc);
  const dim3 grd((unsigned)((int64_t)YT * ZT)), blk(256);
  if (resid)
    hipLaunchKernelGGL((heat7_tbk<T, RY, K, WXN, true>), grd, blk, 0, s, in, out, g, r, zc, YT, resid);
  else
    hipLaunchKernelGGL((heat7_tbk<T, RY, K, WXN, false>), grd, blk, 0, s, in, out, g, r, zc, YT, resid);
}

template <class T, int RY, int K>
static void launch_tbk_t(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  constexpr int WX = 64 * VT<T>::N;
  if (g.pitch > 2 * WX)
    launch_tbk_w<T, RY, K, 4>(g, in, out, r, resid, s);
  else if (g.pitch > WX)
    launch_tbk_w<T, RY, K, 2>(g, in, out, r, resid, s);
  else
    launch_tbk_w<T, RY, K, 1>(g, in, out, r, resid, s);
}

// Two fused steps. Rows per tile: 4 (1 on very short columns): RY 4 1351 GCells/s vs 3 1199, 2 1189
// (profiles/archive/r01_tbk/ab_1024_f32.log).
template <class T>
void launch_heat7_tbk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  // region contract: u0 is read on [lz_begin - K, lz_end + K)
  MDFX_CHECK(steps == 2 && g.lz_begin >= steps && g.lz_end + steps <= g.lz_max,
             format("heat7_tbk: %d fused steps need %d valid planes around [%lld, %lld) of %lld", steps, steps,
                    (long long)g.lz_begin, (long long)g.lz_end, (long long)g.lz_max));
  MDFX_CHECK(g.pitch <= 4 * 64 * VT<T>::N, "heat7_tbk: the row must fit one block");
  MDFX_CHECK(g.ny < ((int64_t)1 << 30) && g.lz_max < ((int64_t)1 << 30) && g.gnz < ((int64_t)1 << 30) &&
                 g.gz_off > -((int64_t)1 << 30) && g.gz_off < ((int64_t)1 << 30),
             "heat7_tbk: row / plane counts must fit 32-bit indices");
  if (g.ny < 8)
    launch_tbk_t<T, 1, 2>(g, in, out, r, resid, s);
  else
    launch_tbk_t<T, 4, 2>(g, in, out, r, resid, s);
}
template void launch_heat7_tbk<float>(const Geo&, const float*, float*, float, int, double*, hipStream_t);
template void launch_heat7_tbk<double>(const Geo&, const double*, double*, double, int, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
