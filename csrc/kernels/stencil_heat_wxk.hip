// Deep temporal blocking for the 3D 7-point stencil with the y halo EXCHANGED between the waves of
// a band instead of recomputed (heat7_wxk): K = 3 or 4 fused steps per sweep (fp32 also K = 5, in
// rows of 2 cells per lane), one block barrier per plane, bitwise equal to K single steps.
//
// heat7_wtk (stencil_heat_wtk.hip) makes every wave of a y band compute the RY + 2(K-l) rows that
// its own level l+1 needs: at K = 3, 3-row waves, 15 row updates per plane for 9 output rows. Most
// of those extra rows are rows the neighbouring wave of the same band computes anyway. Here a
// wave computes only its own RY rows at every level; the rows just above and below it come from
// its neighbours through a small LDS seam table. Only the band's first and last waves still
// compute a one-sided trapezoid of K-l extra rows (the rows outside the band). Row updates per
// output row, 8-wave bands: 1.06 (K = 3, 4-row waves) / 1.13 (K = 4, 3-row waves), against 1.67
// for heat7_wtk's 3-row waves at K = 3.
//
// Why one barrier per plane is still enough: the plane loop streams u0 plane q in and finishes
// level l at plane m = q - l. The z neighbours of u_l(m) are the wave's own rows
// (u_{l-1}(m-1), u_{l-1}(m+1): the latter is computed earlier in the same step), and its in-plane
// neighbours are u_{l-1}(m), which every wave computed in the PREVIOUS step. So a wave publishes
// the first and last of its own rows of levels 1..K-1 into the seam table as it computes them
// (parity q & 1), and after the next plane's barrier the neighbours read them. The in-plane
// partial sum S = (((xm + xp) + ym) + yp) + zm of u_l(m) is therefore formed at the top of the
// step, from the two stored planes m-1, m of level l-1 and the seam rows, and the step finishes
// u_l(m) = fma(r, fma(-6, C, S + zp), C) with zp = u_{l-1}(m+1) the moment that row is computed:
// one row cascades through all K levels (sm::heat7's operation order, so the result is bitwise
// that of K single steps).
//
// Per row and level the state is two stored planes of level l-1 (ping-ponged between the two
// halves of a 2-plane unrolled loop, so no row is ever copied); level 1 keeps heat7_wtk's
// (S, C) pair fed straight from the u0 window. x: overlapping segments of 64 lanes x N cells
// (OV lanes per side), DPP lane shifts -- as heat7_wtk. u0: the band's rows stream by LDS DMA into
// a double-buffered window one plane ahead -- as heat7_wtk. Boundaries: held cells get a zero
// coefficient; the band-edge waves' trapezoid rows outside the grid read clamped (finite) rows and
// never feed an unheld cell.
//
// The band's first, inner and last waves run different compiled copies of the march (their row
// counts differ). Each copy executes exactly one s_barrier per plane step over the same block-
// uniform step range, and gfx9's s_barrier counts arriving waves rather than requiring one code
// path, so the copies meet at every barrier (tests: bands with every role, tall and short grids).
//
// Region contract (as heat7_wtk): output storage planes [lz_begin, lz_end) (and optionally a
// second region [lz2_begin, lz2_end)) need u0 valid on [lz_begin - K, lz_end + K).
//
// Reference parity: the generation update MDF_kernel.cu:10-22 (here in 3D, K generations per
// pass over HBM instead of one generation per host round trip, MDF_kernel.cu:155-188).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <type_traits>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "wxk_common.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int64_t resident_blocks(const void* kfn, int block);

// PEN: the pencil copy (output rows [ly_begin, ly_end) of storage rows holding ghost rows, global
// row = storage row + gy_off). Slabs run the copy without it: the four extra row bounds held in
// scalars cost the slab sweep ~4 % (six more vmcnt(0) waits in front of window reads, round 4).
// One block's arrival at the folded boundary (one out-of-line copy for every march variant): the
// wave's stores of the lower planes complete (vmcnt 0: acknowledged by this XCD's L2), the block
// barrier, then one lane counts the arrival; the block that completes the count re-arms it and bumps
// the sweep counter sig[16]. No cache maintenance here by default (see fold_release below): the
// halo stream's counter-wait kernel ends with the dispatch packet's release, which writes back
// every XCD's L2 before the exchange reads the face. (A per-block agent-scope release - an L2 writeback, and with acq_rel an L2 invalidate, by
// each of the 235 blocks - slowed the whole sweep by ~25 %.) The upper boundary launch and the
// interior sweep count on separate counter blocks (Solver::Slab::sig), and each launch follows the
// previous one on its stream, so no block of a launch arrives before the re-arm of the last one
// that used its counters. (A monotonic count compared modulo `tiles` would need no re-arm, but
// its 64-bit division around this out-of-line call makes the sweep spill.)
// fold_release (MDFX_FOLD_RELEASE=1, opt-in): the leader first writes back its XCD's L2 with a
// system-scope release fence (no invalidate), after every wave's stores of the block are in that L2,
// so each signalling block publishes its own face tiles to memory instead of relying on the halo
// stream's counter-wait dispatch to write every L2 back. (A release by the last-arriving block
// alone would not do: buffer_wbl2 writes back only the L2 of the XCD that executes it.) Round 6
// A/B, interleaved on one box: rank proxy N = 8 2,111 / 2,041 GCells/s without, 2,009 / 2,026 with
// (-2.8 %), N = 4 2,449 vs 2,409 (-1.7 %); the K = 4 / 5 folded ipc and proxy tests pass with it
// (profiles/r06_session_d/). Over the 1 % budget, so it stays opt-in.
// What the default relies on: the counter-wait kernel on the halo stream ends with its dispatch
// packet's system-scope release, which the HIP runtime implements as a writeback of every XCD's
// L2 (the whole cache, not only that kernel's lines). The exchange's copies are dispatched after
// it on the same stream. That whole-L2 writeback is an implementation property, not an HSA
// guarantee; tests/test_gpu_ipc.py checks it for blit and SDMA readers (SDMA, like a peer GPU over
// xGMI, reads memory without going through this device's L2).
__device__ __noinline__ void wxk_fold_signal(unsigned long long* sig, int tiles, bool leader, bool release) {
  wait_vm0();
  lds_barrier();
  if (leader) {
    if (release) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      wait_vm0();  // the writeback has completed before the arrival is counted
    }
    const unsigned long long n = __hip_atomic_fetch_add(sig, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
    if (n == (unsigned long long)tiles) {
      __hip_atomic_store(sig, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(sig + 16, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// SIG: the folded-boundary copy (Geo::sig): the blocks of the chunks starting at lz_begin publish their
// output planes [lz_begin, sig_z) and signal, so the halo exchange of the lower face overlaps the
// rest of the same sweep (no separate boundary launch for that face).
// CN = kRowOps2: fp32 rows of 2 cells per lane (RowOps2f; the 5-step sweep), the window filled by
// 4-byte LDS DMAs (an x segment of 2-cell lanes starts 2 cells off a 16-B vector, so neither a 16-B
// nor an 8-B DMA lane would line up with the grid's column 0).
template <class T, int RY, int RE, int K, int WB, bool RES, bool PEN = false, bool SIG = false, int CN = 0>
__global__ __launch_bounds__(WB * 64) void heat7_wxk(const T* __restrict__ in, T* __restrict__ out, Geo g, T r,
                                                     int zc, int XT, int YT, int ntasks, double* __restrict__ resid) {
  constexpr bool NAR = CN != 0;  // narrow rows: 8 bytes per lane (fp32 2 cells, fp64 1 cell)
  static_assert(CN != kRowOps2 || sizeof(T) == 4, "heat7_wxk: 2-cell lanes are fp32");
  static_assert(CN != kRowOps1 || sizeof(T) == 8, "heat7_wxk: 1-cell lanes are fp64");
  using RO = typename std::conditional<
      CN == kRowOps2, RowOps2f,
      typename std::conditional<CN == kRowOps1, RowOps1d,
                                typename std::conditional<sizeof(T) == 4, RowOpsN, RowOps<T>>::type>::type>::type;
  using V = typename RO::V;
  using Row = typename RO::Row;
  constexpr int N = CN == kRowOps2 ? 2 : CN == kRowOps1 ? 1 : VT<T>::N;
  constexpr int OV = (K + N - 1) / N;     // overlap lanes per side
  constexpr int SEG = (64 - 2 * OV) * N;  // owned columns per wave
  constexpr int BR = 2 * RE + (WB - 2) * RY;  // output rows of a band
  constexpr int RB = BR + 2 * K;              // u0 window rows of a band: yb-K .. yb+BR+K-1
  constexpr int NM = RY > RE + K - 1 ? RY : RE + K - 1;  // most rows any wave computes at level 1
  static_assert(WB >= 2 && K >= 2, "heat7_wxk: bands of at least two waves, at least two levels");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // work: block-uniform task = one z chunk of one (x segment, y band) tile; x segments fastest, then
  // y bands, then z chunks (the first region's chunks, then the second region's)
  const int b = (int)xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntasks) return;
  // two window buffers: the u0 plane DMA runs one plane ahead of the plane being computed
  __shared__ V win[2][RB][64];
  // seam[parity][level-1][boundary between waves s and s+1][0: first row of wave s+1, 1: last row of wave s]
  __shared__ V seam[2][K - 1][WB - 1][2][64];
  // (A second plane in flight does not help this sweep: a third window buffer with one seam table
  // and a second barrier lost in round 3 (profiles/archive/r03_session_r/); an L2 prefetch of plane q + 2 by
  // 4-byte LDS DMAs lost 15-24 % in round 4 (profiles/r04_session_b/) and 15 % in round 5; the DMA
  // two planes ahead in these two buffers (a second barrier per step right after the window reads)
  // lost 4-6 %, non-temporal window DMAs 19 % (profiles/r05_session_b/, r05_session_c/).)
  const int tiles = XT * YT;
  const int t = b % tiles, zt = b / tiles;
  const int P0 = (int)(g.lz_end - g.lz_begin);
  const int zt1 = (P0 + zc - 1) / zc;
  int zs, ze;
  if (zt < zt1) {
    zs = (int)g.lz_begin + zt * zc;
    ze = min((int)g.lz_end, zs + zc);
  } else {
    zs = (int)g.lz2_begin + (zt - zt1) * zc;
    ze = min((int)g.lz2_end, zs + zc);
  }
  const int xt = t % XT, yt = t / XT;
  const int64_t xs = (int64_t)xt * SEG - OV * N;  // column of lane 0
  const int64_t x = xs + (int64_t)lane * N;
  const int ny = (int)g.ny, lzmax = (int)g.lz_max, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  // rows: storage rows [0, ny) (a pencil's include ghost rows), output rows [ly0, ly1), global row =
  // storage row + gyoff of gny (slabs: ly0 = 0, ly1 = ny = gny, gyoff = 0)
  const int ly0 = PEN ? (int)g.ly_begin : 0, ly1 = PEN ? (int)g.ly_end : ny, gyoff = PEN ? (int)g.gy_off : 0,
            gny = PEN ? (int)g.gny : ny;
  const int yb = ly0 + yt * BR;                        // first row of the band
  const int y0 = yb + (w == 0 ? 0 : RE + (w - 1) * RY);  // first own row of this wave
  const int rown = (w == 0 || w == WB - 1) ? RE : RY;    // own rows of this wave
  const int64_t pitch = g.pitch, plane = g.plane;
  const bool xin = x >= 0 && x < pitch;
  const bool own = lane >= OV && lane <= 63 - OV && xin;
  // Output stores are non-temporal except in the two owned lanes at each end of the x segment: the
  // 116-column segments of the 5-step sweep split a 32-B sector at every other seam, and the two
  // blocks' non-temporal partial-sector writes reached memory separately (1.066 fields written per
  // K = 5 sweep, 6.1 M 32-B requests); plain stores merge in the L2 first: 1.009 fields, kernel A/B
  // +0.9 % (round 6, profiles/r06_session_d/; all-plain stores write the same bytes)
  const bool seam_lane = lane <= OV + 1 || lane >= 62 - OV;
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e == 0) || (x + e >= g.nx - 1);
  const Row rx = RO::coef(r, xb);
  const Row r0 = RO::zero();
  // block-uniform: every row the band computes at any level is y-interior (globally), so no wave
  // needs the per-row held test (bands at global y = 0 / gny-1 run the tested copy, all their waves
  // together)
  const bool yint = yb - (K - 1) + gyoff >= 1 && yb + BR + K - 2 + gyoff <= gny - 2;
  const int nsto = __builtin_amdgcn_ballot_w64(own) != 0 ? max(0, min(rown, ly1 - y0)) : 0;
  int nst = 0;  // output stores issued since this wave's last DMA

  // u0 plane lz -> window buffer `buf` by LDS DMA; rows outside [0, ny) and lanes outside the row
  // read the nearest valid row / vector. Wave w fetches rows w, w + WB, ... of the window.
  const uint32_t xcb = (uint32_t)((x < 0 ? 0 : x >= pitch ? pitch - N : x) * (int64_t)sizeof(T));
  // (narrow rows: the window row's 512 bytes as two halves of one dword per lane: fp32 2-cell lanes
  // fetch cells xs + 64 h + lane, fp64 1-cell lanes dword 64 h + lane of the segment, i.e. half of
  // cell xs + 32 h + lane / 2; cells outside the row clamp to the nearest valid one)
  constexpr int DPC = (int)sizeof(T) / 4;  // dwords per cell
  uint32_t xch[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int d = h * 64 + lane;
    const int64_t xh = xs + d / DPC;
    xch[h] = (uint32_t)(((xh < 0 ? 0 : xh >= pitch ? pitch - 1 : xh) * DPC + d % DPC) * 4);
  }
  auto issue = [&](int lz, int buf) {
    const int lzc = lz < 0 ? 0 : lz >= lzmax ? lzmax - 1 : lz;
#pragma unroll
    for (int j = 0; j < (RB + WB - 1) / WB; ++j) {
      const int k = w + j * WB;
      if (k < RB) {
        const int y = yb - K + k;
        const int yc = y < 0 ? 0 : y >= ny ? ny - 1 : y;
        // the row's address is wave-uniform: pinned in SGPRs, so the DMA takes the scalar-base +
        // 32-bit lane-offset form instead of a 64-bit VGPR address per row held across the loop
        uint64_t rb = (uint64_t)(uintptr_t)(in + (int64_t)lzc * plane + (int64_t)yc * pitch);
        asm volatile("" : "+s"(rb));
        // fp64: buffer-descriptor DMA (blds16 / blds4), so the step's LDS reads get partial lgkmcnt
        // waits (2048^3 + residual every 12 / 20: 1048 / 1160 vs 1031 / 1138 GCells/s); fp32 keeps
        // global_load_lds: 1024^3 within +-1 %, 3072^3 2272-2310 vs 2450-2493 with the buffer form
        // (profiles/r06_session_{p,s}/)
        if constexpr (sizeof(T) == 8) {
          const __amdgpu_buffer_rsrc_t rs = row_rsrc((const void*)(uintptr_t)rb);
          if constexpr (NAR) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + (xch[h] & ~(uint32_t)(sizeof(T) - 1))), 1);
              blds4(rs, xch[h], (char*)&win[buf][k][0] + h * 256);
            }
          } else {
            dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + xcb), N);
            blds16(rs, xcb, &win[buf][k][0]);
          }
        } else if constexpr (NAR) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const char* a = (const char*)(uintptr_t)rb + xch[h];
            dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + (xch[h] & ~(uint32_t)(sizeof(T) - 1))), 1);
            glds4(a, (char*)&win[buf][k][0] + h * 256);
          }
        } else {
          const T* a = (const T*)((const char*)(uintptr_t)rb + xcb);
          dcheck(g, in, a, N);
          glds16(a, &win[buf][k][0]);
        }
      }
    }
  };
  const int qlast = ze - 1 + K;  // last u0 plane of the march
  const bool sig_blk = SIG && zs == (int)g.lz_begin;
  const int sig_last = SIG ? (int)g.sig_z - 1 : 0;
  issue(zs - K, 0);
  T* ob = out + (int64_t)y0 * pitch;
  const uint32_t xob = (uint32_t)((xin ? x : 0) * (int64_t)sizeof(T));
  double acc = 0.0;
  // LDS addresses pinned in VGPRs with the wave-uniform parts folded in; compile-time parts go to
  // the instructions' offset fields. Window rows from y0 - K (so every offset is non-negative).
  typedef __attribute__((address_space(3))) V LV;
  LV* const wrow = lds_vptr(&win[0][y0 - yb][lane]);
  const int wu = w > 0 ? w - 1 : 0, wd = w < WB - 1 ? w : WB - 2;
  // (the seam reads index `seam` itself: through a laundered pointer hipcc cannot tell them from
  // the window's in-flight DMA and drains it with vmcnt(0) first)
  LV* const s_first = lds_vptr(&seam[0][0][wu][0][lane]);  // my first row (write, w > 0)
  LV* const s_last = lds_vptr(&seam[0][0][wd][1][lane]);   // my last row (write, w < WB-1)
  constexpr int WIN_BUF = RB * 64;  // V elements per window buffer
  constexpr int SEAM_PAR = (K - 1) * (WB - 1) * 2 * 64, SEAM_LVL = (WB - 1) * 2 * 64;
  auto st = [](LV* p, const V& v) {
    if constexpr (sizeof(V) == 16)
      asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
    else
      asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };

  auto march = [&](auto role_c, auto edge_c) __attribute__((always_inline)) {
    constexpr int ROLE = decltype(role_c)::value;
    constexpr bool EDGE = decltype(edge_c)::value;
    using SH = WxRows<ROLE, RY, RE, K>;
    // level 1: running partial S1 and centre of u0 (ping-pong CA / CB); levels 2..K: the two
    // stored planes of the level below, H[l-2][0 / 1] (which is which alternates with the parity)
    Row S1[NM], CA[NM], CB[NM], H[K - 1][2][NM];
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      S1[i] = RO::zero();
      CA[i] = RO::zero();
      CB[i] = RO::zero();
#pragma unroll
      for (int l = 0; l < K - 1; ++l) H[l][0][i] = H[l][1][i] = RO::zero();
    }
    auto step = [&](int q, auto par_c) __attribute__((always_inline)) {
      constexpr int P = decltype(par_c)::value;
      Row(&Cin)[NM] = P == 0 ? CA : CB;
      Row(&Cout)[NM] = P == 0 ? CB : CA;
      // no instruction moves across a plane boundary (the two planes of an unrolled trip would
      // otherwise interleave, with both planes' rows live at once)
      __builtin_amdgcn_sched_barrier(0);
      // plane q's DMA has landed (the stores issued after it stay in flight); the barrier
      // publishes it and last step's seam rows, and certifies that every wave is done with the
      // other window buffer and the other seam parity
      wait_vm_le(nst);
      lds_barrier();
      if (q < qlast) issue(q + 1, P ^ 1);
      constexpr int SR = P ^ 1;  // seam parity read this step
      // z-held planes: coefficient 0 through a wave-uniform 0 / 1 factor (exact). (A copy of the
      // march without these factors for the z-interior middle gained 3.5 % in the kernel A/B but
      // nothing in the driver form, sessions r05_b / r05_c: not shipped.)
      Row rl[K + 1];
#pragma unroll
      for (int l = 1; l <= K; ++l) {
        const int gz = q - l + gzoff;
        rl[l] = RO::scale(rx, (gz <= 0 || gz >= gnz - 1) ? T(0) : T(1));
      }
      LV* const wbuf = wrow + P * WIN_BUF;
      // every LDS row this step reads (the seam rows of levels 1..K-1 and the u0 window rows) is
      // read up front: the reads overlap each other and the level-(1) arithmetic instead of each
      // waiting out a full LDS round trip right before its use (round 5: 1024^3 kernel A/B 0.4170
      // vs 0.4313 ms per step, profiles/r05_session_a/)
      constexpr int NU = SH::n(1) + 2;
      // (the residual copies of the 4-row K = 3 band read the window rows where they are used: with
      // them held the band needs 4-10 VGPRs more than it has)
      constexpr bool LAZY = RES && K == 3 && RY == 4;
      Row UP[K - 1], DN[K - 1], U[NU];
#pragma unroll
      for (int j = 1; j < K; ++j) {
        UP[j - 1] = DN[j - 1] = RO::zero();
        if (ROLE != 0) UP[j - 1] = RO::fromv(seam[SR][j - 1][wu][1][lane]);
        if (ROLE != 2) DN[j - 1] = RO::fromv(seam[SR][j - 1][wd][0][lane]);
      }
#pragma unroll
      for (int k = 0; k < NU; ++k)
        if constexpr (!LAZY) U[k] = RO::fromv(V(wbuf[(SH::lo(1) - 1 + k + K) * 64]));
      // (1) levels 2..K: S_l(m), m = q - l, into the slot of u_{l-1}(m-1) (its zm, consumed here)
#pragma unroll
      for (int l = 2; l <= K; ++l) {
        const int j = l - 1;  // level of the inputs
        const Row& up = UP[j - 1];
        const Row& dn = DN[j - 1];
#pragma unroll
        for (int i = SH::lo(l); i < SH::hi(l); ++i) {
          const int ij = i - SH::lo(j);
          const Row& c = H[j - 1][P ^ 1][ij];
          const Row& ym = (i - 1 < SH::lo(j)) ? up : H[j - 1][P ^ 1][ij - 1];
          const Row& yp = (i + 1 >= SH::hi(j)) ? dn : H[j - 1][P ^ 1][ij + 1];
          const T lft = lane_up1(RO::last(c));
          const T rgt = lane_down1(RO::first(c));
          Row& a = H[j - 1][P][ij];
          a = RO::partial(c, lft, rgt, ym, yp, a);
          RO::pin(a);
        }
      }
      // (2) level 1 row by row from the u0 window, each new row cascading up through the levels.
      // (A scheduling barrier that keeps (1), which needs only the seam rows read first, ahead of the
      // window rows' waits measured 2-3 % slower at 1024^3, round 6 session P: not shipped.)
      Row X[3];
      auto urow = [&](int i) -> Row {
        if constexpr (LAZY) return RO::fromv(V(wbuf[(i + K) * 64]));
        else return U[i - (SH::lo(1) - 1)];
      };
      X[0] = urow(SH::lo(1) - 1);
      X[1] = urow(SH::lo(1));
      const bool valid = q - K >= zs && q <= qlast;  // u_K(q - K) is an owned output plane
      const int lz = q - K;
#pragma unroll
      for (int i = SH::lo(1); i < SH::hi(1); ++i) {
        const int i1 = i - SH::lo(1);
        X[(i1 + 2) % 3] = urow(i + 1);
        const Row& xm = X[i1 % 3];
        const Row& cen = X[(i1 + 1) % 3];
        const Row& xp = X[(i1 + 2) % 3];
        const bool yh = EDGE && (y0 + i + gyoff == 0 || y0 + i + gyoff == gny - 1);
        Row ri = rl[1];
        if (yh) ri = r0;
        const Row cold = Cin[i1];
        Row cur = RO::fin(S1[i1], cen, cold, ri);  // u_1(q - 1), row i
        const T lft = lane_up1(RO::last(cen));
        const T rgt = lane_down1(RO::first(cen));
        S1[i1] = RO::partial(cen, lft, rgt, xm, xp, cold);
        RO::pin(S1[i1]);
        Cout[i1] = cen;
        // cascade: cur = u_j(q - j) for j = 1, 2, ...
#pragma unroll
        for (int j = 1; j <= K; ++j) {
          if (j == K) {  // the sweep's output row
            if (valid && i >= 0 && i < SH::R && y0 + i < ly1 && own) {
              T* a = (T*)((char*)(ob + (int64_t)lz * plane + (int64_t)i * pitch) + xob);
              dcheck(g, (const T*)out, a, N);
              if (seam_lane)
                *(V*)a = RO::vec(cur);
              else
                store_nt((V*)a, RO::vec(cur));
            }
            break;
          }
          const int ij = i - SH::lo(j);
          const bool next = i >= SH::lo(j + 1) && i < SH::hi(j + 1);  // row i exists at level j + 1
          Row nxt = cur;
          if (next) {
            Row rj = rl[j + 1];
            if (yh) rj = r0;
            const Row& bc = H[j - 1][P ^ 1][ij];  // u_j(q - j - 1): the centre of u_{j+1}(q - j - 1)
            nxt = RO::fin(H[j - 1][P][ij], cur, bc, rj);
            if (RES && j + 1 == K && valid && i >= 0 && i < SH::R && y0 + i < ly1 && own) {
#pragma unroll
              for (int e = 0; e < N; ++e)
                if (x + e < g.nx) {
                  const double d = (double)RO::get(nxt, e) - (double)RO::get(bc, e);
                  acc += d * d;
                }
            }
          }
          H[j - 1][P][ij] = cur;  // next step's centre plane of level j
          // seam rows of level j for the neighbours' next step
          if (ROLE != 0 && i == 0) st(s_first + P * SEAM_PAR + (j - 1) * SEAM_LVL, RO::vec(cur));
          if (ROLE != 2 && i == SH::R - 1) st(s_last + P * SEAM_PAR + (j - 1) * SEAM_LVL, RO::vec(cur));
          if (!next) break;
          cur = nxt;
        }
      }
      nst = valid ? nsto : 0;
      if constexpr (SIG) {
        if (sig_blk && lz == sig_last) {  // block-uniform: every wave takes this branch together
          // this wave's stores of the lower planes are acknowledged by this XCD's L2 (vmcnt 0; no
          // release: they may still sit dirty in that L2); after the barrier one lane counts the
          // block's arrival, and the last block of the launch to arrive bumps the sweep counter the
          // halo stream waits for. Visibility to the exchange rests on the counter-wait kernel's
          // end-of-dispatch release (hip_region_signals, kernels.hpp)
          wxk_fold_signal(g.sig, tiles, w == 0 && lane == 0, g.fold_release != 0);
        }
      }
    };
    // an odd plane count ends with one extra step (q = qlast + 1): no DMA, nothing stored
    for (int q = zs - K; q <= qlast; q += 2) {
      step(q, IC<0>{});
      step(q + 1, IC<1>{});
    }
  };
  if (w == 0) {
    if (yint) march(IC<0>{}, std::false_type{});
    else march(IC<0>{}, std::true_type{});
  } else if (w == WB - 1) {
    if (yint) march(IC<2>{}, std::false_type{});
    else march(IC<2>{}, std::true_type{});
  } else {
    if (yint) march(IC<1>{}, std::false_type{});
    else march(IC<1>{}, std::true_type{});
  }
  wait_vm0();  // no DMA may outlive the wave
  if (RES) wave_atomic_add(resid, acc);
}

// launch geometry of one shape: tiles, z chunks, and the rounds of resident blocks they take
struct WxGeo {
  int XT = 0, YT = 0, zc = 0;
  int64_t ntasks = 0, resident = 0, rounds = 0;
};
template <class T, int RY, int RE, int K, int WB, int CN = 0>
static WxGeo wxk_geo(const Geo& g) {
  constexpr int N = CN == kRowOps2 ? 2 : CN == kRowOps1 ? 1 : VT<T>::N, OV = (K + N - 1) / N, SEG = (64 - 2 * OV) * N;
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  WxGeo w;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int64_t planes2 = g.lz2_end > g.lz2_begin ? g.lz2_end - g.lz2_begin : 0;
  w.XT = (int)((g.nx + SEG - 1) / SEG);
  w.YT = (int)((g.ly_end - g.ly_begin + BR - 1) / BR);
  const int64_t tiles = (int64_t)w.XT * w.YT;
  w.resident = resident_blocks((const void*)&heat7_wxk<T, RY, RE, K, WB, false, false, false, CN>, 64 * WB);
  // (2-wave strip bands: the strip is on the sweep's critical path, before the exchange; chunks down
  // to K planes spread its few tiles over the device)
  w.zc = wx_zc(planes, tiles, w.resident, K, 2 * K, g.min_rounds, WB == 2 ? K : 0);
  if (planes2 > 0) w.zc = (int)std::max(planes, planes2);
  const int ZT = (int)((planes + w.zc - 1) / w.zc) + (planes2 > 0 ? (int)((planes2 + w.zc - 1) / w.zc) : 0);
  w.ntasks = tiles * ZT;
  w.rounds = (w.ntasks + w.resident - 1) / w.resident;
  return w;
}

static bool pen_geo(const Geo& g) { return g.ly_begin != 0 || g.ly_end != g.ny || g.gy_off != 0 || g.gny != g.ny; }

template <class T, int RY, int RE, int K, int WB, int CN = 0>
static void launch_wxk(const Geo& g, const T* in, T* out, T r, double* resid, hipStream_t s) {
  const WxGeo wg = wxk_geo<T, RY, RE, K, WB, CN>(g);
  const int XT = wg.XT, YT = wg.YT, zc = wg.zc;
  // only the blocks of the first z chunk signal: it must hold every plane the signal covers (a
  // chunk shorter than that would leave the halo stream waiting for a signal never sent)
  MDFX_CHECK(!g.sig || zc >= g.sig_z - g.lz_begin,
             format("heat7_wxk: z chunks of %d planes cannot carry the folded boundary's %lld planes", zc,
                    (long long)(g.sig_z - g.lz_begin)));
  const int64_t ntasks = wg.ntasks;
  MDFX_CHECK(ntasks < (int64_t)1 << 31, "heat7_wxk: too many tasks");
  const dim3 grd((unsigned)ntasks), blk(64 * WB);
  const bool pen = pen_geo(g);
  // one instance per (residual, pencil rows, folded-boundary signal) combination the engine uses
  auto go = [&](auto res_c, auto pen_c, auto sig_c) {
    hipLaunchKernelGGL((heat7_wxk<T, RY, RE, K, WB, decltype(res_c)::value, decltype(pen_c)::value,
                                  decltype(sig_c)::value, CN>),
                       grd, blk, 0, s, in, out, g, r, zc, XT, YT, (int)ntasks, resid);
  };
  using F = std::false_type;
  using Tr = std::true_type;
  if constexpr (CN != 0) {  // (the 5-step narrow-row sweeps: slabs, with or without the folded boundary)
    MDFX_CHECK(!pen, "heat7_wxk: the 5-step sweep is for slabs");
    if (g.sig) {
      MDFX_CHECK(g.lz2_end <= g.lz2_begin, "heat7_wxk: folded boundaries are for one-region slab sweeps");
      if (resid) go(Tr{}, F{}, Tr{});
      else go(F{}, F{}, Tr{});
    } else {
      if (resid) go(Tr{}, F{}, F{});
      else go(F{}, F{}, F{});
    }
  } else {
    if constexpr (WB != 8) {
      MDFX_CHECK(!g.sig, "heat7_wxk: folded boundaries run in bands of 8 waves");
    } else if (g.sig) {
      MDFX_CHECK(!pen && g.lz2_end <= g.lz2_begin, "heat7_wxk: folded boundaries are for one-region slab sweeps");
      if (resid) go(Tr{}, F{}, Tr{});
      else go(F{}, F{}, Tr{});
      return;
    }
    if (resid) {
      if (pen) go(Tr{}, Tr{}, F{});
      else go(Tr{}, F{}, F{});
      return;
    }
    if (pen) go(F{}, Tr{}, F{});
    else go(F{}, F{}, F{});
  }
}

bool heat7_wxk_supported(int steps) { return steps == 3 || steps == 4; }

// Shipped bands of 8 waves: fp32 K = 4 in 2 + 6 x 3 + 2 rows (3-row inner waves, 2-row edge
// waves): 1024^3 2387-2394 GCells/s on every box measured; 4-row inner waves ran 2415-2454 on one
// box and 2095-2138 on two others (near the LDS limit, 156 KB), 2-row waves 2247-2253; on thin slabs the 3-row band also
// fills one round of resident blocks best (N = 8 proxy: 1798 vs 1657 for 4 rows)
// (profiles/archive/r03_wxk/). fp32 K = 3 (step-count remainders): 4-row waves. fp64 K = 3: 3 + 1-row bands
// (2048^3 + residual: 897 vs 861 for 3 + 2, 862 for 2 + 2); fp64 K = 4: 2 + 1-row bands (254 VGPRs;
// the 2 + 2, 3 + 1 and 3 + 2-row bands spill), 1024^3 1112-1124 GCells/s against 418 for heat7_wtk's
// 1-row K = 4 and 870-885 at K = 3 (profiles/r04_session_o/). fp32 K = 4 in 3 + 1 and 2 + 1-row
// bands measured slower (1024^3 kernel A/B 2256 / 2223 vs 2523 GCells/s, driver form 2148 / 2121 vs
// 2372; profiles/r04_session_r/). Round 3's other shapes (4-wave bands, 2-row fp32 bands, the 5-step
// sweep, 3 window buffers /
// one seam table) measured slower and were removed in round 4; their numbers stay in
// profiles/archive/r03_wxk/ and profiles/archive/r03_session_r/.
// fp32 K = 5 (round 5): rows of 2 cells per lane (RowOps2f: half the registers per row, so a fifth
// level fits), 5 + 4-row bands of 8 waves (38 rows; 9 x segments of 116 columns x 27 bands = 243
// tiles at 1024 cells, one round; 245 VGPRs). 1024^3 kernel A/B 2689 vs 2426 GCells/s for K = 4,
// 768^3 2349 vs 1954, 512^3 2187 vs 2039, 1024^2 x 128 2536 vs 2384 (profiles/r05_session_t/,
// r05_session_u/); 6 + 1-row bands measured 3 % slower; K = 6 spills in every band that fits one
// round.
// fp64 K = 5 (round 6): rows of 1 cell per lane (RowOps1d: the register footprint of the fp32 2-cell
// rows, 243 VGPRs in the same 5 + 4-row bands; each x neighbour costs two DPP moves, and a segment
// owns 54 of its 64 lanes' columns at one cell per lane). 2048^3 + residual every 20 1120 vs 1058
// GCells/s for K = 4; 1024^3 1011-1035 vs 1062-1080 (19 x 27 = 513 tiles on 256 CUs), so the auto
// depth takes it from 2048-cell rows only (hip_fused_depth; profiles/r06_session_b/).
template <class T>
void launch_heat7_wxk(const Geo& g, const T* in, T* out, T r, int steps, double* resid, hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  MDFX_CHECK((steps >= 3 && steps <= 5) && g.lz_begin >= steps && g.lz_end + steps <= g.lz_max,
             format("heat7_wxk: %d fused steps need %d valid planes around [%lld, %lld) of %lld", steps, steps,
                    (long long)g.lz_begin, (long long)g.lz_end, (long long)g.lz_max));
  MDFX_CHECK(g.lz2_end <= g.lz2_begin || (g.lz2_begin >= g.lz_end && g.lz2_end + steps <= g.lz_max),
             "heat7_wxk: the second region must follow the first and have its planes + ghosts allocated");
  MDFX_CHECK(g.pitch % VT<T>::N == 0, "heat7_wxk: the row pitch must be a whole number of vectors");
  MDFX_CHECK(g.ny < ((int64_t)1 << 30) && g.gny < ((int64_t)1 << 30) && g.lz_max < ((int64_t)1 << 30) &&
                 g.gnz < ((int64_t)1 << 30) && g.gy_off > -((int64_t)1 << 30) && g.gy_off < ((int64_t)1 << 30) &&
                 g.gz_off > -((int64_t)1 << 30) && g.gz_off < ((int64_t)1 << 30),
             "heat7_wxk: row / plane counts must fit 32-bit indices");
  // a pencil's y-boundary strip (K rows next to a y neighbour, over the interior planes): bands of
  // 2 + 2 rows in 2-wave blocks instead of 22-row bands of 8 waves that would compute 4 useful rows
  // (and 4 blocks per CU, so the strip's few tiles split into many z chunks)
  const bool strip = g.ly_end - g.ly_begin <= 4 && (g.ly_begin != 0 || g.ly_end != g.ny);
  // (round 6: only the fp32 K = 4 strip, the pencils' default depth, keeps its 2-wave instance; the
  // K = 3 strips (step-count tails) and fp64 strips run in the regular 8-wave bands, which compute
  // more rows than the strip needs but are correct for any row range: 8 fewer kernel instances,
  // ~320 KB of code object, and no more 322-VGPR fp64 K = 4 strip copy spilling into AGPRs)
  if constexpr (sizeof(T) == 4) {
    if (strip && steps == 4) {
      launch_wxk<T, 2, 2, 4, 2>(g, in, out, r, resid, s);
      return;
    }
  }
  if constexpr (sizeof(T) == 4) {
    if (steps == 5) {
      launch_wxk<T, 5, 4, 5, 8, kRowOps2>(g, in, out, r, resid, s);
      return;
    }
    if (steps == 3) launch_wxk<T, 4, 4, 3, 8>(g, in, out, r, resid, s);
    else launch_wxk<T, 3, 2, 4, 8>(g, in, out, r, resid, s);
  } else {
    if (steps == 5) {  // (1 cell per lane: RowOps1d, the 2-cell fp32 sweep's register footprint)
      launch_wxk<T, 5, 4, 5, 8, kRowOps1>(g, in, out, r, resid, s);
      return;
    }
    // (K = 4: 2 + 1-row bands, 254 VGPRs; 2 + 2, 3 + 1 and 3 + 2 rows spill)
    if (steps == 3) launch_wxk<T, 3, 1, 3, 8>(g, in, out, r, resid, s);
    else launch_wxk<T, 2, 1, 4, 8>(g, in, out, r, resid, s);
  }
}
template void launch_heat7_wxk<float>(const Geo&, const float*, float*, float, int, double*, hipStream_t);
template void launch_heat7_wxk<double>(const Geo&, const double*, double*, double, int, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
