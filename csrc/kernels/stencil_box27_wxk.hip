// Deep temporal blocking for the 3D 27-point stencil with the y halo exchanged between the waves
// of a band (box27_wxk): K = 3 fused steps per sweep, one block barrier per plane, bitwise equal to
// K single box27_zw steps.
//
// The update is box27_zw's per-plane factorisation: for a plane k and an output column (x, y),
//   H(y) = v(x-1,y) + v(x+1,y);  cross = H(y) + (v(x,y-1) + v(x,y+1));  diag = H(y-1) + H(y+1)
//   A(k) = c3*diag + c2*cross + c1*v;  B(k) = c2*diag + c1*cross + c0*v      (sm::box27_A / _B)
//   u'(m) = (A(m-1) + B(m)) + A(m+1)                                        (sm::box27_combine)
// so every level keeps, per row, the running sum S(m) = A(m-1) + B(m) and the last A.
//
// Band organisation as heat7_wxk (stencil_heat_wxk.hip): WB waves stacked along y on one x segment
// (overlapping segments, DPP lane shifts), the band's u0 rows streamed by LDS DMA into a
// double-buffered window, each wave computing only its own rows at every level (the band's edge
// waves add a one-sided trapezoid). The difference from the 7-point: A(m+1) needs the in-plane
// neighbours (y +- 1) of plane m+1 of the level below, not just its centre column, so a level
// cannot use a plane its neighbours finish in the same step. Each level above the first therefore
// runs one plane later: level l finishes plane q - (2l - 1) at step q, from the plane its level
// below finished (and published into the LDS seam table) one step earlier. Level 1 reads u0 from
// the window, which holds whole band rows, and finishes plane q - 1.
//
// Held cells: per-cell coefficient rows (x): c0 -> 1 and c1 = c2 = c3 -> 0, so A = 0 and B = the
// centre, and the cell keeps its value; rows y = 0 / ny-1 take that held coefficient set per row;
// planes gz = 0 / gnz-1 through a 0 / 1 factor on the A terms (u' = fma(z, A, S), S = fma(z, A, B)
// with B = the centre there). Those two run in a general copy of the plane step that only bands
// touching y = 0 / ny-1 take, and other bands only in the step pairs that touch the first / last
// global plane. (A held cell holding -0.0 comes back as +0.0, as in every fused kernel:
// 0 * t + (-0) rounds to +0.)
//
// Region contract (as box27_tb2): output storage planes [lz_begin, lz_end) (and optionally a second
// region [lz2_begin, lz2_end)) need u0 valid on [lz_begin - K, lz_end + K).
//
// Reference parity: the generation update MDF_kernel.cu:10-22 generalised to the 27-point weighted
// stencil of BASELINE.json config 4.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "kcommon.hpp"
#include "rowops.hpp"
#include "wxk_common.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int64_t resident_blocks(const void* kfn, int block);

// XW = 0: one wave per x segment, neighbouring segments overlapping by OV lanes (any row width).
// XW >= 1: the whole row in one block (nx <= XW * 64 * N): XW waves side by side in x with no
// overlap. The x neighbour of a wave's first / last cell comes from the LDS: level 1 reads it from
// the neighbour's window row, level l > 1 from an edge table in which every wave leaves the first
// and last cell of each row it finishes at levels 1..K-1 (written one step before it is read, like
// the y seams). A block is then XW x WB waves.
// CN = kRowOps2 (XW = 0 only): fp32 rows of 2 cells per lane (RowOps2f), half the registers per
// row, so a CU holds two 8-wave bands (rows of 1024 cells: 1641 vs 1582 GCells/s in 4-cell lanes,
// profiles/r06_session_n/). The window is then filled by 4-byte DMA halves (a segment's start is
// not 16-byte aligned), as heat7_wxk's narrow rows.
// Round 6 also measured (profiles/r06_session_{j,k,m}/): 2-cell lanes in whole-row blocks of 16 /
// 12 / 8 waves at 512-cell rows (1235 / 957 / 1129 vs 1379), 1-cell fp64 lanes (554-638 vs 692-830),
// a third window buffer with the DMA two planes ahead (-4.4 % fp32, -2.6 % fp64), level 1's x
// neighbours read from the window instead of lane shifts (10 % fewer VALU slots, -3 %): the march is
// set by the plane step's latency chain, not by occupancy, HBM latency or VALU count.
template <class T, int RY, int RE, int K, int WB, bool RES, int XW = 0, int CN = 0>
__global__ __launch_bounds__((XW > 0 ? XW : 1) * WB * 64) void box27_wxk(const T* __restrict__ in, T* __restrict__ out,
                                                                         Geo g, T c0, T c1, T c2, T c3, int zc, int XT,
                                                                         int YT, int ntasks, double* __restrict__ resid) {
  constexpr bool NAR = CN != 0;
  static_assert(CN != kRowOps2 || sizeof(T) == 4, "box27_wxk: 2-cell lanes are fp32");
  static_assert(CN != kRowOps1 || sizeof(T) == 8, "box27_wxk: 1-cell lanes are fp64");
  static_assert(CN == 0 || XW == 0, "box27_wxk: narrow rows in overlapping segments only");
  using RO = typename std::conditional<
      CN == kRowOps2, RowOps2f,
      typename std::conditional<CN == kRowOps1, RowOps1d,
                                typename std::conditional<sizeof(T) == 4, RowOpsN, RowOps<T>>::type>::type>::type;
  using V = typename std::conditional<NAR, typename RO::V, typename VT<T>::type>::type;
  using Row = typename RO::Row;
  constexpr int N = CN == kRowOps2 ? 2 : CN == kRowOps1 ? 1 : VT<T>::N;
  constexpr int XN = XW > 0 ? XW : 1;
  constexpr int OV = XW > 0 ? 0 : (K + N - 1) / N;
  constexpr int SEG = (64 - 2 * OV) * N;
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  constexpr int RB = BR + 2 * K;
  constexpr int RX = BR + 2 * (K - 1);  // band rows levels 1..K-1 finish: -(K-1) .. BR+K-2
  constexpr int NM = RY > RE + K - 1 ? RY : RE + K - 1;
  constexpr int LAG = 2 * K - 1;  // level K finishes plane q - LAG at step q
  static_assert(WB >= 2 && K >= 2, "box27_wxk: bands of at least two waves, at least two levels");
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int w = wid / XN, wx = wid % XN;  // y wave of the band, x wave of the row
  const int b = (int)xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntasks) return;
  __shared__ V win[2][XN][RB][64];
  __shared__ V seam[2][XN][K - 1][WB - 1][2][64];
  // x-edge table (XW >= 1) and the slots the other 62 lanes of an edge store write into
  constexpr int XE = XW > 0 ? 2 * (K - 1) * XN * RX * 2 : 1;
  __shared__ T xe[XE], xd[XW > 0 ? XE + 64 : 1];
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
  const int64_t x = XW > 0 ? (int64_t)(wx * 64 + lane) * N : (int64_t)xt * SEG - OV * N + (int64_t)lane * N;
  const int ny = (int)g.ny, lzmax = (int)g.lz_max, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  // bands tile the interior rows 1 .. ny-2; the held rows 0 / ny-1 a band does not reach are copied
  // from the window (their value never changes) by the band's edge wave next to them
  const int yb = 1 + yt * BR;
  const int y0 = yb + (w == 0 ? 0 : RE + (w - 1) * RY);
  const int rown = (w == 0 || w == WB - 1) ? RE : RY;
  const int64_t pitch = g.pitch, plane = g.plane;
  const bool xin = x >= 0 && x < pitch;
  const bool own = lane >= OV && lane <= 63 - OV && xin;
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e <= 0) || (x + e >= g.nx - 1);
  // per-cell coefficients: held x cells keep their centre (A = 0, B = centre)
  const Row k0 = RO::coefv(c0, T(1), xb), k1 = RO::coefv(c1, T(0), xb), k2 = RO::coefv(c2, T(0), xb),
            k3 = RO::coefv(c3, T(0), xb);
  // no row of the band (trapezoid included) at y = 0 / ny-1: the plane steps may skip the row tests
  const bool yint = yb - (K - 1) >= 1 && yb + BR + K - 2 <= ny - 2;
  const bool anyown = __builtin_amdgcn_ballot_w64(own) != 0;
  const int nsto = anyown ? max(0, min(rown, ny - y0)) : 0;
  const bool held0 = anyown && yt == 0 && w == 0;                   // row 0 = this wave's row -1
  const bool held1 = anyown && w == WB - 1 && yb + BR == ny - 1;  // row ny-1 = this wave's row RE
  int nst = 0;

  // byte offset of this lane's vector in x chunk kx (clamped into the row: finite values for the
  // held cells past the pitch)
  auto xcb_of = [&](int kx) -> uint32_t {
    const int64_t xx = XW > 0 ? (int64_t)(kx * 64 + lane) * N : x;
    return (uint32_t)((xx < 0 ? 0 : xx >= pitch ? pitch - N : xx) * (int64_t)sizeof(T));
  };
  const uint32_t xcb = xcb_of(0);
  // narrow rows: dword d = 64 h + lane of the segment's row (heat7_wxk's layout)
  constexpr int DPC = (int)sizeof(T) / 4;
  uint32_t xch[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int d = h * 64 + lane;
    const int64_t xh = (int64_t)xt * SEG - OV * N + d / DPC;
    xch[h] = (uint32_t)(((xh < 0 ? 0 : xh >= pitch ? pitch - 1 : xh) * DPC + d % DPC) * 4);
  }
  // u0 plane lz -> window buffer `buf`. Buffer-descriptor DMAs on the wave-uniform row base (blds16 /
  // blds4): with a global_load_lds in flight hipcc made every LDS read of the plane step wait for
  // all of them (lgkmcnt(0)) before the first use; with these the waits are partial, so level K starts
  // on its seam rows while level 1's window rows are still arriving (512^3 fp32 1440 vs 1402, fp64
  // 735 vs 696 GCells/s with the read order and level barriers below, profiles/r06_session_n/)
  auto issue = [&](int lz, int buf) {
    const int lzc = lz < 0 ? 0 : lz >= lzmax ? lzmax - 1 : lz;
    constexpr int NW = XN * WB, NR = XN * RB;
#pragma unroll
    for (int j = 0; j < (NR + NW - 1) / NW; ++j) {
      const int k = wid + j * NW;
      if (k < NR) {
        const int kx = k / RB, kr = k - kx * RB;
        const int y = yb - K + kr;
        const int yc = y < 0 ? 0 : y >= ny ? ny - 1 : y;
        uint64_t rb = (uint64_t)(uintptr_t)(in + (int64_t)lzc * plane + (int64_t)yc * pitch);
        asm volatile("" : "+s"(rb));
        const __amdgpu_buffer_rsrc_t rs = row_rsrc((const void*)(uintptr_t)rb);
        if constexpr (NAR) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + (xch[h] & ~(uint32_t)(sizeof(T) - 1))), 1);
            blds4(rs, xch[h], (char*)&win[buf][kx][kr][0] + h * 256);
          }
        } else {
          const uint32_t o = XW > 1 ? xcb_of(kx) : xcb;
          dcheck(g, in, (const T*)((const char*)(uintptr_t)rb + o), N);
          blds16(rs, o, &win[buf][kx][kr][0]);
        }
      }
    }
  };

  const int qdma = ze - 1 + K;    // last u0 plane any valid output needs
  const int qend = ze - 1 + LAG;  // the step that finishes the chunk's last output plane
  issue(zs - K, 0);
  T* ob = out + (int64_t)y0 * pitch;
  const uint32_t xob = (uint32_t)((xin ? x : 0) * (int64_t)sizeof(T));
  double acc = 0.0;
  typedef __attribute__((address_space(3))) V LV;
  typedef __attribute__((address_space(3))) T LT;
  LV* const wrow = lds_vptr(&win[0][wx][y0 - yb][lane]);
  const int wu = w > 0 ? w - 1 : 0, wd = w < WB - 1 ? w : WB - 2;
  LV* const s_first = lds_vptr(&seam[0][wx][0][wu][0][lane]);
  LV* const s_last = lds_vptr(&seam[0][wx][0][wd][1][lane]);
  // the neighbours' rows this wave reads (through laundered pointers: indexed with the runtime x
  // wave, the direct seam reads made hipcc drain the window DMA just issued, vmcnt(0), every step)
  LV* const s_rdu = lds_vptr(&seam[0][wx][0][wu][1][lane]);
  LV* const s_rdd = lds_vptr(&seam[0][wx][0][wd][0][lane]);
  constexpr int WIN_BUF = XN * RB * 64;
  constexpr int SEAM_PAR = XN * (K - 1) * (WB - 1) * 2 * 64, SEAM_LVL = (WB - 1) * 2 * 64;
  // x edges (XW >= 1). Lane 0 takes its left neighbour's last cell, lane 63 its right neighbour's
  // first; at the row's ends (held cells, the value only meets a zero coefficient) a lane reads a
  // finite cell of its own wave instead. Window: row r of buffer P at e_win[(P * WIN_BUF + r * 64) * N]
  // with r = y0 - yb + i + K; table: [P][level][x wave][i + K - 1][side] from this wave's row i.
  const int wl = wx > 0 ? wx - 1 : 0, wr = wx < XN - 1 ? wx + 1 : XN - 1;
  auto cell = [](V* v, int e) -> T* { return (T*)v + e; };
  LT* const e_win = lds_vptr(lane == 63 ? (wx < XN - 1 ? cell(&win[0][wx + 1][y0 - yb][0], 0) : cell(&win[0][wx][y0 - yb][63], N - 1))
                                        : (wx > 0 ? cell(&win[0][wx - 1][y0 - yb][63], N - 1) : cell(&win[0][wx][y0 - yb][0], 0)));
  constexpr int XE_PAR = (K - 1) * XN * RX * 2, XE_LVL = XN * RX * 2;
  const int xrow0 = (y0 - yb) * 2;  // row i = -(K-1) of this wave in the table
  LT* const e_tab = lds_vptr(lane == 63 ? &xe[(wr * RX) * 2 + xrow0 + (wx < XN - 1 ? 0 : 1)]
                                        : &xe[(wl * RX) * 2 + xrow0 + (wx > 0 ? 1 : 0)]);
  LT* const e_put = lds_vptr(lane == 0 ? &xe[(wx * RX) * 2 + xrow0] : lane == 63 ? &xe[(wx * RX) * 2 + xrow0 + 1] : &xd[lane]);
  auto st = [](LV* p, const V& v) {
    if constexpr (sizeof(V) == 16)
      asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
    else
      asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };
  auto st1 = [](LT* p, T v) {
    if constexpr (sizeof(T) == 4)
      asm volatile("ds_write_b32 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
    else
      asm volatile("ds_write_b64 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };
  auto hs = [](const Row& v) -> Row { return RO::hsum(v, lane_up1(RO::last(v)), lane_down1(RO::first(v))); };
  auto hsx = [](const Row& v, T e) -> Row {
    return RO::hsum(v, lane_up1_or(e, RO::last(v)), lane_down1_or(e, RO::first(v)));
  };

  auto march = [&](auto role_c, auto ygen_c) __attribute__((always_inline)) {
    constexpr int ROLE = decltype(role_c)::value;
    constexpr bool YGEN = decltype(ygen_c)::value;  // the band has rows at y = 0 / ny-1
    using SH = WxRows<ROLE, RY, RE, K>;
    // per level l (index l-1): running sums S, the last two A (ping-pong), and for l < K the two
    // stored output planes H (ping-pong) the level above reads
    Row S[K][NM], Ap[K][2][NM], H[K - 1][2][NM];
#pragma unroll
    for (int l = 0; l < K; ++l)
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        S[l][i] = Ap[l][0][i] = Ap[l][1][i] = RO::zero();
        if (l < K - 1) H[l][0][i] = H[l][1][i] = RO::zero();
      }
    auto step = [&](int q, auto par_c, auto gen_c) __attribute__((always_inline)) {
      constexpr bool GEN = decltype(gen_c)::value;  // held rows / planes may occur in this step
      constexpr int P = decltype(par_c)::value;
      __builtin_amdgcn_sched_barrier(0);
      wait_vm_le(nst);
      lds_barrier();
      if (q < qdma) issue(q + 1, P ^ 1);
      constexpr int WO = P * WIN_BUF;
      const int lzo = q - LAG;  // level K's output plane
      const bool valid = lzo >= zs && lzo < ze;
      // the step's LDS rows (every upper level's two seam rows and x edges, level 1's u0 window rows)
      // are read up front, so the reads overlap each other instead of each waiting out a round trip
      // right before its use (round 5: 512^3 fp64 678 vs 640 GCells/s, profiles/r05_session_a/), in
      // the order the levels use them (top-down): the waits before each level are partial
      constexpr int NU = SH::n(1) + 2;
      Row U[NU], SU[K], SD[K];
      T E1[NU], EX[K][NM + 2];
#pragma unroll
      for (int j = K - 1; j >= 1; --j) {
        // level j's two seam rows (the neighbour waves' rows level j + 1 reads) and, XW > 1, the x
        // edges of level j + 1's input rows from the table level j filled in the previous step
        SU[j] = SD[j] = RO::zero();
        if (SH::lo(j + 1) - 1 < SH::lo(j)) SU[j] = RO::fromv(V(s_rdu[(P ^ 1) * SEAM_PAR + (j - 1) * SEAM_LVL]));
        if (SH::hi(j + 1) >= SH::hi(j)) SD[j] = RO::fromv(V(s_rdd[(P ^ 1) * SEAM_PAR + (j - 1) * SEAM_LVL]));
        if constexpr (XW > 1) {
#pragma unroll
          for (int k = 0; k < SH::n(j + 1) + 2; ++k)
            EX[j][k] = e_tab[(P ^ 1) * XE_PAR + (j - 1) * XE_LVL + (SH::lo(j + 1) - 1 + k + K - 1) * 2];
        }
      }
#pragma unroll
      for (int k = 0; k < NU; ++k) U[k] = RO::fromv(V(wrow[WO + (SH::lo(1) - 1 + k + K) * 64]));
      if constexpr (XW > 1) {
#pragma unroll
        for (int k = 0; k < NU; ++k) E1[k] = e_win[(WO + (SH::lo(1) - 1 + k + K) * 64) * N];
      }
      // levels top-down: level l reads its inputs (the level below's plane from the previous step)
      // before that level overwrites its other stored plane
#pragma unroll
      for (int l = K; l >= 1; --l) {
        // no level's arithmetic moves ahead of the level above (it would pull that level's waits
        // for the later LDS reads forward)
        if (l < K) __builtin_amdgcn_sched_barrier(0);
        const int m = q - (2 * l - 1);  // output plane of level l; its inputs are plane p = m + 1
        T zm = T(1), zp = T(1);
        bool zhp = false;
        if (GEN) {
          const int gm = m + gzoff, gp = m + 1 + gzoff;
          zm = (gm <= 0 || gm >= gnz - 1) ? T(0) : T(1);
          zhp = gp <= 0 || gp >= gnz - 1;
          zp = zhp ? T(0) : T(1);
        }
        // input rows of level l-1 at plane p: rows lo(l)-1 .. hi(l)
        auto vin = [&](int i) -> Row {
          if (l == 1) return U[i - (SH::lo(1) - 1)];
          const int j = l - 1;
          if (i < SH::lo(j)) return SU[j];
          if (i >= SH::hi(j)) return SD[j];
          return H[j - 1][P ^ 1][i - SH::lo(j)];
        };
        auto hsi = [&](const Row& v, int i) -> Row {
          if constexpr (XW > 1) return hsx(v, l == 1 ? E1[i - (SH::lo(1) - 1)] : EX[l - 1][i - (SH::lo(l) - 1)]);
          else return hs(v);
        };
        Row vm = vin(SH::lo(l) - 1), vc = vin(SH::lo(l));
        Row hm = hsi(vm, SH::lo(l) - 1), hc = hsi(vc, SH::lo(l));
#pragma unroll
        for (int i = SH::lo(l); i < SH::hi(l); ++i) {
          const int il = i - SH::lo(l);
          const Row vp = vin(i + 1);
          const Row hp = hsi(vp, i + 1);
          const Row cross = RO::add(hc, RO::add(vm, vp));
          const Row diag = RO::add(hm, hp);
          Row a, bb;
          const bool yh = GEN && (y0 + i == 0 || y0 + i == ny - 1);
          if (yh) {
            a = RO::zero();
            bb = vc;
          } else {
            a = RO::lin3r(vc, cross, diag, k1, k2, k3);   // sm::box27_A
            bb = RO::lin3r(vc, cross, diag, k0, k1, k2);  // sm::box27_B
          }
          if (GEN && zhp) bb = vc;
          // u_l(m) = (A(m-1) + B(m)) + A(m+1), then S(p) = A(m) + B(p)
          const Row o = GEN ? RO::fmaz(zm, a, S[l - 1][il]) : RO::add(S[l - 1][il], a);
          S[l - 1][il] = GEN ? RO::fmaz(zp, Ap[l - 1][P ^ 1][il], bb) : RO::add(Ap[l - 1][P ^ 1][il], bb);
          Ap[l - 1][P][il] = a;
          if (l == K) {
            if (valid && i >= 0 && i < SH::R && y0 + i < ny && own) {
              T* ad = (T*)((char*)(ob + (int64_t)lzo * plane + (int64_t)i * pitch) + xob);
              dcheck(g, (const T*)out, ad, N);
              store_nt((V*)ad, RO::vec(o));
              if (RES) {
                const Row& cen = H[K - 2][P][i - SH::lo(K - 1)];  // u_{K-1}(m): still the stored plane m
#pragma unroll
                for (int e = 0; e < N; ++e)
                  if (x + e < g.nx) {
                    const double d = (double)RO::get(o, e) - (double)RO::get(cen, e);
                    acc += d * d;
                  }
              }
            }
          } else {
            H[l - 1][P][il] = o;
            if (ROLE != 0 && i == 0) st(s_first + P * SEAM_PAR + (l - 1) * SEAM_LVL, RO::vec(o));
            if (ROLE != 2 && i == SH::R - 1) st(s_last + P * SEAM_PAR + (l - 1) * SEAM_LVL, RO::vec(o));
            if constexpr (XW > 1)
              st1(e_put + P * XE_PAR + (l - 1) * XE_LVL + (i + K - 1) * 2, lane == 63 ? RO::last(o) : RO::first(o));
          }
          vm = vc;
          vc = vp;
          hm = hc;
          hc = hp;
        }
      }
      nst = valid ? nsto : 0;
      if constexpr (GEN && ROLE != 1) {
        if ((ROLE == 0 ? held0 : held1) && q >= zs && q < ze) {  // u0 plane q is output plane q there
          constexpr int ih = ROLE == 0 ? -1 : SH::R;
          if (own) {
            T* ad = (T*)((char*)(ob + (int64_t)q * plane + (int64_t)ih * pitch) + xob);
            dcheck(g, (const T*)out, ad, N);
            store_nt((V*)ad, RO::vec(U[ih - (SH::lo(1) - 1)]));
          }
          ++nst;
        }
      }
    };
    // in a y-interior band, the step pairs whose levels all finish and read z-interior planes take
    // the copy without the held-row / held-plane tests (at 512^3 two of the three z chunks touch a
    // global boundary plane, but only in their first or last 2K - 1 steps)
    using Tr = std::true_type;
    using F = std::false_type;
    int q = zs - K;
    if constexpr (!YGEN) {
      auto zfree = [&](int qq) { return qq - LAG + gzoff >= 1 && qq + 1 + gzoff <= gnz - 2; };  // qq and qq + 1
      for (; q <= qend && !zfree(q); q += 2) {
        step(q, IC<0>{}, Tr{});
        step(q + 1, IC<1>{}, Tr{});
      }
      for (; q <= qend && zfree(q); q += 2) {
        step(q, IC<0>{}, F{});
        step(q + 1, IC<1>{}, F{});
      }
    }
    for (; q <= qend; q += 2) {
      step(q, IC<0>{}, Tr{});
      step(q + 1, IC<1>{}, Tr{});
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
  wait_vm0();
  if (RES) wave_atomic_add(resid, acc);
}

// (Round 3 also had an x-pair variant for rows of 257..512 cells, box27_wxp: two 256-cell halves
// side by side in one block with an LDS table of edge cells instead of overlapping lanes. Its
// 6-row bands fetched twice the window rows per output row and it ran 909 vs 1017-1026 GCells/s
// at 512^3 (profiles/archive/r03_session_t/); removed in round 4.)

template <class T, int RY, int RE, int K, int WB, int XW = 0, int CN = 0>
static void launch_b27x(const Geo& g, const T* in, T* out, const StencilCoef& cf, double* resid, hipStream_t s) {
  constexpr int N = CN == kRowOps2 ? 2 : CN == kRowOps1 ? 1 : VT<T>::N, OV = XW > 0 ? 0 : (K + N - 1) / N, SEG = (64 - 2 * OV) * N;
  constexpr int BR = 2 * RE + (WB - 2) * RY, NT = 64 * WB * (XW > 0 ? XW : 1);
  if (XW > 0) MDFX_CHECK(g.nx <= XW * 64 * N, "box27_wxk: whole-row blocks need nx <= XW * 64 * N");
  const int64_t planes = g.lz_end - g.lz_begin;
  const int64_t planes2 = g.lz2_end > g.lz2_begin ? g.lz2_end - g.lz2_begin : 0;
  const int XT = XW > 0 ? 1 : (int)((g.nx + SEG - 1) / SEG);
  const int YT = (int)std::max<int64_t>(1, (g.ny - 2 + BR - 1) / BR);  // bands over rows 1 .. ny-2
  const int64_t tiles = (int64_t)XT * YT;
  const void* kfn = (const void*)&box27_wxk<T, RY, RE, K, WB, false, XW, CN>;
  const int64_t resident = resident_blocks(kfn, NT);
  int zc = wx_zc(planes, tiles, resident, K, 3 * K - 1, g.min_rounds);
  if (planes2 > 0) zc = (int)std::max(planes, planes2);
  const int ZT = (int)((planes + zc - 1) / zc) + (planes2 > 0 ? (int)((planes2 + zc - 1) / zc) : 0);
  const int64_t ntasks = tiles * ZT;
  MDFX_CHECK(ntasks < (int64_t)1 << 31, "box27_wxk: too many tasks");
  const dim3 grd((unsigned)ntasks), blk(NT);
  const T c0 = (T)cf.c0, c1 = (T)cf.c1, c2 = (T)cf.c2, c3 = (T)cf.c3;
  if (resid)
    hipLaunchKernelGGL((box27_wxk<T, RY, RE, K, WB, true, XW, CN>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, XT, YT,
                       (int)ntasks, resid);
  else
    hipLaunchKernelGGL((box27_wxk<T, RY, RE, K, WB, false, XW, CN>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, XT,
                       YT, (int)ntasks, resid);
}

template <class T>
void launch_box27_wxk(const Geo& g, const T* in, T* out, const StencilCoef& cf, int steps, double* resid,
                      hipStream_t s) {
  if (g.lz_end <= g.lz_begin) return;
  MDFX_CHECK(steps == 3 && g.lz_begin >= steps && g.lz_end + steps <= g.lz_max,
             format("box27_wxk: %d fused steps need %d valid planes around [%lld, %lld) of %lld", steps, steps,
                    (long long)g.lz_begin, (long long)g.lz_end, (long long)g.lz_max));
  MDFX_CHECK(g.lz2_end <= g.lz2_begin || (g.lz2_begin >= g.lz_end && g.lz2_end + steps <= g.lz_max),
             "box27_wxk: the second region must follow the first and have its planes + ghosts allocated");
  MDFX_CHECK(g.pitch % VT<T>::N == 0, "box27_wxk: the row pitch must be a whole number of vectors");
  MDFX_CHECK(g.ny < ((int64_t)1 << 30) && g.lz_max < ((int64_t)1 << 30) && g.gnz < ((int64_t)1 << 30) &&
                 g.gz_off > -((int64_t)1 << 30) && g.gz_off < ((int64_t)1 << 30),
             "box27_wxk: row / plane counts must fit 32-bit indices");
  // 2-row inner waves, 1-row edge waves, bands of 8 (14 rows): the 3-row shapes need more than
  // 256 VGPRs; 1-row waves in bands of 8 and 2-row waves in bands of 4 measured slower at 512^3
  // (fp64 500 / 603 vs 640 GCells/s, fp32 845 / 957 vs 1007: profiles/r04_session_n/)
  // fp32 rows of at most 512 cells: whole-row blocks of 2 x 4 waves with the x edges exchanged through
  // the LDS (no lane of a 512-cell row computed twice; bands over rows 1..ny-2 fill 255 blocks in
  // three z chunks): 512^3 1332 GCells/s against 1009 in three overlapping segments and 1092 for
  // box27_tb2n K = 2 (profiles/r05_session_f/)
  if constexpr (std::is_same<T, float>::value) {
    // (2-cell lanes in 5 overlapping segments at 512-cell rows: 1262-1266 vs 1397-1401 GCells/s,
    // profiles/r06_session_q/)
    if (g.nx <= 512) return launch_b27x<T, 2, 1, 3, 4, 2>(g, in, out, cf, resid, s);
    return launch_b27x<T, 2, 1, 3, 8, 0, kRowOps2>(g, in, out, cf, resid, s);
  } else {
    // (fp64 at 512-cell rows fills only 185 of 256 CUs in one round (5 segments x 37 bands); round 6
    // measured the shapes that fill more: 6-wave bands of 10 rows (255 tiles) 570-575, 1-row waves
    // in 8-row bands 559-563, 4-wave bands in 2 blocks per CU (425 tiles) 659-683, against 705-707
    // GCells/s for these 14-row bands: the march is latency-bound per wave, so more waves per tile
    // pay, more tiles do not (profiles/r06_session_h/))
    launch_b27x<T, 2, 1, 3, 8>(g, in, out, cf, resid, s);
  }
}
template void launch_box27_wxk<float>(const Geo&, const float*, float*, const StencilCoef&, int, double*, hipStream_t);
template void launch_box27_wxk<double>(const Geo&, const double*, double*, const StencilCoef&, int, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
