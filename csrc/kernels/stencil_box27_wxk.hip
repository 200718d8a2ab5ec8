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
// with B = the centre there). Those two run in a general copy of the march that only bands touching
// y = 0 / ny-1 and chunks touching the first / last global plane take. (A held cell holding -0.0
// comes back as +0.0, as in every fused kernel: 0 * t + (-0) rounds to +0.)
//
// Region contract (as box27_tb2): output storage planes [lz_begin, lz_end) (and optionally a second
// region [lz2_begin, lz2_end)) need u0 valid on [lz_begin - K, lz_end + K).
//
// Reference parity: the generation update MDF_kernel.cu:10-22 generalised to the 27-point weighted
// stencil of BASELINE.json config 4.
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

template <class T, int RY, int RE, int K, int WB, bool RES>
__global__ __launch_bounds__(WB * 64) void box27_wxk(const T* __restrict__ in, T* __restrict__ out, Geo g, T c0, T c1,
                                                     T c2, T c3, int zc, int XT, int YT, int ntasks,
                                                     double* __restrict__ resid) {
  using V = typename VT<T>::type;
  using RO = typename std::conditional<sizeof(T) == 4, RowOpsN, RowOps<T>>::type;
  using Row = typename RO::Row;
  constexpr int N = VT<T>::N;
  constexpr int OV = (K + N - 1) / N;
  constexpr int SEG = (64 - 2 * OV) * N;
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  constexpr int RB = BR + 2 * K;
  constexpr int NM = RY > RE + K - 1 ? RY : RE + K - 1;
  constexpr int LAG = 2 * K - 1;  // level K finishes plane q - LAG at step q
  static_assert(WB >= 2 && K >= 2, "box27_wxk: bands of at least two waves, at least two levels");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = (int)xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntasks) return;
  __shared__ V win[2][RB][64];
  __shared__ V seam[2][K - 1][WB - 1][2][64];
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
  const int64_t x = (int64_t)xt * SEG - OV * N + (int64_t)lane * N;
  const int ny = (int)g.ny, lzmax = (int)g.lz_max, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  const int yb = yt * BR;
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
  // the fast march: no band row at y = 0 / ny-1 and no global boundary plane anywhere in the chunk
  const bool yint = yb - (K - 1) >= 1 && yb + BR + K - 2 <= ny - 2;
  const bool zint = zs - K + gzoff >= 1 && ze + K - 1 + gzoff <= gnz - 2;
  const int nsto = __builtin_amdgcn_ballot_w64(own) != 0 ? max(0, min(rown, ny - y0)) : 0;
  int nst = 0;

  const uint32_t xcb = (uint32_t)((x < 0 ? 0 : x >= pitch ? pitch - N : x) * (int64_t)sizeof(T));
  auto issue = [&](int lz, int buf) {
    const int lzc = lz < 0 ? 0 : lz >= lzmax ? lzmax - 1 : lz;
#pragma unroll
    for (int j = 0; j < (RB + WB - 1) / WB; ++j) {
      const int k = w + j * WB;
      if (k < RB) {
        const int y = yb - K + k;
        const int yc = y < 0 ? 0 : y >= ny ? ny - 1 : y;
        const T* a = (const T*)((const char*)(in + (int64_t)lzc * plane + (int64_t)yc * pitch) + xcb);
        dcheck(g, in, a, N);
        glds16(a, &win[buf][k][0]);
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
  LV* const wrow = lds_vptr(&win[0][y0 - yb][lane]);
  const int wu = w > 0 ? w - 1 : 0, wd = w < WB - 1 ? w : WB - 2;
  LV* const s_first = lds_vptr(&seam[0][0][wu][0][lane]);
  LV* const s_last = lds_vptr(&seam[0][0][wd][1][lane]);
  constexpr int WIN_BUF = RB * 64;
  constexpr int SEAM_PAR = (K - 1) * (WB - 1) * 2 * 64, SEAM_LVL = (WB - 1) * 2 * 64;
  auto st = [](LV* p, const V& v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };
  auto hs = [](const Row& v) -> Row { return RO::hsum(v, lane_up1(RO::last(v)), lane_down1(RO::first(v))); };

  auto march = [&](auto role_c, auto gen_c) __attribute__((always_inline)) {
    constexpr int ROLE = decltype(role_c)::value;
    constexpr bool GEN = decltype(gen_c)::value;  // held rows / planes may occur
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
    auto step = [&](int q, auto par_c) __attribute__((always_inline)) {
      constexpr int P = decltype(par_c)::value;
      __builtin_amdgcn_sched_barrier(0);
      wait_vm_le(nst);
      lds_barrier();
      if (q < qdma) issue(q + 1, P ^ 1);
      const int lzo = q - LAG;  // level K's output plane
      const bool valid = lzo >= zs && lzo < ze;
      // levels top-down: level l reads its inputs (the level below's plane from the previous step)
      // before that level overwrites its other stored plane
#pragma unroll
      for (int l = K; l >= 1; --l) {
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
          if (l == 1) return RO::fromv(V(wrow[P * WIN_BUF + (i + K) * 64]));
          const int j = l - 1;
          if (i < SH::lo(j)) return RO::fromv(seam[P ^ 1][j - 1][wu][1][lane]);
          if (i >= SH::hi(j)) return RO::fromv(seam[P ^ 1][j - 1][wd][0][lane]);
          return H[j - 1][P ^ 1][i - SH::lo(j)];
        };
        Row vm = vin(SH::lo(l) - 1), vc = vin(SH::lo(l));
        Row hm = hs(vm), hc = hs(vc);
#pragma unroll
        for (int i = SH::lo(l); i < SH::hi(l); ++i) {
          const int il = i - SH::lo(l);
          const Row vp = vin(i + 1);
          const Row hp = hs(vp);
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
          }
          vm = vc;
          vc = vp;
          hm = hc;
          hc = hp;
        }
      }
      nst = valid ? nsto : 0;
    };
    for (int q = zs - K; q <= qend; q += 2) {
      step(q, IC<0>{});
      step(q + 1, IC<1>{});
    }
  };
  const bool fast = yint && zint;
  if (w == 0) {
    if (fast) march(IC<0>{}, std::false_type{});
    else march(IC<0>{}, std::true_type{});
  } else if (w == WB - 1) {
    if (fast) march(IC<2>{}, std::false_type{});
    else march(IC<2>{}, std::true_type{});
  } else {
    if (fast) march(IC<1>{}, std::false_type{});
    else march(IC<1>{}, std::true_type{});
  }
  wait_vm0();
  if (RES) wave_atomic_add(resid, acc);
}

// x-pair variant for rows of 257..512 cells (box27_wxp): the row is split into two halves of 256
// cells (64 lanes x 4) that sit side by side in one block, 2 x WB waves, with no overlapping lanes.
// box27_wxk's overlapping x segments cover a 512-cell row with 3 segments of 248 owned cells, so a
// third of its lanes compute nothing that is kept; here every lane's cells are its own. The cells
// just beyond a half's edge (x = 255 for the right half's lane 0, x = 256 for the left half's lane
// 63) come from the other half: for level 1 straight from the shared u0 window (it holds both
// halves), for the levels above from a small LDS table of edge cells that every wave publishes for
// each row it computes (parity q & 1, read after the next plane's barrier, like the y seams). The
// y seams are kept per half. Everything else -- the level schedule (level l one plane later than
// level l-1), the held-cell coefficients, the band roles -- is box27_wxk's, so the result is
// bitwise that of K box27_zw steps.
template <class T, int RY, int RE, int K, int WB, bool RES>
__global__ __launch_bounds__(2 * WB * 64) void box27_wxp(const T* __restrict__ in, T* __restrict__ out, Geo g, T c0,
                                                         T c1, T c2, T c3, int zc, int YT, int ntasks,
                                                         double* __restrict__ resid) {
  static_assert(sizeof(T) == 4, "box27_wxp: fp32 rows (64 lanes x 4 cells = 256 per half)");
  using V = typename VT<T>::type;
  using RO = RowOpsN;
  using Row = typename RO::Row;
  constexpr int N = 4;
  constexpr int HX = 64 * N;  // cells per half
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  constexpr int RB = BR + 2 * K;
  constexpr int NM = RY > RE + K - 1 ? RY : RE + K - 1;
  constexpr int LAG = 2 * K - 1;
  constexpr int NW = 2 * WB;
  static_assert(WB >= 2 && K >= 2, "box27_wxp: bands of at least two waves, at least two levels");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int xh = w / WB, wy = w % WB;  // x half, wave of the band
  const int b = (int)xcd_remap(blockIdx.x, gridDim.x);
  if (b >= ntasks) return;
  __shared__ V win[2][RB][2][64];
  // [half][parity][level-1][boundary][first of s+1 / last of s][lane]: the half outermost (with it
  // inside, hipcc loses track of which LDS array a seam read touches and drains the window's
  // in-flight DMA with vmcnt(0) before it)
  __shared__ V seam[2][2][K - 1][WB - 1][2][64];
  // x edge rows: the left half publishes the LAST cell of every lane of each row it computes, the
  // right half the FIRST (whole rows of floats: one non-divergent ds_write_b32; the other half reads
  // lane 63's / lane 0's entry)
  __shared__ T xs[2][K - 1][RB][2][64];           // [parity][level-1][window row][half][lane]
  const int zt = b / YT, yt = b % YT;
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
  const int x = xh * HX + lane * N;
  const int ny = (int)g.ny, lzmax = (int)g.lz_max, gzoff = (int)g.gz_off, gnz = (int)g.gnz;
  const int yb = yt * BR;
  const int y0 = yb + (wy == 0 ? 0 : RE + (wy - 1) * RY);
  const int rown = (wy == 0 || wy == WB - 1) ? RE : RY;
  const int64_t pitch = g.pitch, plane = g.plane;
  const bool own = x < pitch;
  bool xb[N];
#pragma unroll
  for (int e = 0; e < N; ++e) xb[e] = (x + e <= 0) || (x + e >= g.nx - 1);
  const Row k0 = RO::coefv(c0, T(1), xb), k1 = RO::coefv(c1, T(0), xb), k2 = RO::coefv(c2, T(0), xb),
            k3 = RO::coefv(c3, T(0), xb);
  const bool yint = yb - (K - 1) >= 1 && yb + BR + K - 2 <= ny - 2;
  const bool zint = zs - K + gzoff >= 1 && ze + K - 1 + gzoff <= gnz - 2;
  const int nsto = __builtin_amdgcn_ballot_w64(own) != 0 ? max(0, min(rown, ny - y0)) : 0;
  int nst = 0;

  // u0 plane lz -> window buffer `buf`: 2 RB half rows of 64 lanes, wave w fetching w, w + 2WB, ..
  // (always half w & 1: 2WB is even). The lane's byte offset in the row stays in one VGPR for the
  // whole march, so the DMA takes the SGPR-base form and no address register is ever recycled
  // under an in-flight DMA (a recycled one makes hipcc drain it with vmcnt(0)).
  const uint32_t xcb = (uint32_t)(std::min<int64_t>((int64_t)(w & 1) * HX + lane * N, pitch - N) * (int64_t)sizeof(T));
  auto issue = [&](int lz, int buf) {
    const int lzc = lz < 0 ? 0 : lz >= lzmax ? lzmax - 1 : lz;
#pragma unroll
    for (int j = 0; j < (2 * RB + NW - 1) / NW; ++j) {
      const int k = w + j * NW;
      if (k < 2 * RB) {
        const int r = k >> 1, h = k & 1;
        const int y = yb - K + r;
        const int yc = y < 0 ? 0 : y >= ny ? ny - 1 : y;
        // the row base is laundered through SGPRs so hipcc cannot hoist `in + xcb` into a 64-bit
        // VGPR pair: the DMA keeps the SGPR-base form with xcb's own long-lived VGPR
        const char* rb = (const char*)(in + (int64_t)lzc * plane + (int64_t)yc * pitch);
        asm volatile("" : "+s"(rb));
        const T* a = (const T*)(rb + xcb);
        dcheck(g, in, a, N);
        glds16(a, &win[buf][r][h][0]);
      }
    }
  };

  const int qdma = ze - 1 + K;
  const int qend = ze - 1 + LAG;
  issue(zs - K, 0);
  T* ob = out + (int64_t)y0 * pitch + x;
  double acc = 0.0;
  typedef __attribute__((address_space(3))) V LV;
  typedef __attribute__((address_space(3))) T LT;
  LV* const wrow = lds_vptr(&win[0][y0 - yb][xh][lane]);
  // the other half's edge cell of u0 window row r (lane 0 of the right half needs x = 255, lane 63
  // of the left half x = 256); the outer ends (x = -1, x = 512) feed held cells only: 0
  const int wu = wy > 0 ? wy - 1 : 0, wd = wy < WB - 1 ? wy : WB - 2;
  LV* const s_first = lds_vptr(&seam[xh][0][0][wu][0][lane]);
  LV* const s_last = lds_vptr(&seam[xh][0][0][wd][1][lane]);
  constexpr int WIN_BUF = RB * 2 * 64, WROW = 2 * 64;           // V elements
  constexpr int SEAM_PAR = (K - 1) * (WB - 1) * 2 * 64, SEAM_LVL = (WB - 1) * 2 * 64;
  constexpr int XS_PAR = (K - 1) * RB * 2 * 64, XS_LVL = RB * 2 * 64;
  // this wave's edge-cell slots: lane 0 publishes its first cell, lane 63 its last
  LT* const xs_mine = lds_vptr(&xs[0][0][y0 - yb + K][xh][lane]);
  // LDS byte addresses of the other half's edge cells: of u0 window row r (buffer 0) and of edge
  // row r (parity 0, level 1); buffers / parities / levels are fixed strides from there
  const uint32_t a_win = (uint32_t)(uintptr_t)(LT*)(xh == 1 ? &((T*)&win[0][0][0][63])[3] : &((T*)&win[0][0][1][0])[0]);
  const uint32_t a_xs = (uint32_t)(uintptr_t)(LT*)(xh == 1 ? &xs[0][0][0][0][63] : &xs[0][0][0][1][0]);
  constexpr uint32_t WIN_ROW_B = 2 * 64 * sizeof(V), WIN_BUF_B = RB * WIN_ROW_B;
  constexpr uint32_t XS_ROW_B = 2 * 64 * sizeof(T), XS_LVL_B = RB * XS_ROW_B, XS_PAR_B = (K - 1) * XS_LVL_B;
  auto st = [](LV* p, const V& v) {
    asm volatile("ds_write_b128 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };
  auto st1 = [](LT* p, T v) {
    asm volatile("ds_write_b32 %0, %1" ::"v"((unsigned)(uintptr_t)p), "v"(v) : "memory");
  };
  // x sums of a row whose cells beyond the half's ends are `eo` (the other half's edge cell)
  // (both shifts always take the edge operand -- the outer ends x = -1 / 512 only ever feed held
  // cells -- so the half's choice is a select of the operand, not a branch around the shift)
  const bool right = xh == 1;
  auto hs = [&](const Row& v, T eo) -> Row {
    const T l = lane_up1_or(right ? eo : T(0), RO::last(v));
    const T r = lane_down1_or(right ? T(0) : eo, RO::first(v));
    return RO::hsum(v, l, r);
  };

  auto march = [&](auto role_c, auto gen_c) __attribute__((always_inline)) {
    constexpr int ROLE = decltype(role_c)::value;
    constexpr bool GEN = decltype(gen_c)::value;
    using SH = WxRows<ROLE, RY, RE, K>;
    Row S[K][NM], Ap[K][2][NM], H[K - 1][2][NM];
#pragma unroll
    for (int l = 0; l < K; ++l)
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        S[l][i] = Ap[l][0][i] = Ap[l][1][i] = RO::zero();
        if (l < K - 1) H[l][0][i] = H[l][1][i] = RO::zero();
      }
    // The other half's edge cells a step uses: for level l, input rows lo(l)-1 .. hi(l) (level 1 from
    // the u0 window of this step's plane, levels above from the edge rows of the previous step).
    // Entry e of that list is fetched by lane e with ONE ds_read_b32 right after the plane's barrier
    // and handed to the row code by readlane: one LDS round trip per step instead of one per row.
    constexpr auto eidx = [](int l, int i) constexpr {  // entry of (level l, row i)
      int e = 0;
      for (int ll = K; ll > l; --ll) e += SH::n(ll) + 2;
      return e + (i - (SH::lo(l) - 1));
    };
    static_assert(eidx(1, SH::hi(1)) < 64, "box27_wxp: one lane per edge cell");
    uint32_t ea[2] = {a_win, a_win};  // per-lane address of entry `lane`, per parity
#pragma unroll
    for (int l = K; l >= 1; --l)
#pragma unroll
      for (int i = SH::lo(l) - 1; i <= SH::hi(l); ++i) {
        const uint32_t r = (uint32_t)(y0 - yb + K + i);  // window / edge row
        if (lane == eidx(l, i)) {
#pragma unroll
          for (int p = 0; p < 2; ++p)
            ea[p] = l == 1 ? a_win + p * WIN_BUF_B + r * WIN_ROW_B
                           : a_xs + (p ^ 1) * XS_PAR_B + (l - 2) * XS_LVL_B + r * XS_ROW_B;
        }
      }
    auto step = [&](int q, auto par_c) __attribute__((always_inline)) {
      constexpr int P = decltype(par_c)::value;
      __builtin_amdgcn_sched_barrier(0);
      wait_vm_le(nst);
      lds_barrier();
      if (q < qdma) issue(q + 1, P ^ 1);
      // (outside hipcc's view, so it is not ordered against the in-flight window DMA; the u0 rows it
      // reads landed before the barrier)
      T ev;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(ev) : "v"(ea[P]) : "memory");
      auto eo_at = [&](int e) -> T {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ev), e));
      };
      const int lzo = q - LAG;
      const bool valid = lzo >= zs && lzo < ze;
#pragma unroll
      for (int l = K; l >= 1; --l) {
        const int m = q - (2 * l - 1);
        T zm = T(1), zp = T(1);
        bool zhp = false;
        if (GEN) {
          const int gm = m + gzoff, gp = m + 1 + gzoff;
          zm = (gm <= 0 || gm >= gnz - 1) ? T(0) : T(1);
          zhp = gp <= 0 || gp >= gnz - 1;
          zp = zhp ? T(0) : T(1);
        }
        // input rows of level l-1 at plane p = m + 1 (rows lo(l)-1 .. hi(l)) and their x sums
        auto vin = [&](int i) -> Row {
          if (l == 1) return RO::fromv(V(wrow[P * WIN_BUF + (i + K) * WROW]));
          const int j = l - 1;
          if (i < SH::lo(j)) return RO::fromv(seam[xh][P ^ 1][j - 1][wu][1][lane]);
          if (i >= SH::hi(j)) return RO::fromv(seam[xh][P ^ 1][j - 1][wd][0][lane]);
          return H[j - 1][P ^ 1][i - SH::lo(j)];
        };
        auto eo = [&](int i) -> T { return eo_at(eidx(l, i)); };
        Row vm = vin(SH::lo(l) - 1), vc = vin(SH::lo(l));
        Row hm = hs(vm, eo(SH::lo(l) - 1)), hc = hs(vc, eo(SH::lo(l)));
#pragma unroll
        for (int i = SH::lo(l); i < SH::hi(l); ++i) {
          const int il = i - SH::lo(l);
          const Row vp = vin(i + 1);
          const Row hp = hs(vp, eo(i + 1));
          const Row cross = RO::add(hc, RO::add(vm, vp));
          const Row diag = RO::add(hm, hp);
          Row a, bb;
          const bool yh = GEN && (y0 + i == 0 || y0 + i == ny - 1);
          if (yh) {
            a = RO::zero();
            bb = vc;
          } else {
            a = RO::lin3r(vc, cross, diag, k1, k2, k3);
            bb = RO::lin3r(vc, cross, diag, k0, k1, k2);
          }
          if (GEN && zhp) bb = vc;
          const Row o = GEN ? RO::fmaz(zm, a, S[l - 1][il]) : RO::add(S[l - 1][il], a);
          S[l - 1][il] = GEN ? RO::fmaz(zp, Ap[l - 1][P ^ 1][il], bb) : RO::add(Ap[l - 1][P ^ 1][il], bb);
          Ap[l - 1][P][il] = a;
          if (l == K) {
            if (valid && i >= 0 && i < SH::R && y0 + i < ny && own) {
              T* ad = ob + (int64_t)lzo * plane + (int64_t)i * pitch;
              dcheck(g, (const T*)out, ad, N);
              store_nt((V*)ad, RO::vec(o));
              if (RES) {
                const Row& cen = H[K - 2][P][i - SH::lo(K - 1)];
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
            st1(xs_mine + P * XS_PAR + (l - 1) * XS_LVL + i * 2 * 64, right ? RO::first(o) : RO::last(o));
          }
          vm = vc;
          vc = vp;
          hm = hc;
          hc = hp;
        }
      }
      nst = valid ? nsto : 0;
    };
    for (int q = zs - K; q <= qend; q += 2) {
      step(q, IC<0>{});
      step(q + 1, IC<1>{});
    }
  };
  const bool fast = yint && zint;
  if (wy == 0) {
    if (fast) march(IC<0>{}, std::false_type{});
    else march(IC<0>{}, std::true_type{});
  } else if (wy == WB - 1) {
    if (fast) march(IC<2>{}, std::false_type{});
    else march(IC<2>{}, std::true_type{});
  } else {
    if (fast) march(IC<1>{}, std::false_type{});
    else march(IC<1>{}, std::true_type{});
  }
  wait_vm0();
  if (RES) wave_atomic_add(resid, acc);
}

template <class T, int RY, int RE, int K, int WB>
static void launch_b27p(const Geo& g, const T* in, T* out, const StencilCoef& cf, double* resid, hipStream_t s) {
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int64_t planes2 = g.lz2_end > g.lz2_begin ? g.lz2_end - g.lz2_begin : 0;
  const int YT = (int)((g.ny + BR - 1) / BR);
  const void* kfn = (const void*)&box27_wxp<T, RY, RE, K, WB, false>;
  const int64_t resident = resident_blocks(kfn, 2 * 64 * WB);
  int zc = knobs().zc > 0 ? knobs().zc : wx_zc(planes, YT, resident, K, 3 * K - 1, g.min_rounds);
  if (planes2 > 0) zc = (int)std::max(planes, planes2);
  const int ZT = (int)((planes + zc - 1) / zc) + (planes2 > 0 ? (int)((planes2 + zc - 1) / zc) : 0);
  const int64_t ntasks = (int64_t)YT * ZT;
  if (knobs().debug_zc)
    fprintf(stderr, "[mdfx] box27_wxp K=%d RY=%d RE=%d WB=%d: %lld planes x %d bands, %lld slots -> zc %d\n", K, RY, RE,
            WB, (long long)planes, YT, (long long)resident, zc);
  MDFX_CHECK(ntasks < (int64_t)1 << 31, "box27_wxp: too many tasks");
  const dim3 grd((unsigned)ntasks), blk(2 * 64 * WB);
  const T c0 = (T)cf.c0, c1 = (T)cf.c1, c2 = (T)cf.c2, c3 = (T)cf.c3;
  if (resid)
    hipLaunchKernelGGL((box27_wxp<T, RY, RE, K, WB, true>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT,
                       (int)ntasks, resid);
  else
    hipLaunchKernelGGL((box27_wxp<T, RY, RE, K, WB, false>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, YT,
                       (int)ntasks, resid);
}

template <class T, int RY, int RE, int K, int WB>
static void launch_b27x(const Geo& g, const T* in, T* out, const StencilCoef& cf, double* resid, hipStream_t s) {
  constexpr int N = VT<T>::N, OV = (K + N - 1) / N, SEG = (64 - 2 * OV) * N;
  constexpr int BR = 2 * RE + (WB - 2) * RY;
  const int64_t planes = g.lz_end - g.lz_begin;
  const int64_t planes2 = g.lz2_end > g.lz2_begin ? g.lz2_end - g.lz2_begin : 0;
  const int XT = (int)((g.nx + SEG - 1) / SEG);
  const int YT = (int)((g.ny + BR - 1) / BR);
  const int64_t tiles = (int64_t)XT * YT;
  const void* kfn = (const void*)&box27_wxk<T, RY, RE, K, WB, false>;
  const int64_t resident = resident_blocks(kfn, 64 * WB);
  int zc = knobs().zc > 0 ? knobs().zc : wx_zc(planes, tiles, resident, K, 3 * K - 1, g.min_rounds);
  if (planes2 > 0) zc = (int)std::max(planes, planes2);
  const int ZT = (int)((planes + zc - 1) / zc) + (planes2 > 0 ? (int)((planes2 + zc - 1) / zc) : 0);
  const int64_t ntasks = tiles * ZT;
  if (knobs().debug_zc)
    fprintf(stderr, "[mdfx] box27_wxk K=%d RY=%d RE=%d WB=%d: %lld planes x %d x %d tiles, %lld slots -> zc %d\n", K, RY,
            RE, WB, (long long)planes, XT, YT, (long long)resident, zc);
  MDFX_CHECK(ntasks < (int64_t)1 << 31, "box27_wxk: too many tasks");
  const dim3 grd((unsigned)ntasks), blk(64 * WB);
  const T c0 = (T)cf.c0, c1 = (T)cf.c1, c2 = (T)cf.c2, c3 = (T)cf.c3;
  if (resid)
    hipLaunchKernelGGL((box27_wxk<T, RY, RE, K, WB, true>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, XT, YT,
                       (int)ntasks, resid);
  else
    hipLaunchKernelGGL((box27_wxk<T, RY, RE, K, WB, false>), grd, blk, 0, s, in, out, g, c0, c1, c2, c3, zc, XT, YT,
                       (int)ntasks, resid);
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
  // fp32 rows of 257..512 cells with MDFX_B27_WXP = 1: the x-pair kernel (two 256-cell halves, no
  // overlapping lanes, bands of 4 waves per half). Off by default: its 6-row bands fetch twice the
  // window rows per output row and it ran 909 vs 1017-1026 GCells/s for the overlapping segments at
  // 512^3 (profiles/r03_session_t/)
  if constexpr (sizeof(T) == 4) {
    if (g.pitch > 256 && g.pitch <= 512 && knobs().b27_wxp != 0) {
      launch_b27p<T, 2, 1, 3, 4>(g, in, out, cf, resid, s);
      return;
    }
  }
  // 2-row inner waves, 1-row edge waves, bands of 8 (14 rows): the 3-row shapes need more than
  // 256 VGPRs
  launch_b27x<T, 2, 1, 3, 8>(g, in, out, cf, resid, s);
}
template void launch_box27_wxk<float>(const Geo&, const float*, float*, const StencilCoef&, int, double*, hipStream_t);
template void launch_box27_wxk<double>(const Geo&, const double*, double*, const StencilCoef&, int, double*, hipStream_t);

}  // namespace dev
}  // namespace mdfx
