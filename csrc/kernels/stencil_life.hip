// Tuned gfx950 Game-of-Life kernel (Moore-8, B3/S23) on uint8 cells, 16 cells per lane.
//
// Each wave is an independent task (1024 cells of a row x zc rows) marching down the rows. Per
// row the lane loads 16 cells with one dwordx4 and evaluates them bit-parallel (SWAR) in two
// 64-bit words: column sums S = north + centre + south (bytes <= 3), then T = S(x-1) + S + S(x+1)
// via byte shifts with the carry byte taken from the neighbouring lane (DPP shift) or, at the
// wave edge, from scalar loads; alive' = ((T - alive) | alive) == 3 (the B3/S23 rule in one
// exact per-byte comparison, life_next). Reference: game_of_life kernel.cu:10-68 (one int per
// cell, 8 scalar loads per cell, dead edge branches D9) -> 1 B read + 1 B written per cell here.
#include <algorithm>

#include "kcommon.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target);

struct U2 {
  uint64_t lo, hi;
};

// B3/S23 on 8 cells at once. t = 3x3 sum including the cell (bytes 0..9), c = the cell (0 / 1).
// With n = t - c the neighbour count, the cell lives next iff n == 3 or (c and n == 2), i.e.
// iff (n | c) == 3: one byte compare instead of two. u = (n | c) ^ 3 is at most 11 per byte, so
// u + 0x7F sets bit 7 exactly when u != 0 and never carries into the next byte. 0x01 per live byte.
__device__ __forceinline__ uint64_t life_next(uint64_t t, uint64_t c) {
  const uint64_t u = ((t - c) | c) ^ 0x0303030303030303ull;
  return (~(u + 0x7F7F7F7F7F7F7F7Full) & 0x8080808080808080ull) >> 7;
}

template <bool RES>
__global__ __launch_bounds__(256) void life_wave(const uint8_t* __restrict__ in,
                                                 uint8_t* __restrict__ out, Geo g, int zc, int XT,
                                                 int ntasks, double* __restrict__ resid) {
  constexpr int N = 16;
  constexpr int WX = 64 * N;
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform, no barriers
  const int xt = task % XT, zt = task / XT;
  const int64_t x = (int64_t)xt * WX + (int64_t)lane * N;
  const int64_t lzs = g.lz_begin + (int64_t)zt * zc;
  const int64_t lze = min(g.lz_end, lzs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t plane = g.plane;
  auto ld = [&](int64_t lz) -> U2 {
    U2 v{0, 0};
    if (xin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x, N);
      const uint4 q = *(const uint4*)(in + lz * plane + x);
      v.lo = (uint64_t)q.x | ((uint64_t)q.y << 32);
      v.hi = (uint64_t)q.z | ((uint64_t)q.w << 32);
    }
    return v;
  };
  auto ldl = [&](int64_t lz) -> uint64_t {
    if (lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x - 1, 1);
      return in[lz * plane + x - 1];
    }
    return 0;
  };
  auto ldr = [&](int64_t lz) -> uint64_t {
    if (lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x + N, 1);
      return in[lz * plane + x + N];
    }
    return 0;
  };
  U2 P = ld(lzs - 1), C = ld(lzs), Nx = ld(lzs + 1);
  uint64_t elP = ldl(lzs - 1), elC = ldl(lzs), elN = ldl(lzs + 1);
  uint64_t erP = ldr(lzs - 1), erC = ldr(lzs), erN = ldr(lzs + 1);
  double acc = 0.0;
  for (int64_t lz = lzs; lz < lze; ++lz) {
    const U2 NN = ld(lz + 2);
    const uint64_t elNN = ldl(lz + 2), erNN = ldr(lz + 2);
    const int64_t gz = lz + g.gz_off;
    U2 o = C;
    if (gz != 0 && gz != g.gnz - 1) {
      const U2 S{P.lo + C.lo + Nx.lo, P.hi + C.hi + Nx.hi};
      // carry bytes from the neighbouring lanes (DPP row shifts; lanes 0 / 63 are replaced below)
      uint64_t sl = (uint32_t)lane_up1((int)(S.hi >> 56));
      uint64_t sr = (uint32_t)lane_down1((int)(S.lo & 0xFF));
      if (lane == 0) sl = elP + elC + elN;
      if (lane == 63) sr = erP + erC + erN;
      const U2 L{(S.lo << 8) | sl, (S.hi << 8) | (S.lo >> 56)};
      const U2 R{(S.lo >> 8) | (S.hi << 56), (S.hi >> 8) | (sr << 56)};
      const U2 T{L.lo + S.lo + R.lo, L.hi + S.hi + R.hi};
      o.lo = life_next(T.lo, C.lo);
      o.hi = life_next(T.hi, C.hi);
      if (x == 0 || x + N > g.nx - 1) {  // frame or pad cells in this lane: copy through
#pragma unroll
        for (int e = 0; e < N; ++e) {
          const int64_t xe = x + e;
          if (xe == 0 || xe >= g.nx - 1) {
            const uint64_t m = 0xFFull << (8 * (e & 7));
            if (e < 8)
              o.lo = (o.lo & ~m) | (C.lo & m);
            else
              o.hi = (o.hi & ~m) | (C.hi & m);
          }
        }
      }
    }
    if (xin) {
      uint4 q;
      q.x = (uint32_t)o.lo;
      q.y = (uint32_t)(o.lo >> 32);
      q.z = (uint32_t)o.hi;
      q.w = (uint32_t)(o.hi >> 32);
      dcheck(g, (const uint8_t*)out, out + lz * plane + x, N);
      *(uint4*)(out + lz * plane + x) = q;
      if (RES) {
        uint64_t dlo = o.lo ^ C.lo, dhi = o.hi ^ C.hi;
        int cnt = 0;
        // only cells with x < nx count
        for (int e = 0; e < N; ++e)
          if (x + e < g.nx) cnt += (int)(((e < 8 ? dlo : dhi) >> (8 * (e & 7))) & 1);
        acc += (double)cnt;
      }
    }
    P = C;
    C = Nx;
    Nx = NN;
    elP = elC;
    elC = elN;
    elN = elNN;
    erP = erC;
    erC = erN;
    erN = erNN;
  }
  if (RES) wave_atomic_add(resid, acc);
}

void launch_life(const Geo& g, const uint8_t* in, uint8_t* out, double* resid, hipStream_t s) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int WX = 64 * 16;
  const int XT = (int)((g.nx + WX - 1) / WX);
  // 32768^2: zc 64 beats 128 (profiles/archive/r01_ab_life_u8.json), zc 32 beats 64 once the carry bytes
  // moved to DPP (2414 vs 2351 GCells/s, profiles/archive/r01_life_tb2.txt)
  const int zc = pick_zc(planes, XT, 256, 4 * 8192);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL(life_wave<true>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL(life_wave<false>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
}

// ---- two generations per sweep ---------------------------------------------------------------
//
// Like jacobi5_tb2: per row c a wave computes generation t+1 of row c for its 1024 cells and, in
// lanes 0 / 63, of the one cell beyond each segment edge (from a 4-byte load of the two cells
// beyond the edge), then generation t+2 of row c-1. 1 B read + 1 B written per cell per TWO
// generations; bitwise equal to two life_wave steps.
__device__ __forceinline__ U2 ld_u2(const uint8_t* p) {
  const uint4 q = *(const uint4*)p;
  return U2{(uint64_t)q.x | ((uint64_t)q.y << 32), (uint64_t)q.z | ((uint64_t)q.w << 32)};
}

template <bool RES>
__global__ __launch_bounds__(256) void life_tb2(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                Geo g, int zc, int XT, int ntasks, double* __restrict__ resid) {
  constexpr int N = 16;
  constexpr int WX = 64 * N;
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform, no barriers
  const int xt = task % XT, zt = task / XT;
  const int64_t x0 = (int64_t)xt * WX;
  const int64_t x = x0 + (int64_t)lane * N;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  const bool xin = x < g.pitch;
  const int64_t plane = g.plane;
  // lane 0: cells x0-2, x0-1 (bytes 2, 3 of the word at x0-4); lane 63: x0+WX, x0+WX+1 (bytes 0, 1)
  const bool hin = (lane == 0 && x0 > 0) || (lane == 63 && x0 + WX < g.pitch);
  const int64_t hoff = lane == 0 ? x0 - 4 : x0 + WX;
  const int64_t hcol = lane == 0 ? x0 - 1 : x0 + WX;
  const bool hframe = hcol <= 0 || hcol >= g.nx - 1;
  const bool frame = x == 0 || x + N > g.nx - 1;  // frame or pad cells in this lane
  auto ld = [&](int64_t lz) -> U2 {
    if (xin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + x, N);
      return ld_u2(in + lz * plane + x);
    }
    return U2{0, 0};
  };
  auto ldh = [&](int64_t lz) -> uint32_t {
    if (hin && lz >= 0 && lz < g.lz_max) {
      dcheck(g, in, in + lz * plane + hoff, 4);
      return *(const uint32_t*)(in + lz * plane + hoff);
    }
    return 0u;
  };
  // the two halo cells as (adjacent, next): lane 0 -> (byte 3, byte 2), lane 63 -> (byte 0, byte 1)
  auto hadj = [&](uint32_t w) -> uint64_t { return lane == 0 ? (w >> 24) & 0xFF : w & 0xFF; };
  auto hnext = [&](uint32_t w) -> uint64_t { return lane == 0 ? (w >> 16) & 0xFF : (w >> 8) & 0xFF; };
  // own cell next to the halo: lane 0 -> cell 0, lane 63 -> cell 15
  auto own = [&](const U2& v) -> uint64_t { return lane == 0 ? v.lo & 0xFF : v.hi >> 56; };
  // one SWAR generation of the lane's 16 cells; esum = 3-row sum of the cell beyond the lane's
  // wave edge (lane 0: left, lane 63: right)
  auto gen = [&](const U2& P, const U2& C, const U2& Nn, uint64_t esum) -> U2 {
    const U2 S{P.lo + C.lo + Nn.lo, P.hi + C.hi + Nn.hi};
    uint64_t sl = (uint32_t)lane_up1((int)(S.hi >> 56));
    uint64_t sr = (uint32_t)lane_down1((int)(S.lo & 0xFF));
    if (lane == 0) sl = esum;
    if (lane == 63) sr = esum;
    const U2 L{(S.lo << 8) | sl, (S.hi << 8) | (S.lo >> 56)};
    const U2 R{(S.lo >> 8) | (S.hi << 56), (S.hi >> 8) | (sr << 56)};
    const U2 T{L.lo + S.lo + R.lo, L.hi + S.hi + R.hi};
    U2 o{life_next(T.lo, C.lo), life_next(T.hi, C.hi)};
    if (frame) {
#pragma unroll
      for (int e = 0; e < N; ++e) {
        const int64_t xe = x + e;
        if (xe == 0 || xe >= g.nx - 1) {
          const uint64_t m = 0xFFull << (8 * (e & 7));
          if (e < 8)
            o.lo = (o.lo & ~m) | (C.lo & m);
          else
            o.hi = (o.hi & ~m) | (C.hi & m);
        }
      }
    }
    return o;
  };

  U2 P = ld(zs - 2), C = ld(zs - 1), Nx = ld(zs);
  uint32_t hP = ldh(zs - 2), hC = ldh(zs - 1), hN = ldh(zs);
  U2 Ua{0, 0}, Ub{0, 0};
  uint64_t ha = 0, hb = 0;  // generation t+1 of the halo cell, rows c-2 and c-1
  double acc = 0.0;
  for (int64_t c = zs - 1; c <= ze; ++c) {
    const U2 NN = ld(c + 2);
    const uint32_t hNN = ldh(c + 2);
    // ---- generation t+1 of row c (segment + halo cell)
    const int64_t gz = c + g.gz_off;
    U2 Uc = C;
    uint64_t hc = hadj(hC);
    if (gz > 0 && gz < g.gnz - 1) {
      Uc = gen(P, C, Nx, hadj(hP) + hadj(hC) + hadj(hN));
      if (!hframe) {
        const uint64_t t = (hadj(hP) + hadj(hC) + hadj(hN)) + (hnext(hP) + hnext(hC) + hnext(hN)) +
                           (own(P) + own(C) + own(Nx));
        hc = (uint64_t)sm::life_rule((unsigned)t, (unsigned char)hadj(hC));
      }
    }
    // ---- generation t+2 of row c-1
    if (c >= zs + 1) {
      const int64_t lz = c - 1;
      const int64_t gz2 = lz + g.gz_off;
      U2 o = Ub;
      if (gz2 != 0 && gz2 != g.gnz - 1) o = gen(Ua, Ub, Uc, ha + hb + hc);
      if (xin) {
        uint4 q;
        q.x = (uint32_t)o.lo;
        q.y = (uint32_t)(o.lo >> 32);
        q.z = (uint32_t)o.hi;
        q.w = (uint32_t)(o.hi >> 32);
        dcheck(g, (const uint8_t*)out, out + lz * plane + x, N);
        *(uint4*)(out + lz * plane + x) = q;
        if (RES) {
          const uint64_t dlo = o.lo ^ Ub.lo, dhi = o.hi ^ Ub.hi;
          int cnt = 0;
          for (int e = 0; e < N; ++e)
            if (x + e < g.nx) cnt += (int)(((e < 8 ? dlo : dhi) >> (8 * (e & 7))) & 1);
          acc += (double)cnt;
        }
      }
    }
    P = C;
    C = Nx;
    Nx = NN;
    hP = hC;
    hC = hN;
    hN = hNN;
    Ua = Ub;
    Ub = Uc;
    ha = hb;
    hb = hc;
  }
  if (RES) wave_atomic_add(resid, acc);
}

void launch_life_tb2(const Geo& g, const uint8_t* in, uint8_t* out, double* resid, hipStream_t s) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int WX = 64 * 16;
  const int XT = (int)((g.nx + WX - 1) / WX);
  const int zc = pick_zc(planes, XT, 256, 4 * 8192);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL(life_tb2<true>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL(life_tb2<false>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
}

// (Round 4's SWAR K-generation kernel, life_tbk: 7,656-7,960 GCells/s at 32768^2 against life_bits'
// 21,268-22,430, profiles/archive/r02_life.txt, reachable only through a switch, was removed in round 5.)

// ---- K generations per sweep, bit-sliced (life_bits) ---------------------------------------------
//
// One bit per cell inside the sweep: each lane loads 32 u8 cells of a row (two 16-B vectors), packs
// them into a 32-bit word (bit j = cell x + j: per 4 cells one multiply-gather, v_mul + v_bfe),
// runs K generations on the words and unpacks the last one back to bytes for the store. A
// generation of 32 cells is ~22 bitwise ops instead of ~100 SWAR byte ops for 16:
//   row sums on arrival (L / R = the row shifted by one cell, the cell beyond the lane through a
//   DPP lane shift and v_alignbit):  2-sum c = L + R  (c0 = L ^ R, c1 = L & R),
//                                     3-sum s = L + X + R  (s0 = c0 ^ X, s1 = maj(L, X, R))
//   neighbours of row r: N = s(r-1) + s(r+1) + c(r) (a 4-bit ripple of full adders, 10 ops)
//   B3/S23: alive' = (N | alive) == 3  ->  n1 & (n0 | alive) & ~(n2 | n3)
// Each level keeps the 3-sums of its last two input rows, the 2-sum and the cells of the last row.
// Waves overlap by one lane per side (a generation corrupts one more cell of the halo lanes from the
// outside in: K <= 32). Held cells (x = 0, x >= nx - 1, the first / last row)
// keep their state through a per-lane bit mask. Bitwise equal to K single generations.
__device__ __forceinline__ uint32_t life_pack4(uint32_t d) {  // bytes 0/1 -> bits 0..3
  return __builtin_amdgcn_ubfe(d * 0x01020408u, 24, 4);
}
__device__ __forceinline__ uint32_t life_unpack4(uint32_t w, int k) {  // bits 4k..4k+3 -> bytes 0/1
  return (__builtin_amdgcn_ubfe(w, 4 * k, 4) * 0x00204081u) & 0x01010101u;
}

template <int K, bool RES>
__global__ __launch_bounds__(256) void life_bits(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                 Geo g, int zc, int XT, int ntasks, double* __restrict__ resid) {
  constexpr int CW = 32;        // cells per lane
  constexpr int SEG = 62 * CW;  // owned cells per wave
  static_assert(K >= 1 && K <= CW, "generations must not reach past the halo lanes");
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;  // wave-uniform, no barriers
  const int xt = task % XT, zt = task / XT;
  const int64_t x = (int64_t)xt * SEG - CW + (int64_t)lane * CW;
  const int64_t zs = g.lz_begin + (int64_t)zt * zc;
  const int64_t ze = min(g.lz_end, zs + (int64_t)zc);
  // pitch is a multiple of 256 cells, x of 32: a lane is wholly inside the row or wholly outside
  const bool xin = x >= 0 && x < g.pitch;
  const bool own = lane >= 1 && lane <= 62 && xin;
  const int64_t plane = g.plane;
  // held cells (x + j == 0 or x + j >= nx - 1) and cells inside the grid (x + j < nx)
  const int64_t hf = g.nx - 1 - x, vf = g.nx - x;
  const uint32_t hm = (x == 0 ? 1u : 0u) | (hf <= 0 ? ~0u : hf >= 32 ? 0u : ~0u << hf);
  const uint32_t vm = vf >= 32 ? ~0u : vf <= 0 ? 0u : (1u << vf) - 1u;
  // lanes outside the row read the nearest in-row vectors, rows past the storage its last row:
  // finite values that only meet halo lanes or held cells
  const uint8_t* ib = in + (x < 0 ? 0 : x >= g.pitch ? g.pitch - CW : x);
  auto ld = [&](int64_t lz) -> uint32_t {
    const int64_t lzc = lz < 0 ? 0 : lz >= g.lz_max ? g.lz_max - 1 : lz;
    dcheck(g, in, ib + lzc * plane, CW);
    const uint4* p = (const uint4*)(ib + lzc * plane);
    const uint4 a = p[0], b = p[1];
    return life_pack4(a.x) | life_pack4(a.y) << 4 | life_pack4(a.z) << 8 | life_pack4(a.w) << 12 |
           life_pack4(b.x) << 16 | life_pack4(b.y) << 20 | life_pack4(b.z) << 24 | life_pack4(b.w) << 28;
  };
  struct RowSums {
    uint32_t s0, s1, c0, c1;
  };
  auto sums = [&](uint32_t X) -> RowSums {
    const uint32_t up = (uint32_t)lane_up1((int)X), dn = (uint32_t)lane_down1((int)X);
    const uint32_t L = __builtin_amdgcn_alignbit(X, up, 31);  // cell x + j - 1
    const uint32_t R = __builtin_amdgcn_alignbit(dn, X, 1);   // cell x + j + 1
    RowSums r;
    r.c0 = L ^ R;
    r.c1 = L & R;
    r.s0 = r.c0 ^ X;
    r.s1 = (r.c0 & X) | (~r.c0 & L);  // maj(L, X, R)
    return r;
  };
  // next state of row r from the 3-sums of rows r - 1 (a) and r + 1 (b) and row r's 2-sum / cells
  auto gen = [&](const RowSums& a, const RowSums& b, const RowSums& c, uint32_t self) -> uint32_t {
    const uint32_t x0 = a.s0 ^ b.s0;
    const uint32_t n0 = x0 ^ c.c0;
    const uint32_t k0 = (x0 & c.c0) | (~x0 & a.s0);  // maj(a0, b0, c0)
    const uint32_t y1 = a.s1 ^ b.s1;
    const uint32_t k1a = (y1 & c.c1) | (~y1 & a.s1);  // maj(a1, b1, c1)
    const uint32_t z1 = y1 ^ c.c1;
    const uint32_t n1 = z1 ^ k0;
    const uint32_t k1b = z1 & k0;
    const uint32_t hi = k1a | k1b;  // n2 | n3
    const uint32_t o = n1 & (n0 | self) & ~hi;
    return (hm & self) | (~hm & o);
  };
  RowSums P2[K], P1[K], Cs[K];  // level l = 1..K at index l - 1: 3-sums of rows q-2 / q-1, row q-1
  uint32_t Xp[K];
#pragma unroll
  for (int l = 0; l < K; ++l) {
    P2[l] = P1[l] = Cs[l] = RowSums{0, 0, 0, 0};
    Xp[l] = 0;
  }
  {
    const uint32_t a = ld(zs - K - 1), b = ld(zs - K);
    P2[0] = sums(a);
    P1[0] = Cs[0] = sums(b);
    Xp[0] = b;
  }
  uint32_t nxt = ld(zs - K + 1);
  double acc = 0.0;
  for (int64_t q = zs - K + 1; q <= ze - 1 + K; ++q) {
    uint32_t X = nxt;  // u0(q)
    nxt = ld(q + 1);
    const int64_t lz = q - K;
#pragma unroll
    for (int l = 1; l <= K; ++l) {
      const RowSums sq = sums(X);
      const uint32_t self = Xp[l - 1];
      const int64_t row = q - l;  // the row this level finishes
      const int64_t gz = row + g.gz_off;
      const bool bnd = l < K ? (gz <= 0 || gz >= g.gnz - 1) : (gz == 0 || gz == g.gnz - 1);
      const uint32_t o = bnd ? self : gen(P2[l - 1], sq, Cs[l - 1], self);
      P2[l - 1] = P1[l - 1];
      P1[l - 1] = Cs[l - 1] = sq;
      Xp[l - 1] = X;
      if (l < K) {
        X = o;
      } else if (lz >= zs && own) {
        uint4 qa, qb;
        qa.x = life_unpack4(o, 0);
        qa.y = life_unpack4(o, 1);
        qa.z = life_unpack4(o, 2);
        qa.w = life_unpack4(o, 3);
        qb.x = life_unpack4(o, 4);
        qb.y = life_unpack4(o, 5);
        qb.z = life_unpack4(o, 6);
        qb.w = life_unpack4(o, 7);
        uint4* p = (uint4*)(out + lz * plane + x);
        dcheck(g, (const uint8_t*)out, (const uint8_t*)p, CW);
        p[0] = qa;
        p[1] = qb;
        if (RES) acc += (double)__builtin_popcount((o ^ self) & vm);
      }
    }
  }
  if (RES) wave_atomic_add(resid, acc);
}

template <int K>
static void launch_life_bits_k(const Geo& g, const uint8_t* in, uint8_t* out, double* resid, hipStream_t s) {
  const int64_t planes = g.lz_end - g.lz_begin;
  if (planes <= 0) return;
  constexpr int SEG = 62 * 32;
  const int XT = (int)((g.nx + SEG - 1) / SEG);
  const int zc = pick_zc(planes, XT, 256, 4 * 2048);
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL((life_bits<K, true>), grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL((life_bits<K, false>), grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
}

void launch_life_tbk(const Geo& g, const uint8_t* in, uint8_t* out, int steps, double* resid, hipStream_t s) {
  // K > 2 generations per sweep, bit-sliced (two generations: life_tb2)
  switch (steps) {
    case 3: launch_life_bits_k<3>(g, in, out, resid, s); return;
    case 4: launch_life_bits_k<4>(g, in, out, resid, s); return;
    case 6: launch_life_bits_k<6>(g, in, out, resid, s); return;
    case 8: launch_life_bits_k<8>(g, in, out, resid, s); return;
    case 12: launch_life_bits_k<12>(g, in, out, resid, s); return;
    case 16: launch_life_bits_k<16>(g, in, out, resid, s); return;
    default: MDFX_FAIL(format("life: no %d-generation sweep (3, 4, 6, 8, 12, 16)", steps));
  }
}

}  // namespace dev
}  // namespace mdfx
