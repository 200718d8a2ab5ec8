// Tuned gfx950 Game-of-Life kernel (Moore-8, B3/S23) on uint8 cells, 16 cells per lane.
//
// Each wave is an independent task (1024 cells of a row x zc rows) marching down the rows. Per
// row the lane loads 16 cells with one dwordx4 and evaluates them bit-parallel (SWAR) in two
// 64-bit words: column sums S = north + centre + south (bytes <= 3), then T = S(x-1) + S + S(x+1)
// via byte shifts with the carry byte taken from the neighbouring lane (ds_bpermute) or, at the
// wave edge, from scalar loads; alive' = (T == 3) | (alive & (T == 4)) with exact per-byte
// equality tests. Reference: game_of_life kernel.cu:10-68 (one int per cell, 8 scalar loads per
// cell, dead edge branches D9) -> 1 B read + 1 B written per cell here.
#include <algorithm>

#include "kcommon.hpp"
#include "mdfx/kernels.hpp"
#include "mdfx/stencil_math.hpp"

namespace mdfx {
namespace dev {

int pick_zc(int64_t planes, int64_t columns, int zc_max, int blocks_target);
int env_int(const char* name, int dflt);

struct U2 {
  uint64_t lo, hi;
};

__device__ __forceinline__ uint64_t bytes_eq(uint64_t t, uint64_t k) {
  // bytes of t are < 0x80: exact zero-byte detection of t ^ k, result 0x01 per equal byte.
  const uint64_t x = t ^ (k * 0x0101010101010101ull);
  const uint64_t z = ~((x + 0x7F7F7F7F7F7F7F7Full) | x) & 0x8080808080808080ull;
  return z >> 7;
}

template <bool RES>
__global__ __launch_bounds__(256) void life_wave(const uint8_t* __restrict__ in,
                                                 uint8_t* __restrict__ out, Geo g, int zc, int XT,
                                                 int ntasks, double* __restrict__ resid) {
  constexpr int N = 16;
  constexpr int WX = 64 * N;
  const int lane = threadIdx.x & 63;
  const int task = (int)xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
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
      const uint4 q = *(const uint4*)(in + lz * plane + x);
      v.lo = (uint64_t)q.x | ((uint64_t)q.y << 32);
      v.hi = (uint64_t)q.z | ((uint64_t)q.w << 32);
    }
    return v;
  };
  auto ldl = [&](int64_t lz) -> uint64_t {
    if (lane == 0 && x > 0 && lz >= 0 && lz < g.lz_max) return in[lz * plane + x - 1];
    return 0;
  };
  auto ldr = [&](int64_t lz) -> uint64_t {
    if (lane == 63 && x + N < g.pitch && lz >= 0 && lz < g.lz_max) return in[lz * plane + x + N];
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
      uint64_t sl = __shfl_up(S.hi >> 56, 1, 64);
      uint64_t sr = __shfl_down(S.lo & 0xFF, 1, 64);
      if (lane == 0) sl = elP + elC + elN;
      if (lane == 63) sr = erP + erC + erN;
      const U2 L{(S.lo << 8) | sl, (S.hi << 8) | (S.lo >> 56)};
      const U2 R{(S.lo >> 8) | (S.hi << 56), (S.hi >> 8) | (sr << 56)};
      const U2 T{L.lo + S.lo + R.lo, L.hi + S.hi + R.hi};
      o.lo = bytes_eq(T.lo, 3) | (C.lo & bytes_eq(T.lo, 4));
      o.hi = bytes_eq(T.hi, 3) | (C.hi & bytes_eq(T.hi, 4));
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
  int zc = env_int("MDFX_ZC", 0);
  if (zc <= 0) zc = pick_zc(planes, XT, 256, 4 * 4096);  // 32768^2: zc 64 beats 128 (profiles/r01_ab_life_u8.json)
  const int ZT = (int)((planes + zc - 1) / zc);
  const int ntasks = XT * ZT;
  const dim3 grd((unsigned)((ntasks + 3) / 4)), blk(256);
  if (resid)
    hipLaunchKernelGGL(life_wave<true>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
  else
    hipLaunchKernelGGL(life_wave<false>, grd, blk, 0, s, in, out, g, zc, XT, ntasks, resid);
}

}  // namespace dev
}  // namespace mdfx
