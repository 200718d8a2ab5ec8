// Shared pieces of the y-halo-exchange kernels (heat7_wxk, box27_wxk): the per-role row ranges of
// a band's waves and the z-chunk plan.
#pragma once

#include <algorithm>
#include <cstdint>
#include <type_traits>

namespace mdfx {
namespace dev {

// rows of level l (1..K) a wave computes, relative to its first own row y0: [lo, hi)
// ROLE 0 = the band's first wave (trapezoid above), 1 = inner waves, 2 = the band's last wave.
// Inner waves own RY rows, the two edge waves RE: an edge wave also computes the K-l trapezoid
// rows outside the band at level l, so RE < RY evens out the waves' work per plane (every wave
// waits for the slowest at the plane barrier)
template <int ROLE, int RY, int RE, int K>
struct WxRows {
  static constexpr int R = ROLE == 1 ? RY : RE;  // own rows
  static constexpr int lo(int l) { return ROLE == 0 ? -(K - l) : 0; }
  static constexpr int hi(int l) { return R + (ROLE == 2 ? K - l : 0); }
  static constexpr int n(int l) { return hi(l) - lo(l); }
};

template <int V>
using IC = std::integral_constant<int, V>;

// chunked schedule of a streaming sweep over `planes` planes of `tiles` tiles on `resident` block
// slots, every chunk paying `fill` extra plane steps: the chunk count minimising rounds x (zc + fill)
// (chunks of at least `min_chunk` planes, default 4K; at least `min_rounds` rounds when asked)
inline int wx_zc(int64_t planes, int64_t tiles, int64_t resident, int K, int64_t fill, int min_rounds,
                 int64_t min_chunk = 0) {
  const int64_t zmax = std::max<int64_t>(1, planes / (min_chunk > 0 ? min_chunk : 4 * K));
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

}  // namespace dev
}  // namespace mdfx
