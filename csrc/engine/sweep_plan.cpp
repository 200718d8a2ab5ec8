// Sweep plan (mdfx/sweep_plan.hpp). Each stretch runs depth-T sweeps and a tail of fewer than 2T
// steps cut so that the summed sweep cost is least (ties keep the deepest sweeps first). The depth-T
// sweeps run first (replayed in pairs from the prepared graphs), the tail's sweeps deepest first,
// and the residual is evaluated by the stretch's last sweep.
#include "mdfx/sweep_plan.hpp"

#include <algorithm>

namespace mdfx {

namespace {

// The cheapest cut of r < 2T steps into supported depths: best[l][d] is the least cost of l steps
// in sweeps of at most d steps (ties take the deeper sweep); *first gets the cut's deepest sweep.
double tail_plan(const SweepCosts& c, int r, int* first) {
  const int T = c.T;
  double best[33][17];
  bool use[33][17];
  for (int l = 0; l <= r; ++l)
    for (int d = 1; d <= T; ++d) {
      use[l][d] = false;
      if (l == 0) {
        best[l][d] = 0.0;
        continue;
      }
      if (d == 1) {
        best[l][d] = best[l - 1][1] + c.cost[1];
        use[l][d] = true;
        continue;
      }
      best[l][d] = best[l][d - 1];
      if (c.ok[d] && l >= d) {
        const double v = c.cost[d] + best[l - d][d];
        if (v <= best[l][d] + 1e-9) {
          best[l][d] = v;
          use[l][d] = true;
        }
      }
    }
  if (first) {
    int d = T;
    while (d > 1 && !use[r][d]) --d;
    *first = r > 0 ? d : 1;
  }
  return best[r][T];
}

}  // namespace

int plan_next_sweep(const SweepCosts& c, int64_t len, bool res_end, int64_t* graphable) {
  *graphable = 0;
  const int T = std::max(1, std::min(c.T, 16));
  if (T <= 1 || len <= 1) {  // single steps: all but the residual step replay in pairs
    *graphable = len - (res_end ? 1 : 0);
    return 1;
  }
  SweepCosts cc = c;
  cc.T = T;
  // candidate tails: len mod T and one more sweep's worth; the rest runs at depth T
  const int64_t m = len % T;
  int64_t best_r = -1;
  double best_c = 0.0;
  for (int64_t r : {m, m + T}) {
    if (r > len || r >= 2 * T) continue;
    const double v = (double)((len - r) / T) * cc.cost[T] + tail_plan(cc, (int)r, nullptr);
    if (best_r < 0 || v < best_c - 1e-9) {
      best_r = r;
      best_c = v;
    }
  }
  const int64_t full = (len - best_r) / T;  // depth-T sweeps ahead of the tail
  if (full > 0) {
    // back-to-back depth-T sweeps before the residual sweep (the last one when the tail is empty)
    *graphable = full - ((res_end && best_r == 0) ? 1 : 0);
    return T;
  }
  int first = 1;
  tail_plan(cc, (int)best_r, &first);
  return first;
}

std::vector<std::pair<int, bool>> plan_sweeps(const SweepCosts& c, int64_t steps, int64_t start,
                                              int64_t residual_every) {
  std::vector<std::pair<int, bool>> out;
  int64_t done = 0, at = start;
  while (done < steps) {
    int64_t to_res = steps - done + 1;
    if (residual_every > 0) to_res = ((at / residual_every) + 1) * residual_every - at;
    int64_t graphable = 0;
    const int k = plan_next_sweep(c, std::min(steps - done, to_res), to_res <= steps - done, &graphable);
    out.emplace_back(k, to_res == k);
    done += k;
    at += k;
  }
  return out;
}

int interval_depth(const SweepCosts& c, int64_t residual_every, bool uniform) {
  const int T0 = std::max(1, std::min(c.T, 16));
  if (T0 <= 1 || residual_every <= 0) return T0;
  if (uniform) {
    // several ranks: the deepest depth whose interval is whole sweeps of that depth (a shallower
    // sweep on a deeper layout exchanges and recomputes the deeper halo)
    for (int T = T0; T > 1; --T) {
      if (!c.ok[T]) continue;
      SweepCosts cc = c;
      cc.T = T;
      bool all = true;
      for (const auto& kr : plan_sweeps(cc, residual_every, 0, residual_every)) all = all && kr.first == T;
      if (all) return T;
    }
  }
  int best_t = T0;
  double best = -1.0;
  for (int T = T0; T >= 1; --T) {
    if (T > 1 && !c.ok[T]) continue;
    SweepCosts cc = c;
    cc.T = T;
    double sum = 0.0;
    bool uses = T == 1;
    for (const auto& kr : plan_sweeps(cc, residual_every, 0, residual_every)) {
      sum += kr.first <= 1 ? 1.0 : c.cost[kr.first];
      uses = uses || kr.first == T;
    }
    // (a depth whose plan never sweeps it costs the same as the next one down, with a wider halo)
    if (uses && (best < 0.0 || sum < best - 1e-9)) {
      best = sum;
      best_t = T;
    }
  }
  return best_t;
}

}  // namespace mdfx
