// Sweep plan of the engine's step loop (Solver::run): how a run of time steps is cut into fused
// sweeps. A host-side pure function of the supported depths and their costs, so it is unit-tested
// on the CPU with the GPU's cost tables (tests/test_cpu_engine.py).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace mdfx {

struct SweepCosts {
  int T = 1;              // deepest fused depth (every slab supports it)
  double cost[17] = {};   // cost[k]: relative time of one k-step sweep (cost[1] = one single step)
  bool ok[17] = {false, true};  // ok[k]: a k-step sweep exists on every slab
};

// Depth of the next sweep of a `len`-step stretch (the steps up to the next residual evaluation, or
// to the end of the run; res_end: the stretch ends at a residual step), and in *graphable how many
// depth-T sweeps follow back to back without a residual (the sweeps replayed in pairs).
int plan_next_sweep(const SweepCosts& c, int64_t len, bool res_end, int64_t* graphable);

// The (depth, residual sweep) list of `steps` steps from step `start` with a residual every
// `residual_every` steps (0: none): plan_next_sweep applied the way Solver::run applies it.
std::vector<std::pair<int, bool>> plan_sweeps(const SweepCosts& c, int64_t steps, int64_t start,
                                              int64_t residual_every);

// The fused depth (at most c.T) for a run with a residual every `residual_every` steps (c.T itself
// without one). One rank: the depth whose sweep plan of one interval costs least, among the depths
// whose plan runs a sweep of that depth (ties: the deeper) - the plan at depth T cuts the interval
// into T-step sweeps and a cheapest tail of < 2T steps, so a shallower depth can plan a cheaper
// cut. Several ranks (`uniform`): the deepest depth whose interval is whole sweeps of that depth,
// else the one-rank rule - every sweep of a run exchanges and recomputes boundary regions as deep
// as the layout's halo, so a 4- or 3-step sweep on a 5-plane halo pays for 5 planes (round 6,
// 2048^3 fp64, residual every 12: one GPU 1022 GCells/s at depth 5 (5 + 4 + 3) against 961-985 at
// depth 4 (4 + 4 + 4), but the N = 8 rank proxy 841-849 against 878-880; profiles/r06_session_g/).
int interval_depth(const SweepCosts& c, int64_t residual_every, bool uniform = false);

}  // namespace mdfx
