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

// The maximum depth (at most c.T) whose sweep plan of one residual interval costs least, among the
// depths whose plan runs a sweep of that depth (ties: the deeper; c.T itself without a residual).
// The plan at depth T cuts the interval into T-step sweeps and a cheapest tail of < 2T steps, so
// it can miss a cheaper all-shallower cut: a residual every 12 steps at depth 5 plans 5 + 4 + 3
// (fp64 costs 3.91) where depth 4's 4 + 4 + 4 costs 3.75, and the depth-5 layout also exchanges
// and recomputes 5-plane boundary regions every sweep (round 6: 2048^3 fp64 1,041.6 GCells/s and
// rank proxy N = 8 834.9 at depth 5, against 1,057 / 900.5 at depth 4; profiles/r06_session_e/).
int interval_depth(const SweepCosts& c, int64_t residual_every);

}  // namespace mdfx
