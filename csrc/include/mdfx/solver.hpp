// mdfx engine: the overlapped, double-buffered time-step scheduler.
//
// Reference parity: the per-rank generation loops of MDF_kernel.cu:155-222 / kernel.cu:202-269
// (C12/C13). The reference launched middle_kernel and border_kernel on two streams but then
// serialised everything with cudaDeviceSynchronize (MDF_kernel.cu:175), raced the two streams on
// d_new_univ (D6) and d_univ (D7), and never swapped buffers (D1). Here, per step and per slab:
//
//   halo stream:  wait(interior t-1) -> boundary planes (cur -> nxt)
//                                 -> record(bnd) -> exchange faces of nxt (RCCL / loopback)
//   compute stream:               wait(boundary t-1) -> interior planes (cur -> nxt)
//                                 -> record(int)
//   swap(cur, nxt)
//
// so the interior sweep of step t overlaps the boundary kernel and the halo exchange of step t
// (and the exchange may run on into step t+1's interior). No host synchronisation inside the loop.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "mdfx/runtime.hpp"
#include "mdfx/sweep_plan.hpp"

namespace mdfx {

struct SolverOptions {
  bool overlap = true;        // interior || (boundary + exchange) on two streams
  bool sync_debug = false;    // device-synchronise after every phase (race differential tests)
  int residual_every = 0;     // compute the global L2 update norm every k steps (0 = never)
  bool graph = false;         // replay a captured 2-step cycle as a hipGraph (HIP only)
  double timeout_s = 0.0;     // watchdog for synchronize() / residual / blocking transport calls:
                              // abort the transport and throw instead of hanging (0 = off)
  // Temporal blocking: time steps fused per sweep over memory (1 or 2). With 2 the slabs keep two
  // ghost planes per side, exchanged once per fused step, and every sweep reads u^t once and writes
  // u^{t+2} once (bitwise identical to two single steps). Fixed at construction.
  int temporal = 1;
  // Per-phase hipEvent timing of slab 0 (boundary / interior / exchange / whole step); syncs the
  // host once per step, so it is a diagnostic mode, not a benchmark mode.
  bool profile = false;
  // Minimum whole rounds of resident blocks per streaming fused sweep (RegionArgs::min_rounds):
  // 0 = automatic (2 with several slabs, so exchange kernels that need CUs find some mid-sweep; 1
  // otherwise). Fewer rounds mean longer z chunks, hence less pipeline fill per chunk.
  int min_rounds = 0;
  // Pencil decomposition: subdomains per slab along y (1 = slabs along z only). The nranks
  // subdomains form a (nranks / py) x py grid of (z, y) pencils, each with `temporal` ghost rows
  // per split y side as well as ghost planes. 3D grids only; fixed at construction.
  int py = 1;
  // Folded lower boundary (Solver::fold_ok): -1 = the transport's default (fold_by_default: ipc,
  // proxy, loopback yes, rccl no), 0 = never, 1 = wherever the layout and kernels allow it.
  int fold = -1;
};

// Whether a step may fold, given the fold option and the transport's default.
inline bool fold_allowed(int fold_opt, bool transport_default) {
  return fold_opt > 0 || (fold_opt < 0 && transport_default);
}

struct PhaseStats {
  int64_t steps = 0;  // sweeps profiled
  double boundary_ms = 0, interior_ms = 0, exchange_ms = 0, step_ms = 0;
  // how long the halo stream (the exchange) ran on past the end of the sweep's last kernel: the
  // part of the exchange the sweep did not hide (HIP profile only; 0 on the host clock)
  double exposed_ms = 0;
};

struct StepStats {
  int64_t steps = 0;
  double last_residual = -1.0;  // sqrt(sum over the grid of (u_new - u_old)^2), -1 if never
  int64_t residual_step = -1;
  int64_t graph_replays = 0;  // 2-sweep cycles replayed from a captured hipGraph
  int64_t graph_captures = 0;  // cycles captured + instantiated (prepare_graphs() or on demand)
  int64_t folded_sweeps = 0;   // eager sweeps whose lower boundary ran inside the interior sweep
  // device spin-wait nodes found in the captured graphs: all of them, and those that wait on a
  // slab's own fold counters (a folded boundary inside a capture; must stay 0, see Solver::step)
  int64_t graph_wait_nodes = 0;
  int64_t graph_fold_waits = 0;
};

// The per-step schedule the engine runs for a layout and transport (Solver::boundary_on_cs and
// fold_ok decide it; Solver::schedule() reports it): "serialised" (no overlap: the exchange, then one
// sweep on the halo stream), "two-stream" (boundary kernels + exchange on the halo stream, interior
// on the compute stream; several slabs per process or a host-side exchange), "boundary-on-compute"
// (one slab per process and a stream-ordered exchange: boundary kernels then interior on the
// compute stream, only the exchange on the halo stream) and "folded" (the same with the lower
// boundary region computed inside the interior sweep, heat7_wxk fused sweeps).
const char* step_schedule(bool overlap, size_t local_slabs, bool stream_ordered, bool fold);

// Auto fused depth for a residual interval on the device: interval_depth over the hip_sweep_cost
// tables and the depths hip_supports_steps has on a `want`-deep layout of grid g (uniform sweeps
// with several ranks). want itself when residual_every <= 0.
int hip_interval_depth(const StencilSpec& spec, Extent3 g, int want, int64_t residual_every, int nranks = 1);

class Solver {
 public:
  // local_ranks[i] is the global slab index owned by backends[i] in this process.
  Solver(const StencilSpec& spec, Extent3 global, int nranks, std::vector<int> local_ranks,
         std::vector<std::unique_ptr<Backend>> backends, std::unique_ptr<Transport> transport,
         SolverOptions opt = SolverOptions());
  ~Solver();
  Solver(const Solver&) = delete;
  Solver& operator=(const Solver&) = delete;

  void init(const InitSpec& s);
  void run(int64_t steps);
  // Capture the 2-sweep hipGraph cycles of both buffer parities now (graph option on and the
  // configuration capturable), so a later run() only replays: a benchmark calls this before its
  // warmup and no capture or instantiation ever falls inside a timed region. Returns the number of
  // cycles held (0 if graphs are off or not capturable here). init() keeps them (buffers do not
  // move); option changes that alter the captured work drop them.
  int prepare_graphs();
  // Launch every stencil kernel instance that run(steps) would use once (each fused depth, the
  // residual copy included), into the scratch buffer and without any exchange, then synchronize:
  // the first launch of an instance pays one-time costs (code-object and occupancy queries) that a
  // timed run without warm-up steps would otherwise count. The field state is unchanged.
  void warm_kernels(int64_t steps);
  // The sweeps run(steps) would issue from the current step count: (fused depth, residual sweep).
  std::vector<std::pair<int, bool>> sweep_plan(int64_t steps) const;
  // Whether run() would replay captured cycles in this configuration.
  bool graph_eligible() const;
  // The schedule eager steps of the deepest fused sweep run (step_schedule).
  std::string schedule() const;
  void synchronize();
  // Refresh ghost planes of the current buffer (after write_owned / resume).
  void exchange_ghosts();

  const StencilSpec& spec() const { return spec_; }
  const Extent3& global() const { return global_; }
  int nranks() const { return nranks_; }
  int num_local() const { return (int)slabs_.size(); }
  int local_rank(int i) const { return slabs_[i].rank; }
  const FieldLayout& layout(int i) const { return slabs_[i].lay; }
  Backend& backend(int i) { return *slabs_[i].be; }
  Transport& transport() { return *transport_; }
  const SolverOptions& options() const { return opt_; }
  void set_options(const SolverOptions& o);
  int current_index() const { return cur_; }
  void* buffer(int i, int b) { return slabs_[i].buf[b]; }
  void* current(int i) { return slabs_[i].buf[cur_]; }
  void* halo_stream(int i) { return slabs_[i].hs; }
  void* compute_stream(int i) { return slabs_[i].cs; }
  const StepStats& stats() const { return stats_; }
  const PhaseStats& phases() const { return phases_; }
  void reset_phases() { phases_ = PhaseStats(); }
  int64_t owned_cells_global() const { return global_.cells(); }

  // Dense copies of the owned planes (nx*ny*nzl elements, x fastest, no pitch / ghosts).
  void read_owned(int i, void* host) ;
  void write_owned(int i, const void* host);
  // Checkpoint: every process writes its slabs as <dir>/slab_<rank>.bin + .json; resume reads any
  // decomposition (files are in global plane order).
  void save_checkpoint(const std::string& dir);
  void load_checkpoint(const std::string& dir);

 private:
  struct Slab {
    int rank = 0;
    std::unique_ptr<Backend> be;
    FieldLayout lay;
    void* buf[2] = {nullptr, nullptr};
    void* hs = nullptr;  // halo stream
    void* cs = nullptr;  // compute stream
    void* ev_bnd = nullptr;
    void* ev_int = nullptr;
    void* ev_x = nullptr;  // the last exchange's stream work (boundary kernels on the compute stream wait for it)
    void* ev_x2 = nullptr;  // (transports that record ghost events: the second pull stream's ghosts)
    double* resid = nullptr;  // 2 accumulators (halo-stream kernels, compute-stream kernels)
    int64_t lo_b = 0, lo_e = 0, hi_b = 0, hi_e = 0, in_b = 0, in_e = 0;  // storage-plane regions
    // pencils: storage-row regions of the interior planes (y-boundary strips and interior rows;
    // all 0 for slabs: every owned row)
    int64_t ylo_b = 0, ylo_e = 0, yhi_b = 0, yhi_e = 0, yin_b = 0, yin_e = 0;
    // folded lower boundary (fold_ok()): device counters from hip_alloc_uncached, one block of 32
    // words per signalling launch (the upper boundary launch at [0], the interior sweep at [32]):
    // [+0] the launch's block arrivals, [+16] its completed signals; [64] / [80] the halo stream's
    // private expect counters for the two
    unsigned long long* sig = nullptr;
  };
  void step(bool want_resid, int k);
  void boundary_kernels(Slab& s, RegionArgs a, void* stream, bool skip_lo = false);
  void interior_kernel(Slab& s, RegionArgs a, void* stream, bool with_lo = false);
  bool fold_ok(const Slab& s, int k) const;
  void maybe_inject_fault();
  void sync_all();
  bool drain(double limit_s);                  // bounded stream drain (teardown after an abort)
  [[noreturn]] void poison(const std::string& why);  // watchdog escalation, then throw
  void finish_residual();
  void run_graph(int64_t pairs, int k);
  int max_depth() const;  // deepest fused depth every slab runs (the prepared graphs' depth)
  // depth of the next sweep of a `len`-step stretch (ending at a residual step if res_end), and in
  // *graphable how many sweeps of that depth follow back to back without a residual
  int plan_sweep(int64_t len, bool res_end, int64_t* graphable) const;
  double sweep_cost(int k) const;  // relative time of a k-step sweep
  SweepCosts sweep_costs() const;  // the plan's inputs: max_depth(), sweep_cost(k), depth_ok_
  void capture_graph(int parity, int k);
  void count_wait_nodes(void* graph);  // StepStats::graph_wait_nodes / graph_fold_waits of a capture
  void destroy_graph();

  StencilSpec spec_;
  Extent3 global_;
  int nranks_;
  PencilDecomposition decomp_;  // pz x py subdomains (py = 1: slabs)
  std::vector<Slab> slabs_;
  std::unique_ptr<Transport> transport_;
  SolverOptions opt_;
  int cur_ = 0;
  StepStats stats_;
  PhaseStats phases_;
  void* pev_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // timing events (slab 0)
  bool ghosts_dirty_ = false;
  // overlapped schedule: the interior sweep of a step waits for the SAME step's boundary kernels
  // instead of the previous step's, so the short boundary launch gets the whole device before the
  // long interior sweep takes every CU; the exchange still runs under the interior (rank proxy
  // N = 8 1,833 vs 1,759 GCells/s per GPU, N = 4 2,058 vs 1,816: profiles/archive/r03_session_p/; the
  // other order was removed in round 4). With one slab per process and a transport whose exchange
  // is pure stream work, the boundary kernels run on the compute stream ahead of the interior and
  // only the exchange on the halo stream (boundary_on_cs).
  bool boundary_on_cs() const;
  int min_rounds() const;  // effective rounds per streaming sweep (RegionArgs::min_rounds)
  bool poisoned_ = false;  // the watchdog aborted the transport: no further steps, bounded teardown
  bool capturing_ = false;  // capture_graph() is recording steps (no folded boundary inside a graph)
  // hipGraphExec_t of the 2-sweep cycle starting at buffer p (index p), and its fused depth
  void* graph_exec_[2] = {nullptr, nullptr};
  int graph_k_[2] = {0, 0};
  // depth_ok_[k]: every slab can run a k-step fused sweep (k <= temporal); 1 always can
  bool depth_ok_[17] = {false, true};
};

}  // namespace mdfx
