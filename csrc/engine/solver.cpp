// mdfx engine implementation (see solver.hpp for the schedule).
#include "mdfx/solver.hpp"
#include "mdfx/sweep_plan.hpp"

#include <dirent.h>
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <sys/stat.h>
#include <string>
#include <thread>
#include <vector>

#include "mdfx/devsync.hpp"

namespace mdfx {

#define HIPC(x)                                                                          \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("HIP: ") + #x + " -> " + hipGetErrorString(e_)); \
  } while (0)

Solver::Solver(const StencilSpec& spec, Extent3 global, int nranks, std::vector<int> local_ranks,
               std::vector<std::unique_ptr<Backend>> backends, std::unique_ptr<Transport> transport,
               SolverOptions opt)
    : spec_(spec), global_(global), nranks_(nranks), transport_(std::move(transport)), opt_(opt) {
  MDFX_CHECK(!local_ranks.empty(), "a process must own at least one slab");
  MDFX_CHECK(local_ranks.size() == backends.size(), "one backend per local slab");
  MDFX_CHECK(transport_ != nullptr, "transport required");
  if (stencil_is_2d(spec_.kind))
    MDFX_CHECK(global_.ny == 1, "2D stencils store an h x w grid as nx=w, ny=1, nz=h");
  else
    MDFX_CHECK(global_.ny >= 1, "bad ny");
  if (spec_.kind == StencilKind::Life) MDFX_CHECK(spec_.dtype == DType::U8, "life cells are u8");
  if (spec_.kind != StencilKind::Life)
    MDFX_CHECK(spec_.dtype == DType::F32 || spec_.dtype == DType::F64, "stencil dtype must be f32 or f64");
  MDFX_CHECK(opt_.temporal >= 1 && opt_.temporal <= 16, "temporal blocking depth must be 1..16");
  MDFX_CHECK(opt_.py >= 1 && nranks % opt_.py == 0,
             format("%d ranks do not form a grid of pencils with %d along y", nranks, opt_.py));
  MDFX_CHECK(opt_.py == 1 || !stencil_is_2d(spec_.kind), "pencil decompositions split 3D grids (y); 2D grids split rows");
  decomp_ = PencilDecomposition(global_, nranks / opt_.py, opt_.py);
  // several slabs: leave room in each interior sweep for the halo exchange's kernels
  if (!backends.empty() && backends[0]->kind() == DeviceKind::HIP) {
    // a fresh engine starts with the device waits armed (a poisoned predecessor may have raised them)
    hip_set_abort(0);
    hip_clear_wait_error();
  }
  const int halo = opt_.temporal;
  for (size_t i = 0; i < local_ranks.size(); ++i) {
    const int r = local_ranks[i];
    MDFX_CHECK(r >= 0 && r < nranks, format("local rank %d outside [0,%d)", r, nranks));
    Slab s;
    s.rank = r;
    s.be = std::move(backends[i]);
    const int rz = decomp_.rz(r), ry = decomp_.ry(r);
    s.lay = FieldLayout::make(global_, decomp_.z.z0(rz), decomp_.z.z1(rz), halo, spec_.dtype, decomp_.y.z0(ry),
                              decomp_.y.z1(ry), opt_.py > 1 ? halo : 0);
    MDFX_CHECK(s.lay.nzl() >= 1, "every slab needs at least one plane");
    MDFX_CHECK(opt_.py == 1 || s.lay.nyl() >= halo,
               format("pencil %d has %lld rows, fewer than the %d ghost rows temporal blocking exchanges", r,
                      (long long)s.lay.nyl(), halo));
    MDFX_CHECK(decomp_.pz() == 1 || s.lay.nzl() >= halo,
               format("slab %d has %lld planes, fewer than the %d ghost planes temporal blocking exchanges "
                      "(use a smaller --temporal or fewer ranks)",
                      r, (long long)s.lay.nzl(), halo));
    const size_t bytes = s.lay.bytes();
    s.buf[0] = s.be->alloc(bytes);
    s.buf[1] = s.be->alloc(bytes);
    s.be->memset(s.buf[0], 0, bytes, nullptr);
    s.be->memset(s.buf[1], 0, bytes, nullptr);
    s.hs = s.be->create_stream(1);
    s.cs = s.be->create_stream(0);
    s.ev_bnd = s.be->create_event();
    s.ev_int = s.be->create_event();
    s.ev_x = s.be->create_event();
    s.ev_x2 = s.be->create_event();
    s.resid = (double*)s.be->alloc(2 * sizeof(double));
    if (s.be->kind() == DeviceKind::HIP && opt_.py == 1 && local_ranks.size() == 1) {
      s.be->activate();
      s.sig = (unsigned long long*)hip_alloc_uncached(128 * 8);
    }
    for (int kk = 2; kk <= opt_.temporal; ++kk) {
      const bool ok = s.be->kind() != DeviceKind::HIP || hip_supports_steps(spec_, s.lay, kk);
      depth_ok_[kk] = (i == 0 ? true : depth_ok_[kk]) && ok;
    }
    if (opt_.temporal > 1 && s.be->kind() == DeviceKind::HIP)
      MDFX_CHECK(hip_supports_steps(spec_, s.lay, opt_.temporal),
                 format("no fused %d-step kernel for %s %s with nx=%lld (fused depths: 2 for every stencil "
                        "(box27 rows up to 1024 fp32 / 512 fp64); 3, 4, 5 for the 3D 7-point; 3, 4, 6, 8 for the 2D stencils, "
                        "also 12, 16 for Life; pencils: 3, 4 fp32 / 3 fp64 for the 3D 7-point only)",
                        opt_.temporal, stencil_name(spec_.kind), dtype_name(spec_.dtype), (long long)global_.nx));
    // regions (storage planes); owned = [halo, halo + nzl). The boundary regions are the `halo`
    // planes at each end that the exchange sends: they are computed on the halo stream so the
    // exchange can follow them in stream order; everything else is interior.
    const int64_t ob = halo, oe = halo + s.lay.nzl();
    const bool has_lo = decomp_.neighbor(r, 0) >= 0, has_hi = decomp_.neighbor(r, 1) >= 0;
    s.lo_b = ob;
    s.lo_e = has_lo ? std::min(ob + halo, oe) : ob;
    s.hi_e = oe;
    s.hi_b = has_hi ? std::max(oe - halo, s.lo_e) : oe;
    s.in_b = s.lo_e;
    s.in_e = s.hi_b;
    if (opt_.py > 1) {
      // the interior planes' rows next to a y neighbour are boundary strips too (the exchange
      // sends them); the rest is interior
      const int64_t yb = s.lay.hy, ye = s.lay.hy + s.lay.nyl();
      s.ylo_b = yb;
      s.ylo_e = decomp_.neighbor(r, 2) >= 0 ? std::min(yb + halo, ye) : yb;
      s.yhi_e = ye;
      s.yhi_b = decomp_.neighbor(r, 3) >= 0 ? std::max(ye - halo, s.ylo_e) : ye;
      s.yin_b = s.ylo_e;
      s.yin_e = s.yhi_b;
    }
    slabs_.push_back(std::move(s));
  }
  for (auto& s : slabs_) s.be->sync_device();
  if (slabs_[0].be->kind() == DeviceKind::HIP) {
    slabs_[0].be->activate();
    for (auto& e : pev_) HIPC(hipEventCreate((hipEvent_t*)&e));
  }
  std::vector<LocalSlab> ls;
  for (auto& s : slabs_) {
    LocalSlab l;
    l.rank = s.rank;
    l.py = opt_.py;
    l.be = s.be.get();
    l.halo_stream = s.hs;
    l.bnd_event = s.ev_bnd;
    l.ghost_event = s.ev_x;
    l.ghost_event2 = s.ev_x2;
    l.lay = s.lay;
    l.buf[0] = s.buf[0];
    l.buf[1] = s.buf[1];
    ls.push_back(l);
  }
  transport_->set_timeout(opt_.timeout_s);
  transport_->setup(ls, nranks_);
}

Solver::~Solver() {
  if (poisoned_) {
    // the watchdog fired: the transport was aborted and the device waits released, so the streams
    // should drain; if they do not within a bound, leak everything rather than hang the exit
    bool drained = false;
    try {
      drained = drain(10.0);
    } catch (...) {
    }
    if (!drained) {
      (void)transport_.release();
      return;
    }
  } else {
    try {
      sync_all();
    } catch (...) {
    }
  }
  destroy_graph();
  transport_.reset();  // communicators before the memory they reference
  for (auto& e : pev_)
    if (e) (void)hipEventDestroy((hipEvent_t)e);
  for (auto& s : slabs_) {
    s.be->release(s.buf[0]);
    s.be->release(s.buf[1]);
    s.be->release(s.resid);
    if (s.sig) {
      s.be->activate();
      hip_free_uncached(s.sig);
    }
    s.be->destroy_event(s.ev_bnd);
    s.be->destroy_event(s.ev_int);
    s.be->destroy_event(s.ev_x);
    s.be->destroy_event(s.ev_x2);
    s.be->destroy_stream(s.hs);
    s.be->destroy_stream(s.cs);
  }
}

void Solver::set_options(const SolverOptions& o) {
  if (o.graph != opt_.graph || o.overlap != opt_.overlap || o.min_rounds != opt_.min_rounds || o.fold != opt_.fold)
    destroy_graph();
  // a different overlap mode switches the schedule (boundary_on_cs), whose steps wait on events the
  // other schedule never records (ev_x) or stops recording (ev_int): drain the queued steps first
  if (o.overlap != opt_.overlap || o.fold != opt_.fold) sync_all();
  MDFX_CHECK(o.temporal == opt_.temporal, "the temporal blocking depth is fixed at construction");
  opt_ = o;
  transport_->set_timeout(opt_.timeout_s);
}

void Solver::init(const InitSpec& is) {
  // captured cycles stay valid: init rewrites the buffers in place, it does not move them
  for (auto& s : slabs_) {
    s.be->init(is, s.lay, s.buf[0], s.hs);
    s.be->init(is, s.lay, s.buf[1], s.hs);
  }
  sync_all();
  cur_ = 0;
  const int64_t caps = stats_.graph_captures;
  stats_ = StepStats();
  stats_.graph_captures = caps;
  ghosts_dirty_ = false;  // ghosts are generated from the global index too
}

void Solver::sync_all() {
  for (auto& s : slabs_) {
    s.be->activate();
    s.be->sync_stream(s.hs);
    s.be->sync_stream(s.cs);
  }
}

bool Solver::drain(double limit_s) {
  if (slabs_[0].be->kind() != DeviceKind::HIP) return true;
  const auto t0 = std::chrono::steady_clock::now();
  for (auto& s : slabs_) {
    s.be->activate();
    for (void* st : {s.hs, s.cs}) {
      for (;;) {
        const hipError_t q = hipStreamQuery((hipStream_t)st);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return false;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s) return false;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
      }
    }
  }
  return true;
}

void Solver::poison(const std::string& why) {
  poisoned_ = true;
  std::fprintf(stderr, "[mdfx] %s: aborting the transport and releasing device waits\n", why.c_str());
  // what the device waits were waiting for: the fold counters of each slab and the transport's
  // protocol counters (bounded copies on private streams; the stuck streams are not involved)
  try {
    for (auto& s : slabs_) {
      if (!s.sig || s.be->kind() != DeviceKind::HIP) continue;
      s.be->activate();
      unsigned long long v[96] = {0};
      if (hip_read_words(v, s.sig, sizeof(v), 2.0))
        std::fprintf(stderr,
                     "[mdfx] rank %d fold counters: upper launch arrivals %llu signals %llu expected %llu; interior "
                     "arrivals %llu signals %llu expected %llu\n",
                     s.rank, v[0], v[16], v[64], v[32], v[48], v[80]);
    }
    const std::string ts = transport_->debug_state();
    if (!ts.empty()) std::fprintf(stderr, "[mdfx] %s\n", ts.c_str());
  } catch (...) {
  }
  std::fflush(stderr);
  try {
    transport_->abort();
  } catch (...) {
  }
  if (slabs_[0].be->kind() == DeviceKind::HIP) hip_set_abort(1);
  MDFX_FAIL(why);
}

void Solver::synchronize() {
  MDFX_CHECK(!poisoned_, "the engine was aborted by its watchdog; create a new Simulation");
  if (opt_.timeout_s <= 0 || slabs_[0].be->kind() != DeviceKind::HIP) {
    sync_all();
    transport_->check();
    return;
  }
  // watchdog: poll the streams and the transport's error state instead of blocking forever (the
  // reference hangs in MPI_Send). On timeout the transport is aborted (ncclCommAbort /
  // the device abort word), so the process can report and exit instead of hanging in teardown.
  const auto t0 = std::chrono::steady_clock::now();
  for (auto& s : slabs_) {
    s.be->activate();
    for (void* st : {s.hs, s.cs}) {
      for (;;) {
        const hipError_t q = hipStreamQuery((hipStream_t)st);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIPC(q);
        try {
          transport_->check();
        } catch (const Error& e) {
          poison(e.what());
        }
        const double el =
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (el > opt_.timeout_s)
          poison(format("watchdog: step stream of rank %d not done after %.1f s", s.rank, el));
        // 20 us polls: the timed bench loop ends within 20 us of the GPU (6.5 ms for 50 steps at N = 8)
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
  }
  transport_->check();
}

void Solver::exchange_ghosts() {
  // make the current buffer's owned planes visible to the exchange (ordered on the halo stream)
  for (auto& s : slabs_) {
    s.be->record(s.ev_int, opt_.overlap ? s.cs : s.hs);
    s.be->wait(s.hs, s.ev_int);
    s.be->record(s.ev_bnd, s.hs);
  }
  transport_->exchange(cur_);
  synchronize();
  ghosts_dirty_ = false;
}

// Boundary kernels on the compute stream: the step is then boundary -> interior on ONE stream (no
// cross-stream event gap between them, measured 10-13 us each at the N = 8 slab shape, where a
// 4-step sweep takes about 0.3 ms), and the exchange alone on the halo stream, after the boundary
// kernels' event and overlapping the interior sweep. The next step's boundary kernels wait for that
// exchange (ev_x): its ghosts are their input. (The ipc / proxy transports record ev_x / ev_x2 right
// after their two pulls, ahead of their pulled signals and waits: 45 -> 26 -> ~20 us from the end of
// the pulls to the next boundary launch at the N = 8 proxy, profiles/r05_session_{ad,ae}/. The faces
// it sent are overwritten only by the sweep after next, after this exchange on the halo stream.)
// Only for one slab per process (the production layout; 8 slabs in one process ran 1936 vs 2023
// GCells/s with it, rank proxies N = 8 / 4 / 2 1850 / 2073 / 2284 vs 1824 / 2069 / 2259,
// profiles/archive/r03_session_x/) and transports whose exchange is pure stream work on the halo stream
// (a host-side exchange synchronises the halo stream alone).
// Rounds of resident blocks per streaming sweep: the option, else 2 with several slabs (exchange
// kernels that need CUs find some mid-sweep) and 1 for a single slab. Passed with every launch
// (RegionArgs::min_rounds), so eager steps, warm-up launches and captured cycles agree.
// Fold the lower boundary region into the interior sweep (one slab per process with the boundary
// kernels on the compute stream, a lower neighbour, fused sweeps through heat7_wxk): instead of a
// separate launch over both K-plane boundary regions (each needing 3K planes marched for K outputs,
// in two rounds of blocks), the interior sweep starts at the lower boundary, signals a device counter
// once those planes are stored, and the halo stream waits for that counter; only the upper region
// keeps its launch (one round). (Round 4's switch back to two launches was removed in round 5; the
// two-launch schedule measured 6-9 % slower at the N = 8 proxy, profiles/r04_session_{i,k}/.)
bool Solver::fold_ok(const Slab& s, int k) const {
  return fold_allowed(opt_.fold, transport_->fold_by_default()) && s.sig && s.lo_e > s.lo_b && s.in_e > s.in_b && hip_region_signals(spec_, s.lay, k);
}

int Solver::min_rounds() const { return opt_.min_rounds > 0 ? opt_.min_rounds : (nranks_ > 1 ? 2 : 1); }

const char* step_schedule(bool overlap, size_t local_slabs, bool stream_ordered, bool fold) {
  if (!overlap) return "serialised";
  if (local_slabs != 1 || !stream_ordered) return "two-stream";
  return fold ? "folded" : "boundary-on-compute";
}

int hip_interval_depth(const StencilSpec& spec, Extent3 g, int want, int64_t residual_every, int nranks) {
  if (want <= 2 || residual_every <= 0) return want;
  SweepCosts c;
  c.T = std::min(want, 16);
  const FieldLayout lay = FieldLayout::make(g, 0, g.nz, want, spec.dtype);
  for (int k = 1; k <= c.T; ++k) {
    c.cost[k] = hip_sweep_cost(spec, g.nx, k);
    c.ok[k] = k == 1 || hip_supports_steps(spec, lay, k);
  }
  return interval_depth(c, residual_every, nranks > 1);
}

bool Solver::boundary_on_cs() const {
  return opt_.overlap && slabs_.size() == 1 && transport_->stream_ordered();
}

std::string Solver::schedule() const {
  const bool fold = boundary_on_cs() && fold_ok(slabs_[0], max_depth());  // (eager steps; captures never fold)
  return step_schedule(opt_.overlap, slabs_.size(), transport_->stream_ordered(), fold);
}

// The boundary regions of a step: the `halo` planes at each z face with a neighbour (all owned
// rows), and for a pencil the `halo` rows at each y face with a neighbour (interior planes).
// Everything the exchange sends is written here.
void Solver::boundary_kernels(Slab& s, RegionArgs a, void* stream, bool skip_lo) {
  if (skip_lo) {
    // the lower region is folded into the interior sweep (fold_ok); the upper region's launch
    // signals the same device counter once its planes are stored (no event between the two launches)
    if (s.hi_e > s.hi_b) {
      a.lz_begin = s.hi_b;
      a.lz_end = s.hi_e;
      a.sig = s.sig;  // (its own counter block: never shared with the interior sweep's)
      a.sig_z = s.hi_e;
      s.be->stencil(spec_, a, stream);
    }
    return;
  }
  if (s.lo_e > s.lo_b && s.hi_e > s.hi_b) {
    // both z boundary regions in one call (one launch where the kernel supports it)
    a.lz_begin = s.lo_b;
    a.lz_end = s.lo_e;
    a.lz2_begin = s.hi_b;
    a.lz2_end = s.hi_e;
    s.be->stencil(spec_, a, stream);
    a.lz2_begin = a.lz2_end = 0;
  } else if (s.lo_e > s.lo_b) {
    a.lz_begin = s.lo_b;
    a.lz_end = s.lo_e;
    s.be->stencil(spec_, a, stream);
  } else if (s.hi_e > s.hi_b) {
    a.lz_begin = s.hi_b;
    a.lz_end = s.hi_e;
    s.be->stencil(spec_, a, stream);
  }
  if (s.in_e > s.in_b) {
    a.lz_begin = s.in_b;
    a.lz_end = s.in_e;
    for (const auto& yr : {std::make_pair(s.ylo_b, s.ylo_e), std::make_pair(s.yhi_b, s.yhi_e)}) {
      if (yr.second <= yr.first) continue;
      a.ly_begin = yr.first;
      a.ly_end = yr.second;
      s.be->stencil(spec_, a, stream);
    }
  }
}

// The interior region: interior planes, and for a pencil its interior rows.
void Solver::interior_kernel(Slab& s, RegionArgs a, void* stream, bool with_lo) {
  if (with_lo) {
    // folded lower boundary: one upward sweep over [lo_b, in_e) that signals once [lo_b, lo_e) is stored
    a.lz_begin = s.lo_b;
    a.lz_end = s.in_e;
    a.lz2_begin = a.lz2_end = 0;
    a.sig = s.sig + 32;
    a.sig_z = s.lo_e;
    s.be->stencil(spec_, a, stream);
    return;
  }
  if (s.in_e <= s.in_b) return;
  a.lz_begin = s.in_b;
  a.lz_end = s.in_e;
  a.lz2_begin = a.lz2_end = 0;
  if (opt_.py > 1) {
    if (s.yin_e <= s.yin_b) return;
    a.ly_begin = s.yin_b;
    a.ly_end = s.yin_e;
  }
  s.be->stencil(spec_, a, stream);
}

void Solver::step(bool want_resid, int k) {
  const int nb = 1 - cur_;
  const bool bcs = boundary_on_cs();
  const bool prof = opt_.profile;
  const bool prof_hip = prof && pev_[0] != nullptr;
  using clk = std::chrono::steady_clock;
  clk::time_point c0, c1, c2, c3;
  if (prof && !prof_hip) c0 = clk::now();
  for (auto& s : slabs_) {
    const bool p0 = prof_hip && &s == &slabs_[0];
    s.be->activate();
    s.be->trace_push("mdfx.step");
    RegionArgs a;
    a.in = s.buf[cur_];
    a.out = s.buf[nb];
    a.lay = s.lay;
    a.steps = k;
    a.min_rounds = min_rounds();
    void* bs = bcs ? s.cs : s.hs;  // the boundary kernels' stream
    if (want_resid) {
      s.be->memset(s.resid, 0, sizeof(double), bs);
      s.be->memset(s.resid + 1, 0, sizeof(double), opt_.overlap ? s.cs : s.hs);
    }
    // boundary planes of this step, after the previous interior sweep (same stream with bcs) and,
    // with bcs, after the previous exchange
    // (a single slab has no neighbour: its exchange moves nothing and the compute stream waits on
    // nothing; the cross-stream event wait alone put ~12 us between consecutive N = 1 sweeps,
    // profiles/r05_session_g2/prof_driver_kernel_trace.csv)
    // (never inside a capture: the folded exchange is ordered after the interior sweep's stores by a
    // device spin wait alone, with no graph edge, so a replay that put the wait node on a queue ahead
    // of the sweep could spin until the watchdog; captured cycles use the boundary launch + event)
    const bool fold = bcs && !capturing_ && fold_ok(s, k);
    // folded, with per-pull ghost events: the upper boundary launch reads only the upper ghosts
    // (ev_x2, after the hi side's pull; a folded slab holds a lower region, an interior plane and
    // the upper region, so that launch's inputs start above the lower ghosts) and the interior the
    // lower ones (ev_x). (With one neighbour both events follow its pull.) At the N = 8 proxy, whose
    // two pulls end together, this measured neutral (2,073-2,098 vs 2,050-2,128 GCells/s interleaved,
    // profiles/r05_session_al/); it matters when one neighbour's face lands late. (Round 6: the upper
    // launch waiting for both instead saves the 6-7 us between the two launches but lost 4 % at the
    // N = 4 proxy, profiles/r06_session_g/.)
    const bool split = fold && nranks_ > 1 && transport_->records_ghost_event();
    if (bcs) {
      if (nranks_ > 1) {
        if (!split) s.be->wait(s.cs, s.ev_x);
        if (transport_->records_ghost_event()) s.be->wait(s.cs, s.ev_x2);
      }
    } else {
      s.be->wait(s.hs, s.ev_int);
    }
    if (p0) HIPC(hipEventRecord((hipEvent_t)pev_[0], (hipStream_t)bs));
    a.resid = want_resid ? s.resid : nullptr;
    if (fold) ++stats_.folded_sweeps;
    boundary_kernels(s, a, bs, fold);
    if (p0) HIPC(hipEventRecord((hipEvent_t)pev_[1], (hipStream_t)bs));
    if (opt_.sync_debug) s.be->sync_device();
    if (prof && !prof_hip && &s == &slabs_[0]) c1 = clk::now();
    // compute stream: interior, after the previous step's boundary kernels
    void* is = opt_.overlap ? s.cs : s.hs;
    if (bcs && !fold) {
      s.be->record(s.ev_bnd, s.cs);  // this step's boundary kernels: the exchange follows them
      s.be->wait(s.hs, s.ev_bnd);
    } else if (!bcs && opt_.overlap) {
      s.be->record(s.ev_bnd, s.hs);  // this step's boundary kernels (the interior waits for them)
      s.be->wait(s.cs, s.ev_bnd);
    }
    if (p0) HIPC(hipEventRecord((hipEvent_t)pev_[2], (hipStream_t)is));
    a.resid = want_resid ? s.resid + 1 : nullptr;
    if (split) s.be->wait(is, s.ev_x);
    interior_kernel(s, a, is, fold);
    // the exchange sends the faces once the upper boundary launch and the interior sweep have
    // signalled them stored (in that order: both launches are on the compute stream). Folded steps
    // need no boundary event: the interior's signal also orders the exchange, which rewrites the
    // ghosts of `nb`, after the previous step's kernels that read them.
    if (fold) {
      const double to = opt_.timeout_s > 0 ? opt_.timeout_s : 300.0;
      if (s.hi_e > s.hi_b)
        hip_counter_wait((const uint64_t*)(s.sig + 16), (uint64_t*)(s.sig + 64), to, s.hs, 0, nullptr);
      hip_counter_wait((const uint64_t*)(s.sig + 48), (uint64_t*)(s.sig + 80), to, s.hs, 0, nullptr);
    }
    if (p0) HIPC(hipEventRecord((hipEvent_t)pev_[3], (hipStream_t)is));
    if (prof && !prof_hip && &s == &slabs_[0]) c2 = clk::now();
    if (!bcs) {
      s.be->record(s.ev_bnd, s.hs);
      s.be->record(s.ev_int, is);  // (with bcs nothing in the step loop waits for it: no marker between sweeps)
    }
    if (opt_.sync_debug) s.be->sync_device();
    s.be->trace_pop();
  }
  if (!slabs_.empty()) slabs_[0].be->trace_push("mdfx.exchange");
  transport_->exchange(nb);
  if (!slabs_.empty()) slabs_[0].be->trace_pop();
  if (bcs && nranks_ > 1 && !transport_->records_ghost_event())
    for (auto& s : slabs_) s.be->record(s.ev_x, s.hs);
  if (prof_hip) {
    Slab& s0 = slabs_[0];
    s0.be->activate();
    HIPC(hipEventRecord((hipEvent_t)pev_[4], (hipStream_t)s0.hs));
    HIPC(hipEventSynchronize((hipEvent_t)pev_[4]));
    HIPC(hipEventSynchronize((hipEvent_t)pev_[3]));
    float b = 0, i = 0, x = 0, t1 = 0, t2 = 0;
    HIPC(hipEventElapsedTime(&b, (hipEvent_t)pev_[0], (hipEvent_t)pev_[1]));
    HIPC(hipEventElapsedTime(&i, (hipEvent_t)pev_[2], (hipEvent_t)pev_[3]));
    HIPC(hipEventElapsedTime(&x, (hipEvent_t)pev_[1], (hipEvent_t)pev_[4]));
    HIPC(hipEventElapsedTime(&t1, (hipEvent_t)pev_[0], (hipEvent_t)pev_[4]));
    HIPC(hipEventElapsedTime(&t2, (hipEvent_t)pev_[0], (hipEvent_t)pev_[3]));
    phases_.boundary_ms += b;
    phases_.interior_ms += i;
    phases_.exchange_ms += x;
    phases_.step_ms += std::max(t1, t2);
    phases_.exposed_ms += std::max(0.0f, t1 - t2);
    ++phases_.steps;
  } else if (prof) {
    c3 = clk::now();
    auto ms = [](clk::time_point a, clk::time_point b) {
      return std::chrono::duration<double, std::milli>(b - a).count();
    };
    phases_.boundary_ms += ms(c0, c1);
    phases_.interior_ms += ms(c1, c2);
    phases_.exchange_ms += ms(c2, c3);
    phases_.step_ms += ms(c0, c3);
    ++phases_.steps;
  }
  if (opt_.sync_debug) sync_all();
  cur_ = nb;
  stats_.steps += k;
  if (want_resid) finish_residual();
}

void Solver::finish_residual() {
  synchronize();  // polled under the watchdog: a hung peer must not block the residual forever
  double local = 0.0;
  for (auto& s : slabs_) {
    double h[2] = {0, 0};
    s.be->copy(h, s.resid, 2 * sizeof(double), CopyKind::D2H, s.hs);
    s.be->sync_stream(s.hs);
    local += h[0] + h[1];
  }
  double g = 0.0;
  try {
    g = transport_->allreduce_sum(local);
  } catch (const Error& e) {
    poison(e.what());
  }
  stats_.last_residual = std::sqrt(g);
  stats_.residual_step = stats_.steps;
  if (!std::isfinite(stats_.last_residual))
    MDFX_FAIL(format("non-finite residual at step %lld: the solution diverged (unstable coefficient?)",
                     (long long)stats_.steps));
}

// Fault injection for failure-detection tests: MDFX_FAULT=<kind>@<rank>:<step> with kind
// exit (the process dies), hang (it stops responding) or nan (a NaN is written into its slab);
// fires once, when the slab <rank> of this process reaches time step <step>.
namespace {
struct Fault {
  std::string kind;
  int rank = -1;
  int64_t step = -1;
  bool fired = false;
};
Fault& fault() {
  static Fault f = [] {
    Fault x;
    const char* v = std::getenv("MDFX_FAULT");
    if (v && *v) {
      char kind[16] = {0};
      long long st = -1;
      int rk = -1;
      if (std::sscanf(v, "%15[a-z]@%d:%lld", kind, &rk, &st) == 3) {
        x.kind = kind;
        x.rank = rk;
        x.step = st;
      }
    }
    return x;
  }();
  return f;
}
}  // namespace

void Solver::maybe_inject_fault() {
  Fault& f = fault();
  if (f.fired || f.rank < 0 || stats_.steps < f.step) return;
  for (int i = 0; i < num_local(); ++i) {
    if (slabs_[i].rank != f.rank) continue;
    f.fired = true;
    std::fprintf(stderr, "[mdfx] injecting fault '%s' on rank %d at step %lld\n", f.kind.c_str(), f.rank,
                 (long long)stats_.steps);
    std::fflush(stderr);
    if (f.kind == "exit") std::_Exit(42);
    if (f.kind == "hang")
      for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
    if (f.kind == "spin") {  // a device kernel that stops making progress (60 s bound)
      if (slabs_[i].be->kind() == DeviceKind::HIP) {
        slabs_[i].be->activate();
        hip_spin(60.0, slabs_[i].cs);
      } else {
        for (;;) std::this_thread::sleep_for(std::chrono::seconds(1));
      }
    }
    if (f.kind == "nan") {
      Slab& s = slabs_[i];
      sync_all();
      const size_t es = s.lay.esize();
      std::vector<char> v(es, 0);
      if (spec_.dtype == DType::F32) {
        const float q = std::nanf("");
        std::memcpy(v.data(), &q, es);
      } else if (spec_.dtype == DType::F64) {
        const double q = std::nan("");
        std::memcpy(v.data(), &q, es);
      }
      // an interior cell of the first owned plane (not on the Dirichlet frame)
      const size_t off = ((size_t)s.lay.halo * s.lay.plane + (size_t)(s.lay.hy + std::min<int64_t>(1, s.lay.nyl() - 1)) * s.lay.pitch +
                          (size_t)std::min<int64_t>(1, s.lay.global.nx - 1)) * es;
      s.be->copy((char*)s.buf[cur_] + off, v.data(), es, CopyKind::H2D, s.hs);
      s.be->sync_stream(s.hs);
    }
  }
}

// Whether the loaded HIP runtime captures the multi-slab step (see Solver::run).
static bool multislab_graph_ok() {
  static const bool ok = [] {
    int v = 0;
    return hipRuntimeGetVersion(&v) == hipSuccess && v >= 70200000;
  }();
  return ok;
}

int Solver::max_depth() const {
  for (int kk = std::min(opt_.temporal, 16); kk > 1; --kk)
    if (depth_ok_[kk]) return kk;
  return 1;
}

// Sweep plan of a stretch of `len` steps (plan_next_sweep, csrc/engine/sweep_plan.cpp): max_depth()
// sweeps and a tail of at most 2 max_depth() - 1 steps, the tail cut so that the summed sweep cost
// (hip_sweep_cost: time per sweep of each fused depth, in single-step sweeps) is least. Measured:
// 2048^3 fp64 with a residual every 10 steps at depth 3, 3 + 3 + 3 + 1 754.0 vs an even
// 3 + 3 + 2 + 2 731.9 GCells/s (the single-step sweep runs near the copy roof, the fp64 two-step
// kernel does not; profiles/r04_session_n/), which the cost table reproduces; at depth 4 it picks
// 4 + 3 + 3 over 4 + 4 + 2 (937.6 GCells/s, profiles/r04_session_u/).
double Solver::sweep_cost(int k) const {
  if (k <= 1) return 1.0;
  return slabs_[0].be->kind() == DeviceKind::HIP ? hip_sweep_cost(spec_, global_.nx, k) : 1.0 + 0.05 * (k - 1);
}

SweepCosts Solver::sweep_costs() const {
  SweepCosts c;
  c.T = max_depth();
  for (int k = 1; k <= 16; ++k) {
    c.cost[k] = sweep_cost(k);
    c.ok[k] = depth_ok_[k];
  }
  return c;
}

int Solver::plan_sweep(int64_t len, bool res_end, int64_t* graphable) const {
  return plan_next_sweep(sweep_costs(), len, res_end, graphable);
}

std::vector<std::pair<int, bool>> Solver::sweep_plan(int64_t steps) const {
  return plan_sweeps(sweep_costs(), steps, stats_.steps, opt_.residual_every);
}

void Solver::run(int64_t steps) {
  MDFX_CHECK(steps >= 0, "negative step count");
  MDFX_CHECK(!poisoned_, "the engine was aborted by its watchdog; create a new Simulation");
  if (ghosts_dirty_) exchange_ghosts();
  transport_->check();
  int64_t done = 0;
  while (done < steps) {
    // time steps until the next residual evaluation (inclusive), unbounded if none
    int64_t to_res = steps - done + 1;
    if (opt_.residual_every > 0)
      to_res = ((stats_.steps / opt_.residual_every) + 1) * opt_.residual_every - stats_.steps;
    // a fused sweep may not jump over a residual step: the stretch up to the next residual step (or
    // the end of the run) is cut into sweeps by plan_sweep
    int64_t graphable = 0;
    const int k = plan_sweep(std::min(steps - done, to_res), to_res <= steps - done, &graphable);
    const bool res = (to_res == k);
    // graph replay for plain (non-residual, non-debug) stretches of >= 2 sweeps, when the
    // transport's exchange is pure stream work (rccl, loopback, ipc; the callback / host / tcp
    // transports move data on the host and always run eagerly). Several slabs in one process need
    // a HIP runtime >= 7.2: the 7.0 runtime PyTorch bundles segfaults in hipStreamEndCapture on the
    // multi-slab loopback capture (6 streams with cross-slab event waits), while the identical
    // binary and capture replay bitwise under 7.2 (csrc/tests/test_main.cpp test_graph run against
    // both runtimes: profiles/archive/r02_graph_runtime.txt). One slab per process (the production layout)
    // replays under both.
    // A captured cycle's first exchange sends buffer 1 - cur_; it is replayed only when the exchange
    // before it sent the other parity (a repeated parity needs the ipc transport's eager look-ahead
    // wait, ipc_transport.cpp).
    if (!res && graph_eligible() && transport_->last_parity() != 1 - cur_) {
      const int64_t pairs = graphable / 2;
      if (pairs > 0) {
        run_graph(pairs, k);
        done += 2 * k * pairs;
        continue;
      }
    }
    step(res, k);
    done += k;
    maybe_inject_fault();
  }
}

// ---- hipGraph replay of a 2-step cycle --------------------------------------------------------
// Captured from the halo stream of slab 0; every other stream joins the capture through event
// waits (fork) and is joined back at the end, so the replay carries exactly the eager schedule's
// dependencies. graph_exec_[p] is the cycle that starts at buffer p; both are kept until an option
// change alters the captured work (init() rewrites the buffers in place and keeps them).
void Solver::destroy_graph() {
  for (int p = 0; p < 2; ++p) {
    if (graph_exec_[p]) (void)hipGraphExecDestroy((hipGraphExec_t)graph_exec_[p]);
    graph_exec_[p] = nullptr;
    graph_k_[p] = 0;
  }
}

bool Solver::graph_eligible() const {
  const bool hip = slabs_[0].be->kind() == DeviceKind::HIP;
  return opt_.graph && hip && !opt_.sync_debug && !opt_.profile && transport_->graph_capturable() &&
         (slabs_.size() == 1 || multislab_graph_ok()) && fault().rank < 0 && !poisoned_;
}

void Solver::warm_kernels(int64_t steps) {
  MDFX_CHECK(!poisoned_, "the engine was aborted by its watchdog; create a new Simulation");
  if (slabs_.empty() || slabs_[0].be->kind() != DeviceKind::HIP) return;  // (nothing to warm on the CPU)
  bool used[17][2] = {};
  for (const auto& kr : sweep_plan(steps)) used[kr.first][kr.second ? 1 : 0] = true;
  synchronize();
  const int nb = 1 - cur_;
  for (int k = 1; k <= 16; ++k)
    for (int r = 0; r < 2; ++r) {
      if (!used[k][r]) continue;
      for (auto& s : slabs_) {
        s.be->activate();
        RegionArgs a;
        a.in = s.buf[cur_];
        a.out = s.buf[nb];  // scratch: the next step overwrites it
        a.lay = s.lay;
        a.steps = k;
        a.min_rounds = min_rounds();
        a.resid = r ? s.resid : nullptr;  // (step() clears the accumulator before it counts)
        boundary_kernels(s, a, s.hs);
        interior_kernel(s, a, s.hs);
      }
    }
  synchronize();
}

int Solver::prepare_graphs() {
  MDFX_CHECK(!poisoned_, "the engine was aborted by its watchdog; create a new Simulation");
  if (!graph_eligible()) return 0;
  const int k = max_depth();
  // one eager exchange first (it re-sends the current faces, so it changes nothing): transports
  // that set up peer connections on first use (RCCL p2p) do so outside the capture
  exchange_ghosts();
  const int saved = cur_;
  for (int p = 0; p < 2; ++p) {
    if (graph_exec_[p] && graph_k_[p] == k) continue;
    cur_ = p;
    capture_graph(p, k);
  }
  cur_ = saved;
  // the captures recorded the per-slab events inside the graphs: re-arm them for eager work
  for (auto& s : slabs_) {
    s.be->activate();
    s.be->record(s.ev_bnd, s.hs);
    s.be->record(s.ev_int, s.cs);
    s.be->record(s.ev_x, s.hs);
    s.be->record(s.ev_x2, s.hs);
  }
  return (graph_exec_[0] ? 1 : 0) + (graph_exec_[1] ? 1 : 0);
}

static bool graph_debug() {
  static const bool on = [] {
    const char* v = std::getenv("MDFX_DEBUG_GRAPH");
    return v && *v == '1';
  }();
  return on;
}
#define GDBG(msg)                                                 \
  do {                                                            \
    if (graph_debug()) std::fprintf(stderr, "[mdfx graph] %s\n", msg); \
  } while (0)

// The device spin-wait nodes of a captured graph, and among them those that wait on a slab's own
// fold counters. Solver::step never folds while capturing (a fold wait is ordered after the interior
// sweep by the spin alone, with no graph edge, so a replay that put it on a queue ahead of the sweep
// would spin until the watchdog); this checks the captured graph itself (tests/test_gpu_ipc.py).
void Solver::count_wait_nodes(void* graph) {
  hipGraph_t g = (hipGraph_t)graph;
  size_t n = 0;
  HIPC(hipGraphGetNodes(g, nullptr, &n));
  std::vector<hipGraphNode_t> nodes(n);
  if (n) HIPC(hipGraphGetNodes(g, nodes.data(), &n));
  const void* wk = hip_counter_wait_kernel();
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    HIPC(hipGraphNodeGetType(nodes[i], &t));
    if (t != hipGraphNodeTypeKernel) continue;
    hipKernelNodeParams p{};
    HIPC(hipGraphKernelNodeGetParams(nodes[i], &p));
    if (p.func != wk) continue;
    ++stats_.graph_wait_nodes;
    const uint64_t* remote = p.kernelParams ? *(const uint64_t* const*)p.kernelParams[0] : nullptr;
    for (auto& s : slabs_)
      if (s.sig && remote >= (const uint64_t*)s.sig && remote < (const uint64_t*)(s.sig + 128)) ++stats_.graph_fold_waits;
  }
}

// Capture the cycle starting at buffer `parity` (== cur_): two sweeps of depth k. Nothing runs.
void Solver::capture_graph(int parity, int k) {
  GDBG("capture begin");
  if (graph_exec_[parity]) {
    (void)hipGraphExecDestroy((hipGraphExec_t)graph_exec_[parity]);
    graph_exec_[parity] = nullptr;
  }
  Slab& o = slabs_[0];
  o.be->activate();
  hipStream_t origin = (hipStream_t)o.hs;
  std::vector<hipEvent_t> fork(slabs_.size() * 2), join(slabs_.size() * 2);
  for (auto& e : fork) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : join) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPC(hipStreamBeginCapture(origin, hipStreamCaptureModeRelaxed));
  HIPC(hipEventRecord(fork[0], origin));
  for (auto& s : slabs_) {
    s.be->activate();
    for (void* st : {s.hs, s.cs})
      if (st != (void*)origin) HIPC(hipStreamWaitEvent((hipStream_t)st, fork[0], 0));
  }
  // every event the captured steps wait on must itself be recorded inside the capture
  for (auto& s : slabs_) {
    s.be->activate();
    s.be->record(s.ev_bnd, s.hs);
    s.be->record(s.ev_int, s.cs);
    s.be->record(s.ev_x, s.hs);
    s.be->record(s.ev_x2, s.hs);
  }
  const StepStats saved = stats_;
  GDBG("capture: steps");
  capturing_ = true;
  try {
    step(false, k);
    step(false, k);
  } catch (...) {
    capturing_ = false;
    throw;
  }
  capturing_ = false;
  GDBG("capture: join");
  stats_ = saved;  // replay accounts for them
  ++stats_.graph_captures;
  size_t ei = 0;
  for (auto& s : slabs_) {
    s.be->activate();
    for (void* st : {s.hs, s.cs}) {
      if (st != (void*)origin) {
        HIPC(hipEventRecord(join[ei], (hipStream_t)st));
        o.be->activate();
        HIPC(hipStreamWaitEvent(origin, join[ei], 0));
        s.be->activate();
      }
      ++ei;
    }
  }
  o.be->activate();
  hipGraph_t g;
  GDBG("capture: end");
  HIPC(hipStreamEndCapture(origin, &g));
  count_wait_nodes(g);
  GDBG("instantiate");
  hipGraphExec_t ex;
  HIPC(hipGraphInstantiateWithFlags(&ex, g, 0));
  HIPC(hipGraphDestroy(g));
  for (auto& e : fork) (void)hipEventDestroy(e);
  for (auto& e : join) (void)hipEventDestroy(e);
  graph_exec_[parity] = ex;
  graph_k_[parity] = k;
  MDFX_CHECK(cur_ == parity, "graph capture must leave the buffer parity unchanged");
  GDBG("instantiated");
}

void Solver::run_graph(int64_t pairs, int k) {
  if (!graph_exec_[cur_] || graph_k_[cur_] != k) {
    capture_graph(cur_, k);
    // the capture recorded the per-slab events inside the graph: re-arm them before the launch
    for (auto& s : slabs_) {
      s.be->activate();
      s.be->record(s.ev_bnd, s.hs);
      s.be->record(s.ev_int, s.cs);
      s.be->record(s.ev_x, s.hs);
      s.be->record(s.ev_x2, s.hs);
    }
  }
  GDBG("launch");
  // (the bcs step schedule records no per-step interior event: mark every compute stream's tail now)
  for (auto& s : slabs_) {
    s.be->activate();
    s.be->record(s.ev_int, s.cs);
  }
  Slab& o = slabs_[0];
  o.be->activate();
  // the replay starts after all eager work on every slab's streams
  for (auto& s : slabs_) {
    if (&s == &o) continue;
    o.be->wait(o.hs, s.ev_bnd);
    o.be->wait(o.hs, s.ev_int);
    o.be->wait(o.hs, s.ev_x);
    o.be->wait(o.hs, s.ev_x2);
  }
  o.be->wait(o.hs, o.ev_int);
  for (int64_t i = 0; i < pairs; ++i) HIPC(hipGraphLaunch((hipGraphExec_t)graph_exec_[cur_], (hipStream_t)o.hs));
  // later eager work on the other streams must follow the replay
  HIPC(hipEventRecord((hipEvent_t)o.ev_bnd, (hipStream_t)o.hs));
  for (auto& s : slabs_) {
    s.be->activate();
    if (s.cs != o.hs) HIPC(hipStreamWaitEvent((hipStream_t)s.cs, (hipEvent_t)o.ev_bnd, 0));
    if (s.hs != o.hs) HIPC(hipStreamWaitEvent((hipStream_t)s.hs, (hipEvent_t)o.ev_bnd, 0));
  }
  // re-establish per-slab events for the next eager step
  for (auto& s : slabs_) {
    s.be->activate();
    s.be->record(s.ev_bnd, s.hs);
    s.be->record(s.ev_int, s.cs);
    s.be->record(s.ev_x, s.hs);
    s.be->record(s.ev_x2, s.hs);
  }
  // a replayed cycle ends with the exchange of buffer cur_ (the parity is unchanged)
  transport_->set_last_parity(cur_);
  stats_.steps += 2 * (int64_t)k * pairs;
  stats_.graph_replays += pairs;
  GDBG("replayed");
}

// ---- host I/O ----------------------------------------------------------------------------------

void Solver::read_owned(int i, void* host) {
  Slab& s = slabs_[i];
  sync_all();
  const FieldLayout& l = s.lay;
  const size_t es = l.esize();
  std::vector<char> stage((size_t)l.nzl() * l.plane_bytes());
  s.be->copy(stage.data(), (char*)s.buf[cur_] + (size_t)l.halo * l.plane_bytes(), stage.size(),
             CopyKind::D2H, s.hs);
  s.be->sync_stream(s.hs);
  char* dst = (char*)host;
  for (int64_t z = 0; z < l.nzl(); ++z)
    for (int64_t y = 0; y < l.nyl(); ++y) {
      std::memcpy(dst, stage.data() + ((size_t)z * l.plane + (size_t)(l.hy + y) * l.pitch) * es,
                  (size_t)l.global.nx * es);
      dst += (size_t)l.global.nx * es;
    }
}

void Solver::write_owned(int i, const void* host) {
  Slab& s = slabs_[i];
  sync_all();
  const FieldLayout& l = s.lay;
  const size_t es = l.esize();
  std::vector<char> stage((size_t)l.nzl() * l.plane_bytes(), 0);
  const char* src = (const char*)host;
  for (int64_t z = 0; z < l.nzl(); ++z)
    for (int64_t y = 0; y < l.nyl(); ++y) {
      std::memcpy(stage.data() + ((size_t)z * l.plane + (size_t)(l.hy + y) * l.pitch) * es, src,
                  (size_t)l.global.nx * es);
      src += (size_t)l.global.nx * es;
    }
  s.be->copy((char*)s.buf[cur_] + (size_t)l.halo * l.plane_bytes(), stage.data(), stage.size(),
             CopyKind::H2D, s.hs);
  s.be->sync_stream(s.hs);
  ghosts_dirty_ = true;
}

static void mkdir_p(const std::string& d) {
  std::string cur;
  for (size_t i = 0; i < d.size(); ++i) {
    cur.push_back(d[i]);
    if (d[i] == '/' || i + 1 == d.size()) ::mkdir(cur.c_str(), 0755);
  }
}

void Solver::save_checkpoint(const std::string& dir) {
  mkdir_p(dir);
  for (int i = 0; i < num_local(); ++i) {
    const FieldLayout& l = slabs_[i].lay;
    std::vector<char> data((size_t)l.owned_cells() * l.esize());
    read_owned(i, data.data());
    const std::string base = dir + "/slab_" + std::to_string(slabs_[i].rank);
    {
      std::ofstream f(base + ".bin", std::ios::binary);
      MDFX_CHECK(f.good(), "cannot write " + base + ".bin");
      f.write(data.data(), (std::streamsize)data.size());
    }
    std::ofstream j(base + ".json");
    j << "{\"format\": \"mdfx-slab-v1\", \"stencil\": \"" << stencil_name(spec_.kind) << "\", \"dtype\": \""
      << dtype_name(spec_.dtype) << "\", \"nx\": " << global_.nx << ", \"ny\": " << global_.ny
      << ", \"nz\": " << global_.nz << ", \"z0\": " << l.z0 << ", \"z1\": " << l.z1 << ", \"y0\": " << l.y0
      << ", \"y1\": " << l.y1
      << ", \"rank\": " << slabs_[i].rank << ", \"nranks\": " << nranks_
      << ", \"step\": " << stats_.steps << "}\n";
  }
  // a directory reused by an earlier save with more ranks keeps its extra slabs: remove them so
  // no reader can mix them in (readers also take nranks from slab_0 and check every header)
  bool owns0 = false;
  for (auto& s : slabs_) owns0 = owns0 || s.rank == 0;
  if (owns0) {
    if (DIR* d = ::opendir(dir.c_str())) {
      std::vector<std::string> stale;
      while (dirent* e = ::readdir(d)) {
        int r = -1;
        char ext[8] = {0};
        if (std::sscanf(e->d_name, "slab_%d.%7s", &r, ext) == 2 && r >= nranks_ &&
            (std::strcmp(ext, "bin") == 0 || std::strcmp(ext, "json") == 0))
          stale.push_back(dir + "/" + e->d_name);
      }
      ::closedir(d);
      for (auto& f : stale) ::unlink(f.c_str());
    }
  }
}

static bool json_int(const std::string& s, const std::string& key, long long& out) {
  const std::string k = "\"" + key + "\":";
  size_t p = s.find(k);
  if (p == std::string::npos) return false;
  p += k.size();
  out = std::atoll(s.c_str() + p);
  return true;
}

void Solver::load_checkpoint(const std::string& dir) {
  // slabs written by any decomposition: slab_0 names the writer's rank count, and every one of
  // slab_0 .. slab_<nranks-1> must carry that count and the same step
  struct F {
    long long z0, z1, y0, y1, step;
    std::string bin;
  };
  std::vector<F> files;
  long long writer_ranks = -1, writer_step = -1;
  for (int r = 0; writer_ranks < 0 || r < writer_ranks; ++r) {
    const std::string base = dir + "/slab_" + std::to_string(r);
    std::ifstream j(base + ".json");
    if (!j.good()) {
      MDFX_CHECK(r > 0, "no checkpoint slabs in " + dir);
      MDFX_FAIL(format("checkpoint %s is incomplete: slab_%d.json missing (written by %lld ranks)", dir.c_str(), r,
                       writer_ranks));
    }
    std::stringstream ss;
    ss << j.rdbuf();
    const std::string js = ss.str();
    F f;
    long long nx = 0, ny = 0, nz = 0;
    MDFX_CHECK(json_int(js, "z0", f.z0) && json_int(js, "z1", f.z1) && json_int(js, "step", f.step) &&
                   json_int(js, "nx", nx) && json_int(js, "ny", ny) && json_int(js, "nz", nz),
               "malformed checkpoint header " + base + ".json");
    // (y0 / y1: a pencil's rows; slab checkpoints hold every row)
    if (!json_int(js, "y0", f.y0) || !json_int(js, "y1", f.y1)) {
      f.y0 = 0;
      f.y1 = ny;
    }
    MDFX_CHECK(nx == global_.nx && ny == global_.ny && nz == global_.nz,
               "checkpoint grid does not match the solver grid");
    MDFX_CHECK(js.find(std::string("\"dtype\": \"") + dtype_name(spec_.dtype) + "\"") != std::string::npos,
               "checkpoint dtype does not match");
    long long nr = -1;
    MDFX_CHECK(json_int(js, "nranks", nr) && nr >= 1, "checkpoint header without nranks: " + base + ".json");
    if (r == 0) {
      writer_ranks = nr;
      writer_step = f.step;
    }
    MDFX_CHECK(nr == writer_ranks && f.step == writer_step,
               format("checkpoint slab_%d (nranks %lld, step %lld) does not match slab_0 (nranks %lld, step %lld)", r, nr,
                      f.step, writer_ranks, writer_step));
    f.bin = base + ".bin";
    files.push_back(f);
  }
  MDFX_CHECK(!files.empty(), "no checkpoint slabs in " + dir);
  for (int i = 0; i < num_local(); ++i) {
    const FieldLayout& l = slabs_[i].lay;
    const size_t rb = (size_t)global_.nx * l.esize();  // dense row bytes
    std::vector<char> data((size_t)l.nzl() * l.nyl() * rb);
    std::vector<std::ifstream> ins(files.size());
    for (int64_t z = l.z0; z < l.z1; ++z) {
      // the rows of plane z this slab owns, gathered from every file that holds some of them (any
      // slab or pencil decomposition wrote them)
      int64_t got = 0;
      for (size_t fi = 0; fi < files.size(); ++fi) {
        const F& f = files[fi];
        if (z < f.z0 || z >= f.z1) continue;
        const int64_t ya = std::max<int64_t>(l.y0, f.y0), yb = std::min<int64_t>(l.y1, f.y1);
        if (ya >= yb) continue;
        if (!ins[fi].is_open()) ins[fi].open(f.bin, std::ios::binary);
        ins[fi].seekg((std::streamoff)((((z - f.z0) * (f.y1 - f.y0)) + (ya - f.y0)) * (int64_t)rb));
        ins[fi].read(data.data() + ((size_t)(z - l.z0) * l.nyl() + (size_t)(ya - l.y0)) * rb,
                     (std::streamsize)((yb - ya) * (int64_t)rb));
        MDFX_CHECK(ins[fi].good(), "short read in " + f.bin);
        got += yb - ya;
      }
      MDFX_CHECK(got == l.nyl(), format("checkpoint is missing rows of plane %lld", (long long)z));
    }
    write_owned(i, data.data());
    stats_.steps = files[0].step;
  }
  // owned planes of buffer 1 are stale but are fully rewritten by the next step
  exchange_ghosts();
}

}  // namespace mdfx
