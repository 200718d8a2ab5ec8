// Implementation of the mdfx command line (see cli_common.hpp).
#include "cli_common.hpp"

#include <chrono>
#include <csignal>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "mdfx/bootstrap.hpp"
#include "mdfx/solver.hpp"

namespace mdfx {
namespace {

struct Opts {
  std::string stencil;
  std::string dtype;
  int64_t n = 0, nx = 0, ny = 0, nz = 0, h = 0, w = 0;
  int64_t steps = -1, warmup = 0;
  std::string backend = "auto";
  int gpus = 0, ranks = 0;
  std::string transport = "auto";
  std::string init;
  uint64_t seed = 1;
  double lo = 0, hi = 1, value = 0, edge = 100, interior = 0, density = 0.15;
  double r = -1, c0 = 0.25, c1 = 0.05, c2 = 0.025, c3 = 3.0 / 160.0;
  int residual_every = 0;
  bool print = false, json = false, sync_debug = false, overlap = true, graph = false;
  bool verbose = false, quiet = false, share_gpu = false;
  int fold = -1;  // --fold auto|on|off (SolverOptions::fold)
  std::string variant = "auto";
  double timeout = 0;
  int64_t ckpt_every = 0;
  std::string ckpt_dir = "mdfx_ckpt", resume;
  bool compat = false;
  bool ref_precision = false;
  int temporal = 0;  // 0 = auto: hip_fused_depth on HIP where a fused kernel exists, else 1
  int py = 1;        // --py: ranks along y of a (z, y) pencil split
  bool profile = false;
  int dim = 0;
  std::string dump;
};

void usage(const char* prog) {
  std::printf(
      "usage: %s [options]\n"
      "  With no size/step options the reference dialogue runs on stdin (generations, height, width).\n"
      "  --stencil 5|7|27|life     stencil family (5 = 2D MDF heat/Jacobi, 7 = 3D 7-pt, 27 = 3D 27-pt)\n"
      "  --n N | --nx --ny --nz    3D grid (N^3) ; 2D: --h ROWS --w COLS\n"
      "  --steps K (--iters, -g)   time steps / generations ; --warmup W untimed steps first\n"
      "  --dtype f32|f64           element type (life is always u8)\n"
      "  --backend auto|hip|cpu    device backend\n"
      "  --gpus N                  slabs on GPUs 0..N-1 driven by this one process\n"
      "  --ranks P                 P slabs in this process (several per GPU allowed: loopback)\n"
      "  --py Y                    (z, y) pencils: Y ranks along y, P / Y along z (3D; loopback, host, ipc)\n"
      "  --transport auto|rccl|ipc|ipc_sdma|loopback|host|tcp\n"
      "                            multi-process runs (mpirun / torchrun): rccl on GPUs, tcp on CPUs\n"
      "  --share-gpu               ipc: allow several processes on one GPU (tests; one per GPU otherwise)\n"
      "  --fold auto|on|off        fold the lower boundary into the interior sweep (auto: the transport's\n"
      "                            default - ipc yes, rccl no)\n"
      "  --init random|dirichlet|constant|life|compat  --seed --lo --hi --value --edge --interior --density\n"
      "  --r R | --c0 --c1 --c2 --c3   update coefficients\n"
      "  --ref-precision           2D MDF: the reference's fp32-sum / fp64-scale evaluation of the update\n"
      "                            (default in the reference dialogue; single-step sweeps)\n"
      "  --residual-every K        global L2 norm of the update every K steps\n"
      "  --checkpoint-every K --checkpoint-dir D ; --resume D\n"
      "  --print                   dump the final grid like the reference's print_array\n"
      "  --json                    one JSON metrics line ; --verbose per-rank detail ; --quiet\n"
      "  --no-overlap --sync-debug --graph --variant auto|tuned|naive --timeout S\n"
      "  --temporal 0..16          time steps fused per memory sweep (0 = auto on GPUs: 5 for the\n"
      "                            fp32 3D 7-point and fp64 rows of 2048+ cells (fp64 4 below) where\n"
      "                            heat7_wxk covers the row, 3 for the 27-point in fp64 or at rows of\n"
      "                            1024+ cells, else 2 for 3D; 8 for the 2D MDF, 12 for Life; 1 on the\n"
      "                            CPU; shallower until slabs are 4 sweeps deep, and fitted to the\n"
      "                            --residual-every interval)\n"
      "  --profile                 per-phase timing of rank 0 (boundary / interior / exchange)\n"
      "  --dim 2|3                 default stencil of that dimension (5 / 7) ; --bc V = --edge V ; --coef R = --r R\n"
      "  --dump DIR                write the final grid (per-slab raw + JSON header, checkpoint format)\n"
      "  --trace                   roctx ranges around every phase (rocprofv3 --marker-trace)\n",
      prog);
}

Opts parse(int argc, char** argv, const char* prog) {
  Opts o;
  auto need = [&](int& i) -> const char* {
    if (i + 1 >= argc) MDFX_FAIL(std::string("missing value for ") + argv[i]);
    return argv[++i];
  };
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-h" || a == "--help") {
      usage(prog);
      std::exit(0);
    } else if (a == "--stencil") o.stencil = need(i);
    else if (a == "--dtype") o.dtype = need(i);
    else if (a == "--n") o.n = std::atoll(need(i));
    else if (a == "--nx") o.nx = std::atoll(need(i));
    else if (a == "--ny") o.ny = std::atoll(need(i));
    else if (a == "--nz") o.nz = std::atoll(need(i));
    else if (a == "--h" || a == "--height") o.h = std::atoll(need(i));
    else if (a == "--w" || a == "--width") o.w = std::atoll(need(i));
    else if (a == "--steps" || a == "--iters" || a == "-g" || a == "--generations") o.steps = std::atoll(need(i));
    else if (a == "--warmup") o.warmup = std::atoll(need(i));
    else if (a == "--backend") o.backend = need(i);
    else if (a == "--gpus") o.gpus = std::atoi(need(i));
    else if (a == "--ranks") o.ranks = std::atoi(need(i));
    else if (a == "--transport") o.transport = need(i);
    else if (a == "--share-gpu") o.share_gpu = true;
    else if (a == "--fold") {
      const std::string v = need(i);
      MDFX_CHECK(v == "auto" || v == "on" || v == "off", "--fold takes auto, on or off");
      o.fold = v == "on" ? 1 : v == "off" ? 0 : -1;
    }
    else if (a == "--init") o.init = need(i);
    else if (a == "--seed") o.seed = std::strtoull(need(i), nullptr, 10);
    else if (a == "--lo") o.lo = std::atof(need(i));
    else if (a == "--hi") o.hi = std::atof(need(i));
    else if (a == "--value") o.value = std::atof(need(i));
    else if (a == "--edge" || a == "--bc") o.edge = std::atof(need(i));
    else if (a == "--interior") o.interior = std::atof(need(i));
    else if (a == "--density") o.density = std::atof(need(i));
    else if (a == "--r" || a == "--coef") o.r = std::atof(need(i));
    else if (a == "--c0") o.c0 = std::atof(need(i));
    else if (a == "--c1") o.c1 = std::atof(need(i));
    else if (a == "--c2") o.c2 = std::atof(need(i));
    else if (a == "--c3") o.c3 = std::atof(need(i));
    else if (a == "--residual-every") o.residual_every = std::atoi(need(i));
    else if (a == "--checkpoint-every") o.ckpt_every = std::atoll(need(i));
    else if (a == "--checkpoint-dir") o.ckpt_dir = need(i);
    else if (a == "--resume") o.resume = need(i);
    else if (a == "--print") o.print = true;
    else if (a == "--json") o.json = true;
    else if (a == "--verbose") o.verbose = true;
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--no-overlap") o.overlap = false;
    else if (a == "--sync-debug") o.sync_debug = true;
    else if (a == "--graph") o.graph = true;
    else if (a == "--variant") o.variant = need(i);
    else if (a == "--timeout") o.timeout = std::atof(need(i));
    else if (a == "--compat") o.compat = true;
    else if (a == "--ref-precision") o.ref_precision = true;
    else if (a == "--temporal") o.temporal = std::atoi(need(i));
    else if (a == "--py") o.py = std::atoi(need(i));
    else if (a == "--profile") o.profile = true;
    else if (a == "--dim") o.dim = std::atoi(need(i));
    else if (a == "--dump") o.dump = need(i);
    else if (a == "--trace") setenv("MDFX_TRACE", "1", 1);
    else MDFX_FAIL("unknown option " + a + " (try --help)");
  }
  return o;
}

// print_array (kernel.cu:115-129) over the dense global grid, plane by plane for 3D grids.
template <class T>
void print_rows(const T* v, int64_t rows, int64_t nx) {
  std::printf("\n");
  for (int64_t i = 0; i < rows * nx; ++i) {
    std::fputs(v[i] == (T)1 ? "0" : " ", stdout);
    if ((i + 1) % nx == 0) std::fputs("\n", stdout);
  }
  std::printf("\n");
}

template <class T>
void print_grid(const std::vector<char>& g, int64_t nx, int64_t ny, int64_t nz) {
  const T* v = (const T*)g.data();
  if (ny == 1) {  // 2D: rows are the z axis
    print_rows(v, nz, nx);
    return;
  }
  for (int64_t z = 0; z < nz; ++z) {
    std::printf("z=%lld", (long long)z);
    print_rows(v + z * ny * nx, ny, nx);
  }
}

}  // namespace

int run_cli(int argc, char** argv, const char* default_stencil, const char* prog) {
  // one hardware queue for hipGraph execution (before the HIP runtime starts): see
  // docs/DESIGN.md "hipGraph replay" - the multi-queue graph executor runs a captured cycle's
  // branches 1.4-2x slower than eager launches, one queue matches them
  setenv("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1", 0);
  try {
    Opts o = parse(argc, argv, prog);
    const ProcEnv env = detect_proc_env();
    std::unique_ptr<Rendezvous> rv;
    if (env.world > 1) rv.reset(new Rendezvous(env));
    const bool root = env.rank == 0;
    MDFX_CHECK(o.dim == 0 || o.dim == 2 || o.dim == 3, "--dim is 2 or 3");
    if (o.stencil.empty()) o.stencil = o.dim == 3 ? "7" : (o.dim == 2 ? "5" : default_stencil);
    const StencilKind kind = stencil_from_name(o.stencil);
    const bool is2d = stencil_is_2d(kind);
    MDFX_CHECK(o.dim == 0 || (o.dim == 2) == is2d, "--dim does not match --stencil " + o.stencil);

    // ---- reference dialogue (rank 0 reads, everyone receives) -----------------------------
    const bool sized = o.n || o.nx || o.ny || o.nz || o.h || o.w;
    if (o.compat || (o.steps < 0 && !sized)) {
      o.compat = true;
      std::string cfg;
      if (root) {
        int g = 0, h = 0, w = 0;
        std::printf("Enter desired number of generations:\n");
        std::fflush(stdout);
        if (std::scanf("%d", &g) != 1) MDFX_FAIL("expected an integer number of generations on stdin");
        std::printf("Enter desired height of universe:\n");
        std::fflush(stdout);
        if (std::scanf("%d", &h) != 1) MDFX_FAIL("expected an integer height on stdin");
        std::printf("Enter desired width of universe:\n");
        std::fflush(stdout);
        if (std::scanf("%d", &w) != 1) MDFX_FAIL("expected an integer width on stdin");
        cfg = format("%d %d %d", g, h, w);
      }
      if (rv) cfg = rv->bcast(cfg);
      long long g = 0, h = 0, w = 0;
      std::sscanf(cfg.c_str(), "%lld %lld %lld", &g, &h, &w);
      MDFX_CHECK(g >= 0 && h >= 1 && w >= 1, "generations >= 0, height and width >= 1");
      o.steps = g;
      if (is2d) {
        o.h = h;
        o.w = w;
      } else {  // a 3D stencil from the 2D dialogue: height x width planes, `height` deep
        o.nx = w;
        o.ny = h;
        o.nz = h;
      }
    }
    if (o.steps < 0) o.steps = 100;

    Extent3 g;
    if (is2d) {
      g.nx = o.w ? o.w : (o.nx ? o.nx : (o.n ? o.n : 256));
      g.ny = 1;
      g.nz = o.h ? o.h : (o.nz ? o.nz : (o.n ? o.n : 256));
    } else {
      const int64_t d = o.n ? o.n : 256;
      g.nx = o.nx ? o.nx : d;
      g.ny = o.ny ? o.ny : d;
      g.nz = o.nz ? o.nz : d;
    }
    StencilSpec spec;
    spec.kind = kind;
    spec.dtype = kind == StencilKind::Life ? DType::U8 : dtype_from_name(o.dtype.empty() ? "f32" : o.dtype);
    spec.coef.r = o.r;
    spec.coef.c0 = o.c0;
    spec.coef.c1 = o.c1;
    spec.coef.c2 = o.c2;
    spec.coef.c3 = o.c3;
    // the reference dialogue reproduces the reference's arithmetic too (MDF_kernel.cu:20, D17)
    spec.coef.ref_precision = kind == StencilKind::Jacobi5 && (o.ref_precision || o.compat);
    hip_set_kernel_variant(o.variant.c_str());

    // ---- backend / slabs / transport ------------------------------------------------------
    const int ndev = hip_device_count();
    bool hip = o.backend == "hip" || (o.backend == "auto" && ndev > 0);
    if (o.backend == "cpu") hip = false;
    if (hip) MDFX_CHECK(ndev > 0, "--backend hip but no HIP device is visible");
    int nranks = 1;
    std::vector<int> local_ranks, devices;
    std::string tname = o.transport;
    if (env.world > 1) {
      nranks = env.world;
      local_ranks = {env.rank};
      devices = {hip ? env.local_rank % ndev : -1};
      if (tname == "auto") tname = hip ? "rccl" : "tcp";
    } else {
      nranks = o.ranks ? o.ranks : (o.gpus ? o.gpus : 1);
      for (int r = 0; r < nranks; ++r) {
        local_ranks.push_back(r);
        devices.push_back(hip ? (o.gpus ? r % std::min(o.gpus, ndev) : 0) : -1);
      }
      if (tname == "auto") tname = hip ? ((o.gpus > 1 && !o.ranks) ? "rccl" : "loopback") : "host";
    }
    std::vector<std::unique_ptr<Backend>> bes;
    for (int d : devices) bes.push_back(d < 0 ? make_cpu_backend() : make_hip_backend(d));
    std::unique_ptr<Transport> tr;
    if (tname == "rccl") {
      std::string uid;
      if (root) uid = rccl_unique_id();
      if (rv) uid = rv->bcast(uid);
      tr = make_rccl_transport(uid);
    } else if (tname == "loopback") {
      tr = make_loopback_transport();
    } else if (tname == "host") {
      tr = make_host_transport();
    } else if (tname == "tcp") {
      MDFX_CHECK(rv != nullptr, "tcp transport needs a multi-process launch (mpirun / torchrun)");
      tr = make_tcp_transport(*rv);
    } else if (tname == "ipc" || tname == "ipc_sdma") {
      MDFX_CHECK(rv != nullptr && hip, "ipc transport needs a multi-process launch on HIP devices");
      Rendezvous* r = rv.get();
      CallbackFns f;
      f.allgather = [r](const std::string& mine) { return r->allgather(mine); };
      f.allreduce_sum = [r](double v) { return r->allreduce_sum(v); };
      f.allreduce_max = [r](double v) { return r->allreduce_max(v); };
      f.barrier = [r]() { r->barrier(); };
      tr = make_ipc_transport(std::move(f), tname == "ipc_sdma" ? 1 : -1, o.share_gpu);
    } else {
      MDFX_FAIL("unknown transport " + tname);
    }
    if (o.temporal <= 0 && o.py > 1) {
      // pencils: the fused 7-point sweep (heat7_wxk K = 4) is the one with y ghost rows
      const int want = spec.kind == StencilKind::Heat7 ? 4 : 1;
      const int64_t pz = nranks / o.py;
      o.temporal = hip && want > 1 && g.nz >= 4 * want * pz && g.ny >= 4 * want * o.py ? want : 1;
    }
    if (o.temporal <= 0) {  // auto: deepest fused sweep with a kernel, slabs >= 4 sweeps deep
      int want = hip ? hip_fused_depth(spec, g.nx) : 1;
      while (want > 1 && g.nz < 4 * (int64_t)want * nranks) want = shallower_depth(want);
      o.temporal = (hip && want > 1 &&
                    hip_supports_steps(spec, FieldLayout::make(g, 0, g.nz, want, spec.dtype), want))
                       ? want
                       : 1;
      // (a depth one residual interval's plan never runs would only widen the halo)
      if (hip && o.temporal > 2) o.temporal = hip_interval_depth(spec, g, o.temporal, o.residual_every, nranks);
    }
    SolverOptions so;
    so.overlap = o.overlap;
    so.sync_debug = o.sync_debug;
    so.residual_every = o.residual_every;
    so.graph = o.graph;
    so.timeout_s = o.timeout;
    so.temporal = o.temporal;
    so.py = o.py;
    so.fold = o.fold;
    Solver solver(spec, g, nranks, local_ranks, std::move(bes), std::move(tr), so);

    // ---- initial condition ----------------------------------------------------------------
    std::string ik = o.init;
    if (ik.empty())
      ik = kind == StencilKind::Jacobi5 ? "dirichlet"
                                        : (kind == StencilKind::Life ? (o.compat ? "compat" : "life") : "random");
    if (!o.resume.empty()) {
      solver.load_checkpoint(o.resume);
    } else if (ik == "compat") {
      MDFX_CHECK(kind == StencilKind::Life, "--init compat reproduces the reference Game-of-Life grid");
      std::vector<uint8_t> full((size_t)(g.nz * g.nx));
      cpu_life_compat_init(full.data(), g.nz, g.nx, o.density, (unsigned)o.seed);
      InitSpec zero;
      zero.kind = InitKind::Constant;
      zero.value = 0;
      solver.init(zero);
      for (int i = 0; i < solver.num_local(); ++i) {
        const FieldLayout& l = solver.layout(i);
        solver.write_owned(i, full.data() + (size_t)(l.z0 * g.nx));
      }
    } else {
      InitSpec is;
      if (ik == "random") is.kind = InitKind::Random;
      else if (ik == "dirichlet") is.kind = InitKind::Dirichlet;
      else if (ik == "constant") is.kind = InitKind::Constant;
      else if (ik == "life") is.kind = InitKind::LifeRandom;
      else MDFX_FAIL("unknown --init " + ik);
      is.seed = o.seed;
      is.lo = o.lo;
      is.hi = o.hi;
      is.value = o.value;
      is.edge = o.edge;
      is.interior = o.interior;
      is.density = o.density;
      solver.init(is);
    }

    // ---- run ------------------------------------------------------------------------------
    if (o.graph) solver.prepare_graphs();  // capture both cycles before the timed loop
    solver.run(o.warmup);
    // first launches of the kernel instances outside the timed loop (the reference dialogue has no
    // warm-up steps; the state is left unchanged)
    solver.warm_kernels(o.steps);
    solver.synchronize();
    solver.transport().barrier();
    const auto t0 = std::chrono::steady_clock::now();
    int64_t left = o.steps;
    while (left > 0) {
      int64_t k = left;
      if (o.ckpt_every > 0) k = std::min(k, o.ckpt_every - solver.stats().steps % o.ckpt_every);
      solver.run(k);
      left -= k;
      if (o.ckpt_every > 0 && solver.stats().steps % o.ckpt_every == 0) solver.save_checkpoint(o.ckpt_dir);
    }
    solver.synchronize();
    const double dt_local = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double dt = solver.transport().allreduce_max(dt_local);
    solver.transport().barrier();

    // ---- output ---------------------------------------------------------------------------
    const double cells = (double)g.cells();
    const double gcs = dt > 0 ? cells * (double)o.steps / dt / 1e9 : 0.0;
    const int ngpu = hip ? (env.world > 1 ? env.world : (o.gpus ? o.gpus : 1)) : 0;
    if (o.verbose)
      for (int i = 0; i < solver.num_local(); ++i) {
        const FieldLayout& l = solver.layout(i);
        std::fprintf(stderr, "[rank %d] planes [%lld, %lld) device %d pitch %lld local time %.6f s\n",
                     solver.local_rank(i), (long long)l.z0, (long long)l.z1, solver.backend(i).device(),
                     (long long)l.pitch, dt_local);
      }
    if (o.print) {
      // gather the dense global grid on rank 0
      std::vector<char> full;
      std::string mine;
      for (int i = 0; i < solver.num_local(); ++i) {
        const FieldLayout& l = solver.layout(i);
        std::string s((size_t)l.owned_cells() * l.esize(), '\0');
        solver.read_owned(i, &s[0]);
        mine += s;
      }
      if (rv) {
        const auto all = rv->allgather(mine);
        for (auto& s : all) full.insert(full.end(), s.begin(), s.end());
      } else {
        full.assign(mine.begin(), mine.end());
      }
      if (root) {
        if (spec.dtype == DType::U8) print_grid<uint8_t>(full, g.nx, g.ny, g.nz);
        else if (spec.dtype == DType::F32) print_grid<float>(full, g.nx, g.ny, g.nz);
        else print_grid<double>(full, g.nx, g.ny, g.nz);
      }
    }
    if (!o.dump.empty()) solver.save_checkpoint(o.dump);  // the state after --steps, before --profile
    double ph_b = -1, ph_i = -1, ph_x = -1, ph_s = -1;
    if (o.profile) {
      // profiled separately from the timed loop (profiling syncs the host every sweep); every
      // rank runs the extra steps, rank 0 reports its slab
      SolverOptions po = solver.options();
      po.profile = true;
      solver.set_options(po);
      solver.run(std::min<int64_t>(std::max<int64_t>(o.steps, 2), 50));
      solver.synchronize();
      const PhaseStats& ph = solver.phases();
      const double n = ph.steps ? (double)ph.steps : 1.0;
      ph_b = ph.boundary_ms / n;
      ph_i = ph.interior_ms / n;
      ph_x = ph.exchange_ms / n;
      ph_s = ph.step_ms / n;
      // the profiled steps ran after the last barrier: no rank may free its exported mailboxes
      // (ipc) while a slower neighbour still pulls from them
      if (root) std::fprintf(stderr,
                   "profile (rank 0, %lld sweeps, per sweep): boundary %.4f ms | interior %.4f ms | "
                   "exchange %.4f ms | step %.4f ms | overlap %.0f%%\n",
                   (long long)ph.steps, ph.boundary_ms / n, ph.interior_ms / n, ph.exchange_ms / n,
                   ph.step_ms / n,
                   ph.step_ms > 0 ? 100.0 * (ph.boundary_ms + ph.exchange_ms + ph.interior_ms - ph.step_ms) /
                                        std::max(1e-9, std::min(ph.boundary_ms + ph.exchange_ms, ph.interior_ms))
                                  : 0.0);
    }
    // teardown guard: every rank's queued exchanges are complete before any Solver is destroyed
    solver.synchronize();
    solver.transport().barrier();
    if (root && o.json) {
      std::string extra;
      if (ph_s > 0)
        extra = format(", \"phase_ms\": {\"boundary\": %.5f, \"interior\": %.5f, \"exchange\": %.5f, \"sweep\": %.5f}, "
                       "\"halo_fraction\": %.4f",
                       ph_b, ph_i, ph_x, ph_s, (ph_b + ph_x) / ph_s);
      std::printf(
          "{\"metric\": \"GCells/s\", \"value\": %.4f, \"unit\": \"GCells/s\", \"stencil\": \"%s\", \"dtype\": \"%s\", "
          "\"grid\": [%lld, %lld, %lld], \"steps\": %lld, \"seconds\": %.6f, \"ms_per_step\": %.4f, "
          "\"ranks\": %d, \"n_gpus\": %d, \"transport\": \"%s\", \"overlap\": %s, \"graph\": %s, \"residual\": %.9g, \"gcells_per_gpu\": %.4f, \"temporal\": %d%s}\n",
          gcs, stencil_name(kind), dtype_name(spec.dtype), (long long)g.nx, (long long)g.ny, (long long)g.nz,
          (long long)o.steps, dt, o.steps ? dt / o.steps * 1e3 : 0.0, nranks, ngpu, solver.transport().name(),
          o.overlap ? "true" : "false", solver.stats().graph_replays > 0 ? "true" : "false", solver.stats().last_residual,
          ngpu ? gcs / ngpu : gcs, solver.options().temporal, extra.c_str());
    } else if (root && !o.compat && !o.quiet) {
      std::printf("mdfx: %s %lldx%lldx%lld %s | %d slab(s), %s transport, %s | %lld steps in %.4f s | "
                  "%.4f ms/step | %.2f GCells/s total, %.2f per GPU",
                  stencil_name(kind), (long long)g.nx, (long long)g.ny, (long long)g.nz, dtype_name(spec.dtype),
                  nranks, solver.transport().name(), hip ? "hip" : "cpu", (long long)o.steps, dt,
                  o.steps ? dt / o.steps * 1e3 : 0.0, gcs, ngpu ? gcs / ngpu : gcs);
      if (solver.stats().last_residual >= 0) std::printf(" | residual %.6g", solver.stats().last_residual);
      std::printf("\n");
    }
    std::fflush(stdout);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s: error: %s\n", prog, e.what());
    std::fflush(stderr);
    return 1;
  }
}

}  // namespace mdfx
