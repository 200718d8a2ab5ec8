// pybind11 bindings: module `_mdfx` (built in-tree into mpi_cuda_process_amd/).
//
// Deliberately torch-header-free (fast builds, no ABI coupling): tensors cross the boundary as raw
// pointers checked by the Python layer, and device memory owned by the engine is exported
// zero-copy through DLPack capsules (torch.from_dlpack).
#include <pybind11/functional.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "mdfx/devsync.hpp"
#include "mdfx/solver.hpp"
#include "mdfx/sweep_plan.hpp"

namespace py = pybind11;
using namespace mdfx;

namespace {

// ---- minimal DLPack ABI (v0.8 "dltensor" capsule) -------------------------------------------
struct DLDevice {
  int32_t device_type;  // kDLCPU = 1, kDLROCM = 10
  int32_t device_id;
};
struct DLDataType {
  uint8_t code;  // 0 int, 1 uint, 2 float
  uint8_t bits;
  uint16_t lanes;
};
struct DLTensor {
  void* data;
  DLDevice device;
  int32_t ndim;
  DLDataType dtype;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
};
struct DLManagedTensor {
  DLTensor dl_tensor;
  void* manager_ctx;
  void (*deleter)(DLManagedTensor*);
};
struct DLCtx {
  std::vector<int64_t> shape, strides;
};

void dl_deleter(DLManagedTensor* t) {
  delete (DLCtx*)t->manager_ctx;
  delete t;
}

py::capsule make_dlpack(void* data, int device, DType dt, std::vector<int64_t> shape,
                        std::vector<int64_t> strides) {
  auto* ctx = new DLCtx{std::move(shape), std::move(strides)};
  auto* t = new DLManagedTensor();
  t->dl_tensor.data = data;
  t->dl_tensor.device = DLDevice{device < 0 ? 1 : 10, device < 0 ? 0 : device};
  t->dl_tensor.ndim = (int32_t)ctx->shape.size();
  switch (dt) {
    case DType::F32: t->dl_tensor.dtype = DLDataType{2, 32, 1}; break;
    case DType::F64: t->dl_tensor.dtype = DLDataType{2, 64, 1}; break;
    case DType::U8: t->dl_tensor.dtype = DLDataType{1, 8, 1}; break;
  }
  t->dl_tensor.shape = ctx->shape.data();
  t->dl_tensor.strides = ctx->strides.data();
  t->dl_tensor.byte_offset = 0;
  t->manager_ctx = ctx;
  t->deleter = dl_deleter;
  return py::capsule(t, "dltensor", [](PyObject* cap) {
    // only delete if the consumer never took ownership (name still "dltensor")
    if (PyCapsule_IsValid(cap, "dltensor")) {
      auto* m = (DLManagedTensor*)PyCapsule_GetPointer(cap, "dltensor");
      if (m && m->deleter) m->deleter(m);
    }
  });
}

StencilSpec make_spec(const std::string& kind, const std::string& dtype, double r, double c0,
                      double c1, double c2, double c3, bool ref_precision = false) {
  StencilSpec s;
  s.coef.ref_precision = ref_precision;
  s.kind = stencil_from_name(kind);
  s.dtype = dtype_from_name(dtype);
  s.coef.r = r;
  s.coef.c0 = c0;
  s.coef.c1 = c1;
  s.coef.c2 = c2;
  s.coef.c3 = c3;
  return s;
}

InitSpec make_init(const std::string& kind, uint64_t seed, double lo, double hi, double value,
                   double edge, double interior, double density) {
  InitSpec s;
  if (kind == "constant")
    s.kind = InitKind::Constant;
  else if (kind == "dirichlet")
    s.kind = InitKind::Dirichlet;
  else if (kind == "random")
    s.kind = InitKind::Random;
  else if (kind == "life" || kind == "life_random")
    s.kind = InitKind::LifeRandom;
  else
    throw Error("unknown init kind '" + kind + "' (constant|dirichlet|random|life)");
  s.seed = seed;
  s.lo = lo;
  s.hi = hi;
  s.value = value;
  s.edge = edge;
  s.interior = interior;
  s.density = density;
  return s;
}

py::dict layout_dict(const FieldLayout& l) {
  py::dict d;
  d["nx"] = l.global.nx;
  d["ny"] = l.global.ny;
  d["nz"] = l.global.nz;
  d["z0"] = l.z0;
  d["z1"] = l.z1;
  d["halo"] = l.halo;
  d["pitch"] = l.pitch;
  d["plane"] = l.plane;
  d["planes"] = l.planes();
  d["nzl"] = l.nzl();
  d["y0"] = l.y0;
  d["y1"] = l.y1;
  d["hy"] = l.hy;
  d["nyl"] = l.nyl();
  d["rows"] = l.rows();
  d["bytes"] = l.bytes();
  d["esize"] = l.esize();
  d["dtype"] = dtype_name(l.dtype);
  return d;
}

py::dtype np_dtype(DType t) {
  switch (t) {
    case DType::F32: return py::dtype::of<float>();
    case DType::F64: return py::dtype::of<double>();
    case DType::U8: return py::dtype::of<uint8_t>();
  }
  return py::dtype::of<float>();
}

// Host callables from a dict {"exchange", "allreduce_sum", "allreduce_max", "barrier",
// "allgather"}; each re-acquires the GIL (the engine runs with it released).
CallbackFns callback_fns(py::object callbacks) {
  if (callbacks.is_none()) throw Error("this transport needs callbacks");
  py::dict cb = callbacks.cast<py::dict>();
  CallbackFns f;
  // callables may be released from a thread that does not hold the GIL (close() releases it)
  auto keep = [](py::object o) {
    return std::shared_ptr<py::object>(new py::object(std::move(o)), [](py::object* q) {
      py::gil_scoped_acquire g;
      delete q;
    });
  };
  if (cb.contains("exchange")) {
    auto ex = keep(cb["exchange"]);
    f.exchange = [ex](int b) {
      py::gil_scoped_acquire g;
      (*ex)(b);
    };
  }
  if (cb.contains("allreduce_sum")) {
    auto ar = keep(cb["allreduce_sum"]);
    f.allreduce_sum = [ar](double v) {
      py::gil_scoped_acquire g;
      return (*ar)(v).cast<double>();
    };
  }
  if (cb.contains("allreduce_max")) {
    auto am = keep(cb["allreduce_max"]);
    f.allreduce_max = [am](double v) {
      py::gil_scoped_acquire g;
      return (*am)(v).cast<double>();
    };
  }
  if (cb.contains("barrier")) {
    auto ba = keep(cb["barrier"]);
    f.barrier = [ba]() {
      py::gil_scoped_acquire g;
      (*ba)();
    };
  }
  if (cb.contains("allgather")) {
    auto ag = keep(cb["allgather"]);
    f.allgather = [ag](const std::string& mine) {
      py::gil_scoped_acquire g;
      std::vector<std::string> out;
      for (auto item : (*ag)(py::bytes(mine))) out.push_back(item.cast<std::string>());
      return out;
    };
  }
  return f;
}

class PySolver {
 public:
  PySolver(const std::string& kind, const std::string& dtype, int64_t nx, int64_t ny, int64_t nz,
           int nranks, std::vector<int> local_ranks, std::vector<int> devices,
           const std::string& transport, py::bytes unique_id, py::object callbacks, bool overlap,
           bool sync_debug, int residual_every, bool graph, double timeout_s, double r, double c0,
           double c1, double c2, double c3, int temporal, bool ref_precision, int pencil_py, bool share_gpu) {
    const StencilSpec spec = make_spec(kind, dtype, r, c0, c1, c2, c3, ref_precision);
    if (devices.size() == 1 && local_ranks.size() > 1) devices.assign(local_ranks.size(), devices[0]);
    if (devices.size() != local_ranks.size())
      throw Error("devices must have one entry per local rank (or a single entry)");
    std::vector<std::unique_ptr<Backend>> bes;
    for (int d : devices) bes.push_back(d < 0 ? make_cpu_backend() : make_hip_backend(d));
    std::unique_ptr<Transport> tr;
    if (transport == "host") {
      tr = make_host_transport();
    } else if (transport == "loopback") {
      tr = make_loopback_transport();
    } else if (transport == "rccl") {
      tr = make_rccl_transport(std::string(unique_id));
    } else if (transport == "callback") {
      CallbackFns f = callback_fns(callbacks);
      if (!f.exchange) throw Error("callback transport needs an exchange callback");
      tr = make_callback_transport(std::move(f));
    } else if (transport == "ipc" || transport == "ipc_sdma") {
      CallbackFns f = callback_fns(callbacks);
      if (!f.allgather) throw Error("ipc transport needs an allgather callback");
      tr = make_ipc_transport(std::move(f), transport == "ipc_sdma" ? 1 : -1, share_gpu);
    } else if (transport == "proxy" || transport == "proxy_sdma") {
      tr = make_proxy_transport(transport == "proxy_sdma" ? 1 : -1);
    } else {
      throw Error("unknown transport '" + transport + "' (host|loopback|rccl|ipc|ipc_sdma|callback|proxy|proxy_sdma)");
    }
    SolverOptions o;
    o.overlap = overlap;
    o.sync_debug = sync_debug;
    o.residual_every = residual_every;
    o.graph = graph;
    o.timeout_s = timeout_s;
    o.temporal = temporal;
    o.py = pencil_py;
    py::gil_scoped_release nogil;  // RCCL comm init may block on peers
    s_.reset(new Solver(spec, Extent3{nx, ny, nz}, nranks, std::move(local_ranks), std::move(bes),
                        std::move(tr), o));
  }

  Solver& s() { return *s_; }
  void close() {
    py::gil_scoped_release nogil;
    s_.reset();
  }
  Solver& chk() {
    if (!s_) throw Error("solver is closed");
    return *s_;
  }

  std::unique_ptr<Solver> s_;
};

}  // namespace

PYBIND11_MODULE(_mdfx, m) {
  m.doc() = "mdfx: MI355X-native multi-GPU finite-difference stencil engine (native core)";
  py::register_exception<Error>(m, "MdfxError", PyExc_RuntimeError);

  m.def("hip_device_count", &hip_device_count);
  m.def("hip_wait_error", &hip_wait_error, "1 after a device-side halo wait timed out");
  m.def(
      "ipc_peer_problem",
      [](py::dict mine, py::dict peer, int expect_rank, bool peer_access) {
        auto info = [](py::dict d) {
          IpcPeerInfo i;
          i.rank = d["rank"].cast<int>();
          i.device = d["device"].cast<int>();
          i.pid = d["pid"].cast<int>();
          i.face_bytes = d["face_bytes"].cast<uint64_t>();
          i.magic_ok = d.contains("magic_ok") ? d["magic_ok"].cast<bool>() : true;
          return i;
        };
        return ipc_peer_problem(info(mine), info(peer), expect_rank, peer_access);
      },
      "host-side check of an ipc neighbour record: '' if usable, else the reason");
  m.def("ipc_shared_gpu_problem", &ipc_shared_gpu_problem, py::arg("pid_pci"), py::arg("share_gpu") = false,
        "host-side check of every rank's (pid, GPU PCI bus id): '' unless engine processes share a GPU");
  m.def("ipc_export_retry_selftest", [](int fail, int max_retries) {
    // the export retry loop with a stand-in for hipIpcGetMemHandle that fails `fail` times with
    // "invalid argument" (1), then succeeds (0); no device needed
    int n = 0;
    return ipc_export_retry([&]() { return n++ < fail ? 1 : 0; }, nullptr, max_retries, 0);
  }, py::arg("fail"), py::arg("max_retries") = 80, "retries the ipc export loop takes for `fail` failures");
  m.def("rccl_unique_id", []() { return py::bytes(rccl_unique_id()); });
  m.def("rccl_traits", []() {
    py::dict d;
    d["stream_ordered"] = rccl_stream_ordered();
    d["graph_capturable"] = rccl_graph_capturable();
    d["fold_by_default"] = rccl_fold_by_default();
    return d;
  }, "what the rccl transport reports to the engine (it is never constructed for this)");
  m.def("step_schedule", &step_schedule, py::arg("overlap"), py::arg("local_slabs"), py::arg("stream_ordered"),
        py::arg("fold"), "the engine's per-step schedule for a layout and transport (Solver::schedule)");
  m.def("fold_allowed", &fold_allowed, py::arg("fold_opt"), py::arg("transport_default"),
        "whether a step may fold its lower boundary (SolverOptions::fold, Transport::fold_by_default)");
  m.def("set_kernel_variant", [](const std::string& v) { hip_set_kernel_variant(v.c_str()); });
  m.def("reload_knobs", &hip_reload_knobs, "re-read the MDFX_* kernel tuning knobs from the environment");
  m.def("poison_lds", &hip_poison_lds, "fill every CU's LDS with NaN (tests for stale-LDS reads)");
  m.def("hip_runtime_version", &hip_runtime_version,
        "version of the HIP runtime the process loaded (PyTorch's bundled one under torch), 0 if none");
  m.def("kernel_variant", []() { return std::string(hip_kernel_variant()); });
  m.def("face_copy_mode", []() { return std::string(face_copy_mode() == 1 ? "sdma" : "blit"); },
        "default engine of the ipc / proxy halo face copies (blit; ipc_sdma / proxy_sdma pick SDMA)");
  m.def("ipc_direct_ok", [](size_t bytes) { return ipc_direct_ok(bytes); },
        "whether the ipc transport pulls straight from field buffers of this size (MDFX_IPC_DIRECT)");
  m.def("layout", [](int64_t nx, int64_t ny, int64_t nz, int64_t z0, int64_t z1, int halo,
                     const std::string& dtype, int64_t y0, int64_t y1, int hy) {
    return layout_dict(FieldLayout::make(Extent3{nx, ny, nz}, z0, z1, halo, dtype_from_name(dtype), y0, y1, hy));
  }, py::arg("nx"), py::arg("ny"), py::arg("nz"), py::arg("z0"), py::arg("z1"), py::arg("halo") = 1,
        py::arg("dtype") = "f32", py::arg("y0") = 0, py::arg("y1") = -1, py::arg("hy") = 0);
  m.def("slab_bounds", [](int64_t nz, int parts) {
    SlabDecomposition d(nz, parts);
    std::vector<std::pair<int64_t, int64_t>> out;
    for (int p = 0; p < parts; ++p) out.emplace_back(d.z0(p), d.z1(p));
    return out;
  });

  // Kernel-level entry: one region update on caller-owned memory (torch tensors in the tests).
  m.def(
      "stencil",
      [](const std::string& kind, const std::string& dtype, uintptr_t in, uintptr_t out, int64_t nx,
         int64_t ny, int64_t nz, int64_t z0, int64_t z1, int halo, int64_t lz_begin, int64_t lz_end,
         int device, uintptr_t stream, uintptr_t resid, double r, double c0, double c1, double c2,
         double c3, int steps, bool ref_precision, int64_t lz2_begin, int64_t lz2_end) {
        RegionArgs a;
        a.lz2_begin = lz2_begin;
        a.lz2_end = lz2_end;
        a.in = (const void*)in;
        a.out = (void*)out;
        a.lay = FieldLayout::make(Extent3{nx, ny, nz}, z0, z1, halo, dtype_from_name(dtype));
        a.lz_begin = lz_begin;
        a.lz_end = lz_end;
        a.resid = (double*)resid;
        a.steps = steps;
        const StencilSpec spec = make_spec(kind, dtype, r, c0, c1, c2, c3, ref_precision);
        if (device < 0)
          cpu_stencil(spec, a);
        else
          hip_stencil(spec, a, (void*)stream);
      },
      py::arg("kind"), py::arg("dtype"), py::arg("in_ptr"), py::arg("out_ptr"), py::arg("nx"),
      py::arg("ny"), py::arg("nz"), py::arg("z0"), py::arg("z1"), py::arg("halo"),
      py::arg("lz_begin"), py::arg("lz_end"), py::arg("device"), py::arg("stream") = 0,
      py::arg("resid_ptr") = 0, py::arg("r") = -1.0, py::arg("c0") = 0.25, py::arg("c1") = 0.05,
      py::arg("c2") = 0.025, py::arg("c3") = 3.0 / 160.0, py::arg("steps") = 1, py::arg("ref_precision") = false,
      py::arg("lz2_begin") = 0, py::arg("lz2_end") = 0);
  m.def(
      "init_field",
      [](const std::string& kind, const std::string& dtype, uintptr_t buf, int64_t nx, int64_t ny,
         int64_t nz, int64_t z0, int64_t z1, int halo, int device, uintptr_t stream, uint64_t seed,
         double lo, double hi, double value, double edge, double interior, double density) {
        const FieldLayout l = FieldLayout::make(Extent3{nx, ny, nz}, z0, z1, halo, dtype_from_name(dtype));
        const InitSpec s = make_init(kind, seed, lo, hi, value, edge, interior, density);
        if (device < 0)
          cpu_init(s, l, (void*)buf);
        else
          hip_init(s, l, (void*)buf, (void*)stream);
      },
      py::arg("kind"), py::arg("dtype"), py::arg("buf_ptr"), py::arg("nx"), py::arg("ny"),
      py::arg("nz"), py::arg("z0"), py::arg("z1"), py::arg("halo"), py::arg("device"),
      py::arg("stream") = 0, py::arg("seed") = 1, py::arg("lo") = 0.0, py::arg("hi") = 1.0,
      py::arg("value") = 0.0, py::arg("edge") = 100.0, py::arg("interior") = 0.0,
      py::arg("density") = 0.15);
  m.def("hip_supports_steps", [](const std::string& kind, const std::string& dtype, int64_t nx, int64_t ny,
                                 int64_t nz, int halo, int steps, bool ref_precision) {
    StencilSpec s = make_spec(kind, dtype, -1, 0, 0, 0, 0, ref_precision);
    return hip_supports_steps(s, FieldLayout::make(Extent3{nx, ny, nz}, 0, nz, halo, dtype_from_name(dtype)), steps);
  }, py::arg("kind"), py::arg("dtype"), py::arg("nx"), py::arg("ny"), py::arg("nz"), py::arg("halo"),
     py::arg("steps"), py::arg("ref_precision") = false);
  m.def("hip_fused_depth", [](const std::string& kind, const std::string& dtype, int64_t nx, bool ref_precision) {
    StencilSpec s = make_spec(kind, dtype, -1, 0, 0, 0, 0, ref_precision);
    return hip_fused_depth(s, nx);
  }, py::arg("kind"), py::arg("dtype"), py::arg("nx"), py::arg("ref_precision") = false);
  m.def("plan_sweeps", [](int64_t steps, int64_t start, int64_t residual_every, int temporal,
                          std::vector<double> cost, std::vector<bool> ok) {
    SweepCosts c;
    c.T = temporal;
    for (size_t k = 0; k < cost.size() && k < 17; ++k) c.cost[k] = cost[k];
    for (size_t k = 0; k < ok.size() && k < 17; ++k) c.ok[k] = ok[k];
    c.ok[1] = true;
    return plan_sweeps(c, steps, start, residual_every);
  }, py::arg("steps"), py::arg("start"), py::arg("residual_every"), py::arg("temporal"), py::arg("cost"),
     py::arg("ok"), "the engine's sweep plan for given per-depth costs (cost[k], ok[k] indexed by depth)");
  m.def("interval_depth", [](int64_t residual_every, int temporal, std::vector<double> cost, std::vector<bool> ok,
                             bool uniform) {
    SweepCosts c;
    c.T = temporal;
    for (size_t k = 0; k < cost.size() && k < 17; ++k) c.cost[k] = cost[k];
    for (size_t k = 0; k < ok.size() && k < 17; ++k) c.ok[k] = ok[k];
    c.ok[1] = true;
    return interval_depth(c, residual_every, uniform);
  }, py::arg("residual_every"), py::arg("temporal"), py::arg("cost"), py::arg("ok"), py::arg("uniform") = false,
     "the deepest depth <= temporal that one residual interval's sweep plan runs (interval_depth)");
  m.def("hip_auto_depth", [](const std::string& kind, const std::string& dtype, int64_t nx, int64_t ny, int64_t nz,
                             int want, int64_t residual_every, bool ref_precision, int nranks) {
    StencilSpec s = make_spec(kind, dtype, -1, 0, 0, 0, 0, ref_precision);
    return hip_interval_depth(s, Extent3{nx, ny, nz}, want, residual_every, nranks);
  }, py::arg("kind"), py::arg("dtype"), py::arg("nx"), py::arg("ny"), py::arg("nz"), py::arg("want"),
     py::arg("residual_every"), py::arg("ref_precision") = false, py::arg("nranks") = 1,
     "want, made shallower until one residual interval's plan runs a sweep of that depth (HIP cost tables)");
  m.def("hip_sweep_cost", [](const std::string& kind, const std::string& dtype, int64_t nx, int steps) {
    return hip_sweep_cost(make_spec(kind, dtype, -1, 0, 0, 0, 0, false), nx, steps);
  }, py::arg("kind"), py::arg("dtype"), py::arg("nx"), py::arg("steps"));
  m.def("life_compat_init", [](int64_t h, int64_t w, double density, unsigned seed) {
    py::array_t<uint8_t> a({h, w});
    cpu_life_compat_init(a.mutable_data(), h, w, density, seed);
    return a;
  }, py::arg("h"), py::arg("w"), py::arg("density") = 0.15, py::arg("seed") = 1);

  py::class_<PySolver>(m, "Solver")
      .def(py::init<const std::string&, const std::string&, int64_t, int64_t, int64_t, int,
                    std::vector<int>, std::vector<int>, const std::string&, py::bytes, py::object,
                    bool, bool, int, bool, double, double, double, double, double, double, int, bool, int, bool>(),
           py::arg("kind"), py::arg("dtype"), py::arg("nx"), py::arg("ny"), py::arg("nz"),
           py::arg("nranks"), py::arg("local_ranks"), py::arg("devices"), py::arg("transport"),
           py::arg("unique_id") = py::bytes(""), py::arg("callbacks") = py::none(),
           py::arg("overlap") = true, py::arg("sync_debug") = false, py::arg("residual_every") = 0,
           py::arg("graph") = false, py::arg("timeout_s") = 0.0, py::arg("r") = -1.0,
           py::arg("c0") = 0.25, py::arg("c1") = 0.05, py::arg("c2") = 0.025,
           py::arg("c3") = 3.0 / 160.0, py::arg("temporal") = 1, py::arg("ref_precision") = false, py::arg("py") = 1,
           py::arg("share_gpu") = false)
      .def("close", &PySolver::close)
      .def("phase_times",
           [](PySolver& p) {
             const PhaseStats& ph = p.chk().phases();
             py::dict d;
             d["sweeps"] = ph.steps;
             d["boundary_ms"] = ph.boundary_ms;
             d["interior_ms"] = ph.interior_ms;
             d["exchange_ms"] = ph.exchange_ms;
             d["step_ms"] = ph.step_ms;
             d["exposed_ms"] = ph.exposed_ms;
             return d;
           })
      .def("reset_phases", [](PySolver& p) { p.chk().reset_phases(); })
      .def("init",
           [](PySolver& p, const std::string& kind, uint64_t seed, double lo, double hi, double value,
              double edge, double interior, double density) {
             const InitSpec s = make_init(kind, seed, lo, hi, value, edge, interior, density);
             py::gil_scoped_release nogil;
             p.chk().init(s);
           },
           py::arg("kind") = "random", py::arg("seed") = 1, py::arg("lo") = 0.0, py::arg("hi") = 1.0,
           py::arg("value") = 0.0, py::arg("edge") = 100.0, py::arg("interior") = 0.0,
           py::arg("density") = 0.15)
      .def("run",
           [](PySolver& p, int64_t steps) {
             py::gil_scoped_release nogil;
             p.chk().run(steps);
           })
      .def("synchronize",
           [](PySolver& p) {
             py::gil_scoped_release nogil;
             p.chk().synchronize();
           })
      .def("exchange_ghosts",
           [](PySolver& p) {
             py::gil_scoped_release nogil;
             p.chk().exchange_ghosts();
           })
      .def("set_options",
           [](PySolver& p, py::kwargs kw) {
             // only the options named change; the rest keep their current values
             SolverOptions o = p.chk().options();
             for (auto item : kw) {
               const std::string k = py::str(item.first);
               if (k == "overlap") o.overlap = item.second.cast<bool>();
               else if (k == "sync_debug") o.sync_debug = item.second.cast<bool>();
               else if (k == "residual_every") o.residual_every = item.second.cast<int>();
               else if (k == "graph") o.graph = item.second.cast<bool>();
               else if (k == "timeout_s") o.timeout_s = item.second.cast<double>();
               else if (k == "min_rounds") o.min_rounds = item.second.cast<int>();
               else if (k == "profile") o.profile = item.second.cast<bool>();
               else if (k == "fold") o.fold = item.second.cast<int>();
               else throw py::key_error("unknown solver option " + k);
             }
             p.chk().set_options(o);
           })
      .def("options",
           [](PySolver& p) {
             const SolverOptions& o = p.chk().options();
             py::dict d;
             d["overlap"] = o.overlap;
             d["sync_debug"] = o.sync_debug;
             d["residual_every"] = o.residual_every;
             d["graph"] = o.graph;
             d["timeout_s"] = o.timeout_s;
             d["profile"] = o.profile;
             d["temporal"] = o.temporal;
             d["min_rounds"] = o.min_rounds;
             d["py"] = o.py;
             d["fold"] = o.fold;
             return d;
           })
      .def_property_readonly("num_local", [](PySolver& p) { return p.chk().num_local(); })
      .def_property_readonly("temporal", [](PySolver& p) { return p.chk().options().temporal; })
      .def_property_readonly("nranks", [](PySolver& p) { return p.chk().nranks(); })
      .def_property_readonly("steps", [](PySolver& p) { return p.chk().stats().steps; })
      .def_property_readonly("residual", [](PySolver& p) { return p.chk().stats().last_residual; })
      .def_property_readonly("residual_step", [](PySolver& p) { return p.chk().stats().residual_step; })
      .def_property_readonly("graph_replays", [](PySolver& p) { return p.chk().stats().graph_replays; })
      .def_property_readonly("graph_captures", [](PySolver& p) { return p.chk().stats().graph_captures; })
      .def_property_readonly("folded_sweeps", [](PySolver& p) { return p.chk().stats().folded_sweeps; })
      .def_property_readonly("graph_wait_nodes", [](PySolver& p) { return p.chk().stats().graph_wait_nodes; })
      .def_property_readonly("graph_fold_waits", [](PySolver& p) { return p.chk().stats().graph_fold_waits; })
      .def("prepare_graphs", [](PySolver& p) { return p.chk().prepare_graphs(); },
           "capture both parities' 2-sweep hipGraph cycles now (0 if graphs are off / not capturable)")
      .def("sweep_plan", [](PySolver& p, int64_t steps) { return p.chk().sweep_plan(steps); }, py::arg("steps"),
           "the sweeps run(steps) would issue from here: a list of (fused depth, residual sweep)")
      .def("warm_kernels", [](PySolver& p, int64_t steps) { p.chk().warm_kernels(steps); }, py::arg("steps"),
           py::call_guard<py::gil_scoped_release>(),
           "launch every kernel instance run(steps) would use once, into the scratch buffer (state unchanged)")
      .def_property_readonly("graph_eligible", [](PySolver& p) { return p.chk().graph_eligible(); })
      .def_property_readonly("schedule", [](PySolver& p) { return p.chk().schedule(); },
                             "the per-step schedule eager steps run (step_schedule)")
      .def_property_readonly("current_index", [](PySolver& p) { return p.chk().current_index(); })
      .def_property_readonly("transport_name", [](PySolver& p) { return std::string(p.chk().transport().name()); })
      .def("local_rank", [](PySolver& p, int i) { return p.chk().local_rank(i); })
      .def("layout", [](PySolver& p, int i) { return layout_dict(p.chk().layout(i)); })
      .def("device", [](PySolver& p, int i) { return p.chk().backend(i).device(); })
      .def("buffer_ptr", [](PySolver& p, int i, int b) { return (uintptr_t)p.chk().buffer(i, b); })
      .def("halo_stream", [](PySolver& p, int i) { return (uintptr_t)p.chk().halo_stream(i); })
      .def("compute_stream", [](PySolver& p, int i) { return (uintptr_t)p.chk().compute_stream(i); })
      .def("halo_spans",
           [](PySolver& p, int i, int b) {
             Solver& s = p.chk();
             LocalSlab ls;
             ls.rank = s.local_rank(i);
             ls.lay = s.layout(i);
             ls.buf[0] = s.buffer(i, 0);
             ls.buf[1] = s.buffer(i, 1);
             ls.py = s.options().py;
             py::list out;
             // pencils: the y faces (sides 2, 3: height pieces of width bytes, stride apart) come
             // first; the z faces (0, 1) carry the y ghost rows, so they go once those have landed
             const std::vector<int> sides = ls.py > 1 ? std::vector<int>{2, 3, 0, 1} : std::vector<int>{0, 1};
             for (int side : sides) {
               const HaloSpan h = halo_span(ls, b, side, s.nranks());
               py::dict d;
               d["side"] = side;
               d["peer"] = h.peer;
               d["send"] = (uintptr_t)h.send;
               d["recv"] = (uintptr_t)h.recv;
               d["bytes"] = h.bytes;
               d["width"] = h.width;
               d["height"] = h.height;
               d["stride"] = h.stride;
               out.append(d);
             }
             return out;
           })
      .def("view",
           [](PySolver& p, int i, int b) {
             Solver& s = p.chk();
             const FieldLayout& l = s.layout(i);
             return make_dlpack(s.buffer(i, b), s.backend(i).device(), l.dtype,
                                {l.planes(), l.rows(), l.pitch}, {l.plane, l.pitch, 1});
           })
      .def("bytes_view",
           [](PySolver& p, int i, uintptr_t ptr, int64_t nbytes) {
             Solver& s = p.chk();
             return make_dlpack((void*)ptr, s.backend(i).device(), DType::U8, {nbytes}, {1});
           })
      .def("read_owned",
           [](PySolver& p, int i) {
             Solver& s = p.chk();
             const FieldLayout& l = s.layout(i);
             py::array a(np_dtype(l.dtype), std::vector<int64_t>{l.nzl(), l.nyl(), l.global.nx});
             void* dst = a.mutable_data();
             {
               py::gil_scoped_release nogil;
               s.read_owned(i, dst);
             }
             return a;
           })
      .def("write_owned",
           [](PySolver& p, int i, py::array a) {
             Solver& s = p.chk();
             const FieldLayout& l = s.layout(i);
             if ((size_t)a.nbytes() != (size_t)l.owned_cells() * l.esize())
               throw Error("write_owned: array size does not match the slab");
             py::array c = py::array::ensure(a, py::array::c_style);
             const void* src = c.data();
             py::gil_scoped_release nogil;
             s.write_owned(i, src);
           })
      .def("save_checkpoint",
           [](PySolver& p, const std::string& d) {
             py::gil_scoped_release nogil;
             p.chk().save_checkpoint(d);
           })
      .def("load_checkpoint", [](PySolver& p, const std::string& d) {
        py::gil_scoped_release nogil;
        p.chk().load_checkpoint(d);
      });
}
