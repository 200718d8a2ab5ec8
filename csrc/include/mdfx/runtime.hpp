// mdfx runtime: device backends (HIP / CPU) and halo transports.
//
// Reference parity:
//   CUDA runtime calls (MDF_kernel.cu:114-121,141-144,161,171,175,177,226-231; layer L0) ->
//   Backend, with RAII ownership and every call checked (D18).
//   MPI p2p halo loops (MDF_kernel.cu:167-169,180-183, one 4-byte message per cell, D5) ->
//   Transport::exchange: one whole-plane message per neighbour per step, device-resident, on a
//   dedicated halo stream.
#pragma once

#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "mdfx/kernels.hpp"

namespace mdfx {

enum class CopyKind : int { H2D = 0, D2H = 1, D2D = 2, H2H = 3 };

class Backend {
 public:
  virtual ~Backend() = default;
  virtual DeviceKind kind() const = 0;
  virtual int device() const = 0;  // HIP ordinal; -1 for CPU
  virtual void activate() const {}
  virtual void* alloc(size_t bytes) = 0;
  virtual void release(void* p) = 0;
  virtual void* create_stream(int priority) = 0;  // priority: 0 normal, 1 high
  virtual void destroy_stream(void* s) = 0;
  virtual void* create_event() = 0;
  virtual void destroy_event(void* e) = 0;
  virtual void record(void* ev, void* stream) = 0;
  virtual void wait(void* stream, void* ev) = 0;
  virtual void sync_stream(void* stream) = 0;
  virtual void sync_device() = 0;
  virtual void memset(void* p, int v, size_t n, void* stream) = 0;
  virtual void copy(void* dst, const void* src, size_t n, CopyKind k, void* stream) = 0;
  virtual void stencil(const StencilSpec& s, const RegionArgs& a, void* stream) = 0;
  virtual void init(const InitSpec& s, const FieldLayout& l, void* buf, void* stream) = 0;
  virtual void trace_push(const char*) {}
  virtual void trace_pop() {}
};

std::unique_ptr<Backend> make_cpu_backend();
std::unique_ptr<Backend> make_hip_backend(int device);
int hip_device_count();

// What a transport needs to know about one subdomain owned by this process.
struct LocalSlab {
  int rank = 0;               // global subdomain index (0..nranks-1)
  int py = 1;                 // pencil decomposition: subdomains per slab along y (1 = slabs)
  Backend* be = nullptr;
  void* halo_stream = nullptr;
  void* bnd_event = nullptr;  // recorded right after this step's boundary kernel(s)
  // recorded by transports whose records_ghost_event() is true, the moment this slab's ghosts of
  // the exchange have landed: ghost_event on the halo stream after its pull, ghost_event2 on the
  // stream of the other pull (the halo stream too when there is one pull); the solver's ev_x / ev_x2
  void* ghost_event = nullptr;
  void* ghost_event2 = nullptr;
  FieldLayout lay;
  void* buf[2] = {nullptr, nullptr};
};

// Byte ranges of one side of a halo exchange for buffer b. Sides 0 / 1 are the z faces (the first /
// last `halo` owned planes, whole planes with any ghost rows: one contiguous span), sides 2 / 3
// the y faces of a pencil (the first / last `hy` owned rows of every owned plane: `height` pieces
// of `width` bytes, `stride` bytes apart, on both ends). A pencil exchanges y first, then z, so the
// z faces carry the y ghosts just received and fill the corner ghosts (the fused K-step sweeps
// read them).
struct HaloSpan {
  int peer = -1;            // neighbouring subdomain, -1 if none (global boundary)
  void* send = nullptr;     // first piece of the owned cells sent
  void* recv = nullptr;     // first piece of the ghost cells received
  size_t bytes = 0;         // width * height
  size_t width = 0;         // contiguous bytes per piece
  size_t height = 1;        // pieces (1: contiguous)
  size_t stride = 0;        // bytes from one piece to the next
};
HaloSpan halo_span(const LocalSlab& s, int b, int side /*0 z-lo, 1 z-hi, 2 y-lo, 3 y-hi*/, int nranks);
// Throws unless every slab is a slab of a 1-D decomposition (transports without y faces).
void require_slabs(const std::vector<LocalSlab>& locals, const char* transport);
// Stream-ordered device-to-device copy of a halo face (same device or a mapped peer): mode 0 the
// runtime's blit kernels (hipMemcpyDeviceToDevice: copy shaders on the CUs), 1 the SDMA copy
// engines (hipMemcpyDeviceToDeviceNoCU: no CUs, lower bandwidth on one device), -1 the process
// default (face_copy_mode(): blit).
void hip_face_copy(void* dst, const void* src, size_t n, void* stream, int mode = -1);
// The same for a 2-D face (a pencil's y face: `height` pieces of `width` bytes, each side at its own
// pitch) ...
void hip_face_copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t width, size_t height, void* stream,
                     int mode = -1);
// ... and the copy of span `s` (the sender's, data at `src`) into span `d` (the receiver's, at `dst`),
// 1-D or 2-D by the spans' geometry.
void hip_face_copy(void* dst, const HaloSpan& d, const void* src, const HaloSpan& s, void* stream, int mode = -1);
int face_copy_mode();
// hipEventCreateWithFlags flags of the engine's and transports' stream-ordering events
bool hip_read_words(void* host, const void* dev, size_t bytes, double timeout_s);  // bounded D2H read (diagnostics)
int halo_stream_priority(bool halo);  // HIP stream priority of a halo (true) or compute stream
unsigned sync_event_flags();

class Transport {
 public:
  virtual ~Transport() = default;
  virtual const char* name() const = 0;
  virtual void setup(const std::vector<LocalSlab>& locals, int nranks) = 0;
  // Enqueue the exchange of buffer b (just written by the boundary kernels) on every local
  // slab's halo stream. On return, work later enqueued on a halo stream sees the ghosts, and
  // the sent planes may be overwritten by later work on the sender's halo stream.
  virtual void exchange(int b) = 0;
  // Blocking host-side reductions across all processes.
  virtual double allreduce_sum(double v) = 0;
  virtual double allreduce_max(double v) = 0;
  virtual void barrier() = 0;
  virtual bool in_process_only() const { return true; }  // every rank lives in this process
  // Optional async-error poll (RCCL, IPC counters); throws if a peer failed.
  virtual void check() {}
  // Whether exchange() only enqueues stream work on the halo streams (no host-side data movement
  // or blocking): rccl (grouped send / recv), loopback, ipc, proxy. The engine's folded,
  // boundary-on-the-compute-stream schedule (Solver::boundary_on_cs) needs exactly this.
  virtual bool stream_ordered() const { return false; }
  // Whether the loaded HIP runtime can also capture that stream work into a hipGraph that replays
  // it faithfully (stream_ordered() and capturable: RCCL's grouped send / recv only under HIP >= 7.2).
  virtual bool graph_capturable() const { return stream_ordered(); }
  // Whether exchange() records every local slab's ghost_event / ghost_event2 as soon as that slab's
  // ghosts have landed (each on the stream of the pull it follows), ahead of the exchange's
  // remaining bookkeeping (the ipc protocol's pulled signals and waits for the neighbours to have
  // pulled this slab's faces, which only the sweep after next, writing that buffer again, depends
  // on; the halo stream orders it). The solver then orders the next sweep after those two events
  // instead of after the whole exchange: no cross-stream join on the critical path.
  virtual bool records_ghost_event() const { return false; }
  // Whether the engine folds the lower boundary region into the interior sweep by default
  // (SolverOptions::fold = -1). A folded face is published by a device counter from inside the
  // sweep, not by a kernel boundary; its visibility to the exchange rests on the halo stream's
  // counter-wait kernel ending with the dispatch's system-scope release (hip_region_signals,
  // kernels.hpp). The ipc / proxy pulls are checked under it on one GPU (tests/test_gpu_ipc.py);
  // RCCL's p2p kernels as readers are not, so rccl opts out and folds only when asked (bench.py's
  // gated `rccl_fold` candidate).
  virtual bool fold_by_default() const { return true; }
  // Watchdog bound for blocking transport calls and device-side waits (seconds; 0 = default).
  virtual void set_timeout(double) {}
  // Watchdog escalation: make every outstanding transport operation return (ncclCommAbort, the
  // device abort word) so the streams drain and the process can exit instead of hanging.
  virtual void abort() {}
  // Watchdog diagnostics: the transport's device counters (the ipc protocol's ready / pulled
  // words, its private expect counters and its neighbours' words), printed before an abort.
  virtual std::string debug_state() { return ""; }
  // Parity of the buffer the last exchange() sent (-1: none yet, or the transport does not track
  // it). The ipc transport uses it to reuse a mailbox slot safely when a parity repeats.
  virtual int last_parity() const { return -1; }
  // The engine replayed captured exchanges (which bypass exchange()); the last one sent parity b.
  virtual void set_last_parity(int) {}
};

// CPU, all subdomains in this process: memcpy.
std::unique_ptr<Transport> make_host_transport();
// HIP, all subdomains in this process (one or several devices): D2D / peer copies with
// event ordering. Used for multi-rank testing on one GPU (RCCL refuses two ranks on one GPU).
std::unique_ptr<Transport> make_loopback_transport();
// RCCL send/recv over xGMI. `unique_id` is the 128-byte ncclUniqueId shared by all processes.
std::unique_ptr<Transport> make_rccl_transport(const std::string& unique_id);
// The rccl transport's schedule traits (what its Transport overrides return; the CPU tier asserts
// the engine schedule they select without constructing a communicator)
bool rccl_stream_ordered();
bool rccl_graph_capturable();
bool rccl_fold_by_default();
std::string rccl_unique_id();
// Host callbacks (the Python layer plugs torch.distributed in here, e.g. gloo on CPU).
struct CallbackFns {
  std::function<void(int)> exchange;
  std::function<double(double)> allreduce_sum;
  std::function<double(double)> allreduce_max;
  std::function<void()> barrier;
  // Gather one byte string from every process, indexed by rank (the ipc transport's handle swap).
  std::function<std::vector<std::string>(const std::string&)> allgather;
};
std::unique_ptr<Transport> make_callback_transport(CallbackFns fns);
// HIP IPC, one slab per process (any number of processes per GPU): faces pulled from the
// neighbours' mapped buffers by the copy engines, ordered by device-side counters
// (csrc/comm/ipc_transport.cpp). Needs fns.allgather; residual / barrier go through fns too.
// copy_mode: the face copy engine (hip_face_copy; -1 = process default). Named "ipc" (blit) or
// "ipc_sdma".
// share_gpu: allow several engine processes on one GPU (tests only; see ipc_shared_gpu_problem).
std::unique_ptr<Transport> make_ipc_transport(CallbackFns fns, int copy_mode = -1, bool share_gpu = false);
// Whether the ipc transport pulls faces straight from the neighbours' exported field buffers (one
// copy per face) rather than through mailboxes (two): buffers of at most 1900 MiB, since torch's
// HIP 7.0 runtime stalls mapping exported buffers of 2 GiB and more; MDFX_IPC_DIRECT=0 / 1 forces.
bool ipc_direct_ok(size_t field_bytes);
// The ipc transport's export with its bounded retry: calls get() (a hipError_t as int) until it
// succeeds, retrying "invalid argument" up to max_retries times sleep_us apart (logging a diagnosis
// of p on the first failure); returns the retries taken, throws on any other error or when they run
// out. MDFX_IPC_EXPORT_FAIL=n injects n failures per process (tests).
int ipc_export_retry(const std::function<int()>& get, void* p, int max_retries, int sleep_us);
// Rank proxy (HIP): ONE slab of an N-way decomposition alone on a GPU, exchanging with itself
// through the ipc transport's mailbox copies and device counters (csrc/comm/proxy_transport.cpp):
// the per-GPU schedule of an N-GPU run, measurable on one GPU. Ghost values are the slab's own
// faces, so results are exact only away from the proxied boundaries.
std::unique_ptr<Transport> make_proxy_transport(int copy_mode = -1);
// What the ipc transport knows about one process's slab when it maps a neighbour (the host-side
// part of its handle record).
struct IpcPeerInfo {
  int rank = -1, device = -1, pid = 0;
  uint64_t face_bytes = 0;
  bool magic_ok = true;
};
// Host-only validation of a neighbour's record (CPU-testable): "" if the pair can exchange, else
// why not. `peer_access` is hipDeviceCanAccessPeer(mine.device -> peer.device) for devices that
// differ (ignored on one device).
std::string ipc_peer_problem(const IpcPeerInfo& mine, const IpcPeerInfo& peer, int expect_rank, bool peer_access);
// Host-only check over every rank's (pid, GPU PCI bus id) record (CPU-testable): "" unless two
// engine processes would share one GPU without share_gpu. The exchange and the folded boundary order
// their work by device-side spin waits (counter_wait_kernel, csrc/kernels/sync_kernels.hip), which
// rely on the hardware scheduler running every producer queue: with several processes' queues
// oversubscribing one GPU a waiting queue can starve the producing one (round 4, session T:
// profiles/r04_session_t/). One process per GPU, the production layout, never does; the one-GPU
// multi-process tests opt in with share_gpu. Every rank sees the same records, so all refuse together.
std::string ipc_shared_gpu_problem(const std::vector<std::pair<int, std::string>>& pid_pci, bool share_gpu);

}  // namespace mdfx
