// HIP-IPC halo transport: one process per slab; the neighbours pull each other's boundary faces
// straight into their ghost planes (over xGMI between GPUs), ordered by device-side counters instead
// of host synchronisation. Two copy engines: "ipc" (the default) pulls with the runtime's blit
// kernels (hipMemcpyDeviceToDevice: __amd_rocclr_copyBuffer on the CUs), "ipc_sdma" with the SDMA
// copy engines (hipMemcpyDeviceToDeviceNoCU: no CUs beyond one-wave counter kernels, but slower
// than a blit between buffers of one device); bench.py times both (hip_face_copy, backends.cpp).
//
// Why a second device-resident transport next to RCCL: RCCL's p2p send/recv runs as kernels that
// occupy CUs the interior sweep wants, and RCCL refuses two ranks on one GPU. The ipc transport
// also runs with several processes on one device, which is how the device-resident multi-process
// path is tested on a one-GPU box (tests/test_gpu_ipc.py; share_gpu: a test-only opt-in, see
// ipc_shared_gpu_problem).
//
// Two protocols, by field-buffer size:
//   direct  (buffers below ~1.9 GiB, e.g. 1024^3 fp32 at N >= 4): each process exports its two
//           field buffers and pulls the neighbour's face straight out of them: one copy per face.
//   mailbox (larger buffers): the HIP runtime PyTorch bundles (ROCm 7.0) stalls forever in
//           hipIpcOpenMemHandle on an exported hipMalloc of 2 GiB or more (scripts/ipc_probe.py on
//           one MI355X: 1900 MiB maps at once, 2048 MiB and 2 GiB + 16 MiB stall with torch's
//           runtime loaded, and the same 2 GiB + 16 MiB maps at once under /opt/rocm 7.2's) — the
//           field buffer of a 1024^3 fp32 slab at N = 2 is 2 GiB + 16 MiB. Each process then
//           publishes its faces into a small exported mailbox (2 parities x 2 sides x `halo`
//           planes) with one local copy per face, and the neighbours pull from there.
// MDFX_IPC_DIRECT=0 / 1 forces one (ipc_direct_ok).
//
// Mailbox protocol for exchange e (every process calls exchange() the same number of times;
// e = 1, 2, ..) on the slab's halo stream, after the boundary kernels that wrote the faces of buffer b:
//
//   for each neighbour n:  wait(n.pulled[mine] >= e - 2)   n is done with mailbox slot b (exchange e-2)
//                          (>= e - 1 when exchange e-1 used the same parity b: a re-send of the
//                          current buffer after init() / write_owned(), so slot b was used last)
//   copy my faces of b -> mailbox[b][side]               (local)
//   signal(ready)                                        exchange e published
//   for each neighbour n:  wait(n.ready >= e)
//                          copy n.mailbox[b][other side] -> my ghost(b)
//                          signal(pulled[side])
//
// `pulled` starts at 2 so the first two exchanges need no special case. All counters live in
// device memory (private `expect` counters advance inside the wait kernel), so the enqueued work is
// identical for every exchange and a captured hipGraph replays correctly.
//
// Direct protocol for exchange e (same counters; `pulled` starts at 1):
//
//   signal(ready)                                        my faces of b are final
//   for each neighbour n:  wait(n.ready >= e)
//                          copy n.buf[b].face(other side) -> my ghost(b)
//                          signal(pulled[side])
//   for each neighbour n:  wait(n.pulled[mine] >= e - 1) n pulled exchange e-1, which sent the faces
//                                                        of buffer 1-b that the next step's boundary
//                                                        kernels overwrite (they follow this exchange)
//
// A re-sent parity (exchange_ghosts) needs no look-ahead here: the last wait is already the
// stronger condition.
//
// (z, y) pencils (direct protocol only) have four neighbours and exchange in two phases, because a
// z face spans the y ghost rows too (they carry the edge and corner cells of the 27-point stencil):
//
//   signal(ready)
//   for each y neighbour n:  wait(n.ready >= e); 2-D copy n's y face -> my ghost rows; signal(pulled[side])
//   signal(readyZ)                                        my y ghost rows of b landed
//   for each z neighbour n:  wait(n.readyZ >= e); copy n's z face -> my ghost planes; signal(pulled[side])
//   for each neighbour n:    wait(n.pulled[mine] >= e - 1)
//
// Reference parity: the per-element host-staged MPI_Send/MPI_Recv loops of
// MDF_kernel.cu:167-169,180-183 (D5, D12) with their rank-1 self-addressing (D3).
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "mdfx/devsync.hpp"
#include "mdfx/runtime.hpp"

namespace mdfx {

#define HIPC(x)                                                                          \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("HIP: ") + #x + " -> " + hipGetErrorString(e_)); \
  } while (0)

void ipc_enable_peer(int mine, int peer, int peer_rank);

namespace {

// Counter block (one uncached allocation per process), 64-bit words on separate 128-B lines.
constexpr int kReady = 0;                 // public: exchanges whose faces I published
constexpr int kPulled = 16;               // public: [kPulled + side] pulls I completed from side
constexpr int kExpReady = 48;             // private: [kExpReady + side]
constexpr int kExpPulled = 64;            // private: [kExpPulled + side]
constexpr int kReadyZ = 96;               // public: exchanges whose y ghost rows landed (pencils)
constexpr size_t kCounterBytes = 128 * 8;

struct IpcRecord {
  char magic[8];
  int32_t rank = -1, device = -1, pid = 0, direct = 0, pencil = 0, pad = 0;
  uint64_t face_bytes[4] = {0, 0, 0, 0};    // per side (z lo, z hi, y lo, y hi); the mailbox holds 4 z faces
  uint64_t face_off[4] = {0, 0, 0, 0};      // byte offsets of each face in the field buffers (direct)
  uint64_t face_stride[4] = {0, 0, 0, 0};   // bytes between a face's pieces (a y face: one per plane)
  char pci[32] = {0};       // PCI bus id of the device: a stable identity across HIP_VISIBLE_DEVICES
  hipIpcMemHandle_t mbox;   // (mailbox protocol)
  hipIpcMemHandle_t buf[2];  // the two field buffers (direct protocol)
  hipIpcMemHandle_t ctr;
};

}  // namespace

// IPC export of a fresh allocation. When engines are built and closed in turn by several processes
// on one GPU (bench.py's trial loop), the export of a new field buffer failed with "invalid
// argument" once in round 5 (8-process churn after the whole GPU tier, profiles/r05_session_ag/),
// although every rank had unmapped its neighbours' exports before any rank freed (~IpcTransport).
// Suspected cause, not confirmed: the runtime releases a closed import asynchronously, so a range
// a neighbour still held could be handed out again before the release. ~IpcTransport now waits
// for its closes (hipDeviceSynchronize) before the meeting that lets the neighbours free, and a
// failing export logs what is known about the pointer (its attributes, its allocation's range, and
// whether that range overlaps an import this process closed earlier) before a bounded retry (up to
// ~2 s), so the next occurrence names its cause. MDFX_IPC_EXPORT_FAIL=n makes the first n exports
// of the process fail with "invalid argument" (tests: the retry and logging path runs on demand).
namespace {
struct ClosedRange {
  uintptr_t base = 0;
  size_t size = 0;
};
std::vector<ClosedRange>& closed_imports() {
  static std::vector<ClosedRange> v;
  return v;
}
void note_closed_import(void* p) {
  void* base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, p) != hipSuccess) {
    (void)hipGetLastError();
    base = p;
    size = 1;
  }
  auto& v = closed_imports();
  if (v.size() >= 64) v.erase(v.begin());
  v.push_back(ClosedRange{(uintptr_t)base, size});
}
std::string export_diagnosis(void* p) {
  if (!p) return "null pointer";
  std::string out;
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) == hipSuccess)
    out += format("type %d device %d devicePointer %p", (int)at.type, at.device, at.devicePointer);
  else {
    (void)hipGetLastError();
    out += "no pointer attributes";
  }
  void* base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, p) == hipSuccess) {
    out += format("; allocation [%p, +%zu)", base, size);
    int hits = 0;
    for (const ClosedRange& c : closed_imports())
      if ((uintptr_t)base < c.base + c.size && c.base < (uintptr_t)base + size) ++hits;
    out += format("; overlaps %d import(s) this process closed earlier (of %zu recorded)", hits,
                  closed_imports().size());
  } else {
    (void)hipGetLastError();
    out += "; no allocation range";
  }
  return out;
}
int export_fail_budget() {
  static int n = [] {
    const char* v = std::getenv("MDFX_IPC_EXPORT_FAIL");
    return v && *v ? std::atoi(v) : 0;
  }();
  return n;
}
}  // namespace

int ipc_export_retry(const std::function<int()>& get, void* p, int max_retries, int sleep_us) {
  static int injected = 0;
  for (int i = 0;; ++i) {
    hipError_t e;
    if (injected < export_fail_budget()) {
      ++injected;
      e = hipErrorInvalidValue;
    } else {
      e = (hipError_t)get();
    }
    if (e == hipSuccess) {
      if (i > 0) std::fprintf(stderr, "mdfx ipc: hipIpcGetMemHandle succeeded after %d retries\n", i);
      return i;
    }
    if (i == 0) std::fprintf(stderr, "mdfx ipc: hipIpcGetMemHandle(%p) -> %s: %s; retrying\n", p,
                             hipGetErrorString(e), export_diagnosis(p).c_str());
    if (e != hipErrorInvalidValue || i >= max_retries)
      throw_error(__FILE__, __LINE__,
                  format("HIP: hipIpcGetMemHandle(%p) -> %s (after %d retries)", p, hipGetErrorString(e), i));
    (void)hipGetLastError();
    if (sleep_us > 0) usleep(sleep_us);
  }
}

namespace {

void ipc_export(hipIpcMemHandle_t* h, void* p) {
  (void)ipc_export_retry([&]() { return (int)hipIpcGetMemHandle(h, p); }, p, 80, 25000);
}

// This process's ordinal of the device with PCI bus id `pci` (-1 if it is not visible here).
int local_device_of(const char* pci) {
  if (!pci[0]) return -1;
  int d = -1;
  if (hipDeviceGetByPCIBusId(&d, pci) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return d;
}

class IpcTransport final : public Transport {
 public:
  IpcTransport(CallbackFns f, int copy_mode, bool share_gpu) : f_(std::move(f)), copy_(copy_mode), share_gpu_(share_gpu) {
    MDFX_CHECK((bool)f_.allgather, "ipc transport needs an allgather control plane");
  }
  ~IpcTransport() override {
    if (!dev_ok_) return;
    (void)hipSetDevice(self_.be->device());
    if (aux_) (void)hipStreamDestroy(aux_);
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    bool mapped = false;
    for (auto& p : peers_) {
      mapped = mapped || p.mbox || p.buf[0] || p.ctr;
      for (void* q : {p.mbox, p.buf[0], p.buf[1], p.ctr}) {
        if (!q) continue;
        note_closed_import(q);
        (void)hipIpcCloseMemHandle(q);
      }
    }
    // the closes complete before the meeting below lets the neighbours free what they exported
    if (mapped) (void)hipDeviceSynchronize();
    // Every rank unmaps its neighbours' exports before any rank frees its own (the engine frees the
    // field buffers right after this destructor). Without this meeting a rank could free and
    // re-allocate memory a neighbour still had mapped, and the next engine's hipIpcGetMemHandle on
    // the new buffer failed with "invalid argument" (round-4 8-process rehearsal of bench.py's
    // trial loop, which builds and closes engines in turn; scripts/ipc_churn.py). Skipped once the
    // transport was aborted (a peer may be gone).
    if (mapped && setup_done_ && !aborted_ && f_.barrier) {
      try {
        f_.barrier();
      } catch (...) {
      }
    }
    if (mbox_) (void)hipFree(mbox_);
    hip_free_uncached(ctr_);
    hip_words_free(words_);
  }
  const char* name() const override { return copy_ == 1 ? "ipc_sdma" : "ipc"; }
  bool in_process_only() const override { return false; }
  bool stream_ordered() const override { return true; }
  bool records_ghost_event() const override { return true; }
  void set_timeout(double s) override { timeout_s_ = s > 0 ? s : 300.0; }

  void setup(const std::vector<LocalSlab>& locals, int nranks) override {
    MDFX_CHECK(locals.size() == 1, "ipc transport: one slab per process");
    self_ = locals[0];
    nranks_ = nranks;
    pencil_ = self_.py > 1 && self_.lay.hy > 0;
    MDFX_CHECK(self_.be->kind() == DeviceKind::HIP, "ipc transport needs a HIP backend");
    self_.be->activate();
    ctr_ = (uint64_t*)hip_alloc_uncached(kCounterBytes);
    words_ = hip_words_alloc();  // this transport's own abort / wait-error words
    dev_ok_ = true;
    // the hi-side pull runs on a second stream, concurrently with the lo-side pull on the halo
    // stream: two neighbours are two different xGMI links (or two blits on one device)
    HIPC(hipStreamCreateWithPriority(&aux_, hipStreamNonBlocking, halo_stream_priority(true)));
    HIPC(hipEventCreateWithFlags(&ev_fork_, sync_event_flags()));
    HIPC(hipEventCreateWithFlags(&ev_join_, sync_event_flags()));
    // every face has the same size (halo planes of one field layout)
    face_ = (size_t)self_.lay.halo * self_.lay.plane_bytes();
    // the protocol is agreed below (every rank must use the same one); counters start per protocol
    const bool want_direct = ipc_direct_ok(self_.lay.bytes());

    IpcRecord mine;
    std::memcpy(mine.magic, "MDFXIPC4", 8);
    mine.rank = self_.rank;
    mine.device = self_.be->device();
    mine.pid = (int32_t)::getpid();
    mine.direct = want_direct ? 1 : 0;
    mine.pencil = pencil_ ? 1 : 0;
    for (int side = 0; side < 4; ++side) {
      const HaloSpan h = halo_span(self_, 0, side, nranks_);
      if (h.peer < 0) continue;
      mine.face_bytes[side] = h.bytes;
      mine.face_off[side] = (uint64_t)((char*)h.send - (char*)self_.buf[0]);
      mine.face_stride[side] = h.stride;
    }
    if (hipDeviceGetPCIBusId(mine.pci, (int)sizeof(mine.pci) - 1, mine.device) != hipSuccess) {
      (void)hipGetLastError();
      mine.pci[0] = 0;
    }
    ipc_export(&mine.ctr, ctr_);
    if (want_direct) {
      for (int b = 0; b < 2; ++b) ipc_export(&mine.buf[b], self_.buf[b]);
    }
    // the mailbox exists in both protocols (a rank that cannot go direct makes everyone fall back)
    HIPC(hipMalloc(&mbox_, 4 * face_));
    HIPC(hipMemset(mbox_, 0, 4 * face_));
    ipc_export(&mine.mbox, mbox_);
    HIPC(hipDeviceSynchronize());
    const std::vector<std::string> all =
        f_.allgather(std::string((const char*)&mine, sizeof(mine)));  // also the setup barrier
    MDFX_CHECK((int)all.size() == nranks_, format("ipc allgather returned %zu records for %d ranks", all.size(), nranks_));
    direct_ = true;
    bool any_pencil = false;
    std::vector<std::pair<int, std::string>> pid_pci;
    for (const std::string& rec : all) {
      MDFX_CHECK(rec.size() == sizeof(IpcRecord), "ipc: malformed handle record");
      IpcRecord r;
      std::memcpy(&r, rec.data(), sizeof(r));
      direct_ = direct_ && r.direct != 0;
      any_pencil = any_pencil || r.pencil != 0;
      r.pci[sizeof(r.pci) - 1] = 0;
      pid_pci.emplace_back(r.pid, std::string(r.pci));
    }
    const std::string shared = ipc_shared_gpu_problem(pid_pci, share_gpu_);
    MDFX_CHECK(shared.empty(), shared);
    // (every rank reaches the same verdict from the same records: all fail together)
    MDFX_CHECK(direct_ || !any_pencil, "ipc transport: a pencil decomposition needs the direct protocol (field buffers "
                                       "up to 1900 MiB on every rank, or MDFX_IPC_DIRECT=1)");
    const uint64_t pulled0 = direct_ ? 1 : 2;  // the first exchange(s) find their faces / slots free
    for (int side = 0; side < 4; ++side) HIPC(hipMemcpy(ctr_ + kPulled + side, &pulled0, 8, hipMemcpyHostToDevice));
    HIPC(hipDeviceSynchronize());

    for (int side = 0; side < 4; ++side) {
      Peer& p = peers_[side];
      p.rank = halo_span(self_, 0, side, nranks_).peer;
      if (p.rank < 0) continue;
      IpcRecord r;
      std::memcpy(&r, all[p.rank].data(), sizeof(r));
      // the neighbour's device as THIS process numbers it (PCI bus id): with per-rank
      // HIP_VISIBLE_DEVICES both sides call their GPU "device 0"
      const int their = local_device_of(r.pci);
      const bool same = mine.pci[0] && r.pci[0] ? std::strcmp(mine.pci, r.pci) == 0 : r.device == mine.device;
      // the neighbour's face that borders me is its opposite side's
      IpcPeerInfo me{mine.rank, mine.device, mine.pid, mine.face_bytes[side], true};
      IpcPeerInfo them{r.rank, same ? mine.device : (their >= 0 ? their : -1), r.pid, r.face_bytes[side ^ 1],
                       std::memcmp(r.magic, "MDFXIPC4", 8) == 0};
      int can = 1;
      if (!same && their >= 0) HIPC(hipDeviceCanAccessPeer(&can, mine.device, their));
      const std::string why = ipc_peer_problem(me, them, p.rank, can != 0);
      MDFX_CHECK(why.empty(), why);
      // explicit peer enable where the neighbour's GPU is visible here; otherwise the IPC open's
      // lazy peer mapping is all there is
      if (!same && their >= 0) ipc_enable_peer(mine.device, their, p.rank);
      if (direct_) {
        for (int b = 0; b < 2; ++b) {
          void* q = nullptr;
          HIPC(hipIpcOpenMemHandle(&q, r.buf[b], hipIpcMemLazyEnablePeerAccess));
          p.buf[b] = q;
        }
        p.face = halo_span(self_, 0, side, nranks_);  // its geometry as my ghost receives it ...
        p.face.stride = r.face_stride[side ^ 1];      // ... read at the neighbour's pitch
        p.face_off = r.face_off[side ^ 1];
      } else {
        HIPC(hipIpcOpenMemHandle(&p.mbox, r.mbox, hipIpcMemLazyEnablePeerAccess));
      }
      HIPC(hipIpcOpenMemHandle(&p.ctr, r.ctr, hipIpcMemLazyEnablePeerAccess));
    }
    f_.barrier ? f_.barrier() : (void)f_.allgather("");
    setup_done_ = true;
  }

  // mailbox slot of buffer parity b, side s (0 = lo, 1 = hi), in a process's mailbox
  char* slot(void* mbox, int b, int s) const { return (char*)mbox + (size_t)(2 * b + s) * face_; }

  void exchange(int b) override {
    self_.be->activate();
    hipStream_t hs = (hipStream_t)self_.halo_stream;
    // inside a graph capture the pair alternates parities and the engine replays it only after an
    // exchange of the other parity: no look-ahead, and last_b_ tracks real (eager) exchanges only
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPC(hipStreamIsCapturing(hs, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    // the two pulls: lo side on the halo stream, hi side on the aux stream (fused_pulls; pencils:
    // phase below), joined back before the exchange ends
    if (direct_) {
      // one pair of faces: the lo side's pull on the halo stream, the hi side's on the aux stream.
      // After the last pair the ghosts are complete: the ghost event goes on the halo stream right
      // after both pulls, ahead of the pulled signals and of the waits for the neighbours' pulls
      // of my faces (only the sweep after next overwrites those; the halo stream still orders it)
      auto phase = [&](int s0, int ready, bool last) {
        const bool two = peers_[s0].rank >= 0 && peers_[s0 + 1].rank >= 0;
        if (two) {
          HIPC(hipEventRecord(ev_fork_, hs));
          HIPC(hipStreamWaitEvent(aux_, ev_fork_, 0));
        }
        for (int side = s0; side < s0 + 2; ++side) {
          const Peer& p = peers_[side];
          if (p.rank < 0) continue;
          const HaloSpan mine = halo_span(self_, b, side, nranks_);
          MDFX_CHECK(mine.peer == p.rank, "ipc: neighbour mismatch");
          hipStream_t ps = two && side == s0 + 1 ? aux_ : hs;
          hip_counter_wait((const uint64_t*)p.ctr + ready, ctr_ + kExpReady + side, timeout_s_, ps, 0, &words_);
          hip_face_copy(mine.recv, mine, (const char*)p.buf[b] + p.face_off, p.face, ps, copy_);
        }
        if (last && self_.ghost_event) {  // (each pull's own stream: no join on the critical path)
          HIPC(hipEventRecord((hipEvent_t)self_.ghost_event, hs));
          HIPC(hipEventRecord((hipEvent_t)self_.ghost_event2, two ? aux_ : hs));
        }
        for (int side = s0; side < s0 + 2; ++side) {
          if (peers_[side].rank < 0) continue;
          hip_counter_signal(ctr_ + kPulled + side, two && side == s0 + 1 ? aux_ : hs);
        }
        if (two) {
          HIPC(hipEventRecord(ev_join_, aux_));
          HIPC(hipStreamWaitEvent(hs, ev_join_, 0));
        }
      };
      if (pencil_) {
        hip_counter_signal(ctr_ + kReady, hs);
        // y faces first; readyZ tells the z neighbours my y ghost rows (inside my z faces) landed
        phase(2, kReady, false);
        hip_counter_signal(ctr_ + kReadyZ, hs);
        phase(0, kReadyZ, true);
      } else {
        fused_pulls(b, [&](int side) { return (const char*)peers_[side].buf[b] + peers_[side].face_off; },
                    [&](int side) { return peers_[side].face; });
      }
      for (int side = 0; side < 4; ++side) {
        const Peer& p = peers_[side];
        if (p.rank < 0) continue;
        hip_counter_wait((const uint64_t*)p.ctr + kPulled + (side ^ 1), ctr_ + kExpPulled + side, timeout_s_, hs, 0,
                         &words_);
      }
      if (!capturing) last_b_ = b;
      return;
    }
    const uint64_t ahead = (!capturing && last_b_ == b) ? 1 : 0;
    // publish: the neighbour on `side` must be done with slot b (exchange e-2) before it is reused
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      const HaloSpan mine = halo_span(self_, b, side, nranks_);
      MDFX_CHECK(mine.bytes == face_ && mine.peer == p.rank, "ipc: face geometry mismatch");
      hip_counter_wait((const uint64_t*)p.ctr + kPulled + (1 - side), ctr_ + kExpPulled + side, timeout_s_, hs,
                       ahead, &words_);
      hip_face_copy(slot(mbox_, b, side), mine.send, face_, hs, copy_);
    }
    fused_pulls(b, [&](int side) { return (const char*)slot(peers_[side].mbox, b, 1 - side); },
                [&](int side) { return halo_span(self_, b, side, nranks_); });
    if (!capturing) last_b_ = b;
  }
  // The slab pulls (both protocols) with the ready signal fused into the first halo-stream wait: the
  // hi-side pull's stream forks off BEFORE the signal, so its wait for the upper neighbour runs
  // beside the signal, and the halo stream's signal and lo-side wait are one dispatch. Round 6
  // rank-proxy traces (profiles/r06_session_{f,g}/): signal (6 us) -> 8 us launch gap -> wait (9 us)
  // -> pull put the pulls 22 us behind the fold wait's end, fused 16 us (N = 2 / 4 proxies +0.3-0.8
  // %, N = 8 within noise). src(side) / span(side): where the face comes from (the neighbour's field
  // buffer or its mailbox slot) and its geometry.
  template <class Src, class Span>
  void fused_pulls(int b, Src src, Span span) {
    hipStream_t hs = (hipStream_t)self_.halo_stream;
    const bool two = peers_[0].rank >= 0 && peers_[1].rank >= 0;
    if (two) {
      HIPC(hipEventRecord(ev_fork_, hs));
      HIPC(hipStreamWaitEvent(aux_, ev_fork_, 0));
    }
    bool signalled = false;
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      const HaloSpan mine = halo_span(self_, b, side, nranks_);
      MDFX_CHECK(mine.peer == p.rank, "ipc: neighbour mismatch");
      hipStream_t ps = two && side == 1 ? aux_ : hs;
      if (ps == hs && !signalled) {
        hip_counter_signal_wait(ctr_ + kReady, (const uint64_t*)p.ctr + kReady, ctr_ + kExpReady + side, timeout_s_,
                                hs, 0, &words_);
        signalled = true;
      } else {
        hip_counter_wait((const uint64_t*)p.ctr + kReady, ctr_ + kExpReady + side, timeout_s_, ps, 0, &words_);
      }
      hip_face_copy(mine.recv, mine, src(side), span(side), ps, copy_);
    }
    if (!signalled) hip_counter_signal(ctr_ + kReady, hs);
    if (self_.ghost_event) {  // (each pull's own stream: no join on the critical path)
      HIPC(hipEventRecord((hipEvent_t)self_.ghost_event, hs));
      HIPC(hipEventRecord((hipEvent_t)self_.ghost_event2, two ? aux_ : hs));
    }
    for (int side = 0; side < 2; ++side)
      if (peers_[side].rank >= 0) hip_counter_signal(ctr_ + kPulled + side, two && side == 1 ? aux_ : hs);
    if (two) {
      HIPC(hipEventRecord(ev_join_, aux_));
      HIPC(hipStreamWaitEvent(hs, ev_join_, 0));
    }
  }

  std::string debug_state() override {
    if (!dev_ok_ || !ctr_) return "";
    self_.be->activate();
    uint64_t c[128] = {0};
    if (!hip_read_words(c, ctr_, sizeof(c), 2.0)) return "ipc: counters unreadable";
    std::string out = format("ipc rank %d (%s): ready %llu readyZ %llu", self_.rank, direct_ ? "direct" : "mailbox",
                             (unsigned long long)c[kReady], (unsigned long long)c[kReadyZ]);
    for (int side = 0; side < 4; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      uint64_t r[128] = {0};
      const bool ok = p.ctr && hip_read_words(r, p.ctr, sizeof(r), 2.0);
      out += format("; side %d (rank %d): pulled %llu expReady %llu expPulled %llu | its ready %lld readyZ %lld "
                    "pulled[mine] %lld",
                    side, p.rank, (unsigned long long)c[kPulled + side], (unsigned long long)c[kExpReady + side],
                    (unsigned long long)c[kExpPulled + side], ok ? (long long)r[kReady] : -1LL,
                    ok ? (long long)r[kReadyZ] : -1LL, ok ? (long long)r[kPulled + (side ^ 1)] : -1LL);
    }
    return out;
  }
  void set_last_parity(int b) override { last_b_ = b; }
  // a captured 2-exchange cycle bakes the look-ahead of its first wait: the engine replays one only
  // when the exchange before it used the other parity (Solver::run)
  int last_parity() const override { return last_b_; }

  double allreduce_sum(double v) override { return f_.allreduce_sum ? f_.allreduce_sum(v) : v; }
  double allreduce_max(double v) override { return f_.allreduce_max ? f_.allreduce_max(v) : v; }
  void barrier() override {
    if (f_.barrier) f_.barrier();
  }
  void check() override {
    if (!words_.host) return;
    if (words_.wait_error())
      MDFX_FAIL(format("ipc transport: rank %d timed out after %.0f s waiting for a neighbour's halo counter "
                       "(a peer process died or hung)", self_.rank, timeout_s_));
    if (words_.abort_raised())
      MDFX_FAIL(format("ipc transport: rank %d was aborted; its halo copies are no longer ordered", self_.rank));
  }
  void abort() override {
    aborted_ = true;
    if (words_.host) words_.set_abort(1);
  }

 private:
  struct Peer {
    int rank = -1;
    void* mbox = nullptr;
    void* buf[2] = {nullptr, nullptr};  // the neighbour's field buffers (direct protocol)
    uint64_t face_off = 0;              // byte offset of its face that borders this slab
    HaloSpan face;                      // that face's geometry (width, height, the neighbour's stride)
    void* ctr = nullptr;
  };
  CallbackFns f_;
  int copy_ = 0;  // face copy engine: 0 blit kernels, 1 SDMA (hip_face_copy)
  hipStream_t aux_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  LocalSlab self_;
  int nranks_ = 1;
  uint64_t* ctr_ = nullptr;
  HipWords words_;
  int last_b_ = -1;  // parity of the previous exchange
  void* mbox_ = nullptr;
  size_t face_ = 0;
  bool dev_ok_ = false;
  bool direct_ = false;
  bool pencil_ = false;  // (z, y) pencil: y faces first, then the z faces (which carry the y ghosts)
  bool setup_done_ = false, aborted_ = false, share_gpu_ = false;
  Peer peers_[4];
  double timeout_s_ = 300.0;
};

}  // namespace

std::string ipc_peer_problem(const IpcPeerInfo& mine, const IpcPeerInfo& peer, int expect_rank, bool peer_access) {
  if (!peer.magic_ok || peer.rank != expect_rank)
    return format("ipc: handle record mismatch (expected rank %d, got %d)", expect_rank, peer.rank);
  if (peer.pid == mine.pid) return "ipc transport: neighbouring slabs must live in different processes";
  if (peer.face_bytes != mine.face_bytes)
    return format("ipc: neighbour face size %llu does not match this slab's %llu", (unsigned long long)peer.face_bytes,
                  (unsigned long long)mine.face_bytes);
  if (peer.device != mine.device && !peer_access)
    return format("ipc transport: device %d cannot access device %d (rank %d's) with peer copies over xGMI / PCIe; "
                  "use --transport rccl", mine.device, peer.device, peer.rank);
  return "";
}

// A neighbour on another GPU is reached by peer copies over xGMI: enable peer access explicitly
// (an already-enabled pair is fine) instead of relying on the lazy mapping of the IPC open.
void ipc_enable_peer(int mine, int peer, int peer_rank) {
  if (mine == peer) return;
  int cur = 0;
  HIPC(hipGetDevice(&cur));
  HIPC(hipSetDevice(mine));
  const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  (void)hipSetDevice(cur);
  if (e == hipErrorPeerAccessAlreadyEnabled) {
    (void)hipGetLastError();  // clear the "already enabled" status
    return;
  }
  if (e != hipSuccess)
    MDFX_FAIL(format("ipc transport: enabling peer access from device %d to device %d (rank %d) failed: %s", mine,
                     peer, peer_rank, hipGetErrorString(e)));
}

// The direct protocol maps the neighbours' field buffers; torch's HIP 7.0 runtime stalls in
// hipIpcOpenMemHandle from 2 GiB up, so only buffers of at most 1900 MiB (probed good) go direct.

bool ipc_direct_ok(size_t field_bytes) {
  const char* v = std::getenv("MDFX_IPC_DIRECT");  // (read per call: tests switch it within a process)
  const int force = v && *v ? std::atoi(v) : -1;
  if (force >= 0) return force != 0;
  return field_bytes <= ((size_t)1900 << 20);
}

std::string ipc_shared_gpu_problem(const std::vector<std::pair<int, std::string>>& pid_pci, bool share_gpu) {
  if (share_gpu) return "";
  for (size_t i = 0; i < pid_pci.size(); ++i)
    for (size_t j = i + 1; j < pid_pci.size(); ++j) {
      const auto& a = pid_pci[i];
      const auto& b = pid_pci[j];
      if (a.second.empty() || a.second != b.second || a.first == b.first) continue;
      return format("ipc transport: ranks %zu and %zu are two engine processes on one GPU (%s). Their halo "
                    "exchange waits on device counters that need the hardware scheduler to run every producer "
                    "queue, which several processes oversubscribing one GPU do not guarantee: run one process "
                    "per GPU (share_gpu=True / bench.py --share-gpu allow it for tests)",
                    i, j, a.second.c_str());
    }
  return "";
}

std::unique_ptr<Transport> make_ipc_transport(CallbackFns fns, int copy_mode, bool share_gpu) {
  return std::unique_ptr<Transport>(
      new IpcTransport(std::move(fns), copy_mode < 0 ? face_copy_mode() : copy_mode, share_gpu));
}

}  // namespace mdfx
