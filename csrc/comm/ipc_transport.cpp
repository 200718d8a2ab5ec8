// HIP-IPC halo transport: one process per slab; each process publishes its boundary faces in a
// small exported "mailbox" allocation, and the neighbours pull them straight into their ghost
// planes with the copy engines, ordered by device-side counters instead of host synchronisation.
//
// Why a second device-resident transport next to RCCL: RCCL's p2p send/recv runs as kernels that
// occupy CUs the interior sweep wants, and RCCL refuses two ranks on one GPU. A pull through the
// copy engine (SDMA over xGMI across GPUs, or a blit on the same GPU) takes no CUs beyond a
// one-wave counter kernel, and works for any number of processes sharing a device — which is how
// the device-resident multi-process path is tested on a one-GPU box (tests/test_gpu_ipc.py).
//
// Why mailboxes instead of mapping the neighbours' whole field buffers: only the faces ever cross
// a process boundary, and the HIP runtime PyTorch bundles (ROCm 7.0) stalls forever in
// hipIpcOpenMemHandle on an exported hipMalloc of 2 GiB or more (scripts/ipc_probe.py on one
// MI355X: 1900 MiB maps at once, 2048 MiB and 2 GiB + 16 MiB stall with torch's runtime loaded,
// and the same 2 GiB + 16 MiB maps at once under /opt/rocm 7.2's) — the field buffer of a 1024^3
// fp32 slab at N = 2 is 2 GiB + 16 MiB. A mailbox holds 2 parities x 2 sides x
// `halo` planes (32 MiB at 1024^2 fp32, K = 2); publishing costs one local D2D copy per face.
//
// Protocol for exchange e (every process calls exchange() the same number of times; e = 1, 2, ..)
// on the slab's halo stream, after the boundary kernels that wrote the faces of buffer b:
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
// Reference parity: the per-element host-staged MPI_Send/MPI_Recv loops of
// MDF_kernel.cu:167-169,180-183 (D5, D12) with their rank-1 self-addressing (D3).
#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <cstring>

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
constexpr size_t kCounterBytes = 128 * 8;

struct IpcRecord {
  char magic[8];
  int32_t rank = -1, device = -1, pid = 0, pad = 0;
  uint64_t face_bytes = 0;  // one face (halo planes); the mailbox holds 4
  hipIpcMemHandle_t mbox;
  hipIpcMemHandle_t ctr;
};

class IpcTransport final : public Transport {
 public:
  explicit IpcTransport(CallbackFns f) : f_(std::move(f)) {
    MDFX_CHECK((bool)f_.allgather, "ipc transport needs an allgather control plane");
  }
  ~IpcTransport() override {
    if (!dev_ok_) return;
    (void)hipSetDevice(self_.be->device());
    for (auto& p : peers_) {
      if (p.mbox) (void)hipIpcCloseMemHandle(p.mbox);
      if (p.ctr) (void)hipIpcCloseMemHandle(p.ctr);
    }
    if (mbox_) (void)hipFree(mbox_);
    hip_free_uncached(ctr_);
    hip_words_free(words_);
  }
  const char* name() const override { return "ipc"; }
  bool in_process_only() const override { return false; }
  bool graph_capturable() const override { return true; }
  void set_timeout(double s) override { timeout_s_ = s > 0 ? s : 300.0; }

  void setup(const std::vector<LocalSlab>& locals, int nranks) override {
    MDFX_CHECK(locals.size() == 1, "ipc transport: one slab per process");
    self_ = locals[0];
    nranks_ = nranks;
    MDFX_CHECK(self_.be->kind() == DeviceKind::HIP, "ipc transport needs a HIP backend");
    self_.be->activate();
    ctr_ = (uint64_t*)hip_alloc_uncached(kCounterBytes);
    words_ = hip_words_alloc();  // this transport's own abort / wait-error words
    const uint64_t two = 2;  // exchanges 1 and 2 find their mailbox slot free
    HIPC(hipMemcpy(ctr_ + kPulled + 0, &two, 8, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(ctr_ + kPulled + 1, &two, 8, hipMemcpyHostToDevice));
    dev_ok_ = true;
    // every face has the same size (halo planes of one field layout)
    face_ = (size_t)self_.lay.halo * self_.lay.plane_bytes();
    HIPC(hipMalloc(&mbox_, 4 * face_));
    HIPC(hipMemset(mbox_, 0, 4 * face_));
    HIPC(hipDeviceSynchronize());

    IpcRecord mine;
    std::memcpy(mine.magic, "MDFXIPC2", 8);
    mine.rank = self_.rank;
    mine.device = self_.be->device();
    mine.pid = (int32_t)::getpid();
    mine.face_bytes = face_;
    HIPC(hipIpcGetMemHandle(&mine.mbox, mbox_));
    HIPC(hipIpcGetMemHandle(&mine.ctr, ctr_));
    const std::vector<std::string> all =
        f_.allgather(std::string((const char*)&mine, sizeof(mine)));  // also the setup barrier
    MDFX_CHECK((int)all.size() == nranks_, format("ipc allgather returned %zu records for %d ranks", all.size(), nranks_));

    const SlabDecomposition dec(self_.lay.global.nz, nranks_);
    for (int side = 0; side < 2; ++side) {
      Peer& p = peers_[side];
      p.rank = side == 0 ? dec.lo_neighbor(self_.rank) : dec.hi_neighbor(self_.rank);
      if (p.rank < 0) continue;
      IpcRecord r;
      MDFX_CHECK(all[p.rank].size() == sizeof(IpcRecord), "ipc: malformed handle record");
      std::memcpy(&r, all[p.rank].data(), sizeof(r));
      IpcPeerInfo me{mine.rank, mine.device, mine.pid, mine.face_bytes, true};
      IpcPeerInfo them{r.rank, r.device, r.pid, r.face_bytes, std::memcmp(r.magic, "MDFXIPC2", 8) == 0};
      int can = 1;
      if (r.device != mine.device) HIPC(hipDeviceCanAccessPeer(&can, mine.device, r.device));
      const std::string why = ipc_peer_problem(me, them, p.rank, can != 0);
      MDFX_CHECK(why.empty(), why);
      ipc_enable_peer(mine.device, r.device, p.rank);
      HIPC(hipIpcOpenMemHandle(&p.mbox, r.mbox, hipIpcMemLazyEnablePeerAccess));
      HIPC(hipIpcOpenMemHandle(&p.ctr, r.ctr, hipIpcMemLazyEnablePeerAccess));
      p.device = r.device;
    }
    f_.barrier ? f_.barrier() : (void)f_.allgather("");
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
    const uint64_t ahead = (!capturing && last_b_ == b) ? 1 : 0;
    // publish: the neighbour on `side` must be done with slot b (exchange e-2) before it is reused
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      const HaloSpan mine = halo_span(self_, b, side, nranks_);
      MDFX_CHECK(mine.bytes == face_ && mine.peer == p.rank, "ipc: face geometry mismatch");
      hip_counter_wait((const uint64_t*)p.ctr + kPulled + (1 - side), ctr_ + kExpPulled + side, timeout_s_, hs,
                       ahead, &words_);
      HIPC(hipMemcpyAsync(slot(mbox_, b, side), mine.send, face_, hipMemcpyDeviceToDevice, hs));
    }
    hip_counter_signal(ctr_ + kReady, hs);
    // pull: the neighbour on `side` published its (1 - side) face of exchange e
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      const HaloSpan mine = halo_span(self_, b, side, nranks_);
      hip_counter_wait((const uint64_t*)p.ctr + kReady, ctr_ + kExpReady + side, timeout_s_, hs, 0, &words_);
      HIPC(hipMemcpyAsync(mine.recv, slot(p.mbox, b, 1 - side), face_, hipMemcpyDeviceToDevice, hs));
      hip_counter_signal(ctr_ + kPulled + side, hs);
    }
    if (!capturing) last_b_ = b;
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
    if (words_.host) words_.set_abort(1);
  }

 private:
  struct Peer {
    int rank = -1;
    int device = -1;
    void* mbox = nullptr;
    void* ctr = nullptr;
  };
  CallbackFns f_;
  LocalSlab self_;
  int nranks_ = 1;
  uint64_t* ctr_ = nullptr;
  HipWords words_;
  int last_b_ = -1;  // parity of the previous exchange
  void* mbox_ = nullptr;
  size_t face_ = 0;
  bool dev_ok_ = false;
  Peer peers_[2];
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

std::unique_ptr<Transport> make_ipc_transport(CallbackFns fns) {
  return std::unique_ptr<Transport>(new IpcTransport(std::move(fns)));
}

}  // namespace mdfx
