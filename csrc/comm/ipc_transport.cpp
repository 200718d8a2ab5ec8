// HIP-IPC halo transport: one process per slab, faces pulled straight out of the neighbour's
// device buffers (mapped with hipIpcOpenMemHandle) by the copy engines, ordered by device-side
// counters instead of host synchronisation.
//
// Why a second device-resident transport next to RCCL: RCCL's p2p send/recv runs as kernels that
// occupy CUs the interior sweep wants, and RCCL refuses two ranks on one GPU. A pull through the
// copy engine (SDMA over xGMI across GPUs, or a blit on the same GPU) takes no CUs beyond a
// one-wave counter kernel, and works for any number of processes sharing a device — which is how
// the device-resident multi-process path is tested on a one-GPU box (tests/test_gpu_ipc.py).
//
// Protocol for exchange e (every process calls exchange() the same number of times; e = 1, 2, ..)
// on the slab's halo stream, after the boundary kernels that wrote the faces of buffer b:
//
//   signal(ready)                                   faces of b published
//   for each neighbour n:  wait(n.ready >= e)        n's faces of b published
//                          copy n.face(b) -> my ghost(b)
//                          signal(pulled[side])      I am done reading n's buffer b
//   for each neighbour n:  wait(n.pulled[mine] >= e-1)
//
// The last wait keeps the next boundary kernel (which rewrites the faces of buffer 1-b, sent in
// exchange e-1) from overwriting faces a neighbour has not pulled yet; `pulled` starts at 1 so the
// first exchange needs no special case. All counters live in device memory (private `expect`
// counters advance inside the wait kernel), so the enqueued work is identical for every exchange
// and a captured hipGraph replays correctly.
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
  uint64_t bytes = 0;  // per field buffer
  hipIpcMemHandle_t buf[2];
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
      for (void* q : p.buf)
        if (q) (void)hipIpcCloseMemHandle(q);
      if (p.ctr) (void)hipIpcCloseMemHandle(p.ctr);
    }
    hip_free_uncached(ctr_);
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
    const uint64_t one = 1;
    HIPC(hipMemcpy(ctr_ + kPulled + 0, &one, 8, hipMemcpyHostToDevice));
    HIPC(hipMemcpy(ctr_ + kPulled + 1, &one, 8, hipMemcpyHostToDevice));
    HIPC(hipDeviceSynchronize());
    dev_ok_ = true;

    IpcRecord mine;
    std::memcpy(mine.magic, "MDFXIPC1", 8);
    mine.rank = self_.rank;
    mine.device = self_.be->device();
    mine.pid = (int32_t)::getpid();
    mine.bytes = self_.lay.bytes();
    HIPC(hipIpcGetMemHandle(&mine.buf[0], self_.buf[0]));
    HIPC(hipIpcGetMemHandle(&mine.buf[1], self_.buf[1]));
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
      MDFX_CHECK(std::memcmp(r.magic, "MDFXIPC1", 8) == 0 && r.rank == p.rank, "ipc: handle record mismatch");
      MDFX_CHECK(r.pid != mine.pid, "ipc transport: neighbouring slabs must live in different processes");
      for (int b = 0; b < 2; ++b)
        HIPC(hipIpcOpenMemHandle(&p.buf[b], r.buf[b], hipIpcMemLazyEnablePeerAccess));
      HIPC(hipIpcOpenMemHandle(&p.ctr, r.ctr, hipIpcMemLazyEnablePeerAccess));
      p.device = r.device;
      // the neighbour's slab, addressed through the mapped buffers
      p.slab.rank = p.rank;
      p.slab.lay = FieldLayout::make(self_.lay.global, dec.z0(p.rank), dec.z1(p.rank), self_.lay.halo, self_.lay.dtype);
      MDFX_CHECK(p.slab.lay.bytes() == r.bytes, "ipc: neighbour buffer size does not match its layout");
      p.slab.buf[0] = p.buf[0];
      p.slab.buf[1] = p.buf[1];
    }
    f_.barrier ? f_.barrier() : (void)f_.allgather("");
  }

  void exchange(int b) override {
    self_.be->activate();
    void* hs = self_.halo_stream;
    hip_counter_signal(ctr_ + kReady, hs);
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      const HaloSpan mine = halo_span(self_, b, side, nranks_);
      const HaloSpan theirs = halo_span(p.slab, b, 1 - side, nranks_);
      MDFX_CHECK(mine.bytes == theirs.bytes && mine.peer == p.rank, "ipc: face geometry mismatch");
      hip_counter_wait((const uint64_t*)p.ctr + kReady, ctr_ + kExpReady + side, timeout_s_, hs);
      HIPC(hipMemcpyAsync(mine.recv, theirs.send, mine.bytes, hipMemcpyDeviceToDevice, (hipStream_t)hs));
      hip_counter_signal(ctr_ + kPulled + side, hs);
    }
    for (int side = 0; side < 2; ++side) {
      const Peer& p = peers_[side];
      if (p.rank < 0) continue;
      // the neighbour on `side` pulls from me as its (1 - side) neighbour
      hip_counter_wait((const uint64_t*)p.ctr + kPulled + (1 - side), ctr_ + kExpPulled + side, timeout_s_, hs);
    }
  }

  double allreduce_sum(double v) override { return f_.allreduce_sum ? f_.allreduce_sum(v) : v; }
  double allreduce_max(double v) override { return f_.allreduce_max ? f_.allreduce_max(v) : v; }
  void barrier() override {
    if (f_.barrier) f_.barrier();
  }
  void check() override {
    if (hip_wait_error())
      MDFX_FAIL(format("ipc transport: rank %d timed out after %.0f s waiting for a neighbour's halo counter "
                       "(a peer process died or hung)", self_.rank, timeout_s_));
  }
  void abort() override { hip_set_abort(1); }

 private:
  struct Peer {
    int rank = -1;
    int device = -1;
    void* buf[2] = {nullptr, nullptr};
    void* ctr = nullptr;
    LocalSlab slab;
  };
  CallbackFns f_;
  LocalSlab self_;
  int nranks_ = 1;
  uint64_t* ctr_ = nullptr;
  bool dev_ok_ = false;
  Peer peers_[2];
  double timeout_s_ = 300.0;
};

}  // namespace

std::unique_ptr<Transport> make_ipc_transport(CallbackFns fns) {
  return std::unique_ptr<Transport>(new IpcTransport(std::move(fns)));
}

}  // namespace mdfx
