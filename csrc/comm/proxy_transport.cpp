// Rank-proxy halo transport: ONE slab (or pencil) of an N-way decomposition, alone on one GPU,
// exchanging with itself through the ipc transport's machinery.
//
// Purpose: measure on a single MI355X what each GPU of an N-GPU run does per step, which the
// one-GPU pool cannot otherwise show (the whole-node bench is the driver's). The slab is exactly
// rank r's (its owned planes of the global grid plus K ghost planes per side), the engine runs its
// real schedule (both boundary regions on the halo stream, the interior on the compute stream,
// event joins, graph replay), and every exchange moves the same bytes through the same stream work
// as an ipc exchange between processes: per face a publish copy into a mailbox slot, a "ready"
// counter signal, a device counter wait, a pull copy from the mailbox into the ghost planes and a
// "pulled" signal (ipc_transport.cpp). The only difference is where the pulled face comes from:
// the slab's own mailbox (its own face, copied into its own ghost) instead of the neighbour's, so
// the copies run at local HBM speed instead of over xGMI, and the ghost values are not the
// neighbour's. Results are therefore exact only at planes farther from a proxied boundary than the
// steps run (tests/test_gpu_proxy.py), and every number measured this way is labelled a proxy.
// The two ipc protocols are both modelled: the mailbox (publish copy + pull copy per face) and the
// direct pull from the field buffer (one copy per face), chosen by the same rule as the ipc
// transport (ipc_direct_ok: field buffers below 2 GiB) or forced with MDFX_IPC_DIRECT=0 / 1.
//
// Reference parity: the per-rank generation loop of MDF_kernel.cu:155-188 (C12/C13) with its
// halo exchange MDF_kernel.cu:166-172,180-183, measured for one rank at a time.
#include <hip/hip_runtime_api.h>

#include "mdfx/devsync.hpp"
#include "mdfx/runtime.hpp"

namespace mdfx {

#define HIPC(x)                                                                          \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("HIP: ") + #x + " -> " + hipGetErrorString(e_)); \
  } while (0)

namespace {

// counter block layout as the ipc transport's (64-bit words on separate 128-B lines)
constexpr int kReady = 0, kPulled = 16, kExpReady = 48, kExpPulled = 64, kReadyZ = 96;
constexpr size_t kCounterBytes = 128 * 8;

class ProxyTransport final : public Transport {
 public:
  explicit ProxyTransport(int copy_mode) : copy_(copy_mode) {}
  ~ProxyTransport() override {
    if (!ok_) return;
    (void)hipSetDevice(self_.be->device());
    if (aux_) (void)hipStreamDestroy(aux_);
    if (ev_fork_) (void)hipEventDestroy(ev_fork_);
    if (ev_join_) (void)hipEventDestroy(ev_join_);
    if (mbox_) (void)hipFree(mbox_);
    hip_free_uncached(ctr_);
    hip_words_free(words_);
  }
  const char* name() const override { return "proxy"; }
  bool stream_ordered() const override { return true; }
  bool records_ghost_event() const override { return true; }
  void set_timeout(double s) override { timeout_s_ = s > 0 ? s : 300.0; }

  void setup(const std::vector<LocalSlab>& locals, int nranks) override {
    MDFX_CHECK(locals.size() == 1, "proxy transport: exactly one slab (rank r of an N-way split) per process");
    self_ = locals[0];
    nranks_ = nranks;
    MDFX_CHECK(self_.be->kind() == DeviceKind::HIP, "proxy transport needs a HIP backend");
    self_.be->activate();
    ctr_ = (uint64_t*)hip_alloc_uncached(kCounterBytes);
    words_ = hip_words_alloc();
    face_ = (size_t)self_.lay.halo * self_.lay.plane_bytes();
    direct_ = ipc_direct_ok(self_.lay.bytes());
    pencil_ = self_.py > 1 && self_.lay.hy > 0;
    MDFX_CHECK(direct_ || !pencil_, "proxy transport: a pencil needs the direct protocol (field buffers up to 1900 MiB "
                                    "or MDFX_IPC_DIRECT=1)");
    // the first exchange(s) find their faces (direct) / mailbox slots free
    const uint64_t pulled0 = direct_ ? 1 : 2;
    for (int side = 0; side < 4; ++side) HIPC(hipMemcpy(ctr_ + kPulled + side, &pulled0, 8, hipMemcpyHostToDevice));
    if (!direct_) {
      HIPC(hipMalloc(&mbox_, 4 * face_));
      HIPC(hipMemset(mbox_, 0, 4 * face_));
    }
    HIPC(hipStreamCreateWithPriority(&aux_, hipStreamNonBlocking, halo_stream_priority(true)));
    HIPC(hipEventCreateWithFlags(&ev_fork_, sync_event_flags()));
    HIPC(hipEventCreateWithFlags(&ev_join_, sync_event_flags()));
    HIPC(hipDeviceSynchronize());
    ok_ = true;
  }

  char* slot(int b, int s) const { return (char*)mbox_ + (size_t)(2 * b + s) * face_; }

  void exchange(int b) override {
    self_.be->activate();
    hipStream_t hs = (hipStream_t)self_.halo_stream;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIPC(hipStreamIsCapturing(hs, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    const uint64_t ahead = (!capturing && last_b_ == b) ? 1 : 0;
    // the ipc transport's stream layout: per pair of faces the hi-side pull on a second stream,
    // concurrent with the lo-side pull on the halo stream
    // (the ghost event after the last pair's pulls, as in the ipc transport)
    auto phase = [&](int s0, int ready, bool last) {
      const bool both = halo_span(self_, b, s0, nranks_).peer >= 0 &&
                        halo_span(self_, b, s0 + 1, nranks_).peer >= 0;
      if (both) {
        HIPC(hipEventRecord(ev_fork_, hs));
        HIPC(hipStreamWaitEvent(aux_, ev_fork_, 0));
      }
      for (int side = s0; side < s0 + 2; ++side) {
        const HaloSpan h = halo_span(self_, b, side, nranks_);
        if (h.peer < 0) continue;
        hipStream_t ps = both && side == s0 + 1 ? aux_ : hs;
        hip_counter_wait(ctr_ + ready, ctr_ + kExpReady + side, timeout_s_, ps, 0, &words_);
        hip_face_copy(h.recv, h, h.send, h, ps, copy_);
      }
      if (last && self_.ghost_event) {  // (each pull's own stream: no join on the critical path)
        HIPC(hipEventRecord((hipEvent_t)self_.ghost_event, hs));
        HIPC(hipEventRecord((hipEvent_t)self_.ghost_event2, both ? aux_ : hs));
      }
      for (int side = s0; side < s0 + 2; ++side) {
        if (halo_span(self_, b, side, nranks_).peer < 0) continue;
        hip_counter_signal(ctr_ + kPulled + side, both && side == s0 + 1 ? aux_ : hs);
      }
      if (both) {
        HIPC(hipEventRecord(ev_join_, aux_));
        HIPC(hipStreamWaitEvent(hs, ev_join_, 0));
      }
    };
    const bool both = halo_span(self_, b, 0, nranks_).peer >= 0 &&
                      halo_span(self_, b, 1, nranks_).peer >= 0;
    // the ipc transport's fused slab pulls (IpcTransport::fused_pulls): the aux stream forks first,
    // the halo stream's ready signal and first wait are one dispatch
    auto fused = [&](auto src) {
      const bool two = both;
      if (two) {
        HIPC(hipEventRecord(ev_fork_, hs));
        HIPC(hipStreamWaitEvent(aux_, ev_fork_, 0));
      }
      bool signalled = false;
      for (int side = 0; side < 2; ++side) {
        const HaloSpan h = halo_span(self_, b, side, nranks_);
        if (h.peer < 0) continue;
        hipStream_t ps = two && side == 1 ? aux_ : hs;
        if (ps == hs && !signalled) {
          hip_counter_signal_wait(ctr_ + kReady, ctr_ + kReady, ctr_ + kExpReady + side, timeout_s_, hs, 0, &words_);
          signalled = true;
        } else {
          hip_counter_wait(ctr_ + kReady, ctr_ + kExpReady + side, timeout_s_, ps, 0, &words_);
        }
        hip_face_copy(h.recv, h, src(side, h), h, ps, copy_);
      }
      if (!signalled) hip_counter_signal(ctr_ + kReady, hs);
      if (self_.ghost_event) {
        HIPC(hipEventRecord((hipEvent_t)self_.ghost_event, hs));
        HIPC(hipEventRecord((hipEvent_t)self_.ghost_event2, two ? aux_ : hs));
      }
      for (int side = 0; side < 2; ++side)
        if (halo_span(self_, b, side, nranks_).peer >= 0)
          hip_counter_signal(ctr_ + kPulled + side, two && side == 1 ? aux_ : hs);
      if (two) {
        HIPC(hipEventRecord(ev_join_, aux_));
        HIPC(hipStreamWaitEvent(hs, ev_join_, 0));
      }
    };
    if (direct_) {
      // the ipc direct sequence: ready, then per face wait + pull from the (own) field buffer +
      // pulled, then the wait that frees the faces the next boundary kernels overwrite. A pencil
      // pulls its y faces first and signals readyZ once they landed: its z faces carry those ghost rows
      if (!pencil_) {
        fused([&](int, const HaloSpan& h) { return (const void*)h.send; });
        for (int side = 0; side < 2; ++side) {
          if (halo_span(self_, b, side, nranks_).peer < 0) continue;
          hip_counter_wait(ctr_ + kPulled + side, ctr_ + kExpPulled + side, timeout_s_, hs, 0, &words_);
        }
        if (!capturing) last_b_ = b;
        return;
      }
      hip_counter_signal(ctr_ + kReady, hs);
      phase(2, kReady, false);
      hip_counter_signal(ctr_ + kReadyZ, hs);
      phase(0, kReadyZ, true);
      for (int side = 0; side < 4; ++side) {
        if (halo_span(self_, b, side, nranks_).peer < 0) continue;
        hip_counter_wait(ctr_ + kPulled + side, ctr_ + kExpPulled + side, timeout_s_, hs, 0, &words_);
      }
      if (!capturing) last_b_ = b;
      return;
    }
    // publish (the ipc sequence, with this slab as its own neighbour on both sides)
    for (int side = 0; side < 2; ++side) {
      const HaloSpan h = halo_span(self_, b, side, nranks_);
      if (h.peer < 0) continue;
      MDFX_CHECK(h.bytes == face_, "proxy: face geometry mismatch");
      hip_counter_wait(ctr_ + kPulled + side, ctr_ + kExpPulled + side, timeout_s_, hs, ahead, &words_);
      hip_face_copy(slot(b, side), h.send, face_, hs, copy_);
    }
    fused([&](int side, const HaloSpan&) { return (const void*)slot(b, side); });
    if (!capturing) last_b_ = b;
  }
  int last_parity() const override { return last_b_; }
  void set_last_parity(int b) override { last_b_ = b; }

  double allreduce_sum(double v) override { return v; }
  double allreduce_max(double v) override { return v; }
  void barrier() override {}
  void check() override {
    if (!words_.host) return;
    if (words_.wait_error()) MDFX_FAIL(format("proxy transport: a halo counter wait timed out after %.0f s", timeout_s_));
    if (words_.abort_raised()) MDFX_FAIL("proxy transport was aborted");
  }
  void abort() override {
    if (words_.host) words_.set_abort(1);
  }

 private:
  int copy_ = -1;  // face copy engine (hip_face_copy)
  hipStream_t aux_ = nullptr;
  hipEvent_t ev_fork_ = nullptr, ev_join_ = nullptr;
  LocalSlab self_;
  int nranks_ = 1;
  uint64_t* ctr_ = nullptr;
  HipWords words_;
  void* mbox_ = nullptr;
  size_t face_ = 0;
  bool ok_ = false;
  bool direct_ = false;
  bool pencil_ = false;  // (z, y) pencil: y faces first, then the z faces
  int last_b_ = -1;
  double timeout_s_ = 300.0;
};

}  // namespace

std::unique_ptr<Transport> make_proxy_transport(int copy_mode) {
  return std::unique_ptr<Transport>(new ProxyTransport(copy_mode));
}

}  // namespace mdfx
