// RCCL halo transport: whole-face ncclSend/ncclRecv between slab neighbours over xGMI.
//
// One process per GPU (torchrun / mpirun; the 128-byte ncclUniqueId is distributed by the
// caller: torch.distributed in Python, a TCP rendezvous in the C++ CLI), or one process driving
// several GPUs (every local rank's comm initialised inside one ncclGroup). Each step the sends
// and receives of all local slabs go into ONE ncclGroupStart/End on each slab's
// halo stream, so the exchange is ordered after the boundary kernel and before the next step's
// boundary kernel by stream order alone, while the interior sweep runs on the compute stream.
// Slab neighbours are single peers: each face rides one xGMI link (≈153 GB/s); a 1024^2 fp32 face
// is 4 MiB ≈ 27 µs.
//
// Reference parity: replaces the per-element blocking MPI_Send/MPI_Recv loops of
// MDF_kernel.cu:167-169,180-183 (D5) and their self-addressed rank-1 branch (D3, D4).
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "mdfx/runtime.hpp"

namespace mdfx {

#define NCCLC(x)                                                                              \
  do {                                                                                        \
    ncclResult_t r_ = (x);                                                                    \
    if (r_ != ncclSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("RCCL: ") + #x + " -> " + ncclGetErrorString(r_)); \
  } while (0)
#define HIPC(x)                                                                          \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("HIP: ") + #x + " -> " + hipGetErrorString(e_)); \
  } while (0)

std::string rccl_unique_id() {
  ncclUniqueId id;
  NCCLC(ncclGetUniqueId(&id));
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

// The grouped send / recv is pure stream work on the halo stream under every runtime
bool rccl_stream_ordered() { return true; }
// ... but the folded boundary is not the default with RCCL: no run has yet shown RCCL's p2p kernels
// reading a face published by a mid-sweep device counter (Transport::fold_by_default); the bench
// gates and verifies the folded schedule as its own candidate (`rccl_fold`) instead
bool rccl_fold_by_default() { return false; }
// ... but RCCL's group joins its own internal streams to the caller's with events, and the HIP 7.0
// runtime PyTorch bundles segfaults in hipStreamEndCapture on such multi-stream captures
// (profiles/archive/r02_graph_runtime.txt): RCCL steps are captured only under HIP >= 7.2
bool rccl_graph_capturable() {
  static const bool ok = [] {
    int v = 0;
    return hipRuntimeGetVersion(&v) == hipSuccess && v >= 70200000;
  }();
  return ok;
}

namespace {

class RcclTransport final : public Transport {
 public:
  explicit RcclTransport(const std::string& uid) {
    MDFX_CHECK(uid.size() == NCCL_UNIQUE_ID_BYTES, "ncclUniqueId must be 128 bytes");
    std::memcpy(id_.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
  }
  ~RcclTransport() override {
    if (aborted_) return;  // streams may hold RCCL work that never ran: leak rather than block
    for (size_t i = 0; i < comms_.size(); ++i) {
      if (scratch_[i]) {
        (void)hipSetDevice(locals_[i].be->device());
        (void)hipFree(scratch_[i]);
      }
      if (i < ystage_.size() && ystage_[i]) {
        (void)hipSetDevice(locals_[i].be->device());
        (void)hipFree(ystage_[i]);
      }
      if (aux_[i]) (void)hipStreamDestroy(aux_[i]);
      if (comms_[i]) (void)ncclCommDestroy(comms_[i]);
    }
  }
  const char* name() const override { return "rccl"; }
  bool in_process_only() const override { return false; }
  // RCCL gets the engine's single-stream boundary schedule under every runtime (stream_ordered),
  // folded only on request (fold_by_default), and graph capture only where the runtime supports it
  bool stream_ordered() const override { return rccl_stream_ordered(); }
  bool fold_by_default() const override { return rccl_fold_by_default(); }
  bool graph_capturable() const override { return rccl_graph_capturable(); }
  void set_timeout(double s) override { timeout_s_ = s; }
  void abort() override {
    if (aborted_) return;
    aborted_ = true;
    for (auto c : comms_)
      if (c) (void)ncclCommAbort(c);
  }

  // Bounded bootstrap: the communicators are created non-blocking and polled under the watchdog
  // bound (timeout_s, or 600 s when the watchdog is off), so a rank that never joins makes every
  // other rank abort its half-built communicator and fail with a message instead of blocking in
  // ncclCommInitRank forever (the reference's D4 hang class starts at its MPI_Init / first send).
  void setup(const std::vector<LocalSlab>& locals, int nranks) override {
    locals_ = locals;
    nranks_ = nranks;
    comms_.assign(locals_.size(), nullptr);
    scratch_.assign(locals_.size(), nullptr);
    aux_.assign(locals_.size(), nullptr);
    for (auto& s : locals_) MDFX_CHECK(s.be->kind() == DeviceKind::HIP, "rccl transport needs HIP backends");
    maybe_hang_before_init();
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    if (locals_.size() == 1) {
      locals_[0].be->activate();
      accept(ncclCommInitRankConfig(&comms_[0], nranks_, id_, locals_[0].rank, &cfg), "ncclCommInitRankConfig");
    } else {
      NCCLC(ncclGroupStart());
      for (size_t i = 0; i < locals_.size(); ++i) {
        locals_[i].be->activate();
        accept(ncclCommInitRankConfig(&comms_[i], nranks_, id_, locals_[i].rank, &cfg), "ncclCommInitRankConfig");
      }
      accept(ncclGroupEnd(), "ncclGroupEnd (init)");
    }
    wait_ready("bootstrap (ncclCommInitRankConfig)", 1000);
    for (size_t i = 0; i < locals_.size(); ++i) {
      locals_[i].be->activate();
      HIPC(hipMalloc(&scratch_[i], 2 * sizeof(double)));
      HIPC(hipStreamCreateWithFlags(&aux_[i], hipStreamNonBlocking));
    }
    // (z, y) pencils: a y face is `nzl` pieces of `hy` rows, one per plane; RCCL moves contiguous
    // bytes, so each y face travels through a staging buffer (2-D copies on the halo stream around
    // a first send / recv group; the z faces, which carry the fresh y ghost rows, follow in a second)
    ystage_.assign(locals_.size(), nullptr);
    for (size_t i = 0; i < locals_.size(); ++i) {
      const LocalSlab& ls = locals_[i];
      if (ls.py <= 1 || ls.lay.hy == 0) continue;
      const size_t yb = halo_span(ls, 0, 2, nranks_).bytes ? halo_span(ls, 0, 2, nranks_).bytes
                                                            : halo_span(ls, 0, 3, nranks_).bytes;
      if (!yb) continue;
      ls.be->activate();
      HIPC(hipMalloc(&ystage_[i], 4 * yb));  // send / recv for each of the two y sides
      ystage_bytes_ = yb;
      pencil_ = true;
    }
  }

  void exchange(int b) override {
    if (pencil_) {
      // phase 1: the y faces through the staging buffers
      for (size_t i = 0; i < locals_.size(); ++i) {
        const LocalSlab& s = locals_[i];
        if (!ystage_[i]) continue;
        s.be->activate();
        for (int side = 2; side < 4; ++side) {
          const HaloSpan h = halo_span(s, b, side, nranks_);
          if (h.peer < 0) continue;
          MDFX_CHECK(h.bytes == ystage_bytes_, "rccl: y face sizes differ between pencils");
          char* snd = (char*)ystage_[i] + (size_t)(2 * (side - 2)) * ystage_bytes_;
          HIPC(hipMemcpy2DAsync(snd, h.width, h.send, h.stride, h.width, h.height, hipMemcpyDeviceToDevice,
                                (hipStream_t)s.halo_stream));
        }
      }
      NCCLC(ncclGroupStart());
      for (size_t i = 0; i < locals_.size(); ++i) {
        const LocalSlab& s = locals_[i];
        if (!ystage_[i]) continue;
        for (int side = 2; side < 4; ++side) {
          const HaloSpan h = halo_span(s, b, side, nranks_);
          if (h.peer < 0) continue;
          char* snd = (char*)ystage_[i] + (size_t)(2 * (side - 2)) * ystage_bytes_;
          char* rcv = snd + ystage_bytes_;
          accept(ncclRecv(rcv, h.bytes, ncclUint8, h.peer, comms_[i], (hipStream_t)s.halo_stream), "ncclRecv");
          accept(ncclSend(snd, h.bytes, ncclUint8, h.peer, comms_[i], (hipStream_t)s.halo_stream), "ncclSend");
        }
      }
      if (accept(ncclGroupEnd(), "ncclGroupEnd (y faces)") == ncclInProgress) wait_ready("halo exchange launch", 50);
      for (size_t i = 0; i < locals_.size(); ++i) {
        const LocalSlab& s = locals_[i];
        if (!ystage_[i]) continue;
        s.be->activate();
        for (int side = 2; side < 4; ++side) {
          const HaloSpan h = halo_span(s, b, side, nranks_);
          if (h.peer < 0) continue;
          const char* rcv = (char*)ystage_[i] + (size_t)(2 * (side - 2) + 1) * ystage_bytes_;
          HIPC(hipMemcpy2DAsync(h.recv, h.stride, rcv, h.width, h.width, h.height, hipMemcpyDeviceToDevice,
                                (hipStream_t)s.halo_stream));
        }
      }
    }
    NCCLC(ncclGroupStart());
    for (size_t i = 0; i < locals_.size(); ++i) {
      const LocalSlab& s = locals_[i];
      for (int side = 0; side < 2; ++side) {
        const HaloSpan h = halo_span(s, b, side, nranks_);
        if (h.peer < 0) continue;
        accept(ncclRecv(h.recv, h.bytes, ncclUint8, h.peer, comms_[i], (hipStream_t)s.halo_stream), "ncclRecv");
        accept(ncclSend(h.send, h.bytes, ncclUint8, h.peer, comms_[i], (hipStream_t)s.halo_stream), "ncclSend");
      }
    }
    // non-blocking communicators: a group whose p2p connections are still being set up (the first
    // exchange with a peer) returns ncclInProgress; wait for the launch before anything else
    if (accept(ncclGroupEnd(), "ncclGroupEnd (exchange)") == ncclInProgress) wait_ready("halo exchange launch", 50);
  }

  double allreduce(double v, ncclRedOp_t op) {
    // the engine already combined its local slabs: slab 0 contributes v, the others the identity
    std::vector<double> in(locals_.size()), out(locals_.size());
    for (size_t i = 0; i < locals_.size(); ++i) {
      in[i] = (i == 0) ? v : (op == ncclSum ? 0.0 : -1e308);
      locals_[i].be->activate();
      HIPC(hipMemcpyAsync(scratch_[i], &in[i], sizeof(double), hipMemcpyHostToDevice, aux_[i]));
    }
    NCCLC(ncclGroupStart());
    for (size_t i = 0; i < locals_.size(); ++i)
      accept(ncclAllReduce(scratch_[i], (char*)scratch_[i] + sizeof(double), 1, ncclFloat64, op, comms_[i], aux_[i]),
             "ncclAllReduce");
    if (accept(ncclGroupEnd(), "ncclGroupEnd (all-reduce)") == ncclInProgress) wait_ready("all-reduce launch", 50);
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < locals_.size(); ++i) {
      locals_[i].be->activate();
      HIPC(hipMemcpyAsync(&out[i], (char*)scratch_[i] + sizeof(double), sizeof(double),
                          hipMemcpyDeviceToHost, aux_[i]));
      // poll instead of blocking: a dead peer surfaces as an RCCL async error or the watchdog
      for (;;) {
        const hipError_t q = hipStreamQuery(aux_[i]);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) HIPC(q);
        check();
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s_ > 0 && el > timeout_s_) {
          abort();
          MDFX_FAIL(format("watchdog: RCCL all-reduce not done after %.1f s (peer dead or hung)", el));
        }
        std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    return out[0];
  }
  double allreduce_sum(double v) override { return allreduce(v, ncclSum); }
  double allreduce_max(double v) override { return allreduce(v, ncclMax); }
  void barrier() override { (void)allreduce(0.0, ncclSum); }

  void check() override {
    if (aborted_) MDFX_FAIL("RCCL communicator was aborted");
    for (auto c : comms_) {
      ncclResult_t ae = ncclSuccess;
      NCCLC(ncclCommGetAsyncError(c, &ae));
      if (ae != ncclSuccess && ae != ncclInProgress) {
        abort();
        MDFX_FAIL(std::string("RCCL async error: ") + ncclGetErrorString(ae));
      }
    }
  }

 private:
  // ncclSuccess or (non-blocking communicator) ncclInProgress; anything else throws
  static ncclResult_t accept(ncclResult_t r, const char* what) {
    if (r != ncclSuccess && r != ncclInProgress)
      ::mdfx::throw_error(__FILE__, __LINE__, std::string("RCCL: ") + what + " -> " + ncclGetErrorString(r));
    return r;
  }
  // Poll every communicator until no operation is in progress, bounded by the watchdog (600 s when
  // it is off); on expiry or error abort the communicators and throw.
  void wait_ready(const char* what, int poll_us) {
    const double limit = timeout_s_ > 0 ? timeout_s_ : 600.0;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      bool busy = false;
      for (auto c : comms_) {
        if (!c) continue;
        ncclResult_t st = ncclSuccess;
        const ncclResult_t q = ncclCommGetAsyncError(c, &st);
        if (q != ncclSuccess && q != ncclInProgress) {
          abort();
          MDFX_FAIL(std::string("RCCL ") + what + ": ncclCommGetAsyncError -> " + ncclGetErrorString(q));
        }
        if (st == ncclInProgress) busy = true;
        else if (st != ncclSuccess) {
          abort();
          MDFX_FAIL(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(st));
        }
      }
      if (!busy) return;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > limit) {
        abort();
        MDFX_FAIL(format("RCCL %s not complete after %.1f s on rank %d of %d: a peer rank never joined or hung "
                         "(communicators aborted)", what, el, locals_.empty() ? -1 : locals_[0].rank, nranks_));
      }
      std::this_thread::sleep_for(std::chrono::microseconds(poll_us));
    }
  }
  // Fault injection for the bootstrap tests: MDFX_FAULT=inithang@<rank> makes that rank stop
  // before it joins the communicator (it sleeps until killed, at most an hour).
  void maybe_hang_before_init() const {
    const char* v = std::getenv("MDFX_FAULT");
    int rk = -1;
    if (!v || std::sscanf(v, "inithang@%d", &rk) != 1) return;
    for (auto& s : locals_)
      if (s.rank == rk) {
        std::fprintf(stderr, "[mdfx] injecting fault 'inithang' on rank %d before ncclCommInitRankConfig\n", rk);
        std::fflush(stderr);
        for (int i = 0; i < 3600; ++i) std::this_thread::sleep_for(std::chrono::seconds(1));
      }
  }

  ncclUniqueId id_;
  std::vector<LocalSlab> locals_;
  int nranks_ = 1;
  std::vector<ncclComm_t> comms_;
  std::vector<void*> ystage_;  // pencils: per slab 4 y-face staging buffers (send / recv x 2 sides)
  size_t ystage_bytes_ = 0;
  bool pencil_ = false;
  std::vector<void*> scratch_;
  std::vector<hipStream_t> aux_;
  double timeout_s_ = 0.0;
  bool aborted_ = false;
};

}  // namespace

std::unique_ptr<Transport> make_rccl_transport(const std::string& unique_id) {
  return std::unique_ptr<Transport>(new RcclTransport(unique_id));
}

}  // namespace mdfx
