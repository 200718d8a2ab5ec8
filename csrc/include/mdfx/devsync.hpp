// mdfx device-side synchronisation: stream-ordered counters for cross-process halo exchange, the
// process-wide abort word, and the device spin used by fault injection.
//
// Reference parity: the reference orders its halo exchange with blocking host MPI calls after a
// cudaDeviceSynchronize (MDF_kernel.cu:167-175,180-183) and hangs forever when a peer misbehaves
// (SURVEY D4). Here a process publishes "faces ready" / "faces pulled" as 64-bit counters in
// uncached device memory that its neighbours map through HIP IPC; waits are tiny kernels on the
// halo stream, so the host never blocks inside the step loop. Every device wait is bounded: it
// returns when the counter arrives, when the host raises the abort word (watchdog), or after its
// timeout, in which case it raises the host-visible error word that Transport::check() reports.
#pragma once

#include <cstdint>

namespace mdfx {

// Process-wide host-mapped words (allocated on first use; valid for the process lifetime).
void hip_set_abort(int v);          // non-zero: every spinning device wait returns at once
int hip_abort_raised();
int hip_wait_error();               // non-zero after a device wait timed out
void hip_clear_wait_error();

// Counters live in memory from hip_alloc_uncached (coherent across XCDs, processes and devices).
void* hip_alloc_uncached(size_t bytes);
void hip_free_uncached(void* p);

// Stream-ordered: *ctr += 1 (system-scope release: everything earlier on `stream` is visible to
// any agent that then observes the new value). Single writer per counter.
void hip_counter_signal(uint64_t* ctr, void* stream);
// An abort word ([0]) and a wait-error word ([16]) of one owner (a transport), host-mapped and
// coherent, so one engine's watchdog releases only its own device waits and reports only its own
// timeouts (the process-wide words above serve the fault-injection spin and owners without a pair).
struct HipWords {
  int* host = nullptr;
  int* dev = nullptr;
  void set_abort(int v) const { __atomic_store_n(&host[0], v, __ATOMIC_SEQ_CST); }
  int abort_raised() const { return __atomic_load_n(&host[0], __ATOMIC_SEQ_CST); }
  int wait_error() const { return __atomic_load_n(&host[16], __ATOMIC_SEQ_CST); }
};
HipWords hip_words_alloc();
void hip_words_free(HipWords& w);

// Stream-ordered: ++*expect (a private device counter), then wait until *remote >= *expect + ahead
// with a system-scope acquire. Bounded by timeout_s and the abort word (the owner's pair when
// `own` is given, else the process-wide one); a timeout raises the matching error word.
void hip_counter_wait(const uint64_t* remote, uint64_t* expect, double timeout_s, void* stream,
                      uint64_t ahead = 0, const HipWords* own = nullptr);
// hip_counter_signal(signal) and hip_counter_wait(remote, ...) in ONE dispatch: the signal first,
// then the wait (the exchange's ready signal fused with its first pull's wait).
void hip_counter_signal_wait(uint64_t* signal, const uint64_t* remote, uint64_t* expect, double timeout_s,
                             void* stream, uint64_t ahead = 0, const HipWords* own = nullptr);
// The wait's kernel (its first argument is `remote`): the engine finds its nodes in captured graphs.
const void* hip_counter_wait_kernel();

// Tests: leave a quiet-NaN pattern in every CU's LDS (synchronous, current device), so a kernel
// that reads LDS it never wrote produces NaN instead of silently using stale finite data.
void hip_poison_lds();

// Fault injection (MDFX_FAULT=spin@rank:step): a one-wave kernel that busy-waits on `stream` for
// `seconds` of device wall clock or until the abort word is raised.
void hip_spin(double seconds, void* stream);

}  // namespace mdfx
