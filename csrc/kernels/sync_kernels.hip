// Device-side synchronisation kernels (see mdfx/devsync.hpp): cross-process counters, the abort
// word and the fault-injection spin. Each kernel is one wave; only lane 0 touches memory, with
// vector (global) loads / stores and system-scope atomics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <string>

#include "mdfx/common.hpp"
#include "mdfx/devsync.hpp"

namespace mdfx {

#define HIPC(x)                                                                          \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) ::mdfx::throw_error(__FILE__, __LINE__, std::string("HIP: ") + #x + " -> " + hipGetErrorString(e_)); \
  } while (0)

namespace {

// [0] abort word, [16] wait-error word (separate 64-B lines); host-mapped, coherent.
int* g_words = nullptr;
std::once_flag g_words_once;

int* words() {
  std::call_once(g_words_once, [] {
    void* p = nullptr;
    HIPC(hipHostMalloc(&p, 4096, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::fill((int*)p, (int*)p + 1024, 0);
    g_words = (int*)p;
  });
  return g_words;
}

// device addresses of the words (coherent mapped host memory: the same on every device)
int* dev_words() {
  static int* d = [] {
    void* p = nullptr;
    HIPC(hipHostGetDevicePointer(&p, words(), 0));
    return (int*)p;
  }();
  return d;
}

uint64_t ticks_for(double seconds) {
  static int khz_cache[64] = {0};  // per device; queried once (this runs on every exchange)
  int dev = 0;
  HIPC(hipGetDevice(&dev));
  int khz = dev < 64 ? __atomic_load_n(&khz_cache[dev], __ATOMIC_RELAXED) : 0;
  if (khz == 0) {
    HIPC(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    if (khz <= 0) khz = 100000;  // gfx9 constant 100 MHz wall clock
    if (dev < 64) __atomic_store_n(&khz_cache[dev], khz, __ATOMIC_RELAXED);
  }
  const double t = std::max(0.0, seconds) * 1e3 * (double)khz;
  return t > 1.8e19 ? ~0ull : (uint64_t)t;
}

__global__ __launch_bounds__(64) void counter_signal_kernel(uint64_t* ctr) {
  if (threadIdx.x != 0) return;
  const uint64_t v = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(ctr, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Forward-progress assumption. This one-wave kernel spins on the halo stream until a producer (the
// interior sweep's folded-boundary signal, or a neighbour's ready / pulled counter) advances. The
// producer runs on ANOTHER hardware queue, so nothing orders the two: the wait relies on the
// hardware scheduler keeping the producing queue mapped and dispatching its blocks while this wave
// spins. With one engine process per GPU (two queues of ours plus the runtime's) that holds. With
// several processes oversubscribing one GPU's hardware queues it did not: round 4 session T, 8
// processes, one sweep stopped at 177 of 235 tile arrivals while high-priority waits spun
// (profiles/r04_session_t/). Hence normal stream priority everywhere, the ipc transport's refusal of
// shared GPUs without share_gpu (ipc_shared_gpu_problem), captured graphs never containing a folded
// wait (Solver::step), and the wall-clock bound below: a wait that cannot complete turns into an
// error word the host watchdog reports, never into a hang.
// Visibility guarantee relied on by the folded boundary: when this kernel, waiting for a fold
// counter, completes, its dispatch packet's system-scope release is carried out by the runtime as
// a writeback of every XCD's L2 (the whole cache), so the face tiles the still-running sweep stored
// earlier (s_waitcnt vmcnt(0) before its arrival counted) are in memory before the exchange's
// copies, dispatched after this kernel on the same stream, read them - blit kernels on other XCDs,
// SDMA engines or a peer GPU over xGMI. An HSA release only promises the kernel's own writes; the
// whole-L2 writeback is the implementation's behaviour, checked on one GPU with blit and SDMA
// readers (tests/test_gpu_ipc.py::test_ipc_fp32_fused_k5_folded). MDFX_FOLD_RELEASE=1 makes every
// signalling block write its own XCD's L2 back first instead (wxk_fold_signal; 1.7-2.8 % slower).
// `signal` (optional): bumped first, as counter_signal_kernel does, so one dispatch both publishes
// this process's counter and waits for the neighbour's (the exchange's "ready" signal and its first
// pull's wait: one kernel launch fewer ahead of the pull, hip_counter_signal_wait). The kernel
// boundary before it has already made the stream's earlier work visible.
__global__ __launch_bounds__(64) void counter_wait_kernel(const uint64_t* remote, uint64_t* expect, uint64_t ahead,
                                                          uint64_t ticks, const int* abort_w, int* err_w,
                                                          uint64_t* signal) {
  if (threadIdx.x != 0) return;
  if (signal) {
    const uint64_t v = __hip_atomic_load(signal, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(signal, v + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const uint64_t next = __hip_atomic_load(expect, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __hip_atomic_store(expect, next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t want = next + ahead;
  // once one wait has timed out the exchange is broken: later waits return at once, so the queued
  // steps drain in microseconds and the host reports the error (Transport::check)
  if (__hip_atomic_load(err_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const uint64_t t0 = (uint64_t)wall_clock64();
  for (;;) {
    if (__hip_atomic_load(remote, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) >= want) return;
    if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
    if ((uint64_t)wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ __launch_bounds__(64) void spin_kernel(uint64_t ticks, const int* abort_w) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = (uint64_t)wall_clock64();
  while ((uint64_t)wall_clock64() - t0 < ticks &&
         __hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0)
    __builtin_amdgcn_s_sleep(64);
}

// Fills its 40 KiB of LDS with a quiet-NaN pattern: four resident blocks cover a CU's 160 KiB,
// so kernels that run next find NaN wherever they read LDS they did not write (tests).
__global__ __launch_bounds__(256) void lds_poison_kernel() {
  __shared__ uint32_t buf[10240];
  for (int i = threadIdx.x; i < 10240; i += 256) buf[i] = 0x7fc00001u;
  __syncthreads();
}

void check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) MDFX_FAIL(std::string(what) + " launch failed: " + hipGetErrorString(e));
}

}  // namespace

void hip_set_abort(int v) { __atomic_store_n(&words()[0], v, __ATOMIC_SEQ_CST); }
int hip_abort_raised() { return __atomic_load_n(&words()[0], __ATOMIC_SEQ_CST); }
int hip_wait_error() { return __atomic_load_n(&words()[16], __ATOMIC_SEQ_CST); }
void hip_clear_wait_error() { __atomic_store_n(&words()[16], 0, __ATOMIC_SEQ_CST); }

void* hip_alloc_uncached(size_t bytes) {
  void* p = nullptr;
  HIPC(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached));
  HIPC(hipMemset(p, 0, bytes));
  HIPC(hipDeviceSynchronize());
  return p;
}

void hip_free_uncached(void* p) {
  if (p) (void)hipFree(p);
}

void hip_counter_signal(uint64_t* ctr, void* stream) {
  hipLaunchKernelGGL(counter_signal_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ctr);
  check_launch("counter_signal");
}

const void* hip_counter_wait_kernel() { return (const void*)&counter_wait_kernel; }

void hip_counter_wait(const uint64_t* remote, uint64_t* expect, double timeout_s, void* stream, uint64_t ahead,
                      const HipWords* own) {
  int* w = own ? own->dev : dev_words();
  hipLaunchKernelGGL(counter_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, remote, expect, ahead,
                     ticks_for(timeout_s), (const int*)w, w + 16, (uint64_t*)nullptr);
  check_launch("counter_wait");
}

void hip_counter_signal_wait(uint64_t* signal, const uint64_t* remote, uint64_t* expect, double timeout_s,
                             void* stream, uint64_t ahead, const HipWords* own) {
  int* w = own ? own->dev : dev_words();
  hipLaunchKernelGGL(counter_wait_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, remote, expect, ahead,
                     ticks_for(timeout_s), (const int*)w, w + 16, signal);
  check_launch("counter_signal_wait");
}

HipWords hip_words_alloc() {
  HipWords h;
  void* p = nullptr;
  HIPC(hipHostMalloc(&p, 4096, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
  std::fill((int*)p, (int*)p + 1024, 0);
  h.host = (int*)p;
  void* d = nullptr;
  HIPC(hipHostGetDevicePointer(&d, p, 0));
  h.dev = (int*)d;
  return h;
}

void hip_words_free(HipWords& h) {
  if (h.host) (void)hipHostFree(h.host);
  h.host = h.dev = nullptr;
}

void hip_poison_lds() {
  int dev = 0, cus = 0;
  HIPC(hipGetDevice(&dev));
  HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipLaunchKernelGGL(lds_poison_kernel, dim3(8 * std::max(cus, 1)), dim3(256), 0, nullptr);
  check_launch("lds_poison");
  HIPC(hipDeviceSynchronize());
}

void hip_spin(double seconds, void* stream) {
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks_for(seconds),
                     (const int*)dev_words());
  check_launch("spin");
}

}  // namespace mdfx
