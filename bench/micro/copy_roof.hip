// HBM copy-roof micro-benchmark: which load / store flavour reaches the measured 6.29 TB/s float4
// copy (MI355X_MICROARCH.md) on this box, and what the streaming kernels' own access path (LDS DMA
// in, non-temporal 16-B stores out) costs against it. Standalone: make micro; build/bin/copy_roof
//
//   v0 plain      global_load_dwordx4 -> global_store_dwordx4, grid-stride, 4 vectors per lane
//   v1 nt store   same, stores non-temporal (what the stencil kernels write with)
//   v2 nt both    non-temporal loads and stores
//   v3 lds dma    global_load_lds_dwordx4 into a per-wave LDS slot, ds_read_b128, nt store (the
//                 heat7_tbk / box27_tbk input path), one vector per lane per step
//   v4 lds dma4   four global_load_lds_dword (4 B per lane: the fp32 K = 5 / fp64 K = 5 heat7_wxk
//                 window path) per wave and step, ds_read_b128, nt 16-B store
//   v5 dma4 st8   the same with two nt 8-B stores per lane (each 512 contiguous bytes per wave: the
//                 narrow-row sweeps' output stores)
// Run under rocprofv3 --pmc with the L2's memory-side counters, v0 / v4 / v5 calibrate how many
// bytes a read / write request stands for on each path (the copy's bytes are known exactly).
//
// Every variant copies the same N floats (a multiple of the grid's stride, checked on the host)
// and the result is compared with the source on the host once.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      std::exit(1);                                                                      \
    }                                                                                    \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ in, f4* __restrict__ out, long n4) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += 4 * stride) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long j = i + k * stride;
      if (j < n4) v[k] = MODE == 2 ? __builtin_nontemporal_load(in + j) : in[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long j = i + k * stride;
      if (j < n4) {
        if (MODE == 0)
          out[j] = v[k];
        else
          __builtin_nontemporal_store(v[k], out + j);
      }
    }
  }
}

// one 16-B vector per lane per step through LDS DMA, as the streaming stencil kernels read planes
__global__ __launch_bounds__(256) void copy_lds(const f4* __restrict__ in, f4* __restrict__ out, long n4) {
  __shared__ f4 slot[4][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + w * 64; i0 < n4; i0 += stride) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(in + i0 + lane),
                                     (__attribute__((address_space(3))) void*)&slot[w][0], 16, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    const f4 v = slot[w][lane];
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): read before the next DMA overwrites
    __builtin_nontemporal_store(v, out + i0 + lane);
  }
}

// 4-byte LDS DMAs: dword d of the wave's 1 KiB chunk lands at LDS byte 4 d (d = 64 h + lane)
template <bool ST8>
__global__ __launch_bounds__(256) void copy_lds4(const f4* __restrict__ in, f4* __restrict__ out, long n4) {
  __shared__ f4 slot[4][64];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i0 = (long)blockIdx.x * blockDim.x + w * 64; i0 < n4; i0 += stride) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)((const float*)(in + i0) + h * 64 + lane),
                                       (__attribute__((address_space(3))) void*)((char*)&slot[w][0] + h * 256), 4, 0, 0);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    if constexpr (ST8) {
      typedef float f2 __attribute__((ext_vector_type(2)));
      const f2 a = ((const f2*)&slot[w][0])[lane], b = ((const f2*)&slot[w][0])[64 + lane];
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_nontemporal_store(a, (f2*)(out + i0) + lane);
      __builtin_nontemporal_store(b, (f2*)(out + i0) + 64 + lane);
    } else {
      const f4 v = slot[w][lane];
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): read before the next DMA overwrites
      __builtin_nontemporal_store(v, out + i0 + lane);
    }
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : (1L << 30);  // floats (4 GiB)
  const int blocks = argc > 2 ? std::atoi(argv[2]) : 256 * 16, threads = 256;
  const long n4 = n / 4, stride = (long)blocks * threads;
  if (n4 % stride != 0) {
    std::fprintf(stderr, "n/4 must be a multiple of %ld\n", stride);
    return 1;
  }
  f4 *in, *out;
  CK(hipMalloc(&in, n4 * sizeof(f4)));
  CK(hipMalloc(&out, n4 * sizeof(f4)));
  CK(hipMemset(in, 0x3f, n4 * sizeof(f4)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const char* names[] = {"plain", "nt store", "nt both", "lds dma", "lds dma4", "dma4 st8"};
  const int only = argc > 3 ? std::atoi(argv[3]) : -1;  // one mode (profiler passes), or all
  for (int mode = 0; mode < 6; ++mode) {
    if (only >= 0 && mode != only) continue;
    CK(hipMemset(out, 0, n4 * sizeof(f4)));
    float best = 1e30f;
    for (int rep = 0; rep < 8; ++rep) {
      CK(hipEventRecord(a));
      switch (mode) {
        case 0: hipLaunchKernelGGL(copy_k<0>, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
        case 1: hipLaunchKernelGGL(copy_k<1>, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
        case 2: hipLaunchKernelGGL(copy_k<2>, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
        case 3: hipLaunchKernelGGL(copy_lds, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
        case 4: hipLaunchKernelGGL(copy_lds4<false>, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
        default: hipLaunchKernelGGL(copy_lds4<true>, dim3(blocks), dim3(threads), 0, 0, in, out, n4); break;
      }
      CK(hipGetLastError());
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    std::vector<float> h(1 << 20), g(1 << 20);
    CK(hipMemcpy(h.data(), (float*)out + (n - (1 << 20)), (1 << 20) * sizeof(float), hipMemcpyDeviceToHost));
    CK(hipMemcpy(g.data(), (float*)in + (n - (1 << 20)), (1 << 20) * sizeof(float), hipMemcpyDeviceToHost));
    const bool ok = h == g;
    std::printf("%-10s %8.3f ms  %6.2f TB/s  %s\n", names[mode], best, 2.0 * n * 4 / (best * 1e-3) / 1e12,
                ok ? "ok" : "MISMATCH");
  }
  {  // the runtime's own device-to-device copy
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      CK(hipEventRecord(a));
      CK(hipMemcpyAsync(out, in, n4 * sizeof(f4), hipMemcpyDeviceToDevice, 0));
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;
    }
    std::printf("%-10s %8.3f ms  %6.2f TB/s  (blocks %d)\n", "hipMemcpy", best, 2.0 * n * 4 / (best * 1e-3) / 1e12, blocks);
  }
  CK(hipFree(in));
  CK(hipFree(out));
  return 0;
}
