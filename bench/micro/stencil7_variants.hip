// Standalone micro-benchmark: 3D 7-point Jacobi/heat update, fp32, single MI355X.
// Compares kernel structures (naive 1-cell-per-lane, z-marching register blocking
// with RY rows per lane, LDS variants) against a float4 copy kernel (the HBM roof).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 stencil7_variants.hip -o s7v
// Run:   ./s7v [n=1024] [iters=20]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIP_CHECK(x)                                                                 \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, \
              __LINE__, #x);                                                         \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

struct Geo {
  int nx, ny, nz;
  long long plane;  // nx*ny (pitch == nx here)
};

typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_nt(float* p, float4 o) {
  f4v v = {o.x, o.y, o.z, o.w};
  __builtin_nontemporal_store(v, (f4v*)p);
}
__device__ __forceinline__ float upd(float c, float s, float r) {
  return fmaf(r, fmaf(-6.f, c, s), c);
}

__device__ __forceinline__ unsigned xcd_remap(unsigned b, unsigned nwg) {
  const unsigned q = nwg / 8, r = nwg % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

__global__ void k_init(float* a, long long n, unsigned seed) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (long long)gridDim.x * blockDim.x) {
    unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull + seed;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
    a[i] = (float)((h >> 40) * (1.0 / 16777216.0));
  }
}

__global__ __launch_bounds__(256) void k_copy(const float4* __restrict__ a, float4* __restrict__ b,
                                              long long n4) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  long long st = (long long)gridDim.x * blockDim.x;
  for (; i < n4; i += st) b[i] = a[i];
}

// ---------------- naive: one float4 per lane, all neighbours from global/L1/L2 -------------
__global__ __launch_bounds__(256) void k_naive(const float* __restrict__ in, float* __restrict__ out,
                                               Geo g, float r) {
  const int x = (blockIdx.x * 64 + threadIdx.x) * 4;
  const int y = blockIdx.y * 4 + threadIdx.y;
  const int z = blockIdx.z;
  if (x >= g.nx || y >= g.ny) return;
  const long long idx = z * g.plane + (long long)y * g.nx + x;
  const float4 c = *(const float4*)(in + idx);
  float4 o = c;
  if (!(y == 0 || y == g.ny - 1 || z == 0 || z == g.nz - 1)) {
    const float l = x > 0 ? in[idx - 1] : 0.f;
    const float rr = x + 4 < g.nx ? in[idx + 4] : 0.f;
    const float4 ym = *(const float4*)(in + idx - g.nx);
    const float4 yp = *(const float4*)(in + idx + g.nx);
    const float4 zm = *(const float4*)(in + idx - g.plane);
    const float4 zp = *(const float4*)(in + idx + g.plane);
    o.x = upd(c.x, ((((l + c.y) + ym.x) + yp.x) + zm.x) + zp.x, r);
    o.y = upd(c.y, ((((c.x + c.z) + ym.y) + yp.y) + zm.y) + zp.y, r);
    o.z = upd(c.z, ((((c.y + c.w) + ym.z) + yp.z) + zm.z) + zp.z, r);
    o.w = upd(c.w, ((((c.z + rr) + ym.w) + yp.w) + zm.w) + zp.w, r);
    if (x == 0) o.x = c.x;
    if (x + 3 == g.nx - 1) o.w = c.w;
  }
  *(float4*)(out + idx) = o;
}

// ---------------- z-march: 4 waves stacked in y, RY rows per lane, ZC planes per block -------
template <int RY, bool NT>
__global__ __launch_bounds__(256) void k_zmarch(const float* __restrict__ in, float* __restrict__ out,
                                                Geo g, float r, int zc, int XT, int YT) {
  const unsigned nwg = gridDim.x;
  const unsigned t = xcd_remap(blockIdx.x, nwg);
  const int xt = t % XT;
  const int yt = (t / XT) % YT;
  const int zt = t / (XT * YT);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int x = xt * 256 + lane * 4;
  const int y0 = yt * (4 * RY) + w * RY;
  const int zs = zt * zc;
  const int ze = min(g.nz, zs + zc);
  if (y0 >= g.ny) return;  // wave-uniform
  const long long nx = g.nx, plane = g.plane;
  auto ld = [&](int z, int y) -> float4 {
    if (z < 0 || z >= g.nz || y < 0 || y >= g.ny) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *(const float4*)(in + z * plane + y * nx + x);
  };
  auto ldl = [&](int z, int y) -> float {
    if (lane != 0 || x == 0 || z < 0 || z >= g.nz || y >= g.ny) return 0.f;
    return in[z * plane + y * nx + x - 1];
  };
  auto ldr = [&](int z, int y) -> float {
    if (lane != 63 || x + 4 >= g.nx || z < 0 || z >= g.nz || y >= g.ny) return 0.f;
    return in[z * plane + y * nx + x + 4];
  };
  float4 P[RY], C[RY], N[RY];
  float EL[RY], ER[RY];
#pragma unroll
  for (int i = 0; i < RY; ++i) {
    P[i] = ld(zs - 1, y0 + i);
    C[i] = ld(zs, y0 + i);
    N[i] = ld(zs + 1, y0 + i);
    EL[i] = ldl(zs, y0 + i);
    ER[i] = ldr(zs, y0 + i);
  }
  float4 HL = ld(zs, y0 - 1), HH = ld(zs, y0 + RY);
  for (int z = zs; z < ze; ++z) {
    float4 NN[RY];
    float ELN[RY], ERN[RY];
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      NN[i] = ld(z + 2, y0 + i);
      ELN[i] = ldl(z + 1, y0 + i);
      ERN[i] = ldr(z + 1, y0 + i);
    }
    const float4 HLN = ld(z + 1, y0 - 1), HHN = ld(z + 1, y0 + RY);
    const bool zb = (z == 0 || z == g.nz - 1);
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      const int y = y0 + i;
      if (y >= g.ny) break;
      const float4 c = C[i];
      float4 o = c;
      float l = __shfl_up(c.w, 1);
      float rr = __shfl_down(c.x, 1);
      if (lane == 0) l = EL[i];
      if (lane == 63) rr = ER[i];
      if (!zb && y != 0 && y != g.ny - 1) {
        const float4 ym = i > 0 ? C[i - 1] : HL;
        const float4 yp = i < RY - 1 ? C[i + 1] : HH;
        const float4 zm = P[i], zp = N[i];
        o.x = upd(c.x, ((((l + c.y) + ym.x) + yp.x) + zm.x) + zp.x, r);
        o.y = upd(c.y, ((((c.x + c.z) + ym.y) + yp.y) + zm.y) + zp.y, r);
        o.z = upd(c.z, ((((c.y + c.w) + ym.z) + yp.z) + zm.z) + zp.z, r);
        o.w = upd(c.w, ((((c.z + rr) + ym.w) + yp.w) + zm.w) + zp.w, r);
        if (x == 0) o.x = c.x;
        if (x + 3 == g.nx - 1) o.w = c.w;
      }
      float4* dst = (float4*)(out + z * plane + (long long)y * nx + x);
      if (NT)
        st_nt((float*)dst, o);
      else
        *dst = o;
    }
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      P[i] = C[i];
      C[i] = N[i];
      N[i] = NN[i];
      EL[i] = ELN[i];
      ER[i] = ERN[i];
    }
    HL = HLN;
    HH = HHN;
  }
}

// ---------------- z-march with the block's planes exchanged through LDS ----------------------
// Block = 4 waves covering 1024 x-values (one wave per 256-wide segment) x RY rows; x-halo of a
// wave segment comes from the neighbouring wave through LDS instead of global edge loads; the
// y-halo rows are loaded from global (2 per RY rows).
template <int RY>
__global__ __launch_bounds__(256) void k_zmarch_wide(const float* __restrict__ in,
                                                     float* __restrict__ out, Geo g, float r,
                                                     int zc, int XT, int YT) {
  // XT counts 1024-wide tiles here.
  __shared__ float edge[2][4][RY][2];  // [buf][wave][row][left/right value]
  const unsigned nwg = gridDim.x;
  const unsigned t = xcd_remap(blockIdx.x, nwg);
  const int xt = t % XT;
  const int yt = (t / XT) % YT;
  const int zt = t / (XT * YT);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int x = xt * 1024 + w * 256 + lane * 4;
  const int y0 = yt * RY;
  const int zs = zt * zc;
  const int ze = min(g.nz, zs + zc);
  const long long nx = g.nx, plane = g.plane;
  const bool xin = x < g.nx;
  auto ld = [&](int z, int y) -> float4 {
    if (!xin || z < 0 || z >= g.nz || y < 0 || y >= g.ny) return make_float4(0.f, 0.f, 0.f, 0.f);
    return *(const float4*)(in + z * plane + y * nx + x);
  };
  float4 P[RY], C[RY], N[RY];
#pragma unroll
  for (int i = 0; i < RY; ++i) {
    P[i] = ld(zs - 1, y0 + i);
    C[i] = ld(zs, y0 + i);
    N[i] = ld(zs + 1, y0 + i);
  }
  float4 HL = ld(zs, y0 - 1), HH = ld(zs, y0 + RY);
  // block-edge x halo (only at 1024-tile boundaries), from global
  auto ldl = [&](int z, int y) -> float {
    if (w != 0 || lane != 0 || x == 0 || z < 0 || z >= g.nz || y >= g.ny) return 0.f;
    return in[z * plane + y * nx + x - 1];
  };
  auto ldr = [&](int z, int y) -> float {
    if (w != 3 || lane != 63 || x + 4 >= g.nx || z < 0 || z >= g.nz || y >= g.ny) return 0.f;
    return in[z * plane + y * nx + x + 4];
  };
  float EL[RY], ER[RY];
#pragma unroll
  for (int i = 0; i < RY; ++i) {
    EL[i] = ldl(zs, y0 + i);
    ER[i] = ldr(zs, y0 + i);
  }
  int buf = 0;
  for (int z = zs; z < ze; ++z) {
    float4 NN[RY];
    float ELN[RY], ERN[RY];
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      NN[i] = ld(z + 2, y0 + i);
      ELN[i] = ldl(z + 1, y0 + i);
      ERN[i] = ldr(z + 1, y0 + i);
    }
    const float4 HLN = ld(z + 1, y0 - 1), HHN = ld(z + 1, y0 + RY);
    // publish wave-edge values of plane z
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < RY; ++i) edge[buf][w][i][0] = C[i].x;
    }
    if (lane == 63) {
#pragma unroll
      for (int i = 0; i < RY; ++i) edge[buf][w][i][1] = C[i].w;
    }
    __syncthreads();
    const bool zb = (z == 0 || z == g.nz - 1);
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      const int y = y0 + i;
      if (y >= g.ny) break;
      const float4 c = C[i];
      float4 o = c;
      float l = __shfl_up(c.w, 1);
      float rr = __shfl_down(c.x, 1);
      if (lane == 0) l = w > 0 ? edge[buf][w - 1][i][1] : EL[i];
      if (lane == 63) rr = w < 3 ? edge[buf][w + 1][i][0] : ER[i];
      if (!zb && y != 0 && y != g.ny - 1) {
        const float4 ym = i > 0 ? C[i - 1] : HL;
        const float4 yp = i < RY - 1 ? C[i + 1] : HH;
        const float4 zm = P[i], zp = N[i];
        o.x = upd(c.x, ((((l + c.y) + ym.x) + yp.x) + zm.x) + zp.x, r);
        o.y = upd(c.y, ((((c.x + c.z) + ym.y) + yp.y) + zm.y) + zp.y, r);
        o.z = upd(c.z, ((((c.y + c.w) + ym.z) + yp.z) + zm.z) + zp.z, r);
        o.w = upd(c.w, ((((c.z + rr) + ym.w) + yp.w) + zm.w) + zp.w, r);
        if (x == 0) o.x = c.x;
        if (x + 3 == g.nx - 1) o.w = c.w;
      }
      if (xin) st_nt(out + z * plane + (long long)y * nx + x, o);
    }
    buf ^= 1;
#pragma unroll
    for (int i = 0; i < RY; ++i) {
      P[i] = C[i];
      C[i] = N[i];
      N[i] = NN[i];
      EL[i] = ELN[i];
      ER[i] = ERN[i];
    }
    HL = HLN;
    HH = HHN;
  }
}

// ------------------------------------------------------------------------------------------
struct Variant {
  const char* name;
  void (*launch)(const float*, float*, Geo, float, hipStream_t, int);
  int zc;
};

static void L_naive(const float* a, float* b, Geo g, float r, hipStream_t s, int) {
  dim3 blk(64, 4), grd((g.nx / 4 + 63) / 64, (g.ny + 3) / 4, g.nz);
  hipLaunchKernelGGL(k_naive, grd, blk, 0, s, a, b, g, r);
}
template <int RY, bool NT>
static void L_zm(const float* a, float* b, Geo g, float r, hipStream_t s, int zc) {
  int XT = g.nx / 256, YT = (g.ny + 4 * RY - 1) / (4 * RY), ZT = (g.nz + zc - 1) / zc;
  hipLaunchKernelGGL((k_zmarch<RY, NT>), dim3(XT * YT * ZT), dim3(256), 0, s, a, b, g, r, zc, XT, YT);
}
template <int RY>
static void L_zw(const float* a, float* b, Geo g, float r, hipStream_t s, int zc) {
  int XT = (g.nx + 1023) / 1024, YT = (g.ny + RY - 1) / RY, ZT = (g.nz + zc - 1) / zc;
  hipLaunchKernelGGL((k_zmarch_wide<RY>), dim3(XT * YT * ZT), dim3(256), 0, s, a, b, g, r, zc, XT,
                     YT);
}

int main(int argc, char** argv) {
  int n = argc > 1 ? atoi(argv[1]) : 1024;
  int iters = argc > 2 ? atoi(argv[2]) : 20;
  Geo g{n, n, n, (long long)n * n};
  const long long cells = (long long)n * n * n;
  const float r = 1.f / 6.f;
  float *A, *B, *R;
  HIP_CHECK(hipMalloc(&A, cells * 4 + 1024));
  HIP_CHECK(hipMalloc(&B, cells * 4 + 1024));
  HIP_CHECK(hipMalloc(&R, cells * 4 + 1024));
  hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, A, cells, 1234u);
  HIP_CHECK(hipDeviceSynchronize());
  hipStream_t s;
  HIP_CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));

  // copy roof
  {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      HIP_CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; ++i)
        hipLaunchKernelGGL(k_copy, dim3(256 * 8 * 4), dim3(256), 0, s, (const float4*)(i & 1 ? B : A),
                           (float4*)(i & 1 ? A : B), cells / 4);
      HIP_CHECK(hipEventRecord(e1, s));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms / iters);
    }
    printf("copy: %.3f ms  %.1f GB/s  (=> %.1f GCells/s at 8 B/cell)\n", best,
           cells * 8.0 / best / 1e6, cells / best / 1e6);
  }
  hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, A, cells, 1234u);
  L_naive(A, R, g, r, s, 0);
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<float> hr(cells), hb(cells);
  HIP_CHECK(hipMemcpy(hr.data(), R, cells * 4, hipMemcpyDeviceToHost));

  std::vector<Variant> vs = {
      {"naive", L_naive, 0},
      {"zm RY1 zc64", L_zm<1, true>, 64},
      {"zm RY2 zc64", L_zm<2, true>, 64},
      {"zm RY2 zc128", L_zm<2, true>, 128},
      {"zm RY2 zc64 plainst", L_zm<2, false>, 64},
      {"zm RY4 zc64", L_zm<4, true>, 64},
      {"zm RY4 zc128", L_zm<4, true>, 128},
      {"zm RY8 zc128", L_zm<8, true>, 128},
      {"zw RY1 zc64", L_zw<1>, 64},
      {"zw RY2 zc64", L_zw<2>, 64},
      {"zw RY4 zc64", L_zw<4>, 64},
      {"zw RY4 zc128", L_zw<4>, 128},
      {"zw RY8 zc128", L_zw<8>, 128},
  };
  // correctness
  for (auto& v : vs) {
    HIP_CHECK(hipMemset(B, 0, cells * 4));
    v.launch(A, B, g, r, s, v.zc);
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipMemcpy(hb.data(), B, cells * 4, hipMemcpyDeviceToHost));
    long long bad = 0, first = -1;
    for (long long i = 0; i < cells; ++i)
      if (memcmp(&hb[i], &hr[i], 4) != 0) {
        if (first < 0) first = i;
        ++bad;
      }
    printf("check %-22s mismatches=%lld first=%lld\n", v.name, bad, first);
  }
  // timing: interleaved rounds
  const int rounds = 3;
  std::vector<std::vector<float>> t(vs.size());
  for (int rd = 0; rd < rounds; ++rd)
    for (size_t k = 0; k < vs.size(); ++k) {
      auto& v = vs[k];
      v.launch(A, B, g, r, s, v.zc);
      HIP_CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; ++i) v.launch(i & 1 ? B : A, i & 1 ? A : B, g, r, s, v.zc);
      HIP_CHECK(hipEventRecord(e1, s));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      t[k].push_back(ms / iters);
    }
  for (size_t k = 0; k < vs.size(); ++k) {
    std::sort(t[k].begin(), t[k].end());
    float best = t[k][0], med = t[k][t[k].size() / 2];
    printf("%-22s best %.3f ms  med %.3f ms  %.1f GCells/s  (%.1f GB/s @8B)\n", vs[k].name, best,
           med, cells / best / 1e6, cells * 8.0 / best / 1e6);
  }
  return 0;
}
