// mdfx — MI355X-native multi-GPU finite-difference stencil engine.
// Common types, enums and error handling shared by every layer.
//
// Reference parity: the reference (Rodrigovicente/MPI-CUDA-Process) checks no return codes at all
// (SURVEY.md §0.3 D18); every HIP / RCCL / system call here goes through MDFX_* checks that throw
// mdfx::Error carrying file:line, so a failing rank fails loudly instead of hanging (D4).
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <cmath>
#include <string>

namespace mdfx {

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

[[noreturn]] void throw_error(const char* file, int line, const std::string& msg);

#define MDFX_CHECK(cond, msg)                                                      \
  do {                                                                             \
    if (!(cond)) ::mdfx::throw_error(__FILE__, __LINE__, std::string("check failed: ") + #cond + " — " + (msg)); \
  } while (0)

#define MDFX_FAIL(msg) ::mdfx::throw_error(__FILE__, __LINE__, (msg))

// Element types of a field. U8 is the Game-of-Life cell type (the reference used int, 4x the
// bytes for a 1-bit state: kernel.cu:10).
enum class DType : int { F32 = 0, F64 = 1, U8 = 2 };

inline size_t dtype_size(DType t) {
  switch (t) {
    case DType::F32: return 4;
    case DType::F64: return 8;
    case DType::U8: return 1;
  }
  return 0;
}
const char* dtype_name(DType t);
DType dtype_from_name(const std::string& s);

// Stencil families. 2D kinds store an h x w grid as (nx = w, ny = 1, nz = h): rows are the
// split ("plane") axis, exactly like the reference's row-slab split (MDF_kernel.cu:30,54).
enum class StencilKind : int {
  Jacobi5 = 0,  // 2D 5-point heat / Jacobi (reference MDF update, MDF_kernel.cu:20)
  Life = 1,     // 2D Moore-8 B3/S23 Game of Life (reference kernel.cu:66)
  Heat7 = 2,    // 3D 7-point heat / Jacobi (BASELINE.json configs 2, 3, 5)
  Box27 = 3,    // 3D 27-point weighted stencil (BASELINE.json config 4)
};
const char* stencil_name(StencilKind k);
StencilKind stencil_from_name(const std::string& s);
inline bool stencil_is_2d(StencilKind k) { return k == StencilKind::Jacobi5 || k == StencilKind::Life; }

// Coefficients. Jacobi5/Heat7: u' = u + r * (sum_neighbours - 2d * u). Box27:
// u' = c0*u + c1*sum(6 faces) + c2*sum(12 edges) + c3*sum(8 corners).
struct StencilCoef {
  double r = -1.0;  // < 0 -> default 1/(2d) (Jacobi)
  double c0 = 0.25, c1 = 1.0 / 20.0, c2 = 1.0 / 40.0, c3 = 3.0 / 160.0;
  // 2D MDF only: evaluate the update exactly as the reference does (sm::jacobi5_ref: fp32 sum and
  // -4u, fp64 scale and add, one more rounding at the store) instead of wholly in the field type.
  // See StencilSpec::mixed_update() for when the two can differ at all.
  bool ref_precision = false;
};

struct StencilSpec {
  StencilKind kind = StencilKind::Heat7;
  DType dtype = DType::F32;
  StencilCoef coef;
  double rate() const {  // effective r for 5/7-pt
    if (coef.r >= 0) return coef.r;
    return kind == StencilKind::Jacobi5 ? 0.25 : 1.0 / 6.0;
  }
  // Whether ref_precision can change a single bit of the result. The reference evaluates
  // round_f32(round_f64(r*t + u)) with t = fma_f32(-4, u, s); the field-type update is fma_f32(r, t, u)
  // = round_f32(r*t + u), one rounding of the exact value. When r is a power of two, r*t is exact
  // with 24 significant bits, so r*t + u is exact in fp64 unless the two exponents are more than 28
  // apart; then the smaller term is under 2^-28 of the larger, both the exact and the fp64-rounded
  // sum lie strictly inside the larger term's half-ulp interval, and both round to it. So with a
  // power-of-two r (the reference's 0.25) the two evaluations are bitwise identical for every input
  // (subnormals included: fp64 holds every fp32 subnormal product exactly), and the fused field-type
  // kernels serve ref_precision. An fp64 field evaluates the reference's update in one fp64 fma
  // either way. Only fp32 with another r needs the mixed kernels (tests/test_cpu_engine.py).
  bool mixed_update() const {
    if (!coef.ref_precision || kind != StencilKind::Jacobi5 || dtype != DType::F32) return false;
    int e = 0;
    const float r = (float)rate();
    return !(r > 0.0f && std::frexp(r, &e) == 0.5f);
  }
};

struct Extent3 {
  int64_t nx = 1, ny = 1, nz = 1;
  int64_t cells() const { return nx * ny * nz; }
};

// Where a field lives. CPU is the reference/oracle backend; HIP is the gfx950 device path.
enum class DeviceKind : int { CPU = 0, HIP = 1 };

std::string format(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

}  // namespace mdfx
