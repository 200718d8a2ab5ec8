// mdfx core: error helpers, enum names, layout and slab decomposition math.
#include <csignal>
#include <cstdarg>
#include <cstdlib>
#include <execinfo.h>
#include <unistd.h>
#include <cstdio>
#include <string>

#include "mdfx/common.hpp"
#include "mdfx/grid.hpp"

namespace mdfx {

namespace {
// MDFX_SEGV_BACKTRACE=1: print the native stack on a crash (host-side debugging on the GPU box,
// where debuggers are not available).
void segv_handler(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "\n[mdfx] fatal signal, native backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
struct SegvInstaller {
  SegvInstaller() {
    const char* v = std::getenv("MDFX_SEGV_BACKTRACE");
    if (v && *v == '1') {
      void* warm[4];
      (void)backtrace(warm, 4);  // load the unwinder now, not inside the handler
      struct sigaction sa {};
      sa.sa_handler = segv_handler;
      sa.sa_flags = SA_RESETHAND | SA_NODEFER;
      sigaction(SIGSEGV, &sa, nullptr);
      sigaction(SIGABRT, &sa, nullptr);
    }
  }
} g_segv_installer;
}  // namespace

void throw_error(const char* file, int line, const std::string& msg) {
  const char* base = file;
  for (const char* p = file; *p; ++p)
    if (*p == '/') base = p + 1;
  throw Error(std::string("[mdfx ") + base + ":" + std::to_string(line) + "] " + msg);
}

std::string format(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return std::string(buf);
}

const char* dtype_name(DType t) {
  switch (t) {
    case DType::F32: return "f32";
    case DType::F64: return "f64";
    case DType::U8: return "u8";
  }
  return "?";
}

DType dtype_from_name(const std::string& s) {
  if (s == "f32" || s == "float32" || s == "float") return DType::F32;
  if (s == "f64" || s == "float64" || s == "double") return DType::F64;
  if (s == "u8" || s == "uint8") return DType::U8;
  MDFX_FAIL("unknown dtype '" + s + "' (f32|f64|u8)");
}

const char* stencil_name(StencilKind k) {
  switch (k) {
    case StencilKind::Jacobi5: return "jacobi5";
    case StencilKind::Life: return "life";
    case StencilKind::Heat7: return "heat7";
    case StencilKind::Box27: return "box27";
  }
  return "?";
}

StencilKind stencil_from_name(const std::string& s) {
  if (s == "jacobi5" || s == "5" || s == "mdf" || s == "5pt") return StencilKind::Jacobi5;
  if (s == "life" || s == "gol") return StencilKind::Life;
  if (s == "heat7" || s == "7" || s == "jacobi7" || s == "7pt") return StencilKind::Heat7;
  if (s == "box27" || s == "27" || s == "27pt") return StencilKind::Box27;
  MDFX_FAIL("unknown stencil '" + s + "' (5|7|27|life)");
}

FieldLayout FieldLayout::make(Extent3 g, int64_t z0, int64_t z1, int halo, DType dt, int64_t y0, int64_t y1, int hy) {
  MDFX_CHECK(g.nx >= 1 && g.ny >= 1 && g.nz >= 1, "grid extents must be positive");
  MDFX_CHECK(0 <= z0 && z0 <= z1 && z1 <= g.nz, "owned plane range out of the grid");
  MDFX_CHECK(halo >= 1, "halo must be >= 1");
  if (y1 < 0) y1 = g.ny;
  MDFX_CHECK(0 <= y0 && y0 < y1 && y1 <= g.ny, "owned row range out of the grid");
  MDFX_CHECK(hy >= 0 && (hy == 0 || g.ny > 1), "ghost rows need a 3D grid");
  FieldLayout l;
  l.global = g;
  l.z0 = z0;
  l.z1 = z1;
  l.halo = halo;
  l.y0 = y0;
  l.y1 = y1;
  l.hy = hy;
  l.dtype = dt;
  const int64_t align = kRowAlignBytes / (int64_t)dtype_size(dt);
  l.pitch = (g.nx + align - 1) / align * align;
  l.plane = l.pitch * l.rows();
  return l;
}

SlabDecomposition::SlabDecomposition(int64_t nz_, int parts_) : nz(nz_), parts(parts_) {
  MDFX_CHECK(parts >= 1, "need at least one part");
  MDFX_CHECK(nz >= parts, format("cannot split %lld planes over %d ranks", (long long)nz, parts));
}

int64_t SlabDecomposition::z0(int p) const {
  // first (nz % parts) parts get one extra plane
  const int64_t base = nz / parts, rem = nz % parts;
  return (int64_t)p * base + std::min<int64_t>(p, rem);
}

int SlabDecomposition::owner(int64_t gz) const {
  MDFX_CHECK(gz >= 0 && gz < nz, "plane outside the grid");
  const int64_t base = nz / parts, rem = nz % parts;
  const int64_t split = rem * (base + 1);
  if (gz < split) return (int)(gz / (base + 1));
  return (int)(rem + (gz - split) / base);
}

}  // namespace mdfx
