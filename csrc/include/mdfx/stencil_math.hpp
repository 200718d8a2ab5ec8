// Canonical point-update arithmetic, shared verbatim by the gfx950 kernels and the CPU oracle so
// that results are bitwise reproducible across backends, kernel variants and decompositions.
//
// Reference parity:
//   MDF update  MDF_kernel.cu:20  new = 0.25*(E+W+N+S - 4u) + u, evaluated there with an fp32 sum
//               and an fp64 scale/add. Here the whole update stays in the field's
//               dtype: s = ((W+E)+N)+S; u' = fma(r, fma(-4, u, s), u).
//   GoL rule    kernel.cu:66   alive' = n==3 || (n==2 && alive). With T = 3x3 sum including self
//               this is T==3 || (T==4 && alive).
#pragma once

#include <cmath>

#if defined(__HIPCC__)
#define MDFX_HDI __host__ __device__ __forceinline__
#else
#define MDFX_HDI inline
#endif

namespace mdfx {
namespace sm {

MDFX_HDI float fmaT(float a, float b, float c) { return fmaf(a, b, c); }
MDFX_HDI double fmaT(double a, double b, double c) { return fma(a, b, c); }

// 3D 7-point heat / Jacobi: s = ((((xm+xp)+ym)+yp)+zm)+zp ; u' = u + r*(s - 6u)
template <class T>
MDFX_HDI T heat7(T c, T xm, T xp, T ym, T yp, T zm, T zp, T r) {
  const T s = ((((xm + xp) + ym) + yp) + zm) + zp;
  return fmaT(r, fmaT(T(-6), c, s), c);
}

// 2D 5-point (rows are the z axis): s = ((xm+xp)+zm)+zp ; u' = u + r*(s - 4u)
template <class T>
MDFX_HDI T jacobi5(T c, T xm, T xp, T zm, T zp, T r) {
  const T s = ((xm + xp) + zm) + zp;
  return fmaT(r, fmaT(T(-4), c, s), c);
}

// The reference's own evaluation of the MDF update (MDF_kernel.cu:20), for pinning its
// semantics bit for bit: the fp32 neighbour sum ((E+W)+N)+S and the -4u term contracted into an
// fp32 fma by hipcc, then `0.25*(...) + u` with a double literal, i.e. one fp64 fma on the widened
// values, rounded back to the field type by the store. (E+W == W+E: IEEE addition commutes.)
template <class T>
MDFX_HDI T jacobi5_ref(T c, T xm, T xp, T zm, T zp, T r) {
  const T s = ((xm + xp) + zm) + zp;
  const T t = fmaT(T(-4), c, s);
  return (T)fma((double)r, (double)t, (double)c);
}

// 3D 27-point as a sum of per-plane partials. For one plane and one output column (x, y):
//   center = v(x,y); cross = (v(x-1,y)+v(x+1,y)) + (v(x,y-1)+v(x,y+1));
//   diag   = (v(x-1,y-1)+v(x+1,y-1)) + (v(x-1,y+1)+v(x+1,y+1))
//   A (off-plane contribution) = c3*diag + c2*cross + c1*center
//   B (in-plane contribution)  = c2*diag + c1*cross + c0*center
//   u'(z) = (A(z-1) + B(z)) + A(z+1)
// which equals c0*u + c1*faces(6) + c2*edges(12) + c3*corners(8).
template <class T>
MDFX_HDI T box27_A(T center, T cross, T diag, T c1, T c2, T c3) {
  return fmaT(c3, diag, fmaT(c2, cross, c1 * center));
}
template <class T>
MDFX_HDI T box27_B(T center, T cross, T diag, T c0, T c1, T c2) {
  return fmaT(c2, diag, fmaT(c1, cross, c0 * center));
}
template <class T>
MDFX_HDI T box27_combine(T a_m, T b_c, T a_p) {
  return (a_m + b_c) + a_p;
}

// Life: T = sum of the 3x3 block including self.
MDFX_HDI unsigned char life_rule(unsigned t, unsigned char alive) {
  return (unsigned char)((t == 3u) | ((t == 4u) & (alive != 0)));
}

}  // namespace sm
}  // namespace mdfx
