// Register layouts and arithmetic of one lane's 16-B row slice for the streaming multi-level
// kernels (heat7_tbk, box27_tbk, jacobi5_tbk), plus the flat per-level state indexing they share.
#pragma once

#include "kcommon.hpp"

namespace mdfx {
namespace dev {

// first row of level k (1..K) in the flat per-level state arrays
template <int RY, int K>
__host__ __device__ constexpr int tbk_off(int k) {
  return (k - 1) * RY + 2 * ((k - 1) * K - (k - 1) * k / 2);
}

// One lane's slice of a row, in the register layout the arithmetic wants.
//  fp32: the 4 cells as two aligned pairs a = (e1, e2), b = (e0, e3). Then
//        x sums (xm + xp) = { (l, rr) + a , b + swap(a) }  -> 2 v_pk_add_f32,
//        and every y / z / update operation is one packed op per pair, with no lane shuffles
//        or register moves to form misaligned pairs (natural (e0,e1),(e2,e3) pairs need them).
//  fp64: the 2 cells as they are (no packed fp64 arithmetic on CDNA).
// `E` is the edge pair (e0, e_{N-1}) the neighbouring waves need.
template <class T>
struct RowOps;

template <>
struct RowOps<float> {
  typedef float T2 __attribute__((ext_vector_type(2)));
  typedef float V __attribute__((ext_vector_type(4)));
  struct Row {
    T2 a, b;
  };
  // natural 16-B vector at p (one ds_read_b128), regrouped into the pair layout
  static __device__ __forceinline__ Row lds(const float* p) {
    const V v = *(const V*)p;
    Row r;
    r.a = T2{v.y, v.z};
    r.b = T2{v.x, v.w};
    return r;
  }
  // the same from two ds_read2_b32 that land each pair in an aligned register pair (a 16-B read
  // would need 4 moves to regroup). The caller waits for lgkmcnt(0) and then passes the row
  // through fence() before the first use.
  static __device__ __forceinline__ Row lds_pairs(const float* p) {
    const unsigned a = (unsigned)(uintptr_t)((const __attribute__((address_space(3))) float*)p);
    Row r;
    asm volatile("ds_read2_b32 %0, %2 offset0:1 offset1:2\n\tds_read2_b32 %1, %2 offset1:3"
                 : "=&v"(r.a), "=&v"(r.b)
                 : "v"(a));
    return r;
  }
  static __device__ __forceinline__ void fence(Row& r) { asm volatile("" : "+v"(r.a), "+v"(r.b)); }
  static __device__ __forceinline__ void pin(Row&) {}
  static __device__ __forceinline__ Row zero() { return Row{T2{0.f, 0.f}, T2{0.f, 0.f}}; }
  static __device__ __forceinline__ float first(const Row& c) { return c.b.x; }
  static __device__ __forceinline__ float last(const Row& c) { return c.b.y; }
  static __device__ __forceinline__ T2 edges(const Row& c) { return c.b; }
  // (((xm + xp) + ym) + yp) + zm
  static __device__ __forceinline__ Row partial(const Row& c, float l, float rr, const Row& ym, const Row& yp,
                                                const Row& zm) {
    const T2 lr = T2{l, rr};
    const T2 sa = T2{c.a.y, c.a.x};
    Row s;
    s.b = lr + c.a;  // (l + e1, rr + e2)
    s.a = c.b + sa;  // (e0 + e2, e3 + e1)
    s.a = ((s.a + ym.a) + yp.a) + zm.a;
    s.b = ((s.b + ym.b) + yp.b) + zm.b;
    return s;
  }
  // fma(r, fma(-6, c, S + zp), c) with a per-cell coefficient in the Row layout (0 = held)
  static __device__ __forceinline__ Row fin(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m6 = T2{-6.f, -6.f};
    Row o;
    o.a = __builtin_elementwise_fma(rc.a, __builtin_elementwise_fma(m6, c.a, S.a + zp.a), c.a);
    o.b = __builtin_elementwise_fma(rc.b, __builtin_elementwise_fma(m6, c.b, S.b + zp.b), c.b);
    return o;
  }
  static __device__ __forceinline__ Row partial5(const Row& c, float l, float rr, const Row& zm) {
    return add(hsum(c, l, rr), zm);
  }
  // fma(r, fma(-4, c, S + zp), c): sm::jacobi5 with S = (xm + xp) + zm
  static __device__ __forceinline__ Row fin4(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m4 = T2{-4.f, -4.f};
    Row o;
    o.a = __builtin_elementwise_fma(rc.a, __builtin_elementwise_fma(m4, c.a, S.a + zp.a), c.a);
    o.b = __builtin_elementwise_fma(rc.b, __builtin_elementwise_fma(m4, c.b, S.b + zp.b), c.b);
    return o;
  }
  // sm::jacobi5_ref: t = fma(-4, c, S + zp) in fp32, then (float)fma((double)r, (double)t, (double)c)
  static __device__ __forceinline__ Row fin4_ref(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m4 = T2{-4.f, -4.f};
    const T2 ta = __builtin_elementwise_fma(m4, c.a, S.a + zp.a);
    const T2 tb = __builtin_elementwise_fma(m4, c.b, S.b + zp.b);
    Row o;
    o.a.x = (float)__builtin_fma((double)rc.a.x, (double)ta.x, (double)c.a.x);
    o.a.y = (float)__builtin_fma((double)rc.a.y, (double)ta.y, (double)c.a.y);
    o.b.x = (float)__builtin_fma((double)rc.b.x, (double)tb.x, (double)c.b.x);
    o.b.y = (float)__builtin_fma((double)rc.b.y, (double)tb.y, (double)c.b.y);
    return o;
  }
  static __device__ __forceinline__ Row coef(float r, const bool* held) {
    return Row{T2{held[1] ? 0.f : r, held[2] ? 0.f : r}, T2{held[0] ? 0.f : r, held[3] ? 0.f : r}};
  }
  static __device__ __forceinline__ float get(const Row& c, int e) {
    return e == 0 ? c.b.x : e == 1 ? c.a.x : e == 2 ? c.a.y : c.b.y;
  }
  static __device__ __forceinline__ void set(Row& c, int e, float v) {
    if (e == 0) c.b.x = v;
    else if (e == 1) c.a.x = v;
    else if (e == 2) c.a.y = v;
    else c.b.y = v;
  }
  static __device__ __forceinline__ V vec(const Row& c) { return V{c.b.x, c.a.x, c.a.y, c.b.y}; }
  // ---- 27-point helpers (box27_tbk) ----
  static __device__ __forceinline__ Row add(const Row& x, const Row& y) { return Row{x.a + y.a, x.b + y.b}; }
  // x * s for a wave-uniform s (2 packed multiplies instead of 8 selects for a 0 / 1 choice)
  static __device__ __forceinline__ Row scale(const Row& x, float s) { return Row{x.a * T2{s, s}, x.b * T2{s, s}}; }
  // xm + xp of every cell; l / rr are the cells beyond the slice's ends
  static __device__ __forceinline__ Row hsum(const Row& c, float l, float rr) {
    Row h;
    h.b = T2{l, rr} + c.a;           // (l + e1, rr + e2)
    h.a = c.b + T2{c.a.y, c.a.x};    // (e0 + e2, e3 + e1)
    return h;
  }
  // fma(k2, d, fma(k1, x, k0 * c)): sm::box27_A / box27_B
  static __device__ __forceinline__ Row lin3(const Row& c, const Row& x, const Row& d, float k0, float k1, float k2) {
    const T2 K0{k0, k0}, K1{k1, k1}, K2{k2, k2};
    Row o;
    o.a = __builtin_elementwise_fma(K2, d.a, __builtin_elementwise_fma(K1, x.a, K0 * c.a));
    o.b = __builtin_elementwise_fma(K2, d.b, __builtin_elementwise_fma(K1, x.b, K0 * c.b));
    return o;
  }
  // per cell: held ? h : o
  static __device__ __forceinline__ Row sel(const bool* held, const Row& h, const Row& o) {
    Row r;
    r.b.x = held[0] ? h.b.x : o.b.x;
    r.a.x = held[1] ? h.a.x : o.a.x;
    r.a.y = held[2] ? h.a.y : o.a.y;
    r.b.y = held[3] ? h.b.y : o.b.y;
    return r;
  }
};

template <>
struct RowOps<double> {
  typedef double T2 __attribute__((ext_vector_type(2)));
  typedef T2 V;
  struct Row {
    T2 v;
  };
  static __device__ __forceinline__ Row lds(const double* p) { return Row{*(const T2*)p}; }
  static __device__ __forceinline__ Row fromv(const V& v) { return Row{v}; }
  static __device__ __forceinline__ Row lds_pairs(const double* p) { return lds(p); }
  static __device__ __forceinline__ void fence(Row&) {}
  static __device__ __forceinline__ void pin(Row&) {}
  static __device__ __forceinline__ Row zero() { return Row{T2{0.0, 0.0}}; }
  static __device__ __forceinline__ double first(const Row& c) { return c.v.x; }
  static __device__ __forceinline__ double last(const Row& c) { return c.v.y; }
  static __device__ __forceinline__ T2 edges(const Row& c) { return c.v; }
  static __device__ __forceinline__ Row partial(const Row& c, double l, double rr, const Row& ym, const Row& yp,
                                                const Row& zm) {
    Row s;
    s.v = T2{l + c.v.y, c.v.x + rr};
    s.v = ((s.v + ym.v) + yp.v) + zm.v;
    return s;
  }
  static __device__ __forceinline__ Row fin(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m6 = T2{-6.0, -6.0};
    return Row{__builtin_elementwise_fma(rc.v, __builtin_elementwise_fma(m6, c.v, S.v + zp.v), c.v)};
  }
  static __device__ __forceinline__ Row fin4(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m4 = T2{-4.0, -4.0};
    return Row{__builtin_elementwise_fma(rc.v, __builtin_elementwise_fma(m4, c.v, S.v + zp.v), c.v)};
  }
  static __device__ __forceinline__ Row fin4_ref(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    return fin4(S, zp, c, rc);  // fp64 fields: the reference's widening is the identity
  }
  static __device__ __forceinline__ Row partial5(const Row& c, double l, double rr, const Row& zm) {
    return Row{T2{l + c.v.y, c.v.x + rr} + zm.v};
  }
  static __device__ __forceinline__ Row coef(double r, const bool* held) {
    return Row{T2{held[0] ? 0.0 : r, held[1] ? 0.0 : r}};
  }
  static __device__ __forceinline__ double get(const Row& c, int e) { return e == 0 ? c.v.x : c.v.y; }
  static __device__ __forceinline__ void set(Row& c, int e, double v) {
    if (e == 0) c.v.x = v;
    else c.v.y = v;
  }
  static __device__ __forceinline__ V vec(const Row& c) { return c.v; }
  static __device__ __forceinline__ Row add(const Row& x, const Row& y) { return Row{x.v + y.v}; }
  static __device__ __forceinline__ Row scale(const Row& x, double s) { return Row{x.v * T2{s, s}}; }
  static __device__ __forceinline__ Row hsum(const Row& c, double l, double rr) {
    return Row{T2{l + c.v.y, c.v.x + rr}};
  }
  static __device__ __forceinline__ Row lin3r(const Row& c, const Row& x, const Row& d, const Row& k0, const Row& k1,
                                              const Row& k2) {
    return Row{__builtin_elementwise_fma(k2.v, d.v, __builtin_elementwise_fma(k1.v, x.v, k0.v * c.v))};
  }
  static __device__ __forceinline__ Row fmaz(double z, const Row& a, const Row& s) {
    return Row{__builtin_elementwise_fma(T2{z, z}, a.v, s.v)};
  }
  static __device__ __forceinline__ Row coefv(double v, double h, const bool* held) {
    return Row{T2{held[0] ? h : v, held[1] ? h : v}};
  }
  static __device__ __forceinline__ Row splat(double v) { return Row{T2{v, v}}; }
  static __device__ __forceinline__ Row lin3(const Row& c, const Row& x, const Row& d, double k0, double k1,
                                             double k2) {
    const T2 K0{k0, k0}, K1{k1, k1}, K2{k2, k2};
    return Row{__builtin_elementwise_fma(K2, d.v, __builtin_elementwise_fma(K1, x.v, K0 * c.v))};
  }
  static __device__ __forceinline__ Row sel(const bool* held, const Row& h, const Row& o) {
    return Row{T2{held[0] ? h.v.x : o.v.x, held[1] ? h.v.y : o.v.y}};
  }
};

// fp32 rows in the NATURAL pair layout p = (e0, e1), q = (e2, e3): a 16-B LDS or global vector is
// already two aligned register pairs, so nothing is regrouped after a ds_read_b128. The x sums are
// four scalar adds, two of them with the neighbour lane's cell as a DPP operand
// (v_add_f32_dpp wave_shr / wave_shl: the lane shift costs no instruction of its own), and every
// y / z / update operation is one packed op per pair. Issue slots per row update: 4 scalar x adds
// + 12 packed ops, against 2 DPP moves + 14 packed ops + about 5 regrouping moves in RowOps<float>.
// Needs -fno-slp-vectorize on the translation unit, or the two plain x adds get packed into one
// v_pk_add_f32 whose halves then have to be moved apart (Makefile / CMakeLists.txt).
struct RowOpsN {
  typedef float T2 __attribute__((ext_vector_type(2)));
  typedef float V __attribute__((ext_vector_type(4)));
  struct Row {
    T2 p, q;
  };
  static __device__ __forceinline__ Row lds(const float* a) {
    const V v = *(const V*)a;
    return Row{T2{v.x, v.y}, T2{v.z, v.w}};
  }
  static __device__ __forceinline__ Row fromv(const V& v) { return Row{T2{v.x, v.y}, T2{v.z, v.w}}; }
  static __device__ __forceinline__ Row zero() { return Row{T2{0.f, 0.f}, T2{0.f, 0.f}}; }
  // one scalar add the backend cannot pair with its neighbour into a v_pk_add_f32 (e0 + e2 and
  // e1 + e3 would pack, and their halves then need two moves to reach (e0,e1) / (e2,e3))
  static __device__ __forceinline__ float add1(float a, float b) {
    float r;
    asm("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
  }
  static __device__ __forceinline__ float first(const Row& c) { return c.p.x; }
  static __device__ __forceinline__ float last(const Row& c) { return c.q.y; }
  // (((xm + xp) + ym) + yp) + zm; l / rr are the cells beyond the slice's ends (lane shifts the
  // compiler folds into the adds as DPP operands)
  static __device__ __forceinline__ Row partial(const Row& c, float l, float rr, const Row& ym, const Row& yp,
                                                const Row& zm) {
    Row s;
    s.p.x = l + c.p.y;    // e0: xm + xp
    s.p.y = add1(c.p.x, c.q.x);  // e1
    s.q.x = add1(c.p.y, c.q.y);  // e2
    s.q.y = rr + c.q.x;   // e3
    s.p = ((s.p + ym.p) + yp.p) + zm.p;
    s.q = ((s.q + ym.q) + yp.q) + zm.q;
    return s;
  }
  static __device__ __forceinline__ Row fin(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m6 = T2{-6.f, -6.f};
    Row o;
    o.p = __builtin_elementwise_fma(rc.p, __builtin_elementwise_fma(m6, c.p, S.p + zp.p), c.p);
    o.q = __builtin_elementwise_fma(rc.q, __builtin_elementwise_fma(m6, c.q, S.q + zp.q), c.q);
    return o;
  }
  static __device__ __forceinline__ Row coef(float r, const bool* held) {
    return Row{T2{held[0] ? 0.f : r, held[1] ? 0.f : r}, T2{held[2] ? 0.f : r, held[3] ? 0.f : r}};
  }
  // ---- 27-point helpers (box27_tb2n) ----
  static __device__ __forceinline__ Row add(const Row& x, const Row& y) { return Row{x.p + y.p, x.q + y.q}; }
  // xm + xp of every cell; l / rr are the cells beyond the slice's ends
  static __device__ __forceinline__ Row hsum(const Row& c, float l, float rr) {
    Row h;
    h.p.x = l + c.p.y;
    h.p.y = add1(c.p.x, c.q.x);
    h.q.x = add1(c.p.y, c.q.y);
    h.q.y = rr + c.q.x;
    return h;
  }
  // fma(k2, d, fma(k1, x, k0 * c)): sm::box27_A / box27_B
  static __device__ __forceinline__ Row lin3(const Row& c, const Row& x, const Row& d, float k0, float k1, float k2) {
    const T2 K0{k0, k0}, K1{k1, k1}, K2{k2, k2};
    Row o;
    o.p = __builtin_elementwise_fma(K2, d.p, __builtin_elementwise_fma(K1, x.p, K0 * c.p));
    o.q = __builtin_elementwise_fma(K2, d.q, __builtin_elementwise_fma(K1, x.q, K0 * c.q));
    return o;
  }
  // per cell: held ? h : o
  static __device__ __forceinline__ Row sel(const bool* held, const Row& h, const Row& o) {
    Row r;
    r.p.x = held[0] ? h.p.x : o.p.x;
    r.p.y = held[1] ? h.p.y : o.p.y;
    r.q.x = held[2] ? h.q.x : o.q.x;
    r.q.y = held[3] ? h.q.y : o.q.y;
    return r;
  }
  // 2D 5-point: (xm + xp) + zm, and fma(r, fma(-4, c, S + zp), c) (sm::jacobi5)
  static __device__ __forceinline__ Row partial5(const Row& c, float l, float rr, const Row& zm) {
    Row s;
    s.p.x = l + c.p.y;
    s.p.y = add1(c.p.x, c.q.x);
    s.q.x = add1(c.p.y, c.q.y);
    s.q.y = rr + c.q.x;
    s.p = s.p + zm.p;
    s.q = s.q + zm.q;
    return s;
  }
  static __device__ __forceinline__ Row fin4(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m4 = T2{-4.f, -4.f};
    Row o;
    o.p = __builtin_elementwise_fma(rc.p, __builtin_elementwise_fma(m4, c.p, S.p + zp.p), c.p);
    o.q = __builtin_elementwise_fma(rc.q, __builtin_elementwise_fma(m4, c.q, S.q + zp.q), c.q);
    return o;
  }
  // sm::jacobi5_ref: t = fma(-4, c, S + zp) in fp32, then (float)fma((double)r, (double)t, (double)c)
  static __device__ __forceinline__ Row fin4_ref(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m4 = T2{-4.f, -4.f};
    const T2 tp = __builtin_elementwise_fma(m4, c.p, S.p + zp.p);
    const T2 tq = __builtin_elementwise_fma(m4, c.q, S.q + zp.q);
    Row o;
    o.p.x = (float)__builtin_fma((double)rc.p.x, (double)tp.x, (double)c.p.x);
    o.p.y = (float)__builtin_fma((double)rc.p.y, (double)tp.y, (double)c.p.y);
    o.q.x = (float)__builtin_fma((double)rc.q.x, (double)tq.x, (double)c.q.x);
    o.q.y = (float)__builtin_fma((double)rc.q.y, (double)tq.y, (double)c.q.y);
    return o;
  }
  static __device__ __forceinline__ Row scale(const Row& x, float s) { return Row{x.p * T2{s, s}, x.q * T2{s, s}}; }
  static __device__ __forceinline__ float get(const Row& c, int e) {
    return e == 0 ? c.p.x : e == 1 ? c.p.y : e == 2 ? c.q.x : c.q.y;
  }
  static __device__ __forceinline__ V vec(const Row& c) { return V{c.p.x, c.p.y, c.q.x, c.q.y}; }
  // ---- 27-point with per-cell coefficients (box27_wxk) ----
  // fma(k2, d, fma(k1, x, k0 * c)) with per-cell coefficient rows
  static __device__ __forceinline__ Row lin3r(const Row& c, const Row& x, const Row& d, const Row& k0, const Row& k1,
                                              const Row& k2) {
    Row o;
    o.p = __builtin_elementwise_fma(k2.p, d.p, __builtin_elementwise_fma(k1.p, x.p, k0.p * c.p));
    o.q = __builtin_elementwise_fma(k2.q, d.q, __builtin_elementwise_fma(k1.q, x.q, k0.q * c.q));
    return o;
  }
  // fma(z, a, s) for a wave-uniform z in {0, 1}: s + a (z = 1, one rounding as an add) or s (z = 0)
  static __device__ __forceinline__ Row fmaz(float z, const Row& a, const Row& s) {
    const T2 zz{z, z};
    return Row{__builtin_elementwise_fma(zz, a.p, s.p), __builtin_elementwise_fma(zz, a.q, s.q)};
  }
  // per cell: held ? h : v
  static __device__ __forceinline__ Row coefv(float v, float h, const bool* held) {
    return Row{T2{held[0] ? h : v, held[1] ? h : v}, T2{held[2] ? h : v, held[3] ? h : v}};
  }
  static __device__ __forceinline__ Row splat(float v) { return Row{T2{v, v}, T2{v, v}}; }
  // materialise a loop-carried row where it is computed: otherwise hipcc carries the INPUTS of the
  // partial sum across the back edge and forms it in the next iteration, where the lane-shift
  // moves can no longer fold into the adds as DPP operands (DPP combining works inside a block)
  static __device__ __forceinline__ void pin(Row& r) { asm volatile("" : "+v"(r.p), "+v"(r.q)); }
  // the same without `volatile`: still materialises the row, but is no scheduling barrier
  static __device__ __forceinline__ void pin_nv(Row& r) { asm("" : "+v"(r.p), "+v"(r.q)); }
};

// fp32 rows of 2 cells per lane (one 8-B vector; heat7_wxk's 5-step sweep): half the registers per
// row of RowOpsN at the same issue count per cell (2 x adds, both with the neighbour lane's cell as
// a DPP operand, + 6 packed ops per row update), so a wave holds the rows of a fifth level
static constexpr int kRowOps2 = 2;
struct RowOps2f {
  typedef float T2 __attribute__((ext_vector_type(2)));
  typedef T2 V;
  struct Row {
    T2 v;
  };
  static __device__ __forceinline__ Row fromv(const V& v) { return Row{v}; }
  static __device__ __forceinline__ Row zero() { return Row{T2{0.f, 0.f}}; }
  static __device__ __forceinline__ float first(const Row& c) { return c.v.x; }
  static __device__ __forceinline__ float last(const Row& c) { return c.v.y; }
  // (((xm + xp) + ym) + yp) + zm; l / rr are the cells beyond the slice's ends
  static __device__ __forceinline__ Row partial(const Row& c, float l, float rr, const Row& ym, const Row& yp,
                                                const Row& zm) {
    Row s;
    s.v.x = l + c.v.y;
    s.v.y = c.v.x + rr;
    s.v = ((s.v + ym.v) + yp.v) + zm.v;
    return s;
  }
  static __device__ __forceinline__ Row fin(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    const T2 m6 = T2{-6.f, -6.f};
    return Row{__builtin_elementwise_fma(rc.v, __builtin_elementwise_fma(m6, c.v, S.v + zp.v), c.v)};
  }
  static __device__ __forceinline__ Row coef(float r, const bool* held) {
    return Row{T2{held[0] ? 0.f : r, held[1] ? 0.f : r}};
  }
  static __device__ __forceinline__ Row scale(const Row& x, float s) { return Row{x.v * T2{s, s}}; }
  static __device__ __forceinline__ float get(const Row& c, int e) { return e == 0 ? c.v.x : c.v.y; }
  static __device__ __forceinline__ V vec(const Row& c) { return c.v; }
  // (as RowOpsN::pin: the row is formed where it is computed, so the lane shifts fold into the
  // adds as DPP operands; a non-volatile pin that lets rows interleave measured the same, +0.4-0.8 %
  // in the kernel A/B, profiles/r05_session_w/)
  static __device__ __forceinline__ void pin(Row& r) { asm volatile("" : "+v"(r.v)); }
  // ---- 27-point with per-cell coefficients (box27_wxk narrow rows; RowOpsN's arithmetic) ----
  static __device__ __forceinline__ Row add(const Row& x, const Row& y) { return Row{x.v + y.v}; }
  static __device__ __forceinline__ Row hsum(const Row& c, float l, float rr) { return Row{T2{l + c.v.y, c.v.x + rr}}; }
  static __device__ __forceinline__ Row lin3r(const Row& c, const Row& x, const Row& d, const Row& k0, const Row& k1,
                                              const Row& k2) {
    return Row{__builtin_elementwise_fma(k2.v, d.v, __builtin_elementwise_fma(k1.v, x.v, k0.v * c.v))};
  }
  static __device__ __forceinline__ Row fmaz(float z, const Row& a, const Row& s) {
    return Row{__builtin_elementwise_fma(T2{z, z}, a.v, s.v)};
  }
  static __device__ __forceinline__ Row coefv(float v, float h, const bool* held) {
    return Row{T2{held[0] ? h : v, held[1] ? h : v}};
  }
};

// fp64 rows of 1 cell per lane (one 8-B value; heat7_wxk's fp64 5-step sweep): the register footprint
// of RowOps2f, so a wave holds the same five levels of 5 + 4-row bands. Each x neighbour is two
// v_mov_b32_dpp (64-bit VALU ops take no DPP operand on gfx9), and a 64-lane segment owns only
// 64 - 2K columns (OV = K overlap lanes per side at one cell per lane)
static constexpr int kRowOps1 = 1;
struct RowOps1d {
  typedef double V;
  struct Row {
    double v;
  };
  static __device__ __forceinline__ Row fromv(const V& v) { return Row{v}; }
  static __device__ __forceinline__ Row zero() { return Row{0.0}; }
  static __device__ __forceinline__ double first(const Row& c) { return c.v; }
  static __device__ __forceinline__ double last(const Row& c) { return c.v; }
  // (((xm + xp) + ym) + yp) + zm; l / rr are the neighbour lanes' cells
  static __device__ __forceinline__ Row partial(const Row&, double l, double rr, const Row& ym, const Row& yp,
                                                const Row& zm) {
    return Row{(((l + rr) + ym.v) + yp.v) + zm.v};
  }
  static __device__ __forceinline__ Row fin(const Row& S, const Row& zp, const Row& c, const Row& rc) {
    return Row{__builtin_fma(rc.v, __builtin_fma(-6.0, c.v, S.v + zp.v), c.v)};
  }
  static __device__ __forceinline__ Row coef(double r, const bool* held) { return Row{held[0] ? 0.0 : r}; }
  static __device__ __forceinline__ Row scale(const Row& x, double s) { return Row{x.v * s}; }
  static __device__ __forceinline__ double get(const Row& c, int) { return c.v; }
  static __device__ __forceinline__ V vec(const Row& c) { return c.v; }
  static __device__ __forceinline__ void pin(Row& r) { asm volatile("" : "+v"(r.v)); }
};

}  // namespace dev
}  // namespace mdfx
