// rc_device.hpp — per-pixel device routines of the MI355X raycaster.
//
// Bit-exact restatement of the reference render semantics (C/raycast.c:79-758,
// C/v3math.c:19-192, C/ppm.c:350-359) for gfx950.  Compiled with -ffp-contract=off and
// IEEE f32/f64 division and square root, so every float/double operation below rounds
// exactly as the x86-64 gcc -O3 build does (SSE2, no FMA).  The two libm calls are replaced
// by exact constructions:
//   pow(x, 0.5)  -> sqrt(x)                         (byte-identical output)
//   pow(x, 20)   -> x^20 in double-double, rounded once (correctly rounded)
//   pow(a, n)    -> a^n in double-double for integer spot exponents
//
// Structure on CDNA4: one lane per pixel; the shape loop is wave-uniform (every lane tests
// shape k together), so shape records are read with scalar loads into SGPRs and the
// per-type branch is a scalar branch.  Hit post-processing (hit point, normal) is deferred
// to after the loop: it depends only on (ray, t, shape), so computing it once for the final
// winner is identical to the reference's write-on-every-accept (C/raycast.c:460-470).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rc_scene.h"

namespace rc {

constexpr int kModeFast = 0;      // reflection miss ends the bounce loop
constexpr int kModeParityA = 1;   // parity, phase A: stop at a first-bounce miss (DEP pixel)
constexpr int kModeParityC = 2;   // parity, phase C: first-bounce miss reads the given carry
constexpr int kModeClassify = 3;  // parity, phase A without shading: class, DEP record, carry

constexpr uint8_t kClsIdent = 0;  // pixel never writes the carry
constexpr uint8_t kClsWriter = 1; // first bounce hit: carry-out independent of carry-in
constexpr uint8_t kClsDep = 2;    // first bounce missed: needs the scan-order carry

struct Scene {
  const rc_shape* __restrict__ shapes;   // n + 1 records (n = phantom)
  const rc_light* __restrict__ lights;   // m records
  const rc_shade_pair* __restrict__ pairs;
  // Per-lane (divergent) record reads — the winner's frame, its shading record and colour
  // pairs — go through these: LDS copies when the kernel staged the scene (stage_scene),
  // else the global records.  Uniform loops over shapes/lights keep the scalar path above.
  const rc_shape* lshapes;
  const rc_shade_pair* lpairs;
  int n, m;
  unsigned long long refl_mask;          // bit k: shape k has reflectivity > 0 (k < 64)
  int has_quadric;                       // any quadric: picks the evaluator specialisation;
                                         // 2: none of them has cross terms (quad_x0)
  int o0_ok;                             // primary rays may use rc_shape::o0 (nearest_primary)
  // Clean DEP entries (no bounce level hits at their carry-in) take their colour from phase
  // A's primary shade: set when every level's shade of such an entry is exactly zero (black
  // phantom, finite reflectivities; host check in upload_scene).
  int dep_fast;
};

// refl[obj] > 0 (C/raycast.c:352) from a register bitmask when n <= 64
__device__ __forceinline__ bool reflective(const Scene& sc, int obj) {
  if (sc.n <= 64) return (sc.refl_mask >> obj) & 1ull;
  return sc.lshapes[obj].refl > 0.0f;
}

struct Cam {
  double hx, hy;   // (0.0 - cw/2.0) and (0.0 + ch/2.0)      C/raycast.c:115-116
  float pw, ph;    // cw/(float)W, ch/(float)H                C/raycast.c:109-110
};

struct V3 {
  float x, y, z;
};

__device__ __forceinline__ V3 v3(float x, float y, float z) { return V3{x, y, z}; }

// C/v3math.c:69-71
__device__ __forceinline__ float dot(V3 a, V3 b) {
  float s = a.x * b.x;
  s = s + a.y * b.y;
  return s + a.z * b.z;
}
__device__ __forceinline__ V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }

// Quotients n / d of the resolver's shape test through one shared reciprocal.  This is the
// compiler's IEEE f64 division sequence (v_rcp_f64, two Newton steps, q0 = n*y, the residual
// r = n - d*q0 and q = q0 + r*y, each rounded once) without its v_div_scale / v_div_fmas /
// v_div_fixup steps, which change nothing unless an operand is extreme: they rescale only for
// |n| < 2^-969, |d| > 2^1021 or exponent gaps beyond 768, and fix up zero, inf and NaN
// operands.  The tests' operands are float-derived (|n| in [2^-201, 2^130] or 0, |d| in
// [2^-148, 2^130]), so every finite quotient is bit-identical to n / d; where n or d is 0, inf
// or NaN the value differs (NaN or an unsigned zero instead of +-inf or -0) but such a t is
// rejected either way (t > 0 and t < inf; a zero or infinite denominator never yields an
// accepted root), which is all the callers use it for.
#ifndef RC_NRDIV
#define RC_NRDIV 1
#endif
__device__ __forceinline__ double recip_nr(double d) {
  double y = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, y, 1.0);
  y = __builtin_fma(y, e, y);
  e = __builtin_fma(-d, y, 1.0);
  return __builtin_fma(y, e, y);
}
__device__ __forceinline__ double div_nr(double n, double d, double y) {
  const double q0 = n * y;
  const double r = __builtin_fma(-d, q0, n);
  return __builtin_fma(r, y, q0);
}

// Correctly rounded f64 sqrt for s = +-0, s >= 2^-767, +inf or NaN — every value it is used
// on here: sums of squares of floats (0 or >= 2^-298) and non-negative floats widened to
// double (0 or >= 2^-149).  This is the compiler's own rsq + Goldschmidt/Newton sequence
// without its range scaling, which it applies only below 2^-767, so results are identical.
__device__ __forceinline__ double sqrt_ns(double s) {
  const double y = __builtin_amdgcn_rsq(s);
  double g = s * y, h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, s);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, s);
  g = __builtin_fma(d, h, g);
  return (s == 0.0 || s == __builtin_inf()) ? s : g;
}

// ((x^2 + y^2) + z^2) in double for floats x, y, z, each addition rounded once: the square of
// a float is exact in double (48 significant bits), so fma(y, y, x*x) rounds exactly the sum
// the reference rounds — one instruction per term instead of a multiply and an add.
__device__ __forceinline__ double sumsq3(double x, double y, double z) {
  return __builtin_fma(z, z, __builtin_fma(y, y, x * x));
}

// Discriminants b*b - p with b a float and p an exact double product (4*a*c of floats, or a
// float widened): b*b is exact too, so fma(b, b, -p) rounds the same difference once.

// C/v3math.c:169-172 — (float)sqrt of an exact double sum of squares
__device__ __forceinline__ float length(V3 a) {
  return (float)sqrt_ns(sumsq3((double)a.x, (double)a.y, (double)a.z));
}

// a_i / len for the three components through one f64 reciprocal: r = 1/len to within
// 2^-52 (rcp + two Newton steps), q = (double)a_i * r within 2^-51.4 of a_i/len.  A quotient
// of two 24-bit floats is either a float or at least 2^-49 (relative) away from every
// rounding midpoint of the float grid, so RN32(q) = RN32(a_i/len), the IEEE f32 quotient.
// len = +inf: r = 0 gives a_i/inf (+-0, NaN for inf a_i); len NaN gives NaN; len = 0 is the
// caller's case.
__device__ __forceinline__ V3 div3(V3 a, float len) {
  const double L = (double)len;
  double r = __builtin_amdgcn_rcp(L);
  double e = __builtin_fma(-L, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-L, r, 1.0);
  r = __builtin_fma(r, e, r);
  r = len == __builtin_inff() ? 0.0 : r;
  return v3((float)((double)a.x * r), (float)((double)a.y * r), (float)((double)a.z * r));
}

// C/v3math.c:180-192 — a zero length leaves the vector unchanged (and is counted: the
// reference prints a stderr line per event).
__device__ __forceinline__ V3 normalize(V3 a, int& zero_events) {
  float len = length(a);
  if (len == 0.0f) {
    zero_events++;
    return a;
  }
  return div3(a, len);
}

// Materialise a value in a register as an opaque definition.  Codegen otherwise turns a
// select whose operand is an expensive single-use op (f64 division, sqrt) into a branch that
// computes the operand conditionally, which serialises the independent quotients.
template <class T>
__device__ __forceinline__ T pin(T x) {
  asm("" : "+v"(x));
  return x;
}

// component-wise select (a struct-valued ?: becomes a pointer select over stack copies)
__device__ __forceinline__ V3 sel(bool p, V3 a, V3 b) {
  return v3(p ? a.x : b.x, p ? a.y : b.y, p ? a.z : b.z);
}

__device__ __forceinline__ V3 normalize_sel(V3 a) {
  const float len = length(a);
  const V3 q = div3(a, len);
  return sel(len == 0.0f, a, v3(pin(q.x), pin(q.y), pin(q.z)));
}

// C/v3math.c:144-160 — v - n*(2*dot(v,n))
__device__ __forceinline__ V3 reflect(V3 v, V3 n) {
  float s = 2.0f * dot(v, n);
  return v3(v.x - n.x * s, v.y - n.y * s, v.z - n.z * s);
}

// ------------------------------------------------------------- double-double power --
struct DD {
  double hi, lo;
};
__device__ __forceinline__ DD dd_mul(DD a, DD b) {
  double p = a.hi * b.hi;
  double e = __builtin_fma(a.hi, b.hi, -p);
  e = e + (a.hi * b.lo + a.lo * b.hi);
  double s = p + e;
  return DD{s, e - (s - p)};
}
__device__ __forceinline__ DD dd_from_prod(double a, double b) {
  double p = a * b;
  return DD{p, __builtin_fma(a, b, -p)};
}
__device__ __forceinline__ double dd_round(DD a) { return a.hi + a.lo; }

// pow(x, 20) for the specular term (C/raycast.c:755-757); x = (double)float, so x*x is
// exact in double and x^20 = (x^2)^8 * (x^2)^2 is built in double-double and rounded once.
__device__ __forceinline__ double pow20(double x) {
  double x2 = x * x;                  // exact: x has 24 significant bits
  DD x4 = dd_from_prod(x2, x2);       // exact
  DD x8 = dd_mul(x4, x4);
  DD x16 = dd_mul(x8, x8);
  DD x20 = dd_mul(x16, x4);
  return dd_round(x20);
}

// pow(a, n) for an integer spot exponent (C/raycast.c:695), a = (double)float.
__device__ __forceinline__ double pown_dd(double a, int n) {
  if (n == 0) return 1.0;
  // a = (double)float: a and a*a are exact doubles (24 and 48 significant bits), which the
  // double-double loop below would return rounded — the same value, ~15 f64 operations less
  // (the examples' spot lights use angular-a0 2)
  if (n == 1) return a;
  if (n == 2) return a * a;
  unsigned e = n < 0 ? (unsigned)(-n) : (unsigned)n;
  DD base{a, 0.0}, acc{1.0, 0.0};
  while (e) {
    if (e & 1u) acc = dd_mul(acc, base);
    e >>= 1;
    if (e) base = dd_mul(base, base);
  }
  if (n > 0) return dd_round(acc);
  // 1 / acc in double-double, rounded once
  double q = 1.0 / acc.hi;
  DD qa = dd_mul(DD{q, 0.0}, acc);
  double r = (1.0 - qa.hi) - qa.lo;
  return q + q * r / 1.0;
}

// ------------------------------------------------------------------ intersections --
// Per-ray sphere constants: `a` depends only on the ray direction (C/raycast.c:583), so it
// is computed once per ray for every sphere test — the same value the reference recomputes.
struct RayK {
  float a4;     // 4 * a               (float, C/raycast.c:587)
  double den;   // 2.0 * (double)a     (C/raycast.c:593)
  double yden;  // recip_nr(den): the sphere quotients' shared reciprocal (RC_NRDIV)
};
__device__ __forceinline__ RayK ray_consts(V3 D) {
  float a = (float)sumsq3((double)D.x, (double)D.y, (double)D.z);
  const double den = 2.0 * (double)a;
  return RayK{4.0f * a, den, RC_NRDIV ? recip_nr(den) : 0.0};
}

// The candidate t = (float)(num / den) of a shape test (accepted only when 0 < t < inf):
// through the shared reciprocal y = recip_nr(den) (RC_NRDIV; bit-identical for every finite
// quotient, a rejected t for zero, infinite or NaN operands either way), else as written.
__device__ __forceinline__ float tquot(double num, double den, double y) {
#if RC_NRDIV
  return (float)div_nr(num, den, y);
#else
  (void)y;
  return (float)(num / den);
#endif
}

// C/raycast.c:576-600
__device__ __forceinline__ bool hit_sphere(V3 O, V3 D, const rc_shape& s, RayK k, float& t) {
  V3 tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
  float b = 2.0f * dot(D, tv);
  float c = (float)((double)dot(tv, tv) - s.r2);
  float fac = k.a4 * c;
  float disc = (float)__builtin_fma((double)b, (double)b, -(double)fac);
  if (disc < 0.0f) return false;
  double sq = sqrt_ns((double)disc);
  // both roots, then a select (with the shared reciprocal the second costs three operations,
  // less than the branch around it)
  const float t1 = pin(tquot((double)(-b) - sq, k.den, k.yden));
  const float t2 = pin(tquot((double)(-b) + sq, k.den, k.yden));
  t = t1 < 0.0f ? t2 : t1;
  return true;
}

// C/raycast.c:545-562
__device__ __forceinline__ bool hit_plane(V3 O, V3 D, const rc_shape& s, float& t) {
  V3 n = v3(s.n[0], s.n[1], s.n[2]);
  float num = dot(v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]), n);
  float den = dot(D, n);
  if (den == 0.0f) return false;
  float tt = (-num) / den;
  if (tt < 0.0f) return false;
  t = tt;
  return true;
}

// Quadrics without cross terms (d = e = f = 0 for every quadric of the scene, as in every
// example scene; quad_x0).  Each cross term is (+-0 coefficient) * (float operands):
//   a: (qd*D.x)*D.y, (qe*D.x)*D.z, (qf*D.y)*D.z      NaN iff some D component is inf/NaN
//   c: (qd*O.x)*O.y, (qe*O.x)*O.z, (qf*O.y)*O.z      NaN iff some O component is inf/NaN
//   b: qd*(O.x*D.y + O.y*D.x), qe*(..), qf*(..)      NaN iff one of the three float sums is
//                                                    inf/NaN
// and +-0 otherwise.  Adding +-0 to a double accumulator leaves it unchanged unless it is
// itself zero, so dropping the terms can change only the SIGN of a zero a, b or c, which no
// result of the test sees: a zero a takes the linear branch either way, b enters the
// discriminant squared and the roots as -b +- sqrt(disc) (a zero sqrt makes both roots +-0,
// rejected by t > 0), a zero b in the linear branch gives t = +-inf or NaN (rejected by
// best > t / t > 0), and a zero c makes 4ac = +-0, which leaves b*b unchanged.  A NaN term
// makes a, b or c NaN, and then every branch of the test ends in t = NaN, which every caller
// rejects (best > t, t > 0, quot_class).  So the short form plus one per-ray flag —
// x0_reject: some cross term would be NaN, the quadric is rejected — is bit-identical.
__device__ __forceinline__ bool quad_x0(const Scene& sc) { return sc.has_quadric == 2; }
__device__ __forceinline__ bool nonfinite3(float a, float b, float c) {
  return !__builtin_isfinite(a) | !__builtin_isfinite(b) | !__builtin_isfinite(c);
}
__device__ __forceinline__ bool x0_reject(V3 O, V3 D) {
  return nonfinite3(D.x, D.y, D.z) | nonfinite3(O.x, O.y, O.z) |
         nonfinite3(O.x * D.y + O.y * D.x, O.x * D.z + O.z * D.x, O.y * D.z + O.z * D.y);
}

// The quadric's a, b, c (C/raycast.c:614-641): double accumulations in source order, float
// products as written; kX0 drops the cross terms (quad_x0 with x0_reject, above).
__device__ __forceinline__ void quad_abc(V3 O, V3 D, const rc_shape& q, float& aq, float& bq,
                                         float& cq, bool x0) {
  // c, a, b: the order the resolver's evaluator has always used (its schedule is sensitive)
  double acc;
  acc = q.A * ((double)O.x * (double)O.x);
  acc = acc + q.B * ((double)O.y * (double)O.y);
  acc = acc + q.C * ((double)O.z * (double)O.z);
  if (!x0) {
    acc = acc + (double)(q.qd * O.x * O.y);
    acc = acc + (double)(q.qe * O.x * O.z);
    acc = acc + (double)(q.qf * O.y * O.z);
  }
  acc = acc + (double)(q.qg * O.x);
  acc = acc + (double)(q.qh * O.y);
  acc = acc + (double)(q.qi * O.z);
  acc = acc + (double)q.qj;
  cq = (float)acc;

  acc = q.A * ((double)D.x * (double)D.x);
  acc = acc + q.B * ((double)D.y * (double)D.y);
  acc = acc + q.C * ((double)D.z * (double)D.z);
  if (!x0) {
    acc = acc + (double)(q.qd * D.x * D.y);
    acc = acc + (double)(q.qe * D.x * D.z);
    acc = acc + (double)(q.qf * D.y * D.z);
  }
  aq = (float)acc;

  acc = 2.0 * q.A * (double)O.x * (double)D.x;
  acc = acc + 2.0 * q.B * (double)O.y * (double)D.y;
  acc = acc + 2.0 * q.C * (double)O.z * (double)D.z;
  if (!x0) {
    acc = acc + (double)(q.qd * (O.x * D.y + O.y * D.x));
    acc = acc + (double)(q.qe * (O.x * D.z + O.z * D.x));
    acc = acc + (double)(q.qf * (O.y * D.z + O.z * D.y));
  }
  acc = acc + (double)(q.qg * D.x);
  acc = acc + (double)(q.qh * D.y);
  acc = acc + (double)(q.qi * D.z);
  bq = (float)acc;
}

// C/raycast.c:614-656; x0 = quad_x0 (uniform), rej = x0 && x0_reject(O, D)
__device__ __forceinline__ bool hit_quadric(V3 O, V3 D, const rc_shape& q, float& t, bool x0,
                                            bool rej) {
  float aq, bq, cq;
  quad_abc(O, D, q, aq, bq, cq, x0);
  if (rej) return false;
  if ((double)aq == 0.0) {
    t = tquot(-1.0 * (double)cq, (double)bq, RC_NRDIV ? recip_nr((double)bq) : 0.0);
    return true;
  }
  const float disc = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
  if ((double)disc < 0.0) return false;
  const double den = 2.0 * (double)aq;
  const double sq = sqrt_ns((double)disc);
  const double y = RC_NRDIV ? recip_nr(den) : 0.0;
  const float t1 = pin(tquot((double)(-bq) - sq, den, y));
  const float t2 = pin(tquot((double)(-bq) + sq, den, y));
  t = t1 <= 0.0f ? t2 : t1;
  return true;
}

// Shape test k for ray (O, D); `skip` is the bounce ray's skip index (-1 for primary and
// shadow-from-phantom rays).  Returns whether the shape would be accepted as a candidate
// with distance t (before the nearest/positive check).  Type is wave-uniform.
__device__ __forceinline__ bool test_shape(const rc_shape& s, V3 O, V3 D, RayK rk, int skip,
                                           float& t, bool x0 = false, bool rej = false) {
  const int type = s.type;
  if (type == RC_SHAPE_SPHERE) return hit_sphere(O, D, s, rk, t);
  if (type == RC_SHAPE_PLANE) return hit_plane(O, D, s, t);
  if (type == RC_SHAPE_QUADRIC) {
    if (!hit_quadric(O, D, s, t, x0, rej)) return false;
    // C/raycast.c:492-494: for bounce rays a quadric hit below the origin's z is ignored
    if (skip != -1 && (O.z + t * D.z) < O.z) return false;
    return true;
  }
  return false;
}

// C/raycast.c:441-531 (shadow_test = false): index of the nearest accepted shape, its t.
__device__ __forceinline__ int nearest(const Scene& sc, V3 O, V3 D, int skip, float& tbest) {
  const RayK rk = ray_consts(D);
  const bool x0 = quad_x0(sc), rej = x0 && x0_reject(O, D);
  float best = __builtin_inff();
  int idx = -1;
  for (int k = 0; k < sc.n; ++k) {
    float t = 0.0f;
    const bool hit = test_shape(sc.shapes[k], O, D, rk, skip, t, x0, rej);
    if (hit && k != skip && best > t && t > 0.0f) {
      best = t;
      idx = k;
    }
  }
  tbest = best;
  return idx;
}
// ------------------------------------------------------------------ primary rays --
// The primary ray of every pixel starts at O = (0,0,0) (C/raycast.c:118-121).  Each test's
// origin-only term is then a per-shape constant (rc_shape::o0, computed on the host by the
// same operations at O = +0: bit-identical), and the quadric's b loses its O terms: with
// finite coefficients each is a signed zero, and x + (+-0) = x for x != 0, so b equals
// ((g*Dx + h*Dy) + i*Dz) up to the sign of a zero result — which no caller can see: b enters
// disc only squared, a zero disc makes both roots +-0 (rejected by t > 0), and the linear
// case's c / +-0 is +-inf or NaN (rejected by best > t / t > 0 alike).
__device__ __forceinline__ bool hit_sphere_o0(V3 D, const rc_shape& s, RayK k, float& t) {
  const V3 tv = v3(0.0f - s.p[0], 0.0f - s.p[1], 0.0f - s.p[2]);
  float b = 2.0f * dot(D, tv);
  float fac = k.a4 * s.o0;
  float disc = (float)__builtin_fma((double)b, (double)b, -(double)fac);
  if (disc < 0.0f) return false;
  double sq = sqrt_ns((double)disc);
  const float t1 = pin(tquot((double)(-b) - sq, k.den, k.yden));
  const float t2 = pin(tquot((double)(-b) + sq, k.den, k.yden));
  t = t1 < 0.0f ? t2 : t1;
  return true;
}

__device__ __forceinline__ bool hit_plane_o0(V3 D, const rc_shape& s, float& t) {
  float den = dot(D, v3(s.n[0], s.n[1], s.n[2]));
  if (den == 0.0f) return false;
  float tt = (-s.o0) / den;
  if (tt < 0.0f) return false;
  t = tt;
  return true;
}

__device__ __forceinline__ bool hit_quadric_o0(V3 D, const rc_shape& q, float& t, bool x0) {
  double acc;
  acc = q.A * ((double)D.x * (double)D.x);
  acc = acc + q.B * ((double)D.y * (double)D.y);
  acc = acc + q.C * ((double)D.z * (double)D.z);
  if (!x0) {   // cross terms (quad_x0)
    acc = acc + (double)(q.qd * D.x * D.y);
    acc = acc + (double)(q.qe * D.x * D.z);
    acc = acc + (double)(q.qf * D.y * D.z);
  }
  const float aq = (float)acc;
  acc = (double)(q.qg * D.x);
  acc = acc + (double)(q.qh * D.y);
  acc = acc + (double)(q.qi * D.z);
  const float bq = (float)acc;
  const float cq = q.o0;
  if ((double)aq == 0.0) {
    t = tquot(-1.0 * (double)cq, (double)bq, RC_NRDIV ? recip_nr((double)bq) : 0.0);
    return true;
  }
  const float disc = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
  if ((double)disc < 0.0) return false;
  const double den = 2.0 * (double)aq;
  const double sq = sqrt_ns((double)disc);
  const double y = RC_NRDIV ? recip_nr(den) : 0.0;
  const float t1 = pin(tquot((double)(-bq) - sq, den, y));
  const float t2 = pin(tquot((double)(-bq) + sq, den, y));
  t = t1 <= 0.0f ? t2 : t1;
  return true;
}

// nearest(sc, (0,0,0), D, -1, tbest) for a primary ray.
__device__ __forceinline__ int nearest_primary(const Scene& sc, V3 D, float& tbest) {
  if (!sc.o0_ok) return nearest(sc, v3(0.0f, 0.0f, 0.0f), D, -1, tbest);
  const RayK rk = ray_consts(D);
  const bool x0 = quad_x0(sc), rej = x0 && x0_reject(v3(0.0f, 0.0f, 0.0f), D);
  float best = __builtin_inff();
  int idx = -1;
  for (int k = 0; k < sc.n; ++k) {
    const rc_shape& s = sc.shapes[k];
    float t = 0.0f;
    bool hit = false;
    if (s.type == RC_SHAPE_SPHERE) hit = hit_sphere_o0(D, s, rk, t);
    else if (s.type == RC_SHAPE_PLANE) hit = hit_plane_o0(D, s, t);
    else if (s.type == RC_SHAPE_QUADRIC)
      hit = hit_quadric_o0(D, s, t, x0) && !rej;
    if (hit && best > t && t > 0.0f) {
      best = t;
      idx = k;
    }
  }
  tbest = best;
  return idx;
}

// ------------------------------------------------------------------- shadow rays --
// A shadow ray only asks whether some shape is hit with 0 < t < inf (C/raycast.c:441-531
// with shadow_test = true); t itself is never used.  t = (float)(num / den) with an IEEE
// double quotient, so its class follows from the operands' signs and exponents alone when
// both are normal doubles whose biased exponents differ by e in [-148, 126]: then
// |num/den| lies in (2^(e-1), 2^(e+1)), which RN64 and then RN32 (both monotone, both
// bounds representable) keep inside [2^-149, 2^127] — a non-zero finite float of the
// quotient's sign.  Anything else (a zero, subnormal, inf or NaN operand, or an extreme
// ratio) takes the division as written.  Saves one or two f64 divisions per shadow test.
constexpr int kQNeg = 0, kQZero = 1, kQPos = 2, kQOther = 3;   // t < 0, t = +-0, 0<t<inf, inf/NaN
__device__ __forceinline__ int quot_class(double num, double den) {
  const unsigned hn = (unsigned)__double2hiint(num), hd = (unsigned)__double2hiint(den);
  const int en = (int)((hn >> 20) & 0x7ffu), ed = (int)((hd >> 20) & 0x7ffu);
  const int e = en - ed;
  if (en != 0 && en != 0x7ff && ed != 0 && ed != 0x7ff && e >= -148 && e <= 126)
    return ((hn ^ hd) >> 31) ? kQNeg : kQPos;
  const float t = (float)(num / den);
  if (t < 0.0f) return kQNeg;
  if (t == 0.0f) return kQZero;
  return t < __builtin_inff() ? kQPos : kQOther;
}

// hit_sphere as a shadow test: the first root unless it is negative (C/raycast.c:593-597)
__device__ __forceinline__ bool shadow_sphere(V3 O, V3 D, const rc_shape& s, RayK k) {
  V3 tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
  float b = 2.0f * dot(D, tv);
  float c = (float)((double)dot(tv, tv) - s.r2);
  float fac = k.a4 * c;
  float disc = (float)__builtin_fma((double)b, (double)b, -(double)fac);
  if (disc < 0.0f) return false;
  double sq = sqrt_ns((double)disc);
  int q = quot_class((double)(-b) - sq, k.den);
  if (q == kQNeg) q = quot_class((double)(-b) + sq, k.den);
  return q == kQPos;
}

// hit_quadric + the bounce rays' z rule as a shadow test.  The z rule (C/raycast.c:492-494)
// needs t itself when it can fire, i.e. for a positive t only if D.z < 0: then the chosen
// root's quotient is formed exactly as in hit_quadric.
__device__ __forceinline__ bool shadow_quadric(V3 O, V3 D, const rc_shape& q, int skip, bool x0,
                                               bool rej) {
  float aq, bq, cq;
  quad_abc(O, D, q, aq, bq, cq, x0);
  if (rej) return false;

  double num, den;
  int cls;
  if ((double)aq == 0.0) {
    num = -1.0 * (double)cq;
    den = (double)bq;
    cls = quot_class(num, den);
  } else {
    const float disc = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
    if ((double)disc < 0.0) return false;
    den = 2.0 * (double)aq;
    const double sq = sqrt_ns((double)disc);
    num = (double)(-bq) - sq;
    cls = quot_class(num, den);
    if (cls == kQNeg || cls == kQZero) {
      num = (double)(-bq) + sq;
      cls = quot_class(num, den);
    }
  }
  if (cls != kQPos) return false;
  if (skip != -1 && D.z < 0.0f) {
    const float t = tquot(num, den, RC_NRDIV ? recip_nr(den) : 0.0);   // a positive finite t (cls)
    if ((O.z + t * D.z) < O.z) return false;
  }
  return true;
}

// C/raycast.c:441-531 (shadow_test = true): is any shape hit with 0 < t < inf?  The first
// such shape is always accepted, so the loop may stop there.
__device__ __forceinline__ bool shadowed(const Scene& sc, V3 O, V3 D, int skip) {
#if RC_EXP_NOSHADOW   // timing attribution builds only (wrong images): no shadow rays
  return false;
#endif
  const RayK rk = ray_consts(D);
  const bool x0 = quad_x0(sc), rej = x0 && x0_reject(O, D);
  for (int k = 0; k < sc.n; ++k) {
    if (k == skip) continue;
    const rc_shape& s = sc.shapes[k];
    const int type = s.type;
    bool hit = false;
    if (type == RC_SHAPE_SPHERE) {
      hit = shadow_sphere(O, D, s, rk);
    } else if (type == RC_SHAPE_PLANE) {
      float t = 0.0f;
      hit = hit_plane(O, D, s, t) && __builtin_inff() > t && t > 0.0f;
    } else if (type == RC_SHAPE_QUADRIC) {
      hit = shadow_quadric(O, D, s, skip, x0, rej);
    }
    if (hit) return true;
  }
  return false;
}
// Hit point and normal of the accepted shape (C/raycast.c:461-523).
__device__ __forceinline__ void hit_frame(const Scene& sc, int idx, V3 O, V3 D, float t, V3& P,
                                          V3& N, int& zero_events) {
  P = v3(O.x + D.x * t, O.y + D.y * t, O.z + D.z * t);
  const rc_shape& s = sc.lshapes[idx];
  const int type = s.type;
  if (type == RC_SHAPE_SPHERE) {
    const float inv = s.inv_r;
    N = normalize(v3((P.x - s.p[0]) * inv, (P.y - s.p[1]) * inv, (P.z - s.p[2]) * inv),
                  zero_events);
  } else if (type == RC_SHAPE_PLANE) {
    N = v3(s.n[0], s.n[1], s.n[2]);
  } else {
    double n0 = 2.0 * s.A * (double)P.x;
    n0 = n0 + (double)(s.qd * P.y);
    n0 = n0 + (double)(s.qe * P.z);
    n0 = n0 + (double)s.qg;
    double n1 = 2.0 * s.B * (double)P.y;
    n1 = n1 + (double)(s.qd * P.x);
    n1 = n1 + (double)(s.qf * P.z);
    n1 = n1 + (double)s.qh;
    double n2 = 2.0 * s.C * (double)P.z;
    n2 = n2 + (double)(s.qe * P.x);
    n2 = n2 + (double)(s.qf * P.y);
    n2 = n2 + (double)s.qi;
    N = normalize(v3((float)n0, (float)n1, (float)n2), zero_events);
    if (dot(N, D) > 0.0f) N = v3(N.x * -1.0f, N.y * -1.0f, N.z * -1.0f);
  }
}

// calc_color (C/raycast.c:381-421) for shape `idx` (sc.n = the phantom shapes_list[-1]).
__device__ __forceinline__ V3 shade(const Scene& sc, int idx, V3 P, V3 N, V3 D, int& zero_events) {
#if RC_EXP_NOSHADE   // timing attribution builds only (wrong images): no shading at all
  return v3(0.0f, 0.0f, 0.0f);
#endif
  const rc_shape& o = sc.lshapes[idx];
  const float opacity = o.opacity;
  V3 out = v3(0.0f, 0.0f, 0.0f);
  if (!(opacity > 0.0f)) return out;
  const int skip = (idx == sc.n) ? -1 : idx;
  const rc_shade_pair* pr = sc.lpairs + (size_t)idx * sc.m;
  for (int l = 0; l < sc.m; ++l) {
    const rc_light& L = sc.lights[l];
    V3 ld = v3(L.pos[0] - P.x, L.pos[1] - P.y, L.pos[2] - P.z);
    const float dist = length(ld);
    // normalize(ld, zero_events) with its length taken from dist (the same operations)
    if (dist == 0.0f) zero_events++;
    else ld = div3(ld, dist);
    // radial attenuation C/raycast.c:666-669
    const float lin = L.r0 + L.r1 * dist;
    const float rad =
        (float)(1.0 / ((double)lin + (double)L.r2 * ((double)dist * (double)dist)));
    // angular attenuation C/raycast.c:679-696.  v = normalize(P - L.pos): P - L.pos is -ld
    // component for component (round-to-nearest is sign-symmetric), so v = -ld and
    // alpha = -dot(ld, dir) exactly.  A zero-length ld (P on the light) is +0 in every
    // component either way: then v = ld, and the reference counts a second zero event
    // (only when the light is not shadowed: it is counted below, after the shadow test).
    float ang = 1.0f;
    const bool z = dist == 0.0f;
    if (L.type == RC_LIGHT_SPOT) {
      const float a = dot(ld, v3(L.dir[0], L.dir[1], L.dir[2]));
      const float alpha = z ? a : -a;
      if (alpha < L.cos_theta) {
        ang = 0.0f;
      } else if (L.a0_kind == RC_A0_INT) {
        ang = (float)pown_dd((double)alpha, L.a0_int);
      } else {
        ang = (float)pow((double)alpha, (double)L.a0);   // parity unpinned
      }
    }
    const float th = dot(N, ld);
    // A light behind the surface (th <= 0) contributes ((0 + 0) * rad) * ang = +-0 when rad
    // and ang are finite, and out + (+-0) == out (out starts at +0 and a round-to-nearest
    // sum is -0 only if both terms are): the reference's shadow ray (C/raycast.c:401-402)
    // cannot change the colour then, so it is not traced.  P on a spot light (a counted
    // zero-normalize event after the shadow test) keeps the test.
    const bool inert = th <= 0.0f && __builtin_isfinite(rad) && __builtin_isfinite(ang) &&
                       !(z && L.type == RC_LIGHT_SPOT);
    if (inert) continue;
    if (shadowed(sc, P, ld, skip)) continue;
    if (L.type == RC_LIGHT_SPOT) zero_events += z ? 1 : 0;
    // diffuse C/raycast.c:708-720, specular C/raycast.c:733-758
    float dr = 0.0f, dg = 0.0f, db = 0.0f, sr = 0.0f, sg = 0.0f, sb = 0.0f;
    if (!(th <= 0.0f)) {   // C/raycast.c:713,740: a NaN theta is not <= 0
      const rc_shade_pair& p = pr[l];
      dr = p.dl[0] * th;
      dg = p.dl[1] * th;
      db = p.dl[2] * th;
      const V3 view = v3(D.x * -1.0f, D.y * -1.0f, D.z * -1.0f);
      const double angle = (double)dot(view, reflect(ld, N));
      if (!(angle > 0.0)) {
        const double p20 = pow20(angle);
        sr = (float)((double)p.sl[0] * p20);
        sg = (float)((double)p.sl[1] * p20);
        sb = (float)((double)p.sl[2] * p20);
      }
    }
    out.x = out.x + ((dr + sr) * rad) * ang;
    out.y = out.y + ((dg + sg) * rad) * ang;
    out.z = out.z + ((db + sb) * rad) * ang;
  }
  return v3(out.x * opacity, out.y * opacity, out.z * opacity);
}

// Primary ray of pixel (x, y) (C/raycast.c:115-118).
__device__ __forceinline__ V3 primary_dir(const Cam& cam, int x, int y, int& zero_events) {
  V3 d;
  d.x = (float)(cam.hx + (double)cam.pw * ((double)x + 0.5));
  d.y = (float)(cam.hy - (double)cam.ph * ((double)y + 0.5));
  d.z = -1.0f;
  return normalize(d, zero_events);
}

// ppm_clamp (C/ppm.c:350-359) + the float -> uint8_t store (C/raycast.c:122-126).
// v_cvt_i32_f32 truncates and maps NaN to 0, like x86 cvttss2si's low byte.
__device__ __forceinline__ uint8_t quant(float c) {
  float v = c * 255.0f;
  if (v > 255.0f) v = 255.0f;
  if (v < 0.0f) v = 0.0f;
  return (uint8_t)(int)v;
}

// State a first-bounce-miss (DEP) pixel carries from phase A to phases B/C.
// A DEP pixel's transfer-function inputs.  Neither bounce direction below depends on the
// carry, so phase A computes them once: `a` = level 2's direction normalize(reflect(d1, n0)),
// and `b` = level 3's direction if level 2 also misses, normalize(reflect(a, n0))
// (C/raycast.c:349-350 with the stale normal of a miss).  The record also holds the pixel's
// primary shade (Scene::dep_fast, C/raycast.c:377), so phase A writes each DEP pixel as ONE
// naturally aligned 64-byte line: the round-3 48-byte record plus a 16-byte shade slot beside
// it cost partial-line writes (k_phase_a WRITE_SIZE 1.24x its algorithmic bytes in flight).
// The resolver reads only the 48-byte record (its registers and LDS windows hold DepRec);
// phase C reads the line.
struct DepRec {
  float ax, ay, az;      // level-2 direction
  float n0x, n0y, n0z;   // primary normal (misses never update the normal)
  int obj0;              // primary shape (stale object of the loop, C/raycast.c:359-362)
  int pad;
  float bx, by, bz;      // level-3 direction when level 2 misses
  int pad2;
};
struct alignas(16) DepLine {   // 64-byte stride: pixel-indexed lines stay aligned
  DepRec r;
  float px, py, pz;      // primary shade (dep_fast; phase C's clean entries are exactly this)
  int pad3;
};
static_assert(sizeof(DepRec) == 48 && sizeof(DepLine) == 64, "one 64-byte line per DEP pixel");
__device__ __forceinline__ V3 dep_pcol(const DepLine* l) { return v3(l->px, l->py, l->pz); }

struct PixelOut {
  V3 rgb;
  uint8_t cls;
  V3 carry;     // carry-out for writers (last bounce-hit point)
  DepRec dep;   // DEP pixels
  V3 pcol;      // DEP pixels under dep_fast: the primary shade (C/raycast.c:377)
};

// iterative_shoot (C/raycast.c:315-379) for one pixel under MODE.
//  kModeFast     : miss ends the loop.
//  kModeParityA  : a miss at level 1 stops here (cls = DEP, dep record filled).
//  kModeParityC  : `carry` is this pixel's scan-order carry-in.
//  kModeClassify : kModeParityA's control flow and carry without any shading (rgb = 0).
// Under sc.dep_fast phase A also shades a DEP pixel's primary hit (po.pcol) and counts the
// events of everything it computed for it (phase C resumes at level 2: shade_dep_cont).
template <int MODE>
__device__ __forceinline__ void shoot(const Scene& sc, V3 d, int maxrec, V3 carry, PixelOut& po,
                                      int& zero_events) {
  po.rgb = v3(0.0f, 0.0f, 0.0f);
  po.cls = kClsIdent;
  int zp = 0;   // events of the primary part (a DEP pixel's share of phase A)
  float t0;
  const int i0 = nearest_primary(sc, d, t0);
  if (i0 < 0) return;                                   // C/raycast.c:328-331
  V3 P0, N0;
  hit_frame(sc, i0, v3(0.0f, 0.0f, 0.0f), d, t0, P0, N0, zp);
  // The primary hit's shade is added last (C/raycast.c:377-378) but depends on the primary hit
  // alone: shading it first is the same arithmetic, added in the same order at the end, and
  // P0 / N0 / d need not stay live through the bounce loop (register pressure: phase A spills).
  V3 prim = v3(0.0f, 0.0f, 0.0f);
  if (MODE != kModeClassify) prim = shade(sc, i0, P0, N0, d, zp);

  int obj = i0, S = i0;
  V3 O = P0, D = d, N = N0, C = carry;
  float T = sc.lshapes[i0].refl;
  V3 out = v3(0.0f, 0.0f, 0.0f);
  bool wrote = false;
  for (int lvl = 1; lvl < maxrec; ++lvl) {              // C/raycast.c:348-376
    if (!reflective(sc, obj)) break;
    int ze = 0;
    D = normalize(reflect(D, N), ze);
    if (lvl == 1) zp += ze;
    else zero_events += ze;
    float t;
    const int i = nearest(sc, O, D, S, t);
    if (i >= 0) {
      hit_frame(sc, i, O, D, t, C, N, zero_events);    // writes the carry
      obj = i;
      wrote = true;
    } else {
      if (MODE == kModeFast) break;                     // CUDA/raycast.cu:224-237
      if ((MODE == kModeParityA || MODE == kModeClassify) && lvl == 1) {
        po.cls = kClsDep;
        const V3 A = normalize_sel(reflect(D, N));
        const V3 B = normalize_sel(reflect(A, N));
        po.dep = DepRec{A.x, A.y, A.z, N.x, N.y, N.z, obj, 0, B.x, B.y, B.z, 0};
        if (MODE == kModeParityA && sc.dep_fast) po.pcol = prim;
        zero_events += zp;
        return;
      }
    }
    if (MODE != kModeClassify) {
      V3 col = shade(sc, i >= 0 ? i : sc.n, C, N, D, zero_events);
      out.x = out.x + col.x * T;
      out.y = out.y + col.y * T;
      out.z = out.z + col.z * T;
      T = T * sc.lshapes[obj].refl;
    }
    O = C;
    S = i;
  }
  if (MODE != kModeClassify)                            // C/raycast.c:377-378
    out = v3(out.x + prim.x, out.y + prim.y, out.z + prim.z);
  zero_events += zp;
  po.rgb = out;
  po.cls = wrote ? kClsWriter : kClsIdent;
  po.carry = C;
}

// Phase C of a DEP pixel under dep_fast, from its carry-in c: the bounce loop of
// iterative_shoot (C/raycast.c:348-376) resumed at level 2, then the primary shade phase A
// computed (the record's p*, C/raycast.c:377-378).  Level 1 missed: its shade is the black phantom's
// (exactly zero), O = C = c, S = -1, N = N0, obj = obj0, T = refl[obj0]^2, and level 2's
// direction normalize(reflect(D1, N0)) is the record's `a`.
// The primary shade is read from the record after the bounce loop, so it does not stay live
// through it (register pressure: phase C spills).
__device__ __forceinline__ V3 shade_dep_cont(const Scene& sc, const DepLine* __restrict__ rp,
                                             int maxrec, V3 c, int& zero_events) {
  const DepRec& r = rp->r;
  int obj = r.obj0, S = -1;
  const float T0 = sc.lshapes[obj].refl;
  float T = T0 * sc.lshapes[obj].refl;
  V3 O = c, C = c, D = v3(r.ax, r.ay, r.az), N = v3(r.n0x, r.n0y, r.n0z);
  V3 out = v3(0.0f, 0.0f, 0.0f);
  for (int lvl = 2; lvl < maxrec; ++lvl) {
    if (!reflective(sc, obj)) break;
    if (lvl > 2) D = normalize(reflect(D, N), zero_events);
    float t;
    const int i = nearest(sc, O, D, S, t);
    if (i >= 0) {
      hit_frame(sc, i, O, D, t, C, N, zero_events);
      obj = i;
    }
    const V3 col = shade(sc, i >= 0 ? i : sc.n, C, N, D, zero_events);
    out.x = out.x + col.x * T;
    out.y = out.y + col.y * T;
    out.z = out.z + col.z * T;
    T = T * sc.lshapes[obj].refl;
    O = C;
    S = i;
  }
  const V3 k = dep_pcol(rp);
  return v3(out.x + k.x, out.y + k.y, out.z + k.z);
}

// Carry-only continuation of a DEP pixel from carry-in c (levels 2..maxrec-1): the
// phase-B transfer function f_p(c).  No shading: only the bounce-hit points matter.
// `hit`: some level hit (the entry is not clean, see Scene::dep_fast).
__device__ __forceinline__ V3 carry_path(const Scene& sc, const DepRec& r, int maxrec, V3 c,
                                         int& zero_events, bool& hit) {
  V3 D = v3(r.ax, r.ay, r.az), N = v3(r.n0x, r.n0y, r.n0z), C = c;   // level 2's direction
  int obj = r.obj0, S = -1;
  hit = false;
  for (int lvl = 2; lvl < maxrec; ++lvl) {
    if (!reflective(sc, obj)) break;
    if (lvl > 2) D = normalize(reflect(D, N), zero_events);
    float t;
    const int i = nearest(sc, C, D, S, t);
    if (i >= 0) {
      V3 P;
      hit_frame(sc, i, C, D, t, P, N, zero_events);
      C = P;
      obj = i;
      hit = true;
    }
    S = i;
  }
  return C;
}

}  // namespace rc

namespace rc {

// ---------------------------------------------------------- cooperative evaluation --
// One entry's transfer function evaluated by a group of G lanes (G = power of two >= n):
// lane k of the group tests shape k, then the group takes the lexicographic minimum of
// (t, k) over the valid candidates.  That is exactly the reference's nearest object
// (C/raycast.c:449-528): the scan accepts strictly smaller t in file order, so the winner
// is the smallest valid t and, among equal t, the smallest index.  The latency of a level is
// one shape test (per type present) instead of n of them.
struct LaneShape {
  rc_shape s;
  bool has;
};

// Cross-lane moves inside 16-lane rows use DPP (a VALU modifier, a few cycles) instead of
// ds_bpermute (an LDS round trip, ~50 cycles): this argmin sits on the serial chain.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL,
                                                    0xF, 0xF, false));
}
constexpr int kDppXor1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int kDppXor2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int kDppHalfMirror = 0x141; // row_half_mirror: lane i <-> 7-i within 8 lanes
constexpr int kDppRor8 = 0x128;       // row_ror:8: the other 8-lane half of a 16-lane row

__device__ __forceinline__ void argmin_step(float& t, int& k, float t2, int k2) {
  if (t2 < t || (t2 == t && k2 < k)) {
    t = t2;
    k = k2;
  }
}

__device__ __forceinline__ int group_argmin(float& t, int k, int G) {
  if (G >= 2) argmin_step(t, k, dpp_f<kDppXor1>(t), dpp_i<kDppXor1>(k));
  if (G >= 4) argmin_step(t, k, dpp_f<kDppXor2>(t), dpp_i<kDppXor2>(k));
  // after the quad steps every lane of a quad holds the quad minimum, so mirroring the
  // 8-lane half pairs quad 0 with quad 1
  if (G >= 8) argmin_step(t, k, dpp_f<kDppHalfMirror>(t), dpp_i<kDppHalfMirror>(k));
  if (G >= 16) argmin_step(t, k, dpp_f<kDppRor8>(t), dpp_i<kDppRor8>(k));
  for (int off = 16; off < G; off <<= 1)
    argmin_step(t, k, __shfl_xor(t, off, 64), __shfl_xor(k, off, 64));
  return k;
}

// Branch-free form for candidates with t in (0, +inf] (misses carry t = +inf, k = kNone):
// positive floats order like their bit patterns, so the lexicographic (t, k) minimum is a
// u32 min over t's bits, then a u32 min over k among the lanes holding that t.  Each step is
// one DPP-fed v_min_u32 — no compare/select chains or exec-mask branches on the serial path.
template <int CTRL>
__device__ __forceinline__ unsigned dpp_min_u(unsigned v) {
  return __builtin_elementwise_min(v, (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF,
                                                                         false));
}
template <int GT>
__device__ __forceinline__ unsigned group_min_u(unsigned v, int Grt) {
  const int G = GT ? GT : Grt;
  if (G >= 2) v = dpp_min_u<kDppXor1>(v);
  if (G >= 4) v = dpp_min_u<kDppXor2>(v);
  if (G >= 8) v = dpp_min_u<kDppHalfMirror>(v);
  if (G >= 16) v = dpp_min_u<kDppRor8>(v);
  for (int off = 16; off < G; off <<= 1)
    v = __builtin_elementwise_min(v, (unsigned)__shfl_xor((int)v, off, 64));
  return v;
}
template <int GT>
__device__ __forceinline__ int group_argmin_pos(float& t, int k, int G) {
  const unsigned tb = group_min_u<GT>(__float_as_uint(t), G);
  const unsigned kb = group_min_u<GT>(__float_as_uint(t) == tb ? (unsigned)k : 0xffffffffu, G);
  t = __uint_as_float(tb);
  return (int)kb;
}

__device__ __forceinline__ V3 carry_path_coop(const Scene& sc, const LaneShape& ls, int kself,
                                              int G, const DepRec& r, int maxrec, V3 c,
                                              int& zero_events, bool& anyhit) {
  constexpr int kNone = 0x7fffffff;
  V3 D = v3(r.ax, r.ay, r.az), N = v3(r.n0x, r.n0y, r.n0z), C = c;   // level 2's direction
  int obj = r.obj0, S = -1;
  anyhit = false;
  for (int lvl = 2; lvl < maxrec; ++lvl) {
    if (!reflective(sc, obj)) break;
    if (lvl > 2) D = normalize(reflect(D, N), zero_events);
    const RayK rk = ray_consts(D);
    float t = __builtin_inff();
    int k = kNone;
    if (ls.has && kself != S) {
      float tt = 0.0f;
      if (test_shape(ls.s, C, D, rk, S, tt) && __builtin_inff() > tt && tt > 0.0f) {
        t = tt;
        k = kself;
      }
    }
    const int win = group_argmin(t, k, G);
    if (win != kNone) {
      V3 P;
      hit_frame(sc, win, C, D, t, P, N, zero_events);
      C = P;
      obj = win;
      S = win;
      anyhit = true;
    } else {
      S = -1;
    }
  }
  return C;
}

}  // namespace rc

namespace rc {

// Diagnostic build only (-DRC_STAMPS=1, `make stamps`): per-section cycle sums of the
// speculative evaluator, read by the resolver trace.  The shipped library has no stamps.
#if RC_STAMPS
struct Stamps {
  unsigned long long acc[4];
  unsigned long long last;
};
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define RC_STAMP_DECL Stamps* st_
#define RC_STAMP_ARG , st_
#if RC_STAMPS == 1   // per-section stamps inside the evaluator (2: coarse, per step only)
#define RC_STAMP(i)                                  \
  do {                                               \
    const unsigned long long n_ = stamp_now();       \
    st_->acc[i] += n_ - st_->last;                   \
    st_->last = n_;                                  \
  } while (0)
#else
#define RC_STAMP(i) \
  do {              \
  } while (0)
#endif
#else
#define RC_STAMP(i) \
  do {              \
  } while (0)
#endif

// ------------------------------------------------------ branch-free lane evaluation --
// The cooperative groups hold one shape per lane, so a wave holds every shape type at once
// and type-divergent code runs each type's branch (each with its own sqrt and divisions)
// one after the other, with nothing to overlap on a lone wave.  The forms below compute
// every type's prelude in straight-line code and share ONE f64 sqrt and two parallel f64
// divisions, selecting by type at the end; each value is produced by the same operations in
// the same order as hit_sphere / hit_plane / hit_quadric, so results are bit-identical.
// The plane's f32 quotient (-num)/den is taken as (float)((double)(-num) / (double)den):
// double rounding is innocuous for division when 53 >= 2*24 + 2.

// test_shape() for any type, branch-free.  kQuad = false: the scene has no quadric, so the
// quadric part is compiled out (every quadric term below is dead).
template <bool kQuad, bool kX0 = false>
__device__ __forceinline__ bool test_unified(const rc_shape& s, V3 O, V3 D, RayK rk, int skip,
                                             float& t) {
  const int type = s.type;
  const bool isS = type == RC_SHAPE_SPHERE, isP = type == RC_SHAPE_PLANE,
             isQ = kQuad && type == RC_SHAPE_QUADRIC;
  // origin-only parts (sphere c, plane num, quadric cq)
  const V3 tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
  const float cS = (float)((double)dot(tv, tv) - s.r2);
  const float numP = pin(dot(tv, v3(s.n[0], s.n[1], s.n[2])));
  // direction parts (sphere b and disc, plane den)
  const float bS = 2.0f * dot(D, tv);
  const float facS = rk.a4 * cS;
  const float discS = (float)__builtin_fma((double)bS, (double)bS, -(double)facS);
  const float denP = dot(D, v3(s.n[0], s.n[1], s.n[2]));
  float cq = 0.0f, aq = 0.0f, bq = 0.0f, discQ = 0.0f;
  bool lin = false;
  if constexpr (kQuad && kX0) {
    quad_abc(O, D, s, aq, bq, cq, true);   // no cross terms (quad_x0)
  } else if constexpr (kQuad) {
    // written out in this order (c, a, b): the lone resolver wave's schedule is sensitive to
    // it (the same terms through quad_abc's a, b, c order: lone resolver 4.22 -> 4.44 ms)
    double acc;
    acc = s.A * ((double)O.x * (double)O.x);
    acc = acc + s.B * ((double)O.y * (double)O.y);
    acc = acc + s.C * ((double)O.z * (double)O.z);
    acc = acc + (double)(s.qd * O.x * O.y);
    acc = acc + (double)(s.qe * O.x * O.z);
    acc = acc + (double)(s.qf * O.y * O.z);
    acc = acc + (double)(s.qg * O.x);
    acc = acc + (double)(s.qh * O.y);
    acc = acc + (double)(s.qi * O.z);
    acc = acc + (double)s.qj;
    cq = (float)acc;
    acc = s.A * ((double)D.x * (double)D.x);
    acc = acc + s.B * ((double)D.y * (double)D.y);
    acc = acc + s.C * ((double)D.z * (double)D.z);
    acc = acc + (double)(s.qd * D.x * D.y);
    acc = acc + (double)(s.qe * D.x * D.z);
    acc = acc + (double)(s.qf * D.y * D.z);
    aq = (float)acc;
    acc = 2.0 * s.A * (double)O.x * (double)D.x;
    acc = acc + 2.0 * s.B * (double)O.y * (double)D.y;
    acc = acc + 2.0 * s.C * (double)O.z * (double)D.z;
    acc = acc + (double)(s.qd * (O.x * D.y + O.y * D.x));
    acc = acc + (double)(s.qe * (O.x * D.z + O.z * D.x));
    acc = acc + (double)(s.qf * (O.y * D.z + O.z * D.y));
    acc = acc + (double)(s.qg * D.x);
    acc = acc + (double)(s.qh * D.y);
    acc = acc + (double)(s.qi * D.z);
    bq = (float)acc;
  }
  if constexpr (kQuad) {
    discQ = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
    lin = (double)aq == 0.0;
  }
  // shared tail: one sqrt, two quotients
  const float B = kQuad ? (isS ? bS : bq) : bS;
  const float disc = kQuad ? (isS ? discS : discQ) : discS;
  const double sq = pin(sqrt_ns((double)disc));
  const double nb = (double)(-B);
  const bool qlin = isQ & lin;
  const double n1q = pin(nb - sq), n1p = pin((double)(-numP));
  const double n1l = kQuad ? pin(-1.0 * (double)cq) : 0.0;
  const double num1 = isP ? n1p : (qlin ? n1l : n1q);
  const double den1 =
      isP ? (double)denP : (qlin ? (double)bq : ((isS || !kQuad) ? rk.den : 2.0 * (double)aq));
  const double num2 = nb + sq;
#if RC_NRDIV
  const double y1 = recip_nr(den1);
  const float q1 = (float)pin(div_nr(num1, den1, y1));
  const float q2 = (float)pin(div_nr(num2, den1, y1));
#else
  const float q1 = (float)pin(num1 / den1);
  const float q2 = (float)pin(num2 / den1);
#endif
  // sphere: second root if the first is negative; quadric: if it is not positive
  const bool second = (isS & (q1 < 0.0f)) | (isQ & !lin & (q1 <= 0.0f));
  const float tt = second ? q2 : q1;
  const bool okS = isS & !(disc < 0.0f);
  const bool okP = isP & (denP != 0.0f) & !(q1 < 0.0f);
  const bool okQ = isQ & (lin | !((double)disc < 0.0));
  // C/raycast.c:492-494: a bounce ray ignores quadric hits below its origin's z
  const bool below = isQ & (skip != -1) & ((O.z + tt * D.z) < O.z);
  const bool ok = (okS | okP | okQ) & !below;
  t = tt;
  return ok;
}

// hit_frame() without type branches; `s` is the winner's record.  kQuad as in test_unified.
template <bool kQuad>
__device__ __forceinline__ void hit_frame_sel(const rc_shape& s, V3 O, V3 D, float t, V3& P,
                                              V3& N) {
  P = v3(O.x + D.x * t, O.y + D.y * t, O.z + D.z * t);
  const int type = s.type;
  const float inv = s.inv_r;
  const V3 vs = v3((P.x - s.p[0]) * inv, (P.y - s.p[1]) * inv, (P.z - s.p[2]) * inv);
  const bool isS = type == RC_SHAPE_SPHERE, isP = type == RC_SHAPE_PLANE;
  V3 v = vs;
  if constexpr (kQuad) {
    double n0 = 2.0 * s.A * (double)P.x;
    n0 = n0 + (double)(s.qd * P.y);
    n0 = n0 + (double)(s.qe * P.z);
    n0 = n0 + (double)s.qg;
    double n1 = 2.0 * s.B * (double)P.y;
    n1 = n1 + (double)(s.qd * P.x);
    n1 = n1 + (double)(s.qf * P.z);
    n1 = n1 + (double)s.qh;
    double n2 = 2.0 * s.C * (double)P.z;
    n2 = n2 + (double)(s.qe * P.x);
    n2 = n2 + (double)(s.qf * P.y);
    n2 = n2 + (double)s.qi;
    v = sel(isS, vs, v3((float)n0, (float)n1, (float)n2));
  }
  V3 n = normalize_sel(v);
  // quadric normals face the ray (a plane's own normal is taken below, unflipped)
  if constexpr (kQuad) n = sel(!isS && dot(n, D) > 0.0f, v3(n.x * -1.0f, n.y * -1.0f, n.z * -1.0f), n);
  N = sel(isP, v3(s.n[0], s.n[1], s.n[2]), n);
}

// Cooperative evaluation with level speculation: the 2G lanes of one entry form two
// groups.  Group h=0 evaluates bounce level L; group h=1 evaluates level L+1 assuming level
// L misses — then its ray is fully known in advance: same origin C, direction
// normalize(reflect(D_L, N)), skip -1, and the object test refl[obj] > 0 unchanged
// (C/raycast.c:349-367 with the stale object/normal of a miss).  If level L misses, both
// levels retire in one step.  The carry creep of dense segments alternates hit/miss, so
// five levels retire in three steps.  Each step is one basic block (selects, no branches)
// so the scheduler can overlap the independent chains of a lone wave.  GT = the group size
// as a compile-time constant (4, 8, 16), or 0 for the runtime value Grt; kQ = 0: the scene has
// no quadric, 1: it has, 2: none of its quadrics has cross terms (quad_x0, quad_abc).
#ifndef RC_LAST_SKIP
#define RC_LAST_SKIP 0   // measured: lone resolver 4.21 -> 4.37 ms (the branch splits the step)
#endif
template <int GT, int kQ>
__device__ __forceinline__ V3 carry_path_spec(const Scene& sc, const LaneShape& ls, int kself,
                                              int Grt, int half, const DepRec& r, int maxrec,
                                              V3 c, int& zero_events, bool& anyhit
#if RC_STAMPS
                                              , Stamps* st_
#endif
) {
  (void)zero_events;
  constexpr bool kQuad = kQ != 0;
  anyhit = false;
  const int G = GT ? GT : Grt;
  constexpr int kNone = 0x7fffffff;
  V3 N = v3(r.n0x, r.n0y, r.n0z), C = c;
  // the first step's two directions come with the record; each later step's are computed
  // at the end of the step before it
  V3 D1 = v3(r.ax, r.ay, r.az), D2 = v3(r.bx, r.by, r.bz);
  int obj = r.obj0, S = -1;
  const int lane = threadIdx.x & 63;
  const int lead0 = lane & ~(2 * G - 1);   // group h=0 leader of this entry
  const int lead1 = lead0 + G;             // group h=1 leader
  int lvl = 2;
  while (lvl < maxrec) {
    if (!reflective(sc, obj)) break;
#if RC_STAMPS == 1
    st_->last = stamp_now();   // acc[0] is the wave's LANE passes (wave_window)
#endif
    const V3 myD = sel(half, D2, D1);
    const int myS = half ? -1 : S;
    const RayK rk = ray_consts(myD);
    float tt = 0.0f;
    // kQ = 2: quadrics without cross terms, rejected where a cross term would be NaN
    // (quad_abc, x0_reject)
    // (bitwise, not short-circuit: a branch here would split the step's basic block)
    bool rejq = false;
    if constexpr (kQ == 2) rejq = (ls.s.type == RC_SHAPE_QUADRIC) & x0_reject(C, myD);
    const bool tok = test_unified<kQuad, kQ == 2>(ls.s, C, myD, rk, myS, tt) & !rejq;
    const bool ok = tok && ls.has && kself != myS && __builtin_inff() > tt && tt > 0.0f;
    float t = ok ? tt : __builtin_inff();
    int k = ok ? kself : kNone;
    RC_STAMP(1);
    k = group_argmin_pos<GT>(t, k, G);
    int ko;
    float to;
    if (GT == 8) {          // the two halves are the 8-lane halves of one 16-lane row
      ko = dpp_i<kDppRor8>(k);
      to = dpp_f<kDppRor8>(t);
    } else if (GT == 4) {   // the two quads of an 8-lane half (each quad holds its minimum)
      ko = dpp_i<kDppHalfMirror>(k);
      to = dpp_f<kDppHalfMirror>(t);
    } else {
      ko = __shfl(k, half ? lead0 : lead1, 64);
      to = __shfl(t, half ? lead0 : lead1, 64);
    }
    const int w0 = half ? ko : k, w1 = half ? k : ko;
    const float t0 = half ? to : t, t1 = half ? t : to;
    RC_STAMP(2);
    // level L hits: retire L.  Level L misses and L+1 exists: retire both (L+1 may miss).
    const bool hitL = w0 != kNone;
    const bool two = !hitL && lvl + 1 < maxrec;
    const int w = hitL ? w0 : (two ? w1 : kNone);
    const float tw = hitL ? t0 : t1;
    const V3 Dw = sel(two, D2, D1);
    const bool hit = w != kNone;
    anyhit = anyhit | hit;
#if RC_LAST_SKIP
    // Every path of the wave ends at this level (the last level, or a non-reflective object):
    // the carry is the hit point alone, so the normal and its normalisation are skipped (a
    // wave-uniform branch; a changer's last level costs ~75 instructions less).
    {
      const int lnext = lvl + (two ? 2 : 1);
      const bool last = lnext >= maxrec || !reflective(sc, hit ? w : obj);
      if (__ballot(!last) == 0) {
        C = sel(hit, v3(C.x + Dw.x * tw, C.y + Dw.y * tw, C.z + Dw.z * tw), C);
        break;
      }
    }
#endif
    V3 P, Nw;
    hit_frame_sel<kQuad>(sc.lshapes[hit ? w : 0], C, Dw, tw, P, Nw);   // divergent: LDS copy
    C = sel(hit, P, C);
    N = sel(hit, Nw, N);
    obj = hit ? w : obj;
    S = hit ? w : -1;
    lvl += two ? 2 : 1;
    if (lvl >= maxrec || !reflective(sc, obj)) break;
    RC_STAMP(3);
    D1 = normalize_sel(reflect(Dw, N));
    D2 = normalize_sel(reflect(D1, N));
  }
  return C;
}

}  // namespace rc
