// rc_cudasem.hpp — the CUDA port's per-pixel semantics (RC_MODE_CUDA).
//
// CUDA/raycast.cu renders every pixel independently: a reflection miss ends the bounce loop
// (CUDA/raycast.cu:224-237), the loop runs up to MAX_ITER = 50 bounces (:13) and the
// arithmetic calls powf on floats where the C port calls pow on doubles
// (CUDA/raycast.cu:462-528,545,572,632-634, CUDA/v3math.cu:168).  The routines below restate
// that arithmetic under the contract of oracle/rc_oracle_cuda.c: every operation as written,
// C promotion rules, no contraction, powf correctly rounded (powf(x,2) = x*x, powf(x,0.5) =
// the correctly rounded sqrtf, powf(a,20) and integer spot exponents = the float of the exact
// double power).  Parity against the CUDA binary itself is unpinned (no nvcc here; its default
// --fmad=true contracts where it chooses) — DESIGN.md §8.
//
// Same CDNA4 structure as the parity/fast kernels (rc_device.hpp): one lane per pixel, the
// shape loop wave-uniform over scalar-loaded records; the C-port helpers that are identical in
// the CUDA port (dot, reflect, plane test, quadric b, hit normals' double sums, the uint8
// store) are shared.
#pragma once

#include "rc_device.hpp"

namespace rc {
namespace cusem {

// powf(x, 0.5) for x a float: sqrt in double rounded to float is the correctly rounded sqrtf
// (53 >= 2*24 + 2); x here is a sum of float squares or a discriminant >= 0.
__device__ __forceinline__ float sqrtf_cr(float x) { return (float)sqrt_ns((double)x); }

// CUDA/v3math.cu:167-170 — powf(powf(a0,2)+powf(a1,2)+powf(a2,2), 0.5) in float
__device__ __forceinline__ float cu_length(V3 a) {
  float s = a.x * a.x;
  s = s + a.y * a.y;
  s = s + a.z * a.z;
  return sqrtf_cr(s);
}

// CUDA/v3math.cu:172-185 — no zero-length guard: a zero length gives IEEE inf/NaN quotients
// (div3 is the IEEE f32 quotient for every finite non-zero len, rc_device.hpp)
__device__ __forceinline__ V3 cu_normalize(V3 a) {
  const float len = cu_length(a);
  if (len == 0.0f || !__builtin_isfinite(len)) return v3(a.x / len, a.y / len, a.z / len);
  return div3(a, len);
}

// CUDA/raycast.cu:455-477
__device__ __forceinline__ bool cu_sphere(V3 O, V3 D, const rc_shape& s, float a, float& t) {
  const V3 tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
  const float b = 2.0f * dot(D, tv);
  const float c = dot(tv, tv) - s.r * s.r;
  const float disc = b * b - (4.0f * a) * c;
  if (disc < 0.0f) return false;
  const double den = 2.0 * (double)a;
  const float sq = sqrtf_cr(disc);
  float tt = (float)((double)(-b - sq) / den);
  if (tt < 0.0f) tt = (float)((double)(-b + sq) / den);
  t = tt;
  return true;
}

// CUDA/raycast.cu:491-532 — a_q and c_q in float, b_q in double (as in the C port)
__device__ __forceinline__ bool cu_quadric(V3 O, V3 D, const rc_shape& q, float& t) {
  float aq = q.qa * (D.x * D.x);
  aq = aq + q.qb * (D.y * D.y);
  aq = aq + q.qc * (D.z * D.z);
  aq = aq + q.qd * D.x * D.y;
  aq = aq + q.qe * D.x * D.z;
  aq = aq + q.qf * D.y * D.z;

  double acc = 2.0 * q.A * (double)O.x * (double)D.x;
  acc = acc + 2.0 * q.B * (double)O.y * (double)D.y;
  acc = acc + 2.0 * q.C * (double)O.z * (double)D.z;
  acc = acc + (double)(q.qd * (O.x * D.y + O.y * D.x));
  acc = acc + (double)(q.qe * (O.x * D.z + O.z * D.x));
  acc = acc + (double)(q.qf * (O.y * D.z + O.z * D.y));
  acc = acc + (double)(q.qg * D.x);
  acc = acc + (double)(q.qh * D.y);
  acc = acc + (double)(q.qi * D.z);
  const float bq = (float)acc;

  float cq = q.qa * (O.x * O.x);
  cq = cq + q.qb * (O.y * O.y);
  cq = cq + q.qc * (O.z * O.z);
  cq = cq + q.qd * O.x * O.y;
  cq = cq + q.qe * O.x * O.z;
  cq = cq + q.qf * O.y * O.z;
  cq = cq + q.qg * O.x;
  cq = cq + q.qh * O.y;
  cq = cq + q.qi * O.z;
  cq = cq + q.qj;

  if ((double)aq == 0.0) {                                    // :517-519
    t = (float)((-1.0 * (double)cq) / (double)bq);
    return true;
  }
  const float disc = (float)((double)(bq * bq) - 4.0 * (double)aq * (double)cq);
  if ((double)disc < 0.0) return false;
  const double den = 2.0 * (double)aq;
  const float sq = sqrtf_cr(disc);
  float tt = (float)((double)(-bq - sq) / den);
  if (tt <= 0.0f) tt = (float)((double)(-bq + sq) / den);
  t = tt;
  return true;
}

__device__ __forceinline__ bool cu_test(const rc_shape& s, V3 O, V3 D, float a, int skip,
                                           float& t) {
  const int type = s.type;
  if (type == RC_SHAPE_SPHERE) return cu_sphere(O, D, s, a, t);
  if (type == RC_SHAPE_PLANE) return hit_plane(O, D, s, t);
  if (type == RC_SHAPE_QUADRIC) {
    if (!cu_quadric(O, D, s, t)) return false;
    if (skip != -1 && (O.z + t * D.z) < O.z) return false;   // CUDA/raycast.cu:388-390
    return true;
  }
  return false;
}

// the sphere test's a = d0*d0 + d1*d1 + d2*d2 (float) depends on the ray only
__device__ __forceinline__ float ray_a(V3 D) {
  float a = D.x * D.x;
  a = a + D.y * D.y;
  return a + D.z * D.z;
}

// CUDA/raycast.cu:330-430 (shadow_test = false): nearest accepted shape and its t
__device__ __forceinline__ int cu_nearest(const Scene& sc, V3 O, V3 D, int skip, float& tbest) {
  const float a = ray_a(D);
  float best = __builtin_inff();
  int idx = -1;
  for (int k = 0; k < sc.n; ++k) {
    float t = 0.0f;
    const bool hit = k != skip && cu_test(sc.shapes[k], O, D, a, skip, t);
    if (hit && best > t && t > 0.0f) {
      best = t;
      idx = k;
    }
  }
  tbest = best;
  return idx;
}

// shadow_test = true: any shape with 0 < t < inf
__device__ __forceinline__ bool cu_shadowed(const Scene& sc, V3 O, V3 D, int skip) {
  const float a = ray_a(D);
  for (int k = 0; k < sc.n; ++k) {
    float t = 0.0f;
    const bool hit = k != skip && cu_test(sc.shapes[k], O, D, a, skip, t);
    if (hit && __builtin_inff() > t && t > 0.0f) return true;
  }
  return false;
}

// hit point and normal of the accepted shape (CUDA/raycast.cu:351-424)
__device__ __forceinline__ void cu_hit_frame(const Scene& sc, int idx, V3 O, V3 D, float t, V3& P,
                                          V3& N) {
  P = v3(O.x + D.x * t, O.y + D.y * t, O.z + D.z * t);
  const rc_shape& s = sc.lshapes[idx];
  const int type = s.type;
  if (type == RC_SHAPE_SPHERE) {
    const float inv = s.inv_r;
    N = cu_normalize(v3((P.x - s.p[0]) * inv, (P.y - s.p[1]) * inv, (P.z - s.p[2]) * inv));
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
    N = cu_normalize(v3((float)n0, (float)n1, (float)n2));
    if (dot(N, D) > 0.0f) N = v3(N.x * -1.0f, N.y * -1.0f, N.z * -1.0f);
  }
}

// calc_color (CUDA/raycast.cu:260-302) with radial/angular attenuation and the light terms
// of :544-634
__device__ __forceinline__ V3 cu_shade(const Scene& sc, int idx, V3 P, V3 N, V3 D) {
  const rc_shape& o = sc.lshapes[idx];
  V3 out = v3(0.0f, 0.0f, 0.0f);
  if (!(o.opacity > 0.0f)) return out;
  const rc_shade_pair* pr = sc.lpairs + (size_t)idx * sc.m;
  for (int l = 0; l < sc.m; ++l) {
    const rc_light& L = sc.lights[l];
    V3 ld = v3(L.pos[0] - P.x, L.pos[1] - P.y, L.pos[2] - P.z);
    const float dist = cu_length(ld);
    ld = cu_normalize(ld);
    const float th = dot(N, ld);
    // the shadow ray decides whether the light counts at all (:276-279); a light behind the
    // surface adds ((0 + 0) * rad) * ang = +-0 when rad and ang are finite, which leaves the
    // colour unchanged, so that ray is not traced (the same argument as rc_device.hpp shade)
    float den = L.r0 + L.r1 * dist;
    den = den + L.r2 * (dist * dist);
    const float rad = (float)(1.0 / (double)den);             // :544-546
    float ang = 1.0f;
    if (L.type == RC_LIGHT_SPOT) {                            // :556-573
      const V3 v = cu_normalize(v3(P.x - L.pos[0], P.y - L.pos[1], P.z - L.pos[2]));
      const float alpha = dot(v, v3(L.dir[0], L.dir[1], L.dir[2]));
      if (alpha < L.cos_theta) ang = 0.0f;
      else if (L.a0_kind == RC_A0_INT) ang = (float)pown_dd((double)alpha, L.a0_int);
      else ang = (float)pow((double)alpha, (double)L.a0);
    }
    const bool inert = th <= 0.0f && __builtin_isfinite(rad) && __builtin_isfinite(ang);
    if (inert) continue;
    if (cu_shadowed(sc, P, ld, idx)) continue;
    float dr = 0.0f, dg = 0.0f, db = 0.0f, sr = 0.0f, sg = 0.0f, sb = 0.0f;
    if (!(th <= 0.0f)) {
      const rc_shade_pair& p = pr[l];
      dr = p.dl[0] * th;
      dg = p.dl[1] * th;
      db = p.dl[2] * th;
      const V3 view = v3(D.x * -1.0f, D.y * -1.0f, D.z * -1.0f);
      const double angle = (double)dot(view, reflect(ld, N));
      if (!(angle > 0.0)) {                                   // :632-634: powf(float, 20)
        const float p20 = (float)pow20(angle);
        sr = p.sl[0] * p20;
        sg = p.sl[1] * p20;
        sb = p.sl[2] * p20;
      }
    }
    out.x = out.x + ((dr + sr) * rad) * ang;
    out.y = out.y + ((dg + sg) * rad) * ang;
    out.z = out.z + ((db + sb) * rad) * ang;
  }
  return v3(out.x * o.opacity, out.y * o.opacity, out.z * o.opacity);
}

// raytrace_engine's primary ray (CUDA/raycast.cu:154-158) + iterative_shoot (:183-246)
__device__ __forceinline__ V3 render_pixel(const Scene& sc, const Cam& cam, int x, int y,
                                           int max_iter) {
  V3 d;
  d.x = (float)(cam.hx + (double)cam.pw * ((double)x + 0.5));
  d.y = (float)(cam.hy - (double)cam.ph * ((double)y + 0.5));
  d.z = -1.0f;
  d = cu_normalize(d);
  float t0;
  const int i0 = cu_nearest(sc, v3(0.0f, 0.0f, 0.0f), d, -1, t0);
  if (i0 < 0) return v3(0.0f, 0.0f, 0.0f);
  V3 P0, N0;
  cu_hit_frame(sc, i0, v3(0.0f, 0.0f, 0.0f), d, t0, P0, N0);
  // the primary hit's shade is added last (:244-245); computed first, same arithmetic
  const V3 prim = cu_shade(sc, i0, P0, N0, d);
  int obj = i0, S = i0;
  V3 O = P0, D = d, N = N0;
  float T = sc.lshapes[i0].refl;
  V3 out = v3(0.0f, 0.0f, 0.0f);
  for (int it = 0; it < max_iter; ++it) {
    if (!reflective(sc, obj)) break;
    D = cu_normalize(reflect(D, N));
    float t;
    const int i = cu_nearest(sc, O, D, S, t);
    if (i < 0) break;                                          // :236-238
    V3 P;
    cu_hit_frame(sc, i, O, D, t, P, N);
    obj = i;
    const V3 col = cu_shade(sc, i, P, N, D);
    out.x = out.x + col.x * T;
    out.y = out.y + col.y * T;
    out.z = out.z + col.z * T;
    T = T * sc.lshapes[obj].refl;
    O = P;
    S = i;
  }
  return v3(out.x + prim.x, out.y + prim.y, out.z + prim.z);
}

}  // namespace cusem
}  // namespace rc
