// spec_exp.hpp — measurement tooling: experimental forms of rc_device.hpp carry_path_spec for
// scripts/step_bench.hip (each checked there bit for bit against the oracle's carries before it
// is timed).  A form that wins moves into rc_device.hpp.
//   VAR 1: every lane computes the hit frame of its OWN shape (its record is in registers) while
//          the group's argmin runs; the winner's point and normal are then taken from the winner
//          lane by an OR over the entry's lanes (DPP).  The argmin and the LDS read of the
//          winner's record leave the serial chain.
#pragma once
#include "rc_device.hpp"

namespace rc {

template <int CTRL>
__device__ __forceinline__ unsigned dpp_or_u(unsigned v) {
  return v | (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
// OR over the 2*GT lanes of an entry (GT = 4: 8 lanes, 8: 16 lanes)
template <int GT>
__device__ __forceinline__ unsigned entry_or(unsigned v) {
  v = dpp_or_u<kDppXor1>(v);
  v = dpp_or_u<kDppXor2>(v);
  v = dpp_or_u<kDppHalfMirror>(v);
  if (GT >= 8) v = dpp_or_u<kDppRor8>(v);
  return v;
}

// VAR bit 1: the origin-only terms of the next step's test (sphere c, plane numerator,
// quadric c: they depend on the new origin alone) are computed as soon as the origin is known,
// beside the two reflections, instead of at the top of the next step.
struct OTerms {
  V3 tv;
  float cS, numP, cq;
};
template <bool kQuad>
__device__ __forceinline__ OTerms origin_terms(const rc_shape& s, V3 O) {
  OTerms o;
  o.tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
  o.cS = (float)((double)dot(o.tv, o.tv) - s.r2);
  o.numP = pin(dot(o.tv, v3(s.n[0], s.n[1], s.n[2])));
  o.cq = 0.0f;
  if constexpr (kQuad) {
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
    o.cq = (float)acc;
  }
  return o;
}
// test_unified (kX0 = false) with the origin terms given
template <bool kQuad>
__device__ __forceinline__ bool test_dir(const rc_shape& s, const OTerms& ot, V3 O, V3 D, RayK rk,
                                         int skip, float& t) {
  const int type = s.type;
  const bool isS = type == RC_SHAPE_SPHERE, isP = type == RC_SHAPE_PLANE,
             isQ = kQuad && type == RC_SHAPE_QUADRIC;
  const V3 tv = ot.tv;
  const float cS = ot.cS, numP = ot.numP, cq = ot.cq;
  const float bS = 2.0f * dot(D, tv);
  const float facS = rk.a4 * cS;
  const float discS = (float)__builtin_fma((double)bS, (double)bS, -(double)facS);
  const float denP = dot(D, v3(s.n[0], s.n[1], s.n[2]));
  float aq = 0.0f, bq = 0.0f, discQ = 0.0f;
  bool lin = false;
  if constexpr (kQuad) {
    double acc;
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
    discQ = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
    lin = (double)aq == 0.0;
  }
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
  const double y1 = recip_nr(den1);
  const float q1 = (float)pin(div_nr(num1, den1, y1));
  const float q2 = (float)pin(div_nr(num2, den1, y1));
  const bool second = (isS & (q1 < 0.0f)) | (isQ & !lin & (q1 <= 0.0f));
  const float tt = second ? q2 : q1;
  const bool okS = isS & !(disc < 0.0f);
  const bool okP = isP & (denP != 0.0f) & !(q1 < 0.0f);
  const bool okQ = isQ & (lin | !((double)disc < 0.0));
  const bool below = isQ & (skip != -1) & ((O.z + tt * D.z) < O.z);
  const bool ok = (okS | okP | okQ) & !below;
  t = tt;
  return ok;
}

template <int GT, int kQ, int VAR>
__device__ __forceinline__ V3 carry_path_x(const Scene& sc, const LaneShape& ls, int kself,
                                           int Grt, int half, const DepRec& r, int maxrec, V3 c,
                                           int& zero_events, bool& anyhit) {
  (void)zero_events;
  static_assert(GT == 4 || GT == 8, "DPP entry OR");
  constexpr bool kQuad = kQ != 0;
  anyhit = false;
  constexpr int G = GT;
  (void)Grt;
  constexpr int kNone = 0x7fffffff;
  V3 N = v3(r.n0x, r.n0y, r.n0z), C = c;
  V3 D1 = v3(r.ax, r.ay, r.az), D2 = v3(r.bx, r.by, r.bz);
  int obj = r.obj0, S = -1;
  int lvl = 2;
  constexpr bool kOwn = (VAR & 1) != 0, kPipe = (VAR & 2) != 0;
  static_assert(!kPipe || kQ != 2, "origin pipelining: the full quadric form only");
  OTerms ot{};
  if constexpr (kPipe) ot = origin_terms<kQuad>(ls.s, C);
  while (lvl < maxrec) {
    if (!reflective(sc, obj)) break;
    const V3 myD = sel(half, D2, D1);
    const int myS = half ? -1 : S;
    const RayK rk = ray_consts(myD);
    float tt = 0.0f;
    bool rejq = false;
    if constexpr (kQ == 2) rejq = (ls.s.type == RC_SHAPE_QUADRIC) & x0_reject(C, myD);
    bool tok;
    if constexpr (kPipe) tok = test_dir<kQuad>(ls.s, ot, C, myD, rk, myS, tt);
    else tok = test_unified<kQuad, kQ == 2>(ls.s, C, myD, rk, myS, tt) & !rejq;
    const bool ok = tok && ls.has && kself != myS && __builtin_inff() > tt && tt > 0.0f;
    // this lane's own shape, as if it won (discarded unless it does)
    V3 Pm, Nm;
    if constexpr (kOwn) hit_frame_sel<kQuad>(ls.s, C, myD, tt, Pm, Nm);
    float t = ok ? tt : __builtin_inff();
    int k = ok ? kself : kNone;
    k = group_argmin_pos<GT>(t, k, G);
    int ko;
    float to;
    if (GT == 8) {
      ko = dpp_i<kDppRor8>(k);
      to = dpp_f<kDppRor8>(t);
    } else {
      ko = dpp_i<kDppHalfMirror>(k);
      to = dpp_f<kDppHalfMirror>(t);
    }
    const int w0 = half ? ko : k, w1 = half ? k : ko;
    const float t0 = half ? to : t, t1 = half ? t : to;
    const bool hitL = w0 != kNone;
    const bool two = !hitL && lvl + 1 < maxrec;
    const int w = hitL ? w0 : (two ? w1 : kNone);
    const V3 Dw = sel(two, D2, D1);
    const bool hit = w != kNone;
    anyhit = anyhit | hit;
    V3 P, Nw;
    if constexpr (kOwn) {
      const bool mine = hit && (half == (hitL ? 0 : 1)) && kself == w;
      P = v3(__uint_as_float(entry_or<GT>(mine ? __float_as_uint(Pm.x) : 0u)),
             __uint_as_float(entry_or<GT>(mine ? __float_as_uint(Pm.y) : 0u)),
             __uint_as_float(entry_or<GT>(mine ? __float_as_uint(Pm.z) : 0u)));
      Nw = v3(__uint_as_float(entry_or<GT>(mine ? __float_as_uint(Nm.x) : 0u)),
              __uint_as_float(entry_or<GT>(mine ? __float_as_uint(Nm.y) : 0u)),
              __uint_as_float(entry_or<GT>(mine ? __float_as_uint(Nm.z) : 0u)));
    } else if constexpr ((VAR & 8) != 0) {   // knock-out: the hit point only, N unchanged
      const float tw = hitL ? t0 : t1;
      P = v3(C.x + Dw.x * tw, C.y + Dw.y * tw, C.z + Dw.z * tw);
      Nw = N;
    } else {
      const float tw = hitL ? t0 : t1;
      hit_frame_sel<kQuad>(sc.lshapes[hit ? w : 0], C, Dw, tw, P, Nw);
    }
    C = sel(hit, P, C);
    N = sel(hit, Nw, N);
    obj = hit ? w : obj;
    S = hit ? w : -1;
    lvl += two ? 2 : 1;
    if (lvl >= maxrec || !reflective(sc, obj)) break;
    if constexpr (kPipe) ot = origin_terms<kQuad>(ls.s, C);
    D1 = normalize_sel(reflect(Dw, N));
    // knock-out builds (timing attribution only: wrong carries): bit 4 drops D2's chain
    if constexpr ((VAR & 4) != 0) D2 = D1;
    else D2 = normalize_sel(reflect(D1, N));
  }
  return C;
}

}  // namespace rc
