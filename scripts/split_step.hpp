// split_step.hpp — measurement tooling (not the product): the team leader's cooperative
// block step split by shape class across the workgroup's waves, for
// scripts/block_bench.hip variant 2.  Bit-exact against the oracle's carry-ins, and measured
// slower than the product's unified step (profiles/r06_evaluator_experiments.txt): the
// quadric class alone issues as many instructions per level as the unified step, and the
// per-level exchange comes on top.  Included after rc_kernels.hip.
#pragma once

namespace rc {

typedef float SplitX[2][16][2][5];   // [class][entry][half] {t, shape, normal}, per parity

// Shape tests and hit frames for ONE shape class (round 6, the team leader's split step in
// rc_kernels.hip): kCls = 1 the scene's quadrics, 2 its spheres and planes.  Every value is
// produced by test_unified / hit_frame_sel's operations in their order (the other class's
// prelude folded away), so results are bit-identical to theirs — and to hit_sphere /
// hit_plane / hit_quadric — for every shape of the class.  A wave that holds one class issues
// only that class's instructions (the quadric prelude alone is most of test_unified's f64
// work).  Cross terms are kept (the resolver's form, RC_X0_RESOLVE 0).
template <int kCls>
__device__ __forceinline__ bool test_cls(const rc_shape& s, V3 O, V3 D, RayK rk, int skip,
                                         float& t) {
  constexpr bool kQ = kCls == 1, kSP = kCls == 2;
  const int type = s.type;
  const bool isS = kSP && type == RC_SHAPE_SPHERE, isP = kSP && type == RC_SHAPE_PLANE,
             isQ = kQ;   // a quadric-class lane holds a quadric (or no shape: masked by the caller)
  float cS = 0.0f, numP = 0.0f, bS = 0.0f, discS = 0.0f, denP = 0.0f;
  if constexpr (kSP) {
    const V3 tv = v3(O.x - s.p[0], O.y - s.p[1], O.z - s.p[2]);
    cS = (float)((double)dot(tv, tv) - s.r2);
    numP = pin(dot(tv, v3(s.n[0], s.n[1], s.n[2])));
    bS = 2.0f * dot(D, tv);
    const float facS = rk.a4 * cS;
    discS = (float)__builtin_fma((double)bS, (double)bS, -(double)facS);
    denP = dot(D, v3(s.n[0], s.n[1], s.n[2]));
  }
  float cq = 0.0f, aq = 0.0f, bq = 0.0f, discQ = 0.0f;
  bool lin = false;
  if constexpr (kQ) {
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
    discQ = (float)__builtin_fma((double)bq, (double)bq, -(4.0 * (double)aq * (double)cq));
    lin = (double)aq == 0.0;
  }
  const float B = kQ ? bq : bS;
  const float disc = kQ ? discQ : discS;
  const double sq = pin(sqrt_ns((double)disc));
  const double nb = (double)(-B);
  const bool qlin = isQ & lin;
  const double n1q = pin(nb - sq);
  const double n1p = kSP ? pin((double)(-numP)) : 0.0;
  const double n1l = kQ ? pin(-1.0 * (double)cq) : 0.0;
  const double num1 = isP ? n1p : (qlin ? n1l : n1q);
  const double den1 = kQ ? (qlin ? (double)bq : 2.0 * (double)aq) : (isP ? (double)denP : rk.den);
  const double num2 = nb + sq;
#if RC_NRDIV
  const double y1 = recip_nr(den1);
  const float q1 = (float)pin(div_nr(num1, den1, y1));
  const float q2 = (float)pin(div_nr(num2, den1, y1));
#else
  const float q1 = (float)pin(num1 / den1);
  const float q2 = (float)pin(num2 / den1);
#endif
  const bool second = (isS & (q1 < 0.0f)) | (isQ & !lin & (q1 <= 0.0f));
  const float tt = second ? q2 : q1;
  const bool okS = isS & !(disc < 0.0f);
  const bool okP = isP & (denP != 0.0f) & !(q1 < 0.0f);
  const bool okQ = isQ & (lin | !((double)disc < 0.0));
  const bool below = isQ & (skip != -1) & ((O.z + tt * D.z) < O.z);
  t = tt;
  return (okS | okP | okQ) & !below;
}

template <int kCls>
__device__ __forceinline__ void hit_frame_cls(const rc_shape& s, V3 O, V3 D, float t, V3& P,
                                              V3& N) {
  P = v3(O.x + D.x * t, O.y + D.y * t, O.z + D.z * t);
  if constexpr (kCls == 1) {
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
    const V3 n = normalize_sel(v3((float)n0, (float)n1, (float)n2));
    N = sel(dot(n, D) > 0.0f, v3(n.x * -1.0f, n.y * -1.0f, n.z * -1.0f), n);
  } else {
    const float inv = s.inv_r;
    const V3 n = normalize_sel(v3((P.x - s.p[0]) * inv, (P.y - s.p[1]) * inv,
                                  (P.z - s.p[2]) * inv));
    N = sel(s.type == RC_SHAPE_PLANE, v3(s.n[0], s.n[1], s.n[2]), n);
  }
}

// The cooperative step split by shape class (round 6).  A block step evaluates 16 entries at
// one carry, each with its two speculative levels; in the unified step every lane runs every
// shape type's test (a wave holds all types) and the leader's chain is issue-bound on them.
// Here waves 0-1 test only the scene's quadrics and waves 2-3 only its spheres and planes
// (test_cls / hit_frame_cls), 8 entries per wave: lane = entry (8 lanes) | half (4) | the
// class's shape k (<= 4 of each class).  After each level every wave publishes its class's
// nearest candidate (t, shape, normal) per entry and half, and one barrier later every lane
// takes the lexicographic (t, shape) minimum over both classes — the reference's nearest
// object, as in group_argmin_pos — and carries on with carry_path_spec's state machine.  The
// step's trip count must be the same in every wave (one barrier per level), so each lane
// also tracks the level and object of the entry 8 slots away (its "twin", held by the other
// wave pair) from the exchanged (t, shape) alone.
struct SplitLane {
  rc_shape s;   // this lane's shape (if has)
  int k;        // its index in the scene (file order)
  bool has;
  bool on;      // the scene fits the layout (both classes present, <= 4 shapes each)
};
__device__ __forceinline__ SplitLane split_lane(const Scene& sc, int wave, int lane) {
  SplitLane sl;
  sl.has = false;
  sl.k = 0x7fffffff;
  int nq = 0, nsp = 0;
  const int cls = wave < 2 ? 1 : 2, kl = lane & 3;
  for (int i = 0; i < sc.n; ++i) {   // wave-uniform: file order within each class
    const bool q = sc.shapes[i].type == RC_SHAPE_QUADRIC;
    const int idx = q ? nq++ : nsp++;
    if ((q ? 1 : 2) == cls && idx == kl) sl.k = i;
  }
  sl.on = nq >= 1 && nq <= 4 && nsp >= 1 && nsp <= 4 && sc.n <= 8;
  sl.has = sl.k != 0x7fffffff;
  sl.s = sc.shapes[sl.has ? sl.k : 0];
  return sl;
}

template <int kCls>
__device__ __forceinline__ V3 split_coop(const Scene& sc, BlockWinShared& bw, SplitX* sx,
                                         const SplitLane& sl,
                                         int pos, int nvalid, int maxrec, V3 c, bool& anyhit) {
  constexpr int kNone = 0x7fffffff;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int es = (wave & 1) * 8 + (lane >> 3), et = es ^ 8, half = (lane >> 2) & 1;
  const int i = pos + es, it = pos + et;
  const DepRec r = bw.rec[i < nvalid ? i : pos];
  V3 N = v3(r.n0x, r.n0y, r.n0z), C = c;
  V3 D1 = v3(r.ax, r.ay, r.az), D2 = v3(r.bx, r.by, r.bz);
  int obj = r.obj0, S = -1, lvl = 2;
  bool done = i >= nvalid || lvl >= maxrec || !reflective(sc, obj);
  int tobj = bw.rec[it < nvalid ? it : pos].obj0, tlvl = 2;
  bool tdone = it >= nvalid || tlvl >= maxrec || !reflective(sc, tobj);
  anyhit = false;
  int par = 0;
  // every exchanged value is read into registers first and chosen by selects (pointer or
  // short-circuit choices here compile to exec-masked branches and split the step)
  struct Cand {
    float t;
    int k;
    V3 n;
  };
  auto rd = [&](int cls, int e, int h) {
    const float* x = sx[par][cls][e][h];
    return Cand{x[0], __float_as_int(x[1]), v3(x[2], x[3], x[4])};
  };
  auto rdk = [&](int cls, int e, int h) {
    const float* x = sx[par][cls][e][h];
    return Cand{x[0], __float_as_int(x[1]), v3(0.0f, 0.0f, 0.0f)};
  };
  // lexicographic (t, k) minimum of two candidates (misses: t = inf, k = kNone), bitwise
  auto lexmin = [](const Cand& a, const Cand& b) {
    const bool tb = (b.t < a.t) | ((b.t == a.t) & (b.k < a.k));
    return Cand{tb ? b.t : a.t, tb ? b.k : a.k, sel(tb, b.n, a.n)};
  };
  while (__ballot(!done || !tdone) != 0) {   // the same decision in every wave (twins)
    const V3 myD = sel(half, D2, D1);
    const int myS = half ? -1 : S;
    const RayK rk = ray_consts(myD);
    float tt = 0.0f;
    const bool tok = test_cls<kCls>(sl.s, C, myD, rk, myS, tt);
    const bool ok = tok & sl.has & (sl.k != myS) & (__builtin_inff() > tt) & (tt > 0.0f);
    float t = ok ? tt : __builtin_inff();
    const int k = group_argmin_pos<4>(t, ok ? sl.k : kNone, 4);
    V3 P, Nw;
    hit_frame_cls<kCls>(sc.lshapes[k != kNone ? k : 0], C, myD, t, P, Nw);
    if ((lane & 3) == 0) {
      float* x = sx[par][kCls - 1][es][half];
      x[0] = t;
      x[1] = __int_as_float(k);
      x[2] = Nw.x;
      x[3] = Nw.y;
      x[4] = Nw.z;
    }
    __syncthreads();
    const Cand h0 = lexmin(rd(0, es, 0), rd(1, es, 0));   // this entry, level L
    const Cand h1 = lexmin(rd(0, es, 1), rd(1, es, 1));   // level L+1 if L misses
    const Cand u0 = lexmin(rdk(0, et, 0), rdk(1, et, 0)); // the twin entry
    const Cand u1 = lexmin(rdk(0, et, 1), rdk(1, et, 1));
    const bool hitL = h0.k != kNone;
    const bool two = !hitL & (lvl + 1 < maxrec);
    const int w = hitL ? h0.k : (two ? h1.k : kNone);
    const float tw = hitL ? h0.t : h1.t;
    const V3 nw = sel(hitL, h0.n, h1.n);
    const V3 Dw = sel(two, D2, D1);
    const bool hit = (w != kNone) & !done;
    anyhit = anyhit | hit;
    // P = C + Dw * tw: the operations of hit_frame_cls, on the winner's t
    C = sel(hit, v3(C.x + Dw.x * tw, C.y + Dw.y * tw, C.z + Dw.z * tw), C);
    N = sel(hit, nw, N);
    obj = hit ? w : obj;
    S = done ? S : (hit ? w : -1);
    lvl = done ? lvl : lvl + (two ? 2 : 1);
    done = done | (lvl >= maxrec) | !reflective(sc, obj);
    D1 = normalize_sel(reflect(Dw, N));
    D2 = normalize_sel(reflect(D1, N));
    {   // the twin entry's level and object, from its (t, shape) records alone
      const bool thitL = u0.k != kNone;
      const bool ttwo = !thitL & (tlvl + 1 < maxrec);
      const int tw_ = thitL ? u0.k : (ttwo ? u1.k : kNone);
      tobj = ((tw_ != kNone) & !tdone) ? tw_ : tobj;
      tlvl = tdone ? tlvl : tlvl + (ttwo ? 2 : 1);
      tdone = tdone | (tlvl >= maxrec) | !reflective(sc, tobj);
    }
    par ^= 1;
  }
  return C;
}


// One window of cooperative steps at 16 entries per step (block_window's coop branch with K
// large: no LANE passes, no predictor), the evaluation split by class.  Publishes every
// entry's carry-in like block_window.
__device__ __forceinline__ void split_block_window(const Scene& sc, int maxrec, BlockWinShared& bw,
                                                   SplitX* sx, const SplitLane& sl, int base,
                                                   int nvalid, V3& c, CinG* __restrict__ cin,
                                                   unsigned tag, WinStats& ws) {
  constexpr int kNo = 0x7fffffff;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  int pos = 0, par = 0;
  while (pos < nvalid) {
    ++ws.coop;
    bool hg = false;
    const V3 oc = wv < 2 ? split_coop<1>(sc, bw, sx, sl, pos, nvalid, maxrec, c, hg)
                         : split_coop<2>(sc, bw, sx, sl, pos, nvalid, maxrec, c, hg);
    const int i = pos + (wv & 1) * 8 + (lane >> 3);
    const bool act = wv < 2 && (lane & 7) == 0 && i < nvalid;
    if (act) bw.hit[i] = hg ? 1 : 0;
    const unsigned long long mc = __ballot(act && !same_bits(oc, c));
    const int g = mc ? (__ffsll((long long)mc) - 1) / 8 : -1;
    if (lane == 0) bw.wpos[par][wave] = g >= 0 ? pos + (wv & 1) * 8 + g : kNo;
    if (g >= 0 && lane == g * 8) {
      bw.wout[par][wave][0] = oc.x;
      bw.wout[par][wave][1] = oc.y;
      bw.wout[par][wave][2] = oc.z;
    }
    __syncthreads();
    int wb = 0, best = bw.wpos[par][0];
    for (int q = 1; q < 4; ++q)
      if (bw.wpos[par][q] < best) {
        best = bw.wpos[par][q];
        wb = q;
      }
    const bool hit = best != kNo;
    const int last = hit ? best : (pos + 16 < nvalid ? pos + 16 : nvalid) - 1;
    const V3 cn = hit ? v3(bw.wout[par][wb][0], bw.wout[par][wb][1], bw.wout[par][wb][2]) : c;
    const int w0 = wave * 64;
    const int lo = pos - w0 > 0 ? pos - w0 : 0;
    const int hi = last + 1 - w0 < 64 ? last + 1 - w0 : 64;
    const unsigned long long hm = __ballot(bw.hit[t] != 0);
    if (lo < hi) cin_put_wave_uniform(cin, base + w0, lo, hi, c, tag, hm);
    if (hit) ++ws.changers;
    pos = last + 1;
    c = cn;
    par ^= 1;
  }
}

}  // namespace rc
