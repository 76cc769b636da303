// rtw_world.hip — the general-world kernel: the reference's render loop and
// rayColor (main.zig:378-402, :103-122, emission included) over the full
// Hittable vocabulary (hittable.zig:22-608: spheres, moving spheres, xy/xz/yz
// rects, boxes, Translate, RotateY), all materials (material.zig:16-121,
// DiffuseLight included) and textures (texture.zig:10-144: solid, checker,
// Perlin noise, image), for every scene of main.zig and BASELINE.json
// configs[4] (globe + 10k spheres).  f64, the reference's arithmetic.
//
// Closest hit: wave-cooperative BVH2 traversal (both child boxes in the
// parent node; one stack per wave in LDS; scalar-loaded nodes and
// primitives), or a wave-uniform linear loop for small worlds.  The reference's HittableList.hit picks the object of
// minimal effective root, ties to the later object — an order-independent
// rule — so visiting primitives in BVH order returns the
// same winner as long as no box that could hold a winner is pruned: every
// box test is widened by `margin` (rtw_world_capi.hip bvh_margin: > the
// largest deviation of a computed root from the exact intersection) and is
// inclusive at tmax.  A NaN root (the reference's acceptance is then order
// dependent) sends the lane through the literal sequential loop.
//
// Per lane: the megakernel's work units (pixel, chunk of samples) with
// lane-level regeneration; per sample: the Tier-B counter RNG, rayColor
// evaluated forward (rad += T * emitted at a light, rad += T * background on a
// miss).  oracle/rtw_world.h Tier B is the written contract.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rtw_device.hpp"
#include "rtw_libm.hpp"

// (Measured choices that are now the only code: the BVH stack's top entry in a
// register, profiles/r02/world_topcache_ab.txt; the node visit's decisions as
// scalar refs made before its leaf tests, profiles/r04/world_decide_refs_ab.txt;
// the lane's state flags as bits of one word, profiles/r04/world_lane_flags_ab.txt;
// the left child's record line touched with every node visit,
// profiles/r04/world_touch_next_ab.txt.)

namespace rtwk {

// MODE 2 (-DRTW_MEASURE, RTW_WORLD_PHASE=1): s_memtime stamps per phase,
// summed per wave (diagnostic; rtw_world_capi.hip prints the shares).
#define WSTAMP(slot)                                                             \
  if constexpr (MODE == 2) {                                                     \
    __builtin_amdgcn_sched_barrier(0);                                           \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                           \
    st.ph[slot] += t_ - st.t_last;                                               \
    st.t_last = t_;                                                              \
  }

using D = double;
using V = V3<D>;

// FEAT: the features a world uses (rtw_world_capi.hip world_features); each
// kernel instantiation compiles only the paths of its features, so a world
// of plain spheres does not carry the register budget of Perlin noise,
// transform chains or rects (the budget sets the spills at 4 waves/SIMD).
constexpr int kFeatNoise = 1, kFeatImage = 2, kFeatXform = 4, kFeatRect = 8;
constexpr int kFeatAll = kFeatNoise | kFeatImage | kFeatXform | kFeatRect;
// Not a world feature: the sphere-world instantiation that traverses the BVH
// per lane (closest_lane) instead of as the wave's union (closest).
constexpr int kFeatLane = 16;
// ... reading each child's ref from its lower bounds' low bits (rtw_world_capi.hip pack_refs).
constexpr int kFeatPacked = 32;

__device__ __forceinline__ const uint32_t* meta_of(const D* r) { return reinterpret_cast<const uint32_t*>(r + 14); }

// Translate / RotateY chains (hittable.zig:478-491, :561-600), op 0 outermost.
template <typename P>
__device__ __forceinline__ void to_object(P xf, V& o, V& d) {
  const uint32_t h = (uint32_t)__builtin_bit_cast(uint64_t, (D)xf[0]);
  const uint32_t n = h & 0xFFu;
#pragma unroll
  for (uint32_t i = 0; i < kMaxXfOps; ++i) {  // unrolled: o, d stay in registers
    if (i >= n) break;
    const auto v = xf + 4 + 3 * i;
    if (((h >> (8 + 4 * i)) & 0xFu) == 0u) {
      o = sub(o, mk((D)v[0], (D)v[1], (D)v[2]));
    } else {
      const D sn = v[0], cs = v[1];
      const V o0 = o, d0 = d;
      o.x = cs * o0.x - sn * o0.z;
      o.z = sn * o0.x + cs * o0.z;
      d.x = cs * d0.x - sn * d0.z;
      d.z = sn * d0.x + cs * d0.z;
    }
  }
}
__device__ __forceinline__ void to_world(const D* xf, V& p, V& nrm) {
  const uint32_t h = *reinterpret_cast<const uint32_t*>(xf);
  const int n = (int)(h & 0xFFu);
#pragma unroll
  for (int i = (int)kMaxXfOps - 1; i >= 0; --i) {
    if (i >= n) continue;
    const D* v = xf + 4 + 3 * i;
    if (((h >> (8 + 4 * i)) & 0xFu) == 0u) {
      p = add(p, ld3(v));
    } else {
      const D sn = v[0], cs = v[1];
      const V p0 = p, n0 = nrm;
      p.x = cs * p0.x + sn * p0.z;
      p.z = -sn * p0.x + cs * p0.z;
      nrm.x = cs * n0.x + sn * n0.z;
      nrm.z = -sn * n0.x + cs * n0.z;
    }
  }
}

// The fields of a primitive record the closest-hit test reads (doubles 0-10
// and the meta words), loaded in one place so the linear loop can prefetch
// the next record (scalar loads through the constant address space) while
// the current one is tested.
struct PrimRec {
  D v[11];
  uint32_t meta0, orig;
};
template <typename P>
__device__ __forceinline__ PrimRec load_rec(P r) {
  PrimRec q;
#pragma unroll
  for (int i = 0; i < 11; ++i) q.v[i] = r[i];
  // meta u32 {kind | xform+1 << 8, mat, orig, 0} occupies doubles 14-15
  q.meta0 = (uint32_t)__builtin_bit_cast(uint64_t, (D)r[14]);
  q.orig = (uint32_t)__builtin_bit_cast(uint64_t, (D)r[15]);
  return q;
}

// The per-lane walk's record load: doubles 0-10 and the {kind, list index}
// copy in double 11 (rtw_world_capi.hip), one 96-B span = six 16-B loads.
template <typename P>
__device__ __forceinline__ PrimRec load_rec_lane(P r) {
  PrimRec q;
#pragma unroll
  for (int i = 0; i < 11; ++i) q.v[i] = r[i];
  const uint64_t m = __builtin_bit_cast(uint64_t, (D)r[11]);
  q.meta0 = (uint32_t)m;
  q.orig = (uint32_t)(m >> 32);
  return q;
}

// A ray in one primitive space with Sphere.hit's `a` = |d|^2 (hittable.zig:97)
// and ia = RN(1/a): the root divisions run as Markstein div_rn (rtw_math.hpp:
// RN(x / b) from RN(1 / b), IEEE division outside the normal range), the same
// bits as x / a.  (Reciprocals for the rect plane divisions measured slower on
// the Cornell box: three divisions per transform change plus register
// pressure, against one division per rect.)
struct RaySp {
  V o, d;
  D a, ia;
};
__device__ __forceinline__ RaySp ray_space(const V& o, const V& d, uint32_t flags) {
  RaySp s;
  s.o = o, s.d = d;
  s.a = norm2(d);
  s.ia = (flags & kWorldHasSpheres) ? (D)1 / s.a : (D)0;  // wave-uniform flag
  return s;
}

// XY / XZ / YZ rect (hittable.zig:305-331, :364-390, :423-449): k is the
// rect's constant axis, (a, b) the in-plane axes.
__device__ __forceinline__ bool rect_root(const D* r, D ok, D oa, D ob, D dk, D da, D db, D tmin, D& t) {
  const D tt = (r[4] - ok) / dk;
  if (tt < tmin) return false;
  const D x = oa + tt * da, y = ob + tt * db;
  if (x < r[0] || x > r[1] || y < r[2] || y > r[3]) return false;
  t = tt;
  return true;
}

// The primitive's effective root for ray (o, d) in world space: Sphere.hit /
// MovingSphere.hit root selection (hittable.zig:96-116, :166-187) or the rect
// plane hit with its containment test (:278-286, :333-341, :388-396).
// Returns false when the primitive cannot be hit at t >= tmin; t may be NaN.
// root_obj: the ray already in the primitive's object space; RCP: use the
// ray space's a and RN(1/a) (else plain IEEE divisions; same results).
template <bool RCP, int FEAT>
__device__ __forceinline__ bool root_obj(const PrimRec& q, const RaySp& s, D time, D tmin, D& t) {
  const D* r = q.v;
  const V& o = s.o;
  const V& d = s.d;
  const uint32_t kind = q.meta0 & 0xFFu;
  if (!(FEAT & kFeatRect) || kind <= 1u) {
    V c = mk(r[0], r[1], r[2]);
    if (kind == 1u)  // hittable.zig:219-221; r[10] = RN(1 / (time1 - time0))
      c = add(c, mul(mk(r[3], r[4], r[5]), rtwm::div_rn(time - r[7], r[8], r[10])));
    const V oc = sub(o, c);
    const D a = RCP ? s.a : norm2(d);
    const D hb = dot(oc, d);
    const D cc = norm2(oc) - r[9];
    const D disc = hb * hb - a * cc;
    if (disc < 0.0) return false;
    const D sq = sqrt(disc);
    D root = RCP ? rtwm::div_rn(-hb - sq, a, s.ia) : (-hb - sq) / a;
    if (root < tmin) root = RCP ? rtwm::div_rn(-hb + sq, a, s.ia) : (-hb + sq) / a;
    t = root;
    return !(root < tmin);
  }
  // one copy per axis-aligned kind (a select of the axes is turned into a
  // dynamically indexed stack copy of o and d by the optimiser)
  if (kind == 2u) return rect_root(r, o.z, o.x, o.y, d.z, d.x, d.y, tmin, t);
  if (kind == 3u) return rect_root(r, o.y, o.x, o.z, d.y, d.x, d.z, tmin, t);
  return rect_root(r, o.x, o.y, o.z, d.x, d.y, d.z, tmin, t);
}
template <int FEAT, typename WV>
__device__ __forceinline__ bool prim_root(const WV& W, const PrimRec& q, V o, V d, D time, D tmin, D& t) {
  const int xf = (int)(q.meta0 >> 8) - 1;
  if ((FEAT & kFeatXform) && xf >= 0) to_object(W.xform + kWorldRec * xf, o, d);
  RaySp s;
  s.o = o, s.d = d;
  return root_obj<false, FEAT>(q, s, time, tmin, t);
}

// fmaxf / fminf of two quiet operands as one v_max_f32 / v_min_f32: the
// compiler otherwise re-quiets (v_max x, x) the loop-carried tmin / tmax
// bounds on every node visit (IEEE mode); the instruction's NaN rule is
// fmaxf's (a quiet NaN operand yields the other one).
__device__ __forceinline__ float max_q(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float min_q(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ float max3_q(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float min3_q(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// The adjacent f32 toward +inf / -inf (finite or infinite x; NaN kept).
__device__ __forceinline__ float next_up(float x) {
  if (!(x < __builtin_inff())) return x;
  if (x == 0.0f) return __uint_as_float(1u);
  const uint32_t b = __float_as_uint(x);
  return __uint_as_float(x > 0.0f ? b + 1u : b - 1u);
}
__device__ __forceinline__ float next_down(float x) { return -next_up(-x); }

// a * {p[SP], p[SP]} + {q[SQ], q[SQ]} as one v_pk_fma_f32: op_sel / op_sel_hi
// pick the 32-bit half of each 64-bit operand for the low / high result, so
// two broadcast operands share one register pair (bc() pairs hold one value twice).
template <int SP, int SQ>
__device__ __forceinline__ f2 pk_fma_sel(f2 a, f2 p, f2 q) {
  f2 r;
  if constexpr (SP == 0 && SQ == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(a), "v"(p), "v"(q));
  else if constexpr (SP == 1 && SQ == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,0]" : "=v"(r) : "v"(a), "v"(p), "v"(q));
  else if constexpr (SP == 0 && SQ == 1)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(p), "v"(q));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,1] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(a), "v"(p), "v"(q));
  return r;
}

struct WHit {
  int pos;     // stored position of the winner (-1: miss)
  int orig;    // its list index
  D t;
  uint32_t nan;  // a NaN root was seen (a u32, not a bool: it stays in a VGPR instead of a lane-mask phi
                 // the traversal loop would copy through exec on every node visit)
};
__device__ __forceinline__ void accept(WHit& h, D t, int pos, int orig, D tmin) {
  h.nan |= (uint32_t)(t != t);
  if (!(t < tmin) & ((t < h.t) | ((t == h.t) & (orig > h.orig)))) {
    h.t = t;
    h.pos = pos;
    h.orig = orig;
  }
}

// The reference's literal sequential loop (HittableList.hit, :231-244) over
// the list in its original order; `order` maps list index -> stored position.
template <int FEAT, typename WV>
__device__ __forceinline__ void seq_hit(const WV& W, const uint32_t* order, V o, V d, D time, D tmin,
                                        WHit& h) {
  h.pos = -1;
  h.orig = -1;
  h.t = (D)__builtin_huge_val();
  for (uint32_t i = 0; i < W.n_prims; ++i) {
    const uint32_t k = order[i];
    D t;
    if (!prim_root<FEAT>(W, load_rec(W.prim + kWorldRec * k), o, d, time, tmin, t)) continue;
    if (h.t < t) continue;  // `t_max < root` rejects; NaN roots are accepted (as in the reference)
    h.t = t;
    h.pos = (int)k;
    h.orig = (int)i;
  }
}

template <int MODE, int FEAT, typename WV>
__device__ __forceinline__ void closest(const WV& W, D m, uint32_t* stack, const V& o, const V& d, D time,
                                        D tmin, WHit& h, unsigned long long& nv, unsigned long long& nt,
                                        KStats& st) {
  h.pos = -1;
  h.orig = -1;
  h.t = (D)__builtin_huge_val();
  h.nan = 0u;
  if (W.n_nodes == 0) {  // linear: wave-uniform loop, scalar-loaded records, one-ahead prefetch
    const RTW_CONST D* pr = cptr(W.prim);
    PrimRec cur = load_rec(pr);  // (a padding record follows the last primitive)
    int xf_cur = -1;             // wave-uniform: the transform the cached object-space ray is for
    RaySp s = ray_space(o, d, W.flags);
    for (uint32_t k = 0; k < W.n_prims; ++k) {
      const PrimRec nxt = load_rec(pr + kWorldRec * (k + 1));
      const int xf = (int)(cur.meta0 >> 8) - 1;
      if ((FEAT & kFeatXform) && xf != xf_cur) {  // consecutive primitives share a chain (a Box's six rects)
        xf_cur = xf;
        V oo = o, od = d;
        if (xf >= 0) to_object(cptr(W.xform) + kWorldRec * xf, oo, od);
        s = ray_space(oo, od, W.flags);
      }
      D t;
      if (MODE == 1) ++nt;
      if (root_obj<true, FEAT>(cur, s, time, tmin, t)) accept(h, t, (int)k, (int)cur.orig, tmin);
      cur = nxt;
    }
    return;
  }
  // Wave-cooperative BVH traversal: the wave walks ONE stack (wave-uniform,
  // in LDS) and descends into a child when ANY of its active lanes' rays
  // hits the child's box; a leaf's primitives are tested by every active
  // lane.  Node and primitive records are therefore wave-uniform (scalar
  // loads, no per-lane memory divergence, no divergent control flow), and
  // testing a primitive whose box a lane missed is harmless: acceptance is
  // the exact rule of §5.1, the box test only prunes.
  // Packed-f32 slab tests (two children per v_pk_fma_f32), conservative: the
  // f32 node bounds are rounded outward and every box is widened by a margin
  // that also covers the f32 rounding; the interval is
  // compared with tmin rounded down and the closest root rounded up.
  const V inv = mk((D)1 / d.x, (D)1 / d.y, (D)1 / d.z);
  const f2 ix = bc((float)inv.x), iy = bc((float)inv.y), iz = bc((float)inv.z);
  // slab t = fma(bound, RN(1/d), RN(-RN(o) RN(1/d)) -/+ RN(m |RN(1/d)|)): the margin is folded
  // into the per-lane offsets, lower bounds moved down and upper bounds up
  const float mf = (float)m;
  const float pxo = -(float)o.x * ix[0], pyo = -(float)o.y * iy[0], pzo = -(float)o.z * iz[0];
  const float mx = mf * fabsf(ix[0]), my = mf * fabsf(iy[0]), mz = mf * fabsf(iz[0]);
  const float sx = ix[0] < 0.0f ? -1.0f : 1.0f, sy = iy[0] < 0.0f ? -1.0f : 1.0f, sz = iz[0] < 0.0f ? -1.0f : 1.0f;
  const f2 oxl = bc(pxo - sx * mx), oxh = bc(pxo + sx * mx);
  const f2 oyl = bc(pyo - sy * my), oyh = bc(pyo + sy * my);
  const f2 ozl = bc(pzo - sz * mz), ozh = bc(pzo + sz * mz);
  const float tminf = next_down((float)tmin);
  auto round_up = [](D x) { return (D)(float)x < x ? next_up((float)x) : (float)x; };
  float tmaxf = round_up(h.t);
  const RTW_CONST float* cn = cptr(W.node);
  const RTW_CONST D* pr = cptr(W.prim);
  const RaySp ws = ray_space(o, d, W.flags);
  // Leaf pretest (kCullBit leaves): the megakernel's packed-f32 bound
  // (rtw_cull.hpp) for the leaf's <= 2 spheres; x < 0 proves the sphere's
  // exact discriminant negative for this lane, and a sphere no lane can hit
  // skips its exact test (the test would reject it in every lane).
  const float af = (float)ws.a;
  const rtwc::LaneCull lc = rtwc::lane_cull((float)o.x, (float)o.y, (float)o.z, af, W.cull_cmax);
  const rtwc::LaneConst lk = rtwc::lane_const(af, lc.alpha, W.cull_rho);
  const RTW_CONST f2* ct = reinterpret_cast<const RTW_CONST f2*>(cptr(W.cull));
  // Lane masks, fixed for the traversal (its control is wave-uniform): the
  // votes below combine them with one compare's ballot in scalar ops.
  const uint64_t act = wballot(true), cull_ok = wballot(lc.ok);
  uint32_t sp = 0, node = 0;  // wave-uniform
  uint32_t top = 0;  // the stack's top entry (valid while sp > 0); stack[0 .. sp-1] hold the ones below it
  auto leaf = [&](uint32_t ref) {
    WSTAMP(2)  // (MODE 2: node visits up to here)
    const uint32_t first = ref & 0x7FFFFFu, cnt = (ref >> 23) & kLeafCountMask;
    auto test_prim = [&](uint32_t k, const PrimRec& q) {
      const int xf = (int)(q.meta0 >> 8) - 1;
      D t;
      if (MODE == 1) ++nt;
      bool ok;
      if (!(FEAT & kFeatXform) || xf < 0) {  // separate calls: no copies of (o, d) on the untransformed path
        ok = root_obj<true, FEAT>(q, ws, time, tmin, t);
      } else {
        RaySp s;
        s.o = o, s.d = d;
        to_object(cptr(W.xform) + kWorldRec * xf, s.o, s.d);
        ok = root_obj<false, FEAT>(q, s, time, tmin, t);
      }
      if (ok) accept(h, t, (int)k, (int)q.orig, tmin);
    };
    bool need0 = true, need1 = true;
    if ((FEAT & ~(kFeatImage | kFeatLane)) == 0 && (ref & kCullBit)) {  // sphere worlds (the others ignore the bit)
      const f2 x = cull_pair<1>(ld_pair(ct, first), bc((float)o.x), bc((float)o.y), bc((float)o.z), bc((float)d.x),
                                bc((float)d.y), bc((float)d.z), bc(lk.na), bc(lk.k), bc((float)time));
      need0 = (act & ~(cull_ok & wballot(x.x < 0.0f))) != 0;  // some lane not proven to miss
      need1 = (act & ~(cull_ok & wballot(x.y < 0.0f))) != 0;
    }
    // (Loading the first primitive's record together with the pretest record,
    // one latency instead of two in a row, measured within noise:
    // profiles/r03/world_leaf_prefetch_ab.txt.)
    for (uint32_t k = first; k < first + cnt; ++k) {
      if (!(k == first ? need0 : (k == first + 1 ? need1 : true))) continue;  // wave-uniform
      test_prim(k, load_rec(pr + kWorldRec * k));
    }
    tmaxf = round_up(h.t);
    WSTAMP(3)  // leaf primitives
  };
  for (;;) {
    if (MODE == 1) ++nv;
    // 32-bit byte offset: the node's scalar loads take it as their SGPR offset.
    // (An LDS copy of the top levels, breadth-first, read with broadcast
    // ds_reads instead: 7 % slower, profiles/r03/world_lds_nodes_ab.txt.)
    const RTW_CONST float* nd =
        reinterpret_cast<const RTW_CONST float*>(reinterpret_cast<const RTW_CONST char*>(cn) + (node << 6));
    static_assert(kNodeWords * 4 == 64, "node record size");
    // The first word of record node + 1 — the left child whenever that child
    // is interior (depth-first layout, rtw_world_capi.hip Builder) — loaded
    // with this node's record (one wait covers both): the child's visit then
    // finds its line in the scalar cache.  (A padding record follows the last;
    // record node + 2 as well: 3 % slower, profiles/r04/world_touch_next_ab.txt.)
    const float touch = nd[kNodeWords];
    const uint32_t r0 = __float_as_uint(nd[12]), r1 = __float_as_uint(nd[13]);
    asm volatile("" ::"s"(touch), "s"(r0));  // (the touch's wait is the record's wait)
    // {child 0, child 1} per axis: words {lo0, lo1} x3 then {hi0, hi1} x3
    const f2 x0 = pfma(f2{nd[0], nd[1]}, ix, oxl), x1 = pfma(f2{nd[6], nd[7]}, ix, oxh);
    const f2 y0 = pfma(f2{nd[2], nd[3]}, iy, oyl), y1 = pfma(f2{nd[8], nd[9]}, iy, oyh);
    const f2 z0 = pfma(f2{nd[4], nd[5]}, iz, ozl), z1 = pfma(f2{nd[10], nd[11]}, iz, ozh);
    float tn[2];
    bool hit[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const float n = fmaxf(fmaxf(fminf(x0[c], x1[c]), fminf(y0[c], y1[c])), max_q(fminf(z0[c], z1[c]), tminf));
      const float f = fminf(fminf(fmaxf(x0[c], x1[c]), fmaxf(y0[c], y1[c])), min_q(fmaxf(z0[c], z1[c]), tmaxf));
      tn[c] = n;
      hit[c] = n <= f;
    }
    // (the ballots are reused by the vote below: ballots of hit[] made again
    // there would first rebuild hit[] in VGPRs from these lane masks)
    const uint64_t b0 = wballot(hit[0]), b1 = wballot(hit[1]);
    // The visit's decisions as 32-bit refs (kNoRef: none) made before the leaf
    // tests (which do not change them), by scalar compares and selects in asm:
    // as C++ bools, LLVM kept them across the leaf calls as 64-bit lane masks
    // (s_cselect -1 / 0, re-combined through exec at the joins), and as
    // integers made from bools it went through VGPRs (v_cndmask +
    // v_readfirstlane).  Globe SALU per wave-iteration 3,848 -> 3,151, -2.4 %
    // time (profiles/r04/world_decide_refs_ab.txt).
    constexpr uint32_t kNoRef = 0xFFFFFFFFu;  // (never a ref: interior refs < kLeafBit, leaf counts <= 2)
    // per child c: t = (some lane hit c) ? r_c : kNoRef; then by the leaf bit of r_c,
    // leaf ref l_c = leaf ? t : kNoRef and interior ref i_c = leaf ? kNoRef : t
    uint32_t la, lb, ia, ib;
    asm("s_cmp_lg_u64 %4, 0\n\ts_cselect_b32 %0, %6, -1\n\ts_bitcmp1_b32 %6, 31\n\t"
        "s_cselect_b32 %2, -1, %0\n\ts_cselect_b32 %0, %0, -1\n\t"
        "s_cmp_lg_u64 %5, 0\n\ts_cselect_b32 %1, %7, -1\n\ts_bitcmp1_b32 %7, 31\n\t"
        "s_cselect_b32 %3, -1, %1\n\ts_cselect_b32 %1, %1, -1"
        : "=&s"(la), "=&s"(lb), "=&s"(ia), "=&s"(ib)
        : "s"(b0), "s"(b1), "s"(r0), "s"(r1)
        : "scc");
    uint32_t nx = ia & ib, ps = kNoRef;  // at most one interior child hit: its ref (or kNoRef)
    if ((ia | ib) < kLeafBit) {          // both: the nearer first, by the vote of the #else branch
      const uint64_t le = wballot(tn[0] <= tn[1]), gt = wballot(tn[1] < tn[0]);
      const uint32_t v0 = popc64(b0 & (~b1 | le)), v1 = popc64(b1 & (~b0 | gt));
      nx = v0 >= v1 ? r0 : r1;
      ps = v0 >= v1 ? r1 : r0;
    }
    if (la != kNoRef) leaf(la);
    if (lb != kNoRef) leaf(lb);
    if (ps != kNoRef) {
      stack[sp++] = top;  // (entry 0 is a dummy when the stack was empty)
      top = ps;
    }
    if (nx != kNoRef) {
      node = nx;
    } else {
      if (sp == 0) {
        WSTAMP(2)
        break;
      }
      node = (uint32_t)__builtin_amdgcn_readfirstlane((int)top);
      top = stack[--sp];
    }
  }
}

// Per-lane BVH traversal (sphere worlds, FEAT & kFeatLane; VERDICT r4 ask 2):
// every lane walks its OWN path through the tree — its own stack (a column of
// this wave's LDS block, entry e of lane l at e * 64 + l: conflict-free),
// its own node loads (per-lane vector loads; the 371-KB globe BVH stays in
// L2), nearer child first by its own entry distance — instead of the wave
// walking the union of its 64 lanes' paths (86.6 wave-level node visits per
// segment on the globe against ~16 per lane).  While-while structure with
// speculative leaves (Aila & Laine): the lanes holding an interior node step
// until every lane holds a leaf (postponed, one per lane) or is out of work,
// then every lane at a leaf tests its <= 2 primitives.  Same slab arithmetic,
// margins and inclusive bounds as the union walk, the same
// order-independent acceptance (§5.1) and NaN fallback, so the same winner.
//
// Resumable: a wave's traversal loop runs to its longest path, so the phase
// YIELDS once fewer than `yield_lanes` of its lanes are still walking (and
// the wave has other work): the walking lanes keep their state (node, leaf,
// stack, closest hit: LaneTrav rows in LDS) and continue in the next
// iteration of the persistent loop, while the others shade their hits and
// start their next segments (dynamic ray fetch).  No result depends on when a
// walk pauses.
constexpr uint32_t kNoRef = 0xFFFFFFFFu;  // (never a ref: interior refs < kLeafBit, leaf counts <= 2)
// LaneTrav rows, [field][lane]: ref, pend, top; (pos + 1) | sp << 26 | nan << 31;
// orig; t (2 words).  The walk's f32 bound tmaxf is round_up(t), remade on
// resume.  (7 words: with the lane's attenuation rows, the per-lane kernel's
// LDS is 40 KB per 4-wave workgroup, four per CU: world_lds_bytes.)
constexpr uint32_t kTravWords = 7;
struct LaneTravRows {                     // one wave's rows, [field][lane]
  uint32_t w[kTravWords][64];
};
// A wave's dynamic LDS in the per-lane kernel, in 32-bit words: the stack
// columns, the LaneTrav rows and the attenuation rows (3 f64 per lane).  With
// the static tail rows (5 words per lane) and chunk sums (3 f64) a 4-wave
// workgroup holds 40 KB: four fit the CU's 160 KB (4 waves per SIMD).
constexpr uint32_t kLaneWaveWords = (kLaneStackLds + kTravWords + 6u) * 64u;
// (+ the node cache: 48 B per cached node record, once per workgroup)
static_assert(((kLaneWaveWords + (5u + 6u) * 64u) * 4u * (kWorldBlock / 64) + kNodeCache * 48u) * 4u <= 160u * 1024u,
              "per-lane kernel: four 4-wave workgroups per CU");
typedef float nf4 __attribute__((ext_vector_type(4)));
// Starts a walk from the root for this lane (no hit yet).
__device__ __forceinline__ void trav_begin(LaneTravRows* R, uint32_t lid) {
  R->w[0][lid] = 0u;  // the root node
  R->w[1][lid] = kNoRef;
  R->w[2][lid] = kNoRef;
  R->w[3][lid] = 0u;           // pos -1, sp 0, no NaN
  R->w[4][lid] = 0xFFFFFFFFu;  // orig -1
  const uint64_t tb = __builtin_bit_cast(uint64_t, (D)__builtin_huge_val());
  R->w[5][lid] = (uint32_t)tb;
  R->w[6][lid] = (uint32_t)(tb >> 32);
}
// One traversal phase of the lanes with `walking` set; returns true for the
// lanes whose walk finished in it (`h` = the closest hit).  Wave-converged.
template <int MODE, int FEAT, typename WV>
__device__ __forceinline__ bool trav_phase(const WV& W, D m, uint32_t* lstack, LaneTravRows* R, const nf4* ncache,
                                           uint32_t lid,
                                           bool walking, uint32_t yield_lanes, const V& o, const V& d, D time, D tmin,
                                           WHit& h, unsigned long long& nv, unsigned long long& nt,
                                           unsigned long long& wi, unsigned long long& wl) {
  if (!wany(walking)) return false;
  auto round_up = [](D x) { return (D)(float)x < x ? next_up((float)x) : (float)x; };
  uint32_t ref = kNoRef, pend = kNoRef, top = kNoRef, sp = 0u;
  float tmaxf = 0.0f;
  if (walking) {
    ref = R->w[0][lid];
    pend = R->w[1][lid];
    top = R->w[2][lid];
    const uint32_t w3 = R->w[3][lid];
    h.pos = (int)(w3 & ((1u << kTravPosBits) - 1u)) - 1;
    sp = (w3 >> kTravPosBits) & 31u;
    h.nan = w3 >> 31;
    h.orig = (int)R->w[4][lid];
    h.t = __builtin_bit_cast(D, (uint64_t)R->w[5][lid] | ((uint64_t)R->w[6][lid] << 32));
    tmaxf = round_up(h.t);  // (the walk keeps tmaxf == round_up(h.t): at its start, after every leaf)
  }
  const V inv = mk((D)1 / d.x, (D)1 / d.y, (D)1 / d.z);
  // The union walk's slab constants (closest), held two to a 64-bit register
  // pair instead of one value twice (bc): the per-lane walk's node bounds are
  // VGPRs, so its v_pk_fma_f32 broadcasts each constant from the half of the
  // pair op_sel names (pk_fma_sel) — 9 VGPRs fewer across the walk, which at the
  // 4-wave budget (128 VGPRs) is what kept the loop off scratch (the globe's
  // per-lane kernel spilled 80 B/lane, rewritten in its loop: DESIGN.md §6.3).
  const float ixf = (float)inv.x, iyf = (float)inv.y, izf = (float)inv.z;
  const float mf = (float)m;
  const float pxo = -(float)o.x * ixf, pyo = -(float)o.y * iyf, pzo = -(float)o.z * izf;
  const float mx = mf * fabsf(ixf), my = mf * fabsf(iyf), mz = mf * fabsf(izf);
  const float sx = ixf < 0.0f ? -1.0f : 1.0f, sy = iyf < 0.0f ? -1.0f : 1.0f, sz = izf < 0.0f ? -1.0f : 1.0f;
  const float tminf = next_down((float)tmin);
  const f2 I1 = f2{ixf, iyf}, I2 = f2{izf, tminf};
  const f2 O1 = f2{pxo - sx * mx, pyo - sy * my};  // lower x, y offsets
  const f2 O2 = f2{pzo - sz * mz, pxo + sx * mx};  // lower z, upper x
  const f2 O3 = f2{pyo + sy * my, pzo + sz * mz};  // upper y, z
  // the node and primitive tables' addresses, read from the kernel argument
  // once per phase (re-read in the loop, the scalar load's lgkmcnt wait also
  // waited for the stack pop's LDS read, which `top` is there to hide)
  using GF = const __attribute__((address_space(1))) float;  // global: vector memory loads, not flat
  GF* nodes = (GF*)W.node;
  // PACKED: refs in the lower bounds' low bytes, as 24 bits (rtw_world_capi.hip pack_refs): a leaf
  // is LB | (count - 1) << 22 | first; the walk keeps refs in that form (kNoRef stays kNoRef).
  constexpr bool PACKED = (FEAT & kFeatPacked) != 0;
  constexpr uint32_t LB = PACKED ? 0x800000u : kLeafBit;
  using GD = const __attribute__((address_space(1))) D;
  GD* pr = (GD*)W.prim;
  asm volatile("" : "+s"(nodes), "+s"(pr));
  const RaySp ws = ray_space(o, d, W.flags);
  // the stack's top entry lives in a register (`top`, kNoRef when empty;
  // entries below it in LDS): a pop waits on no LDS read
  auto pop = [&]() -> uint32_t {
    const uint32_t r = top;
    top = sp ? lstack[(--sp) * 64u + lid] : kNoRef;
    return r;
  };
  auto push = [&](uint32_t r) {
    if (top != kNoRef) lstack[(sp++) * 64u + lid] = top;
    top = r;
  };
  bool yielded = false;
  // (a phase yields only after some walk finished in it: every phase makes progress)
  const uint32_t start = popc64(wballot(walking));
  for (;;) {
    // Interior steps.  A lane that reaches a leaf postpones it (one slot) and
    // keeps walking; the phase ends once every lane holds a leaf or is out of
    // work (speculative while-while): the leaf tests then run with most lanes busy.
    for (;;) {
      const bool step = ref < LB;
      if (!wany(step & (pend == kNoRef))) break;
      const uint32_t nact = popc64(wballot((ref != kNoRef) | (pend != kNoRef)));
      if (nact < yield_lanes && nact < start) {
        yielded = true;  // few lanes left: pause the walk, let the others take new rays
        break;
      }
      if (MODE == 1 && lid == 0) ++wi;
      if (step) {
        if (MODE == 1) ++nv;
        // (a 32-bit byte offset from the SGPR base: the loads' saddr form, no 64-bit address math)
        typedef nf4 f4;
        const __attribute__((address_space(1))) f4* nd = reinterpret_cast<const __attribute__((address_space(1))) f4*>(
            reinterpret_cast<const __attribute__((address_space(1))) char*>(nodes) + (ref << 6));
        f4 q0, q1, q2;
        if (PACKED && kNodeCache > 0 && ref < kNodeCache) {  // the top of the tree: the workgroup's LDS copy
          q0 = ncache[3u * ref], q1 = ncache[3u * ref + 1u], q2 = ncache[3u * ref + 2u];
        } else {
          q0 = nd[0], q1 = nd[1], q2 = nd[2];
        }
#if RTW_LANE_TOUCH  // A/B builds: also touch record ref + 1 (child 0 when interior: depth-first layout;
                    // 5.8 % slower on the globe, profiles/r06/world_touch_ab.txt)
        const float touch = nd[4].x;
#endif
        // {child 0, child 1} per axis: words {lo0, lo1} x3 then {hi0, hi1} x3 (refs in words 12-13);
        // the per-lane constants two to a register pair (pk_fma_sel)
        const f2 x0 = pk_fma_sel<0, 0>(f2{q0.x, q0.y}, I1, O1), x1 = pk_fma_sel<0, 1>(f2{q1.z, q1.w}, I1, O2);
        const f2 y0 = pk_fma_sel<1, 1>(f2{q0.z, q0.w}, I1, O1), y1 = pk_fma_sel<1, 0>(f2{q2.x, q2.y}, I1, O3);
        const f2 z0 = pk_fma_sel<0, 0>(f2{q1.x, q1.y}, I2, O2), z1 = pk_fma_sel<0, 1>(f2{q2.z, q2.w}, I2, O3);
        float tn[2];
        bool hit[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          // (all in asm: the compiler would re-quiet the asm FMAs' outputs before each fminf / fmaxf,
          // but an FMA returns quiet NaNs only, so v_min / v_max on them are fminf / fmaxf)
          const float n = max3_q(min_q(x0[c], x1[c]), min_q(y0[c], y1[c]), max_q(min_q(z0[c], z1[c]), I2[1]));
          const float f = min3_q(max_q(x0[c], x1[c]), max_q(y0[c], y1[c]), min_q(max_q(z0[c], z1[c]), tmaxf));
          tn[c] = n;
          hit[c] = n <= f;
        }
        uint32_t r0, r1;
        if constexpr (PACKED) {  // child c's ref: the low bytes of its lower x / y / z bounds
          // v_perm_b32: byte i of the result = byte sel_i of {S0 (bytes 4-7), S1 (bytes 0-3)}, 0x0C = 0
          const uint32_t t0 = __builtin_amdgcn_perm(__float_as_uint(q0.z), __float_as_uint(q0.x), 0x0C0C0400u);
          const uint32_t t1 = __builtin_amdgcn_perm(__float_as_uint(q0.w), __float_as_uint(q0.y), 0x0C0C0400u);
          r0 = __builtin_amdgcn_perm(__float_as_uint(q1.x), t0, 0x0C040100u);
          r1 = __builtin_amdgcn_perm(__float_as_uint(q1.y), t1, 0x0C040100u);
        } else {
          const f4 q3 = nd[3];
          r0 = __float_as_uint(q3.x), r1 = __float_as_uint(q3.y);
        }
        const bool first0 = tn[0] <= tn[1];
        uint32_t nx = hit[0] ? r0 : (hit[1] ? r1 : kNoRef);
        if (hit[0] && hit[1]) {
          push(first0 ? r1 : r0);
          nx = first0 ? r0 : r1;
        }
        ref = nx != kNoRef ? nx : pop();
#if RTW_LANE_TOUCH
        asm volatile("" ::"v"(touch));  // (its wait here, at the end of the step)
#endif
        if (ref != kNoRef && ref >= LB && pend == kNoRef) {  // postpone the leaf, keep walking
          pend = ref;
          ref = pop();
        }
      }
    }
    if (yielded) break;
    // Leaf tests: the postponed leaf, else a leaf the lane stopped at.
    uint32_t lf = pend;
    if (lf == kNoRef && ref != kNoRef && ref >= LB) {
      lf = ref;
      ref = pop();
    }
    pend = kNoRef;
    if (!wany(lf != kNoRef)) {
      if (!wany(ref != kNoRef)) break;
      continue;
    }
    if (MODE == 1 && lid == 0) ++wl;
    if (lf != kNoRef) {  // 1 .. kMaxLeafPrims primitives
      static_assert(kWorldRec * sizeof(D) == 128, "primitive record size");
      const uint32_t first = PACKED ? (lf & 0x3FFFFFu) : (lf & 0x7FFFFFu);
      const uint32_t cnt = PACKED ? ((lf >> 22) & 1u) + 1u : (lf >> 23) & kLeafCountMask;
      for (uint32_t k = first; k < first + cnt; ++k) {
        if (MODE == 1) ++nt;
        D t;
        const PrimRec q = load_rec_lane(reinterpret_cast<GD*>(
            reinterpret_cast<const __attribute__((address_space(1))) char*>(pr) + (k << 7)));  // (kWorldRec doubles = 128 B)
        if (root_obj<true, FEAT>(q, ws, time, tmin, t)) accept(h, t, (int)k, (int)q.orig, tmin);
      }
      tmaxf = round_up(h.t);
    }
  }
  const bool finished = walking && ref == kNoRef && pend == kNoRef;
  if (walking && !finished) {  // paused: keep the walk's state for the next phase
    R->w[0][lid] = ref;
    R->w[1][lid] = pend;
    R->w[2][lid] = top;
    R->w[3][lid] = (uint32_t)(h.pos + 1) | (sp << kTravPosBits) | (h.nan << 31);
    R->w[4][lid] = (uint32_t)h.orig;
    const uint64_t tb = __builtin_bit_cast(uint64_t, h.t);
    R->w[5][lid] = (uint32_t)tb;
    R->w[6][lid] = (uint32_t)(tb >> 32);
  }
  return finished;
}

// Texture.value (texture.zig:36-144) for the winner's record.
template <int FEAT, typename WV>
__device__ __forceinline__ V tex_value(const WV& W, uint32_t ti, D u, D v, V p) {
  const D* t = W.tex + kWorldRec * ti;
  const uint32_t* th = reinterpret_cast<const uint32_t*>(t);
  switch (th[0]) {
    case 1u:  // checker: only the sign of sin(10x) sin(10y) sin(10z) matters (rtw_math.hpp)
      return rtwm::checker_odd((D)10 * p.x, (D)10 * p.y, (D)10 * p.z) ? ld3(t + 5) : ld3(t + 8);
    case 2u: {  // noise
      if constexpr (!(FEAT & kFeatNoise)) return mk(0.0, 0.0, 0.0);  // (no noise texture in this world), texture.zig:101-105 + Perlin.turb/noise (perlin.zig:49-91)
      const D* pr = W.perlin + (size_t)th[1] * (256 * 3 + 384);
      const uint32_t* perm = reinterpret_cast<const uint32_t*>(pr + 256 * 3);
      D accum = 0.0, weight = 1.0;
      V q = p;
      // Rolled loops (one corner at a time): unrolled, the 56 corner
      // evaluations would set the whole kernel's register budget.
#pragma unroll 1
      for (int oct = 0; oct < 7; ++oct) {
        const D fx = floor(q.x), fy = floor(q.y), fz = floor(q.z);
        const D uu0 = q.x - fx, vv0 = q.y - fy, ww0 = q.z - fz;
        const D uu = uu0 * uu0 * (3 - 2 * uu0), vv = vv0 * vv0 * (3 - 2 * vv0), ww = ww0 * ww0 * (3 - 2 * ww0);
        const int i = (int)fx, j = (int)fy, k = (int)fz;
        D nz = 0.0;
#pragma unroll 1
        for (int cr = 0; cr < 8; ++cr) {  // perlinInterp's i, j, k loops (perlin.zig:104-124), in order
          const int di = cr >> 2, dj = (cr >> 1) & 1, dk = cr & 1;
          const uint32_t ix = (uint32_t)(i + di) & 255u, iy = (uint32_t)(j + dj) & 255u, iz = (uint32_t)(k + dk) & 255u;
          const D* c = pr + 3 * (perm[ix] ^ perm[256 + iy] ^ perm[512 + iz]);
          const D ti = (D)di, tj = (D)dj, tk = (D)dk;
          const V wgt = mk(uu - ti, vv - tj, ww - tk);
          nz += (ti * uu + (1.0 - ti) * (1.0 - uu)) * (tj * vv + (1.0 - tj) * (1.0 - vv)) *
                (tk * ww + (1.0 - tk) * (1.0 - ww)) * dot(ld3(c), wgt);
        }
        accum += weight * nz;
        weight *= 0.5;
        q = mk(q.x * 2.0, q.y * 2.0, q.z * 2.0);
      }
      const D kk = 0.5 * (1.0 + rtwl::sin(t[11] * p.z + 10.0 * fabs(accum)));
      return mk(1 * kk, 1 * kk, 1 * kk);
    }
    case 3u: {  // image
      if constexpr (!(FEAT & kFeatImage)) return mk(0.0, 0.0, 0.0);  // (no image texture in this world), texture.zig:121-144 (row clamp: rtw_world.h)
      const uint32_t* im = W.image + 4 * th[2];
      const uint32_t w = im[0], hgt = im[1];
      const D uc = fmax(0.0, fmin(u, 1.0));
      const D vc = 1.0 - fmax(0.0, fmin(v, 1.0));
      const uint64_t i = (uint64_t)(uc * (D)w), j = (uint64_t)(vc * (D)hgt);
      const uint64_t i_ = i < w - 1 ? i : w - 1;
      uint64_t j_ = j < w - 1 ? j : w - 1;
      if (j_ > hgt - 1) j_ = hgt - 1;
      const uint8_t* px = W.pixels + ((uint64_t)im[2] | ((uint64_t)im[3] << 32)) + (j_ * w + i_) * 4;
      const uchar4 c = *reinterpret_cast<const uchar4*>(px);
      if (c.w == 0) return mk(0.0, 0.0, 1.0);
      const D s = 1.0 / 255.0;
      return mk(s * (D)c.x, s * (D)c.y, s * (D)c.z);
    }
    default:
      return ld3(t + 2);
  }
}

// OCC: minimum resident workgroups per CU asked of the register allocator
// (1 = unconstrained; chosen by A/B on MI355X, rtw_world_capi.hip).
template <int MODE, int OCC, int FEAT>
__global__ void __launch_bounds__(kWorldBlock, OCC) world_kernel(WorldArgs A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  // this wave's BVH stack: one column per lane (per-lane traversal) or one
  // wave-uniform stack (the union walk)
  uint32_t* stack = reinterpret_cast<uint32_t*>(lds_raw) +
                    (threadIdx.x >> 6) * ((FEAT & kFeatLane) ? kLaneWaveWords : kBvhStack);
  // per-lane traversal: this wave's LaneTrav rows follow its stack columns,
  // and the lanes' attenuation rows (T) follow them
  LaneTravRows* trav_rows = reinterpret_cast<LaneTravRows*>(stack + kLaneStackLds * 64u);
  double(*t_rows)[64] = reinterpret_cast<double(*)[64]>(stack + (kLaneStackLds + kTravWords) * 64u);
  // the per-lane walk's node cache (packed refs): the top kNodeCache records, words 0-11
  constexpr bool NCACHE = (FEAT & kFeatLane) != 0 && (FEAT & kFeatPacked) != 0 && kNodeCache > 0;
  const nf4* node_cache = nullptr;  // (staged below; no LDS at all when NCACHE is off)
  // Tail dealing rows of this wave's lanes (lane = the owner of a unit): the
  // first sample handed to other lanes (samples [hi, s_end) are theirs), the
  // ring entries they filled, the unit's pixel; and the dealing list.
  // (Row addresses formed at each use from the wave-uniform index: held as
  // pointers they cost registers across the whole loop.)
  __shared__ uint32_t tail_rows[kWorldBlock / 64][5][64];
  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
#define TL_HI tail_rows[wv][0]
#define TL_READY tail_rows[wv][1]
#define TL_PXLY tail_rows[wv][2]
#define TL_LIST tail_rows[wv][3]
#define TL_OWN tail_rows[wv][4]  // a helper's owner lane
#define TL_C tail_rows[wv][4]    // an owner's chunk (one row: a lane helps only once it owns no unit)
  // The lane's f64 chunk sum (a helper's: the radiance of the sample it
  // traces) lives in LDS too: it changes only when a sample ends.
  __shared__ double home_sum[kWorldBlock / 64][3][64];
#define HS(k) home_sum[wv][k][lid]
  // (The unit's pixel and chunk live only in these rows, read where used —
  // sample start, chunk-sum publish — instead of VGPRs across the loop.)
  // The world's fields are re-read from the kernel argument where used
  // (scalar loads through a laundered kernarg pointer) instead of living in
  // SGPRs for the whole kernel: at the 100-SGPR limit they spill to VGPR
  // lanes (v_writelane / v_readlane in the traversal loop).  As the
  // megakernel's scene fields (rtw_trace.hip VAR bit 512); +1.4 % on the
  // globe and Cornell (profiles/r02/world_karg_ab.txt).
  const RTW_CONST WorldView& W =
      opaque((const RTW_CONST WorldArgs*)__builtin_amdgcn_kernarg_segment_ptr())->w;
  // The loop's other argument fields too (as the megakernel's VAR bit 1024):
  // read where used, through the same laundered pointer.
#define WKA(f) (opaque((const RTW_CONST WorldArgs*)__builtin_amdgcn_kernarg_segment_ptr())->f)
  const uint32_t* order = W.order;
  const uint32_t lid = lane_id();
  if constexpr (NCACHE) {  // stage the node cache (every thread reaches this before the persistent loop)
    __shared__ nf4 ncache_lds[(kNodeCache > 0 ? kNodeCache : 1u) * 3u];
    const uint32_t nn = min(W.n_nodes, kNodeCache);
    const nf4* gn = reinterpret_cast<const nf4*>(W.node);
    for (uint32_t i = threadIdx.x; i < 3u * nn; i += kWorldBlock) ncache_lds[i] = gn[(i / 3u) * 4u + i % 3u];
    __syncthreads();
    node_cache = ncache_lds;
  }
  Lane<D> L;
  L.px = L.ly = L.c = L.s = L.s_end = L.depth = 0;
  L.rs = 0;
  L.skip = -1;
  // The path attenuation T (rayColor's product of attenuations, main.zig:117)
  // of the per-lane kernel lives in LDS rows: it changes only when a segment
  // is shaded, and held in VGPRs across the BVH walk it was what the 4-wave
  // budget spilled (written back every iteration of the persistent loop).
  auto t_get = [&]() -> V {
    if constexpr ((FEAT & kFeatLane) != 0) return mk(t_rows[0][lid], t_rows[1][lid], t_rows[2][lid]);
    return L.T;
  };
  auto t_set = [&](const V& v) {
    if constexpr ((FEAT & kFeatLane) != 0) {
      t_rows[0][lid] = v.x, t_rows[1][lid] = v.y, t_rows[2][lid] = v.z;
    } else {
      L.T = v;
    }
  };
  // rayColor forward (main.zig:103-122): a sample's radiance is nonzero only at
  // the event that ends it (a miss adds T * background, a light T * emitted),
  // so that one term joins the chunk sum directly: sx + (0 + x) == sx + x
  // (x >= +0), the oracle's `rad` (rtw_world.c sample_b) without its registers.
  // The lane's state flags as bits of ONE word (a VGPR): as bools, each was a
  // 64-bit lane mask in SGPRs for the whole loop, and at the traversal's SGPR
  // peak the compiler spilled SGPRs to VGPR lanes (v_writelane / v_readlane,
  // VALU instructions) around it.
  uint32_t lane_flags = 0u;
  LaneFlag<1u> have_unit{lane_flags};
  LaneFlag<2u> have_ray{lane_flags};
  LaneFlag<4u> done{lane_flags};
  LaneFlag<8u> waiting{lane_flags};   // owner: its own samples done, waiting for the ones other lanes trace
  LaneFlag<16u> helping{lane_flags};  // helper: traces sample L.s of lane TL_OWN[lid]'s unit
  LaneFlag<32u> walking{lane_flags};  // per-lane traversal: a paused BVH walk (state in its LaneTrav row)
  uint32_t qnext = 0, qend = 0;
  unsigned long long n_samples = 0, n_segments = 0, n_visits = 0, n_tests = 0, n_iters = 0;
  unsigned long long n_wi = 0, n_wl = 0;  // per-lane traversal: interior / leaf wave iterations
  KStats st;  // MODE 2: phase stamps
  if constexpr (MODE == 2) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st.t_last)::"memory");
  // The loop body, compiled twice: without the tail dealing for the bulk of
  // the launch, and with it once the queue ran dry for some lane of the wave
  // (its variables then are not live in the bulk loop's register allocation).
  // Returns 1 when every lane is done.
  auto body = [&](auto tail_tag) -> int {
    constexpr bool TAIL = decltype(tail_tag)::value;
    if (MODE == 1) ++n_iters;  // wave iterations (lane utilisation = segments / (64 x iterations))
    // ---- take units (wave-uniform; rtw_trace.hip step 1) ----
    const bool need = !have_unit && !done;
    const uint64_t needmask = __ballot(need);
    if (needmask) {
      const uint32_t n = (uint32_t)__popcll(needmask);
      const uint32_t rank = mbcnt64(needmask);
      const uint32_t rem = qend - qnext;
      uint32_t base2 = 0;
      if (n > rem) {
        uint32_t b = 0;
        if (lid == 0) b = atomicAdd(WKA(t.counter), kBatch);
        base2 = __shfl(b, 0);
      }
      if (need) {
        const uint32_t raw = rank < rem ? qnext + rank : base2 + (rank - rem);
        if (raw >= WKA(t.total_units)) {
          done = true;
        } else {
          const uint32_t unit = dealt_unit(raw, WKA(t));
          const uint32_t units_per_tile = kTileW * kTileH * WKA(t.n_chunks);
          const uint32_t tile = rtwm::udiv(unit, WKA(t.upt_m), WKA(t.upt_sh));  // unit / units_per_tile
          const uint32_t r = unit - tile * units_per_tile;
          const uint32_t tiles_x = WKA(t.tiles_x);
          const uint32_t ty = rtwm::udiv(tile, WKA(t.tx_m), WKA(t.tx_sh)), tx = tile - ty * tiles_x;
          const uint32_t px = tx * kTileW + ((r & 63u) & 7u), ly = ty * kTileH + ((r & 63u) >> 3);
          if (px < WKA(t.W) && ly < WKA(t.row_count)) {
            have_unit = true;
            L.s = (r >> 6) * WKA(t.chunk);
            TL_C[lid] = r >> 6;
            L.s_end = min(L.s + WKA(t.chunk), WKA(t.spp));
            HS(0) = HS(1) = HS(2) = 0.0;
            TL_HI[lid] = L.s_end;
            TL_READY[lid] = 0u;
            TL_PXLY[lid] = px | (ly << 16);
          }
        }
      }
      if (n > rem) {
        qnext = base2 + (n - rem);
        qend = base2 + kBatch;
      } else {
        qnext += n;
      }
    }
    if (!__any(have_unit)) {
      if (__all(done)) return 1;
      return 0;
    }
    // ---- tail: once the queue ran dry for some lane of the wave, the lanes
    // left without a unit trace the LAST samples of the wave's other units
    // (one per offering unit per pass, up to kTailWin of a unit), each
    // sample's radiance going to its owner's ring; an owner stops at the
    // first sample it handed out and folds the ring in sample order
    // (main.zig:393), the other engines' addition sequence.  A world unit
    // runs ~84 wave iterations, so without this the launch ends with lanes
    // idle while the last units finish.
    constexpr bool tail = TAIL;
    if constexpr (tail) {
      for (;;) {
        const bool free_lane = done && !have_unit && !helping;
        const uint64_t needm = wballot(free_lane);
        if (!needm) break;
        uint32_t hi = 0;
        bool offer = false;
        if (have_unit && !waiting) {  // (L.s: the sample in flight or the next to start)
          hi = TL_HI[lid];
          offer = hi > max(L.s + 1u, L.s_end > kTailWin ? L.s_end - kTailWin : 0u);
        }
        const uint64_t offm = wballot(offer);
        if (!offm) break;
        const uint32_t ro = mbcnt64(offm);
        if (offer) {
          TL_LIST[ro] = lid | ((hi - 1u) << 6);
          if (ro < popc64(needm)) TL_HI[lid] = hi - 1u;
        }
        wave_lds_sync();
        const uint32_t rw = mbcnt64(needm);
        if (free_lane && rw < popc64(offm)) {
          const uint32_t e = TL_LIST[rw];
          helping = true;
          TL_OWN[lid] = e & 63u;
          L.s = e >> 6;
          HS(0) = HS(1) = HS(2) = 0.0;
        }
        wave_lds_sync();
      }
    }
    // ---- new sample ----
    if (((have_unit && !waiting) || helping) && !have_ray) {
      D u, v, dk[2];
      const uint32_t pl = TL_PXLY[helping ? TL_OWN[lid] : lid];  // the unit's pixel (this lane's or its owner's)
      L.px = pl & 0xFFFFu;
      L.ly = pl >> 16;
      start_sample_uv<D>(kargs<D>(), L, u, v);
      for (;;) {  // randomPointInUnitDisk, rand.zig:30-36
        dk[0] = rrange_m11<D>(L.rs);
        dk[1] = rrange_m11<D>(L.rs);
        if (in_unit_ball<D, 2>(dk)) break;
      }
      start_sample_ray<D>(kargs<D>(), L, u, v, dk[0], dk[1]);
      t_set(L.T);  // (= 1, 1, 1: start_sample_ray)
      have_ray = true;
    }
    // ---- one segment ----
    bool ended = false;
    // The hit record, texture and scatter of a lane whose closest hit is h
    // (written once, used by both traversals).
    auto shade = [&](WHit& h) {
      if (__builtin_expect(h.nan != 0u, 0)) seq_hit<FEAT>(W, order, L.o, L.d, L.time, WKA(t.tmin), h);
      if (h.pos < 0) {  // miss: background (main.zig:109-112)
        const V c = mulv(t_get(), ld3(opaque(kargs<D>())->bg));
        HS(0) += c.x;
        HS(1) += c.y;
        HS(2) += c.z;
        ended = true;
      } else {
        // Hit record of the winner (object space, then the wrappers back).
        const D* r = W.prim + kWorldRec * h.pos;
        const uint32_t* mt = meta_of(r);
        const uint32_t kind = mt[0] & 0xFFu;
        const int xf = (int)(mt[0] >> 8) - 1;
        V o = L.o, d = L.d;
        if ((FEAT & kFeatXform) && xf >= 0) to_object(W.xform + kWorldRec * xf, o, d);
        V p = add(o, mul(d, h.t)), nrm;
        bool front;
        D tu = 0.0, tv = 0.0;
        const D* mp = W.mat + 8 * mt[1];
        const uint32_t* mh = reinterpret_cast<const uint32_t*>(mp);
        const uint32_t mkind = mh[0], mtex = mh[1];
        const bool image_tex = (FEAT & kFeatImage) &&
            (mkind == 0u || mkind == 3u) && *reinterpret_cast<const uint32_t*>(W.tex + kWorldRec * mtex) == 3u;
        if (!(FEAT & kFeatRect) || kind <= 1u) {
          V c = ld3(r);
          if (kind == 1u) c = add(c, mul(ld3(r + 3), (L.time - r[7]) / r[8]));
          const V outward = divs(sub(p, c), r[6]);
          front = dot(outward, d) < 0.0;
          nrm = front ? outward : mul(outward, -1.0);
          if (kind == 0u && image_tex) {  // getSphereUv (hittable.zig:145-150)
            const D pi = 3.14159265358979323846;
            tu = (rtwl::atan2(-outward.z, outward.x) + pi) / (2.0 * pi);
            tv = rtwl::acos(-outward.y) / pi;
          }
        } else {
          D oa, ob, da, db;
          V n0;
          if (kind == 2u) {
            oa = o.x, ob = o.y, da = d.x, db = d.y, n0 = mk(0.0, 0.0, 1.0);
          } else if (kind == 3u) {
            oa = o.x, ob = o.z, da = d.x, db = d.z, n0 = mk(0.0, 1.0, 0.0);
          } else {
            oa = o.y, ob = o.z, da = d.y, db = d.z, n0 = mk(1.0, 0.0, 0.0);
          }
          tu = (oa + h.t * da - r[0]) / r[5];
          tv = (ob + h.t * db - r[2]) / r[6];
          front = dot(n0, d) < 0.0;
          nrm = front ? n0 : mul(n0, -1.0);
        }
        if ((FEAT & kFeatXform) && xf >= 0) to_world(W.xform + kWorldRec * xf, p, nrm);
        if (mkind == 3u) {  // DiffuseLight: emitted, no scatter (material.zig:94-110)
          const V c = mulv(t_get(), tex_value<FEAT>(W, mtex, tu, tv, p));
          HS(0) += c.x;
          HS(1) += c.y;
          HS(2) += c.z;
          ended = true;
        } else {
          V ndir, att;
          bool absorbed = false;
          // Lambertian and Metal draw their unit-ball point in ONE per-lane
          // rejection loop (randomPointInUnitSphere, rand.zig:22-28; the wave
          // would otherwise run the two loops one after the other), and every
          // lane makes one normalisation: the ball point (Lambertian) or the
          // ray direction (Metal, Dielectric).  Same draws, same operations.
          D b3[3] = {0.0, 0.0, 0.0};
          if (mkind <= 1u) {
            for (;;) {
              b3[0] = rrange_m11<D>(L.rs);
              b3[1] = rrange_m11<D>(L.rs);
              b3[2] = rrange_m11<D>(L.rs);
              if (in_unit_ball<D, 3>(b3)) break;
            }
          }
          const V nv = normalized(mkind == 0u ? mk(b3[0], b3[1], b3[2]) : L.d);
          if (mkind == 0u) {  // Lambertian (material.zig:44-52)
            ndir = add(nrm, nv);
            if (fabs(ndir.x) < 1e-8 && fabs(ndir.y) < 1e-8 && fabs(ndir.z) < 1e-8) ndir = nrm;
            att = tex_value<FEAT>(W, mtex, tu, tv, p);
          } else {
            // reflect(ud, nrm) (material.zig:112-114) for Metal and Dielectric;
            // the Dielectric's dot(-ud, nrm) (:75) is exactly -dun
            const V& ud = nv;
            const D dun = dot(ud, nrm);
            const V refl = sub(ud, mul(nrm, 2 * dun));
            if (mkind == 1u) {  // Metal (material.zig:59-65)
              ndir = add(refl, mul(mk(b3[0], b3[1], b3[2]), mp[4]));
              att = ld3(mp + 1);
              absorbed = !(dot(refl, nrm) > 0.0);
            } else {  // Dielectric (material.zig:72-91)
              const D ir = mp[5];
              const D ratio = front ? 1.0 / ir : ir;
              const D cos_t = fmin(-dun, 1.0);
              const D sin_t = sqrt(1.0 - cos_t * cos_t);
              bool refr = false;
              if (ratio * sin_t <= 1.0) {
                const D r0 = (1.0 - ratio) / (1.0 + ratio);
                const D r1 = r0 * r0;
                const D x = 1.0 - cos_t, x2 = x * x;
                refr = r1 + (1.0 - r1) * (x * (x2 * x2)) < rnd<D>(L.rs);  // Zig pow(x, 5.0)
              }
              if (refr) {  // refract (:116-121); its cos_theta is cos_t
                const V perp = mul(add(ud, mul(nrm, cos_t)), ratio);
                ndir = add(perp, mul(nrm, -sqrt(fabs(1.0 - norm2(perp)))));
              } else {
                ndir = refl;
              }
              att = mk(1.0, 1.0, 1.0);
            }
          }
          if (absorbed) {
            ended = true;
          } else {
            t_set(mulv(t_get(), att));
            L.o = p;
            L.d = ndir;
            L.depth++;
          }
        }
      }
    };
    if constexpr ((FEAT & kFeatLane) != 0) {
      if (have_ray && !walking) {
        if (L.depth == WKA(t.max_depth)) {
          ended = true;  // rayColor(depth == 0) is black (main.zig:105-108)
        } else {
          walking = true;
          trav_begin(trav_rows, lid);
          if (MODE == 1) ++n_segments;
        }
      }
      WSTAMP(1)  // sample start (+ take units, loop control)
      // (walks yield in the tail copy of the loop too: the lanes that stopped
      // walking then take the wave's other units' samples.  A `wall(done)` test
      // here never held while a lane walked — a done lane without a unit only
      // walks as a helper, and helpers exist only while an owner, not done,
      // holds its unit: ADVICE r5 — and is gone.)
      const uint32_t yl = WKA(lane_yield);
      WHit h;
      if (trav_phase<MODE, FEAT>(W, WKA(margin), stack, trav_rows, node_cache, lid, walking, yl, L.o, L.d, L.time, WKA(t.tmin),
                                 h, n_visits, n_tests, n_wi, n_wl)) {
        walking = false;
        shade(h);
      }
    } else if (have_ray) {
      if (L.depth == WKA(t.max_depth)) {
        ended = true;  // rayColor(depth == 0) is black (main.zig:105-108)
      } else {
        if (MODE == 1) ++n_segments;
        WHit h;
        WSTAMP(1)  // sample start (+ take units, loop control)
        closest<MODE, FEAT>(W, WKA(margin), stack, L.o, L.d, L.time, WKA(t.tmin), h, n_visits, n_tests, st);
        shade(h);
      }
    }
    WSTAMP(4)  // hit record, texture, scatter (+ the NaN fallback)
    if (ended && helping) {  // a sample of another lane's unit: its radiance to that lane's ring
      const uint32_t j = L.s % kTailWin, o = TL_OWN[lid];
      double* rg = WKA(ring) + ((size_t)(blockIdx.x * kWorldBlock + wv * 64u + o) * kTailWin + j) * 3;
      rg[0] = HS(0);
      rg[1] = HS(1);
      rg[2] = HS(2);
      atomicOr(&TL_READY[o], 1u << j);
      helping = false;
      have_ray = false;
      if (MODE == 1) ++n_samples;
    } else if (ended) {  // (its radiance joined the chunk sum above, main.zig:393)
      L.s++;
      have_ray = false;
      if (MODE == 1) ++n_samples;
      if (L.s != L.s_end && tail && L.s == TL_HI[lid]) waiting = true;  // the rest went to other lanes
      if (L.s == L.s_end) {
        const uint32_t npix = WKA(t.row_count) * WKA(t.W);
        const uint32_t pl = TL_PXLY[lid];
        double* dst = WKA(t.partial) + ((size_t)TL_C[lid] * npix + (size_t)(pl >> 16) * WKA(t.W) + (pl & 0xFFFFu)) * 3;
        dst[0] = HS(0);
        dst[1] = HS(1);
        dst[2] = HS(2);
        have_unit = false;
      }
    }
    // ---- owners waiting on other lanes' samples fold their ring in order ----
    if constexpr (tail) {
      // the ring entries written above, read by other lanes of this wave
      // (wavefront scope: as wf_drain's ring, rtw_wavefront.hip)
      wave_lds_sync();
      if (waiting) {
        uint32_t rdy = TL_READY[lid];
        const double* rb = WKA(ring) + (size_t)(blockIdx.x * kWorldBlock + threadIdx.x) * kTailWin * 3;
        double sx = HS(0), sy = HS(1), sz = HS(2);
        while (L.s != L.s_end && ((rdy >> (L.s % kTailWin)) & 1u)) {
          const uint32_t j = L.s % kTailWin;
          sx += rb[3 * j];
          sy += rb[3 * j + 1];
          sz += rb[3 * j + 2];
          rdy &= ~(1u << j);
          L.s++;
        }
        HS(0) = sx, HS(1) = sy, HS(2) = sz;
        TL_READY[lid] = rdy;
        if (L.s == L.s_end) {
          const uint32_t npix = WKA(t.row_count) * WKA(t.W);
          const uint32_t pl = TL_PXLY[lid];
          double* dst = WKA(t.partial) + ((size_t)TL_C[lid] * npix + (size_t)(pl >> 16) * WKA(t.W) + (pl & 0xFFFFu)) * 3;
          dst[0] = sx;
          dst[1] = sy;
          dst[2] = sz;
          have_unit = false;
          waiting = false;
        }
      }
    }
    return 0;
  };
  for (;;) {
    if (body(std::false_type{}) == 1) break;
    if (WKA(tail_deal) != 0u && __any(done)) {
      while (body(std::true_type{}) != 1) {
      }
      break;
    }
  }
#undef TL_HI
#undef TL_READY
#undef TL_PXLY
#undef TL_LIST
#undef TL_OWN
#undef TL_C
#undef HS
  if constexpr (MODE == 2) {
    WSTAMP(0)
    if (lid == 0)
      for (int i = 0; i < 5; ++i) atomicAdd(A.counts + 8 + i, (unsigned long long)st.ph[i]);
  }
  if constexpr (MODE == 1) {
    atomicAdd(A.counts + 0, n_samples);
    atomicAdd(A.counts + 1, n_segments);
    atomicAdd(A.counts + 2, n_visits);
    atomicAdd(A.counts + 3, n_tests);
    if (lid == 0) atomicAdd(A.counts + 4, n_iters);
    if ((FEAT & kFeatLane) && lid == 0) {
      atomicAdd(A.counts + 5, n_wi);
      atomicAdd(A.counts + 6, n_wl);
    }
  }
}

size_t world_lds_bytes(uint32_t, int fs) {
  return (size_t)((fs & kFeatLane) ? kLaneWaveWords : kBvhStack) * (kWorldBlock / 64) * sizeof(uint32_t);
}

template <int OCC, int FEAT>
static void launch_occ(const WorldArgs& a, uint32_t grid, size_t lds, hipStream_t s, int mode) {
#ifdef RTW_MEASURE
  if (mode == 2) {
    hipLaunchKernelGGL((world_kernel<2, OCC, FEAT>), dim3(grid), dim3(kWorldBlock), lds, s, a);
    return;
  }
#endif
  if (mode == 1)
    hipLaunchKernelGGL((world_kernel<1, OCC, FEAT>), dim3(grid), dim3(kWorldBlock), lds, s, a);
  else
    hipLaunchKernelGGL((world_kernel<0, OCC, FEAT>), dim3(grid), dim3(kWorldBlock), lds, s, a);
}
template <int FEAT>
static void launch_feat(const WorldArgs& a, uint32_t grid, size_t lds, hipStream_t s, int mode, int occ) {
#ifdef RTW_WORLD_ISA_QUICK  // (ISA inspection of the globe's kernel only: tools/isa_world.sh)
  if constexpr (FEAT == (kFeatImage | kFeatLane | kFeatPacked)) hipLaunchKernelGGL((world_kernel<0, 4, FEAT>), dim3(grid), dim3(kWorldBlock), lds, s, a);
#else
  if (occ >= 4)
    launch_occ<4, FEAT>(a, grid, lds, s, mode);
  else if (occ == 3)
    launch_occ<3, FEAT>(a, grid, lds, s, mode);
  else
    launch_occ<1, FEAT>(a, grid, lds, s, mode);
#endif
}
// Instantiated feature sets: spheres with solid / checker / image textures
// (scenes 1, 2, 4 and configs[4]'s globe), rects + transforms + lights without
// noise / image (the Cornell box, scene 5's light), and everything.
int world_feature_set(uint32_t feat, bool lane, bool packed) {
  if ((feat & ~(uint32_t)kFeatImage) == 0u)
    return lane ? (packed ? (kFeatImage | kFeatLane | kFeatPacked) : (kFeatImage | kFeatLane)) : kFeatImage;
  if ((feat & ~(uint32_t)(kFeatXform | kFeatRect)) == 0u) return kFeatXform | kFeatRect;
  return kFeatAll;
}
hipError_t launch_world(const WorldArgs& a, uint32_t grid, size_t lds, hipStream_t s, int mode, int occ, int fs) {
  if (fs == (kFeatImage | kFeatLane | kFeatPacked))
    launch_feat<kFeatImage | kFeatLane | kFeatPacked>(a, grid, lds, s, mode, occ);
  else if (fs == (kFeatImage | kFeatLane))
    launch_feat<kFeatImage | kFeatLane>(a, grid, lds, s, mode, occ);
  else if (fs == kFeatImage)
    launch_feat<kFeatImage>(a, grid, lds, s, mode, occ);
  else if (fs == (kFeatXform | kFeatRect))
    launch_feat<kFeatXform | kFeatRect>(a, grid, lds, s, mode, occ);
  else
    launch_feat<kFeatAll>(a, grid, lds, s, mode, occ);
  return hipGetLastError();
}

template <int FEAT>
static int bpc_feat(size_t lds, int occ) {
  int nb = 0;
  hipError_t e;
#ifdef RTW_WORLD_ISA_QUICK
  e = hipSuccess, nb = 1, (void)lds, (void)occ;
#else
  if (occ >= 4)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, world_kernel<0, 4, FEAT>, kWorldBlock, lds);
  else if (occ == 3)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, world_kernel<0, 3, FEAT>, kWorldBlock, lds);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, world_kernel<0, 1, FEAT>, kWorldBlock, lds);
#endif
  return (e == hipSuccess && nb > 0) ? nb : 1;
}
int world_blocks_per_cu(size_t lds, int occ, int fs) {
  if (fs == (kFeatImage | kFeatLane | kFeatPacked)) return bpc_feat<kFeatImage | kFeatLane | kFeatPacked>(lds, occ);
  if (fs == (kFeatImage | kFeatLane)) return bpc_feat<kFeatImage | kFeatLane>(lds, occ);
  if (fs == kFeatImage) return bpc_feat<kFeatImage>(lds, occ);
  if (fs == (kFeatXform | kFeatRect)) return bpc_feat<kFeatXform | kFeatRect>(lds, occ);
  return bpc_feat<kFeatAll>(lds, occ);
}

}  // namespace rtwk
