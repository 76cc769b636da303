// rtw_trace.hip — CDNA4 (gfx950) megakernel for the RTIOW cover-scene render
// loop: the reference's main.zig:378-402 loop + rayColor (main.zig:103-122)
// + HittableList/Sphere/MovingSphere.hit (hittable.zig:95-244) +
// Lambertian/Metal/Dielectric.scatter (material.zig:44-121) + Solid/Checker
// textures (texture.zig:46-83), re-designed for 64-wide wavefronts.
//
// Design (DESIGN.md has the full rationale):
//  * Work unit = (pixel, chunk of `chunk` samples).  Units are dealt from ONE
//    device counter in batches of 64 per wave (one atomic per 64 units); a
//    lane that finishes its unit takes the next one from the wave's batch at
//    once ("lane-level regeneration"), so lanes never wait for the slowest
//    path of the wave and the end-of-launch drain is one chunk long.
//  * Per lane, one loop iteration = [take a unit] -> [start a sample: seed the
//    per-sample Xoshiro256++, camera ray] -> [one bounce segment].  Paths of
//    different length share the wave without padding to the longest.
//  * The closest-hit loop over the sphere list is wave-UNIFORM: every lane
//    tests sphere k at the same time, so sphere k's record is fetched with
//    scalar loads (s_load, SGPR operands of the VALU ops): zero VGPRs and zero
//    LDS traffic for the hottest data.  The per-lane lookups that follow (the
//    winning sphere, its material) index LDS copies of the tables.
//  * Arithmetic follows the reference operation by operation (compiled with
//    -ffp-contract=off): precision 0 is the reference's f64; precision 1 is
//    f32 with wide (radius >= 100) spheres solved in f64 and convex self-skip.
//  * Per-chunk sums (f64) go to HBM; a second kernel adds chunks in order and
//    quantises exactly like main.zig:395-400.
// The oracle's tierb_core.h is the written contract this file implements.
#include <hip/hip_runtime.h>

#include "rtw_internal.hpp"

namespace rtwk {

// ------------------------------------------------------------------ vec --
template <typename R>
struct V3 {
  R x, y, z;
};
template <typename R>
__device__ __forceinline__ V3<R> mk(R x, R y, R z) {
  return V3<R>{x, y, z};
}
template <typename R>
__device__ __forceinline__ V3<R> add(V3<R> a, V3<R> b) {
  return mk(a.x + b.x, a.y + b.y, a.z + b.z);
}
template <typename R>
__device__ __forceinline__ V3<R> sub(V3<R> a, V3<R> b) {
  return mk(a.x - b.x, a.y - b.y, a.z - b.z);
}
template <typename R>
__device__ __forceinline__ V3<R> mul(V3<R> a, R t) {
  return mk(a.x * t, a.y * t, a.z * t);
}
template <typename R>
__device__ __forceinline__ V3<R> mulv(V3<R> a, V3<R> b) {
  return mk(a.x * b.x, a.y * b.y, a.z * b.z);
}
template <typename R>
__device__ __forceinline__ V3<R> divs(V3<R> a, R t) {
  return mk(a.x / t, a.y / t, a.z / t);
}
template <typename R>
__device__ __forceinline__ R dot(V3<R> a, V3<R> b) {
  return a.x * b.x + a.y * b.y + a.z * b.z;  // vec.zig:20-22, left to right
}
template <typename R>
__device__ __forceinline__ R norm2(V3<R> a) {
  return a.x * a.x + a.y * a.y + a.z * a.z;
}
template <typename R>
__device__ __forceinline__ V3<R> normalized(V3<R> v) {  // vec.zig:32-39
  const R n = sqrt(norm2(v));
  return (n == (R)0) ? v : divs(v, n);
}
template <typename R>
__device__ __forceinline__ V3<R> ld3(const R* p) {
  return mk(p[0], p[1], p[2]);
}

// ------------------------------------------------------------------ RNG --
// Zig 0.14 std.Random: SplitMix64 seeding of Xoshiro256 (xoshiro256++),
// Random.float(f64) / float(f32).  Re-seeded per (seed, pixel, sample).
struct Xo {
  uint64_t s0, s1, s2, s3;
};
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
__device__ __forceinline__ uint64_t sm_next(uint64_t& st) {
  st += 0x9e3779b97f4a7c15ULL;
  uint64_t z = st;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ void xo_seed(Xo& r, uint64_t key) {
  uint64_t st = key;
  r.s0 = sm_next(st);
  r.s1 = sm_next(st);
  r.s2 = sm_next(st);
  r.s3 = sm_next(st);
}
__device__ __forceinline__ uint64_t xo_next(Xo& r) {
  const uint64_t res = rotl64(r.s0 + r.s3, 23) + r.s0;
  const uint64_t t = r.s1 << 17;
  r.s2 ^= r.s0;
  r.s3 ^= r.s1;
  r.s1 ^= r.s2;
  r.s0 ^= r.s3;
  r.s2 ^= t;
  r.s3 = rotl64(r.s3, 45);
  return res;
}
__device__ __forceinline__ uint32_t clz64(uint64_t v) { return v ? (uint32_t)__clzll((long long)v) : 64u; }

__device__ __forceinline__ uint64_t f64_extra_lz(Xo& r) {  // taken with probability 2^-12
  uint64_t lz = 12;
  for (;;) {
    const uint64_t addl = clz64(xo_next(r));
    lz += addl;
    if (addl != 64) break;
    if (lz >= 1022) {
      lz = 1022;
      break;
    }
  }
  return lz;
}
__device__ __forceinline__ double rnd_f64(Xo& r) {
  const uint64_t v = xo_next(r);
  uint64_t lz = clz64(v);
  if (__builtin_expect(lz >= 12, 0)) lz = f64_extra_lz(r);
  const uint64_t bits = ((1022 - lz) << 52) | (v & ((1ULL << 52) - 1));
  return __longlong_as_double((long long)bits);
}
__device__ __forceinline__ uint32_t f32_extra_lz(Xo& r) {  // probability 2^-41
  uint32_t lz = 41 + clz64(xo_next(r));
  if (lz == 41 + 64) lz += (uint32_t)__clz((int)((uint32_t)xo_next(r) | 0x7FFu));
  return lz;
}
__device__ __forceinline__ float rnd_f32(Xo& r) {
  const uint64_t v = xo_next(r);
  uint32_t lz = clz64(v);
  if (__builtin_expect(lz >= 41, 0)) lz = f32_extra_lz(r);
  const uint32_t bits = ((126u - lz) << 23) | ((uint32_t)v & ((1u << 23) - 1));
  return __uint_as_float(bits);
}
template <typename R>
__device__ __forceinline__ R rnd(Xo& r);
template <>
__device__ __forceinline__ double rnd<double>(Xo& r) {
  return rnd_f64(r);
}
template <>
__device__ __forceinline__ float rnd<float>(Xo& r) {
  return rnd_f32(r);
}
template <typename R>
__device__ __forceinline__ R rrange(Xo& r, R mn, R mx) {  // rand.zig:18-20
  return mn + rnd<R>(r) * (mx - mn);
}

// ------------------------------------------------------------- kernel ----
// Scene tables read with a wave-uniform index are accessed through the
// constant address space (4): the compiler may then use scalar loads (s_load
// into SGPRs) although the kernel also stores to global memory.
#define RTW_CONST __attribute__((address_space(4)))
template <typename T>
__device__ __forceinline__ const RTW_CONST T* cptr(const T* p) {
  return (const RTW_CONST T*)(p);
}

template <typename R>
struct Lane {
  V3<R> o, d, T;
  R time;
  Xo rng;
  double sx, sy, sz;  // f64 chunk sum (main.zig:388-393 accumulates in f64)
  uint32_t px, ly, c, s, s_end, depth;
  int skip;
};

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Camera.getRay (main.zig:91-100) after the u,v jitter (main.zig:390-391).
template <typename R>
__device__ __forceinline__ void start_sample(const TraceArgs<R>& A, Lane<R>& L) {
  const uint32_t y = A.row_begin + L.ly * A.row_stride;  // image row (top-first)
  const uint32_t j = A.H - 1 - y;                        // reference row index
  const uint64_t pixel = (uint64_t)y * A.W + L.px;
  xo_seed(L.rng, A.seed_base ^ ((pixel << 24) | (uint64_t)L.s));
  const R u = ((R)L.px + rnd<R>(L.rng)) / ((R)A.W - (R)1);
  const R v = ((R)j + rnd<R>(L.rng)) / ((R)A.H - (R)1);
  R dx, dy;
  for (;;) {  // rand.zig:30-36; sqrt(x) >= 1 <=> x >= 1 for correctly rounded sqrt
    dx = rrange<R>(L.rng, (R)-1, (R)1);
    dy = rrange<R>(L.rng, (R)-1, (R)1);
    if (!(dx * dx + dy * dy + (R)0 * (R)0 >= (R)1)) break;
  }
  const V3<R> rd = mk(dx * A.lens_radius, dy * A.lens_radius, (R)0 * A.lens_radius);
  const V3<R> cu = ld3(A.cu), cv = ld3(A.cv), org = ld3(A.origin);
  const V3<R> offset = add(mul(cu, rd.x), mul(cv, rd.y));
  L.d = sub(sub(add(add(ld3(A.llc), mul(ld3(A.horizontal), u)), mul(ld3(A.vertical), v)), org), offset);
  L.o = add(org, offset);
  L.time = rrange<R>(L.rng, A.time0, A.time1);
  L.T = mk((R)1, (R)1, (R)1);
  L.depth = 0;
  L.skip = -1;
}

// f64 quadratic for a wide sphere in f32 mode (tierb_core.h TBF(test), wide branch).
__device__ __forceinline__ bool wide_test(const RTW_CONST double* w, uint32_t meta, const RTW_CONST double* tgd, V3<float> o,
                                          V3<float> d, float time, float tmin, float& tmax) {
  double cx = w[0], cy = w[1], cz = w[2];
  if (meta & kMoving) {
    const uint32_t g = (meta >> 2) & 63u;
    const double fr = ((double)time - tgd[2 * g]) / (tgd[2 * g + 1] - tgd[2 * g]);
    cx = cx + w[3] * fr;
    cy = cy + w[4] * fr;
    cz = cz + w[5] * fr;
  }
  const double ox = (double)o.x - cx, oy = (double)o.y - cy, oz = (double)o.z - cz;
  const double dx = d.x, dy = d.y, dz = d.z;
  const double ad = dx * dx + dy * dy + dz * dz;
  const double hb = ox * dx + oy * dy + oz * dz;
  const double c = (ox * ox + oy * oy + oz * oz) - w[6];
  const double disc = hb * hb - ad * c;
  if (disc < 0.0) return false;
  const double sq = sqrt(disc);
  double root = (-hb - sq) / ad;
  if (root < (double)tmin || (double)tmax < root) {
    root = (-hb + sq) / ad;
    if (root < (double)tmin || (double)tmax < root) return false;
  }
  tmax = (float)root;
  return true;
}

template <typename R, bool F32, bool STATS>
__global__ void __launch_bounds__(kTraceBlock) trace_kernel(TraceArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const SceneView<R> S = A.sc;
  // LDS copies of the per-lane lookup tables (winning sphere, its material).
  R* l_sph = reinterpret_cast<R*>(lds_raw);
  R* l_mat = l_sph + 8 * S.n;
  R* l_tg = l_mat + 8 * S.nm;
  uint32_t* l_meta = reinterpret_cast<uint32_t*>(l_tg + 2 * S.ng);
  uint32_t* l_kind = l_meta + S.n;
  for (uint32_t i = threadIdx.x; i < 8 * S.n; i += blockDim.x) l_sph[i] = S.sph[i];
  for (uint32_t i = threadIdx.x; i < 8 * S.nm; i += blockDim.x) l_mat[i] = S.mat[i];
  for (uint32_t i = threadIdx.x; i < 2 * S.ng; i += blockDim.x) l_tg[i] = S.tg[i];
  for (uint32_t i = threadIdx.x; i < S.n; i += blockDim.x) l_meta[i] = S.meta[i];
  for (uint32_t i = threadIdx.x; i < S.nm; i += blockDim.x) l_kind[i] = S.kind[i];
  __syncthreads();

  const uint32_t lid = lane_id();
  const uint32_t npix = A.row_count * A.W;
  const uint32_t units_per_tile = kTileW * kTileH * A.n_chunks;
  const R tmin = A.tmin;
  const R kInf = (R)__builtin_huge_val();

  Lane<R> L;
  L.px = L.ly = L.c = L.s = L.s_end = L.depth = 0;
  L.sx = L.sy = L.sz = 0.0;
  L.skip = -1;
  bool have_unit = false;  // lane owns a (pixel, chunk) unit
  bool have_ray = false;   // lane has a live path
  bool done = false;       // queue exhausted for this lane
  uint32_t qnext = 0, qend = 0;  // wave-uniform batch [qnext, qend)
  unsigned long long st_samples = 0, st_segments = 0, st_skipped = 0;

  for (;;) {
    // ---- 1. take units for lanes that need one (wave-uniform control) ----
    const bool need = !have_unit && !done;
    const uint64_t needmask = __ballot(need);
    if (needmask) {
      const uint32_t n = (uint32_t)__popcll(needmask);
      const uint32_t rank = mbcnt64(needmask);
      const uint32_t rem = qend - qnext;
      uint32_t base2 = 0;
      if (n > rem) {
        uint32_t b = 0;
        if (lid == 0) b = atomicAdd(A.counter, kBatch);
        base2 = __shfl(b, 0);
      }
      if (need) {
        const uint32_t unit = rank < rem ? qnext + rank : base2 + (rank - rem);
        if (unit >= A.total_units) {
          done = true;
        } else {
          const uint32_t tile = unit / units_per_tile;
          const uint32_t r = unit - tile * units_per_tile;
          const uint32_t c = r >> 6;
          const uint32_t l = r & 63u;
          const uint32_t ty = tile / A.tiles_x;
          const uint32_t tx = tile - ty * A.tiles_x;
          const uint32_t px = tx * kTileW + (l & 7u);
          const uint32_t ly = ty * kTileH + (l >> 3);
          if (px < A.W && ly < A.row_count) {  // else: padding unit, take another
            have_unit = true;
            L.px = px;
            L.ly = ly;
            L.c = c;
            L.s = c * A.chunk;
            L.s_end = min(L.s + A.chunk, A.spp);
            L.sx = L.sy = L.sz = 0.0;
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
      if (__all(done)) break;
      continue;
    }

    // ---- 2. new samples: per-sample RNG + camera ray ----
    if (have_unit && !have_ray) {
      start_sample<R>(A, L);
      have_ray = true;
    }

    // ---- 3. one bounce segment ----
    if (have_ray) {
      bool ended = false;
      V3<R> col = mk((R)0, (R)0, (R)0);
      if (L.depth == A.max_depth) {  // rayColor depth == 0 (main.zig:105-108)
        ended = true;
      } else {
        if (STATS) st_segments++;
        const R a = norm2(L.d);
        R tmax = kInf;
        int hit = -1;
        int tg_cur = -1;
        R frac = (R)0;
        // HittableList.hit (hittable.zig:231-244): every lane tests sphere k
        // together; the record comes through scalar loads.
        const RTW_CONST uint32_t* c_meta = cptr(S.meta);
        const RTW_CONST R* c_sph = cptr(S.sph);
        const RTW_CONST R* c_tg = cptr(S.tg);
        for (uint32_t k = 0; k < S.n; ++k) {
          const uint32_t meta = c_meta[k];
          if constexpr (F32) {
            if (meta & kWide) {
              float tm = tmax;
              if ((int)k != L.skip && wide_test(cptr(S.wide_d) + 8 * k, meta, cptr(S.tg_d), L.o, L.d, L.time, tmin, tm)) {
                tmax = tm;
                hit = (int)k;
              }
              continue;
            }
          }
          const RTW_CONST R* sp = c_sph + 8 * k;
          R cx = sp[0], cy = sp[1], cz = sp[2];
          if (meta & kMoving) {  // MovingSphere.center (hittable.zig:219-221)
            const int g = (int)((meta >> 2) & 63u);
            if (g != tg_cur) {
              tg_cur = g;
              frac = (L.time - c_tg[2 * g]) / (c_tg[2 * g + 1] - c_tg[2 * g]);
            }
            cx = cx + sp[3] * frac;
            cy = cy + sp[4] * frac;
            cz = cz + sp[5] * frac;
          }
          const R ocx = L.o.x - cx, ocy = L.o.y - cy, ocz = L.o.z - cz;
          const R hb = ocx * L.d.x + ocy * L.d.y + ocz * L.d.z;
          const R cc = (ocx * ocx + ocy * ocy + ocz * ocz) - sp[6];
          const R disc = hb * hb - a * cc;
          bool cand = !(disc < (R)0);
          if (F32) cand = cand && ((int)k != L.skip);
          if (cand) {
            const R sq = sqrt(disc);
            R root = (-hb - sq) / a;
            bool ok = !(root < tmin || tmax < root);
            if (!ok) {
              root = (-hb + sq) / a;
              ok = !(root < tmin || tmax < root);
            }
            if (ok) {
              tmax = root;
              hit = (int)k;
            }
          }
        }
        if (STATS && L.skip >= 0) st_skipped++;

        if (hit < 0) {  // miss: background (main.zig:109-112)
          ended = true;
          col = mulv(L.T, ld3(A.bg));
        } else {
          // Hit record of the winner (hittable.zig:118-128, :189-198).
          const R* sp = l_sph + 8 * hit;
          const uint32_t meta = l_meta[hit];
          const V3<R> p = add(L.o, mul(L.d, tmax));
          V3<R> center = ld3(sp);
          if (meta & kMoving) {
            const uint32_t g = (meta >> 2) & 63u;
            const R fr = (L.time - l_tg[2 * g]) / (l_tg[2 * g + 1] - l_tg[2 * g]);
            center = add(center, mul(ld3(sp + 3), fr));
          }
          const V3<R> outward = divs(sub(p, center), sp[7]);
          const bool front = dot(outward, L.d) < (R)0;
          const V3<R> normal = front ? outward : mul(outward, (R)-1);
          const uint32_t mi = meta >> 8;
          const uint32_t kind = l_kind[mi];
          const R* mp = l_mat + 8 * mi;
          // Material.scatter (material.zig:22-29), lanes of one kind together.
          V3<R> ud = L.d;
          if (kind >= 2u) ud = normalized(L.d);  // metal / dielectric
          V3<R> rs = mk((R)0, (R)0, (R)0);
          if (kind <= 2u) {  // randomPointInUnitSphere (rand.zig:22-28)
            for (;;) {
              rs.x = rrange<R>(L.rng, (R)-1, (R)1);
              rs.y = rrange<R>(L.rng, (R)-1, (R)1);
              rs.z = rrange<R>(L.rng, (R)-1, (R)1);
              if (!(norm2(rs) >= (R)1)) break;
            }
          }
          V3<R> ndir, att;
          bool absorbed = false;
          if (kind <= 1u) {  // Lambertian (material.zig:44-52)
            ndir = add(normal, normalized(rs));
            if (fabs(ndir.x) < (R)1e-8 && fabs(ndir.y) < (R)1e-8 && fabs(ndir.z) < (R)1e-8) ndir = normal;
            att = ld3(mp);
            if (kind == 1u) {  // CheckerTexture.value (texture.zig:79-82)
              const R sines = sin((R)10 * p.x) * sin((R)10 * p.y) * sin((R)10 * p.z);
              if (sines < (R)0) att = ld3(mp + 3);
            }
          } else if (kind == 2u) {  // Metal (material.zig:59-65)
            const V3<R> refl = sub(ud, mul(normal, (R)2 * dot(ud, normal)));
            ndir = add(refl, mul(rs, mp[6]));
            att = ld3(mp);
            absorbed = !(dot(refl, normal) > (R)0);
          } else {  // Dielectric (material.zig:72-91)
            const R ir = mp[7];
            const R ratio = front ? (R)1 / ir : ir;
            const R cos_t = fmin(dot(mul(ud, (R)-1), normal), (R)1);
            const R sin_t = sqrt((R)1 - cos_t * cos_t);
            bool refr = false;
            if (ratio * sin_t <= (R)1) {
              const R r0 = ((R)1 - ratio) / ((R)1 + ratio);
              const R r1 = r0 * r0;
              const R x = (R)1 - cos_t;
              const R x2 = x * x;
              const R refl_p = r1 + ((R)1 - r1) * (x * (x2 * x2));  // Zig pow(x, 5.0)
              refr = refl_p < rnd<R>(L.rng);
            }
            if (refr) {  // refract (material.zig:116-121)
              const R ct = fmin(dot(mul(ud, (R)-1), normal), (R)1);
              const V3<R> perp = mul(add(ud, mul(normal, ct)), ratio);
              const V3<R> par = mul(normal, -sqrt(fabs((R)1 - norm2(perp))));
              ndir = add(perp, par);
            } else {
              ndir = sub(ud, mul(normal, (R)2 * dot(ud, normal)));
            }
            att = mk((R)1, (R)1, (R)1);
          }
          if (absorbed) {
            ended = true;  // emitted == 0 (material.zig:31-38)
          } else {
            L.T = mulv(L.T, att);
            if (F32) L.skip = (dot(ndir, outward) > (R)0) ? hit : -1;
            L.o = p;
            L.d = ndir;
            L.depth++;
          }
        }
      }
      if (ended) {
        L.sx += (double)col.x;
        L.sy += (double)col.y;
        L.sz += (double)col.z;
        L.s++;
        have_ray = false;
        if (STATS) st_samples++;
        if (L.s == L.s_end) {  // unit done: publish the chunk sum
          double* dst = A.partial + ((size_t)L.c * npix + (size_t)L.ly * A.W + L.px) * 3;
          dst[0] = L.sx;
          dst[1] = L.sy;
          dst[2] = L.sz;
          have_unit = false;
        }
      }
    }
  }
  if (STATS) {
    atomicAdd(A.stats + 0, st_samples);
    atomicAdd(A.stats + 1, st_segments);
    atomicAdd(A.stats + 2, st_skipped);
  }
}

// Chunk sums added in order, then main.zig:395-400 quantisation.
__global__ void __launch_bounds__(256) finalize_kernel(FinalizeArgs F) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < F.npix; i += gridDim.x * blockDim.x) {
    double t[3] = {0.0, 0.0, 0.0};
    for (uint32_t c = 0; c < F.n_chunks; ++c) {
      const double* p = F.partial + ((size_t)c * F.npix + i) * 3;
      t[0] += p[0];
      t[1] += p[1];
      t[2] += p[2];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double g = sqrt(t[k] * F.scale);
      const double cl = fmax(0.0, fmin(g, 0.999));
      F.rgb[(size_t)i * 3 + k] = (uint8_t)(256.0 * cl);
      if (F.mean) F.mean[(size_t)i * 3 + k] = (float)(t[k] * F.scale);
    }
  }
}

template <typename R, bool F32>
static hipError_t launch_trace(const TraceArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats) {
  if (stats)
    hipLaunchKernelGGL((trace_kernel<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else
    hipLaunchKernelGGL((trace_kernel<R, F32, false>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_trace_f64(const TraceArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats) {
  return launch_trace<double, false>(a, grid, lds, s, stats);
}
hipError_t launch_trace_f32(const TraceArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats) {
  return launch_trace<float, true>(a, grid, lds, s, stats);
}
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  const uint32_t grid = min((a.npix + 255u) / 256u, 4096u);
  hipLaunchKernelGGL(finalize_kernel, dim3(grid ? grid : 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

int trace_blocks_per_cu(int precision, size_t lds) {
  int nb = 0;
  hipError_t e;
  if (precision == 1)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, trace_kernel<float, true, false>, kTraceBlock, lds);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, trace_kernel<double, false, false>, kTraceBlock, lds);
  if (e != hipSuccess || nb <= 0) nb = 1;
  return nb;
}

}  // namespace rtwk
