// rtw_device.hpp — device code shared by the megakernel (rtw_trace.hip) and
// the wavefront engine (rtw_wavefront.hip): Vec3 ops (vec.zig), the Tier-B
// counter RNG (rand.zig + Zig std.Random), the cooperative rejection sampler,
// Camera.getRay (main.zig:91-100), the closest-hit search over the sphere list
// (hittable.zig:95-244) and Material.scatter (material.zig:22-121).
// Arithmetic follows the reference operation by operation; every translation
// unit that includes this file is compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>

#include "rtw_cull.hpp"
#include "rtw_internal.hpp"
#include "rtw_math.hpp"

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
template <typename R>
__device__ __forceinline__ V3<R> ld3(const __attribute__((address_space(4))) R* p) {
  return mk(p[0], p[1], p[2]);
}

// sqrt of the hot path: rtwm::sqrt_rn (same bits as sqrt, fewer instructions)
// for f64 when VAR has kVarFastSqrt.
constexpr int kVarFastSqrt = 32768;
// Dielectric: Schlick's r0^2 for both ratios precomputed in the material
// record (rtw_capi.hip: doubles 0, 1 of a dielectric; its albedo is unused).
constexpr int kVarR0Table = 131072;
// Pretest: pairs flagged y-only (rtw_capi.hip cull_tg bit 16) skip the x/z
// centre updates.
constexpr int kVarYOnly = 65536;
// Trace loop rotated so that the lens-disk points of new samples and the
// unit-ball points of Lambertian / Metal hits come from ONE coop_reject_mixed
// pass per iteration (rtw_trace.hip).
constexpr int kVarMergedStart = 262144;
// With kVarMergedStart: the sample's time draw and the dielectric's draw are
// made inside the same cooperative pass (coop_reject_mixed `raw`).
constexpr int kVarPreDraw = 524288;
// Unit refill: each 64-unit batch's (tile, chunk) decoded once per batch.
constexpr int kVarBatchDecode = 1048576;
// kVarPathLds (with kVarHomeLds and kVarMergedStart): the lane's attenuation T and
// RNG state live in its LDS home block between the phases that use them
// (sampler, scatter, sample start, miss), so neither is held in VGPRs across
// the closest hit (measurement: within noise).
constexpr int kVarPathLds = 33554432;
// kVarUnitBase (with kVarHomeLds): the unit's RNG block base
// seed_base + (pixel << 40) * gamma and its f64 pixel column / reference row
// are made once per unit (home block); a sample's state is then
// base + s * (gamma << 16) — the same value as (((pixel << 24) | s) << 16) *
// gamma + seed_base mod 2^64, since s < 2^24 (rtw_validate_params) makes the
// | an addition — and u, v add the stored f64 coordinates (measurement:
// within noise).
constexpr int kVarUnitBase = 67108864;
// kVarLaneDisk (with kVarMergedStart): new samples' lens-disk points from each
// lane's own rejection loop after the cooperative pass, not inside it
// (measurement: 4.8 % slower, profiles/r06/mk_var_ab.txt).
constexpr int kVarLaneDisk = 134217728;
// f64 pretest over spatial clusters of narrow spheres (SceneView ccull...):
// a wave skips a cluster's member pretests when every lane's line provably
// misses the cluster's bounding sphere.
constexpr int kVarCluster = 2097152;
// Measurement only (phase duplication): the clustered path's survivor
// loop runs twice, the first pass's result discarded (same image).
constexpr int kVarDupSurvivors = 8388608;
// Megakernel: the lane's unit fields (pixel, chunk, sample end) and f64
// chunk sum live in LDS instead of VGPRs (rtw_trace.hip HomeLds).
constexpr int kVarHomeLds = kVarHomeLdsBit;
template <typename R, int VAR>
__device__ __forceinline__ R sqrt_k(R x) {
  if constexpr ((VAR & kVarFastSqrt) != 0 && sizeof(R) == 8)
    return rtwm::sqrt_rn(x);
  else
    return sqrt(x);
}

// ------------------------------------------------------------- work units --
// The unit a work-queue index deals.  Unit ids run over 8x8 pixel tiles in
// image-row order, top rows first, each tile's chunks in order (one 64-unit
// batch = one (tile, chunk)); order 1 deals them last-first.  Which lane runs
// a unit, and when, changes no bit of its chunk sum; the order moves which
// units run together and which end the launch (measured per engine:
// rtw_capi.hip fill_args, profiles/r03/unit_order_ab.txt).
template <typename A>
__device__ __forceinline__ uint32_t dealt_unit(uint32_t raw, const A& a) {
  return a.unit_order ? a.total_units - 1u - raw : raw;
}

// ------------------------------------------------------------------ RNG --
// Counter-based Tier-B generator over SplitMix64's Weyl sequence: sample
// (pixel p, sample s) owns the 2^16 Weyl states starting at
// base + (((p << 24) | s) << 16) * gamma; its draws are the mixer sm_mix of
// the next states, turned into reals by Zig's Random.float
// (oracle/rtw_oracle.c tierb_state / ro_tb_mix / ro_sm_f64 / ro_sm_f32).
// Every draw is exactly one Weyl step: the rare extra words Random.float needs
// for a tiny value come from the draw's own extension stream (the Weyl states
// from state ^ kExt, same mixer), so draw k of a block sits at state
// W + (k + 1) * gamma and any lane can evaluate any draw (coop_reject).
constexpr uint64_t kGamma = 0x9e3779b97f4a7c15ULL;
constexpr uint64_t kExt = 0x5851F42D4C957F2DULL;
// z * c mod 2^64 on 32-bit lanes as three chained v_mad_u64_u32: the low
// product lo*c_lo, then the high word accumulated as lo32(hi*c_lo + ph) and
// lo32(lo*c_hi + that) (the laundering keeps each mad 64-bit, which the
// optimiser would otherwise narrow back to v_mul_lo_u32 + v_add3_u32: four
// instructions per product).  Same bits as the C multiply.
template <uint64_t C>
__device__ __forceinline__ uint64_t mul64c(uint64_t z) {
  const uint32_t lo = (uint32_t)z, hi = (uint32_t)(z >> 32);
  const uint64_t p = (uint64_t)lo * (uint32_t)C;
  uint64_t q = (uint64_t)hi * (uint32_t)C + (p >> 32);
  asm("" : "+v"(q));
  // q's high word is don't-care: only the low word of r is used, so q goes
  // in whole as the third product's addend (no zero-extension move)
  uint64_t r = (uint64_t)lo * (uint32_t)(C >> 32) + q;
  asm("" : "+v"(r));
  return (r << 32) | (uint32_t)p;
}
// z ^ (z >> k): one v_lshrrev_b64 + two v_xor_b32 (from 32-bit v_alignbit /
// shift / xor instead: 1.3 % slower, profiles/r04/xsh32_scalar_decide_ab.txt)
template <int K>
__device__ __forceinline__ uint64_t xsh(uint64_t z) {
  return z ^ (z >> K);
}
#ifndef RTW_RNG_MIX
#define RTW_RNG_MIX 10
#endif
#if RTW_RNG_MIX != 10 && !defined(RTW_MEASURE)
#error "RTW_RNG_MIX other than 10 (the Tier-B contract) exists only in the -DRTW_MEASURE build (A/B timing)"
#endif
// One Feistel half-round on the state's 32-bit words: t = x * M as ONE
// v_mad_u64_u32 (the full 64-bit product), the other word ^= hi(t), x = lo(t).
template <uint32_t M>
__device__ __forceinline__ void feistel(uint32_t& x, uint32_t& y) {
  const uint64_t t = (uint64_t)x * M;
  y ^= (uint32_t)(t >> 32);
  x = (uint32_t)t;
}
// The Tier-B mixer of a Weyl state (oracle/rtw_oracle.c ro_tb_mix).
//  10 (the contract since round 5): four Feistel half-rounds, the first on the
//     high word — 4 v_mad_u64_u32 + 4 v_xor_b32 (tests/native/rng_stats.c
//     mixer 10: passes the battery over 2^32 draws of the render's layout);
//   0: Zig's SplitMix64 (rounds 1-4): 2 x (3 v_mad_u64_u32) + 3 x 64-bit
//     xorshift;  1: its 32-bit-fold form (MurmurHash3 fmix64 with >> 32).
__device__ __forceinline__ uint64_t sm_mix(uint64_t z) {
#if RTW_RNG_MIX == 10
  uint32_t a = (uint32_t)(z >> 32), b = (uint32_t)z;
  feistel<0xD2511F53u>(a, b);
  feistel<0xCD9E8D57u>(b, a);
  feistel<0x9E3779B1u>(a, b);
  feistel<0x85EBCA6Bu>(b, a);
  return ((uint64_t)a << 32) | b;
#elif RTW_RNG_MIX == 1
  z = mul64c<0xff51afd7ed558ccdULL>(xsh<32>(z));
  z = mul64c<0xc4ceb9fe1a85ec53ULL>(xsh<32>(z));
  return xsh<32>(z);
#elif RTW_RNG_MIX == 2  // (measurement only: fails the battery's neighbour-pixel tests)
  return xsh<32>(mul64c<0xd6e8feb86659fd93ULL>(xsh<32>(z)));
#else
  z = mul64c<0xbf58476d1ce4e5b9ULL>(xsh<30>(z));
  z = mul64c<0x94d049bb133111ebULL>(xsh<27>(z));
  return xsh<31>(z);
#endif
}
__device__ __forceinline__ uint64_t sm_next(uint64_t& st) {
  st += kGamma;
  return sm_mix(st);
}
__device__ __forceinline__ uint32_t clz64(uint64_t v) { return v ? (uint32_t)__clzll((long long)v) : 64u; }

__device__ __forceinline__ uint32_t f64_long_lz(uint64_t draw_state) {  // probability 2^-12 per draw
  uint64_t st = draw_state ^ kExt;
  uint32_t lz = 12;
  for (;;) {
    const uint32_t addl = clz64(sm_next(st));
    lz += addl;
    if (addl != 64) break;
    if (lz >= 1022) {
      lz = 1022;
      break;
    }
  }
  return lz;
}
// Leading zeros of x as the hardware counts them (v_ffbh_u32: 0xFFFFFFFF for
// x == 0, a defined value, unlike __builtin_clz(0)); the callers override the
// x < 2^20 case (f64_long_lz), so only x != 0 values reach the result.
__device__ __forceinline__ uint32_t ffbh_u32(uint32_t x) {
  uint32_t r;
  asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// High word of Random.float(f64) for the drawn word's high half `hi` and its
// leading-zero count `lz`: in the common case (leading one in the top 12
// bits) three VALU ops — ffbh (clz without the zero fix: the rare branch
// overrides it), and_or for the mantissa and the exponent base, the exponent.
__device__ __forceinline__ uint32_t f64_hi_bits(uint32_t hi, uint32_t lz) {
  // ((1022 - lz) << 20) | (hi & 0xFFFFF) as one v_bfi_b32 on the exponent
  // field (the compiler turns the or into and + sub + add: 4 ops, not 3)
  const uint32_t e = (1022u - lz) << 20;
  uint32_t r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "s"(0x000FFFFFu), "v"(hi), "v"(e));
  return r;
}
__device__ __forceinline__ double rnd_f64(uint64_t& st) {  // Random.float(f64)
  const uint64_t v = sm_next(st);
  const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
  // exponent = 1022 - clz(v); mantissa = low 52 bits.  Common case: the
  // leading one is in the top 12 bits, i.e. in `hi`.
  uint32_t lz = ffbh_u32(hi);  // (hi < 2^20, incl. 0: overridden below)
  if (__builtin_expect(hi < 0x00100000u, 0)) lz = f64_long_lz(st);
  return __hiloint2double((int)f64_hi_bits(hi, lz), (int)lo);
}
__device__ __forceinline__ float rnd_f32(uint64_t& st) {  // Random.float(f32)
  const uint64_t v = sm_next(st);
  uint32_t lz = clz64(v);
  if (__builtin_expect(lz >= 41, 0)) {  // probability 2^-41
    uint64_t ext = st ^ kExt;
    lz = 41 + clz64(sm_next(ext));
    if (lz == 41 + 64) lz += (uint32_t)__clz((int)((uint32_t)sm_next(ext) | 0x7FFu));
  }
  const uint32_t bits = ((126u - lz) << 23) | ((uint32_t)v & ((1u << 23) - 1));
  return __uint_as_float(bits);
}
// Three consecutive draws (states s + gamma, s + 2 gamma, s + 3 gamma) as
// Random.float(f64) (rnd_f64 x 3, the same bits); the rare long-leading-zero
// fix-up (probability 3 * 2^-12) takes one branch for the three.  s2: the
// state after the second draw.
__device__ __forceinline__ void rnd3_f64(uint64_t s, double& a, double& b, double& c, uint64_t& s2) {
  const uint64_t t1 = s + kGamma, t2 = t1 + kGamma, t3 = t2 + kGamma;
  s2 = t2;
  const uint64_t v1 = sm_mix(t1), v2 = sm_mix(t2), v3 = sm_mix(t3);
  const uint32_t h1 = (uint32_t)(v1 >> 32), h2 = (uint32_t)(v2 >> 32), h3 = (uint32_t)(v3 >> 32);
  uint32_t z1 = ffbh_u32(h1), z2 = ffbh_u32(h2), z3 = ffbh_u32(h3);
  if (__builtin_expect(min(min(h1, h2), h3) < 0x00100000u, 0)) {
    if (h1 < 0x00100000u) z1 = f64_long_lz(t1);
    if (h2 < 0x00100000u) z2 = f64_long_lz(t2);
    if (h3 < 0x00100000u) z3 = f64_long_lz(t3);
  }
  a = __hiloint2double((int)f64_hi_bits(h1, z1), (int)(uint32_t)v1);
  b = __hiloint2double((int)f64_hi_bits(h2, z2), (int)(uint32_t)v2);
  c = __hiloint2double((int)f64_hi_bits(h3, z3), (int)(uint32_t)v3);
}
__device__ __forceinline__ void rnd3_f32(uint64_t s, float& a, float& b, float& c, uint64_t& s2) {
  uint64_t t = s;
  a = rnd_f32(t);
  b = rnd_f32(t);
  s2 = t;
  c = rnd_f32(t);
}
template <typename R>
__device__ __forceinline__ void rnd3(uint64_t s, R& a, R& b, R& c, uint64_t& s2) {
  if constexpr (sizeof(R) == 8)
    rnd3_f64(s, a, b, c, s2);
  else
    rnd3_f32(s, a, b, c, s2);
}

template <typename R>
__device__ __forceinline__ R rnd(uint64_t& st);
template <>
__device__ __forceinline__ double rnd<double>(uint64_t& st) {
  return rnd_f64(st);
}
template <>
__device__ __forceinline__ float rnd<float>(uint64_t& st) {
  return rnd_f32(st);
}
template <typename R>
__device__ __forceinline__ R rrange(uint64_t& st, R mn, R mx) {  // rand.zig:18-20
  return mn + rnd<R>(st) * (mx - mn);
}
// randomReal(-1, 1) = -1 + r*2: r*2 is exact, so one FMA rounds identically.
template <typename R>
__device__ __forceinline__ R rrange_m11(uint64_t& st) {
  return fma(rnd<R>(st), (R)2, (R)-1);
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
// A pointer the compiler cannot see through: loads through it are issued
// where they are written (not hoisted into loop-invariant SGPRs), which keeps
// the camera block out of the SGPR budget of the sphere loop.
template <typename T>
__device__ __forceinline__ const RTW_CONST T* opaque(const RTW_CONST T* p) {
  asm volatile("" : "+s"(p));
  return p;
}
// The kernel's only argument (TraceArgs) sits at offset 0 of the kernarg segment.
template <typename R>
__device__ __forceinline__ const RTW_CONST TraceArgs<R>* kargs() {
  return (const RTW_CONST TraceArgs<R>*)__builtin_amdgcn_kernarg_segment_ptr();
}

// ---------------------------------------------------- packed-f32 pretest --
// Two spheres per v_pk_fma_f32 (rtw_cull.hpp: the bound and the scalar
// statement of the same operations).  Record of pair p (64 B, scalar-loaded):
// {c.x, c.y, c.z, ndc.x, ndc.y, ndc.z, nr2, unused}, each as {sphere 2p, 2p+1}.
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 bc(float x) { return f2{x, x}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
struct PairRec {
  f2 v[8];
};
__device__ __forceinline__ PairRec ld_pair(const __attribute__((address_space(4))) f2* t, uint32_t p) {
  PairRec r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.v[i] = t[8 * p + i];
  return r;
}
// MOVING: 0 static, 1 moving, 2 moving along y only (ndc.x = ndc.z = 0 for
// both spheres: the x and z updates would add exact zeros).
template <int MOVING>
__device__ __forceinline__ f2 cull_pair(const PairRec& R_, f2 ox, f2 oy, f2 oz, f2 dx, f2 dy, f2 dz, f2 na, f2 k,
                                        f2 frac) {
  const f2* P = R_.v;
  f2 ocx = ox - P[0], ocy = oy - P[1], ocz = oz - P[2];
  if constexpr (MOVING == 1) ocx = pfma(P[3], frac, ocx);
  if constexpr (MOVING != 0) ocy = pfma(P[4], frac, ocy);
  if constexpr (MOVING == 1) ocz = pfma(P[5], frac, ocz);
  const f2 hb = pfma(ocz, dz, pfma(ocy, dy, ocx * dx));
  const f2 cc = pfma(ocz, ocz, pfma(ocy, ocy, pfma(ocx, ocx, P[6])));
  return pfma(na, cc, pfma(hb, hb, k));
}

// The same bound with the lane's broadcast operands held two to a 64-bit
// register pair: {ox, oy}, {oz, dx}, {dy, dz}, {na, k} (8 VGPRs instead of 16
// for bc() pairs, which hold one value twice).  Each VOP3P operand names the
// 32-bit half it broadcasts by op_sel / op_sel_hi (lo: 0 / 0, hi: 1 / 1).  The
// same operations in the same order as cull_pair, so the same bits; inline
// asm because the compiler materialises a broadcast as a register pair.
// KP: the pair holding k (its half KH: 0 lo, 1 hi).
struct CullPairs {
  f2 oxy, ozdx, dyz, nk;
};
__device__ __forceinline__ CullPairs cull_pairs(float ox, float oy, float oz, float dx, float dy, float dz, float na,
                                                float k) {
  return {f2{ox, oy}, f2{oz, dx}, f2{dy, dz}, f2{na, k}};
}
// {a[H], a[H]} - p (p: an SGPR pair of the record)
template <int H>
__device__ __forceinline__ f2 pk_bsub(f2 a, f2 p) {
  f2 r;
  if constexpr (H == 0)
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "s"(p));
  else
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "s"(p));
  return r;
}
// x * {b[1], b[1]}
__device__ __forceinline__ f2 pk_mul_bhi(f2 x, f2 b) {
  f2 r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1]" : "=v"(r) : "v"(x), "v"(b));
  return r;
}
// x * {b[H], b[H]} + c
template <int H>
__device__ __forceinline__ f2 pk_fma_b1(f2 x, f2 b, f2 c) {
  f2 r;
  if constexpr (H == 0)
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(x), "v"(b), "v"(c));
  else
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(x), "v"(b), "v"(c));
  return r;
}
// x * x + {c[H], c[H]}
template <int H>
__device__ __forceinline__ f2 pk_sq_b2(f2 x, f2 c) {
  f2 r;
  if constexpr (H == 0)
    asm("v_pk_fma_f32 %0, %1, %1, %2 op_sel_hi:[1,1,0]" : "=v"(r) : "v"(x), "v"(c));
  else
    asm("v_pk_fma_f32 %0, %1, %1, %2 op_sel:[0,0,1] op_sel_hi:[1,1,1]" : "=v"(r) : "v"(x), "v"(c));
  return r;
}
// {a[0], a[0]} * x + c
__device__ __forceinline__ f2 pk_fma_b0lo(f2 a, f2 x, f2 c) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "v"(a), "v"(x), "v"(c));
  return r;
}
// o - c of both spheres of a record (computed before the callers branch on the
// record's kind: as asm, the compiler would not share it between the branches)
struct CullOc {
  f2 x, y, z;
};
__device__ __forceinline__ CullOc cull_oc(const PairRec& R_, const CullPairs& C) {
  return {pk_bsub<0>(C.oxy, R_.v[0]), pk_bsub<1>(C.oxy, R_.v[1]), pk_bsub<0>(C.ozdx, R_.v[2])};
}
template <int MOVING, int KH = 1>
__device__ __forceinline__ f2 cull_pair_sel(const PairRec& R_, const CullOc& oc, const CullPairs& C, f2 kp, f2 frac) {
  const f2* P = R_.v;
  f2 ocx = oc.x, ocy = oc.y, ocz = oc.z;
  if constexpr (MOVING == 1) ocx = pfma(P[3], frac, ocx);
  if constexpr (MOVING != 0) ocy = pfma(P[4], frac, ocy);
  if constexpr (MOVING == 1) ocz = pfma(P[5], frac, ocz);
  const f2 hb = pk_fma_b1<1>(ocz, C.dyz, pk_fma_b1<0>(ocy, C.dyz, pk_mul_bhi(ocx, C.ozdx)));
  const f2 cc = pfma(ocz, ocz, pfma(ocy, ocy, pfma(ocx, ocx, P[6])));
  return pk_fma_b0lo(C.nk, cc, pk_sq_b2<KH>(hb, kp));
}

template <typename R>
struct Rec {  // one sphere record of the closest-hit loop
  uint32_t meta;
  R c[3], dc[3], r2;
};

template <typename R>
struct Lane {
  V3<R> o, d, T;
  R time;
  uint64_t rs;        // SplitMix64 Weyl state of the current sample
  double sx, sy, sz;  // f64 chunk sum (main.zig:388-393 accumulates in f64)
  uint32_t px, ly, c, s, s_end, depth;
  int skip;
};

// Wave votes on a bool, straight to the lane-mask builtin: HIP's __ballot /
// __any / __all take an int, and the bool -> int -> bool round trip costs a
// v_cndmask + v_cmp per vote where the predicate crosses a block.  Over the
// ACTIVE lanes, as __ballot / __any / __all.
__device__ __forceinline__ uint64_t wballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ bool wany(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ bool wall(bool p) { return __builtin_amdgcn_ballot_w64(!p) == 0; }
// Population count of a lane mask as two 32-bit counts (scalar s_bcnt1_i32_b32;
// the 64-bit form's i64 result turns compares of counts into VALU ops).
__device__ __forceinline__ uint32_t popc64(uint64_t m) {
  return (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32));
}
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ------------------------------------------------- cooperative rejection ----
// The reference's rejection loops (rand.zig:22-28 randomPointInUnitSphere,
// rand.zig:30-36 randomPointInUnitDisk) take the FIRST candidate inside the
// unit ball.  Per lane that is ~1.9 (ball) / ~1.3 (disk) candidates, but a
// wave waits for its unluckiest lane (~6.9 / ~3.6 wave iterations).  Because
// candidate q of a D-dim loop whose state is B uses the draws at states
// B + (D*q + i + 1) * gamma (one Weyl step per draw), the wave can instead
// deal the candidates of its still-pending lanes to ALL 64 lanes: with m
// pending lanes each gets c = 2^floor(log2(64/m)) candidates per round,
// evaluated in parallel; the owner takes the lowest accepted one.  Same
// candidate order, same result bits, ~3 rounds instead of ~7 iterations.
// Must be called in wave-converged control flow (every lane of the wave).
struct CoopSlots {
  uint64_t st[64];  // pending lane's state B, by rank
  uint32_t q[64];   // its next candidate index
};
constexpr size_t kCoopBytesPerWave = sizeof(CoopSlots);
static_assert(kCoopBytesPerWave * (kTraceBlock / 64) == kCoopLdsBytes, "rtw_internal.hpp kCoopLdsBytes");

// Lane (addr >> 2) & 63's value of x (ds_bpermute; __shfl without its
// width arithmetic).
__device__ __forceinline__ float bperm(uint32_t addr, float x) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute((int)addr, __float_as_int(x)));
}
__device__ __forceinline__ double bperm(uint32_t addr, double x) {
  const uint64_t b = (uint64_t)__double_as_longlong(x);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)(uint32_t)b);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)addr, (int)(uint32_t)(b >> 32));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <typename R, int D>
__device__ __forceinline__ bool in_unit_ball(const R (&x)[D]) {
  if constexpr (D == 2)
    return !(x[0] * x[0] + x[1] * x[1] + (R)0 * (R)0 >= (R)1);  // rand.zig:34: vec3(x, y, 0)
  else
    return !(x[0] * x[0] + x[1] * x[1] + x[2] * x[2] >= (R)1);  // rand.zig:26; sqrt(t) >= 1 <=> t >= 1
}

// One bit of a per-lane flag word, used like a bool: a lane's state flags kept
// as bits of one u32 (a VGPR) instead of bools, which the compiler holds as
// 64-bit lane masks in SGPRs for a whole loop (rtw_world.hip
// RTW_WORLD_LANE_FLAGS, rtw_trace.hip RTW_TRACE_LANE_FLAGS).
template <uint32_t BIT>
struct LaneFlag {
  uint32_t& w;
  __device__ __forceinline__ operator bool() const { return (w & BIT) != 0u; }
  __device__ __forceinline__ LaneFlag& operator=(bool v) {
    w = v ? (w | BIT) : (w & ~BIT);
    return *this;
  }
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <typename R, int D, bool COOP>
__device__ __forceinline__ void coop_reject(bool need, uint64_t& st, R (&x)[D], CoopSlots* slots, uint32_t lid) {
  if constexpr (!COOP) {  // the literal per-lane loop (tuning variant 16)
    if (need) {
      for (;;) {
#pragma unroll
        for (int i = 0; i < D; ++i) x[i] = rrange_m11<R>(st);
        if (in_unit_ball<R, D>(x)) break;
      }
    }
    return;
  }
  bool pending = false;
  if (need) {  // round 0: every lane its own first candidate
#pragma unroll
    for (int i = 0; i < D; ++i) x[i] = rrange_m11<R>(st);
    pending = !in_unit_ball<R, D>(x);
  }
  uint64_t P = __ballot(pending);
  uint32_t nextq = 0;  // candidates are counted from B = st
  while (P) {
    const uint32_t m = (uint32_t)__popcll(P);
    const uint32_t lc = (uint32_t)__clz((int)(m - 1u)) - 26u;  // c = 2^lc = 2^floor(log2(64/m)), c*m <= 64
    const uint32_t r = mbcnt64(P);
    if (pending) {
      slots->st[r] = st;
      slots->q[r] = nextq;
    }
    wave_lds_sync();
    const uint32_t orank = lid >> lc;
    bool ok = false;
    R y[D];
#pragma unroll
    for (int i = 0; i < D; ++i) y[i] = (R)0;
    if (orank < m) {
      uint64_t s = slots->st[orank] + (uint64_t)(D * (slots->q[orank] + (lid & ((1u << lc) - 1u)))) * kGamma;
#pragma unroll
      for (int i = 0; i < D; ++i) y[i] = rrange_m11<R>(s);
      ok = in_unit_ball<R, D>(y);
    }
    const uint64_t acc = __ballot(ok);
    wave_lds_sync();  // slots are rewritten next round
    const uint32_t first = (r << lc) & 63u;  // pending lanes: r*c < 64
    const uint64_t mine = (acc >> first) & (~0ull >> (64u - (1u << lc)));
    const uint32_t jj = (uint32_t)__builtin_ctzll(mine);  // (mine == 0: unused)
    const uint32_t addr = ((first + jj) & 63u) << 2;
    R z[D];
#pragma unroll
    for (int i = 0; i < D; ++i) z[i] = bperm(addr, y[i]);
    if (pending) {
      if (mine) {
#pragma unroll
        for (int i = 0; i < D; ++i) x[i] = z[i];
        st += (uint64_t)(D * (nextq + jj + 1u)) * kGamma;
        pending = false;
      } else {
        nextq += 1u << lc;
      }
    }
    P = __ballot(pending);
  }
}

// coop_reject for a MIX of requests in one converged pass: dim 3 =
// randomPointInUnitSphere (rand.zig:22-28), dim 2 = randomPointInUnitDisk
// (rand.zig:30-36), dim 1 = the next single draw (the dielectric's, read
// speculatively: the state is NOT advanced), dim 0 = no request.  The rounds
// are coop_reject's with the dimension carried per pending lane (slot q =
// dim << 24 | next candidate): every candidate evaluates three draws (SIMT),
// a disk candidate q of state B uses the first two, at B + (2q + i + 1) *
// gamma, and the owner advances its state by its own dimension — the same
// candidate and state as the lane's sequential loop.  x[2] is unspecified for
// dim 2.  `raw` returns Random.float of the draw right after the accepted
// disk candidate (the sample's time draw, main.zig:99, computed as the
// candidate's spare third draw; the state is not advanced past it) or, for
// dim 1, of the next draw.  Wave-converged only.
template <typename R>
__device__ __forceinline__ bool in_ball_dim(uint32_t dim, R x0, R x1, R x2) {
  return dim == 3u ? !(x0 * x0 + x1 * x1 + x2 * x2 >= (R)1)   // rand.zig:26
                   : !(x0 * x0 + x1 * x1 + (R)0 * (R)0 >= (R)1);  // rand.zig:34: vec3(x, y, 0)
}
template <typename R>
__device__ __forceinline__ void coop_reject_mixed(uint32_t dim, uint64_t& st, R (&x)[3], R& raw,
                                                  CoopSlots* slots, uint32_t lid) {
  bool pending = false;
  if (dim != 0u) {  // round 0: every requesting lane its own first candidate
    R r0, r1, r2;
    uint64_t s2;
    rnd3<R>(st, r0, r1, r2, s2);
    x[0] = fma(r0, (R)2, (R)-1);  // randomReal(-1, 1) (rrange_m11)
    x[1] = fma(r1, (R)2, (R)-1);
    x[2] = fma(r2, (R)2, (R)-1);
    raw = dim == 1u ? r0 : r2;
    st = dim == 3u ? s2 + kGamma : (dim == 2u ? s2 : st);
    pending = dim >= 2u && !in_ball_dim<R>(dim, x[0], x[1], x[2]);
  }
  uint64_t P = __ballot(pending);
  uint32_t nextq = 0;  // candidates are counted from B = st
  // (Round 0 with each pending lane's second candidate as well, before any
  // dealing round: 1,483 VALU per wave-iteration, 0.5 % slower;
  // profiles/r04/coop_round0_ab.txt.)
  while (P) {
    const uint32_t m = (uint32_t)__popcll(P);  // wave-uniform (scalar)
    // c = 2^lc = 2^floor(log2(64/m)) = 2^(6 - ceil(log2 m)) (c*m <= 64): one
    // scalar clz instead of a division (clz(0) = 32: m = 1 gives lc = 6)
    const uint32_t lc = (uint32_t)__clz((int)(m - 1u)) - 26u;
    const uint32_t r = mbcnt64(P);
    if (pending) {
      slots->st[r] = st;
      slots->q[r] = nextq | (dim << 24);
    }
    wave_lds_sync();
    // Every lane evaluates a candidate (lanes past the dealt ones repeat the
    // last pending lane's slot and never accept): no divergent branch, no
    // zero-initialised copies.
    const uint32_t orank = lid >> lc;
    const uint32_t ork = min(orank, m - 1u);
    const uint32_t qw = slots->q[ork];
    const uint32_t d = qw >> 24;
    const uint64_t sb = slots->st[ork] + (uint64_t)(d * ((qw & 0xFFFFFFu) + (lid & ((1u << lc) - 1u)))) * kGamma;
    R y0, y1, yraw;
    uint64_t s2;
    rnd3<R>(sb, y0, y1, yraw, s2);
    y0 = fma(y0, (R)2, (R)-1);
    y1 = fma(y1, (R)2, (R)-1);
    const R y2f = fma(yraw, (R)2, (R)-1);
    const bool ok = (orank < m) & in_ball_dim<R>(d, y0, y1, y2f);
    // dim 3 takes the third coordinate, dim 2 the spare third draw as its
    // time draw (x[2] is unspecified for dim 2, raw unused for dim 3)
    const R y2 = d == 3u ? y2f : yraw;
    const uint64_t acc = __ballot(ok);
    wave_lds_sync();  // slots are rewritten next round
    // the owner's c candidates are lanes [first, first + c): its lowest
    // accepted one (pending lanes: r*c < 64; the mask is wave-uniform)
    const uint32_t first = (r << lc) & 63u;
    const uint64_t mine = (acc >> first) & (~0ull >> (64u - (1u << lc)));
    const uint32_t jj = (uint32_t)__builtin_ctzll(mine);  // (mine == 0: unused)
    const uint32_t addr = ((first + jj) & 63u) << 2;     // ds_bpermute byte address of the source lane
    const R z0 = bperm(addr, y0), z1 = bperm(addr, y1), z2 = bperm(addr, y2);
    if (pending) {
      if (mine) {
        x[0] = z0;
        x[1] = z1;
        x[2] = z2;
        raw = z2;
        st += (uint64_t)(dim * (nextq + jj + 1u)) * kGamma;
        pending = false;
      } else {
        nextq += 1u << lc;
      }
    }
    P = __ballot(pending);
  }
}

// v / |v| with the three divisions done against RN(1/|v|) (rtw_math.hpp div_rn).
template <typename R, int VAR = 0>
__device__ __forceinline__ V3<R> normalized_rn(V3<R> v) {  // vec.zig:32-39
  const R n = sqrt_k<R, VAR>(norm2(v));
  if (n == (R)0) return v;
  const R y = (R)1 / n;
  return mk(rtwm::div_rn(v.x, n, y), rtwm::div_rn(v.y, n, y), rtwm::div_rn(v.z, n, y));
}

// Camera.getRay (main.zig:91-100) after the u,v jitter (main.zig:390-391).
// Part 1: the sample's RNG block and the u, v jitter (main.zig:390-391).
template <typename R>
__device__ __forceinline__ void start_sample_uv(const RTW_CONST TraceArgs<R>* Ap, Lane<R>& L, R& u, R& v) {
  const RTW_CONST TraceArgs<R>& A = *opaque(Ap);
  const uint32_t y = A.row_begin + L.ly * A.row_stride;  // image row (top-first)
  const uint32_t j = A.H - 1 - y;                        // reference row index
  const uint64_t pixel = (uint64_t)y * A.W + L.px;
  L.rs = A.seed_base + ((((pixel << 24) | (uint64_t)L.s)) << 16) * kGamma;
  u = rtwm::div_rn((R)L.px + rnd<R>(L.rs), (R)A.W - (R)1, A.inv_w1);
  v = rtwm::div_rn((R)j + rnd<R>(L.rs), (R)A.H - (R)1, A.inv_h1);
}
// start_sample_uv with the unit's precomputed base and coordinates (kVarUnitBase)
template <typename R>
__device__ __forceinline__ void start_sample_uv_base(const RTW_CONST TraceArgs<R>* Ap, Lane<R>& L, uint64_t base,
                                                     R px, R j, R& u, R& v) {
  const RTW_CONST TraceArgs<R>& A = *opaque(Ap);
  L.rs = base + (uint64_t)L.s * (kGamma << 16);
  u = rtwm::div_rn(px + rnd<R>(L.rs), (R)A.W - (R)1, A.inv_w1);
  v = rtwm::div_rn(j + rnd<R>(L.rs), (R)A.H - (R)1, A.inv_h1);
}
// Part 2, after the lens-disk point (rand.zig:30-36, coop_reject<R, 2>).
// PRE: the time draw was made by coop_reject_mixed (`traw`, the draw at
// state L.rs + gamma): use it and step the state past it.
template <typename R, bool PRE = false>
__device__ __forceinline__ void start_sample_ray(const RTW_CONST TraceArgs<R>* Ap, Lane<R>& L, R u, R v, R dx,
                                                 R dy, R traw = (R)0) {
  const RTW_CONST TraceArgs<R>& A = *opaque(Ap);
  const V3<R> rd = mk(dx * A.lens_radius, dy * A.lens_radius, (R)0 * A.lens_radius);
  const V3<R> cu = ld3(A.cu), cv = ld3(A.cv), org = ld3(A.origin);
  const V3<R> offset = add(mul(cu, rd.x), mul(cv, rd.y));
  L.d = sub(sub(add(add(ld3(A.llc), mul(ld3(A.horizontal), u)), mul(ld3(A.vertical), v)), org), offset);
  L.o = add(org, offset);
  if constexpr (PRE) {
    L.time = A.time0 + traw * (A.time1 - A.time0);  // rrange (rand.zig:18-20) of the same draw
    L.rs += kGamma;
  } else {
    L.time = rrange<R>(L.rs, A.time0, A.time1);
  }
  L.T = mk((R)1, (R)1, (R)1);
  L.depth = 0;
  L.skip = -1;
}

// f64 quadratic for a wide sphere in f32 mode (tierb_core.h TBF(test), wide
// branch): the roots are solved in f64 and rounded to f32 before any
// comparison, so a wide sphere competes with the others on f32 roots.
// Returns false when the line misses (disc < 0); else `root` is the sphere's
// effective root (root1 if root1 >= tmin, else root2).
__device__ __forceinline__ bool wide_root(const RTW_CONST double* w, uint32_t meta, const RTW_CONST double* tgd,
                                          V3<float> o, V3<float> d, float time, float tmin, float& root) {
  double cx = w[0], cy = w[1], cz = w[2];
  if (meta & kMoving) {
    const uint32_t g = (meta >> 2) & 63u;
    const double fr = ((double)time - tgd[4 * g]) / (tgd[4 * g + 1] - tgd[4 * g]);
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
  root = (float)((-hb - sq) / ad);
  if (root < tmin) root = (float)((-hb + sq) / ad);
  return true;
}

// The reference's literal closest-hit loop (hittable.zig:231-244 with
// Sphere/MovingSphere.hit's root selection), in list order, from LDS tables;
// used only for lanes that met a NaN in the grouped loops.
template <typename R, bool F32, typename SV>
__device__ __forceinline__ void seq_closest_hit(const SV& S, const R* l_sph, const R* l_rad,
                                             const uint32_t* l_meta, const R* l_tg, const uint32_t* l_perm,
                                             const Lane<R>& L, R a, R tmin, R& tmax, int& hit) {
  tmax = (R)__builtin_huge_val();
  hit = -1;
  for (uint32_t i = 0; i < S.n; ++i) {
    const uint32_t k = l_perm[i];
    const uint32_t meta = l_meta[k];
    if (F32 && (int)k == L.skip) continue;
    if constexpr (F32) {
      if (meta & kWide) {
        float root = 0.0f;
        if (!wide_root(cptr(S.wide_d) + 8 * k, meta, cptr(S.tg_d), L.o, L.d, L.time, tmin, root)) continue;
        if (root < tmin || tmax < root) continue;
        tmax = root;
        hit = (int)k;
        continue;
      }
    }
    const R* sp = l_sph + 8 * k;
    R cx = sp[0], cy = sp[1], cz = sp[2];
    if (meta & kMoving) {
      const uint32_t g = (meta >> 2) & 63u;
      const R fr = (L.time - l_tg[4 * g]) / (l_tg[4 * g + 1] - l_tg[4 * g]);
      cx = cx + sp[3] * fr;
      cy = cy + sp[4] * fr;
      cz = cz + sp[5] * fr;
    }
    const R ocx = L.o.x - cx, ocy = L.o.y - cy, ocz = L.o.z - cz;
    const R hb = ocx * L.d.x + ocy * L.d.y + ocz * L.d.z;
    const R cc = (ocx * ocx + ocy * ocy + ocz * ocz) - sp[6];
    const R disc = hb * hb - a * cc;
    if (disc < (R)0) continue;
    const R sq = sqrt(disc);
    R root = (-hb - sq) / a;
    if (root < tmin || tmax < root) {
      root = (-hb + sq) / a;
      if (root < tmin || tmax < root) continue;
    }
    tmax = root;
    hit = (int)k;
  }
  (void)l_rad;
}

// ------------------------------------------------------- LDS scene tables --
// Per-workgroup LDS copies of the per-lane lookup tables (winning sphere, its
// material, time groups), after the per-wave coop_reject slots.
template <typename R>
struct LdsTables {
  CoopSlots* slots;  // this wave's coop_reject slots
  R* sph;
  R* rad;
  R* mat;
  R* tg;
  uint32_t* meta;
  uint32_t* kind;
  uint32_t* perm;  // original list index -> table position
  uint32_t* cpos;  // clustered pretest: slot -> table position
};
template <typename R>
__device__ __forceinline__ LdsTables<R> stage_tables(const SceneView<R>& S, unsigned char* lds_raw) {
  LdsTables<R> T;
  T.slots = reinterpret_cast<CoopSlots*>(lds_raw) + (threadIdx.x >> 6);
  T.sph = reinterpret_cast<R*>(lds_raw + kCoopBytesPerWave * (kTraceBlock / 64));
  T.rad = T.sph + 8 * (S.n + 1);
  T.mat = T.rad + S.n;
  T.tg = T.mat + 8 * S.nm;
  T.meta = reinterpret_cast<uint32_t*>(T.tg + 4 * S.ng);
  T.kind = T.meta + S.n + 1;
  T.perm = T.kind + S.nm;
  T.cpos = T.perm + S.n;
  for (uint32_t i = threadIdx.x; i < 8 * (S.n + 1); i += blockDim.x) T.sph[i] = S.sph[i];
  for (uint32_t i = threadIdx.x; i < S.n; i += blockDim.x) T.rad[i] = S.rad[i];
  for (uint32_t i = threadIdx.x; i < 8 * S.nm; i += blockDim.x) T.mat[i] = S.mat[i];
  for (uint32_t i = threadIdx.x; i < 4 * S.ng; i += blockDim.x) T.tg[i] = S.tg[i];
  for (uint32_t i = threadIdx.x; i < S.n + 1; i += blockDim.x) T.meta[i] = S.meta[i];
  for (uint32_t i = threadIdx.x; i < S.nm; i += blockDim.x) T.kind[i] = S.kind[i];
  for (uint32_t i = threadIdx.x; i < S.n; i += blockDim.x) T.perm[i] = S.perm[i];
  for (uint32_t i = threadIdx.x; i < kClusterSlots * S.n_clusters; i += blockDim.x) T.cpos[i] = S.cpos[i];
  __syncthreads();
  return T;
}

// Kernel statistics (MODE 1) and diagnostic phase stamps (MODE 2: s_memtime
// between phases, summed per wave in SGPRs; never part of the product
// build's timing, rtw_render_counts).
struct KStats {
  unsigned long long samples = 0, segments = 0, skipped = 0;
  unsigned long long candwave = 0, candlane = 0, disc = 0, wave_iters = 0;
  unsigned long long cull_lanes = 0, cull_iters = 0;
  unsigned long long cl_tests = 0, cl_skips = 0;  // clustered pretest: (wave, cluster) pairs, skipped ones
  uint64_t ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t t_last = 0;
};
#define RTW_STAMP(slot)                                                          \
  if constexpr (MODE == 2) {                                                     \
    __builtin_amdgcn_sched_barrier(0);                                           \
    uint64_t t_;                                                                 \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                           \
    st.ph[slot] += t_ - st.t_last;                                               \
    st.t_last = t_;                                                              \
  }

// ------------------------------------------------------------ closest hit --
// HittableList.hit (hittable.zig:231-244) over Sphere/MovingSphere.hit
// (hittable.zig:95-131, :165-201) for lane L's ray; returns the table position
// of the winner in `hit` (-1: miss) and its root in `tmax`.  `tmax` must be
// +inf and `hit` -1 on entry.  Wave-converged control is NOT required, but the
// wide-sphere and pretest loops are wave-uniform (scalar-loaded records).
// VAR: rtw_trace.hip trace_kernel tuning bits (1, 2, 64 are read here).
// SV: SceneView<R> (a copy in registers) or `const RTW_CONST SceneView<R>`
// (the kernel argument itself, re-read with scalar loads where used: keeps
// the scene fields out of the SGPR budget of the rest of the loop).
template <typename R, bool F32, int MODE, int VAR, typename SV>
__device__ __forceinline__ void closest_hit(const SV& S, const LdsTables<R>& T, const Lane<R>& L, R tmin,
                                            R pre_k, uint32_t lid, KStats& st, int& hit, R& tmax) {
  constexpr bool STATS = MODE == 1;
  constexpr bool CULL = !(VAR & 64);  // packed-f32 pretest for narrow spheres
  constexpr int kSphUnroll = (VAR & 2) ? 2 : 1;
  const R a = norm2(L.d);
  const R inv_a = (R)1 / a;          // RN(1/a): roots via div_rn
  const R pre_lim = pre_k * a;     // "both roots behind" prefilter bound
  int tg_cur = -1;
  R frac = (R)0;
  const RTW_CONST uint32_t* c_meta = cptr(S.meta);
  const RTW_CONST R* c_sph = cptr(S.sph);
  const RTW_CONST R* c_tg = cptr(S.tg);
  // HittableList.hit (hittable.zig:231-244): every lane tests sphere k
  // together; the record comes through scalar loads.
  // Closest hit.  The reference's sequential HittableList.hit returns the
  // sphere of minimal effective root (root1 if root1 >= tmin, else root2;
  // root2 >= root1 always), ties to the LAST in list order — an
  // order-independent rule.  So the table is
  // grouped [static-wide | static | moving-wide | moving] and each group
  // runs as its own branch-free loop; ties compare original indices.
  int hit_orig = -1;
  bool nan_seen = false;
  auto accept = [&](R root, int pos, int orig) {
    if (root != root) nan_seen = true;  // NaN: sequential fallback below
    if (!(root < tmin) & ((root < tmax) | ((root == tmax) & (orig > hit_orig)))) {
      tmax = root;
      hit = pos;
      hit_orig = orig;
    }
  };
  auto test = [&](uint32_t k, uint32_t meta, R cx, R cy, R cz, R r2) {
    const R ocx = L.o.x - cx, ocy = L.o.y - cy, ocz = L.o.z - cz;
    const R hb = ocx * L.d.x + ocy * L.d.y + ocz * L.d.z;
    const R cc = (ocx * ocx + ocy * ocy + ocz * ocz) - r2;
    const R disc = hb * hb - a * cc;
    // Candidate unless disc < 0, or provably both roots < tmin: origin
    // outside (cc > 0) and sphere behind (hb > 0) give root1 <= 0 and
    // root2 <= ~2u*hb/a < tmin while hb < pre_k*a.
    // One compare on the hot path; ~97 % of tests end here.  A NaN disc
    // also enters (reference: `disc < 0` is false for NaN).
    if (!(disc < (R)0)) {
      // (bitwise &: no short-circuit branches)
      const bool pre = (hb > (R)0) & (cc > (R)0) & (hb < pre_lim);
      bool cand = !pre;
      if (F32) cand = cand & ((int)k != L.skip);
      if constexpr (STATS) {
        const uint64_t cm = __ballot(cand);
        if (cm && lid == (uint32_t)__builtin_ctzll(__ballot(true))) st.candwave++;
        st.candlane += cand ? 1 : 0;
        st.disc += 1;
      }
      if (cand) {
        const R sq = sqrt_k<R, VAR>(disc);
        R root = rtwm::div_rn(-hb - sq, a, inv_a);
        if (root < tmin) root = rtwm::div_rn(-hb + sq, a, inv_a);
        accept(root, (int)k, (int)(meta >> 20));
      }
    }
  };
  auto rec_at = [&](uint32_t k) {
    Rec<R> r;
    if constexpr (VAR & 1) {
      const R* sp = T.sph + 8 * k;
      r.meta = T.meta[k];
      r.c[0] = sp[0], r.c[1] = sp[1], r.c[2] = sp[2], r.dc[0] = sp[3], r.dc[1] = sp[4], r.dc[2] = sp[5];
      r.r2 = sp[6];
    } else {
      const RTW_CONST R* sp = c_sph + 8 * k;
      r.meta = c_meta[k];
      r.c[0] = sp[0], r.c[1] = sp[1], r.c[2] = sp[2], r.dc[0] = sp[3], r.dc[1] = sp[4], r.dc[2] = sp[5];
      r.r2 = sp[6];
    }
    return r;
  };
  // f32 mode: wide spheres (radius >= 100), solved in f64.
  if constexpr (F32) {
    auto wide_range = [&](uint32_t b, uint32_t e) {
      for (uint32_t k = b; k < e; ++k) {
        const uint32_t meta = c_meta[k];
        float root = 0.0f;
        if ((int)k != L.skip && wide_root(cptr(S.wide_d) + 8 * k, meta, cptr(S.tg_d), L.o, L.d, L.time, tmin, root))
          accept(root, (int)k, (int)(meta >> 20));
      }
    };
    wide_range(0, S.g_static_wide);
    wide_range(S.g_static, S.g_moving_wide);
  }
  // static spheres: records stream one step ahead (padding record at the end)
  auto static_range = [&](uint32_t b, uint32_t e) {
    if (b < e) {
      Rec<R> cur = rec_at(b);
#pragma unroll kSphUnroll
      for (uint32_t k = b; k < e; ++k) {
        const Rec<R> nxt = rec_at(k + 1);
        test(k, cur.meta, cur.c[0], cur.c[1], cur.c[2], cur.r2);
        cur = nxt;
      }
    }
  };
  // moving spheres: centre(t) = c0 + (c1 - c0) * frac (hittable.zig:219-221)
  auto moving_range = [&](uint32_t b, uint32_t e) {
    if (b < e) {
      Rec<R> cur = rec_at(b);
#pragma unroll kSphUnroll
      for (uint32_t k = b; k < e; ++k) {
        const Rec<R> nxt = rec_at(k + 1);
        const int g = (int)((cur.meta >> 2) & 63u);
        if (g != tg_cur) {  // wave-uniform: recomputed only when the time group changes
          tg_cur = g;
          frac = rtwm::div_rn(L.time - c_tg[4 * g], c_tg[4 * g + 1] - c_tg[4 * g], c_tg[4 * g + 2]);
        }
        test(k, cur.meta, cur.c[0] + cur.dc[0] * frac, cur.c[1] + cur.dc[1] * frac, cur.c[2] + cur.dc[2] * frac,
             cur.r2);
        cur = nxt;
      }
    }
  };
  if (!CULL || !S.cull_on) {
    static_range(F32 ? S.g_static_wide : 0u, S.g_static);
    moving_range(F32 ? S.g_moving_wide : S.g_static, S.n);
  } else {
    if constexpr (!F32) {  // wide spheres: exact, wave-uniform
      static_range(0u, S.g_static_wide);
      moving_range(S.g_static, S.g_moving_wide);
    }
    // Narrow spheres: the packed-f32 pretest (rtw_cull.hpp) proves
    // disc < 0 for most (lane, sphere) pairs; each lane then runs the
    // exact test only on the spheres it could not rule out.
    const float af = (float)a;
    const rtwc::LaneCull lc = rtwc::lane_cull((float)L.o.x, (float)L.o.y, (float)L.o.z, af, S.cull_cmax);
    const rtwc::LaneConst lk = rtwc::lane_const(af, lc.alpha, S.cull_rho);
#ifndef RTW_CULL_BC  // (the bc() pair form: -DRTW_CULL_BC, measurement builds)
    const CullPairs cp = cull_pairs((float)L.o.x, (float)L.o.y, (float)L.o.z, (float)L.d.x, (float)L.d.y, (float)L.d.z,
                                    lk.na, lk.k);
#define RTW_CULL_OC(rec) const CullOc oc_ = cull_oc(rec, cp)
#define RTW_CULL(M, rec, fr) cull_pair_sel<M>(rec, oc_, cp, cp.nk, fr)
#define RTW_CULL_K(M, rec, kp, fr) cull_pair_sel<M, 0>(rec, cull_oc(rec, cp), cp, kp, fr)
#else
    const f2 ox = bc((float)L.o.x), oy = bc((float)L.o.y), oz = bc((float)L.o.z);
    const f2 dx = bc((float)L.d.x), dy = bc((float)L.d.y), dz = bc((float)L.d.z);
    const f2 na = bc(lk.na), alpha = bc(lk.k);
#define RTW_CULL_OC(rec) (void)0
#define RTW_CULL(M, rec, fr) cull_pair<M>(rec, ox, oy, oz, dx, dy, dz, na, alpha, fr)
#define RTW_CULL_K(M, rec, kp, fr) cull_pair<M>(rec, ox, oy, oz, dx, dy, dz, na, kp, fr)
#endif
    const RTW_CONST f2* ct = reinterpret_cast<const RTW_CONST f2*>(cptr(S.cull));
    const RTW_CONST uint32_t* ctg = cptr(S.cull_tg);
    const RTW_CONST float* ctf = cptr(S.tg_f);
    const float tf = (float)L.time;
    const uint32_t np_static = S.n_sn >> 1;  // pairs with two static spheres
    int fr_g = -1;  // phase B: time group of fr_v
    R fr_v = (R)0;
    // The pretest of one 64-sphere block: bit 31-r of sk[h] set = sphere
    // base+32h+r proven to miss.
    auto pretest_block = [&](uint32_t base, uint32_t (&sk)[2]) {
      sk[0] = sk[1] = 0u;
      uint32_t tgp_cur = ~0u;
      f2 fr2 = bc(0.0f);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t p0 = (base >> 1) + 16u * h, p1 = min(p0 + 16u, (S.nn + 1u) >> 1);
        // pair records stream one step ahead (the table has a padding pair)
        if (p0 < p1) {
          PairRec cur = ld_pair(ct, p0);
          uint32_t tgp_nxt = ctg[p0];
          for (uint32_t p = p0; p < p1; ++p) {
            const PairRec nxt = ld_pair(ct, p + 1);
            const uint32_t tgp = tgp_nxt;
            tgp_nxt = ctg[p + 1];
            f2 x;
            RTW_CULL_OC(cur);
            if (p < np_static) {
              x = RTW_CULL(0, cur, fr2);
            } else {
              if ((tgp & 0xFFFFu) != tgp_cur) {  // wave-uniform
                tgp_cur = tgp & 0xFFFFu;
                const uint32_t g0 = tgp & 0xFFu, g1 = (tgp >> 8) & 0xFFu;
                fr2 = f2{(tf - ctf[4 * g0]) * ctf[4 * g0 + 2], (tf - ctf[4 * g1]) * ctf[4 * g1 + 2]};
              }
              if ((VAR & kVarYOnly) != 0 && (tgp >> 16) != 0u)
                x = RTW_CULL(2, cur, fr2);
              else
                x = RTW_CULL(1, cur, fr2);
            }
            sk[h] = __builtin_amdgcn_alignbit(sk[h], __float_as_uint(x.x), 31);
            sk[h] = __builtin_amdgcn_alignbit(sk[h], __float_as_uint(x.y), 31);
            cur = nxt;
          }
        }
        // fewer than 16 pairs: move sphere r of the chunk to bit 31 - r
        const uint32_t cnt = p1 > p0 ? 2u * (p1 - p0) : 0u;
        sk[h] = cnt == 0u ? 0u : (cnt == 32u ? sk[h] : sk[h] << (32u - cnt));
      }
    };
    // Per lane: the exact test on the survivors of a 64-slot block (bit 31-r
    // of m0 / m1 = slot base+r / base+32+r); `clustered`: slots of the
    // clustered tables (T.cpos), else the narrow order of the cull table.
    // (Dealing the survivors across the wave instead — owners list their
    // pairs in LDS, every lane tests one with its owner's ray via ds_bpermute
    // — was 18 % slower: profiles/r03/survivor_compaction_ab.txt.)
    auto run_survivors = [&](uint32_t m0, uint32_t m1, uint32_t base, bool clustered) {
        while (m0 | m1) {  // per lane: the exact test on the survivors
          if constexpr (STATS) {
            if (lid == (uint32_t)__builtin_ctzll(__ballot(true))) st.cull_iters++;
          }
          uint32_t r;
          if (m0) {
            r = __clz(m0);
            m0 &= ~(0x80000000u >> r);
          } else {
            r = __clz(m1);
            m1 &= ~(0x80000000u >> r);
            r += 32u;
          }
          const uint32_t j = base + r;
          const uint32_t k = clustered ? T.cpos[j] : (j < S.n_sn ? S.g_static_wide + j : S.g_moving_wide + (j - S.n_sn));
          const R* sp = T.sph + 8 * k;
          const uint32_t meta = T.meta[k];
          R cx = sp[0], cy = sp[1], cz = sp[2];
          if (meta & kMoving) {
            const int g = (int)((meta >> 2) & 63u);
            if (g != fr_g) {  // per lane: usually once per segment
              fr_g = g;
              fr_v = rtwm::div_rn(L.time - T.tg[4 * g], T.tg[4 * g + 1] - T.tg[4 * g], T.tg[4 * g + 2]);
            }
            cx = cx + sp[3] * fr_v;
            cy = cy + sp[4] * fr_v;
            cz = cz + sp[5] * fr_v;
          }
          test(k, meta, cx, cy, cz, sp[6]);
        }
    };
    bool clustered_done = false;
    if constexpr ((VAR & kVarCluster) != 0 && !F32) {
      if (S.cluster_on) {  // kernel argument: wave-uniform
        clustered_done = true;
        const f2 kcl = bc(lc.alpha * S.cull_rho_cl);
        const RTW_CONST f2* cct = reinterpret_cast<const RTW_CONST f2*>(cptr(S.ccull));
        const RTW_CONST f2* ccl = reinterpret_cast<const RTW_CONST f2*>(cptr(S.cclus));
        const RTW_CONST uint32_t* cctg = cptr(S.ccull_tg);
        const RTW_CONST uint32_t* cval = cptr(S.cvalid);
        constexpr uint32_t CS = kClusterSlots, CPB = 64u / kClusterSlots;  // slots per cluster, clusters per block
        for (uint32_t cb = 0; cb < S.n_clusters; cb += CPB) {  // one 64-slot block
          const uint32_t nb = min(CPB, S.n_clusters - cb);
          // cluster pretest (bounding spheres as static pair records): bit c = proven miss
          uint32_t cmiss = 0u;
          for (uint32_t q = 0; 2u * q < nb; ++q) {
            const f2 x = RTW_CULL_K(0, ld_pair(ccl, (cb >> 1) + q), kcl, bc(0.0f));
            cmiss |= ((__float_as_uint(x.x) >> 31) << (2u * q)) | ((__float_as_uint(x.y) >> 31) << (2u * q + 1u));
          }
          if (!lc.ok) cmiss = 0u;
          uint64_t sk64 = 0u;  // slot bits, cluster cb first (MSB side after the final shift)
          uint32_t tgp_cur = ~0u;
          f2 fr2 = bc(0.0f);
#pragma unroll 1
          for (uint32_t c = 0; c < nb; ++c) {
            constexpr uint32_t kAll = (1u << CS) - 1u;
            uint32_t b8 = kAll;  // every slot proven missed
            const bool need = __ballot(((cmiss >> c) & 1u) == 0u) != 0;  // some lane's line may meet the cluster
            if constexpr (STATS) {
              if (lid == (uint32_t)__builtin_ctzll(__ballot(true))) {
                st.cl_tests++;
                st.cl_skips += need ? 0u : 1u;
              }
            }
            if (need) {
              b8 = 0u;
              const uint32_t p0 = (cb + c) * (CS / 2u);
#pragma unroll
              for (uint32_t i = 0; i < CS / 2u; ++i) {
                const uint32_t p = p0 + i;
                const PairRec rec = ld_pair(cct, p);
                const uint32_t tgp = cctg[p];
                f2 x;
                RTW_CULL_OC(rec);
                if (tgp & (1u << 17)) {
                  x = RTW_CULL(0, rec, fr2);
                } else {
                  if ((tgp & 0xFFFFu) != tgp_cur) {  // wave-uniform
                    tgp_cur = tgp & 0xFFFFu;
                    const uint32_t g0 = tgp & 0xFFu, g1 = (tgp >> 8) & 0xFFu;
                    fr2 = f2{(tf - ctf[4 * g0]) * ctf[4 * g0 + 2], (tf - ctf[4 * g1]) * ctf[4 * g1 + 2]};
                  }
                  x = (tgp & (1u << 16)) ? RTW_CULL(2, rec, fr2) : RTW_CULL(1, rec, fr2);
                }
                b8 = __builtin_amdgcn_alignbit(b8, __float_as_uint(x.x), 31);
                b8 = __builtin_amdgcn_alignbit(b8, __float_as_uint(x.y), 31);
              }
              b8 = (b8 & kAll) | (((cmiss >> c) & 1u) ? kAll : 0u);
            }
            sk64 = (sk64 << CS) | b8;
          }
          sk64 <<= CS * (CPB - nb);
          const uint32_t sk[2] = {(uint32_t)(sk64 >> 32), (uint32_t)sk64};
          uint32_t m0 = cval[2u * (cb / CPB)], m1 = cval[2u * (cb / CPB) + 1u];
          if (lc.ok) {
            m0 &= ~sk[0];
            m1 &= ~sk[1];
          }
          if constexpr (STATS) st.cull_lanes += __popc(m0) + __popc(m1);
          RTW_STAMP(2)
          if constexpr ((VAR & kVarDupSurvivors) != 0) {  // measurement: the survivors' exact tests twice
            int h2 = hit, o2 = hit_orig;
            R t2 = tmax;
            bool n2 = nan_seen;
            uint32_t q0 = m0, q1 = m1;
            asm volatile("" : "+v"(q0), "+v"(q1));
            run_survivors(q0, q1, cb * CS, true);
            hit = h2, hit_orig = o2, tmax = t2, nan_seen = n2;
          }
          run_survivors(m0, m1, cb * CS, true);
          RTW_STAMP(6)
        }
      }
    }
    if (!clustered_done)
    for (uint32_t base = 0; base < S.nn; base += 64) {
      uint32_t sk[2];
      pretest_block(base, sk);
      if constexpr ((VAR & 2048) != 0) {  // measurement: the block twice (same image; round 1's phase costs)
        uint32_t base2 = base;
        asm volatile("" : "+s"(base2));
        uint32_t sk2[2];
        pretest_block(base2, sk2);
        asm volatile("" ::"v"(sk2[0]), "v"(sk2[1]));
      }
      const uint32_t rem = S.nn - base;  // real spheres in this block
      const uint32_t v0 = rem >= 32u ? ~0u : ~(~0u >> rem);
      const uint32_t v1 = rem >= 64u ? ~0u : (rem <= 32u ? 0u : ~(~0u >> (rem - 32u)));
      uint32_t m0 = v0, m1 = v1;
      if (lc.ok) {
        m0 &= ~sk[0];
        m1 &= ~sk[1];
      }
      if constexpr (STATS) st.cull_lanes += __popc(m0) + __popc(m1);
      RTW_STAMP(2)
      run_survivors(m0, m1, base, false);
      RTW_STAMP(6)
    }
  }
  // A NaN anywhere makes the reference's acceptance order-dependent:
  // redo such lanes with its literal sequential loop.
  if (__builtin_expect(__any(nan_seen), 0)) {
    if (nan_seen) seq_closest_hit<R, F32>(S, T.sph, T.rad, T.meta, T.tg, T.perm, L, a, tmin, tmax, hit);
  }
  if (STATS && L.skip >= 0) st.skipped++;
  RTW_STAMP(2)
}

// ---------------------------------------------------------------- scatter --
// Hit record of the winner + Material.scatter (material.zig:22-121) for lane
// L, given the unit-ball point b3 (Lambertian / Metal; coop_reject).  Returns
// true when the ray is absorbed (Metal, material.zig:64); else L's ray,
// attenuation product and depth move to the next segment.
// PRE: the dielectric's draw was made by coop_reject_mixed (`draw`, the draw
// at state L.rs + gamma); it is consumed only when the reference draws it.
// POINT: L.o already holds the hit point p = o + tmax * d (the wavefront's
// path form, made with these operations where the hit was found), tmax unused.
template <typename R, bool F32, int VAR = 0, bool PRE = false, bool POINT = false>
__device__ __forceinline__ bool scatter_hit(const LdsTables<R>& T, Lane<R>& L, int hit, R tmax, uint32_t kind,
                                            const R (&b3)[3], R draw = (R)0) {
  // Hit record of the winner (hittable.zig:118-128, :189-198).
  const R* sp = T.sph + 8 * hit;
  const uint32_t meta = T.meta[hit];
  const V3<R> p = POINT ? L.o : add(L.o, mul(L.d, tmax));  // ray.at(t) (ray.zig)
  V3<R> center = ld3(sp);
  if (meta & kMoving) {
    const uint32_t g = (meta >> 2) & 63u;
    const R fr = rtwm::div_rn(L.time - T.tg[4 * g], T.tg[4 * g + 1] - T.tg[4 * g], T.tg[4 * g + 2]);
    center = add(center, mul(ld3(sp + 3), fr));
  }
  const R rad = T.rad[hit], inv_r = sp[7];
  const V3<R> q = sub(p, center);
  const V3<R> outward = mk(rtwm::div_rn(q.x, rad, inv_r), rtwm::div_rn(q.y, rad, inv_r),
                           rtwm::div_rn(q.z, rad, inv_r));
  const bool front = dot(outward, L.d) < (R)0;
  const V3<R> normal = front ? outward : mul(outward, (R)-1);
  const R* mp = T.mat + 8 * ((meta >> 8) & 0xFFFu);
  // Material.scatter (material.zig:22-29), lanes of one kind together.
  // One normalisation per lane: the unit-ball point (Lambertian) or the
  // ray direction (Metal, Dielectric).
  const V3<R> rs = mk(b3[0], b3[1], b3[2]);
  const V3<R> nv = normalized_rn<R, VAR>(kind <= 1u ? rs : L.d);
  const V3<R> ud = nv;
  // Metal and Dielectric share reflect(ud, normal) (material.zig:112-114) and
  // its dot product (the wave runs both branches): the Dielectric's
  // dot(-ud, normal) (:75) is exactly -dun (negation commutes with rounding).
  const R dun = dot(ud, normal);
  const V3<R> refl = sub(ud, mul(normal, (R)2 * dun));
  V3<R> ndir, att;
  bool absorbed = false;
  if (kind <= 1u) {  // Lambertian (material.zig:44-52)
    ndir = add(normal, nv);
    if (fabs(ndir.x) < (R)1e-8 && fabs(ndir.y) < (R)1e-8 && fabs(ndir.z) < (R)1e-8) ndir = normal;
    att = ld3(mp);
    // CheckerTexture.value (texture.zig:79-82): only the sign matters.
    if (kind == 1u && rtwm::checker_odd((double)((R)10 * p.x), (double)((R)10 * p.y), (double)((R)10 * p.z)))
      att = ld3(mp + 3);
  } else if (kind == 2u) {  // Metal (material.zig:59-65)
    ndir = add(refl, mul(rs, mp[6]));
    att = ld3(mp);
    absorbed = !(dot(refl, normal) > (R)0);
  } else {  // Dielectric (material.zig:72-91); mp[6] = RN(1/ir)
    const R ir = mp[7];
    const R ratio = front ? mp[6] : ir;
    const R cos_t = fmin(-dun, (R)1);
    const R sin_t = sqrt_k<R, VAR>((R)1 - cos_t * cos_t);
    bool refr = false;
    if (ratio * sin_t <= (R)1) {
      R r1;
      if constexpr ((VAR & kVarR0Table) != 0) {
        r1 = front ? mp[0] : mp[1];  // host: RN(RN((1-ratio)/(1+ratio))^2) per ratio
      } else {
        const R r0 = ((R)1 - ratio) / ((R)1 + ratio);
        r1 = r0 * r0;
      }
      const R x = (R)1 - cos_t;
      const R x2 = x * x;
      const R refl_p = r1 + ((R)1 - r1) * (x * (x2 * x2));  // Zig pow(x, 5.0)
      if constexpr (PRE) {
        refr = refl_p < draw;
        L.rs += kGamma;
      } else {
        refr = refl_p < rnd<R>(L.rs);
      }
    }
    if (refr) {  // refract (material.zig:116-121); its cos_theta is cos_t
      const V3<R> perp = mul(add(ud, mul(normal, cos_t)), ratio);
      const V3<R> par = mul(normal, -sqrt_k<R, VAR>(fabs((R)1 - norm2(perp))));
      ndir = add(perp, par);
    } else {
      ndir = refl;
    }
    att = mk((R)1, (R)1, (R)1);
  }
  if (absorbed) return true;  // emitted == 0 (material.zig:31-38)
  {
    L.T = mulv(L.T, att);
    if (F32) L.skip = (dot(ndir, outward) > (R)0) ? hit : -1;
    L.o = p;
    L.d = ndir;
    L.depth++;
  }
  return false;
}

}  // namespace rtwk
