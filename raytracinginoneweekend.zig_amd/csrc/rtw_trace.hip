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
//  * Per lane, one loop iteration = [take a unit] -> [start a sample: the
//    sample's counter-RNG block, camera ray] -> [one bounce segment].  Paths
//    of different length share the wave without padding to the longest.  The
//    default variant rotates the iteration so that the lens-disk points of the
//    new samples and the unit-ball points of the hits come from ONE
//    cooperative rejection pass (kVarMergedStart, below).
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

#include "rtw_device.hpp"

// (Round 4) The lane's state flags (have_unit, have_ray, done, shading) as bits of one
// u32 (rtw_device.hpp LaneFlag) instead of bools: as bools they were 64-bit
// lane masks in SGPRs for the whole loop, and at the 100-SGPR limit the loop
// spilled SGPRs to VGPR lanes and one 8-B pair to scratch.  Hot loop: 14 -> 6
// lane ops, 2 -> 1 scratch pairs; -1.4 % per configs[1] frame
// (profiles/r04/trace_lane_flags_ab.txt).

namespace rtwk {


// VAR (tuning variants, selected at launch): bit0 = sphere records from LDS
// instead of scalar loads; bit1 = unroll the sphere loop by 2; bit2 = ask for
// 4 waves per SIMD (VGPR budget 128); bit3 = 5 waves per SIMD (budget 96);
// bit4 = per-lane rejection loops instead of coop_reject; bit5 = coop_reject
// for the lens disk too; bit6 = no narrow-sphere pretest (every lane tests
// every sphere exactly); bit9 (512) = scene fields re-read from the kernel
// argument; bit10 (1024) = the loop's other argument fields too; bits 11-14 =
// phase-duplication measurement builds (RTW_MEASURE); rtw_device.hpp: 32768
// kVarFastSqrt, 65536 kVarYOnly, 131072 kVarR0Table, 262144 kVarMergedStart,
// 524288 kVarPreDraw, 1048576 kVarBatchDecode.  Defaults: rtw_capi.hip
// kernel_variant; A/B tables: profiles/r01/ab_*.txt.
template <typename R, bool F32, int MODE, int VAR>
__global__ void __launch_bounds__(kTraceBlock, (VAR & 8) ? 5 : ((VAR & 4) ? 4 : 1)) trace_kernel(TraceArgs<R> A) {
  constexpr bool STATS = MODE == 1;
  constexpr bool COOP = !(VAR & 16);               // unit-ball point (scatter)
  constexpr bool COOP_DISK = COOP && (VAR & 32);  // lens-disk point (camera ray)
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const SceneView<R> S = A.sc;
  // LDS: per-wave coop_reject slots, then copies of the per-lane lookup
  // tables (winning sphere, its material).
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  CoopSlots* slots = T.slots;

  const uint32_t lid = lane_id();
  // VAR kVarHomeLds: the lane's unit fields (pixel, chunk, sample end) and its
  // f64 chunk sum live in this wave's LDS home block (SoA, one entry per
  // lane) instead of 10 VGPRs held across the closest hit; they are touched
  // only when a unit starts or ends, a sample starts, or a path misses.
  constexpr bool HOME = (VAR & kVarHomeLds) != 0;
  double* h_sum = nullptr;    // [3][64]
  uint32_t* h_u32 = nullptr;  // px[64], ly[64], c[64], s_end[64]
  R* h_t = nullptr;           // kVarPathLds: T [3][64] (8-B slots)
  uint64_t* h_base = nullptr; // kVarUnitBase: the unit's RNG block base [64]
  R* h_pxj = nullptr;         // kVarUnitBase: its f64 pixel column and reference row [2][64] (8-B slots)
  uint64_t* h_rs = nullptr;   // kVarPathLds: RNG state [64]
  if constexpr (HOME) {
    const size_t off = (size_t)(reinterpret_cast<unsigned char*>(T.cpos + kClusterSlots * S.n_clusters) - lds_raw);
    constexpr size_t kPathB = (VAR & kVarPathLds) ? kPathLdsBytesPerWave : 0;
    constexpr size_t kHomeStride =
        kHomeLdsBytesPerWave + kPathB + ((VAR & kVarUnitBase) ? kUnitBaseLdsBytesPerWave : 0);
    unsigned char* hb = lds_raw + ((off + 7) & ~(size_t)7) + (threadIdx.x >> 6) * kHomeStride;
    h_sum = reinterpret_cast<double*>(hb);
    h_u32 = reinterpret_cast<uint32_t*>(hb + 3 * 64 * 8);
    h_t = reinterpret_cast<R*>(hb + 2560);
    h_rs = reinterpret_cast<uint64_t*>(hb + 2560 + 3 * 64 * 8);
    h_base = reinterpret_cast<uint64_t*>(hb + 2560 + kPathB);
    h_pxj = reinterpret_cast<R*>(hb + 2560 + kPathB + 64 * 8);
  }
  constexpr bool UBASE = HOME && (VAR & kVarUnitBase) != 0;
  constexpr bool PLDS = HOME && (VAR & kVarPathLds) != 0 && (VAR & kVarMergedStart) != 0;
  constexpr uint32_t TS = 8 / sizeof(R);  // (8-B slots: T component k of lane l at h_t[(k * 64 + l) * TS])
  auto t_load = [&]() -> V3<R> { return mk(h_t[lid * TS], h_t[(64 + lid) * TS], h_t[(128 + lid) * TS]); };
  auto t_store = [&](const V3<R>& v) {
    h_t[lid * TS] = v.x, h_t[(64 + lid) * TS] = v.y, h_t[(128 + lid) * TS] = v.z;
  };
  // VAR bit 10: the loop's kernel-argument fields are re-read where used
  // (scalar loads through a laundered kernarg pointer) instead of living in
  // SGPRs for the whole kernel: the SGPR budget is the limit (spills become
  // v_readlane/v_writelane VALU instructions).
#define RTW_KA(f) ((VAR & 1024) ? opaque(kargs<R>())->f : A.f)
  const R tmin = A.tmin;
  const R kInf = (R)__builtin_huge_val();

  Lane<R> L;
  L.px = L.ly = L.c = L.s = L.s_end = L.depth = 0;
  L.sx = L.sy = L.sz = 0.0;
  L.rs = 0;
  L.skip = -1;
  uint32_t lane_flags = 0u;  // (rtw_device.hpp LaneFlag)
  LaneFlag<1u> have_unit{lane_flags};
  LaneFlag<2u> have_ray{lane_flags};
  LaneFlag<4u> done{lane_flags};
  uint32_t qnext = 0, qend = 0;  // wave-uniform batch [qnext, qend)
  KStats st;
  if constexpr (MODE == 2) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st.t_last)::"memory");

  // (tile x, tile y, chunk) of the wave's current unit batch and of a newly
  // fetched one (VAR kVarBatchDecode; wave-uniform).
  uint32_t cur_tx = 0, cur_ty = 0, cur_c = 0, nb_tx = 0, nb_ty = 0, nb_c = 0;
  auto decode_batch = [&](uint32_t base, uint32_t& tx, uint32_t& ty, uint32_t& c) {
    const uint32_t b64 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(base >> 6));
    const uint32_t nc = RTW_KA(n_chunks), txs = RTW_KA(tiles_x);
    const uint32_t tile = b64 / nc;
    c = b64 - tile * nc;
    ty = tile / txs;
    tx = tile - ty * txs;
  };
  // ---- take units for lanes that need one (wave-uniform control) ----
  auto take_units = [&]() {
    const bool need = !have_unit && !done;
    const uint64_t needmask = __ballot(need);
    if (needmask) {
      const uint32_t n = (uint32_t)__popcll(needmask);
      const uint32_t rank = mbcnt64(needmask);
      const uint32_t rem = qend - qnext;
      uint32_t base2 = 0;
      if (n > rem) {
        uint32_t b = 0;
        if (lid == 0) b = atomicAdd(RTW_KA(counter), kBatch);
        base2 = __shfl(b, 0);
      }
      if constexpr ((VAR & kVarBatchDecode) != 0) {
        // A batch is 64 aligned units = one (tile, chunk): decoded once per
        // batch (wave-uniform) instead of two integer divisions per refill.
        if (n > rem)  // (a dealt batch is a 64-aligned batch in every order)
          decode_batch(dealt_unit(base2, *opaque(kargs<R>())) & ~63u, nb_tx, nb_ty, nb_c);
      }
      if (need) {
        const uint32_t unit = rank < rem ? qnext + rank : base2 + (rank - rem);
        if (unit >= RTW_KA(total_units)) {
          done = true;
        } else {
          uint32_t tx, ty, c;
          const uint32_t du = dealt_unit(unit, *opaque(kargs<R>()));
          const uint32_t l = du & 63u;
          if constexpr ((VAR & kVarBatchDecode) != 0) {
            const bool in_cur = rank < rem;
            tx = in_cur ? cur_tx : nb_tx;
            ty = in_cur ? cur_ty : nb_ty;
            c = in_cur ? cur_c : nb_c;
          } else {
            const uint32_t units_per_tile = kTileW * kTileH * RTW_KA(n_chunks);
            const uint32_t tile = rtwm::udiv(du, RTW_KA(upt_m), RTW_KA(upt_sh));  // du / units_per_tile
            const uint32_t r = du - tile * units_per_tile;
            c = r >> 6;
            ty = rtwm::udiv(tile, RTW_KA(tx_m), RTW_KA(tx_sh));  // tile / tiles_x
            tx = tile - ty * RTW_KA(tiles_x);
          }
          const uint32_t px = tx * kTileW + (l & 7u);
          const uint32_t ly = ty * kTileH + (l >> 3);
          if (px < RTW_KA(W) && ly < RTW_KA(row_count)) {  // else: padding unit, take another
            have_unit = true;
            L.s = c * RTW_KA(chunk);
            if constexpr (HOME) {
              double z = 0.0;  // (laundered: a hoisted constant would hold registers)
              asm volatile("" : "+v"(z));
              h_u32[lid] = px;
              h_u32[64 + lid] = ly;
              h_u32[128 + lid] = c;
              h_u32[192 + lid] = min(L.s + RTW_KA(chunk), RTW_KA(spp));
              h_sum[lid] = h_sum[64 + lid] = h_sum[128 + lid] = z;
              if constexpr (UBASE) {  // start_sample_uv's per-pixel part, once per unit
                const uint32_t y = RTW_KA(row_begin) + ly * RTW_KA(row_stride);
                const uint64_t pixel = (uint64_t)y * RTW_KA(W) + px;
                h_base[lid] = RTW_KA(seed_base) + (pixel << 40) * kGamma;
                constexpr uint32_t TS = 8 / sizeof(R);
                h_pxj[lid * TS] = (R)px;
                h_pxj[(64 + lid) * TS] = (R)(RTW_KA(H) - 1 - y);
              }
            } else {
              L.px = px;
              L.ly = ly;
              L.c = c;
              L.s_end = min(L.s + RTW_KA(chunk), RTW_KA(spp));
              L.sx = L.sy = L.sz = 0.0;
            }
          }
        }
      }
      if (n > rem) {
        qnext = base2 + (n - rem);
        qend = base2 + kBatch;
        if constexpr ((VAR & kVarBatchDecode) != 0) cur_tx = nb_tx, cur_ty = nb_ty, cur_c = nb_c;
      } else {
        qnext += n;
      }
    }
  };

  // A finished sample joins its chunk sum (main.zig:393); a finished unit is
  // published.  (A miss added its colour; depth limit and absorption add 0.)
  auto finish_sample = [&]() {
    L.s++;
    have_ray = false;
    if (STATS) st.samples++;
    if constexpr (HOME) {
      if (L.s == h_u32[192 + lid]) {
        const uint32_t npix = RTW_KA(row_count) * RTW_KA(W);
        double* dst = RTW_KA(partial) +
                      ((size_t)h_u32[128 + lid] * npix + (size_t)h_u32[64 + lid] * RTW_KA(W) + h_u32[lid]) * 3;
        dst[0] = h_sum[lid];
        dst[1] = h_sum[64 + lid];
        dst[2] = h_sum[128 + lid];
        have_unit = false;
      }
    } else if (L.s == L.s_end) {
      const uint32_t npix = RTW_KA(row_count) * RTW_KA(W);
      double* dst = RTW_KA(partial) + ((size_t)L.c * npix + (size_t)L.ly * RTW_KA(W) + L.px) * 3;
      dst[0] = L.sx;
      dst[1] = L.sy;
      dst[2] = L.sz;
      have_unit = false;
    }
  };
  // One closest-hit step for a lane with a live ray (main.zig:103-112).
  // Returns 1 when the sample ended (depth limit or miss), 2 when the hit is
  // to be shaded.  (A result code, not two bool& outputs: the optimiser merged
  // their stores through a selected pointer, which put both flags in scratch
  // memory — a store + load per iteration on the critical path.)
  auto bounce = [&](uint32_t& kind, int& hit, R& tmax) -> int {
    if (L.depth == RTW_KA(max_depth)) {  // rayColor depth == 0 (main.zig:105-108)
      return 1;
    }
    if (STATS) st.segments++;
    if constexpr (STATS) {
      if (lid == (uint32_t)__builtin_ctzll(__ballot(true))) st.wave_iters++;
    }
    if constexpr (VAR & 512)  // scene fields re-read from the kernel argument (SGPR budget)
      closest_hit<R, F32, MODE, VAR>(opaque(kargs<R>())->sc, T, L, RTW_KA(tmin), RTW_KA(pre_k), lid, st, hit,
                                     tmax);
    else
      closest_hit<R, F32, MODE, VAR>(S, T, L, tmin, A.pre_k, lid, st, hit, tmax);
    if (hit < 0) {  // miss: background (main.zig:109-112)
      V3<R> tt = L.T;
      if constexpr (PLDS) tt = t_load();
      const V3<R> col = mulv(tt, ld3(opaque(kargs<R>())->bg));
      if constexpr (HOME) {
        h_sum[lid] += (double)col.x;
        h_sum[64 + lid] += (double)col.y;
        h_sum[128 + lid] += (double)col.z;
      } else {
        L.sx += (double)col.x;
        L.sy += (double)col.y;
        L.sz += (double)col.z;
      }
      return 1;
    }
    kind = T.kind[(T.meta[hit] >> 8) & 0xFFFu];
    return 2;
  };

  if constexpr ((VAR & kVarMergedStart) != 0) {
    // Rotated loop: [take units] -> [u, v of new samples] -> ONE coop pass:
    // lens-disk points (new samples) + unit-ball points (the Lambertian /
    // Metal hits of the previous step) -> [scatter; camera rays] -> [closest
    // hit].  A lane whose path missed starts its next sample in the next
    // iteration before that iteration's closest hit, as in the default loop;
    // each sample's draws are in the reference's order.
    LaneFlag<8u> shading{lane_flags};
    uint32_t kind = 0;
    int hit = -1;
    R tmax = kInf;
    for (;;) {
      RTW_STAMP(5)
      take_units();
      if (!__any(have_unit)) {
        if (__all(done)) break;
        continue;
      }
      RTW_STAMP(0)
      const bool ns = have_unit && !have_ray;
      if constexpr (PLDS) L.rs = h_rs[lid];
      R u = (R)0, v = (R)0;
      if (ns) {
        if constexpr (UBASE) {
          start_sample_uv_base<R>(kargs<R>(), L, h_base[lid], h_pxj[lid * TS], h_pxj[(64 + lid) * TS], u, v);
        } else {
          if constexpr (HOME) {
            L.px = h_u32[lid];
            L.ly = h_u32[64 + lid];
          }
          start_sample_uv<R>(kargs<R>(), L, u, v);
        }
      }
      RTW_STAMP(1)
      // dim: 3 unit ball (Lambertian, Metal), 1 the dielectric's draw, 2 lens disk (+ time)
      constexpr bool PRE = (VAR & kVarPreDraw) != 0;
      constexpr bool LDISK = (VAR & kVarLaneDisk) != 0;  // new samples' disk points from each lane's own loop
      const uint32_t dim = shading ? (kind <= 2u ? 3u : (PRE ? 1u : 0u)) : (ns && !LDISK ? 2u : 0u);
      R pt[3] = {(R)0, (R)0, (R)0}, raw = (R)0;
      if (__any(dim != 0u)) coop_reject_mixed<R>(dim, L.rs, pt, raw, slots, lid);
      RTW_STAMP(7)
      if (shading) {
        if constexpr (PLDS) L.T = t_load();
        if (scatter_hit<R, F32, VAR, PRE>(T, L, hit, tmax, kind, pt, raw)) finish_sample();  // absorbed
      }
      if (ns) {
        if constexpr (LDISK) {
          R dk[2];
          for (;;) {  // randomPointInUnitDisk (rand.zig:30-36)
            dk[0] = rrange_m11<R>(L.rs);
            dk[1] = rrange_m11<R>(L.rs);
            if (in_unit_ball<R, 2>(dk)) break;
          }
          start_sample_ray<R>(kargs<R>(), L, u, v, dk[0], dk[1]);
        } else {
          start_sample_ray<R, PRE>(kargs<R>(), L, u, v, pt[0], pt[1], raw);
        }
        have_ray = true;
      }
      if constexpr (PLDS) {
        if (shading || ns) t_store(L.T);
        h_rs[lid] = L.rs;
      }
      RTW_STAMP(8)
      shading = false;
      hit = -1;
      tmax = kInf;
      bool ended = false;
      if (have_ray) {
        const int b = bounce(kind, hit, tmax);
        ended = b == 1;
        shading = b == 2;
      }
      RTW_STAMP(3)
      if (ended) finish_sample();
    }
  } else {
  for (;;) {
    RTW_STAMP(5)
    take_units();
    if (!__any(have_unit)) {
      if (__all(done)) break;
      continue;
    }
    RTW_STAMP(0)

    // ---- 2. new samples: per-sample RNG block + camera ray ----
    {
      const bool ns = have_unit && !have_ray;
      if constexpr (COOP_DISK) {
        if (__any(ns)) {  // wave-uniform: coop_reject runs converged
          R u = (R)0, v = (R)0, dk[2];
          if (ns) start_sample_uv<R>(kargs<R>(), L, u, v);
          coop_reject<R, 2, true>(ns, L.rs, dk, slots, lid);
          if (ns) {
            start_sample_ray<R>(kargs<R>(), L, u, v, dk[0], dk[1]);
            have_ray = true;
          }
        }
      } else if (ns) {
        if constexpr ((VAR & 8192) != 0) {  // measurement: sample start twice (same image)
          Lane<R> L2 = L;
          asm volatile("" : "+v"(L2.px));
          R u2, v2, dk2[2];
          start_sample_uv<R>(kargs<R>(), L2, u2, v2);
          coop_reject<R, 2, false>(true, L2.rs, dk2, slots, lid);
          start_sample_ray<R>(kargs<R>(), L2, u2, v2, dk2[0], dk2[1]);
          asm volatile("" ::"v"(L2.d.x), "v"(L2.d.y), "v"(L2.d.z), "v"(L2.o.x), "v"(L2.o.y), "v"(L2.o.z),
                       "v"(L2.time), "v"(L2.rs));
        }
        R u, v, dk[2];
        start_sample_uv<R>(kargs<R>(), L, u, v);
        coop_reject<R, 2, false>(true, L.rs, dk, slots, lid);
        start_sample_ray<R>(kargs<R>(), L, u, v, dk[0], dk[1]);
        have_ray = true;
      }
    }
    RTW_STAMP(1)

    // ---- 3. one bounce segment ----
    // 3a. closest hit (lanes with a live ray); 3b. the unit-ball point for
    // diffuse/metal lanes (converged); 3c. hit record + scatter.  Only the
    // winner, its distance and its material cross 3b (register pressure).
    bool ended = false, shading = false;
    uint32_t kind = 0;
    int hit = -1;
    R tmax = kInf;
    if (have_ray) {
      const int b = bounce(kind, hit, tmax);
      ended = b == 1;
      shading = b == 2;
    }
    RTW_STAMP(3)
    {
      // randomPointInUnitSphere (rand.zig:22-28) for Lambertian and Metal.
      const bool nb = shading && kind <= 2u;
      R b3[3] = {(R)0, (R)0, (R)0};
      if constexpr ((VAR & 4096) != 0) {  // measurement: the unit-ball sampler twice (same image)
        if (__any(nb)) {
          uint64_t rs2 = L.rs;
          asm volatile("" : "+v"(rs2));
          R c3[3];
          coop_reject<R, 3, COOP>(nb, rs2, c3, slots, lid);
          asm volatile("" ::"v"(c3[0]), "v"(c3[1]), "v"(c3[2]), "v"(rs2));
        }
      }
      if (__any(nb)) coop_reject<R, 3, COOP>(nb, L.rs, b3, slots, lid);
      RTW_STAMP(7)
      if constexpr ((VAR & 16384) != 0) {  // measurement: hit record + scatter twice (same image)
        if (shading) {
          Lane<R> L2 = L;
          asm volatile("" : "+v"(L2.o.x));
          const int e2 = scatter_hit<R, F32, VAR>(T, L2, hit, tmax, kind, b3) ? 1 : 0;
          asm volatile("" ::"v"(L2.d.x), "v"(L2.d.y), "v"(L2.d.z), "v"(L2.T.x), "v"(L2.T.y), "v"(L2.T.z),
                       "v"(L2.o.x), "v"(L2.o.y), "v"(L2.o.z), "v"(e2), "v"(L2.rs));
        }
      }
      if (shading) {
        if (scatter_hit<R, F32, VAR>(T, L, hit, tmax, kind, b3)) ended = true;
      }
    }
    RTW_STAMP(8)
    if (ended) finish_sample();
  }
  }  // default loop
  if (STATS) {
    atomicAdd(A.stats + 0, st.samples);
    atomicAdd(A.stats + 1, st.segments);
    atomicAdd(A.stats + 2, st.skipped);
    atomicAdd(A.stats + 3, st.candwave);
    atomicAdd(A.stats + 4, st.candlane);
    atomicAdd(A.stats + 5, st.disc);
    atomicAdd(A.stats + 6, st.wave_iters);
    atomicAdd(A.stats + 7, st.cull_lanes);
    atomicAdd(A.stats + 8, st.cull_iters);
    atomicAdd(A.stats + 11, st.cl_tests);
    atomicAdd(A.stats + 12, st.cl_skips);
  }
  if constexpr (MODE == 2) {
    RTW_STAMP(4)
    if (lid == 0)
      for (int i = 0; i < 10; ++i) atomicAdd(A.stats + 16 + i, (unsigned long long)st.ph[i]);
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

template <typename R, bool F32, int VAR>
static void launch_var(const TraceArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s, int mode) {
  if (mode == 1)
    hipLaunchKernelGGL((trace_kernel<R, F32, 1, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
#ifdef RTW_MEASURE  // per-phase s_memtime stamps (diagnostic)
  else if (mode == 2)
    hipLaunchKernelGGL((trace_kernel<R, F32, 2, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
#endif
  else
    hipLaunchKernelGGL((trace_kernel<R, F32, 0, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
}

// The product library holds ONE variant per precision (kDefaultVarF64 /
// kDefaultVarF32, rtw_internal.hpp).  The A/B variants of round 1
// (profiles/r01/ab_*.txt) are compiled only into the measurement build
// (-DRTW_MEASURE, tools/); any other value is refused (trace_variant_built).
#ifdef RTW_MEASURE
#define RTW_AB_VARIANTS(X)                                                                                     \
  X(0) X(1) X(5) X(9) X(16) X(24) X(32) X(36) X(20) X(68) X(72) X(40) X(4) X(8) X(516) X(1540) X(520) X(1544)  \
  X(33284) X(66052) X(131588) X(229892) X(197128) X(164356) X(131592) X(426500) X(393736) X(1999364)         \
  X(1966600) X(950792) X(1016324) X(2064900) X(918020) X(2564) X(4612) X(8708) X(16900)                    \
  X(950788) X(3047940) X(3048964) X(918024) /* round-1 f64 default (the r02 A/B baseline), round-2 default  \
                                     before bit 1024, round-2 f64 / f32 defaults (before kVarHomeLds) */
#endif

template <bool F32>
constexpr int default_var() {
  return F32 ? kDefaultVarF32 : kDefaultVarF64;
}

bool trace_variant_built(int precision, int var) {
  if (var == (precision == 1 ? kDefaultVarF32 : kDefaultVarF64)) return true;
#ifdef RTW_MEASURE
  switch (var) {
#define RTW_CASE(v) case v:
    RTW_AB_VARIANTS(RTW_CASE)
#undef RTW_CASE
    return true;
  }
#endif
  return false;
}

template <typename R, bool F32>
static hipError_t launch_trace(const TraceArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s, int mode,
                               int var) {
  if (var == default_var<F32>()) {
    launch_var<R, F32, default_var<F32>()>(a, grid, lds, s, mode);
    return hipGetLastError();
  }
#ifdef RTW_MEASURE
  switch (var) {
#define RTW_CASE(v) \
  case v: launch_var<R, F32, v>(a, grid, lds, s, mode); return hipGetLastError();
    RTW_AB_VARIANTS(RTW_CASE)
#undef RTW_CASE
  }
#endif
  return hipErrorInvalidValue;  // not built (rtw_capi.hip checks trace_variant_built first)
}

hipError_t launch_trace_f64(const TraceArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, int mode,
                            int var) {
  return launch_trace<double, false>(a, grid, lds, s, mode, var);
}
hipError_t launch_trace_f32(const TraceArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, int mode,
                            int var) {
  return launch_trace<float, true>(a, grid, lds, s, mode, var);
}
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s) {
  const uint32_t grid = min((a.npix + 255u) / 256u, 4096u);
  hipLaunchKernelGGL(finalize_kernel, dim3(grid ? grid : 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <typename R, bool F32, int VAR>
static int occ(size_t lds) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, trace_kernel<R, F32, 0, VAR>, kTraceBlock, lds) != hipSuccess)
    nb = 0;
  return nb;
}
// Resident workgroups per CU of a built variant; 0 for a variant not built.
int trace_blocks_per_cu(int precision, size_t lds, int var) {
  if (!trace_variant_built(precision, var)) return 0;
  int nb = 0;
  if (precision == 1 && var == kDefaultVarF32) nb = occ<float, true, kDefaultVarF32>(lds);
  else if (precision != 1 && var == kDefaultVarF64) nb = occ<double, false, kDefaultVarF64>(lds);
#ifdef RTW_MEASURE
  else switch (var) {
#define RTW_CASE(v) \
  case v: nb = precision == 1 ? occ<float, true, v>(lds) : occ<double, false, v>(lds); break;
    RTW_AB_VARIANTS(RTW_CASE)
#undef RTW_CASE
  }
#endif
  return nb > 0 ? nb : 1;
}

}  // namespace rtwk
