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
  bool have_unit = false;  // lane owns a (pixel, chunk) unit
  bool have_ray = false;   // lane has a live path
  bool done = false;       // queue exhausted for this lane
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
        if (n > rem) decode_batch(base2, nb_tx, nb_ty, nb_c);
      }
      if (need) {
        const uint32_t unit = rank < rem ? qnext + rank : base2 + (rank - rem);
        if (unit >= RTW_KA(total_units)) {
          done = true;
        } else {
          uint32_t tx, ty, c;
          const uint32_t l = unit & 63u;
          if constexpr ((VAR & kVarBatchDecode) != 0) {
            const bool in_cur = rank < rem;
            tx = in_cur ? cur_tx : nb_tx;
            ty = in_cur ? cur_ty : nb_ty;
            c = in_cur ? cur_c : nb_c;
          } else {
            const uint32_t units_per_tile = kTileW * kTileH * RTW_KA(n_chunks);
            const uint32_t tile = unit / units_per_tile;
            const uint32_t r = unit - tile * units_per_tile;
            c = r >> 6;
            ty = tile / RTW_KA(tiles_x);
            tx = tile - ty * RTW_KA(tiles_x);
          }
          const uint32_t px = tx * kTileW + (l & 7u);
          const uint32_t ly = ty * kTileH + (l >> 3);
          if (px < RTW_KA(W) && ly < RTW_KA(row_count)) {  // else: padding unit, take another
            have_unit = true;
            L.px = px;
            L.ly = ly;
            L.c = c;
            L.s = c * RTW_KA(chunk);
            L.s_end = min(L.s + RTW_KA(chunk), RTW_KA(spp));
            L.sx = L.sy = L.sz = 0.0;
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
    if (L.s == L.s_end) {
      const uint32_t npix = RTW_KA(row_count) * RTW_KA(W);
      double* dst = RTW_KA(partial) + ((size_t)L.c * npix + (size_t)L.ly * RTW_KA(W) + L.px) * 3;
      dst[0] = L.sx;
      dst[1] = L.sy;
      dst[2] = L.sz;
      have_unit = false;
    }
  };
  // One closest-hit step for a lane with a live ray (main.zig:103-112).
  auto bounce = [&](bool& ended, bool& shading, uint32_t& kind, int& hit, R& tmax) {
    if (L.depth == RTW_KA(max_depth)) {  // rayColor depth == 0 (main.zig:105-108)
      ended = true;
      return;
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
      const V3<R> col = mulv(L.T, ld3(opaque(kargs<R>())->bg));
      L.sx += (double)col.x;
      L.sy += (double)col.y;
      L.sz += (double)col.z;
      ended = true;
    } else {
      kind = T.kind[(T.meta[hit] >> 8) & 0xFFFu];
      shading = true;
    }
  };

  if constexpr ((VAR & kVarMergedStart) != 0) {
    // Rotated loop: [take units] -> [u, v of new samples] -> ONE coop pass:
    // lens-disk points (new samples) + unit-ball points (the Lambertian /
    // Metal hits of the previous step) -> [scatter; camera rays] -> [closest
    // hit].  A lane whose path missed starts its next sample in the next
    // iteration before that iteration's closest hit, as in the default loop;
    // each sample's draws are in the reference's order.
    bool shading = false;
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
      R u = (R)0, v = (R)0;
      if (ns) start_sample_uv<R>(kargs<R>(), L, u, v);
      RTW_STAMP(1)
      // dim: 3 unit ball (Lambertian, Metal), 1 the dielectric's draw, 2 lens disk (+ time)
      constexpr bool PRE = (VAR & kVarPreDraw) != 0;
      const uint32_t dim = shading ? (kind <= 2u ? 3u : (PRE ? 1u : 0u)) : (ns ? 2u : 0u);
      R pt[3] = {(R)0, (R)0, (R)0}, raw = (R)0;
      if (__any(dim != 0u)) coop_reject_mixed<R>(dim, L.rs, pt, raw, slots, lid);
      RTW_STAMP(7)
      if (shading) {
        if (scatter_hit<R, F32, VAR, PRE>(T, L, hit, tmax, kind, pt, raw)) finish_sample();  // absorbed
      }
      if (ns) {
        start_sample_ray<R, PRE>(kargs<R>(), L, u, v, pt[0], pt[1], raw);
        have_ray = true;
      }
      RTW_STAMP(8)
      shading = false;
      hit = -1;
      tmax = kInf;
      bool ended = false;
      if (have_ray) bounce(ended, shading, kind, hit, tmax);
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
    if (have_ray) bounce(ended, shading, kind, hit, tmax);
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
#ifndef RTW_ISA_QUICK  // (register-pressure experiments: product variants only)
  if (mode == 1)
    hipLaunchKernelGGL((trace_kernel<R, F32, 1, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (mode == 2)
    hipLaunchKernelGGL((trace_kernel<R, F32, 2, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else
#endif
    hipLaunchKernelGGL((trace_kernel<R, F32, 0, VAR>), dim3(grid), dim3(kTraceBlock), lds, s, a);
}
template <typename R, bool F32>
static hipError_t launch_trace(const TraceArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s, int mode,
                               int var) {
  switch (var) {
#ifndef RTW_ISA_QUICK
    case 1: launch_var<R, F32, 1>(a, grid, lds, s, mode); break;
    case 5: launch_var<R, F32, 5>(a, grid, lds, s, mode); break;
    case 9: launch_var<R, F32, 9>(a, grid, lds, s, mode); break;
    case 16: launch_var<R, F32, 16>(a, grid, lds, s, mode); break;
    case 24: launch_var<R, F32, 24>(a, grid, lds, s, mode); break;
    case 32: launch_var<R, F32, 32>(a, grid, lds, s, mode); break;
    case 36: launch_var<R, F32, 36>(a, grid, lds, s, mode); break;
    case 20: launch_var<R, F32, 20>(a, grid, lds, s, mode); break;
    case 68: launch_var<R, F32, 68>(a, grid, lds, s, mode); break;
    case 72: launch_var<R, F32, 72>(a, grid, lds, s, mode); break;
    case 40: launch_var<R, F32, 40>(a, grid, lds, s, mode); break;
#endif
    case 4: launch_var<R, F32, 4>(a, grid, lds, s, mode); break;
    case 8: launch_var<R, F32, 8>(a, grid, lds, s, mode); break;
    case 516: launch_var<R, F32, 516>(a, grid, lds, s, mode); break;
    case 1540: launch_var<R, F32, 1540>(a, grid, lds, s, mode); break;
    case 520: launch_var<R, F32, 520>(a, grid, lds, s, mode); break;
    case 1544: launch_var<R, F32, 1544>(a, grid, lds, s, mode); break;
    case 33284: launch_var<R, F32, 33284>(a, grid, lds, s, mode); break;
    case 66052: launch_var<R, F32, 66052>(a, grid, lds, s, mode); break;
    case 131588: launch_var<R, F32, 131588>(a, grid, lds, s, mode); break;
    case 229892: launch_var<R, F32, 229892>(a, grid, lds, s, mode); break;
    case 197128: launch_var<R, F32, 197128>(a, grid, lds, s, mode); break;
    case 164356: launch_var<R, F32, 164356>(a, grid, lds, s, mode); break;
    case 131592: launch_var<R, F32, 131592>(a, grid, lds, s, mode); break;
    case 164356 + 262144: launch_var<R, F32, 164356 + 262144>(a, grid, lds, s, mode); break;
    case 131592 + 262144: launch_var<R, F32, 131592 + 262144>(a, grid, lds, s, mode); break;
    case 426500 + 524288: launch_var<R, F32, 426500 + 524288>(a, grid, lds, s, mode); break;
    case 393736 + 524288: launch_var<R, F32, 393736 + 524288>(a, grid, lds, s, mode); break;
    case 950788 + 1048576: launch_var<R, F32, 950788 + 1048576>(a, grid, lds, s, mode); break;
    case 918024 + 1048576: launch_var<R, F32, 918024 + 1048576>(a, grid, lds, s, mode); break;
    case 950792: launch_var<R, F32, 950792>(a, grid, lds, s, mode); break;
    case 950788 + 65536: launch_var<R, F32, 950788 + 65536>(a, grid, lds, s, mode); break;
    case 950788 + 65536 + 1048576: launch_var<R, F32, 950788 + 65536 + 1048576>(a, grid, lds, s, mode); break;
    case 918020: launch_var<R, F32, 918020>(a, grid, lds, s, mode); break;
#ifdef RTW_MEASURE  // phase-duplication measurement builds (tools/)
    case 516 + 2048: launch_var<R, F32, 516 + 2048>(a, grid, lds, s, mode); break;
    case 516 + 4096: launch_var<R, F32, 516 + 4096>(a, grid, lds, s, mode); break;
    case 516 + 8192: launch_var<R, F32, 516 + 8192>(a, grid, lds, s, mode); break;
    case 516 + 16384: launch_var<R, F32, 516 + 16384>(a, grid, lds, s, mode); break;
#endif
    default: launch_var<R, F32, 0>(a, grid, lds, s, mode); break;
  }
  return hipGetLastError();
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
int trace_blocks_per_cu(int precision, size_t lds, int var) {
  int nb = 0;
  switch (var) {
#define RTW_OCC_CASE(v) \
  case v: nb = precision == 1 ? occ<float, true, v>(lds) : occ<double, false, v>(lds); break;
#ifndef RTW_ISA_QUICK
    RTW_OCC_CASE(1) RTW_OCC_CASE(5) RTW_OCC_CASE(9) RTW_OCC_CASE(16) RTW_OCC_CASE(24) RTW_OCC_CASE(32) RTW_OCC_CASE(36) RTW_OCC_CASE(20) RTW_OCC_CASE(68) RTW_OCC_CASE(72) RTW_OCC_CASE(40)
#endif
    RTW_OCC_CASE(0) RTW_OCC_CASE(4) RTW_OCC_CASE(8) RTW_OCC_CASE(516) RTW_OCC_CASE(1540) RTW_OCC_CASE(520) RTW_OCC_CASE(1544) RTW_OCC_CASE(33284) RTW_OCC_CASE(66052) RTW_OCC_CASE(131588) RTW_OCC_CASE(229892) RTW_OCC_CASE(197128) RTW_OCC_CASE(164356) RTW_OCC_CASE(131592) RTW_OCC_CASE(426500) RTW_OCC_CASE(393736) RTW_OCC_CASE(950788) RTW_OCC_CASE(918024) RTW_OCC_CASE(1999364) RTW_OCC_CASE(1966600) RTW_OCC_CASE(950792) RTW_OCC_CASE(918020) RTW_OCC_CASE(1016324) RTW_OCC_CASE(2064900)
#ifdef RTW_MEASURE
    RTW_OCC_CASE(2564) RTW_OCC_CASE(4612) RTW_OCC_CASE(8708) RTW_OCC_CASE(16900)
#endif
#undef RTW_OCC_CASE
  }
  return nb > 0 ? nb : 1;
}

}  // namespace rtwk
