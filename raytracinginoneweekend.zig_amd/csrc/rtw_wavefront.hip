// rtw_wavefront.hip — the wavefront engine (BASELINE.json configs[3]): the
// reference's render loop + rayColor (main.zig:378-402, :103-122) as
// per-bounce kernels over SoA path queues in HBM.
//
//   generate : every home slot takes a (pixel, chunk) unit and starts its
//              first sample (Camera.getRay, main.zig:91-100) -> queue A
// A wave owns fixed queue segments of kSegCap paths for the whole frame
// (rtw_internal.hpp): compaction is wave-local, units come from a per-segment
// reservoir, and a segment stays on one XCD (fixed grid, persistent waves).
//   extend   : closest hit (HittableList.hit, hittable.zig:231-244) for every
//              path of the input queue -> (hit root, winner) per position
//   shade    : background on a miss (main.zig:109-112) or Material.scatter
//              (material.zig:22-121); a finished sample adds to its slot's
//              f64 chunk sum, a finished chunk publishes it and the slot takes
//              the next unit; the slot's next sample starts at once, so the
//              queue stays full until the units run out.  Live paths are
//              appended, in order, to the wave's segment of the output queue.
//
// Arithmetic: the same device functions as the megakernel (rtw_device.hpp),
// so every sample is bit-identical to the megakernel and the Tier-B oracle;
// chunk sums add a unit's samples in sample order (one slot owns a unit).
// Bytes per bounce segment: extend reads o, d, time (+ skip) and writes the
// hit; shade reads the whole path + hit and writes the whole path.
#include <hip/hip_runtime.h>

#include <cstddef>

#include "rtw_device.hpp"


namespace rtwk {


static_assert(offsetof(WfArgs<double>, t) == 0 && offsetof(WfArgs<float>, t) == 0,
              "kargs<R>() reads TraceArgs at kernarg offset 0");

template <typename R>
__device__ __forceinline__ void load_path(const PathBuf<R>& B, uint32_t i, Lane<R>& L, uint32_t& slot) {
  L.o = mk(B.ox[i], B.oy[i], B.oz[i]);
  L.d = mk(B.dx[i], B.dy[i], B.dz[i]);
  L.T = mk(B.tx[i], B.ty[i], B.tz[i]);
  L.time = B.tm[i];
  L.rs = B.rs[i];
  slot = B.slot[i];
  const uint32_t dsk = B.dsk[i];
  L.depth = dsk & 0xFFFFu;
  L.skip = (int)(dsk >> 16) - 1;
}
template <typename R>
__device__ __forceinline__ void store_path(const PathBuf<R>& B, uint32_t i, const Lane<R>& L, uint32_t slot) {
  B.ox[i] = L.o.x, B.oy[i] = L.o.y, B.oz[i] = L.o.z;
  B.dx[i] = L.d.x, B.dy[i] = L.d.y, B.dz[i] = L.d.z;
  B.tx[i] = L.T.x, B.ty[i] = L.T.y, B.tz[i] = L.T.z;
  B.tm[i] = L.time;
  B.rs[i] = L.rs;
  B.slot[i] = slot;
  B.dsk[i] = L.depth | ((uint32_t)(L.skip + 1) << 16);
}

// Unit id -> (px, output row ly, chunk c): 8x8 pixel tiles x chunks, the same
// numbering as the megakernel's queue (rtw_trace.hip step 1).
template <typename R>
__device__ __forceinline__ bool decode_unit(const TraceArgs<R>& A, uint32_t unit, uint32_t& px, uint32_t& ly,
                                            uint32_t& c) {
  const uint32_t upt = kTileW * kTileH * A.n_chunks;
  const uint32_t tile = rtwm::udiv(unit, A.upt_m, A.upt_sh);  // unit / upt
  const uint32_t r = unit - tile * upt;
  c = r >> 6;
  const uint32_t l = r & 63u;
  const uint32_t ty = rtwm::udiv(tile, A.tx_m, A.tx_sh);  // tile / tiles_x
  const uint32_t tx = tile - ty * A.tiles_x;
  px = tx * kTileW + (l & 7u);
  ly = ty * kTileH + (l >> 3);
  return px < A.W && ly < A.row_count;  // else a padding unit of an edge tile
}

// Lanes with `need` take units from the wave's reservoir [qnext, qend)
// (wave-uniform), refilled `batch` units at a time from the device queue —
// the megakernel's dealing (rtw_trace.hip step 1) with smaller batches, so
// little work sits in reservoirs when the queue runs dry.  Wave-converged.  On return
// `got` lanes own `unit`; lanes that found the queue exhausted do not.
template <typename R>
__device__ __forceinline__ bool take_unit(const TraceArgs<R>& A, uint32_t batch, bool need, uint32_t lid,
                                          uint32_t& qnext, uint32_t& qend, uint32_t& unit) {
  bool got = false;
  for (;;) {
    const uint64_t m = __ballot(need);
    if (!m) break;
    const uint32_t n = (uint32_t)__popcll(m);
    const uint32_t rank = mbcnt64(m);
    const uint32_t rem = qend - qnext;
    const uint32_t grab = max(batch, n - rem);  // (used only when n > rem)
    uint32_t base2 = 0;
    if (n > rem) {
      uint32_t b = 0;
      if (lid == 0) b = atomicAdd(A.counter, grab);
      base2 = __shfl(b, 0);
    }
    if (need) {
      const uint32_t raw = rank < rem ? qnext + rank : base2 + (rank - rem);
      uint32_t px, ly, c;
      if (raw >= A.total_units) {
        need = false;  // queue exhausted: the slot retires
      } else {
        const uint32_t u = dealt_unit(raw, A);
        if (decode_unit(A, u, px, ly, c)) {
          need = false;
          got = true;
          unit = u;
        }
      }
    }
    if (n > rem) {
      qnext = base2 + (n - rem);
      qend = base2 + grab;
    } else {
      qnext += n;
    }
  }
  return got;
}

// Start sample s of `unit` in lane L (start_sample_uv / lens disk /
// start_sample_ray: main.zig:390-391, :91-100).  Per-lane disk rejection
// (the megakernel's default; every variant gives the same bits).
template <typename R>
__device__ __forceinline__ void start_path(const TraceArgs<R>& A, uint32_t unit, uint32_t s, Lane<R>& L) {
  uint32_t px, ly, c;
  decode_unit(A, unit, px, ly, c);
  L.px = px;
  L.ly = ly;
  L.s = s;
  R u, v, dk[2];
  start_sample_uv<R>(kargs<R>(), L, u, v);
  for (;;) {  // randomPointInUnitDisk (rand.zig:30-36)
    dk[0] = rrange_m11<R>(L.rs);
    dk[1] = rrange_m11<R>(L.rs);
    if (in_unit_ball<R, 2>(dk)) break;
  }
  start_sample_ray<R>(kargs<R>(), L, u, v, dk[0], dk[1]);
}

// The same for the lanes with `need` (wave-converged): the lens-disk points
// from one cooperative pass (coop_reject_mixed, dim 2: the megakernel's
// merged start) with the sample's time draw made in it, instead of each
// lane's own rejection loop — the same candidates and states, so the same bits.
template <typename R>
__device__ __forceinline__ void start_path_coop(const TraceArgs<R>& A, uint32_t unit, uint32_t s, bool need,
                                                Lane<R>& L, CoopSlots* slots, uint32_t lid) {
  R u = (R)0, v = (R)0;
  if (need) {
    uint32_t px, ly, c;
    decode_unit(A, unit, px, ly, c);
    L.px = px;
    L.ly = ly;
    L.s = s;
    start_sample_uv<R>(kargs<R>(), L, u, v);
  }
  R pt[3] = {(R)0, (R)0, (R)0}, raw = (R)0;
  if (__any(need)) coop_reject_mixed<R>(need ? 2u : 0u, L.rs, pt, raw, slots, lid);
  if (need) start_sample_ray<R, true>(kargs<R>(), L, u, v, pt[0], pt[1], raw);
}

// Append the wave's live lanes to its own segment of queue `out` at
// positions out_n, out_n+1, ... (order kept; no atomics).
template <typename R>
__device__ __forceinline__ void push_path(const PathBuf<R>& out, uint32_t seg_base, uint32_t& out_n, bool live,
                                          const Lane<R>& L, uint32_t slot) {
  const uint64_t m = __ballot(live);
  if (live) store_path(out, seg_base + out_n + mbcnt64(m), L, slot);
  out_n += (uint32_t)__popcll(m);
}

// The same with the path's closest hit (fused engine): its table position;
// L.o is already the hit point (to_hit_point), so the root is not stored.
template <typename R>
__device__ __forceinline__ void push_path_hit(const PathBuf<R>& out, uint32_t seg_base, uint32_t& out_n, bool live,
                                              const Lane<R>& L, uint32_t slot, int hit) {
  const uint64_t m = __ballot(live);
  if (live) {
    const uint32_t i = seg_base + out_n + mbcnt64(m);
    store_path(out, i, L, slot);
    out.hk[i] = hit;
  }
  out_n += (uint32_t)__popcll(m);
}

// Round 6: a path that found its closest hit carries the hit POINT in its
// origin from then on: p = o + t * d — ray.at(t), the operations scatter_hit
// makes (rtw_device.hpp, POINT = false), made here instead, so the same bits.
// The shading reads p (scatter_hit POINT), never o and t; the queues move
// p (24 B) instead of o and the root (32 B): 200 instead of 216 B per bounce
// segment of the fused engine.
template <typename R>
__device__ __forceinline__ void to_hit_point(Lane<R>& L, int hit, R tmax) {
  if (hit >= 0) L.o = add(L.o, mul(L.d, tmax));
}

template <typename R>
__device__ __forceinline__ uint32_t chunk_end(const TraceArgs<R>& A, uint32_t c) {
  return min(c * A.chunk + A.chunk, A.spp);
}

// A wave-uniform word this wave may have written earlier in the same launch:
// a vector load at device scope (past the CU's L1), not a scalar load (the
// scalar cache does not see vector stores).
__device__ __forceinline__ uint32_t ld_wave_u32(const uint32_t* p) {
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Between two queue passes of one launch: this wave's stores have completed
// before it reads the lines back (workgroup scope: the same CU's L1, which its
// own stores keep current; no L2 write-back).
__device__ __forceinline__ void wave_own_writes_visible() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

// Waves are persistent over segments: wave w owns segments w, w + nwaves, ...
// for the whole frame (the host launches the same grid every time).
// (wave-uniform by construction, made so for the compiler: as a per-lane value the
// segment loop's index lived in a VGPR pair that wf_step spilled to scratch)
__device__ __forceinline__ uint32_t wave_id() {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kTraceBlock / 64) + (threadIdx.x >> 6)));
}
__device__ __forceinline__ uint32_t wave_count() { return gridDim.x * (kTraceBlock / 64); }

// Workgroup-uniform: does any segment of this workgroup's waves hold paths?
// (Drain phase: most workgroups skip the LDS staging and exit.)
template <typename R>
__device__ __forceinline__ bool group_has_work(const WfArgs<R>& A) {
  bool work = false;
  for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) work |= A.seg_in[seg] != 0u;
  return __syncthreads_or(work) != 0;
}

// One shading step of a lane's path (`valid`): background on a miss
// (main.zig:109-112) or Material.scatter (material.zig:22-121); a finished
// sample adds to its slot's f64 chunk sum, a finished chunk publishes it and
// the slot takes the next unit from the segment's reservoir; the slot's next
// sample starts at once.  Wave-converged (coop_reject, take_unit).  Returns
// whether the lane holds a live path afterwards.  STATS: count finished
// samples and shaded segments (rtw_render_counts); FIN: also as the
// in-register drain's own counts (stats 9, 10: rtw_render_counts_ex).
// scatter_hit's variant bits: the megakernel's exact fast f64 sqrt and the
// host's Schlick r0^2 table (both bit-identical forms); -0.9 % per frame on top
// of the clustered pretest (profiles/r06/wf_step_ab.txt).
#ifndef RTW_WF_SCATTER_VAR  // (A/B builds override it; 0: the plain forms)
#define RTW_WF_SCATTER_VAR (kVarFastSqrt | kVarR0Table)
#endif
template <typename R>
constexpr int kWfScatterVar = RTW_WF_SCATTER_VAR;
#ifndef RTW_WF_PREDRAW
#define RTW_WF_PREDRAW 0  // A/B builds: the dielectric's draw inside the bounce's cooperative pass (neutral;
                          // profiles/r06/wf_step_ab.txt item 6)
#endif
constexpr bool kWfPreDraw = RTW_WF_PREDRAW != 0;
#ifndef RTW_WF_COOP_DISK
#define RTW_WF_COOP_DISK 0  // A/B builds: shade_step's new samples take their lens-disk points cooperatively
                            // (2.5 % slower; wf_step_ab.txt item 6)
#endif
constexpr bool kWfCoopDisk = RTW_WF_COOP_DISK != 0;
#ifndef RTW_WF_LANE_BALL
#define RTW_WF_LANE_BALL 0  // A/B builds: the bounce's unit-ball points from each lane's own loop (1.0 %
                            // slower; wf_step_ab.txt item 7)
#endif
constexpr bool kWfLaneBall = RTW_WF_LANE_BALL != 0;

// The bounce of a lane's path (`valid`) on its closest hit: background on a
// miss, else Material.scatter; `ended` when the sample is over (miss,
// absorbed, or the depth bound).  Wave-converged (coop_reject).
template <typename R, bool F32>
__device__ __forceinline__ void bounce(const WfArgs<R>& A, const LdsTables<R>& T, uint32_t lid, bool valid, Lane<R>& L,
                                       int hit, R tmax, bool& ended, bool& miss) {
  bool shading = false;
  ended = miss = false;
  uint32_t kind = 0;
  if (valid) {
    if (hit < 0) {  // miss: background (main.zig:109-112)
      miss = true;
      ended = true;
    } else {
      kind = T.kind[(T.meta[hit] >> 8) & 0xFFFu];
      shading = true;
    }
  }
  // randomPointInUnitSphere (rand.zig:22-28) for Lambertian and Metal
  // (kWfPreDraw: and the dielectric's draw, in the same cooperative pass).
  R b3[3] = {(R)0, (R)0, (R)0}, raw = (R)0;
  if constexpr (kWfPreDraw) {
    const uint32_t dim = shading ? (kind <= 2u ? 3u : 1u) : 0u;
    if (__any(dim != 0u)) coop_reject_mixed<R>(dim, L.rs, b3, raw, T.slots, lid);
  } else if constexpr (kWfLaneBall) {
    if (shading && kind <= 2u)
      for (;;) {  // each lane's own rejection loop (rand.zig:22-28)
        b3[0] = rrange_m11<R>(L.rs);
        b3[1] = rrange_m11<R>(L.rs);
        b3[2] = rrange_m11<R>(L.rs);
        if (in_unit_ball<R, 3>(b3)) break;
      }
  } else {
    const bool nb = shading && kind <= 2u;
    if (__any(nb)) coop_reject<R, 3, true>(nb, L.rs, b3, T.slots, lid);
  }
  if (shading) {
    if (scatter_hit<R, F32, kWfScatterVar<R>, kWfPreDraw, true>(T, L, hit, tmax, kind, b3, raw))
      ended = true;  // absorbed: emitted == 0 (material.zig:31-38)
    else if (L.depth == A.t.max_depth)
      ended = true;  // rayColor(depth == 0) is black (main.zig:105-108)
  }
}

template <typename R, bool F32, bool STATS, bool FIN = false>
__device__ __forceinline__ bool shade_step(const WfArgs<R>& A, const LdsTables<R>& T, uint32_t lid, bool valid,
                                           Lane<R>& L, uint32_t slot, int hit, R tmax, uint32_t& qnext,
                                           uint32_t& qend) {
  const uint32_t npix = A.t.row_count * A.t.W;
  bool ended, miss;
  bounce<R, F32>(A, T, lid, valid, L, hit, tmax, ended, miss);
  // A finished sample adds to its slot's chunk sum (main.zig:393).
  bool need_unit = false, need_sample = false;
  uint32_t unit = 0, s = 0;
  if (ended) {
    HomeRec& h = A.home[slot];
    unit = h.unit;
    s = h.s + 1u;
    double* hs = h.sum;
    double sx = hs[0], sy = hs[1], sz = hs[2];
    if (miss) {
      const V3<R> col = mulv(L.T, ld3(opaque(kargs<R>())->bg));
      sx += (double)col.x;
      sy += (double)col.y;
      sz += (double)col.z;
    }
    uint32_t px, ly, c;
    decode_unit(A.t, unit, px, ly, c);
    if (s == chunk_end(A.t, c)) {  // unit done: publish the chunk sum
      double* dst = A.t.partial + ((size_t)c * npix + (size_t)ly * A.t.W + px) * 3;
      dst[0] = sx;
      dst[1] = sy;
      dst[2] = sz;
      need_unit = true;
    } else {
      if (miss) hs[0] = sx, hs[1] = sy, hs[2] = sz;
      h.s = s;
      need_sample = true;
    }
  }
  if (take_unit(A.t, A.batch, need_unit, lid, qnext, qend, unit)) {
    uint32_t px, ly, c;
    decode_unit(A.t, unit, px, ly, c);
    s = c * A.t.chunk;
    HomeRec& h = A.home[slot];
    h.unit = unit;
    h.s = s;
    double* hs = h.sum;
    // A zero the optimiser cannot hoist: hoisted out of the kernel's loop, the
    // constant vector of this store was kept in scratch (24 B per lane written
    // every launch: ~20 GB per frame of the fused engine's PMC traffic).
    double z = 0.0;
    asm volatile("" : "+v"(z));
    hs[0] = hs[1] = hs[2] = z;
    need_sample = true;
  }
  if constexpr (kWfCoopDisk)
    start_path_coop(A.t, unit, s, need_sample, L, T.slots, lid);
  else if (need_sample)
    start_path(A.t, unit, s, L);
  if constexpr (STATS) {
    const uint32_t ns = (uint32_t)__popcll(__ballot(ended)), nv = (uint32_t)__popcll(__ballot(valid));
    if (lid == 0) {
      atomicAdd(A.t.stats + 0, (unsigned long long)ns);
      atomicAdd(A.t.stats + 1, (unsigned long long)nv);
      if (FIN) {
        atomicAdd(A.t.stats + 9, (unsigned long long)nv);
        atomicAdd(A.t.stats + 10, (unsigned long long)ns);
      }
    }
  }
  return valid && (!ended || need_sample);
}

#ifndef RTW_WF_EXT_OCC
#define RTW_WF_EXT_OCC 5  // 6 measured 4 % faster per launch but spills 44 B/lane (wf_extend PMC traffic 104 vs 60 GB/frame)
#endif
constexpr int kWfExtendOcc = RTW_WF_EXT_OCC;
// (The clustered pretest, +5 % in the megakernel, made the fused engine 12 % slower
// in round 2: profiles/r02/wf_cluster_ab.txt — its extra registers spilled in
// wf_step.  Without spills since round 6 it is the default: RTW_WF_VAR_EXTRA.)
template <typename R>
constexpr int kWfExtendVar = sizeof(R) == 8 ? (kVarFastSqrt | RTW_WF_VAR_EXTRA) : 0;

// ---------------------------------------------------------------- generate --
// Every slot of the wave's segments takes a unit and starts its first sample.
// HIT (fused engine): also the first closest hit of every new path.
template <typename R, bool F32, bool HIT>
__global__ void __launch_bounds__(kTraceBlock) wf_generate(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const uint32_t lid = lane_id();
  LdsTables<R> T{};
  if constexpr (HIT) T = stage_tables<R>(A.t.sc, lds_raw);
  KStats st;
  for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) {
    const uint32_t base = seg * kSegCap;
    uint32_t qnext = 0, qend = 0, out_n = 0;
    for (uint32_t k = 0; k < kSegCap; k += 64) {
      const uint32_t slot = base + k + lid;
      uint32_t unit = 0;
      const bool got = take_unit(A.t, A.batch, true, lid, qnext, qend, unit);
      Lane<R> L{};
      if (got) {
        uint32_t px, ly, c;
        decode_unit(A.t, unit, px, ly, c);
        const uint32_t s = c * A.t.chunk;
        HomeRec& h = A.home[slot];
        h.unit = unit;
        h.s = s;
        h.sum[0] = h.sum[1] = h.sum[2] = 0.0;
        start_path(A.t, unit, s, L);
      }
      if constexpr (HIT) {
        int hit = -1;
        R tmax = (R)__builtin_huge_val();
        if (got) {
          closest_hit<R, F32, 0, kWfExtendVar<R>>(opaque(kargs<R>())->sc, T, L, A.t.tmin, A.t.pre_k, lid, st, hit, tmax);
          to_hit_point(L, hit, tmax);
        }
        push_path_hit(A.out, base, out_n, got, L, slot, hit);
      } else {
        push_path(A.out, base, out_n, got, L, slot);
      }
    }
    if (lid == 0) {
      A.seg_out[seg] = out_n;
      A.seg_resv[2 * seg] = qnext;
      A.seg_resv[2 * seg + 1] = qend;
    }
  }
}

// ------------------------------------------------------------------ extend --
// The megakernel's closest-hit instantiation: scene fields re-read from the
// kernel argument inside closest_hit (trace VAR bit 512: the SceneView copy
// would sit in SGPRs for the whole kernel, at the 100-SGPR limit), the exact
// fast f64 sqrt (kVarFastSqrt), and a waves-per-SIMD target for the register
// allocator (kWfExtendOcc, chosen by A/B on MI355X).
template <typename R, bool F32>
__global__ void __launch_bounds__(kTraceBlock, kWfExtendOcc) wf_extend(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  if (!group_has_work(A)) return;
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  const uint32_t lid = lane_id();
  const R tmin = A.t.tmin, pre_k = A.t.pre_k;
  KStats st;
  // Software-pipelined over the wave's segments: the next segment's ray is
  // loaded while this one's closest hit runs.
  auto load = [&](uint32_t seg, Lane<R>& L, bool& ok) {
    ok = seg < A.n_segs && lid < A.seg_in[seg];
    if (ok) {
      const uint32_t i = seg * kSegCap + lid;
      L.o = mk(A.in.ox[i], A.in.oy[i], A.in.oz[i]);
      L.d = mk(A.in.dx[i], A.in.dy[i], A.in.dz[i]);
      L.time = A.in.tm[i];
      L.skip = F32 ? (int)(A.in.dsk[i] >> 16) - 1 : -1;
    }
  };
  static_assert(kSegCap == 64, "one path per lane per segment");
  Lane<R> cur;
  bool cur_ok;
  load(wave_id(), cur, cur_ok);
  for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) {
    Lane<R> nxt;
    bool nxt_ok;
    load(seg + wave_count(), nxt, nxt_ok);
    if (cur_ok) {
      int hit = -1;
      R tmax = (R)__builtin_huge_val();
      closest_hit<R, F32, 0, kWfExtendVar<R>>(opaque(kargs<R>())->sc, T, cur, tmin, pre_k, lid, st, hit, tmax);
      const uint32_t i = seg * kSegCap + lid;
      A.hit_t[i] = tmax;
      A.hit_k[i] = hit;
    }
    cur = nxt;
    cur_ok = nxt_ok;
  }
}

// ------------------------------------------------------------------- shade --
// STATS: count finished samples and shaded segments (rtw_render_counts) —
// with the megakernel's counts they prove every sample ran exactly once.
template <typename R, bool F32, bool STATS>
__global__ void __launch_bounds__(kTraceBlock) wf_shade(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const uint32_t lid = lane_id();
  if (!group_has_work(A)) {  // every segment of the group is empty: so is its output
    if (lid == 0)
      for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) A.seg_out[seg] = 0u;
    return;
  }
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) {
  const uint32_t n_in = A.seg_in[seg];
  if (n_in == 0u) {
    if (lid == 0) A.seg_out[seg] = 0u;
    continue;
  }
  const uint32_t base = seg * kSegCap;
  uint32_t qnext = A.seg_resv[2 * seg], qend = A.seg_resv[2 * seg + 1], out_n = 0;
  for (uint32_t k = 0; k < n_in; k += 64) {  // wave-uniform: coop_reject runs converged
    const uint32_t i = base + k + lid;
    const bool valid = k + lid < n_in;
    Lane<R> L{};
    L.skip = -1;
    uint32_t slot = 0;
    int hit = -1;
    R tmax = (R)0;
    if (valid) {
      load_path(A.in, i, L, slot);
      hit = A.hit_k[i];
      tmax = A.hit_t[i];
      to_hit_point(L, hit, tmax);
    }
    const bool live = shade_step<R, F32, STATS>(A, T, lid, valid, L, slot, hit, tmax, qnext, qend);
    push_path(A.out, base, out_n, live, L, slot);
  }
  if (lid == 0) {
    A.seg_out[seg] = out_n;
    A.seg_resv[2 * seg] = qnext;
    A.seg_resv[2 * seg + 1] = qend;
  }
  }
}

// -------------------------------------------------------- step (fused) --
// The fused engine's bounce kernel: shade_step on the path's stored hit, then
// the closest hit of the lane's next ray (the bounced ray or the next
// sample's camera ray) in registers; live paths are appended to the output
// queue WITH their hit, so no separate extend launch re-reads the rays.
// Per bounce segment: path + hit read (100 B f64: the hit point in o, no root), path + hit written.
#ifndef RTW_WF_STEP_OCC
#define RTW_WF_STEP_OCC 5  // profiles/r02/wf_step_ab.txt: 5 waves (32-B spill) ~3 % faster than 4
#endif
// wf_step / wf_drain read their arguments through the kernarg pointer where
// used: held in SGPRs for the whole kernel (30 queue pointers among them) they
// were spilled to VGPR lanes around the closest hit (wf_step 93 -> 34,
// wf_drain 291 -> 93 v_readlane / v_writelane); -0.6 to -0.9 % per wavefront
// frame (profiles/r04/wf_karg_ab.txt).
// The kernel's argument (WfArgs, at offset 0 of the kernarg segment) through
// a pointer the compiler cannot see through (rtw_device.hpp opaque): its
// fields are scalar-loaded where used instead of held in SGPRs.
template <typename R>
__device__ __forceinline__ const WfArgs<R>& wkargs() {
  return *(const WfArgs<R>*)opaque((const RTW_CONST WfArgs<R>*)__builtin_amdgcn_kernarg_segment_ptr());
}
// The host's poll without a kernel of its own (round 6): each workgroup of a
// wf_step launch sums its waves' final segment path counts (lane 0's `sum`)
// and adds (sum << 20) + 1 to the 64-bit word live_acc: one relaxed atomic
// carries both the count and a ticket (low 20 bits; grids stay far below
// 2^20), so the workgroup that takes the last ticket holds the launch's total
// in the value its add returns — no fences.  (A first form with agent-scope
// release / acquire around a separate ticket made the engine 50% slower:
// every workgroup's fences wrote back and invalidated its XCD's L2 under the
// waves still running.)  The last workgroup writes the total to the host's
// pinned poll word and zeroes the accumulator for the next launch; the
// kernel's end makes the host word visible to the event the host waits on.
// It replaces, per polled batch, a wf_count launch and the copy of its result.
template <typename R>
__device__ __forceinline__ void publish_live(const WfArgs<R>& A, uint32_t sum) {
  if (!A.poll_out) return;  // (wave-uniform: a kernel argument)
  __shared__ uint32_t wg_sum[kTraceBlock / 64];
  if ((threadIdx.x & 63u) == 0u) wg_sum[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t g = 0;
    for (uint32_t w = 0; w < kTraceBlock / 64; ++w) g += wg_sum[w];
    uint64_t* acc = reinterpret_cast<uint64_t*>(A.live_acc);
    const uint64_t old = __hip_atomic_fetch_add(acc, (g << 20) + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((old & 0xFFFFFu) + 1u == gridDim.x) {
      __hip_atomic_store(A.poll_out, (uint32_t)((old >> 20) + g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(acc, uint64_t{0}, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <typename R, bool F32, bool STATS>
__global__ void __launch_bounds__(kTraceBlock, RTW_WF_STEP_OCC) wf_step([[maybe_unused]] WfArgs<R> A_arg) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const WfArgs<R>& A = wkargs<R>();  // (A_arg is the same record, read where used)
  const uint32_t lid = lane_id();
  if (!group_has_work(A)) {  // every segment of the group is empty: so is its output
    if (lid == 0 && (A.passes & 1u) != 0u)  // (an even pass count ends in seg_in, already all zero)
      for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) A.seg_out[seg] = 0u;
    publish_live(A, 0u);
    return;
  }
  const LdsTables<R> T = stage_tables<R>(A.t.sc, lds_raw);
  KStats st;
  static_assert(kSegCap == 64, "one path per lane per segment");
  // One queue pass over a segment: qin -> qout.  The segment's count and
  // reservoir are read with vector loads (a later pass of this launch reads
  // what lane 0 wrote in the pass before; the scalar cache would not see it).
  uint32_t live_sum = 0u;  // (lane 0) the wave's segment counts after the launch's last pass
  auto step_segment = [&](uint32_t seg, const PathBuf<R>& qin, const PathBuf<R>& qout, const uint32_t* sin,
                          uint32_t* sout, bool last) {
    const uint32_t base = seg * kSegCap;
    const uint32_t i = base + lid;
#ifndef RTW_WF_LOAD_AFTER_COUNT
    // The segment's count, reservoir and paths are loaded together: the path
    // loads of every lane (in bounds: a segment holds kSegCap positions) are
    // issued before the count is known, so the segment start waits for one
    // memory latency, not for the count's and then the paths' (a dependent
    // chain).  Lanes past the count ignore what they loaded.
    const uint32_t n_in = ld_wave_u32(sin + seg);
    uint32_t qnext = ld_wave_u32(A.seg_resv + 2 * seg), qend = ld_wave_u32(A.seg_resv + 2 * seg + 1), out_n = 0;
    int hit = qin.hk[i];
    R tmax = (R)0;  // (the stored path's o is its hit point)
    Lane<R> L{};
    uint32_t slot = 0;
    load_path(qin, i, L, slot);
    const bool valid = lid < n_in;  // (an empty segment runs through with no lane valid: out_n = 0)
#else
    const uint32_t n_in = ld_wave_u32(sin + seg);
    if (n_in == 0u) {
      if (lid == 0) sout[seg] = 0u;
      return;
    }
    uint32_t qnext = ld_wave_u32(A.seg_resv + 2 * seg), qend = ld_wave_u32(A.seg_resv + 2 * seg + 1), out_n = 0;
    const bool valid = lid < n_in;
    Lane<R> L{};
    L.skip = -1;
    uint32_t slot = 0;
    int hit = -1;
    R tmax = (R)0;
    if (valid) {
      load_path(qin, i, L, slot);
      hit = qin.hk[i];
    }
#endif
    // A.bounces (>= 1) bounce segments per path in this launch: shade, then
    // the next ray's closest hit, with the path kept in registers between
    // them (one queue read and one write per A.bounces segments; the same
    // per-sample arithmetic in the same order, so the same bits).
    bool live = valid;
    int nh = hit;
    R nt = tmax;
    for (uint32_t b = 0; b < A.bounces; ++b) {
      live = shade_step<R, F32, STATS>(A, T, lid, live, L, slot, nh, nt, qnext, qend);
      nh = -1;
      nt = (R)__builtin_huge_val();
      if (live) {
        closest_hit<R, F32, 0, kWfExtendVar<R>>(opaque(kargs<R>())->sc, T, L, A.t.tmin, A.t.pre_k, lid, st, nh, nt);
        to_hit_point(L, nh, nt);
      }
      if (!wany(live)) break;
    }
    push_path_hit(qout, base, out_n, live, L, slot, nh);
    if (lid == 0) {
      sout[seg] = out_n;
      A.seg_resv[2 * seg] = qnext;
      A.seg_resv[2 * seg + 1] = qend;
      if (last) live_sum += out_n;
    }
  };
  // (Segments dealt at run time instead, one ticket of a device counter per
  // segment, was 2.5x slower: ~16K same-address atomics per launch serialise
  // at ~8.5 ns each; profiles/r03/wf_dynamic_ab.txt.)
  // A.passes queue passes per launch: in -> out, out -> in, ...  A wave owns
  // its segments for the whole frame and a path never leaves its segment, so
  // a pass needs only this wave's own writes of the pass before: every path
  // still crosses the queues once per A.bounces segments, without the launch.
  for (uint32_t q = 0; q < A.passes; ++q) {
    const bool odd = (q & 1u) != 0u;
    const PathBuf<R>& qin = odd ? A.out : A.in;
    const PathBuf<R>& qout = odd ? A.in : A.out;
    const uint32_t* sin = odd ? A.seg_out : A.seg_in;
    uint32_t* sout = odd ? A.seg_in : A.seg_out;
    if (q > 0) wave_own_writes_visible();
    for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count())
      step_segment(seg, qin, qout, sin, sout, q + 1u == A.passes);
  }
  publish_live(A, live_sum);
}

// ------------------------------------------------------------------ finish --
// The drain in registers: once the unit queue runs dry the queue empties
// slowly (a slot runs the rest of its unit's samples one after another, and
// long glass paths finish last), and each (extend, shade) pair would move a
// sparse queue through HBM for a few paths per segment.  wf_finish runs once,
// one wave per segment: the wave loads its segment's live paths (queue A,
// ready for extend) and loops closest hit + shade_step in registers until
// every lane's slot is done — the same per-sample arithmetic and chunk-sum
// order, so the same bits; slots still take units from the segment's
// reservoir and the device queue, so the kernel is correct whenever it runs.
template <typename R, bool F32, bool STATS>
__global__ void __launch_bounds__(kTraceBlock) wf_finish(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const uint32_t lid = lane_id();
  if (!group_has_work(A)) return;
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  const R tmin = A.t.tmin, pre_k = A.t.pre_k;
  KStats st;
  static_assert(kSegCap == 64, "one path per lane per segment");
  for (uint32_t seg = wave_id(); seg < A.n_segs; seg += wave_count()) {
    const uint32_t n_in = A.seg_in[seg];
    if (n_in == 0u) continue;  // every slot of the segment retired: no unit is left for it
    uint32_t qnext = A.seg_resv[2 * seg], qend = A.seg_resv[2 * seg + 1];
    Lane<R> L{};
    L.skip = -1;
    uint32_t slot = 0;
    bool live = lid < n_in;
    int hit0 = -1;
    if (live) {
      load_path(A.in, seg * kSegCap + lid, L, slot);
      if (A.hit_form) hit0 = A.in.hk[seg * kSegCap + lid];
    }
    bool stored = A.hit_form != 0u;  // the queued paths carry their hit: shade it first
    while (__any(live)) {  // wave-converged loop; a lane's path advances one segment per pass
      int hit = -1;
      R tmax = (R)__builtin_huge_val();
      if (stored) {
        hit = hit0;
      } else if (live) {
        closest_hit<R, F32, 0, 0>(S, T, L, tmin, pre_k, lid, st, hit, tmax);
        to_hit_point(L, hit, tmax);
      }
      stored = false;
      live = shade_step<R, F32, STATS, true>(A, T, lid, live, L, slot, hit, tmax, qnext, qend);
    }
    if (lid == 0) {
      A.seg_in[seg] = 0u;
      A.seg_resv[2 * seg] = qnext;
      A.seg_resv[2 * seg + 1] = qend;
    }
  }
}

// ------------------------------------------------------------------- drain --
// The drain dealt per SAMPLE (default; RTW_WF_DRAIN=0: wf_finish).  In
// wf_finish a lane is its slot: it runs the rest of its unit's samples one
// after another, so a wave lasts as long as its slowest slot (up to a whole
// chunk of samples) while lanes whose slot retired idle — the drain ran at
// about half the bounce kernels' segment rate.  Here the segment's slots only
// OWN units (a row of `tab` in LDS, lane = slot): their remaining samples are
// dealt to whichever lanes of the wave are free, so the wave stays full until
// the segment's last samples.  A sample's radiance (T * background at a miss;
// nothing for an absorbed or depth-bounded path) goes to a ring entry of its
// unit (`drain_buf`, kDrainWin entries per slot), and the owner folds the
// entries into the unit's f64 chunk sum strictly in sample order — the
// addition sequence of every other engine, so the same bits.  At most
// kDrainWin samples of a unit are dealt ahead of its fold (the ring's size).
// A unit done publishes its chunk sum; its slot then takes the next unit from
// the segment's reservoir / the device queue (retiring when there is none),
// so the kernel is correct whenever it runs, as wf_finish — provided the grid
// holds one wave per segment (it has no segment loop; the host always launches
// ceil(segments / waves per block) blocks, rtw_capi.hip run_wavefront).
struct DrainUnit {  // 64 B per slot
  uint32_t unit, next, end, fold;  // unit id, next sample to deal, sample end, next sample to fold
  uint32_t ready, miss, live, pad; // ring bits (sample % kDrainWin): radiance stored / sample missed; unit held
  double sum[3];                   // chunk sum of the folded samples
  double pad2;
};
static_assert(sizeof(DrainUnit) == 64, "DrainUnit layout");

template <typename R, bool F32, bool STATS>
__global__ void __launch_bounds__(kTraceBlock) wf_drain([[maybe_unused]] WfArgs<R> A_arg) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const WfArgs<R>& A = wkargs<R>();  // (A_arg is the same record, read where used)
  __shared__ DrainUnit tab_all[kTraceBlock / 64][kSegCap];
  __shared__ uint32_t list_all[kTraceBlock / 64][64];
  const uint32_t lid = lane_id();
  // One wave per segment (the hardware dispatcher balances the waves; ordering
  // the segments by the units their reservoirs hold, most first, measured
  // equal: profiles/r03/wf_drain_ab.txt).
  const uint32_t seg = wave_id();
  const uint32_t n_in = seg < A.n_segs ? A.seg_in[seg] : 0u;
  if (__syncthreads_or(n_in != 0u) == 0) return;
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  const R tmin = A.t.tmin, pre_k = A.t.pre_k;
  const uint32_t npix = A.t.row_count * A.t.W;
  KStats st;
  DrainUnit* tab = tab_all[threadIdx.x >> 6];
  uint32_t* list = list_all[threadIdx.x >> 6];
  static_assert(kSegCap == 64, "one slot per lane");
  if (n_in != 0u) {  // (else every slot of the segment retired: no unit is left for it)
    const uint32_t base = seg * kSegCap;
    uint32_t qnext = A.seg_resv[2 * seg], qend = A.seg_resv[2 * seg + 1];
    tab[lid].live = 0u;  // a slot without a live path has retired
    wave_lds_sync();
    Lane<R> L{};
    L.skip = -1;
    uint32_t k = 0;  // the slot whose sample this lane traces
    bool have = lid < n_in;
    int stored = -2;  // hit_form: the queued path's hit, shaded before the lane traces again (-2: none)
    if (have) {  // the in-flight sample of slot k, from queue A
      uint32_t slot;
      load_path(A.in, base + lid, L, slot);
      if (A.hit_form) stored = A.in.hk[base + lid];
      k = slot - base;
      const uint32_t unit = A.home[slot].unit, s = A.home[slot].s;
      uint32_t px, ly, c;
      decode_unit(A.t, unit, px, ly, c);
      L.s = s;
      DrainUnit& u = tab[k];
      u.unit = unit;
      u.next = s + 1u;
      u.end = chunk_end(A.t, c);
      u.fold = s;
      u.ready = u.miss = 0u;
      u.live = 1u;
      const double* hs = A.home[slot].sum;
      u.sum[0] = hs[0], u.sum[1] = hs[1], u.sum[2] = hs[2];
    }
    wave_lds_sync();
    for (;;) {
      // 1. Deal: each pass gives every free lane one sample of a unit with
      // samples left in its window (the offering units in slot order).
      bool fresh = false;
      uint32_t fu = 0, fs = 0;
      for (;;) {
        const uint64_t needm = wballot(!have);
        if (!needm) break;
        const uint32_t o_next = tab[lid].next, o_end = tab[lid].end, o_fold = tab[lid].fold;
        const bool offer = tab[lid].live != 0u && o_next < min(o_end, o_fold + kDrainWin);
        const uint64_t offm = wballot(offer);
        if (!offm) break;
        const uint32_t nn = popc64(needm), ro = mbcnt64(offm);
        if (offer) {
          list[ro] = lid;
          if (ro < nn) tab[lid].next = o_next + 1u;  // its sample o_next is dealt now
        }
        wave_lds_sync();
        const uint32_t rw = mbcnt64(needm);
        if (!have && rw < popc64(offm)) {
          k = list[rw];
          fu = tab[k].unit;
          fs = tab[k].next - 1u;
          fresh = have = true;
        }
        wave_lds_sync();
      }
      if (!wany(have)) break;  // nothing in flight, nothing left to deal
      if (fresh) start_path(A.t, fu, fs, L);
      // 2. One segment of every lane's path.
      int hit = -1;
      R tmax = (R)__builtin_huge_val();
      if (have) {
        if (stored != -2) {  // (its o is the hit point already)
          hit = stored;
          stored = -2;
        } else {
          closest_hit<R, F32, 0, 0>(S, T, L, tmin, pre_k, lid, st, hit, tmax);
          to_hit_point(L, hit, tmax);
        }
      }
      bool ended, miss;
      bounce<R, F32>(A, T, lid, have, L, hit, tmax, ended, miss);
      if constexpr (STATS) {
        const uint32_t ns = popc64(wballot(ended)), nv = popc64(wballot(have));
        if (lid == 0) {
          atomicAdd(A.t.stats + 0, (unsigned long long)ns);
          atomicAdd(A.t.stats + 1, (unsigned long long)nv);
          atomicAdd(A.t.stats + 9, (unsigned long long)nv);
          atomicAdd(A.t.stats + 10, (unsigned long long)ns);
          atomicAdd(A.t.stats + 13, 1ull);  // drain wave iterations (lane utilisation, RTW_COUNTS_VERBOSE)
        }
      }
      // 3. A finished sample's radiance goes to its unit's ring entry.
      if (ended) {
        const uint32_t bit = 1u << (L.s % kDrainWin);
        if (miss) {
          const V3<R> col = mulv(L.T, ld3(opaque(kargs<R>())->bg));
          R* b = A.drain_buf + ((size_t)(base + k) * kDrainWin + L.s % kDrainWin) * 3;
          b[0] = col.x;
          b[1] = col.y;
          b[2] = col.z;
          atomicOr(&tab[k].miss, bit);
        }
        atomicOr(&tab[k].ready, bit);
        have = false;
      }
      // The ring entries written above are read by other lanes of THIS wave:
      // a wavefront-scope release / acquire (no cache or counter wait — the
      // lanes of one wave see each other's vector memory operations in order,
      // AMDGPU memory model), not a workgroup-scope one, whose release would
      // wait for every store of the wave to complete each iteration.
      wave_lds_sync();
      // 4. Owners fold their ready samples in sample order (main.zig:393); a
      // unit done publishes its chunk sum and the slot takes the next unit.
      bool need_unit = false;
      if (tab[lid].live) {
        uint32_t fold = tab[lid].fold, ready = tab[lid].ready;
        const uint32_t mm = tab[lid].miss, end = tab[lid].end;
        double sx = tab[lid].sum[0], sy = tab[lid].sum[1], sz = tab[lid].sum[2];
        while ((ready >> (fold % kDrainWin)) & 1u) {
          const uint32_t j = fold % kDrainWin;
          if ((mm >> j) & 1u) {  // only a miss adds (the other engines' `sx += col`)
            const R* b = A.drain_buf + ((size_t)(base + lid) * kDrainWin + j) * 3;
            sx += (double)b[0];
            sy += (double)b[1];
            sz += (double)b[2];
          }
          ready &= ~(1u << j);
          ++fold;
        }
        tab[lid].fold = fold;
        tab[lid].ready = ready;
        tab[lid].miss = mm & ready;  // bits of folded samples cleared with their ready bits
        tab[lid].sum[0] = sx, tab[lid].sum[1] = sy, tab[lid].sum[2] = sz;
        if (fold == end) {
          uint32_t px, ly, c;
          decode_unit(A.t, tab[lid].unit, px, ly, c);
          double* dst = A.t.partial + ((size_t)c * npix + (size_t)ly * A.t.W + px) * 3;
          dst[0] = sx;
          dst[1] = sy;
          dst[2] = sz;
          tab[lid].live = 0u;
          need_unit = true;
        }
      }
      uint32_t unit = 0;
      if (take_unit(A.t, A.batch, need_unit, lid, qnext, qend, unit)) {
        uint32_t px, ly, c;
        decode_unit(A.t, unit, px, ly, c);
        DrainUnit& u = tab[lid];
        u.unit = unit;
        u.next = u.fold = c * A.t.chunk;
        u.end = chunk_end(A.t, c);
        u.ready = u.miss = 0u;
        u.live = 1u;
        u.sum[0] = u.sum[1] = u.sum[2] = 0.0;
      }
      wave_lds_sync();
    }
    if (lid == 0) {
      A.seg_in[seg] = 0u;
      A.seg_resv[2 * seg] = qnext;
      A.seg_resv[2 * seg + 1] = qend;
    }
  }
}

// Live paths of a queue = sum of its segment counts (the host's poll word).
__global__ void __launch_bounds__(1024) wf_count(const uint32_t* seg, uint32_t n, uint32_t* live) {
  __shared__ uint32_t part[16];
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += 1024) s += seg[i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < 16; ++w) t += part[w];
    *live = t;
  }
}
// End-of-frame check (after the last bounce batch or wf_finish): every
// segment's queue is empty, no reservoir still holds a unit below
// total_units, and the device queue head passed total_units.  Writes the
// number of violations to *bad (the host reads it; 0 = every unit ran).
__global__ void __launch_bounds__(1024) wf_check_drained(const uint32_t* seg, const uint32_t* resv, uint32_t n,
                                                          const uint32_t* head, uint32_t total_units, uint32_t* bad) {
  __shared__ uint32_t part[16];
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += 1024)
    s += (seg[i] != 0u) + (resv[2 * i] < min(resv[2 * i + 1], total_units));
  for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = *head < total_units;
    for (int w = 0; w < 16; ++w) t += part[w];
    *bad = t;
  }
}
hipError_t launch_wf_check_drained(const uint32_t* seg, const uint32_t* resv, uint32_t n, const uint32_t* head,
                                   uint32_t total_units, uint32_t* bad, hipStream_t s) {
  hipLaunchKernelGGL(wf_check_drained, dim3(1), dim3(1024), 0, s, seg, resv, n, head, total_units, bad);
  return hipGetLastError();
}
hipError_t launch_wf_count(const uint32_t* seg, uint32_t n, uint32_t* live, hipStream_t s) {
  hipLaunchKernelGGL(wf_count, dim3(1), dim3(1024), 0, s, seg, n, live);
  return hipGetLastError();
}

// ----------------------------------------------------------------- launch --
template <typename R, bool F32>
static hipError_t launch3(int k, const WfArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s) {
  if (k == 0)
    hipLaunchKernelGGL((wf_generate<R, F32, false>), dim3(grid), dim3(kTraceBlock), 0, s, a);
  else if (k == 6)
    hipLaunchKernelGGL((wf_generate<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 7)
    hipLaunchKernelGGL((wf_step<R, F32, false>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 8)
    hipLaunchKernelGGL((wf_step<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 1)
    hipLaunchKernelGGL((wf_extend<R, F32>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 2)
    hipLaunchKernelGGL((wf_shade<R, F32, false>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 3)
    hipLaunchKernelGGL((wf_shade<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 9)
    hipLaunchKernelGGL((wf_drain<R, F32, false>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 10)
    hipLaunchKernelGGL((wf_drain<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else if (k == 4)
    hipLaunchKernelGGL((wf_finish<R, F32, false>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else
    hipLaunchKernelGGL((wf_finish<R, F32, true>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_wf_generate_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(0, a, g, l, s);
}
hipError_t launch_wf_extend_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(1, a, g, l, s);
}
hipError_t launch_wf_shade_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<double, false>(stats ? 3 : 2, a, g, l, s);
}
hipError_t launch_wf_finish_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<double, false>(stats ? 5 : 4, a, g, l, s);
}
hipError_t launch_wf_finish_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<float, true>(stats ? 5 : 4, a, g, l, s);
}
hipError_t launch_wf_drain_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<double, false>(stats ? 10 : 9, a, g, l, s);
}
hipError_t launch_wf_drain_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<float, true>(stats ? 10 : 9, a, g, l, s);
}
hipError_t launch_wf_generate_hit_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(6, a, g, l, s);
}
hipError_t launch_wf_generate_hit_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(6, a, g, l, s);
}
hipError_t launch_wf_step_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<double, false>(stats ? 8 : 7, a, g, l, s);
}
hipError_t launch_wf_step_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<float, true>(stats ? 8 : 7, a, g, l, s);
}
hipError_t launch_wf_generate_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(0, a, g, l, s);
}
hipError_t launch_wf_extend_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(1, a, g, l, s);
}
hipError_t launch_wf_shade_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
  return launch3<float, true>(stats ? 3 : 2, a, g, l, s);
}

template <typename R, bool F32>
static int occ_wf(int kernel, size_t lds) {
  int n = 0;
  const hipError_t e =
      kernel == 1   ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wf_extend<R, F32>, kTraceBlock, lds)
      : kernel == 3 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wf_step<R, F32, false>, kTraceBlock, lds)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wf_shade<R, F32, false>, kTraceBlock, lds);
  return (e == hipSuccess && n > 0) ? n : 1;
}
int wf_blocks_per_cu(int precision, int kernel, size_t lds) {
  return precision == 1 ? occ_wf<float, true>(kernel, lds) : occ_wf<double, false>(kernel, lds);
}

}  // namespace rtwk
