// rtw_wavefront.hip — the wavefront engine (BASELINE.json configs[3]): the
// reference's render loop + rayColor (main.zig:378-402, :103-122) as
// per-bounce kernels over SoA path queues in HBM, persistent-grid launches.
//
//   generate : every home slot takes a (pixel, chunk) unit and starts its
//              first sample (Camera.getRay, main.zig:91-100) -> queue A
//   extend   : closest hit (HittableList.hit, hittable.zig:231-244) for every
//              path of the input queue -> (hit root, winner) per position
//   shade    : background on a miss (main.zig:109-112) or Material.scatter
//              (material.zig:22-121); a finished sample adds to its slot's
//              f64 chunk sum, a finished chunk publishes it and the slot takes
//              the next unit; the slot's next sample starts at once, so the
//              queue stays full until the units run out.  Live paths are
//              appended to the output queue (one atomic per wave, coalesced).
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
  const uint32_t tile = unit / upt;
  const uint32_t r = unit - tile * upt;
  c = r >> 6;
  const uint32_t l = r & 63u;
  const uint32_t ty = tile / A.tiles_x;
  const uint32_t tx = tile - ty * A.tiles_x;
  px = tx * kTileW + (l & 7u);
  ly = ty * kTileH + (l >> 3);
  return px < A.W && ly < A.row_count;  // else a padding unit of an edge tile
}

// Lanes with `need` take units from the device queue (wave-converged; one
// atomic per wave per round).  On return `got` lanes own `unit`; lanes that
// found the queue exhausted have need == false and got == false.
template <typename R>
__device__ __forceinline__ bool take_unit(const TraceArgs<R>& A, bool need, uint32_t lid, uint32_t& unit) {
  bool got = false;
  for (;;) {
    const uint64_t m = __ballot(need);
    if (!m) break;
    const uint32_t n = (uint32_t)__popcll(m);
    uint32_t b = 0;
    if (lid == 0) b = atomicAdd(A.counter, n);
    b = __shfl(b, 0);
    if (need) {
      const uint32_t u = b + mbcnt64(m);
      uint32_t px, ly, c;
      if (u >= A.total_units) {
        need = false;  // queue exhausted: the slot retires
      } else if (decode_unit(A, u, px, ly, c)) {
        need = false;
        got = true;
        unit = u;
      }
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

// Append the wave's live lanes to queue `out` (positions contiguous per wave).
template <typename R>
__device__ __forceinline__ void push_path(const WfArgs<R>& A, bool live, uint32_t lid, const Lane<R>& L,
                                          uint32_t slot) {
  const uint64_t m = __ballot(live);
  if (!m) return;
  uint32_t b = 0;
  if (lid == 0) b = atomicAdd(A.count_out, (uint32_t)__popcll(m));
  b = __shfl(b, 0);
  if (live) store_path(A.out, b + mbcnt64(m), L, slot);
}

template <typename R>
__device__ __forceinline__ uint32_t chunk_end(const TraceArgs<R>& A, uint32_t c) {
  return min(c * A.chunk + A.chunk, A.spp);
}

// ---------------------------------------------------------------- generate --
template <typename R, bool F32>
__global__ void __launch_bounds__(kTraceBlock) wf_generate(WfArgs<R> A) {
  const uint32_t lid = lane_id();
  const uint32_t wave = (blockIdx.x * kTraceBlock + threadIdx.x) >> 6;
  const uint32_t nwaves = gridDim.x * (kTraceBlock / 64);
  for (uint32_t base = wave * 64; base < A.n_slots; base += nwaves * 64) {  // wave-uniform
    const uint32_t slot = base + lid;
    uint32_t unit = 0;
    const bool got = take_unit(A.t, slot < A.n_slots, lid, unit);
    Lane<R> L{};
    if (got) {
      uint32_t px, ly, c;
      decode_unit(A.t, unit, px, ly, c);
      const uint32_t s = c * A.t.chunk;
      A.home_unit[slot] = unit;
      A.home_s[slot] = s;
      A.home_sum[3 * slot] = A.home_sum[3 * slot + 1] = A.home_sum[3 * slot + 2] = 0.0;
      start_path(A.t, unit, s, L);
    }
    push_path(A, got, lid, L, slot);
  }
}

// ------------------------------------------------------------------ extend --
template <typename R, bool F32>
__global__ void __launch_bounds__(kTraceBlock) wf_extend(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  if (blockIdx.x == 0 && threadIdx.x == 0) *A.count_out = 0u;  // shade appends to it next
  const uint32_t n_in = *A.count_in;
  const uint32_t lid = lane_id();
  const R tmin = A.t.tmin, pre_k = A.t.pre_k;
  KStats st;
  for (uint32_t i = blockIdx.x * kTraceBlock + threadIdx.x; i < n_in; i += gridDim.x * kTraceBlock) {
    Lane<R> L;
    L.o = mk(A.in.ox[i], A.in.oy[i], A.in.oz[i]);
    L.d = mk(A.in.dx[i], A.in.dy[i], A.in.dz[i]);
    L.time = A.in.tm[i];
    L.skip = F32 ? (int)(A.in.dsk[i] >> 16) - 1 : -1;
    int hit = -1;
    R tmax = (R)__builtin_huge_val();
    closest_hit<R, F32, 0, 0>(S, T, L, tmin, pre_k, lid, st, hit, tmax);
    A.hit_t[i] = tmax;
    A.hit_k[i] = hit;
  }
}

// ------------------------------------------------------------------- shade --
template <typename R, bool F32>
__global__ void __launch_bounds__(kTraceBlock) wf_shade(WfArgs<R> A) {
  extern __shared__ __align__(16) unsigned char lds_raw[];
  const SceneView<R> S = A.t.sc;
  const LdsTables<R> T = stage_tables<R>(S, lds_raw);
  const uint32_t n_in = *A.count_in;
  const uint32_t lid = lane_id();
  const uint32_t wave = (blockIdx.x * kTraceBlock + threadIdx.x) >> 6;
  const uint32_t nwaves = gridDim.x * (kTraceBlock / 64);
  const uint32_t npix = A.t.row_count * A.t.W;
  for (uint32_t base = wave * 64; base < n_in; base += nwaves * 64) {  // wave-uniform: coop_reject converged
    const uint32_t i = base + lid;
    const bool valid = i < n_in;
    Lane<R> L{};
    L.skip = -1;
    uint32_t slot = 0;
    int hit = -1;
    R tmax = (R)0;
    if (valid) {
      load_path(A.in, i, L, slot);
      hit = A.hit_k[i];
      tmax = A.hit_t[i];
    }
    bool ended = false, shading = false, miss = false;
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
    // randomPointInUnitSphere (rand.zig:22-28) for Lambertian and Metal.
    const bool nb = shading && kind <= 2u;
    R b3[3] = {(R)0, (R)0, (R)0};
    if (__any(nb)) coop_reject<R, 3, true>(nb, L.rs, b3, T.slots, lid);
    if (shading) {
      if (scatter_hit<R, F32>(T, L, hit, tmax, kind, b3))
        ended = true;  // absorbed: emitted == 0 (material.zig:31-38)
      else if (L.depth == A.t.max_depth)
        ended = true;  // rayColor(depth == 0) is black (main.zig:105-108)
    }
    // A finished sample adds to its slot's chunk sum (main.zig:393).
    bool need_unit = false, need_sample = false;
    uint32_t unit = 0, s = 0;
    if (ended) {
      unit = A.home_unit[slot];
      s = A.home_s[slot] + 1u;
      double* hs = A.home_sum + 3 * (size_t)slot;
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
        A.home_s[slot] = s;
        need_sample = true;
      }
    }
    if (take_unit(A.t, need_unit, lid, unit)) {
      uint32_t px, ly, c;
      decode_unit(A.t, unit, px, ly, c);
      s = c * A.t.chunk;
      A.home_unit[slot] = unit;
      A.home_s[slot] = s;
      double* hs = A.home_sum + 3 * (size_t)slot;
      hs[0] = hs[1] = hs[2] = 0.0;
      need_sample = true;
    }
    if (need_sample) start_path(A.t, unit, s, L);
    push_path(A, valid && (!ended || need_sample), lid, L, slot);
  }
}

// ----------------------------------------------------------------- launch --
template <typename R, bool F32>
static hipError_t launch3(int k, const WfArgs<R>& a, uint32_t grid, size_t lds, hipStream_t s) {
  if (k == 0)
    hipLaunchKernelGGL((wf_generate<R, F32>), dim3(grid), dim3(kTraceBlock), 0, s, a);
  else if (k == 1)
    hipLaunchKernelGGL((wf_extend<R, F32>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  else
    hipLaunchKernelGGL((wf_shade<R, F32>), dim3(grid), dim3(kTraceBlock), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_wf_generate_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(0, a, g, l, s);
}
hipError_t launch_wf_extend_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(1, a, g, l, s);
}
hipError_t launch_wf_shade_f64(const WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<double, false>(2, a, g, l, s);
}
hipError_t launch_wf_generate_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(0, a, g, l, s);
}
hipError_t launch_wf_extend_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(1, a, g, l, s);
}
hipError_t launch_wf_shade_f32(const WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
  return launch3<float, true>(2, a, g, l, s);
}

template <typename R, bool F32>
static int occ3(int k, size_t lds) {
  int nb = 0;
  hipError_t e;
  if (k == 0)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, wf_generate<R, F32>, kTraceBlock, 0);
  else if (k == 1)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, wf_extend<R, F32>, kTraceBlock, lds);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, wf_shade<R, F32>, kTraceBlock, lds);
  return (e == hipSuccess && nb > 0) ? nb : 1;
}
int wf_blocks_per_cu(int precision, int kernel, size_t lds) {
  return precision == 1 ? occ3<float, true>(kernel, lds) : occ3<double, false>(kernel, lds);
}

}  // namespace rtwk
