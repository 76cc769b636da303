// rtw_internal.hpp — device-side scene layout and kernel launch interface,
// shared by rtw_trace.hip (kernels) and rtw_capi.hip (C ABI).
//
// HBM layout of a scene (uploaded once by rtw_scene_create):
//   sph_R  : n x 8 R    {c0.x, c0.y, c0.z, dc.x, dc.y, dc.z, r*r, RN(1/r)}   (dc = c1 - c0, in f64)
//   rad_R  : n x R      radius
//   meta   : n x u32    bit0 moving | bit1 wide | bits2-7 time group | bits8-19 material
//                       | bits20-31 original list index (tie-break)
//   perm   : n x u32    original list index -> table position
// Table order: [static wide | static | moving wide | moving] (SceneView g_*
// offsets), each group in list order; sph / meta carry one padding record.
//   mat_R  : nm x 8 R   {albedo.xyz, odd.xyz, fuzz (metal) | RN(1/ir) (dielectric), ir}
//   kind   : nm x u32   rtw_material_kind
//   tg_R   : ng x 4 R   {t0, t1, RN(1/(t1-t0)), 0} per distinct MovingSphere (time0, time1)
//   wide_d : n x 8 f64  f64 copy of sph (f32 mode solves wide spheres in f64)
//   tg_d   : ng x 4 f64
//   cull   : nn_pad/2 x 16 f32  pretest pairs over the narrow spheres in table
//            order (static narrow, then moving narrow; rtw_cull.hpp)
//   cull_tg: nn_pad/2 x u32     time groups of each pair
// R = double (precision 0) and float (precision 1) copies are both kept.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtwk {

constexpr uint32_t kMoving = 1u;
constexpr uint32_t kWide = 2u;
constexpr uint32_t kMaxTimeGroups = 64;
constexpr uint32_t kTileW = 8, kTileH = 8;  // 64 pixels = one wave's batch
constexpr uint32_t kBatch = 64;             // work units fetched per atomic
constexpr double kWideRadius = 100.0;       // f32 mode: radius >= this -> f64 quadratic

template <typename R>
struct SceneView {
  const R* sph;
  const R* rad;
  const uint32_t* meta;
  const R* mat;
  const uint32_t* kind;
  const R* tg;
  const double* wide_d;
  const double* tg_d;
  const uint32_t* perm;
  const float* cull;     // pretest records, nn_pad / 2 pairs x 16 f32 (rtw_trace.hip cull_pair)
  const uint32_t* cull_tg;  // per pair: time group of sphere 2p | (of 2p+1) << 8
  const float* tg_f;     // f32 time groups (t0, t1, 1/(t1-t0), 0) for the pretest
  uint32_t n, nm, ng;
  uint32_t g_static_wide, g_static, g_moving_wide;  // group ends; the moving group ends at n
  uint32_t nn, nn_pad, n_sn;  // narrow spheres (static narrow first), padded to 32; static narrow count
  uint32_t cull_on;           // pretest usable for this scene (rtw_cull.hpp limits)
  float cull_cmax;            // max |c0|_inf + |c1 - c0|_inf over narrow spheres (rounded up)
  float cull_rho;             // max 2 r^2 + 1 over narrow spheres (rounded up)
  // Clustered pretest (trace VAR kVarCluster, f64): the narrow spheres in
  // spatial clusters of <= 8 slots (cluster c = slots 8c..8c+7, padded with
  // dummy slots); a bounding sphere per cluster, pretested first, lets a wave
  // skip every member's pretest when no lane's ray line can meet it.
  const float* ccull;         // pair records in slot order (PairRec, 16 f32 per slot pair); kClusterSlots per cluster
  const uint32_t* ccull_tg;   // per slot pair: time groups (bits 0-15), y-only (16), static pair (17)
  const float* cclus;         // cluster bounding spheres as static pair records (2 clusters per record)
  const uint32_t* cpos;       // slot -> table position (dummy slots: 0)
  const uint32_t* cvalid;     // per 64-slot block: 2 words, bit 31 - r of word h = slot 32h + r real
  uint32_t n_clusters;        // clusters (blocks of 8 -> 64 slots)
  uint32_t cluster_on;        // clusters usable (set per render: camera times within every time group)
  float cull_rho_cl;          // max 2 R^2 + 1 over the cluster bounding spheres (rounded up)
};

#ifndef RTW_CLUSTER_SLOTS  // (A/B builds override it: 4 or 8)
#define RTW_CLUSTER_SLOTS 8
#endif
constexpr uint32_t kClusterSlots = RTW_CLUSTER_SLOTS;  // slots per cluster (even, divides 64)
static_assert(kClusterSlots % 2 == 0 && 64 % kClusterSlots == 0, "cluster slots");

template <typename R>
struct TraceArgs {
  SceneView<R> sc;
  R origin[3], horizontal[3], vertical[3], llc[3], cu[3], cv[3];
  R lens_radius, time0, time1;
  R bg[3];
  R tmin;
  R inv_w1, inv_h1;               // RN(1/(W-1)), RN(1/(H-1))
  R pre_k;                        // prefilter bound: tmin / (2.5 * unit roundoff)
  uint32_t W, H, spp, max_depth, chunk, n_chunks;
  uint32_t row_begin, row_stride, row_count, tiles_x;
  uint32_t total_units;
  uint32_t upt_m, upt_sh, tx_m, tx_sh;  // rtwm::udiv magic of units per tile (64 * n_chunks) and tiles_x
  uint32_t unit_order;            // rtw_device.hpp dealt_unit: 0 image order, 1 last-first
  uint64_t seed_base;             // SplitMix64(seed).next()
  double* partial;                // [n_chunks][row_count*W][3] chunk sums
  uint32_t* counter;              // work-queue head (zeroed before launch)
  unsigned long long* stats;      // counts {samples, segments, skipped} [0..2]; phase cycles [8..13]
};

struct FinalizeArgs {
  const double* partial;
  uint8_t* rgb;
  float* mean;
  uint32_t npix, n_chunks;
  double scale;  // 1.0 / spp
};

// Launchers (rtw_trace.hip).  Return hipError_t of the launch.
// mode: 0 = product, 1 = counts (segments/samples), 2 = diagnostic phase stamps
// var: tuning variant (rtw_trace.hip trace_kernel VAR bits)
hipError_t launch_trace_f64(const TraceArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, int mode, int var);
hipError_t launch_trace_f32(const TraceArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, int mode, int var);
hipError_t launch_finalize(const FinalizeArgs& a, hipStream_t s);
// Resident workgroups per CU for the trace kernel (occupancy query); 0 when
// `var` is not compiled into this library.
int trace_blocks_per_cu(int precision, size_t lds, int var);
// The trace_kernel variant of each precision in the product library (VAR bits
// of rtw_device.hpp / rtw_trace.hip, chosen by the in-process A/B on MI355X,
// profiles/r01/ab_defaults.txt): scalar sphere records + 512 (scene fields from
// the kernel argument) + kVarR0Table + kVarMergedStart + kVarPreDraw; f64 also
// 4 waves/SIMD (4) + kVarFastSqrt + kVarCluster (round 2, +5.4 %,
// profiles/r02/cluster_ab.txt) + 1024 (the loop's argument fields re-read from
// the kernel argument too: +0.6 %, profiles/r02/var1024_ab.txt) + kVarHomeLds
// (round 3, +0.6 %, profiles/r03/home_lds_ab.txt), f32 5 waves/SIMD (8) +
// kVarHomeLds (+1.3 %, profiles/r03/home_lds_f32_ab.txt).
// Every other variant exists only in the -DRTW_MEASURE build.
#ifndef RTW_DEFAULT_VAR_F64  // (A/B builds override it)
#define RTW_DEFAULT_VAR_F64 (4 + 512 + 1024 + 32768 + 131072 + 262144 + 524288 + 2097152 + 16777216)  // 19826180
#endif
constexpr int kDefaultVarF64 = RTW_DEFAULT_VAR_F64;
constexpr int kVarClusterBit = 2097152;  // rtw_device.hpp kVarCluster (clustered pretest, f64)
// The wavefront engine's closest-hit variant bits beyond kVarFastSqrt (f64;
// rtw_wavefront.hip kWfExtendVar): with kVarClusterBit its kernels run the
// clustered pretest and the host stages the cluster tables for them.  Round 6
// default: -3.0 % per configs[1] frame (profiles/r06/wf_step_ab.txt; round 2
// measured it 12 % slower when it spilled in wf_step, which no longer spills).
#ifndef RTW_WF_VAR_EXTRA  // (A/B builds override it; 0: the flat pretest)
#define RTW_WF_VAR_EXTRA kVarClusterBit
#endif
constexpr bool kWfCluster = (RTW_WF_VAR_EXTRA & kVarClusterBit) != 0;
// rtw_device.hpp kVarHomeLds: the lane's unit fields and f64 chunk sum in LDS
// (megakernel), kHomeLdsBytesPerWave per wave after the scene tables.
constexpr int kVarHomeLdsBit = 16777216;
constexpr size_t kHomeLdsBytesPerWave = 2560;
// + (kVarPathLds) the lane's path attenuation T (3 x 8 B) and RNG state (8 B) after it
constexpr int kVarPathLdsBit = 33554432;
constexpr size_t kPathLdsBytesPerWave = 4 * 64 * 8;
// + (kVarUnitBase) the unit's RNG base and f64 pixel column / reference row
constexpr int kVarUnitBaseBit = 67108864;
constexpr size_t kUnitBaseLdsBytesPerWave = 3 * 64 * 8;
#ifndef RTW_DEFAULT_VAR_F32  // (A/B builds override it)
#define RTW_DEFAULT_VAR_F32 (8 + 512 + 131072 + 262144 + 524288 + 16777216)  // 17695240
#endif
constexpr int kDefaultVarF32 = RTW_DEFAULT_VAR_F32;
bool trace_variant_built(int precision, int var);
constexpr int kTraceBlock = 256;
// Per-wave LDS slots of coop_reject (rtw_trace.hip CoopSlots: 64 x u64 + 64 x u32).
constexpr size_t kCoopLdsBytes = (kTraceBlock / 64) * 768;

// ------------------------------------------------------ wavefront engine --
// rtw_wavefront.hip (BASELINE.json configs[3]): the same Tier-B render as the
// megakernel, split into per-bounce kernels over SoA path queues in HBM.
// A path = one in-flight sample: its ray, attenuation product, time, RNG
// state, depth and the home slot that owns its (pixel, chunk) unit.  Two
// queues ping-pong: extend(in) writes the closest hit per queue position,
// shade(in -> out) scatters, finishes samples, refills units/samples and
// appends the live paths to `out`.
// The queues are cut into SEGMENTS of kSegCap paths, each owned by one
// persistent wave: a wave always extends / shades its own segments, compacts
// survivors within a segment (no global atomics), deals units from the
// segment's reservoir (one global atomic per kWfBatch units), and a segment
// runs on the same XCD every launch (fixed grid, round-robin dispatch).
constexpr uint32_t kSegCap = 64;  // paths per segment (one 64-lane wave round)
constexpr uint32_t kDrainWin = 32;  // wf_drain: samples of a unit dealt ahead of its fold (ring entries per slot)
// A home slot of the wavefront engine, one 32-B record (one memory sector):
// a sample end reads and updates the three fields together (separate arrays
// touched three sectors per access, partially).
struct alignas(32) HomeRec {
  double sum[3];      // f64 chunk sum of the unit's finished samples
  uint32_t unit, s;   // the unit, the sample in flight
};
static_assert(sizeof(HomeRec) == 32, "HomeRec is one 32-B sector");
template <typename R>
struct PathBuf {
  R *ox, *oy, *oz, *dx, *dy, *dz, *tx, *ty, *tz, *tm;
  uint64_t* rs;
  uint32_t* slot;  // home slot
  uint32_t* dsk;   // depth | (skip + 1) << 16
  int32_t* hk;     // fused engine: the table position of the path's closest hit, -1 = miss; with hk >= 0 the path's
                   // o holds the hit point o + t * d (made where the hit was found: wavefront.hip to_hit_point)
};
// Moving bytes per path (one PathBuf entry).
template <typename R>
constexpr size_t kPathBytes = 10 * sizeof(R) + 8 + 4 + 4;
// Home bytes per slot: f64x3 chunk sum, unit id, sample index.
constexpr size_t kHomeBytes = 24 + 4 + 4;

template <typename R>
struct WfArgs {
  TraceArgs<R> t;  // MUST stay at offset 0: kargs<R>() reads it
  PathBuf<R> in, out;
  R* hit_t;         // [queue position of `in`] root of the winner
  int32_t* hit_k;   // [queue position of `in`] table position of the winner, -1 = miss
  HomeRec* home;    // [slot] the slot's unit, sample index and f64 chunk sum
  uint32_t* seg_in;    // [segment] live paths in `in`
  uint32_t* seg_out;   // [segment] live paths written to `out` (shade)
  uint32_t* seg_resv;  // [segment][2] unit reservoir [next, end)
  uint32_t* live;      // wf_count: sum of seg_in (host poll word)
  R* drain_buf;        // wf_drain: [slot][kDrainWin][3] radiance of finished samples awaiting their fold (R: the
                       // sample's radiance is an R value; widened to f64 when folded, as the other engines add it)
  uint32_t n_slots, n_segs;
  uint32_t batch;      // units per reservoir refill (one atomic on the device queue)
  uint32_t bounces;    // wf_step: bounce segments per path per launch (>= 1), the path kept in registers between them
  uint32_t passes;     // wf_step: queue passes per launch (>= 1): in -> out, out -> in, ... (every segment through the queues)
  uint32_t* live_acc;  // wf_step (fused): 8-B aligned 64-bit word, (sum of the launch's final segment counts << 20)
                       // + workgroups finished; zero between launches (the last workgroup resets it)
  uint32_t* poll_out;  // wf_step (fused): the host's pinned poll word, written by the launch's last workgroup
  uint32_t hit_form;   // 1: queue `in` holds paths WITH their hit (fused engine: hk, and o = the hit point); the drains
                       // then shade the stored hit first instead of tracing the segment again
};

hipError_t launch_wf_generate_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_extend_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_shade_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_generate_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_extend_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_shade_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_finish_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_finish_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_drain_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_drain_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
// Resident workgroups per CU of a bounce kernel (1 = extend, 2 = shade): the
// persistent grid of that kernel is CUs x this.
int wf_blocks_per_cu(int precision, int kernel, size_t lds);
// live = sum of seg_in[0..n_segs) (one workgroup).
hipError_t launch_wf_count(const uint32_t* seg_in, uint32_t n_segs, uint32_t* live, hipStream_t s);
// Fused engine (default): generate + the first closest hit, then one kernel
// per bounce (shade + the next closest hit; the hit travels with the path).
hipError_t launch_wf_generate_hit_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_generate_hit_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s);
hipError_t launch_wf_step_f64(const WfArgs<double>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
hipError_t launch_wf_step_f32(const WfArgs<float>& a, uint32_t grid, size_t lds, hipStream_t s, bool stats);
// *bad = violations of the drained state (non-empty segment, unit left in a
// reservoir, queue head below total_units); 0 after a complete frame.
hipError_t launch_wf_check_drained(const uint32_t* seg_in, const uint32_t* resv, uint32_t n_segs, const uint32_t* head,
                                   uint32_t total_units, uint32_t* bad, hipStream_t s);

// ---------------------------------------------------------- world engine --
// rtw_world.hip / rtw_world_capi.hip: the general-world kernel (all scenes
// of main.zig, BASELINE.json configs[4]).  f64 tables in HBM, 16 doubles
// (128 B) per record:
//   prim   : sphere  {c0.xyz, dc.xyz = c1 - c0, r, t0, t1 - t0, r*r, -, -, -, -, meta(2 x u32 x 2)}
//            rect    {a0, a1, b0, b1, k, a1 - a0, b1 - b0, ...,                  meta}
//            meta = {kind | xform+1 << 8, mat, orig list index, -} in doubles 14-15
//   xform  : {u32 n | op_i << (8 + 4 i)}, v[i].xyz at doubles 4 + 3i
//   texture: {u32 kind, perlin, image, -}, color, odd, even, scale at doubles 2, 5, 8, 11
//   material (8 doubles): {u32 kind, tex}, albedo, fuzz, ir at 1, 4, 5
//   perlin : ranvec 256 x 3 f64, then perm 3 x 256 u32 (per perlin)
//   image  : {width, height, byte offset} + one RGBA8 byte pool
//   node   : 64 B, BVH2 with both child boxes in the parent: f32 lo0.xyz, hi0.xyz,
//            lo1.xyz, hi1.xyz (each f64 box bound rounded OUTWARD to f32, so a box only
//            grows), u32 ref0, ref1; ref bit 31 = leaf {first (bits 0-22), count (23-29),
//            bit 30 = the leaf's spheres have a packed-f32 pretest record cull[first]}
//   cull   : 64 B per stored position (used at a leaf's first position): the
//            megakernel's pair record (rtw_device.hpp PairRec) of the leaf's <= 2 spheres
//   order  : list index -> stored position (the NaN fallback's sequential loop)
// Prims are stored in BVH leaf order; `orig` keeps the list index for the
// reference's tie rule (later object wins).
constexpr uint32_t kWorldRec = 16;   // doubles per prim / xform / texture record
constexpr uint32_t kMaxXfOps = 4;    // ops per transform chain (== RTW_MAX_XFORM_OPS)
constexpr uint32_t kNodeWords = 16;  // 32-bit words per BVH node
constexpr uint32_t kLeafBit = 0x80000000u;
constexpr uint32_t kCullBit = 0x40000000u;  // leaf ref: pretest record present
constexpr uint32_t kLeafCountMask = 0x7Fu;  // leaf ref: count = (ref >> 23) & mask
constexpr uint32_t kBvhStack = 32;  // per-wave LDS stack entries (the builder caps the depth)
// per-LANE stack entries of the per-lane traversal (rtw_world.hip closest_lane):
// a BVH of depth <= kLaneStack never overflows it (a push per level at most);
// deeper BVHs take the union walk
constexpr uint32_t kLaneStack = 16;
// ... of which kLaneStack - 1 in LDS rows: the walk keeps the stack's top entry
// in a register, and a tree of depth D holds at most D pending nodes (one
// sibling per level of the current path: pops take the deepest), so D - 1 rows
// (RTW_LANE_STACK_LDS: the rows built; the default keeps kLaneStack, one to spare)
#ifndef RTW_LANE_STACK_LDS
#define RTW_LANE_STACK_LDS kLaneStack
#endif
constexpr uint32_t kLaneStackLds = RTW_LANE_STACK_LDS;
static_assert(kLaneStackLds + 1 >= kLaneStack, "a depth-kLaneStack tree must fit the LDS rows + the top register");
// The per-lane walk's node cache: the first kNodeCache node records (the top
// of the tree in breadth-first order, rtw_world_capi.hip top_first) staged in
// LDS once per workgroup; a lane visiting one reads it with ds_read instead of
// three vector loads through the TA/TD pipe that bounds the walk.  0: none —
// the default: 21 records (with RTW_LANE_STACK_LDS 15 to fit four workgroups
// per CU) measured equal on the globe, 31.67 vs 31.29 ms (the walk pays per
// wave iteration, ~41 per segment for ~18 visits per lane, not per lane-load);
// profiles/r06/world_ncache_ab.txt.
#ifndef RTW_NODE_CACHE
#define RTW_NODE_CACHE 0
#endif
constexpr uint32_t kNodeCache = RTW_NODE_CACHE;
// per-lane walk: a paused walk keeps its closest hit's stored position + 1 in
// the low kTravPosBits of one LDS word (rtw_world.hip LaneTravRows)
constexpr uint32_t kTravPosBits = 26;
#ifndef RTW_MAX_LEAF_PRIMS
#define RTW_MAX_LEAF_PRIMS 2  // BVH leaf size (profiles/r01/world_leaf_ab.txt; experiment builds override it)
#endif
constexpr uint32_t kMaxLeafPrims = RTW_MAX_LEAF_PRIMS;

struct WorldView {
  const double* prim;
  const double* xform;
  const double* tex;
  const double* mat;
  const double* perlin;
  const uint32_t* image;   // n_images x {width, height, offset_lo, offset_hi}
  const uint8_t* pixels;
  const float* node;
  const uint32_t* order;
  const float* cull;             // leaf pretest records (kCullBit leaves)
  uint32_t n_prims, n_nodes, n_perlins, flags;
  float cull_cmax, cull_rho;     // rtw_cull.hpp Cmax and rho_max over the pretested spheres
};
constexpr uint32_t kWorldHasSpheres = 1;  // WorldView.flags

struct WorldArgs {
  TraceArgs<double> t;  // MUST stay at offset 0 (kargs<double>()); t.sc unused
  WorldView w;
  double margin;        // BVH test widening (rtw_world_capi.hip bvh_margin)
  unsigned long long* counts;  // stats pass: {samples, segments, node visits, prim tests}
  double* ring;         // tail dealing: [lane of the grid][kTailWin][3] radiance of samples traced for that lane's unit
  uint32_t tail_deal;   // 1: lanes the queue left without a unit trace samples of the wave's other units
  uint32_t lane_yield;  // per-lane traversal: a phase pauses once fewer lanes than this still walk (0: never)
};
constexpr uint32_t kTailWin = 32;  // world kernel: the last samples of a unit other lanes may trace (ring entries)

// occ: register-allocation target (workgroups per CU): 1 (none), 3 or 4.
// fs: the kernel's feature set, world_feature_set(features of the world, per-lane
// traversal): bits 1 noise texture, 2 image texture, 4 transform chains, 8 rects,
// 16 per-lane BVH traversal (sphere worlds only).
int world_feature_set(uint32_t feat, bool lane, bool packed);
hipError_t launch_world(const WorldArgs& a, uint32_t grid, size_t lds, hipStream_t s, int mode, int occ, int fs);
int world_blocks_per_cu(size_t lds, int occ, int fs);
constexpr int kWorldBlock = 256;
size_t world_lds_bytes(uint32_t n_perlins, int fs);

}  // namespace rtwk
