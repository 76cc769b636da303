// rtw_world_capi.hip — C ABI of the general-world path (include/rtw_hip.h
// "general worlds"): validation of an rtw_world_desc, packing into the
// device records of rtw_internal.hpp, the BVH build, the render launches.
// Replaces the render loop of main.zig:378-402 for scenes 2-6 (and 1, 7).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rtw_hip.h"
#include "rtw_cull.hpp"
#include "rtw_internal.hpp"

// rtw_capi.hip helpers shared by both paths (same library).
int rtw_fail(int status, const char* fmt, ...);
int rtw_validate_params(const rtw_params* p);
const char* rtw_dev_knob(const char* name);  // environment, -DRTW_MEASURE builds only
size_t rtw_ws_total(const rtw_params* p);
int rtw_device_cus(int dev);
void rtw_fill_trace_args(rtwk::TraceArgs<double>& a, const rtw_camera* cam, const rtw_params* p, unsigned char* ws);
int rtw_launch_finalize(const rtw_params* p, unsigned char* ws, uint8_t* d_rgb, float* d_mean, hipStream_t s);
size_t rtw_ws_stats_off(const rtw_params* p);
size_t rtw_ws_counter_off(const rtw_params* p);
uint32_t rtw_total_units(const rtw_params* p);
int rtw_timer_mark(rtw_timer t, hipStream_t s, bool start);

namespace {

struct Box {
  double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], b.lo[k]), hi[k] = std::max(hi[k], b.hi[k]);
  }
  void grow(const double p[3]) {
    for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], p[k]), hi[k] = std::max(hi[k], p[k]);
  }
  double area() const {
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return dx < 0 ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

// World-space bounding box of a primitive: the reference's boudingBox
// (hittable.zig:133-143 sphere, :203-217 moving sphere over the camera
// shutter [0, 1], :304-317 / :359-372 / :414-427 rects padded by 1e-4)
// through its Translate / RotateY chain (:493-501, :514-556).
Box prim_box(const rtw_prim& p, const rtw_xform* xf) {
  Box b;
  if (p.kind <= RTW_PRIM_MOVING_SPHERE) {
    const double r = std::fabs(p.a[6]);
    for (int s = 0; s < (p.kind == RTW_PRIM_MOVING_SPHERE ? 2 : 1); ++s) {
      double c[3];
      for (int k = 0; k < 3; ++k) {
        c[k] = p.kind == RTW_PRIM_MOVING_SPHERE ? p.a[k] + (p.a[3 + k] - p.a[k]) * (((double)s - p.a[7]) / (p.a[8] - p.a[7]))
                                                : p.a[k];
      }
      Box cb;
      for (int k = 0; k < 3; ++k) cb.lo[k] = c[k] - r, cb.hi[k] = c[k] + r;
      b.grow(cb);
    }
  } else {
    const int ax_k = p.kind == RTW_PRIM_XY_RECT ? 2 : (p.kind == RTW_PRIM_XZ_RECT ? 1 : 0);
    const int ax_a = p.kind == RTW_PRIM_YZ_RECT ? 1 : 0, ax_b = p.kind == RTW_PRIM_XY_RECT ? 1 : 2;
    b.lo[ax_a] = p.a[0], b.hi[ax_a] = p.a[1];
    b.lo[ax_b] = p.a[2], b.hi[ax_b] = p.a[3];
    b.lo[ax_k] = p.a[4] - 0.0001, b.hi[ax_k] = p.a[4] + 0.0001;
  }
  if (xf) {
    for (int i = (int)xf->n - 1; i >= 0; --i) {
      if (xf->op[i] == RTW_XF_TRANSLATE) {
        for (int k = 0; k < 3; ++k) b.lo[k] += xf->v[i][k], b.hi[k] += xf->v[i][k];
      } else {
        const double sn = xf->v[i][0], cs = xf->v[i][1];
        Box nb;
        for (int c = 0; c < 8; ++c) {
          const double x = (c & 1) ? b.hi[0] : b.lo[0], y = (c & 2) ? b.hi[1] : b.lo[1],
                       z = (c & 4) ? b.hi[2] : b.lo[2];
          const double q[3] = {cs * x + sn * z, y, -sn * x + cs * z};
          nb.grow(q);
        }
        b = nb;
      }
    }
  }
  return b;
}

struct Bvh {
  std::vector<float> nodes;  // kNodeWords per node
  std::vector<uint32_t> order;  // stored position -> original prim index
  uint32_t n_nodes = 0, n_leaves = 0, max_depth = 0, max_leaf = 0;
  bool packed = false;  // pack_refs: the child refs also in the low bits of the lower bounds
};

// The per-lane walk loads a node's 12 bounds (48 B, three 16-B loads) and not
// its refs (words 12-13): each child's ref, as 24 bits (an interior node
// index < 2^23, or 0x800000 | (count - 1) << 22 | first primitive < 2^22),
// rides in the low byte of that child's three lower bounds (words 0 / 2 / 4
// for child 0, 1 / 3 / 5 for child 1; one byte each, gathered by two
// v_perm_b32), each bound moved DOWN to the nearest float whose low byte is
// the payload (< 512 ulps: the box only grows, so the test stays
// conservative; the union walk reads the same bounds and words 12-13).  The per-lane walk's loads are bound by the vector memory pipeline
// (TD busy ~0.85, profiles/r05/world_ta_pmc.txt): one load of four per visit.
uint32_t compact_ref(uint32_t r) {
  if (r < rtwk::kLeafBit) return r;
  return 0x800000u | ((((r >> 23) & rtwk::kLeafCountMask) - 1u) << 22) | (r & 0x7FFFFFu);
}
float lower_with_low8(float f, uint32_t payload) {  // the largest float <= f whose low byte is `payload`
  uint32_t b;
  std::memcpy(&b, &f, 4);
  if (!(b & 0x80000000u) && b >= 256u && f != 0.0f) {  // positive: smaller bit patterns are smaller
    uint32_t c = (b & ~255u) | payload;
    if (c > b) c -= 256u;
    std::memcpy(&f, &c, 4);
    return f;
  }
  const uint32_t m = b & 0x7FFFFFFFu;  // zero, tiny or negative: a larger magnitude below zero
  uint32_t c = (m & ~255u) | payload;
  if (c < m) c += 256u;
  c |= 0x80000000u;
  std::memcpy(&f, &c, 4);
  return f;
}
// The per-lane walk's node cache (rtw_world.hip, kNodeCache records in LDS)
// holds the first records: renumber so that the top of the tree comes first,
// breadth-first from the root; the other records keep their depth-first order
// (child 0 of an interior node is still its next record below the top).  Only
// the layout changes: every traversal follows refs, so no result can.
void top_first(Bvh& b, uint32_t k) {
  if (b.n_nodes <= 1 || k <= 1) return;
  std::vector<uint32_t> first{0u};
  for (size_t i = 0; i < first.size() && first.size() < k; ++i)
    for (int c = 0; c < 2 && first.size() < k; ++c) {
      uint32_t ref;
      std::memcpy(&ref, b.nodes.data() + (size_t)rtwk::kNodeWords * first[i] + 12 + c, 4);
      if (!(ref & rtwk::kLeafBit)) first.push_back(ref);
    }
  std::vector<uint32_t> id(b.n_nodes, ~0u);
  for (uint32_t i = 0; i < first.size(); ++i) id[first[i]] = i;
  uint32_t next = (uint32_t)first.size();
  for (uint32_t n = 0; n < b.n_nodes; ++n)
    if (id[n] == ~0u) id[n] = next++;
  std::vector<float> out(b.nodes.size(), 0.0f);  // (the same size: the padding record after the last stays)
  for (uint32_t n = 0; n < b.n_nodes; ++n) {
    float* d = out.data() + (size_t)rtwk::kNodeWords * id[n];
    std::memcpy(d, b.nodes.data() + (size_t)rtwk::kNodeWords * n, rtwk::kNodeWords * 4);
    for (int c = 0; c < 2; ++c) {
      uint32_t ref;
      std::memcpy(&ref, d + 12 + c, 4);
      if (!(ref & rtwk::kLeafBit)) {
        ref = id[ref];
        std::memcpy(d + 12 + c, &ref, 4);
      }
    }
  }
  b.nodes.swap(out);
}

bool pack_refs(Bvh& b, uint32_t n_prims, bool debug) {
  if (b.n_nodes >= 0x800000u || n_prims >= 0x400000u || b.max_leaf > 2u) return false;
  std::vector<float> packed(b.nodes);
  for (uint32_t n = 0; n < b.n_nodes; ++n) {
    float* nd = packed.data() + (size_t)rtwk::kNodeWords * n;
    for (int c = 0; c < 2; ++c) {
      uint32_t r;
      std::memcpy(&r, nd + 12 + c, 4);
      const uint32_t v = compact_ref(r);
      for (int k = 0; k < 3; ++k) {
        const float old = nd[2 * k + c], nw = lower_with_low8(old, (v >> (8 * k)) & 255u);
        if (!(nw <= old) || !std::isfinite(nw)) return false;  // (never: the bounds are finite)
        nd[2 * k + c] = nw;
      }
    }
  }
  if (debug) {  // the device's gather (rtw_world.hip trace_phase PACKED) restated, against every ref
    uint32_t bad = 0, worst = 0;
    for (uint32_t n = 0; n < b.n_nodes; ++n) {
      const float* nd = packed.data() + (size_t)rtwk::kNodeWords * n;
      const float* od = b.nodes.data() + (size_t)rtwk::kNodeWords * n;
      for (int c = 0; c < 2; ++c) {
        uint32_t r, w[3], v = 0;
        std::memcpy(&r, nd + 12 + c, 4);
        for (int k = 0; k < 3; ++k) {
          std::memcpy(&w[k], nd + 2 * k + c, 4);
          v |= (w[k] & 255u) << (8 * k);
          uint32_t ob;
          std::memcpy(&ob, od + 2 * k + c, 4);
          const bool neg = (w[k] | ob) & 0x80000000u;  // ulps between the two (same-sign or across zero)
          const uint32_t d = neg ? (w[k] & 0x7FFFFFFFu) + ((ob & 0x80000000u) ? 0u - (ob & 0x7FFFFFFFu) : ob)
                                 : ob - w[k];
          worst = std::max(worst, d);
          if (!(nd[2 * k + c] <= od[2 * k + c])) ++bad;
        }
        if (v != compact_ref(r)) ++bad;
      }
    }
    fprintf(stderr, "[rtw bvh] packed refs: %u nodes, %u mismatches, bounds moved down by <= %u ulps\n", b.n_nodes,
            bad, worst);
  }
  b.nodes.swap(packed);
  b.packed = true;
  return true;
}

// Leaf size: worlds of >= kLeafOneMin primitives (those AUTO walks per lane:
// >= 2 x kLaneNodes) get leaves of ONE primitive, smaller ones kMaxLeafPrims.
// Per lane, a leaf's primitives are tested one after another by the lanes
// that reach it: the globe at leaf 1 vs 2 is +4.3 % (1.98 vs 3.45 primitive
// tests, 17.6 vs 16.3 node visits per segment), 10 of 10 alternations; leaves
// of 3 and 4 are slower; the union walk on scene 1 (48 primitives) prefers 2
// (-6 % at 1): profiles/r05/world_leaf_ab.txt.
constexpr size_t kLeafOneMin = 512;

class Builder {
 public:
  // depth_cap: the tree's depth (interior levels on a root-to-leaf path) stays
  // <= depth_cap - 1 for the union walk's kBvhStack and <= depth_cap for
  // depth_cap = kLaneStack (the per-lane walk's rebuild, below): SAH splits
  // while a median subtree of the rest still fits, median splits after that.
  Builder(const std::vector<Box>& boxes, Bvh& out, uint32_t depth_cap = rtwk::kBvhStack)
      : boxes_(boxes), out_(out), leaf_max_(boxes.size() >= kLeafOneMin ? 1u : rtwk::kMaxLeafPrims),
        cap_(depth_cap), lane_cap_(depth_cap != rtwk::kBvhStack) {
    idx_.resize(boxes.size());
    for (size_t i = 0; i < idx_.size(); ++i) idx_[i] = (uint32_t)i;
    for (const Box& b : boxes) {
      double m[3];
      for (int k = 0; k < 3; ++k) m[k] = 0.5 * (b.lo[k] + b.hi[k]);
      cent_.push_back({m[0], m[1], m[2]});
    }
  }
  void run() {
    const uint32_t root = alloc();
    node(root, 0, (uint32_t)idx_.size(), 0);
    out_.order = idx_;
  }

 private:
  const std::vector<Box>& boxes_;
  Bvh& out_;
  const uint32_t leaf_max_;  // primitives per leaf (<= rtwk::kMaxLeafPrims)
  const uint32_t cap_;       // depth cap (see the constructor)
  const bool lane_cap_;      // the per-lane walk's cap: SAH while depth + need < cap (else + 2 < cap)
  std::vector<uint32_t> idx_;
  std::vector<std::array<double, 3>> cent_;

  uint32_t alloc() {
    out_.nodes.resize(out_.nodes.size() + rtwk::kNodeWords, 0.0f);
    return out_.n_nodes++;
  }
  Box range_box(uint32_t b, uint32_t e) const {
    Box r;
    for (uint32_t i = b; i < e; ++i) r.grow(boxes_[idx_[i]]);
    return r;
  }
  uint32_t leaf(uint32_t b, uint32_t e) {
    out_.n_leaves++;
    out_.max_leaf = std::max(out_.max_leaf, e - b);
    return rtwk::kLeafBit | ((e - b) << 23) | b;
  }
  // Binned SAH split of [b, e); falls back to the median of the widest axis.
  uint32_t split(uint32_t b, uint32_t e, bool sah) {
    Box cb;
    for (uint32_t i = b; i < e; ++i) cb.grow(cent_[idx_[i]].data());
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
    if (sah && cb.hi[axis] > cb.lo[axis]) {
#ifndef RTW_SAH_BINS
#define RTW_SAH_BINS 256  // profiles/r01/world_sah_bins_ab.txt
#endif
      constexpr int kBins = RTW_SAH_BINS;
      double best = INFINITY;
      int best_axis = -1, best_bin = -1;
      for (int k = 0; k < 3; ++k) {
        const double ext = cb.hi[k] - cb.lo[k];
        if (!(ext > 0)) continue;
        Box bb[kBins];
        uint32_t cnt[kBins] = {0};
        for (uint32_t i = b; i < e; ++i) {
          int t = (int)((cent_[idx_[i]][k] - cb.lo[k]) / ext * kBins);
          t = std::min(std::max(t, 0), kBins - 1);
          bb[t].grow(boxes_[idx_[i]]);
          cnt[t]++;
        }
        Box left[kBins];
        uint32_t lc[kBins];
        Box acc;
        uint32_t ac = 0;
        for (int t = 0; t < kBins; ++t) acc.grow(bb[t]), ac += cnt[t], left[t] = acc, lc[t] = ac;
        acc = Box();
        ac = 0;
        for (int t = kBins - 1; t > 0; --t) {
          acc.grow(bb[t]);
          ac += cnt[t];
          const double cost = left[t - 1].area() * lc[t - 1] + acc.area() * ac;
          if (lc[t - 1] > 0 && ac > 0 && cost < best) best = cost, best_axis = k, best_bin = t;
        }
      }
      if (best_axis >= 0) {
        const double ext = cb.hi[best_axis] - cb.lo[best_axis];
        auto mid = std::partition(idx_.begin() + b, idx_.begin() + e, [&](uint32_t i) {
          int t = (int)((cent_[i][best_axis] - cb.lo[best_axis]) / ext * kBins);
          return std::min(std::max(t, 0), kBins - 1) < best_bin;
        });
        const uint32_t m = (uint32_t)(mid - idx_.begin());
        if (m > b && m < e) return m;
      }
    }
    const uint32_t m = b + (e - b) / 2;
    std::nth_element(idx_.begin() + b, idx_.begin() + m, idx_.begin() + e,
                     [&](uint32_t x, uint32_t y) { return cent_[x][axis] < cent_[y][axis]; });
    return m;
  }
  uint32_t child(uint32_t b, uint32_t e, uint32_t depth) {
    // Leaves: few primitives, or the depth cap of the per-lane LDS stack
    // (node() switches to median splits while they still fit the cap).
    if (e - b <= leaf_max_ || (depth >= (lane_cap_ ? cap_ : cap_ - 1) && e - b <= rtwk::kLeafCountMask))
      return leaf(b, e);
    const uint32_t n = alloc();
    node(n, b, e, depth);
    return n;
  }
  void node(uint32_t n, uint32_t b, uint32_t e, uint32_t depth) {
    out_.max_depth = std::max(out_.max_depth, depth + 1);
    uint32_t m;
    if (e - b <= leaf_max_) {  // root of a tiny world: one leaf + an empty one
      m = e;
    } else {
      // SAH while the median-split depth of the rest still fits the stack.
      uint32_t need = 0;
      for (uint32_t c = e - b; c > leaf_max_; c = (c + 1) / 2) ++need;
      m = split(b, e, lane_cap_ ? depth + need < cap_ : depth + need + 2 < cap_);
    }
    // Child 0 is built first, so an interior child 0 is record n + 1, the line
    // the traversal loads with node n (rtw_world.hip RTW_WORLD_TOUCH_NEXT).
    // (The child of larger surface area first instead: equal, profiles/r04/
    // world_touch_next_ab.txt.)
    const uint32_t lo0 = b, hi0 = m, lo1 = m, hi1 = e;
    const uint32_t c0 = m == e ? leaf(b, e) : child(lo0, hi0, depth + 1);
    const uint32_t c1 = m == e ? (rtwk::kLeafBit | e) : child(lo1, hi1, depth + 1);
    const Box b0 = range_box(lo0, hi0), b1 = range_box(lo1, hi1);
    float* nd = out_.nodes.data() + (size_t)rtwk::kNodeWords * n;
    auto down = [](double x) {  // largest float <= x
      float f = (float)x;
      if ((double)f > x) f = std::nextafter(f, -INFINITY);
      return f;
    };
    auto up = [](double x) {  // smallest float >= x
      float f = (float)x;
      if ((double)f < x) f = std::nextafter(f, INFINITY);
      return f;
    };
    for (int k = 0; k < 3; ++k) {  // {lo0, lo1} and {hi0, hi1} pairs per axis (packed-f32 operands)
      nd[2 * k] = down(b0.lo[k]), nd[2 * k + 1] = down(b1.lo[k]);
      nd[6 + 2 * k] = up(b0.hi[k]), nd[7 + 2 * k] = up(b1.hi[k]);
    }
    uint32_t refs[2] = {c0, c1};
    std::memcpy(nd + 12, refs, sizeof(refs));
  }
};

}  // namespace

struct rtw_world_s {
  int device = 0;
  void* buf = nullptr;
  rtwk::WorldView view{};
  Box bounds;
  bool has_moving = false;
  uint32_t feat = 0;  // features used (rtw_world.hip kFeat*): picks the kernel instantiation
  uint32_t info[4] = {0, 0, 0, 0};
  bool packed = false;  // the BVH carries the refs in its bounds' low bits (pack_refs)
};

extern "C" {

int rtw_world_create(const rtw_world_desc* d, uint32_t flags, rtw_world* out) {
  if (!out || !d) return rtw_fail(RTW_EINVAL, "rtw_world_create: desc/out is NULL");
  *out = nullptr;
  if ((d->n_prims && !d->prims) || (d->n_xforms && !d->xforms) || (d->n_textures && !d->textures) ||
      (d->n_mats && !d->mats) || (d->n_perlins && !d->perlins) || (d->n_images && !d->images))
    return rtw_fail(RTW_EINVAL, "rtw_world_create: NULL array with a non-zero count");
  if (d->n_prims >= (1u << 23)) return rtw_fail(RTW_UNSUPPORTED, "%u primitives exceed 2^23", d->n_prims);
  for (uint32_t i = 0; i < d->n_xforms; ++i) {
    if (d->xforms[i].n > RTW_MAX_XFORM_OPS) return rtw_fail(RTW_EINVAL, "xform %u: %u ops", i, d->xforms[i].n);
    for (uint32_t k = 0; k < d->xforms[i].n; ++k)
      if (d->xforms[i].op[k] > RTW_XF_ROTATE_Y) return rtw_fail(RTW_EINVAL, "xform %u: op %u", i, d->xforms[i].op[k]);
  }
  for (uint32_t i = 0; i < d->n_images; ++i)
    if (!d->images[i].rgba || !d->images[i].width || !d->images[i].height)
      return rtw_fail(RTW_EINVAL, "image %u is empty", i);
  for (uint32_t i = 0; i < d->n_textures; ++i) {
    const rtw_texture& t = d->textures[i];
    if (t.kind > RTW_TEX_IMAGE) return rtw_fail(RTW_EINVAL, "texture %u: kind %u", i, t.kind);
    if (t.kind == RTW_TEX_NOISE && t.perlin >= d->n_perlins) return rtw_fail(RTW_EINVAL, "texture %u: perlin", i);
    if (t.kind == RTW_TEX_IMAGE && t.image >= d->n_images) return rtw_fail(RTW_EINVAL, "texture %u: image", i);
  }
  for (uint32_t i = 0; i < d->n_mats; ++i) {
    const rtw_wmaterial& m = d->mats[i];
    if (m.kind > RTW_WMAT_LIGHT) return rtw_fail(RTW_EINVAL, "material %u: kind %u", i, m.kind);
    if ((m.kind == RTW_WMAT_LAMBERT || m.kind == RTW_WMAT_LIGHT) && m.tex >= d->n_textures)
      return rtw_fail(RTW_EINVAL, "material %u: texture %u >= %u", i, m.tex, d->n_textures);
  }
  rtw_world_s* w = new rtw_world_s;
  std::vector<Box> boxes(d->n_prims);
  for (uint32_t i = 0; i < d->n_prims; ++i) {
    const rtw_prim& p = d->prims[i];
    if (p.kind > RTW_PRIM_YZ_RECT || p.mat >= d->n_mats || p.xform >= (int32_t)d->n_xforms || p.xform < -1) {
      delete w;
      return rtw_fail(RTW_EINVAL, "prim %u: kind %u / material %u / xform %d out of range", i, p.kind, p.mat, p.xform);
    }
    // MovingSphere.center divides by time1 - time0 (hittable.zig:219-221): an
    // empty or reversed shutter gives a NaN centre, whose box no BVH node
    // could hold (the BVH would prune what the linear list tests).
    if (p.kind == RTW_PRIM_MOVING_SPHERE && !(p.a[8] > p.a[7])) {
      delete w;
      return rtw_fail(RTW_EINVAL, "prim %u: moving sphere needs time1 > time0 (got %g, %g)", i, p.a[7], p.a[8]);
    }
    boxes[i] = prim_box(p, p.xform >= 0 ? &d->xforms[p.xform] : nullptr);
    w->bounds.grow(boxes[i]);
    w->has_moving |= p.kind == RTW_PRIM_MOVING_SPHERE;
    if (p.xform >= 0) w->feat |= 4u;
    if (p.kind >= RTW_PRIM_XY_RECT) w->feat |= 8u;
  }
  Bvh bvh;
  // Small worlds (<= kLinearMax primitives: the Cornell box, the Perlin and
  // earth scenes) run the wave-uniform linear loop: every lane tests the same
  // scalar-loaded record, which beat the divergent per-lane BVH walk on
  // MI355X; RTW_WORLD_LINEAR forces it for any size.
  constexpr uint32_t kLinearMax = 32;
  const bool use_bvh = !(flags & RTW_WORLD_LINEAR) && d->n_prims > kLinearMax;
  if (use_bvh) {
    Builder(boxes, bvh).run();
    // The per-lane walk (sphere worlds of >= kLeafOneMin primitives, leaves
    // of one) keeps its stack in kLaneStack LDS entries per lane: a tree
    // deeper than that is rebuilt with SAH splits only while a median subtree
    // of the rest still fits (depth <= kLaneStack), so the lane walk stays
    // available; the globe's SAH tree (depth 16) is already within it.
    const uint32_t unconstrained_depth = bvh.max_depth;
    if (bvh.max_leaf == 1 && bvh.max_depth > rtwk::kLaneStack) {
      Bvh capped;
      Builder(boxes, capped, rtwk::kLaneStack).run();
      if (capped.max_depth <= rtwk::kLaneStack && capped.max_leaf == 1) bvh = std::move(capped);
    }
    if (flags & RTW_WORLD_DEBUG_BVH)
      fprintf(stderr, "[rtw bvh] %u nodes, depth %u (unconstrained SAH: %u), max leaf %u\n", bvh.n_nodes,
              bvh.max_depth, unconstrained_depth, bvh.max_leaf);
    if (flags & RTW_WORLD_DEBUG_BVH) {  // root's two children: leaf (prims) or node, and their boxes
      for (int c = 0; c < 2; ++c) {
        uint32_t ref;
        std::memcpy(&ref, bvh.nodes.data() + 12 + c, 4);
        const float* nd = bvh.nodes.data();
        fprintf(stderr, "[rtw bvh] root child %d: %s %u, box x [%g, %g] y [%g, %g] z [%g, %g]\n", c,
                (ref & rtwk::kLeafBit) ? "leaf of" : "node", (ref & rtwk::kLeafBit) ? (ref >> 23) & rtwk::kLeafCountMask : ref,
                nd[0 + c], nd[6 + c], nd[2 + c], nd[8 + c], nd[4 + c], nd[10 + c]);
      }
    }
    // (leaf-of-one trees are the per-lane walk's: its node cache wants the top first)
    if (bvh.max_leaf == 1) top_first(bvh, rtwk::kNodeCache);
    (void)pack_refs(bvh, d->n_prims, (flags & RTW_WORLD_DEBUG_BVH) != 0);  // (after the diagnostic: it prints the boxes as built)
  } else {
    for (uint32_t i = 0; i < d->n_prims; ++i) bvh.order.push_back(i);
  }
  // Device records, in stored (leaf) order; `order_dev` maps list index -> stored position.
  const uint32_t n = d->n_prims;
  std::vector<double> prim((size_t)rtwk::kWorldRec * (n + 1), 0.0);  // + a zero padding record (prefetch)
  std::vector<uint32_t> list_to_pos(n);
  for (uint32_t pos = 0; pos < n; ++pos) {
    const uint32_t li = bvh.order[pos];
    list_to_pos[li] = pos;
    const rtw_prim& p = d->prims[li];
    double* r = prim.data() + (size_t)rtwk::kWorldRec * pos;
    if (p.kind <= RTW_PRIM_MOVING_SPHERE) {
      for (int k = 0; k < 3; ++k) r[k] = p.a[k];
      if (p.kind == RTW_PRIM_MOVING_SPHERE) {
        for (int k = 0; k < 3; ++k) r[3 + k] = p.a[3 + k] - p.a[k];  // center1.sub(center0)
        r[7] = p.a[7];
        r[8] = p.a[8] - p.a[7];  // time1 - time0
        r[10] = 1.0 / r[8];      // its reciprocal (Markstein division in the kernel)
      }
      r[6] = p.a[6];
      r[9] = p.a[6] * p.a[6];  // sphere.radius * sphere.radius
    } else {
      for (int k = 0; k < 5; ++k) r[k] = p.a[k];
      r[5] = p.a[1] - p.a[0];
      r[6] = p.a[3] - p.a[2];
    }
    const uint32_t meta[4] = {p.kind | ((uint32_t)(p.xform + 1) << 8), p.mat, li, 0u};
    std::memcpy(r + 14, meta, sizeof(meta));
    // the kind and list index again in double 11, so the per-lane walk's root
    // test reads doubles 0-11 only: six 16-B loads per primitive, not seven
    // (rtw_world.hip load_rec_lane)
    const uint32_t meta_lane[2] = {meta[0], meta[2]};
    std::memcpy(r + 11, meta_lane, sizeof(meta_lane));
  }
  // Leaf pretest records (rtw_cull.hpp, the megakernel's packed-f32 bound):
  // a BVH leaf of <= 2 spheres that are untransformed, narrow (|r| < 100) and
  // static or moving over the shutter [0, 1] (their f32 time fraction is the
  // ray's f32 time, as in the cover scene) gets the pair record of its
  // spheres at cull[first] and kCullBit in its ref; the kernel skips a
  // sphere's exact test when no lane's pretest survives.
  std::vector<float> cull;
  float cull_cmax = 0.0f, cull_rho = 0.0f;
  if (use_bvh) {
    auto eligible = [&](uint32_t pos) {
      const rtw_prim& p = d->prims[bvh.order[pos]];
      if (p.xform >= 0 || !(std::fabs(p.a[6]) < 100.0)) return false;
      return p.kind == RTW_PRIM_SPHERE || (p.kind == RTW_PRIM_MOVING_SPHERE && p.a[7] == 0.0 && p.a[8] == 1.0);
    };
    std::vector<uint32_t> leaf_refs;  // (node, child) slots whose leaf qualifies
    double cmax_c = 0.0, cmax_d = 0.0, rho_max = 1.0;
    for (uint32_t nd = 0; nd < bvh.n_nodes; ++nd) {
      for (uint32_t c = 0; c < 2; ++c) {
        uint32_t ref;
        std::memcpy(&ref, bvh.nodes.data() + (size_t)rtwk::kNodeWords * nd + 12 + c, 4);
        const uint32_t first = ref & 0x7FFFFFu, cnt = (ref >> 23) & rtwk::kLeafCountMask;
        if (!(ref & rtwk::kLeafBit) || cnt == 0 || cnt > 2) continue;
        bool ok = true;
        for (uint32_t k = first; k < first + cnt; ++k) ok = ok && eligible(k);
        if (!ok) continue;
        leaf_refs.push_back(2 * nd + c);
        for (uint32_t k = first; k < first + cnt; ++k) {
          const double* r = prim.data() + (size_t)rtwk::kWorldRec * k;
          for (int j = 0; j < 3; ++j) cmax_c = std::max(cmax_c, std::fabs(r[j])), cmax_d = std::max(cmax_d, std::fabs(r[3 + j]));
          rho_max = std::max(rho_max, 2.0 * r[9] + 1.0);
        }
      }
    }
    cull_cmax = std::nextafter((float)(cmax_c + cmax_d), INFINITY);
    cull_rho = std::nextafter((float)rho_max, INFINITY);
    const char* nc = rtw_dev_knob("RTW_WORLD_NOCULL");  // development knob (A/B): no leaf pretest
    if (!leaf_refs.empty() && cull_cmax <= rtwc::kCmaxLimit && !(nc && *nc)) {
      cull.assign((size_t)16 * n, 0.0f);
      for (uint32_t slot : leaf_refs) {
        float* nw = bvh.nodes.data() + (size_t)rtwk::kNodeWords * (slot / 2) + 12 + (slot & 1);
        uint32_t ref;
        std::memcpy(&ref, nw, 4);
        const uint32_t first = ref & 0x7FFFFFu, cnt = (ref >> 23) & rtwk::kLeafCountMask;
        for (uint32_t j = 0; j < cnt; ++j) {  // sphere j of the leaf -> lane j of each f2
          const double* r = prim.data() + (size_t)rtwk::kWorldRec * (first + j);
          float* q = cull.data() + (size_t)16 * first + j;
          for (int k = 0; k < 3; ++k) q[2 * k] = (float)r[k], q[2 * (3 + k)] = -(float)r[3 + k];
          const float rf = (float)r[6];
          q[12] = -(rf * rf);
        }
        ref |= rtwk::kCullBit;  // (cnt <= 2 here, so no ref is all ones: the traversal's kNoRef, rtw_world.hip)
        std::memcpy(nw, &ref, 4);
      }
    }
  }
  std::vector<double> xf((size_t)rtwk::kWorldRec * std::max(d->n_xforms, 1u), 0.0);
  for (uint32_t i = 0; i < d->n_xforms; ++i) {
    double* r = xf.data() + (size_t)rtwk::kWorldRec * i;
    uint32_t h = d->xforms[i].n;
    for (uint32_t k = 0; k < d->xforms[i].n; ++k) {
      h |= d->xforms[i].op[k] << (8 + 4 * k);
      for (int c = 0; c < 3; ++c) r[4 + 3 * k + c] = d->xforms[i].v[k][c];
    }
    std::memcpy(r, &h, 4);
  }
  std::vector<double> tex((size_t)rtwk::kWorldRec * std::max(d->n_textures, 1u), 0.0);
  for (uint32_t i = 0; i < d->n_textures; ++i) {
    const rtw_texture& t = d->textures[i];
    double* r = tex.data() + (size_t)rtwk::kWorldRec * i;
    const uint32_t h[4] = {t.kind, t.perlin, t.image, 0u};
    std::memcpy(r, h, sizeof(h));
    for (int c = 0; c < 3; ++c) r[2 + c] = t.color[c], r[5 + c] = t.odd[c], r[8 + c] = t.even[c];
    r[11] = t.scale;
  }
  std::vector<double> mat((size_t)8 * std::max(d->n_mats, 1u), 0.0);
  for (uint32_t i = 0; i < d->n_mats; ++i) {
    const rtw_wmaterial& m = d->mats[i];
    double* r = mat.data() + (size_t)8 * i;
    const uint32_t h[2] = {m.kind, m.tex};
    std::memcpy(r, h, sizeof(h));
    for (int c = 0; c < 3; ++c) r[1 + c] = m.albedo[c];
    r[4] = m.fuzz, r[5] = m.ir;
  }
  constexpr size_t kPerlinDoubles = 256 * 3 + 384;
  std::vector<double> perl(kPerlinDoubles * std::max(d->n_perlins, 1u), 0.0);
  for (uint32_t i = 0; i < d->n_perlins; ++i) {
    double* r = perl.data() + kPerlinDoubles * i;
    for (int j = 0; j < 256; ++j)
      for (int c = 0; c < 3; ++c) r[3 * j + c] = d->perlins[i].ranvec[j][c];
    std::memcpy(r + 256 * 3, d->perlins[i].perm, sizeof(d->perlins[i].perm));
  }
  std::vector<uint32_t> img(4 * std::max(d->n_images, 1u), 0u);
  size_t pix_bytes = 0;
  for (uint32_t i = 0; i < d->n_images; ++i) {
    img[4 * i] = d->images[i].width, img[4 * i + 1] = d->images[i].height;
    img[4 * i + 2] = (uint32_t)pix_bytes, img[4 * i + 3] = (uint32_t)(pix_bytes >> 32);
    pix_bytes += (size_t)d->images[i].width * d->images[i].height * 4;
  }
  // One allocation: prim | xform | tex | mat | perlin | image | pixels | nodes | order
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t o_prim = 0, o_xf = o_prim + al(prim.size() * 8), o_tex = o_xf + al(xf.size() * 8);
  const size_t o_mat = o_tex + al(tex.size() * 8), o_perl = o_mat + al(mat.size() * 8);
  const size_t o_img = o_perl + al(perl.size() * 8), o_pix = o_img + al(img.size() * 4);
  const size_t o_node = o_pix + al(std::max(pix_bytes, (size_t)4));
  // (+ two zero padding records: the traversal may load the records after the last)
  const size_t o_order = o_node + al(bvh.nodes.size() * 4 + 2 * (size_t)rtwk::kNodeWords * 4);
  const size_t o_cull = o_order + al((size_t)std::max(n, 1u) * 4);
  const size_t total = o_cull + al(std::max(cull.size() * 4, (size_t)4));
  std::vector<unsigned char> host(total, 0);
  std::memcpy(host.data() + o_prim, prim.data(), prim.size() * 8);
  std::memcpy(host.data() + o_xf, xf.data(), xf.size() * 8);
  std::memcpy(host.data() + o_tex, tex.data(), tex.size() * 8);
  std::memcpy(host.data() + o_mat, mat.data(), mat.size() * 8);
  std::memcpy(host.data() + o_perl, perl.data(), perl.size() * 8);
  std::memcpy(host.data() + o_img, img.data(), img.size() * 4);
  for (uint32_t i = 0; i < d->n_images; ++i)
    std::memcpy(host.data() + o_pix + ((size_t)img[4 * i + 2] | ((size_t)img[4 * i + 3] << 32)), d->images[i].rgba,
                (size_t)d->images[i].width * d->images[i].height * 4);
  if (!bvh.nodes.empty()) std::memcpy(host.data() + o_node, bvh.nodes.data(), bvh.nodes.size() * 4);
  if (n) std::memcpy(host.data() + o_order, list_to_pos.data(), (size_t)n * 4);
  if (!cull.empty()) std::memcpy(host.data() + o_cull, cull.data(), cull.size() * 4);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    delete w;
    return rtw_fail(RTW_ENODEV, "no HIP device");
  }
  if (hipMalloc(&w->buf, total) != hipSuccess) {
    delete w;
    return rtw_fail(RTW_ENOMEM, "rtw_world_create: hipMalloc(%zu)", total);
  }
  if (hipMemcpy(w->buf, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(w->buf);
    delete w;
    return rtw_fail(RTW_EHIP, "rtw_world_create: hipMemcpy failed");
  }
  auto* base = static_cast<unsigned char*>(w->buf);
  w->device = dev;
  w->view.prim = reinterpret_cast<const double*>(base + o_prim);
  w->view.xform = reinterpret_cast<const double*>(base + o_xf);
  w->view.tex = reinterpret_cast<const double*>(base + o_tex);
  w->view.mat = reinterpret_cast<const double*>(base + o_mat);
  w->view.perlin = reinterpret_cast<const double*>(base + o_perl);
  w->view.image = reinterpret_cast<const uint32_t*>(base + o_img);
  w->view.pixels = base + o_pix;
  w->view.node = reinterpret_cast<const float*>(base + o_node);
  w->view.order = reinterpret_cast<const uint32_t*>(base + o_order);
  w->view.cull = reinterpret_cast<const float*>(base + o_cull);
  w->view.cull_cmax = cull_cmax;
  w->view.cull_rho = cull_rho;
  for (uint32_t i = 0; i < d->n_textures; ++i)
    w->feat |= d->textures[i].kind == RTW_TEX_NOISE ? 1u : (d->textures[i].kind == RTW_TEX_IMAGE ? 2u : 0u);
  w->view.n_prims = n;
  for (uint32_t i = 0; i < n; ++i)
    if (d->prims[i].kind <= RTW_PRIM_MOVING_SPHERE) w->view.flags |= rtwk::kWorldHasSpheres;
  w->view.n_nodes = bvh.n_nodes;
  w->view.n_perlins = d->n_perlins;
  w->info[0] = bvh.n_nodes, w->info[1] = bvh.n_leaves, w->info[2] = bvh.max_depth, w->info[3] = bvh.max_leaf;
  w->packed = bvh.packed;
  *out = w;
  return RTW_OK;
}

int rtw_world_destroy(rtw_world w) {
  if (!w) return RTW_OK;
  if (w->buf) (void)hipFree(w->buf);
  delete w;
  return RTW_OK;
}

int rtw_world_bvh_info(rtw_world w, uint32_t info_out[4]) {
  if (!w || !info_out) return rtw_fail(RTW_EINVAL, "world/info is NULL");
  std::memcpy(info_out, w->info, sizeof(w->info));
  return RTW_OK;
}

}  // extern "C"

namespace {

// Default register-allocation target (waves per SIMD) from the A/Bs on MI355X
// (DESIGN.md §6.3): 4 waves hide the BVH's dependent node loads; worlds with
// rects or transforms (the Cornell box) run 2 % faster at the 3-wave budget
// since round 4's register work (profiles/r04/world_occ_ab.txt; round 1: 4 was
// best); Perlin-textured worlds keep the 2-wave budget because their noise
// loops spill badly.
static_assert(rtwk::kMaxXfOps == RTW_MAX_XFORM_OPS, "transform chain length");
int world_occ_default(const rtw_world_s* w) {
  if (w->view.n_perlins) return 1;
  return (w->feat & (4u | 8u)) ? 3 : 4;  // rtw_world.hip kFeatXform | kFeatRect
}

// Widening of every BVH box test.  A computed sphere root deviates from the
// exact intersection by at most ~sqrt(u * (hb^2 + |a c|)) / a (u = 2^-53; the
// sqrt of a discriminant with absolute error u*(hb^2 + |ac|)), i.e. in space
// by <= sqrt(u) * sqrt(2 |o - c|^2 + r^2) <= 2.2e-8 * L, where L bounds
// |o - c| + r over every ray origin o (camera or a surface point) and
// primitive.  Rect roots and the slab arithmetic are accurate to a few u * L.
// margin = 1e-7 * L with L = 2 * (max |coordinate| of the scene box and the
// camera) + 1 covers both with a 4x safety factor.  The kernel evaluates the
// slabs in packed f32 (t = fma(b, RN(1/d), RN(-RN(o) RN(1/d)))): expressed in
// space, its rounding is <= 4 u32 (|o| + |b|) <= 2^-22 L (u32 = 2^-24; the
// f32 bounds are rounded outward), so 2^-20 L more (4x) is added.  A box
// that holds a primitive the linear list would accept is never pruned.
double bvh_margin(const rtw_world_s* w, const rtw_camera* cam) {
  double m = 0;
  for (int k = 0; k < 3; ++k) {
    if (std::isfinite(w->bounds.lo[k])) m = std::max(m, std::fabs(w->bounds.lo[k]));
    if (std::isfinite(w->bounds.hi[k])) m = std::max(m, std::fabs(w->bounds.hi[k]));
    m = std::max(m, std::fabs(cam->origin[k]) + cam->lens_radius * 2);
  }
  const double L = 2.0 * m + 1.0;
  return 1e-7 * L + 0x1p-20 * L;
}

// The launch configuration of a world render on device `dev`: kernel
// instantiation (feature set), register budget, LDS, persistent grid, and the
// tail dealing's ring bytes (one kTailWin-entry f64x3 ring per lane of the
// grid, WorldArgs::ring), which live in the caller's workspace after the
// common region (rtw_ws_total), so renders on different streams with their
// own workspaces never share one.
struct WorldLaunchCfg {
  int fs, oi, bpc;
  size_t lds;
  uint32_t grid;
  size_t ring_off, ring_bytes;  // ring: [ring_off, ring_off + ring_bytes) of the workspace
};
constexpr uint32_t kLaneYield = 16;   // (A/B of RTW_WORLD_YIELD 12 / 16 / 24 / 32: profiles/r05/world_lane_ab.txt)
constexpr uint32_t kLaneNodes = 256;  // AUTO traversal: per lane from this BVH size on
WorldLaunchCfg world_cfg(const rtw_world_s* w, const rtw_params* p, int dev) {
  WorldLaunchCfg c;
  // Kernel instantiation for the world's features (params.world_features
  // RTW_WORLD_FEATURES_ALL: the general kernel; every set gives the same bits)
  // and its BVH traversal (params.world_traversal): per lane for sphere worlds
  // whose BVH fits the per-lane stack, else the wave's union walk.
  const uint32_t feat = p->world_features == RTW_WORLD_FEATURES_ALL ? 15u : w->feat;
  // AUTO: per lane on BVHs of >= kLaneNodes nodes (configs[4]'s globe: 5,802
  // nodes, +30 %); the union walk on small trees, where the lanes' paths
  // mostly coincide (scene 1's 23 nodes: the union 17 % faster).
  const bool lane_ok = w->view.n_nodes > 0 && w->info[2] <= rtwk::kLaneStack && w->info[3] <= rtwk::kMaxLeafPrims &&
                       w->view.n_prims + 1u < (1u << rtwk::kTravPosBits);
  const bool lane = lane_ok && (p->world_traversal == RTW_WORLD_TRAVERSAL_LANE ||
                                (p->world_traversal == RTW_WORLD_TRAVERSAL_AUTO && w->view.n_nodes >= kLaneNodes));
  const char* up = rtw_dev_knob("RTW_WORLD_UNPACKED");  // development knob (A/B): the per-lane walk loads the refs
  const bool packed = lane && w->packed && !(up && *up == '1');
  c.fs = rtwk::world_feature_set(feat, lane, packed);
  c.lds = rtwk::world_lds_bytes(w->view.n_perlins, c.fs);
  // Register-allocation target in waves per SIMD (params.world_waves, 0 = the
  // feature set's default).
  const int occ = p->world_waves ? (int)p->world_waves : world_occ_default(w);
  c.oi = occ >= 4 ? 4 : (occ == 3 ? 3 : 1);
  static std::mutex mu;
  static int bpc_cache[64][5] = {};
  static size_t bpc_lds[64][5] = {};
  int bpc;
  {
    std::lock_guard<std::mutex> lk(mu);
    if (bpc_cache[c.fs][c.oi] == 0 || bpc_lds[c.fs][c.oi] != c.lds)
      bpc_cache[c.fs][c.oi] = rtwk::world_blocks_per_cu(c.lds, c.oi, c.fs), bpc_lds[c.fs][c.oi] = c.lds;
    bpc = bpc_cache[c.fs][c.oi];
  }
  c.bpc = bpc;
  const uint32_t units = rtw_total_units(p);
  const uint32_t want = (units + 255) / 256;
  c.grid = std::max(1u, std::min((uint32_t)(rtw_device_cus(dev) * bpc), want));
  c.ring_off = (rtw_ws_total(p) + 255) & ~(size_t)255;
  c.ring_bytes = (size_t)c.grid * rtwk::kWorldBlock * rtwk::kTailWin * 3 * sizeof(double);
  return c;
}

int world_launch(rtw_world w, const rtw_camera* cam, const rtw_params* p, void* ws, size_t ws_bytes,
                 uint8_t* d_rgb, float* d_mean, hipStream_t stream, rtw_timer timer, int mode,
                 uint32_t* tail_ran = nullptr) {
  if (!w || !cam) return rtw_fail(RTW_EINVAL, "world/camera is NULL");
  const int v = rtw_validate_params(p);
  if (v != RTW_OK) return v;
  if (p->precision != RTW_PRECISION_F64 || p->engine != RTW_ENGINE_MEGAKERNEL)
    return rtw_fail(RTW_UNSUPPORTED, "world renders run in f64 on the megakernel engine");
  if (w->has_moving && w->view.n_nodes && (cam->time0 < 0.0 || cam->time1 > 1.0))
    return rtw_fail(RTW_UNSUPPORTED, "BVH boxes of moving spheres cover shutter times [0, 1] only");
  const size_t need = rtw_ws_total(p);
  if (!ws || ws_bytes < need) return rtw_fail(RTW_EINVAL, "workspace %zu bytes < required %zu", ws_bytes, need);
  if ((reinterpret_cast<uintptr_t>(ws) & 255) != 0) return rtw_fail(RTW_EINVAL, "workspace not 256-B aligned");
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return rtw_fail(RTW_ENODEV, "no HIP device");
  if (dev != w->device) return rtw_fail(RTW_EINVAL, "world lives on device %d, current is %d", w->device, dev);
  auto* wsb = static_cast<unsigned char*>(ws);
  if (hipMemsetAsync(wsb + rtw_ws_counter_off(p), 0, 512, stream) != hipSuccess)
    return rtw_fail(RTW_EHIP, "workspace reset failed");
  rtwk::WorldArgs a;
  std::memset(&a, 0, sizeof(a));
  rtw_fill_trace_args(a.t, cam, p, wsb);
  a.w = w->view;
  a.margin = bvh_margin(w, cam);
  a.counts = reinterpret_cast<unsigned long long*>(wsb + rtw_ws_stats_off(p));
  const WorldLaunchCfg c = world_cfg(w, p, dev);
  // Tail dealing (default; development knob RTW_WORLD_TAIL=0: off) needs the
  // rings in the workspace (rtw_world_workspace_bytes); a workspace of only
  // rtw_workspace_bytes(params) renders without it — the same image, and
  // rtw_world_render_counts_ex reports which ran.
  const char* te = rtw_dev_knob("RTW_WORLD_TAIL");
  a.tail_deal = ((te && *te == '0') || ws_bytes < c.ring_off + c.ring_bytes) ? 0u : 1u;
  a.ring = a.tail_deal ? reinterpret_cast<double*>(wsb + c.ring_off) : nullptr;
  // per-lane traversal: pause a wave's walks once fewer than this many lanes
  // still walk (development knob RTW_WORLD_YIELD)
  const char* ye = rtw_dev_knob("RTW_WORLD_YIELD");
  a.lane_yield = (ye && *ye) ? (uint32_t)atoi(ye) : kLaneYield;
  if (tail_ran) *tail_ran = a.tail_deal;
  const size_t lds = c.lds;
  const uint32_t grid = c.grid;
  const int oi = c.oi, fs = c.fs;
  if (timer && rtw_timer_mark(timer, stream, true) != RTW_OK) return RTW_EHIP;
  hipError_t e = rtwk::launch_world(a, grid, lds, stream, mode, oi, fs);
  if (e != hipSuccess) return rtw_fail(RTW_EHIP, "world kernel launch: %s", hipGetErrorString(e));
  if (timer && rtw_timer_mark(timer, stream, false) != RTW_OK) return RTW_EHIP;
  if (d_rgb) return rtw_launch_finalize(p, wsb, d_rgb, d_mean, stream);
  return RTW_OK;
}

}  // namespace

extern "C" {

size_t rtw_world_workspace_bytes(rtw_world w, const rtw_params* p) {
  if (!w || rtw_validate_params(p) != RTW_OK) return 0;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev != w->device) {
    rtw_fail(RTW_EINVAL, "rtw_world_workspace_bytes: the world's device must be current");
    return 0;
  }
  const WorldLaunchCfg c = world_cfg(w, p, dev);
  return c.ring_off + c.ring_bytes;
}

int rtw_world_launch_info(rtw_world w, const rtw_params* p, uint32_t info_out[6]) {
  if (!w || !info_out) return rtw_fail(RTW_EINVAL, "world/info is NULL");
  const int v = rtw_validate_params(p);
  if (v != RTW_OK) return v;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev != w->device)
    return rtw_fail(RTW_EINVAL, "rtw_world_launch_info: the world's device must be current");
  const WorldLaunchCfg c = world_cfg(w, p, dev);
  info_out[0] = w->view.n_nodes == 0 ? RTW_WORLD_TRAVERSAL_LINEAR
                                     : ((c.fs & 16) ? RTW_WORLD_TRAVERSAL_LANE : RTW_WORLD_TRAVERSAL_UNION);
  info_out[1] = (uint32_t)c.fs;
  info_out[2] = (uint32_t)c.oi;
  info_out[3] = (uint32_t)c.bpc;
  info_out[4] = c.grid;
  info_out[5] = (uint32_t)c.lds;
  return RTW_OK;
}

int rtw_world_render_device(rtw_world w, const rtw_camera* cam, const rtw_params* p, void* ws, size_t ws_bytes,
                            uint8_t* d_rgb, float* d_mean, void* stream, rtw_timer timer) {
  if (!d_rgb) return rtw_fail(RTW_EINVAL, "d_rgb is NULL");
  return world_launch(w, cam, p, ws, ws_bytes, d_rgb, d_mean, static_cast<hipStream_t>(stream), timer, 0);
}

int rtw_world_render_counts_ex(rtw_world w, const rtw_camera* cam, const rtw_params* p, void* ws, size_t ws_bytes,
                               uint64_t counts_out[8]) {
  if (!counts_out) return rtw_fail(RTW_EINVAL, "counts is NULL");
#ifdef RTW_MEASURE
  // RTW_WORLD_PHASE=1 (diagnostic build): a phase-stamp pass first; its wave-cycle
  // shares go to stderr (tools/world_bench.py --phase).
  const char* ph = rtw_dev_knob("RTW_WORLD_PHASE");
  if (ph && *ph == '1') {
    int st2 = world_launch(w, cam, p, ws, ws_bytes, nullptr, nullptr, nullptr, nullptr, 2);
    if (st2 != RTW_OK) return st2;
    unsigned long long q[5];
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(q, static_cast<unsigned char*>(ws) + rtw_ws_stats_off(p) + 8 * 8, sizeof(q), hipMemcpyDeviceToHost) !=
            hipSuccess)
      return rtw_fail(RTW_EHIP, "world phase pass failed");
    double tot = 0;
    for (auto x : q) tot += (double)x;
    const char* nm[5] = {"tail/loop", "sample start + units", "node visits", "leaf primitives", "shading"};
    for (int i = 0; i < 5; ++i) fprintf(stderr, "[world phase] %-22s %6.2f %%\n", nm[i], 100.0 * (double)q[i] / tot);
  }
#endif
  uint32_t tail = 0;
  const int st = world_launch(w, cam, p, ws, ws_bytes, nullptr, nullptr, nullptr, nullptr, 1, &tail);
  if (st != RTW_OK) return st;
  if (hipDeviceSynchronize() != hipSuccess) return rtw_fail(RTW_EHIP, "world counts pass failed");
  unsigned long long c[7];
  if (hipMemcpy(c, static_cast<unsigned char*>(ws) + rtw_ws_stats_off(p), sizeof(c), hipMemcpyDeviceToHost) !=
      hipSuccess)
    return rtw_fail(RTW_EHIP, "counts copy failed");
  for (int i = 0; i < 5; ++i) counts_out[i] = c[i];  // samples, segments, node visits, primitive tests, wave iterations
  counts_out[5] = tail;
  counts_out[6] = c[5];  // per-lane traversal: interior-step wave iterations
  counts_out[7] = c[6];  // and leaf-test wave iterations
  return RTW_OK;
}

int rtw_world_render_counts(rtw_world w, const rtw_camera* cam, const rtw_params* p, void* ws, size_t ws_bytes,
                            uint64_t counts_out[4]) {
  if (!counts_out) return rtw_fail(RTW_EINVAL, "counts is NULL");
  uint64_t c[8];
  const int st = rtw_world_render_counts_ex(w, cam, p, ws, ws_bytes, c);
  if (st == RTW_OK)
    for (int i = 0; i < 4; ++i) counts_out[i] = c[i];
  return st;
}

int rtw_world_render(const rtw_camera* cam, const rtw_world_desc* desc, const rtw_params* p, uint8_t* rgb_out,
                     float* mean_out) {
  if (!cam || !desc || !rgb_out) return rtw_fail(RTW_EINVAL, "camera/desc/rgb_out is NULL");
  const int v = rtw_validate_params(p);
  if (v != RTW_OK) return v;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return rtw_fail(RTW_ENODEV, "no HIP device visible");
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return rtw_fail(RTW_EHIP, "hipGetDevice failed");
  const int dev = p->device < 0 ? prev : p->device;
  if (dev >= ndev) return rtw_fail(RTW_EINVAL, "device %d >= device count %d", dev, ndev);
  if (hipSetDevice(dev) != hipSuccess) return rtw_fail(RTW_EHIP, "hipSetDevice failed");
  rtw_world w = nullptr;
  int st = rtw_world_create(desc, 0, &w);
  const size_t wsb = st == RTW_OK ? rtw_world_workspace_bytes(w, p) : 0, pix = (size_t)p->row_count * p->width * 3;
  void *ws = nullptr, *d_rgb = nullptr, *d_mean = nullptr;
  if (st == RTW_OK && (hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(&d_rgb, pix) != hipSuccess ||
                       (mean_out && hipMalloc(&d_mean, pix * sizeof(float)) != hipSuccess)))
    st = rtw_fail(RTW_ENOMEM, "rtw_world_render: device allocation failed");
  if (st == RTW_OK)
    st = world_launch(w, cam, p, ws, wsb, static_cast<uint8_t*>(d_rgb), static_cast<float*>(d_mean), nullptr,
                      nullptr, 0);
  if (st == RTW_OK && hipDeviceSynchronize() != hipSuccess) st = rtw_fail(RTW_EHIP, "world render failed on the device");
  if (st == RTW_OK && hipMemcpy(rgb_out, d_rgb, pix, hipMemcpyDeviceToHost) != hipSuccess)
    st = rtw_fail(RTW_EHIP, "copy of rgb_out failed");
  if (st == RTW_OK && mean_out && hipMemcpy(mean_out, d_mean, pix * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    st = rtw_fail(RTW_EHIP, "copy of mean_out failed");
  if (ws) (void)hipFree(ws);
  if (d_rgb) (void)hipFree(d_rgb);
  if (d_mean) (void)hipFree(d_mean);
  rtw_world_destroy(w);
  (void)hipSetDevice(prev);
  return st;
}

}  // extern "C"
