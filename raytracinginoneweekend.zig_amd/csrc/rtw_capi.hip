// rtw_capi.hip — the C ABI (include/rtw_hip.h): validation, scene upload,
// workspace sizing, kernel launches.  Replaces the render loop of
// src/main.zig:378-402.  No exception and no C++ type crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "rtw_hip.h"
#include "rtw_cull.hpp"
#include "rtw_internal.hpp"
#include "rtw_math.hpp"

namespace {

thread_local std::string g_err;

int fail(int status, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return status;
}
#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return fail(RTW_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// Development knobs (tools/, A/B measurement) are read from the environment
// only in the -DRTW_MEASURE build; the product library's behaviour depends on
// its arguments alone (engine configuration: rtw_params, ABI v4).
const char* dev_knob(const char* name) {
#ifdef RTW_MEASURE
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

uint64_t splitmix_first(uint64_t seed) {  // SplitMix64.init(seed).next()
  uint64_t z = seed + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct DevInfo {
  int cus = 0;
  std::map<std::pair<int, int>, std::pair<size_t, int>> bpc;  // (precision, var) -> (lds, blocks per CU)
};
std::mutex g_dev_mu;
std::map<int, DevInfo> g_dev;

int device_cus(int dev) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto& d = g_dev[dev];
  if (d.cus == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    d.cus = v;
  }
  return d.cus;
}
int blocks_per_cu(int dev, int prec, size_t lds, int var) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto& d = g_dev[dev];
  auto& e = d.bpc[{prec, var}];
  if (e.second == 0 || e.first != lds) e = {lds, rtwk::trace_blocks_per_cu(prec, lds, var)};
  return e.second;
}
// Wavefront bounce kernels: resident workgroups per CU (cached per device).
int wf_bpc(int dev, int prec, int kernel, size_t lds) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto& e = g_dev[dev].bpc[{prec, -kernel}];
  if (e.second == 0 || e.first != lds) e = {lds, rtwk::wf_blocks_per_cu(prec, kernel, lds)};
  return e.second;
}
// Kernel tuning variant (rtw_trace.hip VAR bits): the product library holds
// one per precision (rtw_internal.hpp kDefaultVarF64 / kDefaultVarF32).
// RTW_VARIANT selects another one of a -DRTW_MEASURE build (tools/); a value
// that was not compiled in is refused by launch_all.
int kernel_variant(uint32_t precision) {
  const char* v = dev_knob("RTW_VARIANT");
  if (v && *v) return atoi(v);
  return precision == RTW_PRECISION_F32 ? rtwk::kDefaultVarF32 : rtwk::kDefaultVarF64;
}

}  // namespace

struct rtw_scene_s {
  int device = 0;
  uint32_t n = 0, nm = 0, ng = 0;
  uint32_t n_static = 0, n_moving = 0, n_wide = 0;
  void* buf = nullptr;  // one allocation holding every table
  std::vector<std::pair<double, double>> groups;  // moving-sphere time groups (t0, t1)
  float cull_cmax_cl = 0.0f;                       // Cmax over members and cluster centres
  rtwk::SceneView<double> v64{};
  rtwk::SceneView<float> v32{};
};

struct rtw_timer_s {
  hipEvent_t start = nullptr, stop = nullptr;
  bool recorded = false;
};

struct rtw_sclk_probe_s {
  double* d = nullptr;  // [0] = MHz (device)
  hipStream_t s = nullptr;
};

namespace {
// One wave: spin (s_sleep between reads) until `ticks` of the constant-rate
// s_memrealtime counter passed; the SIMD clock = delta(s_memtime) /
// delta(s_memrealtime) x the counter's rate (hipDeviceAttributeWallClockRate,
// 100 MHz on MI355X; MI355X_MICROARCH.md: in-kernel clock).  Lane 0 writes it.
__global__ void __launch_bounds__(64) sclk_probe_kernel(unsigned long long ticks, double rt_mhz, double* out) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r = r0;
  while (r - r0 < ticks) {
    __builtin_amdgcn_s_sleep(63);
    r = __builtin_amdgcn_s_memrealtime();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = (double)(t1 - t0) / (double)(r - r0) * rt_mhz;
}
}  // namespace

extern "C" {

int rtw_abi_version(void) { return RTW_ABI_VERSION; }

const char* rtw_last_error(void) { return g_err.c_str(); }

int rtw_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int rtw_scene_create(const rtw_sphere* spheres, uint32_t n, const rtw_material* mats, uint32_t nm,
                     rtw_scene* out) {
  if (!out) return fail(RTW_EINVAL, "rtw_scene_create: out is NULL");
  *out = nullptr;
  if (n > 0 && !spheres) return fail(RTW_EINVAL, "rtw_scene_create: spheres is NULL");
  if (nm > 0 && !mats) return fail(RTW_EINVAL, "rtw_scene_create: materials is NULL");
  if (n > RTW_MAX_SPHERES || nm > RTW_MAX_SPHERES)
    return fail(RTW_UNSUPPORTED, "rtw_scene_create: %u spheres / %u materials exceeds %u (BVH path not built)",
                n, nm, RTW_MAX_SPHERES);
  for (uint32_t i = 0; i < nm; ++i) {
    if (mats[i].kind > RTW_DIELECTRIC)
      return fail(RTW_UNSUPPORTED, "material %u: kind %u not supported on the GPU path", i, mats[i].kind);
  }
  // Distinct (t0, t1) pairs of moving spheres -> time groups.
  std::vector<std::pair<double, double>> groups;
  std::vector<uint32_t> meta_orig(n, 0u);
  uint32_t n_moving = 0, n_wide = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const rtw_sphere& s = spheres[i];
    if (s.mat >= nm) return fail(RTW_EINVAL, "sphere %u: material index %u >= %u", i, s.mat, nm);
    if (s.moving > 1) return fail(RTW_EINVAL, "sphere %u: moving flag %u", i, s.moving);
    uint32_t m = (s.mat << 8) | (i << 20);
    if (s.moving) {
      ++n_moving;
      uint32_t g = 0;
      while (g < groups.size() && !(groups[g].first == s.t0 && groups[g].second == s.t1)) ++g;
      if (g == groups.size()) {
        if (groups.size() >= rtwk::kMaxTimeGroups)
          return fail(RTW_UNSUPPORTED, "more than %u distinct moving-sphere time ranges", rtwk::kMaxTimeGroups);
        groups.emplace_back(s.t0, s.t1);
      }
      m |= rtwk::kMoving | (g << 2);
    }
    if (s.radius >= rtwk::kWideRadius) {
      m |= rtwk::kWide;
      ++n_wide;
    }
    meta_orig[i] = m;
  }
  // Table order [static wide | static | moving wide | moving], list order within
  // each group (rtw_internal.hpp); pos_of[i] = table position of sphere i.
  std::vector<uint32_t> order;
  order.reserve(n);
  for (int grp = 0; grp < 4; ++grp)
    for (uint32_t i = 0; i < n; ++i) {
      const bool mv = (meta_orig[i] & rtwk::kMoving) != 0, wd = (meta_orig[i] & rtwk::kWide) != 0;
      if ((int)mv * 2 + (int)!wd == grp) order.push_back(i);
    }
  uint32_t g_end[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i < n; ++i) {
    const bool mv = (meta_orig[i] & rtwk::kMoving) != 0, wd = (meta_orig[i] & rtwk::kWide) != 0;
    for (int grp = (int)mv * 2 + (int)!wd; grp < 4; ++grp) ++g_end[grp];
  }
  std::vector<uint32_t> meta(n + 1, 0u), perm(n, 0u);
  for (uint32_t k = 0; k < n; ++k) {
    meta[k] = meta_orig[order[k]];
    perm[order[k]] = k;
  }
  const uint32_t ng = (uint32_t)groups.size();
  // Host tables (rtw_internal.hpp has the layout).  Reciprocals are correctly
  // rounded IEEE divisions: the kernel's div_rn needs y = RN(1/b).
  // sph / meta carry one zero padding record: the sphere loop prefetches k+1.
  std::vector<double> sph64((size_t)8 * (n + 1), 0.0), rad64(n), mat64((size_t)8 * nm), tg64((size_t)4 * ng);
  std::vector<float> sph32((size_t)8 * (n + 1), 0.0f), rad32(n), mat32((size_t)8 * nm), tg32((size_t)4 * ng);
  std::vector<uint32_t> kind(nm);
  for (uint32_t i = 0; i < n; ++i) {  // i = table position
    const rtw_sphere& s = spheres[order[i]];
    const double rec[8] = {s.c0[0], s.c0[1], s.c0[2], s.c1[0] - s.c0[0], s.c1[1] - s.c0[1], s.c1[2] - s.c0[2],
                           s.radius * s.radius, 1.0 / s.radius};
    for (int k = 0; k < 8; ++k) sph64[8 * i + k] = rec[k];
    for (int k = 0; k < 6; ++k) sph32[8 * i + k] = (float)rec[k];
    const float rf = (float)s.radius;
    sph32[8 * i + 6] = rf * rf;  // f32 mode: r*r in f32 (tierb_core.h prep)
    sph32[8 * i + 7] = 1.0f / rf;
    rad64[i] = s.radius;
    rad32[i] = rf;
  }
  for (uint32_t i = 0; i < nm; ++i) {
    const rtw_material& m = mats[i];
    const bool diel = m.kind == RTW_DIELECTRIC;
    const double rec[8] = {m.albedo[0], m.albedo[1], m.albedo[2], m.albedo_odd[0], m.albedo_odd[1],
                           m.albedo_odd[2], diel ? 1.0 / m.ir : m.fuzz, m.ir};
    for (int k = 0; k < 8; ++k) {
      mat64[8 * i + k] = rec[k];
      mat32[8 * i + k] = (float)rec[k];
    }
    if (diel) {
      mat32[8 * i + 6] = 1.0f / (float)m.ir;
      // Schlick's r0^2 (material.zig:87-91) for ratio = RN(1/ir) (front face)
      // and ir (back face), with the kernel's operations in each precision.
      for (int f = 0; f < 2; ++f) {
        const double rd = f == 0 ? mat64[8 * i + 6] : m.ir;
        const double r0d = (1.0 - rd) / (1.0 + rd);
        mat64[8 * i + f] = r0d * r0d;
        const float rf = f == 0 ? mat32[8 * i + 6] : (float)m.ir;
        const float r0f = (1.0f - rf) / (1.0f + rf);
        mat32[8 * i + f] = r0f * r0f;
      }
    }
    kind[i] = m.kind;
  }
  for (uint32_t g = 0; g < ng; ++g) {
    const double t0 = groups[g].first, t1 = groups[g].second;
    tg64[4 * g] = t0;
    tg64[4 * g + 1] = t1;
    tg64[4 * g + 2] = 1.0 / (t1 - t0);
    const float f0 = (float)t0, f1 = (float)t1;
    tg32[4 * g] = f0;
    tg32[4 * g + 1] = f1;
    tg32[4 * g + 2] = 1.0f / (f1 - f0);
  }
  // Pretest records (rtw_cull.hpp) over the narrow spheres in table order.
  const uint32_t n_sn = g_end[1] - g_end[0], nn = n_sn + (n - g_end[2]);
  const uint32_t nn_pad = (nn + 31u) & ~31u;
  std::vector<float> cull((size_t)8 * nn_pad + 16, 0.0f);  // + one padding pair (prefetch)
  std::vector<uint32_t> cull_tg(nn_pad / 2 + 1, 0u);
  double cmax_c = 0.0, cmax_d = 0.0, rho_max = 1.0;
  for (uint32_t j = 0; j < nn; ++j) {
    const uint32_t pos = j < n_sn ? g_end[0] + j : g_end[2] + (j - n_sn);
    const double* r = &sph64[8 * pos];
    float* q = &cull[(size_t)16 * (j / 2) + (j & 1)];
    for (int k = 0; k < 3; ++k) {
      q[2 * k] = (float)r[k];
      q[2 * (3 + k)] = -(float)r[3 + k];
      cmax_c = std::max(cmax_c, std::fabs(r[k]));
      cmax_d = std::max(cmax_d, std::fabs(r[3 + k]));
    }
    const float rf = (float)rad64[pos];
    q[12] = -(rf * rf);
    rho_max = std::max(rho_max, 2.0 * r[6] + 1.0);
    const uint32_t g = (meta[pos] & rtwk::kMoving) ? (meta[pos] >> 2) & 63u : 0u;
    cull_tg[j / 2] |= g << (8 * (j & 1));
  }
  for (uint32_t j = nn; j < nn_pad; ++j)  // padding: same time group as its partner
    if (j & 1) cull_tg[j / 2] |= (cull_tg[j / 2] & 0xFFu) << 8;
  for (uint32_t j = 0; j + 1 < nn; j += 2) {  // static half of a mixed pair: partner's group
    const bool m0 = j >= n_sn, m1 = j + 1 >= n_sn;
    if (!m0 && m1) cull_tg[j / 2] = (cull_tg[j / 2] & 0xFF00u) | (cull_tg[j / 2] >> 8);
  }
  // bit 16: both spheres of the pair move along y only (ndc.x == ndc.z == 0):
  // the kernel's pretest then skips the x and z centre updates.
  for (uint32_t p = 0; p < nn_pad / 2; ++p) {
    const float* q = &cull[(size_t)16 * p];
    if (q[6] == 0.0f && q[7] == 0.0f && q[10] == 0.0f && q[11] == 0.0f) cull_tg[p] |= 1u << 16;
  }
  const float cmax = std::nextafter((float)(cmax_c + cmax_d), INFINITY);
  const float rho = std::nextafter((float)rho_max, INFINITY);
  const uint32_t cull_on = (nn > 0 && cmax <= rtwc::kCmaxLimit) ? 1u : 0u;
  // Clustered pretest tables (SceneView ccull..., trace VAR kVarCluster).
  // kd-split of the narrow spheres (by the centre of their swept box over
  // the shutter) into clusters of <= 8; members static first, so pairs are
  // static-static where possible.  Bounding sphere of cluster c: centre
  // C = f32(centre of the members' swept box), radius R = max over members
  // of max(|c0 - C|, |c1 - C|) + |r|, widened by 1e-4 (1 + R): a line whose
  // f64 discriminant for (C, R) is negative passes every member at a distance
  // above its radius + 1e-4, far beyond the f64 rounding of the member's own
  // exact test, which therefore rejects it.  Valid for
  // sphere times within each time group's [t0, t1] (checked per render).
  std::vector<uint32_t> cl_items;  // j (narrow index) per slot, ~0u = dummy
  std::vector<float> cclus;
  double cmax_cl = 0.0, rho_cl = 1.0;
  {
    auto cen_of = [&](uint32_t j, int k) {
      const uint32_t pos = j < n_sn ? g_end[0] + j : g_end[2] + (j - n_sn);
      const double* r = &sph64[8 * pos];
      return r[k] + 0.5 * r[3 + k];
    };
    std::vector<std::vector<uint32_t>> groups;
    std::vector<uint32_t> all(nn);
    for (uint32_t j = 0; j < nn; ++j) all[j] = j;
    if (nn) groups.push_back(all);
    for (bool again = true; again;) {
      again = false;
      for (size_t gi = 0; gi < groups.size(); ++gi) {
        if (groups[gi].size() <= rtwk::kClusterSlots) continue;
        std::vector<uint32_t> g = groups[gi];
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t j : g)
          for (int k = 0; k < 3; ++k) lo[k] = std::min(lo[k], cen_of(j, k)), hi[k] = std::max(hi[k], cen_of(j, k));
        int ax = 0;
        for (int k = 1; k < 3; ++k)
          if (hi[k] - lo[k] > hi[ax] - lo[ax]) ax = k;
        std::stable_sort(g.begin(), g.end(), [&](uint32_t a, uint32_t b) { return cen_of(a, ax) < cen_of(b, ax); });
        // Split sizes: whole clusters of 8 on the left, ceil(n/8) clusters in
        // all (profiles/r02/cluster_ab.txt: fewer, fuller clusters beat
        // smaller ones whose bounds are tighter: each cluster costs a ballot
        // and a branch per wave-iteration).
        constexpr size_t CS = rtwk::kClusterSlots;
        const size_t h = CS * (((g.size() + CS - 1) / CS) / 2);
        groups[gi].assign(g.begin(), g.begin() + h);
        groups.emplace_back(g.begin() + h, g.end());
        again = true;
      }
    }
    for (auto& g : groups) {
      std::stable_sort(g.begin(), g.end(), [&](uint32_t a, uint32_t b) { return (a >= n_sn) < (b >= n_sn); });
      double mc0[rtwk::kClusterSlots][3], mdc[rtwk::kClusterSlots][3], mr[rtwk::kClusterSlots];
      for (size_t i = 0; i < g.size(); ++i) {
        const uint32_t pos = g[i] < n_sn ? g_end[0] + g[i] : g_end[2] + (g[i] - n_sn);
        for (int k = 0; k < 3; ++k) mc0[i][k] = sph64[8 * pos + k], mdc[i][k] = sph64[8 * pos + 3 + k];
        mr[i] = rad64[pos];
      }
      float cf[3], rf;
      rtwc::cluster_sphere(mc0, mdc, mr, (int)g.size(), cf, rf);
      const size_t c = cl_items.size() / rtwk::kClusterSlots;
      if (cclus.size() < 16 * (c / 2 + 1)) cclus.resize(16 * (c / 2 + 1), 0.0f);
      float* q = &cclus[16 * (c / 2) + (c & 1)];
      for (int k = 0; k < 3; ++k) q[2 * k] = cf[k], cmax_cl = std::max(cmax_cl, (double)std::fabs(cf[k]));
      q[12] = -(rf * rf);
      rho_cl = std::max(rho_cl, 2.0 * (double)rf * (double)rf + 1.0);
      for (uint32_t i = 0; i < rtwk::kClusterSlots; ++i) cl_items.push_back(i < g.size() ? g[i] : ~0u);
    }
  }
  const uint32_t n_clusters = (uint32_t)(cl_items.size() / rtwk::kClusterSlots);
  const uint32_t n_cslots = rtwk::kClusterSlots * n_clusters;
  // slot tables; a dummy slot's record (c = 0, nr2 = +3e38) is a proven miss for every lane
  std::vector<float> ccull((size_t)8 * n_cslots + 16, 0.0f);
  std::vector<uint32_t> ccull_tg(n_cslots / 2 + 1, 0u), cpos(std::max(n_cslots, 1u), 0u);
  std::vector<uint32_t> cvalid(2 * ((n_cslots + 63) / 64) + 2, 0u);
  for (uint32_t sl = 0; sl < n_cslots; ++sl) {
    float* q = &ccull[(size_t)16 * (sl / 2) + (sl & 1)];
    const uint32_t j = cl_items[sl];
    if (j == ~0u) {
      q[12] = 3e38f;
      continue;
    }
    const uint32_t pos = j < n_sn ? g_end[0] + j : g_end[2] + (j - n_sn);
    const float* src = &cull[(size_t)16 * (j / 2) + (j & 1)];  // the member's own pretest record
    for (int k = 0; k < 7; ++k) q[2 * k] = src[2 * k];
    cpos[sl] = pos;
    cvalid[2 * (sl / 64) + ((sl % 64) >> 5)] |= 0x80000000u >> (sl & 31u);
    const uint32_t g = (meta[pos] & rtwk::kMoving) ? (meta[pos] >> 2) & 63u : 0u;
    ccull_tg[sl / 2] |= g << (8 * (sl & 1));
  }
  for (uint32_t p = 0; p < n_cslots / 2; ++p) {
    const uint32_t j0 = cl_items[2 * p], j1 = cl_items[2 * p + 1];
    const bool m0 = j0 != ~0u && j0 >= n_sn, m1 = j1 != ~0u && j1 >= n_sn;
    if (!m0 && !m1) ccull_tg[p] |= 1u << 17;  // static pair (dummies count as static)
    if (!m0 && m1) ccull_tg[p] = (ccull_tg[p] & 0xFF00u) | ((ccull_tg[p] >> 8) & 0xFFu) | (ccull_tg[p] & ~0xFFFFu);
    if (m0 && !m1) ccull_tg[p] = (ccull_tg[p] & 0xFFu) | ((ccull_tg[p] & 0xFFu) << 8) | (ccull_tg[p] & ~0xFFFFu);
    const float* q = &ccull[(size_t)16 * p];
    if (q[6] == 0.0f && q[7] == 0.0f && q[10] == 0.0f && q[11] == 0.0f) ccull_tg[p] |= 1u << 16;
  }
  if (cclus.empty()) cclus.assign(16, 0.0f);
  const float cmax_all = std::max(cmax, std::nextafter((float)cmax_cl, INFINITY));
  const float rho_c = std::nextafter((float)rho_cl, INFINITY);
  // One device allocation, 256-B aligned sub-buffers.
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  size_t off = 0;
  auto place = [&](size_t bytes) {
    const size_t o = off;
    off += al(bytes + 8);
    return o;
  };
  const size_t o_sph64 = place(sph64.size() * 8), o_rad64 = place(rad64.size() * 8);
  const size_t o_mat64 = place(mat64.size() * 8), o_tg64 = place(tg64.size() * 8);
  const size_t o_sph32 = place(sph32.size() * 4), o_rad32 = place(rad32.size() * 4);
  const size_t o_mat32 = place(mat32.size() * 4), o_tg32 = place(tg32.size() * 4);
  const size_t o_meta = place(meta.size() * 4), o_kind = place(kind.size() * 4), o_perm = place(perm.size() * 4);
  const size_t o_cull = place(cull.size() * 4), o_cull_tg = place(cull_tg.size() * 4);
  const size_t o_ccull = place(ccull.size() * 4), o_ccull_tg = place(ccull_tg.size() * 4);
  const size_t o_cclus = place(cclus.size() * 4), o_cpos = place(cpos.size() * 4), o_cvalid = place(cvalid.size() * 4);
  const size_t total = off;
  std::vector<unsigned char> host(total, 0);
  auto cp = [&](size_t o, const void* p, size_t bytes) {
    if (bytes) std::memcpy(host.data() + o, p, bytes);
  };
  cp(o_sph64, sph64.data(), sph64.size() * 8);
  cp(o_rad64, rad64.data(), rad64.size() * 8);
  cp(o_mat64, mat64.data(), mat64.size() * 8);
  cp(o_tg64, tg64.data(), tg64.size() * 8);
  cp(o_sph32, sph32.data(), sph32.size() * 4);
  cp(o_rad32, rad32.data(), rad32.size() * 4);
  cp(o_mat32, mat32.data(), mat32.size() * 4);
  cp(o_tg32, tg32.data(), tg32.size() * 4);
  cp(o_meta, meta.data(), meta.size() * 4);
  cp(o_kind, kind.data(), kind.size() * 4);
  cp(o_perm, perm.data(), perm.size() * 4);
  cp(o_cull, cull.data(), cull.size() * 4);
  cp(o_cull_tg, cull_tg.data(), cull_tg.size() * 4);
  cp(o_ccull, ccull.data(), ccull.size() * 4);
  cp(o_ccull_tg, ccull_tg.data(), ccull_tg.size() * 4);
  cp(o_cclus, cclus.data(), cclus.size() * 4);
  cp(o_cpos, cpos.data(), cpos.size() * 4);
  cp(o_cvalid, cvalid.data(), cvalid.size() * 4);

  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  void* d = nullptr;
  if (hipMalloc(&d, total) != hipSuccess) return fail(RTW_ENOMEM, "rtw_scene_create: hipMalloc(%zu)", total);
  if (hipMemcpy(d, host.data(), total, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(d);
    return fail(RTW_EHIP, "rtw_scene_create: hipMemcpy failed");
  }
  auto* sc = new rtw_scene_s;
  sc->device = dev;
  sc->n = n;
  sc->nm = nm;
  sc->ng = ng;
  sc->n_moving = n_moving;
  sc->n_static = n - n_moving;
  sc->n_wide = n_wide;
  sc->buf = d;
  auto* b = static_cast<unsigned char*>(d);
  auto D = [&](size_t o) { return reinterpret_cast<const double*>(b + o); };
  auto F = [&](size_t o) { return reinterpret_cast<const float*>(b + o); };
  auto U = [&](size_t o) { return reinterpret_cast<const uint32_t*>(b + o); };
  // cluster_on (per render, fill_args): usable when the scene's bound allows (cmax_all within the limit)
  const uint32_t cl_ok = (n_clusters > 0 && cull_on && cmax_all <= rtwc::kCmaxLimit) ? 1u : 0u;
  sc->v64 = {D(o_sph64), D(o_rad64), U(o_meta), D(o_mat64), U(o_kind), D(o_tg64), D(o_sph64), D(o_tg64), U(o_perm),
             F(o_cull), U(o_cull_tg), F(o_tg32), n, nm, ng, g_end[0], g_end[1], g_end[2], nn, nn_pad, n_sn, cull_on,
             cl_ok ? cmax_all : cmax, rho, F(o_ccull), U(o_ccull_tg), F(o_cclus), U(o_cpos), U(o_cvalid), n_clusters,
             cl_ok, rho_c};
  sc->v32 = {F(o_sph32), F(o_rad32), U(o_meta), F(o_mat32), U(o_kind), F(o_tg32), D(o_sph64), D(o_tg64), U(o_perm),
             F(o_cull), U(o_cull_tg), F(o_tg32), n, nm, ng, g_end[0], g_end[1], g_end[2], nn, nn_pad, n_sn, cull_on,
             cmax, rho, F(o_ccull), U(o_ccull_tg), F(o_cclus), U(o_cpos), U(o_cvalid), n_clusters, 0u, rho_c};
  sc->cull_cmax_cl = cmax_all;
  sc->groups = groups;
  *out = sc;
  return RTW_OK;
}

int rtw_scene_destroy(rtw_scene sc) {
  if (!sc) return RTW_OK;
  if (sc->buf) (void)hipFree(sc->buf);
  delete sc;
  return RTW_OK;
}

}  // extern "C"

namespace {

uint32_t eff_chunk(const rtw_params* p) {
  const uint32_t c = p->chunk ? p->chunk : RTW_DEFAULT_CHUNK;
  return std::min(c, p->spp);
}
uint32_t n_chunks(const rtw_params* p) {
  const uint32_t c = eff_chunk(p);
  return (p->spp + c - 1) / c;
}

int validate(const rtw_params* p) {
  if (!p) return fail(RTW_EINVAL, "params is NULL");
  if (p->width < 2 || p->height < 2)
    return fail(RTW_EINVAL, "image %ux%u: width and height must be >= 2 (main.zig:390-391 divide by W-1, H-1)",
                p->width, p->height);
  if (p->spp == 0) return fail(RTW_EINVAL, "spp must be >= 1");
  if ((uint64_t)p->width * p->height > (1ull << 24))
    return fail(RTW_UNSUPPORTED, "image of %llu pixels exceeds 2^24 (per-sample RNG key layout)",
                (unsigned long long)p->width * p->height);
  if (p->spp > (1u << 24)) return fail(RTW_UNSUPPORTED, "spp %u exceeds 2^24", p->spp);
  if (p->row_stride == 0 || p->row_count == 0) return fail(RTW_EINVAL, "row_stride and row_count must be >= 1");
  if ((uint64_t)p->row_begin + (uint64_t)(p->row_count - 1) * p->row_stride >= p->height)
    return fail(RTW_EINVAL, "rows %u + k*%u (k < %u) exceed height %u", p->row_begin, p->row_stride,
                p->row_count, p->height);
  if (p->precision > RTW_PRECISION_F32) return fail(RTW_EINVAL, "precision %u", p->precision);
  if (p->engine > RTW_ENGINE_WAVEFRONT) return fail(RTW_EINVAL, "engine %u", p->engine);
  if (p->wf_sets > RTW_MAX_WF_SETS) return fail(RTW_EINVAL, "wf_sets %u outside [0, %u]", p->wf_sets, RTW_MAX_WF_SETS);
  if (p->wf_drain > RTW_WF_DRAIN_NONE) return fail(RTW_EINVAL, "wf_drain %u", p->wf_drain);
  if (p->wf_form > RTW_WF_SPLIT) return fail(RTW_EINVAL, "wf_form %u", p->wf_form);
  if (p->world_waves > 4 || p->world_waves == 2)  // (compiled budgets: 1 = unconstrained, 3, 4)
    return fail(RTW_EINVAL, "world_waves %u is not 0, 1, 3 or 4", p->world_waves);
  if (p->world_features > RTW_WORLD_FEATURES_ALL) return fail(RTW_EINVAL, "world_features %u", p->world_features);
  if (p->world_traversal > RTW_WORLD_TRAVERSAL_LANE) return fail(RTW_EINVAL, "world_traversal %u", p->world_traversal);
  if (p->wf_bounces > 16) return fail(RTW_EINVAL, "wf_bounces %u outside [0, 16]", p->wf_bounces);
  if (p->wf_passes > 64) return fail(RTW_EINVAL, "wf_passes %u outside [0, 64]", p->wf_passes);
  if (p->engine == RTW_ENGINE_WAVEFRONT && (p->wf_paths > (1u << 28) || (p->wf_paths && p->wf_paths < 64)))
    return fail(RTW_EINVAL, "wf_paths %u outside [64, 2^28]", p->wf_paths);
  if (p->engine == RTW_ENGINE_WAVEFRONT && p->max_depth > 0xFFFFu)
    return fail(RTW_UNSUPPORTED, "wavefront engine: max_depth %u > 65535", p->max_depth);
  const uint64_t tiles = (uint64_t)((p->width + rtwk::kTileW - 1) / rtwk::kTileW) *
                         ((p->row_count + rtwk::kTileH - 1) / rtwk::kTileH);
  const uint64_t units = tiles * 64ull * n_chunks(p);
  if (units > 0x7FFFFFFFull)  // headroom: waves overshoot the queue by < 2^31 units
    return fail(RTW_UNSUPPORTED, "%llu work units exceed the 32-bit queue; raise params.chunk",
                (unsigned long long)units);
  return RTW_OK;
}

// Wavefront queue sets (params.wf_sets, default kWfSets): the in-flight paths
// are split over independent sets (queues, home slots, segment counts,
// reservoirs, drain ring), each driven on its own HIP stream, so one set's
// launch ramps, tails and drain overlap the other sets' bounce launches.  All
// sets take units from the one device queue: a unit belongs to one slot of
// one set, its chunk sum keeps its sample order, the image keeps its bits.
constexpr uint32_t kWfMaxSets = RTW_MAX_WF_SETS;
constexpr uint32_t kWfSets = RTW_DEFAULT_WF_SETS;
uint32_t wf_sets(const rtw_params* p) { return p->wf_sets ? p->wf_sets : kWfSets; }  // (validated: 1-4)
// The in-register drain (params.wf_drain): wf_drain (RTW_WF_DRAIN_SAMPLES,
// samples dealt to the wave's free lanes, default), wf_finish
// (RTW_WF_DRAIN_SLOTS: a lane runs its own slot's samples) or none.  Only
// wf_drain uses the drain ring, so only it reserves one.
bool wf_per_sample_drain(const rtw_params* p) { return p->wf_drain == RTW_WF_DRAIN_SAMPLES; }
// Segments of one queue set: its share of wf_paths rounded up to whole
// segments (one per wave).
uint32_t wf_segs(const rtw_params* p) {
  const uint32_t n = p->wf_paths ? p->wf_paths : RTW_DEFAULT_WF_PATHS;
  const uint32_t per_set = (n + wf_sets(p) - 1) / wf_sets(p);
  return std::max(1u, (per_set + rtwk::kSegCap - 1) / rtwk::kSegCap);
}

// Workspace: partial chunk sums | counters (unit queue head, one live-path
// poll word per queue set) | stats | wavefront region (engine 1 only,
// rtw_internal.hpp WfArgs): per queue set two path queues, the hit arrays,
// the home slots, per-segment counts (x2), unit reservoirs and (wf_drain
// only) the drain ring.
struct WsLayout {
  size_t partial_off, partial_bytes, counter_off, live_off, stats_off;
  size_t wf_off, wf_set_bytes, total;
};
size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }
// Byte size of one SoA path queue of n entries (10 R arrays, rs, slot, dsk, + the fused engine's hit root, winner).
// (10 R fields, the RNG state, slot, depth|skip, the fused engine's hit winner; round 6 dropped the
// hit root: a queued hit path carries its hit point in o)
size_t wf_queue_bytes(size_t n, size_t r) { return 10 * al256(n * r) + al256(n * 8) + 3 * al256(n * 4); }
WsLayout ws_layout(const rtw_params* p) {
  WsLayout w;
  w.partial_off = 0;
  w.partial_bytes = (size_t)n_chunks(p) * p->row_count * p->width * 3 * sizeof(double);
  w.counter_off = al256(w.partial_bytes);
  w.live_off = w.counter_off + 64;  // kWfMaxSets words; + 128: wf_step's live_acc pairs (kWfMaxSets x 2 words)
  w.stats_off = w.counter_off + 256;
  w.total = w.stats_off + 256;  // stats: 32 x u64
  w.wf_off = w.total;
  w.wf_set_bytes = 0;
  if (p->engine == RTW_ENGINE_WAVEFRONT) {
    const size_t segs = wf_segs(p), n = segs * rtwk::kSegCap;
    const size_t r = p->precision == RTW_PRECISION_F32 ? 4 : 8;
    w.wf_set_bytes = 2 * wf_queue_bytes(n, r) + al256(n * r) + al256(n * 4) + al256(n * sizeof(rtwk::HomeRec)) +
                     2 * al256(segs * 4) + al256(segs * 8) +
                     (wf_per_sample_drain(p) ? al256(n * rtwk::kDrainWin * 3 * r) : 0);
    w.total += wf_sets(p) * w.wf_set_bytes;
  }
  return w;
}

// Unit dealing order (rtw_device.hpp dealt_unit): the development knob
// RTW_UNIT_ORDER=fwd|rev overrides the engine's default (-DRTW_MEASURE only).
uint32_t unit_order(uint32_t dflt) {
  const char* uo = dev_knob("RTW_UNIT_ORDER");
  if (uo && std::strcmp(uo, "fwd") == 0) return 0u;
  if (uo && std::strcmp(uo, "rev") == 0) return 1u;
  return dflt;
}
constexpr uint32_t kWorldUnitOrder = 1u;

template <typename R>
void fill_args(rtwk::TraceArgs<R>& a, const rtwk::SceneView<R>& v, const rtw_camera* cam, const rtw_params* p,
               unsigned char* ws, const WsLayout& L) {
  std::memset(&a, 0, sizeof(a));
  a.sc = v;
  for (int k = 0; k < 3; ++k) {
    a.origin[k] = (R)cam->origin[k];
    a.horizontal[k] = (R)cam->horizontal[k];
    a.vertical[k] = (R)cam->vertical[k];
    a.llc[k] = (R)cam->lower_left_corner[k];
    a.cu[k] = (R)cam->u[k];
    a.cv[k] = (R)cam->v[k];
    a.bg[k] = (R)p->background[k];
  }
  a.lens_radius = (R)cam->lens_radius;
  a.time0 = (R)cam->time0;
  a.time1 = (R)cam->time1;
  a.tmin = (R)0.001;  // rayColor's t_min (main.zig:109)
  a.inv_w1 = (R)1 / ((R)p->width - (R)1);
  a.inv_h1 = (R)1 / ((R)p->height - (R)1);
  // Prefilter bound: root2 <= 2u(1+u)^2 * hb/a < tmin
  // whenever hb < pre_k * a, u = unit roundoff of R.
  const double u = sizeof(R) == 8 ? 0x1p-53 : 0x1p-24;
  a.pre_k = (R)((double)a.tmin / (2.5 * u));
  a.W = p->width;
  a.H = p->height;
  a.spp = p->spp;
  a.max_depth = p->max_depth;
  a.chunk = eff_chunk(p);
  a.n_chunks = n_chunks(p);
  a.row_begin = p->row_begin;
  a.row_stride = p->row_stride;
  a.row_count = p->row_count;
  a.tiles_x = (p->width + rtwk::kTileW - 1) / rtwk::kTileW;
  const uint32_t tiles_y = (p->row_count + rtwk::kTileH - 1) / rtwk::kTileH;
  a.total_units = a.tiles_x * tiles_y * 64u * a.n_chunks;
  const rtwm::UDivMagic mu = rtwm::udiv_magic(rtwk::kTileW * rtwk::kTileH * a.n_chunks), mt = rtwm::udiv_magic(a.tiles_x);
  a.upt_m = mu.m, a.upt_sh = mu.sh, a.tx_m = mt.m, a.tx_sh = mt.sh;
  a.seed_base = splitmix_first(p->seed);
  // Unit dealing order (rtw_device.hpp dealt_unit): image order, top rows
  // first, for the cover-scene engines, last-first for the world kernel
  // (rtw_fill_trace_args), each the faster in the in-process A/Bs
  // (profiles/r03/unit_order_ab.txt); RTW_UNIT_ORDER=fwd|rev overrides.
  a.unit_order = unit_order(0u);
  a.partial = reinterpret_cast<double*>(ws + L.partial_off);
  a.counter = reinterpret_cast<uint32_t*>(ws + L.counter_off);
  a.stats = reinterpret_cast<unsigned long long*>(ws + L.stats_off);
}

// n_clusters: clusters whose slot -> position table (cpos) is staged, 0 unless
// the launched kernel runs the clustered pretest (f64 megakernel with
// kVarCluster and clusters_usable): other paths neither read nor stage it.
size_t lds_bytes(const rtw_scene_s* sc, int prec, uint32_t n_clusters) {
  const size_t r = prec == 1 ? 4 : 8;
  return rtwk::kCoopLdsBytes + r * (8 * ((size_t)sc->n + 1) + (size_t)sc->n + 8 * (size_t)sc->nm + 4 * (size_t)sc->ng) +
         4 * ((size_t)sc->n + 1 + sc->nm + sc->n + rtwk::kClusterSlots * (size_t)n_clusters) + 16;
}

// The clustered pretest's bounding spheres hold each moving member over its
// time group's [t0, t1]: usable only when the camera's shutter lies inside
// every group's range (else the members' centres leave the bounds).
uint32_t clusters_usable(const rtw_scene_s* sc, const rtw_camera* cam) {
  if (!sc->v64.cluster_on) return 0u;
  for (const auto& g : sc->groups)
    if (!(cam->time0 >= g.first && cam->time1 <= g.second)) return 0u;
  return 1u;
}

// ---------------------------------------------------------- wavefront ----
template <typename R>
struct WfLaunch;
template <>
struct WfLaunch<double> {
  static hipError_t gen(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_generate_f64(a, g, l, s);
  }
  static hipError_t ext(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_extend_f64(a, g, l, s);
  }
  static hipError_t shd(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_shade_f64(a, g, l, s, stats);
  }
  static hipError_t fin(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_finish_f64(a, g, l, s, stats);
  }
  static hipError_t drain(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_drain_f64(a, g, l, s, stats);
  }
  static hipError_t gen_hit(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_generate_hit_f64(a, g, l, s);
  }
  static hipError_t step(const rtwk::WfArgs<double>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_step_f64(a, g, l, s, stats);
  }
};
template <>
struct WfLaunch<float> {
  static hipError_t gen(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_generate_f32(a, g, l, s);
  }
  static hipError_t ext(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_extend_f32(a, g, l, s);
  }
  static hipError_t shd(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_shade_f32(a, g, l, s, stats);
  }
  static hipError_t fin(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_finish_f32(a, g, l, s, stats);
  }
  static hipError_t drain(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_drain_f32(a, g, l, s, stats);
  }
  static hipError_t gen_hit(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s) {
    return rtwk::launch_wf_generate_hit_f32(a, g, l, s);
  }
  static hipError_t step(const rtwk::WfArgs<float>& a, uint32_t g, size_t l, hipStream_t s, bool stats) {
    return rtwk::launch_wf_step_f32(a, g, l, s, stats);
  }
};

template <typename R>
rtwk::PathBuf<R> carve_queue(unsigned char*& b, size_t n) {
  rtwk::PathBuf<R> q;
  R** arr[10] = {&q.ox, &q.oy, &q.oz, &q.dx, &q.dy, &q.dz, &q.tx, &q.ty, &q.tz, &q.tm};
  for (R** a : arr) {
    *a = reinterpret_cast<R*>(b);
    b += al256(n * sizeof(R));
  }
  q.rs = reinterpret_cast<uint64_t*>(b);
  b += al256(n * 8);
  q.slot = reinterpret_cast<uint32_t*>(b);
  b += al256(n * 4);
  q.dsk = reinterpret_cast<uint32_t*>(b);
  b += al256(n * 4);
  q.hk = reinterpret_cast<int32_t*>(b);
  b += al256(n * 4);
  return q;
}

// Thread-local pinned words the host polls for the queue lengths (two per
// queue set: batches are checked one behind).
// Mapped: the fused engine's wf_step writes its batch's word from the device
// (poll_words_dev: the device address of the same words).
uint32_t* poll_words() {
  thread_local uint32_t* w = nullptr;
  if (!w && hipHostMalloc(reinterpret_cast<void**>(&w), 4 * kWfMaxSets * sizeof(uint32_t),
                          hipHostMallocPortable | hipHostMallocMapped) != hipSuccess)
    w = nullptr;
  return w;
}
uint32_t* poll_words_dev(uint32_t* host) {
  void* d = nullptr;
  return host && hipHostGetDevicePointer(&d, host, 0) == hipSuccess ? static_cast<uint32_t*>(d) : nullptr;
}

// Side streams of the wavefront queue sets 1.. (set 0 runs on the caller's
// stream): created once per device for the whole process (not per host
// thread, so a process does not accumulate streams beyond the hardware
// queues, where HIP would map them round-robin onto shared queues and a set
// could land on its caller's queue — correct, but serial); non-blocking,
// joined to the caller's stream by events on every render; kept for the
// life of the process.  Concurrent wavefront renders on one device from several
// threads share them (stream-ordered: still correct).
// The streams live for the process and are never destroyed: a
// static destructor would run during exit, possibly after the HIP runtime's
// own teardown (registered at the first HIP call, after this object was
// constructed), where hipStreamDestroy may crash or hang.  The runtime
// releases them with the process.
struct SideStreams {
  std::mutex mu;
  std::map<std::pair<int, uint32_t>, hipStream_t> s;
};
SideStreams& g_side = *new SideStreams;  // (leaked on purpose: no exit-time destructor)
hipStream_t wf_side_stream(int dev, uint32_t k) {
  std::lock_guard<std::mutex> lk(g_side.mu);
  hipStream_t& s = g_side.s[{dev, k}];
  if (!s) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess || cur != dev ||
        hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
      s = nullptr;
  }
  return s;
}

// One queue set of the wavefront engine: its region of the workspace, its
// stream and its host-side progress.
template <typename R>
struct WfSet {
  rtwk::WfArgs<R> a;
  rtwk::PathBuf<R> qa, qb;
  uint32_t *seg_a = nullptr, *seg_b = nullptr;
  hipStream_t s = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  uint64_t batch = 0;
  bool done = false;
  bool started = false;  // its generate kernel was enqueued
};

// Wavefront render: per queue set, generate, then batches of kWfIters bounce
// launches; after each batch wf_count sums the segment counts of the set's
// queue A and the total is copied to pinned memory.  The host stops a set
// once a batch (checked one batch behind, so the GPU never idles on the poll)
// left its queue empty, or hands the set's drain to wf_drain / wf_finish once
// its live count shows retiring slots.  Empty batches cost only the
// launches: every wave reads its count first.  Sets run on their own streams,
// forked from and joined back to the caller's stream.
constexpr uint32_t kWfBatch = 64;
constexpr int kWfIters = 8;  // even: each batch ends with the live paths in queue A
template <typename R>
int run_wavefront(const rtwk::TraceArgs<R>& ta, const rtw_params* p, unsigned char* ws, const WsLayout& L, int dev,
                  size_t lds, hipStream_t stream, bool stats) {
  if (ta.max_depth == 0) {  // rayColor(depth 0) is black (main.zig:105-108): no segment to trace
    HIP_TRY(hipMemsetAsync(ws + L.partial_off, 0, L.partial_bytes, stream));
    return RTW_OK;
  }
  const uint32_t segs = wf_segs(p), nsets = wf_sets(p);
  const size_t n = (size_t)segs * rtwk::kSegCap;
  const bool per_sample = wf_per_sample_drain(p);
  // Units per reservoir refill (kWfBatch; development knob RTW_WF_BATCH): the
  // refills' atomics against the work a reservoir still holds when the queue
  // runs dry.
  const char* be = dev_knob("RTW_WF_BATCH");
  const uint32_t refill = (be && *be) ? (uint32_t)std::max(1, atoi(be)) : kWfBatch;
  // Bounce segments per path per wf_step launch (params.wf_bounces, 0 = 1):
  // the path stays in registers between them.
  const uint32_t bounces = p->wf_bounces ? p->wf_bounces : 1u;
  // Persistent grids: every resident wave slot of each bounce kernel (at most
  // one wave per segment); the same grids for every launch of the frame.
  // The drains always run max_grid = ceil(segs / waves per block) blocks: one
  // wave per segment (wf_drain has no segment loop; grid_of never sizes them).
  const uint32_t max_grid = (segs + rtwk::kTraceBlock / 64 - 1) / (rtwk::kTraceBlock / 64);
  // RTW_WF_GRID (development knob): N > 0 = N x the resident grid, capped at one wave per segment.
  const char* gk = dev_knob("RTW_WF_GRID");
  const uint32_t gmul = (gk && *gk) ? (uint32_t)std::max(1, atoi(gk)) : 1u;
  // RTW_WF_SET_GRID (development knob): each set's bounce grid = the resident grid / N.
  const char* sg = dev_knob("RTW_WF_SET_GRID");
  const uint32_t gdiv = (sg && *sg) ? (uint32_t)std::max(1, atoi(sg)) : 1u;
  auto grid_of = [&](int kernel) {
    const uint32_t per_cu = (uint32_t)wf_bpc(dev, (int)(sizeof(R) == 4), kernel, lds);
    return std::max(1u, std::min((uint32_t)device_cus(dev) * per_cu * gmul / gdiv, max_grid));
  };
  const uint32_t grid = grid_of(2), grid_ext = grid_of(1), grid_step = grid_of(3);
  // Fused engine (default; params.wf_form RTW_WF_SPLIT: separate extend and
  // shade kernels): one kernel per bounce, the closest hit computed where the
  // ray is made.
  const bool fused = p->wf_form == RTW_WF_FUSED;
  // Queue passes per wf_step launch (params.wf_passes, fused form): each pass
  // moves every path through the queues; a batch holds >= kWfIters passes.
  const uint32_t passes = !fused ? 1u : p->wf_passes ? p->wf_passes : RTW_DEFAULT_WF_PASSES;
  const int iters = std::max(2, (kWfIters / (int)passes) & ~1);  // even: the batch ends with the paths in queue A
  uint32_t* poll = poll_words();
  if (!poll) return fail(RTW_EHIP, "hipHostMalloc of the poll words failed");
  uint32_t* poll_dev = poll_words_dev(poll);
  if (!poll_dev) return fail(RTW_EHIP, "hipHostGetDevicePointer of the poll words failed");
  // development knobs: RTW_WF_POLL_KERNEL=1 polls the fused engine through
  // wf_count + copy as the split form does; RTW_WF_POLL_CHECK=1 runs both and
  // reports on stderr a batch whose published count differs from wf_count's
  const char* pk = dev_knob("RTW_WF_POLL_KERNEL");
  const char* pc = dev_knob("RTW_WF_POLL_CHECK");
  const bool poll_check = fused && pc && *pc == '1';
  const bool publish = fused && !(pk && *pk == '1');
  if (publish && grid_step >= (1u << 20)) return fail(RTW_EINVAL, "wf_step grid %u exceeds the poll ticket's 20 bits", grid_step);
  WfSet<R> set[kWfMaxSets];
  int st = RTW_OK;
  hipEvent_t fork = nullptr;
  if (hipEventCreateWithFlags(&fork, hipEventDisableTiming) != hipSuccess || hipEventRecord(fork, stream) != hipSuccess)
    st = fail(RTW_EHIP, "wavefront fork event failed");
  for (uint32_t k = 0; k < nsets && st == RTW_OK; ++k) {
    WfSet<R>& S = set[k];
    rtwk::WfArgs<R>& a = S.a;
    std::memset(&a, 0, sizeof(a));
    a.t = ta;
    unsigned char* b = ws + L.wf_off + k * L.wf_set_bytes;
    S.qa = carve_queue<R>(b, n);
    S.qb = carve_queue<R>(b, n);
    auto take = [&](size_t bytes) {
      unsigned char* q = b;
      b += al256(bytes);
      return q;
    };
    a.hit_t = reinterpret_cast<R*>(take(n * sizeof(R)));
    a.hit_k = reinterpret_cast<int32_t*>(take(n * 4));
    a.home = reinterpret_cast<rtwk::HomeRec*>(take(n * sizeof(rtwk::HomeRec)));
    S.seg_a = reinterpret_cast<uint32_t*>(take(segs * 4));
    S.seg_b = reinterpret_cast<uint32_t*>(take(segs * 4));
    a.seg_resv = reinterpret_cast<uint32_t*>(take(segs * 8));
    a.drain_buf = per_sample ? reinterpret_cast<R*>(take(n * rtwk::kDrainWin * 3 * sizeof(R))) : nullptr;
    a.live = reinterpret_cast<uint32_t*>(ws + L.live_off) + k;
    a.n_slots = (uint32_t)n;
    a.n_segs = segs;
    a.batch = refill;
    a.bounces = bounces;
    a.passes = passes;
    a.hit_form = fused ? 1u : 0u;  // fused: queued paths carry their hit (hk, o = the hit point)
    a.live_acc = reinterpret_cast<uint32_t*>(ws + L.counter_off + 128) + 2 * k;  // (zeroed with the queue head)
    a.poll_out = nullptr;  // (set per batch)
    S.s = k == 0 ? stream : wf_side_stream(dev, k);  // (set 0: the caller's stream, NULL = the default stream)
    if (k > 0 && !S.s) {
      st = fail(RTW_EHIP, "wavefront side stream creation failed");
      break;
    }
    for (auto& x : S.ev)
      if (hipEventCreateWithFlags(&x, hipEventDisableTiming) != hipSuccess) st = fail(RTW_EHIP, "hipEventCreate failed");
    if (st != RTW_OK) break;
    if (k > 0 && hipStreamWaitEvent(S.s, fork, 0) != hipSuccess) {
      st = fail(RTW_EHIP, "wavefront fork wait failed");
      break;
    }
    // generate -> queue A
    a.out = S.qa;
    a.seg_out = S.seg_a;
    const hipError_t e = fused ? WfLaunch<R>::gen_hit(a, grid_step, lds, S.s) : WfLaunch<R>::gen(a, grid, 0, S.s);
    if (e != hipSuccess) st = fail(RTW_EHIP, "wavefront generate launch: %s", hipGetErrorString(e));
    S.started = true;
  }
  // Termination bound (never reached by a correct kernel): every iteration
  // advances every live path by one segment.
  const uint64_t max_batches = (uint64_t)ta.total_units * ta.chunk * (ta.max_depth + 1ull) / (uint64_t)(iters * passes) + 4;
  // Wall-clock guard as well (300 s; development knob RTW_WF_TIMEOUT_S): a
  // queue that never drains is reported instead of hanging the caller.
  const char* tos = dev_knob("RTW_WF_TIMEOUT_S");
  const double timeout_s = (tos && *tos) ? atof(tos) : 300.0;
  const auto t_start = std::chrono::steady_clock::now();
  // Drain in registers once a set's polled live count falls below fin_frac x
  // its slots: 1 as soon as slots start to retire, i.e. the unit queue ran
  // dry; 0 with RTW_WF_DRAIN_NONE (through the queues to the end); the
  // development knob RTW_WF_FINISH sets another fraction.
  const char* fe = dev_knob("RTW_WF_FINISH");
  const double fin_frac = p->wf_drain == RTW_WF_DRAIN_NONE ? 0.0 : (fe && *fe) ? atof(fe) : 1.0;
  uint32_t left = st == RTW_OK ? nsets : 0u;
  while (left > 0 && st == RTW_OK) {
    // Enqueue one batch on every running set, then look at each set's
    // previous batch (so every stream holds a batch while the host waits).
    for (uint32_t k = 0; k < nsets && st == RTW_OK; ++k) {
      WfSet<R>& S = set[k];
      if (S.done) continue;
      rtwk::WfArgs<R>& a = S.a;
      hipError_t e = hipSuccess;
      // fused: the batch's wf_step launches publish the live count into this
      // batch's pinned word themselves (wf_step publish_live); split: wf_count + copy
      a.poll_out = publish ? poll_dev + 2 * k + (S.batch & 1) : nullptr;
      for (int i = 0; i < iters && e == hipSuccess; ++i) {
        const bool even = (i & 1) == 0 || (passes & 1u) == 0u;  // (an even pass count returns to its input queue)
        a.in = even ? S.qa : S.qb;
        a.out = even ? S.qb : S.qa;
        a.seg_in = even ? S.seg_a : S.seg_b;
        a.seg_out = even ? S.seg_b : S.seg_a;
        if (fused)
          e = WfLaunch<R>::step(a, grid_step, lds, S.s, stats);
        else if ((e = WfLaunch<R>::ext(a, grid_ext, lds, S.s)) == hipSuccess)
          e = WfLaunch<R>::shd(a, grid, lds, S.s, stats);
      }
      if (e != hipSuccess) {
        st = fail(RTW_EHIP, "wavefront bounce launch: %s", hipGetErrorString(e));
        break;
      }
      uint32_t* pw = poll + (publish ? 2 * kWfMaxSets : 0u) + 2 * k + (S.batch & 1);
      if (((!publish || poll_check) && (rtwk::launch_wf_count(S.seg_a, segs, a.live, S.s) != hipSuccess ||
                      hipMemcpyAsync(pw, a.live, 4, hipMemcpyDeviceToHost, S.s) != hipSuccess)) ||
          hipEventRecord(S.ev[S.batch & 1], S.s) != hipSuccess)
        st = fail(RTW_EHIP, "wavefront poll enqueue failed");
      a.poll_out = nullptr;  // (the drains and checks below do not publish)
    }
    for (uint32_t k = 0; k < nsets && st == RTW_OK; ++k) {
      WfSet<R>& S = set[k];
      if (S.done) continue;
      const uint64_t b = S.batch++;
      if (b == 0) continue;
      if (hipEventSynchronize(S.ev[(b - 1) & 1]) != hipSuccess) {
        st = fail(RTW_EHIP, "wavefront batch failed on the device");
        break;
      }
      const uint32_t live = poll[2 * k + ((b - 1) & 1)];
      if (poll_check && publish && live != poll[2 * kWfMaxSets + 2 * k + ((b - 1) & 1)])
        std::fprintf(stderr, "[rtw wf poll] set %u batch %llu: published %u, wf_count %u\n", k,
                     (unsigned long long)(b - 1), live, poll[2 * kWfMaxSets + 2 * k + ((b - 1) & 1)]);
      if (live != 0u && (double)live < fin_frac * (double)n) {  // queue A holds the paths after this batch
        rtwk::WfArgs<R>& a = S.a;
        a.in = S.qa;
        a.seg_in = S.seg_a;
        const hipError_t e = per_sample ? WfLaunch<R>::drain(a, max_grid, lds, S.s, stats)
                                        : WfLaunch<R>::fin(a, max_grid, lds, S.s, stats);
        if (e != hipSuccess) st = fail(RTW_EHIP, "wavefront finish launch: %s", hipGetErrorString(e));
      }
      if (live == 0u || (double)live < fin_frac * (double)n) {
        S.done = true;
        --left;
      } else if (b > max_batches ||
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count() > timeout_s) {
        st = fail(RTW_EHIP, "wavefront queue did not drain after %llu batches", (unsigned long long)b);
      }
    }
  }
  // Every unit must have run: the drains ran outside the batch guard above,
  // so check each set's end state on the device, then join its stream.
  for (uint32_t k = 0; k < nsets; ++k) {
    WfSet<R>& S = set[k];
    if (!S.started) continue;
    if (st == RTW_OK) {
      if (rtwk::launch_wf_check_drained(S.seg_a, S.a.seg_resv, segs, ta.counter, ta.total_units, S.a.live, S.s) !=
              hipSuccess ||
          hipMemcpyAsync(&poll[2 * k], S.a.live, 4, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
          !S.ev[0] || hipEventRecord(S.ev[0], S.s) != hipSuccess)
        st = fail(RTW_EHIP, "wavefront drain check failed to run");
    }
    if (k > 0 && S.ev[1]) {  // join: the caller's stream waits for this set
      if (hipEventRecord(S.ev[1], S.s) != hipSuccess || hipStreamWaitEvent(stream, S.ev[1], 0) != hipSuccess) {
        (void)hipStreamSynchronize(S.s);
        if (st == RTW_OK) st = fail(RTW_EHIP, "wavefront join failed");
      }
    }
  }
  for (uint32_t k = 0; k < nsets && st == RTW_OK; ++k) {
    if (hipEventSynchronize(set[k].ev[0]) != hipSuccess)
      st = fail(RTW_EHIP, "wavefront drain check failed to run");
    else if (poll[2 * k] != 0u)
      st = fail(RTW_EHIP, "wavefront drain of set %u left %u segments/reservoirs with work undone", k, poll[2 * k]);
  }
  for (uint32_t k = 0; k < nsets; ++k)
    for (auto& x : set[k].ev)
      if (x) (void)hipEventDestroy(x);
  if (fork) (void)hipEventDestroy(fork);
  return st;
}

int launch_all(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace, size_t ws_bytes,
               uint8_t* d_rgb, float* d_mean, hipStream_t stream, rtw_timer timer, int mode) {
  const WsLayout L = ws_layout(p);
  if (!workspace || ws_bytes < L.total)
    return fail(RTW_EINVAL, "workspace %zu bytes < required %zu", ws_bytes, L.total);
  if ((reinterpret_cast<uintptr_t>(workspace) & 255) != 0) return fail(RTW_EINVAL, "workspace not 256-B aligned");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (dev != sc->device)
    return fail(RTW_EINVAL, "scene lives on device %d but the current device is %d", sc->device, dev);
  auto* ws = static_cast<unsigned char*>(workspace);
  HIP_TRY(hipMemsetAsync(ws + L.counter_off, 0, 512, stream));  // queue head + stats
  const int var = kernel_variant(p->precision);
  if (p->engine != RTW_ENGINE_WAVEFRONT && !rtwk::trace_variant_built((int)p->precision, var))
    return fail(RTW_EINVAL, "RTW_VARIANT=%d: trace kernel variant not built into this library", var);
  // The clustered pretest runs only in the f64 megakernel variants with
  // kVarCluster (or the wavefront kernels built with it: kWfCluster), and only
  // when the shutter lies in every time group.
  const uint32_t cl_on = (p->precision == RTW_PRECISION_F64 &&
                          (p->engine == RTW_ENGINE_MEGAKERNEL ? (var & rtwk::kVarClusterBit) != 0 : rtwk::kWfCluster))
                             ? clusters_usable(sc, cam)
                             : 0u;
  size_t lds = lds_bytes(sc, (int)p->precision, cl_on ? sc->v64.n_clusters : 0u);
  if (p->engine == RTW_ENGINE_MEGAKERNEL && (var & rtwk::kVarHomeLdsBit) != 0)
    lds += 8 + (rtwk::kHomeLdsBytesPerWave + ((var & rtwk::kVarPathLdsBit) ? rtwk::kPathLdsBytesPerWave : 0) +
                ((var & rtwk::kVarUnitBaseBit) ? rtwk::kUnitBaseLdsBytesPerWave : 0)) *
                   (rtwk::kTraceBlock / 64);  // (8: alignment of the home block)
  if (lds > 64 * 1024) return fail(RTW_UNSUPPORTED, "scene tables need %zu B of LDS", lds);
  const int bpc = blocks_per_cu(dev, (int)p->precision, lds, var);
  const int cus = device_cus(dev);
  uint32_t total_units = 0;
  hipError_t e;
  if (timer) HIP_TRY(hipEventRecord(timer->start, stream));
  if (p->engine == RTW_ENGINE_WAVEFRONT) {
    if (mode == 2) return fail(RTW_UNSUPPORTED, "phase profile runs on the megakernel engine");
    int st;
    if (p->precision == RTW_PRECISION_F32) {
      rtwk::TraceArgs<float> a;
      fill_args(a, sc->v32, cam, p, ws, L);
      a.sc.n_clusters = 0u;  // f32: no clustered pretest
      st = run_wavefront<float>(a, p, ws, L, dev, lds, stream, mode == 1);
    } else {
      rtwk::TraceArgs<double> a;
      fill_args(a, sc->v64, cam, p, ws, L);
      a.sc.cluster_on = cl_on;  // (0 unless the bounce kernels were built with the clustered pretest)
      if (!cl_on) a.sc.n_clusters = 0u;
      st = run_wavefront<double>(a, p, ws, L, dev, lds, stream, mode == 1);
    }
    if (st != RTW_OK) return st;
    e = hipSuccess;
  } else if (p->precision == RTW_PRECISION_F32) {
    rtwk::TraceArgs<float> a;
    fill_args(a, sc->v32, cam, p, ws, L);
    a.sc.n_clusters = 0u;  // f32: no clustered pretest
    total_units = a.total_units;
    const uint32_t want = (total_units + 255) / 256;
    const uint32_t grid = std::max(1u, std::min((uint32_t)(cus * bpc), want));
    e = rtwk::launch_trace_f32(a, grid, lds, stream, mode, var);
  } else {
    rtwk::TraceArgs<double> a;
    fill_args(a, sc->v64, cam, p, ws, L);
    a.sc.cluster_on = cl_on;
    if (!cl_on) a.sc.n_clusters = 0u;  // nothing to stage (lds_bytes above)
    total_units = a.total_units;
    const uint32_t want = (total_units + 255) / 256;
    const uint32_t grid = std::max(1u, std::min((uint32_t)(cus * bpc), want));
    e = rtwk::launch_trace_f64(a, grid, lds, stream, mode, var);
  }
  if (e != hipSuccess) return fail(RTW_EHIP, "trace kernel launch: %s", hipGetErrorString(e));
  if (timer) {
    HIP_TRY(hipEventRecord(timer->stop, stream));
    timer->recorded = true;
  }
  if (d_rgb) {
    rtwk::FinalizeArgs f;
    f.partial = reinterpret_cast<const double*>(ws + L.partial_off);
    f.rgb = d_rgb;
    f.mean = d_mean;
    f.npix = p->row_count * p->width;
    f.n_chunks = n_chunks(p);
    f.scale = 1.0 / (double)p->spp;
    e = rtwk::launch_finalize(f, stream);
    if (e != hipSuccess) return fail(RTW_EHIP, "finalize kernel launch: %s", hipGetErrorString(e));
  }
  return RTW_OK;
}

}  // namespace

extern "C" {

size_t rtw_workspace_bytes(const rtw_params* p) {
  if (validate(p) != RTW_OK) return 0;
  return ws_layout(p).total;
}

int rtw_timer_create(rtw_timer* out) {
  if (!out) return fail(RTW_EINVAL, "timer out is NULL");
  auto* t = new rtw_timer_s;
  if (hipEventCreate(&t->start) != hipSuccess || hipEventCreate(&t->stop) != hipSuccess) {
    delete t;
    return fail(RTW_EHIP, "hipEventCreate failed");
  }
  *out = t;
  return RTW_OK;
}
int rtw_timer_destroy(rtw_timer t) {
  if (!t) return RTW_OK;
  (void)hipEventDestroy(t->start);
  (void)hipEventDestroy(t->stop);
  delete t;
  return RTW_OK;
}
int rtw_sclk_probe_begin(void* stream, double wall_ms, rtw_sclk_probe* out) {
  if (!out) return fail(RTW_EINVAL, "probe out is NULL");
  *out = nullptr;
  if (!(wall_ms > 0.0 && wall_ms < 600e3)) return fail(RTW_EINVAL, "probe window %g ms outside (0, 600 s)", wall_ms);
  // the s_memrealtime rate of the current device (kHz), not an assumed 100 MHz
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0)
    return fail(RTW_EHIP, "probe: wall-clock rate of device %d unavailable", dev);
  auto* p = new rtw_sclk_probe_s;
  p->s = static_cast<hipStream_t>(stream);
  if (hipMalloc(reinterpret_cast<void**>(&p->d), sizeof(double)) != hipSuccess) {
    delete p;
    return fail(RTW_ENOMEM, "probe: hipMalloc failed");
  }
  hipLaunchKernelGGL(sclk_probe_kernel, dim3(1), dim3(64), 0, p->s, (unsigned long long)(wall_ms * khz),
                     (double)khz * 1e-3, p->d);
  if (hipGetLastError() != hipSuccess) {
    (void)hipFree(p->d);
    delete p;
    return fail(RTW_EHIP, "probe kernel launch failed");
  }
  *out = p;
  return RTW_OK;
}
int rtw_sclk_probe_end(rtw_sclk_probe p, double* mhz) {
  if (!p || !mhz) return fail(RTW_EINVAL, "probe/mhz is NULL");
  int st = RTW_OK;
  if (hipStreamSynchronize(p->s) != hipSuccess || hipMemcpy(mhz, p->d, sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    st = fail(RTW_EHIP, "probe read failed");
  (void)hipFree(p->d);
  delete p;
  return st;
}

int rtw_timer_elapsed_ms(rtw_timer t, float* ms) {
  if (!t || !ms) return fail(RTW_EINVAL, "timer/ms is NULL");
  if (!t->recorded) return fail(RTW_EINVAL, "timer was never recorded");
  HIP_TRY(hipEventSynchronize(t->stop));
  HIP_TRY(hipEventElapsedTime(ms, t->start, t->stop));
  return RTW_OK;
}

int rtw_render_device(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace,
                      size_t ws_bytes, uint8_t* d_rgb, float* d_mean, void* stream, rtw_timer timer) {
  if (!sc || !cam) return fail(RTW_EINVAL, "scene/camera is NULL");
  if (!d_rgb) return fail(RTW_EINVAL, "d_rgb is NULL");
  const int v = validate(p);
  if (v != RTW_OK) return v;
  return launch_all(sc, cam, p, workspace, ws_bytes, d_rgb, d_mean, static_cast<hipStream_t>(stream), timer, 0);
}

// The statistics pass: one render in counting mode, the kernels' 32 statistics
// words copied back (rtw_hip.h RTW_STAT_*; words 16.. are the diagnostic
// build's phase stamps).
static int stats_pass(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace, size_t ws_bytes,
               unsigned long long (&st)[32]) {
  if (!sc || !cam) return fail(RTW_EINVAL, "scene/camera is NULL");
  const int v = validate(p);
  if (v != RTW_OK) return v;
  // RTW_PHASE_PROFILE=1: diagnostic build with per-phase s_memtime stamps.
  const char* prof = dev_knob("RTW_PHASE_PROFILE");
  const int mode = (prof && prof[0] == '1') ? 2 : 1;
#ifndef RTW_MEASURE
  if (mode == 2) return fail(RTW_UNSUPPORTED, "RTW_PHASE_PROFILE needs the -DRTW_MEASURE build (tools/gpu_phase.sh)");
#endif
  const int r = launch_all(sc, cam, p, workspace, ws_bytes, nullptr, nullptr, nullptr, nullptr, mode);
  if (r != RTW_OK) return r;
  HIP_TRY(hipDeviceSynchronize());
  for (auto& x : st) x = 0;
  const WsLayout L = ws_layout(p);
  HIP_TRY(hipMemcpy(st, static_cast<unsigned char*>(workspace) + L.stats_off, sizeof(st), hipMemcpyDeviceToHost));
  if (mode == 1 && dev_knob("RTW_COUNTS_VERBOSE")) {
    fprintf(stderr, "[rtw counts] samples %llu segments %llu skipped %llu cand_wave_iters %llu cand_lanes %llu "
            "disc_ge0_lanes %llu sphere_loop_wave_iters %llu cull_survivor_lanes %llu cull_exact_wave_iters %llu "
            "cluster_wave_tests %llu cluster_wave_skips %llu\n", st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8],
            st[11], st[12]);
    if (st[13])  // wavefront engine, wf_drain
      fprintf(stderr, "[rtw counts] drain wave iterations %llu, drained segments per wave iteration %.2f of 64\n",
              st[13], (double)st[9] / (double)st[13]);
  }
  if (mode == 2) {
    const char* names[10] = {"refill",  "start_sample", "wide+pretest", "hit+kind",    "tail",
                             "loop_top", "exact_survivors", "coop_ball", "hitrec+scatter", "-"};
    unsigned long long tot = 0;
    for (int i = 0; i < 10; ++i) tot += st[16 + i];
    for (int i = 0; i < 9; ++i)
      fprintf(stderr, "[rtw phase] %-15s %6.2f%%  (%llu wave-cycles)\n", names[i], tot ? 100.0 * st[16 + i] / tot : 0.0,
              st[16 + i]);
  }
  return RTW_OK;
}

int rtw_render_stats(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace, size_t ws_bytes,
                     uint64_t stats_out[RTW_STATS_WORDS]) {
  if (!stats_out) return fail(RTW_EINVAL, "stats is NULL");
  unsigned long long st[32];
  const int r = stats_pass(sc, cam, p, workspace, ws_bytes, st);
  if (r != RTW_OK) return r;
  for (int i = 0; i < RTW_STATS_WORDS; ++i) stats_out[i] = st[i];
  return RTW_OK;
}

int rtw_render_counts_ex(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace,
                         size_t ws_bytes, uint64_t counts_out[6]) {
  if (!counts_out) return fail(RTW_EINVAL, "counts is NULL");
  unsigned long long st[32];
  const int r = stats_pass(sc, cam, p, workspace, ws_bytes, st);
  if (r != RTW_OK) return r;
  counts_out[0] = st[0];
  counts_out[1] = st[1];
  // every segment tests every sphere; f32 mode skips one small sphere per segment with a skip set
  counts_out[2] = st[1] * sc->n_static;
  counts_out[3] = st[1] * sc->n_moving;
  if (p->precision == RTW_PRECISION_F32) counts_out[2] -= st[2];
  counts_out[4] = st[9];  // wf_finish (rtw_wavefront.hip shade_step FIN)
  counts_out[5] = st[10];
  return RTW_OK;
}

int rtw_render_counts(rtw_scene sc, const rtw_camera* cam, const rtw_params* p, void* workspace,
                      size_t ws_bytes, uint64_t counts_out[4]) {
  if (!counts_out) return fail(RTW_EINVAL, "scene/camera/counts is NULL");
  uint64_t c[6];
  const int r = rtw_render_counts_ex(sc, cam, p, workspace, ws_bytes, c);
  if (r == RTW_OK)
    for (int i = 0; i < 4; ++i) counts_out[i] = c[i];
  return r;
}

int rtw_render(const rtw_camera* cam, const rtw_sphere* spheres, uint32_t n, const rtw_material* mats, uint32_t nm,
               const rtw_params* p, uint8_t* rgb_out, float* mean_out) {
  if (!cam || !rgb_out) return fail(RTW_EINVAL, "camera/rgb_out is NULL");
  const int v = validate(p);
  if (v != RTW_OK) return v;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(RTW_ENODEV, "no HIP device visible");
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  const int dev = p->device < 0 ? prev : p->device;
  if (dev >= ndev) return fail(RTW_EINVAL, "device %d >= device count %d", dev, ndev);
  HIP_TRY(hipSetDevice(dev));
  rtw_scene sc = nullptr;
  int st = rtw_scene_create(spheres, n, mats, nm, &sc);
  if (st != RTW_OK) {
    (void)hipSetDevice(prev);
    return st;
  }
  const size_t wsb = ws_layout(p).total;
  const size_t pix = (size_t)p->row_count * p->width * 3;
  void *ws = nullptr, *d_rgb = nullptr, *d_mean = nullptr;
  hipStream_t s = nullptr;
  st = RTW_OK;
  if (hipMalloc(&ws, wsb) != hipSuccess || hipMalloc(&d_rgb, pix) != hipSuccess ||
      (mean_out && hipMalloc(&d_mean, pix * sizeof(float)) != hipSuccess)) {
    st = fail(RTW_ENOMEM, "rtw_render: device allocation failed");
  }
  if (st == RTW_OK && hipStreamCreate(&s) != hipSuccess) st = fail(RTW_EHIP, "hipStreamCreate failed");
  if (st == RTW_OK)
    st = launch_all(sc, cam, p, ws, wsb, static_cast<uint8_t*>(d_rgb), static_cast<float*>(d_mean), s, nullptr,
                    0);
  if (st == RTW_OK && hipStreamSynchronize(s) != hipSuccess) st = fail(RTW_EHIP, "render failed on the device");
  if (st == RTW_OK && hipMemcpy(rgb_out, d_rgb, pix, hipMemcpyDeviceToHost) != hipSuccess)
    st = fail(RTW_EHIP, "copy of rgb_out failed");
  if (st == RTW_OK && mean_out &&
      hipMemcpy(mean_out, d_mean, pix * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
    st = fail(RTW_EHIP, "copy of mean_out failed");
  if (s) (void)hipStreamDestroy(s);
  if (ws) (void)hipFree(ws);
  if (d_rgb) (void)hipFree(d_rgb);
  if (d_mean) (void)hipFree(d_mean);
  rtw_scene_destroy(sc);
  (void)hipSetDevice(prev);
  return st;
}

}  // extern "C"

// ---- helpers shared with the world path (rtw_world_capi.hip) ----
int rtw_fail(int status, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fail(status, "%s", buf);
}
int rtw_validate_params(const rtw_params* p) { return validate(p); }
const char* rtw_dev_knob(const char* name) { return dev_knob(name); }
size_t rtw_ws_total(const rtw_params* p) { return ws_layout(p).total; }
size_t rtw_ws_stats_off(const rtw_params* p) { return ws_layout(p).stats_off; }
size_t rtw_ws_counter_off(const rtw_params* p) { return ws_layout(p).counter_off; }
int rtw_device_cus(int dev) { return device_cus(dev); }
uint32_t rtw_total_units(const rtw_params* p) {
  const uint32_t tiles_x = (p->width + rtwk::kTileW - 1) / rtwk::kTileW;
  const uint32_t tiles_y = (p->row_count + rtwk::kTileH - 1) / rtwk::kTileH;
  return tiles_x * tiles_y * 64u * n_chunks(p);  // = TraceArgs::total_units (fill_args)
}
void rtw_fill_trace_args(rtwk::TraceArgs<double>& a, const rtw_camera* cam, const rtw_params* p, unsigned char* ws) {
  fill_args(a, rtwk::SceneView<double>{}, cam, p, ws, ws_layout(p));
  a.unit_order = unit_order(kWorldUnitOrder);  // the world kernel's default (fill_args)
}
int rtw_launch_finalize(const rtw_params* p, unsigned char* ws, uint8_t* d_rgb, float* d_mean, hipStream_t s) {
  const WsLayout L = ws_layout(p);
  rtwk::FinalizeArgs f;
  f.partial = reinterpret_cast<const double*>(ws + L.partial_off);
  f.rgb = d_rgb;
  f.mean = d_mean;
  f.npix = p->row_count * p->width;
  f.n_chunks = n_chunks(p);
  f.scale = 1.0 / (double)p->spp;
  const hipError_t e = rtwk::launch_finalize(f, s);
  if (e != hipSuccess) return fail(RTW_EHIP, "finalize kernel launch: %s", hipGetErrorString(e));
  return RTW_OK;
}
int rtw_timer_mark(rtw_timer t, hipStream_t s, bool start) {
  if (hipEventRecord(start ? t->start : t->stop, s) != hipSuccess) return fail(RTW_EHIP, "timer event record failed");
  if (!start) t->recorded = true;
  return RTW_OK;
}
