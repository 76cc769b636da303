// rtw_host.cpp — host-side rtw API mirror (see rtw_host.hpp) and the C-ABI
// host helpers rtw_camera_init / rtw_image_height / rtw_cover_scene.
// Compiled with -ffp-contract=off: one IEEE op per Zig f64 op.
#include "rtw_host.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>

namespace rtw {

double Vec3::norm() const { return std::sqrt(normSquared()); }          // vec.zig:12-14
Vec3 Vec3::normalized() const {                                          // vec.zig:32-39
  const double n = norm();
  return n == 0.0 ? *this : div(n);
}

// ---- std.Random.DefaultPrng restatement (Zig 0.14) ----
static inline uint64_t splitmix64_next(uint64_t& s) {  // std/Random/SplitMix64.zig
  s += 0x9e3779b97f4a7c15ULL;
  uint64_t z = s;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static inline uint64_t rotl(uint64_t x, unsigned k) { return (x << k) | (x >> (64 - k)); }

Random Random::init(uint64_t seed) {  // Xoshiro256.seed
  Random r;
  uint64_t sm = seed;
  for (auto& w : r.s_) w = splitmix64_next(sm);
  return r;
}
uint64_t Random::next() {  // Xoshiro256.next (xoshiro256++)
  const uint64_t res = rotl(s_[0] + s_[3], 23) + s_[0];
  const uint64_t t = s_[1] << 17;
  s_[2] ^= s_[0];
  s_[3] ^= s_[1];
  s_[1] ^= s_[2];
  s_[0] ^= s_[3];
  s_[2] ^= t;
  s_[3] = rotl(s_[3], 45);
  return res;
}
static inline uint64_t clz64(uint64_t x) { return x ? (uint64_t)__builtin_clzll(x) : 64u; }
double Random::float64() {  // std/Random.zig float(f64)
  const uint64_t rnd = next();
  uint64_t lz = clz64(rnd);
  if (lz >= 12) {
    lz = 12;
    for (;;) {
      const uint64_t addl = clz64(next());
      lz += addl;
      if (addl != 64) break;
      if (lz >= 1022) {
        lz = 1022;
        break;
      }
    }
  }
  const uint64_t bits = ((1022 - lz) << 52) | (rnd & ((1ULL << 52) - 1));
  double d;
  std::memcpy(&d, &bits, 8);
  return d;
}
void Random::state(uint64_t out[4]) const { std::memcpy(out, s_, sizeof(s_)); }

double randomReal01(Random& rng) { return rng.float64(); }
double randomReal(Random& rng, double min, double max) { return min + randomReal01(rng) * (max - min); }
Vec3 random01(Random& rng) {
  Vec3 v;
  v.x = randomReal01(rng);
  v.y = randomReal01(rng);
  v.z = randomReal01(rng);
  return v;
}
Vec3 randomVec(Random& rng, double min, double max) {
  Vec3 v;
  v.x = randomReal(rng, min, max);
  v.y = randomReal(rng, min, max);
  v.z = randomReal(rng, min, max);
  return v;
}

Texture Texture::makeSolid(Color c) {
  Texture t;
  t.kind = Kind::solid;
  t.color = c;
  return t;
}
Texture Texture::makeChecker(Color odd, Color even) {
  Texture t;
  t.kind = Kind::checker;
  t.odd = odd;
  t.even = even;
  return t;
}
std::shared_ptr<Material> Material::diffuse(Texture t) {
  auto m = std::make_shared<Material>();
  m->kind = Kind::diffuse;
  m->albedo = t;
  return m;
}
std::shared_ptr<Material> Material::metal(Color albedo, double fuzz) {
  auto m = std::make_shared<Material>();
  m->kind = Kind::metal;
  m->metal_albedo = albedo;
  m->fuzz = fuzz;
  return m;
}
std::shared_ptr<Material> Material::dielectric(double ir) {
  auto m = std::make_shared<Material>();
  m->kind = Kind::dielectric;
  m->ir = ir;
  return m;
}

Hittable Hittable::makeSphere(Point3 c, double r, std::shared_ptr<Material> m) {
  Hittable h;
  h.kind = Kind::sphere;
  h.center0 = h.center1 = c;
  h.radius = r;
  h.material = std::move(m);
  return h;
}
Hittable Hittable::makeMovingSphere(Point3 c0, Point3 c1, double t0, double t1, double r,
                                    std::shared_ptr<Material> m) {
  Hittable h;
  h.kind = Kind::movingSphere;
  h.center0 = c0;
  h.center1 = c1;
  h.time0 = t0;
  h.time1 = t1;
  h.radius = r;
  h.material = std::move(m);
  return h;
}
Hittable Hittable::makeList(std::vector<Hittable> objs) {
  Hittable h;
  h.kind = Kind::list;
  h.objects = std::move(objs);
  return h;
}

Camera Camera::init(Point3 look_from, Point3 look_at, Vec3 vup, double vfov, double aspect_ratio,
                    double aperture, double focus_dist, double time0, double time1) {
  const double theta = vfov * M_PI / 180.0;  // deg2rad, main.zig:36-38
  const double h = std::tan(theta / 2);
  const double viewport_height = 2.0 * h;
  const double viewport_width = aspect_ratio * viewport_height;
  const Vec3 w = look_from.sub(look_at).normalized();
  const Vec3 u = vup.cross(w).normalized();
  const Vec3 v = w.cross(u);
  Camera c;
  c.origin = look_from;
  c.horizontal = u.mul(viewport_width * focus_dist);
  c.vertical = v.mul(viewport_height * focus_dist);
  c.lower_left_corner = c.origin.sub(c.horizontal.div(2.0)).sub(c.vertical.div(2.0)).sub(w.mul(focus_dist));
  c.u = u;
  c.v = v;
  c.w = w;
  c.lens_radius = aperture / 2.0;
  c.time0 = time0;
  c.time1 = time1;
  return c;
}

static void put3(double d[3], const Vec3& v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}
rtw_camera Camera::to_c() const {
  rtw_camera c;
  put3(c.origin, origin);
  put3(c.horizontal, horizontal);
  put3(c.vertical, vertical);
  put3(c.lower_left_corner, lower_left_corner);
  put3(c.u, u);
  put3(c.v, v);
  put3(c.w, w);
  c.lens_radius = lens_radius;
  c.time0 = time0;
  c.time1 = time1;
  return c;
}

Hittable generateRandomScene(Random& rng) {  // main.zig:157-221
  std::vector<Hittable> objs;
  auto checker = Texture::makeChecker(rgb(0.2, 0.3, 0.1), rgb(0.9, 0.9, 0.9));
  auto mat_ground = Material::diffuse(checker);
  auto mat1 = Material::dielectric(1.5);
  auto mat2 = Material::diffuse(Texture::makeSolid(rgb(0.4, 0.2, 0.1)));
  auto mat3 = Material::metal(rgb(0.7, 0.6, 0.5), 0.0);
  objs.push_back(Hittable::makeSphere({0, -1000, 0}, 1000, mat_ground));
  objs.push_back(Hittable::makeSphere({0, 1, 0}, 1.0, mat1));
  objs.push_back(Hittable::makeSphere({-4, 1, 0}, 1.0, mat2));
  objs.push_back(Hittable::makeSphere({4, 1, 0}, 1.0, mat3));
  for (int a = -3; a < 3; ++a) {
    for (int b = -3; b < 3; ++b) {
      const double choose_mat = randomReal01(rng);
      Point3 center;
      center.x = (double)a + 0.9 * randomReal01(rng);
      center.y = 0.2;
      center.z = (double)b + 0.9 * randomReal01(rng);
      if (center.sub({4, 0.2, 0}).norm() <= 0.9) continue;
      if (choose_mat < 0.8) {  // diffuse, moving (main.zig:193-205)
        const Color a1 = random01(rng);
        const Color a2 = random01(rng);
        auto m = Material::diffuse(Texture::makeSolid(a1.mulV(a2)));
        const Point3 center1 = center.add({0, randomReal(rng, 0, 0.5), 0});
        objs.push_back(Hittable::makeMovingSphere(center, center1, 0, 1, 0.2, m));
      } else if (choose_mat < 0.95) {  // metal (main.zig:206-211)
        const Color albedo = randomVec(rng, 0.5, 1);
        const double fuzz = randomReal(rng, 0, 0.5);
        objs.push_back(Hittable::makeSphere(center, 0.2, Material::metal(albedo, fuzz)));
      } else {  // glass (main.zig:212-215)
        objs.push_back(Hittable::makeSphere(center, 0.2, Material::dielectric(1.5)));
      }
    }
  }
  return Hittable::makeList(std::move(objs));
}

static rtw_material flat_material(const Material& m) {
  rtw_material r;
  std::memset(&r, 0, sizeof(r));
  switch (m.kind) {
    case Material::Kind::diffuse:
      if (m.albedo.kind == Texture::Kind::solid) {
        r.kind = RTW_LAMBERT_SOLID;
        put3(r.albedo, m.albedo.color);
      } else if (m.albedo.kind == Texture::Kind::checker) {
        r.kind = RTW_LAMBERT_CHECKER;
        put3(r.albedo, m.albedo.even);
        put3(r.albedo_odd, m.albedo.odd);
      } else {
        r.kind = RTW_DIFFUSE_LIGHT;  // noise / image: not on the cover path (rtw_world_* renders them)
      }
      break;
    case Material::Kind::metal:
      r.kind = RTW_METAL;
      put3(r.albedo, m.metal_albedo);
      r.fuzz = m.fuzz;
      break;
    case Material::Kind::dielectric:
      r.kind = RTW_DIELECTRIC;
      r.ir = m.ir;
      break;
    case Material::Kind::diffuse_light:
      r.kind = RTW_DIFFUSE_LIGHT;
      break;
  }
  return r;
}

static void flatten_into(const Hittable& h, FlatScene& out, std::map<const Material*, uint32_t>& ids) {
  if (h.kind == Hittable::Kind::list) {
    for (const auto& o : h.objects) flatten_into(o, out, ids);
    return;
  }
  if (h.kind != Hittable::Kind::sphere && h.kind != Hittable::Kind::movingSphere)
    throw Error(RTW_UNSUPPORTED, "the cover-scene path renders spheres only (use flattenWorld / rtw_world_*)");
  if (!h.material) throw Error(RTW_EINVAL, "hittable without material");
  auto it = ids.find(h.material.get());
  uint32_t mid;
  if (it == ids.end()) {
    mid = (uint32_t)out.materials.size();
    out.materials.push_back(flat_material(*h.material));
    ids[h.material.get()] = mid;
  } else {
    mid = it->second;
  }
  rtw_sphere s;
  std::memset(&s, 0, sizeof(s));
  put3(s.c0, h.center0);
  put3(s.c1, h.kind == Hittable::Kind::movingSphere ? h.center1 : h.center0);
  s.radius = h.radius;
  s.t0 = h.time0;
  s.t1 = h.time1;
  s.moving = h.kind == Hittable::Kind::movingSphere ? 1u : 0u;
  s.mat = mid;
  out.spheres.push_back(s);
}

FlatScene flatten(const Hittable& world) {
  FlatScene f;
  std::map<const Material*, uint32_t> ids;
  flatten_into(world, f, ids);
  return f;
}

uint32_t imageHeight(uint32_t width, double aspect_ratio) {
  return (uint32_t)std::trunc((double)width / aspect_ratio);
}

std::vector<uint8_t> render(const Camera& cam, const Hittable& world, const RenderSettings& s, uint32_t height) {
  const FlatScene f = flatten(world);
  rtw_params p;
  std::memset(&p, 0, sizeof(p));
  p.width = s.width;
  p.height = height;
  p.spp = s.samples_per_pixel;
  p.max_depth = s.max_depth;
  p.seed = s.seed;
  put3(p.background, s.background);
  p.row_begin = 0;
  p.row_stride = 1;
  p.row_count = height;
  p.chunk = s.chunk;
  p.precision = s.precision;
  p.device = -1;
  p.engine = s.engine;
  const rtw_camera c = cam.to_c();
  std::vector<uint8_t> rgb((size_t)s.width * height * 3);
  const int st = rtw_render(&c, f.spheres.data(), (uint32_t)f.spheres.size(), f.materials.data(),
                            (uint32_t)f.materials.size(), &p, rgb.data(), nullptr);
  if (st != RTW_OK) throw Error(st, rtw_last_error());
  return rgb;
}

void writePPM(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw Error(RTW_EINVAL, "cannot open " + path);
  std::fprintf(f, "P6\n%u %u\n255\n", w, h);
  std::fwrite(rgb.data(), 1, rgb.size(), f);
  std::fclose(f);
}

}  // namespace rtw

// ------------------------------------------------------- C-ABI helpers ----
extern "C" int rtw_camera_init(rtw_camera* cam, const double look_from[3], const double look_at[3],
                               const double vup[3], double vfov, double aspect_ratio, double aperture,
                               double focus_dist, double time0, double time1) {
  if (!cam || !look_from || !look_at || !vup) return RTW_EINVAL;
  const rtw::Camera c = rtw::Camera::init({look_from[0], look_from[1], look_from[2]},
                                          {look_at[0], look_at[1], look_at[2]}, {vup[0], vup[1], vup[2]},
                                          vfov, aspect_ratio, aperture, focus_dist, time0, time1);
  *cam = c.to_c();
  return RTW_OK;
}

extern "C" uint32_t rtw_image_height(uint32_t width, double aspect_ratio) {
  return rtw::imageHeight(width, aspect_ratio);
}

extern "C" int rtw_cover_scene(uint64_t seed, rtw_sphere* spheres, uint32_t* n_spheres, rtw_material* mats,
                               uint32_t* n_mats, uint64_t rng_state_out[4]) {
  if (!n_spheres || !n_mats) return RTW_EINVAL;
  rtw::Random rng = rtw::Random::init(seed);
  const rtw::Hittable world = rtw::generateRandomScene(rng);
  const rtw::FlatScene f = rtw::flatten(world);
  const uint32_t cap_s = *n_spheres, cap_m = *n_mats;
  *n_spheres = (uint32_t)f.spheres.size();
  *n_mats = (uint32_t)f.materials.size();
  if (rng_state_out) rng.state(rng_state_out);
  if (!spheres || !mats) return RTW_OK;  // size query
  if (cap_s < f.spheres.size() || cap_m < f.materials.size()) return RTW_EINVAL;
  std::memcpy(spheres, f.spheres.data(), f.spheres.size() * sizeof(rtw_sphere));
  std::memcpy(mats, f.materials.data(), f.materials.size() * sizeof(rtw_material));
  return RTW_OK;
}
