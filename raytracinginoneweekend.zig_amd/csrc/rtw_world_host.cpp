// rtw_world_host.cpp — host-side mirror of the reference's general scene
// vocabulary (rects, box, translate, rotateY, diffuse light, noise and image
// textures, Perlin; hittable.zig:270-608, material.zig:94-110,
// texture.zig:85-144, perlin.zig:10-124), the scene builders of main.zig
// (scenes 2-6) plus the configs[4] globe scene, the flattening of a world
// into the rtw_world_desc arrays, and the C-ABI scene-build helpers.
// Compiled with -ffp-contract=off: one IEEE op per Zig f64 op.
#include <cmath>
#include <cstring>
#include <map>

#include "rtw_hip.h"
#include "rtw_host.hpp"
#include "rtw_libm.hpp"

namespace rtw {

static void put3(double d[3], const Vec3& v) {
  d[0] = v.x;
  d[1] = v.y;
  d[2] = v.z;
}

// Zig 0.14 std.Random.uintLessThan(u64) (Lemire's multiply-shift with the
// pcg "extra tweak") behind intRangeLessThan for unsigned T; r.int(u64) is
// one Xoshiro256.next().
uint64_t randomIntLessThan(Random& rng, uint64_t at_least, uint64_t less_than) {
  const uint64_t lt = less_than - at_least;
  uint64_t x = rng.next();
  unsigned __int128 m = (unsigned __int128)x * lt;
  uint64_t l = (uint64_t)m;
  if (l < lt) {
    uint64_t t = 0 - lt;
    if (t >= lt) {
      t -= lt;
      if (t >= lt) t %= lt;
    }
    while (l < t) {
      x = rng.next();
      m = (unsigned __int128)x * lt;
      l = (uint64_t)m;
    }
  }
  return at_least + (uint64_t)(m >> 64);
}

std::shared_ptr<Perlin> Perlin::init(Random& rng) {  // perlin.zig:18-40
  auto p = std::make_shared<Perlin>();
  for (int i = 0; i < 256; ++i) {
    p->ranvec[i] = randomVec(rng, -1, 1).normalized();
    p->perm[0][i] = p->perm[1][i] = p->perm[2][i] = (uint32_t)i;
  }
  for (auto& q : p->perm) {  // permute, perlin.zig:93-102 (target in [0, i))
    for (uint64_t i = 255; i > 0; --i) {
      const uint64_t target = randomIntLessThan(rng, 0, i);
      std::swap(q[i], q[target]);
    }
  }
  return p;
}

Texture Texture::makeNoise(double scale, Random& rng) {
  Texture t;
  t.kind = Kind::noise;
  t.perlin = Perlin::init(rng);
  t.scale = scale;
  return t;
}
Texture Texture::makeImage(std::shared_ptr<Image> image) {
  Texture t;
  t.kind = Kind::image;
  t.image = std::move(image);
  return t;
}
std::shared_ptr<Material> Material::diffuseLight(Texture emit) {
  auto m = std::make_shared<Material>();
  m->kind = Kind::diffuse_light;
  m->albedo = std::move(emit);
  return m;
}

static Hittable rect(Hittable::Kind k, double a0, double a1, double b0, double b1, double kk,
                     std::shared_ptr<Material> m) {
  Hittable h;
  h.kind = k;
  h.a0 = a0, h.a1 = a1, h.b0 = b0, h.b1 = b1, h.k = kk;
  h.material = std::move(m);
  return h;
}
Hittable Hittable::makeXyRect(double x0, double x1, double y0, double y1, double k, std::shared_ptr<Material> m) {
  return rect(Kind::xyRect, x0, x1, y0, y1, k, std::move(m));
}
Hittable Hittable::makeXzRect(double x0, double x1, double z0, double z1, double k, std::shared_ptr<Material> m) {
  return rect(Kind::xzRect, x0, x1, z0, z1, k, std::move(m));
}
Hittable Hittable::makeYzRect(double y0, double y1, double z0, double z1, double k, std::shared_ptr<Material> m) {
  return rect(Kind::yzRect, y0, y1, z0, z1, k, std::move(m));
}
Hittable Hittable::makeBox(Point3 p0, Point3 p1, std::shared_ptr<Material> m) {  // Box.init, hittable.zig:434-452
  Hittable h;
  h.kind = Kind::box;
  h.box_min = p0;
  h.box_max = p1;
  h.objects.push_back(makeXyRect(p0.x, p1.x, p0.y, p1.y, p1.z, m));
  h.objects.push_back(makeXyRect(p0.x, p1.x, p0.y, p1.y, p0.z, m));
  h.objects.push_back(makeXzRect(p0.x, p1.x, p0.z, p1.z, p1.y, m));
  h.objects.push_back(makeXzRect(p0.x, p1.x, p0.z, p1.z, p0.y, m));
  h.objects.push_back(makeYzRect(p0.y, p1.y, p0.z, p1.z, p1.x, m));
  h.objects.push_back(makeYzRect(p0.y, p1.y, p0.z, p1.z, p0.x, m));
  return h;
}
Hittable Hittable::makeTranslate(std::shared_ptr<Hittable> obj, Vec3 offset) {
  Hittable h;
  h.kind = Kind::translate;
  h.object = std::move(obj);
  h.offset = offset;
  return h;
}
Hittable Hittable::makeRotateY(std::shared_ptr<Hittable> obj, double angle) {  // RotateY.init, :514-517
  Hittable h;
  h.kind = Kind::rotateY;
  h.object = std::move(obj);
  h.sin_t = rtwl::sin(angle);  // std.math.sin / cos (musl algorithms, rtw_libm.hpp)
  h.cos_t = rtwl::cos(angle);
  h.angle = angle;
  return h;
}

static double deg2rad(double degree) { return degree * 3.14159265358979323846 / 180.0; }  // main.zig:36-38

Hittable generateTwoSpheres(Random& rng) {  // main.zig:123-138
  (void)rng;
  const Texture checker = Texture::makeChecker(rgb(0.2, 0.3, 0.1), rgb(0.9, 0.9, 0.9));
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeSphere({0, -10, 0}, 10, Material::diffuse(checker)));
  objs.push_back(Hittable::makeSphere({0, 10, 0}, 10, Material::diffuse(checker)));
  return Hittable::makeList(std::move(objs));
}
Hittable generateTwoPerlinSpheres(Random& rng) {  // main.zig:140-155
  const Texture perlin = Texture::makeNoise(4.0, rng);
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeSphere({0, -1000, 0}, 1000, Material::diffuse(perlin)));
  objs.push_back(Hittable::makeSphere({0, 2, 0}, 2, Material::diffuse(perlin)));
  return Hittable::makeList(std::move(objs));
}
Hittable generateEarthScene(std::shared_ptr<Image> earth) {  // main.zig:223-233
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeSphere({0, 0, 0}, 2, Material::diffuse(Texture::makeImage(std::move(earth)))));
  return Hittable::makeList(std::move(objs));
}
Hittable generateSimpleLightScene(Random& rng) {  // main.zig:235-254
  const Texture perlin = Texture::makeNoise(4.0, rng);
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeSphere({0, -1000, 0}, 1000, Material::diffuse(perlin)));
  objs.push_back(Hittable::makeSphere({0, 2, 0}, 2, Material::diffuse(perlin)));
  objs.push_back(Hittable::makeXyRect(3.0, 5.0, 1.0, 3.0, -2.0, Material::diffuseLight(Texture::makeSolid(rgb(4, 4, 4)))));
  return Hittable::makeList(std::move(objs));
}
Hittable generateCornellBox() {  // main.zig:256-290
  auto red = Material::diffuse(Texture::makeSolid(rgb(0.65, 0.05, 0.05)));
  auto white = Material::diffuse(Texture::makeSolid(rgb(0.73, 0.73, 0.73)));
  auto green = Material::diffuse(Texture::makeSolid(rgb(0.12, 0.45, 0.15)));
  auto light = Material::diffuseLight(Texture::makeSolid(rgb(15, 15, 15)));
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeYzRect(0, 555, 0, 555, 555, green));
  objs.push_back(Hittable::makeYzRect(0, 555, 0, 555, 0, red));
  objs.push_back(Hittable::makeXzRect(213, 343, 227, 332, 554, light));
  objs.push_back(Hittable::makeXzRect(0, 555, 0, 555, 0, white));
  objs.push_back(Hittable::makeXzRect(0, 555, 0, 555, 555, white));
  objs.push_back(Hittable::makeXyRect(0, 555, 0, 555, 555, white));
  auto box1 = std::make_shared<Hittable>(Hittable::makeBox({0, 0, 0}, {165, 330, 165}, white));
  auto box1r = std::make_shared<Hittable>(Hittable::makeRotateY(box1, deg2rad(15)));
  objs.push_back(Hittable::makeTranslate(box1r, {265, 0, 295}));
  auto box2 = std::make_shared<Hittable>(Hittable::makeBox({0, 0, 0}, {165, 165, 165}, white));
  auto box2r = std::make_shared<Hittable>(Hittable::makeRotateY(box2, deg2rad(-18)));
  objs.push_back(Hittable::makeTranslate(box2r, {130, 0, 65}));
  return Hittable::makeList(std::move(objs));
}

// configs[4] (BASELINE.json): the earth texture on a radius-2 globe at
// (0, 2, 0) over the cover scene's checker ground, and the cover scene's
// random-sphere rule (main.zig:177-218) on a 100 x 100 grid (a, b in
// [-50, 50)), excluding cells within 2.5 of the globe's foot: ~10k spheres.
// Not a reference scene: its builder follows the reference's conventions.
Hittable generateGlobeScene(Random& rng, std::shared_ptr<Image> earth) {
  std::vector<Hittable> objs;
  objs.push_back(Hittable::makeSphere(
      {0, -1000, 0}, 1000, Material::diffuse(Texture::makeChecker(rgb(0.2, 0.3, 0.1), rgb(0.9, 0.9, 0.9)))));
  objs.push_back(Hittable::makeSphere({0, 2, 0}, 2, Material::diffuse(Texture::makeImage(std::move(earth)))));
  for (int a = -50; a < 50; ++a) {
    for (int b = -50; b < 50; ++b) {
      const double choose_mat = randomReal01(rng);
      Point3 center;
      center.x = (double)a + 0.9 * randomReal01(rng);
      center.y = 0.2;
      center.z = (double)b + 0.9 * randomReal01(rng);
      if (center.sub({0, 0.2, 0}).norm() <= 2.5) continue;
      if (choose_mat < 0.8) {
        const Color a1 = random01(rng);
        const Color a2 = random01(rng);
        auto m = Material::diffuse(Texture::makeSolid(a1.mulV(a2)));
        const Point3 center1 = center.add({0, randomReal(rng, 0, 0.5), 0});
        objs.push_back(Hittable::makeMovingSphere(center, center1, 0, 1, 0.2, m));
      } else if (choose_mat < 0.95) {
        const Color albedo = randomVec(rng, 0.5, 1);
        const double fuzz = randomReal(rng, 0, 0.5);
        objs.push_back(Hittable::makeSphere(center, 0.2, Material::metal(albedo, fuzz)));
      } else {
        objs.push_back(Hittable::makeSphere(center, 0.2, Material::dielectric(1.5)));
      }
    }
  }
  return Hittable::makeList(std::move(objs));
}

// ------------------------------------------------------------- flatten ----
namespace {
struct Flattener {
  FlatWorld& f;
  std::map<const Material*, uint32_t> mat_ids;
  std::map<const Perlin*, uint32_t> perlin_ids;
  std::map<const Image*, uint32_t> image_ids;

  uint32_t perlin_id(const std::shared_ptr<Perlin>& p) {
    auto it = perlin_ids.find(p.get());
    if (it != perlin_ids.end()) return it->second;
    rtw_perlin q;
    for (int i = 0; i < 256; ++i) put3(q.ranvec[i], p->ranvec[i]);
    std::memcpy(q.perm, p->perm, sizeof(q.perm));
    f.perlins.push_back(q);
    return perlin_ids[p.get()] = (uint32_t)f.perlins.size() - 1;
  }
  uint32_t image_id(const std::shared_ptr<Image>& im) {
    auto it = image_ids.find(im.get());
    if (it != image_ids.end()) return it->second;
    f.images.push_back(im);
    return image_ids[im.get()] = (uint32_t)f.images.size() - 1;
  }
  uint32_t texture(const Texture& t) {  // one table entry per material (textures are values in Zig)
    rtw_texture r;
    std::memset(&r, 0, sizeof(r));
    switch (t.kind) {
      case Texture::Kind::solid: r.kind = RTW_TEX_SOLID; put3(r.color, t.color); break;
      case Texture::Kind::checker: r.kind = RTW_TEX_CHECKER; put3(r.odd, t.odd); put3(r.even, t.even); break;
      case Texture::Kind::noise: r.kind = RTW_TEX_NOISE; r.perlin = perlin_id(t.perlin); r.scale = t.scale; break;
      case Texture::Kind::image:
        if (!t.image) throw Error(RTW_EINVAL, "image texture without an image");
        r.kind = RTW_TEX_IMAGE;
        r.image = image_id(t.image);
        break;
    }
    f.textures.push_back(r);
    return (uint32_t)f.textures.size() - 1;
  }
  uint32_t material(const std::shared_ptr<Material>& m) {  // Rc(Material) -> index
    if (!m) throw Error(RTW_EINVAL, "hittable without material");
    auto it = mat_ids.find(m.get());
    if (it != mat_ids.end()) return it->second;
    rtw_wmaterial r;
    std::memset(&r, 0, sizeof(r));
    switch (m->kind) {
      case Material::Kind::diffuse: r.kind = RTW_WMAT_LAMBERT; r.tex = texture(m->albedo); break;
      case Material::Kind::metal: r.kind = RTW_WMAT_METAL; put3(r.albedo, m->metal_albedo); r.fuzz = m->fuzz; break;
      case Material::Kind::dielectric: r.kind = RTW_WMAT_DIELECTRIC; r.ir = m->ir; break;
      case Material::Kind::diffuse_light: r.kind = RTW_WMAT_LIGHT; r.tex = texture(m->albedo); break;
    }
    f.materials.push_back(r);
    return mat_ids[m.get()] = (uint32_t)f.materials.size() - 1;
  }
  int32_t xform(const std::vector<std::pair<uint32_t, Vec3>>& chain) {
    if (chain.empty()) return -1;
    if (chain.size() > RTW_MAX_XFORM_OPS) throw Error(RTW_UNSUPPORTED, "more than 4 nested Translate/RotateY");
    rtw_xform x;
    std::memset(&x, 0, sizeof(x));
    x.n = (uint32_t)chain.size();
    for (size_t i = 0; i < chain.size(); ++i) {
      x.op[i] = chain[i].first;
      put3(x.v[i], chain[i].second);
    }
    for (size_t i = 0; i < f.xforms.size(); ++i)
      if (std::memcmp(&f.xforms[i], &x, sizeof(x)) == 0) return (int32_t)i;
    f.xforms.push_back(x);
    return (int32_t)f.xforms.size() - 1;
  }
  void walk(const Hittable& h, std::vector<std::pair<uint32_t, Vec3>>& chain) {
    rtw_prim p;
    std::memset(&p, 0, sizeof(p));
    switch (h.kind) {
      case Hittable::Kind::list:
      case Hittable::Kind::box:  // Box.hit = its sides' HittableList.hit (hittable.zig:454-456)
        for (const auto& o : h.objects) walk(o, chain);
        return;
      case Hittable::Kind::translate:
      case Hittable::Kind::rotateY:
        if (!h.object) throw Error(RTW_EINVAL, "wrapper without an object");
        chain.push_back(h.kind == Hittable::Kind::translate
                            ? std::make_pair((uint32_t)RTW_XF_TRANSLATE, h.offset)
                            : std::make_pair((uint32_t)RTW_XF_ROTATE_Y, Vec3{h.sin_t, h.cos_t, h.angle}));
        walk(*h.object, chain);
        chain.pop_back();
        return;
      case Hittable::Kind::sphere:
      case Hittable::Kind::movingSphere: {
        const bool mv = h.kind == Hittable::Kind::movingSphere;
        p.kind = mv ? RTW_PRIM_MOVING_SPHERE : RTW_PRIM_SPHERE;
        put3(p.a, h.center0);
        put3(p.a + 3, mv ? h.center1 : h.center0);
        p.a[6] = h.radius;
        p.a[7] = mv ? h.time0 : 0.0;
        p.a[8] = mv ? h.time1 : 0.0;
        break;
      }
      default:
        p.kind = h.kind == Hittable::Kind::xyRect ? RTW_PRIM_XY_RECT
                 : h.kind == Hittable::Kind::xzRect ? RTW_PRIM_XZ_RECT : RTW_PRIM_YZ_RECT;
        p.a[0] = h.a0, p.a[1] = h.a1, p.a[2] = h.b0, p.a[3] = h.b1, p.a[4] = h.k;
        break;
    }
    p.mat = material(h.material);
    p.xform = xform(chain);
    f.prims.push_back(p);
  }
};
}  // namespace

FlatWorld flattenWorld(const Hittable& world) {
  FlatWorld f;
  Flattener fl{f, {}, {}, {}};
  std::vector<std::pair<uint32_t, Vec3>> chain;
  fl.walk(world, chain);
  for (const auto& im : f.images) f.image_views.push_back(rtw_image{im->width, im->height, im->rgba.data()});
  return f;
}

rtw_world_desc FlatWorld::desc() const {
  rtw_world_desc d;
  d.prims = prims.data(), d.n_prims = (uint32_t)prims.size();
  d.xforms = xforms.data(), d.n_xforms = (uint32_t)xforms.size();
  d.textures = textures.data(), d.n_textures = (uint32_t)textures.size();
  d.mats = materials.data(), d.n_mats = (uint32_t)materials.size();
  d.perlins = perlins.data(), d.n_perlins = (uint32_t)perlins.size();
  d.images = image_views.data(), d.n_images = (uint32_t)image_views.size();
  return d;
}

rtw_scene_settings sceneSettings(uint32_t id) {  // main.zig:303-376
  rtw_scene_settings s;
  std::memset(&s, 0, sizeof(s));
  auto set = [&](Vec3 lf, Vec3 la, double vfov, double aperture, Color bg) {
    put3(s.look_from, lf);
    put3(s.look_at, la);
    s.vfov = vfov, s.aperture = aperture;
    put3(s.background, bg);
    s.aspect = 3.0 / 2.0, s.width = 600, s.spp = 50;  // main.zig:304-308
    s.height = imageHeight(600, 3.0 / 2.0);
  };
  const Color sky = rgb(0.70, 0.80, 1.00), black = rgb(0, 0, 0);
  switch (id) {
    case 1: set({13, 2, 3}, {0, 0, 0}, 20.0, 0.1, sky); break;
    case 2: case 3: case 4: set({13, 2, 3}, {0, 0, 0}, 20.0, 0.0, sky); break;
    case 5: set({26, 3, 6}, {0, 2, 0}, 20.0, 0.0, black); s.spp = 400; break;
    case 6:
      set({278, 278, -800}, {278, 278, 0}, 40.0, 0.0, black);
      s.aspect = 1.0, s.width = 600, s.height = 600, s.spp = 200;
      break;
    case 7:
      set({13, 2, 3}, {0, 1, 0}, 20.0, 0.1, sky);
      s.aspect = 16.0 / 9.0, s.width = 1200, s.height = imageHeight(1200, 16.0 / 9.0), s.spp = 100;
      break;
    default: throw Error(RTW_EINVAL, "scene id must be 1..7");
  }
  return s;
}

}  // namespace rtw

// ------------------------------------------------------- C-ABI helpers ----
struct rtw_built_scene_s {
  rtw::FlatWorld world;
  rtw_scene_settings settings;
  uint64_t rng_after[4];
};

extern "C" int rtw_build_scene(uint32_t id, uint64_t seed, const rtw_image* image, rtw_built_scene* out) {
  if (!out) return RTW_EINVAL;
  *out = nullptr;
  try {
    if ((id == 4 || id == 7) && (!image || !image->rgba || image->width == 0 || image->height == 0))
      return RTW_EINVAL;
    std::shared_ptr<rtw::Image> earth;
    if (image && image->rgba) {
      earth = std::make_shared<rtw::Image>();
      earth->width = image->width, earth->height = image->height;
      earth->rgba.assign(image->rgba, image->rgba + (size_t)image->width * image->height * 4);
    }
    rtw::Random rng = rtw::Random::init(seed);  // main.zig:300
    rtw::Hittable world;
    switch (id) {
      case 1: world = rtw::generateRandomScene(rng); break;
      case 2: world = rtw::generateTwoSpheres(rng); break;
      case 3: world = rtw::generateTwoPerlinSpheres(rng); break;
      case 4: world = rtw::generateEarthScene(earth); break;
      case 5: world = rtw::generateSimpleLightScene(rng); break;
      case 6: world = rtw::generateCornellBox(); break;
      case 7: world = rtw::generateGlobeScene(rng, earth); break;
      default: return RTW_EINVAL;
    }
    auto* b = new rtw_built_scene_s;
    b->world = rtw::flattenWorld(world);
    b->settings = rtw::sceneSettings(id);
    rng.state(b->rng_after);
    *out = b;
    return RTW_OK;
  } catch (const rtw::Error& e) {
    return e.status;
  } catch (...) {
    return RTW_ENOMEM;
  }
}

extern "C" int rtw_built_scene_desc(rtw_built_scene b, rtw_world_desc* desc, rtw_scene_settings* settings,
                                    uint64_t rng_state_after[4]) {
  if (!b) return RTW_EINVAL;
  if (desc) *desc = b->world.desc();
  if (settings) *settings = b->settings;
  if (rng_state_after) std::memcpy(rng_state_after, b->rng_after, sizeof(b->rng_after));
  return RTW_OK;
}

extern "C" int rtw_built_scene_free(rtw_built_scene b) {
  delete b;
  return RTW_OK;
}
