// rtw_host.hpp — C++ host-side mirror of the reference's src/rtw API for the
// cover-scene path (the reference's host is Zig, which this image cannot
// build; INTEGRATION.md shows the Zig binding a maintainer would add).
//
// Same names, argument meaning and behaviour as the Zig module:
//   rtw::Vec3 / Point3 / Color      src/rtw/vec.zig:8-109
//   rtw::Random (DefaultPrng)       std.Random.DefaultPrng, used at main.zig:300
//   rtw::rand helpers               src/rtw/rand.zig:1-40
//   rtw::Texture                    src/rtw/texture.zig:10-144 (solid, checker, noise, image)
//   rtw::Perlin                     src/rtw/perlin.zig:10-124
//   rtw::Material                   src/rtw/material.zig:16-110
//   rtw::Hittable                   src/rtw/hittable.zig:22-608 (sphere, movingSphere, list,
//                                   xy/xz/yzRect, box, translate, rotateY)
//   rtw::Camera                     src/main.zig:40-101
//   rtw::generate*                  src/main.zig:123-290 (scenes 1-6) + the configs[4] globe
//                                   scene (rtw_world_host.cpp)
//   rtw::render                     replaces src/main.zig:378-402 via rtw_render()
// Zig error unions map to rtw::Error exceptions on the C++ side only; nothing
// crosses the C ABI except status codes.
#pragma once
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "rtw_hip.h"

namespace rtw {

struct Error : std::runtime_error {
  int status;
  Error(int st, const std::string& m) : std::runtime_error(m), status(st) {}
};

struct Vec3 {
  double x = 0, y = 0, z = 0;
  double normSquared() const { return x * x + y * y + z * z; }
  double norm() const;
  double dot(const Vec3& v) const { return x * v.x + y * v.y + z * v.z; }
  Vec3 cross(const Vec3& v) const { return {y * v.z - z * v.y, z * v.x - x * v.z, x * v.y - y * v.x}; }
  Vec3 normalized() const;
  Vec3 add(const Vec3& v) const { return {x + v.x, y + v.y, z + v.z}; }
  Vec3 sub(const Vec3& v) const { return {x - v.x, y - v.y, z - v.z}; }
  Vec3 mul(double t) const { return {x * t, y * t, z * t}; }
  Vec3 mulV(const Vec3& v) const { return {x * v.x, y * v.y, z * v.z}; }
  Vec3 div(double t) const { return {x / t, y / t, z / t}; }
};
using Point3 = Vec3;
using Color = Vec3;
inline Color rgb(double r, double g, double b) { return {r, g, b}; }

// std.Random.DefaultPrng = Xoshiro256 (xoshiro256++), SplitMix64-seeded.
class Random {
 public:
  static Random init(uint64_t seed);
  uint64_t next();
  double float64();  // Random.float(f64)
  void state(uint64_t out[4]) const;

 private:
  uint64_t s_[4] = {0, 0, 0, 0};
};

// rand.zig
double randomReal01(Random& rng);                          // rand.zig:13-15
double randomReal(Random& rng, double min, double max);    // rand.zig:18-20
Vec3 random01(Random& rng);                                // vec.zig:82-88
Vec3 randomVec(Random& rng, double min, double max);       // vec.zig:90-96

// Random.intRangeLessThan for u64 (Zig std, Lemire; rand.zig:8-10).
uint64_t randomIntLessThan(Random& rng, uint64_t at_least, uint64_t less_than);

struct Perlin {  // perlin.zig:10-124
  Vec3 ranvec[256];
  uint32_t perm[3][256];
  static std::shared_ptr<Perlin> init(Random& rng);  // perlin.zig:18-40
};

struct Image {  // zigimg Image, decoded to RGBA8 (texture.zig:107-118)
  uint32_t width = 0, height = 0;
  std::vector<uint8_t> rgba;
};

struct Texture {
  enum class Kind { solid, checker, noise, image } kind = Kind::solid;
  Color color;      // solid
  Color odd, even;  // checker (texture.zig:57-83)
  std::shared_ptr<Perlin> perlin;  // noise (texture.zig:85-105)
  double scale = 1;
  std::shared_ptr<Image> image;    // image (texture.zig:107-144)
  static Texture makeSolid(Color c);
  static Texture makeChecker(Color odd, Color even);        // texture.zig:17-23
  static Texture makeNoise(double scale, Random& rng);      // texture.zig:28-30
  static Texture makeImage(std::shared_ptr<Image> image);   // texture.zig:32-34
};

struct Material {
  enum class Kind { diffuse, metal, dielectric, diffuse_light } kind = Kind::diffuse;
  Texture albedo;      // diffuse albedo / diffuse_light emit
  Color metal_albedo;  // metal
  double fuzz = 0;     // metal
  double ir = 1;       // dielectric
  static std::shared_ptr<Material> diffuse(Texture t);
  static std::shared_ptr<Material> metal(Color albedo, double fuzz);
  static std::shared_ptr<Material> dielectric(double ir);
  static std::shared_ptr<Material> diffuseLight(Texture emit);  // material.zig:94-110
};

struct Hittable {
  enum class Kind { sphere, movingSphere, list, xyRect, xzRect, yzRect, box, translate, rotateY } kind = Kind::list;
  Point3 center0, center1;
  double time0 = 0, time1 = 1, radius = 0;
  double a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0;  // rects (first, second in-plane axis; plane offset)
  Point3 box_min, box_max;                       // box (sides in `objects`)
  Vec3 offset;                                   // translate
  double sin_t = 0, cos_t = 1, angle = 0;        // rotateY
  std::shared_ptr<Hittable> object;              // translate / rotateY: Rc(Hittable)
  std::shared_ptr<Material> material;  // Rc(Material) (src/rc.zig)
  std::vector<Hittable> objects;       // list, box sides
  static Hittable makeSphere(Point3 c, double r, std::shared_ptr<Material> m);  // main.zig:26-34
  static Hittable makeMovingSphere(Point3 c0, Point3 c1, double t0, double t1, double r,
                                   std::shared_ptr<Material> m);
  static Hittable makeList(std::vector<Hittable> objs);
  static Hittable makeXyRect(double x0, double x1, double y0, double y1, double k, std::shared_ptr<Material> m);
  static Hittable makeXzRect(double x0, double x1, double z0, double z1, double k, std::shared_ptr<Material> m);
  static Hittable makeYzRect(double y0, double y1, double z0, double z1, double k, std::shared_ptr<Material> m);
  static Hittable makeBox(Point3 p0, Point3 p1, std::shared_ptr<Material> m);             // hittable.zig:34-36
  static Hittable makeTranslate(std::shared_ptr<Hittable> obj, Vec3 offset);            // hittable.zig:38-40
  static Hittable makeRotateY(std::shared_ptr<Hittable> obj, double angle_rad);         // hittable.zig:42-44
};

struct Camera {  // main.zig:40-101
  Point3 origin, lower_left_corner;
  Vec3 horizontal, vertical, u, v, w;
  double lens_radius = 0, time0 = 0, time1 = 0;
  static Camera init(Point3 look_from, Point3 look_at, Vec3 vup, double vfov, double aspect_ratio,
                     double aperture, double focus_dist, double time0, double time1);
  rtw_camera to_c() const;
};

// main.zig:157-221
Hittable generateRandomScene(Random& rng);
// main.zig:123-155, :223-290, and the configs[4] globe scene (rtw_world_host.cpp)
Hittable generateTwoSpheres(Random& rng);
Hittable generateTwoPerlinSpheres(Random& rng);
Hittable generateEarthScene(std::shared_ptr<Image> earth);
Hittable generateSimpleLightScene(Random& rng);
Hittable generateCornellBox();
Hittable generateGlobeScene(Random& rng, std::shared_ptr<Image> earth);

// The general world -> flat arrays of the world ABI (rtw_world_desc).
struct FlatWorld {
  std::vector<rtw_prim> prims;
  std::vector<rtw_xform> xforms;
  std::vector<rtw_texture> textures;
  std::vector<rtw_wmaterial> materials;
  std::vector<rtw_perlin> perlins;
  std::vector<std::shared_ptr<Image>> images;
  std::vector<rtw_image> image_views;
  rtw_world_desc desc() const;
};
FlatWorld flattenWorld(const Hittable& world);
// Scene settings of main() (main.zig:303-376) for scene ids 1-7.
rtw_scene_settings sceneSettings(uint32_t scene_id);

// The world -> flat arrays of the C ABI (Rc(Material) pointers -> indices).
struct FlatScene {
  std::vector<rtw_sphere> spheres;
  std::vector<rtw_material> materials;
};
FlatScene flatten(const Hittable& world);

// Image parameters of the reference main() (main.zig:303-310, :320-326).
struct RenderSettings {
  uint32_t width = 600;
  double aspect_ratio = 3.0 / 2.0;
  uint32_t samples_per_pixel = 50;
  uint32_t max_depth = 50;
  uint64_t seed = 42;
  Color background = rgb(0.70, 0.80, 1.00);
  uint32_t precision = RTW_PRECISION_F64;
  uint32_t chunk = 0;
  uint32_t engine = RTW_ENGINE_MEGAKERNEL;  // or RTW_ENGINE_WAVEFRONT (same image)
};
uint32_t imageHeight(uint32_t width, double aspect_ratio);  // main.zig:306

// Replaces main.zig:378-402: returns rgb24 (top row first, main.zig:396).
std::vector<uint8_t> render(const Camera& cam, const Hittable& world, const RenderSettings& s,
                            uint32_t height);

void writePPM(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h);

}  // namespace rtw
