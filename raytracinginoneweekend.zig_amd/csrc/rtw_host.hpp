// rtw_host.hpp — C++ host-side mirror of the reference's src/rtw API for the
// cover-scene path (the reference's host is Zig, which this image cannot
// build; INTEGRATION.md shows the Zig binding a maintainer would add).
//
// Same names, argument meaning and behaviour as the Zig module:
//   rtw::Vec3 / Point3 / Color      src/rtw/vec.zig:8-109
//   rtw::Random (DefaultPrng)       std.Random.DefaultPrng, used at main.zig:300
//   rtw::rand helpers               src/rtw/rand.zig:1-40
//   rtw::Texture                    src/rtw/texture.zig:10-83 (solid, checker)
//   rtw::Material                   src/rtw/material.zig:16-92
//   rtw::Hittable                   src/rtw/hittable.zig:22-268 (sphere, movingSphere, list)
//   rtw::Camera                     src/main.zig:40-101
//   rtw::generateRandomScene        src/main.zig:157-221
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

struct Texture {
  enum class Kind { solid, checker } kind = Kind::solid;
  Color color;      // solid
  Color odd, even;  // checker (texture.zig:57-83)
  static Texture makeSolid(Color c);
  static Texture makeChecker(Color odd, Color even);  // texture.zig:17-23
};

struct Material {
  enum class Kind { diffuse, metal, dielectric, diffuse_light } kind = Kind::diffuse;
  Texture albedo;      // diffuse
  Color metal_albedo;  // metal
  double fuzz = 0;     // metal
  double ir = 1;       // dielectric
  static std::shared_ptr<Material> diffuse(Texture t);
  static std::shared_ptr<Material> metal(Color albedo, double fuzz);
  static std::shared_ptr<Material> dielectric(double ir);
};

struct Hittable {
  enum class Kind { sphere, movingSphere, list } kind = Kind::list;
  Point3 center0, center1;
  double time0 = 0, time1 = 1, radius = 0;
  std::shared_ptr<Material> material;  // Rc(Material) (src/rc.zig)
  std::vector<Hittable> objects;       // list
  static Hittable makeSphere(Point3 c, double r, std::shared_ptr<Material> m);  // main.zig:26-34
  static Hittable makeMovingSphere(Point3 c0, Point3 c1, double t0, double t1, double r,
                                   std::shared_ptr<Material> m);
  static Hittable makeList(std::vector<Hittable> objs);
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
};
uint32_t imageHeight(uint32_t width, double aspect_ratio);  // main.zig:306

// Replaces main.zig:378-402: returns rgb24 (top row first, main.zig:396).
std::vector<uint8_t> render(const Camera& cam, const Hittable& world, const RenderSettings& s,
                            uint32_t height);

void writePPM(const std::string& path, const std::vector<uint8_t>& rgb, uint32_t w, uint32_t h);

}  // namespace rtw
