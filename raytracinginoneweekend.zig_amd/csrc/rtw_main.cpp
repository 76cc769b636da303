// rtw_main.cpp — command-line renderer: the reference's main() (main.zig:295-405)
// for scene 1 with the render loop replaced by rtw_render (GPU).  Writes PPM
// (the reference writes PNG via zigimg; the bytes are identical, main.zig:396).
//   rtw_render [--width W] [--aspect A|W:H] [--spp N] [--depth D] [--seed S]
//              [--precision f64|f32] [--chunk C] [--out out.ppm]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "rtw_host.hpp"

static double parse_aspect(const char* s) {
  const char* c = std::strchr(s, ':');
  if (c) return std::atof(s) / std::atof(c + 1);
  return std::atof(s);
}

int main(int argc, char** argv) {
  rtw::RenderSettings s;  // main.zig:303-310 defaults (600 wide, 3:2, 50 spp, depth 50)
  std::string out = "out.ppm";
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--width") s.width = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--aspect") s.aspect_ratio = parse_aspect(v);
    else if (k == "--spp") s.samples_per_pixel = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--depth") s.max_depth = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--seed") s.seed = std::strtoull(v, nullptr, 10);
    else if (k == "--precision") s.precision = std::string(v) == "f32" ? RTW_PRECISION_F32 : RTW_PRECISION_F64;
    else if (k == "--chunk") s.chunk = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--out") out = v;
    else {
      std::fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  try {
    rtw::Random rng = rtw::Random::init(s.seed);                 // main.zig:300-301
    const rtw::Hittable world = rtw::generateRandomScene(rng);    // main.zig:321
    const uint32_t height = rtw::imageHeight(s.width, s.aspect_ratio);
    const rtw::Camera cam = rtw::Camera::init({13, 2, 3}, {0, 0, 0}, {0, 1, 0}, 20.0, s.aspect_ratio, 0.1, 10.0,
                                              0, 1);              // main.zig:323-326, :366-376
    const auto rgb = rtw::render(cam, world, s, height);         // main.zig:378-402
    rtw::writePPM(out, rgb, s.width, height);                    // main.zig:405
    std::fprintf(stderr, "wrote %s (%ux%u, %u spp)\n", out.c_str(), s.width, height, s.samples_per_pixel);
  } catch (const rtw::Error& e) {
    std::fprintf(stderr, "rtw_render: %s (status %d)\n", e.what(), e.status);
    return 1;
  }
  return 0;
}
