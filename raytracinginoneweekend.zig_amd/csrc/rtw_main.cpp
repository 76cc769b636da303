// rtw_main.cpp — command-line renderer: the reference's main() (main.zig:295-405)
// with the render loop replaced by the GPU (rtw_render for the cover scene's
// megakernel, rtw_world_render for every other scene).  Writes PPM (the
// reference writes PNG via zigimg; the pixel bytes are identical, main.zig:396).
//   rtw_render [--scene 1..7] [--width W] [--aspect A|W:H] [--spp N] [--depth D]
//              [--seed S] [--precision f64|f32] [--engine megakernel|wavefront]
//              [--chunk C] [--image earth.png] [--out out.ppm]
// Defaults are the reference's: scene 6 (main.zig:313) with that scene's own
// size, spp, camera and background (main.zig:316-362); --width/--aspect/--spp
// override them.  Scenes 4 and 7 need --image (assets/sekaichizu.png).
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtw_host.hpp"

static double parse_aspect(const char* s) {
  const char* c = std::strchr(s, ':');
  if (c) return std::atof(s) / std::atof(c + 1);
  return std::atof(s);
}

static uint32_t be32(const unsigned char* p) { return (uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]; }

// 8-bit non-interlaced PNG -> RGBA8 (what zigimg hands texture.zig:133-140 for
// an RGBA file; grey / RGB / palette are expanded to RGBA).
static std::shared_ptr<rtw::Image> loadPNG(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw rtw::Error(RTW_EINVAL, "cannot open " + path);
  std::vector<unsigned char> d;
  unsigned char buf[65536];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
  std::fclose(f);
  if (d.size() < 8 || std::memcmp(d.data(), "\x89PNG\r\n\x1a\n", 8) != 0) throw rtw::Error(RTW_EINVAL, path + ": not a PNG");
  uint32_t w = 0, h = 0;
  int depth = 0, ctype = 0, interlace = 0;
  std::vector<unsigned char> idat, plte, trns;
  for (size_t i = 8; i + 12 <= d.size();) {
    const uint32_t len = be32(&d[i]);
    const std::string typ(reinterpret_cast<const char*>(&d[i + 4]), 4);
    const unsigned char* body = &d[i + 8];
    if (typ == "IHDR") {
      w = be32(body), h = be32(body + 4), depth = body[8], ctype = body[9], interlace = body[12];
    } else if (typ == "PLTE") {
      plte.assign(body, body + len);
    } else if (typ == "tRNS") {
      trns.assign(body, body + len);
    } else if (typ == "IDAT") {
      idat.insert(idat.end(), body, body + len);
    } else if (typ == "IEND") {
      break;
    }
    i += 12 + len;
  }
  if (depth != 8 || interlace != 0) throw rtw::Error(RTW_UNSUPPORTED, path + ": only 8-bit non-interlaced PNGs");
  const int ch = ctype == 6 ? 4 : ctype == 2 ? 3 : ctype == 4 ? 2 : 1;
  const size_t stride = (size_t)w * ch;
  std::vector<unsigned char> raw((stride + 1) * h);
  uLongf rl = (uLongf)raw.size();
  if (uncompress(raw.data(), &rl, idat.data(), (uLong)idat.size()) != Z_OK || rl != raw.size())
    throw rtw::Error(RTW_EINVAL, path + ": bad image data");
  std::vector<unsigned char> px(stride * h), prev(stride, 0);
  for (uint32_t y = 0; y < h; ++y) {  // scanline filters (PNG spec section 9)
    const unsigned char ft = raw[y * (stride + 1)];
    const unsigned char* line = &raw[y * (stride + 1) + 1];
    unsigned char* cur = &px[y * stride];
    for (size_t x = 0; x < stride; ++x) {
      const int a = x >= (size_t)ch ? cur[x - ch] : 0, b = prev[x], c = x >= (size_t)ch ? prev[x - ch] : 0;
      int pred = 0;
      if (ft == 1) pred = a;
      else if (ft == 2) pred = b;
      else if (ft == 3) pred = (a + b) >> 1;
      else if (ft == 4) {
        const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
        pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
      }
      cur[x] = (unsigned char)(line[x] + pred);
    }
    std::memcpy(prev.data(), cur, stride);
  }
  auto im = std::make_shared<rtw::Image>();
  im->width = w, im->height = h;
  im->rgba.resize((size_t)w * h * 4);
  for (size_t i = 0; i < (size_t)w * h; ++i) {
    unsigned char* o = &im->rgba[4 * i];
    const unsigned char* s = &px[ch * i];
    if (ctype == 6) std::memcpy(o, s, 4);
    else if (ctype == 2) o[0] = s[0], o[1] = s[1], o[2] = s[2], o[3] = 255;
    else if (ctype == 4) o[0] = o[1] = o[2] = s[0], o[3] = s[1];
    else if (ctype == 0) o[0] = o[1] = o[2] = s[0], o[3] = 255;
    else {
      o[0] = plte[3 * s[0]], o[1] = plte[3 * s[0] + 1], o[2] = plte[3 * s[0] + 2];
      o[3] = s[0] < trns.size() ? trns[s[0]] : 255;
    }
  }
  return im;
}

int main(int argc, char** argv) {
  uint32_t scene = 6;  // main.zig:313
  uint32_t width = 0, spp = 0, depth = 50, chunk = 0, precision = RTW_PRECISION_F64, engine = RTW_ENGINE_MEGAKERNEL;
  double aspect = 0;
  uint64_t seed = 42;
  std::string out = "out.ppm", image_path;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--scene") scene = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--width") width = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--aspect") aspect = parse_aspect(v);
    else if (k == "--spp") spp = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--depth") depth = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--seed") seed = std::strtoull(v, nullptr, 10);
    else if (k == "--precision") precision = std::string(v) == "f32" ? RTW_PRECISION_F32 : RTW_PRECISION_F64;
    else if (k == "--engine") engine = std::string(v) == "wavefront" ? RTW_ENGINE_WAVEFRONT : RTW_ENGINE_MEGAKERNEL;
    else if (k == "--chunk") chunk = (uint32_t)std::strtoul(v, nullptr, 10);
    else if (k == "--image") image_path = v;
    else if (k == "--out") out = v;
    else {
      std::fprintf(stderr, "unknown option %s\n", k.c_str());
      return 2;
    }
  }
  try {
    const rtw_scene_settings st = rtw::sceneSettings(scene);  // main.zig:303-362
    const double asp = aspect > 0 ? aspect : st.aspect;
    const uint32_t W = width ? width : st.width;
    const uint32_t H = (width || aspect > 0) ? rtw::imageHeight(W, asp) : st.height;
    const uint32_t S = spp ? spp : st.spp;
    const rtw::Camera cam = rtw::Camera::init({st.look_from[0], st.look_from[1], st.look_from[2]},
                                              {st.look_at[0], st.look_at[1], st.look_at[2]}, {0, 1, 0}, st.vfov, asp,
                                              st.aperture, 10.0, 0, 1);  // main.zig:366-376
    rtw::Random rng = rtw::Random::init(seed);                           // main.zig:300-301
    std::vector<uint8_t> rgb((size_t)W * H * 3);
    if (scene == 1) {  // the cover scene: the sphere megakernel (or the wavefront engine)
      rtw::RenderSettings rs;
      rs.width = W, rs.aspect_ratio = asp, rs.samples_per_pixel = S, rs.max_depth = depth, rs.seed = seed;
      rs.precision = precision, rs.chunk = chunk, rs.engine = engine;
      rs.background = {st.background[0], st.background[1], st.background[2]};
      const rtw::Hittable world = rtw::generateRandomScene(rng);
      rgb = rtw::render(cam, world, rs, H);  // main.zig:378-402
    } else {
      std::shared_ptr<rtw::Image> earth;
      if (scene == 4 || scene == 7) {
        if (image_path.empty()) throw rtw::Error(RTW_EINVAL, "scenes 4 and 7 need --image assets/sekaichizu.png");
        earth = loadPNG(image_path);
      }
      rtw::Hittable world;
      switch (scene) {
        case 2: world = rtw::generateTwoSpheres(rng); break;
        case 3: world = rtw::generateTwoPerlinSpheres(rng); break;
        case 4: world = rtw::generateEarthScene(earth); break;
        case 5: world = rtw::generateSimpleLightScene(rng); break;
        case 6: world = rtw::generateCornellBox(); break;
        case 7: world = rtw::generateGlobeScene(rng, earth); break;
        default: throw rtw::Error(RTW_EINVAL, "scene must be 1..7");
      }
      const rtw::FlatWorld fw = rtw::flattenWorld(world);
      const rtw_world_desc desc = fw.desc();
      rtw_params p;
      std::memset(&p, 0, sizeof(p));
      p.width = W, p.height = H, p.spp = S, p.max_depth = depth, p.seed = seed;
      for (int k = 0; k < 3; ++k) p.background[k] = st.background[k];
      p.row_begin = 0, p.row_stride = 1, p.row_count = H, p.chunk = chunk, p.precision = RTW_PRECISION_F64;
      p.device = -1, p.engine = RTW_ENGINE_MEGAKERNEL;
      const rtw_camera c = cam.to_c();
      const int rc = rtw_world_render(&c, &desc, &p, rgb.data(), nullptr);  // main.zig:378-402
      if (rc != RTW_OK) throw rtw::Error(rc, rtw_last_error());
    }
    rtw::writePPM(out, rgb, W, H);  // main.zig:405
    std::fprintf(stderr, "wrote %s (scene %u, %ux%u, %u spp)\n", out.c_str(), scene, W, H, S);
  } catch (const rtw::Error& e) {
    std::fprintf(stderr, "rtw_render: %s (status %d)\n", e.what(), e.status);
    return 1;
  }
  return 0;
}
