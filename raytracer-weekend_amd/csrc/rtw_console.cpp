// rtw_console.cpp — the build's console_app (console_app/src/main.rs:15-96) on the GPU core.
//
//   rtw_console <scene> [-w|--width 400] [-a|--aspect-ratio 1.7777778] [-s|--samples-per-pixel 100]
//               [--seed 0] [--models models] [--out render]
// Same Opts and defaults (main.rs:15-26), height = round(width / aspect) (:33), camera
// aspect = width / height as f32 (:38-41), tonemap (:68-90), PNG to render/image_0000.png (:92-94).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <zlib.h>

#include <string>
#include <vector>

#include "rtw.hpp"

static void put32(std::vector<uint8_t>& v, uint32_t x) {
  for (int s = 24; s >= 0; s -= 8) v.push_back((uint8_t)(x >> s));
}
static void chunk(FILE* f, const char* type, const std::vector<uint8_t>& data) {
  std::vector<uint8_t> buf;
  put32(buf, (uint32_t)data.size());
  buf.insert(buf.end(), type, type + 4);
  buf.insert(buf.end(), data.begin(), data.end());
  uint32_t crc = (uint32_t)crc32(0, buf.data() + 4, (uInt)(buf.size() - 4));
  put32(buf, crc);
  fwrite(buf.data(), 1, buf.size(), f);
}
static bool write_png(const char* path, const uint8_t* rgb, uint32_t w, uint32_t h) {
  FILE* f = fopen(path, "wb");
  if (!f) return false;
  static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
  fwrite(sig, 1, 8, f);
  std::vector<uint8_t> ihdr;
  put32(ihdr, w);
  put32(ihdr, h);
  ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});
  chunk(f, "IHDR", ihdr);
  std::vector<uint8_t> raw;
  raw.reserve((size_t)h * (w * 3 + 1));
  for (uint32_t y = 0; y < h; ++y) {
    raw.push_back(0);
    raw.insert(raw.end(), rgb + (size_t)y * w * 3, rgb + (size_t)(y + 1) * w * 3);
  }
  uLongf n = compressBound((uLong)raw.size());
  std::vector<uint8_t> z(n);
  compress2(z.data(), &n, raw.data(), (uLong)raw.size(), 6);
  z.resize(n);
  chunk(f, "IDAT", z);
  chunk(f, "IEND", {});
  return fclose(f) == 0;
}

int main(int argc, char** argv) {
  std::string scene, models = "models", out_dir = "render";
  uint32_t width = 400, spp = 100;
  double aspect = 1.7777778;
  uint64_t seed = 0;
  for (int k = 1; k < argc; ++k) {
    std::string a = argv[k];
    auto next = [&](const char* what) -> const char* {
      if (k + 1 >= argc) { fprintf(stderr, "missing value for %s\n", what); exit(2); }
      return argv[++k];
    };
    if (a == "-w" || a == "--width") width = (uint32_t)atoi(next("--width"));
    else if (a == "-a" || a == "--aspect-ratio") aspect = atof(next("--aspect-ratio"));
    else if (a == "-s" || a == "--samples-per-pixel") spp = (uint32_t)atoi(next("--samples-per-pixel"));
    else if (a == "--seed") seed = strtoull(next("--seed"), nullptr, 0);
    else if (a == "--models") models = next("--models");
    else if (a == "--out") out_dir = next("--out");
    else if (a == "-h" || a == "--help") {
      printf("usage: rtw_console <jumpy-balls|two-spheres|two-perlin-spheres|earth|simple-light|cornell-box|"
             "smokey-cornell-box|book2-final-scene|animated-book2-final-scene|simple-triangle|wavefront-cow-obj|"
             "wavefront-suspension-obj|textured-monument> [-w W] [-a ASPECT] [-s SPP] [--seed N] [--models DIR] "
             "[--out DIR]\n");
      return 0;
    } else if (scene.empty()) scene = a;
    else { fprintf(stderr, "unexpected argument '%s'\n", a.c_str()); return 2; }
  }
  if (scene.empty()) { fprintf(stderr, "missing scene subcommand (try --help)\n"); return 2; }
  const uint32_t height = (uint32_t)llround((double)width / aspect);  // main.rs:33 (f64 round)
  try {
    rtw::World world;
    rtw::Camera cam;
    rtw::Color bg;
    const float cam_aspect = (float)width / (float)height;  // main.rs:38-41
    world.preset(scene, cam_aspect, seed, models, cam, bg);
    world.commit();  // flattened and uploaded once, reused by every camera (main.rs:47-56)
    const std::vector<rtw::Camera> cams = rtw::World::preset_cameras(scene, cam_aspect, models);
    mkdir(out_dir.c_str(), 0755);
    for (size_t frame = 0; frame < cams.size(); ++frame) {
      rtw::Raytracer rt(world, cams[frame], bg, width, height, spp, seed);
      rtw_stats st;
      std::vector<float> sums = rt.render_sums(&st);
      std::vector<uint8_t> img(sums.size());
      rtw::check(rtw_tonemap(sums.data(), width * height, spp, img.data()));
      char name[32];
      snprintf(name, sizeof name, "/image_%04zu.png", frame);  // main.rs:92-94
      std::string path = out_dir + name;
      if (!write_png(path.c_str(), img.data(), width, height)) { fprintf(stderr, "cannot write %s\n", path.c_str()); return 1; }
      printf("%s %ux%u %u spp: %.1f ms kernel, %llu rays, %.1f Mrays/s -> %s\n", scene.c_str(), width, height, spp,
             st.kernel_ms, (unsigned long long)st.rays, st.rays / (st.kernel_ms * 1e3), path.c_str());
    }
  } catch (const rtw::Error& e) {
    fprintf(stderr, "error %d: %s\n", e.code, e.what());
    return 1;
  }
  return 0;
}
