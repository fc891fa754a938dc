// tests/native/sanitize_driver.cpp — TEST ONLY. The host code that parses untrusted files (the
// COLLADA loader, the OpenEXR reader, the camera-settings reader), the scene preparation
// (bdpt_scene.cpp: BVH builds, flattening) and the device core's CPU build (bdpt_core.h via
// core_cpu.cpp) linked into one executable built with -fsanitize=address,undefined by
// tests/test_sanitizers.py (ASan/UBSan on host code). It runs the real inputs and
// then mutated copies of them (truncations, byte flips): every load must either succeed or fail
// with an error code — never read or write out of bounds. Exit 0 = clean run; a sanitizer report
// aborts (halt_on_error).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <random>
#include <string>
#include <vector>

#include "bdpt/bdpt.h"
#include "bdpt_scene.h"

namespace bdpt { thread_local std::string g_err; }

extern "C" int core_cpu_render(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed, int s0,
                               int count, const int* pixels, int npix, double* eye, double* light, double* stats,
                               int lds_mode, int rr);

static std::vector<char> slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  return std::vector<char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}
static void spit(const std::string& p, const std::vector<char>& b) {
  std::ofstream f(p, std::ios::binary);
  f.write(b.data(), (std::streamsize)b.size());
}

static int load_scene(const std::string& path, int W, int H, bool render, int lds_mode) {
  bdpt_dae* dae = nullptr;
  int rc = bdpt_dae_load(path.c_str(), W, H, &dae);
  if (rc != BDPT_OK) return rc;
  bdpt_scene_desc d;
  bdpt_dae_get_desc(dae, &d);
  bdpt::HostScene hs;
  std::string err;
  rc = bdpt::build_host_scene(&d, hs, err);
  if (rc == BDPT_E_UNSUPPORTED) {   // lights / materials only the PathTracer takes
    bdpt::HostScene hp;
    rc = bdpt::build_host_scene(&d, hp, err, true);
    render = false;
  }
  if (rc == BDPT_OK && render) {
    std::vector<double> eye((size_t)W * H * 3), light((size_t)W * H * 3), st(8);
    rc = core_cpu_render(&d, W, H, 1, 5, 5489, 0, 1, nullptr, 0, eye.data(), light.data(), st.data(), lds_mode, 0);
  }
  bdpt_dae_free(dae);
  return rc;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: sanitize_driver <tmpdir> <files...> (.dae / .exr / .txt camera settings)\n");
    return 2;
  }
  const std::string tmp = argv[1];
  std::mt19937 rng(12345);
  int loads = 0, failures = 0;
  for (int a = 2; a < argc; a++) {
    const std::string p = argv[a];
    const std::string ext = p.substr(p.find_last_of('.') + 1);
    auto run = [&](const std::string& f, bool real) {
      int rc = BDPT_OK;
      if (ext == "dae") {
        rc = load_scene(f, 24, 18, real, 0);
        if (real && rc == BDPT_OK) rc = load_scene(f, 24, 18, true, 1);
      } else if (ext == "exr") {
        int32_t w = 0, h = 0;
        float* rgb = nullptr;
        rc = bdpt_exr_load(f.c_str(), &w, &h, &rgb);
        if (rc == BDPT_OK) {
          double s = 0;
          for (size_t k = 0; k < (size_t)w * h * 3; k++) s += rgb[k];
          if (s != s && real) rc = -100;
          bdpt_exr_free(rgb);
        }
      } else if (ext == "txt") {
        bdpt_camera cam;
        memset(&cam, 0, sizeof cam);
        rc = bdpt_camera_load_settings(f.c_str(), &cam);
      }
      loads++;
      if (rc != BDPT_OK) failures++;
      if (real && rc != BDPT_OK) {
        fprintf(stderr, "real input failed: %s rc=%d %s\n", f.c_str(), rc, bdpt::g_err.c_str());
        exit(3);
      }
    };
    run(p, true);
    const std::vector<char> orig = slurp(p);
    if (orig.empty()) continue;
    const std::string m = tmp + "/mut." + ext;
    // truncations at 8 cut points, then 24 copies with 1-16 random bytes changed
    for (int k = 1; k <= 8; k++) {
      std::vector<char> b(orig.begin(), orig.begin() + (long)(orig.size() * k / 9));
      spit(m, b);
      run(m, false);
    }
    for (int k = 0; k < 24; k++) {
      std::vector<char> b = orig;
      const int nflip = 1 + (int)(rng() % 16);
      for (int q = 0; q < nflip; q++) b[rng() % b.size()] = (char)(rng() & 0xff);
      spit(m, b);
      run(m, false);
    }
  }
  printf("sanitize_driver: %d loads, %d rejected inputs, no sanitizer report\n", loads, failures);
  return 0;
}
