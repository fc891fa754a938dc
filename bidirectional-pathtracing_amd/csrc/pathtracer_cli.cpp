// pathtracer_cli.cpp — the reference's `pathtracer` command line (src/application/main.cpp:62-200)
// in windowless mode, rendering through libbdpt_amd.so on MI355X GPUs.
//
//   pathtracer [-s spp] [-m max_depth] [-r W H] [-f out.png] [-p x y dx dy] [-t threads] [-c cam.txt]
//              [-l n] [-e envmap.exr] [--rr] [-g gpus] [-S seed] [--dump-scene scene.json]
//              [--pt [-a batch tol] [-H] [-b lens] [-d focal]] scene.dae
//
// Same flags and defaults as the reference (-s 1, -m 1, 800x600 when -r is absent; -t / -l are
// accepted and do not apply to the GPU path; -p renders one cell). -g N splits the sample range
// over N devices (one context and one host thread per device) and sums the frames on the devices with
// one RCCL reduce into device 0's (bdpt_reduce_frames, inside the timed region). -e loads an
// environment map as the reference's -e does (load_exr, main.cpp:115-119) — under BDPT, which the
// reference cannot run with it; --rr turns on Russian roulette (bidirection.cpp:87-93).
// --pt selects the reference's unidirectional PathTracer (pathtracer.cpp:47-340) with its flags
// -l, -a, -H, -b, -d (main.cpp:107-141); its -g N splits the frame into row bands (whole pixels).
// Output: the tonemapped PNG and the "_rate.png" sampling-rate image, as render_to_file writes
// them (raytraced_renderer.cpp:330-347, 690-761). The "Rendering... 100%! (Xs)" time covers the
// production kernel's render, the frame reduce and the frame read-back; bdpt_create (BVH build + upload) runs before
// the timer starts, as the reference's starts after build_accel. The report's ray / test counts
// come from a second, untimed render of the same samples by the instrumented kernel (--no-stats
// skips it).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "bdpt/bdpt.h"
#include "image_io.h"

namespace {

void usage(const char* b) {
  printf("Usage: %s [options] <scenefile>\n", b);
  printf("Program Options:\n");
  printf("  -s  <INT>        Number of camera rays per pixel\n");
  printf("  -l  <INT>        Number of samples per area light (unused by BDPT)\n");
  printf("  -t  <INT>        Number of render threads (GPU path: ignored)\n");
  printf("  -m  <INT>        Maximum ray depth\n");
  printf("  --pt             Unidirectional PathTracer instead of BDPT\n");
  printf("  -a  <INT> <FLOAT> PathTracer: samples per batch and tolerance (adaptive sampling)\n");
  printf("  -H               PathTracer: hemisphere sampling for direct lighting\n");
  printf("  -b  <FLOAT>      PathTracer: lens radius\n");
  printf("  -d  <FLOAT>      PathTracer: focal distance\n");
  printf("  -e  <PATH>       Path to environment map\n");
  printf("  --rr             Russian roulette on both subpaths\n");
  printf("  -c  <FILENAME>   Load camera settings file (Camera::dump_settings format)\n");
  printf("  -f  <FILENAME>   Image (.png) file to save output to\n");
  printf("  -r  <INT> <INT>  Width and height of output image\n");
  printf("  -p  <x> <y> <dx> <dy>  Render only this cell\n");
  printf("  -g  <INT>        Number of GPUs (default 1)\n");
  printf("  --devices <LIST> Device of each of the -g workers, comma-separated (default 0..N-1)\n");
  printf("  -S  <INT>        RNG seed (default 5489)\n");
  printf("  --dump-scene <FILE>  Write the loaded scene as JSON\n");
  printf("  --no-stats       Skip the ray / intersection-test counters of the end-of-render report\n");
  printf("  --tonemap <in.f64> <W> <H> <out.png>  Output stage only: raw float64 RGB (row 0 =\n"
         "                   bottom) -> PNG + _rate.png, as render_to_file writes them\n");
  printf("  -h               Print this help message\n");
}

int fail(const char* what) {
  fprintf(stderr, "[PathTracer] %s: %s\n", what, bdpt_last_error());
  return 1;
}

}  // namespace

int main(int argc, char** argv) {
  int spp = 1, max_depth = 1, w = 0, h = 0, gpus = 1;
  long cx = -1, cy = 0, cdx = 0, cdy = 0;
  unsigned long long seed = 5489;
  std::string out, dump, scene, envpath, cam_settings;
  std::vector<int> devices;
  bool rr = false, pt = false, hemi = false, stats = true;
  int nal = 1, batch = 32;
  float tol = 0.05f;
  double lens = 0.0, focal = 4.7;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto need = [&](int n) {
      if (i + n >= argc) { usage(argv[0]); exit(1); }
    };
    if (a == "-s") { need(1); spp = atoi(argv[++i]); }
    else if (a == "-m") { need(1); max_depth = atoi(argv[++i]); }
    else if (a == "-t") { need(1); ++i; }
    else if (a == "-l") { need(1); nal = atoi(argv[++i]); }
    else if (a == "--pt") pt = true;
    else if (a == "-a") { need(2); batch = atoi(argv[i + 1]); tol = (float)atof(argv[i + 2]); i += 2; }
    else if (a == "-H") hemi = true;
    else if (a == "-b") { need(1); lens = atof(argv[++i]); }
    else if (a == "-d") { need(1); focal = atof(argv[++i]); }
    else if (a == "-f") { need(1); out = argv[++i]; }
    else if (a == "-r") { need(2); w = atoi(argv[i + 1]); h = atoi(argv[i + 2]); i += 2; }
    else if (a == "-p") { need(4); cx = atol(argv[i + 1]); cy = atol(argv[i + 2]); cdx = atol(argv[i + 3]); cdy = atol(argv[i + 4]); i += 4; }
    else if (a == "-g") { need(1); gpus = atoi(argv[++i]); }
    else if (a == "--devices") {   // device of each -g worker (default 0..N-1), e.g. 0,0 on a one-GPU box
      need(1);
      devices.clear();
      for (const char* q = argv[++i]; *q;) {
        char* end;
        devices.push_back((int)strtol(q, &end, 10));
        if (end == q) break;
        q = *end == ',' ? end + 1 : end;
      }
    }
    else if (a == "-S") { need(1); seed = strtoull(argv[++i], nullptr, 10); }
    else if (a == "--dump-scene") { need(1); dump = argv[++i]; }
    else if (a == "-e") { need(1); envpath = argv[++i]; }
    else if (a == "--rr") rr = true;
    else if (a == "--no-stats") stats = false;
    else if (a == "--tonemap") {
      need(4);
      const int tw = atoi(argv[i + 2]), tht = atoi(argv[i + 3]);
      std::vector<double> hdr((size_t)tw * tht * 3);
      FILE* f = fopen(argv[i + 1], "rb");
      if (!f || fread(hdr.data(), sizeof(double), hdr.size(), f) != hdr.size()) {
        fprintf(stderr, "[PathTracer] cannot read %s\n", argv[i + 1]);
        return 1;
      }
      fclose(f);
      const std::string o = argv[i + 4];
      if (!bdpt::write_png(o, bdpt::tonemap(hdr.data(), tw, tht), tw, tht)) return 1;
      return bdpt::write_rate_png(o, std::vector<float>((size_t)tw * tht, 1.0f), tw, tht) ? 0 : 1;
    }
    else if (a == "-c") { need(1); cam_settings = argv[++i]; }
    else if (a == "-h" || (a.size() > 1 && a[0] == '-')) { usage(argv[0]); return 1; }
    else scene = a;
  }
  if (scene.empty() || gpus < 1) { usage(argv[0]); return 1; }
  fprintf(stderr, "[PathTracer] Input scene file: %s\n", scene.c_str());
  bdpt_dae* dae = nullptr;
  if (bdpt_dae_load(scene.c_str(), w, h, &dae) != BDPT_OK) return fail("loading scene");
  if (!dump.empty() && bdpt_dae_dump_json(dae, dump.c_str()) != BDPT_OK) return fail("dumping scene");
  if (out.empty() && dump.empty()) {
    fprintf(stderr, "[PathTracer] no -f: the interactive viewer is not part of this build\n");
    return 1;
  }
  if (out.empty()) return 0;
  if (w <= 0 || h <= 0) { w = 800; h = 600; }
  bdpt_scene_desc desc;
  bdpt_dae_get_desc(dae, &desc);
  // -c: after the -r resize, before rendering (main.cpp:172-178); the file's focal distance and lens
  // radius replace -d / -b, which set_camera gave the camera before (raytraced_renderer.cpp:141-142)
  if (!cam_settings.empty() &&
      bdpt_camera_load_settings_lens(cam_settings.c_str(), &desc.camera, &focal, &lens) != BDPT_OK)
    fprintf(stderr, "[PathTracer] %s (camera unchanged)\n", bdpt_last_error());
  bdpt_envmap env;
  float* env_rgb = nullptr;
  if (!envpath.empty()) {
    fprintf(stderr, "[PathTracer] Loading environment map %s\n", envpath.c_str());
    if (bdpt_exr_load(envpath.c_str(), &env.width, &env.height, &env_rgb) != BDPT_OK) return fail("loading environment map");
    env.rgb = env_rgb;
    desc.envmap = &env;
  }
  fprintf(stderr, "[PathTracer] %d primitives, %d materials, %d lights; %dx%d, %d spp, max depth %d, %d GPU(s)\n",
          desc.nprim, desc.nmat, desc.nlight, w, h, spp, max_depth, gpus);

  std::vector<bdpt_tile> tiles;
  if (cx >= 0) tiles.push_back(bdpt_tile{(int32_t)cx, (int32_t)cy, (int32_t)cdx, (int32_t)cdy});
  std::vector<int> rcs(gpus, 0);
  std::vector<std::string> errs(gpus);
  std::vector<bdpt_stats> st(gpus);
  std::vector<void*> ctxs(gpus, nullptr);
  std::vector<std::vector<bdpt_tile>> mine(gpus, tiles);
  std::vector<int> s0(gpus), s1(gpus);
  auto params = [&](int g, bool count) {
    bdpt_params p;
    memset(&p, 0, sizeof p);
    p.width = w; p.height = h; p.spp = spp; p.max_depth = max_depth; p.seed = seed;
    p.device = g < (int)devices.size() ? devices[g] : g;
    p.russian_roulette = rr ? 1 : 0;
    p.collect_stats = count ? 1 : 0;
    if (pt) {
      p.integrator = BDPT_INTEGRATOR_PT;
      p.ns_area_light = nal; p.samples_per_batch = batch; p.max_tolerance = tol;
      p.direct_hemisphere_sample = hemi ? 1 : 0; p.lens_radius = lens; p.focal_distance = focal;
    }
    return p;
  };
  for (int g = 0; g < gpus; g++) {
    s0[g] = (int)((long long)spp * g / gpus);
    s1[g] = (int)((long long)spp * (g + 1) / gpus);
    if (pt) {   // whole pixels: GPU g takes a band of rows (or of the -p cell)
      bdpt_tile area = tiles.empty() ? bdpt_tile{0, 0, (int32_t)w, (int32_t)h} : tiles[0];
      const int r0 = area.y0 + (int)((long long)area.h * g / gpus), r1 = area.y0 + (int)((long long)area.h * (g + 1) / gpus);
      mine[g].assign(1, bdpt_tile{area.x0, r0, area.w, r1 - r0});
      s0[g] = 0; s1[g] = r1 > r0 ? spp : 0;
    }
  }
  // one host thread per device; `phase` 0 = bdpt_create (BVH build + upload: the reference's
  // build_accel, outside its render timer, raytraced_renderer.cpp:350-374), 1 = the timed render of
  // the production kernel, 2 = the report's ray / test counters from the instrumented kernel on the
  // same samples, untimed
  auto run = [&](int phase) {
    std::vector<std::thread> th;
    for (int g = 0; g < gpus; g++) {
      th.emplace_back([&, g] {
        int rc = BDPT_OK;
        if (phase == 0) {
          bdpt_params p = params(g, false);
          rc = bdpt_create(&desc, &p, &ctxs[g]);
        } else if (phase == 1) {
          if (s1[g] > s0[g])
            rc = bdpt_render(ctxs[g], mine[g].empty() ? nullptr : mine[g].data(), (int32_t)mine[g].size(), s0[g], s1[g] - s0[g]);
        } else {
          bdpt_params p = params(g, true);
          void* sc = nullptr;
          rc = bdpt_create(&desc, &p, &sc);
          if (rc == BDPT_OK && s1[g] > s0[g])
            rc = bdpt_render(sc, mine[g].empty() ? nullptr : mine[g].data(), (int32_t)mine[g].size(), s0[g], s1[g] - s0[g]);
          if (rc == BDPT_OK) rc = bdpt_get_stats(sc, &st[g]);
          if (sc) bdpt_destroy(sc);
        }
        if (rc != BDPT_OK) errs[g] = bdpt_last_error();
        rcs[g] = rc;
      });
    }
    for (auto& t : th) t.join();
    for (int g = 0; g < gpus; g++)
      if (rcs[g] != BDPT_OK) {
        fprintf(stderr, "[PathTracer] GPU %d: %s\n", g, errs[g].c_str());
        return false;
      }
    return true;
  };
  bdpt_reducer* red = nullptr;
  auto release = [&] {   // the render contexts, before the stats pass creates its own
    bdpt_reduce_destroy(red);
    red = nullptr;
    for (void*& c : ctxs)
      if (c) { bdpt_destroy(c); c = nullptr; }
  };
  auto cleanup = [&] {
    release();
    bdpt_dae_free(dae);
    bdpt_exr_free(env_rgb);
  };
  if (!run(0)) { cleanup(); return 1; }
  // the frame reduce over the N contexts (RCCL, bdpt_reduce_*): its communicator is set up here,
  // outside the timer like the contexts; the reduce itself runs inside it. One context holds the
  // whole frame already: -g 1 needs neither RCCL nor a reduce.
  if (gpus > 1 && bdpt_reduce_create(ctxs.data(), gpus, &red) != BDPT_OK) {
    fail("creating the frame reduce");
    cleanup();
    return 1;
  }
  std::vector<float> img((size_t)w * h * 3, 0.0f);
  std::vector<int32_t> count((size_t)w * h, 0);
  auto t0 = std::chrono::steady_clock::now();
  if (!run(1)) { cleanup(); return 1; }
  // every device's partial frame summed into context 0's over xGMI, then one read-back
  if ((red && bdpt_reduce_frames(red, 0) != BDPT_OK) || bdpt_read_frame(ctxs[0], BDPT_FRAME_SAMPLE, img.data()) != BDPT_OK ||
      bdpt_read_sample_counts(ctxs[0], count.data()) != BDPT_OK) {
    fail("reducing the frames");
    cleanup();
    return 1;
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  release();
  if (stats && !run(2)) { cleanup(); return 1; }
  const double samples = (double)(tiles.empty() ? (long long)w * h : cdx * cdy) * spp;
  // the reference's end-of-render report (raytraced_renderer.cpp:679-682), on stdout: time, rays
  // traced (closest-hit walk rays + connection rays), Mrays/s, primitive tests per ray
  fprintf(stdout, "[PathTracer] Rendering... 100%%! (%.4fs)\n", secs);
  if (stats) {
    unsigned long long rays = 0, isects = 0;
    for (int g = 0; g < gpus; g++) {
      rays += st[g].rays;
      isects += st[g].tri_tests + st[g].sph_tests;
    }
    fprintf(stdout, "[PathTracer] BVH traced %llu rays.\n", rays);
    fprintf(stdout, "[PathTracer] Average speed %.4f million rays per second.\n", (double)rays / secs * 1e-6);
    fprintf(stdout, "[PathTracer] Averaged %f intersection tests per ray.\n", rays ? (double)isects / rays : 0.0);
  }
  fflush(stdout);
  fprintf(stderr, "[PathTracer] %.2f Msamples/s\n", samples / secs / 1e6);
  const std::vector<double> hdr(img.begin(), img.end());
  const std::vector<uint32_t> rgba = bdpt::tonemap(hdr.data(), w, h);
  fprintf(stderr, "[PathTracer] Saving to file: %s... ", out.c_str());
  if (tiles.empty()) {
    if (!bdpt::write_png(out, rgba, w, h)) { fprintf(stderr, "failed\n"); return 1; }
  } else {
    // the cell render saves the cell only (raytrace_cell copies the cell of the frame buffer into a
    // dx x dy buffer, save_image writes that, raytraced_renderer.cpp:622-646, 690-728); the rate
    // image below stays whole-frame, as save_sampling_rate_image reads the whole sampleCountBuffer
    const int x0 = std::max(0L, cx), y0 = std::max(0L, cy);
    const int cw = std::max(0, (int)std::min((long)w, cx + cdx) - x0), ch = std::max(0, (int)std::min((long)h, cy + cdy) - y0);
    std::vector<uint32_t> cell((size_t)cw * ch);
    for (int y = 0; y < ch; y++)
      for (int x = 0; x < cw; x++) cell[(size_t)y * cw + x] = rgba[(size_t)(y0 + y) * w + x0 + x];
    if (!bdpt::write_png(out, cell, cw, ch)) { fprintf(stderr, "failed\n"); return 1; }
  }
  fprintf(stderr, "Done!\n");
  std::vector<float> rate((size_t)w * h, 0.0f);
  if (pt) {   // sampleCountBuffer[k] * 1.0f / ns_aa (save_sampling_rate_image, raytraced_renderer.cpp:737)
    for (size_t k = 0; k < rate.size(); k++) rate[k] = count[k] * 1.0f / spp;   // summed by the reduce
  } else if (tiles.empty()) {
    std::fill(rate.begin(), rate.end(), 1.0f);   // every pixel got ns_aa samples (bidirection.cpp:539)
  } else {
    for (long y = std::max(0L, cy); y < std::min((long)h, cy + cdy); y++)
      for (long x = std::max(0L, cx); x < std::min((long)w, cx + cdx); x++) rate[(size_t)y * w + x] = 1.0f;
  }
  bdpt::write_rate_png(out, rate, w, h);
  fprintf(stdout, "[PathTracer] Job completed.\n");
  cleanup();
  return 0;
}
