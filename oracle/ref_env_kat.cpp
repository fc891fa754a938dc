// oracle/ref_env_kat.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Known-answer dump of the reference's own environment-light code, built from its sources where
// they lie under /root/reference (oracle/ref.mk -> oracle/_ref/ref_env_kat):
//   * load_exr (src/application/main.cpp:40-77, restated here because main.cpp holds main();
//     it drives the reference's vendored tinyexr, CGL/include/CGL/tinyexr.h) -> the decoded
//     HDRImageBuffer,
//   * EnvironmentLight::init (environment_light.cpp:18-62) -> pdf_envmap, marginal_y, conds_y,
//   * the first N EnvironmentLight::sample_L calls of a fresh process (:126-156) -> wi, pdf, L,
//   * EnvironmentLight::sample_dir (:159-168) for M directions given on the command line file.
// usage: ref_env_kat map.exr N dirs.txt out.json   (run in a scratch directory: init() writes
//        probability_debug.png into the working directory, environment_light.cpp:57-59)
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define TINYEXR_IMPLEMENTATION
#include "CGL/tinyexr.h"

#define private public
#define protected public
#include "CGL/CGL.h"
#include "util/image.h"
#include "scene/environment_light.h"
#undef private
#undef protected

using namespace CGL;

// main.cpp:40-77
static HDRImageBuffer* load_exr(const char* file_path) {
  const char* err;
  EXRImage exr;
  InitEXRImage(&exr);
  int ret = ParseMultiChannelEXRHeaderFromFile(&exr, file_path, &err);
  if (ret != 0) { fprintf(stderr, "exr header: %s\n", err); return nullptr; }
  for (int i = 0; i < exr.num_channels; i++)
    if (exr.pixel_types[i] == TINYEXR_PIXELTYPE_HALF) exr.requested_pixel_types[i] = TINYEXR_PIXELTYPE_FLOAT;
  ret = LoadMultiChannelEXRFromFile(&exr, file_path, &err);
  if (ret != 0) { fprintf(stderr, "exr load: %s\n", err); return nullptr; }
  HDRImageBuffer* envmap = new HDRImageBuffer();
  envmap->resize(exr.width, exr.height);
  float* channel_r = (float*)exr.images[2];
  float* channel_g = (float*)exr.images[1];
  float* channel_b = (float*)exr.images[0];
  for (size_t i = 0; i < (size_t)exr.width * exr.height; i++)
    envmap->data[i] = Vector3D(channel_r[i], channel_g[i], channel_b[i]);
  return envmap;
}

static void arr(FILE* f, const char* name, const double* v, size_t n, bool last = false) {
  fprintf(f, "\"%s\": [", name);
  for (size_t i = 0; i < n; i++) fprintf(f, "%s%.17g", i ? ", " : "", v[i]);
  fprintf(f, "]%s\n", last ? "" : ",");
}

int main(int argc, char** argv) {
  if (argc < 5) { fprintf(stderr, "usage: %s map.exr N dirs.txt out.json\n", argv[0]); return 1; }
  HDRImageBuffer* env = load_exr(argv[1]);
  if (!env) return 2;
  const int n = atoi(argv[2]);
  std::vector<double> dirs;
  if (FILE* fd = fopen(argv[3], "r")) {
    double v;
    while (fscanf(fd, "%lf", &v) == 1) dirs.push_back(v);
    fclose(fd);
  }
  SceneObjects::EnvironmentLight L(env);
  const size_t w = env->w, h = env->h, np = w * h;
  FILE* f = fopen(argv[4], "w");
  if (!f) return 3;
  fprintf(f, "{\"width\": %zu, \"height\": %zu,\n", w, h);
  std::vector<double> rgb(3 * np);
  for (size_t i = 0; i < np; i++)
    for (int c = 0; c < 3; c++) rgb[3 * i + c] = env->data[i][c];
  arr(f, "rgb", rgb.data(), rgb.size());
  arr(f, "pdf_envmap", L.pdf_envmap, np);
  arr(f, "marginal_y", L.marginal_y, h);
  arr(f, "conds_y", L.conds_y, np);
  std::vector<double> wi(3 * n), pdf(n), rad(3 * n);
  for (int k = 0; k < n; k++) {
    Vector3D d;
    double dist, p;
    Vector3D r = L.sample_L(Vector3D(0, 0, 0), &d, &dist, &p);
    for (int c = 0; c < 3; c++) { wi[3 * k + c] = d[c]; rad[3 * k + c] = r[c]; }
    pdf[k] = p;
  }
  arr(f, "sample_wi", wi.data(), wi.size());
  arr(f, "sample_pdf", pdf.data(), pdf.size());
  arr(f, "sample_L", rad.data(), rad.size());
  const size_t m = dirs.size() / 3;
  std::vector<double> look(3 * m);
  for (size_t k = 0; k < m; k++) {
    Ray r(Vector3D(0, 0, 0), Vector3D(dirs[3 * k], dirs[3 * k + 1], dirs[3 * k + 2]));
    Vector3D v = L.sample_dir(r);
    for (int c = 0; c < 3; c++) look[3 * k + c] = v[c];
  }
  arr(f, "dirs", dirs.data(), dirs.size());
  arr(f, "sample_dir", look.data(), look.size(), true);
  fprintf(f, "}\n");
  fclose(f);
  return 0;
}
