// tests/native/core_cpu.cpp — TEST ONLY. Compiles the device-side pipeline (bdpt_core.h) and the
// host scene preparation (bdpt_scene.cpp) with g++ so the per-sample arithmetic can be checked
// against the oracle on the CPU before it runs on the GPU. Never linked into the product.
#include <cstdio>
#include <vector>

#include "bdpt_core.h"
#include "bdpt_scene.h"

using namespace bdpt;

struct HostSink {
  std::vector<double>* light;
  int W;
  void splat(int x, int y, f3 v) {
    size_t k = 3 * ((size_t)x + (size_t)y * W);
    (*light)[k] += v.x; (*light)[k + 1] += v.y; (*light)[k + 2] += v.z;
  }
};

template <int MAXV, int LM>
static int run(const HostScene& hs, int W, int H, int spp, int M, uint64_t seed, int s0, int count,
               const int* pixels, int npix, double* eye, double* light, double* stats) {
  SceneView S;
  const HostBvh& T = hs.tree(lm_width(LM));
  S.nodes = (const float4*)T.nodes.data();
  S.geom = (const float4*)hs.geom.data();
  S.shade = (const float4*)hs.shade.data();
  S.mats = hs.mats.data();
  S.lights = hs.lights.data();
  S.nlights = (int)hs.lights.size();
  S.root = T.root;
  // LM 1 reads the "LDS copy": on the CPU the same arrays (exercises the LDS-mode tree)
  S.lnodes = LM == 1 ? S.nodes : nullptr;
  S.lgeom = LM == 1 ? S.geom : nullptr;
  S.ntop = 0;
  S.cam = hs.cam;
  SampleParams sp;
  sp.W = W; sp.H = H; sp.spp = spp; sp.max_depth = M; sp.seed = seed;
  std::vector<double> lb((size_t)W * H * 3, 0.0);
  HostSink sink{&lb, W};
  Counters cnt = {0, 0, 0, 0, 0, 0};
  Paths<MAXV>* P = new Paths<MAXV>();
  float inv = 1.0f / (float)spp;
  int total = pixels ? npix : W * H;
  for (int q = 0; q < total; q++) {
    int x = pixels ? pixels[2 * q] : q % W, y = pixels ? pixels[2 * q + 1] : q / W;
    for (int s = s0; s < s0 + count; s++) {
      f3 v = render_sample<MAXV, LM>(S, sp, *P, cnt, x, y, (uint32_t)s, sink);
      size_t k = 3 * ((size_t)x + (size_t)y * W);
      eye[k] += (double)(v.x * inv); eye[k + 1] += (double)(v.y * inv); eye[k + 2] += (double)(v.z * inv);
    }
  }
  delete P;
  for (size_t k = 0; k < lb.size(); k++) light[k] += lb[k];
  if (stats) {
    stats[0] = cnt.closest + cnt.shadow; stats[1] = cnt.closest; stats[2] = cnt.shadow;
    stats[3] = cnt.nodes; stats[4] = cnt.tris; stats[5] = cnt.sphs; stats[6] = cnt.hits;
  }
  return 0;
}

template <int LM>
static int render_lm(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed, int s0,
                     int count, const int* pixels, int npix, double* eye, double* light, double* stats) {
  HostScene hs;
  std::string err;
  int rc = build_host_scene(d, hs, err);
  if (rc) { fprintf(stderr, "core_cpu: %s\n", err.c_str()); return rc; }
  int need = M < 1 ? 1 : M;
  if (need <= 5) return run<5, LM>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats);
  if (need <= 8) return run<8, LM>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats);
  if (need <= 16) return run<16, LM>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats);
  return BDPT_E_UNSUPPORTED;
}

// lds_mode 0: the HBM tree (lm_width(0) children per node); 1: the LDS-mode tree (lm_width(1))
extern "C" int core_cpu_render(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed, int s0,
                               int count, const int* pixels, int npix, double* eye, double* light, double* stats,
                               int lds_mode) {
  if (lds_mode == 1) return render_lm<1>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats);
  return render_lm<0>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats);
}

extern "C" int core_cpu_scene_info(const bdpt_scene_desc* d, int* depth, int* ref_nodes, int* prim_ref) {
  HostScene hs;
  std::string err;
  int rc = build_host_scene(d, hs, err);
  if (rc) return rc;
  *depth = hs.depth;
  *ref_nodes = hs.ref_nodes;
  for (size_t i = 0; i < hs.ref_order.size(); i++) prim_ref[i] = hs.ref_order[i];
  return 0;
}
