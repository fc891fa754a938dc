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

template <int MAXV, int LM, bool EXT>
static int run(const HostScene& hs, int W, int H, int spp, int M, uint64_t seed, int s0, int count,
               const int* pixels, int npix, double* eye, double* light, double* stats, int rr) {
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
  // LM 2 reads its BFS treelet [0, n_top) from the "LDS copy" (the same array on the CPU)
  S.lnodes = LM == 1 || LM == 2 ? S.nodes : nullptr;
  S.lgeom = LM == 1 || LM == 3 ? S.geom : nullptr;
  S.lshade = LM == 3 ? S.shade : nullptr;
  S.lleaves = hs.leaf_refs.data();
  S.nleaves = (int)hs.leaf_refs.size();
  S.fn = flat_prims(hs, &S.fsph);
  S.ntop = LM == 2 ? T.n_top : 0;
  S.lstack = nullptr;
  S.cam = hs.cam;
  const size_t np = (size_t)hs.env_w * hs.env_h;
  S.env.light = hs.env_light;
  S.env.w = hs.env_w;
  S.env.h = hs.env_h;
  S.env.marg = hs.env.data();
  S.env.cond = hs.env.data() + hs.env_h;
  S.env.pdf = hs.env.data() + hs.env_h + np;
  S.env.rgb = hs.env.data() + hs.env_h + 2 * np;
  S.env.gmarg = hs.env.empty() ? nullptr : (const int*)(hs.env.data() + hs.env_h + 5 * np);
  S.env.gcond = hs.env.empty() ? nullptr : S.env.gmarg + hs.env_gm + 1;
  S.env.gm = hs.env_gm;
  S.env.gc = hs.env_gc;
  S.env.cx = hs.env_c[0]; S.env.cy = hs.env_c[1]; S.env.cz = hs.env_c[2];
  S.env.rad = hs.env_rad;
  SampleParams sp;
  sp.W = W; sp.H = H; sp.spp = spp; sp.max_depth = M; sp.seed = seed;
  sp.rr = rr;
  std::vector<double> lb((size_t)W * H * 3, 0.0);
  HostSink sink{&lb, W};
  Counters cnt = {0, 0, 0, 0, 0, 0};
  Paths<MAXV>* P = new Paths<MAXV>();
  float inv = 1.0f / (float)spp;
  int total = pixels ? npix : W * H;
  for (int q = 0; q < total; q++) {
    int x = pixels ? pixels[2 * q] : q % W, y = pixels ? pixels[2 * q + 1] : q / W;
    for (int s = s0; s < s0 + count; s++) {
      f3 v = render_sample<MAXV, LM, EXT>(S, sp, *P, cnt, x, y, (uint32_t)s, sink);
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

template <int LM, bool EXT>
static int render_maxv(const HostScene& hs, int W, int H, int spp, int M, uint64_t seed, int s0, int count,
                       const int* pixels, int npix, double* eye, double* light, double* stats, int rr) {
  int need = M < 1 ? 1 : M;
  if (need <= 5) return run<5, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (need <= 8) return run<8, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (need <= 16) return run<16, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (need <= 32) return run<32, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (need <= 62) return run<62, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (need <= 126) return run<126, LM, EXT>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  return BDPT_E_UNSUPPORTED;
}

template <int LM>
static int render_lm(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed, int s0,
                     int count, const int* pixels, int npix, double* eye, double* light, double* stats, int rr) {
  HostScene hs;
  std::string err;
  int rc = build_host_scene(d, hs, err);
  if (rc) { fprintf(stderr, "core_cpu: %s\n", err.c_str()); return rc; }
  // the kernel selection of bdpt_create: EXT kernels for an environment light or roulette
  if (hs.env_light >= 0 || rr)
    return render_maxv<LM, true>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  return render_maxv<LM, false>(hs, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
}

// lds_mode 0: the HBM tree (lm_width(0) children per node); 1: the LDS-mode tree (lm_width(1));
// 2: the HBM tree with its BFS treelet read through the LDS path (same array on the CPU); 3: flat list
extern "C" int core_cpu_render(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed, int s0,
                               int count, const int* pixels, int npix, double* eye, double* light, double* stats,
                               int lds_mode, int rr) {
  if (lds_mode == 1) return render_lm<1>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (lds_mode == 2) return render_lm<2>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  if (lds_mode == 3) return render_lm<3>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
  return render_lm<0>(d, W, H, spp, M, seed, s0, count, pixels, npix, eye, light, stats, rr);
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

// The unidirectional PathTracer (bdpt_core.h pt_pixel) for the whole frame: image = W*H*3
// (sampleBuffer), counts = W*H (sampleCountBuffer).
// LDS mode 3's flat primitive run (flat_prims): its length, or 0 when the leaves are not one run
extern "C" int core_cpu_flat_prims(const bdpt_scene_desc* d, uint32_t* sph_mask) {
  HostScene hs;
  std::string err;
  if (build_host_scene(d, hs, err) != BDPT_OK) return -1;
  return flat_prims(hs, sph_mask);
}

extern "C" int core_cpu_pt_render(const bdpt_scene_desc* d, int W, int H, int spp, int M, uint64_t seed,
                                  int ns_area_light, int batch, float tol, int hemisphere, double lens,
                                  double focal, double* image, int* counts) {
  HostScene hs;
  std::string err;
  int rc = build_host_scene(d, hs, err, true);
  if (rc) { fprintf(stderr, "core_cpu: %s\n", err.c_str()); return rc; }
  SceneView S;
  const HostBvh& T = hs.tree(lm_width(0));
  S.nodes = (const float4*)T.nodes.data();
  S.geom = (const float4*)hs.geom.data();
  S.shade = (const float4*)hs.shade.data();
  S.mats = hs.mats.data();
  S.lights = hs.lights.data();
  S.nlights = (int)hs.lights.size();
  S.root = T.root;
  S.lnodes = nullptr;
  S.lgeom = nullptr;
  S.lshade = nullptr;
  S.lleaves = nullptr;
  S.nleaves = 0;
  S.fn = 0;
  S.fsph = 0;
  S.ntop = 0;
  S.lstack = nullptr;
  S.cam = hs.cam;
  const size_t np = (size_t)hs.env_w * hs.env_h;
  S.env.light = hs.env_light;
  S.env.w = hs.env_w;
  S.env.h = hs.env_h;
  S.env.marg = hs.env.data();
  S.env.cond = hs.env.data() + hs.env_h;
  S.env.pdf = hs.env.data() + hs.env_h + np;
  S.env.rgb = hs.env.data() + hs.env_h + 2 * np;
  S.env.gmarg = hs.env.empty() ? nullptr : (const int*)(hs.env.data() + hs.env_h + 5 * np);
  S.env.gcond = hs.env.empty() ? nullptr : S.env.gmarg + hs.env_gm + 1;
  S.env.gm = hs.env_gm;
  S.env.gc = hs.env_gc;
  S.env.cx = hs.env_c[0]; S.env.cy = hs.env_c[1]; S.env.cz = hs.env_c[2];
  S.env.rad = hs.env_rad;
  PtParams pp;
  pp.W = W; pp.H = H; pp.spp = spp; pp.max_depth = M; pp.seed = seed;
  pp.ns_area_light = ns_area_light; pp.batch = batch; pp.hemisphere = hemisphere; pp.tol = tol;
  pp.lens_radius = (float)lens; pp.focal_distance = (float)focal;
  Counters cnt = {0, 0, 0, 0, 0, 0};
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const size_t k = (size_t)x + (size_t)y * W;
      const f3 v = pt_pixel<0>(S, pp, cnt, x, y, counts + k);
      image[3 * k] = v.x; image[3 * k + 1] = v.y; image[3 * k + 2] = v.z;
    }
  return 0;
}

// the device tree's depth and node count (binary tree before the 4-wide collapse), as built under
// the current BDPT_BVH / BDPT_SAH_* settings
extern "C" int core_cpu_dev_tree(const bdpt_scene_desc* d, int* depth, int* nodes) {
  HostScene hs;
  std::string err;
  int rc = build_host_scene(d, hs, err);
  if (rc) return rc;
  *depth = hs.dev_depth;
  *nodes = hs.dev_nodes;
  return 0;
}

// Closest hits of the device traversal (lds_mode 0, 1 or 2) against a brute-force loop over every
// primitive with the same tests and tie rule, for n rays with origins spread over the scene's box and
// directions with exact zero (and -0) components: axis-aligned and in the coordinate planes (a zero
// component once gave an infinite inverse and NaN / -inf plane distances, bdpt_core.h safe_inv).
// Returns the number of rays whose hit (primitive, t) differs; *hits = rays that hit something.
template <int LM>
static SceneView trace_view(const HostScene& hs) {
  SceneView S = {};
  const HostBvh& T = hs.tree(lm_width(LM));
  S.nodes = (const float4*)T.nodes.data();
  S.geom = (const float4*)hs.geom.data();
  S.shade = (const float4*)hs.shade.data();
  S.root = T.root;
  S.lnodes = LM == 1 || LM == 2 ? S.nodes : nullptr;
  S.lgeom = LM == 1 ? S.geom : nullptr;
  S.ntop = LM == 2 ? T.n_top : 0;
  return S;
}

template <int LM>
static int trace_check_lm(const HostScene& hs, int n, uint64_t seed, int* hits) {
  const SceneView S = trace_view<LM>(hs);
  const int np = (int)(hs.geom.size() / 12);
  float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
  for (int i = 0; i < np; i++) {
    const float* g = &hs.geom[12 * i];
    const bool sph = __float_as_int(hs.shade[12 * i + 10]) != 0;
    for (int v = 0; v < (sph ? 1 : 3); v++)
      for (int k = 0; k < 3; k++) {
        const float e = v == 0 ? 0.0f : (v == 1 ? g[3 + k] : g[6 + k]);
        const float x = g[k] + e;
        lo[k] = fminf(lo[k], x); hi[k] = fmaxf(hi[k], x);
      }
  }
  uint64_t st = seed;
  auto rnd = [&]() { st = st * 6364136223846793005ull + 1442695040888963407ull; return (float)((st >> 40) & 0xffffff) / 16777216.0f; };
  int bad = 0;
  *hits = 0;
  Counters cnt = {};
  for (int q = 0; q < n; q++) {
    f3 o = mk3(lo[0] + (hi[0] - lo[0]) * rnd(), lo[1] + (hi[1] - lo[1]) * rnd(), lo[2] + (hi[2] - lo[2]) * rnd());
    float dv[3] = {rnd() * 2 - 1, rnd() * 2 - 1, rnd() * 2 - 1};
    const int pat = q % 7;   // which components are zeroed: one axis (3), two axes (3), none
    if (pat < 3) dv[pat] = (q & 8) ? -0.0f : 0.0f;
    else if (pat < 6) { dv[(pat + 1) % 3] = 0.0f; dv[(pat + 2) % 3] = (q & 8) ? -0.0f : 0.0f; }
    f3 d = normalize(mk3(dv[0], dv[1], dv[2]));
    if (!(norm2(d) > 0.5f)) continue;
    Hit h;
    trace_closest<LM, kWalkStack>(S, o, d, 1e-5f, 1e30f, h, cnt);
    float bt = 1e30f;
    int bp = -1, bk = -1;
    for (int i = 0; i < np; i++) {
      const float4* g = S.geom + 3 * i;
      float t, b1, b2;
      bool ok;
      int key;
      if (__float_as_int(hs.shade[12 * i + 10]) != 0) {
        ok = sph_test(g[0], o, d, 1e-5f, bt, &t);
        key = __float_as_int(g[1].x);
      } else {
        ok = tri_test(g[0], g[1], g[2], o, d, 1e-5f, bt, &t, &b1, &b2);
        key = __float_as_int(g[2].y);
      }
      if (ok && (t < bt || key > bk)) { bt = t; bp = i; bk = key; }
    }
    if (bp >= 0) (*hits)++;
    // compared as scene primitives: a primitive that spatial splits reference from two leaves has a
    // record at two positions, and either may be the one a walk or the loop meets first
    const int sp = bp >= 0 ? hs.prim_ref[bp] : -1, hp = h.prim >= 0 ? hs.prim_ref[h.prim] : -1;
    if (sp != hp || (bp >= 0 && bt != h.t)) bad++;
  }
  return bad;
}

extern "C" int core_cpu_trace_check(const bdpt_scene_desc* d, int lds_mode, int n, uint64_t seed, int* hits) {
  HostScene hs;
  std::string err;
  if (build_host_scene(d, hs, err) != BDPT_OK) return -1;
  if (lds_mode == 1) return trace_check_lm<1>(hs, n, seed, hits);
  return lds_mode == 2 ? trace_check_lm<2>(hs, n, seed, hits) : trace_check_lm<0>(hs, n, seed, hits);
}

// bdpt_trace_rays (k_trace_rays) on the CPU: rays = n x (o, d, tmin, tmax); closest hit t and the
// primitive's scene index (-1: none), or for any_hit whether anything lies in [tmin, tmax]
template <int LM>
static void trace_rays_lm(const HostScene& hs, const float* rays, int n, int any_hit, float* out_t, int* out_prim) {
  const SceneView S = trace_view<LM>(hs);
  Counters c = {};
  for (int i = 0; i < n; i++) {
    const float* r = rays + 8 * (size_t)i;
    const f3 o = mk3(r[0], r[1], r[2]), d = mk3(r[3], r[4], r[5]);
    if (any_hit) {
      const bool h = trace_any<LM, kConnStack>(S, o, d, r[6], r[7], c);
      out_t[i] = h ? 0.0f : INFINITY;
      out_prim[i] = h ? 0 : -1;
    } else {
      Hit h;
      const bool ok = trace_closest<LM, kWalkStack>(S, o, d, r[6], r[7], h, c);
      out_t[i] = ok ? h.t : INFINITY;
      out_prim[i] = ok ? hs.prim_ref[h.prim] : -1;
    }
  }
}

extern "C" int core_cpu_trace_rays(const bdpt_scene_desc* d, int lds_mode, const float* rays, int n, int any_hit,
                                   float* out_t, int* out_prim) {
  HostScene hs;
  std::string err;
  if (build_host_scene(d, hs, err) != BDPT_OK) return -1;
  if (lds_mode == 1) trace_rays_lm<1>(hs, rays, n, any_hit, out_t, out_prim);
  else if (lds_mode == 2) trace_rays_lm<2>(hs, rays, n, any_hit, out_t, out_prim);
  else trace_rays_lm<0>(hs, rays, n, any_hit, out_t, out_prim);
  return 0;
}

#if defined(BDPT_STEP_HIST)
// diagnostics (tools/anyhit_probe.py): collect the any-hit rays of the following renders (max_rays,
// 0 = stop), then copy up to max_rays of them out; returns the number collected
static std::vector<float> g_rays;
extern "C" void core_cpu_ray_dump(int on) {
  g_rays.clear();
  ray_dump() = on == 1 ? &g_rays : nullptr;          // 1: any-hit queries
  ray_dump_closest() = on == 2 ? &g_rays : nullptr;  // 2: closest-hit queries
}
extern "C" long long core_cpu_ray_dump_get(float* out, long long max_rays) {
  const long long n = std::min<long long>(max_rays, (long long)g_rays.size() / 8);
  std::copy(g_rays.begin(), g_rays.begin() + 8 * n, out);
  return (long long)g_rays.size() / 8;
}
// diagnostics (tools/step_hist.py): node steps per closest-hit query since the last call
extern "C" void core_cpu_step_hist(unsigned long long* out1024) {
  for (int k = 0; k < 1024; k++) { out1024[k] = step_hist()[k]; step_hist()[k] = 0; }
}
#endif
