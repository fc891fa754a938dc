// integration/bidirection_amd.h — the reference-side binding a maintainer adds to
// src/pathtracer/ to run dongmingli-Ben/bidirectional-pathtracing's BDPT loop on MI355X through
// libbdpt_amd.so (include/bdpt/bdpt.h). INTEGRATION.md walks through it.
//
// BidirectionalPathTracerAMD replaces BidirectionalPathTracer (bidirection.h:51-92) behind the
// PathTracer interface (pathtracer.h:23-104). The one change to the reference is the class the
// renderer constructs (raytraced_renderer.cpp:53):
//     -  pt = new BidirectionalPathTracer();
//     +  pt = new BidirectionalPathTracerAMD();
// Everything else — render_to_file, start_raytracing, the worker threads' raytrace_tile loop of
// raytrace_pixel calls, write_to_framebuffer after every tile, save_image — runs unmodified:
//   * start_raytracing calls clear() and set_frame_size(), then sets bvh / camera / scene
//     (:280-285); the first raytrace_pixel() of the frame attaches the scene (bdpt_create over
//     scene->objects' primitives in build_accel's collection order, scene->lights, *camera and
//     envLight's map);
//   * the workers call raytrace_pixel() per pixel of a 32x32 tile, row-major (:293-298, 610-615):
//     the tile's first pixel renders the whole tile with ONE bdpt_render and copies the tile's
//     pixels of the device frame into sampleBuffer (and sampleCountBuffer = ns_aa, as
//     bidirection.cpp:539), the others are no-ops, so the write_to_framebuffer after the tile
//     (:619, non-virtual, pathtracer.cpp:42-45) shows it;
//   * when the last pixel of the frame has been rendered the whole frame — light-tracing splats
//     land anywhere (bidirection.cpp:457-466) — goes to sampleBuffer / eyeBuffer / lightBuffer,
//     so the last write_to_framebuffer and save_image see the final image.
// A pixel that no 32x32 tile covers (the -p cell path, 8x8 tiles at an arbitrary corner) is a 1x1
// tile. attach() / raytrace_tile() / raytrace_frame() / finish() remain for callers that drive
// whole tiles or frames themselves.
//
// Flattening reads the reference's scene objects: Triangle p1..p3 / n1..n3, Sphere o / r, the
// BSDF parameters, the light fields and the camera (hFov, vFov, nClip, fClip, pos, c2w, w2c). The
// BSDF members and Camera's state are private in the reference; a maintainer gives this class read
// access (a `friend class BidirectionalPathTracerAMD;` line in Camera and each BSDF class) — the
// compile check in tests/test_integration.py builds it with the same read access the oracle's
// ref_driver uses.
//
// Threading: the reference's worker threads call raytrace_pixel concurrently (on disjoint tiles);
// the binding's tile bookkeeping is under a mutex, and bdpt_render serialises launches per context.
#ifndef BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H
#define BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "bdpt/bdpt.h"
#include "pathtracer/bidirection.h"
#include "pathtracer/bsdf.h"
#include "pathtracer/camera.h"
#include "scene/environment_light.h"
#include "scene/light.h"
#include "scene/sphere.h"
#include "scene/triangle.h"

namespace CGL {

class BidirectionalPathTracerAMD : public BidirectionalPathTracer {
 public:
  // bdpt_create over the scene the reference's build_accel sees (primitives in its collection
  // order — the tie-break key of equal-t hits is their position in the reference BVH's leaf order,
  // which bdpt_create rebuilds from this order), its lights, camera and optional -e envmap.
  // Returns the BDPT_* status; bdpt_last_error() has the text.
  int attach(const std::vector<SceneObjects::Primitive*>& prims,
             const std::vector<SceneObjects::SceneLight*>& lights, const Camera& cam,
             const HDRImageBuffer* envmap = nullptr, uint64_t seed = 5489) {
    type_.clear(); geom_.clear(); mat_.clear(); mats_.clear(); lights_.clear();
    std::map<const BSDF*, int32_t> mat_index;
    for (const SceneObjects::Primitive* p : prims) {
      double g[18] = {0};
      if (auto* t = dynamic_cast<const SceneObjects::Triangle*>(p)) {
        const Vector3D* v[6] = {&t->p1, &t->p2, &t->p3, &t->n1, &t->n2, &t->n3};
        for (int k = 0; k < 6; k++)
          for (int c = 0; c < 3; c++) g[3 * k + c] = (*v[k])[c];
        type_.push_back(BDPT_PRIM_TRIANGLE);
      } else if (auto* s = dynamic_cast<const SceneObjects::Sphere*>(p)) {
        for (int c = 0; c < 3; c++) g[c] = s->o[c];
        g[3] = s->r;
        type_.push_back(BDPT_PRIM_SPHERE);
      } else {
        return fail("unsupported primitive type");
      }
      geom_.insert(geom_.end(), g, g + 18);
      const BSDF* b = p->get_bsdf();
      auto it = mat_index.find(b);
      if (it == mat_index.end()) {
        it = mat_index.emplace(b, (int32_t)mats_.size()).first;
        mats_.push_back(material(b));
      }
      mat_.push_back(it->second);
    }
    for (const SceneObjects::SceneLight* l : lights) {
      bdpt_light d = {};
      if (auto* a = dynamic_cast<const SceneObjects::AreaLight*>(l)) {
        d.type = BDPT_LIGHT_AREA;
        copy3(d.radiance, a->radiance); copy3(d.position, a->position); copy3(d.direction, a->direction);
        copy3(d.dim_x, a->dim_x); copy3(d.dim_y, a->dim_y);
        d.area = a->area;
      } else if (auto* pl = dynamic_cast<const SceneObjects::PointLight*>(l)) {
        d.type = BDPT_LIGHT_POINT;
        copy3(d.radiance, pl->radiance); copy3(d.position, pl->position);
      } else if (dynamic_cast<const SceneObjects::EnvironmentLight*>(l)) {
        continue;   // comes in through desc.envmap (raytraced_renderer.cpp:117-119 appends it last)
      } else {
        d.type = BDPT_LIGHT_OTHER;   // bdpt_create rejects it under BDPT, as the reference asserts
      }
      lights_.push_back(d);
    }
    bdpt_scene_desc desc = {};
    desc.nprim = (int32_t)type_.size();
    desc.prim_type = type_.data();
    desc.prim_geom = geom_.data();
    desc.prim_mat = mat_.data();
    desc.nmat = (int32_t)mats_.size();
    desc.mats = mats_.data();
    desc.nlight = (int32_t)lights_.size();
    desc.lights = lights_.data();
    desc.camera = camera_desc(cam);
    bdpt_envmap env = {};
    if (envmap) {   // HDRImageBuffer data[w * j + i] as float RGB (main.cpp:40-77 layout)
      env_rgb_.resize(envmap->w * envmap->h * 3);
      for (size_t k = 0; k < envmap->w * envmap->h; k++)
        for (int c = 0; c < 3; c++) env_rgb_[3 * k + c] = (float)envmap->data[k][c];
      env.width = (int32_t)envmap->w;
      env.height = (int32_t)envmap->h;
      env.rgb = env_rgb_.data();
      desc.envmap = &env;
    }
    bdpt_params p = {};
    p.width = (int32_t)sampleBuffer.w;
    p.height = (int32_t)sampleBuffer.h;
    p.spp = (int32_t)ns_aa;
    p.max_depth = (int32_t)max_ray_depth;
    p.seed = seed;
    if (ctx_) { bdpt_destroy(ctx_); ctx_ = nullptr; }
    return bdpt_create(&desc, &p, &ctx_);
  }

  // ---- the PathTracer contract, driven by the reference's unmodified RaytracedRenderer ----
  void set_frame_size(size_t width, size_t height) override {
    BidirectionalPathTracer::set_frame_size(width, height);
    drop_frame();
  }
  // The renderer's per-pixel call (raytraced_renderer.cpp:610-615; bidirection.cpp:503-542). It
  // runs on the renderer's worker threads, where an exception would end the process, so a failure
  // (no device, bdpt_* error) is recorded — error() — and the frame's remaining pixels are skipped.
  void raytrace_pixel(size_t x, size_t y) override {
    const size_t W = sampleBuffer.w, H = sampleBuffer.h;
    if (x >= W || y >= H || failed_.load(std::memory_order_acquire)) return;
    if (done_ && done_[x + y * W].load(std::memory_order_acquire)) return;   // rendered with its tile
    std::lock_guard<std::mutex> lk(mu_);
    if (failed_.load(std::memory_order_relaxed)) return;
    try {
      render_pixel_locked(x, y, W, H);
    } catch (const std::exception& e) {
      err_ = e.what();
      failed_.store(true, std::memory_order_release);
    }
  }
  // empty, or the first failure of the frame's raytrace_pixel calls
  std::string error() const { return failed_.load() ? err_ : std::string(); }
  size_t launches() const { return launches_; }   // bdpt_render calls since the last frame reset

 private:
  void render_pixel_locked(size_t x, size_t y, size_t W, size_t H) {
    if (!ctx_) {
      if (!scene || !camera) throw std::runtime_error("BidirectionalPathTracerAMD: no scene / camera");
      std::vector<SceneObjects::Primitive*> prims;   // build_accel's collection order (:352-360)
      for (SceneObjects::SceneObject* obj : scene->objects) {
        const std::vector<SceneObjects::Primitive*>& op = obj->get_primitives();
        prims.insert(prims.end(), op.begin(), op.end());
      }
      const HDRImageBuffer* env = envLight ? static_cast<const SceneObjects::EnvironmentLight*>(envLight)->envMap : nullptr;
      check(attach(prims, scene->lights, *camera, env));
    }
    if (!done_) {
      done_.reset(new std::atomic<uint8_t>[W * H]);
      for (size_t k = 0; k < W * H; k++) done_[k].store(0, std::memory_order_relaxed);
      rendered_ = 0;
    }
    if (done_[x + y * W].load(std::memory_order_relaxed)) return;
    // the tile whose first pixel this is (tiles start at multiples of imageTileSize = 32,
    // raytraced_renderer.cpp:83,293-298), else this pixel alone
    const bool corner = x % kTile == 0 && y % kTile == 0;
    const size_t tw = corner ? std::min(kTile, W - x) : 1, th = corner ? std::min(kTile, H - y) : 1;
    raytrace_tile((int)x, (int)y, (int)tw, (int)th);
    for (size_t yy = y; yy < y + th; yy++)
      for (size_t xx = x; xx < x + tw; xx++) {
        sampleCountBuffer[xx + yy * W] = ns_aa;   // bidirection.cpp:539
        if (!done_[xx + yy * W].exchange(1, std::memory_order_release)) rendered_++;
      }
    if (rendered_ == W * H) {
      finish();   // the frame is complete: every splat is in, sampleBuffer <- the whole image
    } else {
      std::vector<float> rgb(tw * th * 3);
      check(bdpt_read_frame_rect(ctx_, BDPT_FRAME_SAMPLE, (int32_t)x, (int32_t)y, (int32_t)tw, (int32_t)th, rgb.data()));
      for (size_t yy = 0; yy < th; yy++)
        for (size_t xx = 0; xx < tw; xx++) {
          const float* v = &rgb[3 * (xx + yy * tw)];
          sampleBuffer.data[(x + xx) + (y + yy) * W] = Vector3D(v[0], v[1], v[2]);
        }
    }
  }

 public:
  void raytrace_tile(int tx, int ty, int w, int h) {    // RaytracedRenderer::raytrace_tile's unit
    bdpt_tile t = {tx, ty, w, h};
    check(bdpt_render(ctx_, &t, 1, 0, (int32_t)ns_aa));
    launches_++;
  }
  void raytrace_frame() {
    check(bdpt_render(ctx_, nullptr, 0, 0, (int32_t)ns_aa));
    launches_++;
  }
  // start_raytracing (:280) clears before every frame: the next raytrace_pixel attaches again
  void clear() override {
    BidirectionalPathTracer::clear();
    drop_frame();
  }
  // sampleBuffer / eyeBuffer / lightBuffer <- the device frames, before save_image
  void finish() {
    const size_t n = sampleBuffer.w * sampleBuffer.h;
    std::vector<float> rgb(n * 3);
    HDRImageBuffer* dst[3] = {&sampleBuffer, &eyeBuffer, &lightBuffer};
    const int32_t which[3] = {BDPT_FRAME_SAMPLE, BDPT_FRAME_EYE, BDPT_FRAME_LIGHT};
    for (int b = 0; b < 3; b++) {
      if (dst[b]->w * dst[b]->h != n) continue;
      check(bdpt_read_frame(ctx_, which[b], rgb.data()));
      for (size_t k = 0; k < n; k++) dst[b]->data[k] = Vector3D(rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]);
    }
  }
  ~BidirectionalPathTracerAMD() {
    if (ctx_) bdpt_destroy(ctx_);
  }

 private:
  static void copy3(double* d, const Vector3D& v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }
  static void check(int rc) {
    if (rc != BDPT_OK) throw std::runtime_error(bdpt_last_error());
  }
  static int fail(const char*) { return BDPT_E_UNSUPPORTED; }
  static bdpt_material material(const BSDF* b) {   // bsdf.h:132-304
    bdpt_material m = {};
    if (auto* d = dynamic_cast<const DiffuseBSDF*>(b)) {
      m.type = BDPT_MAT_DIFFUSE; copy3(m.a, d->reflectance);
    } else if (auto* e = dynamic_cast<const EmissionBSDF*>(b)) {
      m.type = BDPT_MAT_EMISSION; copy3(m.a, e->radiance);
    } else if (auto* mi = dynamic_cast<const MirrorBSDF*>(b)) {
      m.type = BDPT_MAT_MIRROR; copy3(m.a, mi->reflectance);
    } else if (auto* g = dynamic_cast<const GlassBSDF*>(b)) {
      m.type = BDPT_MAT_GLASS; copy3(m.a, g->reflectance); copy3(m.b, g->transmittance);
      m.ior = g->ior; m.roughness = g->roughness;
    } else if (auto* r = dynamic_cast<const RefractionBSDF*>(b)) {
      m.type = BDPT_MAT_REFRACTION; copy3(m.b, r->transmittance);
      m.ior = r->ior; m.roughness = r->roughness;
    } else {
      m.type = BDPT_MAT_MICROFACET;   // rejected by bdpt_create under BDPT (sample_pdf asserts)
    }
    return m;
  }
  void drop_frame() {   // a new frame (size / scene / camera may have changed): attach again
    std::lock_guard<std::mutex> lk(mu_);
    if (ctx_) { bdpt_destroy(ctx_); ctx_ = nullptr; }
    done_.reset();
    rendered_ = 0;
    launches_ = 0;
    failed_.store(false);
    err_.clear();
  }
  static bdpt_camera camera_desc(const Camera& c) {   // camera.h:104-125
    bdpt_camera d = {};
    copy3(d.pos, c.pos);
    for (int col = 0; col < 3; col++)
      for (int row = 0; row < 3; row++) {
        d.c2w[3 * col + row] = c.c2w(row, col);
        d.w2c[3 * col + row] = c.w2c(row, col);
      }
    d.hfov_deg = c.hFov;
    d.vfov_deg = c.vFov;
    d.nclip = c.nClip;
    d.fclip = c.fClip;
    return d;
  }

  static constexpr size_t kTile = 32;   // RaytracedRenderer::imageTileSize (raytraced_renderer.cpp:83)
  void* ctx_ = nullptr;
  std::mutex mu_;
  std::unique_ptr<std::atomic<uint8_t>[]> done_;   // per pixel: rendered with its tile
  size_t rendered_ = 0, launches_ = 0;
  std::atomic<bool> failed_{false};
  std::string err_;
  std::vector<int32_t> type_, mat_;
  std::vector<double> geom_;
  std::vector<bdpt_material> mats_;
  std::vector<bdpt_light> lights_;
  std::vector<float> env_rgb_;
};

}  // namespace CGL

#endif  // BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H
