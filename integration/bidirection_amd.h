// integration/bidirection_amd.h — the reference-side binding a maintainer adds to
// src/pathtracer/ to run dongmingli-Ben/bidirectional-pathtracing's BDPT loop on MI355X through
// libbdpt_amd.so (include/bdpt/bdpt.h). INTEGRATION.md walks through it.
//
// BidirectionalPathTracerAMD replaces BidirectionalPathTracer (bidirection.h:51-92) behind the
// PathTracer interface (pathtracer.h:23-104): RaytracedRenderer creates it at
// raytraced_renderer.cpp:53, calls attach() where build_accel collects the primitives
// (raytraced_renderer.cpp:350-374), its workers call raytrace_tile() per tile (:595-620) — or one
// thread renders the whole frame with raytrace_frame() — and finish() copies the frame into
// sampleBuffer before save_image. raytrace_pixel() stays available as a 1x1 tile.
//
// Flattening reads the reference's scene objects: Triangle p1..p3 / n1..n3, Sphere o / r, the
// BSDF parameters, the light fields and the camera (hFov, vFov, nClip, fClip, pos, c2w, w2c). The
// BSDF members and Camera's state are private in the reference; a maintainer gives this class read
// access (a `friend class BidirectionalPathTracerAMD;` line in Camera and each BSDF class) — the
// compile check in tests/test_integration.py builds it with the same read access the oracle's
// ref_driver uses.
//
// Threading: the reference's worker threads may call raytrace_tile concurrently; bdpt_render locks
// its context, so concurrent tiles are serialised on the GPU queue (include/bdpt/bdpt.h).
#ifndef BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H
#define BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H

#include <map>
#include <stdexcept>
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

  void raytrace_pixel(size_t x, size_t y) override {   // the reference's per-pixel entry: a 1x1 tile
    raytrace_tile((int)x, (int)y, 1, 1);
  }
  void raytrace_tile(int tx, int ty, int w, int h) {    // RaytracedRenderer::raytrace_tile's unit
    bdpt_tile t = {tx, ty, w, h};
    check(bdpt_render(ctx_, &t, 1, 0, (int32_t)ns_aa));
  }
  void raytrace_frame() { check(bdpt_render(ctx_, nullptr, 0, 0, (int32_t)ns_aa)); }
  void clear() override {
    BidirectionalPathTracer::clear();
    if (ctx_) check(bdpt_clear(ctx_));
  }
  // sampleBuffer <- the device frame (eyeBuffer + lightBuffer), before save_image
  void finish() {
    std::vector<float> rgb(sampleBuffer.w * sampleBuffer.h * 3);
    check(bdpt_read_frame(ctx_, BDPT_FRAME_SAMPLE, rgb.data()));
    for (size_t k = 0; k < sampleBuffer.w * sampleBuffer.h; k++)
      sampleBuffer.data[k] = Vector3D(rgb[3 * k], rgb[3 * k + 1], rgb[3 * k + 2]);
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

  void* ctx_ = nullptr;
  std::vector<int32_t> type_, mat_;
  std::vector<double> geom_;
  std::vector<bdpt_material> mats_;
  std::vector<bdpt_light> lights_;
  std::vector<float> env_rgb_;
};

}  // namespace CGL

#endif  // BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H
