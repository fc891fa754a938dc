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
//   * start_raytracing calls clear() and set_frame_size() on its own thread, then sets bvh /
//     camera / scene (:280-285); the first raytrace_pixel() of the frame attaches the scene
//     (bdpt_create over scene->objects' primitives in build_accel's collection order,
//     scene->lights, *camera and envLight's map);
//   * the workers call raytrace_pixel() per pixel of a 32x32 tile, row-major (:293-298, 610-615):
//     the tile's first pixel queues the whole tile (sampleCountBuffer = ns_aa, as
//     bidirection.cpp:539) and returns; the others are no-ops. Queued tiles go to the device in
//     batches, one bdpt_render per batch: the worker that finds no launch in flight launches what
//     is queued, waits for it, copies those pixels into sampleBuffer (batches of up to 16 tiles;
//     a larger one waits for the frame's end) and repeats while more tiles were queued meanwhile
//     (by workers that returned at once). A later write_to_framebuffer (:619, non-virtual,
//     pathtracer.cpp:42-45) shows the tiles whose batch has been copied;
//   * the call that queues the frame's last pixel waits for the last batch and then takes the
//     whole frame — light-tracing splats land anywhere (bidirection.cpp:457-466) — into
//     sampleBuffer / eyeBuffer / lightBuffer, so the last write_to_framebuffer and save_image see
//     the final image.
// The -p cell path (8x8 tiles from the cell's corner, :300-318) cannot be told apart from a tile
// loop by the pixels alone: a cell may hold a 32-aligned pixel, which would queue a whole 32x32
// tile past the cell's edge. A host that renders cells names the cell first — set_cell(x, y, dx,
// dy), the one line a maintainer adds to render_to_file's cell branch (:338-345, next to cell_tl /
// cell_br) — and the frame's first cell pixel then queues the whole cell as one rectangle: one
// launch, one copy of the cell's pixels, and every worker returns only once the cell is in
// sampleBuffer (the cell render copies frameBuffer as soon as the workers end, :640-645). Without
// it, a pixel that no 32x32 tile covers is queued alone; lone pixels of a batch merge into
// rectangles, and their call returns once its batch (and every pixel queued before it, refreshed
// within their bounding box) is in sampleBuffer. attach() / raytrace_tile() / raytrace_frame() /
// finish() remain for callers that drive whole tiles or frames themselves.
//
// Flattening reads the reference's scene objects: Triangle p1..p3 / n1..n3, Sphere o / r, the
// BSDF parameters, the light fields and the camera (hFov, vFov, nClip, fClip, pos, c2w, w2c). The
// BSDF members and Camera's state are private in the reference; a maintainer gives this class read
// access (a `friend class BidirectionalPathTracerAMD;` line in Camera and each BSDF class) — the
// compile check in tests/test_integration.py builds it with the same read access the oracle's
// ref_driver uses.
//
// Several GPUs: BDPT_DEVICES=0,1,... (environment, read by attach) gives the binding one context per
// listed device. Queued tile batches go to whichever context is free, so up to N batches render at
// once; every context renders whole pixels (all ns_aa samples) of its tiles, and since the t = 1
// splats land anywhere the frame is the sum of the contexts' frames: finish() reduces them into the
// first context's with the C-ABI's RCCL reduce (bdpt_reduce_frames) before it reads the image. The
// per-tile copy into sampleBuffer reads the launching context's pixels (their splats from other
// contexts arrive with finish(), as later tiles' splats do on one device). A cell render (set_cell,
// or lone pixels) uses the first context only. A device listed twice shares its GPU (tests).
//
// Threading: the reference's worker threads call raytrace_pixel concurrently (on disjoint tiles).
// The per-pixel "queued" flags are allocated while the renderer is single-threaded
// (set_frame_size); the queue, the counters and every bdpt_* call on the context are under one
// mutex, released while a batch runs on the device (only the launching thread touches the
// context then).
#ifndef BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H
#define BDPT_AMD_INTEGRATION_BIDIRECTION_AMD_H

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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
    release();
    for (int dev : devices()) {   // one context per BDPT_DEVICES entry (default: device 0)
      p.device = dev;
      void* c = nullptr;
      const int rc = bdpt_create(&desc, &p, &c);
      if (rc != BDPT_OK) { release(); return rc; }
      ctxs_.push_back(c);
    }
    ctx_ = ctxs_[0];
    busy_.assign(ctxs_.size(), 0);
    if (ctxs_.size() > 1) {   // the frame is the sum of the contexts' frames (finish)
      const int rc = bdpt_reduce_create(ctxs_.data(), (int32_t)ctxs_.size(), &red_);
      if (rc != BDPT_OK) { release(); return rc; }
    }
    return BDPT_OK;
  }
  // the devices of BDPT_DEVICES ("0,1,..."; default {0})
  static std::vector<int> devices() {
    std::vector<int> d;
    const char* e = std::getenv("BDPT_DEVICES");
    for (const char* q = e; q && *q;) {
      char* end = nullptr;
      const long v = std::strtol(q, &end, 10);
      if (end == q) break;
      d.push_back((int)v);
      q = *end == ',' ? end + 1 : end;
    }
    if (d.empty()) d.push_back(0);
    return d;
  }
  size_t contexts() { std::lock_guard<std::mutex> lk(mu_); return ctxs_.size(); }

  // ---- the PathTracer contract, driven by the reference's unmodified RaytracedRenderer ----
  // start_raytracing calls clear() and then set_frame_size() before it starts the workers
  // (raytraced_renderer.cpp:280-281, 326): the per-pixel flags are allocated, zeroed, here.
  void set_frame_size(size_t width, size_t height) override {
    BidirectionalPathTracer::set_frame_size(width, height);
    drop_frame();
  }
  // start_raytracing (:280) clears before every frame: the next raytrace_pixel attaches again
  void clear() override {
    BidirectionalPathTracer::clear();
    drop_frame();
  }
  // The renderer's per-pixel call (raytraced_renderer.cpp:610-615; bidirection.cpp:503-542). It
  // runs on the renderer's worker threads, where an exception would end the process, so a failure
  // (no device, bdpt_* error) is recorded — error() — and the frame's remaining pixels are skipped.
  void raytrace_pixel(size_t x, size_t y) override {
    const size_t W = sampleBuffer.w, H = sampleBuffer.h;
    if (x >= W || y >= H || !done_ || failed_.load(std::memory_order_acquire)) return;
    if (done_[x + y * W].load(std::memory_order_acquire)) return;   // queued with its tile
    std::unique_lock<std::mutex> lk(mu_);
    if (failed_.load(std::memory_order_relaxed)) return;
    try {
      const bool lone = enqueue_locked(x, y, W, H);
      const size_t mine = seq_;
      pump(lk);
      if (lone)   // -p cell path: return once this pixel is in sampleBuffer
        cv_.wait(lk, [&] { return copied_ >= mine || failed_.load(); });
      if (queued_ == W * H && !finished_ && !failed_.load()) {
        // the frame's last pixel: wait for the batch in flight, then take the whole frame
        cv_.wait(lk, [&] { return (nbusy_ == 0 && pending_.empty()) || failed_.load(); });
        if (!failed_.load() && !finished_) {
          finished_ = true;
          finish();   // every splat is in (bidirection.cpp:457-466): sampleBuffer <- the image
        }
      }
    } catch (const std::exception& e) {
      record_failure_locked(e.what());
    }
  }
  // The -p cell (render_to_file's cell branch, raytraced_renderer.cpp:338-345): the rectangle
  // [x, x+dx) x [y, y+dy) that the coming frames' raytrace_pixel calls cover (kept across clear()
  // and set_frame_size(), which start_raytracing runs first); clear_cell() returns to whole frames.
  void set_cell(size_t x, size_t y, size_t dx, size_t dy) {
    std::lock_guard<std::mutex> lk(mu_);
    cell_ = bdpt_tile{(int32_t)x, (int32_t)y, (int32_t)dx, (int32_t)dy};
    has_cell_ = dx > 0 && dy > 0;
  }
  void clear_cell() {
    std::lock_guard<std::mutex> lk(mu_);
    has_cell_ = false;
  }
  // empty, or the first failure of the frame's raytrace_pixel calls
  std::string error() {
    std::lock_guard<std::mutex> lk(mu_);
    return failed_.load() ? err_ : std::string();
  }
  size_t launches() { std::lock_guard<std::mutex> lk(mu_); return launches_; }   // bdpt_render calls this frame
  size_t tiles_queued() { std::lock_guard<std::mutex> lk(mu_); return seq_; }    // tiles / lone pixels queued
  // seconds the launching threads spent in bdpt_render + the batches' copies into sampleBuffer
  double device_seconds() { std::lock_guard<std::mutex> lk(mu_); return busy_s_; }

 private:
  // Queues the whole cell when one is set (set_cell; returns true: the caller waits for it), else
  // the tile whose first pixel (x, y) is — tiles start at multiples of imageTileSize = 32,
  // raytraced_renderer.cpp:83,293-298 — or else the pixel alone (returns true then). mu_ held.
  bool enqueue_locked(size_t x, size_t y, size_t W, size_t H) {
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
    if (done_[x + y * W].load(std::memory_order_relaxed)) return false;
    size_t x0 = x, y0 = y, tw = 1, th = 1;
    bool wait = true;
    if (has_cell_ && (int64_t)x >= cell_.x0 && (int64_t)x < (int64_t)cell_.x0 + cell_.w && (int64_t)y >= cell_.y0 &&
        (int64_t)y < (int64_t)cell_.y0 + cell_.h) {
      // the cell, clipped to the frame, as one rectangle
      x0 = (size_t)std::max<int64_t>(0, cell_.x0);
      y0 = (size_t)std::max<int64_t>(0, cell_.y0);
      tw = (size_t)std::min<int64_t>((int64_t)W, (int64_t)cell_.x0 + cell_.w) - x0;
      th = (size_t)std::min<int64_t>((int64_t)H, (int64_t)cell_.y0 + cell_.h) - y0;
    } else if (!has_cell_ && x % kTile == 0 && y % kTile == 0) {
      tw = std::min(kTile, W - x);
      th = std::min(kTile, H - y);
      wait = false;
    }
    if (wait) single_ = true;   // a cell or lone pixels: the first context only (its copies are whole)
    for (size_t yy = y0; yy < y0 + th; yy++)
      for (size_t xx = x0; xx < x0 + tw; xx++) {
        sampleCountBuffer[xx + yy * W] = ns_aa;   // bidirection.cpp:539
        if (!done_[xx + yy * W].exchange(1, std::memory_order_release)) queued_++;
      }
    // the bounding box of everything queued this frame: what a lone batch refreshes
    qx0_ = std::min(qx0_, x0); qy0_ = std::min(qy0_, y0);
    qx1_ = std::max(qx1_, x0 + tw); qy1_ = std::max(qy1_, y0 + th);
    pending_.push_back(bdpt_tile{(int32_t)x0, (int32_t)y0, (int32_t)tw, (int32_t)th});
    seq_++;
    return wait;
  }

  // Launches the queued tiles in batches. The caller that finds no launch in flight becomes the
  // launcher and goes on until nothing is queued; tiles queued meanwhile by the other workers
  // (who return at once) go out together in the next bdpt_render. mu_ held on entry and exit,
  // released while the device works.
  void pump(std::unique_lock<std::mutex>& lk) {
    while (!pending_.empty() && !failed_.load()) {
      // a free context (the first only in a cell render): its launcher goes on while tiles are queued
      int k = -1;
      for (size_t c = 0; c < (single_ ? 1 : ctxs_.size()); c++)
        if (!busy_[c]) { k = (int)c; break; }
      if (k < 0) return;   // every context busy: their launchers take what is queued
      busy_[k] = 1;
      nbusy_++;
      void* ctx = ctxs_[k];
      std::vector<bdpt_tile> batch;
      batch.swap(pending_);
      const size_t upto = seq_;
      // the frame's last batch: finish() reads the whole frame right after it, so its own copy
      // into sampleBuffer is skipped (only its completion is waited for)
      const bool last = queued_ == sampleBuffer.w * sampleBuffer.h;
      const bool lone = coalesce(batch);
      const bdpt_tile box = {(int32_t)qx0_, (int32_t)qy0_, (int32_t)(qx1_ - qx0_), (int32_t)(qy1_ - qy0_)};
      lk.unlock();
      const auto t0 = std::chrono::steady_clock::now();
      int rc = BDPT_E_INVALID;
      std::string what;
      try {   // nothing may leave this section with mu_ released (and the context still busy)
        rc = bdpt_render(ctx, batch.data(), (int32_t)batch.size(), 0, (int32_t)ns_aa);
        if (rc == BDPT_OK) rc = last ? bdpt_sync(ctx) : copy_back(ctx, batch, lone, box);   // waits for the launch
        if (rc != BDPT_OK) what = bdpt_last_error();
      } catch (const std::exception& e) {
        what = e.what();
        rc = BDPT_E_INVALID;
      }
      const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      lk.lock();
      busy_[k] = 0;
      nbusy_--;
      launches_++;
      busy_s_ += dt;
      copied_ = std::max(copied_, upto);
      if (rc != BDPT_OK) record_failure_locked(what);
      cv_.notify_all();
    }
    cv_.notify_all();
  }

  // sampleBuffer <- the batch's pixels, one rectangle read per tile. A large batch of whole tiles
  // (more than 16: the workers queued faster than the device rendered, as without the reference's
  // per-tile tonemap) is not copied: finish() brings the whole frame in when the last pixel is
  // queued, and the copy would only delay the next launch. A batch with lone pixels (their
  // callers wait for them, the -p cell path without set_cell) refreshes every queued pixel, read
  // as one rectangle: `box`, the bounding box of what the frame has queued.
  int copy_back(void* ctx, const std::vector<bdpt_tile>& batch, bool lone, const bdpt_tile& box) {
    if (batch.size() > 16 && !lone) return bdpt_sync(ctx);
    const size_t W = sampleBuffer.w;
    std::vector<float> rgb;
    if (lone) {
      // The cell path never queues the whole frame, so finish() never runs: every batch refreshes
      // all pixels queued so far, so the splats of later samples (bidirection.cpp:457-466) reach
      // the cell's earlier pixels too, and the cell's last batch leaves it complete.
      rgb.resize((size_t)box.w * box.h * 3);
      int rc = bdpt_read_frame_rect(ctx, BDPT_FRAME_SAMPLE, box.x0, box.y0, box.w, box.h, rgb.data());
      if (rc != BDPT_OK) return rc;
      for (int32_t yy = 0; yy < box.h; yy++)
        for (int32_t xx = 0; xx < box.w; xx++) {
          const size_t k = (size_t)(box.x0 + xx) + (size_t)(box.y0 + yy) * W;
          const float* v = &rgb[3 * ((size_t)xx + (size_t)yy * box.w)];
          if (done_[k].load(std::memory_order_relaxed)) sampleBuffer.data[k] = Vector3D(v[0], v[1], v[2]);
        }
      return BDPT_OK;
    }
    for (const bdpt_tile& t : batch) {
      rgb.resize((size_t)t.w * t.h * 3);
      int rc = bdpt_read_frame_rect(ctx, BDPT_FRAME_SAMPLE, t.x0, t.y0, t.w, t.h, rgb.data());
      if (rc != BDPT_OK) return rc;
      for (int32_t yy = 0; yy < t.h; yy++)
        for (int32_t xx = 0; xx < t.w; xx++) {
          const float* v = &rgb[3 * (xx + yy * t.w)];
          sampleBuffer.data[(t.x0 + xx) + (t.y0 + yy) * W] = Vector3D(v[0], v[1], v[2]);
        }
    }
    return BDPT_OK;
  }

  // Lone pixels merge into rectangles: runs along a row, then equal runs on consecutive rows (an
  // 8x8 cell tile becomes one tile instead of 64 one-pixel blocks). The set of pixels, and so the
  // image, is unchanged.
  // Returns whether the batch held lone pixels.
  static bool coalesce(std::vector<bdpt_tile>& batch) {
    std::vector<bdpt_tile> out, px;
    for (const bdpt_tile& t : batch) (t.w == 1 && t.h == 1 ? px : out).push_back(t);
    if (px.size() < 2) return !px.empty();
    std::sort(px.begin(), px.end(), [](const bdpt_tile& a, const bdpt_tile& b) {
      return a.y0 != b.y0 ? a.y0 < b.y0 : a.x0 < b.x0;
    });
    std::vector<bdpt_tile> runs;
    for (const bdpt_tile& p : px) {
      if (!runs.empty() && runs.back().y0 == p.y0 && runs.back().x0 + runs.back().w == p.x0) runs.back().w++;
      else runs.push_back(p);
    }
    std::sort(runs.begin(), runs.end(), [](const bdpt_tile& a, const bdpt_tile& b) {
      return a.x0 != b.x0 ? a.x0 < b.x0 : a.w != b.w ? a.w < b.w : a.y0 < b.y0;
    });
    std::vector<bdpt_tile> rects;
    for (const bdpt_tile& r : runs) {
      bdpt_tile* b = rects.empty() ? nullptr : &rects.back();
      if (b && b->x0 == r.x0 && b->w == r.w && b->y0 + b->h == r.y0) b->h++;
      else rects.push_back(r);
    }
    out.insert(out.end(), rects.begin(), rects.end());
    batch.swap(out);
    return true;
  }

  void record_failure_locked(const std::string& what) {
    if (!failed_.load()) err_ = what;
    failed_.store(true, std::memory_order_release);
    cv_.notify_all();
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
  // After attach(): one untimed one-pixel launch (the process's first launch loads the kernel's
  // code object), then the frames are cleared again — for hosts that time their frames.
  void warm_up() {
    bdpt_tile t = {0, 0, 1, 1};
    check(bdpt_render(ctx_, &t, 1, 0, 1));
    check(bdpt_sync(ctx_));
    check(bdpt_clear(ctx_));
    check(bdpt_sync(ctx_));
  }
  // sampleBuffer / eyeBuffer / lightBuffer <- the device frames, before save_image. The sample
  // frame is the fp32 sum eye + light (what bdpt_read_frame(BDPT_FRAME_SAMPLE) returns, formed here
  // from the two frames already read). The conversion to the reference's double buffers (3 x W*H
  // Vector3D) is split over up to 16 host threads: 1080p is 6 M vectors.
  void finish() {
    const size_t n = sampleBuffer.w * sampleBuffer.h;
    if (red_) check(bdpt_reduce_frames(red_, 0));   // every context's frame into the first's
    std::vector<float> eye(n * 3), light(n * 3);
    check(bdpt_read_frame(ctx_, BDPT_FRAME_EYE, eye.data()));
    check(bdpt_read_frame(ctx_, BDPT_FRAME_LIGHT, light.data()));
    const bool el = eyeBuffer.w * eyeBuffer.h == n && lightBuffer.w * lightBuffer.h == n;
    auto convert = [&](size_t k0, size_t k1) {
      for (size_t k = k0; k < k1; k++) {
        const float* e = &eye[3 * k];
        const float* l = &light[3 * k];
        sampleBuffer.data[k] = Vector3D(e[0] + l[0], e[1] + l[1], e[2] + l[2]);
        if (el) {
          eyeBuffer.data[k] = Vector3D(e[0], e[1], e[2]);
          lightBuffer.data[k] = Vector3D(l[0], l[1], l[2]);
        }
      }
    };
    const size_t nt = std::max<size_t>(1, std::min<size_t>({16, (size_t)std::thread::hardware_concurrency(), n / 65536 + 1}));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; t++) th.emplace_back(convert, n * t / nt, n * (t + 1) / nt);
    convert(0, n / nt);
    for (std::thread& x : th) x.join();
  }
  ~BidirectionalPathTracerAMD() { release(); }

 private:
  // the reduce before the contexts it reads (bdpt_reduce_destroy), then the contexts
  void release() {
    if (red_) { bdpt_reduce_destroy(red_); red_ = nullptr; }
    for (void* c : ctxs_) bdpt_destroy(c);
    ctxs_.clear();
    ctx_ = nullptr;
  }
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
  // a new frame (size / scene / camera may have changed): attach again. Called on the renderer's
  // thread with no worker running (set_frame_size / clear, :280-281).
  void drop_frame() {
    std::lock_guard<std::mutex> lk(mu_);
    release();
    const size_t n = sampleBuffer.w * sampleBuffer.h;
    done_.reset(n ? new std::atomic<uint8_t>[n]() : nullptr);   // value-initialised: all 0
    pending_.clear();
    qx0_ = qy0_ = SIZE_MAX;
    qx1_ = qy1_ = 0;
    queued_ = seq_ = copied_ = launches_ = 0;
    busy_s_ = 0.0;
    nbusy_ = 0;
    busy_.assign(busy_.size(), 0);
    single_ = finished_ = false;
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
  void* ctx_ = nullptr;                            // the first context (ctxs_[0])
  std::vector<void*> ctxs_;                        // one per BDPT_DEVICES entry
  bdpt_reducer* red_ = nullptr;                    // their frame reduce (more than one context)
  std::vector<char> busy_;                         // per context: a launcher is using it
  int nbusy_ = 0;
  bool single_ = false;                            // a cell / lone pixels this frame: first context only
  std::mutex mu_;
  std::condition_variable cv_;
  std::unique_ptr<std::atomic<uint8_t>[]> done_;   // per pixel: queued (with its tile)
  std::vector<bdpt_tile> pending_;                 // queued, not yet launched
  size_t queued_ = 0;                              // pixels queued this frame
  size_t qx0_ = SIZE_MAX, qy0_ = SIZE_MAX, qx1_ = 0, qy1_ = 0;   // their bounding box
  bdpt_tile cell_ = {0, 0, 0, 0};                  // set_cell: the -p cell, kept across frames
  bool has_cell_ = false;
  size_t seq_ = 0, copied_ = 0;                    // tiles queued / tiles whose batch is in sampleBuffer
  size_t launches_ = 0;
  double busy_s_ = 0.0;
  bool finished_ = false;
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
