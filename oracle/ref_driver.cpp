// oracle/ref_driver.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).
//
// Headless driver around the reference's own hot-path sources (compiled where they lie under
// /root/reference by oracle/ref.mk into oracle/_ref/). It mirrors the windowless `-f` branch of
// the reference CLI (src/application/main.cpp:157-181): ColladaParser::load -> the scene
// assembly of Application::load (src/application/application.cpp:228-304; restated here
// because application.cpp needs GLU, which this image lacks) -> Application::resize ->
// set_up_pathtracer (application.cpp:633-639) -> RaytracedRenderer::render_to_file
// (raytraced_renderer.cpp:330-347) with -t threads. Afterwards it dumps
//   * the HDR buffers of BidirectionalPathTracer (sampleBuffer / eyeBuffer / lightBuffer,
//     bidirection.h:81, pathtracer.h:90) as float64 .npy (row 0 = bottom, as the reference),
//   * the static scene the integrator saw (primitives in scene order, BSDF parameters,
//     lights, camera state) as JSON with round-trip (%.17g) doubles,
//   * BVH statistics and the DFS primitive order of the leaves (bvh.cpp:51-129).
// These outputs become the golden fixtures under tests/golden/ (see tools/make_golden.py).
// Options beyond the reference CLI's: -e map.exr loads an environment map exactly as main.cpp's
// -e (load_exr, restated in oracle/ref_env_kat.cpp's shared copy below); -U swaps the integrator
// for the reference's unidirectional PathTracer (pathtracer.cpp:47-340; the reference constructs
// only the BDPT one, raytraced_renderer.cpp:53) with -a batch tol as main.cpp's -a — used as the
// converged-image cross-check of the environment light (tests/test_env.py).

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <map>
#include <set>
#include <list>
#include <thread>
#include <mutex>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <stack>
#include <random>
#include <algorithm>
#include <sstream>
#include <fstream>
#include <iostream>
#include <unordered_map>
#include <functional>
#include <getopt.h>

#define TINYEXR_IMPLEMENTATION
#include "CGL/tinyexr.h"

// Read-only access to the reference's private state (buffers, camera, BSDF parameters).
#define private public
#define protected public
#include "CGL/CGL.h"
#include "scene/collada/collada.h"
#include "scene/gl_scene/scene.h"
#include "scene/gl_scene/mesh.h"
#include "scene/gl_scene/sphere.h"
#include "scene/gl_scene/area_light.h"
#include "scene/gl_scene/point_light.h"
#include "scene/gl_scene/directional_light.h"
#include "scene/gl_scene/ambient_light.h"
#include "scene/gl_scene/spot_light.h"
#include "scene/scene.h"
#ifdef BDPT_INTEGRATION
#include "bidirection_amd.h"   // integration/: the reference-side binding to libbdpt_amd.so
#endif
#include "scene/light.h"
#include "scene/triangle.h"
#include "scene/sphere.h"
#include "scene/bvh.h"
#include "pathtracer/bsdf.h"
#include "pathtracer/camera.h"
#include "pathtracer/raytraced_renderer.h"
#include "pathtracer/bidirection.h"
#undef private
#undef protected

using namespace CGL;
using namespace CGL::Collada;

static void write_npy(const std::string& path, const HDRImageBuffer& b) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) { perror(path.c_str()); exit(2); }
  char hdr[128];
  int n = snprintf(hdr, sizeof hdr, "{'descr': '<f8', 'fortran_order': False, 'shape': (%zu, %zu, 3), }",
                   b.h, b.w);
  int total = 10 + n + 1;
  int pad = (64 - total % 64) % 64;
  unsigned short hl = (unsigned short)(n + pad + 1);
  fwrite("\x93NUMPY\x01\x00", 1, 8, f);
  fwrite(&hl, 2, 1, f);
  fwrite(hdr, 1, n, f);
  for (int i = 0; i < pad; i++) fputc(' ', f);
  fputc('\n', f);
  for (size_t i = 0; i < b.w * b.h; i++) {
    double v[3] = {b.data[i].x, b.data[i].y, b.data[i].z};
    fwrite(v, 8, 3, f);
  }
  fclose(f);
}

static std::string v3(const Vector3D& v) {
  char buf[128];
  snprintf(buf, sizeof buf, "[%.17g, %.17g, %.17g]", v.x, v.y, v.z);
  return buf;
}
static std::string d1(double d) {
  char buf[64];
  snprintf(buf, sizeof buf, "%.17g", d);
  return buf;
}

struct BvhStats { size_t nodes = 0, leaves = 0, depth = 0; };
static void walk_bvh(SceneObjects::BVHNode* n, size_t depth, BvhStats& st,
                     const std::map<const SceneObjects::Primitive*, size_t>& idx,
                     std::vector<size_t>& order) {
  st.nodes++;
  st.depth = std::max(st.depth, depth);
  if (n->isLeaf()) {
    st.leaves++;
    for (auto p = n->start; p != n->end; p++) order.push_back(idx.at(*p));
    return;
  }
  walk_bvh(n->l, depth + 1, st, idx, order);
  walk_bvh(n->r, depth + 1, st, idx, order);
}

static void dump_scene(const std::string& path, RaytracedRenderer* rr, Camera& cam) {
  SceneObjects::Scene* sc = rr->scene;
  std::vector<SceneObjects::Primitive*> prims;
  for (auto* obj : sc->objects) {
    const auto& p = obj->get_primitives();
    prims.insert(prims.end(), p.begin(), p.end());
  }
  std::map<const BSDF*, size_t> mat_id;
  std::vector<const BSDF*> mats;
  auto mat_of = [&](const BSDF* b) {
    auto it = mat_id.find(b);
    if (it != mat_id.end()) return it->second;
    mat_id[b] = mats.size();
    mats.push_back(b);
    return mats.size() - 1;
  };
  std::ostringstream tris, sphs, porder;
  bool ft = true, fs = true;
  size_t nt = 0, ns = 0;
  for (auto* p : prims) {
    if (nt + ns) porder << ",";
    if (dynamic_cast<SceneObjects::Triangle*>(p)) porder << "[\"t\"," << nt++ << "]";
    else porder << "[\"s\"," << ns++ << "]";
    if (auto* t = dynamic_cast<SceneObjects::Triangle*>(p)) {
      tris << (ft ? "" : ",\n") << "  [" << v3(t->p1) << "," << v3(t->p2) << "," << v3(t->p3) << ","
           << v3(t->n1) << "," << v3(t->n2) << "," << v3(t->n3) << "," << mat_of(t->bsdf) << "]";
      ft = false;
    } else if (auto* s = dynamic_cast<SceneObjects::Sphere*>(p)) {
      sphs << (fs ? "" : ",\n") << "  [" << v3(s->o) << "," << d1(s->r) << "," << mat_of(s->get_bsdf()) << "]";
      fs = false;
    }
  }
  // BVH over the same primitive list (a fresh build gives the identical tree:
  // construct_bvh is deterministic, bvh.cpp:51-129).
  SceneObjects::BVHAccel bvh(prims, 4);
  std::map<const SceneObjects::Primitive*, size_t> pidx;
  for (size_t i = 0; i < prims.size(); i++) pidx[prims[i]] = i;
  BvhStats st;
  std::vector<size_t> order;
  walk_bvh(bvh.root, 0, st, pidx, order);

  std::ofstream o(path);
  o << "{\n\"source\": \"reference (oracle/_ref/ref_driver)\",\n";
  o << "\"camera\": {\"pos\": " << v3(cam.pos) << ", \"target\": " << v3(cam.targetPos)
    << ", \"c2w_cols\": [" << v3(cam.c2w[0]) << "," << v3(cam.c2w[1]) << "," << v3(cam.c2w[2]) << "]"
    << ", \"w2c_cols\": [" << v3(cam.w2c[0]) << "," << v3(cam.w2c[1]) << "," << v3(cam.w2c[2]) << "]"
    << ", \"hFov\": " << d1(cam.hFov) << ", \"vFov\": " << d1(cam.vFov) << ", \"ar\": " << d1(cam.ar)
    << ", \"nClip\": " << d1(cam.nClip) << ", \"fClip\": " << d1(cam.fClip)
    << ", \"phi\": " << d1(cam.phi) << ", \"theta\": " << d1(cam.theta) << ", \"r\": " << d1(cam.r)
    << ", \"screenW\": " << cam.screenW << ", \"screenH\": " << cam.screenH
    << ", \"screenDist\": " << d1(cam.screenDist) << "},\n";
  o << "\"lights\": [";
  bool fl = true;
  for (auto* l : sc->lights) {
    o << (fl ? "\n" : ",\n");
    fl = false;
    if (auto* a = dynamic_cast<SceneObjects::AreaLight*>(l)) {
      o << "  {\"type\": \"area\", \"radiance\": " << v3(a->radiance) << ", \"position\": " << v3(a->position)
        << ", \"direction\": " << v3(a->direction) << ", \"dim_x\": " << v3(a->dim_x)
        << ", \"dim_y\": " << v3(a->dim_y) << ", \"area\": " << d1(a->area) << "}";
    } else if (auto* pl = dynamic_cast<SceneObjects::PointLight*>(l)) {
      o << "  {\"type\": \"point\", \"radiance\": " << v3(pl->radiance) << ", \"position\": " << v3(pl->position) << "}";
    } else if (auto* hl = dynamic_cast<SceneObjects::InfiniteHemisphereLight*>(l)) {
      o << "  {\"type\": \"hemisphere\", \"radiance\": " << v3(hl->radiance) << "}";
    } else if (auto* dl = dynamic_cast<SceneObjects::DirectionalLight*>(l)) {
      o << "  {\"type\": \"directional\", \"radiance\": " << v3(dl->radiance) << ", \"direction\": "
        << v3(dl->dirToLight) << "}";
    } else {
      o << "  {\"type\": \"unsupported\"}";
    }
  }
  o << "],\n\"materials\": [";
  for (size_t i = 0; i < mats.size(); i++) {
    const BSDF* b = mats[i];
    o << (i ? ",\n  " : "\n  ");
    if (auto* d = dynamic_cast<const DiffuseBSDF*>(b))
      o << "{\"type\": \"diffuse\", \"reflectance\": " << v3(d->reflectance) << "}";
    else if (auto* e = dynamic_cast<const EmissionBSDF*>(b))
      o << "{\"type\": \"emission\", \"radiance\": " << v3(e->radiance) << "}";
    else if (auto* m = dynamic_cast<const MirrorBSDF*>(b))
      o << "{\"type\": \"mirror\", \"reflectance\": " << v3(m->reflectance) << "}";
    else if (auto* g = dynamic_cast<const GlassBSDF*>(b))
      o << "{\"type\": \"glass\", \"reflectance\": " << v3(g->reflectance) << ", \"transmittance\": "
        << v3(g->transmittance) << ", \"roughness\": " << d1(g->roughness) << ", \"ior\": " << d1(g->ior) << "}";
    else if (auto* r = dynamic_cast<const RefractionBSDF*>(b))
      o << "{\"type\": \"refraction\", \"transmittance\": " << v3(r->transmittance) << ", \"roughness\": "
        << d1(r->roughness) << ", \"ior\": " << d1(r->ior) << "}";
    else if (auto* mf = dynamic_cast<const MicrofacetBSDF*>(b))
      o << "{\"type\": \"microfacet\", \"eta\": " << v3(mf->eta) << ", \"k\": " << v3(mf->k)
        << ", \"alpha\": " << d1(mf->alpha) << "}";
    else
      o << "{\"type\": \"unknown\"}";
  }
  o << "],\n\"bvh\": {\"nodes\": " << st.nodes << ", \"leaves\": " << st.leaves << ", \"depth\": " << st.depth
    << ", \"dfs_prim_order\": [";
  for (size_t i = 0; i < order.size(); i++) o << (i ? "," : "") << order[i];
  o << "]},\n\"prim_order\": [" << porder.str() << "],\n\"triangles\": [\n" << tris.str() << "],\n\"spheres\": [\n" << sphs.str() << "]\n}\n";
}

// main.cpp:40-77
static HDRImageBuffer* load_exr(const char* file_path) {
  const char* err;
  EXRImage exr;
  InitEXRImage(&exr);
  if (ParseMultiChannelEXRHeaderFromFile(&exr, file_path, &err) != 0) return nullptr;
  for (int i = 0; i < exr.num_channels; i++)
    if (exr.pixel_types[i] == TINYEXR_PIXELTYPE_HALF) exr.requested_pixel_types[i] = TINYEXR_PIXELTYPE_FLOAT;
  if (LoadMultiChannelEXRFromFile(&exr, file_path, &err) != 0) return nullptr;
  HDRImageBuffer* envmap = new HDRImageBuffer();
  envmap->resize(exr.width, exr.height);
  float* channel_r = (float*)exr.images[2];
  float* channel_g = (float*)exr.images[1];
  float* channel_b = (float*)exr.images[0];
  for (size_t i = 0; i < (size_t)exr.width * exr.height; i++)
    envmap->data[i] = Vector3D(channel_r[i], channel_g[i], channel_b[i]);
  return envmap;
}

int main(int argc, char** argv) {
  size_t ns_aa = 1, max_depth = 1, threads = 1, w = 0, h = 0, batch = 32, nal = 1;
  size_t cx = (size_t)-1, cy = 0, cdx = 0, cdy = 0;   // -p: the cell render (main.cpp:97-103, 180)
  float tol = 0.05f;
  bool hemi = false;
  double lens = 0.0, focal = 4.7;
  std::string png = "/dev/null", npy_prefix, scene_json, cam_settings;
  bool render = true, uni = false, amd = false, amd_loop = false, tile_loop = false, no_cell_hook = false;
  HDRImageBuffer* envmap = nullptr;
  int opt;
  while ((opt = getopt(argc, argv, "s:t:m:r:f:o:j:ne:Ua:Hb:d:l:c:GABCp:")) != -1) {
    switch (opt) {
      case 's': ns_aa = atoi(optarg); break;
      case 't': threads = atoi(optarg); break;
      case 'm': max_depth = atoi(optarg); break;
      case 'r': w = atoi(argv[optind - 1]); h = atoi(argv[optind]); optind++; break;  // main.cpp:93-97
      case 'f': png = optarg; break;
      case 'o': npy_prefix = optarg; break;
      case 'j': scene_json = optarg; break;
      case 'n': render = false; break;
      case 'e': envmap = load_exr(optarg); if (!envmap) return 4; break;
      case 'U': uni = true; break;
      case 'H': hemi = true; break;                      // main.cpp:138-141
      case 'l': nal = atoi(optarg); break;               // main.cpp:107-109
      case 'b': lens = atof(optarg); break;              // main.cpp:128-130
      case 'd': focal = atof(optarg); break;             // main.cpp:131-133
      case 'a': batch = atoi(argv[optind - 1]); tol = atof(argv[optind]); optind++; break;   // main.cpp:134-137
      case 'c': cam_settings = optarg; break;            // main.cpp:120-121
      case 'G': amd = true; break;                       // integration check (BDPT_INTEGRATION builds)
      case 'A': amd_loop = true; break;                  // the binding under the reference's own render loop
      case 'B': amd_loop = true; tile_loop = true; break;   // ... its worker loop without the per-tile tonemap
      case 'C': no_cell_hook = true; break;              // -A -p without the binding's set_cell line
      case 'p':                                          // main.cpp:97-103
        cx = atoi(argv[optind - 1]); cy = atoi(argv[optind]); cdx = atoi(argv[optind + 1]); cdy = atoi(argv[optind + 2]);
        optind += 3;
        break;
      default: fprintf(stderr, "usage: ref_driver [-s spp] [-t thr] [-m depth] [-r W H] [-f png] [-o npy_prefix] [-j scene.json] [-n] scene.dae\n"); return 1;
    }
  }
  if (optind >= argc) return 1;
  SceneInfo* info = new SceneInfo();
  if (ColladaParser::load(argv[optind], info) < 0) return 3;

  // --- Application::init (application.cpp:52-104), windowless part ---
  size_t screenW = 800, screenH = 600;
  Camera camera;
  {
    CameraInfo ci;
    ci.hFov = 50; ci.vFov = 35; ci.nClip = 0.01; ci.fClip = 100;
    camera.configure(ci, screenW, screenH);
  }
  // --- Application::load (application.cpp:228-304) ---
  std::vector<GLScene::SceneLight*> lights;
  std::vector<GLScene::SceneObject*> objects;
  Vector3D c_pos, c_dir;
  for (auto& node : info->nodes) {
    Instance* inst = node.instance;
    const Matrix4x4& T = node.transform;
    switch (inst->type) {
      case Instance::CAMERA: {
        CameraInfo* c = static_cast<CameraInfo*>(inst);
        c_pos = (T * Vector4D(c_pos, 1)).to3D();
        c_dir = (T * Vector4D(c->view_dir, 1)).to3D().unit();
        camera.configure(*c, screenW, screenH);  // init_camera, application.cpp:306-312
        break;
      }
      case Instance::LIGHT: {
        LightInfo& li = static_cast<LightInfo&>(*inst);
        GLScene::SceneLight* l = nullptr;
        switch (li.light_type) {                 // init_light, application.cpp:318-336
          case LightType::AMBIENT: l = new GLScene::AmbientLight(li); break;
          case LightType::DIRECTIONAL: l = new GLScene::DirectionalLight(li, T); break;
          case LightType::AREA: l = new GLScene::AreaLight(li, T); break;
          case LightType::POINT: l = new GLScene::PointLight(li, T); break;
          case LightType::SPOT: l = new GLScene::SpotLight(li, T); break;
          default: break;
        }
        lights.push_back(l);
        break;
      }
      case Instance::SPHERE: {                   // init_sphere, application.cpp:345-351
        SphereInfo& si = static_cast<SphereInfo&>(*inst);
        const Vector3D& position = (T * Vector4D(0, 0, 0, 1)).projectTo3D();
        double scale = (T * Vector4D(1, 0, 0, 0)).to3D().norm();
        objects.push_back(new GLScene::Sphere(si, position, scale));
        break;
      }
      case Instance::POLYMESH:                   // init_polymesh, application.cpp:353-356
        objects.push_back(new GLScene::Mesh(static_cast<PolymeshInfo&>(*inst), T));
        break;
      default: break;                            // materials: parsed already (collada.cpp:854-938)
    }
  }
  GLScene::Scene* scene = new GLScene::Scene(objects, lights);
  const BBox& bbox = scene->get_bbox();
  if (!bbox.empty()) {
    Vector3D target = bbox.centroid();
    double canonical_view_distance = bbox.extent.norm() / 2 * 1.5;
    double view_distance = canonical_view_distance * 2;
    double min_view_distance = canonical_view_distance / 10.0;
    double max_view_distance = canonical_view_distance * 20.0;
    camera.place(target, acos(c_dir.y), atan2(c_dir.x, c_dir.z), view_distance,
                 min_view_distance, max_view_distance);
  }
  // --- main.cpp:172-173 -> Application::resize (application.cpp:188-200) ---
  if (w && h) { screenW = w; screenH = h; camera.set_screen_size(w, h); }
  // --- main.cpp:177-178 -> Application::load_camera (application.h:114-116) ---
  if (!cam_settings.empty()) camera.load_settings(cam_settings);

  // --- Application ctor (application.cpp:21-40) with AppConfig defaults (application.h:45-65) ---
  RaytracedRenderer* rr = new RaytracedRenderer(ns_aa, max_depth, nal, 1, 1, 1, threads, batch, tol,
                                                envmap, hemi, "", lens, focal);
  if (uni) {   // the reference's unidirectional integrator with the same settings (:53-74)
    PathTracer* u = new PathTracer();
    PathTracer* b = rr->pt;
    u->ns_aa = b->ns_aa; u->max_ray_depth = b->max_ray_depth; u->ns_area_light = b->ns_area_light;
    u->ns_diff = b->ns_diff; u->ns_glsy = b->ns_glsy; u->ns_refr = b->ns_refr;
    u->samplesPerBatch = b->samplesPerBatch; u->maxTolerance = b->maxTolerance;
    u->direct_hemisphere_sample = b->direct_hemisphere_sample; u->envLight = b->envLight;
    rr->pt = u;
  }
#ifdef BDPT_INTEGRATION
  BidirectionalPathTracerAMD* amd_pt = nullptr;
  if (amd_loop) {
    // The integration's one-line change at raytraced_renderer.cpp:53 — the renderer holds a
    // BidirectionalPathTracerAMD instead of a BidirectionalPathTracer, with the same settings
    // (:55-75) — made here right after construction; set_camera / set_scene / set_frame_size and
    // render_to_file (worker threads, raytrace_tile -> raytrace_pixel, write_to_framebuffer,
    // save_image) below run as the reference wrote them.
    PathTracer* b = rr->pt;
    amd_pt = new BidirectionalPathTracerAMD();
    amd_pt->ns_aa = b->ns_aa; amd_pt->max_ray_depth = b->max_ray_depth; amd_pt->ns_area_light = b->ns_area_light;
    amd_pt->ns_diff = b->ns_diff; amd_pt->ns_glsy = b->ns_glsy; amd_pt->ns_refr = b->ns_refr;
    amd_pt->samplesPerBatch = b->samplesPerBatch; amd_pt->maxTolerance = b->maxTolerance;
    amd_pt->direct_hemisphere_sample = b->direct_hemisphere_sample; amd_pt->envLight = b->envLight;
    rr->pt = amd_pt;
  }
#else
  if (amd_loop) {
    fprintf(stderr, "[ref_driver] -A needs the BDPT_INTEGRATION build (oracle/_ref/ref_driver_amd)\n");
    return 2;
  }
#endif
  // --- set_up_pathtracer (application.cpp:633-639) ---
  rr->set_camera(&camera);
  rr->set_scene(scene->get_static_scene());
  rr->set_frame_size(screenW, screenH);
  if (!scene_json.empty()) dump_scene(scene_json, rr, camera);
  if (!render) return 0;
  if (amd) {
#ifdef BDPT_INTEGRATION
    // integration/bidirection_amd.h in place of the reference's BidirectionalPathTracer: the
    // primitives in build_accel's collection order (raytraced_renderer.cpp:352-360), the scene's
    // lights (the env light appended last, :117-119) and the camera, then one whole-frame render
    // through libbdpt_amd.so; -o writes its sampleBuffer like the reference path does.
    BidirectionalPathTracerAMD gpu;
    gpu.ns_aa = rr->pt->ns_aa;
    gpu.max_ray_depth = rr->pt->max_ray_depth;
    gpu.set_frame_size(screenW, screenH);
    std::vector<SceneObjects::Primitive*> prims;
    for (SceneObjects::SceneObject* obj : rr->scene->objects) {
      const std::vector<SceneObjects::Primitive*>& op = obj->get_primitives();
      prims.insert(prims.end(), op.begin(), op.end());
    }
    const int rc = gpu.attach(prims, rr->scene->lights, camera, envmap);
    if (rc != BDPT_OK) {
      fprintf(stderr, "[ref_driver] BidirectionalPathTracerAMD::attach: %d (%s)\n", rc, bdpt_last_error());
      return 20 - rc;   // BDPT_E_DEVICE (-3) -> 23
    }
    gpu.raytrace_frame();
    gpu.finish();
    if (!npy_prefix.empty()) write_npy(npy_prefix + "_sample.npy", gpu.sampleBuffer);
    fprintf(stdout, "[ref_driver] rendered through libbdpt_amd.so\n");
    return 0;
#else
    fprintf(stderr, "[ref_driver] -G needs the BDPT_INTEGRATION build (oracle/_ref/ref_driver_amd)\n");
    return 2;
#endif
  }
#ifdef BDPT_INTEGRATION
  if (tile_loop) {
    // -B: the binding's own throughput. The reference's worker loop (raytraced_renderer.cpp:
    // 654-666 -> raytrace_tile :595-617: `threads` workers take the 32x32 tiles of
    // start_raytracing's queue in raster order, :293-298, and call raytrace_pixel on every pixel,
    // row-major) WITHOUT the whole-frame write_to_framebuffer after each tile (:619), whose cost
    // grows with the frame's pixels times its tiles and does not depend on the integrator. The
    // scene is attached (bdpt_create: BVH build + upload, the reference's build_accel) before
    // the timer starts, and one untimed one-pixel launch loads the kernel (warm_up).
    amd_pt->clear();
    amd_pt->set_frame_size(screenW, screenH);
    std::vector<SceneObjects::Primitive*> prims;
    for (SceneObjects::SceneObject* obj : rr->scene->objects) {
      const std::vector<SceneObjects::Primitive*>& op = obj->get_primitives();
      prims.insert(prims.end(), op.begin(), op.end());
    }
    amd_pt->bvh = rr->bvh; amd_pt->camera = &camera; amd_pt->scene = rr->scene;
    const int rc = amd_pt->attach(prims, rr->scene->lights, camera, envmap);
    if (rc != BDPT_OK) {
      fprintf(stderr, "[ref_driver] BidirectionalPathTracerAMD::attach: %d (%s)\n", rc, bdpt_last_error());
      return 20 - rc;
    }
    amd_pt->warm_up();   // the first launch loads the kernel's code object: not part of a frame
    const size_t T = 32;
    std::vector<std::pair<size_t, size_t>> tiles;
    for (size_t y = 0; y < screenH; y += T)
      for (size_t x = 0; x < screenW; x += T) tiles.emplace_back(x, y);
    std::atomic<size_t> next{0};
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ws;
    for (size_t t = 0; t < threads; t++)
      ws.emplace_back([&] {
        for (size_t k; (k = next.fetch_add(1)) < tiles.size();)
          for (size_t y = tiles[k].second; y < std::min(tiles[k].second + T, screenH); y++)
            for (size_t x = tiles[k].first; x < std::min(tiles[k].first + T, screenW); x++) amd_pt->raytrace_pixel(x, y);
      });
    for (auto& w : ws) w.join();
    const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!amd_pt->error().empty()) {
      fprintf(stderr, "[ref_driver] BidirectionalPathTracerAMD: %s\n", amd_pt->error().c_str());
      return 24;
    }
    fprintf(stdout, "[ref_driver] binding tile loop: %.4f s, %.3f Msamples/s, %zu tiles, %zu bdpt_render "
            "launches, %.4f s in launches, %zu device context(s)\n", secs,
            (double)screenW * screenH * ns_aa / secs * 1e-6, amd_pt->tiles_queued(), amd_pt->launches(),
            amd_pt->device_seconds(), amd_pt->contexts());
    if (!npy_prefix.empty()) {
      write_npy(npy_prefix + "_sample.npy", amd_pt->sampleBuffer);
      write_npy(npy_prefix + "_eye.npy", amd_pt->eyeBuffer);
      write_npy(npy_prefix + "_light.npy", amd_pt->lightBuffer);
    }
    return 0;
  }
  std::chrono::steady_clock::time_point loop_t0 = std::chrono::steady_clock::now();
#endif
#ifdef BDPT_INTEGRATION
  // the maintainer's second line, for -p cell renders: render_to_file's cell branch
  // (raytraced_renderer.cpp:338-345) names the cell to the binding next to cell_tl / cell_br
  if (amd_pt && cx != (size_t)-1 && !no_cell_hook) amd_pt->set_cell(cx, cy, cdx, cdy);
#endif
  try {
    rr->render_to_file(png, cx, cy, cdx, cdy);   // x = -1: the whole frame
  } catch (const std::exception& e) {   // the binding reports bdpt_* failures as exceptions
    fprintf(stderr, "[ref_driver] %s\n", e.what());
    return 23;
  }
#ifdef BDPT_INTEGRATION
  if (amd_pt && !amd_pt->error().empty()) {
    fprintf(stderr, "[ref_driver] BidirectionalPathTracerAMD: %s\n", amd_pt->error().c_str());
    return amd_pt->error() == "no HIP device" ? 23 : 24;
  }
  if (amd_pt)
    fprintf(stdout, "[ref_driver] bdpt_render launches: %zu for %zu tiles; %.4f s in launches of %.4f s in "
            "render_to_file; %zu device context(s)\n", amd_pt->launches(), amd_pt->tiles_queued(),
            amd_pt->device_seconds(), std::chrono::duration<double>(std::chrono::steady_clock::now() - loop_t0).count(),
            amd_pt->contexts());
#endif
  if (!npy_prefix.empty() && uni) {
    write_npy(npy_prefix + "_sample.npy", rr->pt->sampleBuffer);
    FILE* fc = fopen((npy_prefix + "_count.bin").c_str(), "wb");   // sampleCountBuffer, int32 row-major
    if (fc) {
      fwrite(rr->pt->sampleCountBuffer.data(), sizeof(int), rr->pt->sampleCountBuffer.size(), fc);
      fclose(fc);
    }
  } else if (!npy_prefix.empty()) {
    BidirectionalPathTracer* pt = (BidirectionalPathTracer*)rr->pt;
    write_npy(npy_prefix + "_sample.npy", pt->sampleBuffer);
    write_npy(npy_prefix + "_eye.npy", pt->eyeBuffer);
    write_npy(npy_prefix + "_light.npy", pt->lightBuffer);
    fprintf(stdout, "[ref_driver] rays=%llu isects=%llu\n", (unsigned long long)rr->bvh->total_rays,
            (unsigned long long)rr->bvh->total_isects);
  }
  return 0;
}
