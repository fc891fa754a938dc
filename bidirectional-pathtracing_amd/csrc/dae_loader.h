// dae_loader.h — host-side COLLADA (.dae) scene loader for the BDPT path.
//
// Produces the scene exactly as the reference hands it to its path tracer: ColladaParser::load
// (src/scene/collada/collada.cpp:129-941) for the document, Application::load
// (src/application/application.cpp:228-304) for camera placement / lights / objects,
// GLScene::Mesh + HalfedgeMesh::build (src/scene/gl_scene/mesh.cpp:22-43,
// src/util/halfEdgeMesh.cpp:29-404) for the triangle vertex order and the area-weighted vertex
// normals (halfEdgeMesh.h:492-515), GLScene::{Sphere,AreaLight,PointLight}, and Camera::configure /
// place / set_screen_size (src/pathtracer/camera.cpp:29-147). Primitives come out in the
// reference's order (scene nodes in document post-order, faces in mesh order), so the BVH built
// by bdpt_create has the reference's leaf order.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "bdpt/bdpt.h"

namespace bdpt {

struct DaeScene {
  std::vector<int32_t> prim_type;
  std::vector<double> prim_geom;   // 18 per primitive (bdpt_scene_desc layout)
  std::vector<int32_t> prim_mat;
  std::vector<bdpt_material> mats;
  std::vector<bdpt_light> lights;
  bdpt_camera cam;
  // camera state beyond the ABI (for the scene dump)
  double target[3], phi, theta, r, ar, screen_dist;
  int screen_w, screen_h;
  int n_tris, n_sphs;
  bdpt_scene_desc desc() const;
};

// Loads `path`; width/height > 0 apply Camera::set_screen_size (the CLI's -r W H, whose FOV
// follows the frame size with screenDist fixed at 800x600). Returns BDPT_OK or an error code
// with the message in err.
int load_dae(const char* path, int width, int height, DaeScene& out, std::string& err);

// Writes the scene in the JSON dump format of tests/golden/scenes/*.json.
int dump_scene_json(const DaeScene& s, const char* path, std::string& err);

}  // namespace bdpt
