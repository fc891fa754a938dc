// bdpt_scene.h — host-side scene preparation for the device path.
//
// Replaces RaytracedRenderer::build_accel (raytraced_renderer.cpp:350-374) + BVHAccel's
// construct_bvh (bvh.cpp:51-129): the BVH topology is the reference's (longest centroid axis,
// spatial midpoint, leaf <= 4, stable partition, built in fp64 on the reference's bboxes), then
// flattened for HBM:
//   nodes : per tree width W (2 and 4, the second collapsed from the first; same leaves), one
//           node_bytes(W) record per node = the children's fp32 AABBs (outward-rounded and padded
//           by 2^-16 of the box scale, so the fp32 slab test is conservative) + child refs; the
//           layouts are at node_step (bdpt_core.h)
//   geom  : 48 B per primitive reference in DFS leaf order (triangle p0,e1,e2 | sphere c,r); a
//           primitive referenced from two leaves (spatial splits) has a record at both positions
//   shade : 48 B per primitive reference (triangle n1,n2,n3 | sphere flag) + material id
//   prim_ref: DFS position -> scene primitive index
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "bdpt/bdpt.h"
#include "bdpt_core.h"

namespace bdpt {

struct HostBvh {
  std::vector<float> nodes;   // 4 * node_f4(W) floats per node
  int root = 0;               // root child reference (node index or encoded leaf)
  int n_top = 0;              // leading nodes in BFS order (LDS treelet candidates)
  int depth = 0;              // node levels below the root
};

struct HostScene {
  HostBvh bvh2, bvh4;         // the device tree with 2 / 4 children per node
  const HostBvh& tree(int W) const { return W == 4 ? bvh4 : bvh2; }
  std::vector<float> geom;    // 12 floats per prim
  std::vector<float> shade;   // 12 floats per prim
  std::vector<int32_t> prim_ref;    // device DFS position -> scene primitive index
  std::vector<int32_t> leaf_refs;   // every leaf of the device tree (encoded refs, DFS order)
  std::vector<int32_t> ref_order;   // the reference tree's DFS leaf order (scene indices)
  std::vector<DMat> mats;
  std::vector<DLight> lights;
  DCam cam;
  int depth = 0;              // reference BVH depth (root = 0)
  int ref_nodes = 0;          // node count of the reference binary tree
  int dev_nodes = 0, dev_depth = 0;   // the device tree (SAH by default), binary
  int nprim = 0;
  // environment light (bdpt_scene_desc.envmap): EnvironmentLight::init's tables
  // (environment_light.cpp:18-62) built in fp64 and rounded, and the emission sphere
  int env_light = -1;         // index in `lights`, -1 = none
  int env_w = 0, env_h = 0;
  std::vector<float> env;     // marginal_y[h] | conds_y[w*h] | pdf_envmap[w*h] | rgb[w*h*3] |
                              // guide tables (int32 bits): marginal[gm+1] | per row conditional[h*(gc+1)]
  int env_gm = 0, env_gc = 0; // guide-table cells (powers of two)
  float env_c[3] = {0, 0, 0}, env_rad = 0;
};

constexpr int kTopNodes = 1024;
// Spatial splits in the device tree (SBVH, bdpt_scene.cpp SahBuilder): tried at a node whose best
// object split leaves children overlapping by more than kSbvhAlpha x the root's surface area, up
// to kSbvhBudget x n extra primitive references, in scenes of >= kSbvhMinPrims primitives (the
// flat-list and all-in-LDS scenes stay unsplit). kSbvhAlpha 0 = off. Run-time A/B: BDPT_SBVH=alpha,
// BDPT_SBVH_BUDGET=fraction.
constexpr int kSbvhMinPrims = 256;
constexpr double kSbvhAlpha = 1e-5;
constexpr double kSbvhBudget = 0.3;

// LM 3's flat list as one run of primitives: when the device tree's leaves, in DFS order, hold
// primitives 0, 1, ..., n-1 consecutively (the builder emits them so), returns n and sets *sph to
// the sphere mask of those n (n <= 32); else 0 (the kernels then walk the leaf list).
inline int flat_prims(const HostScene& hs, uint32_t* sph) {
  *sph = 0;
  int next = 0;
  for (int32_t r : hs.leaf_refs) {
    const uint32_t u = ~(uint32_t)r;
    const int st = (int)(u >> 7), cnt = (int)(u & 7u), m = (int)((u >> 3) & 15u);
    if (st != next || next + cnt > 32) return 0;
    *sph |= (uint32_t)m << st;
    next += cnt;
  }
  return next;
}

// Returns BDPT_OK or an error code; err receives a message.
// pt: the scene is for the unidirectional PathTracer (microfacet materials allowed).
int build_host_scene(const bdpt_scene_desc* d, HostScene& out, std::string& err, bool pt = false);

}  // namespace bdpt
