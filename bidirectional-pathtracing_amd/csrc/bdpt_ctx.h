// bdpt_ctx.h — the device context behind the C-ABI handle (shared by the kernels' TU,
// bdpt_hip.hip, and the multi-GPU frame reduce, bdpt_reduce.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "bdpt/bdpt.h"
#include "bdpt_core.h"
#include "bdpt_err.h"
#include "bdpt_scene.h"

namespace bdpt {

// bdpt_last_error() text: bdpt_err.h

struct Ctx {
  HostScene hs;
  bool ext = false;            // environment light or Russian roulette: the EXT kernels
  bdpt_params prm;
  int device = 0;
  hipStream_t own = nullptr, stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  float* d_nodes2 = nullptr;   // HostScene::bvh2 / bvh4
  float* d_nodes4 = nullptr;
  float* d_geom = nullptr;
  float* d_shade = nullptr;
  DMat* d_mats = nullptr;
  DLight* d_lights = nullptr;
  int* d_prim_ref = nullptr;
  int* d_leaves = nullptr;     // HostScene::leaf_refs (LM 3 staging source)
  float* d_env = nullptr;      // HostScene::env (environment light tables + map)
  int* d_count = nullptr;      // PathTracer::sampleCountBuffer (W*H)
  unsigned* d_work8 = nullptr;  // 8 per-XCD-group ticket counters, 128 B apart
  bool pt = false;             // bdpt_params.integrator == BDPT_INTEGRATOR_PT
  float* d_eye = nullptr;
  float* d_light = nullptr;
  float* d_sample = nullptr;
  // [0..7] counters, [12..14] environment-table reads, [15] tickets, [16..31] phase profile,
  // [32..47] lane-use profile (BDPT_PHASE_PROF builds)
  static constexpr int kStatSlots = 48;
  unsigned long long* d_stats = nullptr;
  // Tile-block lists of bdpt_render: a ring of pinned staging + device buffers, each slot reused
  // only after the event recorded behind the launch that read it, so back-to-back tile renders
  // (raytrace_tile / raytrace_pixel callers) never wait for the GPU.
  struct BlockSlot {
    int4* h = nullptr;
    int4* d = nullptr;
    size_t cap = 0;
    hipEvent_t done = nullptr;
    bool pending = false;
  };
  static constexpr int kBlockSlots = 4;
  BlockSlot blk[kBlockSlots];
  int blk_next = 0;
  // Every entry point locks the ctx: the reference drives raytrace_pixel / raytrace_tile from N
  // worker threads (raytraced_renderer.cpp:325-327,610-615); calls on one ctx are serialised here.
  std::recursive_mutex mu;
  // Diagnostics read once at bdpt_create (BDPT_LDS_MODE, BDPT_NTOP_MAX, BDPT_BLOCK_MAJOR,
  // BDPT_XCD_GROUPS): -1 = not set.
  int env_lds_mode = -1, env_ntop_max = -1, block_major = 1, xcd = 0;
  int last_lm = -1;            // LDS mode of the last BDPT / PathTracer launch
  int maxv = 5;
  int ncu = 256;
  size_t npix = 0;
};

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      ::bdpt::g_err = std::string(#x) + ": " + hipGetErrorString(e_);               \
      return BDPT_E_DEVICE;                                                         \
    }                                                                               \
  } while (0)

// The scene as a kernel of LDS mode LM sees it (its tree width: lm_width(LM)).
inline SceneView view_of(const Ctx* c, int LM) {
  SceneView S;
  const int W = lm_width(LM);
  // the device copy of the very tree the kernels of this width traverse (hs.tree(W))
  S.nodes = (const float4*)(&c->hs.tree(W) == &c->hs.bvh4 ? c->d_nodes4 : c->d_nodes2);
  S.geom = (const float4*)c->d_geom;
  S.shade = (const float4*)c->d_shade;
  S.mats = c->d_mats;
  S.lights = c->d_lights;
  S.nlights = (int)c->hs.lights.size();
  S.root = c->hs.tree(W).root;
  S.lnodes = nullptr;
  S.lgeom = nullptr;
  S.lshade = nullptr;
  S.lleaves = c->d_leaves;
  S.nleaves = (int)c->hs.leaf_refs.size();
  S.fn = flat_prims(c->hs, &S.fsph);
  S.ntop = 0;
  S.lstack = nullptr;
  S.cam = c->hs.cam;
  const HostScene& hs = c->hs;
  S.env.light = hs.env_light;
  S.env.w = hs.env_w;
  S.env.h = hs.env_h;
  const size_t np = (size_t)hs.env_w * hs.env_h;
  S.env.marg = c->d_env;
  S.env.cond = c->d_env ? c->d_env + hs.env_h : nullptr;
  S.env.pdf = c->d_env ? c->d_env + hs.env_h + np : nullptr;
  S.env.rgb = c->d_env ? c->d_env + hs.env_h + 2 * np : nullptr;
  S.env.gmarg = c->d_env ? (const int*)(c->d_env + hs.env_h + 5 * np) : nullptr;
  S.env.gcond = S.env.gmarg ? S.env.gmarg + hs.env_gm + 1 : nullptr;
  S.env.gm = hs.env_gm;
  S.env.gc = hs.env_gc;
  S.env.cx = hs.env_c[0]; S.env.cy = hs.env_c[1]; S.env.cz = hs.env_c[2];
  S.env.rad = hs.env_rad;
  return S;
}

}  // namespace bdpt
