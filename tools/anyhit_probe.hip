// Probe (diagnostics, not the product): how fast do the megakernel's connection rays trace in a
// kernel of their own? k_probe_any runs trace_any (bdpt_core.h, the product's any-hit traversal)
// over a host-supplied array of rays (o, d, tmin, tmax) — the north star's own connection rays,
// dumped by the CPU build (tools/anyhit_probe.py) — at 4 or 8 waves per SIMD, with the tree in HBM
// (LM 0) or its BFS treelet in LDS (LM 2), each lane taking rays grid-stride as a flush takes 64.
// Build (tools/anyhit_probe.py does it): hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -fno-slp-vectorize -shared -fPIC -Iinclude -Ibidirectional-pathtracing_amd/csrc
//   tools/anyhit_probe.hip bidirectional-pathtracing_amd/csrc/bdpt_scene.cpp -o tools/bin/libanyhit_probe.so
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

#include "bdpt_core.h"
#include "bdpt_scene.h"

using namespace bdpt;

constexpr int kProbeBlock = 1024;   // = kLdsStackStride: the LDS stack slots' lane stride
static_assert(kProbeBlock == kLdsStackStride, "probe block = LDS stack stride");

template <int LM, int WPE>
__global__ __launch_bounds__(kProbeBlock, WPE) void k_probe_any(SceneView S, const float* rays, int n, int* out,
                                                                int ntop) {
  extern __shared__ __align__(16) unsigned char smem[];
  if (LM == 2) {
    S.lstack = (int*)smem;
    float4* sc = (float4*)(smem + (size_t)kLdsStack * kProbeBlock * sizeof(int));
    const int n4 = node_f4(lm_width(2)) * ntop;
    for (int k = threadIdx.x; k < n4; k += blockDim.x) sc[k] = S.nodes[k];
    __syncthreads();
    S.lnodes = sc;
    S.ntop = ntop;
  }
  Counters c = {};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const float* r = rays + 8 * i;
    const bool h = trace_any<LM, kConnStack>(S, mk3(r[0], r[1], r[2]), mk3(r[3], r[4], r[5]), r[6], r[7], c);
    out[i] = h ? 1 : 0;
  }
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "probe: %s: %s\n", #x, hipGetErrorString(e_));                   \
      return -1;                                                                       \
    }                                                                                  \
  } while (0)

template <int LM, int WPE>
static int run(const HostScene& hs, const float* d_rays, int n, int* d_out, int reps, float* ms, int* occ, int* ntop_out) {
  const HostBvh& T = hs.tree(lm_width(LM));
  float4 *d_nodes = nullptr, *d_geom = nullptr;
  CK(hipMalloc(&d_nodes, T.nodes.size() * sizeof(float)));
  CK(hipMalloc(&d_geom, hs.geom.size() * sizeof(float)));
  CK(hipMemcpy(d_nodes, T.nodes.data(), T.nodes.size() * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_geom, hs.geom.data(), hs.geom.size() * sizeof(float), hipMemcpyHostToDevice));
  SceneView S = {};
  S.nodes = d_nodes;
  S.geom = d_geom;
  S.root = T.root;
  // LDS: stack slots + as many treelet nodes as fit in the block's share of 160 KB
  const size_t stack = (size_t)kLdsStack * kProbeBlock * sizeof(int);
  const int blocks_per_cu = WPE * 4 * 64 / kProbeBlock;
  const size_t share = 160 * 1024 / blocks_per_cu - 512;
  int ntop = 0;
  if (LM == 2) ntop = (int)std::min<size_t>((size_t)T.n_top, (share - stack) / node_bytes(lm_width(2)));
  const size_t lds = LM == 2 ? stack + (size_t)ntop * node_bytes(lm_width(2)) : 0;
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_probe_any<LM, WPE>, kProbeBlock, lds));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int grid = std::max(1, per_cu) * pr.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_probe_any<LM, WPE>), dim3(grid), dim3(kProbeBlock), lds, 0, S, d_rays, n, d_out, ntop);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((k_probe_any<LM, WPE>), dim3(grid), dim3(kProbeBlock), lds, 0, S, d_rays, n, d_out, ntop);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(ms, e0, e1));
  *ms /= reps;
  *occ = per_cu * kProbeBlock / 64 / 4;
  *ntop_out = ntop;
  (void)hipFree(d_nodes);
  (void)hipFree(d_geom);
  return 0;
}

// lm 0 / 2, wpe 4 / 8 (waves per SIMD asked of the compiler); returns the number of occluded rays,
// ms = mean kernel time over reps, occ = resident waves per SIMD, ntop = treelet nodes in LDS
extern "C" int probe_any(const bdpt_scene_desc* d, const float* rays, int n, int lm, int wpe, int reps, float* ms,
                         int* occ, int* ntop) {
  HostScene hs;
  std::string err;
  if (build_host_scene(d, hs, err) != BDPT_OK) { fprintf(stderr, "probe: %s\n", err.c_str()); return -1; }
  float* d_rays = nullptr;
  int* d_out = nullptr;
  CK(hipMalloc(&d_rays, (size_t)n * 8 * sizeof(float)));
  CK(hipMalloc(&d_out, (size_t)n * sizeof(int)));
  CK(hipMemcpy(d_rays, rays, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice));
  int rc;
  if (lm == 2) rc = wpe == 8 ? run<2, 8>(hs, d_rays, n, d_out, reps, ms, occ, ntop) : run<2, 4>(hs, d_rays, n, d_out, reps, ms, occ, ntop);
  else rc = wpe == 8 ? run<0, 8>(hs, d_rays, n, d_out, reps, ms, occ, ntop) : run<0, 4>(hs, d_rays, n, d_out, reps, ms, occ, ntop);
  if (rc) return rc;
  std::vector<int> out(n);
  CK(hipMemcpy(out.data(), d_out, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  (void)hipFree(d_rays);
  (void)hipFree(d_out);
  long long occl = 0;
  for (int v : out) occl += v;
  return (int)occl;
}
