// Probe (diagnostics, not the product): the walk's closest-hit queries in a kernel of their own,
// traced by the product's trace_closest (bdpt_core.h) or by trace_closest_coop (lane donation: idle
// lanes take over pending subtrees of the lanes still tracing), to measure what the donation buys
// before it goes into the megakernel. The rays (o, d, tmin, tmax) are the closest-hit queries of a
// CPU-build render of the stand-in (tools/closest_probe.py). Every lane takes rays grid-stride in a
// wave-uniform loop (the coop form needs the whole wave in every call); LM 2 stages the BFS
// treelet and the LDS stack slots as the megakernel does; 4 waves per SIMD.
// Build (tools/closest_probe.py does it): hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//   -fno-slp-vectorize -shared -fPIC -Iinclude -Ibidirectional-pathtracing_amd/csrc
//   tools/closest_probe.hip bidirectional-pathtracing_amd/csrc/bdpt_scene.cpp -o tools/bin/libclosest_probe.so
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

#include "bdpt_core.h"
#include "bdpt_scene.h"

using namespace bdpt;

// The cooperative traversals (measured here in round 6, not in the product: DESIGN.md §5). They were
// in bdpt_core.h while measured; the megakernel integration lost 9 % (the walk loop made wave-uniform
// for the helpers doubled the spills) and the donation itself cut the wave-level node steps by only
// 16 % (the tail is a sequential descent, not a set of pending subtrees).
namespace bdpt {
// ------------------------------------------------------------------------------------------------
// Cooperative traversal (lane donation). The wave pays for its slowest lane: a walk query takes ~6
// node steps on average but the wave iterates ~27 (the tail of the per-query distribution,
// DESIGN.md §5). Here the lanes whose query has finished take over pending subtrees of the lanes
// still tracing: whenever at most kCoopThresh lanes still trace, every tracing lane with a non-empty
// stack hands its top entry (with its ray and its current best distance) to an idle lane, which
// traverses that subtree with a stack of its own and merges its closest hit back into the owner's
// (a readlane per field). The candidate set of every query is unchanged and the merge keeps the
// tie rule (smaller t, then the larger reference-tree key), so the result is the same bits as
// trace_closest. Every lane of the wave must call it together (`have` = this lane has a query).
constexpr int kCoopThresh = 16;   // donate once at most this many lanes still trace
constexpr bool kCoopBottom = true;  // donate the oldest stack entry (the largest pending subtree)
constexpr int kCoopPasses = 2;      // donation passes per leaf round

BDPT_HD bool hit_better(float t, int key, float bt, int bkey) { return t < bt || (t == bt && key > bkey); }

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ int coop_bperm(int src, int v) { return __builtin_amdgcn_ds_bpermute(src << 2, v); }
__device__ __forceinline__ float coop_bperm(int src, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(v)));
}
__device__ __forceinline__ int lanes_below_ull(unsigned long long m) {   // set bits of m below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ int coop_readlane(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float coop_readlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
// position of the k-th (0-based) set bit of m (k < popcount(m))
__device__ __forceinline__ int select_kth(unsigned long long m, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int cnt = __popcll(m & ((1ull << w) - 1));
    if (k >= cnt) { k -= cnt; m >>= w; pos += w; }
  }
  return pos;
}
#endif

template <int LM = 0, int K = 0, int THRESH = kCoopThresh, bool BOT = kCoopBottom, int PASSES = kCoopPasses>
BDPT_HD bool trace_closest_coop(const SceneView& S, f3 o, f3 d, float tmin, float tmax, Hit& h, Counters& c,
                                bool have) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (!have) return false;   // the host build runs one lane: nothing to share
  return trace_closest<LM, K>(S, o, d, tmin, tmax, h, c);
#else
  static_assert(spec_trav(LM), "the cooperative traversal is the speculative while-while of LM 0 / 2");
  const int lane = (int)__lane_id();
  RayInv r = make_rayinv(o, d);   // the ray this lane works on (its own, or a borrowed one)
  float wtmin = tmin;
  Hit w;                          // the closest hit of the current work unit
  w.t = tmax; w.prim = -1; w.key = -1; w.b1 = 0; w.b2 = 0;
  Hit mine = w;                   // this lane's own query, with its helpers' hits merged in
  int stack_mem[kStackMax];
  TravStack<K, BOT> stk(stack_mem, LM == 2 ? lane_stack(S) : nullptr);
  int ref = have ? S.root : kTravDone;
  int pend = 0;
  int owner = have ? lane : -1;   // whose query the current work unit belongs to; -1 = idle
  if (have) c.closest++;
  float4 a0, a1, a2;
  auto test_leaf = [&](int lf) {
    const int st = leaf_start(lf), cnt = leaf_count(lf), sm = leaf_sph_mask(lf);
    a0 = ld_geom<LM>(S, 3 * st); a1 = ld_geom<LM>(S, 3 * st + 1); a2 = ld_geom<LM>(S, 3 * st + 2);
    for (int k = 0; k < cnt; k++) {
      BDPT_LANE_PROF(c, LP_CPRIM);
      const int pi = st + k;
      float t, b1 = 0, b2 = 0;
      bool ok;
      int key;
      const float4 g0 = a0, g1 = a1, g2 = a2;
      const int nx = 3 * (k + 1 < cnt ? pi + 1 : pi);
      a0 = ld_geom<LM>(S, nx); a1 = ld_geom<LM>(S, nx + 1); a2 = ld_geom<LM>(S, nx + 2);
      if ((sm >> k) & 1) {
        c.sphs++;
        ok = sph_test(g0, r.o, r.d, wtmin, w.t, &t);
        key = __float_as_int(g1.x);
      } else {
        c.tris++;
        ok = tri_test(g0, g1, g2, r.o, r.d, wtmin, w.t, &t, &b1, &b2);
        key = __float_as_int(g2.y);
      }
      if (ok && (t < w.t || key > w.key)) {
        w.t = t; w.prim = pi; w.key = key; w.b1 = b1; w.b2 = b2;
      }
    }
  };
  for (;;) {
    // speculative while-while over the current work units (as trace_closest)
    while (ref >= 0) {
      BDPT_LANE_PROF(c, LP_CNODE);
      ref = node_step<K, LM, kClosestOrd>(S, r, ref, wtmin, w.t, stk, c);
      if (ref < 0 && ref != kTravDone && pend == 0) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
      if (wave_count(pend == 0 && ref >= 0) == 0) break;
    }
    while (pend != 0) {
      test_leaf(pend);
      pend = 0;
      if (ref < 0 && ref != kTravDone) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
    }
    // work units that ended: an own unit merges into `mine`, a borrowed one into its owner's
    const bool fin = owner >= 0 && ref == kTravDone;
    const bool own_working = owner == lane && !fin;
    if (fin && owner == lane && w.prim >= 0 && hit_better(w.t, w.key, mine.t, mine.key)) mine = w;
    unsigned long long mm = __ballot(fin && owner != lane && w.prim >= 0);
    while (mm) {
      const int hl = __builtin_ctzll(mm);
      mm &= mm - 1;
      const int ow = coop_readlane(owner, hl), hk = coop_readlane(w.key, hl), hp = coop_readlane(w.prim, hl);
      const float ht = coop_readlane(w.t, hl), hb1 = coop_readlane(w.b1, hl), hb2 = coop_readlane(w.b2, hl);
      if (lane == ow) {
        if (own_working) {   // still tracing its own query: the hit also tightens its pruning
          if (hit_better(ht, hk, w.t, w.key)) { w.t = ht; w.key = hk; w.prim = hp; w.b1 = hb1; w.b2 = hb2; }
        } else if (hit_better(ht, hk, mine.t, mine.key)) {
          mine.t = ht; mine.key = hk; mine.prim = hp; mine.b1 = hb1; mine.b2 = hb2;
        }
      }
    }
    if (fin) owner = -1;
    const unsigned long long mW = __ballot(owner >= 0);
    if (mW == 0) break;
    if (__popcll(mW) > THRESH) continue;
    // donation: each tracing lane with a pending subtree hands a stack entry (the oldest with BOT,
    // else the newest) to an idle lane, PASSES times per round
#pragma unroll 1
    for (int pass = 0; pass < PASSES; pass++) {
    const bool can = owner >= 0 && (BOT ? stk.can_pop_bottom() : stk.size() > 0);
    const unsigned long long mI = __ballot(owner < 0), mD = __ballot(can);
    if (mI == 0 || mD == 0) break;
    const int ki = lanes_below_ull(mI), kd = lanes_below_ull(mD);
    const bool take = owner < 0 && ki < __popcll(mD);
    const bool give = can && kd < __popcll(mI);
    int e = kTravDone;
    if (give) {
      if (BOT) stk.pop_bottom(e);
      else stk.pop(e);
    }
    const int src = take ? select_kth(mD, ki) : lane;
    const int e_in = coop_bperm(src, e), ow_in = coop_bperm(src, owner);
    const float t_in = coop_bperm(src, w.t), tmin_in = coop_bperm(src, wtmin);
    RayInv rin;
    rin.o = mk3(coop_bperm(src, r.o.x), coop_bperm(src, r.o.y), coop_bperm(src, r.o.z));
    rin.d = mk3(coop_bperm(src, r.d.x), coop_bperm(src, r.d.y), coop_bperm(src, r.d.z));
    rin.inv = mk3(coop_bperm(src, r.inv.x), coop_bperm(src, r.inv.y), coop_bperm(src, r.inv.z));
    rin.oi = mk3(coop_bperm(src, r.oi.x), coop_bperm(src, r.oi.y), coop_bperm(src, r.oi.z));
    const int nn = coop_bperm(src, r.nx | (r.ny << 8) | (r.nz << 16));
    if (take) {
      r = rin;
      r.nx = nn & 0xff; r.ny = (nn >> 8) & 0xff; r.nz = (nn >> 16) & 0xff;
      wtmin = tmin_in;
      w.t = t_in; w.prim = -1; w.key = -1; w.b1 = 0; w.b2 = 0;
      owner = ow_in;
      stk.clear();
      if (e_in >= 0) { ref = e_in; pend = 0; }
      else { pend = e_in; ref = kTravDone; }   // a leaf entry: tested in the next leaf phase
    }
    }
  }
  h = mine;
  if (h.prim >= 0) c.hits++;
  return h.prim >= 0;
#endif
}

// Any hit, cooperatively (as trace_closest_coop): a borrowed subtree that holds a hit answers its
// owner's query; a work unit whose owner's query is answered is dropped.
template <int LM = 0, int K = 0, int THRESH = kCoopThresh, bool BOT = kCoopBottom, int PASSES = kCoopPasses>
BDPT_HD bool trace_any_coop(const SceneView& S, f3 o, f3 d, float tmin, float tmax, Counters& c, bool have) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (!have) return false;
  return trace_any<LM, K>(S, o, d, tmin, tmax, c);
#else
  static_assert(spec_trav(LM), "the cooperative traversal is the speculative while-while of LM 0 / 2");
  const int lane = (int)__lane_id();
  RayInv r = make_rayinv(o, d);
  float wtmin = tmin, wtmax = tmax;
  bool whit = false;   // the current work unit found a hit
  bool mine = false;   // this lane's own query is answered (occluded)
  int stack_mem[kStackMax];
  TravStack<K, BOT> stk(stack_mem, LM == 2 ? lane_stack(S) : nullptr);
  int ref = have ? S.root : kTravDone;
  int pend = 0;
  int owner = have ? lane : -1;
  if (have) c.shadow++;
  float4 a0, a1, a2;
  auto test_leaf = [&](int lf) -> bool {
    const int st = leaf_start(lf), cnt = leaf_count(lf), sm = leaf_sph_mask(lf);
    a0 = ld_geom<LM>(S, 3 * st); a1 = ld_geom<LM>(S, 3 * st + 1); a2 = ld_geom<LM>(S, 3 * st + 2);
    for (int k = 0; k < cnt; k++) {
      BDPT_LANE_PROF(c, LP_APRIM);
      const int pi = st + k;
      float t, b1, b2;
      bool ok;
      const float4 g0 = a0, g1 = a1, g2 = a2;
      const int nx = 3 * (k + 1 < cnt ? pi + 1 : pi);
      a0 = ld_geom<LM>(S, nx); a1 = ld_geom<LM>(S, nx + 1); a2 = ld_geom<LM>(S, nx + 2);
      if ((sm >> k) & 1) {
        c.sphs++;
        ok = sph_test(g0, r.o, r.d, wtmin, wtmax, &t);
      } else {
        c.tris++;
        ok = tri_test(g0, g1, g2, r.o, r.d, wtmin, wtmax, &t, &b1, &b2);
      }
      if (ok) return true;
    }
    return false;
  };
  for (;;) {
    while (ref >= 0) {
      BDPT_LANE_PROF(c, LP_ANODE);
      ref = node_step<K, LM, kAnyOrd>(S, r, ref, wtmin, wtmax, stk, c);
      if (ref < 0 && ref != kTravDone && pend == 0) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
      if (wave_count(pend == 0 && ref >= 0) == 0) break;
    }
    while (pend != 0) {
      if (test_leaf(pend)) { whit = true; ref = kTravDone; pend = 0; break; }
      pend = 0;
      if (ref < 0 && ref != kTravDone) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
    }
    const bool fin = owner >= 0 && ref == kTravDone;
    if (fin && owner == lane && whit) mine = true;
    unsigned long long mm = __ballot(fin && owner != lane && whit);
    while (mm) {
      const int hl = __builtin_ctzll(mm);
      mm &= mm - 1;
      if (lane == coop_readlane(owner, hl)) mine = true;
    }
    // a unit still running whose owner's query is answered stops (its own lane's included)
    const bool answered = coop_bperm(owner < 0 ? lane : owner, (int)mine) != 0;
    if (fin || (owner >= 0 && answered)) { owner = -1; ref = kTravDone; pend = 0; }
    const unsigned long long mW = __ballot(owner >= 0);
    if (mW == 0) break;
    if (__popcll(mW) > THRESH) continue;
#pragma unroll 1
    for (int pass = 0; pass < PASSES; pass++) {
    const bool can = owner >= 0 && (BOT ? stk.can_pop_bottom() : stk.size() > 0);
    const unsigned long long mI = __ballot(owner < 0), mD = __ballot(can);
    if (mI == 0 || mD == 0) break;
    const int ki = lanes_below_ull(mI), kd = lanes_below_ull(mD);
    const bool take = owner < 0 && ki < __popcll(mD);
    const bool give = can && kd < __popcll(mI);
    int e = kTravDone;
    if (give) {
      if (BOT) stk.pop_bottom(e);
      else stk.pop(e);
    }
    const int src = take ? select_kth(mD, ki) : lane;
    const int e_in = coop_bperm(src, e), ow_in = coop_bperm(src, owner);
    const float tmax_in = coop_bperm(src, wtmax), tmin_in = coop_bperm(src, wtmin);
    RayInv rin;
    rin.o = mk3(coop_bperm(src, r.o.x), coop_bperm(src, r.o.y), coop_bperm(src, r.o.z));
    rin.d = mk3(coop_bperm(src, r.d.x), coop_bperm(src, r.d.y), coop_bperm(src, r.d.z));
    rin.inv = mk3(coop_bperm(src, r.inv.x), coop_bperm(src, r.inv.y), coop_bperm(src, r.inv.z));
    rin.oi = mk3(coop_bperm(src, r.oi.x), coop_bperm(src, r.oi.y), coop_bperm(src, r.oi.z));
    const int nn = coop_bperm(src, r.nx | (r.ny << 8) | (r.nz << 16));
    if (take) {
      r = rin;
      r.nx = nn & 0xff; r.ny = (nn >> 8) & 0xff; r.nz = (nn >> 16) & 0xff;
      wtmin = tmin_in;
      wtmax = tmax_in;
      whit = false;
      owner = ow_in;
      stk.clear();
      if (e_in >= 0) { ref = e_in; pend = 0; }
      else { pend = e_in; ref = kTravDone; }
    }
    }
  }
  return mine;
#endif
}


// Two queries per lane in one traversal loop (round 6 probe): a lane traces its ray A, then at once
// its ray B, without waiting for the wave between them, so the wave iterates max over lanes of
// (steps A + steps B) instead of max(steps A) + max(steps B). This is what tracing a lane's eye and
// light walk rays together would buy.
template <int LM = 0, int K = 0, bool ANY = false>
__device__ void trace_dual(const SceneView& S, const float* ra, const float* rb, bool has_a, bool has_b, Hit& ha,
                           Hit& hb, Counters& c) {
  RayInv r;
  float wtmin = 0;
  Hit w;
  w.t = 0; w.prim = -1; w.key = -1; w.b1 = 0; w.b2 = 0;
  ha = w; hb = w;
  int stack_mem[kStackMax];
  TravStack<K> stk(stack_mem, LM == 2 ? lane_stack(S) : nullptr);
  int ref = kTravDone, pend = 0, phase = 2;
  auto start = [&](const float* q, int ph) {
    r = make_rayinv(mk3(q[0], q[1], q[2]), mk3(q[3], q[4], q[5]));
    wtmin = q[6];
    w.t = q[7]; w.prim = -1; w.key = -1; w.b1 = 0; w.b2 = 0;
    stk.clear();
    ref = S.root;
    pend = 0;
    phase = ph;
    if (ANY) c.shadow++;
    else c.closest++;
  };
  if (has_a) start(ra, 0);
  else if (has_b) start(rb, 1);
  float4 a0, a1, a2;
  bool found = false;   // any hit: the current ray is occluded
  auto test_leaf = [&](int lf) -> bool {
    const int st = leaf_start(lf), cnt = leaf_count(lf), sm = leaf_sph_mask(lf);
    a0 = ld_geom<LM>(S, 3 * st); a1 = ld_geom<LM>(S, 3 * st + 1); a2 = ld_geom<LM>(S, 3 * st + 2);
    for (int k = 0; k < cnt; k++) {
      BDPT_LANE_PROF(c, ANY ? LP_APRIM : LP_CPRIM);
      const int pi = st + k;
      float t, b1 = 0, b2 = 0;
      bool ok;
      int key;
      const float4 g0 = a0, g1 = a1, g2 = a2;
      const int nx = 3 * (k + 1 < cnt ? pi + 1 : pi);
      a0 = ld_geom<LM>(S, nx); a1 = ld_geom<LM>(S, nx + 1); a2 = ld_geom<LM>(S, nx + 2);
      if ((sm >> k) & 1) {
        c.sphs++;
        ok = sph_test(g0, r.o, r.d, wtmin, w.t, &t);
        key = __float_as_int(g1.x);
      } else {
        c.tris++;
        ok = tri_test(g0, g1, g2, r.o, r.d, wtmin, w.t, &t, &b1, &b2);
        key = __float_as_int(g2.y);
      }
      if (ANY && ok) return true;
      if (ok && (t < w.t || key > w.key)) {
        w.t = t; w.prim = pi; w.key = key; w.b1 = b1; w.b2 = b2;
      }
    }
    return false;
  };
  for (;;) {
    while (ref >= 0) {
      BDPT_LANE_PROF(c, ANY ? LP_ANODE : LP_CNODE);
      ref = node_step<K, LM, ANY ? kAnyOrd : kClosestOrd>(S, r, ref, wtmin, w.t, stk, c);
      if (ref < 0 && ref != kTravDone && pend == 0) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
      if (wave_count(pend == 0 && ref >= 0) == 0) break;
    }
    while (pend != 0) {
      if (test_leaf(pend)) { found = true; ref = kTravDone; pend = 0; break; }
      pend = 0;
      if (ref < 0 && ref != kTravDone) {
        pend = ref;
        if (!stk.pop(ref)) ref = kTravDone;
      }
    }
    if (phase < 2 && ref == kTravDone) {   // this ray is done: record it, start the other
      if (ANY) w.prim = found ? 1 : -1;
      found = false;
      if (phase == 0) {
        ha = w;
        if (has_b) start(rb, 1);
        else phase = 2;
      } else {
        hb = w;
        phase = 2;
      }
    }
    if (wave_count(phase < 2) == 0) break;
  }
}
}  // namespace bdpt

constexpr int kProbeBlock = 1024;   // = kLdsStackStride: the LDS stack slots' lane stride
static_assert(kProbeBlock == kLdsStackStride, "probe block = LDS stack stride");

// coop configurations: 0 = plain; 1.. = (threshold, bottom entries, passes) below
template <int CFG> struct CoopCfg;
template <> struct CoopCfg<1> { static constexpr int T = 16; static constexpr bool BOT = false; static constexpr int P = 1; };
template <> struct CoopCfg<2> { static constexpr int T = 16; static constexpr bool BOT = true; static constexpr int P = 2; };
template <> struct CoopCfg<3> { static constexpr int T = 32; static constexpr bool BOT = true; static constexpr int P = 2; };
template <> struct CoopCfg<4> { static constexpr int T = 48; static constexpr bool BOT = true; static constexpr int P = 4; };
template <> struct CoopCfg<5> { static constexpr int T = 64; static constexpr bool BOT = true; static constexpr int P = 4; };
template <> struct CoopCfg<6> { static constexpr int T = 32; static constexpr bool BOT = false; static constexpr int P = 4; };
constexpr const char* kCfgName[] = {"plain", "t16 top x1", "t16 bot x2", "t32 bot x2", "t48 bot x4", "t64 bot x4",
                                     "t32 top x4", "dual (2/lane)"};

template <int LM, int COOP, bool ANY>
__global__ __launch_bounds__(kProbeBlock, 4) void k_probe_closest(SceneView S, const float* rays, int n, int2* out,
                                                                  int ntop, unsigned long long* steps) {
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
  const long long stride = (long long)gridDim.x * blockDim.x;
  // wave-uniform loop: the wave runs while any of its lanes has a ray left
  const long long wave0 = (long long)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  if constexpr (COOP == 7) {
    // ray pairs (2 j, 2 j + 1) per lane, one traversal loop for both
    const long long np = (n + 1) / 2;
    for (long long j = (long long)blockIdx.x * blockDim.x + threadIdx.x, wb = wave0; wb < np; j += stride, wb += stride) {
      const long long ia = 2 * j, ib = 2 * j + 1;
      const bool ha_ = ia < n, hb_ = ib < n;
      Hit h1, h2;
      trace_dual<LM, ANY ? kConnStack : kWalkStack, ANY>(S, rays + 8 * (ha_ ? ia : 0), rays + 8 * (hb_ ? ib : 0), ha_, hb_, h1,
                                                          h2, c);
      if (ANY) {
        if (ha_) out[ia] = make_int2(0, h1.prim >= 0 ? 1 : -1);
        if (hb_) out[ib] = make_int2(0, h2.prim >= 0 ? 1 : -1);
      } else {
        if (ha_) out[ia] = h1.prim >= 0 ? make_int2(__float_as_int(h1.t), h1.key) : make_int2(0, -1);
        if (hb_) out[ib] = h2.prim >= 0 ? make_int2(__float_as_int(h2.t), h2.key) : make_int2(0, -1);
      }
    }
  } else {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x, wb = wave0; wb < n; i += stride, wb += stride) {
      const bool have = i < n;
      const float* r = rays + 8 * (have ? i : 0);
      Hit h;
      h.t = 0; h.key = -1;
      bool ok;
      if constexpr (ANY) {
        const f3 o = mk3(r[0], r[1], r[2]), d = mk3(r[3], r[4], r[5]);
        if constexpr (COOP > 0) {
          using Q = CoopCfg<COOP>;
          ok = trace_any_coop<LM, kConnStack, Q::T, Q::BOT, Q::P>(S, o, d, r[6], r[7], c, have);
        } else {
          ok = have && trace_any<LM, kConnStack>(S, o, d, r[6], r[7], c);
        }
        h.key = ok ? 1 : -1;
      } else if constexpr (COOP > 0 && COOP < 7) {
        using Q = CoopCfg<COOP>;
        ok = trace_closest_coop<LM, kWalkStack, Q::T, Q::BOT, Q::P>(S, mk3(r[0], r[1], r[2]), mk3(r[3], r[4], r[5]), r[6],
                                                                    r[7], h, c, have);
      } else {
        ok = false;
        if (have) ok = trace_closest<LM, kWalkStack>(S, mk3(r[0], r[1], r[2]), mk3(r[3], r[4], r[5]), r[6], r[7], h, c);
      }
      if (have) out[i] = ok ? make_int2(__float_as_int(h.t), h.key) : make_int2(0, -1);
    }
  }
  atomicAdd(steps, (unsigned long long)c.nodes);
#ifdef BDPT_PHASE_PROF
  // lane-use profile (bdpt_core.h BDPT_LANE_PROF): steps[1 + k] = wave-level iterations / active lanes
  for (int k = 0; k < 8; k++) atomicAdd(steps + 1 + k, (unsigned long long)c.lp[k]);
#endif
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "probe: %s: %s\n", #x, hipGetErrorString(e_));                   \
      return -1;                                                                       \
    }                                                                                  \
  } while (0)

template <int LM, int COOP, bool ANY>
static int run(const HostScene& hs, const float* d_rays, int n, int2* d_out, int reps, float* ms, int* ntop_out,
               unsigned long long* nodes) {
  const HostBvh& T = hs.tree(lm_width(LM));
  float4 *d_nodes = nullptr, *d_geom = nullptr;
  unsigned long long* d_steps = nullptr;
  CK(hipMalloc(&d_nodes, T.nodes.size() * sizeof(float)));
  CK(hipMalloc(&d_geom, hs.geom.size() * sizeof(float)));
  CK(hipMalloc(&d_steps, 9 * sizeof(unsigned long long)));
  CK(hipMemcpy(d_nodes, T.nodes.data(), T.nodes.size() * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_geom, hs.geom.data(), hs.geom.size() * sizeof(float), hipMemcpyHostToDevice));
  SceneView S = {};
  S.nodes = d_nodes;
  S.geom = d_geom;
  S.root = T.root;
  // LDS: stack slots + the treelet nodes that fit in one block's 160 KB (one 1024-lane block per CU)
  const size_t stack = (size_t)kLdsStack * kProbeBlock * sizeof(int);
  int ntop = 0;
  if (LM == 2) ntop = (int)std::min<size_t>((size_t)T.n_top, (160 * 1024 - 512 - stack) / node_bytes(lm_width(2)));
  const size_t lds = LM == 2 ? stack + (size_t)ntop * node_bytes(lm_width(2)) : 0;
  int per_cu = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_probe_closest<LM, COOP, ANY>, kProbeBlock, lds));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int grid = std::max(1, per_cu) * pr.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipMemset(d_steps, 0, 9 * sizeof(unsigned long long)));
  hipLaunchKernelGGL((k_probe_closest<LM, COOP, ANY>), dim3(grid), dim3(kProbeBlock), lds, 0, S, d_rays, n, d_out, ntop, d_steps);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(nodes, d_steps, 9 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((k_probe_closest<LM, COOP, ANY>), dim3(grid), dim3(kProbeBlock), lds, 0, S, d_rays, n, d_out, ntop, d_steps);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(ms, e0, e1));
  *ms /= reps;
  *ntop_out = ntop;
  (void)hipFree(d_nodes);
  (void)hipFree(d_geom);
  (void)hipFree(d_steps);
  return 0;
}

extern "C" const char* probe_cfg_name(int k) { return k >= 0 && k <= 7 ? kCfgName[k] : "?"; }

// lm 0 / 2, coop 0 (plain) / 1..6 (CoopCfg), any 0 (closest hit) / 1 (any hit); out = n x (t bits, reference key) (key -1 =
// no hit; any hit: key 1 = occluded); ms = mean kernel time
extern "C" int probe_closest(const bdpt_scene_desc* d, const float* rays, int n, int lm, int coop, int any, int reps,
                             float* ms, int* ntop, int* out, unsigned long long* nodes) {
  HostScene hs;
  std::string err;
  if (build_host_scene(d, hs, err) != BDPT_OK) { fprintf(stderr, "probe: %s\n", err.c_str()); return -1; }
  float* d_rays = nullptr;
  int2* d_out = nullptr;
  CK(hipMalloc(&d_rays, (size_t)n * 8 * sizeof(float)));
  CK(hipMalloc(&d_out, (size_t)n * sizeof(int2)));
  CK(hipMemcpy(d_rays, rays, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice));
  int rc;
#define RUN(L, C, A) run<L, C, A>(hs, d_rays, n, d_out, reps, ms, ntop, nodes)
#define RUNC(C, A) (lm == 2 ? RUN(2, C, A) : RUN(0, C, A))
#define RUNA(A)                                                                                       \
  (coop == 0 ? RUNC(0, A) : coop == 1 ? RUNC(1, A) : coop == 2 ? RUNC(2, A) : coop == 3 ? RUNC(3, A)   \
   : coop == 4 ? RUNC(4, A) : coop == 5 ? RUNC(5, A) : coop == 6 ? RUNC(6, A) : RUNC(7, A))
  rc = any ? RUNA(true) : RUNA(false);
#undef RUNA
#undef RUNC
#undef RUN
  if (rc) return rc;
  CK(hipMemcpy(out, d_out, (size_t)n * sizeof(int2), hipMemcpyDeviceToHost));
  (void)hipFree(d_rays);
  (void)hipFree(d_out);
  return 0;
}
