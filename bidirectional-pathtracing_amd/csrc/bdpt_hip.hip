// bdpt_hip.hip — HIP kernels for gfx950 + the C-ABI of include/bdpt/bdpt.h (libbdpt_amd.so).
//
// k_bdpt_sample: one lane per (pixel, chunk of samples). Lanes of a wave cover an 8x8 pixel block
// at the same sample index (coherent primary rays and BVH paths). Each lane runs the reference's
// per-sample estimator (bdpt_core.h: eye walk, light walk, all s x t connections with MIS),
// accumulates its eye-image value in registers and adds it once per chunk to the fp32 eye frame;
// t = 1 light-tracing splats (bidirection.cpp:457-466) are fp32 atomics into the light frame —
// the device form of update_pixel under update_lock (bidirection.cpp:544-551).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (see __graft_entry__.build).

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "bdpt/bdpt.h"
#include "bdpt_core.h"
#include "bdpt_ctx.h"
#include "bdpt_scene.h"

using namespace bdpt;

thread_local std::string bdpt::g_err;

namespace {

struct KParams {
  SceneView S;
  SampleParams sp;
  float* eye;        // W*H*3
  float* light;      // W*H*3
  unsigned long long* stats;  // 8 counters
  unsigned long long* prof;   // phase cycle counters (BDPT_PHASE_PROF builds only)
  const int4* blocks;         // tile blocks (x0, y0, w, h) of <= 8x8 pixels; null = full frame
  int nblocks;
  int nbx;                    // full-frame: blocks per row
  int spp_begin, spp_end, spl;
  unsigned nitems;            // work items = nblocks * ceil(spp_count / spl)
  unsigned nchunks;           // ceil(spp_count / spl)
  int block_major;            // 1: consecutive tickets walk one pixel block's chunks
  unsigned* work;             // ticket counter (zeroed before each launch)
  unsigned* work8;            // XCD mode: 8 ticket counters, 128 B apart (zeroed before each launch)
  unsigned region;            // XCD mode: items per group, ceil(nitems / 8)
  int xcd;                    // 1: blocks b, b+8, ... (one XCD) take items from their own eighth first
  int n_node4, n_geom4;       // float4 counts of the node / geometry arrays (LDS staging)
  int nmat;
  unsigned item_lo;           // first item of this launch (tickets count from it)
  int lstack_on;              // the traversal stacks' LDS overflow slots are staged (LM 1 / 2)
};

__device__ __forceinline__ unsigned wave_sum(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int ctz_mask(uint32_t m) { return __builtin_ctz(m); }
__device__ __forceinline__ int ctz_mask(uint64_t m) { return __builtin_ctzll(m); }
__device__ __forceinline__ int ctz_mask(unsigned __int128 m) {   // the m <= 126 kernels' 128-bit masks
  const uint64_t lo = (uint64_t)m;
  return lo ? __builtin_ctzll(lo) : 64 + __builtin_ctzll((uint64_t)(m >> 64));
}
// number of set bits of m below this lane (ballot + mbcnt prefix sum)
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}

// Wave-local ring of deferred connection rays in LDS (SoA, 128 slots per wave).
constexpr int QCAP = 128;
struct WaveQ {
  float ox[QCAP], oy[QCAP], oz[QCAP], dx[QCAP], dy[QCAP], dz[QCAP], tmax[QCAP];
  float vx[QCAP], vy[QCAP], vz[QCAP];
  int tgt[QCAP];            // >= 0: light-image pixel (t = 1 splat); < 0: ~owner lane (eye image)
  float acc[3][64];         // eye-image accumulators of the wave's 64 lanes
};

__device__ __forceinline__ float wave_sumf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Resolve n (<= 64) queued connection rays, one per lane: any-hit test, then add the value of the
// unoccluded ones to the owner's eye accumulator (LDS atomic) or splat it (global atomic).
// Splats aimed at the flush's most common kind of target — the first splatting lane's pixel — are
// summed across the wave first: a point light's own vertex projects to the same pixel for every
// sample (t = 1, s = 1), and unaggregated that one address serialises ~all global atomics.
template <int LM>
__device__ __forceinline__ void flush_queue(const SceneView& S, WaveQ& q, int head, int n, int lane, float* light,
                                            Counters& cnt) {
  bool vis = false;
  float vx = 0, vy = 0, vz = 0;
  int tgt = -1;
#ifdef BDPT_PHASE_PROF
  if (lane == 0) cnt.lp[2 * LP_FLUSH]++;
  if (lane < n) cnt.lp[2 * LP_FLUSH + 1]++;
#endif
  if (lane < n) {
    const int k = (head + lane) & (QCAP - 1);
    f3 o = mk3(q.ox[k], q.oy[k], q.oz[k]), d = mk3(q.dx[k], q.dy[k], q.dz[k]);
    const float tmax = q.tmax[k];
    vx = q.vx[k]; vy = q.vy[k]; vz = q.vz[k];
    tgt = q.tgt[k];
    vis = !trace_any<LM, kConnStack>(S, o, d, BDPT_EPS_F, tmax, cnt);
  }
  if (vis && tgt < 0) {
    const int ow = ~tgt;
    atomicAdd(&q.acc[0][ow], vx);
    atomicAdd(&q.acc[1][ow], vy);
    atomicAdd(&q.acc[2][ow], vz);
  }
  const bool splat = vis && tgt >= 0;
  const unsigned long long m = __ballot(splat);
  if (m == 0) return;
  const int lead = __builtin_ctzll(m);
  const int t0 = __shfl(tgt, lead, 64);
  const bool same = splat && tgt == t0;
  const unsigned long long ms = __ballot(same);
  if (__popcll(ms) > 1) {
    const float sx = wave_sumf(same ? vx : 0.0f), sy = wave_sumf(same ? vy : 0.0f), sz = wave_sumf(same ? vz : 0.0f);
    if (lane == lead) {
      float* p = light + 3 * (size_t)t0;
      atomicAdd(p, sx);
      atomicAdd(p + 1, sy);
      atomicAdd(p + 2, sz);
    }
  } else if (same) {
    float* p = light + 3 * (size_t)t0;
    atomicAdd(p, vx);
    atomicAdd(p + 1, vy);
    atomicAdd(p + 2, vz);
  }
  if (splat && !same) {
    float* p = light + 3 * (size_t)tgt;
    atomicAdd(p, vx);
    atomicAdd(p + 1, vy);
    atomicAdd(p + 2, vz);
  }
}

// k_bdpt_sample: each lane owns one pixel and a chunk of its samples. Per sample the lane builds
// both subpaths (random walks, closest-hit traversal) and then enumerates its (i, j) connections
// in the reference's order; every connection that needs a visibility ray is pushed (ballot +
// mbcnt compaction) into the wave's LDS ring, and whenever 64 are queued the whole wave traces
// them together — all 64 lanes busy on shadow rays regardless of per-lane path lengths.
// 4 waves per SIMD = 128 VGPRs: measured best (round 1: 2: 160, 3: 220, 4: 259, 5: 151 Msamples/s;
// round 4, with 0 instead of 38-51 spilled VGPRs at 3 waves: still -13..-16% on every workload,
// profiles/r04c_ab_waves.log)
constexpr int kMinWaves = 4;
constexpr int kBlock = 256 * kMinWaves;   // one block per CU: one LDS scene copy shared by its 16 waves
constexpr int kWavesPerBlock = kBlock / 64;

// Connections: every strategy from per-lane compacted lists (connect_sample) instead of the
// wave-uniform max|E| x max|L| grid. History: the general (i, j >= 2) pairs from lists, the special
// strategies wave-uniform, paid only for m > 5 (C5-shaped 446 -> 470, CBgems m7 +0.9 %; the m5 north
// star -1.7 %). Round 5 put the special strategies on lists too (the s = 0 list holds only the
// emitter / environment vertices), and the lists now win at m5 as well: north star 721.7 -> 730.4,
// CBspheres 674 -> 684 Msamples/s, C5-shaped and CBgems m7 unchanged (profiles/r05za_ab_conn_lists.log).
// Materials and lights copied to LDS (static arrays) when they fit: per-lane material / light
// reads in the walk and in every connection become ds_reads instead of vector-memory loads.
// (measured: C2 +3%, Lucy stand-in +1%, CBgems +1%)
constexpr int kLdsMats = 48, kLdsLights = 8;
constexpr size_t kLdsStackBytes = (size_t)kLdsStack * kBlock * sizeof(int);   // LM 1 (when it fits) and 2

constexpr size_t kStaticLds = kLdsMats * sizeof(DMat) + kLdsLights * sizeof(DLight);
constexpr int kMaxDepth = 126;   // the deepest k_bdpt_sample instantiation (MAXV = 126: vertex index <= 127, 128-bit delta masks)
#define BDPT_STR2(x) #x
#define BDPT_STR(x) BDPT_STR2(x)

#ifdef BDPT_PHASE_PROF
#define PH_STAMP(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define PH_STAMP(v)
#endif

// Stages the block's LDS copy of the scene (LM 1: whole tree + geometry; LM 2: the BFS treelet;
// LM 3: the flat leaf list with its geometry and shading records) behind the wave queues, and the
// materials / lights, and points kp.S at them.
template <int LM>
__device__ __forceinline__ void stage_scene(KParams& kp, unsigned char* smem, DMat* s_mats, DLight* s_lights) {
  static_assert(kLdsStackStride == kBlock, "LDS stack stride = lanes per block");
  const bool lst = (LM == 1 || LM == 2) && kLdsStack > 0 && kp.lstack_on;
  if (lst)   // the traversal stacks' LDS overflow slots, behind the wave queues
    kp.S.lstack = (int*)(smem + kWavesPerBlock * sizeof(WaveQ));
  if (LM != 0) {
    float4* sc = (float4*)(smem + kWavesPerBlock * sizeof(WaveQ) + (lst ? kLdsStackBytes : 0));
    const int nn = LM == 1 ? kp.n_node4 : LM == 3 ? 0 : node_f4(lm_width(LM)) * kp.S.ntop;
    const int n4 = nn + (LM == 1 || LM == 3 ? kp.n_geom4 : 0);
    for (int k = threadIdx.x; k < n4; k += blockDim.x)
      sc[k] = k < nn ? kp.S.nodes[k] : kp.S.geom[k - nn];
    if (LM == 3) {
      int* lv = (int*)(sc + n4);
      for (int k = threadIdx.x; k < kp.S.nleaves; k += blockDim.x) lv[k] = kp.S.lleaves[k];
      kp.S.lleaves = lv;
      float4* ls = sc + n4 + (kp.S.nleaves + 3) / 4;   // shading records after the leaf list
      for (int k = threadIdx.x; k < kp.n_geom4; k += blockDim.x) ls[k] = kp.S.shade[k];
      kp.S.lshade = ls;
    }
    __syncthreads();
    kp.S.lnodes = sc;
    kp.S.lgeom = sc + nn;
  }
  if (kp.nmat <= kLdsMats && kp.S.nlights <= kLdsLights) {
    for (int k = threadIdx.x; k < kp.nmat; k += blockDim.x) s_mats[k] = kp.S.mats[k];
    for (int k = threadIdx.x; k < kp.S.nlights; k += blockDim.x) s_lights[k] = kp.S.lights[k];
    __syncthreads();
    kp.S.mats = s_mats;
    kp.S.lights = s_lights;
  }
}

// Persistent waves: each wave takes work items (8x8 pixel block, chunk of spl samples) from a
// global ticket counter until none are left, so per-item cost differences (path lengths, scene
// regions) never leave CUs idle at the tail of the launch. Returns false at the first ticket past
// the end (every wave reaches it). XCD mode: blocks b and b + 8 share an XCD (round-robin dealing,
// MI355X_MICROARCH.md), so group g = b % 8 works through its own contiguous eighth of the items (a
// contiguous band of pixel blocks, whose BVH region then stays in that XCD's L2) and only then
// helps the other groups. Items are numbered from kp.item_lo.
struct Item {
  int x, y, s0, my_n;   // this lane's pixel and sample range [s0, s0 + my_n)
  unsigned idx;         // item index relative to kp.item_lo
};
__device__ __forceinline__ bool next_item(const KParams& kp, int lane, int grp, int& cur, Item& it) {
  unsigned item = 0;
  if (kp.xcd) {
    item = 0xffffffffu;
    if (lane == 0) {
      for (; cur < 8; cur++) {
        const unsigned gg = (unsigned)((grp + cur) & 7);
        const unsigned lo = gg * kp.region;
        if (lo >= kp.nitems) continue;
        const unsigned t = atomicAdd(kp.work8 + 32 * gg, 1u);
        if (t < kp.region && lo + t < kp.nitems) { item = lo + t; break; }
      }
    }
    item = __shfl(item, 0, 64);
    cur = __shfl(cur, 0, 64);
    if (item == 0xffffffffu) return false;
  } else {
    if (lane == 0) item = atomicAdd(kp.work, 1u);
    item = __shfl(item, 0, 64);
    if (item >= kp.nitems) return false;
  }
  it.idx = item;
  item += kp.item_lo;
  int chunk, blk;
  if (kp.block_major) {
    blk = (int)(item / kp.nchunks);
    chunk = (int)(item - (unsigned)blk * kp.nchunks);
  } else {
    chunk = (int)(item / (unsigned)kp.nblocks);
    blk = (int)(item - (unsigned)chunk * (unsigned)kp.nblocks);
  }
  int bx0, by0, bw, bh;
  if (kp.blocks) {
    int4 bb = kp.blocks[blk];
    bx0 = bb.x; by0 = bb.y; bw = bb.z; bh = bb.w;
  } else {
    bx0 = (blk % kp.nbx) * 8;
    by0 = (blk / kp.nbx) * 8;
    bw = min(8, kp.sp.W - bx0);
    bh = min(8, kp.sp.H - by0);
  }
  const int qx = lane & 7, qy = lane >> 3;
  it.x = 0; it.y = 0;
  int s0 = 0, s1 = 0;
  if (qx < bw && qy < bh) {
    it.x = bx0 + qx;
    it.y = by0 + qy;
    s0 = kp.spp_begin + chunk * kp.spl;
    s1 = min(s0 + kp.spl, kp.spp_end);
  }
  it.s0 = s0;
  it.my_n = max(0, s1 - s0);
  return true;
}

// Per-wave connection state of one work item: the wave-uniform ring indices (the eye accumulators,
// direct s = 0 contributions included, live in the ring's LDS).
struct ConnState {
  int head = 0, tail = 0;
#ifdef BDPT_PHASE_PROF
  unsigned long long ph_gen = 0, ph_flush = 0;
#endif
};

// The connections of one pixel-sample (est_radiance_global_illumination's s x t loop,
// bidirection.cpp:472-500): one strategy kind at a time, each lane walking its own list of usable
// vertices, so the j == 1 (fresh light sample) and i == 1 (camera connection) bodies run once per
// iteration for all lanes instead of interleaving with the general case; every connection that
// needs a visibility ray is pushed (ballot + mbcnt compaction) into the wave's LDS ring, and
// whenever 64 are queued the wave traces them together. PA: the path accessor (PathsInRegs over the
// lane's private Paths).
template <int LM, bool EXT, bool STATS, class PA>
__device__ __forceinline__ void connect_sample(const KParams& kp, WaveQ& q, const PA& PP, Rng& g, int nE, int nL,
                                               int lane, float inv, ConnState& cs, Counters& cnt) {
#ifdef BDPT_PHASE_PROF
  const unsigned long long tg0 = __builtin_amdgcn_s_memtime();
  unsigned long long tp0, tp1;
#endif
  // one (i, j) connection per lane (active lanes only), its ray pushed into the wave's ring, the
  // ring flushed whenever 64 rays are queued
  auto conn_step = [&](int i, int j, bool active, const Vtx* ev_pre = nullptr, const Vtx* lv_pre = nullptr) {
    int kind = CONN_NONE;
    Conn cn;
    if (active) {
      BDPT_LANE_PROF(cnt, LP_CONN);
      kind = make_conn<EXT>(kp.S, kp.sp, PP, g, i, j, cn, ev_pre, lv_pre, EXT && STATS ? &cnt : nullptr);
      if (kind == CONN_DIRECT) {
        // straight into this lane's accumulator in the wave's LDS (only this wave writes it, and
        // not while a flush runs): no registers held across the walks
        q.acc[0][lane] += cn.val.x * inv;
        q.acc[1][lane] += cn.val.y * inv;
        q.acc[2][lane] += cn.val.z * inv;
      }
    }
    const bool push = kind == CONN_RAY;
    const unsigned long long m = __ballot(push);
    if (push) {
      const int slot = (cs.tail + lanes_below(m)) & (QCAP - 1);
      q.ox[slot] = cn.o.x; q.oy[slot] = cn.o.y; q.oz[slot] = cn.o.z;
      q.dx[slot] = cn.d.x; q.dy[slot] = cn.d.y; q.dz[slot] = cn.d.z;
      q.tmax[slot] = cn.tmax;
      const bool eye_t = cn.splat < 0;
      q.vx[slot] = eye_t ? cn.val.x * inv : cn.val.x;
      q.vy[slot] = eye_t ? cn.val.y * inv : cn.val.y;
      q.vz[slot] = eye_t ? cn.val.z * inv : cn.val.z;
      q.tgt[slot] = eye_t ? ~lane : cn.splat;
    }
    cs.tail += __popcll(m);
    if (cs.tail - cs.head >= 64) {
      PH_STAMP(tp0);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      flush_queue<LM>(kp.S, q, cs.head, 64, lane, kp.light, cnt);
      __builtin_amdgcn_wave_barrier();
      cs.head += 64;
      PH_STAMP(tp1);
#ifdef BDPT_PHASE_PROF
      cs.ph_flush += tp1 - tp0;
#endif
    }
  };
  // Per-lane lists (bit masks, built by the walk as it stores the vertices) of the vertices each
  // strategy can use: connectable eye / light vertices (cq > 0), and the eye vertices an s = 0 path
  // ends on (an emitter, or the environment in EXT kernels) — the only ones make_conn does not
  // reject at once for these strategies
  using Mask = decltype(PP.dE);   // 32 bits, or 64 for the m <= 32 / 62 kernels
  // (a lane without a sample in this step, nE = 0, still holds its previous sample's paths)
  const bool has = nE > 0;
  Mask mE = has ? PP.conn_e() : Mask(0), mL = has ? PP.conn_l() : Mask(0), m0 = has ? PP.src_e() : Mask(0);
  // The special strategies one kind at a time (each iteration runs one make_conn body for all
  // lanes), every lane walking its own list in the reference's index order, so the wave iterates
  // the longest list instead of the longest subpath: s = 0 (j = 0), the fresh light sample (j = 1:
  // the camera, i = 1, and every connectable eye vertex), light tracing to the camera (i = 1, j >= 2)
  auto each = [&](Mask m, int fixed, bool fixed_is_j) {
    while (__ballot(m != 0)) {
      const bool act = m != 0;
      const int k = act ? ctz_mask(m) : 0;
      conn_step(fixed_is_j ? k : fixed, fixed_is_j ? fixed : k, act);
      if (act) m &= m - 1;
    }
  };
  each(m0, 0, true);
  each(nL > 1 ? Mask(mE | Mask(2u)) : Mask(0), 1, true);
  each(mL, 1, false);
  // ... then the general (i >= 2, j >= 2) pairs from the same lists: a lane walks its own (i, j)
  // pairs, so the wave iterates max(pairs) times instead of max|E| x max|L| (most cells of that
  // grid are empty for most lanes)
  if (mL == 0) mE = 0;
  Mask jm = mL;
  while (__ballot(mE != 0)) {
    const bool act = mE != 0;
    const int ci = act ? ctz_mask(mE) : 0, cj = act ? ctz_mask(jm) : 0;
    conn_step(ci, cj, act);
    if (act) {
      jm &= jm - 1;
      if (jm == 0) { mE &= mE - 1; jm = mL; }
    }
  }
#ifdef BDPT_PHASE_PROF
  cs.ph_gen += __builtin_amdgcn_s_memtime() - tg0;
#endif
}

// End of a work item: the queued rays are traced and every lane adds its eye-image sum once.
template <int LM>
__device__ __forceinline__ void finish_item(const KParams& kp, WaveQ& q, const Item& it, int lane, ConnState& cs,
                                            Counters& cnt) {
  if (cs.tail > cs.head) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    flush_queue<LM>(kp.S, q, cs.head, cs.tail - cs.head, lane, kp.light, cnt);
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (it.my_n > 0) {
    float ax = q.acc[0][lane], ay = q.acc[1][lane], az = q.acc[2][lane];
    float* e = kp.eye + 3 * ((size_t)it.x + (size_t)it.y * kp.sp.W);
    if (ax != 0) atomicAdd(e, ax);
    if (ay != 0) atomicAdd(e + 1, ay);
    if (az != 0) atomicAdd(e + 2, az);
  }
  __builtin_amdgcn_wave_barrier();
}

template <bool STATS>
__device__ __forceinline__ void flush_stats(const KParams& kp, int lane, unsigned nsamp, const Counters& cnt) {
  if (STATS) {
    // slots 0..7 the scene counters, 12..14 the environment-table reads (15: tickets, 16..31: phase profile)
    unsigned v[11] = {nsamp, cnt.closest, cnt.shadow, cnt.nodes, cnt.tris, cnt.sphs, cnt.hits, cnt.lnodes,
                      cnt.env_s, cnt.env_l, cnt.env_p};
#pragma unroll
    for (int k = 0; k < 11; k++) {
      unsigned s = wave_sum(v[k]);
      if (lane == 0 && s) atomicAdd(kp.stats + (k < 8 ? k : k + 4), (unsigned long long)s);
    }
  }
}

// LM (LDS mode): 0 = scene read from HBM/L2; 1 = whole BVH + geometry staged in LDS by every
// block; 2 = the top n_top BFS-ordered nodes (the part every ray traverses) staged in LDS.
// EXT: environment light and/or Russian roulette; EXT = false is the reference-only
// path with no trace of either in the generated code.
template <int MAXV, bool STATS, int LM, bool EXT>
__global__ __launch_bounds__(kBlock, kMinWaves) void k_bdpt_sample(KParams kp) {
  // One dynamic LDS array: [wave queues][optional scene / treelet copy]
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ DMat s_mats[kLdsMats];
  __shared__ DLight s_lights[kLdsLights];
  stage_scene<LM>(kp, smem, s_mats, s_lights);
  WaveQ* qs = (WaveQ*)smem;
  const int lane = threadIdx.x & 63;
  WaveQ& q = qs[threadIdx.x >> 6];
  Counters cnt = {0, 0, 0, 0, 0, 0};
  unsigned nsamp = 0;
  const float inv = 1.0f / (float)kp.sp.spp;
  Paths<MAXV> P;
#ifdef BDPT_PHASE_PROF
  unsigned long long ph_prep = 0, ph_gen = 0, ph_flush = 0, tp0, tp1;
  unsigned long long ph_walk_wave = 0, ph_walk_lane = 0;   // walk iterations: wave (max) / lane sums
  unsigned long long ph_cells = 0, ph_pairs = 0;           // connection grid cells / (i, j) pairs
#endif
  const int grp = blockIdx.x & 7;
  int cur = 0;   // wave-uniform: XCD groups exhausted so far
  Item it;
  while (next_item(kp, lane, grp, cur, it)) {
    const int wave_n = wave_max(it.my_n);
    q.acc[0][lane] = 0;
    q.acc[1][lane] = 0;
    q.acc[2][lane] = 0;
    ConnState cs;
    for (int t = 0; t < wave_n; t++) {
      Rng g;
      int nE = 0, nL = 0;
      PH_STAMP(tp0);
#ifdef BDPT_PHASE_PROF
      const uint32_t c0 = cnt.closest;
#endif
      if (t < it.my_n) {
        prepare_sample<MAXV, LM, EXT>(kp.S, kp.sp, P, cnt, g, it.x, it.y, (uint32_t)(it.s0 + t));
        nE = P.nE;
        nL = P.nL;
        nsamp++;
      }
      PH_STAMP(tp1);
#ifdef BDPT_PHASE_PROF
      ph_prep += tp1 - tp0;
      const int wi = (int)(cnt.closest - c0);
      ph_walk_wave += (unsigned)wave_max(wi);
      ph_walk_lane += (unsigned)wi;
      ph_cells += (unsigned)(max(wave_max(nE) - 1, 0) * wave_max(nL));
      ph_pairs += (unsigned)(max(nE - 1, 0) * nL);
#endif
      connect_sample<LM, EXT, STATS>(kp, q, PathsInRegs<MAXV, EXT>(P), g, nE, nL, lane, inv, cs, cnt);
    }
    finish_item<LM>(kp, q, it, lane, cs, cnt);
#ifdef BDPT_PHASE_PROF
    ph_gen += cs.ph_gen;
    ph_flush += cs.ph_flush;
#endif
  }
#ifdef BDPT_PHASE_PROF
  {
    // the wave-level clocks were added by whichever lane was the lowest active one (BDPT_WAVE_CLK)
    const unsigned long long ct = wave_sum64(cnt.clk_walk_trace), cl = wave_sum64(cnt.clk_light),
                             cv = wave_sum64(cnt.clk_vertex);
    if (lane == 0) {
      atomicAdd((unsigned long long*)kp.prof + 0, ph_prep);
      atomicAdd((unsigned long long*)kp.prof + 1, ph_gen - ph_flush);
      atomicAdd((unsigned long long*)kp.prof + 2, ph_flush);
      atomicAdd((unsigned long long*)kp.prof + 3, ct);
      atomicAdd((unsigned long long*)kp.prof + 4, ph_walk_wave);
      atomicAdd((unsigned long long*)kp.prof + 6, ph_cells);
      atomicAdd((unsigned long long*)kp.prof + 8, cl);
      atomicAdd((unsigned long long*)kp.prof + 9, cv);
    }
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {   // lane-use profile: prof[16 + k]
    const unsigned long long s = (unsigned long long)wave_sum(cnt.lp[k]);
    if (lane == 0 && s) atomicAdd((unsigned long long*)kp.prof + 16 + k, s);
  }
  {
    const unsigned long long wl = (unsigned long long)wave_sum((unsigned)ph_walk_lane);
    const unsigned long long wp = (unsigned long long)wave_sum((unsigned)ph_pairs);
    if (lane == 0) {
      atomicAdd((unsigned long long*)kp.prof + 5, wl);
      atomicAdd((unsigned long long*)kp.prof + 7, wp);
    }
  }
#endif
  flush_stats<STATS>(kp, lane, nsamp, cnt);
}

// k_pt: the unidirectional PathTracer (bdpt_core.h pt_pixel). Persistent waves take 8x8 pixel
// blocks from a ticket counter; a lane owns one pixel and runs its adaptive batches to the end
// (PathTracer::raytrace_pixel), then stores the mean (update_pixel) and the sample count.
struct PtKParams {
  SceneView S;
  PtParams pp;
  float* eye;                 // the frame (sampleBuffer)
  int* count;                 // sampleCountBuffer
  unsigned long long* stats;
  const int4* blocks;
  int nblocks, nbx;
  unsigned* work;
  int n_node4, n_geom4;
};

template <bool STATS, int LM>
__global__ __launch_bounds__(kBlock, kMinWaves) void k_pt(PtKParams kp) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int lane = threadIdx.x & 63;
  if (LM != 0) {
    float4* sc = (float4*)smem;
    const int nn = LM == 1 ? kp.n_node4 : LM == 3 ? 0 : node_f4(lm_width(LM)) * kp.S.ntop;
    const int n4 = nn + (LM == 1 || LM == 3 ? kp.n_geom4 : 0);
    for (int k = threadIdx.x; k < n4; k += blockDim.x) sc[k] = k < nn ? kp.S.nodes[k] : kp.S.geom[k - nn];
    if (LM == 3) {
      int* lv = (int*)(sc + n4);
      for (int k = threadIdx.x; k < kp.S.nleaves; k += blockDim.x) lv[k] = kp.S.lleaves[k];
      kp.S.lleaves = lv;
      float4* ls = sc + n4 + (kp.S.nleaves + 3) / 4;   // shading records after the leaf list
      for (int k = threadIdx.x; k < kp.n_geom4; k += blockDim.x) ls[k] = kp.S.shade[k];
      kp.S.lshade = ls;
    }
    __syncthreads();
    kp.S.lnodes = sc;
    kp.S.lgeom = sc + nn;
  }
  Counters cnt = {0, 0, 0, 0, 0, 0};
  unsigned nsamp = 0;
  for (;;) {
    unsigned item = 0;
    if (lane == 0) item = atomicAdd(kp.work, 1u);
    item = __shfl(item, 0, 64);
    if (item >= (unsigned)kp.nblocks) break;
    int bx0, by0, bw, bh;
    if (kp.blocks) {
      const int4 bb = kp.blocks[item];
      bx0 = bb.x; by0 = bb.y; bw = bb.z; bh = bb.w;
    } else {
      bx0 = ((int)item % kp.nbx) * 8;
      by0 = ((int)item / kp.nbx) * 8;
      bw = min(8, kp.pp.W - bx0);
      bh = min(8, kp.pp.H - by0);
    }
    const int qx = lane & 7, qy = lane >> 3;
    if (qx < bw && qy < bh) {
      const int x = bx0 + qx, y = by0 + qy;
      int n = 0;
      const f3 v = pt_pixel<LM>(kp.S, kp.pp, cnt, x, y, &n);
      const size_t k = (size_t)x + (size_t)y * kp.pp.W;
      kp.eye[3 * k] = v.x;
      kp.eye[3 * k + 1] = v.y;
      kp.eye[3 * k + 2] = v.z;
      kp.count[k] = n;
      nsamp += (unsigned)n;
    }
  }
  if (STATS) {
    unsigned v[8] = {nsamp, cnt.closest, cnt.shadow, cnt.nodes, cnt.tris, cnt.sphs, cnt.hits, cnt.lnodes};
#pragma unroll
    for (int k = 0; k < 8; k++) {
      unsigned s = wave_sum(v[k]);
      if (lane == 0 && s) atomicAdd(kp.stats + k, (unsigned long long)s);
    }
  }
}

__global__ void k_trace_rays(SceneView S, const float* rays, int n, int any_hit, float* out_t, int* out_prim,
                             const int* prim_ref) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = rays + 8 * (size_t)i;
  f3 o = mk3(r[0], r[1], r[2]), d = mk3(r[3], r[4], r[5]);
  Counters c = {0, 0, 0, 0, 0, 0};
  if (any_hit) {
    bool h = trace_any(S, o, d, r[6], r[7], c);
    out_t[i] = h ? 0.0f : INFINITY;
    out_prim[i] = h ? 0 : -1;
  } else {
    Hit h;
    bool ok = trace_closest(S, o, d, r[6], r[7], h, c);
    out_t[i] = ok ? h.t : INFINITY;
    out_prim[i] = ok ? prim_ref[h.prim] : -1;
  }
}

__global__ void k_combine(const float* a, const float* b, float* out, long long n) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

// LDS budget for the scene copy: 160 KB per CU shared by the blocks that the 4-waves/SIMD VGPR
// budget admits (16 waves per CU), minus their wave queues.
constexpr size_t kLdsPerCu = 160 * 1024;
// scenes up to this many primitives use the flat leaf-list traversal (LM 3)
constexpr int kFlatMaxPrims = 24;   // flat leaf list up to this many primitives; measured: CBspheres 488 -> 511 Msamples/s, CBspheres_lambertian +6%, CBempty -1%
constexpr size_t kBlocksPerCu = 4 * kMinWaves / kWavesPerBlock;
constexpr size_t kLdsSceneMax = kLdsPerCu / kBlocksPerCu - kWavesPerBlock * sizeof(WaveQ) - 256 - kStaticLds;
// LM 2's treelet gets kLdsSceneMax - kLdsStackBytes (an unsigned difference): it must hold at least
// one node, or the subtraction wraps and the treelet size is no longer capped by the LDS budget
static_assert(kLdsSceneMax > kLdsStackBytes + (size_t)node_bytes(lm_width(2)), "LDS budget: wave queues + stack slots leave no treelet");

// Persistent launch: as many blocks as are co-resident (occupancy query with this launch's LDS),
// never more waves than work items.
template <class K>
int launch_persistent(Ctx* c, K kernel, size_t lds, const KParams& kp) {
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds));
  if (per_cu <= 0) { g_err = "k_bdpt_sample cannot be resident (LDS/VGPR budget)"; return BDPT_E_DEVICE; }
  long long grid = std::min<long long>((long long)per_cu * c->ncu,
                                       ((long long)kp.nitems + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(kBlock), lds, c->stream, kp);
  HIPCHK(hipGetLastError());
  return BDPT_OK;
}

// The LDS mode of a BDPT launch and the dynamic LDS it needs (wave queues + the scene copy).
int pick_lm(Ctx* c, KParams& kp, size_t* lds) {
  const size_t q = kWavesPerBlock * sizeof(WaveQ);
  const size_t full = (c->hs.tree(lm_width(1)).nodes.size() + c->hs.geom.size()) * sizeof(float);
  const bool has_nodes = !c->hs.bvh2.nodes.empty();
  // LM 3's LDS: geometry, leaf list (padded to 16 B), shading records
  const size_t flat = 2 * c->hs.geom.size() * sizeof(float) + (c->hs.leaf_refs.size() + 3) / 4 * 16;
  int lm = c->env_lds_mode >= 0 ? c->env_lds_mode   // diagnostics: BDPT_LDS_MODE forces 0 / 1 / 2 / 3
               : (c->hs.nprim <= kFlatMaxPrims && flat <= kLdsSceneMax) ? 3
               : (full <= kLdsSceneMax ? 1 : has_nodes ? 2 : 0);
  if (lm == 3 && flat > kLdsSceneMax) lm = 1;
  if (lm == 1 && full > kLdsSceneMax) lm = 2;
  if (lm == 2 && !has_nodes) lm = 0;
  kp.S = view_of(c, lm);
  kp.n_node4 = (int)(c->hs.tree(lm_width(lm)).nodes.size() / 4);
  if (lm == 2) kp.S.ntop = (int)std::min<size_t>((size_t)c->hs.tree(lm_width(2)).n_top,
                                                 (kLdsSceneMax - kLdsStackBytes) / node_bytes(lm_width(2)));
  if (lm == 2 && c->env_ntop_max >= 0) kp.S.ntop = std::min(kp.S.ntop, c->env_ntop_max);   // diagnostics
  c->last_lm = lm;
  // LM 2 always gives the stacks their LDS slots (the treelet makes room); LM 1 when the whole
  // scene and the slots fit together (CBgems: +0.5 .. +0.8 %, profiles/r04o_ab_stack_lm1.log)
  kp.lstack_on = lm == 2 || (lm == 1 && full + kLdsStackBytes <= kLdsSceneMax);
  *lds = q + (kp.lstack_on ? kLdsStackBytes : 0) +
         (lm == 3 ? flat : lm == 1 ? full : lm == 2 ? (size_t)kp.S.ntop * node_bytes(lm_width(2)) : 0);
  return lm;
}

template <int MAXV, bool STATS, bool EXT>
int launch_lm(Ctx* c, KParams& kp) {
  size_t lds = 0;
  const int lm = pick_lm(c, kp, &lds);
  if (lm == 3) return launch_persistent(c, k_bdpt_sample<MAXV, STATS, 3, EXT>, lds, kp);
  if (lm == 1) return launch_persistent(c, k_bdpt_sample<MAXV, STATS, 1, EXT>, lds, kp);
  if (lm == 2) return launch_persistent(c, k_bdpt_sample<MAXV, STATS, 2, EXT>, lds, kp);
  return launch_persistent(c, k_bdpt_sample<MAXV, STATS, 0, EXT>, lds, kp);
}

template <int MAXV>
int launch_maxv(Ctx* c, KParams& kp) {
  if (c->ext) return c->prm.collect_stats ? launch_lm<MAXV, true, true>(c, kp) : launch_lm<MAXV, false, true>(c, kp);
  return c->prm.collect_stats ? launch_lm<MAXV, true, false>(c, kp) : launch_lm<MAXV, false, false>(c, kp);
}

template <class K, class KP>
int launch_persistent_pt(Ctx* c, K kernel, size_t lds, const KP& kp, long long items) {
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds));
  if (per_cu <= 0) { g_err = "k_pt cannot be resident (LDS/VGPR budget)"; return BDPT_E_DEVICE; }
  long long grid = std::min<long long>((long long)per_cu * c->ncu, (items + kWavesPerBlock - 1) / kWavesPerBlock);
  hipLaunchKernelGGL(kernel, dim3((unsigned)std::max(1LL, grid)), dim3(kBlock), lds, c->stream, kp);
  HIPCHK(hipGetLastError());
  return BDPT_OK;
}

template <bool STATS>
int launch_pt(Ctx* c, PtKParams& kp) {
  const size_t full = (c->hs.tree(lm_width(1)).nodes.size() + c->hs.geom.size()) * sizeof(float);
  const size_t lds_max = kLdsPerCu / kBlocksPerCu - 256;
  // LM 3's LDS: geometry, leaf list (padded to 16 B), shading records
  const size_t flat = 2 * c->hs.geom.size() * sizeof(float) + (c->hs.leaf_refs.size() + 3) / 4 * 16;
  int lm = c->env_lds_mode >= 0 ? c->env_lds_mode
               : (c->hs.nprim <= kFlatMaxPrims && flat <= lds_max) ? 3 : (full <= lds_max ? 1 : 2);
  if (lm == 3 && flat > lds_max) lm = 1;
  if (lm == 1 && full > lds_max) lm = 2;
  c->last_lm = lm;
  kp.S = view_of(c, lm);
  kp.n_node4 = (int)(c->hs.tree(lm_width(lm)).nodes.size() / 4);
  kp.n_geom4 = (int)(c->hs.geom.size() / 4);
  if (lm == 2) kp.S.ntop = (int)std::min<size_t>((size_t)c->hs.tree(lm_width(2)).n_top, lds_max / node_bytes(lm_width(2)));
  if (lm == 3) return launch_persistent_pt(c, k_pt<STATS, 3>, flat, kp, kp.nblocks);
  if (lm == 1) return launch_persistent_pt(c, k_pt<STATS, 1>, full, kp, kp.nblocks);
  if (lm == 2) return launch_persistent_pt(c, k_pt<STATS, 2>, (size_t)kp.S.ntop * node_bytes(lm_width(2)), kp, kp.nblocks);
  return launch_persistent_pt(c, k_pt<STATS, 0>, 0, kp, kp.nblocks);
}

void free_ctx(Ctx* c) {
  if (!c) return;
  void* bufs[] = {c->d_nodes2, c->d_nodes4, c->d_geom, c->d_shade, c->d_mats, c->d_lights, c->d_prim_ref, c->d_env, c->d_count, c->d_work8, c->d_leaves,
                  c->d_eye, c->d_light, c->d_sample, c->d_stats};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  for (Ctx::BlockSlot& b : c->blk) {
    if (b.d) (void)hipFree(b.d);
    if (b.h) (void)hipHostFree(b.h);
    if (b.done) (void)hipEventDestroy(b.done);
  }
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

template <class T>
int upload(T** dst, const std::vector<T>& v) {
  size_t bytes = std::max<size_t>(sizeof(T), v.size() * sizeof(T));
  HIPCHK(hipMalloc((void**)dst, bytes));
  if (!v.empty()) HIPCHK(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return BDPT_OK;
}

}  // namespace

extern "C" {

int bdpt_abi_version(void) { return BDPT_ABI_VERSION; }
const char* bdpt_last_error(void) { return g_err.c_str(); }

int bdpt_create(const bdpt_scene_desc* scene, const bdpt_params* params, void** ctx_out) {
  if (!scene || !params || !ctx_out) { g_err = "null argument"; return BDPT_E_INVALID; }
  *ctx_out = nullptr;
  const bdpt_params& p = *params;
  if (p.width <= 0 || p.height <= 0 || p.spp <= 0 || p.max_depth < 0) {
    g_err = "invalid frame size / spp / max_depth";
    return BDPT_E_INVALID;
  }
  // the kernels hold a subpath in a fixed array: instantiations for m <= 5, 8, 16, 32, 62 and 126
  // (the reference's vectors have no cap, bidirection.cpp:84-86; deeper paths are rejected cleanly:
  // a subpath's vertex index must fit the 128-bit delta masks)
  int need = p.max_depth < 1 ? 1 : p.max_depth;
  if (need > kMaxDepth) {
    g_err = "max_depth " + std::to_string(p.max_depth) + " > " + std::to_string(kMaxDepth) +
            ": the deepest kernel holds subpaths of up to 126 bounces";
    return BDPT_E_UNSUPPORTED;
  }
  // 0 = auto = 1: the persistent megakernel. 2 was the wavefront pipeline (per-bounce kernels with
  // ballot-compacted ray queues), retired in round 5 after it had fallen to 0.32-0.50x of the
  // megakernel and never ran the environment light / roulette.
  if (p.integrator == BDPT_INTEGRATOR_PT && p.max_depth > kPtMaxVerts) {   // k_pt records <= 21 vertices
    g_err = "PathTracer max_depth " + std::to_string(p.max_depth) + " > " + std::to_string(kPtMaxVerts) +
            ": its walk records up to 21 vertices (the reference's own roulette cap, pathtracer.cpp:215)";
    return BDPT_E_UNSUPPORTED;
  }
  if (p.pipeline == 2) {
    g_err = "pipeline 2 (wavefront) was retired: it ran at 0.32-0.50x of the megakernel (DESIGN.md §5); use 0 or 1";
    return BDPT_E_UNSUPPORTED;
  }
  if (p.pipeline < 0 || p.pipeline > 2) { g_err = "bad pipeline (0 = auto, 1 = megakernel)"; return BDPT_E_INVALID; }
  Ctx* c = new Ctx();
  c->prm = p;
  c->maxv = need <= 5 ? 5 : need <= 8 ? 8 : need <= 16 ? 16 : need <= 32 ? 32 : need <= 62 ? 62 : 126;
  // diagnostics / A-B switches, read once per ctx (tests set them before bdpt_create)
  auto env_int = [](const char* name, int dflt) { const char* v = getenv(name); return v ? atoi(v) : dflt; };
  c->env_lds_mode = env_int("BDPT_LDS_MODE", -1);
  c->env_ntop_max = env_int("BDPT_NTOP_MAX", -1);
  c->block_major = env_int("BDPT_BLOCK_MAJOR", 1);
  c->xcd = env_int("BDPT_XCD_GROUPS", 0);
  if (c->env_lds_mode > 3) { g_err = "BDPT_LDS_MODE must be 0..3"; delete c; return BDPT_E_INVALID; }
  c->pt = p.integrator == BDPT_INTEGRATOR_PT;
  if (p.integrator != BDPT_INTEGRATOR_BDPT && !c->pt) { g_err = "unknown integrator"; delete c; return BDPT_E_INVALID; }
  if (c->pt && (p.ns_area_light < 0 || p.samples_per_batch < 0 || p.lens_radius < 0)) {
    g_err = "invalid PathTracer settings"; delete c; return BDPT_E_INVALID;
  }
  int rc = build_host_scene(scene, c->hs, g_err, c->pt);
  if (rc) { delete c; return rc; }
  // host-side shape check before anything runs: each tree holds whole nodes of the stride its
  // kernels read (hs.tree(lm_width(LM)) is what view_of hands the LDS mode LM)
  for (int lm = 0; lm < 3; lm++) {
    const int W = lm_width(lm);
    if (c->hs.tree(W).nodes.size() % (4 * (size_t)node_f4(W)) != 0) {
      g_err = "device tree layout does not match the kernels' node width";
      delete c;
      return BDPT_E_INVALID;
    }
  }
  c->ext = c->hs.env_light >= 0 || p.russian_roulette != 0;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    g_err = "no HIP device";
    delete c;
    return BDPT_E_DEVICE;
  }
  if (p.device < 0 || p.device >= ndev) { g_err = "bad device ordinal"; delete c; return BDPT_E_INVALID; }
  c->device = p.device;
  auto fail = [&](int code) { free_ctx(c); return code; };
  if (hipSetDevice(c->device) != hipSuccess) { g_err = "hipSetDevice failed"; return fail(BDPT_E_DEVICE); }
  if (hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || c->ncu <= 0)
    c->ncu = 256;
  if ((rc = upload(&c->d_nodes2, c->hs.bvh2.nodes))) return fail(rc);
  if ((rc = upload(&c->d_nodes4, c->hs.bvh4.nodes))) return fail(rc);
  if ((rc = upload(&c->d_geom, c->hs.geom))) return fail(rc);
  if ((rc = upload(&c->d_shade, c->hs.shade))) return fail(rc);
  if ((rc = upload(&c->d_mats, c->hs.mats))) return fail(rc);
  if ((rc = upload(&c->d_lights, c->hs.lights))) return fail(rc);
  if ((rc = upload(&c->d_prim_ref, c->hs.prim_ref))) return fail(rc);
  if ((rc = upload(&c->d_leaves, c->hs.leaf_refs))) return fail(rc);
  if (c->hs.env_light >= 0 && (rc = upload(&c->d_env, c->hs.env))) return fail(rc);
  c->npix = (size_t)p.width * p.height;
  size_t fb = c->npix * 3 * sizeof(float);
  if (hipMalloc((void**)&c->d_eye, fb) != hipSuccess || hipMalloc((void**)&c->d_light, fb) != hipSuccess ||
      hipMalloc((void**)&c->d_sample, fb) != hipSuccess ||
      hipMalloc((void**)&c->d_count, c->npix * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&c->d_work8, 8 * 32 * sizeof(unsigned)) != hipSuccess ||
      hipMalloc((void**)&c->d_stats, Ctx::kStatSlots * sizeof(unsigned long long)) != hipSuccess) {
    g_err = "out of device memory";
    return fail(BDPT_E_NOMEM);
  }
  bool ev_ok = true;
  for (Ctx::BlockSlot& b : c->blk) ev_ok = ev_ok && hipEventCreateWithFlags(&b.done, hipEventDisableTiming) == hipSuccess;
  if (!ev_ok || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
    g_err = "stream/event creation failed";
    return fail(BDPT_E_DEVICE);
  }
  c->stream = c->own;
  if (hipMemsetAsync(c->d_eye, 0, fb, c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_light, 0, fb, c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_count, 0, c->npix * sizeof(int), c->stream) != hipSuccess ||
      hipMemsetAsync(c->d_stats, 0, Ctx::kStatSlots * sizeof(unsigned long long), c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) { g_err = "init sync failed"; return fail(BDPT_E_DEVICE); }
  *ctx_out = c;
  return BDPT_OK;
}

void bdpt_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return;
  {
    std::lock_guard<std::recursive_mutex> lk(c->mu);   // waits for a call in flight on another thread
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
  }
  free_ctx(c);
}

int bdpt_set_stream(void* ctx, void* stream) {
  Ctx* c = (Ctx*)ctx;
  if (!c) { g_err = "null ctx"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  c->stream = stream ? (hipStream_t)stream : c->own;
  return BDPT_OK;
}

int bdpt_clear(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) { g_err = "null ctx"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  size_t fb = c->npix * 3 * sizeof(float);
  HIPCHK(hipMemsetAsync(c->d_eye, 0, fb, c->stream));
  HIPCHK(hipMemsetAsync(c->d_light, 0, fb, c->stream));
  HIPCHK(hipMemsetAsync(c->d_count, 0, c->npix * sizeof(int), c->stream));
  HIPCHK(hipMemsetAsync(c->d_stats, 0, Ctx::kStatSlots * sizeof(unsigned long long), c->stream));
  return BDPT_OK;
}

int bdpt_render(void* ctx, const bdpt_tile* tiles, int32_t ntiles, int32_t spp_begin, int32_t spp_count) {
  Ctx* c = (Ctx*)ctx;
  if (!c) { g_err = "null ctx"; return BDPT_E_INVALID; }
  if (spp_begin < 0 || spp_count < 0 || ntiles < 0) { g_err = "negative argument"; return BDPT_E_INVALID; }
  if ((int64_t)spp_begin + spp_count > INT32_MAX) { g_err = "spp_begin + spp_count overflows int32"; return BDPT_E_INVALID; }
  if (spp_count == 0) return BDPT_OK;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  const int W = c->prm.width, H = c->prm.height;
  KParams kp;
  kp.S = view_of(c, 0);   // launch_lm sets the LDS mode's view
  kp.sp.W = W; kp.sp.H = H; kp.sp.spp = c->prm.spp; kp.sp.max_depth = c->prm.max_depth; kp.sp.seed = c->prm.seed;
  kp.sp.rr = c->prm.russian_roulette != 0;
  kp.eye = c->d_eye;
  kp.light = c->d_light;
  kp.stats = c->d_stats;
  kp.prof = c->d_stats + 16;
  kp.n_geom4 = (int)(c->hs.geom.size() / 4);
  kp.nmat = (int)c->hs.mats.size();
  kp.item_lo = 0;
  kp.lstack_on = 0;
  kp.blocks = nullptr;
  kp.nbx = (W + 7) / 8;
  kp.nblocks = kp.nbx * ((H + 7) / 8);
  Ctx::BlockSlot* slot = nullptr;
  if (tiles && ntiles > 0) {
    // Tiles (raytrace_tile clips them to the frame, raytraced_renderer.cpp:600-604) -> 8x8 blocks.
    std::vector<int4> blk;
    for (int t = 0; t < ntiles; t++) {
      int x0 = std::max(0, tiles[t].x0), y0 = std::max(0, tiles[t].y0);
      int x1 = std::min(W, tiles[t].x0 + tiles[t].w), y1 = std::min(H, tiles[t].y0 + tiles[t].h);
      for (int by = y0; by < y1; by += 8)
        for (int bx = x0; bx < x1; bx += 8) blk.push_back(make_int4(bx, by, std::min(8, x1 - bx), std::min(8, y1 - by)));
    }
    if (blk.empty()) return BDPT_OK;
    // next slot of the staging ring: wait only for the launch that last read it
    slot = &c->blk[c->blk_next];
    c->blk_next = (c->blk_next + 1) % Ctx::kBlockSlots;
    if (slot->pending) HIPCHK(hipEventSynchronize(slot->done));
    slot->pending = false;
    if (blk.size() > slot->cap) {
      if (slot->d) { (void)hipFree(slot->d); slot->d = nullptr; }
      if (slot->h) { (void)hipHostFree(slot->h); slot->h = nullptr; }
      slot->cap = 0;
      HIPCHK(hipMalloc((void**)&slot->d, blk.size() * sizeof(int4)));
      HIPCHK(hipHostMalloc((void**)&slot->h, blk.size() * sizeof(int4)));
      slot->cap = blk.size();
    }
    memcpy(slot->h, blk.data(), blk.size() * sizeof(int4));
    HIPCHK(hipMemcpyAsync(slot->d, slot->h, blk.size() * sizeof(int4), hipMemcpyHostToDevice, c->stream));
    kp.blocks = slot->d;
    kp.nblocks = (int)blk.size();
  }
  // the slot is free again once everything enqueued below has run (on every return path)
  struct SlotRelease {
    Ctx::BlockSlot* s;
    hipStream_t st;
    ~SlotRelease() {
      if (s && hipEventRecord(s->done, st) == hipSuccess) s->pending = true;
      else if (s) (void)hipStreamSynchronize(st);
    }
  } slot_release{slot, c->stream};
  if (c->pt) {   // the PathTracer renders whole pixels (adaptive sampling decides per pixel)
    if (spp_begin != 0 || spp_count != c->prm.spp) {
      g_err = "the PathTracer renders whole pixels: spp_begin must be 0 and spp_count the ctx's spp";
      return BDPT_E_INVALID;
    }
    PtKParams pk;
    pk.pp.W = W; pk.pp.H = H; pk.pp.spp = c->prm.spp; pk.pp.max_depth = c->prm.max_depth;
    pk.pp.seed = c->prm.seed;
    pk.pp.ns_area_light = c->prm.ns_area_light > 0 ? c->prm.ns_area_light : 1;
    pk.pp.batch = c->prm.samples_per_batch > 0 ? c->prm.samples_per_batch : 32;
    pk.pp.hemisphere = c->prm.direct_hemisphere_sample != 0;
    pk.pp.tol = c->prm.max_tolerance;
    pk.pp.lens_radius = (float)c->prm.lens_radius;
    pk.pp.focal_distance = (float)(c->prm.focal_distance > 0 ? c->prm.focal_distance : 4.7);
    pk.eye = c->d_eye;
    pk.count = c->d_count;
    pk.stats = c->d_stats;
    pk.blocks = kp.blocks;
    pk.nblocks = kp.nblocks;
    pk.nbx = kp.nbx;
    pk.work = (unsigned*)(c->d_stats + 15);
    HIPCHK(hipMemsetAsync(pk.work, 0, sizeof(unsigned), c->stream));
    HIPCHK(hipEventRecord(c->ev0, c->stream));
    int rc = c->prm.collect_stats ? launch_pt<true>(c, pk) : launch_pt<false>(c, pk);
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev1, c->stream));
    c->timed = true;
    return BDPT_OK;
  }
  int spl = c->prm.samples_per_lane;
  if (spl <= 0) {
    // small work items (8x8 pixels x 2 samples): measured against the earlier "~16 items per
    // co-resident wave" rule (spl 6 on C2, 43 on the 1080p stand-in): C2 586 -> 591, Lucy stand-in
    // 1080p 532 -> 536-539 Msamples/s; with block-major order spl 2 vs 4: CBgems 313 vs 305, C2 and
    // the stand-in equal; spl 8 / 16 / 32 lose 1-14% (tools/gpu_spl.sh)
    spl = (int)std::min<long long>(spp_count, 2);
  }
  kp.spl = spl;
  kp.spp_begin = spp_begin;
  kp.spp_end = spp_begin + spp_count;
  const long long nchunks = (spp_count + spl - 1) / spl;
  const long long nitems = nchunks * kp.nblocks;
  if (nitems >= 0x7fffffffLL) { g_err = "launch too large; split spp"; return BDPT_E_INVALID; }
  kp.nitems = (unsigned)nitems;
  kp.nchunks = (unsigned)nchunks;
  // consecutive tickets take one pixel block's sample chunks in turn (measured: C2 +1.2%, CBgems
  // +2%, Lucy stand-in 1080p +-0 over chunk-major order); BDPT_BLOCK_MAJOR=0 restores chunk-major
  kp.block_major = c->block_major;
  kp.work = (unsigned*)(c->d_stats + 15);
  HIPCHK(hipMemsetAsync(kp.work, 0, sizeof(unsigned), c->stream));
  kp.work8 = c->d_work8;
  kp.region = (kp.nitems + 7u) / 8u;
  kp.xcd = c->xcd;
  if (kp.xcd) HIPCHK(hipMemsetAsync(kp.work8, 0, 8 * 32 * sizeof(unsigned), c->stream));
  HIPCHK(hipEventRecord(c->ev0, c->stream));
#ifdef BDPT_ONLY_MAXV   // A/B variant builds (tools/build_variants.sh): one depth class, a faster compile
  if (c->maxv != BDPT_ONLY_MAXV) { g_err = "variant build: only max_depth class " BDPT_STR(BDPT_ONLY_MAXV); return BDPT_E_UNSUPPORTED; }
  int rc = launch_maxv<BDPT_ONLY_MAXV>(c, kp);
#else
  int rc = c->maxv == 5 ? launch_maxv<5>(c, kp) : c->maxv == 8 ? launch_maxv<8>(c, kp)
           : c->maxv == 16 ? launch_maxv<16>(c, kp) : c->maxv == 32 ? launch_maxv<32>(c, kp)
           : c->maxv == 62 ? launch_maxv<62>(c, kp) : launch_maxv<126>(c, kp);
#endif
  if (rc) return rc;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  c->timed = true;
  return BDPT_OK;
}

int bdpt_sync(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (!c) { g_err = "null ctx"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  return BDPT_OK;
}

int bdpt_frame_device_ptr(void* ctx, int32_t which, void** dptr) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !dptr) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (which == BDPT_FRAME_EYE) { *dptr = c->d_eye; return BDPT_OK; }
  if (which == BDPT_FRAME_LIGHT) { *dptr = c->d_light; return BDPT_OK; }
  if (which != BDPT_FRAME_SAMPLE) { g_err = "bad frame id"; return BDPT_E_INVALID; }
  long long n = (long long)c->npix * 3;
  hipLaunchKernelGGL(k_combine, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->d_eye, c->d_light,
                     c->d_sample, n);
  HIPCHK(hipGetLastError());
  *dptr = c->d_sample;
  return BDPT_OK;
}

int bdpt_copy_frame(void* ctx, int32_t which, void* dst_device) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !dst_device) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  void* p = nullptr;
  int rc = bdpt_frame_device_ptr(ctx, which, &p);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(dst_device, p, c->npix * 3 * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
  return BDPT_OK;
}

int bdpt_read_frame(void* ctx, int32_t which, float* rgb) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !rgb) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  void* p = nullptr;
  int rc = bdpt_frame_device_ptr(ctx, which, &p);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(rgb, p, c->npix * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return BDPT_OK;
}

int bdpt_read_frame_rect(void* ctx, int32_t which, int32_t x0, int32_t y0, int32_t w, int32_t h, float* rgb) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !rgb) { g_err = "null argument"; return BDPT_E_INVALID; }
  const int W = c->prm.width, H = c->prm.height;
  if (x0 < 0 || y0 < 0 || w < 0 || h < 0 || (int64_t)x0 + w > W || (int64_t)y0 + h > H) {
    g_err = "rectangle outside the frame";
    return BDPT_E_INVALID;
  }
  if (w == 0 || h == 0) return BDPT_OK;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  void* p = nullptr;
  int rc = bdpt_frame_device_ptr(ctx, which, &p);
  if (rc) return rc;
  const size_t row = (size_t)W * 3 * sizeof(float);
  HIPCHK(hipMemcpy2DAsync(rgb, (size_t)w * 3 * sizeof(float), (const char*)p + ((size_t)y0 * W + x0) * 3 * sizeof(float), row,
                          (size_t)w * 3 * sizeof(float), (size_t)h, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return BDPT_OK;
}

int bdpt_read_sample_counts(void* ctx, int32_t* counts) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !counts) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->pt) {
    HIPCHK(hipMemcpy(counts, c->d_count, c->npix * sizeof(int), hipMemcpyDeviceToHost));
  } else {   // BidirectionalPathTracer::raytrace_pixel records ns_aa (bidirection.cpp:539)
    for (size_t k = 0; k < c->npix; k++) counts[k] = c->prm.spp;
  }
  return BDPT_OK;
}

int bdpt_get_stats(void* ctx, bdpt_stats* out) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !out) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  unsigned long long s[16];
  HIPCHK(hipMemcpy(s, c->d_stats, sizeof s, hipMemcpyDeviceToHost));
  memset(out, 0, sizeof *out);
  out->samples = s[0];
  out->closest_rays = s[1];
  out->shadow_rays = s[2];
  out->rays = s[1] + s[2];
  out->node_visits = s[3];
  out->tri_tests = s[4];
  out->sph_tests = s[5];
  out->hits = s[6];
  float ms = 0;
  if (c->timed) HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
  out->last_kernel_ms = ms;
  out->bvh_nodes = (uint64_t)c->hs.ref_nodes;
  out->bvh_depth = (uint64_t)c->hs.depth;
  out->lds_node_visits = s[7];
  out->lds_mode = c->last_lm;
  out->env_samples = s[12];
  out->env_lookups = s[13];
  out->env_pdf_lookups = s[14];
  return BDPT_OK;
}

int bdpt_debug_lane_counters(void* ctx, uint64_t* out16) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !out16) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out16, c->d_stats + 32, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return BDPT_OK;
}

int bdpt_debug_counters(void* ctx, uint64_t* out16) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !out16) { g_err = "null argument"; return BDPT_E_INVALID; }
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out16, c->d_stats + 16, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return BDPT_OK;
}

int bdpt_trace_rays(void* ctx, const float* rays, int32_t n, int32_t any_hit, float* out_t, int32_t* out_prim) {
  Ctx* c = (Ctx*)ctx;
  if (!c || (!rays && n) || n < 0) { g_err = "bad argument"; return BDPT_E_INVALID; }
  if (n == 0) return BDPT_OK;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  HIPCHK(hipSetDevice(c->device));
  float *d_r = nullptr, *d_t = nullptr;
  int* d_p = nullptr;
  struct Frees {   // every exit path (HIPCHK returns early) releases the temporaries
    void** p[3];
    ~Frees() { for (void** q : p) if (*q) (void)hipFree(*q); }
  } frees{{(void**)&d_r, (void**)&d_t, (void**)&d_p}};
  HIPCHK(hipMalloc((void**)&d_r, (size_t)n * 8 * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_t, (size_t)n * sizeof(float)));
  HIPCHK(hipMalloc((void**)&d_p, (size_t)n * sizeof(int)));
  HIPCHK(hipMemcpy(d_r, rays, (size_t)n * 8 * sizeof(float), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_trace_rays, dim3((n + 127) / 128), dim3(128), 0, c->stream, view_of(c, 0), d_r, n, any_hit,
                     d_t, d_p, c->d_prim_ref);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipMemcpy(out_t, d_t, (size_t)n * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(out_prim, d_p, (size_t)n * sizeof(int), hipMemcpyDeviceToHost));
  return BDPT_OK;
}

}  // extern "C"
