// bdpt_wavefront.hip — wavefront form of the BDPT hot path for gfx950 (the default pipeline).
//
// The per-sample estimator of bdpt_core.h (BidirectionalPathTracer::raytrace_pixel,
// bidirection.cpp:503-542) is split into stages that each run one lane per *work item* over
// compacted queues in HBM, instead of one lane per pixel-sample walking every stage in lockstep:
//
//   k_wf_gen      slot -> camera ray + light vertex L[1] + first light ray   (:20-118, :515-524)
//   k_wf_trace    closest hit of every queued walk ray (BVHAccel::intersect, bvh.cpp:161-188)
//   k_wf_shade    hit -> path vertex (store) + sample_f -> next ray, ballot-compacted (:39-102)
//      (trace + shade repeat once per bounce; eye and light rays share the queues)
//   k_wf_cand     per slot: MIS path constants + the list of (i, j) connections that can be
//                 nonzero (diffuse endpoints seen from the front, emitters for s = 0)
//   k_wf_connect  one lane per candidate: estimate_bidirection_radiance up to its visibility
//                 test (:296-469) + power-heuristic MIS (:121-293) -> shadow-ray queue
//   k_wf_shadow   any-hit of every connection ray; unoccluded values are added to the eye image
//                 (pixel of the slot) or splatted into the light image (update_pixel, :544-551)
//
// A slot is one pixel-sample of the current batch: slot = (k * nblocks + block) * 64 + lane,
// sample = batch_s0 + k, pixel = lane's position in the 8x8 block. Every stage is a persistent
// grid-stride loop of whole waves over a device-side count, so no host synchronisation happens
// inside a render. Path vertices live in an SoA vertex store (3 x float4 per vertex per slot).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "bdpt_ctx.h"

namespace bdpt {

namespace {

constexpr int kBlock = 256;           // gen / shade / cand / connect
constexpr int kTraceBlock = 512;      // trace / shadow: one LDS scene copy per 8 waves
constexpr size_t kTraceLds = 40 * 1024;
constexpr int kWfRegStack = 8;
constexpr int kRegStack = kWfRegStack;   // traversal stack entries held in VGPRs

// Queues are striped: NS sub-queues, each with its own counter on its own 128-B line and its
// own region of cap_s entries. A producer wave working on input chunk c pushes into stripe
// c % NS, so a counter sees 1/NS of the wave-level atomics (one device-scope counter saturates
// near 88 atomics/us, MI355X_MICROARCH.md "dequeue"), and the capacity bound of every stripe
// follows from the number of input chunks it can receive. Consumers walk the stripes' chunks
// through a prefix sum of the NS counts held one per lane.
constexpr int NS = 64;
constexpr int CTR_STRIDE = 32;   // words between stripe counters
// counter blocks (NS * CTR_STRIDE words each, zeroed per batch)
enum { Q_CAND = 0, Q_SHADOW = 1, Q_RAYS = 2 /* + bounce */ };
constexpr int kMaxQueues = Q_RAYS + 18;

struct WfParams {
  SceneView S;
  SampleParams sp;
  float* eye;
  float* light;
  unsigned long long* stats;
  const int4* blocks;
  int nblocks, nbx;       // blocks of this batch (a window of the render's block list)
  int block0;             // first block of the window
  int batch_s0, spp_end;
  unsigned nslots;        // active slots of this batch
  unsigned stride;        // allocated slots (vertex-store stride)
  int capE, capL;         // vertices per eye / light path in the store
  float4 *vA, *vB, *vC;   // (pos, fwd) (n, gp) (alpha, mat | conn << 16)
  uint4* hdr;             // (nE | nL << 8, dE, dL, l1_dir_pdf)
  float4 *w0, *w1, *w2;   // walk state per path: (alpha, pdf) (f, count | dmask << 8) (n, rng pos)
  float4* w3;             //   previous vertex: (fwd, gp, mat, light dir_pdf)
  float4 *qo_in, *qd_in;  // ray queue in: (o, tmin) (d, tmax)
  unsigned* qid_in;       //   path index = slot * 2 + (0 eye | 1 light)
  float4 *qo_out, *qd_out;
  unsigned* qid_out;
  float4* hits;           // (t, prim, b1, b2) per queue entry
  unsigned* cand;         // slot | i << 22 | j << 27
  float4 *so, *sd, *sv;   // shadow queue: (o, tmax) (d, target) (value)
  unsigned char* svis;    // per shadow entry: 1 = unoccluded (refill traversal -> k_wf_resolve)
  unsigned* ctr;          // kMaxQueues counter blocks
  int cin, cout;          // counter blocks of the in / out ray queues
  unsigned cap_ray, cap_cand, cap_sh;   // entries per stripe
  int n_node4, n_geom4;
  float inv_spp;
  int point_light;        // scene has a point light: its t = 1, s = 1 splats all hit one pixel
  unsigned lds_scene;     // bytes of LDS scene copy (the wave pools follow it)
};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
__device__ __forceinline__ unsigned wave_sum_u(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned* qctr(const WfParams& p, int q) { return p.ctr + (size_t)q * NS * CTR_STRIDE; }
// Entry index of this lane for a push of 0/1 items per lane into stripe `chunk % NS`.
__device__ __forceinline__ unsigned push1(unsigned* cq, unsigned cap_s, unsigned chunk, bool push) {
  const unsigned st = chunk % NS;
  const unsigned long long m = __ballot(push);
  unsigned base = 0;
  if (lane_id() == 0 && m) base = atomicAdd(cq + st * CTR_STRIDE, (unsigned)__popcll(m));
  base = __shfl(base, 0, 64);
  return st * cap_s + base + (unsigned)lanes_below(m);
}
// First entry index of this lane for a push of n items per lane into stripe `chunk % NS`.
__device__ __forceinline__ unsigned pushn(unsigned* cq, unsigned cap_s, unsigned chunk, unsigned n) {
  const int lane = lane_id();
  const unsigned st = chunk % NS;
  unsigned incl = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    unsigned t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  const unsigned total = __shfl(incl, 63, 64);
  unsigned base = 0;
  if (lane == 0 && total) base = atomicAdd(cq + st * CTR_STRIDE, total);
  base = __shfl(base, 0, 64);
  return st * cap_s + base + incl - n;
}
// Consumer view of a striped queue: lane l holds stripe l's count and the inclusive prefix of
// chunk counts; chunk(c) maps a wave-uniform chunk index to (entry index, valid) of this lane.
struct QView {
  unsigned cnt, cincl, total, cap_s;
  __device__ void init(const unsigned* cq, unsigned cap) {
    const int lane = lane_id();
    cap_s = cap;
    cnt = __hip_atomic_load(cq + lane * CTR_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned incl = (cnt + 63u) >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      unsigned t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    cincl = incl;
    total = __shfl(incl, 63, 64);
  }
  __device__ bool entry(unsigned c, unsigned& idx) const {
    const unsigned st = (unsigned)__popcll(__ballot(cincl <= c));
    const unsigned before = st ? (unsigned)__shfl((int)cincl, (int)st - 1, 64) : 0u;
    const unsigned n = (unsigned)__shfl((int)cnt, (int)st, 64);
    const unsigned k = (c - before) * 64u + (unsigned)lane_id();
    idx = st * cap_s + k;
    return k < n;
  }
};

__device__ __forceinline__ void flush_stats(unsigned long long* st, unsigned samples, const Counters& c) {
  unsigned v[8] = {samples, c.closest, c.shadow, c.nodes, c.tris, c.sphs, c.hits, c.lnodes};
#pragma unroll
  for (int k = 0; k < 8; k++) {
    unsigned s = wave_sum_u(v[k]);
    if (lane_id() == 0 && s) atomicAdd(st + k, (unsigned long long)s);
  }
}

// slot -> pixel / global sample index; false for padding lanes of ragged blocks.
__device__ __forceinline__ bool slot_pixel(const WfParams& p, unsigned slot, int& x, int& y, int& smp) {
  const unsigned per = (unsigned)p.nblocks * 64u;
  const unsigned k = slot / per, rem = slot - k * per;
  const int blk = p.block0 + (int)(rem >> 6), q = (int)(rem & 63u);
  int bx0, by0, bw, bh;
  if (p.blocks) {
    const int4 b = p.blocks[blk];
    bx0 = b.x; by0 = b.y; bw = b.z; bh = b.w;
  } else {
    bx0 = (blk % p.nbx) * 8;
    by0 = (blk / p.nbx) * 8;
    bw = min(8, p.sp.W - bx0);
    bh = min(8, p.sp.H - by0);
  }
  const int qx = q & 7, qy = q >> 3;
  smp = p.batch_s0 + (int)k;
  x = bx0 + qx;
  y = by0 + qy;
  return qx < bw && qy < bh && smp < p.spp_end;
}

__device__ __forceinline__ unsigned vbits(int mat, int conn) { return ((unsigned)mat & 0xffffu) | ((unsigned)conn << 16); }

// Path accessor over the vertex store (make_conn / mis_weight, bdpt_core.h).
struct PathsStore {
  const float4 *A, *B, *C;
  unsigned stride, slot;
  int capE;
  uint32_t dE, dL;
  __device__ Vtx ld(int v) const {
    const size_t k = (size_t)v * stride + slot;
    const float4 a = A[k], b = B[k], c = C[k];
    Vtx r;
    r.pos = mk3(a.x, a.y, a.z);
    r.fwd = a.w;
    r.n = mk3(b.x, b.y, b.z);
    r.gp = b.w;
    r.zh = r.n;   // make_frame_hit (bdpt_core.h); L[1]'s zh is never read
    r.alpha = mk3(c.x, c.y, c.z);
    const unsigned bits = __float_as_uint(c.w);
    r.mat = (int)(short)(bits & 0xffffu);
    r.cq = (bits >> 16) ? 1.0f : 0.0f;   // no roulette in this pipeline: q = 1
    return r;
  }
  __device__ Vtx e(int k) const { return ld(k - 2); }
  __device__ Vtx l(int k) const { return ld(capE + k - 1); }
};

// Scene staging into LDS for the traversal kernels (LM 1: whole BVH + geometry, LM 2: treelet).
template <int LM>
__device__ __forceinline__ void stage_scene(WfParams& p, float4* sc) {
  if (LM == 0) return;
  const int nn = LM == 1 ? p.n_node4 : node_f4(lm_width(LM)) * p.S.ntop;
  const int n4 = nn + (LM == 1 ? p.n_geom4 : 0);
  for (int k = threadIdx.x; k < n4; k += blockDim.x) sc[k] = k < nn ? p.S.nodes[k] : p.S.geom[k - nn];
  __syncthreads();
  p.S.lnodes = sc;
  p.S.lgeom = sc + nn;
}

// ---------------------------------------------------------------------------------------------
template <bool STATS>
__global__ __launch_bounds__(kBlock) void k_wf_gen(WfParams p) {
  const int lane = lane_id();
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  unsigned nsamp = 0;
  for (unsigned base = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64u; base < p.nslots; base += nw * 64u) {
    const unsigned slot = base + lane;
    int x = 0, y = 0, smp = 0;
    const bool ok = slot < p.nslots && slot_pixel(p, slot, x, y, smp);
    f3 cam = mk3(p.S.cam.pos[0], p.S.cam.pos[1], p.S.cam.pos[2]);
    f3 rd = splat3(0), lo = splat3(0), ld = splat3(0);
    if (ok) {
      nsamp++;
      const SceneView& S = p.S;
      Rng g;
      rng_init(g, p.sp.seed, (uint32_t)(x + y * p.sp.W), (uint32_t)smp);
      float px, py;
      grid2d(g, &px, &py);
      px = px + (float)x;
      py = py + (float)y;
      rd = camera_dir(S.cam, px / (float)p.sp.W, py / (float)p.sp.H);
      const unsigned pe = 2 * slot, pl = 2 * slot + 1;
      p.w0[pe] = make_float4(1.0f, 1.0f, 1.0f, 1.0f);   // alpha = init_rad / point_pdf, pdf = dir_pdf
      p.w1[pe] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(0u));
      p.w2[pe] = make_float4(rd.x, rd.y, rd.z, __uint_as_float(g.pos));
      p.w3[pe] = make_float4(1.0f, 0.0f, __int_as_float(-1), 0.0f);
      // sample_light_ray (bidirection.cpp:105-118), AreaLight/PointLight::sample_Le
      rng_stream(g, 1);
      int lid = (int)(rng_next(g) * (float)S.nlights);
      if (lid >= S.nlights) lid = S.nlights - 1;
      const DLight& L0 = S.lights[lid];
      f3 ln;
      float lpp, ldp;
      const f3 lrad = mk3(L0.rad[0], L0.rad[1], L0.rad[2]);
      if (L0.type == LIGHT_POINT) {
        float z = rng_next(g) * 2 - 1;
        float sinT = sqrtf(fmaxf(0.0f, 1.0f - z * z));
        float u = rng_next(g);
        float c, s;
        cos_sin_2pi(u, &c, &s);
        ld = mk3(c * sinT, s * sinT, z);
        lo = mk3(L0.pos[0], L0.pos[1], L0.pos[2]);
        lpp = 1;
        ldp = 0.25f / BDPT_PI_F;
        ln = ld;
      } else {
        float sx, sy;
        grid2d(g, &sx, &sy);
        sx = sx - 0.5f;
        sy = sy - 0.5f;
        lo = add(add(mk3(L0.pos[0], L0.pos[1], L0.pos[2]), smul(sx, mk3(L0.dx[0], L0.dx[1], L0.dx[2]))),
                 smul(sy, mk3(L0.dy[0], L0.dy[1], L0.dy[2])));
        f3 dl = cosine_hemi(g, &ldp);
        Frame lf;
        lf.X = mk3(L0.fx[0], L0.fx[1], L0.fx[2]);
        lf.Y = mk3(L0.fy[0], L0.fy[1], L0.fy[2]);
        lf.Z = mk3(L0.fz[0], L0.fz[1], L0.fz[2]);
        ld = to_world(lf, dl);
        lpp = 1.0f / L0.area;
        ln = mk3(L0.dir[0], L0.dir[1], L0.dir[2]);
      }
      lpp = lpp / (float)S.nlights;
      const f3 la = divs(lrad, lpp);
      const size_t v1 = (size_t)p.capE * p.stride + slot;   // L[1]
      p.vA[v1] = make_float4(lo.x, lo.y, lo.z, lpp);           // fwd of L[1] = point pdf
      p.vB[v1] = make_float4(ln.x, ln.y, ln.z, 0.0f);
      p.vC[v1] = make_float4(la.x, la.y, la.z, __uint_as_float(vbits(-1, 0)));
      p.w0[pl] = make_float4(la.x, la.y, la.z, ldp);
      p.w1[pl] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(0u));
      p.w2[pl] = make_float4(ln.x, ln.y, ln.z, __uint_as_float(g.pos));
      p.w3[pl] = make_float4(lpp, 0.0f, __int_as_float(-1), ldp);   // L[1]: fwd = point pdf, gp = 0
    }
    // two rays per live slot: eye (camera ray on [nClip, fClip]) and light (on [EPS_F, inf))
    const unsigned q = pushn(qctr(p, p.cout), p.cap_ray, base >> 6, ok ? 2u : 0u);
    if (ok) {
      p.qo_out[q] = make_float4(cam.x, cam.y, cam.z, p.S.cam.nclip);
      p.qd_out[q] = make_float4(rd.x, rd.y, rd.z, p.S.cam.fclip);
      p.qid_out[q] = 2 * slot;
      p.qo_out[q + 1] = make_float4(lo.x, lo.y, lo.z, BDPT_EPS_F);
      p.qd_out[q + 1] = make_float4(ld.x, ld.y, ld.z, INFINITY);
      p.qid_out[q + 1] = 2 * slot + 1;
    }
  }
  if (STATS) {
    Counters c = {0, 0, 0, 0, 0, 0};
    flush_stats(p.stats, nsamp, c);
  }
}

template <int LM, bool STATS>
__global__ __launch_bounds__(kTraceBlock) void k_wf_trace(WfParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_scene<LM>(p, (float4*)smem);
  QView qv;
  qv.init(qctr(p, p.cin), p.cap_ray);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  Counters cnt = {0, 0, 0, 0, 0, 0};
  for (unsigned c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < qv.total; c += nw) {
    unsigned r;
    if (qv.entry(c, r)) {
      const float4 o = p.qo_in[r], d = p.qd_in[r];
      Hit h;
      h.prim = -1;
      const bool ok = trace_closest<LM, kRegStack>(p.S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), o.w, d.w, h, cnt);
      p.hits[r] = make_float4(h.t, __int_as_float(ok ? h.prim : -1), h.b1, h.b2);
    }
  }
  if (STATS) flush_stats(p.stats, 0, cnt);
}

// One bounce of both walks (prepare_bidirectional_subpath's loop body, bidirection.cpp:48-99).
__global__ __launch_bounds__(kBlock) void k_wf_shade(WfParams p) {
  QView qv;
  qv.init(qctr(p, p.cin), p.cap_ray);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const SceneView& S = p.S;
  for (unsigned c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < qv.total; c += nw) {
    unsigned r;
    const bool valid = qv.entry(c, r);
    bool push = false;
    f3 no = splat3(0), nd = splat3(0);
    unsigned pi = 0;
    if (valid) {
      const float4 hh = p.hits[r];
      Hit h;
      h.t = hh.x;
      h.prim = __float_as_int(hh.y);
      h.b1 = hh.z;
      h.b2 = hh.w;
      pi = p.qid_in[r];
      if (h.prim >= 0) {
        const unsigned slot = pi >> 1, kind = pi & 1u;
        const float4 qo = p.qo_in[r], qd = p.qd_in[r];
        const f3 ro = mk3(qo.x, qo.y, qo.z), rd = mk3(qd.x, qd.y, qd.z);
        const float4 a0 = p.w0[pi], a1 = p.w1[pi], a2 = p.w2[pi];
        const f3 prev_alpha = mk3(a0.x, a0.y, a0.z), prev_f = mk3(a1.x, a1.y, a1.z), prev_n = mk3(a2.x, a2.y, a2.z);
        const float prev_pdf = a0.w;
        unsigned cd = __float_as_uint(a1.w);
        int count = (int)(cd & 0xffu);
        unsigned dm = cd >> 8;
        f3 nrm;
        int mat;
        shade_hit(S, h, ro, rd, &nrm, &mat);
        const DMat M = S.mats[mat];
        const Frame fr = make_frame_hit(nrm);
        const f3 hit_p = add(ro, muls(rd, h.t));
        const float cp = dot(prev_n, rd);
        const f3 alpha = divs(mul(muls(prev_alpha, fabsf(cp)), prev_f), prev_pdf);
        const int i = count + 2;   // reference vertex index
        // MIS path constants of the new vertex, as eye_constants / light_constants (bdpt_core.h)
        // compute them from this vertex and the previous one (ray origin ro, walk state w2/w3):
        // conn, fwd (pdf of reaching it from the previous vertex), gp (Horner prefix G_{i-1},
        // which needs the reverse pdf of the previous vertex, evaluated from this one).
        const float4 a3 = p.w3[pi];
        const f3 zh = fr.Z;
        const int conn = M.type == MAT_DIFFUSE && lz(normalize(sub(ro, hit_p)), zh) >= 0 && nonzero3(alpha);
        float fwd = 1.0f * 1.0f, gp = 0.0f;
        if (kind != 0 || i > 2) {
          const f3 pzh = (kind != 0 && i == 2) ? zaxis(prev_n) : prev_n;   // L[1] / a hit (make_frame_hit)
          f3 dw;
          const float g2 = step_g(hit_p, nrm, ro, pzh, &dw);
          const float pf = (kind != 0 && i == 2) ? a3.w : pdf_b(S.mats[__float_as_int(a3.z)], prev_n, pzh, dw) * 1.0f;
          fwd = pf * g2;
          f3 dr;
          const float g = step_g(ro, prev_n, hit_p, zh, &dr);
          const float pr = pdf_b(M, nrm, zh, dr) * 1.0f;
          gp = mis_horner((pr * g) / a3.x, !((dm >> (i - 2)) & 3u), a3.y);
        }
        const size_t v = (size_t)(kind == 0 ? count : p.capE + 1 + count) * p.stride + slot;
        p.vA[v] = make_float4(hit_p.x, hit_p.y, hit_p.z, fwd);
        p.vB[v] = make_float4(nrm.x, nrm.y, nrm.z, gp);
        p.vC[v] = make_float4(alpha.x, alpha.y, alpha.z, __uint_as_float(vbits(mat, conn)));
        if (is_delta(M.type)) dm |= 1u << i;
        count++;
        if (!(i >= p.sp.max_depth + 1 || count >= p.capE)) {
          int x, y, smp;
          (void)slot_pixel(p, slot, x, y, smp);
          Rng g;
          rng_init(g, p.sp.seed, (uint32_t)(x + y * p.sp.W), (uint32_t)smp);
          rng_stream(g, kind);
          g.pos = __float_as_uint(a2.w);
          const f3 w_out = to_local(fr, neg(rd));
          f3 wi;
          float pdf;
          const f3 fv = sample_f(M, g, w_out, &wi, &pdf);
          nd = normalize(to_world(fr, wi));
          no = hit_p;
          push = true;
          p.w0[pi] = make_float4(alpha.x, alpha.y, alpha.z, pdf * 1.0f);
          p.w2[pi] = make_float4(nrm.x, nrm.y, nrm.z, __uint_as_float(g.pos));
          p.w1[pi] = make_float4(fv.x, fv.y, fv.z, __uint_as_float((unsigned)count | (dm << 8)));
          p.w3[pi] = make_float4(fwd, gp, __int_as_float(mat), a3.w);
        } else {
          p.w1[pi] = make_float4(a1.x, a1.y, a1.z, __uint_as_float((unsigned)count | (dm << 8)));
        }
      }
    }
    const unsigned q = push1(qctr(p, p.cout), p.cap_ray, c, push);
    if (push) {
      p.qo_out[q] = make_float4(no.x, no.y, no.z, BDPT_EPS_F);
      p.qd_out[q] = make_float4(nd.x, nd.y, nd.z, INFINITY);
      p.qid_out[q] = pi;
    }
  }
}

// Per slot: the list of (i, j) connections that can be nonzero (make_conn's early exits that
// depend only on vertex properties) + the slot header for k_wf_connect.
__global__ __launch_bounds__(kBlock) void k_wf_cand(WfParams p) {
  const int lane = lane_id();
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  const SceneView& S = p.S;
  for (unsigned base = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64u; base < p.nslots; base += nw * 64u) {
    const unsigned slot = base + lane;
    int x = 0, y = 0, smp = 0;
    const bool ok = slot < p.nslots && slot_pixel(p, slot, x, y, smp);
    int nE = 0, nL = 0;
    unsigned connE = 0, emE = 0, connL = 0;   // bit k: reference vertex k
    unsigned ne = 0;
    if (ok) {
      const unsigned ce = __float_as_uint(p.w1[2 * slot].w), cl = __float_as_uint(p.w1[2 * slot + 1].w);
      const int cntE = (int)(ce & 0xffu), cntL = (int)(cl & 0xffu);
      nE = cntE + 2;
      nL = cntL + 2;
      for (int k = 0; k < cntE; k++) {
        const unsigned bits = __float_as_uint(p.vC[(size_t)k * p.stride + slot].w);
        const int mat = (int)(short)(bits & 0xffffu);
        connE |= (bits >> 16) << (k + 2);
        emE |= (S.mats[mat].type == MAT_EMISSION ? 1u : 0u) << (k + 2);
      }
      for (int k = 2; k < nL; k++)
        connL |= (__float_as_uint(p.vC[(size_t)(p.capE + k - 1) * p.stride + slot].w) >> 16) << k;
      p.hdr[slot] = make_uint4((unsigned)nE | ((unsigned)nL << 8), ce >> 8, cl >> 8, 0u);
      const unsigned nlc = 1u + (unsigned)__popc(connL);   // j == 1 (fresh light sample) + j >= 2
      ne = (unsigned)__popc(emE) + (1u + (unsigned)__popc(connE)) * nlc;
    }
    unsigned q = pushn(qctr(p, Q_CAND), p.cap_cand, base >> 6, ne);
    if (ok) {
      for (int i = 1; i < nE; i++) {
        const unsigned ib = slot | ((unsigned)i << 22);
        if ((emE >> i) & 1u) p.cand[q++] = ib;
        if (i >= 2 && !((connE >> i) & 1u)) continue;
        p.cand[q++] = ib | (1u << 27);
        for (int j = 2; j < nL; j++)
          if ((connL >> j) & 1u) p.cand[q++] = ib | ((unsigned)j << 27);
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_wf_connect(WfParams p) {
  QView qv;
  qv.init(qctr(p, Q_CAND), p.cap_cand);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  for (unsigned cc = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; cc < qv.total; cc += nw) {
    unsigned r;
    const bool valid = qv.entry(cc, r);
    int kind = CONN_NONE;
    Conn cn;
    int pix = 0;
    bool hot = false;
    if (valid) {
      const unsigned c = p.cand[r];
      const unsigned slot = c & 0x3fffffu;
      const int i = (int)((c >> 22) & 31u), j = (int)(c >> 27);
      hot = p.point_light && i == 1 && j == 1;
      int x, y, smp;
      (void)slot_pixel(p, slot, x, y, smp);
      pix = x + y * p.sp.W;
      const uint4 hd = p.hdr[slot];
      PathsStore st{p.vA, p.vB, p.vC, p.stride, slot, p.capE, hd.y, hd.z};
      Rng g;
      rng_init(g, p.sp.seed, (uint32_t)pix, (uint32_t)smp);
      kind = make_conn(p.S, p.sp, st, g, i, j, cn);
      if (kind == CONN_DIRECT) {
        float* e = p.eye + 3 * (size_t)pix;
        atomicAdd(e, cn.val.x * p.inv_spp);
        atomicAdd(e + 1, cn.val.y * p.inv_spp);
        atomicAdd(e + 2, cn.val.z * p.inv_spp);
      }
    }
    const bool push = kind == CONN_RAY;
    const unsigned q = push1(qctr(p, Q_SHADOW), p.cap_sh, cc, push);
    if (push) {
      const bool eye_t = cn.splat < 0;
      const int tgt = eye_t ? ~pix : cn.splat;
      const f3 v = eye_t ? muls(cn.val, p.inv_spp) : cn.val;
      p.so[q] = make_float4(cn.o.x, cn.o.y, cn.o.z, cn.tmax);
      p.sd[q] = make_float4(cn.d.x, cn.d.y, cn.d.z, __int_as_float(tgt));
      p.sv[q] = make_float4(v.x, v.y, v.z, hot ? 1.0f : 0.0f);
    }
  }
}

// Adds v to frame[3*t] for every lane with `on`, one atomic per run of equal targets in lane
// order (segmented inclusive scan; connection rays of one slot are queued next to each other).
__device__ __forceinline__ void seg_add(float* frame, bool on, int t, f3 v) {
  if (__ballot(on) == 0) return;
  const int lane = lane_id();
  const int key = on ? t : -1 - lane;
  const int prev = __shfl_up(key, 1, 64), next = __shfl_down(key, 1, 64);
  bool head = lane == 0 || prev != key;
  const bool tail = lane == 63 || next != key;
  float x = on ? v.x : 0.0f, y = on ? v.y : 0.0f, z = on ? v.z : 0.0f;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float ux = __shfl_up(x, o, 64), uy = __shfl_up(y, o, 64), uz = __shfl_up(z, o, 64);
    const bool uh = __shfl_up((int)head, o, 64) != 0;
    if (lane >= o && !head) {
      x += ux; y += uy; z += uz;
      head = uh;
    }
  }
  if (on && tail) {
    float* f = frame + 3 * (size_t)t;
    atomicAdd(f, x);
    atomicAdd(f + 1, y);
    atomicAdd(f + 2, z);
  }
}

// Adds v to frame[3*t] for every lane with `on`; lanes aiming at the same pixel as the first
// pending lane are summed across the wave first (a few rounds), the rest use plain atomics.
__device__ __forceinline__ void wave_add(float* frame, bool on, int t, f3 v, int rounds) {
#pragma unroll 1
  for (int round = 0; round < rounds; round++) {
    const unsigned long long m = __ballot(on);
    if (m == 0) return;
    const int lead = __builtin_ctzll(m);
    const int t0 = __shfl(t, lead, 64);
    const bool same = on && t == t0;
    if (__popcll(__ballot(same)) < 2) break;
    const float sx = wave_sum_f(same ? v.x : 0.0f), sy = wave_sum_f(same ? v.y : 0.0f),
                sz = wave_sum_f(same ? v.z : 0.0f);
    if (lane_id() == lead) {
      float* f = frame + 3 * (size_t)t0;
      atomicAdd(f, sx);
      atomicAdd(f + 1, sy);
      atomicAdd(f + 2, sz);
    }
    on = on && !same;
  }
  if (on) {
    float* f = frame + 3 * (size_t)t;
    atomicAdd(f, v.x);
    atomicAdd(f + 1, v.y);
    atomicAdd(f + 2, v.z);
  }
}

template <int LM, bool STATS>
__global__ __launch_bounds__(kTraceBlock) void k_wf_shadow(WfParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_scene<LM>(p, (float4*)smem);
  QView qv;
  qv.init(qctr(p, Q_SHADOW), p.cap_sh);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  Counters cnt = {0, 0, 0, 0, 0, 0};
  for (unsigned c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < qv.total; c += nw) {
    unsigned r;
    const bool valid = qv.entry(c, r);
    bool vis = false, hot = false;
    int tgt = 0;
    f3 v = splat3(0);
    if (valid) {
      const float4 o = p.so[r], d = p.sd[r];
      tgt = __float_as_int(d.w);
      vis = !trace_any<LM, kRegStack>(p.S, mk3(o.x, o.y, o.z), mk3(d.x, d.y, d.z), BDPT_EPS_F, o.w, cnt);
      if (vis) {
        const float4 w = p.sv[r];
        v = mk3(w.x, w.y, w.z);
        hot = w.w != 0.0f;
      }
    }
    seg_add(p.eye, vis && tgt < 0, ~tgt, v);
    wave_add(p.light, vis && tgt >= 0 && hot, tgt, v, 8);
    wave_add(p.light, vis && tgt >= 0 && !hot, tgt, v, 1);
  }
  if (STATS) flush_stats(p.stats, 0, cnt);
}

// ---------------------------------------------------------------------------------------------
// Traversal with lane refill (Aila & Laine 2009, "persistent while-while with dynamic fetch"): a
// lane whose ray is finished takes the next queued ray instead of idling until the slowest lane
// of its wave is done. Each wave owns a 128-entry LDS pool of queue indices, refilled chunk by
// chunk (64 entries) from its static share of the striped queue; lanes advance one leaf visit
// at a time and the wave refills while it is less than 3/4 busy.
constexpr int kPool = 128;
constexpr int kWfRefillBelow = 48;
constexpr int kRefillBelow = kWfRefillBelow;

struct WavePool {
  int* ids;
  unsigned next;     // next chunk of this wave's static share (wave-uniform)
  int head, count;   // wave-uniform
  __device__ void refill(const QView& qv, unsigned nw) {
    while (count < 64 && next < qv.total) {
      unsigned r;
      const bool v = qv.entry(next, r);
      const unsigned long long m = __ballot(v);
      if (v) ids[(head + count + lanes_below(m)) & (kPool - 1)] = (int)r;
      count += __popcll(m);
      next += nw;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  // returns true for an idle lane that received entry *rid
  __device__ bool assign(bool active, unsigned* rid) {
    const unsigned long long idle = __ballot(!active);
    const int take = min(__popcll(idle), count);
    bool got = false;
    if (!active) {
      const int rank = lanes_below(idle);
      if (rank < take) {
        *rid = (unsigned)ids[(head + rank) & (kPool - 1)];
        got = true;
      }
    }
    head += take;
    count -= take;
    __builtin_amdgcn_wave_barrier();
    return got;
  }
  __device__ bool more(const QView& qv) const { return count > 0 || next < qv.total; }
};

template <int LM, bool STATS>
__global__ __launch_bounds__(kTraceBlock) void k_wf_trace_rf(WfParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_scene<LM>(p, (float4*)smem);
  QView qv;
  qv.init(qctr(p, p.cin), p.cap_ray);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  WavePool pool{(int*)(smem + p.lds_scene) + (threadIdx.x >> 6) * kPool, (blockIdx.x * blockDim.x + threadIdx.x) >> 6, 0, 0};
  Counters cnt = {0, 0, 0, 0, 0, 0};
  bool active = false;
  unsigned rid = 0;
  f3 o = splat3(0), d = splat3(0);
  float tmin = 0;
  RayInv r = make_rayinv(mk3(1, 1, 1), mk3(1, 1, 1));
  Hit h;
  h.t = 0; h.prim = -1; h.key = -1; h.b1 = 0; h.b2 = 0;
  int ref = 0;
  int stack_mem[kStackMax];
  TravStack<kRegStack> stk(stack_mem);
  for (;;) {
    pool.refill(qv, nw);
    if (pool.assign(active, &rid)) {
      const float4 a = p.qo_in[rid], b = p.qd_in[rid];
      o = mk3(a.x, a.y, a.z);
      d = mk3(b.x, b.y, b.z);
      tmin = a.w;
      r = make_rayinv(o, d);
      h.t = b.w; h.prim = -1; h.key = -1; h.b1 = 0; h.b2 = 0;
      ref = p.S.root;
      stk.nreg = 0;
      stk.clear();
      cnt.closest++;
      active = true;
    }
    if (__ballot(active) == 0) break;
    for (;;) {
      if (active && closest_step<LM, kRegStack>(p.S, r, o, d, tmin, h, ref, stk, cnt)) {
        if (h.prim >= 0) cnt.hits++;
        p.hits[rid] = make_float4(h.t, __int_as_float(h.prim), h.b1, h.b2);
        active = false;
      }
      const int na = __popcll(__ballot(active));
      if (na == 0 || (na < kRefillBelow && pool.more(qv))) break;
    }
  }
  if (STATS) flush_stats(p.stats, 0, cnt);
}

template <int LM, bool STATS>
__global__ __launch_bounds__(kTraceBlock) void k_wf_shadow_rf(WfParams p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  stage_scene<LM>(p, (float4*)smem);
  QView qv;
  qv.init(qctr(p, Q_SHADOW), p.cap_sh);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  WavePool pool{(int*)(smem + p.lds_scene) + (threadIdx.x >> 6) * kPool, (blockIdx.x * blockDim.x + threadIdx.x) >> 6, 0, 0};
  Counters cnt = {0, 0, 0, 0, 0, 0};
  bool active = false;
  unsigned rid = 0;
  f3 o = splat3(0), d = splat3(0);
  float tmax = 0;
  RayInv r = make_rayinv(mk3(1, 1, 1), mk3(1, 1, 1));
  int ref = 0;
  int stack_mem[kStackMax];
  TravStack<kRegStack> stk(stack_mem);
  for (;;) {
    pool.refill(qv, nw);
    if (pool.assign(active, &rid)) {
      const float4 a = p.so[rid], b = p.sd[rid];
      o = mk3(a.x, a.y, a.z);
      d = mk3(b.x, b.y, b.z);
      tmax = a.w;
      r = make_rayinv(o, d);
      ref = p.S.root;
      stk.nreg = 0;
      stk.clear();
      cnt.shadow++;
      active = true;
    }
    if (__ballot(active) == 0) break;
    for (;;) {
      bool hit = false;
      if (active && any_step<LM, kRegStack>(p.S, r, o, d, BDPT_EPS_F, tmax, ref, stk, &hit, cnt)) {
        p.svis[rid] = hit ? 0 : 1;   // resolved into the frames by k_wf_resolve
        active = false;
      }
      const int na = __popcll(__ballot(active));
      if (na == 0 || (na < kRefillBelow && pool.more(qv))) break;
    }
  }
  if (STATS) flush_stats(p.stats, 0, cnt);
}

// Adds the unoccluded connection values to the frames, walking the shadow queue in its own order:
// a slot's connection rays sit next to each other, so eye-image values reduce to one atomic per
// run of equal pixels (seg_add) and point-light t=1 splats to one per wave (wave_add).
__global__ __launch_bounds__(kBlock) void k_wf_resolve(WfParams p) {
  QView qv;
  qv.init(qctr(p, Q_SHADOW), p.cap_sh);
  const unsigned nw = (gridDim.x * blockDim.x) >> 6;
  for (unsigned c = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; c < qv.total; c += nw) {
    unsigned r;
    const bool valid = qv.entry(c, r);
    const bool vis = valid && p.svis[r] != 0;
    int tgt = 0;
    bool hot = false;
    f3 v = splat3(0);
    if (vis) {
      tgt = __float_as_int(p.sd[r].w);
      const float4 w = p.sv[r];
      v = mk3(w.x, w.y, w.z);
      hot = w.w != 0.0f;
    }
    seg_add(p.eye, vis && tgt < 0, ~tgt, v);
    wave_add(p.light, vis && tgt >= 0 && hot, tgt, v, 8);
    wave_add(p.light, vis && tgt >= 0 && !hot, tgt, v, 1);
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
struct WfState {
  int capE = 0, capL = 0;
  unsigned stride = 0;     // allocated slots
  size_t ncand = 0;        // candidate / shadow capacity (entries)
  float4 *vA = nullptr, *vB = nullptr, *vC = nullptr;
  uint4* hdr = nullptr;
  float4 *w0 = nullptr, *w1 = nullptr, *w2 = nullptr, *w3 = nullptr;
  float4 *qo[2] = {nullptr, nullptr}, *qd[2] = {nullptr, nullptr};
  unsigned* qid[2] = {nullptr, nullptr};
  float4* hits = nullptr;
  unsigned* cand = nullptr;
  float4 *so = nullptr, *sd = nullptr, *sv = nullptr;
  unsigned char* svis = nullptr;
  unsigned* ctr = nullptr;
  unsigned cap_ray = 0, cap_cand = 0, cap_sh = 0;   // entries per stripe
  int lm = -1, ntop = 0;
  size_t lds = 0;
};

void wf_free(Ctx* c) {
  WfState* w = c->wf;
  if (!w) return;
  void* bufs[] = {w->vA, w->vB, w->vC, w->hdr, w->w0, w->w1, w->w2, w->w3, w->qo[0], w->qo[1], w->qd[0], w->qd[1],
                  w->qid[0], w->qid[1], w->hits, w->cand, w->so, w->sd, w->sv, w->svis, w->ctr};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  delete w;
  c->wf = nullptr;
}

namespace {

template <class T>
int dalloc(T** p, size_t n) {
  HIPCHK(hipMalloc((void**)p, std::max<size_t>(1, n) * sizeof(T)));
  return BDPT_OK;
}

int wf_alloc(Ctx* c) {
  if (c->wf) return BDPT_OK;
  WfState* w = new WfState();
  c->wf = w;
  const int M = c->prm.max_depth;
  w->capE = std::max(1, M);
  w->capL = w->capE + 1;
  // connection candidates per slot <= (|E| - 1) * |L| (bidirection.cpp:490-491)
  const size_t per_slot_cand = (size_t)(w->capE + 1) * (w->capL + 1);
  const char* env = getenv("BDPT_WF_SLOTS");
  size_t slots = env ? (size_t)atoll(env) : (per_slot_cand <= 64 ? (1u << 20) : (1u << 18));
  slots = std::min<size_t>(std::max<size_t>(slots, 64), 1u << 22);   // slot ids are 22 bits
  w->stride = (unsigned)slots;
  const size_t chunks_s = (slots / 64 + NS - 1) / NS;   // slot chunks per stripe
  w->cap_ray = (unsigned)(((2 * slots / 64 + NS - 1) / NS + 2) * 64);
  w->cap_cand = (unsigned)(chunks_s * 64 * per_slot_cand);
  w->cap_sh = w->cap_cand + 64;
  w->ncand = (size_t)NS * w->cap_sh;
  const size_t nray = (size_t)NS * w->cap_ray;
  const size_t nv = (size_t)(w->capE + w->capL) * slots;
  int rc;
  if ((rc = dalloc(&w->vA, nv)) || (rc = dalloc(&w->vB, nv)) || (rc = dalloc(&w->vC, nv)) ||
      (rc = dalloc(&w->hdr, slots)) || (rc = dalloc(&w->w0, 2 * slots)) || (rc = dalloc(&w->w1, 2 * slots)) ||
      (rc = dalloc(&w->w2, 2 * slots)) || (rc = dalloc(&w->w3, 2 * slots)) || (rc = dalloc(&w->qo[0], nray)) || (rc = dalloc(&w->qo[1], nray)) ||
      (rc = dalloc(&w->qd[0], nray)) || (rc = dalloc(&w->qd[1], nray)) ||
      (rc = dalloc(&w->qid[0], nray)) || (rc = dalloc(&w->qid[1], nray)) ||
      (rc = dalloc(&w->hits, nray)) || (rc = dalloc(&w->cand, w->ncand)) || (rc = dalloc(&w->so, w->ncand)) ||
      (rc = dalloc(&w->sd, w->ncand)) || (rc = dalloc(&w->sv, w->ncand)) || (rc = dalloc(&w->svis, w->ncand)) ||
      (rc = dalloc(&w->ctr, (size_t)kMaxQueues * NS * CTR_STRIDE))) {
    wf_free(c);
    return rc;
  }
  // LDS staging for the traversal kernels: whole scene if it fits, else the BFS treelet.
  const size_t full = (c->hs.tree(lm_width(1)).nodes.size() + c->hs.geom.size()) * sizeof(float);
  const char* lenv = getenv("BDPT_LDS_MODE");
  w->lm = lenv ? atoi(lenv) : (full <= kTraceLds ? 1 : 2);
  if (w->lm == 1 && full > kTraceLds) w->lm = 2;
  if (w->lm == 2) {
    w->ntop = (int)std::min<size_t>((size_t)c->hs.tree(lm_width(2)).n_top, kTraceLds / node_bytes(lm_width(2)));
    if (w->ntop <= 0) w->lm = 0;
  }
  w->lds = w->lm == 1 ? full : w->lm == 2 ? (size_t)w->ntop * node_bytes(lm_width(2)) : 0;
  return BDPT_OK;
}

template <class K>
int launch(Ctx* c, K kernel, int block, size_t lds, const WfParams& p, long long work) {
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds));
  if (per_cu <= 0) { g_err = "wavefront kernel cannot be resident"; return BDPT_E_DEVICE; }
  long long grid = (long long)per_cu * c->ncu;
  if (work >= 0) grid = std::min<long long>(grid, std::max<long long>(1, (work + block - 1) / block));
  hipLaunchKernelGGL(kernel, dim3((unsigned)grid), dim3(block), lds, c->stream, p);
  HIPCHK(hipGetLastError());
  return BDPT_OK;
}

// BDPT_WF_REFILL: bit 0 = refill traversal for walk rays (default on), bit 1 = refill traversal
// for connection rays + separate k_wf_resolve (default off: the fused kernel overlaps its frame
// atomics with traversal, which measured faster)
int wf_refill_mask() {
  static const int m = getenv("BDPT_WF_REFILL") ? atoi(getenv("BDPT_WF_REFILL")) : 1;
  return m;
}
bool wf_refill() { return (wf_refill_mask() & 2) != 0; }

template <bool STATS>
int trace_launch(Ctx* c, WfParams& p, bool shadow, long long work) {
  WfState* w = c->wf;
  p.S.ntop = w->ntop;
  p.lds_scene = (unsigned)((w->lds + 15) & ~(size_t)15);
  const bool rf = shadow ? wf_refill() : (wf_refill_mask() & 1) != 0;
  if (rf) {
    const size_t lds = p.lds_scene + (size_t)(kTraceBlock / 64) * kPool * sizeof(int);
    if (shadow) {
      if (w->lm == 1) return launch(c, k_wf_shadow_rf<1, STATS>, kTraceBlock, lds, p, work);
      if (w->lm == 2) return launch(c, k_wf_shadow_rf<2, STATS>, kTraceBlock, lds, p, work);
      return launch(c, k_wf_shadow_rf<0, STATS>, kTraceBlock, lds, p, work);
    }
    if (w->lm == 1) return launch(c, k_wf_trace_rf<1, STATS>, kTraceBlock, lds, p, work);
    if (w->lm == 2) return launch(c, k_wf_trace_rf<2, STATS>, kTraceBlock, lds, p, work);
    return launch(c, k_wf_trace_rf<0, STATS>, kTraceBlock, lds, p, work);
  }
  if (shadow) {
    if (w->lm == 1) return launch(c, k_wf_shadow<1, STATS>, kTraceBlock, w->lds, p, work);
    if (w->lm == 2) return launch(c, k_wf_shadow<2, STATS>, kTraceBlock, w->lds, p, work);
    return launch(c, k_wf_shadow<0, STATS>, kTraceBlock, 0, p, work);
  }
  if (w->lm == 1) return launch(c, k_wf_trace<1, STATS>, kTraceBlock, w->lds, p, work);
  if (w->lm == 2) return launch(c, k_wf_trace<2, STATS>, kTraceBlock, w->lds, p, work);
  return launch(c, k_wf_trace<0, STATS>, kTraceBlock, 0, p, work);
}

}  // namespace

int wf_render(Ctx* c, const int4* blocks, int nblocks, int nbx, int spp_begin, int spp_count) {
  int rc = wf_alloc(c);
  if (rc) return rc;
  WfState* w = c->wf;
  const bool stats = c->prm.collect_stats != 0;
  WfParams p;
  memset(&p, 0, sizeof p);
  p.S = view_of(c, w->lm);
  p.sp.W = c->prm.width; p.sp.H = c->prm.height; p.sp.spp = c->prm.spp; p.sp.max_depth = c->prm.max_depth;
  p.sp.seed = c->prm.seed;
  p.eye = c->d_eye;
  p.light = c->d_light;
  p.stats = c->d_stats;
  p.blocks = blocks;
  p.nblocks = nblocks;
  p.nbx = nbx;
  p.spp_end = spp_begin + spp_count;
  p.stride = w->stride;
  p.capE = w->capE;
  p.capL = w->capL;
  p.vA = w->vA; p.vB = w->vB; p.vC = w->vC; p.hdr = w->hdr;
  p.w0 = w->w0; p.w1 = w->w1; p.w2 = w->w2; p.w3 = w->w3;
  p.hits = w->hits;
  p.cand = w->cand;
  p.so = w->so; p.sd = w->sd; p.sv = w->sv; p.svis = w->svis;
  p.ctr = w->ctr;
  p.cap_ray = w->cap_ray;
  p.cap_cand = w->cap_cand;
  p.cap_sh = w->cap_sh;
  p.n_node4 = (int)(c->hs.tree(lm_width(w->lm)).nodes.size() / 4);
  p.n_geom4 = (int)(c->hs.geom.size() / 4);
  p.inv_spp = 1.0f / (float)c->prm.spp;
  for (const DLight& l : c->hs.lights) p.point_light |= l.type == LIGHT_POINT;
  // a batch = a window of <= stride/64 blocks x K samples
  const int win = (int)std::min<long long>(nblocks, w->stride / 64);
  const int K = (int)std::max<long long>(1, w->stride / ((long long)win * 64));
  for (int b0 = 0; b0 < nblocks; b0 += win)
  for (int s0 = spp_begin; s0 < p.spp_end; s0 += K) {
    const int k = std::min(K, p.spp_end - s0);
    p.block0 = b0;
    p.nblocks = std::min(win, nblocks - b0);
    p.batch_s0 = s0;
    p.nslots = (unsigned)((long long)k * p.nblocks * 64);
    HIPCHK(hipMemsetAsync(w->ctr, 0, (size_t)(Q_RAYS + w->capE + 1) * NS * CTR_STRIDE * sizeof(unsigned), c->stream));
    // gen -> ray queue of bounce 0
    p.qo_out = w->qo[0]; p.qd_out = w->qd[0]; p.qid_out = w->qid[0];
    p.cout = Q_RAYS;
    if ((rc = stats ? launch(c, k_wf_gen<true>, kBlock, 0, p, p.nslots) : launch(c, k_wf_gen<false>, kBlock, 0, p, p.nslots)))
      return rc;
    for (int b = 0; b < w->capE; b++) {
      const int in = b & 1, out = in ^ 1;
      p.qo_in = w->qo[in]; p.qd_in = w->qd[in]; p.qid_in = w->qid[in];
      p.qo_out = w->qo[out]; p.qd_out = w->qd[out]; p.qid_out = w->qid[out];
      p.cin = Q_RAYS + b;
      p.cout = Q_RAYS + b + 1;
      const long long maxr = 2LL * p.nslots;
      if ((rc = stats ? trace_launch<true>(c, p, false, maxr) : trace_launch<false>(c, p, false, maxr))) return rc;
      if ((rc = launch(c, k_wf_shade, kBlock, 0, p, maxr))) return rc;
    }
    if ((rc = launch(c, k_wf_cand, kBlock, 0, p, p.nslots))) return rc;
    if ((rc = launch(c, k_wf_connect, kBlock, 0, p, -1))) return rc;
    if ((rc = stats ? trace_launch<true>(c, p, true, -1) : trace_launch<false>(c, p, true, -1))) return rc;
    if (wf_refill() && (rc = launch(c, k_wf_resolve, kBlock, 0, p, -1))) return rc;
  }
  return BDPT_OK;
}

}  // namespace bdpt
