// bdpt_core.h — device-side BDPT per-sample pipeline for MI355X (gfx950), single-source so the
// host part of libbdpt_amd.so can precompute light frames with the same arithmetic.
//
// What it computes is the reference's per-pixel-sample estimator
//   BidirectionalPathTracer::raytrace_pixel / est_radiance_global_illumination
//   (src/pathtracer/bidirection.cpp:472-542)
// in the fp32 "device semantics" of DESIGN.md §fp32: every expression keeps the reference's
// operation order (CGL Vector3D semantics), uniforms come from Philox4x32-10 keyed by
// (seed, pixel, sample), sin/cos(2*pi*u) from a fixed polynomial, cos(acos z) = z, integer
// powers by products, and the sphere quadratic in fp64. The oracle's COUNTER32 mode
// (oracle/bdpt_oracle.cpp) restates the same semantics independently; parity is per sample.
//
// How it differs from the reference's *structure* (output-identical):
//  * BVH2 with both child boxes in the parent, near-first ordered traversal, t-culling against
//    conservatively padded fp32 boxes; ties in t resolved to the larger DFS leaf position, which
//    is what the reference's l->r exhaustive traversal with `t <= max_t` yields (bvh.cpp:161-188).
//  * Connection (shadow) rays use an any-hit traversal: only their boolean is consumed
//    (bidirection.cpp:428-433).
//  * The MIS walk (bidirection.cpp:121-293) is O(i+j) multiplies per connection: the per-vertex
//    ratios nom/denom of the non-endpoint steps are path constants, evaluated once per subpath
//    with the reference's exact operations and reused; only the two endpoint steps are evaluated
//    per connection.
//  * Connections whose contribution is identically zero (non-diffuse endpoint BSDF, f = 0
//    hemisphere test, zero throughput) skip their shadow ray (quirk 17).

#pragma once

#include <stdint.h>

#include <type_traits>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BDPT_HD __host__ __device__ __forceinline__
#define BDPT_D __device__ __forceinline__
#else
#include <cmath>
#define BDPT_HD inline
#define BDPT_D inline
#include <cstring>
using std::sqrt;
struct float4 {
  float x, y, z, w;
};
inline int __float_as_int(float f) { int i; std::memcpy(&i, &f, 4); return i; }
inline float __int_as_float(int i) { float f; std::memcpy(&f, &i, 4); return f; }
#endif

namespace bdpt {

// ------------------------------------------------------------------------------------------------
// Constants (CGL/include/CGL/misc.h:11-14)
#define BDPT_PI_F 3.14159265358979323f
#define BDPT_EPS_F 0.00001f

// ------------------------------------------------------------------------------------------------
// fp32 3-vectors with CGL Vector3D operation order (vector3D.h)
struct f3 {
  float x, y, z;
};
BDPT_HD f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
BDPT_HD f3 add(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
BDPT_HD f3 sub(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
BDPT_HD f3 mul(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
BDPT_HD f3 muls(f3 a, float c) { return mk3(a.x * c, a.y * c, a.z * c); }      // v * c
BDPT_HD f3 smul(float c, f3 a) { return mk3(c * a.x, c * a.y, c * a.z); }      // c * v
BDPT_HD f3 divs(f3 a, float c) { float rc = 1.0f / c; return mk3(rc * a.x, rc * a.y, rc * a.z); }
BDPT_HD f3 neg(f3 a) { return mk3(-a.x, -a.y, -a.z); }
BDPT_HD float dot(f3 u, f3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
BDPT_HD float norm2(f3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
BDPT_HD float norm(f3 a) { return sqrtf(norm2(a)); }
BDPT_HD f3 normalize(f3 a) { float rc = 1.0f / norm(a); return mk3(a.x * rc, a.y * rc, a.z * rc); }
BDPT_HD f3 cross(f3 u, f3 v) {
  return mk3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}
BDPT_HD f3 splat3(float c) { return mk3(c, c, c); }

// make_coord_space (bsdf.cpp:21-41): columns X, Y, Z of o2w.
struct Frame {
  f3 X, Y, Z;
};
template <bool UNIT = false>
BDPT_HD Frame make_frame_t(f3 n) {
  f3 z = n, h = n;
  if (fabsf(h.x) <= fabsf(h.y) && fabsf(h.x) <= fabsf(h.z)) h.x = 1.0f;
  else if (fabsf(h.y) <= fabsf(h.x) && fabsf(h.y) <= fabsf(h.z)) h.y = 1.0f;
  else h.z = 1.0f;
  if (!UNIT) z = normalize(z);
  f3 y = normalize(cross(h, z));
  f3 x = normalize(cross(z, y));
  Frame f;
  f.X = x; f.Y = y; f.Z = z;
  return f;
}
BDPT_HD Frame make_frame(f3 n) { return make_frame_t<false>(n); }
// The frame of a surface hit. Its shading normal is already normalize()d (shade_hit), so the
// fp32 semantics take Z = n instead of normalising it a second time (which moves a component by
// at most an ulp, in about 1 of 4 normals): one normalize less per vertex, and a stored path
// vertex needs no separate shading axis (oracle mode 2 does the same).
BDPT_HD Frame make_frame_hit(f3 n) { return make_frame_t<true>(n); }
// o2w * v (matrix3x3.cpp:110-114) and w2o * v = o2w.T() * v
BDPT_HD f3 to_world(const Frame& f, f3 v) { return add(add(smul(v.x, f.X), smul(v.y, f.Y)), smul(v.z, f.Z)); }
BDPT_HD float lz(f3 v, f3 Z) { return v.x * Z.x + v.y * Z.y + v.z * Z.z; }   // (w2o*v).z
BDPT_HD f3 to_local(const Frame& f, f3 v) { return mk3(lz(v, f.X), lz(v, f.Y), lz(v, f.Z)); }
BDPT_HD f3 zaxis(f3 n) { return normalize(n); }   // make_coord_space(n).Z without X, Y
BDPT_HD bool nonzero3(f3 v) { return (v.x != 0) | (v.y != 0) | (v.z != 0); }

// ------------------------------------------------------------------------------------------------
// Counter RNG: Philox4x32-10, counter (pixel, sample, block, 0xB1D1), key (seed lo, hi).
// Sub-streams of one pixel-sample (identical in oracle/bdpt_oracle.cpp CounterStream):
// 0 = camera jitter + eye walk, 1 = light choice + light walk, 2 + i = the fresh light sample of
// connection (i, j = 1). Counter = (pixel, sample, block, 0xB1D1 + (stream << 16)), so phases and
// connections can be evaluated in any order and skipped connections consume nothing.
struct Rng {
  uint32_t k0, k1, pix, smp;
  uint32_t pos;   // uniform index within the stream: block = pos >> 2, word = pos & 3
  uint32_t cur;   // block held in b0..b3 (0xffffffff: none)
  uint32_t tag;   // 0xB1D1 + (stream << 16)
  uint32_t b0, b1, b2, b3;
};
BDPT_HD void rng_init(Rng& r, uint64_t seed, uint32_t pixel, uint32_t sample) {
  r.k0 = (uint32_t)seed; r.k1 = (uint32_t)(seed >> 32); r.pix = pixel; r.smp = sample;
  r.pos = 0; r.cur = 0xffffffffu; r.tag = 0xB1D1u;
}
BDPT_HD void rng_stream(Rng& r, uint32_t s) {
  r.pos = 0; r.cur = 0xffffffffu; r.tag = 0xB1D1u + (s << 16);
}
BDPT_HD void philox(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
BDPT_HD float u_of(uint32_t x) { return ((float)(x >> 9) + 0.5f) * 1.1920928955078125e-07f; }
BDPT_HD float rng_next(Rng& r) {
  const uint32_t blk = r.pos >> 2;
  if (blk != r.cur) {
    r.b0 = r.pix; r.b1 = r.smp; r.b2 = blk; r.b3 = r.tag;
    philox(r.b0, r.b1, r.b2, r.b3, r.k0, r.k1);
    r.cur = blk;
  }
  const uint32_t w = r.pos & 3u;
  uint32_t x = w == 0 ? r.b0 : w == 1 ? r.b1 : w == 2 ? r.b2 : r.b3;
  r.pos++;
  return u_of(x);
}
// Consume n uniforms without using them (a connection whose value is known to be zero still
// advances the stream exactly as the reference's draws would).
BDPT_HD void rng_skip(Rng& r, uint32_t n) { r.pos += n; }

// cos/sin(2*pi*u), u in (0,1): quadrant split + Taylor polynomials (same as the oracle's).
BDPT_HD void cos_sin_2pi(float u, float* c, float* s) {
  float t = u * 4.0f;
  int k = (int)(t + 0.5f);
  float f = u - (float)k * 0.25f;
  float f2 = f * f;
  float sp = f * (6.2831854820251465f +
                  f2 * (-41.34170150756836f +
                        f2 * (81.6052474975586f + f2 * (-76.70585632324219f + f2 * 42.058692932128906f))));
  float cp = 1.0f + f2 * (-19.739208221435547f +
                          f2 * (64.93939208984375f +
                                f2 * (-85.45681762695312f + f2 * (60.2446403503418f + f2 * -26.42625617980957f))));
  int q = k & 3;
  float cc = q == 0 ? cp : q == 1 ? -sp : q == 2 ? -cp : sp;
  float ss = q == 0 ? sp : q == 1 ? cp : q == 2 ? -sp : -cp;
  *c = cc;
  *s = ss;
}

// atan2(y, x) for the environment map's direction -> (theta, phi) (environment_light.cpp:97-102):
// octant reduction + the Cephes atanf polynomial (|err| ~ 1e-7), plain fp32 operations so the
// oracle's mode 2 (oracle/bdpt_oracle.cpp atan2_f32) evaluates it bit-identically.
BDPT_HD float atan2_det(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  if (ax == 0.0f && ay == 0.0f) return 0.0f;
  float t = ay <= ax ? ay / ax : ax / ay;   // [0, 1]
  float off = 0.0f;
  if (t > 0.41421356237309503f) {           // tan(pi/8): atan t = pi/4 + atan((t-1)/(t+1))
    off = 0.78539816339744831f;
    t = (t - 1.0f) / (t + 1.0f);
  }
  const float z = t * t;
  float r = ((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) * z) * t + t;
  r = off + r;
  if (ay > ax) r = 1.57079632679489662f - r;
  if (x < 0.0f) r = 3.14159265358979323f - r;
  return y < 0.0f ? -r : r;
}
// lround for x >= 0 (std::lround: halves away from zero), exact: x - floor(x) is exact.
BDPT_HD int lround_pos(float x) {
  const float f = floorf(x);
  return (int)f + ((x - f) >= 0.5f ? 1 : 0);
}

// ------------------------------------------------------------------------------------------------
// Scene layout in HBM (see DESIGN.md §Data layout)
enum { MAT_DIFFUSE = 0, MAT_EMISSION = 1, MAT_MIRROR = 2, MAT_GLASS = 3, MAT_REFRACTION = 4, MAT_MICROFACET = 5 };
// Vtx::mat of a vertex without BSDF: -1 camera / area or point light vertex, MAT_ENV_V a vertex
// of the environment light (an escaped eye ray, or an env light subpath's first vertex).
enum { MAT_ENV_V = -2 };
enum { LIGHT_AREA = 0, LIGHT_POINT = 1, LIGHT_ENV = 2, LIGHT_HEMI = 3, LIGHT_DIR = 4 };   // HEMI, DIR: PathTracer only
// Russian roulette (bdpt_params.russian_roulette): vertices with index i > BDPT_RR_MIN continue
// with p_keep = min(1, |f| / pdf) (the rule commented out at bidirection.cpp:87-93).
#define BDPT_RR_MIN 3

struct DMat {
  int type;
  float a[3];    // microfacet: eta
  float b[3];    // microfacet: k
  float ior;
  float alpha;   // microfacet roughness (PathTracer only: BDPT rejects microfacet)
};
struct DLight {
  int type;
  float rad[3], pos[3], dir[3], dx[3], dy[3];
  float area;                 // LIGHT_ENV: pi R^2 of the scene's bounding sphere (emission disk)
  float fx[3], fy[3], fz[3];  // make_coord_space(dir)
};

// Environment light (EnvironmentLight, environment_light.cpp): the map and its sampling tables
// (init(), :18-62) built in fp64 on the host and rounded to fp32, plus the scene's bounding
// sphere that sample_Le emits from.
struct EnvView {
  const float* marg;   // h: marginal_y (CDF over rows)
  const float* cond;   // w*h: conds_y (per-row CDFs)
  const float* pdf;    // w*h: pdf_envmap
  const float* rgb;    // w*h*3: data[w*j + i]
  const int* gmarg;    // gm+1: guide table of marg (null: plain binary search)
  const int* gcond;    // h*(gc+1): guide tables of the rows of cond
  int gm, gc;
  int w, h;
  int light;           // index of the env light in the light list (-1: none)
  float cx, cy, cz, rad;
};
struct DCam {
  float pos[3];
  float c2w[9];  // column-major
  float w2c[9];
  float tanh_, tanv_;  // tan(hFov*PI/360) in fp64, rounded (camera.cpp:199-200)
  float nclip, fclip;
};

// Child reference: >= 0 internal node index; < 0 leaf: ~ref = start << 7 | sphere_mask << 3 | count.
BDPT_HD bool ref_is_leaf(int r) { return r < 0; }
BDPT_HD int leaf_start(int r) { return (int)(((uint32_t)~r) >> 7); }
BDPT_HD int leaf_count(int r) { return (int)((uint32_t)~r & 7u); }
BDPT_HD int leaf_sph_mask(int r) { return (int)((((uint32_t)~r) >> 3) & 15u); }

struct SceneView {
  const float4* nodes;   // node_f4(lm_width(LM)) float4 per node (layouts at node_step)
  const float4* geom;    // 3 x float4 per prim (DFS order): tri p0,e1,e2 | sphere c,r
  const float4* shade;   // 3 x float4 per prim: n1 n2 n3 (tri) ; w of the 3rd = material (bits)
  const DMat* mats;
  const DLight* lights;
  int nlights;
  int root;              // root child reference
  const float4* lnodes;  // LDS copy of nodes [0, ntop) (LM 1: all nodes; LM 2: BFS treelet)
  const float4* lgeom;   // LDS copy of the geometry (LM 1 and 3)
  const float4* lshade;  // LDS copy of the shading records (LM 3)
  const int* lleaves;    // LM 3: every leaf reference (LDS), nleaves of them
  int nleaves;
  int fn;                // LM 3: > 0 when the leaves hold primitives 0 .. fn-1 in order (flat_prims)
  uint32_t fsph;         // LM 3: sphere mask of those primitives
  int ntop;
  int* lstack;           // LM 1 / 2: the traversal stacks' first kLdsStack overflow slots in LDS (slot k of
                         // lane t at lstack[k * kLdsStackStride + t]); null: all overflow in scratch
  DCam cam;
  EnvView env;
};

// ------------------------------------------------------------------------------------------------
// Counters for the roofline (algorithmic bytes)
struct Counters {
  uint32_t nodes, tris, sphs, closest, shadow, hits;
  uint32_t lnodes = 0;   // of `nodes`: child AABBs read from the block's LDS copy (LM 1, LM 2 treelet)
  uint32_t env_s = 0, env_l = 0, env_p = 0;   // environment-light samples / radiance / pdf lookups
#ifdef BDPT_PHASE_PROF
  // wave-level cycles (each interval counted by the wave's lowest active lane, BDPT_WAVE_CLK; the
  // kernel sums its lanes): in the walk's closest-hit queries, drawing the light vertex L[1]
  // (sample_light_ray), and from a hit to the next ray (shading record, vertex, sample_f)
  unsigned long long clk_walk_trace = 0;
  unsigned long long clk_light = 0;
  unsigned long long clk_vertex = 0;
  // lane use per phase: [2k] wave-level iterations (counted by the wave's lowest active lane),
  // [2k + 1] active lanes summed over them (every active lane counts itself); k = LP_*
  uint32_t lp[2 * 8] = {};
#endif
};

// Phases of the lane-use profile (BDPT_PHASE_PROF builds, bdpt_debug_lane_counters).
enum {
  LP_CNODE = 0,   // closest-hit node steps (walk rays)
  LP_CPRIM = 1,   // closest-hit primitive tests
  LP_ANODE = 2,   // any-hit node steps (connection rays)
  LP_APRIM = 3,   // any-hit primitive tests
  LP_SHADE = 4,   // walk: hit -> next ray (shading record, vertex, MIS constants, sample_f)
  LP_WALK = 5,    // walk iterations (one closest-hit query each)
  LP_CONN = 6,    // connection evaluations (make_conn)
  LP_FLUSH = 7    // connection-ray flushes: wave-level flushes / rays traced
};
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define BDPT_LANE_PROF(c, k)                                                                      \
  do {                                                                                            \
    const unsigned long long m_ = __ballot(1);                                                    \
    if ((unsigned)__lane_id() == (unsigned)__builtin_ctzll(m_)) (c).lp[2 * (k)]++;                \
    (c).lp[2 * (k) + 1]++;                                                                        \
  } while (0)
// a wave-level interval of dt cycles (s_memtime is the wave's clock): added once, by the lowest
// active lane, so that an interval is counted whichever lanes take part in it
#define BDPT_WAVE_CLK(acc, dt)                                                                    \
  do {                                                                                            \
    const unsigned long long m_ = __ballot(1);                                                    \
    if ((unsigned)__lane_id() == (unsigned)__builtin_ctzll(m_)) (acc) += (dt);                    \
  } while (0)
#else
#define BDPT_LANE_PROF(c, k) \
  do {                       \
  } while (0)
#endif

struct Hit {
  float t;
  int prim;   // position in the device tree's leaf order, -1 = none
  int key;    // position in the reference tree's DFS leaf order (tie-break)
  float b1, b2;
};

// Both predicates with non-short-circuit & / |: each term a lane mask, combined without a branch.
// Written with && / || (and the early-outs joined by ||), the compiler emitted an exec-mask branch
// per term — ~40 scalar / vector instructions per check in the leaf loops; flat, the north-star
// kernel has 650 fewer static instructions and runs +3.3 % (CBspheres +14 %, CBgems m7 +5 %,
// profiles/r06v_ab_tri_flat.log). Same predicates, same results.
BDPT_HD bool quot_neg(float n, float d) {
  return (((n < 0) & (d > 0)) | ((n > 0) & (d < 0))) & (fabsf(n) >= fabsf(d) * 8.67361738e-19f);  // 2^-60
}
BDPT_HD bool quot_gt1(float n, float d) {
  return (((n > 0) & (d > 0)) | ((n < 0) & (d < 0))) & (fabsf(n) > fabsf(d));
}

// Möller–Trumbore exactly as Triangle::intersect (triangle.cpp:57-95), fp32.
BDPT_HD bool tri_test(const float4 g0, const float4 g1, const float4 g2, f3 o, f3 d, float tmin, float tmax,
                      float* t_out, float* b1_out, float* b2_out) {
  f3 p0 = mk3(g0.x, g0.y, g0.z);
  f3 e1 = mk3(g0.w, g1.x, g1.y);
  f3 e2 = mk3(g1.z, g1.w, g2.x);
  f3 s = sub(o, p0);
  f3 s1 = cross(d, e2);
  float denom = dot(s1, e1);
  float n1 = dot(s1, s);
  // Exact early-outs before the three correctly-rounded divisions: only when the rounded
  // quotient is certainly < 0 (opposite signs, |q| >= 2^-60 so it cannot round to -0) or > 1
  // (|n| > |denom| implies fl(n/denom) > 1), i.e. exactly when the reference test fails anyway.
  if (quot_neg(n1, denom) | quot_gt1(n1, denom)) return false;
  f3 s2 = cross(s, e1);
  float n2 = dot(s2, d);
  if (quot_neg(n2, denom) | quot_gt1(n2, denom)) return false;
  float nt = dot(s2, e2);
  if ((tmin >= 0) & quot_neg(nt, denom)) return false;
  float t = nt / denom;
  float b1 = n1 / denom;
  float b2 = n2 / denom;
  *t_out = t; *b1_out = b1; *b2_out = b2;
  return (t >= tmin) & (t <= tmax) & (b1 >= 0) & (b2 >= 0) & (b1 + b2 <= 1);
}

// Sphere::test + intersect (sphere.cpp:11-35,61-93) with the quadratic in fp64.
BDPT_HD bool sph_test(const float4 g0, f3 o, f3 d, float tmin, float tmax, float* t_out) {
  {
    // Conservative fp32 miss test: squared distance of the centre from the ray's line exceeds r^2
    // by far more than the fp32 error (~1e-6 |o-c|^2), so the fp64 discriminant is < 0 too.
    f3 f = sub(o, mk3(g0.x, g0.y, g0.z));
    float a = norm2(d), bh = dot(f, d), ff = norm2(f);
    float dl2a = ff * a - bh * bh;   // a * dist^2(centre, line)
    if (dl2a > a * (g0.w * g0.w * 1.001f + ff * 1e-5f)) return false;
  }
  double ox = o.x, oy = o.y, oz = o.z, dx = d.x, dy = d.y, dz = d.z;
  double cx = g0.x, cy = g0.y, cz = g0.z, r = g0.w;
  double r2 = r * r;
  double a = dx * dx + dy * dy + dz * dz;
  double fx = ox - cx, fy = oy - cy, fz = oz - cz;
  double b = 2 * (fx * dx + fy * dy + fz * dz);
  double c = (fx * fx + fy * fy + fz * fz) - r2;
  double delta = b * b - 4 * a * c;
  if (delta < 0) return false;
  double root = sqrt(delta);
  double t1 = (-b - root) / (2 * a);
  double t2 = (-b + root) / (2 * a);
  const bool in1 = (t1 >= (double)tmin) & (t1 <= (double)tmax), in2 = (t2 >= (double)tmin) & (t2 <= (double)tmax);
  const double t = in1 ? t1 : in2 ? t2 : -1.0;
  if (t > 0) {
    *t_out = (float)t;
    return true;
  }
  return false;
}

}  // namespace bdpt

namespace bdpt {

// ------------------------------------------------------------------------------------------------
// BVH traversal (replaces BVHAccel::intersect, bvh.cpp:161-188; see header comment).
constexpr int kStackMax = 64;
// Register-stack entries of the megakernel's walk / connection-ray traversals (TravStack<K>).
// Measured (Lucy stand-in 1080p / CBspheres / CBgems, Msamples/s): K 0: 440 / 438 / 273,
// K 2: 465 / 452 / 284, K 4: 465 / 450 / 290 (walk 8 or connection 8: no further gain). Round 4,
// with 8 LDS slots behind them (kLdsStack): walk / connection 2/2, 3/3, 2/4, 4/2 lose 0.6 .. 1.7 %
// on the north star (profiles/r04k_ab_regstack.log). Round 5, with the LDS slots: 0 / 0 and 0 / 4
// -0.5 % on the north star, 4 / 0 +-0.2 %; with the tree in HBM (no LDS slots) 0 / 0 -10 %, and on
// CBgems (LM 1) -2 % (profiles/r05y_ab_regstack.log). Round 6, after the leaner node step: 3 / 3,
// 2 / 2, 4 / 2, 2 / 4 lose 0.4 .. 1 % on the north star, up to 2 % on CBgems (r06z3_ab_regstack.log).
#ifndef BDPT_WALK_STACK
#define BDPT_WALK_STACK 4
#endif
#ifndef BDPT_CONN_STACK
#define BDPT_CONN_STACK 4
#endif
constexpr int kWalkStack = BDPT_WALK_STACK;   // variant builds may override (-DBDPT_WALK_STACK=...)
constexpr int kConnStack = BDPT_CONN_STACK;
// Children per BVH node: 2 (64-B nodes) or 4 (128-B nodes: half the dependent node fetches per
// ray, four independent slab tests per fetch). The host emits both trees over the same leaves;
// a kernel traverses the one its LDS mode selects: scenes fetched from HBM (LM 0, LM 2's nodes below
// the treelet) gain from the shorter dependent chain, a scene held whole in LDS (LM 1) does not
// (its fetches are short, and the wider test costs instructions). Measured, DESIGN.md §5.
constexpr int kBvhWidth = 4;       // LM 0 / 2
constexpr int kLdsBvhWidth = 2;   // LM 1
static_assert((kBvhWidth == 2 || kBvhWidth == 4) && (kLdsBvhWidth == 2 || kLdsBvhWidth == 4),
              "BVH widths must be 2 or 4");
// Child visiting order of the 4-wide node step: 0 = slot order (any-hit connection rays),
// 1 = near-first by a sorting network (closest-hit queries).
constexpr int kAnyOrd = 0, kClosestOrd = 1;

// BVH leaves: the next primitive's record is loaded before the current one is tested, where the
// geometry comes from HBM (LM 0 / 2). Measured: Lucy stand-in 1080p 489 -> 516, CBbunny 800x600
// 351 -> 370 Msamples/s; with the geometry in LDS (LM 1, CBgems) 303 -> 299, so off there. LM 3
// walks its flat list the same way (S.fn > 0).
BDPT_HD constexpr bool leaf_prefetch(int LM) { return LM == 0 || LM == 2; }

// Speculative while-while (Aila & Laine 2009; trace_closest / trace_any): a lane holding a
// postponed leaf keeps descending while other lanes still look for theirs; leaves are tested once
// every lane holds one (or is done). Where the nodes come from HBM (LM 0 / 2) the extra node steps
// fill the lanes that would otherwise wait: Lucy stand-in 601 -> 631, C5-shaped 468 -> 485
// Msamples/s; with the whole tree in LDS (LM 1) the longer steps cost more than the latency they
// hide (CBgems m7 269 -> 247), so only LM 0 / 2. Variants measured and removed: two
// postponed leaves per lane, stopping the descent once fewer than 4 / 8 / 16 lanes still look.
BDPT_HD constexpr bool spec_trav(int LM) { return LM == 0 || LM == 2; }
// active lanes of the wave for which the predicate holds (the host build runs one lane)
BDPT_HD int wave_count(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __popcll(__ballot(p));
#else
  return p ? 1 : 0;
#endif
}
// LM 3 (flat): tiny scenes test every leaf in order, no node fetches, no stack, no divergence
// in the traversal loop (same hits and tie rule as a tree walk, bdpt_scene.cpp leaf_refs).
BDPT_HD constexpr int lm_width(int LM) { return LM == 1 || LM == 3 ? kLdsBvhWidth : kBvhWidth; }
BDPT_HD constexpr int node_f4(int W) { return W == 4 ? 8 : 4; }        // float4 per node (stride)
BDPT_HD constexpr int node_used_f4(int W) { return W == 4 ? 7 : 4; }   // float4 a traversal reads
BDPT_HD constexpr int node_bytes(int W) { return 16 * node_f4(W); }

// Traversal stack: the newest K entries in registers (shifted on push/pop, fully unrolled), older
// ones in a private array (K = 0: all of it). Near-first traversal of these trees rarely holds more
// than ~8 entries; a few register entries keep most pushes/pops off scratch.
// The overflow below the register entries: its first kLdsStack slots in LDS when the kernel gives
// the stack an LDS area (SceneView::lstack, LM 1 / 2; one lane's slot k at lstack[k * stride + lane], no
// bank conflicts), deeper ones in the private array. A pop from LDS puts the next node address on
// the critical path after an LDS read instead of a scratch (L1 / L2) read. The 32 KB come out of the
// LM-2 treelet (~430 -> ~180 nodes). Measured (profiles/r04i_ab_lds_stack.log, Msamples/s, 0 / 4 /
// 8 / 12 slots): north star 681 / 690 / 689 / 679, C5-shaped 580 / 586 / 590 / 579, C3 465 / 471 /
// 471 / 465, CBbunny 800x600 510 / 517 / 515 / 508.
constexpr int kLdsStack = 8;
constexpr int kLdsStackStride = 1024;   // lanes per block (bdpt_hip.hip kBlock)

// this lane's LDS overflow slots (device, LM 1 / 2 kernels that staged them), else null
BDPT_HD int* lane_stack(const SceneView& S) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kLdsStack > 0 && S.lstack ? S.lstack + threadIdx.x : nullptr;
#else
  return nullptr;
#endif
}

#if defined(BDPT_STEP_HIST) && !defined(__HIP_DEVICE_COMPILE__)
}  // namespace bdpt
#include <vector>
namespace bdpt {
inline unsigned long long* step_hist() { static thread_local unsigned long long h[1024]; return h; }
inline int& step_hist_nested() { static thread_local int n = 0; return n; }
// diagnostics: the any-hit queries' rays (o, d, tmin, tmax) while a sink is set (tools/anyhit_probe.py)
inline std::vector<float>*& ray_dump() { static thread_local std::vector<float>* v = nullptr; return v; }
// ... and the closest-hit queries' (tools/closest_probe.py)
inline std::vector<float>*& ray_dump_closest() { static thread_local std::vector<float>* v = nullptr; return v; }
#endif
// BOT (the cooperative traversals): entries can also be taken from the bottom (the oldest, highest
// in the tree), pop_bottom; the memory part is then [lo, msp).
template <int K, bool BOT = false>
struct TravStack {
  int s[K > 0 ? K : 1];
  int nreg, msp;
  int lo;     // BOT: first valid memory entry (0 otherwise)
  int* mem;   // a separate private array, so that s[] / nreg / msp stay in registers
  int* lds;   // this lane's LDS overflow slots (stride kLdsStackStride), or null
  BDPT_HD explicit TravStack(int* m, int* l = nullptr) : nreg(0), msp(0), lo(0), mem(m), lds(l) {}
  BDPT_HD void clear() { nreg = 0; msp = 0; lo = 0; }
  BDPT_HD int size() const { return nreg + msp - (BOT ? lo : 0); }
  BDPT_HD void put(int k, int v) {
#if defined(__HIP_DEVICE_COMPILE__)
    if (kLdsStack > 0 && lds && k < kLdsStack) {
      *(__attribute__((address_space(3))) int*)(lds + k * kLdsStackStride) = v;
      return;
    }
#endif
    mem[k] = v;
  }
  BDPT_HD int get(int k) const {
#if defined(__HIP_DEVICE_COMPILE__)
    if (kLdsStack > 0 && lds && k < kLdsStack) return *(const __attribute__((address_space(3))) int*)(lds + k * kLdsStackStride);
#endif
    return mem[k];
  }
  BDPT_HD void push(int v) {
    if (K == 0) {
      if (BOT && msp == lo) { msp = 0; lo = 0; }
      put(msp++, v);
      return;
    }
    if (nreg == K) {
      if (BOT && msp == lo) { msp = 0; lo = 0; }
      put(msp++, s[K - 1]);
    } else {
      nreg++;
    }
#pragma unroll
    for (int k = K - 1; k > 0; k--) s[k] = s[k - 1];
    s[0] = v;
  }
  BDPT_HD bool pop(int& v) {
    if (K > 0 && nreg > 0) {
      v = s[0];
#pragma unroll
      for (int k = 0; k + 1 < K; k++) s[k] = s[k + 1];
      nreg--;
      return true;
    }
    if (msp == (BOT ? lo : 0)) return false;
    v = get(--msp);
    return true;
  }
  // the oldest entry (BOT); the memory part only while its indices stay low (the array holds
  // kStackMax entries and lo only grows until the memory part empties)
  BDPT_HD bool can_pop_bottom() const { return size() > 0 && msp < kStackMax / 2; }
  BDPT_HD bool pop_bottom(int& v) {
    if (msp > lo) {
      v = get(lo++);
      if (lo == msp) { lo = 0; msp = 0; }
      return true;
    }
    if (K > 0 && nreg > 0) {
      v = s[0];
#pragma unroll
      for (int k = 1; k < K; k++)
        if (k < nreg) v = s[k];
      nreg--;
      return true;
    }
    return false;
  }
};

struct RayInv {
  f3 o, d, inv, oi;   // oi = o * inv: slab planes are fma(p, inv, -oi)
  // 4-wide nodes: byte offset (0 or 16) of each axis' near plane row within its lo / hi row pair
  // (the hi row when the direction component is negative), so that a lane loads its near and far
  // rows directly and the per-axis min / max of the two plane distances disappears
  int nx, ny, nz;
};
// A zero direction component would give an infinite inverse and NaN / wrong-signed plane distances
// (inf - inf); it is replaced by +-2^-100, whose plane distances are huge and of the right sign, so a
// parallel ray is inside a slab exactly when its origin is (up to the boxes' padding).
BDPT_HD float safe_inv(float x) {
  const float tiny = 7.88860905e-31f;   // 2^-100
  return 1.0f / (fabsf(x) < tiny ? copysignf(tiny, x) : x);
}
BDPT_HD RayInv make_rayinv(f3 o, f3 d) {
  RayInv r;
  r.o = o; r.d = d;
  r.inv = mk3(safe_inv(d.x), safe_inv(d.y), safe_inv(d.z));
  r.oi = mk3(o.x * r.inv.x, o.y * r.inv.y, o.z * r.inv.z);
  r.nx = r.inv.x < 0.0f ? 16 : 0;
  r.ny = r.inv.y < 0.0f ? 16 : 0;
  r.nz = r.inv.z < 0.0f ? 16 : 0;
  return r;
}
// Slab test against a padded (conservative) box (2-wide nodes; 4-wide nodes load the near and far
// rows directly, node_step). The fused form rounds differently from (p - o) * inv by at most ulp(o * inv) in t, far inside
// the 2^-16 box padding, so it never culls a box a hit lies in (results do not depend on it).
BDPT_HD void slab(const RayInv& r, float lx, float ly, float lz_, float hx, float hy, float hz,
                  float* tn, float* tf) {
  const float t0x = fmaf(lx, r.inv.x, -r.oi.x), t1x = fmaf(hx, r.inv.x, -r.oi.x);
  const float t0y = fmaf(ly, r.inv.y, -r.oi.y), t1y = fmaf(hy, r.inv.y, -r.oi.y);
  const float t0z = fmaf(lz_, r.inv.z, -r.oi.z), t1z = fmaf(hz, r.inv.z, -r.oi.z);
  const float n = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fminf(t0z, t1z));
  const float f = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fmaxf(t0z, t1z));
  *tn = n;
  *tf = f * 1.00000024f;
}

// Traversal loops are "while-while" (Aila & Laine 2009): an inner loop descends internal nodes
// until this lane stands on a leaf (or its stack is empty), then the leaf's primitives are tested.
// In a wave, every lane runs node steps together and then leaf tests together, instead of each
// iteration paying for both code paths. Each lane visits nodes in the same near-first order as a
// plain loop, so hits and counters do not change.
constexpr int kTravDone = (int)0x80000000;   // not a valid leaf reference (start would be 2^24)

// Scene fetches with explicit address spaces on the device: the LDS copy is read with ds_read and
// the HBM arrays with global_load (through a generic pointer both would compile to flat_load).
BDPT_HD float4 ld_lds4(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(3))) float4*)p;
#else
  return *p;
#endif
}
BDPT_HD float4 ld_glb4(const float4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(1))) float4*)p;
#else
  return *p;
#endif
}
// geometry record k (3 float4 per primitive): LDS copy in LDS mode 1, else HBM
template <int LM>
BDPT_HD float4 ld_geom(const SceneView& S, int k) {
  return LM == 1 || LM == 3 ? ld_lds4(S.lgeom + k) : ld_glb4(S.geom + k);
}
// primitive pi's whole record (3 float4). From HBM: the array's base as the scalar part of the
// address, a 32-bit per-lane offset, the rows' 0 / 16 / 32 in the immediate field.
template <int LM>
BDPT_HD void ld_rec3(const SceneView& S, int pi, float4& a0, float4& a1, float4& a2) {
  if (LM == 1 || LM == 3) {
    a0 = ld_lds4(S.lgeom + 3 * pi); a1 = ld_lds4(S.lgeom + 3 * pi + 1); a2 = ld_lds4(S.lgeom + 3 * pi + 2);
  } else {
    const char* b = (const char*)S.geom;
    const size_t o = (size_t)((uint32_t)pi * 48u);
    a0 = ld_glb4((const float4*)(b + o));
    a1 = ld_glb4((const float4*)(b + 16 + o));
    a2 = ld_glb4((const float4*)(b + 32 + o));
  }
}
BDPT_HD int ld_lds_i(const int* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *(const __attribute__((address_space(3))) int*)p;
#else
  return *p;
#endif
}
// A 4-wide node's rows as the ray sees them: v[0] / v[1] = the x plane rows nearer / farther along
// the ray (lo.x / hi.x, swapped when the direction's x is negative), v[2] / v[3] y, v[4] / v[5] z,
// v[6] the child references. Byte offsets within node ref: near = 128 ref + 32 a + n_a, far =
// 128 ref + 32 a + 16 - n_a. The address is the node array's base (wave-uniform: the scalar part of
// a global load) plus a 32-bit per-lane byte offset, the row's constant part in the immediate field:
// against a 64-bit address per row (round 6, profiles/r06qrs_ab_lean_node.log) the per-ray offsets
// take 6 VGPRs instead of 12 and the north-star kernel's static scratch instructions fall 236 -> 187.
// 32-bit offsets suffice: a scene holds < 2^24 primitive references (bdpt_scene.cpp), so < 2^25 binary
// and fewer 4-wide nodes, 128 ref + 112 < 2^32; the records (ld_rec3) are < 48 * 2^24 bytes.
BDPT_HD void ld_node4_oct_glb(const float4* nodes, int ref, const RayInv& r, float4* v) {
  const char* b = (const char*)nodes;
  const uint32_t o = (uint32_t)ref * 128u;
  const uint32_t nx = (uint32_t)r.nx, ny = (uint32_t)r.ny, nz = (uint32_t)r.nz;
  v[0] = ld_glb4((const float4*)(b + (size_t)(o + nx)));
  v[1] = ld_glb4((const float4*)(b + (size_t)(o + (16u - nx))));
  v[2] = ld_glb4((const float4*)(b + 32 + (size_t)(o + ny)));
  v[3] = ld_glb4((const float4*)(b + 32 + (size_t)(o + (16u - ny))));
  v[4] = ld_glb4((const float4*)(b + 64 + (size_t)(o + nz)));
  v[5] = ld_glb4((const float4*)(b + 64 + (size_t)(o + (16u - nz))));
  v[6] = ld_glb4((const float4*)(b + 96 + (size_t)o));
}
// The same as one asm block: the seven loads issue back to back under one wait. LM 0 (every node from
// HBM) needs it: left to the compiler, its loads were spaced by waits and the reference row (needed
// only once a child is hit) sank behind the slab tests, a second dependent fetch per step (LM 0
// 703 -> 647). LM 2's HBM path (waves with a lane below the treelet) runs faster with the compiler's
// schedule (north star 782 asm vs 792), so it keeps the C++ form.
BDPT_HD void ld_node4_oct_glb_asm(const float4* nodes, int ref, const RayInv& r, float4* v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const char* b = (const char*)nodes;
  const uint32_t o = (uint32_t)ref * 128u;
  const uint32_t nx = (uint32_t)r.nx, ny = (uint32_t)r.ny, nz = (uint32_t)r.nz;
  typedef float v4f __attribute__((ext_vector_type(4)));
  v4f t[7];
  asm volatile(
      "global_load_dwordx4 %0, %7, %14\n\t"
      "global_load_dwordx4 %1, %8, %14\n\t"
      "global_load_dwordx4 %2, %9, %14 offset:32\n\t"
      "global_load_dwordx4 %3, %10, %14 offset:32\n\t"
      "global_load_dwordx4 %4, %11, %14 offset:64\n\t"
      "global_load_dwordx4 %5, %12, %14 offset:64\n\t"
      "global_load_dwordx4 %6, %13, %14 offset:96\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6])
      : "v"(o + nx), "v"(o + (16u - nx)), "v"(o + ny), "v"(o + (16u - ny)), "v"(o + nz), "v"(o + (16u - nz)),
        "v"(o), "s"(b));
#pragma unroll
  for (int k = 0; k < 7; k++) v[k] = make_float4(t[k].x, t[k].y, t[k].z, t[k].w);
#else
  ld_node4_oct_glb(nodes, ref, r, v);
#endif
}
// the same from the LDS copy
BDPT_HD void ld_node4_oct_lds(const float4* p, const RayInv& r, float4* v) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef float v4f __attribute__((ext_vector_type(4)));
  const uint32_t a = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float4*)p;
  const int nx = r.nx, ny = r.ny, nz = r.nz;
  v4f t[7];
  // one asm block of ds_read_b128 and a single wait (a node fetch that may come from LDS or HBM, as in
  // the treelet mode, otherwise compiles to flat_load for both): near rows at a + n + 32 axis, far
  // rows at a - n + 32 axis + 16
  asm volatile(
      "ds_read_b128 %0, %7\n\t"
      "ds_read_b128 %1, %8 offset:16\n\t"
      "ds_read_b128 %2, %9 offset:32\n\t"
      "ds_read_b128 %3, %10 offset:48\n\t"
      "ds_read_b128 %4, %11 offset:64\n\t"
      "ds_read_b128 %5, %12 offset:80\n\t"
      "ds_read_b128 %6, %13 offset:96\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "=&v"(t[5]), "=&v"(t[6])
      : "v"(a + nx), "v"(a - nx), "v"(a + ny), "v"(a - ny), "v"(a + nz), "v"(a - nz), "v"(a));
#pragma unroll
  for (int k = 0; k < 7; k++) v[k] = make_float4(t[k].x, t[k].y, t[k].z, t[k].w);
#else
  ld_node4_oct_glb(p, 0, r, v);
#endif
}

// One node of the descent: slab-test the children, continue with the nearest hit child, push the
// other hit children (farther first, so they pop near-first); pop when none is hit.
// Width 2, 4 float4: lo_l.xyz hi_l.x | hi_l.yz lo_r.xy | lo_r.z hi_r.xyz | refs
// Width 4, 8 float4: lo.x[4] | hi.x[4] | lo.y[4] | hi.y[4] | lo.z[4] | hi.z[4] | refs[4] | pad,
// fetched in near / far order per axis (ld_node4_oct_*)
// ORD: visit hit children near-first (closest-hit queries); any-hit queries take them in slot order.
// A child is entered when its slab interval, clipped to [tmin, tmax], is non-empty.
template <int K, int LM, int ORD = 1, bool BOT = false>
BDPT_HD int node_step(const SceneView& S, const RayInv& r, int ref, float tmin, float tmax, TravStack<K, BOT>& stk,
                      Counters& c) {
  constexpr int W = lm_width(LM), NU = node_used_f4(W);
  float4 v[NU];
  if (W == 4) {
    // rows in near / far order (ld_node4_oct_*). LM 2: the treelet (LDS) and HBM lanes of one wave
    // would run a lane-divergent if / else over the same registers — the global loads, a wait for
    // them (the ds_reads would overwrite their registers), then the ds_reads: HBM latency + LDS
    // latency. So only a wave whose lanes are all in the treelet reads LDS; any other wave fetches
    // every lane's node from HBM (the treelet nodes are there too, and hot in L2).
    if (LM == 2) {
      const bool in_lds = ref < S.ntop;
#if defined(__HIP_DEVICE_COMPILE__)
      const bool all_lds = __ballot(in_lds) == __ballot(true);
#else
      const bool all_lds = in_lds;
#endif
      if (all_lds) {
        ld_node4_oct_lds(S.lnodes + node_f4(W) * ref, r, v);
        c.lnodes += W;
      } else {
        ld_node4_oct_glb(S.nodes, ref, r, v);
      }
    } else if (LM == 1) {
      ld_node4_oct_lds(S.lnodes + node_f4(W) * ref, r, v);
      c.lnodes += W;
    } else {
      ld_node4_oct_glb_asm(S.nodes, ref, r, v);
    }
  } else if (LM == 1) {   // 2-wide, all nodes in LDS: plain ds_reads the compiler schedules
#pragma unroll
    for (int k = 0; k < NU; k++) v[k] = ld_lds4(S.lnodes + node_f4(W) * ref + k);
    c.lnodes += W;
  } else {
#pragma unroll
    for (int k = 0; k < NU; k++) v[k] = ld_glb4(S.nodes + node_f4(W) * ref + k);
  }
  if (W == 2) {
    const float4 a = v[0], b = v[1], cc = v[2], e = v[3 % NU];
    c.nodes += 2;
    float tnl, tfl, tnr, tfr;
    slab(r, a.x, a.y, a.z, a.w, b.x, b.y, &tnl, &tfl);
    slab(r, b.z, b.w, cc.x, cc.y, cc.z, cc.w, &tnr, &tfr);
    const bool hl = fmaxf(tnl, tmin) <= fminf(tfl, tmax);
    const bool hr = fmaxf(tnr, tmin) <= fminf(tfr, tmax);
    const int lref = __float_as_int(e.x), rref = __float_as_int(e.y);
    if (hl && hr) {
      const bool lfirst = ORD == 0 || tnl <= tnr;
      stk.push(lfirst ? rref : lref);
      return lfirst ? lref : rref;
    }
    if (hl) return lref;
    if (hr) return rref;
    int nx;
    return stk.pop(nx) ? nx : kTravDone;
  } else {
    c.nodes += 4;
    int r0, r1, r2, r3;
    float tn0, tn1, tn2, tn3;
    bool h0, h1, h2, h3;
    const float4 lx = v[0], hx = v[1], ly = v[2 % NU], hy = v[3 % NU];
    const float4 lz = v[4 % NU], hz = v[5 % NU], e = v[6 % NU];
    r0 = __float_as_int(e.x); r1 = __float_as_int(e.y); r2 = __float_as_int(e.z); r3 = __float_as_int(e.w);
    float tf;
    // lx / ly / lz are the near rows, hx / hy / hz the far rows (ld_node4_oct_*): with a finite
    // inverse the near plane's distance is the smaller of the two (the fma is monotone in the plane
    // coordinate), so this is slab()'s test without its per-axis min / max — 6 fewer VALU per child,
    // the same visits. Measured against slab() (profiles/r05l_ab_oct_rows.log): north star +0.3 %,
    // C5-shaped +1.2 %, CBbunny +0.3 %, the stand-in with the tree in HBM (LM 0) +2.5 %.
#define BDPT_SLAB_OCT(C, TN, TF)                                                             \
  {                                                                                          \
    TN = fmaxf(fmaxf(fmaf(lx.C, r.inv.x, -r.oi.x), fmaf(ly.C, r.inv.y, -r.oi.y)),            \
               fmaf(lz.C, r.inv.z, -r.oi.z));                                                \
    TF = fminf(fminf(fmaf(hx.C, r.inv.x, -r.oi.x), fmaf(hy.C, r.inv.y, -r.oi.y)),            \
               fmaf(hz.C, r.inv.z, -r.oi.z)) * 1.00000024f;                                  \
  }
    // An empty slot (reference kTravDone) holds an inverted infinite box (bdpt_scene.cpp): its near
    // distance is +inf and its far one -inf, so its test fails without a look at the reference, and
    // the reference row is needed only once a child is hit (round 6: north star +1.7 % by itself).
    BDPT_SLAB_OCT(x, tn0, tf);
    h0 = fmaxf(tn0, tmin) <= fminf(tf, tmax);
    BDPT_SLAB_OCT(y, tn1, tf);
    h1 = fmaxf(tn1, tmin) <= fminf(tf, tmax);
    BDPT_SLAB_OCT(z, tn2, tf);
    h2 = fmaxf(tn2, tmin) <= fminf(tf, tmax);
    BDPT_SLAB_OCT(w, tn3, tf);
    h3 = fmaxf(tn3, tmin) <= fminf(tf, tmax);
#undef BDPT_SLAB_OCT
    if (ORD == 0) {
      // continue with the lowest hit slot, push the others
      int nx = kTravDone;
      if (h3) nx = r3;
      if (h2) { if (nx != kTravDone) stk.push(nx); nx = r2; }
      if (h1) { if (nx != kTravDone) stk.push(nx); nx = r1; }
      if (h0) { if (nx != kTravDone) stk.push(nx); nx = r0; }
      if (nx == kTravDone && !stk.pop(nx)) return kTravDone;
      return nx;
    }
    // sort key: entry distance of a hit child, +inf for a miss or an empty slot
    float k0 = h0 ? tn0 : INFINITY, k1 = h1 ? tn1 : INFINITY, k2 = h2 ? tn2 : INFINITY, k3 = h3 ? tn3 : INFINITY;
    // 5-comparator sorting network on (key, ref)
#define BDPT_CSWAP(ka, ra, kb, rb)                          \
  {                                                         \
    const bool sw = kb < ka;                                \
    const float tk = sw ? kb : ka; kb = sw ? ka : kb; ka = tk; \
    const int tr = sw ? rb : ra; rb = sw ? ra : rb; ra = tr;   \
  }
    BDPT_CSWAP(k0, r0, k1, r1);
    BDPT_CSWAP(k2, r2, k3, r3);
    BDPT_CSWAP(k0, r0, k2, r2);
    BDPT_CSWAP(k1, r1, k3, r3);
    BDPT_CSWAP(k1, r1, k2, r2);
#undef BDPT_CSWAP
    if (!(k0 < INFINITY)) {
      int nx;
      return stk.pop(nx) ? nx : kTravDone;
    }
    // the keys are sorted, so a later child is hit only if the earlier ones are: nested, a wave skips
    // the deeper pushes unless one of its lanes has that many hit children (against three flat
    // conditional pushes: north star +1.4 %, C5-shaped +1.8 %, profiles/r06z6_ab_push_nest.log)
    if (k1 < INFINITY) {
      if (k2 < INFINITY) {
        if (k3 < INFINITY) stk.push(r3);
        stk.push(r2);
      }
      stk.push(r1);
    }
    return r0;
  }
}

// Closest hit in [tmin, tmax]; ties in t go to the larger DFS position (reference order).
template <int LM = 0, int K = 0>
BDPT_HD bool trace_closest(const SceneView& S, f3 o, f3 d, float tmin, float tmax, Hit& h, Counters& c) {
  RayInv r = make_rayinv(o, d);
  h.t = tmax;
  h.prim = -1;
  h.key = -1;
  h.b1 = 0; h.b2 = 0;
  int stack_mem[kStackMax];
  TravStack<K> stk(stack_mem, LM == 1 || LM == 2 ? lane_stack(S) : nullptr);
  int ref = S.root;
  c.closest++;
#if defined(BDPT_STEP_HIST) && !defined(__HIP_DEVICE_COMPILE__)
  // CPU diagnostics (tools/step_hist.py): the histogram of node steps per closest-hit query
  struct StepHist {
    const Counters& c;
    uint32_t n0;
    ~StepHist() {
      if (step_hist_nested()) return;
      const uint32_t s = (c.nodes - n0) / (uint32_t)lm_width(LM);
      step_hist()[s < 255 ? s : 255]++;
    }
  } step_hist_{c, c.nodes};
  if (ray_dump_closest() && !step_hist_nested()) {
    const float rv[8] = {o.x, o.y, o.z, d.x, d.y, d.z, tmin, tmax};
    ray_dump_closest()->insert(ray_dump_closest()->end(), rv, rv + 8);
  }
#endif
  int li = 0;
  if (LM == 3 && S.fn > 0) {
    // the flat list as one run of primitives, the next record's loads issued before this test
    float4 a0, a1, a2;
    ld_rec3<LM>(S, 0, a0, a1, a2);
    for (int pi = 0; pi < S.fn; pi++) {
      BDPT_LANE_PROF(c, LP_CPRIM);
      const float4 g0 = a0, g1 = a1, g2 = a2;
      ld_rec3<LM>(S, pi + 1 < S.fn ? pi + 1 : pi, a0, a1, a2);
      float t, b1 = 0, b2 = 0;
      bool ok;
      int key;
      if ((S.fsph >> pi) & 1u) {
        c.sphs++;
        ok = sph_test(g0, o, d, tmin, h.t, &t);
        key = __float_as_int(g1.x);
      } else {
        c.tris++;
        ok = tri_test(g0, g1, g2, o, d, tmin, h.t, &t, &b1, &b2);
        key = __float_as_int(g2.y);
      }
      if (ok & ((t < h.t) | (key > h.key))) {
        h.t = t; h.prim = pi; h.key = key; h.b1 = b1; h.b2 = b2;
      }
    }
    if (h.prim >= 0) c.hits++;
    return h.prim >= 0;
  }
  float4 a0, a1, a2;
  // the primitives of leaf lf, closest hit so far in h
  auto test_leaf = [&](int lf) {
    const int st = leaf_start(lf), cnt = leaf_count(lf), sm = leaf_sph_mask(lf);
    if constexpr (leaf_prefetch(LM)) {
      ld_rec3<LM>(S, st, a0, a1, a2);
    }
    for (int k = 0; k < cnt; k++) {
      BDPT_LANE_PROF(c, LP_CPRIM);
      const int pi = st + k;
      float t, b1 = 0, b2 = 0;
      bool ok;
      int key;
      if constexpr (leaf_prefetch(LM)) {
        // this record was loaded one test ahead; issue the next one's loads (if any) before testing it
        const float4 g0 = a0, g1 = a1, g2 = a2;
        if (k + 1 < cnt) ld_rec3<LM>(S, pi + 1, a0, a1, a2);
        if ((sm >> k) & 1) {
          c.sphs++;
          ok = sph_test(g0, o, d, tmin, h.t, &t);
          key = __float_as_int(g1.x);
        } else {
          c.tris++;
          ok = tri_test(g0, g1, g2, o, d, tmin, h.t, &t, &b1, &b2);
          key = __float_as_int(g2.y);
        }
      } else {
        if ((sm >> k) & 1) {
          c.sphs++;
          ok = sph_test(ld_geom<LM>(S, 3 * pi), o, d, tmin, h.t, &t);
          key = ok ? __float_as_int(ld_geom<LM>(S, 3 * pi + 1).x) : 0;
        } else {
          c.tris++;
          const float4 g2 = ld_geom<LM>(S, 3 * pi + 2);
          ok = tri_test(ld_geom<LM>(S, 3 * pi), ld_geom<LM>(S, 3 * pi + 1), g2, o, d, tmin, h.t, &t, &b1, &b2);
          key = __float_as_int(g2.y);
        }
      }
      // t <= h.t here; an equal t replaces the hit only if it comes later in the reference's DFS
      // leaf order (the reference keeps the last of equal-t hits)
      if (ok & ((t < h.t) | (key > h.key))) {
        h.t = t; h.prim = pi; h.key = key; h.b1 = b1; h.b2 = b2;
      }
    }
  };
  if constexpr (spec_trav(LM)) {
    // speculative while-while: a lane's first leaf is postponed and the lane goes on descending its
    // stack while other lanes still look for theirs; leaves are tested once every lane has one
    int pend = 0;
    for (;;) {
      while (ref >= 0) {
        BDPT_LANE_PROF(c, LP_CNODE);
        ref = node_step<K, LM, kClosestOrd>(S, r, ref, tmin, h.t, stk, c);
        if ((ref < 0) & (ref != kTravDone) & (pend == 0)) {
          pend = ref;
          if (!stk.pop(ref)) ref = kTravDone;
        }
        if (wave_count((pend == 0) & (ref >= 0)) == 0) break;
      }
      while (pend != 0) {
        test_leaf(pend);
        pend = 0;
        if ((ref < 0) & (ref != kTravDone)) {
          pend = ref;
          if (!stk.pop(ref)) ref = kTravDone;
        }
      }
      if (ref == kTravDone) break;
    }
  } else {
    for (;;) {
      if (LM == 3) {
        if (li >= S.nleaves) break;
        ref = ld_lds_i(S.lleaves + li++);
      }
      while (ref >= 0) {
        BDPT_LANE_PROF(c, LP_CNODE);
        ref = node_step<K, LM, kClosestOrd>(S, r, ref, tmin, h.t, stk, c);
      }
      if (ref == kTravDone) break;
      test_leaf(ref);
      if (LM != 3 && !stk.pop(ref)) break;
    }
  }
  if (h.prim >= 0) c.hits++;
#if defined(BDPT_STEP_HIST) && !defined(__HIP_DEVICE_COMPILE__)
  // entries 512..767: node steps of the same query given its final hit distance up front (the
  // ordering-independent part); 768..1023: node steps of the queries that hit nothing
  if (!step_hist_nested()) {
    step_hist_nested() = 1;
    Counters c2 = {};
    Hit h2;
    trace_closest<LM, K>(S, o, d, tmin, h.prim >= 0 ? h.t * 1.000001f : tmax, h2, c2);
    const uint32_t s2 = c2.nodes / (uint32_t)lm_width(LM);
    step_hist()[512 + (s2 < 255 ? s2 : 255)]++;
    if (h.prim < 0) step_hist()[768 + (s2 < 255 ? s2 : 255)]++;
    step_hist_nested() = 0;
  }
#endif
  return h.prim >= 0;
}

// Any hit in [tmin, tmax] (connection rays, bidirection.cpp:418-433).
template <int LM = 0, int K = 0>
BDPT_HD bool trace_any(const SceneView& S, f3 o, f3 d, float tmin, float tmax, Counters& c) {
  RayInv r = make_rayinv(o, d);
  int stack_mem[kStackMax];
  TravStack<K> stk(stack_mem, LM == 1 || LM == 2 ? lane_stack(S) : nullptr);
  int ref = S.root;
  c.shadow++;
#if defined(BDPT_STEP_HIST) && !defined(__HIP_DEVICE_COMPILE__)
  struct StepHistAny {   // any-hit queries: histogram entries 256..511
    const Counters& c;
    uint32_t n0;
    ~StepHistAny() {
      if (step_hist_nested()) return;
      const uint32_t s = (c.nodes - n0) / (uint32_t)lm_width(LM);
      step_hist()[256 + (s < 255 ? s : 255)]++;
    }
  } step_hist_{c, c.nodes};
  if (ray_dump() && !step_hist_nested()) {
    const float rv[8] = {o.x, o.y, o.z, d.x, d.y, d.z, tmin, tmax};
    ray_dump()->insert(ray_dump()->end(), rv, rv + 8);
  }
#endif
  int li = 0;
  if (LM == 3 && S.fn > 0) {
    float4 a0, a1, a2;
    ld_rec3<LM>(S, 0, a0, a1, a2);
    for (int pi = 0; pi < S.fn; pi++) {
      BDPT_LANE_PROF(c, LP_APRIM);
      const float4 g0 = a0, g1 = a1, g2 = a2;
      ld_rec3<LM>(S, pi + 1 < S.fn ? pi + 1 : pi, a0, a1, a2);
      float t, b1, b2;
      bool ok;
      if ((S.fsph >> pi) & 1u) {
        c.sphs++;
        ok = sph_test(g0, o, d, tmin, tmax, &t);
      } else {
        c.tris++;
        ok = tri_test(g0, g1, g2, o, d, tmin, tmax, &t, &b1, &b2);
      }
      if (ok) return true;
    }
    return false;
  }
  float4 a0, a1, a2;
  // true if a primitive of leaf lf is hit on [tmin, tmax]
  auto test_leaf = [&](int lf) -> bool {
    const int st = leaf_start(lf), cnt = leaf_count(lf), sm = leaf_sph_mask(lf);
    if constexpr (leaf_prefetch(LM)) {
      ld_rec3<LM>(S, st, a0, a1, a2);
    }
    for (int k = 0; k < cnt; k++) {
      BDPT_LANE_PROF(c, LP_APRIM);
      const int pi = st + k;
      float t, b1, b2;
      bool ok;
      if constexpr (leaf_prefetch(LM)) {
        const float4 g0 = a0, g1 = a1, g2 = a2;
        if (k + 1 < cnt) ld_rec3<LM>(S, pi + 1, a0, a1, a2);
        if ((sm >> k) & 1) {
          c.sphs++;
          ok = sph_test(g0, o, d, tmin, tmax, &t);
        } else {
          c.tris++;
          ok = tri_test(g0, g1, g2, o, d, tmin, tmax, &t, &b1, &b2);
        }
      } else {
        if ((sm >> k) & 1) {
          c.sphs++;
          ok = sph_test(ld_geom<LM>(S, 3 * pi), o, d, tmin, tmax, &t);
        } else {
          c.tris++;
          ok = tri_test(ld_geom<LM>(S, 3 * pi), ld_geom<LM>(S, 3 * pi + 1), ld_geom<LM>(S, 3 * pi + 2), o, d, tmin, tmax, &t, &b1, &b2);
        }
      }
      if (ok) return true;
    }
    return false;
  };
  if constexpr (spec_trav(LM)) {
    // speculative while-while, as in trace_closest
    int pend = 0;
    for (;;) {
      while (ref >= 0) {
        BDPT_LANE_PROF(c, LP_ANODE);
        ref = node_step<K, LM, kAnyOrd>(S, r, ref, tmin, tmax, stk, c);
        if ((ref < 0) & (ref != kTravDone) & (pend == 0)) {
          pend = ref;
          if (!stk.pop(ref)) ref = kTravDone;
        }
        if (wave_count((pend == 0) & (ref >= 0)) == 0) break;
      }
      while (pend != 0) {
        if (test_leaf(pend)) return true;
        pend = 0;
        if ((ref < 0) & (ref != kTravDone)) {
          pend = ref;
          if (!stk.pop(ref)) ref = kTravDone;
        }
      }
      if (ref == kTravDone) return false;
    }
  } else {
    for (;;) {
      if (LM == 3) {
        if (li >= S.nleaves) return false;
        ref = ld_lds_i(S.lleaves + li++);
      }
      while (ref >= 0) {
        BDPT_LANE_PROF(c, LP_ANODE);
        ref = node_step<K, LM, kAnyOrd>(S, r, ref, tmin, tmax, stk, c);
      }
      if (ref == kTravDone) return false;
      if (test_leaf(ref)) return true;
      if (LM != 3 && !stk.pop(ref)) return false;
    }
  }
}

// Shading record of a closest hit: interpolated normal (triangle.cpp:80-82) or sphere normal
// (sphere.cpp:78-81), and the material.
template <int LM = 0>
BDPT_HD void shade_hit(const SceneView& S, const Hit& h, f3 o, f3 d, f3* n_out, int* mat_out) {
  float4 s0, s1, s2;
  if (LM == 3) {   // the flat list's shading records are staged in LDS with its geometry
    const float4* sh = S.lshade + 3 * h.prim;
    s0 = ld_lds4(sh); s1 = ld_lds4(sh + 1); s2 = ld_lds4(sh + 2);
  } else {
    const float4* sh = S.shade + 3 * h.prim;
    s0 = ld_glb4(sh); s1 = ld_glb4(sh + 1); s2 = ld_glb4(sh + 2);
  }
  *mat_out = __float_as_int(s2.y);
  if (__float_as_int(s2.z) != 0) {   // sphere: center in geom
    float4 g = ld_geom<LM>(S, 3 * h.prim);
    f3 p = add(o, smul(h.t, d));
    *n_out = normalize(sub(p, mk3(g.x, g.y, g.z)));
  } else {
    f3 n1 = mk3(s0.x, s0.y, s0.z), n2 = mk3(s0.w, s1.x, s1.y), n3 = mk3(s1.z, s1.w, s2.x);
    f3 n = add(add(muls(n1, 1 - h.b1 - h.b2), smul(h.b1, n2)), smul(h.b2, n3));
    *n_out = normalize(n);
  }
}

// ------------------------------------------------------------------------------------------------
// Samplers (sampler.cpp) and BSDFs (bsdf.cpp, advanced_bsdf.cpp)
BDPT_HD void grid2d(Rng& g, float* x, float* y) {   // Vector2D(U(), U()): y is drawn first
  float b = rng_next(g);
  float a = rng_next(g);
  *x = a;
  *y = b;
}
BDPT_HD f3 cosine_hemi(Rng& g, float* pdf) {   // sampler.cpp:76-86
  float Xi1 = rng_next(g);
  float Xi2 = rng_next(g);
  float r = sqrtf(Xi1);
  *pdf = sqrtf(1 - Xi1) / BDPT_PI_F;
  float c, s;
  cos_sin_2pi(Xi2, &c, &s);
  return mk3(r * c, r * s, sqrtf(1 - Xi1));
}
BDPT_HD float cosine_pdf_z(float z) { return z > 0 ? z / BDPT_PI_F : 0.0f; }   // sampler.cpp:92-95

BDPT_HD bool is_delta(int type) { return type == MAT_MIRROR || type == MAT_GLASS || type == MAT_REFRACTION; }

BDPT_HD bool refract_dir(f3 wo, f3* wi, float ior) {   // advanced_bsdf.cpp:279-303
  bool enter = wo.z > 0;
  float eta = enter ? 1.0f / ior : ior;
  float z_sq = 1 - eta * eta * (1 - wo.z * wo.z);
  if (z_sq < 0) return false;
  float sgn = enter ? -1.0f : 1.0f;
  *wi = mk3(-eta * wo.x, -eta * wo.y, sgn * sqrtf(z_sq));
  return true;
}

// MicrofacetBSDF (advanced_bsdf.cpp:46-142, bsdf.h:176-184) in the device semantics (PathTracer
// only): cos(acos z) = z, tan(acos z) = sqrt(1 - z^2) / z, integer powers by products, erf / exp /
// log from the fp32 math library (oracle mode 2 restates it, oracle/bdpt_oracle.cpp mf_*).
BDPT_HD float mf_lambda(float alpha, f3 w) {
  const float c = fminf(fmaxf(w.z, (float)(-1.0 + 1e-5)), (float)(1.0 - 1e-5));
  const float t = sqrtf(1.0f - c * c) / c;
  const float a = 1.0f / (alpha * t);
  return 0.5f * (erff(a) - 1.0f + expf(-a * a) / (a * BDPT_PI_F));
}
BDPT_HD float mf_G(float alpha, f3 wo, f3 wi) { return 1.0f / (1.0f + mf_lambda(alpha, wi) + mf_lambda(alpha, wo)); }
BDPT_HD float mf_D(float alpha, f3 h) {
  const float c = h.z;
  const float t = sqrtf(fmaxf(0.0f, 1.0f - c * c)) / c;
  const float q = t / alpha;
  const float c2 = c * c;
  return expf(-(q * q)) / (BDPT_PI_F * alpha * alpha * (c2 * c2));
}
BDPT_HD f3 mf_F(const DMat& M, f3 wi) {   // (Rs + Rp) / 2, CGL operator order
  const f3 eta = mk3(M.a[0], M.a[1], M.a[2]), k = mk3(M.b[0], M.b[1], M.b[2]);
  const float c = fabsf(wi.z) / norm(wi);
  const float c2 = c * c;
  const f3 e2k2 = add(mul(eta, eta), mul(k, k));
  const f3 t = muls(smul(2.0f, eta), c);
  const f3 Rs = mk3((e2k2.x - t.x + c2) / (e2k2.x + t.x + c2), (e2k2.y - t.y + c2) / (e2k2.y + t.y + c2),
                    (e2k2.z - t.z + c2) / (e2k2.z + t.z + c2));
  const f3 e = muls(e2k2, c2);
  const f3 Rp = mk3((e.x - t.x + 1.0f) / (e.x + t.x + 1.0f), (e.y - t.y + 1.0f) / (e.y + t.y + 1.0f),
                    (e.z - t.z + 1.0f) / (e.z + t.z + 1.0f));
  return divs(add(Rs, Rp), 2.0f);
}
BDPT_HD f3 mf_f(const DMat& M, f3 wo, f3 wi) {
  if (wo.z <= BDPT_EPS_F || wi.z <= BDPT_EPS_F) return splat3(0);
  const f3 h = normalize(add(wo, wi));
  return divs(muls(muls(mf_F(M, wi), mf_G(M.alpha, wo, wi)), mf_D(M.alpha, h)), 4.0f * wo.z * wi.z);
}
BDPT_HD f3 mf_sample_f(const DMat& M, Rng& g, f3 wo, f3* wi, float* pdf) {
  float rx, ry;
  grid2d(g, &rx, &ry);
  const float alpha = M.alpha;
  const float tt = sqrtf(-alpha * alpha * logf(1.0f - rx));   // tan(theta)
  const float ct = 1.0f / sqrtf(1.0f + tt * tt);
  const float st = tt * ct;
  float cp, sp;
  cos_sin_2pi(ry, &cp, &sp);
  const f3 h = mk3(st * cp, st * sp, ct);
  const float costheta = dot(wo, h) / norm(wo);
  const f3 d = sub(wo, muls(muls(h, costheta), norm(wo)));
  *wi = normalize(sub(muls(muls(h, costheta), norm(wo)), d));
  if (wo.z <= BDPT_EPS_F || wi->z <= BDPT_EPS_F) {
    *pdf = 1;
    *wi = mk3(0, 0, 1);
    return splat3(0);
  }
  const float q = tt / alpha, c2 = ct * ct;
  const float p_theta = 2.0f * st * expf(-(q * q)) / (alpha * alpha * (c2 * ct));
  const float p_phi = 1.0f / (2.0f * BDPT_PI_F);
  const float pdf_h = p_theta * p_phi / st;
  *pdf = pdf_h / (4.0f * dot(*wi, h));
  return mf_f(M, wo, *wi);
}

BDPT_HD f3 sample_f(const DMat& M, Rng& g, f3 wo, f3* wi, float* pdf) {
  f3 A = mk3(M.a[0], M.a[1], M.a[2]);
  switch (M.type) {
    case MAT_MICROFACET: return mf_sample_f(M, g, wo, wi, pdf);
    case MAT_DIFFUSE: {
      *wi = cosine_hemi(g, pdf);
      if (wo.z < 0 || wi->z < 0) return splat3(0);
      return divs(A, BDPT_PI_F);
    }
    case MAT_EMISSION: {
      *pdf = 1.0f / BDPT_PI_F;
      *wi = cosine_hemi(g, pdf);
      return splat3(0);
    }
    case MAT_MIRROR: {
      *wi = mk3(-wo.x, -wo.y, wo.z);
      *pdf = 1;
      float ct = fabsf(wi->z) / norm(*wi);
      return divs(A, ct);
    }
    case MAT_REFRACTION: {
      f3 B = mk3(M.b[0], M.b[1], M.b[2]);
      if (!refract_dir(wo, wi, M.ior)) { *pdf = 1; return splat3(0); }
      *pdf = 1;
      float eta = wo.z > 0 ? 1.0f / M.ior : M.ior;
      float ct = fabsf(wi->z) / norm(*wi);
      return divs(divs(B, ct), eta * eta);
    }
    default: {   // glass (advanced_bsdf.cpp:198-237)
      f3 B = mk3(M.b[0], M.b[1], M.b[2]);
      f3 wr = mk3(-wo.x, -wo.y, wo.z), wt;
      bool tir = !refract_dir(wo, &wt, M.ior);
      if (tir) {
        *pdf = 1;
        *wi = wr;
        float ct = fabsf(wi->z) / norm(wo);
        return divs(A, ct);
      }
      float cref = fabsf(wt.z) / norm(wt);
      float eta = wo.z > 0 ? 1.0f / M.ior : M.ior;
      float x = (1 - eta) / (1 + eta);
      float R0 = x * x;
      float m = 1 - cref, m2 = m * m, m4 = m2 * m2;
      float Rf = R0 + (1 - R0) * (m4 * m);
      if (rng_next(g) < Rf) {
        *wi = wr;
        *pdf = Rf;
        float ct = fabsf(wi->z) / norm(*wi);
        return divs(smul(Rf, A), ct);
      }
      *wi = wt;
      *pdf = 1 - Rf;
      float ct = fabsf(wi->z) / norm(*wi);
      return divs(divs(smul(1 - Rf, B), ct), eta * eta);
    }
  }
}

// BSDF::sample_pdf with wo = 0 (as every MIS call site passes, bidirection.cpp:150,189,...).
// `n` is the vertex normal (the frame is rebuilt only for glass, which needs wi.x, wi.y).
BDPT_HD float pdf_b(const DMat& M, f3 n, f3 zh, f3 dw) {
  switch (M.type) {
    case MAT_DIFFUSE:
    case MAT_EMISSION: return cosine_pdf_z(lz(dw, zh));
    case MAT_MIRROR:
    case MAT_REFRACTION: return 1.0f;
    default: {
      Frame f = make_frame_hit(n);
      f3 wi = to_local(f, dw), wt;
      if (!refract_dir(wi, &wt, M.ior)) return 1.0f;
      float c = fabsf(wt.z) / norm(wt);
      float eta = M.ior;   // wo = 0: wo.z > 0 is false (advanced_bsdf.cpp:251)
      float x = (1 - eta) / (1 + eta);
      float R0 = x * x;
      float m = 1 - c, m2 = m * m, m4 = m2 * m2;
      float Rf = R0 + (1 - R0) * (m4 * m);
      if (wi.z > 0) return Rf;
      return 1 - Rf;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// EnvironmentLight (environment_light.cpp) in the device semantics: w points from the scene toward
// the environment (sample_L's *wi, sample_dir's r.d).
BDPT_HD int upper_idx(const float* a, int n, float u) {   // std::upper_bound(a, a + n, u) - a, <= n - 1
  int lo = 0, cnt = n;
  while (cnt > 0) {
    const int st = cnt >> 1, m = lo + st;
    if (!(u < a[m])) { lo = m + 1; cnt -= st + 1; }
    else cnt = st;
  }
  return lo < n ? lo : n - 1;
}
// The same index through a guide table gd[0..G] (gd[k] = upper_bound(a, a + n, k / G), G a power of
// two, bdpt_scene.cpp): u * G is exact, so the answer lies in [gd[k], gd[k + 1]] for k = floor(u * G)
// and only that range is searched (one or two dependent loads instead of log2 n).
BDPT_HD int upper_idx_guided(const float* a, int n, const int* gd, int G, float u) {
  int k = (int)(u * (float)G);
  k = k < 0 ? 0 : k > G - 1 ? G - 1 : k;
  int lo = gd[k], cnt = gd[k + 1] - lo;
  while (cnt > 0) {
    const int st = cnt >> 1, m = lo + st;
    if (!(u < a[m])) { lo = m + 1; cnt -= st + 1; }
    else cnt = st;
  }
  return lo < n ? lo : n - 1;
}
BDPT_HD f3 env_texel(const EnvView& E, int k) {
  const float* p = E.rgb + 3 * (size_t)k;
  return mk3(p[0], p[1], p[2]);
}
BDPT_HD f3 env_bilerp(const EnvView& E, float x, float y) {   // bilerp (:106-123)
  int right = lround_pos(x), left, v = lround_pos(y);
  const float u1 = ((float)right - x) + 0.5f;
  float v1;
  if (right == 0 || right == E.w) { left = E.w - 1; right = 0; }
  else left = right - 1;
  if (v == 0) { v = 1; v1 = 1.0f; }
  else if (v == E.h) { v = E.h - 1; v1 = 0.0f; }
  else v1 = ((float)v - y) + 0.5f;
  const int bottom = E.w * v, top = bottom - E.w;
  const float u0 = 1 - u1;
  const f3 a = add(muls(env_texel(E, top + left), u1), muls(env_texel(E, top + right), u0));
  const f3 b = add(muls(env_texel(E, bottom + left), u1), muls(env_texel(E, bottom + right), u0));
  return add(muls(a, v1), muls(b, 1 - v1));
}
// theta_phi_to_dir(xy_to_theta_phi(x, y)) (:88-104): phi = 2 pi x / w, theta = pi y / h;
// (cos(phi - pi) sin t, cos t, -sin(phi - pi) sin t) = (-cos phi sin t, cos t, sin phi sin t).
BDPT_HD f3 env_xy_to_dir(const EnvView& E, float x, float y, float* sin_theta) {
  float cp, sp, ct, st;
  cos_sin_2pi(x / (float)E.w, &cp, &sp);
  cos_sin_2pi((y / (float)E.h) * 0.5f, &ct, &st);
  *sin_theta = st;
  return mk3(-cp * st, ct, sp * st);
}
// theta_phi_to_xy(dir_to_theta_phi(u)) (:81-86, 97-102) for a unit u: theta = acos(u.y),
// phi = atan2(-u.z, u.x) + pi; sin(theta) as sqrt((1 - y)(1 + y)).
BDPT_HD void env_dir_to_xy(const EnvView& E, f3 u, float* x, float* y, float* sin_theta) {
  const float st = sqrtf(fmaxf(0.0f, (1.0f - u.y) * (1.0f + u.y)));
  const float th = atan2_det(st, u.y);
  const float ph = atan2_det(-u.z, u.x) + BDPT_PI_F;
  *x = ph / 2.0f / BDPT_PI_F * (float)E.w;
  *y = th / BDPT_PI_F * (float)E.h;
  *sin_theta = st;
}
// sample_dir (:159-168): the radiance arriving along -u from direction u
BDPT_HD f3 env_radiance(const EnvView& E, f3 u) {
  float x, y, st;
  env_dir_to_xy(E, u, &x, &y, &st);
  return env_bilerp(E, x, y);
}
// Solid-angle density of sample_L choosing direction u (the pdf sample_L returns, :152, for the
// texel u falls in); 0 at the poles.
BDPT_HD float env_pdf_dir(const EnvView& E, f3 u) {
  float x, y, st;
  env_dir_to_xy(E, u, &x, &y, &st);
  if (!(st > 0.0f)) return 0.0f;
  const int xi = (int)x, yi = (int)y;
  const int i = xi < E.w - 1 ? xi : E.w - 1, j = yi < E.h - 1 ? yi : E.h - 1;
  return E.pdf[E.w * j + i] * (float)(E.w * E.h) / (2.0f * BDPT_PI_F * BDPT_PI_F * st);
}
// sample_L's direction sampling (:126-156): row by the marginal CDF, column by the row's CDF, then
// a uniform jitter inside the texel; returns bilerp(xy) (4 uniforms).
BDPT_HD f3 env_sample_dir(const EnvView& E, Rng& g, f3* w, float* pdf) {
  float ux, uy;
  grid2d(g, &ux, &uy);
  int y, x;
  if (E.gmarg) {
    y = upper_idx_guided(E.marg, E.h, E.gmarg, E.gm, uy);
    x = upper_idx_guided(E.cond + (size_t)E.w * y, E.w, E.gcond + (size_t)(E.gc + 1) * y, E.gc, ux);
  } else {
    y = upper_idx(E.marg, E.h, uy);
    x = upper_idx(E.cond + (size_t)E.w * y, E.w, ux);
  }
  const float xf = (float)x + rng_next(g);
  const float yf = (float)y + rng_next(g);
  float st;
  *w = env_xy_to_dir(E, xf, yf, &st);
  *pdf = E.pdf[E.w * y + x] * (float)(E.w * E.h) / (2.0f * BDPT_PI_F * BDPT_PI_F * st);
  return env_bilerp(E, xf, yf);
}

// ------------------------------------------------------------------------------------------------
// Path vertices (PathVertex, bidirection.h:29-46) with the MIS path constants attached.
struct Vtx {
  f3 pos, n, zh, alpha;
  float fwd;   // MIS denominator of the step at this vertex (bidirection.cpp:194-211 / 257-280)
  float gp;    // MIS prefix: G of the vertex one step inward (see mis_horner), 0 at E[2] / L[1];
               // during the walk it holds the vertex's roulette probability q (PathVertex.q)
               // until the *_constants pass has consumed it
  int mat;     // -1: no BSDF (camera / light vertex); MAT_ENV_V: environment vertex
  float cq;    // > 0: can receive a connection — diffuse (the only BSDF with f != 0,
               // bsdf.cpp:52-62), seen from its front side (wo.z >= 0 toward the previous vertex),
               // alpha != 0 — and then equal to q; 0: cannot
};

struct LightSample {
  f3 pos, n, zh, alpha;
  float dir_pdf;
  float fwd;   // point_pdf / nL (the MIS denominator of the light end in environment scenes)
  bool env;    // environment light: n = zh = -w, pos unused
};

// A vertex as the path store holds it: the shading axis zh is not stored (it is zaxis(n), or n
// itself for an environment vertex, and is recomputed where a connection reads it), and in the
// reference-only kernels (EXT = false) the connectability flag rides in bit 16 of the material
// word, so a vertex is 12 dwords (48 B) instead of 16; EXT kernels keep cq (the roulette
// probability of a connectable vertex) as a 13th dword. The private segment is lane-interleaved
// per dword, so the dwords a kernel never touches cost no traffic.
struct VtxS {
  f3 pos;
  float fwd;
  f3 n;
  float gp;
  f3 alpha;
  int mb;     // material id (low 16 bits, signed); EXT = false: bit 16 = can_connect
  float cq;   // EXT only
};
BDPT_HD int vs_mat(const VtxS& s) { return (int)(short)(s.mb & 0xffff); }
template <bool EXT>
BDPT_HD void vtx_store(VtxS& s, const Vtx& v) {
  s.pos = v.pos; s.fwd = v.fwd; s.n = v.n; s.gp = v.gp; s.alpha = v.alpha;
  s.mb = (v.mat & 0xffff) | (!EXT && v.cq > 0.0f ? 0x10000 : 0);
  if (EXT) s.cq = v.cq;
}
template <bool EXT>
BDPT_HD Vtx vtx_load(const VtxS& s) {
  Vtx v;
  v.pos = s.pos; v.fwd = s.fwd; v.n = s.n; v.gp = s.gp; v.alpha = s.alpha;
  v.mat = vs_mat(s);
  v.cq = EXT ? s.cq : ((s.mb >> 16) != 0 ? 1.0f : 0.0f);
  v.zh = v.n;   // hit vertices: make_frame_hit; environment vertices: n = zh = -w; L[1]'s zh is never read
  return v;
}

// Per-subpath bit masks indexed by the reference's vertex index k <= MAXV + 1: 32 bits up to the
// m = 16 kernels (unchanged code), 64 for the m <= 32 and m <= 62 ones.
template <int MAXV>
using DeltaMask = typename std::conditional<
    (MAXV > 62), unsigned __int128, typename std::conditional<(MAXV > 29), uint64_t, uint32_t>::type>::type;
static_assert(sizeof(DeltaMask<62>) * 8 >= 62 + 2, "delta mask holds vertex indices up to MAXV + 1");
static_assert(sizeof(DeltaMask<126>) * 8 >= 126 + 2, "delta mask holds vertex indices up to MAXV + 1");

template <int MAXV>
struct Paths {
  VtxS E[MAXV];       // E[k] at index k-2 (k >= 2): eye hits
  VtxS L[MAXV + 1];   // L[k] at index k-1 (k >= 1): L[1] = light vertex, then hits
  int nE, nL;        // path sizes including v0, v1 (reference's vector sizes)
  DeltaMask<MAXV> dE, dL;   // delta-BSDF bit masks: bit k set <=> E[k] / L[k] is_delta()
  DeltaMask<MAXV> cE, cL;   // connectable vertices: bit k set <=> E[k] / L[k] has cq > 0
  DeltaMask<MAXV> sE;       // s = 0 sources: bit k set <=> E[k] is on an emitter or the environment
  float l1_dir_pdf;
  f3 l1_d;           // the light walk's first direction and its pdf (read back when it starts)
  float l1_pdf;
#ifdef BDPT_BOUND_WB2
  VtxS W2[2 * MAXV + 1];   // bound experiment (timing only): a second copy of every stored vertex
#endif
};
#ifdef BDPT_BOUND_WB2
// the copy is written with ordinary (vector) stores; one dword of it at an index the compiler cannot
// see is read back per sample (BDPT_WB2_USE), so that none of the stores can be dropped
template <bool EXT, int MAXV>
BDPT_HD void vtx_store_dup(Paths<MAXV>& P, const VtxS* slot, const Vtx& v) {
  vtx_store<EXT>(P.W2[slot - P.E], v);
}
template <int MAXV>
BDPT_HD void wb2_use(const Paths<MAXV>& P) {
#if defined(__HIP_DEVICE_COMPILE__)
  int k;
  asm volatile("v_mov_b32 %0, 0" : "=v"(k));
  const float x = P.W2[k].fwd;
  asm volatile("; wb2 use %0" ::"v"(x));
#endif
}
#define BDPT_WB2_DUP(P, slot, v) vtx_store_dup<EXT>(P, slot, v)
#define BDPT_WB2_USE(P) wb2_use(P)
#else
#define BDPT_WB2_DUP(P, slot, v) do {} while (0)
#define BDPT_WB2_USE(P) do {} while (0)
#endif

struct SampleParams {
  int W, H, spp, max_depth;
  uint64_t seed;
  int rr;   // Russian roulette (bdpt_params.russian_roulette; honoured by EXT kernels only)
};

// Power-heuristic sums in Horner form. Along a subpath walked from the connection endpoint
// inward, the reference accumulates ratio_k = f_end * ... * f_k and adds ratio_k^2 when neither
// vertex of step k is delta (t_k). Innermost first, the same sum is G_k = f_k^2 (t_k + G_{k-1});
// every interior factor f_k is a path constant (rev/fwd pdf ratio), so G up to the vertex below
// the endpoint is cached per vertex (Vtx::gp) and a connection costs O(1) instead of O(i + j).
// A term whose inner sum is exactly zero stays zero (no inf * 0); the oracle's mode 2 evaluates
// the identical expression (oracle/bdpt_oracle.cpp horner_step).
BDPT_HD float mis_horner(float f, bool t, float g) {
  const float s = t ? 1.0f + g : g;
  return s == 0.0f ? 0.0f : (f * f) * s;
}

// MIS step quantities between a vertex `cur` and a neighbour `oth` whose BSDF/frame is used:
// d = normalize(cur - oth), g = |(w2o(oth)*d).z * dot(d, cur.n)| / dist^2 (bidirection.cpp:151-158).
BDPT_HD float step_g(f3 cur_pos, f3 cur_n, f3 oth_pos, f3 oth_zh, f3* dw_out) {
  f3 dw = sub(cur_pos, oth_pos);
  float dist = norm(dw);
  dw = normalize(dw);
  float wz = lz(dw, oth_zh);
  *dw_out = dw;
  return fabsf(wz * dot(dw, cur_n)) / (dist * dist);
}
// The same with environment vertices: an env vertex sits at infinity in direction
// w, with n = zh = -w. oth env: d = -w and g = |dot(d, cur.n)| (the emission disk's planar density
// projected onto cur); cur env: d = w and g = 1 (densities of an env vertex are solid-angle ones).
BDPT_HD float step_gx(f3 cur_pos, f3 cur_n, bool cur_env, f3 oth_pos, f3 oth_zh, bool oth_env, f3* dw_out) {
  if (cur_env) { *dw_out = neg(cur_n); return 1.0f; }
  if (oth_env) { *dw_out = oth_zh; return fabsf(dot(oth_zh, cur_n)); }
  return step_g(cur_pos, cur_n, oth_pos, oth_zh, dw_out);
}
BDPT_HD bool is_env(const Vtx& v) { return v.mat == MAT_ENV_V; }

// AreaLight/PointLight BDPT methods (light.cpp:115-153, 219-284).
BDPT_HD bool light_contains(const DLight& l, f3 p) {
  f3 lp = mk3(l.pos[0], l.pos[1], l.pos[2]);
  if (l.type == LIGHT_POINT) return norm(sub(p, lp)) < BDPT_EPS_F;
  f3 d = normalize(sub(lp, p));
  return fabsf(dot(d, mk3(l.dir[0], l.dir[1], l.dir[2]))) < BDPT_EPS_F;
}
// sample_pdf's dir_pdf for a point known to be on the light; wi = direction of travel.
BDPT_HD float light_dir_pdf(const DLight& l, f3 wi) {
  if (l.type == LIGHT_POINT) return 0.25f / BDPT_PI_F;
  if (l.type == LIGHT_ENV) return 1.0f / l.area;   // planar density of the emission disk (§9)
  Frame f;
  f.X = mk3(l.fx[0], l.fx[1], l.fx[2]);
  f.Y = mk3(l.fy[0], l.fy[1], l.fy[2]);
  f.Z = mk3(l.fz[0], l.fz[1], l.fz[2]);
  f3 wl = normalize(to_local(f, neg(wi)));
  return cosine_pdf_z(wl.z);
}

BDPT_HD LightSample light_sample_point(const DLight& l, int nlights, Rng& g, f3 p, float* lpp_out) {
  LightSample s;
  f3 rad = mk3(l.rad[0], l.rad[1], l.rad[2]);
  f3 dirv = mk3(l.dir[0], l.dir[1], l.dir[2]);
  float lpp;
  if (l.type == LIGHT_POINT) {
    f3 lp = mk3(l.pos[0], l.pos[1], l.pos[2]);
    f3 d = sub(lp, p);
    f3 wi = normalize(d);
    lpp = 1.0f;
    s.dir_pdf = 0.25f / BDPT_PI_F;
    s.n = neg(wi);
    s.pos = lp;
  } else {
    float sx, sy;
    grid2d(g, &sx, &sy);
    sx = sx - 0.5f;
    sy = sy - 0.5f;
    f3 pt = add(add(mk3(l.pos[0], l.pos[1], l.pos[2]), smul(sx, mk3(l.dx[0], l.dx[1], l.dx[2]))),
                smul(sy, mk3(l.dy[0], l.dy[1], l.dy[2])));
    f3 d = sub(pt, p);
    float cosT = dot(d, dirv);
    float dd = sqrtf(norm2(d));
    f3 wi = divs(d, dd);
    lpp = 1.0f / l.area;
    s.n = dirv;
    s.pos = pt;
    s.dir_pdf = cosine_pdf_z(lz(neg(wi), mk3(l.fz[0], l.fz[1], l.fz[2])));
    if (!(cosT < 0)) rad = splat3(0);
  }
  lpp = lpp / (float)nlights;
  s.alpha = divs(rad, lpp);
  s.zh = zaxis(s.n);
  s.fwd = lpp;
  s.env = false;
  *lpp_out = lpp;
  return s;
}
// sample_Le_point of the environment light: a direction w from sample_L's
// importance sampling; point_pdf = its solid-angle pdf / nL, dir_pdf = the emission disk's planar
// density 1/(pi R^2); the vertex sits at infinity (n = zh = -w).
BDPT_HD LightSample env_sample_point(const SceneView& S, Rng& g, f3 p) {
  LightSample s;
  f3 w;
  float pw;
  const f3 rad = env_sample_dir(S.env, g, &w, &pw);
  const float lpp = pw / (float)S.nlights;
  s.pos = p;
  s.n = neg(w);
  s.zh = s.n;
  s.dir_pdf = 1.0f / S.lights[S.env.light].area;
  s.alpha = divs(rad, lpp);
  s.fwd = lpp;
  s.env = true;
  return s;
}

// Camera::generate_ray (camera.cpp:191-212)
BDPT_HD f3 camera_dir(const DCam& c, float x, float y) {
  float rx = (2 * x - 1) * c.tanh_;
  float ry = (2 * y - 1) * c.tanv_;
  float rz = -1;
  f3 w = add(add(smul(rx, mk3(c.c2w[0], c.c2w[1], c.c2w[2])), smul(ry, mk3(c.c2w[3], c.c2w[4], c.c2w[5]))),
             smul(rz, mk3(c.c2w[6], c.c2w[7], c.c2w[8])));
  return normalize(w);
}

struct EyeSample {
  f3 pos, n, zh, alpha;
  float dir_pdf;
  int x, y;
};
// Camera::sample_ray_pdf (camera.cpp:214-248) with cos(acos z) = z.
BDPT_HD EyeSample camera_sample(const DCam& c, int W, int H, f3 p) {
  EyeSample e;
  f3 cam = mk3(c.pos[0], c.pos[1], c.pos[2]);
  f3 wi = sub(cam, p);
  float dist = norm(wi);
  wi = normalize(wi);
  f3 mw = neg(wi);
  f3 wc = add(add(smul(mw.x, mk3(c.w2c[0], c.w2c[1], c.w2c[2])), smul(mw.y, mk3(c.w2c[3], c.w2c[4], c.w2c[5]))),
              smul(mw.z, mk3(c.w2c[6], c.w2c[7], c.w2c[8])));
  wc.z = -wc.z;
  float ct = wc.z;
  float c2 = ct * ct;
  float denom = 4 * c.tanh_ * c.tanv_ / (c2 * c2);
  e.dir_pdf = (dist * dist) / ct;
  e.n = neg(wi);
  float rz = 1.0f / wc.z;
  wc = mk3(wc.x * rz, wc.y * rz, wc.z * rz);
  float fx = ((wc.x / c.tanh_ + 1) * 0.5f) * (float)W;
  float fy = ((wc.y / c.tanv_ + 1) * 0.5f) * (float)H;
  e.x = (fx > -1.0f && fx < (float)W) ? (int)fx : -1;
  e.y = (fy > -1.0f && fy < (float)H) ? (int)fy : -1;
  e.alpha = divs(splat3(1.0f / denom), 1.0f);
  e.pos = cam;
  e.zh = zaxis(e.n);
  return e;
}


// multiple_importance_sampling_weight (bidirection.cpp:121-293) with cached path constants.
// PA: path accessor — e(k) / l(k) return reference vertices E[k] (k >= 2) / L[k] (k >= 1) and
// dE / dL the delta masks; PathsInRegs below (one lane's Paths) or the wavefront vertex store.
// i, j: reference vertex indices; ls: fresh light sample (j == 1); es: camera sample (i == 1);
// dc, dist: normalize(vl - ve) and |vl - ve| of the connection (j >= 1), which are exactly the
// endpoint-step directions the reference recomputes (normalize(-v) == -normalize(v) in IEEE).
template <bool EXT = false, class PA>
BDPT_HD float mis_weight(const SceneView& S, const PA& P, const Vtx* ev, const Vtx* lv, int i, int j,
                         const LightSample& ls, const EyeSample& es, int eye_light, f3 dc, float dist) {
  float ge = 0.0f, gl = 0.0f;
  if (i >= 2) {
    const Vtx& cur = *ev;
    const bool cenv = EXT && is_env(cur);
    float nom;
    if (j == 0) {
      const DLight& EL = S.lights[eye_light];
      float p = EL.type == LIGHT_POINT ? 1.0f
                : (EXT && EL.type == LIGHT_ENV) ? env_pdf_dir(S.env, neg(cur.n)) / (float)S.nlights
                                                : 1.0f / EL.area;
      nom = p * 1.0f;
    } else {
      f3 pzh = j == 1 ? ls.zh : lv->zh;
      f3 dw = neg(dc);   // normalize(E[i] - vl)
      float g = (EXT && j == 1 && ls.env) ? fabsf(dot(dw, cur.n))
                                          : fabsf(lz(dw, pzh) * dot(dw, cur.n)) / (dist * dist);
      float p = j == 1 ? ls.dir_pdf * 1.0f : pdf_b(S.mats[lv->mat], lv->n, pzh, dw) * (EXT ? lv->cq : 1.0f);
      nom = p * g;
    }
    float below = cur.gp;   // G_{i-1}
    if (j == 0 && i >= 3) {  // the step below the emitter uses the light's dir_pdf (:224-232)
      const Vtx v = P.e(i - 1);
      f3 dr;
      const float revg = EXT ? step_gx(v.pos, v.n, false, cur.pos, cur.zh, cenv, &dr)
                             : step_g(v.pos, v.n, cur.pos, cur.zh, &dr);   // g of the step E[i-1] <- E[i]
      f3 dw = cenv ? cur.n : normalize(sub(v.pos, cur.pos));
      float dp = light_dir_pdf(S.lights[eye_light], neg(dw));
      below = mis_horner(((dp * 1.0f) * revg) / v.fwd, !((P.dE >> (i - 2)) & 3u), v.gp);
    }
    // delta(E[i]) || delta(E[i-1]); an escaped camera ray (i = 2) has no camera-connection strategy
    const bool t = !((P.dE >> (i - 1)) & 3u) && !(cenv && i == 2);
    ge = mis_horner(nom / cur.fwd, t, below);
  }
  if (j >= 1) {
    if (EXT && j == 1 && S.env.light >= 0) {
      // environment scenes: the light end of (i, 1) is the fresh sample itself
      f3 dw;
      float g;
      if (ls.env) { dw = dc; g = 1.0f; }
      else g = step_g(ls.pos, ls.n, i == 1 ? es.pos : ev->pos, i == 1 ? es.zh : ev->zh, &dw);
      float p = i <= 1 ? es.dir_pdf * 1.0f : pdf_b(S.mats[ev->mat], ev->n, ev->zh, dw) * ev->cq;
      gl = mis_horner((p * g) / ls.fwd, true, 0.0f);
    } else {
      const Vtx& cur = *lv;   // j == 1: the original L[1], not the fresh sample (quirk 5)
      f3 pzh = i == 1 ? es.zh : ev->zh;
      f3 dw;
      float g;
      if (j >= 2) {   // cur = L[j] = vl: normalize(L[j] - ve) = dc
        dw = dc;
        g = fabsf(lz(dw, pzh) * dot(dw, cur.n)) / (dist * dist);
      } else {
        f3 ppos = i == 1 ? es.pos : ev->pos;
        g = step_g(cur.pos, cur.n, ppos, pzh, &dw);
      }
      float p = i <= 1 ? es.dir_pdf * 1.0f : pdf_b(S.mats[ev->mat], ev->n, pzh, dw) * (EXT ? ev->cq : 1.0f);
      gl = mis_horner((p * g) / cur.fwd, !((P.dL >> (j - 1)) & 3u), cur.gp);
    }
  }
  return 1.0f / ((1.0f + ge) + gl);
}

// Path accessor over one lane's Paths (megakernel, host tests).
template <int MAXV, bool EXT>
struct PathsInRegs {
  const Paths<MAXV>& P;
  DeltaMask<MAXV> dE, dL;
  BDPT_HD explicit PathsInRegs(const Paths<MAXV>& p) : P(p), dE(p.dE), dL(p.dL) {}
  BDPT_HD DeltaMask<MAXV> conn_e() const { return P.cE; }   // connectable eye / light vertices
  BDPT_HD DeltaMask<MAXV> conn_l() const { return P.cL; }
  BDPT_HD DeltaMask<MAXV> src_e() const { return P.sE; }    // s = 0 sources
  BDPT_HD Vtx e(int k) const { return vtx_load<EXT>(P.E[k - 2]); }
  BDPT_HD Vtx l(int k) const { return vtx_load<EXT>(P.L[k - 1]); }
};

// The next vertex's throughput alpha = prev_alpha * |cos| * f / pdf (prepare_bidirectional_subpath
// :60-62), formed when its ray is: one f3 live across the traversal instead of alpha, f and pdf
BDPT_HD f3 walk_next_alpha(f3 pa, f3 pn, f3 d, f3 f, float pdf) { return divs(mul(muls(pa, fabsf(dot(pn, d))), f), pdf); }

// The state of one lane's fused eye + light walk between two iterations (walk_step).
template <int MAXV>
struct WalkState {
  f3 ro, rd, prev_n, nalpha;   // the next ray, the previous vertex's normal, the next vertex's throughput
  float rmin, rmax;
  float pv_fwd, pv_gp, pv_q;   // the previous vertex's fwd / prefix / roulette probability
  int i, count, pv_mat;        // reference vertex index, vertices stored on this subpath, previous material
  DeltaMask<MAXV> dm;          // delta mask of this subpath
  DeltaMask<MAXV> cm, em;      // its connectable vertices (cq > 0); the eye subpath's s = 0 sources
  uint32_t lpos;               // the light stream's position after L[1]
  bool light, l1env;           // walking the light subpath; its L[1] is an environment vertex
};

// Starts one pixel-sample's walk: the camera ray (raytrace_pixel's jitter, bidirection.cpp:515-524)
// and the light vertex L[1] with the light walk's first ray (sample_light_ray, :105-118).
template <int MAXV, bool EXT = false>
BDPT_HD void walk_begin(const SceneView& S, const SampleParams& sp, Paths<MAXV>& P, Counters& cnt, Rng& g,
                        WalkState<MAXV>& w, int x, int y, uint32_t sample) {
  rng_init(g, sp.seed, (uint32_t)(x + y * sp.W), sample);
  float px, py;
  grid2d(g, &px, &py);
  px = px + (float)x;
  py = py + (float)y;
  float dx = px / (float)sp.W, dy = py / (float)sp.H;
  const f3 cam = mk3(S.cam.pos[0], S.cam.pos[1], S.cam.pos[2]);
  f3 rd = camera_dir(S.cam, dx, dy);
  // sample_light_ray (bidirection.cpp:105-118), AreaLight/PointLight::sample_Le, on stream 1: the
  // light vertex L[1] and the light walk's first ray, drawn before the eye walk and kept in the path
  // store (read back when the light walk starts), so the ~17 registers of the light sample are not
  // live across the eye walk's traversals (drawing them at the switch instead spilled more).
  bool l1env = false;
  float mis_p = 0.0f;   // L[1]'s MIS point density (differs from lpp only for the env light)
  auto sample_light = [&](Rng& gl, f3& lo, f3& ld, f3& ln, f3& alpha1, float& ldp) {
    rng_stream(gl, 1);
    int lid = (int)(rng_next(gl) * (float)S.nlights);
    if (lid >= S.nlights) lid = S.nlights - 1;
    const DLight& L0 = S.lights[lid];
    f3 lrad = mk3(L0.rad[0], L0.rad[1], L0.rad[2]);
    float lpp, mis_dir;
    if (EXT && L0.type == LIGHT_ENV) {
      // sample_Le of the environment light: direction by sample_L's importance
      // sampling, origin uniform on the disk of radius R facing -w, tangent to the bounding sphere
      f3 w;
      float pw;
      lrad = env_sample_dir(S.env, gl, &w, &pw);
      cnt.env_s++;
      const float u1 = rng_next(gl), u2 = rng_next(gl);
      const float r = S.env.rad * sqrtf(u1);
      float c, sn;
      cos_sin_2pi(u2, &c, &sn);
      const Frame wf = make_frame(w);
      lo = add(add(add(mk3(S.env.cx, S.env.cy, S.env.cz), smul(S.env.rad, w)), smul(r * c, wf.X)), smul(r * sn, wf.Y));
      ld = neg(w);
      ln = ld;
      lpp = 1.0f / L0.area;
      ldp = pw;
      mis_p = pw;
      mis_dir = 1.0f / L0.area;
      l1env = true;
    } else if (L0.type == LIGHT_POINT) {
      float z = rng_next(gl) * 2 - 1;
      float sinT = sqrtf(fmaxf(0.0f, 1.0f - z * z));
      float u = rng_next(gl);
      float c, s;
      cos_sin_2pi(u, &c, &s);
      ld = mk3(c * sinT, s * sinT, z);
      lo = mk3(L0.pos[0], L0.pos[1], L0.pos[2]);
      lpp = 1;
      ldp = 0.25f / BDPT_PI_F;
      ln = ld;
      mis_p = lpp;
      mis_dir = ldp;
    } else {
      float sx, sy;
      grid2d(gl, &sx, &sy);
      sx = sx - 0.5f;
      sy = sy - 0.5f;
      lo = add(add(mk3(L0.pos[0], L0.pos[1], L0.pos[2]), smul(sx, mk3(L0.dx[0], L0.dx[1], L0.dx[2]))),
               smul(sy, mk3(L0.dy[0], L0.dy[1], L0.dy[2])));
      f3 dl = cosine_hemi(gl, &ldp);
      Frame lf;
      lf.X = mk3(L0.fx[0], L0.fx[1], L0.fx[2]);
      lf.Y = mk3(L0.fy[0], L0.fy[1], L0.fy[2]);
      lf.Z = mk3(L0.fz[0], L0.fz[1], L0.fz[2]);
      ld = to_world(lf, dl);
      lpp = 1.0f / L0.area;
      ln = mk3(L0.dir[0], L0.dir[1], L0.dir[2]);
      mis_p = lpp;
      mis_dir = ldp;
    }
    lpp = lpp / (float)S.nlights;
    mis_p = mis_p / (float)S.nlights;
    alpha1 = divs(lrad, lpp);
    Vtx v1;
    v1.pos = lo;
    v1.n = ln;
    v1.zh = l1env ? ln : zaxis(ln);
    v1.alpha = alpha1;
    v1.mat = l1env ? (int)MAT_ENV_V : -1;
    v1.gp = 0; v1.cq = 0;
    v1.fwd = mis_p;   // light_constants' L[1] value (set here for the fused walk)
    vtx_store<EXT>(P.L[0], v1);
    BDPT_WB2_DUP(P, &P.L[0], v1);
    P.l1_dir_pdf = mis_dir;
  };
  Rng gl0 = g;
  f3 lo, ld, ln, la1;
  float ldp;
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long tl0 = __builtin_amdgcn_s_memtime();
#endif
  sample_light(gl0, lo, ld, ln, la1, ldp);
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
  BDPT_WAVE_CLK(cnt.clk_light, __builtin_amdgcn_s_memtime() - tl0);
#endif
  w.lpos = gl0.pos;
  P.l1_d = ld;
  P.l1_pdf = ldp;
  w.l1env = false;   // re-read with the rest when the light walk starts
  // the walk: eye first (camera ray on [nClip, fClip], alpha = 1, pdf = 1, n = d), then light
  w.ro = cam;
  w.rmin = S.cam.nclip;
  w.rmax = S.cam.fclip;
  w.prev_n = rd;
  w.rd = rd;
  w.nalpha = walk_next_alpha(divs(splat3(1.0f), 1.0f), rd, rd, splat3(1.0f), 1.0f);
  w.i = 2;
  w.count = 0;
  w.dm = 0;
  w.cm = 0;
  w.em = 0;
  w.light = false;
  w.pv_mat = -1;
  w.pv_fwd = 1.0f; w.pv_gp = 0.0f; w.pv_q = 1.0f;
}
// One iteration of the fused walk: trace the next ray, store the vertex it hits (with its MIS
// constants), sample the continuation. Returns true once the light subpath has ended (both
// subpaths and P.nE / P.nL / P.dE / P.dL complete).
template <int MAXV, int LM = 0, bool EXT = false>
BDPT_HD bool walk_step(const SceneView& S, const SampleParams& sp, Paths<MAXV>& P, Counters& cnt, Rng& g,
                       WalkState<MAXV>& w) {
  f3 ro = w.ro, rd = w.rd, prev_n = w.prev_n, nalpha = w.nalpha;
  float rmin = w.rmin, rmax = w.rmax, pv_fwd = w.pv_fwd, pv_gp = w.pv_gp, pv_q = w.pv_q;
  int i = w.i, count = w.count, pv_mat = w.pv_mat;
  DeltaMask<MAXV> dm = w.dm, cm = w.cm, em = w.em;
  bool light = w.light, l1env = w.l1env;
  auto next_alpha = walk_next_alpha;
  bool done = false;
  {
    Hit h;
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long tq0 = __builtin_amdgcn_s_memtime();
#endif
    BDPT_LANE_PROF(cnt, LP_WALK);
    bool end = !trace_closest<LM, kWalkStack>(S, ro, rd, rmin, rmax, h, cnt);
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long tq1 = __builtin_amdgcn_s_memtime();
    BDPT_WAVE_CLK(cnt.clk_walk_trace, tq1 - tq0);
#endif
    if (EXT && end && !light && S.env.light >= 0) {
      // an escaped eye ray ends on the environment light: vertex at infinity in direction rd
      Vtx v;
      v.alpha = nalpha;
      v.pos = ro;
      v.n = neg(rd);
      v.zh = v.n;
      v.mat = MAT_ENV_V;
      v.fwd = 1; v.gp = 1; v.cq = 0;
      // eye_constants of an env vertex: g = 1 toward it, the previous vertex's BSDF density of rd
      // times its roulette probability; no prefix (the j = 0 weight recomputes this step)
      if (count > 0) {
        const f3 pn = EXT ? P.E[count - 1].n : prev_n;
        const int pm = EXT ? vs_mat(P.E[count - 1]) : pv_mat;
        v.fwd = pdf_b(S.mats[pm], pn, pn, rd) * pv_q * 1.0f;
      }
      v.gp = 0.0f;
      em |= DeltaMask<MAXV>(1) << i;   // an s = 0 source (vertex index i = count + 2)
      BDPT_WB2_DUP(P, &P.E[count], v);
      vtx_store<EXT>(P.E[count++], v);
    }
    if (!end) {
      BDPT_LANE_PROF(cnt, LP_SHADE);
      f3 n;
      int mat;
      shade_hit<LM>(S, h, ro, rd, &n, &mat);
      const DMat M = S.mats[mat];
      const Frame fr = make_frame_hit(n);
      const f3 hit_p = add(ro, muls(rd, h.t));
      Vtx v;
      v.alpha = nalpha;
      v.pos = hit_p;
      v.n = n;
      v.zh = fr.Z;
      v.mat = mat;
      v.fwd = 1; v.gp = EXT ? 1.0f : 0.0f; v.cq = 0;
      VtxS* slot = (light ? P.L + 1 : P.E) + count++;
      if (is_delta(M.type)) dm |= DeltaMask<MAXV>(1) << i;
      if (!light && M.type == MAT_EMISSION) em |= DeltaMask<MAXV>(1) << i;   // an s = 0 source
      // eye_constants / light_constants of this vertex at its creation. The previous vertex is the
      // one just below it on the same subpath (camera: no step; the light vertex L[1] for the
      // light's first hit) and is still in registers: position ro, normal prev_n (shading axis
      // normalize(prev_n), as make_frame / zaxis compute it; an environment L[1] keeps n itself),
      // material, fwd, prefix, roulette probability. The prefix and the connectability need this
      // vertex's own roulette probability, known after its sample_f below (EXT), so they are
      // finished there: gp = horner(((pp * q) * g) / fwd_prev, t, gp_prev), cq = conn ? q : 0.
      const bool conn = M.type == MAT_DIFFUSE && lz(normalize(sub(ro, v.pos)), v.zh) >= 0 && nonzero3(v.alpha);
      const bool first_eye = !light && count == 1;
      // the previous vertex. EXT kernels read it back from the path store (it was stored before
      // this traversal) rather than hold it in registers across the traversal: C5 +1.5%; the
      // reference-only kernels keep the registers (-0.3 .. -1.5% otherwise, profiles/r03_ab_pv_reload.log)
      f3 pn = prev_n;
      int pmat = pv_mat;
      float pfwd = pv_fwd, pgp = pv_gp;
      if (EXT) {
        if (first_eye) {
          pn = rd; pmat = -1; pfwd = 1.0f; pgp = 0.0f;
        } else {
          const VtxS& pvx = light ? P.L[count - 1] : P.E[count - 2];
          pn = pvx.n; pmat = vs_mat(pvx); pfwd = pvx.fwd; pgp = pvx.gp;
        }
      }
      float gp_pp = 0.0f, gp_g = 0.0f;
      if (first_eye) {
        v.fwd = 1.0f * 1.0f;
      } else {
        const bool nx_env = EXT && light && count == 1 && l1env;
        // the previous vertex's shading axis: a surface hit's is its normal (make_frame_hit), the
        // light vertex L[1]'s is zaxis(n) (an environment L[1] keeps n)
        const f3 nx_zh = (nx_env || !(light && count == 1)) ? pn : zaxis(pn);
        f3 dw;
        const float g2 = EXT ? step_gx(v.pos, v.n, false, ro, nx_zh, nx_env, &dw) : step_g(v.pos, v.n, ro, nx_zh, &dw);
        const float p = (light && count == 1) ? P.l1_dir_pdf
                                              : pdf_b(S.mats[pmat], pn, nx_zh, dw) * (EXT ? pv_q : 1.0f);
        v.fwd = p * g2;
        gp_g = EXT ? step_gx(ro, pn, nx_env, v.pos, v.zh, false, &dw) : step_g(ro, pn, v.pos, v.zh, &dw);
        gp_pp = pdf_b(M, v.n, v.zh, dw);
      }
      const bool gp_t = !((dm >> (i - 2)) & 3u);
      auto finish = [&](float q) {   // q: this vertex's roulette probability (1 without roulette)
        v.cq = conn ? (EXT ? q : 1.0f) : 0.0f;
        if (v.cq > 0.0f) cm |= DeltaMask<MAXV>(1) << i;   // connectable (i: this vertex's index)
        v.gp = first_eye ? 0.0f : mis_horner(((EXT ? gp_pp * q : gp_pp) * gp_g) / pfwd, gp_t, pgp);
        pv_mat = v.mat; pv_fwd = v.fwd; pv_gp = v.gp; pv_q = q;
      };
      if (!EXT) finish(1.0f);
      vtx_store<EXT>(*slot, v);
      BDPT_WB2_DUP(P, slot, v);
      if (i >= sp.max_depth + 1 || count >= MAXV) {
        end = true;
        if (EXT) {
          finish(1.0f);
          slot->gp = v.gp; slot->cq = v.cq;
        }
      } else {
        f3 wi;
        float pdf;
        const f3 fv = sample_f(M, g, to_local(fr, neg(rd)), &wi, &pdf);
        float q = 1.0f;
        if (EXT && sp.rr && i > BDPT_RR_MIN) {
          // p_keep = min(1, |f| / pdf), PathVertex.q, then coin_flip(p_keep) (bidirection.cpp:87-93)
          q = pdf > 0.0f ? fminf(1.0f, norm(fv) / pdf) : 0.0f;
          slot->gp = q;
          if (!(rng_next(g) < q)) end = true;
        }
        if (EXT) {
          finish(q);
          slot->gp = v.gp; slot->cq = v.cq;
        }
        ro = hit_p;
        rd = normalize(to_world(fr, wi));
        rmin = BDPT_EPS_F;
        rmax = INFINITY;
        prev_n = n;
        nalpha = next_alpha(v.alpha, n, rd, fv, pdf * q);
        i++;
        // A subpath whose throughput is exactly zero (the vertex's f = 0: an emitter, a diffuse
        // surface seen from behind, bsdf.cpp:56-58,99-110) would walk on to the depth cap with
        // alpha = 0: every later vertex has alpha = 0, so no
        // connection can use it (can_connect, make_conn's contrib gate) and no weight of another
        // connection reads it, and the walk's draws come from its own counter stream. Ending it
        // here is output-identical (tests/test_core_cpu.py vs the oracle, which walks on) and
        // saves 3-4% of the walk rays at the north star's 1080p FOV.
        if (!nonzero3(nalpha)) end = true;
      }
#if defined(BDPT_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
      BDPT_WAVE_CLK(cnt.clk_vertex, __builtin_amdgcn_s_memtime() - tq1);
#endif
    }
    if (end) {
      if (light) {
        P.nL = count + 2;
        P.dL = dm;
        P.cL = cm;
        done = true;
      } else {
      P.nE = count + 2;
      P.dE = dm;
      P.cE = cm;
      P.sE = em;
      light = true;
      // the light sample drawn before the eye walk, read back from the path store (not held in
      // registers across the eye walk)
      rng_stream(g, 1);
      g.pos = w.lpos;
      ro = P.L[0].pos; rd = P.l1_d; prev_n = P.L[0].n;
      nalpha = next_alpha(P.L[0].alpha, prev_n, rd, splat3(1.0f), P.l1_pdf);
      const float mis_p = P.L[0].fwd;
      l1env = vs_mat(P.L[0]) == (int)MAT_ENV_V;
      rmin = BDPT_EPS_F; rmax = INFINITY;
      i = 2; count = 0; dm = 0; cm = 0;
      pv_mat = -1; pv_fwd = mis_p; pv_gp = 0.0f; pv_q = 1.0f;   // the light vertex L[1]
      }
    }
  }
  w.ro = ro; w.rd = rd; w.prev_n = prev_n; w.nalpha = nalpha;
  w.rmin = rmin; w.rmax = rmax; w.pv_fwd = pv_fwd; w.pv_gp = pv_gp; w.pv_q = pv_q;
  w.i = i; w.count = count; w.pv_mat = pv_mat; w.dm = dm; w.cm = cm; w.em = em; w.light = light; w.l1env = l1env;
  return done;
}

// Eye and light subpaths of one pixel-sample plus their MIS constants
// (est_radiance_global_illumination, bidirection.cpp:472-488; raytrace_pixel :515-524;
// prepare_bidirectional_subpath :20-102 for both walks). The two walks run as ONE loop: a lane whose
// eye walk ends starts its light walk in the next iteration, so a wave iterates
// max(|E| + |L|) times instead of max |E| + max |L|. The RNG sub-streams (eye walk: 0, light
// sample + walk: 1) make the interleaving invisible in the results.
template <int MAXV, int LM = 0, bool EXT = false>
BDPT_HD void prepare_sample(const SceneView& S, const SampleParams& sp, Paths<MAXV>& P, Counters& cnt, Rng& g,
                            int x, int y, uint32_t sample) {
  WalkState<MAXV> w;
  walk_begin<MAXV, EXT>(S, sp, P, cnt, g, w, x, y, sample);
  while (!walk_step<MAXV, LM, EXT>(S, sp, P, cnt, g, w)) {
  }
  BDPT_WB2_USE(P);
}
// What estimate_bidirection_radiance (bidirection.cpp:296-469) computes for pair (i, j) up to its
// visibility test: either nothing (zero contribution), a direct eye-image value (s = 0, no ray),
// or a connection ray on [EPS_F, tmax] whose value (MIS-weighted) counts if it is unoccluded.
enum { CONN_NONE = 0, CONN_DIRECT = 1, CONN_RAY = 2 };
struct Conn {
  f3 o, d;
  float tmax;
  f3 val;      // eye image: ill; light image: ill / ns_aa
  int splat;   // -1: eye image of this sample's pixel; else x + y*W of the t = 1 splat
};

// A vertex that can receive a connection: diffuse (f != 0 only for DiffuseBSDF, bsdf.cpp:52-62),
// viewed from its front side (wo.z >= 0) and carrying throughput.
BDPT_HD bool can_connect(const Vtx& v) { return v.cq > 0.0f; }
// ev_pre / lv_pre: E[i] / L[j] already loaded by the caller (kept across the megakernel's inner
// connection loop), or null.
// ec: environment-table read counters (stats builds), or null.
template <bool EXT = false, class PA>
BDPT_HD int make_conn(const SceneView& S, const SampleParams& sp, const PA& P, Rng& g, int i, int j, Conn& cn,
                      const Vtx* ev_pre = nullptr, const Vtx* lv_pre = nullptr, Counters* ec = nullptr) {
  const f3 cam = mk3(S.cam.pos[0], S.cam.pos[1], S.cam.pos[2]);
  const bool eye_cam = i == 1;
  Vtx ev, lv;
  LightSample ls;
  ls.env = false;
  EyeSample es;
  es.x = -1; es.y = -1;
  cn.splat = -1;
  if (!eye_cam) ev = ev_pre ? *ev_pre : P.e(i);
  if (j == 0) {
    if (eye_cam) return CONN_NONE;
    if (EXT && is_env(ev)) {   // an escaped eye ray: the environment light contains it (§9)
      const f3 c = env_radiance(S.env, neg(ev.n));
      if (ec) ec->env_l++;
      f3 contrib = mul(mul(ev.alpha, splat3(1.0f)), c);
      float w = 0;
      if (norm(contrib) > BDPT_EPS_F) {
        w = mis_weight<EXT>(S, P, &ev, &lv, i, 0, ls, es, S.env.light, splat3(0), 0);
        if (ec) ec->env_p++;   // the j = 0 weight's env_pdf_dir
      }
      cn.val = muls(contrib, w);
      return CONN_DIRECT;
    }
    const DMat& M = S.mats[ev.mat];
    if (M.type != MAT_EMISSION) return CONN_NONE;
    f3 c = mk3(M.a[0], M.a[1], M.a[2]);
    if (!(norm(c) > BDPT_EPS_F)) return CONN_NONE;
    int eye_light = -1;
    for (int l = 0; l < S.nlights; l++)
      if ((!EXT || S.lights[l].type != LIGHT_ENV) && light_contains(S.lights[l], ev.pos)) { eye_light = l; break; }
    if (eye_light < 0) return CONN_NONE;
    f3 prevp = i == 2 ? cam : P.e(i - 1).pos;
    f3 wi = normalize(sub(ev.pos, prevp));
    const DLight& EL = S.lights[eye_light];
    if (!(light_dir_pdf(EL, wi) > 0)) return CONN_NONE;
    c = mk3(EL.rad[0], EL.rad[1], EL.rad[2]);
    f3 contrib = mul(mul(ev.alpha, splat3(1.0f)), c);
    float w = 0;
    if (norm(contrib) > BDPT_EPS_F) w = mis_weight<EXT>(S, P, &ev, &lv, i, 0, ls, es, eye_light, splat3(0), 0);
    cn.val = muls(contrib, w);
    return CONN_DIRECT;
  }
  // Zero-contribution connections (f_eye = 0 or f_light = 0 or zero throughput) end here.
  if (!eye_cam && !can_connect(ev)) return CONN_NONE;
  lv = lv_pre ? *lv_pre : P.l(j);   // j == 1: the original L[1] (MIS quirk); j >= 2: the light endpoint
  if (j >= 2 && !can_connect(lv)) return CONN_NONE;
  f3 vl_pos, vl_n, la;
  if (j == 1) {   // fresh light sample (bidirection.cpp:332-358)
    const f3 epos = eye_cam ? cam : ev.pos;
    rng_stream(g, 2u + (uint32_t)i);
    int id = (int)(rng_next(g) * (float)S.nlights);
    if (id >= S.nlights) id = S.nlights - 1;
    if (EXT && S.lights[id].type == LIGHT_ENV) {
      if (eye_cam) return CONN_NONE;   // no camera connection to a vertex at infinity (§9)
      ls = env_sample_point(S, g, epos);
      if (ec) ec->env_s++;
    } else {
      float lp;
      ls = light_sample_point(S.lights[id], S.nlights, g, epos, &lp);
    }
    vl_pos = ls.pos; vl_n = ls.n; la = ls.alpha;
  } else {
    vl_pos = lv.pos; vl_n = lv.n; la = lv.alpha;
  }
  f3 ve_pos, ve_n, ea;
  if (eye_cam) {   // camera sample (bidirection.cpp:360-383)
    es = camera_sample(S.cam, sp.W, sp.H, vl_pos);
    if (!(es.x >= 0 && es.y >= 0 && es.x < sp.W && es.y < sp.H)) return CONN_NONE;   // not splatted
    ve_pos = es.pos; ve_n = es.n; ea = es.alpha;
  } else {
    ve_pos = ev.pos; ve_n = ev.n; ea = ev.alpha;
  }
  f3 eal = mul(ea, la);
  if (!nonzero3(eal)) return CONN_NONE;
  // One direction serves the f() hemisphere tests, the connection ray and both MIS endpoint steps.
  const bool lenv = EXT && ls.env;
  f3 dc;
  float dist;
  if (lenv) {
    dc = neg(ls.n);   // toward the environment, unbounded
    dist = INFINITY;
  } else {
    dc = sub(vl_pos, ve_pos);
    dist = norm(dc);
    dc = normalize(dc);
  }
  f3 f_eye = splat3(1.0f), f_light = splat3(1.0f);
  if (!eye_cam) {
    if (lz(dc, ev.zh) < 0) return CONN_NONE;   // f_eye = 0 (bsdf.cpp:56-58)
    const DMat& M = S.mats[ev.mat];
    f_eye = divs(mk3(M.a[0], M.a[1], M.a[2]), BDPT_PI_F);
  }
  if (j >= 2) {
    if (lz(neg(dc), lv.zh) < 0) return CONN_NONE;   // f_light = 0
    const DMat& M = S.mats[lv.mat];
    f_light = divs(mk3(M.a[0], M.a[1], M.a[2]), BDPT_PI_F);
  }
  float gg = lenv ? fabsf(dot(ve_n, dc)) : fabsf(dot(vl_n, dc) * dot(ve_n, dc)) / (dist * dist);
  f3 c = mul(muls(f_eye, gg), f_light);
  f3 contrib = mul(eal, c);
  if (!(norm(contrib) > BDPT_EPS_F)) return CONN_NONE;   // w = 0
  float w = mis_weight<EXT>(S, P, &ev, &lv, i, j, ls, es, -1, dc, dist);
  f3 ill = muls(contrib, w);
  cn.o = ve_pos;
  cn.d = dc;
  cn.tmax = dist - BDPT_EPS_F;
  if (eye_cam) {
    cn.val = divs(ill, (float)sp.spp);
    cn.splat = es.x + es.y * sp.W;
  } else {
    cn.val = ill;
  }
  return CONN_RAY;
}

// One pixel-sample, connections resolved in the reference's (i, j) order (host/test use; the
// device kernel defers the connection rays to a wave-compacted queue instead).
template <int MAXV, int LM = 0, bool EXT = false, class Sink>
BDPT_HD f3 render_sample(const SceneView& S, const SampleParams& sp, Paths<MAXV>& P, Counters& cnt,
                         int x, int y, uint32_t sample, Sink& sink) {
  Rng g;
  prepare_sample<MAXV, LM, EXT>(S, sp, P, cnt, g, x, y, sample);
  f3 eye_sum = splat3(0);
  for (int i = 1; i < P.nE; i++) {
    for (int j = 0; j < P.nL; j++) {
      Conn cn;
      int kind = make_conn<EXT>(S, sp, PathsInRegs<MAXV, EXT>(P), g, i, j, cn);
      if (kind == CONN_DIRECT) {
        eye_sum = add(eye_sum, cn.val);
      } else if (kind == CONN_RAY) {
        if (trace_any<LM>(S, cn.o, cn.d, BDPT_EPS_F, cn.tmax, cnt)) continue;
        if (cn.splat >= 0) sink.splat(cn.splat % sp.W, cn.splat / sp.W, cn.val);
        else eye_sum = add(eye_sum, cn.val);
      }
    }
  }
  return eye_sum;
}

// ================================================================================================
// The unidirectional PathTracer (pathtracer.cpp:47-340) in the device
// semantics. The reference recurses (at_least_one_bounce, :181-262) and adds each vertex's
// continuation after the deeper vertices return; the walk here runs forward and keeps what each
// vertex contributes (NEE, f, cos, pdf, the next hit's emission), then folds innermost-first so the
// fp32 operation order is the reference's (oracle mode 2 runs the recursion itself, bit-exact).
struct PtParams {
  int W, H, spp, max_depth;   // max_depth 0: roulette (coin_flip(0.3), depth < 20)
  uint64_t seed;
  int ns_area_light, batch, hemisphere;
  float tol;                  // maxTolerance (adaptive sampling, :320-334)
  float lens_radius, focal_distance;
};
constexpr int kPtMaxVerts = 21;   // depths 0..20 (the roulette cap, :215)

BDPT_HD bool mat_is_delta(const SceneView& S, int m) { return is_delta(S.mats[m].type); }
BDPT_HD f3 mat_emission(const SceneView& S, int m) {
  const DMat& M = S.mats[m];
  return M.type == MAT_EMISSION ? mk3(M.a[0], M.a[1], M.a[2]) : splat3(0);
}
BDPT_HD f3 bsdf_f_pt(const DMat& M, f3 wo, f3 wi) {   // BSDF::f of every kind (bsdf.cpp, advanced_bsdf.cpp)
  if (M.type == MAT_DIFFUSE) {
    if (wo.z < 0 || wi.z < 0) return splat3(0);
    return divs(mk3(M.a[0], M.a[1], M.a[2]), BDPT_PI_F);
  }
  if (M.type == MAT_MICROFACET) return mf_f(M, wo, wi);
  return splat3(0);
}
// SceneLight::sample_L (light.cpp:103-113, 205-217; environment_light.cpp:126-156)
BDPT_HD f3 light_sample_L(const SceneView& S, const DLight& L, Rng& g, f3 p, f3* wi, float* dist, float* pdf) {
  if (L.type == LIGHT_ENV) {
    *dist = INFINITY;
    return env_sample_dir(S.env, g, wi, pdf);
  }
  if (L.type == LIGHT_POINT) {
    const f3 d = sub(mk3(L.pos[0], L.pos[1], L.pos[2]), p);
    *wi = normalize(d);
    *dist = norm(d);
    *pdf = 1.0f;
    return mk3(L.rad[0], L.rad[1], L.rad[2]);
  }
  if (L.type == LIGHT_DIR) {    // DirectionalLight::sample_L (light.cpp:17-23)
    *wi = mk3(L.dir[0], L.dir[1], L.dir[2]);
    *dist = INFINITY;
    *pdf = 1.0f;
    return mk3(L.rad[0], L.rad[1], L.rad[2]);
  }
  if (L.type == LIGHT_HEMI) {   // InfiniteHemisphereLight::sample_L (light.cpp:62-70, sampler.cpp:36-49)
    const float Xi1 = rng_next(g);
    const float Xi2 = rng_next(g);
    float c, s;
    cos_sin_2pi(Xi2, &c, &s);
    const float st = sqrtf(fmaxf(0.0f, 1.0f - Xi1 * Xi1));   // theta = acos(Xi1)
    *wi = mk3(st * c, Xi1, -(st * s));                        // sampleToWorld * (x, y, z) = (x, z, -y)
    *dist = INFINITY;
    *pdf = (float)(1.0 / (2.0 * 3.14159265358979323));   // 1 / (2 PI) in fp64, rounded once
    return mk3(L.rad[0], L.rad[1], L.rad[2]);
  }
  float sx, sy;
  grid2d(g, &sx, &sy);
  sx = sx - 0.5f;
  sy = sy - 0.5f;
  const f3 d = sub(add(add(mk3(L.pos[0], L.pos[1], L.pos[2]), smul(sx, mk3(L.dx[0], L.dx[1], L.dx[2]))),
                       smul(sy, mk3(L.dy[0], L.dy[1], L.dy[2]))), p);
  const float cosT = dot(d, mk3(L.dir[0], L.dir[1], L.dir[2]));
  const float sq = norm2(d);
  const float dd = sqrtf(sq);
  *wi = divs(d, dd);
  *dist = dd;
  *pdf = sq / (L.area * fabsf(cosT));
  return cosT < 0 ? mk3(L.rad[0], L.rad[1], L.rad[2]) : splat3(0);
}

// Direct lighting at a non-delta hit (estimate_direct_lighting_importance :99-169 /
// _hemisphere :47-97).
template <int LM>
BDPT_HD f3 pt_direct(const SceneView& S, const PtParams& pp, Rng& g, const Frame& fr, f3 hit_p, f3 w_out, f3 n,
                     const DMat& M, Counters& cnt) {
  f3 L_out = splat3(0);
  if (pp.hemisphere) {
    const int num = S.nlights * pp.ns_area_light;
    for (int i = 0; i < num; i++) {
      f3 wi;
      float pdf;
      const f3 f = sample_f(M, g, w_out, &wi, &pdf);
      const f3 wiw = normalize(to_world(fr, wi));
      Hit h;
      if (!trace_closest<LM, kWalkStack>(S, hit_p, wiw, BDPT_EPS_F, INFINITY, h, cnt)) continue;
      f3 hn;
      int hm;
      shade_hit<LM>(S, h, hit_p, wiw, &hn, &hm);
      const float ct = fabsf(dot(wiw, n));
      L_out = add(L_out, divs(muls(mul(mat_emission(S, hm), f), ct), pdf));
    }
    return divs(L_out, (float)num);
  }
  for (int l = 0; l < S.nlights; l++) {
    const DLight& L = S.lights[l];
    const int ns = (L.type == LIGHT_POINT || L.type == LIGHT_DIR) ? 1 : pp.ns_area_light;   // is_delta_light
    f3 L_o = splat3(0);
    for (int i = 0; i < ns; i++) {
      f3 wiw;
      float dist, pdf;
      const f3 Le = light_sample_L(S, L, g, hit_p, &wiw, &dist, &pdf);
      const f3 f = bsdf_f_pt(M, w_out, to_local(fr, wiw));
      if (trace_any<LM, kConnStack>(S, hit_p, wiw, BDPT_EPS_F, dist - BDPT_EPS_F, cnt)) continue;
      const float ct = fabsf(dot(wiw, n));
      const f3 L_in = dist >= INFINITY ? Le : divs(Le, dist * dist);
      L_o = add(L_o, divs(muls(mul(L_in, f), ct), pdf));
    }
    L_out = add(L_out, divs(L_o, (float)ns));
  }
  return L_out;
}

// One camera sample (raytrace_pixel :304-316 -> est_radiance_global_illumination :264-290).
template <int LM>
BDPT_HD f3 pt_sample(const SceneView& S, const PtParams& pp, Counters& cnt, int x, int y, uint32_t sample) {
  Rng g;
  rng_init(g, pp.seed, (uint32_t)(x + y * pp.W), sample);
  float px, py, lx, ly;
  grid2d(g, &px, &py);
  px = px + (float)x;
  py = py + (float)y;
  const float dx = px / (float)pp.W, dy = py / (float)pp.H;
  grid2d(g, &lx, &ly);
  // Camera::generate_ray_for_thin_lens (camera_lens.cpp:22-43)
  float lc, ls;
  cos_sin_2pi(ly, &lc, &ls);
  const f3 pLens = mk3(pp.lens_radius * sqrtf(lx) * lc, pp.lens_radius * sqrtf(lx) * ls, 0.0f);
  const f3 rdir = mk3((2 * dx - 1) * S.cam.tanh_, (2 * dy - 1) * S.cam.tanv_, -1.0f);
  const f3 rd0 = sub(muls(rdir, pp.focal_distance), pLens);
  const f3 c0 = mk3(S.cam.c2w[0], S.cam.c2w[1], S.cam.c2w[2]), c1 = mk3(S.cam.c2w[3], S.cam.c2w[4], S.cam.c2w[5]),
           c2 = mk3(S.cam.c2w[6], S.cam.c2w[7], S.cam.c2w[8]);
  f3 rd = normalize(add(add(smul(rd0.x, c0), smul(rd0.y, c1)), smul(rd0.z, c2)));
  f3 ro = add(mk3(S.cam.pos[0], S.cam.pos[1], S.cam.pos[2]),
              add(add(smul(pLens.x, c0), smul(pLens.y, c1)), smul(pLens.z, c2)));
  Hit h;
  if (!trace_closest<LM, kWalkStack>(S, ro, rd, S.cam.nclip, S.cam.fclip, h, cnt))
    return S.env.light >= 0 ? env_radiance(S.env, rd) : splat3(0);
  f3 n;
  int mat;
  shade_hit<LM>(S, h, ro, rd, &n, &mat);
  const f3 E0 = mat_emission(S, mat);
  // forward walk: per vertex k the NEE value, and for a continued walk f, cos, pdf, the roulette
  // flag and the next hit's emission (used when vertex k is delta)
  f3 nee[kPtMaxVerts], fk[kPtMaxVerts], enext[kPtMaxVerts];
  float ck[kPtMaxVerts], pk[kPtMaxVerts];
  unsigned delta_m = 0, cont_m = 0;
  const bool roulette = pp.max_depth == 0;
  int k = 0;
  for (;; k++) {
    const DMat M = S.mats[mat];
    const Frame fr = make_frame_hit(n);
    const f3 hit_p = add(ro, muls(rd, h.t));
    const f3 w_out = to_local(fr, neg(rd));
    const bool dl = is_delta(M.type);
    if (dl) delta_m |= 1u << k;
    nee[k] = dl ? splat3(0) : pt_direct<LM>(S, pp, g, fr, hit_p, w_out, n, M, cnt);
    bool trace;
    if (roulette) trace = (rng_next(g) < 0.3f) && k < 20;
    else trace = k < pp.max_depth - 1;
    if (!trace || k + 1 >= kPtMaxVerts) break;
    f3 wi;
    float pdf;
    const f3 f = sample_f(M, g, w_out, &wi, &pdf);
    const f3 wiw = normalize(to_world(fr, wi));
    Hit h2;
    if (!trace_closest<LM, kWalkStack>(S, hit_p, wiw, BDPT_EPS_F, INFINITY, h2, cnt)) break;
    f3 n2;
    int m2;
    shade_hit<LM>(S, h2, hit_p, wiw, &n2, &m2);
    fk[k] = f;
    ck[k] = fabsf(dot(wiw, n));
    pk[k] = pdf;
    enext[k] = mat_emission(S, m2);
    cont_m |= 1u << k;
    ro = hit_p; rd = wiw; h = h2; n = n2; mat = m2;
  }
  // fold innermost-first: L_k = nee_k + (L_{k+1} [+ E_{k+1} if delta_k]) * f_k * cos_k / pdf_k [/ 0.3]
  f3 L = splat3(0);
  for (int j = k; j >= 0; j--) {
    f3 Lj = add(splat3(0), nee[j]);
    if ((cont_m >> j) & 1u) {
      f3 L_in = L;
      if ((delta_m >> j) & 1u) L_in = add(L_in, enext[j]);
      f3 t = divs(muls(mul(L_in, fk[j]), ck[j]), pk[j]);
      if (roulette) t = divs(t, 0.3f);
      Lj = add(Lj, add(splat3(0), t));
    }
    L = Lj;
  }
  return add(E0, L);
}

// PathTracer::raytrace_pixel's adaptive batches (:292-338): samples in batches of pp.batch until
// the 95% interval of the illuminance is within tol * mean (or pp.spp is reached).
template <int LM>
BDPT_HD f3 pt_pixel(const SceneView& S, const PtParams& pp, Counters& cnt, int x, int y, int* count) {
  int num = 0;
  f3 illum = splat3(0);
  float s1 = 0, s2 = 0;
  for (int i = 0; i < pp.spp; i += pp.batch) {
    for (int j = 0; j < pp.batch; j++) {
      const f3 ill = pt_sample<LM>(S, pp, cnt, x, y, (uint32_t)(i + j));
      illum = add(illum, ill);
      const float il = 0.2126f * ill.x + 0.7152f * ill.y + 0.0722f * ill.z;   // Vector3D::illum
      s1 += il;
      s2 += il * il;
    }
    num = i + pp.batch;
    const float mu = s1 / (float)num;
    const float sigma = sqrtf((s2 - s1 * s1 / (float)num) / (float)(num - 1));
    const float ci = 1.96f * sigma / sqrtf((float)num);
    if (ci <= pp.tol * mu && mu > BDPT_EPS_F) break;
  }
  *count = num;
  return divs(illum, (float)num);
}

}  // namespace bdpt
