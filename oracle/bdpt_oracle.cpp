// oracle/bdpt_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference's per-pixel BDPT loop (dongmingli-Ben/bidirectional-pathtracing,
// src/pathtracer/bidirection.cpp and what it calls). It is the checker for the HIP path: only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. Nothing in the
// product (bidirectional-pathtracing_amd/) links or calls this file.
//
// One template, three instantiations (see DESIGN.md §Parity chain):
//   mode 0  REF_STREAM  fp64 + the reference's RNG streams (two per-TU std::mt19937(5489) engines,
//                       util/random_util.h:10-22, plus glibc rand() for light choice,
//                       sampler.h:25-28) + glibc libm, tiles in raster order (single thread).
//                       Pinned bit-exactly against oracle/_ref (the reference itself) dumps in
//                       tests/golden/.
//   mode 1  COUNTER64   fp64 + libm, but uniforms from the counter RNG (Philox4x32-10) — the bridge
//                       between the reference semantics and the fp32 device semantics.
//   mode 2  COUNTER32   fp32 + counter RNG + the device's deterministic transcendentals
//                       (sincos of 2*pi*u by polynomial, cos(acos z) = z, integer powers by
//                       products) — the per-sample parity partner of the HIP kernel.
// Every arithmetic expression below follows the reference's operation order (CGL Vector3D
// semantics: v/c = v*(1/c), normalize = *= 1/norm, dot = (x*x'+y*y')+z*z', CGL/include/CGL/
// vector3D.h) so that mode 0 reproduces the reference's fp64 bits. Build: -O2 -ffp-contract=off.

#include <cmath>
#include <type_traits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <limits>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "bdpt/bdpt.h"

namespace orc {

static const double PI_D = 3.14159265358979323;  // CGL/include/CGL/misc.h:11
static const float EPS_F = 0.00001f;              // misc.h:13

// ----------------------------------------------------------------------------------------------
// CGL Vector3D semantics (vector3D.h)
template <class R>
struct V3 {
  R x, y, z;
  V3() : x(0), y(0), z(0) {}
  V3(R a, R b, R c) : x(a), y(b), z(c) {}
  explicit V3(R c) : x(c), y(c), z(c) {}
  R& operator[](int i) { return (&x)[i]; }
  const R& operator[](int i) const { return (&x)[i]; }
  V3 operator-() const { return V3(-x, -y, -z); }
  V3 operator+(const V3& v) const { return V3(x + v.x, y + v.y, z + v.z); }
  V3 operator-(const V3& v) const { return V3(x - v.x, y - v.y, z - v.z); }
  V3 operator*(const V3& v) const { return V3(x * v.x, y * v.y, z * v.z); }
  V3 operator/(const V3& v) const { return V3(x / v.x, y / v.y, z / v.z); }
  V3 operator*(R c) const { return V3(x * c, y * c, z * c); }
  V3 operator/(R c) const {                       // vector3D.h: rc = 1/c; rc*x
    const R rc = R(1) / c;
    return V3(rc * x, rc * y, rc * z);
  }
  void operator+=(const V3& v) { x += v.x; y += v.y; z += v.z; }
  void operator*=(R c) { x *= c; y *= c; z *= c; }
  void operator/=(R c) { (*this) *= (R(1) / c); }
  R norm2() const { return x * x + y * y + z * z; }
  R norm() const { return std::sqrt(norm2()); }
  V3 unit() const { R rn = R(1) / norm(); return (*this) * rn; }
  void normalize() { (*this) /= norm(); }
};
template <class R> inline V3<R> operator*(R c, const V3<R>& v) { return V3<R>(c * v.x, c * v.y, c * v.z); }
template <class R> inline R dot(const V3<R>& u, const V3<R>& v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
template <class R> inline V3<R> cross(const V3<R>& u, const V3<R>& v) {
  return V3<R>(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x);
}

// Matrix3x3 with columns X,Y,Z = o2w (bsdf.cpp:21-41). o2w*v = v.x*X + v.y*Y + v.z*Z
// (matrix3x3.cpp:110-114); w2o*v = o2w.T()*v = (dot(v,X), dot(v,Y), dot(v,Z)).
template <class R>
struct Frame {
  V3<R> X, Y, Z;
  V3<R> to_world(const V3<R>& v) const { return v.x * X + v.y * Y + v.z * Z; }
  V3<R> to_local(const V3<R>& v) const {
    return V3<R>(v.x * X.x + v.y * X.y + v.z * X.z, v.x * Y.x + v.y * Y.y + v.z * Y.z,
                 v.x * Z.x + v.y * Z.y + v.z * Z.z);
  }
};

// make_coord_space (bsdf.cpp:21-41)
template <class R>
Frame<R> make_coord_space(const V3<R>& n) {
  V3<R> z(n.x, n.y, n.z);
  V3<R> h = z;
  if (std::fabs(h.x) <= std::fabs(h.y) && std::fabs(h.x) <= std::fabs(h.z))
    h.x = 1.0;
  else if (std::fabs(h.y) <= std::fabs(h.x) && std::fabs(h.y) <= std::fabs(h.z))
    h.y = 1.0;
  else
    h.z = 1.0;
  z.normalize();
  V3<R> y = cross(h, z);
  y.normalize();
  V3<R> x = cross(z, y);
  x.normalize();
  return Frame<R>{x, y, z};
}

// The frame of a surface hit (isect.mat >= 0). Mode 2 restates the device's fp32 semantics,
// which take Z = n for a hit normal (already unit length: the intersection normalises it) instead
// of normalising it again (bdpt_core.h make_frame_hit); modes 0 and 1 (fp64) keep
// the reference's make_coord_space, so mode 0 stays bit-exact with the reference.
// oracle_set_hit_frame_ref(1): mode 2 with the reference's make_coord_space for hits too (the
// device semantics minus the Z = n shortcut), so tests can bound what the shortcut alone changes.
static int g_hit_frame_ref = 0;
extern "C" void oracle_set_hit_frame_ref(int on) { g_hit_frame_ref = on; }

template <class R>
Frame<R> hit_coord_space(const V3<R>& n) {
  if (!std::is_same<R, float>::value || g_hit_frame_ref) return make_coord_space(n);
  V3<R> z(n.x, n.y, n.z);
  V3<R> h = z;
  if (std::fabs(h.x) <= std::fabs(h.y) && std::fabs(h.x) <= std::fabs(h.z))
    h.x = 1.0;
  else if (std::fabs(h.y) <= std::fabs(h.x) && std::fabs(h.y) <= std::fabs(h.z))
    h.y = 1.0;
  else
    h.z = 1.0;
  V3<R> y = cross(h, z);
  y.normalize();
  V3<R> x = cross(z, y);
  x.normalize();
  return Frame<R>{x, y, z};
}

// ----------------------------------------------------------------------------------------------
// Random numbers.
// Philox4x32-10 (Salmon et al. 2011). Counter (pixel, sample, block, 0xB1D1), key (seed lo, hi).
inline void philox4x32_10(uint32_t ctr[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ ctr[1] ^ k0;
    uint32_t n2 = hi0 ^ ctr[3] ^ k1;
    ctr[0] = n0; ctr[1] = lo1; ctr[2] = n2; ctr[3] = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
}
// u = ((x >> 9) + 0.5) * 2^-23 : exact in fp32 (24 significant bits), in [2^-24, 1 - 2^-24].
inline float u24(uint32_t x) { return ((float)(x >> 9) + 0.5f) * 1.1920928955078125e-07f; }

// Counter modes: every pixel-sample owns independent sub-streams, so the device can run its
// phases in any order: 0 = camera jitter + eye walk, 1 = light choice + light walk,
// 2 + i = the fresh light sample of connection (i, j = 1) (bidirection.cpp:332-358).
// Counter = (pixel, sample, block, 0xB1D1 + (stream << 16)).
struct CounterStream {
  uint32_t k0, k1, pix, smp, block, tag;
  uint32_t buf[4];
  int idx;
  void init(uint64_t seed, uint32_t pixel, uint32_t sample) {
    k0 = (uint32_t)seed; k1 = (uint32_t)(seed >> 32); pix = pixel; smp = sample; block = 0; idx = 4; tag = 0;
  }
  void select(uint32_t s) { tag = s; block = 0; idx = 4; }
  float next() {
    if (idx == 4) {
      buf[0] = pix; buf[1] = smp; buf[2] = block++; buf[3] = 0xB1D1u + (tag << 16);
      philox4x32_10(buf, k0, k1);
      idx = 0;
    }
    return u24(buf[idx++]);
  }
};

// Reference streams: util/random_util.h:10-22 (per-TU static engine, default seed 5489;
// rmax = 1/(max-min); U = clamp(x*rmax, 1e-7, 0.99999999)).
struct RefStreams {
  std::mt19937 S;   // sampler.cpp's engine (all Sampler2D/3D draws)
  std::mt19937 G;   // advanced_bsdf.cpp's engine (GlassBSDF coin_flip)
  std::mt19937 P;   // pathtracer.cpp's engine (PathTracer's roulette coin_flip)
  std::mt19937 E;   // environment_light.cpp's engine (sample_L's texel jitter)
  double rmax = 1.0 / (double)(4294967295u);
  static double clampd(double x) { return std::min(std::max(x, 0.0000001), 0.99999999); }
  double uS() { return clampd(double(S()) * rmax); }
  double uG() { return clampd(double(G()) * rmax); }
  double uP() { return clampd(double(P()) * rmax); }
  double uE() { return clampd(double(E()) * rmax); }
};

// ----------------------------------------------------------------------------------------------
// Policies: arithmetic type + RNG source + transcendentals.
struct PolicyRef {              // mode 0
  typedef double R;
  static const bool kHornerMis = false;
  RefStreams* rs;
  R uS() { return rs->uS(); }
  R uG() { return rs->uG(); }
  R uP() { return rs->uP(); }
  R uE() { return rs->uE(); }
  int rand_light(int n) { return 0 + std::rand() % (n - 1 - 0 + 1); }   // sampler.h:25-28
  void stream(uint32_t) {}                                                  // one sequential stream
  static void cos_sin_2pi(R xi, R* c, R* s) { R th = 2. * PI_D * xi; *c = std::cos(th); *s = std::sin(th); }
  static R cos_acos(R z) { return std::cos(std::acos(z)); }
  static R pow2(R x) { return std::pow(x, 2); }
  static R pow4(R x) { return std::pow(x, 4); }
  static R pow5(R x) { return std::pow(x, 5); }
  static R tan_half_fov(double fov_deg) { return std::tan(fov_deg * PI_D / 360); }
  static const bool kDevEnv = false;   // environment map math: the reference's libm formulas
};
struct PolicyC64 {              // mode 1
  typedef double R;
  static const bool kHornerMis = false;
  CounterStream* cs;
  R uS() { return (double)cs->next(); }
  R uG() { return (double)cs->next(); }
  R uP() { return (double)cs->next(); }
  R uE() { return (double)cs->next(); }
  int rand_light(int n) { int k = (int)((double)cs->next() * n); return k < n ? k : n - 1; }
  void stream(uint32_t k) { cs->select(k); }
  static void cos_sin_2pi(R xi, R* c, R* s) { R th = 2. * PI_D * xi; *c = std::cos(th); *s = std::sin(th); }
  static R cos_acos(R z) { return std::cos(std::acos(z)); }
  static R pow2(R x) { return std::pow(x, 2); }
  static R pow4(R x) { return std::pow(x, 4); }
  static R pow5(R x) { return std::pow(x, 5); }
  static R tan_half_fov(double fov_deg) { return std::tan(fov_deg * PI_D / 360); }
  static const bool kDevEnv = false;
};

// Deterministic fp32 sin/cos of 2*pi*u, u in (0,1): quadrant reduction (exact by Sterbenz) and
// Taylor polynomials to degree 9/10 in f = u - k/4, |f| <= 1/8. Same op order as the device.
static inline void cos_sin_2pi_f32(float u, float* c, float* s) {
  float t = u * 4.0f;
  int k = (int)(t + 0.5f);                 // t >= 0
  float f = u - (float)k * 0.25f;          // exact
  float f2 = f * f;
  // sin(2*pi*f) = f*(a1 + f2*(a3 + f2*(a5 + f2*(a7 + f2*a9))))
  float sp = f * (6.2831854820251465f +
                  f2 * (-41.34170150756836f +
                        f2 * (81.6052474975586f + f2 * (-76.70585632324219f + f2 * 42.058692932128906f))));
  // cos(2*pi*f) = 1 + f2*(b2 + f2*(b4 + f2*(b6 + f2*(b8 + f2*b10))))
  float cp = 1.0f + f2 * (-19.739208221435547f +
                          f2 * (64.93939208984375f +
                                f2 * (-85.45681762695312f + f2 * (60.2446403503418f + f2 * -26.42625617980957f))));
  switch (k & 3) {
    case 0: *c = cp; *s = sp; break;
    case 1: *c = -sp; *s = cp; break;
    case 2: *c = -cp; *s = -sp; break;
    default: *c = sp; *s = -cp; break;
  }
}

// Deterministic fp32 atan2 (octant reduction + the Cephes atanf polynomial), the device's
// atan2_det in the same operation order: the environment map's direction -> (theta, phi) in mode 2.
static inline float atan2_f32(float y, float x) {
  const float ax = std::fabs(x), ay = std::fabs(y);
  if (ax == 0.0f && ay == 0.0f) return 0.0f;
  float t = ay <= ax ? ay / ax : ax / ay;
  float off = 0.0f;
  if (t > 0.41421356237309503f) {
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
// std::lround for x >= 0 (halves away from zero)
template <class R>
static inline long lround_pos(R x) {
  const R f = std::floor(x);
  return (long)f + ((x - f) >= R(0.5) ? 1 : 0);
}

struct PolicyC32 {              // mode 2
  typedef float R;
  // The device sums the power-heuristic terms in Horner form over per-vertex prefixes
  // (bdpt_core.h mis_weight); mode 2 evaluates the same factors in the same order.
  static const bool kHornerMis = true;
  CounterStream* cs;
  R uS() { return cs->next(); }
  R uG() { return cs->next(); }
  R uP() { return cs->next(); }
  R uE() { return cs->next(); }
  int rand_light(int n) { int k = (int)(cs->next() * (float)n); return k < n ? k : n - 1; }
  void stream(uint32_t k) { cs->select(k); }
  static void cos_sin_2pi(R xi, R* c, R* s) { cos_sin_2pi_f32(xi, c, s); }
  static R cos_acos(R z) { return z; }
  static R pow2(R x) { return x * x; }
  static R pow4(R x) { R x2 = x * x; return x2 * x2; }
  static R pow5(R x) { R x2 = x * x; R x4 = x2 * x2; return x4 * x; }
  static R tan_half_fov(double fov_deg) { return (float)std::tan(fov_deg * PI_D / 360); }
  static const bool kDevEnv = true;    // environment map math: the device's deterministic forms
};

// ----------------------------------------------------------------------------------------------
// Scene in precision R.
template <class R>
struct BBoxT {            // bbox.h:19-136
  V3<R> mx, mn;
  BBoxT() : mx(-INFINITY, -INFINITY, -INFINITY), mn(INFINITY, INFINITY, INFINITY) {}
  explicit BBoxT(const V3<R>& p) : mx(p), mn(p) {}
  BBoxT(const V3<R>& a, const V3<R>& b) : mx(b), mn(a) {}
  void expand(const BBoxT& b) {
    mn.x = std::min(mn.x, b.mn.x); mn.y = std::min(mn.y, b.mn.y); mn.z = std::min(mn.z, b.mn.z);
    mx.x = std::max(mx.x, b.mx.x); mx.y = std::max(mx.y, b.mx.y); mx.z = std::max(mx.z, b.mx.z);
  }
  void expand(const V3<R>& p) {
    mn.x = std::min(mn.x, p.x); mn.y = std::min(mn.y, p.y); mn.z = std::min(mn.z, p.z);
    mx.x = std::max(mx.x, p.x); mx.y = std::max(mx.y, p.y); mx.z = std::max(mx.z, p.z);
  }
  V3<R> centroid() const { return (mn + mx) / R(2); }
};

template <class R>
struct Ray {               // ray.h:20-71 (min_t/max_t are mutable there)
  V3<R> o, d;
  R min_t, max_t;
};

template <class R>
struct Prim {
  int type;
  V3<R> p1, p2, p3, n1, n2, n3;  // triangle
  V3<R> c; R r, r2;              // sphere (sphere.h:23)
  int mat;
  BBoxT<R> bbox;
};

template <class R>
struct Mat {
  int type;
  V3<R> a, b;          // microfacet: a = eta, b = k (MicrofacetBSDF, bsdf.h:170-205)
  R ior;
  R alpha = 0;         // microfacet roughness (collada.cpp:891, parsed as float)
};

template <class R>
struct Light {
  int type;
  V3<R> radiance, position, direction, dim_x, dim_y;
  R area;
};

// The environment light (EnvironmentLight, environment_light.cpp): its map, the
// sampling tables of init() (:18-62) in fp64 rounded to R, and the emission sphere.
static const int LIGHT_ENV_ORC = 100;   // Light::type of the environment light (internal)
template <class R>
struct EnvMap {
  int w = 0, h = 0;
  std::vector<R> marg, cond, pdf;
  std::vector<V3<R>> rgb;
  V3<R> center;
  R rad = 0, area = 0;   // area = pi R^2 (the emission disk)
};

struct BvhNode {
  int l = -1, r = -1;      // children (-1: leaf)
  int start = 0, end = 0;  // leaf range into leaf_prims
};

template <class R>
struct Scene {
  std::vector<Prim<R>> prims;
  std::vector<Mat<R>> mats;
  std::vector<Light<R>> lights;
  std::vector<BvhNode> nodes;
  std::vector<BBoxT<R>> node_box;  // box used by the traversal in precision R
  std::vector<int> leaf_prims;     // prim indices in DFS leaf order
  std::vector<int> dfs_rank;       // prim -> position in DFS leaf order
  int root = 0;
  int depth = 0;
  // camera
  V3<R> cam_pos;
  V3<R> c2w[3], w2c[3];  // columns
  double hfov_deg, vfov_deg;
  R nclip, fclip;
  EnvMap<R> env;
  int env_light = -1;              // index in lights, -1: none
};

// BVH build: construct_bvh (bvh.cpp:51-129) in fp64 on the reference's bboxes.
struct BuildCtx {
  const std::vector<BBoxT<double>>* pb;
  std::vector<BvhNode>* nodes;
  std::vector<BBoxT<double>>* boxes;
  std::vector<int>* leaf_prims;
  int depth;
};
static int construct_bvh(BuildCtx& B, std::vector<int> prims, int depth) {
  const auto& pb = *B.pb;
  B.depth = std::max(B.depth, depth);
  if (prims.size() <= 4) {
    BBoxT<double> bbox = pb[prims[0]];
    for (int p : prims) bbox.expand(pb[p]);
    int id = (int)B.nodes->size();
    BvhNode n;
    n.start = (int)B.leaf_prims->size();
    for (int p : prims) B.leaf_prims->push_back(p);
    n.end = (int)B.leaf_prims->size();
    B.nodes->push_back(n);
    B.boxes->push_back(bbox);
    return id;
  }
  double x_max = 0, x_min = 0, y_max = 0, y_min = 0, z_max = 0, z_min = 0;
  for (size_t i = 0; i < prims.size(); i++) {
    V3<double> c = pb[prims[i]].centroid();
    x_max = i == 0 ? c.x : std::max(x_max, c.x);
    x_min = i == 0 ? c.x : std::min(x_min, c.x);
    y_max = i == 0 ? c.y : std::max(y_max, c.y);
    y_min = i == 0 ? c.y : std::min(y_min, c.y);
    z_max = i == 0 ? c.z : std::max(z_max, c.z);
    z_min = i == 0 ? c.z : std::min(z_min, c.z);
  }
  double ranges[3] = {x_max - x_min, y_max - y_min, z_max - z_min};
  double mins[3] = {x_min, y_min, z_min};
  double max_range = std::max(ranges[0], std::max(ranges[1], ranges[2]));
  int axis;
  for (axis = 0; axis < 3; axis++)
    if (ranges[axis] == max_range) break;
  if (!(max_range > 0) || axis == 3) return -1;  // reference asserts (bvh.cpp:94)
  double midpoint = mins[axis] + ranges[axis] / 2;
  std::vector<int> left, right;
  for (int p : prims) {
    if (pb[p].centroid()[axis] <= midpoint) left.push_back(p);
    else right.push_back(p);
  }
  if (left.empty() || right.empty()) return -1;   // bvh.cpp:117-118
  int id = (int)B.nodes->size();
  B.nodes->push_back(BvhNode());
  B.boxes->push_back(BBoxT<double>());
  int l = construct_bvh(B, left, depth + 1);
  int r = construct_bvh(B, right, depth + 1);
  if (l < 0 || r < 0) return -1;
  BBoxT<double> bb((*B.boxes)[l].mn, (*B.boxes)[l].mx);
  bb.expand((*B.boxes)[r]);
  (*B.nodes)[id].l = l;
  (*B.nodes)[id].r = r;
  (*B.boxes)[id] = bb;
  return id;
}

static inline V3<double> v3d(const double* p) { return V3<double>(p[0], p[1], p[2]); }

template <class R>
static V3<R> cvt(const V3<double>& v) { return V3<R>((R)v.x, (R)v.y, (R)v.z); }

// Conservative fp32 box: round outward and pad by 2^-16 of the larger of |extent| and |coord|.
static float pad_down(double v, double ext) {
  double m = std::max(std::fabs(v), ext) * (1.0 / 65536.0) + 1e-30;
  float f = (float)(v - m);
  if ((double)f > v - m) f = std::nextafter(f, -INFINITY);
  return f;
}
static float pad_up(double v, double ext) {
  double m = std::max(std::fabs(v), ext) * (1.0 / 65536.0) + 1e-30;
  float f = (float)(v + m);
  if ((double)f < v + m) f = std::nextafter(f, INFINITY);
  return f;
}

template <class R>
static int load_scene(const bdpt_scene_desc* d, Scene<R>& sc, std::string& err, bool pt = false) {
  // Primitives (Triangle ctor triangle.cpp:9-21; Sphere sphere.h:23) in fp64, then precision R.
  std::vector<BBoxT<double>> pb(d->nprim);
  sc.prims.resize(d->nprim);
  for (int i = 0; i < d->nprim; i++) {
    const double* g = d->prim_geom + 18 * (size_t)i;
    Prim<R>& P = sc.prims[i];
    P.type = d->prim_type[i];
    P.mat = d->prim_mat[i];
    if (P.mat < 0 || P.mat >= d->nmat) { err = "bad material index"; return BDPT_E_INVALID; }
    if (P.type == BDPT_PRIM_TRIANGLE) {
      V3<double> p1 = v3d(g), p2 = v3d(g + 3), p3 = v3d(g + 6);
      BBoxT<double> b(p1);
      b.expand(p2);
      b.expand(p3);
      pb[i] = b;
      P.p1 = cvt<R>(p1); P.p2 = cvt<R>(p2); P.p3 = cvt<R>(p3);
      P.n1 = cvt<R>(v3d(g + 9)); P.n2 = cvt<R>(v3d(g + 12)); P.n3 = cvt<R>(v3d(g + 15));
    } else if (P.type == BDPT_PRIM_SPHERE) {
      V3<double> c = v3d(g);
      double r = g[3];
      pb[i] = BBoxT<double>(c - V3<double>(r, r, r), c + V3<double>(r, r, r));
      P.c = cvt<R>(c);
      P.r = (R)r;
      P.r2 = (sizeof(R) == 8) ? (R)(r * r) : P.r * P.r;  // sphere.h:23 r2(r*r)
    } else {
      err = "bad primitive type";
      return BDPT_E_INVALID;
    }
  }
  for (int i = 0; i < d->nmat; i++) {
    const bdpt_material& m = d->mats[i];
    if ((m.type == BDPT_MAT_MICROFACET && !pt) || m.type < 0 || m.type > BDPT_MAT_MICROFACET) {
      err = "unsupported material (microfacet sample_pdf asserts under BDPT)";
      return BDPT_E_UNSUPPORTED;
    }
    Mat<R> M;
    M.type = m.type;
    M.a = cvt<R>(v3d(m.a));
    M.b = cvt<R>(v3d(m.b));
    M.ior = (R)m.ior;
    M.alpha = (R)m.roughness;
    sc.mats.push_back(M);
  }
  if (d->nlight < 1 && !d->envmap) { err = "scene has no light"; return BDPT_E_INVALID; }
  for (int i = 0; i < d->nlight; i++) {
    const bdpt_light& l = d->lights[i];
    // InfiniteHemisphereLight (light.cpp:55-98) only implements sample_L: PathTracer only
    const bool ok = l.type == BDPT_LIGHT_AREA || l.type == BDPT_LIGHT_POINT ||
                    (pt && (l.type == BDPT_LIGHT_HEMISPHERE || l.type == BDPT_LIGHT_DIRECTIONAL));
    if (!ok) {
      err = "unsupported light type under BDPT";
      return BDPT_E_UNSUPPORTED;
    }
    Light<R> L;
    L.type = l.type;
    L.radiance = cvt<R>(v3d(l.radiance));
    L.position = cvt<R>(v3d(l.position));
    L.direction = cvt<R>(v3d(l.direction));
    L.dim_x = cvt<R>(v3d(l.dim_x));
    L.dim_y = cvt<R>(v3d(l.dim_y));
    L.area = (R)l.area;
    sc.lights.push_back(L);
  }
  // BVH (fp64 build, reference topology).
  std::vector<BBoxT<double>> boxes;
  BuildCtx B{&pb, &sc.nodes, &boxes, &sc.leaf_prims, 0};
  std::vector<int> all(d->nprim);
  for (int i = 0; i < d->nprim; i++) all[i] = i;
  if (d->nprim == 0) { err = "empty scene"; return BDPT_E_INVALID; }
  sc.root = construct_bvh(B, all, 0);
  if (sc.root < 0) { err = "degenerate BVH split"; return BDPT_E_INVALID; }
  sc.depth = B.depth;
  sc.dfs_rank.assign(d->nprim, 0);
  for (size_t i = 0; i < sc.leaf_prims.size(); i++) sc.dfs_rank[sc.leaf_prims[i]] = (int)i;
  sc.node_box.resize(boxes.size());
  for (size_t i = 0; i < boxes.size(); i++) {
    if (sizeof(R) == 8) {
      sc.node_box[i].mn = cvt<R>(boxes[i].mn);
      sc.node_box[i].mx = cvt<R>(boxes[i].mx);
    } else {
      V3<double> e = boxes[i].mx - boxes[i].mn;
      double ext = std::max(e.x, std::max(e.y, e.z));
      for (int k = 0; k < 3; k++) {
        sc.node_box[i].mn[k] = (R)pad_down(boxes[i].mn[k], ext);
        sc.node_box[i].mx[k] = (R)pad_up(boxes[i].mx[k], ext);
      }
    }
  }
  // Environment light, appended after the scene's lights (raytraced_renderer.cpp:117-119); tables
  // as EnvironmentLight::init (environment_light.cpp:18-62) in fp64.
  if (d->envmap) {
    const bdpt_envmap& em = *d->envmap;
    if (em.width <= 0 || em.height <= 0 || !em.rgb) { err = "bad environment map"; return BDPT_E_INVALID; }
    const int w = em.width, h = em.height;
    const size_t np = (size_t)w * h;
    std::vector<double> pdf(np), marg(h), cond(np);
    double sum = 0;
    for (int j = 0; j < h; ++j) {
      for (int i = 0; i < w; ++i) {
        const float* t = em.rgb + 3 * ((size_t)w * j + i);
        V3<double> px(t[0], t[1], t[2]);                                      // main.cpp:70-74
        float illum = 0.2126f * px.x + 0.7152f * px.y + 0.0722f * px.z;        // vector3D.h:231-233
        pdf[(size_t)w * j + i] = illum * std::sin(PI_D * (j + .5) / h);
        sum += pdf[(size_t)w * j + i];
      }
    }
    if (!(sum > 0)) { err = "environment map has no positive radiance"; return BDPT_E_INVALID; }
    for (int j = 0; j < h; ++j) {
      double prev = j == 0 ? 0 : marg[j - 1];
      marg[j] = prev;
      for (int i = 0; i < w; ++i) {
        pdf[(size_t)w * j + i] /= sum;
        marg[j] += pdf[(size_t)w * j + i];
      }
      double py = marg[j] - prev;
      for (int i = 0; i < w; i++) {   // (a zero row, never selected, gets a finite CDF)
        size_t k = (size_t)w * j + i;
        cond[k] = i == 0 ? 0 : cond[k - 1];
        cond[k] += py > 0 ? pdf[k] / py : 1.0 / w;
      }
    }
    EnvMap<R>& E = sc.env;
    E.w = w;
    E.h = h;
    E.marg.assign(marg.begin(), marg.end());
    E.cond.assign(cond.begin(), cond.end());
    E.pdf.assign(pdf.begin(), pdf.end());
    E.rgb.resize(np);
    for (size_t k = 0; k < np; k++) E.rgb[k] = V3<R>((R)em.rgb[3 * k], (R)em.rgb[3 * k + 1], (R)em.rgb[3 * k + 2]);
    // bounding sphere of all primitives: centre of the box, radius half its diagonal
    BBoxT<double> all_box = pb[0];
    for (int i = 1; i < d->nprim; i++) all_box.expand(pb[i]);
    V3<double> ctr((all_box.mn.x + all_box.mx.x) / 2, (all_box.mn.y + all_box.mx.y) / 2,
                   (all_box.mn.z + all_box.mx.z) / 2);
    V3<double> ext = all_box.mx - all_box.mn;
    double rad = std::sqrt(ext.x * ext.x + ext.y * ext.y + ext.z * ext.z) / 2;
    E.center = cvt<R>(ctr);
    E.rad = (R)rad;
    E.area = (R)(PI_D * rad * rad);
    Light<R> L;
    L.type = LIGHT_ENV_ORC;
    L.area = E.area;
    sc.env_light = (int)sc.lights.size();
    sc.lights.push_back(L);
  }
  // Camera
  const bdpt_camera& c = d->camera;
  sc.cam_pos = cvt<R>(v3d(c.pos));
  for (int k = 0; k < 3; k++) {
    sc.c2w[k] = cvt<R>(v3d(c.c2w + 3 * k));
    sc.w2c[k] = cvt<R>(v3d(c.w2c + 3 * k));
  }
  sc.hfov_deg = c.hfov_deg;
  sc.vfov_deg = c.vfov_deg;
  sc.nclip = (R)c.nclip;
  sc.fclip = (R)c.fclip;
  return BDPT_OK;
}

// ----------------------------------------------------------------------------------------------
// EnvironmentLight math (environment_light.cpp). Modes 0/1 (P::kDevEnv false) follow the
// reference's libm expressions exactly (pinned by tests/test_env.py against the reference's own
// EnvironmentLight); mode 2 the device's deterministic forms (bdpt_core.h env_*).
template <class R>
static int upper_idx(const std::vector<R>& a, size_t off, int n, R u) {   // std::upper_bound, <= n-1
  int k = (int)(std::upper_bound(a.begin() + off, a.begin() + off + n, u) - (a.begin() + off));
  return k < n ? k : n - 1;
}
template <class R>
static V3<R> env_bilerp(const EnvMap<R>& E, R x, R y) {                      // :106-123
  long right = lround_pos(x), left, v = lround_pos(y);
  R u1 = right - x + R(.5), v1;
  if (right == 0 || right == E.w) {
    left = E.w - 1;
    right = 0;
  } else left = right - 1;
  if (v == 0) v1 = v = 1;
  else if (v == E.h) {
    v = E.h - 1;
    v1 = 0;
  } else v1 = v - y + R(.5);
  long bottom = E.w * v, top = bottom - E.w;
  R u0 = 1 - u1;
  return (E.rgb[top + left] * u1 + E.rgb[top + right] * u0) * v1 +
         (E.rgb[bottom + left] * u1 + E.rgb[bottom + right] * u0) * (1 - v1);
}
// xy_to_theta_phi + theta_phi_to_dir (:88-104)
// glibc's sincos() and sin() can differ in the last bit. The compiler fuses the sin and cos of
// theta_phi_to_dir (environment_light.cpp:110-112) into one sincos() call, but sample_L's pdf
// (:166) calls sin() on its own: a non-inlined sin keeps that call plain here too.
__attribute__((noinline)) static double plain_sin(double x) { return std::sin(x); }
template <class P, class R>
static V3<R> env_xy_to_dir(const EnvMap<R>& E, R x, R y, R* sin_theta) {
  if (P::kDevEnv) {
    R cp, sp, ct, st;
    P::cos_sin_2pi(x / R(E.w), &cp, &sp);
    P::cos_sin_2pi((y / R(E.h)) * R(0.5), &ct, &st);
    *sin_theta = st;
    return V3<R>(-cp * st, ct, sp * st);
  }
  double phi = x / E.w * 2.0 * PI_D;
  double theta = y / E.h * PI_D;
  *sin_theta = (R)plain_sin(theta);   // sample_L's own sin() (:166), not the sincos() of :110-112
  return V3<R>((R)(std::cos(phi - PI_D) * std::sin(theta)), (R)std::cos(theta),
               (R)(-std::sin(phi - PI_D) * std::sin(theta)));
}
// dir_to_theta_phi + theta_phi_to_xy (:81-86, 97-102). Mode 2 takes the direction as unit.
template <class P, class R>
static void env_dir_to_xy(const EnvMap<R>& E, const V3<R>& d, R* x, R* y, R* sin_theta) {
  if (P::kDevEnv) {
    const R st = std::sqrt(std::max(R(0), (R(1) - d.y) * (R(1) + d.y)));
    const R th = atan2_f32(st, d.y);
    const R ph = atan2_f32(-d.z, d.x) + R(PI_D);
    *x = ph / R(2) / R(PI_D) * R(E.w);
    *y = th / R(PI_D) * R(E.h);
    *sin_theta = st;
    return;
  }
  V3<R> u = d.unit();
  double theta = std::acos(u.y);
  double phi = std::atan2(-u.z, u.x) + PI_D;
  *x = (R)(phi / 2. / PI_D * E.w);
  *y = (R)(theta / PI_D * E.h);
  *sin_theta = (R)std::sin(theta);
}
template <class P, class R>
static V3<R> env_radiance(const EnvMap<R>& E, const V3<R>& d) {             // sample_dir (:159-168)
  R x, y, st;
  env_dir_to_xy<P>(E, d, &x, &y, &st);
  return env_bilerp(E, x, y);
}
// solid-angle pdf of sample_L choosing direction d; 0 at the poles
template <class P, class R>
static R env_pdf_dir(const EnvMap<R>& E, const V3<R>& d) {
  R x, y, st;
  env_dir_to_xy<P>(E, d, &x, &y, &st);
  if (!(st > 0)) return 0;
  int i = std::min((int)x, E.w - 1), j = std::min((int)y, E.h - 1);
  return E.pdf[(size_t)E.w * j + i] * R(E.w * E.h) / (R(2) * R(PI_D) * R(PI_D) * st);
}
// sample_L's direction sampling (:126-156) from explicit uniforms: (ux, uy) the grid sample,
// (jx, jy) the texel jitter.
template <class P, class R>
static V3<R> env_sample_dir(const EnvMap<R>& E, R ux, R uy, R jx, R jy, V3<R>* wi, R* pdf) {
  int y = upper_idx(E.marg, 0, E.h, uy);
  int x = upper_idx(E.cond, (size_t)E.w * y, E.w, ux);
  R xf = x + jx, yf = y + jy;
  R st;
  *wi = env_xy_to_dir<P>(E, xf, yf, &st);
  *pdf = E.pdf[(size_t)E.w * y + x] * R(E.w * E.h) / (R(2) * R(PI_D) * R(PI_D) * st);
  return env_bilerp(E, xf, yf);
}

// ----------------------------------------------------------------------------------------------
struct Stats {
  uint64_t rays = 0, closest = 0, shadow = 0, nodes = 0, tri = 0, sph = 0, hits = 0;
};

template <class P>
struct Tracer {
  typedef typename P::R R;
  typedef V3<R> V;
  const Scene<R>& sc;
  P pol;
  int max_depth, W, H, ns_aa;
  R tanh_, tanv_;
  Stats st;
  bool rr = false;   // Russian roulette: PathVertex.q, bidirection.cpp:87-93
  // L[1]'s MIS densities when the light subpath starts on the environment light
  bool l1_env = false;
  R l1_mis_p = 0, l1_mis_dir = 0;
  // splat sink (lightBuffer & sampleBuffer updates, bidirection.cpp:457-466)
  std::vector<double>* light_buf = nullptr;   // W*H*3
  std::vector<double>* sample_buf = nullptr;  // mode 0 only (exact sampleBuffer order)

  struct Isect {            // intersection.h:21-34
    R t = (R)INFINITY;
    int prim = -1;
    V n;
    int mat = -1;           // bsdf == NULL
  };
  struct Vertex {           // bidirection.h:29-46
    Isect isect;
    R p = 1, q = 1;
    V alpha = V(1), position;
    bool is_light = false, new_sample = false;
    R dir_pdf = 0;
    bool env = false;       // environment vertex at infinity: isect.n = -w
  };

  Tracer(const Scene<R>& s, P p, int md, int w, int h, int spp)
      : sc(s), pol(p), max_depth(md), W(w), H(h), ns_aa(spp) {
    tanh_ = P::tan_half_fov(sc.hfov_deg);
    tanv_ = P::tan_half_fov(sc.vfov_deg);
  }

  // ---------------- geometry ----------------
  // BBox::intersect (bbox.cpp:10-56): rejects only when tmax < tmin.
  bool box_hit(const BBoxT<R>& b, const Ray<R>& r) const {
    R tmin_x = (b.mn.x - r.o.x) / r.d.x, tmax_x = (b.mx.x - r.o.x) / r.d.x;
    if (tmax_x < tmin_x) std::swap(tmin_x, tmax_x);
    R tmin_y = (b.mn.y - r.o.y) / r.d.y, tmax_y = (b.mx.y - r.o.y) / r.d.y;
    if (tmax_y < tmin_y) std::swap(tmin_y, tmax_y);
    R tmin_z = (b.mn.z - r.o.z) / r.d.z, tmax_z = (b.mx.z - r.o.z) / r.d.z;
    if (tmax_z < tmin_z) std::swap(tmin_z, tmax_z);
    R tmin = std::max(tmin_x, std::max(tmin_y, tmin_z));
    R tmax = std::min(tmax_x, std::min(tmax_y, tmax_z));
    if (tmax < tmin) return false;
    return true;
  }
  // Triangle::intersect (triangle.cpp:57-95)
  bool tri_hit(const Prim<R>& T, Ray<R>& r, Isect* is, int idx) {
    st.tri++;
    V o = r.o, d = r.d, p0 = T.p1, p1 = T.p2, p2 = T.p3;
    V e1 = p1 - p0, e2 = p2 - p0, s = o - p0;
    V s1 = cross(d, e2), s2 = cross(s, e1);
    R denom = dot(s1, e1);
    R t = dot(s2, e2) / denom;
    R b1 = dot(s1, s) / denom;
    R b2 = dot(s2, d) / denom;
    if (t >= r.min_t && t <= r.max_t && b1 >= 0 && b2 >= 0 && b1 + b2 <= 1) {
      V normal = T.n1 * (1 - b1 - b2) + b1 * T.n2 + b2 * T.n3;
      normal.normalize();
      r.max_t = t;
      is->t = t;
      is->n = normal;
      is->prim = idx;
      is->mat = T.mat;
      return true;
    }
    return false;
  }
  // Sphere::test/intersect (sphere.cpp:11-35,61-93). The quadratic is always solved in fp64
  // (in mode 2 from the fp32 ray and sphere): in fp32 the reference's b*b - 4ac cancels
  // catastrophically for rays from the camera (|o-c|^2 ~ 20 vs r^2 = 0.09), which moves hits by
  // ~1e-5 and self-shadows the EPS_F-offset connection rays (DESIGN.md §fp32 semantics).
  bool sph_hit(const Prim<R>& S, Ray<R>& r, Isect* is, int idx) {
    st.sph++;
    V3<double> o((double)r.o.x, (double)r.o.y, (double)r.o.z), d((double)r.d.x, (double)r.d.y, (double)r.d.z);
    V3<double> vc((double)S.c.x, (double)S.c.y, (double)S.c.z);
    double r2 = (sizeof(R) == 8) ? (double)S.r2 : (double)S.r * (double)S.r;
    double a = d.norm2();
    double b = 2 * dot(o - vc, d);
    double c = (o - vc).norm2() - r2;
    double delta = b * b - 4 * a * c;
    if (delta < 0) return false;
    double root = std::sqrt(delta);
    double t1 = (-b - root) / (2 * a);
    double t2 = (-b + root) / (2 * a);
    double t = -1;
    if (t1 >= (double)r.min_t && t1 <= (double)r.max_t) t = t1;
    else if (t2 >= (double)r.min_t && t2 <= (double)r.max_t) t = t2;
    if (t > 0) {
      R tr = (R)t;
      r.max_t = tr;
      V p = r.o + tr * r.d;
      V normal = p - S.c;
      normal.normalize();
      is->t = tr;
      is->n = normal;
      is->prim = idx;
      is->mat = S.mat;
      return true;
    }
    return false;
  }
  // BVHAccel::intersect (bvh.cpp:161-188): visit every child whose slab test passes, l then r.
  bool node_hit(Ray<R>& r, Isect* is, int node) {
    st.nodes++;
    if (!box_hit(sc.node_box[node], r)) return false;
    const BvhNode& N = sc.nodes[node];
    if (N.l < 0) {
      bool hit = false, h;
      for (int k = N.start; k < N.end; k++) {
        int pi = sc.leaf_prims[k];
        const Prim<R>& pr = sc.prims[pi];
        h = (pr.type == BDPT_PRIM_TRIANGLE) ? tri_hit(pr, r, is, pi) : sph_hit(pr, r, is, pi);
        hit = h || hit;
      }
      return hit;
    }
    bool h1 = node_hit(r, is, N.l);
    bool h2 = node_hit(r, is, N.r);
    return h1 || h2;
  }
  bool intersect(Ray<R> r, Isect* is, bool closest) {
    st.rays++;
    if (closest) st.closest++; else st.shadow++;
    bool h = node_hit(r, is, sc.root);
    if (h && closest) st.hits++;
    return h;
  }

  // ---------------- samplers (sampler.cpp) ----------------
  void grid2d(R* x, R* y) {        // Vector2D(random_uniform(), random_uniform()): y drawn first
    R b = pol.uS();
    R a = pol.uS();
    *x = a;
    *y = b;
  }
  V cosine_hemi(R* pdf) {          // sampler.cpp:76-86
    R Xi1 = pol.uS();
    R Xi2 = pol.uS();
    R r = std::sqrt(Xi1);
    *pdf = std::sqrt(1 - Xi1) / R(PI_D);
    R c, s;
    P::cos_sin_2pi(Xi2, &c, &s);
    return V(r * c, r * s, std::sqrt(1 - Xi1));
  }
  static R cosine_pdf(const V& v) { return v.z > 0 ? v.z / R(PI_D) : R(0); }   // sampler.cpp:92-95
  V sphere_uniform() {             // sampler.cpp:17-25
    R z = pol.uS() * 2 - 1;
    R sinTheta = std::sqrt(std::max(R(0), R(1.0f) - z * z));
    R u = pol.uS();
    R c, s;
    P::cos_sin_2pi(u, &c, &s);
    return V(c * sinTheta, s * sinTheta, z);
  }

  // ---------------- BSDFs ----------------
  static void reflect(const V& wo, V* wi) { *wi = V(-wo.x, -wo.y, wo.z); }   // advanced_bsdf.cpp:272-277
  static bool refract(const V& wo, V* wi, R ior) {                            // :279-303
    bool enter = wo.z > 0;
    R eta = enter ? R(1) / ior : ior;
    R z_sq = 1 - eta * eta * (1 - wo.z * wo.z);
    if (z_sq < 0) return false;
    R sgn = enter ? R(-1) : R(1);
    *wi = V(-eta * wo.x, -eta * wo.y, sgn * std::sqrt(z_sq));
    return true;
  }
  // ---------------- MicrofacetBSDF (advanced_bsdf.cpp:46-142, bsdf.h:176-184) ----------------
  // Modes 0/1: the reference's libm expressions; mode 2 (P::kDevEnv): the device's fp32 forms
  // (cos(acos z) = z, tan(acos z) = sqrt(1 - z^2) / z, integer powers by products; erf / exp / log
  // / sqrt from the fp32 math library).
  R mf_lambda(R alpha, const V& w) const {
    if (P::kDevEnv) {
      const R c = std::min(std::max(w.z, R(-1.0 + 1e-5)), R(1.0 - 1e-5));
      const R t = std::sqrt(R(1) - c * c) / c;
      const R a = R(1) / (alpha * t);
      return R(0.5) * (std::erf(a) - R(1) + std::exp(-a * a) / (a * R(PI_D)));
    }
    double theta = std::acos(std::min(std::max((double)w.z, -1.0 + 1e-5), 1.0 - 1e-5));
    double a = 1.0 / (alpha * std::tan(theta));
    return (R)(0.5 * (std::erf(a) - 1.0 + std::exp(-a * a) / (a * PI_D)));
  }
  R mf_G(R alpha, const V& wo, const V& wi) const { return R(1.0) / (R(1.0) + mf_lambda(alpha, wi) + mf_lambda(alpha, wo)); }
  R mf_D(R alpha, const V& h) const {
    if (P::kDevEnv) {
      const R c = h.z;
      const R t = std::sqrt(std::max(R(0), R(1) - c * c)) / c;
      const R q = t / alpha;
      const R c2 = c * c;
      return std::exp(-(q * q)) / (R(PI_D) * alpha * alpha * (c2 * c2));
    }
    double theta = std::acos(h.z);
    double nom = std::exp(-std::pow(std::tan(theta) / alpha, 2));
    double denom = PI_D * alpha * alpha * std::pow(std::cos(theta), 4);
    return (R)(nom / denom);
  }
  V mf_F(const Mat<R>& M, const V& wi) const {
    R c = std::fabs(wi.z) / wi.norm();
    R c2 = P::pow2(c);
    V e2k2 = M.a * M.a + M.b * M.b;
    V Rs = (e2k2 - R(2) * M.a * c + V(c2)) / (e2k2 + R(2) * M.a * c + V(c2));
    V Rp = (e2k2 * c2 - R(2) * M.a * c + V(R(1))) / (e2k2 * c2 + R(2) * M.a * c + V(R(1)));
    return (Rs + Rp) / R(2);
  }
  V mf_f(const Mat<R>& M, const V& wo, const V& wi) const {
    if (wo.z <= R(EPS_F) || wi.z <= R(EPS_F)) return V();
    V h = wo + wi;
    h.normalize();
    return mf_F(M, wi) * mf_G(M.alpha, wo, wi) * mf_D(M.alpha, h) / (R(4) * wo.z * wi.z);
  }
  V mf_sample_f(const Mat<R>& M, const V& wo, V* wi, R* pdf) {
    R rx, ry;
    grid2d(&rx, &ry);
    const R alpha = M.alpha;
    R st, ct, sp, cp, th_t;   // sin/cos theta, sin/cos phi, tan theta
    if (P::kDevEnv) {
      th_t = std::sqrt(-alpha * alpha * std::log(R(1) - rx));
      ct = R(1) / std::sqrt(R(1) + th_t * th_t);
      st = th_t * ct;
      P::cos_sin_2pi(ry, &cp, &sp);
    } else {
      double theta = std::atan(std::sqrt(-alpha * alpha * std::log(1 - rx)));
      double phi = 2 * PI_D * ry;
      st = std::sin(theta); ct = std::cos(theta); sp = std::sin(phi); cp = std::cos(phi);
      th_t = std::tan(theta);
    }
    V h(st * cp, st * sp, ct);
    R costheta = dot(wo, h) / wo.norm();
    V d = wo - h * costheta * wo.norm();
    *wi = h * costheta * wo.norm() - d;
    wi->normalize();
    if (wo.z <= R(EPS_F) || wi->z <= R(EPS_F)) {
      *pdf = 1;
      *wi = V(0, 0, 1);
      return V();
    }
    R p_theta;
    if (P::kDevEnv) {
      const R q = th_t / alpha, c2 = ct * ct;
      p_theta = R(2) * st * std::exp(-(q * q)) / (alpha * alpha * (c2 * ct));
    } else {
      double theta = std::atan(std::sqrt(-alpha * alpha * std::log(1 - rx)));
      p_theta = (R)(2 * std::sin(theta) * std::exp(-std::pow(std::tan(theta) / alpha, 2)) /
                    (alpha * alpha * std::pow(std::cos(theta), 3)));
    }
    R p_phi = R(1.) / (R(2) * R(PI_D));
    R pdf_h = p_theta * p_phi / st;
    *pdf = pdf_h / (R(4) * dot(*wi, h));
    return mf_f(M, wo, *wi);
  }

  V bsdf_f(int m, const V& wo, const V& wi) const {
    const Mat<R>& M = sc.mats[m];
    if (M.type == BDPT_MAT_DIFFUSE) {                                         // bsdf.cpp:52-62
      if (wo.z < 0. || wi.z < 0.) return V();
      return M.a / R(PI_D);
    }
    if (M.type == BDPT_MAT_MICROFACET) return mf_f(M, wo, wi);              // PathTracer only
    return V();                                      // emission/mirror/glass/refraction f = 0
  }
  V bsdf_sample_f(int m, const V& wo, V* wi, R* pdf) {
    const Mat<R>& M = sc.mats[m];
    switch (M.type) {
      case BDPT_MAT_DIFFUSE: {                                                // bsdf.cpp:67-77
        *wi = cosine_hemi(pdf);
        return bsdf_f(m, wo, *wi);
      }
      case BDPT_MAT_EMISSION: {                                               // bsdf.cpp:103-108
        *pdf = R(1.0) / R(PI_D);
        *wi = cosine_hemi(pdf);
        return V();
      }
      case BDPT_MAT_MICROFACET: return mf_sample_f(M, wo, wi, pdf);            // :89-142
      case BDPT_MAT_MIRROR: {                                                 // advanced_bsdf.cpp:21-29
        reflect(wo, wi);
        *pdf = 1;
        R costheta = std::fabs(wi->z) / wi->norm();
        return M.a / costheta;
      }
      case BDPT_MAT_REFRACTION: {                                             // :163-178
        if (!refract(wo, wi, M.ior)) { *pdf = 1; return V(); }  // reference leaves pdf unset
        *pdf = 1;
        R eta = wo.z > 0 ? R(1) / M.ior : M.ior;
        R costheta = std::fabs(wi->z) / wi->norm();
        return M.b / costheta / (eta * eta);
      }
      default: {                                                              // glass :198-237
        V wi_reflect, wi_refract;
        reflect(wo, &wi_reflect);
        bool tir = !refract(wo, &wi_refract, M.ior);
        if (tir) {
          *pdf = 1;
          *wi = wi_reflect;
          R costheta = std::fabs(wi->z) / wo.norm();
          return M.a / costheta;
        }
        R c_ref = std::fabs(wi_refract.z) / wi_refract.norm();
        R eta = wo.z > 0 ? R(1) / M.ior : M.ior;
        R R0 = P::pow2((1 - eta) / (1 + eta));
        R Rf = R0 + (1 - R0) * P::pow5(1 - c_ref);
        if (pol.uG() < Rf) {                                                  // coin_flip(R)
          *wi = wi_reflect;
          *pdf = Rf;
          R costheta = std::fabs(wi->z) / wi->norm();
          return Rf * M.a / costheta;
        } else {
          *wi = wi_refract;
          *pdf = 1 - Rf;
          R costheta = std::fabs(wi->z) / wi->norm();
          return (1 - Rf) * M.b / costheta / (eta * eta);
        }
      }
    }
  }
  R bsdf_sample_pdf(int m, const V& wo, const V& wi) const {
    const Mat<R>& M = sc.mats[m];
    switch (M.type) {
      case BDPT_MAT_DIFFUSE:
      case BDPT_MAT_EMISSION: return cosine_pdf(wi);                           // bsdf.cpp:81-85,112-117
      case BDPT_MAT_MIRROR:
      case BDPT_MAT_REFRACTION: return 1.;                                     // advanced_bsdf.cpp:32,181
      default: {                                                               // glass :240-259
        V wo_reflect, wo_refract, wi_ = wi;
        reflect(wi_, &wo_reflect);
        bool tir = !refract(wi_, &wo_refract, M.ior);
        if (tir) return 1.;
        R c = std::fabs(wo_refract.z) / wo_refract.norm();
        R eta = wo.z > 0 ? R(1) / M.ior : M.ior;
        R R0 = P::pow2((1 - eta) / (1 + eta));
        R Rf = R0 + (1 - R0) * P::pow5(1 - c);
        if (wi.z > 0.) return Rf;
        return 1 - Rf;
      }
    }
  }
  V get_emission(int m) const { return sc.mats[m].type == BDPT_MAT_EMISSION ? sc.mats[m].a : V(); }
  bool is_delta(int m) const {
    if (m < 0) return false;
    int t = sc.mats[m].type;
    return t == BDPT_MAT_MIRROR || t == BDPT_MAT_GLASS || t == BDPT_MAT_REFRACTION;
  }

  // ---------------- lights (light.cpp) ----------------
  V light_sample_Le(const Light<R>& L, Ray<R>* ray, R* point_pdf, R* dir_pdf, V* normal) {
    l1_env = false;
    if (L.type == LIGHT_ENV_ORC) {   // importance-sampled w, origin on the disk facing -w
      const EnvMap<R>& E = sc.env;
      R ux, uy;
      grid2d(&ux, &uy);
      R jx = pol.uE();
      R jy = pol.uE();
      V w;
      R pw;
      V Le = env_sample_dir<P>(E, ux, uy, jx, jy, &w, &pw);
      R u1 = pol.uS(), u2 = pol.uS();
      R r = E.rad * std::sqrt(u1);
      R c, s;
      P::cos_sin_2pi(u2, &c, &s);
      Frame<R> f = make_coord_space(w);
      ray->o = E.center + E.rad * w + (r * c) * f.X + (r * s) * f.Y;
      ray->d = -w; ray->min_t = 0; ray->max_t = (R)INFINITY;
      *point_pdf = R(1) / E.area;
      *dir_pdf = pw;
      *normal = -w;
      l1_env = true;
      l1_mis_p = pw;
      l1_mis_dir = R(1) / E.area;
      return Le;
    }
    if (L.type == BDPT_LIGHT_POINT) {                                        // :115-123
      V d = sphere_uniform();
      ray->o = L.position; ray->d = d; ray->min_t = 0; ray->max_t = (R)INFINITY;
      *point_pdf = 1;
      *dir_pdf = R(0.25) / R(PI_D);
      *normal = d;
      return L.radiance;
    }
    R sx, sy;                                                                 // :219-232
    grid2d(&sx, &sy);
    sx = sx - R(0.5f);
    sy = sy - R(0.5f);
    V o = L.position + sx * L.dim_x + sy * L.dim_y;
    V d = cosine_hemi(dir_pdf);
    Frame<R> f = make_coord_space(L.direction);
    ray->o = o; ray->d = f.to_world(d); ray->min_t = 0; ray->max_t = (R)INFINITY;
    *point_pdf = R(1.) / L.area;
    *normal = L.direction;
    return L.radiance;
  }
  V light_sample_Le_point(const Light<R>& L, const V& p, V* wi, V* point, R* dist, R* point_pdf,
                          R* dir_pdf, V* normal) {
    if (L.type == LIGHT_ENV_ORC) {   // a vertex at infinity in direction w
      R ux, uy;
      grid2d(&ux, &uy);
      R jx = pol.uE();
      R jy = pol.uE();
      R pw;
      V Le = env_sample_dir<P>(sc.env, ux, uy, jx, jy, wi, &pw);
      *point = p;
      *dist = (R)INFINITY;
      *point_pdf = pw;
      *dir_pdf = R(1) / sc.env.area;
      *normal = -(*wi);
      return Le;
    }
    if (L.type == BDPT_LIGHT_POINT) {                                        // :125-137
      V d = L.position - p;
      *wi = d.unit();
      *dist = d.norm();
      *point_pdf = 1.0;
      *dir_pdf = R(0.25) / R(PI_D);
      *normal = -(*wi);
      *point = L.position;
      return L.radiance;
    }
    R sx, sy;                                                                 // :234-255
    grid2d(&sx, &sy);
    sx = sx - R(0.5f);
    sy = sy - R(0.5f);
    *point = L.position + sx * L.dim_x + sy * L.dim_y;
    V d = *point - p;
    R cosTheta = dot(d, L.direction);
    R sqDist = d.norm2();
    R dd = std::sqrt(sqDist);
    *wi = d / dd;
    *dist = dd;
    *point_pdf = R(1.) / L.area;
    *normal = L.direction;
    Frame<R> f = make_coord_space(L.direction);
    *dir_pdf = cosine_pdf(f.to_local(-(*wi)));
    return cosTheta < 0 ? L.radiance : V();
  }
  bool light_contain_point(const Light<R>& L, const V& p) const {
    if (L.type == BDPT_LIGHT_POINT) return (p - L.position).norm() < R(EPS_F);   // :139-142
    V d = L.position - p;                                                     // :257-262
    d.normalize();
    return std::fabs(dot(d, L.direction)) < R(EPS_F);
  }
  // env light: only ever asked about an environment vertex (direction -n) or, for
  // the step below one, about the planar density of its emission disk
  V env_light_pdf(const Vertex& v, R* point_pdf, R* dir_pdf) const {
    const V w = -v.isect.n;
    *point_pdf = env_pdf_dir<P>(sc.env, w) / R(sc.lights.size());
    *dir_pdf = R(1) / sc.env.area;
    return env_radiance<P>(sc.env, w);
  }
  V light_sample_pdf(const Light<R>& L, const V& p, const V& wi, R* point_pdf, R* dir_pdf) const {
    if (!light_contain_point(L, p)) { *point_pdf = 0.; *dir_pdf = 0.; return V(); }
    if (L.type == BDPT_LIGHT_POINT) {                                        // :144-153
      *point_pdf = 1.0;
      *dir_pdf = R(0.25) / R(PI_D);
      return L.radiance;
    }
    *point_pdf = R(1.) / L.area;                                              // :264-284
    Frame<R> f = make_coord_space(L.direction);
    V wl = f.to_local(-wi);
    wl.normalize();
    *dir_pdf = cosine_pdf(wl);
    return *dir_pdf > 0. ? L.radiance : V();
  }

  // sample_L (light.cpp:18-23, 103-113, 205-217; environment_light.cpp:126-156): the PathTracer's
  // next-event estimation. AreaLight's pdf is the solid-angle one; the caller divides by dist^2
  // once more (pathtracer.cpp:147, the reference's own convention).
  V light_sample_L(const Light<R>& L, const V& p, V* wi, R* dist, R* pdf) {
    if (L.type == LIGHT_ENV_ORC) {
      R ux, uy;
      grid2d(&ux, &uy);
      R jx = pol.uE();
      R jy = pol.uE();
      *dist = (R)INFINITY;
      return env_sample_dir<P>(sc.env, ux, uy, jx, jy, wi, pdf);
    }
    if (L.type == BDPT_LIGHT_POINT) {
      V d = L.position - p;
      *wi = d.unit();
      *dist = d.norm();
      *pdf = 1.0;
      return L.radiance;
    }
    if (L.type == BDPT_LIGHT_DIRECTIONAL) {  // light.cpp:17-23
      *wi = L.direction;
      *dist = (R)INFINITY;
      *pdf = 1.0;
      return L.radiance;
    }
    if (L.type == BDPT_LIGHT_HEMISPHERE) {   // light.cpp:62-70 with sampler.cpp:36-49
      R Xi1 = pol.uS();
      R Xi2 = pol.uS();
      V dir;
      if (P::kDevEnv) {                       // the device's form: cos(acos x) = x, sin = sqrt(1-x^2)
        R c, s;
        P::cos_sin_2pi(Xi2, &c, &s);
        const R st = std::sqrt(std::max(R(0), R(1) - Xi1 * Xi1));
        dir = V(st * c, st * s, Xi1);
      } else {                                // fp64 theta/phi through the float libm calls
        const double theta = std::acos((double)Xi1);
        const double phi = 2.0 * PI_D * (double)Xi2;
        dir = V((R)(sinf(theta) * cosf(phi)), (R)(sinf(theta) * sinf(phi)), (R)cosf(theta));
      }
      *wi = V(dir.x, dir.z, -dir.y);          // sampleToWorld = [x, -z, y] columns (:55-60)
      *dist = (R)INFINITY;
      *pdf = R(1.0 / (2.0 * PI_D));
      return L.radiance;
    }
    R sx, sy;
    grid2d(&sx, &sy);
    sx = sx - R(0.5f);
    sy = sy - R(0.5f);
    V d = L.position + sx * L.dim_x + sy * L.dim_y - p;
    R cosTheta = dot(d, L.direction);
    R sqDist = d.norm2();
    R dd = std::sqrt(sqDist);
    *wi = d / dd;
    *dist = dd;
    *pdf = sqDist / (L.area * std::fabs(cosTheta));
    return cosTheta < 0 ? L.radiance : V();
  }
  bool light_is_delta(const Light<R>& L) const {
    return L.type == BDPT_LIGHT_POINT || L.type == BDPT_LIGHT_DIRECTIONAL;
  }

  // ---------------- camera (camera.cpp) ----------------
  Ray<R> generate_ray(R x, R y) const {                                       // :191-212
    V rd;
    rd.x = (2 * x - 1) * tanh_;
    rd.y = (2 * y - 1) * tanv_;
    rd.z = -1;
    V wd = rd.x * sc.c2w[0] + rd.y * sc.c2w[1] + rd.z * sc.c2w[2];
    wd.normalize();
    Ray<R> r;
    r.o = sc.cam_pos;
    r.d = wd;
    r.min_t = sc.nclip;
    r.max_t = sc.fclip;
    return r;
  }
  // Camera::generate_ray_for_thin_lens (camera_lens.cpp:22-43)
  R lens_radius = 0, focal_distance = R(4.7);
  // uTheta: the lens sample's y; the reference passes rndTheta = uTheta * 2.0 * PI
  // (pathtracer.cpp:315), mode 2 takes cos/sin(2 pi u) from the device polynomial.
  Ray<R> generate_ray_thin_lens(R x, R y, R rndR, R uTheta) const {
    V pLens;
    if (P::kDevEnv) {
      R c, s;
      P::cos_sin_2pi(uTheta, &c, &s);
      pLens = V(lens_radius * std::sqrt(rndR) * c, lens_radius * std::sqrt(rndR) * s, 0);
    } else {
      R rndTheta = uTheta * 2.0 * PI_D;
      pLens = V(lens_radius * std::sqrt(rndR) * std::cos(rndTheta), lens_radius * std::sqrt(rndR) * std::sin(rndTheta), 0);
    }
    V rayDir((2 * x - 1) * tanh_, (2 * y - 1) * tanv_, -1);
    V pFocus = rayDir * focal_distance;
    rayDir = pFocus - pLens;
    V wd = rayDir.x * sc.c2w[0] + rayDir.y * sc.c2w[1] + rayDir.z * sc.c2w[2];
    wd.normalize();
    V lo = pLens.x * sc.c2w[0] + pLens.y * sc.c2w[1] + pLens.z * sc.c2w[2];
    Ray<R> r;
    r.o = sc.cam_pos + lo;
    r.d = wd;
    r.min_t = sc.nclip;
    r.max_t = sc.fclip;
    return r;
  }

  V sample_ray_pdf(const V& p, V* wi, V* eye_point, R* dist, R* point_pdf, R* dir_pdf, V* normal,
                   int* x, int* y) const {                                     // :214-248
    *wi = sc.cam_pos - p;
    *dist = wi->norm();
    wi->normalize();
    *eye_point = sc.cam_pos;
    *point_pdf = 1.0;
    V mw = -(*wi);
    V wc = mw.x * sc.w2c[0] + mw.y * sc.w2c[1] + mw.z * sc.w2c[2];
    wc.z = -wc.z;
    R cos_t = P::cos_acos(wc.z);
    R denom = 4 * tanh_ * tanv_ / P::pow4(cos_t);
    *dir_pdf = ((*dist) * (*dist)) / cos_t;
    *normal = -(*wi);
    wc /= wc.z;
    R fx = ((wc.x / tanh_ + 1) * R(0.5)) * W;
    R fy = ((wc.y / tanv_ + 1) * R(0.5)) * H;
    // C++ float->int truncation; NaN / out-of-int-range -> -1 (never splatted), see DESIGN.md.
    *x = (fx > R(-1) && fx < R(W)) ? (int)fx : -1;
    *y = (fy > R(-1) && fy < R(H)) ? (int)fy : -1;
    return V(R(1.)) / denom;
  }

  // ---------------- BDPT (bidirection.cpp) ----------------
  void prepare_subpath(Ray<R> r, R point_pdf, R dir_pdf, std::vector<Vertex>& path,
                       const V& init_radiance, const V& init_normal, bool is_light) {  // :20-102
    Vertex v;
    path.push_back(v);
    v.p = point_pdf;
    v.alpha = init_radiance / point_pdf;
    v.isect.n = init_normal;
    v.position = r.o;
    v.q = 1.;
    v.is_light = is_light;
    v.dir_pdf = dir_pdf;
    path.push_back(v);
    if (is_light && l1_env) {   // env light: L[1]'s MIS densities
      path[1].env = true;
      path[1].p = l1_mis_p / R(sc.lights.size());
      path[1].dir_pdf = l1_mis_dir;
    }
    v.env = false;
    int i = 2;
    Isect isect;
    R prev_pdf = dir_pdf;
    V prev_f(1., 1., 1.), prev_n(init_normal);
    for (;;) {
      if (!intersect(r, &isect, true)) {
        if (!is_light && sc.env_light >= 0) {   // the escaped eye ray ends on the environment
          Vertex e;
          e.env = true;
          e.isect.n = -r.d;
          e.position = r.o;
          e.alpha = path[i - 1].alpha * std::fabs(dot(prev_n, r.d)) * prev_f / prev_pdf;
          e.q = 1.;
          path.push_back(e);
        }
        break;
      }
      r.max_t = isect.t;  // (not read again: the next ray is rebuilt below)
      Frame<R> f = hit_coord_space(isect.n);
      const V hit_p = r.o + r.d * isect.t;
      const V w_out = f.to_local(-r.d);
      V wi, fv, wi_world;
      R pdf;
      fv = bsdf_sample_f(isect.mat, w_out, &wi, &pdf);
      wi_world = f.to_world(wi);
      wi_world.normalize();
      v.isect = isect;
      R g = std::fabs(dot(prev_n, r.d) * dot(isect.n, r.d)) / (isect.t * isect.t);
      v.p = path[i - 1].p * prev_pdf * g;
      v.alpha = path[i - 1].alpha * std::fabs(dot(prev_n, r.d)) * prev_f / prev_pdf;
      v.position = hit_p;
      v.is_light = false;
      Ray<R> ray;
      ray.o = hit_p; ray.d = wi_world; ray.min_t = R(EPS_F); ray.max_t = (R)INFINITY;
      r = ray;
      R p_keep = 1;
      v.q = p_keep;
      path.push_back(v);
      if (i >= max_depth + 1) break;
      if (rr && i > 3) {   // bidirection.cpp:87-93 with min_subpath_length = 3 (BDPT_RR_MIN)
        p_keep = pdf > 0 ? std::min(R(1), fv.norm() / pdf) : R(0);
        path.back().q = p_keep;
        if (!(pol.uS() < p_keep)) break;   // coin_flip(p_keep)
      }
      prev_f = fv;
      prev_n = isect.n;
      prev_pdf = pdf * p_keep;
      i++;
    }
  }
  Ray<R> sample_light_ray(R& point_pdf, R& dir_pdf, V& init_radiance, V& init_normal) {  // :105-118
    int n = (int)sc.lights.size();
    int id = pol.rand_light(n);
    Ray<R> r;
    V rad = light_sample_Le(sc.lights[id], &r, &point_pdf, &dir_pdf, &init_normal);
    point_pdf /= R(n);
    init_radiance = rad;
    r.min_t = R(EPS_F);
    return r;
  }

  // One Horner step of the mode-2 MIS sum; a term whose inner sum is zero stays exactly zero
  // (no inf * 0) — the same convention as the device (bdpt_core.h mis_horner).
  static R horner_step(R f, bool t, R g) {
    R s = t ? R(1.) + g : g;
    return s == R(0.) ? R(0.) : (f * f) * s;
  }

  // One MIS step (bidirection.cpp:151-158 and the five copies that follow): d = unit(cur - oth),
  // g = |(frame(oth.n)^T d).z * dot(d, cur.n)| / dist^2, with the environment rules of DESIGN.md §9
  // (oth env: d = oth.n = -w, g = |dot(d, cur.n)|; cur env: d = -cur.n = w, g = 1).
  R step(const Vertex& cur, const Vertex& oth, V* d_out) const {
    if (cur.env) { *d_out = -cur.isect.n; return R(1.); }
    if (oth.env) { *d_out = oth.isect.n; return std::fabs(dot(oth.isect.n, cur.isect.n)); }
    Frame<R> f = oth.isect.mat >= 0 ? hit_coord_space(oth.isect.n) : make_coord_space(oth.isect.n);
    V wi_world = cur.position - oth.position;
    R dist = wi_world.norm();
    wi_world.normalize();
    V wi = f.to_local(wi_world);
    *d_out = wi_world;
    return std::fabs(wi.z * dot(wi_world, cur.isect.n)) / (dist * dist);
  }
  R pdf_from(const Vertex& v, const V& d) const {   // v.bsdf->sample_pdf(0, frame(v.n)^T d)
    V wo;
    return bsdf_sample_pdf(v.isect.mat, wo, hit_coord_space(v.isect.n).to_local(d));
  }

  R mis_weight(int i_eye, int i_light, const std::vector<Vertex>& E, const std::vector<Vertex>& L,
               const Vertex& LS, const Vertex& ES) {                          // :121-293
    R w_inv = 0., ratio = 1.;
    w_inv += ratio;
    R fE[64], fL[64];
    bool tE[64], tL[64];
    int eye_light = -1;
    for (int i = i_eye; i > 1; i--) {
      const Vertex& cur = E[i];
      const Vertex& prv = (i == i_eye) ? (i_light == 1 ? LS : L[i_light]) : E[i + 1];
      const Vertex& nxt = E[i - 1];
      R nom, denom, p = 0, g;
      V d;
      if (i_light == 0 && i == i_eye) {
        // the light containing cur: the env light for an environment vertex, else the first
        // area / point light whose contain_point holds (the env light contains no surface point)
        if (cur.env) {
          eye_light = sc.env_light;
        } else {
          for (size_t j = 0; j < sc.lights.size(); j++)
            if (sc.lights[j].type != LIGHT_ENV_ORC && light_contain_point(sc.lights[j], cur.position)) {
              eye_light = (int)j;
              break;
            }
        }
        if (eye_light < 0) return 0.;
        g = 1.;
        R pp, dp;
        if (cur.env) env_light_pdf(cur, &pp, &dp);
        else light_sample_pdf(sc.lights[eye_light], cur.position, V(), &pp, &dp);
        p = pp;
      } else {
        g = step(cur, prv, &d);
        if (i_light == 1 && i == i_eye) {
          p = LS.dir_pdf * LS.q;
        } else if (i_light == 0 && i == i_eye - 1) {
          R pp, dp;
          if (prv.env) env_light_pdf(prv, &pp, &dp);
          else light_sample_pdf(sc.lights[eye_light], prv.position, -d, &pp, &dp);
          p = dp * L[1].q;
        } else {
          p = pdf_from(prv, d) * prv.q;
        }
      }
      nom = p * g;
      g = step(cur, nxt, &d);
      if (i == 2) {
        p = 1.;
        g = 1.;
      } else {
        p = pdf_from(nxt, d) * nxt.q;
      }
      denom = p * g;
      // an environment vertex right after the camera has no camera-connection strategy (§9)
      const bool t = !(is_delta(cur.isect.mat) || is_delta(nxt.isect.mat)) && !(cur.env && i == 2);
      if (P::kHornerMis) {
        fE[i] = nom / denom;
        tE[i] = t;
        continue;
      }
      ratio *= nom / denom;
      if (!t) continue;
      w_inv += ratio * ratio;
    }
    ratio = 1.;
    for (int i = i_light; i > 0; i--) {
      // environment scenes: the light end of (i, 1) is the fresh sample itself;
      // otherwise the reference's original L[1] (quirk 5)
      const Vertex& cur = (i == 1 && i_light == 1 && sc.env_light >= 0) ? LS : L[i];
      const Vertex& prv = (i == i_light) ? (i_eye == 1 ? ES : E[i_eye]) : L[i + 1];
      const Vertex& nxt = L[i - 1];
      R nom, denom, p, g;
      V d;
      g = step(cur, prv, &d);
      if (i_eye <= 1 && i == i_light) p = ES.dir_pdf * ES.q;
      else p = pdf_from(prv, d) * prv.q;
      nom = p * g;
      if (i > 1) {
        g = step(cur, nxt, &d);
        if (i == 2) p = nxt.dir_pdf;
        else p = pdf_from(nxt, d) * nxt.q;
        denom = p * g;
      } else {
        denom = cur.p;
      }
      const bool t = !(is_delta(cur.isect.mat) || is_delta(nxt.isect.mat));
      if (P::kHornerMis) {
        fL[i] = nom / denom;
        tL[i] = t;
        continue;
      }
      ratio *= nom / denom;
      if (!t) continue;
      w_inv += ratio * ratio;
    }
    if (P::kHornerMis) {
      // sum_k t_k (f_k ... f_end)^2 = G_end with G_k = f_k^2 (t_k + G_{k-1}), innermost vertex first
      R ge = 0, gl = 0;
      for (int k = 2; k <= i_eye; k++) ge = horner_step(fE[k], tE[k], ge);
      for (int k = 1; k <= i_light; k++) gl = horner_step(fL[k], tL[k], gl);
      return R(1.) / ((R(1.) + ge) + gl);
    }
    return R(1.) / w_inv;
  }

  // ---------------- the unidirectional PathTracer (pathtracer.cpp:47-340) ----------------
  int ns_area_light = 1;
  bool hemisphere = false;   // direct_hemisphere_sample (-H)
  V pt_direct_hemisphere(const Ray<R>& r, const Isect& isect) {              // :47-97
    Frame<R> o2w = hit_coord_space(isect.n);
    const V hit_p = r.o + r.d * isect.t;
    const V w_out = o2w.to_local(-r.d);
    int num_samples = (int)sc.lights.size() * ns_area_light;
    V L_out;
    for (int i = 0; i < num_samples; i++) {
      R pdf;
      V wi, f, wi_world;
      f = bsdf_sample_f(isect.mat, w_out, &wi, &pdf);
      wi_world = o2w.to_world(wi);
      wi_world.normalize();
      Ray<R> ray;
      ray.o = hit_p; ray.d = wi_world; ray.min_t = R(EPS_F); ray.max_t = (R)INFINITY;
      Isect is2;
      if (!intersect(ray, &is2, true)) continue;
      R costhetha = std::fabs(dot(wi_world, isect.n));
      V L_in = get_emission(is2.mat);
      L_out += L_in * f * costhetha / pdf;
    }
    L_out /= R(num_samples);
    return L_out;
  }
  V pt_direct_importance(const Ray<R>& r, const Isect& isect) {              // :99-169
    Frame<R> o2w = hit_coord_space(isect.n);
    const V hit_p = r.o + r.d * isect.t;
    const V w_out = o2w.to_local(-r.d);
    V L_out;
    for (const Light<R>& light : sc.lights) {
      int n_samples = light_is_delta(light) ? 1 : ns_area_light;
      R pdf, distToLight;
      V wi, f, wi_world, emit_radiance, L_o;
      for (int i = 0; i < n_samples; i++) {
        emit_radiance = light_sample_L(light, hit_p, &wi_world, &distToLight, &pdf);
        wi = o2w.to_local(wi_world);
        f = bsdf_f(isect.mat, w_out, wi);
        Ray<R> ray;
        ray.o = hit_p; ray.d = wi_world; ray.min_t = R(EPS_F); ray.max_t = distToLight - R(EPS_F);
        Isect is2;
        if (intersect(ray, &is2, false)) continue;
        R costhetha = std::fabs(dot(wi_world, isect.n));
        V L_in = distToLight >= (R)INFINITY ? emit_radiance : emit_radiance / (distToLight * distToLight);
        L_o += L_in * f * costhetha / pdf;
      }
      L_o /= R(n_samples);
      L_out += L_o;
    }
    return L_out;
  }
  V pt_at_least_one_bounce(const Ray<R>& r, int depth, const Isect& isect) {   // :181-262
    Frame<R> o2w = hit_coord_space(isect.n);
    V hit_p = r.o + r.d * isect.t;
    V w_out = o2w.to_local(-r.d);
    V L_out, L_o;
    if (!is_delta(isect.mat)) L_out += hemisphere ? pt_direct_hemisphere(r, isect) : pt_direct_importance(r, isect);
    bool trace = true, roulette = false;
    R cpdf = R(0.3);
    if (max_depth == 0) {
      roulette = true;
      if (!(pol.uP() < cpdf) || depth >= 20) trace = false;
    } else if (depth >= max_depth - 1) {
      trace = false;
    }
    if (!trace) return L_out;
    V wi, f, wi_world;
    R pdf;
    f = bsdf_sample_f(isect.mat, w_out, &wi, &pdf);
    wi_world = o2w.to_world(wi);
    wi_world.normalize();
    Ray<R> ray;
    ray.o = hit_p; ray.d = wi_world; ray.min_t = R(EPS_F); ray.max_t = (R)INFINITY;
    Isect is2;
    if (!intersect(ray, &is2, true)) return L_out;
    R costhetha = std::fabs(dot(wi_world, isect.n));
    V L_in = pt_at_least_one_bounce(ray, depth + 1, is2);
    if (is_delta(isect.mat)) L_in += get_emission(is2.mat);
    if (roulette) L_o += L_in * f * costhetha / pdf / cpdf;
    else L_o += L_in * f * costhetha / pdf;
    L_out += L_o;
    return L_out;
  }
  V pt_est_radiance(const Ray<R>& r) {                                       // :264-290
    Isect isect;
    V L_out;
    if (!intersect(r, &isect, true)) return sc.env_light >= 0 ? env_radiance<P>(sc.env, r.d) : L_out;
    L_out = get_emission(isect.mat);
    L_out += pt_at_least_one_bounce(r, 0, isect);
    return L_out;
  }
  // One camera sample of pixel (x, y) (:304-316).
  V pt_sample(int x, int y) {
    R px, py, lx, ly;
    grid2d(&px, &py);
    px = px + R(x);
    py = py + R(y);
    R dx = px / R(W), dy = py / R(H);
    grid2d(&lx, &ly);
    return pt_est_radiance(generate_ray_thin_lens(dx, dy, lx, ly));
  }

  void splat(int x, int y, const V& s) {
    size_t k = 3 * ((size_t)x + (size_t)y * W);
    for (int c = 0; c < 3; c++) (*light_buf)[k + c] += (double)s[c];
    if (sample_buf)
      for (int c = 0; c < 3; c++) (*sample_buf)[k + c] += (double)s[c];
  }

  V estimate(int i_eye, int i_light, const std::vector<Vertex>& E, const std::vector<Vertex>& L) {  // :296-469
    Vertex ve, vl, LS, ES;
    int eye_x = -1, eye_y = -1;
    if (i_eye > 1 && E[i_eye].env && i_light >= 1) return V();   // nothing connects to infinity
    ve = E[i_eye];
    vl = L[i_light];
    V c;
    if (i_light == 0) {
      if (i_eye > 1 && E[i_eye].env) {   // an escaped eye ray: the environment's radiance (§9)
        R pp, dp;
        c = env_light_pdf(E[i_eye], &pp, &dp);
      } else if (i_eye > 1) {
        c = get_emission(E[i_eye].isect.mat);
        if (c.norm() > R(EPS_F)) {
          bool hit = false;
          for (size_t j = 0; j < sc.lights.size(); j++) {
            if (sc.lights[j].type != LIGHT_ENV_ORC && light_contain_point(sc.lights[j], E[i_eye].position)) {
              hit = true;
              R pp, dp;
              V wi = E[i_eye].position - E[i_eye - 1].position;
              wi.normalize();
              c = light_sample_pdf(sc.lights[j], E[i_eye].position, wi, &pp, &dp);
              break;
            }
          }
          if (!hit) c = V();
        }
      }
    } else {
      V f_eye, f_light, connect;
      if (i_light == 1) {
        pol.stream(2u + (uint32_t)i_eye);
        int n = (int)sc.lights.size();
        int id = pol.rand_light(n);
        V ldir, lpoint, ln;
        R lpp, ldp, dist;
        V rad = light_sample_Le_point(sc.lights[id], E[i_eye].position, &ldir, &lpoint, &dist, &lpp,
                                      &ldp, &ln);
        lpp /= R(n);
        LS.p = lpp;
        LS.alpha = rad / lpp;
        LS.q = 1.;
        LS.position = lpoint;
        LS.isect.n = ln;
        LS.is_light = true;
        LS.new_sample = true;
        LS.dir_pdf = ldp;
        LS.env = sc.lights[id].type == LIGHT_ENV_ORC;
        f_light = V(1., 1., 1.);
        vl = LS;
        if (LS.env && i_eye == 1) return V();   // no camera connection to infinity (§9)
      }
      if (i_eye == 1) {
        V edir, epoint, en;
        R epp, edp, dist;
        V rad = sample_ray_pdf(vl.position, &edir, &epoint, &dist, &epp, &edp, &en, &eye_x, &eye_y);
        ES.p = epp;
        ES.alpha = rad / epp;
        ES.q = 1.;
        ES.position = epoint;
        ES.isect.n = en;
        ES.is_light = false;
        ES.new_sample = true;
        ES.dir_pdf = edp;
        f_eye = V(1., 1., 1.);
        ve = ES;
      }
      if (i_eye > 1) {
        Frame<R> f = hit_coord_space(E[i_eye].isect.n);
        V er = E[i_eye - 1].position - E[i_eye].position;
        er.normalize();
        er = f.to_local(er);
        if (vl.env) {
          connect = -vl.isect.n;
        } else {
          connect = vl.position - E[i_eye].position;
          connect.normalize();
        }
        connect = f.to_local(connect);
        f_eye = bsdf_f(E[i_eye].isect.mat, er, connect);
      }
      if (i_light > 1) {
        Frame<R> f = hit_coord_space(L[i_light].isect.n);
        V lr = L[i_light - 1].position - L[i_light].position;
        lr.normalize();
        lr = f.to_local(lr);
        connect = ve.position - L[i_light].position;
        connect.normalize();
        connect = f.to_local(connect);
        f_light = bsdf_f(L[i_light].isect.mat, connect, lr);
      }
      R dist;
      if (vl.env) {   // toward the environment, unbounded; G = |cos| at the eye end only (§9)
        connect = -vl.isect.n;
        dist = (R)INFINITY;
      } else {
        connect = vl.position - ve.position;
        dist = connect.norm();
        connect.normalize();
      }
      Ray<R> r;
      r.o = ve.position;
      r.d = connect;
      r.min_t = R(EPS_F);
      r.max_t = dist - R(EPS_F);
      Isect is;
      if (intersect(r, &is, false)) return V();
      R g = vl.env ? std::fabs(dot(ve.isect.n, connect))
                   : std::fabs(dot(vl.isect.n, connect) * dot(ve.isect.n, connect)) / (dist * dist);
      c = f_eye * g * f_light;
    }
    V la = i_light == 1 ? LS.alpha : L[i_light].alpha;
    V ea = i_eye == 1 ? ES.alpha : E[i_eye].alpha;
    R w = 0.;
    V contrib = ea * la * c;
    if (contrib.norm() > R(EPS_F)) w = mis_weight(i_eye, i_light, E, L, LS, ES);
    V ill = contrib * w;
#ifdef ORC_DEBUG2
    fprintf(stderr, "  (%d,%d) c=(%.6g %.6g %.6g) w=%.6g ill=(%.6g %.6g %.6g)\n", i_eye, i_light, (double)c.x,
            (double)c.y, (double)c.z, (double)w, (double)ill.x, (double)ill.y, (double)ill.z);
#endif
#ifdef ORC_DEBUG
    if (!(std::isfinite((double)ill.x))) {
      fprintf(stderr, "NaN ill at i=%d j=%d contrib=(%g %g %g) w=%g c=(%g %g %g) ea=(%g) la=(%g)\n", i_eye, i_light,
              (double)contrib.x, (double)contrib.y, (double)contrib.z, (double)w, (double)c.x, (double)c.y, (double)c.z,
              (double)ea.x, (double)la.x);
      for (size_t k = 0; k < E.size(); k++) fprintf(stderr, " E%zu pos=(%g %g %g) n=(%g %g %g) p=%g a=%g mat=%d\n", k,
        (double)E[k].position.x, (double)E[k].position.y, (double)E[k].position.z, (double)E[k].isect.n.x,
        (double)E[k].isect.n.y, (double)E[k].isect.n.z, (double)E[k].p, (double)E[k].alpha.x, E[k].isect.mat);
      for (size_t k = 0; k < L.size(); k++) fprintf(stderr, " L%zu pos=(%g %g %g) n=(%g %g %g) p=%g a=%g mat=%d\n", k,
        (double)L[k].position.x, (double)L[k].position.y, (double)L[k].position.z, (double)L[k].isect.n.x,
        (double)L[k].isect.n.y, (double)L[k].isect.n.z, (double)L[k].p, (double)L[k].alpha.x, L[k].isect.mat);
    }
#endif
    if (i_eye == 1) {
      if (eye_x >= 0 && eye_y >= 0 && eye_x < W && eye_y < H) splat(eye_x, eye_y, ill / R(ns_aa));
      return V();
    }
    return ill;
  }

  V est_radiance(const Ray<R>& r) {                                           // :472-500
    V L_out;
    std::vector<Vertex> E, L;
    E.reserve(max_depth + 2);
    L.reserve(max_depth + 2);
    prepare_subpath(r, 1., 1., E, V(1., 1., 1.), r.d, false);
    R lpp, ldp;
    V lrad, ln;
    pol.stream(1);
    Ray<R> lr = sample_light_ray(lpp, ldp, lrad, ln);
    prepare_subpath(lr, lpp, ldp, L, lrad, ln, true);
#ifdef ORC_DEBUG2
    for (size_t k = 0; k < E.size(); k++) fprintf(stderr, " E%zu pos=(%.8g %.8g %.8g) n=(%.6g %.6g %.6g) p=%.6g a=%.6g mat=%d\n", k,
        (double)E[k].position.x, (double)E[k].position.y, (double)E[k].position.z, (double)E[k].isect.n.x,
        (double)E[k].isect.n.y, (double)E[k].isect.n.z, (double)E[k].p, (double)E[k].alpha.x, E[k].isect.mat);
    for (size_t k = 0; k < L.size(); k++) fprintf(stderr, " L%zu pos=(%.8g %.8g %.8g) n=(%.6g %.6g %.6g) p=%.6g a=%.6g mat=%d\n", k,
        (double)L[k].position.x, (double)L[k].position.y, (double)L[k].position.z, (double)L[k].isect.n.x,
        (double)L[k].isect.n.y, (double)L[k].isect.n.z, (double)L[k].p, (double)L[k].alpha.x, L[k].isect.mat);
#endif
    for (int i = 1; i < (int)E.size(); i++)
      for (int j = 0; j < (int)L.size(); j++) L_out += estimate(i, j, E, L);
    return L_out;
  }

  // One sample of pixel (x,y) (bidirection.cpp:515-533).
  V one_sample(int x, int y) {
    R px, py;
    grid2d(&px, &py);
    px = px + R(x);
    py = py + R(y);
    R dx = px / R(W), dy = py / R(H);
    Ray<R> ray = generate_ray(dx, dy);
    return est_radiance(ray);
  }
};

// ----------------------------------------------------------------------------------------------
template <class R>
static int render_counter(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, uint64_t seed,
                          int s0, int sc_count, int nthreads, double* eye, double* light, double* stats,
                          int rr) {
  Scene<R> sc;
  std::string err;
  int rc = load_scene<R>(d, sc, err);
  if (rc) { fprintf(stderr, "oracle: %s\n", err.c_str()); return rc; }
  if (nthreads < 1) nthreads = 1;
  std::vector<std::vector<double>> lbuf(nthreads, std::vector<double>((size_t)W * H * 3, 0.0));
  std::vector<Stats> sts(nthreads);
  auto work = [&](int t) {
    for (int y = t; y < H; y += nthreads) {
      for (int x = 0; x < W; x++) {
        double acc[3] = {0, 0, 0};
        for (int s = s0; s < s0 + sc_count; s++) {
          CounterStream cs;
          cs.init(seed, (uint32_t)(x + y * W), (uint32_t)s);
          typedef typename std::conditional<sizeof(R) == 8, PolicyC64, PolicyC32>::type P;
          P pol;
          pol.cs = &cs;
          Tracer<P> tr(sc, pol, max_depth, W, H, spp);
          tr.rr = rr != 0;
          tr.light_buf = &lbuf[t];
          V3<R> ill = tr.one_sample(x, y);
          R inv = R(1.) / R(spp);
          for (int c = 0; c < 3; c++) acc[c] += (double)(ill[c] * inv);
          Stats& S = sts[t];
          S.rays += tr.st.rays; S.closest += tr.st.closest; S.shadow += tr.st.shadow;
          S.nodes += tr.st.nodes; S.tri += tr.st.tri; S.sph += tr.st.sph; S.hits += tr.st.hits;
        }
        size_t k = 3 * ((size_t)x + (size_t)y * W);
        for (int c = 0; c < 3; c++) eye[k + c] += acc[c];
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; t++) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  for (int t = 0; t < nthreads; t++)
    for (size_t k = 0; k < (size_t)W * H * 3; k++) light[k] += lbuf[t][k];
  if (stats) {
    Stats S;
    for (auto& s : sts) {
      S.rays += s.rays; S.closest += s.closest; S.shadow += s.shadow; S.nodes += s.nodes;
      S.tri += s.tri; S.sph += s.sph; S.hits += s.hits;
    }
    stats[0] = (double)S.rays; stats[1] = (double)S.closest; stats[2] = (double)S.shadow;
    stats[3] = (double)S.nodes; stats[4] = (double)S.tri; stats[5] = (double)S.sph;
    stats[6] = (double)S.hits; stats[7] = (double)sc.nodes.size();
  }
  return 0;
}

template <class P>
static int env_kat(const bdpt_scene_desc* d, int n, const double* u, double* wi, double* pdf, double* rad) {
  typedef typename P::R R;
  Scene<R> sc;
  std::string err;
  if (!d || !d->envmap || load_scene<R>(d, sc, err)) return BDPT_E_INVALID;
  for (int k = 0; k < n; k++) {
    V3<R> w;
    R p;
    V3<R> L = env_sample_dir<P>(sc.env, (R)u[4 * k], (R)u[4 * k + 1], (R)u[4 * k + 2], (R)u[4 * k + 3], &w, &p);
    for (int c = 0; c < 3; c++) { wi[3 * k + c] = w[c]; rad[3 * k + c] = L[c]; }
    pdf[k] = p;
  }
  return 0;
}
template <class P>
static int env_lookup(const bdpt_scene_desc* d, int n, const double* dirs, double* rad, double* pdf) {
  typedef typename P::R R;
  Scene<R> sc;
  std::string err;
  if (!d || !d->envmap || load_scene<R>(d, sc, err)) return BDPT_E_INVALID;
  for (int k = 0; k < n; k++) {
    V3<R> w((R)dirs[3 * k], (R)dirs[3 * k + 1], (R)dirs[3 * k + 2]);
    V3<R> L = env_radiance<P>(sc.env, w);
    for (int c = 0; c < 3; c++) rad[3 * k + c] = L[c];
    pdf[k] = env_pdf_dir<P>(sc.env, w);
  }
  return 0;
}
// PathTracer::raytrace_pixel (pathtracer.cpp:292-338): adaptive batches of camera samples.
struct PtSettings {
  int ns_area_light, batch, hemisphere;
  float tol;
  double lens_radius, focal_distance;
};
template <class P>
static void pt_pixel(Tracer<P>& tr, int x, int y, int ns_aa, const PtSettings& ps, CounterStream* cs,
                     uint64_t seed, double* out, int* count) {
  typedef typename P::R R;
  int num_samples = 0;
  V3<R> illumination(0, 0, 0);
  R s1 = 0, s2 = 0;
  for (int i = 0; i < ns_aa; i = i + ps.batch) {
    for (int j = 0; j < ps.batch; j++) {
      if (cs) cs->init(seed, (uint32_t)(x + y * tr.W), (uint32_t)(i + j));
      V3<R> ill = tr.pt_sample(x, y);
      illumination += ill;
      R il;
      if (sizeof(R) == 8) il = (float)(0.2126f * ill.x + 0.7152f * ill.y + 0.0722f * ill.z);   // illum() is float
      else il = R(0.2126f) * ill.x + R(0.7152f) * ill.y + R(0.0722f) * ill.z;
      s1 += il;
      s2 += il * il;
    }
    num_samples = i + ps.batch;
    R mu = s1 / R(num_samples);
    R sigma = std::sqrt((s2 - s1 * s1 / R(num_samples)) / R(num_samples - 1));
    R ci = R(1.96) * sigma / std::sqrt(R(num_samples));
    if (ci <= R((double)ps.tol) * mu && mu > R(EPS_F)) break;
  }
  illumination /= R(num_samples);
  for (int c = 0; c < 3; c++) out[c] = (double)illumination[c];
  *count = num_samples;
}

template <class R>
static int pt_render_counter(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, uint64_t seed,
                             const PtSettings& ps, int nthreads, double* image, int* counts, double* stats) {
  Scene<R> sc;
  std::string err;
  int rc = load_scene<R>(d, sc, err, true);
  if (rc) { fprintf(stderr, "oracle: %s\n", err.c_str()); return rc; }
  if (nthreads < 1) nthreads = 1;
  std::vector<Stats> sts(nthreads);
  typedef typename std::conditional<sizeof(R) == 8, PolicyC64, PolicyC32>::type P;
  auto work = [&](int t) {
    CounterStream cs;
    cs.init(seed, 0, 0);
    P pol;
    pol.cs = &cs;
    Tracer<P> tr(sc, pol, max_depth, W, H, spp);
    tr.ns_area_light = ps.ns_area_light;
    tr.hemisphere = ps.hemisphere != 0;
    tr.lens_radius = (R)ps.lens_radius;
    tr.focal_distance = (R)ps.focal_distance;
    for (int y = t; y < H; y += nthreads)
      for (int x = 0; x < W; x++) {
        size_t k = (size_t)x + (size_t)y * W;
        pt_pixel(tr, x, y, spp, ps, &cs, seed, image + 3 * k, counts + k);
      }
    sts[t] = tr.st;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nthreads; t++) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  if (stats) {
    Stats S;
    for (auto& q : sts) {
      S.rays += q.rays; S.closest += q.closest; S.shadow += q.shadow; S.nodes += q.nodes;
      S.tri += q.tri; S.sph += q.sph; S.hits += q.hits;
    }
    stats[0] = (double)S.rays; stats[1] = (double)S.closest; stats[2] = (double)S.shadow;
    stats[3] = (double)S.nodes; stats[4] = (double)S.tri; stats[5] = (double)S.sph;
    stats[6] = (double)S.hits; stats[7] = (double)sc.nodes.size();
  }
  return 0;
}

}  // namespace orc

using namespace orc;

extern "C" {

// mode 0: the reference's own sequence (tiles of 32 in raster order, pixels row-major inside a
// tile, ns_aa samples per pixel; raytraced_renderer.cpp:297-301,610-615); writes eye, light and the
// reference-ordered sample buffer (all fp64). modes 1/2: counter RNG, samples [s0, s0+count).
// rr: Russian roulette (counter modes only, the reference cannot run it; nor an
// environment light under BDPT, which mode 0 therefore rejects).
int oracle_render_ex(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, int mode,
                     uint64_t seed, int s0, int count, int nthreads, double* eye, double* light,
                     double* sample, double* stats, int rr) {
  if (!d || W <= 0 || H <= 0 || spp <= 0 || max_depth < 0) return BDPT_E_INVALID;
  if (mode == 1) return render_counter<double>(d, W, H, spp, max_depth, seed, s0, count, nthreads, eye, light, stats, rr);
  if (mode == 2) return render_counter<float>(d, W, H, spp, max_depth, seed, s0, count, nthreads, eye, light, stats, rr);
  if (mode != 0) return BDPT_E_INVALID;
  if (rr || d->envmap) return BDPT_E_UNSUPPORTED;
  Scene<double> sc;
  std::string err;
  int rc = load_scene<double>(d, sc, err);
  if (rc) { fprintf(stderr, "oracle: %s\n", err.c_str()); return rc; }
  RefStreams rs;                 // fresh engines: the reference's static engines at process start
  std::srand(1);
  PolicyRef pol;
  pol.rs = &rs;
  Tracer<PolicyRef> tr(sc, pol, max_depth, W, H, spp);
  std::vector<double> lb((size_t)W * H * 3, 0.0), sb((size_t)W * H * 3, 0.0);
  tr.light_buf = &lb;
  tr.sample_buf = &sb;
  const int TS = 32;
  for (int ty = 0; ty < H; ty += TS)
    for (int tx = 0; tx < W; tx += TS)
      for (int y = ty; y < std::min(ty + TS, H); y++)
        for (int x = tx; x < std::min(tx + TS, W); x++) {
          V3<double> illum(0, 0, 0);                                           // :514-541
          for (int s = 0; s < spp; s++) illum += tr.one_sample(x, y);
          illum /= (double)spp;
          size_t k = 3 * ((size_t)x + (size_t)y * W);
          for (int c = 0; c < 3; c++) { eye[k + c] = illum[c]; sb[k + c] += illum[c]; }
        }
  memcpy(light, lb.data(), lb.size() * sizeof(double));
  if (sample) memcpy(sample, sb.data(), sb.size() * sizeof(double));
  if (stats) {
    stats[0] = (double)tr.st.rays; stats[1] = (double)tr.st.closest; stats[2] = (double)tr.st.shadow;
    stats[3] = (double)tr.st.nodes; stats[4] = (double)tr.st.tri; stats[5] = (double)tr.st.sph;
    stats[6] = (double)tr.st.hits; stats[7] = (double)sc.nodes.size();
  }
  return 0;
}

int oracle_render(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, int mode,
                  uint64_t seed, int s0, int count, int nthreads, double* eye, double* light,
                  double* sample, double* stats) {
  return oracle_render_ex(d, W, H, spp, max_depth, mode, seed, s0, count, nthreads, eye, light, sample, stats, 0);
}

// Environment-light known answers (tests/test_env.py): the fp64 tables of EnvironmentLight::init
// (marg[h], cond[w*h], pdf[w*h]); sample_L from explicit uniforms (u = ux, uy, jx, jy) -> wi[3],
// pdf, radiance[3]; sample_dir / the direction pdf for n directions -> rad[3n], pdf[n]. mode 1:
// the reference's fp64 libm formulas; mode 2: the device's fp32 semantics.
int oracle_env_tables(const bdpt_scene_desc* d, double* marg, double* cond, double* pdf) {
  Scene<double> sc;
  std::string err;
  if (!d || !d->envmap || load_scene<double>(d, sc, err)) return BDPT_E_INVALID;
  const size_t np = (size_t)sc.env.w * sc.env.h;
  memcpy(marg, sc.env.marg.data(), sc.env.h * sizeof(double));
  memcpy(cond, sc.env.cond.data(), np * sizeof(double));
  memcpy(pdf, sc.env.pdf.data(), np * sizeof(double));
  return 0;
}
int oracle_env_sample(const bdpt_scene_desc* d, int mode, int n, const double* u, double* wi, double* pdf,
                      double* rad) {
  if (mode == 2) return env_kat<PolicyC32>(d, n, u, wi, pdf, rad);
  return env_kat<PolicyC64>(d, n, u, wi, pdf, rad);
}
int oracle_env_lookup(const bdpt_scene_desc* d, int mode, int n, const double* dirs, double* rad, double* pdf) {
  if (mode == 2) return env_lookup<PolicyC32>(d, n, dirs, rad, pdf);
  return env_lookup<PolicyC64>(d, n, dirs, rad, pdf);
}

// The unidirectional PathTracer (pathtracer.cpp:47-340). mode 0: the
// reference's own sequence (its four TU-static engines, tiles of 32 in raster order, -t 1); modes
// 1/2: counter RNG keyed by (pixel, sample index within the pixel). image: W*H*3 (row 0 = bottom)
// = sampleBuffer, counts: W*H = sampleCountBuffer.
int oracle_pt_render(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, int mode, uint64_t seed,
                     int ns_area_light, int samples_per_batch, float max_tolerance, int hemisphere,
                     double lens_radius, double focal_distance, int nthreads, double* image, int* counts,
                     double* stats) {
  if (!d || W <= 0 || H <= 0 || spp <= 0 || max_depth < 0 || samples_per_batch <= 0 || ns_area_light <= 0)
    return BDPT_E_INVALID;
  PtSettings ps{ns_area_light, samples_per_batch, hemisphere, max_tolerance, lens_radius, focal_distance};
  if (mode == 1) return pt_render_counter<double>(d, W, H, spp, max_depth, seed, ps, nthreads, image, counts, stats);
  if (mode == 2) return pt_render_counter<float>(d, W, H, spp, max_depth, seed, ps, nthreads, image, counts, stats);
  if (mode != 0) return BDPT_E_INVALID;
  Scene<double> sc;
  std::string err;
  int rc = load_scene<double>(d, sc, err, true);
  if (rc) { fprintf(stderr, "oracle: %s\n", err.c_str()); return rc; }
  RefStreams rs;
  std::srand(1);
  PolicyRef pol;
  pol.rs = &rs;
  Tracer<PolicyRef> tr(sc, pol, max_depth, W, H, spp);
  tr.ns_area_light = ns_area_light;
  tr.hemisphere = hemisphere != 0;
  tr.lens_radius = lens_radius;
  tr.focal_distance = focal_distance;
  const int TS = 32;
  for (int ty = 0; ty < H; ty += TS)
    for (int tx = 0; tx < W; tx += TS)
      for (int y = ty; y < std::min(ty + TS, H); y++)
        for (int x = tx; x < std::min(tx + TS, W); x++) {
          size_t k = (size_t)x + (size_t)y * W;
          pt_pixel(tr, x, y, spp, ps, nullptr, seed, image + 3 * k, counts + k);
        }
  if (stats) {
    stats[0] = (double)tr.st.rays; stats[1] = (double)tr.st.closest; stats[2] = (double)tr.st.shadow;
    stats[3] = (double)tr.st.nodes; stats[4] = (double)tr.st.tri; stats[5] = (double)tr.st.sph;
    stats[6] = (double)tr.st.hits; stats[7] = (double)sc.nodes.size();
  }
  return 0;
}

// BVH facts of the oracle's reference build: nodes, depth, DFS leaf order (prim indices).
int oracle_bvh_info(const bdpt_scene_desc* d, int* nodes, int* depth, int* leaf_order) {
  Scene<double> sc;
  std::string err;
  int rc = load_scene<double>(d, sc, err);
  if (rc) return rc;
  *nodes = (int)sc.nodes.size();
  *depth = sc.depth;
  if (leaf_order)
    for (size_t i = 0; i < sc.leaf_prims.size(); i++) leaf_order[i] = sc.leaf_prims[i];
  return 0;
}

// Closest-hit / any-hit queries (mode 1: fp64 boxes; mode 2: fp32 conservative boxes).
int oracle_trace_rays(const bdpt_scene_desc* d, int mode, const float* rays, int n, int any_hit,
                      float* out_t, int* out_prim) {
  if (mode == 2) {
    Scene<float> sc;
    std::string err;
    if (load_scene<float>(d, sc, err)) return BDPT_E_INVALID;
    CounterStream cs;
    cs.init(0, 0, 0);
    PolicyC32 pol;
    pol.cs = &cs;
    Tracer<PolicyC32> tr(sc, pol, 1, 1, 1, 1);
    for (int i = 0; i < n; i++) {
      const float* r = rays + 8 * (size_t)i;
      Ray<float> ray;
      ray.o = V3<float>(r[0], r[1], r[2]);
      ray.d = V3<float>(r[3], r[4], r[5]);
      ray.min_t = r[6];
      ray.max_t = r[7];
      Tracer<PolicyC32>::Isect is;
      bool h = tr.intersect(ray, &is, !any_hit);
      out_t[i] = h ? (any_hit ? 0.0f : is.t) : INFINITY;
      out_prim[i] = h ? (any_hit ? 0 : is.prim) : -1;
    }
    return 0;
  }
  Scene<double> sc;
  std::string err;
  if (load_scene<double>(d, sc, err)) return BDPT_E_INVALID;
  CounterStream cs;
  cs.init(0, 0, 0);
  PolicyC64 pol;
  pol.cs = &cs;
  Tracer<PolicyC64> tr(sc, pol, 1, 1, 1, 1);
  for (int i = 0; i < n; i++) {
    const float* r = rays + 8 * (size_t)i;
    Ray<double> ray;
    ray.o = V3<double>(r[0], r[1], r[2]);
    ray.d = V3<double>(r[3], r[4], r[5]);
    ray.min_t = r[6];
    ray.max_t = r[7];
    Tracer<PolicyC64>::Isect is;
    bool h = tr.intersect(ray, &is, !any_hit);
    out_t[i] = h ? (any_hit ? 0.0f : (float)is.t) : INFINITY;
    out_prim[i] = h ? (any_hit ? 0 : is.prim) : -1;
  }
  return 0;
}

// One sample's eye-image contribution (debug / per-sample parity); splats go to light_out (W*H*3).
int oracle_sample(const bdpt_scene_desc* d, int W, int H, int spp, int max_depth, int mode,
                  uint64_t seed, int x, int y, int s, double* eye_out, double* light_out) {
  if (mode != 1 && mode != 2) return BDPT_E_INVALID;
  std::vector<double> lb((size_t)W * H * 3, 0.0);
  if (mode == 1) {
    Scene<double> sc; std::string err;
    if (load_scene<double>(d, sc, err)) return BDPT_E_INVALID;
    CounterStream cs; cs.init(seed, (uint32_t)(x + y * W), (uint32_t)s);
    PolicyC64 pol; pol.cs = &cs;
    Tracer<PolicyC64> tr(sc, pol, max_depth, W, H, spp);
    tr.light_buf = &lb;
    V3<double> v = tr.one_sample(x, y);
    for (int c = 0; c < 3; c++) eye_out[c] = v[c];
  } else {
    Scene<float> sc; std::string err;
    if (load_scene<float>(d, sc, err)) return BDPT_E_INVALID;
    CounterStream cs; cs.init(seed, (uint32_t)(x + y * W), (uint32_t)s);
    PolicyC32 pol; pol.cs = &cs;
    Tracer<PolicyC32> tr(sc, pol, max_depth, W, H, spp);
    tr.light_buf = &lb;
    V3<float> v = tr.one_sample(x, y);
    for (int c = 0; c < 3; c++) eye_out[c] = v[c];
  }
  if (light_out) memcpy(light_out, lb.data(), lb.size() * sizeof(double));
  return 0;
}

// Known-answer helpers for the RNG and the deterministic transcendentals.
void oracle_philox(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t block, uint32_t out[4]) {
  out[0] = pixel; out[1] = sample; out[2] = block; out[3] = 0xB1D1u;
  philox4x32_10(out, (uint32_t)seed, (uint32_t)(seed >> 32));
}
void oracle_cos_sin_2pi(float u, float* c, float* s) { cos_sin_2pi_f32(u, c, s); }
double oracle_mt_first(int n, double* out) {   // first n U of a fresh reference engine
  RefStreams rs;
  for (int i = 0; i < n; i++) out[i] = rs.uS();
  return n > 0 ? out[0] : 0.0;
}

}  // extern "C"
