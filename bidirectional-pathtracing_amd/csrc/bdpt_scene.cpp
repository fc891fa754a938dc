// bdpt_scene.cpp — host-side scene preparation (see bdpt_scene.h).
#include "bdpt_scene.h"

#include <algorithm>
#include <array>
#include <functional>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>

namespace bdpt {

namespace {

struct Box {  // BBox (bbox.h:19-136), fp64
  double mn[3], mx[3];
  void from_point(const double* p) {
    for (int k = 0; k < 3; k++) mn[k] = mx[k] = p[k];
  }
  void expand(const Box& b) {
    for (int k = 0; k < 3; k++) {
      mn[k] = std::min(mn[k], b.mn[k]);
      mx[k] = std::max(mx[k], b.mx[k]);
    }
  }
  void expand_pt(const double* p) {
    for (int k = 0; k < 3; k++) {
      mn[k] = std::min(mn[k], p[k]);
      mx[k] = std::max(mx[k], p[k]);
    }
  }
  double centroid(int k) const { return 0.5 * (mn[k] + mx[k]); }   // (min + max) / 2
};

struct Node {
  int l = -1, r = -1;
  int start = 0, count = 0;
  Box box;
};

struct Builder {
  const std::vector<Box>* pb;
  std::vector<Node> nodes;
  std::vector<int> leaf_prims;
  int depth = 0;

  int make_leaf(const std::vector<int>& prims) {
    Node n;
    n.box = (*pb)[prims[0]];
    for (int p : prims) n.box.expand((*pb)[p]);
    n.start = (int)leaf_prims.size();
    n.count = (int)prims.size();
    for (int p : prims) leaf_prims.push_back(p);
    nodes.push_back(n);
    return (int)nodes.size() - 1;
  }

  // construct_bvh (bvh.cpp:51-129). Where the reference asserts (no extent / empty side) the
  // list is split in half in input order instead (documented divergence: the reference aborts).
  int build(const std::vector<int>& prims, int d) {
    depth = std::max(depth, d);
    const auto& B = *pb;
    if (prims.size() <= 4) return make_leaf(prims);
    double xmax = 0, xmin = 0, ymax = 0, ymin = 0, zmax = 0, zmin = 0;
    for (size_t i = 0; i < prims.size(); i++) {
      const Box& b = B[prims[i]];
      double cx = b.centroid(0), cy = b.centroid(1), cz = b.centroid(2);
      xmax = i == 0 ? cx : std::max(xmax, cx);
      xmin = i == 0 ? cx : std::min(xmin, cx);
      ymax = i == 0 ? cy : std::max(ymax, cy);
      ymin = i == 0 ? cy : std::min(ymin, cy);
      zmax = i == 0 ? cz : std::max(zmax, cz);
      zmin = i == 0 ? cz : std::min(zmin, cz);
    }
    double ranges[3] = {xmax - xmin, ymax - ymin, zmax - zmin};
    double mins[3] = {xmin, ymin, zmin};
    double max_range = std::max(ranges[0], std::max(ranges[1], ranges[2]));
    int axis;
    for (axis = 0; axis < 3; axis++)
      if (ranges[axis] == max_range) break;
    std::vector<int> left, right;
    if (max_range > 0 && axis < 3) {
      double mid = mins[axis] + ranges[axis] / 2;
      for (int p : prims) {
        if (B[p].centroid(axis) <= mid) left.push_back(p);
        else right.push_back(p);
      }
    }
    if (left.empty() || right.empty()) {
      left.assign(prims.begin(), prims.begin() + prims.size() / 2);
      right.assign(prims.begin() + prims.size() / 2, prims.end());
    }
    int id = (int)nodes.size();
    nodes.push_back(Node());
    int l = build(left, d + 1);
    int r = build(right, d + 1);
    Box bb = nodes[l].box;
    bb.expand(nodes[r].box);
    nodes[id].l = l;
    nodes[id].r = r;
    nodes[id].box = bb;
    return id;
  }
};

// Device tree: binned SAH (16 bins per axis on centroid bounds, leaves of <= 2 primitives with SAH
// termination; the leaf encoding allows up to 4), optionally with spatial splits (SBVH, Stich et
// al. 2009: a triangle straddling a split plane is referenced from both sides, each side bounding
// only its clipped part). Which tree the device traverses does not change any result: closest
// hits are decided by t, ties by the primitive's position in the REFERENCE tree's DFS leaf order
// (the reference keeps the last of equal-t hits, bvh.cpp:161-188; a primitive referenced twice
// gives the same t and key both times), and any-hit is order free.
struct SahBuilder {
  struct Ref {
    int prim;
    Box box;   // the part of the primitive this reference bounds (its whole box unless clipped)
  };
  const std::vector<Box>* pb;
  const bdpt_scene_desc* desc = nullptr;   // triangle vertices for the spatial-split clipping
  std::vector<Node> nodes;
  std::vector<int> leaf_prims;
  int depth = 0;
  // Leaves: split until a node holds <= leaf_max primitives; with ct > 0 (SAH termination) such a
  // node stays a leaf only when n <= ct + (A_l n_l + A_r n_r) / A (traversal cost ct, unit test
  // cost). Measured (Msamples/s, leaf_max 4 / ct 0 -> leaf_max 2 / ct 1): Lucy stand-in 1080p
  // 532 -> 579, CBgems 311 -> 381, CBbunny 800x600 393 -> 428; triangle tests per Lucy sample
  // 63.3 -> 26.2 (large wall triangles no longer share leaves with the mesh).
  int leaf_max = 2;
  double ct = 1.0;
  int nb = 16;          // centroid bins per axis (<= kMaxBins)
  static constexpr int kMaxBins = 64;
  // spatial splits: tried at a node when its best object split's children overlap by more than
  // alpha x the root's area; at most budget x n references in all (0 = off)
  double alpha = 0;
  double budget = 0;
  int nsb = 32;         // spatial bins per axis (<= kMaxBins)
  size_t max_refs = 0, nrefs = 0;
  double root_area = 0;
  static double area(const Box& b) {
    const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return dx < 0 ? 0 : 2 * (dx * dy + dy * dz + dz * dx);
  }
  static Box empty_box() {
    Box b;
    for (int k = 0; k < 3; k++) { b.mn[k] = INFINITY; b.mx[k] = -INFINITY; }
    return b;
  }
  static Box intersect(const Box& a, const Box& b) {
    Box r;
    for (int k = 0; k < 3; k++) { r.mn[k] = std::max(a.mn[k], b.mn[k]); r.mx[k] = std::min(a.mx[k], b.mx[k]); }
    return r;
  }
  static bool valid(const Box& b) { return b.mn[0] <= b.mx[0] && b.mn[1] <= b.mx[1] && b.mn[2] <= b.mx[2]; }
  // the box of the part of reference r within [lo, hi] along axis ax: a triangle is clipped as a
  // polygon (its vertices inside the slab and its edges' crossings of the two planes), anything
  // else by its box; the result is also within r's own box (earlier clips)
  Box clip(const Ref& r, int ax, double lo, double hi) const {
    Box b = empty_box();
    if (desc->prim_type[r.prim] == BDPT_PRIM_TRIANGLE) {
      const double* g = desc->prim_geom + 18 * (size_t)r.prim;
      for (int e = 0; e < 3; e++) {
        const double* a = g + 3 * e;
        const double* c = g + 3 * ((e + 1) % 3);
        if (a[ax] >= lo && a[ax] <= hi) b.expand_pt(a);
        for (double pl : {lo, hi}) {
          if ((a[ax] < pl && c[ax] > pl) || (a[ax] > pl && c[ax] < pl)) {
            const double t = (pl - a[ax]) / (c[ax] - a[ax]);
            double q[3];
            for (int k = 0; k < 3; k++) q[k] = a[k] + t * (c[k] - a[k]);
            q[ax] = pl;
            b.expand_pt(q);
          }
        }
      }
    } else {
      b = (*pb)[r.prim];
    }
    Box slab = r.box;
    slab.mn[ax] = std::max(slab.mn[ax], lo);
    slab.mx[ax] = std::min(slab.mx[ax], hi);
    return intersect(b, slab);
  }
  int make_leaf(const Ref* refs, int n) {
    Node nd;
    nd.box = refs[0].box;
    for (int k = 0; k < n; k++) nd.box.expand(refs[k].box);
    nd.start = (int)leaf_prims.size();
    nd.count = n;
    for (int k = 0; k < n; k++) leaf_prims.push_back(refs[k].prim);
    nodes.push_back(nd);
    return (int)nodes.size() - 1;
  }
  int build_root(int n) {
    std::vector<Ref> refs(n);
    for (int i = 0; i < n; i++) refs[i] = Ref{i, (*pb)[i]};
    Box all = refs[0].box;
    for (int i = 1; i < n; i++) all.expand(refs[i].box);
    root_area = area(all);
    nrefs = (size_t)n;
    max_refs = (size_t)((double)n * (1.0 + std::max(0.0, budget)));
    return build(refs, 0);
  }
  int build(std::vector<Ref>& refs, int d) {
    depth = std::max(depth, d);
    const int n = (int)refs.size();
    if (n <= 1 || (n <= leaf_max && ct <= 0)) return make_leaf(refs.data(), n);
    Box cb = empty_box();
    for (int i = 0; i < n; i++) {
      double c[3] = {refs[i].box.centroid(0), refs[i].box.centroid(1), refs[i].box.centroid(2)};
      cb.expand_pt(c);
    }
    const int NB = nb;
    double best = INFINITY;
    int best_axis = -1, best_split = 0;
    Box best_l, best_r;
    for (int ax = 0; ax < 3; ax++) {
      const double lo = cb.mn[ax], ext = cb.mx[ax] - cb.mn[ax];
      if (!(ext > 0)) continue;
      Box bb[kMaxBins];
      int cnt[kMaxBins] = {0};
      for (int b = 0; b < NB; b++) bb[b] = empty_box();
      for (int i = 0; i < n; i++) {
        int b = (int)((refs[i].box.centroid(ax) - lo) / ext * NB);
        b = std::min(NB - 1, std::max(0, b));
        cnt[b]++;
        bb[b].expand(refs[i].box);
      }
      double ra[kMaxBins];
      int rc[kMaxBins];
      Box rb[kMaxBins];
      Box acc = empty_box();
      int c = 0;
      for (int b = NB - 1; b > 0; b--) {
        acc.expand(bb[b]);
        c += cnt[b];
        ra[b] = area(acc);
        rc[b] = c;
        rb[b] = acc;
      }
      acc = empty_box();
      c = 0;
      for (int b = 0; b < NB - 1; b++) {
        acc.expand(bb[b]);
        c += cnt[b];
        if (c == 0 || rc[b + 1] == 0) continue;
        const double cost = area(acc) * c + ra[b + 1] * rc[b + 1];
        if (cost < best) { best = cost; best_axis = ax; best_split = b + 1; best_l = acc; best_r = rb[b + 1]; }
      }
    }
    if (n <= leaf_max && ct > 0) {
      Box nb_ = refs[0].box;
      for (int i = 1; i < n; i++) nb_.expand(refs[i].box);
      const double an = area(nb_);
      if (best_axis < 0 || !(an > 0) || (double)n <= ct + best / an) return make_leaf(refs.data(), n);
    }
    // spatial split: only where the object split's children overlap and the reference budget lasts
    int sp_axis = -1;
    double sp_pos = 0;
    if (alpha > 0 && n > leaf_max && nrefs < max_refs && best_axis >= 0) {
      const Box ov = intersect(best_l, best_r);
      if (valid(ov) && area(ov) > alpha * root_area) {
        Box nbx = refs[0].box;
        for (int i = 1; i < n; i++) nbx.expand(refs[i].box);
        const int SB = nsb;
        double sbest = best;
        for (int ax = 0; ax < 3; ax++) {
          const double lo = nbx.mn[ax], ext = nbx.mx[ax] - nbx.mn[ax];
          if (!(ext > 0)) continue;
          Box bb[kMaxBins];
          int ent[kMaxBins] = {0}, ex[kMaxBins] = {0};
          for (int b = 0; b < SB; b++) bb[b] = empty_box();
          auto bin_of = [&](double v) { return std::min(SB - 1, std::max(0, (int)((v - lo) / ext * SB))); };
          for (int i = 0; i < n; i++) {
            const int b0 = bin_of(refs[i].box.mn[ax]), b1 = bin_of(refs[i].box.mx[ax]);
            ent[b0]++;
            ex[b1]++;
            for (int b = b0; b <= b1; b++) {
              const Box cbx = b0 == b1 ? refs[i].box
                                       : clip(refs[i], ax, lo + ext * b / SB, b + 1 == SB ? nbx.mx[ax] : lo + ext * (b + 1) / SB);
              if (valid(cbx)) bb[b].expand(cbx);
            }
          }
          double ra[kMaxBins];
          int rc[kMaxBins];
          Box acc = empty_box();
          int c = 0;
          for (int b = SB - 1; b > 0; b--) {
            acc.expand(bb[b]);
            c += ex[b];
            ra[b] = area(acc);
            rc[b] = c;
          }
          acc = empty_box();
          c = 0;
          for (int b = 0; b < SB - 1; b++) {
            acc.expand(bb[b]);
            c += ent[b];
            if (c == 0 || rc[b + 1] == 0) continue;
            const double cost = area(acc) * c + ra[b + 1] * rc[b + 1];
            if (cost < sbest) { sbest = cost; sp_axis = ax; sp_pos = lo + ext * (b + 1) / SB; }
          }
        }
      }
    }
    std::vector<Ref> left, right;
    if (sp_axis >= 0) {
      for (const Ref& r : refs) {
        if (r.box.mx[sp_axis] <= sp_pos) { left.push_back(r); continue; }
        if (r.box.mn[sp_axis] >= sp_pos) { right.push_back(r); continue; }
        const Box lb = clip(r, sp_axis, -INFINITY, sp_pos), rbx = clip(r, sp_axis, sp_pos, INFINITY);
        const bool lv = valid(lb), rv = valid(rbx);
        if (lv) left.push_back(Ref{r.prim, lb});
        if (rv) right.push_back(Ref{r.prim, rbx});
        if (!lv && !rv) left.push_back(r);   // degenerate clip: keep the reference whole
        if (lv && rv) nrefs++;
      }
      if (left.empty() || right.empty()) {   // nothing gained: fall back to the object split
        nrefs -= left.size() + right.size() - refs.size();
        left.clear();
        right.clear();
        sp_axis = -1;
      }
    }
    if (sp_axis < 0) {
      int nl;
      if (best_axis < 0) {
        nl = n / 2;   // coincident centroids: split in input order
      } else {
        const double lo = cb.mn[best_axis], ext = cb.mx[best_axis] - cb.mn[best_axis];
        auto mid = std::stable_partition(refs.begin(), refs.end(), [&](const Ref& r) {
          int b = (int)((r.box.centroid(best_axis) - lo) / ext * NB);
          return std::min(NB - 1, std::max(0, b)) < best_split;
        });
        nl = (int)(mid - refs.begin());
        if (nl == 0 || nl == n) nl = n / 2;
      }
      left.assign(refs.begin(), refs.begin() + nl);
      right.assign(refs.begin() + nl, refs.end());
    }
    std::vector<Ref>().swap(refs);
    const int id = (int)nodes.size();
    nodes.push_back(Node());
    const int l = build(left, d + 1);
    const int r = build(right, d + 1);
    Box bb = nodes[l].box;
    bb.expand(nodes[r].box);
    nodes[id].l = l;
    nodes[id].r = r;
    nodes[id].box = bb;
    return id;
  }
};

float pad_down(double v, double ext) {
  double m = std::max(std::fabs(v), ext) * (1.0 / 65536.0) + 1e-30;
  float f = (float)(v - m);
  if ((double)f > v - m) f = std::nextafter(f, -INFINITY);
  return f;
}
float pad_up(double v, double ext) {
  double m = std::max(std::fabs(v), ext) * (1.0 / 65536.0) + 1e-30;
  float f = (float)(v + m);
  if ((double)f < v + m) f = std::nextafter(f, INFINITY);
  return f;
}

float i2f(int v) {
  float f;
  std::memcpy(&f, &v, 4);
  return f;
}

}  // namespace

int build_host_scene(const bdpt_scene_desc* d, HostScene& out, std::string& err, bool pt) {
  if (!d || d->nprim <= 0 || !d->prim_type || !d->prim_geom || !d->prim_mat) {
    err = "scene has no primitives";
    return BDPT_E_INVALID;
  }
  if (d->nmat <= 0 || !d->mats) { err = "scene has no materials"; return BDPT_E_INVALID; }
  // the path store keeps a vertex's material id in 16 signed bits (bdpt_core.h VtxS::mb; the
  // negative ids mark environment / camera vertices)
  if (d->nmat > 32767) { err = "more than 32767 materials (the path vertex stores a 16-bit id)"; return BDPT_E_UNSUPPORTED; }
  if ((d->nlight <= 0 || !d->lights) && !d->envmap) { err = "scene has no light (BDPT needs one)"; return BDPT_E_INVALID; }
  if (d->nprim >= (1 << 24)) { err = "too many primitives for the leaf encoding (2^24)"; return BDPT_E_INVALID; }
  // materials (collada.cpp:854-938 -> bsdf.h classes)
  out.mats.clear();
  for (int i = 0; i < d->nmat; i++) {
    const bdpt_material& m = d->mats[i];
    if (m.type == BDPT_MAT_MICROFACET && !pt) {
      err = "MicrofacetBSDF::sample_pdf is assert(0) under BDPT (advanced_bsdf.cpp:144-148)";
      return BDPT_E_UNSUPPORTED;
    }
    if (m.type < BDPT_MAT_DIFFUSE || m.type > BDPT_MAT_MICROFACET) { err = "unknown material type"; return BDPT_E_INVALID; }
    DMat M;
    M.type = m.type;
    for (int k = 0; k < 3; k++) { M.a[k] = (float)m.a[k]; M.b[k] = (float)m.b[k]; }
    M.ior = (float)m.ior;
    M.alpha = (float)m.roughness;
    out.mats.push_back(M);
  }
  // lights (light.cpp:102-284)
  out.lights.clear();
  for (int i = 0; i < d->nlight; i++) {
    const bdpt_light& l = d->lights[i];
    if ((l.type == BDPT_LIGHT_HEMISPHERE || l.type == BDPT_LIGHT_DIRECTIONAL) && !pt) {
      err = "ambient (InfiniteHemisphereLight) and directional lights only implement sample_L: the BDPT light "
            "API asserts (light.cpp:25-51,72-98); use the PathTracer integrator";
      return BDPT_E_UNSUPPORTED;
    }
    if (l.type != BDPT_LIGHT_AREA && l.type != BDPT_LIGHT_POINT && l.type != BDPT_LIGHT_HEMISPHERE &&
        l.type != BDPT_LIGHT_DIRECTIONAL) {
      err = "only area and point lights implement the BDPT light API (light.cpp:25-51,168-194,299-364)";
      return BDPT_E_UNSUPPORTED;
    }
    DLight L;
    std::memset(&L, 0, sizeof L);
    L.type = l.type;
    for (int k = 0; k < 3; k++) {
      L.rad[k] = (float)l.radiance[k];
      L.pos[k] = (float)l.position[k];
      L.dir[k] = (float)l.direction[k];
      L.dx[k] = (float)l.dim_x[k];
      L.dy[k] = (float)l.dim_y[k];
    }
    L.area = (float)l.area;
    Frame f = make_frame(mk3(L.dir[0], L.dir[1], L.dir[2]));
    L.fx[0] = f.X.x; L.fx[1] = f.X.y; L.fx[2] = f.X.z;
    L.fy[0] = f.Y.x; L.fy[1] = f.Y.y; L.fy[2] = f.Y.z;
    L.fz[0] = f.Z.x; L.fz[1] = f.Z.y; L.fz[2] = f.Z.z;
    out.lights.push_back(L);
  }
  // camera (camera.cpp:191-248): tan(hFov*PI/360) evaluated in fp64 then rounded
  const bdpt_camera& c = d->camera;
  const double PI_D = 3.14159265358979323;
  for (int k = 0; k < 3; k++) out.cam.pos[k] = (float)c.pos[k];
  for (int k = 0; k < 9; k++) { out.cam.c2w[k] = (float)c.c2w[k]; out.cam.w2c[k] = (float)c.w2c[k]; }
  out.cam.tanh_ = (float)std::tan(c.hfov_deg * PI_D / 360);
  out.cam.tanv_ = (float)std::tan(c.vfov_deg * PI_D / 360);
  out.cam.nclip = (float)c.nclip;
  out.cam.fclip = (float)c.fclip;

  // primitive bboxes (triangle.cpp:9-21 / sphere.h:32-34)
  const int n = d->nprim;
  std::vector<Box> pb(n);
  for (int i = 0; i < n; i++) {
    const double* g = d->prim_geom + 18 * (size_t)i;
    int m = d->prim_mat[i];
    if (m < 0 || m >= d->nmat) { err = "primitive material index out of range"; return BDPT_E_INVALID; }
    if (d->prim_type[i] == BDPT_PRIM_TRIANGLE) {
      pb[i].from_point(g);
      pb[i].expand_pt(g + 3);
      pb[i].expand_pt(g + 6);
    } else if (d->prim_type[i] == BDPT_PRIM_SPHERE) {
      for (int k = 0; k < 3; k++) { pb[i].mn[k] = g[k] - g[3]; pb[i].mx[k] = g[k] + g[3]; }
    } else {
      err = "unknown primitive type";
      return BDPT_E_INVALID;
    }
  }
  // environment light: appended after the scene's lights (raytraced_renderer.cpp:117-119)
  out.env_light = -1;
  out.env.clear();
  if (d->envmap) {
    const bdpt_envmap& em = *d->envmap;
    if (em.width <= 0 || em.height <= 0 || !em.rgb || (long long)em.width * em.height > (1LL << 26)) {
      err = "bad environment map";
      return BDPT_E_INVALID;
    }
    const int w = em.width, h = em.height;
    const size_t np = (size_t)w * h;
    std::vector<double> pdf(np), marg(h), cond(np);
    double sum = 0;
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) {
        const float* t = em.rgb + 3 * ((size_t)w * j + i);
        const double r = t[0], g = t[1], b = t[2];
        const float il = (float)(0.2126f * r + 0.7152f * g + 0.0722f * b);   // Vector3D::illum() (float)
        pdf[(size_t)w * j + i] = il * std::sin(PI_D * (j + .5) / h);
        sum += pdf[(size_t)w * j + i];
      }
    if (!(sum > 0) || !std::isfinite(sum)) { err = "environment map has no positive radiance"; return BDPT_E_INVALID; }
    for (int j = 0; j < h; ++j) {
      const double prev = j == 0 ? 0 : marg[j - 1];
      marg[j] = prev;
      for (int i = 0; i < w; ++i) {
        pdf[(size_t)w * j + i] /= sum;
        marg[j] += pdf[(size_t)w * j + i];
      }
      const double py = marg[j] - prev;
      for (int i = 0; i < w; i++) {   // a zero row is never selected; keep its CDF finite
        const size_t k = (size_t)w * j + i;
        cond[k] = (i == 0 ? 0 : cond[k - 1]) + (py > 0 ? pdf[k] / py : 1.0 / w);
      }
    }
    out.env_w = w;
    out.env_h = h;
    // guide tables (cut-point method) for the device's CDF inversions: cell k of a CDF a[0..n) holds
    // upper_bound(a, a + n, k / G), so upper_bound(u) lies in [guide[k], guide[k + 1]] for
    // k = floor(u * G) (exact for a power-of-two G) and a short search finds the reference's index
    int gm = 1, gc = 1;
    while (gm < h) gm <<= 1;
    while (gc < w) gc <<= 1;
    out.env_gm = gm;
    out.env_gc = gc;
    out.env.resize((size_t)h + np * 2 + np * 3 + (size_t)(gm + 1) + (size_t)h * (gc + 1));
    float* o = out.env.data();
    const float* fmarg = o;
    for (int j = 0; j < h; j++) *o++ = (float)marg[j];
    const float* fcond = o;
    for (size_t k = 0; k < np; k++) *o++ = (float)cond[k];
    for (size_t k = 0; k < np; k++) *o++ = (float)pdf[k];
    for (size_t k = 0; k < np * 3; k++) *o++ = em.rgb[k];
    auto guide = [&o](const float* a, int n, int g) {
      for (int k = 0; k <= g; k++) {
        const int32_t v = (int32_t)(std::upper_bound(a, a + n, (float)k / (float)g) - a);
        std::memcpy(o++, &v, sizeof v);
      }
    };
    guide(fmarg, h, gm);
    for (int j = 0; j < h; j++) guide(fcond + (size_t)w * j, w, gc);
    // bounding sphere of the primitives (the emission disk's radius and centre)
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < n; i++)
      for (int k = 0; k < 3; k++) { mn[k] = std::min(mn[k], pb[i].mn[k]); mx[k] = std::max(mx[k], pb[i].mx[k]); }
    double ext2 = 0;
    for (int k = 0; k < 3; k++) {
      out.env_c[k] = (float)((mn[k] + mx[k]) / 2);
      ext2 += (mx[k] - mn[k]) * (mx[k] - mn[k]);
    }
    const double R = std::sqrt(ext2) / 2;
    out.env_rad = (float)R;
    DLight L;
    std::memset(&L, 0, sizeof L);
    L.type = LIGHT_ENV;
    L.area = (float)(PI_D * R * R);
    out.env_light = (int)out.lights.size();
    out.lights.push_back(L);
  }
  // the reference's tree: its DFS leaf order is the tie-break key of every primitive
  Builder R;
  R.pb = &pb;
  std::vector<int> all(n);
  for (int i = 0; i < n; i++) all[i] = i;
  const int ref_root = R.build(all, 0);
  out.depth = R.depth;
  out.ref_nodes = (int)R.nodes.size();
  out.nprim = n;
  out.ref_order = R.leaf_prims;
  std::vector<int> ref_pos(n);
  for (int k = 0; k < n; k++) ref_pos[R.leaf_prims[k]] = k;
  // the device's tree (BDPT_BVH=ref traverses the reference's own tree instead)
  const char* bvh_env = getenv("BDPT_BVH");
  const bool use_ref = bvh_env && std::string(bvh_env) == "ref";
  Builder Bs;
  int root = ref_root;
  if (!use_ref) {
    SahBuilder S;
    S.pb = &pb;
    S.desc = d;
    // diagnostics / A-B: leaf size and SAH termination of the device tree (no effect on results)
    if (const char* e = getenv("BDPT_SAH_LEAF")) S.leaf_max = std::max(1, std::min(4, atoi(e)));
    if (const char* e = getenv("BDPT_SAH_CT")) S.ct = atof(e);
    if (const char* e = getenv("BDPT_SAH_BINS")) S.nb = std::max(2, std::min(SahBuilder::kMaxBins, atoi(e)));
    // spatial splits (scenes of >= kSbvhMinPrims primitives): alpha and the reference budget
    if (n >= kSbvhMinPrims) {
      S.alpha = kSbvhAlpha;
      S.budget = kSbvhBudget;
    }
    if (const char* e = getenv("BDPT_SBVH")) S.alpha = n >= kSbvhMinPrims ? atof(e) : 0.0;
    if (const char* e = getenv("BDPT_SBVH_BUDGET")) S.budget = atof(e);
    root = S.build_root(n);
    Bs.nodes = std::move(S.nodes);
    Bs.leaf_prims = std::move(S.leaf_prims);
    Bs.depth = S.depth;
  }
  Builder& T = use_ref ? R : Bs;
  out.dev_depth = T.depth;
  out.dev_nodes = (int)T.nodes.size();

  // primitives in the device tree's DFS leaf order (a primitive that a spatial split references
  // from two leaves has a record at both positions)
  const int nref = (int)T.leaf_prims.size();
  if (nref >= (1 << 24)) { err = "too many primitive references for the leaf encoding (2^24)"; return BDPT_E_UNSUPPORTED; }
  out.prim_ref = T.leaf_prims;
  out.geom.assign(12 * (size_t)nref, 0.0f);
  out.shade.assign(12 * (size_t)nref, 0.0f);
  for (int k = 0; k < nref; k++) {
    int i = T.leaf_prims[k];
    const double* g = d->prim_geom + 18 * (size_t)i;
    float* G = &out.geom[12 * (size_t)k];
    float* S = &out.shade[12 * (size_t)k];
    if (d->prim_type[i] == BDPT_PRIM_TRIANGLE) {
      float p1[3], p2[3], p3[3];
      for (int c3 = 0; c3 < 3; c3++) { p1[c3] = (float)g[c3]; p2[c3] = (float)g[3 + c3]; p3[c3] = (float)g[6 + c3]; }
      float e1[3], e2[3];
      for (int c3 = 0; c3 < 3; c3++) { e1[c3] = p2[c3] - p1[c3]; e2[c3] = p3[c3] - p1[c3]; }
      G[0] = p1[0]; G[1] = p1[1]; G[2] = p1[2]; G[3] = e1[0];
      G[4] = e1[1]; G[5] = e1[2]; G[6] = e2[0]; G[7] = e2[1];
      G[8] = e2[2];
      G[9] = i2f(ref_pos[i]);   // tie-break key (third float4 .y)
      for (int c3 = 0; c3 < 9; c3++) S[c3] = (float)g[9 + c3];
      S[9] = i2f(d->prim_mat[i]);
      S[10] = i2f(0);
    } else {
      G[0] = (float)g[0]; G[1] = (float)g[1]; G[2] = (float)g[2]; G[3] = (float)g[3];
      G[4] = i2f(ref_pos[i]);   // tie-break key (second float4 .x)
      S[9] = i2f(d->prim_mat[i]);
      S[10] = i2f(1);
    }
  }
  for (int W : {2, 4}) {
    HostBvh& B = W == 4 ? out.bvh4 : out.bvh2;
    auto sarea = [](const Box& b) {
      const double dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
      return 2 * (dx * dy + dy * dz + dz * dx);
    };
    // Wide nodes (W children) by the collapse that minimises the wide tree's SAH cost: dynamic
    // programming over the binary tree, F[n][i] = the cheapest way to represent n's subtree as at
    // most i roots (a leaf: its area x c_prim per primitive; n itself as a wide node: its area x
    // c_node plus the best split of its W slots between its two binary children), Fk the choice
    // (0 = n itself, k = k slots to the left child). Measured against pulling in the grandchildren
    // of the largest-area children (round 4 and before): node steps per walk query 6.95 -> 5.76,
    // expected wave-level steps 28.8 -> 27.5 (CPU build, tools/step_hist.py); north star 702 -> 724,
    // CBbunny 800x600 520 -> 537, C5-shaped 599 -> 618 Msamples/s (profiles/r05h_ab_sah_collapse.log).
    // Results do not depend on the tree shape (closest hit by t, then DFS key).
    const double c_node = 1.0, c_prim = 0.5;
    std::vector<std::array<double, 9>> F(T.nodes.size());
    std::vector<std::array<int, 9>> Fk(T.nodes.size());
    if (W > 2 && T.nodes[root].l >= 0) {
      const double inf = 1e300;
      std::vector<int> post, st{root};
      while (!st.empty()) {   // pre-order; walked backwards = children before parents
        const int id = st.back();
        st.pop_back();
        post.push_back(id);
        if (T.nodes[id].l >= 0) { st.push_back(T.nodes[id].l); st.push_back(T.nodes[id].r); }
      }
      for (auto it = post.rbegin(); it != post.rend(); ++it) {
        const int id = *it;
        const Node& nd = T.nodes[id];
        const double a = sarea(nd.box);
        if (nd.l < 0) {
          for (int i = 0; i <= W; i++) { F[id][i] = i ? a * c_prim * nd.count : inf; Fk[id][i] = 0; }
          continue;
        }
        double g = inf;
        for (int k = 1; k < W; k++) g = std::min(g, F[nd.l][k] + F[nd.r][W - k]);
        F[id][0] = inf;
        F[id][1] = a * c_node + g;
        Fk[id][1] = 0;
        for (int i = 2; i <= W; i++) {
          F[id][i] = F[id][1];
          Fk[id][i] = 0;
          for (int k = 1; k < i; k++)
            if (F[nd.l][k] + F[nd.r][i - k] < F[id][i]) { F[id][i] = F[nd.l][k] + F[nd.r][i - k]; Fk[id][i] = k; }
        }
      }
    }
    auto children = [&](int id) {
      std::vector<int> ch;
      const Node& nd = T.nodes[id];
      if (W == 2) return std::vector<int>{nd.l, nd.r};
      std::function<void(int, int)> expand = [&](int m, int i) {
        if (i <= 1 || T.nodes[m].l < 0 || Fk[m][i] == 0) { ch.push_back(m); return; }
        expand(T.nodes[m].l, Fk[m][i]);
        expand(T.nodes[m].r, i - Fk[m][i]);
      };
      int bk = 1;
      double bc = 1e300;
      for (int k = 1; k < W; k++)
        if (F[nd.l][k] + F[nd.r][W - k] < bc) { bc = F[nd.l][k] + F[nd.r][W - k]; bk = k; }
      expand(nd.l, bk);
      expand(nd.r, W - bk);
      return ch;
    };
    // node order: the top kTopNodes wide nodes in BFS order (the LDS treelet: every ray starts
    // there), then the rest in DFS pre-order (subtrees contiguous for the global fetches).
    std::vector<int> dev_index(T.nodes.size(), -1);
    std::vector<int> order;
    std::vector<std::vector<int>> kids;   // per emitted node, its binary child ids
    int wdepth = 0;
    if (T.nodes[root].l >= 0) {
      std::vector<int> bfs{root};
      for (size_t h = 0; h < bfs.size() && (int)order.size() < kTopNodes; h++) {
        int id = bfs[h];
        dev_index[id] = (int)order.size();
        order.push_back(id);
        kids.push_back(children(id));
        for (int ch : kids.back())
          if (T.nodes[ch].l >= 0) bfs.push_back(ch);
      }
      B.n_top = (int)order.size();
      std::vector<std::pair<int, int>> st{{root, 0}};
      while (!st.empty()) {
        const int id = st.back().first, dd = st.back().second;
        st.pop_back();
        wdepth = std::max(wdepth, dd);
        if (dev_index[id] < 0) {
          dev_index[id] = (int)order.size();
          order.push_back(id);
          kids.push_back(children(id));
        }
        const std::vector<int>& ch = kids[dev_index[id]];
        for (int k = (int)ch.size() - 1; k >= 0; k--)
          if (T.nodes[ch[k]].l >= 0) st.push_back({ch[k], dd + 1});
      }
    }
    B.depth = wdepth;
    if ((W - 1) * (wdepth + 1) + 2 > kStackMax) {
      err = "BVH deeper than the traversal stack";
      return BDPT_E_UNSUPPORTED;
    }
    bool wide_sph_leaf = false;
    auto ref_of = [&](int id) -> int {
      const Node& nd = T.nodes[id];
      if (nd.l >= 0) return dev_index[id];
      int mask = 0;
      for (int k = 0; k < nd.count; k++) {
        int i = T.leaf_prims[nd.start + k];
        if (d->prim_type[i] == BDPT_PRIM_SPHERE) mask |= 1 << k;
      }
      if (mask >> 4) wide_sph_leaf = true;   // the reference's sphere mask has 4 bits
      uint32_t enc = ((uint32_t)nd.start << 7) | ((uint32_t)mask << 3) | (uint32_t)nd.count;
      return (int)~enc;
    };
    // padded fp32 child boxes: lo.xyz, hi.xyz
    auto child_box = [&](int id, float v[6]) {
      const Box& b = T.nodes[id].box;
      double ext = std::max(b.mx[0] - b.mn[0], std::max(b.mx[1] - b.mn[1], b.mx[2] - b.mn[2]));
      for (int c3 = 0; c3 < 3; c3++) {
        v[c3] = pad_down(b.mn[c3], ext);
        v[3 + c3] = pad_up(b.mx[c3], ext);
      }
    };
    B.nodes.assign((size_t)4 * node_f4(W) * order.size(), 0.0f);
    for (size_t k = 0; k < order.size(); k++) {
      float* N = &B.nodes[(size_t)4 * node_f4(W) * k];
      const std::vector<int>& ch = kids[k];
      if (W == 2) {
        // lo_l.xyz hi_l.x | hi_l.yz lo_r.xy | lo_r.z hi_r.xyz | refs
        child_box(ch[0], N);
        child_box(ch[1], N + 6);
        N[12] = i2f(ref_of(ch[0]));
        N[13] = i2f(ref_of(ch[1]));
      } else {
        // SoA over the children: lo.x[4] hi.x[4] lo.y[4] hi.y[4] lo.z[4] hi.z[4] | refs[4] | pad;
        // an empty slot has ref kTravDone and an inverted infinite box (lo +inf, hi -inf): whatever
        // the direction's signs, its near plane distance is +inf and its far one -inf (no NaN for a
        // finite inverse), so its slab test fails without looking at the reference
        for (int s = 0; s < W; s++) {
          float v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
          int rf = kTravDone;
          if (s < (int)ch.size()) {
            child_box(ch[s], v);
            rf = ref_of(ch[s]);
          }
          for (int c3 = 0; c3 < 3; c3++) {
            N[8 * c3 + s] = v[c3];
            N[8 * c3 + 4 + s] = v[3 + c3];
          }
          N[24 + s] = i2f(rf);
        }
      }
    }
    B.root = ref_of(root);
    if (W == 2) {   // every leaf reference in DFS order: the flat traversal of tiny scenes (LM 3)
      out.leaf_refs.clear();
      std::vector<int> st{root};
      while (!st.empty()) {
        const int id = st.back();
        st.pop_back();
        if (T.nodes[id].l < 0) { out.leaf_refs.push_back(ref_of(id)); continue; }
        st.push_back(T.nodes[id].r);
        st.push_back(T.nodes[id].l);
      }
    }
    if (wide_sph_leaf) {
      err = "a BVH leaf holds a sphere past its 4th primitive (the leaf reference's sphere mask has 4 bits)";
      return BDPT_E_UNSUPPORTED;
    }
  }
  return BDPT_OK;
}

}  // namespace bdpt
