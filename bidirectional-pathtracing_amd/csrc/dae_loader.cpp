// dae_loader.cpp — COLLADA scene loader (see dae_loader.h for the reference functions restated).
// Arithmetic follows the reference build (-O3 -mavx2, CGL double vectors): v/c = v*(1/c),
// normalize = *= 1/norm, left-to-right sums, Matrix4x4 * Matrix4x4 as its __AVX__ branch computes
// it (matrix4x4.cpp:125-144: C(i,j) = dot(column i of A, column j of B)), parsed COLLADA floats
// rounded to float where the reference stores float.
#include "dae_loader.h"

#include "bdpt_err.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <set>
#include <sstream>
#include <utility>

namespace bdpt {

namespace {

constexpr double kPi = 3.14159265358979323;   // CGL/include/CGL/misc.h:11
constexpr float kEpsF = 0.00001f;             // misc.h:13

// ---------------------------------------------------------------------------------------------
// Minimal XML DOM (elements, attributes, text; comments / declarations skipped).
struct XEl {
  std::string name, text;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<std::unique_ptr<XEl>> kids;
  XEl* parent = nullptr;
  const char* attr(const char* k) const {
    for (auto& a : attrs)
      if (a.first == k) return a.second.c_str();
    return nullptr;
  }
  XEl* first(const char* n) const {
    for (auto& k : kids)
      if (!n || k->name == n) return k.get();
    return nullptr;
  }
  XEl* next(const char* n) const {   // next sibling (with name n, or any)
    if (!parent) return nullptr;
    bool seen = false;
    for (auto& k : parent->kids) {
      if (seen && (!n || k->name == n)) return k.get();
      if (k.get() == this) seen = true;
    }
    return nullptr;
  }
};

std::string xml_unescape(const std::string& s) {
  if (s.find('&') == std::string::npos) return s;
  std::string o;
  for (size_t i = 0; i < s.size(); i++) {
    if (s[i] == '&') {
      size_t e = s.find(';', i);
      if (e != std::string::npos) {
        std::string ent = s.substr(i + 1, e - i - 1);
        const char* rep = ent == "lt" ? "<" : ent == "gt" ? ">" : ent == "amp" ? "&" : ent == "quot" ? "\"" : ent == "apos" ? "'" : nullptr;
        if (rep) { o += rep; i = e; continue; }
      }
    }
    o += s[i];
  }
  return o;
}

bool parse_xml(const std::string& src, XEl& root, std::string& err) {
  size_t i = 0, n = src.size();
  XEl* cur = &root;
  while (i < n) {
    if (src[i] != '<') {
      size_t j = src.find('<', i);
      if (j == std::string::npos) j = n;
      cur->text += xml_unescape(src.substr(i, j - i));
      i = j;
      continue;
    }
    if (src.compare(i, 4, "<!--") == 0) {
      size_t j = src.find("-->", i);
      if (j == std::string::npos) { err = "unterminated comment"; return false; }
      i = j + 3;
      continue;
    }
    if (src.compare(i, 2, "<?") == 0 || src.compare(i, 2, "<!") == 0) {
      size_t j = src.find('>', i);
      if (j == std::string::npos) { err = "unterminated declaration"; return false; }
      i = j + 1;
      continue;
    }
    if (src.compare(i, 2, "</") == 0) {
      size_t j = src.find('>', i);
      if (j == std::string::npos || !cur->parent) { err = "bad closing tag"; return false; }
      cur = cur->parent;
      i = j + 1;
      continue;
    }
    // start tag
    size_t j = i + 1;
    while (j < n && !isspace((unsigned char)src[j]) && src[j] != '>' && src[j] != '/') j++;
    auto el = std::make_unique<XEl>();
    el->name = src.substr(i + 1, j - i - 1);
    el->parent = cur;
    bool selfclose = false;
    for (;;) {
      while (j < n && isspace((unsigned char)src[j])) j++;
      if (j >= n) { err = "unterminated tag"; return false; }
      if (src[j] == '>') { j++; break; }
      if (src[j] == '/') { selfclose = true; j = src.find('>', j) + 1; break; }
      size_t k = j;
      while (k < n && src[k] != '=' && !isspace((unsigned char)src[k])) k++;
      std::string key = src.substr(j, k - j);
      k = src.find_first_of("\"'", k);
      if (k == std::string::npos) { err = "bad attribute"; return false; }
      char q = src[k];
      size_t e = src.find(q, k + 1);
      if (e == std::string::npos) { err = "bad attribute"; return false; }
      el->attrs.emplace_back(key, xml_unescape(src.substr(k + 1, e - k - 1)));
      j = e + 1;
    }
    XEl* raw = el.get();
    cur->kids.push_back(std::move(el));
    if (!selfclose) cur = raw;
    i = j;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// CGL math (double).
struct V3 {
  double x = 0, y = 0, z = 0;
  V3() {}
  V3(double a, double b, double c) : x(a), y(b), z(c) {}
  V3 operator+(const V3& v) const { return V3(x + v.x, y + v.y, z + v.z); }
  V3 operator-(const V3& v) const { return V3(x - v.x, y - v.y, z - v.z); }
  V3 operator*(double c) const { return V3(x * c, y * c, z * c); }
  V3 operator/(double c) const { double rc = 1.0 / c; return V3(rc * x, rc * y, rc * z); }
  void operator+=(const V3& v) { x += v.x; y += v.y; z += v.z; }
  double norm() const { return std::sqrt(x * x + y * y + z * z); }
  void normalize() { double rc = 1.0 / norm(); x *= rc; y *= rc; z *= rc; }
  V3 unit() const { double rn = 1.0 / norm(); return (*this) * rn; }
};
V3 cross(const V3& u, const V3& v) { return V3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x); }

struct V4 {
  double x = 0, y = 0, z = 0, w = 0;
  V4() {}
  V4(double a, double b, double c, double d) : x(a), y(b), z(c), w(d) {}
  V4(const V3& v, double d) : x(v.x), y(v.y), z(v.z), w(d) {}
  double operator[](int i) const { return i == 0 ? x : i == 1 ? y : i == 2 ? z : w; }
  V3 to3D() const { return V3(x, y, z); }
  V3 projectTo3D() const { double iw = 1.0 / w; return V3(x * iw, y * iw, z * iw); }
};

struct M4 {   // column-major: col[j] is column j; (i, j) = col[j][i]
  V4 col[4];
  double& at(int i, int j) { return (&col[j].x)[i]; }
  double at(int i, int j) const { return (&col[j].x)[i]; }
  static M4 identity() {
    M4 m;
    for (int k = 0; k < 4; k++) m.at(k, k) = 1.0;
    return m;
  }
  V4 operator*(const V4& v) const {   // x0*c0 + x1*c1 + x2*c2 + x3*c3 (matrix4x4.cpp:146-149)
    V4 r;
    for (int k = 0; k < 4; k++) {
      const V4& c = col[k];
      const double s = v[k];
      if (k == 0) r = V4(s * c.x, s * c.y, s * c.z, s * c.w);
      else r = V4(r.x + s * c.x, r.y + s * c.y, r.z + s * c.z, r.w + s * c.w);
    }
    return r;
  }
};
// Matrix4x4::operator*(Matrix4x4) in the reference's AVX build (matrix4x4.cpp:131-132):
// C(i, j) = dot(A[i], B column j) with A[i] the i-th COLUMN of A, i.e. C = A^T * B.
M4 mat_mul_ref(const M4& A, const M4& B) {
  M4 C;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      C.at(i, j) = A.at(0, i) * B.at(0, j) + A.at(1, i) * B.at(1, j) + A.at(2, i) * B.at(2, j) +
                   A.at(3, i) * B.at(3, j);
  return C;
}

double radians(double d) { return d * (kPi / 180); }
double degrees(double r) { return r * (180 / kPi); }

std::vector<std::string> tokens(const std::string& s) {
  std::vector<std::string> t;
  std::istringstream ss(s);
  std::string w;
  while (ss >> w) t.push_back(w);
  return t;
}
V3 spectrum_of(const char* s) {   // spectrum_from_string: doubles
  std::istringstream ss(s ? s : "");
  V3 v;
  ss >> v.x >> v.y >> v.z;
  return v;
}

// ---------------------------------------------------------------------------------------------
// COLLADA document -> instances (collada.cpp)
enum InstType { I_NONE, I_CAMERA, I_LIGHT, I_MESH, I_SPHERE };
enum LightKind { LK_NONE, LK_AMBIENT, LK_DIRECTIONAL, LK_AREA, LK_POINT, LK_SPOT };

struct Material {   // one per instance_material (each builds a new BSDF, collada.cpp:854-938)
  int type = BDPT_MAT_DIFFUSE;
  V3 a, b;
  double ior = 0, roughness = 0;
};

struct Node {
  InstType type = I_NONE;
  M4 T;
  // camera
  float hfov = 50, vfov = 35, nclip = 0.001f, fclip = 1000;
  V3 view_dir, up_dir;
  // light
  LightKind lk = LK_NONE;
  V3 spectrum = V3(1, 1, 1), lpos = V3(0, 0, 0), ldir = V3(0, 0, -1), lup = V3(0, 1, 0);
  // mesh
  std::vector<V3> verts;
  std::vector<std::vector<size_t>> polys;
  // sphere
  float radius = 0;
  bool has_mat = false;
  Material mat;
};

struct Parser {
  std::map<std::string, XEl*> ids;
  M4 transform = M4::identity();
  V3 up;
  std::vector<Node> nodes;
  std::string err;

  void uri_load(XEl* e) {
    if (const char* id = e->attr("id")) ids[id] = e;
    for (auto& k : e->kids) uri_load(k.get());
  }
  XEl* uri_find(const std::string& id) {
    auto it = ids.find(id);
    return it == ids.end() ? nullptr : it->second;
  }
  XEl* get(XEl* x, const std::string& q) {   // get_element: path of first children + url hop
    std::istringstream ss(q);
    std::string tok;
    XEl* e = x;
    while (e && std::getline(ss, tok, '/')) e = e->first(tok.c_str());
    if (e) {
      if (const char* url = e->attr("url")) e = uri_find(url_id(url));
    }
    return e;
  }
  XEl* technique_common(XEl* x) {
    if (XEl* p = x->first("profile_COMMON")) {
      for (XEl* t = p->first("technique"); t; t = t->next("technique")) {
        const char* sid = t->attr("sid");
        if (sid && std::string(sid) == "common") return t;
      }
    }
    return x->first("technique_common");
  }
  XEl* technique_cgl(XEl* x) {
    for (XEl* t = get(x, "extra/technique"); t; t = t->next("technique")) {
      const char* pr = t->attr("profile");
      if (pr && std::string(pr) == "CGL") return t;
    }
    return nullptr;
  }

  bool load(XEl* root) {
    uri_load(root);
    if (XEl* asset = get(root, "asset")) {
      XEl* ua = get(asset, "up_axis");
      if (!ua) { err = "no up_axis"; return false; }
      std::string u = tokens(ua->text).empty() ? "" : tokens(ua->text)[0];
      transform = M4::identity();
      if (u == "X_UP") {
        transform.at(0, 0) = 0; transform.at(0, 1) = 1;
        transform.at(1, 0) = 1; transform.at(1, 1) = 0;
        transform.at(2, 2) = -1;
        up = V3(1, 0, 0);
      } else if (u == "Z_UP") {
        transform.at(1, 1) = 0; transform.at(1, 2) = 1;
        transform.at(2, 1) = 1; transform.at(2, 2) = 0;
        transform.at(0, 0) = -1;
        up = V3(0, 0, 1);
      } else if (u == "Y_UP") {
        up = V3(0, 1, 0);
      } else {
        err = "invalid up_axis";
        return false;
      }
    }
    XEl* sc = get(root, "scene/instance_visual_scene");
    if (!sc) { err = "no visual scene"; return false; }
    for (XEl* n = get(sc, "node"); n; n = n->next("node"))
      if (!parse_node(n)) return false;
    return true;
  }

  bool parse_node(XEl* x) {
    Node node;
    node.T = M4::identity();
    for (auto& kp : x->kids) {
      XEl* e = kp.get();
      const std::vector<std::string> t = tokens(e->text);
      auto num = [&](size_t k) { return k < t.size() ? strtod(t[k].c_str(), nullptr) : 0.0; };
      if (e->name == "matrix") {
        M4 m;
        for (int i = 0; i < 4; i++)
          for (int j = 0; j < 4; j++) m.at(i, j) = num(4 * i + j);
        node.T = m;
        break;
      }
      if (e->name == "rotate") {   // collada.cpp:274-299, restated as written
        M4 m;
        const char* sid = e->attr("sid");
        char ax = sid && *sid ? sid[strlen(sid) - 1] : 0;
        if (ax == 'X') { m.at(1, 1) = num(0); m.at(1, 2) = num(1); m.at(2, 1) = num(2); m.at(2, 2) = num(3); }
        if (ax == 'Y') { m.at(0, 0) = num(0); m.at(2, 0) = num(1); m.at(0, 2) = num(2); m.at(2, 2) = num(3); }
        if (ax == 'Z') { m.at(0, 0) = num(0); m.at(0, 1) = num(1); m.at(1, 0) = num(2); m.at(1, 1) = num(3); }
        node.T = mat_mul_ref(m, node.T);
      }
      if (e->name == "translate") {
        M4 m;
        m.at(0, 3) = num(0); m.at(1, 3) = num(1); m.at(2, 3) = num(2);
        node.T = mat_mul_ref(m, node.T);
      }
      if (e->name == "scale") {
        M4 m;
        m.at(0, 0) = num(0); m.at(1, 1) = num(1); m.at(1, 1) = num(2);
        node.T = mat_mul_ref(m, node.T);
      }
    }
    const M4 saved = transform;
    node.T = mat_mul_ref(transform, node.T);
    transform = node.T;
    for (XEl* c = get(x, "node"); c; c = c->next("node"))
      if (!parse_node(c)) return false;
    transform = saved;

    XEl* ecam = get(x, "instance_camera");
    XEl* elight = get(x, "instance_light");
    XEl* egeo = get(x, "instance_geometry");
    if (ecam) {
      if (!parse_camera(ecam, node)) return false;
    } else if (elight) {
      if (!parse_light(elight, node)) return false;
    } else if (egeo) {
      if (get(egeo, "mesh")) {
        if (!parse_mesh(egeo, node)) return false;
      } else if (get(egeo, "extra")) {
        if (!parse_sphere(egeo, node)) return false;
      }
      if (node.type != I_NONE) {
        if (XEl* im = get(x, "instance_geometry/bind_material/technique_common/instance_material")) {
          const char* tg = im->attr("target");
          if (!tg) { err = "instance_material without target"; return false; }
          XEl* m = uri_find(url_id(tg));
          if (!m) { err = std::string("unknown material ") + tg; return false; }
          if (!parse_material(m, node.mat)) return false;
          node.has_mat = true;
        }
      }
    }
    nodes.push_back(std::move(node));
    return true;
  }

  bool parse_camera(XEl* x, Node& n) {
    n.type = I_CAMERA;
    n.up_dir = up;
    n.view_dir = V3(0, 0, -1);
    XEl* p = get(x, "optics/technique_common/perspective");
    if (!p) { err = "camera without perspective"; return false; }
    XEl *ex = p->first("xfov"), *ey = p->first("yfov"), *en = p->first("znear"), *ef = p->first("zfar");
    n.hfov = ex ? (float)atof(ex->text.c_str()) : 50.0f;
    n.vfov = ey ? (float)atof(ey->text.c_str()) : 35.0f;
    n.nclip = en ? (float)atof(en->text.c_str()) : 0.001f;
    n.fclip = ef ? (float)atof(ef->text.c_str()) : 1000.0f;
    if (!ey) {
      XEl* ar = get(p, "aspect_ratio");
      if (!ar) { err = "camera: no yfov and no aspect_ratio"; return false; }
      float a = (float)atof(ar->text.c_str());
      n.vfov = (float)(2 * degrees(atan(tan(radians(0.5 * n.hfov)) / a)));
    }
    return true;
  }

  bool parse_light(XEl* x, Node& n) {
    n.type = I_LIGHT;
    XEl* tc = technique_common(x);
    XEl* tg = technique_cgl(x);
    XEl* t = tg ? tg : tc;
    if (!t) { err = "light without profile"; return false; }
    XEl* e = t->first(nullptr);
    if (!e) return true;
    const std::string ty = e->name;
    XEl* col = get(e, "color");
    if (ty == "ambient") n.lk = LK_AMBIENT;
    else if (ty == "directional") n.lk = LK_DIRECTIONAL;
    else if (ty == "area") n.lk = LK_AREA;
    else if (ty == "point") n.lk = LK_POINT;
    else if (ty == "spot") n.lk = LK_SPOT;
    else { err = "unknown light type " + ty; return false; }
    if (!col) { err = "light without color"; return false; }
    if ((n.lk == LK_POINT || n.lk == LK_SPOT) &&
        !(get(e, "constant_attenuation") && get(e, "linear_attenuation") && get(e, "quadratic_attenuation"))) {
      err = "incomplete point/spot light";
      return false;
    }
    n.spectrum = spectrum_of(col->text.c_str());
    return true;
  }

  bool parse_sphere(XEl* x, Node& n) {
    XEl* t = technique_cgl(x);
    if (!t) { err = "sphere without CGL technique"; return false; }
    XEl* r = get(t, "sphere/radius");
    if (!r) { err = "sphere without radius"; return false; }
    n.type = I_SPHERE;
    n.radius = (float)atof(r->text.c_str());
    return true;
  }

  // "#id" of a source / url attribute ("" when absent)
  static std::string url_id(const char* a) { return !a ? std::string() : std::string(a[0] == '#' ? a + 1 : a); }

  bool parse_mesh(XEl* x, Node& n) {
    XEl* m = x->first("mesh");
    if (!m) { err = "geometry without mesh"; return false; }
    std::map<std::string, std::vector<float>> src;
    for (XEl* s = m->first("source"); s; s = s->next("source")) {
      XEl* fa = s->first("float_array");
      if (!fa) continue;
      const char* cnt = fa->attr("count");
      size_t nf = cnt ? (size_t)atol(cnt) : 0;
      std::vector<float> f;
      f.reserve(std::min(nf, fa->text.size() / 2 + 1));   // a count beyond the text reads what is there
      const char* p = fa->text.c_str();
      for (size_t i = 0; i < nf; i++) {
        char* end;
        float v = strtof(p, &end);
        if (end == p) break;
        f.push_back(v);
        p = end;
      }
      const char* id = s->attr("id");
      src[id ? id : ""] = std::move(f);
    }
    XEl* ev = m->first("vertices");
    if (!ev) { err = "mesh without vertices"; return false; }
    const std::string vid = ev->attr("id") ? ev->attr("id") : "";
    std::vector<V3> verts;
    for (XEl* in = ev->first("input"); in; in = in->next("input")) {
      const char* sem = in->attr("semantic");
      if (!sem || std::string(sem) != "POSITION") continue;
      auto it = src.find(url_id(in->attr("source")));
      if (it == src.end()) { err = "bad POSITION source"; return false; }
      for (size_t i = 0; i + 2 < it->second.size(); i += 3)
        verts.emplace_back(it->second[i], it->second[i + 1], it->second[i + 2]);
    }
    n.type = I_MESH;
    XEl* pl = m->first("polylist");
    if (!pl) return true;   // only polylists are read (collada.cpp:681)
    bool hv = false, hn = false, ht = false;
    size_t vo = 0;
    for (XEl* in = pl->first("input"); in; in = in->next("input")) {
      const std::string sem = in->attr("semantic") ? in->attr("semantic") : "";
      const size_t off = in->attr("offset") ? (size_t)atol(in->attr("offset")) : 0;
      if (sem == "VERTEX") {
        hv = true;
        vo = off;
        if (url_id(in->attr("source")) != vid) { err = "VERTEX source mismatch"; return false; }
        n.verts = verts;
      }
      if (sem == "NORMAL") hn = true;
      if (sem == "TEXCOORD") ht = true;
    }
    const size_t npoly = pl->attr("count") ? (size_t)atol(pl->attr("count")) : 0;
    const size_t stride = (hv ? 1 : 0) + (hn ? 1 : 0) + (ht ? 1 : 0);
    XEl* vc = pl->first("vcount");
    XEl* pp = pl->first("p");
    if (!vc || !pp) { err = "polylist without vcount / p"; return false; }
    std::vector<size_t> sizes;
    size_t nidx = 0;
    {
      // malformed files (counts beyond the lists, offsets beyond the stride) are rejected here;
      // the reference's parser would read past its arrays on them
      const char* p = vc->text.c_str();
      for (size_t i = 0; i < npoly; i++) {
        char* end;
        size_t s = strtoul(p, &end, 10);
        if (end == p || s > pp->text.size()) { err = "polylist vcount does not match its count"; return false; }
        p = end;
        sizes.push_back(s);
        nidx += s * stride;
      }
    }
    if (hv && vo >= stride) { err = "polylist input offset beyond its stride"; return false; }
    if (nidx > pp->text.size()) { err = "polylist p shorter than its vcount"; return false; }
    std::vector<size_t> idx;
    idx.reserve(nidx);
    {
      const char* p = pp->text.c_str();
      for (size_t i = 0; i < nidx; i++) {
        char* end;
        size_t v = strtoul(p, &end, 10);
        if (end == p) { err = "polylist p shorter than its vcount"; return false; }
        p = end;
        idx.push_back(v);
      }
    }
    if (hv) {
      size_t k = 0;
      n.polys.resize(npoly);
      for (size_t i = 0; i < npoly; i++)
        for (size_t j = 0; j < sizes[i]; j++, k++) n.polys[i].push_back(idx[k * stride + vo]);
    }
    return true;
  }

  bool parse_material(XEl* x, Material& mat) {
    XEl* fx = get(x, "instance_effect");
    if (!fx) { err = "material without effect"; return false; }
    XEl* tc = technique_common(fx);
    XEl* tg = technique_cgl(fx);
    mat = Material();
    if (tg) {
      for (XEl* b = tg->first(nullptr); b; b = b->next(nullptr)) {
        const std::string ty = b->name;
        auto txt = [&](const char* q) -> const char* {
          XEl* e = get(b, q);
          return e ? e->text.c_str() : nullptr;
        };
        if (ty == "emission") {
          mat = Material();
          mat.type = BDPT_MAT_EMISSION;
          mat.a = spectrum_of(txt("radiance"));
        } else if (ty == "mirror") {
          mat = Material();
          mat.type = BDPT_MAT_MIRROR;
          mat.a = spectrum_of(txt("reflectance"));
        } else if (ty == "microfacet") {   // collada.cpp:886-895: a = eta, b = k, alpha as float
          mat = Material();
          mat.type = BDPT_MAT_MICROFACET;
          mat.a = spectrum_of(txt("eta"));
          mat.b = spectrum_of(txt("k"));
          mat.roughness = (float)atof(txt("alpha") ? txt("alpha") : "0");
        } else if (ty == "refraction") {
          mat = Material();
          mat.type = BDPT_MAT_REFRACTION;
          mat.b = spectrum_of(txt("transmittance"));
          mat.roughness = (float)atof(txt("roughness") ? txt("roughness") : "0");
          mat.ior = (float)atof(txt("ior") ? txt("ior") : "0");
        } else if (ty == "glass") {
          mat = Material();
          mat.type = BDPT_MAT_GLASS;
          mat.b = spectrum_of(txt("transmittance"));
          mat.a = spectrum_of(txt("reflectance"));
          mat.roughness = (float)atof(txt("roughness") ? txt("roughness") : "0");
          mat.ior = (float)atof(txt("ior") ? txt("ior") : "0");
        }
      }
    } else if (tc) {
      XEl* d = get(tc, "phong/diffuse/color");
      mat.type = BDPT_MAT_DIFFUSE;
      mat.a = d ? spectrum_of(d->text.c_str()) : V3(.5f, .5f, .5f);
    } else {
      mat.type = BDPT_MAT_DIFFUSE;
      mat.a = V3(.5f, .5f, .5f);
    }
    return true;
  }
};

// ---------------------------------------------------------------------------------------------
// HalfedgeMesh::build (halfEdgeMesh.cpp:29-404): only what fixes the triangle vertex order and the
// vertex normals. Containers are creation-ordered like the reference's std::lists.
struct HalfedgeMesh {
  struct HE { int next = -1, twin = -1, vertex = -1, face = -1; };
  struct Face { int he = -1; bool boundary = false; };
  std::vector<HE> h;
  std::vector<int> vhe;        // vertex -> halfedge
  std::vector<V3> vpos, vnrm;
  std::vector<Face> faces;     // real faces first (polygon order), then boundary loops

  bool build(const std::vector<std::vector<size_t>>& polys, const std::vector<V3>& positions, std::string& err) {
    std::map<size_t, int> index_to_vertex;
    for (const auto& p : polys) {
      if (p.size() < 3) { err = "polygon with < 3 vertices"; return false; }
      std::set<size_t> distinct(p.begin(), p.end());
      if (distinct.size() < p.size()) { err = "polygon with repeated vertices"; return false; }
      for (size_t i : p)
        if (!index_to_vertex.count(i)) {
          index_to_vertex[i] = (int)vhe.size();
          vhe.push_back(-1);
        }
    }
    const int nreal = (int)polys.size();
    faces.resize(nreal);
    std::map<std::pair<size_t, size_t>, int> pair_he;
    for (int f = 0; f < nreal; f++) {
      const auto& p = polys[f];
      const size_t deg = p.size();
      std::vector<int> fh;
      for (size_t i = 0; i < deg; i++) {
        const size_t a = p[i], b = p[(i + 1) % deg];
        if (pair_he.count({a, b})) { err = "non-manifold or inconsistently oriented mesh"; return false; }
        const int hab = (int)h.size();
        h.push_back(HE());
        pair_he[{a, b}] = hab;
        h[hab].face = f;
        faces[f].he = hab;
        h[hab].vertex = index_to_vertex[a];
        vhe[index_to_vertex[a]] = hab;
        fh.push_back(hab);
        auto it = pair_he.find({b, a});
        if (it != pair_he.end()) {
          h[hab].twin = it->second;
          h[it->second].twin = hab;
        }
      }
      for (size_t i = 0; i < deg; i++) h[fh[i]].next = fh[(i + 1) % deg];
    }
    // boundary vertices point at a boundary halfedge
    for (size_t v = 0; v < vhe.size(); v++) {
      const int start = vhe[v];
      int e = start;
      do {
        if (h[e].twin < 0) { vhe[v] = e; break; }
        e = h[h[e].twin].next;
      } while (e != start);
    }
    // boundary loops (the loop also visits halfedges appended meanwhile; they have twins)
    for (size_t e0 = 0; e0 < h.size(); e0++) {
      if (h[e0].twin >= 0) continue;
      const int b = (int)faces.size();
      faces.push_back(Face{-1, true});
      std::vector<int> bh;
      int i = (int)e0;
      do {
        const int t = (int)h.size();
        h.push_back(HE());
        bh.push_back(t);
        h[i].twin = t;
        h[t].twin = i;
        h[t].face = b;
        h[t].vertex = h[h[i].next].vertex;
        i = h[i].next;
        while (i != (int)e0 && h[i].twin >= 0) i = h[h[i].twin].next;
      } while (i != (int)e0);
      faces[b].he = bh.empty() ? -1 : bh[0];
      const size_t deg = bh.size();
      for (size_t q = 0; q < deg; q++) h[bh[q]].next = bh[(q + deg - 1) % deg];
    }
    for (size_t v = 0; v < vhe.size(); v++) vhe[v] = h[h[vhe[v]].twin].next;
    if (positions.size() != vhe.size()) { err = "mesh has unused vertices"; return false; }
    vpos.resize(vhe.size());
    {
      int k = 0;
      for (auto& kv : index_to_vertex) vpos[kv.second] = positions[k++];
    }
    vnrm.resize(vhe.size());
    for (size_t v = 0; v < vhe.size(); v++) vnrm[v] = vertex_normal((int)v);
    return true;
  }
  bool vertex_on_boundary(int v) const {
    int e = vhe[v];
    do {
      if (faces[h[e].face].boundary) return true;
      e = h[h[e].twin].next;
    } while (e != vhe[v]);
    return false;
  }
  V3 vertex_normal(int v) const {   // Vertex::computeNormal (halfEdgeMesh.h:492-515)
    V3 nrm(0., 0., 0.);
    const V3 pi = vpos[v];
    int e = vhe[v];
    const bool bnd = vertex_on_boundary(v);
    do {
      const V3 pj = vpos[h[h[e].next].vertex];
      const V3 pk = vpos[h[h[h[e].next].next].vertex];
      nrm += cross(pj - pi, pk - pi);
      e = bnd ? h[h[e].next].twin : h[h[e].twin].next;
    } while (e != vhe[v]);
    nrm.normalize();
    return nrm;
  }
};

// ---------------------------------------------------------------------------------------------
// Camera (camera.cpp:29-147); double state like the reference's Camera.
struct Camera {
  size_t sw = 0, sh = 0;
  double nclip = 0, fclip = 0, hfov = 0, vfov = 0, ar = 0, screen_dist = 0;
  V3 target, pos;
  double phi = 0, theta = 0, r = 0, minr = 0, maxr = 0;
  V3 c2w[3];   // columns
  double w2c[3][3];   // (row, col)

  void configure(float h, float v, float nc, float fc, size_t w, size_t hh) {
    sw = w; sh = hh;
    nclip = nc; fclip = fc;
    hfov = h; vfov = v;
    const double ar1 = tan(radians(hfov) / 2) / tan(radians(vfov) / 2);
    ar = static_cast<double>(sw) / sh;
    if (ar1 < ar) hfov = 2 * degrees(atan(tan(radians(vfov) / 2) * ar));
    else if (ar1 > ar) vfov = 2 * degrees(atan(tan(radians(hfov) / 2) / ar));
    screen_dist = ((double)sh) / (2.0 * tan(radians(vfov) / 2));
  }
  void place(V3 t, double ph, double th, double rr, double mn, double mx) {
    const double r_ = std::min(std::max(rr, mn), mx);
    const double phi_ = (sin(ph) == 0) ? (ph + kEpsF) : ph;
    target = t; phi = phi_; theta = th; r = r_; minr = mn; maxr = mx;
    compute_position();
  }
  void set_screen_size(size_t w, size_t hh) {
    sw = w; sh = hh;
    ar = 1.0 * sw / sh;
    hfov = 2 * degrees(atan(((double)sw) / (2 * screen_dist)));
    vfov = 2 * degrees(atan(((double)sh) / (2 * screen_dist)));
  }
  void compute_position() {
    double sp = sin(phi);
    if (sp == 0) { phi += kEpsF; sp = sin(phi); }
    const V3 dir(r * sp * sin(theta), r * cos(phi), r * sp * cos(theta));
    pos = target + dir;
    const V3 upv(0, sp > 0 ? 1 : -1, 0);
    V3 sx = cross(upv, dir);
    sx.normalize();
    V3 sy = cross(dir, sx);
    sy.normalize();
    c2w[0] = sx; c2w[1] = sy; c2w[2] = dir.unit();
    // Matrix3x3::inv (matrix3x3.cpp:129-140): adjugate * (1 / det)
    auto A = [&](int i, int j) { const V3& c = c2w[j]; return i == 0 ? c.x : i == 1 ? c.y : c.z; };
    double B[3][3];
    B[0][0] = -A(1, 2) * A(2, 1) + A(1, 1) * A(2, 2); B[0][1] = A(0, 2) * A(2, 1) - A(0, 1) * A(2, 2); B[0][2] = -A(0, 2) * A(1, 1) + A(0, 1) * A(1, 2);
    B[1][0] = A(1, 2) * A(2, 0) - A(1, 0) * A(2, 2); B[1][1] = -A(0, 2) * A(2, 0) + A(0, 0) * A(2, 2); B[1][2] = A(0, 2) * A(1, 0) - A(0, 0) * A(1, 2);
    B[2][0] = -A(1, 1) * A(2, 0) + A(1, 0) * A(2, 1); B[2][1] = A(0, 1) * A(2, 0) - A(0, 0) * A(2, 1); B[2][2] = -A(0, 1) * A(1, 0) + A(0, 0) * A(1, 1);
    const double det = -A(0, 2) * A(1, 1) * A(2, 0) + A(0, 1) * A(1, 2) * A(2, 0) + A(0, 2) * A(1, 0) * A(2, 1) -
                       A(0, 0) * A(1, 2) * A(2, 1) - A(0, 1) * A(1, 0) * A(2, 2) + A(0, 0) * A(1, 1) * A(2, 2);   // :31-37
    const double rx = 1. / det;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) w2c[i][j] = B[i][j] * rx;
  }
};

void set3(double* d, const V3& v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }

}  // namespace

bdpt_scene_desc DaeScene::desc() const {
  bdpt_scene_desc d;
  memset(&d, 0, sizeof d);
  d.nprim = (int32_t)prim_type.size();
  d.prim_type = prim_type.data();
  d.prim_geom = prim_geom.data();
  d.prim_mat = prim_mat.data();
  d.nmat = (int32_t)mats.size();
  d.mats = mats.data();
  d.nlight = (int32_t)lights.size();
  d.lights = lights.data();
  d.camera = cam;
  return d;
}

int load_dae(const char* path, int width, int height, DaeScene& out, std::string& err) {
  FILE* f = fopen(path, "rb");
  if (!f) { err = std::string("cannot open ") + path; return BDPT_E_INVALID; }
  std::string src;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) src.append(buf, n);
  fclose(f);
  XEl doc;
  if (!parse_xml(src, doc, err)) { err = std::string(path) + ": XML: " + err; return BDPT_E_INVALID; }
  XEl* root = doc.first("COLLADA");
  if (!root) { err = std::string(path) + ": not a COLLADA file"; return BDPT_E_INVALID; }
  Parser P;
  if (!P.load(root)) { err = std::string(path) + ": " + P.err; return BDPT_E_INVALID; }

  // Application::init / load (application.cpp:52-104, 228-304)
  size_t sw = 800, sh = 600;
  Camera cam;
  cam.configure(50, 35, 0.01f, 100, sw, sh);
  V3 c_pos, c_dir;
  struct Obj { bool sphere; const Node* node; V3 center; double radius; HalfedgeMesh mesh; };
  std::vector<Obj> objs;
  out = DaeScene();
  for (const Node& nd : P.nodes) {
    const M4& T = nd.T;
    if (nd.type == I_CAMERA) {
      c_pos = (T * V4(c_pos, 1)).to3D();
      c_dir = (T * V4(nd.view_dir, 1)).to3D().unit();
      cam.configure(nd.hfov, nd.vfov, nd.nclip, nd.fclip, sw, sh);
    } else if (nd.type == I_LIGHT) {
      bdpt_light l;
      memset(&l, 0, sizeof l);
      set3(l.radiance, nd.spectrum);
      if (nd.lk == LK_AREA) {   // GLScene::AreaLight (gl_scene/area_light.h:14-27), light.cpp:199-203
        const V3 p = (T * V4(nd.lpos, 1)).to3D();
        V3 dir = (T * V4(nd.ldir, 1)).to3D() - p;
        dir.normalize();
        const V3 dy = nd.lup, dx = cross(nd.lup, nd.ldir);
        const V3 dimx = (T * V4(dx, 1)).to3D() - p, dimy = (T * V4(dy, 1)).to3D() - p;
        l.type = BDPT_LIGHT_AREA;
        set3(l.position, p);
        set3(l.direction, dir);
        set3(l.dim_x, dimx);
        set3(l.dim_y, dimy);
        l.area = dimx.norm() * dimy.norm();
      } else if (nd.lk == LK_POINT) {   // gl_scene/point_light.h:17-22
        l.type = BDPT_LIGHT_POINT;
        set3(l.position, (T * V4(nd.lpos, 1)).to3D());
      } else if (nd.lk == LK_AMBIENT) {   // gl_scene/ambient_light.h:19-23: InfiniteHemisphereLight
        l.type = BDPT_LIGHT_HEMISPHERE;
      } else if (nd.lk == LK_DIRECTIONAL) {
        // gl_scene/directional_light.h:14-19 (a w = 1 transform of the COLLADA direction, negated,
        // normalised), then DirectionalLight's dirToLight = -direction.unit() (light.cpp:11-15)
        V3 d = (T * V4(nd.ldir, 1)).to3D();
        d = V3(-d.x, -d.y, -d.z);
        d.normalize();
        const V3 u = d.unit();
        l.type = BDPT_LIGHT_DIRECTIONAL;
        set3(l.direction, V3(-u.x, -u.y, -u.z));
      } else {
        l.type = BDPT_LIGHT_OTHER;   // spot
      }
      out.lights.push_back(l);
    } else if (nd.type == I_SPHERE) {   // application.cpp:345-351, gl_scene/sphere.cpp:12-20
      Obj o;
      o.sphere = true;
      o.node = &nd;
      o.center = (T * V4(0, 0, 0, 1)).projectTo3D();
      const double scale = (T * V4(1, 0, 0, 0)).to3D().norm();
      o.radius = nd.radius * scale;
      objs.push_back(std::move(o));
    } else if (nd.type == I_MESH) {   // gl_scene/mesh.cpp:22-43
      Obj o;
      o.sphere = false;
      o.node = &nd;
      std::vector<V3> vs = nd.verts;
      for (auto& v : vs) v = (T * V4(v, 1)).projectTo3D();
      if (!o.mesh.build(nd.polys, vs, err)) { err = std::string(path) + ": " + err; return BDPT_E_INVALID; }
      objs.push_back(std::move(o));
    }
  }
  // scene bbox (gl_scene/scene.cpp:10-16) -> camera placement
  const double inf = INFINITY;
  V3 bmin(inf, inf, inf), bmax(-inf, -inf, -inf);
  auto expand = [&](const V3& lo, const V3& hi) {
    bmin = V3(std::min(bmin.x, lo.x), std::min(bmin.y, lo.y), std::min(bmin.z, lo.z));
    bmax = V3(std::max(bmax.x, hi.x), std::max(bmax.y, hi.y), std::max(bmax.z, hi.z));
  };
  for (const Obj& o : objs) {
    if (o.sphere) {
      expand(V3(o.center.x - o.radius, o.center.y - o.radius, o.center.z - o.radius),
             V3(o.center.x + o.radius, o.center.y + o.radius, o.center.z + o.radius));
    } else {
      V3 lo(inf, inf, inf), hi(-inf, -inf, -inf);
      for (const V3& p : o.mesh.vpos) {
        lo = V3(std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z));
        hi = V3(std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z));
      }
      expand(lo, hi);
    }
  }
  if (!objs.empty() && bmax.x >= bmin.x) {
    const V3 ext = bmax - bmin;
    const V3 target = (bmin + bmax) / 2;
    const double canonical = ext.norm() / 2 * 1.5;
    cam.place(target, acos(c_dir.y), atan2(c_dir.x, c_dir.z), canonical * 2, canonical / 10.0, canonical * 20.0);
  }
  if (width > 0 && height > 0) cam.set_screen_size((size_t)width, (size_t)height);

  // static scene: primitives in object order (object.cpp:16-56, raytraced_renderer.cpp:350-374);
  // every instance_material (and every default) is its own BSDF
  auto add_mat = [&](const Node& nd) {
    bdpt_material m;
    memset(&m, 0, sizeof m);
    if (nd.has_mat) {
      m.type = nd.mat.type;
      set3(m.a, nd.mat.a);
      set3(m.b, nd.mat.b);
      m.ior = nd.mat.ior;
      m.roughness = nd.mat.roughness;
    } else {
      m.type = BDPT_MAT_DIFFUSE;
      set3(m.a, V3(0.5f, 0.5f, 0.5f));
    }
    out.mats.push_back(m);
    return (int32_t)out.mats.size() - 1;
  };
  for (const Obj& o : objs) {
    const int32_t mid = add_mat(*o.node);
    if (o.sphere) {
      double g[18] = {0};
      g[0] = o.center.x; g[1] = o.center.y; g[2] = o.center.z; g[3] = o.radius;
      out.prim_type.push_back(BDPT_PRIM_SPHERE);
      out.prim_geom.insert(out.prim_geom.end(), g, g + 18);
      out.prim_mat.push_back(mid);
      out.n_sphs++;
      continue;
    }
    const HalfedgeMesh& M = o.mesh;
    for (size_t fi = 0; fi < M.faces.size(); fi++) {
      if (M.faces[fi].boundary) continue;
      const int e = M.faces[fi].he;
      const int v[3] = {M.h[e].vertex, M.h[M.h[e].next].vertex, M.h[M.h[M.h[e].next].next].vertex};
      double g[18];
      for (int k = 0; k < 3; k++) {
        g[3 * k] = M.vpos[v[k]].x; g[3 * k + 1] = M.vpos[v[k]].y; g[3 * k + 2] = M.vpos[v[k]].z;
        g[9 + 3 * k] = M.vnrm[v[k]].x; g[10 + 3 * k] = M.vnrm[v[k]].y; g[11 + 3 * k] = M.vnrm[v[k]].z;
      }
      out.prim_type.push_back(BDPT_PRIM_TRIANGLE);
      out.prim_geom.insert(out.prim_geom.end(), g, g + 18);
      out.prim_mat.push_back(mid);
      out.n_tris++;
    }
  }
  // camera for the ABI (bdpt_camera: c2w / w2c column-major)
  memset(&out.cam, 0, sizeof out.cam);
  set3(out.cam.pos, cam.pos);
  for (int c = 0; c < 3; c++) {
    out.cam.c2w[3 * c] = cam.c2w[c].x;
    out.cam.c2w[3 * c + 1] = cam.c2w[c].y;
    out.cam.c2w[3 * c + 2] = cam.c2w[c].z;
    for (int r = 0; r < 3; r++) out.cam.w2c[3 * c + r] = cam.w2c[r][c];
  }
  out.cam.hfov_deg = cam.hfov;
  out.cam.vfov_deg = cam.vfov;
  out.cam.nclip = cam.nclip;
  out.cam.fclip = cam.fclip;
  set3(out.target, cam.target);
  out.phi = cam.phi;
  out.theta = cam.theta;
  out.r = cam.r;
  out.ar = cam.ar;
  out.screen_dist = cam.screen_dist;
  out.screen_w = (int)cam.sw;
  out.screen_h = (int)cam.sh;
  return BDPT_OK;
}

int dump_scene_json(const DaeScene& s, const char* path, std::string& err) {
  FILE* f = fopen(path, "w");
  if (!f) { err = std::string("cannot write ") + path; return BDPT_E_INVALID; }
  auto v3 = [&](const double* v) { fprintf(f, "[%.17g, %.17g, %.17g]", v[0], v[1], v[2]); };
  fprintf(f, "{\n\"source\": \"bdpt_amd dae_loader\",\n\"camera\": {\"pos\": ");
  v3(s.cam.pos);
  fprintf(f, ", \"target\": ");
  v3(s.target);
  fprintf(f, ", \"c2w_cols\": [");
  for (int c = 0; c < 3; c++) { if (c) fprintf(f, ","); v3(s.cam.c2w + 3 * c); }
  fprintf(f, "], \"w2c_cols\": [");
  for (int c = 0; c < 3; c++) { if (c) fprintf(f, ","); v3(s.cam.w2c + 3 * c); }
  fprintf(f, "], \"hFov\": %.17g, \"vFov\": %.17g, \"ar\": %.17g, \"nClip\": %.17g, \"fClip\": %.17g, "
             "\"phi\": %.17g, \"theta\": %.17g, \"r\": %.17g, \"screenW\": %d, \"screenH\": %d, \"screenDist\": %.17g},\n",
          s.cam.hfov_deg, s.cam.vfov_deg, s.ar, s.cam.nclip, s.cam.fclip, s.phi, s.theta, s.r, s.screen_w, s.screen_h,
          s.screen_dist);
  fprintf(f, "\"lights\": [");
  for (size_t i = 0; i < s.lights.size(); i++) {
    const bdpt_light& l = s.lights[i];
    fprintf(f, "%s\n  ", i ? "," : "");
    if (l.type == BDPT_LIGHT_AREA) {
      fprintf(f, "{\"type\": \"area\", \"radiance\": "); v3(l.radiance);
      fprintf(f, ", \"position\": "); v3(l.position);
      fprintf(f, ", \"direction\": "); v3(l.direction);
      fprintf(f, ", \"dim_x\": "); v3(l.dim_x);
      fprintf(f, ", \"dim_y\": "); v3(l.dim_y);
      fprintf(f, ", \"area\": %.17g}", l.area);
    } else if (l.type == BDPT_LIGHT_POINT) {
      fprintf(f, "{\"type\": \"point\", \"radiance\": "); v3(l.radiance);
      fprintf(f, ", \"position\": "); v3(l.position);
      fprintf(f, "}");
    } else if (l.type == BDPT_LIGHT_HEMISPHERE) {
      fprintf(f, "{\"type\": \"hemisphere\", \"radiance\": "); v3(l.radiance);
      fprintf(f, "}");
    } else if (l.type == BDPT_LIGHT_DIRECTIONAL) {
      fprintf(f, "{\"type\": \"directional\", \"radiance\": "); v3(l.radiance);
      fprintf(f, ", \"direction\": "); v3(l.direction);
      fprintf(f, "}");
    } else {
      fprintf(f, "{\"type\": \"unsupported\"}");
    }
  }
  fprintf(f, "],\n\"materials\": [");
  for (size_t i = 0; i < s.mats.size(); i++) {
    const bdpt_material& m = s.mats[i];
    fprintf(f, "%s\n  ", i ? "," : "");
    switch (m.type) {
      case BDPT_MAT_DIFFUSE: fprintf(f, "{\"type\": \"diffuse\", \"reflectance\": "); v3(m.a); fprintf(f, "}"); break;
      case BDPT_MAT_EMISSION: fprintf(f, "{\"type\": \"emission\", \"radiance\": "); v3(m.a); fprintf(f, "}"); break;
      case BDPT_MAT_MIRROR: fprintf(f, "{\"type\": \"mirror\", \"reflectance\": "); v3(m.a); fprintf(f, "}"); break;
      case BDPT_MAT_GLASS:
        fprintf(f, "{\"type\": \"glass\", \"reflectance\": "); v3(m.a);
        fprintf(f, ", \"transmittance\": "); v3(m.b);
        fprintf(f, ", \"roughness\": %.17g, \"ior\": %.17g}", m.roughness, m.ior);
        break;
      case BDPT_MAT_REFRACTION:
        fprintf(f, "{\"type\": \"refraction\", \"transmittance\": "); v3(m.b);
        fprintf(f, ", \"roughness\": %.17g, \"ior\": %.17g}", m.roughness, m.ior);
        break;
      default:
        fprintf(f, "{\"type\": \"microfacet\", \"eta\": "); v3(m.a);
        fprintf(f, ", \"k\": "); v3(m.b);
        fprintf(f, ", \"alpha\": %.17g}", m.roughness);
        break;
    }
  }
  fprintf(f, "],\n\"prim_order\": [");
  int nt = 0, ns = 0;
  for (size_t i = 0; i < s.prim_type.size(); i++)
    fprintf(f, "%s[\"%s\",%d]", i ? "," : "", s.prim_type[i] == BDPT_PRIM_SPHERE ? "s" : "t",
            s.prim_type[i] == BDPT_PRIM_SPHERE ? ns++ : nt++);
  fprintf(f, "],\n\"triangles\": [");
  bool first = true;
  for (size_t i = 0; i < s.prim_type.size(); i++) {
    if (s.prim_type[i] != BDPT_PRIM_TRIANGLE) continue;
    const double* g = &s.prim_geom[18 * i];
    fprintf(f, "%s\n  [", first ? "" : ",");
    first = false;
    for (int k = 0; k < 6; k++) { v3(g + 3 * k); fprintf(f, ","); }
    fprintf(f, "%d]", s.prim_mat[i]);
  }
  fprintf(f, "],\n\"spheres\": [");
  first = true;
  for (size_t i = 0; i < s.prim_type.size(); i++) {
    if (s.prim_type[i] != BDPT_PRIM_SPHERE) continue;
    const double* g = &s.prim_geom[18 * i];
    fprintf(f, "%s\n  [", first ? "" : ",");
    first = false;
    v3(g);
    fprintf(f, ",%.17g,%d]", g[3], s.prim_mat[i]);
  }
  fprintf(f, "]\n}\n");
  fclose(f);
  return BDPT_OK;
}

}  // namespace bdpt

// ---------------------------------------------------------------------------------------------
// C-ABI (include/bdpt/bdpt.h)
extern "C" {

struct bdpt_dae {
  bdpt::DaeScene s;
};

int bdpt_dae_load(const char* path, int32_t width, int32_t height, bdpt_dae** out) {
  if (!path || !out) { bdpt::g_err = "null argument"; return BDPT_E_INVALID; }
  *out = nullptr;
  bdpt_dae* d = new bdpt_dae();
  std::string err;
  int rc = bdpt::load_dae(path, width, height, d->s, err);
  if (rc) {
    bdpt::g_err = err;
    delete d;
    return rc;
  }
  *out = d;
  return BDPT_OK;
}

int bdpt_dae_get_desc(const bdpt_dae* d, bdpt_scene_desc* out) {
  if (!d || !out) { bdpt::g_err = "null argument"; return BDPT_E_INVALID; }
  *out = d->s.desc();
  return BDPT_OK;
}

int bdpt_dae_dump_json(const bdpt_dae* d, const char* path) {
  if (!d || !path) { bdpt::g_err = "null argument"; return BDPT_E_INVALID; }
  std::string err;
  int rc = bdpt::dump_scene_json(d->s, path, err);
  if (rc) bdpt::g_err = err;
  return rc;
}

void bdpt_dae_free(bdpt_dae* d) { delete d; }

int bdpt_camera_load_settings(const char* path, bdpt_camera* cam) {
  return bdpt_camera_load_settings_lens(path, cam, nullptr, nullptr);
}

int bdpt_camera_load_settings_lens(const char* path, bdpt_camera* cam, double* focal_distance, double* lens_radius) {
  if (!path || !cam) { bdpt::g_err = "null argument"; return BDPT_E_INVALID; }
  std::ifstream file(path);
  if (!file.is_open()) { bdpt::g_err = std::string("cannot open camera settings ") + path; return BDPT_E_INVALID; }
  // Camera::load_settings (camera.cpp:172-186): the same extractions into the same types, so a
  // short or malformed file leaves / zeroes the same members the reference's would
  double hFov = cam->hfov_deg, vFov = cam->vfov_deg, ar = 0, nClip = cam->nclip, fClip = cam->fclip;
  double pos[3] = {cam->pos[0], cam->pos[1], cam->pos[2]}, target[3] = {0, 0, 0};
  double phi = 0, theta = 0, r = 0, minR = 0, maxR = 0;
  double c2w[3][3];   // (row, col)
  for (int i = 0; i < 9; ++i) c2w[i / 3][i % 3] = cam->c2w[3 * (i % 3) + i / 3];
  size_t screenW = 0, screenH = 0;
  double screenDist = 0, focalDistance = focal_distance ? *focal_distance : 0,
         lensRadius = lens_radius ? *lens_radius : 0;
  file >> hFov >> vFov >> ar >> nClip >> fClip;
  for (int i = 0; i < 3; ++i) file >> pos[i];
  for (int i = 0; i < 3; ++i) file >> target[i];
  file >> phi >> theta >> r >> minR >> maxR;
  for (int i = 0; i < 9; ++i) file >> c2w[i / 3][i % 3];
  file >> screenW >> screenH >> screenDist;
  file >> focalDistance >> lensRadius;
  cam->hfov_deg = hFov;
  cam->vfov_deg = vFov;
  cam->nclip = nClip;
  cam->fclip = fClip;
  for (int i = 0; i < 3; ++i) cam->pos[i] = pos[i];
  for (int i = 0; i < 9; ++i) cam->c2w[3 * (i % 3) + i / 3] = c2w[i / 3][i % 3];   // column-major
  if (focal_distance) *focal_distance = focalDistance;
  if (lens_radius) *lens_radius = lensRadius;
  fprintf(stderr, "[Camera] Loaded settings from %s\n", path);
  return BDPT_OK;
}

}  // extern "C"
