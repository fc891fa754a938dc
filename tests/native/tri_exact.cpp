// Test-only: bdpt::tri_test (with its exact quotient-sign / > 1 early-outs) against the plain Möller–Trumbore
// predicate it must reproduce (three correctly rounded divisions, then the reference's
// comparisons, triangle.cpp:57-95), on random and on near-boundary cases (b1 + b2 close to 1,
// t close to tmax, tiny and huge denominators). Prints the number of mismatches.
#include <cmath>
#include <cstdio>
#include <random>

#include "bdpt_core.h"

using namespace bdpt;

static bool plain(const float4 g0, const float4 g1, const float4 g2, f3 o, f3 d, float tmin, float tmax,
                  float* t_out, float* b1_out, float* b2_out) {
  f3 p0 = mk3(g0.x, g0.y, g0.z), e1 = mk3(g0.w, g1.x, g1.y), e2 = mk3(g1.z, g1.w, g2.x);
  f3 s = sub(o, p0), s1 = cross(d, e2);
  float denom = dot(s1, e1), n1 = dot(s1, s);
  f3 s2 = cross(s, e1);
  float n2 = dot(s2, d), nt = dot(s2, e2);
  float t = nt / denom, b1 = n1 / denom, b2 = n2 / denom;
  *t_out = t; *b1_out = b1; *b2_out = b2;
  return t >= tmin && t <= tmax && b1 >= 0 && b2 >= 0 && b1 + b2 <= 1;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<float> U(-1.0f, 1.0f);
  long bad = 0, hits = 0;
  for (long k = 0; k < n; k++) {
    const int kind = (int)(k % 4);
    const float sc = kind == 3 ? std::ldexp(1.0f, (int)(k % 60) - 30) : 1.0f;   // tiny / huge triangles
    f3 p0 = mk3(U(rng), U(rng), U(rng)), e1 = muls(mk3(U(rng), U(rng), U(rng)), sc),
       e2 = muls(mk3(U(rng), U(rng), U(rng)), sc);
    f3 o = mk3(U(rng) * 3, U(rng) * 3, U(rng) * 3);
    // aim at a point of the triangle's plane: b1 + b2 near 1 (kind 1) or anywhere (kind 0)
    float a = 0.5f + 0.5f * U(rng), b = 0.5f + 0.5f * U(rng);
    if (kind == 1) { a = 0.5f + 0.5f * U(rng); b = 1.0f - a + U(rng) * 1e-6f; }
    f3 target = add(p0, add(muls(e1, a), muls(e2, b)));
    f3 d = normalize(sub(target, o));
    float tmax = kind == 2 ? norm(sub(target, o)) * (1.0f + U(rng) * 1e-6f) : (k % 7 == 0 ? INFINITY : 10.0f);
    const float tmin = (k % 11 == 0) ? -1.0f : 1e-5f;
    float4 g0, g1, g2;
    g0.x = p0.x; g0.y = p0.y; g0.z = p0.z; g0.w = e1.x;
    g1.x = e1.y; g1.y = e1.z; g1.z = e2.x; g1.w = e2.y;
    g2.x = e2.z; g2.y = 0; g2.z = 0; g2.w = 0;
    float t1 = 0, u1 = 0, v1 = 0, t2 = 0, u2 = 0, v2 = 0;
    const bool r1 = tri_test(g0, g1, g2, o, d, tmin, tmax, &t1, &u1, &v1);
    const bool r2 = plain(g0, g1, g2, o, d, tmin, tmax, &t2, &u2, &v2);
    if (r2) hits++;
    if (r1 != r2 || (r1 && (t1 != t2 || u1 != u2 || v1 != v2))) {
      if (bad < 5) std::printf("mismatch k=%ld kind=%d: %d vs %d t %a %a\n", k, kind, r1, r2, t1, t2);
      bad++;
    }
  }
  std::printf("cases %ld hits %ld mismatches %ld\n", n, hits, bad);
  return bad != 0;
}
