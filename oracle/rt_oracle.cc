// oracle/rt_oracle.cc -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the
// reference's render path, used by tests/ (and bench.py's cpu_baseline leg)
// as the CHECKER.  Never linked into, or called by, the product
// (librtow.so / the CLIs); the product fails loudly without its HIP build.
//
// Two modes, both written from the reference's semantics (not copied):
//
//  * reference mode (rto_reference_render): single-threaded fp64 restatement
//    of src/cpu -- one std::mt19937 (seed 5489) + uniform_real_distribution
//    <double> stream shared by scene construction and rendering
//    (src/cpu/rtweekend.h:27-31), rejection sampling, recursive ray_color,
//    closed hit interval, g++ argument evaluation order.  Pinned: byte-
//    identical PPM to the reference binary built from /root/reference by
//    oracle/Makefile (tests/golden/ref_c0_*.ppm.gz, SHA-256 736ab8c6...).
//
//  * kernel mode (rto_kernel_render): fp32 restatement of the algorithm the
//    HIP kernel runs (DESIGN.md "Kernel algorithm"): normalised directions,
//    expanded quadratic, pcg4d counter RNG, closed-form sampling.  Written
//    independently of ray-tracing-in-one-weekend_amd/csrc/rt_render.hip from
//    the same specification; with -ffp-contract=off and explicit fmaf it is
//    the bit-exact per-pixel parity partner of the GPU kernel.
//
// Reference anchors are cited per function (paths under /root/reference).
#include "rt_oracle.h"
#include "rt_turn_table.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <cstdlib>
#include <vector>

namespace {

// =====================================================================
// reference mode (fp64)
// =====================================================================

struct d3 {
  double x, y, z;
};
inline d3 operator+(d3 a, d3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline d3 operator-(d3 a) { return {-a.x, -a.y, -a.z}; }
inline d3 operator*(d3 a, d3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline d3 operator*(double t, d3 v) { return {t * v.x, t * v.y, t * v.z}; }  // vec3.h:83-85
inline d3 operator/(d3 v, double t) { return (1 / t) * v; }                    // vec3.h:91
inline double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline double len2(d3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline d3 cross(d3 u, d3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
inline d3 unit(d3 v) { return v / std::sqrt(len2(v)); }  // vec3.h:103

// rtweekend.h:27-36
struct rng64 {
  std::mt19937 gen;
  std::uniform_real_distribution<double> dist{0.0, 1.0};
  double operator()() { return dist(gen); }
  double operator()(double lo, double hi) { return lo + (hi - lo) * (*this)(); }
};

// vec3.h:105-112 random_in_unit_sphere; vec3::random(-1,1) draws z,y,x (g++)
d3 in_unit_sphere(rng64 &r) {
  while (true) {
    d3 p;
    p.z = r(-1, 1);
    p.y = r(-1, 1);
    p.x = r(-1, 1);
    if (len2(p) >= 1) continue;
    return p;
  }
}

// vec3.h:133-140 random_in_unit_disk; vec3(rd(-1,1), rd(-1,1), 0): y drawn first
d3 in_unit_disk(rng64 &r) {
  while (true) {
    d3 p;
    p.z = 0;
    p.y = r(-1, 1);
    p.x = r(-1, 1);
    if (len2(p) >= 1) continue;
    return p;
  }
}

struct dsphere {
  d3 c;
  double r;
  int kind;
  d3 albedo;
  double param;
};

struct dhit {
  d3 p, n;
  double t;
  bool front;
  int obj;
};

// sphere.h:24-51
bool sphere_hit(const dsphere &s, d3 o, d3 d, double tmin, double tmax, dhit &rec) {
  d3 oc = o - s.c;
  double a = len2(d);
  double half_b = dot(oc, d);
  double c = len2(oc) - s.r * s.r;
  double disc = half_b * half_b - a * c;
  if (disc < 0) return false;
  double sq = std::sqrt(disc);
  double root = (-half_b - sq) / a;
  if (root < tmin || tmax < root) {
    root = (-half_b + sq) / a;
    if (root < tmin || tmax < root) return false;
  }
  rec.t = root;
  rec.p = o + root * d;                   // ray.h at()
  d3 outward = (rec.p - s.c) / s.r;
  rec.front = dot(d, outward) < 0;        // hittable.h:16-19
  rec.n = rec.front ? outward : -outward;
  return true;
}

unsigned long long g_last_trapped = 0;  // rto_reference_trapped
unsigned long long g_last_capped = 0;   // rto_reference_capped
std::atomic<unsigned long long> g_kcapped{0};  // rto_kernel_capped
// kernel mode, attribution only (rto_kernel_attrib): spurious-root skips,
// first hits on the inside of a sealed sphere, and those of them whose ray
// had just been moved on by a skip
std::atomic<unsigned long long> g_skips{0}, g_inner{0}, g_inner_after_skip{0};
// ... and the first 4096 entries: (sphere entered, previous segment's sphere, depth, t_min * 1e6)
std::atomic<unsigned> g_ev_n{0};
long long g_ev[4096][4];

struct dworld {
  std::vector<dsphere> s;
  unsigned long long calls = 0;
  // attribution only (rto_reference_trapped): the sealed spheres of the
  // opaque-inside rule (sealed_of on the fp64 scene) and the segments the
  // reference traces after a path's first hit on the inside of one
  std::vector<uint8_t> sealed;
  unsigned long long trapped = 0;
  unsigned long long capped = 0;  // paths ended at the depth cap (rto_reference_capped)
  // hittable_list.h:28-43
  bool hit(d3 o, d3 d, double tmin, double tmax, dhit &rec) {
    ++calls;
    dhit tmp;
    bool any = false;
    double closest = tmax;
    for (size_t i = 0; i < s.size(); ++i) {
      if (sphere_hit(s[i], o, d, tmin, closest, tmp)) {
        any = true;
        closest = tmp.t;
        rec = tmp;
        rec.obj = (int)i;
      }
    }
    return any;
  }
};

d3 reflect(d3 v, d3 n) { return v - (2 * dot(v, n)) * n; }  // vec3.h:122

d3 refract(d3 uv, d3 n, double eta) {  // vec3.h:126-131
  double cos_theta = std::fmin(dot(-uv, n), 1.0);
  d3 perp = eta * (uv + cos_theta * n);
  d3 par = (-std::sqrt(std::fabs(1.0 - len2(perp)))) * n;
  return perp + par;
}

double reflectance(double cosine, double ref_idx) {  // material.h:82-87
  double r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  return r0 + (1 - r0) * std::pow((1 - cosine), 5);
}

// material.h scatter functions; returns false when absorbed
bool scatter(const dsphere &m, d3 din, const dhit &rec, rng64 &r, d3 &att, d3 &dout) {
  if (m.kind == RT_LAMBERTIAN) {  // material.h:19-30
    d3 dir = rec.n + unit(in_unit_sphere(r));
    const double s = 1e-8;
    if (std::fabs(dir.x) < s && std::fabs(dir.y) < s && std::fabs(dir.z) < s) dir = rec.n;
    dout = dir;
    att = m.albedo;
    return true;
  }
  if (m.kind == RT_METAL) {  // material.h:40-46
    d3 refl = reflect(unit(din), rec.n);
    dout = refl + m.param * in_unit_sphere(r);
    att = m.albedo;
    return dot(dout, rec.n) > 0;
  }
  // dielectric, material.h:57-76
  att = {1.0, 1.0, 1.0};
  double ratio = rec.front ? (1.0 / m.param) : m.param;
  d3 ud = unit(din);
  double cos_t = std::fmin(dot(-ud, rec.n), 1.0);
  double sin_t = std::sqrt(1.0 - cos_t * cos_t);
  bool cannot = ratio * sin_t > 1.0;
  if (cannot || reflectance(cos_t, ratio) > r())
    dout = reflect(ud, rec.n);
  else
    dout = refract(ud, rec.n, ratio);
  return true;
}

// main.cc:12-30 (recursive); trapped: the path has hit a sealed sphere from
// inside (counted in w.trapped, nothing else changes)
d3 ray_color(d3 o, d3 d, dworld &w, rng64 &r, int depth, bool trapped = false) {
  if (depth <= 0) {
    ++w.capped;
    return {0, 0, 0};
  }
  dhit rec;
  if (trapped) ++w.trapped;
  if (w.hit(o, d, 0.001, INFINITY, rec)) {
    d3 att, dir;
    const bool in = trapped || (!w.sealed.empty() && w.sealed[rec.obj] && !rec.front);
    if (scatter(w.s[rec.obj], d, rec, r, att, dir)) return att * ray_color(rec.p, dir, w, r, depth - 1, in);
    return {0, 0, 0};
  }
  d3 ud = unit(d);
  double t = 0.5 * (ud.y + 1.0);
  return (1.0 - t) * d3{1.0, 1.0, 1.0} + t * d3{0.5, 0.7, 1.0};
}

// main.cc:32-76 random_scene, g++ draw order
void final_scene(rng64 &r, int half, std::vector<dsphere> &s) {
  s.push_back({{0, -1000, 0}, 1000, RT_LAMBERTIAN, {0.5, 0.5, 0.5}, 0});
  for (int a = -half; a < half; a++) {
    for (int b = -half; b < half; b++) {
      double choose = r();
      d3 c;
      c.y = 0.2;
      c.z = b + 0.9 * r();
      c.x = a + 0.9 * r();
      if (std::sqrt(len2(c - d3{4, 0.2, 0})) > 0.9) {
        if (choose < 0.8) {
          d3 rhs, lhs;
          rhs.z = r(); rhs.y = r(); rhs.x = r();
          lhs.z = r(); lhs.y = r(); lhs.x = r();
          s.push_back({c, 0.2, RT_LAMBERTIAN, lhs * rhs, 0});
        } else if (choose < 0.95) {
          d3 alb;
          alb.z = r(0.5, 1); alb.y = r(0.5, 1); alb.x = r(0.5, 1);
          double fuzz = r(0, 0.5);
          s.push_back({c, 0.2, RT_METAL, alb, fuzz < 1 ? fuzz : 1});
        } else {
          s.push_back({c, 0.2, RT_DIELECTRIC, {1, 1, 1}, 1.5});
        }
      }
    }
  }
  s.push_back({{0, 1, 0}, 1.0, RT_DIELECTRIC, {1, 1, 1}, 1.5});
  s.push_back({{-4, 1, 0}, 1.0, RT_LAMBERTIAN, {0.4, 0.2, 0.1}, 0});
  s.push_back({{4, 1, 0}, 1.0, RT_METAL, {0.7, 0.6, 0.5}, 0.0});
}

void five_scene(std::vector<dsphere> &s) {
  s.push_back({{0.0, -100.5, -1.0}, 100.0, RT_LAMBERTIAN, {0.8, 0.8, 0.0}, 0});
  s.push_back({{0.0, 0.0, -1.0}, 0.5, RT_LAMBERTIAN, {0.1, 0.2, 0.5}, 0});
  s.push_back({{-1.0, 0.0, -1.0}, 0.5, RT_DIELECTRIC, {1, 1, 1}, 1.5});
  s.push_back({{-1.0, 0.0, -1.0}, -0.4, RT_DIELECTRIC, {1, 1, 1}, 1.5});
  s.push_back({{1.0, 0.0, -1.0}, 0.5, RT_METAL, {0.8, 0.6, 0.2}, 0.0});
}

inline uint8_t tonemap(double v, double scale) {  // color.h:8-23
  double x = std::sqrt(scale * v);
  if (x < 0.0) x = 0.0;
  if (x > 0.999) x = 0.999;
  return (uint8_t)(int)(256 * x);
}

// =====================================================================
// kernel mode (fp32) -- the specification the HIP kernel implements
// =====================================================================

inline float fmaf_(float a, float b, float c) { return std::fmaf(a, b, c); }

// debug tracing of one sample (rto_trace): prints every segment and every
// candidate sphere (root, discriminant) -- test tooling only
FILE *g_trace = nullptr;
long g_trace_sample = -1;

struct u4 {
  uint32_t x, y, z, w;
};

// pcg4d, Jarzynski & Olano, JCGT 9(3) 2020
u4 pcg4d(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  uint32_t x = a * 1664525u + 1013904223u;
  uint32_t y = b * 1664525u + 1013904223u;
  uint32_t z = c * 1664525u + 1013904223u;
  uint32_t w = d * 1664525u + 1013904223u;
  x += y * w;
  y += z * x;
  z += x * y;
  w += y * z;
  x ^= x >> 16;
  y ^= y >> 16;
  z ^= z >> 16;
  w ^= w >> 16;
  x += y * w;
  y += z * x;
  z += x * y;
  w += y * z;
  return {x, y, z, w};
}

inline float unif(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

// the kernel's sin/cos of 2 pi u (rt_render.hip sincos_turn): the (cos, sin)
// table of include/rt_turn_table.h at i = floor(1024 u), rotated by the
// remainder d with cos d = 1 - d^2/2, sin d = d (1 - d^2/6)
const float *turn_table() {
  static const std::vector<float> tab = [] {
    std::vector<float> t(2 * RT_TURN_TABLE);
    rt_turn_table(t.data());
    return t;
  }();
  return tab.data();
}
void sincos_turn(float u, float &s, float &c) {
  const float t = u * (float)RT_TURN_TABLE;
  const float fl = std::floor(t);
  const float *e = turn_table() + 2 * (int)fl;
  const float d = (t - fl) * (6.28318530717958648f / (float)RT_TURN_TABLE);
  const float x2 = d * d;
  const float cd = fmaf_(x2, -0.5f, 1.0f);
  const float sd = d * fmaf_(x2, -0.166666667f, 1.0f);
  c = fmaf_(e[0], cd, -(e[1] * sd));
  s = fmaf_(e[1], cd, e[0] * sd);
}

// the kernel's radius of a uniform point in the unit ball (radius law of
// random_in_unit_sphere, vec3.h:105-112: CDF r^3): the largest of three
// uniforms -- the hash's z and w draws and the low bytes of x, y, z
float ball_radius(const u4 &r) {
  const uint32_t lo = ((r.x & 0xffu) << 24) | ((r.y & 0xffu) << 16) | ((r.z & 0xffu) << 8);
  return std::fmax(std::fmax(unif(r.z), unif(r.w)), unif(lo));
}

// sqrtf(max(x, 2^-96)): the kernel's sqrt_k (rt_render.hip) -- correctly
// rounded, argument clamped below
inline float sqrt_k(float x) { return std::sqrt(std::fmax(x, 0x1p-96f)); }

void unit_vec(float u1, float u2, float &x, float &y, float &z) {
  z = fmaf_(-2.0f, u1, 1.0f);
  float r = sqrt_k(fmaf_(-z, z, 1.0f));
  float s, c;
  sincos_turn(u2, s, c);
  x = r * c;
  y = r * s;
}

inline float dot3(float ax, float ay, float az, float bx, float by, float bz) {
  return fmaf_(az, bz, fmaf_(ay, by, ax * bx));
}

// the kernel's normalize3: integer-seeded inverse sqrt + 3 Newton steps;
// returns the length it divided by, l2 * r (|x| within a few ulp)
float normalize3(float &x, float &y, float &z) {
  const float l2 = dot3(x, y, z, x, y, z);
  uint32_t i;
  std::memcpy(&i, &l2, 4);
  i = 0x5f375a86u - (i >> 1);
  float r;
  std::memcpy(&r, &i, 4);
  const float h = 0.5f * l2;
  for (int k = 0; k < 3; ++k) r = r * fmaf_(-h, r * r, 1.5f);
  x *= r;
  y *= r;
  z *= r;
  return l2 * r;
}

// t_min of a ray whose direction was normalised from length len (DESIGN.md
// 2, step 2): the reference tests its roots against 0.001 in units of the
// ray's UNnormalised direction (src/cpu/main.cc:19 world.hit(r, 0.001, ..);
// src/gpu/camera.h:117 interval(0.001, inf); sphere.h:37-41 roots in units of
// d), i.e. 0.001 |d| in world units on the normalised ray.  tmin_world: the
// round-1..4 specification, 0.001 world units whatever |d| was.
inline float tmin_of(bool tmin_world, float len) { return tmin_world ? 0.001f : 0.001f * len; }

struct kscene {
  std::vector<float> cx, cy, cz, ks, inv_r, radius, ar, ag, ab, param, inv_param, r0;
  std::vector<uint32_t> kind;
  std::vector<uint8_t> sealed;  // the opaque-inside rule applies (sealed_of)
  double max_albedo = 0.0;      // largest lambertian / metal albedo channel
};

struct kctx {
  const kscene *sc;
  const rt_camera *cam;
  const rt_params *p;
  uint32_t seed32;
  bool open, metal_unit;
  double *exact = nullptr;  // rto_kernel_render_exact: fp64 sums of the unquantised radiance
  const float *out0 = nullptr;  // ... indexed like the frame tile out0
  bool no_dither = false;   // ... and the format without stochastic rounding (truncation only)
  bool tmin_world = false;  // t_min in world units (the round-4 specification, RTO_OPT_TMIN_WORLD)
  bool no_sealed = false;   // without the opaque-inside rule (RTO_OPT_NO_SEALED, attribution only)
  bool fp64_roots = false;  // candidates' roots in fp64 (RTO_OPT_FP64_ROOTS, attribution only)
  bool same_exit = true;    // the same-sphere exit rule (RTO_OPT_NO_SAME_EXIT turns it off)
  bool fp64_hit = false;    // the winner's root, hit point and normal in fp64 (RTO_OPT_FP64_HIT, attribution only)
};

// the sum format's dither draw (rt_kernel.hip dither_u): pcg4d keyed by the
// pixel and the sample with the bit-inverted seed
inline float dither_u(uint32_t pix, uint32_t sample, uint32_t seed32) {
  return unif(pcg4d(pix, sample, 0u, ~seed32).x);
}

// returns the ray's t_min (tmin_of its unnormalised direction's length)
float camera_ray(const kctx &k, uint32_t pix, int col, int grow, uint32_t sample, float o[3],
                 float d[3]) {
  const rt_camera &c = *k.cam;
  u4 r = pcg4d(pix, sample, 0u, k.seed32);
  float u1 = unif(r.x), u2 = unif(r.y);
  float fs, ft;
  if (c.model == RT_CAMERA_CPU) {
    int j = k.p->height - 1 - grow;
    // 1/(W-1) and 1/(H-1) rounded once to fp32 (main.cc:116-117 divides)
    fs = ((float)col + u1) * (float)(1.0 / (k.p->width - 1));
    ft = ((float)j + u2) * (float)(1.0 / (k.p->height - 1));
  } else {
    fs = (float)col + (u1 - 0.5f);
    ft = (float)grow + (u2 - 0.5f);
  }
  float t[3];
  for (int a = 0; a < 3; ++a) t[a] = fmaf_(ft, c.vert[a], fmaf_(fs, c.horiz[a], c.corner[a]));
  for (int a = 0; a < 3; ++a) o[a] = c.eye[a];
  if (c.has_lens) {
    float rr = sqrt_k(unif(r.z));
    float s, cc;
    sincos_turn(unif(r.w), s, cc);
    float ddx = rr * cc, ddy = rr * s;
    for (int a = 0; a < 3; ++a) o[a] = fmaf_(ddy, c.lens_v[a], fmaf_(ddx, c.lens_u[a], o[a]));
  }
  for (int a = 0; a < 3; ++a) d[a] = t[a] - o[a];
  return tmin_of(k.tmin_world, normalize3(d[0], d[1], d[2]));
}

// one pixel, all samples; returns number of closest-hit queries
unsigned long long kernel_pixel(const kctx &k, int col, int grow, float acc[3]) {
  const kscene &sc = *k.sc;
  const uint32_t pix = (uint32_t)grow * (uint32_t)k.p->width + (uint32_t)col;
  const size_t n = sc.cx.size();
  unsigned long long segs = 0;
  // fixed-point pixel sum (the kernel's spec): a sample's
  // radiance v (at most 1) adds q(v 2^F) to a uint32 sum, F = 31 -
  // floor(log2(spp)); the pixel is sum 2^-F.  q truncates for F >= 20 and
  // rounds stochastically below, trunc(x) + (frac(x) > u).  Integer addition
  // does not depend on the order, so any lanes, waves, launches or GPUs may
  // trace a pixel's samples
  acc[0] = acc[1] = acc[2] = 0.0f;
  double ex[3] = {0.0, 0.0, 0.0};
  if (k.p->max_depth <= 0 || k.p->spp <= 0) return 0;  // ray_color(.., 0) is black, no hit test
  // the sum format (rt_api.cpp sum_format): albedos above 1 make 64-bit sums
  // with a radiance clamp vcap = min(A^(max_depth - 1), 2^24) rounded down to
  // fp32, F = 62 - floor(log2 spp) - ceil(log2 vcap)
  int f = 31;
  for (int s = k.p->spp; s > 1; s >>= 1) --f;
  const bool wide = sc.max_albedo > 1.0;
  float vcap = 1.0f;
  if (wide) {
    double v = k.p->max_depth > 1 ? std::pow(sc.max_albedo, (double)(k.p->max_depth - 1)) : 1.0;
    v = std::min(std::max(v, 1.0), 16777216.0);
    vcap = (float)v;
    if ((double)vcap > v) vcap = std::nextafter(vcap, 0.0f);
    int e = 0;
    const double m = std::frexp((double)vcap, &e);
    f += 31 - (m == 0.5 ? e - 1 : e);
  }
  const float qscale = std::ldexp(1.0f, f), qinv = std::ldexp(1.0f, -f);
  const bool dither = f < 20 && !k.no_dither;
  uint64_t q[3] = {0u, 0u, 0u};
  for (uint32_t sample = 0; sample < (uint32_t)k.p->spp; ++sample) {
    float o[3], d[3];
    float tmin = camera_ray(k, pix, col, grow, sample, o, d);
    float th[3] = {1.0f, 1.0f, 1.0f};
    bool after_skip = false, inner_seen = false;  // rto_kernel_attrib
    long prev_best = -2;
    long origin_sphere = -1;  // the sphere the ray starts on (-1: a camera ray)
    for (int depth = 0;;) {
      ++segs;
      // closest hit: expanded quadratic with |d| = 1
      const float nk1 = -dot3(o[0], o[1], o[2], d[0], d[1], d[2]);
      const float o2 = dot3(o[0], o[1], o[2], o[0], o[1], o[2]);
      const float ox2 = -2.0f * o[0], oy2 = -2.0f * o[1], oz2 = -2.0f * o[2];
      float tmax = INFINITY;
      long best = -1;
      bool near = true;  // which root the winner was taken at
      const bool tr = g_trace && (long)sample == g_trace_sample;
      if (tr)
        std::fprintf(g_trace, "seg %d O=(%.9g %.9g %.9g) D=(%.9g %.9g %.9g) |O|^2=%.9g\n", depth, o[0],
                     o[1], o[2], d[0], d[1], d[2], o2);
      auto closest = [&]() {
        tmax = INFINITY;
        best = -1;
        near = true;
        // the per-sphere test in blocks of 64: a branch-free pass the compiler
        // vectorises (h and the discriminant's excess for every sphere), then
        // the candidates in index order -- the same arithmetic per sphere
        constexpr size_t kB = 64;
        float hb[kB], eb[kB];
        for (size_t i0 = 0; i0 < n; i0 += kB) {
          const size_t m = std::min(kB, n - i0);
          const float *cx = &sc.cx[i0], *cy = &sc.cy[i0], *cz = &sc.cz[i0], *ks = &sc.ks[i0];
          for (size_t j = 0; j < m; ++j) {
            const float h = fmaf_(cz[j], d[2], fmaf_(cx[j], d[0], fmaf_(cy[j], d[1], nk1)));
            const float g = fmaf_(cz[j], oz2, fmaf_(cx[j], ox2, fmaf_(cy[j], oy2, o2)));
            hb[j] = h;
            eb[j] = fmaf_(h, h, -g) - ks[j];  // >= 0 <=> e >= ks (exact for finite floats)
          }
          for (size_t j = 0; j < m; ++j) {
          if (!(eb[j] >= 0.0f)) continue;
          const size_t i = i0 + j;
          const float h = hb[j];
          {
            // sphere.h:34-44: the root offered is t0 if past t_min, else t1; it
            // wins if closer than tmax (ties: last index for the closed src/cpu
            // interval, first for the open src/gpu one -- what a sequential scan
            // does, stated so that any visiting order gives the same winner)
            const float sq = sqrt_k(eb[j]);
            float t0 = h - sq, t1 = h + sq;
            if (k.fp64_roots) {  // the same ray and sphere, roots in fp64
              const double ocx = (double)o[0] - sc.cx[i], ocy = (double)o[1] - sc.cy[i], ocz = (double)o[2] - sc.cz[i];
              const double b = ocx * d[0] + ocy * d[1] + ocz * d[2];
              const double r = sc.radius[i];
              const double c = ocx * ocx + ocy * ocy + ocz * ocz - r * r;
              const double dd = b * b - c;
              if (!(dd >= 0.0)) continue;
              const double s = std::sqrt(dd);
              t0 = (float)(-b - s);
              t1 = (float)(-b + s);
            }
            const bool use0 = k.open ? t0 > tmin : t0 >= tmin;
            const float root = use0 ? t0 : t1;
            const bool above = k.open ? root > tmin : root >= tmin;
            const bool closer = root < tmax || (root == tmax && (k.open ? (long)i < best : (long)i > best));
            if (tr)
              std::fprintf(g_trace, "   cand %zu disc=%.9g t0=%.9g t1=%.9g root=%.9g above=%d closer=%d\n", i,
                           eb[j], t0, t1, root, (int)above, (int)closer);
            if (above && closer) {
              tmax = root;
              near = use0;
              best = (long)i;
            }
          }
          }
        }
      };
      // refine the winner's chosen root with the better-conditioned forms
      // (DESIGN.md "Kernel algorithm", step 3); bb = (O - C).D
      auto refine = [&](size_t b, float &bb) {
        float t = tmax;
        const float r2 = sc.radius[b] * sc.radius[b];
        const float ocx = o[0] - sc.cx[b], ocy = o[1] - sc.cy[b], ocz = o[2] - sc.cz[b];
        bb = dot3(ocx, ocy, ocz, d[0], d[1], d[2]);
        float cc;
        if (r2 < o2 + std::fabs(sc.ks[b])) {
          cc = fmaf_(ocz, ocz, fmaf_(ocy, ocy, fmaf_(ocx, ocx, -r2)));
        } else {
          const float g = fmaf_(sc.cz[b], oz2, fmaf_(sc.cy[b], oy2, fmaf_(sc.cx[b], ox2, o2)));
          cc = g + sc.ks[b];
        }
        float disc;
        if (r2 < bb * bb) {
          const float fx = fmaf_(-bb, d[0], ocx), fy = fmaf_(-bb, d[1], ocy),
                      fz = fmaf_(-bb, d[2], ocz);
          disc = fmaf_(-fz, fz, fmaf_(-fy, fy, fmaf_(-fx, fx, r2)));
        } else {
          disc = fmaf_(bb, bb, -cc);
        }
        const float sq = sqrt_k(disc);
        const float q = -(bb + (bb < 0.0f ? -sq : sq));
        if (q != 0.0f) {
          const float ta = q, tb = cc * (1.0f / q);  // c RN(1/q), the kernel's rcp_k
          const float tr = near ? std::fmin(ta, tb) : std::fmax(ta, tb);
          if (std::isfinite(tr)) t = tr;
        }
        return t;
      };
      closest();
      float t = 0.0f;
      if (best >= 0) {
        float bb;
        t = refine((size_t)best, bb);
        // A refined root before t_min on a sphere the ray moves away from: the
        // ray starts on that sphere and leaves its ball, which in exact
        // arithmetic it cannot meet again (src/cpu, fp64, never does at
        // t >= 0.001); the expanded quadratic's root was an fp32 artefact (for
        // spheres far from the origin it can trap the path inside the
        // sphere).  So is (round 5) the exiting root of the sphere the ray
        // starts on when it moves away from that sphere's centre: t = 0 in
        // exact arithmetic, an fp32 hit point an ulp inside the ball with a
        // tiny t_min (lambertian n + u, u ~ -n) otherwise.  Not a segment: the
        // ray moves on to the scan's root point and walks again, same
        // direction.  (the ray keeps its t_min: same direction, same unit)
        if (bb > 0.0f && (t < tmin || (k.same_exit && best == origin_sphere && !near))) {
          if (tr) std::fprintf(g_trace, "  spurious best %ld t %.9g: skipped\n", best, tmax);
          g_skips.fetch_add(1, std::memory_order_relaxed);
          after_skip = true;
          if (t < tmin) {
            for (int a = 0; a < 3; ++a) o[a] = fmaf_(tmax, d[a], o[a]);
          } else {  // the same origin, t_min just past the scan's root (the kernel's bit step)
            tmin = std::nextafter(tmax, INFINITY);
          }
          normalize3(d[0], d[1], d[2]);
          --segs;
          continue;
        }
      }
      if (tr) std::fprintf(g_trace, "  -> best %ld t %.9g near %d\n", best, tmax, (int)near);
      if (best < 0) {  // sky, main.cc:27-29
        const float a = 0.5f * (d[1] + 1.0f);
        const float s0 = 1.0f - a;
        const float v[3] = {th[0] * fmaf_(a, 0.5f, s0), th[1] * fmaf_(a, 0.7f, s0), th[2] * (s0 + a)};
        const float u = dither ? dither_u(pix, sample, k.seed32) : 0.0f;
        for (int j = 0; j < 3; ++j) {
          const float x = (wide ? std::fmin(v[j], vcap) : v[j]) * qscale;
          const uint64_t qx = wide ? (uint64_t)x : (uint64_t)(uint32_t)x;
          q[j] += qx + (dither && x - std::floor(x) > u ? 1u : 0u);
          ex[j] += (double)v[j];
        }
        break;
      }
      const size_t b = (size_t)best;
      float p[3], nn[3];
      for (int a = 0; a < 3; ++a) p[a] = fmaf_(t, d[a], o[a]);
      nn[0] = (p[0] - sc.cx[b]) * sc.inv_r[b];
      nn[1] = (p[1] - sc.cy[b]) * sc.inv_r[b];
      nn[2] = (p[2] - sc.cz[b]) * sc.inv_r[b];
      // front face from the root taken (exact-arithmetic equivalent of
      // dot(d, outward) < 0, hittable.h:16-19; outward flips for r < 0)
      if (k.fp64_hit) {
        // attribution only (RTO_OPT_FP64_HIT): the winner's root from the
        // fp64 quadratic on the fp32 ray and sphere (the reference's
        // sphere::hit arithmetic, sphere.h:24-51, |d| = 1 here), and the hit
        // point and normal from it in fp64, rounded once to fp32
        const double c3[3] = {sc.cx[b], sc.cy[b], sc.cz[b]}, rr = sc.radius[b];
        double oc[3], hb = 0.0, cq = -rr * rr, dd = 0.0;
        for (int a = 0; a < 3; ++a) {
          oc[a] = (double)o[a] - c3[a];
          hb += oc[a] * (double)d[a];
          cq += oc[a] * oc[a];
          dd += (double)d[a] * (double)d[a];
        }
        const double disc = hb * hb - dd * cq;
        if (disc >= 0.0) {
          const double sq = std::sqrt(disc);
          const double td = (near ? (-hb - sq) : (-hb + sq)) / dd;
          for (int a = 0; a < 3; ++a) {
            const double pd = (double)o[a] + td * (double)d[a];
            p[a] = (float)pd;
            nn[a] = (float)((pd - c3[a]) / rr);
          }
        }
      }
      const bool front = near != (sc.inv_r[b] < 0.0f);
      if (!front)
        for (int a = 0; a < 3; ++a) nn[a] = -nn[a];
      const u4 r = pcg4d(pix, sample, (uint32_t)(depth + 1), k.seed32);
      float sd[3];
      bool scattered = true;
      if (sc.kind[b] == RT_LAMBERTIAN) {
        float u[3];
        unit_vec(unif(r.x), unif(r.y), u[0], u[1], u[2]);
        for (int a = 0; a < 3; ++a) sd[a] = nn[a] + u[a];
        const float eps = 1e-8f;
        if (std::fabs(sd[0]) < eps && std::fabs(sd[1]) < eps && std::fabs(sd[2]) < eps)
          for (int a = 0; a < 3; ++a) sd[a] = nn[a];
        th[0] *= sc.ar[b];
        th[1] *= sc.ag[b];
        th[2] *= sc.ab[b];
      } else if (sc.kind[b] == RT_METAL) {
        const float kk = -2.0f * dot3(d[0], d[1], d[2], nn[0], nn[1], nn[2]);
        float rf[3], u[3];
        for (int a = 0; a < 3; ++a) rf[a] = fmaf_(kk, nn[a], d[a]);
        unit_vec(unif(r.x), unif(r.y), u[0], u[1], u[2]);
        float fz = sc.param[b];
        if (!k.metal_unit) fz *= ball_radius(r);
        for (int a = 0; a < 3; ++a) sd[a] = fmaf_(fz, u[a], rf[a]);
        scattered = dot3(sd[0], sd[1], sd[2], nn[0], nn[1], nn[2]) > 0.0f;
        th[0] *= sc.ar[b];
        th[1] *= sc.ag[b];
        th[2] *= sc.ab[b];
      } else {
        const float ratio = front ? sc.inv_param[b] : sc.param[b];
        const float cos_t = std::fmin(-dot3(d[0], d[1], d[2], nn[0], nn[1], nn[2]), 1.0f);
        // ratio sin > 1 (material.h:64), squared (the kernel's form)
        const bool cannot = (ratio * ratio) * fmaf_(-cos_t, cos_t, 1.0f) > 1.0f;
        const float r0 = sc.r0[b];  // ((1-ior)/(1+ior))^2, same for ior and 1/ior
        const float x = 1.0f - cos_t;
        const float x2 = x * x;
        const float refl = fmaf_(1.0f - r0, x2 * x2 * x, r0);
        if (cannot || refl > unif(r.x)) {
          const float kk = -2.0f * dot3(d[0], d[1], d[2], nn[0], nn[1], nn[2]);
          for (int a = 0; a < 3; ++a) sd[a] = fmaf_(kk, nn[a], d[a]);
        } else {
          float q[3];
          for (int a = 0; a < 3; ++a) q[a] = ratio * fmaf_(cos_t, nn[a], d[a]);
          const float m = -sqrt_k(std::fabs(1.0f - dot3(q[0], q[1], q[2], q[0], q[1], q[2])));
          for (int a = 0; a < 3; ++a) sd[a] = fmaf_(m, nn[a], q[a]);
        }
      }
      // the opaque-inside rule: a sealed lambertian
      // sphere hit at its exiting root ends the path (in the reference's
      // arithmetic every later chord inside it is t = |r|, to the depth cap)
      if (sc.kind[b] == RT_LAMBERTIAN && sc.sealed[b] && !near && !inner_seen) {
        inner_seen = true;
        g_inner.fetch_add(1, std::memory_order_relaxed);
        if (after_skip) g_inner_after_skip.fetch_add(1, std::memory_order_relaxed);
        const unsigned e = g_ev_n.fetch_add(1);
        if (e < 4096) {
          g_ev[e][0] = (long long)b;
          g_ev[e][1] = prev_best;
          g_ev[e][2] = depth;
          g_ev[e][3] = (long long)(tmin * 1e6f);
        }
      }
      prev_best = (long)b;
      after_skip = false;
      if (sc.kind[b] == RT_LAMBERTIAN && sc.sealed[b] && !near && !k.no_sealed) scattered = false;
      if (wide)  // albedos above 1: the throughput stays finite (the kernel's clamp)
        for (int a = 0; a < 3; ++a) th[a] = std::fmin(th[a], 0x1p100f);
      ++depth;
      if (scattered && depth >= k.p->max_depth) g_kcapped.fetch_add(1, std::memory_order_relaxed);
      if (!scattered || depth >= k.p->max_depth) break;
      for (int a = 0; a < 3; ++a) {
        o[a] = p[a];
        d[a] = sd[a];
      }
      origin_sphere = (long)b;
      tmin = tmin_of(k.tmin_world, normalize3(d[0], d[1], d[2]));
    }
  }
  for (int a = 0; a < 3; ++a) acc[a] = (wide ? (float)q[a] : (float)(uint32_t)q[a]) * qinv;
  if (k.exact) {
    double *e = k.exact + 3 * ((size_t)(&acc[0] - k.out0) / 3);
    for (int a = 0; a < 3; ++a) e[a] = ex[a];
  }
  return segs;
}

// ---------------------------------------------------------------------
// src/gpu restatement (rto_gpuref_render): the reference CUDA path's own
// per-sample arithmetic, fp32, as src/gpu/camera.h:112-195, sphere.h:15-44,
// material.h:20-104 and rtweekend.h:42-69 write it -- for attributing the
// brightness difference between the kernel specification (GPU semantics
// flags) and gallery/gpu/image23.png.  Each switch replaces one
// part of the kernel specification with src/gpu's form:
//   GREF_NAIVE_HIT: sphere::hit's quadratic (oc = O - C, a = |d|^2, roots
//                   (-half_b -+ sqrt(disc)) / a, the open interval, the scan's
//                   shrinking t_max), hit point O + t d, set_face_normal by
//                   dot(d, outward) -- no refinement, no spurious-root rule, no
//                   opaque-inside rule;
//   GREF_UNNORM:    directions left unnormalised (the camera's pixel_sample -
//                   origin, scatter directions as built), unit_vector(d) =
//                   d (1 / |d|) where src/gpu takes one (needs GREF_NAIVE_HIT:
//                   the kernel's quadratic assumes |d| = 1);
//   GREF_REJECT:    random_in_unit_sphere / random_in_unit_disk by rejection
//                   (random_unit_vector = its unit_vector), uniforms from
//                   pcg4d batches of 4;
//   GREF_FP32_SUM:  pixel sums in fp32 (camera.h:189-194) instead of the
//                   fixed-point sums.
// nvcc contracts a*b+c into fma by default (-fmad=true): the dot products and
// o + t d are written as fma chains.  Uniforms come from pcg4d (src/gpu draws
// curand XORWOW): equal in distribution, a different stream.
enum { GREF_NAIVE_HIT = 1, GREF_UNNORM = 2, GREF_REJECT = 4, GREF_FP32_SUM = 8 };

struct gvec {
  float x, y, z;
};
inline gvec gadd(gvec a, gvec b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline gvec gsub(gvec a, gvec b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline gvec gmul(float t, gvec v) { return {t * v.x, t * v.y, t * v.z}; }
inline float gdot(gvec a, gvec b) { return fmaf_(a.z, b.z, fmaf_(a.y, b.y, a.x * b.x)); }
inline gvec gfma(float t, gvec d, gvec o) { return {fmaf_(t, d.x, o.x), fmaf_(t, d.y, o.y), fmaf_(t, d.z, o.z)}; }
inline gvec gunit(gvec v) { return gmul(1.0f / std::sqrt(gdot(v, v)), v); }  // vec3.h: v / length, operator/ = (1/t) v

// a stream of uniforms for one (pixel, sample, bounce): pcg4d batches
struct gdraws {
  uint32_t pix, sample, slot, seed, batch = 0, k = 4;
  u4 cur{};
  float next() {
    if (k == 4) {
      cur = pcg4d(pix, sample, slot | (batch++ << 16), seed);
      k = 0;
    }
    const uint32_t v[4] = {cur.x, cur.y, cur.z, cur.w};
    return unif(v[k++]);
  }
};

gvec g_in_unit_sphere(gdraws &r) {  // rtweekend.h:42-49
  while (true) {
    const float x = fmaf_(2.0f, r.next(), -1.0f), y = fmaf_(2.0f, r.next(), -1.0f), z = fmaf_(2.0f, r.next(), -1.0f);
    const gvec p{x, y, z};
    if (gdot(p, p) < 1.0f) return p;
  }
}

unsigned long long gpuref_pixel(const kctx &k, int col, int grow, float acc[3], int mode) {
  const kscene &sc = *k.sc;
  const rt_camera &c = *k.cam;
  const uint32_t pix = (uint32_t)grow * (uint32_t)k.p->width + (uint32_t)col;
  const size_t n = sc.cx.size();
  const bool naive = mode & GREF_NAIVE_HIT, unnorm = (mode & GREF_UNNORM) && naive, reject = mode & GREF_REJECT;
  unsigned long long segs = 0;
  float fsum[3] = {0.0f, 0.0f, 0.0f};
  uint32_t q[3] = {0u, 0u, 0u};
  int f = 31;
  for (int s = k.p->spp; s > 1; s >>= 1) --f;
  const float qscale = std::ldexp(1.0f, f), qinv = std::ldexp(1.0f, -f);
  for (uint32_t sample = 0; sample < (uint32_t)k.p->spp; ++sample) {
    // get_ray (camera.h:153-167): the kernel's camera arithmetic for the
    // target; the lens by rejection or the polar draw
    const u4 r0 = pcg4d(pix, sample, 0u, k.seed32);
    float fs, ft;
    if (c.model == RT_CAMERA_CPU) {
      fs = ((float)col + unif(r0.x)) * (float)(1.0 / (k.p->width - 1));
      ft = ((float)(k.p->height - 1 - grow) + unif(r0.y)) * (float)(1.0 / (k.p->height - 1));
    } else {
      fs = (float)col + (unif(r0.x) - 0.5f);
      ft = (float)grow + (unif(r0.y) - 0.5f);
    }
    gvec tgt, o{c.eye[0], c.eye[1], c.eye[2]};
    tgt.x = fmaf_(ft, c.vert[0], fmaf_(fs, c.horiz[0], c.corner[0]));
    tgt.y = fmaf_(ft, c.vert[1], fmaf_(fs, c.horiz[1], c.corner[1]));
    tgt.z = fmaf_(ft, c.vert[2], fmaf_(fs, c.horiz[2], c.corner[2]));
    if (c.has_lens) {
      float dx, dy;
      if (reject) {  // random_in_unit_disk, rtweekend.h:61-69
        gdraws dr{pix, sample, 0u, k.seed32};
        dr.k = 2;  // r0's z and w first
        dr.cur = r0;
        do {
          dx = fmaf_(2.0f, dr.next(), -1.0f);
          dy = fmaf_(2.0f, dr.next(), -1.0f);
        } while (!(fmaf_(dy, dy, dx * dx) < 1.0f));
      } else {
        const float rr = sqrt_k(unif(r0.z));
        float sn, cs;
        sincos_turn(unif(r0.w), sn, cs);
        dx = rr * cs;
        dy = rr * sn;
      }
      o.x = fmaf_(dy, c.lens_v[0], fmaf_(dx, c.lens_u[0], o.x));
      o.y = fmaf_(dy, c.lens_v[1], fmaf_(dx, c.lens_u[1], o.y));
      o.z = fmaf_(dy, c.lens_v[2], fmaf_(dx, c.lens_u[2], o.z));
    }
    gvec d = gsub(tgt, o);
    // t_min in units of the unnormalised direction (tmin_of); with GREF_UNNORM
    // the roots are in those units already
    float tmin = 0.001f;
    if (!unnorm) tmin = tmin_of(k.tmin_world, normalize3(d.x, d.y, d.z));
    gvec att{1.0f, 1.0f, 1.0f};
    gvec col3{0.0f, 0.0f, 0.0f};
    for (int depth = 0; depth < k.p->max_depth; ++depth) {
      ++segs;
      long best = -1;
      float tbest = INFINITY;
      gvec p{}, nrm{};
      bool front = true;
      bool inside = false;  // the winner was taken at its exiting root (specification only)
      if (naive) {
        // hittable_list::hit (hittable_list.h:49-65) over sphere::hit (sphere.h:15-44)
        const float a = gdot(d, d);
        for (size_t i = 0; i < n; ++i) {
          const gvec oc = gsub(o, gvec{sc.cx[i], sc.cy[i], sc.cz[i]});
          const float hb = gdot(oc, d);
          const float cc = fmaf_(-sc.radius[i], sc.radius[i], gdot(oc, oc));
          const float disc = fmaf_(hb, hb, -(a * cc));
          if (disc < 0.0f) continue;
          const float sq = std::sqrt(disc);
          float root = (-hb - sq) / a;
          if (!(root > tmin && root < tbest)) {  // interval::surrounds
            root = (-hb + sq) / a;
            if (!(root > tmin && root < tbest)) continue;
          }
          tbest = root;
          best = (long)i;
        }
        if (best >= 0) {
          const size_t b = (size_t)best;
          p = gfma(tbest, d, o);
          const gvec outward = gmul(1.0f / sc.radius[b], gsub(p, gvec{sc.cx[b], sc.cy[b], sc.cz[b]}));
          front = gdot(d, outward) < 0.0f;  // hittable.h:16-19
          nrm = front ? outward : gvec{-outward.x, -outward.y, -outward.z};
        }
      } else {
        // the kernel specification's closest hit, refinement and shading normal
        const float nk1 = -dot3(o.x, o.y, o.z, d.x, d.y, d.z);
        const float o2 = dot3(o.x, o.y, o.z, o.x, o.y, o.z);
        const float ox2 = -2.0f * o.x, oy2 = -2.0f * o.y, oz2 = -2.0f * o.z;
        bool near = true;
        for (size_t i = 0; i < n; ++i) {
          const float h = fmaf_(sc.cz[i], d.z, fmaf_(sc.cx[i], d.x, fmaf_(sc.cy[i], d.y, nk1)));
          const float g = fmaf_(sc.cz[i], oz2, fmaf_(sc.cx[i], ox2, fmaf_(sc.cy[i], oy2, o2)));
          const float e = fmaf_(h, h, -g);
          if (!(e >= sc.ks[i])) continue;
          const float sq = sqrt_k(e - sc.ks[i]);
          const float t0 = h - sq, t1 = h + sq;
          const bool use0 = t0 > tmin;
          const float root = use0 ? t0 : t1;
          if (root > tmin && (root < tbest || (root == tbest && (long)i < best))) {
            tbest = root;
            near = use0;
            best = (long)i;
          }
        }
        if (best >= 0) {
          const size_t b = (size_t)best;
          // refine
          const float r2 = sc.radius[b] * sc.radius[b];
          const float ocx = o.x - sc.cx[b], ocy = o.y - sc.cy[b], ocz = o.z - sc.cz[b];
          const float bb = dot3(ocx, ocy, ocz, d.x, d.y, d.z);
          float cc;
          if (r2 < o2 + std::fabs(sc.ks[b])) cc = fmaf_(ocz, ocz, fmaf_(ocy, ocy, fmaf_(ocx, ocx, -r2)));
          else cc = fmaf_(sc.cz[b], oz2, fmaf_(sc.cy[b], oy2, fmaf_(sc.cx[b], ox2, o2))) + sc.ks[b];
          float disc;
          if (r2 < bb * bb) {
            const float fx = fmaf_(-bb, d.x, ocx), fy = fmaf_(-bb, d.y, ocy), fz = fmaf_(-bb, d.z, ocz);
            disc = fmaf_(-fz, fz, fmaf_(-fy, fy, fmaf_(-fx, fx, r2)));
          } else {
            disc = fmaf_(bb, bb, -cc);
          }
          const float sq = sqrt_k(disc);
          const float qq = -(bb + (bb < 0.0f ? -sq : sq));
          float t = tbest;
          if (qq != 0.0f) {
            const float ta = qq, tb = cc * (1.0f / qq);
            const float tr = near ? std::fmin(ta, tb) : std::fmax(ta, tb);
            if (std::isfinite(tr)) t = tr;
          }
          if (t < tmin && bb > 0.0f) {  // spurious root: move on, not a segment
            o = gfma(tbest, d, o);
            --segs;
            --depth;
            continue;
          }
          p = gfma(t, d, o);
          nrm = gvec{(p.x - sc.cx[b]) * sc.inv_r[b], (p.y - sc.cy[b]) * sc.inv_r[b], (p.z - sc.cz[b]) * sc.inv_r[b]};
          front = near != (sc.inv_r[b] < 0.0f);
          inside = !near;
          if (!front) nrm = gvec{-nrm.x, -nrm.y, -nrm.z};
        }
      }
      if (best < 0) {  // camera.h:118-124
        const gvec ud = unnorm ? gunit(d) : d;
        const float a = 0.5f * (ud.y + 1.0f);
        const float s0 = 1.0f - a;
        col3 = gvec{att.x * fmaf_(a, 0.5f, s0), att.y * fmaf_(a, 0.7f, s0), att.z * (s0 + a)};
        break;
      }
      const size_t b = (size_t)best;
      gdraws dr{pix, sample, (uint32_t)(depth + 1), k.seed32};
      auto unit_vector = [&]() -> gvec {
        if (reject) return gunit(g_in_unit_sphere(dr));
        gvec u;
        unit_vec(dr.next(), dr.next(), u.x, u.y, u.z);
        return u;
      };
      gvec sd;
      bool scattered = true;
      if (sc.kind[b] == RT_LAMBERTIAN) {  // material.h:20-40
        sd = gadd(nrm, unit_vector());
        const float e = 1e-8f;
        if (std::fabs(sd.x) < e && std::fabs(sd.y) < e && std::fabs(sd.z) < e) sd = nrm;
        if (!naive && inside && sc.sealed[b]) scattered = false;  // the specification's opaque-inside rule
      } else if (sc.kind[b] == RT_METAL) {  // material.h:42-64
        const gvec ud = unnorm ? gunit(d) : d;
        const float kk = -2.0f * gdot(ud, nrm);
        const gvec refl = gfma(kk, nrm, ud);
        const gvec u = unit_vector();
        sd = gfma(sc.param[b], u, refl);
        scattered = gdot(sd, nrm) > 0.0f;
      } else {  // material.h:66-104
        const float ratio = front ? sc.inv_param[b] : sc.param[b];
        const gvec ud = unnorm ? gunit(d) : d;
        const float cos_t = std::fmin(-gdot(ud, nrm), 1.0f);
        const float sin_t = std::sqrt(fmaf_(-cos_t, cos_t, 1.0f));
        const bool cannot = ratio * sin_t > 1.0f;
        const float r0 = sc.r0[b];
        const float refl = fmaf_(1.0f - r0, std::pow(1.0f - cos_t, 5.0f), r0);
        if (cannot || refl > dr.next()) {
          const float kk = -2.0f * gdot(ud, nrm);
          sd = gfma(kk, nrm, ud);
        } else {
          const gvec qv = gmul(ratio, gfma(cos_t, nrm, ud));
          const float m = -std::sqrt(std::fabs(1.0f - gdot(qv, qv)));
          sd = gfma(m, nrm, qv);
        }
      }
      if (!scattered) break;
      att = gvec{att.x * sc.ar[b], att.y * sc.ag[b], att.z * sc.ab[b]};
      o = p;
      d = sd;
      if (!unnorm) tmin = tmin_of(k.tmin_world, normalize3(d.x, d.y, d.z));
    }
    const float v[3] = {col3.x, col3.y, col3.z};
    for (int j = 0; j < 3; ++j) {
      fsum[j] += v[j];
      const float x = v[j] * qscale;
      q[j] += (uint32_t)x;
    }
  }
  for (int a = 0; a < 3; ++a) acc[a] = (mode & GREF_FP32_SUM) ? fsum[a] : (float)q[a] * qinv;
  return segs;
}

// The opaque-inside rule's sealed spheres (restates rt_accel.cpp
// sealed_spheres): lambertian, |r| > 2 t_min, and no
// other sphere's ball overlaps its ball (fp64; touching at one point allowed).
// Brute force over all pairs, independent of the product's sweep.
std::vector<uint8_t> sealed_of(const rt_scene_view &v) {
  std::vector<uint8_t> over(v.n, 0), out(v.n, 0);
  for (uint32_t i = 0; i < v.n; ++i)
    for (uint32_t j = i + 1; j < v.n; ++j) {
      const double dx = (double)v.cx[i] - v.cx[j];
      const double rs = std::fabs((double)v.radius[i]) + std::fabs((double)v.radius[j]);
      if (std::fabs(dx) >= rs) continue;
      const double dy = (double)v.cy[i] - v.cy[j], dz = (double)v.cz[i] - v.cz[j];
      if (dx * dx + dy * dy + dz * dz < rs * rs) over[i] = over[j] = 1;
    }
  for (uint32_t i = 0; i < v.n; ++i)
    out[i] = v.mat_kind[i] == RT_LAMBERTIAN && !over[i] && std::fabs((double)v.radius[i]) > 0.002;
  return out;
}

kscene make_kscene(const rt_scene_view &v) {
  kscene s;
  s.sealed = sealed_of(v);
  for (uint32_t i = 0; i < v.n; ++i)
    for (int a = 0; a < 3 && v.mat_kind[i] != RT_DIELECTRIC; ++a)
      s.max_albedo = std::max(s.max_albedo, (double)v.albedo_rgb[3 * i + a]);
  for (uint32_t i = 0; i < v.n; ++i) {
    const double x = v.cx[i], y = v.cy[i], z = v.cz[i], r = v.radius[i];
    s.cx.push_back(v.cx[i]);
    s.cy.push_back(v.cy[i]);
    s.cz.push_back(v.cz[i]);
    s.ks.push_back((float)(x * x + y * y + z * z - r * r));
    s.inv_r.push_back(1.0f / v.radius[i]);
    s.radius.push_back(v.radius[i]);
    s.ar.push_back(v.albedo_rgb[3 * i + 0]);
    s.ag.push_back(v.albedo_rgb[3 * i + 1]);
    s.ab.push_back(v.albedo_rgb[3 * i + 2]);
    // metal fuzz clamped to 1 (material.h:38), as rt_scene_upload does
    s.param.push_back(v.mat_kind[i] == RT_METAL ? std::min(v.mat_param[i], 1.0f) : v.mat_param[i]);
    const double ior = v.mat_param[i];
    s.inv_param.push_back((float)(1.0 / ior));
    const double r0 = (1.0 - ior) / (1.0 + ior);
    s.r0.push_back((float)(r0 * r0));
    s.kind.push_back(v.mat_kind[i]);
  }
  return s;
}

}  // namespace

extern "C" {

namespace {
// main.cc:78-130 from the camera on, for a world already built (and the rng
// at the state the scene left it in)
int reference_render_world(dworld &w, rng64 &r, d3 lookfrom, d3 lookat, double aperture, double focus,
                           int width, double aspect, int spp, int max_depth, uint8_t *rgb_out,
                           unsigned long long *segments);
}  // namespace

int rto_sealed(const rt_scene_view *scene, uint8_t *out) {
  if (!scene || !out) return -1;
  const std::vector<uint8_t> v = sealed_of(*scene);
  std::copy(v.begin(), v.end(), out);
  return 0;
}

// The kernel's sampling draws on n pcg4d keys (i, 7, 3, seed), for the
// distribution tests (tests/test_oracle.py): kind 0 a unit vector (lambertian
// and metal), 1 a point of the unit ball (metal fuzz: ball_radius x unit
// vector, random_in_unit_sphere's law), 2 a point of the unit disk (the
// lens, random_in_unit_disk), 3 a lambertian direction about the normal
// (0, 0, 1), normalised as the kernel does.  3 floats per draw.
int rto_sample_probe(int kind, uint32_t n, uint32_t seed, float *out) {
  if (!out || kind < 0 || kind > 3) return -1;
  for (uint32_t i = 0; i < n; ++i) {
    const u4 r = pcg4d(i, 7u, 3u, seed);
    float v[3] = {0, 0, 0};
    if (kind == 2) {
      const float rr = sqrt_k(unif(r.z));
      float s, c;
      sincos_turn(unif(r.w), s, c);
      v[0] = rr * c;
      v[1] = rr * s;
    } else {
      unit_vec(unif(r.x), unif(r.y), v[0], v[1], v[2]);
      if (kind == 1) {
        const float rho = ball_radius(r);
        for (float &x : v) x *= rho;
      } else if (kind == 3) {
        v[2] += 1.0f;
        normalize3(v[0], v[1], v[2]);
      }
    }
    for (int a = 0; a < 3; ++a) out[3 * (size_t)i + a] = v[a];
  }
  return 0;
}

int rto_reference_render(int width, double aspect, int spp, int max_depth, int scene,
                         uint8_t *rgb_out, int *height_out, unsigned long long *segments) {
  if (width < 2 || !(aspect > 0) || spp < 1 || max_depth < 0) return -1;
  const int height = (int)(width / aspect);  // main.cc:84
  if (height < 2) return -1;
  if (height_out) *height_out = height;
  if (!rgb_out) return 0;  // size query
  rng64 r;
  dworld w;
  d3 lookfrom{13, 2, 3}, lookat{0, 0, 0};
  double aperture = 0.1, focus = 10.0;
  if (scene == 1) {
    five_scene(w.s);
    lookfrom = {-2, 2, 1};
    lookat = {0, 0, -1};
    aperture = 0.0;
    focus = 3.4;
  } else {
    final_scene(r, 11, w.s);
  }
  return reference_render_world(w, r, lookfrom, lookat, aperture, focus, width, aspect, spp, max_depth,
                                rgb_out, segments);
}

int rto_reference_render_view(const rt_scene_view *scene, int width, double aspect, int spp, int max_depth,
                              uint8_t *rgb_out, int *height_out, unsigned long long *segments) {
  if (!scene || width < 2 || !(aspect > 0) || spp < 1 || max_depth < 0) return -1;
  const int height = (int)(width / aspect);
  if (height < 2) return -1;
  if (height_out) *height_out = height;
  if (!rgb_out) return 0;
  rng64 r;  // no scene draws: the stream starts at the first sample
  dworld w;
  for (uint32_t i = 0; i < scene->n; ++i) {
    const uint32_t k = scene->mat_kind[i];
    const double p = scene->mat_param[i];
    const d3 alb{scene->albedo_rgb[3 * i], scene->albedo_rgb[3 * i + 1], scene->albedo_rgb[3 * i + 2]};
    // material.h:38: metal(a, f) keeps fuzz(f < 1 ? f : 1); dielectrics carry no albedo
    w.s.push_back({{scene->cx[i], scene->cy[i], scene->cz[i]}, scene->radius[i], (int)k,
                   k == RT_DIELECTRIC ? d3{1, 1, 1} : alb, k == RT_METAL ? (p < 1 ? p : 1) : p});
  }
  return reference_render_world(w, r, {13, 2, 3}, {0, 0, 0}, 0.1, 10.0, width, aspect, spp, max_depth,
                                rgb_out, segments);
}

namespace {
int reference_render_world(dworld &w, rng64 &r, d3 lookfrom, d3 lookat, double aperture, double focus,
                           int width, double aspect, int spp, int max_depth, uint8_t *rgb_out,
                           unsigned long long *segments) {
  const int height = (int)(width / aspect);
  {  // the sealed spheres (sealed_of's rule on the fp64 scene), for rto_reference_trapped
    const size_t n = w.s.size();
    std::vector<uint8_t> over(n, 0);
    for (size_t i = 0; i < n; ++i)
      for (size_t j = i + 1; j < n; ++j) {
        const d3 e = w.s[i].c - w.s[j].c;
        const double rs = std::fabs(w.s[i].r) + std::fabs(w.s[j].r);
        if (dot(e, e) < rs * rs) over[i] = over[j] = 1;
      }
    w.sealed.assign(n, 0);
    for (size_t i = 0; i < n; ++i)
      w.sealed[i] = w.s[i].kind == RT_LAMBERTIAN && !over[i] && std::fabs(w.s[i].r) > 0.002 && w.s[i].r > 0;
  }
  // camera.h:8-26
  const double pi = 3.1415926535897932385;
  double theta = 20.0 * pi / 180.0;
  double hh = std::tan(theta / 2);
  double vh = 2.0 * hh, vw = aspect * vh;
  d3 cw = unit(lookfrom - lookat);
  d3 cu = unit(cross(d3{0, 1, 0}, cw));
  d3 cv = cross(cw, cu);
  d3 origin = lookfrom;
  d3 horizontal = (focus * vw) * cu;
  d3 vertical = (focus * vh) * cv;
  d3 llc = origin - horizontal / 2 - vertical / 2 - focus * cw;
  double lens_radius = aperture / 2;
  const double scale = 1.0 / spp;
  size_t k = 0;
  for (int j = height - 1; j >= 0; --j) {  // main.cc:111-123
    for (int i = 0; i < width; ++i) {
      d3 pc{0, 0, 0};
      for (int s = 0; s < spp; ++s) {
        double u = (i + r()) / (width - 1);
        double v = (j + r()) / (height - 1);
        d3 rd = lens_radius * in_unit_disk(r);  // camera.h:29-33
        d3 offset = rd.x * cu + rd.y * cv;
        d3 ro = origin + offset;
        d3 rdir = llc + u * horizontal + v * vertical - origin - offset;
        pc = pc + ray_color(ro, rdir, w, r, max_depth);
      }
      rgb_out[k++] = tonemap(pc.x, scale);
      rgb_out[k++] = tonemap(pc.y, scale);
      rgb_out[k++] = tonemap(pc.z, scale);
    }
  }
  if (segments) *segments = w.calls;
  g_last_trapped = w.trapped;
  g_last_capped = w.capped;
  return 0;
}
}  // namespace

unsigned long long rto_reference_trapped() { return g_last_trapped; }
unsigned long long rto_reference_capped() { return g_last_capped; }
unsigned long long rto_kernel_capped(int reset) {
  const unsigned long long v = g_kcapped.load();
  if (reset) g_kcapped = 0;
  return v;
}

void rto_kernel_attrib(unsigned long long *out, int reset) {
  out[0] = g_skips.load();
  out[1] = g_inner.load();
  out[2] = g_inner_after_skip.load();
  if (reset) g_skips = g_inner = g_inner_after_skip = 0;
}

int rto_kernel_attrib_events(long long *out, int n, int reset) {
  const int m = (int)std::min<unsigned>(g_ev_n.load(), std::min(n, 4096));
  std::memcpy(out, g_ev, sizeof(long long) * 4 * (size_t)m);
  if (reset) g_ev_n = 0;
  return m;
}

int rto_kernel_render_exact(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p,
                            float *out, double *exact, int opts, unsigned long long *segments,
                            int threads) {
  if (!scene || !cam || !p || !out || p->width < 1 || p->height < 1 || p->row_block < 1 ||
      p->band_stride < 1 || p->local_rows < 0 || p->spp < 0 || p->spp >= (1 << 24))
    return -1;
  const kscene sc = make_kscene(*scene);
  kctx k{&sc, cam, p, (uint32_t)p->seed ^ ((uint32_t)(p->seed >> 32) * 0x9E3779B9u),
         (p->flags & RT_FLAG_OPEN_INTERVAL) != 0, (p->flags & RT_FLAG_METAL_UNIT_VECTOR) != 0};
  k.exact = exact;
  k.out0 = out;
  k.no_dither = (opts & RTO_OPT_NO_DITHER) != 0;
  k.tmin_world = (opts & RTO_OPT_TMIN_WORLD) != 0;
  k.no_sealed = (opts & RTO_OPT_NO_SEALED) != 0;
  k.fp64_roots = (opts & RTO_OPT_FP64_ROOTS) != 0;
  k.same_exit = (opts & RTO_OPT_NO_SAME_EXIT) == 0;
  k.fp64_hit = (opts & RTO_OPT_FP64_HIT) != 0;
  if (exact) std::memset(exact, 0, 3 * sizeof(double) * (size_t)p->local_rows * (size_t)p->width);
  if (threads < 1) {
    // the machine's cores, but no more than OMP_NUM_THREADS (16 on the GPU
    // box, whose nproc shows the whole host) or 16
    threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char *e = std::getenv("OMP_NUM_THREADS")) {
      const int k = std::atoi(e);
      if (k >= 1) threads = std::min(threads, k);
    }
  }
  // work items of 64 pixels (a band of 8 rows still spreads over every thread)
  const long long n_px = (long long)p->local_rows * p->width;
  std::atomic<long long> next{0};
  std::atomic<unsigned long long> total{0};
  auto worker = [&]() {
    unsigned long long segs = 0;
    for (long long i0; (i0 = next.fetch_add(64)) < n_px;) {
      for (long long i = i0; i < std::min(n_px, i0 + 64); ++i) {
        const int lr = (int)(i / p->width), col = (int)(i % p->width);
        const int band = lr / p->row_block;
        const int grow = (band * p->band_stride + p->band_offset) * p->row_block + lr % p->row_block;
        float *o = out + 3 * (size_t)i;
        if (grow >= p->height) {
          o[0] = o[1] = o[2] = 0.0f;
          continue;
        }
        segs += kernel_pixel(k, col, grow, o);
      }
    }
    total += segs;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
  worker();
  for (auto &t : pool) t.join();
  if (segments) *segments = total.load();
  return 0;
}

int rto_kernel_render(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p,
                      float *out, unsigned long long *segments, int threads) {
  return rto_kernel_render_exact(scene, cam, p, out, nullptr, 0, segments, threads);
}

int rto_gpuref_render(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p, int mode,
                      float *out, unsigned long long *segments, int threads) {
  if (!scene || !cam || !p || !out || p->width < 1 || p->height < 1 || p->row_block < 1 ||
      p->band_stride < 1 || p->local_rows < 0 || p->spp < 0 || p->spp >= (1 << 24))
    return -1;
  const kscene sc = make_kscene(*scene);
  kctx k{&sc, cam, p, (uint32_t)p->seed ^ ((uint32_t)(p->seed >> 32) * 0x9E3779B9u), true, true};
  if (threads < 1) threads = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const long long n_px = (long long)p->local_rows * p->width;
  std::atomic<long long> next{0};
  std::atomic<unsigned long long> total{0};
  auto worker = [&]() {
    unsigned long long segs = 0;
    for (long long i0; (i0 = next.fetch_add(64)) < n_px;) {
      for (long long i = i0; i < std::min(n_px, i0 + 64); ++i) {
        const int lr = (int)(i / p->width), col = (int)(i % p->width);
        const int band = lr / p->row_block;
        const int grow = (band * p->band_stride + p->band_offset) * p->row_block + lr % p->row_block;
        float *o = out + 3 * (size_t)i;
        if (grow >= p->height) {
          o[0] = o[1] = o[2] = 0.0f;
          continue;
        }
        segs += gpuref_pixel(k, col, grow, o, mode);
      }
    }
    total += segs;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(worker);
  worker();
  for (auto &t : pool) t.join();
  if (segments) *segments = total.load();
  return 0;
}

int rto_trace(const rt_scene_view *scene, const rt_camera *cam, const rt_params *p, int col,
              int grow, long sample) {
  if (!scene || !cam || !p) return -1;
  const kscene sc = make_kscene(*scene);
  kctx k{&sc, cam, p, (uint32_t)p->seed ^ ((uint32_t)(p->seed >> 32) * 0x9E3779B9u),
         (p->flags & RT_FLAG_OPEN_INTERVAL) != 0, (p->flags & RT_FLAG_METAL_UNIT_VECTOR) != 0};
  g_trace = stdout;
  g_trace_sample = sample;
  float acc[3];
  kernel_pixel(k, col, grow, acc);
  std::fflush(stdout);
  g_trace = nullptr;
  g_trace_sample = -1;
  return 0;
}

int rto_reference_scene(int half_extent, double *rows, size_t capacity, size_t *n_out,
                        double *rng_next) {
  rng64 r;
  std::vector<dsphere> s;
  final_scene(r, half_extent, s);
  if (n_out) *n_out = s.size();
  if (rng_next) *rng_next = r();
  if (!rows) return 0;
  if (capacity < s.size()) return -1;
  for (size_t i = 0; i < s.size(); ++i) {
    double *q = rows + 9 * i;
    q[0] = s[i].kind;
    q[1] = s[i].c.x;
    q[2] = s[i].c.y;
    q[3] = s[i].c.z;
    q[4] = s[i].r;
    q[5] = s[i].albedo.x;
    q[6] = s[i].albedo.y;
    q[7] = s[i].albedo.z;
    q[8] = s[i].param;
  }
  return 0;
}

}  // extern "C"
