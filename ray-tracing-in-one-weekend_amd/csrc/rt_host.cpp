// rt_host.cpp -- host-side pieces of the render path that run once per frame:
// scene construction, camera setup, tonemap and PPM output.  Pure C++17, no
// HIP calls (the device half lives in rt_kernel.hip and rt_api.cpp).
//
// Scene construction restates random_scene() (src/cpu/main.cc:32-76) with the
// std::mt19937 draws SEQUENCED EXPLICITLY in the order g++ 11 evaluates the
// reference's argument lists, so the scene is the same whatever compiler
// builds this file (hipcc/clang evaluates left-to-right and would otherwise
// produce a different 484-sphere scene -- SURVEY 0.2 / 8a-1).
#include "rt_internal.h"

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

// src/cpu/rtweekend.h:27-36: a single static mt19937 (default seed 5489)
// feeding uniform_real_distribution<double>(0,1).
struct ref_rng {
  std::mt19937 gen;
  std::uniform_real_distribution<double> dist{0.0, 1.0};
  double next() { return dist(gen); }
  double next(double lo, double hi) { return lo + (hi - lo) * next(); }
};

struct dvec3 {
  double x, y, z;
};

// vec3::random() (src/cpu/vec3.h:11-13) as g++ evaluates it: the three
// arguments of the vec3 constructor are drawn right to left (z, y, x).
dvec3 random_vec(ref_rng &r) {
  dvec3 v;
  v.z = r.next();
  v.y = r.next();
  v.x = r.next();
  return v;
}

dvec3 random_vec(ref_rng &r, double lo, double hi) {
  dvec3 v;
  v.z = r.next(lo, hi);
  v.y = r.next(lo, hi);
  v.x = r.next(lo, hi);
  return v;
}

struct scene_writer {
  rt_scene_buf *out;
  bool overflow = false;
  void add(double cx, double cy, double cz, double r, rt_material_kind k,
           double ar, double ag, double ab, double param) {
    if (out->n >= out->capacity) {
      overflow = true;
      return;
    }
    uint32_t i = out->n++;
    out->cx[i] = (float)cx;
    out->cy[i] = (float)cy;
    out->cz[i] = (float)cz;
    out->radius[i] = (float)r;
    out->mat_kind[i] = (uint32_t)k;
    out->albedo_rgb[3 * i + 0] = (float)ar;
    out->albedo_rgb[3 * i + 1] = (float)ag;
    out->albedo_rgb[3 * i + 2] = (float)ab;
    out->mat_param[i] = (float)param;
  }
};

bool buf_ok(const rt_scene_buf *b) {
  return b && b->cx && b->cy && b->cz && b->radius && b->mat_kind &&
         b->albedo_rgb && b->mat_param;
}

struct v3 {
  double x, y, z;
};
v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
v3 scale(double t, v3 a) { return {t * a.x, t * a.y, t * a.z}; }
double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
v3 cross(v3 u, v3 v) {
  return {u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x};
}
v3 unit(v3 v) { return scale(1 / std::sqrt(dot(v, v)), v); }
v3 ld(const double *p) { return {p[0], p[1], p[2]}; }
void st(float *d, v3 v) {
  d[0] = (float)v.x;
  d[1] = (float)v.y;
  d[2] = (float)v.z;
}

constexpr double kPi = 3.1415926535897932385;

thread_local int g_last_hip_error = 0;

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

const char *rt_strerror(int status) {
  switch (status) {
    case RT_OK: return "ok";
    case RT_ERR_INVALID: return "invalid argument";
    case RT_ERR_HIP: return "HIP runtime error";
    case RT_ERR_NOMEM: return "out of memory";
    case RT_ERR_NO_DEVICE: return "no such HIP device";
    case RT_ERR_CAPACITY: return "output buffer too small";
    case RT_ERR_NO_SCENE: return "no scene uploaded";
    case RT_ERR_IO: return "I/O error";
    default: return "unknown status";
  }
}

int rt_last_hip_error(void) { return g_last_hip_error; }
void rt_internal_set_hip_error(int e) { g_last_hip_error = e; }

int rt_scene_final(int half_extent, rt_scene_buf *out, double *rng_next) {
  if (!buf_ok(out) || half_extent < 0 || half_extent > 4096) return RT_ERR_INVALID;
  out->n = 0;
  scene_writer w{out};
  ref_rng rng;
  // main.cc:35-36 ground
  w.add(0, -1000, 0, 1000, RT_LAMBERTIAN, 0.5, 0.5, 0.5, 0);
  // main.cc:38-64 grid
  for (int a = -half_extent; a < half_extent; a++) {
    for (int b = -half_extent; b < half_extent; b++) {
      double choose_mat = rng.next();                 // main.cc:40
      double cz = b + 0.9 * rng.next();               // main.cc:41, drawn first by g++
      double cx = a + 0.9 * rng.next();
      double cy = 0.2;
      double dx = cx - 4, dy = cy - 0.2, dz = cz - 0;  // main.cc:43
      if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {
        if (choose_mat < 0.8) {
          // main.cc:48: color::random() * color::random(); g++ evaluates the
          // right operand first (pinned by tests/golden/scene_final_gcc.txt)
          dvec3 rhs = random_vec(rng);
          dvec3 lhs = random_vec(rng);
          w.add(cx, cy, cz, 0.2, RT_LAMBERTIAN, lhs.x * rhs.x, lhs.y * rhs.y,
                lhs.z * rhs.z, 0);
        } else if (choose_mat < 0.95) {
          dvec3 albedo = random_vec(rng, 0.5, 1);  // main.cc:53
          double fuzz = rng.next(0, 0.5);          // main.cc:54
          // metal::metal clamps fuzz to 1 (material.h:38)
          w.add(cx, cy, cz, 0.2, RT_METAL, albedo.x, albedo.y, albedo.z,
                fuzz < 1 ? fuzz : 1);
        } else {
          w.add(cx, cy, cz, 0.2, RT_DIELECTRIC, 1, 1, 1, 1.5);  // main.cc:59
        }
      }
    }
  }
  // main.cc:66-73
  w.add(0, 1, 0, 1.0, RT_DIELECTRIC, 1, 1, 1, 1.5);
  w.add(-4, 1, 0, 1.0, RT_LAMBERTIAN, 0.4, 0.2, 0.1, 0);
  w.add(4, 1, 0, 1.0, RT_METAL, 0.7, 0.6, 0.5, 0.0);
  if (rng_next) *rng_next = rng.next();
  return w.overflow ? RT_ERR_CAPACITY : RT_OK;
}

int rt_scene_five(rt_scene_buf *out) {
  if (!buf_ok(out)) return RT_ERR_INVALID;
  out->n = 0;
  scene_writer w{out};
  // archive-gpu/image22/main.cu:23-38
  w.add(0.0, -100.5, -1.0, 100.0, RT_LAMBERTIAN, 0.8, 0.8, 0.0, 0);
  w.add(0.0, 0.0, -1.0, 0.5, RT_LAMBERTIAN, 0.1, 0.2, 0.5, 0);
  w.add(-1.0, 0.0, -1.0, 0.5, RT_DIELECTRIC, 1, 1, 1, 1.5);
  w.add(-1.0, 0.0, -1.0, -0.4, RT_DIELECTRIC, 1, 1, 1, 1.5);
  w.add(1.0, 0.0, -1.0, 0.5, RT_METAL, 0.8, 0.6, 0.2, 0.0);
  return w.overflow ? RT_ERR_CAPACITY : RT_OK;
}

int rt_camera_cpu(const double lookfrom[3], const double lookat[3],
                  const double vup[3], double vfov_deg, double aspect,
                  double aperture, double focus_dist, rt_camera *out) {
  if (!lookfrom || !lookat || !vup || !out || !(aspect > 0)) return RT_ERR_INVALID;
  // camera.h:8-26, same operation order in fp64
  double theta = vfov_deg * kPi / 180.0;
  double h = std::tan(theta / 2);
  double viewport_height = 2.0 * h;
  double viewport_width = aspect * viewport_height;
  v3 w = unit(sub(ld(lookfrom), ld(lookat)));
  v3 u = unit(cross(ld(vup), w));
  v3 v = cross(w, u);
  v3 origin = ld(lookfrom);
  v3 horizontal = scale(focus_dist * viewport_width, u);
  v3 vertical = scale(focus_dist * viewport_height, v);
  v3 llc = sub(sub(sub(origin, scale(1 / 2.0, horizontal)), scale(1 / 2.0, vertical)),
               scale(focus_dist, w));
  double lens_radius = aperture / 2;
  std::memset(out, 0, sizeof(*out));
  out->model = RT_CAMERA_CPU;
  out->has_lens = lens_radius != 0.0;
  st(out->eye, origin);
  st(out->corner, llc);
  st(out->horiz, horizontal);
  st(out->vert, vertical);
  st(out->lens_u, scale(lens_radius, u));
  st(out->lens_v, scale(lens_radius, v));
  return RT_OK;
}

int rt_camera_gpu(const double lookfrom[3], const double lookat[3],
                  const double vup[3], double vfov_deg, int width, int height,
                  double defocus_angle_deg, double focus_dist, rt_camera *out) {
  if (!lookfrom || !lookat || !vup || !out || width < 1 || height < 1)
    return RT_ERR_INVALID;
  // new_camera, src/gpu/camera.h:75-109
  double theta = vfov_deg / 180.0 * kPi;
  double h = std::tan(theta / 2.0);
  double viewport_height = 2.0 * h * focus_dist;
  double viewport_width = viewport_height * ((double)width / height);
  v3 w = unit(sub(ld(lookfrom), ld(lookat)));
  v3 u = unit(cross(ld(vup), w));
  v3 v = cross(w, u);
  v3 center = ld(lookfrom);
  v3 viewport_u = scale(viewport_width, u);
  v3 viewport_v = scale(-viewport_height, v);
  v3 du = scale(1.0 / width, viewport_u);
  v3 dv = scale(1.0 / height, viewport_v);
  v3 upper_left = sub(sub(sub(center, scale(focus_dist, w)), scale(0.5, viewport_u)),
                      scale(0.5, viewport_v));
  v3 p00 = {upper_left.x + 0.5 * (du.x + dv.x), upper_left.y + 0.5 * (du.y + dv.y),
            upper_left.z + 0.5 * (du.z + dv.z)};
  double defocus_radius = focus_dist * std::tan(defocus_angle_deg / 2.0 / 180.0 * kPi);
  std::memset(out, 0, sizeof(*out));
  out->model = RT_CAMERA_GPU;
  out->has_lens = defocus_angle_deg > 0.0;  // camera.h:161-163
  st(out->eye, center);
  st(out->corner, p00);
  st(out->horiz, du);
  st(out->vert, dv);
  st(out->lens_u, scale(defocus_radius, u));
  st(out->lens_v, scale(defocus_radius, v));
  return RT_OK;
}

}  // extern "C"

namespace {

// host worker count for the output helpers: at most 16 threads, one per
// ~4 M channels, 1 for small frames
unsigned host_threads(size_t work) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  return (unsigned)std::max<size_t>(1, std::min<size_t>({(size_t)hw, (size_t)16, work >> 22}));
}

template <class F>
void parallel_ranges(size_t n, F f) {
  const unsigned t = host_threads(n);
  if (t <= 1) {
    f((size_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  for (unsigned k = 0; k < t; ++k) th.emplace_back(f, n * k / t, n * (k + 1) / t);
  for (auto &x : th) x.join();
}

// write_color, src/cpu/color.h:8-23 (fp64)
inline uint8_t level_cpu(float s, double scale) {
  double x = std::sqrt(scale * (double)s);
  if (x < 0.0) x = 0.0;
  if (x > 0.999) x = 0.999;
  if (!(x == x)) x = 0.0;  // NaN sums (never produced) map to 0
  return (uint8_t)(int)(256 * x);
}

// write_color, src/gpu/color.h:16-38 (fp32: r *= 1.0f/spp, sqrtf, interval(0, 0.999f).clamp)
inline uint8_t level_gpu(float s, float scale) {
  float x = std::sqrt(s * scale);
  if (x < 0.000f) x = 0.000f;
  if (x > 0.999f) x = 0.999f;
  if (!(x == x)) x = 0.0f;
  return (uint8_t)(int)(256.0f * x);
}

bool write_all(int fd, const char *p, size_t left) {
  while (left) {
    ssize_t k = ::write(fd, p, left);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += k;
    left -= (size_t)k;
  }
  return true;
}

}  // namespace

extern "C" {

int rt_tonemap_u8_mode(const float *sums_rgb, size_t n_pixels, int spp, int mode, uint8_t *out_rgb) {
  if ((!sums_rgb || !out_rgb) && n_pixels) return RT_ERR_INVALID;
  if (spp < 1 || (mode != RT_TONEMAP_CPU && mode != RT_TONEMAP_GPU)) return RT_ERR_INVALID;
  const double scale = 1.0 / spp;
  const float scale_f = 1.0f / (float)spp;
  parallel_ranges(3 * n_pixels, [&](size_t b, size_t e) {
    if (mode == RT_TONEMAP_CPU)
      for (size_t i = b; i < e; ++i) out_rgb[i] = level_cpu(sums_rgb[i], scale);
    else
      for (size_t i = b; i < e; ++i) out_rgb[i] = level_gpu(sums_rgb[i], scale_f);
  });
  return RT_OK;
}

int rt_tonemap_u8(const float *sums_rgb, size_t n_pixels, int spp, uint8_t *out_rgb) {
  return rt_tonemap_u8_mode(sums_rgb, n_pixels, spp, RT_TONEMAP_CPU, out_rgb);
}

int rt_write_ppm(int fd, const uint8_t *rgb, int width, int height, int binary) {
  if (fd < 0 || width < 0 || height < 0 || (!rgb && width && height)) return RT_ERR_INVALID;
  // both references print "P3\nW H\n255\n" (src/cpu/main.cc:109,
  // src/gpu/camera.h:201)
  const std::string head = std::string(binary ? "P6\n" : "P3\n") + std::to_string(width) + " " +
                           std::to_string(height) + "\n255\n";
  if (!write_all(fd, head.data(), head.size())) return RT_ERR_IO;
  const size_t n = (size_t)width * height;
  if (binary) return write_all(fd, reinterpret_cast<const char *>(rgb), 3 * n) ? RT_OK : RT_ERR_IO;
  // P3: "r g b\n" per pixel (color.h:20-22).  Chunks of kChunk pixels are
  // formatted by up to 16 threads into their own buffers and written in
  // order; memory stays at threads x kChunk x 12 bytes whatever the frame.
  static constexpr size_t kChunk = 1 << 16;
  struct digits {
    char c[4];
    uint8_t len;
  };
  static const std::vector<digits> tab = [] {
    std::vector<digits> t(256);
    for (int v = 0; v < 256; ++v) t[v].len = (uint8_t)std::snprintf(t[v].c, 4, "%d", v);
    return t;
  }();
  auto format = [&](size_t b, size_t e, std::string &out) {
    out.resize(12 * (e - b));
    char *p = &out[0];
    for (size_t i = b; i < e; ++i) {
      for (int k = 0; k < 3; ++k) {
        const digits &d = tab[rgb[3 * i + k]];
        std::memcpy(p, d.c, 4);  // (the table entry is padded; only len bytes count)
        p += d.len;
        *p++ = k < 2 ? ' ' : '\n';
      }
    }
    out.resize((size_t)(p - out.data()));
  };
  const size_t n_chunks = (n + kChunk - 1) / kChunk;
  const unsigned t = (unsigned)std::max<size_t>(1, std::min<size_t>(host_threads(3 * n), n_chunks));
  std::vector<std::string> buf(t);
  for (size_t c0 = 0; c0 < n_chunks; c0 += t) {
    const size_t m = std::min<size_t>(t, n_chunks - c0);
    auto job = [&](size_t j) { format((c0 + j) * kChunk, std::min(n, (c0 + j + 1) * kChunk), buf[j]); };
    if (m == 1) {
      job(0);
    } else {
      std::vector<std::thread> th;
      for (size_t j = 0; j < m; ++j) th.emplace_back(job, j);
      for (auto &x : th) x.join();
    }
    for (size_t j = 0; j < m; ++j)
      if (!write_all(fd, buf[j].data(), buf[j].size())) return RT_ERR_IO;
  }
  return RT_OK;
}

}  // extern "C"
