// oracle/ref_harness.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured
// as the product).  Builds the reference's own CPU tracer (src/cpu) from the
// sources where they lie under /root/reference, by textual inclusion, and adds
// a thin driver so the reference can be run at any image size and dump its
// scene / known-answer vectors.  Nothing of the reference is copied into this
// repository: the Makefile in this directory compiles this file with
// -I/root/reference/src/cpu and writes the binary to oracle/_ref/.
//
// What it reuses verbatim from the reference (by #include):
//   random_scene()            src/cpu/main.cc:32-76
//   ray_color()               src/cpu/main.cc:12-30
//   camera / get_ray          src/cpu/camera.h:8-34
//   write_color               src/cpu/color.h:8-23
//   sphere::hit, materials    src/cpu/sphere.h, src/cpu/material.h
//   random_double (mt19937)   src/cpu/rtweekend.h:27-31
// The render loop below restates src/cpu/main.cc:109-123 exactly (same draw
// order, same output formatting), so `render` is byte-identical to the
// reference binary with its compile-time constants patched.
//
// Usage:
//   ref_harness scene                       -> scene dump (%.17g), then "next <rnd>"
//   ref_harness render W ASPN ASPD SPP [DEPTH] [scene=final|five|file:PATH] [SKIP]
//                      [APERTURE FOCUS_DIST]
//        SKIP = number of random_double() draws discarded after the scene is
//        built (an independent stream, for the oracle's own noise floor)
//        file:PATH = spheres read from a dump in `scene`'s format (e.g. the
//        10 000-sphere stress scene), built with the reference's own
//        sphere / lambertian / metal / dielectric classes
//        APERTURE FOCUS_DIST override the camera's lens (depth of field)
//        PPM (P3) on stdout; on stderr a JSON stats line with samples,
//        segments (= hittable_list::hit calls), sphere_tests and seconds.
//   ref_harness hits PATH   -> sphere::hit (t_min 0.001) on the cases in PATH,
//        one `o[3] d[3] c[3] r` per line, as kat-format JSON lines
//   ref_harness cameras PATH -> the camera basis (camera.h:8-26) for each
//        `lookfrom[3] lookat[3] vup[3] vfov aspect aperture focus` line of PATH
//   ref_harness colors PATH  -> write_color's line for each `r g b spp` line
//   ref_harness vectors PATH -> reflect / refract / reflectance for each
//        `v[3] n[3] eta cosine ref_idx` line
//   ref_harness kat                         -> known-answer vectors (JSON lines)
// standard headers first so the access override below touches only the
// reference's own classes
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <limits>
#include <memory>
#include <random>
#include <sstream>
#include <string>
#include <vector>
#define private public  // test access to camera / dielectric internals
#define main ref_main
#include "main.cc"
#undef main
#undef private

namespace {

struct counting_world : hittable {
  const hittable_list &w;
  mutable unsigned long long calls = 0;
  explicit counting_world(const hittable_list &world) : w(world) {}
  bool hit(const ray &r, double t_min, double t_max,
           hit_record &rec) const override {
    ++calls;
    return w.hit(r, t_min, t_max, rec);
  }
};

const char *mat_kind(const material *m, double *a, double *param) {
  if (auto l = dynamic_cast<const lambertian *>(m)) {
    a[0] = l->albedo.x(); a[1] = l->albedo.y(); a[2] = l->albedo.z();
    *param = 0;
    return "L";
  }
  if (auto me = dynamic_cast<const metal *>(m)) {
    a[0] = me->albedo.x(); a[1] = me->albedo.y(); a[2] = me->albedo.z();
    *param = me->fuzz;
    return "M";
  }
  if (auto d = dynamic_cast<const dielectric *>(m)) {
    a[0] = a[1] = a[2] = 1.0;
    *param = d->ir;
    return "D";
  }
  return "?";
}

void dump_world(const hittable_list &world) {
  for (const auto &obj : world.objects) {
    auto s = std::dynamic_pointer_cast<sphere>(obj);
    double a[3], p;
    const char *k = mat_kind(s->mat_ptr.get(), a, &p);
    std::printf("%s %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", k,
                s->center.x(), s->center.y(), s->center.z(), s->radius, a[0],
                a[1], a[2], p);
  }
}

// Book scene used by archive-gpu/image22 (5 spheres incl. a hollow glass
// sphere of negative radius), expressed with the src/cpu classes.
hittable_list five_scene() {
  hittable_list world;
  auto ground = make_shared<lambertian>(color(0.8, 0.8, 0.0));
  auto center = make_shared<lambertian>(color(0.1, 0.2, 0.5));
  auto left = make_shared<dielectric>(1.5);
  auto right = make_shared<metal>(color(0.8, 0.6, 0.2), 0.0);
  world.add(make_shared<sphere>(point3(0.0, -100.5, -1.0), 100.0, ground));
  world.add(make_shared<sphere>(point3(0.0, 0.0, -1.0), 0.5, center));
  world.add(make_shared<sphere>(point3(-1.0, 0.0, -1.0), 0.5, left));
  world.add(make_shared<sphere>(point3(-1.0, 0.0, -1.0), -0.4, left));
  world.add(make_shared<sphere>(point3(1.0, 0.0, -1.0), 0.5, right));
  return world;
}

// "K cx cy cz r a0 a1 a2 param" per line (K = L | M | D), as dump_world prints
hittable_list file_scene(const char *path) {
  hittable_list world;
  FILE *f = std::fopen(path, "r");
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path);
    std::exit(2);
  }
  char k[8];
  double c[3], r, a[3], p;
  while (std::fscanf(f, "%7s %lf %lf %lf %lf %lf %lf %lf %lf", k, &c[0], &c[1], &c[2], &r, &a[0], &a[1], &a[2],
                     &p) == 9) {
    shared_ptr<material> m;
    if (k[0] == 'L') m = make_shared<lambertian>(color(a[0], a[1], a[2]));
    else if (k[0] == 'M') m = make_shared<metal>(color(a[0], a[1], a[2]), p);
    else m = make_shared<dielectric>(p);
    world.add(make_shared<sphere>(point3(c[0], c[1], c[2]), r, m));
  }
  std::fclose(f);
  return world;
}

int cmd_scene() {
  auto world = random_scene();
  dump_world(world);
  std::printf("next %.17g\n", random_double());
  return 0;
}

int cmd_render(int argc, char **argv) {
  if (argc < 6) return 2;
  const int image_width = std::atoi(argv[2]);
  const double aspect_ratio = std::atof(argv[3]) / std::atof(argv[4]);
  const int image_height = static_cast<int>(image_width / aspect_ratio);
  const int samples_per_pixel = std::atoi(argv[5]);
  const int max_depth = argc > 6 ? std::atoi(argv[6]) : 50;
  const std::string scene = argc > 7 ? argv[7] : "final";
  const long long skip = argc > 8 ? std::atoll(argv[8]) : 0;

  hittable_list world;
  point3 lookfrom(13, 2, 3), lookat(0, 0, 0);
  double vfov = 20, aperture = 0.1, dist_to_focus = 10.0;
  if (scene == "five") {
    world = five_scene();
    lookfrom = point3(-2, 2, 1);
    lookat = point3(0, 0, -1);
    aperture = 0.0;
    dist_to_focus = 3.4;
  } else if (scene.compare(0, 5, "file:") == 0) {
    world = file_scene(scene.c_str() + 5);
  } else {
    world = random_scene();
  }
  if (argc > 10) {
    aperture = std::atof(argv[9]);
    dist_to_focus = std::atof(argv[10]);
  }
  for (long long k = 0; k < skip; ++k) (void)random_double();
  vec3 vup(0, 1, 0);
  camera cam(lookfrom, lookat, vup, vfov, aspect_ratio, aperture, dist_to_focus);
  counting_world counted(world);

  auto start = std::chrono::steady_clock::now();
  std::cout << "P3\n" << image_width << " " << image_height << "\n255\n";
  for (int j = image_height - 1; j >= 0; --j) {
    for (int i = 0; i < image_width; ++i) {
      color pixel_color(0, 0, 0);
      for (int s = 0; s < samples_per_pixel; ++s) {
        auto u = (i + random_double()) / (image_width - 1);
        auto v = (j + random_double()) / (image_height - 1);
        ray r = cam.get_ray(u, v);
        pixel_color += ray_color(r, counted, max_depth);
      }
      write_color(std::cout, pixel_color, samples_per_pixel);
    }
  }
  std::cout.flush();
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count();
  unsigned long long samples = 1ull * image_width * image_height * samples_per_pixel;
  std::fprintf(stderr,
               "{\"width\": %d, \"height\": %d, \"spp\": %d, \"depth\": %d, "
               "\"spheres\": %zu, \"samples\": %llu, \"segments\": %llu, "
               "\"sphere_tests\": %llu, \"seconds\": %.6f}\n",
               image_width, image_height, samples_per_pixel, max_depth,
               world.objects.size(), samples, counted.calls,
               counted.calls * (unsigned long long)world.objects.size(), secs);
  return 0;
}

void pv(const char *name, const vec3 &v) {
  std::printf("\"%s\": [%.17g, %.17g, %.17g]", name, v.x(), v.y(), v.z());
}

int cmd_kat() {
  // camera basis for the final-scene camera at aspect 16/9 (camera.h:8-26)
  {
    camera cam(point3(13, 2, 3), point3(0, 0, 0), vec3(0, 1, 0), 20, 16.0 / 9.0, 0.1, 10.0);
    std::printf("{\"kind\": \"camera\", \"aspect\": %.17g, ", 16.0 / 9.0);
    pv("origin", cam.origin); std::printf(", ");
    pv("lower_left_corner", cam.lower_left_corner); std::printf(", ");
    pv("horizontal", cam.horizontal); std::printf(", ");
    pv("vertical", cam.vertical); std::printf(", ");
    pv("u", cam.u); std::printf(", ");
    pv("v", cam.v); std::printf(", ");
    pv("w", cam.w);
    std::printf(", \"lens_radius\": %.17g}\n", cam.lens_radius);
  }
  // sphere::hit (sphere.h:24-51) on a fixed set of rays
  {
    struct { double o[3], d[3], c[3], r; } cases[] = {
        {{0, 0, 0}, {0, 0, -1}, {0, 0, -3}, 1.0},
        {{0, 0, 0}, {0, 0, -2}, {0, 0, -3}, 1.0},        // unnormalised dir
        {{0, 0, -3}, {0, 1, 0}, {0, 0, -3}, 1.0},        // from inside
        {{0, 0, 0}, {0, 1, 0}, {0, 0, -3}, 1.0},         // miss
        {{13, 2, 3}, {-13, -2, -3}, {0, 1, 0}, 1.0},
        {{5, 0.001, 5}, {0.3, 0.9, -0.1}, {0, -1000, 0}, 1000.0},
        {{-1, 0, 0}, {1, 0, -1}, {-1, 0, -1}, -0.4},     // negative radius
        {{0, 0.2, 0}, {1, 0, 0}, {2, 0.2, 0}, 0.2},
    };
    for (auto &c : cases) {
      auto mat = make_shared<lambertian>(color(0.5, 0.5, 0.5));
      sphere s(point3(c.c[0], c.c[1], c.c[2]), c.r, mat);
      ray r(point3(c.o[0], c.o[1], c.o[2]), vec3(c.d[0], c.d[1], c.d[2]));
      hit_record rec;
      bool h = s.hit(r, 0.001, infinity, rec);
      std::printf("{\"kind\": \"sphere_hit\", \"o\": [%.17g, %.17g, %.17g], \"d\": [%.17g, %.17g, %.17g], "
                  "\"c\": [%.17g, %.17g, %.17g], \"r\": %.17g, \"hit\": %s",
                  c.o[0], c.o[1], c.o[2], c.d[0], c.d[1], c.d[2], c.c[0], c.c[1], c.c[2], c.r,
                  h ? "true" : "false");
      if (h) {
        std::printf(", \"t\": %.17g, ", rec.t);
        pv("p", rec.p); std::printf(", ");
        pv("normal", rec.normal);
        std::printf(", \"front_face\": %s", rec.front_face ? "true" : "false");
      }
      std::printf("}\n");
    }
  }
  // reflect / refract / reflectance (vec3.h:122-131, material.h:82-87)
  {
    vec3 vs[] = {unit_vector(vec3(1, -1, 0)), unit_vector(vec3(0.3, -0.9, 0.2)),
                 unit_vector(vec3(-0.7, -0.1, 0.5))};
    vec3 n(0, 1, 0);
    for (auto &v : vs) {
      std::printf("{\"kind\": \"reflect\", ");
      pv("v", v); std::printf(", "); pv("n", n); std::printf(", ");
      pv("out", reflect(v, n)); std::printf("}\n");
      for (double eta : {1.0 / 1.5, 1.5}) {
        std::printf("{\"kind\": \"refract\", \"eta\": %.17g, ", eta);
        pv("v", v); std::printf(", "); pv("n", n); std::printf(", ");
        pv("out", refract(v, n, eta)); std::printf("}\n");
      }
    }
    for (double cosine : {0.0, 0.1, 0.5, 0.9, 1.0})
      for (double idx : {1.0 / 1.5, 1.5})
        std::printf("{\"kind\": \"reflectance\", \"cosine\": %.17g, \"ref_idx\": %.17g, \"out\": %.17g}\n",
                    cosine, idx, dielectric::reflectance(cosine, idx));
  }
  // write_color (color.h:8-23)
  {
    double sums[][3] = {{0, 0, 0}, {10, 5, 2.5}, {0.001, 9.99, 10}, {123.4, 0.5, 77.7}, {1e9, 1e-9, 3.3}};
    int spps[] = {10, 10, 10, 500, 7};
    for (int k = 0; k < 5; ++k) {
      std::ostringstream os;
      write_color(os, color(sums[k][0], sums[k][1], sums[k][2]), spps[k]);
      std::string line = os.str();
      line.pop_back();
      std::printf("{\"kind\": \"write_color\", \"sum\": [%.17g, %.17g, %.17g], \"spp\": %d, \"out\": \"%s\"}\n",
                  sums[k][0], sums[k][1], sums[k][2], spps[k], line.c_str());
    }
  }
  return 0;
}

// sphere::hit (sphere.h:24-51) on cases read from a file, one per line:
// o[3] d[3] c[3] r -> one kat-format JSON line each (t_min 0.001, t_max inf)
int cmd_hits(const char *path) {
  FILE *f = std::fopen(path, "r");
  if (!f) return 2;
  double v[10];
  while (std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf %lf", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5],
                     &v[6], &v[7], &v[8], &v[9]) == 10) {
    auto mat = make_shared<lambertian>(color(0.5, 0.5, 0.5));
    sphere s(point3(v[6], v[7], v[8]), v[9], mat);
    ray r(point3(v[0], v[1], v[2]), vec3(v[3], v[4], v[5]));
    hit_record rec;
    const bool h = s.hit(r, 0.001, infinity, rec);
    std::printf("{\"kind\": \"sphere_hit\", \"o\": [%.17g, %.17g, %.17g], \"d\": [%.17g, %.17g, %.17g], "
                "\"c\": [%.17g, %.17g, %.17g], \"r\": %.17g, \"hit\": %s",
                v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], h ? "true" : "false");
    if (h) {
      std::printf(", \"t\": %.17g, ", rec.t);
      pv("p", rec.p); std::printf(", ");
      pv("normal", rec.normal);
      std::printf(", \"front_face\": %s", rec.front_face ? "true" : "false");
    }
    std::printf("}\n");
  }
  std::fclose(f);
  return 0;
}

// camera (camera.h:8-26) on parameter sets read from a file, one per line:
// lookfrom[3] lookat[3] vup[3] vfov aspect aperture focus_dist -> its basis
int cmd_cameras(const char *path) {
  FILE *f = std::fopen(path, "r");
  if (!f) return 2;
  double v[13];
  while (std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf %lf", &v[0], &v[1], &v[2], &v[3], &v[4],
                     &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12]) == 13) {
    camera cam(point3(v[0], v[1], v[2]), point3(v[3], v[4], v[5]), vec3(v[6], v[7], v[8]), v[9], v[10], v[11],
               v[12]);
    std::printf("{\"kind\": \"camera\", \"args\": [");
    for (int k = 0; k < 13; ++k) std::printf(k ? ", %.17g" : "%.17g", v[k]);
    std::printf("], ");
    pv("origin", cam.origin); std::printf(", ");
    pv("lower_left_corner", cam.lower_left_corner); std::printf(", ");
    pv("horizontal", cam.horizontal); std::printf(", ");
    pv("vertical", cam.vertical); std::printf(", ");
    pv("u", cam.u); std::printf(", ");
    pv("v", cam.v); std::printf(", ");
    pv("w", cam.w);
    std::printf(", \"lens_radius\": %.17g}\n", cam.lens_radius);
  }
  std::fclose(f);
  return 0;
}

// write_color (color.h:8-23) on sums read from a file, one `r g b spp` per
// line -> the reference's output line for each
int cmd_colors(const char *path) {
  FILE *f = std::fopen(path, "r");
  if (!f) return 2;
  double r, g, b;
  int spp;
  while (std::fscanf(f, "%lf %lf %lf %d", &r, &g, &b, &spp) == 4) {
    std::ostringstream os;
    write_color(os, color(r, g, b), spp);
    std::fputs(os.str().c_str(), stdout);
  }
  std::fclose(f);
  return 0;
}

// reflect / refract (vec3.h:124-131) and dielectric::reflectance
// (material.h:82-87) on cases read from a file, one `v[3] n[3] eta cosine
// ref_idx` per line -> kat-format JSON lines (reflect, refract, reflectance)
int cmd_vectors(const char *path) {
  FILE *f = std::fopen(path, "r");
  if (!f) return 2;
  double a[9];
  while (std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf", &a[0], &a[1], &a[2], &a[3], &a[4], &a[5], &a[6],
                     &a[7], &a[8]) == 9) {
    const vec3 v(a[0], a[1], a[2]), n(a[3], a[4], a[5]);
    std::printf("{\"kind\": \"reflect\", ");
    pv("v", v); std::printf(", "); pv("n", n); std::printf(", ");
    pv("out", reflect(v, n)); std::printf("}\n");
    std::printf("{\"kind\": \"refract\", \"eta\": %.17g, ", a[6]);
    pv("v", v); std::printf(", "); pv("n", n); std::printf(", ");
    pv("out", refract(v, n, a[6])); std::printf("}\n");
    std::printf("{\"kind\": \"reflectance\", \"cosine\": %.17g, \"ref_idx\": %.17g, \"out\": %.17g}\n",
                a[7], a[8], dielectric::reflectance(a[7], a[8]));
  }
  std::fclose(f);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s scene|render|kat ...\n", argv[0]);
    return 2;
  }
  if (!std::strcmp(argv[1], "scene")) return cmd_scene();
  if (!std::strcmp(argv[1], "render")) return cmd_render(argc, argv);
  if (!std::strcmp(argv[1], "kat")) return cmd_kat();
  if (!std::strcmp(argv[1], "hits") && argc > 2) return cmd_hits(argv[2]);
  if (!std::strcmp(argv[1], "cameras") && argc > 2) return cmd_cameras(argv[2]);
  if (!std::strcmp(argv[1], "colors") && argc > 2) return cmd_colors(argv[2]);
  if (!std::strcmp(argv[1], "vectors") && argc > 2) return cmd_vectors(argv[2]);
  return 2;
}
