// tools/host_sanitize.cpp -- drives the library's host code under ASan + UBSan
// on the CPU (no device): the scene builders, both cameras, the BVH / layer-grid
// builder (rt_internal_accel_info), both tonemaps and the P3 / P6 writers, on
// the reference scenes and on ragged / degenerate inputs.  Built and run by
// tools/host_sanitize.sh; exits non-zero on any failed check (the sanitizers
// abort on their own findings).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <fcntl.h>
#include <unistd.h>
#include <vector>

#include "rt_internal.h"

#define CHECK(x)                                                    \
  do {                                                              \
    if (!(x)) {                                                     \
      std::fprintf(stderr, "check failed: %s (line %d)\n", #x, __LINE__); \
      std::exit(1);                                                 \
    }                                                               \
  } while (0)

struct scene {
  std::vector<float> cx, cy, cz, r, alb, par;
  std::vector<uint32_t> kind;
  rt_scene_buf buf(uint32_t cap) {
    cx.resize(cap), cy.resize(cap), cz.resize(cap), r.resize(cap), par.resize(cap);
    alb.resize(3 * (size_t)cap), kind.resize(cap);
    return rt_scene_buf{cap, 0, cx.data(), cy.data(), cz.data(), r.data(), kind.data(), alb.data(), par.data()};
  }
  rt_scene_view view(uint32_t n) const {
    return rt_scene_view{n, cx.data(), cy.data(), cz.data(), r.data(), kind.data(), alb.data(), par.data()};
  }
};

static void accel(const rt_scene_view &v, bool expect_layer) {
  // every grid placement (auto, LDS, cells in LDS, global) and a few cell scales
  for (int place = 0; place <= 3; ++place)
    for (double scale : {0.0, 0.5, 1.3}) {
      uint64_t info[RT_ACCEL_INFO_N];
      CHECK(rt_internal_accel_info(&v, place, scale, info, RT_ACCEL_INFO_N) == RT_OK);
      CHECK((info[2] != 0) == expect_layer);
      if (info[7]) CHECK(info[11] == 1 && info[12] == 1 && info[10] <= 15 && info[16] >= 1);
    }
  uint64_t two[2];
  CHECK(rt_internal_accel_info(&v, 0, 0.0, two, 2) == RT_OK);  // a short buffer is filled, no more
  CHECK(rt_internal_accel_info(&v, 4, 0.0, two, 2) != RT_OK);
}

int main() {
  // the final scene at several sizes (half extent 11: 486 spheres; 50: 10k)
  for (int he : {0, 1, 3, 11, 50}) {
    scene s;
    const uint32_t cap = (uint32_t)(4 * he * he + 8);
    rt_scene_buf b = s.buf(cap);
    double next = 0;
    CHECK(rt_scene_final(he, &b, &next) == RT_OK);
    CHECK(b.n <= cap);
    accel(s.view(b.n), he >= 11);
    // the grid fitter (RT_OPT_GRID_FIT's host model) for two frame geometries
    if (he == 11 || he == 50) {
      rt_camera cam;
      const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
      CHECK(rt_camera_cpu(from, at, up, 20.0, 16.0 / 9.0, 0.1, 10.0, &cam) == RT_OK);
      const rt_scene_view v = s.view(b.n);
      double scale = -1, costs[2 * 40];
      size_t n = 0;
      CHECK(rt_internal_grid_fit(&v, &cam, 3840, 2160, &scale, costs, 40, &n) == RT_OK);
      CHECK(scale > 0 && n >= 1 && n <= 31);
      CHECK(rt_internal_grid_fit(&v, &cam, 64, 64, &scale, nullptr, 0, &n) == RT_OK);
    }
  }
  {  // too small a buffer is refused
    scene s;
    rt_scene_buf b = s.buf(3);
    CHECK(rt_scene_final(11, &b, nullptr) != RT_OK);
  }
  {  // the five-sphere scene (no layer), and an empty scene
    scene s;
    rt_scene_buf b = s.buf(8);
    CHECK(rt_scene_five(&b) == RT_OK);
    accel(s.view(b.n), false);
    accel(s.view(0), false);
  }
  {  // a dense layer: 300 overlapping spheres in 1.5 x 1.5 (the builder shrinks cells or gives up)
    scene s;
    s.buf(300);
    for (int i = 0; i < 300; ++i) {
      s.cx[i] = 1.5f * (float)((i * 37) % 100) / 100.0f;
      s.cz[i] = 1.5f * (float)((i * 61) % 100) / 100.0f;
      s.cy[i] = 0.2f;
      s.r[i] = 0.2f;
      s.kind[i] = RT_LAMBERTIAN;
      s.alb[3 * i] = s.alb[3 * i + 1] = s.alb[3 * i + 2] = 0.5f;
    }
    uint64_t info[RT_ACCEL_INFO_N];
    const rt_scene_view v = s.view(300);
    CHECK(rt_internal_accel_info(&v, 0, 0.0, info, RT_ACCEL_INFO_N) == RT_OK);
    if (info[7]) CHECK(info[11] == 1 && info[12] == 1 && info[10] <= 15);
  }
  // cameras (both models, with and without a lens)
  rt_camera cam;
  const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  CHECK(rt_camera_cpu(from, at, up, 20.0, 16.0 / 9.0, 0.1, 10.0, &cam) == RT_OK);
  CHECK(rt_camera_gpu(from, at, up, 20.0, 1920, 1080, 0.6, 10.0, &cam) == RT_OK);
  // tonemaps (both modes) and the writers, on ragged sizes
  for (int w : {1, 7, 333}) {
    const int h = 5;
    std::vector<float> sums(3 * (size_t)w * h);
    for (size_t i = 0; i < sums.size(); ++i) sums[i] = (float)(i % 97) * 0.37f;
    std::vector<uint8_t> rgb(sums.size());
    for (int spp : {1, 10, 500}) {
      CHECK(rt_tonemap_u8_mode(sums.data(), (size_t)w * h, spp, RT_TONEMAP_CPU, rgb.data()) == RT_OK);
      CHECK(rt_tonemap_u8_mode(sums.data(), (size_t)w * h, spp, RT_TONEMAP_GPU, rgb.data()) == RT_OK);
    }
    const int fd = open("/dev/null", O_WRONLY);
    CHECK(fd >= 0);
    CHECK(rt_write_ppm(fd, rgb.data(), w, h, 0) == RT_OK);
    CHECK(rt_write_ppm(fd, rgb.data(), w, h, 1) == RT_OK);
    close(fd);
  }
  // launch plans (rt_internal_launch_plan): frames from one pixel to C4's,
  // spp up to the ABI's maximum, budgets from 1 sample to 2^40
  for (int w : {1, 9, 3840, 16384}) {
    for (int spp : {0, 1, 16, 2000, (1 << 24) - 1}) {
      for (double budget : {0.0, 1.0, 1e6, 4294967296.0, 1099511627776.0}) {
        rt_params p;
        std::memset(&p, 0, sizeof p);
        p.width = w;
        p.height = w;
        p.spp = spp;
        p.max_depth = 50;
        p.row_block = w;
        p.band_stride = 1;
        p.local_rows = w;
        p.flags = RT_FLAG_ACCEL_BVH | RT_FLAG_PILOT_SCHEDULE;
        uint64_t plan[RT_LAUNCH_PLAN_N];
        CHECK(rt_internal_launch_plan(&p, budget, plan, RT_LAUNCH_PLAN_N) == RT_OK);
        CHECK(plan[0] >= 1 && plan[1] >= 1 && plan[2] >= 1 && plan[4] == plan[0] * plan[1] && plan[4] <= 65536);
        CHECK(plan[0] <= plan[3] && (spp == 0 || plan[1] <= (uint64_t)spp));
      }
    }
  }
  std::printf("host_sanitize: ok\n");
  return 0;
}
