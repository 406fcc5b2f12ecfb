// cli.cpp -- drop-in process surface for cpu_ray_tracer / gpu_ray_tracer.
//
// Same conventions as the reference executables: P3 PPM on stdout, progress
// and timing on stderr (src/cpu/main.cc:103-132, src/gpu/main.cu:121-139),
// exit code 99 on a device error (src/gpu/cuda_utility.h:8-18).  The
// personality is chosen by argv[0]:
//   cpu_ray_tracer : 1200x800 (3:2), 500 spp, depth 50, src/cpu camera and
//                    semantics (src/cpu/main.cc:82-99)
//   gpu_ray_tracer : 1920x1080 (16:9), 500 spp, depth 50, src/gpu camera
//                    (defocus 0.6 deg) and semantics, seed = time(nullptr)
//                    (src/gpu/main.cu:88, src/gpu/camera.h:58-71)
//   rtow           : cpu_ray_tracer defaults
// Everything renders on the GPU through librtow.so; flags override defaults:
//   --width N --height N --spp N --depth N --seed N --spheres K (grid half
//   extent; 11 = reference, 50 = 10k spheres) --scene final|five
//   --camera cpu|gpu --semantics cpu|gpu --accel bvh|scan --gpus N --device N
//   --devices D0,D1,... --gather rccl|host --out FILE --p6 --quiet
// With --gpus N > 1 the frame is split into interleaved 8-row bands, one
// context and stream per device; each device tonemaps its tile to bytes
// (rt_tonemap_async) and the byte tiles are gathered to device 0 with one
// RCCL ncclGather over xGMI (single process, ncclCommInitAll); device 0's
// gathered frame is copied to the host once.  --gather host copies each tile
// back instead (no RCCL); --gather rccl forces the RCCL path also on 1 GPU.
// --devices names the device of each band; a device may repeat (bands on one
// GPU, host gather only: RCCL takes one rank per device), which runs the
// N-band split, per-band contexts and the assembly on a single-GPU machine.
#include <fcntl.h>
#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "rt.h"

namespace {

struct options {
  int width = 1200, height = 800, spp = 500, depth = 50;
  unsigned long long seed = 0;
  bool seed_set = false;
  int half_extent = 11;
  std::string scene = "final";
  int camera = RT_CAMERA_CPU;
  unsigned flags = 0;
  bool bvh = true;  // BVH walk (bit-identical to the scan)
  int gpus = 1, device = 0;
  std::vector<int> devices;  // --devices: the device of each band (default 0..gpus-1)
  std::string gather = "auto";  // auto: rccl when gpus > 1
  std::string out;
  bool p6 = false, quiet = false;
  double launch_samples = 0.0;  // RT_OPT_LAUNCH_SAMPLES (0: the library's default)
};

[[noreturn]] void die(const char *what, int st) {
  std::fprintf(stderr, "rtow error = %d (%s) at '%s'\n", st, rt_strerror(st), what);
  std::exit(99);  // src/gpu/cuda_utility.h:16
}

void check(int st, const char *what) {
  if (st != RT_OK) die(what, st);
}

[[noreturn]] void usage(const char *argv0) {
  std::fprintf(stderr,
               "usage: %s [--width N] [--height N] [--spp N] [--depth N] [--seed N]\n"
               "          [--spheres HALF_EXTENT] [--scene final|five] [--camera cpu|gpu]\n"
               "          [--semantics cpu|gpu] [--accel bvh|scan] [--gpus N] [--device N]\n"
               "          [--devices D0,D1,...] [--gather rccl|host] [--out FILE] [--p6] [--quiet]\n"
               "          [--launch-samples N]\n",
               argv0);
  std::exit(2);
}

struct gpu_job {
  int device;
  rt_params params;
  rt_stats stats{};
};

}  // namespace

int main(int argc, char **argv) {
  options o;
  std::string name = argv[0];
  if (auto s = name.rfind('/'); s != std::string::npos) name = name.substr(s + 1);
  const bool gpu_mode = name == "gpu_ray_tracer";
  if (gpu_mode) {
    o.width = 1920;
    o.height = 1080;  // static_cast<int>(1920 / (16/9)), src/gpu/camera.h:60-62
    o.camera = RT_CAMERA_GPU;
    o.flags = RT_FLAG_GPU_SEMANTICS;
  }
  bool height_set = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char * {
      if (i + 1 >= argc) usage(argv[0]);
      return argv[++i];
    };
    if (a == "--width") o.width = std::atoi(next());
    else if (a == "--height") { o.height = std::atoi(next()); height_set = true; }
    else if (a == "--spp") o.spp = std::atoi(next());
    else if (a == "--depth") o.depth = std::atoi(next());
    else if (a == "--seed") { o.seed = std::strtoull(next(), nullptr, 10); o.seed_set = true; }
    else if (a == "--spheres") o.half_extent = std::atoi(next());
    else if (a == "--scene") o.scene = next();
    else if (a == "--camera") o.camera = std::string(next()) == "gpu" ? RT_CAMERA_GPU : RT_CAMERA_CPU;
    else if (a == "--semantics") o.flags = std::string(next()) == "gpu" ? RT_FLAG_GPU_SEMANTICS : 0u;
    else if (a == "--accel") o.bvh = std::string(next()) != "scan";
    else if (a == "--gpus") o.gpus = std::atoi(next());
    else if (a == "--device") o.device = std::atoi(next());
    else if (a == "--devices") {
      // one device per band, comma separated; a device may repeat (several
      // bands rendered by one GPU, each with its own context and stream)
      o.devices.clear();
      for (std::string list = next(); !list.empty();) {
        const size_t c = list.find(',');
        o.devices.push_back(std::atoi(list.substr(0, c).c_str()));
        list = c == std::string::npos ? std::string() : list.substr(c + 1);
      }
    }
    else if (a == "--gather") o.gather = next();
    else if (a == "--out") o.out = next();
    else if (a == "--p6") o.p6 = true;
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--launch-samples") o.launch_samples = std::atof(next());
    else usage(argv[0]);
  }
  if (!height_set && (o.width != (gpu_mode ? 1920 : 1200))) {
    // keep the reference aspect ratio when only the width is given
    o.height = gpu_mode ? (int)(o.width / (16.0f / 9.0f)) : (int)(o.width / (3.0 / 2.0));
  }
  if (gpu_mode && !o.seed_set) o.seed = (unsigned long long)std::time(nullptr);  // main.cu:88
  if (o.width < 2 || o.height < 2 || o.spp < 0 || o.depth < 0 || o.gpus < 1) usage(argv[0]);
  if (o.gather != "auto" && o.gather != "rccl" && o.gather != "host") usage(argv[0]);
  bool repeated = false;
  if (!o.devices.empty()) {
    if ((int)o.devices.size() != o.gpus) usage(argv[0]);
    for (int g = 0; g < o.gpus; ++g)
      for (int k = 0; k < g; ++k) repeated |= o.devices[k] == o.devices[g];
    if (repeated && o.gather == "rccl") {
      std::fprintf(stderr, "rtow: --gather rccl needs distinct devices\n");
      std::exit(2);
    }
    if (repeated) o.gather = "host";
  }

  // ---- scene (random_scene / new_world) ----
  const uint32_t cap = (uint32_t)(4 * o.half_extent * o.half_extent + 16);
  std::vector<float> cx(cap), cy(cap), cz(cap), rad(cap), alb(3 * cap), par(cap);
  std::vector<uint32_t> kind(cap);
  rt_scene_buf buf{cap, 0, cx.data(), cy.data(), cz.data(), rad.data(), kind.data(), alb.data(), par.data()};
  if (o.scene == "five") check(rt_scene_five(&buf), "rt_scene_five");
  else check(rt_scene_final(o.half_extent, &buf, nullptr), "rt_scene_final");
  rt_scene_view view{buf.n, cx.data(), cy.data(), cz.data(), rad.data(), kind.data(), alb.data(), par.data()};

  // ---- camera ----
  rt_camera cam;
  const bool five = o.scene == "five";
  const double from_f[3] = {13, 2, 3}, at_f[3] = {0, 0, 0};
  const double from_5[3] = {-2, 2, 1}, at_5[3] = {0, 0, -1};
  const double vup[3] = {0, 1, 0};
  const double *from = five ? from_5 : from_f, *at = five ? at_5 : at_f;
  if (o.camera == RT_CAMERA_GPU)
    check(rt_camera_gpu(from, at, vup, 20.0, o.width, o.height, five ? 10.0 : 0.6, five ? 3.4 : 10.0, &cam),
          "rt_camera_gpu");
  else
    check(rt_camera_cpu(from, at, vup, 20.0, (double)o.width / o.height, five ? 0.0 : 0.1,
                        five ? 3.4 : 10.0, &cam),
          "rt_camera_cpu");

  int ndev = 0;
  check(rt_device_count(&ndev), "rt_device_count");
  if (ndev < 1) die("no HIP device", RT_ERR_NO_DEVICE);
  if (o.devices.empty() && o.gpus > ndev) {
    // no silent clamp: a run asked for N GPUs must not report a 1-GPU time as N
    std::fprintf(stderr, "rtow: --gpus %d but only %d HIP device(s) visible\n", o.gpus, ndev);
    std::exit(2);
  }
  for (int d : o.devices)
    if (d < 0 || d >= ndev) {
      std::fprintf(stderr, "rtow: --devices names device %d but only %d HIP device(s) visible\n", d, ndev);
      std::exit(2);
    }

  // the reference's stderr surface, per personality (src/cpu/main.cc:103-105,
  // src/gpu/main.cu:121-125); our extra lines follow the timing
  if (!o.quiet) {
    std::fprintf(stderr, "Image Size = %d x %d\n", o.width, o.height);
    std::fprintf(stderr, "Samples Per Pixel = %d\n", o.spp);
    if (gpu_mode) {
      std::fprintf(stderr, "Block Dim (a x b threads) = %d x %d\n", 8, 8);  // one wave64 per 8x8 tile
      std::fprintf(stderr, "Random Seed = %llu\n", o.seed);
    } else {
      std::fprintf(stderr, "Number of CPU threads = %d\n", 1);  // one host thread drives the GPUs
      if (o.seed_set) std::fprintf(stderr, "Random Seed = %llu\n", o.seed);
    }
  }

  // ---- render: one context and stream per GPU, interleaved row bands ----
  const int row_block = 8;
  std::vector<gpu_job> jobs(o.gpus);
  for (int g = 0; g < o.gpus; ++g) {
    rt_params p{};
    p.width = o.width;
    p.height = o.height;
    p.spp = o.spp;
    p.max_depth = o.depth;
    p.seed = o.seed;
    // (no RT_FLAG_PILOT_SCHEDULE: the pilot pays off over repeated frames of
    // one geometry, not in a one-frame process -- its first launch also loads
    // the instrumented kernel)
    p.flags = o.flags | (o.bvh ? RT_FLAG_ACCEL_BVH : 0u);
    if (o.gpus == 1) {
      p.row_block = o.height;
      p.band_stride = 1;
      p.band_offset = 0;
      p.local_rows = o.height;
    } else {
      const int band_rows = row_block * o.gpus;
      p.row_block = row_block;
      p.band_stride = o.gpus;
      p.band_offset = g;
      p.local_rows = (o.height + band_rows - 1) / band_rows * row_block;
    }
    jobs[g].device = !o.devices.empty() ? o.devices[g] : o.gpus == 1 ? o.device : g;
    jobs[g].params = p;
  }
  std::vector<rt_context *> ctxs(o.gpus, nullptr);
  for (int g = 0; g < o.gpus; ++g) {
    check(rt_context_create(jobs[g].device, &ctxs[g]), "rt_context_create");
    if (o.launch_samples > 0.0)
      check(rt_context_set_option(ctxs[g], RT_OPT_LAUNCH_SAMPLES, o.launch_samples), "rt_context_set_option");
    check(rt_scene_upload(ctxs[g], &view), "rt_scene_upload");
  }
  const bool use_rccl = o.gather == "rccl" || (o.gather == "auto" && o.gpus > 1);
  // Every device renders its tile (fp32 sums) and tonemaps it on the device
  // (write_color, src/cpu/color.h or src/gpu/color.h by personality) into 3 B
  // per pixel; the byte tiles are gathered to device 0 with one RCCL
  // ncclGather over xGMI (or copied back one by one with --gather host) and
  // written by the streaming PPM writer: the host never holds fp32 sums.
  const int tone_mode = (o.flags & RT_FLAG_GPU_SEMANTICS) == RT_FLAG_GPU_SEMANTICS ? RT_TONEMAP_GPU
                                                                                 : RT_TONEMAP_CPU;
  const size_t tile_px = (size_t)o.width * jobs[0].params.local_rows;
  std::vector<int> devs(o.gpus);
  for (int g = 0; g < o.gpus; ++g) devs[g] = jobs[g].device;
  std::vector<hipStream_t> streams(o.gpus);
  std::vector<float *> d_tile(o.gpus, nullptr);
  std::vector<uint8_t *> d_u8(o.gpus, nullptr);
  uint8_t *d_all = nullptr;
  std::vector<ncclComm_t> comms;
  if (use_rccl) {
    comms.resize(o.gpus);
    // RCCL prints a version banner on stdout, which carries the PPM: send it
    // to stderr while the communicators are created
    std::fflush(stdout);
    const int saved_stdout = ::dup(1);
    ::dup2(2, 1);
    const ncclResult_t init = ncclCommInitAll(comms.data(), o.gpus, devs.data());
    std::fflush(stdout);
    ::dup2(saved_stdout, 1);
    ::close(saved_stdout);
    if (init != ncclSuccess) die("ncclCommInitAll", RT_ERR_HIP);
  }
  for (int g = 0; g < o.gpus; ++g) {
    if (hipSetDevice(devs[g]) != hipSuccess ||
        hipStreamCreateWithFlags(&streams[g], hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&d_tile[g], 3 * tile_px * sizeof(float)) != hipSuccess ||
        hipMalloc(&d_u8[g], 3 * tile_px) != hipSuccess)
      die("device buffers", RT_ERR_HIP);
    if (use_rccl && g == 0 && hipMalloc(&d_all, 3 * tile_px * o.gpus) != hipSuccess)
      die("gather buffer", RT_ERR_HIP);
  }
  // per device: events before the render, after it, after write_color and
  // after the gather, for the per-device lines on stderr
  std::vector<hipEvent_t> ev(4 * (size_t)o.gpus, nullptr);
  for (int g = 0; g < o.gpus; ++g) {
    (void)hipSetDevice(devs[g]);
    for (int k = 0; k < 4; ++k)
      if (hipEventCreate(&ev[4 * g + k]) != hipSuccess) die("hipEventCreate", RT_ERR_HIP);
    (void)hipDeviceSynchronize();
  }
  const auto start = std::chrono::high_resolution_clock::now();
  for (int g = 0; g < o.gpus; ++g) {
    (void)hipSetDevice(devs[g]);
    (void)hipEventRecord(ev[4 * g + 0], streams[g]);
    check(rt_render_async(ctxs[g], &cam, &jobs[g].params, d_tile[g], streams[g]), "rt_render_async");
    (void)hipEventRecord(ev[4 * g + 1], streams[g]);
    check(rt_tonemap_async(ctxs[g], d_tile[g], tile_px, o.spp > 0 ? o.spp : 1, tone_mode, d_u8[g], streams[g]),
          "rt_tonemap_async");
    (void)hipEventRecord(ev[4 * g + 2], streams[g]);
  }
  if (use_rccl) {
    if (ncclGroupStart() != ncclSuccess) die("ncclGroupStart", RT_ERR_HIP);
    for (int g = 0; g < o.gpus; ++g)
      if (ncclGather(d_u8[g], g == 0 ? d_all : nullptr, 3 * tile_px, ncclUint8, 0, comms[g], streams[g]) !=
          ncclSuccess)
        die("ncclGather", RT_ERR_HIP);
    if (ncclGroupEnd() != ncclSuccess) die("ncclGroupEnd", RT_ERR_HIP);
  }
  for (int g = 0; g < o.gpus; ++g) {
    (void)hipSetDevice(devs[g]);
    (void)hipEventRecord(ev[4 * g + 3], streams[g]);
  }
  // progress while the bounded launches run (the reference's "Scanlines
  // remaining", src/cpu/main.cc:112): a render of many launches reports each
  // one as it completes, and a device fault ends the run after the launch it
  // happened in, not at the end of the frame.  One launch per device: no
  // polling, the streams are synchronised at once; otherwise the poll sleeps
  // 1 ms, so the reference-style "Time Cost" below overshoots by < 1 ms
  // (it slept 20 ms before: ADVICE r3)
  bool single = true;
  for (int g = 0; g < o.gpus; ++g) {
    uint32_t d = 0, t = 0;
    check(rt_render_progress(ctxs[g], &d, &t), "rt_render_progress");
    single = single && t <= 1;
  }
  for (unsigned last = ~0u; !single;) {
    unsigned done = 0, total = 0;
    for (int g = 0; g < o.gpus; ++g) {
      uint32_t d = 0, t = 0;
      check(rt_render_progress(ctxs[g], &d, &t), "rt_render_progress");
      done += d;
      total += t;
    }
    if (!o.quiet && total > (unsigned)o.gpus && total - done != last) {
      std::fprintf(stderr, "\rLaunches remaining: %u ", total - done);
      std::fflush(stderr);
      last = total - done;
    }
    if (done == total) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  for (int g = 0; g < o.gpus; ++g) {
    (void)hipSetDevice(devs[g]);
    if (hipStreamSynchronize(streams[g]) != hipSuccess) die("render", RT_ERR_HIP);
  }
  const auto end = std::chrono::high_resolution_clock::now();
  // byte tiles, rank-major, to the host
  std::vector<uint8_t> tiles(3 * tile_px * o.gpus);
  if (use_rccl) {
    (void)hipSetDevice(devs[0]);
    if (hipMemcpy(tiles.data(), d_all, tiles.size(), hipMemcpyDeviceToHost) != hipSuccess)
      die("gather copy", RT_ERR_HIP);
  } else {
    for (int g = 0; g < o.gpus; ++g) {
      (void)hipSetDevice(devs[g]);
      if (hipMemcpy(&tiles[3 * tile_px * g], d_u8[g], 3 * tile_px, hipMemcpyDeviceToHost) != hipSuccess)
        die("tile copy", RT_ERR_HIP);
    }
  }
  for (int g = 0; g < o.gpus; ++g) check(rt_collect_stats(ctxs[g], &jobs[g].stats), "rt_collect_stats");

  // main.cu:134-139 / main.cc:125-130 timing lines
  float ms = std::chrono::duration<float, std::milli>(end - start).count();
  int time_cost_in_ms = (int)(ms + 0.999f);
  int time_cost_in_sec = (time_cost_in_ms + 999) / 1000;
  unsigned long long segs = 0, samples = 0;
  for (auto &j : jobs) {
    segs += j.stats.segments;
    samples += j.stats.samples;
  }
  if (!o.quiet) {
    if (!gpu_mode) std::fprintf(stderr, "\rScanlines remaining: %d ", 0);  // main.cc:112, all rendered at once
    std::fprintf(stderr, "%sTime Cost (ms) = %d ms\n", gpu_mode ? "" : "\n", time_cost_in_ms);
    std::fprintf(stderr, "Time Cost (sec) = %d sec\n", time_cost_in_sec);
    std::fprintf(stderr, "Number of GPUs = %d, spheres = %u\n", o.gpus, buf.n);
    std::fprintf(stderr, "Throughput = %.1f Mray/s, %.1f Msample/s (%llu segments)\n",
                 segs / (ms * 1e3), samples / (ms * 1e3), segs);
    // per device: render (its launches), write_color, and the wait for the
    // gather (the RCCL gather of the byte tiles ends on every device's stream)
    for (int g = 0; g < o.gpus; ++g) {
      float r = 0.f, t = 0.f, x = 0.f;
      (void)hipSetDevice(devs[g]);
      (void)hipEventElapsedTime(&r, ev[4 * g + 0], ev[4 * g + 1]);
      (void)hipEventElapsedTime(&t, ev[4 * g + 1], ev[4 * g + 2]);
      (void)hipEventElapsedTime(&x, ev[4 * g + 2], ev[4 * g + 3]);
      std::fprintf(stderr, "GPU %d (device %d): render %.3f ms in %llu launch(es), write_color %.3f ms, %s %.3f ms\n",
                   g, devs[g], r, (unsigned long long)jobs[g].stats.launches, t,
                   use_rccl ? "gather (RCCL)" : "gather (none)", x);
    }
  }

  // ---- assemble rows + PPM (output_image, src/gpu/camera.h:197-210) ----
  std::vector<uint8_t> rgb(3 * (size_t)o.width * o.height, 0);
  for (int g = 0; g < o.gpus; ++g) {
    const rt_params &p = jobs[g].params;
    const uint8_t *src = &tiles[3 * tile_px * g];
    for (int r = 0; r < p.local_rows; ++r) {
      const int band = r / p.row_block;
      const int grow = (band * p.band_stride + p.band_offset) * p.row_block + r % p.row_block;
      if (grow >= o.height) continue;
      std::memcpy(&rgb[3 * (size_t)grow * o.width], &src[3 * (size_t)r * o.width], 3 * (size_t)o.width);
    }
  }
  std::vector<uint8_t>().swap(tiles);
  int fd = 1;
  if (!o.out.empty()) {
    fd = ::open(o.out.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) die(o.out.c_str(), RT_ERR_IO);
  }
  check(rt_write_ppm(fd, rgb.data(), o.width, o.height, o.p6 ? 1 : 0), "rt_write_ppm");
  if (fd != 1) ::close(fd);
  for (int g = 0; g < o.gpus; ++g) {
    (void)hipSetDevice(devs[g]);
    for (int k = 0; k < 4; ++k) (void)hipEventDestroy(ev[4 * g + k]);
    (void)hipFree(d_tile[g]);
    (void)hipFree(d_u8[g]);
    (void)hipStreamDestroy(streams[g]);
    if (use_rccl) ncclCommDestroy(comms[g]);
  }
  if (d_all) {
    (void)hipSetDevice(devs[0]);
    (void)hipFree(d_all);
  }
  for (auto *c : ctxs) rt_context_destroy(c);
  if (!o.quiet && !gpu_mode) std::fprintf(stderr, "\nDone.\n");  // main.cc:132
  return 0;
}
