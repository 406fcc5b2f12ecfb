// tools/seed_search_image23.c -- recover the time seed of the reference's
// gallery/gpu/image23.png (src/gpu/main.cu:88 seeds new_world's curand XORWOW
// with time(nullptr)).  For every candidate second and both argument orders it
// builds the scene's draw sequence (main.cu:18-75), projects the diffuse
// spheres nearest the camera (radius > 40 px) through src/gpu's camera, and
// scores how many of their centre pixels have the predicted chroma
// (sqrt(albedo), sky-tinted).  The true seed scores ~all of them; others stay
// at noise (tests/gallery_lib.py records the result).  Build container only:
//   python -c "from PIL import Image; import numpy as np; np.asarray(Image.open(
//     '/root/reference/gallery/gpu/image23.png').convert('RGB')).tofile('/tmp/g23.rgb')"
//   gcc -O3 -fopenmp -o /tmp/seed23 tools/seed_search_image23.c -lm
//   /tmp/seed23 1640995200 1760572800 /tmp/g23.rgb      (~15 min on 8 cores)
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
typedef struct { uint32_t v[5], d; } xw;
static void xw_init(xw *s, uint64_t seed) {
  uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u, s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
  uint32_t t0 = 1099087573u * s0, t1 = 2591861531u * s1;
  s->d = 6615241u + t1 + t0;
  s->v[0] = 123456789u + t0; s->v[1] = 362436069u ^ t0; s->v[2] = 521288629u + t1;
  s->v[3] = 88675123u ^ t1; s->v[4] = 5783321u + t0;
}
static inline uint32_t xw_next(xw *s) {
  uint32_t t = s->v[0] ^ (s->v[0] >> 2);
  s->v[0] = s->v[1]; s->v[1] = s->v[2]; s->v[2] = s->v[3]; s->v[3] = s->v[4];
  s->v[4] = (s->v[4] ^ (s->v[4] << 4)) ^ (t ^ (t << 1));
  s->d += 362437u;
  return s->v[4] + s->d;
}
static inline float rf(xw *s) { float u = (float)xw_next(s) * 2.3283064e-10f + 1.1641532e-10f; return 1.0f - u; }
static unsigned char *img;
static double E[3], U[3], V[3], W[3];
static double vw, vh;
// pixel of a world point (src/gpu camera: 1920x1080, vfov 20, focus 10)
static int project(double x, double y, double z, double *pi, double *pj, double *scale) {
  double d[3] = {x - E[0], y - E[1], z - E[2]};
  double dw = d[0] * W[0] + d[1] * W[1] + d[2] * W[2];
  if (dw >= -1e-3) return 0;
  double s = 10.0 / (-dw);
  double px = (d[0] * U[0] + d[1] * U[1] + d[2] * U[2]) * s, py = (d[0] * V[0] + d[1] * V[1] + d[2] * V[2]) * s;
  *pi = (px + vw / 2) / vw * 1920.0 - 0.5;
  *pj = (vh / 2 - py) / vh * 1080.0 - 0.5;
  *scale = s * 1920.0 / vw;  // pixels per world unit at the sphere
  return *pi >= 8 && *pi < 1912 && *pj >= 8 && *pj < 1072;
}
typedef struct { float cx, cz, a[3]; int mat; } sph;
static int gen(uint64_t seed, int rev, sph *out) {
  xw s; xw_init(&s, seed); int n = 0;
  for (int a = -11; a < 11; a++)
    for (int b = -11; b < 11; b++) {
      float choose = rf(&s), r1, r2;
      if (!rev) { r1 = rf(&s); r2 = rf(&s); } else { r2 = rf(&s); r1 = rf(&s); }
      float cx = a + 0.9f * r1, cz = b + 0.9f * r2;
      float dx = cx - 4.0f, dz = cz;
      if (sqrtf(dx * dx + dz * dz) <= 0.9f) continue;
      sph q; q.cx = cx; q.cz = cz;
      if (choose < 0.8f) {
        float v1[3], v2[3];
        for (int k = 0; k < 3; ++k) v1[rev ? 2 - k : k] = rf(&s);
        for (int k = 0; k < 3; ++k) v2[rev ? 2 - k : k] = rf(&s);
        for (int k = 0; k < 3; ++k) q.a[k] = v1[k] * v2[k];
        q.mat = 0;
      } else if (choose < 0.95f) {
        for (int k = 0; k < 3; ++k) q.a[rev ? 2 - k : k] = 0.5f + 0.5f * rf(&s);
        (void)rf(&s); q.mat = 1;
      } else { q.a[0] = q.a[1] = q.a[2] = 1; q.mat = 2; }
      out[n++] = q;
    }
  return n;
}
static double score(const sph *sp, int n, int *nd) {
  double sc = 0; int cnt = 0;
  for (int k = 0; k < n; ++k) {
    if (sp[k].mat != 0 || sp[k].cx < 4.0f) continue;
    double pi, pj, pxu;
    if (!project(sp[k].cx, 0.2, sp[k].cz, &pi, &pj, &pxu)) continue;
    if (0.2 * pxu < 40) continue;  // near spheres only (radius > 40 px)
    int i0 = (int)pi, j0 = (int)pj; double o[3] = {0, 0, 0};
    for (int dj = -3; dj <= 3; ++dj) for (int di = -3; di <= 3; ++di)
      for (int c = 0; c < 3; ++c) o[c] += img[((j0 + dj) * 1920 + (i0 + di)) * 3 + c];
    double os = o[0] + o[1] + o[2] + 1e-9, p[3], ps = 0;
    for (int c = 0; c < 3; ++c) { p[c] = sqrt(sp[k].a[c] * (c == 2 ? 1.0 : (c == 1 ? 0.85 : 0.75))); ps += p[c]; }
    double dist = 0;
    for (int c = 0; c < 3; ++c) dist += fabs(o[c] / os - p[c] / (ps + 1e-9));
    sc += dist < 0.12 ? 1.0 : -0.3; ++cnt;
  }
  *nd = cnt;
  return sc;
}
int main(int argc, char **argv) {
  uint64_t lo = strtoull(argv[1], 0, 10), hi = strtoull(argv[2], 0, 10);
  FILE *f = fopen(argc > 3 ? argv[3] : "/tmp/g23.rgb", "rb");
  img = malloc(1920 * 1080 * 3);
  if (!f || fread(img, 1, 1920 * 1080 * 3, f) != 1920 * 1080 * 3) return 1;
  fclose(f);
  double la[3] = {0, 0, 0}, vup[3] = {0, 1, 0};
  E[0] = 13; E[1] = 2; E[2] = 3;
  double w[3] = {E[0] - la[0], E[1] - la[1], E[2] - la[2]}, wl = sqrt(w[0]*w[0]+w[1]*w[1]+w[2]*w[2]);
  for (int c = 0; c < 3; ++c) W[c] = w[c] / wl;
  double u[3] = {vup[1]*W[2]-vup[2]*W[1], vup[2]*W[0]-vup[0]*W[2], vup[0]*W[1]-vup[1]*W[0]};
  double ul = sqrt(u[0]*u[0]+u[1]*u[1]+u[2]*u[2]);
  for (int c = 0; c < 3; ++c) U[c] = u[c] / ul;
  V[0] = W[1]*U[2]-W[2]*U[1]; V[1] = W[2]*U[0]-W[0]*U[2]; V[2] = W[0]*U[1]-W[1]*U[0];
  vh = 2 * tan(10.0 * M_PI / 180) * 10; vw = vh * 1920.0 / 1080.0;
  double best = -1e9;
#pragma omp parallel
  {
    sph sp[500];
#pragma omp for schedule(dynamic, 65536)
    for (uint64_t seed = lo; seed < hi; ++seed)
      for (int rev = 0; rev < 2; ++rev) {
        int n = gen(seed, rev, sp), nd;
        double sc = score(sp, n, &nd);
        if (sc >= 5 && sc >= best - 1) {
#pragma omp critical
          { if (sc > best) best = sc; printf("seed %llu rev %d score %.1f of %d\n", (unsigned long long)seed, rev, sc, nd); fflush(stdout); }
        }
      }
  }
  return 0;
}
