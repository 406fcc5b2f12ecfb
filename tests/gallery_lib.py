"""Test infrastructure: src/gpu's final scene as the reference's own CUDA run
that made gallery/gpu/image23.png built it, restated on the host so that the
image can be re-rendered here.  Used only by tests (never by the product).

src/gpu/main.cu:18-75 builds the scene on the device from curand XORWOW with
curand_init(seed, 0, 0), seed = time(nullptr) (main.cu:88), drawing
random_float = 1 - curand_uniform (src/gpu/rtweekend.h:20-29).  XORWOW is
restated from cuRAND's published algorithm (Marsaglia's xorwow plus a Weyl
sequence, curand_init's seed scrambling, curand_uniform = x 2^-32 + 2^-33).
The gallery run's seed, IMAGE23_SEED = 1694284176 (2023-09-09 18:29:36 UTC),
was found by a search over 2022-2025 that projects each candidate scene's
nearest diffuse spheres into the image and compares their colours
(tools/seed_search_image23.c): it scores 13.7 of 15 spheres against at most
7.8 for any other second in those four years.  Function arguments are drawn
left to right (the other order scores at noise level).
"""
import numpy as np

IMAGE23_SEED = 1694284176
M32 = 0xFFFFFFFF


class Xorwow:
    """curandStateXORWOW after curand_init(seed, 0, 0)."""

    def __init__(self, seed):
        s0 = (seed & M32) ^ 0xAAD26B49
        s1 = ((seed >> 32) & M32) ^ 0xF7DCEFDD
        t0 = (1099087573 * s0) & M32
        t1 = (2591861531 * s1) & M32
        self.d = (6615241 + t1 + t0) & M32
        self.v = [(123456789 + t0) & M32, 362436069 ^ t0, (521288629 + t1) & M32, 88675123 ^ t1,
                  (5783321 + t0) & M32]

    def next_u32(self):
        v = self.v
        t = v[0] ^ (v[0] >> 2)
        v[0], v[1], v[2], v[3] = v[1], v[2], v[3], v[4]
        v[4] = (v[4] ^ ((v[4] << 4) & M32)) ^ (t ^ ((t << 1) & M32))
        self.d = (self.d + 362437) & M32
        return (v[4] + self.d) & M32

    def random_float(self, lo=None, hi=None):
        """1 - curand_uniform, optionally scaled to [lo, hi) (rtweekend.h:20-29)."""
        f = np.float32
        r = f(1) - f(f(self.next_u32()) * f(2.3283064e-10) + f(1.1641532e-10))
        return r if lo is None else f(f(lo) + f(f(hi) - f(lo)) * r)


def src_gpu_final_scene(rtow, seed=IMAGE23_SEED):
    """src/gpu/main.cu:18-75 new_world(seed) as an rtow.Scene (fp32, draws in
    argument order left to right)."""
    rng = Xorwow(seed)
    f = np.float32
    rows = [((0.0, -1000.0, 0.0), 1000.0, rtow.RT_LAMBERTIAN, (0.5, 0.5, 0.5), 0.0)]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rng.random_float()
            cx = f(a) + f(0.9) * rng.random_float()
            cz = f(b) + f(0.9) * rng.random_float()
            dx, dz = f(cx - f(4.0)), f(cz)
            if f(np.sqrt(f(dx * dx + dz * dz))) <= f(0.9):
                continue
            if choose < f(0.8):
                v1 = [rng.random_float() for _ in range(3)]
                v2 = [rng.random_float() for _ in range(3)]
                rows.append(((cx, 0.2, cz), 0.2, rtow.RT_LAMBERTIAN, tuple(float(x * y) for x, y in zip(v1, v2)), 0.0))
            elif choose < f(0.95):
                alb = [rng.random_float(0.5, 1.0) for _ in range(3)]
                fuzz = rng.random_float(0.0, 0.5)
                rows.append(((cx, 0.2, cz), 0.2, rtow.RT_METAL, tuple(map(float, alb)), float(fuzz)))
            else:
                rows.append(((cx, 0.2, cz), 0.2, rtow.RT_DIELECTRIC, (1.0, 1.0, 1.0), 1.5))
    rows.append(((0.0, 1.0, 0.0), 1.0, rtow.RT_DIELECTRIC, (1.0, 1.0, 1.0), 1.5))
    rows.append(((-4.0, 1.0, 0.0), 1.0, rtow.RT_LAMBERTIAN, (0.4, 0.2, 0.1), 0.0))
    rows.append(((4.0, 1.0, 0.0), 1.0, rtow.RT_METAL, (0.7, 0.6, 0.5), 0.0))
    c = np.array([r[0] for r in rows], np.float32)
    return rtow.Scene(c[:, 0].copy(), c[:, 1].copy(), c[:, 2].copy(), np.array([r[1] for r in rows], np.float32),
                      np.array([r[2] for r in rows], np.uint32), np.array([r[3] for r in rows], np.float32),
                      np.array([r[4] for r in rows], np.float32))
