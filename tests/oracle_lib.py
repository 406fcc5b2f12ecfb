"""ctypes binding of oracle/librt_oracle.so -- the CHECKER (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
import ctypes
import gzip
import json
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "librt_oracle.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            raise RuntimeError(f"{ORACLE_SO} missing: run `make -C oracle`")
        # built with -mfma (oracle/Makefile): the host CPU needs FMA3
        with open("/proc/cpuinfo") as f:
            if " fma " not in f.read().replace("\n", " "):
                raise RuntimeError("the oracle is built with -mfma but this CPU has no FMA3")
        L = ctypes.CDLL(ORACLE_SO)
        L.rto_reference_render.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_ulonglong)]
        L.rto_kernel_render.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong),
                                        ctypes.c_int]
        L.rto_reference_scene.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def reference_render(width, aspect, spp, max_depth=50, scene=0):
    """fp64 restatement of src/cpu -> (uint8 [H, W, 3] top row first, segments)."""
    L = lib()
    h = ctypes.c_int()
    assert L.rto_reference_render(width, aspect, spp, max_depth, scene, None, ctypes.byref(h), None) == 0
    out = np.zeros((h.value, width, 3), np.uint8)
    seg = ctypes.c_ulonglong()
    assert L.rto_reference_render(width, aspect, spp, max_depth, scene, out.ctypes.data,
                                  ctypes.byref(h), ctypes.byref(seg)) == 0
    return out, seg.value


def reference_render_view(scene, width, aspect, spp, max_depth=50):
    """fp64 restatement of src/cpu on any scene, with the final scene's camera
    (what oracle/_ref/ref_harness renders for a `file:` scene)
    -> (uint8 [H, W, 3] top row first, segments)."""
    L = lib()
    L.rto_reference_render_view.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                            ctypes.POINTER(ctypes.c_ulonglong)]
    v = scene.view()
    h = ctypes.c_int()
    assert L.rto_reference_render_view(ctypes.addressof(v), width, aspect, spp, max_depth, None,
                                       ctypes.byref(h), None) == 0
    out = np.zeros((h.value, width, 3), np.uint8)
    seg = ctypes.c_ulonglong()
    assert L.rto_reference_render_view(ctypes.addressof(v), width, aspect, spp, max_depth, out.ctypes.data,
                                       ctypes.byref(h), ctypes.byref(seg)) == 0
    return out, seg.value


# rto_kernel_render_exact's opts bits (oracle/rt_oracle.h): superseded forms
# of the specification, for the tests that show why they changed
RTO_OPT_NO_DITHER = 1
RTO_OPT_TMIN_WORLD = 2
RTO_OPT_NO_SEALED = 4
RTO_OPT_FP64_ROOTS = 8
RTO_OPT_NO_SAME_EXIT = 16
RTO_OPT_FP64_HIT = 32


def kernel_render(scene, cam, params, threads=0, tmin_world=False, no_sealed=False):
    """fp32 restatement of the kernel algorithm -> (float32 [rows, W, 3], segments).
    tmin_world: t_min 0.001 in world units on the normalised ray (the
    round-1..4 specification) instead of the reference's unit, 0.001 |d|.
    no_sealed: without the opaque-inside rule (attribution only)."""
    if tmin_world or no_sealed:
        opts = (RTO_OPT_TMIN_WORLD if tmin_world else 0) | (RTO_OPT_NO_SEALED if no_sealed else 0)
        out, _, segs = _kernel_render_opts(scene, cam, params, opts, False, threads)
        return out, segs
    v = scene.view()
    out = np.zeros((params.local_rows, params.width, 3), np.float32)
    seg = ctypes.c_ulonglong()
    assert lib().rto_kernel_render(ctypes.addressof(v), ctypes.addressof(cam), ctypes.addressof(params),
                                   out.ctypes.data, ctypes.byref(seg), threads) == 0
    return out, seg.value


def _kernel_render_opts(scene, cam, params, opts, want_exact, threads):
    v = scene.view()
    out = np.zeros((params.local_rows, params.width, 3), np.float32)
    exact = np.zeros((params.local_rows, params.width, 3), np.float64) if want_exact else None
    seg = ctypes.c_ulonglong()
    L = lib()
    L.rto_kernel_render_exact.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int, ctypes.POINTER(ctypes.c_ulonglong),
                                                                   ctypes.c_int]
    assert L.rto_kernel_render_exact(ctypes.addressof(v), ctypes.addressof(cam), ctypes.addressof(params),
                                     out.ctypes.data, exact.ctypes.data if want_exact else None, int(opts),
                                     ctypes.byref(seg), threads) == 0
    return out, exact, seg.value


def kernel_render_exact(scene, cam, params, no_dither=False, threads=0):
    """kernel_render plus each pixel's fp64 sum of the unquantised sample
    radiances (the reference's fp64 accumulation, src/cpu/main.cc:114-119, of
    the same samples) -> (float32 sums, float64 exact sums, segments).
    no_dither: the sum format without stochastic rounding (truncation)."""
    return _kernel_render_opts(scene, cam, params, RTO_OPT_NO_DITHER if no_dither else 0, True, threads)


def trace(scene, cam, params, col, row, sample, max_depth=50):
    """Print one sample's segments and candidate spheres (debug tooling)."""
    import copy
    v = scene.view()
    p = copy.copy(params)
    p.max_depth = max_depth
    lib().rto_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_long]
    lib().rto_trace(ctypes.addressof(v), ctypes.addressof(cam), ctypes.addressof(p), col, row, sample)


def reference_scene(half_extent=11):
    L = lib()
    n = ctypes.c_size_t()
    nxt = ctypes.c_double()
    L.rto_reference_scene(half_extent, None, 0, ctypes.byref(n), None)
    rows = np.zeros((n.value, 9), np.float64)
    assert L.rto_reference_scene(half_extent, rows.ctypes.data, n.value, ctypes.byref(n),
                                 ctypes.byref(nxt)) == 0
    return rows, nxt.value


# ---------------------------------------------------------------- fixtures --

def read_ppm_bytes(data):
    """Parse P3/P6 bytes -> uint8 [H, W, 3]."""
    if data[:2] == b"P6":
        parts = data.split(b"\n", 3)
        w, h = map(int, parts[1].split())
        return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)
    toks = data.split()
    assert toks[0] == b"P3"
    w, h = int(toks[1]), int(toks[2])
    vals = np.array(toks[4:], dtype=np.int64)
    return vals.astype(np.uint8).reshape(h, w, 3)


def golden_ppm(name):
    with gzip.open(os.path.join(GOLDEN, name + ".ppm.gz"), "rb") as f:
        return f.read()


def golden_stats():
    with open(os.path.join(GOLDEN, "ref_stats.json")) as f:
        return json.load(f)


def golden_scene_rows():
    rows = []
    for line in open(os.path.join(GOLDEN, "scene_final_gcc.txt")):
        t = line.split()
        if t[0] == "next":
            nxt = float(t[1])
            continue
        rows.append([{"L": 0, "M": 1, "D": 2}[t[0]]] + [float(x) for x in t[1:]])
    return np.array(rows, np.float64), nxt


def golden_kat():
    with open(os.path.join(GOLDEN, "kat.jsonl")) as f:
        return [json.loads(l) for l in f if l.strip()]


def ppm_p3_bytes(rgb):
    """Format like write_color (src/cpu/color.h:20-22) + header main.cc:109."""
    h, w = rgb.shape[:2]
    flat = rgb.reshape(-1, 3)
    body = "".join("%d %d %d\n" % (r, g, b) for r, g, b in flat)
    return ("P3\n%d %d\n255\n" % (w, h) + body).encode()


def color_kat():
    """tests/golden/kat_colors.txt (make_color_kat.py): [(float32 sums[3], spp,
    reference levels[3])], fp32 sums within a few ulps of write_color's level
    thresholds."""
    out = []
    with open(os.path.join(GOLDEN, "kat_colors.txt")) as f:
        for line in f:
            left, right = line.split("|")
            v = left.split()
            out.append((np.array([float(x) for x in v[:3]], np.float32), int(v[3]),
                        [int(x) for x in right.split()]))
    return out


def sample_probe(kind, n, seed=1):
    """The kernel's sampling draws (rto_sample_probe): float32 [n, 3]."""
    L = lib()
    L.rto_sample_probe.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    out = np.zeros((n, 3), np.float32)
    assert L.rto_sample_probe(kind, n, seed, out.ctypes.data) == 0
    return out


def sealed(scene):
    """The oracle's sealed spheres (the kernel specification's opaque-inside
    rule): a bool array, one per sphere."""
    v = scene.view()
    out = np.zeros(max(scene.n, 1), np.uint8)
    L = lib()
    L.rto_sealed.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    assert L.rto_sealed(ctypes.addressof(v), out.ctypes.data) == 0
    return out[:scene.n].astype(bool)
