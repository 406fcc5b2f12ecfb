"""rtow -- Python binding (ctypes) of librtow.so, the MI355X render path.

This is the host-side mirror of the reference's process surface for tests,
bench.py and scripting.  Every call goes straight to the C ABI in
include/rt.h; there is no Python or CPU fallback for the render itself: if
librtow.so is missing, or no HIP device is present, the calls raise.

Reference anchors:
  final_scene()   random_scene()        src/cpu/main.cc:32-76
  camera_cpu()    camera::camera        src/cpu/camera.h:8-26
  camera_gpu()    new_camera            src/gpu/camera.h:53-110
  Context.render  render<<<>>>          src/gpu/camera.h:169-195
  tonemap()       write_color           src/cpu/color.h:8-23
  write_ppm()     main.cc:109 / output_image src/gpu/camera.h:197-210
"""
import ctypes
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# RTOW_LIB: load an alternative build (A/B experiments on the GPU box)
LIB_PATH = os.environ.get("RTOW_LIB") or os.path.join(HERE, "librtow.so")

RT_LAMBERTIAN, RT_METAL, RT_DIELECTRIC = 0, 1, 2
RT_ERR_INVALID = -1
RT_CAMERA_CPU, RT_CAMERA_GPU = 0, 1
RT_FLAG_OPEN_INTERVAL = 1
RT_FLAG_METAL_UNIT_VECTOR = 2
RT_FLAG_GPU_SEMANTICS = 3
RT_FLAG_KEEP_COUNTERS = 1 << 8
RT_FLAG_ACCEL_BVH = 1 << 9
RT_FLAG_COUNT_WORK = 1 << 10
RT_FLAG_PILOT_SCHEDULE = 1 << 11  # launch expensive tiles first (4-spp pilot per frame geometry)
RT_FLAG_LAYER_BVH = 1 << 12  # layer scenes: walk the layer BVH instead of the layer grid
RT_CHUNK_SPP = 64  # include/rt.h: kept for compatibility (pixel sums are exact integers, units split evenly)
RT_TONEMAP_CPU, RT_TONEMAP_GPU = 0, 1  # write_color of src/cpu (fp64) / src/gpu (fp32)
RT_KAT_SPHERE_HIT, RT_KAT_REFLECT, RT_KAT_REFRACT, RT_KAT_REFLECTANCE = 0, 1, 2, 3
ABI_VERSION = 6
# rt_context_set_option (include/rt.h): placement / shape / launch options, never semantics
RT_OPT_GRID_PLACEMENT, RT_OPT_GRID_SCALE, RT_OPT_BVH_LEAF = 1, 2, 3
RT_OPT_BVH_COLLAPSE, RT_OPT_BVH_SIDE, RT_OPT_LAUNCH_SAMPLES, RT_OPT_GRID_FIT = 4, 5, 6, 7
RT_OPT_INTERNAL_GRID_PHASE_X, RT_OPT_INTERNAL_GRID_PHASE_Z = 8, 9  # include/rt_internal.h
RT_GRID_AUTO, RT_GRID_LDS, RT_GRID_CELLS_LDS, RT_GRID_GLOBAL = 0, 1, 2, 3
GRID_PLACEMENTS = {"auto": RT_GRID_AUTO, "lds": RT_GRID_LDS, "cells": RT_GRID_CELLS_LDS, "global": RT_GRID_GLOBAL}

_f = ctypes.POINTER(ctypes.c_float)
_u32 = ctypes.POINTER(ctypes.c_uint32)


class SceneView(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("cx", _f), ("cy", _f), ("cz", _f), ("radius", _f),
                ("mat_kind", _u32), ("albedo_rgb", _f), ("mat_param", _f)]


class SceneBuf(ctypes.Structure):
    _fields_ = [("capacity", ctypes.c_uint32), ("n", ctypes.c_uint32), ("cx", _f), ("cy", _f),
                ("cz", _f), ("radius", _f), ("mat_kind", _u32), ("albedo_rgb", _f),
                ("mat_param", _f)]


class Camera(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int32), ("has_lens", ctypes.c_int32),
                ("eye", ctypes.c_float * 3), ("corner", ctypes.c_float * 3),
                ("horiz", ctypes.c_float * 3), ("vert", ctypes.c_float * 3),
                ("lens_u", ctypes.c_float * 3), ("lens_v", ctypes.c_float * 3)]


class Params(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32),
                ("spp", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("row_block", ctypes.c_int32),
                ("band_stride", ctypes.c_int32), ("band_offset", ctypes.c_int32),
                ("local_rows", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("units", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [("segments", ctypes.c_uint64), ("samples", ctypes.c_uint64),
                ("bf_tests", ctypes.c_uint64), ("sphere_tests", ctypes.c_uint64),
                ("box_tests", ctypes.c_uint64), ("box_hits", ctypes.c_uint64),
                ("wave_steps", ctypes.c_uint64),
                ("kernel_ms", ctypes.c_double), ("root_tests", ctypes.c_uint64),
                ("launches", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def lib():
    """Load librtow.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; "
                               "g.build()'` (or make -C ray-tracing-in-one-weekend_amd)")
        # torch's bundled HIP runtime has the same soname as the system one
        # librtow links (libamdhip64.so.7): whichever loads first serves the
        # process, and torch cannot enumerate devices through the system's.
        # So torch, when present, loads first ("Loading").
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        d3 = ctypes.POINTER(ctypes.c_double)
        L.rt_abi_version.restype = ctypes.c_int
        L.rt_strerror.restype = ctypes.c_char_p
        L.rt_strerror.argtypes = [ctypes.c_int]
        L.rt_last_hip_error.restype = ctypes.c_int
        L.rt_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.rt_scene_final.argtypes = [ctypes.c_int, ctypes.POINTER(SceneBuf), d3]
        L.rt_scene_five.argtypes = [ctypes.POINTER(SceneBuf)]
        L.rt_camera_cpu.argtypes = [d3, d3, d3, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.POINTER(Camera)]
        L.rt_camera_gpu.argtypes = [d3, d3, d3, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_double, ctypes.c_double, ctypes.POINTER(Camera)]
        L.rt_context_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        L.rt_context_destroy.argtypes = [ctypes.c_void_p]
        L.rt_context_destroy.restype = None
        L.rt_scene_upload.argtypes = [ctypes.c_void_p, ctypes.POINTER(SceneView)]
        L.rt_render_async.argtypes = [ctypes.c_void_p, ctypes.POINTER(Camera), ctypes.POINTER(Params),
                                      ctypes.c_void_p, ctypes.c_void_p]
        L.rt_render.argtypes = [ctypes.c_void_p, ctypes.POINTER(Camera), ctypes.POINTER(Params),
                                ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.rt_collect_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats)]
        L.rt_reset_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        if hasattr(L, "rt_render_progress"):
            L.rt_render_progress.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint32)]
        L.rt_tonemap_u8.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
        L.rt_tonemap_u8_mode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p]
        L.rt_tonemap_async.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.rt_device_kat.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p]
        L.rt_write_ppm.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int]
        L.rt_internal_accel_info.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                             ctypes.c_void_p, ctypes.c_size_t]
        if hasattr(L, "rt_internal_launch_plan"):
            L.rt_internal_launch_plan.argtypes = [ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p,
                                                  ctypes.c_size_t]
        if hasattr(L, "rt_internal_sealed"):
            L.rt_internal_sealed.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        if hasattr(L, "rt_context_set_option"):  # (absent in pre-ABI-4 builds loaded for A/B runs)
            L.rt_context_set_option.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_double]
        _lib = L
    return _lib


class RTError(RuntimeError):
    def __init__(self, status, where):
        L = lib()
        msg = L.rt_strerror(status).decode()
        if status == -2:
            msg += f" (hipError {L.rt_last_hip_error()})"
        super().__init__(f"{where}: {msg} [{status}]")
        self.status = status


def check(status, where):
    if status != 0:
        raise RTError(status, where)


def device_code_sha16(path=None):
    """Fingerprint of the gfx950 code in a built library: sha256 of its
    .hip_fatbin section (the device code objects only; host-side edits leave it
    unchanged, and rebuilding the same source gives the same bytes).  PMC
    summaries record it so that bench.py can flag counters collected on other
    kernel code."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as f:
        b = f.read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = secs[shstrndx][4]
    for s in secs:
        if b[names + s[0]:b.index(b"\0", names + s[0])] == b".hip_fatbin":
            return hashlib.sha256(b[s[4]:s[4] + s[5]]).hexdigest()[:16]
    return None


def _ptr(a, t):
    return a.ctypes.data_as(t)


@dataclass
class Scene:
    """Sphere scene as SoA numpy arrays (fp32)."""
    cx: np.ndarray
    cy: np.ndarray
    cz: np.ndarray
    radius: np.ndarray
    kind: np.ndarray
    albedo: np.ndarray  # (n, 3)
    param: np.ndarray
    rng_next: float = float("nan")

    @property
    def n(self):
        return int(self.cx.shape[0])

    def view(self):
        """A SceneView pointing into this object's arrays (keep self alive)."""
        for name in ("cx", "cy", "cz", "radius", "albedo", "param"):
            a = getattr(self, name)
            if a.dtype != np.float32 or not a.flags.c_contiguous:
                setattr(self, name, np.ascontiguousarray(a, dtype=np.float32))
        if self.kind.dtype != np.uint32 or not self.kind.flags.c_contiguous:
            self.kind = np.ascontiguousarray(self.kind, dtype=np.uint32)
        return SceneView(self.n, _ptr(self.cx, _f), _ptr(self.cy, _f), _ptr(self.cz, _f),
                         _ptr(self.radius, _f), _ptr(self.kind, _u32), _ptr(self.albedo, _f),
                         _ptr(self.param, _f))


def _scene_from(fill, capacity):
    arr = {k: np.zeros(capacity, np.float32) for k in ("cx", "cy", "cz", "radius", "param")}
    kind = np.zeros(capacity, np.uint32)
    albedo = np.zeros((capacity, 3), np.float32)
    buf = SceneBuf(capacity, 0, _ptr(arr["cx"], _f), _ptr(arr["cy"], _f), _ptr(arr["cz"], _f),
                   _ptr(arr["radius"], _f), _ptr(kind, _u32), _ptr(albedo, _f),
                   _ptr(arr["param"], _f))
    nxt = fill(buf)
    n = buf.n
    return Scene(arr["cx"][:n].copy(), arr["cy"][:n].copy(), arr["cz"][:n].copy(),
                 arr["radius"][:n].copy(), kind[:n].copy(), albedo[:n].copy(),
                 arr["param"][:n].copy(), nxt)


def final_scene(half_extent=11):
    """The final random-spheres scene (486 spheres at half_extent=11)."""
    cap = (2 * half_extent) ** 2 + 8

    def fill(buf):
        nxt = ctypes.c_double()
        check(lib().rt_scene_final(half_extent, ctypes.byref(buf), ctypes.byref(nxt)), "rt_scene_final")
        return nxt.value
    return _scene_from(fill, cap)


def five_scene():
    def fill(buf):
        check(lib().rt_scene_five(ctypes.byref(buf)), "rt_scene_five")
        return float("nan")
    return _scene_from(fill, 8)


def _d3(v):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


def camera_cpu(lookfrom=(13, 2, 3), lookat=(0, 0, 0), vup=(0, 1, 0), vfov=20.0,
               aspect=16.0 / 9.0, aperture=0.1, focus_dist=10.0):
    cam = Camera()
    check(lib().rt_camera_cpu(_d3(lookfrom), _d3(lookat), _d3(vup), vfov, aspect, aperture,
                              focus_dist, ctypes.byref(cam)), "rt_camera_cpu")
    return cam


def camera_gpu(width, height, lookfrom=(13, 2, 3), lookat=(0, 0, 0), vup=(0, 1, 0), vfov=20.0,
               defocus_angle=0.6, focus_dist=10.0):
    cam = Camera()
    check(lib().rt_camera_gpu(_d3(lookfrom), _d3(lookat), _d3(vup), vfov, width, height,
                              defocus_angle, focus_dist, ctypes.byref(cam)), "rt_camera_gpu")
    return cam


def make_params(width, height, spp, max_depth=50, seed=0, flags=0, rank=0, world=1, row_block=8,
                units=0):
    """Params for rank `rank` of `world` (interleaved row bands of row_block rows).

    units: waves sharing each tile's samples in even shares (0 = automatic);
    scheduling only, the image is the same for every value (fixed-point sums)."""
    if world == 1:
        return Params(width, height, spp, max_depth, seed, max(1, height), 1, 0, height, flags, units)
    band_rows = row_block * world
    n_bands = -(-height // band_rows)  # every rank gets the same number of bands
    return Params(width, height, spp, max_depth, seed, row_block, world, rank, n_bands * row_block,
                  flags, units)


def local_to_global_rows(p):
    r = np.arange(p.local_rows)
    band = r // p.row_block
    return (band * p.band_stride + p.band_offset) * p.row_block + r % p.row_block


def device_count():
    n = ctypes.c_int()
    check(lib().rt_device_count(ctypes.byref(n)), "rt_device_count")
    return n.value


class Context:
    """One HIP device + uploaded scene (rt_context)."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        check(lib().rt_context_create(device, ctypes.byref(h)), "rt_context_create")
        self._h = h
        self.device = device
        self.scene = None

    def close(self):
        if self._h:
            lib().rt_context_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, option, value):
        """rt_context_set_option: placement / shape / launch granularity (0 = default)."""
        check(lib().rt_context_set_option(self._h, option, float(value)), "rt_context_set_option")

    def upload(self, scene, grid_mode=None, grid_scale=None, grid_phase=None):
        """rt_scene_upload; grid_mode ("auto", "lds", "cells", "global") and
        grid_scale / grid_phase ((x, z) cell fractions) set the layer grid's
        options first (the image is the same).
        Options are the context's: they stay set for later uploads until set
        again (0 / "auto" restores the default)."""
        if grid_mode is not None:
            self.set_option(RT_OPT_GRID_PLACEMENT, GRID_PLACEMENTS[grid_mode])
        if grid_scale is not None:
            self.set_option(RT_OPT_GRID_SCALE, grid_scale)
        if grid_phase is not None:
            self.set_option(RT_OPT_INTERNAL_GRID_PHASE_X, grid_phase[0])
            self.set_option(RT_OPT_INTERNAL_GRID_PHASE_Z, grid_phase[1])
        v = scene.view()
        check(lib().rt_scene_upload(self._h, ctypes.byref(v)), "rt_scene_upload")
        self.scene = scene

    def grid_scale(self):
        """The cell scale of the context's current layer grid (RT_OPT_GRID_FIT
        refits it per frame geometry); 0.0 without a grid."""
        lib().rt_internal_grid_scale.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]
        g = ctypes.c_double()
        check(lib().rt_internal_grid_scale(self._h, ctypes.byref(g)), "rt_internal_grid_scale")
        return g.value

    def render(self, cam, params):
        """Render synchronously; returns (sums float32 [rows, W, 3], Stats)."""
        out = np.zeros((params.local_rows, params.width, 3), np.float32)
        st = Stats()
        check(lib().rt_render(self._h, ctypes.byref(cam), ctypes.byref(params),
                              out.ctypes.data, ctypes.byref(st)), "rt_render")
        return out, st

    def render_async(self, cam, params, dev_ptr, stream=0):
        """Enqueue into a device pointer (e.g. torch tensor.data_ptr()) on a hipStream_t."""
        check(lib().rt_render_async(self._h, ctypes.byref(cam), ctypes.byref(params),
                                    ctypes.c_void_p(dev_ptr), ctypes.c_void_p(stream)),
              "rt_render_async")

    def tonemap_async(self, dev_sums, n_pixels, spp, dev_out, mode=RT_TONEMAP_CPU, stream=0):
        """write_color on the device: fp32 sums -> bytes, both device pointers."""
        check(lib().rt_tonemap_async(self._h, ctypes.c_void_p(dev_sums), n_pixels, spp, mode,
                                     ctypes.c_void_p(dev_out), ctypes.c_void_p(stream)), "rt_tonemap_async")

    def progress(self):
        """rt_render_progress: (launches done, launches total) of the last render."""
        d, t = ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().rt_render_progress(self._h, ctypes.byref(d), ctypes.byref(t)), "rt_render_progress")
        return d.value, t.value

    def reset_stats(self, stream=0):
        check(lib().rt_reset_stats(self._h, ctypes.c_void_p(stream)), "rt_reset_stats")

    def collect_stats(self):
        st = Stats()
        check(lib().rt_collect_stats(self._h, ctypes.byref(st)), "rt_collect_stats")
        return st


def tonemap(sums, spp, mode=RT_TONEMAP_CPU):
    """write_color on the host: src/cpu's fp64 levels, or src/gpu's fp32 ones."""
    sums = np.ascontiguousarray(sums, dtype=np.float32)
    out = np.zeros(sums.shape, np.uint8)
    n_pix = sums.size // 3
    check(lib().rt_tonemap_u8_mode(sums.ctypes.data, n_pix, spp, mode, out.ctypes.data),
          "rt_tonemap_u8_mode")
    return out


def device_kat(kind, cases, device=0):
    """Evaluate the render kernel's device arithmetic on known-answer cases
    (rt_device_kat): cases [n, <=10] float64 -> [n, 9] float64."""
    cases = np.asarray(cases, np.float64)
    inp = np.zeros((cases.shape[0], 10), np.float64)
    inp[:, :cases.shape[1]] = cases
    out = np.zeros((cases.shape[0], 9), np.float64)
    check(lib().rt_device_kat(device, kind, inp.ctypes.data, inp.shape[0], out.ctypes.data), "rt_device_kat")
    return out


ACCEL_INFO_KEYS = ("nodes_per_order", "bvh_slots", "layer_mode", "extra_pair0", "n_extra_pairs",
                   "grid_nx", "grid_nz", "grid_items", "grid_lds_bytes", "grid_fits_lds",
                   "max_items_per_cell", "grid_starts_ok", "grid_ring_empty", "oref_milli",
                   "layer_slots", "listed_cells", "grid_placement", "grid_scale_milli")


def accel_info(scene, grid_mode="auto", grid_scale=0.0):
    """What rt_scene_upload would build for `scene` with those grid options,
    computed on the host (rt_internal_accel_info; no device): a dict of
    ACCEL_INFO_KEYS."""
    v = scene.view()
    out = np.zeros(len(ACCEL_INFO_KEYS), np.uint64)
    check(lib().rt_internal_accel_info(ctypes.byref(v), GRID_PLACEMENTS[grid_mode], float(grid_scale),
                                       out.ctypes.data, out.size), "rt_internal_accel_info")
    return {k: int(x) for k, x in zip(ACCEL_INFO_KEYS, out)}


def grid_fit(scene, cam, width, height, phase=(0.0, 0.0)):
    """What RT_OPT_GRID_FIT picks for `scene` seen by `cam` in a width x height
    frame, computed on the host (rt_internal_grid_fit_phase; no device), with
    the grid origin shifted by `phase` cells (RT_OPT_INTERNAL_GRID_PHASE_X / _Z): (cell
    scale or 0.0 without an LDS grid, [(candidate scale, modelled cost)])."""
    L = lib()
    L.rt_internal_grid_fit_phase.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_double, ctypes.c_double,
                                             ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_size_t)]
    v = scene.view()
    sc, n = ctypes.c_double(), ctypes.c_size_t()
    costs = np.zeros(2 * 64, np.float64)
    check(L.rt_internal_grid_fit_phase(ctypes.byref(v), ctypes.byref(cam), width, height, float(phase[0]),
                                       float(phase[1]), ctypes.byref(sc), costs.ctypes.data, 64,
                                       ctypes.byref(n)), "rt_internal_grid_fit_phase")
    return sc.value, [(float(costs[2 * i]), float(costs[2 * i + 1])) for i in range(min(64, n.value))]


def sealed(scene):
    """Per sphere, whether the kernel's opaque-inside rule applies to it (a
    sealed lambertian sphere), computed on the host
    (rt_internal_sealed; no device): a bool array."""
    v = scene.view()
    out = np.zeros(max(scene.n, 1), np.uint8)
    check(lib().rt_internal_sealed(ctypes.byref(v), out.ctypes.data, scene.n), "rt_internal_sealed")
    return out[:scene.n].astype(bool)


LAUNCH_PLAN_KEYS = ("ranges", "chunks", "units", "entries", "launches")


def launch_plan(params, launch_samples=0.0):
    """How rt_render would cut a render with `params` into launches under a
    launch-sample budget (0 = default), computed on the host
    (rt_internal_launch_plan; no device): a dict of LAUNCH_PLAN_KEYS."""
    out = np.zeros(len(LAUNCH_PLAN_KEYS), np.uint64)
    check(lib().rt_internal_launch_plan(ctypes.byref(params), float(launch_samples), out.ctypes.data, out.size),
          "rt_internal_launch_plan")
    return {k: int(x) for k, x in zip(LAUNCH_PLAN_KEYS, out)}


def write_ppm(path, rgb, binary=False):
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w = rgb.shape[0], rgb.shape[1]
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    try:
        check(lib().rt_write_ppm(fd, rgb.ctypes.data, w, h, 1 if binary else 0), "rt_write_ppm")
    finally:
        os.close(fd)
