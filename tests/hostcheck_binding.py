"""Builds and binds tests/hostcheck (the GPU kernel's per-lane code compiled for the CPU).
TEST INFRASTRUCTURE ONLY."""
import ctypes as C
import os
import subprocess

import numpy as np

from blenderraytracer_amd import capi

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "hostcheck", "pt_hostcheck.cpp")
DEPS = [SRC] + [os.path.join(ROOT, "blenderraytracer_amd", "csrc", f) for f in ("pt_core.h", "pt_path.h", "scene_pack.h",
                                                                          "pool_order.h", "js_math.h")]
LIB = os.path.join(HERE, "hostcheck", "_build", "libpt_hostcheck.so")
_lib = None


def build(defines=(), name="libpt_hostcheck.so"):
    target = os.path.join(os.path.dirname(LIB), name)
    os.makedirs(os.path.dirname(target), exist_ok=True)
    if os.path.exists(target) and all(os.path.getmtime(target) >= os.path.getmtime(d) for d in DEPS):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = "%s.tmp%d" % (target, os.getpid())     # parallel test workers: build aside, rename atomically
    subprocess.check_call([hipcc, "--offload-host-only", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                           *[f"-D{d}" for d in defines], "-I", os.path.join(ROOT, "include"), SRC, "-o", tmp])
    os.replace(tmp, target)
    return target


def _bind(L):
    L.ptc_render.argtypes = [C.POINTER(capi.SceneDesc), C.POINTER(capi.Settings), C.POINTER(C.c_double),
                             C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    L.ptc_bvh_check.argtypes = [C.POINTER(capi.SceneDesc), C.c_longlong, C.c_uint, C.POINTER(C.c_longlong)]
    L.ptc_bvh_check.restype = C.c_longlong
    L.ptc_bvh_info.argtypes = [C.POINTER(capi.SceneDesc)] + [C.POINTER(C.c_int)] * 4
    L.ptc_away_check.argtypes = [C.c_longlong, C.c_uint, C.POINTER(C.c_longlong)]
    L.ptc_away_check.restype = C.c_longlong
    L.ptc_bvh_rays.argtypes = [C.POINTER(capi.SceneDesc), C.c_longlong, C.c_uint, C.c_longlong, C.POINTER(C.c_double),
                               C.POINTER(C.c_double), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.ptc_bvh_rays.restype = C.c_longlong
    return L


def lib(defines=()):
    """The hostcheck library; `defines` builds (and caches) a variant with -D flags."""
    global _lib
    if defines:
        return _bind(C.CDLL(build(defines, "libpt_hostcheck_%s.so" % "_".join(d.replace("=", "") for d in defines))))
    if _lib is None:
        _lib = _bind(C.CDLL(build()))
    return _lib


def bvh_info(packed, L=None):
    """(deepest leaf of the binary trees, two-child nodes)"""
    return bvh_shape(packed, L)[:2]


def bvh_shape(packed, L=None):
    """(deepest leaf, two-child nodes, sphere indices of the dominant spheres tested before the walk)"""
    depth, nodes2, nbig, big = C.c_int(), C.c_int(), C.c_int(), (C.c_int * 8)()
    (L or lib()).ptc_bvh_info(C.byref(packed.desc), C.byref(depth), C.byref(nodes2), C.byref(nbig), big)
    return depth.value, nodes2.value, list(big[:nbig.value])


def bvh_check(packed, n, seed):
    """(rays whose brute-force and BVH closest hits differ, rays that hit something)"""
    hits = C.c_longlong()
    bad = lib().ptc_bvh_check(C.byref(packed.desc), n, seed, C.byref(hits))
    assert bad >= 0
    return bad, hits.value


def bvh_rays(packed, n, seed, host_n=None):
    """The BVH stress rays (n x 6 float64: origin, direction) and the host's World-order closest hit
    (t, kind, index) of the first host_n of them (default all) — the kernel's own code compiled for the
    CPU."""
    host_n = n if host_n is None else host_n
    rays = np.zeros((n, 6))
    t = np.full(n, np.nan)
    kind = np.full(n, -2, dtype=np.int32)
    idx = np.full(n, -2, dtype=np.int32)
    m = lib().ptc_bvh_rays(C.byref(packed.desc), n, seed, host_n, rays.ctypes.data_as(C.POINTER(C.c_double)),
                           t.ctypes.data_as(C.POINTER(C.c_double)), kind.ctypes.data_as(C.POINTER(C.c_int)),
                           idx.ctypes.data_as(C.POINTER(C.c_int)))
    assert m >= 0
    return rays[:m], t[:m], kind[:m], idx[:m]


EVENTS = ["f64_sphere_tests", "disc_nonneg", "second_root", "accept", "lambertian", "metal", "dielectric", "emissive",
          "miss", "samples", "sphere_draw_rounds", "disk_draw_rounds", "filter_tests", "dielectric_schlick",
          "tri_filter_tests", "tri_tests"]


def event_counts(packed, settings_list, walk):
    """Events per segment of the kernel's own code run on the CPU over the given crops (pt_core.h
    RT_HCOUNT; the instruction-floor model of bench.py): walk "grid" | "bvh" | "brute" as the GPU runs it."""
    L = lib(("RT_HOST_COUNTERS=1",))
    L.ptc_work.argtypes = [C.POINTER(capi.SceneDesc), C.POINTER(capi.Settings), C.POINTER(C.c_double)]
    L.ptc_host_counts.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    cnt = (C.c_ulonglong * 16)()
    L.ptc_host_counts(cnt, 1)
    out = (C.c_double * 4)()
    tot = [0.0] * 4
    for st in settings_list:
        st.accel = {"grid": 4, "bvh": capi.RT_ACCEL_BVH, "brute": capi.RT_ACCEL_BRUTE}[walk]
        assert L.ptc_work(C.byref(packed.desc), C.byref(st), out) == 0
        tot = [a + b for a, b in zip(tot, out)]
    L.ptc_host_counts(cnt, 1)
    seg = max(tot[0], 1.0)
    res = {"segments": tot[0], "walk_steps": tot[1] / seg, "sphere_tests_work": tot[2] / seg, "tri_tests": tot[3] / seg}
    res.update({n: cnt[k] / seg for k, n in enumerate(EVENTS)})
    return res


def render(packed, settings, L=None):
    """Per-pixel linear means, segment and draw counts computed by the kernel's own code on the CPU
    (`L`: a variant library from lib(defines))."""
    cw = settings.crop_w or settings.width
    ch = settings.crop_h or settings.height
    s = np.zeros((ch, cw, 3))
    segs = np.zeros((ch, cw), dtype=np.uint32)
    draws = np.zeros((ch, cw), dtype=np.uint32)
    rc = (L or lib()).ptc_render(C.byref(packed.desc), C.byref(settings), s.ctypes.data_as(C.POINTER(C.c_double)),
                          segs.ctypes.data_as(C.POINTER(C.c_uint32)), draws.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert rc == 0
    return {"mean": s / settings.samples, "segments": segs, "draws": draws}


def pool_order(cw, ch, chunks, one_wave=True):
    """The pool's visiting order (pool_order.h): (items by workgroup / queue position, RT_TILE_BLOCK,
    RT_XCD_RUN, tiles)."""
    import numpy as np
    L = lib()
    L.ptc_pool_order.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint32), C.POINTER(C.c_int)]
    L.ptc_pool_order.restype = C.c_longlong
    tiles = ((cw + 7) // 8) * ((ch + 7) // 8)
    out = np.zeros(tiles * chunks, dtype=np.uint32)
    par = (C.c_int * 3)()
    n = L.ptc_pool_order(cw, ch, chunks, int(one_wave), out.ctypes.data_as(C.POINTER(C.c_uint32)), par)
    assert n == tiles * chunks
    return out, par[0], par[1], par[2]
