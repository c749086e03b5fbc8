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
DEPS = [SRC] + [os.path.join(ROOT, "blenderraytracer_amd", "csrc", f) for f in ("pt_core.h", "pt_path.h", "scene_pack.h")]
LIB = os.path.join(HERE, "hostcheck", "_build", "libpt_hostcheck.so")
_lib = None


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(d) for d in DEPS):
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.check_call([hipcc, "--offload-host-only", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                           "-I", os.path.join(ROOT, "include"), SRC, "-o", LIB])
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.ptc_render.argtypes = [C.POINTER(capi.SceneDesc), C.POINTER(capi.Settings), C.POINTER(C.c_double),
                                    C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
        _lib.ptc_bvh_check.argtypes = [C.POINTER(capi.SceneDesc), C.c_longlong, C.c_uint, C.POINTER(C.c_longlong)]
        _lib.ptc_bvh_check.restype = C.c_longlong
    return _lib


def bvh_check(packed, n, seed):
    """(rays whose brute-force and BVH closest hits differ, rays that hit something)"""
    hits = C.c_longlong()
    bad = lib().ptc_bvh_check(C.byref(packed.desc), n, seed, C.byref(hits))
    assert bad >= 0
    return bad, hits.value


def render(packed, settings):
    """Per-pixel linear means, segment and draw counts computed by the kernel's own code on the CPU."""
    cw = settings.crop_w or settings.width
    ch = settings.crop_h or settings.height
    s = np.zeros((ch, cw, 3))
    segs = np.zeros((ch, cw), dtype=np.uint32)
    draws = np.zeros((ch, cw), dtype=np.uint32)
    rc = lib().ptc_render(C.byref(packed.desc), C.byref(settings), s.ctypes.data_as(C.POINTER(C.c_double)),
                          segs.ctypes.data_as(C.POINTER(C.c_uint32)), draws.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert rc == 0
    return {"mean": s / settings.samples, "segments": segs, "draws": draws}
