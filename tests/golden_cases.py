"""Loader for the reference-generated golden fixtures (tests/golden/, made by
oracle/ref_harness/run_reference.mjs from the real /root/reference renderer)."""
import gzip
import json
import os

import numpy as np

from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import load_scene_json

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
_manifest = None


def manifest():
    global _manifest
    if _manifest is None:
        with open(os.path.join(GOLDEN, "manifest.json")) as f:
            _manifest = json.load(f)
    return _manifest


# cases whose CPU renders take a minute or more (the reference's brute-force 50k-triangle mesh at 16x16 x
# 256 spp, 1.5 M RTOW samples): pinned by the C oracle, the kernel's host build and the GPU tests, left
# out of the slower JS CPU path's run and of repeated CPU passes
HEAVY = ("cfg5_mesh50k_256spp_wide", "cfg3_rtow_crop_512spp_wide")


def case_names(heavy=True):
    return sorted(k for k in manifest()["cases"] if heavy or k not in HEAVY)


def load_array(case, key):
    c = manifest()["cases"][case]
    dt = {"linear": np.float64, "post": np.float64, "rgba8": np.uint8, "segs": np.uint32, "draws": np.uint32,
          "denoised": np.float32}[key]
    raw = gzip.open(os.path.join(GOLDEN, c["files"][key])).read()
    _, _, cw, ch = c["crop"]
    comp = {"linear": 3, "post": 3, "rgba8": 4, "segs": 1, "draws": 1, "denoised": 4}[key]
    a = np.frombuffer(raw, dtype=dt).reshape(ch, cw, comp)
    return a[..., 0] if comp == 1 else a


def has(case, key):
    return key in manifest()["cases"][case]["files"]


def kats():
    with gzip.open(os.path.join(GOLDEN, "kats.json.gz")) as f:
        return decode(json.load(f))


def decode(v):
    if isinstance(v, str) and v in ("NaN", "Infinity", "-Infinity"):
        return float(v.replace("Infinity", "inf"))
    if isinstance(v, list):
        return [decode(x) for x in v]
    if isinstance(v, dict):
        return {k: decode(x) for k, x in v.items()}
    return v


def tracer_for(case, precision=capi.RT_PREC_F64, device=0):
    """GpuRayTracer configured exactly as the harness configured the reference RayTracer."""
    c = manifest()["cases"][case]
    w, h = c["requested"]
    rt = GpuRayTracer(w, h, seed=c["seed"], device=device, precision=precision)
    assert rt.load_from_json(load_scene_json(c["scene"]))
    rt.update_render_settings(c["settings_in"])
    if c["background_in"]:
        rt.update_background(c["background_in"]["type"], c["background_in"]["intensity"])
    assert (rt.width, rt.height) == (c["width"], c["height"])
    return rt, c


def ensure_mesh50k_file():
    """scenes/mesh50k.json is git-ignored: the Node tools read it from disk, so write it once."""
    from blenderraytracer_amd.scene import SCENES_DIR
    p = os.path.join(SCENES_DIR, "mesh50k.json")
    if not os.path.exists(p) or os.path.getsize(p) == 0:
        data = load_scene_json("mesh50k")  # generated before the file exists (no empty-file race)
        tmp = p + f".tmp{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(data, f)
        os.replace(tmp, p)
