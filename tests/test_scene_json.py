"""The C++ scene-JSON loader (include/rt_scene_json.h, librt_hip.so; host code, runs without a GPU)
against the Python host's loader, which tests/test_js_host.py pins to the reference's own objects
(SceneLoader.loadFromJSON, scene-loader.js:20-284, through RayTracer.loadFromJSON,
ray-tracer.js:304-333).  Same objects in World order, same materials, bit-identical camera vectors,
plane/triangle normals and Perlin permutation."""
import ctypes as C
import json
import os

import numpy as np
import pytest

import golden_cases as gc
from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import SCENES_DIR, load_scene_json

SCENES = sorted(f for f in os.listdir(SCENES_DIR) if f.endswith(".json") and f != "mesh50k.json")


class JsonScene:
    def __init__(self, text, width, height, seed):
        self.lib = capi.load_library()
        self.h = C.c_void_p()
        raw = text.encode() if isinstance(text, str) else text
        self.status = self.lib.rt_json_scene_load(raw, len(raw), width, height, seed, C.byref(self.h))
        self.error = self.lib.rt_last_error().decode() if self.status else ""

    def desc(self):
        return self.lib.rt_json_scene_desc(self.h).contents

    def size(self):
        w, h = C.c_int32(), C.c_int32()
        self.lib.rt_json_scene_size(self.h, C.byref(w), C.byref(h))
        return w.value, h.value

    def close(self):
        if self.h:
            self.lib.rt_json_scene_destroy(self.h)
            self.h = C.c_void_p()


def canonical(d):
    """Per-object (type, geometry, resolved material, triangles): independent of material dedup."""
    out = []
    for i in range(d.num_objects):
        o = d.objects[i]
        m = d.materials[o.material]
        mat = (m.type, tuple(m.albedo), m.roughness, m.ior, tuple(m.emission))
        if o.type in (capi.RT_OBJ_TRIANGLE, capi.RT_OBJ_MESH):
            tris = np.ctypeslib.as_array(d.triangles, shape=(max(1, d.num_triangles) * 12,))
            geo = tris[o.first * 12:(o.first + o.count) * 12].tobytes()
            out.append((o.type, o.count, geo, mat))
        else:
            out.append((o.type, np.array(list(o.g)).tobytes(), mat))
    return out


def camera_bits(d):
    c = d.camera
    vals = [*c.origin, *c.lower_left, *c.horizontal, *c.vertical, *c.u, *c.v, *c.w, c.lens_radius]
    return np.array(vals).tobytes(), c.type


def check_same(text, width, height, seed):
    data = json.loads(text)
    rt = GpuRayTracer(width, height, seed=seed)
    ok = rt.load_from_json(data)
    js = JsonScene(text, width, height, seed)
    try:
        assert (js.status == 0) == ok, js.error
        if not ok:
            return js.error
        p = rt.packed().desc
        d = js.desc()
        assert js.size() == (rt.width, rt.height)
        assert canonical(d) == canonical(p)
        assert camera_bits(d) == camera_bits(p)
        assert (d.background, d.sky_intensity, tuple(d.solid_color)) == (p.background, p.sky_intensity, tuple(p.solid_color))
        assert list(d.perm) == list(p.perm)
        assert d.abi_version == capi.RT_ABI_VERSION
    finally:
        js.close()
    return None


@pytest.mark.parametrize("scene", SCENES)
def test_scene_files(scene):
    with open(os.path.join(SCENES_DIR, scene)) as f:
        text = f.read()
    for (w, h, seed) in ((256, 256, 1), (1920, 1080, 42), (640, 360, 0xFFFFFFFF)):
        assert check_same(text, w, h, seed) is None


def test_mesh50k():
    text = json.dumps(load_scene_json("mesh50k"))
    assert check_same(text, 1920, 1080, 5) is None


@pytest.mark.parametrize("case", gc.case_names())
def test_golden_cases_load_like_python(case):
    c = gc.manifest()["cases"][case]
    text = json.dumps(load_scene_json(c["scene"]))
    w, h = c["requested"]
    assert check_same(text, w, h, c["seed"]) is None


EDGE = {
    # sphere radius 0 -> 1 (`radius || 1.0`), metal roughness clamped, unknown material -> default,
    # missing material -> Lambertian 0.8, unknown object type skipped, object without type skipped
    "defaults": {"objects": [
        {"type": "sphere", "center": [0, 0, -2], "radius": 0, "material": {"type": "metal", "color": [1, 0, 0], "roughness": 7}},
        {"type": "SPHERE", "center": [1, 0, -2], "radius": -0.5, "material": {"type": "unobtainium"}},
        {"type": "sphere", "center": [1, 0]},
        {"type": "cone", "center": [0, 0, 0]},
        {"center": [0, 0, 0]},
        {"type": "plane", "point": [0, -1, 0], "normal": [0, 7, 1], "material": {"type": "emissive", "color": [1, 1, 1], "intensity": 3}},
        {"type": "box", "min": [0, 0, 0], "max": [1, 1, 1], "material": {"type": "dielectric"}},
        {"type": "triangle", "v0": [0, 0, 0], "v1": [1, 0, 0], "v2": [0, 1, 0], "material": {"type": "Emissive"}},
        {"type": "mesh", "vertices": [[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 1]],
         "indices": [0, 1, 2, 2, 9, 3, 1.5, 2, 3, -1, 0, 1, 0, 1]},
        {"type": "mesh", "vertices": [[0, 0, 0]], "indices": []},
        {"type": "mesh", "vertices": [[0, 0, 0]]},
    ], "camera": {"position": [0, 0, 0.5], "lookAt": [0, 0, 0], "fov": 60, "aperture": 0.2}},
    "resolution_resize": {"objects": [{"type": "sphere", "center": [0, 0, -1], "radius": 0.5}],
                          "camera": {"position": [1, 2, 3], "lookAt": [0, 0, -1], "resolution": [320, 200],
                                     "focusDist": 4, "aspect": 2.5}},
    "orthographic_and_bg": {"objects": [], "camera": {"type": "orthographic", "aspect": 0},
                            "background": {"type": "procedural_sky", "intensity": 0.25}},
    "json_solid_bug": {"objects": [], "background": {"type": "solid", "color": [1, 0, 0]}},
    "no_camera": {"objects": [{"type": "box", "min": [-1, -1, -3], "max": [1, 1, -2]}],
                  "background": {"type": "weird", "intensity": 0}},
    "null_values": {"objects": [{"type": "sphere", "center": [None, 1, False], "radius": None,
                                 "material": {"type": "metal", "roughness": None, "color": [True, 0.5, None]}}],
                    "camera": {"position": [0, 1, 5], "fov": None, "focusDist": None}},
}


@pytest.mark.parametrize("name", sorted(EDGE))
def test_loader_semantics_edge_cases(name):
    assert check_same(json.dumps(EDGE[name]), 200, 100, 9) is None


@pytest.mark.parametrize("text", ["", "{", '{"objects": [}', "[1, 2]", '{"a": 1} x', '{"a": "\\q"}',
                                  '{"objects": [{"type": 5}]}', '{"objects": [null]}'])
def test_malformed_input_is_rejected(text):
    js = JsonScene(text, 64, 64, 1)
    assert js.status == -1 and js.error                      # RT_ERR_INVALID, like loadFromJSON's false
    js.close()
    try:                                                      # the Python host agrees where JSON parses
        data = json.loads(text)
    except ValueError:
        return
    assert not GpuRayTracer(64, 64, seed=1).load_from_json(data)


def test_json_parser_details():
    """Escapes, unicode, exponents, duplicate keys (last wins, as JSON.parse)."""
    text = ('{"objects": [{"type": "sph\\u0065re", "center": [1e0, -0.5E+1, 2.5e-1], "radius": 1e-3,'
            ' "radius": 0.75, "name": "caf\\u00e9 \\ud83d\\ude00 \\"q\\""}], "camera": {"fov": 3.0e1}}')
    assert check_same(text, 100, 50, 3) is None
    js = JsonScene(text, 100, 50, 3)
    d = js.desc()
    assert d.objects[0].type == capi.RT_OBJ_SPHERE and list(d.objects[0].g)[:4] == [1.0, -5.0, 0.25, 0.75]
    js.close()


LOADER_CASES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "loader_cases.json")))["cases"]


@pytest.mark.parametrize("name", sorted(LOADER_CASES))
def test_loader_cases_match_reference(name):
    """Loader-only fixtures from the REAL reference (oracle/ref_harness/run_reference.mjs --loader):
    RayTracer.loadFromJSON's verdict on each scene — e.g. a light whose `type` is a truthy non-string
    makes _createLight's type.toLowerCase() throw (scene-loader.js:187) and the load fail, while a
    non-string camera type loads (camera.js compares it with === only) — and, when it loads, the
    camera vectors bit for bit.  Both the Python host and the C++ loader (check_same: they also agree
    with each other object by object) must give the reference's verdict."""
    c = LOADER_CASES[name]
    err = check_same(json.dumps(c["scene"]), 32, 24, 1)
    assert (err is None) == c["ok"], (name, err)
    if c["ok"]:
        rt = GpuRayTracer(32, 24, seed=1)
        assert rt.load_from_json(c["scene"])
        cam = rt.packed().desc.camera
        got = [list(cam.origin), list(cam.lower_left), list(cam.horizontal), list(cam.vertical)]
        assert got == c["camera"], name
        assert cam.type == (capi.RT_CAM_ORTHOGRAPHIC if c["camera_type"] == "orthographic" else capi.RT_CAM_PERSPECTIVE)
