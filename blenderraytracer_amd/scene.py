"""Host-side scene model: the reference's scene-JSON semantics, packed for the C ABI.

Restates, in IEEE double exactly as the JavaScript evaluates it (Python floats are binary64 and
never fused):
  SceneLoader.loadFromJSON / _createObject / _createMaterial / _createCamera  js/scene-loader.js:20-284
  Camera constructor                                                          js/camera.js:8-36
  Plane normal / Triangle normal / TriangleMesh construction                  js/geometry.js:50-53,140-146,193-237
  RayTracer default scene, setupCamera (resize), updateBackground             js/ray-tracer.js:42-77,439-474,568-585
The packed form is include/rt_hip.h's rt_scene_desc (objects in World.objects insertion order).
Lights are parsed by the reference but never used by the renderer, so they are dropped.
"""
import ctypes as C
import json
import math
import os

import numpy as np

from . import capi
from .jsmath import js_tan
from .rng import permutation

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES_DIR = os.path.join(REPO, "scenes")


# ---- JS value semantics -------------------------------------------------------------------------
def truthy(v):
    """JavaScript ToBoolean for JSON values (`a || b`)."""
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return not (v == 0 or v != v)
    if isinstance(v, str):
        return v != ""
    return True


def js_or(a, b):
    return a if truthy(a) else b


def num(v):
    """JS ToNumber for the values JSON can hold in a numeric slot (null -> 0)."""
    if v is None or v is False:
        return 0.0
    if v is True:
        return 1.0
    return float(v)


def parse_vec3(arr):  # scene-loader.js:268-273
    if isinstance(arr, list) and len(arr) >= 3:
        return (num(arr[0]), num(arr[1]), num(arr[2]))
    return (0.0, 0.0, 0.0)


# ---- Vec3 (js/math.js:6-19), tuples of doubles ----------------------------------------------------
def vadd(a, b): return (a[0] + b[0], a[1] + b[1], a[2] + b[2])
def vsub(a, b): return (a[0] - b[0], a[1] - b[1], a[2] - b[2])
def vmul(a, s): return (a[0] * s, a[1] * s, a[2] * s)
def vdiv(a, s): return (a[0] / s, a[1] / s, a[2] / s)
def vdot(a, b): return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]
def vcross(a, b): return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])
def vlen(a): return math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2])


def vnorm(a):
    n = vlen(a)
    return vdiv(a, n) if n > 0 else (0.0, 0.0, 0.0)


# ---- Camera (js/camera.js:8-36) -------------------------------------------------------------------
class Camera:
    def __init__(self, look_from, look_at, vup, vfov, aspect, aperture, focus_dist, type="perspective"):
        self.type = type
        self.aperture = aperture
        self.focus_dist = focus_dist
        self.fov = vfov
        theta = vfov * math.pi / 180
        h = js_tan(theta / 2)                 # V8's Math.tan (camera.js:15; jsmath.py)
        vh = 2.0 * h
        vw = aspect * vh
        self.w = vnorm(vsub(look_from, look_at))
        self.u = vnorm(vcross(vup, self.w))
        self.v = vcross(self.w, self.u)
        self.origin = look_from
        if type == "perspective":
            self.horizontal = vmul(self.u, vw * focus_dist)
            self.vertical = vmul(self.v, vh * focus_dist)
            self.lower_left = vsub(vsub(vsub(self.origin, vdiv(self.horizontal, 2)), vdiv(self.vertical, 2)),
                                   vmul(self.w, focus_dist))
        else:
            self.horizontal = vmul(self.u, vw)
            self.vertical = vmul(self.v, vh)
            self.lower_left = vsub(vsub(self.origin, vdiv(self.horizontal, 2)), vdiv(self.vertical, 2))
        self.lens_radius = aperture / 2

    def desc(self):
        d = capi.CameraDesc()
        for name, src in (("origin", self.origin), ("lower_left", self.lower_left), ("horizontal", self.horizontal),
                          ("vertical", self.vertical), ("u", self.u), ("v", self.v), ("w", self.w)):
            getattr(d, name)[:] = src
        d.lens_radius = self.lens_radius
        # getRay branches on === 'orthographic' (camera.js:40); the constructor on === 'perspective'
        d.type = capi.RT_CAM_ORTHOGRAPHIC if self.type == "orthographic" else capi.RT_CAM_PERSPECTIVE
        return d


# ---- materials / objects ------------------------------------------------------------------------
def _material(m):  # scene-loader.js:143-173 + materials.js constructors
    if not m or not isinstance(m, dict) or not truthy(m.get("type")):
        return ("lambertian", (0.8, 0.8, 0.8))
    t = _js_lower(m["type"], "material")
    if t == "lambertian":
        return ("lambertian", parse_vec3(m.get("color")))
    if t == "metal":
        r = m["roughness"] if "roughness" in m else 0.0
        return ("metal", parse_vec3(m.get("color")), min(num(r), 1.0))  # Math.min(roughness, 1)
    if t == "dielectric":
        return ("dielectric", num(m["ior"]) if "ior" in m else 1.5)
    if t == "emissive":
        inten = num(m["intensity"]) if "intensity" in m else 1.0
        return ("emissive", vmul(parse_vec3(m.get("color")), inten))
    return ("lambertian", (0.8, 0.8, 0.8))


class World:
    """World (js/world.js:8-16): objects in insertion order, background, skyIntensity, perm."""

    def __init__(self, perm):
        self.objects = []      # (kind, material, payload)
        self.background = capi.RT_BG_GRADIENT
        self.sky_intensity = 1.0
        self.solid_color = (0.1, 0.1, 0.1)
        self.perm = list(perm)

    def add(self, kind, material, payload):
        self.objects.append((kind, material, payload))

    def triangle_count(self):
        return sum(len(p) if k == "mesh" else 1 for k, _, p in self.objects if k in ("mesh", "triangle"))


def _triangle(v0, v1, v2):  # geometry.js:138-146: normal = normalize(cross(v1-v0, v2-v0))
    return (v0, v1, v2, vnorm(vcross(vsub(v1, v0), vsub(v2, v0))))


def _is_index(i):
    return isinstance(i, (int, float)) and not isinstance(i, bool) and float(i).is_integer() and i >= 0


def _mesh(vertices, indices):  # geometry.js:193-237
    tris = []
    n = len(vertices)
    for i in range(0, len(indices), 3):
        if i + 2 >= len(indices):
            continue                                   # incomplete triangle
        idx = indices[i:i + 3]
        if any(isinstance(x, (int, float)) and not isinstance(x, bool) and x >= n for x in idx):
            continue                                   # idx >= vertices.length
        vs = [vertices[int(x)] if _is_index(x) else (0.0, 0.0, 0.0) for x in idx]   # undefined -> _ensureVec3 -> 0
        tris.append(_triangle(*vs))
    return tris


def _js_lower(t, what):
    """`x.type.toLowerCase()`: throws (so loadFromJSON returns false) unless x.type is a string."""
    if not isinstance(t, str):
        raise TypeError(f"{what}.type.toLowerCase is not a function")
    return t.lower()


def _create_object(o, world):  # scene-loader.js:90-137
    if o is None:
        raise TypeError("Cannot read property 'type' of null")
    if not isinstance(o, dict) or not truthy(o.get("type")):
        return
    mat = _material(o.get("material") if truthy(o.get("material")) else {"type": "lambertian", "color": [0.8, 0.8, 0.8]})
    t = _js_lower(o["type"], "object")
    if t == "sphere":
        world.add("sphere", mat, (parse_vec3(o.get("center")), num(js_or(o.get("radius"), 1.0))))
    elif t == "plane":
        world.add("plane", mat, (parse_vec3(o.get("point")), vnorm(parse_vec3(o.get("normal")))))
    elif t == "box":
        world.add("box", mat, (parse_vec3(o.get("min")), parse_vec3(o.get("max"))))
    elif t == "triangle":
        world.add("triangle", mat, _triangle(parse_vec3(o.get("v0")), parse_vec3(o.get("v1")), parse_vec3(o.get("v2"))))
    elif t == "mesh":
        if not truthy(o.get("vertices")) or not truthy(o.get("indices")):
            return
        verts = [parse_vec3(v) for v in o["vertices"]]
        world.add("mesh", mat, _mesh(verts, o["indices"]))


def create_camera(cam, aspect):  # scene-loader.js:205-262
    position = parse_vec3(js_or(cam.get("position"), [0, 0, 5]))
    look_at = parse_vec3(js_or(cam.get("lookAt"), [0, 0, 0]))
    up = parse_vec3(js_or(cam.get("up"), [0, 1, 0]))
    fov = num(cam["fov"]) if "fov" in cam else 45
    aperture = num(cam["aperture"]) if "aperture" in cam else 0.0
    if vlen(vsub(position, look_at)) < 1.0:
        direction = vmul(vnorm(vsub(position, look_at)), -1)
        look_at = vadd(position, vmul(direction, 100))
    focus = cam.get("focusDist") if "focusDist" in cam else None
    focus = vlen(vsub(position, look_at)) if focus is None and "focusDist" not in cam else num(focus)
    ctype = js_or(cam.get("type"), "perspective")
    final_aspect = num(js_or(cam.get("aspect"), aspect))
    return Camera(position, look_at, up, fov, final_aspect, aperture, focus, ctype)


def load_from_json(data, width, height, perm):
    """SceneLoader.loadFromJSON (scene-loader.js:20-84) -> (world, camera|None, new_dims|None)."""
    new_dims = None
    cam = data.get("camera")
    if truthy(cam) and truthy(cam.get("resolution")):
        new_dims = (int(cam["resolution"][0]), int(cam["resolution"][1]))
        width, height = new_dims
    world = World(perm)
    bg = data.get("background")
    if truthy(bg):
        t = bg.get("type")
        if t == "gradient":
            world.background = capi.RT_BG_GRADIENT
        elif t in ("solid", "hdri"):
            world.background = capi.RT_BG_NAN      # bound factory -> NaN radiance (scene-loader.js:41-45)
        elif t == "procedural_sky":
            world.background = capi.RT_BG_PROCEDURAL_SKY
        else:
            world.background = capi.RT_BG_GRADIENT
        if "intensity" in bg:
            world.sky_intensity = num(bg["intensity"])
    objs = data.get("objects")
    if isinstance(objs, list):
        for o in objs:
            _create_object(o, world)
    # lights (scene-loader.js:69-76) are parsed but never rendered; _createLight calls
    # lightData.type.toLowerCase() (:187), which throws for a truthy non-string type: the load fails
    lights = data.get("lights")
    if isinstance(lights, list):
        for lt in lights:
            if isinstance(lt, dict) and truthy(lt.get("type")):
                _js_lower(lt["type"], "light")
    camera = create_camera(cam, width / height) if truthy(cam) else None
    return world, camera, new_dims


def default_scene(width, height, perm):
    """RayTracer.setupDefaultScene (ray-tracer.js:42-77)."""
    w = World(perm)
    w.add("plane", ("lambertian", (0.5, 0.5, 0.5)), ((0.0, -0.5, 0.0), vnorm((0.0, 1.0, 0.0))))
    w.add("sphere", ("lambertian", (0.7, 0.3, 0.3)), ((0.0, 0.0, -1.0), 0.5))
    w.add("sphere", ("dielectric", 1.5), ((-1.0, 0.0, -1.0), 0.5))
    w.add("sphere", ("metal", (0.8, 0.8, 0.9), 0.1), ((1.0, 0.0, -1.0), 0.5))
    w.add("sphere", ("emissive", vmul((1.0, 1.0, 1.0), 5)), ((0.0, 1.5, -1.0), 0.3))
    cam = Camera((3.0, 2.0, 2.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0), 45, width / height, 0.0, 10.0)
    return w, cam


def setup_camera(cam, width, height):
    """RayTracer.setupCamera after a resize (ray-tracer.js:439-474): aspect becomes W/H."""
    look_at = vsub(cam.origin, vmul(cam.w, cam.focus_dist))
    return Camera(cam.origin, look_at, cam.v, js_or(cam.fov, 45), width / height, js_or(cam.aperture, 0.0),
                  js_or(cam.focus_dist, 10.0), js_or(cam.type, "perspective"))


# ---- packing into rt_scene_desc ------------------------------------------------------------------
_MAT_CODE = {"lambertian": capi.RT_MAT_LAMBERTIAN, "metal": capi.RT_MAT_METAL,
             "dielectric": capi.RT_MAT_DIELECTRIC, "emissive": capi.RT_MAT_EMISSIVE}

# canonical record bytes per primitive test at f32: sphere 16, plane 24, box 24, tri 36
RECORD_BYTES = {"sphere": 16, "plane": 24, "box": 24, "triangle": 36}


class PackedScene:
    """Owns the arrays an rt_scene_desc points into (keep it alive while the desc is used)."""

    def __init__(self, world, camera):
        mats, mat_index = [], {}
        objs = []
        tris = []
        for kind, mat, payload in world.objects:
            key = repr(mat)
            if key not in mat_index:
                mat_index[key] = len(mats)
                mats.append(mat)
            o = capi.ObjectDesc()
            o.material = mat_index[key]
            if kind == "sphere":
                o.type = capi.RT_OBJ_SPHERE
                o.g[:] = (*payload[0], payload[1], 0.0, 0.0)
            elif kind == "plane":
                o.type = capi.RT_OBJ_PLANE
                o.g[:] = (*payload[0], *payload[1])
            elif kind == "box":
                o.type = capi.RT_OBJ_BOX
                o.g[:] = (*payload[0], *payload[1])
            elif kind == "triangle":
                o.type = capi.RT_OBJ_TRIANGLE
                o.first, o.count = len(tris), 1
                tris.append(payload)
            elif kind == "mesh":
                o.type = capi.RT_OBJ_MESH
                o.first, o.count = len(tris), len(payload)
                tris.extend(payload)
            objs.append(o)
        self.objects = (capi.ObjectDesc * max(1, len(objs)))(*objs)
        self.materials = (capi.MaterialDesc * max(1, len(mats)))()
        for i, m in enumerate(mats):
            d = self.materials[i]
            d.type = _MAT_CODE[m[0]]
            if m[0] in ("lambertian", "metal"):
                d.albedo[:] = m[1]
            if m[0] == "metal":
                d.roughness = m[2]
            if m[0] == "dielectric":
                d.ior = m[1]
            if m[0] == "emissive":
                d.emission[:] = m[1]
        self.triangles = np.zeros((max(1, len(tris)), 12), dtype=np.float64)
        for i, t in enumerate(tris):
            self.triangles[i] = (*t[0], *t[1], *t[2], *t[3])
        self.num_objects, self.num_materials, self.num_triangles = len(objs), len(mats), len(tris)
        self.kinds = [k for k, _, _ in world.objects]
        self.desc = capi.SceneDesc()
        d = self.desc
        d.abi_version = capi.RT_ABI_VERSION
        d.num_objects = self.num_objects
        d.objects = self.objects
        d.num_materials = self.num_materials
        d.num_triangles = self.num_triangles
        d.materials = self.materials
        d.triangles = self.triangles.ctypes.data_as(C.POINTER(C.c_double))
        d.camera = camera.desc()
        d.background = world.background
        d.sky_intensity = world.sky_intensity
        d.solid_color[:] = world.solid_color
        d.perm[:] = world.perm

    def record_bytes_per_segment(self):
        """Σ canonical record bytes over every primitive one world.hit call tests."""
        total = 0
        for k, o in zip(self.kinds, self.objects):
            total += RECORD_BYTES["triangle"] * o.count if k in ("mesh", "triangle") else RECORD_BYTES[k]
        return total

    def primitives_per_segment(self):
        return sum(o.count if k in ("mesh", "triangle") else 1 for k, o in zip(self.kinds, self.objects))


def scene_path(name):
    p = name if os.path.isabs(name) else os.path.join(SCENES_DIR, name if name.endswith(".json") else name + ".json")
    return p


def load_scene_json(name):
    """Scene JSON by file name under scenes/ (mesh50k is generated on demand)."""
    p = scene_path(name)
    if os.path.basename(p) == "mesh50k.json" and (not os.path.exists(p) or os.path.getsize(p) == 0):
        import importlib.util
        spec = importlib.util.spec_from_file_location("scenes_generate", os.path.join(SCENES_DIR, "generate.py"))
        gen = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(gen)
        return gen.mesh50k()
    with open(p) as f:
        return json.load(f)


def keyed_permutation(seed):
    return permutation(seed)
