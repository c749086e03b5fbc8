"""Deterministic generators for the benchmark / parity scenes (BASELINE.json configs 2, 3, 5).

All scenes use the reference's scene-JSON format (`/root/reference/docs/scene_format.md`,
parsed by `js/scene-loader.js:20-284`).  The generated JSON files are committed next to this
script (except the ~50k-triangle mesh, which is rebuilt on demand because it is ~2.5 MB):

  cornell.json      config 2: 5 planes + 2 spheres (Lambertian / Emissive), SURVEY §8(d)
  rtow.json         config 3/4: "Ray Tracing in One Weekend" random spheres, seed 42
  kitchen_sink.json coverage scene: boxes, single triangles, a mesh with bad indices,
                    hollow glass, coincident spheres (tie order), defaults and unknown types
  mesh50k (memory)  config 5: sample_mesh.json with the cube replaced by a 176x142 UV sphere
                    (49,984 triangles, Metal 0.8 roughness 0.1), camera aspect 16/9

Run `python scenes/generate.py` to rewrite the committed files.
"""
import copy
import json
import math
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


def cornell():
    white = {"type": "lambertian", "color": [0.73, 0.73, 0.73]}
    return {
        "name": "Cornell-style box (config 2)",
        "objects": [
            {"type": "plane", "name": "Back", "point": [0, 0, -5], "normal": [0, 0, 1], "material": white},
            {"type": "plane", "name": "Floor", "point": [0, -2.5, 0], "normal": [0, 1, 0], "material": white},
            {"type": "plane", "name": "Ceiling", "point": [0, 2.5, 0], "normal": [0, -1, 0], "material": white},
            {"type": "plane", "name": "Left", "point": [-2.5, 0, 0], "normal": [1, 0, 0],
             "material": {"type": "lambertian", "color": [0.65, 0.05, 0.05]}},
            {"type": "plane", "name": "Right", "point": [2.5, 0, 0], "normal": [-1, 0, 0],
             "material": {"type": "lambertian", "color": [0.12, 0.45, 0.15]}},
            {"type": "sphere", "name": "Light", "center": [0, 2.5, -3.0], "radius": 0.7,
             "material": {"type": "emissive", "color": [1, 1, 1], "intensity": 15}},
            {"type": "sphere", "name": "Ball", "center": [-0.6, -1.7, -3.4], "radius": 0.8, "material": white},
        ],
        "lights": [],
        "camera": {"position": [0, 0, 2], "lookAt": [0, 0, -1], "up": [0, 1, 0], "fov": 40,
                   "aspect": 1.0, "aperture": 0.0, "type": "perspective"},
        # black via intensity 0: JSON "solid" would hit the reference's NaN bug
        "background": {"type": "gradient", "intensity": 0},
    }


def rtow(seed=42):
    rng = random.Random(seed)
    objs = [{"type": "sphere", "name": "ground", "center": [0, -1000, 0], "radius": 1000,
             "material": {"type": "lambertian", "color": [0.5, 0.5, 0.5]}}]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = rng.random()
            c = [a + 0.9 * rng.random(), 0.2, b + 0.9 * rng.random()]
            if math.sqrt((c[0] - 4) ** 2 + (c[1] - 0.2) ** 2 + c[2] ** 2) <= 0.9:
                continue
            if choose < 0.8:
                col = [rng.random() * rng.random() for _ in range(3)]
                mat = {"type": "lambertian", "color": col}
            elif choose < 0.95:
                col = [0.5 + 0.5 * rng.random() for _ in range(3)]
                mat = {"type": "metal", "color": col, "roughness": 0.5 * rng.random()}
            else:
                mat = {"type": "dielectric", "ior": 1.5}
            objs.append({"type": "sphere", "center": c, "radius": 0.2, "material": mat})
    objs.append({"type": "sphere", "center": [0, 1, 0], "radius": 1.0, "material": {"type": "dielectric", "ior": 1.5}})
    objs.append({"type": "sphere", "center": [-4, 1, 0], "radius": 1.0,
                 "material": {"type": "lambertian", "color": [0.4, 0.2, 0.1]}})
    objs.append({"type": "sphere", "center": [4, 1, 0], "radius": 1.0,
                 "material": {"type": "metal", "color": [0.7, 0.6, 0.5], "roughness": 0.0}})
    return {
        "name": "RTOW random spheres (configs 3-4), seed %d" % seed,
        "objects": objs,
        "lights": [],
        "camera": {"position": [13, 2, 3], "lookAt": [0, 0, 0], "up": [0, 1, 0], "fov": 20,
                   "aspect": 16 / 9, "aperture": 0.1, "focusDist": 10.0, "type": "perspective"},
        "background": {"type": "gradient", "intensity": 1.0},
    }


def kitchen_sink():
    """Exercises every loader default and every primitive / material branch."""
    return {
        "name": "coverage scene",
        "objects": [
            {"type": "plane", "name": "floor", "point": [0, -1, 0], "normal": [0, 3, 0.2],
             "material": {"type": "lambertian", "color": [0.5, 0.55, 0.5]}},
            # two coincident spheres: World.hit keeps the FIRST (js/world.js:26, strict <)
            {"type": "sphere", "center": [-1.6, -0.4, -3], "radius": 0.6,
             "material": {"type": "lambertian", "color": [0.9, 0.1, 0.1]}},
            {"type": "sphere", "center": [-1.6, -0.4, -3], "radius": 0.6,
             "material": {"type": "lambertian", "color": [0.1, 0.9, 0.1]}},
            # hollow glass bubble: negative radius flips the normal (geometry.js:34)
            {"type": "sphere", "center": [0, -0.3, -2.2], "radius": 0.7, "material": {"type": "dielectric", "ior": 1.5}},
            {"type": "sphere", "center": [0, -0.3, -2.2], "radius": -0.6, "material": {"type": "dielectric", "ior": 1.5}},
            {"type": "sphere", "center": [1.5, -0.5, -2.6], "radius": 0.5, "material": {"type": "dielectric", "ior": 2.4}},
            # radius 0 -> 1 (scene-loader.js:101); missing material -> Lambertian 0.8
            {"type": "sphere", "center": [0.5, 1.8, -6], "radius": 0},
            {"type": "box", "min": [-0.9, -1, -4.2], "max": [-0.1, 0.2, -3.4],
             "material": {"type": "metal", "color": [0.8, 0.6, 0.2], "roughness": 0.3}},
            {"type": "box", "min": [0.6, -1, -4.4], "max": [1.4, -0.6, -3.6],
             "material": {"type": "metal", "color": [0.9, 0.9, 0.9]}},
            {"type": "box", "min": [-0.6, 2.2, -3.5], "max": [0.6, 2.25, -2.5],
             "material": {"type": "emissive", "color": [1, 0.9, 0.7], "intensity": 6}},
            {"type": "triangle", "v0": [-3, -1, -5], "v1": [-1, -1, -5.5], "v2": [-2, 1.5, -5.2],
             "material": {"type": "metal", "color": [0.7, 0.7, 0.9], "roughness": 2.5}},
            {"type": "triangle", "v0": [2.5, -1, -5], "v1": [3.5, 1, -5.5], "v2": [1.5, 1.2, -5.2],
             "material": {"type": "unobtainium"}},
            {"type": "mesh", "name": "tetra",
             "vertices": [[2.2, -1, -3.2], [3.0, -1, -3.4], [2.6, -1, -2.6], [2.6, 0.0, -3.05]],
             "indices": [0, 1, 3, 1, 2, 3, 2, 0, 3, 0, 2, 1, 0, 1, 9, 2, 3],
             "material": {"type": "lambertian", "color": [0.2, 0.4, 0.8]}},
            {"type": "mesh", "name": "no-indices", "vertices": [[0, 0, 0]]},
            {"type": "torus", "center": [0, 0, 0]},
            {"name": "typeless"},
            {"type": "sphere", "center": [-2.4, 1.4, -4], "radius": 0.35, "material": {"type": "emissive", "color": [0.4, 0.6, 1.0]}},
        ],
        "lights": [{"type": "point", "position": [0, 5, 0], "intensity": 9}, {"type": "spot"}],
        "camera": {"position": [0.3, 0.6, 2.5], "lookAt": [0, -0.2, -3], "up": [0, 1, 0], "fov": 55,
                   "aperture": 0.04, "type": "perspective"},
        "background": {"type": "gradient", "intensity": 0.8},
    }


def uv_sphere_mesh(nu=176, nv=142, radius=1.2):
    """A UV sphere with nu*nv quads = 2*nu*nv triangles (49,984 for the defaults)."""
    verts = []
    for r in range(nv + 1):
        th = math.pi * r / nv
        for s in range(nu):
            ph = 2 * math.pi * s / nu
            verts.append([radius * math.sin(th) * math.cos(ph), radius * math.cos(th), radius * math.sin(th) * math.sin(ph)])
    idx = []
    for r in range(nv):
        for s in range(nu):
            a = r * nu + s
            b = r * nu + (s + 1) % nu
            c = (r + 1) * nu + s
            d = (r + 1) * nu + (s + 1) % nu
            idx += [a, c, b, b, c, d]
    return verts, idx


def mesh50k(sample_mesh_path=os.path.join(HERE, "sample_mesh.json")):
    with open(sample_mesh_path) as f:
        scene = json.load(f)
    scene = copy.deepcopy(scene)
    verts, idx = uv_sphere_mesh()
    scene["name"] = "sample_mesh with a 49,984-triangle UV sphere (config 5)"
    scene["objects"][0] = {"type": "mesh", "name": "UVSphere", "vertices": verts, "indices": idx,
                           "material": {"type": "metal", "color": [0.8, 0.8, 0.8], "roughness": 0.1}}
    scene["camera"]["aspect"] = 16 / 9
    return scene


def kitchen_sink_solid_json():
    """JSON "solid" background: the reference binds a function, yielding NaN radiance."""
    s = kitchen_sink()
    s["background"] = {"type": "solid", "color": [0.2, 0.3, 0.4], "intensity": 1.0}
    return s


def kitchen_sink_ortho():
    s = kitchen_sink()
    s["camera"] = dict(s["camera"], type="orthographic", aperture=0.0, fov=70)
    return s


def kitchen_sink_resolution():
    """camera.resolution triggers resizeCanvas + setupCamera (ray-tracer.js:319-326, 439-474)."""
    s = kitchen_sink()
    s["camera"] = dict(s["camera"], resolution=[40, 28], aspect=1.2)
    return s


def close_lookat():
    """lookAt < 1 unit away is pushed 100 units out; focusDist then defaults to 100 (scene-loader.js:213-233)."""
    s = cornell()
    s["camera"] = {"position": [0, 0, 2], "lookAt": [0.1, 0.2, 1.6], "fov": 60}
    s["background"] = {"type": "gradient", "intensity": 0.3}
    return s


def empty_scene():
    return {"name": "empty", "camera": {"position": [0, 0.2, 0], "lookAt": [0, 0.5, -4], "fov": 90}}


DERIVED = {
    "kitchen_sink_solid_json": kitchen_sink_solid_json,
    "kitchen_sink_ortho": kitchen_sink_ortho,
    "kitchen_sink_resolution": kitchen_sink_resolution,
    "close_lookat": close_lookat,
    "empty_scene": empty_scene,
}


def write_all():
    items = [("cornell", cornell), ("rtow", rtow), ("kitchen_sink", kitchen_sink)] + sorted(DERIVED.items())
    for name, fn in items:
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fn(), f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    write_all()
    with open(os.path.join(HERE, "mesh50k.json"), "w") as f:  # git-ignored, rebuilt on demand
        json.dump(mesh50k(), f)
    print("spheres in rtow:", len(rtow()["objects"]))
