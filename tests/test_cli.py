"""rt_render_cli (blenderraytracer_amd/csrc/rt_cli.cpp): the Node-free front end — scene JSON through
the C++ loader, rt_render, image out.  On the GPU its image equals the Python host's render of the
same scene and settings byte for byte."""
import json
import os
import subprocess

import numpy as np
import pytest

from blenderraytracer_amd import capi
from blenderraytracer_amd.renderer import GpuRayTracer
from blenderraytracer_amd.scene import SCENES_DIR, load_scene_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "blenderraytracer_amd", "lib", "rt_render_cli")

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="rt_render_cli not built")


def read_pam(path):
    with open(path, "rb") as f:
        data = f.read()
    head, _, body = data.partition(b"ENDHDR\n")
    fields = dict(line.split(" ", 1) for line in head.decode().splitlines()[1:])
    w, h = int(fields["WIDTH"]), int(fields["HEIGHT"])
    return np.frombuffer(body, dtype=np.uint8).reshape(h, w, 4)


def run_cli(*args):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)


def test_cli_without_device_fails_loudly():
    lib = capi.load_library()
    import ctypes as C
    n = C.c_int()
    if lib.rt_device_count(C.byref(n)) == 0 and n.value > 0:
        pytest.skip("a GPU is visible")
    r = run_cli(os.path.join(SCENES_DIR, "sample_scene.json"), "--width", "32", "--height", "32")
    assert r.returncode == 2 and "no HIP device" in r.stderr


def test_cli_rejects_bad_scene(tmp_path):
    p = tmp_path / "bad.json"
    p.write_text('{"objects": [')
    r = run_cli(str(p))
    assert r.returncode == 2 and "loading the scene" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("scene,args,settings", [
    ("sample_scene.json", ["--width", "96", "--height", "64", "--spp", "6", "--depth", "4", "--seed", "3"],
     dict(w=96, h=64, seed=3, s={"samples": 6, "maxBounces": 4})),
    ("kitchen_sink.json", ["--width", "80", "--height", "60", "--spp", "4", "--seed", "11", "--aa", "stochastic",
                           "--tone", "aces", "--precision", "f64", "--accel", "brute"],
     dict(w=80, h=60, seed=11, s={"samples": 4, "antiAliasing": "stochastic", "toneMapping": "aces"})),
    ("cornell.json", ["--width", "64", "--height", "64", "--spp", "8", "--seed", "2", "--denoise", "0.8"],
     dict(w=64, h=64, seed=2, s={"samples": 8, "denoising": True, "denoiseStrength": 0.8})),
])
def test_cli_image_matches_python_host(gpu, tmp_path, scene, args, settings):
    out = tmp_path / "img.pam"
    r = run_cli(os.path.join(SCENES_DIR, scene), *args, "--out", str(out))
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["msamples_per_s"] > 0
    img = read_pam(out)
    rt = GpuRayTracer(settings["w"], settings["h"], seed=settings["seed"])
    assert rt.load_from_json(load_scene_json(scene))
    rt.update_render_settings(settings["s"])
    ref = rt.render()["rgba8"]
    assert img.shape == ref.shape
    # denoise weights: glibc exp in both hosts -> identical bytes
    assert np.array_equal(img, ref)
    rt.close()


@pytest.mark.gpu
def test_cli_resolution_from_json(gpu, tmp_path):
    """kitchen_sink_resolution sets camera.resolution: the CLI renders at that size."""
    out = tmp_path / "img.ppm"
    r = run_cli(os.path.join(SCENES_DIR, "kitchen_sink_resolution.json"), "--spp", "1", "--out", str(out))
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    res = load_scene_json("kitchen_sink_resolution.json")["camera"]["resolution"]
    assert (line["width"], line["height"]) == tuple(res)
    assert os.path.getsize(out) > 3 * res[0] * res[1]
