"""The JS CPU path (oracle/js/pt_cpu.mjs: the reference's per-pixel loop restated clean-room over the
packed scene arrays) against the reference's golden fixtures.  It runs on the same V8 as the
reference (same Math.pow / Math.exp / Math.sqrt), so the bar is bit-exact: every linear mean,
world.hit count and RNG draw count identical.  This is what bench.py times as the JS CPU baseline."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import golden_cases as gc
from blenderraytracer_amd.scene import load_scene_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "oracle", "js", "cpu_tool.mjs")
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


@pytest.fixture(scope="module")
def js_outputs(tmp_path_factory):
    gc.ensure_mesh50k_file()                       # generated on demand (git-ignored)
    out = tmp_path_factory.mktemp("jscpu")
    subprocess.run([NODE, TOOL, "golden", str(out), *gc.case_names(heavy=False)], check=True, timeout=900)
    return out


@pytest.mark.parametrize("case", gc.case_names(heavy=False))
def test_js_cpu_path_bit_exact(js_outputs, case):
    c = gc.manifest()["cases"][case]
    _, _, cw, ch = c["crop"]
    ld = lambda k, dt: np.fromfile(os.path.join(js_outputs, f"{case}.{k}.bin"), dtype=dt)
    ns = 1 if c["resolved"]["antiAliasing"] == "none" else c["resolved"]["samples"]
    mean = (ld("sum", np.float64) / ns).reshape(ch, cw, 3)          # color.div(sampleCount)
    assert np.array_equal(ld("segs", np.uint32).reshape(ch, cw), gc.load_array(case, "segs"))
    assert np.array_equal(ld("draws", np.uint32).reshape(ch, cw), gc.load_array(case, "draws"))
    assert np.array_equal(mean, gc.load_array(case, "linear"), equal_nan=True)


def test_js_cpu_bench_bands_match_one_thread(tmp_path):
    """cpu_tool.mjs bench: N worker_threads over row bands render exactly the samples of one thread
    (same segment count and colour checksum)."""
    scene = os.path.join(tmp_path, "rtow.json")
    with open(scene, "w") as f:
        json.dump(load_scene_json("rtow.json"), f)
    args = dict(scene=scene, width=1920, height=1080, spp=4, depth=5, seed=1, crop=[900, 500, 24, 12])
    one = json.loads(subprocess.run([NODE, TOOL, "bench", json.dumps(dict(args, workers=1))], check=True,
                                    capture_output=True, text=True, timeout=300).stdout)
    four = json.loads(subprocess.run([NODE, TOOL, "bench", json.dumps(dict(args, workers=4))], check=True,
                                     capture_output=True, text=True, timeout=300).stdout)
    assert one["workers"] == 1 and four["workers"] == 4
    assert one["samples"] == four["samples"] == 24 * 12 * 4
    assert one["segments"] == four["segments"]
    assert abs(one["checksum"] - four["checksum"]) <= 1e-9 * abs(one["checksum"])
