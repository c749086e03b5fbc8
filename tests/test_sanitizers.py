"""ASan + UBSan over the host-side code of the path: the C++ scene-JSON loader, the host
scene packing and BVH builder, the kernel's per-lane code compiled for the CPU and the C oracle,
built with -fsanitize=address,undefined (tests/sanitize/Makefile) and run on every scene of the
repository; the three must also agree pixel for pixel (tests/sanitize/asan_driver.cpp)."""
import glob
import os
import subprocess

import pytest

from blenderraytracer_amd.scene import load_scene_json

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")


@pytest.fixture(scope="module")
def driver():
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    subprocess.run(["make", "-s", "-j4"], cwd=SAN, check=True, timeout=900)
    return os.path.join(SAN, "_build", "asan_driver")


def test_host_code_clean_under_asan_ubsan(driver):
    load_scene_json("mesh50k")                          # generated on demand (git-ignored)
    scenes = sorted(glob.glob(os.path.join(ROOT, "scenes", "*.json")))
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([driver, *scenes], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
    assert r.stdout.count(" ok") == len(scenes)
