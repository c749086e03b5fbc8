"""tri_exit_bound (blenderraytracer_amd/csrc/pt_core.h leaves_tri_hull, scene_pack.h build_tri_exit): a ray
leaving the triangle it just hit, away from every triangle of the scene, skips the next segment's triangle
walk.  The skip must never drop a triangle the reference's binary64 test (geometry.js:148-188) would accept.

tests/hostcheck/tri_exit_check.cpp makes rays hit a triangle through the binary64 test (the point as
hit_record computes it), leaves it at angles from steep down to 1e-14 (grazing) on either side, and tests
every triangle of the mesh whenever the check says "skip".  The GPU side — images of skipping kernels
bit-identical to the brute-force World-order kernel and to the reference's goldens — is
tests/test_gpu_parity.py (test_bvh_bit_identical_to_brute_mesh50k, the mesh goldens).
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "hostcheck", "tri_exit_check.cpp")
DEPS = [SRC] + [os.path.join(ROOT, "blenderraytracer_amd", "csrc", f) for f in ("pt_core.h", "pt_path.h", "scene_pack.h")]
BIN = os.path.join(HERE, "hostcheck", "_build", "tri_exit_check")


@pytest.fixture(scope="module")
def checker():
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    if not os.path.exists(BIN) or any(os.path.getmtime(BIN) < os.path.getmtime(p) for p in DEPS):
        tmp = "%s.tmp%d" % (BIN, os.getpid())    # parallel test workers: build aside, rename atomically
        hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
        subprocess.check_call([hipcc, "--offload-host-only", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread",
                               "-I", os.path.join(ROOT, "include"), SRC, "-o", tmp])
        os.replace(tmp, BIN)
    return BIN


def run(binary, mesh, rays, seed, mutation=0):
    out = subprocess.run([binary, mesh, str(rays), str(seed), str(mutation)], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    return {k: int(v) for k, v in re.findall(r"(\w+)=(\d+)", out)}


@pytest.mark.parametrize("mesh,rays", [("sphere", 6000), ("sphere_off", 6000), ("cube", 20000), ("torus", 20000),
                                       ("bowl", 8000), ("grid", 20000), ("pair", 8000)])
def test_skipped_segments_hit_no_triangle(checker, mesh, rays):
    r = run(checker, mesh, rays, 7)
    assert r["rays"] == rays
    assert r["violations"] == 0, r
    assert r["skips"] > rays // 20, r          # the check does let exits skip


def test_convex_mesh_every_face_is_an_exit_face(checker):
    """config 5's UV sphere: every face with a unit normal gets a finite bound on its outer side (the pole
    rows' zero-area triangles have none)."""
    r = run(checker, "sphere", 0, 1)
    assert r["exit_faces"] >= 49984 - 2 * 176


@pytest.mark.parametrize("mesh,mutation", [("torus", 1), ("bowl", 1), ("sphere_off", 1), ("sphere_off", 2), ("pair", 1)])
def test_checker_catches_wrong_bounds(checker, mesh, mutation):
    """Mutations: C from the face's own vertices only (1), the two sides' bounds swapped (2) — both skip
    segments that do hit a triangle, and the checker sees it."""
    r = run(checker, mesh, 4000, 3, mutation)
    assert r["violations"] > 0, r
