"""bench.py's instruction-floor model (roofline_binding.floor): the kernel's own per-lane code on the CPU
(tests/hostcheck built with -DRT_HOST_COUNTERS) counts events per segment on a few crops, and the
model prices them in VALU issue slots.  CPU-only: checks the counts are those of the walk the GPU
runs and the floor lands in a sane range."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_floor_rtow_grid():
    rt = bench.make_tracer(bench.CONFIGS["rtow"], "f64", 1, 0)
    fl = bench.instruction_floor(rt, bench.CONFIGS["rtow"], side=16, spp=4)
    ev = fl["events_per_segment"]
    assert fl["walk"] == "grid"
    assert 0.9 <= ev["walk_steps"] <= 3.0                      # cells per segment
    assert ev["filter_tests"] >= ev["f64_sphere_tests"] >= ev["disc_nonneg"] > 0
    assert abs(ev["hit"] + ev["miss"] - 1.0) < 1e-9
    assert 0.2 <= ev["samples"] <= 1.0                         # 1 / segments per sample
    assert 300 <= fl["lane_slots_per_segment"] <= 1500


def test_floor_cornell_brute_force():
    rt = bench.make_tracer(bench.CONFIGS["cornell"], "f64", 1, 0)
    fl = bench.instruction_floor(rt, bench.CONFIGS["cornell"], side=16, spp=4)
    assert fl["walk"] == "brute"
    assert fl["events_per_segment"]["plane_tests"] == 5.0
    assert fl["lane_slots_per_segment"] > 5 * bench.FLOOR_COST["plane_tests"]
