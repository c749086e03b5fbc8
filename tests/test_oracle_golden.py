"""The CPU oracle (oracle/pt_oracle.c) against fixtures produced by the REAL reference renderer
(oracle/ref_harness/run_reference.mjs running /root/reference/js under Node with the keyed RNG).

This pins the oracle: per-pixel linear means, post-gamma values, RGBA8 bytes, world.hit segment
counts and RNG draw counts, all bit for bit — since round 6 the oracle evaluates Math.pow / exp / sin /
cos with V8's own algorithms (oracle/pt_oracle.c v8_pow, v8_exp, v8_sincos; tests/test_js_host.py::
test_js_math_vs_v8), where glibc's differed in the last ulp (procedural sky, gamma, stochastic AA)."""
import numpy as np
import pytest

import golden_cases as gc
from oracle import binding


@pytest.mark.parametrize("case", gc.case_names())
def test_oracle_matches_reference(case):
    rt, c = gc.tracer_for(case)
    r = binding.render(rt.packed(), rt.settings(crop=c["crop"]))
    lin = gc.load_array(case, "linear")
    post = gc.load_array(case, "post")
    nan = np.isnan(lin)
    assert np.array_equal(nan, np.isnan(r["mean"])), "NaN positions differ"
    ok = ~nan
    assert np.array_equal(r["mean"][ok], lin[ok]), "linear mean differs from the reference"
    okp = ~np.isnan(post)
    assert np.array_equal(np.isnan(r["post"]), ~okp)
    assert np.array_equal(r["post"][okp], post[okp]), "post-gamma value differs from the reference"
    assert np.array_equal(r["rgba8"], gc.load_array(case, "rgba8"))     # denoised when the case denoises
    if gc.has(case, "denoised"):
        assert np.array_equal(r["denoised"], gc.load_array(case, "denoised")), "PostProcessor.denoise differs"
    assert np.array_equal(r["segments"], gc.load_array(case, "segs")), "world.hit counts differ"
    assert np.array_equal(r["draws"], gc.load_array(case, "draws")), "Math.random draw counts differ"


def test_fixtures_are_bit_exact():
    """Across all fixtures, every linear-mean channel is bitwise identical to the reference."""
    same = total = 0
    for case in gc.case_names(heavy=False):
        rt, c = gc.tracer_for(case)
        r = binding.render(rt.packed(), rt.settings(crop=c["crop"]))
        lin = gc.load_array(case, "linear")
        eq = (r["mean"] == lin) | (np.isnan(lin) & np.isnan(r["mean"]))
        same += int(eq.sum())
        total += eq.size
    assert same == total


def test_nan_bug_is_reproduced():
    """JSON 'solid' backgrounds render NaN in the reference (stored as 0 in RGBA8)."""
    lin = gc.load_array("json_solid_nan_bug", "linear")
    assert np.isnan(lin).mean() > 0.5
    rgba = gc.load_array("json_solid_nan_bug", "rgba8")
    assert np.all(rgba[np.isnan(lin[..., 0])][:, 0] == 0)
