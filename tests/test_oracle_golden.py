"""The CPU oracle (oracle/pt_oracle.c) against fixtures produced by the REAL reference renderer
(oracle/ref_harness/run_reference.mjs running /root/reference/js under Node with the keyed RNG).

This pins the oracle: per-pixel linear means, post-gamma values, RGBA8 bytes, world.hit segment
counts and RNG draw counts.  Bit-exact except where V8's fdlibm pow/exp and glibc's differ in the
last ulp (procedural-sky background): there the tolerance is 4 ulp of the value."""
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
    tol = 4 * np.spacing(np.abs(lin[ok]))
    assert np.all(np.abs(r["mean"][ok] - lin[ok]) <= tol), "linear mean differs from the reference"
    okp = ~np.isnan(post)
    assert np.all(np.abs(r["post"][okp] - post[okp]) <= 4 * np.spacing(np.abs(post[okp])) + 1e-300)
    assert np.array_equal(r["rgba8"], gc.load_array(case, "rgba8"))     # denoised when the case denoises
    if gc.has(case, "denoised"):
        dn = gc.load_array(case, "denoised")
        assert np.all(np.abs(r["denoised"] - dn) <= np.spacing(np.abs(dn))), "PostProcessor.denoise differs"
    assert np.array_equal(r["segments"], gc.load_array(case, "segs")), "world.hit counts differ"
    assert np.array_equal(r["draws"], gc.load_array(case, "draws")), "Math.random draw counts differ"


def test_fixtures_are_mostly_bit_exact():
    """Across all fixtures, >99.9% of linear-mean channels are bitwise identical to the reference."""
    same = total = 0
    for case in gc.case_names(heavy=False):
        rt, c = gc.tracer_for(case)
        r = binding.render(rt.packed(), rt.settings(crop=c["crop"]))
        lin = gc.load_array(case, "linear")
        eq = (r["mean"] == lin) | (np.isnan(lin) & np.isnan(r["mean"]))
        same += int(eq.sum())
        total += eq.size
    assert same / total > 0.999


def test_nan_bug_is_reproduced():
    """JSON 'solid' backgrounds render NaN in the reference (stored as 0 in RGBA8)."""
    lin = gc.load_array("json_solid_nan_bug", "linear")
    assert np.isnan(lin).mean() > 0.5
    rgba = gc.load_array("json_solid_nan_bug", "rgba8")
    assert np.all(rgba[np.isnan(lin[..., 0])][:, 0] == 0)
