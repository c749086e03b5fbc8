"""pt_core.h root_div (RT_ROOT_RCP): the sphere roots' divisions by a = d.d as a Markstein correction
from RN(1/a), run by the kernel's own code on the CPU (tests/hostcheck): bit-identical to the IEEE
division over the sphere test's ranges, and the plain division outside its guards."""
import ctypes as C

import numpy as np

from tests import hostcheck_binding as hc


def _root_div(x, a, dtype=np.float64):
    L = hc.lib(("RT_ROOT_RCP=1",))            # the Markstein path in both precisions, whatever the default
    fn, ct = (L.ptc_root_div, C.c_double) if dtype == np.float64 else (L.ptc_root_div_f32, C.c_float)
    fn.argtypes = [C.POINTER(ct)] * 3 + [C.c_longlong]
    x = np.ascontiguousarray(x, dtype=dtype)
    a = np.ascontiguousarray(a, dtype=dtype)
    out = np.empty_like(x)
    p = lambda v: v.ctypes.data_as(C.POINTER(ct))   # noqa: E731
    fn(p(x), p(a), p(out), len(x))
    return out


def test_root_div_equals_division():
    rng = np.random.default_rng(7)
    n = 2_000_000
    # a = d.d of ray directions (unit-ish, scattered: up to ~4, tiny and huge too); x = -hb -+ sqrt(disc)
    a = np.concatenate([rng.uniform(0.25, 4.0, n // 2), np.exp2(rng.uniform(-420, 420, n // 2))])
    x = np.concatenate([rng.normal(0, 10, n // 2), np.exp2(rng.uniform(-520, 520, n // 2)) * rng.choice([-1, 1], n // 2)])
    # significands next to a power of two and all-ones significands (1.111...1 x 2^k)
    edge = np.array([np.nextafter(1.0, 2.0), np.nextafter(2.0, 1.0), 1.0, 3.0, np.nextafter(4.0, 1.0)])
    a = np.concatenate([a, np.repeat(edge, 1000)])
    x = np.concatenate([x, rng.normal(0, 5, edge.size * 1000)])
    with np.errstate(all="ignore"):
        ref = x / a
    got = _root_div(x, a)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), int(np.count_nonzero(got != ref))


def test_root_div_edges():
    x = np.array([0.0, -0.0, 1e-300, 5e-324, np.inf, -np.inf, np.nan, 1.0, 1.0, 1.0])
    a = np.array([1.0, 1.0, 1.0, 3.0, 1.0, 2.0, 1.0, 0.0, np.inf, 1e-200])
    with np.errstate(all="ignore"):
        ref = x / a
    got = _root_div(x, a)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert np.array_equal(got[~np.isnan(ref)].view(np.uint64), ref[~np.isnan(ref)].view(np.uint64))


def test_root_div_equals_division_binary32():
    """The binary32 fast mode's form (RT_ROOT_RCP's default): the same Markstein correction in binary32."""
    rng = np.random.default_rng(11)
    n = 2_000_000
    a = np.concatenate([rng.uniform(0.25, 4.0, n // 2), np.exp2(rng.uniform(-45, 45, n // 2))]).astype(np.float32)
    x = np.concatenate([rng.normal(0, 10, n // 2), np.exp2(rng.uniform(-65, 65, n // 2)) * rng.choice([-1, 1], n // 2)]).astype(np.float32)
    with np.errstate(all="ignore"):
        ref = x / a
    got = _root_div(x, a, np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), int(np.count_nonzero(got != ref))
