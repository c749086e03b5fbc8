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


def _hard_f64_pairs(n, seed):
    """Binary64 (x, s) whose quotient lies within a few 2^-105 of a midpoint between two binary64 numbers
    (or of a binary64 number): with integer significands X, S in [2^52, 2^53), X 2^53 - S Q = N for a small
    N, so x / s = (Q + N / S) 2^-53 — the cases a division through a reciprocal can round the wrong way."""
    rng = np.random.default_rng(seed)
    xs, ss = [], []
    two53 = 1 << 53
    while len(xs) < n:
        S = int(rng.integers(1 << 52, 1 << 53)) | 1
        N = int(rng.choice([-3, -2, -1, 1, 2, 3]))
        X = (N * pow(two53, -1, S)) % S
        while X < (1 << 52):
            X += S
        if X >= two53:
            continue
        assert (X * two53 - N) % S == 0
        e = int(rng.integers(-60, 60))
        xs.append(np.ldexp(float(X), e - 52) * (1 if rng.random() < 0.5 else -1))
        ss.append(np.ldexp(float(S), int(rng.integers(-60, 60)) - 52))
    return np.array(xs), np.array(ss)


def test_vdiv_rcp_f64_hard_cases():
    """vdiv_rcp's binary64 division (two Markstein corrections) on near-midpoint quotients and random
    pairs: bit-identical to the IEEE division.  The single correction of round 4 is reported, not used."""
    L = hc.lib()
    L.ptc_div_rcp_f64.argtypes = [C.POINTER(C.c_double)] * 4 + [C.c_longlong]
    xh, sh = _hard_f64_pairs(60_000, 3)
    rng = np.random.default_rng(5)
    xr = rng.normal(0, 1, 200_000) * np.exp2(rng.uniform(-400, 400, 200_000))
    sr = rng.uniform(0.5, 2, 200_000) * np.exp2(rng.uniform(-300, 300, 200_000))
    x, s = np.concatenate([xh, xr]), np.concatenate([sh, sr])
    out2, out1 = np.empty_like(x), np.empty_like(x)
    p = lambda v: v.ctypes.data_as(C.POINTER(C.c_double))   # noqa: E731
    L.ptc_div_rcp_f64(p(x), p(s), p(out2), p(out1), len(x))
    ref = x / s
    assert np.array_equal(out2.view(np.uint64), ref.view(np.uint64)), int(np.count_nonzero(out2 != ref))
    print(f"single correction: {int(np.count_nonzero(out1 != ref))} of {len(x)} differ "
          f"({int(np.count_nonzero(out1[:len(xh)] != ref[:len(xh)]))} of {len(xh)} hard cases)")


def test_vdiv_rcp_f32_every_significand():
    """vdiv_rcp's binary32 division (one Markstein correction): every significand of x against 64
    all-ones-adjacent and 16 random divisor significands (671 M divisions), bit-identical to IEEE."""
    L = hc.lib()
    L.ptc_div_rcp_f32_exhaustive.argtypes = [C.c_int, C.c_uint]
    L.ptc_div_rcp_f32_exhaustive.restype = C.c_longlong
    assert L.ptc_div_rcp_f32_exhaustive(80, 99) == 0


def test_normalize_unit_guard_f32():
    """normalize<float> through vdiv_rcp_unit (one min3 + three compares as the guard, pt_core.h) equals
    three IEEE divisions by the same length, bit for bit, on 2 M vectors whose components mix zeros,
    subnormals, squares that overflow and magnitudes 2^-149 .. 2^70."""
    L = hc.lib()
    L.ptc_normalize_check.argtypes = [C.c_longlong, C.c_uint]
    L.ptc_normalize_check.restype = C.c_longlong
    assert L.ptc_normalize_check(2_000_000, 7) == 0
