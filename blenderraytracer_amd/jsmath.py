"""JavaScript's Math functions as the reference's V8 (Node 12) computes them, for the Python host.

The host evaluates a few values the reference computes in JS before the render: the denoise weights
(`Math.exp`, post-processor.js:60) and the camera's `Math.tan(theta / 2)` (camera.js:15).  V8's
Math.exp and Math.tan are fdlibm's e_exp.c and s_tan.c / k_tan.c / e_rem_pio2.c, restated here in
binary64 Python floats (IEEE round-to-nearest, the same operations in the same order) — equal to Node's
Math.exp / Math.tan bit for bit (tests/test_js_host.py::test_js_math_vs_v8), where glibc's (math.exp,
math.tan) differ in the last bit on a few percent of arguments.  The kernel's own copy is
csrc/js_math.h.
"""
import struct

_u = struct.Struct("<Q")
_d = struct.Struct("<d")


def _bits(hi, lo):
    return _d.unpack(_u.pack((hi << 32) | lo))[0]


def _hi(x):
    return _u.unpack(_d.pack(x))[0] >> 32


def _lo(x):
    return _u.unpack(_d.pack(x))[0] & 0xFFFFFFFF


def _with_hi(x, h):
    return _d.unpack(_u.pack(((h & 0xFFFFFFFF) << 32) | _lo(x)))[0]


_HUGE = 1.0e300
_TWOM1000 = _bits(0x01700000, 0)
_O_THRESHOLD = _bits(0x40862E42, 0xFEFA39EF)
_U_THRESHOLD = _bits(0xC0874910, 0xD52D3051)
_LN2HI = _bits(0x3FE62E42, 0xFEE00000)
_LN2LO = _bits(0x3DEA39EF, 0x35793C76)
_INVLN2 = _bits(0x3FF71547, 0x652B82FE)
_P1 = _bits(0x3FC55555, 0x5555553E)
_P2 = _bits(0xBF66C16C, 0x16BEBD93)
_P3 = _bits(0x3F11566A, 0xAF25DE2C)
_P4 = _bits(0xBEBBBD41, 0xC5D26BF1)
_P5 = _bits(0x3E663769, 0x72BEA4D0)


def js_exp(x):
    """Math.exp(x) as V8 7.8 computes it (fdlibm e_exp.c)."""
    x = float(x)
    hx = _hi(x)
    xsb = (hx >> 31) & 1
    hx &= 0x7FFFFFFF
    hi = lo = 0.0
    k = 0
    if hx >= 0x40862E42:                                   # |x| >= 709.78...
        if hx >= 0x7FF00000:
            if ((hx & 0xFFFFF) | _lo(x)) != 0:
                return x + x                               # NaN
            return x if xsb == 0 else 0.0                  # exp(+-inf) = inf, 0
        if x > _O_THRESHOLD:
            return _HUGE * _HUGE
        if x < _U_THRESHOLD:
            return _TWOM1000 * _TWOM1000
    if hx > 0x3FD62E42:                                    # |x| > 0.5 ln2
        if hx < 0x3FF0A2B2:                                # and < 1.5 ln2
            hi = x + _LN2HI if xsb else x - _LN2HI
            lo = -_LN2LO if xsb else _LN2LO
            k = 1 - xsb - xsb
        else:
            k = int(_INVLN2 * x + (-0.5 if xsb else 0.5))  # C's (int) truncates toward zero
            t = float(k)
            hi = x - t * _LN2HI
            lo = t * _LN2LO
        x = hi - lo
    elif hx < 0x3E300000:                                  # |x| < 2^-28
        if _HUGE + x > 1.0:
            return 1.0 + x
    else:
        k = 0
    t = x * x
    c = x - t * (_P1 + t * (_P2 + t * (_P3 + t * (_P4 + t * _P5))))
    if k == 0:
        return 1.0 - ((x * c) / (c - 2.0) - x)
    y = 1.0 - ((lo - (x * c) / (2.0 - c)) - hi)
    if k >= -1021:
        return _with_hi(y, _hi(y) + (k << 20))
    return _with_hi(y, _hi(y) + ((k + 1000) << 20)) * _TWOM1000


# ---- Math.tan (fdlibm s_tan.c, k_tan.c, e_rem_pio2.c for |x| <= 2^19 pi/2): the camera's tan(fov / 2),
# camera.js:15 ----------------------------------------------------------------------------------------

def _with_lo(x, lo):
    return _d.unpack(_u.pack((_u.unpack(_d.pack(x))[0] & 0xFFFFFFFF00000000) | lo))[0]


def _s32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


_T = [_bits(0x3FD55555, 0x55555563), _bits(0x3FC11111, 0x1110FE7A), _bits(0x3FABA1BA, 0x1BB341FE),
      _bits(0x3F9664F4, 0x8406D637), _bits(0x3F8226E3, 0xE96E8493), _bits(0x3F6D6D22, 0xC9560328),
      _bits(0x3F57DBC8, 0xFEE08315), _bits(0x3F4344D8, 0xF2F26501), _bits(0x3F3026F7, 0x1A8D1068),
      _bits(0x3F147E88, 0xA03792A6), _bits(0x3F12B80F, 0x32F0A7E9), _bits(0xBEF375CB, 0xDB605373),
      _bits(0x3EFB2A70, 0x74BF7AD4)]
_PIO4 = _bits(0x3FE921FB, 0x54442D18)
_PIO4LO = _bits(0x3C81A626, 0x33145C07)
_INVPIO2 = _bits(0x3FE45F30, 0x6DC9C883)
_PIO2 = [(_bits(0x3FF921FB, 0x54400000), _bits(0x3DD0B461, 0x1A626331)),
         (_bits(0x3DD0B461, 0x1A600000), _bits(0x3BA3198A, 0x2E037073)),
         (_bits(0x3BA3198A, 0x2E000000), _bits(0x397B839A, 0x252049C1))]
_NPIO2_HW = [0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C, 0x4025FDBB, 0x402921FB,
             0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C, 0x40346B9C, 0x4035FDBB, 0x40378FDB, 0x403921FB,
             0x403AB41B, 0x403C463A, 0x403DD85A, 0x403F6A7A, 0x40407E4C, 0x4041475C, 0x4042106C, 0x4042D97C,
             0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB, 0x4046C6CB, 0x40478FDB, 0x404858EB, 0x404921FB]


def _c_int(v):
    """C's (int) conversion of a finite double: truncation toward zero."""
    return int(v)


def _k_tan(x, y, iy):
    hx = _s32(_hi(x))
    ix = hx & 0x7FFFFFFF
    if ix < 0x3E300000 and _c_int(x) == 0:                 # |x| < 2^-28
        if ((ix | _lo(x)) | (iy + 1)) == 0:
            return 1.0 / abs(x)
        if iy == 1:
            return x
        w = x + y
        z = _with_lo(w, 0)
        v = y - (z - x)
        a = -1.0 / w
        t = _with_lo(a, 0)
        s = 1.0 + t * z
        return t + a * (s + t * v)
    if ix >= 0x3FE59428:                                   # |x| >= 0.6744
        if hx < 0:
            x, y = -x, -y
        z = _PIO4 - x
        w = _PIO4LO - y
        x = z + w
        y = 0.0
    z = x * x
    w = z * z
    T = _T
    r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))))
    v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))))
    s = z * x
    r = y + z * (s * (r + v) + y)
    r += T[0] * s
    w = x + r
    if ix >= 0x3FE59428:
        v = float(iy)
        return float(1 - ((hx >> 30) & 2)) * (v - 2.0 * (x - (w * w / (w + v) - r)))
    if iy == 1:
        return w
    z = _with_lo(w, 0)
    v = r - (z - x)
    a = -1.0 / w
    t = _with_lo(a, 0)
    s = 1.0 + t * z
    return t + a * (s + t * v)


def _rem_pio2(x):
    """(n, y0, y1) with x = n pi/2 + y0 + y1, or None beyond 2^19 pi/2 (fdlibm e_rem_pio2.c)."""
    hx = _s32(_hi(x))
    ix = hx & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return 0, x, 0.0
    p1, p1t = _PIO2[0]
    p2, p2t = _PIO2[1]
    if ix < 0x4002D97C:                                    # |x| < 3 pi / 4
        if hx > 0:
            z = x - p1
            if ix != 0x3FF921FB:
                y0 = z - p1t
                return 1, y0, (z - y0) - p1t
            z -= p2
            y0 = z - p2t
            return 1, y0, (z - y0) - p2t
        z = x + p1
        if ix != 0x3FF921FB:
            y0 = z + p1t
            return -1, y0, (z - y0) + p1t
        z += p2
        y0 = z + p2t
        return -1, y0, (z - y0) + p2t
    if ix > 0x413921FB:
        return None
    t = abs(x)
    n = _c_int(t * _INVPIO2 + 0.5)
    fn = float(n)
    r = t - fn * p1
    w = fn * p1t
    y0 = r - w
    if not (n < 32 and ix != _NPIO2_HW[n - 1]):
        j = ix >> 20
        i = j - ((_hi(y0) >> 20) & 0x7FF)
        if i > 16:
            t = r
            w = fn * p2
            r = t - w
            w = fn * p2t - ((t - r) - w)
            y0 = r - w
            i = j - ((_hi(y0) >> 20) & 0x7FF)
            if i > 49:
                p3, p3t = _PIO2[2]
                t = r
                w = fn * p3
                r = t - w
                w = fn * p3t - ((t - r) - w)
                y0 = r - w
    y1 = (r - y0) - w
    if hx < 0:
        return -n, -y0, -y1
    return n, y0, y1


def js_tan(x):
    """Math.tan(x) as V8 7.8 computes it (fdlibm s_tan.c); beyond 2^19 pi/2 the platform's tan."""
    import math
    x = float(x)
    ix = _hi(x) & 0x7FFFFFFF
    if ix <= 0x3FE921FB:
        return _k_tan(x, 0.0, 1)
    if ix >= 0x7FF00000:
        return x - x
    red = _rem_pio2(x)
    if red is None:
        return math.tan(x)
    n, y0, y1 = red
    return _k_tan(y0, y1, 1 - ((n & 1) << 1))
