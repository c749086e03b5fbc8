// JavaScript's Math.pow and Math.exp as the reference's own runtime computes them, for host and device.
//
// The reference's materials.js:82 (`Math.pow(1 - cosine, 5)`, Schlick), world.js:46-72 (the procedural
// sky's `Math.pow(sd, 512)`, `Math.pow(corona, 2)`) and post-processor.js (`Math.pow(c, 1 / gamma)`)
// run on Node 12's V8 (7.8), whose Math.pow is v8::base::ieee754::pow: fdlibm's e_pow.c (Sun
// Microsystems, the published algorithm restated below) with one change in its final step — V8
// divides z·t1 by ((t1 − 2) − (w + z·w)) where fdlibm computes z·t1 / (t1 − 2) − (w + z·w).  With that
// change this restatement equals Node's Math.pow bit for bit (tests/test_js_host.py::test_js_pow_vs_v8:
// millions of arguments over the reference's uses plus special values); fdlibm's own final step
// differs on 4.5 % of x^5 arguments, and the correctly rounded power on 9.6 %.
//
// Math.exp is v8::base::ieee754::exp, fdlibm's e_exp.c unchanged (restated below; equal to Node's
// Math.exp bit for bit, same test): the procedural sky's horizon glow (world.js:60) and the denoise
// weights (post-processor.js:60).  Math.sin / Math.cos / Math.tan are fdlibm's s_sin.c / s_cos.c /
// s_tan.c with their kernels and e_rem_pio2.c's reduction for |x| <= 2^19 pi/2 (the stochastic AA's
// cos / sin of 2 pi r, ray-tracer.js:130-131; the camera's tan(fov / 2), camera.js:15); beyond that
// the platform's own function (not bit-pinned; never on the path).
//
// Plain binary64 arithmetic only (no FMA contraction: the library builds with -ffp-contract=off), so the
// device and the host compute the same bits.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef RT_JS_HD
#if defined(__HIPCC__)
#define RT_JS_HD __host__ __device__ inline
#else
#define RT_JS_HD inline
#endif
#endif

namespace jsm {

RT_JS_HD int hi(double x) { uint64_t b; memcpy(&b, &x, 8); return (int)(b >> 32); }
RT_JS_HD uint32_t lo(double x) { uint64_t b; memcpy(&b, &x, 8); return (uint32_t)b; }
RT_JS_HD double with_lo(double x, uint32_t l) {
    uint64_t b; memcpy(&b, &x, 8); b = (b & 0xffffffff00000000ULL) | l; memcpy(&x, &b, 8); return x;
}
RT_JS_HD double with_hi(double x, int h) {
    uint64_t b; memcpy(&b, &x, 8); b = (b & 0xffffffffULL) | ((uint64_t)(uint32_t)h << 32); memcpy(&x, &b, 8); return x;
}
RT_JS_HD double bits(uint32_t h, uint32_t l) { const uint64_t b = ((uint64_t)h << 32) | l; double d; memcpy(&d, &b, 8); return d; }

// x^y (ECMAScript Math.pow on V8 7.8)
RT_JS_HD double pow(double x, double y) {
    const double one = 1.0, two = 2.0, zero = 0.0, two53 = bits(0x43400000, 0);
    const double huge = 1.0e300, tiny = 1.0e-300;
    const double L1 = bits(0x3FE33333, 0x33333303), L2 = bits(0x3FDB6DB6, 0xDB6FABFF), L3 = bits(0x3FD55555, 0x518F264D),
                 L4 = bits(0x3FD17460, 0xA91D4101), L5 = bits(0x3FCD864A, 0x93C9DB65), L6 = bits(0x3FCA7E28, 0x4A454EEF);
    const double P1 = bits(0x3FC55555, 0x5555553E), P2 = bits(0xBF66C16C, 0x16BEBD93), P3 = bits(0x3F11566A, 0xAF25DE2C),
                 P4 = bits(0xBEBBBD41, 0xC5D26BF1), P5 = bits(0x3E663769, 0x72BEA4D0);
    const double lg2 = bits(0x3FE62E42, 0xFEFA39EF), lg2_h = bits(0x3FE62E43, 0), lg2_l = bits(0xBE205C61, 0x0CA86C39);
    const double ovt = 8.0085662595372944372e-17;
    const double cp = bits(0x3FEEC709, 0xDC3A03FD), cp_h = bits(0x3FEEC709, 0xE0000000), cp_l = bits(0xBE3E2FE0, 0x145B01F5);
    const double ivln2 = bits(0x3FF71547, 0x652B82FE), ivln2_h = bits(0x3FF71547, 0x60000000),
                 ivln2_l = bits(0x3E54AE0B, 0xF85DDF44);
    const double dp_h1 = bits(0x3FE2B803, 0x40000000), dp_l1 = bits(0x3E4CFDEB, 0x43CFD006);

    const int hx = hi(x), hy = hi(y);
    const uint32_t lx = lo(x), ly = lo(y);
    int ix = hx & 0x7fffffff;
    const int iy = hy & 0x7fffffff;

    if ((iy | ly) == 0) return one;                                           // x^0 = 1
    if (ix > 0x7ff00000 || (ix == 0x7ff00000 && lx != 0) || iy > 0x7ff00000 || (iy == 0x7ff00000 && ly != 0))
        return x + y;                                                         // NaN
    // yisint: 0 y not an integer, 1 odd, 2 even (only needed for x < 0)
    int yisint = 0;
    if (hx < 0) {
        if (iy >= 0x43400000) yisint = 2;
        else if (iy >= 0x3ff00000) {
            const int k = (iy >> 20) - 0x3ff;
            if (k > 20) {
                const uint32_t j = ly >> (52 - k);
                if ((j << (52 - k)) == ly) yisint = 2 - (int)(j & 1);
            } else if (ly == 0) {
                const int j = iy >> (20 - k);
                if ((j << (20 - k)) == iy) yisint = 2 - (j & 1);
            }
        }
    }
    if (ly == 0) {                                                            // special y
        if (iy == 0x7ff00000) {                                               // +-inf
            if (((ix - 0x3ff00000) | (int)lx) == 0) return y - y;             // (+-1)^+-inf = NaN
            else if (ix >= 0x3ff00000) return hy >= 0 ? y : zero;
            else return hy < 0 ? -y : zero;
        }
        if (iy == 0x3ff00000) return hy < 0 ? one / x : x;                    // +-1
        if (hy == 0x40000000) return x * x;                                   // 2
        if (hy == 0x3fe00000 && hx >= 0) return sqrt(x);                      // 0.5
    }
    double ax = fabs(x);
    if (lx == 0 && (ix == 0x7ff00000 || ix == 0 || ix == 0x3ff00000)) {       // x = +-0, +-inf, +-1
        double z = ax;
        if (hy < 0) z = one / z;
        if (hx < 0) {
            if (((ix - 0x3ff00000) | yisint) == 0) z = (z - z) / (z - z);     // (-1)^non-int
            else if (yisint == 1) z = -z;
        }
        return z;
    }
    int n = (int)((uint32_t)hx >> 31) ^ 1;                                    // (hx >> 31) + 1: 1 for x > 0
    if ((n | yisint) == 0) return (x - x) / (x - x);                          // (x < 0)^non-int
    double s = one;
    if ((n | (yisint - 1)) == 0) s = -one;                                    // (x < 0)^odd

    double t1, t2;
    if (iy > 0x41e00000) {                                                    // |y| > 2^31
        if (iy > 0x43f00000) {                                                // |y| > 2^64: over/underflow
            if (ix <= 0x3fefffff) return hy < 0 ? huge * huge : tiny * tiny;
            if (ix >= 0x3ff00000) return hy > 0 ? huge * huge : tiny * tiny;
        }
        if (ix < 0x3fefffff) return hy < 0 ? s * huge * huge : s * tiny * tiny;
        if (ix > 0x3ff00000) return hy > 0 ? s * huge * huge : s * tiny * tiny;
        // |1 - x| <= 2^-20: log(x) by x - x^2/2 + x^3/3 - x^4/4
        const double t = ax - one;
        const double w = (t * t) * (0.5 - t * (0.3333333333333333333333 - t * 0.25));
        const double u = ivln2_h * t;
        const double v = t * ivln2_l - w * ivln2;
        t1 = with_lo(u + v, 0);
        t2 = v - (t1 - u);
    } else {
        n = 0;
        if (ix < 0x00100000) {                                                // subnormal x
            ax *= two53;
            n -= 53;
            ix = hi(ax);
        }
        n += (ix >> 20) - 0x3ff;
        const int j = ix & 0x000fffff;
        int k;
        ix = j | 0x3ff00000;                                                  // normalize ix
        if (j <= 0x3988E) k = 0;                                              // |x| < sqrt(3/2)
        else if (j < 0xBB67A) k = 1;                                          // |x| < sqrt(3)
        else { k = 0; n += 1; ix -= 0x00100000; }
        ax = with_hi(ax, ix);
        const double bp = k ? 1.5 : 1.0, dp_h = k ? dp_h1 : zero, dp_l = k ? dp_l1 : zero;
        // ss = s_h + s_l = (x - 1) / (x + 1) or (x - 1.5) / (x + 1.5)
        double u = ax - bp;
        double v = one / (ax + bp);
        const double ss = u * v;
        const double s_h = with_lo(ss, 0);
        double t_h = with_hi(zero, ((ix >> 1) | 0x20000000) + 0x00080000 + (k << 18));
        double t_l = ax - (t_h - bp);
        const double s_l = v * ((u - s_h * t_h) - s_h * t_l);
        // log(ax)
        double s2 = ss * ss;
        double r = s2 * s2 * (L1 + s2 * (L2 + s2 * (L3 + s2 * (L4 + s2 * (L5 + s2 * L6)))));
        r += s_l * (s_h + ss);
        s2 = s_h * s_h;
        t_h = with_lo(3.0 + s2 + r, 0);
        t_l = r - ((t_h - 3.0) - s2);
        u = s_h * t_h;
        v = s_l * t_h + t_l * ss;
        const double p_h = with_lo(u + v, 0);
        const double p_l = v - (p_h - u);
        const double z_h = cp_h * p_h;
        const double z_l = cp_l * p_h + p_l * cp + dp_l;
        const double t = (double)n;
        t1 = with_lo(((z_h + z_l) + dp_h) + t, 0);
        t2 = z_l - (((t1 - t) - dp_h) - z_h);
    }
    // (y1 + y2) * (t1 + t2)
    const double y1 = with_lo(y, 0);
    const double p_l = (y - y1) * t1 + y * t2;
    double p_h = y1 * t1;
    double z = p_l + p_h;
    int j = hi(z);
    const int i = (int)lo(z);
    if (j >= 0x40900000) {                                                    // z >= 1024
        if (((j - 0x40900000) | i) != 0) return s * huge * huge;
        if (p_l + ovt > z - p_h) return s * huge * huge;
    } else if ((j & 0x7fffffff) >= 0x4090cc00) {                              // z <= -1075
        if ((((uint32_t)j - 0xc090cc00u) | (uint32_t)i) != 0) return s * tiny * tiny;
        if (p_l <= z - p_h) return s * tiny * tiny;
    }
    // 2^(p_h + p_l)
    const int ii = j & 0x7fffffff;
    int k = (ii >> 20) - 0x3ff;
    n = 0;
    if (ii > 0x3fe00000) {                                                    // |z| > 0.5: n = [z + 0.5]
        n = j + (0x00100000 >> (k + 1));
        k = ((n & 0x7fffffff) >> 20) - 0x3ff;
        const double t = with_hi(zero, n & ~(0x000fffff >> k));
        n = ((n & 0x000fffff) | 0x00100000) >> (20 - k);
        if (j < 0) n = -n;
        p_h -= t;
    }
    const double t = with_lo(p_l + p_h, 0);
    const double u = t * lg2_h;
    const double v = (p_l - (t - p_h)) * lg2 + t * lg2_l;
    z = u + v;
    const double w = v - (z - u);
    const double tt = z * z;
    const double tz = z - tt * (P1 + tt * (P2 + tt * (P3 + tt * (P4 + tt * P5))));
    const double r = (z * tz) / ((tz - two) - (w + z * w));                  // V8's final step (fdlibm: / (tz - two) - (w + z * w))
    z = one - (r - z);
    j = hi(z) + (int)((uint32_t)n << 20);
    if ((j >> 20) <= 0) z = ldexp(z, n);                                      // subnormal result
    else z = with_hi(z, hi(z) + (int)((uint32_t)n << 20));
    return s * z;
}

// e^x (ECMAScript Math.exp on V8 7.8: fdlibm's e_exp.c)
RT_JS_HD double exp(double x) {
    const double one = 1.0, huge = 1.0e300, twom1000 = bits(0x01700000, 0);
    const double o_threshold = bits(0x40862E42, 0xFEFA39EF), u_threshold = bits(0xc0874910, 0xD52D3051);
    const double ln2HI = bits(0x3fe62e42, 0xfee00000), ln2LO = bits(0x3dea39ef, 0x35793c76);
    const double invln2 = bits(0x3ff71547, 0x652b82fe);
    const double P1 = bits(0x3FC55555, 0x5555553E), P2 = bits(0xBF66C16C, 0x16BEBD93), P3 = bits(0x3F11566A, 0xAF25DE2C),
                 P4 = bits(0xBEBBBD41, 0xC5D26BF1), P5 = bits(0x3E663769, 0x72BEA4D0);
    double hi_ = 0, lo_ = 0;
    int k = 0;
    uint32_t hx = (uint32_t)hi(x);
    const int xsb = (int)((hx >> 31) & 1);
    hx &= 0x7fffffff;
    if (hx >= 0x40862E42) {                                                   // |x| >= 709.78...
        if (hx >= 0x7ff00000) {
            if (((hx & 0xfffff) | lo(x)) != 0) return x + x;                  // NaN
            return xsb == 0 ? x : 0.0;                                        // exp(+-inf) = inf, 0
        }
        if (x > o_threshold) return huge * huge;
        if (x < u_threshold) return twom1000 * twom1000;
    }
    if (hx > 0x3fd62e42) {                                                    // |x| > 0.5 ln2
        if (hx < 0x3FF0A2B2) {                                                // and < 1.5 ln2
            hi_ = xsb ? x + ln2HI : x - ln2HI;
            lo_ = xsb ? -ln2LO : ln2LO;
            k = 1 - xsb - xsb;
        } else {
            k = (int)(invln2 * x + (xsb ? -0.5 : 0.5));
            const double t = k;
            hi_ = x - t * ln2HI;
            lo_ = t * ln2LO;
        }
        x = hi_ - lo_;
    } else if (hx < 0x3e300000) {                                             // |x| < 2^-28
        if (huge + x > one) return one + x;
    } else {
        k = 0;
    }
    const double t = x * x;
    const double c = x - t * (P1 + t * (P2 + t * (P3 + t * (P4 + t * P5))));
    if (k == 0) return one - ((x * c) / (c - 2.0) - x);
    const double y = one - ((lo_ - (x * c) / (2.0 - c)) - hi_);
    if (k >= -1021) return with_hi(y, hi(y) + (int)((uint32_t)k << 20));
    return with_hi(y, hi(y) + (int)((uint32_t)(k + 1000) << 20)) * twom1000;
}

// fdlibm k_sin.c / k_cos.c / k_tan.c on [-pi/4, pi/4] (x + y the reduced argument)
RT_JS_HD double k_sin(double x, double y, int iy) {
    const double S1 = bits(0xBFC55555, 0x55555549), S2 = bits(0x3F811111, 0x1110F8A6), S3 = bits(0xBF2A01A0, 0x19C161D5),
                 S4 = bits(0x3EC71DE3, 0x57B1FE7D), S5 = bits(0xBE5AE5E6, 0x8A2B9CEB), S6 = bits(0x3DE5D93A, 0x5ACFD57C);
    const int ix = hi(x) & 0x7fffffff;
    if (ix < 0x3e400000 && (int)x == 0) return x;                            // |x| < 2^-27
    const double z = x * x, v = z * x;
    const double r = S2 + z * (S3 + z * (S4 + z * (S5 + z * S6)));
    if (iy == 0) return x + v * (S1 + z * r);
    return x - ((z * (0.5 * y - v * r) - y) - v * S1);
}
RT_JS_HD double k_cos(double x, double y) {
    const double C1 = bits(0x3FA55555, 0x5555554C), C2 = bits(0xBF56C16C, 0x16C15177), C3 = bits(0x3EFA01A0, 0x19CB1590),
                 C4 = bits(0xBE927E4F, 0x809C52AD), C5 = bits(0x3E21EE9E, 0xBDB4B1C4), C6 = bits(0xBDA8FAE9, 0xBE8838D4);
    const int ix = hi(x) & 0x7fffffff;
    if (ix < 0x3e400000 && (int)x == 0) return 1.0;                          // |x| < 2^-27
    const double z = x * x;
    const double r = z * (C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6)))));
    if (ix < 0x3FD33333) return 1.0 - (0.5 * z - (z * r - x * y));           // |x| < 0.3
    const double qx = ix > 0x3fe90000 ? 0.28125 : with_hi(0.0, ix - 0x00200000);   // x / 4
    const double hz = 0.5 * z - qx, a = 1.0 - qx;
    return a - (hz - (z * r - x * y));
}
RT_JS_HD double k_tan(double x, double y, int iy) {
    const double T[13] = {bits(0x3FD55555, 0x55555563), bits(0x3FC11111, 0x1110FE7A), bits(0x3FABA1BA, 0x1BB341FE),
                          bits(0x3F9664F4, 0x8406D637), bits(0x3F8226E3, 0xE96E8493), bits(0x3F6D6D22, 0xC9560328),
                          bits(0x3F57DBC8, 0xFEE08315), bits(0x3F4344D8, 0xF2F26501), bits(0x3F3026F7, 0x1A8D1068),
                          bits(0x3F147E88, 0xA03792A6), bits(0x3F12B80F, 0x32F0A7E9), bits(0xBEF375CB, 0xDB605373),
                          bits(0x3EFB2A70, 0x74BF7AD4)};
    const double pio4 = bits(0x3FE921FB, 0x54442D18), pio4lo = bits(0x3C81A626, 0x33145C07);
    double z, r, v, w, s;
    const int hx = hi(x), ix = hx & 0x7fffffff;
    if (ix < 0x3e300000 && (int)x == 0) {                                    // |x| < 2^-28
        if (((ix | (int)lo(x)) | (iy + 1)) == 0) return 1.0 / fabs(x);
        if (iy == 1) return x;
        w = x + y;
        z = with_lo(w, 0);
        v = y - (z - x);
        const double a = -1.0 / w, t = with_lo(a, 0);
        s = 1.0 + t * z;
        return t + a * (s + t * v);
    }
    if (ix >= 0x3FE59428) {                                                   // |x| >= 0.6744
        if (hx < 0) { x = -x; y = -y; }
        z = pio4 - x;
        w = pio4lo - y;
        x = z + w;
        y = 0.0;
    }
    z = x * x;
    w = z * z;
    r = T[1] + w * (T[3] + w * (T[5] + w * (T[7] + w * (T[9] + w * T[11]))));
    v = z * (T[2] + w * (T[4] + w * (T[6] + w * (T[8] + w * (T[10] + w * T[12])))));
    s = z * x;
    r = y + z * (s * (r + v) + y);
    r += T[0] * s;
    w = x + r;
    if (ix >= 0x3FE59428) {
        v = (double)iy;
        return (double)(1 - ((hx >> 30) & 2)) * (v - 2.0 * (x - (w * w / (w + v) - r)));
    }
    if (iy == 1) return w;
    z = with_lo(w, 0);
    v = r - (z - x);
    const double a = -1.0 / w, t = with_lo(a, 0);
    s = 1.0 + t * z;
    return t + a * (s + t * v);
}

// fdlibm e_rem_pio2.c for |x| <= 2^19 pi/2: x = n pi/2 + (y0 + y1); returns n, or INT32_MIN (|x| beyond)
RT_JS_HD int rem_pio2(double x, double& y0, double& y1) {
    const double invpio2 = bits(0x3FE45F30, 0x6DC9C883), pio2_1 = bits(0x3FF921FB, 0x54400000),
                 pio2_1t = bits(0x3DD0B461, 0x1A626331), pio2_2 = bits(0x3DD0B461, 0x1A600000),
                 pio2_2t = bits(0x3BA3198A, 0x2E037073), pio2_3 = bits(0x3BA3198A, 0x2E000000),
                 pio2_3t = bits(0x397B839A, 0x252049C1);
    const int hx = hi(x), ix = hx & 0x7fffffff;
    if (ix <= 0x3fe921fb) { y0 = x; y1 = 0; return 0; }
    if (ix < 0x4002d97c) {                                                    // |x| < 3 pi / 4: n = +-1
        if (hx > 0) {
            double z = x - pio2_1;
            if (ix != 0x3ff921fb) { y0 = z - pio2_1t; y1 = (z - y0) - pio2_1t; }
            else { z -= pio2_2; y0 = z - pio2_2t; y1 = (z - y0) - pio2_2t; }
            return 1;
        }
        double z = x + pio2_1;
        if (ix != 0x3ff921fb) { y0 = z + pio2_1t; y1 = (z - y0) + pio2_1t; }
        else { z += pio2_2; y0 = z + pio2_2t; y1 = (z - y0) + pio2_2t; }
        return -1;
    }
    if (ix > 0x413921fb) return (int)0x80000000;                              // the large-argument path
    // high words of n pi / 2, n = 1 .. 32
    const int npio2_hw[32] = {0x3FF921FB, 0x400921FB, 0x4012D97C, 0x401921FB, 0x401F6A7A, 0x4022D97C, 0x4025FDBB,
                              0x402921FB, 0x402C463A, 0x402F6A7A, 0x4031475C, 0x4032D97C, 0x40346B9C, 0x4035FDBB,
                              0x40378FDB, 0x403921FB, 0x403AB41B, 0x403C463A, 0x403DD85A, 0x403F6A7A, 0x40407E4C,
                              0x4041475C, 0x4042106C, 0x4042D97C, 0x4043A28C, 0x40446B9C, 0x404534AC, 0x4045FDBB,
                              0x4046C6CB, 0x40478FDB, 0x404858EB, 0x404921FB};
    double t = fabs(x);
    const int n = (int)(t * invpio2 + 0.5);
    const double fn = (double)n;
    double r = t - fn * pio2_1;
    double w = fn * pio2_1t;
    if (n < 32 && ix != npio2_hw[n - 1]) {
        y0 = r - w;
    } else {
        const int j = ix >> 20;
        y0 = r - w;
        int i = j - ((hi(y0) >> 20) & 0x7ff);
        if (i > 16) {                                                         // 2nd iteration
            t = r;
            w = fn * pio2_2;
            r = t - w;
            w = fn * pio2_2t - ((t - r) - w);
            y0 = r - w;
            i = j - ((hi(y0) >> 20) & 0x7ff);
            if (i > 49) {                                                     // 3rd iteration
                t = r;
                w = fn * pio2_3;
                r = t - w;
                w = fn * pio2_3t - ((t - r) - w);
                y0 = r - w;
            }
        }
    }
    y1 = (r - y0) - w;
    if (hx < 0) { y0 = -y0; y1 = -y1; return -n; }
    return n;
}

RT_JS_HD double sin(double x) {
    const int ix = hi(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_sin(x, 0.0, 0);
    if (ix >= 0x7ff00000) return x - x;
    double y0, y1;
    const int n = rem_pio2(x, y0, y1);
    if (n == (int)0x80000000) return ::sin(x);
    switch (n & 3) {
        case 0: return k_sin(y0, y1, 1);
        case 1: return k_cos(y0, y1);
        case 2: return -k_sin(y0, y1, 1);
        default: return -k_cos(y0, y1);
    }
}
RT_JS_HD double cos(double x) {
    const int ix = hi(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_cos(x, 0.0);
    if (ix >= 0x7ff00000) return x - x;
    double y0, y1;
    const int n = rem_pio2(x, y0, y1);
    if (n == (int)0x80000000) return ::cos(x);
    switch (n & 3) {
        case 0: return k_cos(y0, y1);
        case 1: return -k_sin(y0, y1, 1);
        case 2: return -k_cos(y0, y1);
        default: return k_sin(y0, y1, 1);
    }
}
RT_JS_HD double tan(double x) {
    const int ix = hi(x) & 0x7fffffff;
    if (ix <= 0x3fe921fb) return k_tan(x, 0.0, 1);
    if (ix >= 0x7ff00000) return x - x;
    double y0, y1;
    const int n = rem_pio2(x, y0, y1);
    if (n == (int)0x80000000) return ::tan(x);
    return k_tan(y0, y1, 1 - ((n & 1) << 1));
}

}  // namespace jsm
