// Keyed counter-based RNG that replaces the reference's global Math.random()
// (js/math.js:21-31, js/materials.js:62, js/ray-tracer.js:128-140, js/noise.js:12).
//
// Draw k of sample s of pixel p under seed S:
//   seedm = lowbias32(S ^ 0x3C6EF372)
//   pkey  = lowbias32(seedm ^ p)                       p = (H-1-j)*W + i  (top-down row-major)
//   skey  = lowbias32(pkey ^ lowbias32(s + 0x1B873593))
//   u32   = lowbias32(skey ^ (k * 0x9E3779B9))
//   r     = (u32 >>> 8) * 2^-24                        in [0, 1), exact in f32 and f64
// The Perlin permutation of World (js/noise.js:6-18) is drawn from pixel = sample = 0xFFFFFFFF.
// The same definition is implemented in oracle/pt_oracle.c, blenderraytracer_amd/csrc/pt_core.h
// and blenderraytracer_amd/rng.py; every implementation must agree bit for bit.

export function lowbias32(x) {
    x = x >>> 0;
    x ^= x >>> 16;
    x = Math.imul(x, 0x7feb352d);
    x ^= x >>> 15;
    x = Math.imul(x, 0x846ca68b);
    x ^= x >>> 16;
    return x >>> 0;
}

export const PERM_STREAM = 0xFFFFFFFF;
const INV24 = 1 / 16777216;

export function seedMix(seed) { return lowbias32((seed ^ 0x3C6EF372) >>> 0); }
export function pixelKey(seedm, pixel) { return lowbias32((seedm ^ pixel) >>> 0); }
export function sampleKey(pkey, sample) { return lowbias32((pkey ^ lowbias32((sample + 0x1B873593) >>> 0)) >>> 0); }
export function drawU32(skey, k) { return lowbias32((skey ^ Math.imul(k, 0x9E3779B9)) >>> 0); }
export function draw(skey, k) { return (drawU32(skey, k) >>> 8) * INV24; }

// A stateful stream: what Math.random() becomes while one (pixel, sample) is being traced.
export class KeyedStream {
    constructor(seed) { this.seedm = seedMix(seed); this.key = 0; this.k = 0; }
    select(pixel, sample) { this.key = sampleKey(pixelKey(this.seedm, pixel >>> 0), sample >>> 0); this.k = 0; }
    next() { return draw(this.key, this.k++); }
}

// Perlin permutation p[512] exactly as js/noise.js:6-18 shuffles it, drawing from the perm stream.
export function permutation(seed) {
    const st = new KeyedStream(seed);
    st.select(PERM_STREAM, PERM_STREAM);
    const p = [];
    for (let i = 0; i < 256; i++) p[i] = i;
    for (let i = 255; i >= 0; i--) {
        const j = Math.floor(st.next() * (i + 1));
        const t = p[i]; p[i] = p[j]; p[j] = t;
    }
    for (let i = 0; i < 256; i++) p[256 + i] = p[i];
    return p;
}
