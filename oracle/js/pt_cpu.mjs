// pt_cpu.mjs — the reference's JS CPU path, restated clean-room for Node: the per-pixel loop of
// RayTracer.render (js/ray-tracer.js:189-208) with rayColor (:102-123), World.hit (js/world.js:20-33),
// the Sphere/Plane/Box/Triangle/TriangleMesh hits (js/geometry.js:15-262), the materials
// (js/materials.js:14-96), Camera.getRay (js/camera.js:38-51), getAntiAliasSample (:125-149) and the
// backgrounds (js/world.js:35-110, js/noise.js:29-61), over the packed scene arrays of pack.mjs.
//
// TEST INFRASTRUCTURE / CPU BASELINE ONLY: tests/test_js_cpu.py checks it against the reference's
// golden fixtures (it runs on the same V8 as the reference, so every linear mean is bit-identical),
// and bench.py's cpu_baseline times it on the GPU box's host cores (oracle/js/cpu_tool.mjs bench).  The
// product never loads it.
//
// Same binary64 operations in the same order as the reference (Vec3 methods, js/math.js:6-32, inlined
// as scalar locals instead of allocated objects); rayColor's recursion is unrolled into a forward pass
// that records (emitted, attenuation) per bounce and a backward fold emitted + attenuation * inner —
// exactly the recursion's additions and products.  Math.random() is the keyed RNG (keyed-rng.mjs).

const INV24 = 1 / 16777216;
const OBJ_SPHERE = 0, OBJ_PLANE = 1, OBJ_BOX = 2, OBJ_TRIANGLE = 3, OBJ_MESH = 4;
const MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_EMISSIVE = 3;

function lowbias32(x) {
    x ^= x >>> 16; x = Math.imul(x, 0x7feb352d);
    x ^= x >>> 15; x = Math.imul(x, 0x846ca68b);
    x ^= x >>> 16;
    return x >>> 0;
}

// ---- the RNG stream of the current (pixel, sample): Math.random() of the reference ----------------
let KEY = 0, K = 0;
function rnd() {
    const h = lowbias32((KEY ^ Math.imul(K, 0x9E3779B9)) >>> 0);
    K++;
    return (h >>> 8) * INV24;
}

// Decoded scene (objects in World.objects order, materials, triangles, camera, background).
export function makeScene(p) {
    const n = p.objects.byteLength / 64;
    const ov = new DataView(p.objects.buffer, p.objects.byteOffset, p.objects.byteLength);
    const type = new Int32Array(n), mat = new Int32Array(n), first = new Int32Array(n), count = new Int32Array(n);
    const g = new Float64Array(6 * n);
    for (let i = 0; i < n; i++) {
        type[i] = ov.getInt32(64 * i, true); mat[i] = ov.getInt32(64 * i + 4, true);
        first[i] = ov.getInt32(64 * i + 8, true); count[i] = ov.getInt32(64 * i + 12, true);
        for (let k = 0; k < 6; k++) g[6 * i + k] = ov.getFloat64(64 * i + 16 + 8 * k, true);
    }
    const nm = p.materials.byteLength / 72;
    const mv = new DataView(p.materials.buffer, p.materials.byteOffset, p.materials.byteLength);
    const mtype = new Int32Array(nm), mval = new Float64Array(8 * nm);   // albedo3, rough, ior, emit3
    for (let i = 0; i < nm; i++) {
        mtype[i] = mv.getInt32(72 * i, true);
        for (let k = 0; k < 8; k++) mval[8 * i + k] = mv.getFloat64(72 * i + 8 + 8 * k, true);
    }
    return {
        n, type, mat, first, count, g, tris: Float64Array.from(p.triangles), mtype, mval,
        cam: Float64Array.from(p.camera), ortho: p.cameraType === 1, bg: p.background, sky: p.skyIntensity,
        solid: Float64Array.from(p.solidColor), perm: Int32Array.from(p.perm),
    };
}

// ---- World.hit: the winner's (t, object, triangle) in H* ---------------------------------------------
let HT = 0, HOBJ = -1, HTRI = -1;

// Triangle.hit (geometry.js:148-188) with tMax; returns t (possibly NaN, as the reference would) or
// -Infinity for a miss
function triHit(T, b, ox, oy, oz, dx, dy, dz, tMin, tMax) {
    const e1x = T[b + 3] - T[b], e1y = T[b + 4] - T[b + 1], e1z = T[b + 5] - T[b + 2];
    const e2x = T[b + 6] - T[b], e2y = T[b + 7] - T[b + 1], e2z = T[b + 8] - T[b + 2];
    const hx = dy * e2z - dz * e2y, hy = dz * e2x - dx * e2z, hz = dx * e2y - dy * e2x;
    const a = e1x * hx + e1y * hy + e1z * hz;
    if (Math.abs(a) < 0.0001) return -Infinity;
    const f = 1.0 / a;
    const sx = ox - T[b], sy = oy - T[b + 1], sz = oz - T[b + 2];
    const u = f * (sx * hx + sy * hy + sz * hz);
    if (u < 0 || u > 1) return -Infinity;
    const qx = sy * e1z - sz * e1y, qy = sz * e1x - sx * e1z, qz = sx * e1y - sy * e1x;
    const v = f * (dx * qx + dy * qy + dz * qz);
    if (v < 0 || u + v > 1) return -Infinity;
    const t = f * (e2x * qx + e2y * qy + e2z * qz);
    if (t < tMin || t > tMax) return -Infinity;
    return t;
}

function worldHit(S, ox, oy, oz, dx, dy, dz) {
    const tMin = 0.001, G = S.g, T = S.tris;
    let closest = Infinity, found = false;
    for (let i = 0; i < S.n; i++) {
        const b = 6 * i;
        let t = NaN, tri = -1;                    // NaN: no candidate (t < closest fails, as for a NaN hit)
        switch (S.type[i]) {
        case OBJ_SPHERE: {                                                     // geometry.js:15-45
            const ocx = ox - G[b], ocy = oy - G[b + 1], ocz = oz - G[b + 2], r = G[b + 3];
            const a = dx * dx + dy * dy + dz * dz;
            const hb = ocx * dx + ocy * dy + ocz * dz;
            const c = (ocx * ocx + ocy * ocy + ocz * ocz) - r * r;
            const disc = hb * hb - a * c;
            if (disc < 0) break;
            const sq = Math.sqrt(disc);
            let root = (-hb - sq) / a;
            if (root < tMin || closest < root) {
                root = (-hb + sq) / a;
                if (root < tMin || closest < root) break;
            }
            t = root;
            break;
        }
        case OBJ_PLANE: {                                                      // geometry.js:56-74
            const denom = G[b + 3] * dx + G[b + 4] * dy + G[b + 5] * dz;
            if (Math.abs(denom) < 1e-6) break;
            const tt = ((G[b] - ox) * G[b + 3] + (G[b + 1] - oy) * G[b + 4] + (G[b + 2] - oz) * G[b + 5]) / denom;
            if (tt < tMin || tt > closest) break;
            t = tt;
            break;
        }
        case OBJ_BOX: {                                                        // geometry.js:85-117
            let t0 = (G[b] - ox) / dx, t1 = (G[b + 3] - ox) / dx;
            if (t0 > t1) { const s = t0; t0 = t1; t1 = s; }
            let ty0 = (G[b + 1] - oy) / dy, ty1 = (G[b + 4] - oy) / dy;
            if (ty0 > ty1) { const s = ty0; ty0 = ty1; ty1 = s; }
            if (t0 > ty1 || ty0 > t1) break;
            t0 = Math.max(t0, ty0);
            t1 = Math.min(t1, ty1);
            let tz0 = (G[b + 2] - oz) / dz, tz1 = (G[b + 5] - oz) / dz;
            if (tz0 > tz1) { const s = tz0; tz0 = tz1; tz1 = s; }
            if (t0 > tz1 || tz0 > t1) break;
            t0 = Math.max(t0, tz0);
            t1 = Math.min(t1, tz1);
            const tt = t0 > tMin ? t0 : t1;
            if (tt < tMin || tt > closest) break;                              // NaN passes here ...
            t = tt;
            break;
        }
        case OBJ_TRIANGLE: {
            const tt = triHit(T, 12 * S.first[i], ox, oy, oz, dx, dy, dz, tMin, closest);
            if (tt !== -Infinity) { t = tt; tri = S.first[i]; }
            break;
        }
        case OBJ_MESH: {                                                       // geometry.js:248-262
            let cl = closest, any = false;
            for (let k = S.first[i], e = k + S.count[i]; k < e; k++) {
                const tt = triHit(T, 12 * k, ox, oy, oz, dx, dy, dz, tMin, cl);
                if (tt !== -Infinity) { cl = tt; tri = k; any = true; }   // the last equal-t triangle wins
            }
            if (any) t = cl;
            break;
        }
        }
        if (t < closest) {                                                     // ... and fails here
            closest = t; HT = t; HOBJ = i; HTRI = tri; found = true;
        }
    }
    return found;
}

// ---- backgrounds (world.js:35-110) into BG* ------------------------------------------------------
let BX = 0, BY = 0, BZ = 0;
function fade(t) { return t * t * t * (t * (t * 6 - 15) + 10); }
function lerp(t, a, b) { return a + t * (b - a); }
function grad(hash, x, y, z) {
    const h = hash & 15;
    const u = h < 8 ? x : y;
    const v = h < 4 ? y : (h === 12 || h === 14) ? x : z;
    return ((h & 1) === 0 ? u : -u) + ((h & 2) === 0 ? v : -v);
}
function perlin(p, x, y, z) {                                                  // noise.js:29-61
    const fx0 = Math.floor(x), fy0 = Math.floor(y), fz0 = Math.floor(z);
    const X = fx0 & 255, Y = fy0 & 255, Z = fz0 & 255;
    const fx = x - fx0, fy = y - fy0, fz = z - fz0;
    const u = fade(fx), v = fade(fy), w = fade(fz);
    const A = p[X] + Y, AA = p[A] + Z, AB = p[A + 1] + Z;
    const B = p[X + 1] + Y, BA = p[B] + Z, BB = p[B + 1] + Z;
    return lerp(w,
        lerp(v, lerp(u, grad(p[AA], fx, fy, fz), grad(p[BA], fx - 1, fy, fz)),
            lerp(u, grad(p[AB], fx, fy - 1, fz), grad(p[BB], fx - 1, fy - 1, fz))),
        lerp(v, lerp(u, grad(p[AA + 1], fx, fy, fz - 1), grad(p[BA + 1], fx - 1, fy, fz - 1)),
            lerp(u, grad(p[AB + 1], fx, fy - 1, fz - 1), grad(p[BB + 1], fx - 1, fy - 1, fz - 1))));
}
function unit(x, y, z) {   // Vec3.normalize into BX/BY/BZ
    const l = Math.sqrt(x * x + y * y + z * z);
    if (l > 0) { BX = x / l; BY = y / l; BZ = z / l; } else { BX = 0; BY = 0; BZ = 0; }
}
const SUN_P = (() => { unit(0.3, 0.6, 0.8); return [BX, BY, BZ]; })();
const SUN_H = (() => { unit(-0.3, 0.6, -0.5); return [BX, BY, BZ]; })();

function background(S, dx, dy, dz) {
    const I = S.sky;
    switch (S.bg) {
    case 0: {                                                                  // skyGradient :35-40
        unit(dx, dy, dz);
        const t = 0.5 * (BY + 1.0);
        BX = (1.0 * (1.0 - t) + 0.5 * t) * I; BY = (1.0 * (1.0 - t) + 0.7 * t) * I; BZ = (1.0 * (1.0 - t) + 1.0 * t) * I;
        return;
    }
    case 1:                                                                    // solidBackground :42-44
        BX = S.solid[0] * I; BY = S.solid[1] * I; BZ = S.solid[2] * I;
        return;
    case 2: {                                                                  // hdriBackground :74-110
        unit(dx, dy, dz);
        const x = BX, y = BY, z = BZ;
        const sd = Math.max(0, x * SUN_H[0] + y * SUN_H[1] + z * SUN_H[2]);
        const mask = sd > (1.0 - 0.04) ? 1.0 : 0.0;
        const sm = mask * 20;
        const corona = Math.max(0, (sd - (1.0 - 0.2)) / 0.2);
        const cm = Math.pow(corona, 2) * 3;
        const si = Math.max(0, y * 0.5 + 0.5) * 2;
        const gb = Math.max(0, -y * 0.3);
        const scat = Math.pow(Math.max(0, 1.0 - Math.abs(y)), 2) * 0.3;
        BX = ((((0.3 * si + 0.2 * gb) + 0.8 * scat) + 1.0 * sm) + 1.0 * cm) * I;
        BY = ((((0.5 * si + 0.15 * gb) + 0.9 * scat) + 0.95 * sm) + 0.8 * cm) * I;
        BZ = ((((0.8 * si + 0.1 * gb) + 1.0 * scat) + 0.8 * sm) + 0.6 * cm) * I;
        return;
    }
    case 3: {                                                                  // proceduralSky :46-72
        unit(dx, dy, dz);
        const x = BX, y = BY, z = BZ;
        const sd = Math.max(0, x * SUN_P[0] + y * SUN_P[1] + z * SUN_P[2]);
        const sun = Math.pow(sd, 512) * 10;
        const hb = Math.max(0, y) * 0.8;
        const glow = Math.exp(-Math.abs(y) * 4) * 0.3;
        const gnd = Math.max(0, -y * 0.5);
        const cloud = Math.max(0, perlin(S.perm, x * 10, y * 3 + 2, z * 10) * 0.8 + 0.2);
        const cl = cloud * Math.max(0, y) * 0.5;
        BX = ((((0.4 * hb + 1.0 * glow) + 0.1 * gnd) + 1.0 * sun) + 0.9 * cl) * I;
        BY = ((((0.7 * hb + 0.8 * glow) + 0.15 * gnd) + 0.95 * sun) + 0.9 * cl) * I;
        BZ = ((((1.0 * hb + 0.6 * glow) + 0.1 * gnd) + 0.8 * sun) + 1.0 * cl) * I;
        return;
    }
    default:                                                                   // JSON solid/hdri: NaN
        BX = NaN; BY = NaN; BZ = NaN;
    }
}

// ---- rayColor (ray-tracer.js:102-123) -----------------------------------------------------------------
// forward: per bounce the emitted radiance and the attenuation; backward: e + att * inner
let LX = 0, LY = 0, LZ = 0, SEGS = 0;
let STACK = new Float64Array(6 * 8);

function rayColor(S, ox, oy, oz, dx, dy, dz, depth) {
    if (STACK.length < 6 * depth) STACK = new Float64Array(6 * depth);
    const st = STACK, MV = S.mval;
    let lvl = 0, ix = 0, iy = 0, iz = 0;
    for (;;) {
        if (depth <= 0) break;                                                 // rayColor(ray, 0) = 0
        SEGS++;
        if (!worldHit(S, ox, oy, oz, dx, dy, dz)) {
            background(S, dx, dy, dz);
            ix = BX; iy = BY; iz = BZ;
            break;
        }
        const i = HOBJ, t = HT, G = S.g, b = 6 * i;
        const px = ox + dx * t, py = oy + dy * t, pz = oz + dz * t;            // ray.at(t)
        let nx, ny, nz;
        switch (S.type[i]) {
        case OBJ_SPHERE: { const r = G[b + 3]; nx = (px - G[b]) / r; ny = (py - G[b + 1]) / r; nz = (pz - G[b + 2]) / r; break; }
        case OBJ_PLANE: nx = G[b + 3]; ny = G[b + 4]; nz = G[b + 5]; break;
        case OBJ_BOX: {                                                        // geometry.js:118-126
            const eps = 1e-6;
            nx = 0; ny = 0; nz = 1;
            if (Math.abs(px - G[b]) < eps) { nx = -1; nz = 0; }
            else if (Math.abs(px - G[b + 3]) < eps) { nx = 1; nz = 0; }
            else if (Math.abs(py - G[b + 1]) < eps) { ny = -1; nz = 0; }
            else if (Math.abs(py - G[b + 4]) < eps) { ny = 1; nz = 0; }
            else if (Math.abs(pz - G[b + 2]) < eps) { nz = -1; }
            break;
        }
        default: { const q = 12 * HTRI; nx = S.tris[q + 9]; ny = S.tris[q + 10]; nz = S.tris[q + 11]; }
        }
        const front = (dx * nx + dy * ny + dz * nz) < 0;                       // setFaceNormal
        if (!front) { nx = nx * -1; ny = ny * -1; nz = nz * -1; }
        const m = S.mat[i], mt = S.mtype[m], mb = 8 * m;
        let ex = 0, ey = 0, ez = 0;
        if (mt === MAT_EMISSIVE) { ix = MV[mb + 5]; iy = MV[mb + 6]; iz = MV[mb + 7]; break; }
        let sdx, sdy, sdz, ax, ay, az;
        if (mt === MAT_LAMBERTIAN) {                                           // materials.js:20-25
            let rx, ry, rz;
            do { rx = rnd() * 2 - 1; ry = rnd() * 2 - 1; rz = rnd() * 2 - 1; } while (rx * rx + ry * ry + rz * rz >= 1.0);
            const l = Math.sqrt(rx * rx + ry * ry + rz * rz);
            if (l > 0) { rx = rx / l; ry = ry / l; rz = rz / l; } else { rx = 0; ry = 0; rz = 0; }
            sdx = nx + rx; sdy = ny + ry; sdz = nz + rz;
            ax = MV[mb]; ay = MV[mb + 1]; az = MV[mb + 2];
        } else if (mt === MAT_METAL) {                                         // materials.js:36-41
            const l = Math.sqrt(dx * dx + dy * dy + dz * dz);
            let ux = 0, uy = 0, uz = 0;
            if (l > 0) { ux = dx / l; uy = dy / l; uz = dz / l; }
            const k2 = 2 * (ux * nx + uy * ny + uz * nz);
            const fx = ux - nx * k2, fy = uy - ny * k2, fz = uz - nz * k2;
            let rx, ry, rz;
            do { rx = rnd() * 2 - 1; ry = rnd() * 2 - 1; rz = rnd() * 2 - 1; } while (rx * rx + ry * ry + rz * rz >= 1.0);
            const rough = MV[mb + 3];
            sdx = fx + rx * rough; sdy = fy + ry * rough; sdz = fz + rz * rough;
            if (!((sdx * nx + sdy * ny + sdz * nz) > 0)) { ix = ex; iy = ey; iz = ez; break; }   // absorbed
            ax = MV[mb]; ay = MV[mb + 1]; az = MV[mb + 2];
        } else {                                                               // Dielectric :51-70
            const ior = MV[mb + 4];
            const ratio = front ? (1.0 / ior) : ior;
            const l = Math.sqrt(dx * dx + dy * dy + dz * dz);
            let ux = 0, uy = 0, uz = 0;
            if (l > 0) { ux = dx / l; uy = dy / l; uz = dz / l; }
            const cosT = Math.min((ux * -1) * nx + (uy * -1) * ny + (uz * -1) * nz, 1.0);
            const sinT = Math.sqrt(1.0 - cosT * cosT);
            let reflect = ratio * sinT > 1.0;
            if (!reflect) {
                let r0 = (1 - ratio) / (1 + ratio);
                r0 = r0 * r0;
                reflect = r0 + (1 - r0) * Math.pow((1 - cosT), 5) > rnd();
            }
            if (reflect) {
                const k2 = 2 * (ux * nx + uy * ny + uz * nz);
                sdx = ux - nx * k2; sdy = uy - ny * k2; sdz = uz - nz * k2;
            } else {                                                           // refract :72-77
                const ct = Math.min((ux * -1) * nx + (uy * -1) * ny + (uz * -1) * nz, 1.0);
                const px2 = (ux + nx * ct) * ratio, py2 = (uy + ny * ct) * ratio, pz2 = (uz + nz * ct) * ratio;
                const k = -Math.sqrt(Math.abs(1.0 - (px2 * px2 + py2 * py2 + pz2 * pz2)));
                sdx = px2 + nx * k; sdy = py2 + ny * k; sdz = pz2 + nz * k;
            }
            ax = 1; ay = 1; az = 1;
        }
        const o6 = 6 * lvl++;
        st[o6] = ex; st[o6 + 1] = ey; st[o6 + 2] = ez; st[o6 + 3] = ax; st[o6 + 4] = ay; st[o6 + 5] = az;
        ox = px; oy = py; oz = pz; dx = sdx; dy = sdy; dz = sdz;
        depth--;
    }
    while (lvl > 0) {                                                          // emitted.add(att * scattered)
        const o6 = 6 * --lvl;
        ix = st[o6] + st[o6 + 3] * ix; iy = st[o6 + 1] + st[o6 + 4] * iy; iz = st[o6 + 2] + st[o6 + 5] * iz;
    }
    LX = ix; LY = iy; LZ = iz;
}

// ---- RayTracer.render's loop nest over a crop window (ray-tracer.js:189-208) -------------------------
// st: {width, height, samples (sampleCount), maxDepth, aaMode (0 super, 1 stochastic, 2 centre), seed}
// crop: [x0, y0, w, h] in top-down rows; rows: [r0, r1, step] — the crop rows r0, r0 + step, ... < r1
// to render (a worker's share; interleaved rows balance cheap sky rows against expensive ones).
// Returns the per-pixel colour sums (before .div(sampleCount)), world.hit counts and RNG draws of
// those rows, in order.
export function renderCrop(S, st, crop, rows) {
    const W = st.width, H = st.height, ns = st.samples;
    const [x0, y0, cw, ch] = crop || [0, 0, W, H];
    const [r0, r1, step] = rows || [0, ch, 1];
    const nrows = r1 > r0 ? Math.ceil((r1 - r0) / step) : 0, n = nrows * cw;
    const sum = new Float64Array(3 * n), segs = new Uint32Array(n), draws = new Uint32Array(n);
    const seedm = lowbias32((st.seed ^ 0x3C6EF372) >>> 0);
    const C = S.cam;
    for (let rr = 0; rr < nrows; rr++) {
        const row = y0 + r0 + rr * step, j = H - 1 - row;
        for (let i = x0; i < x0 + cw; i++) {
            const q = rr * cw + (i - x0);
            const pkey = lowbias32((seedm ^ ((row * W + i) >>> 0)) >>> 0);
            let cx = 0, cy = 0, cz = 0, nd = 0;
            SEGS = 0;
            for (let s = 0; s < ns; s++) {
                KEY = lowbias32((pkey ^ lowbias32((s + 0x1B873593) >>> 0)) >>> 0);
                K = 0;
                let u, v;
                if (st.aaMode === 1) {                                         // getAntiAliasSample
                    const r1_ = rnd(), r2 = rnd();
                    const offX = Math.sqrt(r1_) * Math.cos(2 * Math.PI * r2);
                    const offY = Math.sqrt(r1_) * Math.sin(2 * Math.PI * r2);
                    u = (i + 0.5 + offX * 0.5) / W; v = (j + 0.5 + offY * 0.5) / H;
                } else if (st.aaMode === 0) {
                    u = (i + rnd()) / W; v = (j + rnd()) / H;
                } else {
                    u = (i + 0.5) / W; v = (j + 0.5) / H;
                }
                let rx, ry;                                                    // Camera.getRay
                do { rx = rnd() * 2 - 1; ry = rnd() * 2 - 1; } while (rx * rx + ry * ry + 0 * 0 >= 1.0);
                const lr = C[21];
                rx = rx * lr; ry = ry * lr;
                let ox, oy, oz, dx, dy, dz;
                const bx = (C[3] + C[6] * u) + C[9] * v, by = (C[4] + C[7] * u) + C[10] * v, bz = (C[5] + C[8] * u) + C[11] * v;
                if (S.ortho) {
                    ox = (C[0] + C[12] * rx) + C[15] * ry; oy = (C[1] + C[13] * rx) + C[16] * ry; oz = (C[2] + C[14] * rx) + C[17] * ry;
                    const ex = (bx - ox) + C[18] * -1, ey = (by - oy) + C[19] * -1, ez = (bz - oz) + C[20] * -1;
                    const l = Math.sqrt(ex * ex + ey * ey + ez * ez);
                    if (l > 0) { dx = ex / l; dy = ey / l; dz = ez / l; } else { dx = 0; dy = 0; dz = 0; }
                } else {
                    ox = C[0] + (C[12] * rx + C[15] * ry); oy = C[1] + (C[13] * rx + C[16] * ry); oz = C[2] + (C[14] * rx + C[17] * ry);
                    dx = bx - ox; dy = by - oy; dz = bz - oz;
                }
                rayColor(S, ox, oy, oz, dx, dy, dz, st.maxDepth);
                cx = cx + LX; cy = cy + LY; cz = cz + LZ;                      // color = color.add(rayColor)
                nd += K;
            }
            sum[3 * q] = cx; sum[3 * q + 1] = cy; sum[3 * q + 2] = cz;
            segs[q] = SEGS; draws[q] = nd;
        }
    }
    return { sum, segs, draws };
}
