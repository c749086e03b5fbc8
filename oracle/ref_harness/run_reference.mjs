// Golden-vector generator: runs the REAL reference renderer (/root/reference/js) under Node with
// Math.random replaced by the keyed RNG (blenderraytracer_amd/js/keyed-rng.mjs) and writes the
// fixtures under tests/golden/.  TEST INFRASTRUCTURE ONLY — runs in the build container, never on
// the GPU box, never imported by product code.
//
// The reference is browser ES-module code; to run it on Node 12 this script
//   (1) copies /root/reference/js to a temp dir with {"type":"module"} (no repo copy is made),
//   (2) rewrites `this.camera?.X` -> `(this.camera && this.camera.X)` in ray-tracer.js:504-508
//       (optional chaining does not parse on Node 12; the lines are in updateCamera, off the path),
//   (3) provides window.renderCancelled, performance.now and a 2D-canvas stand-in holding imageData.
// Float outputs are captured with per-instance wrappers (SURVEY §8c): getAntiAliasSample selects
// the keyed stream for (pixel, sample); toneMap captures the linear per-pixel mean; gammaCorrect the
// post-gamma value; world.hit counts ray segments.
//
// usage: node oracle/ref_harness/run_reference.mjs [--only name,name] [--kats]
import fs from 'fs';
import os from 'os';
import path from 'path';
import zlib from 'zlib';
import { fileURLToPath, pathToFileURL } from 'url';
import { KeyedStream, permutation } from '../../blenderraytracer_amd/js/keyed-rng.mjs';

const HERE = path.dirname(fileURLToPath(import.meta.url));
const REPO = path.resolve(HERE, '..', '..');
const REF = process.env.RT_REFERENCE || '/root/reference';
const OUT = path.join(REPO, 'tests', 'golden');

function prepareReference() {
    const dir = fs.mkdtempSync(path.join(os.tmpdir(), 'rt-ref-'));
    fs.mkdirSync(path.join(dir, 'js'));
    for (const f of fs.readdirSync(path.join(REF, 'js'))) {
        let src = fs.readFileSync(path.join(REF, 'js', f), 'utf8');
        if (f === 'ray-tracer.js') src = src.replace(/this\.camera\?\.([A-Za-z]+)/g, '(this.camera && this.camera.$1)');
        fs.writeFileSync(path.join(dir, 'js', f), src);
    }
    fs.writeFileSync(path.join(dir, 'package.json'), '{"type":"module"}');
    return dir;
}

// ---- browser globals -------------------------------------------------------------------------
global.window = { renderCancelled: false };
global.performance = { now: () => Date.now() };
const realLog = console.log;
console.log = () => {};
console.warn = () => {};
console.error = () => {};

function makeCanvas(w, h) {
    return {
        width: w, height: h, style: {},
        getContext: () => ({
            createImageData: (cw, ch) => ({ width: cw, height: ch, data: new Uint8ClampedArray(cw * ch * 4) }),
            putImageData() {},
        }),
    };
}

// ---- keyed Math.random ------------------------------------------------------------------------
let stream = new KeyedStream(0);
let drawCounter = null;   // per-pixel draw counts while rendering
let curPix = -1;
Math.random = () => { if (drawCounter && curPix >= 0) drawCounter[curPix]++; return stream.next(); };

function enc(v) {
    if (typeof v === 'number') {
        if (Number.isNaN(v)) return 'NaN';
        if (v === Infinity) return 'Infinity';
        if (v === -Infinity) return '-Infinity';
        return v;
    }
    if (Array.isArray(v)) return v.map(enc);
    if (v && typeof v === 'object') { const o = {}; for (const k of Object.keys(v)) o[k] = enc(v[k]); return o; }
    return v;
}
const v3 = (v) => [v.x, v.y, v.z];

function loadScene(name) {
    const file = name.endsWith('.json') ? name : name + '.json';
    return JSON.parse(fs.readFileSync(path.join(REPO, 'scenes', file), 'utf8'));
}

function writeGz(file, typed) {
    fs.writeFileSync(path.join(OUT, file), zlib.gzipSync(Buffer.from(typed.buffer, typed.byteOffset, typed.byteLength), { level: 9 }));
}

async function runCase(mods, c) {
    const { RayTracer, Vec3 } = mods;
    const canvas = makeCanvas(c.width, c.height);
    stream = new KeyedStream(c.seed);
    stream.select(0xFFFFFFFE, 0xFFFFFFFE);           // constructor's default scene: irrelevant stream
    const rt = new RayTracer(canvas);
    stream.select(0xFFFFFFFF, 0xFFFFFFFF);           // PERM stream for the loaded World's PerlinNoise
    const ok = rt.loadFromJSON(loadScene(c.scene));
    if (!ok) throw new Error('loadFromJSON failed for ' + c.name);
    rt.updateRenderSettings(c.settings);
    if (c.background) rt.updateBackground(c.background.type, c.background.intensity);
    const W = rt.width, H = rt.height;
    const perm = rt.world.cloudNoise.p.slice();
    const permExpect = permutation(c.seed);
    if (perm.some((x, i) => x !== permExpect[i])) throw new Error('perm stream mismatch');

    // crop window in output (top-down) coordinates
    const [x0, y0, cw, ch] = c.crop || [0, 0, W, H];
    const n = cw * ch;
    const linear = new Float64Array(n * 3), post = new Float64Array(n * 3);
    const rgba = new Uint8Array(n * 4);
    const segs = new Uint32Array(n), draws = new Uint32Array(n);
    const fullSegs = new Uint32Array(W * H), fullDraws = new Uint32Array(W * H);
    drawCounter = fullDraws;

    const localIndex = (p) => { const row = Math.floor(p / W), col = p % W; return (row - y0) * cw + (col - x0); };
    const origAA = rt.getAntiAliasSample.bind(rt);
    rt.getAntiAliasSample = (i, j, s) => {
        curPix = (H - 1 - j) * W + i;
        stream.select(curPix, s);
        return origAA(i, j, s);
    };
    const origTM = rt.toneMap.bind(rt);
    rt.toneMap = (color) => { const q = localIndex(curPix); linear.set(v3(color), q * 3); return origTM(color); };
    const origGC = rt.gammaCorrect.bind(rt);
    rt.gammaCorrect = (color) => { const r = origGC(color); post.set(v3(r), localIndex(curPix) * 3); return r; };
    const world = rt.world;
    const origHit = world.hit.bind(world);
    world.hit = (ray, a, b) => { fullSegs[curPix]++; return origHit(ray, a, b); };

    const sampleCount = rt.antiAliasing === 'none' ? 1 : rt.samples;
    // PostProcessor.denoise (post-processor.js:45-77) output, when render() applies it (ray-tracer.js:266-276)
    let denoised = null;
    const PP = mods.PostProcessor;
    const origDenoise = PP.denoise;
    PP.denoise = (data, w, h, strength) => { denoised = origDenoise.call(PP, data, w, h, strength); return denoised; };
    const t0 = process.hrtime.bigint();
    if (!c.crop) {
        await rt.render();
        const data = rt.imageData.data;
        rgba.set(data);
    } else {
        // Same loop body as RayTracer.render (ray-tracer.js:189-252), restricted to the crop rows/cols.
        const tmp = new Uint8ClampedArray(4);
        for (let j = H - 1; j >= 0; j--) {
            const row = H - 1 - j;
            if (row < y0 || row >= y0 + ch) continue;
            for (let i = x0; i < x0 + cw; i++) {
                let color = new Vec3(0, 0, 0);
                for (let s = 0; s < sampleCount; s++) {
                    const sm = rt.getAntiAliasSample(i, j, s);
                    const ray = rt.camera.getRay(sm.u, sm.v);
                    color = color.add(rt.rayColor(ray, rt.maxBounces));
                }
                color = color.div(sampleCount);
                color = rt.toneMap(color);
                color = rt.gammaCorrect(color);
                tmp[0] = Math.min(255, Math.max(0, Math.floor(color.x * 255)));
                tmp[1] = Math.min(255, Math.max(0, Math.floor(color.y * 255)));
                tmp[2] = Math.min(255, Math.max(0, Math.floor(color.z * 255)));
                tmp[3] = 255;
                rgba.set(tmp, ((row - y0) * cw + (i - x0)) * 4);
            }
        }
    }
    const secs = Number(process.hrtime.bigint() - t0) / 1e9;
    PP.denoise = origDenoise;
    drawCounter = null; curPix = -1;
    for (let r = 0; r < ch; r++) for (let x = 0; x < cw; x++) {
        const p = (y0 + r) * W + (x0 + x);
        segs[r * cw + x] = fullSegs[p]; draws[r * cw + x] = fullDraws[p];
    }
    const cam = rt.camera;
    const files = {};
    const arrays = { linear, post, rgba8: rgba, segs, draws };
    if (denoised) arrays.denoised = denoised;
    for (const [k, arr] of Object.entries(arrays)) {
        files[k] = `${c.name}.${k}.gz`;
        writeGz(files[k], arr);
    }
    return {
        name: c.name, scene: c.scene, seed: c.seed, requested: [c.width, c.height], width: W, height: H,
        crop: [x0, y0, cw, ch], settings_in: c.settings, background_in: c.background,
        resolved: {
            maxBounces: rt.maxBounces, samples: rt.samples, gamma: rt.gamma, exposure: rt.exposure,
            toneMapping: rt.toneMapping, antiAliasing: rt.antiAliasing, denoising: rt.denoising,
            denoiseStrength: rt.denoiseStrength,
            skyIntensity: rt.world.skyIntensity,
        },
        camera: {
            origin: v3(cam.origin), lowerLeftCorner: v3(cam.lowerLeftCorner), horizontal: v3(cam.horizontal),
            vertical: v3(cam.vertical), u: v3(cam.u), v: v3(cam.v), w: v3(cam.w), lensRadius: cam.lensRadius,
            type: cam.type, fov: cam.fov, focusDist: cam.focusDist, aperture: cam.aperture,
        },
        perm_head: perm.slice(0, 16),
        files,
        js_seconds: secs,
        js_samples: n * sampleCount,
    };
}

// ---- per-function known-answer vectors ----------------------------------------------------------
function kats(mods) {
    const { Vec3, Ray, Sphere, Plane, Box, Triangle, TriangleMesh, Lambertian, Metal, Dielectric, Emissive,
        Camera, World, PostProcessor, HitRecord } = mods;
    const gen = new KeyedStream(424242);
    stream = new KeyedStream(4242);                  // scatter / getRay draws: seed 4242, keyed (pixel, sample)
    let gk = 0;
    const U = (a, b) => { gen.select(7, gk++); return a + (b - a) * gen.next(); };
    const randVec = (a, b) => new Vec3(U(a, b), U(a, b), U(a, b));
    const hitOut = (h) => h ? { t: h.t, point: v3(h.point), normal: v3(h.normal), frontFace: h.frontFace } : null;
    const out = { primitives: [], scatter: [], camera: [], background: [], post: [] };

    const shapes = [
        { kind: 'sphere', args: [[0, 0, -1], 0.5], make: () => new Sphere(new Vec3(0, 0, -1), 0.5, null) },
        { kind: 'sphere', args: [[0.2, -0.1, -1.3], -0.45], make: () => new Sphere(new Vec3(0.2, -0.1, -1.3), -0.45, null) },
        { kind: 'sphere', args: [[0, -1000, 0], 1000], make: () => new Sphere(new Vec3(0, -1000, 0), 1000, null) },
        { kind: 'plane', args: [[0, -0.5, 0], [0, 2, 0.3]], make: () => new Plane(new Vec3(0, -0.5, 0), new Vec3(0, 2, 0.3), null) },
        { kind: 'box', args: [[-0.5, -0.5, -1.5], [0.5, 0.25, -0.5]], make: () => new Box(new Vec3(-0.5, -0.5, -1.5), new Vec3(0.5, 0.25, -0.5), null) },
        { kind: 'box', args: [[-10, -2, -30], [12, 3, -11]], make: () => new Box(new Vec3(-10, -2, -30), new Vec3(12, 3, -11), null) },
        { kind: 'triangle', args: [[-1, -1, -2], [1, -1, -2.5], [0, 1, -2.2]], make: () => new Triangle(new Vec3(-1, -1, -2), new Vec3(1, -1, -2.5), new Vec3(0, 1, -2.2), null) },
        { kind: 'triangle', args: [[0, 0, -1], [1e-3, 0, -1], [0, 1e-3, -1]], make: () => new Triangle(new Vec3(0, 0, -1), new Vec3(1e-3, 0, -1), new Vec3(0, 1e-3, -1), null) },
    ];
    const rays = [];
    for (let r = 0; r < 160; r++) {
        const o = r < 120 ? randVec(-1.5, 1.5) : new Vec3(0, 0, [0, 1, -1, -0.5][r % 4]);
        let d;
        if (r % 10 === 3) d = new Vec3(0, 0, -1);                          // axis parallel: Inf/NaN in Box
        else if (r % 10 === 7) d = new Vec3(U(-1, 1), 0, -1);
        else d = new Vec3(U(-1, 1), U(-1, 1), U(-1.5, 0.5)).mul(U(0.2, 3));
        const tMax = r % 5 === 0 ? U(0.1, 2) : Infinity;
        rays.push({ o, d, tMin: 0.001, tMax });
    }
    rays.push({ o: new Vec3(-0.5, 0, 0), d: new Vec3(0, 0, -1), tMin: 0.001, tMax: Infinity });   // box edge: 0/0
    for (const sh of shapes) {
        const obj = sh.make();
        for (const r of rays) {
            const h = obj.hit(new Ray(r.o, r.d), r.tMin, r.tMax);
            out.primitives.push({ kind: sh.kind, args: sh.args, o: v3(r.o), d: v3(r.d), tMin: r.tMin, tMax: r.tMax, hit: hitOut(h) });
        }
    }
    // mesh tie-order: two coincident triangles with opposite winding -> last one wins (<=)
    {
        const verts = [[0, 0, -2], [1, 0, -2], [0, 1, -2], [0, 0, -2], [0, 1, -2], [1, 0, -2]];
        const mesh = new TriangleMesh(verts.map((a) => new Vec3(a[0], a[1], a[2])), [0, 1, 2, 3, 4, 5, 0, 1], null);
        for (const r of rays.slice(0, 40)) {
            const h = mesh.hit(new Ray(r.o, r.d), r.tMin, r.tMax);
            out.primitives.push({ kind: 'mesh', args: [verts, [0, 1, 2, 3, 4, 5, 0, 1]], o: v3(r.o), d: v3(r.d), tMin: r.tMin, tMax: r.tMax, hit: hitOut(h) });
        }
    }
    // scatter: given (ray, hit record) and stream (pixel, sample) -> result + draws consumed
    const mats = [
        { m: { type: 'lambertian', albedo: [0.7, 0.3, 0.2] }, make: () => new Lambertian(new Vec3(0.7, 0.3, 0.2)) },
        { m: { type: 'metal', albedo: [0.8, 0.8, 0.9], roughness: 0 }, make: () => new Metal(new Vec3(0.8, 0.8, 0.9), 0) },
        { m: { type: 'metal', albedo: [0.8, 0.6, 0.2], roughness: 0.45 }, make: () => new Metal(new Vec3(0.8, 0.6, 0.2), 0.45) },
        { m: { type: 'dielectric', ior: 1.5 }, make: () => new Dielectric(1.5) },
        { m: { type: 'dielectric', ior: 2.4 }, make: () => new Dielectric(2.4) },
        { m: { type: 'emissive', emit: [3, 3, 2.4] }, make: () => new Emissive(new Vec3(1, 1, 0.8), 3) },
    ];
    for (const mm of mats) {
        const mat = mm.make();
        for (let q = 0; q < 60; q++) {
            const d = randVec(-1, 1).mul(U(0.3, 2));
            let n = randVec(-1, 1).normalize();
            const rec = new HitRecord();
            rec.t = U(0.1, 3); rec.point = randVec(-2, 2);
            rec.setFaceNormal(new Ray(new Vec3(0, 0, 0), d), n);
            stream.select(1000 + q, 77);
            const before = stream.k;
            const sr = mat.scatter(new Ray(new Vec3(0, 0, 0), d), rec);
            const used = stream.k - before;
            out.scatter.push({
                material: mm.m, d: v3(d), point: v3(rec.point), normal: v3(rec.normal), frontFace: rec.frontFace,
                seed: 4242, pixel: 1000 + q, sample: 77, draws: used,
                result: sr ? { origin: v3(sr.scattered.origin), dir: v3(sr.scattered.direction), attenuation: v3(sr.attenuation) } : null,
                emitted: v3(mat.emitted(0, 0, rec.point)),
            });
        }
    }
    // camera: constructor vectors + getRay
    const camSpecs = [
        [[3, 2, 2], [0, 0, -1], [0, 1, 0], 45, 1.5, 0.0, 10.0, 'perspective'],
        [[13, 2, 3], [0, 0, 0], [0, 1, 0], 20, 16 / 9, 0.1, 10.0, 'perspective'],
        [[0, 2, 3], [0, 0, -1], [0, 1, 0], 40, 1.5, 0.05, 4.0, 'perspective'],
        [[1, 4, 2], [0, 0, -1], [0.2, 1, 0], 70, 1.0, 0.3, 3.0, 'orthographic'],
    ];
    for (const cs of camSpecs) {
        const cam = new Camera(new Vec3(...cs[0]), new Vec3(...cs[1]), new Vec3(...cs[2]), cs[3], cs[4], cs[5], cs[6], cs[7]);
        const rays2 = [];
        for (let q = 0; q < 24; q++) {
            const s = U(0, 1), t = U(0, 1);
            stream.select(500 + q, 3);
            const ray = cam.getRay(s, t);
            rays2.push({ s, t, seed: 4242, pixel: 500 + q, sample: 3, draws: stream.k, origin: v3(ray.origin), dir: v3(ray.direction) });
        }
        out.camera.push({
            spec: cs, origin: v3(cam.origin), lowerLeftCorner: v3(cam.lowerLeftCorner), horizontal: v3(cam.horizontal),
            vertical: v3(cam.vertical), u: v3(cam.u), v: v3(cam.v), w: v3(cam.w), lensRadius: cam.lensRadius, rays: rays2,
        });
    }
    // backgrounds (working updateBackground semantics) for the keyed perm of seed 99
    stream = new KeyedStream(99);
    stream.select(0xFFFFFFFF, 0xFFFFFFFF);
    const world = new World();
    world.skyIntensity = 1.25;
    const dirs = [];
    for (let q = 0; q < 64; q++) dirs.push(randVec(-1, 1).mul(U(0.2, 4)));
    dirs.push(new Vec3(0.3, 0.6, 0.8), new Vec3(-0.3, 0.6, -0.5), new Vec3(0, 1, 0), new Vec3(0, -1, 0));
    const bgs = {
        gradient: world.skyGradient.bind(world), solid: world.solidBackground(new Vec3(0.1, 0.1, 0.1)),
        hdri: world.hdriBackground(), procedural_sky: world.proceduralSky.bind(world),
    };
    for (const [type, fn] of Object.entries(bgs)) {
        for (const d of dirs) out.background.push({ type, intensity: 1.25, seed: 99, d: v3(d), color: v3(fn(new Ray(new Vec3(0, 0, 0), d))) });
    }
    const noisePts = [];
    for (let q = 0; q < 40; q++) { const p = randVec(-30, 30); noisePts.push({ p: v3(p), n: world.cloudNoise.noise(p) }); }
    out.noise = { seed: 99, perm: world.cloudNoise.p.slice(), points: noisePts };
    // post processing
    for (let q = 0; q < 50; q++) {
        const c = q < 45 ? randVec(0, 4) : new Vec3([0, -0.5, NaN, 1e6, 0.25][q - 45], 0.5, 2);
        const exp = U(0.5, 2), gamma = U(1.8, 2.6);
        out.post.push({
            c: v3(c), exposure: exp, gamma,
            reinhard: v3(PostProcessor.reinhardToneMap(c, exp)), aces: v3(PostProcessor.acesToneMap(c, exp)),
            linear: v3(c.mul(exp)), gammaCorrect: v3(PostProcessor.gammaCorrect(c, gamma)),
        });
    }
    return out;
}

// Loader-only cases (cases.json loader_cases): RayTracer.loadFromJSON's verdict and what the World
// holds afterwards -> tests/golden/loader_cases.json
function loaderCases(mods, spec) {
    const out = { generator: 'oracle/ref_harness/run_reference.mjs --loader', cases: {} };
    for (const c of spec.loader_cases || []) {
        stream.select(0xFFFFFFFE, 0xFFFFFFFE);
        const rt = new mods.RayTracer(makeCanvas(32, 24));
        stream.select(0xFFFFFFFF, 0xFFFFFFFF);
        const ok = rt.loadFromJSON(JSON.parse(JSON.stringify(c.scene)));
        const cam = rt.camera;
        out.cases[c.name] = {
            scene: c.scene, ok, objects: rt.world.objects.length, lights: rt.world.lights.length,
            camera: cam ? [cam.origin, cam.lowerLeftCorner, cam.horizontal, cam.vertical].map((v) => [v.x, v.y, v.z]) : null,
            camera_type: cam ? String(cam.type) : null,
        };
    }
    return out;
}

async function main() {
    const argv = process.argv.slice(2);
    const only = argv.includes('--only') ? argv[argv.indexOf('--only') + 1].split(',') : null;
    const dir = prepareReference();
    const url = (f) => pathToFileURL(path.join(dir, 'js', f)).href;
    const mods = {
        ...(await import(url('ray-tracer.js'))), ...(await import(url('math.js'))), ...(await import(url('geometry.js'))),
        ...(await import(url('materials.js'))), ...(await import(url('camera.js'))), ...(await import(url('world.js'))),
        ...(await import(url('post-processor.js'))),
    };
    fs.mkdirSync(OUT, { recursive: true });
    const spec = JSON.parse(fs.readFileSync(path.join(HERE, 'cases.json'), 'utf8'));
    if (argv.includes('--loader')) {
        const l = loaderCases(mods, spec);
        fs.writeFileSync(path.join(OUT, 'loader_cases.json'), JSON.stringify(l, null, 1) + '\n');
        realLog(`loader cases: ${Object.keys(l.cases).length} (${Object.values(l.cases).filter((c) => !c.ok).length} rejected)`);
        fs.rmSync ? fs.rmSync(dir, { recursive: true, force: true }) : fs.rmdirSync(dir, { recursive: true });
        return;
    }
    const manifestPath = path.join(OUT, 'manifest.json');
    const manifest = fs.existsSync(manifestPath) ? JSON.parse(fs.readFileSync(manifestPath, 'utf8')) : { cases: {} };
    manifest.generator = 'oracle/ref_harness/run_reference.mjs';
    manifest.node = process.version;
    for (const c of spec.cases) {
        if (only && !only.includes(c.name)) continue;
        const rec = await runCase(mods, c);
        manifest.cases[c.name] = enc(rec);
        realLog(`${c.name}: ${rec.width}x${rec.height} crop ${rec.crop} ${rec.js_samples} samples in ${rec.js_seconds.toFixed(2)} s (${(rec.js_samples / rec.js_seconds / 1e6).toFixed(4)} Msamples/s)`);
    }
    if (!only || argv.includes('--kats')) {
        const k = kats(mods);
        fs.writeFileSync(path.join(OUT, 'kats.json.gz'), zlib.gzipSync(JSON.stringify(enc(k)), { level: 9 }));
        realLog(`kats: ${k.primitives.length} primitive, ${k.scatter.length} scatter, ${k.camera.length} cameras, ${k.background.length} background, ${k.post.length} post`);
    }
    fs.writeFileSync(manifestPath, JSON.stringify(manifest, null, 1) + '\n');
    fs.rmSync ? fs.rmSync(dir, { recursive: true, force: true }) : fs.rmdirSync(dir, { recursive: true });
}

main().catch((e) => { realLog(e && e.stack || e); process.exit(1); });
