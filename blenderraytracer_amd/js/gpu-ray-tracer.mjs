// GpuRayTracer — drop-in for the reference's RayTracer.render (js/ray-tracer.js:166-281) on MI355X.
//
// Two ways to use it:
//   1. installGpuRender(rayTracer, opts): replaces render() on an instance of the REFERENCE's own
//      RayTracer class.  Everything else (loadFromJSON, presets, updateCamera, UI) stays the
//      reference's code; render() packs this.world / this.camera (pack.mjs), traces on the GPU
//      through rt_napi.node -> librt_hip.so, and fills this.imageData like the reference does.
//   2. new GpuRayTracer(canvasOrSize, opts): a DOM-free RayTracer twin for Node (bench, tests, GPU
//      box) with the reference's loadFromJSON / updateRenderSettings / updateBackground semantics
//      restated in scene-model.mjs.
// Randomness: Math.random is replaced by the keyed RNG (keyed-rng.mjs); opts.seed selects it.
import { createRequire } from 'module';
import path from 'path';
import { fileURLToPath } from 'url';
import { packScene } from './pack.mjs';
import { Vec3, BG, defaultScene, loadFromJSON, setupCamera, permutation } from './scene-model.mjs';

const HERE = path.dirname(fileURLToPath(import.meta.url));
let native = null;

export function loadNative() {
    if (!native) {
        const require = createRequire(import.meta.url);
        const p = process.env.RT_NAPI_ADDON || path.join(HERE, '..', 'lib', 'rt_napi.node');
        native = require(p);   // throws if the addon (or librt_hip.so) is missing: no CPU fallback
    }
    return native;
}

export const AA = { supersampling: 0, stochastic: 1 };            // anything else: pixel centre (2)
export const TONE = { aces: 1, linear: 2 };                        // anything else: reinhard (0)
export const PRECISION = { f64: 0, f32: 1 };
export const ACCEL = { auto: 0, brute: 1, bvh: 2 };

// rt_settings from RayTracer fields (ray-tracer.js:23-33, :201, :125-161)
export function settingsOf(rt, opts = {}) {
    return {
        width: rt.width, height: rt.height,
        samples: rt.antiAliasing === 'none' ? 1 : rt.samples,
        maxDepth: rt.maxBounces,
        aaMode: AA[rt.antiAliasing] !== undefined ? AA[rt.antiAliasing] : 2,
        toneMap: TONE[rt.toneMapping] !== undefined ? TONE[rt.toneMapping] : 0,
        exposure: rt.exposure, gamma: rt.gamma,
        seed: (opts.seed || 0) >>> 0,
        precision: PRECISION[opts.precision || 'f64'],
        batchSamples: batchSamplesOf(rt, opts),
        // progressive display: the frame of the samples so far goes into imageData at every progress call
        preview: opts.preview ? 1 : 0,
        // 'sample': every pixel adds its samples in sample order (the reference's loop order); default: the
        // sample pool's order (faster; the RGBA8 frame can differ by one at a floor(c*255) boundary)
        sumOrder: opts.sumOrder === 'sample' ? 1 : 0,
        accel: ACCEL[opts.accel || 'auto'],
        // multi-GPU: every sample batch split over these HIP devices (rt_settings.devices)
        devices: opts.devices ? Array.from(opts.devices) : [],
        // continue a cancelled render from its checkpoint (rt_render_resume): the sums still on the device
        // (a lazy checkpointState nobody has read), or {sums, samplesDone} from the host
        ...(opts.resume ? (opts.resume.resident
            ? { resumeResident: 1, resumeSamplesDone: opts.resume.samplesDone }
            : { resumeSums: opts.resume.sums, resumeSamplesDone: opts.resume.samplesDone }) : {}),
        cropX0: opts.crop ? opts.crop[0] : 0, cropY0: opts.crop ? opts.crop[1] : 0,
        cropW: opts.crop ? opts.crop[2] : 0, cropH: opts.crop ? opts.crop[3] : 0,
        wantMean: opts.wantMean ? 1 : 0, wantCounts: opts.wantCounts ? 1 : 0,
        // the post-gamma Float32 frame: render() keeps it (this.floatData) only on request
        wantPost: opts.wantPost === false ? 0 : 1,
        // PostProcessor.denoise weights, evaluated with V8's Math.exp exactly as post-processor.js:55 does
        denoise: rt.denoising ? 1 : 0,
        denoiseW1: Math.exp(-(1) / (2 * rt.denoiseStrength * rt.denoiseStrength)),
        denoiseW2: Math.exp(-(2) / (2 * rt.denoiseStrength * rt.denoiseStrength)),
    };
}

// Progress granularity.  The reference reports progress and repaints after every row
// (ray-tracer.js:224-261); the GPU renders whole frames, so render() splits the samples into about
// `progressSteps` batches (default 16; opts.batchSamples overrides, 0 = one batch): after each batch
// onProgress fires and imageData shows the frame of the samples done so far.  The library sizes the
// batches (rt_settings.batch_samples = -steps) to a multiple of the sample pool's chunk, so progress
// costs no work-item splits (mesh50k at 256 spp: 22 batches of 12 instead of 16 of 16, DESIGN.md §1).
export const DEFAULT_PROGRESS_STEPS = 16;
function batchSamplesOf(rt, opts) {
    if (opts.batchSamples !== undefined) return opts.batchSamples || 0;
    if (!opts.intoImageData) return 0;
    return -(opts.progressSteps || DEFAULT_PROGRESS_STEPS);
}

const isCancelled = () => typeof window !== 'undefined' && window && window.renderCancelled;

const bytesOf = (a) => Buffer.from(a.buffer, a.byteOffset, a.byteLength);
function samePacked(a, b) {
    if (!a || !b) return false;
    for (const k of ['objects', 'materials', 'triangles', 'camera', 'solidColor', 'perm'])
        if (!bytesOf(a[k]).equals(bytesOf(b[k]))) return false;
    return a.cameraType === b.cameraType && a.background === b.background && Object.is(a.skyIntensity, b.skyIntensity);
}

// The scene resident on the GPU for this RayTracer: packed from world / camera at every render (cheap)
// and compared byte for byte with the cached one, so the upload and the BVH build happen only when
// the scene or the camera changed (presets, loadFromJSON, updateCamera, updateBackground...).
function residentScene(rt, nat, device) {
    const packed = packScene(rt.world, rt.camera);
    const c = rt.__gpuScene;
    if (c && c.device === device && samePacked(c.packed, packed)) return c.scene;
    if (c) nat.destroyScene(c.scene);
    rt.__gpuScene = null;
    const scene = nat.createScene(packed, device);
    Object.defineProperty(rt, '__gpuScene', { value: { scene, packed, device }, writable: true, configurable: true, enumerable: false });
    return scene;
}

// Drop the GPU copy of the scene (it is also freed when the RayTracer is garbage collected).
export function releaseGpuScene(rt) {
    if (rt.__gpuScene) { loadNative().destroyScene(rt.__gpuScene.scene); rt.__gpuScene = null; }
}

// The checkpoint of a cancelled render, lazily: samplesDone at once, the float64 sums (50 MB at 1080p)
// copied from the device only when `.sums` is read — the cancel returns without that copy, and resume()
// continues from the sums still on the device.  Valid until the RayTracer's next render (or a change of
// its scene): read `.sums` before rendering again to keep it.
function lazyCheckpoint(rt, nat, scene, samplesDone) {
    const gen = rt.__renderGen;
    let sums = null;
    const live = () => gen === rt.__renderGen && rt.__gpuScene && rt.__gpuScene.scene === scene;
    return {
        samplesDone,
        get resident() { return sums === null && live(); },
        get sums() {
            if (sums === null) {
                if (!live()) throw new Error('checkpointState: superseded by a later render (read .sums before rendering again)');
                sums = nat.checkpoint(scene).sums;
            }
            return sums;
        },
    };
}

// The GPU body of render(): trace, epilogue and readback; returns the native result (or null when
// cancelled, like the reference which then stops silently, ray-tracer.js:256,264).
export async function gpuRender(rt, onProgress, opts = {}) {
    const nat = loadNative();
    const scene = residentScene(rt, nat, opts.device || 0);
    // a resident checkpoint is resumed from the device (decided before this render supersedes it)
    const resume = opts.resume && opts.resume.resident ? { resident: true, samplesDone: opts.resume.samplesDone }
        : opts.resume ? { sums: opts.resume.sums, samplesDone: opts.resume.samplesDone } : undefined;
    Object.defineProperty(rt, '__renderGen', { value: (rt.__renderGen || 0) + 1, writable: true, configurable: true, enumerable: false });
    const st = settingsOf(rt, { preview: !!opts.intoImageData, ...opts, resume });
    // render() proper: the RGBA8 frame lands in this.imageData.data (full frame only), and with
    // st.preview every progress call first copies the running frame into it (the addon does that on
    // the main thread), so putImageData shows it like the reference's per-row repaint
    const into = opts.intoImageData && !opts.crop && rt.imageData && rt.imageData.data.length === rt.width * rt.height * 4;
    if (into) st.outRgba8 = rt.imageData.data;
    else st.preview = 0;
    const repaint = () => { if (into && rt.ctx && rt.ctx.putImageData) rt.ctx.putImageData(rt.imageData, 0, 0); };
    try {
        return await nat.render(scene, st, (f) => {
            if (st.preview) repaint();
            if (onProgress) onProgress(f);
            if (isCancelled()) nat.cancel(scene);
        });
    } catch (e) {
        if (e && e.status === -4) {                               // RT_ERR_CANCELLED
            // like the reference (ray-tracer.js:256,264): stop silently, leaving the partial frame on the
            // canvas: imageData holds the frame of the checkpointed samples; render({resume:
            // rt.checkpointState}) continues from them
            if (st.preview) repaint();
            rt.checkpointState = lazyCheckpoint(rt, nat, scene, nat.checkpointSamples(scene));
            return null;
        }
        throw e;
    }
}

function blit(rt, res) {
    // ray-tracer.js:215-276: RGBA8 top-down row-major, alpha 255, denoised when rt.denoising (all on the GPU)
    if (res.rgba8 !== rt.imageData.data) rt.imageData.data.set(res.rgba8);
    if (res.post) rt.floatData = res.post;                         // opts.keepFloatData
    if (rt.ctx && rt.ctx.putImageData) rt.ctx.putImageData(rt.imageData, 0, 0);
}

// Option 1: swap the render() of a reference RayTracer instance for the GPU path.
// opts: {seed, precision: 'f64'|'f32', accel, batchSamples | progressSteps (default 16), device,
//        devices: [HIP ordinals], sumOrder: 'pool' | 'sample',
//        keepFloatData: also read back the post-gamma Float32 frame into this.floatData}
export function installGpuRender(rayTracer, opts = {}) {
    rayTracer.render = async function render(onProgress) {
        const res = await gpuRender(this, onProgress, { ...opts, intoImageData: true, wantPost: !!opts.keepFloatData });
        if (!res) return;
        blit(this, res);
        this.lastStats = res.stats;
        if (onProgress) onProgress(1.0);
    };
    return rayTracer;
}

// Option 2: the DOM-free twin.
export class GpuRayTracer {
    constructor(canvas, opts = {}) {
        this.canvas = canvas && canvas.getContext ? canvas : null;
        this.ctx = this.canvas ? this.canvas.getContext('2d') : null;
        this.width = canvas.width;
        this.height = canvas.height;
        this.opts = opts;
        this.imageData = this.ctx ? this.ctx.createImageData(this.width, this.height) : { width: this.width, height: this.height, data: new Uint8ClampedArray(this.width * this.height * 4) };
        this.maxBounces = 5; this.samples = 4; this.gamma = 2.2; this.exposure = 1.0;
        this.toneMapping = 'reinhard'; this.antiAliasing = 'supersampling';
        this.denoising = false; this.denoiseStrength = 0.5;
        const d = defaultScene(this.width, this.height, permutation(opts.seed || 0));
        this.world = d.world;
        this.camera = d.camera;
    }

    loadFromJSON(json) {                                             // ray-tracer.js:305-334
        try {
            const r = loadFromJSON(json, this.width, this.height, permutation(this.opts.seed || 0));
            this.world = r.world;
            if (r.camera) this.camera = r.camera;
            if (r.newDimensions) this.resizeCanvas(r.newDimensions.width, r.newDimensions.height);
            return true;
        } catch (e) {
            return false;
        }
    }

    resizeCanvas(width, height) {                                    // ray-tracer.js:598-614
        this.width = width; this.height = height;
        if (this.canvas) { this.canvas.width = width; this.canvas.height = height; }
        this.imageData = { width, height, data: new Uint8ClampedArray(width * height * 4) };
        if (this.camera) this.camera = setupCamera(this.camera, width, height);
    }

    updateRenderSettings(p) {                                        // ray-tracer.js:554-566
        this.maxBounces = p.maxBounces || 5;
        this.samples = p.samples || 4;
        this.gamma = p.gamma || 2.2;
        this.exposure = p.exposure || 1.0;
        this.toneMapping = p.toneMapping || 'reinhard';
        this.antiAliasing = p.antiAliasing || 'supersampling';
        this.denoising = p.denoising || false;
        this.denoiseStrength = p.denoiseStrength || 0.5;
    }

    updateBackground(type, intensity = 1.0) {                        // ray-tracer.js:568-585
        this.world.skyIntensity = intensity;
        this.world.backgroundKind = BG[type] !== undefined && type !== 'nan' ? BG[type] : BG.gradient;
        this.world.solidColor = new Vec3(0.1, 0.1, 0.1);
    }

    async render(onProgress) {
        const res = await gpuRender(this, onProgress, { ...this.opts, intoImageData: true, wantPost: !!this.opts.keepFloatData });
        if (!res) return;
        blit(this, res);
        this.lastStats = res.stats;
        if (onProgress) onProgress(1.0);
    }

    // Continue the last cancelled render (window.renderCancelled) from its checkpoint.
    async resume(onProgress) {
        if (!this.checkpointState) return this.render(onProgress);
        const res = await gpuRender(this, onProgress, { ...this.opts, resume: this.checkpointState, intoImageData: true,
                                                        wantPost: !!this.opts.keepFloatData });
        if (!res) return;
        this.checkpointState = null;
        blit(this, res);
        this.lastStats = res.stats;
        if (onProgress) onProgress(1.0);
    }

    // Everything render() computes, plus diagnostics (linear mean, per-pixel segments / draws).
    async renderBuffers(opts = {}) {
        return gpuRender(this, opts.onProgress, { ...this.opts, ...opts });
    }
}
