// Node end-to-end timing of the drop-in (bench.py's end_to_end_node): GpuRayTracer.render() — the same
// gpuRender() that installGpuRender() puts on the reference's RayTracer — on a bench workload.
// The first render() uploads the scene and builds the BVHs; the timed ones reuse the resident scene
// (packScene + byte compare), trace in the default 16 progressive sample batches (onProgress and the
// running frame in imageData after each), run the epilogue and copy the RGBA8 frame into imageData (the
// reference's render() output; the Float32 frame only with keepFloatData).  Median of `reps` timed
// renders after one warm-up (SURVEY §8d), for the default render and two references: the same frame
// without preview frames and as one sample batch.
//   node scripts/node_e2e.mjs '{"scene": path, "width", "height", "spp", "depth", "seed", "precision", "reps"}'
import fs from 'fs';
import { GpuRayTracer } from '../blenderraytracer_amd/js/gpu-ray-tracer.mjs';

const a = JSON.parse(process.argv[2]);
const reps = a.reps || 5;
const ms = () => Number(process.hrtime.bigint()) * 1e-6;
const median = (v) => { const s = [...v].sort((x, y) => x - y); return s[Math.floor(s.length / 2)]; };

function tracer(opts) {
    const rt = new GpuRayTracer({ width: a.width, height: a.height }, { seed: a.seed, precision: a.precision || 'f64', ...opts });
    if (!rt.loadFromJSON(JSON.parse(fs.readFileSync(a.scene, 'utf8')))) throw new Error('loadFromJSON failed');
    if (rt.width !== a.width || rt.height !== a.height) rt.resizeCanvas(a.width, a.height);
    rt.updateRenderSettings({ samples: a.spp, maxBounces: a.depth });
    return rt;
}

async function timed(rt, withProgress) {
    const walls = [], kernels = [], inner = [];
    let calls = 0;
    for (let r = 0; r < reps; r++) {
        const progress = [];
        const t = ms();
        await rt.render(withProgress ? (f) => progress.push(f) : undefined);
        walls.push(ms() - t);
        kernels.push(rt.lastStats.kernelMs);
        inner.push(rt.lastStats.wallMs);
        calls = progress.length;
    }
    return { wall: median(walls), walls, kernel: median(kernels), inner: median(inner), calls };
}

(async () => {
    const rt = tracer({});
    let t = ms();
    await rt.render();
    const first = ms() - t;
    const d = await timed(rt, true);
    const np = tracer({ preview: false });
    await np.render();
    const n0 = await timed(np, true);
    const one = tracer({ batchSamples: 0 });
    await one.render();
    const o1 = await timed(one, false);
    const n = a.width * a.height * a.spp;
    process.stdout.write(JSON.stringify({
        value: n / (d.wall * 1e-3) / 1e6, wall_ms: d.wall, walls_ms: d.walls, first_call_ms: first, kernel_ms: d.kernel,
        rt_render_wall_ms: d.inner, progress_calls: d.calls, reps, no_preview_wall_ms: n0.wall,
        one_batch_wall_ms: o1.wall, one_batch_kernel_ms: o1.kernel }) + '\n');
})().catch((e) => { process.stderr.write(String(e.stack || e) + '\n'); process.exit(1); });
