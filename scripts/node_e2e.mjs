// Node end-to-end timing of the drop-in (bench.py's end_to_end_node): GpuRayTracer.render() — the same
// gpuRender() that installGpuRender() puts on the reference's RayTracer — on a bench workload.
// The first render() uploads the scene and builds the BVHs; the timed second one reuses the resident
// scene (packScene + byte compare), traces, runs the epilogue and copies the RGBA8 frame into
// imageData (the reference's render() output; the Float32 frame only with keepFloatData).
//   node scripts/node_e2e.mjs '{"scene": path, "width", "height", "spp", "depth", "seed", "precision"}'
import fs from 'fs';
import { GpuRayTracer } from '../blenderraytracer_amd/js/gpu-ray-tracer.mjs';

const a = JSON.parse(process.argv[2]);
const rt = new GpuRayTracer({ width: a.width, height: a.height }, { seed: a.seed, precision: a.precision || 'f64' });
if (!rt.loadFromJSON(JSON.parse(fs.readFileSync(a.scene, 'utf8')))) throw new Error('loadFromJSON failed');
if (rt.width !== a.width || rt.height !== a.height) rt.resizeCanvas(a.width, a.height);
rt.updateRenderSettings({ samples: a.spp, maxBounces: a.depth });
const ms = () => Number(process.hrtime.bigint()) * 1e-6;
(async () => {
    let t = ms();
    await rt.render();
    const first = ms() - t;
    const progress = [];
    t = ms();
    await rt.render((f) => progress.push(f));
    const wall = ms() - t;
    const kernel = rt.lastStats ? rt.lastStats.kernelMs : null;
    // the same frame as ONE sample batch (no progress calls, no preview frames): what the default
    // 16-batch progressive render costs over it
    const one = new GpuRayTracer({ width: a.width, height: a.height }, { seed: a.seed, precision: a.precision || 'f64', batchSamples: 0 });
    one.loadFromJSON(JSON.parse(fs.readFileSync(a.scene, 'utf8')));
    if (one.width !== a.width || one.height !== a.height) one.resizeCanvas(a.width, a.height);
    one.updateRenderSettings({ samples: a.spp, maxBounces: a.depth });
    await one.render();
    t = ms();
    await one.render();
    const wallOne = ms() - t;
    const n = a.width * a.height * a.spp;
    process.stdout.write(JSON.stringify({ value: n / (wall * 1e-3) / 1e6, wall_ms: wall, first_call_ms: first,
                                          kernel_ms: kernel, progress_calls: progress.length,
                                          one_batch_wall_ms: wallOne }) + '\n');
})().catch((e) => { process.stderr.write(String(e.stack || e) + '\n'); process.exit(1); });
