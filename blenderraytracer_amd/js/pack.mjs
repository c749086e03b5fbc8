// Packs a World + Camera into the rt_scene_desc records of include/rt_hip.h.
//
// Duck-typed on the reference's object protocol (SURVEY §1 L4), so it accepts both the reference's
// own js/world.js / js/geometry.js / js/materials.js / js/camera.js instances (the browser drop-in)
// and the restated model of scene-model.mjs (Node).  World.objects order is preserved: it decides
// ties (js/world.js:24-30).
const OBJ = { sphere: 0, plane: 1, box: 2, triangle: 3, mesh: 4 };
const MAT = { lambertian: 0, metal: 1, dielectric: 2, emissive: 3 };
export const BG_CODE = { gradient: 0, solid: 1, hdri: 2, procedural_sky: 3, nan: 4 };
export const OBJECT_BYTES = 64;
export const MATERIAL_BYTES = 72;

function materialRecord(m) {
    if (m == null) throw new Error('object without material');
    if (m.texture !== undefined) throw new Error('textured materials are not reachable from render() (SURVEY §0) and not supported');
    if (m.refractionIndex !== undefined) return { type: MAT.dielectric, ior: m.refractionIndex };
    if (m.intensity !== undefined && m.color !== undefined) {
        // materials.js:95: emitted = color.mul(intensity), evaluated in double exactly as the reference does
        const e = typeof m.emitted === 'function' ? m.emitted(0, 0, null) : { x: m.color.x * m.intensity, y: m.color.y * m.intensity, z: m.color.z * m.intensity };
        return { type: MAT.emissive, emit: [e.x, e.y, e.z] };
    }
    if (m.albedo !== undefined && m.roughness !== undefined) return { type: MAT.metal, albedo: [m.albedo.x, m.albedo.y, m.albedo.z], roughness: m.roughness };
    if (m.albedo !== undefined) return { type: MAT.lambertian, albedo: [m.albedo.x, m.albedo.y, m.albedo.z] };
    throw new Error('unsupported material');
}

// World.background is a function in the reference; recover which one (ray-tracer.js:568-585,
// scene-loader.js:38-51).  Our own World carries backgroundKind directly.
function backgroundOf(world) {
    if (world.backgroundKind !== undefined) {
        const c = world.solidColor || { x: 0.1, y: 0.1, z: 0.1 };
        return { code: world.backgroundKind, solid: [c.x, c.y, c.z] };
    }
    const fn = world.background;
    const name = fn && fn.name;
    if (name === 'bound skyGradient') return { code: BG_CODE.gradient, solid: [0, 0, 0] };
    if (name === 'bound proceduralSky') return { code: BG_CODE.procedural_sky, solid: [0, 0, 0] };
    if (name === 'bound solidBackground' || name === 'bound hdriBackground') return { code: BG_CODE.nan, solid: [0, 0, 0] };
    if (typeof fn === 'function' && fn.length === 0) {            // solidBackground(color) closure
        const saved = world.skyIntensity;
        world.skyIntensity = 1;
        const c = fn();
        world.skyIntensity = saved;
        return { code: BG_CODE.solid, solid: [c.x, c.y, c.z] };
    }
    if (typeof fn === 'function' && fn.length === 1) return { code: BG_CODE.hdri, solid: [0, 0, 0] };  // hdriBackground() closure
    throw new Error('unsupported world.background');
}

// (indexed stores, no temporary array: packScene runs on every render() to detect scene changes, and
// a 50k-triangle mesh is 600k values)
function triangleRecord(t, out, k) {
    const b = 12 * k, v0 = t.v0, v1 = t.v1, v2 = t.v2, n = t.normal;
    out[b] = v0.x; out[b + 1] = v0.y; out[b + 2] = v0.z;
    out[b + 3] = v1.x; out[b + 4] = v1.y; out[b + 5] = v1.z;
    out[b + 6] = v2.x; out[b + 7] = v2.y; out[b + 8] = v2.z;
    out[b + 9] = n.x; out[b + 10] = n.y; out[b + 11] = n.z;
}

export function packScene(world, camera) {
    const mats = [];
    const matIndex = new Map();
    const matOf = (m) => {
        if (!matIndex.has(m)) { matIndex.set(m, mats.length); mats.push(materialRecord(m)); }
        return matIndex.get(m);
    };
    let ntri = 0;
    for (const o of world.objects) if (o.triangles) ntri += o.triangles.length; else if (o.v0) ntri += 1;
    const tris = new Float64Array(Math.max(1, ntri) * 12);
    // records through typed-array views (little-endian hosts, as the C ABI's x86-64 / aarch64 peers):
    // plain indexed stores, no DataView calls or temporaries
    const objects = new ArrayBuffer(OBJECT_BYTES * world.objects.length);
    const oi = new Int32Array(objects), of = new Float64Array(objects);
    let k = 0;
    const objs = world.objects;
    for (let i = 0; i < objs.length; i++) {
        const o = objs[i];
        const gi = i * (OBJECT_BYTES / 8) + 2;                    // g[0] at byte 16
        const g = (a, b, c, d, e, f) => {
            of[gi] = a; of[gi + 1] = b; of[gi + 2] = c; of[gi + 3] = d;
            if (e !== undefined) { of[gi + 4] = e; of[gi + 5] = f; }
        };
        let type, mat, first = 0, count = 0;
        if (o.triangles) {                                            // TriangleMesh
            type = OBJ.mesh;
            first = k; count = o.triangles.length;
            mat = count ? matOf(o.triangles[0].material) : matOf(o.material || { albedo: { x: 0, y: 0, z: 0 } });
            const ts = o.triangles, m0 = count ? ts[0].material : null;
            for (let j = 0; j < count; j++) {
                const t = ts[j];
                if (t.material !== m0) throw new Error('mesh triangles with different materials');
                triangleRecord(t, tris, k++);
            }
        } else if (o.v0) {                                            // Triangle
            type = OBJ.triangle; mat = matOf(o.material); first = k; count = 1;
            triangleRecord(o, tris, k++);
        } else if (o.center !== undefined && o.radius !== undefined) {
            type = OBJ.sphere; mat = matOf(o.material); g(o.center.x, o.center.y, o.center.z, o.radius);
        } else if (o.point !== undefined && o.normal !== undefined) {
            type = OBJ.plane; mat = matOf(o.material); g(o.point.x, o.point.y, o.point.z, o.normal.x, o.normal.y, o.normal.z);
        } else if (o.min !== undefined && o.max !== undefined) {
            type = OBJ.box; mat = matOf(o.material); g(o.min.x, o.min.y, o.min.z, o.max.x, o.max.y, o.max.z);
        } else {
            throw new Error(`world.objects[${i}]: unsupported object`);
        }
        const ii = i * (OBJECT_BYTES / 4);
        oi[ii] = type; oi[ii + 1] = mat; oi[ii + 2] = first; oi[ii + 3] = count;
    }
    const materials = new ArrayBuffer(MATERIAL_BYTES * Math.max(1, mats.length));
    const mi = new Int32Array(materials), mf = new Float64Array(materials);
    for (let i = 0; i < mats.length; i++) {
        const m = mats[i], b = i * (MATERIAL_BYTES / 8);
        mi[2 * b] = m.type;
        const al = m.albedo || [0, 0, 0], em = m.emit || [0, 0, 0];
        mf[b + 1] = al[0]; mf[b + 2] = al[1]; mf[b + 3] = al[2];
        mf[b + 4] = m.roughness || 0;
        mf[b + 5] = m.ior || 0;
        mf[b + 6] = em[0]; mf[b + 7] = em[1]; mf[b + 8] = em[2];
    }
    const c = camera;
    const cam = new Float64Array(22);
    [c.origin, c.lowerLeftCorner, c.horizontal, c.vertical, c.u, c.v, c.w].forEach((v, j) => cam.set([v.x, v.y, v.z], 3 * j));
    cam[21] = c.lensRadius;
    const bg = backgroundOf(world);
    return {
        objects: new Uint8Array(objects),
        materials: new Uint8Array(materials, 0, MATERIAL_BYTES * mats.length),
        triangles: tris.subarray(0, ntri * 12),
        camera: cam,
        cameraType: c.type === 'orthographic' ? 1 : 0,        // getRay branches on === 'orthographic'
        background: bg.code,
        skyIntensity: world.skyIntensity,
        solidColor: new Float64Array(bg.solid),
        perm: Int32Array.from(world.cloudNoise.p),
    };
}
