/*
 * rt_hip.h — C ABI of the MI355X path-tracing backend (librt_hip.so).
 *
 * Drop-in boundary for the per-pixel path-tracing loop of Shinzef/BlenderRayTracer:
 *   RayTracer.prototype.render(onProgress)            js/ray-tracer.js:166-281
 *     -> rayColor(ray, depth)                          js/ray-tracer.js:102-123
 *     -> World.hit / background                        js/world.js:20-110
 *     -> Sphere/Plane/Box/Triangle/TriangleMesh.hit    js/geometry.js:15-262
 *     -> Lambertian/Metal/Dielectric/Emissive          js/materials.js:14-96
 *     -> Camera.getRay                                 js/camera.js:38-51
 *     -> toneMap / gammaCorrect epilogue               js/ray-tracer.js:151-165, post-processor.js:9-42
 * The host (JS GpuRayTracer over N-API, or Python over ctypes) packs the reference's duck-typed
 * World/Camera objects into the plain arrays below; everything under render() runs on the GPU.
 *
 * Conventions: plain C types, caller owns every host buffer, the library owns device buffers.
 * Every int-returning entry point returns 0 on success and a negative rt_status on failure;
 * rt_last_error() then holds a thread-local message.  No C++ exception crosses this ABI.
 * Randomness: the keyed counter RNG documented in DESIGN.md §RNG replaces Math.random().
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3      /* 2: rt_settings.device_count / devices (multi-GPU sample split)
                                 3: rt_settings.sum_order, rt_output.preview_rgba8, rt_closest_hits */

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,     /* bad argument / descriptor */
    RT_ERR_DEVICE = -2,      /* HIP runtime error */
    RT_ERR_NOMEM = -3,
    RT_ERR_CANCELLED = -4,   /* rt_cancel() / progress() stopped the render before its last sample */
    RT_ERR_NO_DEVICE = -5    /* no HIP device visible: the backend never falls back to the CPU */
} rt_status;

/* World object kinds, in the reference's World.objects insertion order (js/world.js:20-33). */
typedef enum rt_object_type {
    RT_OBJ_SPHERE = 0,    /* geometry.js:15-45   g = {cx, cy, cz, radius}                     */
    RT_OBJ_PLANE = 1,     /* geometry.js:56-74   g = {px, py, pz, nx, ny, nz} (n normalized)  */
    RT_OBJ_BOX = 2,       /* geometry.js:85-132  g = {minx, miny, minz, maxx, maxy, maxz}     */
    RT_OBJ_TRIANGLE = 3,  /* geometry.js:148-188 one world object = triangles[first]          */
    RT_OBJ_MESH = 4       /* geometry.js:248-262 triangles[first .. first+count), last tie wins */
} rt_object_type;

typedef enum rt_material_type {
    RT_MAT_LAMBERTIAN = 0, /* materials.js:14-26 */
    RT_MAT_METAL = 1,      /* materials.js:29-42 */
    RT_MAT_DIELECTRIC = 2, /* materials.js:45-84 */
    RT_MAT_EMISSIVE = 3    /* materials.js:87-96 */
} rt_material_type;

typedef enum rt_background_type {
    RT_BG_GRADIENT = 0,        /* World.skyGradient      world.js:35-40  */
    RT_BG_SOLID = 1,           /* World.solidBackground  world.js:42-44 (updateBackground form) */
    RT_BG_HDRI = 2,            /* World.hdriBackground   world.js:74-110 (updateBackground form) */
    RT_BG_PROCEDURAL_SKY = 3,  /* World.proceduralSky    world.js:46-72  */
    RT_BG_NAN = 4              /* JSON "solid"/"hdri": the loader binds a factory, radiance is NaN
                                  (scene-loader.js:41-45) */
} rt_background_type;

#define RT_MAX_DEVICES 8

typedef enum rt_camera_type { RT_CAM_PERSPECTIVE = 0, RT_CAM_ORTHOGRAPHIC = 1 } rt_camera_type;
/* getAntiAliasSample (ray-tracer.js:125-149): any string other than 'stochastic' and
 * 'supersampling' samples the pixel centre (RT_AA_CENTER) */
typedef enum rt_aa_mode { RT_AA_SUPERSAMPLING = 0, RT_AA_STOCHASTIC = 1, RT_AA_CENTER = 2 } rt_aa_mode;
typedef enum rt_tone_map { RT_TM_REINHARD = 0, RT_TM_ACES = 1, RT_TM_LINEAR = 2 } rt_tone_map;

/* Arithmetic of the path kernel.  F64 is the reference's own arithmetic (JS numbers are IEEE
 * binary64, no FMA contraction): ray paths agree with the reference decision for decision.
 * F32 is the fast mode; its per-channel RMS vs the reference is measured in tests. */
typedef enum rt_precision { RT_PREC_F64 = 0, RT_PREC_F32 = 1 } rt_precision;

/* World.hit evaluation.  BRUTE walks World.objects in order (world.js:24-30); BVH walks one bounding
 * volume hierarchy over the spheres and one over the triangles (built by rt_scene_create) with the
 * same tie-breaking, so both give bit-identical renders.  AUTO picks BVH for large scenes. */
typedef enum rt_accel { RT_ACCEL_AUTO = 0, RT_ACCEL_BRUTE = 1, RT_ACCEL_BVH = 2 } rt_accel;

/* Order in which a pixel's sample radiances are added into its binary64 sum (the reference adds them
 * in sample order, ray-tracer.js:202-208).  Every path decision, segment and draw count is the same in
 * both; only the rounding of the binary64 sums differs (~1e-16 relative).
 *   RT_SUM_POOL (default, fastest): the sample pool adds a tile's samples in the order its wave
 *     finishes them, then the chunk partials in chunk order.  Deterministic (the same render reproduces
 *     its bits), but an RGBA8 byte can differ from a sample-order sum by one at a floor(c*255) boundary.
 *   RT_SUM_SAMPLE_ORDER: one lane per pixel adds samples [sample_begin, sample_end) in sample order,
 *     exactly the reference's loop order (slower: DESIGN.md §4). */
typedef enum rt_sum_order { RT_SUM_POOL = 0, RT_SUM_SAMPLE_ORDER = 1 } rt_sum_order;

typedef struct rt_material_desc {
    int32_t type;          /* rt_material_type */
    int32_t _pad;
    double albedo[3];      /* Lambertian / Metal albedo */
    double roughness;      /* Metal: already Math.min(roughness, 1) (materials.js:33) */
    double ior;            /* Dielectric refractionIndex */
    double emission[3];    /* Emissive: color.mul(intensity) (materials.js:95), evaluated in double */
} rt_material_desc;        /* 72 bytes */

typedef struct rt_object_desc {
    int32_t type;          /* rt_object_type */
    int32_t material;      /* index into rt_scene_desc.materials */
    int32_t first;         /* TRIANGLE / MESH: first triangle */
    int32_t count;         /* TRIANGLE: 1; MESH: number of triangles (may be 0) */
    double g[6];           /* geometry, see rt_object_type */
} rt_object_desc;          /* 64 bytes */

typedef struct rt_camera_desc {  /* vectors exactly as js/camera.js:8-36 computes them */
    double origin[3];
    double lower_left[3];
    double horizontal[3];
    double vertical[3];
    double u[3], v[3], w[3];
    double lens_radius;
    int32_t type;          /* rt_camera_type ("orthographic" => normalized, focal length 1) */
    int32_t _pad;
} rt_camera_desc;

typedef struct rt_scene_desc {
    int32_t abi_version;                 /* RT_ABI_VERSION */
    int32_t num_objects;
    const rt_object_desc* objects;
    int32_t num_materials;
    int32_t num_triangles;
    const rt_material_desc* materials;
    const double* triangles;             /* 12 doubles each: v0, v1, v2, unit geometric normal
                                            normalize(cross(v1-v0, v2-v0)) (geometry.js:143-145) */
    rt_camera_desc camera;
    int32_t background;                  /* rt_background_type */
    int32_t _pad;
    double sky_intensity;                /* World.skyIntensity */
    double solid_color[3];               /* RT_BG_SOLID color (updateBackground uses 0.1,0.1,0.1) */
    int32_t perm[512];                   /* World.cloudNoise.p (noise.js:6-18) */
} rt_scene_desc;

typedef struct rt_settings {
    int32_t width, height;     /* full image; pixel key p = (H-1-j)*W + i (ray-tracer.js:215) */
    int32_t samples;           /* sampleCount of ray-tracer.js:201, resolved by the host:
                                  1 for antiAliasing 'none', else this.samples */
    int32_t max_depth;         /* this.maxBounces */
    int32_t aa_mode;           /* rt_aa_mode */
    int32_t tone_map;          /* rt_tone_map */
    double exposure;
    double gamma;
    uint32_t seed;             /* keyed RNG seed */
    int32_t sample_begin;      /* render samples [sample_begin, sample_end) of every pixel   */
    int32_t sample_end;        /* <= 0 means sampleCount                                       */
    int32_t crop_x0, crop_y0;  /* output window (top-down rows), crop_w/h == 0 -> full image   */
    int32_t crop_w, crop_h;
    int32_t precision;         /* rt_precision */
    int32_t batch_samples;     /* samples per launch (progress/cancel granularity); 0 = all;
                                  -N = about N batches, each a multiple of the sample pool's chunk
                                  (the Node drop-in's default, -16)                               */
    int32_t denoise;           /* this.denoising: PostProcessor.denoise after gamma (ray-tracer.js:266-276);
                                  needs the full frame (crop_w/h = 0 or the whole image) */
    double denoise_weights[2]; /* Math.exp(-1/(2s*s)), Math.exp(-2/(2s*s)), s = denoiseStrength, evaluated by
                                  the host with its own exp (post-processor.js:55) */
    int32_t accel;             /* rt_accel: how World.hit is evaluated (results are identical) */
    int32_t device_count;      /* 0 or 1: the scene's own device.  N in 2..RT_MAX_DEVICES:
                                  with the sample pool (sum_order RT_SUM_POOL), WHOLE sample batches are
                                  dealt round-robin — batch k traced on devices[k % N] — and each batch's
                                  chunk partials are copied to the scene's device and added there in
                                  batch order, so the sums are bit-identical to the same batches on one
                                  device (checkpoint/resume unchanged).  The batch size is then
                                  min(batch_samples, ceil((samples - sample_begin) / N)) so that every
                                  device gets work; batch_samples = 0 gives N batches.  With
                                  RT_SUM_SAMPLE_ORDER (or when the partial slots do not fit) every batch is
                                  instead split into N contiguous sample ranges, range k on devices[k],
                                  their sums added on the scene's device in range order (equal to one
                                  device up to the order of those additions).  A device may be listed more
                                  than once (its batches run on separate streams).  The scene is uploaded
                                  to each listed device on first use and kept. */
    int32_t devices[8];        /* HIP ordinals of the devices (device_count of them).  Peer access to the
                                  scene's device is enabled where the topology has it; without it the
                                  copies are staged through host memory (reported once on stderr) */
    int32_t sum_order;         /* rt_sum_order */
} rt_settings;

/* Host outputs of rt_render, each optional (NULL = not wanted). n = crop_w*crop_h pixels,
 * top-down row-major like imageData. */
typedef struct rt_output {
    double* mean;          /* n*3: per-pixel linear mean, the toneMap() input (ray-tracer.js:208) */
    float* post;           /* n*4: post-gamma floats + alpha 1.0 (the floatData of ray-tracer.js:216-219);
                              with denoise: the denoised floats the RGBA8 bytes are made from */
    uint8_t* rgba8;        /* n*4: min(255,max(0,floor(c*255))), NaN -> 0, alpha 255 (ray-tracer.js:226-252) */
    uint32_t* segments;    /* n: world.hit calls per pixel (diagnostic; enables device counting) */
    uint32_t* draws;       /* n: RNG draws per pixel (diagnostic) */
    uint8_t* preview_rgba8;   /* n*4, progressive display (ray-tracer.js:224-241 putImageData per row): with
                                 more than one sample batch, before every progress() call this buffer holds
                                 the RGBA8 frame of the samples traced so far (mean over those samples, tone
                                 map, gamma; no denoise, like the reference's rows before its final pass;
                                 the gamma pow of these running frames is binary32, so a pixel within ~1e-7 of
                                 an RGBA8 rounding boundary may differ by one step from rgba8's exact frame).
                                 After a cancel the buffer holds the exact frame of the checkpointed samples.  A batch
                                 whose successor has already finished when the host gets to it is skipped
                                 (the buffer keeps the previous frame until the newer one is copied) */
    int32_t* preview_samples; /* optional out: the samples (from sample_begin) in preview_rgba8's frame,
                                 updated with it */
} rt_output;

typedef struct rt_stats {
    double kernel_ms;            /* device time of the path-tracing launches (HIP events on the device's
                                    accumulation stream, from the render's set-up to its last batch's
                                    merge; the maximum over devices).  With several batches and a
                                    progress callback this includes any time the GPU waited for the host */
    double finalize_ms;          /* device time of the epilogue */
    double wall_ms;              /* host wall time of the call */
    uint64_t samples;            /* pixels x samples traced */
    uint64_t segments;           /* world.hit calls (ray segments) */
    uint64_t prim_tests;         /* primitives tested: segments x primitives (brute force), counted (BVH) */
    double algorithmic_bytes;    /* SURVEY §8(d) record bytes the tests read + 12 B/pixel framebuffer:
                                    brute force: segments x sum of primitive record bytes;
                                    BVH: 64 B/node visited + 16 B/sphere + 36 B/triangle tested
                                    + segments x 24 B per plane and box */
    uint64_t node_visits;        /* BVH nodes visited (0 for brute force) */
    uint64_t sphere_tests;       /* BVH: sphere / triangle tests in visited leaves (0 for brute force) */
    uint64_t tri_tests;
} rt_stats;

typedef struct rt_scene rt_scene;   /* opaque: scene resident in HBM of one device */

/* Library / device info. */
int rt_abi_version(void);
const char* rt_last_error(void);
int rt_device_count(int* count);

/* Scene lifetime: copies the descriptor into device memory of `device` (HIP ordinal). */
int rt_scene_create(const rt_scene_desc* desc, int device, rt_scene** out);
void rt_scene_destroy(rt_scene* scene);

/* Full render into host buffers: trace, finalize (tone map, gamma, RGBA8) and copy back.
 * Replaces RayTracer.render (ray-tracer.js:166-281) minus the DOM. Synchronous.
 * progress(fraction, user) is called between sample batches from the calling thread; a non-zero
 * return value cancels (like window.renderCancelled, ray-tracer.js:190,196), as does rt_cancel from any
 * thread.  Batches are pipelined: on one device (up to 64 batches whose partials fit RT_FUSED_MB) all
 * of them are traced by ONE launch and each batch is added as soon as its last item is done; otherwise
 * up to 3 per device are queued on the GPU beyond the one the host waits for.  With the sample pool and
 * several batches a cancel stops the batches at their next 8x8 tile x sample-chunk item: the persistent
 * (LDS) pool launches read no cancel word — rt_cancel moves each in-flight launch's work queue past its
 * last item from a high-priority stream, so every wave's next take ends its loop and only the items
 * already taken finish (about 7 ms to return on config 3) — and the one-wave pool kernel's workgroups
 * read the cancel word as they start.  The render returns once the GPU has drained; the checkpoint holds
 * the batches fully added before that.  Otherwise (sample order, one batch, partials that do not fit)
 * it is observed between batches and the queued ones complete.
 * RT_ERR_CANCELLED unless every sample was traced.
 * Threading: one call in flight per scene (rt_render, rt_render_resume, rt_trace_device,
 * rt_finalize_device, rt_render_checkpoint), as for the reference's render(); calls on different
 * scenes may run concurrently from different threads.  Asynchronous device calls on different streams
 * are ordered by the scene itself (its scratch buffers are event-guarded). */
typedef int (*rt_progress_fn)(double fraction, void* user);
int rt_render(rt_scene* scene, const rt_settings* settings, const rt_output* out,
              rt_progress_fn progress, void* user, rt_stats* stats);

/* Progressive rendering (the reference's row-by-row progress, ray-tracer.js:258-261,
 * at sample granularity).  After rt_render / rt_render_resume returns — finished or cancelled
 * (RT_ERR_CANCELLED; the checkpoint is always a whole number of batches) — the scene holds the per-pixel float64 radiance sums
 * of samples [sample_begin, samples_done).  rt_render_checkpoint copies them out (count must be
 * 3 x crop pixels) so a host can persist them; rt_render_resume traces samples
 * [samples_done, sample_end) on top of such sums and finishes like rt_render.  Every pixel still
 * adds its samples in order, so a resumed render is bit-identical to an uninterrupted one.
 * Resident checkpoints (no host copy of the sums): rt_render_checkpoint(scene, NULL, 0, &done)
 * returns only samples_done, and rt_render_resume(..., sums = NULL, samples_done, ...) continues from
 * the sums the scene still holds on its device — valid until the scene's next render (the call fails
 * with RT_ERR_INVALID unless samples_done, the frame size, the crop window, sample_begin, precision,
 * seed, aa_mode and max_depth are the checkpoint's; a render that fails before its sums are consistent
 * leaves no checkpoint). */
int rt_render_checkpoint(rt_scene* scene, double* sums, size_t count, int32_t* samples_done);
int rt_render_resume(rt_scene* scene, const rt_settings* settings, const double* sums, int32_t samples_done,
                     const rt_output* out, rt_progress_fn progress, void* user, rt_stats* stats);

/* Device-level building blocks for multi-GPU (one process per GPU): trace samples
 * [sample_begin, sample_end) and ADD per-pixel radiance sums into d_sum (device, n*3 doubles,
 * caller zeroes it); segment counting goes to stats.  Asynchronous on `hip_stream`
 * (a hipStream_t, NULL = default stream); stats are filled after the stream is synchronized
 * when `sync` is non-zero. */
int rt_trace_device(rt_scene* scene, const rt_settings* settings, double* d_sum, void* hip_stream,
                    int sync, rt_stats* stats);

/* rt_trace_device with the frame delivered band by band, so a multi-GPU caller can reduce the first
 * bands across GPUs while the later ones still trace.  The crop's 8-pixel tile rows are
 * split into `bands` horizontal bands (at most 64 and the tile rows); the trace runs on the scene's own
 * stream (after the caller's work on `hip_stream` so far) with its work items band-major, and as soon as
 * band b's items are done its sums are added into d_sum on `hip_stream` and band_ready(b, row0, rows,
 * user) is called from this thread: the caller may enqueue work on rows [row0, row0 + rows) of d_sum on
 * hip_stream (or a stream that waits for it), which runs beside the later bands' trace.  A non-zero return
 * stops the delivery (RT_ERR_CANCELLED; the trace itself completes).  Returns once every band was
 * delivered and hip_stream has been ordered after the whole trace.  d_sum ends up equal to
 * rt_trace_device's, bit for bit (same work items, same chunk partials, same order of additions). */
typedef int (*rt_band_fn)(int32_t band, int32_t row0, int32_t rows, void* user);
int rt_trace_device_bands(rt_scene* scene, const rt_settings* settings, double* d_sum, void* hip_stream, int32_t bands,
                          rt_band_fn band_ready, void* user, rt_stats* stats);

/* Epilogue on device: mean = sum / sampleCount, toneMap, gammaCorrect, optional denoise, RGBA8
 * (ray-tracer.js:208-276).  Any output pointer may be NULL.  All pointers are device pointers; the
 * scene provides the scratch buffer the denoise pass reads from. */
int rt_finalize_device(rt_scene* scene, const rt_settings* settings, const double* d_sum, double* d_mean,
                       float* d_post, uint8_t* d_rgba8, void* hip_stream);

/* Diagnostic (tests): World.hit for `n` rays on the scene's device — the device arithmetic of the
 * trace kernel's closest-hit stage (brute force in World.objects order, or the BVH walk), so the
 * BVH's bit-identity proof is checked on the instructions the GPU runs.  rays: host, n x 6 doubles
 * (origin xyz, direction xyz; rounded to binary32 first in RT_PREC_F32).  Outputs (host, n each, any may
 * be NULL): t (binary64 of the winning parameter, +inf when nothing is hit), kind (-1 none, 0 sphere,
 * 1 plane, 2 box, 3 triangle), index (primitive index within its kind, in World.objects order; mesh
 * triangles in mesh order). */
int rt_closest_hits(rt_scene* scene, int32_t precision, int32_t accel, const double* rays, size_t n,
                    double* t, int32_t* kind, int32_t* index);

/* Diagnostic: the walk a render with these precision / accel settings runs on this scene — 0 World.objects
 * order (brute force), 1 a BVH tree walk, 2 the uniform grid over the spheres (sphere-only scenes where
 * the host's sampled cost estimate prefers it, scene_pack.h choose_walk); < 0 an error status.  Every
 * walk finds the same closest hit; they differ in speed only. */
int rt_scene_walk(rt_scene* scene, int32_t precision, int32_t accel);

/* Request cancellation of an in-flight rt_render on `scene` (the pool kernels read it between items;
 * see rt_render). */
int rt_cancel(rt_scene* scene);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
