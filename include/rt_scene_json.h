/*
 * rt_scene_json.h — scene-JSON loader of librt_hip.so (host code, no GPU needed).
 *
 * Replaces, for hosts without Node (the C++ bench CLI, C/C++ embedders):
 *   RayTracer.prototype.loadFromJSON(jsonData)      js/ray-tracer.js:304-333
 *     -> SceneLoader.loadFromJSON / _createObject / _createMaterial / _createCamera / _parseVec3
 *                                                  js/scene-loader.js:20-284
 *     -> RayTracer.resizeCanvas + setupCamera on a camera "resolution" entry
 *                                                  js/ray-tracer.js:319-326, 439-474, 598-614
 *     -> new World() (its PerlinNoise permutation)  js/world.js:8-16, js/noise.js:6-18
 * and packs the result into the rt_scene_desc of rt_hip.h, with the same JavaScript value
 * semantics (`||` defaults, `!== undefined` defaults, ToNumber of null/booleans, Math.min on the
 * metal roughness, Plane normal normalization, TriangleMesh index validation).  Lights are parsed by
 * the reference but never used by render(), so they are ignored.  Without a "camera" entry the
 * RayTracer keeps its constructor camera (ray-tracer.js:42-77: (3,2,2) -> (0,0,-1), fov 45,
 * aspect W/H, aperture 0, focus 10), which is what the loader returns then.
 * Like the reference's loadFromJSON (which catches and returns false), malformed input returns
 * RT_ERR_INVALID with rt_last_error() describing it.
 */
#ifndef RT_SCENE_JSON_H
#define RT_SCENE_JSON_H

#include "rt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Owns the arrays its rt_scene_desc points into. */
typedef struct rt_json_scene rt_json_scene;

/* Parse `len` bytes of scene JSON for a RayTracer of width x height whose World permutation comes
 * from the keyed stream of `seed`.  On success *out owns the packed scene. */
int rt_json_scene_load(const char* json, size_t len, int32_t width, int32_t height, uint32_t seed,
                       rt_json_scene** out);

/* The packed scene, valid until rt_json_scene_destroy. */
const rt_scene_desc* rt_json_scene_desc(const rt_json_scene* scene);

/* The RayTracer's width/height after loading (changed by a camera "resolution" entry). */
void rt_json_scene_size(const rt_json_scene* scene, int32_t* width, int32_t* height);

void rt_json_scene_destroy(rt_json_scene* scene);

#ifdef __cplusplus
}
#endif

#endif /* RT_SCENE_JSON_H */
