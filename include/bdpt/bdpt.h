/* include/bdpt/bdpt.h — C-ABI of the MI355X-native BDPT hot path (libbdpt_amd.so).
 *
 * Drop-in boundary for the reference's per-pixel BDPT loop:
 *   reference interface                          replaced by
 *   PathTracer::set_frame_size   pathtracer.h:36  -> bdpt_create (frame size in bdpt_params)
 *   PathTracer::clear            pathtracer.h:43  -> bdpt_clear
 *   PathTracer::raytrace_pixel   pathtracer.h:69  -> bdpt_render over a 1x1 tile
 *     (BidirectionalPathTracer::raytrace_pixel, src/pathtracer/bidirection.cpp:503-542)
 *   RaytracedRenderer::raytrace_tile             -> bdpt_render over a list of tiles
 *     (src/pathtracer/raytraced_renderer.cpp:595-620)
 *   BidirectionalPathTracer::{sampleBuffer, eyeBuffer, lightBuffer}
 *     (bidirection.h:81, pathtracer.h:90)         -> bdpt_read_frame (BDPT_FRAME_*)
 *   RaytracedRenderer::set_scene / build_accel    -> bdpt_create (scene desc; the BVH is built
 *     (raytraced_renderer.cpp:105-127,350-374)       inside: the reference's midpoint-split tree,
 *                                                    bvh.cpp:51-129, for its DFS leaf order (the
 *                                                    equal-t tie key), and a binned-SAH device tree
 *                                                    over the same primitives)
 *
 * Threading: one ctx per GPU. Every entry point taking a ctx locks it, so the reference's model of
 * N worker threads calling raytrace_pixel / raytrace_tile on one PathTracer
 * (raytraced_renderer.cpp:325-327,610-615) is safe; the calls are serialised per ctx.
 *
 * Plain C types only: no torch, no HIP types in any signature (a stream is passed as void*).
 * Every call returns 0 (BDPT_OK) or a negative BDPT_E_* code; bdpt_last_error() gives the text.
 * No C++ exception crosses this boundary. Unsupported features that the reference can only
 * assert(0) on under BDPT (microfacet sample_pdf, advanced_bsdf.cpp:144-148; directional / spot /
 * sphere / mesh lights, light.cpp:25-51,168-194) are rejected at bdpt_create with
 * BDPT_E_UNSUPPORTED instead of aborting.
 *
 * Extensions beyond what the reference can run (semantics in DESIGN.md §9):
 *   - the environment light under BDPT (the reference's EnvironmentLight has sample_L / sample_dir
 *     but asserts in sample_Le / sample_Le_point / sample_pdf / contain_point,
 *     environment_light.cpp:182-208): bdpt_scene_desc.envmap, loaded by bdpt_exr_load (-e);
 *   - Russian roulette on both subpaths through PathVertex.q (bidirection.h:36, the rule commented
 *     out at bidirection.cpp:87-93): bdpt_params.russian_roulette.
 * And the reference's second integrator: the unidirectional PathTracer
 * (pathtracer.cpp:47-340 — NEE, adaptive sampling, thin lens, roulette at -m 0, the environment
 * light, MicrofacetBSDF), selected by bdpt_params.integrator = BDPT_INTEGRATOR_PT (ABI v3).
 */
#ifndef BDPT_AMD_BDPT_H
#define BDPT_AMD_BDPT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BDPT_ABI_VERSION 9

enum bdpt_status {
  BDPT_OK = 0,
  BDPT_E_INVALID = -1,      /* bad argument / malformed scene */
  BDPT_E_UNSUPPORTED = -2,  /* feature the reference BDPT cannot run (see header comment) */
  BDPT_E_DEVICE = -3,       /* HIP runtime error (no device, launch failure, ...) */
  BDPT_E_NOMEM = -4
};

/* Primitive kinds (src/scene/triangle.h, src/scene/sphere.h). */
enum bdpt_prim_type { BDPT_PRIM_TRIANGLE = 0, BDPT_PRIM_SPHERE = 1 };

/* BSDF kinds (src/pathtracer/bsdf.h:117-306). */
enum bdpt_mat_type {
  BDPT_MAT_DIFFUSE = 0,     /* a = reflectance                                  bsdf.cpp:52-85   */
  BDPT_MAT_EMISSION = 1,    /* a = radiance                                     bsdf.cpp:99-118  */
  BDPT_MAT_MIRROR = 2,      /* a = reflectance                          advanced_bsdf.cpp:17-35   */
  BDPT_MAT_GLASS = 3,       /* a = reflectance, b = transmittance, ior  advanced_bsdf.cpp:198-259 */
  BDPT_MAT_REFRACTION = 4,  /* b = transmittance, ior                   advanced_bsdf.cpp:163-184 */
  BDPT_MAT_MICROFACET = 5   /* rejected: sample_pdf asserts under BDPT  advanced_bsdf.cpp:144-148 */
};

/* Light kinds (src/scene/light.h). Only area and point lights have BDPT methods in the reference;
 * the environment light comes in through bdpt_scene_desc.envmap, never through this list. */
enum bdpt_light_type {
  BDPT_LIGHT_AREA = 0, BDPT_LIGHT_POINT = 1,
  BDPT_LIGHT_OTHER = 2,       /* spot: rejected (SpotLight::sample_L leaves its outputs unset,
                                 light.cpp:163-166)                                            */
  BDPT_LIGHT_HEMISPHERE = 3,  /* an ambient light = InfiniteHemisphereLight (light.cpp:55-70):
                                 PathTracer only (BDPT: sample_Le asserts, :72-77)             */
  BDPT_LIGHT_DIRECTIONAL = 4  /* DirectionalLight (light.cpp:11-23): `direction` = dirToLight, the
                                 unit world direction towards the light; PathTracer only        */
};

typedef struct bdpt_material {
  int32_t type;
  double a[3];
  double b[3];
  double ior;
  double roughness;
} bdpt_material;

typedef struct bdpt_light {
  int32_t type;
  double radiance[3];
  double position[3];
  double direction[3];  /* area: unit emitting normal                                */
  double dim_x[3];      /* area: rectangle edge vectors (light.cpp:199-203)          */
  double dim_y[3];
  double area;          /* |dim_x| * |dim_y|                                         */
} bdpt_light;

/* Pinhole camera state after Camera::configure/place/set_screen_size (camera.cpp:29-147). */
typedef struct bdpt_camera {
  double pos[3];
  double c2w[9];        /* column-major: c2w[3*col + row] (CGL Matrix3x3 columns)     */
  double w2c[9];        /* = c2w.inv() as the reference computes it                    */
  double hfov_deg;
  double vfov_deg;
  double nclip;
  double fclip;
} bdpt_camera;

/* The HDRImageBuffer of an environment map (main.cpp:40-77 load_exr; data[w*j + i], row j = 0 at
 * theta = 0, i.e. +y): EnvironmentLight(envMap) (environment_light.cpp:6-62). */
typedef struct bdpt_envmap {
  int32_t width, height;
  const float* rgb;           /* width*height*3                                          */
} bdpt_envmap;

/* Scene in the reference's primitive order (objects in scene order, faces in mesh order:
 * RaytracedRenderer::build_accel, raytraced_renderer.cpp:350-374). The BVH is built from it. */
typedef struct bdpt_scene_desc {
  int32_t nprim;
  const int32_t* prim_type;   /* nprim, bdpt_prim_type                                   */
  const double* prim_geom;    /* nprim*18: triangle p1,p2,p3,n1,n2,n3; sphere c[3],r,... */
  const int32_t* prim_mat;    /* nprim, index into mats                                  */
  int32_t nmat;
  const bdpt_material* mats;
  int32_t nlight;
  const bdpt_light* lights;
  bdpt_camera camera;
  /* NULL = none. Otherwise an EnvironmentLight appended after `lights` (the renderer pushes
   * pt->envLight onto scene->lights last, raytraced_renderer.cpp:117-119). ABI v2. */
  const bdpt_envmap* envmap;
} bdpt_scene_desc;

/* Random-number semantics of the device path: Philox4x32-10 keyed by seed, counter
 * (pixel = x + y*W, global sample index, block, 0xB1D1). See DESIGN.md §RNG. */
typedef struct bdpt_params {
  int32_t width;              /* frame size (PathTracer::set_frame_size)                 */
  int32_t height;
  int32_t spp;                /* ns_aa: the 1/ns_aa weight of every sample                */
  int32_t max_depth;          /* max_ray_depth (-m); BDPT: 0..62, PathTracer: 0..21      */
  uint64_t seed;
  int32_t samples_per_lane;   /* 0 = auto                                                 */
  int32_t device;             /* HIP device ordinal                                       */
  int32_t collect_stats;      /* 1 = kernel also counts node/prim tests (roofline bytes)  */
  int32_t pipeline;           /* 0 = auto = 1, the megakernel; 2 (the wavefront pipeline) was
                                 retired in round 5: BDPT_E_UNSUPPORTED                      */
  int32_t russian_roulette;   /* 1 = PathVertex.q roulette on both subpaths (ABI v2)       */
  /* ABI v3: the integrator and the PathTracer's settings (PathTracer fields, pathtracer.h:73-85;
   * CLI -l -a -H -b -d, main.cpp:107-141; AppConfig defaults application.h:45-65) */
  int32_t integrator;         /* BDPT_INTEGRATOR_BDPT (0, the reference's) / _PT (1)         */
  int32_t ns_area_light;      /* -l: samples per area light (0 = 1)                          */
  int32_t samples_per_batch;  /* -a batch: adaptive sampling batch (0 = 32)                  */
  float max_tolerance;        /* -a tol: stop when 1.96 sigma / sqrt(n) <= tol * mean        */
  int32_t direct_hemisphere_sample;  /* -H: hemisphere instead of light sampling            */
  double lens_radius;         /* -b (0: pinhole)                                             */
  double focal_distance;      /* -d (0 = 4.7)                                                */
  int32_t reserved[4];
} bdpt_params;

enum bdpt_integrator { BDPT_INTEGRATOR_BDPT = 0, BDPT_INTEGRATOR_PT = 1 };

typedef struct bdpt_tile {
  int32_t x0, y0, w, h;       /* clipped to the frame like raytrace_tile does            */
} bdpt_tile;

enum bdpt_frame { BDPT_FRAME_SAMPLE = 0, BDPT_FRAME_EYE = 1, BDPT_FRAME_LIGHT = 2 };

typedef struct bdpt_stats {
  uint64_t samples;           /* pixel-samples rendered since the last clear            */
  uint64_t rays;              /* closest-hit + connection queries                        */
  uint64_t closest_rays;      /* walk rays (closest hit)                                 */
  uint64_t shadow_rays;       /* connection rays (any hit)                               */
  uint64_t node_visits;       /* AABBs fetched                                            */
  uint64_t tri_tests;
  uint64_t sph_tests;
  uint64_t hits;              /* closest-hit queries that hit (shading record fetched)   */
  double last_kernel_ms;      /* duration of the last bdpt_render's kernels (hipEvents)  */
  uint64_t bvh_nodes;
  uint64_t bvh_depth;
  /* ABI v4: where the scene reads of the last launches were served from */
  uint64_t lds_node_visits;   /* of node_visits: AABBs read from the CU's LDS copy          */
  int32_t lds_mode;           /* 0 scene in HBM, 1 whole scene in LDS, 2 BFS treelet in LDS +
                                 HBM below it, 3 flat primitive list in LDS; -1 none yet     */
  int32_t reserved0;
  /* ABI v6: environment-light table reads, counted like the scene reads above */
  uint64_t env_samples;       /* importance-sampled directions: 2 guide cells + 2 CDF entries per
                                 axis, the texel pdf, 4 texels (76 B)                          */
  uint64_t env_lookups;       /* radiance lookups along a direction: 4 texels (48 B)          */
  uint64_t env_pdf_lookups;   /* texel pdf lookups (4 B)                                      */
} bdpt_stats;

int bdpt_abi_version(void);
const char* bdpt_last_error(void);

/* Builds the BVH, flattens it, deep-copies the scene to HBM. The caller may free its arrays
 * after this returns. */
int bdpt_create(const bdpt_scene_desc* scene, const bdpt_params* params, void** ctx_out);
void bdpt_destroy(void* ctx);

/* All later work is enqueued on `stream` (a hipStream_t; NULL = the ctx's own stream). */
int bdpt_set_stream(void* ctx, void* stream);

/* Zeroes the frame buffers and counters (PathTracer::clear / set_frame_size). Async. */
int bdpt_clear(void* ctx);

/* Renders global sample indices [spp_begin, spp_begin+spp_count) of every pixel of the tiles.
 * Asynchronous on the ctx stream. ntiles == 0 or tiles == NULL means the whole frame. The
 * PathTracer renders whole pixels (its adaptive sampling decides per pixel): spp_begin must be 0
 * and spp_count the ctx's spp; shard its work across GPUs by tiles. */
int bdpt_render(void* ctx, const bdpt_tile* tiles, int32_t ntiles, int32_t spp_begin,
                int32_t spp_count);

int bdpt_sync(void* ctx);

/* Copies a W*H*3 float frame (row 0 = bottom, as HDRImageBuffer) to host memory (sync). Under
 * the PathTracer, BDPT_FRAME_SAMPLE is its sampleBuffer (per-pixel means, update_pixel). */
int bdpt_read_frame(void* ctx, int32_t which, float* rgb);

/* ABI v8: the pixels [x0, x0 + w) x [y0, y0 + h) of a frame as w*h*3 floats, row 0 = y0 (sync):
 * what a per-tile caller copies into sampleBuffer after raytrace_tile (the renderer reads the
 * whole sampleBuffer through the non-virtual write_to_framebuffer after every tile,
 * raytraced_renderer.cpp:619, pathtracer.cpp:42-45). The rectangle must lie inside the frame. */
int bdpt_read_frame_rect(void* ctx, int32_t which, int32_t x0, int32_t y0, int32_t w, int32_t h, float* rgb);

/* PathTracer::sampleCountBuffer (pathtracer.h:94): W*H samples per pixel, row 0 = bottom (sync).
 * Under BDPT every rendered pixel reports the samples rendered for it. */
int bdpt_read_sample_counts(void* ctx, int32_t* counts);

/* Device pointer of a frame (W*H*3 float) for in-HBM consumers (RCCL reduce). */
int bdpt_frame_device_ptr(void* ctx, int32_t which, void** dptr);

/* Enqueues a device-to-device copy of a frame into caller device memory (W*H*3 floats) on the
 * ctx stream — e.g. into a torch tensor that RCCL then reduces. Async. */
int bdpt_copy_frame(void* ctx, int32_t which, void* dst_device);

int bdpt_get_stats(void* ctx, bdpt_stats* out);

/* ABI v9: the multi-GPU frame reduce. The reference renders with N CPU threads
 * into one shared frame (raytraced_renderer.cpp:325-327); here N contexts — one per GPU, each
 * rendering its own sample range of every pixel — hold partial W*H*3 frames, and because the t = 1
 * light splats land on any pixel (bidirection.cpp:457-466) the image is their whole-frame sum.
 * bdpt_reduce_create builds one RCCL communicator clique over the contexts' distinct devices
 * (ncclCommInitAll; contexts sharing a device are summed on it first). bdpt_reduce_frames then
 * enqueues one grouped ncclReduce (sum, fp32) of every context's eye and light frames into the
 * `root` context's frames, on the contexts' streams (under the PathTracer the sampleCountBuffer is
 * summed too); afterwards bdpt_read_frame(root, ...) returns the whole image. The other contexts'
 * frames are unchanged. Async; later work on any listed ctx is ordered after it. The contexts must
 * outlive the reducer and share the frame size and integrator. RCCL is loaded on first use
 * (librccl.so.1); without it these calls fail with BDPT_E_DEVICE. */
typedef struct bdpt_reducer bdpt_reducer;
int bdpt_reduce_create(void* const* ctxs, int32_t n, bdpt_reducer** out);
int bdpt_reduce_frames(bdpt_reducer* r, int32_t root);
/* RCCL ranks of the reducer's communicator (= distinct devices), or BDPT_E_INVALID. */
int bdpt_reduce_ranks(const bdpt_reducer* r);
/* ncclGetVersion of the RCCL that the reducer uses (loads it), or a negative BDPT_E_* code. */
int bdpt_reduce_rccl_version(void);
void bdpt_reduce_destroy(bdpt_reducer* r);

/* Test hook: closest-hit / any-hit queries for a batch of rays through the device BVH
 * (BVHAccel::intersect, bvh.cpp:161-188). rays: n*8 floats {o.xyz, d.xyz, min_t, max_t};
 * out_t[n] (INFINITY if no hit), out_prim[n] (reference primitive index or -1). Sync. */
int bdpt_trace_rays(void* ctx, const float* rays, int32_t n, int32_t any_hit, float* out_t,
                    int32_t* out_prim);

/* Diagnostic hook: the 16 phase-profile words of a BDPT_PHASE_PROF build (cycles of the walks,
 * connection generation and connection rays, walk traversal; walk iterations per wave / per lane;
 * connection-grid cells / pairs). Sync. */
int bdpt_debug_counters(void* ctx, uint64_t* out16);
/* Diagnostic hook (ABI v9): the lane-use profile of a BDPT_PHASE_PROF build — per phase k (closest-hit
 * node steps, closest-hit primitive tests, any-hit node steps, any-hit primitive tests, walk
 * shading, walk iterations, connection evaluations, connection-ray flushes) out16[2k] = wave-level
 * iterations and out16[2k+1] = active lanes summed over them. Sync. Zero in product builds. */
int bdpt_debug_lane_counters(void* ctx, uint64_t* out16);

/* Host-side COLLADA loader: the reference CLI's scene path (ColladaParser::load,
 * collada.cpp:129-941, + Application::load, application.cpp:228-304). width/height > 0 apply
 * Camera::set_screen_size (-r W H). The desc returned by bdpt_dae_get_desc points into the
 * loaded scene and stays valid until bdpt_dae_free. No device is touched. */
typedef struct bdpt_dae bdpt_dae;
int bdpt_dae_load(const char* path, int32_t width, int32_t height, bdpt_dae** out);
int bdpt_dae_get_desc(const bdpt_dae* scene, bdpt_scene_desc* out);
/* Writes the scene in the JSON dump format of tests/golden/scenes (round-trip doubles). */
int bdpt_dae_dump_json(const bdpt_dae* scene, const char* path);
void bdpt_dae_free(bdpt_dae* scene);

/* ABI v5: the CLI's -c camera-settings file (main.cpp:120-121,177-178 -> Application::load_camera
 * -> Camera::load_settings, camera.cpp:172-186), read with the reference's stream extraction order
 * (hFov vFov ar nClip fClip, pos, targetPos, phi theta r minR maxR, c2w row by row, screenW
 * screenH screenDist, focalDistance lensRadius: the format Camera::dump_settings writes). It
 * replaces cam's hfov_deg, vfov_deg, nclip, fclip, pos and c2w. w2c is kept: load_settings does
 * not recompute it (w2c = c2w.inv() only happens in compute_position, camera.cpp:146), so the
 * reference's t = 1 camera connections keep using the placement's inverse — reproduced here.
 * A file that cannot be opened leaves cam unchanged (as the reference's ifstream does) and returns
 * BDPT_E_INVALID. */
int bdpt_camera_load_settings(const char* path, bdpt_camera* cam);
/* ABI v7: the same, also returning the file's focalDistance and lensRadius (its last line), which
 * Camera::load_settings writes over the thin-lens settings the renderer's config gave the camera
 * (raytraced_renderer.cpp:141-142 set_camera runs first, main.cpp:177 load_camera after, and
 * PathTracer::raytrace_pixel reads them in generate_ray_for_thin_lens, pathtracer.cpp:312).
 * *focal_distance / *lens_radius carry the current values in (a short file leaves or zeroes them
 * as the reference's extractions would). Either pointer may be null. */
int bdpt_camera_load_settings_lens(const char* path, bdpt_camera* cam, double* focal_distance, double* lens_radius);

/* Host-side OpenEXR reader for the -e environment map (main.cpp:40-77 load_exr, tinyexr):
 * scanline files with NONE / RLE / ZIPS / ZIP compression and HALF / FLOAT / UINT channels.
 * Like load_exr, the channels are taken in the file's (alphabetical) channel-list order and
 * r, g, b = channels 2, 1, 0 (an RGB file: R, G, B). *rgb_out (width*height*3 floats) is freed
 * with bdpt_exr_free. */
int bdpt_exr_load(const char* path, int32_t* width, int32_t* height, float** rgb_out);
void bdpt_exr_free(float* rgb);

#ifdef __cplusplus
}
#endif

#endif /* BDPT_AMD_BDPT_H */
