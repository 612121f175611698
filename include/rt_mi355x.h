/*
 * rt_mi355x.h — C ABI of the MI355X-native Monte-Carlo sample loop.
 *
 * Drop-in boundary for semicolonTransistor/rust-ray-tracing's hot path:
 *   trait Renderer { fn render(&self, max_bounces, samples_per_pixel, &Arc<Scene>, &Arc<Camera>)
 *                    -> (RgbImage, RenderStat) }                     (src/renderer.rs:38-40)
 * whose live implementation is TileRenderer::render (src/renderer.rs:243-387) driving
 * TileRenderTask::render_vectorized2 (src/renderer.rs:141-176) ->
 * Scene::trace_vectorized2 (src/ray_tracing.rs:375-505).  A GPU renderer is a new
 * `impl Renderer` that flattens Scene/Camera into the structs below and calls rt_render
 * (or the device-resident rt_context_* API); the Rust-side binding is in INTEGRATION.md.
 *
 * Everything is plain C: pointers + sizes, caller-owned buffers, int status codes.
 * Thread-safety: rt_render may be called from any thread; one rt_context must not be
 * used concurrently from two threads.
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (the reference panics instead; see rt_last_error) ---- */
#define RT_OK 0
#define RT_ERR_INVALID 1     /* bad argument: NULL pointer, spp == 0, material index out of range ...
                                (reference: unwrap()/panic!, e.g. objects.rs:296, materials.rs:31) */
#define RT_ERR_HIP 2         /* HIP runtime failure (no device, launch failure, OOM) */
#define RT_ERR_RANGE 3       /* a pixel channel exceeded 2.0 after /spp: the reference panics in
                                Color::to_u8_array (color.rs:55-57); the image is still written */
#define RT_ERR_UNSUPPORTED 4 /* configuration this build cannot run (e.g. spp > 2^20) */

/* Largest max_bounces an RT_FLAG_F32 render accepts (RT_ERR_UNSUPPORTED above): fp32 draws Philox2x32-10
 * with the counter (pixel, sample | code << 20), code 257 + bounce for the scatter, which must stay below
 * 2^12.  fp64 (Philox4x32-10, the bounce in its own counter word) has no such limit. */
#define RT_MAX_BOUNCES_F32 3839u

/* ---- materials (src/materials.rs:41-155) ---- */
#define RT_LAMBERTIAN 0u
#define RT_METAL 1u
#define RT_DIELECTRIC 2u

typedef struct rt_material {
    uint32_t kind;       /* RT_LAMBERTIAN / RT_METAL / RT_DIELECTRIC */
    uint32_t hollow;     /* Dielectric::hollow (materials.rs:111-114) */
    double albedo[3];    /* Lambertian::albedo / Metal::albedo */
    double fuzz;         /* Metal::fuzzy_factor, already clamped by Metal::new (materials.rs:79-88) */
    double ior;          /* Dielectric::index_of_refraction */
} rt_material;           /* 48 bytes */

/* ---- scene: spheres in scene order (closest-hit ties resolve to the later sphere,
 *      objects.rs:141), Scene::objects (ray_tracing.rs:102-104) flattened SoA ---- */
typedef struct rt_scene {
    uint32_t n_spheres;
    uint32_t n_materials;
    const double* center;         /* [n_spheres][3] */
    const double* radius;         /* [n_spheres] */
    const uint32_t* material;     /* [n_spheres], index into materials */
    const rt_material* materials; /* [n_materials] */
} rt_scene;

/* ---- camera: the precomputed fields of Camera (ray_tracing.rs:15-24) ---- */
typedef struct rt_camera {
    uint32_t image_width, image_height;
    double center[3];   /* Camera::center */
    double ulc[3];      /* Camera::viewport_upper_left_corner */
    double vu[3];       /* Camera::viewport_u */
    double vv[3];       /* Camera::viewport_v */
    double du[3];       /* Camera::defocus_u */
    double dv[3];       /* Camera::defocus_v */
} rt_camera;

/* Pixel set to render: rows row_begin + i*row_step (i < row_count), columns
 * [col_begin, col_begin + col_count).  Outputs are compact over the set:
 * element (i, c) at index i*col_count + c.  NULL = whole image (== RgbImage layout). */
typedef struct rt_tile_range {
    uint32_t row_begin, row_step, row_count;
    uint32_t col_begin, col_count;
} rt_tile_range;

/* RenderStat (renderer.rs:11-34) plus the work counters the roofline needs. */
typedef struct rt_stats {
    double seconds;          /* wall time of the call (host clock) */
    double kernel_ms;        /* device time of the trace kernel(s), HIP events */
    double pixels_per_second;
    uint64_t pixels;
    uint64_t samples;        /* pixels * spp */
    uint64_t ray_segments;   /* enabled rays traced, summed over bounces (ray_tracing.rs:396-401) */
    uint64_t lane_slots;     /* SIMD lanes issued for those traces (64 per wave-bounce);
                                (ray_segments - direct_sky_samples) / lane_slots = lane utilisation */
    uint64_t bounce_iters;   /* bounce-loop iterations executed, summed over pixels */
    /* Executed work of the culls and exact tests, in wave-level tests (each runs all 64 lanes of a
     * wave); DESIGN.md §5 turns them into executed FLOP for the roofline:
     *   box_groups          general sweep, 4 boxes each: 18 v_pk_fma_f32 = 72 fp32 FLOP per lane
     *   filter_groups       general sweep, 4 spheres each: 14 v_pk_fma_f32 = 56 fp32 FLOP per lane
     *   exact_tests         general sweep, one sphere each through Sphere::hit_packed's test
     *                       (objects.rs:252-257): 17 FLOP per lane in the render's precision
     *   cone_tests          camera sweep, 64 cone records each: 23 fp32 FLOP per lane
     *   camera_exact_tests  camera sweep, one sphere each from the camera-origin table: 8 FLOP per
     *                       lane in the render's precision */
    uint64_t box_groups, filter_groups, exact_tests, cone_tests, camera_exact_tests;
    /* Samples of pixels finished when they are claimed, without tracing: a pinhole camera's pixel
     * whose camera candidate list is empty (no primary ray of the pixel can hit a sphere, so every
     * sample escapes at bounce 0).  Their primary segments are in ray_segments (the reference traces
     * them, ray_tracing.rs:396-401) but occupy no SIMD lane, so they are not in lane_slots. */
    uint64_t direct_sky_samples;
    /* The kernel the last collected render ran (RT_KERNEL_* fields below; 0 = none) and how many of
     * its 4-wave workgroups were resident per CU (hipOccupancyMaxActiveBlocksPerMultiprocessor): equal
     * to the kernel's waves-per-SIMD target unless LDS or registers cut its occupancy. */
    uint32_t kernel_id;
    uint32_t kernel_wg_per_cu;
} rt_stats;

/* rt_stats.kernel_id: trace_paths<T, W, ROOT2, MODE, CAMQ, MEGA> of rt_kernel.hip, one bit field each.
 * Bit 15 is set for any kernel, so 0 means "no render collected". */
#define RT_KERNEL_F64(id) ((id) & 1u)            /* T = double (else float) */
#define RT_KERNEL_WAVES(id) (((id) >> 1) & 7u)   /* W: waves per SIMD the register allocation targets */
#define RT_KERNEL_ROOT2(id) (((id) >> 4) & 1u)   /* quirk Q1 off */
#define RT_KERNEL_MODE(id) (((id) >> 5) & 3u)    /* 0 live path, 1 vectorized, 2 scalar, 3 vectorized3 */
#define RT_KERNEL_CAMQ(id) (((id) >> 7) & 1u)    /* pinhole camera batches */
#define RT_KERNEL_MEGA(id) (((id) >> 8) & 1u)    /* four-level sweep (mega boxes; scenes of > 8 super groups) */

/* ---- flags ---- */
#define RT_FLAG_F32 0x1u     /* compute in fp32 (default: fp64, the reference's arithmetic) */
#define RT_FLAG_ROOT2 0x2u   /* quirk Q1 off: accept the far root like scalar Sphere::hit
                                (objects.rs:228-234) instead of testing root1 twice (objects.rs:273) */
/* Semantics modes (at most one; default = the live path, TileRenderTask::render_vectorized2 ->
 * Scene::trace_vectorized2, renderer.rs:141-176, quirks Q1-Q3 as the reference has them):
 *   RT_FLAG_MODE_VECTORIZED: render_vectorized -> Scene::trace_vectorized (renderer.rs:102-139,
 *     ray_tracing.rs:312-373): each sample keeps its own value and the sky uses its own final
 *     direction (Q2, Q3 off); hit_packed is shared, so Q1 still applies unless RT_FLAG_ROOT2.
 *   RT_FLAG_MODE_VECTORIZED3: render_vectorized3 -> Scene::trace_vectorized3 (renderer.rs:178-213,
 *     ray_tracing.rs:508-628): each sample's own value as in _VECTORIZED, summed in the order an
 *     in-place swap partition (CombinedIndex, :113-214, :561-607) leaves the slots in; the missing
 *     lanes of a partial chunk add sky(0) (white at depth 0).
 *   RT_FLAG_MODE_SCALAR: TileRenderTask::render -> Scene::trace_rays (renderer.rs:68-100,
 *     ray_tracing.rs:264-306): scalar Sphere::hit (objects.rs:216-247; no FMA, both roots, normal
 *     divided by the signed radius), the first of equal hits wins (min_by_key), Color::average. */
#define RT_FLAG_MODE_VECTORIZED 0x4u
#define RT_FLAG_MODE_SCALAR 0x8u
#define RT_FLAG_MODE_VECTORIZED3 0x10u
#define RT_FLAG_ALL 0x1Fu     /* any other bit, or two mode bits, is RT_ERR_INVALID */

/* Camera::new (ray_tracing.rs:27-62).  view_angle and defocus_angle in degrees. */
int rt_camera_new(rt_camera* out, uint32_t image_width, uint32_t image_height, double focal_length,
                  double view_angle_deg, const double center[3], const double look_at[3],
                  const double up[3], double defocus_angle_deg);

/* Metal::new's clamp (materials.rs:79-88): fuzz < 1 ? fuzz : 1. */
double rt_metal_clamp_fuzz(double fuzz);

/* One-shot render, host buffers in/out (replaces TileRenderer::render, renderer.rs:243-387,
 * on the device; scene upload and PCIe copies included).
 *   rgb8:   [pixels][3] RGB8, Color::to_u8_array of (sum / spp)   (may be NULL)
 *   linear: [pixels][3] f64 pixel colour after /spp, before gamma (may be NULL)
 *   stats:  may be NULL
 *   seed:   keys the counter-based draws that replace thread_rng() (ray_tracing.rs:78-79).  fp64
 *           keys Philox4x32-10 with the whole 64-bit seed.  fp32 (RT_FLAG_F32) keys Philox2x32-10,
 *           whose key is 32 bits: seed lo ^ fmix32(seed hi) (murmur3's finaliser; fmix32(0) = 0), so
 *           2^32 seed pairs share each fp32 key, but no structured pattern such as hi == lo does.
 * Returns RT_OK, RT_ERR_RANGE (image written; reference would have panicked) or an error. */
int rt_render(const rt_scene* scene, const rt_camera* camera, uint32_t max_bounces, uint32_t spp,
              uint64_t seed, uint32_t flags, const rt_tile_range* range, uint8_t* rgb8,
              double* linear, rt_stats* stats);

/* ---- device-resident API: scene kept in HBM across calls, outputs in device memory ---- */
typedef struct rt_context rt_context;

/* The renderer object: TileRenderer::new (renderer.rs:232-241) and its drop; one per GPU. */
int rt_context_create(int device, rt_context** out);
int rt_context_destroy(rt_context* ctx);
/* Upload (replace) the scene, the Arc<Scene> handed to Renderer::render (main.rs:43,
 * renderer.rs:38-40); copies fp64 and fp32 SoA images into HBM. */
int rt_context_set_scene(rt_context* ctx, const rt_scene* scene);
/* Enqueue one render on `stream` (a hipStream_t; NULL = the HIP null stream, as in every HIP
 * API): the pixels of `range` through TileRenderTask::render_vectorized2 (renderer.rs:141-176),
 * i.e. one share of TileRenderer::render's tile loop (renderer.rs:248-296).  d_rgb8 / d_linear are device pointers (either may be NULL).  Asynchronous.  Renders on
 * one context share its work counter, scratch and camera table: a render on a different stream
 * than the previous one first synchronises the previous stream, so they never overlap.  Use one
 * context per concurrent stream for overlap. */
int rt_render_async(rt_context* ctx, const rt_camera* camera, uint32_t max_bounces, uint32_t spp,
                    uint64_t seed, uint32_t flags, const rt_tile_range* range, void* d_rgb8,
                    void* d_linear, void* stream);
/* RenderStat (renderer.rs:11-34) for the renders since the last call.
 * Synchronise `stream` (NULL = null stream), then report and reset the counters accumulated by the renders
 * enqueued since the last call (ray_segments, work counters, error flag).  kernel_ms = device time
 * between the first and last enqueued render (HIP events on that stream); pixels_per_second =
 * pixels / kernel_ms (the per-shard px/s the reference prints per tile, renderer.rs:339);
 * seconds = 0 (rt_render fills in its wall time). */
int rt_context_collect(rt_context* ctx, void* stream, rt_stats* stats);
/* Device memory helpers (so hosts without a HIP toolchain can drive the async API); no reference
 * counterpart (the reference has no device memory). */
int rt_device_alloc(rt_context* ctx, size_t bytes, void** out);
int rt_device_free(rt_context* ctx, void* ptr);
int rt_memcpy_d2h(rt_context* ctx, void* dst, const void* src, size_t bytes);   /* synchronises the device */

/* Last error message of the calling thread ("" if none). */
const char* rt_last_error(void);
/* Build/version string: "rt_mi355x <version> gfx950 <product|experiment> src=<source hash>". */
const char* rt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_MI355X_H */
