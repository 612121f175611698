/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of semicolonTransistor/rust-ray-tracing's live packed path
 * (TileRenderTask::render_vectorized2 -> Scene::trace_vectorized2), used as the
 * parity checker for the HIP megakernel and as the timed CPU baseline in
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library; the product path never links it.
 *
 * PARITY STATUS: "parity unpinned" w.r.t. the real reference binary.
 *   - The reference has no tests, fixtures or golden vectors and
 *     cannot be built here (Rust nightly + crates.io deps; no rustc/cargo).
 *   - The reference draws from rand::thread_rng() (unseedable ChaCha12, rand 0.8.5)
 *     and rand_distr 0.4.3 Normal; those streams cannot be reproduced.  This oracle
 *     substitutes keyed Philox4x32-10 (f64) and Philox2x32-10 (f32) streams with the same distributions
 *     (see oracle_impl.h "RNG boundary").
 *   - What IS pinned: every deterministic formula (camera, sphere test, hit-record
 *     finalize, scatter, compaction, sky, final buffer read, quantization) follows
 *     the reference file:line cited next to it, checked by source-derived
 *     known-answer tests (tests/test_oracle_kat.py) and Philox's published KATs.
 *
 * The struct layouts below intentionally match include/rt_mi355x.h so tests can
 * hand the same ctypes structures to both; they are declared independently.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_material {
    uint32_t kind;      /* 0 lambertian, 1 metal, 2 dielectric */
    uint32_t hollow;    /* dielectric only */
    double albedo[3];   /* lambertian / metal */
    double fuzz;        /* metal, already clamped <= 1 by Metal::new (materials.rs:79-88) */
    double ior;         /* dielectric */
} or_material;

typedef struct or_scene {
    uint32_t n_spheres;
    uint32_t n_materials;
    const double* center;      /* [n_spheres][3], scene order (tie rule depends on it) */
    const double* radius;      /* [n_spheres] */
    const uint32_t* material;  /* [n_spheres] index into materials */
    const or_material* materials;
} or_scene;

typedef struct or_camera {
    uint32_t image_width, image_height;
    double center[3], ulc[3], vu[3], vv[3], du[3], dv[3];
} or_camera;

/* flag bits (same values as RT_FLAG_* in include/rt_mi355x.h) */
#define OR_FLAG_ROOT2 0x2u   /* Q1 off: accept root2 like scalar Sphere::hit (objects.rs:228-234) */
/* Semantics modes (default: trace_vectorized2 via render_vectorized2, renderer.rs:141-176):
 *   VECTORIZED: trace_vectorized (ray_tracing.rs:312-373) via render_vectorized (renderer.rs:102-139)
 *               — per-chunk, final-ray sky (Q2 off), every ray keeps its own value (Q3 off);
 *               hit_packed is shared with the default mode, so Q1 / OR_FLAG_ROOT2 still apply.
 *   SCALAR:     trace_rays (ray_tracing.rs:264-306) via render (renderer.rs:68-100) — scalar
 *               Sphere::hit (objects.rs:216-247: both roots, no FMA, normal / signed radius),
 *               first minimum wins ties, Color::average in sample order. */
#define OR_FLAG_MODE_VECTORIZED 0x4u
#define OR_FLAG_MODE_SCALAR 0x8u
/* OR_FLAG_MODE_VECTORIZED3: TileRenderTask::render_vectorized3 -> Scene::trace_vectorized3
 *               (renderer.rs:178-213, ray_tracing.rs:508-628): in-place swap partition, own-direction
 *               sky, colours white for every lane (missing lanes of a partial chunk add sky(0)). */
#define OR_FLAG_MODE_VECTORIZED3 0x10u

/* Render the listed pixels (global index row*W+col; NULL = all W*H in order).
 * rgb_out: n*3 bytes, lin_out: n*3 doubles (pixel colour after /spp, before
 * gamma), either may be NULL.  *segments (may be NULL) receives the number of
 * enabled rays traced (sum over bounces of enabled lanes).
 * Returns 0, or 3 if some channel exceeded 2.0 (the reference panics there,
 * color.rs:55-57), or 1 on bad arguments (including both mode bits set), or 4 when the
 * RNG counter cannot hold the configuration (spp > 2^20; f32: max_bounces > 3839, the
 * C ABI's RT_ERR_UNSUPPORTED). */
int oracle_render_f64(const or_scene* sc, const or_camera* cam, uint32_t max_bounces,
                      uint32_t spp, uint64_t seed, uint32_t flags,
                      const uint32_t* pixels, uint32_t n_pixels,
                      uint8_t* rgb_out, double* lin_out, uint64_t* segments, int n_threads);
int oracle_render_f32(const or_scene* sc, const or_camera* cam, uint32_t max_bounces,
                      uint32_t spp, uint64_t seed, uint32_t flags,
                      const uint32_t* pixels, uint32_t n_pixels,
                      uint8_t* rgb_out, double* lin_out, uint64_t* segments, int n_threads);

/* Camera::new (ray_tracing.rs:27-62). */
int oracle_camera_new(or_camera* out, uint32_t w, uint32_t h, double focal_length,
                      double view_angle_deg, const double center[3], const double look_at[3],
                      const double up[3], double defocus_angle_deg);

/* Philox4x32-10 block (for KATs). */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Philox2x32-10 block: the fp32 build's draws (for KATs). */
void oracle_philox2x32_10(const uint32_t ctr[2], uint32_t key, uint32_t out[2]);
/* The fp32 key fold: seed lo ^ oracle_fmix32(seed hi) (murmur3's finaliser). */
uint32_t oracle_fmix32(uint32_t h);

/* Primitive probes for known-answer tests. */
void oracle_sincos2pi_f64(double u, double* s, double* c);
void oracle_to_u8(const double rgb[3], uint8_t out[3], int* panics);
void oracle_get_ray_f64(const or_camera* cam, uint32_t col, uint32_t row, uint32_t sample,
                        uint64_t seed, double origin[3], double dir[3]);

/* The reference-shaped CPU baseline (packed_avx2.h): the same results as oracle_render_f64, computed
 * the way the reference runs them (4-lane f64 AVX2 packets, 128x128 tiles through a shared queue).
 * rgb_out / lin_out are full-frame (W*H*3); only the listed tiles (row-major tile grid; NULL = all)
 * are written. */
int packed_render_f64(const or_scene* sc, const or_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                      uint32_t tile, const uint32_t* tiles, uint32_t n_tiles, uint8_t* rgb_out, double* lin_out,
                      uint64_t* segments, uint64_t* pixels_out, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
