/*
 * packed_avx2.h — TEST INFRASTRUCTURE / CPU BASELINE ONLY (bench.py's cpu_baseline.packed leg).
 *
 * The reference's live packed path as the reference itself runs it on a CPU, restated with explicit
 * 4-lane f64 AVX2: PackedRays<4> as __m256d lanes (ray.rs:36-43, Simd<f64, 4>), Sphere::hit_packed
 * with _mm256_fmadd_pd where the reference writes mul_add (objects.rs:249-290; geometry.rs:434-436,
 * 466-468), the any() gate as a movemask (objects.rs:259-261), masked_select / PackedHitRecords::update
 * as blendv (simd_util.rs:39-60, objects.rs:140-155), PackedHitRecords::finalize packed (:157-162), the
 * per-lane material scatter scalar (ray_tracing.rs:406-426), the two-buffer stable shuffle
 * (:430-481) and the (C-1)%2 final read (:486-504); the image in 128x128 tiles pulled by
 * every thread from one shared counter (TileRenderer's MPMC tile channel, renderer.rs:243-296).
 * Same operations in the same order as the scalar oracle (oracle_impl.h), so it is bit-identical to
 * oracle_render_f64 (tests/test_oracle_packed.py) -- it only runs them the way the reference does.
 * The loop-invariant a = |d|^2 and 1/a (objects.rs:253-254) are computed once per chunk, as an
 * optimising compiler hoists them out of the inlined sphere loop.
 *
 * Included at the end of oracle.c (it uses the f64 instantiation's static helpers).
 */
#include <immintrin.h>

typedef struct {
    double ox[4], oy[4], oz[4], dx[4], dy[4], dz[4];
    double en[4];       /* mask lanes: all ones = enabled (Mask<i64, 4>) */
    uint32_t sid[4];
} __attribute__((aligned(32))) pk_rays;
typedef struct { double r[4], g[4], b[4]; } __attribute__((aligned(32))) pk_col;

static inline double pk_on(void) { uint64_t b = ~0ull; double d; memcpy(&d, &b, 8); return d; }
static inline int pk_lane_on(double m) { uint64_t b; memcpy(&b, &m, 8); return b != 0; }

typedef struct {
    uint32_t C;
    pk_rays* rays0;
    pk_rays* buf[2];
    pk_col* col[2];
    double* sky[2];     /* [C][4] masks */
} pk_ws;

static int pk_ws_init(pk_ws* w, uint32_t C) {
    w->C = C;
    const size_t nr = ((size_t)C * sizeof(pk_rays) + 31) & ~(size_t)31, nc = ((size_t)C * sizeof(pk_col) + 31) & ~(size_t)31;
    const size_t ns = ((size_t)C * 4 * sizeof(double) + 31) & ~(size_t)31;
    w->rays0 = (pk_rays*)aligned_alloc(32, nr);
    w->buf[0] = (pk_rays*)aligned_alloc(32, nr); w->buf[1] = (pk_rays*)aligned_alloc(32, nr);
    w->col[0] = (pk_col*)aligned_alloc(32, nc); w->col[1] = (pk_col*)aligned_alloc(32, nc);
    w->sky[0] = (double*)aligned_alloc(32, ns); w->sky[1] = (double*)aligned_alloc(32, ns);
    return w->rays0 && w->buf[0] && w->buf[1] && w->col[0] && w->col[1] && w->sky[0] && w->sky[1];
}
static void pk_ws_free(pk_ws* w) {
    free(w->rays0);
    for (int i = 0; i < 2; ++i) { free(w->buf[i]); free(w->col[i]); free(w->sky[i]); }
}

/* One chunk against every sphere: Sphere::hit_packed + PackedHitRecords::update per sphere
 * (ray_tracing.rs:399-401), then finalize (:403).  Returns the hit mask (bit l: lane l hit). */
static inline int pk_hit_chunk(const scene_r_f64* S, const double* r2s, const pk_rays* R, double px[4], double py[4],
                               double pz[4], double nx_[4], double ny_[4], double nz_[4], int front[4], uint32_t mat[4]) {
    const __m256d ox = _mm256_load_pd(R->ox), oy = _mm256_load_pd(R->oy), oz = _mm256_load_pd(R->oz);
    const __m256d dx = _mm256_load_pd(R->dx), dy = _mm256_load_pd(R->dy), dz = _mm256_load_pd(R->dz);
    const __m256d en = _mm256_load_pd(R->en);
    const __m256d a = _mm256_fmadd_pd(dz, dz, _mm256_fmadd_pd(dy, dy, _mm256_mul_pd(dx, dx)));   /* :253 */
    const __m256d inv_a = _mm256_div_pd(_mm256_set1_pd(1.0), a);                                /* :254 */
    const __m256d sgn = _mm256_set1_pd(-0.0);
    const __m256d na = _mm256_xor_pd(a, sgn);   /* -a */
    const __m256d tmin = _mm256_set1_pd(0.001), inf = _mm256_set1_pd(INFINITY), zero = _mm256_setzero_pd();
    __m256d t = inf, nx = zero, ny = zero, nz = zero, hit = zero;                                 /* default() :124-133 */
    int mat_l[4] = {0, 0, 0, 0};
    for (uint32_t i = 0; i < S->n; ++i) {
        const __m256d cx = _mm256_set1_pd(S->cx[i]), cy = _mm256_set1_pd(S->cy[i]), cz = _mm256_set1_pd(S->cz[i]);
        const __m256d ocx = _mm256_sub_pd(ox, cx), ocy = _mm256_sub_pd(oy, cy), ocz = _mm256_sub_pd(oz, cz);   /* :252 */
        const __m256d hb = _mm256_fmadd_pd(ocz, dz, _mm256_fmadd_pd(ocy, dy, _mm256_mul_pd(ocx, dx)));         /* :255 */
        const __m256d c = _mm256_sub_pd(_mm256_fmadd_pd(ocz, ocz, _mm256_fmadd_pd(ocy, ocy, _mm256_mul_pd(ocx, ocx))),
                                        _mm256_set1_pd(r2s[i]));                                                  /* :256 */
        const __m256d disc = _mm256_fmadd_pd(hb, hb, _mm256_mul_pd(na, c));                                       /* :257 */
        const __m256d gate = _mm256_and_pd(_mm256_cmp_pd(disc, zero, _CMP_GE_OQ), en);                          /* :259 */
        if (_mm256_movemask_pd(gate) == 0) continue;                                                              /* :261 any() */
        const __m256d sd = _mm256_sqrt_pd(disc);                                                                  /* :263 */
        const __m256d r1 = _mm256_mul_pd(_mm256_sub_pd(_mm256_xor_pd(hb, sgn), sd), inv_a);                      /* :270 */
        const __m256d r1v = _mm256_and_pd(_mm256_cmp_pd(r1, tmin, _CMP_GE_OQ), _mm256_cmp_pd(r1, inf, _CMP_LT_OQ)); /* :272 */
        /* Q1: root2_valid tests root1 again (:273), so root = masked_select(.., root1, root1_valid) = root1 */
        const __m256d upd = _mm256_and_pd(_mm256_and_pd(r1v, en), _mm256_cmp_pd(r1, t, _CMP_LE_OQ));            /* :141 */
        const int um = _mm256_movemask_pd(upd);
        if (um == 0) continue;
        t = _mm256_blendv_pd(t, r1, upd);
        const __m256d lx = _mm256_add_pd(ox, _mm256_mul_pd(dx, r1));                                             /* at_t */
        const __m256d ly = _mm256_add_pd(oy, _mm256_mul_pd(dy, r1));
        const __m256d lz = _mm256_add_pd(oz, _mm256_mul_pd(dz, r1));
        nx = _mm256_blendv_pd(nx, _mm256_sub_pd(lx, cx), upd);                                                    /* :280 */
        ny = _mm256_blendv_pd(ny, _mm256_sub_pd(ly, cy), upd);
        nz = _mm256_blendv_pd(nz, _mm256_sub_pd(lz, cz), upd);
        hit = _mm256_or_pd(hit, upd);
        for (int l = 0; l < 4; ++l) if (um >> l & 1) mat_l[l] = (int)S->mat[i];
    }
    /* finalize, objects.rs:157-162: N <- unit(N) (packed length), P <- at_t(t), front face, flip */
    const __m256d len = _mm256_sqrt_pd(_mm256_fmadd_pd(nz, nz, _mm256_fmadd_pd(ny, ny, _mm256_mul_pd(nx, nx))));
    nx = _mm256_div_pd(nx, len); ny = _mm256_div_pd(ny, len); nz = _mm256_div_pd(nz, len);
    _mm256_storeu_pd(px, _mm256_add_pd(ox, _mm256_mul_pd(dx, t)));
    _mm256_storeu_pd(py, _mm256_add_pd(oy, _mm256_mul_pd(dy, t)));
    _mm256_storeu_pd(pz, _mm256_add_pd(oz, _mm256_mul_pd(dz, t)));
    const __m256d fr = _mm256_cmp_pd(_mm256_fmadd_pd(dz, nz, _mm256_fmadd_pd(dy, ny, _mm256_mul_pd(dx, nx))), zero, _CMP_LT_OQ);
    nx = _mm256_blendv_pd(_mm256_xor_pd(nx, sgn), nx, fr);
    ny = _mm256_blendv_pd(_mm256_xor_pd(ny, sgn), ny, fr);
    nz = _mm256_blendv_pd(_mm256_xor_pd(nz, sgn), nz, fr);
    _mm256_storeu_pd(nx_, nx); _mm256_storeu_pd(ny_, ny); _mm256_storeu_pd(nz_, nz);
    const int fm = _mm256_movemask_pd(fr);
    for (int l = 0; l < 4; ++l) { front[l] = fm >> l & 1; mat[l] = (uint32_t)mat_l[l]; }
    return _mm256_movemask_pd(hit);
}

static inline void pk_copy_slot(pk_ws* w, int fs, uint32_t fc, int fl, int ts, uint32_t tc, int tl, double en) {
    const pk_rays* a = &w->buf[fs][fc];
    pk_rays* b = &w->buf[ts][tc];
    b->ox[tl] = a->ox[fl]; b->oy[tl] = a->oy[fl]; b->oz[tl] = a->oz[fl];
    b->dx[tl] = a->dx[fl]; b->dy[tl] = a->dy[fl]; b->dz[tl] = a->dz[fl];
    b->en[tl] = en; b->sid[tl] = a->sid[fl];
    w->col[ts][tc].r[tl] = w->col[fs][fc].r[fl];
    w->col[ts][tc].g[tl] = w->col[fs][fc].g[fl];
    w->col[ts][tc].b[tl] = w->col[fs][fc].b[fl];
    w->sky[ts][tc * 4 + tl] = w->sky[fs][fc * 4 + fl];
}

/* Scene::trace_vectorized2 (ray_tracing.rs:375-505) for one pixel's chunks in w->rays0. */
static void pk_trace_pixel(const scene_r_f64* S, const double* r2s, pk_ws* w, uint32_t depth, uint32_t pix, uint32_t k0,
                           uint32_t k1, double out[3], uint64_t* segs) {
    const uint32_t C = w->C;
    const double on = pk_on();
    for (uint32_t j = 0; j < C; ++j) {                                                      /* :382-384 */
        w->buf[0][j] = w->rays0[j];
        memset(&w->buf[1][j], 0, sizeof(pk_rays));
        for (int l = 0; l < 4; ++l) {
            w->buf[1][j].en[l] = on;
            for (int s = 0; s < 2; ++s) {
                w->col[s][j].r[l] = 1.0; w->col[s][j].g[l] = 1.0; w->col[s][j].b[l] = 1.0;
                w->sky[s][j * 4 + l] = 0.0;
            }
        }
    }
    uint32_t last = C;                                                                      /* :386 */
    uint64_t nseg = 0;
    for (uint32_t k = 0; k < depth && last != 0; ++k) {                                     /* :388-392 */
        const int sel = (int)(k % 2);
        for (uint32_t j = 0; j < last; ++j) {                                               /* :396 */
            pk_rays* R = &w->buf[sel][j];
            double px[4], py[4], pz[4], nx[4], ny[4], nz[4];
            int front[4];
            uint32_t mat[4];
            for (int l = 0; l < 4; ++l) nseg += pk_lane_on(R->en[l]);
            const int hm = pk_hit_chunk(S, r2s, R, px, py, pz, nx, ny, nz, front, mat);
            for (int l = 0; l < 4; ++l) {                                                   /* :406-426, per lane */
                if (hm >> l & 1) {
                    v3_f64 nd;
                    double att[3];
                    scatter_f64(&S->mats[mat[l]], mk_f64(R->dx[l], R->dy[l], R->dz[l]), mk_f64(px[l], py[l], pz[l]),
                                mk_f64(nx[l], ny[l], nz[l]), front[l], pix, R->sid[l], k, k0, k1, &nd, att);
                    pk_col* cc = &w->col[sel][j];
                    cc->r[l] = cc->r[l] * att[0]; cc->g[l] = cc->g[l] * att[1]; cc->b[l] = cc->b[l] * att[2];
                    R->ox[l] = px[l]; R->oy[l] = py[l]; R->oz[l] = pz[l];
                    R->dx[l] = nd.x; R->dy[l] = nd.y; R->dz[l] = nd.z;
                    R->en[l] = on;
                } else {
                    R->en[l] = 0.0;                                                         /* :422 */
                    w->sky[sel][j * 4 + l] = on;                                            /* :423 */
                }
            }
        }
        const int ns = 1 - sel;                                                             /* :430-481 */
        uint32_t oc = 0;
        int os = 0;
        for (uint32_t i = 0; i < last; ++i)
            for (int l = 0; l < 4; ++l)
                if (pk_lane_on(w->buf[sel][i].en[l])) {
                    pk_copy_slot(w, sel, i, l, ns, oc, os, on);
                    if (++os >= 4) { os = 0; ++oc; }
                }
        const uint32_t nl = os == 0 ? oc : oc + 1;
        for (uint32_t i = 0; i < last; ++i)
            for (int l = 0; l < 4; ++l)
                if (!pk_lane_on(w->buf[sel][i].en[l])) {
                    pk_copy_slot(w, sel, i, l, ns, oc, os, 0.0);
                    if (++os >= 4) { os = 0; ++oc; }
                }
        last = nl;
    }
    /* :486-504: buffer (C-1)%2, sky of the ORIGINAL rays, black where still enabled, per-lane sums */
    const int sel = (int)((C - 1) % 2);
    __m256d ar = _mm256_setzero_pd(), ag = _mm256_setzero_pd(), ab = _mm256_setzero_pd();
    const __m256d one = _mm256_set1_pd(1.0), half = _mm256_set1_pd(0.5), zero = _mm256_setzero_pd();
    for (uint32_t j = 0; j < C; ++j) {
        const __m256d a = _mm256_mul_pd(_mm256_add_pd(_mm256_load_pd(w->rays0[j].dy), one), half);   /* :490 */
        const __m256d oma = _mm256_add_pd(_mm256_xor_pd(a, _mm256_set1_pd(-0.0)), one);
        const __m256d sr = _mm256_add_pd(_mm256_mul_pd(one, oma), _mm256_mul_pd(_mm256_set1_pd(0.5), a));
        const __m256d sg = _mm256_add_pd(_mm256_mul_pd(one, oma), _mm256_mul_pd(_mm256_set1_pd(0.7), a));
        const __m256d sb = _mm256_add_pd(_mm256_mul_pd(one, oma), _mm256_mul_pd(one, a));
        const __m256d sk = _mm256_load_pd(&w->sky[sel][j * 4]);
        const __m256d en = _mm256_load_pd(w->buf[sel][j].en);
        __m256d cr = _mm256_load_pd(w->col[sel][j].r), cg = _mm256_load_pd(w->col[sel][j].g),
                cb = _mm256_load_pd(w->col[sel][j].b);
        cr = _mm256_blendv_pd(cr, _mm256_mul_pd(cr, sr), sk);                               /* :494-495 */
        cg = _mm256_blendv_pd(cg, _mm256_mul_pd(cg, sg), sk);
        cb = _mm256_blendv_pd(cb, _mm256_mul_pd(cb, sb), sk);
        cr = _mm256_blendv_pd(cr, zero, en); cg = _mm256_blendv_pd(cg, zero, en); cb = _mm256_blendv_pd(cb, zero, en);   /* :496 */
        ar = _mm256_add_pd(ar, cr); ag = _mm256_add_pd(ag, cg); ab = _mm256_add_pd(ab, cb);       /* :500-502 */
    }
    double acc[3][4];
    _mm256_storeu_pd(acc[0], ar); _mm256_storeu_pd(acc[1], ag); _mm256_storeu_pd(acc[2], ab);
    for (int ch = 0; ch < 3; ++ch) out[ch] = ((0.0 + acc[ch][0]) + acc[ch][1] + acc[ch][2]) + acc[ch][3];   /* PackedColor::sum */
    *segs += nseg;
}

typedef struct {
    const scene_r_f64* S;
    const double* r2s;
    const cam_r_f64* cam;
    uint32_t depth, spp, k0, k1, tile, tiles_x;
    const uint32_t* tiles;
    uint32_t n_tiles;
    uint8_t* rgb; double* lin;
    volatile uint32_t next;   /* the shared tile channel (renderer.rs:251-284) */
    uint64_t segs, pixels;
    int panic;
    pthread_mutex_t mu;
} pk_job;

static void* pk_worker(void* arg) {
    pk_job* J = (pk_job*)arg;
    const uint32_t C = (J->spp + 3u) / 4u;
    pk_ws w;
    if (!pk_ws_init(&w, C)) { pk_ws_free(&w); return NULL; }
    const double on = pk_on();
    uint64_t segs = 0, npx = 0;
    int panic = 0;
    for (;;) {
        const uint32_t ti = __atomic_fetch_add(&J->next, 1u, __ATOMIC_RELAXED);
        if (ti >= J->n_tiles) break;
        const uint32_t t = J->tiles ? J->tiles[ti] : ti;
        const uint32_t c0 = (t % J->tiles_x) * J->tile, r0 = (t / J->tiles_x) * J->tile;
        const uint32_t c1 = c0 + J->tile < J->cam->W ? c0 + J->tile : J->cam->W;
        const uint32_t r1 = r0 + J->tile < J->cam->H ? r0 + J->tile : J->cam->H;
        for (uint32_t row = r0; row < r1; ++row)
            for (uint32_t col = c0; col < c1; ++col) {
                const uint32_t pix = row * J->cam->W + col;
                for (uint32_t j = 0; j < C; ++j) {                 /* renderer.rs:155-159, ray.rs:136-153 */
                    pk_rays* P = &w.rays0[j];
                    memset(P, 0, sizeof(*P));
                    for (int l = 0; l < 4; ++l) {
                        const uint32_t s = j * 4u + (uint32_t)l;
                        P->sid[l] = s;
                        if (s < J->spp) {
                            v3_f64 o, d;
                            get_ray_f64(J->cam, col, row, pix, s, J->k0, J->k1, &o, &d);
                            P->ox[l] = o.x; P->oy[l] = o.y; P->oz[l] = o.z;
                            P->dx[l] = d.x; P->dy[l] = d.y; P->dz[l] = d.z;
                            P->en[l] = on;
                        }
                    }
                }
                double sum[3];
                pk_trace_pixel(J->S, J->r2s, &w, J->depth, pix, J->k0, J->k1, sum, &segs);
                for (int ch = 0; ch < 3; ++ch) {
                    const double v = sum[ch] / (double)J->spp;     /* renderer.rs:161 */
                    if (!(v <= 2.0)) panic = 1;                    /* color.rs:55-57 */
                    if (J->rgb) J->rgb[(size_t)pix * 3 + ch] = q8_f64(v);
                    if (J->lin) J->lin[(size_t)pix * 3 + ch] = v;
                }
                ++npx;
            }
    }
    pk_ws_free(&w);
    pthread_mutex_lock(&J->mu);
    J->segs += segs;
    J->pixels += npx;
    J->panic |= panic;
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

/* The image (full-frame rgb_out / lin_out, either may be NULL) in tile x tile blocks, the listed
 * block indices only (row-major block grid; NULL = every block), n_threads workers pulling blocks.
 * *pixels_out: pixels rendered.  Returns 0, 3 on a channel > 2.0, 1 on bad arguments. */
int packed_render_f64(const or_scene* sc, const or_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                      uint32_t tile, const uint32_t* tiles, uint32_t n_tiles, uint8_t* rgb_out, double* lin_out,
                      uint64_t* segments, uint64_t* pixels_out, int n_threads) {
    if (!sc || !cam || spp == 0 || tile == 0 || cam->image_width == 0 || cam->image_height == 0) return 1;
    if (sc->n_spheres && (!sc->center || !sc->radius || !sc->material || !sc->materials)) return 1;
    for (uint32_t i = 0; i < sc->n_spheres; ++i)
        if (sc->material[i] >= sc->n_materials) return 1;
    scene_r_f64 S;
    S.n = sc->n_spheres;
    S.cx = (double*)malloc(sizeof(double) * (S.n + 1));
    S.cy = (double*)malloc(sizeof(double) * (S.n + 1));
    S.cz = (double*)malloc(sizeof(double) * (S.n + 1));
    S.r = (double*)malloc(sizeof(double) * (S.n + 1));
    double* r2s = (double*)malloc(sizeof(double) * (S.n + 1));
    S.mat = sc->material;
    S.mats = (mat_r_f64*)malloc(sizeof(mat_r_f64) * (sc->n_materials + 1));
    for (uint32_t i = 0; i < S.n; ++i) {
        S.cx[i] = sc->center[3 * i]; S.cy[i] = sc->center[3 * i + 1]; S.cz[i] = sc->center[3 * i + 2];
        S.r[i] = sc->radius[i];
        r2s[i] = S.r[i] * S.r[i];   /* radius.powi(2), objects.rs:256 */
    }
    for (uint32_t i = 0; i < sc->n_materials; ++i) {
        const or_material* m = &sc->materials[i];
        mat_r_f64* o = &S.mats[i];
        o->kind = m->kind; o->hollow = m->hollow;
        o->ar = m->albedo[0]; o->ag = m->albedo[1]; o->ab = m->albedo[2];
        o->fuzz = m->fuzz; o->ior = m->ior;
    }
    cam_r_f64 C = cam_to_r64(cam);
    pk_job J;
    memset(&J, 0, sizeof(J));
    J.S = &S; J.r2s = r2s; J.cam = &C; J.depth = max_bounces; J.spp = spp;
    J.k0 = (uint32_t)seed; J.k1 = (uint32_t)(seed >> 32);
    J.tile = tile;
    J.tiles_x = (cam->image_width + tile - 1) / tile;
    const uint32_t all = J.tiles_x * ((cam->image_height + tile - 1) / tile);
    J.tiles = tiles; J.n_tiles = tiles ? n_tiles : all;
    for (uint32_t i = 0; tiles && i < n_tiles; ++i)
        if (tiles[i] >= all) { free(S.cx); free(S.cy); free(S.cz); free(S.r); free(r2s); free(S.mats); return 1; }
    J.rgb = rgb_out; J.lin = lin_out;
    pthread_mutex_init(&J.mu, NULL);
    if (n_threads < 1) n_threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], NULL, pk_worker, &J);
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&J.mu);
    free(S.cx); free(S.cy); free(S.cz); free(S.r); free(r2s); free(S.mats);
    if (segments) *segments = J.segs;
    if (pixels_out) *pixels_out = J.pixels;
    return J.panic ? 3 : 0;
}
