// rt_kernel.hip — MI355X (gfx950) megakernel for the reference's per-pixel sample loop.
//
// Replaces TileRenderTask::render_vectorized2 (src/renderer.rs:141-176) and everything it
// calls: Camera::get_ray (ray_tracing.rs:77-89), Scene::trace_vectorized2
// (ray_tracing.rs:375-505), Sphere::hit_packed (objects.rs:249-290), PackedHitRecords
// (objects.rs:121-176), Material::get_hit_result (materials.rs:54-147), the final sky pass and
// reduction (ray_tracing.rs:486-504), /spp and Color::to_u8_array (renderer.rs:161,
// color.rs:54-64).
//
// Mapping:
//   * path regeneration: a persistent wave keeps one ray per lane from its camera ray to its
//     termination, then takes the next sample (of this pixel or of the next one its workgroup
//     claims from an atomic block counter; up to kSlots pixels in flight).  Every ray's bounce k depends only
//     on its own state and the counter-based RNG key (sample, pixel, k, stream), so no ray waits
//     for the others; lane utilisation is ~1.0.
//   * each sweep finds every sphere the reference could hit through conservative fp32 culls and
//     runs the reference's exact test on those only: spheres stream through the scalar cache in
//     64-byte groups (s_load_dwordx16 into SGPRs, a free broadcast to all 64 lanes), two spheres
//     per packed-FP32 instruction; bounced rays first slab-test 16-sphere cluster boxes, then a
//     per-sphere distance filter on the clusters some lane may hit (nearest_hit).
//   * pinhole cameras: primary rays run in full-wave camera batches; a cone around the batch's
//     rays culls clusters and spheres with lanes as spheres (camera_sweep), survivors get the
//     exact test from a per-launch camera-origin table (oc and c are the same for every primary
//     ray); hits wait in an LDS queue for free lanes.
//   * the reference's positions (its per-bounce stable shuffle) are a function of the per-sample
//     termination bounces alone; when a pixel's last sample ends, finish_pixel replays them,
//     applies quirk Q3's buffer read ("retire rule") and sums in the reference's order, so fp64
//     and fp32 results are bit-identical to the CPU restatement in oracle/.
//
// Source layout (one translation unit): rt_experiments.hpp (build kinds), rt_common.hpp (layouts,
// kernel arguments, scalar-load pipelines), rt_sweep.hpp (general sweep), rt_camera.hpp (primary
// rays, scatter), rt_finish.hpp (replay + reduction), rt_trace.hpp (the persistent kernel),
// rt_layout.hpp (host-side scene layout); this file holds the C ABI.
#include "rt_trace.hpp"
#include "rt_layout.hpp"

#include <chrono>
#include <mutex>
#include <string>

// ============================== host side ==============================
using namespace rt;

static thread_local std::string g_err;
static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(x)                                                                     \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev_first = nullptr, ev_last = nullptr;
    bool have_first = false;
    // scene, fp64 and fp32 images
    void* sph64 = nullptr; void* sph32 = nullptr;   // grouped sphere records
    void* fsph64 = nullptr; void* fsph32 = nullptr; // fp32 filter streams (for fp64 / fp32 rays)
    uint32_t n_fgroups = 0;
    float f_cmax64 = 0, f_r2max64 = 0, f_cmax32 = 0, f_r2max32 = 0, f_r2min64 = 0, f_r2min32 = 0;
    void* cam64 = nullptr; void* cam32 = nullptr;   // camera-origin tables (same size; rebuilt per launch)
    void* camf64 = nullptr; void* camf32 = nullptr; // camera filter tables (fp32 layout; rebuilt per launch)
    void* cen64 = nullptr; void* cen32 = nullptr;   // AoS centre tables
    void* camx64 = nullptr; void* camx32 = nullptr; // per-sphere camera-origin records (rebuilt per launch)
    void* cull64 = nullptr; void* cull32 = nullptr; // camera cone-cull records (fp32; rebuilt per launch)
    uint32_t n_cull = 0;                            // records: n_spheres rounded up to 64, + 64 padding
    void* rsph64 = nullptr; void* rsph32 = nullptr; // general sweep: slot-order exact groups
    void* rfsph64 = nullptr; void* rfsph32 = nullptr; // slot-order fp32 filter groups
    void* top64 = nullptr; void* top32 = nullptr;   // cluster bounds (fp32 top groups)
    void* sup64 = nullptr; void* sup32 = nullptr;   // super boxes (4 clusters each)
    void* meg64 = nullptr; void* meg32 = nullptr;   // mega boxes (4 supers each; big scenes only)
    void* lfs64 = nullptr; void* lfs32 = nullptr;   // cluster-local filter groups (big scenes only)
    void* lbx64[4] = {}; void* lbx32[4] = {};       // local box levels: cluster boxes, supers, megas, gigas
    uint32_t n_gg = 0;
    float l_r2max64 = 0, l_r2min64 = 0, l_r2max32 = 0, l_r2min32 = 0;
    uint32_t n_mg = 0;
    void* mtiers = nullptr;                         // the mega walk's order table (pack_mega_tiers)
    float mt_lo[3] = {0, 0, 0}, mt_inv = 0;
    uint32_t mt_n[3] = {1, 1, 1};
    uint32_t* ridx = nullptr;
    void* clus64 = nullptr; void* clus32 = nullptr;   // cluster bounding spheres {C, R} (double)
    void* cullc64 = nullptr; void* cullc32 = nullptr; // per-cluster camera cull records (rebuilt per launch)
    uint32_t n_cslots = 0, n_clp = 0;                 // slot-order cull records; cluster records (x64)
    uint32_t n_supc = 0;                              // super records after them (x64; 0: none)
    uint32_t n_top = 0, n_xg = 0, n_xs = 0;
    uint32_t n_groups64 = 0, n_groups32 = 0;
    void* mat64 = nullptr; void* mat32 = nullptr;     // per-sphere material records
    uint32_t n_spheres = 0, n_materials = 0;
    unsigned long long* segs = nullptr;
    uint32_t* err = nullptr;
    uint32_t* counter = nullptr;   // persistent-kernel claim-stream counters (zeroed before each launch)
    void* scratch = nullptr;       // per-wave ray state (grown on demand)
    size_t scratch_bytes = 0;
    int n_cu = 0;
    uint64_t samples = 0, pixels = 0;
    hipStream_t last_stream = nullptr;   // stream of the previous render (they share scratch and tables)
    bool have_last = false;
    // The camera tables of each precision (build_cam_table) depend only on the scene, the camera centre,
    // the scalar mode and RT_FILTER_OFF: a launch with the same key reuses them (bench frames, shards).
    uint64_t scene_gen = 0;
    struct CamKey { bool valid = false; uint64_t gen = 0; double center[3] = {0, 0, 0}; uint32_t scalar = 0, off = 0; };
    CamKey camkey[2];   // [0] fp32 tables, [1] fp64
    uint32_t last_kernel_id = 0, last_wg_per_cu = 0;   // rt_stats.kernel_id / kernel_wg_per_cu of the last launch
};

extern "C" const char* rt_last_error(void) { return g_err.c_str(); }
// "rt_mi355x <version> gfx950 <product|experiment> src=<hash of the sources it was built from>"
extern "C" const char* rt_version(void) { return "rt_mi355x 0.3 gfx950 " RT_BUILD_KIND " src=" RT_SRC_HASH; }

extern "C" double rt_metal_clamp_fuzz(double fuzz) { return fuzz < 1.0 ? fuzz : 1.0; }

// Camera::new, ray_tracing.rs:27-62 (f64, Vec3 ops without FMA; compiled -ffp-contract=off).
extern "C" int rt_camera_new(rt_camera* out, uint32_t w, uint32_t h, double focal_length, double view_angle_deg,
                             const double center[3], const double look_at[3], const double up[3],
                             double defocus_angle_deg) {
    if (!out || !center || !look_at || !up || w == 0 || h == 0) return fail(RT_ERR_INVALID, "rt_camera_new: bad argument");
    const double rads_per_deg = 3.141592653589793 / 180.0;              // f64::to_radians
    const double aspect = (double)w / (double)h;                         // :28
    const double vh = std::tan((view_angle_deg * rads_per_deg) / 2.0) * focal_length * 2.0;  // :29
    const double vw = vh * aspect;                                       // :32
    auto unit3 = [](const double a[3], double o[3]) {
        const double l = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
        o[0] = a[0] / l; o[1] = a[1] / l; o[2] = a[2] / l;
    };
    double dirv[3] = {look_at[0] - center[0], look_at[1] - center[1], look_at[2] - center[2]};
    double dir[3]; unit3(dirv, dir);                                     // :34
    const double wv[3] = {-dir[0], -dir[1], -dir[2]};                    // :35
    const double cr[3] = {up[1] * wv[2] - up[2] * wv[1], up[2] * wv[0] - up[0] * wv[2], up[0] * wv[1] - up[1] * wv[0]};
    double u[3]; unit3(cr, u);                                           // :36
    const double v[3] = {wv[1] * u[2] - wv[2] * u[1], wv[2] * u[0] - wv[0] * u[2], wv[0] * u[1] - wv[1] * u[0]};  // :37
    const double dr = focal_length * std::tan((defocus_angle_deg / 2.0) * rads_per_deg);  // :43
    out->image_width = w; out->image_height = h;
    for (int i = 0; i < 3; ++i) {
        out->center[i] = center[i];
        out->vu[i] = u[i] * vw;                                          // :39
        out->vv[i] = (-v[i]) * vh;                                       // :40
        out->ulc[i] = ((center[i] - wv[i] * focal_length) - out->vu[i] / 2.0) - out->vv[i] / 2.0;  // :41
        out->du[i] = u[i] * dr;                                          // :44
        out->dv[i] = v[i] * dr;                                          // :45
    }
    return RT_OK;
}

extern "C" int rt_context_create(int device, rt_context** out) {
    if (!out) return fail(RT_ERR_INVALID, "rt_context_create: out is NULL");
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(RT_ERR_INVALID, "rt_context_create: no such device");
    HIPCHK(hipSetDevice(device));
    rt_context* c = new rt_context();
    c->device = device;
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev_first));
    HIPCHK(hipEventCreate(&c->ev_last));
    HIPCHK(hipMalloc((void**)&c->segs, sizeof(unsigned long long) * kSegShards * kSegStride));
    HIPCHK(hipMalloc((void**)&c->err, 16));
    HIPCHK(hipMalloc((void**)&c->counter, kStreams * kCtrStride * sizeof(uint32_t)));   // claim streams (rt_trace.hpp)
    HIPCHK(hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device));
    HIPCHK(hipMemset(c->segs, 0, sizeof(unsigned long long) * kSegShards * kSegStride));
    HIPCHK(hipMemset(c->err, 0, 16));
    *out = c;
    return RT_OK;
}

static void free_scene(rt_context* c) {
    (void)hipFree(c->sph64); (void)hipFree(c->sph32); (void)hipFree(c->mat64); (void)hipFree(c->mat32);
    (void)hipFree(c->cam64); (void)hipFree(c->cam32);
    c->cam64 = c->cam32 = nullptr;
    (void)hipFree(c->camf64); (void)hipFree(c->camf32);
    c->camf64 = c->camf32 = nullptr;
    (void)hipFree(c->fsph64); (void)hipFree(c->fsph32);
    c->fsph64 = c->fsph32 = nullptr;
    (void)hipFree(c->cen64); (void)hipFree(c->cen32);
    (void)hipFree(c->camx64); (void)hipFree(c->camx32); (void)hipFree(c->cull64); (void)hipFree(c->cull32);
    c->camx64 = c->camx32 = c->cull64 = c->cull32 = nullptr;
    (void)hipFree(c->rsph64); (void)hipFree(c->rsph32); (void)hipFree(c->rfsph64); (void)hipFree(c->rfsph32);
    (void)hipFree(c->top64); (void)hipFree(c->top32); (void)hipFree(c->ridx);
    (void)hipFree(c->sup64); (void)hipFree(c->sup32);
    c->sup64 = c->sup32 = nullptr;
    (void)hipFree(c->meg64); (void)hipFree(c->meg32);
    (void)hipFree(c->lfs64); (void)hipFree(c->lfs32);
    c->lfs64 = c->lfs32 = nullptr;
    for (int lv = 0; lv < 4; ++lv) {
        (void)hipFree(c->lbx64[lv]); (void)hipFree(c->lbx32[lv]);
        c->lbx64[lv] = c->lbx32[lv] = nullptr;
    }
    c->meg64 = c->meg32 = nullptr;
    c->n_mg = 0;
    c->n_gg = 0;
    (void)hipFree(c->mtiers);
    c->mtiers = nullptr;
    (void)hipFree(c->clus64); (void)hipFree(c->clus32); (void)hipFree(c->cullc64); (void)hipFree(c->cullc32);
    c->clus64 = c->clus32 = c->cullc64 = c->cullc32 = nullptr;
    c->n_cslots = c->n_clp = c->n_supc = 0;
    c->rsph64 = c->rsph32 = c->rfsph64 = c->rfsph32 = c->top64 = c->top32 = nullptr;
    c->ridx = nullptr;
    c->n_top = c->n_xg = c->n_xs = 0;
    c->sph64 = c->sph32 = c->mat64 = c->mat32 = c->cen64 = c->cen32 = nullptr;
    c->n_spheres = c->n_materials = 0;
}

extern "C" int rt_context_destroy(rt_context* c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    (void)hipFree(c->segs); (void)hipFree(c->err); (void)hipFree(c->counter); (void)hipFree(c->scratch);
    (void)hipEventDestroy(c->ev_first); (void)hipEventDestroy(c->ev_last);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return RT_OK;
}

extern "C" int rt_context_set_scene(rt_context* c, const rt_scene* s) {
    if (!c || !s) return fail(RT_ERR_INVALID, "rt_context_set_scene: NULL argument");
    if (s->n_spheres && (!s->center || !s->radius || !s->material || !s->materials))
        return fail(RT_ERR_INVALID, "rt_context_set_scene: NULL array");
    for (uint32_t i = 0; i < s->n_spheres; ++i)
        if (s->material[i] >= s->n_materials)
            return fail(RT_ERR_INVALID, "rt_context_set_scene: material index out of range (objects.rs:296 would panic)");
    for (uint32_t i = 0; i < s->n_materials; ++i)
        if (s->materials[i].kind > RT_DIELECTRIC)
            return fail(RT_ERR_INVALID, "rt_context_set_scene: unknown material kind (materials.rs:31 would panic)");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    free_scene(c);
    ++c->scene_gen;   // camera tables built for the previous scene are stale
    c->camkey[0].valid = c->camkey[1].valid = false;
    std::vector<double> g64, c64; std::vector<MatT<double>> m64;
    std::vector<float> g32, c32; std::vector<MatT<float>> m32;
    pack_scene(s, g64, c64, m64, c->n_groups64);
    pack_scene(s, g32, c32, m32, c->n_groups32);
    std::vector<uint32_t> sm(s->n_spheres ? s->n_spheres : 1, 0);
    for (uint32_t i = 0; i < s->n_spheres; ++i) sm[i] = s->material[i];
    auto up = [&](void** dst, const void* src, size_t bytes) -> int {
        HIPCHK(hipMalloc(dst, bytes));
        HIPCHK(hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
        return RT_OK;
    };
    int rc;
    if ((rc = up(&c->sph64, g64.data(), g64.size() * sizeof(double))) != RT_OK) return rc;
    if ((rc = up(&c->sph32, g32.data(), g32.size() * sizeof(float))) != RT_OK) return rc;
    {
        std::vector<float> f64g, f32g, fr64, fr32;
        uint32_t nf = 0;
        pack_filter(c64, s->n_spheres, f64g, nf, c->f_cmax64, c->f_r2max64, c->f_r2min64, fr64);
        pack_filter(c32, s->n_spheres, f32g, c->n_fgroups, c->f_cmax32, c->f_r2max32, c->f_r2min32, fr32);
        if ((rc = up(&c->fsph64, f64g.data(), f64g.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->fsph32, f32g.data(), f32g.size() * sizeof(float))) != RT_OK) return rc;
        const SweepLayout L = build_layout(s);
        std::vector<double> rg64; std::vector<float> rg32, rf64, rf32, t64, t32, s64, s32, m64, m32;
        std::vector<float> lf64, lf32, lr64, lr32;   // the mega kernels' local streams (uploaded inline below)
        pack_sweep(c64, fr64, L, rg64, rf64, t64, c->f_cmax64, c->f_r2max64, s64, m64);
        pack_sweep(c32, fr32, L, rg32, rf32, t32, c->f_cmax32, c->f_r2max32, s32, m32);
        if ((rc = up(&c->sup64, s64.data(), s64.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->sup32, s32.data(), s32.size() * sizeof(float))) != RT_OK) return rc;
        c->n_mg = m32.empty() ? 0u : (uint32_t)(m32.size() / kBoxFloats - 1);   // groups, without the empty one
        if (c->n_mg) {
            if ((rc = up(&c->meg64, m64.data(), m64.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->meg32, m32.data(), m32.size() * sizeof(float))) != RT_OK) return rc;
            std::vector<float> q64, q32;
            pack_local(c64, L, t64, lf64, lr64, q64);
            pack_local(c32, L, t32, lf32, lr32, q32);
            std::vector<float> b64[4], b32[4];
            pack_local_boxes(c64, L, q64, b64[0], b64[1], b64[2], b64[3], c->l_r2max64, c->l_r2min64);
            std::vector<float> wme;
            pack_local_boxes(c32, L, q32, b32[0], b32[1], b32[2], b32[3], c->l_r2max32, c->l_r2min32, &wme);
            c->n_gg = L.giga && c->n_mg <= 16u ? (c->n_mg + 3u) / 4u : 0u;
            {
                const MegaTiers M = pack_mega_tiers(wme, (L.members.size() / 4 + 3) / 4);
                if ((rc = up(&c->mtiers, M.t.data(), M.t.size() * sizeof(uint64_t))) != RT_OK) return rc;
                for (int a = 0; a < 3; ++a) { c->mt_lo[a] = M.lo[a]; c->mt_n[a] = M.n[a]; }
                c->mt_inv = M.inv;
            }
            for (int lv = 0; lv < 4; ++lv) {
                if ((rc = up(&c->lbx64[lv], b64[lv].data(), b64[lv].size() * sizeof(float))) != RT_OK) return rc;
                if ((rc = up(&c->lbx32[lv], b32[lv].data(), b32[lv].size() * sizeof(float))) != RT_OK) return rc;
            }
        }
        c->n_top = (uint32_t)(L.members.size() / 4);
        c->n_xg = L.n_xg;
        c->n_xs = L.n_xs;
        // slot -> scene index (0xFFFFFFFF: dummy), padded past the last cluster by one block of 64
        // (the camera sweep's empty quarters read the slots of cluster index n_clusters)
        const uint32_t ncl = (uint32_t)L.members.size();
        c->n_cslots = 4u * L.n_xg + 16u * ncl + 64u;
        c->n_clp = (ncl + 63u) / 64u * 64u;
        std::vector<uint32_t> ridx(c->n_cslots, 0xFFFFFFFFu);
        for (size_t i = 0; i < L.slot.size(); ++i) if (L.slot[i] >= 0) ridx[i] = (uint32_t)L.slot[i];
        // cluster bounding spheres for the camera cull, per precision: centre = the members' AABB
        // centre, R >= max |c_i - C| + |r_i| over the members' T-precision centres and radii.  Scenes
        // with more than 128 clusters (config E) also get super records, the bounding spheres of the
        // 4 clusters of each super (camera_sweep tests them first), stored after the cluster records.
        const uint32_t nsup = ncl / 4u;
        c->n_supc = ncl > 128u ? (nsup + 63u) / 64u * 64u : 0u;
        auto bounds = [&](auto const& cen, std::vector<double>& out) {
            out.assign((size_t)4 * ((c->n_clp + c->n_supc) ? c->n_clp + c->n_supc : 1), 0.0);
            for (size_t k = 0; k < out.size() / 4; ++k) out[4 * k + 3] = -INFINITY;
            auto sphere = [&](size_t at, uint32_t k0, uint32_t nk) {   // the members of clusters k0 .. k0+nk-1
                double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                bool any = false;
                for (uint32_t k = k0; k < k0 + nk; ++k)
                    for (uint32_t i : L.members[k]) {
                        any = true;
                        for (int a = 0; a < 3; ++a) {
                            const double r = std::fabs((double)cen[4 * i + 3]);
                            lo[a] = std::min(lo[a], (double)cen[4 * i + a] - r);
                            hi[a] = std::max(hi[a], (double)cen[4 * i + a] + r);
                        }
                    }
                if (!any) return;
                double C[3], R = 0.0;
                for (int a = 0; a < 3; ++a) C[a] = 0.5 * (lo[a] + hi[a]);
                for (uint32_t k = k0; k < k0 + nk; ++k)
                    for (uint32_t i : L.members[k]) {
                        const double dx = (double)cen[4 * i] - C[0], dy = (double)cen[4 * i + 1] - C[1],
                                     dz = (double)cen[4 * i + 2] - C[2];
                        R = std::max(R, std::sqrt(dx * dx + dy * dy + dz * dz) + std::fabs((double)cen[4 * i + 3]));
                    }
                out[4 * at] = C[0]; out[4 * at + 1] = C[1]; out[4 * at + 2] = C[2];
                out[4 * at + 3] = std::isfinite(R) ? R * (1.0 + 0x1.0p-40) : INFINITY;
            };
            for (uint32_t k = 0; k < ncl; ++k) sphere(k, k, 1);
            if (c->n_supc)
                for (uint32_t k = 0; k < nsup; ++k) sphere(c->n_clp + k, 4 * k, 4);
        };
        std::vector<double> cl64, cl32;
        bounds(c64, cl64);
        bounds(c32, cl32);
        if ((rc = up(&c->clus64, cl64.data(), cl64.size() * sizeof(double))) != RT_OK) return rc;
        if ((rc = up(&c->clus32, cl32.data(), cl32.size() * sizeof(double))) != RT_OK) return rc;
        HIPCHK(hipMalloc(&c->cullc64, cl64.size() / 4 * 4 * sizeof(float)));
        HIPCHK(hipMalloc(&c->cullc32, cl32.size() / 4 * 4 * sizeof(float)));
        if ((rc = up(&c->rsph64, rg64.data(), rg64.size() * sizeof(double))) != RT_OK) return rc;
        if ((rc = up(&c->rsph32, rg32.data(), rg32.size() * sizeof(float))) != RT_OK) return rc;
        // General-sweep filter streams, inline layout (nearest_hit): the always-exact groups, then per cluster its 4
        // filter groups, 4 records of 8 words {r^2 of pair 0 (2), r^2 of pair 1 (2), 4 scene indices} (r^2: the
        // fp32 scene-frame stream, whose exact test takes the centres from the filter group; in the mega kernels'
        // local streams the r^2 words of records 0 and 1 hold the cluster's frame record); then a dummy group (the
        // loop's prefetch).  96 floats per cluster keep every group on its own 64-byte line.  A
        // taken group's record and a walked cluster's frame are loads from the pointer the walk already holds.
        auto inline_stream = [&](const std::vector<float>& src, bool r2, const std::vector<float>* frame) {
            const size_t blk = 96, ngf = src.size() / 16 - 1, nxg = c->n_xg, nk = (ngf - nxg) / 4;
            std::vector<float> rx((size_t)16 * nxg + blk * nk + 32, 0.0f);
            for (size_t g = 0; g < 16 * nxg; ++g) rx[g] = src[g];
            for (size_t k = 0; k < nk; ++k) {
                float* b = &rx[16 * nxg + blk * k];
                for (size_t j = 0; j < 64; ++j) b[j] = src[16 * (nxg + 4 * k) + j];
                for (size_t q = 0; q < 4; ++q) {
                    const size_t g = nxg + 4 * k + q;
                    uint32_t rec[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
                    if (r2) for (int h = 0; h < 4; ++h) memcpy(&rec[h], &rg32[16 * g + 8 * (h / 2) + 6 + (h % 2)], 4);
                    for (int j = 0; j < 4; ++j) rec[4 + j] = 4 * g + j < ridx.size() ? ridx[4 * g + j] : 0xFFFFFFFFu;
                    memcpy(b + 64 + 8 * q, rec, 32);
                }
                if (frame) for (size_t j = 0; j < 4; ++j) { b[64 + j] = (*frame)[8 * k + j]; b[72 + j] = (*frame)[8 * k + 4 + j]; }
            }
            for (size_t j = 0; j < 16; ++j) rx[16 * nxg + blk * nk + j] = src[16 * ngf + j];   // the dummy group
            return rx;
        };
        {
            const std::vector<float> rx32 = inline_stream(rf32, true, nullptr), rx64 = inline_stream(rf64, false, nullptr);
            if ((rc = up(&c->rfsph32, rx32.data(), rx32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->rfsph64, rx64.data(), rx64.size() * sizeof(float))) != RT_OK) return rc;
        }
        if (c->n_mg) {
            const std::vector<float> lx32 = inline_stream(lf32, false, &lr32), lx64 = inline_stream(lf64, false, &lr64);
            if ((rc = up(&c->lfs32, lx32.data(), lx32.size() * sizeof(float))) != RT_OK) return rc;
            if ((rc = up(&c->lfs64, lx64.data(), lx64.size() * sizeof(float))) != RT_OK) return rc;
        }
        if ((rc = up(&c->top64, t64.data(), t64.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up(&c->top32, t32.data(), t32.size() * sizeof(float))) != RT_OK) return rc;
        if ((rc = up((void**)&c->ridx, ridx.data(), ridx.size() * sizeof(uint32_t))) != RT_OK) return rc;
        HIPCHK(hipMalloc(&c->camf64, f64g.size() * sizeof(float)));
        HIPCHK(hipMalloc(&c->camf32, f32g.size() * sizeof(float)));
    }
    HIPCHK(hipMalloc(&c->cam64, g64.size() * sizeof(double)));
    HIPCHK(hipMalloc(&c->cam32, g32.size() * sizeof(float)));
    c->n_cull = (s->n_spheres + 63u) / 64u * 64u + 64u;
    HIPCHK(hipMalloc(&c->camx64, (size_t)4 * c->n_cslots * sizeof(double)));
    HIPCHK(hipMalloc(&c->camx32, (size_t)4 * c->n_cslots * sizeof(float)));
    HIPCHK(hipMalloc(&c->cull64, (size_t)4 * c->n_cslots * sizeof(float)));
    HIPCHK(hipMalloc(&c->cull32, (size_t)4 * c->n_cslots * sizeof(float)));
    if ((rc = up(&c->cen64, c64.data(), c64.size() * sizeof(double))) != RT_OK) return rc;
    if ((rc = up(&c->cen32, c32.data(), c32.size() * sizeof(float))) != RT_OK) return rc;
    {
        // per-sphere records: next_ray gathers a hit sphere's material in one dependent load
        std::vector<MatT<double>> s64(sm.size());
        std::vector<MatT<float>> s32(sm.size());
        for (size_t i = 0; i < sm.size(); ++i)
            if (sm[i] < m64.size()) { s64[i] = m64[sm[i]]; s32[i] = m32[sm[i]]; }
        if ((rc = up(&c->mat64, s64.data(), s64.size() * sizeof(MatT<double>))) != RT_OK) return rc;
        if ((rc = up(&c->mat32, s32.data(), s32.size() * sizeof(MatT<float>))) != RT_OK) return rc;
    }
    c->n_spheres = s->n_spheres;
    c->n_materials = s->n_materials;
    return RT_OK;
}

static bool check_range(const rt_camera* cam, const rt_tile_range* r) {
    if (r->row_count == 0 || r->col_count == 0 || r->row_step == 0) return false;
    if (r->col_begin + (uint64_t)r->col_count > cam->image_width) return false;
    const uint64_t last_row = r->row_begin + (uint64_t)(r->row_count - 1) * r->row_step;
    return last_row < cam->image_height;
}

static int ensure_scratch(rt_context* c, size_t bytes, hipStream_t st);

// The kernel instantiation for (flags, waves-per-SIMD target, camera batches, mega level).  W < 0:
// the defaults (RT_WAVES unset).  The mega level (scenes with more than 8 super groups) has its own
// live-path kernels (fp32 at 5 or 6 waves, default 6; fp64 at 4); at other W such scenes are swept
// from the super boxes (the same result, more box tests).  id: rt_stats.kernel_id (rt_mi355x.h).
template <typename T> struct KernelPick {
    void (*fn)(KParams<T>);
    uint32_t id;
    int W;
};
template <typename T, int W, bool ROOT2, int MODE, bool CAMQ, bool MEGA = false>
static KernelPick<T> kp() {
    const uint32_t id = 0x8000u | (sizeof(T) == 8 ? 1u : 0u) | ((uint32_t)W << 1) | (ROOT2 ? 1u << 4 : 0u) |
                        ((uint32_t)MODE << 5) | (CAMQ ? 1u << 7 : 0u) | (MEGA ? 1u << 8 : 0u);
    return KernelPick<T>{trace_paths<T, W, ROOT2, MODE, CAMQ, MEGA>, id, W};
}
template <typename T, bool CAMQ>
static KernelPick<T> pick_kernel(uint32_t flags, int W, bool mega, bool big) {
    const bool r2 = (flags & RT_FLAG_ROOT2) != 0u;
    constexpr bool F32 = sizeof(T) == 4;
    constexpr int WM = kWavesModes<T>;
    if (flags & RT_FLAG_MODE_SCALAR) return kp<T, WM, false, kModeScalar, CAMQ>();
    if (flags & RT_FLAG_MODE_VECTORIZED3)
        return r2 ? kp<T, WM, true, kModeV3, CAMQ>() : kp<T, WM, false, kModeV3, CAMQ>();
    if (flags & RT_FLAG_MODE_VECTORIZED)
        return r2 ? kp<T, WM, true, kModeV1, CAMQ>() : kp<T, WM, false, kModeV1, CAMQ>();
    if (r2) return kp<T, WM, true, kModeV2, CAMQ>();
    if (mega) {
        const int Wm = W < 0 ? (F32 ? (big ? kWavesMegaF32 : 5) : kWavesF64) : W;
        if constexpr (F32) {
            if (Wm == 5) return kp<T, 5, false, kModeV2, CAMQ, true>();
            if (Wm == 6) return kp<T, 6, false, kModeV2, CAMQ, true>();
        } else {
            if (Wm == 4) return kp<T, 4, false, kModeV2, CAMQ, true>();
        }
    }
    if (W < 0) W = F32 ? (big ? kWavesF32 : 5) : kWavesF64;
    // RT_WAVES above what the kernel's LDS allows is clamped: fp32 6 (round 2's W7 build lost its
    // seventh workgroup to the camera lists and the parking: 5 resident), fp64 5 (its W6 build: 3)
    if constexpr (F32) {
        return W >= 6 ? kp<T, 6, false, kModeV2, CAMQ>() : W >= 5 ? kp<T, 5, false, kModeV2, CAMQ>()
                                                         : kp<T, 4, false, kModeV2, CAMQ>();
    } else {
        return W >= 5 ? kp<T, 5, false, kModeV2, CAMQ>() : kp<T, 4, false, kModeV2, CAMQ>();
    }
}

template <typename T>
static int launch_t(rt_context* c, const rt_camera* cam, uint32_t depth, uint32_t spp, uint64_t seed, uint32_t flags,
                    const rt_tile_range& rg, void* d_rgb, void* d_lin, hipStream_t st) {
    KParams<T> p;
    memset(&p, 0, sizeof(p));
    const bool f64 = sizeof(T) == 8;
    p.sph = (const T*)(f64 ? c->sph64 : c->sph32);
    p.cen = (const T*)(f64 ? c->cen64 : c->cen32);
    p.n_groups = f64 ? c->n_groups64 : c->n_groups32;
    p.fsph = (const float*)(f64 ? c->fsph64 : c->fsph32);
    p.n_fgroups = c->n_fgroups;
    p.rsph = (const T*)(f64 ? c->rsph64 : c->rsph32);
    p.rfsph = (const float*)(f64 ? c->rfsph64 : c->rfsph32);
    p.ftop = (const float*)(f64 ? c->top64 : c->top32);
    p.fsup = (const float*)(f64 ? c->sup64 : c->sup32);
    p.fmeg = (const float*)(f64 ? c->meg64 : c->meg32);
    p.n_mg = c->n_mg;
    p.lfsph = (const float*)(f64 ? c->lfs64 : c->lfs32);
    p.lclb = (const float*)(f64 ? c->lbx64[0] : c->lbx32[0]);
    p.lsup = (const float*)(f64 ? c->lbx64[1] : c->lbx32[1]);
    p.lmeg = (const float*)(f64 ? c->lbx64[2] : c->lbx32[2]);
    p.lgig = (const float*)(f64 ? c->lbx64[3] : c->lbx32[3]);
    p.n_gg = c->n_gg;
    p.mtiers = (const uint64_t*)c->mtiers;
    for (int a = 0; a < 3; ++a) { p.mt_lo[a] = c->mt_lo[a]; p.mt_n[a] = c->mt_n[a]; }
    p.mt_inv = c->mt_inv;
    {
        auto up32 = [](double v) -> float {
            float f = (float)v;
            if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
            return f;
        };
        const double r2m = (double)(f64 ? c->l_r2min64 : c->l_r2min32);
        p.l_r2max = f64 ? c->l_r2max64 : c->l_r2max32;
        p.l_hir2 = up32((double)kFilterMargin * 0.5 / r2m);
        p.l_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m));
    }
    p.ridx = c->ridx;
    p.n_top = c->n_top;
    p.n_xg = c->n_xg;
    p.n_xs = c->n_xs;
    p.f_cmax = f64 ? c->f_cmax64 : c->f_cmax32;
    p.f_r2max = f64 ? c->f_r2max64 : c->f_r2max32;
    p.f_r2min = f64 ? c->f_r2min64 : c->f_r2min32;
    {
        auto up32 = [](double v) -> float {
            float f = (float)v;
            if ((double)f < v) f = std::nextafter(f, std::numeric_limits<float>::infinity());
            return f;
        };
        const double r2m = (double)p.f_r2min;   // 0 (no filtered sphere) gives +inf: every basis is zero
        p.f_ir2 = up32(1.0 / r2m);
        p.f_hir2 = up32(0.5 / r2m);
        p.f_isr = up32(8.0 * 0x1.0p-24 / std::sqrt(r2m));
    }
    bool filter_off = false;
    {   // diagnostics: every general-sweep and camera-sweep group through the exact test
        const char* e = getenv("RT_FILTER_OFF");
        filter_off = e && atoi(e) != 0;
        if (filter_off) p.f_cmax = std::numeric_limits<float>::infinity();
    }
    p.mats = (const MatT<T>*)(f64 ? c->mat64 : c->mat32);
    p.n_spheres = c->n_spheres;
    p.W = cam->image_width; p.H = cam->image_height;
    p.rW = p.W < (1u << 20) ? 1.0 / (double)p.W : 0.0;   // div_dim
    p.rH = p.H < (1u << 20) ? 1.0 / (double)p.H : 0.0;
    for (int i = 0; i < 3; ++i) {
        p.center[i] = (T)cam->center[i]; p.ulc[i] = (T)cam->ulc[i]; p.vu[i] = (T)cam->vu[i];
        p.vv[i] = (T)cam->vv[i]; p.du[i] = (T)cam->du[i]; p.dv[i] = (T)cam->dv[i];
    }
    p.spp = spp;
    p.C = (spp + 3) / 4;
    p.P = 4 * p.C;
    p.depth = depth;
    p.flags = flags;
    {
        bool pinhole = true;
        for (int i = 0; i < 3; ++i) {
            if (p.du[i] != T(0) || p.dv[i] != T(0)) pinhole = false;
            if (p.center[i] == T(0) && std::signbit(p.center[i])) pinhole = false;
        }
        if (pinhole) p.flags |= kFlagPinholeInternal;
    }
    p.s_sel = (p.C - 1) % 2;   // ray_tracing.rs:486
    // fp64: Philox4x32-10 keyed by (seed lo, seed hi).  fp32: Philox2x32-10 has a 32-bit key, folded here as
    // seed lo ^ fmix32(seed hi) (rng<float> reads k0 only): fmix32(0) = 0, so a seed below 2^32 keys as itself,
    // and seeds such as (m << 32) | m no longer all key as 0.
    if (f64) { p.k0 = (uint32_t)seed; p.k1 = (uint32_t)(seed >> 32); }
    else { p.k0 = (uint32_t)seed ^ fmix32((uint32_t)(seed >> 32)); p.k1 = 0u; }
    p.row_begin = rg.row_begin; p.row_step = rg.row_step; p.col_begin = rg.col_begin; p.col_count = rg.col_count;
    p.rgb = (uint8_t*)d_rgb;
    p.lin = (double*)d_lin;
    p.segs = c->segs;
    p.err = c->err;
    p.counter = c->counter;
    p.n_items = rg.row_count * rg.col_count;

    // Persistent grid: as many 4-wave workgroups as stay resident, never more waves than pixels.
    // Minimum waves per SIMD the register allocation targets.  RT_WAVES (4..7; read at every
    // launch, so one process can compare them) overrides it for the live-path kernels (pinhole and
    // defocus cameras); the ROOT2 and semantics-mode kernels always run at kWavesModes.
    const char* waves_env = getenv("RT_WAVES");
    const int W = waves_env && atoi(waves_env) > 0 ? atoi(waves_env) : -1;
    // Camera batches + camera-origin table when every primary ray starts at the centre.
    const bool camq = (p.flags & kFlagPinholeInternal) && depth >= 1u;
    const bool big = (uint64_t)p.n_items >= kW6PixelsPerWave * 24u * (uint64_t)c->n_cu;   // 24 W6 waves per CU
    const KernelPick<T> pick = camq ? pick_kernel<T, true>(flags, W, p.n_mg > 0, big)
                                    : pick_kernel<T, false>(flags, W, p.n_mg > 0, big);
    void (*kern)(KParams<T>) = pick.fn;
    if (camq) {
        p.camsph = (const T*)(f64 ? c->cam64 : c->cam32);
        p.camf = (const float*)(f64 ? c->camf64 : c->camf32);
        p.camx = (const T*)(f64 ? c->camx64 : c->camx32);
        p.cull = (const float*)(f64 ? c->cull64 : c->cull32);
        const uint32_t n_slots = (p.n_groups + 1) * kGroup<T>, n_fslots = (p.n_fgroups + 1) * 4;
        p.cullc = (const float*)(f64 ? c->cullc64 : c->cullc32);
        p.n_clp = c->n_clp;
        p.n_supc = c->n_supc;
        const uint32_t n_thr = std::max(std::max(std::max(n_slots, n_fslots), c->n_cull),
                                        std::max(c->n_cslots, c->n_clp + c->n_supc));
        rt_context::CamKey& ck = c->camkey[f64 ? 1 : 0];
        const uint32_t scalar = (flags & RT_FLAG_MODE_SCALAR) ? 1u : 0u;
        double cen[3] = {(double)p.center[0], (double)p.center[1], (double)p.center[2]};
        const bool same = ck.valid && ck.gen == c->scene_gen && ck.scalar == scalar && ck.off == (uint32_t)filter_off &&
                          memcmp(ck.center, cen, sizeof(cen)) == 0;   // bit for bit (-0 is not +0)
        if (!same) {
            auto build = scalar ? build_cam_table<T, true> : build_cam_table<T, false>;
            hipLaunchKernelGGL(build, dim3((n_thr + 255) / 256), dim3(256), 0, st, p.sph, (T*)p.camsph, n_slots,
                               (float*)p.camf, n_fslots, p.center[0], p.center[1], p.center[2], (uint32_t)filter_off,
                               (T*)p.camx, (float*)p.cull, c->n_cull, c->n_spheres, c->ridx, c->n_cslots,
                               (const double*)(f64 ? c->clus64 : c->clus32), (float*)p.cullc, c->n_clp + c->n_supc);
            HIPCHK(hipGetLastError());
            ck.valid = true;
            ck.gen = c->scene_gen;
            ck.scalar = scalar;
            ck.off = (uint32_t)filter_off;
            memcpy(ck.center, cen, sizeof(cen));
        }
    }
    int per_cu = 0;
    HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 256, 0));
    if (per_cu < 1) per_cu = 1;
    // 4-wave workgroups: W waves per SIMD is W workgroups per CU.  Fewer means the kernel's LDS (or
    // registers) cut its occupancy below the target it was built for (kParkC takes fp32 W6 to 26.8 of the
    // 27.3 KB six workgroups allow): an error, in every build kind, so that neither the product nor an
    // A/B build is ever measured at an occupancy other than the one it names (rt_stats reports both).
    c->last_kernel_id = 0;   // 0: no kernel (ids have bit 15 set)
    c->last_wg_per_cu = 0;
    if (per_cu < pick.W)
        return fail(RT_ERR_UNSUPPORTED, std::string(RT_BUILD_KIND) + " build: " + std::to_string(per_cu) +
                                            " workgroups per CU resident, kernel built for " + std::to_string(pick.W) +
                                            " (its LDS or registers grew past the occupancy target)");
    c->last_kernel_id = pick.id;   // only a kernel that passed the check is ever reported
    c->last_wg_per_cu = (uint32_t)per_cu;
    uint64_t nblocks = (uint64_t)c->n_cu * (uint64_t)per_cu;
    const uint64_t need = ((uint64_t)p.n_items + 3) / 4;
    if (nblocks > need) nblocks = need;
    {   // G: the largest power of two <= min(kMaxBlock, kBlockSamples / spp, pixels per wave / kBlockShare),
        // raised to kClaimSpp / spp (claim rate, below) where the share bound would go under it
        const uint64_t per_wave = (uint64_t)p.n_items / (4u * nblocks);
        const uint64_t g = std::max<uint64_t>({1u, std::min<uint64_t>({(uint64_t)kMaxBlock, kBlockSamples / spp,
                                                                       per_wave / kBlockShare}),
                                               std::min<uint64_t>((uint64_t)kMaxBlock, (kClaimSpp + spp - 1) / spp)});
        uint32_t G = 1;
        while (2u * G <= g) G *= 2u;
        // diagnostics (tools/waves_ab.py --block): RT_BLOCK_G overrides the largest block (1..16, a power of two)
        const char* ge = getenv("RT_BLOCK_G");
        if (ge && atoi(ge) >= 1 && atoi(ge) <= (int)kMaxBlock && (atoi(ge) & (atoi(ge) - 1)) == 0) G = (uint32_t)atoi(ge);
        p.blk_g = G;
    }
    p.swide = paths_wide(p.P, depth);
    p.vbytes = paths_vbytes(p.P, p.swide, (flags & RT_FLAG_MODE_VECTORIZED3) != 0u);
    p.sbytes = paths_sbytes(p.P, sizeof(T), p.swide);
    p.scratch_stride = (size_t)p.vbytes + (size_t)kSlots * p.sbytes;
    // Keep the scratch within a fixed budget: fewer resident waves for very large spp.
    const uint64_t kScratchBudget = 24ull << 30;
    const uint64_t max_blocks = kScratchBudget / (4 * p.scratch_stride);
    if (nblocks > max_blocks) nblocks = max_blocks > 0 ? max_blocks : 1;
    const int rc = ensure_scratch(c, p.scratch_stride * nblocks * 4, st);
    if (rc != RT_OK) return rc;
    p.scratch = (char*)c->scratch;
    HIPCHK(hipMemsetAsync(c->counter, 0, kStreams * kCtrStride * sizeof(uint32_t), st));
    hipLaunchKernelGGL(kern, dim3((uint32_t)nblocks), dim3(256), 0, st, p);
    HIPCHK(hipGetLastError());
    return RT_OK;
}

static int ensure_scratch(rt_context* c, size_t bytes, hipStream_t st) {
    if (bytes <= c->scratch_bytes) return RT_OK;
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipDeviceSynchronize());
    if (c->scratch) HIPCHK(hipFree(c->scratch));
    c->scratch = nullptr;
    c->scratch_bytes = 0;
    HIPCHK(hipMalloc(&c->scratch, bytes));
    c->scratch_bytes = bytes;
    return RT_OK;
}

extern "C" int rt_render_async(rt_context* c, const rt_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                               uint32_t flags, const rt_tile_range* range, void* d_rgb8, void* d_linear, void* stream) {
    if (!c || !cam) return fail(RT_ERR_INVALID, "rt_render_async: NULL argument");
    if (spp == 0) return fail(RT_ERR_INVALID, "rt_render_async: spp == 0 (the reference panics: 0/0 in to_u8_array)");
    if (flags & ~RT_FLAG_ALL) return fail(RT_ERR_INVALID, "rt_render_async: unknown flag bits");
    {
        const uint32_t modes = flags & (RT_FLAG_MODE_VECTORIZED | RT_FLAG_MODE_SCALAR | RT_FLAG_MODE_VECTORIZED3);
        if (modes & (modes - 1u))
            return fail(RT_ERR_INVALID, "rt_render_async: the RT_FLAG_MODE_* flags are exclusive");
    }
    if (spp > (1u << 20)) return fail(RT_ERR_UNSUPPORTED, "rt_render_async: spp > 2^20");
    if ((flags & RT_FLAG_F32) && max_bounces > RT_MAX_BOUNCES_F32)   // rng<float>'s counter (rt_device.hpp)
        return fail(RT_ERR_UNSUPPORTED, "rt_render_async: fp32 with max_bounces > RT_MAX_BOUNCES_F32 (3839)");
    if (cam->image_width == 0 || cam->image_height == 0) return fail(RT_ERR_INVALID, "rt_render_async: empty image");
    if ((uint64_t)cam->image_width * cam->image_height > 0xFFFFFFFFull) return fail(RT_ERR_UNSUPPORTED, "image too large");
    rt_tile_range rg = range ? *range : rt_tile_range{0, 1, cam->image_height, 0, cam->image_width};
    if (!check_range(cam, &rg)) return fail(RT_ERR_INVALID, "rt_render_async: tile range outside the image");
    if ((uint64_t)rg.row_count * rg.col_count > 0x7FFFFFFFull) return fail(RT_ERR_UNSUPPORTED, "too many pixels in one call");
    const bool f32 = (flags & RT_FLAG_F32) != 0;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream
    // Renders on one context share its work counter, scratch and camera table: a render on a new
    // stream first waits for the previous stream, so cross-stream use serialises instead of racing.
    if (c->have_last && c->last_stream != st) HIPCHK(hipStreamSynchronize(c->last_stream));
    c->last_stream = st;
    c->have_last = true;
    if (!c->have_first) {
        HIPCHK(hipEventRecord(c->ev_first, st));
        c->have_first = true;
    }
    const int rc = f32 ? launch_t<float>(c, cam, max_bounces, spp, seed, flags, rg, d_rgb8, d_linear, st)
                       : launch_t<double>(c, cam, max_bounces, spp, seed, flags, rg, d_rgb8, d_linear, st);
    if (rc != RT_OK) return rc;
    HIPCHK(hipEventRecord(c->ev_last, st));
    c->pixels += (uint64_t)rg.row_count * rg.col_count;
    c->samples += (uint64_t)rg.row_count * rg.col_count * spp;
    return RT_OK;
}

extern "C" int rt_context_collect(rt_context* c, void* stream, rt_stats* out) {
    if (!c) return fail(RT_ERR_INVALID, "rt_context_collect: NULL context");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t st = (hipStream_t)stream;   // NULL = the HIP null stream
    HIPCHK(hipStreamSynchronize(st));
    std::vector<unsigned long long> segs(kSegShards * kSegStride);
    uint32_t err = 0;
    HIPCHK(hipMemcpy(segs.data(), c->segs, segs.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(&err, c->err, sizeof(uint32_t), hipMemcpyDeviceToHost));
    float ms = 0.f;
    if (c->have_first) HIPCHK(hipEventElapsedTime(&ms, c->ev_first, c->ev_last));
    HIPCHK(hipMemset(c->segs, 0, segs.size() * sizeof(unsigned long long)));
    HIPCHK(hipMemset(c->err, 0, 16));
    uint64_t total = 0, slots = 0, iters = 0, dsky = 0, kst[8] = {0, 0, 0, 0, 0, 0, 0, 0}, work[kNWork] = {};
    for (int i = 0; i < kSegShards; ++i)
        for (int j = 0; j < 8; ++j) kst[j] += segs[(size_t)i * kSegStride + 3 + j];
    if (kst[0] | kst[1] | kst[2] | kst[3])   // instrumented build (make kstats) only
        fprintf(stderr, "rt_kstats: general taken_groups %llu sweeps %llu clusters %llu top_groups %llu  camera "
                "candidates %llu sweeps %llu  finish_pixel %llu  filter_lanes_passing %llu\n",
                (unsigned long long)kst[0], (unsigned long long)kst[1], (unsigned long long)kst[4],
                (unsigned long long)kst[5], (unsigned long long)kst[2], (unsigned long long)kst[3],
                (unsigned long long)kst[6], (unsigned long long)kst[7]);
    for (int i = 0; i < kSegShards; ++i) {
        total += segs[(size_t)i * kSegStride];
        slots += segs[(size_t)i * kSegStride + 1];
        iters += segs[(size_t)i * kSegStride + 2];
        dsky += segs[(size_t)i * kSegStride + kDirectSkySlot];
        for (uint32_t j = 0; j < kNWork; ++j) work[j] += segs[(size_t)i * kSegStride + kWorkSlot + j];
    }
    if (out) {
        memset(out, 0, sizeof(*out));
        out->kernel_ms = ms;
        out->pixels = c->pixels;
        out->samples = c->samples;
        out->ray_segments = total;
        out->lane_slots = slots;
        out->bounce_iters = iters;
        out->pixels_per_second = ms > 0.f ? (double)c->pixels / ((double)ms * 1e-3) : 0.0;
        out->box_groups = work[kWBox];
        out->filter_groups = work[kWFilt];
        out->exact_tests = work[kWExact];
        out->cone_tests = work[kWCone];
        out->camera_exact_tests = work[kWCExact];
        out->direct_sky_samples = dsky;
        out->kernel_id = c->last_kernel_id;
        out->kernel_wg_per_cu = c->last_wg_per_cu;
    }
    c->have_first = false;
    c->pixels = c->samples = 0;
    c->last_kernel_id = c->last_wg_per_cu = 0;
    if (err) return fail(RT_ERR_RANGE, "a pixel channel exceeded 2.0 (Color::to_u8_array would panic, color.rs:55-57)");
    return RT_OK;
}

extern "C" int rt_device_alloc(rt_context* c, size_t bytes, void** out) {
    if (!c || !out) return fail(RT_ERR_INVALID, "rt_device_alloc: NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(out, bytes ? bytes : 1));
    return RT_OK;
}
extern "C" int rt_device_free(rt_context* c, void* ptr) {
    if (!c) return fail(RT_ERR_INVALID, "rt_device_free: NULL context");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipFree(ptr));
    return RT_OK;
}
extern "C" int rt_memcpy_d2h(rt_context* c, void* dst, const void* src, size_t bytes) {
    if (!c || !dst || !src) return fail(RT_ERR_INVALID, "rt_memcpy_d2h: NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

extern "C" int rt_render(const rt_scene* scene, const rt_camera* cam, uint32_t max_bounces, uint32_t spp, uint64_t seed,
                         uint32_t flags, const rt_tile_range* range, uint8_t* rgb8, double* linear, rt_stats* stats) {
    if (!scene || !cam) return fail(RT_ERR_INVALID, "rt_render: NULL argument");
    const auto t0 = std::chrono::steady_clock::now();
    rt_context* c = nullptr;
    int rc = rt_context_create(0, &c);
    if (rc != RT_OK) return rc;
    struct Guard { rt_context* c; void* a = nullptr; void* b = nullptr;
        ~Guard() { if (a) rt_device_free(c, a); if (b) rt_device_free(c, b); rt_context_destroy(c); } } g{c};
    rc = rt_context_set_scene(c, scene);
    if (rc != RT_OK) return rc;
    const rt_tile_range rg = range ? *range : rt_tile_range{0, 1, cam->image_height, 0, cam->image_width};
    const size_t npx = (size_t)rg.row_count * rg.col_count;
    if (rgb8 && (rc = rt_device_alloc(c, npx * 3, &g.a)) != RT_OK) return rc;
    if (linear && (rc = rt_device_alloc(c, npx * 3 * sizeof(double), &g.b)) != RT_OK) return rc;
    rc = rt_render_async(c, cam, max_bounces, spp, seed, flags, &rg, g.a, g.b, nullptr);
    if (rc != RT_OK) return rc;
    rt_stats st;
    const int crc = rt_context_collect(c, nullptr, &st);
    if (crc != RT_OK && crc != RT_ERR_RANGE) return crc;
    if (rgb8 && (rc = rt_memcpy_d2h(c, rgb8, g.a, npx * 3)) != RT_OK) return rc;
    if (linear && (rc = rt_memcpy_d2h(c, linear, g.b, npx * 3 * sizeof(double))) != RT_OK) return rc;
    st.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    st.pixels_per_second = st.seconds > 0 ? (double)st.pixels / st.seconds : 0.0;
    if (stats) *stats = st;
    if (crc == RT_ERR_RANGE) return fail(RT_ERR_RANGE, "a pixel channel exceeded 2.0 (Color::to_u8_array would panic, color.rs:55-57)");
    return RT_OK;
}
