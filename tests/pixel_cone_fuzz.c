// Fuzz of the per-pixel camera cone (rt_camera.hpp: pixel_list), test infrastructure for
// tests/test_filter_margin.py.  Claims checked, for random cameras (Camera::new, ray_tracing.rs:27-62),
// image sizes and pixels:
//  (1) containment: every primary ray of the pixel as the kernel computes it in T (Camera::get_ray,
//      ray_tracing.rs:77-89, jitter in [0, 1) including its extremes; fp32 or fp64) lies inside the
//      pixel cone: sin(angle(d, a)) <= S, where the axis a and S are computed as pixel_list does
//      (fp32 footprint corners, v_rsq/v_rcp/v_sqrt modelled as +-1 ulp).  Reported: the worst
//      (sin - S0) / margin, S0 = the cone's S without the pixel margin 2^-20 M / |Dc| (M = |ulc|_1 +
//      |vu|_1 + |vv|_1 + |centre|_1, Dc the footprint centre's direction: the rounding of the corners
//      and of the rays scales with the coordinates' magnitudes over the focal distance); must stay < 1,
//      the test asks for 4x headroom;
//  (2) end to end: a sphere placed near tangency to one of those rays, that the reference's sphere
//      test (hit_packed under Q1, with root2, or the scalar Sphere::hit) finds a root for, passes the
//      pixel cone's cull with the same rp record as camera_sweep (build_cam_table).
// Usage: pixel_cone_fuzz N F64(0|1) [SEED]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static double U() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1.0p-53; }
static double N() { double a = U(), b = U(); return sqrt(-2 * log(a + 1e-300)) * cos(6.283185307179586 * b); }
static float up32(double v) { float f = (float)v; if ((double)f < v) f = nextafterf(f, INFINITY); return f; }
static uint32_t bits(float x) { uint32_t b; memcpy(&b, &x, 4); return b; }
static float fbits(uint32_t b) { float x; memcpy(&x, &b, 4); return x; }
static float jitter(float r) {
    const double v = U();
    return v < 1.0 / 3 ? nextafterf(r, 0.0f) : v < 2.0 / 3 ? nextafterf(r, INFINITY) : r;
}
static float rsq(float x) { return jitter(1.0f / sqrtf(x)); }
static float rcp(float x) { return jitter(1.0f / x); }
static float vsqrt(float x) { return jitter(sqrtf(x)); }

static int hits_f(const float oc[3], float r, const float d[3]) {
    const float r2 = r * r;
    const float a = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
    const float hb = fmaf(oc[2], d[2], fmaf(oc[1], d[1], oc[0] * d[0]));
    const float c = fmaf(oc[2], oc[2], fmaf(oc[1], oc[1], oc[0] * oc[0])) - r2;
    const float disc = fmaf(hb, hb, (-a) * c);
    const float sd = sqrtf(disc), ia = 1.0f / a;
    const float r1 = (-hb - sd) * ia, rr2 = (-hb + sd) * ia;
    if ((r1 >= 0.001f && r1 < INFINITY) || (rr2 >= 0.001f && rr2 < INFINITY)) return 1;
    const float as = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const float hs = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const float cs = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r2;
    const float ds = hs * hs - as * cs;
    const float sds = sqrtf(ds);
    const float q1 = (-hs - sds) / as, q2 = (-hs + sds) / as;
    return (q1 >= 0.001f && q1 < INFINITY) || (q2 >= 0.001f && q2 < INFINITY);
}
static int hits_d(const double oc[3], double r, const double d[3]) {
    const double r2 = r * r;
    const double a = fma(d[2], d[2], fma(d[1], d[1], d[0] * d[0]));
    const double hb = fma(oc[2], d[2], fma(oc[1], d[1], oc[0] * d[0]));
    const double c = fma(oc[2], oc[2], fma(oc[1], oc[1], oc[0] * oc[0])) - r2;
    const double disc = fma(hb, hb, (-a) * c);
    const double sd = sqrt(disc), ia = 1.0 / a;
    const double r1 = (-hb - sd) * ia, rr2 = (-hb + sd) * ia;
    if ((r1 >= 0.001 && r1 < INFINITY) || (rr2 >= 0.001 && rr2 < INFINITY)) return 1;
    const double as = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double hs = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const double cs = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r2;
    const double ds = hs * hs - as * cs;
    const double sds = sqrt(ds);
    const double q1 = (-hs - sds) / as, q2 = (-hs + sds) / as;
    return (q1 >= 0.001 && q1 < INFINITY) || (q2 >= 0.001 && q2 < INFINITY);
}

static void unit3(const double a[3], double o[3]) {
    const double l = sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    for (int k = 0; k < 3; ++k) o[k] = a[k] / l;
}

int main(int argc, char** argv) {
    const long n = atol(argv[1]);
    const int f64 = atoi(argv[2]);
    if (argc > 3) s = strtoull(argv[3], 0, 0) | 1;
    long rays = 0, outside = 0, hits = 0, miss = 0, culled = 0, over = 0;
    double worst = -1e300;
    for (long it = 0; it < n; ++it) {
        // Camera::new (ray_tracing.rs:27-62), f64, no FMA
        const uint32_t W = 1 + (uint32_t)(pow(2.0, 12 * U())), H = 1 + (uint32_t)(pow(2.0, 12 * U()));
        const double sc = pow(10.0, -1 + 4 * U());
        const double ctr[3] = {N() * sc, N() * sc, N() * sc};
        const double la[3] = {ctr[0] + N(), ctr[1] + N(), ctr[2] + N()};
        const double up[3] = {N(), N(), N()};
        const double vfov = 1.0 + 119.0 * U(), fl = pow(10.0, -1 + 3 * U());
        const double deg = 3.141592653589793 / 180.0;
        const double vh = tan((vfov * deg) / 2.0) * fl * 2.0, vw = vh * ((double)W / (double)H);
        double dv_[3] = {la[0] - ctr[0], la[1] - ctr[1], la[2] - ctr[2]}, dir[3], u[3];
        unit3(dv_, dir);
        const double w[3] = {-dir[0], -dir[1], -dir[2]};
        const double cr[3] = {up[1] * w[2] - up[2] * w[1], up[2] * w[0] - up[0] * w[2], up[0] * w[1] - up[1] * w[0]};
        unit3(cr, u);
        const double v[3] = {w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2], w[0] * u[1] - w[1] * u[0]};
        double vu[3], vv[3], ulc[3];
        for (int k = 0; k < 3; ++k) {
            vu[k] = u[k] * vw;
            vv[k] = (-v[k]) * vh;
            ulc[k] = ((ctr[k] - w[k] * fl) - vu[k] / 2.0) - vv[k] / 2.0;
        }
        const uint32_t col = (uint32_t)(U() * W), row = (uint32_t)(U() * H);
        // pixel_list: the cone in fp32 from the camera constants (T -> float)
        float cf[4][3], df[4][3] = {{0}};
        float tc[3], tu[3], tv[3], tl[3];
        for (int k = 0; k < 3; ++k) {
            tc[k] = f64 ? (float)ctr[k] : (float)(float)ctr[k];
            tu[k] = (float)vu[k]; tv[k] = (float)vv[k]; tl[k] = (float)ulc[k];
        }
        float Dc[5][3];
        for (int l = 0; l < 5; ++l) {
            const float fx = l < 4 ? (float)(l & 1) : 0.5f, fy = l < 4 ? (float)(l >> 1) : 0.5f;
            const float s1 = ((float)col + fx) / (float)W, s2 = ((float)row + fy) / (float)H;
            for (int k = 0; k < 3; ++k) Dc[l][k] = (tl[k] + (tu[k] * s1 + tv[k] * s2)) - tc[k];
        }
        (void)cf; (void)df;
        float ax = Dc[4][0], ay = Dc[4][1], az = Dc[4][2];
        const float ia = rsq(fmaf(az, az, fmaf(ay, ay, ax * ax)));
        ax *= ia; ay *= ia; az *= ia;
        uint32_t sm = 0;
        int all = 0;
        for (int l = 0; l < 4; ++l) {
            const float Dx = Dc[l][0], Dy = Dc[l][1], Dz = Dc[l][2];
            const float cx = fmaf(Dy, az, -(Dz * ay)), cy = fmaf(Dz, ax, -(Dx * az)), cz = fmaf(Dx, ay, -(Dy * ax));
            const float dn2 = fmaf(Dz, Dz, fmaf(Dy, Dy, Dx * Dx));
            const float s2 = fmaf(cz, cz, fmaf(cy, cy, cx * cx)) * rcp(dn2) * (1.0f + 0x1.0p-22f);
            const float dt = fmaf(Dz, az, fmaf(Dy, ay, Dx * ax)) * rsq(dn2);
            if (!(dt > 0.5f)) all = 1;
            if (bits(s2) > sm) sm = bits(s2);
        }
        const float root = vsqrt(fbits(sm));
        float M = 0.0f;
        for (int k = 0; k < 3; ++k) M += ((fabsf(tl[k]) + fabsf(tu[k])) + fabsf(tv[k])) + fabsf(tc[k]);
        const float dnc = fmaf(Dc[4][2], Dc[4][2], fmaf(Dc[4][1], Dc[4][1], Dc[4][0] * Dc[4][0]));
        const float margin = (M * 0x1.0p-20f) * rsq(dnc);
        const float S0 = fmaf(root, 1.0f + 0x1.0p-22f, 0x1.0p-21f);
        const float Sn = fmaf(root, 1.0f + 0x1.0p-22f, 0x1.0p-21f + margin);
        const double kPixelMargin = margin;
        if (!(Sn < 0.5f)) all = 1;
        if (all) { ++over; continue; }   // pixel_list gives up: the batches sweep per batch
        const float Cc = vsqrt(fmaf(-Sn, Sn, 1.0f));
        const double A[3] = {ax, ay, az};
        const double An = sqrt(A[0] * A[0] + A[1] * A[1] + A[2] * A[2]);
        // rays of the pixel, as the kernel computes them in T (pinhole: origin = centre)
        double D[16][3];
        const int nr = 16;
        for (int i = 0; i < nr; ++i) {
            double jx = U(), jy = U();
            if (i == 0) { jx = 0.0; jy = 0.0; }
            if (i == 1) { jx = 1.0 - 0x1.0p-53; jy = 1.0 - 0x1.0p-53; }
            if (i == 2) { jx = 0.0; jy = 1.0 - 0x1.0p-53; }
            if (i == 3) { jx = 1.0 - 0x1.0p-53; jy = 0.0; }
            if (f64) {
                const double s1 = ((double)col + jx) / (double)W, s2 = ((double)row + jy) / (double)H;
                double pc[3];
                for (int k = 0; k < 3; ++k) pc[k] = ulc[k] + (vu[k] * s1 + vv[k] * s2);
                double vv3[3] = {pc[0] - ctr[0], pc[1] - ctr[1], pc[2] - ctr[2]};
                unit3(vv3, D[i]);
            } else {
                const float fjx = i == 1 || i == 3 ? 1.0f - 0x1.0p-24f : (float)jx;
                const float fjy = i == 1 || i == 2 ? 1.0f - 0x1.0p-24f : (float)jy;
                // the kernel's div_dim (rt_common.hpp): RN_f(RN_d(x * RN_d(1/W))) for W < 2^20 (equal to
                // RN_f(x / W), tests/test_div_dim.py; modelled literally here)
                const float s1 = (float)((double)((float)col + fjx) * (1.0 / (double)W));
                const float s2 = (float)((double)((float)row + fjy) * (1.0 / (double)H));
                float pc[3], vf[3];
                for (int k = 0; k < 3; ++k) pc[k] = tl[k] + (tu[k] * s1 + tv[k] * s2);
                for (int k = 0; k < 3; ++k) vf[k] = pc[k] - (float)ctr[k];
                // unit() (rt_device.hpp, Vec3::length + division, geometry.rs:106-112): no FMA
                const float l = sqrtf((vf[0] * vf[0] + vf[1] * vf[1]) + vf[2] * vf[2]);
                for (int k = 0; k < 3; ++k) D[i][k] = vf[k] / l;
            }
            // (1) containment, in double: sin of the angle between the ray and the fp32 axis
            const double c0 = D[i][1] * A[2] - D[i][2] * A[1], c1 = D[i][2] * A[0] - D[i][0] * A[2],
                         c2 = D[i][0] * A[1] - D[i][1] * A[0];
            const double dl = sqrt(D[i][0] * D[i][0] + D[i][1] * D[i][1] + D[i][2] * D[i][2]);
            const double sn = sqrt(c0 * c0 + c1 * c1 + c2 * c2) / (dl * An);
            ++rays;
            if (sn > (double)Sn) ++outside;
            const double need = (sn - (double)S0) / (double)kPixelMargin;
            if (need > worst) worst = need;
        }
        // (2) end to end: a sphere near tangency to ray j, the record and cull of camera_sweep
        const int j = (int)(U() * nr);
        const double r = sc * pow(10.0, -4 + 4 * U());
        const double tpar = pow(10.0, -3 + 4 * U()) * sc;
        double px[3] = {N(), N(), N()};
        const double pd = px[0] * D[j][0] + px[1] * D[j][1] + px[2] * D[j][2];
        for (int k = 0; k < 3; ++k) px[k] -= pd * D[j][k];
        const double pl = sqrt(px[0] * px[0] + px[1] * px[1] + px[2] * px[2]);
        double rho = r * (1 + (U() - 0.5) * 1e-3 * pow(10.0, -6 * U()));
        const double O[3] = {f64 ? ctr[0] : (double)(float)ctr[0], f64 ? ctr[1] : (double)(float)ctr[1],
                             f64 ? ctr[2] : (double)(float)ctr[2]};
        double C[3];
        for (int k = 0; k < 3; ++k) C[k] = O[k] + tpar * D[j][k] + px[k] / pl * rho;
        double oc64[3], r2t;
        int any = 0;
        if (f64) {
            for (int k = 0; k < 3; ++k) oc64[k] = O[k] - C[k];
            r2t = r * r;
            for (int i = 0; i < nr; ++i) any |= hits_d(oc64, r, D[i]);
        } else {
            const float rf = (float)r;
            float ocf[3];
            for (int k = 0; k < 3; ++k) { ocf[k] = (float)O[k] - (float)C[k]; oc64[k] = ocf[k]; }
            r2t = (double)(rf * rf);
            for (int i = 0; i < nr; ++i) { float d[3] = {(float)D[i][0], (float)D[i][1], (float)D[i][2]}; any |= hits_f(ocf, rf, d); }
        }
        const float wx = -(float)oc64[0], wy = -(float)oc64[1], wz = -(float)oc64[2];
        const double wn2 = oc64[0] * oc64[0] + oc64[1] * oc64[1] + oc64[2] * oc64[2];
        const double vr = sqrt(r2t * (1.0 + 0x1.0p-20) + 0x1.0p-18 * wn2) + 0x1.0p-19 * sqrt(wn2) + 1e-30;
        const float rp = vr < 1e30 ? up32(vr) : INFINITY;
        const float t = fmaf(wz, az, fmaf(wy, ay, wx * ax));
        const float qx = fmaf(wy, az, -(wz * ay)), qy = fmaf(wz, ax, -(wx * az)), qz = fmaf(wx, ay, -(wy * ax));
        const float pp = vsqrt(fmaf(qz, qz, fmaf(qy, qy, qx * qx)));
        const float f = fmaf(pp, Cc, -(t * Sn));
        const int pass = !(f > rp);
        if (!pass) ++culled;
        if (any) { ++hits; if (!pass) ++miss; }
    }
    printf("f64=%d cases %ld rays %ld outside %ld over %ld hits %ld misses %ld culled %ld worst margin fraction %.4f\n",
           f64, n, rays, outside, over, hits, miss, culled, worst);
    return outside != 0 || miss != 0;
}
