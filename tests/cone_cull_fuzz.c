// Fuzz of the camera-batch cone cull (rt_kernel.hip: camera_sweep, build_cam_table's rp), test
// infrastructure for tests/test_filter_margin.py.  Claim checked: whenever the reference's sphere
// test finds a valid root for ANY ray of a camera batch -- hit_packed under Q1 (objects.rs:249-290,
// root1 only), hit_packed with root2 (Q1 off) or the scalar Sphere::hit (objects.rs:216-247) --
// the cull, computed as the kernel does in fp32 (axis = the first ray's direction, sin(theta) =
// max |d^ x a| inflated, w = c - O, f = |w x a| cos(theta) - (w.a) sin(theta)), passes the sphere:
// !(f > rp) with rp = sqrt(r^2 (1 + 2^-20) + 64 u |w|^2) + 32 u |w| rounded up.
// Cases: batches of 1..64 rays with angular spreads 1e-7..0.3 rad, spheres placed near tangency to
// one ray of the batch, cameras near and inside spheres, scales 0.1..1000, fp32 and fp64 rays.
// Prints the worst fraction of the margin used over all hits: (f - r) / (rp - r).
// Usage: cone_cull_fuzz N F64(0|1) [SEED]
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
// v_rsq_f32 / v_rcp_f32 (1 ulp): the correctly rounded value moved by -1, 0 or +1 ulp at random
static float jitter(float r) {
    const double v = U();
    return v < 1.0 / 3 ? nextafterf(r, 0.0f) : v < 2.0 / 3 ? nextafterf(r, INFINITY) : r;
}
static float rsq(float x) { return jitter(1.0f / sqrtf(x)); }
static float rcp(float x) { return jitter(1.0f / x); }
static float vsqrt(float x) { return jitter(sqrtf(x)); }   // v_sqrt_f32 (1 ulp)
static float fbits(uint32_t b) { float x; memcpy(&x, &b, 4); return x; }

// Does any of the three reference tests find a valid root?  (T = float)
static int hits_f(const float oc[3], float r, const float d[3]) {
    const float r2 = r * r;
    // hit_packed (objects.rs:252-273), fma where the reference writes mul_add
    const float a = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
    const float hb = fmaf(oc[2], d[2], fmaf(oc[1], d[1], oc[0] * d[0]));
    const float c = fmaf(oc[2], oc[2], fmaf(oc[1], oc[1], oc[0] * oc[0])) - r2;
    const float disc = fmaf(hb, hb, (-a) * c);
    const float sd = sqrtf(disc), ia = 1.0f / a;
    const float r1 = (-hb - sd) * ia, rr2 = (-hb + sd) * ia;
    if ((r1 >= 0.001f && r1 < INFINITY) || (rr2 >= 0.001f && rr2 < INFINITY)) return 1;
    // Sphere::hit (objects.rs:217-234): no fma, both roots, / a
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

int main(int argc, char** argv) {
    long n = atol(argv[1]);
    int f64 = atoi(argv[2]);
    if (argc > 3) s = strtoull(argv[3], 0, 0) | 1;
    long hits = 0, miss = 0, culled = 0, batches_all = 0, cmiss = 0;
    double worst = -1e300;
    for (long it = 0; it < n; ++it) {
        const double S = pow(10.0, -1 + 4 * U());
        const double O[3] = {N() * S, N() * S, N() * S};
        // batch: nr rays around a random axis, spread up to `spread` rad, each unit() in T
        const int nr = 1 + (int)(U() * 64);
        const double spread = pow(10.0, -7 + 6.5 * U());
        double ax0[3] = {N(), N(), N()};
        const double al = sqrt(ax0[0] * ax0[0] + ax0[1] * ax0[1] + ax0[2] * ax0[2]);
        for (int k = 0; k < 3; ++k) ax0[k] /= al;
        double D[64][3];
        float Df[64][3];
        for (int i = 0; i < nr; ++i) {
            double v[3];
            for (int k = 0; k < 3; ++k) v[k] = ax0[k] + spread * (2 * U() - 1);
            if (f64) {
                const double l = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);   // unit(): v / sqrt(len2)
                for (int k = 0; k < 3; ++k) D[i][k] = v[k] / l;
            } else {
                float w[3] = {(float)v[0], (float)v[1], (float)v[2]};
                const float l = sqrtf(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
                for (int k = 0; k < 3; ++k) D[i][k] = w[k] / l;
            }
            for (int k = 0; k < 3; ++k) Df[i][k] = (float)D[i][k];
        }
        // sphere near tangency to ray j of the batch
        const int j = (int)(U() * nr);
        const double r = S * pow(10.0, -4 + 4 * U());
        double tpar = pow(10.0, -3 + 4 * U()) * S * (U() < 0.9 ? 1 : -1);
        if (U() < 0.2) tpar = r * (0.5 + U());   // camera near (or inside) the sphere
        double px[3] = {N(), N(), N()};
        const double pd = px[0] * D[j][0] + px[1] * D[j][1] + px[2] * D[j][2];
        for (int k = 0; k < 3; ++k) px[k] -= pd * D[j][k];
        const double pl = sqrt(px[0] * px[0] + px[1] * px[1] + px[2] * px[2]);
        double rho = r * (1 + (U() - 0.5) * 1e-3 * pow(10.0, -6 * U()));
        if (U() < 0.1) rho = r * U();
        double C[3];
        for (int k = 0; k < 3; ++k) C[k] = O[k] + tpar * D[j][k] + px[k] / pl * rho;
        // the reference's oc (and the camera-origin table's) in T, r^2 in T
        double oc64[3], r2t;
        float ocf[3];
        int any = 0;
        if (f64) {
            for (int k = 0; k < 3; ++k) oc64[k] = O[k] - C[k];
            r2t = r * r;
            for (int i = 0; i < nr; ++i) any |= hits_d(oc64, r, D[i]);
        } else {
            const float rf = (float)r;
            for (int k = 0; k < 3; ++k) { ocf[k] = (float)O[k] - (float)C[k]; oc64[k] = ocf[k]; }
            r2t = (double)(rf * rf);
            for (int i = 0; i < nr; ++i) { float d[3] = {Df[i][0], Df[i][1], Df[i][2]}; any |= hits_f(ocf, rf, d); }
        }
        // build_cam_table: w = -(float)oc, rp
        const float wx = -(float)oc64[0], wy = -(float)oc64[1], wz = -(float)oc64[2];
        const double wn2 = oc64[0] * oc64[0] + oc64[1] * oc64[1] + oc64[2] * oc64[2];
        const double v = sqrt(r2t * (1.0 + 0x1.0p-20) + 0x1.0p-18 * wn2) + 0x1.0p-19 * sqrt(wn2) + 1e-30;
        const float rp = v < 1e30 ? up32(v) : INFINITY;
        // camera_sweep: the cone, as the kernel computes it
        float ax = Df[0][0], ay = Df[0][1], az = Df[0][2];
        const float ia = rsq(fmaf(az, az, fmaf(ay, ay, ax * ax)));
        ax = ax * ia; ay = ay * ia; az = az * ia;
        uint32_t sm = 0;
        int all = 0;
        for (int i = 0; i < nr; ++i) {
            const float fdx = Df[i][0], fdy = Df[i][1], fdz = Df[i][2];
            const float cx = fmaf(fdy, az, -(fdz * ay)), cy = fmaf(fdz, ax, -(fdx * az)), cz = fmaf(fdx, ay, -(fdy * ax));
            const float dn2 = fmaf(fdz, fdz, fmaf(fdy, fdy, fdx * fdx));
            const float s2 = fmaf(cz, cz, fmaf(cy, cy, cx * cx)) * rcp(dn2) * (1.0f + 0x1.0p-22f);
            const float dt = fmaf(fdz, az, fmaf(fdy, ay, fdx * ax));
            if (!(dt > 0.5f)) all = 1;
            if (bits(s2) > sm) sm = bits(s2);
        }
        const float Sn = fmaf(vsqrt(fbits(sm)), 1.0f + 0x1.0p-22f, 0x1.0p-21f);
        if (!(Sn < 0.5f)) all = 1;
        const float Cc = vsqrt(fmaf(-Sn, Sn, 1.0f));
        const float t = fmaf(wz, az, fmaf(wy, ay, wx * ax));
        const float qx = fmaf(wy, az, -(wz * ay)), qy = fmaf(wz, ax, -(wx * az)), qz = fmaf(wx, ay, -(wy * ax));
        const float pp = vsqrt(fmaf(qz, qz, fmaf(qy, qy, qx * qx)));
        const float f = fmaf(pp, Cc, -(t * Sn));
        const int pass = all || !(f > rp);
        // the sphere's cluster (set_scene's bounds + build_cam_table's record): the target plus up to
        // 15 neighbours; AABB centre C, R >= max |c_i - C| + r_i, rp_k as the kernel computes it
        double cl[16][4];
        const int nk = 1 + (int)(U() * 16);
        for (int k = 0; k < 3; ++k) cl[0][k] = f64 ? C[k] : (double)(float)C[k];
        cl[0][3] = f64 ? r : (double)(float)r;
        for (int m = 1; m < nk; ++m) {
            for (int k = 0; k < 3; ++k) cl[m][k] = C[k] + N() * S * 0.05;
            cl[m][3] = r * pow(10.0, 2 * U() - 1);
            if (!f64) for (int k = 0; k < 4; ++k) cl[m][k] = (float)cl[m][k];
        }
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, CC[3], RR = 0.0;
        for (int m = 0; m < nk; ++m)
            for (int k = 0; k < 3; ++k) { lo[k] = fmin(lo[k], cl[m][k] - cl[m][3]); hi[k] = fmax(hi[k], cl[m][k] + cl[m][3]); }
        for (int k = 0; k < 3; ++k) CC[k] = 0.5 * (lo[k] + hi[k]);
        for (int m = 0; m < nk; ++m) {
            const double dx = cl[m][0] - CC[0], dy = cl[m][1] - CC[1], dz = cl[m][2] - CC[2];
            RR = fmax(RR, sqrt(dx * dx + dy * dy + dz * dz) + cl[m][3]);
        }
        RR *= 1.0 + 0x1.0p-40;
        const double Ox = f64 ? O[0] : (double)(float)O[0], Oy = f64 ? O[1] : (double)(float)O[1],
                     Oz = f64 ? O[2] : (double)(float)O[2];
        const double Wx = CC[0] - Ox, Wy = CC[1] - Oy, Wz = CC[2] - Oz, Wn = sqrt(Wx * Wx + Wy * Wy + Wz * Wz);
        const double vk = RR * (1.0 + 0x1.0p-20) + (0x1.0p-9 + 0x1.0p-16) * (Wn + RR) + 1e-30;
        const float rpk = vk < 1e30 ? up32(vk) : INFINITY;
        const float Wf[3] = {(float)Wx, (float)Wy, (float)Wz};
        const float tk = fmaf(Wf[2], az, fmaf(Wf[1], ay, Wf[0] * ax));
        const float kx = fmaf(Wf[1], az, -(Wf[2] * ay)), ky = fmaf(Wf[2], ax, -(Wf[0] * az)), kz = fmaf(Wf[0], ay, -(Wf[1] * ax));
        const float pk = vsqrt(fmaf(kz, kz, fmaf(ky, ky, kx * kx)));
        const int pass_k = all || !(fmaf(pk, Cc, -(tk * Sn)) > rpk);
        if (pass && !pass_k) ++cmiss;
        batches_all += all;
        if (!pass) ++culled;
        if (any) {
            ++hits;
            if (!pass || !pass_k) ++miss;
            if (!all) {
                const double fd = f;
                const double need = fd > sqrt(r2t) ? (fd - sqrt(r2t)) / ((double)rp - sqrt(r2t)) : 0.0;
                if (need > worst) worst = need;
            }
        }
    }
    printf("f64=%d cases %ld hits %ld misses %ld culled %ld all %ld worst margin fraction %.4f\n", f64, n, hits, miss, culled,
           batches_all, worst);
    printf("cluster records stricter than a passing member: %ld\n", cmiss);
    return miss != 0 || cmiss != 0;
}
