// Fuzz of the general sweep's cluster boxes (rt_kernel.hip: pack_sweep's boxes, nearest_hit's
// per-lane slab constants, box_pair), test infrastructure for tests/test_filter_margin.py.
// Claim checked: whenever the reference's sphere test finds a valid root -- hit_packed under Q1
// (objects.rs:249-290), hit_packed with root2, or the scalar Sphere::hit (objects.rs:216-247), in
// fp32 or fp64 -- for a member of a cluster, the kernel's slab test of that ray against the
// cluster's box passes, and passes with the best-hit bound at that root too (box_pair's bt: the
// computed near time is <= the smallest root any of those tests reports, so a box entered only past
// the lane's best hit can be skipped).  The box and the lane's margin are computed exactly as the host and the
// kernel do (fp32 filter records, floored r2f, kappa from m = 48 u (pm^2 + r2max)).  A second
// evaluation with a quarter of the widening (kappa / 4) must pass too (>= 4x headroom).
// Cases: clusters of 1..16 spheres with radii spanning 4 decades, rays aimed near tangency to a
// member from outside, inside and behind the box, axis-parallel rays, scales 0.1..1000.
// LOCAL = 1: the MEGA kernels' local frames (pack_local): the case is moved up to 1000x its size from
// the origin, r2f is floored per cluster only (2^-10 of its largest), the box is re-centred on a group
// frame S (C' = RN_f(C - S), H widened by 2^-22 |C'|), the lane uses o' = o - S and the margin from
// pm = |o'|_1 + |C'|_1 + |H'|_1.
// Usage: box_cull_fuzz N F64(0|1) [SEED] [LOCAL]
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
static uint64_t s = 88172645463325252ull;
static double U() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1.0p-53; }
static double N() { double a = U(), b = U(); return sqrt(-2 * log(a + 1e-300)) * cos(6.283185307179586 * b); }
static float up32(double v) { float f = (float)v; if ((double)f < v) f = nextafterf(f, INFINITY); return f; }
// v_rcp_f32 (1 ulp): the correctly rounded value moved by -1, 0 or +1 ulp at random
static float rcp(float x) {
    float r = 1.0f / x;
    const double v = U();
    if (v < 1.0 / 3) r = nextafterf(r, 0.0f); else if (v < 2.0 / 3) r = nextafterf(r, copysignf(INFINITY, r));
    return r;
}

static double vmin(double t, double x, double lo) { return (x >= lo && x < INFINITY && x < t) ? x : t; }
static double hits_f(const float o[3], const float d[3], const float c[3], float r) {
    const float oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]}, r2 = r * r;
    const float a = fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0]));
    const float hb = fmaf(oc[2], d[2], fmaf(oc[1], d[1], oc[0] * d[0]));
    const float cc = fmaf(oc[2], oc[2], fmaf(oc[1], oc[1], oc[0] * oc[0])) - r2;
    const float disc = fmaf(hb, hb, (-a) * cc);
    const float sd = sqrtf(disc), ia = 1.0f / a;
    const float r1 = (-hb - sd) * ia, rr2 = (-hb + sd) * ia;
    double t = INFINITY;
    t = vmin(t, r1, 0.001f); t = vmin(t, rr2, 0.001f);
    const float as = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const float hs = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const float cs = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r2;
    const float ds = hs * hs - as * cs, sds = sqrtf(ds);
    const float q1 = (-hs - sds) / as, q2 = (-hs + sds) / as;
    t = vmin(t, q1, 0.001f); t = vmin(t, q2, 0.001f);
    return t;
}
static double hits_d(const double o[3], const double d[3], const double c[3], double r) {
    const double oc[3] = {o[0] - c[0], o[1] - c[1], o[2] - c[2]}, r2 = r * r;
    const double a = fma(d[2], d[2], fma(d[1], d[1], d[0] * d[0]));
    const double hb = fma(oc[2], d[2], fma(oc[1], d[1], oc[0] * d[0]));
    const double cc = fma(oc[2], oc[2], fma(oc[1], oc[1], oc[0] * oc[0])) - r2;
    const double disc = fma(hb, hb, (-a) * cc);
    const double sd = sqrt(disc), ia = 1.0 / a;
    const double r1 = (-hb - sd) * ia, rr2 = (-hb + sd) * ia;
    double t = INFINITY;
    t = vmin(t, r1, 0.001); t = vmin(t, rr2, 0.001);
    const double as = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double hs = oc[0] * d[0] + oc[1] * d[1] + oc[2] * d[2];
    const double cs = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r2;
    const double ds = hs * hs - as * cs, sds = sqrt(ds);
    const double q1 = (-hs - sds) / as, q2 = (-hs + sds) / as;
    t = vmin(t, q1, 0.001); t = vmin(t, q2, 0.001);
    return t;
}

// box_pair's test for one box (kernel arithmetic, fp32)
static int box_pass(const float C[3], const float h[3], const float i[3], const float A[3], const float J[3]) {
    float n[3], f[3];
    for (int a = 0; a < 3; ++a) {
        const float u = fmaf(C[a], i[a], A[a]);
        n[a] = fmaf(h[a], -J[a], u);
        f[a] = fmaf(h[a], J[a], u);
    }
    const float tn = fmaxf(fmaxf(n[0], n[1]), n[2]), tf = fminf(fminf(f[0], f[1]), f[2]);
    return !(tf - tn < 0.0f) && !(tf < 0.0f);
}
// the same with the best-hit bound bt (box_pair: max(tn, 0) <= min(tf, bt)), as the kernel orders it
static int box_pass_bt(const float C[3], const float h[3], const float i[3], const float A[3], const float J[3], float bt) {
    float n[3], f[3];
    for (int a = 0; a < 3; ++a) {
        const float u = fmaf(C[a], i[a], A[a]);
        n[a] = fmaf(h[a], -J[a], u);
        f[a] = fmaf(h[a], J[a], u);
    }
    const float tn = fmaxf(fmaxf(fmaxf(n[0], n[1]), n[2]), 0.0f), tf = fminf(fminf(fminf(f[0], f[1]), f[2]), bt);
    return !(tf < tn);
}

int main(int argc, char** argv) {
    const long n = atol(argv[1]);
    const int f64 = atoi(argv[2]);
    if (argc > 3) s = strtoull(argv[3], 0, 0) | 1;
    const int local = argc > 4 ? atoi(argv[4]) : 0;
    const float u = 0x1.0p-24f;
    long hits = 0, miss = 0, miss_q = 0, miss_0 = 0, culled = 0;
    for (long it = 0; it < n; ++it) {
        const double S = pow(10.0, -1 + 4 * U());
        double P[3] = {N() * S, N() * S, N() * S};   // cluster position
        if (local) { const double tm = S * pow(10.0, 3 * U()); for (int a = 0; a < 3; ++a) P[a] += N() * tm; }
        const int k = 1 + (int)(U() * 16);
        double cd[16][3], rd[16];
        float cf[16][3], r2f[16];
        const double rs = S * pow(10.0, -3 + 2.5 * U());
        double cm = 0.0, rm = 0.0;
        for (int j = 0; j < k; ++j) {
            for (int a = 0; a < 3; ++a) cd[j][a] = P[a] + N() * S * 0.05 * (a == 1 && U() < 0.5 ? 0.01 : 1.0);
            rd[j] = rs * pow(10.0, -1.5 * U());
            if (!f64) { for (int a = 0; a < 3; ++a) cd[j][a] = (float)cd[j][a]; rd[j] = (float)rd[j]; }
            for (int a = 0; a < 3; ++a) cf[j][a] = (float)cd[j][a];
            const double c1 = fabs((double)cf[j][0]) + fabs((double)cf[j][1]) + fabs((double)cf[j][2]);
            cm = fmax(cm, c1);
            rm = fmax(rm, f64 ? rd[j] * rd[j] : (double)((float)rd[j] * (float)rd[j]));
        }
        // pack_filter: floored r2f; pack_sweep: the box; margins (cmax includes |C|_1 + |h|_1)
        const double floor2 = local ? rm * 0x1.0p-10 : fmax(rm * 0x1.0p-10, cm * cm * 0x1.0p-16);
        double r2max = 0.0, r2min = INFINITY;
        for (int j = 0; j < k; ++j) {
            const double r2 = f64 ? rd[j] * rd[j] : (double)((float)rd[j] * (float)rd[j]);
            r2f[j] = up32(fmax(r2, floor2));
            r2max = fmax(r2max, r2f[j]);
            r2min = fmin(r2min, r2f[j]);
        }
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int j = 0; j < k; ++j)
            for (int a = 0; a < 3; ++a) {
                lo[a] = fmin(lo[a], (double)cf[j][a] - sqrt((double)r2f[j]));
                hi[a] = fmax(hi[a], (double)cf[j][a] + sqrt((double)r2f[j]));
            }
        float C[3], H[3];
        double cb = 0.0;
        for (int a = 0; a < 3; ++a) {
            C[a] = (float)(0.5 * (lo[a] + hi[a]));
            const double hh = fmax(hi[a] - (double)C[a], (double)C[a] - lo[a]);
            H[a] = up32(hh * (1.0 + 0x1.0p-20) + 0x1.0p-22 * fabs((double)C[a]));
            cb += fabs((double)C[a]) + (double)H[a];
        }
        float cmax = up32(fmax(cm, cb));
        const float fr2max = up32(r2max), fr2min = (float)r2min;
        float Sg[3] = {0, 0, 0};
        if (local) {   // a group frame near the box; the box in it
            double hs = 0.0;
            for (int a = 0; a < 3; ++a) hs = fmax(hs, (double)H[a]);
            double cl = 0.0;
            for (int a = 0; a < 3; ++a) {
                Sg[a] = (float)((double)C[a] + N() * hs * 2.0 * U());
                const float Cl = (float)((double)C[a] - (double)Sg[a]);
                H[a] = up32((double)H[a] + 0x1.0p-22 * fabs((double)Cl));
                C[a] = Cl;
                cl += fabs((double)C[a]) + (double)H[a];
            }
            cmax = up32(cl);
        }
        // a ray near tangency to member j (from outside, inside or behind)
        const int j = (int)(U() * k);
        double D[3] = {N(), N(), N()};
        if (U() < 0.1) { const int ax = (int)(U() * 3); D[0] = D[1] = D[2] = 0.0; D[ax] = U() < 0.5 ? 1.0 : -1.0;
                         D[(ax + 1) % 3] = U() < 0.5 ? 0.0 : 1e-9 * N(); }
        const double dl = sqrt(D[0] * D[0] + D[1] * D[1] + D[2] * D[2]);
        for (int a = 0; a < 3; ++a) D[a] /= dl;
        double px[3] = {N(), N(), N()};
        const double pd = px[0] * D[0] + px[1] * D[1] + px[2] * D[2];
        for (int a = 0; a < 3; ++a) px[a] -= pd * D[a];
        const double pl = sqrt(px[0] * px[0] + px[1] * px[1] + px[2] * px[2]);
        double rho = rd[j] * (1 + (U() - 0.5) * 1e-3 * pow(10.0, -6 * U()));
        if (U() < 0.2) rho = rd[j] * U();
        double tpar = -(pow(10.0, -3 + 4 * U()) * S);   // origin before the sphere ...
        if (U() < 0.15) tpar = -tpar;                   // ... or past it (hits only with root2 / inside)
        if (U() < 0.15) tpar = rd[j] * (U() - 0.5);     // or inside / at it
        double O[3];
        for (int a = 0; a < 3; ++a) O[a] = cd[j][a] + tpar * D[a] + px[a] / pl * rho;
        if (U() < 0.3) {   // graze the box face where the sphere touches it: tangent at an extreme point
            int ext = 0;
            const int ax = (int)(U() * 3), sg = U() < 0.5 ? 1 : -1;
            for (int m = 1; m < k; ++m) if (sg * (cd[m][ax] + sg * rd[m]) > sg * (cd[ext][ax] + sg * rd[ext])) ext = m;
            double T[3] = {N(), N(), N()};
            T[ax] = 0.0;
            const double tl = sqrt(T[0] * T[0] + T[1] * T[1] + T[2] * T[2]);
            const double e = rd[ext] * (1e-7 * N());
            for (int a = 0; a < 3; ++a) {
                D[a] = T[a] / tl;
                O[a] = cd[ext][a] + (a == ax ? sg * (rd[ext] + e) : 0.0) - D[a] * S * pow(10.0, -2 + 3 * U());
            }
            if (!f64) for (int a = 0; a < 3; ++a) { O[a] = (float)O[a]; D[a] = (float)D[a]; }
        }
        if (!f64) for (int a = 0; a < 3; ++a) { O[a] = (float)O[a]; D[a] = (float)D[a]; }
        double tmin = INFINITY;   // the smallest root any of the reference's tests reports for a member
        for (int m = 0; m < k; ++m) {
            if (f64) tmin = fmin(tmin, hits_d(O, D, cd[m], rd[m]));
            else {
                const float of[3] = {(float)O[0], (float)O[1], (float)O[2]}, df[3] = {(float)D[0], (float)D[1], (float)D[2]};
                const float cc[3] = {(float)cd[m][0], (float)cd[m][1], (float)cd[m][2]};
                tmin = fmin(tmin, hits_f(of, df, cc, (float)rd[m]));
            }
        }
        const int any = tmin < INFINITY;
        // the best-hit bound at that root: the kernel's bt for a best hit t* (fp64: rounded up)
        const float bt = f64 ? (float)tmin * (1.0f + 0x1.0p-22f) : (float)tmin;
        // nearest_hit's per-lane constants (fp32)
        const float fd[3] = {(float)D[0], (float)D[1], (float)D[2]};
        float fo[3] = {(float)O[0], (float)O[1], (float)O[2]};
        if (local) for (int a = 0; a < 3; ++a) fo[a] = f64 ? (float)(O[a] - (double)Sg[a]) : fo[a] - Sg[a];   // o' = o - S
        const float on = fabsf(fo[0]) + fabsf(fo[1]) + fabsf(fo[2]);
        const float pm = cmax + on;
        const float isr = up32(8.0 * 0x1.0p-24 / sqrt((double)fr2min));
        // the sweep's constant (nearest_hit) and the mega kernels' local form (lmask)
        const float kap = local ? fmaf(fmaf(pm, pm, fr2max), up32(48.0 * 0x1.0p-24 * 0.5 / fr2min), fmaf(pm, isr, 1.0f))
                                : 1.0f + fmaf(48.0f * 0x1.0p-24f * fmaf(pm, pm, fr2max), up32(0.5 / fr2min), pm * isr);
        const float kq = 1.0f + (kap - 1.0f) * 0.25f;
        float I[3], A[3], J[3], Jq[3], J0[3];
        for (int a = 0; a < 3; ++a) {
            I[a] = rcp(fabsf(fd[a]) >= 1e-20f ? fd[a] : copysignf(1e-20f, fd[a]));
            A[a] = -(fo[a] * I[a]);
            J[a] = fabsf(I[a]) * kap;
            Jq[a] = fabsf(I[a]) * kq;
            J0[a] = fabsf(I[a]);
        }
        const int pass = box_pass(C, H, I, A, J), pass_q = box_pass(C, H, I, A, Jq), pass_0 = box_pass(C, H, I, A, J0);
        const int pass_b = box_pass_bt(C, H, I, A, J, bt), pass_bq = box_pass_bt(C, H, I, A, Jq, bt);
        if (!pass) ++culled;
        if (any) {
            ++hits;
            if (!pass || !pass_b) ++miss;
            if (!pass_q || !pass_bq) ++miss_q;
            if (!pass_0) ++miss_0;
        }
    }
    printf("f64=%d cases %ld hits %ld culled %ld misses %ld quarter-margin-misses %ld (no-margin misses %ld)\n", f64, n,
           hits, culled, miss, miss_q, miss_0);
    return miss != 0;
}
