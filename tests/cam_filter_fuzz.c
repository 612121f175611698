// Fuzz of the camera-batch filter (rt_kernel.hip: build_cam_table's sc, nearest_hit CAMT under
// Q1, cam_filter_group), test infrastructure for tests/test_filter_margin.py.  Claim checked:
// whenever hit_packed (objects.rs:249-290, Q1: root1 only) finds a VALID root1 for a ray from the
// camera, the filter's t = hb' + sc, computed as the kernel does (hb' = oc.d^ in fp32 with
// d^ = d / sqrt(|d|^2), sc = sqrt(c) - 24 u |oc| - 1e-20 rounded down, +inf for c <= 0), has its
// sign bit set.  Cases: spheres near tangency, cameras near and inside spheres, scales 0.1..1000.
// Usage: cam_filter_fuzz N F64(0|1) [SEED]
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static double U() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1.0p-53; }
static double N() { double a = U(), b = U(); return sqrt(-2 * log(a + 1e-300)) * cos(6.283185307179586 * b); }
static float down32(double v) { float f = (float)v; if ((double)f > v) f = nextafterf(f, -INFINITY); return f; }
int main(int argc, char** argv) {
    long n = atol(argv[1]); int f64 = atoi(argv[2]);
    if (argc > 3) s = strtoull(argv[3], 0, 0) | 1;
    long valid = 0, miss = 0; double worst = -1e300;
    const double u = 0x1.0p-24;
    for (long it = 0; it < n; ++it) {
        double S = pow(10.0, -1 + 4 * U());
        double O[3] = {N() * S, N() * S, N() * S};
        double dd[3] = {N(), N(), N()}; double dl = sqrt(dd[0]*dd[0]+dd[1]*dd[1]+dd[2]*dd[2]);
        double D[3] = {dd[0]/dl, dd[1]/dl, dd[2]/dl};
        if (!f64) for (int k = 0; k < 3; ++k) { O[k] = (float)O[k]; D[k] = (float)D[k]; }
        double r = S * pow(10.0, -4 + 4 * U());
        double tpar = pow(10.0, -3 + 4 * U()) * S * (U() < 0.9 ? 1 : -1);
        if (U() < 0.2) tpar = r * (0.5 + U());   // camera near the sphere
        double px[3] = {N(), N(), N()};
        double pd = px[0]*D[0]+px[1]*D[1]+px[2]*D[2];
        for (int k = 0; k < 3; ++k) px[k] -= pd * D[k];
        double pl = sqrt(px[0]*px[0]+px[1]*px[1]+px[2]*px[2]);
        double rho = r * (1 + (U() - 0.5) * 1e-3 * pow(10.0, -6 * U()));
        if (U() < 0.1) rho = r * U();
        double C[3];
        for (int k = 0; k < 3; ++k) C[k] = O[k] + tpar * D[k] + px[k] / pl * rho;
        int ok; double oc64[3], c64;
        float ocf[3];
        if (!f64) {
            float cx = C[0], cy = C[1], cz = C[2], rr = r, r2 = rr * rr;
            float ox = O[0], oy = O[1], oz = O[2], dx = D[0], dy = D[1], dz = D[2];
            float ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;
            float c = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx)) - r2;
            float a = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
            float hb = fmaf(ocz, dz, fmaf(ocy, dy, ocx * dx));
            float disc = fmaf(hb, hb, (-a) * c);
            float inv_a = 1.0f / a;
            float r1 = (-hb - sqrtf(disc)) * inv_a;
            ok = r1 >= 0.001f && r1 < INFINITY;
            oc64[0] = ocx; oc64[1] = ocy; oc64[2] = ocz; c64 = c;
        } else {
            double oc[3] = {O[0]-C[0], O[1]-C[1], O[2]-C[2]}, r2 = r * r;
            double c = fma(oc[2], oc[2], fma(oc[1], oc[1], oc[0] * oc[0])) - r2;
            double a = fma(D[2], D[2], fma(D[1], D[1], D[0] * D[0]));
            double hb = fma(oc[2], D[2], fma(oc[1], D[1], oc[0] * D[0]));
            double disc = fma(hb, hb, -(a * c));
            double r1 = (-hb - sqrt(disc)) * (1.0 / a);
            ok = r1 >= 0.001 && r1 < INFINITY;
            for (int k = 0; k < 3; ++k) oc64[k] = oc[k];
            c64 = c;
        }
        for (int k = 0; k < 3; ++k) ocf[k] = (float)oc64[k];
        // table: sc = sqrt(c) - 24u|oc| - 1e-20, rounded down; +inf if c <= 0
        double ocn = sqrt(oc64[0]*oc64[0] + oc64[1]*oc64[1] + oc64[2]*oc64[2]);
        float sc = (c64 > 0) ? down32(sqrt(c64) - 24 * u * ocn - 1e-20) : INFINITY;
        // lane: d^ = d * (1/sqrt(a)) in fp32
        float fdx = D[0], fdy = D[1], fdz = D[2];
        float fa = fmaf(fdz, fdz, fmaf(fdy, fdy, fdx * fdx));
        float inv = 1.0f / sqrtf(fa);
        float hx = fdx * inv, hy = fdy * inv, hz = fdz * inv;
        float hbp = fmaf(ocf[2], hz, fmaf(ocf[1], hy, ocf[0] * hx));
        float t = hbp + sc;
        uint32_t bits; memcpy(&bits, &t, 4);
        if (ok) {
            ++valid;
            if (!(bits >> 31)) ++miss;
            double need = (hbp + (double)sqrt(c64 > 0 ? c64 : 0)) / (u * ocn);   // how far inside the margin
            if (need > worst) worst = need;
        }
    }
    printf("f64=%d cases %ld valid %ld misses %ld worst (hb'+sqrt c)/(u|oc|) %.2f\n", f64, n, valid, miss, worst);
    return miss != 0;
}
