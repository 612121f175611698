// Fuzz of the general-sweep distance filter (rt_kernel.hip: nearest_hit / filter_group), test
// infrastructure for tests/test_filter_margin.py.  Claim checked: whenever the reference's own
// discriminant is >= 0 for a (ray, sphere) -- so the reference may hit it -- the filter's
// D = r2f - y'^2 - x'^2, computed exactly as the kernel does (basis scaled by 1/sqrt(1 + m/r2min),
// margin m = 48 u ((max|c|_1 + |o|_1)^2 + max r2f)), has its sign bit clear, i.e. the filter
// passes the sphere and the exact test decides.  Cases are adversarial: the centre is put
// at distance r(1 +- 5e-4 * 10^-6U) from the ray's line (near tangency), scene scales 0.1..1000,
// radii 1e-3..1 of the scale, near-vertical and non-unit directions.
// The reference formulas are objects.rs:252-257 (hit_packed, FMA where it writes mul_add) and
// objects.rs:217-222 (Sphere::hit, no FMA).
// mode 0: fp32 hit_packed; 1: fp32 scalar Sphere::hit; 2: fp64 hit_packed; 3: fp64 scalar.
// LOCAL = 1: the MEGA kernels' cluster-local frame (pack_local + nearest_hit): the whole case is moved
// far from the origin (up to 1000x its size), a cluster centre Ck (fp32) is put 1..100 radii from the
// sphere, and the filter sees c' = RN_f(c - Ck), o' = o - Ck (fp64 rays: in double, then rounded) with
// the margin 48 u ((|c'|_1 + |o'|_1)^2 + r2f): the same formula in local magnitudes.
// Usage: filter_margin_fuzz N MODE [SEED] [LOCAL] -> prints misses and the worst margin needed, in u.
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static double U() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (s >> 11) * 0x1.0p-53; }
static double N() { double a = U(), b = U(); return sqrt(-2 * log(a + 1e-300)) * cos(6.283185307179586 * b); }
static const float KM = 48.0f * 0x1.0p-24f;
// v_rsq_f32 (1 ulp): the correctly rounded value moved by -1, 0 or +1 ulp at random
static float rsq(float x) {
    float r = 1.0f / sqrtf(x);
    const double v = U();
    if (v < 1.0 / 3) r = nextafterf(r, 0.0f); else if (v < 2.0 / 3) r = nextafterf(r, INFINITY);
    return r;
}
static float up32(double v) { float f = (float)v; if ((double)f < v) f = nextafterf(f, INFINITY); return f; }
int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 10000000;
    const int mode = argc > 2 ? atoi(argv[2]) : 0;
    if (argc > 3) s = strtoull(argv[3], 0, 0) | 1;
    const int local = argc > 4 ? atoi(argv[4]) : 0;
    long acc = 0, miss = 0; double worst = 0;
    for (long it = 0; it < n; ++it) {
        double S = pow(10.0, -1 + 4 * U());
        double O[3] = {N() * S, N() * S, N() * S};
        double dd[3] = {N(), N(), N()};
        if (U() < 0.1) { dd[0] *= 1e-3; dd[2] *= 1e-3; }
        double dl = sqrt(dd[0]*dd[0]+dd[1]*dd[1]+dd[2]*dd[2]);
        double sc = U() < 0.3 ? 3.7 : 1.0;
        double D[3] = {dd[0]/dl*sc, dd[1]/dl*sc, dd[2]/dl*sc};
        if (mode < 2) for (int k = 0; k < 3; ++k) { O[k] = (float)O[k]; D[k] = (float)D[k]; }
        double r = S * pow(10.0, -3 + 3 * U());
        double tpar = (U() * 4 - 1) * S * 3;
        double px[3] = {N(), N(), N()};
        double a0 = D[0]*D[0]+D[1]*D[1]+D[2]*D[2];
        double pd = (px[0]*D[0]+px[1]*D[1]+px[2]*D[2]) / a0;
        for (int k = 0; k < 3; ++k) px[k] -= pd * D[k];
        double pl = sqrt(px[0]*px[0]+px[1]*px[1]+px[2]*px[2]);
        double rho = r * (1 + (U() - 0.5) * 1e-3 * pow(10.0, -6 * U()));
        double C[3];
        for (int k = 0; k < 3; ++k) C[k] = O[k] + tpar * D[k] / sqrt(a0) + px[k] / pl * rho;
        float Ck[3] = {0, 0, 0};
        if (local) {   // far from the origin; a cluster centre near the sphere
            const double tm = S * pow(10.0, 3 * U());
            const double g = r * pow(10.0, 2 * U());
            for (int k = 0; k < 3; ++k) {
                const double t = N() * tm;
                O[k] += t; C[k] += t;
                Ck[k] = (float)(C[k] + N() * g);
            }
            if (mode < 2) for (int k = 0; k < 3; ++k) O[k] = (float)O[k];
        }
        if (mode < 2) for (int k = 0; k < 3; ++k) C[k] = (float)C[k];
        int ref_ok;
        float r2f;
        if (mode < 2) {
            float rr = (float)r, r2 = rr * rr;
            float ox = O[0], oy = O[1], oz = O[2], dx = D[0], dy = D[1], dz = D[2], cx = C[0], cy = C[1], cz = C[2];
            float ocx = ox - cx, ocy = oy - cy, ocz = oz - cz, disc;
            if (mode == 0) {
                float a = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
                float hb = fmaf(ocz, dz, fmaf(ocy, dy, ocx * dx));
                float c = fmaf(ocz, ocz, fmaf(ocy, ocy, ocx * ocx)) - r2;
                disc = fmaf(hb, hb, (-a) * c);
            } else {
                float a = (dx * dx + dy * dy) + dz * dz;
                float hb = (ocx * dx + ocy * dy) + ocz * dz;
                float c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r2;
                disc = hb * hb - a * c;
            }
            ref_ok = disc >= 0.0f;
            r2f = r2;
        } else {
            double rr = r, r2 = rr * rr;
            double oc[3] = {O[0]-C[0], O[1]-C[1], O[2]-C[2]}, disc;
            if (mode == 2) {
                double a = fma(D[2], D[2], fma(D[1], D[1], D[0] * D[0]));
                double hb = fma(oc[2], D[2], fma(oc[1], D[1], oc[0] * D[0]));
                double c = fma(oc[2], oc[2], fma(oc[1], oc[1], oc[0] * oc[0])) - r2;
                disc = fma(hb, hb, -(a * c));
            } else {
                double a = (D[0]*D[0] + D[1]*D[1]) + D[2]*D[2];
                double hb = (oc[0]*D[0] + oc[1]*D[1]) + oc[2]*D[2];
                double c = ((oc[0]*oc[0] + oc[1]*oc[1]) + oc[2]*oc[2]) - r2;
                disc = hb * hb - a * c;
            }
            ref_ok = disc >= 0.0;
            r2f = (float)r2;
            if ((double)r2f < r2) r2f = nextafterf(r2f, INFINITY);
        }
        // filter (kernel formula), fp32
        float fdx = D[0], fdy = D[1], fdz = D[2], fox = O[0], foy = O[1], foz = O[2];
        float cx = C[0], cy = C[1], cz = C[2];
        float L = fmaf(fdz, fdz, fdx * fdx);
        float af = fmaf(fdz, fdz, fmaf(fdy, fdy, fdx * fdx));
        float s1 = rsq(L), s2 = rsq(L * af);
        float on = fabsf(fox) + fabsf(foy) + fabsf(foz);
        // the kernel's m uses the scene-wide max |c|_1 and max r2f, and its r2min is the scene's
        // smallest r2f; this sphere's own values bound those from the unfavourable side, so the
        // inflation tested here (r2f * (1 + m / r2f) = r2f + m) is never larger than the kernel's
        if (local) {   // pack_local's c' and the kernel's o'
            cx = (float)((double)C[0] - (double)Ck[0]); cy = (float)((double)C[1] - (double)Ck[1]);
            cz = (float)((double)C[2] - (double)Ck[2]);
            if (mode < 2) { fox = fox - Ck[0]; foy = foy - Ck[1]; foz = foz - Ck[2]; }
            else { fox = (float)(O[0] - (double)Ck[0]); foy = (float)(O[1] - (double)Ck[1]); foz = (float)(O[2] - (double)Ck[2]); }
            on = ((fabsf(fox) + fabsf(foy)) + fabsf(foz));
        }
        float cmax = fabsf(cx) + fabsf(cy) + fabsf(cz);
        float pm = cmax + on;
        float m = KM * fmaf(pm, pm, r2f);
        float r2min = r2f;
        // basis scaled by sigma = 1/sqrt(1 + m/r2min): the test x'^2 + y'^2 <= r2f is
        // x^2 + y^2 <= r2f (1 + m/r2min) >= r2f + m, with no per-pair add
        float sg = rsq(fmaf(m, up32(1.0 / r2min), 1.0f));
        float t1 = s1 * sg, t2 = s2 * sg;
        float e1x = fdz * t1, e1z = -fdx * t1;
        float e2x = -(fdx * fdy) * t2, e2y = L * t2, e2z = -(fdy * fdz) * t2;
        float oe1 = fmaf(foz, e1z, fox * e1x), oe2 = fmaf(foz, e2z, fmaf(foy, e2y, fox * e2x));
        float x = fmaf(cx, e1x, fmaf(cz, e1z, -oe1));
        float y = fmaf(cx, e2x, fmaf(cy, e2y, fmaf(cz, e2z, -oe2)));
        float Dv = fmaf(-x, x, fmaf(-y, y, r2f));
        uint32_t bits; memcpy(&bits, &Dv, 4);
        if (ref_ok) {
            ++acc;
            if (bits >> 31) ++miss;
            double need = (((double)x * x + (double)y * y) / ((double)sg * sg) - r2f) / ((double)pm * pm + r2f) / 0x1.0p-24;
            if (need > worst) worst = need;
        }
    }
    printf("mode %d: cases %ld ref-accepted %ld  filter misses %ld  worst need %.2f u\n", mode, n, acc, miss, worst);
    return miss != 0;
}
