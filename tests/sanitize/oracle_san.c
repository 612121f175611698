/*
 * oracle_san.c — TEST HARNESS: drives the CPU oracle (oracle/oracle.c, test infrastructure) built with
 * -fsanitize=address,undefined by tests/test_sanitizers.py.  Reads render cases as whitespace-separated
 * text from stdin (doubles written with %.17g, so exact), renders each with oracle_render_f64 /
 * oracle_render_f32 / packed_render_f64, and prints "rc segments" and then every linear channel as a hex
 * float (%a) per case, so the test can compare bit for bit with the ordinary build.
 *
 * case: prec flags depth spp seed W H threads n_pixels
 *       camera: center[3] ulc[3] vu[3] vv[3] du[3] dv[3]
 *       n_spheres n_materials, spheres (cx cy cz r m), materials (kind hollow a0 a1 a2 fuzz ior)
 *       pixels[n_pixels] (n_pixels = 0: the whole image)
 * prec: 0 oracle f64, 1 oracle f32, 2 packed f64 (the AVX2 baseline; whole image, one 8x8-tile grid).
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../oracle/oracle.h"

static void rd(const char* fmt, void* p) {
    if (scanf(fmt, p) != 1) { fprintf(stderr, "oracle_san: bad input\n"); exit(2); }
}

int main(void) {
    unsigned n_cases = 0;
    rd("%u", &n_cases);
    for (unsigned ci = 0; ci < n_cases; ++ci) {
        unsigned prec, flags, depth, spp, W, H, threads, n_pix, ns, nm;
        uint64_t seed;
        rd("%u", &prec); rd("%u", &flags); rd("%u", &depth); rd("%u", &spp); rd("%" SCNu64, &seed);
        rd("%u", &W); rd("%u", &H); rd("%u", &threads); rd("%u", &n_pix);
        or_camera cam;
        cam.image_width = W; cam.image_height = H;
        double* cv[6] = {cam.center, cam.ulc, cam.vu, cam.vv, cam.du, cam.dv};
        for (int v = 0; v < 6; ++v)
            for (int a = 0; a < 3; ++a) rd("%lf", &cv[v][a]);
        rd("%u", &ns); rd("%u", &nm);
        double* cen = malloc(sizeof(double) * 3 * (ns ? ns : 1));
        double* rad = malloc(sizeof(double) * (ns ? ns : 1));
        uint32_t* mat = malloc(sizeof(uint32_t) * (ns ? ns : 1));
        or_material* mats = malloc(sizeof(or_material) * (nm ? nm : 1));
        for (unsigned i = 0; i < ns; ++i) {
            rd("%lf", &cen[3 * i]); rd("%lf", &cen[3 * i + 1]); rd("%lf", &cen[3 * i + 2]); rd("%lf", &rad[i]);
            rd("%u", &mat[i]);
        }
        for (unsigned i = 0; i < nm; ++i) {
            rd("%u", &mats[i].kind); rd("%u", &mats[i].hollow);
            rd("%lf", &mats[i].albedo[0]); rd("%lf", &mats[i].albedo[1]); rd("%lf", &mats[i].albedo[2]);
            rd("%lf", &mats[i].fuzz); rd("%lf", &mats[i].ior);
        }
        uint32_t* pix = n_pix ? malloc(sizeof(uint32_t) * n_pix) : NULL;
        for (unsigned i = 0; i < n_pix; ++i) rd("%u", &pix[i]);
        const or_scene sc = {ns, nm, cen, rad, mat, mats};
        const size_t n_out = n_pix ? n_pix : (size_t)W * H;
        uint8_t* rgb = malloc(3 * n_out);
        double* lin = malloc(sizeof(double) * 3 * n_out);
        uint64_t segs = 0, px = 0;
        int rc;
        if (prec == 2)
            rc = packed_render_f64(&sc, &cam, depth, spp, seed, 8, NULL, 0, rgb, lin, &segs, &px, (int)threads);
        else
            rc = (prec ? oracle_render_f32 : oracle_render_f64)(&sc, &cam, depth, spp, seed, flags, pix, n_pix, rgb,
                                                                  lin, &segs, (int)threads);
        printf("%d %" PRIu64 "\n", rc, segs);
        for (size_t i = 0; i < 3 * n_out; ++i) printf("%a\n", lin[i]);
        free(cen); free(rad); free(mat); free(mats); free(pix); free(rgb); free(lin);
    }
    return 0;
}
