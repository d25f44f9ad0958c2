/* sanitize_driver.c — TEST INFRASTRUCTURE: drives the CPU oracle (mfx_oracle.c) through every
 * entry point on a small scene with all three primitive kinds, for an AddressSanitizer +
 * UndefinedBehaviorSanitizer build (tests/test_oracle_sanitizers.py; SURVEY.md §5 "ASan/UBSan on
 * the CPU oracle"). Exit status 0 and no sanitizer report is the pass condition. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mafrix_rt.h"

typedef struct OScene OScene;
OScene* oracle_create(const mfx_scene_desc* d);
void oracle_destroy(OScene* s);
int oracle_sample(const OScene* s, uint64_t seed, int32_t spp, int64_t sample_base, int32_t nthreads, double* frame,
                  double* stats);
int oracle_closest_hit(const OScene* s, int64_t n, const double* rays, double tmin, double tmax, double* t_out,
                       int32_t* prim_out, double* normal_out);
int oracle_any_hit(const OScene* s, int64_t n, const double* rays, double tmin, const double* tmax, int32_t* occ);
int oracle_bvh_leaves(const OScene* s, int32_t* indices, int32_t* leaf_first, int32_t* leaf_count, int32_t* nleaves);
int oracle_post_rgba8(const double* frame, int32_t w, int32_t h, uint8_t* rgba);

static void set3(double* p, double x, double y, double z) { p[0] = x; p[1] = y; p[2] = z; }

int main(void) {
    enum { NT = 40, NP = NT + 3 };
    mfx_prim prims[NP];
    memset(prims, 0, sizeof(prims));
    uint64_t r = 0x9e3779b97f4a7c15ULL;
    for (int i = 0; i < NT; i++) { /* a band of small triangles, some duplicated */
        prims[i].kind = MFX_PRIM_TRIANGLE;
        prims[i].material = i % 2;
        double cx = -0.8 + 1.6 * (double)(i % 8) / 7.0, cy = 0.2 + 0.1 * (double)(i / 8), cz = -1.0;
        if (i % 10 == 9) { cx = -0.8; cy = 0.2; } /* duplicate of triangle 0's position */
        r = r * 6364136223846793005ULL + 1442695040888963407ULL;
        double j = (double)(r >> 40) / 16777216.0 * 0.05;
        set3(prims[i].p[0], cx, cy, cz + j);
        set3(prims[i].p[1], cx + 0.1, cy, cz);
        set3(prims[i].p[2], cx, cy + 0.1, cz);
    }
    prims[NT].kind = MFX_PRIM_RECT; /* floor */
    set3(prims[NT].p[0], -4, 0, -4);
    set3(prims[NT].p[1], -4, 0, 4);
    set3(prims[NT].p[2], 4, 0, 4);
    set3(prims[NT].p[3], 4, 0, -4);
    prims[NT + 1].kind = MFX_PRIM_SPHERE;
    set3(prims[NT + 1].p[0], 0.6, 0.5, -1.5);
    prims[NT + 1].p[1][0] = 0.5;
    prims[NT + 2].kind = MFX_PRIM_SPHERE;
    prims[NT + 2].material = 1;
    set3(prims[NT + 2].p[0], -0.6, 0.5, -1.5);
    prims[NT + 2].p[1][0] = 0.5;
    double albedo[2][3] = {{0.725, 0.71, 0.68}, {0.63, 0.065, 0.05}};
    mfx_scene_desc d;
    memset(&d, 0, sizeof(d));
    d.prims = prims;
    d.nprims = NP;
    d.albedo = &albedo[0][0];
    d.nmat = 2;
    d.width = 24;
    d.height = 16;
    d.max_depth = 3;
    set3(d.light.p[0], -0.5, 2.0, -1.5);
    set3(d.light.p[1], -0.5, 2.0, -0.5);
    set3(d.light.p[2], 0.5, 2.0, -0.5);
    set3(d.light.p[3], 0.5, 2.0, -1.5);
    set3(d.light.normal, 0, -1, 0);
    set3(d.light.intensity, 10, 10, 10);
    set3(d.camera.position, 0, 1, 3);
    set3(d.camera.direction, 0, -0.2, -1);
    d.camera.fov = 120;
    d.camera.aspect = 1.5;

    OScene* s = oracle_create(&d);
    if (!s) return 2;
    const int64_t npix = (int64_t)d.width * d.height;
    double* frame = calloc((size_t)npix * 4, sizeof(double));
    double stats[8];
    if (oracle_sample(s, 0x4D414652ULL, 3, 0, 1, frame, stats) != 0) return 3;
    uint8_t* rgba = calloc((size_t)npix * 4, 1);
    if (oracle_post_rgba8(frame, d.width, d.height, rgba) != 0) return 4;
    enum { NR = 500 };
    double rays[NR * 6], t[NR], nrm[NR * 3], tmax[NR];
    int32_t prim[NR], occ[NR];
    for (int k = 0; k < NR; k++) {
        r = r * 6364136223846793005ULL + 1442695040888963407ULL;
        double a = (double)(r >> 40) / 16777216.0 * 6.283185307179586, b = (double)((r >> 16) & 0xffffff) / 16777216.0;
        set3(rays + 6 * k, 0, 1, 3);
        double dx = cos(a) * b, dy = -0.3 - 0.5 * b, dz = -1.0;
        double l = sqrt(dx * dx + dy * dy + dz * dz);
        set3(rays + 6 * k + 3, dx / l, dy / l, dz / l);
        tmax[k] = 1.0 + 4.0 * b;
    }
    if (oracle_closest_hit(s, NR, rays, 1e-6, 99999999., t, prim, nrm) != 0) return 5;
    if (oracle_any_hit(s, NR, rays, 1e-6, tmax, occ) != 0) return 6;
    int32_t idx[NP], lf[NP], lc[NP], nl = 0;
    if (oracle_bvh_leaves(s, idx, lf, lc, &nl) != 0 || nl < 1) return 7;
    int hits = 0;
    for (int k = 0; k < NR; k++) hits += prim[k] >= 0;
    printf("sanitized oracle run: %d of %d rays hit, %d reference leaves, %.0f rays traced\n", hits, NR, nl,
           stats[0] + stats[1] + stats[2]);
    free(frame);
    free(rgba);
    oracle_destroy(s);
    return 0;
}
