/* tests/native/oracle_sanitize.c — runs the oracle restatement (oracle/rt_oracle.c,
 * test infrastructure) under AddressSanitizer + UndefinedBehaviorSanitizer
 * (tests/test_sanitizers.py): every scene, both RNG modes and both media orders, a
 * clipped output rectangle, the quantiser, the PPM writer and the RNG helpers.
 * Exit 0 = every render returned 0 and no sanitizer fired. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"

int main(void) {
    int bad = 0;
    static float img[24 * 16 * 3];
    static uint8_t rgb[24 * 16 * 3];
    static char text[24 * 16 * 16 + 64];
    for (int scene = 0; scene <= ORACLE_SCENE_EDGE_DEGENERATE; scene++) {
        if (scene == ORACLE_SCENE_EARTH) {   /* a synthetic 5x3 RGBA image for the texture */
            static uint8_t tex[5 * 3 * 4];
            for (int i = 0; i < (int)sizeof tex; i++) tex[i] = (uint8_t)(i * 37);
            oracle_set_image(tex, 5, 3, 4);
        }
        for (int mode = 0; mode < 2; mode++) {
            oracle_params p;
            memset(&p, 0, sizeof p);
            p.scene = scene;
            p.nx = 24; p.ny = 16; p.ns = 2;
            p.max_depth = 50;
            p.background = scene == ORACLE_SCENE_RANDOM || scene == ORACLE_SCENE_RANDOM_MOTION ||
                           scene == ORACLE_SCENE_EARTH || scene == ORACLE_SCENE_TWO_SPHERES;
            p.tmin = 0.001f;
            p.camera = scene == ORACLE_SCENE_CORNELL || scene == ORACLE_SCENE_CORNELL_SMOKE ? ORACLE_CAM_CORNELL
                     : scene == ORACLE_SCENE_FINAL ? ORACLE_CAM_FINAL_ALT : ORACLE_CAM_RANDOM;
            p.rng = mode;
            p.media_after = mode;
            p.forward = mode;
            p.chunk = mode ? 1 : 0;
            if (mode) { p.x0 = 3; p.y0 = 2; p.w = 11; p.h = 9; }
            p.threads = 1;
            p.seed = 5;
            oracle_stats st;
            if (oracle_render(&p, img, &st) != 0) { printf("scene %d mode %d: render failed\n", scene, mode); bad++; }
            const int n = mode ? 11 * 9 : 24 * 16;
            oracle_quantize(img, n, rgb);
            const long need = oracle_ppm_text(rgb, mode ? 11 : 24, mode ? 9 : 16, text, (long)sizeof text);
            if (need <= 0 || need > (long)sizeof text) { printf("scene %d: ppm %ld\n", scene, need); bad++; }
        }
    }
    double d[64];
    oracle_drand48(0, 64, d);
    oracle_counter_draws(1, 2, 3, 64, d);
    (void)oracle_medium_draw(1, 2, 3, 4, 5, 6);
    float ranvec[768];
    int32_t perm[768];
    oracle_perlin_tables(ranvec, perm);
    static char dump[1 << 20];
    for (int scene = 0; scene <= ORACLE_SCENE_EDGE_DEGENERATE; scene++)
        if (oracle_scene_dump(scene, dump, (long)sizeof dump) <= 0 && scene != ORACLE_SCENE_EDGE_EMPTY) {
            printf("scene %d: dump failed\n", scene);
            bad++;
        }
    printf(bad ? "FAILED %d\n" : "OK\n", bad);
    return bad ? 1 : 0;
}
