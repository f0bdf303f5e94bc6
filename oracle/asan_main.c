/* ASan/UBSan driver for the oracle (test infrastructure, SURVEY 5: a
 * sanitizer build of the CPU restatement).  `make -C oracle asan` builds it
 * with -fsanitize=address,undefined and runs detect+describe (upright,
 * rotated, extended, doubled) and the matcher on seeded synthetic frames,
 * including a tiny and a flat frame. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "surf_oracle.h"

static uint64_t rng = 0x5EED0000u;
static uint32_t next(void)
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)rng;
}

static int run(int w, int h, int pitch, const uint8_t* img, int upright, int extend, int doubled)
{
    or_param p;
    if (or_init_param(&p, 4, 2.f, doubled, 9, 2, upright, extend, 4) != 0) return -1;
    const int max_pts = 8192;
    or_point* pts = calloc(max_pts, sizeof(or_point));
    float* desc = calloc((size_t)max_pts * p.nfeatures, sizeof(float));
    int nc = 0;
    const int n = or_detect_and_compute(&p, img, w, h, pitch, pts, max_pts, desc, &nc);
    if (n > 1) or_match(pts, pts, desc, desc, n, n, p.nfeatures, 1);
    free(pts);
    free(desc);
    return n;
}

int main(void)
{
    const int sizes[][2] = {{320, 240}, {97, 61}, {33, 33}};
    for (int k = 0; k < 3; k++) {
        const int w = sizes[k][0], h = sizes[k][1], pitch = (w + 127) / 128 * 128;
        uint8_t* img = malloc((size_t)pitch * h);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < pitch; x++) {
                const int v = ((x / 7 + y / 5) & 1) ? 200 : 40;
                img[(size_t)y * pitch + x] = (uint8_t)(v + (int)(next() % 30));
            }
        for (int mode = 0; mode < 5; mode++) {
            const int n = run(w, h, pitch, img, mode == 0 || mode == 2, mode == 2 || mode == 3, mode == 4);
            printf("%dx%d mode %d: %d points\n", w, h, mode, n);
            if (n < 0) return 1;
        }
        memset(img, 128, (size_t)pitch * h);                  /* flat: no points */
        if (run(w, h, pitch, img, 0, 0, 0) != 0) return 1;
        free(img);
    }
    printf("asan ok\n");
    return 0;
}
