/*
 * synth.c -- deterministic synthetic grayscale frames and PGM I/O.
 *
 * Host-side tooling shared by the bench and the tests (no GPU, no oracle).
 * Frame f of a batch is seeded with 0x5EED0000 + f:
 * a smooth linear gradient, K Gaussian blobs with sigma in [1.5, 80] px drawn
 * with density ~ sigma^-3 (equal image area per scale band, like natural
 * images) and amplitude +-U[20, 90], and +-4 uniform noise, clamped to
 * [0, 255].  K defaults to 8000 per 1920x1080 (scaled with the area), which
 * yields ~3k keypoints per 1080p frame at thresh=4 and responses in every
 * octave, so the reference's counter-chain restart (surfd.cu:825-826) never
 * triggers.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SYNTH_SEED_BASE 0x5EED0000ull

static inline uint64_t splitmix64(uint64_t* s)
{
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double u01(uint64_t* s) { return (double)(splitmix64(s) >> 11) * (1.0 / 9007199254740992.0); }
static inline double uab(uint64_t* s, double a, double b) { return a + (b - a) * u01(s); }

/* Default blob count for a w x h frame. */
int surf_synth_default_blobs(int w, int h)
{
    const double k = 8000.0 * ((double)w * h) / (1920.0 * 1080.0);
    return k < 64.0 ? 64 : (int)(k + 0.5);
}

/* One frame into dst (row pitch `pitch` bytes); nblobs <= 0 selects the
 * default density. */
int surf_synth_frame(uint8_t* dst, int w, int h, int pitch, uint64_t seed, int nblobs)
{
    if (w <= 0 || h <= 0 || pitch < w) return -1;
    if (nblobs <= 0) nblobs = surf_synth_default_blobs(w, h);
    float* acc = (float*)malloc(sizeof(float) * (size_t)w * h);
    float* ex = (float*)malloc(sizeof(float) * (size_t)w);
    float* ey = (float*)malloc(sizeof(float) * (size_t)h);
    if (!acc || !ex || !ey) { free(acc); free(ex); free(ey); return -2; }
    uint64_t st = seed;
    const double g0 = uab(&st, 70.0, 180.0);
    const double gx = uab(&st, -50.0, 50.0) / w;
    const double gy = uab(&st, -50.0, 50.0) / h;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++)
            acc[(size_t)y * w + x] = (float)(g0 + gx * x + gy * y);
    for (int k = 0; k < nblobs; k++) {
        const double cx = uab(&st, 0.0, (double)w);
        const double cy = uab(&st, 0.0, (double)h);
        /* sigma in [1.5, 80] with density ~ sigma^-3 (equal image area per
         * scale band, like natural images): inverse CDF of that density */
        const double ia = 1.0 / (1.5 * 1.5), ib = 1.0 / (80.0 * 80.0);
        const double sigma = 1.0 / sqrt(ia - u01(&st) * (ia - ib));
        const double amp = uab(&st, 20.0, 90.0) * (u01(&st) < 0.5 ? -1.0 : 1.0);
        const double inv = 1.0 / (2.0 * sigma * sigma);
        const int R = (int)ceil(3.5 * sigma);
        int x0 = (int)floor(cx) - R, x1 = (int)floor(cx) + R;
        int y0 = (int)floor(cy) - R, y1 = (int)floor(cy) + R;
        if (x0 < 0) x0 = 0;
        if (y0 < 0) y0 = 0;
        if (x1 > w - 1) x1 = w - 1;
        if (y1 > h - 1) y1 = h - 1;
        for (int x = x0; x <= x1; x++) ex[x] = (float)exp(-((x - cx) * (x - cx)) * inv);
        for (int y = y0; y <= y1; y++) ey[y] = (float)(amp * exp(-((y - cy) * (y - cy)) * inv));
        for (int y = y0; y <= y1; y++) {
            float* row = acc + (size_t)y * w;
            const float a = ey[y];
            for (int x = x0; x <= x1; x++) row[x] += a * ex[x];
        }
    }
    for (int y = 0; y < h; y++) {
        uint8_t* out = dst + (size_t)y * pitch;
        const float* row = acc + (size_t)y * w;
        for (int x = 0; x < w; x++) {
            const double v = row[x] + uab(&st, -4.0, 4.0);
            long q = lrint(v);
            out[x] = (uint8_t)(q < 0 ? 0 : (q > 255 ? 255 : q));
        }
        for (int x = w; x < pitch; x++) out[x] = 0;
    }
    free(acc);
    free(ex);
    free(ey);
    return 0;
}

typedef struct {
    uint8_t* dst;
    int n, w, h, pitch, first, nthreads, tid, nblobs;
    size_t stride;
    int err;
} synth_job;

static void* synth_worker(void* arg)
{
    synth_job* j = (synth_job*)arg;
    for (int f = j->tid; f < j->n; f += j->nthreads) {
        int e = surf_synth_frame(j->dst + (size_t)f * j->stride, j->w, j->h, j->pitch,
                                 SYNTH_SEED_BASE + (uint64_t)(j->first + f), j->nblobs);
        if (e) j->err = e;
    }
    return NULL;
}

/* Frames first .. first+n-1 into dst (frame stride `stride` bytes). */
int surf_synth_frames(uint8_t* dst, int n, int w, int h, int pitch, size_t stride,
                      int first, int nblobs, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n) nthreads = n > 0 ? n : 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
    synth_job* jobs = (synth_job*)calloc(nthreads, sizeof(synth_job));
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (synth_job){dst, n, w, h, pitch, first, nthreads, t, nblobs, stride, 0};
        pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
    }
    int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].err) err = jobs[t].err;
    }
    free(th);
    free(jobs);
    return err;
}

/* Binary PGM (P5, maxval 255) header probe: fills w, h; returns the byte
 * offset of the pixel data or -1. */
long surf_pgm_info(const char* path, int* w, int* h)
{
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    char magic[3] = {0};
    int maxv = 0;
    long off = -1;
    if (fscanf(f, "%2s", magic) == 1 && strcmp(magic, "P5") == 0) {
        int vals[3], got = 0;
        while (got < 3) {
            int c = fgetc(f);
            if (c == EOF) break;
            if (c == '#') { while (c != '\n' && c != EOF) c = fgetc(f); continue; }
            if (c >= '0' && c <= '9') { ungetc(c, f); if (fscanf(f, "%d", &vals[got]) == 1) got++; }
        }
        if (got == 3) {
            fgetc(f);  /* single whitespace before raster */
            *w = vals[0]; *h = vals[1]; maxv = vals[2];
            if (maxv == 255) off = ftell(f);
        }
    }
    fclose(f);
    return off;
}

/* Read the raster into dst with row pitch `pitch` (>= w). */
int surf_pgm_read(const char* path, uint8_t* dst, int pitch)
{
    int w = 0, h = 0;
    long off = surf_pgm_info(path, &w, &h);
    if (off < 0) return -1;
    FILE* f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, off, SEEK_SET);
    int rc = 0;
    for (int y = 0; y < h && !rc; y++) {
        if (fread(dst + (size_t)y * pitch, 1, (size_t)w, f) != (size_t)w) rc = -2;
        for (int x = w; x < pitch; x++) dst[(size_t)y * pitch + x] = 0;
    }
    fclose(f);
    return rc;
}

/* 2x2 box average (round half up), used to derive the 640x480 config #1
 * frame from the 1280x960 data/left.pgm. */
void surf_downsample2(const uint8_t* src, int w, int h, int spitch, uint8_t* dst, int dpitch)
{
    for (int y = 0; y < h / 2; y++)
        for (int x = 0; x < w / 2; x++) {
            const uint8_t* a = src + (size_t)(2 * y) * spitch + 2 * x;
            const int s = a[0] + a[1] + a[spitch] + a[spitch + 1];
            dst[(size_t)y * dpitch + x] = (uint8_t)((s + 2) / 4);
        }
}
