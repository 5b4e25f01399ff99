/*
 * oracle_cli.c -- CPU-baseline driver for the oracle (TEST INFRASTRUCTURE ONLY).
 * Times LBGQuantizer::quantize (src/Quantizer.cpp:122-143) as restated in lbg_oracle.c
 * on a synthetic image or a P6 PPM, SCALED colour space, like
 * CompressedImage::compress (src/Compressor.cpp:118-123) times tiling + quantize.
 *   oracle_cli gen <S> <seed> <bw> <bh> <bits> <threads> [reps]
 *   oracle_cli ppm <path> <bw> <bh> <bits> <threads> [reps]
 * Prints one JSON line per rep.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

void orc_gen_image(uint32_t S, uint64_t seed, uint8_t *rgb);
size_t orc_num_blocks(int xSize, int ySize, int w, int h);
void orc_tile(const uint8_t *rgb, int xSize, int ySize, int w, int h, int cs, double *X, uint8_t *codes,
              uint8_t pad_code);
int orc_lbg(const double *X, size_t N, int D, int bits, double eps, int sum_mode, int threads, double *C_out,
            uint32_t *A_out, double *distortion_out, double *C_split_dump, uint32_t *A_dump);

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static uint8_t *read_ppm(const char *path, int *xs, int *ys) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    char magic[3] = {0};
    int mx;
    if (fscanf(f, "%2s %d %d %d", magic, xs, ys, &mx) != 4) { fclose(f); return NULL; }
    fgetc(f);
    size_t n = (size_t)(*xs) * (*ys) * 3;
    uint8_t *p = (uint8_t *)malloc(n);
    if (fread(p, 1, n, f) != n) { free(p); fclose(f); return NULL; }
    fclose(f);
    return p;
}

int main(int argc, char **argv) {
    if (argc < 2) { fprintf(stderr, "usage: see header\n"); return 2; }
    int xs, ys, bw, bh, bits, threads, reps = 1, a = 2;
    uint8_t *rgb;
    if (!strcmp(argv[1], "gen") && argc >= 8) {
        uint32_t S = (uint32_t)atoi(argv[2]);
        uint64_t seed = strtoull(argv[3], NULL, 0);
        xs = ys = (int)S;
        rgb = (uint8_t *)malloc((size_t)S * S * 3);
        orc_gen_image(S, seed, rgb);
        a = 4;
    } else if (!strcmp(argv[1], "ppm") && argc >= 7) {
        rgb = read_ppm(argv[2], &xs, &ys);
        if (!rgb) { fprintf(stderr, "cannot read %s\n", argv[2]); return 1; }
        a = 3;
    } else { fprintf(stderr, "bad args\n"); return 2; }
    bw = atoi(argv[a]); bh = atoi(argv[a + 1]); bits = atoi(argv[a + 2]); threads = atoi(argv[a + 3]);
    if (argc > a + 4) reps = atoi(argv[a + 4]);
    int D = 3 * bw * bh;
    size_t N = orc_num_blocks(xs, ys, bw, bh);
    double *X = (double *)malloc(N * D * sizeof(double));
    double *C = (double *)malloc(((size_t)1 << bits) * D * sizeof(double));
    uint32_t *A = (uint32_t *)malloc(N * sizeof(uint32_t));
    for (int r = 0; r < reps; r++) {
        double t0 = now();
        orc_tile(rgb, xs, ys, bw, bh, 1, X, NULL, 0);
        double t1 = now();
        double dist;
        int rc = orc_lbg(X, N, D, bits, 1e-6, 0, threads, C, A, &dist, NULL, NULL);
        double t2 = now();
        printf("{\"rc\": %d, \"N\": %zu, \"D\": %d, \"bits\": %d, \"threads\": %d, \"tile_s\": %.6f, "
               "\"quantize_s\": %.6f, \"distortion\": %.17g}\n",
               rc, N, D, bits, threads, t1 - t0, t2 - t1, dist);
        fflush(stdout);
    }
    return 0;
}
