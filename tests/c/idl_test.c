/* C consumer of the orbslam3_extractFeatures replacement (include/orbgpu.h), compiled with gcc as
 * plain C the way the FastRPC host wrapper (LynxHardwareAccelerator.cpp:146-152) would call it.
 * Reads one side-by-side 2W x H Y8 frame from argv[1] (raw bytes), prints the counts and an FNV-1a
 * hash of every output array; tests/test_wire.py checks them against the oracle. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "orbgpu.h"

#define CAP 20000

static uint64_t fnv(const void* p, size_t n, uint64_t h) {
    const uint8_t* b = (const uint8_t*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

int main(int argc, char** argv) {
    if (argc < 4) return 2;
    const int W = atoi(argv[2]), H = atoi(argv[3]);
    const size_t len = (size_t)W * H * 2;
    uint8_t* img = (uint8_t*)malloc(len);
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(img, 1, len, f) != len) return 3;
    fclose(f);
    orbgpu_params prm = {2000, 1.2f, 8, 20, 7};
    orbgpu_ctx* ctx = NULL;
    if (orbgpu_create(&prm, 0, W, H, 2, &ctx) != ORBGPU_OK) {
        fprintf(stderr, "create: %s\n", orbgpu_last_error());
        return 4;
    }
    static int32_t x[2][CAP], y[2][CAP], ang[2][CAP], lvl[2][CAP];
    static uint8_t orb[2][CAP * 32];
    static int16_t idx[CAP], d1[CAP], d2[CAP];
    int n[2] = {0, 0}, mono[2] = {0, 0};
    const int rc = orbgpu_extract_features(ctx, img, (int)len, W, H, 2 * W, 20, 300, W, 0, W - 300, &n[0], x[0],
                                           y[0], ang[0], lvl[0], orb[0], &n[1], x[1], y[1], ang[1], lvl[1], orb[1],
                                           CAP, &mono[0], &mono[1], idx, d1, d2, CAP);
    if (rc != ORBGPU_OK) {
        fprintf(stderr, "extract: %s\n", orbgpu_last_error());
        return 5;
    }
    const int nq = n[0] - mono[0];
    for (int e = 0; e < 2; ++e) {
        uint64_t h = 1469598103934665603ull;
        h = fnv(x[e], 4 * (size_t)n[e], h);
        h = fnv(y[e], 4 * (size_t)n[e], h);
        h = fnv(ang[e], 4 * (size_t)n[e], h);
        h = fnv(lvl[e], 4 * (size_t)n[e], h);
        h = fnv(orb[e], 32 * (size_t)n[e], h);
        printf("eye %d n %d mono %d hash %016llx\n", e, n[e], mono[e], (unsigned long long)h);
    }
    uint64_t h = 1469598103934665603ull;
    h = fnv(idx, 2 * (size_t)nq, h);
    h = fnv(d1, 2 * (size_t)nq, h);
    h = fnv(d2, 2 * (size_t)nq, h);
    printf("matches %d hash %016llx\n", nq, (unsigned long long)h);
    orbgpu_destroy(ctx);
    free(img);
    return 0;
}
