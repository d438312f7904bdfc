/* abi_caller.c -- a plain C11 caller of include/orbslam_gpu.h, linked against
 * liborbslam_gpu.so the way the reference's C++ adapter would link it.
 *
 * Always (no device needed): the host-only entry points answer as the reference would --
 * ORBmatcher::DescriptorDistance (ORBmatcher.cc:1647-1663) and the glibc rand() stream
 * (DUtils::Random::RandomInt's source, Random.cpp:47-50).  Without a device every create()
 * must fail with ORB_E_NODEVICE (no CPU fallback).  With a device: ORBextractor::operator()
 * (ORBextractor.cc:1043-1105) on a seeded 640x480 image, from a host buffer to host
 * buffers; keypoints and descriptors are written to argv[1] for the test to compare. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "orbslam_gpu.h"

#define W 640
#define H 480
#define CAP 4096

static int fail(const char* what, int rc) {
    fprintf(stderr, "abi_caller: %s (rc %d)\n", what, rc);
    return 1;
}

/* the same generator as tests/test_library.py::_abi_image */
static void make_image(uint8_t* img) {
    uint32_t s = 12345u;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            s = s * 1664525u + 1013904223u;
            const int base = ((x / 40) * 37 + (y / 30) * 91) % 200;
            img[y * W + x] = (uint8_t)(base + (int)((s >> 24) & 31));
        }
}

int main(int argc, char** argv) {
    uint8_t a[32], b[32];
    /* the library implements the ABI revision this caller was compiled against */
    if (orbgpu_abi_version() != ORBGPU_ABI_VERSION) return fail("ABI revision mismatch", orbgpu_abi_version());
    for (int i = 0; i < 32; i++) {
        a[i] = (uint8_t)(i * 37 + 1);
        b[i] = (uint8_t)(i * 11 + 5);
    }
    int expect = 0;
    for (int i = 0; i < 32; i++) expect += __builtin_popcount((unsigned)(a[i] ^ b[i]));
    if (ORBmatcher_DescriptorDistance(a, b) != expect) return fail("DescriptorDistance", -1);
    if (ORBmatcher_DescriptorDistance(a, a) != 0) return fail("DescriptorDistance(a, a)", -1);

    orb_rng g;
    orb_rng_seed(&g, 1);
    if (orb_rng_rand(&g) != 1804289383) return fail("rand() after srand(1)", -1);

    const int dev = orbgpu_device_available();
    ORBextractor_h ex = NULL;
    int rc = ORBextractor_create(1000, 1.2f, 8, 20, 7, W, H, 1, &ex);
    if (!dev) {
        ORBmatcher_h m = NULL;
        if (rc != ORB_E_NODEVICE || ex != NULL) return fail("ORBextractor_create without a device", rc);
        rc = ORBmatcher_create(0.9f, 1, &m);
        if (rc != ORB_E_NODEVICE || m != NULL) return fail("ORBmatcher_create without a device", rc);
        printf("abi_caller ok: host entry points, ORB_E_NODEVICE without a device\n");
        return 0;
    }
    if (rc != ORB_OK) return fail("ORBextractor_create", rc);
    uint8_t* img = (uint8_t*)malloc((size_t)W * H);
    orb_kp* kps = (orb_kp*)malloc(sizeof(orb_kp) * CAP);
    uint8_t* desc = (uint8_t*)malloc((size_t)CAP * 32);
    if (!img || !kps || !desc) return fail("malloc", -1);
    make_image(img);
    int n = -1;
    rc = ORBextractor_extract(ex, img, W, H, W, kps, desc, CAP, &n);
    if (rc != ORB_OK || n <= 0) return fail("ORBextractor_extract", rc);
    int levels = 0;
    float sf = 0.f;
    if (ORBextractor_get_levels(ex, &levels, &sf) != ORB_OK || levels != 8 || sf != 1.2f) return fail("get_levels", -1);
    ORBextractor_destroy(ex);
    if (argc > 1) {
        FILE* f = fopen(argv[1], "wb");
        if (!f) return fail("fopen", -1);
        fwrite(&n, sizeof n, 1, f);
        fwrite(kps, sizeof(orb_kp), (size_t)n, f);
        fwrite(desc, 32, (size_t)n, f);
        fclose(f);
    }
    printf("abi_caller ok: %d keypoints\n", n);
    free(img);
    free(kps);
    free(desc);
    return 0;
}
