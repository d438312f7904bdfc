/*
 * rng.c -- TEST INFRASTRUCTURE ONLY (parity oracle).
 *
 * glibc rand() restatement (stdlib/random_r.c, TYPE_3: degree 31, separation
 * 3, additive feedback, 310 warm-up draws) and DUtils::Random::RandomInt
 * (reference Thirdparty/DBoW2/DUtils/Random.cpp:47-50).  Pinned against the
 * host libc rand() in tests/test_oracle_kat.py.
 */
#include "orb_oracle.h"

void ora_rng_seed(ora_rng* g, unsigned int seed)
{
    if (seed == 0) seed = 1;
    int32_t word = (int32_t)seed;
    g->tbl[0] = word;
    for (int i = 1; i < 31; i++) {
        long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        g->tbl[i] = word;
    }
    g->f = 3;
    g->r = 0;
    for (int i = 0; i < 310; i++) (void)ora_rng_rand(g);
}

int ora_rng_rand(ora_rng* g)
{
    uint32_t val = (uint32_t)g->tbl[g->f] + (uint32_t)g->tbl[g->r];
    g->tbl[g->f] = (int32_t)val;
    int result = (int)(val >> 1);
    if (++g->f >= 31) { g->f = 0; ++g->r; }
    else if (++g->r >= 31) g->r = 0;
    return result;
}

int ora_rng_random_int(ora_rng* g, int min, int max)
{
    int d = max - min + 1;
    return (int)(((double)ora_rng_rand(g) / ((double)2147483647 + 1.0)) * d) + min;
}
