// TEST INFRASTRUCTURE ONLY: a C-ABI shim over the reference's own DUtils::Random
// (/root/reference/Thirdparty/DBoW2/DUtils/Random.cpp, compiled from the reference
// sources by oracle/ref/Makefile into oracle/_ref/).  It lets the CPU tests pin the
// RANSAC draw stream (Random.cpp:47-50) to the reference code itself.
#include "Random.h"
#include <cstdlib>

extern "C" {
void ref_seed_rand(int seed) { DUtils::Random::SeedRand(seed); }            // Random.cpp:33-36
void ref_seed_rand_once(int seed) { DUtils::Random::SeedRandOnce(seed); }   // Random.cpp:38-45
int ref_random_int(int mn, int mx) { return DUtils::Random::RandomInt(mn, mx); }   // Random.cpp:47-50
int ref_libc_rand(void) { return rand(); }
}
