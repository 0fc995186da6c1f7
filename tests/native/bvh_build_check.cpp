/* Host check of pm_build.cpp's threaded SAH build (tests/test_bvh_quant.py):
 * prints a hash of the binary nodes, refs and quantized 4-wide nodes of a
 * random triangle-box soup; the test runs it with PM_BUILD_THREADS 1 and N
 * and requires the same hash (the threaded build numbers subtrees exactly
 * as the serial recursion does, so the tree is identical). */
#include "pm_build.h"
#include <cstdio>
#include <random>
#include <cstring>
using namespace pm;
int main(int argc, char **argv) {
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(30.f, 525.f), E(-4.f, 4.f);
    std::vector<BuildPrim> prims(argc > 1 ? atoi(argv[1]) : 300000);
    for (size_t i = 0; i < prims.size(); ++i) {
        float c[3] = {U(rng), U(rng), U(rng)};
        for (int a = 0; a < 3; ++a) { float e = E(rng); prims[i].lo[a] = std::min(c[a], c[a] + e); prims[i].hi[a] = std::max(c[a], c[a] + e); }
        prims[i].ref = (uint32_t)i;
    }
    BvhOut b; build_bvh(prims, 60, b);
    Bvh4Out w; collapse_bvh4(b, 1, w);
    std::vector<uint32_t> q; quantize_bvh4(w.nodes, b.refs, q);
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t n) { const unsigned char *c = (const unsigned char *)p; for (size_t i = 0; i < n; ++i) { h ^= c[i]; h *= 1099511628211ull; } };
    mix(b.nodes.data(), b.nodes.size() * 4); mix(b.refs.data(), b.refs.size() * 4); mix(q.data(), q.size() * 4);
    printf("%zu nodes depth %d hash %016llx\n", b.nodes.size() / 16, b.depth, h);
}
