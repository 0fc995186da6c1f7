/* SAH build vs PLOC on C3's triangle soup (boxes as pm_commit pads them):
 * 4-wide surface-area cost, depth, stack bound and build time.
 *   g++ -O2 -std=c++17 -pthread -ffp-contract=off -Icuda-raytrace_amd/csrc -Iinclude \
 *       tools/bvh_quality.cpp cuda-raytrace_amd/csrc/pm_build.cpp -o /tmp/bq && /tmp/bq 1000000 8 16 */
#include "pm_build.h"
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
using namespace pm;
static double ms(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
}
int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000000;
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(30.f, 525.f), E(-4.f, 4.f);
    std::vector<BuildPrim> prims(n);
    for (int i = 0; i < n; ++i) {
        float c[3] = {U(rng), U(rng), U(rng)}, p[3][3];
        for (int a = 0; a < 3; ++a) { p[0][a] = c[a]; p[1][a] = c[a] + E(rng); p[2][a] = c[a] + E(rng); }
        for (int a = 0; a < 3; ++a) {
            float lo = std::min(p[0][a], std::min(p[1][a], p[2][a])), hi = std::max(p[0][a], std::max(p[1][a], p[2][a]));
            float pad = 1e-4f * std::max(1.0f, std::max(std::fabs(lo), std::fabs(hi)));
            prims[i].lo[a] = lo - pad; prims[i].hi[a] = hi + pad;
        }
        prims[i].ref = (uint32_t)i;
    }
    auto report = [&](const char *name, const BvhOut &b, double t) {
        Bvh4Out w;
        collapse_bvh4(b, 1, w);
        printf("%-10s build %8.1f ms  binary depth %3d  bvh4 nodes %8zu depth %3d max_stack %3d  SAH4 %.2f\n", name, t,
               b.depth, w.nodes.size() / 32, w.depth, w.max_stack, bvh4_sah_cost(w.nodes));
    };
    {
        std::vector<BuildPrim> p = prims;
        auto t0 = std::chrono::steady_clock::now();
        BvhOut b;
        build_bvh(p, 60, b);
        report("sah", b, ms(t0));
    }
    for (int k = 2; k < argc; ++k) {
        const int r = atoi(argv[k]);
        auto t0 = std::chrono::steady_clock::now();
        PlocTree t;
        build_ploc(prims, r, t);
        BvhOut b;
        ploc_to_bvh(prims, t, b);
        char name[32];
        snprintf(name, sizeof name, "ploc r%d", r);
        report(name, b, ms(t0));
        printf("           rounds %d\n", t.rounds);
    }
}
