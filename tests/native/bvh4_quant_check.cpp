/* Host check of pm_build.cpp quantize_bvh4 (tests/test_bvh_quant.py): every
 * decoded child box, computed with the device decode o + q * 2^e in float,
 * contains the float box of collapse_bvh4; codes and counts round-trip. */
#include "pm_build.h"
#include <cstdio>
#include <cstring>
#include <cmath>
#include <random>
#include <cstdlib>
using namespace pm;
int main(int argc, char **argv) {
    std::mt19937 rng(3);
    std::uniform_real_distribution<float> U(30.f, 525.f), E(-4.f, 4.f);
    std::vector<BuildPrim> prims(argc > 1 ? atoi(argv[1]) : 50000);
    for (size_t i = 0; i < prims.size(); ++i) {
        float c[3] = {U(rng), U(rng), U(rng)};
        for (int a = 0; a < 3; ++a) { float e = E(rng); prims[i].lo[a] = std::min(c[a], c[a] + e); prims[i].hi[a] = std::max(c[a], c[a] + e); }
        prims[i].ref = (uint32_t)i;
    }
    BvhOut b; build_bvh(prims, 60, b);
    Bvh4Out w; collapse_bvh4(b, 1, w);
    std::vector<uint32_t> q;
    if (!quantize_bvh4(w.nodes, q)) { printf("encode failed\n"); return 1; }
    size_t nn = w.nodes.size() / 32; double vol_f = 0, vol_q = 0; long bad = 0;
    for (size_t i = 0; i < nn; ++i) {
        const float *n = &w.nodes[i * 32]; const uint32_t *u = &q[i * 16];
        int codes[4], counts[4]; memcpy(codes, n + 24, 16); memcpy(counts, n + 28, 16);
        for (int k = 0; k < 4; ++k) {
            int cn = (int)(int16_t)((u[10 + k / 2] >> (16 * (k & 1))) & 0xffff);
            if (cn != counts[k] || (int)u[12 + k] != codes[k]) bad++;
            if (counts[k] == -1) continue;
            double vf = 1, vq = 1;
            for (int a = 0; a < 3; ++a) {
                float o; memcpy(&o, &u[a], 4);
                uint32_t eb = (u[3] >> (8 * a)) & 0xff; uint32_t bits = (eb - 1u) << 23; float s; memcpy(&s, &bits, 4);
                float lo = o + (float)((u[4 + a] >> (8 * k)) & 0xff) * s, hi = o + (float)((u[7 + a] >> (8 * k)) & 0xff) * s;
                if (lo > n[4 * a + k] || hi < n[4 * (3 + a) + k]) bad++;
                vf *= n[4 * (3 + a) + k] - n[4 * a + k]; vq *= hi - lo;
            }
            vol_f += vf; vol_q += vq;
        }
    }
    printf("nodes %zu bad %ld volume ratio %.3f\n", nn, bad, vol_q / vol_f);
    return bad != 0;
}
