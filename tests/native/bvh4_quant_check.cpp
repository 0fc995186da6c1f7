/* Host check of pm_build.cpp quantize_bvh4 (tests/test_bvh_quant.py): every
 * decoded child box, computed with the device decode o + q * 2^e in float,
 * contains the float box of collapse_bvh4; codes and counts round-trip.
 * Mode "refs": the scene's refs are passed (triangles at storage slots
 * ref + 5, every 97th ref a disk): a leaf is coded LEAF_TRIS with ~first slot
 * exactly when all its refs are triangles at consecutive slots. Mode
 * "bigleaf": a leaf of >= LEAF_TRIS primitives cannot be coded (false). */
#include "pm_build.h"
#include <cstdio>
#include <cstring>
#include <cmath>
#include <random>
#include <cstdlib>
using namespace pm;
int main(int argc, char **argv) {
    const bool with_refs = argc > 2 && !strcmp(argv[2], "refs");
    if (argc > 2 && !strcmp(argv[2], "bigleaf")) {
        std::vector<float> node(32, 0.f);
        int codes[4] = {~0, 0, 0, 0}, counts[4] = {LEAF_TRIS, -1, -1, -1};
        for (int a = 0; a < 3; ++a) node[4 * (3 + a)] = 1.f;
        memcpy(&node[24], codes, 16); memcpy(&node[28], counts, 16);
        std::vector<uint32_t> q, refs(LEAF_TRIS);
        for (int i = 0; i < LEAF_TRIS; ++i) refs[i] = (uint32_t)i;
        const bool a = quantize_bvh4(node, q), b = quantize_bvh4(node, refs, q);
        counts[0] = LEAF_TRIS - 1; memcpy(&node[28], counts, 16);
        const bool c = quantize_bvh4(node, refs, q);
        const int cn = (int)(int16_t)(q[10] & 0xffff);
        printf("bigleaf %d %d fits %d count %x bad %d\n", a, b, c, cn, (a || b || !c || cn != (LEAF_TRIS | (LEAF_TRIS - 1))) ? 1 : 0);
        return (a || b || !c || cn != (LEAF_TRIS | (LEAF_TRIS - 1))) ? 1 : 0;
    }
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
    std::vector<uint32_t> q, refs;
    if (with_refs) {
        refs.resize(b.refs.size());
        for (size_t k = 0; k < refs.size(); ++k) refs[k] = k % 97 == 13 ? (1u << 30) | (uint32_t)k : (uint32_t)k + 5u;
    }
    if (!quantize_bvh4(w.nodes, refs, q)) { printf("encode failed\n"); return 1; }
    long flagged = 0;
    size_t nn = w.nodes.size() / 32; double vol_f = 0, vol_q = 0; long bad = 0;
    for (size_t i = 0; i < nn; ++i) {
        const float *n = &w.nodes[i * 32]; const uint32_t *u = &q[i * 16];
        int codes[4], counts[4]; memcpy(codes, n + 24, 16); memcpy(counts, n + 28, 16);
        for (int k = 0; k < 4; ++k) {
            int cn = (int)(int16_t)((u[10 + k / 2] >> (16 * (k & 1))) & 0xffff);
            int code = codes[k];
            if (with_refs && counts[k] > 0) {
                const uint32_t f = (uint32_t)~codes[k];
                bool tris = true;
                for (int j = 0; j < counts[k]; ++j) tris = tris && (refs[f + j] >> 30) == 0u;
                if (tris) { code = ~(int)(f + 5u); cn &= ~LEAF_TRIS; flagged++;
                            if (!(((u[10 + k / 2] >> (16 * (k & 1))) & 0xffff) & LEAF_TRIS)) bad++; }
                else if (cn & LEAF_TRIS) bad++;
            }
            if (cn != counts[k] || (int)u[12 + k] != code) bad++;
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
    printf("nodes %zu bad %ld volume ratio %.3f leaf_tris %ld\n", nn, bad, vol_q / vol_f, flagged);
    if (with_refs && flagged == 0) bad++;
    return bad != 0;
}
