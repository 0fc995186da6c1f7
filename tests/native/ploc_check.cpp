/* Host check of pm_build.cpp's PLOC restatement (tests/test_bvh_quant.py):
 * on a random triangle-box soup, the tree is a binary tree over all n
 * leaves (every Morton position reached once from the root, n - 1 internal
 * nodes), each internal box is exactly the union of its children's boxes,
 * the order is a permutation sorted by Morton code, and the 4-wide collapse
 * quantizes with every decoded box containing its float box. Prints a hash
 * of the tree so the test can require the same tree for 1 and N threads. */
#include "pm_build.h"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <random>
using namespace pm;
static int fail(const char *m) { printf("FAIL %s\n", m); return 1; }
int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 50000, radius = argc > 2 ? atoi(argv[2]) : 3;
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> U(30.f, 525.f), E(-4.f, 4.f);
    std::vector<BuildPrim> prims(n);
    for (int i = 0; i < n; ++i) {
        float c[3] = {U(rng), U(rng), U(rng)};
        for (int a = 0; a < 3; ++a) { float e = E(rng); prims[i].lo[a] = std::min(c[a], c[a] + e); prims[i].hi[a] = std::max(c[a], c[a] + e); }
        prims[i].ref = (uint32_t)i;
    }
    PlocTree t;
    build_ploc(prims, radius, t);
    if ((int)t.order.size() != n || (int)t.left.size() != n - 1 || t.root != 2 * n - 2) return fail("sizes / root");
    std::vector<char> seen(n, 0);
    for (uint32_t o : t.order) { if (o >= (uint32_t)n || seen[o]) return fail("order not a permutation"); seen[o] = 1; }
    for (int p = 1; p < n; ++p)
        if (ploc_morton(prims[t.order[p - 1]], t.frame_lo, t.frame_scale) > ploc_morton(prims[t.order[p]], t.frame_lo, t.frame_scale) ||
            (ploc_morton(prims[t.order[p - 1]], t.frame_lo, t.frame_scale) == ploc_morton(prims[t.order[p]], t.frame_lo, t.frame_scale) &&
             t.order[p - 1] > t.order[p]))
            return fail("not in Morton order");
    auto box = [&](int id, float lo[3], float hi[3]) {
        if (id < n) { std::memcpy(lo, prims[t.order[id]].lo, 12); std::memcpy(hi, prims[t.order[id]].hi, 12); }
        else { std::memcpy(lo, &t.box[(size_t)(id - n) * 6], 12); std::memcpy(hi, &t.box[(size_t)(id - n) * 6 + 3], 12); }
    };
    std::vector<char> reach(2 * n - 1, 0);
    std::vector<int> st{t.root};
    while (!st.empty()) {
        const int id = st.back(); st.pop_back();
        if (reach[id]++) return fail("node reached twice");
        if (id < n) continue;
        const int k = id - n, ch[2] = {t.left[k], t.right[k]};
        float lo[3], hi[3], a[3], b[3], c2[3], d[3];
        box(id, lo, hi); box(ch[0], a, b); box(ch[1], c2, d);
        for (int x = 0; x < 3; ++x)
            if (lo[x] != std::min(a[x], c2[x]) || hi[x] != std::max(b[x], d[x])) return fail("box is not the union");
        st.push_back(ch[0]); st.push_back(ch[1]);
    }
    for (int i = 0; i < 2 * n - 1; ++i) if (!reach[i]) return fail("node unreachable");
    BvhOut b; ploc_to_bvh(prims, t, b);
    Bvh4Out w; collapse_bvh4(b, 1, w);
    bvh4_bfs_order(w.nodes);
    std::vector<uint32_t> q;
    if (!quantize_bvh4(w.nodes, b.refs, q)) return fail("quantize");
    unsigned long long h = 1469598103934665603ull;
    auto mix = [&](const void *p, size_t m) { const unsigned char *c = (const unsigned char *)p; for (size_t i = 0; i < m; ++i) { h ^= c[i]; h *= 1099511628211ull; } };
    mix(t.order.data(), t.order.size() * 4); mix(t.left.data(), t.left.size() * 4); mix(t.right.data(), t.right.size() * 4);
    mix(q.data(), q.size() * 4);
    printf("ok rounds %d bvh4 %zu depth %d stack %d hash %016llx\n", t.rounds, w.nodes.size() / 32, w.depth, w.max_stack, h);
    return 0;
}
