/* Node visits per ray of a W-wide BVH (W = 2, 4, 8) collapsed from the same
 * binned-SAH binary tree over C3's triangle soup — a CPU estimate of what an
 * 8-wide tree would save k_trace_pool (whose time per 1M paths tracks its
 * node visits). Closest-hit traversal, hit internal children
 * entered nearest first, leaves (one triangle each) tested when their box is
 * hit; rays from random points of the soup's box in uniform directions.
 *   g++ -O2 -std=c++17 -pthread -ffp-contract=off -Icuda-raytrace_amd/csrc -Iinclude \
 *       tools/bvh_width_sim.cpp cuda-raytrace_amd/csrc/pm_build.cpp -o /tmp/bws && /tmp/bws 1000000 20000 */
#include "pm_build.h"
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
using namespace pm;

struct Child { float lo[3], hi[3]; int code; int count; };  /* count 0: internal node `code`; >0: leaf refs [~code, ..) */
struct Node { std::vector<Child> ch; };

static const BvhOut *B;
static std::vector<Node> W;

static Child bin_child(int node, int k) {
    const float *n = &B->nodes[(size_t)node * 16];
    Child c;
    for (int a = 0; a < 3; ++a) { c.lo[a] = n[6 * k + a]; c.hi[a] = n[6 * k + 3 + a]; }
    int ints[4];
    std::memcpy(ints, &n[12], sizeof(ints));
    c.code = ints[k]; c.count = ints[2 + k];
    return c;
}
static float area(const Child &c) {
    const float dx = c.hi[0] - c.lo[0], dy = c.hi[1] - c.lo[1], dz = c.hi[2] - c.lo[2];
    return dx * dy + dy * dz + dz * dx;
}
static int collapse(int node, int width) {
    std::vector<Child> ch;
    for (int k = 0; k < 2; ++k) { Child c = bin_child(node, k); if (c.count >= 0) ch.push_back(c); }
    while ((int)ch.size() < width) {
        int best = -1;
        for (size_t i = 0; i < ch.size(); ++i)
            if (ch[i].count == 0 && (best < 0 || area(ch[i]) > area(ch[best]))) best = (int)i;
        if (best < 0) break;
        const int inner = ch[best].code;
        ch.erase(ch.begin() + best);
        for (int k = 0; k < 2; ++k) { Child c = bin_child(inner, k); if (c.count >= 0) ch.push_back(c); }
    }
    const int me = (int)W.size();
    W.push_back(Node{});
    for (Child &c : ch)
        if (c.count == 0) c.code = collapse(c.code, width);
    W[me].ch = ch;
    return me;
}

struct Tri { float p0[3], p1[3], p2[3]; };
static std::vector<Tri> T;

static bool isect(const Tri &t, const float o[3], const float d[3], float tmax, float &th) {
    float e0[3], e1[3], n[3], e2[3], i[3];
    for (int a = 0; a < 3; ++a) { e0[a] = t.p1[a] - t.p0[a]; e1[a] = t.p0[a] - t.p2[a]; }
    n[0] = e1[1] * e0[2] - e1[2] * e0[1]; n[1] = e1[2] * e0[0] - e1[0] * e0[2]; n[2] = e1[0] * e0[1] - e1[1] * e0[0];
    const float den = n[0] * d[0] + n[1] * d[1] + n[2] * d[2];
    const float r = 1.f / den;
    for (int a = 0; a < 3; ++a) e2[a] = (t.p0[a] - o[a]) * r;
    i[0] = d[1] * e2[2] - d[2] * e2[1]; i[1] = d[2] * e2[0] - d[0] * e2[2]; i[2] = d[0] * e2[1] - d[1] * e2[0];
    const float b = i[0] * e1[0] + i[1] * e1[1] + i[2] * e1[2], g = i[0] * e0[0] + i[1] * e0[1] + i[2] * e0[2];
    const float tt = n[0] * e2[0] + n[1] * e2[1] + n[2] * e2[2];
    if (tt > 1e-3f && tt < tmax && b >= 0.f && g >= 0.f && b + g <= 1.f) { th = tt; return true; }
    return false;
}
static float slab(const Child &c, const float o[3], const float inv[3], float tmax) {
    float tn = 0.f, tf = tmax;
    for (int a = 0; a < 3; ++a) {
        float t0 = (c.lo[a] - o[a]) * inv[a], t1 = (c.hi[a] - o[a]) * inv[a];
        if (t0 > t1) std::swap(t0, t1);
        tn = std::max(tn, t0); tf = std::min(tf, t1);
    }
    return tn <= tf ? tn : INFINITY;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 1000000, nrays = argc > 2 ? atoi(argv[2]) : 20000;
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(30.f, 525.f), E(-4.f, 4.f);
    std::vector<BuildPrim> prims(n);
    T.resize(n);
    for (int i = 0; i < n; ++i) {
        float c[3] = {U(rng), U(rng), U(rng)};
        for (int a = 0; a < 3; ++a) { T[i].p0[a] = c[a]; T[i].p1[a] = c[a] + E(rng); T[i].p2[a] = c[a] + E(rng); }
        for (int a = 0; a < 3; ++a) {
            float lo = std::min(T[i].p0[a], std::min(T[i].p1[a], T[i].p2[a]));
            float hi = std::max(T[i].p0[a], std::max(T[i].p1[a], T[i].p2[a]));
            float pad = 1e-4f * std::max(1.0f, std::max(std::fabs(lo), std::fabs(hi)));
            prims[i].lo[a] = lo - pad; prims[i].hi[a] = hi + pad;
        }
        prims[i].ref = (uint32_t)i;
    }
    BvhOut bvh;
    build_bvh(prims, 60, bvh);
    B = &bvh;
    std::mt19937 rr(7);
    std::uniform_real_distribution<float> P(0.f, 555.f), Z(-1.f, 1.f), Ph(0.f, 6.2831853f);
    std::vector<float> ro(3 * nrays), rd(3 * nrays);
    for (int r = 0; r < nrays; ++r) {
        for (int a = 0; a < 3; ++a) ro[3 * r + a] = P(rr);
        const float z = Z(rr), ph = Ph(rr), s = std::sqrt(std::max(0.f, 1.f - z * z));
        rd[3 * r] = s * std::cos(ph); rd[3 * r + 1] = s * std::sin(ph); rd[3 * r + 2] = z;
    }
    for (int width : {2, 4, 8}) {
        W.clear();
        collapse(0, width);
        double visits = 0, tests = 0, boxes = 0, hits = 0;
        for (int r = 0; r < nrays; ++r) {
            const float *o = &ro[3 * r], *d = &rd[3 * r];
            const float inv[3] = {1.f / d[0], 1.f / d[1], 1.f / d[2]};
            float best = 1e30f;
            bool hit = false;
            std::vector<std::pair<float, int>> stack;
            stack.push_back({0.f, 0});
            while (!stack.empty()) {
                auto [tn, nd] = stack.back();
                stack.pop_back();
                if (tn >= best) continue;
                visits += 1;
                std::vector<std::pair<float, int>> in;
                for (const Child &c : W[nd].ch) {
                    boxes += 1;
                    const float t = slab(c, o, inv, best);
                    if (t == INFINITY) continue;
                    if (c.count > 0) {
                        for (int q = 0; q < c.count; ++q) {
                            tests += 1;
                            float th;
                            const uint32_t ref = bvh.refs[~c.code + q] & 0x3fffffffu;
                            if (isect(T[ref], o, d, best, th)) { best = th; hit = true; }
                        }
                    } else in.push_back({t, c.code});
                }
                std::sort(in.begin(), in.end(), [](auto &a, auto &b) { return a.first > b.first; });
                for (auto &e : in) stack.push_back(e); /* nearest on top */
            }
            hits += hit;
        }
        printf("width %d: nodes %zu  node visits/ray %.2f  box tests/ray %.1f  prim tests/ray %.2f  hit %.3f\n", width,
               W.size(), visits / nrays, boxes / nrays, tests / nrays, hits / nrays);
    }
    return 0;
}
