/*
 * pm_build.cpp — host builders (see pm_build.h).
 */
#include "pm_build.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

namespace pm {

namespace {

constexpr int NBINS = 32;

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float *l, const float *h) {
        for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], l[a]); hi[a] = std::max(hi[a], h[a]); }
    }
    void grow(const Box &b) { grow(b.lo, b.hi); }
    float half_area() const {
        float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0.f;
        return dx * dy + dy * dz + dz * dx;
    }
};

inline float centroid(const BuildPrim &p, int a) { return 0.5f * (p.lo[a] + p.hi[a]); }

/* host threads for the builders: this process's CPU share (OMP_NUM_THREADS,
 * 16 per GPU on the MI355X boxes), else the hardware's, at most 32 */
int build_threads() {
    static const int t = [] {
        const char *e = std::getenv("PM_BUILD_THREADS");
        if (!e) e = std::getenv("OMP_NUM_THREADS");
        int n = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(32, n));
    }();
    return t;
}
/* f(chunk, begin, end) over [b, e) in `parts` contiguous chunks, in parallel */
void parallel_chunks(int b, int e, int parts, const std::function<void(int, int, int)> &f) {
    if (parts <= 1) { f(0, b, e); return; }
    std::vector<std::thread> th;
    const int n = e - b;
    for (int k = 0; k < parts; ++k) {
        const int cb = b + (int)((int64_t)n * k / parts), ce = b + (int)((int64_t)n * (k + 1) / parts);
        th.emplace_back(f, k, cb, ce);
    }
    for (auto &t : th) t.join();
}
/* ranges this large bin in parallel (the top levels, where few subtrees
 * run at once); the merge of per-chunk bins is exact (counts, min / max) */
constexpr int PAR_BIN_MIN = 1 << 16;
/* ranges this large build their left subtree in another thread */
constexpr int SUBTREE_TASK_MIN = 1 << 14;

struct BvhBuilder {
    std::vector<BuildPrim> &P;
    std::vector<float> &nodes;
    int max_depth;
    BvhCost cost;
    int depth_seen = 0;
    int threads = 1; /* binning threads for large ranges */

    int alloc() {
        int id = (int)(nodes.size() / 16);
        nodes.resize(nodes.size() + 16, 0.f);
        return id;
    }

    void write_node(int id, const Box &lb, int lcode, int lcount, const Box &rb, int rcode, int rcount) {
        float *n = &nodes[(size_t)id * 16];
        n[0] = lb.lo[0]; n[1] = lb.lo[1]; n[2] = lb.lo[2]; n[3] = lb.hi[0];
        n[4] = lb.hi[1]; n[5] = lb.hi[2]; n[6] = rb.lo[0]; n[7] = rb.lo[1];
        n[8] = rb.lo[2]; n[9] = rb.hi[0]; n[10] = rb.hi[1]; n[11] = rb.hi[2];
        int ints[4] = {lcode, rcode, lcount, rcount};
        std::memcpy(&n[12], ints, sizeof(ints));
    }

    /* binned SAH; returns split position or -1 for "make a leaf" */
    int find_split(int b, int e) {
        int n = e - b;
        const int parts = n >= PAR_BIN_MIN ? std::min(threads, n / (PAR_BIN_MIN / 4)) : 1;
        Box cb, full;
        if (parts == 1) {
            for (int i = b; i < e; ++i) {
                float c[3] = {centroid(P[i], 0), centroid(P[i], 1), centroid(P[i], 2)};
                cb.grow(c, c);
                full.grow(P[i].lo, P[i].hi);
            }
        } else {
            std::vector<Box> pc(parts), pf(parts);
            parallel_chunks(b, e, parts, [&](int k, int cb0, int ce0) {
                for (int i = cb0; i < ce0; ++i) {
                    float c[3] = {centroid(P[i], 0), centroid(P[i], 1), centroid(P[i], 2)};
                    pc[k].grow(c, c);
                    pf[k].grow(P[i].lo, P[i].hi);
                }
            });
            for (int k = 0; k < parts; ++k) { cb.grow(pc[k]); full.grow(pf[k]); }
        }
        float best_cost = INFINITY;
        int best_axis = -1, best_bin = -1;
        /* the three axes' bins in one pass over the range */
        Box bins[3][NBINS];
        int cnt[3][NBINS] = {{0}};
        float k3[3];
        for (int a = 0; a < 3; ++a) { const float ext = cb.hi[a] - cb.lo[a]; k3[a] = ext > 0.f ? NBINS / ext : 0.f; }
        if (parts == 1) {
            for (int a = 0; a < 3; ++a) {
                if (!(k3[a] > 0.f)) continue;
                for (int i = b; i < e; ++i) {
                    int bi = (int)((centroid(P[i], a) - cb.lo[a]) * k3[a]);
                    bi = std::min(NBINS - 1, std::max(0, bi));
                    cnt[a][bi]++;
                    bins[a][bi].grow(P[i].lo, P[i].hi);
                }
            }
        } else {
            struct Part { Box bins[3][NBINS]; int cnt[3][NBINS]; };
            std::vector<Part> pp(parts);
            parallel_chunks(b, e, parts, [&](int k, int cb0, int ce0) {
                Part &q = pp[k];
                std::memset(q.cnt, 0, sizeof(q.cnt));
                for (int a = 0; a < 3; ++a)
                    for (int i2 = 0; i2 < NBINS; ++i2) q.bins[a][i2] = Box();
                for (int i = cb0; i < ce0; ++i)
                    for (int a = 0; a < 3; ++a) {
                        if (!(k3[a] > 0.f)) continue;
                        int bi = (int)((centroid(P[i], a) - cb.lo[a]) * k3[a]);
                        bi = std::min(NBINS - 1, std::max(0, bi));
                        q.cnt[a][bi]++;
                        q.bins[a][bi].grow(P[i].lo, P[i].hi);
                    }
            });
            for (int k = 0; k < parts; ++k)
                for (int a = 0; a < 3; ++a)
                    for (int i2 = 0; i2 < NBINS; ++i2) { cnt[a][i2] += pp[k].cnt[a][i2]; bins[a][i2].grow(pp[k].bins[a][i2]); }
        }
        for (int a = 0; a < 3; ++a) {
            float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.f)) continue;
            float rarea[NBINS];
            int rcnt[NBINS];
            Box acc;
            int c = 0;
            for (int i = NBINS - 1; i > 0; --i) {
                acc.grow(bins[a][i]); c += cnt[a][i];
                rarea[i] = acc.half_area(); rcnt[i] = c;
            }
            Box lacc;
            int lc = 0;
            for (int i = 0; i < NBINS - 1; ++i) {
                lacc.grow(bins[a][i]); lc += cnt[a][i];
                if (lc == 0 || rcnt[i + 1] == 0) continue;
                float cost = lacc.half_area() * lc + rarea[i + 1] * rcnt[i + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = a; best_bin = i; }
            }
        }
        float A = full.half_area();
        if (best_axis < 0) {
            /* all centroids coincide: median split by index */
            return n > cost.leaf_max ? b + n / 2 : -1;
        }
        /* SAH: C_trav + sum_child (A_child / A) N_child C_isect vs a leaf's N C_isect */
        float split_cost = cost.c_trav + (A > 0.f ? best_cost / A : (float)n) * cost.c_isect;
        if (n <= cost.leaf_max && (float)n * cost.c_isect <= split_cost) return -1;
        float ext = cb.hi[best_axis] - cb.lo[best_axis];
        float k = NBINS / ext;
        int a = best_axis;
        auto mid = std::partition(P.begin() + b, P.begin() + e, [&](const BuildPrim &p) {
            int bi = (int)((centroid(p, a) - cb.lo[a]) * k);
            bi = std::min(NBINS - 1, std::max(0, bi));
            return bi <= best_bin;
        });
        int m = (int)(mid - P.begin());
        if (m == b || m == e) {
            m = b + n / 2;
            std::nth_element(P.begin() + b, P.begin() + m, P.begin() + e,
                             [&](const BuildPrim &x, const BuildPrim &y) { return centroid(x, a) < centroid(y, a); });
        }
        return m;
    }

    Box range_box(int b, int e) const {
        const int parts = e - b >= PAR_BIN_MIN ? std::min(threads, (e - b) / (PAR_BIN_MIN / 4)) : 1;
        if (parts == 1) {
            Box box;
            for (int i = b; i < e; ++i) box.grow(P[i].lo, P[i].hi);
            return box;
        }
        std::vector<Box> pb(parts);
        parallel_chunks(b, e, parts, [&](int k, int cb0, int ce0) {
            for (int i = cb0; i < ce0; ++i) pb[k].grow(P[i].lo, P[i].hi);
        });
        Box box;
        for (auto &x : pb) box.grow(x);
        return box;
    }
    void child(int b, int e, int depth, int &code, int &count, Box &box) {
        box = range_box(b, e);
        int split = -1;
        if (e - b > 1 && depth < max_depth) split = find_split(b, e);
        if (split < 0) { code = ~b; count = e - b; return; }
        int id = alloc();
        depth_seen = std::max(depth_seen, depth + 1);
        Box lb, rb;
        int lc, lcnt, rc, rcnt;
        if (threads > 1 && e - b >= SUBTREE_TASK_MIN) {
            /* the left subtree in its own builder and thread, numbered as the
             * serial recursion numbers it: its nodes follow this node, the
             * right subtree's follow them (identical tree and ids) */
            std::vector<float> lnodes;
            BvhBuilder L{P, lnodes, max_depth, cost, 0, std::max(1, threads / 2)};
            std::thread t([&] { L.child(b, split, depth + 1, lc, lcnt, lb); });
            BvhBuilder R{P, rnodes_scratch(), max_depth, cost, 0, std::max(1, threads - threads / 2)};
            R.child(split, e, depth + 1, rc, rcnt, rb);
            t.join();
            const int lbase = (int)(nodes.size() / 16), nl = (int)(lnodes.size() / 16);
            append(lnodes, lbase);
            append(R.nodes, lbase + nl);
            if (lcnt == 0) lc += lbase;
            if (rcnt == 0) rc += lbase + nl;
            depth_seen = std::max({depth_seen, L.depth_seen, R.depth_seen});
            R.nodes.clear();
        } else {
            child(b, split, depth + 1, lc, lcnt, lb);
            child(split, e, depth + 1, rc, rcnt, rb);
        }
        write_node(id, lb, lc, lcnt, rb, rc, rcnt);
        code = id; count = 0;
    }
    /* a subtree's nodes (ids from 0) appended at id base: internal child ids shift */
    void append(const std::vector<float> &sub, int base) {
        const size_t off = nodes.size();
        nodes.insert(nodes.end(), sub.begin(), sub.end());
        for (size_t i = off; i < nodes.size(); i += 16) {
            int ints[4];
            std::memcpy(ints, &nodes[i + 12], sizeof(ints));
            for (int k = 0; k < 2; ++k)
                if (ints[2 + k] == 0) ints[k] += base;
            std::memcpy(&nodes[i + 12], ints, sizeof(ints));
        }
    }
    std::vector<float> own_scratch;
    std::vector<float> &rnodes_scratch() { own_scratch.clear(); return own_scratch; }
};

} // namespace

namespace {
struct Bin { /* a binary-tree child: leaf (start, count) or internal node */
    float lo[3], hi[3];
    int code, count; /* count > 0 leaf with refs [~code, ~code + count); 0 internal */
    float area() const {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx < 0 || dy < 0 || dz < 0 ? 0.f : dx * dy + dy * dz + dz * dx;
    }
};

struct Collapse {
    const BvhOut &bin;
    int leaf_prims;
    std::vector<float> &out;
    std::vector<int> first, total; /* per binary node: first ref, number of prims below */
    int depth = 0;

    Bin child_of(int node, int k) const {
        const float *n = &bin.nodes[(size_t)node * 16];
        Bin b;
        for (int a = 0; a < 3; ++a) { b.lo[a] = n[6 * k + a]; b.hi[a] = n[6 * k + 3 + a]; }
        int ints[4];
        std::memcpy(ints, &n[12], sizeof(ints));
        b.code = ints[k]; b.count = ints[2 + k];
        return b;
    }
    /* prims below a binary child, and its first ref (subtrees are contiguous) */
    void range(const Bin &b, int &f, int &t) const {
        if (b.count > 0) { f = ~b.code; t = b.count; }
        else if (b.count < 0) { f = 0; t = 0; }
        else { f = first[b.code]; t = total[b.code]; }
    }
    void ranges(int node) {
        int f0, t0, f1, t1;
        for (int k = 0; k < 2; ++k) {
            const Bin c = child_of(node, k);
            if (c.count == 0) ranges(c.code);
        }
        range(child_of(node, 0), f0, t0);
        range(child_of(node, 1), f1, t1);
        first[node] = t0 ? (t1 ? std::min(f0, f1) : f0) : f1;
        total[node] = t0 + t1;
    }
    /* a small internal subtree becomes one leaf over its contiguous refs */
    Bin as_leaf(const Bin &b) const {
        if (b.count != 0) return b;
        int f, t;
        range(b, f, t);
        if (t > leaf_prims) return b;
        Bin l = b;
        l.code = ~f; l.count = t;
        return l;
    }
    int width = 4; /* children per node: 4 (collapse_bvh4) or 8 (collapse_bvh8) */
    /* emits the W-wide node of binary node `node` (8 W floats); returns (its index, stack need) */
    int emit(int node, int level, int &need) {
        depth = std::max(depth, level + 1);
        const int W = width, NF = 8 * W;
        std::vector<Bin> ch;
        for (int k = 0; k < 2; ++k) {
            Bin c = child_of(node, k);
            if (c.count >= 0) ch.push_back(as_leaf(c));
        }
        while ((int)ch.size() < W) { /* open the largest internal child */
            int best = -1;
            for (size_t i = 0; i < ch.size(); ++i)
                if (ch[i].count == 0 && (best < 0 || ch[i].area() > ch[best].area())) best = (int)i;
            if (best < 0) break;
            const int inner = ch[best].code;
            ch.erase(ch.begin() + best);
            for (int k = 0; k < 2; ++k) {
                Bin c = child_of(inner, k);
                if (c.count >= 0) ch.push_back(as_leaf(c));
            }
        }
        const int id = (int)(out.size() / NF);
        out.resize(out.size() + NF, 0.f);
        int internal = 0, sub = 0;
        int codes[8], counts[8];
        float box[6][8];
        for (int k = 0; k < W; ++k) {
            if (k < (int)ch.size()) {
                for (int a = 0; a < 3; ++a) { box[a][k] = ch[k].lo[a]; box[3 + a][k] = ch[k].hi[a]; }
                codes[k] = ch[k].code; counts[k] = ch[k].count;
            } else {
                for (int a = 0; a < 3; ++a) { box[a][k] = INFINITY; box[3 + a][k] = -INFINITY; }
                codes[k] = 0; counts[k] = -1;
            }
        }
        for (int k = 0; k < (int)ch.size(); ++k)
            if (counts[k] == 0) {
                int cn = 0;
                codes[k] = emit(codes[k], level + 1, cn);
                ++internal;
                sub = std::max(sub, cn);
            }
        float *n = &out[(size_t)id * NF];
        for (int r = 0; r < 6; ++r)
            for (int k = 0; k < W; ++k) n[W * r + k] = box[r][k];
        std::memcpy(&n[6 * W], codes, W * sizeof(int));
        std::memcpy(&n[7 * W], counts, W * sizeof(int));
        /* entering this node pushes all hit internal children but one */
        need = (internal > 0 ? internal - 1 : 0) + sub;
        return id;
    }
};
} // namespace

static void collapse_bvhw(const BvhOut &bin, int leaf_prims, int width, Bvh4Out &out) {
    out.nodes.clear();
    const size_t nn = bin.nodes.size() / 16;
    Collapse C{bin, std::max(1, leaf_prims), out.nodes, std::vector<int>(nn, 0), std::vector<int>(nn, 0)};
    C.width = width;
    C.ranges(0);
    int need = 0;
    C.emit(0, 0, need);
    out.depth = C.depth;
    out.max_stack = need + 1;
}
void collapse_bvh4(const BvhOut &bin, int leaf_prims, Bvh4Out &out) { collapse_bvhw(bin, leaf_prims, 4, out); }
void collapse_bvh8(const BvhOut &bin, int leaf_prims, Bvh4Out &out) { collapse_bvhw(bin, leaf_prims, 8, out); }

void bvh4_bfs_order(std::vector<float> &nodes) {
    const size_t nn = nodes.size() / 32;
    if (nn == 0) return;
    std::vector<int> order, newid(nn, -1);
    order.reserve(nn);
    order.push_back(0);
    newid[0] = 0;
    for (size_t h = 0; h < order.size(); ++h) {
        const float *n = &nodes[(size_t)order[h] * 32];
        int codes[4], counts[4];
        std::memcpy(codes, &n[24], sizeof(codes));
        std::memcpy(counts, &n[28], sizeof(counts));
        for (int k = 0; k < 4; ++k)
            if (counts[k] == 0 && newid[codes[k]] < 0) { newid[codes[k]] = (int)order.size(); order.push_back(codes[k]); }
    }
    std::vector<float> out(order.size() * 32);
    for (size_t i = 0; i < order.size(); ++i) {
        float *n = &out[i * 32];
        std::memcpy(n, &nodes[(size_t)order[i] * 32], 32 * sizeof(float));
        int codes[4], counts[4];
        std::memcpy(codes, &n[24], sizeof(codes));
        std::memcpy(counts, &n[28], sizeof(counts));
        for (int k = 0; k < 4; ++k)
            if (counts[k] == 0) codes[k] = newid[codes[k]];
        std::memcpy(&n[24], codes, sizeof(codes));
    }
    nodes.swap(out);
}

/* the device's decode of a quantized bound (traverse4 / trav_step): o + q * 2^e,
 * the power of two s = 2^e passed exactly */
static float qdecode(float o, uint32_t q, float s) { return o + (float)q * s; }

static bool quantize_nodes(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q,
                           int i0, int i1);
bool quantize_bvh4(const std::vector<float> &nodes, std::vector<uint32_t> &q) {
    return quantize_bvh4(nodes, std::vector<uint32_t>(), q);
}

bool quantize_bvh4(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q) {
    const size_t nn = nodes.size() / 32;
    q.assign(nn * 16, 0u);
    std::atomic<bool> ok{true};
    /* nodes encode independently: chunks of nodes in parallel */
    const int parts = nn >= 4096 ? build_threads() : 1;
    parallel_chunks(0, (int)nn, parts, [&](int, int i0, int i1) { if (!quantize_nodes(nodes, refs, q, i0, i1)) ok = false; });
    return ok;
}

static bool quantize_nodes(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q,
                           int i0, int i1) {
    for (size_t i = (size_t)i0; i < (size_t)i1; ++i) {
        const float *n = &nodes[i * 32];
        int codes[4], counts[4];
        std::memcpy(codes, &n[24], sizeof(codes));
        std::memcpy(counts, &n[28], sizeof(counts));
        uint32_t *w = &q[i * 16];
        uint32_t ebytes = 0;
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int k = 0; k < 4; ++k)
                if (counts[k] != -1) { lo = std::min(lo, n[4 * a + k]); hi = std::max(hi, n[4 * (3 + a) + k]); }
            if (!(lo <= hi)) lo = hi = 0.f; /* no children (empty scene root) */
            const double ext = (double)hi - (double)lo;
            /* the smallest e >= -126 with 255 * 2^e >= ext (a linear search
             * from -126 cost ~400 ldexp calls per node) */
            int e = -126;
            if (ext > 0.0) {
                int ex = 0;
                (void)std::frexp(ext / 255.0, &ex);
                e = std::max(-126, std::min(127, ex - 1));
                while (e > -126 && std::ldexp(255.0, e - 1) >= ext) --e;
            }
            while (e < 127 && std::ldexp(255.0, e) < ext) ++e;
            const double s = std::ldexp(1.0, e);
            const float sf = std::ldexp(1.0f, e);
            std::memcpy(&w[a], &lo, 4);
            ebytes |= (uint32_t)(e + 128) << (8 * a);
            uint32_t ql = 0, qh = 0;
            for (int k = 0; k < 4; ++k) {
                uint32_t bl = 0, bh = 0;
                if (counts[k] != -1) {
                    const float clo = n[4 * a + k], chi = n[4 * (3 + a) + k];
                    bl = (uint32_t)std::min(255.0, std::max(0.0, std::floor(((double)clo - lo) / s)));
                    bh = (uint32_t)std::min(255.0, std::max(0.0, std::ceil(((double)chi - lo) / s)));
                    while (bl > 0 && qdecode(lo, bl, sf) > clo) --bl;
                    while (bh < 255 && qdecode(lo, bh, sf) < chi) ++bh;
                    if (qdecode(lo, bl, sf) > clo || qdecode(lo, bh, sf) < chi) return false;
                }
                ql |= bl << (8 * k);
                qh |= bh << (8 * k);
            }
            w[4 + a] = ql;
            w[7 + a] = qh;
        }
        w[3] = ebytes;
        for (int k = 0; k < 4; ++k) {
            if (counts[k] >= LEAF_TRIS) return false;
            if (counts[k] > 0 && !refs.empty()) { /* triangles-only leaf at consecutive slots? */
                const uint32_t f = (uint32_t)~codes[k], s0 = refs[f] & 0x3fffffffu;
                bool tris = true;
                for (int j = 0; j < counts[k] && tris; ++j)
                    tris = (refs[f + j] >> 30) == 0u && (refs[f + j] & 0x3fffffffu) == s0 + (uint32_t)j;
                if (tris) { codes[k] = ~(int)s0; counts[k] |= LEAF_TRIS; }
            }
            w[10 + k / 2] |= (uint32_t)(uint16_t)(int16_t)counts[k] << (16 * (k & 1));
        }
        std::memcpy(&w[12], codes, sizeof(codes));
    }
    return true;
}

/* 8-wide nodes (collapse_bvh8, 64 floats) -> 32 u32 (pm_build.h quantize_bvh8) */
static bool quantize_nodes8(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q,
                            int i0, int i1) {
    for (size_t i = (size_t)i0; i < (size_t)i1; ++i) {
        const float *n = &nodes[i * 64];
        int codes[8], counts[8];
        std::memcpy(codes, &n[48], sizeof(codes));
        std::memcpy(counts, &n[56], sizeof(counts));
        uint32_t *w = &q[i * 32];
        uint32_t ebytes = 0;
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (int k = 0; k < 8; ++k)
                if (counts[k] != -1) { lo = std::min(lo, n[8 * a + k]); hi = std::max(hi, n[8 * (3 + a) + k]); }
            if (!(lo <= hi)) lo = hi = 0.f;
            const double ext = (double)hi - (double)lo;
            int e = -126;
            if (ext > 0.0) {
                int ex = 0;
                (void)std::frexp(ext / 255.0, &ex);
                e = std::max(-126, std::min(127, ex - 1));
                while (e > -126 && std::ldexp(255.0, e - 1) >= ext) --e;
            }
            while (e < 127 && std::ldexp(255.0, e) < ext) ++e;
            const double s = std::ldexp(1.0, e);
            const float sf = std::ldexp(1.0f, e);
            std::memcpy(&w[a], &lo, 4);
            ebytes |= (uint32_t)(e + 128) << (8 * a);
            uint32_t ql[2] = {0, 0}, qh[2] = {0, 0};
            for (int k = 0; k < 8; ++k) {
                uint32_t bl = 0, bh = 0;
                if (counts[k] != -1) {
                    const float clo = n[8 * a + k], chi = n[8 * (3 + a) + k];
                    bl = (uint32_t)std::min(255.0, std::max(0.0, std::floor(((double)clo - lo) / s)));
                    bh = (uint32_t)std::min(255.0, std::max(0.0, std::ceil(((double)chi - lo) / s)));
                    while (bl > 0 && qdecode(lo, bl, sf) > clo) --bl;
                    while (bh < 255 && qdecode(lo, bh, sf) < chi) ++bh;
                    if (qdecode(lo, bl, sf) > clo || qdecode(lo, bh, sf) < chi) return false;
                }
                ql[k / 4] |= bl << (8 * (k & 3));
                qh[k / 4] |= bh << (8 * (k & 3));
            }
            w[4 + 2 * a] = ql[0]; w[5 + 2 * a] = ql[1];
            w[10 + 2 * a] = qh[0]; w[11 + 2 * a] = qh[1];
        }
        w[3] = ebytes;
        for (int k = 0; k < 8; ++k) {
            int32_t word;
            if (counts[k] == 0) word = codes[k];                   /* internal node */
            else if (counts[k] < 0) word = (int32_t)0x80000000;    /* empty slot (its box never hits) */
            else {
                if (counts[k] >= 16) return false;
                uint32_t f = (uint32_t)~codes[k], tris = 0;
                if (!refs.empty()) { /* a triangle run at consecutive storage slots? */
                    const uint32_t s0 = refs[f] & 0x3fffffffu;
                    bool t = true;
                    for (int j = 0; j < counts[k] && t; ++j)
                        t = (refs[f + j] >> 30) == 0u && (refs[f + j] & 0x3fffffffu) == s0 + (uint32_t)j;
                    if (t) { f = s0; tris = 1; }
                }
                if (f >= (1u << 26)) return false;
                word = ~(int32_t)((f << 5) | (tris << 4) | (uint32_t)counts[k]);
            }
            w[16 + k] = (uint32_t)word;
        }
    }
    return true;
}

bool quantize_bvh8(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q) {
    const size_t nn = nodes.size() / 64;
    q.assign(nn * 32, 0u);
    std::atomic<bool> ok{true};
    const int parts = nn >= 4096 ? build_threads() : 1;
    parallel_chunks(0, (int)nn, parts, [&](int, int i0, int i1) { if (!quantize_nodes8(nodes, refs, q, i0, i1)) ok = false; });
    return ok;
}

int host_threads() { return build_threads(); }
void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)> &f, int64_t min_per_thread) {
    const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(build_threads(), n / std::max<int64_t>(1, min_per_thread)));
    if (parts <= 1) { f(0, n); return; }
    std::vector<std::thread> th;
    for (int k = 0; k < parts; ++k) th.emplace_back(f, n * k / parts, n * (k + 1) / parts);
    for (auto &t : th) t.join();
}

void build_bvh(std::vector<BuildPrim> &prims, int max_depth, BvhOut &out, const BvhCost &cost) {
    out.nodes.clear();
    out.refs.clear();
    BvhBuilder B{prims, out.nodes, max_depth, cost, 0, (int)prims.size() >= SUBTREE_TASK_MIN ? build_threads() : 1};
    int n = (int)prims.size();
    Box empty;
    if (n == 0) {
        int id = B.alloc();
        B.write_node(id, empty, ~0, -1, empty, ~0, -1);
    } else {
        int root = B.alloc();
        int split = n > 1 ? B.find_split(0, n) : -1;
        if (split < 0) {
            Box all;
            for (auto &p : prims) all.grow(p.lo, p.hi);
            B.write_node(root, all, ~0, n, empty, ~0, -1);
        } else {
            Box lb, rb;
            int lc, lcnt, rc, rcnt;
            B.child(0, split, 1, lc, lcnt, lb);
            B.child(split, n, 1, rc, rcnt, rb);
            B.write_node(root, lb, lc, lcnt, rb, rc, rcnt);
        }
    }
    out.depth = B.depth_seen + 1;
    /* renumber nodes breadth-first: the first K nodes are then the top levels
     * of the tree, which the traversal kernels stage in LDS */
    {
        const size_t nn = out.nodes.size() / 16;
        std::vector<int> order, newidx(nn, -1);
        order.reserve(nn);
        order.push_back(0);
        newidx[0] = 0;
        for (size_t h = 0; h < order.size(); ++h) {
            const float *nd = &out.nodes[(size_t)order[h] * 16];
            int ints[4];
            std::memcpy(ints, &nd[12], sizeof(ints));
            for (int k = 0; k < 2; ++k)
                if (ints[2 + k] == 0 && ints[k] >= 0) { /* internal child */
                    newidx[ints[k]] = (int)order.size();
                    order.push_back(ints[k]);
                }
        }
        std::vector<float> bfs(order.size() * 16);
        for (size_t i = 0; i < order.size(); ++i) {
            std::memcpy(&bfs[i * 16], &out.nodes[(size_t)order[i] * 16], 16 * sizeof(float));
            int ints[4];
            std::memcpy(ints, &bfs[i * 16 + 12], sizeof(ints));
            for (int k = 0; k < 2; ++k)
                if (ints[2 + k] == 0 && ints[k] >= 0) ints[k] = newidx[ints[k]];
            std::memcpy(&bfs[i * 16 + 12], ints, sizeof(ints));
        }
        out.nodes.swap(bfs);
    }
    out.refs.resize(prims.size());
    for (size_t i = 0; i < prims.size(); ++i) out.refs[i] = prims[i].ref;
}

/* ------------------------------------------------------------------ PLOC */
void ploc_morton_frame(const std::vector<BuildPrim> &prims, float lo[3], float scale[3]) {
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int a = 0; a < 3; ++a) lo[a] = INFINITY;
    for (const BuildPrim &p : prims)
        for (int a = 0; a < 3; ++a) {
            const float c = centroid(p, a);
            lo[a] = std::min(lo[a], c); hi[a] = std::max(hi[a], c);
        }
    for (int a = 0; a < 3; ++a) {
        if (!(lo[a] <= hi[a])) lo[a] = hi[a] = 0.f;
        const float ext = hi[a] - lo[a];
        scale[a] = ext > 0.f ? 1024.f / ext : 0.f;
    }
}
static inline uint32_t expand10(uint32_t v) { /* 10 bits -> every third bit */
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
uint32_t ploc_morton(const BuildPrim &p, const float lo[3], const float scale[3]) {
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        const float u = (centroid(p, a) - lo[a]) * scale[a];
        q[a] = u >= 1023.f ? 1023u : u > 0.f ? (uint32_t)u : 0u;
    }
    return (expand10(q[0]) << 2) | (expand10(q[1]) << 1) | expand10(q[2]);
}

namespace {
struct PBox { float lo[3], hi[3]; };
inline float union_area(const PBox &a, const PBox &b) {
    const float dx = std::max(a.hi[0], b.hi[0]) - std::min(a.lo[0], b.lo[0]);
    const float dy = std::max(a.hi[1], b.hi[1]) - std::min(a.lo[1], b.lo[1]);
    const float dz = std::max(a.hi[2], b.hi[2]) - std::min(a.lo[2], b.lo[2]);
    return dx * dy + dy * dz + dz * dx;
}
} // namespace

void build_ploc(const std::vector<BuildPrim> &prims, int radius, PlocTree &t) {
    const int n = (int)prims.size();
    t = PlocTree();
    if (n == 0) return;
    radius = std::max(1, radius);
    ploc_morton_frame(prims, t.frame_lo, t.frame_scale);
    std::vector<uint64_t> keys((size_t)n);
    parallel_for(n, [&](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i)
            keys[i] = ((uint64_t)ploc_morton(prims[i], t.frame_lo, t.frame_scale) << 32) | (uint64_t)i;
    });
    std::sort(keys.begin(), keys.end());
    t.order.resize((size_t)n);
    for (int i = 0; i < n; ++i) t.order[i] = (uint32_t)(keys[i] & 0xffffffffu);
    t.left.resize((size_t)std::max(0, n - 1));
    t.right.resize((size_t)std::max(0, n - 1));
    t.box.resize((size_t)std::max(0, n - 1) * 6);
    std::vector<int> id((size_t)n), nid((size_t)n), nn((size_t)n);
    std::vector<PBox> box((size_t)n), nbox((size_t)n);
    for (int i = 0; i < n; ++i) {
        const BuildPrim &p = prims[t.order[i]];
        id[i] = i;
        for (int a = 0; a < 3; ++a) { box[i].lo[a] = p.lo[a]; box[i].hi[a] = p.hi[a]; }
    }
    int nc = n, created = 0;
    while (nc > 1) {
        parallel_for(nc, [&](int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {
                const int j0 = (int)std::max<int64_t>(0, i - radius), j1 = (int)std::min<int64_t>(nc - 1, i + radius);
                float best = INFINITY;
                int bj = -1;
                for (int j = j0; j <= j1; ++j) {
                    if (j == i) continue;
                    const float a = union_area(box[i], box[j]);
                    if (bj < 0 || a < best) { best = a; bj = j; }
                }
                nn[i] = bj;
            }
        }, 1 << 12);
        int m = 0;
        for (int i = 0; i < nc; ++i) {
            const int j = nn[i];
            const bool mutual = nn[j] == i;
            if (mutual && i > j) continue; /* merged into cluster j */
            if (mutual) {
                const int k = created++;
                t.left[k] = id[i]; t.right[k] = id[j];
                PBox u;
                for (int a = 0; a < 3; ++a) {
                    u.lo[a] = std::min(box[i].lo[a], box[j].lo[a]);
                    u.hi[a] = std::max(box[i].hi[a], box[j].hi[a]);
                }
                std::memcpy(&t.box[(size_t)k * 6], &u, sizeof(u));
                nid[m] = n + k; nbox[m] = u;
            } else {
                nid[m] = id[i]; nbox[m] = box[i];
            }
            ++m;
        }
        id.swap(nid);
        box.swap(nbox);
        nc = m;
        ++t.rounds;
    }
    t.root = id[0];
}

void ploc_to_bvh(const std::vector<BuildPrim> &prims, const PlocTree &t, BvhOut &out) {
    out.nodes.clear();
    out.refs.clear();
    const int n = (int)prims.size();
    Box empty;
    auto leaf_box = [&](int p) {
        Box b;
        b.grow(prims[t.order[p]].lo, prims[t.order[p]].hi);
        return b;
    };
    auto node_box = [&](int id) {
        if (id < n) return leaf_box(id);
        Box b;
        b.grow(&t.box[(size_t)(id - n) * 6], &t.box[(size_t)(id - n) * 6 + 3]);
        return b;
    };
    auto write = [&](int at, const Box &lb, int lc, int lcnt, const Box &rb, int rc, int rcnt) {
        float *nd = &out.nodes[(size_t)at * 16];
        for (int a = 0; a < 3; ++a) { nd[a] = lb.lo[a]; nd[3 + a] = lb.hi[a]; nd[6 + a] = rb.lo[a]; nd[9 + a] = rb.hi[a]; }
        int ints[4] = {lc, rc, lcnt, rcnt};
        std::memcpy(&nd[12], ints, sizeof(ints));
    };
    if (n <= 1) {
        out.nodes.assign(16, 0.f);
        if (n == 0) write(0, empty, ~0, -1, empty, ~0, -1);
        else write(0, leaf_box(0), ~0, 1, empty, ~0, -1);
        out.depth = 1;
    } else {
        /* breadth-first over the internal nodes from the root */
        std::vector<int> q;
        q.reserve((size_t)n - 1);
        q.push_back(t.root);
        std::vector<int> level(1, 0);
        out.nodes.assign((size_t)(n - 1) * 16, 0.f);
        int depth = 0;
        for (size_t h = 0; h < q.size(); ++h) {
            const int k = q[h] - n, lv = level[h];
            depth = std::max(depth, lv + 1);
            const int ch[2] = {t.left[k], t.right[k]};
            int code[2], cnt[2];
            for (int s = 0; s < 2; ++s) {
                if (ch[s] < n) { code[s] = ~ch[s]; cnt[s] = 1; }
                else { code[s] = (int)q.size(); cnt[s] = 0; q.push_back(ch[s]); level.push_back(lv + 1); }
            }
            write((int)h, node_box(ch[0]), code[0], cnt[0], node_box(ch[1]), code[1], cnt[1]);
        }
        out.depth = depth;
    }
    out.refs.resize((size_t)n);
    for (int p = 0; p < n; ++p) out.refs[p] = prims[t.order[p]].ref;
}

double bvh4_sah_cost(const std::vector<float> &nodes, double c_node, double c_prim) {
    const size_t nn = nodes.size() / 32;
    if (nn == 0) return 0.0;
    auto area = [](double dx, double dy, double dz) { return dx < 0 || dy < 0 || dz < 0 ? 0.0 : dx * dy + dy * dz + dz * dx; };
    double root = 0.0, total = 0.0;
    {
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = 0; k < 4; ++k) {
            int cnt;
            std::memcpy(&cnt, &nodes[28 + k], 4);
            if (cnt == -1) continue;
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], (double)nodes[4 * a + k]); hi[a] = std::max(hi[a], (double)nodes[4 * (3 + a) + k]); }
        }
        root = area(hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]);
    }
    if (root <= 0.0) return 0.0;
    total = c_node * root;
    for (size_t i = 0; i < nn; ++i) {
        const float *nd = &nodes[i * 32];
        for (int k = 0; k < 4; ++k) {
            int cnt;
            std::memcpy(&cnt, &nd[28 + k], 4);
            if (cnt == -1) continue;
            const double a = area((double)nd[12 + k] - nd[k], (double)nd[16 + k] - nd[4 + k], (double)nd[20 + k] - nd[8 + k]);
            total += cnt == 0 ? c_node * a : c_prim * a * cnt;
        }
    }
    return total / root;
}

int64_t build_kdtree_pbrt(const pm_photon *slots, int64_t nslots, std::vector<pm_photon> &nodes) {
    std::vector<pm_photon> ph;
    ph.reserve((size_t)nslots);
    for (int64_t i = 0; i < nslots; ++i)
        if (slots[i].bits & 1u) ph.push_back(slots[i]);
    const int64_t m = (int64_t)ph.size();
    nodes.resize((size_t)m);
    if (m == 0) return 0;
    std::vector<uint32_t> idx((size_t)m);
    for (int64_t i = 0; i < m; ++i) idx[i] = (uint32_t)i;

    struct Task { int64_t start, end; int64_t parent; int kind; uint32_t node; };
    std::vector<Task> st;
    st.push_back(Task{0, m, -1, 0, 0});
    uint32_t next_free = 1;
    while (!st.empty()) {
        Task t = st.back();
        st.pop_back();
        uint32_t node = t.node;
        if (t.kind == 2) { /* right child: numbered once its left sibling's subtree is done */
            node = next_free++;
            pm_photon &par = nodes[(size_t)t.parent];
            par.bits = (par.bits & 7u) | (node << 3);
        }
        if (t.start + 1 == t.end) {
            nodes[node] = ph[idx[(size_t)t.start]];
            nodes[node].bits = (3u << 1) | (PM_PHOTON_MAX_RIGHT_CHILD << 3);
            continue;
        }
        float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int64_t i = t.start; i < t.end; ++i) {
            const float *p = ph[idx[(size_t)i]].p;
            for (int a = 0; a < 3; ++a) { mn[a] = std::min(mn[a], p[a]); mx[a] = std::max(mx[a], p[a]); }
        }
        float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        int axis = (dx > dy && dx > dz) ? 0 : (dy > dz ? 1 : 2);
        int64_t mid = (t.start + t.end) / 2;
        std::nth_element(idx.begin() + t.start, idx.begin() + mid, idx.begin() + t.end,
                         [&](uint32_t a, uint32_t b) {
                             float pa = ph[a].p[axis], pb = ph[b].p[axis];
                             return pa == pb ? a < b : pa < pb;
                         });
        nodes[node] = ph[idx[(size_t)mid]];
        uint32_t bits = ((uint32_t)axis << 1) | (PM_PHOTON_MAX_RIGHT_CHILD << 3);
        bool has_left = t.start < mid, has_right = mid + 1 < t.end;
        if (has_left) bits |= 1u;
        nodes[node].bits = bits;
        if (has_right) st.push_back(Task{mid + 1, t.end, (int64_t)node, 2, 0});
        if (has_left) st.push_back(Task{t.start, mid, (int64_t)node, 1, next_free++});
    }
    return m;
}

} // namespace pm
