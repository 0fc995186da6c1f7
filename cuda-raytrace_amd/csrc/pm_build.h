/*
 * pm_build.h — host-side acceleration-structure builders.
 *
 *  - build_bvh: binned-SAH binary BVH in the two-children-per-node layout the
 *    traversal kernels read (replaces OptiX's "Sbvh" build triggered at
 *    cudarender.cpp:38-75). Depth is capped so the per-lane LDS stack
 *    (BVH_STACK) can never overflow.
 *  - build_kdtree_pbrt: the canonical pbrt-v2 KdTree median split in the
 *    reference's CudaPhoton node layout (CreatePhotonMap,
 *    photon_mapping/photonmappingrenderer.cpp:150-180). Ties on the split
 *    coordinate break by position in the valid-photon list, so the tree is
 *    unique (implementation-independent).
 */
#pragma once
#include <stdint.h>

#include <functional>
#include <vector>

#include "../../include/pm_api.h"

namespace pm {

struct BuildPrim {
    float lo[3], hi[3];
    uint32_t ref;
};

struct BvhOut {
    std::vector<float> nodes; /* 16 floats per node */
    std::vector<uint32_t> refs;
    int depth = 0;
};

/* SAH cost model: a node visit (two box tests) costs c_trav, a primitive
 * test c_isect; leaves hold at most leaf_max primitives */
struct BvhCost {
    float c_trav = 1.0f, c_isect = 1.0f;
    int leaf_max = 1;
};
void build_bvh(std::vector<BuildPrim> &prims, int max_depth, BvhOut &out, const BvhCost &cost = BvhCost());

/* host threads of the builders (PM_BUILD_THREADS, else OMP_NUM_THREADS, else
 * the hardware's; at most 32) and a parallel loop over [0, n) in contiguous
 * chunks of at least min_per_thread: f(begin, end) */
int host_threads();
void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)> &f, int64_t min_per_thread = 1 << 15);

/* 4-wide BVH collapsed from the binary one (each node takes its binary
 * node's children and opens the largest internal child until it has four):
 * 32 floats = 128 B per node, one L2 line, SoA child boxes
 *   lox[4] loy[4] loz[4] hix[4] hiy[4] hiz[4] child[4] count[4]
 * child >= 0: internal node; child < 0: leaf, refs [~child, ~child + count);
 * count -1: empty slot (box lo = +inf, hi = -inf). Binary subtrees of at
 * most leaf_prims primitives become one leaf (their refs are contiguous).
 * max_stack: entries a traversal stack needs (pushes all hit children but
 * the nearest), so a kernel can size its LDS stack exactly. */
struct Bvh4Out {
    std::vector<float> nodes;
    int depth = 0;
    int max_stack = 0;
};
void collapse_bvh4(const BvhOut &bin, int leaf_prims, Bvh4Out &out);

/* 64-B quantized copy of the 4-wide nodes (16 u32 per node, half the bytes
 * of a node visit): [0..2] node origin o (float: min corner of its
 * children), [3] per-axis step exponents e + 128 (bytes 0..2; step 2^e,
 * 255 steps span the node); [4..9] lox loy loz hix hiy hiz, one byte per
 * child (child k in byte k); [10..11] counts as int16 pairs (children 0|1,
 * 2|3); [12..15] child codes. A bound decodes as o + q * 2^e in float
 * (q * 2^e exact, one rounding in the add); q is floor / ceil of the exact
 * offset, so by monotone rounding every decoded box contains the float box,
 * which is checked here: the culling test only gets more conservative.
 * Returns false if a node cannot be encoded (leaf count > 16383 = 0x3fff: bit 14 is the LEAF_TRIS flag). */
bool quantize_bvh4(const std::vector<float> &nodes, std::vector<uint32_t> &q);
/* With the scene's refs (kind << 30 | storage index): a leaf whose refs
 * are all triangles at consecutive storage slots s0, s0 + 1, ... is coded
 * ~s0 with LEAF_TRIS set in its count, so the traversal tests
 * tri_geo[s0 ..] directly, without loading the refs (one dependent load
 * less per leaf). */
constexpr int LEAF_TRIS = 0x4000;
/* renumbers collapse_bvh4's nodes (depth-first) breadth-first, root 0: the
 * top levels become the first nodes (the LDS nodelets of k_trace_pool) */
void bvh4_bfs_order(std::vector<float> &nodes);
bool quantize_bvh4(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q);
/* 8-wide (round 6): the same collapse with eight children per node, 64
 * floats = lox[8] loy[8] loz[8] hix[8] hiy[8] hiz[8] child[8] count[8] */
void collapse_bvh8(const BvhOut &bin, int leaf_prims, Bvh4Out &out);
/* 128-B quantized 8-wide nodes (32 u32): [0..2] origin, [3] exponent bytes
 * (as quantize_bvh4), [4 + 2a, 5 + 2a] lo bytes of axis a (children 0-3,
 * 4-7), [10 + 2a, 11 + 2a] hi bytes, [16..23] child words: an internal node
 * index >= 0, INT_MIN for an empty slot, else a leaf ~((s << 5) | (tris << 4)
 * | n): n < 16 refs from s, or (tris) n triangles at storage slots s ..
 * (LEAF_TRIS), s < 2^26; [24..31] 0. False if a leaf cannot be coded so. */
bool quantize_bvh8(const std::vector<float> &nodes, const std::vector<uint32_t> &refs, std::vector<uint32_t> &q);

/* PLOC (parallel locally-ordered clustering, Meister & Bittner 2018), the
 * GPU builder's algorithm (pm_bvh_gpu.hip) restated on the host — the
 * device tree's test oracle and the A/B path of PM_BVH_BUILD=ploc-host.
 *  1. primitives sorted by the 30-bit Morton code of their box centroid in
 *     the centroid bounds (ploc_morton: q = (c - lo) * scale per axis, scale =
 *     1024 / extent, clamped to 1023), ties by primitive index;
 *  2. rounds over the cluster list (initially the sorted leaves): every
 *     cluster takes as nearest neighbour the cluster within `radius` list
 *     positions whose union box has the smallest surface area (ties: the
 *     lower position — a strict order on pairs, so the global minimum pair
 *     is always mutual); mutual pairs merge into a new internal node at the
 *     lower position (ids in creation order: n + k, ranked by position
 *     within a round), the higher one leaves, the list keeps its order.
 * Leaf ids are Morton positions p (< n), internal ids n + k; the root is
 * the last node created. */
struct PlocTree {
    std::vector<uint32_t> order;  /* primitive index at Morton position p */
    std::vector<int32_t> left, right;
    std::vector<float> box;       /* internal node k: lo[3] hi[3] */
    int root = -1;                /* node id (-1: no primitives) */
    int rounds = 0;
    float frame_lo[3] = {0, 0, 0}, frame_scale[3] = {0, 0, 0};
};
void ploc_morton_frame(const std::vector<BuildPrim> &prims, float lo[3], float scale[3]);
uint32_t ploc_morton(const BuildPrim &p, const float lo[3], const float scale[3]);
void build_ploc(const std::vector<BuildPrim> &prims, int radius, PlocTree &t);
/* the PLOC tree in build_bvh's layout (breadth-first, root 0, leaves of one
 * primitive at Morton positions, refs in Morton order) */
void ploc_to_bvh(const std::vector<BuildPrim> &prims, const PlocTree &t, BvhOut &out);
/* surface-area cost of a 4-wide tree (pm_build.h node layout): sum over
 * nodes of area(node box) * c_node + over leaves area * prims, / root area */
double bvh4_sah_cost(const std::vector<float> &nodes, double c_node = 1.0, double c_prim = 1.0);

/* returns the number of nodes (= valid photons); nodes sized >= that */
int64_t build_kdtree_pbrt(const pm_photon *slots, int64_t nslots, std::vector<pm_photon> &nodes);

} // namespace pm
