/*
 * pm_bvh_gpu.hip — the scene BVH built on the device. The reference has
 * OptiX build its Sbvh / Bvh acceleration structure on the GPU at the first
 * launch (cudarender.cpp:38-75 declares it, :118-119 launches); the host SAH
 * build this replaces for large scenes took 0.28 s of C3's 0.5 s commit.
 *
 * Algorithm: PLOC (parallel locally-ordered clustering, Meister & Bittner
 * 2018) over the primitive boxes, then the 4-wide collapse and the 64-B
 * quantized node encoding the traversal kernels read. Every step is
 * restated on the host in pm_build.cpp (build_ploc, ploc_to_bvh,
 * collapse_bvh4, bvh4_bfs_order, quantize_bvh4) and the device tree is that
 * host tree bit for bit (tests/test_bvh_gpu.py), so the test oracle is a
 * plain serial program:
 *   1. Morton codes (30 bit) of the box centroids in the centroid bounds,
 *      radix-sorted (rocPRIM, stable: ties stay in primitive order);
 *   2. PLOC rounds over the cluster list: nearest neighbour within `radius`
 *      list positions by union surface area (LDS tile of the block's list
 *      window), mutual pairs merge at the lower position, two exclusive scans
 *      number the new nodes and compact the list;
 *   3. collapse, breadth-first by level: each 4-wide node takes its binary
 *      node's children and opens the largest-area internal child until it
 *      has four; a scan over the level numbers the next level's nodes;
 *   4. each 4-wide node is quantized as it is written (o + q * 2^e, every
 *      decoded box contains the float box), leaves of one triangle coded
 *      LEAF_TRIS with the triangle's storage slot (triangles are stored in
 *      Morton order), other primitives through refs;
 *   5. the stack bound (pushes per descent, pm_build.cpp Collapse::emit) by
 *      a bottom-up pass over the levels; the triangle records (computed on
 *      the host in triangle-id order) are permuted into storage order.
 * Readbacks: two words per PLOC round and one per level (the host sizes the
 * next launch); everything else stays on the device.
 */
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <vector>

#include "pm_build.h"
#include "pm_kernels.h"

#pragma clang fp contract(off)

namespace pm {
namespace {

constexpr int BB = 256;          /* threads per block of every build kernel */
constexpr int PLOC_RMAX = 32;    /* largest neighbour radius (LDS window) */

/* std::min / std::max exactly (the first argument wins ties and NaN) */
__device__ __forceinline__ float hmin(float a, float b) { return b < a ? b : a; }
__device__ __forceinline__ float hmax(float a, float b) { return a < b ? b : a; }

__device__ __forceinline__ uint32_t expand10(uint32_t v) {
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}
__device__ __forceinline__ uint32_t morton_q(float lo, float hi, float flo, float fs) {
    const float u = (0.5f * (lo + hi) - flo) * fs; /* pm_build.cpp ploc_morton */
    return u >= 1023.f ? 1023u : u > 0.f ? (uint32_t)u : 0u;
}

/* boxes: 2 float4 per primitive, (lo.xyz, ref bits) (hi.xyz, 0) */
__global__ __launch_bounds__(BB) void k_ploc_morton(const float4 *box, int n, float3 flo, float3 fs, uint32_t *key,
                                                    uint32_t *val) {
    const int i = blockIdx.x * BB + threadIdx.x;
    if (i >= n) return;
    const float4 a = box[2 * i], b = box[2 * i + 1];
    key[i] = (expand10(morton_q(a.x, b.x, flo.x, fs.x)) << 2) | (expand10(morton_q(a.y, b.y, flo.y, fs.y)) << 1) |
             expand10(morton_q(a.z, b.z, flo.z, fs.z));
    val[i] = (uint32_t)i;
}

/* leaves in Morton order: leaf boxes, the initial cluster list, triangle flags */
__global__ __launch_bounds__(BB) void k_ploc_init(const float4 *box, const uint32_t *order, int n, float4 *leaf,
                                                  float4 *cb, int *cid, uint32_t *istri) {
    const int p = blockIdx.x * BB + threadIdx.x;
    if (p == 0) istri[n] = 0u;
    if (p >= n) return;
    const uint32_t i = order[p];
    const float4 a = box[2 * i], b = box[2 * i + 1];
    leaf[2 * p] = a; leaf[2 * p + 1] = b;
    cb[2 * p] = a; cb[2 * p + 1] = b;
    cid[p] = p;
    istri[p] = (__float_as_uint(a.w) >> 30) == PRIM_TRI ? 1u : 0u;
}

__device__ __forceinline__ float union_area(float4 alo, float4 ahi, float4 blo, float4 bhi) {
    const float dx = hmax(ahi.x, bhi.x) - hmin(alo.x, blo.x);
    const float dy = hmax(ahi.y, bhi.y) - hmin(alo.y, blo.y);
    const float dz = hmax(ahi.z, bhi.z) - hmin(alo.z, blo.z);
    return dx * dy + dy * dz + dz * dx;
}

/* nearest neighbour of every cluster within R positions: smallest union
 * area, the lowest position on ties (candidates scanned in ascending order,
 * strict <) — pm_build.cpp build_ploc */
__global__ __launch_bounds__(BB) void k_ploc_nn(const float4 *cb, int nc, int R, int *nn) {
    __shared__ float4 sb[2 * (BB + 2 * PLOC_RMAX)];
    const int b0 = blockIdx.x * BB, s0 = b0 - R, cnt = BB + 2 * R;
    for (int t = threadIdx.x; t < cnt; t += BB) {
        const int j = s0 + t;
        if (j >= 0 && j < nc) { sb[2 * t] = cb[2 * j]; sb[2 * t + 1] = cb[2 * j + 1]; }
    }
    __syncthreads();
    const int i = b0 + threadIdx.x;
    if (i >= nc) return;
    const int li = i - s0;
    const float4 alo = sb[2 * li], ahi = sb[2 * li + 1];
    const int j0 = max(0, i - R), j1 = min(nc - 1, i + R);
    float best = 0.f;
    int bj = -1;
    for (int j = j0; j <= j1; ++j) {
        if (j == i) continue;
        const int lj = j - s0;
        const float a = union_area(alo, ahi, sb[2 * lj], sb[2 * lj + 1]);
        if (bj < 0 || a < best) { best = a; bj = j; }
    }
    nn[i] = bj;
}

/* m[i]: cluster i merges with its mutual neighbour (i the lower); k[i]: it
 * stays in the list; entry nc = 0 so the scans' last word is the total */
__global__ __launch_bounds__(BB) void k_ploc_flags(const int *nn, int nc, uint32_t *m, uint32_t *k) {
    const int i = blockIdx.x * BB + threadIdx.x;
    if (i > nc) return;
    if (i == nc) { m[i] = 0u; k[i] = 0u; return; }
    const int j = nn[i];
    const bool mutual = nn[j] == i;
    m[i] = mutual && i < j ? 1u : 0u;
    k[i] = mutual && i > j ? 0u : 1u;
}

__global__ __launch_bounds__(BB) void k_ploc_merge(const int *cid, const float4 *cb, const int *nn, const uint32_t *mpos,
                                                   const uint32_t *kpos, int nc, int n, int created, int *oid,
                                                   float4 *ob, int2 *lr, float4 *nb) {
    const int i = blockIdx.x * BB + threadIdx.x;
    if (i >= nc) return;
    const int j = nn[i];
    const bool mutual = nn[j] == i;
    if (mutual && i > j) return;
    const uint32_t o = kpos[i];
    if (mutual) {
        const int k = created + (int)mpos[i];
        const float4 alo = cb[2 * i], ahi = cb[2 * i + 1], blo = cb[2 * j], bhi = cb[2 * j + 1];
        const float4 ulo = make_float4(hmin(alo.x, blo.x), hmin(alo.y, blo.y), hmin(alo.z, blo.z), 0.f);
        const float4 uhi = make_float4(hmax(ahi.x, bhi.x), hmax(ahi.y, bhi.y), hmax(ahi.z, bhi.z), 0.f);
        lr[k] = make_int2(cid[i], cid[j]);
        nb[2 * k] = ulo; nb[2 * k + 1] = uhi;
        oid[o] = n + k;
        ob[2 * o] = ulo; ob[2 * o + 1] = uhi;
    } else {
        oid[o] = cid[i];
        ob[2 * o] = cb[2 * i]; ob[2 * o + 1] = cb[2 * i + 1];
    }
}

struct Tree {
    const float4 *leaf; /* 2 per Morton position */
    const int2 *lr;     /* internal node k = id - n: children */
    const float4 *nb;   /* 2 per internal node */
    int n;
    __device__ __forceinline__ void box(int id, float4 &lo, float4 &hi) const {
        if (id < n) { lo = leaf[2 * id]; hi = leaf[2 * id + 1]; }
        else { lo = nb[2 * (id - n)]; hi = nb[2 * (id - n) + 1]; }
    }
    __device__ __forceinline__ float area(int id) const { /* pm_build.cpp Bin::area */
        float4 lo, hi;
        box(id, lo, hi);
        const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
        return dx < 0 || dy < 0 || dz < 0 ? 0.f : dx * dy + dy * dz + dz * dx;
    }
};

/* the children of a 4-wide node (binary node fr[f]): open the largest-area
 * internal child until there are four (pm_build.cpp Collapse::emit) */
__global__ __launch_bounds__(BB) void k_bvh4_expand(Tree T, const int *fr, int nf, int4 *ch, uint32_t *nint) {
    const int f = blockIdx.x * BB + threadIdx.x;
    if (f > nf) return;
    if (f == nf) { nint[f] = 0u; return; }
    const int id = fr[f];
    const int2 c01 = T.lr[id - T.n];
    int c[4] = {c01.x, c01.y, -1, -1};
    int cnt = 2;
    while (cnt < 4) {
        int best = -1;
        float ba = 0.f;
        for (int i = 0; i < cnt; ++i)
            if (c[i] >= T.n) {
                const float a = T.area(c[i]);
                if (best < 0 || a > ba) { best = i; ba = a; }
            }
        if (best < 0) break;
        const int2 g = T.lr[c[best] - T.n];
        for (int i = best; i < cnt - 1; ++i) c[i] = c[i + 1];
        c[cnt - 1] = g.x;
        c[cnt] = g.y;
        ++cnt;
    }
    uint32_t k = 0;
    for (int i = 0; i < cnt; ++i) k += c[i] >= T.n ? 1u : 0u;
    ch[f] = make_int4(c[0], c[1], c[2], c[3]);
    nint[f] = k;
}

/* the encoder's decode (pm_build.cpp qdecode; traverse4's FMA rounds the same) */
__device__ __forceinline__ float qdecode(float o, uint32_t q, float s) { return o + (float)q * s; }

/* writes 4-wide node level_base + f, quantized (pm_build.cpp quantize_nodes),
 * and the next level's frontier */
__global__ __launch_bounds__(BB) void k_bvh4_emit(Tree T, const int4 *ch, const uint32_t *ipos, int nf, int level_base,
                                                  int next_base, int *fr_next, const uint32_t *tri_slot, uint4 *wn,
                                                  unsigned int *err) {
    const int f = blockIdx.x * BB + threadIdx.x;
    if (f >= nf) return;
    const int4 cc = ch[f];
    const int c[4] = {cc.x, cc.y, cc.z, cc.w};
    int codes[4], counts[4];
    float blo[3][4], bhi[3][4];
    uint32_t r = ipos[f];
    for (int k = 0; k < 4; ++k) {
        blo[0][k] = blo[1][k] = blo[2][k] = INFINITY;
        bhi[0][k] = bhi[1][k] = bhi[2][k] = -INFINITY;
        if (c[k] < 0) { codes[k] = 0; counts[k] = -1; continue; }
        float4 lo, hi;
        T.box(c[k], lo, hi);
        blo[0][k] = lo.x; blo[1][k] = lo.y; blo[2][k] = lo.z;
        bhi[0][k] = hi.x; bhi[1][k] = hi.y; bhi[2][k] = hi.z;
        if (c[k] >= T.n) {
            codes[k] = next_base + (int)r;
            fr_next[r] = c[k];
            ++r;
            counts[k] = 0;
        } else {
            const uint32_t ref = __float_as_uint(lo.w);
            if ((ref >> 30) == PRIM_TRI) { codes[k] = ~(int)tri_slot[c[k]]; counts[k] = 1 | LEAF_TRIS; }
            else { codes[k] = ~c[k]; counts[k] = 1; }
        }
    }
    uint32_t w[16];
    uint32_t ebytes = 0u;
    bool ok = true;
    for (int a = 0; a < 3; ++a) {
        float lo = INFINITY, hi = -INFINITY;
        for (int k = 0; k < 4; ++k)
            if (counts[k] != -1) { lo = hmin(lo, blo[a][k]); hi = hmax(hi, bhi[a][k]); }
        if (!(lo <= hi)) lo = hi = 0.f;
        const double ext = (double)hi - (double)lo;
        int e = -126;
        if (ext > 0.0) {
            int ex = 0;
            (void)frexp(ext / 255.0, &ex);
            e = max(-126, min(127, ex - 1));
            while (e > -126 && ldexp(255.0, e - 1) >= ext) --e;
        }
        while (e < 127 && ldexp(255.0, e) < ext) ++e;
        const double s = ldexp(1.0, e);
        const float sf = ldexpf(1.0f, e);
        w[a] = __float_as_uint(lo);
        ebytes |= (uint32_t)(e + 128) << (8 * a);
        uint32_t ql = 0u, qh = 0u;
        for (int k = 0; k < 4; ++k) {
            uint32_t bl = 0u, bh = 0u;
            if (counts[k] != -1) {
                const float clo = blo[a][k], chi = bhi[a][k];
                const double fl = floor(((double)clo - lo) / s), cl = ceil(((double)chi - lo) / s);
                const double vl = 0.0 < fl ? fl : 0.0, vh = 0.0 < cl ? cl : 0.0; /* std::max(0.0, x) */
                bl = (uint32_t)(vl < 255.0 ? vl : 255.0);
                bh = (uint32_t)(vh < 255.0 ? vh : 255.0);
                while (bl > 0u && qdecode(lo, bl, sf) > clo) --bl;
                while (bh < 255u && qdecode(lo, bh, sf) < chi) ++bh;
                if (qdecode(lo, bl, sf) > clo || qdecode(lo, bh, sf) < chi) ok = false;
            }
            ql |= bl << (8 * k);
            qh |= bh << (8 * k);
        }
        w[4 + a] = ql;
        w[7 + a] = qh;
    }
    w[3] = ebytes;
    w[10] = w[11] = 0u;
    for (int k = 0; k < 4; ++k) {
        w[10 + k / 2] |= (uint32_t)(uint16_t)(int16_t)counts[k] << (16 * (k & 1));
        w[12 + k] = (uint32_t)codes[k];
    }
    if (!ok) atomicOr(err, 1u);
    uint4 *o = wn + 4 * (size_t)(level_base + f);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o[2] = make_uint4(w[8], w[9], w[10], w[11]);
    o[3] = make_uint4(w[12], w[13], w[14], w[15]);
}

/* stack entries a descent from each node of one level needs: all hit
 * internal children but one pushed, plus the deepest child's need */
__global__ __launch_bounds__(BB) void k_bvh4_need(const uint4 *wn, int level_base, int nl, int *need) {
    const int i = blockIdx.x * BB + threadIdx.x;
    if (i >= nl) return;
    const int node = level_base + i;
    const uint4 w2 = wn[4 * (size_t)node + 2], w3 = wn[4 * (size_t)node + 3];
    const int cnt[4] = {(int)(int16_t)(w2.z & 0xffffu), (int)(int16_t)(w2.z >> 16), (int)(int16_t)(w2.w & 0xffffu),
                        (int)(int16_t)(w2.w >> 16)};
    const int code[4] = {(int)w3.x, (int)w3.y, (int)w3.z, (int)w3.w};
    int internal = 0, sub = 0;
    for (int k = 0; k < 4; ++k)
        if (cnt[k] == 0) { ++internal; sub = max(sub, need[code[k]]); }
    need[node] = (internal > 0 ? internal - 1 : 0) + sub;
}

/* storage order of the triangles (Morton order) and the leaf refs */
__global__ __launch_bounds__(BB) void k_tri_order(const float4 *leaf, const uint32_t *tri_slot, int n, uint32_t *refs,
                                                  uint32_t *tri_order) {
    const int p = blockIdx.x * BB + threadIdx.x;
    if (p >= n) return;
    const uint32_t ref = __float_as_uint(leaf[2 * p].w);
    if ((ref >> 30) == PRIM_TRI) {
        const uint32_t s = tri_slot[p];
        tri_order[s] = ref & 0x3fffffffu;
        refs[p] = (PRIM_TRI << 30) | s;
    } else {
        refs[p] = ref;
    }
}

__global__ __launch_bounds__(BB) void k_tri_permute(const uint32_t *tri_order, int64_t nst, const float4 *src_geo,
                                                    const float4 *src_shade, const int4 *src_info, float4 *geo,
                                                    float4 *shade, uint32_t *tid, int4 *info) {
    const int64_t s = (int64_t)blockIdx.x * BB + threadIdx.x;
    if (s >= nst) return;
    const uint32_t t = tri_order[s];
    geo[3 * s] = src_geo[3 * (size_t)t]; geo[3 * s + 1] = src_geo[3 * (size_t)t + 1]; geo[3 * s + 2] = src_geo[3 * (size_t)t + 2];
    shade[2 * s] = src_shade[2 * (size_t)t]; shade[2 * s + 1] = src_shade[2 * (size_t)t + 1];
    info[s] = src_info[t];
    tid[s] = t;
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + BB - 1) / BB); }

} // namespace

hipError_t gpu_bvh_build(const GpuBvhIn &in, GpuBvhOut &out, hipStream_t s) {
    const int n = in.n;
    if (n < 2 || in.radius < 1 || in.radius > PLOC_RMAX) return hipErrorInvalidValue;
    hipError_t e = hipSuccess;
    /* one arena for every temporary */
    const size_t n1 = (size_t)n + 1;
    size_t sort_bytes = 0;
    if ((e = rocprim::radix_sort_pairs(nullptr, sort_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                       (uint32_t *)nullptr, (uint32_t *)nullptr, (size_t)n, 0u, 30u, s)) != hipSuccess)
        return e;
    const size_t sums_words = scan_scratch_words((int64_t)n1);
    struct Part { void **p; size_t bytes; };
    uint32_t *key0, *key1, *val0, *val1, *mflag, *kflag, *mpos, *kpos, *sums, *istri, *tri_slot, *nint, *ipos;
    float4 *leaf, *cb0, *cb1, *nb;
    int *cid0, *cid1, *nn, *fr0, *fr1, *need;
    int2 *lr;
    int4 *ch;
    void *sort_tmp;
    unsigned int *err;
    const Part parts[] = {
        {(void **)&key0, 4 * n1}, {(void **)&key1, 4 * n1}, {(void **)&val0, 4 * n1}, {(void **)&val1, 4 * n1},
        {(void **)&mflag, 4 * n1}, {(void **)&kflag, 4 * n1}, {(void **)&mpos, 4 * n1}, {(void **)&kpos, 4 * n1},
        {(void **)&sums, 4 * sums_words}, {(void **)&istri, 4 * n1}, {(void **)&tri_slot, 4 * n1},
        {(void **)&nint, 4 * n1}, {(void **)&ipos, 4 * n1}, {(void **)&leaf, 32 * (size_t)n},
        {(void **)&cb0, 32 * (size_t)n}, {(void **)&cb1, 32 * (size_t)n}, {(void **)&nb, 32 * (size_t)n},
        {(void **)&cid0, 4 * (size_t)n}, {(void **)&cid1, 4 * (size_t)n}, {(void **)&nn, 4 * (size_t)n},
        {(void **)&fr0, 4 * (size_t)n}, {(void **)&fr1, 4 * (size_t)n}, {(void **)&need, 4 * (size_t)n},
        {(void **)&lr, 8 * (size_t)n}, {(void **)&ch, 16 * (size_t)n}, {&sort_tmp, sort_bytes + 16},
        {(void **)&err, 16}};
    size_t total = 0;
    for (const Part &p : parts) total += (p.bytes + 255) & ~(size_t)255;
    char *arena = nullptr;
    if ((e = hipMalloc(&arena, total)) != hipSuccess) return e;
    uint32_t *h = nullptr; /* readback words */
    if ((e = hipHostMalloc((void **)&h, 64, hipHostMallocDefault)) != hipSuccess) { (void)hipFree(arena); return e; }
    {
        size_t off = 0;
        for (const Part &p : parts) { *p.p = arena + off; off += (p.bytes + 255) & ~(size_t)255; }
    }
    auto done = [&](hipError_t r) {
        (void)hipStreamSynchronize(s);
        (void)hipHostFree(h);
        (void)hipFree(arena);
        return r;
    };
    auto readback = [&](const uint32_t *a, const uint32_t *b) -> hipError_t {
        hipError_t r;
        if ((r = hipMemcpyAsync(h, a, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return r;
        if (b && (r = hipMemcpyAsync(h + 1, b, 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return r;
        return hipStreamSynchronize(s);
    };
    if ((e = hipMemsetAsync(err, 0, 4, s)) != hipSuccess) return done(e);

    /* 1. Morton order */
    pm_launch(k_ploc_morton, dim3(blocks(n)), dim3(BB), 0, s, in.box, n,
              make_float3(in.frame_lo[0], in.frame_lo[1], in.frame_lo[2]),
              make_float3(in.frame_scale[0], in.frame_scale[1], in.frame_scale[2]), key0, val0);
    if ((e = rocprim::radix_sort_pairs(sort_tmp, sort_bytes, key0, key1, val0, val1, (size_t)n, 0u, 30u, s)) != hipSuccess)
        return done(e);
    pm_launch(k_ploc_init, dim3(blocks(n)), dim3(BB), 0, s, in.box, (const uint32_t *)val1, n, leaf, cb0, cid0, istri);

    /* 2. PLOC rounds */
    int nc = n, created = 0, rounds = 0;
    int *cid = cid0, *cido = cid1;
    float4 *cb = cb0, *cbo = cb1;
    while (nc > 1) {
        pm_launch(k_ploc_nn, dim3(blocks(nc)), dim3(BB), 0, s, (const float4 *)cb, nc, in.radius, nn);
        pm_launch(k_ploc_flags, dim3(blocks((int64_t)nc + 1)), dim3(BB), 0, s, (const int *)nn, nc, mflag, kflag);
        if ((e = launch_exclusive_scan(mflag, (int64_t)nc + 1, mpos, sums, s)) != hipSuccess) return done(e);
        if ((e = launch_exclusive_scan(kflag, (int64_t)nc + 1, kpos, sums, s)) != hipSuccess) return done(e);
        pm_launch(k_ploc_merge, dim3(blocks(nc)), dim3(BB), 0, s, (const int *)cid, (const float4 *)cb,
                  (const int *)nn, (const uint32_t *)mpos, (const uint32_t *)kpos, nc, n, created, cido, cbo, lr, nb);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        if ((e = readback(mpos + nc, kpos + nc)) != hipSuccess) return done(e);
        const int merged = (int)h[0], kept = (int)h[1];
        if (merged < 1 || kept != nc - merged || ++rounds > 1 << 16) return done(hipErrorUnknown); /* no progress */
        created += merged;
        nc = kept;
        std::swap(cid, cido);
        std::swap(cb, cbo);
    }
    if (created != n - 1) return done(hipErrorUnknown);

    /* triangle storage slots (Morton order among the triangles), refs */
    if ((e = launch_exclusive_scan(istri, (int64_t)n + 1, tri_slot, sums, s)) != hipSuccess) return done(e);
    pm_launch(k_tri_order, dim3(blocks(n)), dim3(BB), 0, s, (const float4 *)leaf, (const uint32_t *)tri_slot, n,
              out.refs, out.tri_order);

    /* 3./4. collapse by levels, nodes written quantized; the root is the
     * last cluster's node (an internal node: n >= 2) */
    Tree T{leaf, lr, nb, n};
    if ((e = hipMemcpyAsync(fr0, cid, 4, hipMemcpyDeviceToDevice, s)) != hipSuccess) return done(e);
    std::vector<int> level_base, level_count;
    int nf = 1, base = 0;
    int *fr = fr0, *frn = fr1;
    while (nf > 0) {
        if (base + nf > out.max_nodes) return done(hipErrorInvalidValue);
        pm_launch(k_bvh4_expand, dim3(blocks((int64_t)nf + 1)), dim3(BB), 0, s, T, (const int *)fr, nf, ch, nint);
        if ((e = launch_exclusive_scan(nint, (int64_t)nf + 1, ipos, sums, s)) != hipSuccess) return done(e);
        pm_launch(k_bvh4_emit, dim3(blocks(nf)), dim3(BB), 0, s, T, (const int4 *)ch, (const uint32_t *)ipos, nf, base,
                  base + nf, frn, (const uint32_t *)tri_slot, out.wnodes, err);
        if ((e = hipGetLastError()) != hipSuccess) return done(e);
        if ((e = readback(ipos + nf, nullptr)) != hipSuccess) return done(e);
        level_base.push_back(base);
        level_count.push_back(nf);
        base += nf;
        nf = (int)h[0];
        std::swap(fr, frn);
    }
    /* 5. stack bound, deepest level first */
    for (int l = (int)level_base.size() - 1; l >= 0; --l)
        pm_launch(k_bvh4_need, dim3(blocks(level_count[l])), dim3(BB), 0, s, (const uint4 *)out.wnodes, level_base[l],
                  level_count[l], need);
    if ((e = readback((const uint32_t *)need, (const uint32_t *)err)) != hipSuccess) return done(e);
    if (h[1] != 0u) return done(hipErrorUnknown); /* a box the quantized decode would not contain */
    out.nodes = base;
    out.depth = (int)level_base.size();
    out.max_stack = (int)h[0] + 1;
    out.rounds = rounds;
    if ((e = readback(tri_slot + n, nullptr)) != hipSuccess) return done(e);
    out.n_tris = (int64_t)h[0];
    return done(hipGetLastError());
}

hipError_t launch_tri_permute(const uint32_t *tri_order, int64_t nst, const float4 *src_geo, const float4 *src_shade,
                              const int4 *src_info, float4 *geo, float4 *shade, uint32_t *tid, int4 *info,
                              hipStream_t s) {
    if (nst <= 0) return hipSuccess;
    pm_launch(k_tri_permute, dim3(blocks(nst)), dim3(BB), 0, s, tri_order, nst, src_geo, src_shade, src_info, geo, shade,
              tid, info);
    return hipGetLastError();
}

} // namespace pm
