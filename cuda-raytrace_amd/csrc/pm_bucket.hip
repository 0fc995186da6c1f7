/*
 * pm_bucket.hip — photon-map build on the GPU (replaces CreatePhotonMap,
 * photon_mapping/photonmappingrenderer.cpp:150-180, which copies the slots to
 * the host and builds a pbrt KdTree there).
 *
 * Photon buckets = a dense uniform grid over the scene box, cell edge
 * >= 2 r_max, photons stored cell-contiguously:
 *   1. k_bucket_count  cell key of each valid slot; rank = returning atomicAdd
 *                      on that cell's counter (atomics spread over ~10^5
 *                      cells; there is no single hot word). Skipped when the
 *                      trace kernel already counted its deposits (fused
 *                      counting, pm_trace.hip: the atomics then overlap the
 *                      latency-bound trace instead of costing a pass).
 *   2. exclusive scan  of the ncells+1 counters (tile sums, then per tile:
 *                      prefix of the earlier tile sums + local scan; 16-B
 *                      vector loads) -> cell_start; cell_start[ncells] =
 *                      number of valid photons. The counters are zeroed as
 *                      they are read, so the next pass needs no memset.
 *   3. k_bucket_fill   slot -> cell_start[key] + rank, written straight into
 *                      the arrays the gather reads: ph_a (position, wi.x;
 *                      16 B, streamed by every range test) and ph_b (alpha,
 *                      wi.y | wi.z, pad: one 32-B sector, read only for
 *                      photons inside the radius)
 * The order inside a bucket depends on atomic arrival order. Results do not:
 * the bucket gather (pm_gather.hip) sums flux in exact 64-bit fixed point
 * and counts photons as integers, so any order gives identical bits.
 */
#include <hip/hip_runtime.h>

#include "pm_kernels.h"

#pragma clang fp contract(off)

namespace pm {

/* 2048 counters per block: at C2's 2.7 M cells, 1,320 blocks instead of 660
 * with 16 per thread (build 37.2 -> 34.3 us: the scan kernels were short of
 * waves to hide their latency); 4 per thread measured the same */
#ifndef PM_SCAN_ITEMS
#define PM_SCAN_ITEMS 8
#endif
constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = PM_SCAN_ITEMS, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__global__ __launch_bounds__(256) void k_bucket_count(const pm_photon *slots, int64_t n, GridDesc g,
                                                      uint32_t *count, uint32_t *key_out, uint32_t *rank_out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float2 *q = reinterpret_cast<const float2 *>(slots + i);
    const float2 a = q[0], b = q[1];
    uint32_t key = 0xffffffffu, rank = 0u;
    if ((uint32_t)__float_as_int(a.x) & 1u) {
        const uint32_t cx = cell_axis(a.y, g.gx, g.inv_cs, g.dx);
        const uint32_t cy = cell_axis(b.x, g.gy, g.inv_cs, g.dy);
        const uint32_t cz = cell_axis(b.y, g.gz, g.inv_cs, g.dz);
        key = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx + cx;
        rank = atomicAdd(&count[key], 1u);
    }
    key_out[i] = key;
    rank_out[i] = rank;
}

PMD uint32_t wave_incl_scan(uint32_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t t = __shfl_up(v, off);
        if (lane >= off) v += t;
    }
    return v;
}

/* block-wide exclusive scan of one value per thread; returns the block total */
PMD uint32_t block_excl_scan(uint32_t v, uint32_t *excl, uint32_t *lds /* >= 4 */) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    uint32_t off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_BLOCK / 64; ++w) {
        uint32_t s = lds[w];
        if (w < wave) off += s;
        tot += s;
    }
    __syncthreads();
    *excl = off + inc - v;
    return tot;
}

/* per-tile sums; thread t owns SCAN_ITEMS contiguous words (16-B loads) */
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_reduce(const uint32_t *in, int64_t n, uint32_t *sums) {
    __shared__ uint32_t lds[4];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t s = 0;
    if (base + SCAN_ITEMS <= n) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS / 4; ++k) { uint4 v = p[k]; s += v.x + v.y + v.z + v.w; }
    } else {
        for (int64_t k = base; k < n; ++k) s += in[k];
    }
    uint32_t excl;
    uint32_t tot = block_excl_scan(s, &excl, lds);
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

/* clear != nullptr: the tile of `in` is zeroed after it is read (the bucket
 * counters then start the next pass at zero without a memset launch) */
__global__ __launch_bounds__(SCAN_BLOCK) void k_scan_down(const uint32_t *in, int64_t n, const uint32_t *sums,
                                                          uint32_t *out, uint32_t *clear) {
    __shared__ uint32_t lds[4];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE + (int64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    const bool full = base + SCAN_ITEMS <= n;
    if (full) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + base);
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS / 4; ++k) {
            uint4 q = p[k];
            v[4 * k] = q.x; v[4 * k + 1] = q.y; v[4 * k + 2] = q.z; v[4 * k + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k) v[k] = (base + k < n) ? in[base + k] : 0u;
    }
    if (clear) {
        if (full) {
            /* only the 16-B groups that counted something (most cells of a
             * pass's grid stay empty: C2 552 K photons in 2.7 M cells) */
            uint4 *p = reinterpret_cast<uint4 *>(clear + base);
#pragma unroll
            for (int k = 0; k < SCAN_ITEMS / 4; ++k)
                if ((v[4 * k] | v[4 * k + 1] | v[4 * k + 2] | v[4 * k + 3]) != 0u) p[k] = make_uint4(0u, 0u, 0u, 0u);
        } else {
            for (int64_t k = base; k < n; ++k) clear[k] = 0u;
        }
    }
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) s += v[k];
    uint32_t excl;
    block_excl_scan(s, &excl, lds);
    /* this tile's offset: the sum of all earlier tile sums (a few hundred
     * values, read by every block) — no separate scan of the sums, and no
     * block ever waits on another */
    uint32_t prev = 0;
    for (int t = threadIdx.x; t < (int)blockIdx.x; t += SCAN_BLOCK) prev += sums[t];
    uint32_t prev_excl;
    prev = block_excl_scan(prev, &prev_excl, lds);
    uint32_t run = prev + excl;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; ++k) { uint32_t t = v[k]; v[k] = run; run += t; }
    if (full) {
        uint4 *p = reinterpret_cast<uint4 *>(out + base);
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS / 4; ++k) p[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else {
#pragma unroll
        for (int k = 0; k < SCAN_ITEMS; ++k)
            if (base + k < n) out[base + k] = v[k];
    }
}

__global__ __launch_bounds__(256) void k_bucket_fill(const pm_photon *slots, int64_t n, const uint32_t *key,
                                                     const uint32_t *rank, const uint32_t *cell_start, float4 *ph_a,
                                                     float4 *ph_b, int64_t key_np, int mpc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    /* keys / ranks of the trace's fused count may be plane-major (TraceParams::key_np) */
    const int64_t ki = key_np > 0 ? (i % mpc) * key_np + i / mpc : i;
    const uint32_t k = key[ki];
    if (k == 0xffffffffu) return;
    const uint32_t dst = cell_start[k] + rank[ki];
    const float2 *q = reinterpret_cast<const float2 *>(slots + i);
    const float2 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
    /* a = (bits, p.x) b = (p.y, p.z) c = (alpha.x, alpha.y) d = (alpha.z, wi.x) e = (wi.y, wi.z) */
    ph_a[dst] = make_float4(a.y, b.x, b.y, d.y);
    /* one whole 32-B sector per photon: scattered stores cost a sector
     * write-back each, so (alpha, wi.y) + wi.z as one sector instead of two
     * arrays saves a third of the fill's write traffic */
    ph_b[2 * (size_t)dst] = make_float4(c.x, c.y, d.x, e.x);
    /* + the slot index: the kNN estimator's tie-break and its handle on the
     * photon (pm_gather.hip k_gather_knn) */
    ph_b[2 * (size_t)dst + 1] = make_float4(e.y, __uint_as_float((uint32_t)i), 0.f, 0.f);
}
/* Measured (PMC WRITE_SIZE): ~55 MB written per launch for ~20 MB of photon
 * data — the scattered 16-B stores cost whole-line write-backs. Giving each
 * XCD its own contiguous destination window (blocks b, b+8 share an XCD;
 * eight equal-photon key ranges from the scan) left the write bytes at
 * ~58 MB and read every key 8x: 41 us vs 29 us, so not used. */

__global__ __launch_bounds__(256) void k_zero_invalid_slots(pm_photon *slots, const uint32_t *key, int64_t n,
                                                            int64_t key_np, int mpc) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int64_t ki = key_np > 0 ? (i % mpc) * key_np + i / mpc : i;
    if (key[ki] != 0xffffffffu) return;
    float2 *q = reinterpret_cast<float2 *>(slots + i);
    const float2 z = make_float2(0.f, 0.f);
    q[0] = z; q[1] = z; q[2] = z; q[3] = z; q[4] = z;
}
hipError_t launch_zero_invalid_slots(pm_photon *slots, const uint32_t *key, int64_t n, int64_t key_np, int mpc,
                                     hipStream_t s) {
    if (n <= 0) return hipSuccess;
    pm_launch(k_zero_invalid_slots, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slots, key, n, key_np,
              mpc > 0 ? mpc : 1);
    return hipGetLastError();
}

size_t scan_scratch_words(int64_t n) { return (size_t)((n + SCAN_TILE - 1) / SCAN_TILE) + 16; }

hipError_t launch_exclusive_scan(const uint32_t *in, int64_t n, uint32_t *out, uint32_t *sums, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int ntile = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
    pm_launch(k_scan_reduce, dim3(ntile), dim3(SCAN_BLOCK), 0, s, in, n, sums);
    pm_launch(k_scan_down, dim3(ntile), dim3(SCAN_BLOCK), 0, s, in, n, sums, out, nullptr);
    return hipGetLastError();
}
size_t bucket_scratch_words(int64_t n_slots, uint32_t ncells) {
    const int64_t ntile = ((int64_t)ncells + 1 + SCAN_TILE - 1) / SCAN_TILE;
    return (size_t)(2 * n_slots + ntile + 16);
}

hipError_t launch_bucket_build(const pm_photon *slots, int64_t n, GridDesc g, uint32_t *count, uint32_t *cell_start,
                               uint32_t *scratch, float4 *ph_a, float4 *ph_b, bool counted, hipStream_t s,
                               int64_t key_np, int mpc) {
    if (!counted || key_np * mpc != n) key_np = 0; /* k_bucket_count writes slot order */
    const int64_t nc = (int64_t)g.ncells + 1; /* last counter stays 0 -> cell_start[ncells] = total */
    uint32_t *key = scratch, *rank = scratch + n, *sums = scratch + 2 * n;
    if (n > 0 && !counted)
        pm_launch(k_bucket_count, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slots, n, g, count, key,
                           rank);
    const int ntile = (int)((nc + SCAN_TILE - 1) / SCAN_TILE);
    pm_launch(k_scan_reduce, dim3(ntile), dim3(SCAN_BLOCK), 0, s, count, nc, sums);
    /* the counters are zeroed as they are scanned: ready for the next pass */
    pm_launch(k_scan_down, dim3(ntile), dim3(SCAN_BLOCK), 0, s, count, nc, sums, cell_start, count);
    if (n > 0)
        pm_launch(k_bucket_fill, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, slots, n, key, rank,
                           cell_start, ph_a, ph_b, key_np, mpc > 0 ? mpc : 1);
    return hipGetLastError();
}

} // namespace pm
