/*
 * pm_gather.hip — fixed-radius range query + PPM update (gathering.cu:17-126)
 * over photon buckets (grid) or the reference kd-tree layout, the PPM update
 * of reduced partials, final radiance + sanitisation (gathering.cu:129-146,
 * photonmappingrenderer.cpp:251-268) and the per-step record reset.
 *
 * wave64; 8x8 pixel tiles map onto one wave so a wave's gather points are
 * spatially coherent and share photon buckets in L1/L2.
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pm_kernels.h"

#pragma clang fp contract(off)

namespace pm {
/* ====================================================================== */
/* gather                                                                 */
/* ====================================================================== */
/* gathering.cu:104-126 PPM update */
PMD void ppm_apply(float4 &st, float &N, int M, v3 L, float alpha) {
    if (M > 0) {
        int totalPhotons = N + alpha * M;
        float ratio = totalPhotons / (N + M);
        st.w = st.w * ratio;
        v3 flux = (xyz(st) + L) * ratio;
        st.x = flux.x; st.y = flux.y; st.z = flux.z;
        N = totalPhotons;
    }
}

/* Exact, order-independent flux sums for the bucket gather: each photon's
 * contribution is rounded once to a 64-bit fixed-point integer (scale 2^S
 * chosen per scene so that 2^23 maximal contributions fit, pm_api.cpp
 * fx_scale) and integers add associatively. The bucket order (atomic
 * arrival order in pm_bucket.hip) and the number of GPUs that hold the
 * photons therefore never change a bit of the result. */
struct Fx3 { long long x, y, z; };
/* where record r's partial goes: its rank in the record view (active records
 * only, -1 = not in the view) or r itself (all-records view) */
PMD int64_t partial_index(const GatherParams &P, int64_t r) {
    if (!P.view_rank) return r;
    const uint32_t k = P.view_rank[r];
    return k == 0xffffffffu ? -1 : (int64_t)k;
}
PMD long long to_fx(float c, float scale) { return (long long)rintf(c * scale); }
/* partial of view record k: (M, L) as four int64, or split into an int32
 * count and three int64 flux words (the "reduce" exchange's layout) */
PMD void write_partial(const GatherParams &P, int64_t k, int M, Fx3 L) {
    if (k < 0) return;
    if (P.count) {
        P.count[k] = M;
        long long *f = P.flux + 3 * k;
        f[0] = L.x; f[1] = L.y; f[2] = L.z;
        return;
    }
    longlong2 *q = reinterpret_cast<longlong2 *>(P.partial + 4 * k);
    q[0] = make_longlong2((long long)M, L.x);
    q[1] = make_longlong2(L.y, L.z);
}

/* Fixed-radius query over photon buckets. Every photon with
 * d^2 < r^2 is inside the visited cells because the cell range is taken
 * over [p - r', p + r'] with r' slightly larger than sqrt(r^2). */
PMD void add_hit(Fx3 &Lf, v3 ns, v3 fv, float4 a, float4 b, float wz, float sc) {
    const v3 wi = mk(a.w, b.w, wz);
    const v3 c = fabsf(dot(ns, wi)) * fv * xyz(b); /* processPhoton, gathering.cu:17-23 */
    Lf.x += to_fx(c.x, sc); Lf.y += to_fx(c.y, sc); Lf.z += to_fx(c.z, sc);
}
PMD bool in_radius(v3 p, float4 a, float r2) { /* gathering.cu:32-36 (DistanceSquared < maxDist2) */
    const v3 diff = p - xyz(a);
    return diff.x * diff.x + diff.y * diff.y + diff.z * diff.z < r2;
}

#ifndef PM_SCAN_PIPE
#define PM_SCAN_PIPE 1
#endif
#ifndef PM_SCAN_BATCH
#define PM_SCAN_BATCH 4 /* 6: 116 VGPRs, 8: 142 — the tile kernel drops to 4 / 3 waves per SIMD */
#endif
/* One lane scans its own cells [x0, x1] x [y0, y1] x [z0, z1] straight from
 * global memory: the census launches (their photons-tested count is the
 * per-record unit bench.py prices), lanes whose radius exceeds the grid's
 * design radius (uploaded records), and tiles whose row union is too wide for
 * k_gather_tile's LDS staging. All eight row bounds are loaded first; rows
 * are read in software-pipelined batches (PIPE, the tile kernel's lanes: C3
 * gather 0.51 -> 0.45 ms, C5 0.28 -> 0.25 ms, same box) or four photons at a
 * time (the census / per-lane kernel, whose 64-VGPR budget the pipeline
 * would spill). */
/* the lane's rows, each one contiguous run [b, e) of photons, passed to RANGE(b, e) */
#define PM_LANE_SCAN_CELLS(RANGE) \
    if (y1 <= y0 + 1 && z1 <= z0 + 1) {                                                     \
        /* all row bounds first: 8 independent loads in flight */                           \
        uint32_t rb[4], re[4];                                                              \
_Pragma("unroll")                                                                           \
        for (int k = 0; k < 4; ++k) {                                                       \
            const uint32_t cy = y0 + (k & 1), cz = z0 + (k >> 1);                           \
            const bool use = cy <= y1 && cz <= z1;                                          \
            const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;               \
            rb[k] = use ? P.cell_start[row + x0] : 0u;                                      \
            re[k] = use ? P.cell_start[row + x1 + 1] : 0u;                                  \
            if (COUNT) { vis += re[k] - rb[k]; rows += use; }                               \
        }                                                                                   \
_Pragma("unroll")                                                                           \
        for (int k = 0; k < 4; ++k) RANGE(rb[k], re[k]);                                    \
    } else { /* radius above the grid's design radius (uploaded records) */                 \
        for (uint32_t cz = z0; cz <= z1; ++cz)                                              \
            for (uint32_t cy = y0; cy <= y1; ++cy) {                                        \
                const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;           \
                const uint32_t b = P.cell_start[row + x0], e = P.cell_start[row + x1 + 1];  \
                if (COUNT) { vis += e - b; rows++; }                                        \
                RANGE(b, e);                                                                \
            }                                                                               \
    }                                                                                       \
    do { } while (0)
template <int COUNT, int PIPE = PM_SCAN_PIPE>
PMD void lane_scan(const GatherParams &P, v3 p, float r2, v3 ns, v3 fv, uint32_t x0, uint32_t x1, uint32_t y0,
                   uint32_t y1, uint32_t z0, uint32_t z1, int &M, Fx3 &Lf, unsigned long long &vis,
                   unsigned long long &rows) {
    const GridDesc &g = P.grid;
    const float sc = P.fx_scale;
    const float *phb = reinterpret_cast<const float *>(P.ph_b);
    auto photon = [&](const float4 a, uint32_t j) {
        if (in_radius(p, a, r2)) {
            M++;
            add_hit(Lf, ns, fv, a, P.ph_b[2 * (size_t)j], phb[8 * (size_t)j + 4], sc);
        }
    };
    if constexpr (PIPE != 0) {
        (void)photon;
        constexpr int SB = PM_SCAN_BATCH;
        /* batches of PM_SCAN_BATCH photons, software-pipelined: the next batch's positions
         * are requested before this batch is tested, and the flux words of all
         * of a batch's hits are requested together before any is summed — one
         * memory round trip per batch instead of one for the positions plus one
         * per hit (dense cells: C5's caustic, the soup's incoherent lanes) */
        auto range = [&](uint32_t j, const uint32_t e) {
            if (j >= e) return;
            float4 a[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) a[i] = P.ph_a[min(j + (uint32_t)i, e - 1u)]; /* past e: masked below */
            for (; j < e; j += SB) {
                float4 cur[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) cur[i] = a[i];
                if (j + (uint32_t)SB < e) {
#pragma unroll
                    for (int i = 0; i < SB; ++i) a[i] = P.ph_a[min(j + (uint32_t)SB + (uint32_t)i, e - 1u)];
                }
                uint32_t m = 0u;
#pragma unroll
                for (int i = 0; i < SB; ++i) m |= (j + (uint32_t)i < e && in_radius(p, cur[i], r2)) ? 1u << i : 0u;
                float4 hb[SB];
                float hc[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) {
                    hb[i] = make_float4(0.f, 0.f, 0.f, 0.f);
                    hc[i] = 0.f;
                    if (m & (1u << i)) { hb[i] = P.ph_b[2 * (size_t)(j + i)]; hc[i] = phb[8 * (size_t)(j + i) + 4]; }
                }
#pragma unroll
                for (int i = 0; i < SB; ++i)
                    if (m & (1u << i)) { M++; add_hit(Lf, ns, fv, cur[i], hb[i], hc[i], sc); }
            }
        };
        PM_LANE_SCAN_CELLS(range);
    } else {
        auto range = [&](uint32_t j, const uint32_t e) {
            for (; j + 4 <= e; j += 4) { /* 4 photon loads in flight */
                const float4 a0 = P.ph_a[j], a1 = P.ph_a[j + 1], a2 = P.ph_a[j + 2], a3 = P.ph_a[j + 3];
                photon(a0, j); photon(a1, j + 1); photon(a2, j + 2); photon(a3, j + 3);
            }
            for (; j < e; ++j) photon(P.ph_a[j], j);
        };
        PM_LANE_SCAN_CELLS(range);
    }
}

/* r' of a record's cell box [p - r', p + r']: hardware sqrt (<= 1 ulp), the
 * 1e-4 relative margin covers it */
PMD float box_reach(float r2) { return __builtin_amdgcn_sqrtf(r2) * 1.0001f + 1e-4f; }

/* k_gather_tile: a record's normal requested with its position and its
 * material as one 16-B load (the compiler otherwise loaded m.w, waited, then
 * m.xyz): two round trips fewer before the row bounds. C2 gather 43.7 -> 42.8
 * us (5 runs each, same box); also issuing the material load after the first
 * group's row bounds spilled 28 B and measured slower (45.4 us) */
#ifndef PM_REC_EARLY
#define PM_REC_EARLY 1
#endif
#ifndef PM_TILE_SIDX
#define PM_TILE_SIDX 1
#endif
/* record prologue shared by the bucket kernels: flags, PPM state, BSDF, cell
 * box of [p - r', p + r'] (small: at most 2 x 2 rows, the grid's design case) */
struct GatherRec {
    bool live = false, small = false, big = false;
    float4 st = make_float4(0.f, 0.f, 0.f, 0.f);
    v3 p = mk(0.f, 0.f, 0.f), ns = mk(0.f, 0.f, 0.f), fv = mk(0.f, 0.f, 0.f);
    float r2 = 0.f;
    uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0, z0 = 0, z1 = 0;
    float4 nrm = make_float4(0.f, 0.f, 0.f, 0.f);
    /* phase 1: position, PPM state and cell box. The state is read with the
     * position (speculatively, also for inactive records) so that the cell
     * box waits for one round trip only; the normal is requested here and
     * consumed by shade() */
    template <int PARTIAL, bool EARLY = false>
    PMD void load(const GatherParams &P, int64_t r) {
        if (r >= P.rec_end) return;
        const float4 pos = P.R.pos[r];
        const float4 st0 = P.fresh ? make_float4(0.f, 0.f, 0.f, P.r2init) : P.R.state[r];
        if (EARLY) { /* the normal requested with the position (one round trip fewer) */
            const float4 n0 = P.R.nrm[r];
            if (accept<PARTIAL>(P, r, pos, st0)) nrm = n0;
        } else if (accept<PARTIAL>(P, r, pos, st0)) {
            nrm = P.R.nrm[r];
        }
    }
    /* the flags, PPM state and cell box of record r < rec_end from its loaded
     * position and state; false: inactive (its partial written) */
    template <int PARTIAL>
    PMD bool accept(const GatherParams &P, int64_t r, float4 pos, float4 st0) {
        const uint32_t flags = (uint32_t)__float_as_int(pos.w);
        if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) {
            if (PARTIAL) write_partial(P, partial_index(P, r), 0, Fx3{0, 0, 0});
            return false;
        }
        live = true;
        st = st0;
        r2 = st.w;
        p = xyz(pos);
        if (r2 > 0.f) {
            const GridDesc &g = P.grid;
            const float rq = box_reach(r2);
            /* cells overlapping [p - r', p + r']: cell edge >= 2 r_max, so at
             * most 2 per axis -> at most 4 (y, z) rows of <= 2 cells in x */
            x0 = cell_axis(p.x - rq, g.gx, g.inv_cs, g.dx); x1 = cell_axis(p.x + rq, g.gx, g.inv_cs, g.dx);
            y0 = cell_axis(p.y - rq, g.gy, g.inv_cs, g.dy); y1 = cell_axis(p.y + rq, g.gy, g.inv_cs, g.dy);
            z0 = cell_axis(p.z - rq, g.gz, g.inv_cs, g.dz); z1 = cell_axis(p.z + rq, g.gz, g.inv_cs, g.dz);
            small = y1 <= y0 + 1 && z1 <= z0 + 1;
            big = !small;
        }
        return true;
    }
    /* phase 2: shading normal and BSDF (Kd / pi for matte, processPhoton) */
    PMD void shade(const GatherParams &P) {
        if (!live) return;
        float4 m = P.materials[__float_as_int(nrm.w)];
#if PM_REC_EARLY
        asm volatile("" : "+v"(m.x), "+v"(m.y), "+v"(m.z), "+v"(m.w)); /* one 16-B load, not m.w then m.xyz */
#endif
        fv = __float_as_int(m.w) == PM_MATTE ? xyz(m) * INV_PI : mk(0.f, 0.f, 0.f);
        ns = xyz(nrm);
    }
    /* fused PPM update (gathering.cu:104-126) from the fixed-point sums as
     * doubles (exact integers) */
    PMD void store_sum(const GatherParams &P, int64_t r, int M, double sx, double sy, double sz) {
        if (!live) return;
        const double inv = P.fx_inv;
        v3 L = mk((float)(sx * inv), (float)(sy * inv), (float)(sz * inv));
        float N = P.fresh ? 0.f : P.R.n[r];
        ppm_apply(st, N, M, L, P.ppm_alpha);
        if (M > 0 || P.fresh) { P.R.state[r] = st; P.R.n[r] = N; }
    }
    /* fused PPM update or the partial of the exchange */
    template <int PARTIAL>
    PMD void store(const GatherParams &P, int64_t r, int M, Fx3 Lf) {
        if (!live) return;
        if (PARTIAL) write_partial(P, partial_index(P, r), M, Lf);
        else store_sum(P, r, M, (double)Lf.x, (double)Lf.y, (double)Lf.z);
    }
};

/* Per-lane bucket gather: one lane per record, its own rows from global
 * memory. Census launches (COUNT) and the PM_GATHER_KERNEL=lane experiment. */
template <int PARTIAL, int COUNT>
__global__ __launch_bounds__(GATHER_BLOCK, 8) void k_gather_grid(GatherParams P) { /* 8 waves/SIMD: latency bound */
    const int64_t r = P.rec_begin + (int64_t)blockIdx.x * GATHER_BLOCK + threadIdx.x;
    unsigned long long vis = 0, hits = 0, rows = 0, act = 0;
    GatherRec R;
    R.load<PARTIAL>(P, r);
    R.shade(P);
    int M = 0;
    Fx3 Lf{0, 0, 0};
    if (R.live && R.r2 > 0.f)
        lane_scan<COUNT, 0>(P, R.p, R.r2, R.ns, R.fv, R.x0, R.x1, R.y0, R.y1, R.z0, R.z1, M, Lf, vis, rows);
    if (COUNT && R.live) { hits += (unsigned long long)M; act++; }
    R.store<PARTIAL>(P, r, M, Lf);
    if (COUNT) count4(P.counters, vis, hits, rows, act);
}

/* ---------------------------------------------------------------------- */
/* Tile gather (default): the 64 records of a wave are one 8x8 pixel tile, so
 * their cell boxes overlap almost entirely. The wave takes the union box of
 * its lanes' boxes (X0..X1 x Y0..Y1 x Z0..Z1 cells), and when it has at most
 * 64 (y, z) rows:
 *   1. lane u loads the bounds of union row u (cells X0..X1: one contiguous
 *      run of photons), a wave prefix sum concatenates the rows -> U photons;
 *   2. the concatenation is staged into this wave's LDS window, TILE_CAP
 *      photons at a time, with coalesced loads (positions lane and lane + 64:
 *      1 KiB per load instruction): ph_a (p, wi.x) and the flux half of ph_b
 *      (alpha, wi.y | wi.z); the row of each position comes from a wave
 *      max-scan over the row-start markers;
 *   3. every lane tests the whole union-x run of each of its <= 4 rows from
 *      LDS (lanes sharing a row read the same address: broadcast), its rows
 *      walked as one flattened sequence, two photons per step.
 * A lane tests a superset of its own cells (the union's x-range); every
 * photon with d^2 < r^2 still lies in exactly one visited run, and the sums
 * are exact fixed point, so M and L are bit-identical to k_gather_grid's.
 * Global memory sees one record read, one row-bounds load per union row and
 * ~3 coalesced loads per 64 photons per tile, instead of ~2 scattered loads
 * per photon per lane. Lanes with an oversized radius and
 * tiles with more than 64 union rows fall back to lane_scan. */
#ifndef PM_TILE_CAP
#define PM_TILE_CAP 128
#endif
constexpr int TILE_CAP = PM_TILE_CAP; /* photons per LDS window (two per lane) */
/* PM_TILE_PAIRS (default): positions stored by aligned pairs, 32 B per pair
 * (x0 x1 y0 y1 | z0 z1 . .), so a pair test reads one ds_read_b128 and one
 * ds_read_b64 at immediate offsets (no per-pair address arithmetic) straight
 * into the register pairs of the packed math; runs start at even positions
 * (an odd start masks its first bit). 0: SoA x / y / z with ds_read2. */
#ifndef PM_TILE_PAIRS
#define PM_TILE_PAIRS 1
#endif
#ifndef PM_TILE_XCDG
#define PM_TILE_XCDG 8
#endif
struct TileLds {
#if PM_TILE_PAIRS
    /* TILE_CAP pairs: a run's aligned pairs reach at most one pair past
     * them (lanes beyond their run, masked): that read lands in b[] below,
     * inside the block's LDS. No padding pairs: 7,680 B per wave (the LDS
     * allocation granule makes 7,744 B fit 18 one-wave blocks per CU, 7,680
     * B 20, the VGPR limit): C2 gather 47.4-48.6 -> 44.4-46.3 us (same box) */
    float4 pr[2 * TILE_CAP];
#else
    /* positions SoA, so that a pair of neighbouring photons is one ds_read2;
     * 2 x TILE_CAP entries: the test loop reads up to TILE_CAP past a run's
     * start (lanes beyond their run) without wrapping the index */
    float x[2 * TILE_CAP], y[2 * TILE_CAP], z[2 * TILE_CAP];
#endif
    float4 b[TILE_CAP]; /* alpha.rgb, wi.y */
    float w[TILE_CAP];  /* wi.x */
    float c[TILE_CAP];  /* wi.z */
    int mark[TILE_CAP]; /* union row starting at this position, -1 = none */
};
/* LDS traffic between lanes of one wave: ds_* of a wave execute in order, so
 * a compiler-level ordering point is all the exchange needs */
PMD void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
/* inclusive wave scans on DPP (row_shr 1/2/4/8 inside rows of 16 lanes,
 * then row_bcast 15/31 into rows 1,3 / 2,3): VALU-rate cross-lane moves
 * instead of an LDS round trip per step (__shfl = ds_bpermute). A lane
 * whose DPP source is out of its row, or whose row the mask leaves out,
 * receives `id`, the operation's identity, so no lane guards are needed.
 * Every lane must be active. */
template <class Op>
PMD int wave_scan_dpp(int v, int id, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x111, 0xf, 0xf, false)); /* row_shr:1 */
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x112, 0xf, 0xf, false)); /* row_shr:2 */
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x114, 0xf, 0xf, false)); /* row_shr:4 */
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x118, 0xf, 0xf, false)); /* row_shr:8 */
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false)); /* row_bcast:15 -> rows 1, 3 */
    v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false)); /* row_bcast:31 -> rows 2, 3 */
    return v;
}
PMD uint32_t wave_incl_sum_u32(uint32_t v) {
    return (uint32_t)wave_scan_dpp((int)v, 0, [](int a, int b) { return (int)((uint32_t)a + (uint32_t)b); });
}
PMD int wave_incl_max_i32(int v) { return wave_scan_dpp(v, -1, [](int a, int b) { return max(a, b); }); }
/* wave-uniform min / max (the scan's last lane) */
PMD uint32_t wave_min_u32(uint32_t v) {
    const int m = wave_scan_dpp((int)v, -1, [](int a, int b) { return (int)min((uint32_t)a, (uint32_t)b); });
    return (uint32_t)__builtin_amdgcn_readlane(m, 63);
}
PMD uint32_t wave_max_u32(uint32_t v) {
    const int m = wave_scan_dpp((int)v, 0, [](int a, int b) { return (int)max((uint32_t)a, (uint32_t)b); });
    return (uint32_t)__builtin_amdgcn_readlane(m, 63);
}
/* two 16-bit minima at once (v_pk_min_u16) */
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
PMD uint32_t wave_min_2x16(uint32_t v) {
    const int m = wave_scan_dpp((int)v, -1, [](int a, int b) {
        return (int)__builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(u16x2, a),
                                                                          __builtin_bit_cast(u16x2, b)));
    });
    return (uint32_t)__builtin_amdgcn_readlane(m, 63);
}
PMD uint32_t uniform_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
/* wave-uniform float minimum / maximum (every lane active) */
PMD float wave_min_f(float v) {
    const int m = wave_scan_dpp(__float_as_int(v), __float_as_int(INFINITY),
                                [](int a, int b) { return __float_as_int(fminf(__int_as_float(a), __int_as_float(b))); });
    return __int_as_float(__builtin_amdgcn_readlane(m, 63));
}
PMD float wave_max_f(float v) {
    const int m = wave_scan_dpp(__float_as_int(v), __float_as_int(-INFINITY),
                                [](int a, int b) { return __float_as_int(fmaxf(__int_as_float(a), __int_as_float(b))); });
    return __int_as_float(__builtin_amdgcn_readlane(m, 63));
}

/* one-wave blocks are dealt round-robin over the 8 XCDs: blocks b, b + 8, ...
 * (one XCD, dispatched close together) take PM_TILE_XCDG neighbouring entries
 * of the tile list, so neighbouring tiles share their photon rows in one L2
 * (C2 gather FETCH 141 -> 96 MB per launch at 8, 118 at 4, 82 at 16; time
 * within noise of each other, ~2 % below no grouping). A bijection on whole
 * groups of 8 x XCDG entries; the tail keeps its order. (The kNN tile kernel
 * measured 1.5 % slower with it: its passes re-stage unions a tile's own
 * wave re-reads, not its neighbours'.) */
PMD int64_t xcd_tile(int64_t w, int64_t nt) {
#if PM_TILE_XCDG > 1
    constexpr int64_t GX = 8 * PM_TILE_XCDG;
    if (w < nt / GX * GX) w = w / GX * GX + (w % 8) * PM_TILE_XCDG + (w / 8) % PM_TILE_XCDG;
#endif
    return w;
}

typedef float f2 __attribute__((ext_vector_type(2)));
/* integer-valued double in [0, 2^53) -> int64, exactly (two 32-bit halves) */
PMD long long d2ll(double d) {
    const uint32_t hi = (uint32_t)(d * 0x1p-32);
    const uint32_t lo = (uint32_t)fma((double)hi, -0x1p32, d);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
/* PM_TILE_STATS builds (make variant VFLAGS=-DPM_TILE_STATS): per-wave event
 * counts of k_gather_tile into counters[8..15] (read with pm_trace_profile):
 * tile waves, windows, test pairs, hit iterations, direct lanes, chunks,
 * wide (> 64 rows) waves, staged photons */
#ifdef PM_TILE_STATS
#define TILE_STAT(k, v) do { const unsigned long long tv_ = (unsigned long long)(v); \
    if ((threadIdx.x & 63) == 0) atomicAdd(&P.counters[8 + (k)], tv_); } while (0)
#elif defined(PM_TILE_TIMES)
/* per-wave counts for the wave timeline records (k_gather_tile only) */
#define TILE_STAT(k, v) do { tstat[(k)] += (uint32_t)(v); } while (0)
#else
#define TILE_STAT(k, v) do { } while (0)
#endif

/* PM_GATHER_PROFILE builds (make variant VFLAGS=-DPM_GATHER_PROFILE): wave
 * clock (s_memtime) per phase of k_gather_tile, summed over waves into
 * counters[8..14] (record, group, stage, test, hits, direct, store) and the
 * wave count into counters[15] (tools/gather_profile.py). A phase's time
 * includes the memory waits of the loads it first consumes. */
struct GProf {
#ifdef PM_GATHER_PROFILE
    uint64_t last = 0, acc[7] = {0, 0, 0, 0, 0, 0, 0};
    PMD void begin() { last = __builtin_amdgcn_s_memtime(); }
    PMD void mark(int i) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        acc[i] += t - last;
        last = t;
    }
    PMD void flush(unsigned long long *out) {
        if (!out || (threadIdx.x & 63) != 0) return;
        for (int i = 0; i < 7; ++i) atomicAdd(&out[8 + i], (unsigned long long)acc[i]);
        atomicAdd(&out[15], 1ull);
    }
#else
    PMD void begin() {}
    PMD void mark(int) {}
    PMD void flush(unsigned long long *) {}
#endif
};

/* the default instance (span 2, non-negative sums) at 5 waves/SIMD, the
 * LDS limit (TileLds): unbounded, the compiler takes more than 102 VGPRs
 * since the cooperative direct scan (4 waves); bounded, none spill. The
 * other instances keep the compiler's choice (bounded they spill) */
#ifndef PM_TILE_WAVES
#define PM_TILE_WAVES 5
#endif
template <int NN, int KR>
constexpr int tile_waves() { return NN && KR == 2 ? PM_TILE_WAVES : 1; }
#define TILE_OCC __attribute__((amdgpu_waves_per_eu(tile_waves<NN, KR>(), 8)))
/* the cell box [X0, X1] x [Y0, Y1] x [Z0, Z1] of the lanes with `in` set */
PMD void union_box6(const GridDesc &g, bool in, uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1, uint32_t z0,
                    uint32_t z1, uint32_t &X0, uint32_t &X1, uint32_t &Y0, uint32_t &Y1, uint32_t &Z0, uint32_t &Z1) {
    if (g.dx < 65536 && g.dy < 65536 && g.dz < 65536) {
        /* three packed 16-bit minima (maxima as minima of 0xffff - c) */
        const uint32_t m0 = wave_min_2x16(in ? (x0 << 16) | y0 : 0xffffffffu);
        const uint32_t m1 = wave_min_2x16(in ? ((0xffffu - x1) << 16) | (0xffffu - y1) : 0xffffffffu);
        const uint32_t m2 = wave_min_2x16(in ? (z0 << 16) | (0xffffu - z1) : 0xffffffffu);
        X0 = m0 >> 16; Y0 = m0 & 0xffffu; X1 = 0xffffu - (m1 >> 16); Y1 = 0xffffu - (m1 & 0xffffu);
        Z0 = m2 >> 16; Z1 = 0xffffu - (m2 & 0xffffu);
    } else {
        X0 = wave_min_u32(in ? x0 : 0xffffffffu); X1 = wave_max_u32(in ? x1 : 0u);
        Y0 = wave_min_u32(in ? y0 : 0xffffffffu); Y1 = wave_max_u32(in ? y1 : 0u);
        Z0 = wave_min_u32(in ? z0 : 0xffffffffu); Z1 = wave_max_u32(in ? z1 : 0u);
    }
}
PMD void union_box(const GridDesc &g, const GatherRec &R, bool in, uint32_t &X0, uint32_t &X1, uint32_t &Y0,
                   uint32_t &Y1, uint32_t &Z0, uint32_t &Z1) {
    union_box6(g, in, R.x0, R.x1, R.y0, R.y1, R.z0, R.z1, X0, X1, Y0, Y1, Z0, Z1);
}
#ifndef PM_GROUP_R
#define PM_GROUP_R 3
#endif
/* a group takes the lanes whose box starts within GROUP_R cells of the
 * leader's: y rows [ly - R, ly + R + 1] fit the row pitch 8, z layers x 8
 * rows fit the 64 lanes */
constexpr uint32_t GROUP_R = PM_GROUP_R;
/* C2 gather: 12 -> 51.9 us, 8 -> 51.3, 4 -> 48.5, 2 -> 48.8, 1 -> 48.9 (C3
 * unchanged): a small LDS group still beats its lanes scanning per lane.
 * Sparse maps are the exception: with under 1/SPARSE_CELLS photons per
 * cell (C1: 52K photons in 2.7M cells) a lane's own cells hold almost
 * nothing and a small group's staging overhead is the larger cost — C1 14.9
 * us with 12, 34.9 us with 4 — so they keep groups of >= 12 lanes. The
 * density is read on the device (cell_start[ncells] = photons in the map). */
#ifndef PM_GROUP_MIN
#define PM_GROUP_MIN 4
#endif
#ifndef PM_GROUP_MIN_SPARSE
#define PM_GROUP_MIN_SPARSE 12
#endif
constexpr int GROUP_MIN = PM_GROUP_MIN, GROUP_MIN_SPARSE = PM_GROUP_MIN_SPARSE;
constexpr uint32_t SPARSE_CELLS = 20;
#ifndef PM_TILE_UMAX
#define PM_TILE_UMAX 512
#endif
constexpr int TILE_UMAX = PM_TILE_UMAX; /* C5 (r02 grid): no cap 2.88 ms, 2048 0.44, 1024 0.41, 512 0.43; adaptive grid (r03): 2048 0.268, 1024 0.24, 512 0.205; C2 unchanged */
/* Dense maps (>= 2 photons per 5 cells: C5's caustic scene, 0.73; C2 0.20)
 * fall back to the per-lane scans from smaller unions on: C5 tile gather
 * 0.153-0.159 ms at 512, 0.145-0.148 at 256, 0.150-0.152 at 192, 0.158-0.161
 * at 128; C2 0.5 % slower at 256, C4 unchanged (round 6, same box,
 * profiles/r06/tile_umax). The density is read on the device, as for
 * GROUP_MIN_SPARSE. */
#ifndef PM_TILE_UMAX_DENSE
#define PM_TILE_UMAX_DENSE 256
#endif
constexpr int TILE_UMAX_DENSE = PM_TILE_UMAX_DENSE;
static_assert(2 * GROUP_R + 2 <= 8, "group rows exceed the 64-lane row map");
/* the updated radii of a wave into the adaptive-grid histogram
 * (GatherParams::r2hist): one atomic per distinct bin of the wave (a tile's
 * radii are alike), in one of R2_COPIES copies by block */
PMD void r2_histogram(const GatherParams &P, bool live, float r2) {
    int b = -1;
    if (live) {
        const float t = r2 * P.r2hist_inv;
        b = t >= 1.f ? 0 : !(t > 0.f) ? R2_BINS - 1 : min(R2_BINS - 1, (int)(-__log2f(t) * (float)R2_PER_OCTAVE));
    }
    unsigned long long pend = __ballot(b >= 0);
    uint32_t *h = P.r2hist + (blockIdx.x % (unsigned)R2_COPIES) * R2_BINS;
    while (pend) {
        const int l = __builtin_ctzll(pend);
        const int bb = __builtin_amdgcn_readlane(b, l);
        const unsigned long long same = __ballot(b == bb);
        if ((threadIdx.x & 63) == (unsigned)l) atomicAdd(&h[bb], (uint32_t)__builtin_popcountll(same));
        pend &= ~same;
    }
}
__global__ __launch_bounds__(R2_BINS) void k_r2hist_reduce(uint32_t *hist, uint32_t *out) {
    const int b = threadIdx.x;
    uint32_t t = 0u;
    for (int k = 0; k < R2_COPIES; ++k) {
        t += hist[k * R2_BINS + b];
        hist[k * R2_BINS + b] = 0u; /* ready for the next histogram */
    }
    out[b] = t;
}
hipError_t launch_r2hist_reduce(uint32_t *hist, uint32_t *out_mapped, hipStream_t s) {
    pm_launch(k_r2hist_reduce, dim3(1), dim3(R2_BINS), 0, s, hist, out_mapped);
    return hipGetLastError();
}
/* KR: cells per axis a lane's box [p - r', p + r'] spans at most, for the
 * grid's design radius (GatherParams::span: cell edge 2 r' / (KR - 1), the
 * cell-edge sweep of DESIGN.md §5). A lane reads KR z-layers, each one
 * contiguous run of <= KR rows of the union; its group radius keeps the union
 * inside the 64-lane row map (2 GR + KR <= 8 rows per axis). */
template <int KR>
constexpr uint32_t tile_group_r() { return KR == 2 ? GROUP_R : (8u - (uint32_t)KR) / 2u; }
struct TileLds;
/* The lanes of `sel` (small boxes: at most KR x KR rows each) all at once:
 * their rows are concatenated (row slot = lane, its owner from a max-scan
 * over the owners' first slots), the rows' photons concatenated again and
 * tested 64 per step, each against its owner's query (shuffled from the
 * owner); hits are added with add_hit — lane_scan's terms — into the
 * owner's int64 sums in LDS (exact, order-free), so M and L equal
 * lane_scan's bit for bit. A step costs the whole wave whatever the number
 * of owners: the cost is ~ the lanes' photons / 64. Every lane active. */
PMD void coop_batch(const GatherParams &P, TileLds &T, int lane, const GatherRec &R, bool &sel, int &M, Fx3 &Lf) {
    const GridDesc &g = P.grid;
    const float sc = P.fx_scale;
    const float *phb = reinterpret_cast<const float *>(P.ph_b);
    /* per-owner sums (M, L.x, L.y, L.z) in the idle staging array: 64 x 32 B */
    unsigned long long *acc = reinterpret_cast<unsigned long long *>(T.b);
    static_assert(sizeof(T.b) >= 64 * 32, "owner sums fit the flux staging array");
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[4 * lane + q] = 0ull;
    const uint32_t ny = sel ? R.y1 - R.y0 + 1u : 0u, nr = sel ? ny * (R.z1 - R.z0 + 1u) : 0u;
    const uint32_t rin = wave_incl_sum_u32(nr), rpre = rin - nr;
    const uint32_t RT = uniform_u32(__builtin_amdgcn_readlane(rin, 63));
    for (uint32_t c0 = 0; c0 < RT; c0 += 64u) {
        /* row slot c0 + lane: its owner, the lane whose slots [rpre, rin) hold it */
        T.mark[lane] = -1;
        wave_lds_sync();
        if (nr > 0u) {
            if (rpre >= c0 && rpre < c0 + 64u) T.mark[rpre - c0] = lane;
            else if (rpre < c0 && rin > c0) T.mark[0] = lane;
        }
        wave_lds_sync();
        const int o = wave_incl_max_i32(T.mark[lane]);
        wave_lds_sync();
        const int os = max(o, 0);
        const uint32_t j = c0 + (uint32_t)lane;
        const uint32_t ox0 = (uint32_t)__shfl((int)R.x0, os), ox1 = (uint32_t)__shfl((int)R.x1, os);
        const uint32_t oy0 = (uint32_t)__shfl((int)R.y0, os), oz0 = (uint32_t)__shfl((int)R.z0, os);
        const uint32_t ony = (uint32_t)__shfl((int)ny, os), orp = (uint32_t)__shfl((int)rpre, os);
        uint32_t B = 0u, len = 0u;
        if (j < RT && o >= 0) {
            const uint32_t k = j - orp;
            const uint32_t cy = oy0 + k % ony, cz = oz0 + k / ony;
            const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
            B = P.cell_start[row + ox0];
            len = P.cell_start[row + ox1 + 1u] - B;
        }
        const uint32_t incl = wave_incl_sum_u32(len), pre = incl - len;
        const uint32_t U = uniform_u32(__builtin_amdgcn_readlane(incl, 63));
        const uint32_t gofs = B - pre;
        for (uint32_t t0 = 0; t0 < U; t0 += 64u) {
            T.mark[lane] = -1;
            wave_lds_sync();
            if (len > 0u) {
                if (pre >= t0 && pre < t0 + 64u) T.mark[pre - t0] = lane;
                else if (pre < t0 && pre + len > t0) T.mark[0] = lane;
            }
            wave_lds_sync();
            const int u = max(wave_incl_max_i32(T.mark[lane]), 0);
            wave_lds_sync();
            const uint32_t t = t0 + (uint32_t)lane;
            const uint32_t gi = t + (uint32_t)__shfl((int)gofs, u);
            const int ow = __shfl(os, u);
            const v3 p = mk(__shfl(R.p.x, ow), __shfl(R.p.y, ow), __shfl(R.p.z, ow));
            const float r2 = __shfl(R.r2, ow);
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            bool h = false;
            if (t < U) {
                a = P.ph_a[gi];
                h = in_radius(p, a, r2);
            }
            if (__ballot(h)) {
                const v3 ns = mk(__shfl(R.ns.x, ow), __shfl(R.ns.y, ow), __shfl(R.ns.z, ow));
                const v3 fv = mk(__shfl(R.fv.x, ow), __shfl(R.fv.y, ow), __shfl(R.fv.z, ow));
                if (h) {
                    Fx3 c{0, 0, 0};
                    add_hit(c, ns, fv, a, P.ph_b[2 * (size_t)gi], phb[8 * (size_t)gi + 4], sc);
                    atomicAdd(&acc[4 * ow], 1ull);
                    atomicAdd(&acc[4 * ow + 1], (unsigned long long)c.x);
                    atomicAdd(&acc[4 * ow + 2], (unsigned long long)c.y);
                    atomicAdd(&acc[4 * ow + 3], (unsigned long long)c.z);
                }
            }
        }
    }
    wave_lds_sync();
    if (sel) {
        M = (int)acc[4 * lane];
        Lf = Fx3{(long long)acc[4 * lane + 1], (long long)acc[4 * lane + 2], (long long)acc[4 * lane + 3]};
        sel = false;
    }
    wave_lds_sync(); /* the sums are read before anything else writes the array */
}

/* COST: record each wave's lifetime into P.tile_cost (the launch that
 * measures the tile list for k_tile_sort); a separate instance, since the
 * clock kept live across the kernel cost the timed instance 12 B of scratch */
template <int PARTIAL, int NN, int KR, bool COST>
__global__ __launch_bounds__(TILE_BLOCK) TILE_OCC void k_gather_tile(GatherParams P) {
    static_assert(KR >= 2 && KR <= 5 && 2 * tile_group_r<KR>() + KR <= 8, "lane box / group radius");
    constexpr uint32_t GR = tile_group_r<KR>();
    __shared__ TileLds tiles[TILE_BLOCK / 64];
    TileLds &T = tiles[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    int64_t r, w = 0;
    const unsigned long long tc0 = COST ? __builtin_amdgcn_s_memrealtime() : 0ull;
    if (P.tiles) { /* only tiles with an active record (no block-level barrier below: a wave may leave) */
        w = (int64_t)blockIdx.x * (TILE_BLOCK / 64) + (threadIdx.x >> 6);
        const int64_t nt = P.n_tiles_dev ? (int64_t)*P.n_tiles_dev : P.n_tiles;
        if (w >= nt) return;
        if (TILE_BLOCK == 64) w = xcd_tile(w, nt);
#if PM_TILE_SIDX
        /* wave-uniform entry through the scalar cache (a vector load of it cost an L2 round trip) */
        w = (int64_t)__builtin_amdgcn_readfirstlane((int)w);
        r = P.rec_begin + (int64_t)((const_u32_ptr)P.tiles)[w] * 64 + lane;
#else
        r = P.rec_begin + (int64_t)P.tiles[w] * 64 + lane;
#endif
    } else {
        r = P.rec_begin + (int64_t)blockIdx.x * TILE_BLOCK + threadIdx.x;
    }
    const GridDesc &g = P.grid;
#ifdef PM_TILE_TIMES
    const unsigned long long tt0 = __builtin_amdgcn_s_memrealtime();
    uint32_t tstat[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    GProf gp;
    gp.begin();
    GatherRec R;
    R.load<PARTIAL, PM_REC_EARLY != 0>(P, r);
    /* a box of <= KR cells per axis takes part in the LDS groups; larger
     * (radius above the grid's design radius) scans its own cells */
    const bool small = R.live && R.r2 > 0.f && R.y1 - R.y0 < (uint32_t)KR && R.z1 - R.z0 < (uint32_t)KR;
    int M = 0;
    Fx3 Lf{0, 0, 0};
    const float sc = P.fx_scale;
    unsigned long long nv = 0, nr = 0; /* lane_scan census (unused) */
    /* NN (no negative contribution possible, GatherParams::fx_nonneg): the
     * integer-valued contributions rint(c * 2^S) are summed in double — exact
     * while the sum stays below 2^53 (checked at the end; partial sums of
     * non-negative terms never exceed it), and 4 instructions per channel
     * instead of a float -> int64 conversion and a 64-bit add */
    double dx = 0.0, dy = 0.0, dz = 0.0;
    R.shade(P);
    const v3 fvs = R.fv * sc;
    const f2 px2 = {R.p.x, R.p.x}, py2 = {R.p.y, R.p.y}, pz2 = {R.p.z, R.p.z};
    const f2 r2v = {R.r2, R.r2};
    /* Groups: the first pending lane leads; every pending lane whose box
     * starts within GR cells of the leader's on each axis joins. A group's
     * union box is at most (2 GR + KR)^3 cells (<= 8 x 8 rows), so it always
     * fits the 64-lane row map; a coherent tile is one group, a tile across a
     * depth edge two or three, never one huge box. */
    bool pend = small;
    bool direct = R.live && R.r2 > 0.f && !small; /* lanes that scan their own cells from global memory */
    const uint64_t n_map = P.cell_start[g.ncells];
    const int group_min = n_map * SPARSE_CELLS < (uint64_t)g.ncells ? GROUP_MIN_SPARSE : GROUP_MIN;
    const uint32_t umax = n_map * 5u >= (uint64_t)g.ncells * 2u ? (uint32_t)TILE_UMAX_DENSE : (uint32_t)TILE_UMAX;
    gp.mark(0);
    while (true) {
        const unsigned long long pm = __ballot(pend);
        if (pm == 0ull) break;
        /* the box of all pending lanes when it fits the row map (the common,
         * coherent tile: one group), else the leader's neighbourhood */
        uint32_t X0, X1, Y0, Y1, Z0, Z1, LY;
        bool mine = pend;
        /* 1. union row u = lane: photons [B, B + len); u = (cz - Z0) * 2^LY +
         * (cy - Y0) (no lane divides; padding rows are empty) */
        uint32_t B = 0u, len = 0u;
        union_box(g, R, mine, X0, X1, Y0, Y1, Z0, Z1);
        /* row pitch: NY rounded up to a power of two, 2^LY */
        LY = Y1 > Y0 ? 32u - (uint32_t)__builtin_clz(Y1 - Y0) : 0u;
        if (LY > 6u || ((uint64_t)(Z1 - Z0 + 1u) << LY) > 64u) {
            const int leader = __builtin_ctzll(pm);
            const uint32_t lx = __builtin_amdgcn_readlane(R.x0, leader), ly = __builtin_amdgcn_readlane(R.y0, leader),
                           lz = __builtin_amdgcn_readlane(R.z0, leader);
            mine = pend && R.x0 + GR - lx <= 2u * GR && R.y0 + GR - ly <= 2u * GR && R.z0 + GR - lz <= 2u * GR;
            /* an incoherent tile (lanes on many far-apart surfaces, e.g. a
             * triangle soup) would need a group per few lanes: below
             * GROUP_MIN lanes the rest scan their own cells per lane */
            if (__builtin_popcountll(__ballot(mine)) < group_min) {
                direct = direct || pend;
                break;
            }
            union_box(g, R, mine, X0, X1, Y0, Y1, Z0, Z1);
            LY = 3u;
        }
        const uint32_t cy = Y0 + ((uint32_t)lane & ((1u << LY) - 1u)), cz = Z0 + ((uint32_t)lane >> LY);
        if (cy <= Y1 && cz <= Z1) {
            const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
            B = P.cell_start[row + X0];
            len = P.cell_start[row + X1 + 1u] - B;
        }
        pend = pend && !mine;
        TILE_STAT(0, 1);
        const uint32_t incl = wave_incl_sum_u32(len), pre = incl - len;
        const uint32_t U = uniform_u32(__builtin_amdgcn_readlane(incl, 63));
        if (U == 0u) continue;
        /* a dense union (many photons per cell, e.g. C5's caustic scene: 4x
         * C2's density) costs more to stage than its lanes read on their own:
         * above TILE_UMAX photons the group's lanes scan their own cells */
        if (U > umax) { direct = direct || mine; continue; }
        const uint32_t gofs = B - pre; /* photon index of concatenated position t in row u: t + gofs_u */
        /* this lane's rows as KR runs of the concatenation: rows (y0 .. y1, z)
         * are neighbours in the union, so each z-layer of the lane's box is
         * one contiguous run [s_k, e_k) */
        const uint32_t ny = mine ? R.y1 - R.y0 + 1u : 1u;
        const uint32_t nz = mine ? R.z1 - R.z0 + 1u : 0u;
        uint32_t sK[KR], eK[KR];
#pragma unroll
        for (int k = 0; k < KR; ++k) {
            /* every lane shuffles: a bpermute from a lane that is inactive at
             * the shuffle reads 0 */
            const int u = mine && (uint32_t)k < nz ? (int)(((R.z0 + (uint32_t)k - Z0) << LY) + (R.y0 - Y0)) : 0;
            const uint32_t s0 = (uint32_t)__shfl((int)pre, u), e0 = (uint32_t)__shfl((int)incl, u + (int)ny - 1);
            sK[k] = (uint32_t)k < nz ? s0 : 0u;
            eK[k] = (uint32_t)k < nz ? e0 : 0u;
        }
        gp.mark(1);
        for (uint32_t T0 = 0; T0 < U; T0 += TILE_CAP) {
            const uint32_t n = min((uint32_t)TILE_CAP, U - T0);
            TILE_STAT(1, 1);
            TILE_STAT(7, n);
            /* 2. stage positions T0 + lane (and T0 + 64 + lane) */
            constexpr int H = TILE_CAP / 64;
            static_assert(H == 1 || H == 2, "TILE_CAP is 64 or 128");
#pragma unroll
            for (int h = 0; h < H; ++h) T.mark[lane + 64 * h] = -1;
            wave_lds_sync();
            if (len > 0u) {
                if (pre >= T0 && pre < T0 + TILE_CAP) T.mark[pre - T0] = lane;
                else if (pre < T0 && pre + len > T0) T.mark[0] = lane; /* row running into the window */
            }
            wave_lds_sync();
            const float *phb = reinterpret_cast<const float *>(P.ph_b);
#if PM_TILE_PAIRS
            static_assert(H == 2, "paired staging: two positions per lane");
            {
                /* lane l stages positions 2 l and 2 l + 1, a whole pair: one
                 * 16-B and one 8-B LDS write instead of three scattered words
                 * per position (bank conflicts) */
                const int2 m2 = *reinterpret_cast<const int2 *>(&T.mark[2 * lane]);
                const int incl = wave_incl_max_i32(max(m2.x, m2.y));
                const int prev = __shfl(incl, (lane + 63) & 63);
                const int u0 = max(lane == 0 ? -1 : prev, m2.x), u1 = incl;
                const uint32_t q0 = 2u * (uint32_t)lane;
                const uint32_t gi0 = T0 + q0 + (uint32_t)__shfl((int)gofs, u0);
                const uint32_t gi1 = T0 + q0 + 1u + (uint32_t)__shfl((int)gofs, u1);
                /* positions at or beyond n re-read position 0's photon (n >= 1) and are never read */
                const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gi0, 0);
                const uint32_t j0 = q0 < n ? gi0 : g0, j1 = q0 + 1u < n ? gi1 : g0;
                const float4 pa0 = P.ph_a[j0], pa1 = P.ph_a[j1];
                const float4 qa0 = P.ph_b[2 * (size_t)j0], qa1 = P.ph_b[2 * (size_t)j1];
                const float ca0 = phb[8 * (size_t)j0 + 4], ca1 = phb[8 * (size_t)j1 + 4];
                T.pr[2 * lane] = make_float4(pa0.x, pa1.x, pa0.y, pa1.y);
                *reinterpret_cast<f2 *>(&T.pr[2 * lane + 1]) = f2{pa0.z, pa1.z};
                *reinterpret_cast<f2 *>(&T.w[q0]) = f2{pa0.w, pa1.w};
                T.b[q0] = qa0; T.b[q0 + 1] = qa1;
                *reinterpret_cast<f2 *>(&T.c[q0]) = f2{ca0, ca1};
            }
#else
            int u[H];
            u[0] = wave_incl_max_i32(T.mark[lane]);
            if (H == 2) u[H - 1] = max(wave_incl_max_i32(T.mark[lane + 64 * (H - 1)]), __builtin_amdgcn_readlane(u[0], 63));
            uint32_t gi[H];
#pragma unroll
            for (int h = 0; h < H; ++h) gi[h] = T0 + 64u * h + (uint32_t)lane + (uint32_t)__shfl((int)gofs, u[h]);
            /* every load in flight, then the LDS writes; positions at or beyond
             * n re-read position 0's photon (n >= 1) and are never read */
            const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gi[0], 0);
            float4 pa[H], qa[H];
            float ca[H];
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const uint32_t j = (uint32_t)lane + 64u * h < n ? gi[h] : g0;
                pa[h] = P.ph_a[j]; qa[h] = P.ph_b[2 * (size_t)j]; ca[h] = phb[8 * (size_t)j + 4];
            }
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const int q = lane + 64 * h;
                T.x[q] = pa[h].x; T.y[q] = pa[h].y; T.z[q] = pa[h].z;
                T.w[q] = pa[h].w;
                T.b[q] = qa[h]; T.c[q] = ca[h];
            }
#endif
            wave_lds_sync();
            gp.mark(2);
            /* 3. each run of this lane within the window: LDS positions [base,
             * base + m). Tested two photons per packed instruction, 32
             * positions at a time, into hit masks; the hits of all runs are
             * then summed in one loop with every lane busy (max over lanes of
             * its hits per chunk, not one masked pass per photon any lane hits). */
#if PM_TILE_PAIRS
            /* the pairs from even position a + v0: cnt (<= 32) positions, bits 2j / 2j + 1 of pair j;
             * positions outside [lo_bit, hi_bit) of this chunk are another run's or the window's */
            auto test32p = [&](uint32_t a, uint32_t v0, uint32_t cnt, uint32_t lo_bit, uint32_t hi_bit) {
                const float4 *pp = &T.pr[a + v0]; /* pair (a + v0) / 2: two float4 each */
                uint32_t bits = 0u;
                const uint32_t np = (cnt + 1u) >> 1;
#ifndef PM_TEST_UNROLL
#define PM_TEST_UNROLL 2 /* 96 VGPRs, 5 waves/SIMD (4: 110 VGPRs, 4 waves): C2 gather 48.9-49.7 -> 47.5-48.4 us, C5 0.217 -> 0.206 ms, C3 0.545 -> 0.563 ms */
#endif
#pragma unroll PM_TEST_UNROLL
                for (uint32_t j = 0; j < np; ++j) {
                    const float4 xy = pp[2 * j];
                    const f2 zz = *reinterpret_cast<const f2 *>(&pp[2 * j + 1]);
                    const f2 ddx = px2 - f2{xy.x, xy.y}, ddy = py2 - f2{xy.z, xy.w}, ddz = pz2 - zz;
                    const f2 d2 = (ddx * ddx + ddy * ddy) + ddz * ddz;
                    /* d2 < r^2 is the sign of min(d2, FLT_MAX) - r^2: exact
                     * for finite d2 (a difference of unequal floats is never
                     * 0, d2 >= +0), and a NaN d2 (non-finite photon or record
                     * coordinates; its sign bit is arbitrary — the packed
                     * subtract negates an operand) becomes FLT_MAX, false as
                     * the comparison is; shifted in with one alignbit per
                     * photon; the first pair ends in the top bits: reversed
                     * below */
                    const f2 df = f2{fminf(d2.x, 0x1.fffffep127f), fminf(d2.y, 0x1.fffffep127f)} - r2v;
                    bits = __builtin_amdgcn_alignbit(bits, __float_as_uint(df.x), 31u);
                    bits = __builtin_amdgcn_alignbit(bits, __float_as_uint(df.y), 31u);
                }
                bits = __builtin_bitreverse32(bits) >> (32u - 2u * np);
                const uint32_t hi_m = hi_bit >= 32u ? 0xffffffffu : (1u << hi_bit) - 1u;
                return bits & hi_m & ~((1u << lo_bit) - 1u);
            };
#endif
#if !PM_TILE_PAIRS
            auto test32 = [&](uint32_t base, uint32_t v0, uint32_t cnt, uint32_t m) {
                const float *xs = T.x + base + v0, *ys = T.y + base + v0, *zs = T.z + base + v0;
                uint32_t bits = 0u;
#pragma unroll 4
                for (uint32_t j = 0; j < cnt; j += 2) {
                    /* in_radius for both photons: ((dx^2 + dy^2) + dz^2) < r^2 */
                    const f2 ddx = px2 - f2{xs[j], xs[j + 1]}, ddy = py2 - f2{ys[j], ys[j + 1]},
                             ddz = pz2 - f2{zs[j], zs[j + 1]};
                    const f2 d2 = (ddx * ddx + ddy * ddy) + ddz * ddz;
                    if (d2.x < R.r2) bits |= 1u << j;
                    if (d2.y < R.r2) bits |= 2u << j;
                }
                /* positions at or beyond m belong to the next run / window */
                const uint32_t left = m > v0 ? m - v0 : 0u;
                return bits & (left >= 32u ? 0xffffffffu : (1u << left) - 1u);
            };
#endif
            auto hit = [&](uint32_t t) {
                const float4 qb4 = T.b[t];
                const v3 wi = mk(T.w[t], qb4.w, T.c[t]);
                if (NN) {
                    /* fvs = fv * 2^S: the power-of-two scale commutes with the
                     * rounding, so this is rint(c * 2^S) for c of processPhoton */
                    const v3 c = fabsf(dot(R.ns, wi)) * fvs * xyz(qb4);
                    dx += (double)rintf(c.x); dy += (double)rintf(c.y); dz += (double)rintf(c.z);
                } else {
                    add_hit(Lf, R.ns, R.fv, make_float4(0.f, 0.f, 0.f, wi.x), qb4, wi.z, sc);
                }
            };
            uint32_t mK[KR], baseK[KR], vK[KR];
            uint32_t vmax = 0u;
#pragma unroll
            for (int k = 0; k < KR; ++k) {
                const uint32_t lo = max(sK[k], T0), hi = min(eK[k], T0 + n);
                mK[k] = hi > lo ? hi - lo : 0u;
                baseK[k] = mK[k] ? lo - T0 : 0u; /* < TILE_CAP */
#if PM_TILE_PAIRS
                /* from the even position below the run: one more position when it starts odd */
                mK[k] += mK[k] ? (baseK[k] & 1u) : 0u;
                baseK[k] &= ~1u;
#endif
                vK[k] = wave_max_u32(mK[k]);
                vmax = max(vmax, vK[k]);
            }
            for (uint32_t vb = 0; vb < vmax; vb += 32) {
                TILE_STAT(5, 1);
                uint32_t bK[KR], any = 0u;
                int nh = 0;
#pragma unroll
                for (int k = 0; k < KR; ++k) {
                    TILE_STAT(2, (min(32u, vK[k] > vb ? vK[k] - vb : 0u) + 1) / 2);
#if PM_TILE_PAIRS
                    {
                        /* the run's first position is odd: bit 0 of its first chunk is not its own */
                        const uint32_t lob = vb == 0u && mK[k] ? (uint32_t)(max(sK[k], T0) - T0 - baseK[k]) : 0u;
                        const uint32_t hib = mK[k] > vb ? mK[k] - vb : 0u;
                        bK[k] = vK[k] > vb ? test32p(baseK[k], vb, min(32u, vK[k] - vb), lob, hib) : 0u;
                    }
#else
                    bK[k] = vK[k] > vb ? test32(baseK[k], vb, min(32u, vK[k] - vb), mK[k]) : 0u;
#endif
                    nh += __builtin_popcount(bK[k]);
                    any |= bK[k];
                }
                M += nh;
                gp.mark(3);
                TILE_STAT(3, wave_max_u32(nh));
                while (any) {
                    /* the first run with a hit left: its lowest position */
                    uint32_t t = 0u;
                    bool took = false;
                    any = 0u;
#pragma unroll
                    for (int k = 0; k < KR; ++k) {
                        if (!took && bK[k]) {
                            t = baseK[k] + vb + (uint32_t)__builtin_ctz(bK[k]);
                            bK[k] &= bK[k] - 1u;
                            took = true;
                        }
                        any |= bK[k];
                    }
                    hit(t);
                }
                gp.mark(4);
            }
            wave_lds_sync(); /* the window is read before the next one overwrites it */
        }
    }
    /* lanes whose radius exceeds the grid's design radius, and the lanes
     * of incoherent tiles, scan their own cells from global memory */
    TILE_STAT(4, __builtin_popcountll(__ballot(direct)));
    if (NN) {
        if (dx < 0x1p53 && dy < 0x1p53 && dz < 0x1p53) { /* NaN / inf fail: int64 path */
            Lf.x = d2ll(dx); Lf.y = d2ll(dy); Lf.z = d2ll(dz);
        } else if (small) { /* inexact (or NaN): this record again in int64 */
            M = 0;
            direct = true;
        }
    }
    gp.mark(4);
    /* Direct lanes with a small box whose cells hold few photons in all (an
     * incoherent tile's lanes no group took, C3: ~12 per wave, ~20 photons
     * each): the whole wave scans each one's cells in turn, 64 photons per
     * load. Many photons (a dense union's group, C5; a tile of unrelated
     * surfaces at a depth edge): each lane its own, side by side — the
     * cooperative scan's time grows with the sum over the lanes, the
     * per-lane scans' with the largest lane. */
    if (__ballot(direct)) {
        const bool cand = direct && small;
        uint32_t own = 0u;
        if (cand) { /* every row of the lane's box (up to KR x KR with finer cells) */
            for (uint32_t cz = R.z0; cz <= R.z1; ++cz)
                for (uint32_t cy = R.y0; cy <= R.y1; ++cy) {
                    const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
                    own += P.cell_start[row + R.x1 + 1u] - P.cell_start[row + R.x0];
                }
        }
        const uint32_t tot = uniform_u32(__builtin_amdgcn_readlane(wave_incl_sum_u32(own), 63));
#ifdef PM_COOP_STATS
        const uint32_t nc = (uint32_t)__builtin_popcountll(__ballot(cand)), nd = (uint32_t)__builtin_popcountll(__ballot(direct));
        if (lane == 0 && P.counters) {
            atomicAdd(&P.counters[8], 1ull); atomicAdd(&P.counters[9], (unsigned long long)nc);
            atomicAdd(&P.counters[10], (unsigned long long)tot); atomicMax(&P.counters[11], (unsigned long long)tot);
            atomicAdd(&P.counters[12], (unsigned long long)nd);
            if (nc > 16) { atomicAdd(&P.counters[13], 1ull); atomicAdd(&P.counters[14], (unsigned long long)tot); }
            atomicMax(&P.counters[15], (unsigned long long)nc);
        }
#endif
        if (tot <= (uint32_t)P.coop_steps * 64u) {
            bool sel = cand;
            coop_batch(P, T, lane, R, sel, M, Lf);
            direct = direct && !cand;
        }
    }
    if (direct) lane_scan<0>(P, R.p, R.r2, R.ns, R.fv, R.x0, R.x1, R.y0, R.y1, R.z0, R.z1, M, Lf, nv, nr);
    gp.mark(5);
    R.store<PARTIAL>(P, r, M, Lf);
    if (!PARTIAL && P.r2hist) r2_histogram(P, R.live, R.st.w);
    if (COST && lane == 0)
        P.tile_cost[w] = (uint16_t)min(__builtin_amdgcn_s_memrealtime() - tc0, 65535ull);
    gp.mark(6);
    gp.flush(P.counters);
#ifdef PM_TILE_TIMES
    if (P.tile_times && lane == 0) {
        uint32_t xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned long long *o = P.tile_times + 8 * (size_t)blockIdx.x;
        o[0] = tt0; o[1] = __builtin_amdgcn_s_memrealtime(); o[2] = xcc; o[3] = hw;
        /* groups | windows << 32, test pairs | hit iterations << 32, direct lanes | chunks << 32, staged | record << 32 */
        o[4] = tstat[0] | ((unsigned long long)tstat[1] << 32);
        o[5] = tstat[2] | ((unsigned long long)tstat[3] << 32);
        o[6] = tstat[4] | ((unsigned long long)tstat[5] << 32);
        o[7] = tstat[7] | ((unsigned long long)(r - lane) << 32);
    }
#endif
}

/* ---------------------------------------------------------------------- */
/* kNN estimator: pbrt-v2 PhotonIntegrator::LPhoton (integrators/photonmap.cpp,
 * diffuse branch) with PhotonProcess / KdTree::Lookup semantics, over the
 * photon buckets. Per record (one lane), the found set is the K photons with
 * the smallest keys (d^2, slot) among those with d^2 < maxD2 — the set pbrt's
 * lookup finds, up to the order among photons at exactly equal d^2, where
 * the lower slot wins here and the first visited in pbrt. r_k^2 = the K-th
 * smallest d^2 once K were found (pbrt's shrunk maxDistSquared), else maxD2.
 *     S = sum over found photons with Dot(Nf, wi) > 0 of
 *         (3/pi (1 - d^2/r_k^2)^2 / r_k^2) * alpha        (kernel(), photonmap.cpp)
 * with Nf = Faceforward(ns, wo) (PM_REC_BACKFACE).
 * Two passes over the buckets: (1) a max-heap of d^2 values alone (4 B per
 * entry, LDS columns [K][64]) finds r_k^2; (2) a rescan bounded by r_k^2 sums
 * the photons with d^2 < r_k^2 and, of those at exactly r_k^2, the lowest
 * slots (slot ids ride in ph_b; a third scan runs only when more ties than
 * places exist). The sum is exact and order-free: integer-valued terms
 * in the record's fixed point (scale: the power of two below knn_fx * r_k^2,
 * every term <= 2^22) added in int32 (Kx3). Fused record update: flux += S, radius2 = r_k^2,
 * photon_count = found; the final pass applies 1/paths and rho/pi = Kd/pi
 * (k_final). Both passes visit rows in rings around the query's row,
 * nearest first, and skip rows / cells beyond the current bound. */
PMD float sq(float x) { return x * x; }
/* kNN sums: each term round(c * sc) is an integer <= 2^22
 * (knn_fx), at most PM_KNN_MAX = 2^6 of them per record, so their int32 sum
 * is exact (< 2^28): order-free like the PPM gather's int64 fixed point, at
 * one rounding, one conversion and one integer add per channel (round 4
 * summed terms <= 2^47 in double: two double-rate operations per term; the
 * scalar-stream SUM pass is 41 % of the kNN gather) */
struct Kx3 { int x, y, z; };
/* a kNN term to the nearest integer, floor(x + 0.5) in one instruction
 * (v_cvt_rpi_i32_f32): an error of at most half a unit of the record's fixed
 * point per term, without the one-sided bias of truncation (round 6) */
PMD int knn_rnd(float x) {
    int r;
    asm("v_cvt_rpi_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
/* Dot(Faceforward(ns, wo), wi) > 0 for the photon's wi = (wx, b.w, wz) */
PMD bool knn_facing(v3 ns, bool back, const float4 &b, float wx, float wz) {
    float dn = dot(ns, mk(wx, b.w, wz));
    if (back) dn = -dn;
    return dn > 0.f;
}
/* pbrt kernel() 3/pi (1 - d^2/r_k^2)^2 / r_k^2 times alpha, inv = 1/r_k^2,
 * in the record's fixed point sc */
PMD void knn_add(Kx3 &a, float d2, float inv, float sc, const float4 &b) {
    const float s = 1.f - d2 * inv;
    const float kk = 3.f * INV_PI * s * s;
    /* sc is a power of two: k * (inv * sc) * alpha rounds like (k * inv * alpha) * sc;
     * terms are rounded to the nearest integer (knn_rnd: <= 1/2 unit each) */
    const float ks = kk * (inv * sc);
    a.x += knn_rnd(ks * b.x); a.y += knn_rnd(ks * b.y); a.z += knn_rnd(ks * b.z);
}
/* distance, in cell units, from coordinate u (cell units) to cell c of an
 * axis with dim cells — the border cells extend to infinity (cell_axis
 * clamps) — less a 1e-3 margin that covers the float rounding of u and of the
 * photons' own d^2, so pruning with it never drops a photon that counts */
PMD float cell_gap(float u, uint32_t c, int dim) {
    const float lo = c == 0 ? -INFINITY : (float)c, hi = (int)c + 1 == dim ? INFINITY : (float)(c + 1);
    return fmaxf(fmaxf(lo - u, u - hi) - 1e-3f, 0.f);
}
/* max-heap of d^2 bits in LDS columns: entry k of this lane at h[k * KNN_BLOCK] */
PMD void heap_push(uint32_t *h, int n, uint32_t d) {
    int i = n;
    while (i > 0) {
        const int pa = (i - 1) >> 1;
        const uint32_t pd = h[pa * KNN_BLOCK];
        if (pd >= d) break;
        h[i * KNN_BLOCK] = pd;
        i = pa;
    }
    h[i * KNN_BLOCK] = d;
}
PMD void heap_replace_top(uint32_t *h, int n, uint32_t d) {
    int i = 0;
    while (true) {
        int c = 2 * i + 1;
        if (c >= n) break;
        uint32_t cd = h[c * KNN_BLOCK];
        if (c + 1 < n) {
            const uint32_t rd = h[(c + 1) * KNN_BLOCK];
            if (rd > cd) { c = c + 1; cd = rd; }
        }
        if (d >= cd) break;
        h[i * KNN_BLOCK] = cd;
        i = c;
    }
    h[i * KNN_BLOCK] = d;
}

/* the bucket rows around p within sqrt(maxd2), nearest rings first; bound()
 * (in world units^2) is re-read per row; visit(j, d2) per photon of the kept
 * cells. Returns nothing; COUNT census through vis / rows. */
struct KnnGrid {
    GridDesc g; /* a copy: a pointer into the kernel arguments would force them into scratch */
    uint32_t x0, x1, y0, y1, z0, z1;
    int cyc, czc, rings;
    float ux, uy, uz, inv2;
    PMD void init(const GridDesc &G, v3 p, float maxd2) {
        g = G;
        const float rq = sqrtf(maxd2) * 1.0001f + 1e-4f;
        x0 = cell_axis(p.x - rq, G.gx, G.inv_cs, G.dx); x1 = cell_axis(p.x + rq, G.gx, G.inv_cs, G.dx);
        y0 = cell_axis(p.y - rq, G.gy, G.inv_cs, G.dy); y1 = cell_axis(p.y + rq, G.gy, G.inv_cs, G.dy);
        z0 = cell_axis(p.z - rq, G.gz, G.inv_cs, G.dz); z1 = cell_axis(p.z + rq, G.gz, G.inv_cs, G.dz);
        cyc = (int)cell_axis(p.y, G.gy, G.inv_cs, G.dy); czc = (int)cell_axis(p.z, G.gz, G.inv_cs, G.dz);
        /* the query point in cell units (cell_axis before the floor) */
        ux = (p.x - G.gx) * G.inv_cs; uy = (p.y - G.gy) * G.inv_cs; uz = (p.z - G.gz) * G.inv_cs;
        inv2 = G.inv_cs * G.inv_cs;
        rings = max((int)(y1 - y0), (int)(z1 - z0));
    }
    template <class B, class V>
    PMD void scan(const uint32_t *cell_start, const float4 *ph_a, v3 p, B bound, V visit, unsigned long long &vis,
                  unsigned long long &rows) const {
        for (int ring = 0; ring <= rings; ++ring)
            for (uint32_t cz = z0; cz <= z1; ++cz)
                for (uint32_t cy = y0; cy <= y1; ++cy) {
                    if (max(abs((int)cy - cyc), abs((int)cz - czc)) != ring) continue;
                    const float gy = cell_gap(uy, cy, g.dy), gz = cell_gap(uz, cz, g.dz);
                    const float lim = bound() * inv2 - (gy * gy + gz * gz);
                    if (lim < 0.f) continue;
                    uint32_t xa = x0, xb = x1;
                    while (xa <= xb && sq(cell_gap(ux, xa, g.dx)) > lim) ++xa;
                    while (xb > xa && sq(cell_gap(ux, xb, g.dx)) > lim) --xb;
                    if (xa > xb) continue;
                    const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
                    const uint32_t b = cell_start[row + xa], e = cell_start[row + xb + 1];
                    vis += e - b; rows++;
                    for (uint32_t j = b; j < e; ++j) {
                        const float4 a = ph_a[j];
                        const v3 diff = p - xyz(a);
                        visit(j, a, diff.x * diff.x + diff.y * diff.y + diff.z * diff.z);
                    }
                }
    }
};

template <int COUNT>
__global__ __launch_bounds__(KNN_BLOCK) void k_gather_knn(GatherParams P) {
    extern __shared__ uint32_t kheap[]; /* [K][KNN_BLOCK] d^2 bits */
    const int K = P.knn_k;
    uint32_t *h = kheap + threadIdx.x;
    const int64_t r = P.rec_begin + (int64_t)blockIdx.x * KNN_BLOCK + threadIdx.x;
    unsigned long long vis = 0, hits = 0, rows = 0, act = 0;
    if (r < P.rec_end) {
        const float4 pos = P.R.pos[r];
        const uint32_t flags = (uint32_t)__float_as_int(pos.w);
        if (!(flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID))) {
            float4 st = P.fresh ? make_float4(0.f, 0.f, 0.f, P.r2init) : P.R.state[r];
            const float4 nrm = P.R.nrm[r];
            const float4 m = P.materials[__float_as_int(nrm.w)];
            const float maxd2 = P.knn_r2;
            const v3 p = xyz(pos), ns = xyz(nrm);
            int cnt = 0;
            float md2 = maxd2;
            Kx3 acc{0, 0, 0};
            float sc = 1.f;
            bool nan = false;
            if (__float_as_int(m.w) == PM_MATTE) { /* non-specular BSDF components only */
                KnnGrid G;
                G.init(P.grid, p, maxd2);
                /* pass 1: r_k^2 */
                uint32_t topd = 0xffffffffu;
                G.scan(P.cell_start, P.ph_a, p, [&]() { return cnt == K ? __uint_as_float(topd) : maxd2; },
                       [&](uint32_t, const float4 &, float d2) {
                           if (!(d2 < maxd2)) return;
                           const uint32_t db = __float_as_uint(d2); /* d2 >= 0: bits order = value order */
                           if (cnt < K) {
                               heap_push(h, cnt, db);
                               if (++cnt == K) topd = h[0];
                           } else if (db < topd) {
                               heap_replace_top(h, K, db);
                               topd = h[0];
                           }
                       }, vis, rows);
                const bool full = cnt == K;
                if (full) md2 = __uint_as_float(topd);
                sc = md2 == 0.f ? 1.f : __uint_as_float(__float_as_uint(P.knn_fx * md2) & 0xff800000u); /* 2^n: exact */
                const bool back = (flags & PM_REC_BACKFACE) != 0;
                const float *phb = reinterpret_cast<const float *>(P.ph_b);
                /* contribution of photon j (LPhoton term) into a */
                const float inv = 1.f / md2;
                auto add = [&](Kx3 &a, uint32_t j, const float4 &pa, float d2) {
                    const float4 b0 = P.ph_b[2 * (size_t)j];
                    if (!knn_facing(ns, back, b0, pa.w, phb[8 * (size_t)j + 4])) return;
                    if (md2 == 0.f) { nan = true; return; } /* K photons at distance 0: kernel() is 0/0 */
                    knn_add(a, d2, inv, sc, b0);
                };
                /* pass 2: every photon below r_k^2 (all below maxD2 when not full);
                 * ties at r_k^2 aside */
                int less = 0, ties = 0;
                Kx3 acc_eq{0, 0, 0};
                G.scan(P.cell_start, P.ph_a, p, [&]() { return md2; },
                       [&](uint32_t j, const float4 &pa, float d2) {
                           if (d2 < md2) { less++; add(acc, j, pa, d2); }
                           else if (full && d2 == md2) { ties++; add(acc_eq, j, pa, d2); }
                       }, vis, rows);
                const int need = full ? K - less : 0;
                if (ties == need) {
                    acc.x += acc_eq.x; acc.y += acc_eq.y; acc.z += acc_eq.z;
                } else {
                    /* more photons at exactly r_k^2 than places: the lowest slots (rare) */
                    uint32_t last = 0u;
                    bool first = true;
                    for (int t = 0; t < need; ++t) {
                        uint32_t best = 0xffffffffu, bj = 0u;
                        float4 ba = make_float4(0.f, 0.f, 0.f, 0.f);
                        G.scan(P.cell_start, P.ph_a, p, [&]() { return md2; },
                               [&](uint32_t j, const float4 &pa, float d2) {
                                   if (d2 != md2) return;
                                   const uint32_t sl = __float_as_uint(phb[8 * (size_t)j + 5]);
                                   if ((first || sl > last) && sl <= best) { best = sl; bj = j; ba = pa; }
                               }, vis, rows);
                        add(acc, bj, ba, md2);
                        last = best;
                        first = false;
                    }
                }
                cnt = full ? K : less;
            }
            if (COUNT) { hits += (unsigned long long)cnt; act++; }
            const double isc = 1.0 / (double)sc;
            v3 L = mk((float)((double)acc.x * isc), (float)((double)acc.y * isc), (float)((double)acc.z * isc));
            if (nan) L = mk(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
            const v3 flux = xyz(st) + L;
            P.R.state[r] = make_float4(flux.x, flux.y, flux.z, md2);
            P.R.n[r] = (float)cnt;
        }
    }
    if (COUNT) count4(P.counters, vis, hits, rows, act);
}

/* ---------------------------------------------------------------------- */
/* kNN tile kernel (default kNN path): k_gather_knn's estimate, bit for bit
 * (same found set, r_k^2, per-record scale and exact sums), for the 64
 * records of an 8x8 tile at once.
 *  - Photon source: the wave stages the union of its lanes' bucket rows (each
 *    lane's box [p - maxD, p + maxD]) into LDS windows of KT_CAP photons with
 *    coalesced loads, as k_gather_tile does; every lane tests every staged
 *    photon against its own d^2 interval. The union is a superset of each
 *    lane's cells and anything at d^2 >= maxD^2 is dropped, so the found set
 *    is unchanged, and the scan loop is wave-uniform instead of 64 lanes
 *    walking their own rows with a divergent heap.
 *  - r_k^2 without a heap: the K-th smallest d^2 is selected exactly by
 *    passes over the same photons. HIST counts each lane's photons of its
 *    interval into 32 bins of a monotone bin function (float subtract,
 *    multiply, clamp, truncate: every step is monotone, so a bin is an
 *    interval of d^2 values) with one LDS add per photon; a prefix walk finds
 *    the bin holding the K-th. COLLECT then keeps that bin's values (<= 12,
 *    in LDS) with their min and max: <= 12 values are ranked directly, equal
 *    values are the answer, otherwise [min, max] is re-binned (the extremes
 *    land in bins 0 and 31, so every level shrinks the set). A deep or
 *    overflowing (>= 2^16 photons) search extracts minima one by one instead.
 *    A record with < K photons inside maxD (r_k^2 = maxD^2) goes from level
 *    0's HIST straight to its SUM pass.
 *  - HIST counts inline in the test loop (no per-hit loop); COLLECT, MIN and
 *    SUM lanes take their hits one per lane per iteration, COLLECT over the
 *    chosen bin's d^2 range only (conservative float bounds, exact bin test).
 *  - Incoherent tiles: k_gather_tile's groups (leader neighbourhoods); lanes
 *    left over in groups of < KT_GROUP_MIN run the same passes over their own
 *    rows from global memory. */
#ifndef PM_KT_CAP
#define PM_KT_CAP 64
#endif
/* C2 kNN: 12 -> 1.07 ms, 4 -> 0.99, 1 -> 0.95: every lane gets an LDS group
 * (its own if need be); per-lane passes remain for grids too coarse for the
 * row map */
#ifndef PM_KT_GROUP_MIN
#define PM_KT_GROUP_MIN 1
#endif
constexpr int KT_CAP = PM_KT_CAP;  /* photons per LDS window (one per lane) */
/* bins / kept values (C2 kNN, ms): 64/8 1.25, 48/8 1.12, 32/16 1.10, 24/12
 * 1.08, 32/10 1.07, 32/12 1.03 — 32/12 keeps the LDS at ~9.8 KB per wave
 * (4 waves/SIMD, the VGPR limit) with few re-binning passes */
#ifndef PM_KT_BINS
#define PM_KT_BINS 32
#endif
#ifndef PM_KT_PIPE
#define PM_KT_PIPE 1
#endif
constexpr int KT_BINS = PM_KT_BINS; /* histogram bins per pass */
#ifndef PM_KT_LIST
#define PM_KT_LIST 12
#endif
constexpr int KT_LIST = PM_KT_LIST; /* values a COLLECT pass keeps per lane */
constexpr int KT_LEVELS = 4;       /* re-binning levels before minimum extraction */
constexpr uint32_t KT_GROUP_R = 1; /* lane boxes span <= 5 cells: a group's union <= 7 per axis */
constexpr int KT_GROUP_MIN = PM_KT_GROUP_MIN;
struct KnnLds {
    float x[KT_CAP + 4], y[KT_CAP + 4], z[KT_CAP + 4]; /* +4: the pair test reads one past the window */
    float4 b[KT_CAP];                                   /* alpha.rgb, wi.y */
    float w[KT_CAP], c[KT_CAP];                         /* wi.x, wi.z */
    int mark[KT_CAP];
    uint32_t hist[KT_BINS / 2][64]; /* two 16-bit counters per word, a column per lane */
    uint32_t list[KT_LIST][64];
};
#define PM_INLINE __attribute__((always_inline))
enum { KP_DONE = 0, KP_HIST = 1, KP_COLLECT = 2, KP_MIN = 3, KP_SUM = 4 };
PMD float next_up(float x) { return __uint_as_float(__float_as_uint(x) + 1u); } /* x >= 0, finite */
/* wave-uniform vector loads through the scalar cache (k_gather_knn_ss) */
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef const f32x16 __attribute__((address_space(4), aligned(4))) sv16;
typedef const f32x8 __attribute__((address_space(4), aligned(4))) sv8;
/* per-record fixed-point scale: the power of two below knn_fx * r_k^2 */
PMD float knn_scale(float fx, float md2) {
    return md2 == 0.f ? 1.f : __uint_as_float(__float_as_uint(fx * md2) & 0xff800000u);
}
/* one lane's selection state */
struct KnnSel {
    int phase = KP_DONE, level = 0, need = 0, kbin = 0;
    float blo = INFINITY, bhi = 0.f; /* this pass's hit interval [blo, bhi) */
    float lo = 0.f, s = 0.f;         /* bin function of HIST / COLLECT */
    uint32_t cntf = 0, cc = 0, tcnt = 0;
    float mn = INFINITY, mx = 0.f, tmin = INFINITY;
    float md2 = 0.f, sc = 1.f;
    int less = 0, ties = 0, cnt = 0;
    bool full = true, tiefix = false, nan = false, nan_eq = false;
    float inv = 0.f; /* 1 / r_k^2 */
    Kx3 acc{0, 0, 0};
    PMD int bin(float d2) const { return (int)fminf((d2 - lo) * s, (float)(KT_BINS - 1)); }
};

__global__ __launch_bounds__(KNN_BLOCK) void k_gather_knn_tile(GatherParams P) {
#ifdef PM_TILE_TIMES
    uint32_t tstat[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* TILE_STAT's sink (unused here) */
    (void)tstat;
#endif
    __shared__ KnnLds L;
    const int lane = threadIdx.x & 63;
    if (P.tiles && P.n_tiles_dev && (int64_t)blockIdx.x >= (int64_t)*P.n_tiles_dev) return; /* one wave per block */
    const int64_t r = P.rec_begin + (P.tiles ? (int64_t)P.tiles[blockIdx.x] * 64 + lane
                                             : (int64_t)blockIdx.x * KNN_BLOCK + threadIdx.x);
    const GridDesc &g = P.grid;
    GProf gp; /* PM_GATHER_PROFILE: record, pass setup, stage, test, hits, pass end, direct + store */
    gp.begin();
    const int K = P.knn_k;
    const float maxd2 = P.knn_r2;
#pragma unroll
    for (int w = 0; w < KT_BINS / 2; ++w) L.hist[w][lane] = 0u;
    /* record */
    bool active = false, live = false, back = false;
    float4 pos = make_float4(0.f, 0.f, 0.f, 0.f), nrm = pos;
    if (r < P.rec_end) {
        pos = P.R.pos[r];
        const uint32_t flags = (uint32_t)__float_as_int(pos.w);
        active = !(flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID));
        back = (flags & PM_REC_BACKFACE) != 0;
        if (active) {
            nrm = P.R.nrm[r];
            live = __float_as_int(P.materials[__float_as_int(nrm.w)].w) == PM_MATTE; /* non-specular BSDF only */
        }
    }
    const v3 p = xyz(pos), ns = xyz(nrm);
    uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0, z0 = 0, z1 = 0;
    if (live) { /* KnnGrid::init's cells */
        const float rq = sqrtf(maxd2) * 1.0001f + 1e-4f;
        x0 = cell_axis(p.x - rq, g.gx, g.inv_cs, g.dx); x1 = cell_axis(p.x + rq, g.gx, g.inv_cs, g.dx);
        y0 = cell_axis(p.y - rq, g.gy, g.inv_cs, g.dy); y1 = cell_axis(p.y + rq, g.gy, g.inv_cs, g.dy);
        z0 = cell_axis(p.z - rq, g.gz, g.inv_cs, g.dz); z1 = cell_axis(p.z + rq, g.gz, g.inv_cs, g.dz);
    }
    KnnSel S;
    if (live) { S.phase = KP_HIST; S.need = K; S.blo = 0.f; S.bhi = maxd2; S.s = (float)KT_BINS / maxd2; }
    if (live && !(S.s <= 3.402823466e38f)) S.s = 3.402823466e38f;

    /* contribution of a found photon (pbrt kernel(), LPhoton diffuse term) into
     * a; returns true when it is pbrt's 0/0 (K photons at distance 0) */
    auto contrib = [&](Kx3 &a, float d2, const float4 &b, float wx, float wz) PM_INLINE {
        if (!knn_facing(ns, back, b, wx, wz)) return false;
        if (S.md2 == 0.f) return true;
        knn_add(a, d2, S.inv, S.sc, b);
        return false;
    };
    /* a photon inside this pass's interval; fl() -> its (b, wi.x, wi.z) */
    auto on_hit = [&](float d2, auto fl) PM_INLINE {
        switch (S.phase) {
        case KP_HIST: { /* per-lane passes only: the tile passes count inline */
            const int b = S.bin(d2);
            atomicAdd(&L.hist[b >> 1][lane], 1u << ((b & 1) * 16));
            S.cntf++;
            break;
        }
        case KP_COLLECT:
            if (S.bin(d2) == S.kbin) {
                if (S.cc < (uint32_t)KT_LIST) L.list[S.cc][lane] = __float_as_uint(d2);
                S.cc++;
                S.mn = fminf(S.mn, d2);
                S.mx = fmaxf(S.mx, d2);
            }
            break;
        case KP_MIN:
            if (d2 < S.tmin) { S.tmin = d2; S.tcnt = 1u; }
            else if (d2 == S.tmin) S.tcnt++;
            break;
        case KP_SUM: {
            float4 fb; float wx, wz;
            fl(fb, wx, wz);
            if (d2 < S.md2) { S.less++; S.nan |= contrib(S.acc, d2, fb, wx, wz); }
            else { /* d2 == r_k^2 (full lookups): the kernel is 0 there; only pbrt's 0/0 matters */
                S.ties++;
                if (S.md2 == 0.f) S.nan_eq |= knn_facing(ns, back, fb, wx, wz);
            }
            break;
        }
        default: break;
        }
    };
    auto begin_sum = [&]() PM_INLINE {
        S.sc = knn_scale(P.knn_fx, S.md2);
        S.inv = 1.f / S.md2;
        S.acc = Kx3{0, 0, 0};
        S.less = S.ties = 0;
        S.nan = S.nan_eq = false;
        S.blo = 0.f; S.bhi = S.full ? next_up(S.md2) : S.md2; /* not full: every d^2 < maxD^2 */
        S.phase = KP_SUM;
    };
    auto begin_min = [&](float lo_incl, float hi_excl) PM_INLINE {
        S.blo = lo_incl; S.bhi = hi_excl;
        S.tmin = INFINITY; S.tcnt = 0u;
        S.phase = KP_MIN;
    };
    /* end of a pass: the next phase */
    auto finish = [&]() PM_INLINE {
        switch (S.phase) {
        case KP_HIST: {
            if (S.level == 0) {
                if (S.cntf < (uint32_t)K) { /* fewer than K inside maxD: r_k^2 = maxD^2 */
                    S.full = false;
                    S.md2 = maxd2;
                    begin_sum();
                    break;
                }
                if (S.cntf >= 65536u) { begin_min(0.f, maxd2); break; } /* 16-bit bins may have wrapped */
            }
            uint32_t cum = 0u;
            bool found = false;
#pragma unroll
            for (int w = 0; w < KT_BINS / 2; ++w) {
                const uint32_t hw = L.hist[w][lane];
                L.hist[w][lane] = 0u;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint32_t c = (hw >> (16 * h)) & 0xffffu;
                    if (!found && cum + c >= (uint32_t)S.need) { found = true; S.kbin = 2 * w + h; }
                    else if (!found) cum += c;
                }
            }
            S.need -= (int)cum;
            S.cc = 0u; S.mn = INFINITY; S.mx = 0.f;
            /* the bin's d^2 range, widened: (d2 - lo) * s is within 2^-23
             * relative of exact, so bin k lies in lo + [k - 0.01, k + 1.01) / s,
             * and two ulps cover the rounding of that bound */
            if (S.kbin > 0) {
                const float cl = S.lo + ((float)S.kbin - 0.01f) / S.s;
                S.blo = fmaxf(S.blo, __uint_as_float(max((int)__float_as_uint(cl) - 2, 0)));
            }
            if (S.kbin < KT_BINS - 1) {
                const float ch = S.lo + ((float)S.kbin + 1.01f) / S.s;
                if (ch < 3.0e38f) S.bhi = fminf(S.bhi, next_up(next_up(ch)));
            }
            S.phase = KP_COLLECT; /* same bin function, exact bin test per hit */
            break;
        }
        case KP_COLLECT:
            if (S.cc <= (uint32_t)KT_LIST) { /* rank the kept values: the need-th smallest */
                uint32_t v[KT_LIST];
#pragma unroll
                for (int a = 0; a < KT_LIST; ++a) v[a] = (uint32_t)a < S.cc ? L.list[a][lane] : 0xffffffffu;
                uint32_t ans = v[0];
#pragma unroll
                for (int a = 0; a < KT_LIST; ++a) {
                    int lt = 0, le = 0;
#pragma unroll
                    for (int b = 0; b < KT_LIST; ++b) { lt += v[b] < v[a]; le += v[b] <= v[a]; }
                    if ((uint32_t)a < S.cc && lt < S.need && S.need <= le) ans = v[a];
                }
                S.md2 = __uint_as_float(ans);
                begin_sum();
            } else if (S.mn == S.mx) {
                S.md2 = S.mn;
                begin_sum();
            } else if (S.level >= KT_LEVELS) {
                begin_min(S.mn, next_up(S.mx));
            } else { /* re-bin [mn, mx] */
                S.level++;
                S.lo = S.mn;
                S.s = (float)KT_BINS / (S.mx - S.mn);
                if (!(S.s <= 3.402823466e38f)) S.s = 3.402823466e38f;
                S.blo = S.mn; S.bhi = next_up(S.mx);
                S.cntf = 0u;
                S.phase = KP_HIST;
            }
            break;
        case KP_MIN:
            if (S.tcnt == 0u || S.tcnt >= (uint32_t)S.need) { S.md2 = S.tcnt ? S.tmin : maxd2; begin_sum(); }
            else { S.need -= (int)S.tcnt; begin_min(next_up(S.tmin), S.bhi); }
            break;
        case KP_SUM:
            if (S.full) {
                /* K found: those below r_k^2 and K - less of the ties; the ties
                 * add 0 unless r_k^2 = 0, where the selected ones decide the NaN */
                if (S.ties == K - S.less) S.nan |= S.nan_eq;
                else if (S.md2 == 0.f) S.tiefix = true;
                S.cnt = K;
            } else {
                S.cnt = S.less;
            }
            S.phase = KP_DONE;
            break;
        default: break;
        }
    };

    const f2 px2 = {p.x, p.x}, py2 = {p.y, p.y}, pz2 = {p.z, p.z};
    bool pend = live, direct = false;
    gp.mark(0);
    while (true) {
        const unsigned long long pm = __ballot(pend);
        if (pm == 0ull) break;
        /* the group: every pending lane if the union box fits the 64-lane row
         * map, else the leader's neighbourhood (k_gather_tile) */
        uint32_t X0, X1, Y0, Y1, Z0, Z1;
        bool mine = pend;
        union_box6(g, mine, x0, x1, y0, y1, z0, z1, X0, X1, Y0, Y1, Z0, Z1);
        uint32_t LY = Y1 > Y0 ? 32u - (uint32_t)__builtin_clz(Y1 - Y0) : 0u;
        if (LY > 6u || ((uint64_t)(Z1 - Z0 + 1u) << LY) > 64u) {
            const int leader = __builtin_ctzll(pm);
            const uint32_t lx = __builtin_amdgcn_readlane(x0, leader), ly = __builtin_amdgcn_readlane(y0, leader),
                           lz = __builtin_amdgcn_readlane(z0, leader);
            mine = pend && x0 + KT_GROUP_R - lx <= 2u * KT_GROUP_R && y0 + KT_GROUP_R - ly <= 2u * KT_GROUP_R &&
                   z0 + KT_GROUP_R - lz <= 2u * KT_GROUP_R;
            if (__builtin_popcountll(__ballot(mine)) < KT_GROUP_MIN) {
                direct = direct || pend;
                break;
            }
            union_box6(g, mine, x0, x1, y0, y1, z0, z1, X0, X1, Y0, Y1, Z0, Z1);
            LY = Y1 > Y0 ? 32u - (uint32_t)__builtin_clz(Y1 - Y0) : 0u;
            if (LY > 6u || ((uint64_t)(Z1 - Z0 + 1u) << LY) > 64u) { /* a grid too coarse for the bound: per lane */
                direct = direct || pend;
                break;
            }
        }
        pend = pend && !mine;
        TILE_STAT(0, 1);
        /* passes until every lane of the group has its estimate */
        while (__ballot(mine && S.phase != KP_DONE)) {
            const bool act = mine && S.phase != KP_DONE;
            TILE_STAT(1, 1);
            /* this pass's union: the cells of [p - r', p + r'] for r'^2 = the
             * pass's upper bound (after level 0 mostly r_k^2, not maxD^2) —
             * a sub-box of the group's, so it fits the row map as well */
            uint32_t PX0 = X0, PX1 = X1, PY0 = Y0, PY1 = Y1, PZ0 = Z0, PZ1 = Z1, PLY = LY;
            {
                uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0, c0 = 0, c1 = 0;
                if (act) {
                    const float rq = sqrtf(S.bhi) * 1.0001f + 1e-4f;
                    a0 = cell_axis(p.x - rq, g.gx, g.inv_cs, g.dx); a1 = cell_axis(p.x + rq, g.gx, g.inv_cs, g.dx);
                    b0 = cell_axis(p.y - rq, g.gy, g.inv_cs, g.dy); b1 = cell_axis(p.y + rq, g.gy, g.inv_cs, g.dy);
                    c0 = cell_axis(p.z - rq, g.gz, g.inv_cs, g.dz); c1 = cell_axis(p.z + rq, g.gz, g.inv_cs, g.dz);
                }
                uint32_t QX0, QX1, QY0, QY1, QZ0, QZ1;
                union_box6(g, act, a0, a1, b0, b1, c0, c1, QX0, QX1, QY0, QY1, QZ0, QZ1);
                const uint32_t QLY = QY1 > QY0 ? 32u - (uint32_t)__builtin_clz(QY1 - QY0) : 0u;
                if (QLY <= 6u && ((uint64_t)(QZ1 - QZ0 + 1u) << QLY) <= 64u) {
                    PX0 = QX0; PX1 = QX1; PY0 = QY0; PY1 = QY1; PZ0 = QZ0; PZ1 = QZ1; PLY = QLY;
                }
            }
            /* union row u = lane: photons [B, B + len) of cells PX0..PX1 */
            uint32_t B = 0u, len = 0u;
            const uint32_t cy = PY0 + ((uint32_t)lane & ((1u << PLY) - 1u)), cz = PZ0 + ((uint32_t)lane >> PLY);
            if (cy <= PY1 && cz <= PZ1) {
                const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
                B = P.cell_start[row + PX0];
                len = P.cell_start[row + PX1 + 1u] - B;
            }
            const uint32_t incl = wave_incl_sum_u32(len), pre = incl - len;
            const uint32_t U = uniform_u32(__builtin_amdgcn_readlane(incl, 63));
            const uint32_t gofs = B - pre;
            TILE_STAT(6, __builtin_popcountll(__ballot(act && S.phase == KP_MIN)));
            TILE_STAT(7, __builtin_popcountll(__ballot(act && S.phase == KP_HIST && S.level > 0)));
            const float blo = act ? S.blo : INFINITY, bhi = act ? S.bhi : 0.f;
            const bool hl = act && S.phase == KP_HIST; /* counts inline */
            const bool hist_any = __ballot(hl) != 0ull;
            const bool other_any = __ballot(act && !hl) != 0ull;
            /* the sums need the photons' flux and direction */
            const bool flux = __ballot(act && S.phase == KP_SUM) != 0ull;
            const f2 lo2 = {S.lo, S.lo}, s2 = {S.s, S.s};
            uint32_t cntf = 0u;
            auto window = [&](uint32_t n, auto DO_HIST, auto DO_OTHER) PM_INLINE {
                /* every lane tests every staged photon, two per packed step,
                 * 32 at a time: HIST lanes count them into their histogram on
                 * the spot, the others collect a hit mask and then take the
                 * hits one per lane per iteration */
                for (uint32_t vb = 0; vb < n; vb += 32) {
                    const uint32_t cnt = min(32u, n - vb);
                    uint32_t bits = 0u;
#pragma unroll 4
                    for (uint32_t j = 0; j < cnt; j += 2) {
                        const f2 ddx = px2 - f2{L.x[vb + j], L.x[vb + j + 1]}, ddy = py2 - f2{L.y[vb + j], L.y[vb + j + 1]},
                                 ddz = pz2 - f2{L.z[vb + j], L.z[vb + j + 1]};
                        const f2 d2 = (ddx * ddx + ddy * ddy) + ddz * ddz;
                        const bool hx = d2.x >= blo && d2.x < bhi && j < cnt, hy = d2.y >= blo && d2.y < bhi && j + 1 < cnt;
                        if (decltype(DO_HIST)::value) {
                            if (hl) {
                                /* S.bin of both, packed: the same IEEE operations.
                                 * Branch-free: a miss adds 0 to bin 0 */
                                const f2 bb = (d2 - lo2) * s2;
                                const int b0 = hx ? (int)fminf(bb.x, (float)(KT_BINS - 1)) : 0;
                                const int b1 = hy ? (int)fminf(bb.y, (float)(KT_BINS - 1)) : 0;
#ifdef PM_KT_BRANCHY
                                if (hx) atomicAdd(&L.hist[b0 >> 1][lane], 1u << ((b0 & 1) * 16));
                                if (hy) atomicAdd(&L.hist[b1 >> 1][lane], 1u << ((b1 & 1) * 16));
#else
                                atomicAdd(&L.hist[b0 >> 1][lane], (uint32_t)hx << ((b0 & 1) * 16));
                                atomicAdd(&L.hist[b1 >> 1][lane], (uint32_t)hy << ((b1 & 1) * 16));
#endif
                                cntf += (uint32_t)hx + (uint32_t)hy;
                            }
                        }
                        if (decltype(DO_OTHER)::value) {
                            if (hx) bits |= 1u << j;
                            if (hy) bits |= 2u << j;
                        }
                    }
                    gp.mark(3);
                    if (decltype(DO_OTHER)::value) {
                        if (hl) bits = 0u;
                        TILE_STAT(4, wave_max_u32(__builtin_popcount(bits)));
                        while (bits) {
                            const uint32_t t = vb + (uint32_t)__builtin_ctz(bits);
                            bits &= bits - 1u;
                            const v3 diff = p - mk(L.x[t], L.y[t], L.z[t]);
                            const float d2 = diff.x * diff.x + diff.y * diff.y + diff.z * diff.z;
                            on_hit(d2, [&](float4 &fb, float &wx, float &wz) PM_INLINE { fb = L.b[t]; wx = L.w[t]; wz = L.c[t]; });
                        }
                    }
                }
            };
            gp.mark(1);
#if PM_KT_PIPE
            /* software-pipelined staging (one photon per lane per window):
             * the next window's positions are requested before this window
             * is written to LDS and tested, so a window's load round trip
             * overlaps the previous window's tests; the flux words (SUM
             * passes only) are requested at the start of their own window */
            static_assert(KT_CAP == 64, "pipelined staging: one photon per lane per window");
            const float *phb = reinterpret_cast<const float *>(P.ph_b);
            /* photon index of this lane's position in window T0: its row from
             * a max scan over the row-start marks; past the union -> the
             * window's first photon (never read) */
            auto window_index = [&](uint32_t T0) PM_INLINE {
                L.mark[lane] = -1;
                wave_lds_sync();
                if (len > 0u) {
                    if (pre >= T0 && pre < T0 + KT_CAP) L.mark[pre - T0] = lane;
                    else if (pre < T0 && pre + len > T0) L.mark[0] = lane;
                }
                wave_lds_sync();
                const int u = wave_incl_max_i32(L.mark[lane]);
                const uint32_t gi = T0 + (uint32_t)lane + (uint32_t)__shfl((int)gofs, u);
                const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gi, 0);
                return (uint32_t)lane < min((uint32_t)KT_CAP, U - T0) ? gi : g0;
            };
            uint32_t jn = U > 0u ? window_index(0u) : 0u;
            float4 pan = U > 0u ? P.ph_a[jn] : make_float4(0.f, 0.f, 0.f, 0.f);
            for (uint32_t T0 = 0; T0 < U; T0 += KT_CAP) {
                const uint32_t n = min((uint32_t)KT_CAP, U - T0);
                TILE_STAT(2, 1);
                TILE_STAT(3, n);
                const uint32_t j = jn;
                const float4 pa = pan;
                float4 qa = make_float4(0.f, 0.f, 0.f, 0.f);
                float ca = 0.f;
                if (flux) { qa = P.ph_b[2 * (size_t)j]; ca = phb[8 * (size_t)j + 4]; }
                if (T0 + KT_CAP < U) {
                    jn = window_index(T0 + KT_CAP);
                    pan = P.ph_a[jn];
                }
                L.x[lane] = pa.x; L.y[lane] = pa.y; L.z[lane] = pa.z;
                if (flux) { L.w[lane] = pa.w; L.b[lane] = qa; L.c[lane] = ca; }
                wave_lds_sync();
                gp.mark(2);
                using T_ = std::true_type;
                using F_ = std::false_type;
                if (hist_any && other_any) window(n, T_{}, T_{});
                else if (hist_any) window(n, T_{}, F_{});
                else window(n, F_{}, T_{});
                gp.mark(4);
                wave_lds_sync(); /* the window is read before the next one overwrites it */
            }
#else
            for (uint32_t T0 = 0; T0 < U; T0 += KT_CAP) {
                const uint32_t n = min((uint32_t)KT_CAP, U - T0);
                TILE_STAT(2, 1);
                TILE_STAT(3, n);
                constexpr int H = KT_CAP / 64;
                /* stage positions T0 + lane + 64 h: the row of each from a max
                 * scan over the row-start marks */
#pragma unroll
                for (int h = 0; h < H; ++h) L.mark[lane + 64 * h] = -1;
                wave_lds_sync();
                if (len > 0u) {
                    if (pre >= T0 && pre < T0 + KT_CAP) L.mark[pre - T0] = lane;
                    else if (pre < T0 && pre + len > T0) L.mark[0] = lane;
                }
                wave_lds_sync();
                int u[H];
                u[0] = wave_incl_max_i32(L.mark[lane]);
#pragma unroll
                for (int h = 1; h < H; ++h) u[h] = max(wave_incl_max_i32(L.mark[lane + 64 * h]), __builtin_amdgcn_readlane(u[h - 1], 63));
                uint32_t gi[H];
#pragma unroll
                for (int h = 0; h < H; ++h) gi[h] = T0 + 64u * h + (uint32_t)lane + (uint32_t)__shfl((int)gofs, u[h]);
                const float *phb = reinterpret_cast<const float *>(P.ph_b);
                const uint32_t g0 = (uint32_t)__builtin_amdgcn_readlane((int)gi[0], 0);
                float4 pa[H], qa[H];
                float ca[H];
#pragma unroll
                for (int h = 0; h < H; ++h) {
                    const uint32_t j = (uint32_t)lane + 64u * h < n ? gi[h] : g0;
                    pa[h] = P.ph_a[j];
                    qa[h] = make_float4(0.f, 0.f, 0.f, 0.f);
                    ca[h] = 0.f;
                    if (flux) { qa[h] = P.ph_b[2 * (size_t)j]; ca[h] = phb[8 * (size_t)j + 4]; }
                }
#pragma unroll
                for (int h = 0; h < H; ++h) {
                    const int q = lane + 64 * h;
                    L.x[q] = pa[h].x; L.y[q] = pa[h].y; L.z[q] = pa[h].z;
                    if (flux) { L.w[q] = pa[h].w; L.b[q] = qa[h]; L.c[q] = ca[h]; }
                }
                wave_lds_sync();
                gp.mark(2);
                using T_ = std::true_type;
                using F_ = std::false_type;
                if (hist_any && other_any) window(n, T_{}, T_{});
                else if (hist_any) window(n, T_{}, F_{});
                else window(n, F_{}, T_{});
                gp.mark(4);
                wave_lds_sync(); /* the window is read before the next one overwrites it */
            }
#endif
            if (hl) S.cntf += cntf;
            if (act) finish();
            gp.mark(5);
        }
    }
    /* lanes of incoherent tiles: the same passes over their own rows */
    TILE_STAT(5, __builtin_popcountll(__ballot(direct)));
    KnnGrid G;
    unsigned long long nv = 0, nr = 0;
    if (__ballot(direct)) {
        if (direct) G.init(P.grid, p, maxd2);
        const float *phb = reinterpret_cast<const float *>(P.ph_b);
        while (__ballot(direct && S.phase != KP_DONE)) {
            if (direct && S.phase != KP_DONE) {
                G.scan(P.cell_start, P.ph_a, p, [&]() { return S.bhi; },
                       [&](uint32_t j, const float4 &a, float d2) {
                           if (!(d2 >= S.blo && d2 < S.bhi)) return;
                           on_hit(d2, [&](float4 &fb, float &wx, float &wz) PM_INLINE {
                               fb = P.ph_b[2 * (size_t)j]; wx = a.w; wz = phb[8 * (size_t)j + 4];
                           });
                       }, nv, nr);
                finish();
            }
        }
    }
    /* r_k^2 = 0 with more photons at the query point than places: the lowest
     * slots are the found ones (k_gather_knn's third scan) */
    if (__ballot(S.tiefix)) {
        if (S.tiefix) {
            if (!direct) G.init(P.grid, p, maxd2);
            const float *phb = reinterpret_cast<const float *>(P.ph_b);
            const int need = K - S.less;
            uint32_t last = 0u;
            bool first = true, nan = false;
            for (int t = 0; t < need; ++t) {
                uint32_t best = 0xffffffffu, bj = 0u;
                float4 ba = make_float4(0.f, 0.f, 0.f, 0.f);
                G.scan(P.cell_start, P.ph_a, p, [&]() { return S.md2; },
                       [&](uint32_t j, const float4 &a, float d2) {
                           if (d2 != S.md2) return;
                           const uint32_t sl = __float_as_uint(phb[8 * (size_t)j + 5]);
                           if ((first || sl > last) && sl <= best) { best = sl; bj = j; ba = a; }
                       }, nv, nr);
                nan |= knn_facing(ns, back, P.ph_b[2 * (size_t)bj], ba.w, phb[8 * (size_t)bj + 4]); /* r_k^2 = 0: 0/0 */
                last = best;
                first = false;
            }
            S.nan |= nan;
        }
    }
    if (active) {
        if (!live) S.md2 = maxd2; /* specular: nothing found, cnt 0 */
        const float4 st = P.fresh ? make_float4(0.f, 0.f, 0.f, P.r2init) : P.R.state[r];
        const double isc = 1.0 / (double)S.sc;
        v3 Lr = mk((float)((double)S.acc.x * isc), (float)((double)S.acc.y * isc), (float)((double)S.acc.z * isc));
        if (S.nan) Lr = mk(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
        const v3 flux = xyz(st) + Lr;
        P.R.state[r] = make_float4(flux.x, flux.y, flux.z, S.md2);
        P.R.n[r] = (float)S.cnt;
    }
    gp.mark(6);
    gp.flush(P.counters);
}

/* ---------------------------------------------------------------------- */
/* kNN scalar-stream kernel (round 4, the default kNN path): the estimate of
 * k_gather_knn_tile / k_gather_knn bit for bit, with the photons streamed
 * through the scalar cache instead of staged into LDS.
 *  - A wave (one 8x8 tile) forms the same groups as k_gather_knn_tile. Per
 *    pass it walks the rows of the union box of its lanes' bounds; a row is a
 *    contiguous run of the cell-sorted photons, read as photon PAIRS
 *    (k_knn_pack: x0 x1 | y0 y1 | z0 z1 | wx0 wx1 ...) with s_load, so one
 *    SGPR pair is the wave-uniform operand of a packed v_pk_* instruction and
 *    every lane tests both photons of the pair against its own record. No
 *    staging, no index mapping, no LDS traffic for the photons at all.
 *  - r_k^2 by radix-style histograms on the d^2 BIT PATTERNS (a non-negative
 *    float orders like its bits): bin = min(sat(bits - A) >> sh, 32), 32 bins
 *    + a sink per lane in LDS (one ds_add per photon, no conversions, exact
 *    bin edges). Level 0 covers the two octaves below maxD^2 at 1/16 octave
 *    (bin 0 also takes everything nearer); the bin holding the K-th value is
 *    COLLECTed into a per-lane list (<= 12) and ranked, or, when it holds
 *    more, histogrammed again at 32x the resolution (or, for a dense lane
 *    whose K-th is in bin 0, over all of [0, hi) in 4-octave bins).
 *  - SUM: every lane adds, for each pair, the pbrt kernel terms of the
 *    photons below its r_k^2 that face it, in the record's fixed point
 *    (rint, exact double sums: order-free), masked per lane; a pair no lane
 *    hits costs only its distance test.
 *  - Passes are phase-serialised per wave (HIST before COLLECT before SUM),
 *    so each pass runs one specialised loop.
 * A tile this kernel does not handle — a lane group whose union box exceeds
 * the 64-row map, r_k^2 = 0 (pbrt's 0/0 and its lowest-slot ties) — is
 * appended to P.knn_ovf and re-run by k_gather_knn_tile. */
/* waves per SIMD (VGPR budget; the 4.25 KB histogram allows 9): C2 kNN gather
 * 5 (81 VGPRs) 0.746-0.757 ms, 6 (73) 0.735, 7 (72) 0.747 (same box) */
#ifndef PM_KS_WAVES
#define PM_KS_WAVES 6
#endif
#define KS_OCC __attribute__((amdgpu_waves_per_eu(PM_KS_WAVES, PM_KS_WAVES)))
constexpr int KS_NB = 32;   /* bins per histogram level (+1 sink), 16-bit counters: two lanes per word */
constexpr int KS_HW = KS_NB / 2 + 1; /* LDS words per lane: (KS_NB + 1) 16-bit counters, or KS_LIST + 1 list rows + a sink row */
#ifndef PM_KS_LIST
#define PM_KS_LIST 12
#endif
constexpr int KS_LIST = PM_KS_LIST; /* values a COLLECT keeps per lane (rows 0..KS_LIST of the histogram, +1 scratch) */
/* (y, z) rows of a group's union box: two per lane. With 64, a tile across a
 * corner of the room (lanes on two walls, the union deeper than 8 x 8 rows)
 * split into leader groups, each running its own passes over nearly the same
 * photons: those tiles took up to 19 passes against 3.65 on average and set
 * the launch's length (tools/tile_times.py knn) */
#ifndef PM_KS_ROWS
#define PM_KS_ROWS 128
#endif
constexpr int KS_ROWS = PM_KS_ROWS;
static_assert(KS_ROWS == 64 || KS_ROWS == 128, "one or two union rows per lane");
enum { KS_HIST = 0, KS_COLLECT = 1, KS_SUM = 2, KS_DONE = 3 };
static_assert(KS_LIST + 1 < KS_HW, "the COLLECT list aliases histogram rows (not the sink's)");

/* photon pairs of the bucket order for the scalar stream: pair k = photons
 * 2k, 2k + 1, P block (x x y y z z wx wx), Q block (r r g g b b wy wy wz wz
 * . .); photons past the map are zero (the stream masks them). Block 0
 * thread 0 also clears the overflow-tile counter of this gather. */
__global__ __launch_bounds__(256) void k_knn_pack(const uint32_t *cell_start, uint32_t ncells, const float4 *ph_a,
                                                  const float4 *ph_b, float4 *pk_p, float4 *pk_q, int64_t npairs,
                                                  uint32_t *ovf_n) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k < 64 && ovf_n) ovf_n[k] = 0u;
    if (k >= npairs) return;
    const int64_t n = cell_start[ncells], j = 2 * k;
    if (j >= n + 16) return; /* a few zero pairs past the map: never read unmasked */
    float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0, b0 = a0, b1 = a0;
    float c0 = 0.f, c1 = 0.f;
    if (j < n) { a0 = ph_a[j]; b0 = ph_b[2 * j]; c0 = ph_b[2 * j + 1].x; }
    if (j + 1 < n) { a1 = ph_a[j + 1]; b1 = ph_b[2 * j + 2]; c1 = ph_b[2 * j + 3].x; }
    pk_p[2 * k] = make_float4(a0.x, a1.x, a0.y, a1.y);
    pk_p[2 * k + 1] = make_float4(a0.z, a1.z, a0.w, a1.w);
    pk_q[3 * k] = make_float4(b0.x, b1.x, b0.y, b1.y);
    pk_q[3 * k + 1] = make_float4(b0.z, b1.z, b0.w, b1.w);
    pk_q[3 * k + 2] = make_float4(c0, c1, 0.f, 0.f);
}

/* gap (cell units) between [lo, hi] and cell c of an axis of dim cells —
 * the border cells extend to infinity (cell_axis clamps) — less a 1e-3
 * margin for the rounding of the cell-unit coordinates */
PMD float box_gap(float lo, float hi, uint32_t c, int dim) {
    const float a = c == 0 ? -INFINITY : (float)c, b = (int)c + 1 == dim ? INFINITY : (float)(c + 1);
    return fmaxf(fmaxf(a - hi, lo - b) - 1e-3f, 0.f);
}
/* cell of a cell-unit coordinate, clamped like cell_axis */
PMD uint32_t cell_u(float u, int dim) {
    const int c = (int)floorf(u);
    return (uint32_t)(c < 0 ? 0 : (c >= dim ? dim - 1 : c));
}
__global__ __launch_bounds__(64) KS_OCC void k_gather_knn_ss(GatherParams P) {
#ifdef PM_TILE_TIMES
    uint32_t tstat[8] = {0, 0, 0, 0, 0, 0, 0, 0}; /* TILE_STAT's sink (unused here) */
    (void)tstat;
#endif
    /* 4.25 KB: HIST counts 16-bit halves (bin h of lane l: half l & 1 of
     * word 32 h + l / 2, bins 0..32); COLLECT lists 32-bit words (entry a of
     * lane l: word 64 a + l, rows 0..KS_LIST, the sink row KS_HW - 1) */
    __shared__ uint32_t H[KS_HW * 64];
    const int lane = threadIdx.x & 63;
    if (P.tiles && P.n_tiles_dev && (int64_t)blockIdx.x >= (int64_t)*P.n_tiles_dev) return;
#ifdef PM_TILE_TIMES
    const unsigned long long tc0 = __builtin_amdgcn_s_memrealtime();
#else
    const unsigned long long tc0 = P.tile_cost ? __builtin_amdgcn_s_memrealtime() : 0ull;
#endif
    /* the wave's lifetime for the cost-ordered tile list (k_tile_sort) */
    auto record_cost = [&]() {
        if (P.tile_cost && lane == 0)
            P.tile_cost[blockIdx.x] = (uint16_t)min(__builtin_amdgcn_s_memrealtime() - tc0, 65535ull);
    };
    const uint32_t tile = P.tiles ? P.tiles[blockIdx.x] : blockIdx.x;
    const int64_t r = P.rec_begin + (int64_t)tile * 64 + lane;
    const int K = P.knn_k;
    const float maxd2 = P.knn_r2;
#pragma unroll
    for (int b = 0; b < KS_HW; ++b) H[b * 64 + lane] = 0u;
    bool active = false, live = false, back = false;
    float4 pos = make_float4(0.f, 0.f, 0.f, 0.f), nrm = pos;
    if (r < P.rec_end) {
        pos = P.R.pos[r];
        const uint32_t flags = (uint32_t)__float_as_int(pos.w);
        active = !(flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID));
        back = (flags & PM_REC_BACKFACE) != 0;
        if (active) {
            nrm = P.R.nrm[r];
            live = __float_as_int(P.materials[__float_as_int(nrm.w)].w) == PM_MATTE; /* non-specular BSDF only */
        }
    }
    const v3 p = xyz(pos);
    /* Faceforward folded into the normal: Dot(-n, w) = -Dot(n, w) exactly */
    const float nsx = back ? -nrm.x : nrm.x, nsy = back ? -nrm.y : nrm.y, nsz = back ? -nrm.z : nrm.z;
    const GridDesc g = P.grid;
    TILE_STAT(0, 1);
    GProf gp; /* PM_GATHER_PROFILE: record + groups, pass setup, HIST, COLLECT, SUM, pass end, store */
    gp.begin();
    uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0, z0 = 0, z1 = 0;
    if (live) { /* KnnGrid::init's cells */
        const float rq = sqrtf(maxd2) * 1.0001f + 1e-4f;
        x0 = cell_axis(p.x - rq, g.gx, g.inv_cs, g.dx); x1 = cell_axis(p.x + rq, g.gx, g.inv_cs, g.dx);
        y0 = cell_axis(p.y - rq, g.gy, g.inv_cs, g.dy); y1 = cell_axis(p.y + rq, g.gy, g.inv_cs, g.dy);
        z0 = cell_axis(p.z - rq, g.gz, g.inv_cs, g.dz); z1 = cell_axis(p.z + rq, g.gz, g.inv_cs, g.dz);
    }
    /* selection state: HIST level (A, sh) counts the values below
     * A + (32 << sh) (bin 0 includes everything below A + (1 << sh)) */
    const uint32_t Bm = __float_as_uint(maxd2);
    uint32_t sh = 19u;
    while (sh > 0u && (32u << sh) > Bm) --sh;
    uint32_t A = Bm - (32u << sh);
    /* lowopen: bin 0 also holds everything below A (level 0, before any
     * refinement); otherwise the K-th is known to be >= A and `base` values
     * lie below A (bin 0 counts them too: every histogram counts global ranks) */
    uint32_t base = 0u;
    int phase = live ? KS_HIST : KS_DONE;
    bool lvl0 = true, full = true, defer = false, lowopen = true;
    uint32_t klo = 0u, kw = 0u, cc = 0u;
    int need = 0, less = 0, cnt = 0;
    float md2 = maxd2, inv = 0.f, sc = 1.f;
    Kx3 acc{0, 0, 0};

    const const_f32_ptr pkp = (const_f32_ptr)P.knn_pk_p;
    const const_f32_ptr pkq = (const_f32_ptr)P.knn_pk_q;
    const f2 px2 = {p.x, p.x}, py2 = {p.y, p.y}, pz2 = {p.z, p.z};
    bool pend = live;
    while (!defer) {
        const unsigned long long pm = __ballot(pend);
        if (pm == 0ull) break;
        /* the group: every pending lane if their union box fits the 64-lane
         * row map, else the first pending lane's neighbourhood */
        uint32_t X0, X1, Y0, Y1, Z0, Z1;
        bool mine = pend;
        union_box6(g, mine, x0, x1, y0, y1, z0, z1, X0, X1, Y0, Y1, Z0, Z1);
        uint32_t LY = Y1 > Y0 ? 32u - (uint32_t)__builtin_clz(Y1 - Y0) : 0u;
        if (LY > 7u || ((uint64_t)(Z1 - Z0 + 1u) << LY) > (uint64_t)KS_ROWS) {
            /* the first pending lane's neighbourhood: the lanes whose box
             * starts within GRk cells of the leader's, for the widest GRk whose
             * union still fits the row map (a surface seen at a grazing angle
             * spreads its tile over several cells: wider groups, fewer of them,
             * each with its own passes) */
            const int leader = __builtin_ctzll(pm);
            const uint32_t lx = __builtin_amdgcn_readlane(x0, leader), ly = __builtin_amdgcn_readlane(y0, leader),
                           lz = __builtin_amdgcn_readlane(z0, leader);
            bool fits = false;
            for (uint32_t GRk = KS_ROWS > 64 ? 4u : KT_GROUP_R; !fits && GRk >= KT_GROUP_R; GRk >>= 1) {
                mine = pend && x0 + GRk - lx <= 2u * GRk && y0 + GRk - ly <= 2u * GRk && z0 + GRk - lz <= 2u * GRk;
                union_box6(g, mine, x0, x1, y0, y1, z0, z1, X0, X1, Y0, Y1, Z0, Z1);
                LY = Y1 > Y0 ? 32u - (uint32_t)__builtin_clz(Y1 - Y0) : 0u;
                fits = LY <= 7u && ((uint64_t)(Z1 - Z0 + 1u) << LY) <= (uint64_t)KS_ROWS;
            }
            if (!fits) { defer = true; break; } /* grid too coarse */
        }
        pend = pend && !mine;
        /* passes until every lane of the group has its estimate (a level
         * descends 5 bits or slides to [0, hi): far fewer than 64 passes;
         * the bound only guarantees that every wave ends) */
        for (int npass = 0;; ++npass) {
            if (npass == 64) { defer = true; break; }
            const bool in = mine && phase != KS_DONE;
            const unsigned long long mh = __ballot(in && phase == KS_HIST), mc = __ballot(in && phase == KS_COLLECT),
                                     ms = __ballot(in && phase == KS_SUM);
            if ((mh | mc | ms) == 0ull) break;
            const int pt = mh ? KS_HIST : (mc ? KS_COLLECT : KS_SUM);
            const bool act = in && phase == pt;
            TILE_STAT(1, 1);
            TILE_STAT(2, pt == KS_HIST);
            gp.mark(0);
            /* this lane's bound (every value the pass needs is below it) */
            float bnd = 0.f;
            if (act) {
                if (pt == KS_HIST) { /* the level's upper edge A + (32 << sh), at most maxD^2 */
                    const uint64_t ub = (uint64_t)A + ((uint64_t)32u << sh);
                    bnd = ub >= (uint64_t)Bm ? maxd2 : __uint_as_float((uint32_t)ub);
                }
                else if (pt == KS_COLLECT) bnd = __uint_as_float(klo + kw);
                else bnd = full ? next_up(md2) : md2;
            }
            /* the pass's union: cells of [p - r', p + r'], r'^2 = bnd: a
             * sub-box of the group's (bnd <= maxD^2), so it fits the row map */
            uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0, c0 = 0, c1 = 0;
            if (act) {
                const float rq = sqrtf(bnd) * 1.0001f + 1e-4f;
                a0 = cell_axis(p.x - rq, g.gx, g.inv_cs, g.dx); a1 = cell_axis(p.x + rq, g.gx, g.inv_cs, g.dx);
                b0 = cell_axis(p.y - rq, g.gy, g.inv_cs, g.dy); b1 = cell_axis(p.y + rq, g.gy, g.inv_cs, g.dy);
                c0 = cell_axis(p.z - rq, g.gz, g.inv_cs, g.dz); c1 = cell_axis(p.z + rq, g.gz, g.inv_cs, g.dz);
            }
            uint32_t PX0, PX1, PY0, PY1, PZ0, PZ1;
            union_box6(g, act, a0, a1, b0, b1, c0, c1, PX0, PX1, PY0, PY1, PZ0, PZ1);
            const uint32_t PLY = PY1 > PY0 ? 32u - (uint32_t)__builtin_clz(PY1 - PY0) : 0u;
            /* rows pruned to the union of the pass's spheres: with the act
             * lanes' positions in the box [Pmin, Pmax] and R the largest
             * bound (cell units), a photon within R_l of lane l lies in a row
             * whose (y, z) gap to the box is <= R and, in that row, within
             * sqrt(R^2 - gap^2) of [Pmin.x, Pmax.x] (KnnGrid::scan's pruning
             * for the whole pass at once; cell_gap's 1e-3 margins) */
            const float ux = (p.x - g.gx) * g.inv_cs, uy = (p.y - g.gy) * g.inv_cs, uz = (p.z - g.gz) * g.inv_cs;
            const float Rq = wave_max_f(act ? (sqrtf(bnd) * 1.0001f + 1e-4f) * g.inv_cs : 0.f);
            const float mnx = wave_min_f(act ? ux : INFINITY), mxx = wave_max_f(act ? ux : -INFINITY);
            const float mny = wave_min_f(act ? uy : INFINITY), mxy = wave_max_f(act ? uy : -INFINITY);
            const float mnz = wave_min_f(act ? uz : INFINITY), mxz = wave_max_f(act ? uz : -INFINITY);
            /* union rows u = lane and lane + 64: photons [Bu, Bu + Lu) of cells
             * xa..xb of its (y, z) */
            uint32_t Bu[2] = {0u, 0u}, Lu[2] = {0u, 0u};
#pragma unroll
            for (int h = 0; h < KS_ROWS / 64; ++h) {
                const uint32_t u = (uint32_t)lane + 64u * (uint32_t)h;
                const uint32_t cy = PY0 + (u & ((1u << PLY) - 1u)), cz = PZ0 + (u >> PLY);
                if (cy <= PY1 && cz <= PZ1) {
                    const float gy = box_gap(mny, mxy, cy, g.dy), gz = box_gap(mnz, mxz, cz, g.dz);
                    const float rem = Rq * Rq - (gy * gy + gz * gz);
                    if (rem >= 0.f) {
                        const float sx = sqrtf(rem) * 1.0001f + 1e-3f;
                        const uint32_t xa = max(PX0, cell_u(mnx - sx, g.dx)), xb = min(PX1, cell_u(mxx + sx, g.dx));
                        if (xa <= xb) {
                            const uint32_t row = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx;
                            Bu[h] = P.cell_start[row + xa];
                            Lu[h] = P.cell_start[row + xb + 1u] - Bu[h];
                        }
                    }
                }
            }
            const unsigned long long rows = __ballot(Lu[0] > 0u), rows_hi = KS_ROWS > 64 ? __ballot(Lu[1] > 0u) : 0ull;
            /* 16-bit bin counters: a union of >= 2^16 photons goes to k_gather_knn_tile */
            if (uniform_u32(__builtin_amdgcn_readlane(wave_incl_sum_u32(Lu[0] + Lu[1]), 63)) >= 65536u) { defer = true; break; }
#ifdef PM_KNN_SS_DBG
            const unsigned long long rows0 = rows | rows_hi;
#endif
            /* per-lane constants of the pass (lanes outside it never hit) */
            const uint32_t hA = act ? A : 0u, hsh = act ? sh : 0u;
            const uint32_t clo = act ? klo : 0u, cw = act ? kw : 0u;
            const float smd = act ? md2 : -1.f, sinv = inv, ssc = sc;
            /* 1/r_k^2 times the power-of-two scale: exact, one multiply per term */
            const float sis = sinv * ssc;
            const f2 inv2 = {sinv, sinv}, is2 = {sis, sis}, one2 = {1.f, 1.f}, c3 = {3.f * INV_PI, 3.f * INV_PI};
            const f2 nx2 = {nsx, nsx}, ny2 = {nsy, nsy}, nz2 = {nsz, nsz};
            uint32_t *hcol = H + lane;
            /* HIST counters: bin h of lane l is the (l & 1) half of word
             * h * 32 + l / 2 (lanes l, l ^ 1 share a word column), so a count
             * is one address op and a per-lane constant increment */
            uint32_t *hpair = H + (lane >> 1);
            /* lanes outside the pass add 0 (their half of each word stays 0) */
            const uint32_t hinc = act ? 1u << ((lane & 1) * 16) : 0u;
            /* COLLECT: the lane's list rows (lanes outside the pass write the sink row) */
            uint32_t *lcol = hcol + (act ? 0 : (KS_HW - 1) * 64);
            uint32_t ccl = 0u;
            /* one specialised loop per pass type over the rows' photon pairs */
            /* one specialised loop per pass type over the rows' photon pairs,
             * NP pairs per batch: the batch's s_loads are issued together and
             * waited on once (the scalar cache returns out of order, so a wave
             * cannot wait for an older load while a younger one is in flight) */
            auto stream = [&](auto PT_) PM_INLINE {
                constexpr int PT = decltype(PT_)::value;
                constexpr int NP = PT == KS_SUM ? 2 : 4;
                unsigned long long rm = rows, rm_hi = rows_hi;
                while (rm | rm_hi) {
                    /* rows 0..63 (Bu[0] of lane u), then 64..127 (Bu[1]) */
                    const bool hi = rm == 0ull;
                    const unsigned long long cur = hi ? rm_hi : rm;
                    const int u = __builtin_ctzll(cur);
                    if (hi) rm_hi &= rm_hi - 1ull;
                    else rm &= rm - 1ull;
                    const uint32_t b = uniform_u32(__builtin_amdgcn_readlane(hi ? Bu[1] : Bu[0], u));
                    const uint32_t e = b + uniform_u32(__builtin_amdgcn_readlane(hi ? Lu[1] : Lu[0], u));
                    const uint32_t k1 = (e + 1u) >> 1;
                    TILE_STAT(3, 1);
                    TILE_STAT(PT == KS_HIST ? 4 : PT == KS_COLLECT ? 5 : 6, k1 - (b >> 1));
                    for (uint32_t k0 = b >> 1; k0 < k1; k0 += NP) {
                        /* the batch (reads past the run stay inside the packed
                         * buffer's zero pairs; their photons are never counted) */
                        /* whole-vector loads: one s_load_dwordx16 per 64 B, none of
                         * them sunk into the per-pair branches below */
                        float pv[NP][8], qv[PT == KS_SUM ? NP : 1][12];
                        const sv16 *q = (const sv16 *)(pkp + 8 * (size_t)k0);
                        if constexpr (PT == KS_SUM) {
                            static_assert(NP == 2, "one P vector + 24 Q floats per batch");
                            f32x16 v = q[0], a = ((const sv16 *)(pkq + 12 * (size_t)k0))[0];
                            f32x8 c8 = ((const sv8 *)(pkq + 12 * (size_t)k0 + 16))[0];
                            asm volatile("" : "+s"(v), "+s"(a), "+s"(c8)); /* the whole batch, one wait */
#pragma unroll
                            for (int c = 0; c < 16; ++c) pv[c / 8][c % 8] = v[c];
#pragma unroll
                            for (int c = 0; c < 12; ++c) qv[0][c] = a[c];
#pragma unroll
                            for (int c = 0; c < 4; ++c) qv[1][c] = a[12 + c];
#pragma unroll
                            for (int c = 0; c < 8; ++c) qv[1][4 + c] = c8[c];
                        } else {
                            static_assert(NP == 4, "two P vectors per batch");
                            f32x16 v0 = q[0], v1 = q[1];
                            asm volatile("" : "+s"(v0), "+s"(v1)); /* the whole batch, one wait */
#pragma unroll
                            for (int c = 0; c < 16; ++c) { pv[c / 8][c % 8] = v0[c]; pv[2 + c / 8][c % 8] = v1[c]; }
                        }
#pragma unroll
                        for (int i = 0; i < NP; ++i) {
                            const uint32_t k = k0 + (uint32_t)i;
                            if (i > 0 && k >= k1) break;
                            f2 X = {pv[i][0], pv[i][1]};
                            const f2 Y = {pv[i][2], pv[i][3]}, Z = {pv[i][4], pv[i][5]};
                            /* the run's ends: a half pair outside [b, e) is pushed to infinity */
                            if (2u * k < b) X.x = INFINITY;
                            if (2u * k + 1u >= e) X.y = INFINITY;
                            const f2 dx = px2 - X, dy = py2 - Y, dz = pz2 - Z;
                            const f2 d2 = (dx * dx + dy * dy) + dz * dz; /* in_radius / KnnGrid::scan's order */
                            const uint32_t u0 = __float_as_uint(d2.x), u1 = __float_as_uint(d2.y);
                            if constexpr (PT == KS_HIST) {
                                const uint32_t h0 = min(__builtin_elementwise_sub_sat(u0, hA) >> hsh, (uint32_t)KS_NB);
                                const uint32_t h1 = min(__builtin_elementwise_sub_sat(u1, hA) >> hsh, (uint32_t)KS_NB);
                                atomicAdd(hpair + h0 * 32u, hinc);
                                atomicAdd(hpair + h1 * 32u, hinc);
                            } else if constexpr (PT == KS_COLLECT) {
                                lcol[ccl * 64u] = u0;
                                ccl += (u0 - clo) < cw ? 1u : 0u;
                                lcol[ccl * 64u] = u1;
                                ccl += (u1 - clo) < cw ? 1u : 0u;
                            } else {
                                const f2 WX = {pv[i][6], pv[i][7]}, R = {qv[i][0], qv[i][1]}, G = {qv[i][2], qv[i][3]};
                                const f2 Bl = {qv[i][4], qv[i][5]}, WY = {qv[i][6], qv[i][7]}, WZ = {qv[i][8], qv[i][9]};
                                const bool h0 = d2.x < smd, h1 = d2.y < smd;
                                less += (int)h0 + (int)h1;
                                if (__ballot(h0 || h1)) {
                                    TILE_STAT(7, 1);
                                    const f2 dn = (nx2 * WX + ny2 * WY) + nz2 * WZ; /* knn_facing */
                                    /* knn_add: s = 1 - d^2 / r_k^2, kernel 3/pi s^2, times 1/r_k^2 and alpha;
                                     * a photon that does not count gets ki = 0, so every term of it is rint(0) = 0 */
                                    const f2 sv = one2 - d2 * inv2;
                                    f2 ki = ((c3 * sv) * sv) * is2;
                                    if (!(h0 && dn.x > 0.f)) ki.x = 0.f;
                                    if (!(h1 && dn.y > 0.f)) ki.y = 0.f;
                                    const f2 cr = ki * R, cg = ki * G, cb = ki * Bl;
                                    acc.x += knn_rnd(cr.x) + knn_rnd(cr.y); /* knn_add's rounding */
                                    acc.y += knn_rnd(cg.x) + knn_rnd(cg.y);
                                    acc.z += knn_rnd(cb.x) + knn_rnd(cb.y);
                                }
                            }
                        }
                    }
                }
            };
            gp.mark(1);
            if (pt == KS_HIST) stream(std::integral_constant<int, KS_HIST>{});
            else if (pt == KS_COLLECT) stream(std::integral_constant<int, KS_COLLECT>{});
            else stream(std::integral_constant<int, KS_SUM>{});
            gp.mark(pt == KS_HIST ? 2 : pt == KS_COLLECT ? 3 : 4);
            if (!act) continue;
            if (pt == KS_HIST) {
                /* the bin holding the K-th value; the column is left zeroed */
                uint32_t cum = 0u, below = 0u, cntb = 0u;
                int bs = -1;
                /* both lanes of a word read it before either clears it (one
                 * instruction each); a neighbour outside the pass counted only
                 * into the sink, so its halves of bins 0..31 are zero anyway */
                const uint32_t hs = (uint32_t)(lane & 1) * 16u;
#pragma unroll 4
                for (int b = 0; b < KS_NB; ++b) {
                    const uint32_t c = (hpair[b * 32] >> hs) & 0xffffu;
                    hpair[b * 32] = 0u;
                    if (bs < 0 && cum + c >= (uint32_t)K) { bs = b; below = cum; cntb = c; }
                    cum += c;
                }
                hpair[KS_NB * 32] = 0u;
                if (lvl0 && cum < (uint32_t)K) { /* fewer than K inside maxD: r_k^2 = maxD^2 */
                    full = false;
                    md2 = maxd2;
                    phase = KS_SUM;
                } else {
                    lvl0 = false;
                    /* the K-th value's bin [lo, hi): bin 0 of an open level
                     * starts at 0; bin 0 of a refined level holds the base
                     * values below A as well, which are not in [A, hi) */
                    const bool open0 = bs == 0 && lowopen && A != 0u;
                    const uint32_t lo = open0 ? 0u : A + ((uint32_t)bs << sh), hi = A + ((uint32_t)(bs + 1) << sh);
                    if (bs == 0 && !open0) { cntb -= base; below = base; }
                    if (sh == 0u && !open0) { /* a bin of one bit pattern */
                        md2 = __uint_as_float(lo);
                        phase = KS_SUM;
                    } else if (cntb <= (uint32_t)KS_LIST) {
                        phase = KS_COLLECT;
                        klo = lo; kw = hi - lo; need = K - (int)below; cc = 0u;
                    } else if (!open0) { /* 32x finer over the bin */
                        A = lo;
                        base = below;
                        sh = sh >= 5u ? sh - 5u : 0u;
                    } else { /* the K-th is below A + 2^sh (a dense lane): the 32 bins
                               * slide down to end at hi, 4x wider (8 octaves at 1/4 octave) */
                        const uint32_t sh2 = min(sh + 2u, 26u);
                        A = hi > (32u << sh2) ? hi - (32u << sh2) : 0u;
                        base = 0u;
                        sh = sh2;
                    }
                    lowopen = open0 && A != 0u && cntb > (uint32_t)KS_LIST;
                }
            } else if (pt == KS_COLLECT) {
                cc = ccl;
                /* rank the kept values (cc of them): the need-th smallest */
                uint32_t v[KS_LIST];
#pragma unroll
                for (int a = 0; a < KS_LIST; ++a) v[a] = (uint32_t)a < cc ? hcol[a * 64] : 0xffffffffu;
                const uint32_t *lcand = hcol;
                uint32_t ans = v[0];
                for (uint32_t a = 0; a < cc; ++a) { /* candidate a (re-read from LDS: a rolled loop) */
                    const uint32_t va = lcand[a * 64];
                    int lt = 0, le = 0;
#pragma unroll
                    for (int bb = 0; bb < KS_LIST; ++bb) { lt += v[bb] < va; le += v[bb] <= va; }
                    if (lt < need && need <= le) ans = va;
                }
#pragma unroll
                for (int a = 0; a <= KS_LIST; ++a) hcol[a * 64] = 0u;
                md2 = __uint_as_float(ans);
                phase = KS_SUM;
                if (md2 == 0.f) defer = true; /* pbrt's 0/0: k_gather_knn_tile's tie rules */
#ifdef PM_KNN_SS_DBG
                if (ans == 0xffffffffu) {
                    const uint32_t i = atomicAdd(P.knn_ovf_n + 1, 1u);
                    if (i < 60u) {
                        uint32_t *d = P.knn_ovf_n + 64 + 16 * i;
                        d[0] = tile; d[1] = lane; d[2] = cc; d[3] = (uint32_t)need; d[4] = klo; d[5] = kw; d[6] = A;
                        d[7] = sh; d[8] = __float_as_uint(p.x); d[9] = __float_as_uint(p.y); d[10] = __float_as_uint(p.z);
                        d[11] = PX0; d[12] = PX1; d[13] = PY0 | (PY1 << 16); d[14] = PZ0 | (PZ1 << 16); d[15] = (uint32_t)__popcll(rows0);
                    }
                }
#endif
            }
            if (phase == KS_SUM && pt != KS_SUM) { /* begin_sum */
                sc = knn_scale(P.knn_fx, md2);
                inv = 1.f / md2;
                acc = Kx3{0, 0, 0};
                less = 0;
            } else if (pt == KS_SUM) {
                cnt = full ? K : less;
                phase = KS_DONE;
            }
        }
        if (__ballot(defer)) defer = true;
        gp.mark(5);
    }
    if (__ballot(defer)) { /* re-run by k_gather_knn_tile */
        if (lane == 0) P.knn_ovf[atomicAdd(P.knn_ovf_n, 1u)] = tile;
        record_cost();
        return;
    }
#ifdef PM_KNN_SS_DBG
    if (active && md2 != md2) atomicAdd(P.knn_ovf_n + 2, 1u);
#endif
    if (active) {
        if (!live) md2 = maxd2; /* specular: nothing found, cnt 0 */
        const float4 st = P.fresh ? make_float4(0.f, 0.f, 0.f, P.r2init) : P.R.state[r];
        const double isc = 1.0 / (double)sc;
        const v3 Lr = mk((float)((double)acc.x * isc), (float)((double)acc.y * isc), (float)((double)acc.z * isc));
        const v3 flux = xyz(st) + Lr;
        P.R.state[r] = make_float4(flux.x, flux.y, flux.z, md2);
        P.R.n[r] = (float)cnt;
    }
    record_cost();
    gp.mark(6);
    gp.flush(P.counters);
#ifdef PM_TILE_TIMES
    if (P.tile_times && lane == 0) {
        uint32_t xcc, hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        unsigned long long *o = P.tile_times + 8 * (size_t)blockIdx.x;
        o[0] = tc0; o[1] = __builtin_amdgcn_s_memrealtime(); o[2] = xcc; o[3] = hw;
        o[4] = tstat[1] | ((unsigned long long)tstat[2] << 32);   /* passes | HIST passes */
        o[5] = tstat[4] | ((unsigned long long)tstat[5] << 32);   /* HIST pairs | COLLECT pairs */
        o[6] = tstat[6] | ((unsigned long long)tstat[3] << 32);   /* SUM pairs | rows */
        o[7] = tstat[7] | ((unsigned long long)(r - lane) << 32); /* hit batches | record */
    }
#endif
}

hipError_t launch_gather_knn(const GatherParams &p, int count, hipStream_t s) {
    if (p.rec_end <= p.rec_begin) return hipSuccess;
    if (p.knn_k < 1 || p.knn_k > PM_KNN_MAX) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((p.rec_end - p.rec_begin + KNN_BLOCK - 1) / KNN_BLOCK);
    /* census launches run the per-lane kernel (its photons-tested count is the
     * per-record unit bench.py prices); the tile kernels find the same set */
    if (!count && p.kernel == PM_GK_TILE) {
        const unsigned g = p.tiles ? (unsigned)p.n_tiles : grid;
        if (!g) return hipSuccess;
        if (p.knn_pk_p && p.knn_r2 > 1e-30f) { /* the level-0 bins need bits(maxD^2) >= 32 << sh */
            /* scalar stream, then k_gather_knn_tile over the tiles it handed back */
            /* the pairs once per photon map (band gathers reuse them); the
             * overflow counters of every gather */
            const int64_t np = p.knn_pk_pairs;
            if (p.knn_pack)
                pm_launch(k_knn_pack, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, p.cell_start, p.grid.ncells,
                          p.ph_a, p.ph_b, p.knn_pk_p, p.knn_pk_q, np, p.knn_ovf_n);
            else {
                const hipError_t e = hipMemsetAsync(p.knn_ovf_n, 0, 64 * sizeof(uint32_t), s);
                if (e != hipSuccess) return e;
            }
            pm_launch(k_gather_knn_ss, dim3(g), dim3(64), 0, s, p);
            GatherParams q = p;
            q.tiles = p.knn_ovf;
            q.n_tiles_dev = p.knn_ovf_n;
            q.rec_begin = p.rec_begin;
            pm_launch(k_gather_knn_tile, dim3(g), dim3(KNN_BLOCK), 0, s, q);
            return hipGetLastError();
        }
        pm_launch(k_gather_knn_tile, dim3(g), dim3(KNN_BLOCK), 0, s, p);
        return hipGetLastError();
    }
    const uint32_t lds = (uint32_t)(p.knn_k * KNN_BLOCK * sizeof(uint32_t));
    if (count) pm_launch(k_gather_knn<1>, dim3(grid), dim3(KNN_BLOCK), lds, s, p);
    else pm_launch(k_gather_knn<0>, dim3(grid), dim3(KNN_BLOCK), lds, s, p);
    return hipGetLastError();
}

/* kd-tree range query in the reference layout (gathering.cu:25-96):
 * same visiting order, same accumulation order -> bit-exact with it. */
template <int PARTIAL, int COUNT>
__global__ __launch_bounds__(GATHER_BLOCK) void k_gather_kd(GatherParams P) {
    __shared__ uint32_t stk[KD_STACK * GATHER_BLOCK];
    uint32_t *stack = stk + threadIdx.x;
    const int64_t r = P.rec_begin + (int64_t)blockIdx.x * GATHER_BLOCK + threadIdx.x;
    unsigned long long vis = 0, hits = 0, rows = 0, act = 0;
    if (r < P.rec_end) {
        float4 pos = P.R.pos[r];
        uint32_t flags = (uint32_t)__float_as_int(pos.w);
        if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) {
            if (PARTIAL) write_partial(P, partial_index(P, r), 0, Fx3{0, 0, 0});
        } else {
            float4 st = P.fresh ? make_float4(0.f, 0.f, 0.f, P.r2init) : P.R.state[r];
            float4 nrm = P.R.nrm[r];
            const float maxDist2 = st.w;
            float4 m = P.materials[__float_as_int(nrm.w)];
            v3 fv = __float_as_int(m.w) == PM_MATTE ? xyz(m) * INV_PI : mk(0.f, 0.f, 0.f);
            const v3 p = xyz(pos), ns = xyz(nrm);
            int M = 0;
            v3 L = mk(0.f, 0.f, 0.f);
            if (P.kd_count > 0) {
                int sp = 0;
                uint32_t nodeNum = 0;
                stack[0] = 0; sp = 1;
                int64_t guard = 0; /* each node is visited at most once */
                const int stack_max = P.kd_stack < KD_STACK ? P.kd_stack : KD_STACK;
                bool overflow = false;
                do {
                    if (++guard > P.kd_count || nodeNum >= (uint64_t)P.kd_count) { /* not a pbrt kd-tree */
                        atomicOr(P.error, PM_GATHER_ERR_TREE);
                        break;
                    }
                    const float2 *q = reinterpret_cast<const float2 *>(P.kd_nodes + nodeNum);
                    float2 q0 = q[0], q1 = q[1];
                    uint32_t bits = (uint32_t)__float_as_int(q0.x);
                    uint32_t axis = (bits >> 1) & 3u, hasLeft = bits & 1u, right = bits >> 3;
                    v3 np = mk(q0.y, q1.x, q1.y);
                    v3 diff = p - np;
                    float dist2 = diff.x * diff.x + diff.y * diff.y + diff.z * diff.z;
                    if (COUNT) vis++;
                    if (dist2 < maxDist2) {
                        M++;
                        float2 q2 = q[2], q3 = q[3], q4 = q[4];
                        v3 al = mk(q2.x, q2.y, q3.x), wi = mk(q3.y, q4.x, q4.y);
                        L = L + fabsf(dot(ns, wi)) * fv * al;
                    }
                    if (axis < 3) {
                        float pa = comp(p, (int)axis), na = comp(np, (int)axis);
                        float d2 = (pa - na) * (pa - na);
                        if (pa <= na) {
                            if (d2 < maxDist2 && right < PM_PHOTON_MAX_RIGHT_CHILD) {
                                if (sp < stack_max) { stack[sp * GATHER_BLOCK] = right; ++sp; } else overflow = true;
                            }
                            if (hasLeft) nodeNum = nodeNum + 1; else { --sp; nodeNum = stack[sp * GATHER_BLOCK]; }
                        } else {
                            if (d2 < maxDist2 && hasLeft) {
                                if (sp < stack_max) { stack[sp * GATHER_BLOCK] = nodeNum + 1; ++sp; } else overflow = true;
                            }
                            if (right < PM_PHOTON_MAX_RIGHT_CHILD) nodeNum = right;
                            else { --sp; nodeNum = stack[sp * GATHER_BLOCK]; }
                        }
                    } else {
                        --sp;
                        nodeNum = stack[sp * GATHER_BLOCK];
                    }
                } while (nodeNum);
                /* a dropped subtree would silently lose photons: the launch reports it */
                if (overflow) atomicOr(P.error, PM_GATHER_ERR_STACK);
            }
            if (COUNT) { hits += (unsigned long long)M; act++; }
            if (PARTIAL) {
                const float sc = P.fx_scale;
                write_partial(P, partial_index(P, r), M, Fx3{to_fx(L.x, sc), to_fx(L.y, sc), to_fx(L.z, sc)});
            } else {
                float N = P.fresh ? 0.f : P.R.n[r];
                ppm_apply(st, N, M, L, P.ppm_alpha);
                if (M > 0 || P.fresh) { P.R.state[r] = st; P.R.n[r] = N; }
            }
        }
    }
    if (COUNT) count4(P.counters, vis, hits, rows, act);
}

template <int PARTIAL, int NN, bool COST>
static void launch_tile_nn(const GatherParams &p, unsigned g, hipStream_t s) {
    switch (p.span) { /* cells per axis of a lane box at the grid's design radius */
    case 2: pm_launch((k_gather_tile<PARTIAL, NN, 2, COST>), dim3(g), dim3(TILE_BLOCK), 0, s, p); break;
    case 3: pm_launch((k_gather_tile<PARTIAL, NN, 3, COST>), dim3(g), dim3(TILE_BLOCK), 0, s, p); break;
    case 4: pm_launch((k_gather_tile<PARTIAL, NN, 4, COST>), dim3(g), dim3(TILE_BLOCK), 0, s, p); break;
    default: pm_launch((k_gather_tile<PARTIAL, NN, 5, COST>), dim3(g), dim3(TILE_BLOCK), 0, s, p); break;
    }
}
template <int PARTIAL>
static void launch_tile(const GatherParams &p, unsigned g, hipStream_t s) {
    /* only a list launch measures tile costs (they index the list) */
    const bool cost = p.tile_cost != nullptr && p.tiles != nullptr;
    if (p.fx_nonneg) cost ? launch_tile_nn<PARTIAL, 1, true>(p, g, s) : launch_tile_nn<PARTIAL, 1, false>(p, g, s);
    else cost ? launch_tile_nn<PARTIAL, 0, true>(p, g, s) : launch_tile_nn<PARTIAL, 0, false>(p, g, s);
}

template <int STRUCT, int PARTIAL, int COUNT>
static void launch_g(const GatherParams &p, hipStream_t s) {
    unsigned grid = (unsigned)((p.rec_end - p.rec_begin + GATHER_BLOCK - 1) / GATHER_BLOCK);
    if (STRUCT == PM_GATHER_GRID && !COUNT && p.kernel == PM_GK_TILE && p.tiles) {
        /* the tile list: only tiles with an active record */
        const int64_t waves = p.n_tiles;
        const unsigned g = (unsigned)((waves + TILE_BLOCK / 64 - 1) / (TILE_BLOCK / 64));
        if (g == 0) return;
        launch_tile<PARTIAL>(p, g, s);
        return;
    }
    /* a counting launch always runs the per-lane kernel: its census (rows and
     * photons per RECORD) is the algorithm's unit count bench.py prices; the
     * tile and wave kernels find exactly the same photons (bit-identical records) */
    if (STRUCT == PM_GATHER_GRID && !COUNT && p.kernel == PM_GK_TILE)
        launch_tile<PARTIAL>(p, (unsigned)((p.rec_end - p.rec_begin + TILE_BLOCK - 1) / TILE_BLOCK), s);
    else if (STRUCT == PM_GATHER_GRID)
        pm_launch((k_gather_grid<PARTIAL, COUNT>), dim3(grid), dim3(GATHER_BLOCK), 0, s, p);
    else
        pm_launch((k_gather_kd<PARTIAL, COUNT>), dim3(grid), dim3(GATHER_BLOCK), 0, s, p);
}

hipError_t launch_gather(const GatherParams &p, int structure, int partial, int count, hipStream_t s) {
    if (p.rec_end <= p.rec_begin) return hipSuccess;
    int key = (structure ? 4 : 0) | (partial ? 2 : 0) | (count ? 1 : 0);
    switch (key) {
    case 0: launch_g<0, 0, 0>(p, s); break;
    case 1: launch_g<0, 0, 1>(p, s); break;
    case 2: launch_g<0, 1, 0>(p, s); break;
    case 3: launch_g<0, 1, 1>(p, s); break;
    case 4: launch_g<1, 0, 0>(p, s); break;
    case 5: launch_g<1, 0, 1>(p, s); break;
    case 6: launch_g<1, 1, 0>(p, s); break;
    default: launch_g<1, 1, 1>(p, s); break;
    }
    return hipGetLastError();
}

/* radius^2 of a record range to / from a contiguous float array: after the
 * owner's PPM update every rank needs the new radii for the next pass's
 * range queries (pmrender/dist.py, "reduce" exchange) */
__global__ __launch_bounds__(256) void k_radius2_io(RecordsDev R, float *buf, int64_t rec_begin, int64_t rec_count,
                                                    int to_records, const uint32_t *view) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rec_count) return;
    const int64_t r = view ? (int64_t)view[rec_begin + i] : rec_begin + i;
    if (to_records) R.state[r].w = buf[i];
    else buf[i] = R.state[r].w;
}

hipError_t launch_radius2_io(const RecordsDev &R, float *buf, int64_t rec_begin, int64_t rec_count, int to_records,
                             const uint32_t *view, hipStream_t s) {
    if (rec_count <= 0) return hipSuccess;
    pm_launch(k_radius2_io, dim3((unsigned)((rec_count + 255) / 256)), dim3(256), 0, s, R, buf, rec_begin,
                       rec_count, to_records, view);
    return hipGetLastError();
}

/* PPM update from summed partials (M, L in fixed point), record chunk */
__global__ __launch_bounds__(256) void k_ppm_update(RecordsDev R, const long long *partial, int64_t rec_begin,
                                                    int64_t rec_count, float alpha, double inv, const uint32_t *view) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= rec_count) return;
    const int64_t r = view ? (int64_t)view[rec_begin + i] : rec_begin + i;
    uint32_t flags = (uint32_t)__float_as_int(R.pos[r].w);
    if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return;
    const longlong2 *q = reinterpret_cast<const longlong2 *>(partial + 4 * i);
    const longlong2 a = q[0], b = q[1];
    const int M = (int)a.x;
    if (M <= 0) return;
    float4 st = R.state[r];
    float N = R.n[r];
    v3 L = mk((float)((double)a.y * inv), (float)((double)b.x * inv), (float)((double)b.y * inv));
    ppm_apply(st, N, M, L, alpha);
    R.state[r] = st;
    R.n[r] = N;
}

hipError_t launch_ppm_update(const GatherParams &p, const long long *partial, int64_t rec_begin, int64_t rec_count,
                             hipStream_t s) {
    if (rec_count <= 0) return hipSuccess;
    pm_launch(k_ppm_update, dim3((unsigned)((rec_count + 255) / 256)), dim3(256), 0, s, p.R, partial,
                       rec_begin, rec_count, p.ppm_alpha, p.fx_inv, p.view_list);
    return hipGetLastError();
}

/* PPM update of the split exchange: every rank holds the global photon
 * count M of every view record (all-reduced), so it updates every radius and
 * photon count itself — no radius exchange — while the summed flux arrives
 * only for its own chunk [v_begin, v_begin + v_count) (reduce-scattered).
 * fresh: the records are in a deferred reset — start from the initial state
 * and write every view record. */
__global__ __launch_bounds__(256) void k_ppm_update_split(RecordsDev R, const int *count, const long long *flux,
                                                          int64_t n_view, int64_t v_begin, int64_t v_count, float alpha,
                                                          double inv, const uint32_t *view, int fresh, float r2init) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_view) return;
    const int64_t r = view ? (int64_t)view[i] : i;
    const uint32_t flags = (uint32_t)__float_as_int(R.pos[r].w);
    if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return;
    const int M = count[i];
    if (M <= 0 && !fresh) return;
    float4 st = fresh ? make_float4(0.f, 0.f, 0.f, r2init) : R.state[r];
    float N = fresh ? 0.f : R.n[r];
    v3 L = mk(0.f, 0.f, 0.f);
    const int64_t k = i - v_begin;
    if (k >= 0 && k < v_count) {
        const long long *f = flux + 3 * k;
        L = mk((float)((double)f[0] * inv), (float)((double)f[1] * inv), (float)((double)f[2] * inv));
    }
    ppm_apply(st, N, M, L, alpha);
    R.state[r] = st;
    R.n[r] = N;
}

/* pm_ppm_update_split in two halves (ppm_apply's operations, split at the
 * ratio): radius2 and N of every view record now, the ratio kept for the
 * owner's flux update after the flux reduce-scatter has landed */
__global__ __launch_bounds__(256) void k_ppm_update_radius(RecordsDev R, const int *count, float *ratio_out,
                                                           int64_t n_view, float alpha, const uint32_t *view,
                                                           int fresh, float r2init) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_view) return;
    const int64_t r = view ? (int64_t)view[i] : i;
    ratio_out[i] = -1.f;
    const uint32_t flags = (uint32_t)__float_as_int(R.pos[r].w);
    if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return;
    const int M = count[i];
    if (M <= 0 && !fresh) return;
    float4 st = fresh ? make_float4(0.f, 0.f, 0.f, r2init) : R.state[r];
    float N = fresh ? 0.f : R.n[r];
    if (M > 0) { /* ppm_apply without the flux */
        int totalPhotons = N + alpha * M;
        float ratio = totalPhotons / (N + M);
        st.w = st.w * ratio;
        N = totalPhotons;
        ratio_out[i] = ratio;
    }
    R.state[r] = st;
    R.n[r] = N;
}
__global__ __launch_bounds__(256) void k_ppm_update_flux(RecordsDev R, const float *ratio, const long long *flux,
                                                         int64_t v_begin, int64_t v_count, double inv,
                                                         const uint32_t *view) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= v_count) return;
    const int64_t i = v_begin + k;
    const float q = ratio[i];
    if (!(q >= 0.f)) return;
    const int64_t r = view ? (int64_t)view[i] : i;
    const long long *f = flux + 3 * k;
    const v3 L = mk((float)((double)f[0] * inv), (float)((double)f[1] * inv), (float)((double)f[2] * inv));
    float4 st = R.state[r];
    const v3 fl = (xyz(st) + L) * q;
    st.x = fl.x; st.y = fl.y; st.z = fl.z;
    R.state[r] = st;
}
hipError_t launch_ppm_update_radius(const GatherParams &p, const int *count, float *ratio, int64_t n_view, int fresh,
                                    hipStream_t s) {
    if (n_view <= 0) return hipSuccess;
    pm_launch(k_ppm_update_radius, dim3((unsigned)((n_view + 255) / 256)), dim3(256), 0, s, p.R, count, ratio, n_view,
              p.ppm_alpha, p.view_list, fresh, p.r2init);
    return hipGetLastError();
}
hipError_t launch_ppm_update_flux(const GatherParams &p, const float *ratio, const long long *flux, int64_t v_begin,
                                  int64_t v_count, hipStream_t s) {
    if (v_count <= 0) return hipSuccess;
    pm_launch(k_ppm_update_flux, dim3((unsigned)((v_count + 255) / 256)), dim3(256), 0, s, p.R, ratio, flux, v_begin,
              v_count, p.fx_inv, p.view_list);
    return hipGetLastError();
}

hipError_t launch_ppm_update_split(const GatherParams &p, const int *count, const long long *flux, int64_t n_view,
                                   int64_t v_begin, int64_t v_count, int fresh, hipStream_t s) {
    if (n_view <= 0) return hipSuccess;
    pm_launch(k_ppm_update_split, dim3((unsigned)((n_view + 255) / 256)), dim3(256), 0, s, p.R, count, flux, n_view,
              v_begin, v_count, p.ppm_alpha, p.fx_inv, p.view_list, fresh, p.r2init);
    return hipGetLastError();
}

/* ====================================================================== */
/* record view (active records, compacted in record order)               */
/* ====================================================================== */
__global__ __launch_bounds__(256) void k_view_flags(RecordsDev R, uint32_t *flags) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r > R.count) return;
    if (r == R.count) { flags[r] = 0u; return; } /* scanned tail -> total */
    const uint32_t f = (uint32_t)__float_as_int(R.pos[r].w);
    flags[r] = (f & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) ? 0u : 1u;
}

__global__ __launch_bounds__(256) void k_view_list(RecordsDev R, const uint32_t *flags, uint32_t *rank,
                                                   uint32_t *list) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R.count) return;
    if (flags[r]) list[rank[r]] = (uint32_t)r;
    else rank[r] = 0xffffffffu;
}

hipError_t launch_record_view(const RecordsDev &R, uint32_t *flags, uint32_t *rank, uint32_t *list, uint32_t *sums,
                              hipStream_t s) {
    const int64_t n = R.count;
    pm_launch(k_view_flags, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, R, flags);
    hipError_t e = launch_exclusive_scan(flags, n + 1, rank, sums, s);
    if (e != hipSuccess) return e;
    pm_launch(k_view_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, R, flags, rank, list);
    return hipGetLastError();
}

/* ====================================================================== */
/* final gathering                                                        */
/* ====================================================================== */
__global__ __launch_bounds__(256) void k_final(FinalParams P) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= P.rec_count) return;
    const int64_t r = P.view ? (int64_t)P.view[P.rec_begin + i] : P.rec_begin + i;
    int64_t o = i;
    if (P.raster) {
        int px, py;
        rec_to_pixel(r, P.W, &px, &py);
        uint32_t fl = (uint32_t)__float_as_int(P.R.pos[r].w);
        if (fl & PM_REC_INVALID) return;
        o = (int64_t)py * P.W + px;
    }
    float4 pos = P.R.pos[r];
    uint32_t flags = (uint32_t)__float_as_int(pos.w);
    v3 out = mk(0.f, 0.f, 0.f);
    if (!(flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID))) {
        float4 dl = P.R.dl[r], st = P.R.state[r];
        float N = P.R.n[r];
        v3 IDL = mk(0.f, 0.f, 0.f);
        if (P.knn) { /* LPhoton: Lr * rho / pi with Lr's 1/nPaths = 1/emitted (passes averaged) */
            const float4 m = P.materials[__float_as_int(P.R.nrm[r].w)];
            const v3 fv = __float_as_int(m.w) == PM_MATTE ? xyz(m) * INV_PI : mk(0.f, 0.f, 0.f);
            IDL = (xyz(st) / P.emitted) * fv;
        } else if (N != 0) {
            IDL = xyz(st) * INV_PI / (st.w * P.emitted);
        }
        out = xyz(dl) + IDL;
        float y = 0.212671f * out.x + 0.715160f * out.y + 0.072169f * out.z;
        if (isnan(out.x) || isnan(out.y) || isnan(out.z) || y < -1e-5f || isinf(y)) out = mk(0.f, 0.f, 0.f);
    }
    P.out[3 * o + 0] = out.x;
    P.out[3 * o + 1] = out.y;
    P.out[3 * o + 2] = out.z;
}

__global__ __launch_bounds__(256) void k_tile_flags(RecordsDev R, uint8_t *flags) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool act = false;
    if (r < R.count) act = !((uint32_t)__float_as_int(R.pos[r].w) & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID));
    const unsigned long long m = __ballot(act);
    if ((threadIdx.x & 63) == 0 && r < R.count) flags[r >> 6] = m != 0ull ? 1 : 0;
}
/* one block compacts the flags in order: 1024 tiles per step, ballot ranks
 * inside each wave, wave totals through LDS */
__global__ __launch_bounds__(1024) void k_tile_compact(const uint8_t *flags, int64_t nt, uint32_t *list,
                                                       uint32_t *count) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t base;
    if (threadIdx.x == 0) base = 0u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    for (int64_t t0 = 0; t0 < nt; t0 += 1024) {
        const int64_t t = t0 + threadIdx.x;
        const bool f = t < nt && flags[t] != 0;
        const unsigned long long m = __ballot(f);
        if (lane == 0u) wsum[w] = (uint32_t)__builtin_popcountll(m);
        __syncthreads();
        uint32_t off = base;
        for (uint32_t k = 0; k < w; ++k) off += wsum[k];
        if (f) list[off + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = (uint32_t)t;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t tot = 0u;
            for (int k = 0; k < 16; ++k) tot += wsum[k];
            base += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *count = base;
}
/* Cost-ordered tile list (one block): the tile gather's launch ends with
 * the waves dispatched last (each a tile's whole lifetime, 9.5 us on average
 * at C2, up to 35 us for the densest tiles), so the order of the list sets
 * the drain. The groups of 8 entries a wave's XCD takes together (xcd_tile)
 * are counting-sorted by the largest lifetime among them, heaviest first, in
 * 256 log-spaced buckets (3 % each); the order inside a bucket is the atomics'
 * (any order gives the same sums). */
__global__ __launch_bounds__(1024) void k_tile_sort(const uint32_t *list, const uint16_t *cost, const uint32_t *n_dev,
                                                    int64_t n_host, uint32_t *out) {
    __shared__ uint32_t hist[256];
    const int tid = threadIdx.x;
    const int64_t n = n_dev ? (int64_t)*n_dev : n_host, S = n / 8;
    if (tid < 256) hist[tid] = 0u;
    __syncthreads();
    auto bucket = [&](int64_t g) {
        uint32_t c = 1u;
        for (int k = 0; k < 8; ++k) c = max(c, (uint32_t)cost[8 * g + k]);
        /* 24 buckets per octave from 16 ticks (0.16 us) up; heaviest -> 0 */
        const int b = (int)(24.f * (__log2f((float)c) - 4.f));
        return 255 - min(max(b, 0), 255);
    };
    for (int64_t g = tid; g < S; g += 1024) atomicAdd(&hist[bucket(g)], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0u;
        for (int b = 0; b < 256; ++b) { const uint32_t c = hist[b]; hist[b] = run; run += c; }
    }
    __syncthreads();
    for (int64_t g = tid; g < S; g += 1024) {
        const uint32_t pos = atomicAdd(&hist[bucket(g)], 1u);
        const uint4 *src = reinterpret_cast<const uint4 *>(list + 8 * g);
        uint4 *dst = reinterpret_cast<uint4 *>(out + 8 * (int64_t)pos);
        dst[0] = src[0];
        dst[1] = src[1];
    }
    for (int64_t i = 8 * S + tid; i < n; i += 1024) out[i] = list[i]; /* the partial group stays last */
}
hipError_t launch_tile_sort(const uint32_t *list, const uint16_t *cost, const uint32_t *n_dev, int64_t n, uint32_t *out,
                            hipStream_t s) {
    pm_launch(k_tile_sort, dim3(1), dim3(1024), 0, s, list, cost, n_dev, n, out);
    return hipGetLastError();
}

hipError_t launch_tile_list(const RecordsDev &R, uint8_t *flags, uint32_t *list, uint32_t *count, hipStream_t s) {
    if (R.count <= 0) return hipSuccess;
    pm_launch(k_tile_flags, dim3((unsigned)((R.count + 255) / 256)), dim3(256), 0, s, R, flags);
    pm_launch(k_tile_compact, dim3(1), dim3(1024), 0, s, (const uint8_t *)flags, (R.count + 63) / 64, list, count);
    return hipGetLastError();
}

hipError_t launch_final(const FinalParams &p, hipStream_t s) {
    if (p.rec_count <= 0) return hipSuccess;
    pm_launch(k_final, dim3((unsigned)((p.rec_count + 255) / 256)), dim3(256), 0, s, p);
    return hipGetLastError();
}

/* restore the eye pass's initial PPM state (flux 0, N 0, r^2 init;
 * raytracing.cu:121-123) so that every benchmark step gathers the same
 * workload as the reference's single pass */
__global__ __launch_bounds__(256) void k_reset_records(RecordsDev R, float r2init) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= R.count) return;
    uint32_t flags = (uint32_t)__float_as_int(R.pos[r].w);
    if (flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return;
    R.state[r] = make_float4(0.f, 0.f, 0.f, r2init);
    R.n[r] = 0.f;
}

hipError_t launch_reset_records(const RecordsDev &R, float r2init, hipStream_t s) {
    if (R.count <= 0) return hipSuccess;
    pm_launch(k_reset_records, dim3((unsigned)((R.count + 255) / 256)), dim3(256), 0, s, R, r2init);
    return hipGetLastError();
}

} // namespace pm
