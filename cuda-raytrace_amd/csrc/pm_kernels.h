/*
 * pm_kernels.h — kernel parameter blocks and launcher declarations shared by
 * the host orchestration (pm_api.cpp) and the HIP kernels (pm_trace.hip, pm_bucket.hip, pm_gather.hip).
 */
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pm_device.h"

namespace pm {

/* Stage timing without marker packets: the API (pm_api.cpp timer_begin /
 * timer_end) points g_stage at an event pair around one stage, and every
 * launch in the stage goes through pm_launch, which binds the start event to
 * the stage's first dispatch and the stop event to each dispatch (the last
 * one wins) — the timestamps come from the kernel dispatches themselves, so
 * timing adds no idle gap between kernels. */
struct StageEvents { hipEvent_t start = nullptr, stop = nullptr; int launched = 0; };
extern thread_local StageEvents *g_stage;

template <typename F, typename... Args>
inline void pm_launch(F kernel, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, Args... args) {
    hipEvent_t a = nullptr, b = nullptr;
    if (StageEvents *st = g_stage) {
        a = st->launched ? nullptr : st->start;
        b = st->stop;
        st->launched++;
    }
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, a, b, 0u, args...);
}

constexpr int EYE_BLOCK = 128;     /* traversal kernels: LDS stack column per lane */
constexpr int TRACE_BLOCK = 256;    /* k_trace: 4 waves compact paths together */
constexpr int BVH_STACK = BVH_STACK_DEPTH; /* >= max BVH depth (builder enforces it) */
/* the 8-wide tree's exact stack bound (seven pushes per level) runs deeper:
 * its stacks hold up to 96 entries (k_trace_pool8 keeps PM_POOL_STACK of them
 * in LDS and spills the rest; the eye pass's LDS columns take the bound) */
constexpr int BVH8_STACK = 96;
constexpr int GATHER_BLOCK = 256;
/* k_gather_tile: waves per block. Its waves never synchronise with each
 * other, and a block's LDS is held until its last wave ends, so with several
 * waves per block a tile that runs long keeps its neighbours' LDS allocated
 * (LDS co-limits the kernel at 5 waves/SIMD). One wave per block: C2
 * gather 47.6 -> 46.5-47.1 us, C3 0.54-0.56 -> 0.53 ms, C5 0.30 -> 0.27 ms
 * (same box, against 256) */
#ifndef PM_TILE_BLOCK
#define PM_TILE_BLOCK 64
#endif
constexpr int TILE_BLOCK = PM_TILE_BLOCK;
enum { PM_GK_TILE = 0, PM_GK_LANE = 1 };
/* error word of a kd-tree gather: a record's traversal stack overflowed (a
 * subtree would have been dropped), or the node links are not a pbrt tree */
enum { PM_GATHER_ERR_STACK = 1u, PM_GATHER_ERR_TREE = 2u };
constexpr int KD_STACK = 32;       /* >= pbrt median kd-tree depth for < 2^31 photons */
constexpr int KNN_BLOCK = 64;      /* k_gather_knn: one wave per block, LDS heaps [K][64] */

/* device SoA record arrays */
struct RecordsDev {
    float4 *pos;    /* pos.xyz, flags (bits) */
    float4 *nrm;    /* ns.xyz, material (bits) */
    float4 *state;  /* flux.xyz, radius2 */
    float *n;       /* photon_count */
    float4 *dl;     /* direct light */
    int64_t count;
};

struct EyeParams {
    SceneDev S;
    RecordsDev R;
    int pinhole, W, H, n2d;
    float4 eye, fwd, right, up;
    const float *rays;
    const float *rand2d;
    float eps, r2init;
    int max_spec;
    uint32_t light_seed;
};

constexpr int R2_BINS = 64, R2_COPIES = 256, R2_PER_OCTAVE = 8; /* radius histogram (adaptive grid) */
struct GridDesc {
    float gx, gy, gz, inv_cs;
    int dx, dy, dz;
    uint32_t ncells;
};

/* bucket coordinate along one axis, clamped (points outside the scene box
 * map to the border cells on both the build and the query side) */
PMD uint32_t cell_axis(float v, float g0, float inv_cs, int dim) {
    int c = (int)floorf((v - g0) * inv_cs);
    c = c < 0 ? 0 : (c >= dim ? dim - 1 : c);
    return (uint32_t)c;
}

struct TraceParams {
    SceneDev S;
    pm_photon *slots;
    uint32_t perm[28];
    uint32_t perm_bits[3]; /* the base 3, 5, 7 tables of perm, 3 bits per digit (permuted_halton4) */
    int64_t path_begin, path_count, slot_path_base;
    int64_t pool_paths; /* > 0: pooled kernel (k_trace_pool, 4-wide BVH scenes), paths per wave; else one path per lane */
    int pass, mpc, max_spec, light_index;
    float eps;
    uint32_t seed;
    unsigned long long *counters; /* census [rays, nodes, prim tests, deposits] */
    unsigned long long *prof;     /* phase cycles (PM_TRACE_PROFILE builds), 8 words */
    /* fused bucket counting (bucket != 0): per slot cell key (0xffffffff =
     * invalid) and rank = atomicAdd(count[key]) of the build's counting pass */
    int bucket;
    GridDesc grid;
    uint32_t *count, *key, *rank;
    /* per-lane / pooled kernels: a path's deposits held in registers and
     * written once per path (pm_trace.hip Held; used when mpc == 4 and the
     * slot buffer is 16-B aligned) */
    int hold;
    /* pooled kernel: LDS stack entries per lane (0: S.stack_depth); deeper
     * entries go to spill (entry i of thread g at spill[(i - pool_stack) *
     * spill_stride + g]) */
    int pool_stack;
    int *spill;
    uint32_t spill_stride;
    /* fused counting: keys / ranks plane-major (deposit k of path i at k * key_np + i) when > 0, else at the slot index */
    int64_t key_np;
    /* fused counting only: 1 = leave a path's unused slots as they are (their
     * keys say invalid; pm_api zeroes them with launch_zero_invalid_slots
     * before anything else reads the slot buffer) */
    int lazy_zero;
};

struct GatherParams {
    RecordsDev R;
    int64_t rec_begin, rec_end; /* records gathered by this launch */
    const float4 *materials;
    float ppm_alpha;
    /* grid */
    GridDesc grid;
    const uint32_t *cell_start; /* ncells + 1 */
    const float4 *ph_a;         /* x, y, z, wi.x */
    const float4 *ph_b;         /* 2 per photon: (alpha.rgb, wi.y), (wi.z, 0, 0, 0) */
    /* kd-tree (reference layout) */
    const pm_photon *kd_nodes;
    int64_t kd_count;
    int kd_stack;         /* traversal stack entries (<= KD_STACK; smaller only to test the overflow report) */
    unsigned int *error;  /* PM_GATHER_ERR_* of the launch (device word, OR-ed) */
    /* fixed-point flux: contribution c -> rint(c * fx_scale), fx_inv = 1/fx_scale (2^-S) */
    float fx_scale;
    double fx_inv;
    /* every contribution is >= 0 (scene emission and albedos and the photon
     * fluxes are non-negative): the tile kernel may sum in double (exact) */
    int fx_nonneg;
    /* partial mode: per record int64 (M, L.x, L.y, L.z) in fixed point, or
     * (count != null) split: int32 M in count[k], three int64 in flux[3k..] */
    long long *partial;
    int *count;
    long long *flux;
    /* fresh: records are in a deferred reset (pm_reset_records): read the
     * initial PPM state (flux 0, N 0, r2init) instead of memory, write it back */
    int fresh;
    float r2init;
    /* record view: view_rank[r] = position of record r in the view (partials),
     * view_list[i] = record of view position i (update); null = all records */
    const uint32_t *view_rank;
    const uint32_t *view_list;
    /* grid gather kernel (PM_GK_*): tile (k_gather_tile, LDS-staged, default),
     * lane (k_gather_grid, per lane from global memory); census launches
     * always run k_gather_grid */
    int kernel;
    int span; /* tile kernel: cells per axis of a lane box at the grid's design radius (2..5) */
    /* tile kernel: a wave's direct lanes with small boxes are scanned by the
     * whole wave together (coop_batch) when their cells hold at most
     * 64 * coop_steps photons, else each lane scans its own */
    uint32_t coop_steps;
    /* non-null: k_gather_tile bins every updated radius, R2_COPIES x R2_BINS
     * counters, bin = floor(-log2(r^2 * r2hist_inv) * R2_PER_OCTAVE) clamped */
    uint32_t *r2hist;
    float r2hist_inv;
    /* kNN estimator (k_gather_knn): knn_k nearest photons with d^2 < knn_r2;
     * per-record fixed-point scale = power of two below knn_fx * r_k^2;
     * slots = the slot buffer the buckets were built from (ph_b carries the
     * slot index) */
    int knn_k;
    float knn_r2, knn_fx;
    const pm_photon *slots;
    unsigned long long *counters; /* [0] visited, [1] in radius */
    /* tile list (non-null: full-range gathers): the launch covers only the
     * n_tiles tiles of 64 records (tile t = records [64 t, 64 t + 64)) that
     * hold an active record, in record order */
    const uint32_t *tiles;
    int64_t n_tiles;
    /* non-null: the list's length is this device word (the host has not read
     * it back yet); n_tiles then bounds the grid (every tile) */
    const uint32_t *n_tiles_dev;
    /* non-null: each tile wave stores its lifetime (s_memrealtime ticks,
     * saturated to 16 bits) at tile_cost[list entry], for the cost-ordered
     * list of the next gathers (launch_tile_sort) */
    uint16_t *tile_cost;
    /* PM_TILE_TIMES diagnostic builds: per launched wave (start, end)
     * s_memrealtime and (XCC_ID, HW_ID), 4 u64 at tile_times[4 * block] */
    unsigned long long *tile_times;
    /* kNN scalar-stream kernel (k_gather_knn_ss): photon pairs (k_knn_pack,
     * knn_pk_pairs of them: 2 float4 + 3 float4 per pair) and the list of
     * tiles it hands back to k_gather_knn_tile (knn_ovf, length *knn_ovf_n) */
    float4 *knn_pk_p, *knn_pk_q;
    int64_t knn_pk_pairs;
    int knn_pack; /* 1: (re)write the pairs (the map changed since the last pack); else only clear the counters */
    uint32_t *knn_ovf, *knn_ovf_n;
};
/* knn_ovf_n[0] = handed-back tiles; [1..63] and the 16-word records at
 * [64, 1024 + 64) are PM_KNN_SS_DBG diagnostics; the list follows */
constexpr int KNN_OVF_HDR = 64 + 1024;

struct FinalParams {
    RecordsDev R;
    int knn;                     /* records hold kNN sums: out = DL + flux / emitted * Kd/pi */
    const float4 *materials;
    float emitted;
    int64_t rec_begin, rec_count;
    float *out;     /* float3 */
    int raster;     /* 1: out indexed by pixel (pinhole), 0: by record - rec_begin */
    int W;
    const uint32_t *view; /* non-null: [rec_begin, rec_begin + rec_count) index the active-record view */
};

/* traversal mode of a scene: LDS-resident blob (brute force when tiny) or HBM */
inline int scene_mode(const SceneDev &S) {
    return S.n_inst > 0 ? MODE_INST : S.lds_bytes ? (S.brute ? MODE_BRUTE : MODE_LDS) : MODE_GLOBAL;
}

hipError_t launch_eye(const EyeParams &p, hipStream_t s);
/* simple renderer (simplerender.cu): direct light per eye sample into out
 * (float3, raster / sample order); only p.R.count of the records is read */
hipError_t launch_simple(const EyeParams &p, float *out, hipStream_t s);
/* writes every slot of its paths (deposits, then zeros); count: census */
/* resident waves of k_trace_pool per CU with `lds` bytes of dynamic LDS per block */
int trace_pool_waves_per_cu(size_t lds, int hold, int w8 = 0);
size_t scan_scratch_words(int64_t n);
int trace_lane_waves_per_cu(const SceneDev &S, size_t lds, int hold);
/* adaptive-grid histogram: sum the R2_COPIES copies into host-mapped
 * out[R2_BINS] with plain stores (no copy engine) and zero the copies */
hipError_t launch_r2hist_reduce(uint32_t *hist, uint32_t *out_mapped, hipStream_t s);
hipError_t launch_trace(const TraceParams &p, int count, hipStream_t s);
/* photon-bucket build (pm_bucket.hip): count + rank, scan, fill.
 * count and cell_start have ncells + 1 entries; cell_start[ncells] = valid
 * photons; scratch holds bucket_scratch_words() uint32: key[n], rank[n], ...
 * counted: key/rank/count were produced by the trace kernel (TraceParams::bucket);
 * otherwise count must arrive zeroed. count leaves zeroed (cleared by the scan). */
size_t bucket_scratch_words(int64_t n_slots, uint32_t ncells);
hipError_t launch_bucket_build(const pm_photon *slots, int64_t n, GridDesc g, uint32_t *count, uint32_t *cell_start,
                               uint32_t *scratch, float4 *ph_a, float4 *ph_b, bool counted, hipStream_t s,
                               int64_t key_np = 0, int mpc = 1);
/* gather: structure 0 grid, 1 kd; mode 0 fused PPM, 1 partial */
hipError_t launch_gather(const GatherParams &p, int structure, int partial, int count, hipStream_t s);
/* kNN estimator (pbrt LPhoton) over the photon buckets, fused record update */
hipError_t launch_gather_knn(const GatherParams &p, int count, hipStream_t s);
hipError_t launch_ppm_update(const GatherParams &p, const long long *partial, int64_t rec_begin, int64_t rec_count,
                             hipStream_t s);
hipError_t launch_ppm_update_split(const GatherParams &p, const int *count, const long long *flux, int64_t n_view,
                                   int64_t v_begin, int64_t v_count, int fresh, hipStream_t s);
hipError_t launch_ppm_update_radius(const GatherParams &p, const int *count, float *ratio, int64_t n_view, int fresh,
                                    hipStream_t s);
hipError_t launch_ppm_update_flux(const GatherParams &p, const float *ratio, const long long *flux, int64_t v_begin,
                                  int64_t v_count, hipStream_t s);
hipError_t launch_final(const FinalParams &p, hipStream_t s);
/* list[0 .. *count) = the tiles (records [64 t, 64 t + 64)) holding an
 * active record, ascending, built on the device (flags: one byte per tile) */
/* the slots of [0, n) whose fused-count key is invalid (0xffffffff) set to
 * zero: the deferred zero fill of a lazy_zero trace (key index as the
 * trace wrote it: plane-major k * key_np + path when key_np > 0) */
hipError_t launch_zero_invalid_slots(pm_photon *slots, const uint32_t *key, int64_t n, int64_t key_np, int mpc,
                                     hipStream_t s);
hipError_t launch_tile_list(const RecordsDev &R, uint8_t *flags, uint32_t *list, uint32_t *count, hipStream_t s);
/* the tile list reordered by measured cost: groups of 8 consecutive entries
 * (a wave's XCD group, xcd_tile) in descending order of their largest
 * tile_cost, the last partial group kept last; n = *n_dev when non-null */
hipError_t launch_tile_sort(const uint32_t *list, const uint16_t *cost, const uint32_t *n_dev, int64_t n, uint32_t *out,
                            hipStream_t s);
hipError_t launch_radius2_io(const RecordsDev &R, float *buf, int64_t rec_begin, int64_t rec_count, int to_records,
                             const uint32_t *view, hipStream_t s);
/* exclusive scan of n uint32 (pm_bucket.hip); in/out 16-B aligned; sums: scan_scratch_words(n) */
size_t scan_scratch_words(int64_t n);
hipError_t launch_exclusive_scan(const uint32_t *in, int64_t n, uint32_t *out, uint32_t *sums, hipStream_t s);
/* active-record view: flags/rank n+1 words, list n words; rank[n] = active count */
hipError_t launch_record_view(const RecordsDev &R, uint32_t *flags, uint32_t *rank, uint32_t *list, uint32_t *sums,
                              hipStream_t s);
hipError_t launch_reset_records(const RecordsDev &R, float r2init, hipStream_t s);

/* scene BVH on the device (pm_bvh_gpu.hip): PLOC over the primitive boxes
 * (box: 2 float4 per primitive, (lo.xyz, ref bits) (hi.xyz, 0); Morton frame
 * of pm_build.h ploc_morton_frame), collapsed into quantized 4-wide nodes —
 * the tree pm_build.h build_ploc + ploc_to_bvh + collapse_bvh4 +
 * bvh4_bfs_order + quantize_bvh4 produce on the host, bit for bit. Outputs:
 * wnodes (<= max_nodes nodes of 4 uint4, breadth-first), refs (n, Morton
 * order; triangles as PRIM_TRI << 30 | storage slot) and tri_order (storage
 * slot -> triangle id, triangles in Morton order). Blocks on the stream. */
struct GpuBvhIn {
    const float4 *box;
    int n;
    float frame_lo[3], frame_scale[3];
    int radius;
};
struct GpuBvhOut {
    uint4 *wnodes;
    uint32_t *refs, *tri_order;
    int64_t max_nodes;
    int64_t nodes = 0, n_tris = 0;
    int depth = 0, max_stack = 0, rounds = 0;
};
hipError_t gpu_bvh_build(const GpuBvhIn &in, GpuBvhOut &out, hipStream_t s);
/* triangle records computed in triangle-id order -> storage order */
hipError_t launch_tri_permute(const uint32_t *tri_order, int64_t nst, const float4 *src_geo, const float4 *src_shade,
                              const int4 *src_info, float4 *geo, float4 *shade, uint32_t *tid, int4 *info,
                              hipStream_t s);

} // namespace pm
