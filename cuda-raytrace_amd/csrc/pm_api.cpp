/*
 * pm_api.cpp — the C-ABI of libpmhip.so (declared in include/pm_api.h):
 * context, scene flattening, BVH build + upload, stage orchestration and
 * the whole-render entry point. Host code only; kernels live in
 * pm_kernels.hip. No CPU fallback: every compute entry point launches HIP
 * kernels and fails with PM_ERR_HIP when the device is unusable.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <functional>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "pm_build.h"
#include "pm_kernels.h"

#pragma clang fp contract(off)

using namespace pm;

namespace {

std::string g_last_error;

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; bytes = 0; }
        if (n == 0) n = 16;
        hipError_t e = hipMalloc(&p, n);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    /* ensure() with 50 % headroom: buffers sized by the photon grid or the
     * valid photons of a pass, which change from pass to pass of a
     * progressive render (the radius shrinks, the grid gains cells): a
     * reallocation's hipFree waits for the device and left a ~250 us bubble
     * in every C5 pass (profiles/r06/c5_realloc) */
    hipError_t ensure_slack(size_t n) { return n <= bytes && p ? hipSuccess : ensure(n + n / 2); }
    bool external = false; /* caller-owned memory: never freed or grown here */
    void release() { if (p && !external) (void)hipFree(p); p = nullptr; bytes = 0; external = false; }
    template <class T> T *as() const { return (T *)p; }
};

struct HMesh { int material, light, has_n, has_uv; };
struct HTri { int v[3]; int mesh; uint32_t gid; }; /* gid: global id (insertion order over all triangles) */
/* two-level instancing: an object mesh stored once in object space, and its
 * instances (pbrt ObjectBegin / ObjectInstance) */
struct HObj {
    std::vector<float> P, N, UV;
    std::vector<int> idx;
    int material = 0, light = -1;
    bool has_n = false, has_uv = false;
};
struct HInst { int obj; float m[16], minv[16]; uint32_t gid_base; };
struct Timer { hipEvent_t a = nullptr, b = nullptr; };
struct TimerPool { std::vector<Timer> ev; size_t used = 0; };

struct Group;
struct Ctx {
    Group *group = nullptr; /* non-null: a multi-device context (pm_config::n_devices), Group below */
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    /* host scene */
    std::vector<float4> materials;
    std::vector<float> P, N, UV;
    std::vector<HMesh> meshes;
    std::vector<HTri> tris;
    int64_t next_tri_id = 0;     /* global ids handed out to triangles (meshes and instances); < 2^31 */
    std::vector<HObj> objs;
    std::vector<HInst> insts;
    int64_t obj_tris_stored = 0; /* object triangles in the committed scene (each mesh once) */
    std::vector<float4> disks;   /* 5 per disk */
    std::vector<float4> spheres; /* 4 per sphere */
    std::vector<float> sphere_o2w;
    std::vector<LightDev> lights;
    int rand2d_total = 0;
    int pinhole = 0, W = 0, H = 0;
    float eye[3] = {0}, fwd[3] = {0}, right[3] = {0}, up[3] = {0};
    std::vector<float> rays, rand2d;
    int64_t nrays = 0;
    int n2d = 0;
    bool committed = false;
    /* device scene */
    DevBuf d_scene, d_rays, d_rand2d; /* d_scene: the scene blob (SceneDev) */
    DevBuf d_tripairs;                /* brute-force scenes: triangle pairs interleaved (SceneDev::tri_pairs_g) */
    SceneDev S{};
    float bbox_lo[3] = {0, 0, 0}, bbox_hi[3] = {0, 0, 0};
    double emit_max = 1.0, kd_max = 1.0; /* bounds for the fixed-point flux scale */
    bool scene_nonneg = true;  /* no negative emission / albedo component (fixed-point sums in double) */
    bool slots_nonneg = true;  /* the slot buffer holds no negative flux (uploaded slots are checked) */
    int bvh_depth = 0;
    /* records */
    DevBuf d_pos, d_nrm, d_state, d_n, d_dl;
    int64_t nrec = 0;
    /* slots */
    DevBuf d_slots;
    int64_t slots_used = 0;
    /* lazy zero fill (TraceParams::lazy_zero): slots [0, slots_dirty) may hold
     * stale data where their fused-count key (d_scratch, dirty_key_np /
     * dirty_mpc) is invalid; materialize_slots zeroes them before any reader
     * but the bucket fill (env PM_LAZY_ZERO=1; by default the trace zeroes them
     * itself: same-box A/B in profiles/r05/trace_writes) */
    int64_t slots_dirty = 0, dirty_key_np = 0;
    int dirty_mpc = 0;
    hipEvent_t dirty_event = nullptr;
    bool lazy_zero = false, slots_exposed = false;
    /* photon buckets */
    DevBuf d_count, d_cell_start, d_scratch, d_pha, d_phb;
    DevBuf d_knnpk, d_knnovf; /* kNN scalar stream: photon pairs, handed-back tiles (+ count) */
    DevBuf d_tile_times;      /* PM_TILE_TIMES diagnostic builds */
    uint64_t map_gen = 0;      /* bumped by every bucket build */
    uint64_t knn_pack_gen = ~0ull; /* the map d_knnpk's pairs were packed from */
    void *knn_pack_ptr = nullptr;  /* ... and the pair buffer they were written to */
    bool knn_ss = true;       /* kNN: k_gather_knn_ss first (PM_KNN_SS=0: k_gather_knn_tile alone) */
    bool fuse_ok = true;      /* trace may fuse the bucket counting (off for the sub-contexts of a multi-device group) */
    struct { bool valid = false; int64_t n = 0; GridDesc grid{}; float r2 = 0.f; int64_t key_np = 0; int mpc = 1; } fused; /* counts made by the last trace (keys plane-major when key_np > 0) */
    GridDesc grid{};
    float grid_r2 = 0.f; /* radius^2 the photon map's grid is designed for */
    int64_t bvh4_nodes = 0; /* 4-wide BVH of an HBM scene (0: binary traversal) */
    int bvh4_depth = 0;
    int map_kind = -1;
    int64_t map_slots = 0;
    /* kd-tree */
    DevBuf d_kd;
    int64_t kd_count = 0;
    /* misc */
    DevBuf d_out, d_counters;
    bool counting = false;
    /* record view (pm_set_record_view): active records compacted in record order */
    bool view_active = false;
    int64_t n_view = 0;
    DevBuf d_vflags, d_vrank, d_vlist, d_vsums;
    /* tiles (64 records) holding an active record, in record order: full-range
     * tile gathers launch over these only (records fixed after the eye pass) */
    DevBuf d_tiles, d_tile_flags, d_tile_count;
    int64_t n_tiles = 0;           /* valid once tile_count_known */
    bool tiles_valid = false;      /* the list on the device matches the records */
    /* the list is reordered once by the measured cost of its tiles (the first
     * full-range tile gather on it records them; launch_tile_sort); env
     * PM_TILE_SORT=0 keeps record order */
    DevBuf d_tile_cost, d_tiles2;
    bool tile_sort = true, tiles_sorted = false;
    bool tile_count_known = false; /* its length read back (pinned copy + event, never waited on) */
    uint32_t *h_tile_count = nullptr;
    hipEvent_t tile_event = nullptr;
    /* pm_reset_records is deferred: records read as (flux 0, N 0, r2 = rec_fresh_r2) */
    bool rec_fresh = false;
    float rec_fresh_r2 = 0.f;
    /* estimator of the last gather: what the records' flux / radius2 /
     * photon_count mean for the final pass (PPM state or kNN sums) */
    int rec_estimator = PM_ESTIMATOR_PPM;
    int kd_stack = KD_STACK;        /* kd gather stack entries (env PM_KD_STACK, tests only) */
    bool trace_pool = true;         /* 4-wide scenes: the pooled trace kernel (env PM_TRACE_POOL=0: one path per lane) */
    bool trace_hold = true;         /* deposits written once per path where it costs no waves (env PM_TRACE_HOLD=0: per deposit) */
    int pool_stack = 31;            /* pooled kernel: LDS stack entries per lane (env PM_POOL_STACK; 0 = the exact bound): 31 lets five blocks share a CU's LDS */
    DevBuf d_spill;                 /* pooled kernel: stack entries beyond pool_stack */
    int gather_kernel = PM_GK_TILE; /* bucket gather kernel (env PM_GATHER_KERNEL=tile|lane) */
    int cell_span = 2;              /* PPM grid: cells per axis of a query box (env PM_CELL_SPAN 2..5) */
    /* adaptive grid radius (progressive PPM: radii shrink pass by pass). The
     * fused tile gather bins every updated r^2 (R2_BINS log bins per copy,
     * 8 copies) into d_r2hist; the histogram is copied to pinned memory
     * behind r2_event and, once landed, sets the next passes' grid radius to
     * the grid_quantile of the records' radii (the rest scan per lane).
     * Staleness is safe (radii only shrink); anything that can raise a
     * radius (eye pass, reset, upload, set_radius2, split / partial updates)
     * invalidates it. env PM_GRID_QUANTILE (default 0.9; <= 0 disables). */
    DevBuf d_r2hist;
    uint32_t *h_r2hist = nullptr, *h_r2hist_dev = nullptr; /* host-mapped R2_BINS words, its device address */
    hipEvent_t r2_event = nullptr;
    hipStream_t r2_stream = nullptr; /* the stream the last histogram reduce ran on (r2_event) */
    bool r2_wanted = false;    /* a progressive pass asked for the radii (no histogram otherwise) */
    bool r2_accum = false;     /* d_r2hist holds bins of this pass's gathers (every band), not yet reduced */
    bool r2_dirty = false;     /* d_r2hist holds bins of invalidated radii: zero before binning again */
    float r2_accum_init = 0.f; /* the r^2 the accumulated bins are relative to */
    bool r2_pending = false;   /* a histogram copy in flight */
    bool r2_valid = false;     /* the last landed / in-flight histogram describes the records */
    float r2_hist_init = 0.f;  /* the r^2 its bins are relative to */
    float design_r2 = 0.f;     /* grid radius^2 of the current photon map (0: initial_radius2) */
    double grid_quantile = 0.9; /* C5 step (same box, 3 runs each): 0.95 0.82-0.85 ms, 0.9 0.784-0.790, 0.8 0.826 */
    /* leading words of d_count known to be zero (the bucket scan clears the
     * counters it reads); valid while d_count.p == count_zero_ptr */
    size_t count_zero_words = 0;
    void *count_zero_ptr = nullptr;
    /* stages that get event pairs: "all", "" (none) or a comma list
     * (pm_set_stage_timing; env PM_STAGE_TIMERS=0 starts with none) */
    std::string timed_stages = "all";
    bool stage_active = false;
    StageEvents stage;             /* the stage being timed (g_stage points here) */
    bool stage_marker = false;
    std::map<std::string, TimerPool> timers;
};

#define FAIL(c, code, ...)                                                     \
    do {                                                                       \
        char _b[512];                                                          \
        snprintf(_b, sizeof(_b), __VA_ARGS__);                                 \
        if (c) (c)->err = _b;                                                  \
        g_last_error = _b;                                                     \
        pm::g_stage = nullptr; /* an error inside a timed stage ends it */    \
        return code;                                                           \
    } while (0)

#define HIPCHK(c, expr)                                                                   \
    do {                                                                                  \
        hipError_t _e = (expr);                                                           \
        if (_e != hipSuccess) FAIL(c, PM_ERR_HIP, "%s: %s", #expr, hipGetErrorString(_e)); \
    } while (0)

#define GETCTX(ptr)                                                                                      \
    Ctx *c = (Ctx *)(ptr);                                                                               \
    if (!c) FAIL((Ctx *)nullptr, PM_ERR_INVALID, "null context");                                        \
    if (c->group)                                                                                        \
        FAIL(c, PM_ERR_INVALID, "%s: a multi-device context takes the scene calls, pm_render and "       \
                                "pm_render_simple (the stage API needs one context per device)", __func__); \
    (void)hipSetDevice(c->device)

hipStream_t pick(Ctx *c, void *s) { return s ? (hipStream_t)s : c->stream; }

/* Single-process multi-device context (north_star: tiles and
 * photon batches over the GPUs of one node, RCCL all-gather of the photon
 * slots before the gather): one sub-context per device holds the whole
 * scene and record set; pm_render shards the paths by global id, all-gathers
 * the 40-B slots into every device's buffer (ncclAllGather over xGMI when the
 * devices are distinct, peer copies otherwise), builds the same map on every
 * device and gathers interleaved 8-row bands per device (pmrender/dist.py
 * _bands: runs of bands dealt round-robin, about four per device). */
struct Group {
    std::vector<Ctx *> subs;
    std::vector<int> devs;
    std::vector<ncclComm_t> comms; /* empty: peer-copy exchange */
    std::vector<hipEvent_t> ev;    /* per sub: end of its trace (peer-copy exchange) */
};
Group *group_of(void *ptr) { return ptr ? ((Ctx *)ptr)->group : nullptr; }
int group_fail(void *ptr, Ctx *sub, int rc) {
    Ctx *c = (Ctx *)ptr;
    c->err = "device " + std::to_string(sub->device) + ": " + sub->err;
    g_last_error = c->err;
    return rc;
}
/* scene calls go to every device's context */
#define GROUP_FWD(ptr, CALL)                                                                                  \
    if (Group *g_ = group_of(ptr)) {                                                                          \
        for (Ctx *sub : g_->subs) {                                                                           \
            const int rc_ = (CALL);                                                                           \
            if (rc_) return group_fail(ptr, sub, rc_);                                                        \
        }                                                                                                     \
        return PM_OK;                                                                                         \
    }

} // namespace
thread_local pm::StageEvents *pm::g_stage = nullptr;
namespace {

/* Every stage launch takes a fresh event pair from a per-stage pool. Kernel
 * stages bind the pair to their own dispatches (pm_launch, pm_kernels.h):
 * no marker packets, so timing leaves no idle gap between kernels. A stage
 * of host work / copies (marker = true) records the pair as markers.
 * Nothing synchronizes until a reader asks. */
bool stage_timed(const Ctx *c, const char *name) {
    const std::string &t = c->timed_stages;
    if (t == "all") return true;
    const size_t n = strlen(name);
    for (size_t i = 0; i < t.size();) {
        size_t j = t.find(',', i);
        if (j == std::string::npos) j = t.size();
        if (j - i == n && t.compare(i, n, name) == 0) return true;
        i = j + 1;
    }
    return false;
}
int timer_begin(Ctx *c, const char *name, hipStream_t s, bool marker = false) {
    c->stage_active = stage_timed(c, name);
    if (!c->stage_active) return 0;
    TimerPool &tp = c->timers[name];
    if (tp.used == tp.ev.size()) {
        Timer t;
        /* timing-only events: no system-scope fence (cache write-back +
         * invalidate) when recorded */
        (void)hipEventCreateWithFlags(&t.a, hipEventDisableSystemFence);
        (void)hipEventCreateWithFlags(&t.b, hipEventDisableSystemFence);
        tp.ev.push_back(t);
    }
    const Timer &t = tp.ev[tp.used];
    c->stage = StageEvents{t.a, t.b, 0};
    c->stage_marker = marker;
    if (marker) {
        (void)hipEventRecord(t.a, s);
        c->stage.launched = 1; /* start taken: kernels only move the stop */
    }
    g_stage = &c->stage;
    return 0;
}
void timer_end(Ctx *c, const char *name, hipStream_t s) {
    if (!c->stage_active) return;
    c->stage_active = false;
    g_stage = nullptr;
    TimerPool &tp = c->timers[name];
    const Timer &t = tp.ev[tp.used];
    if (c->stage.launched == 0) (void)hipEventRecord(t.a, s); /* nothing launched: an empty interval */
    if (c->stage_marker || c->stage.launched == 0) (void)hipEventRecord(t.b, s);
    tp.used++;
}
double pair_ms(const Timer &t) {
    (void)hipEventSynchronize(t.b);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t.a, t.b) != hipSuccess) return -1.0;
    return ms;
}
/* duration of the most recent launch of a stage (k > 1: the sum of the last k) */
double timer_ms(Ctx *c, const char *name, size_t k = 1) {
    auto it = c->timers.find(name);
    if (it == c->timers.end() || it->second.used == 0) return -1.0;
    double ms = 0;
    for (size_t i = it->second.used - std::min(k, it->second.used); i < it->second.used; ++i) ms += pair_ms(it->second.ev[i]);
    return ms;
}

inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
inline float ibits(int v) { float f; std::memcpy(&f, &v, 4); return f; }
inline int fbits_h(float f) { int v; std::memcpy(&v, &f, 4); return v; }
inline float bits_f(uint32_t v) { float f; std::memcpy(&f, &v, 4); return f; }

/* Normalized shading frame of one triangle: the same IEEE float operations
 * in the same order as the closest-hit program (cudatrianglemesh.cu:36-78,
 * then normalize as cudamaterial.cu.h:84-85), so the device reads values
 * bit-identical to computing them per hit. n = e1 x e0 as in tri_geo. */
void tri_frame(const float *p0, const float *p1, const float *p2, const float *UV, const int *v, const float *n,
               float *ns, float *dpdu) {
    float uv0x = 0.f, uv0y = 0.f, uv1x = 1.f, uv1y = 0.f, uv2x = 0.f, uv2y = 1.f;
    if (UV) {
        uv0x = UV[2 * v[0]]; uv0y = UV[2 * v[0] + 1];
        uv1x = UV[2 * v[1]]; uv1y = UV[2 * v[1] + 1];
        uv2x = UV[2 * v[2]]; uv2y = UV[2 * v[2] + 1];
    }
    const float du1 = uv0x - uv2x, du2 = uv1x - uv2x, dv1 = uv0y - uv2y, dv2 = uv1y - uv2y;
    const float determinant = du1 * dv2 - dv1 * du2;
    float d[3];
    if (determinant == 0.0f) {
        if (std::fabs(n[0]) > std::fabs(n[1])) {
            float invLen = 1.f / std::sqrt(n[0] * n[0] + n[2] * n[2]);
            d[0] = -n[2] * invLen; d[1] = 0.f; d[2] = n[0] * invLen;
        } else {
            float invLen = 1.f / std::sqrt(n[1] * n[1] + n[2] * n[2]);
            d[0] = 0.f; d[1] = n[2] * invLen; d[2] = n[1] * invLen;
        }
    } else {
        const float invdet = 1.f / determinant;
        for (int a = 0; a < 3; ++a) {
            float dp1 = p0[a] - p2[a], dp2 = p1[a] - p2[a];
            d[a] = (dv2 * dp1 - dv1 * dp2) * invdet;
        }
    }
    auto normalize3 = [](const float *x, float *out) {
        float inv = 1.0f / std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
        for (int a = 0; a < 3; ++a) out[a] = x[a] * inv;
    };
    normalize3(n, ns);
    normalize3(d, dpdu);
}

int64_t num_records(const Ctx *c) {
    if (c->pinhole) return (int64_t)((c->W + 7) / 8) * ((c->H + 7) / 8) * 64;
    return c->nrays;
}

/* pbrt-v2 PermutedHalton(5, RNG(seed)) table (montecarlo.h GeneratePermutation
 * + Shuffle over MT19937 == std::mt19937; photonmappingrenderer.cpp:216). */
void halton_perm(uint32_t seed, uint32_t out[28]) {
    std::mt19937 rng(seed);
    const uint32_t primes[5] = {2, 3, 5, 7, 11};
    uint32_t *p = out;
    for (int d = 0; d < 5; ++d) {
        uint32_t b = primes[d];
        for (uint32_t i = 0; i < b; ++i) p[i] = i;
        for (uint32_t i = 0; i < b; ++i) {
            uint32_t other = i + ((uint32_t)rng() % (b - i));
            std::swap(p[i], p[other]);
        }
        p += b;
    }
}

/* the records' radii changed in a way that may raise them (eye pass, reset,
 * upload, set_radius2, kNN radii): the adaptive grid falls back to the
 * initial radius, and bins accumulated from the old radii are dropped */
static void r2_invalidate(Ctx *c) {
    c->r2_valid = false;
    c->design_r2 = 0.f;
    if (c->r2_accum) { c->r2_accum = false; c->r2_dirty = true; }
}

/* the deferred zero fill of a lazy_zero trace, on stream s after the trace
 * (s == nullptr: on the trace's own stream, waited for) */
static int materialize_slots(Ctx *c, hipStream_t s) {
    if (c->slots_dirty <= 0) return PM_OK;
    const bool wait = s == nullptr;
    if (wait) s = c->stream;
    HIPCHK(c, hipStreamWaitEvent(s, c->dirty_event, 0));
    HIPCHK(c, launch_zero_invalid_slots(c->d_slots.as<pm_photon>(), c->d_scratch.as<uint32_t>(), c->slots_dirty,
                                        c->dirty_key_np, c->dirty_mpc, s));
    c->slots_dirty = 0;
    if (wait) HIPCHK(c, hipStreamSynchronize(s));
    return PM_OK;
}

template <class T>
int upload(Ctx *c, DevBuf &b, const std::vector<T> &v) {
    HIPCHK(c, b.ensure(std::max<size_t>(v.size() * sizeof(T), 16)));
    if (!v.empty()) HIPCHK(c, hipMemcpy(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return PM_OK;
}

int ensure_records(Ctx *c) {
    int64_t n = num_records(c);
    if (n <= 0) FAIL(c, PM_ERR_INVALID, "no eye samples (call pm_set_pinhole or pm_set_eye_rays)");
    HIPCHK(c, c->d_pos.ensure(n * sizeof(float4)));
    HIPCHK(c, c->d_nrm.ensure(n * sizeof(float4)));
    HIPCHK(c, c->d_state.ensure(n * sizeof(float4)));
    HIPCHK(c, c->d_n.ensure(n * sizeof(float)));
    HIPCHK(c, c->d_dl.ensure(n * sizeof(float4)));
    c->nrec = n;
    c->tiles_valid = false;
    r2_invalidate(c);
    return PM_OK;
}

RecordsDev recs(Ctx *c) {
    RecordsDev R;
    R.pos = c->d_pos.as<float4>(); R.nrm = c->d_nrm.as<float4>(); R.state = c->d_state.as<float4>();
    R.n = c->d_n.as<float>(); R.dl = c->d_dl.as<float4>(); R.count = c->nrec;
    return R;
}

/* cells per axis of a box of width 2 r' (r' of radius2) on grid g: the tile
 * kernel's run count (GatherParams::span), clamped to its instances 2..5
 * (larger boxes scan per lane) */
int grid_span(const GridDesc &g, float radius2) {
    const double rq = sqrt((double)radius2) * 1.0001 + 1e-4;
    const double w = 2.0 * rq * (double)g.inv_cs * (1.0 + 1e-6);
    return std::max(2, std::min(5, (int)std::floor(w) + 2));
}

GatherParams gather_params(Ctx *c, const pm_render_params *p) {
    GatherParams G{};
    G.R = recs(c);
    G.materials = c->S.materials;
    G.ppm_alpha = p->ppm_alpha;
    G.grid = c->grid;
    G.cell_start = c->d_cell_start.as<uint32_t>();
    G.ph_a = c->d_pha.as<float4>(); G.ph_b = c->d_phb.as<float4>();
    G.kd_nodes = c->d_kd.as<pm_photon>(); G.kd_count = c->kd_count;
    G.counters = c->d_counters.as<unsigned long long>();
    G.kernel = c->gather_kernel;
    G.kd_stack = c->kd_stack;
    G.error = reinterpret_cast<unsigned int *>(c->d_counters.as<unsigned long long>() + 16);
    G.fx_nonneg = c->scene_nonneg && c->slots_nonneg ? 1 : 0;
    G.span = grid_span(c->grid, c->grid_r2 > 0.f ? c->grid_r2 : p->initial_radius2);
    /* The cooperative scan of a tile's direct lanes costs the sum of their
     * photons / 64 steps, the per-lane scans the largest lane's photons but
     * one scattered line per lane and load. Scenes traversed from HBM (many
     * small primitives: C3's 1M-triangle soup) give incoherent tiles whose
     * lanes share no cells — the cooperative scan takes them all (same box:
     * C3 gather 0.458 -> 0.216 ms); LDS-sized scenes (the Cornell family)
     * give coherent direct lanes (a dense union's group, C5), which the
     * per-lane scans serve from L1, so only light waves (<= 8 steps) go
     * cooperative (C5: all 0.214 ms vs 0.170 bounded). */
    G.coop_steps = scene_mode(c->S) == MODE_GLOBAL ? 0xffffffu : 8u;
    if (c->view_active) { G.view_rank = c->d_vrank.as<uint32_t>(); G.view_list = c->d_vlist.as<uint32_t>(); }
    /* fixed-point scale 2^S: a single contribution is bounded by
     * alpha_max * Kd_max / pi with alpha_max = emission * Kd_max^mpc (Lambert
     * weight ~Kd, specular weight 1); x4 headroom; 2^40 per contribution
     * leaves 2^23 contributions per record before int64 overflow */
    double cmax = c->emit_max * std::pow(c->kd_max, (double)p->max_photon_count) * (c->kd_max / M_PI) * 4.0;
    int S = (int)std::floor(std::log2(std::ldexp(1.0, 40) / std::max(cmax, 1e-30)));
    S = std::max(-60, std::min(60, S));
    G.fx_scale = (float)std::ldexp(1.0, S);
    G.fx_inv = std::ldexp(1.0, -S);
    return G;
}

/* (re)builds the active-record view from the current records; synchronizes to read its size */
int build_view(Ctx *c, hipStream_t s) {
    const int64_t n = c->nrec;
    HIPCHK(c, c->d_vflags.ensure((size_t)(n + 1) * 4));
    HIPCHK(c, c->d_vrank.ensure((size_t)(n + 1) * 4));
    HIPCHK(c, c->d_vlist.ensure((size_t)std::max<int64_t>(n, 1) * 4));
    HIPCHK(c, c->d_vsums.ensure(scan_scratch_words(n + 1) * 4));
    HIPCHK(c, launch_record_view(recs(c), c->d_vflags.as<uint32_t>(), c->d_vrank.as<uint32_t>(),
                                 c->d_vlist.as<uint32_t>(), c->d_vsums.as<uint32_t>(), s));
    uint32_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, c->d_vrank.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    c->n_view = total;
    return PM_OK;
}

/* number of records the range-based record calls address */
int64_t view_size(const Ctx *c) { return c->view_active ? c->n_view : c->nrec; }
const uint32_t *view_list(Ctx *c) { return c->view_active ? c->d_vlist.as<uint32_t>() : nullptr; }

/* applies a deferred pm_reset_records before a reader that is not a fused full gather */
int materialize_reset(Ctx *c, hipStream_t s) {
    if (!c->rec_fresh) return PM_OK;
    timer_begin(c, "reset", s);
    HIPCHK(c, launch_reset_records(recs(c), c->rec_fresh_r2, s));
    timer_end(c, "reset", s);
    c->rec_fresh = false;
    return PM_OK;
}

int check_params(Ctx *c, const pm_render_params *p) {
    if (!p) FAIL(c, PM_ERR_INVALID, "null params");
    if (!c->committed) FAIL(c, PM_ERR_INVALID, "scene not committed (call pm_commit)");
    if (p->max_photon_count < 1 || p->max_photon_count > 64) FAIL(c, PM_ERR_INVALID, "max_photon_count out of range");
    if (p->light_source_index < 0 || p->light_source_index >= (int)c->lights.size())
        FAIL(c, PM_ERR_INVALID, "light_source_index %d out of range (%zu lights)", p->light_source_index,
             c->lights.size());
    if (!(p->initial_radius2 > 0.f)) FAIL(c, PM_ERR_INVALID, "initial_radius2 must be > 0");
    if (p->estimator != PM_ESTIMATOR_PPM && p->estimator != PM_ESTIMATOR_KNN)
        FAIL(c, PM_ERR_INVALID, "unknown estimator %d", p->estimator);
    if (p->estimator == PM_ESTIMATOR_KNN) {
        if (p->knn_lookup < 1 || p->knn_lookup > PM_KNN_MAX)
            FAIL(c, PM_ERR_INVALID, "knn_lookup must be in [1, %d]", PM_KNN_MAX);
        if (p->gather_structure != PM_GATHER_GRID)
            FAIL(c, PM_ERR_INVALID, "the kNN estimator runs on the photon buckets (PM_GATHER_GRID)");
    }
    return PM_OK;
}

/* where pm_commit put each section of the scene blob */
struct SceneLayout {
    size_t o_nodes = 0, o_refs = 0, o_geo = 0, o_shade = 0, o_tid = 0, o_info = 0, o_norms = 0, o_disks = 0,
           o_spheres = 0, o_mats = 0, o_lights = 0, o_wnodes = 0, bytes = 0;
    size_t o_insts = 0, o_objv = 0, o_objinfo = 0, o_objn = 0, o_objuv = 0, o_objmesh = 0; /* instancing */
    int64_t n_nodes = 0, n_refs = 0, n_tris = 0;
    bool id_order = false;
    int wide = 0, wide_stack = 0;
};

/* per triangle t: (p0, e0, e1, n) for the intersector, the normalized
 * shading frame for hits, vertex ids + mesh */
void tri_record(const Ctx *c, uint32_t t, float4 *geo, float4 *shade, int4 *info) {
    const float *V = c->P.data();
    const HTri &tr = c->tris[t];
    const HMesh &m = c->meshes[tr.mesh];
    const float *p0 = V + 3 * tr.v[0], *p1 = V + 3 * tr.v[1], *p2 = V + 3 * tr.v[2];
    float e0[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    float e1[3] = {p0[0] - p2[0], p0[1] - p2[1], p0[2] - p2[2]};
    float n[3] = {e1[1] * e0[2] - e1[2] * e0[1], e1[2] * e0[0] - e1[0] * e0[2], e1[0] * e0[1] - e1[1] * e0[0]};
    geo[0] = f4(p0[0], p0[1], p0[2], e0[0]);
    geo[1] = f4(e0[1], e0[2], e1[0], e1[1]);
    geo[2] = f4(e1[2], n[0], n[1], n[2]);
    float ns[3], dpdu[3];
    tri_frame(p0, p1, p2, m.has_uv ? &c->UV[0] : nullptr, tr.v, n, ns, dpdu);
    shade[0] = f4(ns[0], ns[1], ns[2], bits_f((uint32_t)m.material | (m.has_n ? 0x80000000u : 0u)));
    shade[1] = f4(dpdu[0], dpdu[1], dpdu[2], bits_f((uint32_t)m.light));
    *info = make_int4(tr.v[0], tr.v[1], tr.v[2], tr.mesh);
}

std::vector<float4> vertex_normals(const Ctx *c) {
    std::vector<float4> norms(c->N.size() / 3);
    for (size_t i = 0; i < norms.size(); ++i) norms[i] = f4(c->N[3 * i], c->N[3 * i + 1], c->N[3 * i + 2], 0.f);
    return norms;
}

/* PLOC neighbour radius (env PM_PLOC_RADIUS, 1..32). C3 trace per 1M paths
 * on the host-built PLOC tree (same box): r 1 5.87 ms, 2 4.70, 3 4.50, 4
 * 4.58–4.63, 8 5.12, 16 5.73; the binned-SAH tree 4.50–4.51 */
int ploc_radius() {
    const char *e = getenv("PM_PLOC_RADIUS");
    return e ? std::max(1, std::min(32, atoi(e))) : 3;
}

/* env PM_BVH_BUILD: "gpu" (the device PLOC build, pm_bvh_gpu.hip), "host"
 * (the binned-SAH host build), "ploc-host" (the device's algorithm on the
 * host: A/B and test oracle); unset or "auto": the device for scenes of at
 * least PM_BVH_GPU_MIN (65,536) primitives, whose host build dominated the
 * scene setup (C3: 0.28 s SAH of a 0.51 s commit) */
bool gpu_bvh_wanted(int64_t nprims) {
    const char *b = getenv("PM_BVH_BUILD");
    const std::string m = b ? b : "auto";
    int64_t gmin = 1 << 16;
    if (const char *e = getenv("PM_BVH_GPU_MIN")) gmin = std::max<int64_t>(2, atoll(e));
    const bool want = m == "gpu" ? nprims >= 2 : (m == "auto" && nprims >= gmin);
    if (!want || PM_BVH4_QUANT == 0) return false;
    /* the breadth-first renumbering of the host tree is a host-path switch */
    return getenv("PM_BVH4_BFS") == nullptr;
}

struct TmpBuf : DevBuf {
    ~TmpBuf() { release(); }
};

/* the scene blob with the BVH built on the device: boxes from the host's
 * parallel pass uploaded, gpu_bvh_build writes the 4-wide nodes and refs in
 * place, the triangle records (computed on the host in triangle-id order
 * while the device builds) are uploaded and permuted into storage order.
 * built = false: the caller runs the host build (the device tree exceeded a
 * limit the traversal has, or the build failed — reported on stderr) */
int commit_gpu_bvh(Ctx *c, const std::vector<BuildPrim> &prims, int64_t nt, SceneLayout &L, bool &built, bool ptimes) {
    built = false;
    const auto t0 = std::chrono::steady_clock::now();
    auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    const int n = (int)prims.size();
    GpuBvhIn in{};
    in.n = n;
    in.radius = ploc_radius();
    ploc_morton_frame(prims, in.frame_lo, in.frame_scale);
    std::vector<float4> geo(3 * (size_t)nt), shade(2 * (size_t)nt);
    std::vector<int4> info((size_t)nt);
    struct Joiner {
        std::thread t;
        ~Joiner() { if (t.joinable()) t.join(); }
    } records;
    records.t = std::thread([&] {
        parallel_for(nt, [&](int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; ++k) tri_record(c, (uint32_t)k, &geo[3 * k], &shade[2 * k], &info[k]);
        });
    });
    std::vector<float4> hb(2 * (size_t)n);
    parallel_for(n, [&](int64_t i0, int64_t i1) {
        for (int64_t i = i0; i < i1; ++i) {
            const BuildPrim &p = prims[i];
            hb[2 * i] = f4(p.lo[0], p.lo[1], p.lo[2], bits_f(p.ref));
            hb[2 * i + 1] = f4(p.hi[0], p.hi[1], p.hi[2], 0.f);
        }
    });
    TmpBuf d_box, d_tord, d_src;
    HIPCHK(c, d_box.ensure(hb.size() * sizeof(float4)));
    HIPCHK(c, hipMemcpy(d_box.p, hb.data(), hb.size() * sizeof(float4), hipMemcpyHostToDevice));
    in.box = d_box.as<float4>();
    /* blob sections in pm_commit's order; no binary tree (a 16-B placeholder) */
    const std::vector<float4> norms = vertex_normals(c);
    size_t off = 0;
    auto sect = [&](size_t bytes) { const size_t o = (off + 15) & ~(size_t)15; off = o + bytes; return o; };
    L.o_nodes = sect(16);
    L.o_refs = sect(4 * (size_t)n);
    L.o_geo = sect(48 * (size_t)nt);
    L.o_shade = sect(32 * (size_t)nt);
    L.o_tid = sect(4 * (size_t)nt);
    L.o_info = sect(16 * (size_t)nt);
    L.o_norms = sect(norms.size() * sizeof(float4));
    L.o_disks = sect(c->disks.size() * sizeof(float4));
    L.o_spheres = sect(c->spheres.size() * sizeof(float4));
    L.o_mats = sect(c->materials.size() * sizeof(float4));
    L.o_lights = sect(c->lights.size() * sizeof(LightDev));
    L.o_wnodes = sect(64 * (size_t)(n - 1));
    /* never LDS-resident: the LDS modes traverse the binary tree this path does not build */
    L.bytes = std::max<size_t>((off + 15) & ~(size_t)15, (size_t)LDS_SCENE_MAX + 16);
    HIPCHK(c, c->d_scene.ensure(L.bytes));
    char *base = c->d_scene.as<char>();
    HIPCHK(c, hipMemsetAsync(base + L.o_nodes, 0, 16, c->stream));
    auto put = [&](size_t o, const void *src, size_t bytes) {
        return bytes ? hipMemcpyAsync(base + o, src, bytes, hipMemcpyHostToDevice, c->stream) : hipSuccess;
    };
    HIPCHK(c, put(L.o_norms, norms.data(), norms.size() * sizeof(float4)));
    HIPCHK(c, put(L.o_disks, c->disks.data(), c->disks.size() * sizeof(float4)));
    HIPCHK(c, put(L.o_spheres, c->spheres.data(), c->spheres.size() * sizeof(float4)));
    HIPCHK(c, put(L.o_mats, c->materials.data(), c->materials.size() * sizeof(float4)));
    HIPCHK(c, put(L.o_lights, c->lights.data(), c->lights.size() * sizeof(LightDev)));
    HIPCHK(c, d_tord.ensure(4 * (size_t)std::max<int64_t>(nt, 1)));
    GpuBvhOut out;
    out.wnodes = reinterpret_cast<uint4 *>(base + L.o_wnodes);
    out.refs = reinterpret_cast<uint32_t *>(base + L.o_refs);
    out.tri_order = d_tord.as<uint32_t>();
    out.max_nodes = n - 1;
    const double t_up = ms();
    const hipError_t e = gpu_bvh_build(in, out, c->stream);
    const double t_build = ms();
    if (e != hipSuccess) {
        (void)hipGetLastError();
        fprintf(stderr, "pm_commit: device BVH build failed (%s); host build\n", hipGetErrorString(e));
        return PM_OK;
    }
    if (out.max_stack > BVH_STACK || out.n_tris != nt) {
        fprintf(stderr, "pm_commit: device BVH stack bound %d (limit %d), %lld triangles; host build\n", out.max_stack,
                BVH_STACK, (long long)out.n_tris);
        return PM_OK;
    }
    records.t.join();
    const double t_rec = ms();
    HIPCHK(c, d_src.ensure(96 * (size_t)std::max<int64_t>(nt, 1)));
    float4 *src_geo = d_src.as<float4>(), *src_shade = src_geo + 3 * nt;
    int4 *src_info = reinterpret_cast<int4 *>(src_shade + 2 * nt);
    HIPCHK(c, hipMemcpyAsync(src_geo, geo.data(), geo.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(src_shade, shade.data(), shade.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(src_info, info.data(), info.size() * sizeof(int4), hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, launch_tri_permute(d_tord.as<uint32_t>(), nt, src_geo, src_shade, src_info,
                                 reinterpret_cast<float4 *>(base + L.o_geo), reinterpret_cast<float4 *>(base + L.o_shade),
                                 reinterpret_cast<uint32_t *>(base + L.o_tid), reinterpret_cast<int4 *>(base + L.o_info),
                                 c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (ptimes)
        fprintf(stderr, "pm_commit: device build: boxes up %.1f ms, PLOC + collapse %.1f ms (%d rounds, %lld nodes, depth %d, "
                        "stack %d), records %.1f ms, permute %.1f ms\n", t_up, t_build - t_up, out.rounds,
                (long long)out.nodes, out.depth, out.max_stack, t_rec, ms());
    c->bvh_depth = out.depth;
    c->bvh4_nodes = out.nodes;
    c->bvh4_depth = out.depth;
    L.n_nodes = out.nodes;
    L.n_refs = n;
    L.n_tris = nt;
    L.id_order = false;
    L.wide = 2;
    L.wide_stack = out.max_stack;
    built = true;
    return PM_OK;
}

} // namespace

extern "C" {

const char *pm_version(void) { return "pmhip 0.1 (gfx950)"; }

void pm_default_params(pm_render_params *p) {
    std::memset(p, 0, sizeof(*p));
    p->scene_epsilon = 0.1f;
    p->initial_radius2 = 4.0f;
    p->ppm_alpha = 0.7f;
    p->max_photon_count = 4;
    p->paths_per_pass = 512 * 512;
    p->passes = 1;
    p->light_source_index = 0;
    p->max_specular_depth = 10;
    p->rng_seed = 777u;
    p->light_rng_seed = 2047u;
    p->gather_structure = PM_GATHER_GRID;
    p->estimator = PM_ESTIMATOR_PPM;
    p->knn_lookup = 50; /* pbrt-v2 PhotonIntegrator "nused" */
}

int pm_create(void **out, const pm_config *cfg) {
    if (!out) FAIL((Ctx *)nullptr, PM_ERR_INVALID, "null output pointer");
    *out = nullptr;
    if (cfg && cfg->n_devices > 0) { /* multi-device context (Group) */
        if (!cfg->devices || cfg->n_devices > 64) FAIL((Ctx *)nullptr, PM_ERR_INVALID, "bad device list");
        Ctx *gc = new Ctx();
        gc->group = new Group();
        Group &G = *gc->group;
        bool distinct = true;
        for (int i = 0; i < cfg->n_devices; ++i) {
            pm_config one{};
            one.device = cfg->devices[i];
            void *sub = nullptr;
            if (pm_create(&sub, &one) != PM_OK) {
                const std::string e = g_last_error;
                pm_destroy(gc);
                FAIL((Ctx *)nullptr, PM_ERR_HIP, "device %d: %s", cfg->devices[i], e.c_str());
            }
            for (int d : G.devs) distinct = distinct && d != one.device;
            /* a device's trace covers one shard of the all-gathered slots, so
             * counts fused into it would never match the build: not made */
            if (cfg->n_devices > 1) ((Ctx *)sub)->fuse_ok = false;
            G.subs.push_back((Ctx *)sub);
            G.devs.push_back(one.device);
            hipEvent_t ev = nullptr;
            (void)hipSetDevice(one.device);
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
                pm_destroy(gc);
                FAIL((Ctx *)nullptr, PM_ERR_HIP, "hipEventCreate on device %d", one.device);
            }
            G.ev.push_back(ev);
        }
        gc->device = G.devs[0];
        const char *re = getenv("PM_GROUP_RCCL"); /* 0: peer copies even on distinct devices */
        if (distinct && !(re && atoi(re) == 0)) {
            G.comms.resize(G.devs.size());
            const ncclResult_t r = ncclCommInitAll(G.comms.data(), (int)G.devs.size(), G.devs.data());
            if (r != ncclSuccess) {
                G.comms.clear();
                pm_destroy(gc);
                FAIL((Ctx *)nullptr, PM_ERR_HIP, "ncclCommInitAll over %d devices: %s", cfg->n_devices, ncclGetErrorString(r));
            }
        } else if (distinct) {
            for (int a : G.devs)
                for (int b : G.devs)
                    if (a != b) { (void)hipSetDevice(a); (void)hipDeviceEnablePeerAccess(b, 0); }
            (void)hipGetLastError(); /* already-enabled peers are not errors here */
        }
        *out = gc;
        return PM_OK;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0)
        FAIL((Ctx *)nullptr, PM_ERR_HIP, "no HIP device available (%s)", hipGetErrorString(e));
    int dev = cfg ? cfg->device : 0;
    if (dev < 0 || dev >= ndev) FAIL((Ctx *)nullptr, PM_ERR_INVALID, "device %d out of range (%d devices)", dev, ndev);
    Ctx *c = new Ctx();
    c->device = dev;
    if (const char *e = getenv("PM_GATHER_KERNEL"))
        c->gather_kernel = !strcmp(e, "lane") ? PM_GK_LANE : PM_GK_TILE;
    if (const char *e = getenv("PM_KNN_SS")) c->knn_ss = atoi(e) != 0;
    if (const char *e = getenv("PM_CELL_SPAN")) c->cell_span = std::max(2, std::min(5, atoi(e)));
    if (const char *e = getenv("PM_TILE_SORT")) c->tile_sort = atoi(e) != 0;
    if (const char *e = getenv("PM_LAZY_ZERO")) c->lazy_zero = atoi(e) != 0;
    if (const char *e = getenv("PM_GRID_QUANTILE")) c->grid_quantile = atof(e);
    if (const char *e = getenv("PM_TRACE_HOLD")) c->trace_hold = atoi(e) != 0;
    if (const char *e = getenv("PM_TRACE_POOL")) c->trace_pool = atoi(e) != 0;
    if (const char *e = getenv("PM_POOL_STACK")) c->pool_stack = std::max(0, atoi(e));
    if (const char *e = getenv("PM_KD_STACK")) c->kd_stack = std::max(1, std::min(KD_STACK, atoi(e)));
    if (const char *e = getenv("PM_STAGE_TIMERS")) if (atoi(e) == 0) c->timed_stages.clear();
    (void)hipSetDevice(dev);
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        FAIL((Ctx *)nullptr, PM_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    e = c->d_counters.ensure(17 * sizeof(unsigned long long)); /* [gather x4][trace x4][trace profile x8][gather error] */
    if (e != hipSuccess) {
        delete c;
        FAIL((Ctx *)nullptr, PM_ERR_HIP, "hipMalloc: %s", hipGetErrorString(e));
    }
    *out = c;
    return PM_OK;
}

void pm_destroy(void *ptr) {
    Ctx *c = (Ctx *)ptr;
    if (!c) return;
    if (Group *g = c->group) {
        for (ncclComm_t cm : g->comms) (void)ncclCommDestroy(cm);
        for (size_t i = 0; i < g->ev.size(); ++i) { (void)hipSetDevice(g->devs[i]); (void)hipEventDestroy(g->ev[i]); }
        for (Ctx *sub : g->subs) pm_destroy(sub);
        delete g;
        delete c;
        return;
    }
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto &kv : c->timers)
        for (Timer &t : kv.second.ev) {
            (void)hipEventDestroy(t.a);
            (void)hipEventDestroy(t.b);
        }
    DevBuf *bufs[] = {&c->d_scene, &c->d_rays, &c->d_rand2d, &c->d_pos, &c->d_nrm, &c->d_state, &c->d_n,
                      &c->d_dl, &c->d_slots, &c->d_count, &c->d_scratch, &c->d_vflags, &c->d_vrank, &c->d_vlist, &c->d_vsums,
                      &c->d_cell_start, &c->d_pha, &c->d_phb, &c->d_knnpk, &c->d_knnovf, &c->d_tile_times, &c->d_tile_cost, &c->d_tiles2,
                      &c->d_kd, &c->d_out, &c->d_counters, &c->d_tiles, &c->d_tile_flags, &c->d_tile_count,
                      &c->d_r2hist, &c->d_spill};
    for (DevBuf *b : bufs) b->release();
    if (c->tile_event) (void)hipEventDestroy(c->tile_event);
    if (c->r2_event) (void)hipEventDestroy(c->r2_event);
    if (c->dirty_event) (void)hipEventDestroy(c->dirty_event);
    if (c->h_r2hist) (void)hipHostFree(c->h_r2hist);
    if (c->h_tile_count) (void)hipHostFree(c->h_tile_count);
    (void)hipStreamDestroy(c->stream);
    delete c;
}

const char *pm_last_error(void *ptr) {
    Ctx *c = (Ctx *)ptr;
    return c ? c->err.c_str() : g_last_error.c_str();
}

int64_t pm_kdtree_build_host(const pm_photon *slots, int64_t nslots, pm_photon *nodes_out) {
    if (!slots || !nodes_out || nslots < 0) return -1;
    std::vector<pm_photon> nodes;
    int64_t m = build_kdtree_pbrt(slots, nslots, nodes);
    if (m > 0) std::memcpy(nodes_out, nodes.data(), (size_t)m * sizeof(pm_photon));
    return m;
}

int pm_halton_permutation(uint32_t seed, uint32_t out[28]) {
    if (!out) return PM_ERR_INVALID;
    halton_perm(seed, out);
    return PM_OK;
}

/* ------------------------------------------------------------------ scene */
int pm_add_material(void *ptr, int type, const float rgb[3], int *out_id) {
    GROUP_FWD(ptr, pm_add_material(sub, type, rgb, out_id));
    GETCTX(ptr);
    if (type != PM_MATTE && type != PM_MIRROR && type != PM_GLASS) FAIL(c, PM_ERR_INVALID, "bad material type %d", type);
    float r = rgb ? rgb[0] : 0.f, g = rgb ? rgb[1] : 0.f, b = rgb ? rgb[2] : 0.f;
    c->materials.push_back(f4(r, g, b, ibits(type)));
    if (out_id) *out_id = (int)c->materials.size() - 1;
    c->committed = false;
    return PM_OK;
}

int pm_add_trimesh(void *ptr, const float *P, int nverts, const int *idx, int ntris, const float *N, const float *uv,
                   int material, int light) {
    GROUP_FWD(ptr, pm_add_trimesh(sub, P, nverts, idx, ntris, N, uv, material, light));
    GETCTX(ptr);
    if (!P || !idx || nverts <= 0 || ntris <= 0) FAIL(c, PM_ERR_INVALID, "empty or null mesh");
    if (material < 0 || material >= (int)c->materials.size()) FAIL(c, PM_ERR_INVALID, "bad material id %d", material);
    for (int64_t i = 0; i < 3 * (int64_t)ntris; ++i)
        if (idx[i] < 0 || idx[i] >= nverts) FAIL(c, PM_ERR_INVALID, "vertex index %d out of range", idx[i]);
    if (c->next_tri_id + ntris >= ((int64_t)1 << 31)) FAIL(c, PM_ERR_INVALID, "too many triangles (global ids reach 2^31)");
    int64_t base = (int64_t)c->P.size() / 3;
    c->P.insert(c->P.end(), P, P + 3 * (size_t)nverts);
    if (N) c->N.insert(c->N.end(), N, N + 3 * (size_t)nverts);
    else c->N.insert(c->N.end(), 3 * (size_t)nverts, 0.f);
    if (uv) c->UV.insert(c->UV.end(), uv, uv + 2 * (size_t)nverts);
    else c->UV.insert(c->UV.end(), 2 * (size_t)nverts, 0.f);
    int mid = (int)c->meshes.size();
    c->meshes.push_back(HMesh{material, light, N != nullptr, uv != nullptr});
    for (int t = 0; t < ntris; ++t)
        c->tris.push_back(HTri{{(int)(base + idx[3 * t]), (int)(base + idx[3 * t + 1]), (int)(base + idx[3 * t + 2])}, mid,
                               (uint32_t)c->next_tri_id++});
    c->committed = false;
    return PM_OK;
}

int pm_add_object_mesh(void *ptr, const float *P, int nverts, const int *idx, int ntris, const float *N,
                       const float *uv, int material, int light, int *out_object) {
    GROUP_FWD(ptr, pm_add_object_mesh(sub, P, nverts, idx, ntris, N, uv, material, light, out_object));
    GETCTX(ptr);
    if (!P || !idx || nverts <= 0 || ntris <= 0) FAIL(c, PM_ERR_INVALID, "empty or null object mesh");
    if (material < 0 || material >= (int)c->materials.size()) FAIL(c, PM_ERR_INVALID, "bad material id %d", material);
    for (int64_t i = 0; i < 3 * (int64_t)ntris; ++i)
        if (idx[i] < 0 || idx[i] >= nverts) FAIL(c, PM_ERR_INVALID, "vertex index %d out of range", idx[i]);
    HObj o;
    o.P.assign(P, P + 3 * (size_t)nverts);
    if (N) o.N.assign(N, N + 3 * (size_t)nverts);
    if (uv) o.UV.assign(uv, uv + 2 * (size_t)nverts);
    o.idx.assign(idx, idx + 3 * (size_t)ntris);
    o.material = material; o.light = light; o.has_n = N != nullptr; o.has_uv = uv != nullptr;
    c->objs.push_back(std::move(o));
    if (out_object) *out_object = (int)c->objs.size() - 1;
    c->committed = false;
    return PM_OK;
}

int pm_add_mesh_instance(void *ptr, int object, const float o2w[16], const float w2o[16]) {
    GROUP_FWD(ptr, pm_add_mesh_instance(sub, object, o2w, w2o));
    GETCTX(ptr);
    if (object < 0 || object >= (int)c->objs.size()) FAIL(c, PM_ERR_INVALID, "bad object id %d", object);
    if (!o2w || !w2o) FAIL(c, PM_ERR_INVALID, "null instance transform");
    if (o2w[12] != 0.f || o2w[13] != 0.f || o2w[14] != 0.f || o2w[15] != 1.f)
        FAIL(c, PM_ERR_INVALID, "instance transform is not affine (flatten it with pm_add_trimesh)");
    /* every instance takes global ids for all of its triangles (as the
     * flattened scene would): heavy instancing must not wrap them */
    const int64_t n_obj_tris = (int64_t)(c->objs[object].idx.size() / 3);
    if (c->next_tri_id + n_obj_tris >= ((int64_t)1 << 31))
        FAIL(c, PM_ERR_INVALID, "too many instanced triangles (global ids reach 2^31)");
    HInst in;
    in.obj = object;
    std::memcpy(in.m, o2w, sizeof in.m);
    std::memcpy(in.minv, w2o, sizeof in.minv);
    in.gid_base = (uint32_t)c->next_tri_id;
    c->next_tri_id += n_obj_tris;
    c->insts.push_back(in);
    c->committed = false;
    return PM_OK;
}

/* an instance's world vertex as pbrt's Transform::operator()(Point) computes
 * it for an affine transform (w == 1): the device's inst_point, bit for bit */
static inline void inst_point_h(const float *m, const float *p, float *o) {
    for (int a = 0; a < 3; ++a) o[a] = m[4 * a] * p[0] + m[4 * a + 1] * p[1] + m[4 * a + 2] * p[2] + m[4 * a + 3];
}

int pm_add_sphere(void *ptr, float radius, const float o2w[16], const float w2o[16], int material, int light) {
    GROUP_FWD(ptr, pm_add_sphere(sub, radius, o2w, w2o, material, light));
    GETCTX(ptr);
    if (!o2w || !w2o || !(radius > 0.f)) FAIL(c, PM_ERR_INVALID, "bad sphere");
    if (material < 0 || material >= (int)c->materials.size()) FAIL(c, PM_ERR_INVALID, "bad material id %d", material);
    c->spheres.push_back(f4(w2o[0], w2o[1], w2o[2], w2o[3]));
    c->spheres.push_back(f4(w2o[4], w2o[5], w2o[6], w2o[7]));
    c->spheres.push_back(f4(w2o[8], w2o[9], w2o[10], w2o[11]));
    c->spheres.push_back(f4(radius, ibits(material), ibits(light), ibits(0)));
    c->sphere_o2w.insert(c->sphere_o2w.end(), o2w, o2w + 16);
    c->committed = false;
    return PM_OK;
}

/* derived uniforms as cudadisk.cpp:24-43 computes them */
int pm_add_disk(void *ptr, const float o[3], const float x[3], const float y[3], const float z[3], float inner,
                float phimax, int material, int light) {
    GROUP_FWD(ptr, pm_add_disk(sub, o, x, y, z, inner, phimax, material, light));
    GETCTX(ptr);
    if (!o || !x || !y || !z) FAIL(c, PM_ERR_INVALID, "null disk vector");
    if (material < 0 || material >= (int)c->materials.size()) FAIL(c, PM_ERR_INVALID, "bad material id %d", material);
    float inv_rx2 = 1.f / (x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    float inv_ry2 = 1.f / (y[0] * y[0] + y[1] * y[1] + y[2] * y[2]);
    float moffset = o[0] * z[0] + o[1] * z[1] + o[2] * z[2];
    c->disks.push_back(f4(o[0], o[1], o[2], inner));
    c->disks.push_back(f4(x[0], x[1], x[2], phimax));
    c->disks.push_back(f4(y[0], y[1], y[2], moffset));
    c->disks.push_back(f4(z[0], z[1], z[2], inv_rx2));
    c->disks.push_back(f4(inv_ry2, ibits(material), ibits(light), ibits(0)));
    c->committed = false;
    return PM_OK;
}

int pm_add_light_point(void *ptr, const float pos[3], const float I[3]) {
    GROUP_FWD(ptr, pm_add_light_point(sub, pos, I));
    GETCTX(ptr);
    if (!pos || !I) FAIL(c, PM_ERR_INVALID, "null point light");
    LightDev L{};
    L.o_type = f4(pos[0], pos[1], pos[2], ibits(PM_LIGHT_POINT));
    L.p1_ns = f4(0, 0, 0, ibits(1)); /* nSample = 1, cudalight.cpp:22 */
    L.p2_r2d = f4(0, 0, 0, ibits(0));
    L.n_area = f4(0, 0, 0, 0);
    L.le = f4(I[0], I[1], I[2], 0);
    c->lights.push_back(L);
    c->committed = false;
    return PM_OK;
}

int pm_add_light_disk(void *ptr, const float o[3], const float p1[3], const float p2[3], const float n[3],
                      const float Le[3], float area, int nsamples) {
    GROUP_FWD(ptr, pm_add_light_disk(sub, o, p1, p2, n, Le, area, nsamples));
    GETCTX(ptr);
    if (!o || !p1 || !p2 || !n || !Le) FAIL(c, PM_ERR_INVALID, "null disk light vector");
    int ns = std::max(1, nsamples);
    LightDev L{};
    L.o_type = f4(o[0], o[1], o[2], ibits(PM_LIGHT_AREA_DISK));
    L.p1_ns = f4(p1[0], p1[1], p1[2], ibits(ns));
    L.p2_r2d = f4(p2[0], p2[1], p2[2], ibits(c->rand2d_total)); /* CudaSample::Add2D offset */
    L.n_area = f4(n[0], n[1], n[2], area);
    L.le = f4(Le[0], Le[1], Le[2], 0);
    c->rand2d_total += ns;
    c->lights.push_back(L);
    c->committed = false;
    return PM_OK;
}

int pm_set_pinhole(void *ptr, const float eye[3], const float fwd[3], const float right[3], const float up[3], int W,
                   int H) {
    GROUP_FWD(ptr, pm_set_pinhole(sub, eye, fwd, right, up, W, H));
    GETCTX(ptr);
    if (W <= 0 || H <= 0 || !eye || !fwd || !right || !up) FAIL(c, PM_ERR_INVALID, "bad pinhole camera");
    c->pinhole = 1; c->W = W; c->H = H;
    std::memcpy(c->eye, eye, 12); std::memcpy(c->fwd, fwd, 12);
    std::memcpy(c->right, right, 12); std::memcpy(c->up, up, 12);
    return PM_OK;
}

int pm_set_eye_rays(void *ptr, const float *rays, int64_t nrays, const float *rand2d, int n2d) {
    GROUP_FWD(ptr, pm_set_eye_rays(sub, rays, nrays, rand2d, n2d));
    GETCTX(ptr);
    if (!rays || nrays <= 0) FAIL(c, PM_ERR_INVALID, "no rays");
    c->pinhole = 0;
    c->nrays = nrays;
    c->rays.assign(rays, rays + 6 * nrays);
    c->n2d = (rand2d && n2d > 0) ? n2d : 0;
    if (c->n2d) c->rand2d.assign(rand2d, rand2d + (size_t)2 * n2d * nrays);
    else c->rand2d.clear();
    HIPCHK(c, c->d_rays.ensure(c->rays.size() * sizeof(float)));
    HIPCHK(c, hipMemcpy(c->d_rays.p, c->rays.data(), c->rays.size() * sizeof(float), hipMemcpyHostToDevice));
    if (c->n2d) {
        HIPCHK(c, c->d_rand2d.ensure(c->rand2d.size() * sizeof(float)));
        HIPCHK(c, hipMemcpy(c->d_rand2d.p, c->rand2d.data(), c->rand2d.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    return PM_OK;
}

/* the object meshes of an instanced scene (two-level trees) */
struct InstLayout {
    std::vector<uint32_t> qn;     /* every object's quantized 4-wide nodes, object 0 first (relocated by the caller) */
    std::vector<float4> insts;    /* 8 per instance (SceneDev::insts) */
    int max_stack = 0;            /* the deepest object tree's stack bound */
    size_t o_objv = 0, o_objinfo = 0, o_objn = 0, o_objuv = 0, o_objmesh = 0;
};

/* quantized 4-wide nodes moved to start at node `base`: internal child codes shift */
static void relocate_bvh4(std::vector<uint32_t> &q, uint32_t base) {
    for (size_t nd = 0; nd + 16 <= q.size(); nd += 16)
        for (int k = 0; k < 4; ++k) {
            const int16_t cnt = (int16_t)((q[nd + 10 + k / 2] >> (16 * (k & 1))) & 0xffffu);
            if (cnt == 0) q[nd + 12 + k] += base;
        }
}

/* Each object mesh once: its triangles (object space) in the leaf order of
 * its own binned-SAH tree, collapsed to 4-wide and quantized (every leaf a
 * LEAF_TRIS run of object slots); the instance records point at them. */
static int commit_objects(Ctx *c, std::vector<unsigned char> &blob,
                          const std::function<size_t(const void *, size_t)> &put, InstLayout &IL) {
    std::vector<float4> objv, objn, objuv;
    std::vector<int4> objinfo, objmesh;
    std::vector<uint32_t> root(c->objs.size()), slot0(c->objs.size());
    std::vector<int> stack(c->objs.size());
    uint32_t vbase = 0;
    for (size_t oi = 0; oi < c->objs.size(); ++oi) {
        const HObj &o = c->objs[oi];
        const int nt = (int)(o.idx.size() / 3);
        std::vector<BuildPrim> prims(nt);
        for (int t = 0; t < nt; ++t) {
            BuildPrim &bp = prims[t];
            for (int a = 0; a < 3; ++a) {
                const float v0 = o.P[3 * o.idx[3 * t] + a], v1 = o.P[3 * o.idx[3 * t + 1] + a], v2 = o.P[3 * o.idx[3 * t + 2] + a];
                const float lo = std::min(v0, std::min(v1, v2)), hi = std::max(v0, std::max(v1, v2));
                const float pad = 1e-4f * std::max(1.0f, std::max(fabsf(lo), fabsf(hi)));
                bp.lo[a] = lo - pad; bp.hi[a] = hi + pad;
            }
            bp.ref = (PRIM_TRI << 30) | (uint32_t)t;
        }
        BvhOut bvh;
        build_bvh(prims, BVH_STACK - 2, bvh);
        Bvh4Out w;
        collapse_bvh4(bvh, 1, w);
        /* storage: the tree's leaf order, at global object slots */
        const uint32_t s0 = (uint32_t)(objv.size() / 3);
        std::vector<uint32_t> refs(bvh.refs.size());
        for (size_t k = 0; k < bvh.refs.size(); ++k) {
            const uint32_t t = bvh.refs[k] & 0x3fffffffu;
            refs[k] = (PRIM_TRI << 30) | (s0 + (uint32_t)k);
            for (int q = 0; q < 3; ++q) {
                const float *v = &o.P[3 * (size_t)o.idx[3 * t + q]];
                objv.push_back(f4(v[0], v[1], v[2], q == 0 ? ibits((int)t) : 0.f));
            }
            objinfo.push_back(make_int4((int)vbase + o.idx[3 * t], (int)vbase + o.idx[3 * t + 1], (int)vbase + o.idx[3 * t + 2],
                                        (int)oi));
        }
        std::vector<uint32_t> qn;
        if (!quantize_bvh4(w.nodes, refs, qn)) FAIL(c, PM_ERR_INVALID, "object mesh %zu: tree not codable", oi);
        for (size_t nd = 0; nd + 16 <= qn.size(); nd += 16)
            for (int k = 0; k < 4; ++k) {
                const int16_t cnt = (int16_t)((qn[nd + 10 + k / 2] >> (16 * (k & 1))) & 0xffffu);
                if (cnt > 0 && !(cnt & LEAF_TRIS)) FAIL(c, PM_ERR_INVALID, "object mesh %zu: a leaf is not a triangle run", oi);
            }
        const uint32_t at = (uint32_t)(IL.qn.size() / 16);
        relocate_bvh4(qn, at);
        root[oi] = at;
        slot0[oi] = s0;
        stack[oi] = w.max_stack;
        IL.max_stack = std::max(IL.max_stack, w.max_stack);
        IL.qn.insert(IL.qn.end(), qn.begin(), qn.end());
        const int nv = (int)(o.P.size() / 3);
        for (int v = 0; v < nv; ++v) {
            objn.push_back(o.has_n ? f4(o.N[3 * v], o.N[3 * v + 1], o.N[3 * v + 2], 0.f) : f4(0.f, 0.f, 0.f, 0.f));
            objuv.push_back(o.has_uv ? f4(o.UV[2 * v], o.UV[2 * v + 1], 0.f, 0.f) : f4(0.f, 0.f, 0.f, 0.f));
        }
        vbase += (uint32_t)nv;
        objmesh.push_back(make_int4(o.material, o.light, o.has_n ? 1 : 0, o.has_uv ? 1 : 0));
    }
    for (const HInst &in : c->insts) {
        for (int r = 0; r < 3; ++r) IL.insts.push_back(f4(in.m[4 * r], in.m[4 * r + 1], in.m[4 * r + 2], in.m[4 * r + 3]));
        for (int r = 0; r < 3; ++r)
            IL.insts.push_back(f4(in.minv[4 * r], in.minv[4 * r + 1], in.minv[4 * r + 2], in.minv[4 * r + 3]));
        const int nt = (int)(c->objs[in.obj].idx.size() / 3);
        IL.insts.push_back(f4(ibits((int)root[in.obj]), ibits((int)slot0[in.obj]), ibits((int)in.gid_base), ibits(nt)));
        /* blas_isect's box pad, 1e-5 (a (2 |o| + W) + k B): a = |w2o|, W
         * bounds the world extent by |o2w| B + |translation|, k = |o2w| |w2o|
         * (infinity norms of the linear parts), B the object's extent */
        double B = 0.0, nm = 0.0, ni_ = 0.0, tr = 0.0;
        const std::vector<float> &P = c->objs[in.obj].P;
        for (float v : P) B = std::max(B, (double)fabsf(v));
        for (int r = 0; r < 3; ++r) {
            nm = std::max(nm, fabs(in.m[4 * r]) + fabs(in.m[4 * r + 1]) + fabs(in.m[4 * r + 2]));
            ni_ = std::max(ni_, fabs(in.minv[4 * r]) + fabs(in.minv[4 * r + 1]) + fabs(in.minv[4 * r + 2]));
            tr = std::max(tr, (double)fabsf(in.m[4 * r + 3]));
        }
        const double W = nm * B + tr;
        IL.insts.push_back(f4(ibits(stack[in.obj]), (float)(ni_ * 1.001), (float)((ni_ * W + nm * ni_ * B) * 1.001), 0.f));
    }
    IL.o_objv = put(objv.data(), objv.size() * sizeof(float4));
    IL.o_objinfo = put(objinfo.data(), objinfo.size() * sizeof(int4));
    IL.o_objn = put(objn.data(), objn.size() * sizeof(float4));
    IL.o_objuv = put(objuv.data(), objuv.size() * sizeof(float4));
    IL.o_objmesh = put(objmesh.data(), objmesh.size() * sizeof(int4));
    c->obj_tris_stored = (int64_t)objinfo.size();
    (void)blob;
    return PM_OK;
}

int pm_commit(void *ptr) {
    GROUP_FWD(ptr, pm_commit(sub));
    GETCTX(ptr);
    if (c->lights.empty()) FAIL(c, PM_ERR_INVALID, "scene has no lights");
    const int64_t nt = (int64_t)c->tris.size(), nd = (int64_t)c->disks.size() / 5,
                  ns = (int64_t)c->spheres.size() / 4;
    if (nt + nd + ns + (int64_t)c->insts.size() == 0) FAIL(c, PM_ERR_INVALID, "scene has no shapes");
    if (nt >= (1 << 30) || nd >= (1 << 30) || ns >= (1 << 30)) FAIL(c, PM_ERR_INVALID, "too many primitives");
    /* global ids: triangles (meshes and instances, in insertion order), then
     * disks, then spheres (tie-break order) */
    const int64_t nt_ids = (int64_t)c->next_tri_id;
    if (nt_ids + nd + ns >= (int64_t)1 << 31) FAIL(c, PM_ERR_INVALID, "too many primitives");
    for (int64_t i = 0; i < nd; ++i) c->disks[5 * i + 4].w = ibits((int)(nt_ids + i));
    for (int64_t i = 0; i < ns; ++i) c->spheres[4 * i + 3].w = ibits((int)(nt_ids + nd + i));
    const int64_t ni = (int64_t)c->insts.size();

    const auto t_commit0 = std::chrono::steady_clock::now();
    std::vector<BuildPrim> prims(nt);
    float blo[3] = {INFINITY, INFINITY, INFINITY}, bhi[3] = {-INFINITY, -INFINITY, -INFINITY};
    auto make_box = [](const float lo[3], const float hi[3], uint32_t ref) {
        BuildPrim bp;
        for (int a = 0; a < 3; ++a) {
            float pad = 1e-4f * std::max(1.0f, std::max(fabsf(lo[a]), fabsf(hi[a])));
            bp.lo[a] = lo[a] - pad; bp.hi[a] = hi[a] + pad;
        }
        bp.ref = ref;
        return bp;
    };
    auto add_box = [&](float lo[3], float hi[3], uint32_t ref) {
        for (int a = 0; a < 3; ++a) { blo[a] = std::min(blo[a], lo[a]); bhi[a] = std::max(bhi[a], hi[a]); }
        prims.push_back(make_box(lo, hi, ref));
    };
    const float *V = c->P.data();
    { /* triangle boxes in parallel chunks; the scene box merged per chunk */
        std::mutex mu;
        parallel_for(nt, [&](int64_t t0, int64_t t1) {
            float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int64_t t = t0; t < t1; ++t) {
                const HTri &tr = c->tris[t];
                float lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {
                    float v0 = V[3 * tr.v[0] + a], v1 = V[3 * tr.v[1] + a], v2 = V[3 * tr.v[2] + a];
                    lo[a] = std::min(v0, std::min(v1, v2)); hi[a] = std::max(v0, std::max(v1, v2));
                    clo[a] = std::min(clo[a], lo[a]); chi[a] = std::max(chi[a], hi[a]);
                }
                prims[t] = make_box(lo, hi, (PRIM_TRI << 30) | (uint32_t)t);
            }
            std::lock_guard<std::mutex> g(mu);
            for (int a = 0; a < 3; ++a) { blo[a] = std::min(blo[a], clo[a]); bhi[a] = std::max(bhi[a], chi[a]); }
        });
    }
    for (int64_t i = 0; i < nd; ++i) {
        const float4 *d = &c->disks[5 * i];
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int sx = -1; sx <= 1; sx += 2)
            for (int sy = -1; sy <= 1; sy += 2) { /* cudadisk.cu:87-96 */
                float p[3] = {d[0].x + sx * d[1].x + sy * d[2].x, d[0].y + sx * d[1].y + sy * d[2].y,
                              d[0].z + sx * d[1].z + sy * d[2].z};
                for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], p[a]); hi[a] = std::max(hi[a], p[a]); }
            }
        add_box(lo, hi, (PRIM_DISK << 30) | (uint32_t)i);
    }
    for (int64_t i = 0; i < ns; ++i) {
        const float *m = &c->sphere_o2w[16 * i];
        float r = c->spheres[4 * i + 3].x;
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int k = 0; k < 8; ++k) {
            float x = (k & 1) ? r : -r, y = (k & 2) ? r : -r, z = (k & 4) ? r : -r;
            float w[3] = {m[0] * x + m[1] * y + m[2] * z + m[3], m[4] * x + m[5] * y + m[6] * z + m[7],
                          m[8] * x + m[9] * y + m[10] * z + m[11]};
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], w[a]); hi[a] = std::max(hi[a], w[a]); }
        }
        add_box(lo, hi, (PRIM_SPHERE << 30) | (uint32_t)i);
    }
    /* instances: the box of the world vertices the device rebuilds */
    for (int64_t i = 0; i < ni; ++i) {
        const HInst &in = c->insts[i];
        const HObj &o = c->objs[in.obj];
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int v : o.idx) {
            float w[3];
            inst_point_h(in.m, &o.P[3 * (size_t)v], w);
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], w[a]); hi[a] = std::max(hi[a], w[a]); }
        }
        add_box(lo, hi, (PRIM_INST << 30) | (uint32_t)i);
    }
    /* env PM_COMMIT_TIMES=1: the build's phases on stderr (setup-time study) */
    const bool ptimes = getenv("PM_COMMIT_TIMES") != nullptr;
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto tms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    SceneLayout L;
    int rc;
    bool built = false;
    /* env PM_BVH8=1 (round 6): scenes traversed from HBM get an 8-wide
     * quantized tree (host build; pm_build.h quantize_bvh8) instead of the
     * 4-wide one; instanced scenes keep 4-wide trees */
    const bool bvh8 = ni == 0 && getenv("PM_BVH8") && atoi(getenv("PM_BVH8")) != 0;
    if (ni == 0 && !bvh8 && gpu_bvh_wanted((int64_t)prims.size())) {
        if ((rc = commit_gpu_bvh(c, prims, nt, L, built, ptimes))) return rc;
        if (ptimes && built) fprintf(stderr, "pm_commit: device build, total %.1f ms\n", tms(t_commit0, tnow()));
    }
    if (!built) {
        L = SceneLayout();
        BvhOut bvh;
        BvhCost cost;
        const auto t_build0 = tnow();
        /* env PM_BVH_BUILD=ploc-host: the device builder's PLOC tree built on
         * the host (A/B of the tree quality; PM_PLOC_RADIUS) */
        const char *bb = getenv("PM_BVH_BUILD");
        if (bb && std::strcmp(bb, "ploc-host") == 0 && prims.size() > 1) {
            PlocTree pt;
            build_ploc(prims, ploc_radius(), pt);
            ploc_to_bvh(prims, pt, bvh);
        } else {
            build_bvh(prims, BVH_STACK - 2, bvh, cost);
        }
        if (ptimes) fprintf(stderr, "pm_commit: %zu prims (boxes %.1f ms), host build %.1f ms\n", prims.size(),
                            tms(t_commit0, t_build0), tms(t_build0, tnow()));
        c->bvh_depth = bvh.depth;
        if (bvh.depth >= BVH_STACK) FAIL(c, PM_ERR_INVALID, "BVH too deep (%d)", bvh.depth);

        /* tiny LDS scenes skip the BVH (MODE_BRUTE). Their triangles are stored
         * in global-id order (brute_isect's tie-break relies on it), others in
         * leaf order. */
        const bool id_order = ni == 0 && (int64_t)bvh.refs.size() <= BRUTE_MAX_PRIMS;
        std::vector<uint32_t> tri_order; /* triangle ids in storage order */
        tri_order.reserve(nt);
        if (id_order) {
            for (int64_t t = 0; t < nt; ++t) tri_order.push_back((uint32_t)t);
        } else {
            for (uint32_t ref : bvh.refs)
                if ((ref >> 30) == PRIM_TRI) tri_order.push_back(ref & 0x3fffffffu);
        }
        std::vector<uint32_t> slot_of(nt);
        for (size_t k = 0; k < tri_order.size(); ++k) slot_of[tri_order[k]] = (uint32_t)k;
        parallel_for((int64_t)bvh.refs.size(), [&](int64_t i0, int64_t i1) {
            for (int64_t i = i0; i < i1; ++i) {
                uint32_t &ref = bvh.refs[i];
                if ((ref >> 30) == PRIM_TRI) ref = (PRIM_TRI << 30) | slot_of[ref & 0x3fffffffu];
            }
        });

        /* per-triangle precomputed (p0, e0, e1, n) for the intersector and the
         * normalized shading frame for hits (in parallel chunks of storage slots) */
        const int64_t nst = (int64_t)tri_order.size();
        std::vector<float4> tri_geo(3 * nst), tri_shade(2 * nst);
        std::vector<int4> tri_info(nst);
        std::vector<uint32_t> tri_id(nst);
        parallel_for(nst, [&](int64_t k0, int64_t k1) {
            for (int64_t k = k0; k < k1; ++k) {
                tri_record(c, tri_order[k], &tri_geo[3 * k], &tri_shade[2 * k], &tri_info[k]);
                tri_id[k] = c->tris[tri_order[k]].gid;
            }
        });
        if (ptimes) fprintf(stderr, "pm_commit: triangle records done at %.1f ms\n", tms(t_commit0, tnow()));
        const std::vector<float4> norms = vertex_normals(c);
        std::vector<float4> nodes4(bvh.nodes.size() / 4);
        std::memcpy(nodes4.data(), bvh.nodes.data(), bvh.nodes.size() * sizeof(float));

        /* one blob of 16-B aligned sections: the same offsets address it in HBM
         * and, for scenes that fit (SceneDev::lds_bytes), in each block's LDS copy */
        std::vector<unsigned char> blob;
        /* one reservation for every section (no regrowth copies of a 250 MB blob) */
        blob.reserve(16 * 16 + nodes4.size() * sizeof(float4) + bvh.refs.size() * 4 + tri_geo.size() * sizeof(float4) +
                     tri_shade.size() * sizeof(float4) + tri_id.size() * 4 + tri_info.size() * sizeof(int4) +
                     norms.size() * sizeof(float4) + (c->disks.size() + c->spheres.size() + c->materials.size()) * sizeof(float4) +
                     c->lights.size() * sizeof(LightDev) + (size_t)(bvh.nodes.size() / 16 + 1) * 64 * 2);
        auto put = [&](const void *src, size_t n) -> size_t {
            size_t off = (blob.size() + 15) & ~(size_t)15;
            blob.resize(off + n, 0);
            if (n) std::memcpy(&blob[off], src, n);
            return off;
        };
        L.o_nodes = put(nodes4.data(), nodes4.size() * sizeof(float4));
        L.o_refs = put(bvh.refs.data(), bvh.refs.size() * sizeof(uint32_t));
        L.o_geo = put(tri_geo.data(), tri_geo.size() * sizeof(float4));
        L.o_shade = put(tri_shade.data(), tri_shade.size() * sizeof(float4));
        L.o_tid = put(tri_id.data(), tri_id.size() * sizeof(uint32_t));
        L.o_info = put(tri_info.data(), tri_info.size() * sizeof(int4));
        L.o_norms = put(norms.data(), norms.size() * sizeof(float4));
        L.o_disks = put(c->disks.data(), c->disks.size() * sizeof(float4));
        L.o_spheres = put(c->spheres.data(), c->spheres.size() * sizeof(float4));
        L.o_mats = put(c->materials.data(), c->materials.size() * sizeof(float4));
        L.o_lights = put(c->lights.data(), c->lights.size() * sizeof(LightDev));
        /* instances: each object mesh's own tree and object-space triangles */
        InstLayout IL;
        if (ni > 0 && (rc = commit_objects(c, blob, put, IL))) return rc;
        /* scenes traversed from HBM also get the 4-wide BVH (half the dependent
         * node fetches per ray; binary leaves of one primitive);
         * instanced scenes always (their objects' trees are 4-wide) */
        bool wide8 = false;
        if (bvh8 && blob.size() > LDS_SCENE_MAX) {
            Bvh4Out w;
            collapse_bvh8(bvh, 1, w);
            std::vector<uint32_t> qn;
            if (quantize_bvh8(w.nodes, bvh.refs, qn) && w.max_stack <= BVH8_STACK) {
                L.o_wnodes = put(qn.data(), qn.size() * sizeof(uint32_t));
                L.wide = 3;
                L.wide_stack = w.max_stack;
                c->bvh4_nodes = (int64_t)(qn.size() / 32);
                c->bvh4_depth = w.depth;
                wide8 = true;
            }
        }
        if (!wide8 && (blob.size() > LDS_SCENE_MAX || ni > 0)) {
            {
                Bvh4Out w;
                const auto t_c0 = tnow();
                collapse_bvh4(bvh, 1, w);
                if (ptimes) fprintf(stderr, "pm_commit: collapse %.1f ms\n", tms(t_c0, tnow()));
                /* node format fixed at build time (pm_device.h PM_BVH4_QUANT) */
                std::vector<uint32_t> qn;
                const bool quant = PM_BVH4_QUANT != 0;
                /* a leaf the quantized count cannot code (>= LEAF_TRIS primitives,
                 * possible at build_bvh's depth limit) keeps the binary traversal,
                 * like a tree whose stack bound exceeds BVH_STACK. env
                 * PM_BVH4_BFS=1 renumbers the tree breadth-first, the order the
                 * device build produces (tests/test_bvh_gpu.py compares them) */
                const char *bf = getenv("PM_BVH4_BFS");
                if (bf && atoi(bf) != 0) bvh4_bfs_order(w.nodes);
                const auto t_q0 = tnow();
                const bool coded = !quant || quantize_bvh4(w.nodes, bvh.refs, qn);
                if (ptimes) fprintf(stderr, "pm_commit: quantize %.1f ms\n", tms(t_q0, tnow()));
                if (ni > 0 && !(coded && quant && w.max_stack + IL.max_stack + 1 <= BVH_STACK))
                    FAIL(c, PM_ERR_INVALID, "instanced scene: top-level tree not codable (stack %d + %d)", w.max_stack,
                         IL.max_stack);
                if (coded && w.max_stack <= BVH_STACK) {
                    if (ni > 0) { /* the objects' nodes follow the top-level tree's */
                        const uint32_t top = (uint32_t)(qn.size() / 16);
                        relocate_bvh4(IL.qn, top);
                        for (int64_t i = 0; i < ni; ++i) IL.insts[8 * i + 6].x = ibits(fbits_h(IL.insts[8 * i + 6].x) + (int)top);
                        qn.insert(qn.end(), IL.qn.begin(), IL.qn.end());
                        L.o_insts = put(IL.insts.data(), IL.insts.size() * sizeof(float4));
                    }
                    L.o_wnodes = quant ? put(qn.data(), qn.size() * sizeof(uint32_t))
                                       : put(w.nodes.data(), w.nodes.size() * sizeof(float));
                    L.wide = quant ? 2 : 1;
                    L.wide_stack = w.max_stack + (ni > 0 ? IL.max_stack : 0);
                    c->bvh4_nodes = (int64_t)(quant ? qn.size() / 16 : w.nodes.size() / 32);
                    c->bvh4_depth = w.depth;
                }
            }
        }
        blob.resize(std::max<size_t>((blob.size() + 15) & ~(size_t)15, 16), 0);
        /* instanced scenes never go LDS-resident (MODE_INST walks the 4-wide trees from HBM) */
        if (ni > 0 && blob.size() <= LDS_SCENE_MAX) blob.resize(LDS_SCENE_MAX + 16, 0);
        L.o_objv = IL.o_objv; L.o_objinfo = IL.o_objinfo; L.o_objn = IL.o_objn; L.o_objuv = IL.o_objuv;
        L.o_objmesh = IL.o_objmesh;
        const auto t_u0 = tnow();
        if ((rc = upload(c, c->d_scene, blob))) return rc;
        if (id_order) {
            /* triangle pairs for the brute-force loop: pair j = storage slots
             * 2j, 2j + 1, each of the 12 (p0, e0, e1, n) components as two
             * adjacent floats, so a scalar load puts the packed operand of
             * both triangles in an aligned SGPR pair */
            const int64_t np = nst / 2;
            std::vector<float> pairs((size_t)std::max<int64_t>(np, 1) * 24, 0.f);
            const float *geo = reinterpret_cast<const float *>(tri_geo.data());
            for (int64_t j = 0; j < np; ++j)
                for (int q = 0; q < 12; ++q)
                    for (int h = 0; h < 2; ++h) pairs[(size_t)j * 24 + 2 * q + h] = geo[(size_t)(2 * j + h) * 12 + q];
            if ((rc = upload(c, c->d_tripairs, pairs))) return rc;
        }
        if (ptimes) fprintf(stderr, "pm_commit: upload %.1f ms (%zu bytes), total %.1f ms\n", tms(t_u0, tnow()), blob.size(),
                            tms(t_commit0, tnow()));
        L.bytes = blob.size();
        L.n_nodes = (int64_t)nodes4.size() / 4;
        /* the traversal loops' guard: with instances it must cover an object's tree too */
        if (ni > 0) L.n_nodes = std::max<int64_t>(L.n_nodes, c->bvh4_nodes);
        L.n_refs = (int64_t)bvh.refs.size();
        L.n_tris = (int64_t)tri_info.size();
        L.id_order = id_order;
    }

    SceneDev &S = c->S;
    const char *base = c->d_scene.as<char>();
    S.blob = base;
    S.blob_bytes = (uint32_t)std::min<size_t>(L.bytes, 0xffffffffu);
    S.lds_bytes = L.bytes <= LDS_SCENE_MAX ? (uint32_t)L.bytes : 0u;
    S.nodes = (const float4 *)(base + L.o_nodes); S.refs = (const uint32_t *)(base + L.o_refs);
    S.tri_geo = (const float4 *)(base + L.o_geo); S.tri_shade = (const float4 *)(base + L.o_shade);
    S.tri_id = (const uint32_t *)(base + L.o_tid); S.tri_info = (const int4 *)(base + L.o_info);
    S.norms = (const float4 *)(base + L.o_norms); S.disks = (const float4 *)(base + L.o_disks);
    S.spheres = (const float4 *)(base + L.o_spheres); S.materials = (const float4 *)(base + L.o_mats);
    S.lights = (const LightDev *)(base + L.o_lights);
    S.n_lights = (int)c->lights.size(); S.n_nodes = (int)L.n_nodes;
    S.n_refs = (int)L.n_refs;
    S.n_tris = (int)L.n_tris; S.n_disks = (int)nd; S.n_spheres = (int)ns;
    S.tri_geo_g = S.tri_geo; S.tri_id_g = S.tri_id;
    S.tri_pairs_g = L.id_order ? c->d_tripairs.as<float>() : nullptr;
    S.n_inst = (int)ni;
    S.insts = ni ? (const float4 *)(base + L.o_insts) : nullptr;
    S.obj_v = ni ? (const float4 *)(base + L.o_objv) : nullptr;
    S.obj_info = ni ? (const int4 *)(base + L.o_objinfo) : nullptr;
    S.obj_n = ni ? (const float4 *)(base + L.o_objn) : nullptr;
    S.obj_uv = ni ? (const float4 *)(base + L.o_objuv) : nullptr;
    S.obj_mesh = ni ? (const int4 *)(base + L.o_objmesh) : nullptr;
    S.brute = (S.lds_bytes > 0 && L.id_order) ? 1 : 0;
    /* a push happens only when descending a level, so depth + 1 entries suffice;
     * sizing the LDS stack by the actual tree keeps occupancy VGPR-bound */
    S.stack_depth = std::min(BVH_STACK, std::max(2, c->bvh_depth + 2));
    S.wide = L.wide;
    S.wnodes = L.wide ? (const float4 *)(base + L.o_wnodes) : nullptr;
    /* wide scenes traverse only the 4-wide tree (traverse() dispatches every
     * MODE_GLOBAL query to traverse4): its exact stack bound sizes the LDS
     * stacks, not the binary tree's depth — k_trace_pool's 256-thread blocks
     * then fit four per CU (its VGPR occupancy) instead of three */
    if (L.wide) S.stack_depth = std::min(L.wide == 3 ? BVH8_STACK : BVH_STACK, std::max(2, L.wide_stack + 1));
    for (int a = 0; a < 3; ++a) { c->bbox_lo[a] = blo[a]; c->bbox_hi[a] = bhi[a]; }
    double em = 0.0, kd = 1.0;
    for (const LightDev &L : c->lights) {
        double le = std::max({std::fabs(L.le.x), std::fabs(L.le.y), std::fabs(L.le.z)});
        em = std::max(em, fbits_h(L.o_type.w) == PM_LIGHT_POINT ? le * 4.0 * M_PI : le * L.n_area.w * 2.0 * M_PI);
    }
    for (const float4 &m : c->materials)
        if (fbits_h(m.w) == PM_MATTE) kd = std::max({kd, (double)m.x, (double)m.y, (double)m.z});
    c->emit_max = std::max(em, 1e-30);
    c->kd_max = kd;
    bool nn = true;
    for (const LightDev &L : c->lights) nn = nn && L.le.x >= 0.f && L.le.y >= 0.f && L.le.z >= 0.f && L.n_area.w >= 0.f;
    for (const float4 &m : c->materials)
        if (fbits_h(m.w) == PM_MATTE) nn = nn && m.x >= 0.f && m.y >= 0.f && m.z >= 0.f;
    c->scene_nonneg = nn;
    c->committed = true;
    return PM_OK;
}

/* ------------------------------------------------------------- stages */
int pm_eye_pass(void *ptr, const pm_render_params *p, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if ((rc = ensure_records(c))) return rc;
    if (!c->pinhole && c->rand2d_total > c->n2d)
        FAIL(c, PM_ERR_INVALID, "eye rays carry %d 2D samples, lights need %d", c->n2d, c->rand2d_total);
    hipStream_t s = pick(c, stream);
    EyeParams E{};
    E.S = c->S;
    E.R = recs(c);
    E.pinhole = c->pinhole; E.W = c->W; E.H = c->H; E.n2d = c->n2d;
    E.eye = f4(c->eye[0], c->eye[1], c->eye[2], 0); E.fwd = f4(c->fwd[0], c->fwd[1], c->fwd[2], 0);
    E.right = f4(c->right[0], c->right[1], c->right[2], 0); E.up = f4(c->up[0], c->up[1], c->up[2], 0);
    E.rays = c->d_rays.as<float>(); E.rand2d = c->d_rand2d.as<float>();
    E.eps = p->scene_epsilon; E.r2init = p->initial_radius2; E.max_spec = p->max_specular_depth;
    E.light_seed = p->light_rng_seed;
    timer_begin(c, "eye", s);
    HIPCHK(c, launch_eye(E, s));
    timer_end(c, "eye", s);
    c->rec_fresh = false; /* the eye pass writes every record */
    c->tiles_valid = false;
    r2_invalidate(c);
    if (c->view_active && (rc = build_view(c, s))) return rc;
    return PM_OK;
}

int pm_reserve_slots(void *ptr, int64_t n, void **d_slots) {
    GETCTX(ptr);
    int rc;
    if (n < 0) FAIL(c, PM_ERR_INVALID, "negative slot count");
    if (d_slots) { /* the caller may read the buffer from now on: no lazy zero fill on it */
        if ((rc = materialize_slots(c, nullptr))) return rc;
        c->slots_exposed = true;
    }
    if ((size_t)n * sizeof(pm_photon) > c->d_slots.bytes) {
        if (c->d_slots.external)
            FAIL(c, PM_ERR_INVALID, "external slot buffer holds %zu slots, %lld needed",
                 c->d_slots.bytes / sizeof(pm_photon), (long long)n);
        /* keep the contents: grow by copy */
        DevBuf nb;
        HIPCHK(c, nb.ensure((size_t)n * sizeof(pm_photon)));
        if (c->d_slots.p) {
            HIPCHK(c, hipStreamSynchronize(c->stream));
            HIPCHK(c, hipMemcpy(nb.p, c->d_slots.p, c->d_slots.bytes, hipMemcpyDeviceToDevice));
            c->d_slots.release();
        }
        c->d_slots = nb;
        nb.p = nullptr;
    }
    if (d_slots) *d_slots = c->d_slots.p;
    return PM_OK;
}

int pm_set_slot_buffer(void *ptr, void *d, int64_t n) {
    GETCTX(ptr);
    int rc;
    if ((rc = materialize_slots(c, nullptr))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->d_slots.release();
    c->fused.valid = false;
    if (d) {
        if (n <= 0) FAIL(c, PM_ERR_INVALID, "external slot buffer needs n_slots > 0");
        c->d_slots.p = d;
        c->d_slots.bytes = (size_t)n * sizeof(pm_photon);
        c->d_slots.external = true;
    }
    c->slots_used = 0;
    return PM_OK;
}

/* photon-bucket grid of a render: cell edge 2 r_max / (span - 1) over the
 * scene box, so a query box [p - r', p + r'] spans <= span cells per axis
 * (PPM radii only shrink, so it holds for every pass of the render) */
/* radius^2 the PPM grid is designed for: the grid_quantile of the records'
 * current radii from the last landed histogram (k_gather_tile), else the
 * initial radius. Refreshed only where a photon map's grid is chosen
 * (pm_trace_photons with fused counting, or pm_build_photon_map without), so
 * the trace and the build of one pass agree. */
static float grid_radius2(Ctx *c, const pm_render_params *p, bool refresh, hipStream_t s) {
    const float init = p->initial_radius2;
    if (p->estimator == PM_ESTIMATOR_KNN || c->grid_quantile <= 0.0) return init;
    if (refresh) {
        /* a new pass. First a landed sum sets the grid radius (if it still
         * describes the records) ... */
        if (c->r2_pending && hipEventQuery(c->r2_event) == hipSuccess) {
            c->r2_pending = false;
            if (c->r2_valid && c->r2_hist_init == init) {
                uint64_t cnt[R2_BINS] = {0}, total = 0;
                for (int b = 0; b < R2_BINS; ++b) cnt[b] = ((volatile uint32_t *)c->h_r2hist)[b];
                for (int b = 0; b < R2_BINS; ++b) total += cnt[b];
                /* bins b.. hold t = r^2 / init <= 2^(-b/8): the largest b that still
                 * covers the quantile */
                int best = 0;
                uint64_t above = total;
                for (int b = 0; b < R2_BINS; ++b) {
                    if ((double)above < c->grid_quantile * (double)total) break;
                    best = b;
                    above -= cnt[b];
                }
                /* the bins come from an approximate log2: a small margin */
                c->design_r2 = total ? std::min(init, (float)(init * std::exp2(-best / (double)R2_PER_OCTAVE) * 1.01)) : 0.f;
            }
        }
        /* ... then the previous pass's gathers — all of its record ranges (a
         * group device's or an all-gather rank's bands) — binned their radii
         * into d_r2hist: sum them once, into host-mapped memory (not while a
         * sum is in flight: the pinned buffer is reused; the bins keep
         * accumulating, and older radii only overestimate) */
        if (c->r2_accum && !c->r2_pending &&
            launch_r2hist_reduce(c->d_r2hist.as<uint32_t>(), c->h_r2hist_dev, s) == hipSuccess &&
            hipEventRecord(c->r2_event, s) == hipSuccess) {
            c->r2_pending = true;
            c->r2_stream = s;
            c->r2_accum = false;
            c->r2_valid = true;
            c->r2_hist_init = c->r2_accum_init;
        }
        /* a pass that continues a render (no reset pending): its gathers bin
         * their radii for the passes after it */
        c->r2_wanted = !c->rec_fresh;
    }
    if (c->rec_fresh || !c->r2_valid || c->r2_hist_init != init) return init;
    return c->design_r2 > 0.f ? c->design_r2 : init;
}

static GridDesc make_grid(const Ctx *c, const pm_render_params *p, float radius2) {
    GridDesc g{};
    const float rq = sqrtf(radius2) * 1.0001f + 1e-4f;
    /* PPM: span 2 by default (cell edge >= 2 r_max: at most 2x2x2 cells;
     * env PM_CELL_SPAN 3..5 for finer cells, DESIGN.md §5 sweep). kNN:
     * r_max / 2 — the query visits rows nearest first and prunes cells
     * beyond the shrinking k-th distance (k_gather_knn) */
    const float f = p->estimator == PM_ESTIMATOR_KNN ? 0.5f : 2.0f / (float)(c->cell_span - 1);
    float cs = f * rq * 1.001f;
    float ext[3];
    for (int a = 0; a < 3; ++a) ext[a] = std::max(c->bbox_hi[a] - c->bbox_lo[a], 1e-3f);
    int64_t dims[3];
    while (true) {
        for (int a = 0; a < 3; ++a) dims[a] = std::max<int64_t>(1, (int64_t)std::ceil(ext[a] / cs) + 1);
        if (dims[0] * dims[1] * dims[2] <= (int64_t)1 << 25) break;
        cs *= 1.25f;
    }
    g.gx = c->bbox_lo[0]; g.gy = c->bbox_lo[1]; g.gz = c->bbox_lo[2];
    g.inv_cs = 1.0f / cs;
    g.dx = (int)dims[0]; g.dy = (int)dims[1]; g.dz = (int)dims[2];
    g.ncells = (uint32_t)(dims[0] * dims[1] * dims[2]);
    return g;
}

static bool same_grid(const GridDesc &a, const GridDesc &b) { return std::memcmp(&a, &b, sizeof(GridDesc)) == 0; }

/* make the first `words` bucket counters zero (a memset only when the last
 * bucket scan did not already leave them cleared) */
static hipError_t count_zeroed(Ctx *c, size_t words, hipStream_t s) {
    if (c->count_zero_ptr == c->d_count.p && c->count_zero_words >= words) return hipSuccess;
    hipError_t e = hipMemsetAsync(c->d_count.p, 0, words * 4, s);
    if (e == hipSuccess) { c->count_zero_words = words; c->count_zero_ptr = c->d_count.p; }
    return e;
}

int pm_trace_photons(void *ptr, const pm_render_params *p, int pass, int64_t path_begin, int64_t path_count,
                     int64_t slot_path_base, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (path_count < 0 || path_begin < slot_path_base) FAIL(c, PM_ERR_INVALID, "bad path range");
    if ((uint64_t)(path_begin + path_count) * (uint64_t)p->max_photon_count > 0xffffffffull)
        FAIL(c, PM_ERR_INVALID, "photon slot index exceeds 32 bits (reference pm_index is a uint)");
    const int64_t mpc = p->max_photon_count;
    const int64_t end_slot = (path_begin + path_count - slot_path_base) * mpc;
    hipStream_t s = pick(c, stream);
    const bool fuse = c->fuse_ok && p->gather_structure == PM_GATHER_GRID && path_begin == slot_path_base;
    /* stale slots of an earlier lazy trace: zeroed now unless this fused
     * trace rewrites (or re-marks) every one of them */
    if (c->slots_dirty > 0 && !(fuse && end_slot >= c->slots_dirty) && (rc = materialize_slots(c, s))) return rc;
    c->slots_dirty = 0;
    if ((rc = pm_reserve_slots(c, end_slot, nullptr))) return rc;
    TraceParams T{};
    T.S = c->S;
    T.slots = c->d_slots.as<pm_photon>();
    halton_perm((uint32_t)pass, T.perm);
    {
        const uint32_t base[3] = {3u, 5u, 7u}, off[3] = {2u, 5u, 10u};
        for (int k = 0; k < 3; ++k) {
            T.perm_bits[k] = 0u;
            for (uint32_t d = 0; d < base[k]; ++d) T.perm_bits[k] |= T.perm[off[k] + d] << (3u * d);
        }
    }
    T.path_begin = path_begin; T.path_count = path_count; T.slot_path_base = slot_path_base;
    T.hold = c->trace_hold ? 1 : 0;
    if (T.hold && !c->S.wide) { /* per-lane kernel: only when the held deposits' LDS costs no resident waves */
        const size_t lds = (size_t)c->S.stack_depth * TRACE_BLOCK * 4 + c->S.lds_bytes;
        if (trace_lane_waves_per_cu(c->S, lds, 1) < trace_lane_waves_per_cu(c->S, lds, 0)) T.hold = 0;
    }
    if (c->S.wide) {
        /* pooled kernel: one occupancy round (resident waves per CU from the
         * occupancy API: VGPRs and the LDS stacks) — each wave with a
         * contiguous pool of a multiple of 64 paths. C3 sweep (1M paths, 256 CUs): 4096 waves 5.25 ms, 8192
         * (two rounds) 5.81, 5462 (1.33 rounds) 6.73, 2048 7.22 */
        /* LDS stack entries per lane (env PM_POOL_STACK; 0 = the tree's exact
         * bound): below the bound, deeper entries spill to global memory and
         * the smaller LDS reservation admits more resident blocks */
        const int lstk = c->pool_stack > 0 && c->pool_stack < c->S.stack_depth ? c->pool_stack : c->S.stack_depth;
        T.pool_stack = lstk;
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0) cus = 256;
        const size_t lds = (size_t)lstk * TRACE_BLOCK * 4 + c->S.lds_bytes;
        const int w8 = c->S.wide == 3;
        int per_cu = trace_pool_waves_per_cu(lds, 0, w8);
        if (T.hold) { /* pooled kernel: the held deposits' LDS must not cost resident waves */
            const int per_cu_h = trace_pool_waves_per_cu(lds, 1, w8);
            if (per_cu_h < per_cu) T.hold = 0;
            else per_cu = per_cu_h;
        }
        const int64_t waves = (int64_t)cus * (per_cu > 0 ? per_cu : 16);
        /* any pool size works (the wave's cursor hands out paths to dead lanes) */
        const int64_t per = std::max<int64_t>(1, (path_count + waves - 1) / waves);
        T.pool_paths = c->trace_pool || c->S.wide == 3 ? per : 0; /* 8-wide: its deeper stacks need the pooled kernel's spill */
        if (lstk < c->S.stack_depth) {
            const int64_t blocks = ((path_count + per - 1) / per + TRACE_BLOCK / 64 - 1) / (TRACE_BLOCK / 64);
            const int64_t threads = blocks * TRACE_BLOCK;
            HIPCHK(c, c->d_spill.ensure((size_t)threads * (size_t)(c->S.stack_depth - lstk) * 4));
            T.spill = c->d_spill.as<int>();
            T.spill_stride = (uint32_t)threads;
        }
    }
    T.pass = pass; T.mpc = (int)mpc; T.max_spec = p->max_specular_depth; T.light_index = p->light_source_index;
    T.eps = p->scene_epsilon; T.seed = p->rng_seed;
    T.counters = c->d_counters.as<unsigned long long>() + 4;
    T.prof = c->d_counters.as<unsigned long long>() + 8;
    if (c->counting) HIPCHK(c, hipMemsetAsync(T.counters, 0, 32, s));
    /* A call that fills the slot buffer from slot 0 also runs the counting pass
     * of the bucket build (keys, ranks, per-cell counts) at deposit time; the
     * build then skips it (c->fused). Any other slot producer invalidates it. */
    c->fused.valid = false;
    if (fuse) {
        c->fused.r2 = grid_radius2(c, p, true, s);
        const GridDesc g = make_grid(c, p, c->fused.r2);
        HIPCHK(c, c->d_count.ensure_slack(((size_t)g.ncells + 1) * 4));
        HIPCHK(c, c->d_scratch.ensure_slack(bucket_scratch_words(end_slot, g.ncells) * 4));
        HIPCHK(c, count_zeroed(c, (size_t)g.ncells + 1, s));
        T.bucket = 1;
        T.grid = g;
        T.count = c->d_count.as<uint32_t>();
        T.key = c->d_scratch.as<uint32_t>();
        T.rank = c->d_scratch.as<uint32_t>() + end_slot;
        /* plane-major keys / ranks; the held deposits write a path's four
         * keys as one 16-B store in slot order */
        T.key_np = !T.hold ? path_count : 0;
        T.lazy_zero = c->lazy_zero && !T.hold && !c->d_slots.external && !c->slots_exposed ? 1 : 0;
    }
    timer_begin(c, "trace", s);
    /* the kernel writes all path_count * mpc slots: deposits, then zeros */
    HIPCHK(c, launch_trace(T, c->counting, s));
    timer_end(c, "trace", s);
    if (fuse) { c->fused.valid = true; c->fused.n = end_slot; c->fused.grid = T.grid; c->fused.key_np = T.key_np; c->fused.mpc = (int)mpc; c->count_zero_words = 0; }
    if (T.lazy_zero) {
        if (!c->dirty_event) HIPCHK(c, hipEventCreateWithFlags(&c->dirty_event, hipEventDisableTiming));
        HIPCHK(c, hipEventRecord(c->dirty_event, s));
        c->slots_dirty = end_slot;
        c->dirty_key_np = T.key_np;
        c->dirty_mpc = (int)mpc;
    }
    /* traced photons carry the scene's signs (scene_nonneg); slots outside
     * the traced range keep theirs, so the flag is reset only when this
     * trace rewrote every slot in use */
    if (path_begin == slot_path_base && end_slot >= c->slots_used) c->slots_nonneg = true;
    c->slots_used = std::max(c->slots_used, end_slot);
    return PM_OK;
}

int pm_build_photon_map(void *ptr, const pm_render_params *p, int64_t n_slots, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (n_slots <= 0) n_slots = c->slots_used;
    if ((size_t)n_slots * sizeof(pm_photon) > c->d_slots.bytes) FAIL(c, PM_ERR_INVALID, "n_slots beyond slot buffer");
    hipStream_t s = pick(c, stream);
    c->map_slots = n_slots;
    if (p->gather_structure == PM_GATHER_KDTREE && (rc = materialize_slots(c, s))) return rc;
    if (p->gather_structure == PM_GATHER_KDTREE) {
        /* reference path (CreatePhotonMap): DtoH, CPU pbrt KdTree, HtoD */
        timer_begin(c, "build", s, true);
        std::vector<pm_photon> h((size_t)n_slots), nodes;
        HIPCHK(c, hipMemcpyAsync(h.data(), c->d_slots.p, n_slots * sizeof(pm_photon), hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        int64_t m = build_kdtree_pbrt(h.data(), n_slots, nodes);
        c->kd_count = m;
        if (m > 0) {
            HIPCHK(c, c->d_kd.ensure(m * sizeof(pm_photon)));
            HIPCHK(c, hipMemcpyAsync(c->d_kd.p, nodes.data(), m * sizeof(pm_photon), hipMemcpyHostToDevice, s));
            HIPCHK(c, hipStreamSynchronize(s));
        }
        timer_end(c, "build", s);
        c->map_kind = PM_GATHER_KDTREE;
        if (m == 0) FAIL(c, PM_ERR_NO_PHOTONS, "0 valid photons");
        return PM_OK;
    }
    /* photon buckets: cell size >= 2 r_max (PPM radii only shrink) */
    GridDesc &g = c->grid;
    /* the grid of the trace's fused counts, if they cover these slots */
    const bool fused_ok = c->fused.valid && c->fused.n == n_slots;
    c->grid_r2 = fused_ok ? c->fused.r2 : grid_radius2(c, p, true, s);
    g = make_grid(c, p, c->grid_r2);
    const bool counted = fused_ok && same_grid(c->fused.grid, g);
    /* the counting pass below reads every slot's valid bit (and overwrites the keys) */
    if (!counted && (rc = materialize_slots(c, s))) return rc;
    const size_t n = (size_t)n_slots;
    HIPCHK(c, c->d_count.ensure_slack(((size_t)g.ncells + 1) * 4));
    HIPCHK(c, c->d_cell_start.ensure_slack(((size_t)g.ncells + 1) * 4));
    if (!counted) {
        HIPCHK(c, c->d_scratch.ensure_slack(bucket_scratch_words(n_slots, g.ncells) * 4));
        HIPCHK(c, count_zeroed(c, (size_t)g.ncells + 1, s));
    }
    HIPCHK(c, c->d_pha.ensure_slack(n * 16)); HIPCHK(c, c->d_phb.ensure_slack(n * 32));
    timer_begin(c, "build", s);
    HIPCHK(c, launch_bucket_build(c->d_slots.as<pm_photon>(), n_slots, g, c->d_count.as<uint32_t>(),
                                  c->d_cell_start.as<uint32_t>(), c->d_scratch.as<uint32_t>(), c->d_pha.as<float4>(),
                                  c->d_phb.as<float4>(), counted, s, counted ? c->fused.key_np : 0, c->fused.mpc));
    ++c->map_gen; /* kNN pairs repacked on the next kNN gather */
    /* the scan left the counters zeroed */
    c->count_zero_words = (size_t)g.ncells + 1;
    c->count_zero_ptr = c->d_count.p;
    timer_end(c, "build", s);
    c->map_kind = PM_GATHER_GRID;
    return PM_OK;
}


/* the tile list of the current records, built on the device without a host
 * wait: flags + an in-order compaction, its length copied to pinned memory
 * behind an event. Until that copy has landed (hipEventQuery, never waited
 * on) the gather kernels read the length from device memory and the grid
 * covers every tile. */
static int ensure_tiles(Ctx *c, hipStream_t s) {
    if (!c->tiles_valid) {
        const int64_t nt = (c->nrec + 63) / 64;
        HIPCHK(c, c->d_tile_flags.ensure(std::max<int64_t>(nt, 16)));
        HIPCHK(c, c->d_tiles.ensure(std::max<int64_t>(nt * 4, 16)));
        HIPCHK(c, c->d_tile_count.ensure(16));
        if (!c->h_tile_count) HIPCHK(c, hipHostMalloc((void **)&c->h_tile_count, 4, hipHostMallocDefault));
        if (!c->tile_event) HIPCHK(c, hipEventCreateWithFlags(&c->tile_event, hipEventDisableTiming));
        /* a previous list's length still in flight (records replaced before
         * any gather read it): let that copy land before the pinned word is reused */
        else if (!c->tile_count_known) HIPCHK(c, hipEventSynchronize(c->tile_event));
        HIPCHK(c, launch_tile_list(recs(c), c->d_tile_flags.as<uint8_t>(), c->d_tiles.as<uint32_t>(),
                                   c->d_tile_count.as<uint32_t>(), s));
        HIPCHK(c, hipMemcpyAsync(c->h_tile_count, c->d_tile_count.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipEventRecord(c->tile_event, s));
        c->tiles_valid = true;
        c->tiles_sorted = false;
        c->tile_count_known = false;
    }
    if (!c->tile_count_known && hipEventQuery(c->tile_event) == hipSuccess) {
        c->n_tiles = (int64_t)*c->h_tile_count;
        c->tile_count_known = true;
    }
    return PM_OK;
}

static int gather_common(Ctx *c, const pm_render_params *p, long long *partial, int64_t rec_begin, int64_t rec_count,
                         void *stream, int *count = nullptr, long long *flux = nullptr) {
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (c->nrec <= 0) FAIL(c, PM_ERR_INVALID, "no records (run pm_eye_pass first)");
    if (c->map_kind != p->gather_structure) FAIL(c, PM_ERR_INVALID, "photon map not built for this gather structure");
    if (p->estimator == PM_ESTIMATOR_KNN && (partial || count))
        FAIL(c, PM_ERR_INVALID, "the kNN estimator is not linear in the photon set: no partial / split gathers "
                                "(multi-GPU: all-gather the photons, then pm_gather_range)");
    if (rec_begin < 0 || rec_count < 0 || rec_begin + rec_count > c->nrec) FAIL(c, PM_ERR_INVALID, "bad record range");
    hipStream_t s = pick(c, stream);
    GatherParams G = gather_params(c, p);
    G.partial = partial;
    G.count = count;
    G.flux = flux;
    G.rec_begin = rec_begin;
    G.rec_end = rec_begin + rec_count;
    /* a pending reset is consumed by a fused gather over all records (it starts
     * from the initial PPM state and writes it); a split partial gather reads
     * the initial radius and leaves the reset to pm_ppm_update_split, which
     * writes every view record; any other gather needs it applied */
    const bool split = count != nullptr;
    const bool consume = c->rec_fresh && !partial && !split && rec_begin == 0 && rec_count == c->nrec;
    if (consume || (split && c->rec_fresh)) { G.fresh = 1; G.r2init = c->rec_fresh_r2; }
    else if ((rc = materialize_reset(c, s))) return rc;
    /* full-range tile gathers skip the tiles without an active record (their
     * records are neither read nor written, except as partials outside a view) */
    if (c->gather_kernel == PM_GK_TILE && !c->counting && rec_begin == 0 && rec_count == c->nrec &&
        p->gather_structure == PM_GATHER_GRID && ((!partial && !split) || c->view_active)) {
        if ((rc = ensure_tiles(c, s))) return rc;
        G.tiles = c->d_tiles.as<uint32_t>();
        if (c->tile_count_known) { G.n_tiles = c->n_tiles; G.n_tiles_dev = nullptr; }
        else { G.n_tiles = (c->nrec + 63) / 64; G.n_tiles_dev = c->d_tile_count.as<uint32_t>(); }
        /* the PPM tile gather and the kNN scalar-stream kernel record the costs */
        if (c->tile_sort && !c->tiles_sorted && (p->estimator == PM_ESTIMATOR_PPM || c->knn_ss)) {
            HIPCHK(c, c->d_tile_cost.ensure((size_t)((c->nrec + 63) / 64 + 8) * 2));
            HIPCHK(c, c->d_tiles2.ensure(c->d_tiles.bytes));
            G.tile_cost = c->d_tile_cost.as<uint16_t>();
        }
        /* fresh PPM gather: every radius is r2init, the first group's box comes from the tile's position box */
    }
    if (c->counting) HIPCHK(c, hipMemsetAsync(c->d_counters.p, 0, 32, s));
    /* a fused PPM tile gather bins the updated radii (grid_radius2) — over
     * all records, or over each of a pass's bands (a device's bands in a
     * group render or an all-gather rank): every gather of the pass adds to
     * the same bins, summed once when the next pass chooses its grid, so the
     * quantile describes every record the context gathers (the grid only
     * sets the cost, never the sums) */
    const bool hist = p->estimator == PM_ESTIMATOR_PPM && p->gather_structure == PM_GATHER_GRID && !partial &&
                      !split && c->gather_kernel == PM_GK_TILE &&
                      !c->counting && c->grid_quantile > 0.0 && c->r2_wanted;
    if (hist) {
        /* the reduce that read and re-zeroed the bins may have run on another
         * stream (a trace issued ahead on a second stream chose its grid:
         * dist.py's pipelined passes): this gather bins (and may clear) only
         * after it — otherwise the two race on d_r2hist */
        if (c->r2_pending && c->r2_stream != s) HIPCHK(c, hipStreamWaitEvent(s, c->r2_event, 0));
        if (c->r2_accum && c->r2_accum_init != p->initial_radius2) { c->r2_accum = false; c->r2_dirty = true; }
        if (!c->d_r2hist.p) {
            HIPCHK(c, c->d_r2hist.ensure(R2_COPIES * R2_BINS * 4));
            c->r2_dirty = true;
        }
        if (c->r2_dirty) { /* the reduce re-zeroes it; anything else left in it is dropped here */
            HIPCHK(c, hipMemsetAsync(c->d_r2hist.p, 0, R2_COPIES * R2_BINS * 4, s));
            c->r2_dirty = false;
        }
        if (!c->h_r2hist) {
            HIPCHK(c, hipHostMalloc((void **)&c->h_r2hist, R2_BINS * 4, hipHostMallocMapped));
            HIPCHK(c, hipHostGetDevicePointer((void **)&c->h_r2hist_dev, c->h_r2hist, 0));
        }
        if (!c->r2_event) HIPCHK(c, hipEventCreateWithFlags(&c->r2_event, hipEventDisableTiming));
        G.r2hist = c->d_r2hist.as<uint32_t>();
        G.r2hist_inv = 1.0f / p->initial_radius2;
    }
    timer_begin(c, "gather", s);
    if (p->estimator == PM_ESTIMATOR_KNN) {
        G.knn_k = p->knn_lookup;
        G.knn_r2 = p->initial_radius2; /* pbrt's maxDistSquared: the buckets cover it */
        /* every term (kernel <= 3/pi < 1) is <= alpha_max / r_k^2: <= 2^22 of
         * the per-record scale per term (x4 headroom in amax), exact as a float
         * and as an int32, and <= PM_KNN_MAX = 2^6 terms sum below 2^28 —
         * exact in int32 */
        const double amax = c->emit_max * std::pow(c->kd_max, (double)p->max_photon_count) * 4.0;
        G.knn_fx = (float)(std::ldexp(1.0, 24) / std::max(amax, 1e-30));
        G.slots = c->d_slots.as<pm_photon>();
        if (c->knn_ss && !c->counting && c->gather_kernel == PM_GK_TILE) {
            const int64_t nph = (int64_t)(c->d_pha.bytes / 16), pairs = (nph + 1) / 2 + 16;
            const int64_t ntiles = (G.rec_end - G.rec_begin + 63) / 64;
            HIPCHK(c, c->d_knnpk.ensure((size_t)pairs * 80));
            HIPCHK(c, c->d_knnovf.ensure((size_t)(ntiles + KNN_OVF_HDR) * 4));
            G.knn_pk_p = c->d_knnpk.as<float4>();
            G.knn_pk_q = G.knn_pk_p + 2 * pairs;
            G.knn_pk_pairs = pairs;
            G.knn_pack = c->knn_pack_gen != c->map_gen || c->knn_pack_ptr != c->d_knnpk.p;
            c->knn_pack_gen = c->map_gen;
            c->knn_pack_ptr = c->d_knnpk.p;
            G.knn_ovf_n = c->d_knnovf.as<uint32_t>();
            G.knn_ovf = G.knn_ovf_n + KNN_OVF_HDR;
        }
#ifdef PM_TILE_TIMES
        const char *tt_path = getenv("PM_TILE_TIMES");
        const int64_t tt_n = (c->nrec + 63) / 64;
        if (tt_path && G.tiles) {
            HIPCHK(c, c->d_tile_times.ensure((size_t)tt_n * 64));
            HIPCHK(c, hipMemsetAsync(c->d_tile_times.p, 0, (size_t)tt_n * 64, s));
            G.tile_times = c->d_tile_times.as<unsigned long long>();
        }
#endif
        HIPCHK(c, launch_gather_knn(G, c->counting, s));
#ifdef PM_TILE_TIMES
        if (G.tile_times) {
            std::vector<unsigned long long> h((size_t)tt_n * 8);
            HIPCHK(c, hipMemcpyAsync(h.data(), G.tile_times, h.size() * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            if (FILE *f = fopen(tt_path, "ab")) {
                const unsigned long long hdr[4] = {0xffffffffffffffffull, (unsigned long long)tt_n, 0, 0};
                fwrite(hdr, 8, 4, f);
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
#endif
        if (G.knn_ovf_n && getenv("PM_KNN_SS_DEBUG")) { /* tiles handed back to k_gather_knn_tile */
            uint32_t nb = 0;
            HIPCHK(c, hipMemcpyAsync(&nb, G.knn_ovf_n, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            fprintf(stderr, "pm knn_ss: %u of %lld tiles handed back\n", nb, (long long)(G.tiles ? G.n_tiles : (G.rec_end - G.rec_begin + 63) / 64));
            std::vector<uint32_t> hdr(KNN_OVF_HDR);
            HIPCHK(c, hipMemcpy(hdr.data(), G.knn_ovf_n, KNN_OVF_HDR * 4, hipMemcpyDeviceToHost));
            if (hdr[1] || hdr[2]) { /* PM_KNN_SS_DBG builds */
                fprintf(stderr, "pm knn_ss dbg: %u bad collects, %u NaN radii\n", hdr[1], hdr[2]);
                for (uint32_t i = 0; i < std::min<uint32_t>(hdr[1], 60); ++i) {
                    fprintf(stderr, "  ");
                    for (int w = 0; w < 16; ++w) fprintf(stderr, " %u", hdr[64 + 16 * i + w]);
                    fprintf(stderr, "\n");
                }
            }
        }
    } else {
        if (p->gather_structure == PM_GATHER_KDTREE) HIPCHK(c, hipMemsetAsync(G.error, 0, 4, s));
#ifdef PM_TILE_TIMES
        /* diagnostic builds: env PM_TILE_TIMES=file appends each tile launch's
         * per-wave (start, end, XCC_ID, HW_ID) records (tools/tile_times.py) */
        const char *tt_path = getenv("PM_TILE_TIMES");
        const int64_t tt_n = (c->nrec + 63) / 64;
        if (tt_path && G.tiles) {
            HIPCHK(c, c->d_tile_times.ensure((size_t)tt_n * 64));
            HIPCHK(c, hipMemsetAsync(c->d_tile_times.p, 0, (size_t)tt_n * 64, s));
            G.tile_times = c->d_tile_times.as<unsigned long long>();
        }
#endif
        HIPCHK(c, launch_gather(G, p->gather_structure, partial != nullptr || split, c->counting, s));
#ifdef PM_TILE_TIMES
        if (G.tile_times) {
            std::vector<unsigned long long> h((size_t)tt_n * 8);
            HIPCHK(c, hipMemcpyAsync(h.data(), G.tile_times, h.size() * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            if (FILE *f = fopen(tt_path, "ab")) {
                const unsigned long long hdr[4] = {0xffffffffffffffffull, (unsigned long long)tt_n, 0, 0};
                fwrite(hdr, 8, 4, f);
                fwrite(h.data(), 8, h.size(), f);
                fclose(f);
            }
        }
#endif
    }
    if (G.tile_cost) { /* the measured wave lifetimes reorder the list for the next gathers */
        HIPCHK(c, launch_tile_sort(G.tiles, G.tile_cost, G.n_tiles_dev, G.n_tiles, c->d_tiles2.as<uint32_t>(), s));
        std::swap(c->d_tiles, c->d_tiles2);
        c->tiles_sorted = true;
    }
    timer_end(c, "gather", s);
    if (p->estimator != PM_ESTIMATOR_KNN && p->gather_structure == PM_GATHER_KDTREE) {
        /* the reference's path (host kd-tree, synchronous like CreatePhotonMap):
         * a truncated traversal is an error, not a silently darker pixel */
        unsigned int err = 0;
        HIPCHK(c, hipMemcpyAsync(&err, G.error, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(c, hipStreamSynchronize(s));
        if (err & PM_GATHER_ERR_STACK) FAIL(c, PM_ERR_INVALID, "kd-tree gather: traversal stack of %d entries overflowed", G.kd_stack);
        if (err & PM_GATHER_ERR_TREE) FAIL(c, PM_ERR_INVALID, "kd-tree gather: node links do not form a pbrt kd-tree");
    }
    c->rec_estimator = p->estimator;
    if (consume) c->rec_fresh = false;
    if (hist) {
        /* summed by grid_radius2 at the next pass, into host-mapped memory by
         * a one-block kernel: no copy-engine transfer in the stream (a
         * per-pass D2H copy cost ~0.5 ms of C2 step) */
        c->r2_accum = true;
        c->r2_accum_init = p->initial_radius2;
    } else if (p->estimator == PM_ESTIMATOR_KNN) {
        r2_invalidate(c); /* r_k^2 replaced the radii */
    }
    return PM_OK;
}

int pm_gather(void *ptr, const pm_render_params *p, void *stream) {
    GETCTX(ptr);
    return gather_common(c, p, nullptr, 0, c->nrec, stream);
}

int pm_gather_range(void *ptr, const pm_render_params *p, int64_t rec_begin, int64_t rec_count, void *stream) {
    GETCTX(ptr);
    return gather_common(c, p, nullptr, rec_begin, rec_count, stream);
}

int pm_gather_partial(void *ptr, const pm_render_params *p, void *d_partial, void *stream) {
    GETCTX(ptr);
    if (!d_partial) FAIL(c, PM_ERR_INVALID, "null partial buffer");
    return gather_common(c, p, (long long *)d_partial, 0, c->nrec, stream);
}

int pm_gather_split(void *ptr, const pm_render_params *p, void *d_count, void *d_flux, void *stream) {
    GETCTX(ptr);
    if (!d_count || !d_flux) FAIL(c, PM_ERR_INVALID, "null count / flux buffer");
    return gather_common(c, p, nullptr, 0, c->nrec, stream, (int *)d_count, (long long *)d_flux);
}

int pm_ppm_update_split(void *ptr, const pm_render_params *p, const void *d_count, const void *d_flux_chunk,
                        int64_t v_begin, int64_t v_count, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    const int64_t n = view_size(c);
    if (!d_count || (v_count > 0 && !d_flux_chunk) || v_begin < 0 || v_count < 0 || v_begin + v_count > n)
        FAIL(c, PM_ERR_INVALID, "bad view chunk");
    hipStream_t s = pick(c, stream);
    GatherParams G = gather_params(c, p);
    const int fresh = c->rec_fresh ? 1 : 0;
    G.r2init = c->rec_fresh_r2;
    timer_begin(c, "update", s);
    HIPCHK(c, launch_ppm_update_split(G, (const int *)d_count, (const long long *)d_flux_chunk, n, v_begin, v_count,
                                      fresh, s));
    timer_end(c, "update", s);
    c->rec_fresh = false; /* every view record written (records outside the view are inactive) */
    return PM_OK;
}

int pm_ppm_update_split_radius(void *ptr, const pm_render_params *p, const void *d_count, void *d_ratio, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    const int64_t n = view_size(c);
    if (!d_count || !d_ratio) FAIL(c, PM_ERR_INVALID, "null count / ratio buffer");
    hipStream_t s = pick(c, stream);
    GatherParams G = gather_params(c, p);
    const int fresh = c->rec_fresh ? 1 : 0;
    G.r2init = c->rec_fresh_r2;
    timer_begin(c, "update", s);
    HIPCHK(c, launch_ppm_update_radius(G, (const int *)d_count, (float *)d_ratio, n, fresh, s));
    timer_end(c, "update", s);
    c->rec_fresh = false; /* every view record written (records outside the view are inactive) */
    return PM_OK;
}

int pm_ppm_update_split_flux(void *ptr, const pm_render_params *p, const void *d_ratio, const void *d_flux_chunk,
                             int64_t v_begin, int64_t v_count, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    const int64_t n = view_size(c);
    if (!d_ratio || (v_count > 0 && !d_flux_chunk) || v_begin < 0 || v_count < 0 || v_begin + v_count > n)
        FAIL(c, PM_ERR_INVALID, "bad view chunk");
    hipStream_t s = pick(c, stream);
    GatherParams G = gather_params(c, p);
    HIPCHK(c, launch_ppm_update_flux(G, (const float *)d_ratio, (const long long *)d_flux_chunk, v_begin, v_count, s));
    return PM_OK;
}

int pm_ppm_update(void *ptr, const pm_render_params *p, const void *d_partial, int64_t rec_begin, int64_t rec_count,
                  void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (!d_partial || rec_begin < 0 || rec_count < 0 || rec_begin + rec_count > view_size(c))
        FAIL(c, PM_ERR_INVALID, "bad record range");
    hipStream_t s = pick(c, stream);
    if ((rc = materialize_reset(c, s))) return rc;
    GatherParams G = gather_params(c, p);
    timer_begin(c, "update", s);
    HIPCHK(c, launch_ppm_update(G, (const long long *)d_partial, rec_begin, rec_count, s));
    timer_end(c, "update", s);
    return PM_OK;
}

int pm_get_radius2(void *ptr, int64_t rec_begin, int64_t rec_count, void *d_out, void *stream) {
    GETCTX(ptr);
    if (!d_out || rec_begin < 0 || rec_count < 0 || rec_begin + rec_count > view_size(c))
        FAIL(c, PM_ERR_INVALID, "bad radius2 range");
    int rc;
    if ((rc = materialize_reset(c, pick(c, stream)))) return rc;
    HIPCHK(c, launch_radius2_io(recs(c), (float *)d_out, rec_begin, rec_count, 0, view_list(c), pick(c, stream)));
    return PM_OK;
}

int pm_set_radius2(void *ptr, const void *d_in, int64_t rec_begin, int64_t rec_count, void *stream) {
    GETCTX(ptr);
    if (!d_in || rec_begin < 0 || rec_count < 0 || rec_begin + rec_count > view_size(c))
        FAIL(c, PM_ERR_INVALID, "bad radius2 range");
    int rc;
    if ((rc = materialize_reset(c, pick(c, stream)))) return rc;
    HIPCHK(c, launch_radius2_io(recs(c), (float *)d_in, rec_begin, rec_count, 1, view_list(c), pick(c, stream)));
    r2_invalidate(c); /* radii may have grown */
    return PM_OK;
}

int pm_final(void *ptr, double emitted, int64_t rec_begin, int64_t rec_count, void *d_out, void *stream) {
    GETCTX(ptr);
    if (!d_out || rec_begin < 0 || rec_count < 0 || rec_begin + rec_count > c->nrec)
        FAIL(c, PM_ERR_INVALID, "bad final range");
    hipStream_t s = pick(c, stream);
    int rc;
    if ((rc = materialize_reset(c, s))) return rc;
    FinalParams F{};
    F.R = recs(c);
    F.knn = c->rec_estimator == PM_ESTIMATOR_KNN; F.materials = c->S.materials;
    F.emitted = (float)emitted; /* gContext["emittingPhotons"]->setFloat((float)totalPhotons) */
    F.rec_begin = rec_begin; F.rec_count = rec_count; F.out = (float *)d_out; F.raster = 0; F.W = c->W;
    timer_begin(c, "final", s);
    HIPCHK(c, launch_final(F, s));
    timer_end(c, "final", s);
    return PM_OK;
}

/* ------------------------------------------------------------ whole render */
/* the all-gather mode's record ranges of each device: 8-row bands (`unit`
 * records each) in runs dealt round-robin, about four runs per device
 * (pmrender/dist.py _bands) */
static std::vector<std::vector<std::pair<int64_t, int64_t>>> device_bands(int64_t n, int64_t unit, int world) {
    std::vector<std::vector<std::pair<int64_t, int64_t>>> owned(world);
    const int64_t units = (n + unit - 1) / unit;
    const int64_t runs = std::max<int64_t>(1, (units + (int64_t)world * 4 - 1) / ((int64_t)world * 4));
    int k = 0;
    for (int64_t u = 0; u < units; u += runs, ++k) {
        const int64_t b = u * unit, e = std::min(n, (u + runs) * unit);
        owned[k % world].push_back({b, e - b});
    }
    return owned;
}

/* one progressive render over the group's devices (Group): per pass every
 * device traces its shard of the global paths into its own slot buffer at
 * the shard's global slot offset, the shards are all-gathered (equal
 * chunks, the last padded with invalid slots), every device builds the full
 * map and gathers its bands; the final pass writes each device's bands into
 * the host image. Bit-identical to one device rendering all the paths (the
 * same valid photons in the map; exact, order-free gather sums). */
static int group_render(Ctx *gc, const pm_render_params *p, float *out_rgb, pm_stats *st) {
    Group &G = *gc->group;
    const int n = (int)G.subs.size();
    if (!p || !out_rgb) FAIL(gc, PM_ERR_INVALID, "null params / output");
    if (p->passes < 1 || p->paths_per_pass < 1) FAIL(gc, PM_ERR_INVALID, "passes and paths_per_pass must be >= 1");
    const int64_t P = p->paths_per_pass, mpc = p->max_photon_count;
    const int64_t chunk = (P + n - 1) / n;                 /* paths per device (the last one may trace fewer) */
    const int64_t total_slots = chunk * n * mpc;
    const size_t chunk_bytes = (size_t)(chunk * mpc) * sizeof(pm_photon);
    int rc;
    auto sub_fail = [&](Ctx *sub, int code) { return group_fail(gc, sub, code); };
    std::vector<pm_photon *> slots(n);
    for (int d = 0; d < n; ++d) {
        Ctx *c = G.subs[d];
        (void)hipSetDevice(c->device);
        if ((rc = pm_eye_pass(c, p, nullptr))) return sub_fail(c, rc);
        if ((rc = pm_reserve_slots(c, total_slots, (void **)&slots[d]))) return sub_fail(c, rc);
    }
    Ctx *c0 = G.subs[0];
    const int64_t nrec = c0->nrec;
    const int64_t unit = c0->pinhole ? (int64_t)((c0->W + 7) / 8) * 64 : 512;
    const auto bands = device_bands(nrec, unit, n);
    int64_t nvalid = 0;
    double t_trace = 0, t_build = 0, t_gather = 0;
    for (int pass = 0; pass < p->passes; ++pass) {
        for (int d = 0; d < n; ++d) {
            Ctx *c = G.subs[d];
            (void)hipSetDevice(c->device);
            const int64_t b = d * chunk, cnt = std::max<int64_t>(0, std::min(chunk, P - b));
            if (cnt > 0 && (rc = pm_trace_photons(c, p, pass, b, cnt, 0, nullptr))) return sub_fail(c, rc);
            if (cnt < chunk) /* padding slots of a short shard: invalid */
                HIPCHK(gc, hipMemsetAsync(slots[d] + (b + cnt) * mpc, 0, (size_t)((chunk - cnt) * mpc) * sizeof(pm_photon),
                                          c->stream));
        }
        /* all-gather of the shards: every buffer gets every device's chunk */
        if (!G.comms.empty()) {
            if (ncclGroupStart() != ncclSuccess) FAIL(gc, PM_ERR_HIP, "ncclGroupStart");
            for (int d = 0; d < n; ++d) {
                Ctx *c = G.subs[d];
                (void)hipSetDevice(c->device);
                const ncclResult_t r = ncclAllGather((const char *)slots[d] + d * chunk_bytes, slots[d], chunk_bytes,
                                                     ncclUint8, G.comms[d], c->stream);
                if (r != ncclSuccess) { (void)ncclGroupEnd(); FAIL(gc, PM_ERR_HIP, "ncclAllGather: %s", ncclGetErrorString(r)); }
            }
            if (ncclGroupEnd() != ncclSuccess) FAIL(gc, PM_ERR_HIP, "ncclGroupEnd");
        } else if (n > 1) {
            for (int d = 0; d < n; ++d) {
                (void)hipSetDevice(G.subs[d]->device);
                HIPCHK(gc, hipEventRecord(G.ev[d], G.subs[d]->stream));
            }
            for (int d = 0; d < n; ++d) {
                Ctx *c = G.subs[d];
                (void)hipSetDevice(c->device);
                for (int q = 0; q < n; ++q) {
                    if (q == d) continue;
                    HIPCHK(gc, hipStreamWaitEvent(c->stream, G.ev[q], 0));
                    HIPCHK(gc, hipMemcpyPeerAsync((char *)slots[d] + q * chunk_bytes, c->device,
                                                  (const char *)slots[q] + q * chunk_bytes, G.subs[q]->device,
                                                  chunk_bytes, c->stream));
                }
            }
        }
        for (int d = 0; d < n; ++d) {
            Ctx *c = G.subs[d];
            (void)hipSetDevice(c->device);
            if ((rc = pm_build_photon_map(c, p, total_slots, nullptr))) {
                if (rc == PM_ERR_NO_PHOTONS) FAIL(gc, PM_ERR_NO_PHOTONS, "0 valid photons (photonmappingrenderer.cpp:165-167)");
                return sub_fail(c, rc);
            }
        }
        if (p->gather_structure == PM_GATHER_GRID) {
            uint32_t nv = 0;
            (void)hipSetDevice(c0->device);
            HIPCHK(gc, hipMemcpyAsync(&nv, c0->d_cell_start.as<uint32_t>() + c0->grid.ncells, 4, hipMemcpyDeviceToHost, c0->stream));
            HIPCHK(gc, hipStreamSynchronize(c0->stream));
            nvalid = nv;
        } else {
            nvalid = c0->kd_count;
        }
        if (nvalid == 0) FAIL(gc, PM_ERR_NO_PHOTONS, "0 valid photons (photonmappingrenderer.cpp:165-167)");
        for (int d = 0; d < n; ++d) {
            Ctx *c = G.subs[d];
            (void)hipSetDevice(c->device);
            for (const auto &bc : bands[d])
                if ((rc = pm_gather_range(c, p, bc.first, bc.second, nullptr))) return sub_fail(c, rc);
        }
        /* the next pass overwrites the slot buffers the peers read */
        for (int d = 0; d < n; ++d) { (void)hipSetDevice(G.subs[d]->device); HIPCHK(gc, hipStreamSynchronize(G.subs[d]->stream)); }
        /* stage times of the slowest device, read once the pass is done (a
         * read inside the loops would wait for one device before the next
         * one's launch) */
        double tt = 0, tb = 0, tg = 0;
        for (int d = 0; d < n; ++d) {
            Ctx *c = G.subs[d];
            if (std::min(chunk, P - d * chunk) > 0) tt = std::max(tt, timer_ms(c, "trace"));
            tb = std::max(tb, timer_ms(c, "build"));
            if (!bands[d].empty()) tg = std::max(tg, timer_ms(c, "gather", bands[d].size()));
        }
        t_trace += tt; t_build += tb; t_gather += tg;
    }
    /* final radiance of each device's bands, straight into the host image */
    const double emitted = (double)P * p->passes;
    const int64_t nout = c0->pinhole ? (int64_t)c0->W * c0->H : nrec;
    for (int d = 0; d < n; ++d) {
        Ctx *c = G.subs[d];
        (void)hipSetDevice(c->device);
        if ((rc = materialize_reset(c, c->stream))) return sub_fail(c, rc);
        HIPCHK(gc, c->d_out.ensure(nout * 3 * sizeof(float)));
        for (const auto &bc : bands[d]) {
            FinalParams F{};
            F.R = recs(c);
            F.knn = c->rec_estimator == PM_ESTIMATOR_KNN; F.materials = c->S.materials;
            F.emitted = (float)emitted;
            F.rec_begin = bc.first; F.rec_count = bc.second; F.raster = c->pinhole; F.W = c->W;
            F.out = c->pinhole ? c->d_out.as<float>() : c->d_out.as<float>() + 3 * bc.first;
            HIPCHK(gc, launch_final(F, c->stream));
            int64_t o0 = bc.first, o1 = bc.first + bc.second; /* output elements of the band */
            if (c->pinhole) {
                const int64_t t0 = bc.first / unit, t1 = (bc.first + bc.second + unit - 1) / unit; /* tile rows */
                o0 = std::min<int64_t>(8 * t0, c->H) * c->W;
                o1 = std::min<int64_t>(8 * t1, c->H) * c->W;
            }
            if (o1 > o0)
                HIPCHK(gc, hipMemcpyAsync(out_rgb + 3 * o0, c->d_out.as<float>() + 3 * o0, (size_t)(o1 - o0) * 3 * sizeof(float),
                                          hipMemcpyDeviceToHost, c->stream));
        }
    }
    for (int d = 0; d < n; ++d) { (void)hipSetDevice(G.subs[d]->device); HIPCHK(gc, hipStreamSynchronize(G.subs[d]->stream)); }
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->paths_emitted = (int64_t)emitted;
        st->photons_valid = nvalid;
        std::vector<float4> pos(nrec);
        (void)hipSetDevice(c0->device);
        HIPCHK(gc, hipMemcpy(pos.data(), c0->d_pos.p, nrec * sizeof(float4), hipMemcpyDeviceToHost));
        int64_t act = 0;
        for (auto &q : pos) act += (fbits_h(q.w) & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) == 0;
        st->gather_points = act;
        st->ms_eye = timer_ms(c0, "eye"); st->ms_trace = t_trace; st->ms_build = t_build; st->ms_gather = t_gather;
    }
    return PM_OK;
}

int pm_render(void *ptr, const pm_render_params *p, float *out_rgb, pm_stats *st) {
    if (group_of(ptr)) return group_render((Ctx *)ptr, p, out_rgb, st);
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (!out_rgb) FAIL(c, PM_ERR_INVALID, "null output");
    if (p->passes < 1 || p->paths_per_pass < 1) FAIL(c, PM_ERR_INVALID, "passes and paths_per_pass must be >= 1");
    hipStream_t s = c->stream;
    double t_eye = 0, t_trace = 0, t_build = 0, t_gather = 0, t_final = 0;
    if ((rc = pm_eye_pass(c, p, s))) return rc;
    t_eye = timer_ms(c, "eye");
    int64_t nvalid = 0;
    int64_t counters[2] = {0, 0};
    for (int pass = 0; pass < p->passes; ++pass) {
        if ((rc = pm_trace_photons(c, p, pass, 0, p->paths_per_pass, 0, s))) return rc;
        t_trace += timer_ms(c, "trace");
        if ((rc = pm_build_photon_map(c, p, p->paths_per_pass * p->max_photon_count, s))) return rc;
        t_build += timer_ms(c, "build");
        if (p->gather_structure == PM_GATHER_GRID) {
            uint32_t nv = 0;
            HIPCHK(c, hipMemcpyAsync(&nv, c->d_cell_start.as<uint32_t>() + c->grid.ncells, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(c, hipStreamSynchronize(s));
            nvalid = nv;
        } else {
            nvalid = c->kd_count;
        }
        if (nvalid == 0) FAIL(c, PM_ERR_NO_PHOTONS, "0 valid photons (photonmappingrenderer.cpp:165-167)");
        if ((rc = pm_gather(c, p, s))) return rc;
        t_gather += timer_ms(c, "gather");
        if (c->counting) {
            unsigned long long hc[2];
            HIPCHK(c, hipMemcpy(hc, c->d_counters.p, 16, hipMemcpyDeviceToHost));
            counters[0] = (int64_t)hc[0]; counters[1] = (int64_t)hc[1];
        }
    }
    const double emitted = (double)p->paths_per_pass * p->passes;
    const int64_t nout = c->pinhole ? (int64_t)c->W * c->H : c->nrec;
    HIPCHK(c, c->d_out.ensure(nout * 3 * sizeof(float)));
    FinalParams F{};
    F.R = recs(c);
    F.knn = c->rec_estimator == PM_ESTIMATOR_KNN; F.materials = c->S.materials;
    F.emitted = (float)emitted;
    F.rec_begin = 0; F.rec_count = c->nrec; F.out = c->d_out.as<float>(); F.raster = c->pinhole; F.W = c->W;
    timer_begin(c, "final", s);
    HIPCHK(c, launch_final(F, s));
    timer_end(c, "final", s);
    HIPCHK(c, hipMemcpyAsync(out_rgb, c->d_out.p, nout * 3 * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    t_final = timer_ms(c, "final");
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->paths_emitted = (int64_t)emitted;
        st->photons_valid = nvalid;
        std::vector<float4> pos(c->nrec);
        HIPCHK(c, hipMemcpy(pos.data(), c->d_pos.p, c->nrec * sizeof(float4), hipMemcpyDeviceToHost));
        int64_t act = 0;
        for (auto &q : pos) act += (fbits_h(q.w) & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) == 0;
        st->gather_points = act;
        st->nodes_visited = counters[0];
        st->photons_in_radius = counters[1];
        st->ms_eye = t_eye; st->ms_trace = t_trace; st->ms_build = t_build; st->ms_gather = t_gather;
        st->ms_final = t_final;
    }
    return PM_OK;
}

/* ------------------------------------------------------- simple renderer */
int pm_simple_pass(void *ptr, const pm_render_params *p, void *d_out, void *stream) {
    GETCTX(ptr);
    if (!p) FAIL(c, PM_ERR_INVALID, "null params");
    if (!c->committed) FAIL(c, PM_ERR_INVALID, "scene not committed (call pm_commit)");
    if (!d_out) FAIL(c, PM_ERR_INVALID, "null output");
    const int64_t n = num_records(c);
    if (n <= 0) FAIL(c, PM_ERR_INVALID, "no eye samples (call pm_set_pinhole or pm_set_eye_rays)");
    if (!c->pinhole && c->rand2d_total > c->n2d)
        FAIL(c, PM_ERR_INVALID, "eye rays carry %d 2D samples, lights need %d", c->n2d, c->rand2d_total);
    hipStream_t s = pick(c, stream);
    EyeParams E{};
    E.S = c->S;
    E.R.count = n; /* the simple renderer keeps no records */
    E.pinhole = c->pinhole; E.W = c->W; E.H = c->H; E.n2d = c->n2d;
    E.eye = f4(c->eye[0], c->eye[1], c->eye[2], 0); E.fwd = f4(c->fwd[0], c->fwd[1], c->fwd[2], 0);
    E.right = f4(c->right[0], c->right[1], c->right[2], 0); E.up = f4(c->up[0], c->up[1], c->up[2], 0);
    E.rays = c->d_rays.as<float>(); E.rand2d = c->d_rand2d.as<float>();
    E.eps = p->scene_epsilon; E.light_seed = p->light_rng_seed;
    timer_begin(c, "simple", s);
    HIPCHK(c, launch_simple(E, (float *)d_out, s));
    timer_end(c, "simple", s);
    return PM_OK;
}

int pm_render_simple(void *ptr, const pm_render_params *p, float *out_rgb, pm_stats *st) {
    if (Group *g_ = group_of(ptr)) { /* direct light only: one device renders it */
        const int rc_ = pm_render_simple(g_->subs[0], p, out_rgb, st);
        return rc_ ? group_fail(ptr, g_->subs[0], rc_) : PM_OK;
    }
    GETCTX(ptr);
    if (!out_rgb) FAIL(c, PM_ERR_INVALID, "null output");
    const int64_t nout = c->pinhole ? (int64_t)c->W * c->H : c->nrays;
    if (nout > 0) HIPCHK(c, c->d_out.ensure(nout * 3 * sizeof(float)));
    hipStream_t s = c->stream;
    int rc;
    if ((rc = pm_simple_pass(c, p, c->d_out.p, s))) return rc;
    HIPCHK(c, hipMemcpyAsync(out_rgb, c->d_out.p, nout * 3 * sizeof(float), hipMemcpyDeviceToHost, s));
    HIPCHK(c, hipStreamSynchronize(s));
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->gather_points = nout;
        st->ms_eye = timer_ms(c, "simple");
    }
    return PM_OK;
}

/* ------------------------------------------------------- buffers / tests */
int64_t pm_num_records(void *ptr) {
    if (Group *g_ = group_of(ptr)) return pm_num_records(g_->subs[0]);
    Ctx *c = (Ctx *)ptr;
    return c ? num_records(c) : -1;
}

int pm_record_pixel(void *ptr, int64_t r, int64_t *pixel) {
    GETCTX(ptr);
    if (!pixel) FAIL(c, PM_ERR_INVALID, "null output");
    if (!c->pinhole) { *pixel = r; return PM_OK; }
    int64_t tile = r >> 6;
    int lane = (int)(r & 63), tilesX = (c->W + 7) / 8;
    int px = (int)(tile % tilesX) * 8 + (lane & 7), py = (int)(tile / tilesX) * 8 + (lane >> 3);
    *pixel = (px >= c->W || py >= c->H) ? -1 : (int64_t)py * c->W + px;
    return PM_OK;
}

int pm_download_slots(void *ptr, pm_photon *out, int64_t n) {
    GETCTX(ptr);
    int rc;
    if (!out || n < 0 || (size_t)n * sizeof(pm_photon) > c->d_slots.bytes) FAIL(c, PM_ERR_INVALID, "bad slot range");
    if ((rc = materialize_slots(c, nullptr))) return rc;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->d_slots.p, n * sizeof(pm_photon), hipMemcpyDeviceToHost));
    return PM_OK;
}

int pm_upload_slots(void *ptr, const pm_photon *in, int64_t n) {
    GETCTX(ptr);
    int rc;
    if (!in || n < 0) FAIL(c, PM_ERR_INVALID, "bad slots");
    if ((rc = materialize_slots(c, nullptr))) return rc;
    if ((rc = pm_reserve_slots(c, n, nullptr))) return rc;
    c->fused.valid = false;
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(c->d_slots.p, in, n * sizeof(pm_photon), hipMemcpyHostToDevice));
    c->slots_used = n;
    c->slots_nonneg = true;
    for (int64_t i = 0; i < n && c->slots_nonneg; ++i)
        if (in[i].bits & 1u) /* valid photon */
            c->slots_nonneg = in[i].alpha[0] >= 0.f && in[i].alpha[1] >= 0.f && in[i].alpha[2] >= 0.f;
    return PM_OK;
}

int pm_download_records(void *ptr, pm_record *out, int64_t n) {
    GETCTX(ptr);
    if (!out || n < 0 || n > c->nrec) FAIL(c, PM_ERR_INVALID, "bad record range");
    int rc;
    if ((rc = materialize_reset(c, c->stream))) return rc;
    HIPCHK(c, hipDeviceSynchronize());
    std::vector<float4> pos(n), nrm(n), st(n), dl(n);
    std::vector<float> N(n);
    HIPCHK(c, hipMemcpy(pos.data(), c->d_pos.p, n * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(nrm.data(), c->d_nrm.p, n * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(st.data(), c->d_state.p, n * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(dl.data(), c->d_dl.p, n * 16, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(N.data(), c->d_n.p, n * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; ++i) {
        pm_record &r = out[i];
        r.pos[0] = pos[i].x; r.pos[1] = pos[i].y; r.pos[2] = pos[i].z; r.flags = (uint32_t)fbits_h(pos[i].w);
        r.ns[0] = nrm[i].x; r.ns[1] = nrm[i].y; r.ns[2] = nrm[i].z; r.material = fbits_h(nrm[i].w);
        r.flux[0] = st[i].x; r.flux[1] = st[i].y; r.flux[2] = st[i].z; r.radius2 = st[i].w;
        r.dl[0] = dl[i].x; r.dl[1] = dl[i].y; r.dl[2] = dl[i].z; r.photon_count = N[i];
    }
    return PM_OK;
}

int pm_upload_records(void *ptr, const pm_record *in, int64_t n) {
    GETCTX(ptr);
    int rc;
    if (!in || n != num_records(c)) FAIL(c, PM_ERR_INVALID, "record count must equal pm_num_records");
    if ((rc = ensure_records(c))) return rc;
    std::vector<float4> pos(n), nrm(n), st(n), dl(n);
    std::vector<float> N(n);
    for (int64_t i = 0; i < n; ++i) {
        const pm_record &r = in[i];
        pos[i] = f4(r.pos[0], r.pos[1], r.pos[2], ibits((int)r.flags));
        nrm[i] = f4(r.ns[0], r.ns[1], r.ns[2], ibits(r.material));
        st[i] = f4(r.flux[0], r.flux[1], r.flux[2], r.radius2);
        dl[i] = f4(r.dl[0], r.dl[1], r.dl[2], 0.f);
        N[i] = r.photon_count;
    }
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(c->d_pos.p, pos.data(), n * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_nrm.p, nrm.data(), n * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_state.p, st.data(), n * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_dl.p, dl.data(), n * 16, hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->d_n.p, N.data(), n * 4, hipMemcpyHostToDevice));
    c->rec_fresh = false; /* every record overwritten */
    c->tiles_valid = false;
    r2_invalidate(c);
    if (c->view_active && (rc = build_view(c, c->stream))) return rc;
    return PM_OK;
}

int64_t pm_kdtree_nodes(void *ptr) {
    Ctx *c = (Ctx *)ptr;
    return c ? c->kd_count : -1;
}

int pm_download_kdtree(void *ptr, pm_photon *out, int64_t n) {
    GETCTX(ptr);
    if (!out || n < 0 || n > c->kd_count) FAIL(c, PM_ERR_INVALID, "bad kd range");
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(out, c->d_kd.p, n * sizeof(pm_photon), hipMemcpyDeviceToHost));
    return PM_OK;
}

int pm_gather_counters(void *ptr, int64_t out[4]) {
    GETCTX(ptr);
    unsigned long long h[4];
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h, c->d_counters.p, 32, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out[i] = (int64_t)h[i];
    return PM_OK;
}

int pm_trace_counters(void *ptr, int64_t out[4]) {
    GETCTX(ptr);
    unsigned long long h[4];
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(h, c->d_counters.as<unsigned long long>() + 4, 32, hipMemcpyDeviceToHost));
    for (int i = 0; i < 4; ++i) out[i] = (int64_t)h[i];
    return PM_OK;
}

int pm_map_info(void *ptr, int64_t out[4]) {
    GETCTX(ptr);
    if (!out) FAIL(c, PM_ERR_INVALID, "null output");
    out[0] = c->map_kind; out[1] = 0; out[2] = c->map_slots; out[3] = 0;
    if (c->map_kind == PM_GATHER_KDTREE) {
        out[1] = c->kd_count;
    } else if (c->map_kind == PM_GATHER_GRID) {
        uint32_t nv = 0;
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(&nv, c->d_cell_start.as<uint32_t>() + c->grid.ncells, 4, hipMemcpyDeviceToHost));
        out[1] = nv;
        out[3] = c->grid.ncells;
    }
    return PM_OK;
}

int pm_scene_info(void *ptr, int64_t out[7]) {
    if (Group *g_ = group_of(ptr)) return pm_scene_info(g_->subs[0], out);
    GETCTX(ptr);
    if (!c->S.blob) FAIL(c, PM_ERR_INVALID, "no scene committed");
    const SceneDev &S = c->S;
    out[0] = c->next_tri_id;   /* triangles rendered: meshes + every instance's */
    out[1] = S.n_disks; out[2] = S.n_spheres;
    /* the tree the kernels traverse: the 4-wide BVH when the scene has one
     * (either builder), else the binary SAH tree */
    out[3] = S.wide ? c->bvh4_nodes : S.n_nodes;
    out[4] = S.wide ? c->bvh4_depth : c->bvh_depth;
    out[5] = scene_mode(S) == MODE_BRUTE ? 2 : scene_mode(S) == MODE_LDS ? 1 : scene_mode(S) == MODE_INST ? 3 : 0;
    out[6] = S.blob_bytes;
    return PM_OK;
}

int pm_scene_section(void *ptr, int section, void *out, int64_t max_bytes, int64_t *bytes) {
    if (Group *g_ = group_of(ptr)) return pm_scene_section(g_->subs[0], section, out, max_bytes, bytes);
    GETCTX(ptr);
    if (!c->S.blob) FAIL(c, PM_ERR_INVALID, "no scene committed");
    const SceneDev &S = c->S;
    const void *src = nullptr;
    int64_t n = 0;
    switch (section) {
    case PM_SCENE_REFS: src = S.refs; n = 4 * (int64_t)S.n_refs; break;
    case PM_SCENE_TRI_GEO: src = S.tri_geo; n = 48 * (int64_t)S.n_tris; break;
    case PM_SCENE_TRI_SHADE: src = S.tri_shade; n = 32 * (int64_t)S.n_tris; break;
    case PM_SCENE_TRI_ID: src = S.tri_id; n = 4 * (int64_t)S.n_tris; break;
    case PM_SCENE_TRI_INFO: src = S.tri_info; n = 16 * (int64_t)S.n_tris; break;
    case PM_SCENE_BVH4: src = S.wnodes; n = S.wide ? (S.wide == 2 ? 64 : 128) * c->bvh4_nodes : 0; break; /* 3: 8-wide, 128 B */
    case PM_SCENE_INSTANCES: src = S.insts; n = 128 * (int64_t)S.n_inst; break;
    case PM_SCENE_OBJ_TRIS: src = S.obj_v; n = S.n_inst ? 48 * c->obj_tris_stored : 0; break;
    default: FAIL(c, PM_ERR_INVALID, "unknown scene section %d", section);
    }
    if (bytes) *bytes = n;
    if (out && n > 0) {
        if (max_bytes < n) FAIL(c, PM_ERR_INVALID, "scene section needs %lld bytes", (long long)n);
        HIPCHK(c, hipStreamSynchronize(c->stream));
        HIPCHK(c, hipMemcpy(out, src, (size_t)n, hipMemcpyDeviceToHost));
    }
    return PM_OK;
}

int pm_trace_profile(void *ptr, int64_t out[8], int reset) {
    GETCTX(ptr);
    unsigned long long h[8];
    HIPCHK(c, hipDeviceSynchronize());
    HIPCHK(c, hipMemcpy(h, c->d_counters.as<unsigned long long>() + 8, 64, hipMemcpyDeviceToHost));
    for (int i = 0; i < 8; ++i) out[i] = (int64_t)h[i];
    if (reset) HIPCHK(c, hipMemset(c->d_counters.as<unsigned long long>() + 8, 0, 64));
    return PM_OK;
}

int pm_final_view(void *ptr, double emitted, int64_t v_begin, int64_t v_count, void *d_out, void *stream) {
    GETCTX(ptr);
    if (!c->view_active) FAIL(c, PM_ERR_INVALID, "no active-record view (pm_set_record_view)");
    if (!d_out || v_begin < 0 || v_count < 0 || v_begin + v_count > c->n_view) FAIL(c, PM_ERR_INVALID, "bad view range");
    hipStream_t s = pick(c, stream);
    int rc;
    if ((rc = materialize_reset(c, s))) return rc;
    FinalParams F{};
    F.R = recs(c);
    F.knn = c->rec_estimator == PM_ESTIMATOR_KNN; F.materials = c->S.materials;
    F.emitted = (float)emitted;
    F.rec_begin = v_begin; F.rec_count = v_count; F.out = (float *)d_out; F.raster = 0; F.W = c->W;
    F.view = c->d_vlist.as<uint32_t>();
    timer_begin(c, "final", s);
    HIPCHK(c, launch_final(F, s));
    timer_end(c, "final", s);
    return PM_OK;
}

int pm_record_view_list(void *ptr, void *d_out, void *stream) {
    GETCTX(ptr);
    if (!c->view_active) FAIL(c, PM_ERR_INVALID, "no active-record view (pm_set_record_view)");
    if (!d_out) FAIL(c, PM_ERR_INVALID, "null output");
    if (c->n_view > 0)
        HIPCHK(c, hipMemcpyAsync(d_out, c->d_vlist.p, (size_t)c->n_view * 4, hipMemcpyDeviceToDevice, pick(c, stream)));
    return PM_OK;
}

int pm_set_record_view(void *ptr, int active_only, int64_t *n_view) {
    GETCTX(ptr);
    if (active_only) {
        if (c->nrec <= 0) FAIL(c, PM_ERR_INVALID, "no records (run pm_eye_pass first)");
        int rc;
        HIPCHK(c, hipDeviceSynchronize());
        if ((rc = build_view(c, c->stream))) return rc;
    }
    c->view_active = active_only != 0;
    if (n_view) *n_view = view_size(c);
    return PM_OK;
}

int pm_set_counting(void *ptr, int enabled) {
    GETCTX(ptr);
    c->counting = enabled != 0;
    return PM_OK;
}

int pm_set_stage_timing(void *ptr, const char *stages) {
    GETCTX(ptr);
    if (c->stage_active) FAIL(c, PM_ERR_INVALID, "stage timing changed inside a stage");
    c->timed_stages = stages ? stages : "";
    return PM_OK;
}

int pm_synchronize(void *ptr) {
    GROUP_FWD(ptr, pm_synchronize(sub));
    GETCTX(ptr);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return PM_OK;
}

int pm_last_kernel_ms(void *ptr, const char *name, double *ms) {
    GETCTX(ptr);
    if (!name || !ms) FAIL(c, PM_ERR_INVALID, "null argument");
    *ms = timer_ms(c, name);
    if (*ms < 0) FAIL(c, PM_ERR_INVALID, "no timing recorded for '%s'", name);
    return PM_OK;
}

int pm_timing_reset(void *ptr) {
    GETCTX(ptr);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (auto &kv : c->timers) kv.second.used = 0;
    return PM_OK;
}

int pm_timing_total(void *ptr, const char *name, int64_t *count, double *total_ms) {
    GETCTX(ptr);
    if (!name || !count || !total_ms) FAIL(c, PM_ERR_INVALID, "null argument");
    *count = 0;
    *total_ms = 0.0;
    auto it = c->timers.find(name);
    if (it == c->timers.end()) return PM_OK;
    for (size_t i = 0; i < it->second.used; ++i) {
        double ms = pair_ms(it->second.ev[i]);
        if (ms < 0) FAIL(c, PM_ERR_HIP, "event timing failed for '%s'", name);
        *total_ms += ms;
    }
    *count = (int64_t)it->second.used;
    return PM_OK;
}

int pm_reset_records(void *ptr, const pm_render_params *p, void *stream) {
    GETCTX(ptr);
    int rc;
    if ((rc = check_params(c, p))) return rc;
    if (c->nrec <= 0) FAIL(c, PM_ERR_INVALID, "no records (run pm_eye_pass first)");
    (void)stream;
    /* deferred: the next fused full gather starts from the initial state, any
     * other reader applies it first (materialize_reset) */
    c->rec_fresh = true;
    c->rec_fresh_r2 = p->initial_radius2;
    r2_invalidate(c);
    return PM_OK;
}

} /* extern "C" */
