/*
 * pm_api.h — C-ABI of the MI355X photon-mapping renderer (libpmhip.so).
 *
 * This is the drop-in boundary. The reference exposes a C++ plugin surface to
 * pbrt-v2 (cuda_render/cudaapi.h:8-19 + class CudaRender : Renderer,
 * cuda_render/cudarender.h:22-91) whose implementation talks to OptiX. Here
 * that surface is kept by a thin C++ adapter (cuda-raytrace_amd/adapter/,
 * see INTEGRATION.md) that flattens pbrt objects into the POD calls below.
 * Every entry point is `extern "C"`, takes plain pointers and sizes, returns
 * an int status (PM_OK = 0) and never throws; the message of the last failure
 * is available from pm_last_error(). Caller-owned input arrays are copied
 * during the call. A context is single-threaded (like the reference's global
 * gContext, cudarender.cpp:14) and bound to one HIP device.
 *
 * Mapping to the reference (file:line of the function each entry replaces):
 *   pm_create / pm_destroy        CudaRenderInit        cudaapi.cpp:4-7, cudarender.cpp:17-36
 *   pm_add_material               CudaMaterial::createCudaMeteral  util/material/cudamaterial.cpp:8-21
 *   pm_add_trimesh                CudaTriangleMesh::setupGeometry  util/shape/cudatrianglemesh.cpp:16-73
 *   pm_add_sphere                 CudaSphere::setupTransform       util/shape/cudasphere.cpp:15-40
 *   pm_add_disk                   CudaDisk::setupGeometry          util/shape/cudadisk.cpp:15-45
 *   pm_add_light_point            CudaLight::setupLight<PointLight>        util/light/cudalight.cpp:16-24
 *   pm_add_light_disk             CudaLight::setupLight<DiffuseAreaLight>  util/light/cudalight.cpp:26-59
 *   pm_set_eye_rays               PbrtCamera::preLaunch (bRays, bRandom2D) util/camera/pbrtcamera.cpp:57-122
 *   pm_set_pinhole                (on-device eye rays for synthetic benches)
 *   pm_commit                     CudaRender::Render → assembleNode (Sbvh build)  cudarender.cpp:38-75,112-123
 *   pm_render                     PhotonMappingRenderer::render    photon_mapping/photonmappingrenderer.cpp:31-45
 *   pm_eye_pass                   RaytracingPass                   photonmappingrenderer.cpp:108-139 (+ raytracing.cu)
 *   pm_trace_photons              PhotonTracingPass                photonmappingrenderer.cpp:204-226 (+ photontracing.cu)
 *   pm_build_photon_map           CreatePhotonMap                  photonmappingrenderer.cpp:150-180
 *   pm_gather                     PhotonGatheringPass              photonmappingrenderer.cpp:228-232 (+ gathering.cu:104-126)
 *   pm_final                      FinalGatheringPass               photonmappingrenderer.cpp:234-277 (+ gathering.cu:129-146)
 *   pm_render_simple              SimpleRenderer::render           simple_render/simplerender.cpp:18-103 (+ simplerender.cu)
 */
#ifndef PM_API_H
#define PM_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define PM_OK 0
#define PM_ERR_INVALID 1     /* bad argument / call order */
#define PM_ERR_HIP 2         /* HIP runtime failure (message has hipGetErrorString) */
#define PM_ERR_NO_PHOTONS 3  /* 0 valid photons: reference raises Severe, photonmappingrenderer.cpp:165-167 */
#define PM_ERR_NOMEM 4

/* ---- enums (values equal the reference's) ----------------------------- */
/* MaterialType, util/common.cu.h:61-63 */
#define PM_MATTE 0
#define PM_MIRROR 1
#define PM_GLASS 2
/* CudaLightDevice::LightType, util/common.cu.h:48 */
#define PM_LIGHT_POINT 1
#define PM_LIGHT_AREA_DISK 3
/* RayTracingRecord flags, photon_mapping/photonmapping.h:25-26 (+ INVALID for padding) */
#define PM_REC_EXCEPTION 0x01u
#define PM_REC_MISS 0x02u
#define PM_REC_INVALID 0x04u
/* the eye ray hit the back of the shading normal: dot(ns, wo) < 0 with
 * wo = -ray.direction (RayTracingRecord::direction, photonmapping.h:18) —
 * what pbrt's Faceforward(nn, wo) needs in the kNN estimator */
#define PM_REC_BACKFACE 0x08u
/* gather structures */
#define PM_GATHER_GRID 0   /* hashed uniform grid of photon buckets (default, fastest) */
#define PM_GATHER_KDTREE 1 /* reference-layout kd-tree (CudaPhoton nodes, pbrt median split) */
/* multi-GPU photon exchange */
#define PM_EXCHANGE_REDUCE 0   /* local maps, per-record (M, L) reduce-scatter */
#define PM_EXCHANGE_ALLGATHER 1 /* all-gather photon slots, replicated map */
/* radiance estimators of the gather (pm_render_params::estimator) */
#define PM_ESTIMATOR_PPM 0 /* the reference's: fixed-radius query + progressive update (gathering.cu:17-146) */
#define PM_ESTIMATOR_KNN 1 /* pbrt-v2 PhotonIntegrator::LPhoton: k nearest photons, Simpson kernel */
#define PM_KNN_MAX 64      /* largest knn_lookup */

/* ---- POD layouts shared with tests / other hosts ----------------------- */

/* Photon slot == kd-node, bit-for-bit the reference's CudaPhoton
 * (photon_mapping/photonmapping.h:32-41): word = hasLeftChild:1 | splitAxis:2
 * | rightChild:29 (LSB first). Before the tree is built bit 0 is the valid
 * bit (photonmapping.h:43-56). 40 bytes. */
typedef struct pm_photon {
    uint32_t bits;
    float p[3];
    float alpha[3];
    float wi[3];
} pm_photon;
#define PM_PHOTON_MAX_RIGHT_CHILD ((1u << 29) - 1u) /* photonmapping.h:41 */

/* Gather-point record (the subset of RayTracingRecord, photonmapping.h:7-24,
 * that the gather and final passes read). 64 bytes, AoS for exchange; the
 * device keeps it as SoA. Under PM_ESTIMATOR_KNN,
 * flux accumulates the per-pass sums, radius2 holds the last pass's r_k^2
 * (pbrt's shrunk maxDistSquared) and photon_count its number of photons
 * found. */
typedef struct pm_record {
    float pos[3];
    uint32_t flags;
    float ns[3];    /* normalized world shading normal */
    int32_t material;
    float flux[3];
    float radius2;
    float dl[3];    /* direct light */
    float photon_count;
} pm_record;

typedef struct pm_config {
    int device;          /* HIP device ordinal (n_devices == 0) */
    /* n_devices > 0: one context over devices[0 .. n_devices) of this node
     * (photon paths sharded by global id, RCCL all-gather of
     * the slots, interleaved 8-row bands per device). It takes the scene
     * calls, pm_render and pm_render_simple; the stage API needs one context
     * per device (one process per GPU, pmrender/dist.py). The reference is
     * single-context (cudarender.cpp:14), so this is new surface. */
    int n_devices;
    const int *devices;
    int reserved[4];
} pm_config;

/* Render parameters. Defaults (pm_default_params) are the reference's
 * hard-coded constants. */
typedef struct pm_render_params {
    float scene_epsilon;     /* 0.1   photonmappingrenderer.cpp:52 */
    float initial_radius2;   /* 4.0   raytracing.cu:123 */
    float ppm_alpha;         /* 0.7   gathering.cu:115 */
    int max_photon_count;    /* 4     photonmappingrenderer.cpp:183 (deposits per path) */
    int64_t paths_per_pass;  /* 262144 = 512*512, photonmappingrenderer.cpp:184-185,214 */
    int passes;              /* 1     photonmappingrenderer.cpp:38 */
    int light_source_index;  /* 0     photonmappingrenderer.cpp:211 */
    int max_specular_depth;  /* 10    raytracing.cu:98 (eye); build cap for photons (SURVEY App.B 5) */
    uint32_t rng_seed;       /* 777   util/random/cudarandom.h:15 */
    uint32_t light_rng_seed; /* 2047  (cudalight.cpp:530, commented-out light RNG seed) */
    int gather_structure;    /* PM_GATHER_GRID */
    /* PM_ESTIMATOR_PPM (default) or PM_ESTIMATOR_KNN: per pass, the knn_lookup
     * nearest photons with d^2 < initial_radius2 (pbrt's maxdist^2) give
     * sum_i Simpson(d_i^2, r_k^2) / r_k^2 * alpha_i over photons on the
     * viewer's side (pbrt photonmap.cpp LPhoton, diffuse branch); passes are
     * averaged. Photon-bucket gather only; not linear in the photon set, so
     * no partial/split gathers (multi-GPU: the all-gather exchange). */
    int estimator;
    int knn_lookup;          /* 50    pbrt PhotonIntegrator "nused" */
    int reserved[4];
} pm_render_params;

typedef struct pm_stats {
    int64_t paths_emitted;    /* total over passes */
    int64_t photons_valid;    /* last pass */
    int64_t gather_points;    /* active records (not MISS/EXC/INVALID) */
    int64_t nodes_visited;    /* last gather pass: photons tested (grid) or kd nodes visited */
    int64_t photons_in_radius;/* last gather pass: sum of M */
    double ms_eye, ms_trace, ms_build, ms_gather, ms_final; /* device time, summed over passes */
} pm_stats;

/* ---- lifecycle -------------------------------------------------------- */
void pm_default_params(pm_render_params *p);
int pm_create(void **ctx, const pm_config *cfg);
void pm_destroy(void *ctx);
const char *pm_last_error(void *ctx);
const char *pm_version(void);

/* ---- scene ------------------------------------------------------------ */
/* returns material id in *out_id. rgb = Kd (matte) / Kr (mirror, ignored by
 * the device as in cudamaterial.cu.h:101-105) / unused (glass). */
int pm_add_material(void *ctx, int type, const float rgb[3], int *out_id);
/* World-space mesh (pbrt TriangleMesh::p is already world space,
 * cudatrianglemesh.cpp:24-30). N and uv may be NULL. light_index = index of
 * the area light this shape emits for, -1 otherwise. */
int pm_add_trimesh(void *ctx, const float *P, int nverts, const int *indices, int ntris,
                   const float *N, const float *uv, int material, int light_index);
/* Object instancing (the reference's CudaObjectInstance, cudaapi.h:17 /
 * cudarender.cpp:88-103: an OptiX Transform over the instance's group).
 * pm_add_object_mesh stores a mesh once, in object space (arguments as
 * pm_add_trimesh), without rendering it; *out_object = its id.
 * pm_add_mesh_instance places it with a row-major affine object-to-world
 * matrix (last row 0 0 0 1, else PM_ERR_INVALID) and its inverse: the scene
 * gets a two-level tree (the object's own 4-wide tree, entered from the
 * top-level one), and every hit, shading frame and photon equals the hit of
 * the mesh flattened to world space with pbrt's Transform (points:
 * m[0]*x + m[1]*y + m[2]*z + m[3] per row, left to right; normals: the
 * transpose of w2o) and added with pm_add_trimesh at this call (global ids
 * in call order). */
int pm_add_object_mesh(void *ctx, const float *P, int nverts, const int *indices, int ntris,
                       const float *N, const float *uv, int material, int light_index, int *out_object);
int pm_add_mesh_instance(void *ctx, int object, const float o2w[16], const float w2o[16]);
/* Object-space sphere (cudasphere.cpp:15-40): row-major 4x4 matrices. */
int pm_add_sphere(void *ctx, float radius, const float o2w[16], const float w2o[16],
                  int material, int light_index);
/* World-space disk, already flattened as in cudadisk.cpp:24-43: o = O2W(0,0,h),
 * x = O2W(r,0,0), y = O2W(0,r,0), z = normalize(O2W(0,0,1)),
 * inner_norm = innerRadius/radius, phi_max in radians. */
int pm_add_disk(void *ctx, const float o[3], const float x[3], const float y[3],
                const float z[3], float inner_norm, float phi_max, int material, int light_index);
int pm_add_light_point(void *ctx, const float pos[3], const float intensity[3]);
/* Disk area light (cudalight.cpp:34-53): o centre, p1/p2 world radius vectors,
 * n normal, Le emitted radiance, area, n_samples shadow samples. */
int pm_add_light_disk(void *ctx, const float o[3], const float p1[3], const float p2[3],
                      const float n[3], const float Le[3], float area, int n_samples);

/* Eye samples. Either a pinhole camera evaluated on the device (records in
 * 8x8-pixel tile order, output in raster order) ... */
int pm_set_pinhole(void *ctx, const float eye[3], const float fwd[3], const float right[3],
                   const float up[3], int width, int height);
/* ... or host-generated rays in sampler order, as PbrtCamera::preLaunch
 * packs them (o.xyz, d.xyz per ray; rand2d = n2d float2 per ray, indexed
 * [ray][random2DStart + s], cudalight.cu.h:34-35). */
int pm_set_eye_rays(void *ctx, const float *rays, int64_t nrays, const float *rand2d, int n2d);

/* Builds the BVH and uploads the scene. Must follow the last pm_add_*. */
int pm_commit(void *ctx);

/* ---- whole render (PhotonMappingRenderer::render) ---------------------- */
/* out_rgb: host float[3 * nrays] (rays mode) or float[3 * W * H] (pinhole,
 * raster order), NaN/negative/inf sanitized to black like
 * photonmappingrenderer.cpp:251-268. stats may be NULL. */
int pm_render(void *ctx, const pm_render_params *params, float *out_rgb, pm_stats *stats);

/* ---- simple renderer (SimpleRenderer::render, simple_render/simplerender.cpp:18-103)
 * Direct light only: closest hit of each eye sample, one shadow-tested sample
 * per light (sample index 0, no pdf division, no emitted term,
 * simplerender.cu:40-72), miss = black; NaN / negative / inf sanitized like
 * simplerender.cpp:70-87. The reference sets scene_epsilon to 0.01 for it
 * (simplerender.cpp:23, PM_SIMPLE_SCENE_EPSILON); params->scene_epsilon is
 * used as given, and params->light_rng_seed feeds the pinhole mode's disk
 * samples. out_rgb as pm_render. */
#define PM_SIMPLE_SCENE_EPSILON 0.01f
int pm_render_simple(void *ctx, const pm_render_params *params, float *out_rgb, pm_stats *stats);
/* the same into a device buffer (float3 per output sample) on `stream` */
int pm_simple_pass(void *ctx, const pm_render_params *params, void *d_out, void *stream);

/* ---- stage-level API (device-resident state, explicit stream) ---------- */
/* `stream` is a hipStream_t (NULL = the context's own stream). */
int pm_eye_pass(void *ctx, const pm_render_params *params, void *stream);
/* Emits paths [path_begin, path_begin + path_count) of `pass` into the
 * context's slot buffer at slot offset (path - slot_path_base) * max_photon_count.
 * Global path ids keep the Halton / Philox streams identical for any sharding. */
int pm_trace_photons(void *ctx, const pm_render_params *params, int pass, int64_t path_begin,
                     int64_t path_count, int64_t slot_path_base, void *stream);
/* Builds the gather structure from the first n_slots slots (n_slots<=0: all). */
int pm_build_photon_map(void *ctx, const pm_render_params *params, int64_t n_slots, void *stream);
/* Fused range query + PPM update over all records ... */
int pm_gather(void *ctx, const pm_render_params *params, void *stream);
/* ... or over records [rec_begin, rec_begin + rec_count) (tile-owned gather). */
int pm_gather_range(void *ctx, const pm_render_params *params, int64_t rec_begin, int64_t rec_count,
                    void *stream);
/* Range query only: writes per record four int64 (M, L.r, L.g, L.b) to
 * d_partial (device pointer, 32 B x records of the view, see
 * pm_set_record_view); L is in the gather's exact fixed point, so partials of
 * photon shards sum to the 1-GPU result. */
int pm_gather_partial(void *ctx, const pm_render_params *params, void *d_partial, void *stream);
/* The "reduce" exchange's split partials: per view record an int32 photon
 * count M (d_count, n_view entries) and the flux sum as three int64 in the
 * gather's fixed point (d_flux, 3 x n_view, record-major). Summed over the
 * photon shards they equal a 1-GPU gather exactly. A pending pm_reset_records
 * is honoured (initial radius) and left to pm_ppm_update_split. */
int pm_gather_split(void *ctx, const pm_render_params *params, void *d_count, void *d_flux, void *stream);
/* PPM update (gathering.cu:115-125) from split partials summed over ranks:
 * radius2 and photon count of EVERY view record from the global counts
 * (d_count, n_view int32: all-reduced, so every rank updates every radius
 * itself and no radius exchange is needed), flux of view records
 * [v_begin, v_begin + v_count) from d_flux_chunk (3 int64 each:
 * reduce-scattered to the owner). Consumes a pending pm_reset_records. */
int pm_ppm_update_split(void *ctx, const pm_render_params *params, const void *d_count, const void *d_flux_chunk,
                        int64_t v_begin, int64_t v_count, void *stream);
/* The same update in two halves, so that the flux reduce-scatter of pass k
 * can still be in flight while pass k + 1 gathers (pmrender/dist.py):
 * pm_ppm_update_split_radius applies the global counts (d_count) to radius2
 * and photon count of every view record and writes each record's ratio
 * N'/(N + M) to d_ratio (n_view floats; < 0: nothing to apply), consuming a
 * pending pm_reset_records (a fresh record's flux is set to 0);
 * pm_ppm_update_split_flux later applies flux = (flux + L) * ratio to view
 * records [v_begin, v_begin + v_count) from d_flux_chunk. Together they are
 * pm_ppm_update_split bit for bit (gathering.cu:115-125 order of operations). */
int pm_ppm_update_split_radius(void *ctx, const pm_render_params *params, const void *d_count, void *d_ratio,
                               void *stream);
int pm_ppm_update_split_flux(void *ctx, const pm_render_params *params, const void *d_ratio,
                             const void *d_flux_chunk, int64_t v_begin, int64_t v_count, void *stream);
/* Record view of pm_gather_partial, pm_ppm_update, pm_get_radius2 and
 * pm_set_radius2 (their rec_begin / rec_count and buffers index the view):
 * active_only = 0 -> all records (default); 1 -> only active records (not
 * MISS / EXCEPTION / INVALID), compacted in record order — what a multi-GPU
 * exchange has to move (53% of the records at C2). The view is rebuilt by
 * every pm_eye_pass / pm_upload_records. *n_view = records in the view. */
int pm_set_record_view(void *ctx, int active_only, int64_t *n_view);
/* With the active view set: final radiance of view records [v_begin,
 * v_begin + v_count) into d_out (float3 each, view order) and the view's
 * record indices (uint32 x n_view) — records outside the view are black. */
int pm_final_view(void *ctx, double emitted, int64_t v_begin, int64_t v_count, void *d_out, void *stream);
int pm_record_view_list(void *ctx, void *d_out, void *stream);
/* PPM update of records [rec_begin, rec_begin+rec_count) from summed partials
 * (d_partial points at the partial of rec_begin). */
int pm_ppm_update(void *ctx, const pm_render_params *params, const void *d_partial,
                  int64_t rec_begin, int64_t rec_count, void *stream);
/* radius^2 of records [rec_begin, rec_begin+rec_count) to / from a device
 * float array (d_out[i] / d_in[i] is record rec_begin + i). The owner of a
 * record chunk publishes its updated radii so every rank queries the next
 * pass with the current radius (multi-GPU "reduce" exchange). */
int pm_get_radius2(void *ctx, int64_t rec_begin, int64_t rec_count, void *d_out, void *stream);
int pm_set_radius2(void *ctx, const void *d_in, int64_t rec_begin, int64_t rec_count, void *stream);
/* Final radiance of records [rec_begin, rec_begin+rec_count) into the device
 * buffer d_out (float3 per record, RECORD order) — emitted = total paths. */
int pm_final(void *ctx, double emitted, int64_t rec_begin, int64_t rec_count, void *d_out, void *stream);

/* ---- buffers, sizes, host transfer (tests / distributed glue) ---------- */
int64_t pm_num_records(void *ctx);
int pm_record_pixel(void *ctx, int64_t rec, int64_t *pixel); /* -1 if padding */
/* slot buffer capacity management; returns device pointer of the slots */
int pm_reserve_slots(void *ctx, int64_t n_slots, void **d_slots);
/* Use a caller-owned device buffer (n_slots pm_photon) as the slot buffer,
 * e.g. a torch tensor that an RCCL all-gather fills; NULL reverts to the
 * context's own buffer. The caller keeps it alive while the context uses it. */
int pm_set_slot_buffer(void *ctx, void *d_slots, int64_t n_slots);
int pm_download_slots(void *ctx, pm_photon *out, int64_t n);
int pm_upload_slots(void *ctx, const pm_photon *in, int64_t n);
int pm_download_records(void *ctx, pm_record *out, int64_t n);
int pm_upload_records(void *ctx, const pm_record *in, int64_t n);
/* kd-tree nodes of the last PM_GATHER_KDTREE build (reference layout) */
int64_t pm_kdtree_nodes(void *ctx);
int pm_download_kdtree(void *ctx, pm_photon *out, int64_t n);
/* counters of the last gather: [0] photons (grid) or kd nodes visited,
 * [1] photons in radius (sum of M), [2] bucket rows read (grid), [3] active records */
int pm_gather_counters(void *ctx, int64_t out[4]);
/* counters of the last pm_trace_photons with counting on: [0] rays traced,
 * [1] BVH nodes entered, [2] primitive intersection tests, [3] photons
 * deposited (the traffic census behind the trace roofline) */
int pm_trace_counters(void *ctx, int64_t out[4]);
/* the loaded scene as the traversal kernels see it: [0] triangles rendered
 * (an instanced mesh counted once per instance), [1] disks, [2] spheres,
 * [3] BVH nodes, [4] BVH depth, [5] traversal mode (0 BVH in HBM, 1 BVH in
 * LDS, 2 brute force over an LDS-sized scene, 3 two-level: top tree over
 * instance boxes + one tree per object mesh), [6] scene bytes.
 * [3] / [4] describe the tree the kernels traverse: with mode 0 that is the
 * 4-wide quantized BVH (its node count and its depth in 4-wide levels),
 * whichever builder made it (device PLOC for >= 65,536 primitives, else the
 * host SAH build collapsed); with mode 1 the binary SAH tree */
int pm_scene_info(void *ctx, int64_t out[7]);
/* diagnostics: one section of the committed scene as the kernels read it
 * (refs; per storage slot the triangle records geo 48 B, shade 32 B, id,
 * info 16 B; the 4-wide nodes, 64 B quantized or 128 B float). *bytes = its
 * size; out may be null to query it, else max_bytes must hold it. Lets a
 * test compare the device-built tree with its host restatement. */
#define PM_SCENE_REFS 0
#define PM_SCENE_TRI_GEO 1
#define PM_SCENE_TRI_SHADE 2
#define PM_SCENE_TRI_ID 3
#define PM_SCENE_TRI_INFO 4
#define PM_SCENE_BVH4 5
#define PM_SCENE_INSTANCES 6 /* 128 B per instance (pm_device.h SceneDev::insts) */
#define PM_SCENE_OBJ_TRIS 7  /* 48 B per stored object triangle (object-space p0, p1, p2) */
int pm_scene_section(void *ctx, int section, void *out, int64_t max_bytes, int64_t *bytes);
/* the current photon map (pm_build_photon_map; the reference's
 * CreatePhotonMap, photonmappingrenderer.cpp:150-180): [0] structure
 * (PM_GATHER_GRID / PM_GATHER_KDTREE, -1 none), [1] valid photons in it,
 * [2] slots it was built from, [3] grid cells (0 for the kd-tree) */
int pm_map_info(void *ctx, int64_t out[4]);
/* Phase profile of the trace kernel, summed over waves and launches since the
 * last reset: shader-clock cycles in [0] emission, [1] BVH traversal,
 * [2] shading + bounce + deposit, [3] compaction barrier, [4] state exchange,
 * [5] unused, [6] wave lifetime, [7] waves. All zero unless the library was
 * built with PROF=1 (lib/libpmhip_prof.so); a measurement hook, not used by
 * the render path. */
int pm_trace_profile(void *ctx, int64_t out[8], int reset);
/* enable/disable census counters in the trace and gather kernels (off by
 * default: costs an atomic per wave) */
int pm_set_counting(void *ctx, int enabled);
int pm_synchronize(void *ctx);
/* Stage timings measured with HIP events recorded on the stream the kernels
 * run on. Stage names: "eye", "trace", "build", "gather", "update", "final",
 * "reset". last = most recent launch; total = sum over launches since
 * pm_timing_reset (synchronizes on the last event only when read). */
int pm_last_kernel_ms(void *ctx, const char *name, double *ms);
/* Which stages record events: "all" (default), "" / NULL (none) or a comma
 * list ("gather"). Each timed stage boundary costs a few us of GPU idle
 * time, so a throughput run times only the stage it reports on. */
int pm_set_stage_timing(void *ctx, const char *stages);
int pm_timing_reset(void *ctx);
int pm_timing_total(void *ctx, const char *name, int64_t *count, double *total_ms);
/* Restores every active record to the eye pass's initial PPM state
 * (flux 0, photon_count 0, radius2 = initial_radius2). */
int pm_reset_records(void *ctx, const pm_render_params *params, void *stream);

/* Host-only (no device needed): the canonical pbrt-v2 KdTree over the valid
 * slots in the reference node layout, i.e. what CreatePhotonMap
 * (photonmappingrenderer.cpp:150-180) uploads. nodes_out holds >= nslots
 * entries; returns the node count (= valid photons). */
int64_t pm_kdtree_build_host(const pm_photon *slots, int64_t nslots, pm_photon *nodes_out);

/* Halton permutation of PermutedHalton(5, RNG(seed)) (28 uints), exposed for tests. */
int pm_halton_permutation(uint32_t seed, uint32_t out[28]);

#ifdef __cplusplus
}
#endif
#endif /* PM_API_H */
