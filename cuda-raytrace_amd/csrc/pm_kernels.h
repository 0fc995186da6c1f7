/*
 * pm_kernels.h — kernel parameter blocks and launcher declarations shared by
 * the host orchestration (pm_api.cpp) and the HIP kernels (pm_kernels.hip).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pm_device.h"

namespace pm {

constexpr int EYE_BLOCK = 128;     /* traversal kernels: LDS stack column per lane */
constexpr int TRACE_BLOCK = 128;
constexpr int BVH_STACK = BVH_STACK_DEPTH; /* >= max BVH depth (builder enforces it) */
constexpr int GATHER_BLOCK = 256;
constexpr int KD_STACK = 32;       /* >= pbrt median kd-tree depth for < 2^31 photons */

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

struct TraceParams {
    SceneDev S;
    pm_photon *slots;
    uint32_t perm[28];
    int64_t path_begin, path_count, slot_path_base;
    int pass, mpc, max_spec, light_index;
    float eps;
    uint32_t seed;
};

struct GridDesc {
    float gx, gy, gz, inv_cs;
    int dx, dy, dz;
    uint32_t ncells;
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
    const float4 *ph_b;         /* alpha.rgb, wi.y */
    const float *ph_c;          /* wi.z */
    /* kd-tree (reference layout) */
    const pm_photon *kd_nodes;
    int64_t kd_count;
    /* partial mode */
    float4 *partial;
    unsigned long long *counters; /* [0] visited, [1] in radius */
};

struct FinalParams {
    RecordsDev R;
    float emitted;
    int64_t rec_begin, rec_count;
    float *out;     /* float3 */
    int raster;     /* 1: out indexed by pixel (pinhole), 0: by record - rec_begin */
    int W;
};

hipError_t launch_eye(const EyeParams &p, hipStream_t s);
hipError_t launch_trace(const TraceParams &p, hipStream_t s);
/* grid build */
hipError_t launch_grid_keys(const pm_photon *slots, int64_t n, GridDesc g, uint32_t *keys, uint32_t *vals,
                            uint32_t *cell_count, uint32_t *n_valid, hipStream_t s);
size_t grid_sort_temp_bytes(int64_t n, uint32_t ncells);
hipError_t launch_grid_sort(void *temp, size_t temp_bytes, uint32_t *keys_in, uint32_t *keys_out,
                            uint32_t *vals_in, uint32_t *vals_out, int64_t n, int end_bit, hipStream_t s);
size_t grid_scan_temp_bytes(uint32_t ncells);
hipError_t launch_grid_scan(void *temp, size_t temp_bytes, const uint32_t *cell_count, uint32_t *cell_start,
                            uint32_t ncells, hipStream_t s);
hipError_t launch_grid_scatter(const pm_photon *slots, const uint32_t *sorted_vals, const uint32_t *n_valid,
                               int64_t n, float4 *ph_a, float4 *ph_b, float *ph_c, hipStream_t s);
/* gather: structure 0 grid, 1 kd; mode 0 fused PPM, 1 partial */
hipError_t launch_gather(const GatherParams &p, int structure, int partial, int count, hipStream_t s);
hipError_t launch_ppm_update(const GatherParams &p, const float4 *partial, int64_t rec_begin, int64_t rec_count,
                             hipStream_t s);
hipError_t launch_final(const FinalParams &p, hipStream_t s);
hipError_t launch_reset_records(const RecordsDev &R, float r2init, hipStream_t s);

} // namespace pm
