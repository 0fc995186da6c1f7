/*
 * pm_trace.hip — eye-pass and photon-pass kernels (HIP/CDNA4).
 *
 *   k_eye        eye pass: camera ray -> specular chain -> gather record +
 *                direct light with shadow rays   (raytracing.cu:19-147)
 *   k_trace      photon emission + bounce, <= max_photon_count deposits per
 *                path into owner-written slots   (photontracing.cu:80-185)
 * (photon buckets: pm_bucket.hip; gather/PPM/final: pm_gather.hip)
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "pm_kernels.h"

#pragma clang fp contract(off)

namespace pm {

/* ====================================================================== */
/* eye pass                                                               */
/* ====================================================================== */
template <int MODE>
__global__ __launch_bounds__(EYE_BLOCK) void k_eye(EyeParams P) {
    extern __shared__ __attribute__((aligned(16))) int stk[]; /* [stack_depth x EYE_BLOCK][scene blob (LDS)] */
    int *stack = stk + threadIdx.x;
    const SceneDev S = scene_view<mode_lds(MODE)>(P.S, reinterpret_cast<uint4 *>(stk + P.S.stack_depth * EYE_BLOCK),
                                                       threadIdx.x, EYE_BLOCK);
    if (mode_lds(MODE)) __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * EYE_BLOCK + threadIdx.x;
    if (r >= P.R.count) return;

    Ray ray;
    int64_t pixel;
    float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (P.pinhole) {
        int px, py;
        rec_to_pixel(r, P.W, &px, &py);
        if (px >= P.W || py >= P.H) {
            P.R.pos[r] = make_float4(0.f, 0.f, 0.f, __int_as_float(PM_REC_INVALID));
            P.R.nrm[r] = zero4; P.R.state[r] = zero4; P.R.n[r] = 0.f; P.R.dl[r] = zero4;
            return;
        }
        pixel = (int64_t)py * P.W + px;
        float sx = (2.0f * ((float)px + 0.5f)) / (float)P.W - 1.0f;
        float sy = 1.0f - (2.0f * ((float)py + 0.5f)) / (float)P.H;
        v3 d = xyz(P.fwd) + sx * xyz(P.right) + sy * xyz(P.up);
        ray.o = xyz(P.eye);
        ray.d = normalize(d);
    } else {
        pixel = r;
        const float *q = P.rays + 6 * r;
        ray.o = mk(q[0], q[1], q[2]);
        ray.d = mk(q[3], q[4], q[5]);
    }
    ray.tmin = P.eps;
    ray.tmax = RT_DEFAULT_MAX;

    int depth = 0;
    Hit h;
    Geo g;
    uint32_t flags = 0;
    while (true) {
        if (!traverse<false, MODE>(S, ray, h, stack, EYE_BLOCK)) { flags = PM_REC_MISS; break; }
        g = shade<MODE == MODE_INST>(S, ray, h);
        const v3 point = ray.o + ray.d * h.t;
        int mtype = fbits(S.materials[g.material].w);
        if (is_specular(mtype)) {
            v3 wi;
            bool ok = material_specular(mtype, g, -ray.d, &wi);
            depth++;
            if (depth > P.max_spec || !ok) { flags = PM_REC_EXCEPTION; break; }
            ray.o = point; ray.d = wi; ray.tmin = P.eps; ray.tmax = RT_DEFAULT_MAX;
            continue;
        }
        ray.o = point; /* keep the hit point; ray.d stays the incident direction */
        break;
    }
    if (flags) {
        P.R.pos[r] = make_float4(0.f, 0.f, 0.f, __int_as_float((int)flags));
        P.R.nrm[r] = zero4; P.R.state[r] = zero4; P.R.n[r] = 0.f; P.R.dl[r] = zero4;
        return;
    }
    const v3 point = ray.o, ns = g.ns, dir = ray.d;

    /* directLight (raytracing.cu:49-84) */
    v3 L = mk(0.f, 0.f, 0.f);
    const int total = S.n_lights;
    if (g.light < total) {
        if (g.light >= 0) L = L + light_le(S.lights[g.light], -dir);
        float4 m = S.materials[g.material];
        v3 fv = fbits(m.w) == PM_MATTE ? xyz(m) * INV_PI : mk(0.f, 0.f, 0.f);
        for (int i = 0; i < total; ++i) {
            const LightDev Lt = S.lights[i];
            const int nS = fbits(Lt.p1_ns.w);
            const int ltype = fbits(Lt.o_type.w);
            for (int s = 0; s < nS; ++s) {
                float u1 = 0.f, u2 = 0.f;
                if (ltype == PM_LIGHT_AREA_DISK) {
                    int slot = fbits(Lt.p2_r2d.w) + s;
                    if (P.pinhole) {
                        uint32_t o4[4];
                        pmdm_philox4x32_10((uint32_t)pixel, (uint32_t)slot, 0u, 0u, P.light_seed, 0u, o4);
                        u1 = pmdm_u01(o4[0]); u2 = pmdm_u01(o4[1]);
                    } else {
                        const float *q = P.rand2d + ((size_t)pixel * P.n2d + slot) * 2;
                        u1 = q[0]; u2 = q[1];
                    }
                }
                v3 uwi; float pdf;
                v3 li = sample_l_shading(Lt, point, u1, u2, &uwi, &pdf);
                Ray sr;
                sr.o = point; sr.d = uwi; sr.tmin = 0.001f; sr.tmax = 1.0f - 0.001f;
                Hit sh;
                float atten = traverse<true, MODE>(S, sr, sh, stack, EYE_BLOCK) ? 0.0f : 1.0f;
                v3 wi = normalize(uwi);
                L = L + (atten * fabsf(dot(ns, wi))) * fv * li / (pdf * nS);
            }
        }
    }
    /* Faceforward(nn, wo) side, for the kNN estimator (the reference keeps
     * record.direction itself, raytracing.cu:117) */
    const uint32_t side = dot(ns, -dir) < 0.f ? PM_REC_BACKFACE : 0u;
    P.R.pos[r] = make_float4(point.x, point.y, point.z, __uint_as_float(side));
    P.R.nrm[r] = make_float4(ns.x, ns.y, ns.z, __int_as_float(g.material));
    P.R.state[r] = make_float4(0.f, 0.f, 0.f, P.r2init);
    P.R.n[r] = 0.f;
    P.R.dl[r] = make_float4(L.x, L.y, L.z, 0.f);
}

hipError_t launch_eye(const EyeParams &p, hipStream_t s) {
    if (p.R.count <= 0) return hipSuccess;
    unsigned grid = (unsigned)((p.R.count + EYE_BLOCK - 1) / EYE_BLOCK);
    const size_t lds = (size_t)p.S.stack_depth * EYE_BLOCK * 4 + p.S.lds_bytes;
    switch (scene_mode(p.S)) {
    case MODE_BRUTE: pm_launch(k_eye<MODE_BRUTE>, dim3(grid), dim3(EYE_BLOCK), lds, s, p); break;
    case MODE_LDS: pm_launch(k_eye<MODE_LDS>, dim3(grid), dim3(EYE_BLOCK), lds, s, p); break;
    case MODE_INST: pm_launch(k_eye<MODE_INST>, dim3(grid), dim3(EYE_BLOCK), lds, s, p); break;
    default: pm_launch(k_eye<MODE_GLOBAL>, dim3(grid), dim3(EYE_BLOCK), lds, s, p); break;
    }
    return hipGetLastError();
}

/* ====================================================================== */
/* simple renderer (direct light only, simple_render/simplerender.cu)     */
/* ====================================================================== */
/* One lane per eye sample: closest hit of the camera ray (no specular
 * chain), then for every light one shadow-tested sample (iSample 0, no pdf
 * division, no emitted term): L += att·|ns·wi|·f·li (simplerender.cu:40-72);
 * a miss is black (:75-79). The host's NaN / negative / infinite check
 * (simplerender.cpp:70-87) is fused into the store. Output: raster order
 * (pinhole) or sample order (host rays), float3 per sample. */
template <int MODE>
__global__ __launch_bounds__(EYE_BLOCK) void k_simple(EyeParams P, float *out) {
    extern __shared__ __attribute__((aligned(16))) int stk[];
    int *stack = stk + threadIdx.x;
    const SceneDev S = scene_view<mode_lds(MODE)>(P.S, reinterpret_cast<uint4 *>(stk + P.S.stack_depth * EYE_BLOCK),
                                                       threadIdx.x, EYE_BLOCK);
    if (mode_lds(MODE)) __syncthreads();
    const int64_t r = (int64_t)blockIdx.x * EYE_BLOCK + threadIdx.x;
    if (r >= P.R.count) return;

    Ray ray;
    int64_t pixel;
    if (P.pinhole) {
        int px, py;
        rec_to_pixel(r, P.W, &px, &py);
        if (px >= P.W || py >= P.H) return;
        pixel = (int64_t)py * P.W + px;
        float sx = (2.0f * ((float)px + 0.5f)) / (float)P.W - 1.0f;
        float sy = 1.0f - (2.0f * ((float)py + 0.5f)) / (float)P.H;
        v3 d = xyz(P.fwd) + sx * xyz(P.right) + sy * xyz(P.up);
        ray.o = xyz(P.eye);
        ray.d = normalize(d);
    } else {
        pixel = r;
        const float *q = P.rays + 6 * r;
        ray.o = mk(q[0], q[1], q[2]);
        ray.d = mk(q[3], q[4], q[5]);
    }
    ray.tmin = P.eps;
    ray.tmax = RT_DEFAULT_MAX;

    v3 L = mk(0.f, 0.f, 0.f);
    Hit h;
    if (traverse<false, MODE>(S, ray, h, stack, EYE_BLOCK)) {
        const Geo g = shade<MODE == MODE_INST>(S, ray, h);
        const v3 point = ray.o + ray.d * h.t;
        const float4 m = S.materials[g.material];
        const v3 fv = fbits(m.w) == PM_MATTE ? xyz(m) * INV_PI : mk(0.f, 0.f, 0.f); /* f(wo, wi) */
        for (int i = 0; i < S.n_lights; ++i) {
            const LightDev Lt = S.lights[i];
            float u1 = 0.f, u2 = 0.f;
            if (fbits(Lt.o_type.w) == PM_LIGHT_AREA_DISK) {
                const int slot = fbits(Lt.p2_r2d.w); /* random2DStart + iSample 0 */
                if (P.pinhole) {
                    uint32_t o4[4];
                    pmdm_philox4x32_10((uint32_t)pixel, (uint32_t)slot, 0u, 0u, P.light_seed, 0u, o4);
                    u1 = pmdm_u01(o4[0]); u2 = pmdm_u01(o4[1]);
                } else {
                    const float *q = P.rand2d + ((size_t)pixel * P.n2d + slot) * 2;
                    u1 = q[0]; u2 = q[1];
                }
            }
            v3 uwi; float pdf;
            const v3 li = sample_l_shading(Lt, point, u1, u2, &uwi, &pdf);
            Ray sr;
            sr.o = point; sr.d = uwi; sr.tmin = 0.001f; sr.tmax = 1.0f - 0.001f;
            Hit sh;
            const float atten = traverse<true, MODE>(S, sr, sh, stack, EYE_BLOCK) ? 0.0f : 1.0f;
            const v3 wi = normalize(uwi);
            L = L + (atten * fabsf(dot(g.ns, wi))) * fv * li;
        }
    }
    const float y = 0.212671f * L.x + 0.715160f * L.y + 0.072169f * L.z; /* pbrt RGBSpectrum::y */
    if (isnan(L.x) || isnan(L.y) || isnan(L.z) || y < -1e-5f || isinf(y)) L = mk(0.f, 0.f, 0.f);
    out[3 * pixel + 0] = L.x;
    out[3 * pixel + 1] = L.y;
    out[3 * pixel + 2] = L.z;
}

hipError_t launch_simple(const EyeParams &p, float *out, hipStream_t s) {
    if (p.R.count <= 0) return hipSuccess;
    unsigned grid = (unsigned)((p.R.count + EYE_BLOCK - 1) / EYE_BLOCK);
    const size_t lds = (size_t)p.S.stack_depth * EYE_BLOCK * 4 + p.S.lds_bytes;
    switch (scene_mode(p.S)) {
    case MODE_BRUTE: pm_launch(k_simple<MODE_BRUTE>, dim3(grid), dim3(EYE_BLOCK), lds, s, p, out); break;
    case MODE_LDS: pm_launch(k_simple<MODE_LDS>, dim3(grid), dim3(EYE_BLOCK), lds, s, p, out); break;
    case MODE_INST: pm_launch(k_simple<MODE_INST>, dim3(grid), dim3(EYE_BLOCK), lds, s, p, out); break;
    default: pm_launch(k_simple<MODE_GLOBAL>, dim3(grid), dim3(EYE_BLOCK), lds, s, p, out); break;
    }
    return hipGetLastError();
}

/* ====================================================================== */
/* photon pass                                                            */
/* ====================================================================== */
PMD void store_photon(pm_photon *dst, v3 p, v3 a, v3 wi) {
    /* 40-B slot, 8-B aligned: five 8-byte stores */
    float2 *q = reinterpret_cast<float2 *>(dst);
    q[0] = make_float2(__int_as_float(1), p.x);
    q[1] = make_float2(p.y, p.z);
    q[2] = make_float2(a.x, a.y);
    q[3] = make_float2(a.z, wi.x);
    q[4] = make_float2(wi.y, wi.z);
}

/* Photon paths (photontracing.cu:80-185) split into ray steps so a block can
 * compact its live paths between steps. Per-path state (12 words) lives in
 * registers and moves through LDS only at compaction. */
struct PathState {
    Ray ray;         /* tmax is RT_DEFAULT_MAX at every step */
    v3 alpha;
    uint32_t pid;    /* global path id */
    uint32_t nI;     /* photons-in-path counter (reference nI) */
    uint32_t spec;   /* specular bounces so far */
    uint32_t stored; /* slots [0, stored) written */
    /* fused counting: the bucket rank of the last deposit is stored one deposit
     * later (or when the path ends), so the wave never waits for the returning
     * atomic right after issuing it */
    uint32_t pslot;  /* slot of the pending rank, PSLOT_NONE if none */
    uint32_t prank;
};
constexpr uint32_t PSLOT_NONE = 0xffffffffu;
/* where the fused bucket count keeps deposit k of path pid: plane-major
 * (k * key_np + path) when key_np > 0, so that the lanes of a wave — paths
 * next to each other — store their keys and ranks into the same lines
 * instead of one 4-B store per 16-B path block; else the slot index */
PMD size_t key_index(const TraceParams &P, uint32_t pid, uint32_t k) {
    const size_t path = (size_t)(pid - (uint64_t)P.slot_path_base);
    return P.key_np > 0 ? (size_t)k * (size_t)P.key_np + path : path * (size_t)P.mpc + k;
}
PMD void flush_rank(const TraceParams &P, PathState &st) {
    if (st.pslot != PSLOT_NONE) { P.rank[st.pslot] = st.prank; st.pslot = PSLOT_NONE; }
}

/* HOLD kernels (k_trace_lane, k_trace_pool when max_photon_count is 4): a
 * path's first three deposits wait in LDS until the path ends, then its
 * 160-B slot block is written with 16-B stores, with its four bucket keys
 * and ranks as one 16-B store each (the fourth deposit ends the path, so it
 * is stored at once, next to the block's other writes). Writing each deposit
 * as it happens (photontracing.cu:141-151's owner-writes) stored five 8-B
 * pieces at a 160-B lane stride at different times, so L2 wrote partial lines
 * back several times (PMC: 2.2x the slot + key + rank bytes at C2, 2.9x at
 * C3). Registers were not an option: holding 36 words cost ~90 VGPRs in
 * the brute-force trace (4 -> 3 waves/SIMD). LDS: HOLD_WORDS x TRACE_BLOCK
 * words after the stacks and the scene blob, a column per thread. */
constexpr int HOLD_MPC = 4;
constexpr int HOLD_WORDS = 27; /* slots 0..2: p, alpha, wi */
struct Held {
    uint32_t *col;    /* this thread's LDS column: word i at col[i * TRACE_BLOCK] */
    uint4 key, rank;  /* shift registers, .x the newest deposit's */
};
PMD void held_clear(Held &h) { (void)h; } /* deposits beyond the path's count are never read */
PMD void held_put(Held &h, const TraceParams &P, size_t slot, uint32_t k, v3 p, v3 a, v3 wi, uint32_t key,
                  uint32_t rank) {
    if (k < 3u) {
        uint32_t *c = h.col + 9u * k * TRACE_BLOCK;
        c[0 * TRACE_BLOCK] = __float_as_uint(p.x); c[1 * TRACE_BLOCK] = __float_as_uint(p.y);
        c[2 * TRACE_BLOCK] = __float_as_uint(p.z); c[3 * TRACE_BLOCK] = __float_as_uint(a.x);
        c[4 * TRACE_BLOCK] = __float_as_uint(a.y); c[5 * TRACE_BLOCK] = __float_as_uint(a.z);
        c[6 * TRACE_BLOCK] = __float_as_uint(wi.x); c[7 * TRACE_BLOCK] = __float_as_uint(wi.y);
        c[8 * TRACE_BLOCK] = __float_as_uint(wi.z);
    } else {
        store_photon(P.slots + slot, p, a, wi); /* the last deposit: the block is written right after */
    }
    h.key = make_uint4(key, h.key.x, h.key.y, h.key.z);
    h.rank = make_uint4(rank, h.rank.x, h.rank.y, h.rank.z);
}
/* the path's slot block (16-B aligned: 160 B per path from a 16-B aligned
 * buffer, launch_trace checks): slots 0..2 from LDS (zero past the n
 * deposits), slot 3 zero unless its deposit was stored; with fused counting
 * the key and rank quads (key 0xffffffff past n) */
PMD void held_write(const TraceParams &P, uint32_t pid, const Held &h, uint32_t n) {
    const size_t path = (size_t)(pid - (uint64_t)P.slot_path_base);
    uint32_t w[HOLD_WORDS];
#pragma unroll
    for (int i = 0; i < HOLD_WORDS; ++i) w[i] = (uint32_t)(i / 9) < n ? h.col[i * TRACE_BLOCK] : 0u;
    const uint32_t va = n > 0u, vb = n > 1u, vc = n > 2u;
    uint4 *dst = reinterpret_cast<uint4 *>(P.slots + path * HOLD_MPC);
    dst[0] = make_uint4(va, w[0], w[1], w[2]);
    dst[1] = make_uint4(w[3], w[4], w[5], w[6]);
    dst[2] = make_uint4(w[7], w[8], vb, w[9]);
    dst[3] = make_uint4(w[10], w[11], w[12], w[13]);
    dst[4] = make_uint4(w[14], w[15], w[16], w[17]);
    dst[5] = make_uint4(vc, w[18], w[19], w[20]);
    dst[6] = make_uint4(w[21], w[22], w[23], w[24]);
    if (n > 3u) {
        reinterpret_cast<uint2 *>(dst + 7)[0] = make_uint2(w[25], w[26]); /* slot 3 already stored */
    } else {
        dst[7] = make_uint4(w[25], w[26], 0u, 0u);
        dst[8] = make_uint4(0u, 0u, 0u, 0u);
        dst[9] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (P.bucket) {
        /* slot j = push n - 1 - j (wraps for j >= n: invalid) */
        const uint32_t q0 = n - 1u, q1 = n - 2u, q2 = n - 3u, q3 = n - 4u;
#define PICKQ(V, Q, DEF) ((Q) == 0u ? V.x : (Q) == 1u ? V.y : (Q) == 2u ? V.z : (Q) == 3u ? V.w : (DEF))
        reinterpret_cast<uint4 *>(P.key)[path] = make_uint4(PICKQ(h.key, q0, 0xffffffffu), PICKQ(h.key, q1, 0xffffffffu),
                                                            PICKQ(h.key, q2, 0xffffffffu), PICKQ(h.key, q3, 0xffffffffu));
        reinterpret_cast<uint4 *>(P.rank)[path] = make_uint4(PICKQ(h.rank, q0, 0u), PICKQ(h.rank, q1, 0u),
                                                             PICKQ(h.rank, q2, 0u), PICKQ(h.rank, q3, 0u));
#undef PICKQ
    }
}

/* Phase profile of k_trace (profiling builds only: `make prof` ->
 * lib/libpmhip_prof.so): per-wave s_memtime cycles accumulated per phase,
 * summed over waves into TraceParams::prof (pm_trace_profile). */
struct TProf {
#ifdef PM_TRACE_PROFILE
    uint64_t last = 0, start = 0, acc[6] = {0, 0, 0, 0, 0, 0};
    PMD void begin() { start = last = __builtin_amdgcn_s_memtime(); }
    PMD void mark(int i) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        acc[i] += t - last;
        last = t;
    }
    PMD void flush(unsigned long long *out) {
        if (!out || (threadIdx.x & 63) != 0) return;
        for (int i = 0; i < 6; ++i) atomicAdd(&out[i], (unsigned long long)acc[i]);
        atomicAdd(&out[6], (unsigned long long)(last - start));
        atomicAdd(&out[7], 1ull);
    }
#else
    PMD void begin() {}
    PMD void mark(int) {}
    PMD void flush(unsigned long long *) {}
#endif
};

/* emission: Halton light sample -> first ray (photontracing.cu:88-117) */
PMD bool emit_path(const TraceParams &P, const SceneDev &S, const uint32_t *perm, uint32_t pid, PathState &st) {
    const uint32_t pm_index = pid * (uint32_t)P.mpc;
    float smp[4];
    permuted_halton4(pm_index, perm, P.perm_bits, smp);
    const LightDev Lt = S.lights[P.light_index];
    v3 N1; float pdf;
    v3 Le = sample_le(Lt, smp[0], smp[1], smp[2], smp[3], P.eps, &st.ray, &N1, &pdf);
    st.pid = pid; st.nI = 0; st.spec = 0; st.stored = 0; st.pslot = PSLOT_NONE;
    if (pdf == 0.0f || is_black(Le)) return false;
    st.ray.tmax = RT_DEFAULT_MAX;
    st.alpha = (absdot(N1, st.ray.d) * Le) / pdf;
    return true;
}

/* one ray of a path: trace, then specular continuation or diffuse deposit +
 * Lambert bounce (photontracing.cu:119-183); false when the path ends */
template <int HOLD, bool INST = false>
PMD bool path_shade(const TraceParams &P, const SceneDev &S, PathState &st, const Hit &h, TProf &prof, Held &held);

template <int MODE, int HOLD, class C>
PMD bool path_step(const TraceParams &P, const SceneDev &S, int *stack, PathState &st, C &cen, TProf &prof,
                   Held &held) {
    Hit h;
    const bool hit = traverse<false, MODE>(S, st.ray, h, stack, TRACE_BLOCK, cen);
    prof.mark(1);
    if (!hit) return false;
    return path_shade<HOLD, MODE == MODE_INST>(P, S, st, h, prof, held);
}

/* the hit of a path's ray: specular continuation, or diffuse deposit +
 * Lambert bounce (photontracing.cu:119-183); false when the path ends.
 * HOLD: the deposit goes to `held` (written at path end, held_write) */
template <int HOLD, bool INST>
PMD bool path_shade(const TraceParams &P, const SceneDev &S, PathState &st, const Hit &h, TProf &prof, Held &held) {
    const uint32_t mpc = (uint32_t)P.mpc;
    Geo g = shade<INST>(S, st.ray, h);
    v3 hit_point = st.ray.o + h.t * st.ray.d;
    float4 m = S.materials[g.material];
    int mtype = fbits(m.w);
    prof.mark(3);
    if (is_specular(mtype)) {
        v3 wi;
        if (!material_specular(mtype, g, -st.ray.d, &wi)) return false;
        if ((int)++st.spec > P.max_spec) return false;
        if (st.nI == 0) st.nI++;
        st.ray.o = hit_point; st.ray.d = wi; st.ray.tmin = P.eps; st.ray.tmax = RT_DEFAULT_MAX;
        return true;
    }
    v3 wo = -st.ray.d;
    if (st.nI >= 1) {
        const size_t slot = (size_t)(st.pid - (uint64_t)P.slot_path_base) * mpc + (st.nI - 1);
        if (!HOLD) store_photon(P.slots + slot, hit_point, st.alpha, wo);
        st.stored = st.nI;
        uint32_t key = 0xffffffffu, rank = 0u;
        if (P.bucket) { /* fused counting pass of the bucket build (pm_bucket.hip k_bucket_count) */
            const GridDesc &g = P.grid;
            const uint32_t cx = cell_axis(hit_point.x, g.gx, g.inv_cs, g.dx);
            const uint32_t cy = cell_axis(hit_point.y, g.gy, g.inv_cs, g.dy);
            const uint32_t cz = cell_axis(hit_point.z, g.gz, g.inv_cs, g.dz);
            key = (cz * (uint32_t)g.dy + cy) * (uint32_t)g.dx + cx;
            rank = atomicAdd(&P.count[key], 1u);
            if (!HOLD) {
                const size_t ki = key_index(P, st.pid, st.nI - 1);
                P.key[ki] = key;
                flush_rank(P, st);
                st.prank = rank; st.pslot = (uint32_t)ki;
            }
        }
        /* HOLD: the returned rank is first read at the path's end */
        if (HOLD) held_put(held, P, slot, st.nI - 1, hit_point, st.alpha, wo, key, rank);
    }
    prof.mark(4);
    if (st.nI >= mpc) return false;
    const uint32_t pm_index = st.pid * mpc;
    uint32_t o4[4];
    pmdm_philox4x32_10(pm_index + st.nI, (uint32_t)P.pass, 0u, 0u, P.seed, 0u, o4);
    float u1 = pmdm_u01(o4[0]), u2 = pmdm_u01(o4[1]);
    v3 wiw; float bpdf;
    v3 fr = sample_f(xyz(m), g, wo, u1, u2, &wiw, &bpdf);
    if (is_black(fr) || bpdf == 0.f) return false;
    v3 anew = st.alpha * fr * absdot(wiw, g.ns) / bpdf;
    st.alpha = anew;
    st.nI++;
    st.ray.o = hit_point; st.ray.d = wiw; st.ray.tmin = P.eps; st.ray.tmax = RT_DEFAULT_MAX;
    prof.mark(5);
    return true;
}

/* a finished path's unused slots are invalid = zero (the reference leaves
 * them stale, DESIGN.md divergences); written here instead of a memset pass */
template <int HOLD = 0>
PMD void finish_path(const TraceParams &P, PathState &st, const Held *held = nullptr) {
    if (HOLD) { held_write(P, st.pid, *held, st.stored); return; }
    flush_rank(P, st);
    const uint32_t mpc = (uint32_t)P.mpc;
    pm_photon *slots = P.slots + (size_t)(st.pid - (uint64_t)P.slot_path_base) * mpc;
    const float2 z = make_float2(0.f, 0.f);
    for (uint32_t k = st.stored; k < mpc; ++k) {
        float2 *q = reinterpret_cast<float2 *>(slots + k);
        /* lazy_zero (fused counting, env PM_LAZY_ZERO=1; off by default):
         * the invalid key alone marks the slot; the bucket fill never reads
         * it, and pm_api zeroes it before any other reader. 20-50 MB fewer
         * trace stores per pass, but no faster C2 trace on a same-box A/B and
         * a slower C4 bucket fill (46.5 -> 69 us; profiles/r05/trace_writes) */
        if (!P.lazy_zero) { q[0] = z; q[1] = z; q[2] = z; q[3] = z; q[4] = z; }
        if (P.bucket) P.key[key_index(P, st.pid, k)] = 0xffffffffu;
    }
}

/* Per-lane photon tracer: one path per lane, no block barriers; a wave lives
 * as long as its longest path (C2: one occupancy round of 4,096 waves, 3.46
 * rays per path on average). Pools of several paths per lane, refilled as
 * lanes finish, and a block-compacting variant were measured slower (DESIGN.md
 * §5) and removed. HOLD: deposits held in LDS and written per path.
 * COUNT: census [rays traced, BVH nodes entered, primitive tests, photons
 * deposited], one atomic per wave (counting launches only, never timed). */
template <int COUNT, int MODE, int HOLD>
__global__ __launch_bounds__(TRACE_BLOCK) void k_trace_lane(TraceParams P) {
    extern __shared__ __attribute__((aligned(16))) int stk[];
    __shared__ uint32_t perm[28];
    const int tid = threadIdx.x;
    if (tid < 28) perm[tid] = P.perm[tid];
    const SceneDev S = scene_view<mode_lds(MODE)>(P.S, reinterpret_cast<uint4 *>(stk + P.S.stack_depth * TRACE_BLOCK),
                                                       tid, TRACE_BLOCK);
    __syncthreads();
    int *stack = stk + tid;
    typename std::conditional<COUNT != 0, Census, NoCensus>::type cen;
    TProf prof;
    uint32_t rays = 0, deposits = 0;
    const int64_t path = (int64_t)blockIdx.x * TRACE_BLOCK + tid;
    PathState st;
    Held held;
    if (HOLD) /* after the stacks and the (16-B padded) scene blob */
        held.col = reinterpret_cast<uint32_t *>(stk + P.S.stack_depth * TRACE_BLOCK + (mode_lds(MODE) ? (int)((P.S.lds_bytes + 15u) / 4u & ~3u) : 0)) + tid;
    prof.begin();
    if (path < P.path_count) {
        if (HOLD) held_clear(held);
        bool alive = emit_path(P, S, perm, (uint32_t)(P.path_begin + path), st);
        prof.mark(0);
        while (alive) {
            ++rays;
            alive = path_step<MODE, HOLD>(P, S, stack, st, cen, prof, held);
            prof.mark(2);
        }
        if (COUNT) deposits += st.stored;
        finish_path<HOLD>(P, st, &held);
    }
    prof.flush(P.prof);
    if (COUNT) {
        uint32_t nodes = 0, prims = 0;
        if constexpr (COUNT != 0) { nodes = cen.nodes; prims = cen.prims; }
        count4(P.counters, rays, nodes, prims, deposits);
    }
}

/* Pooled photon tracer for scenes traversed from HBM with the 4-wide BVH
 * (C3). A ray's traversal lives across iterations of the wave's loop
 * (TravState: node, stack in LDS, pending leaves, best hit), so lanes whose
 * ray ended do not idle until the wave's longest ray ends: they wait until
 * at least POOL_SHADE_MIN lanes are ready (or nothing traverses), then those
 * lanes shade their hits together (deposit / bounce -> next ray) and lanes
 * without a path take the next ones of the wave's pool [wbegin, wend). The
 * rest of the time every iteration runs POOL_STEPS traversal steps for the
 * traversing lanes. Paths, slots and bucket counts are the per-lane
 * kernel's (owner-writes; the fused bucket ranks' order is immaterial). */
#ifndef PM_POOL_SHADE_MIN
#define PM_POOL_SHADE_MIN 16
#endif
#ifndef PM_POOL_STEPS
#define PM_POOL_STEPS 4
#endif
constexpr int POOL_STEPS = PM_POOL_STEPS, POOL_SHADE_MIN = PM_POOL_SHADE_MIN;
enum { PHASE_DEAD = 0, PHASE_TRAV = 1, PHASE_SHADE = 2 };

/* W8: the 8-wide tree (S.wide == 3, TravState8) */
template <int COUNT, int HOLD, int W8>
/* 5 waves/SIMD: 96 VGPRs (102 unconstrained -> 4 waves), no scratch; with
 * the LDS stacks capped at 31 entries (PM_POOL_STACK, the rest spilled) five
 * 256-thread blocks fit a CU. C3 trace (same box): 4.59-4.61 ms at 4 waves,
 * 4.41-4.42 ms at 5 (stack 31 or 24); 6 (80 VGPRs, 100 B of scratch) 4.58 */
#ifndef PM_POOL_EU
#define PM_POOL_EU 5
#endif
#if PM_POOL_EU > 0
#define POOL_OCC __attribute__((amdgpu_waves_per_eu(PM_POOL_EU, PM_POOL_EU)))
#else
#define POOL_OCC
#endif
/* the 8-wide walk needs 117 VGPRs unconstrained: 4 waves/SIMD (113, no
 * scratch) by default; 5 spills 88 B */
#ifndef PM_POOL8_EU
#define PM_POOL8_EU 4
#endif
__device__ __forceinline__ void trace_pool_body(TraceParams P) { /* ~102 VGPRs without SLP: 4 waves/SIMD */
    extern __shared__ __attribute__((aligned(16))) int stk[];
    __shared__ uint32_t perm[28];
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < 28) perm[tid] = P.perm[tid];
    const SceneDev &S = P.S;
    __syncthreads();
    int *stack = stk + tid;
    /* LDS stack entries per lane (P.pool_stack, else the tree's bound); deeper ones spill to global memory */
    const int lstk = P.pool_stack > 0 && P.pool_stack < P.S.stack_depth ? P.pool_stack : P.S.stack_depth;
    const SpillStack sstk{stack, TRACE_BLOCK, lstk, P.spill, P.spill_stride, (uint32_t)(blockIdx.x * TRACE_BLOCK + tid)};
    typename std::conditional<COUNT != 0, Census, NoCensus>::type cen;
    TProf prof;
    uint32_t rays = 0, deposits = 0;
    const int64_t wave_id = ((int64_t)blockIdx.x * TRACE_BLOCK + tid) >> 6;
    const int64_t wbegin = wave_id * P.pool_paths;
    const int64_t wend = wbegin + P.pool_paths < P.path_count ? wbegin + P.pool_paths : P.path_count;
    int64_t cursor = wbegin; /* wave-uniform: next unassigned path of the pool */
    PathState st;
    typename std::conditional<W8 != 0, TravState8, TravState>::type tr;
    Held held;
    if (HOLD) held.col = reinterpret_cast<uint32_t *>(stk + lstk * TRACE_BLOCK) + tid; /* after the stacks */
    int phase = PHASE_DEAD;
    while (true) {
        const unsigned long long travm = __ballot(phase == PHASE_TRAV);
        const unsigned long long shadem = __ballot(phase == PHASE_SHADE);
        const unsigned long long deadm = __ballot(phase == PHASE_DEAD);
        const bool pool_left = cursor < wend;
        if (travm == 0ull && shadem == 0ull && !pool_left) break; /* every lane reaches it together */
        const int waiting = __popcll(shadem) + (pool_left ? __popcll(deadm) : 0);
        if (travm == 0ull || waiting >= POOL_SHADE_MIN) {
            if (phase == PHASE_SHADE) {
                ++rays;
                const bool alive = tr.best.ref != 0xffffffffu && path_shade<HOLD>(P, S, st, tr.best, prof, held);
                if (alive) {
                    trav_begin(st.ray, tr);
                    phase = PHASE_TRAV;
                } else {
                    if (COUNT) deposits += st.stored;
                    finish_path<HOLD>(P, st, &held);
                    phase = PHASE_DEAD;
                }
            }
            const unsigned long long dm = __ballot(phase == PHASE_DEAD);
            if (cursor < wend) {
                const int64_t mine = cursor + __popcll(dm & ((1ull << lane) - 1ull));
                if (phase == PHASE_DEAD && mine < wend) {
                    if (HOLD) held_clear(held);
                    if (emit_path(P, S, perm, (uint32_t)(P.path_begin + mine), st)) {
                        trav_begin(st.ray, tr);
                        phase = PHASE_TRAV;
                    } else {
                        finish_path<HOLD>(P, st, &held);
                    }
                }
                cursor = cursor + __popcll(dm) < wend ? cursor + __popcll(dm) : wend;
            }
            continue;
        }
#pragma unroll 1
        for (int k = 0; k < POOL_STEPS; ++k)
            if (phase == PHASE_TRAV && !trav_step(S, st.ray, tr, sstk, cen)) phase = PHASE_SHADE;
    }
    if (COUNT) {
        uint32_t nodes = 0, prims = 0;
        if constexpr (COUNT != 0) { nodes = cen.nodes; prims = cen.prims; }
        count4(P.counters, rays, nodes, prims, deposits);
    }
}

template <int COUNT, int HOLD>
__global__ __launch_bounds__(TRACE_BLOCK) POOL_OCC void k_trace_pool(TraceParams P) { trace_pool_body<COUNT, HOLD, 0>(P); }
template <int COUNT, int HOLD>
__global__ __launch_bounds__(TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(PM_POOL8_EU, PM_POOL8_EU)))
void k_trace_pool8(TraceParams P) { trace_pool_body<COUNT, HOLD, 1>(P); }

/* resident waves of the pooled kernel per CU at this LDS size (0 if unknown) */
int trace_pool_waves_per_cu(size_t lds, int hold, int w8) { /* lds: the stacks */
    int blocks = 0;
    if (hold) lds += (size_t)HOLD_WORDS * TRACE_BLOCK * 4;
    const hipError_t e =
        w8 ? (hold ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_pool8<0, 1>, TRACE_BLOCK, lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_pool8<0, 0>, TRACE_BLOCK, lds))
           : (hold ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_pool<0, 1>, TRACE_BLOCK, lds)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_pool<0, 0>, TRACE_BLOCK, lds));
    if (e != hipSuccess) return 0;
    return blocks * (TRACE_BLOCK / 64);
}

/* resident waves per CU of the per-lane kernel (scene mode of S) with or
 * without the held deposits' LDS: the host keeps HOLD only when it costs no
 * waves (C2: one occupancy round of 4,096 waves) */
int trace_lane_waves_per_cu(const SceneDev &S, size_t lds, int hold) {
    int blocks = 0;
    hipError_t e;
    if (hold) {
        lds += ((size_t)S.lds_bytes + 15u) / 16u * 16u - S.lds_bytes + (size_t)HOLD_WORDS * TRACE_BLOCK * 4;
        switch (scene_mode(S)) {
        case MODE_BRUTE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_BRUTE, 1>, TRACE_BLOCK, lds); break;
        case MODE_LDS: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_LDS, 1>, TRACE_BLOCK, lds); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_GLOBAL, 1>, TRACE_BLOCK, lds); break;
        }
    } else {
        switch (scene_mode(S)) {
        case MODE_BRUTE: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_BRUTE, 0>, TRACE_BLOCK, lds); break;
        case MODE_LDS: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_LDS, 0>, TRACE_BLOCK, lds); break;
        default: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, k_trace_lane<0, MODE_GLOBAL, 0>, TRACE_BLOCK, lds); break;
        }
    }
    return e == hipSuccess ? blocks * (TRACE_BLOCK / 64) : 0;
}

/* deposits held in registers and written per path (Held): the reference's
 * 4 photons per path, a 16-B aligned slot buffer; env PM_TRACE_HOLD=0 (read
 * by pm_api.cpp into TraceParams::hold) keeps the per-deposit stores */
static bool trace_hold(const TraceParams &p) {
    return p.hold && p.mpc == HOLD_MPC && ((uintptr_t)p.slots & 15u) == 0u;
}

template <int HOLD>
static void launch_lane(const TraceParams &p, dim3 grid, size_t lds, int count, hipStream_t s) {
    switch (scene_mode(p.S)) {
    case MODE_BRUTE:
        if (count) pm_launch((k_trace_lane<1, MODE_BRUTE, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        else pm_launch((k_trace_lane<0, MODE_BRUTE, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        break;
    case MODE_LDS:
        if (count) pm_launch((k_trace_lane<1, MODE_LDS, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        else pm_launch((k_trace_lane<0, MODE_LDS, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        break;
    case MODE_INST: /* instances: the per-lane kernel (the pooled one walks only one level) */
        if (count) pm_launch((k_trace_lane<1, MODE_INST, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        else pm_launch((k_trace_lane<0, MODE_INST, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        break;
    default:
        if (count) pm_launch((k_trace_lane<1, MODE_GLOBAL, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        else pm_launch((k_trace_lane<0, MODE_GLOBAL, HOLD>), grid, dim3(TRACE_BLOCK), lds, s, p);
        break;
    }
}

hipError_t launch_trace(const TraceParams &p, int count, hipStream_t s) {
    if (p.path_count <= 0) return hipSuccess;
    if (p.pool_paths > 0 && scene_mode(p.S) == MODE_GLOBAL && p.S.wide) {
        const int lstk = p.pool_stack > 0 && p.pool_stack < p.S.stack_depth ? p.pool_stack : p.S.stack_depth;
        if (lstk < p.S.stack_depth && !p.spill) return hipErrorInvalidValue;
        const size_t lds = (size_t)lstk * TRACE_BLOCK * 4;
        const int64_t waves = (p.path_count + p.pool_paths - 1) / p.pool_paths;
        const unsigned grid = (unsigned)((waves + TRACE_BLOCK / 64 - 1) / (TRACE_BLOCK / 64));
        const bool hold = trace_hold(p);
        const size_t lds_h = lds + (hold ? (size_t)HOLD_WORDS * TRACE_BLOCK * 4 : 0);
        if (p.S.wide == 3) {
            if (count && hold) pm_launch((k_trace_pool8<1, 1>), dim3(grid), dim3(TRACE_BLOCK), lds_h, s, p);
            else if (count) pm_launch((k_trace_pool8<1, 0>), dim3(grid), dim3(TRACE_BLOCK), lds, s, p);
            else if (hold) pm_launch((k_trace_pool8<0, 1>), dim3(grid), dim3(TRACE_BLOCK), lds_h, s, p);
            else pm_launch((k_trace_pool8<0, 0>), dim3(grid), dim3(TRACE_BLOCK), lds, s, p);
        } else if (count && hold) pm_launch((k_trace_pool<1, 1>), dim3(grid), dim3(TRACE_BLOCK), lds_h, s, p);
        else if (count) pm_launch((k_trace_pool<1, 0>), dim3(grid), dim3(TRACE_BLOCK), lds, s, p);
        else if (hold) pm_launch((k_trace_pool<0, 1>), dim3(grid), dim3(TRACE_BLOCK), lds_h, s, p);
        else pm_launch((k_trace_pool<0, 0>), dim3(grid), dim3(TRACE_BLOCK), lds, s, p);
        return hipGetLastError();
    }
    /* one path per lane */
    const size_t lds = (size_t)p.S.stack_depth * TRACE_BLOCK * 4 + p.S.lds_bytes;
    const unsigned grid = (unsigned)((p.path_count + TRACE_BLOCK - 1) / TRACE_BLOCK);
    if (trace_hold(p))
        launch_lane<1>(p, dim3(grid), lds + ((size_t)p.S.lds_bytes + 15u) / 16u * 16u - p.S.lds_bytes +
                                          (size_t)HOLD_WORDS * TRACE_BLOCK * 4, count, s);
    else launch_lane<0>(p, dim3(grid), lds, count, s);
    return hipGetLastError();
}

} // namespace pm
