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

#include "pm_kernels.h"

#pragma clang fp contract(off)

namespace pm {

/* ====================================================================== */
/* eye pass                                                               */
/* ====================================================================== */
__global__ __launch_bounds__(EYE_BLOCK) void k_eye(EyeParams P) {
    extern __shared__ int stk[]; /* stack_depth x EYE_BLOCK */
    int *stack = stk + threadIdx.x;
    const int64_t r = (int64_t)blockIdx.x * EYE_BLOCK + threadIdx.x;
    if (r >= P.R.count) return;
    const SceneDev &S = P.S;

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
        if (!traverse<false>(S, ray, h, stack, EYE_BLOCK)) { flags = PM_REC_MISS; break; }
        g = shade(S, ray, h);
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
                float atten = traverse<true>(S, sr, sh, stack, EYE_BLOCK) ? 0.0f : 1.0f;
                v3 wi = normalize(uwi);
                L = L + (atten * fabsf(dot(ns, wi))) * fv * li / (pdf * nS);
            }
        }
    }
    P.R.pos[r] = make_float4(point.x, point.y, point.z, __int_as_float(0));
    P.R.nrm[r] = make_float4(ns.x, ns.y, ns.z, __int_as_float(g.material));
    P.R.state[r] = make_float4(0.f, 0.f, 0.f, P.r2init);
    P.R.n[r] = 0.f;
    P.R.dl[r] = make_float4(L.x, L.y, L.z, 0.f);
}

hipError_t launch_eye(const EyeParams &p, hipStream_t s) {
    if (p.R.count <= 0) return hipSuccess;
    unsigned grid = (unsigned)((p.R.count + EYE_BLOCK - 1) / EYE_BLOCK);
    hipLaunchKernelGGL(k_eye, dim3(grid), dim3(EYE_BLOCK), (size_t)p.S.stack_depth * EYE_BLOCK * 4, s, p);
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

__global__ __launch_bounds__(TRACE_BLOCK) void k_trace(TraceParams P) {
    extern __shared__ int stk[]; /* stack_depth x TRACE_BLOCK */
    __shared__ uint32_t perm[28];
    if (threadIdx.x < 28) perm[threadIdx.x] = P.perm[threadIdx.x];
    __syncthreads();
    int *stack = stk + threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * TRACE_BLOCK + threadIdx.x;
    if (i >= P.path_count) return;
    const SceneDev &S = P.S;
    const uint64_t path = (uint64_t)(P.path_begin + i);
    const uint32_t mpc = (uint32_t)P.mpc;
    pm_photon *slots = P.slots + (size_t)(path - (uint64_t)P.slot_path_base) * mpc;
    const uint32_t pm_index = (uint32_t)(path * mpc);

    float smp[4];
    {
        const uint32_t b[4] = {2, 3, 5, 7};
        const uint32_t off[4] = {0, 2, 5, 10};
#pragma unroll
        for (int k = 0; k < 4; ++k) smp[k] = permuted_radical_inverse(pm_index, b[k], perm + off[k]);
    }
    const LightDev Lt = S.lights[P.light_index];
    Ray ray; v3 N1; float pdf;
    v3 Le = sample_le(Lt, smp[0], smp[1], smp[2], smp[3], P.eps, &ray, &N1, &pdf);
    if (pdf == 0.0f || is_black(Le)) return;
    ray.tmax = RT_DEFAULT_MAX;
    v3 alpha = (absdot(N1, ray.d) * Le) / pdf;
    uint32_t nI = 0;
    int spec = 0;
    Hit h;
    while (true) {
        if (!traverse<false>(S, ray, h, stack, TRACE_BLOCK)) return;
        Geo g = shade(S, ray, h);
        v3 hit_point = ray.o + h.t * ray.d;
        float4 m = S.materials[g.material];
        int mtype = fbits(m.w);
        if (is_specular(mtype)) {
            v3 wi;
            if (!material_specular(mtype, g, -ray.d, &wi)) return;
            if (++spec > P.max_spec) return;
            if (nI == 0) nI++;
            ray.o = hit_point; ray.d = wi; ray.tmin = P.eps; ray.tmax = RT_DEFAULT_MAX;
            continue;
        }
        v3 wo = -ray.d;
        if (nI >= 1) store_photon(slots + (nI - 1), hit_point, alpha, wo);
        if (nI >= mpc) return;
        uint32_t o4[4];
        pmdm_philox4x32_10(pm_index + nI, (uint32_t)P.pass, 0u, 0u, P.seed, 0u, o4);
        float u1 = pmdm_u01(o4[0]), u2 = pmdm_u01(o4[1]);
        v3 wiw; float bpdf;
        v3 fr = sample_f(xyz(m), g, wo, u1, u2, &wiw, &bpdf);
        if (is_black(fr) || bpdf == 0.f) return;
        v3 anew = alpha * fr * absdot(wiw, g.ns) / bpdf;
        alpha = anew;
        nI++;
        ray.o = hit_point; ray.d = wiw; ray.tmin = P.eps; ray.tmax = RT_DEFAULT_MAX;
    }
}

hipError_t launch_trace(const TraceParams &p, hipStream_t s) {
    if (p.path_count <= 0) return hipSuccess;
    unsigned grid = (unsigned)((p.path_count + TRACE_BLOCK - 1) / TRACE_BLOCK);
    hipLaunchKernelGGL(k_trace, dim3(grid), dim3(TRACE_BLOCK), (size_t)p.S.stack_depth * TRACE_BLOCK * 4, s, p);
    return hipGetLastError();
}

} // namespace pm
