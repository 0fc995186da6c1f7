/*
 * pm_device.h — device-side building blocks of the MI355X photon mapper:
 * vector math with the reference's (OptiX) rounding semantics, the scene
 * layout in HBM, intersectors, BSDFs, lights and Halton sampling.
 *
 * Numerics contract: compiled with
 * -ffp-contract=off; every expression keeps the operation order of the
 * reference program it restates, so results match the CPU oracle bit for
 * bit. Transcendentals come from include/pm_detmath.h.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pm_api.h"
#include "../../include/pm_detmath.h"

#pragma clang fp contract(off)

#define PMD __device__ __forceinline__

namespace pm {

/* ------------------------------------------------------------------ v3 */
struct v3 { float x, y, z; };
PMD v3 mk(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
PMD v3 operator+(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PMD v3 operator-(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PMD v3 operator-(v3 a) { return mk(-a.x, -a.y, -a.z); }
PMD v3 operator*(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PMD v3 operator*(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PMD v3 operator*(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
/* OptiX float3 / float multiplies by the reciprocal */
/* IEEE correctly rounded 1/x in 3 instructions instead of the ~10 of the
 * scaled division sequence: one FMA Newton step on v_rcp_f32. Checked bit for
 * bit against 1.0f / x for every float with 2^-125 <= |x| < 2^125
 * (tools/rcp_exhaustive.hip: 0 mismatches on gfx950); other inputs (zero,
 * denormal, huge, inf, nan) take the full division. */
PMD float rcp_exact(float x) {
    const float r0 = __builtin_amdgcn_rcpf(x);
    float r = __builtin_fmaf(__builtin_fmaf(-x, r0, 1.0f), r0, r0);
    if (__builtin_expect(((__float_as_uint(x) >> 23) & 0xffu) - 2u > 249u, 0)) r = 1.0f / x;
    return r;
}
PMD v3 operator/(v3 a, float s) { float inv = rcp_exact(s); return a * inv; }
PMD float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PMD v3 cross(v3 a, v3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
PMD v3 normalize(v3 v) { float inv = rcp_exact(sqrtf(dot(v, v))); return v * inv; }
PMD float absdot(v3 a, v3 b) { return fabsf(dot(a, b)); }
PMD bool is_black(v3 s) { return s.x == 0.0f && s.y == 0.0f && s.z == 0.0f; }
PMD v3 xyz(float4 a) { return mk(a.x, a.y, a.z); }
PMD float comp(v3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

constexpr float INV_PI = 0.31830988618379067154f;
constexpr float INV_TWOPI = 0.15915494309189533577f;
constexpr float RT_DEFAULT_MAX = 1.e27f;

/* ---------------------------------------------------------- scene layout */
/* prim ref = (kind << 30) | index */
/* PRIM_INST: an object instance (pm_add_mesh_instance) in the top-level
 * tree; a hit on one of its triangles carries (PRIM_INST << 30) | the
 * object triangle's storage slot, and the triangle's global id */
enum : uint32_t { PRIM_TRI = 0u, PRIM_DISK = 1u, PRIM_SPHERE = 2u, PRIM_INST = 3u };

struct LightDev {      /* CudaLightDevice (common.cu.h:47-59), 80 B */
    float4 o_type;     /* o.xyz, type (int bits) */
    float4 p1_ns;      /* p1.xyz, nSample (int bits) */
    float4 p2_r2d;     /* p2.xyz, random2DStart (int bits) */
    float4 n_area;     /* normal.xyz, area */
    float4 le;         /* intensity.xyz, 0 */
};

struct SceneDev {
    const float4 *nodes;     /* 4 float4 per BVH node */
    const uint32_t *refs;    /* leaf primitive refs */
    const float4 *tri_geo;   /* 3 float4 per triangle: (p0, e0.x) (e0.yz, e1.xy) (e1.z, n) */
    const int4 *tri_info;    /* (v0, v1, v2, mesh) */
    const uint32_t *tri_id;  /* global primitive id (tie-break) */
    /* 2 float4 per triangle, computed on the host with the device's exact
     * IEEE operations (pm_commit): (normalize(n).xyz, material | has_n<<31)
     * (normalize(dpdu).xyz, light). Hit shading is two loads, not ~60 VALU
     * ops + 2 sqrt + 3 divides behind a tri_info -> mesh -> vertex chain. */
    const float4 *tri_shade;
    const float4 *norms;
    const float4 *disks;     /* 5 float4 per disk */
    const float4 *spheres;   /* 4 float4 per sphere */
    const float4 *materials; /* (kd.xyz, type bits) */
    const LightDev *lights;
    int n_lights;
    int n_nodes;
    int stack_depth; /* LDS stack entries per lane (>= BVH depth, <= BVH_STACK_DEPTH) */
    int n_refs;      /* primitives (leaf refs) */
    int n_tris, n_disks, n_spheres;
    int brute;       /* 1: test every primitive wave-uniformly instead of the BVH (tiny LDS scenes) */
    /* HBM copies of tri_geo / tri_id (never rebased to LDS): MODE_BRUTE reads
     * them with wave-uniform indices through the scalar cache into SGPRs */
    const float4 *tri_geo_g;
    const uint32_t *tri_id_g;
    /* brute-force scenes: triangles 2j, 2j + 1 interleaved component by
     * component (24 floats per pair, pm_commit), so each packed operand of
     * isect_tri_pair is one aligned SGPR pair of a scalar load */
    const float *tri_pairs_g;
    /* 4-wide BVH (4 uint4 per quantized node, pm_build.h quantize_bvh4; 8
     * float4 per node in PM_BVH4_QUANT=0 builds, collapse_bvh4) for scenes
     * traversed from HBM (MODE_GLOBAL) when wide != 0; the binary nodes stay
     * for the LDS modes */
    const float4 *wnodes;
    int wide;        /* 4-wide BVH in wnodes: 1 = 128-B float nodes, 2 = 64-B quantized (pm_build.h) */
    /* two-level instancing (pm_add_object_mesh / pm_add_mesh_instance): each
     * object mesh is stored once, in object space, with its own quantized
     * 4-wide tree in wnodes; the top-level tree's instance leaves (PRIM_INST
     * refs) enter it. Per instance 8 float4 (inst_*): the object-to-world
     * rows m[0..11], the world-to-object rows minv[0..11] (pbrt Transform's
     * m and mInv), then (tree root, first object slot, first global id,
     * triangles) and (tree stack bound, 0, 0, 0) as ints. Per object slot:
     * obj_v 3 float4 (object-space p0, p1, p2; p0.w = the triangle's index
     * in its mesh), obj_info (vertex ids into obj_n / obj_uv, mesh). A
     * triangle is intersected and shaded in world space from its vertices
     * transformed exactly as pbrt's Transform does (Transform::operator()),
     * so every hit equals the hit of the instance flattened to world space. */
    const float4 *insts;
    const float4 *obj_v;
    const int4 *obj_info;
    const float4 *obj_n;  /* object vertex normals (xyz) */
    const float4 *obj_uv; /* object vertex uvs (xy) */
    const int4 *obj_mesh; /* per object mesh: material, light, has_n, has_uv */
    int n_inst;
    /* all arrays above are 16-B aligned sections of one blob in HBM */
    const char *blob;
    uint32_t blob_bytes;
    uint32_t lds_bytes; /* = blob_bytes when the blob fits LDS_SCENE_MAX (LDS-resident mode), else 0 */
};

/* Scenes up to this size are copied into each block's LDS and traversed from
 * there (Cornell C2: ~4 KB); larger ones are traversed from HBM/L2. */
constexpr uint32_t LDS_SCENE_MAX = 16384;
/* LDS scenes with at most this many primitives skip the BVH: every lane
 * tests every primitive (MODE_BRUTE) */
constexpr int BRUTE_MAX_PRIMS = 64;

/* how the kernels see the scene (template argument of the traversal kernels) */
enum SceneMode : int { MODE_GLOBAL = 0, MODE_LDS = 1, MODE_BRUTE = 2, MODE_INST = 3 };
/* MODE_INST: a MODE_GLOBAL scene with object instances (two-level 4-wide trees) */
constexpr bool mode_lds(int mode) { return mode == MODE_LDS || mode == MODE_BRUTE; }

struct Ray { v3 o, d; float tmin, tmax; };

constexpr int BVH_STACK_DEPTH = 48; /* LDS stack entries per lane (builder caps depth below it) */

struct Hit {
    uint32_t ref;   /* prim ref of the winner */
    uint32_t gid;   /* global id (tie-break) */
    float t, beta, gamma;
};

PMD int fbits(float f) { return __float_as_int(f); }

/* ------------------------------------------------------------ samplers */
/* util.cu.h:23-65 */
PMD void concentric_sample_disk(float u1, float u2, float *dx, float *dy) {
    float r, theta;
    float sx = 2 * u1 - 1;
    float sy = 2 * u2 - 1;
    if (sx == 0.0f && sy == 0.0f) { *dx = 0.0f; *dy = 0.0f; return; }
    /* the reference's four branches each divide; here the branch only selects
     * (r, numerator, offset) and one IEEE division follows. Bit-identical:
     * c - a/r == c + (-a)/r, and 0 + q == q for the q > 0 of that case. */
    float num, base;
    if (sx >= -sy) {
        if (sx > sy) { r = sx; num = sy; base = (sy > 0.0f) ? 0.0f : 8.0f; }
        else { r = sy; num = -sx; base = 2.0f; }
    } else {
        if (sx <= sy) { r = -sx; num = -sy; base = 4.0f; }
        else { r = -sy; num = sx; base = 6.0f; }
    }
    theta = base + num / r;
    theta = (float)((double)theta * (M_PI / 4.f));
    float st, ct;
    pmdm_sincosf(theta, &st, &ct);
    *dx = r * ct;
    *dy = r * st;
}

/* cudalight.cu.h:66-73 */
PMD v3 uniform_sample_sphere(float u1, float u2) {
    float z = 1.f - 2.f * u1;
    float r = sqrtf(fmaxf(0.f, 1.f - z * z));
    float phi = (float)(2.f * M_PI * (double)u2);
    float sp, cp;
    pmdm_sincosf(phi, &sp, &cp);
    return mk(r * cp, r * sp, z);
}

/* photontracing.cu:19-43 — permutation table in LDS/constant, 28 uints */
PMD float permuted_radical_inverse(uint32_t n, uint32_t base, const uint32_t *p) {
    float val = 0;
    float invBase = 1.f / base, invBi = invBase;
    while (n > 0) {
        uint32_t d_i = p[n % base];
        val += d_i * invBi;
        n = (uint32_t)((float)n * invBase); /* reference quirk: n *= invBase */
        invBi *= invBase;
    }
    return val;
}

/* The four dimensions (bases 2, 3, 5, 7; table offsets 0, 2, 5, 10) of
 * photontracing.cu:33-43, each exactly permuted_radical_inverse:
 *  - base 2 in closed form for n < 2^24: there the quirk n *= 0.5f is an exact
 *    shift, so the digits are the L = bitlength(n) bits of n, and every term
 *    d_i * 2^-(i+1) and partial sum is an exact dyadic fraction (<= 24
 *    significant bits): the loop's float sum equals rev = brev(n) / 2^32
 *    (table (0,1)) or (1 - 2^-L) - rev (table (1,0)) bit for bit;
 *  - bases 3, 5, 7 as three interleaved chains of one loop (independent
 *    digit steps overlap), bounded by base 3, which has the most digits. The
 *    permutation tables come packed, 3 bits per digit (pbits[k] >> 3r & 7:
 *    no LDS load in the digit chain). Below 12,582,912 the quirk's
 *    truncated product equals floor(m / base) for these bases (exhaustive
 *    check over all m < 2^24: first mismatch at 12,582,912 for base 7 and
 *    12,582,914 for base 3), so the digit is m - base * next instead of a
 *    modulo; larger indices (C4/C5) take the modulo. */
template <bool EXACT>
PMD void halton_chains(uint32_t n, const uint32_t pbits[3], float out[3]) {
    const uint32_t base[3] = {3u, 5u, 7u};
    float val[3], invBase[3], invBi[3];
    uint32_t m[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        val[k] = 0.f;
        invBase[k] = 1.f / base[k];
        invBi[k] = invBase[k];
        m[k] = n;
    }
    while ((m[0] | m[1] | m[2]) != 0u) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (m[k] > 0) {
                const uint32_t next = (uint32_t)((float)m[k] * invBase[k]); /* reference quirk: n *= invBase */
                const uint32_t r = EXACT ? m[k] - next * base[k] : m[k] % base[k];
                const uint32_t d_i = (pbits[k] >> (3u * r)) & 7u;
                val[k] += d_i * invBi[k];
                m[k] = next;
                invBi[k] *= invBase[k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) out[k] = val[k];
}
PMD void permuted_halton4(uint32_t n, const uint32_t *p, const uint32_t pbits[3], float out[4]) {
#ifdef PM_EXP_HALTON_CHEAP /* cost experiment only (not bit-exact): make variant */
    for (int k = 0; k < 4; ++k) out[k] = (float)((n * (2654435761u + 2u * k)) >> 8) * (1.0f / 16777216.0f);
    return;
#endif
    if (n < (1u << 24)) {
        const float rev = (float)__builtin_bitreverse32(n) * 0x1p-32f;
        const int L = n ? 32 - __builtin_clz(n) : 0;
        out[0] = p[0] == 0u ? rev : (1.0f - __builtin_ldexpf(1.0f, -L)) - rev;
    } else {
        out[0] = permuted_radical_inverse(n, 2u, p);
    }
    if (n < 12582912u) halton_chains<true>(n, pbits, out + 1);
    else halton_chains<false>(n, pbits, out + 1);
}

/* ------------------------------------------------------------ intersect */
/* OptiX 3 intersect_triangle (cudatrianglemesh.cu:24) on precomputed
 * e0 = p1-p0, e1 = p0-p2, n = e1 x e0 (identical float values). */
PMD bool isect_tri_v(const float4 a, const float4 b, const float4 c, const Ray &ray, float *t, float *beta,
                     float *gamma) {
    v3 p0 = mk(a.x, a.y, a.z), e0 = mk(a.w, b.x, b.y), e1 = mk(b.z, b.w, c.x), n = mk(c.y, c.z, c.w);
    const v3 e2 = rcp_exact(dot(n, ray.d)) * (p0 - ray.o);
    const v3 i = cross(ray.d, e2);
    *beta = dot(i, e1);
    *gamma = dot(i, e0);
    *t = dot(n, e2);
    return (*t < ray.tmax) & (*t > ray.tmin) & (*beta >= 0.0f) & (*gamma >= 0.0f) & (*beta + *gamma <= 1);
}
PMD bool isect_tri(const float4 *g, const Ray &ray, float *t, float *beta, float *gamma) {
    return isect_tri_v(g[0], g[1], g[2], ray, t, beta, gamma);
}

/* cudadisk.cu:18-50 */
PMD bool isect_disk(const float4 *dk, const Ray &ray, float *thit_out) {
    float4 a = dk[0], b = dk[1], c = dk[2], d = dk[3], e = dk[4];
    v3 o = xyz(a), x = xyz(b), y = xyz(c), z = xyz(d);
    float thit = (c.w - dot(z, ray.o)) / dot(z, ray.d);
    if (!(thit > ray.tmin && thit < ray.tmax)) return false;
    v3 phit = ray.o + thit * ray.d;
    v3 local = phit - o;
    float localx = dot(local, x) * d.w;
    float localy = dot(local, y) * e.x;
    float dist2 = localx * localx + localy * localy;
    if (dist2 > 1.f || dist2 < a.w * a.w) return false;
    /* phi <= (float)2pi always, so a full disk (phiMax >= (float)2pi) can
     * never reject here: skip the double-precision atan2 (same result) */
    if (b.w < 6.28318548202514648438f) {
        float phi = pmdm_atan2f(localy, localx);
        if (phi < 0) phi = (float)((double)phi + 2.f * M_PI);
        if (phi > b.w) return false;
    }
    *thit_out = thit;
    return true;
}

PMD void xform_ray(const float4 *m, const Ray &r, v3 *o, v3 *d) {
    float4 r0 = m[0], r1 = m[1], r2 = m[2];
    *o = mk(((r0.x * r.o.x + r0.y * r.o.y) + r0.z * r.o.z) + r0.w,
            ((r1.x * r.o.x + r1.y * r.o.y) + r1.z * r.o.z) + r1.w,
            ((r2.x * r.o.x + r2.y * r.o.y) + r2.z * r.o.z) + r2.w);
    *d = mk((r0.x * r.d.x + r0.y * r.d.y) + r0.z * r.d.z,
            (r1.x * r.d.x + r1.y * r.d.y) + r1.z * r.d.z,
            (r2.x * r.d.x + r2.y * r.d.y) + r2.z * r.d.z);
}
/* rtTransformNormal(RT_OBJECT_TO_WORLD, n) = transpose(W2O) n */
PMD v3 xform_normal(const float4 *m, v3 n) {
    float4 r0 = m[0], r1 = m[1], r2 = m[2];
    return mk((r0.x * n.x + r1.x * n.y) + r2.x * n.z,
              (r0.y * n.x + r1.y * n.y) + r2.y * n.z,
              (r0.z * n.x + r1.z * n.y) + r2.z * n.z);
}

/* cudasphere.cu:7-72 */
PMD bool isect_sphere(const float4 *s, const Ray &ray, float *thit) {
    v3 o, d;
    xform_ray(s, ray, &o, &d);
    float rad = s[3].x;
    float A = dot(d, d);
    float B = 2.f * dot(d, o);
    float C = dot(o, o) - rad * rad;
    float discrim = B * B - 4.f * A * C;
    if (discrim < 0.f) return false;
    float root = sqrtf(discrim);
    float q = (B < 0) ? -.5f * (B - root) : -.5f * (B + root);
    float t0 = q / A, t1 = C / q;
    if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
    if (t0 > ray.tmin && t0 < ray.tmax) { *thit = t0; return true; }
    if (t1 > ray.tmin && t1 < ray.tmax) { *thit = t1; return true; }
    return false;
}

/* ---------------------------------------------------------- traversal */
/* Slab test of one child box; returns tnear (inf = miss). */
/* t = (plane - o) / d as one FMA, plane * inv - o * inv (oinv precomputed per
 * ray). The slab test only culls: its error is about one ulp of the
 * coordinates, and every primitive box is padded by 1e-4 of its coordinate
 * magnitude at commit (thousands of ulps), so no box holding a hit is culled. */
/* slab test; oinvH (default oinv) offsets the high planes: an instance tree
 * widens every box by a pad with oinv = (o' + pad) * inv, oinvH = (o' - pad)
 * * inv at no cost per box (blas_isect) */
PMD float box_near(float lx, float ly, float lz, float hx, float hy, float hz, v3 oinv, v3 inv, float tmin,
                   float tmax, v3 oinvH) {
    float t0x = __builtin_fmaf(lx, inv.x, -oinv.x), t1x = __builtin_fmaf(hx, inv.x, -oinvH.x);
    float t0y = __builtin_fmaf(ly, inv.y, -oinv.y), t1y = __builtin_fmaf(hy, inv.y, -oinvH.y);
    float t0z = __builtin_fmaf(lz, inv.z, -oinv.z), t1z = __builtin_fmaf(hz, inv.z, -oinvH.z);
    float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
    float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
    return tn <= tf ? tn : __int_as_float(0x7f800000);
}
PMD float box_near(float lx, float ly, float lz, float hx, float hy, float hz, v3 oinv, v3 inv, float tmin,
                   float tmax) {
    return box_near(lx, ly, lz, hx, hy, hz, oinv, inv, tmin, tmax, oinv);
}

PMD v3 safe_inv(v3 d) {
    const float tiny = 1e-20f;
    float x = fabsf(d.x) < tiny ? copysignf(tiny, d.x) : d.x;
    float y = fabsf(d.y) < tiny ? copysignf(tiny, d.y) : d.y;
    float z = fabsf(d.z) < tiny ? copysignf(tiny, d.z) : d.z;
    /* hardware reciprocal (<= 1 ulp): the slab test only culls, and every
     * prim box is padded by 1e-4 relative at commit, so an ulp in 1/d never
     * drops a box holding the closest hit (which is order-independent) */
    return mk(__builtin_amdgcn_rcpf(x), __builtin_amdgcn_rcpf(y), __builtin_amdgcn_rcpf(z));
}

/* per-lane traversal census (bench roofline / DESIGN.md): nodes entered and
 * primitive tests; NoCensus compiles to nothing */
struct NoCensus { PMD void node() {} PMD void prim() {} };
struct Census {
    uint32_t nodes = 0, prims = 0;
    PMD void node() { ++nodes; }
    PMD void prim() { ++prims; }
};

/* The scene as a kernel sees it. LDS=true: the whole blob is copied into
 * `lds` by the block (every thread calls; __syncthreads() before use) and
 * every pointer is rebased into it. The rebased pointers derive from a
 * __shared__ array, so the compiler emits ds_read (not flat) loads. */
template <bool LDS>
PMD SceneDev scene_view(const SceneDev &S, uint4 *lds, int tid, int nthreads) {
    if (!LDS) return S;
    const uint4 *src = reinterpret_cast<const uint4 *>(S.blob);
    for (int i = tid; i < (int)(S.lds_bytes / 16); i += nthreads) lds[i] = src[i];
    SceneDev V = S;
    const char *b = reinterpret_cast<const char *>(lds);
#define PM_REBASE(f) V.f = reinterpret_cast<decltype(V.f)>(b + (reinterpret_cast<const char *>(S.f) - S.blob))
    PM_REBASE(nodes); PM_REBASE(refs); PM_REBASE(tri_geo); PM_REBASE(tri_info); PM_REBASE(tri_id);
    PM_REBASE(tri_shade); PM_REBASE(norms); PM_REBASE(disks); PM_REBASE(spheres); PM_REBASE(materials);
    PM_REBASE(lights);
#undef PM_REBASE
    V.blob = b;
    return V;
}

/* closest hit so far: smaller t wins, equal t -> lowest global primitive id
 * (callers pass only t <= best.t), so the result is independent of the order
 * primitives are tested in (BVH or brute force) */
PMD void consider(Hit &best, float t, float b, float g, uint32_t ref, uint32_t gid) {
    if (t < best.t || gid < best.gid) { best.t = t; best.beta = b; best.gamma = g; best.ref = ref; best.gid = gid; }
}

/* MODE_BRUTE: every primitive, wave-uniform loop (same primitive in every
 * lane: broadcast LDS reads, no divergence, no stack) */
typedef const float __attribute__((address_space(4))) *const_f32_ptr;
typedef const uint32_t __attribute__((address_space(4))) *const_u32_ptr;
/* 16 B through the scalar cache (wave-uniform address) */
PMD float4 ldc4(const_f32_ptr q) { return make_float4(q[0], q[1], q[2], q[3]); }

typedef float f2 __attribute__((ext_vector_type(2)));
PMD f2 bc2(float x) { return f2{x, x}; }

/* isect_tri_v for two triangles at once (packed v_pk_mul/add_f32): the same
 * per-component IEEE operations in the same order, so each lane of the pair is
 * bit-identical to the scalar test. */
/* two triangles' (p0, e0, e1, n) as packed pairs, wave-uniform */
struct TriPair { f2 p0x, p0y, p0z, e0x, e0y, e0z, e1x, e1y, e1z, nx, ny, nz; };
/* the ray's origin and direction as packed splats. The components pass
 * through an empty asm first: splatting a value loaded from the path state
 * otherwise became a <2 x float> load of the state, which kept the ray in
 * scratch memory (5 scratch loads per ray in k_trace_lane) */
struct RaySplat { f2 ox, oy, oz, dx, dy, dz; };
PMD RaySplat splat_ray(const Ray &r) {
    float ox = r.o.x, oy = r.o.y, oz = r.o.z, dx = r.d.x, dy = r.d.y, dz = r.d.z;
    asm("" : "+v"(ox), "+v"(oy), "+v"(oz), "+v"(dx), "+v"(dy), "+v"(dz));
    return RaySplat{bc2(ox), bc2(oy), bc2(oz), bc2(dx), bc2(dy), bc2(dz)};
}
PMD void isect_tri_pair(const TriPair &q, const RaySplat &ray, f2 &t, f2 &beta, f2 &gamma) {
    const f2 p0x = q.p0x, p0y = q.p0y, p0z = q.p0z, e0x = q.e0x, e0y = q.e0y, e0z = q.e0z;
    const f2 e1x = q.e1x, e1y = q.e1y, e1z = q.e1z, nx = q.nx, ny = q.ny, nz = q.nz;
    const f2 dx = ray.dx, dy = ray.dy, dz = ray.dz;
    const f2 den = (nx * dx + ny * dy) + nz * dz; /* dot(n, d) */
    /* rcp_exact of both, one range check for the pair (either outside
     * [2^-125, 2^125): both divide; a NaN passes the check and gives NaN
     * either way) and the Newton step as two packed FMAs */
    const f2 r0 = f2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
    f2 inv = __builtin_elementwise_fma(__builtin_elementwise_fma(-den, r0, bc2(1.0f)), r0, r0);
    const float alo = fminf(fabsf(den.x), fabsf(den.y)), ahi = fmaxf(fabsf(den.x), fabsf(den.y));
    if (__builtin_expect(!(alo >= 0x1p-125f) | !(ahi < 0x1p125f), 0)) { inv.x = 1.0f / den.x; inv.y = 1.0f / den.y; }
    const f2 e2x = inv * (p0x - ray.ox), e2y = inv * (p0y - ray.oy), e2z = inv * (p0z - ray.oz);
    const f2 ix = dy * e2z - dz * e2y, iy = dz * e2x - dx * e2z, iz = dx * e2y - dy * e2x; /* cross(d, e2) */
    beta = (ix * e1x + iy * e1y) + iz * e1z;
    gamma = (ix * e0x + iy * e0y) + iz * e0z;
    t = (nx * e2x + ny * e2y) + nz * e2z;
}

/* Brute-force scenes store their triangles in global-id order (pm_api.cpp
 * build_scene), and triangles, disks, spheres are tested in that order, which
 * is ascending global id: a strict t < best.t keeps the first of equal-t hits
 * = the lowest id, the same hit consider() picks in any order — no id loads
 * in the loop. best.gid is left unset (nothing after the query reads it). */
PMD void take(Hit &best, float t, float b, float g, uint32_t ref) {
    best.t = t; best.beta = b; best.gamma = g; best.ref = ref;
}
/* a pair of SceneDev::tri_pairs_g: component c of triangle h at q[2c + h] */
PMD TriPair load_pair_il(const_f32_ptr q) {
    TriPair t;
    t.p0x = f2{q[0], q[1]}; t.p0y = f2{q[2], q[3]}; t.p0z = f2{q[4], q[5]};
    t.e0x = f2{q[6], q[7]}; t.e0y = f2{q[8], q[9]}; t.e0z = f2{q[10], q[11]};
    t.e1x = f2{q[12], q[13]}; t.e1y = f2{q[14], q[15]}; t.e1z = f2{q[16], q[17]};
    t.nx = f2{q[18], q[19]}; t.ny = f2{q[20], q[21]}; t.nz = f2{q[22], q[23]};
    return t;
}
template <bool ANY, class C>
PMD bool brute_isect(const SceneDev &S, const Ray &ray, Hit &best, C &cen) {
    const const_f32_ptr tg = (const_f32_ptr)S.tri_geo_g; /* constant address space: s_load */
    const RaySplat rs = splat_ray(ray);
    int k = 0;
    /* (software-pipelining the next pair's scalar loads measured slower:
     * C2 trace 91 vs 86 us — more live SGPRs, no unroll; so did pipelined
     * vector loads of the pairs into VGPRs: 73.5 -> 99 us, 111 VGPRs) */
    /* the running best in locals (one register per field: with the Hit
     * reference the compiler kept best.t twice, one more move per hit) */
    float bt = best.t, bb = best.beta, bg = best.gamma;
    uint32_t bref = best.ref;
#pragma unroll 2
    for (; k + 1 < S.n_tris; k += 2) {
        cen.prim(); cen.prim();
        f2 t, b, g;
        isect_tri_pair(load_pair_il((const_f32_ptr)S.tri_pairs_g + 12 * k), rs, t, b, g); /* pair k / 2: 24 floats */
        /* closest hit: t < best.t <= ray.tmax (traverse starts best.t at
         * tmax) implies t < tmax, so only the any-hit query tests tmax */
        const bool ok0 = (!ANY || t.x < ray.tmax) & (t.x > ray.tmin) & (b.x >= 0.0f) & (g.x >= 0.0f) & (b.x + g.x <= 1);
        const bool ok1 = (!ANY || t.y < ray.tmax) & (t.y > ray.tmin) & (b.y >= 0.0f) & (g.y >= 0.0f) & (b.y + g.y <= 1);
        if (ANY) { if (ok0 | ok1) return true; continue; }
        if (ok0 && t.x < bt) { bt = t.x; bb = b.x; bg = g.x; bref = (PRIM_TRI << 30) | (uint32_t)k; }
        if (ok1 && t.y < bt) { bt = t.y; bb = b.y; bg = g.y; bref = (PRIM_TRI << 30) | (uint32_t)(k + 1); }
    }
    if (!ANY) { best.t = bt; best.beta = bb; best.gamma = bg; best.ref = bref; }
    if (k < S.n_tris) {
        cen.prim();
        float t, b, g;
        const const_f32_ptr q = tg + 12 * k;
        const float4 a = make_float4(q[0], q[1], q[2], q[3]), bb = make_float4(q[4], q[5], q[6], q[7]),
                     cc = make_float4(q[8], q[9], q[10], q[11]);
        const bool ok = isect_tri_v(a, bb, cc, ray, &t, &b, &g);
        if (ANY && ok) return true;
        if (!ANY && ok && t < best.t) take(best, t, b, g, (PRIM_TRI << 30) | (uint32_t)k);
    }
    for (int k = 0; k < S.n_disks; ++k) {
        cen.prim();
        float t;
        const bool ok = isect_disk(S.disks + 5 * k, ray, &t);
        if (ANY) { if (ok) return true; continue; }
        if (ok && t < best.t) take(best, t, 0.f, 0.f, (PRIM_DISK << 30) | (uint32_t)k);
    }
    for (int k = 0; k < S.n_spheres; ++k) {
        cen.prim();
        float t;
        const bool ok = isect_sphere(S.spheres + 4 * k, ray, &t);
        if (ANY) { if (ok) return true; continue; }
        if (ok && t < best.t) take(best, t, 0.f, 0.f, (PRIM_SPHERE << 30) | (uint32_t)k);
    }
    return false;
}

/* Tests the primitives of one leaf; for ANY=true returns at the first hit.
 * TRIRUN: the leaf comes from a quantized 4-wide node, whose count may carry
 * pm_build.h's LEAF_TRIS flag (only quantize_bvh4 sets it; binary and float
 * 4-wide leaves are always decoded through their refs, whatever their size). */
template <bool ANY, class C>
PMD bool blas_isect(const SceneDev &S, uint32_t inst, const Ray &ray, Hit &best, int *stack, int stride, C &cen);
/* INST: the leaf's refs may be instances (MODE_INST), whose trees are walked
 * with the stack entries above the caller's (stack, stride) */
template <bool ANY, bool TRIRUN = false, class C, bool INST = false>
PMD bool leaf_isect(const SceneDev &S, uint32_t start, uint32_t count, const Ray &ray, Hit &best, C &cen,
                    int *istack = nullptr, int istride = 0) {
    if (TRIRUN && (count & 0x4000u)) { /* LEAF_TRIS: triangles at storage slots [start, start + n), no refs */
        for (uint32_t idx = start; idx < start + (count & 0x3fffu); ++idx) {
            cen.prim();
            float t, b, g;
            const bool ok = isect_tri(S.tri_geo + 3 * idx, ray, &t, &b, &g);
            if (ANY) { if (ok) return true; continue; }
            if (!ok || t > best.t) continue;
            const uint32_t gid = S.tri_id[idx];
            if (t < best.t || gid < best.gid) {
                best.t = t; best.beta = b; best.gamma = g; best.ref = (PRIM_TRI << 30) | idx; best.gid = gid;
            }
        }
        return false;
    }
    for (uint32_t k = start; k < start + count; ++k) {
        cen.prim();
        uint32_t ref = S.refs[k];
        uint32_t kind = ref >> 30, idx = ref & 0x3fffffffu;
        float t, b = 0.f, g = 0.f;
        bool ok;
        uint32_t gid;
        if (INST && kind == PRIM_INST) {
            if (blas_isect<ANY>(S, idx, ray, best, istack, istride, cen) && ANY) return true;
            continue;
        }
        if (kind == PRIM_TRI) {
            ok = isect_tri(S.tri_geo + 3 * idx, ray, &t, &b, &g);
            if (ANY) { if (ok) return true; continue; }
            if (!ok || t > best.t) continue;
            gid = S.tri_id[idx];
        } else if (kind == PRIM_DISK) {
            ok = isect_disk(S.disks + 5 * idx, ray, &t);
            if (ANY) { if (ok) return true; continue; }
            if (!ok || t > best.t) continue;
            gid = (uint32_t)fbits(S.disks[5 * idx + 4].w);
        } else {
            ok = isect_sphere(S.spheres + 4 * idx, ray, &t);
            if (ANY) { if (ok) return true; continue; }
            if (!ok || t > best.t) continue;
            gid = (uint32_t)fbits(S.spheres[4 * idx + 3].w);
        }
        if (t < best.t || gid < best.gid) { /* t <= best.t here: ties -> lowest id */
            best.t = t; best.beta = b; best.gamma = g; best.ref = ref; best.gid = gid;
        }
    }
    return false;
}

/* BVH traversal with a per-lane stack column in LDS (stack[depth*stride]).
 * Closest hit (ANY=false) or occlusion (ANY=true). Node = 4 float4:
 * (l.lo, l.hi.x) (l.hi.yz, r.lo.xy) (r.lo.z, r.hi) (left, right, lcount, rcount);
 * child >= 0 internal node, child < 0 leaf with refs start ~child. */
template <bool ANY, class C, bool INST = false>
PMD bool traverse4(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride, C &cen);
template <bool ANY, class C>
PMD bool traverse8(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride, C &cen);

template <bool ANY, int MODE, class C>
PMD bool traverse(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride, C &cen) {
    best.t = ray.tmax;
    best.gid = 0xffffffffu;
    best.ref = 0xffffffffu;
    const v3 inv = safe_inv(ray.d);
    const v3 oinv = mk(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    int sp = 0;
    int cur = 0; /* next node to enter; -1: none left */
    /* Leaves found while descending are postponed (at most the two children of
     * one node) and tested in a separate loop, so a wave runs the primitive
     * code once for all lanes that reached leaves instead of once per node
     * iteration for a few of them (Aila & Laine's "while-while"). Culling is
     * unchanged: a postponed leaf's box was hit within the current best t. */
    if constexpr (MODE == MODE_BRUTE) {
        cen.node();
        if (brute_isect<ANY>(S, ray, best, cen)) return true;
        return ANY ? false : best.ref != 0xffffffffu;
    }
    if constexpr (MODE == MODE_INST) {
        return traverse4<ANY, C, true>(S, ray, best, stack, stride, cen);
    } else if constexpr (MODE == MODE_GLOBAL) {
        if (S.wide == 3) return traverse8<ANY>(S, ray, best, stack, stride, cen);
        if (S.wide) return traverse4<ANY>(S, ray, best, stack, stride, cen);
    }
    uint32_t l0s = 0, l0n = 0, l1s = 0, l1n = 0; /* pending leaves: first ref, count (0 = none) */
    int guard = 0; /* every node is entered at most once per ray: a bound every lane reaches */
    while (true) {
        while (cur >= 0 && l0n == 0 && guard <= S.n_nodes) {
            ++guard;
            cen.node();
            const float4 *nd = S.nodes + 4 * cur;
            float4 a = nd[0], b = nd[1], c = nd[2];
            int4 ch = *reinterpret_cast<const int4 *>(nd + 3);
            float tl = box_near(a.x, a.y, a.z, a.w, b.x, b.y, oinv, inv, ray.tmin, best.t);
            float tr = box_near(b.z, b.w, c.x, c.y, c.z, c.w, oinv, inv, ray.tmin, best.t);
            bool hl = tl != __int_as_float(0x7f800000) && ch.z >= 0;
            bool hr = tr != __int_as_float(0x7f800000) && ch.w >= 0;
            if (hl && ch.x < 0) { l0s = (uint32_t)~ch.x; l0n = (uint32_t)ch.z; hl = false; }
            if (hr && ch.y < 0) {
                if (l0n == 0) { l0s = (uint32_t)~ch.y; l0n = (uint32_t)ch.w; }
                else { l1s = (uint32_t)~ch.y; l1n = (uint32_t)ch.w; }
                hr = false;
            }
            if (hl && hr && sp < S.stack_depth) {
                int nearc = ch.x, farc = ch.y;
                if (tr < tl) { nearc = ch.y; farc = ch.x; }
                stack[sp * stride] = farc;
                ++sp;
                cur = nearc;
            } else if (hl) {
                cur = ch.x;
            } else if (hr) {
                cur = ch.y;
            } else if (sp > 0) {
                --sp;
                cur = stack[sp * stride];
            } else {
                cur = -1;
            }
        }
        while (l0n != 0) {
            if (leaf_isect<ANY>(S, l0s, l0n, ray, best, cen)) return true;
            l0s = l1s; l0n = l1n; l1n = 0;
        }
        if (cur < 0 || guard > S.n_nodes) break;
    }
    return ANY ? false : best.ref != 0xffffffffu;
}
/* entry distances of the four children of 4-wide node `cur` (INF: missed)
 * and their codes / counts: 64-B quantized nodes (pm_build.h quantize_bvh4:
 * each bound decoded as o + q * 2^e, a box containing the float one; S.wide
 * == 2) or, in builds with PM_BVH4_QUANT=0, 128-B float nodes (S.wide == 1).
 * C3 trace 5.16 -> 4.75 ms per 1M paths (same box): half the bytes per visit,
 * 24 byte conversions + 24 multiply-adds more per node. */
#ifndef PM_QSLAB
#define PM_QSLAB 1 /* quantized planes folded into the slab test (node4_decode) */
#endif
#ifndef PM_BVH4_QUANT
#define PM_BVH4_QUANT 1 /* build-time node format: 1 = quantized 64-B nodes, 0 = 128-B float nodes */
#endif
/* a quantized node's four child boxes against the ray (the node's 64 B
 * already loaded: trav_step requests them ahead) */
PMD void node4_decode(const uint4 w0, const uint4 w1, const uint4 w2, const uint4 w3, const v3 &oinv, const v3 &inv,
                      float tmin, float tmax, float t[4], int c[4], int n[4], const v3 &oinvH);
PMD void node4_test(const SceneDev &S, int cur, const v3 &oinv, const v3 &inv, float tmin, float tmax, float t[4],
                    int c[4], int n[4], const v3 &oinvH) {
    if (PM_BVH4_QUANT) {
        const uint4 *nd = reinterpret_cast<const uint4 *>(S.wnodes) + 4 * cur;
        node4_decode(nd[0], nd[1], nd[2], nd[3], oinv, inv, tmin, tmax, t, c, n, oinvH);
    } else {
        const float4 *nd = S.wnodes + 8 * cur;
        const float4 lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5];
        const int4 ch = *reinterpret_cast<const int4 *>(nd + 6), cn = *reinterpret_cast<const int4 *>(nd + 7);
        t[0] = box_near(lx.x, ly.x, lz.x, hx.x, hy.x, hz.x, oinv, inv, tmin, tmax, oinvH);
        t[1] = box_near(lx.y, ly.y, lz.y, hx.y, hy.y, hz.y, oinv, inv, tmin, tmax, oinvH);
        t[2] = box_near(lx.z, ly.z, lz.z, hx.z, hy.z, hz.z, oinv, inv, tmin, tmax, oinvH);
        t[3] = box_near(lx.w, ly.w, lz.w, hx.w, hy.w, hz.w, oinv, inv, tmin, tmax, oinvH);
        c[0] = ch.x; c[1] = ch.y; c[2] = ch.z; c[3] = ch.w;
        n[0] = cn.x; n[1] = cn.y; n[2] = cn.z; n[3] = cn.w;
    }
}
PMD void node4_decode(const uint4 w0, const uint4 w1, const uint4 w2, const uint4 w3, const v3 &oinv, const v3 &inv,
                      float tmin, float tmax, float t[4], int c[4], int n[4], const v3 &oinvH) {
    {
        const float ox = __uint_as_float(w0.x), oy = __uint_as_float(w0.y), oz = __uint_as_float(w0.z);
        /* step 2^e: exponent field e + 127 = stored byte - 1 */
        const float sx = __uint_as_float(((w0.w & 0xffu) - 1u) << 23);
        const float sy = __uint_as_float((((w0.w >> 8) & 0xffu) - 1u) << 23);
        const float sz = __uint_as_float((((w0.w >> 16) & 0xffu) - 1u) << 23);
#if PM_QSLAB
        /* the plane o + q 2^e and the slab (plane - O) / d folded: t = q a + b
         * with a = 2^e / d, b = o / d - O / d per node, one FMA per plane
         * instead of a decode FMA and a slab FMA. Not the decoded plane's t
         * bit for bit, but within a few ulps of the coordinates, far inside
         * the 1e-4 relative pad of every primitive box (culling stays
         * conservative; closest hits do not depend on it) */
        const float ax = sx * inv.x, ay = sy * inv.y, az = sz * inv.z;
        const float bx = __builtin_fmaf(ox, inv.x, -oinv.x), by = __builtin_fmaf(oy, inv.y, -oinv.y),
                    bz = __builtin_fmaf(oz, inv.z, -oinv.z);
        const float bxH = __builtin_fmaf(ox, inv.x, -oinvH.x), byH = __builtin_fmaf(oy, inv.y, -oinvH.y),
                    bzH = __builtin_fmaf(oz, inv.z, -oinvH.z);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t sh = 8u * (uint32_t)k;
            const float t0x = __builtin_fmaf((float)((w1.x >> sh) & 0xffu), ax, bx);
            const float t0y = __builtin_fmaf((float)((w1.y >> sh) & 0xffu), ay, by);
            const float t0z = __builtin_fmaf((float)((w1.z >> sh) & 0xffu), az, bz);
            const float t1x = __builtin_fmaf((float)((w1.w >> sh) & 0xffu), ax, bxH);
            const float t1y = __builtin_fmaf((float)((w2.x >> sh) & 0xffu), ay, byH);
            const float t1z = __builtin_fmaf((float)((w2.y >> sh) & 0xffu), az, bzH);
            const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
            const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
            t[k] = tn <= tf ? tn : __int_as_float(0x7f800000);
        }
#else
        /* o + q * 2^e as one FMA: the product is exact, so the single
         * rounding is the add's — the encoder's decode, bit for bit */
#define QDEC(o, q, s) __builtin_fmaf((q), (s), (o))
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t sh = 8u * (uint32_t)k;
            const float lx = QDEC(ox, (float)((w1.x >> sh) & 0xffu), sx), ly = QDEC(oy, (float)((w1.y >> sh) & 0xffu), sy);
            const float lz = QDEC(oz, (float)((w1.z >> sh) & 0xffu), sz), hx = QDEC(ox, (float)((w1.w >> sh) & 0xffu), sx);
            const float hy = QDEC(oy, (float)((w2.x >> sh) & 0xffu), sy), hz = QDEC(oz, (float)((w2.y >> sh) & 0xffu), sz);
            t[k] = box_near(lx, ly, lz, hx, hy, hz, oinv, inv, tmin, tmax, oinvH);
        }
#undef QDEC
#endif
        c[0] = (int)w3.x; c[1] = (int)w3.y; c[2] = (int)w3.z; c[3] = (int)w3.w;
        n[0] = (int)(int16_t)(w2.z & 0xffffu); n[1] = (int)(int16_t)(w2.z >> 16);
        n[2] = (int)(int16_t)(w2.w & 0xffffu); n[3] = (int)(int16_t)(w2.w >> 16);
    }
}
PMD void node4_test(const SceneDev &S, int cur, const v3 &oinv, const v3 &inv, float tmin, float tmax, float t[4],
                    int c[4], int n[4]) {
    node4_test(S, cur, oinv, inv, tmin, tmax, t, c, n, oinv);
}

/* 4-wide traversal (MODE_GLOBAL scenes with S.wide): one 128-B node per
 * visit, its four boxes tested at once; hit internal children are ordered
 * near to far with a sorting network, the nearest entered next and the rest
 * pushed (the stack is sized by the builder's max_stack); hit leaves are
 * postponed and tested together as in traverse() (at most four per node). */
template <bool ANY, class C, bool INST>
PMD bool traverse4(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride, C &cen) {
    best.t = ray.tmax;
    best.gid = 0xffffffffu;
    best.ref = 0xffffffffu;
    const v3 inv = safe_inv(ray.d);
    const v3 oinv = mk(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    int sp = 0;
    int cur = 0;
    uint32_t l0s = 0, l0n = 0, l1s = 0, l1n = 0, l2s = 0, l2n = 0, l3s = 0, l3n = 0;
    int guard = 0;
    const float INF = __int_as_float(0x7f800000);
    while (true) {
        while (cur >= 0 && l0n == 0 && guard <= S.n_nodes) {
            ++guard;
            cen.node();
            float t[4];
            int c[4], n[4];
            node4_test(S, cur, oinv, inv, ray.tmin, best.t, t, c, n);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (t[k] != INF && n[k] > 0) { /* leaf: postpone */
                    const uint32_t s0 = (uint32_t)~c[k], n0 = (uint32_t)n[k];
                    if (l0n == 0) { l0s = s0; l0n = n0; }
                    else if (l1n == 0) { l1s = s0; l1n = n0; }
                    else if (l2n == 0) { l2s = s0; l2n = n0; }
                    else { l3s = s0; l3n = n0; }
                }
                if (n[k] != 0) t[k] = INF; /* only internal children stay */
            }
            /* near to far: (0,1) (2,3) (0,2) (1,3) (1,2) */
            auto cs = [&](int a, int b) {
                if (t[b] < t[a]) { const float tt = t[a]; t[a] = t[b]; t[b] = tt; const int cc = c[a]; c[a] = c[b]; c[b] = cc; }
            };
            cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
            if (t[3] != INF) { stack[sp * stride] = c[3]; ++sp; }
            if (t[2] != INF) { stack[sp * stride] = c[2]; ++sp; }
            if (t[1] != INF) { stack[sp * stride] = c[1]; ++sp; }
            if (t[0] != INF) cur = c[0];
            else if (sp > 0) { --sp; cur = stack[sp * stride]; }
            else cur = -1;
        }
        while (l0n != 0) {
            /* instance trees use the stack entries above the ones in use */
            if (leaf_isect<ANY, PM_BVH4_QUANT != 0, C, INST>(S, l0s, l0n, ray, best, cen, stack + sp * stride, stride))
                return true;
            l0s = l1s; l0n = l1n; l1s = l2s; l1n = l2n; l2s = l3s; l2n = l3n; l3n = 0;
        }
        if (cur < 0 || guard > S.n_nodes) break;
    }
    return ANY ? false : best.ref != 0xffffffffu;
}

/* ------------------------------------------------------ instance trees */
/* pbrt Transform::operator()(Point) for an affine transform (its w row is
 * (0, 0, 0, 1), checked at pm_add_mesh_instance, so w == 1 and no divide):
 * the host's flattening evaluates m[0] * x + m[1] * y + m[2] * z + m[3]
 * left to right — the same IEEE operations, in the same order */
PMD v3 inst_point(const float4 *m, float x, float y, float z) {
    const float4 r0 = m[0], r1 = m[1], r2 = m[2];
    return mk(((r0.x * x + r0.y * y) + r0.z * z) + r0.w, ((r1.x * x + r1.y * y) + r1.z * z) + r1.w,
              ((r2.x * x + r2.y * y) + r2.z * z) + r2.w);
}
/* object slot k of instance record I as the world triangle pm_commit would
 * have stored for the flattened mesh (tri_record: p0, e0 = p1 - p0,
 * e1 = p0 - p2, n = e1 x e0) */
PMD void inst_tri(const SceneDev &S, const float4 *I, uint32_t k, v3 &p0, v3 &p1, v3 &p2, float4 g[3]) {
    const float4 a = S.obj_v[3 * k], b = S.obj_v[3 * k + 1], c = S.obj_v[3 * k + 2];
    p0 = inst_point(I, a.x, a.y, a.z);
    p1 = inst_point(I, b.x, b.y, b.z);
    p2 = inst_point(I, c.x, c.y, c.z);
    const v3 e0 = p1 - p0, e1 = p0 - p2;
    const v3 n = mk(e1.y * e0.z - e1.z * e0.y, e1.z * e0.x - e1.x * e0.z, e1.x * e0.y - e1.y * e0.x);
    g[0] = make_float4(p0.x, p0.y, p0.z, e0.x);
    g[1] = make_float4(e0.y, e0.z, e1.x, e1.y);
    g[2] = make_float4(e1.z, n.x, n.y, n.z);
}
/* the instance record holding global triangle id gid (records ascend by id) */
PMD uint32_t inst_of_gid(const SceneDev &S, uint32_t gid) {
    uint32_t lo = 0, hi = (uint32_t)S.n_inst - 1u;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if ((uint32_t)__float_as_int(S.insts[8 * mid + 6].z) <= gid) lo = mid;
        else hi = mid - 1u;
    }
    return lo;
}
/* Closest hit (or any hit) among an instance's triangles. The object tree
 * is walked in object space: the ray taken through w2o (o' = w2o o, d' =
 * w2o d; the same t parameterises both, the transform being affine) and
 * every box widened by pad = 1e-5 (a (2 |o| + W) + k B), a = |w2o| (row
 * sums), W the instance's world extent, k = |o2w| |w2o|, B the object's
 * extent (both per instance, I[7]) — beyond the rounding of o', d' and of
 * the world vertices mapped back (~3 ulps of those magnitudes), so culling
 * is conservative: every triangle that can win is tested. Triangles are
 * rebuilt in world space (inst_tri) and tested with the world ray like a
 * flattened mesh's, so hits equal the flattened scene's bit for bit. The
 * stack entries above the caller's hold the walk (collapse_bvh4's bound). */
template <bool ANY, class C>
PMD bool blas_isect(const SceneDev &S, uint32_t inst, const Ray &ray, Hit &best, int *stack, int stride, C &cen) {
    const float4 *I = S.insts + 8 * inst;
    const float4 hd = I[6], pk = I[7];
    const uint32_t gid0 = (uint32_t)__float_as_int(hd.z);
    const float4 w0 = I[3], w1 = I[4], w2 = I[5];
    const v3 o = inst_point(I + 3, ray.o.x, ray.o.y, ray.o.z);
    const v3 d = mk((w0.x * ray.d.x + w0.y * ray.d.y) + w0.z * ray.d.z, (w1.x * ray.d.x + w1.y * ray.d.y) + w1.z * ray.d.z,
                    (w2.x * ray.d.x + w2.y * ray.d.y) + w2.z * ray.d.z);
    const float on = fmaxf(fabsf(ray.o.x), fmaxf(fabsf(ray.o.y), fabsf(ray.o.z)));
    const float pad = 1e-5f * (pk.y * (2.f * on) + pk.z);
    const v3 inv = safe_inv(d);
    const v3 oL = mk((o.x + pad) * inv.x, (o.y + pad) * inv.y, (o.z + pad) * inv.z);
    const v3 oH = mk((o.x - pad) * inv.x, (o.y - pad) * inv.y, (o.z - pad) * inv.z);
    const float INF = __int_as_float(0x7f800000);
    int sp = 0, cur = __float_as_int(hd.x), guard = 0;
    while (cur >= 0 && guard <= S.n_nodes) {
        ++guard;
        cen.node();
        float t[4];
        int c[4], n[4];
        node4_test(S, cur, oL, inv, ray.tmin, best.t, t, c, n, oH);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (t[k] == INF || n[k] <= 0) continue;
            /* a leaf: its triangles at object slots [~c, ~c + count) (LEAF_TRIS) */
            const uint32_t s0 = (uint32_t)~c[k], cnt = (uint32_t)n[k] & 0x3fffu;
            for (uint32_t q = s0; q < s0 + cnt; ++q) {
                cen.prim();
                v3 p0, p1, p2;
                float4 g[3];
                inst_tri(S, I, q, p0, p1, p2, g);
                float tt, bb, gg;
                const bool ok = isect_tri_v(g[0], g[1], g[2], ray, &tt, &bb, &gg);
                if (ANY) { if (ok) return true; continue; }
                if (!ok || tt > best.t) continue;
                const uint32_t gid = gid0 + (uint32_t)__float_as_int(S.obj_v[3 * q].w);
                if (tt < best.t || gid < best.gid) {
                    best.t = tt; best.beta = bb; best.gamma = gg; best.ref = (PRIM_INST << 30) | q; best.gid = gid;
                }
            }
            t[k] = INF;
        }
        /* internal children: nearest next, the others pushed */
        auto cs = [&](int a, int b) {
            if (t[b] < t[a]) { const float tt = t[a]; t[a] = t[b]; t[b] = tt; const int cc = c[a]; c[a] = c[b]; c[b] = cc; }
        };
        cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
        if (t[3] != INF) { stack[sp * stride] = c[3]; ++sp; }
        if (t[2] != INF) { stack[sp * stride] = c[2]; ++sp; }
        if (t[1] != INF) { stack[sp * stride] = c[1]; ++sp; }
        if (t[0] != INF) cur = c[0];
        else if (sp > 0) { --sp; cur = stack[sp * stride]; }
        else cur = -1;
    }
    return false;
}

/* Resumable closest-hit traversal of the 4-wide BVH for kernels that keep a
 * ray's traversal alive across iterations of an outer loop (k_trace_pool):
 * trav_step advances by one node visit or one leaf; the result equals
 * traverse4's (same culling, same leaf tests, same tie-break). */
struct TravState {
    v3 inv, oinv;
    Hit best;
    int cur, sp, guard;
    uint32_t l0s, l0n, l1s, l1n, l2s, l2n, l3s, l3n;
};
PMD void trav_begin(const Ray &ray, TravState &t) {
    t.best.t = ray.tmax;
    t.best.gid = 0xffffffffu;
    t.best.ref = 0xffffffffu;
    t.best.beta = t.best.gamma = 0.f;
    t.inv = safe_inv(ray.d);
    t.oinv = mk(ray.o.x * t.inv.x, ray.o.y * t.inv.y, ray.o.z * t.inv.z);
    t.cur = 0; t.sp = 0; t.guard = 0;
    t.l0n = t.l1n = t.l2n = t.l3n = 0;
    t.l0s = t.l1s = t.l2s = t.l3s = 0;
}
/* a lane's traversal stack: entries below cap in its LDS column, deeper ones
 * (rare: the bound is exact, typical depths are far below it) in a global
 * spill area, entry i of thread gid at spill[(i - cap) * sstride + gid] —
 * so the LDS a block reserves can be sized for occupancy, not the worst ray */
struct SpillStack {
    int *lds;
    int stride, cap;
    int *spill;
    uint32_t sstride, gid;
    PMD void put(int i, int v) const {
        if (i < cap) lds[i * stride] = v;
        else spill[(size_t)(i - cap) * sstride + gid] = v;
    }
    PMD int get(int i) const { return i < cap ? lds[i * stride] : spill[(size_t)(i - cap) * sstride + gid]; }
};
#ifndef PM_TRAV_FUSE
#define PM_TRAV_FUSE 1
#endif
#ifndef PM_LEAFQ_SHIFT
#define PM_LEAFQ_SHIFT 1 /* trav_step: hit leaves enter the (empty) queue by selects; C3 trace 3.86-3.88 -> 3.81-3.85 ms */
#endif
/* false once the ray is done (best holds its closest hit, if any) */
template <class C>
PMD bool trav_step(const SceneDev &S, const Ray &ray, TravState &T, const SpillStack &stk, C &cen) {
    /* (requesting the node before the pending leaf's test, so a wave's leaf
     * and node loads overlap, measured slower: C3 trace 4.14 -> 4.22-4.27 ms,
     * 88 B of scratch at 5 waves/SIMD or 4.23-4.26 ms at 4; profiles/r05/trace_c3) */
    if (T.l0n != 0) {
        leaf_isect<false, PM_BVH4_QUANT != 0>(S, T.l0s, T.l0n, ray, T.best, cen);
        T.l0s = T.l1s; T.l0n = T.l1n; T.l1s = T.l2s; T.l1n = T.l2n; T.l2s = T.l3s; T.l2n = T.l3n; T.l3n = 0;
#if PM_TRAV_FUSE
        /* the last pending leaf done: this step also visits the next node, so
         * a lane's leaf tests share steps with node visits (the wave runs
         * both codes whenever its lanes differ anyway). C3 trace per 1M paths
         * 4.42-4.43 -> 4.07-4.10 ms (same box); also testing the first leaf a
         * visit finds in the same step: 4.44 (the second leaf code costs every
         * step) */
        if (T.l0n != 0) return true;
#else
        return T.l0n != 0 || T.cur >= 0;
#endif
    }
    if (T.cur < 0 || T.guard > S.n_nodes) return false;
    ++T.guard;
    cen.node();
    const float INF = __int_as_float(0x7f800000);
    float t[4];
    int c[4], n[4];
    node4_test(S, T.cur, T.oinv, T.inv, ray.tmin, T.best.t, t, c, n);
#if PM_LEAFQ_SHIFT
    /* the pending-leaf queue is empty here (a visit follows the last pending
     * leaf's test): the hit leaves, in child order, enter it by shifting from
     * the back — selects only, no branch per child */
    {
        uint32_t a0s = 0, a0n = 0, a1s = 0, a1n = 0, a2s = 0, a2n = 0, a3s = 0, a3n = 0;
#pragma unroll
        for (int k = 3; k >= 0; --k) {
            if (t[k] != INF && n[k] > 0) {
                a3s = a2s; a3n = a2n; a2s = a1s; a2n = a1n; a1s = a0s; a1n = a0n;
                a0s = (uint32_t)~c[k]; a0n = (uint32_t)n[k];
            }
        }
        T.l0s = a0s; T.l0n = a0n; T.l1s = a1s; T.l1n = a1n; T.l2s = a2s; T.l2n = a2n; T.l3s = a3s; T.l3n = a3n;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (n[k] != 0) t[k] = INF;
#else
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (t[k] != INF && n[k] > 0) {
            const uint32_t s0 = (uint32_t)~c[k], n0 = (uint32_t)n[k];
            if (T.l0n == 0) { T.l0s = s0; T.l0n = n0; }
            else if (T.l1n == 0) { T.l1s = s0; T.l1n = n0; }
            else if (T.l2n == 0) { T.l2s = s0; T.l2n = n0; }
            else { T.l3s = s0; T.l3n = n0; }
        }
        if (n[k] != 0) t[k] = INF;
    }
#endif
    auto cs = [&](int a, int b) {
        if (t[b] < t[a]) { const float tt = t[a]; t[a] = t[b]; t[b] = tt; const int cc = c[a]; c[a] = c[b]; c[b] = cc; }
    };
    cs(0, 1); cs(2, 3); cs(0, 2); cs(1, 3); cs(1, 2);
    if (t[3] != INF) { stk.put(T.sp, c[3]); ++T.sp; }
    if (t[2] != INF) { stk.put(T.sp, c[2]); ++T.sp; }
    if (t[1] != INF) { stk.put(T.sp, c[1]); ++T.sp; }
    if (t[0] != INF) T.cur = c[0];
    else if (T.sp > 0) { --T.sp; T.cur = stk.get(T.sp); }
    else T.cur = -1;
    return T.l0n != 0 || T.cur >= 0;
}

/* ------------------------------------------------------- 8-wide trees */
/* S.wide == 3 (round 6, pm_build.h quantize_bvh8): 128-B quantized nodes of
 * eight children; the child word is the internal node index (>= 0), INT_MIN
 * for an empty slot, or a leaf ~((s << 5) | (tris << 4) | n). One visit tests
 * eight boxes: a third fewer node visits per ray than the 4-wide tree on
 * C3's soup (tools/bvh_width_sim.cpp: 30.1 -> 20.1), each a dependent fetch. */
constexpr int BVH8_EMPTY = (int)0x80000000;
PMD void node8_test(const SceneDev &S, int cur, const v3 &oinv, const v3 &inv, float tmin, float tmax, float t[8],
                    int c[8]) {
    const uint4 *nd = reinterpret_cast<const uint4 *>(S.wnodes) + 8 * cur;
    const uint4 w0 = nd[0], w1 = nd[1], w2 = nd[2], w3 = nd[3], w4 = nd[4], w5 = nd[5];
    const float ox = __uint_as_float(w0.x), oy = __uint_as_float(w0.y), oz = __uint_as_float(w0.z);
    const float sx = __uint_as_float(((w0.w & 0xffu) - 1u) << 23);
    const float sy = __uint_as_float((((w0.w >> 8) & 0xffu) - 1u) << 23);
    const float sz = __uint_as_float((((w0.w >> 16) & 0xffu) - 1u) << 23);
    /* node4_decode's folded slab: t = q (2^e / d) + (o - O) / d, one FMA per plane */
    const float ax = sx * inv.x, ay = sy * inv.y, az = sz * inv.z;
    const float bx = __builtin_fmaf(ox, inv.x, -oinv.x), by = __builtin_fmaf(oy, inv.y, -oinv.y),
                bz = __builtin_fmaf(oz, inv.z, -oinv.z);
    /* byte planes: lo x (w1.x, w1.y), lo y (w1.z, w1.w), lo z (w2.x, w2.y),
     * hi x (w2.z, w2.w), hi y (w3.x, w3.y), hi z (w3.z, w3.w) */
    const uint32_t LX[2] = {w1.x, w1.y}, LY[2] = {w1.z, w1.w}, LZ[2] = {w2.x, w2.y};
    const uint32_t HX[2] = {w2.z, w2.w}, HY[2] = {w3.x, w3.y}, HZ[2] = {w3.z, w3.w};
    c[0] = (int)w4.x; c[1] = (int)w4.y; c[2] = (int)w4.z; c[3] = (int)w4.w;
    c[4] = (int)w5.x; c[5] = (int)w5.y; c[6] = (int)w5.z; c[7] = (int)w5.w;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int h = k >> 2;
        const uint32_t sh = 8u * (uint32_t)(k & 3);
        const float t0x = __builtin_fmaf((float)((LX[h] >> sh) & 0xffu), ax, bx);
        const float t0y = __builtin_fmaf((float)((LY[h] >> sh) & 0xffu), ay, by);
        const float t0z = __builtin_fmaf((float)((LZ[h] >> sh) & 0xffu), az, bz);
        const float t1x = __builtin_fmaf((float)((HX[h] >> sh) & 0xffu), ax, bx);
        const float t1y = __builtin_fmaf((float)((HY[h] >> sh) & 0xffu), ay, by);
        const float t1z = __builtin_fmaf((float)((HZ[h] >> sh) & 0xffu), az, bz);
        const float tn = fmaxf(fmaxf(fminf(t0x, t1x), fminf(t0y, t1y)), fmaxf(fminf(t0z, t1z), tmin));
        const float tf = fminf(fminf(fmaxf(t0x, t1x), fmaxf(t0y, t1y)), fminf(fmaxf(t0z, t1z), tmax));
        t[k] = tn <= tf && c[k] != BVH8_EMPTY ? tn : __int_as_float(0x7f800000);
    }
}
/* a leaf child word's test (its refs, or LEAF_TRIS slots) */
template <bool ANY, class C>
PMD bool leaf8_isect(const SceneDev &S, int word, const Ray &ray, Hit &best, C &cen) {
    const uint32_t w = ~(uint32_t)word;
    return leaf_isect<ANY, true>(S, w >> 5, (w & 15u) | ((w & 16u) ? 0x4000u : 0u), ray, best, cen);
}
/* a node's hit internal children near to far: 32-bit keys (the entry t's
 * bits — non-negative floats order like their bits — with the low three
 * replaced by the child's slot; misses and leaves sort last as ~0) through
 * Batcher's odd-even merge network for 8 (19 min/max pairs). The order only
 * steers the walk; hits do not depend on it (lowest-id tie-break). */
PMD void sort8_keys(uint32_t k[8]) {
    auto cs = [&](int a, int b) { const uint32_t lo = min(k[a], k[b]), hi = max(k[a], k[b]); k[a] = lo; k[b] = hi; };
    cs(0, 1); cs(2, 3); cs(4, 5); cs(6, 7);
    cs(0, 2); cs(1, 3); cs(4, 6); cs(5, 7);
    cs(1, 2); cs(5, 6);
    cs(0, 4); cs(1, 5); cs(2, 6); cs(3, 7);
    cs(2, 4); cs(3, 5);
    cs(1, 2); cs(3, 4); cs(5, 6);
}
PMD int child8(const int c[8], uint32_t slot) { /* c[slot & 7] by selects (no dynamic register index) */
    const int a = (slot & 1u) ? c[1] : c[0], b = (slot & 1u) ? c[3] : c[2];
    const int d = (slot & 1u) ? c[5] : c[4], e = (slot & 1u) ? c[7] : c[6];
    const int f = (slot & 2u) ? b : a, g = (slot & 2u) ? e : d;
    return (slot & 4u) ? g : f;
}
/* one node visit of the 8-wide walk: the hit leaves tested at once (every
 * lane's, in one pass of the wave), the hit internal children sorted, the
 * nearest returned in `next` (-1: none) and the others pushed far to near */
template <bool ANY, class C, class Put>
PMD bool visit8(const SceneDev &S, int node, const Ray &ray, const v3 &oinv, const v3 &inv, Hit &best, C &cen, int &next,
                Put &&stack_put) {
    float t[8];
    int c[8];
    node8_test(S, node, oinv, inv, ray.tmin, best.t, t, c);
    const float INF = __int_as_float(0x7f800000);
    uint32_t key[8], lm = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (t[k] != INF && c[k] < 0) lm |= 1u << k;
        key[k] = t[k] != INF && c[k] >= 0 ? (__float_as_uint(t[k]) & ~7u) | (uint32_t)k : 0xffffffffu;
    }
    /* the hit leaves, one per lane per round: as many rounds as the lane with
     * the most (unrolled per slot, the wave ran the leaf code for every slot
     * any lane hit) */
    while (lm != 0u) {
        const uint32_t k = (uint32_t)__builtin_ctz(lm);
        lm &= lm - 1u;
        if (leaf8_isect<ANY>(S, child8(c, k), ray, best, cen) && ANY) return true;
    }
    sort8_keys(key);
#pragma unroll
    for (int k = 7; k >= 1; --k)
        if (key[k] != 0xffffffffu) stack_put(child8(c, key[k]));
    next = key[0] != 0xffffffffu ? child8(c, key[0]) : -1;
    return false;
}
/* one-call closest / any hit on the 8-wide tree (eye pass, shadow rays,
 * per-lane kernels) */
template <bool ANY, class C>
PMD bool traverse8(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride, C &cen) {
    best.t = ray.tmax;
    best.gid = 0xffffffffu;
    best.ref = 0xffffffffu;
    const v3 inv = safe_inv(ray.d);
    const v3 oinv = mk(ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z);
    int sp = 0, cur = 0, guard = 0;
    while (cur >= 0 && guard <= S.n_nodes) {
        ++guard;
        cen.node();
        int next = -1;
        if (visit8<ANY>(S, cur, ray, oinv, inv, best, cen, next, [&](int v) { stack[sp * stride] = v; ++sp; }))
            return true;
        if (next >= 0) cur = next;
        else if (sp > 0) { --sp; cur = stack[sp * stride]; }
        else cur = -1;
    }
    return ANY ? false : best.ref != 0xffffffffu;
}
/* resumable 8-wide traversal for k_trace_pool (trav_step's contract): one
 * node visit per step, its hit leaves tested in the same step (no pending
 * queue: the registers of eight queued leaves spilled the pooled kernel) */
struct TravState8 {
    v3 inv, oinv;
    Hit best;
    int cur, sp, guard;
};
PMD void trav_begin(const Ray &ray, TravState8 &t) {
    t.best.t = ray.tmax;
    t.best.gid = 0xffffffffu;
    t.best.ref = 0xffffffffu;
    t.best.beta = t.best.gamma = 0.f;
    t.inv = safe_inv(ray.d);
    t.oinv = mk(ray.o.x * t.inv.x, ray.o.y * t.inv.y, ray.o.z * t.inv.z);
    t.cur = 0; t.sp = 0; t.guard = 0;
}
template <class C>
PMD bool trav_step(const SceneDev &S, const Ray &ray, TravState8 &T, const SpillStack &stk, C &cen) {
    if (T.cur < 0 || T.guard > S.n_nodes) return false;
    ++T.guard;
    cen.node();
    int next = -1;
    visit8<false>(S, T.cur, ray, T.oinv, T.inv, T.best, cen, next, [&](int v) { stk.put(T.sp, v); ++T.sp; });
    if (next >= 0) T.cur = next;
    else if (T.sp > 0) { --T.sp; T.cur = stk.get(T.sp); }
    else T.cur = -1;
    return T.cur >= 0;
}

template <bool ANY, int MODE>
PMD bool traverse(const SceneDev &S, const Ray &ray, Hit &best, int *stack, int stride) {
    NoCensus none;
    return traverse<ANY, MODE>(S, ray, best, stack, stride, none);
}

/* ------------------------------------------------------------- shading */
struct Geo { v3 ns, dpdu; int material, light; };

/* hit attributes (cudatrianglemesh.cu:20-78, cudadisk.cu:36-47,
 * cudasphere.cu:35-48), transformed and normalized as the closest-hit
 * programs do (raytracing.cu:110-117, cudamaterial.cu.h:84-85). */
/* INST: the scene may hold instances (MODE_INST kernels); the others compile
 * without that branch (its registers cost the pooled trace kernel scratch) */
template <bool INST = true>
PMD Geo shade(const SceneDev &S, const Ray &ray, const Hit &h) {
    Geo g;
    uint32_t kind = h.ref >> 30, idx = h.ref & 0x3fffffffu;
    v3 nsw, dpduw;
    if (INST && kind == PRIM_INST) { /* an instance's triangle: the flattened triangle's frame, rebuilt */
        const float4 *I = S.insts + 8 * inst_of_gid(S, h.gid);
        v3 p0, p1, p2;
        float4 gg[3];
        inst_tri(S, I, idx, p0, p1, p2, gg);
        const v3 n = mk(gg[2].y, gg[2].z, gg[2].w);
        const int4 vi = S.obj_info[idx];
        const int4 mi = S.obj_mesh[vi.w];
        g.material = mi.x; g.light = mi.y;
        /* tri_frame (pm_api.cpp): dp/du from the uvs (cudatrianglemesh.cu:49-58) */
        float uv0x = 0.f, uv0y = 0.f, uv1x = 1.f, uv1y = 0.f, uv2x = 0.f, uv2y = 1.f;
        if (mi.w) {
            const float4 a = S.obj_uv[vi.x], b = S.obj_uv[vi.y], c = S.obj_uv[vi.z];
            uv0x = a.x; uv0y = a.y; uv1x = b.x; uv1y = b.y; uv2x = c.x; uv2y = c.y;
        }
        const float du1 = uv0x - uv2x, du2 = uv1x - uv2x, dv1 = uv0y - uv2y, dv2 = uv1y - uv2y;
        const float det = du1 * dv2 - dv1 * du2;
        v3 d;
        if (det == 0.0f) {
            if (fabsf(n.x) > fabsf(n.y)) {
                const float il = rcp_exact(sqrtf(n.x * n.x + n.z * n.z));
                d = mk(-n.z * il, 0.f, n.x * il);
            } else {
                const float il = rcp_exact(sqrtf(n.y * n.y + n.z * n.z));
                d = mk(0.f, n.z * il, n.y * il);
            }
        } else {
            const float invdet = rcp_exact(det);
            const v3 dp1 = p0 - p2, dp2 = p1 - p2;
            d = mk((dv2 * dp1.x - dv1 * dp2.x) * invdet, (dv2 * dp1.y - dv1 * dp2.y) * invdet,
                   (dv2 * dp1.z - dv1 * dp2.z) * invdet);
        }
        g.dpdu = normalize(d);
        if (!mi.z) { g.ns = normalize(n); return g; }
        /* vertex normals through pbrt's Transform::operator()(Normal) (transpose
         * of mInv), then interpolated per hit as for a flattened mesh */
        const float4 *W = I + 3;
        const v3 n0 = xform_normal(W, xyz(S.obj_n[vi.x])), n1 = xform_normal(W, xyz(S.obj_n[vi.y])),
                 n2 = xform_normal(W, xyz(S.obj_n[vi.z]));
        g.ns = normalize(n1 * h.beta + n2 * h.gamma + n0 * (1.0f - h.beta - h.gamma));
        return g;
    }
    if (kind == PRIM_TRI) {
        /* per-triangle frame (cudatrianglemesh.cu:36-78 + normalize), see tri_shade */
        const float4 s0 = S.tri_shade[2 * idx], s1 = S.tri_shade[2 * idx + 1];
        const int mb = fbits(s0.w);
        g.material = mb & 0x7fffffff; g.light = fbits(s1.w);
        g.dpdu = xyz(s1);
        if (mb >= 0) { g.ns = xyz(s0); return g; }
        const int4 ti = S.tri_info[idx]; /* shading normals: interpolated per hit */
        v3 n0 = xyz(S.norms[ti.x]), n1 = xyz(S.norms[ti.y]), n2 = xyz(S.norms[ti.z]);
        g.ns = normalize(n1 * h.beta + n2 * h.gamma + n0 * (1.0f - h.beta - h.gamma));
        return g;
    } else if (kind == PRIM_DISK) {
        const float4 *dk = S.disks + 5 * idx;
        float4 a = dk[0], b = dk[1], c = dk[2], d = dk[3], e = dk[4];
        v3 x = xyz(b), y = xyz(c);
        v3 phit = ray.o + h.t * ray.d;
        v3 local = phit - xyz(a);
        float localx = dot(local, x) * d.w;
        float localy = dot(local, y) * e.x;
        nsw = xyz(d);
        dpduw = -localy * x + localx * y;
        g.material = fbits(e.y); g.light = fbits(e.z);
    } else {
        const float4 *s = S.spheres + 4 * idx;
        v3 o, d;
        xform_ray(s, ray, &o, &d);
        float rad = s[3].x;
        v3 phit = o + h.t * d;
        if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * rad;
        v3 n = phit / rad;
        v3 dpdu = mk(-n.y, n.x, 0.f);
        nsw = xform_normal(s, n);
        dpduw = xform_normal(s, dpdu);
        g.material = fbits(s[3].y); g.light = fbits(s[3].z);
    }
    g.ns = normalize(nsw);
    g.dpdu = normalize(dpduw);
    return g;
}

PMD v3 world_to_local(v3 v, v3 nn, v3 sn, v3 tn) { return mk(dot(v, sn), dot(v, tn), dot(v, nn)); }
PMD v3 local_to_world(v3 v, v3 nn, v3 sn, v3 tn) {
    return mk(sn.x * v.x + tn.x * v.y + nn.x * v.z, sn.y * v.x + tn.y * v.y + nn.y * v.z,
              sn.z * v.x + tn.z * v.y + nn.z * v.z);
}
PMD bool is_specular(int type) { return type == PM_GLASS || type == PM_MIRROR; }

/* cudamaterial.cu.h:101-165; false on glass TIR */
PMD bool material_specular(int type, const Geo &g, v3 wow, v3 *wiw) {
    const v3 nn = g.ns, sn = g.dpdu, tn = cross(nn, sn);
    v3 wo = world_to_local(wow, nn, sn, tn);
    v3 wi;
    if (type == PM_MIRROR) {
        wi = mk(-wo.x, -wo.y, wo.z);
    } else {
        bool entering = wo.z > 0.f;
        float sini2 = fmaxf(0.f, 1.f - wo.z * wo.z);
        float eta = entering ? 1 / 1.5f : 1.5f;
        float sint2 = eta * eta * sini2;
        if (sint2 >= 1.0f) return false;
        float cost = sqrtf(fmaxf(0.f, 1.f - sint2));
        if (entering) cost = -cost;
        wi = mk(eta * -wo.x, eta * -wo.y, cost);
    }
    *wiw = local_to_world(wi, nn, sn, tn);
    return true;
}

/* cudamaterial.cu.h:50-98 (Lambert lobe); returns f = Kd/pi */
PMD v3 sample_f(v3 kd, const Geo &g, v3 wow, float u1, float u2, v3 *wiw, float *pdf) {
    const v3 nn = g.ns, sn = g.dpdu, tn = cross(nn, sn);
    v3 wo = world_to_local(wow, nn, sn, tn);
    float x, y;
    concentric_sample_disk(u1, u2, &x, &y);
    v3 wi = mk(x, y, sqrtf(fmaxf(0.f, 1.f - x * x - y * y)));
    if (wo.z < 0.f) wi.z *= -1.f;
    *pdf = (wo.z * wi.z > 0.0f) ? fabsf(wi.z) * INV_PI : 0.f;
    *wiw = local_to_world(wi, nn, sn, tn);
    return kd * INV_PI;
}

/* ------------------------------------------------------------- lights */
/* cudalight.cu.h:18-64 */
PMD v3 sample_l_shading(const LightDev &L, v3 point, float u1, float u2, v3 *uwi, float *pdf) {
    int type = fbits(L.o_type.w);
    if (type == PM_LIGHT_POINT) {
        *uwi = xyz(L.o_type) - point;
        float invlength2 = rcp_exact(dot(*uwi, *uwi));
        *pdf = 1.f;
        return xyz(L.le) * invlength2;
    }
    float x, y;
    concentric_sample_disk(u1, u2, &x, &y);
    *uwi = xyz(L.o_type) + x * xyz(L.p1_ns) + y * xyz(L.p2_r2d) - point;
    v3 wi = normalize(*uwi);
    float distanceSquared = dot(*uwi, *uwi);
    float costha = -dot(xyz(L.n_area), wi);
    *pdf = distanceSquared / (costha * L.n_area.w);
    return costha > 0.0f ? xyz(L.le) : mk(0.f, 0.f, 0.f);
}

/* cudalight.cu.h:78-124 — emission */
PMD v3 sample_le(const LightDev &L, float lu1, float lu2, float u1, float u2, float eps, Ray *ray, v3 *Ns,
                 float *pdf) {
    int type = fbits(L.o_type.w);
    if (type == PM_LIGHT_POINT) {
        ray->o = xyz(L.o_type);
        ray->d = uniform_sample_sphere(lu1, lu2);
        ray->tmin = eps;
        *Ns = ray->d;
        *pdf = (float)(1.f / (4.f * M_PI));
        return xyz(L.le);
    }
    float x, y;
    concentric_sample_disk(lu1, lu2, &x, &y);
    v3 org = xyz(L.o_type) + x * xyz(L.p1_ns) + y * xyz(L.p2_r2d);
    v3 dir = uniform_sample_sphere(u1, u2);
    *Ns = xyz(L.n_area);
    if (dot(dir, *Ns) < 0.f) dir = dir * -1.f;
    ray->o = org; ray->d = dir; ray->tmin = 1e-2f;
    *pdf = INV_TWOPI;
    return xyz(L.le) * L.n_area.w;
}

/* cudalight.cu.h:128-138 */
PMD v3 light_le(const LightDev &L, v3 wow) {
    if (dot(xyz(L.n_area), wow) > 0.f) return xyz(L.le);
    return mk(0.f, 0.f, 0.f);
}

/* ------------------------------------------------------------- census */
PMD unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

/* four census counters summed over the wave, one atomic each per wave (only
 * in counting launches, never in timed ones); every lane of the wave calls */
PMD void count4(unsigned long long *c, unsigned long long a, unsigned long long b, unsigned long long d,
                unsigned long long e) {
    a = wave_sum(a); b = wave_sum(b); d = wave_sum(d); e = wave_sum(e);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&c[0], a); atomicAdd(&c[1], b); atomicAdd(&c[2], d); atomicAdd(&c[3], e);
    }
}

/* record index -> pixel of an 8x8-tile ordering */
PMD void rec_to_pixel(int64_t r, int W, int *px, int *py) {
    int64_t tile = r >> 6;
    int lane = (int)(r & 63);
    int tilesX = (W + 7) / 8;
    *px = (int)(tile % tilesX) * 8 + (lane & 7);
    *py = (int)(tile / tilesX) * 8 + (lane >> 3);
}

} // namespace pm
