/*
 * pm_oracle.cpp — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * A plain, scalar, multi-threaded C++17 restatement of the reference
 * photon mapper (wjzhou/cuda-raytrace, cuda_render/) used to check the HIP
 * renderer and as the timed CPU baseline of bench.py. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it; the
 * product library (libpmhip.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned". The reference ships no tests, fixtures or
 * golden vectors and cannot be built here (OptiX 3.0,
 * CUDA 4.2 and the pbrt-v2 submodule are absent). This file
 * is therefore pinned piecewise by analytic known-answer tests derived from
 * the reference source (tests/test_oracle_kat.py) and by the committed
 * fixtures it generates (tests/golden/).
 *
 * Every function cites the reference file:line it restates. Floating-point
 * expressions keep the reference's operation order, with OptiX math
 * semantics (vector / scalar == vector * (1/scalar), normalize ==
 * v * (1/sqrt(dot(v,v)))), and the build compiles with -ffp-contract=off.
 * Transcendentals come from include/pm_detmath.h (deterministic libm).
 *
 * Documented divergences from the reference:
 *  - RNG: Philox4x32-10 keyed (777,0), counter (slot, pass) replaces cuRAND
 *    MTGP32 (photontracing.cu:159-161 reads rand[3*slot], rand[3*slot+1]).
 *  - glass total internal reflection terminates the photon / flags the eye
 *    record EXCEPTION (reference leaves wi uninitialised, cudamaterial.cu.h:124-126).
 *  - point-light photon tmin = scene_epsilon (uninitialised in the reference).
 *  - photon specular chains are capped at max_specular_depth (10).
 *  - closest-hit ties (equal t) resolve to the lowest global primitive id.
 */
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../include/pm_api.h"
#include "../include/pm_detmath.h"

namespace {

/* ------------------------------------------------------------------ math */
struct f3 { float x, y, z; };
inline f3 mk(float x, float y, float z) { return f3{x, y, z}; }
inline f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
inline f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
inline f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
/* optixu_math: operator/(float3,float) multiplies by the reciprocal */
inline f3 operator/(f3 a, float s) { float inv = 1.0f / s; return a * inv; }
inline float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
inline f3 normalize(f3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
inline float absdot(f3 a, f3 b) { return fabsf(dot(a, b)); } /* util.cu.h:13-15 */
inline bool is_black(f3 s) { return s.x == 0.0f && s.y == 0.0f && s.z == 0.0f; } /* util.cu.h:17-19 */
inline f3 ld3(const float *p) { return mk(p[0], p[1], p[2]); }
inline float comp(f3 v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }

const float INV_PI = 0.31830988618379067154f;   /* util.cu.h:3 */
const float INV_TWOPI = 0.15915494309189533577f; /* util.cu.h:4 */
const float RT_DEFAULT_MAX = 1.e27f;             /* OptiX 3 default ray tmax */

/* util.cu.h:23-65 — ConcentricSampleDisk (pbrt-v2 montecarlo). The
 * `theta *= M_PI / 4.f` multiply is a double-precision one, as written. */
void concentric_sample_disk(float u1, float u2, float *dx, float *dy) {
    float r, theta;
    float sx = 2 * u1 - 1;
    float sy = 2 * u2 - 1;
    if (sx == 0.0 && sy == 0.0) { *dx = 0.0; *dy = 0.0; return; }
    if (sx >= -sy) {
        if (sx > sy) { r = sx; if (sy > 0.0) theta = sy / r; else theta = 8.0f + sy / r; }
        else { r = sy; theta = 2.0f - sx / r; }
    } else {
        if (sx <= sy) { r = -sx; theta = 4.0f - sy / r; }
        else { r = -sy; theta = 6.0f + sx / r; }
    }
    theta = (float)((double)theta * (M_PI / 4.f));
    *dx = r * pmdm_cosf(theta);
    *dy = r * pmdm_sinf(theta);
}

/* cudalight.cu.h:66-73 — UniformSampleSphere; 2.f * M_PI * u2 is double. */
f3 uniform_sample_sphere(float u1, float u2) {
    float z = 1.f - 2.f * u1;
    float r = sqrtf(std::max(0.f, 1.f - z * z));
    float phi = (float)(2.f * M_PI * u2);
    return mk(r * pmdm_cosf(phi), r * pmdm_sinf(phi), z);
}

/* ------------------------------------------------------------------ scene */
struct Material { int type; f3 kd; };
struct Mesh { int material, light, has_n, has_uv; int64_t vbase; };
struct Tri { int v[3]; int mesh; };
struct Disk {
    f3 o, x, y, z; float inner, phimax, moffset, inv_rx2, inv_ry2; int material, light;
};
struct Sphere { float r; float o2w[16], w2o[16]; int material, light; };
struct Light {
    int type; f3 o, p1, p2, normal, intensity; float area; int nsample, rand2d_start;
};
struct Ray { f3 o, d; float tmin, tmax; };

struct BNode { float lo[3], hi[3]; int left, right, start, count; };

struct Scene {
    std::vector<Material> mats;
    std::vector<f3> P, N;
    std::vector<float> UV;
    std::vector<Mesh> meshes;
    std::vector<Tri> tris;
    std::vector<Disk> disks;
    std::vector<Sphere> spheres;
    std::vector<Light> lights;
    int rand2d_total = 0;
    /* eye */
    int pinhole = 0, W = 0, H = 0;
    f3 eye{}, fwd{}, right{}, up{};
    std::vector<float> rays, rand2d;
    int n2d = 0;
    int64_t nrays = 0;
    /* bvh */
    std::vector<BNode> nodes;
    std::vector<int> order;
    int64_t nprims() const { return (int64_t)tris.size() + disks.size() + spheres.size(); }
};

/* ----------------------------------------------------------- intersectors */
struct Hit {
    int64_t prim = -1;
    float t = 0.f, beta = 0.f, gamma = 0.f;
};

/* OptiX 3 intersect_triangle (branchless form), used by
 * cudatrianglemesh.cu:24 — SURVEY.md Appendix B item 9. */
bool isect_tri(f3 p0, f3 p1, f3 p2, const Ray &ray, float *t, float *beta, float *gamma) {
    const f3 e0 = p1 - p0;
    const f3 e1 = p0 - p2;
    const f3 n = cross(e1, e0);
    const f3 e2 = (1.0f / dot(n, ray.d)) * (p0 - ray.o);
    const f3 i = cross(ray.d, e2);
    *beta = dot(i, e1);
    *gamma = dot(i, e0);
    *t = dot(n, e2);
    return (*t < ray.tmax) & (*t > ray.tmin) & (*beta >= 0.0f) & (*gamma >= 0.0f) &
           (*beta + *gamma <= 1);
}

/* cudadisk.cu:18-50 */
bool isect_disk(const Disk &dk, const Ray &ray, float *thit_out, float *lx_out, float *ly_out) {
    float thit = (dk.moffset - dot(dk.z, ray.o)) / dot(dk.z, ray.d);
    if (!(thit > ray.tmin && thit < ray.tmax)) return false;
    f3 phit = ray.o + thit * ray.d;
    f3 local = phit - dk.o;
    float localx = dot(local, dk.x) * dk.inv_rx2;
    float localy = dot(local, dk.y) * dk.inv_ry2;
    float dist2 = localx * localx + localy * localy;
    if (dist2 > 1.f || dist2 < dk.inner * dk.inner) return false;
    float phi = pmdm_atan2f(localy, localx);
    if (phi < 0) phi = (float)((double)phi + 2.f * M_PI);
    if (phi > dk.phimax) return false;
    *thit_out = thit; *lx_out = localx; *ly_out = localy;
    return true;
}

/* world -> object transform of a ray for the sphere's Transform node
 * (cudasphere.cpp:27-29): o' = W2O (o,1), d' = W2O (d,0). */
void xform_ray(const float *m, const Ray &r, f3 *o, f3 *d) {
    *o = mk(((m[0] * r.o.x + m[1] * r.o.y) + m[2] * r.o.z) + m[3],
            ((m[4] * r.o.x + m[5] * r.o.y) + m[6] * r.o.z) + m[7],
            ((m[8] * r.o.x + m[9] * r.o.y) + m[10] * r.o.z) + m[11]);
    *d = mk((m[0] * r.d.x + m[1] * r.d.y) + m[2] * r.d.z,
            (m[4] * r.d.x + m[5] * r.d.y) + m[6] * r.d.z,
            (m[8] * r.d.x + m[9] * r.d.y) + m[10] * r.d.z);
}
/* rtTransformNormal(RT_OBJECT_TO_WORLD, n) = transpose(W2O) n */
f3 xform_normal(const float *m, f3 n) {
    return mk((m[0] * n.x + m[4] * n.y) + m[8] * n.z,
              (m[1] * n.x + m[5] * n.y) + m[9] * n.z,
              (m[2] * n.x + m[6] * n.y) + m[10] * n.z);
}

/* cudasphere.cu:7-25 */
bool quadratic(float A, float B, float C, float *t0, float *t1) {
    float discrim = B * B - 4.f * A * C;
    if (discrim < 0.) return false;
    float root = sqrtf(discrim);
    float q;
    if (B < 0) q = -.5f * (B - root);
    else q = -.5f * (B + root);
    *t0 = q / A;
    *t1 = C / q;
    if (*t0 > *t1) std::swap(*t0, *t1);
    return true;
}

/* cudasphere.cu:27-72: nearest root inside (tmin, tmax). */
bool isect_sphere(const Sphere &s, const Ray &ray, float *thit) {
    f3 o, d;
    xform_ray(s.w2o, ray, &o, &d);
    float A = dot(d, d);
    float B = 2.f * dot(d, o);
    float C = dot(o, o) - s.r * s.r;
    float t0, t1;
    if (!quadratic(A, B, C, &t0, &t1)) return false;
    if (t0 > ray.tmin && t0 < ray.tmax) { *thit = t0; return true; }
    if (t1 > ray.tmin && t1 < ray.tmax) { *thit = t1; return true; }
    return false;
}

/* primitive test; returns candidate t */
bool isect_prim(const Scene &S, int64_t pid, const Ray &ray, Hit *h) {
    int64_t nt = S.tris.size(), nd = S.disks.size();
    if (pid < nt) {
        const Tri &tr = S.tris[pid];
        float t, b, g;
        if (!isect_tri(S.P[tr.v[0]], S.P[tr.v[1]], S.P[tr.v[2]], ray, &t, &b, &g)) return false;
        h->t = t; h->beta = b; h->gamma = g;
        return true;
    }
    if (pid < nt + nd) {
        float t, lx, ly;
        if (!isect_disk(S.disks[pid - nt], ray, &t, &lx, &ly)) return false;
        h->t = t;
        return true;
    }
    float t;
    if (!isect_sphere(S.spheres[pid - nt - nd], ray, &t)) return false;
    h->t = t;
    return true;
}

/* -------------------------------------------------------------- oracle BVH
 * A plain median-split BVH (deliberately different from the product's
 * binned-SAH build): closest-hit results do not depend on it. */
void prim_bounds(const Scene &S, int64_t pid, float lo[3], float hi[3]) {
    int64_t nt = S.tris.size(), nd = S.disks.size();
    f3 mn, mx;
    if (pid < nt) {
        const Tri &tr = S.tris[pid];
        f3 a = S.P[tr.v[0]], b = S.P[tr.v[1]], c = S.P[tr.v[2]];
        mn = mk(std::min({a.x, b.x, c.x}), std::min({a.y, b.y, c.y}), std::min({a.z, b.z, c.z}));
        mx = mk(std::max({a.x, b.x, c.x}), std::max({a.y, b.y, c.y}), std::max({a.z, b.z, c.z}));
    } else if (pid < nt + nd) {
        const Disk &d = S.disks[pid - nt]; /* cudadisk.cu:87-96 */
        f3 p[4] = {d.o + d.x + d.y, d.o + d.x - d.y, d.o - d.x + d.y, d.o - d.x - d.y};
        mn = mx = p[0];
        for (int i = 1; i < 4; ++i) {
            mn = mk(std::min(mn.x, p[i].x), std::min(mn.y, p[i].y), std::min(mn.z, p[i].z));
            mx = mk(std::max(mx.x, p[i].x), std::max(mx.y, p[i].y), std::max(mx.z, p[i].z));
        }
    } else {
        const Sphere &s = S.spheres[pid - nt - nd]; /* object box [-r,r]^3 -> world */
        mn = mk(INFINITY, INFINITY, INFINITY); mx = mk(-INFINITY, -INFINITY, -INFINITY);
        for (int c = 0; c < 8; ++c) {
            float x = (c & 1) ? s.r : -s.r, y = (c & 2) ? s.r : -s.r, z = (c & 4) ? s.r : -s.r;
            const float *m = s.o2w;
            f3 w = mk(m[0] * x + m[1] * y + m[2] * z + m[3], m[4] * x + m[5] * y + m[6] * z + m[7],
                      m[8] * x + m[9] * y + m[10] * z + m[11]);
            mn = mk(std::min(mn.x, w.x), std::min(mn.y, w.y), std::min(mn.z, w.z));
            mx = mk(std::max(mx.x, w.x), std::max(mx.y, w.y), std::max(mx.z, w.z));
        }
    }
    float lo_[3] = {mn.x, mn.y, mn.z}, hi_[3] = {mx.x, mx.y, mx.z};
    for (int a = 0; a < 3; ++a) { /* conservative padding */
        float pad = 1e-4f * std::max(1.0f, std::max(fabsf(lo_[a]), fabsf(hi_[a])));
        lo[a] = lo_[a] - pad; hi[a] = hi_[a] + pad;
    }
}

int build_rec(Scene &S, std::vector<float> &blo, std::vector<float> &bhi, int start, int end) {
    int id = (int)S.nodes.size();
    S.nodes.push_back(BNode{});
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = start; i < end; ++i) {
        int p = S.order[i];
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], blo[3 * p + a]); hi[a] = std::max(hi[a], bhi[3 * p + a]);
            float c = 0.5f * (blo[3 * p + a] + bhi[3 * p + a]);
            clo[a] = std::min(clo[a], c); chi[a] = std::max(chi[a], c);
        }
    }
    BNode nd{};
    for (int a = 0; a < 3; ++a) { nd.lo[a] = lo[a]; nd.hi[a] = hi[a]; }
    if (end - start <= 4) {
        nd.left = nd.right = -1; nd.start = start; nd.count = end - start;
        S.nodes[id] = nd;
        return id;
    }
    int axis = 0;
    float ext[3] = {chi[0] - clo[0], chi[1] - clo[1], chi[2] - clo[2]};
    if (ext[1] > ext[axis]) axis = 1;
    if (ext[2] > ext[axis]) axis = 2;
    int mid = (start + end) / 2;
    std::nth_element(S.order.begin() + start, S.order.begin() + mid, S.order.begin() + end,
                     [&](int a, int b) {
                         float ca = blo[3 * a + axis] + bhi[3 * a + axis];
                         float cb = blo[3 * b + axis] + bhi[3 * b + axis];
                         return ca < cb || (ca == cb && a < b);
                     });
    nd.start = nd.count = 0;
    int l = build_rec(S, blo, bhi, start, mid);
    int r = build_rec(S, blo, bhi, mid, end);
    nd.left = l; nd.right = r;
    S.nodes[id] = nd;
    return id;
}

void build_bvh(Scene &S) {
    int64_t n = S.nprims();
    std::vector<float> blo(3 * n), bhi(3 * n);
    for (int64_t i = 0; i < n; ++i) prim_bounds(S, i, &blo[3 * i], &bhi[3 * i]);
    S.order.resize(n);
    for (int64_t i = 0; i < n; ++i) S.order[i] = (int)i;
    S.nodes.clear();
    if (n > 0) build_rec(S, blo, bhi, 0, (int)n);
}

inline bool box_hit(const BNode &nd, const Ray &r, float tmax) {
    float t0 = r.tmin, t1 = tmax;
    float o[3] = {r.o.x, r.o.y, r.o.z}, d[3] = {r.d.x, r.d.y, r.d.z};
    for (int a = 0; a < 3; ++a) {
        float inv = 1.0f / d[a];
        float tn = (nd.lo[a] - o[a]) * inv, tf = (nd.hi[a] - o[a]) * inv;
        if (tn > tf) std::swap(tn, tf);
        if (tn > t0) t0 = tn;
        if (tf < t1) t1 = tf;
        if (t0 > t1) return false;
    }
    return true;
}

/* closest hit; ties on t resolve to the lowest primitive id */
bool closest_hit(const Scene &S, const Ray &ray, Hit *best) {
    if (S.nodes.empty()) return false;
    int stack[128];
    int sp = 0;
    stack[sp++] = 0;
    best->prim = -1;
    float bt = ray.tmax;
    while (sp) {
        const BNode &nd = S.nodes[stack[--sp]];
        if (!box_hit(nd, ray, bt)) continue;
        if (nd.left < 0) {
            for (int i = 0; i < nd.count; ++i) {
                int pid = S.order[nd.start + i];
                Hit h;
                if (!isect_prim(S, pid, ray, &h)) continue;
                /* isect_prim guarantees t < ray.tmax, so the first hit always wins */
                if (h.t < bt || (h.t == bt && pid < best->prim)) {
                    bt = h.t; h.prim = pid; *best = h;
                }
            }
        } else {
            stack[sp++] = nd.left;
            stack[sp++] = nd.right;
        }
    }
    return best->prim >= 0;
}

/* any hit in (tmin, tmax) — shadow_any_hit (raytracing.cu:143-147) */
bool any_hit(const Scene &S, const Ray &ray) {
    if (S.nodes.empty()) return false;
    int stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const BNode &nd = S.nodes[stack[--sp]];
        if (!box_hit(nd, ray, ray.tmax)) continue;
        if (nd.left < 0) {
            for (int i = 0; i < nd.count; ++i) {
                Hit h;
                if (isect_prim(S, S.order[nd.start + i], ray, &h)) return true;
            }
        } else {
            stack[sp++] = nd.left;
            stack[sp++] = nd.right;
        }
    }
    return false;
}

/* --------------------------------------------------------------- shading
 * Hit attributes (cudashape.cu.h:7-11) already transformed to world space
 * with rtTransformNormal and normalized where the closest-hit programs
 * normalize them (raytracing.cu:110-117, photontracing.cu:166-167,
 * cudamaterial.cu.h:84-85). */
struct Geo { f3 ns, dpdu; int material, light; };

Geo shade(const Scene &S, const Ray &ray, const Hit &h) {
    Geo g;
    int64_t nt = S.tris.size(), nd = S.disks.size();
    f3 nsw, dpduw;
    if (h.prim < nt) { /* cudatrianglemesh.cu:20-78 */
        const Tri &tr = S.tris[h.prim];
        const Mesh &m = S.meshes[tr.mesh];
        f3 p0 = S.P[tr.v[0]], p1 = S.P[tr.v[1]], p2 = S.P[tr.v[2]];
        const f3 e0 = p1 - p0, e1 = p0 - p2;
        const f3 n = cross(e1, e0);
        float uv0x, uv0y, uv1x, uv1y, uv2x, uv2y;
        if (!m.has_uv) { uv0x = 0.f; uv0y = 0.f; uv1x = 1.f; uv1y = 0.f; uv2x = 0.f; uv2y = 1.f; }
        else {
            uv0x = S.UV[2 * tr.v[0]]; uv0y = S.UV[2 * tr.v[0] + 1];
            uv1x = S.UV[2 * tr.v[1]]; uv1y = S.UV[2 * tr.v[1] + 1];
            uv2x = S.UV[2 * tr.v[2]]; uv2y = S.UV[2 * tr.v[2] + 1];
        }
        float du1 = uv0x - uv2x, du2 = uv1x - uv2x, dv1 = uv0y - uv2y, dv2 = uv1y - uv2y;
        f3 dp1 = p0 - p2, dp2 = p1 - p2;
        float determinant = du1 * dv2 - dv1 * du2;
        f3 dpdu;
        if (determinant == 0.0f) {
            if (fabsf(n.x) > fabsf(n.y)) {
                float invLen = 1.f / sqrtf(n.x * n.x + n.z * n.z);
                dpdu = mk(-n.z * invLen, 0.f, n.x * invLen);
            } else {
                float invLen = 1.f / sqrtf(n.y * n.y + n.z * n.z);
                dpdu = mk(0.f, n.z * invLen, n.y * invLen);
            }
        } else {
            float invdet = 1.f / determinant;
            dpdu = (dv2 * dp1 - dv1 * dp2) * invdet;
        }
        f3 ns = n;
        if (m.has_n) {
            f3 n0 = S.N[tr.v[0]], n1 = S.N[tr.v[1]], n2 = S.N[tr.v[2]];
            ns = n1 * h.beta + n2 * h.gamma + n0 * (1.0f - h.beta - h.gamma);
        }
        nsw = ns; dpduw = dpdu;
        g.material = m.material; g.light = m.light;
    } else if (h.prim < nt + nd) { /* cudadisk.cu:36-47 */
        const Disk &dk = S.disks[h.prim - nt];
        f3 phit = ray.o + h.t * ray.d;
        f3 local = phit - dk.o;
        float localx = dot(local, dk.x) * dk.inv_rx2;
        float localy = dot(local, dk.y) * dk.inv_ry2;
        nsw = dk.z;
        dpduw = -localy * dk.x + localx * dk.y;
        g.material = dk.material; g.light = dk.light;
    } else { /* cudasphere.cu:35-48 (object space) */
        const Sphere &s = S.spheres[h.prim - nt - nd];
        f3 o, d;
        xform_ray(s.w2o, ray, &o, &d);
        f3 phit = o + h.t * d;
        if (phit.x == 0.f && phit.y == 0.f) phit.x = 1e-5f * s.r;
        f3 n = phit / s.r;
        f3 dpdu = mk(-n.y, n.x, 0.f);
        nsw = xform_normal(s.w2o, n);
        dpduw = xform_normal(s.w2o, dpdu);
        g.material = s.material; g.light = s.light;
    }
    g.ns = normalize(nsw);
    g.dpdu = normalize(dpduw);
    return g;
}

/* cudamaterial.cu.h:57-66 */
inline f3 world_to_local(f3 v, f3 nn, f3 sn, f3 tn) { return mk(dot(v, sn), dot(v, tn), dot(v, nn)); }
inline f3 local_to_world(f3 v, f3 nn, f3 sn, f3 tn) {
    return mk(sn.x * v.x + tn.x * v.y + nn.x * v.z, sn.y * v.x + tn.y * v.y + nn.y * v.z,
              sn.z * v.x + tn.z * v.y + nn.z * v.z);
}

inline bool is_specular(int type) { return type == PM_GLASS || type == PM_MIRROR; } /* cudamaterial.cu.h:168-173 */

/* cudamaterial.cu.h:23-32: Lambert only; specular materials have f = 0 */
inline f3 bsdf_f(const Scene &S, int mat) {
    const Material &m = S.mats[mat];
    if (m.type == PM_MATTE) return m.kd * INV_PI;
    return mk(0.f, 0.f, 0.f);
}

/* cudamaterial.cu.h:101-165 — returns false on glass TIR (build divergence) */
bool material_specular(int type, const Geo &g, f3 wow, f3 *wiw) {
    const f3 nn = g.ns, sn = g.dpdu, tn = cross(nn, sn);
    f3 wo = world_to_local(wow, nn, sn, tn);
    f3 wi;
    if (type == PM_MIRROR) {
        wi = mk(-wo.x, -wo.y, wo.z);
    } else {
        bool entering = wo.z > 0.f;
        float sini2 = std::max(0.f, 1.f - wo.z * wo.z);
        float eta = entering ? 1 / 1.5f : 1.5f;
        float sint2 = eta * eta * sini2;
        if (sint2 >= 1.0f) return false;
        float cost = sqrtf(std::max(0.f, 1.f - sint2));
        if (entering) cost = -cost;
        wi = mk(eta * -wo.x, eta * -wo.y, cost);
    }
    *wiw = local_to_world(wi, nn, sn, tn);
    return true;
}

/* cudamaterial.cu.h:50-98 — Sample_f with the Lambert lobe */
f3 sample_f(const Scene &S, int mat, const Geo &g, f3 wow, float u1, float u2, f3 *wiw, float *pdf) {
    const f3 nn = g.ns, sn = g.dpdu, tn = cross(nn, sn);
    f3 wo = world_to_local(wow, nn, sn, tn);
    float x, y;
    concentric_sample_disk(u1, u2, &x, &y);
    f3 wi = mk(x, y, sqrtf(std::max(0.f, 1.f - x * x - y * y)));
    if (wo.z < 0.) wi.z *= -1.f;
    *pdf = (wo.z * wi.z > 0.0f) ? fabsf(wi.z) * INV_PI : 0.f;
    *wiw = local_to_world(wi, nn, sn, tn);
    return S.mats[mat].kd * INV_PI; /* f_Lambert(materialParameter) */
}

/* ------------------------------------------------------------------ halton
 * photontracing.cu:19-43; table from pbrt-v2 PermutedHalton(5, RNG(seed))
 * (photonmappingrenderer.cpp:216), restated from pbrt-v2 core/montecarlo.h
 * GeneratePermutation + Shuffle and core/rng.h (MT19937 == std::mt19937). */
void halton_permutation(uint32_t seed, uint32_t out[28]) {
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

float permuted_radical_inverse(uint32_t n, uint32_t base, const uint32_t *p) {
    float val = 0;
    float invBase = 1.f / base, invBi = invBase;
    while (n > 0) {
        uint32_t d_i = p[n % base];
        val += d_i * invBi;
        n *= invBase; /* reference quirk: float multiply + truncation */
        invBi *= invBase;
    }
    return val;
}

void halton_sample(uint32_t n, const uint32_t *perm, float out[4]) {
    const uint32_t b[4] = {2, 3, 5, 7};
    const uint32_t *p = perm;
    for (int i = 0; i < 4; ++i) { out[i] = permuted_radical_inverse(n, b[i], p); p += b[i]; }
}

/* ------------------------------------------------------------------ lights */
/* cudalight.cu.h:78-124 — emission. Returns Le (pdf/ray/Ns outputs). */
f3 sample_le(const Light &L, float lu1, float lu2, float u1, float u2, float eps, Ray *ray, f3 *Ns, float *pdf) {
    if (L.type == PM_LIGHT_POINT) {
        ray->o = L.o;
        ray->d = uniform_sample_sphere(lu1, lu2);
        ray->tmin = eps; /* build: reference leaves tmin uninitialised */
        *Ns = ray->d;
        *pdf = (float)(1.f / (4.f * M_PI));
        return L.intensity;
    }
    float x, y;
    concentric_sample_disk(lu1, lu2, &x, &y);
    f3 org = L.o + x * L.p1 + y * L.p2;
    f3 dir = uniform_sample_sphere(u1, u2);
    *Ns = L.normal;
    if (dot(dir, *Ns) < 0.) dir = dir * -1.f;
    ray->o = org; ray->d = dir; ray->tmin = 1e-2f;
    *pdf = INV_TWOPI;
    return L.intensity * L.area;
}

/* cudalight.cu.h:18-64 — sampling a light from a shading point */
f3 sample_l_shading(const Light &L, f3 point, float u1, float u2, f3 *uwi, float *pdf) {
    if (L.type == PM_LIGHT_POINT) {
        *uwi = L.o - point;
        float invlength2 = 1.0f / dot(*uwi, *uwi);
        *pdf = 1.f;
        return L.intensity * invlength2;
    }
    float x, y;
    concentric_sample_disk(u1, u2, &x, &y);
    *uwi = L.o + x * L.p1 + y * L.p2 - point;
    f3 wi = normalize(*uwi);
    float distanceSquared = dot(*uwi, *uwi);
    float costha = -dot(L.normal, wi);
    *pdf = distanceSquared / (costha * L.area);
    return costha > 0.0f ? L.intensity : mk(0.f, 0.f, 0.f);
}

/* cudalight.cu.h:128-138 */
f3 light_le(const Scene &S, int light, f3 wow) {
    if (light >= 0) {
        const Light &L = S.lights[light];
        if (dot(L.normal, wow) > 0.f) return L.intensity;
    }
    return mk(0.f, 0.f, 0.f);
}

/* --------------------------------------------------------------- eye pass */
void rec_to_pixel(int64_t r, int W, int *px, int *py) {
    int64_t tile = r >> 6;
    int lane = (int)(r & 63);
    int tilesX = (W + 7) / 8;
    *px = (int)(tile % tilesX) * 8 + (lane & 7);
    *py = (int)(tile / tilesX) * 8 + (lane >> 3);
}

int64_t num_records(const Scene &S) {
    if (S.pinhole) return (int64_t)((S.W + 7) / 8) * ((S.H + 7) / 8) * 64;
    return S.nrays;
}

/* raytracing.cu:19-25, 87-128 and directLight :49-84 */
void eye_record(const Scene &S, const pm_render_params &P, int64_t r, pm_record *rec) {
    std::memset(rec, 0, sizeof(*rec));
    Ray ray;
    int64_t pixel;
    if (S.pinhole) {
        int px, py;
        rec_to_pixel(r, S.W, &px, &py);
        if (px >= S.W || py >= S.H) { rec->flags = PM_REC_INVALID; return; }
        pixel = (int64_t)py * S.W + px;
        float sx = (2.0f * ((float)px + 0.5f)) / (float)S.W - 1.0f;
        float sy = 1.0f - (2.0f * ((float)py + 0.5f)) / (float)S.H;
        f3 d = S.fwd + sx * S.right + sy * S.up;
        ray.o = S.eye;
        ray.d = normalize(d);
    } else {
        pixel = r;
        ray.o = ld3(&S.rays[6 * r]);
        ray.d = ld3(&S.rays[6 * r + 3]);
    }
    ray.tmin = P.scene_epsilon;
    ray.tmax = RT_DEFAULT_MAX;
    int depth = 0;
    Hit h;
    Geo g;
    while (true) {
        if (!closest_hit(S, ray, &h)) { rec->flags = PM_REC_MISS; return; } /* raytracing_miss :130-133 */
        g = shade(S, ray, h);
        const f3 point = ray.o + ray.d * h.t;
        int mtype = S.mats[g.material].type;
        if (is_specular(mtype)) { /* :89-104 */
            f3 wi;
            bool ok = material_specular(mtype, g, -ray.d, &wi);
            depth++;
            if (depth > P.max_specular_depth || !ok) { rec->flags = PM_REC_EXCEPTION; return; }
            ray.o = point; ray.d = wi; ray.tmin = P.scene_epsilon; ray.tmax = RT_DEFAULT_MAX;
            continue;
        }
        /* Faceforward(nn, wo) side for the kNN estimator; the reference keeps
         * the direction itself (record.direction, raytracing.cu:117) */
        rec->flags = dot(g.ns, -ray.d) < 0.f ? PM_REC_BACKFACE : 0u;
        rec->pos[0] = point.x; rec->pos[1] = point.y; rec->pos[2] = point.z;
        rec->ns[0] = g.ns.x; rec->ns[1] = g.ns.y; rec->ns[2] = g.ns.z;
        rec->material = g.material;
        rec->radius2 = P.initial_radius2;
        rec->photon_count = 0;
        break;
    }
    /* directLight (raytracing.cu:49-84) */
    f3 L = mk(0.f, 0.f, 0.f);
    const f3 point = ld3(rec->pos), ns = g.ns, dir = ray.d;
    int total = (int)S.lights.size();
    if (g.light < total) {
        L = L + light_le(S, g.light, -dir);
        f3 fv = bsdf_f(S, g.material);
        for (int i = 0; i < total; ++i) {
            const Light &Lt = S.lights[i];
            int nS = Lt.nsample;
            for (int s = 0; s < nS; ++s) {
                float u1 = 0.f, u2 = 0.f;
                if (Lt.type == PM_LIGHT_AREA_DISK) {
                    int slot = Lt.rand2d_start + s;
                    if (S.pinhole) {
                        uint32_t o4[4];
                        pmdm_philox4x32_10((uint32_t)pixel, (uint32_t)slot, 0u, 0u, P.light_rng_seed, 0u, o4);
                        u1 = pmdm_u01(o4[0]); u2 = pmdm_u01(o4[1]);
                    } else {
                        const float *q = &S.rand2d[((size_t)pixel * S.n2d + slot) * 2];
                        u1 = q[0]; u2 = q[1];
                    }
                }
                f3 uwi; float pdf;
                f3 li = sample_l_shading(Lt, point, u1, u2, &uwi, &pdf);
                Ray sr{point, uwi, 0.001f, 1.0f - 0.001f};
                float atten = any_hit(S, sr) ? 0.0f : 1.0f;
                f3 wi = normalize(uwi);
                L = L + (atten * fabsf(dot(ns, wi))) * fv * li / (pdf * nS);
            }
        }
    }
    rec->dl[0] = L.x; rec->dl[1] = L.y; rec->dl[2] = L.z;
}

/* ------------------------------------------------------- simple renderer
 * simple_render/simplerender.cu:26-79 (simple_camera, simple_cloest_hit,
 * simple_miss, simple_shadow_any_hit) + the host check of
 * simplerender.cpp:70-87. Writes the sample's output in output order. */
void simple_sample(const Scene &S, const pm_render_params &P, int64_t r, float *out_rgb) {
    Ray ray;
    int64_t pixel;
    if (S.pinhole) {
        int px, py;
        rec_to_pixel(r, S.W, &px, &py);
        if (px >= S.W || py >= S.H) return;
        pixel = (int64_t)py * S.W + px;
        float sx = (2.0f * ((float)px + 0.5f)) / (float)S.W - 1.0f;
        float sy = 1.0f - (2.0f * ((float)py + 0.5f)) / (float)S.H;
        f3 d = S.fwd + sx * S.right + sy * S.up;
        ray.o = S.eye;
        ray.d = normalize(d);
    } else {
        pixel = r;
        ray.o = ld3(&S.rays[6 * r]);
        ray.d = ld3(&S.rays[6 * r + 3]);
    }
    ray.tmin = P.scene_epsilon; /* simple_camera: Ray(o, d, 0, scene_epsilon) :26-32 */
    ray.tmax = RT_DEFAULT_MAX;
    f3 L = mk(0.f, 0.f, 0.f);
    Hit h;
    if (closest_hit(S, ray, &h)) {
        const Geo g = shade(S, ray, h);
        const f3 point = ray.o + ray.d * h.t;            /* :46 */
        const f3 fv = bsdf_f(S, g.material);            /* f(wo, wi): Lambert Kd/pi, else black */
        for (int i = 0; i < (int)S.lights.size(); ++i) { /* :53-72 */
            const Light &Lt = S.lights[i];
            float u1 = 0.f, u2 = 0.f;
            if (Lt.type == PM_LIGHT_AREA_DISK) {
                int slot = Lt.rand2d_start; /* Sample_L(i, point, uwi, pdf, 0) */
                if (S.pinhole) {
                    uint32_t o4[4];
                    pmdm_philox4x32_10((uint32_t)pixel, (uint32_t)slot, 0u, 0u, P.light_rng_seed, 0u, o4);
                    u1 = pmdm_u01(o4[0]); u2 = pmdm_u01(o4[1]);
                } else {
                    const float *q = &S.rand2d[((size_t)pixel * S.n2d + slot) * 2];
                    u1 = q[0]; u2 = q[1];
                }
            }
            f3 uwi; float pdf;
            f3 li = sample_l_shading(Lt, point, u1, u2, &uwi, &pdf);
            Ray sr{point, uwi, 0.001f, 1.0f - 0.001f};
            float atten = any_hit(S, sr) ? 0.0f : 1.0f;
            f3 wi = normalize(uwi);
            L = L + (atten * fabsf(dot(g.ns, wi))) * fv * li;
        }
    }
    float y = 0.212671f * L.x + 0.715160f * L.y + 0.072169f * L.z; /* pbrt RGBSpectrum::y */
    if (std::isnan(L.x) || std::isnan(L.y) || std::isnan(L.z) || y < -1e-5f || std::isinf(y))
        L = mk(0.f, 0.f, 0.f);
    out_rgb[3 * pixel + 0] = L.x; out_rgb[3 * pixel + 1] = L.y; out_rgb[3 * pixel + 2] = L.z;
}

/* ------------------------------------------------------------ photon pass
 * photontracing.cu:80-185 with the recursion unrolled into a loop. */
void trace_path(const Scene &S, const pm_render_params &P, const uint32_t *perm, int pass,
                uint64_t path, pm_photon *slots /* this path's max_photon_count slots */) {
    const uint32_t mpc = (uint32_t)P.max_photon_count;
    uint32_t pm_index = (uint32_t)(path * mpc); /* :82 */
    float smp[4];
    halton_sample(pm_index, perm, smp);
    const Light &Lt = S.lights[P.light_source_index];
    Ray ray; f3 N1; float pdf;
    f3 Le = sample_le(Lt, smp[0], smp[1], smp[2], smp[3], P.scene_epsilon, &ray, &N1, &pdf);
    if (pdf == 0.0f || is_black(Le)) return; /* :91 (slots stay zero = invalid) */
    ray.tmax = RT_DEFAULT_MAX;
    f3 alpha = (absdot(N1, ray.d) * Le) / pdf; /* :97 */
    uint32_t nI = 0;
    int spec = 0;
    Hit h;
    while (true) {
        if (!closest_hit(S, ray, &h)) return; /* photontracing_miss */
        Geo g = shade(S, ray, h);
        f3 hit_point = ray.o + h.t * ray.d;
        int mtype = S.mats[g.material].type;
        if (is_specular(mtype)) { /* :120-133 */
            f3 wi;
            if (!material_specular(mtype, g, -ray.d, &wi)) return;
            if (++spec > P.max_specular_depth) return;
            /* spec weight is 1 (cudamaterial.cu.h:104,133): alpha *= 1 */
            if (nI == 0) nI++;
            ray.o = hit_point; ray.d = wi; ray.tmin = P.scene_epsilon; ray.tmax = RT_DEFAULT_MAX;
            continue;
        }
        f3 wo = -ray.d;
        if (nI >= 1) { /* :141-151 */
            pm_photon &ph = slots[nI - 1];
            ph.bits = 1u;
            ph.p[0] = hit_point.x; ph.p[1] = hit_point.y; ph.p[2] = hit_point.z;
            ph.alpha[0] = alpha.x; ph.alpha[1] = alpha.y; ph.alpha[2] = alpha.z;
            ph.wi[0] = wo.x; ph.wi[1] = wo.y; ph.wi[2] = wo.z;
        }
        if (nI >= mpc) return; /* :153-155 */
        uint32_t o4[4];
        pmdm_philox4x32_10(pm_index + nI, (uint32_t)pass, 0u, 0u, P.rng_seed, 0u, o4);
        float u1 = pmdm_u01(o4[0]), u2 = pmdm_u01(o4[1]); /* :159-161 */
        f3 wiw; float bpdf;
        f3 fr = sample_f(S, g.material, g, wo, u1, u2, &wiw, &bpdf);
        if (is_black(fr) || bpdf == 0.f) return;
        f3 anew = alpha * fr * absdot(wiw, g.ns) / bpdf; /* :166-169 */
        alpha = anew;
        nI++;
        ray.o = hit_point; ray.d = wiw; ray.tmin = P.scene_epsilon; ray.tmax = RT_DEFAULT_MAX;
    }
}

/* ----------------------------------------------------------------- kd-tree
 * pbrt-v2 KdTree<TPhoton> (core/kdtree.h, unvendored)
 * as used by CreatePhotonMap (photonmappingrenderer.cpp:150-180). The
 * comparator's pointer tie-break becomes the index in the valid-photon list. */
struct KdBuild {
    const std::vector<pm_photon> *ph;
    std::vector<int> idx;
    pm_photon *out;
    uint32_t next_free;
    void rec(uint32_t node, int start, int end) {
        const std::vector<pm_photon> &P = *ph;
        if (start + 1 == end) {
            out[node] = P[idx[start]];
            out[node].bits = (3u << 1) | (PM_PHOTON_MAX_RIGHT_CHILD << 3);
            return;
        }
        float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = start; i < end; ++i)
            for (int a = 0; a < 3; ++a) {
                mn[a] = std::min(mn[a], P[idx[i]].p[a]);
                mx[a] = std::max(mx[a], P[idx[i]].p[a]);
            }
        float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        int axis = (dx > dy && dx > dz) ? 0 : (dy > dz ? 1 : 2); /* BBox::MaximumExtent */
        int mid = (start + end) / 2;
        std::nth_element(idx.begin() + start, idx.begin() + mid, idx.begin() + end, [&](int a, int b) {
            float pa = P[a].p[axis], pb = P[b].p[axis];
            return pa == pb ? a < b : pa < pb;
        });
        out[node] = P[idx[mid]];
        uint32_t bits = ((uint32_t)axis << 1) | (PM_PHOTON_MAX_RIGHT_CHILD << 3);
        if (start < mid) {
            bits |= 1u;
            uint32_t child = next_free++;
            rec(child, start, mid);
        }
        if (mid + 1 < end) {
            uint32_t rc = next_free++;
            bits = (bits & 7u) | (rc << 3);
            rec(rc, mid + 1, end);
        }
        out[node].bits = bits;
    }
};

/* gathering.cu:17-23 + 25-96 (explicit-stack lookup, sentinel 0) */
void kd_lookup(const pm_photon *nodes, const pm_record &rec, f3 fv, float maxDist2, int *nLookup,
               f3 *Lout, int64_t *visited) {
    uint32_t stack[64];
    uint32_t sp = 0;
    uint32_t nodeNum = 0;
    f3 L = mk(0.f, 0.f, 0.f);
    const f3 p = ld3(rec.pos), ns = ld3(rec.ns);
    stack[sp++] = 0;
    do {
        const pm_photon &nd = nodes[nodeNum];
        uint32_t axis = (nd.bits >> 1) & 3u, hasLeft = nd.bits & 1u, right = nd.bits >> 3;
        f3 np = ld3(nd.p);
        f3 diff = p - np; /* DistanceSquared(node->p, p), util.cu.h:8-11 */
        float dist2 = diff.x * diff.x + diff.y * diff.y + diff.z * diff.z;
        (*visited)++;
        if (dist2 < maxDist2) {
            (*nLookup)++;
            L = L + fabsf(dot(ns, ld3(nd.wi))) * fv * ld3(nd.alpha);
        }
        if (axis < 3) {
            float pa = comp(p, (int)axis), na = comp(np, (int)axis);
            float d2 = (pa - na) * (pa - na);
            if (pa <= na) {
                if (d2 < maxDist2 && right < PM_PHOTON_MAX_RIGHT_CHILD) stack[sp++] = right;
                if (hasLeft) nodeNum = nodeNum + 1; else nodeNum = stack[--sp];
            } else {
                if (d2 < maxDist2 && hasLeft) stack[sp++] = nodeNum + 1;
                if (right < PM_PHOTON_MAX_RIGHT_CHILD) nodeNum = right; else nodeNum = stack[--sp];
            }
        } else {
            nodeNum = stack[--sp];
        }
    } while (nodeNum);
    *Lout = L;
}

/* gathering.cu:104-126 PPM update */
void ppm_update(pm_record &rec, int M, f3 L, float alpha) {
    if (M > 0) {
        int totalPhotons = rec.photon_count + alpha * M;
        float ratio = totalPhotons / (rec.photon_count + M);
        rec.radius2 = rec.radius2 * ratio;
        f3 flux = (ld3(rec.flux) + L) * ratio;
        rec.flux[0] = flux.x; rec.flux[1] = flux.y; rec.flux[2] = flux.z;
        rec.photon_count = totalPhotons;
    }
}

/* ---- kNN estimator (PM_ESTIMATOR_KNN): pbrt-v2's photon map lookup --------
 * Restated from pbrt-v2 (unvendored submodule):
 * KdTree::privateLookup (core/kdtree.h), PhotonProcess + ClosePhoton + kernel()
 * + LPhoton's diffuse branch (integrators/photonmap.cpp). Parity unpinned. */
struct ClosePhoton {
    const pm_photon *photon;
    float d2;
    bool operator<(const ClosePhoton &o) const { return d2 == o.d2 ? photon < o.photon : d2 < o.d2; }
};
struct PhotonProcess {
    ClosePhoton *photons;
    uint32_t nLookup, nFound;
    void operator()(const pm_photon &ph, float d2, float &maxD2) {
        if (nFound < nLookup) { /* unordered until full, then a max-heap */
            photons[nFound++] = ClosePhoton{&ph, d2};
            if (nFound == nLookup) {
                std::make_heap(photons, photons + nLookup);
                maxD2 = photons[0].d2;
            }
        } else { /* replace the most distant photon */
            std::pop_heap(photons, photons + nLookup);
            photons[nLookup - 1] = ClosePhoton{&ph, d2};
            std::push_heap(photons, photons + nLookup);
            maxD2 = photons[0].d2;
        }
    }
};
/* KdTree::privateLookup: children first (near side, then far side if the
 * splitting plane is within the current radius), then the node itself */
void kd_knn(const pm_photon *nodes, int64_t nnodes, uint32_t nodeNum, f3 p, PhotonProcess &proc, float &maxD2,
            int64_t *visited) {
    const pm_photon &nd = nodes[nodeNum];
    const uint32_t axis = (nd.bits >> 1) & 3u, hasLeft = nd.bits & 1u, right = nd.bits >> 3;
    if (axis != 3) {
        const float pa = comp(p, (int)axis), split = nd.p[axis];
        const float dist2 = (pa - split) * (pa - split);
        if (pa <= split) {
            if (hasLeft) kd_knn(nodes, nnodes, nodeNum + 1, p, proc, maxD2, visited);
            if (dist2 < maxD2 && (int64_t)right < nnodes) kd_knn(nodes, nnodes, right, p, proc, maxD2, visited);
        } else {
            if ((int64_t)right < nnodes) kd_knn(nodes, nnodes, right, p, proc, maxD2, visited);
            if (dist2 < maxD2 && hasLeft) kd_knn(nodes, nnodes, nodeNum + 1, p, proc, maxD2, visited);
        }
    }
    (*visited)++;
    const f3 diff = ld3(nd.p) - p; /* DistanceSquared(nodeData[nodeNum].p, p) */
    const float d2 = diff.x * diff.x + diff.y * diff.y + diff.z * diff.z;
    if (d2 < maxD2) proc(nd, d2, maxD2);
}
/* One pass of LPhoton (diffuse branch) at a record: S = sum over the found
 * photons with Dot(Nf, wi) > 0 of kernel(d2) / maxD2 * alpha, where Nf =
 * Faceforward(nn, wo) and maxD2 is the lookup's shrunk radius. The 1/nPaths
 * and rho/pi = Kd/pi factors are applied at the final pass (final_radiance). */
f3 knn_estimate(const pm_photon *nodes, int64_t nnodes, const pm_record &rec, int K, float maxD2_0, int *nFound,
                float *maxD2_out, int64_t *visited) {
    ClosePhoton buf[PM_KNN_MAX];
    PhotonProcess proc{buf, (uint32_t)std::max(1, std::min(K, PM_KNN_MAX)), 0u};
    float maxD2 = maxD2_0;
    const f3 p = ld3(rec.pos);
    kd_knn(nodes, nnodes, 0, p, proc, maxD2, visited);
    const f3 ns = ld3(rec.ns);
    const f3 Nf = (rec.flags & PM_REC_BACKFACE) ? -ns : ns;
    f3 L = mk(0.f, 0.f, 0.f);
    for (uint32_t i = 0; i < proc.nFound; ++i) {
        const pm_photon &ph = *buf[i].photon;
        if (dot(Nf, ld3(ph.wi)) > 0.f) {
            const float s = (1.f - buf[i].d2 / maxD2);
            const float k = 3.f * INV_PI * s * s; /* kernel(): Simpson */
            L = L + (k / maxD2) * ld3(ph.alpha);
        }
    }
    *nFound = (int)proc.nFound;
    *maxD2_out = maxD2;
    return L;
}

/* gathering.cu:129-146 + host sanity check photonmappingrenderer.cpp:252-268;
 * kNN: L = direct + (sum of the passes' S / paths emitted) * rho/pi */
void final_radiance(const Scene &S, const pm_record &rec, float emitted, int estimator, float out[3]) {
    if ((rec.flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) != 0) {
        out[0] = out[1] = out[2] = 0.f;
        return;
    }
    f3 DL = ld3(rec.dl), IDL = mk(0.f, 0.f, 0.f);
    if (estimator == PM_ESTIMATOR_KNN) IDL = (ld3(rec.flux) / emitted) * bsdf_f(S, rec.material);
    else if (rec.photon_count != 0) IDL = ld3(rec.flux) * INV_PI / (rec.radius2 * emitted);
    f3 o = DL + IDL;
    float y = 0.212671f * o.x + 0.715160f * o.y + 0.072169f * o.z; /* pbrt RGBSpectrum::y */
    if (std::isnan(o.x) || std::isnan(o.y) || std::isnan(o.z) || y < -1e-5f || std::isinf(y))
        o = mk(0.f, 0.f, 0.f);
    out[0] = o.x; out[1] = o.y; out[2] = o.z;
}

template <class F>
void parallel_for(int64_t n, int nthreads, F f) {
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::thread::hardware_concurrency());
    if (n < 256 || nthreads == 1) { for (int64_t i = 0; i < n; ++i) f(i); return; }
    std::atomic<int64_t> next(0);
    const int64_t chunk = 256;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t)
        th.emplace_back([&]() {
            while (true) {
                int64_t b = next.fetch_add(chunk);
                if (b >= n) break;
                int64_t e = std::min(n, b + chunk);
                for (int64_t i = b; i < e; ++i) f(i);
            }
        });
    for (auto &x : th) x.join();
}

} // namespace

/* ======================================================================= */
/* exported C API (ctypes)                                                  */
/* ======================================================================= */
extern "C" {

void *orc_create(void) { return new Scene(); }
void orc_destroy(void *s) { delete (Scene *)s; }

int orc_add_material(void *s, int type, const float rgb[3]) {
    Scene &S = *(Scene *)s;
    S.mats.push_back(Material{type, ld3(rgb)});
    return (int)S.mats.size() - 1;
}

int orc_add_trimesh(void *s, const float *P, int nverts, const int *idx, int ntris, const float *N,
                    const float *uv, int material, int light) {
    Scene &S = *(Scene *)s;
    Mesh m{material, light, N != nullptr, uv != nullptr, (int64_t)S.P.size()};
    int64_t base = S.P.size();
    for (int i = 0; i < nverts; ++i) {
        S.P.push_back(ld3(P + 3 * i));
        S.N.push_back(N ? ld3(N + 3 * i) : mk(0.f, 0.f, 0.f));
        S.UV.push_back(uv ? uv[2 * i] : 0.f);
        S.UV.push_back(uv ? uv[2 * i + 1] : 0.f);
    }
    int mid = (int)S.meshes.size();
    S.meshes.push_back(m);
    for (int t = 0; t < ntris; ++t)
        S.tris.push_back(Tri{{(int)(base + idx[3 * t]), (int)(base + idx[3 * t + 1]), (int)(base + idx[3 * t + 2])}, mid});
    return 0;
}

int orc_add_sphere(void *s, float r, const float o2w[16], const float w2o[16], int material, int light) {
    Scene &S = *(Scene *)s;
    Sphere sp;
    sp.r = r;
    std::memcpy(sp.o2w, o2w, sizeof(sp.o2w));
    std::memcpy(sp.w2o, w2o, sizeof(sp.w2o));
    sp.material = material; sp.light = light;
    S.spheres.push_back(sp);
    return 0;
}

/* cudadisk.cu + derived uniforms of cudadisk.cpp:24-43 */
int orc_add_disk(void *s, const float o[3], const float x[3], const float y[3], const float z[3],
                 float inner_norm, float phi_max, int material, int light) {
    Scene &S = *(Scene *)s;
    Disk d;
    d.o = ld3(o); d.x = ld3(x); d.y = ld3(y); d.z = ld3(z);
    d.inner = inner_norm; d.phimax = phi_max;
    d.inv_rx2 = 1.f / (d.x.x * d.x.x + d.x.y * d.x.y + d.x.z * d.x.z);
    d.inv_ry2 = 1.f / (d.y.x * d.y.x + d.y.y * d.y.y + d.y.z * d.y.z);
    d.moffset = d.o.x * d.z.x + d.o.y * d.z.y + d.o.z * d.z.z;
    d.material = material; d.light = light;
    S.disks.push_back(d);
    return 0;
}

int orc_add_light_point(void *s, const float pos[3], const float I[3]) {
    Scene &S = *(Scene *)s;
    Light L{};
    L.type = PM_LIGHT_POINT; L.o = ld3(pos); L.intensity = ld3(I); L.nsample = 1; /* cudalight.cpp:16-24 */
    S.lights.push_back(L);
    return (int)S.lights.size() - 1;
}

int orc_add_light_disk(void *s, const float o[3], const float p1[3], const float p2[3], const float n[3],
                       const float Le[3], float area, int nsamples) {
    Scene &S = *(Scene *)s;
    Light L{};
    L.type = PM_LIGHT_AREA_DISK; L.o = ld3(o); L.p1 = ld3(p1); L.p2 = ld3(p2); L.normal = ld3(n);
    L.intensity = ld3(Le); L.area = area; L.nsample = std::max(1, nsamples);
    L.rand2d_start = S.rand2d_total; /* CudaSample::Add2D running offset, cudasample.cpp:2-9 */
    S.rand2d_total += L.nsample;
    S.lights.push_back(L);
    return (int)S.lights.size() - 1;
}

int orc_set_pinhole(void *s, const float eye[3], const float fwd[3], const float right[3], const float up[3],
                    int W, int H) {
    Scene &S = *(Scene *)s;
    S.pinhole = 1; S.W = W; S.H = H;
    S.eye = ld3(eye); S.fwd = ld3(fwd); S.right = ld3(right); S.up = ld3(up);
    return 0;
}

int orc_set_eye_rays(void *s, const float *rays, int64_t nrays, const float *rand2d, int n2d) {
    Scene &S = *(Scene *)s;
    S.pinhole = 0;
    S.nrays = nrays;
    S.rays.assign(rays, rays + 6 * nrays);
    S.n2d = n2d;
    if (rand2d && n2d > 0) S.rand2d.assign(rand2d, rand2d + (size_t)2 * n2d * nrays);
    return 0;
}

int orc_commit(void *s) { build_bvh(*(Scene *)s); return 0; }

int64_t orc_num_records(void *s) { return num_records(*(Scene *)s); }

int orc_record_pixel(void *s, int64_t r) {
    Scene &S = *(Scene *)s;
    if (!S.pinhole) return (int)r;
    int px, py;
    rec_to_pixel(r, S.W, &px, &py);
    if (px >= S.W || py >= S.H) return -1;
    return py * S.W + px;
}

void orc_eye_pass(void *s, const pm_render_params *P, pm_record *out, int nthreads) {
    Scene &S = *(Scene *)s;
    parallel_for(num_records(S), nthreads, [&](int64_t r) { eye_record(S, *P, r, &out[r]); });
}

void orc_halton_permutation(uint32_t seed, uint32_t out[28]) { halton_permutation(seed, out); }
void orc_halton_sample(uint32_t n, const uint32_t perm[28], float out[4]) { halton_sample(n, perm, out); }

void orc_trace_photons(void *s, const pm_render_params *P, int pass, int64_t path_begin, int64_t path_count,
                       pm_photon *slots, int nthreads) {
    Scene &S = *(Scene *)s;
    uint32_t perm[28];
    halton_permutation((uint32_t)pass, perm); /* RNG(pass), photonmappingrenderer.cpp:216 */
    std::memset(slots, 0, sizeof(pm_photon) * (size_t)path_count * P->max_photon_count);
    parallel_for(path_count, nthreads, [&](int64_t i) {
        trace_path(S, *P, perm, pass, (uint64_t)(path_begin + i), slots + (size_t)i * P->max_photon_count);
    });
}

/* returns node count (valid photons); nodes_out must hold nslots entries */
int64_t orc_build_kdtree(const pm_photon *slots, int64_t nslots, pm_photon *nodes_out) {
    std::vector<pm_photon> ph;
    ph.reserve(nslots);
    for (int64_t i = 0; i < nslots; ++i)
        if (slots[i].bits & 1u) ph.push_back(slots[i]); /* isValid, photonmappingrenderer.cpp:157-163 */
    if (ph.empty()) return 0;
    KdBuild b;
    b.ph = &ph;
    b.idx.resize(ph.size());
    for (size_t i = 0; i < ph.size(); ++i) b.idx[i] = (int)i;
    b.out = nodes_out;
    b.next_free = 1;
    b.rec(0, 0, (int)ph.size());
    return (int64_t)ph.size();
}

void orc_gather(void *s, const pm_photon *nodes, int64_t nnodes, pm_record *recs, int64_t nrec,
                const pm_render_params *P, int64_t counters[2], int nthreads) {
    Scene &S = *(Scene *)s;
    std::atomic<int64_t> vis(0), hits(0);
    parallel_for(nrec, nthreads, [&](int64_t r) {
        pm_record &rec = recs[r];
        if (rec.flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return; /* :108-111 */
        if (nnodes <= 0) return;
        int M = 0;
        int64_t v = 0;
        f3 L;
        if (P->estimator == PM_ESTIMATOR_KNN) {
            float md2 = P->initial_radius2;
            L = mk(0.f, 0.f, 0.f);
            if (S.mats[rec.material].type == PM_MATTE) /* non-specular BSDF components only */
                L = knn_estimate(nodes, nnodes, rec, P->knn_lookup, P->initial_radius2, &M, &md2, &v);
            const f3 flux = ld3(rec.flux) + L;
            rec.flux[0] = flux.x; rec.flux[1] = flux.y; rec.flux[2] = flux.z;
            rec.radius2 = md2;
            rec.photon_count = (float)M;
        } else {
            kd_lookup(nodes, rec, bsdf_f(S, rec.material), rec.radius2, &M, &L, &v);
            ppm_update(rec, M, L, P->ppm_alpha);
        }
        vis += v;
        hits += M;
    });
    if (counters) { counters[0] = vis.load(); counters[1] = hits.load(); }
}

/* range query only: per-record (M, L.rgb) — the linear part of the PPM
 * estimator that sharded photon maps sum across GPUs */
void orc_gather_partial(void *s, const pm_photon *nodes, int64_t nnodes, const pm_record *recs, int64_t nrec,
                        float *out4, int nthreads) {
    Scene &S = *(Scene *)s;
    parallel_for(nrec, nthreads, [&](int64_t r) {
        const pm_record &rec = recs[r];
        float *o = out4 + 4 * r;
        o[0] = o[1] = o[2] = o[3] = 0.f;
        if (rec.flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) return;
        if (nnodes <= 0) return;
        int M = 0;
        int64_t v = 0;
        f3 L;
        kd_lookup(nodes, rec, bsdf_f(S, rec.material), rec.radius2, &M, &L, &v);
        o[0] = (float)M; o[1] = L.x; o[2] = L.y; o[3] = L.z;
    });
}

/* final radiance in output order (raster for pinhole, ray order otherwise) */
void orc_final_est(void *s, const pm_record *recs, int64_t nrec, double emitted, int estimator, float *out_rgb,
                   int nthreads) {
    Scene &S = *(Scene *)s;
    float E = (float)emitted;
    parallel_for(nrec, nthreads, [&](int64_t r) {
        int64_t pix = r;
        if (S.pinhole) {
            int px, py;
            rec_to_pixel(r, S.W, &px, &py);
            if (px >= S.W || py >= S.H) return;
            pix = (int64_t)py * S.W + px;
        }
        final_radiance(S, recs[r], E, estimator, &out_rgb[3 * pix]);
    });
}
void orc_final(void *s, const pm_record *recs, int64_t nrec, double emitted, float *out_rgb, int nthreads) {
    orc_final_est(s, recs, nrec, emitted, PM_ESTIMATOR_PPM, out_rgb, nthreads);
}

/* whole pipeline: PhotonMappingRenderer::render (photonmappingrenderer.cpp:31-45) */
int orc_render(void *s, const pm_render_params *P, float *out_rgb, pm_stats *st, int nthreads) {
    Scene &S = *(Scene *)s;
    int64_t nrec = num_records(S);
    std::vector<pm_record> recs(nrec);
    orc_eye_pass(s, P, recs.data(), nthreads);
    int64_t nslots = P->paths_per_pass * P->max_photon_count;
    std::vector<pm_photon> slots(nslots), nodes(nslots);
    int64_t counters[2] = {0, 0};
    int64_t nvalid = 0;
    for (int pass = 0; pass < P->passes; ++pass) {
        orc_trace_photons(s, P, pass, 0, P->paths_per_pass, slots.data(), nthreads);
        nvalid = orc_build_kdtree(slots.data(), nslots, nodes.data());
        if (nvalid == 0) return PM_ERR_NO_PHOTONS;
        orc_gather(s, nodes.data(), nvalid, recs.data(), nrec, P, counters, nthreads);
    }
    double emitted = (double)P->paths_per_pass * P->passes;
    orc_final_est(s, recs.data(), nrec, emitted, P->estimator, out_rgb, nthreads);
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->paths_emitted = (int64_t)emitted;
        st->photons_valid = nvalid;
        int64_t act = 0;
        for (auto &r : recs) act += (r.flags & (PM_REC_MISS | PM_REC_EXCEPTION | PM_REC_INVALID)) == 0;
        st->gather_points = act;
        st->nodes_visited = counters[0];
        st->photons_in_radius = counters[1];
    }
    return PM_OK;
}

/* SimpleRenderer::render (simple_render/simplerender.cpp:18-103); out_rgb in
 * output order (raster for pinhole, ray order otherwise), zero-initialised */
void orc_render_simple(void *s, const pm_render_params *P, float *out_rgb, int nthreads) {
    Scene &S = *(Scene *)s;
    parallel_for(num_records(S), nthreads, [&](int64_t r) { simple_sample(S, *P, r, out_rgb); });
}

/* ---- primitive entry points for known-answer tests -------------------- */
void orc_concentric_sample_disk(float u1, float u2, float out[2]) { concentric_sample_disk(u1, u2, &out[0], &out[1]); }
void orc_uniform_sample_sphere(float u1, float u2, float out[3]) {
    f3 v = uniform_sample_sphere(u1, u2); out[0] = v.x; out[1] = v.y; out[2] = v.z;
}
int orc_intersect_triangle(const float p0[3], const float p1[3], const float p2[3], const float o[3],
                           const float d[3], float tmin, float tmax, float out[3]) {
    Ray r{ld3(o), ld3(d), tmin, tmax};
    return isect_tri(ld3(p0), ld3(p1), ld3(p2), r, &out[0], &out[1], &out[2]) ? 1 : 0;
}
int orc_intersect_disk(const float o[3], const float x[3], const float y[3], const float z[3], float inner,
                       float phimax, const float ro[3], const float rd[3], float tmin, float tmax, float *t) {
    Scene S;
    orc_add_disk(&S, o, x, y, z, inner, phimax, 0, -1);
    Ray r{ld3(ro), ld3(rd), tmin, tmax};
    float lx, ly;
    return isect_disk(S.disks[0], r, t, &lx, &ly) ? 1 : 0;
}
int orc_intersect_sphere(float radius, const float o2w[16], const float w2o[16], const float ro[3],
                         const float rd[3], float tmin, float tmax, float *t) {
    Sphere s;
    s.r = radius;
    std::memcpy(s.o2w, o2w, 64); std::memcpy(s.w2o, w2o, 64);
    Ray r{ld3(ro), ld3(rd), tmin, tmax};
    return isect_sphere(s, r, t) ? 1 : 0;
}
void orc_ppm_update(float *radius2, float *photon_count, float flux[3], int M, const float L[3], float alpha) {
    pm_record r{};
    r.radius2 = *radius2; r.photon_count = *photon_count;
    r.flux[0] = flux[0]; r.flux[1] = flux[1]; r.flux[2] = flux[2];
    ppm_update(r, M, ld3(L), alpha);
    *radius2 = r.radius2; *photon_count = r.photon_count;
    flux[0] = r.flux[0]; flux[1] = r.flux[1]; flux[2] = r.flux[2];
}
void orc_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    pmdm_philox4x32_10(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1], out);
}
float orc_sinf(float x) { return pmdm_sinf(x); }
float orc_cosf(float x) { return pmdm_cosf(x); }
float orc_atan2f(float y, float x) { return pmdm_atan2f(y, x); }

} /* extern "C" */
