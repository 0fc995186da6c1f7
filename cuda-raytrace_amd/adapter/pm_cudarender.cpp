/*
 * pm_cudarender.cpp — see pm_cudarender.h. Host-only C++: scene flattening
 * (the reference's CudaShape / CudaMaterial / CudaLight setup code, restated
 * over plain descriptors) and the render driver, all over the C-ABI.
 */
#include "pm_cudarender.h"

#include <cstdlib>

#include <cmath>
#include <cstdio>
#include <cstring>

namespace pmcuda {

/* ------------------------------------------------------------ Transform */
Transform Transform::identity() {
    Transform t;
    for (int i = 0; i < 16; ++i) t.m[i] = t.minv[i] = (i % 5 == 0) ? 1.f : 0.f;
    return t;
}

Transform Transform::translate(float x, float y, float z) {
    Transform t = identity();
    t.m[3] = x; t.m[7] = y; t.m[11] = z;
    t.minv[3] = -x; t.minv[7] = -y; t.minv[11] = -z;
    return t;
}

Transform Transform::rotate_x(float degrees) {
    /* pbrt RotateX: m = [1 0 0 0; 0 c -s 0; 0 s c 0; 0 0 0 1], inverse = transpose */
    const float rad = degrees * 0.01745329251994329577f;
    const float s = std::sin(rad), c = std::cos(rad);
    Transform t = identity();
    t.m[5] = c; t.m[6] = -s; t.m[9] = s; t.m[10] = c;
    t.minv[5] = c; t.minv[6] = s; t.minv[9] = -s; t.minv[10] = c;
    return t;
}

static void matmul(const float *a, const float *b, float *out) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            out[4 * i + j] = a[4 * i] * b[j] + a[4 * i + 1] * b[4 + j] + a[4 * i + 2] * b[8 + j] +
                             a[4 * i + 3] * b[12 + j];
}

Transform Transform::operator*(const Transform &b) const {
    Transform r;
    matmul(m, b.m, r.m);
    matmul(b.minv, minv, r.minv);
    return r;
}

/* pbrt Transform::operator()(Point): homogeneous divide only when w != 1 */
void Transform::point(const float p[3], float out[3]) const {
    float x = m[0] * p[0] + m[1] * p[1] + m[2] * p[2] + m[3];
    float y = m[4] * p[0] + m[5] * p[1] + m[6] * p[2] + m[7];
    float z = m[8] * p[0] + m[9] * p[1] + m[10] * p[2] + m[11];
    float w = m[12] * p[0] + m[13] * p[1] + m[14] * p[2] + m[15];
    if (w == 1.f) { out[0] = x; out[1] = y; out[2] = z; }
    else { const float inv = 1.f / w; out[0] = x * inv; out[1] = y * inv; out[2] = z * inv; } /* pbrt Point/float */
}

void Transform::vector(const float v[3], float out[3]) const {
    out[0] = m[0] * v[0] + m[1] * v[1] + m[2] * v[2];
    out[1] = m[4] * v[0] + m[5] * v[1] + m[6] * v[2];
    out[2] = m[8] * v[0] + m[9] * v[1] + m[10] * v[2];
}

void Transform::normal(const float n[3], float out[3]) const {
    out[0] = minv[0] * n[0] + minv[4] * n[1] + minv[8] * n[2];
    out[1] = minv[1] * n[0] + minv[5] * n[1] + minv[9] * n[2];
    out[2] = minv[2] * n[0] + minv[6] * n[1] + minv[10] * n[2];
}

/* ------------------------------------------------------------ helpers */
static void check(void *ctx, int rc, const char *what) {
    if (rc != PM_OK) throw Error(std::string(what) + ": " + pm_last_error(ctx));
}

static void warning(const char *fmt, const char *arg) {
    std::fprintf(stderr, "Warning: ");
    std::fprintf(stderr, fmt, arg);
    std::fprintf(stderr, "\n");
}

/* pbrt Normalize: v / Length(v), with Vector::operator/ multiplying by 1/f */
static void normalize3(float v[3]) {
    const float inv = 1.f / std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    for (int a = 0; a < 3; ++a) v[a] = v[a] * inv;
}

/* CudaDisk::setupGeometry (cudadisk.cpp:24-43) */
struct DiskFrame { float o[3], x[3], y[3], z[3]; };
static DiskFrame disk_frame(const Shape &d) {
    DiskFrame f;
    const float po[3] = {0.f, 0.f, d.height}, vx[3] = {d.radius, 0.f, 0.f}, vy[3] = {0.f, d.radius, 0.f},
                vz[3] = {0.f, 0.f, 1.f};
    d.o2w.point(po, f.o);
    d.o2w.vector(vx, f.x);
    d.o2w.vector(vy, f.y);
    d.o2w.vector(vz, f.z);
    normalize3(f.z);
    return f;
}

/* ------------------------------------------------------------ CudaRender */
/* PM_DEVICES="0,1,...": one context over those devices of the node
 * (pm_config::n_devices: photon shards, RCCL all-gather, 8-row bands per
 * device), so the plugin pbrt loads renders on the whole node; unset: the
 * one device given (PM_DEVICE in cudaapi.cpp). */
static std::vector<int> device_list_env() {
    std::vector<int> devs;
    const char *e = std::getenv("PM_DEVICES");
    if (!e) return devs;
    std::string s(e);
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        if (j > i) devs.push_back(std::atoi(s.substr(i, j - i).c_str()));
        i = j + 1;
    }
    return devs;
}

CudaRender::CudaRender(int device) {
    pm_config cfg{};
    cfg.device = device;
    const std::vector<int> devs = device_list_env();
    if (!devs.empty()) {
        cfg.n_devices = (int)devs.size();
        cfg.devices = devs.data();
    }
    if (pm_create(&ctx_, &cfg) != PM_OK) throw Error(std::string("pm_create: ") + pm_last_error(nullptr));
}

CudaRender::~CudaRender() {
    delete renderer_;
    pm_destroy(ctx_);
}

int CudaRender::materialId(const Material *m) {
    auto it = materials_.find(m);
    if (it != materials_.end()) return it->second;
    int type = PM_MATTE;
    float rgb[3] = {0.5f, 0.5f, 0.5f}; /* fallback matte 0.5 (cudamaterial.cpp:20,40) */
    if (m && m->kind != Material::Unknown) {
        type = m->kind == Material::Matte ? PM_MATTE : (m->kind == Material::Mirror ? PM_MIRROR : PM_GLASS);
        rgb[0] = m->k.r; rgb[1] = m->k.g; rgb[2] = m->k.b;
    }
    int id = -1;
    check(ctx_, pm_add_material(ctx_, type, rgb, &id), "pm_add_material");
    materials_[m] = id;
    return id;
}

void CudaRender::addPrim(const std::string &name, const Shape &s, int material, int lightIndex) {
    if (committed_) throw Error("shape added after the scene was committed");
    if (name == "trianglemesh") {
        const int nverts = (int)(s.P.size() / 3), ntris = (int)(s.indices.size() / 3);
        const float *N = s.N.size() == s.P.size() && !s.N.empty() ? s.N.data() : nullptr;
        const float *uv = s.uv.size() == 2 * (size_t)nverts && !s.uv.empty() ? s.uv.data() : nullptr;
        check(ctx_, pm_add_trimesh(ctx_, s.P.data(), nverts, s.indices.data(), ntris, N, uv, material, lightIndex),
              "pm_add_trimesh");
    } else if (name == "sphere") {
        check(ctx_, pm_add_sphere(ctx_, s.radius, s.o2w.m, s.o2w.minv, material, lightIndex), "pm_add_sphere");
    } else if (name == "disk") {
        const DiskFrame f = disk_frame(s);
        check(ctx_, pm_add_disk(ctx_, f.o, f.x, f.y, f.z, s.inner_radius / s.radius, s.phi_max, material, lightIndex),
              "pm_add_disk");
    } else {
        warning("shape:%s not implemented yet", name.c_str()); /* cudarender.cpp:141-144 */
    }
}

void CudaRender::createCudaShape(const std::string &name, const Shape &shape, const void *currentInstance,
                                 const Material *material, int lightIndex) {
    if (name != "trianglemesh" && name != "sphere" && name != "disk") {
        warning("shape:%s not implemented yet", name.c_str());
        return;
    }
    const int mat = materialId(material);
    if (currentInstance) { /* inside ObjectBegin/ObjectEnd: kept until instanced */
        instances_[currentInstance].push_back(Prim{name, shape, mat, lightIndex});
        return;
    }
    addPrim(name, shape, mat, lightIndex);
}

/* The reference places an OptiX Transform over the instance's group
 * (cudarender.cpp:88-103). Here a triangle mesh of the group is stored once
 * (pm_add_object_mesh, the first time the group is instanced) and each
 * instance adds a two-level entry with the transform (pm_add_mesh_instance),
 * whose hits equal those of the mesh flattened with this Transform (the
 * device rebuilds each world triangle exactly as Transform::point does).
 * Spheres and disks, and meshes under a projective transform, are flattened:
 * their transforms composed, the vertices / normals transformed here. env
 * PM_INSTANCING=0 flattens everything (the A/B of the two-level trees). */
void CudaRender::objectInstance(const void *instance, const Transform &tr) {
    auto it = instances_.find(instance);
    if (it == instances_.end()) throw Error("Instance not found"); /* cudarender.cpp:96-98 Severe */
    const char *env = std::getenv("PM_INSTANCING");
    const bool two_level = !(env && std::atoi(env) == 0) && tr.m[12] == 0.f && tr.m[13] == 0.f && tr.m[14] == 0.f &&
                           tr.m[15] == 1.f;
    for (size_t k = 0; k < it->second.size(); ++k) {
        const Prim &p = it->second[k];
        if (two_level && p.name == "trianglemesh") {
            if (committed_) throw Error("shape added after the scene was committed");
            auto ob = objects_.find({instance, k});
            if (ob == objects_.end()) {
                const Shape &s = p.shape;
                const int nverts = (int)(s.P.size() / 3), ntris = (int)(s.indices.size() / 3);
                const float *N = s.N.size() == s.P.size() && !s.N.empty() ? s.N.data() : nullptr;
                const float *uv = s.uv.size() == 2 * (size_t)nverts && !s.uv.empty() ? s.uv.data() : nullptr;
                int id = -1;
                check(ctx_, pm_add_object_mesh(ctx_, s.P.data(), nverts, s.indices.data(), ntris, N, uv, p.material,
                                               p.light, &id),
                      "pm_add_object_mesh");
                ob = objects_.emplace(std::make_pair(instance, k), id).first;
            }
            check(ctx_, pm_add_mesh_instance(ctx_, ob->second, tr.m, tr.minv), "pm_add_mesh_instance");
            continue;
        }
        Shape s = p.shape;
        if (p.name == "trianglemesh") {
            for (size_t v = 0; v + 2 < s.P.size(); v += 3) tr.point(&p.shape.P[v], &s.P[v]);
            for (size_t v = 0; v + 2 < s.N.size(); v += 3) tr.normal(&p.shape.N[v], &s.N[v]);
        } else {
            s.o2w = tr * p.shape.o2w;
        }
        addPrim(p.name, s, p.material, p.light);
    }
}

void CudaRender::createSubRenderer(const RenderSettings &settings, const std::string &rendername) {
    delete renderer_;
    renderer_ = nullptr;
    if (rendername == "simple") /* cudarender.cpp:126-134 */
        renderer_ = new SimpleRenderer(settings);
    else
        renderer_ = new PhotonMappingRenderer(settings);
}

/* CudaLight::setupLight (cudalight.cpp:16-59) */
void CudaRender::addLights(const std::vector<Light> &lights) {
    if (lights_added_) return;
    for (const Light &L : lights) {
        if (L.kind == Light::Point) {
            const float I[3] = {L.intensity.r, L.intensity.g, L.intensity.b};
            check(ctx_, pm_add_light_point(ctx_, L.pos, I), "pm_add_light_point");
        } else {
            const DiskFrame f = disk_frame(L.disk);
            float n[3] = {f.x[1] * f.y[2] - f.x[2] * f.y[1], f.x[2] * f.y[0] - f.x[0] * f.y[2],
                          f.x[0] * f.y[1] - f.x[1] * f.y[0]};
            normalize3(n);
            const float Le[3] = {L.Lemit.r, L.Lemit.g, L.Lemit.b};
            const float r = L.disk.radius, ri = L.disk.inner_radius;
            const float area = L.disk.phi_max * 0.5f * (r * r - ri * ri); /* pbrt Disk::Area */
            check(ctx_, pm_add_light_disk(ctx_, f.o, f.x, f.y, n, Le, area, L.n_samples < 1 ? 1 : L.n_samples),
                  "pm_add_light_disk");
        }
    }
    lights_added_ = true;
}

void CudaRender::commit() {
    if (committed_) return;
    check(ctx_, pm_commit(ctx_), "pm_commit");
    committed_ = true;
}

void CudaRender::Render(const std::vector<Light> &lights, Camera &camera) {
    if (!renderer_) throw Error("CreateCudaRenderer was not called");
    addLights(lights);
    commit();
    renderer_->render(this, lights, camera);
}

/* ------------------------------------------------------------ renderer */
static int64_t set_camera(void *ctx, const Camera &camera) {
    if (camera.pinhole) {
        check(ctx, pm_set_pinhole(ctx, camera.eye, camera.fwd, camera.right, camera.up, camera.width, camera.height),
              "pm_set_pinhole");
        return (int64_t)camera.width * camera.height;
    }
    const int64_t n = (int64_t)(camera.rays.size() / 6);
    check(ctx, pm_set_eye_rays(ctx, camera.rays.data(), n, camera.rand2d.empty() ? nullptr : camera.rand2d.data(),
                               camera.n2d),
          "pm_set_eye_rays");
    return n;
}

/* film splat (photonmappingrenderer.cpp:247-272, simplerender.cpp:68-89) */
static void splat(Camera &camera, const std::vector<float> &rgb, int64_t n) {
    if (!camera.film) return;
    for (int64_t i = 0; i < n; ++i) {
        CameraSample cs;
        if (camera.pinhole) {
            cs.imageX = (float)(i % camera.width) + 0.5f;
            cs.imageY = (float)(i / camera.width) + 0.5f;
        } else {
            cs = camera.samples.at((size_t)i);
        }
        camera.film->AddSample(cs, &rgb[3 * i]);
    }
    camera.film->WriteImage();
}

void SimpleRenderer::render(CudaRender *r, const std::vector<Light> &, Camera &camera) {
    void *ctx = r->context();
    const int64_t n = set_camera(ctx, camera);
    rgb.assign((size_t)(3 * n), 0.f);
    check(ctx, pm_render_simple(ctx, &settings.params, rgb.data(), &stats), "pm_render_simple");
    splat(camera, rgb, n);
}

void PhotonMappingRenderer::render(CudaRender *r, const std::vector<Light> &, Camera &camera) {
    void *ctx = r->context();
    const int64_t n = set_camera(ctx, camera);
    /* eye pass -> (photon pass -> photon map -> gather) x passes -> final
     * (photonmappingrenderer.cpp:31-45), NaN / negative / inf -> black */
    rgb.assign((size_t)(3 * n), 0.f);
    check(ctx, pm_render(ctx, &settings.params, rgb.data(), &stats), "pm_render");
    splat(camera, rgb, n);
}

/* ------------------------------------------------------------ cudaapi.h */
static CudaRender *g_render = nullptr;

void CudaRenderInit(int device) { g_render = new CudaRender(device); }

static CudaRender &global() {
    if (!g_render) throw Error("CudaRenderInit must precede all other calls");
    return *g_render;
}

void CreateCudaShape(const std::string &name, const Shape &shape, const void *currentInstance,
                     const Material *material, int lightIndex) {
    global().createCudaShape(name, shape, currentInstance, material, lightIndex);
}

void CudaObjectInstance(const void *key, const Transform &transform) { global().objectInstance(key, transform); }

CudaRender *CreateCudaRenderer(const RenderSettings &settings, const std::string &rendername) {
    CudaRender &r = global();
    r.createSubRenderer(settings, rendername);
    g_render = nullptr; /* ownership passes to the caller */
    return &r;
}

} // namespace pmcuda
