/*
 * pm_cudarender.h — C++ host layer of the MI355X photon mapper that mirrors
 * the reference's pbrt plugin surface (cuda_render/cudaapi.h:8-19 and
 * class CudaRender, cuda_render/cudarender.h:14-91) on top of the C-ABI in
 * include/pm_api.h. It is plain C++ (no HIP headers): every device action
 * goes through libpmhip.so.
 *
 * pbrt-v2 is not vendored with the reference, so this layer
 * takes plain descriptors of what the reference reads out of pbrt objects
 * (Shape, Material, Light, Transform, the camera's sample stream, Film). The
 * pbrt-side glue that fills them is a few lines per type; INTEGRATION.md
 * shows it.
 *
 *   reference (cudaapi.h / cudarender.h)          here
 *   -----------------------------------------------------------------------
 *   void CudaRenderInit()                         pmcuda::CudaRenderInit()
 *   void CreateCudaShape(name, shape, instance,   pmcuda::CreateCudaShape(name, Shape, instance key,
 *        material, lightIndex)                          Material*, lightIndex)
 *   void CudaObjectInstance(key, Transform)       pmcuda::CudaObjectInstance(key, Transform)
 *   Renderer* CreateCudaRenderer(sampler, camera, pmcuda::CreateCudaRenderer(RenderSettings, rendername)
 *        params, rendername)
 *   CudaRender::Render(const Scene*)              CudaRender::Render(lights, Camera&)
 *   CudaRenderer::render(scene, render, camera)   CudaRenderer::render(CudaRender*, lights, Camera&)
 *
 * Error convention follows the reference (cudarender.cpp:141-144,
 * cudalight.cpp:54-55,68, cudamaterial.cpp:20): unsupported shapes / lights
 * warn and are skipped, unknown materials fall back to matte 0.5; fatal
 * errors (no device, failed render) throw pmcuda::Error instead of pbrt's
 * Severe() abort, so a host application can decide.
 */
#pragma once

#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/pm_api.h"

namespace pmcuda {

struct Error : std::runtime_error {
    explicit Error(const std::string &m) : std::runtime_error(m) {}
};

/* pbrt Transform: row-major Matrix4x4 m and its inverse (Transform::GetMatrix /
 * GetInverseMatrix, as cudarender.cpp:100 passes them to OptiX). */
struct Transform {
    float m[16];
    float minv[16];
    static Transform identity();
    static Transform translate(float x, float y, float z);
    static Transform rotate_x(float degrees);
    Transform operator*(const Transform &b) const; /* pbrt composition: (this * b)(p) = this(b(p)) */
    void point(const float in[3], float out[3]) const;
    void vector(const float in[3], float out[3]) const;
    void normal(const float in[3], float out[3]) const; /* inverse transpose */
};

struct RGB { float r, g, b; };

/* what CudaMaterial::createCudaMeteral reads (cudamaterial.cpp:8-75): the
 * Kd / Kr texture evaluated at a default DifferentialGeometry */
struct Material {
    enum Kind { Matte, Mirror, Glass, Unknown } kind = Matte;
    RGB k = {0.5f, 0.5f, 0.5f};
};

/* what CudaShape::CreateCudaShape reads from a pbrt Shape:
 *  "trianglemesh": world-space P (pbrt TriangleMesh::p is world space,
 *                  cudatrianglemesh.cpp:24-30), vertexIndex, optional n, uv
 *  "sphere":       radius + ObjectToWorld        (cudasphere.cpp:15-40)
 *  "disk":         height, radius, innerRadius, phiMax (radians) + ObjectToWorld
 *                  (cudadisk.cpp:15-45) */
struct Shape {
    std::vector<float> P, N, uv;
    std::vector<int> indices;
    Transform o2w = Transform::identity();
    float radius = 1.f, height = 0.f, inner_radius = 0.f, phi_max = 6.28318530717958647692f;
};

/* pbrt lights as CudaLight::setupLight flattens them (cudalight.cpp:16-59):
 * PointLight, or DiffuseAreaLight over disk shapes. */
struct Light {
    enum Kind { Point, AreaDisk } kind = Point;
    float pos[3] = {0, 0, 0}; /* Point */
    RGB intensity = {0, 0, 0};
    Shape disk;               /* AreaDisk: the disk shape (radius, height, o2w) */
    RGB Lemit = {0, 0, 0};
    int n_samples = 1;
};

/* ParamSet of the renderer + the reference's hard-coded constants (see
 * pm_render_params for where each comes from) */
struct RenderSettings {
    pm_render_params params;
    RenderSettings() { pm_default_params(&params); }
};

/* pbrt CameraSample fields Film::AddSample uses */
struct CameraSample { float imageX, imageY; };

struct Film {
    virtual void AddSample(const CameraSample &s, const float rgb[3]) = 0;
    virtual void WriteImage() {}
    virtual ~Film() {}
};

/* CudaCamera (util/camera/cudacamera.h): the eye samples of one render.
 * pinhole: a synthetic camera evaluated on the device (one sample per pixel
 * centre); otherwise rays in sampler order as PbrtCamera::preLaunch packs
 * them (o.xyz, d.xyz), their light 2D randoms and camera samples. */
struct Camera {
    bool pinhole = true;
    float eye[3] = {0, 0, 0}, fwd[3] = {0, 0, 1}, right[3] = {1, 0, 0}, up[3] = {0, 1, 0};
    int width = 0, height = 0;
    std::vector<float> rays, rand2d;
    int n2d = 0;
    std::vector<CameraSample> samples;
    Film *film = nullptr;
};

class CudaRender;

/* strategy interface (cudarender.h:14-19) */
class CudaRenderer {
public:
    virtual void render(CudaRender *render, const std::vector<Light> &lights, Camera &camera) = 0;
    virtual ~CudaRenderer() {}
};

/* PhotonMappingRenderer (photon_mapping/photonmappingrenderer.cpp:31-45):
 * eye pass -> (photon trace -> photon map -> gather) x passes -> final -> splat */
class PhotonMappingRenderer : public CudaRenderer {
public:
    explicit PhotonMappingRenderer(const RenderSettings &s) : settings(s) {}
    void render(CudaRender *render, const std::vector<Light> &lights, Camera &camera) override;
    RenderSettings settings;
    pm_stats stats{};
    std::vector<float> rgb; /* last output: per sample (rays) or raster (pinhole) */
};

/* SimpleRenderer (simple_render/simplerender.cpp:18-103): direct light only,
 * scene_epsilon 0.01 (simplerender.cpp:23) -> pm_render_simple -> splat */
class SimpleRenderer : public CudaRenderer {
public:
    explicit SimpleRenderer(const RenderSettings &s) : settings(s) {
        settings.params.scene_epsilon = PM_SIMPLE_SCENE_EPSILON;
    }
    void render(CudaRender *render, const std::vector<Light> &lights, Camera &camera) override;
    RenderSettings settings;
    pm_stats stats{};
    std::vector<float> rgb;
};

class CudaRender {
public:
    explicit CudaRender(int device = 0);
    ~CudaRender();
    CudaRender(const CudaRender &) = delete;
    CudaRender &operator=(const CudaRender &) = delete;

    void createCudaShape(const std::string &name, const Shape &shape, const void *currentInstance,
                         const Material *material, int lightIndex);
    void objectInstance(const void *instance, const Transform &tr);
    void createSubRenderer(const RenderSettings &settings, const std::string &rendername);
    /* Renderer::Render(scene): lights come from pbrt's scene->lights */
    void Render(const std::vector<Light> &lights, Camera &camera);

    void *context() const { return ctx_; }
    CudaRenderer *subRenderer() const { return renderer_; }
    int materialId(const Material *m); /* dedupe per pbrt Material* (cudarender.cpp:181-192) */
    /* lights must be added before the first render; called by the renderer */
    void addLights(const std::vector<Light> &lights);
    void commit();

private:
    struct Prim {
        std::string name;
        Shape shape;
        int material;
        int light;
    };
    void addPrim(const std::string &name, const Shape &shape, int material, int lightIndex);

    void *ctx_ = nullptr;
    CudaRenderer *renderer_ = nullptr;
    std::map<const Material *, int> materials_;
    std::map<const void *, std::vector<Prim>> instances_; /* pbrt ObjectBegin ... ObjectEnd */
    /* the object meshes already stored (pm_add_object_mesh) per (instance key, prim) */
    std::map<std::pair<const void *, size_t>, int> objects_;
    bool committed_ = false;
    bool lights_added_ = false;
};

/* ---- cudaapi.h free functions (process-global renderer, cudaapi.cpp:3-26) ---- */
void CudaRenderInit(int device = 0);
void CreateCudaShape(const std::string &name, const Shape &shape, const void *currentInstance,
                     const Material *material, int lightIndex);
void CudaObjectInstance(const void *key, const Transform &transform);
/* returns the global CudaRender with its sub-renderer set; ownership passes
 * to the caller as in cudaapi.cpp:22-26 (pbrt deletes its Renderer) */
CudaRender *CreateCudaRenderer(const RenderSettings &settings, const std::string &rendername);

} // namespace pmcuda
