/*
 * cudaapi.cpp — the reference's pbrt plugin surface (cuda_render/cudaapi.cpp,
 * cudarender.cpp:105-196, util/shape/cuda{trianglemesh,sphere,disk}.cpp, util/light/cudalight.cpp:16-59,
 * util/material/cudamaterial.cpp:8-58, util/camera/pbrtcamera.cpp:57-122,
 * photonmappingrenderer.cpp:234-283) with pbrt-v2 types at the boundary and
 * the MI355X renderer underneath: pbrt objects are read exactly where the
 * reference reads them and handed to the C++ host layer (pm_cudarender.h),
 * which drives the C-ABI (include/pm_api.h). No HIP or OptiX header here.
 */
#include "cudaapi.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "core/film.h"
#include "cudarender.h"
#include "lights/diffuse.h"
#include "lights/point.h"
#include "materials/glass.h"
#include "materials/matte.h"
#include "materials/mirror.h"
#include "shapes/disk.h"
#include "shapes/sphere.h"
#include "shapes/trianglemesh.h"

/* ---------------------------------------------------------------- pbrt -> descriptors */
static pmcuda::Transform toPm(const Transform &t) {
    pmcuda::Transform r;
    std::memcpy(r.m, &t.GetMatrix().m[0][0], sizeof r.m);
    std::memcpy(r.minv, &t.GetInverseMatrix().m[0][0], sizeof r.minv);
    return r;
}

static pmcuda::RGB toPm(const Spectrum &s) {
    float c[3];
    s.ToRGB(c);
    return pmcuda::RGB{c[0], c[1], c[2]};
}

/* what CudaShape::CreateCudaShape reads: the world-space triangle mesh
 * (cudatrianglemesh.cpp:18-66), the sphere's radius and transforms
 * (cudasphere.cpp:17-29), the disk's height / radii / phiMax and
 * ObjectToWorld (cudadisk.cpp:17-35). false: a shape the reference skips. */
static bool toPm(const Shape *s, pmcuda::Shape &d) {
    if (const TriangleMesh *tm = dynamic_cast<const TriangleMesh *>(s)) {
        d.P.resize(3 * (size_t)tm->nverts);
        for (int i = 0; i < tm->nverts; ++i) {
            d.P[3 * i] = tm->p[i].x; d.P[3 * i + 1] = tm->p[i].y; d.P[3 * i + 2] = tm->p[i].z;
        }
        d.indices.assign(tm->vertexIndex, tm->vertexIndex + 3 * (size_t)tm->ntris);
        if (tm->n) { /* copied raw, object-space pbrt normals (cudatrianglemesh.cpp:46-51) */
            d.N.resize(3 * (size_t)tm->nverts);
            for (int i = 0; i < tm->nverts; ++i) {
                d.N[3 * i] = tm->n[i].x; d.N[3 * i + 1] = tm->n[i].y; d.N[3 * i + 2] = tm->n[i].z;
            }
        }
        if (tm->uvs) d.uv.assign(tm->uvs, tm->uvs + 2 * (size_t)tm->nverts);
        return true;
    }
    if (const Sphere *sp = dynamic_cast<const Sphere *>(s)) {
        d.radius = sp->radius;
        d.o2w = toPm(*sp->ObjectToWorld);
        return true;
    }
    if (const Disk *dk = dynamic_cast<const Disk *>(s)) {
        d.radius = dk->radius;
        d.height = dk->height;
        d.inner_radius = dk->innerRadius;
        d.phi_max = dk->phiMax;
        d.o2w = toPm(*dk->ObjectToWorld);
        return true;
    }
    return false;
}

/* ---------------------------------------------------------------- CudaRender */
static int device_ordinal() {
    const char *e = std::getenv("PM_DEVICE");
    return e ? std::atoi(e) : 0;
}

CudaRender::CudaRender() : impl_(device_ordinal()), sampler_(NULL), camera_(NULL) {}

CudaRender::~CudaRender() { /* the sub-renderer's pbrt objects (photonmappingrenderer.cpp:25-29) */
    delete sampler_;
    delete camera_;
}

/* CudaMaterial::createCudaMeteral (cudamaterial.cpp:8-21): Kd / Kr evaluated
 * at a default DifferentialGeometry; anything else is matte 0.5 */
const pmcuda::Material *CudaRender::material(const Material *m) {
    auto it = materials_.find(m);
    if (it != materials_.end()) return &it->second;
    pmcuda::Material d;
    DifferentialGeometry dg;
    if (const MatteMaterial *mm = dynamic_cast<const MatteMaterial *>(m)) {
        d.kind = pmcuda::Material::Matte;
        d.k = toPm(mm->Kd->Evaluate(dg));
    } else if (const MirrorMaterial *mi = dynamic_cast<const MirrorMaterial *>(m)) {
        d.kind = pmcuda::Material::Mirror;
        d.k = toPm(mi->Kr->Evaluate(dg));
    } else if (dynamic_cast<const GlassMaterial *>(m)) {
        d.kind = pmcuda::Material::Glass;
        d.k = pmcuda::RGB{1.f, 1.f, 1.f};
    } else {
        d.kind = pmcuda::Material::Unknown;
    }
    return &(materials_[m] = d);
}

void CudaRender::createCudaShape(const std::string &name, Reference<Shape> &shape,
                                 std::vector<Reference<Primitive> > *currentInstance, const Material *kMaterial,
                                 int lightIndex) {
    pmcuda::Shape d;
    if (!toPm(shape.GetPtr(), d)) {
        Warning("shape:%s not implemented yet", name.c_str()); /* cudarender.cpp:141-144 */
        return;
    }
    try {
        impl_.createCudaShape(name, d, currentInstance, material(kMaterial), lightIndex);
    } catch (const pmcuda::Error &e) {
        Severe("%s", e.what());
    }
}

void CudaRender::objectInstance(std::vector<Reference<Primitive> > *instance, const Transform &tr) {
    try {
        impl_.objectInstance(instance, toPm(tr));
    } catch (const pmcuda::Error &e) {
        Severe("%s", e.what());
    }
}

void CudaRender::createSubRenderer(Sampler *sampler, Camera *camera, const ParamSet &params,
                                   const std::string &rendername) {
    sampler_ = sampler;
    camera_ = camera;
    /* the reference hard-codes its constants (pm_render_params defaults);
     * the ParamSet may scale the photon pass, which the reference cannot */
    pmcuda::RenderSettings s;
    s.params.paths_per_pass = params.FindOneInt("photonpaths", (int)s.params.paths_per_pass);
    s.params.passes = params.FindOneInt("passes", s.params.passes);
    if (params.FindOneString("photonmap", "grid") == "kdtree") s.params.gather_structure = PM_GATHER_KDTREE;
    impl_.createSubRenderer(s, rendername);
}

/* Film::AddSample of each eye sample in sampler order, with the reference's
 * host-side sanitising (photonmappingrenderer.cpp:247-272) */
namespace {
struct PbrtFilm : pmcuda::Film {
    ::Film *film;
    const std::vector<CameraSample> *samples;
    size_t next = 0;
    void AddSample(const pmcuda::CameraSample &, const float rgb[3]) override {
        Spectrum result = RGBSpectrum::FromRGB(rgb);
        if (result.HasNaNs()) {
            Error("Not-a-number radiance value returned for image sample.  Setting to black.");
            result = Spectrum(0.f);
        } else if (result.y() < -1e-5f) {
            Error("Negative luminance value, %f, returned for image sample.  Setting to black.", result.y());
            result = Spectrum(0.f);
        } else if (std::isinf(result.y())) {
            Error("Infinite luminance value returned for image sample.  Setting to black.");
            result = Spectrum(0.f);
        }
        film->AddSample((*samples)[next++], result);
    }
    void WriteImage() override { film->WriteImage(); } /* PhotonMappingRenderer::postLaunch */
};
} // namespace

void CudaRender::Render(const Scene *scene) {
    if (!camera_ || !sampler_) Severe("CreateCudaRenderer must precede Render");
    /* lights (CudaLight::preLaunch, cudalight.cpp:105-120): point lights, and
     * the disks of diffuse area lights, each with its 2D light samples
     * registered in sampler order (CudaSample::Add2D rounds the count) */
    std::vector<pmcuda::Light> lights;
    Sample proto(NULL, NULL, NULL, scene);
    uint32_t n2d = 0;
    for (Light *l : scene->lights) {
        if (PointLight *pl = dynamic_cast<PointLight *>(l)) {
            pmcuda::Light L;
            L.kind = pmcuda::Light::Point;
            L.pos[0] = pl->lightPos.x; L.pos[1] = pl->lightPos.y; L.pos[2] = pl->lightPos.z;
            L.intensity = toPm(pl->Intensity);
            lights.push_back(L);
        } else if (DiffuseAreaLight *al = dynamic_cast<DiffuseAreaLight *>(l)) {
            uint32_t samplePerShape = (uint32_t)std::max(1, al->nSamples);
            for (const Reference<Shape> &s : al->shapeSet->shapes) {
                if (const Disk *disk = dynamic_cast<const Disk *>(s.GetPtr())) {
                    samplePerShape = (uint32_t)sampler_->RoundSize((int)samplePerShape);
                    proto.Add2D(samplePerShape);
                    n2d += samplePerShape;
                    pmcuda::Light L;
                    L.kind = pmcuda::Light::AreaDisk;
                    toPm(disk, L.disk);
                    L.Lemit = toPm(al->Lemit);
                    L.n_samples = (int)samplePerShape;
                    lights.push_back(L);
                } else {
                    Warning("UnImplemented Cuda Area Light Source");
                }
            }
        } else {
            Warning("UnImplemented Cuda Light Source");
        }
    }
    /* the eye samples (PbrtCamera::preLaunch, pbrtcamera.cpp:57-122): the
     * sampler's stream in its own order, rays with differentials scaled by
     * 1/sqrt(spp), the light 2D randoms of each sample */
    int xs, xe, ys, ye;
    camera_->film->GetSampleExtent(&xs, &xe, &ys, &ye);
    const int spp = sampler_->samplesPerPixel;
    const int64_t maximal = (int64_t)(xe - xs) * (ye - ys) * spp;
    const int maxSamples = sampler_->MaximumSampleCount();
    Sample *samples = proto.Duplicate(maxSamples);
    RNG rng;
    pmcuda::Camera cam;
    cam.pinhole = false;
    cam.n2d = (int)n2d;
    std::vector<CameraSample> csamples;
    int count;
    while ((count = sampler_->GetMoreSamples(samples, rng)) > 0) {
        for (int i = 0; i < count; ++i) {
            if ((int64_t)csamples.size() >= maximal) Severe("Too many samples. expect:%lld", (long long)maximal);
            RayDifferential rd;
            camera_->GenerateRayDifferential(samples[i], &rd);
            rd.ScaleDifferentials(1.f / std::sqrt((float)spp));
            cam.rays.insert(cam.rays.end(), {rd.o.x, rd.o.y, rd.o.z, rd.d.x, rd.d.y, rd.d.z});
            if (n2d) cam.rand2d.insert(cam.rand2d.end(), samples[i].twoD[0], samples[i].twoD[0] + 2 * n2d);
            csamples.push_back(samples[i]);
            cam.samples.push_back(pmcuda::CameraSample{samples[i].imageX, samples[i].imageY});
        }
    }
    delete[] samples;
    if ((int64_t)csamples.size() != maximal) Warning("pbrt camera do not generate enough samples");
    PbrtFilm film;
    film.film = camera_->film;
    film.samples = &csamples;
    cam.film = &film;
    try {
        impl_.Render(lights, cam);
    } catch (const pmcuda::Error &e) {
        Severe("%s", e.what());
    }
}

/* ---------------------------------------------------------------- cudaapi.cpp:3-26 */
static CudaRender *cudaRender = NULL;

void CudaRenderInit() {
    try {
        cudaRender = new CudaRender();
    } catch (const pmcuda::Error &e) {
        Severe("%s", e.what());
    }
}

void CreateCudaShape(const std::string &name, Reference<Shape> &shape,
                     std::vector<Reference<Primitive> > *currentInstance, const Material *material, int lightIndex) {
    if (!cudaRender) Severe("CudaRenderInit must precede CreateCudaShape");
    cudaRender->createCudaShape(name, shape, currentInstance, material, lightIndex);
}

void CudaObjectInstance(std::vector<Reference<Primitive> > *key, const Transform &transform) {
    if (!cudaRender) Severe("CudaRenderInit must precede CudaObjectInstance");
    cudaRender->objectInstance(key, transform);
}

Renderer *CreateCudaRenderer(Sampler *sampler, Camera *camera, const ParamSet &params,
                             const std::string &rendername) {
    if (!cudaRender) Severe("CudaRenderInit must precede CreateCudaRenderer");
    cudaRender->createSubRenderer(sampler, camera, params, rendername);
    return cudaRender;
}
