/*
 * cudarender.h — class CudaRender : public Renderer, the reference's pbrt
 * Renderer (cuda_render/cudarender.h:22-33), over the C-ABI: only Render does
 * work, Li / Transmittance return black as in the reference. The scene graph
 * calls (createCudaShape, objectInstance, createSubRenderer) convert pbrt
 * objects into the plain descriptors of the host layer (pm_cudarender.h),
 * reading the members the reference reads.
 */
#ifndef cudarender_h__
#define cudarender_h__

#include <map>
#include <string>
#include <vector>

#include "core/camera.h"
#include "core/light.h"
#include "core/material.h"
#include "core/memory.h"
#include "core/paramset.h"
#include "core/pbrt.h"
#include "core/primitive.h"
#include "core/renderer.h"
#include "core/sampler.h"
#include "core/scene.h"
#include "core/spectrum.h"
#include "pm_cudarender.h"

class CudaRender : public Renderer {
public:
    CudaRender();
    ~CudaRender();
    /* cudarender.h:26, cudarender.cpp:112-123: assemble the scene, upload the
     * camera's samples (PbrtCamera::preLaunch), run the sub-renderer, splat
     * through camera->film->AddSample and write the image */
    virtual void Render(const Scene *scene);
    virtual Spectrum Li(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                        MemoryArena &arena, Intersection *isect = NULL, Spectrum *T = NULL) const {
        return Spectrum(0.f);
    }
    virtual Spectrum Transmittance(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                                   MemoryArena &arena) const {
        return Spectrum(0.f);
    }

    void objectInstance(std::vector<Reference<Primitive> > *instance, const Transform &tr);
    void createCudaShape(const std::string &name, Reference<Shape> &shape,
                         std::vector<Reference<Primitive> > *currentInstance, const Material *kMaterial,
                         int lightIndex);
    void createSubRenderer(Sampler *sampler, Camera *camera, const ParamSet &params, const std::string &rendername);

    /* the host layer underneath (context, statistics of the last render) */
    pmcuda::CudaRender &impl() { return impl_; }

private:
    const pmcuda::Material *material(const Material *m);
    pmcuda::CudaRender impl_;
    std::map<const Material *, pmcuda::Material> materials_; /* cudarender.h:74-76 */
    Sampler *sampler_;
    Camera *camera_;
};

#endif // cudarender_h__
