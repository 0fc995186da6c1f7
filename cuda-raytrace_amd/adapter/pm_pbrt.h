/*
 * pm_pbrt.h — a pbrt-v2 scene-file front end for the pbrt-facing layer
 * (pm_cudarender.h). SURVEY.md §8f row 3: the reference is loaded by a pbrt-v2
 * fork whose api.cpp turns scene directives into CudaRenderInit /
 * CreateCudaShape / CudaObjectInstance / CreateCudaRenderer calls
 * (cuda_render/cudaapi.h:8-19). pbrt-v2 is not vendored, so this
 * parser restates the part of pbrt-v2's api.cpp + parser that the plugin sees:
 *
 *   transforms   Identity Translate Scale Rotate LookAt Transform ConcatTransform
 *                CoordinateSystem CoordSysTransform TransformBegin/End
 *   state        WorldBegin/End AttributeBegin/End ReverseOrientation
 *                Material MakeNamedMaterial NamedMaterial Texture (constant)
 *   lights       LightSource "point" (I, scale, from), AreaLightSource "diffuse"
 *                (L, scale, nsamples) on the following shapes
 *   shapes       Shape "trianglemesh" (P in world space as pbrt's TriangleMesh
 *                stores it; N / uv raw), "sphere", "disk"; anything else goes
 *                to CreateCudaShape, which warns and skips it like
 *                cudarender.cpp:141-144
 *   instancing   ObjectBegin/ObjectEnd/ObjectInstance
 *   options      Camera "perspective" (fov, frameaspectratio, screenwindow),
 *                Film (xresolution, yresolution, filename), Renderer
 *                ("photonmapping" | "simple" | "cuda" + "string rendername";
 *                extension params "integer paths", "integer passes",
 *                "string gather" = "grid" | "kdtree")
 *                Sampler / PixelFilter / *Integrator / Accelerator: accepted, ignored
 *   Include      relative to the including file
 *
 * Semantics follow pbrt-v2: float transforms with pbrt's Rotate / LookAt
 * formulas, post-multiplied onto the CTM; CTM reset at WorldBegin; the camera
 * is Inverse(CTM) at the Camera directive; PointLight position =
 * light-to-world(0) + "from" (pbrt-v2 builds Translate(from) * light2world);
 * materials default to pbrt's (matte Kd 0.5, mirror Kr 0.9); unknown
 * material types become the reference's fallback matte 0.5
 * (cudamaterial.cpp:20,40). The camera is evaluated on the device as a
 * pinhole through the pixel centres (pm_set_pinhole).
 */
#pragma once

#include <string>
#include <vector>

#include "pm_cudarender.h"

namespace pmcuda {

/* Receiver of the plugin calls the scene file produces (the pbrt-v2 api.cpp
 * -> cudaapi.h boundary). The default sink forwards to CreateCudaShape /
 * CudaObjectInstance; a test sink can record them. */
struct PbrtSink {
    virtual void shape(const std::string &name, const Shape &shape, const void *instance, const Material *material,
                       int lightIndex) = 0;
    virtual void objectInstance(const void *key, const Transform &tr) = 0;
    virtual ~PbrtSink() {}
};

struct CudaApiSink : PbrtSink {
    void shape(const std::string &name, const Shape &s, const void *instance, const Material *m, int li) override {
        CreateCudaShape(name, s, instance, m, li);
    }
    void objectInstance(const void *key, const Transform &tr) override { CudaObjectInstance(key, tr); }
};

/* Everything outside the world block that the render needs. */
struct PbrtOptions {
    std::vector<Light> lights;   /* pbrt scene->lights order (point + area, declaration order) */
    Camera camera;               /* pinhole: eye, fwd, right, up, width, height */
    std::string renderer = "photonmapping";
    RenderSettings settings;     /* params from the Renderer directive */
    std::string film_filename = "pbrt.pfm";
    int warnings = 0;
};

/* Parses `path` (and its Includes), issuing shapes / instances to `sink`.
 * Materials referenced by issued shapes stay alive as long as the parser
 * object does. Throws pmcuda::Error with file:line on malformed input. */
class PbrtParser {
public:
    PbrtParser();
    ~PbrtParser();
    PbrtParser(const PbrtParser &) = delete;
    PbrtParser &operator=(const PbrtParser &) = delete;
    void parseFile(const std::string &path, PbrtSink &sink, PbrtOptions &opts);
    void parseString(const std::string &text, PbrtSink &sink, PbrtOptions &opts, const std::string &dir = ".");

private:
    struct Impl;
    Impl *impl_;
};

} // namespace pmcuda
