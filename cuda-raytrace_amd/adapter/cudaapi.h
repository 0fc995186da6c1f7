/*
 * cudaapi.h — the reference's pbrt plugin entry points, with its exact
 * signatures (cuda_render/cudaapi.h:8-19). pbrt-v2's api.cpp (the fork)
 * includes this after its own headers; here the pbrt types come from the
 * pbrt-v2 tree on the include path (adapter/pbrt_stub in this repository).
 * Implemented in cudaapi.cpp over the C-ABI (include/pm_api.h).
 */
#ifndef cudaapi_h__
#define cudaapi_h__

#include <string>
#include <vector>

#include "core/camera.h"
#include "core/paramset.h"
#include "core/pbrt.h"
#include "core/primitive.h"
#include "core/renderer.h"
#include "core/sampler.h"
#include "core/shape.h"
#include "core/transform.h"

/* cudaapi.h:8-10 — MakeRenderer("cuda"): the process-global CudaRender with
 * the sub-renderer `rendername` ("simple" or the photon mapper); pbrt owns
 * (and deletes) the returned Renderer, the sub-renderer owns sampler and
 * camera (photonmappingrenderer.cpp:25-29) */
Renderer *CreateCudaRenderer(Sampler *sampler, Camera *camera, const ParamSet &params, const std::string &rendername);

/* cudaapi.h:12 — pbrtInit(): before any other call */
void CudaRenderInit();

/* cudaapi.h:14-16 — pbrtShape(): one call per Shape directive; lightIndex =
 * the area light's index in scene->lights, -1 for plain geometry;
 * currentInstance = RenderOptions::currentInstance inside ObjectBegin/End */
void CreateCudaShape(const std::string &name, Reference<Shape> &shape,
                     std::vector<Reference<Primitive> > *currentInstance, const Material *material, int lightIndex);

/* cudaapi.h:18-19 — pbrtObjectInstance(): the instance's world transform */
void CudaObjectInstance(std::vector<Reference<Primitive> > *key, const Transform &transform);

#endif // cudaapi_h__
