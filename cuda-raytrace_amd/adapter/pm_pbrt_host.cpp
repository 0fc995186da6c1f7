/*
 * pm_pbrt_host.cpp — a pbrt-v2-shaped host for the plugin boundary: it makes
 * the calls pbrt-v2's api.cpp (the reference's fork) makes, in its order,
 * with pbrt objects (adapter/pbrt_stub):
 *   pbrtInit            -> CudaRenderInit()
 *   Shape directives    -> CreateCudaShape(name, Reference<Shape>, currentInstance, Material*, areaLightIndex)
 *   ObjectInstance      -> CudaObjectInstance(&instance, Transform)
 *   MakeRenderer "cuda" -> CreateCudaRenderer(sampler, camera, ParamSet, rendername)
 *   pbrtWorldEnd        -> renderer->Render(scene); delete renderer
 * for the Cornell box of pmrender/scenes.py, with a one-sample-per-pixel
 * sampler (pixel centres, raster order; light 2D randoms from a fixed hash),
 * a pinhole camera and a film that keeps what Film::AddSample receives. The
 * rays, light randoms and film image go to a binary file, so a test can
 * render the same inputs through the stage driver and compare bit for bit.
 *
 * usage: pm_pbrt_host --out f.bin [--width W --height H --paths N
 *        --photonmap grid|kdtree --renderer photonmap|simple --nsamples S --instanced]
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "core/film.h"
#include "cudaapi.h"
#include "lights/diffuse.h"
#include "materials/matte.h"
#include "shapes/disk.h"
#include "shapes/trianglemesh.h"

namespace {

struct Opts {
    int W = 64, H = 48, paths = 16384, nsamples = 1;
    std::string photonmap = "grid", renderer = "photonmap", out;
    bool instanced = false;
};

/* pixel centres in raster order, one sample per pixel; light 2D randoms:
 * a fixed integer hash of (pixel, dimension) */
class CentreSampler : public Sampler {
public:
    CentreSampler(int W, int H) : Sampler(0, W, 0, H, 1, 0.f, 1.f), next(0), W_(W), H_(H) {}
    int GetMoreSamples(Sample *sample, RNG &) {
        if (next >= W_ * H_) return 0;
        const int x = next % W_, y = next / W_;
        sample->imageX = (float)x + 0.5f;
        sample->imageY = (float)y + 0.5f;
        sample->lensU = sample->lensV = 0.5f;
        sample->time = 0.f;
        for (size_t d = 0; d < sample->n2D.size(); ++d)
            for (uint32_t k = 0; k < 2 * sample->n2D[d]; ++k) {
                sample->twoD[d][k] = hash01((uint32_t)next * 977u + (uint32_t)(d * 64 + k));
                rand2d.push_back(sample->twoD[d][k]);
            }
        ++next;
        return 1;
    }
    int MaximumSampleCount() { return 1; }
    int RoundSize(int size) const { return size; }
    std::vector<float> rand2d; /* every light 2D random handed out, in sample order */
private:
    static float hash01(uint32_t v) {
        v ^= v >> 16; v *= 0x7feb352du; v ^= v >> 15; v *= 0x846ca68bu; v ^= v >> 16;
        return (float)(v >> 8) * (1.f / 16777216.f);
    }
    int next, W_, H_;
};

/* the pinhole of pmrender/scenes.py pinhole(): eye (278, 273, -800) looking
 * +z, fov 39.3 deg over the shorter axis, image x towards -x world */
class PinholeCamera : public Camera {
public:
    PinholeCamera(Film *f, int W, int H) : Camera(f), W_(W), H_(H) {
        const double t = std::tan(39.3 * M_PI / 180.0 / 2.0);
        sx = (float)(W >= H ? t * W / H : t);
        sy = (float)(W >= H ? t : t * H / W);
    }
    float GenerateRay(const CameraSample &cs, Ray *ray) const {
        const float u = 2.f * cs.imageX / (float)W_ - 1.f, v = 1.f - 2.f * cs.imageY / (float)H_;
        Vector d(-u * sx, v * sy, 1.f);
        ray->o = Point(278.f, 273.f, -800.f);
        ray->d = Normalize(d);
        return 1.f;
    }
private:
    int W_, H_;
    float sx, sy;
};

class KeepFilm : public Film {
public:
    KeepFilm(int W, int H) : Film(W, H), rgb(3 * (size_t)W * H, 0.f) {}
    void AddSample(const CameraSample &s, const Spectrum &L) {
        const int x = (int)std::floor(s.imageX), y = (int)std::floor(s.imageY);
        if (x < 0 || y < 0 || x >= xResolution || y >= yResolution) return;
        float c[3];
        L.ToRGB(c);
        std::memcpy(&rgb[3 * ((size_t)y * xResolution + x)], c, sizeof c);
        ++added;
    }
    void GetSampleExtent(int *xs, int *xe, int *ys, int *ye) const { *xs = 0; *xe = xResolution; *ys = 0; *ye = yResolution; }
    void WriteImage(float) { ++written; }
    std::vector<float> rgb;
    long added = 0;
    int written = 0;
};

/* records the rays the renderer asked for (for the stage-driver comparison) */
class RecordingCamera : public PinholeCamera {
public:
    using PinholeCamera::PinholeCamera;
    float GenerateRayDifferential(const CameraSample &cs, RayDifferential *rd) const {
        const float w = PinholeCamera::GenerateRayDifferential(cs, rd);
        rays.insert(rays.end(), {rd->o.x, rd->o.y, rd->o.z, rd->d.x, rd->d.y, rd->d.z});
        return w;
    }
    mutable std::vector<float> rays;
};

Reference<Texture<Spectrum> > constant(float r, float g, float b) {
    const float c[3] = {r, g, b};
    return Reference<Texture<Spectrum> >(new ConstantTexture<Spectrum>(RGBSpectrum::FromRGB(c)));
}

Reference<Shape> quads(const Transform *o2w, const std::vector<std::vector<float> > &qs) {
    std::vector<Point> P;
    std::vector<int> idx;
    for (const std::vector<float> &q : qs) {
        const int b = (int)P.size();
        for (int k = 0; k < 4; ++k) P.push_back(Point(q[3 * k], q[3 * k + 1], q[3 * k + 2]));
        idx.insert(idx.end(), {b, b + 1, b + 2, b, b + 2, b + 3});
    }
    return Reference<Shape>(new TriangleMesh(o2w, o2w, false, (int)idx.size() / 3, (int)P.size(), idx.data(), P.data(),
                                             NULL, NULL, NULL));
}

int run(const Opts &o) {
    static const Transform identity;
    /* pbrtInit */
    CudaRenderInit();
    Reference<Material> white(new MatteMaterial(constant(0.73f, 0.73f, 0.73f), NULL, NULL));
    Reference<Material> red(new MatteMaterial(constant(0.63f, 0.065f, 0.05f), NULL, NULL));
    Reference<Material> green(new MatteMaterial(constant(0.14f, 0.45f, 0.091f), NULL, NULL));
    Reference<Material> black(new MatteMaterial(constant(0.f, 0.f, 0.f), NULL, NULL));
    /* WorldBegin ... Shape directives (pmrender/scenes.py cornell_box order) */
    Reference<Shape> s;
    s = quads(&identity, {{552.8f, 0, 0, 0, 0, 0, 0, 0, 559.2f, 549.6f, 0, 559.2f},
                          {556.0f, 548.8f, 0, 556.0f, 548.8f, 559.2f, 0, 548.8f, 559.2f, 0, 548.8f, 0},
                          {549.6f, 0, 559.2f, 0, 0, 559.2f, 0, 548.8f, 559.2f, 556.0f, 548.8f, 559.2f}});
    CreateCudaShape("trianglemesh", s, NULL, white.GetPtr(), -1);
    s = quads(&identity, {{0, 0, 559.2f, 0, 0, 0, 0, 548.8f, 0, 0, 548.8f, 559.2f}});
    CreateCudaShape("trianglemesh", s, NULL, green.GetPtr(), -1);
    s = quads(&identity, {{552.8f, 0, 0, 549.6f, 0, 559.2f, 556.0f, 548.8f, 559.2f, 556.0f, 548.8f, 0}});
    CreateCudaShape("trianglemesh", s, NULL, red.GetPtr(), -1);
    std::vector<Reference<Primitive> > blocks; /* RenderOptions::instances["blocks"] */
    std::vector<Reference<Primitive> > *inst = o.instanced ? &blocks : NULL;
    s = quads(&identity, {{130, 165, 65, 82, 165, 225, 240, 165, 272, 290, 165, 114},
                          {290, 0, 114, 290, 165, 114, 240, 165, 272, 240, 0, 272},
                          {130, 0, 65, 130, 165, 65, 290, 165, 114, 290, 0, 114},
                          {82, 0, 225, 82, 165, 225, 130, 165, 65, 130, 0, 65},
                          {240, 0, 272, 240, 165, 272, 82, 165, 225, 82, 0, 225}});
    CreateCudaShape("trianglemesh", s, inst, white.GetPtr(), -1);
    s = quads(&identity, {{423, 330, 247, 265, 330, 296, 314, 330, 456, 472, 330, 406},
                          {423, 0, 247, 423, 330, 247, 472, 330, 406, 472, 0, 406},
                          {472, 0, 406, 472, 330, 406, 314, 330, 456, 314, 0, 456},
                          {314, 0, 456, 314, 330, 456, 265, 330, 296, 265, 0, 296},
                          {265, 0, 296, 265, 330, 296, 423, 330, 247, 423, 0, 247}});
    CreateCudaShape("trianglemesh", s, inst, white.GetPtr(), -1);
    if (o.instanced) CudaObjectInstance(&blocks, identity); /* ObjectInstance "blocks" */
    /* AttributeBegin; Translate 278 548.7 279.5; Rotate 90 1 0 0;
     * AreaLightSource "diffuse" "rgb L" [17 17 17]; Shape "disk" "float radius" 65 */
    float m[4][4] = {{1, 0, 0, 278.f}, {0, 0, -1, 548.7f}, {0, 1, 0, 279.5f}, {0, 0, 0, 1}};
    float mi[4][4] = {{1, 0, 0, -278.f}, {0, 0, 1, -279.5f}, {0, -1, 0, 548.7f}, {0, 0, 0, 1}};
    static const Transform light2world{Matrix4x4(m), Matrix4x4(mi)}, world2light{Matrix4x4(mi), Matrix4x4(m)};
    Reference<Shape> disk(new Disk(&light2world, &world2light, false, 0.f, 65.f, 0.f, 360.f));
    const float Le[3] = {17.f, 17.f, 17.f};
    DiffuseAreaLight *area = new DiffuseAreaLight(light2world, RGBSpectrum::FromRGB(Le, SPECTRUM_ILLUMINANT),
                                                  o.nsamples, disk);
    Scene scene;
    scene.lights.push_back(area);
    CreateCudaShape("disk", disk, NULL, black.GetPtr(), 0);
    /* MakeRenderer: Renderer "cuda" */
    KeepFilm *film = new KeepFilm(o.W, o.H);
    RecordingCamera *camera = new RecordingCamera(film, o.W, o.H);
    ParamSet params; /* Renderer "cuda" "integer photonpaths" [N] "string photonmap" [...] */
    params.AddInt("photonpaths", &o.paths, 1);
    params.AddString("photonmap", &o.photonmap, 1);
    CentreSampler *sampler = new CentreSampler(o.W, o.H);
    Renderer *renderer = CreateCudaRenderer(sampler, camera, params, o.renderer == "simple" ? "simple" : "photonmap");
    /* pbrtWorldEnd */
    renderer->Render(&scene);
    FILE *f = std::fopen(o.out.c_str(), "wb");
    if (!f) { std::perror("fopen"); return 2; }
    const int hdr[4] = {o.W, o.H, o.nsamples, (int)film->written};
    std::fwrite(hdr, sizeof hdr, 1, f);
    std::fwrite(camera->rays.data(), sizeof(float), camera->rays.size(), f);
    std::fwrite(sampler->rand2d.data(), sizeof(float), sampler->rand2d.size(), f);
    std::fwrite(film->rgb.data(), sizeof(float), film->rgb.size(), f);
    std::fclose(f);
    std::printf("pm_pbrt_host: %ld samples added, image written %d time(s)\n", film->added, film->written);
    delete renderer; /* pbrt deletes its Renderer */
    delete area;
    return 0;
}

} // namespace

int main(int argc, char **argv) {
    Opts o;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
        if (a == "--width") o.W = std::stoi(val());
        else if (a == "--height") o.H = std::stoi(val());
        else if (a == "--paths") o.paths = std::stoi(val());
        else if (a == "--nsamples") o.nsamples = std::stoi(val());
        else if (a == "--photonmap") o.photonmap = val();
        else if (a == "--renderer") o.renderer = val();
        else if (a == "--instanced") o.instanced = true;
        else if (a == "--out") o.out = val();
        else { std::fprintf(stderr, "unknown option %s\n", a.c_str()); return 2; }
    }
    if (o.out.empty()) { std::fprintf(stderr, "usage: %s --out f.bin [options]\n", argv[0]); return 2; }
    return run(o);
}
