/*
 * pm_render_cli — renders a scene through the pbrt-facing C++ layer
 * (pm_cudarender.h), the way pbrt-v2 drives the reference plugin:
 *   CudaRenderInit -> CreateCudaShape x N (ObjectBegin/Instance optional)
 *   -> CreateCudaRenderer -> Render(lights, camera) -> Film::AddSample
 * and writes the image as PFM. Used by tests/test_adapter.py (GPU) to check
 * that this host path produces the same image as the Python stage driver.
 *
 *   pm_render_cli --scene cornell --width W --height H --camera e0 e1 e2 f0 f1 f2 r0 r1 r2 u0 u1 u2
 *                 [--paths N] [--passes P] [--structure grid|kd] [--instanced]
 *                 [--renderer photonmapping|simple] --out img.pfm
 *   pm_render_cli --pbrt scene.pbrt [--out img.pfm] [--renderer R] [--paths N] [--passes P] [--structure S]
 *                 (a pbrt-v2 scene file through pm_pbrt.h; command-line options override the file)
 *   pm_render_cli --pbrt scene.pbrt --dump   (parse only, no device: the plugin calls as JSON)
 *   pm_render_cli --selftest      (host-only checks, no device needed)
 */
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "pm_cudarender.h"
#include "pm_pbrt.h"

using namespace pmcuda;

namespace {

/* one sample per pixel: the film is the pixel grid */
struct PixelFilm : Film {
    int W, H;
    std::vector<float> rgb;
    std::string path;
    PixelFilm(int w, int h, std::string p) : W(w), H(h), rgb((size_t)3 * w * h, 0.f), path(std::move(p)) {}
    void AddSample(const CameraSample &s, const float c[3]) override {
        const int x = (int)std::floor(s.imageX), y = (int)std::floor(s.imageY);
        if (x < 0 || y < 0 || x >= W || y >= H) return;
        float *d = &rgb[3 * ((size_t)y * W + x)];
        d[0] = c[0]; d[1] = c[1]; d[2] = c[2];
    }
    void WriteImage() override { /* PFM: rows bottom to top, little endian */
        FILE *f = std::fopen(path.c_str(), "wb");
        if (!f) throw Error("cannot write " + path);
        std::fprintf(f, "PF\n%d %d\n-1.0\n", W, H);
        for (int y = H - 1; y >= 0; --y) std::fwrite(&rgb[3 * (size_t)y * W], sizeof(float), 3 * (size_t)W, f);
        std::fclose(f);
    }
};

Shape quads(const std::vector<std::vector<float>> &q) {
    Shape s;
    for (const auto &quad : q) {
        const int b = (int)(s.P.size() / 3);
        s.P.insert(s.P.end(), quad.begin(), quad.end());
        const int idx[6] = {b, b + 1, b + 2, b, b + 2, b + 3};
        s.indices.insert(s.indices.end(), idx, idx + 6);
    }
    return s;
}

/* The classic Cornell box of pmrender/scenes.py cornell_box() (C2), issued
 * as pbrt would: world-space triangle meshes, a disk area light under
 * Translate 278 548.7 279.5 + Rotate 90 about x (exact matrix). */
void cornell(bool instanced, std::vector<Light> &lights) {
    static const Material white{Material::Matte, {0.73f, 0.73f, 0.73f}};
    static const Material red{Material::Matte, {0.63f, 0.065f, 0.05f}};
    static const Material green{Material::Matte, {0.14f, 0.45f, 0.091f}};
    static const Material black{Material::Matte, {0.f, 0.f, 0.f}};
    CreateCudaShape("trianglemesh", quads({{552.8f, 0, 0, 0, 0, 0, 0, 0, 559.2f, 549.6f, 0, 559.2f},
                                           {556.0f, 548.8f, 0, 556.0f, 548.8f, 559.2f, 0, 548.8f, 559.2f, 0, 548.8f, 0},
                                           {549.6f, 0, 559.2f, 0, 0, 559.2f, 0, 548.8f, 559.2f, 556.0f, 548.8f, 559.2f}}),
                    nullptr, &white, -1);
    CreateCudaShape("trianglemesh", quads({{0, 0, 559.2f, 0, 0, 0, 0, 548.8f, 0, 0, 548.8f, 559.2f}}), nullptr, &green,
                    -1);
    CreateCudaShape("trianglemesh",
                    quads({{552.8f, 0, 0, 549.6f, 0, 559.2f, 556.0f, 548.8f, 559.2f, 556.0f, 548.8f, 0}}), nullptr,
                    &red, -1);
    const Shape shortb = quads({{130, 165, 65, 82, 165, 225, 240, 165, 272, 290, 165, 114},
                                {290, 0, 114, 290, 165, 114, 240, 165, 272, 240, 0, 272},
                                {130, 0, 65, 130, 165, 65, 290, 165, 114, 290, 0, 114},
                                {82, 0, 225, 82, 165, 225, 130, 165, 65, 130, 0, 65},
                                {240, 0, 272, 240, 165, 272, 82, 165, 225, 82, 0, 225}});
    const Shape tallb = quads({{423, 330, 247, 265, 330, 296, 314, 330, 456, 472, 330, 406},
                               {423, 0, 247, 423, 330, 247, 472, 330, 406, 472, 0, 406},
                               {472, 0, 406, 472, 330, 406, 314, 330, 456, 314, 0, 456},
                               {314, 0, 456, 314, 330, 456, 265, 330, 296, 265, 0, 296},
                               {265, 0, 296, 265, 330, 296, 423, 330, 247, 423, 0, 247}});
    if (instanced) { /* ObjectBegin "blocks" ... ObjectEnd; ObjectInstance "blocks" (identity) */
        static const int key = 0;
        CreateCudaShape("trianglemesh", shortb, &key, &white, -1);
        CreateCudaShape("trianglemesh", tallb, &key, &white, -1);
        CudaObjectInstance(&key, Transform::identity());
    } else {
        CreateCudaShape("trianglemesh", shortb, nullptr, &white, -1);
        CreateCudaShape("trianglemesh", tallb, nullptr, &white, -1);
    }
    Light L;
    L.kind = Light::AreaDisk;
    L.disk.radius = 65.f;
    L.disk.o2w = Transform::identity();
    const float m[16] = {1, 0, 0, 278.f, 0, 0, -1, 548.7f, 0, 1, 0, 279.5f, 0, 0, 0, 1};
    const float mi[16] = {1, 0, 0, -278.f, 0, 0, 1, -279.5f, 0, -1, 0, 548.7f, 0, 0, 0, 1};
    std::memcpy(L.disk.o2w.m, m, sizeof(m));
    std::memcpy(L.disk.o2w.minv, mi, sizeof(mi));
    L.Lemit = {17.f, 17.f, 17.f};
    L.n_samples = 1;
    lights.push_back(L);
    CreateCudaShape("disk", L.disk, nullptr, &black, 0);
}

int selftest() {
    int bad = 0;
    auto near = [&](float a, float b, const char *what) {
        if (std::fabs(a - b) > 1e-5f * (1.f + std::fabs(b))) { std::printf("FAIL %s: %g vs %g\n", what, a, b); ++bad; }
    };
    const Transform t = Transform::translate(1, 2, 3) * Transform::rotate_x(90.f);
    const float p[3] = {0, 0, 1};
    float o[3];
    t.point(p, o); /* rotate (0,0,1) -> (0,-1,0), then translate */
    near(o[0], 1.f, "point.x"); near(o[1], 1.f, "point.y"); near(o[2], 3.f, "point.z");
    const float v[3] = {0, 1, 0};
    t.vector(v, o); /* (0,1,0) -> (0,0,1), translation ignored */
    near(o[0], 0.f, "vector.x"); near(o[1], 0.f, "vector.y"); near(o[2], 1.f, "vector.z");
    float r[16];
    for (int i = 0; i < 4; ++i) /* m * minv == I */
        for (int j = 0; j < 4; ++j) {
            float s = 0.f;
            for (int k = 0; k < 4; ++k) s += t.m[4 * i + k] * t.minv[4 * k + j];
            r[4 * i + j] = s;
            near(s, i == j ? 1.f : 0.f, "m*minv");
        }
    const float n[3] = {0, 0, 1};
    t.normal(n, o); /* normals follow the inverse transpose: same as vectors for a rotation */
    near(o[0], 0.f, "normal.x"); near(o[1], -1.f, "normal.y"); near(o[2], 0.f, "normal.z");
    (void)r;
    std::printf(bad ? "selftest: %d failures\n" : "selftest: ok\n", bad);
    return bad ? 1 : 0;
}

/* --dump: records the plugin calls a scene file produces, as JSON (floats
 * printed round-trip exact) — the parse checked without a device */
struct DumpSink : PbrtSink {
    std::string out;
    std::map<const void *, int> keys;
    static void arr(std::string &o, const float *v, size_t n) {
        o += "[";
        char b[32];
        for (size_t i = 0; i < n; ++i) { std::snprintf(b, sizeof b, "%s%.9g", i ? ", " : "", v[i]); o += b; }
        o += "]";
    }
    int key(const void *k) {
        if (!k) return -1;
        auto it = keys.find(k);
        if (it != keys.end()) return it->second;
        const int id = (int)keys.size();
        keys[k] = id;
        return id;
    }
    void shape(const std::string &name, const Shape &s, const void *inst, const Material *m, int li) override {
        char b[160];
        if (!out.empty()) out += ",\n";
        std::snprintf(b, sizeof b, "{\"call\": \"shape\", \"name\": \"%s\", \"instance\": %d, \"light\": %d, ",
                      name.c_str(), key(inst), li);
        out += b;
        const int kind = !m ? -1 : (int)m->kind;
        const float k[3] = {m ? m->k.r : 0.f, m ? m->k.g : 0.f, m ? m->k.b : 0.f};
        std::snprintf(b, sizeof b, "\"material\": %d, \"k\": ", kind);
        out += b;
        arr(out, k, 3);
        out += ", \"P\": "; arr(out, s.P.data(), s.P.size());
        out += ", \"N\": "; arr(out, s.N.data(), s.N.size());
        out += ", \"uv\": "; arr(out, s.uv.data(), s.uv.size());
        out += ", \"indices\": [";
        for (size_t i = 0; i < s.indices.size(); ++i) out += (i ? ", " : "") + std::to_string(s.indices[i]);
        out += "], \"o2w\": "; arr(out, s.o2w.m, 16);
        out += ", \"w2o\": "; arr(out, s.o2w.minv, 16);
        const float sc[4] = {s.radius, s.height, s.inner_radius, s.phi_max};
        out += ", \"radius_height_inner_phimax\": "; arr(out, sc, 4);
        out += "}";
    }
    void objectInstance(const void *k, const Transform &tr) override {
        if (!out.empty()) out += ",\n";
        out += "{\"call\": \"instance\", \"instance\": " + std::to_string(key(k)) + ", \"o2w\": ";
        arr(out, tr.m, 16);
        out += "}";
    }
};

int dump(const std::string &path) {
    DumpSink sink;
    PbrtOptions o;
    PbrtParser parser;
    parser.parseFile(path, sink, o);
    std::string lights;
    for (const Light &L : o.lights) {
        if (!lights.empty()) lights += ",\n";
        char b[128];
        if (L.kind == Light::Point) {
            const float I[3] = {L.intensity.r, L.intensity.g, L.intensity.b};
            lights += "{\"kind\": \"point\", \"pos\": ";
            DumpSink::arr(lights, L.pos, 3);
            lights += ", \"I\": ";
            DumpSink::arr(lights, I, 3);
        } else {
            const float Le[3] = {L.Lemit.r, L.Lemit.g, L.Lemit.b};
            std::snprintf(b, sizeof b, "{\"kind\": \"disk\", \"nsamples\": %d, \"Le\": ", L.n_samples);
            lights += b;
            DumpSink::arr(lights, Le, 3);
            lights += ", \"o2w\": ";
            DumpSink::arr(lights, L.disk.o2w.m, 16);
            const float sc[4] = {L.disk.radius, L.disk.height, L.disk.inner_radius, L.disk.phi_max};
            lights += ", \"radius_height_inner_phimax\": ";
            DumpSink::arr(lights, sc, 4);
        }
        lights += "}";
    }
    const Camera &c = o.camera;
    std::printf("{\"calls\": [\n%s],\n\"lights\": [\n%s],\n\"camera\": {\"width\": %d, \"height\": %d, \"eye\": ",
                sink.out.c_str(), lights.c_str(), c.width, c.height);
    std::string cam;
    DumpSink::arr(cam, c.eye, 3); cam += ", \"fwd\": ";
    DumpSink::arr(cam, c.fwd, 3); cam += ", \"right\": ";
    DumpSink::arr(cam, c.right, 3); cam += ", \"up\": ";
    DumpSink::arr(cam, c.up, 3);
    const pm_render_params &p = o.settings.params;
    std::printf("%s},\n\"renderer\": \"%s\", \"paths\": %lld, \"passes\": %d, \"gather\": %d, \"film\": \"%s\", "
                "\"warnings\": %d}\n",
                cam.c_str(), o.renderer.c_str(), (long long)p.paths_per_pass, p.passes, p.gather_structure,
                o.film_filename.c_str(), o.warnings);
    return 0;
}

/* a .pbrt scene through the plugin surface, as pbrt-v2 + the reference would run it */
int render_pbrt(const std::string &path, std::string out, const std::string &renderer, long long paths, int passes,
                const std::string &structure) {
    CudaRenderInit(0);
    PbrtOptions o;
    CudaApiSink sink;
    PbrtParser parser;
    parser.parseFile(path, sink, o);
    if (!renderer.empty()) o.renderer = renderer;
    pm_render_params &p = o.settings.params;
    if (paths > 0) p.paths_per_pass = paths;
    if (passes > 0) p.passes = passes;
    if (!structure.empty()) p.gather_structure = structure == "kd" ? PM_GATHER_KDTREE : PM_GATHER_GRID;
    if (out.empty()) out = o.film_filename;
    CudaRender *render = CreateCudaRenderer(o.settings, o.renderer);
    PixelFilm film(o.camera.width, o.camera.height, out);
    o.camera.film = &film;
    render->Render(o.lights, o.camera);
    if (auto *pm = dynamic_cast<PhotonMappingRenderer *>(render->subRenderer()))
        std::printf("{\"renderer\": \"photonmapping\", \"paths_emitted\": %lld, \"photons_valid\": %lld, "
                    "\"gather_points\": %lld}\n",
                    (long long)pm->stats.paths_emitted, (long long)pm->stats.photons_valid,
                    (long long)pm->stats.gather_points);
    else
        std::printf("{\"renderer\": \"simple\", \"samples\": %lld}\n",
                    (long long)static_cast<SimpleRenderer *>(render->subRenderer())->stats.gather_points);
    delete render;
    return 0;
}

} // namespace

int main(int argc, char **argv) {
    std::string scene = "cornell", out, structure, renderer, pbrt;
    bool dump_only = false;
    int W = 64, H = 48;
    long long paths = 512 * 512;
    int passes = 1;
    bool instanced = false, have_cam = false, paths_set = false, passes_set = false;
    float cam[12] = {0};
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--selftest") return selftest();
        else if (a == "--scene") scene = next();
        else if (a == "--width") W = std::atoi(next());
        else if (a == "--height") H = std::atoi(next());
        else if (a == "--paths") { paths = std::atoll(next()); paths_set = true; }
        else if (a == "--passes") { passes = std::atoi(next()); passes_set = true; }
        else if (a == "--structure") structure = next();
        else if (a == "--instanced") instanced = true;
        else if (a == "--renderer") renderer = next();
        else if (a == "--pbrt") pbrt = next();
        else if (a == "--dump") dump_only = true;
        else if (a == "--out") out = next();
        else if (a == "--camera") {
            for (float &c : cam) c = std::strtof(next(), nullptr);
            have_cam = true;
        } else { std::fprintf(stderr, "unknown argument %s\n", a.c_str()); return 2; }
    }
    if (!pbrt.empty()) {
        try {
            if (dump_only) return dump(pbrt);
            return render_pbrt(pbrt, out, renderer, paths_set ? paths : 0, passes_set ? passes : 0, structure);
        } catch (const Error &e) {
            std::fprintf(stderr, "pm_render_cli: %s\n", e.what());
            return 1;
        }
    }
    if (out.empty()) out = "out.pfm";
    if (scene != "cornell" || !have_cam) {
        std::fprintf(stderr, "usage: %s --scene cornell --camera <12 floats> [--width W --height H] --out f.pfm\n",
                     argv[0]);
        return 2;
    }
    try {
        CudaRenderInit(0);
        std::vector<Light> lights;
        cornell(instanced, lights);
        RenderSettings settings;
        settings.params.paths_per_pass = paths;
        settings.params.passes = passes;
        settings.params.gather_structure = structure == "kd" ? PM_GATHER_KDTREE : PM_GATHER_GRID;
        CudaRender *render = CreateCudaRenderer(settings, renderer.empty() ? "photonmapping" : renderer);
        PixelFilm film(W, H, out);
        Camera camera;
        camera.pinhole = true;
        std::memcpy(camera.eye, cam, 12);
        std::memcpy(camera.fwd, cam + 3, 12);
        std::memcpy(camera.right, cam + 6, 12);
        std::memcpy(camera.up, cam + 9, 12);
        camera.width = W;
        camera.height = H;
        camera.film = &film;
        render->Render(lights, camera);
        auto *pmr = dynamic_cast<PhotonMappingRenderer *>(render->subRenderer());
        const pm_stats &st = pmr ? pmr->stats : static_cast<SimpleRenderer *>(render->subRenderer())->stats;
        std::printf("{\"paths_emitted\": %lld, \"photons_valid\": %lld, \"gather_points\": %lld}\n",
                    (long long)st.paths_emitted, (long long)st.photons_valid, (long long)st.gather_points);
        delete render;
    } catch (const Error &e) {
        std::fprintf(stderr, "pm_render_cli: %s\n", e.what());
        return 1;
    }
    return 0;
}
