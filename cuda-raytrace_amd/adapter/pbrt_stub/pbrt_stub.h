/*
 * pbrt_stub.h — the members of pbrt-v2 (the reference's fork,
 * git://github.com/wjzhou/pbrt-v2.git, not vendored with the reference) that
 * the plugin boundary touches, declared with pbrt-v2's
 * class names, member names and signatures so that adapter/cudaapi.cpp
 * compiles here exactly as it would inside a pbrt-v2 tree. Header-only; the
 * few bodies are the obvious ones (vector algebra, Sample memory layout).
 * NOT pbrt: no parser, integrators, BSDFs or accelerators — a real build
 * replaces this directory by pbrt-v2's src/ (see INTEGRATION.md §2).
 *
 * The fork exposes members that upstream pbrt-v2 keeps protected / private
 * (TriangleMesh::p, Sphere::radius, Disk::*, PointLight::lightPos,
 * DiffuseAreaLight::shapeSet, MatteMaterial::Kd, ...); the reference reads
 * them directly (util/shape/cudatrianglemesh.cpp:18-66, cudasphere.cpp:17-29,
 * cudadisk.cpp:17-35, util/light/cudalight.cpp:16-57,
 * util/material/cudamaterial.cpp:26-58), so they are public here too.
 */
#pragma once

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

using std::string;
using std::vector;

/* ---- core/pbrt.h: diagnostics, references -------------------------------- */
inline void pbrtStubMessage(const char *kind, const char *fmt, va_list ap) {
    std::fprintf(stderr, "%s: ", kind);
    std::vfprintf(stderr, fmt, ap);
    std::fprintf(stderr, "\n");
}
inline void Info(const char *fmt, ...) { va_list ap; va_start(ap, fmt); pbrtStubMessage("Info", fmt, ap); va_end(ap); }
inline void Warning(const char *fmt, ...) { va_list ap; va_start(ap, fmt); pbrtStubMessage("Warning", fmt, ap); va_end(ap); }
inline void Error(const char *fmt, ...) { va_list ap; va_start(ap, fmt); pbrtStubMessage("Error", fmt, ap); va_end(ap); }
inline void Severe(const char *fmt, ...) {
    va_list ap; va_start(ap, fmt); pbrtStubMessage("Fatal Error", fmt, ap); va_end(ap);
    std::abort();
}

class ReferenceCounted {
public:
    ReferenceCounted() : nReferences(0) {}
    int nReferences;
private:
    ReferenceCounted(const ReferenceCounted &);
    ReferenceCounted &operator=(const ReferenceCounted &);
};

template <typename T> class Reference {
public:
    Reference(T *p = NULL) : ptr(p) { if (ptr) ++ptr->nReferences; }
    Reference(const Reference<T> &r) : ptr(r.ptr) { if (ptr) ++ptr->nReferences; }
    Reference &operator=(const Reference<T> &r) {
        if (r.ptr) ++r.ptr->nReferences;
        if (ptr && --ptr->nReferences == 0) delete ptr;
        ptr = r.ptr;
        return *this;
    }
    ~Reference() { if (ptr && --ptr->nReferences == 0) delete ptr; }
    T *operator->() { return ptr; }
    const T *operator->() const { return ptr; }
    operator bool() const { return ptr != NULL; }
    const T *GetPtr() const { return ptr; }
private:
    T *ptr;
};

inline float Radians(float deg) { return ((float)M_PI / 180.f) * deg; }

/* ---- core/geometry.h ------------------------------------------------------ */
class Vector {
public:
    Vector() : x(0.f), y(0.f), z(0.f) {}
    Vector(float xx, float yy, float zz) : x(xx), y(yy), z(zz) {}
    Vector operator*(float f) const { return Vector(f * x, f * y, f * z); }
    Vector operator+(const Vector &v) const { return Vector(x + v.x, y + v.y, z + v.z); }
    float Length() const { return std::sqrt(x * x + y * y + z * z); }
    float x, y, z;
};
class Point {
public:
    Point() : x(0.f), y(0.f), z(0.f) {}
    Point(float xx, float yy, float zz) : x(xx), y(yy), z(zz) {}
    float x, y, z;
};
class Normal {
public:
    Normal() : x(0.f), y(0.f), z(0.f) {}
    Normal(float xx, float yy, float zz) : x(xx), y(yy), z(zz) {}
    float x, y, z;
};
inline Vector Cross(const Vector &v1, const Vector &v2) {
    return Vector((v1.y * v2.z) - (v1.z * v2.y), (v1.z * v2.x) - (v1.x * v2.z), (v1.x * v2.y) - (v1.y * v2.x));
}
inline Vector Normalize(const Vector &v) { return v * (1.f / v.Length()); }

class Ray {
public:
    Ray() : mint(0.f), maxt(INFINITY), time(0.f), depth(0) {}
    Point o;
    Vector d;
    mutable float mint, maxt;
    float time;
    int depth;
};
class RayDifferential : public Ray {
public:
    RayDifferential() : hasDifferentials(false) {}
    void ScaleDifferentials(float s) {
        rxOrigin = Point(o.x + (rxOrigin.x - o.x) * s, o.y + (rxOrigin.y - o.y) * s, o.z + (rxOrigin.z - o.z) * s);
        ryOrigin = Point(o.x + (ryOrigin.x - o.x) * s, o.y + (ryOrigin.y - o.y) * s, o.z + (ryOrigin.z - o.z) * s);
        rxDirection = d + Vector(rxDirection.x - d.x, rxDirection.y - d.y, rxDirection.z - d.z) * s;
        ryDirection = d + Vector(ryDirection.x - d.x, ryDirection.y - d.y, ryDirection.z - d.z) * s;
    }
    bool hasDifferentials;
    Point rxOrigin, ryOrigin;
    Vector rxDirection, ryDirection;
};

/* ---- core/transform.h ------------------------------------------------------ */
struct Matrix4x4 {
    Matrix4x4() { for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) m[i][j] = i == j ? 1.f : 0.f; }
    explicit Matrix4x4(const float mat[4][4]) { std::memcpy(m, mat, 16 * sizeof(float)); }
    float m[4][4];
};
class Transform {
public:
    Transform() {}
    Transform(const Matrix4x4 &mat, const Matrix4x4 &minv) : m(mat), mInv(minv) {}
    const Matrix4x4 &GetMatrix() const { return m; }
    const Matrix4x4 &GetInverseMatrix() const { return mInv; }
    Point operator()(const Point &pt) const {
        const float x = pt.x, y = pt.y, z = pt.z;
        const float xp = m.m[0][0] * x + m.m[0][1] * y + m.m[0][2] * z + m.m[0][3];
        const float yp = m.m[1][0] * x + m.m[1][1] * y + m.m[1][2] * z + m.m[1][3];
        const float zp = m.m[2][0] * x + m.m[2][1] * y + m.m[2][2] * z + m.m[2][3];
        const float wp = m.m[3][0] * x + m.m[3][1] * y + m.m[3][2] * z + m.m[3][3];
        if (wp == 1.f) return Point(xp, yp, zp);
        return Point(xp / wp, yp / wp, zp / wp);
    }
    Vector operator()(const Vector &v) const {
        const float x = v.x, y = v.y, z = v.z;
        return Vector(m.m[0][0] * x + m.m[0][1] * y + m.m[0][2] * z, m.m[1][0] * x + m.m[1][1] * y + m.m[1][2] * z,
                      m.m[2][0] * x + m.m[2][1] * y + m.m[2][2] * z);
    }
private:
    Matrix4x4 m, mInv;
};

/* ---- core/spectrum.h (RGB build: Spectrum == RGBSpectrum) ------------------ */
enum SpectrumType { SPECTRUM_REFLECTANCE, SPECTRUM_ILLUMINANT };
class RGBSpectrum {
public:
    RGBSpectrum(float v = 0.f) { c[0] = c[1] = c[2] = v; }
    void ToRGB(float *rgb) const { rgb[0] = c[0]; rgb[1] = c[1]; rgb[2] = c[2]; }
    static RGBSpectrum FromRGB(const float rgb[3], SpectrumType type = SPECTRUM_REFLECTANCE) {
        (void)type;
        RGBSpectrum s;
        s.c[0] = rgb[0]; s.c[1] = rgb[1]; s.c[2] = rgb[2];
        return s;
    }
    bool HasNaNs() const { return std::isnan(c[0]) || std::isnan(c[1]) || std::isnan(c[2]); }
    float y() const { const float YWeight[3] = {0.212671f, 0.715160f, 0.072169f};
                      return YWeight[0] * c[0] + YWeight[1] * c[1] + YWeight[2] * c[2]; }
    float c[3];
};
typedef RGBSpectrum Spectrum;

/* ---- core/diffgeom.h, core/texture.h -------------------------------------- */
class Shape;
struct DifferentialGeometry {
    DifferentialGeometry() : u(0.f), v(0.f), shape(NULL) {}
    Point p;
    Normal nn;
    float u, v;
    const Shape *shape;
};
template <typename T> class Texture : public ReferenceCounted {
public:
    virtual T Evaluate(const DifferentialGeometry &) const = 0;
    virtual ~Texture() {}
};
template <typename T> class ConstantTexture : public Texture<T> {
public:
    ConstantTexture(const T &v) : value(v) {}
    T Evaluate(const DifferentialGeometry &) const { return value; }
private:
    T value;
};

/* ---- core/shape.h, shapes/{trianglemesh,sphere,disk}.h ---------------------------------------------- */
class Shape : public ReferenceCounted {
public:
    Shape(const Transform *o2w, const Transform *w2o, bool ro)
        : ObjectToWorld(o2w), WorldToObject(w2o), ReverseOrientation(ro), TransformSwapsHandedness(false),
          shapeId(0) {}
    virtual ~Shape() {}
    virtual float Area() const { Severe("Unimplemented Shape::Area() method called"); return 0.f; }
    const Transform *ObjectToWorld, *WorldToObject;
    const bool ReverseOrientation, TransformSwapsHandedness;
    const uint32_t shapeId;
};
class ShapeSet {
public:
    explicit ShapeSet(const Reference<Shape> &s) { shapes.push_back(s); }
    vector<Reference<Shape> > shapes;
};
/* pbrt-v2 TriangleMesh: the constructor stores the vertices in WORLD space */
class TriangleMesh : public Shape {
public:
    TriangleMesh(const Transform *o2w, const Transform *w2o, bool ro, int nt, int nv, const int *vi, const Point *P,
                 const Normal *N, const Vector *S, const float *uv)
        : Shape(o2w, w2o, ro), ntris(nt), nverts(nv) {
        vertexIndex = new int[3 * ntris];
        std::memcpy(vertexIndex, vi, 3 * ntris * sizeof(int));
        uvs = NULL; n = NULL; s = NULL;
        if (uv) { uvs = new float[2 * nverts]; std::memcpy(uvs, uv, 2 * nverts * sizeof(float)); }
        p = new Point[nverts];
        if (N) { n = new Normal[nverts]; std::memcpy(n, N, nverts * sizeof(Normal)); }
        if (S) { s = new Vector[nverts]; std::memcpy(s, S, nverts * sizeof(Vector)); }
        for (int i = 0; i < nverts; ++i) p[i] = (*ObjectToWorld)(P[i]);
    }
    ~TriangleMesh() { delete[] vertexIndex; delete[] p; delete[] s; delete[] n; delete[] uvs; }
    int ntris, nverts;
    int *vertexIndex;
    Point *p;
    Normal *n;
    Vector *s;
    float *uvs;
};
class Sphere : public Shape {
public:
    Sphere(const Transform *o2w, const Transform *w2o, bool ro, float rad, float z0, float z1, float pm)
        : Shape(o2w, w2o, ro), radius(rad), zmin(z0), zmax(z1), phiMax(Radians(pm)) {}
    float Area() const { return phiMax * radius * (zmax - zmin); }
    float radius;
    float zmin, zmax;
    float phiMax;
};
class Disk : public Shape {
public:
    Disk(const Transform *o2w, const Transform *w2o, bool ro, float ht, float r, float ri, float tmax)
        : Shape(o2w, w2o, ro), height(ht), radius(r), innerRadius(ri), phiMax(Radians(tmax < 0.f ? 0.f : tmax > 360.f ? 360.f : tmax)) {}
    float Area() const { return phiMax * 0.5f * (radius * radius - innerRadius * innerRadius); }
    float height, radius, innerRadius, phiMax;
};

/* ---- core/material.h, materials/{matte,mirror,glass}.h ---------------------------------------- */
class Material : public ReferenceCounted {
public:
    virtual ~Material() {}
};
class MatteMaterial : public Material {
public:
    MatteMaterial(Reference<Texture<Spectrum> > kd, Reference<Texture<float> > sig, Reference<Texture<float> > bump)
        : Kd(kd), sigma(sig), bumpMap(bump) {}
    Reference<Texture<Spectrum> > Kd;
    Reference<Texture<float> > sigma, bumpMap;
};
class MirrorMaterial : public Material {
public:
    MirrorMaterial(Reference<Texture<Spectrum> > r, Reference<Texture<float> > bump) : Kr(r), bumpMap(bump) {}
    Reference<Texture<Spectrum> > Kr;
    Reference<Texture<float> > bumpMap;
};
class GlassMaterial : public Material {
public:
    GlassMaterial(Reference<Texture<Spectrum> > r, Reference<Texture<Spectrum> > t, Reference<Texture<float> > i,
                  Reference<Texture<float> > bump)
        : Kr(r), Kt(t), index(i), bumpMap(bump) {}
    Reference<Texture<Spectrum> > Kr, Kt;
    Reference<Texture<float> > index, bumpMap;
};

/* ---- core/light.h, lights/point.h, lights/diffuse.h ------------------------ */
class Light {
public:
    virtual ~Light() {}
    Light(const Transform &l2w, int ns = 1) : nSamples(ns < 1 ? 1 : ns), LightToWorld(l2w) {}
    const int nSamples;
protected:
    const Transform LightToWorld;
};
class AreaLight : public Light {
public:
    AreaLight(const Transform &l2w, int ns) : Light(l2w, ns) {}
};
class PointLight : public Light {
public:
    PointLight(const Transform &light2world, const Spectrum &intensity)
        : Light(light2world), lightPos(light2world(Point(0, 0, 0))), Intensity(intensity) {}
    Point lightPos;
    Spectrum Intensity;
};
class DiffuseAreaLight : public AreaLight {
public:
    DiffuseAreaLight(const Transform &light2world, const Spectrum &Le, int ns, const Reference<Shape> &shape)
        : AreaLight(light2world, ns), Lemit(Le), shapeSet(new ShapeSet(shape)), area(shape->Area()) {}
    ~DiffuseAreaLight() { delete shapeSet; }
    Spectrum Lemit;
    ShapeSet *shapeSet;
    float area;
};

/* ---- core/primitive.h, core/scene.h, core/paramset.h, core/rng.h, core/memory.h */
class Primitive : public ReferenceCounted {
public:
    virtual ~Primitive() {}
};
class Scene {
public:
    vector<Light *> lights;
};
class ParamSet { /* the single-value lookups of pbrt-v2's ParamSet */
public:
    void AddInt(const string &name, const int *data, int nItems) { if (nItems > 0) ints.push_back(std::make_pair(name, data[0])); }
    void AddFloat(const string &name, const float *data, int nItems) { if (nItems > 0) floats.push_back(std::make_pair(name, data[0])); }
    void AddString(const string &name, const string *data, int nItems) { if (nItems > 0) strings.push_back(std::make_pair(name, data[0])); }
    int FindOneInt(const string &name, int d) const { return find(ints, name, d); }
    float FindOneFloat(const string &name, float d) const { return find(floats, name, d); }
    string FindOneString(const string &name, const string &d) const { return find(strings, name, d); }
private:
    template <typename T> static T find(const vector<std::pair<string, T> > &v, const string &name, const T &d) {
        for (size_t i = 0; i < v.size(); ++i) if (v[i].first == name) return v[i].second;
        return d;
    }
    vector<std::pair<string, int> > ints;
    vector<std::pair<string, float> > floats;
    vector<std::pair<string, string> > strings;
};
class RNG {
public:
    RNG(uint32_t seed = 5489UL) : state(seed) {}
    uint32_t RandomUInt() const { state = state * 1664525u + 1013904223u; return state; }
    float RandomFloat() const { return (RandomUInt() >> 8) * (1.f / 16777216.f); }
private:
    mutable uint32_t state;
};
class MemoryArena {};
struct Intersection;

/* ---- core/sampler.h: CameraSample, Sample (pbrt's memory layout: every
 * oneD / twoD array of a sample in one contiguous block), Sampler ---------- */
class Sampler;
class SurfaceIntegrator;
class VolumeIntegrator;
struct CameraSample {
    float imageX, imageY;
    float lensU, lensV;
    float time;
};
struct Sample : public CameraSample {
    Sample(Sampler *, SurfaceIntegrator *, VolumeIntegrator *, const Scene *) : oneD(NULL), twoD(NULL) {}
    uint32_t Add1D(uint32_t num) { n1D.push_back(num); return (uint32_t)n1D.size() - 1; }
    uint32_t Add2D(uint32_t num) { n2D.push_back(num); return (uint32_t)n2D.size() - 1; }
    ~Sample() { if (oneD) { std::free(oneD[0]); std::free(oneD); } }
    Sample *Duplicate(int count) const {
        Sample *ret = new Sample[count];
        for (int i = 0; i < count; ++i) {
            ret[i].n1D = n1D;
            ret[i].n2D = n2D;
            ret[i].AllocateSampleMemory();
        }
        return ret;
    }
    vector<uint32_t> n1D, n2D;
    float **oneD, **twoD;
private:
    void AllocateSampleMemory() {
        const size_t nPtrs = n1D.size() + n2D.size();
        if (!nPtrs) { oneD = twoD = NULL; return; }
        oneD = (float **)std::malloc(nPtrs * sizeof(float *));
        twoD = oneD + n1D.size();
        size_t totSamples = 0;
        for (uint32_t i = 0; i < n1D.size(); ++i) totSamples += n1D[i];
        for (uint32_t i = 0; i < n2D.size(); ++i) totSamples += 2 * n2D[i];
        float *mem = (float *)std::calloc(totSamples ? totSamples : 1, sizeof(float));
        for (uint32_t i = 0; i < n1D.size(); ++i) { oneD[i] = mem; mem += n1D[i]; }
        for (uint32_t i = 0; i < n2D.size(); ++i) { twoD[i] = mem; mem += 2 * n2D[i]; }
    }
    Sample() : oneD(NULL), twoD(NULL) {}
};
class Sampler {
public:
    Sampler(int xstart, int xend, int ystart, int yend, int spp, float sopen, float sclose)
        : xPixelStart(xstart), xPixelEnd(xend), yPixelStart(ystart), yPixelEnd(yend), samplesPerPixel(spp),
          shutterOpen(sopen), shutterClose(sclose) {}
    virtual ~Sampler() {}
    virtual int GetMoreSamples(Sample *sample, RNG &rng) = 0;
    virtual int MaximumSampleCount() = 0;
    virtual int RoundSize(int size) const = 0;
    const int xPixelStart, xPixelEnd, yPixelStart, yPixelEnd;
    const int samplesPerPixel;
    const float shutterOpen, shutterClose;
};

/* ---- core/film.h, core/camera.h, core/renderer.h ---------------------------- */
class Film {
public:
    Film(int xres, int yres) : xResolution(xres), yResolution(yres) {}
    virtual ~Film() {}
    virtual void AddSample(const CameraSample &sample, const Spectrum &L) = 0;
    virtual void GetSampleExtent(int *xstart, int *xend, int *ystart, int *yend) const = 0;
    virtual void WriteImage(float splatScale = 1.f) = 0;
    const int xResolution, yResolution;
};
class Camera {
public:
    explicit Camera(Film *f) : film(f) {}
    virtual ~Camera() { delete film; }
    virtual float GenerateRay(const CameraSample &sample, Ray *ray) const = 0;
    virtual float GenerateRayDifferential(const CameraSample &sample, RayDifferential *rd) const {
        float wt = GenerateRay(sample, rd);
        rd->hasDifferentials = false;
        return wt;
    }
    Film *film;
};
class Renderer {
public:
    virtual ~Renderer() {}
    virtual void Render(const Scene *scene) = 0;
    virtual Spectrum Li(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                        MemoryArena &arena, Intersection *isect = NULL, Spectrum *T = NULL) const = 0;
    virtual Spectrum Transmittance(const Scene *scene, const RayDifferential &ray, const Sample *sample, RNG &rng,
                                   MemoryArena &arena) const = 0;
};
