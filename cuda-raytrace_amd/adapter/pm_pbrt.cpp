/*
 * pm_pbrt.cpp — pbrt-v2 scene-file front end, see pm_pbrt.h. Host-only C++.
 */
#include "pm_pbrt.h"

#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <sstream>

namespace pmcuda {

namespace {

/* ------------------------------------------------------------ tokens */
struct Token {
    enum Kind { Word, String, Number, Open, Close, End } kind = End;
    std::string text;
    double num = 0.0;
    int line = 0;
};

class Lexer {
public:
    Lexer(std::string text, std::string file) : s_(std::move(text)), file_(std::move(file)) {}
    Token next() {
        skip();
        Token t;
        t.line = line_;
        if (i_ >= s_.size()) return t;
        const char c = s_[i_];
        if (c == '[') { ++i_; t.kind = Token::Open; return t; }
        if (c == ']') { ++i_; t.kind = Token::Close; return t; }
        if (c == '"') {
            const size_t e = s_.find('"', i_ + 1);
            if (e == std::string::npos) fail(line_, "unterminated string");
            t.kind = Token::String;
            t.text = s_.substr(i_ + 1, e - i_ - 1);
            for (char ch : t.text) line_ += ch == '\n';
            i_ = e + 1;
            return t;
        }
        size_t e = i_;
        while (e < s_.size() && !std::isspace((unsigned char)s_[e]) && s_[e] != '[' && s_[e] != ']' && s_[e] != '"' &&
               s_[e] != '#')
            ++e;
        t.text = s_.substr(i_, e - i_);
        i_ = e;
        char *end = nullptr;
        const double v = std::strtod(t.text.c_str(), &end);
        if (end && *end == '\0' && !t.text.empty() &&
            (std::isdigit((unsigned char)t.text[0]) || t.text[0] == '-' || t.text[0] == '+' || t.text[0] == '.')) {
            t.kind = Token::Number;
            t.num = v;
        } else {
            t.kind = Token::Word;
        }
        return t;
    }
    Token peek() {
        const size_t i = i_;
        const int l = line_;
        Token t = next();
        i_ = i;
        line_ = l;
        return t;
    }
    [[noreturn]] void fail(int line, const char *fmt, ...) const {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        std::vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        throw Error(file_ + ":" + std::to_string(line) + ": " + buf);
    }
    const std::string &file() const { return file_; }

private:
    void skip() {
        while (i_ < s_.size()) {
            const char c = s_[i_];
            if (c == '\n') { ++line_; ++i_; }
            else if (std::isspace((unsigned char)c)) ++i_;
            else if (c == '#') { while (i_ < s_.size() && s_[i_] != '\n') ++i_; }
            else break;
        }
    }
    std::string s_, file_;
    size_t i_ = 0;
    int line_ = 1;
};

/* ------------------------------------------------------------ ParamSet */
struct Param {
    std::string type, name;
    std::vector<double> nums;
    std::vector<std::string> strs;
    mutable bool used = false;
};

struct ParamSet {
    std::vector<Param> params;
    const Param *find(const std::string &name) const {
        for (const Param &p : params)
            if (p.name == name) { p.used = true; return &p; }
        return nullptr;
    }
    float oneFloat(const std::string &n, float d) const {
        const Param *p = find(n);
        return p && !p->nums.empty() ? (float)p->nums[0] : d;
    }
    double oneDouble(const std::string &n, double d) const {
        const Param *p = find(n);
        return p && !p->nums.empty() ? p->nums[0] : d;
    }
    int oneInt(const std::string &n, int d) const {
        const Param *p = find(n);
        return p && !p->nums.empty() ? (int)p->nums[0] : d;
    }
    std::string oneString(const std::string &n, const std::string &d) const {
        const Param *p = find(n);
        return p && !p->strs.empty() ? p->strs[0] : d;
    }
    std::vector<float> floats(const std::string &n) const {
        const Param *p = find(n);
        std::vector<float> v;
        if (p) for (double x : p->nums) v.push_back((float)x);
        return v;
    }
};

/* ------------------------------------------------------------ pbrt-v2 math */
/* Gauss-Jordan inverse (double), as pbrt's Inverse(Matrix4x4) */
bool invert(const float *m, float *out) {
    double a[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) a[i][j] = j < 4 ? m[4 * i + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int piv = c;
        for (int r = c + 1; r < 4; ++r)
            if (std::fabs(a[r][c]) > std::fabs(a[piv][c])) piv = r;
        if (a[piv][c] == 0.0) return false;
        if (piv != c)
            for (int j = 0; j < 8; ++j) std::swap(a[c][j], a[piv][j]);
        const double inv = 1.0 / a[c][c];
        for (int j = 0; j < 8; ++j) a[c][j] *= inv;
        for (int r = 0; r < 4; ++r)
            if (r != c && a[r][c] != 0.0) {
                const double f = a[r][c];
                for (int j = 0; j < 8; ++j) a[r][j] -= f * a[c][j];
            }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = (float)a[i][j + 4];
    return true;
}

Transform from_matrix(const float m[16]) {
    Transform t;
    std::memcpy(t.m, m, sizeof(t.m));
    if (!invert(m, t.minv)) throw Error("singular transform matrix");
    return t;
}

Transform scale(float x, float y, float z) {
    Transform t = Transform::identity();
    t.m[0] = x; t.m[5] = y; t.m[10] = z;
    t.minv[0] = 1.f / x; t.minv[5] = 1.f / y; t.minv[10] = 1.f / z;
    return t;
}

/* pbrt-v2 Radians(float) */
inline float radians(float deg) { return ((float)M_PI / 180.f) * deg; }

struct V { float x, y, z; };
V normalize(V v) {
    const float inv = 1.f / std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    return V{v.x * inv, v.y * inv, v.z * inv};
}

/* pbrt-v2 Rotate(angle, axis) */
Transform rotate(float angle, V axis) {
    const V a = normalize(axis);
    const float s = std::sin(radians(angle)), c = std::cos(radians(angle));
    float m[16] = {0};
    m[0] = a.x * a.x + (1.f - a.x * a.x) * c;
    m[1] = a.x * a.y * (1.f - c) - a.z * s;
    m[2] = a.x * a.z * (1.f - c) + a.y * s;
    m[4] = a.x * a.y * (1.f - c) + a.z * s;
    m[5] = a.y * a.y + (1.f - a.y * a.y) * c;
    m[6] = a.y * a.z * (1.f - c) - a.x * s;
    m[8] = a.x * a.z * (1.f - c) - a.y * s;
    m[9] = a.y * a.z * (1.f - c) + a.x * s;
    m[10] = a.z * a.z + (1.f - a.z * a.z) * c;
    m[15] = 1.f;
    Transform t;
    std::memcpy(t.m, m, sizeof(m));
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) t.minv[4 * i + j] = m[4 * j + i];
    return t;
}

/* pbrt-v2 LookAt: Transform(Inverse(camToWorld), camToWorld). The frame is
 * computed in double (pbrt-v2 normalizes in float: <= 1 ulp apart), so an
 * axis-aligned view gives exact unit axes. */
Transform look_at(V pos, V look, V up) {
    auto nrm = [](double v[3]) {
        const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        for (int a = 0; a < 3; ++a) v[a] /= l;
    };
    auto crs = [](const double a[3], const double b[3], double o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
    };
    double dir[3] = {(double)look.x - pos.x, (double)look.y - pos.y, (double)look.z - pos.z}, u[3] = {up.x, up.y, up.z};
    double left[3], nu[3];
    nrm(dir); nrm(u);
    crs(u, dir, left);
    nrm(left);
    crs(dir, left, nu);
    const float c2w[16] = {(float)left[0], (float)nu[0], (float)dir[0], pos.x, (float)left[1], (float)nu[1],
                           (float)dir[1], pos.y, (float)left[2], (float)nu[2], (float)dir[2], pos.z,
                           0.f, 0.f, 0.f, 1.f};
    Transform t;
    std::memcpy(t.minv, c2w, sizeof(c2w));
    if (!invert(c2w, t.m)) throw Error("LookAt: degenerate camera frame");
    return t;
}

Transform inverse(const Transform &t) {
    Transform r;
    std::memcpy(r.m, t.minv, sizeof(r.m));
    std::memcpy(r.minv, t.m, sizeof(r.minv));
    return r;
}

/* ------------------------------------------------------------ state */
struct GraphicsState {
    const Material *material = nullptr;
    std::string area_light;        /* "" = none */
    ParamSet area_params;
    bool reverse = false;
};

} // namespace

struct PbrtParser::Impl {
    PbrtSink *sink = nullptr;
    PbrtOptions *opts = nullptr;
    Transform ctm = Transform::identity();
    GraphicsState gs;
    std::vector<std::pair<Transform, GraphicsState>> attr_stack;
    std::vector<Transform> xform_stack;
    std::map<std::string, Transform> coord_sys;
    std::deque<Material> materials; /* stable addresses: CudaRender keys materials by pointer */
    std::map<std::string, const Material *> named_materials;
    std::map<std::string, RGB> textures; /* constant spectrum textures */
    std::map<std::string, int> instances; /* node addresses are the instance keys */
    const void *current_instance = nullptr;
    bool in_world = false;
    /* options gathered before WorldBegin */
    Transform camera_to_world = Transform::identity();
    bool have_camera = false;
    ParamSet camera_params;
    int xres = 640, yres = 480; /* pbrt-v2 ImageFilm defaults */

    Impl() {
        materials.push_back(Material{Material::Matte, {0.5f, 0.5f, 0.5f}}); /* pbrt default "matte" Kd 0.5 */
        gs.material = &materials.back();
    }

    void warn(const Lexer &lx, int line, const char *fmt, const std::string &a) {
        std::fprintf(stderr, "Warning: %s:%d: ", lx.file().c_str(), line);
        std::fprintf(stderr, fmt, a.c_str());
        std::fprintf(stderr, "\n");
        opts->warnings++;
    }

    /* ---- parsing helpers */
    static std::string str(Lexer &lx) {
        Token t = lx.next();
        if (t.kind != Token::String) lx.fail(t.line, "expected a quoted string");
        return t.text;
    }
    static double num(Lexer &lx) {
        Token t = lx.next();
        if (t.kind != Token::Number) lx.fail(t.line, "expected a number, got '%s'", t.text.c_str());
        return t.num;
    }
    static std::vector<double> nums(Lexer &lx) { /* "[ n n n ]" or bare numbers */
        std::vector<double> v;
        if (lx.peek().kind == Token::Open) {
            lx.next();
            for (Token t = lx.next(); t.kind != Token::Close; t = lx.next()) {
                if (t.kind != Token::Number) lx.fail(t.line, "expected a number in [ ]");
                v.push_back(t.num);
            }
        } else {
            while (lx.peek().kind == Token::Number) v.push_back(lx.next().num);
        }
        return v;
    }
    static ParamSet params(Lexer &lx) {
        ParamSet ps;
        while (lx.peek().kind == Token::String) {
            Token decl = lx.next();
            std::istringstream is(decl.text);
            Param p;
            if (!(is >> p.type >> p.name)) lx.fail(decl.line, "bad parameter declaration \"%s\"", decl.text.c_str());
            if (p.type == "color") p.type = "rgb";
            if (p.type == "point3") p.type = "point";
            if (p.type == "normal3") p.type = "normal";
            Token t = lx.next();
            auto take = [&](const Token &v) {
                if (v.kind == Token::Number) p.nums.push_back(v.num);
                else if (v.kind == Token::String) p.strs.push_back(v.text);
                else lx.fail(v.line, "bad value for parameter \"%s\"", p.name.c_str());
            };
            if (t.kind == Token::Open) {
                for (Token v = lx.next(); v.kind != Token::Close; v = lx.next()) {
                    if (v.kind == Token::End) lx.fail(t.line, "unterminated [ ] for \"%s\"", p.name.c_str());
                    take(v);
                }
            } else {
                take(t);
            }
            ps.params.push_back(std::move(p));
        }
        return ps;
    }

    /* FindOneSpectrum: rgb only (spectrum / blackbody / xyz: warn, default) */
    RGB spectrum(Lexer &lx, int line, const ParamSet &ps, const std::string &name, RGB dflt) {
        const Param *p = ps.find(name);
        if (!p) return dflt;
        if (p->type == "rgb" && p->nums.size() >= 3) return RGB{(float)p->nums[0], (float)p->nums[1], (float)p->nums[2]};
        if (p->type == "float" && !p->nums.empty()) { const float v = (float)p->nums[0]; return RGB{v, v, v}; }
        warn(lx, line, "spectrum parameter type of \"%s\" not supported; using the default", name);
        return dflt;
    }
    /* GetSpectrumTexture evaluated at a default DifferentialGeometry
     * (cudamaterial.cpp:35-38): constant textures only */
    RGB spectrum_tex(Lexer &lx, int line, const ParamSet &ps, const std::string &name, RGB dflt) {
        const Param *p = ps.find(name);
        if (p && p->type == "texture") {
            auto it = textures.find(p->strs.empty() ? "" : p->strs[0]);
            if (it != textures.end()) return it->second;
            warn(lx, line, "texture \"%s\" is not a constant spectrum texture; using the default",
                 p->strs.empty() ? std::string() : p->strs[0]);
            return dflt;
        }
        return spectrum(lx, line, ps, name, dflt);
    }

    const Material *make_material(Lexer &lx, int line, const std::string &type, const ParamSet &ps) {
        Material m;
        if (type == "matte") {
            m.kind = Material::Matte;
            m.k = spectrum_tex(lx, line, ps, "Kd", RGB{0.5f, 0.5f, 0.5f});
        } else if (type == "mirror") {
            m.kind = Material::Mirror;
            m.k = spectrum_tex(lx, line, ps, "Kr", RGB{0.9f, 0.9f, 0.9f});
        } else if (type == "glass") {
            m.kind = Material::Glass; /* Kr / Kt / index unused by the device (cudamaterial.cpp:69-75) */
            m.k = RGB{1.f, 1.f, 1.f};
        } else {
            warn(lx, line, "material \"%s\" has no MI355X equivalent; using the fallback matte 0.5", type);
            m.kind = Material::Unknown; /* -> matte 0.5 in CudaRender::materialId */
        }
        materials.push_back(m);
        return &materials.back();
    }

    void shape(Lexer &lx, int line, const std::string &name, const ParamSet &ps) {
        Shape s;
        s.o2w = ctm;
        if (name == "trianglemesh") {
            const std::vector<float> P = ps.floats("P");
            const Param *ip = ps.find("indices");
            if (P.empty() || P.size() % 3 || !ip || ip->nums.size() % 3)
                lx.fail(line, "trianglemesh needs \"point P\" and \"integer indices\" (multiples of 3)");
            const int nverts = (int)(P.size() / 3);
            for (double v : ip->nums) {
                if (v < 0 || v >= nverts) lx.fail(line, "trianglemesh index %g out of range", v);
                s.indices.push_back((int)v);
            }
            s.P.resize(P.size());
            for (int v = 0; v < nverts; ++v) ctm.point(&P[3 * v], &s.P[3 * v]); /* pbrt TriangleMesh: world space */
            s.N = ps.floats("N");                                                /* raw, as the mesh keeps them */
            if (!s.N.empty() && s.N.size() != P.size()) { warn(lx, line, "%s: ignoring N of the wrong size", name); s.N.clear(); }
            s.uv = ps.floats("uv");
            if (s.uv.empty()) s.uv = ps.floats("st");
            if (!s.uv.empty() && s.uv.size() != 2 * (size_t)nverts) {
                warn(lx, line, "%s: ignoring uv of the wrong size", name);
                s.uv.clear();
            }
        } else if (name == "sphere") {
            s.radius = ps.oneFloat("radius", 1.f);
        } else if (name == "disk") {
            s.height = ps.oneFloat("height", 0.f);
            s.radius = ps.oneFloat("radius", 1.f);
            s.inner_radius = ps.oneFloat("innerradius", 0.f);
            const float pm = ps.oneFloat("phimax", 360.f);
            s.phi_max = radians(pm < 0.f ? 0.f : (pm > 360.f ? 360.f : pm)); /* Disk ctor */
        }
        int light = -1;
        if (!gs.area_light.empty()) {
            if (current_instance) {
                warn(lx, line, "area lights inside ObjectBegin are not supported (%s)", name);
            } else if (gs.area_light != "diffuse") {
                warn(lx, line, "area light \"%s\" not supported", gs.area_light);
            } else if (name != "disk") { /* cudalight.cpp:35-56: only disks emit */
                warn(lx, line, "UnImplemented Cuda Area Light Source: %s (only disks)", name);
            } else {
                Light L;
                L.kind = Light::AreaDisk;
                L.disk = s;
                const RGB Le = spectrum(lx, line, gs.area_params, "L", RGB{1.f, 1.f, 1.f});
                const RGB sc = spectrum(lx, line, gs.area_params, "scale", RGB{1.f, 1.f, 1.f});
                L.Lemit = RGB{Le.r * sc.r, Le.g * sc.g, Le.b * sc.b};
                L.n_samples = gs.area_params.oneInt("nsamples", 1);
                light = (int)opts->lights.size();
                opts->lights.push_back(L);
            }
        }
        sink->shape(name, s, current_instance, gs.material, light);
    }

    void camera_done() {
        /* pinhole through the pixel centres: d = fwd + sx*right + sy*up,
         * sx, sy in [-1, 1] (pm_set_pinhole); the screen window folds into
         * the three vectors */
        /* the field of view as written (double): pbrt-v2 rounds it to float
         * first, which moves the frustum by < 1e-7 */
        double fov = camera_params.oneDouble("fov", 90.0);
        const double half = camera_params.oneDouble("halffov", -1.0);
        if (half > 0.0) fov = 2.0 * half;
        const double t = std::tan(fov * (M_PI / 180.0) / 2.0);
        /* screen window (pbrt-v2 CreatePerspectiveCamera): the fov spans the
         * shorter image axis */
        double cx = 0.0, cy = 0.0, sx, sy;
        const Param *fp = camera_params.find("frameaspectratio");
        const double frame = fp && !fp->nums.empty() ? (double)(float)fp->nums[0] : (double)xres / (double)yres;
        if (frame > 1.0) { sx = fp ? t * frame : t * xres / yres; sy = t; }
        else { sx = t; sy = fp ? t / frame : t * yres / xres; }
        const std::vector<float> w = camera_params.floats("screenwindow");
        if (w.size() == 4) {
            cx = t * 0.5 * ((double)w[0] + w[1]); cy = t * 0.5 * ((double)w[2] + w[3]);
            sx = t * 0.5 * ((double)w[1] - w[0]); sy = t * 0.5 * ((double)w[3] - w[2]);
        }
        const float o[3] = {0.f, 0.f, 0.f}, X[3] = {1.f, 0.f, 0.f}, Y[3] = {0.f, 1.f, 0.f}, Z[3] = {0.f, 0.f, 1.f};
        float x[3], y[3], z[3];
        Camera &cam = opts->camera;
        camera_to_world.point(o, cam.eye);
        camera_to_world.vector(X, x);
        camera_to_world.vector(Y, y);
        camera_to_world.vector(Z, z);
        for (int a = 0; a < 3; ++a) {
            cam.fwd[a] = (float)(z[a] + cx * x[a] + cy * y[a]);
            cam.right[a] = (float)(x[a] * sx);
            cam.up[a] = (float)(y[a] * sy);
        }
        cam.pinhole = true;
        cam.width = xres;
        cam.height = yres;
    }

    void parse(Lexer &lx, const std::string &dir) {
        for (Token t = lx.next(); t.kind != Token::End; t = lx.next()) {
            if (t.kind != Token::Word) lx.fail(t.line, "expected a directive, got '%s'", t.text.c_str());
            const std::string &d = t.text;
            const int line = t.line;
            if (d == "Identity") ctm = Transform::identity();
            else if (d == "Translate") {
                const float x = (float)num(lx), y = (float)num(lx), z = (float)num(lx);
                ctm = ctm * Transform::translate(x, y, z);
            } else if (d == "Scale") {
                const float x = (float)num(lx), y = (float)num(lx), z = (float)num(lx);
                ctm = ctm * scale(x, y, z);
            } else if (d == "Rotate") {
                const float a = (float)num(lx), x = (float)num(lx), y = (float)num(lx), z = (float)num(lx);
                ctm = ctm * rotate(a, V{x, y, z});
            } else if (d == "LookAt") {
                float v[9];
                for (float &f : v) f = (float)num(lx);
                ctm = ctm * look_at(V{v[0], v[1], v[2]}, V{v[3], v[4], v[5]}, V{v[6], v[7], v[8]});
            } else if (d == "Transform" || d == "ConcatTransform") {
                const std::vector<double> v = nums(lx);
                if (v.size() != 16) lx.fail(line, "%s needs 16 numbers", d.c_str());
                float m[16]; /* pbrt lists the matrix column by column */
                for (int i = 0; i < 4; ++i)
                    for (int j = 0; j < 4; ++j) m[4 * i + j] = (float)v[4 * j + i];
                const Transform tr = from_matrix(m);
                ctm = d == "Transform" ? tr : ctm * tr;
            } else if (d == "CoordinateSystem") coord_sys[str(lx)] = ctm;
            else if (d == "CoordSysTransform") {
                const std::string n = str(lx);
                auto it = coord_sys.find(n);
                if (it == coord_sys.end()) warn(lx, line, "coordinate system \"%s\" not defined", n);
                else ctm = it->second;
            } else if (d == "TransformBegin") xform_stack.push_back(ctm);
            else if (d == "TransformEnd") {
                if (xform_stack.empty()) lx.fail(line, "unmatched TransformEnd");
                ctm = xform_stack.back();
                xform_stack.pop_back();
            } else if (d == "ActiveTransform") lx.next();       /* motion blur: not supported, ignored */
            else if (d == "TransformTimes") { num(lx); num(lx); }
            else if (d == "ReverseOrientation") gs.reverse = !gs.reverse;
            else if (d == "Camera") {
                const std::string n = str(lx);
                camera_params = params(lx);
                if (n != "perspective") lx.fail(line, "camera \"%s\" not supported (perspective only)", n.c_str());
                if (camera_params.oneFloat("lensradius", 0.f) > 0.f)
                    warn(lx, line, "%s: depth of field not supported (pinhole)", n);
                camera_to_world = inverse(ctm);
                coord_sys["camera"] = camera_to_world;
                have_camera = true;
            } else if (d == "Film") {
                str(lx);
                const ParamSet ps = params(lx);
                xres = ps.oneInt("xresolution", 640);
                yres = ps.oneInt("yresolution", 480);
                opts->film_filename = ps.oneString("filename", opts->film_filename);
            } else if (d == "Renderer") {
                const std::string n = str(lx);
                const ParamSet ps = params(lx);
                opts->renderer = ps.oneString("rendername", n == "cuda" ? "photonmapping" : n);
                pm_render_params &p = opts->settings.params;
                p.paths_per_pass = ps.oneInt("paths", (int)p.paths_per_pass);
                p.passes = ps.oneInt("passes", p.passes);
                const std::string g = ps.oneString("gather", "grid");
                p.gather_structure = g == "kdtree" || g == "kd" ? PM_GATHER_KDTREE : PM_GATHER_GRID;
            } else if (d == "Sampler" || d == "PixelFilter" || d == "SurfaceIntegrator" || d == "VolumeIntegrator" ||
                       d == "Accelerator" || d == "Volume") {
                str(lx);
                params(lx);
            } else if (d == "WorldBegin") {
                if (!have_camera) { camera_to_world = inverse(ctm); have_camera = true; }
                camera_done();
                ctm = Transform::identity();
                coord_sys["world"] = ctm;
                in_world = true;
            } else if (d == "WorldEnd") {
                in_world = false;
            } else if (d == "AttributeBegin") attr_stack.emplace_back(ctm, gs);
            else if (d == "AttributeEnd") {
                if (attr_stack.empty()) lx.fail(line, "unmatched AttributeEnd");
                ctm = attr_stack.back().first;
                gs = attr_stack.back().second;
                attr_stack.pop_back();
            } else if (d == "Material") {
                const std::string n = str(lx);
                const ParamSet ps = params(lx);
                gs.material = make_material(lx, line, n, ps);
            } else if (d == "MakeNamedMaterial") {
                const std::string n = str(lx);
                const ParamSet ps = params(lx);
                named_materials[n] = make_material(lx, line, ps.oneString("type", "matte"), ps);
            } else if (d == "NamedMaterial") {
                const std::string n = str(lx);
                auto it = named_materials.find(n);
                if (it == named_materials.end()) warn(lx, line, "named material \"%s\" not defined", n);
                else gs.material = it->second;
            } else if (d == "Texture") {
                const std::string n = str(lx), type = str(lx), cls = str(lx);
                const ParamSet ps = params(lx);
                if ((type == "spectrum" || type == "color") && cls == "constant")
                    textures[n] = spectrum(lx, line, ps, "value", RGB{1.f, 1.f, 1.f});
                else if (type == "spectrum" || type == "color")
                    warn(lx, line, "texture class \"%s\" not supported (constant only)", cls);
            } else if (d == "LightSource") {
                const std::string n = str(lx);
                const ParamSet ps = params(lx);
                if (n == "point") {
                    const RGB I = spectrum(lx, line, ps, "I", RGB{1.f, 1.f, 1.f});
                    const RGB sc = spectrum(lx, line, ps, "scale", RGB{1.f, 1.f, 1.f});
                    const std::vector<float> from = ps.floats("from");
                    const float o[3] = {0.f, 0.f, 0.f};
                    Light L;
                    L.kind = Light::Point;
                    ctm.point(o, L.pos); /* Translate(from) * light2world, applied to the origin */
                    if (from.size() == 3) for (int a = 0; a < 3; ++a) L.pos[a] = L.pos[a] + from[a];
                    L.intensity = RGB{I.r * sc.r, I.g * sc.g, I.b * sc.b};
                    opts->lights.push_back(L);
                } else {
                    warn(lx, line, "UnImplemented Cuda Light Source: %s", n); /* cudalight.cpp:11-14,67-69 */
                }
            } else if (d == "AreaLightSource") {
                gs.area_light = str(lx);
                gs.area_params = params(lx);
            } else if (d == "Shape") {
                const std::string n = str(lx);
                const ParamSet ps = params(lx);
                if (!in_world) lx.fail(line, "Shape outside WorldBegin/WorldEnd");
                shape(lx, line, n, ps);
            } else if (d == "ObjectBegin") {
                const std::string n = str(lx);
                attr_stack.emplace_back(ctm, gs);
                current_instance = &instances[n];
            } else if (d == "ObjectEnd") {
                if (!current_instance || attr_stack.empty()) lx.fail(line, "ObjectEnd outside ObjectBegin");
                current_instance = nullptr;
                ctm = attr_stack.back().first;
                gs = attr_stack.back().second;
                attr_stack.pop_back();
            } else if (d == "ObjectInstance") {
                const std::string n = str(lx);
                auto it = instances.find(n);
                if (it == instances.end()) lx.fail(line, "object \"%s\" not defined", n.c_str());
                sink->objectInstance(&it->second, ctm);
            } else if (d == "Include") {
                std::string f = str(lx);
                if (!f.empty() && f[0] != '/') f = dir + "/" + f;
                parse_file(f);
            } else {
                lx.fail(line, "unknown directive '%s'", d.c_str());
            }
        }
    }

    void parse_file(const std::string &path) {
        std::ifstream in(path, std::ios::binary);
        if (!in) throw Error("cannot open scene file " + path);
        std::stringstream ss;
        ss << in.rdbuf();
        const size_t slash = path.find_last_of('/');
        Lexer lx(ss.str(), path);
        parse(lx, slash == std::string::npos ? "." : path.substr(0, slash));
    }
};

PbrtParser::PbrtParser() : impl_(new Impl) {}
PbrtParser::~PbrtParser() { delete impl_; }

void PbrtParser::parseFile(const std::string &path, PbrtSink &sink, PbrtOptions &opts) {
    impl_->sink = &sink;
    impl_->opts = &opts;
    impl_->parse_file(path);
}

void PbrtParser::parseString(const std::string &text, PbrtSink &sink, PbrtOptions &opts, const std::string &dir) {
    impl_->sink = &sink;
    impl_->opts = &opts;
    Lexer lx(text, "<string>");
    impl_->parse(lx, dir);
}

} // namespace pmcuda
