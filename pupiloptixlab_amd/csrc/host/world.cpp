// world.cpp — the reference's resource::Scene loader and world::World
// preparation, producing the flat pupil_scene_desc the engine consumes.
//
//   Scene::LoadFromXML / LoadXmlObj        framework/resource/scene.cpp:27-227
//   LoadShapeInstanceFromXml + built-ins   framework/resource/shape.cpp:20-217
//   LoadMaterialFromXml + IOR lookup       framework/resource/material.cpp:26-190, render/material/ior.h
//   LoadTransform3D / LoadTextureOrRGB     framework/resource/xml/util_loader.cpp:101-211
//   World::LoadScene                       framework/world/world.cpp:101-139
//   EmitterHelper (area emitters, probs)   framework/world/emitter.cpp:169-337
//   CameraHelper (sample_to_camera)        framework/world/camera.cpp:72-91, util/camera.cpp:7-101
#include <cmath>
#include <cstdio>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/pupil_pt.h"
#include "hmath.h"
#include "xml.h"

namespace Pupil {

void set_last_error(const std::string &m);  // engine.hip (pupil_last_error)

namespace {
int werr(int code, const std::string &m) {
    set_last_error(m);
    return code;
}
void warn(const std::string &m) { std::fprintf(stderr, "[pupil] warning: %s\n", m.c_str()); }

std::vector<std::string> split(const std::string &s, const std::string &delims) {
    std::vector<std::string> out;
    std::string cur;
    for (char c : s) {
        if (delims.find(c) != std::string::npos) {
            if (!cur.empty()) out.push_back(cur);
            cur.clear();
        } else if (c != ' ' || delims.find(' ') == std::string::npos) {
            cur += c;
        }
    }
    if (!cur.empty()) out.push_back(cur);
    return out;
}

float to_float(const std::string &s) { return std::stof(s); }
}  // namespace

namespace image {  // image_load.cpp
bool LoadBitmap(const std::string &path, std::vector<float> &rgba, int &w, int &h, std::string &err);
}

namespace resource {

struct Texture {
    uint32_t type = PUPIL_TEX_RGB;
    util::Float3 c0{0.f, 0.f, 0.f};
    util::Float3 c1{0.f, 0.f, 0.f};
    util::Transform transform{};
    uint32_t width = 0, height = 0, filter = 0;
    std::shared_ptr<std::vector<float>> rgba;
};

Texture ColorTexture(util::Float3 c) {
    Texture t;
    t.type = PUPIL_TEX_RGB;
    t.c0 = c;
    return t;
}

struct Material {
    uint32_t type = PUPIL_MAT_UNKNOWN;
    bool twosided = false;
    float int_ior = 1.f, ext_ior = 1.f;
    bool nonlinear = false;
    Texture tex[4];
};

struct Mesh {
    std::vector<float> positions, normals, texcoords;
    std::vector<uint32_t> indices;
};

struct Shape {
    uint32_t kind = PUPIL_SHAPE_MESH;
    std::string name;  // "rectangle", "cube", "sphere" or file path
    std::shared_ptr<Mesh> mesh;
};

struct ShapeInstance {
    std::string name;
    int shape = -1;
    bool face_normals = false, flip_tex_coords = false, flip_normals = false;
    Material mat;
    bool is_emitter = false;
    Texture radiance;
    util::Transform transform{};
};

struct SceneEmitter {
    uint32_t type = PUPIL_EMITTER_NONE;
    util::Float3 radiance{};
    Texture envmap;
    float scale = 1.f;
    util::Transform transform{};
};

// ---- built-in shapes (shape.cpp:20-66 geometry: unit rectangle/cube)
std::shared_ptr<Mesh> MakeRectangle() {
    auto m = std::make_shared<Mesh>();
    m->positions = {-1, -1, 0, 1, -1, 0, 1, 1, 0, -1, 1, 0};
    m->normals = {0, 0, 1, 0, 0, 1, 0, 0, 1, 0, 0, 1};
    m->texcoords = {0, 0, 1, 0, 1, 1, 0, 1};
    m->indices = {0, 1, 2, 0, 2, 3};
    return m;
}
std::shared_ptr<Mesh> MakeCube() {
    auto m = std::make_shared<Mesh>();
    // six faces, four vertices each: -X, -Z, +X, +Z, +Y, -Y
    const float face_pos[6][4][3] = {
        {{-1, -1, -1}, {-1, -1, 1}, {-1, 1, 1}, {-1, 1, -1}}, {{1, -1, -1}, {-1, -1, -1}, {-1, 1, -1}, {1, 1, -1}},
        {{1, -1, 1}, {1, -1, -1}, {1, 1, -1}, {1, 1, 1}},     {{-1, -1, 1}, {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}},
        {{-1, 1, 1}, {1, 1, 1}, {1, 1, -1}, {-1, 1, -1}},     {{-1, -1, -1}, {1, -1, -1}, {1, -1, 1}, {-1, -1, 1}}};
    const float face_nrm[6][3] = {{-1, 0, 0}, {0, 0, -1}, {1, 0, 0}, {0, 0, 1}, {0, 1, 0}, {0, -1, 0}};
    const float uv[4][2] = {{0, 0}, {1, 0}, {1, 1}, {0, 1}};
    for (int f = 0; f < 6; f++) {
        for (int v = 0; v < 4; v++) {
            for (int k = 0; k < 3; k++) m->positions.push_back(face_pos[f][v][k]);
            for (int k = 0; k < 3; k++) m->normals.push_back(face_nrm[f][k]);
            m->texcoords.push_back(uv[v][0]);
            m->texcoords.push_back(uv[v][1]);
        }
        const uint32_t b = 4 * f;
        for (uint32_t i : {b, b + 1, b + 2, b, b + 2, b + 3}) m->indices.push_back(i);
    }
    return m;
}

// ---- Wavefront OBJ (replaces assimp ReadFile(aiProcess_Triangulate),
// shape.cpp:219-278): one vertex per face corner, fan triangulation.
bool LoadObj(const std::string &path, Mesh &out, std::string &err) {
    std::ifstream f(path);
    if (!f) {
        err = "cannot open " + path;
        return false;
    }
    std::vector<float> v, vt, vn;
    struct Corner {
        int v, t, n;
    };
    std::vector<Corner> corners;
    bool any_t = false, any_n = false;
    // assimp's OBJ importer makes one aiMesh per object ('o') and per material change
    // ('usemtl') that receives faces; the reference loads a file only when it yields
    // exactly one mesh (resource/shape.cpp:230-233), so count them the same way.
    int meshes = 0;
    bool segment_has_faces = false;
    std::string material;
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "o") {
            segment_has_faces = false;
        } else if (tag == "usemtl") {
            std::string m;
            ss >> m;
            if (m != material && segment_has_faces) segment_has_faces = false;
            material = m;
        } else if (tag == "v") {
            float x, y, z;
            ss >> x >> y >> z;
            v.insert(v.end(), {x, y, z});
        } else if (tag == "vt") {
            float x = 0, y = 0;
            ss >> x >> y;
            vt.insert(vt.end(), {x, y});
        } else if (tag == "vn") {
            float x, y, z;
            ss >> x >> y >> z;
            vn.insert(vn.end(), {x, y, z});
        } else if (tag == "f") {
            std::vector<Corner> poly;
            std::string tok;
            while (ss >> tok) {
                Corner c{0, 0, 0};
                const auto parts = [&]() {
                    std::vector<std::string> p(3);
                    size_t k = 0;
                    for (char ch : tok) {
                        if (ch == '/') k++;
                        else if (k < 3) p[k] += ch;
                    }
                    return p;
                }();
                auto fix = [](const std::string &s, size_t n) -> int {
                    if (s.empty()) return 0;
                    int i = std::stoi(s);
                    return i < 0 ? (int)n + i + 1 : i;
                };
                c.v = fix(parts[0], v.size() / 3);
                c.t = fix(parts[1], vt.size() / 2);
                c.n = fix(parts[2], vn.size() / 3);
                poly.push_back(c);
            }
            if (!segment_has_faces && poly.size() >= 3) {
                segment_has_faces = true;
                meshes++;
            }
            for (size_t k = 2; k < poly.size(); k++) {
                corners.push_back(poly[0]);
                corners.push_back(poly[k - 1]);
                corners.push_back(poly[k]);
            }
        }
    }
    if (meshes != 1) {
        err = path + " holds " + std::to_string(meshes) +
              " meshes (objects / materials); only single-mesh OBJ files load (resource/shape.cpp:230-233)";
        return false;
    }
    for (auto &c : corners) {
        if (c.t > 0) any_t = true;
        if (c.n > 0) any_n = true;
    }
    for (size_t i = 0; i < corners.size(); i++) {
        const Corner &c = corners[i];
        if (c.v <= 0 || (size_t)c.v * 3 > v.size()) {
            err = "bad vertex index in " + path;
            return false;
        }
        out.positions.insert(out.positions.end(), {v[3 * (c.v - 1)], v[3 * (c.v - 1) + 1], v[3 * (c.v - 1) + 2]});
        if (any_n) {
            if (c.n > 0 && (size_t)c.n * 3 <= vn.size())
                out.normals.insert(out.normals.end(),
                                   {vn[3 * (c.n - 1)], vn[3 * (c.n - 1) + 1], vn[3 * (c.n - 1) + 2]});
            else
                out.normals.insert(out.normals.end(), {0.f, 0.f, 0.f});
        }
        if (any_t) {
            if (c.t > 0 && (size_t)c.t * 2 <= vt.size())
                out.texcoords.insert(out.texcoords.end(), {vt[2 * (c.t - 1)], vt[2 * (c.t - 1) + 1]});
            else
                out.texcoords.insert(out.texcoords.end(), {0.f, 0.f});
        }
        out.indices.push_back((uint32_t)i);
    }
    if (out.indices.empty()) {
        err = "no faces in " + path;
        return false;
    }
    return true;
}

// util::BitmapTexture::Load (framework/util/texture.cpp:162-174) -> a bitmap
// texture; EXR / HDR / PNG / JPEG / PFM decoding lives in image_load.cpp.
// On failure the caller falls back to black like TextureManager::GetTexture
// (resource/texture.cpp:53-60).
bool LoadImageTexture(const std::string &path, Texture &t, std::string &err) {
    auto data = std::make_shared<std::vector<float>>();
    int w = 0, h = 0;
    if (!Pupil::image::LoadBitmap(path, *data, w, h, err)) return false;
    t.type = PUPIL_TEX_BITMAP;
    t.width = (uint32_t)w;
    t.height = (uint32_t)h;
    t.rgba = data;
    return true;
}

// ---- IOR tables (render/material/ior.h data; values from Hecht / measured n,k)
struct DielectricIor {
    const char *name;
    float value;
};
const DielectricIor kDielectric[] = {
    {"vacuum", 1.0f},        {"helium", 1.000036f},     {"hydrogen", 1.000132f},       {"air", 1.000277f},
    {"carbon dioxide", 1.00045f}, {"water", 1.3330f},   {"acetone", 1.36f},            {"ethanol", 1.361f},
    {"carbon tetrachloride", 1.461f}, {"glycerol", 1.4729f}, {"benzene", 1.501f},       {"silicone oil", 1.52045f},
    {"bromine", 1.661f},     {"water ice", 1.31f},      {"fused quartz", 1.458f},      {"pyrex", 1.470f},
    {"acrylic glass", 1.49f}, {"polypropylene", 1.49f}, {"bk7", 1.5046f},              {"sodium chloride", 1.544f},
    {"amber", 1.55f},        {"pet", 1.5750f},          {"diamond", 2.419f}};
struct ConductorIor {
    const char *name;
    float eta[3], k[3];
};
const ConductorIor kConductor[] = {
    {"a-C", {2.93785f, 2.22242f, 1.96400f}, {0.88555f, 0.79763f, 0.81356f}},
    {"Ag", {0.15494f, 0.11648f, 0.13809f}, {4.81810f, 3.11562f, 2.14240f}},
    {"Al", {1.65394f, 0.87850f, 0.52012f}, {9.20430f, 6.25621f, 4.82675f}},
    {"Au", {0.14282f, 0.37414f, 1.43944f}, {3.97472f, 2.38066f, 1.59981f}},
    {"Cr", {4.36041f, 2.91052f, 1.65119f}, {5.19538f, 4.22239f, 3.74700f}},
    {"Cu", {0.19999f, 0.92209f, 1.09988f}, {3.90464f, 2.44763f, 2.13765f}},
    {"Fe", {2.76404f, 1.95417f, 1.62766f}, {3.83077f, 2.73841f, 2.31812f}},
    {"Hg", {2.39384f, 1.43697f, 0.90762f}, {6.31420f, 4.36266f, 3.41454f}},
    {"Ni", {2.36225f, 1.65983f, 1.46395f}, {4.48929f, 3.04369f, 2.34046f}},
    {"Rh", {2.58031f, 1.85624f, 1.55114f}, {6.76790f, 4.69297f, 3.96766f}},
    {"TiN", {1.64497f, 1.14800f, 1.37685f}, {3.36132f, 1.93936f, 1.09967f}},
    {"W", {4.36142f, 3.29330f, 2.99191f}, {3.49325f, 2.59934f, 2.26838f}},
    {"none", {0.f, 0.f, 0.f}, {1.f, 1.f, 1.f}}};

float LoadDielectricIor(const std::string &s, float def) {
    if (s.empty()) return def;
    try {
        size_t used = 0;
        const float v = std::stof(s, &used);
        if (used == s.size()) return v;
    } catch (...) {
    }
    for (auto &e : kDielectric)
        if (s == e.name) return e.value;
    return def;
}
bool LoadConductorIor(const std::string &name, util::Float3 &eta, util::Float3 &k) {
    if (name.empty()) return false;
    for (auto &e : kConductor)
        if (name == e.name) {
            eta = {e.eta[0], e.eta[1], e.eta[2]};
            k = {e.k[0], e.k[1], e.k[2]};
            return true;
        }
    return false;
}

class Scene {
public:
    std::filesystem::path root;
    int max_depth = 1;
    struct {
        float fov = 90.f, near_clip = 0.01f, far_clip = 10000.f;
        util::Transform transform{};
        int w = 768, h = 576;
    } sensor;
    std::vector<Shape> shapes;
    std::vector<ShapeInstance> instances;
    std::vector<SceneEmitter> emitters;
    int rect = -1, cube = -1, sphere = -1;

    int BuiltinShape(const std::string &name) {
        int *slot = name == "rectangle" ? &rect : name == "cube" ? &cube : name == "sphere" ? &sphere : nullptr;
        if (!slot) return -1;
        if (*slot < 0) {
            Shape s;
            s.name = name;
            if (name == "sphere") s.kind = PUPIL_SHAPE_SPHERE;
            else s.mesh = name == "cube" ? MakeCube() : MakeRectangle();
            shapes.push_back(s);
            *slot = (int)shapes.size() - 1;
        }
        return *slot;
    }

    // ---- xml util loaders (util_loader.cpp)
    static bool LoadInt(const xml::Object *o, const char *n, int &p, int def) {
        auto v = o->GetProperty(n);
        if (v.empty()) {
            p = def;
            return false;
        }
        p = std::stoi(v);
        return true;
    }
    static bool LoadFloat(const xml::Object *o, const char *n, float &p, float def) {
        auto v = o->GetProperty(n);
        if (v.empty()) {
            p = def;
            return false;
        }
        p = to_float(v);
        return true;
    }
    static bool LoadFloat3(const std::string &v, util::Float3 &p, util::Float3 def) {
        if (v.empty()) {
            p = def;
            return false;
        }
        auto xyz = split(v, ",");
        if (xyz.size() == 3) p = {to_float(xyz[0]), to_float(xyz[1]), to_float(xyz[2])};
        else if (xyz.size() == 1) p.x = p.y = p.z = to_float(xyz[0]);
        else {
            warn("float3 property must have 1 or 3 components: " + v);
            return false;
        }
        return true;
    }
    static bool Load3Float(const std::string &v, util::Float3 &p, util::Float3 def) {
        if (v.empty()) {
            p = def;
            return false;
        }
        auto xyz = split(v, ",");
        if (xyz.size() != 3) {
            warn("point property must have 3 components: " + v);
            return false;
        }
        p = {to_float(xyz[0]), to_float(xyz[1]), to_float(xyz[2])};
        return true;
    }
    static bool LoadBool(const xml::Object *o, const char *n, bool &p, bool def) {
        auto v = o->GetProperty(n);
        if (v == "true") p = true;
        else if (v == "false") p = false;
        else {
            p = def;
            return false;
        }
        return true;
    }
    static void LoadTransform3D(const xml::Object *o, util::Transform &t) {
        auto value = o->GetProperty("matrix");
        if (!value.empty()) {
            auto el = split(value, " ");
            if (el.size() == 16) {
                for (int i = 0; i < 16; i++) t.matrix.e[i] = to_float(el[i]);
            } else if (el.size() == 9) {
                for (int i = 0, j = 0; j < 9; j++) {
                    t.matrix.e[i] = to_float(el[j]);
                    ++i;
                    if ((j + 1) % 3 == 0) ++i;
                }
            } else {
                warn("transform matrix size must be 9 or 16");
                for (size_t i = 0; i < el.size() && i < 16; i++) t.matrix.e[i] = to_float(el[i]);
            }
            return;
        }
        if (auto *la = o->GetUniqueSubObject("lookat")) {
            util::Float3 origin{1, 0, 0}, target{0, 0, 0}, up{0, 1, 0};
            Load3Float(la->GetProperty("origin"), origin, {1, 0, 0});
            Load3Float(la->GetProperty("target"), target, {0, 0, 0});
            Load3Float(la->GetProperty("up"), up, {0, 1, 0});
            t.LookAt(origin, target, up);
            for (int r = 0; r < 3; r++) {  // mitsuba +X left / +Z view -> Pupil (util_loader.cpp:168-175)
                t.matrix.at(r, 0) *= -1.f;
                t.matrix.at(r, 2) *= -1.f;
            }
            return;
        }
        util::Float3 scale;
        if (LoadFloat3(o->GetProperty("scale"), scale, {})) t.Scale(scale.x, scale.y, scale.z);
        if (auto *rot = o->GetUniqueSubObject("rotate")) {
            util::Float3 axis;
            float angle;
            if (Load3Float(rot->GetProperty("axis"), axis, {}) && LoadFloat(rot, "angle", angle, 0.f))
                t.Rotate(axis.x, axis.y, axis.z, angle);
        }
        util::Float3 tr;
        if (Load3Float(o->GetProperty("translate"), tr, {})) t.Translate(tr.x, tr.y, tr.z);
    }
    static void LoadTransform(const xml::Object *o, util::Transform &t) {
        if (!o) return;
        if (o->var_name == "to_world") LoadTransform3D(o, t);
        else if (o->var_name == "to_uv") {
            util::Float3 s;
            if (LoadFloat3(o->GetProperty("scale"), s, {})) t.Scale(s.x, s.y, s.z);
        } else {
            warn("transform [" + o->var_name + "] unknown");
        }
    }
    void LoadTexture(const xml::Object *o, Texture &t) {
        if (o->type == "bitmap") {
            const auto path = (root / o->GetProperty("filename")).string();
            Texture loaded;
            std::string err;
            if (!LoadImageTexture(path, loaded, err)) {
                warn("bitmap [" + path + "] not loadable (" + err + "); using black");
                loaded = ColorTexture({0, 0, 0});
            }
            t = loaded;
            t.filter = o->GetProperty("filter_type") == "bilinear" ? 1u : 0u;
        } else if (o->type == "checkerboard") {
            t = Texture{};
            t.type = PUPIL_TEX_CHECKERBOARD;
            LoadFloat3(o->GetProperty("color0"), t.c0, {0.4f, 0.4f, 0.4f});
            LoadFloat3(o->GetProperty("color1"), t.c1, {0.2f, 0.2f, 0.2f});
        } else {
            warn("unknown texture type [" + o->type + "]");
            t = ColorTexture({0, 0, 0});
        }
        LoadTransform(o->GetUniqueSubObject("transform"), t.transform);
    }
    bool LoadTextureOrRGB(const xml::Object *o, const char *name, Texture &t, util::Float3 def) {
        auto [tex, rgb] = o->GetParameter(name);
        if (!tex && rgb.empty()) {
            t = ColorTexture(def);
            return false;
        }
        if (!tex) {
            util::Float3 c;
            LoadFloat3(rgb, c, def);
            t = ColorTexture(c);
        } else {
            LoadTexture(tex, t);
        }
        return true;
    }
    Material LoadMaterial(const xml::Object *o) {
        Material m;
        if (!o) return m;
        const std::string &ty = o->type;
        if (ty == "diffuse") {
            m.type = PUPIL_MAT_DIFFUSE;
            LoadTextureOrRGB(o, "reflectance", m.tex[0], {0.5f, 0.5f, 0.5f});
        } else if (ty == "dielectric" || ty == "roughdielectric") {
            const bool rough = ty == "roughdielectric";
            m.type = rough ? PUPIL_MAT_ROUGH_DIELECTRIC : PUPIL_MAT_DIELECTRIC;
            m.int_ior = LoadDielectricIor(o->GetProperty("int_ior"), 1.5046f);
            m.ext_ior = LoadDielectricIor(o->GetProperty("ext_ior"), 1.000277f);
            int k = 0;
            if (rough) LoadTextureOrRGB(o, "alpha", m.tex[k++], {0.1f, 0.1f, 0.1f});
            LoadTextureOrRGB(o, "specular_reflectance", m.tex[k++], {1, 1, 1});
            LoadTextureOrRGB(o, "specular_transmittance", m.tex[k++], {1, 1, 1});
        } else if (ty == "conductor" || ty == "roughconductor") {
            const bool rough = ty == "roughconductor";
            m.type = rough ? PUPIL_MAT_ROUGH_CONDUCTOR : PUPIL_MAT_CONDUCTOR;
            util::Float3 eta, kk;
            if (!LoadConductorIor(o->GetProperty("material"), eta, kk)) {
                eta = {0, 0, 0};
                kk = {1, 1, 1};
            }
            int k = 0;
            if (rough) LoadTextureOrRGB(o, "alpha", m.tex[k++], {0.1f, 0.1f, 0.1f});
            LoadTextureOrRGB(o, "eta", m.tex[k++], eta);
            LoadTextureOrRGB(o, "k", m.tex[k++], kk);
            LoadTextureOrRGB(o, "specular_reflectance", m.tex[k++], {1, 1, 1});
        } else if (ty == "plastic" || ty == "roughplastic") {
            const bool rough = ty == "roughplastic";
            m.type = rough ? PUPIL_MAT_ROUGH_PLASTIC : PUPIL_MAT_PLASTIC;
            m.int_ior = LoadDielectricIor(o->GetProperty("int_ior"), 1.49f);
            m.ext_ior = LoadDielectricIor(o->GetProperty("ext_ior"), 1.000277f);
            m.nonlinear = o->GetProperty("nonlinear") == "true";
            int k = 0;
            if (rough) LoadTextureOrRGB(o, "alpha", m.tex[k++], {0.1f, 0.1f, 0.1f});
            LoadTextureOrRGB(o, "diffuse_reflectance", m.tex[k++], {0.5f, 0.5f, 0.5f});
            LoadTextureOrRGB(o, "specular_reflectance", m.tex[k++], {1, 1, 1});
        } else if (ty == "twosided") {
            m = LoadMaterial(o->GetUniqueSubObject("bsdf"));
            m.twosided = true;
        } else {
            warn("unknown bsdf [" + ty + "]");
        }
        return m;
    }
    void LoadShape(const xml::Object *o) {
        ShapeInstance ins;
        ins.name = o->id;
        const std::string &ty = o->type;
        if (ty == "rectangle" || ty == "cube") {
            ins.shape = BuiltinShape(ty);
            LoadBool(o, "flip_normals", ins.flip_normals, false);
        } else if (ty == "sphere") {
            util::Float3 center{0, 0, 0};
            float radius;
            Load3Float(o->GetProperty("center"), center, {0, 0, 0});
            LoadFloat(o, "radius", radius, 1.f);
            ins.shape = BuiltinShape("sphere");
            LoadBool(o, "flip_normals", ins.flip_normals, false);
            util::Transform t;
            t.Scale(radius, radius, radius);
            t.Translate(center.x, center.y, center.z);
            ins.transform = t;
        } else if (ty == "obj") {
            const auto path = (root / o->GetProperty("filename")).string();
            int found = -1;
            for (size_t i = 0; i < shapes.size(); i++)
                if (shapes[i].name == path) found = (int)i;
            if (found < 0) {
                Shape s;
                s.name = path;
                s.mesh = std::make_shared<Mesh>();
                std::string err;
                if (!LoadObj(path, *s.mesh, err)) {
                    warn("mesh load failed: " + err);
                    return;
                }
                shapes.push_back(s);
                found = (int)shapes.size() - 1;
            }
            ins.shape = found;
            LoadBool(o, "face_normals", ins.face_normals, false);
            LoadBool(o, "flip_tex_coords", ins.flip_tex_coords, true);
            LoadBool(o, "flip_normals", ins.flip_normals, false);
        } else {
            warn("unknown shape type [" + ty + "]");
            return;
        }
        ins.mat = LoadMaterial(o->GetUniqueSubObject("bsdf"));
        util::Transform t;
        LoadTransform(o->GetUniqueSubObject("transform"), t);
        if (shapes[ins.shape].kind == PUPIL_SHAPE_SPHERE) ins.transform.matrix = t.matrix * ins.transform.matrix;
        else ins.transform = t;
        if (auto *eo = o->GetUniqueSubObject("emitter")) {
            if (eo->type == "area") {
                LoadTextureOrRGB(eo, "radiance", ins.radiance, {0, 0, 0});
                ins.is_emitter = true;
            } else {
                warn("shape emitter not supported");
            }
        }
        instances.push_back(ins);
    }
    void ApplySensor(float fov, char fov_axis, float near_clip, float far_clip, const util::Transform &t, bool flip) {
        sensor.fov = fov;
        sensor.near_clip = near_clip;
        sensor.far_clip = far_clip;
        if (fov_axis == 'x') {  // scene.cpp:122-127
            const float aspect = (float)sensor.h / (float)sensor.w;
            const float radian = sensor.fov * 3.14159265358979323846f / 180.f * 0.5f;
            const float tt = std::tan(radian) * aspect;
            sensor.fov = 2.f * std::atan(tt) * 180.f / 3.14159265358979323846f;
        }
        sensor.transform = t;
        if (flip)
            for (int r = 0; r < 3; r++) {  // scene.cpp:132-139
                sensor.transform.matrix.at(r, 0) *= -1.f;
                sensor.transform.matrix.at(r, 2) *= -1.f;
            }
    }
    bool LoadFromXML(const std::string &file, std::string &err) {
        root = std::filesystem::path(file).parent_path();
        xml::Parser parser;
        xml::Object *scene = parser.LoadFromFile(file, &err);
        if (!scene) return false;
        for (auto *o : scene->sub_object) {
            if (o->obj_name == "integrator") {
                LoadInt(o, "max_depth", max_depth, 1);
            } else if (o->obj_name == "sensor") {
                if (o->type != "perspective") {
                    warn("sensor only supports perspective");
                    continue;
                }
                float fov, nc, fc;
                LoadFloat(o, "fov", fov, 90.f);
                LoadFloat(o, "near_clip", nc, 0.01f);
                LoadFloat(o, "far_clip", fc, 10000.f);
                if (auto *film = o->GetUniqueSubObject("film")) {
                    if (film->type != "hdrfilm") warn("film only supports hdrfilm");
                    else {
                        LoadInt(film, "width", sensor.w, 768);
                        LoadInt(film, "height", sensor.h, 576);
                    }
                }
                char axis = 'x';
                auto v = o->GetProperty("fov_axis");
                if (v == "y" || v == "Y") axis = 'y';
                else if (!v.empty() && v != "x" && v != "X") warn("sensor fov_axis must be x or y");
                util::Transform t;
                LoadTransform(o->GetUniqueSubObject("transform"), t);
                ApplySensor(fov, axis, nc, fc, t, true);
            } else if (o->obj_name == "shape") {
                LoadShape(o);
            } else if (o->obj_name == "emitter") {
                SceneEmitter e;
                if (o->type == "constant") {
                    e.type = PUPIL_EMITTER_CONST_ENV;
                    LoadFloat3(o->GetProperty("radiance"), e.radiance, {0, 0, 0});
                } else if (o->type == "envmap") {
                    e.type = PUPIL_EMITTER_ENV_MAP;
                    LoadFloat(o, "scale", e.scale, 1.f);
                    const auto path = (root / o->GetProperty("filename")).string();
                    std::string err;
                    if (!LoadImageTexture(path, e.envmap, err)) {
                        warn("env map [" + path + "] not loadable (" + err + "); skipped");
                        continue;
                    }
                    e.envmap.filter = 1;
                    LoadTransform(o->GetUniqueSubObject("transform"), e.transform);
                } else {
                    if (o->type != "area") warn("unknown emitter type [" + o->type + "]");
                    continue;
                }
                emitters.push_back(e);
            }
        }
        return true;
    }
};

}  // namespace resource

namespace world {

using resource::Material;
using resource::Texture;

pupil_texture ToDesc(const Texture &t) {
    pupil_texture d;
    std::memset(&d, 0, sizeof(d));
    d.type = t.type;
    d.c0[0] = t.c0.x, d.c0[1] = t.c0.y, d.c0[2] = t.c0.z;
    d.c1[0] = t.c1.x, d.c1[1] = t.c1.y, d.c1[2] = t.c1.z;
    std::memcpy(d.transform, t.transform.matrix.e, sizeof(d.transform));
    d.width = t.width;
    d.height = t.height;
    d.filter = t.filter;
    d.rgba = t.rgba ? t.rgba->data() : nullptr;
    return d;
}

Texture FromDesc(const pupil_texture &d) {
    Texture t;
    t.type = d.type;
    t.c0 = {d.c0[0], d.c0[1], d.c0[2]};
    t.c1 = {d.c1[0], d.c1[1], d.c1[2]};
    std::memcpy(t.transform.matrix.e, d.transform, sizeof(d.transform));
    bool zero = true;
    for (float v : d.transform) zero = zero && v == 0.f;
    if (zero) t.transform = util::Transform{};
    t.width = d.width;
    t.height = d.height;
    t.filter = d.filter;
    if (d.type == PUPIL_TEX_BITMAP && d.rgba)
        t.rgba = std::make_shared<std::vector<float>>(d.rgba, d.rgba + (size_t)d.width * d.height * 4);
    return t;
}

// emitter.cpp:73-101 GetWeight
float GetWeight(const Texture &t) {
    auto mx = [](float r, float g, float b) { return r > g ? (r > b ? r : b) : (g > b ? g : b); };
    if (t.type == PUPIL_TEX_RGB) return mx(t.c0.x, t.c0.y, t.c0.z);
    if (t.type == PUPIL_TEX_CHECKERBOARD) return (mx(t.c0.x, t.c0.y, t.c0.z) + mx(t.c1.x, t.c1.y, t.c1.z)) * 0.5f;
    if (t.type == PUPIL_TEX_BITMAP && t.rgba) {
        float w = 0.f;
        const auto &d = *t.rgba;
        for (size_t i = 0; i < t.width; i++)
            for (size_t j = 0; j < t.height; j++) {
                const size_t k = (i * t.width + j) * 4;
                if (k + 2 < d.size()) w += mx(d[k], d[k + 1], d[k + 2]);
            }
        return w / (1.f * t.width * t.height);
    }
    return 0.f;
}

util::Float3 TransformPoint(util::Float3 p, const util::Mat4 &M) {  // transform.cpp:123-130
    const float *m = M.e;
    const float x = m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3];
    const float y = m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7];
    const float z = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    const float w = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    return {x / w, y / w, z / w};
}
util::Float3 TransformNormal(util::Float3 n, const util::Mat4 &M) {  // transform.cpp:138-146
    const float *m = M.e;
    const float x = m[0] * n.x + m[1] * n.y + m[2] * n.z;
    const float y = m[4] * n.x + m[5] * n.y + m[6] * n.z;
    const float z = m[8] * n.x + m[9] * n.y + m[10] * n.z;
    const float len = std::sqrt(x * x + y * y + z * z);
    return {x / len, y / len, z / len};
}

class World {
public:
    resource::Scene scene;
    // flattened outputs (kept alive for pupil_world_get_desc)
    std::vector<pupil_shape> d_shapes;
    std::vector<pupil_material> d_materials;
    std::vector<pupil_instance> d_instances;
    std::vector<pupil_emitter> d_areas;
    pupil_emitter d_env{};
    bool has_env = false;

    // World::LoadScene(Scene*) + EmitterHelper + CameraHelper
    int Build(pupil_scene_desc &desc) {
        auto &sc = scene;
        d_shapes.clear();
        d_materials.clear();
        d_instances.clear();
        d_areas.clear();
        has_env = false;
        for (auto &s : sc.shapes) {
            pupil_shape ds;
            std::memset(&ds, 0, sizeof(ds));
            ds.kind = s.kind;
            if (s.kind == PUPIL_SHAPE_MESH) {
                ds.num_vertices = (uint32_t)(s.mesh->positions.size() / 3);
                ds.num_faces = (uint32_t)(s.mesh->indices.size() / 3);
                ds.positions = s.mesh->positions.data();
                ds.normals = s.mesh->normals.empty() ? nullptr : s.mesh->normals.data();
                ds.texcoords = s.mesh->texcoords.empty() ? nullptr : s.mesh->texcoords.data();
                ds.indices = s.mesh->indices.data();
            }
            d_shapes.push_back(ds);
        }
        int emitter_offset = 0;
        for (auto &ins : sc.instances) {
            if (ins.shape < 0) continue;
            const resource::Shape &shape = sc.shapes[ins.shape];
            pupil_material dm;
            std::memset(&dm, 0, sizeof(dm));
            dm.type = ins.mat.type;
            dm.twosided = ins.mat.twosided;
            dm.int_ior = ins.mat.int_ior;
            dm.ext_ior = ins.mat.ext_ior;
            dm.nonlinear = ins.mat.nonlinear;
            for (int k = 0; k < 4; k++) dm.tex[k] = ToDesc(ins.mat.tex[k]);
            d_materials.push_back(dm);
            pupil_instance di;
            std::memset(&di, 0, sizeof(di));
            di.shape = (uint32_t)ins.shape;
            di.material = (uint32_t)d_materials.size() - 1;
            std::memcpy(di.to_world, ins.transform.matrix.e, sizeof(di.to_world));
            const util::Mat4 inv = ins.transform.matrix.Inverse();
            std::memcpy(di.to_object, inv.e, sizeof(di.to_object));
            di.flip_normals = ins.flip_normals;
            di.flip_tex_coords = ins.flip_tex_coords;
            di.emitter_offset = -1;
            if (ins.is_emitter) {
                di.emitter_offset = emitter_offset;
                AddAreaEmitter(ins, shape);
                emitter_offset = (int)d_areas.size();
            }
            d_instances.push_back(di);
        }
        for (auto &e : sc.emitters) {
            if (e.type == PUPIL_EMITTER_CONST_ENV) {
                std::memset(&d_env, 0, sizeof(d_env));
                d_env.type = PUPIL_EMITTER_CONST_ENV;
                d_env.color[0] = e.radiance.x, d_env.color[1] = e.radiance.y, d_env.color[2] = e.radiance.z;
                d_env.weight = 1.f;
                has_env = true;
            } else if (e.type == PUPIL_EMITTER_ENV_MAP) {
                std::memset(&d_env, 0, sizeof(d_env));
                d_env.type = PUPIL_EMITTER_ENV_MAP;
                d_env.radiance = ToDesc(e.envmap);
                d_env.scale = e.scale;
                d_env.weight = 1.f;
                const util::Mat4 inv = e.transform.matrix.Inverse();
                for (int r = 0; r < 3; r++)
                    for (int c = 0; c < 3; c++) {
                        d_env.to_world[3 * r + c] = e.transform.matrix.at(r, c);
                        d_env.to_local[3 * r + c] = inv.at(r, c);
                    }
                has_env = true;
            }
        }
        ComputeProbability();
        // camera (CameraHelper::Reset + GetCudaMemory)
        std::memset(&desc, 0, sizeof(desc));
        desc.width = (uint32_t)sc.sensor.w;
        desc.height = (uint32_t)sc.sensor.h;
        desc.max_depth = (uint32_t)(sc.max_depth > 0 ? sc.max_depth : 1);
        const float aspect = (float)sc.sensor.w / (float)sc.sensor.h;
        const util::Mat4 s2c = util::SampleToCamera(sc.sensor.fov, aspect, sc.sensor.near_clip, sc.sensor.far_clip);
        std::memcpy(desc.sample_to_camera, s2c.e, sizeof(desc.sample_to_camera));
        std::memcpy(desc.camera_to_world, sc.sensor.transform.matrix.e, sizeof(desc.camera_to_world));
        desc.num_shapes = (uint32_t)d_shapes.size();
        desc.num_materials = (uint32_t)d_materials.size();
        desc.num_instances = (uint32_t)d_instances.size();
        desc.num_area_emitters = (uint32_t)d_areas.size();
        desc.shapes = d_shapes.data();
        desc.materials = d_materials.data();
        desc.instances = d_instances.data();
        desc.area_emitters = d_areas.data();
        desc.env = has_env ? &d_env : nullptr;
        return PUPIL_OK;
    }

    // EmitterHelper::SetMeshAreaEmitter / SetSphereAreaEmitter (emitter.cpp:169-243)
    void AddAreaEmitter(const resource::ShapeInstance &ins, const resource::Shape &shape) {
        const pupil_texture radiance = ToDesc(ins.radiance);
        const float select_weight = GetWeight(ins.radiance);
        if (shape.kind == PUPIL_SHAPE_SPHERE) {
            pupil_emitter e;
            std::memset(&e, 0, sizeof(e));
            e.type = PUPIL_EMITTER_SPHERE;
            util::Float3 o{0, 0, 0};
            util::Float3 p{o.x + 1.f, o.y, o.z};
            o = TransformPoint(o, ins.transform.matrix);
            p = TransformPoint(p, ins.transform.matrix);
            e.center[0] = o.x, e.center[1] = o.y, e.center[2] = o.z;
            const float dx = o.x - p.x, dy = o.y - p.y, dz = o.z - p.z;
            e.radius = std::sqrt(dx * dx + dy * dy + dz * dz);
            e.area = 4 * 3.14159265358979323846f * e.radius * e.radius;
            e.radiance = radiance;
            e.weight = select_weight * e.area;
            d_areas.push_back(e);
            return;
        }
        const resource::Mesh &mesh = *shape.mesh;
        const util::Mat4 normal_transform = ins.transform.matrix.Inverse().Transpose();
        const size_t nf = mesh.indices.size() / 3;
        for (size_t i = 0; i < nf; i++) {
            pupil_emitter e;
            std::memset(&e, 0, sizeof(e));
            e.type = PUPIL_EMITTER_TRI_AREA;
            util::Float3 p[3];
            for (int v = 0; v < 3; v++) {
                const uint32_t idx = mesh.indices[3 * i + v];
                p[v] = TransformPoint({mesh.positions[3 * idx], mesh.positions[3 * idx + 1], mesh.positions[3 * idx + 2]},
                                      ins.transform.matrix);
                util::Float3 n{0, 0, 1};
                if (!mesh.normals.empty())
                    n = {mesh.normals[3 * idx], mesh.normals[3 * idx + 1], mesh.normals[3 * idx + 2]};
                n = TransformNormal(n, normal_transform);
                e.pos[v][0] = p[v].x, e.pos[v][1] = p[v].y, e.pos[v][2] = p[v].z;
                e.nrm[v][0] = n.x, e.nrm[v][1] = n.y, e.nrm[v][2] = n.z;
                if (!mesh.texcoords.empty()) {
                    e.tex[v][0] = mesh.texcoords[2 * idx];
                    e.tex[v][1] = mesh.texcoords[2 * idx + 1];
                }
            }
            const float v1x = p[1].x - p[0].x, v1y = p[1].y - p[0].y, v1z = p[1].z - p[0].z;
            const float v2x = p[2].x - p[0].x, v2y = p[2].y - p[0].y, v2z = p[2].z - p[0].z;
            const float cx = v1y * v2z - v1z * v2y, cy = v1z * v2x - v1x * v2z, cz = v1x * v2y - v1y * v2x;
            e.area = std::sqrt(cx * cx + cy * cy + cz * cz) * 0.5f;
            e.radiance = radiance;
            e.weight = select_weight * e.area;
            d_areas.push_back(e);
        }
    }

    // EmitterHelper::ComputeProbability (emitter.cpp:321-337)
    void ComputeProbability() {
        float area_weight_sum = 0.f;
        for (auto &e : d_areas) area_weight_sum += e.weight;
        if (!d_areas.empty())
            for (auto &e : d_areas) e.select_probability = e.weight / area_weight_sum * d_areas.size();
        const size_t emitter_num = (has_env ? 1 : 0) + d_areas.size();
        for (auto &e : d_areas) e.select_probability = e.select_probability / emitter_num;
        if (has_env) d_env.select_probability = d_env.weight / emitter_num;
    }
};

}  // namespace world
}  // namespace Pupil

struct pupil_world {
    Pupil::world::World w;
    // materials are per instance in the reference (ShapeInstance::mat); the
    // programmatic API keeps a table and copies into each instance
    std::vector<Pupil::resource::Material> materials;
    pupil_scene_desc desc{};
};

extern "C" {

int pupil_world_create(pupil_world **out) {
    if (!out) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    *out = new pupil_world();
    return PUPIL_OK;
}

void pupil_world_destroy(pupil_world *w) { delete w; }

int pupil_world_load_xml(pupil_world *w, const char *path) {
    if (!w || !path) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    if (!std::filesystem::exists(path)) return Pupil::werr(PUPIL_ERR_IO, std::string("scene file does not exist: ") + path);
    w->w.scene = Pupil::resource::Scene{};
    std::string err;
    try {
        if (!w->w.scene.LoadFromXML(path, err)) return Pupil::werr(PUPIL_ERR_IO, "scene load failed: " + err);
    } catch (const std::exception &e) {
        return Pupil::werr(PUPIL_ERR_INVALID, std::string("scene parse error: ") + e.what());
    }
    return PUPIL_OK;
}

int pupil_world_set_film(pupil_world *w, uint32_t width, uint32_t height, uint32_t max_depth) {
    if (!w || width == 0 || height == 0) return Pupil::werr(PUPIL_ERR_INVALID, "bad film");
    w->w.scene.sensor.w = (int)width;
    w->w.scene.sensor.h = (int)height;
    w->w.scene.max_depth = (int)max_depth;
    return PUPIL_OK;
}

int pupil_world_set_sensor(pupil_world *w, float fov, char fov_axis, float near_clip, float far_clip,
                           const float to_world[16]) {
    if (!w || !to_world) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    Pupil::util::Transform t;
    std::memcpy(t.matrix.e, to_world, sizeof(t.matrix.e));
    w->w.scene.ApplySensor(fov, fov_axis == 'y' || fov_axis == 'Y' ? 'y' : 'x', near_clip, far_clip, t, true);
    return PUPIL_OK;
}

int pupil_world_add_mesh(pupil_world *w, uint32_t nv, uint32_t nf, const float *positions, const float *normals,
                         const float *texcoords, const uint32_t *indices, uint32_t *out_shape) {
    if (!w || !positions || !indices || nv == 0 || nf == 0) return Pupil::werr(PUPIL_ERR_INVALID, "bad mesh");
    Pupil::resource::Shape s;
    s.kind = PUPIL_SHAPE_MESH;
    s.name = "mesh" + std::to_string(w->w.scene.shapes.size());
    s.mesh = std::make_shared<Pupil::resource::Mesh>();
    s.mesh->positions.assign(positions, positions + 3 * (size_t)nv);
    if (normals) s.mesh->normals.assign(normals, normals + 3 * (size_t)nv);
    if (texcoords) s.mesh->texcoords.assign(texcoords, texcoords + 2 * (size_t)nv);
    s.mesh->indices.assign(indices, indices + 3 * (size_t)nf);
    for (uint32_t i : s.mesh->indices)
        if (i >= nv) return Pupil::werr(PUPIL_ERR_INVALID, "mesh index out of range");
    w->w.scene.shapes.push_back(s);
    if (out_shape) *out_shape = (uint32_t)w->w.scene.shapes.size() - 1;
    return PUPIL_OK;
}

int pupil_world_add_builtin_shape(pupil_world *w, const char *name, uint32_t *out_shape) {
    if (!w || !name) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    const int s = w->w.scene.BuiltinShape(name);
    if (s < 0) return Pupil::werr(PUPIL_ERR_INVALID, std::string("unknown built-in shape ") + name);
    if (out_shape) *out_shape = (uint32_t)s;
    return PUPIL_OK;
}

int pupil_world_add_material(pupil_world *w, const pupil_material *m, uint32_t *out_material) {
    if (!w || !m) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    Pupil::resource::Material mat;
    mat.type = m->type;
    mat.twosided = m->twosided != 0;
    mat.int_ior = m->int_ior;
    mat.ext_ior = m->ext_ior;
    mat.nonlinear = m->nonlinear != 0;
    for (int k = 0; k < 4; k++) mat.tex[k] = Pupil::world::FromDesc(m->tex[k]);
    auto &tab = w->materials;
    tab.push_back(mat);
    if (out_material) *out_material = (uint32_t)tab.size() - 1;
    return PUPIL_OK;
}

int pupil_world_add_instance(pupil_world *w, uint32_t shape, uint32_t material, const float to_world[16],
                             uint32_t flip_normals, uint32_t flip_tex_coords, uint32_t is_emitter,
                             const pupil_texture *radiance, uint32_t *out_instance) {
    if (!w || !to_world) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    auto &tab = w->materials;
    if (shape >= w->w.scene.shapes.size()) return Pupil::werr(PUPIL_ERR_INVALID, "shape out of range");
    if (material >= tab.size()) return Pupil::werr(PUPIL_ERR_INVALID, "material out of range");
    Pupil::resource::ShapeInstance ins;
    ins.shape = (int)shape;
    ins.mat = tab[material];
    std::memcpy(ins.transform.matrix.e, to_world, sizeof(ins.transform.matrix.e));
    ins.flip_normals = flip_normals != 0;
    ins.flip_tex_coords = flip_tex_coords != 0;
    ins.is_emitter = is_emitter != 0;
    if (ins.is_emitter) {
        if (!radiance) return Pupil::werr(PUPIL_ERR_INVALID, "emitter without radiance");
        ins.radiance = Pupil::world::FromDesc(*radiance);
    }
    w->w.scene.instances.push_back(ins);
    if (out_instance) *out_instance = (uint32_t)w->w.scene.instances.size() - 1;
    return PUPIL_OK;
}

int pupil_world_set_instance_transform(pupil_world *w, uint32_t instance, const float to_world[16]) {
    if (!w || !to_world) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    // desc instance k = k-th scene instance with a shape (World::Build skips the others)
    uint32_t k = 0;
    for (auto &ins : w->w.scene.instances) {
        if (ins.shape < 0) continue;
        if (k++ == instance) {
            std::memcpy(ins.transform.matrix.e, to_world, sizeof(ins.transform.matrix.e));
            return PUPIL_OK;
        }
    }
    return Pupil::werr(PUPIL_ERR_INVALID, "instance out of range");
}

int pupil_world_add_const_env(pupil_world *w, const float radiance[3]) {
    if (!w || !radiance) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    Pupil::resource::SceneEmitter e;
    e.type = PUPIL_EMITTER_CONST_ENV;
    e.radiance = {radiance[0], radiance[1], radiance[2]};
    w->w.scene.emitters.push_back(e);
    return PUPIL_OK;
}

int pupil_world_get_desc(pupil_world *w, pupil_scene_desc *desc) {
    if (!w || !desc) return Pupil::werr(PUPIL_ERR_INVALID, "null argument");
    if (w->w.scene.instances.empty()) return Pupil::werr(PUPIL_ERR_INVALID, "world has no shape instances");
    const int rc = w->w.Build(w->desc);
    if (rc) return rc;
    *desc = w->desc;
    return PUPIL_OK;
}

}  // extern "C"
